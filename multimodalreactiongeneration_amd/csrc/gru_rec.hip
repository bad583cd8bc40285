// Persistent GRU recurrence for gfx950 (replaces the per-step cell launches of the GRU mixer:
// mixer_block.py:169-208 GRUMixer = torch.nn.GRU, gate order r, z, n; config_gru.yaml:50-52).
//
// Same decomposition as the LSTM recurrence (lstm.hip): gx = X W_ih^T + b_ih comes from one GEMM over
// all steps; the batch is cut into groups of BS rows, each served by G workgroups ("members") that own
// U = H/G hidden units, i.e. R = 3U rows of W_hh (r, z, n), held in VGPRs for the whole sequence.  Per
// step a member
//   1. computes pre[b][row] = sum_k h_{t-1}[b][k] W_hh[row][k] (register-blocked VALU GEMV, DPP reduce),
//   2. runs the cell of its BS x U units:  r = s(gx_r + pre_r + b_hr), z = s(gx_z + pre_z + b_hz),
//      hn = pre_n + b_hn, n = tanh(gx_n + r hn), h = (1 - z) n + z h_{t-1},
//   3. publishes h_t as {tag, value} granules (lstm_common.h) and gathers the group's full h_t.
// G = 1 ("solo", H <= 128): the workgroup holds all of W_hh and exchanges h through its LDS.
// Backward (reverse time): the cell derivative gives dgx = (dr', dz', dn') and dgh = (dr', dz', dn' r);
// a member's partial dh_{t-1} = dgh(own rows) W_hh(own rows, :) is reduce-scattered like the LSTM's,
// and each cell adds its direct term dh_t z_t.  Outputs match the per-step path (gru.hip): y, gates
// (r, z, n), ghn = W_hn h + b_hn, and dGX / dGH for the weight / input gradient GEMMs.
#include "lstm_common.h"

namespace mrg {

struct GruFwdArgs {
  const float* gx; long gx_bs, gx_ts;     // [B, T, 3H] input pre-activations (+ b_ih)
  const float* w_hh; const float* b_hh;   // [3H, H], [3H]
  const float* h0;                        // [B, H] or null
  float* y; long y_bs, y_ts;              // h_t
  float* gates; long g_bs, g_ts;          // r, z, n
  float* ghn; long n_bs, n_ts;            // W_hn h_{t-1} + b_hn
  unsigned long long* xbuf;               // [2][B][H] granules
  int B, T, reverse, local;
  int* err;
};

struct GruBwdArgs {
  const float* w_hh;
  const float* gates; long g_bs, g_ts;
  const float* ghn; long n_bs, n_ts;
  const float* y; long y_bs, y_ts;        // h_t (h_{t-1} of the next step)
  const float* h0;                        // nullable
  const float* dy; long dy_bs, dy_ts;     // nullable
  const float* dhT;                       // nullable [B, H]
  float* dgx; float* dgh; long d_bs, d_ts;
  float* dh0;                             // nullable
  unsigned long long* xbuf;               // [2][B][G][H] granules
  int B, T, reverse, local;
  int* err;
};

// forward tiling: KC = 8 lanes split k, RT rows per lane (4 when the solo H = 128 group would need
// more than 1024 threads at 2)
template <int H, int G>
struct GruFwdCfg {
  static constexpr int U = H / G, R = 3 * U, KC = 8, KL = H / KC;
  static constexpr int RT = (R * KC / 2 > 1024) ? 4 : 2;
  static constexpr int NT = R * KC / RT;
  static constexpr int WPS = (NT / 64 + 3) / 4;
};
// backward tiling: RC = 8 lanes split the member's rows, OT hidden outputs per lane
template <int H, int G>
struct GruBwdCfg {
  static constexpr int U = H / G, R = 3 * U, RC = 8, RL = R / RC;
  static constexpr int OT = (G > 1) ? 4 : 1;
  static constexpr int NT = RC * H / OT;
  static constexpr int WPS = (NT / 64 + 3) / 4;
};

template <int H, int G, int BS>
constexpr bool gru_tile_ok() {
  return BS * (H / G) <= GruFwdCfg<H, G>::NT && BS * (H / G) <= GruBwdCfg<H, G>::NT;
}

template <int H, int G, int BS>
__global__ __launch_bounds__((GruFwdCfg<H, G>::NT), (GruFwdCfg<H, G>::WPS)) void gru_fwd_kernel(GruFwdArgs P) {
  using C = GruFwdCfg<H, G>;
  constexpr int NT = C::NT, U = C::U, R = C::R, KC = C::KC, KL = C::KL, RT = C::RT;
  constexpr bool SOLO = G == 1;
  constexpr int KLP = ((KL / 4) % 2 == 0) ? KL + 4 : KL;
  static_assert((KL % 4) == 0 && RT * NT == R * KC && BS * U <= NT, "bad GRU tiling");
  __shared__ __attribute__((aligned(16))) float hs[BS][KC][KLP];
  __shared__ float pre[BS][R];
  constexpr int CW = (BS * U + 63) / 64;
  constexpr int GOFF = (CW * 64 < NT) ? CW * 64 : 0;
  constexpr int GT = NT - GOFF;
  constexpr int NG = (BS * H + GT - 1) / GT;

  int prob, grp, j;
  const int ngroups = (P.B + BS - 1) / BS;
  decompose(G, ngroups, 1, prob, grp, j);
  const int B = P.B, T = P.T, tid = threadIdx.x, b0 = grp * BS;
  bool dead = false;

  const int rg = tid / KC, kc = tid % KC;
  float w[RT][KL];
#pragma unroll
  for (int q = 0; q < RT; ++q) {
    const int r = rg * RT + q;
    const int grow = (r / U) * H + j * U + (r % U);
#pragma unroll
    for (int i = 0; i < KL; i += 4) {
      float4 v = *reinterpret_cast<const float4*>(P.w_hh + (long)grow * H + kc * KL + i);
      w[q][i] = v.x; w[q][i + 1] = v.y; w[q][i + 2] = v.z; w[q][i + 3] = v.w;
    }
  }
  const bool cell = tid < BS * U;
  const int cb = tid / U, cu = tid % U, bg = b0 + cb;
  const bool cvalid = cell && bg < B;
  const int hcol = j * U + cu;
  float h = 0.0f, bh[3] = {0.f, 0.f, 0.f};
  if (cvalid) {
#pragma unroll
    for (int q = 0; q < 3; ++q) bh[q] = P.b_hh[q * H + hcol];
    if (P.h0) h = P.h0[(long)bg * H + hcol];
  }
  for (int e = tid; e < BS * H; e += NT) {
    const int b = e / H, k = e % H;
    hs[b][k / KL][k % KL] = (P.h0 && b0 + b < B) ? P.h0[(long)(b0 + b) * H + k] : 0.0f;
  }
  float gxv[3] = {0.f, 0.f, 0.f};
  auto load_gx = [&](int t) {
    if (cvalid) {
      const float* g = P.gx + (long)bg * P.gx_bs + (long)t * P.gx_ts + hcol;
#pragma unroll
      for (int q = 0; q < 3; ++q) gxv[q] = g[q * H];
    }
  };
  load_gx(P.reverse ? T - 1 : 0);
  __syncthreads();
  unsigned long long* xb = P.xbuf;
  __shared__ int xcc_flag;
  const int local = (P.local && G > 1) ? group_on_one_xcd<G>(xb + ((long)B + b0) * H, j, P.err, dead, &xcc_flag) : 0;

  for (int tt = 0; tt < T; ++tt) {
    const int t = P.reverse ? T - 1 - tt : tt;
#pragma unroll
    for (int b = 0; b < BS; ++b) {
      float acc[RT];
#pragma unroll
      for (int q = 0; q < RT; ++q) acc[q] = 0.0f;
      const float* hp = &hs[b][kc][0];
#pragma unroll
      for (int i = 0; i < KL; i += 4) {
        float4 hv = *reinterpret_cast<const float4*>(hp + i);
#pragma unroll
        for (int q = 0; q < RT; ++q) {
          acc[q] = fmaf(w[q][i], hv.x, acc[q]);
          acc[q] = fmaf(w[q][i + 1], hv.y, acc[q]);
          acc[q] = fmaf(w[q][i + 2], hv.z, acc[q]);
          acc[q] = fmaf(w[q][i + 3], hv.w, acc[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < RT; ++q) acc[q] = group_sum<KC>(acc[q]);
      if (kc == 0) {
#pragma unroll
        for (int q = 0; q < RT; ++q) pre[b][rg * RT + q] = acc[q];
      }
    }
    __syncthreads();
    const int par = tt & 1;
    if (cvalid) {
      const float r = sigmoidf_(gxv[0] + pre[cb][cu] + bh[0]);
      const float z = sigmoidf_(gxv[1] + pre[cb][U + cu] + bh[1]);
      const float hn = pre[cb][2 * U + cu] + bh[2];
      const float n = tanhf_(gxv[2] + r * hn);
      h = (1.0f - z) * n + z * h;
      if constexpr (SOLO) {
        hs[cb][cu / KL][cu % KL] = h;   // after the GEMV's reads (barrier above), before the next (below)
      } else {
        put_granule(xb + ((long)par * B + bg) * H + hcol, (unsigned)(tt + 1), h, local);
      }
      P.y[(long)bg * P.y_bs + (long)t * P.y_ts + hcol] = h;
      float* gs = P.gates + (long)bg * P.g_bs + (long)t * P.g_ts + hcol;
      gs[0] = r; gs[H] = z; gs[2 * H] = n;
      P.ghn[(long)bg * P.n_bs + (long)t * P.n_ts + hcol] = hn;
      if (tt + 1 < T) load_gx(P.reverse ? t - 1 : t + 1);
    }
    if (!SOLO && tt + 1 < T && tid >= GOFF) {
      const int gt = tid - GOFF;
      const int nvalid = min(BS, B - b0) * H;
      unsigned long long* rb = xb + ((long)par * B + b0) * H;
      float gv[NG];
      int idx[NG];
#pragma unroll
      for (int i = 0; i < NG; ++i) idx[i] = min(gt + i * GT, nvalid - 1);
      get_granules_idx<NG>(rb, idx, (unsigned)(tt + 1), gv, P.err, dead);
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        const int e = gt + i * GT;
        if (e < BS * H) {
          const int b = e / H, k = e % H;
          hs[b][k / KL][k % KL] = (b0 + b < B) ? gv[i] : 0.0f;
        }
      }
    }
    __syncthreads();
  }
}

// Backward with the LSTM backward's division of labour (lstm.hip): the cell threads only poll the
// hand-offs and run the cell; io shadow threads in the waves the cells do not use move the saved
// values HBM -> LDS two steps ahead and write dgx / dgh, so a cell wave's single vmcnt only ever
// covers its own polls (gfx9 counts loads and stores together).  Batch tiles whose cells fill the
// workgroup (no spare waves) let the cells move their own values (SELF_IO).
template <int H, int G, int BS>
__global__ __launch_bounds__((GruBwdCfg<H, G>::NT), (GruBwdCfg<H, G>::WPS)) void gru_bwd_kernel(GruBwdArgs P) {
  using C = GruBwdCfg<H, G>;
  constexpr int NT = C::NT, U = C::U, RC = C::RC, RL = C::RL, OT = C::OT;
  constexpr bool SOLO = G == 1;
  constexpr int RLP = ((RL / 4) % 2 == 0) ? RL + 4 : RL;
  static_assert(OT >= 1 && OT <= RC && OT * NT == RC * H && (RL % 4) == 0 && BS * U <= NT && (U % OT) == 0,
                "bad GRU bwd tiling");
  __shared__ __attribute__((aligned(16))) float dgl[BS][RC][RLP];   // dgh rows of the step (GEMV operand)
  __shared__ float dxn[BS * U];                                     // dgx's n column (dgh's is dn' r)
  __shared__ float sv[2][6][BS * U];   // r, z, n, hn, h_prev, dy of the cells, by step parity
  __shared__ float dhs[SOLO ? BS : 1][SOLO ? H : 1];
  constexpr int CW = (BS * U + 63) / 64;
  constexpr bool SELF_IO = CW * 64 + BS * U > NT;
  constexpr int IOFF = SELF_IO ? 0 : CW * 64;

  int prob, grp, j;
  const int ngroups = (P.B + BS - 1) / BS;
  decompose(G, ngroups, 1, prob, grp, j);
  const int B = P.B, T = P.T, tid = threadIdx.x, b0 = grp * BS;
  bool dead = false;

  const int ogr = tid / RC, rc = tid % RC;
  float w[OT][RL];
#pragma unroll
  for (int i = 0; i < RL; ++i) {
    const int rr = rc * RL + i;
    const int grow = (rr / U) * H + j * U + (rr % U);
#pragma unroll
    for (int o = 0; o < OT; ++o) w[o][i] = P.w_hh[(long)grow * H + ogr * OT + o];
  }
  const bool cell = tid < BS * U;
  const int cb = tid / U, cu = tid % U, bg = b0 + cb;
  const bool cvalid = cell && bg < B;
  const int hcol = j * U + cu;
  float direct = 0.0f;   // dh_{t+1} z_{t+1} of this cell's unit, carried in processing order
  float dhrec = 0.0f;
  if (cvalid && P.dhT) dhrec = P.dhT[(long)bg * H + hcol];

  // io role: the shadow of cell (ib, iu)
  const int iot = tid - IOFF;
  const bool io = iot >= 0 && iot < BS * U;
  const int ib = io ? iot / U : 0, iu = iot % U, ibg = b0 + ib;
  const bool iovalid = io && ibg < B;
  const int iocol = j * U + iu;
  float pf[6];
  auto io_load = [&](int tt2) {   // saved values of processing step tt2 -> pf
    if (!iovalid || tt2 >= T) return;
    const int t = P.reverse ? tt2 : T - 1 - tt2;
    const int tp = P.reverse ? t + 1 : t - 1;
    const float* gs = P.gates + (long)ibg * P.g_bs + (long)t * P.g_ts + iocol;
    pf[0] = gs[0]; pf[1] = gs[H]; pf[2] = gs[2 * H];
    pf[3] = P.ghn[(long)ibg * P.n_bs + (long)t * P.n_ts + iocol];
    pf[4] = (tp >= 0 && tp < T) ? P.y[(long)ibg * P.y_bs + (long)tp * P.y_ts + iocol]
                                : (P.h0 ? P.h0[(long)ibg * H + iocol] : 0.0f);
    pf[5] = P.dy ? P.dy[(long)ibg * P.dy_bs + (long)t * P.dy_ts + iocol] : 0.0f;
  };
  auto io_stage = [&](int tt2) {   // pf -> the sv slot of step tt2
    if (!iovalid || tt2 >= T) return;
#pragma unroll
    for (int q = 0; q < 6; ++q) sv[tt2 & 1][q][iot] = pf[q];
  };
  io_load(0);
  io_stage(0);
  io_load(1);
  __syncthreads();

  unsigned long long* xb = P.xbuf;
  const long xstride_b = (long)G * H;   // per batch row: [dest G][src G][U]
  __shared__ int xcc_flag;
  const int local = (P.local && G > 1) ? group_on_one_xcd<G>(xb + ((long)B + b0) * xstride_b, j, P.err, dead,
                                                             &xcc_flag)
                                       : 0;
  for (int tt = 0; tt < T; ++tt) {
    const int t = P.reverse ? tt : T - 1 - tt;
    const int r0 = cu, r1 = U + cu, r2 = 2 * U + cu;
    if constexpr (!SELF_IO) {   // io waves stage / prefetch while the cells work (as lstm.hip's backward)
      io_stage(tt + 1);
      io_load(tt + 2);
    }
    if (cvalid) {
      if (tt > 0) {
        float s;
        if constexpr (SOLO) {
          s = dhs[cb][cu];
        } else {
          const int par = (tt - 1) & 1;
          unsigned long long* g = xb + ((long)par * B + bg) * xstride_b + (long)j * H + cu;
          float gv[G];
          get_granules<G>(g, U, (unsigned)tt, gv, P.err, dead);
          s = 0.0f;
#pragma unroll
          for (int src = 0; src < G; ++src) s += gv[src];
        }
        dhrec = s + direct;
      }
      const int sl = tt & 1;
      const float r = sv[sl][0][tid], z = sv[sl][1][tid], n = sv[sl][2][tid];
      const float hn = sv[sl][3][tid], hprev = sv[sl][4][tid];
      const float dh = sv[sl][5][tid] + dhrec;
      const float dn = dh * (1.0f - z);
      const float dz = dh * (hprev - n);
      const float dpn = dn * (1.0f - n * n);
      const float dr = dpn * hn;
      direct = dh * z;
      dgl[cb][r0 / RL][r0 % RL] = dr * r * (1.0f - r);
      dgl[cb][r1 / RL][r1 % RL] = dz * z * (1.0f - z);
      dgl[cb][r2 / RL][r2 % RL] = dpn * r;
      dxn[tid] = dpn;
    } else if (cell) {
      dgl[cb][r0 / RL][r0 % RL] = 0.0f;
      dgl[cb][r1 / RL][r1 % RL] = 0.0f;
      dgl[cb][r2 / RL][r2 % RL] = 0.0f;
      dxn[tid] = 0.0f;
    }
    __syncthreads();
    // partial dh_{t-1}[b][hout] = sum over this member's rows of dgh[b][row] W_hh[row][hout]
    const int par = tt & 1;
#pragma unroll
    for (int b = 0; b < BS; ++b) {
      float acc[OT];
#pragma unroll
      for (int o = 0; o < OT; ++o) acc[o] = 0.0f;
      const float* dp = &dgl[b][rc][0];
#pragma unroll
      for (int i = 0; i < RL; i += 4) {
        const float4 dv = *reinterpret_cast<const float4*>(dp + i);
#pragma unroll
        for (int o = 0; o < OT; ++o) {
          acc[o] = fmaf(dv.x, w[o][i], acc[o]);
          acc[o] = fmaf(dv.y, w[o][i + 1], acc[o]);
          acc[o] = fmaf(dv.z, w[o][i + 2], acc[o]);
          acc[o] = fmaf(dv.w, w[o][i + 3], acc[o]);
        }
      }
#pragma unroll
      for (int o = 0; o < OT; ++o) acc[o] = group_sum<RC>(acc[o]);
      if (rc < OT) {
        float v = acc[0];
#pragma unroll
        for (int o = 1; o < OT; ++o) v = (rc == o) ? acc[o] : v;
        const int hout = ogr * OT + rc;
        if constexpr (SOLO) {
          dhs[b][hout] = v;   // all reads of dhs this step were before the barrier above
        } else if (b0 + b < B) {
          const int dest = hout / U, du = hout % U;
          put_granule(xb + ((long)par * B + b0 + b) * xstride_b + (long)dest * H + (long)j * U + du,
                      (unsigned)(tt + 1), v, local);
        }
      }
    }
    if (iovalid) {
      // dgx / dgh of this step (still in LDS until the barrier), then stage step tt+1, prefetch tt+2
      const int ir0 = iu, ir1 = U + iu, ir2 = 2 * U + iu;
      const float gr = dgl[ib][ir0 / RL][ir0 % RL], gz = dgl[ib][ir1 / RL][ir1 % RL];
      float* ox = P.dgx + (long)ibg * P.d_bs + (long)t * P.d_ts + iocol;
      float* oh = P.dgh + (long)ibg * P.d_bs + (long)t * P.d_ts + iocol;
      ox[0] = gr; ox[H] = gz; ox[2 * H] = dxn[iot];
      oh[0] = gr; oh[H] = gz; oh[2 * H] = dgl[ib][ir2 / RL][ir2 % RL];
      if constexpr (SELF_IO) {
        io_stage(tt + 1);
        io_load(tt + 2);
      }
    }
    __syncthreads();
  }
  if (cvalid && P.dh0) {
    float s;
    if constexpr (SOLO) {
      s = dhs[cb][cu];
    } else {
      const int par = (T - 1) & 1;
      unsigned long long* g = xb + ((long)par * B + bg) * xstride_b + (long)j * H + cu;
      float gv[G];
      get_granules<G>(g, U, (unsigned)T, gv, P.err, dead);
      s = 0.0f;
#pragma unroll
      for (int src = 0; src < G; ++src) s += gv[src];
    }
    P.dh0[(long)bg * H + hcol] = s + direct;
  }
}

// ring size at H = 256: 4 members (U = 64, 768 / 512 threads) by default, measured 0.7-1.0 ms faster
// on the GRU config than 8 (U = 32; profiles/r04_gru_persistent.txt); MRG_GRU_GROUP256=8 or
// mrg_gru_config(8) selects 8
static int g_gru_group256 = [] {
  const char* e = getenv("MRG_GRU_GROUP256");
  return (e && atoi(e) == 8) ? 8 : 4;
}();

static int gru_group(int H) {
  switch (H) {
    case 256: return g_gru_group256;
    case 128: case 64: case 32: return 1;
    default: return 0;
  }
}

// launch at batch tile BS when the grid fits the GPU at once; a solo group (no hand-offs, no
// co-residency requirement) also launches at its last candidate tile when none fits
template <typename K, typename A>
static bool gru_try(K kernel, int nt, long nblk, int cus, bool solo_last, hipStream_t s, const A& a) {
  if (!fits(kernel, nt, nblk, cus) && !solo_last) return false;
  klaunch(kernel, nblk, nt, 0, s, a);
  return true;
}

template <int H, int G>
static int gru_launch_fwd(const GruFwdArgs& a, int cus, hipStream_t s) {
  constexpr int NT = GruFwdCfg<H, G>::NT;
  constexpr int BMAX = gru_tile_ok<H, G, 8>() ? 8 : gru_tile_ok<H, G, 4>() ? 4 : 2;
  for (int bs = 1; bs <= BMAX; bs *= 2) {
    const long nblk = (long)((a.B + bs - 1) / bs) * G;
    const bool sl = G == 1 && bs == BMAX;
    bool ok = false;
    switch (bs) {
      case 1: ok = gru_try(gru_fwd_kernel<H, G, 1>, NT, nblk, cus, sl, s, a); break;
      case 2: ok = gru_try(gru_fwd_kernel<H, G, 2>, NT, nblk, cus, sl, s, a); break;
      case 4: if constexpr (gru_tile_ok<H, G, 4>()) ok = gru_try(gru_fwd_kernel<H, G, 4>, NT, nblk, cus, sl, s, a); break;
      default: if constexpr (gru_tile_ok<H, G, 8>()) ok = gru_try(gru_fwd_kernel<H, G, 8>, NT, nblk, cus, sl, s, a); break;
    }
    if (ok) return check_launch("gru_fwd_kernel");
  }
  set_error("gru fwd: persistent grid does not fit the GPU (B=%d H=%d)", a.B, H);
  return 4;
}

template <int H, int G>
static int gru_launch_bwd(const GruBwdArgs& a, int cus, hipStream_t s) {
  constexpr int NT = GruBwdCfg<H, G>::NT;
  constexpr int BMAX = gru_tile_ok<H, G, 8>() ? 8 : gru_tile_ok<H, G, 4>() ? 4 : 2;
  for (int bs = 1; bs <= BMAX; bs *= 2) {
    const long nblk = (long)((a.B + bs - 1) / bs) * G;
    const bool sl = G == 1 && bs == BMAX;
    bool ok = false;
    switch (bs) {
      case 1: ok = gru_try(gru_bwd_kernel<H, G, 1>, NT, nblk, cus, sl, s, a); break;
      case 2: ok = gru_try(gru_bwd_kernel<H, G, 2>, NT, nblk, cus, sl, s, a); break;
      case 4: if constexpr (gru_tile_ok<H, G, 4>()) ok = gru_try(gru_bwd_kernel<H, G, 4>, NT, nblk, cus, sl, s, a); break;
      default: if constexpr (gru_tile_ok<H, G, 8>()) ok = gru_try(gru_bwd_kernel<H, G, 8>, NT, nblk, cus, sl, s, a); break;
    }
    if (ok) return check_launch("gru_bwd_kernel");
  }
  set_error("gru bwd: persistent grid does not fit the GPU (B=%d H=%d)", a.B, H);
  return 4;
}

}  // namespace mrg

using namespace mrg;

MRG_API int mrg_gru_supported_hidden(int H) { return gru_group(H) > 0; }

MRG_API int mrg_gru_config(int group256) {
  MRG_REQUIRE(group256 == 4 || group256 == 8, "mrg_gru_config: group must be 4 or 8");
  const int prev = g_gru_group256;
  g_gru_group256 = group256;
  return prev;
}

// hand-off ring bytes of one persistent GRU launch (fwd and bwd), zeroed by the caller before each
MRG_API size_t mrg_gru_xbuf_bytes(int B, int H) {
  const int G = H == 256 ? 8 : gru_group(H);   // the largest ring a launch may take
  return (size_t)2 * B * (G > 0 ? G : 1) * H * 8;
}

MRG_API int mrg_gru_fwd(int B, int T, int H, const float* gx, long gx_bs, long gx_ts, const float* w_hh,
                        const float* b_hh, const float* h0, float* y, long y_bs, long y_ts, float* gates, long g_bs,
                        long g_ts, float* ghn, long n_bs, long n_ts, int reverse, void* xbuf, int* err, int cus,
                        hipStream_t stream) {
  const int G = gru_group(H);
  MRG_REQUIRE(G > 0, "mrg_gru_fwd: unsupported hidden size %d (256 / 128 / 64 / 32)", H);
  MRG_REQUIRE(((uintptr_t)w_hh & 15) == 0, "mrg_gru_fwd: w_hh must be 16-byte aligned");
  if (B == 0 || T == 0) return 0;
  GruFwdArgs a;
  memset(&a, 0, sizeof(a));
  a.gx = gx; a.gx_bs = gx_bs; a.gx_ts = gx_ts; a.w_hh = w_hh; a.b_hh = b_hh; a.h0 = h0;
  a.y = y; a.y_bs = y_bs; a.y_ts = y_ts; a.gates = gates; a.g_bs = g_bs; a.g_ts = g_ts;
  a.ghn = ghn; a.n_bs = n_bs; a.n_ts = n_ts; a.xbuf = (unsigned long long*)xbuf;
  a.B = B; a.T = T; a.reverse = reverse ? 1 : 0; a.local = 1; a.err = err;
  if (cus <= 0) cus = device_cus();
  switch (H) {
    case 256: return G == 4 ? gru_launch_fwd<256, 4>(a, cus, stream) : gru_launch_fwd<256, 8>(a, cus, stream);
    case 128: return gru_launch_fwd<128, 1>(a, cus, stream);
    case 64: return gru_launch_fwd<64, 1>(a, cus, stream);
    default: return gru_launch_fwd<32, 1>(a, cus, stream);
  }
}

MRG_API int mrg_gru_bwd(int B, int T, int H, const float* w_hh, const float* gates, long g_bs, long g_ts,
                        const float* ghn, long n_bs, long n_ts, const float* y, long y_bs, long y_ts,
                        const float* h0, const float* dy, long dy_bs, long dy_ts, const float* dhT, float* dgx,
                        float* dgh, long d_bs, long d_ts, float* dh0, int reverse, void* xbuf, int* err, int cus,
                        hipStream_t stream) {
  const int G = gru_group(H);
  MRG_REQUIRE(G > 0, "mrg_gru_bwd: unsupported hidden size %d (256 / 128 / 64 / 32)", H);
  if (B == 0 || T == 0) return 0;
  GruBwdArgs a;
  memset(&a, 0, sizeof(a));
  a.w_hh = w_hh; a.gates = gates; a.g_bs = g_bs; a.g_ts = g_ts; a.ghn = ghn; a.n_bs = n_bs; a.n_ts = n_ts;
  a.y = y; a.y_bs = y_bs; a.y_ts = y_ts; a.h0 = h0; a.dy = dy; a.dy_bs = dy_bs; a.dy_ts = dy_ts; a.dhT = dhT;
  a.dgx = dgx; a.dgh = dgh; a.d_bs = d_bs; a.d_ts = d_ts; a.dh0 = dh0; a.xbuf = (unsigned long long*)xbuf;
  a.B = B; a.T = T; a.reverse = reverse ? 1 : 0; a.local = 1; a.err = err;
  if (cus <= 0) cus = device_cus();
  switch (H) {
    case 256: return G == 4 ? gru_launch_bwd<256, 4>(a, cus, stream) : gru_launch_bwd<256, 8>(a, cus, stream);
    case 128: return gru_launch_bwd<128, 1>(a, cus, stream);
    case 64: return gru_launch_bwd<64, 1>(a, cus, stream);
    default: return gru_launch_bwd<32, 1>(a, cus, stream);
  }
}
