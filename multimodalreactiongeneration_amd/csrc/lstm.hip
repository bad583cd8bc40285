// Persistent LSTM recurrence for gfx950 (replaces the cuDNN RNN that nn.LSTM
// lowers to in the reference: LSTMMixer mixer_block.py:237-252, LSTMModule
// lstm_block.py:21-46, LSTMSampler lstm_sampler.py:16-34).
//
// Split of the work (host side, multimodalreactiongeneration_amd/functional.py):
//   Gx = X W_ih^T + b_ih            MFMA GEMM over all B*T rows   (gemm.hip)
//   recurrence over t               THIS FILE, one launch per layer (or per
//                                   batch of independent same-shape layers)
//   dW_ih, dW_hh, dX, db            MFMA GEMMs / column sums over dG
//
// Recurrence layout.  The batch is cut into groups of BS rows; each group is
// served by G workgroups ("members") that each own U = H/G hidden units, i.e.
// R = 4U rows of W_hh (gate order i, f, g, o), held in VGPRs for the whole
// sequence (W_hh is read from HBM once per launch).  Per step a member
//   1. computes pre[b][r] = sum_k h_{t-1}[b][k] W_hh[r][k] for its R rows
//      (VALU fp32 FMA: at fp32 the VALU and the f32 MFMA both run 64 FLOP/clk/
//      SIMD, and the per-group GEMV has only BS <= 8 columns, so a 16/32-wide
//      MFMA tile would idle 2-32x of its lanes),
//   2. applies the gate nonlinearities + cell update for its BS x U cells,
//   3. publishes its h_t slice as 8-byte {tag, value} granules written by ONE
//      agent-scope (sc1) store each, and
//   4. gathers the full h_t of its group by polling the granules with
//      agent-scope loads (no fences: the data is the flag; recipe R2 of
//      cdna_hip_programming.md Guideline 16).  Tags are step+1 and a 2-deep
//      parity ring makes slot reuse safe; the ring is zeroed per launch.
// Group members are placed on one XCD (blocks b and b+8 share an XCD under
// the observed round-robin dispatch) so hand-offs stay in that XCD's L2;
// placement affects speed only, never correctness.  Every spin is bounded and
// reports through *err.
//
// Solo groups (G = 1, H <= 128, the default there: mrg_lstm_set_solo): one workgroup holds all of
// W_hh (at H = 128, 1024 threads x 64 values) and exchanges h / dh through its LDS, so a step has no
// hand-off through L2 and the workgroups of a launch never wait on each other (no co-residency
// requirement: a grid larger than the GPU still completes).
//
// Backward runs the same decomposition in reverse time: a member owns the
// same U units, computes dG for them, then the partial products
// P_j[b][:] = dG_j[b] W_hh[rows_j, :] over ALL H outputs; the exchange is a
// reduce-scatter (each member sums the G partials of its own units), so the
// bytes moved per step equal the forward's (BS x H granules per member).
#include "lstm_common.h"
#include <cstdlib>

namespace mrg {

// Threads per workgroup and resident workgroups per CU for a (hidden size, group size):
//   H = 256, G = 8  : 512 threads (64 W_hh values per lane), 2 workgroups per CU
//   H = 256, G = 16 : 256 threads (64 W_hh values per lane), 4 workgroups per CU
//   H = 256, G = 4  : 1024 threads (64 W_hh values per lane), 1 workgroup per CU
//   H <= 128        : 256 threads, 2 workgroups per CU
// waves_per_simd bounds VGPRs at 512 / waves (128 here) so the whole grid stays resident.
//   H = 128, G = 1  : 1024 threads (64 W_hh values per lane), 1 workgroup per CU (a "solo" group)
template <int H, int G>
struct LstmNT {
  static constexpr int value = ((G == 1 && H == 128) || (G == 4 && H == 256)) ? 1024
                               : (H >= 256 && H / G >= 32)                    ? 512
                                                                              : 256;
  static constexpr int waves_per_simd = (H >= 256 || value == 1024) ? 4 : 2;
};

// batch tiles a (H, G) kernel can hold (every cell thread in the block)
template <int H, int G, int BS>
constexpr bool tile_ok() { return BS * (H / G) <= LstmNT<H, G>::value && (G > 1 || H < 128 || BS <= 8); }

template <int H, int G, int BS>
__global__ __launch_bounds__((LstmNT<H, G>::value), (LstmNT<H, G>::waves_per_simd)) void lstm_fwd_kernel(LstmFwdArgs args) {
  constexpr int NT = LstmNT<H, G>::value;
  constexpr int U = H / G;
  constexpr int R = 4 * U;
  constexpr bool SOLO = G == 1;
  // register blocking of the recurrent GEMV: a thread owns RT gate rows x KL hidden inputs, the
  // KC lanes of a row group split the hidden dimension (DPP-reduced), so every h value read from
  // LDS feeds RT FMAs (the GEMV is LDS-issue bound otherwise)
  // (KC = 8 lanes x 2 rows measured fastest at H = 256: 3 DPP levels, 128-B LDS reads per lane; 16 x 4
  // at batch tiles >= 4 (half the LDS reads of h, one more DPP level) measured 5-23 % slower, r03)
  // (solo groups at H = 128: 8 lanes x 4 rows, half the LDS reads of h per FMA of 4 x 2)
  constexpr int KC = (SOLO && H == 128) ? 8 : (H >= 128) ? (2 * NT / R) : ((H / 4 < 16) ? H / 4 : 16);
  constexpr int RT = R * KC / NT;
  constexpr int KL = H / KC;
  constexpr int KLP = ((KL / 4) % 2 == 0) ? KL + 4 : KL;  // odd 16-B chunk pitch: conflict-free b128
  static_assert(RT >= 1 && RT * NT == R * KC && (KL % 4) == 0 && BS * U <= NT, "bad LSTM tiling");
  __shared__ __attribute__((aligned(16))) float hs[BS][KC][KLP];
  __shared__ float pre[BS][R];
  // cell threads occupy the first CW waves; the rest gather (all threads if the cells fill the block)
  constexpr int CW = (BS * U + 63) / 64;
  constexpr int GOFF = (CW * 64 < NT) ? CW * 64 : 0;
  constexpr int GT = NT - GOFF;
  constexpr int NG = (BS * H + GT - 1) / GT;

  int prob, grp, j;
  const int ngroups = (args.B + BS - 1) / BS;
  decompose(G, ngroups, args.nprob, prob, grp, j);
  const LstmFwdProblem& P = args.p[prob];
  const int B = args.B, T = args.T;
  const int tid = threadIdx.x;
  const int b0 = grp * BS;
  bool dead = false;

  // dot role: row group rg (rows rg*RT .. +RT-1), k-chunk kc
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

  // cell role
  const bool cell = tid < BS * U;
  const int cb = tid / U, cu = tid % U;
  const int bg = b0 + cb;
  const bool cvalid = cell && bg < B;
  const int hcol = j * U + cu;
  float c = 0.0f, h = 0.0f;
  float bh[4] = {0.f, 0.f, 0.f, 0.f};
  if (cvalid) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bh[q] = P.b_hh[q * H + hcol];
    if (P.c0) c = P.c0[(long)bg * P.c0_bs + hcol];
  }

  // initial h_{-1}
  for (int e = tid; e < BS * H; e += NT) {
    int b = e / H, k = e % H;
    float v = 0.0f;
    if (P.h0 && b0 + b < B) v = P.h0[(long)(b0 + b) * P.h0_bs + k];
    hs[b][k / KL][k % KL] = v;
  }
  float gxv[4] = {0.f, 0.f, 0.f, 0.f};
  auto load_gx = [&](int t) {
    if (cvalid) {
      const float* g = P.gx + (long)bg * P.gx_bs + (long)t * P.gx_ts + hcol;
#pragma unroll
      for (int q = 0; q < 4; ++q) gxv[q] = g[q * H];
    }
  };
  load_gx(P.reverse ? T - 1 : 0);
  __syncthreads();

  unsigned long long* xb = P.xbuf;
  __shared__ int xcc_flag;
  const int local = (args.local && G > 1) ? group_on_one_xcd<G>(xb + ((long)B + b0) * H, j, args.err, dead, &xcc_flag)
                                          : 0;
  for (int tt = 0; tt < T; ++tt) {
    const int t = P.reverse ? T - 1 - tt : tt;
    MRG_STAMP(0);
    // 1. recurrent GEMV for this member's R gate rows, one batch row at a time (short live ranges)
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
      if (b == 0) MRG_STAMP(1);
#pragma unroll
      for (int q = 0; q < RT; ++q) acc[q] = group_sum<KC>(acc[q]);
      if (kc == 0) {
#pragma unroll
        for (int q = 0; q < RT; ++q) pre[b][rg * RT + q] = acc[q];
      }
    }
    MRG_STAMP(2);
    __syncthreads();
    MRG_STAMP(3);
    // 2. gates + cell update, 3. publish
    const int par = tt & 1;
    if (cvalid) {
      float zi = pre[cb][0 * U + cu] + gxv[0] + bh[0];
      float zf = pre[cb][1 * U + cu] + gxv[1] + bh[1];
      float zg = pre[cb][2 * U + cu] + gxv[2] + bh[2];
      float zo = pre[cb][3 * U + cu] + gxv[3] + bh[3];
      float ig = sigmoidf_(zi), fg = sigmoidf_(zf), gg = tanhf_(zg), og = sigmoidf_(zo);
      c = fg * c + ig * gg;
      h = og * tanhf_(c);
      if constexpr (SOLO) {
        hs[cb][cu / KL][cu % KL] = h;   // after the GEMV's reads (barrier above), before the next (below)
      } else if (!(args.inject == 1 && j == 0 && tt == 0)) {
        put_granule(xb + ((long)par * B + bg) * H + hcol, (unsigned)(tt + 1), h, local);
      }
      P.y[(long)bg * P.y_bs + (long)t * P.y_ts + hcol] = h;
      float* gs = P.gates + (long)bg * P.g_bs + (long)t * P.g_ts + hcol;
      gs[0] = ig; gs[H] = fg; gs[2 * H] = gg; gs[3 * H] = og;
      P.cs[(long)bg * P.cs_bs + (long)t * P.cs_ts + hcol] = c;
      if (tt + 1 < T) load_gx(P.reverse ? t - 1 : t + 1);
    }
    MRG_STAMP(4);
    // 4. gather h_t of the whole group.  Done by the waves after the cell waves: on gfx9 one vmcnt
    // covers loads and stores, so a wave that just issued the y/gates/cs stores and the gx prefetch
    // would wait for all of them before its first poll returned.
    if (!SOLO && tt + 1 < T && tid >= GOFF) {
      const int gt = tid - GOFF;
      const int nvalid = min(BS, B - b0) * H;
      unsigned long long* rb = xb + ((long)par * B + b0) * H;
      float gv[NG];
      int idx[NG];
#pragma unroll
      for (int i = 0; i < NG; ++i) idx[i] = min(gt + i * GT, nvalid - 1);
      get_granules_idx<NG>(rb, idx, (unsigned)(tt + 1), gv, args.err, dead);
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        int e = gt + i * GT;
        if (e < BS * H) {
          int b = e / H, k = e % H;
          hs[b][k / KL][k % KL] = (b0 + b < B) ? gv[i] : 0.0f;
        }
      }
    }
    MRG_STAMP(5);
    __syncthreads();
    MRG_STAMP(6);
  }
  if (cvalid) {
    if (P.hT) P.hT[(long)bg * H + hcol] = h;
    if (P.cT) P.cT[(long)bg * H + hcol] = c;
  }
}

template <int H, int G, int BS>
__global__ __launch_bounds__((LstmNT<H, G>::value), (LstmNT<H, G>::waves_per_simd)) void lstm_bwd_kernel(LstmBwdArgs args) {
  constexpr int NT = LstmNT<H, G>::value;
  constexpr int U = H / G;
  constexpr int R = 4 * U;
  constexpr bool SOLO = G == 1;
  // a thread owns OT consecutive outputs (hidden units of dh_{t-1}) x RL gate rows; the RC lanes of
  // an output group split the rows (DPP-reduced): each dG value read from LDS feeds OT FMAs
  constexpr int RC = (H >= 128 && !SOLO) ? 8 : 16;
  constexpr int OT = RC * H / NT;
  constexpr int RL = R / RC;
  constexpr int RLP = ((RL / 4) % 2 == 0) ? RL + 4 : RL;
  static_assert(OT >= 1 && OT <= RC && OT * NT == RC * H && RL * RC == R && (RL % 4) == 0 && BS * U <= NT &&
                (U % OT) == 0, "bad LSTM bwd tiling");
  __shared__ __attribute__((aligned(16))) float dgl[BS][RC][RLP];
  __shared__ float sv[2][7][BS * U];  // saved i, f, g, o, c_t, c_{t-1}, dy of the cells, by step parity
  __shared__ float dhs[SOLO ? BS : 1][SOLO ? H : 1];  // solo: dh_{t-1} of the step, summed in place
  constexpr int CW = (BS * U + 63) / 64;
  // no spare waves for the io role at the largest batch tiles: the cell threads then move their own
  // saved activations (same schedule: stage step tt+1, prefetch tt+2, after the step's GEMV)
  constexpr bool SELF_IO = CW * 64 + BS * U > NT;
  constexpr int IOFF = SELF_IO ? 0 : CW * 64;  // first io thread

  int prob, grp, j;
  const int ngroups = (args.B + BS - 1) / BS;
  decompose(G, ngroups, args.nprob, prob, grp, j);
  const LstmBwdProblem& P = args.p[prob];
  const int B = args.B, T = args.T;
  const int tid = threadIdx.x;
  const int b0 = grp * BS;
  bool dead = false;

  // dot role: w[o][i] = W_hh[grow(rc*RL + i)][ogr*OT + o]
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
  const int cb = tid / U, cu = tid % U;
  const int bg = b0 + cb;
  const bool cvalid = cell && bg < B;
  const int hcol = j * U + cu;
  float dcn = 0.0f;  // dc_{t+1} * f_{t+1} carried in processing order
  float dhrec = 0.0f;
  if (cvalid) {
    if (P.dcT) dcn = P.dcT[(long)bg * H + hcol];
    if (P.dhT) dhrec = P.dhT[(long)bg * H + hcol];
  }

  // io role: a shadow thread per cell, in waves the cells do not use, moves the saved activations
  // HBM -> LDS two steps ahead and dG LDS -> HBM, so the cell waves' vmcnt only ever covers
  // hand-off traffic (gfx9 has one vmcnt for loads and stores).
  const int iot = tid - IOFF;
  const bool io = iot >= 0 && iot < BS * U;
  const int ib = io ? iot / U : 0, iu = iot % U;
  const int ibg = b0 + ib;
  const bool iovalid = io && ibg < B;
  const int iocol = j * U + iu;
  float pf[7];
  auto io_load = [&](int tt2) {  // saved values of processing step tt2 -> pf
    if (!iovalid || tt2 >= T) return;
    const int t = P.reverse ? tt2 : T - 1 - tt2;
    const int tp = P.reverse ? t + 1 : t - 1;
    const float* gs = P.gates + (long)ibg * P.g_bs + (long)t * P.g_ts + iocol;
    pf[0] = gs[0]; pf[1] = gs[H]; pf[2] = gs[2 * H]; pf[3] = gs[3 * H];
    pf[4] = P.cs[(long)ibg * P.cs_bs + (long)t * P.cs_ts + iocol];
    pf[5] = (tp >= 0 && tp < T) ? P.cs[(long)ibg * P.cs_bs + (long)tp * P.cs_ts + iocol]
                                : (P.c0 ? P.c0[(long)ibg * P.c0_bs + iocol] : 0.0f);
    pf[6] = P.dy ? P.dy[(long)ibg * P.dy_bs + (long)t * P.dy_ts + iocol] : 0.0f;
  };
  auto io_stage = [&](int tt2) {  // pf -> sv slot of step tt2
    if (!iovalid || tt2 >= T) return;
#pragma unroll
    for (int q = 0; q < 7; ++q) sv[tt2 & 1][q][iot] = pf[q];
  };
  io_load(0);
  io_stage(0);
  io_load(1);
  __syncthreads();

  unsigned long long* xb = P.xbuf;
  const long xstride_b = (long)G * H;  // per batch row: [dest G][src G][U]
  __shared__ int xcc_flag;
  const int local = (args.local && G > 1) ? group_on_one_xcd<G>(xb + ((long)B + b0) * xstride_b, j, args.err, dead,
                                                                &xcc_flag)
                                          : 0;
  for (int tt = 0; tt < T; ++tt) {
    const int t = P.reverse ? tt : T - 1 - tt;
    MRG_STAMP(0);
    if (cvalid) {
      if (tt > 0) {
        if constexpr (SOLO) {
          dhrec = dhs[cb][cu];
        } else {
          const int par = (tt - 1) & 1;
          unsigned long long* g = xb + ((long)par * B + bg) * xstride_b + (long)j * H + cu;
          float gv[G];
          get_granules<G>(g, U, (unsigned)tt, gv, args.err, dead);
          float s = 0.0f;
#pragma unroll
          for (int src = 0; src < G; ++src) s += gv[src];
          dhrec = s;
        }
      }
      MRG_STAMP(1);
      const int sl = tt & 1;
      const float ig = sv[sl][0][tid], fg = sv[sl][1][tid], gg = sv[sl][2][tid], og = sv[sl][3][tid];
      const float cc = sv[sl][4][tid], cp = sv[sl][5][tid], dyv = sv[sl][6][tid];
      const float dh = dhrec + dyv;
      const float tc = tanhf_(cc);
      const float dc = dh * og * (1.0f - tc * tc) + dcn;
      const float d_o = dh * tc * og * (1.0f - og);
      const float d_i = dc * gg * ig * (1.0f - ig);
      const float d_f = dc * cp * fg * (1.0f - fg);
      const float d_g = dc * ig * (1.0f - gg * gg);
      dcn = dc * fg;
      {
        const int r0 = 0 * U + cu, r1 = 1 * U + cu, r2 = 2 * U + cu, r3 = 3 * U + cu;
        dgl[cb][r0 / RL][r0 % RL] = d_i;
        dgl[cb][r1 / RL][r1 % RL] = d_f;
        dgl[cb][r2 / RL][r2 % RL] = d_g;
        dgl[cb][r3 / RL][r3 % RL] = d_o;
      }
      MRG_STAMP(2);
    } else if (cell) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = q * U + cu;
        dgl[cb][rr / RL][rr % RL] = 0.0f;
      }
    }
    __syncthreads();
    MRG_STAMP(3);
    // partial dh_{t-1}[b][hout] = sum over this member's rows of dG[b][row] * W_hh[row][hout]
    {
      const int par = tt & 1;
#pragma unroll
      for (int b = 0; b < BS; ++b) {  // one batch row at a time: short live ranges
        float acc[OT];
#pragma unroll
        for (int o = 0; o < OT; ++o) acc[o] = 0.0f;
        const float* dp = &dgl[b][rc][0];
#pragma unroll
        for (int i = 0; i < RL; i += 4) {
          float4 dv = *reinterpret_cast<const float4*>(dp + i);
#pragma unroll
          for (int o = 0; o < OT; ++o) {
            acc[o] = fmaf(dv.x, w[o][i], acc[o]);
            acc[o] = fmaf(dv.y, w[o][i + 1], acc[o]);
            acc[o] = fmaf(dv.z, w[o][i + 2], acc[o]);
            acc[o] = fmaf(dv.w, w[o][i + 3], acc[o]);
          }
        }
        if (b == 0) MRG_STAMP(4);
#pragma unroll
        for (int o = 0; o < OT; ++o) acc[o] = group_sum<RC>(acc[o]);
        // every lane of the RC group holds the sums: lanes rc < OT each publish granule o = rc, so
        // a wave's puts are contiguous 8-B granules in ONE store instruction (full 128-B lines)
        if constexpr (SOLO) {
          if (rc < OT) {   // all reads of dhs this step were before the barrier above
            float v = acc[0];
#pragma unroll
            for (int o = 1; o < OT; ++o) v = (rc == o) ? acc[o] : v;
            dhs[b][ogr * OT + rc] = v;
          }
        } else if (rc < OT && b0 + b < B && !(args.inject == 2 && j == 0 && tt == 0)) {
          const int h0 = ogr * OT;
          const int dest = h0 / U, du = h0 % U;
          float v = acc[0];
#pragma unroll
          for (int o = 1; o < OT; ++o) v = (rc == o) ? acc[o] : v;
          unsigned long long* gq = xb + ((long)par * B + b0 + b) * xstride_b + (long)dest * H + (long)j * U + du;
          put_granule(gq + rc, (unsigned)(tt + 1), v, local);
        }
      }
    }
    if (iovalid) {
      // dG of this step (still in dgl until the barrier), then stage step tt+1, prefetch tt+2
      float* dgp = P.dG + (long)ibg * P.dG_bs + (long)t * P.dG_ts + iocol;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rr = q * U + iu;
        dgp[q * H] = dgl[ib][rr / RL][rr % RL];
      }
      io_stage(tt + 1);
      io_load(tt + 2);
    }
    MRG_STAMP(5);
    __syncthreads();
    MRG_STAMP(6);
  }
  if (cvalid) {
    if (P.dh0) {
      if constexpr (SOLO) {
        P.dh0[(long)bg * H + hcol] = dhs[cb][cu];
      } else {
        const int par = (T - 1) & 1;
        unsigned long long* g = xb + ((long)par * B + bg) * xstride_b + (long)j * H + cu;
        float gv[G];
        get_granules<G>(g, U, (unsigned)T, gv, args.err, dead);
        float s = 0.0f;
#pragma unroll
        for (int src = 0; src < G; ++src) s += gv[src];
        P.dh0[(long)bg * H + hcol] = s;
      }
    }
    if (P.dc0) P.dc0[(long)bg * H + hcol] = dcn;
  }
}

int launch_fwd_mx(const LstmFwdArgs& a, int cus, hipStream_t s);   // lstm_mx.hip
int launch_bwd_mx(const LstmBwdArgs& a, int cus, hipStream_t s);

// MFMA form of the recurrence (lstm_mx.hip, H = 256, 8 members per group, batch tiles of 16):
// 0 = never, 1 = when the VALU form would need batch tiles >= MX_MIN_BS (default), 2 = whenever it fits
static int g_mx = [] {
  const char* e = getenv("MRG_LSTM_MX");
  return e ? atoi(e) : 1;
}();
static int g_mx_min_bs = [] {
  const char* e = getenv("MRG_LSTM_MX_MIN_BS");
  return e ? atoi(e) : 4;
}();
// the backward's own threshold (MRG_LSTM_MX_MIN_BS_BWD, default: the forward's)
static int g_mx_min_bs_bwd = [] {
  const char* e = getenv("MRG_LSTM_MX_MIN_BS_BWD");
  return e ? atoi(e) : 0;
}();

// batch tile the VALU launchers would pick (smallest fitting; 0 = none fits)
template <typename K1, typename K2, typename K4, typename K8, typename K16>
static int valu_bs(K1 k1, K2 k2, K4 k4, K8 k8, K16 k16, int nt, int nprob, int B, int G, int cus) {
  for (int bs = 1; bs <= 16; bs *= 2) {
    const long nblk = (long)nprob * ((B + bs - 1) / bs) * G;
    const bool ok = bs == 1 ? fits(k1, nt, nblk, cus) : bs == 2 ? fits(k2, nt, nblk, cus)
                  : bs == 4 ? fits(k4, nt, nblk, cus) : bs == 8 ? fits(k8, nt, nblk, cus) : fits(k16, nt, nblk, cus);
    if (ok) return bs;
  }
  return 0;
}

// one candidate batch tile: launch when it fits (or, for a solo group, when it is the last candidate:
// its workgroups never wait on each other, so a grid larger than the GPU still completes)
template <int BS, typename Args, typename K>
static bool try_tile(K kernel, int nt, long nblk, int cus, bool last_solo, hipStream_t s, const Args& a) {
  if (!fits(kernel, nt, nblk, cus) && !last_solo) return false;
  klaunch(kernel, nblk, nt, 0, s, a);
  return true;
}

template <int H, int G>
static int launch_fwd(const LstmFwdArgs& a, int force_bs, int cus, hipStream_t s) {
  constexpr int NT = LstmNT<H, G>::value;
  const long groups1 = a.B;
  if constexpr (H == 256 && G == 8) {
    if (g_mx && force_bs <= 0 && (!a.stamps || g_mx == 2)) {
      const int bs = valu_bs(lstm_fwd_kernel<H, G, 1>, lstm_fwd_kernel<H, G, 2>, lstm_fwd_kernel<H, G, 4>,
                             lstm_fwd_kernel<H, G, 8>, lstm_fwd_kernel<H, G, 16>, NT, a.nprob, a.B, G, cus);
      if (g_mx == 2 || bs == 0 || bs >= g_mx_min_bs) {
        const int r = launch_fwd_mx(a, cus, s);
        if (r != 0) return r < 0 ? 1 : 0;
      }
    }
  }
  constexpr int BMAX = tile_ok<H, G, 16>() ? 16 : tile_ok<H, G, 8>() ? 8 : tile_ok<H, G, 4>() ? 4 : 2;
  for (int bs = 1; bs <= BMAX; bs *= 2) {
    if (force_bs > 0 && bs != force_bs) continue;
    long nblk = (long)a.nprob * ((groups1 + bs - 1) / bs) * G;
    const bool last = G == 1 && (bs == BMAX || bs == force_bs);
    bool ok = false;
    switch (bs) {
      case 1: ok = try_tile<1>(lstm_fwd_kernel<H, G, 1>, NT, nblk, cus, last, s, a); break;
      case 2: ok = try_tile<2>(lstm_fwd_kernel<H, G, 2>, NT, nblk, cus, last, s, a); break;
      case 4: if constexpr (tile_ok<H, G, 4>()) ok = try_tile<4>(lstm_fwd_kernel<H, G, 4>, NT, nblk, cus, last, s, a); break;
      case 8: if constexpr (tile_ok<H, G, 8>()) ok = try_tile<8>(lstm_fwd_kernel<H, G, 8>, NT, nblk, cus, last, s, a); break;
      default: if constexpr (tile_ok<H, G, 16>()) ok = try_tile<16>(lstm_fwd_kernel<H, G, 16>, NT, nblk, cus, last, s, a); break;
    }
    if (ok) return check_launch("lstm_fwd_kernel");
  }
  set_error("lstm fwd: persistent grid does not fit the GPU (nprob=%d B=%d H=%d force_bs=%d)", a.nprob, a.B, H,
            force_bs);
  return 4;
}

static int g_bwd_blocks_per_cu = 0;  // cap on resident workgroups per CU (mrg_lstm_set_blocks_per_cu)

template <int H, int G>
static int launch_bwd(const LstmBwdArgs& a, int force_bs, int cus, hipStream_t s) {
  constexpr int NT = LstmNT<H, G>::value;
  // (the MFMA form runs one workgroup per CU, within a cap of one: mrg_lstm_set_blocks_per_cu)
  if constexpr (H == 256 && G == 8) {
    if (g_mx && force_bs <= 0 && (!a.stamps || g_mx == 2) && g_bwd_blocks_per_cu <= 1) {
      const int bs = valu_bs(lstm_bwd_kernel<H, G, 1>, lstm_bwd_kernel<H, G, 2>, lstm_bwd_kernel<H, G, 4>,
                             lstm_bwd_kernel<H, G, 8>, lstm_bwd_kernel<H, G, 16>, NT, a.nprob, a.B, G, cus);
      if (g_mx == 2 || bs == 0 || bs >= (g_mx_min_bs_bwd > 0 ? g_mx_min_bs_bwd : g_mx_min_bs)) {
        const int r = launch_bwd_mx(a, cus, s);
        if (r != 0) return r < 0 ? 1 : 0;
      }
    }
  }
  constexpr int BMAX = tile_ok<H, G, 16>() ? 16 : tile_ok<H, G, 8>() ? 8 : tile_ok<H, G, 4>() ? 4 : 2;
  for (int bs = 1; bs <= BMAX; bs *= 2) {
    if (force_bs > 0 && bs != force_bs) continue;
    long nblk = (long)a.nprob * ((a.B + bs - 1) / bs) * G;
    const bool last = G == 1 && (bs == BMAX || bs == force_bs);
    if (force_bs <= 0 && g_bwd_blocks_per_cu > 0 && bs < BMAX && nblk > (long)g_bwd_blocks_per_cu * cus) continue;
    bool ok = false;
    switch (bs) {
      case 1: ok = try_tile<1>(lstm_bwd_kernel<H, G, 1>, NT, nblk, cus, last, s, a); break;
      case 2: ok = try_tile<2>(lstm_bwd_kernel<H, G, 2>, NT, nblk, cus, last, s, a); break;
      case 4: if constexpr (tile_ok<H, G, 4>()) ok = try_tile<4>(lstm_bwd_kernel<H, G, 4>, NT, nblk, cus, last, s, a); break;
      case 8: if constexpr (tile_ok<H, G, 8>()) ok = try_tile<8>(lstm_bwd_kernel<H, G, 8>, NT, nblk, cus, last, s, a); break;
      default: if constexpr (tile_ok<H, G, 16>()) ok = try_tile<16>(lstm_bwd_kernel<H, G, 16>, NT, nblk, cus, last, s, a); break;
    }
    if (ok) return check_launch("lstm_bwd_kernel");
  }
  set_error("lstm bwd: persistent grid does not fit the GPU (nprob=%d B=%d H=%d force_bs=%d)", a.nprob, a.B, H,
            force_bs);
  return 4;
}

static int g_group256 = [] {  // members per group at H = 256 (4, 8 or 16), mrg_lstm_config / MRG_LSTM_GROUP256
  const char* e = getenv("MRG_LSTM_GROUP256");
  const int g = e ? atoi(e) : 8;
  return (g == 4 || g == 16) ? g : 8;
}();

// solo groups (G = 1) at H <= 128: MRG_LSTM_SOLO=0 / mrg_lstm_set_solo(0) restores the multi-member groups
static int g_solo = [] {
  const char* e = getenv("MRG_LSTM_SOLO");
  return (e && atoi(e) == 0) ? 0 : 1;
}();

// members per group without solo groups (the hand-off ring is sized for these)
// forward-only ring size at H = 256 (MRG_LSTM_GROUP256_FWD = 4 / 8 / 16; unset: the shared setting)
static int g_fwd_group256 = [] {
  const char* e = getenv("MRG_LSTM_GROUP256_FWD");
  const int g = e ? atoi(e) : 0;
  return (g == 4 || g == 8 || g == 16) ? g : 0;
}();

static int ring_group_size(int H) {
  switch (H) {
    case 256: return g_group256;
    case 128: return 8;
    case 64: return 4;
    case 32: return 2;
    case 16: return 1;
    default: return 0;
  }
}

static int group_size(int H) {
  const int g = ring_group_size(H);
  return (g > 0 && H <= 128 && g_solo) ? 1 : g;
}

}  // namespace mrg

using namespace mrg;

static unsigned long long* g_stamps = nullptr;
static int g_inject = 0;
static int g_local = [] {  // granule stores at workgroup scope (see put_granule); MRG_LSTM_LOCAL=0 disables
  const char* e = getenv("MRG_LSTM_LOCAL");
  return (e && atoi(e) == 0) ? 0 : 1;
}();

// Granule store scope of the recurrences' hand-offs: 1 = workgroup scope (line kept in L2), 0 = agent.
MRG_API int mrg_lstm_set_local_handoff(int on) {
  g_local = on ? 1 : 0;
  return 0;
}

// Tests only: arm a fault for the next forward launch (see mrg.h).
MRG_API int mrg_lstm_debug_inject(int mode) {
  MRG_REQUIRE(mode >= 0 && mode <= 2, "mrg_lstm_debug_inject: mode must be 0, 1 (next fwd) or 2 (next bwd)");
  g_inject = mode;
  return 0;
}

// Diagnostics: next LSTM launches record per-step phase clocks of block 0 into buf ([T][8] u64);
// pass null to disable.  Not for timed runs.
MRG_API int mrg_lstm_debug_stamps(void* buf) {
  g_stamps = (unsigned long long*)buf;
  return 0;
}

// Exchange-ring bytes (zeroed by the caller before every launch).
MRG_API size_t mrg_lstm_fwd_xbuf_bytes(int B, int H) { return (size_t)2 * B * H * 8; }
MRG_API size_t mrg_lstm_bwd_xbuf_bytes(int B, int H) {
  // sized for the largest group the runtime may select, so mrg_lstm_config can change it
  int G = H == 256 ? 16 : ring_group_size(H);
  return (size_t)2 * B * (G > 0 ? G : 1) * H * 8;
}

MRG_API int mrg_lstm_supported_hidden(int H) { return group_size(H) > 0; }

// Backward recurrences take the smallest batch tile whose grid fits `n` workgroups per CU (0 = the
// HW occupancy), leaving the rest of each CU to weight-gradient GEMMs issued beside them.  Returns
// the previous cap.
MRG_API int mrg_lstm_set_blocks_per_cu(int n) {
  const int prev = g_bwd_blocks_per_cu;
  g_bwd_blocks_per_cu = n > 0 ? n : 0;
  return prev;
}

// MFMA form of the H = 256 recurrences (lstm_mx.hip): 0 never, 1 when the VALU form needs batch tiles
// >= min_bs (default 4), 2 whenever its grid fits.  Returns the previous mode.
MRG_API int mrg_lstm_set_mx(int mode, int min_bs) {
  MRG_REQUIRE(mode >= 0 && mode <= 2, "mrg_lstm_set_mx: mode must be 0..2");
  const int prev = g_mx;
  g_mx = mode;
  if (min_bs > 0) g_mx_min_bs = min_bs;
  return prev;
}

// Tuning: solo (one-workgroup) groups at H <= 128 on / off.  Returns the previous setting.
MRG_API int mrg_lstm_set_solo(int on) {
  const int prev = g_solo;
  g_solo = on ? 1 : 0;
  return prev;
}

// Tuning: workgroups per recurrence group at H = 256 (8 or 16).  Affects the bwd xbuf size.
MRG_API int mrg_lstm_config(int group256) {
  MRG_REQUIRE(group256 == 4 || group256 == 8 || group256 == 16, "mrg_lstm_config: group must be 4, 8 or 16");
  g_group256 = group256;
  return 0;
}

// nprob independent same-shape recurrences in one persistent launch.
// Arrays are indexed by problem; strides in elements.  See lstm.hip header.
MRG_API int mrg_lstm_fwd(int nprob, int B, int T, int H,
                         const float* const* gx, const long* gx_bs, const long* gx_ts,
                         const float* const* w_hh, const float* const* b_hh,
                         const float* const* h0, const float* const* c0,
                         float* const* y, const long* y_bs, const long* y_ts,
                         float* const* gates, float* const* cs, float* const* hT, float* const* cT,
                         const int* reverse, void* const* xbuf, const long* lay, int* err, int cus,
                         int force_bs, hipStream_t stream) {
  MRG_REQUIRE(nprob >= 1 && nprob <= MAXP, "mrg_lstm_fwd: nprob %d out of range", nprob);
  int G = group_size(H);
  MRG_REQUIRE(G > 0, "mrg_lstm_fwd: unsupported hidden size %d", H);
  if (H == 256 && g_fwd_group256) G = g_fwd_group256;
  if (B == 0 || T == 0) return 0;
  LstmFwdArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = nprob; a.B = B; a.T = T; a.err = err; a.stamps = g_stamps;
  a.inject = g_inject == 1 ? 1 : 0;
  if (g_inject == 1) g_inject = 0;  // one launch only
  a.local = g_local;
  for (int i = 0; i < nprob; ++i) {
    LstmFwdProblem& p = a.p[i];
    p.gx = gx[i]; p.gx_bs = gx_bs[i]; p.gx_ts = gx_ts[i];
    p.w_hh = w_hh[i]; p.b_hh = b_hh[i]; p.h0 = h0 ? h0[i] : nullptr; p.c0 = c0 ? c0[i] : nullptr;
    p.y = y[i]; p.y_bs = y_bs[i]; p.y_ts = y_ts[i]; p.gates = gates[i]; p.cs = cs[i];
    p.hT = hT ? hT[i] : nullptr; p.cT = cT ? cT[i] : nullptr;
    p.xbuf = (unsigned long long*)xbuf[i]; p.reverse = reverse ? reverse[i] : 0;
    const long* L = lay ? lay + 8 * i : nullptr;  // {gates bs, ts, cs bs, ts, h0 bs, c0 bs}
    p.g_bs = L ? L[0] : (long)T * 4 * H; p.g_ts = L ? L[1] : 4 * H;
    p.cs_bs = L ? L[2] : (long)T * H; p.cs_ts = L ? L[3] : H;
    p.h0_bs = L ? L[4] : H; p.c0_bs = L ? L[5] : H;
    MRG_REQUIRE(((uintptr_t)p.w_hh & 15) == 0, "mrg_lstm_fwd: w_hh must be 16-byte aligned");
  }
  if (cus <= 0) cus = device_cus();
  switch (H) {
    case 256: return G == 8   ? launch_fwd<256, 8>(a, force_bs, cus, stream)
                     : G == 4 ? launch_fwd<256, 4>(a, force_bs, cus, stream)
                              : launch_fwd<256, 16>(a, force_bs, cus, stream);
    case 128: return G == 1 ? launch_fwd<128, 1>(a, force_bs, cus, stream) : launch_fwd<128, 8>(a, force_bs, cus, stream);
    case 64: return G == 1 ? launch_fwd<64, 1>(a, force_bs, cus, stream) : launch_fwd<64, 4>(a, force_bs, cus, stream);
    case 32: return G == 1 ? launch_fwd<32, 1>(a, force_bs, cus, stream) : launch_fwd<32, 2>(a, force_bs, cus, stream);
    case 16: return launch_fwd<16, 1>(a, force_bs, cus, stream);
  }
  return 2;
}

MRG_API int mrg_lstm_bwd(int nprob, int B, int T, int H,
                         const float* const* w_hh, const float* const* gates, const float* const* cs,
                         const float* const* c0, const float* const* dy, const long* dy_bs,
                         const long* dy_ts, const float* const* dhT, const float* const* dcT,
                         float* const* dG, float* const* dh0, float* const* dc0, const int* reverse,
                         void* const* xbuf, const long* lay, int* err, int cus, int force_bs,
                         hipStream_t stream) {
  MRG_REQUIRE(nprob >= 1 && nprob <= MAXP, "mrg_lstm_bwd: nprob %d out of range", nprob);
  int G = group_size(H);
  MRG_REQUIRE(G > 0, "mrg_lstm_bwd: unsupported hidden size %d", H);
  if (B == 0 || T == 0) return 0;
  LstmBwdArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = nprob; a.B = B; a.T = T; a.err = err; a.stamps = g_stamps;
  a.local = g_local;
  a.inject = g_inject == 2 ? 2 : 0;
  if (g_inject == 2) g_inject = 0;  // one launch only
  for (int i = 0; i < nprob; ++i) {
    LstmBwdProblem& p = a.p[i];
    p.w_hh = w_hh[i]; p.gates = gates[i]; p.cs = cs[i]; p.c0 = c0 ? c0[i] : nullptr;
    p.dy = dy ? dy[i] : nullptr; p.dy_bs = dy_bs ? dy_bs[i] : 0; p.dy_ts = dy_ts ? dy_ts[i] : 0;
    p.dhT = dhT ? dhT[i] : nullptr; p.dcT = dcT ? dcT[i] : nullptr; p.dG = dG[i];
    p.dh0 = dh0 ? dh0[i] : nullptr; p.dc0 = dc0 ? dc0[i] : nullptr;
    p.xbuf = (unsigned long long*)xbuf[i]; p.reverse = reverse ? reverse[i] : 0;
    const long* L = lay ? lay + 8 * i : nullptr;  // {gates bs, ts, cs bs, ts, c0 bs, dG bs, ts}
    p.g_bs = L ? L[0] : (long)T * 4 * H; p.g_ts = L ? L[1] : 4 * H;
    p.cs_bs = L ? L[2] : (long)T * H; p.cs_ts = L ? L[3] : H;
    p.c0_bs = L ? L[4] : H;
    p.dG_bs = L ? L[5] : (long)T * 4 * H; p.dG_ts = L ? L[6] : 4 * H;
  }
  if (cus <= 0) cus = device_cus();
  switch (H) {
    case 256: return G == 8   ? launch_bwd<256, 8>(a, force_bs, cus, stream)
                     : G == 4 ? launch_bwd<256, 4>(a, force_bs, cus, stream)
                              : launch_bwd<256, 16>(a, force_bs, cus, stream);
    case 128: return G == 1 ? launch_bwd<128, 1>(a, force_bs, cus, stream) : launch_bwd<128, 8>(a, force_bs, cus, stream);
    case 64: return G == 1 ? launch_bwd<64, 1>(a, force_bs, cus, stream) : launch_bwd<64, 4>(a, force_bs, cus, stream);
    case 32: return G == 1 ? launch_bwd<32, 1>(a, force_bs, cus, stream) : launch_bwd<32, 2>(a, force_bs, cus, stream);
    case 16: return launch_bwd<16, 1>(a, force_bs, cus, stream);
  }
  return 2;
}

// ---------------------------------------------------------------------------------------------
// Single-step LSTM cell (T = 1): the per-frame decode of lstm_with_sampling's scheduled-sampling
// training (LSTMSampler with carried state, LSTMLayerd restarted from zero each frame,
// lstm_with_sample.py:410-433).  A persistent recurrence launch (W_hh into the VGPRs of 512
// workgroups, a zeroed hand-off ring) for one step is pure overhead: the gate pre-activations
// come from the GEMMs (x W_ih^T + b_ih, + h0 W_hh^T when there is a state) and these two
// element-wise kernels do the rest.  Same gate order (i, f, g, o) and the same sigmoid / tanh
// as the persistent kernels.
namespace mrg {

__global__ __launch_bounds__(256) void lstm_cell_fwd_kernel(int B, int H, const float* __restrict__ pre, long pre_ld,
                                                            const float* __restrict__ b_hh,
                                                            const float* __restrict__ c0, float* __restrict__ gates,
                                                            float* __restrict__ c, float* __restrict__ h, long h_ld,
                                                            float* __restrict__ h2) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * H) return;
  const int b = i / H, u = i % H;
  const float* p = pre + (long)b * pre_ld;
  const float zi = p[u] + b_hh[u], zf = p[H + u] + b_hh[H + u];
  const float zg = p[2 * H + u] + b_hh[2 * H + u], zo = p[3 * H + u] + b_hh[3 * H + u];
  const float ig = sigmoidf_(zi), fg = sigmoidf_(zf), gg = tanhf_(zg), og = sigmoidf_(zo);
  const float cc = fg * (c0 ? c0[i] : 0.0f) + ig * gg;
  float* gs = gates + (long)b * 4 * H + u;
  gs[0] = ig; gs[H] = fg; gs[2 * H] = gg; gs[3 * H] = og;
  c[i] = cc;
  const float hv = og * tanhf_(cc);
  h[(long)b * h_ld + u] = hv;
  if (h2) h2[i] = hv;
}

__global__ __launch_bounds__(256) void lstm_cell_bwd_kernel(int B, int H, const float* __restrict__ gates,
                                                            const float* __restrict__ c,
                                                            const float* __restrict__ c0,
                                                            const float* __restrict__ dh, long dh_ld,
                                                            const float* __restrict__ dh2,
                                                            const float* __restrict__ dc, float* __restrict__ dG,
                                                            float* __restrict__ dc0) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * H) return;
  const int b = i / H, u = i % H;
  const float* gs = gates + (long)b * 4 * H + u;
  const float ig = gs[0], fg = gs[H], gg = gs[2 * H], og = gs[3 * H];
  const float cc = c[i], cp = c0 ? c0[i] : 0.0f;
  const float dhv = (dh ? dh[(long)b * dh_ld + u] : 0.0f) + (dh2 ? dh2[i] : 0.0f);
  const float tc = tanhf_(cc);
  const float dcc = dhv * og * (1.0f - tc * tc) + (dc ? dc[i] : 0.0f);
  float* d = dG + (long)b * 4 * H + u;
  d[0] = dcc * gg * ig * (1.0f - ig);
  d[H] = dcc * cp * fg * (1.0f - fg);
  d[2 * H] = dcc * ig * (1.0f - gg * gg);
  d[3 * H] = dhv * tc * og * (1.0f - og);
  if (dc0) dc0[i] = dcc * fg;
}

}  // namespace mrg

// gates [B, 4H], c [B, H], h rows of stride h_ld (and a dense copy in h2, nullable); pre [B, 4H]
// rows of stride pre_ld (b_ih already in); c0 nullable (zero state)
MRG_API int mrg_lstm_cell_fwd(int B, int H, const float* pre, long pre_ld, const float* b_hh, const float* c0,
                              float* gates, float* c, float* h, long h_ld, float* h2, hipStream_t stream) {
  if (B == 0 || H == 0) return 0;
  const long n = (long)B * H;
  klaunch(lstm_cell_fwd_kernel, (unsigned)((n + 255) / 256), 256, 0, stream, B, H, pre, pre_ld, b_hh, c0, gates, c, h,
                                                                        h_ld, h2);
  return check_launch("lstm_cell_fwd_kernel");
}

// dG [B, 4H] = d(gate pre-activations); the h gradient is dh (rows of stride dh_ld) + dh2 (dense);
// dh, dh2, dc, c0, dc0 nullable
MRG_API int mrg_lstm_cell_bwd(int B, int H, const float* gates, const float* c, const float* c0, const float* dh,
                              long dh_ld, const float* dh2, const float* dc, float* dG, float* dc0,
                              hipStream_t stream) {
  if (B == 0 || H == 0) return 0;
  const long n = (long)B * H;
  klaunch(lstm_cell_bwd_kernel, (unsigned)((n + 255) / 256), 256, 0, stream, B, H, gates, c, c0, dh, dh_ld, dh2, dc, dG, dc0);
  return check_launch("lstm_cell_bwd_kernel");
}
