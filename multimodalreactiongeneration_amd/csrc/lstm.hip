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
// Backward runs the same decomposition in reverse time: a member owns the
// same U units, computes dG for them, then the partial products
// P_j[b][:] = dG_j[b] W_hh[rows_j, :] over ALL H outputs; the exchange is a
// reduce-scatter (each member sums the G partials of its own units), so the
// bytes moved per step equal the forward's (BS x H granules per member).
#include "mrg_common.h"

namespace mrg {

static constexpr int NT = 256;
static constexpr int MAXP = 4;

struct LstmFwdProblem {
  const float* gx;  // pre-activations from the input GEMM (+ b_ih)
  long gx_bs, gx_ts;
  const float* w_hh;  // [4H, H]
  const float* b_hh;  // [4H]
  const float* h0;    // [B, H] or null
  const float* c0;    // [B, H] or null
  float* y;           // h_t
  long y_bs, y_ts;
  float* gates;  // [B, T, 4H] post-activation i, f, g, o (saved for backward)
  float* cs;     // [B, T, H] cell states (saved for backward)
  float* hT;     // [B, H] or null
  float* cT;     // [B, H] or null
  unsigned long long* xbuf;  // [2][B][H] granules
  int reverse;
};

struct LstmBwdProblem {
  const float* w_hh;
  const float* gates;
  const float* cs;
  const float* c0;  // nullable
  const float* dy;  // nullable
  long dy_bs, dy_ts;
  const float* dhT;  // nullable
  const float* dcT;  // nullable
  float* dG;         // [B, T, 4H]
  float* dh0;        // nullable
  float* dc0;        // nullable
  unsigned long long* xbuf;  // [2][B][G][H] granules
  int reverse;
};

struct LstmFwdArgs {
  LstmFwdProblem p[MAXP];
  int nprob, B, T;
  int* err;
};
struct LstmBwdArgs {
  LstmBwdProblem p[MAXP];
  int nprob, B, T;
  int* err;
};

static constexpr unsigned SPIN_LIMIT = 1u << 22;

__device__ __forceinline__ unsigned long long make_granule(unsigned tag, float v) {
  return ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v);
}

__device__ __forceinline__ void put_granule(unsigned long long* g, unsigned tag, float v) {
  __hip_atomic_store(g, make_granule(tag, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Poll one granule until its tag matches; bounded.  `dead` latches after a
// timeout so a broken launch drains quickly instead of spinning every step.
__device__ __forceinline__ float get_granule(unsigned long long* g, unsigned tag, int* err, bool& dead) {
  unsigned long long v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((unsigned)(v >> 32) != tag && !dead) {
    unsigned spins = 0;
    do {
      __builtin_amdgcn_s_sleep(1);
      v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (++spins > SPIN_LIMIT) {
        atomicOr(err, 1);
        dead = true;
        break;
      }
    } while ((unsigned)(v >> 32) != tag);
  }
  return __uint_as_float((unsigned)v);
}

// block -> (problem, group, member); members of a group share blockIdx % 8 (one XCD)
__device__ __forceinline__ void decompose(int G, int ngroups_per_prob, int nprob, int& prob, int& grp,
                                          int& member) {
  int b = blockIdx.x;
  int total_groups = ngroups_per_prob * nprob;
  int gid;
  if ((total_groups & 7) == 0) {
    int x = b & 7, idx = b >> 3;
    member = idx % G;
    gid = (idx / G) * 8 + x;
  } else {
    member = b % G;
    gid = b / G;
  }
  prob = gid / ngroups_per_prob;
  grp = gid % ngroups_per_prob;
}

template <int H, int G, int BS>
__global__ __launch_bounds__(NT) void lstm_fwd_kernel(LstmFwdArgs args) {
  constexpr int U = H / G;
  constexpr int R = 4 * U;
  constexpr int KC = NT / R;
  constexpr int KL = H / KC;
  constexpr int KLP = KL + 4;
  static_assert(NT % R == 0 && H % KC == 0 && BS * U <= NT && (KL % 4) == 0, "bad LSTM tiling");
  __shared__ __attribute__((aligned(16))) float hs[BS][KC][KLP];
  __shared__ float pre[BS][R];

  int prob, grp, j;
  const int ngroups = (args.B + BS - 1) / BS;
  decompose(G, ngroups, args.nprob, prob, grp, j);
  const LstmFwdProblem& P = args.p[prob];
  const int B = args.B, T = args.T;
  const int tid = threadIdx.x;
  const int b0 = grp * BS;
  bool dead = false;

  // dot role: gate row r, k-chunk kc
  const int r = tid / KC, kc = tid % KC;
  const int grow = (r / U) * H + j * U + (r % U);
  float w[KL];
#pragma unroll
  for (int i = 0; i < KL; i += 4) {
    float4 v = *reinterpret_cast<const float4*>(P.w_hh + (long)grow * H + kc * KL + i);
    w[i] = v.x; w[i + 1] = v.y; w[i + 2] = v.z; w[i + 3] = v.w;
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
    if (P.c0) c = P.c0[(long)bg * H + hcol];
  }

  // initial h_{-1}
  for (int e = tid; e < BS * H; e += NT) {
    int b = e / H, k = e % H;
    float v = 0.0f;
    if (P.h0 && b0 + b < B) v = P.h0[(long)(b0 + b) * H + k];
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
  for (int tt = 0; tt < T; ++tt) {
    const int t = P.reverse ? T - 1 - tt : tt;
    // 1. recurrent GEMV for this member's R gate rows
    float acc[BS];
#pragma unroll
    for (int b = 0; b < BS; ++b) {
      float s = 0.0f;
      const float* hp = &hs[b][kc][0];
#pragma unroll
      for (int i = 0; i < KL; i += 4) {
        float4 hv = *reinterpret_cast<const float4*>(hp + i);
        s = fmaf(w[i], hv.x, s);
        s = fmaf(w[i + 1], hv.y, s);
        s = fmaf(w[i + 2], hv.z, s);
        s = fmaf(w[i + 3], hv.w, s);
      }
      acc[b] = s;
    }
#pragma unroll
    for (int off = KC / 2; off >= 1; off >>= 1)
#pragma unroll
      for (int b = 0; b < BS; ++b) acc[b] += __shfl_xor(acc[b], off, 64);
    if (kc == 0) {
#pragma unroll
      for (int b = 0; b < BS; ++b) pre[b][r] = acc[b];
    }
    __syncthreads();
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
      put_granule(xb + ((long)par * B + bg) * H + hcol, (unsigned)(tt + 1), h);
      P.y[(long)bg * P.y_bs + (long)t * P.y_ts + hcol] = h;
      float* gs = P.gates + ((long)bg * T + t) * 4 * H + hcol;
      gs[0] = ig; gs[H] = fg; gs[2 * H] = gg; gs[3 * H] = og;
      P.cs[((long)bg * T + t) * H + hcol] = c;
      if (tt + 1 < T) load_gx(P.reverse ? t - 1 : t + 1);
    }
    // 4. gather h_t of the whole group
    if (tt + 1 < T) {
      for (int e = tid; e < BS * H; e += NT) {
        int b = e / H, k = e % H;
        float v = 0.0f;
        if (b0 + b < B)
          v = get_granule(xb + ((long)par * B + b0 + b) * H + k, (unsigned)(tt + 1), args.err, dead);
        hs[b][k / KL][k % KL] = v;
      }
    }
    __syncthreads();
  }
  if (cvalid) {
    if (P.hT) P.hT[(long)bg * H + hcol] = h;
    if (P.cT) P.cT[(long)bg * H + hcol] = c;
  }
}

template <int H, int G, int BS>
__global__ __launch_bounds__(NT) void lstm_bwd_kernel(LstmBwdArgs args) {
  constexpr int U = H / G;
  constexpr int R = 4 * U;
  constexpr int TP = NT / H;  // threads per output column of the partial product
  constexpr int RL = R / TP;  // W rows per thread
  static_assert(NT % H == 0 && R % TP == 0 && BS * U <= NT && (RL % 4) == 0, "bad LSTM bwd tiling");
  __shared__ __attribute__((aligned(16))) float dgl[BS][R];

  int prob, grp, j;
  const int ngroups = (args.B + BS - 1) / BS;
  decompose(G, ngroups, args.nprob, prob, grp, j);
  const LstmBwdProblem& P = args.p[prob];
  const int B = args.B, T = args.T;
  const int tid = threadIdx.x;
  const int b0 = grp * BS;
  bool dead = false;

  // dot role: output column hout, row chunk rc; w[i] = W_hh[grow(rc*RL+i)][hout]
  const int hout = tid / TP, rc = tid % TP;
  float w[RL];
#pragma unroll
  for (int i = 0; i < RL; ++i) {
    int rr = rc * RL + i;
    int grow = (rr / U) * H + j * U + (rr % U);
    w[i] = P.w_hh[(long)grow * H + hout];
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

  unsigned long long* xb = P.xbuf;
  const long xstride_b = (long)G * H;  // per batch row: [dest G][src G][U]
  for (int tt = 0; tt < T; ++tt) {
    const int t = P.reverse ? tt : T - 1 - tt;
    const int tprev = P.reverse ? t + 1 : t - 1;  // forward-time predecessor
    if (cvalid) {
      if (tt > 0) {
        const int par = (tt - 1) & 1;
        unsigned long long* g = xb + ((long)par * B + bg) * xstride_b + (long)j * H + cu;
        float s = 0.0f;
#pragma unroll
        for (int src = 0; src < G; ++src) s += get_granule(g + src * U, (unsigned)tt, args.err, dead);
        dhrec = s;
      }
      float dh = dhrec;
      if (P.dy) dh += P.dy[(long)bg * P.dy_bs + (long)t * P.dy_ts + hcol];
      const float* gs = P.gates + ((long)bg * T + t) * 4 * H + hcol;
      float ig = gs[0], fg = gs[H], gg = gs[2 * H], og = gs[3 * H];
      float cc = P.cs[((long)bg * T + t) * H + hcol];
      float cp = 0.0f;
      if (tprev >= 0 && tprev < T) cp = P.cs[((long)bg * T + tprev) * H + hcol];
      else if (P.c0) cp = P.c0[(long)bg * H + hcol];
      float tc = tanhf_(cc);
      float dc = dh * og * (1.0f - tc * tc) + dcn;
      float d_o = dh * tc * og * (1.0f - og);
      float d_i = dc * gg * ig * (1.0f - ig);
      float d_f = dc * cp * fg * (1.0f - fg);
      float d_g = dc * ig * (1.0f - gg * gg);
      dcn = dc * fg;
      float* dgp = P.dG + ((long)bg * T + t) * 4 * H + hcol;
      dgp[0] = d_i; dgp[H] = d_f; dgp[2 * H] = d_g; dgp[3 * H] = d_o;
      dgl[cb][0 * U + cu] = d_i;
      dgl[cb][1 * U + cu] = d_f;
      dgl[cb][2 * U + cu] = d_g;
      dgl[cb][3 * U + cu] = d_o;
    } else if (cell) {
      dgl[cb][cu] = 0.0f; dgl[cb][U + cu] = 0.0f; dgl[cb][2 * U + cu] = 0.0f; dgl[cb][3 * U + cu] = 0.0f;
    }
    __syncthreads();
    // partial dh_{t-1}[b][hout] = sum over this member's rows of dG[b][row] * W_hh[row][hout]
    // (batch loop kept rolled: the 128 W registers stay resident without spilling)
    {
      const int par = tt & 1;
      const int dest = hout / U, du = hout % U;
#pragma unroll 1
      for (int b = 0; b < BS; ++b) {
        float s = 0.0f;
        const float* dp = &dgl[b][rc * RL];
#pragma unroll
        for (int i = 0; i < RL; i += 4) {
          float4 dv = *reinterpret_cast<const float4*>(dp + i);
          s = fmaf(dv.x, w[i], s);
          s = fmaf(dv.y, w[i + 1], s);
          s = fmaf(dv.z, w[i + 2], s);
          s = fmaf(dv.w, w[i + 3], s);
        }
#pragma unroll
        for (int off = TP / 2; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
        if (rc == 0 && b0 + b < B)
          put_granule(xb + ((long)par * B + b0 + b) * xstride_b + (long)dest * H + (long)j * U + du,
                      (unsigned)(tt + 1), s);
      }
    }
    __syncthreads();
  }
  if (cvalid) {
    if (P.dh0) {
      const int par = (T - 1) & 1;
      unsigned long long* g = xb + ((long)par * B + bg) * xstride_b + (long)j * H + cu;
      float s = 0.0f;
#pragma unroll
      for (int src = 0; src < G; ++src) s += get_granule(g + src * U, (unsigned)T, args.err, dead);
      P.dh0[(long)bg * H + hcol] = s;
    }
    if (P.dc0) P.dc0[(long)bg * H + hcol] = dcn;
  }
}

template <int H, int G>
static int launch_fwd(const LstmFwdArgs& a, int BS, int nblk, hipStream_t s) {
  switch (BS) {
    case 1: lstm_fwd_kernel<H, G, 1><<<nblk, NT, 0, s>>>(a); break;
    case 2: lstm_fwd_kernel<H, G, 2><<<nblk, NT, 0, s>>>(a); break;
    case 4: lstm_fwd_kernel<H, G, 4><<<nblk, NT, 0, s>>>(a); break;
    case 8: lstm_fwd_kernel<H, G, 8><<<nblk, NT, 0, s>>>(a); break;
    default: set_error("lstm fwd: bad BS %d", BS); return 2;
  }
  return check_launch("lstm_fwd_kernel");
}

template <int H, int G>
static int launch_bwd(const LstmBwdArgs& a, int BS, int nblk, hipStream_t s) {
  switch (BS) {
    case 1: lstm_bwd_kernel<H, G, 1><<<nblk, NT, 0, s>>>(a); break;
    case 2: lstm_bwd_kernel<H, G, 2><<<nblk, NT, 0, s>>>(a); break;
    case 4: lstm_bwd_kernel<H, G, 4><<<nblk, NT, 0, s>>>(a); break;
    case 8: lstm_bwd_kernel<H, G, 8><<<nblk, NT, 0, s>>>(a); break;
    default: set_error("lstm bwd: bad BS %d", BS); return 2;
  }
  return check_launch("lstm_bwd_kernel");
}

// members per group for a hidden size (U = 32 at H=256, U = 16 below)
static int group_size(int H) {
  switch (H) {
    case 256: return 8;
    case 128: return 8;
    case 64: return 4;
    case 32: return 2;
    case 16: return 1;
    default: return 0;
  }
}

// batch rows per group: keep the persistent grid <= 2 workgroups per CU
static int pick_bs(int nprob, int B, int G, int cus) {
  for (int bs = 1; bs <= 8; bs *= 2) {
    long groups = (long)nprob * ((B + bs - 1) / bs);
    if (groups * G <= 2L * cus) return bs;
  }
  return 8;
}

}  // namespace mrg

using namespace mrg;

// Exchange-ring bytes (zeroed by the caller before every launch).
MRG_API size_t mrg_lstm_fwd_xbuf_bytes(int B, int H) { return (size_t)2 * B * H * 8; }
MRG_API size_t mrg_lstm_bwd_xbuf_bytes(int B, int H) {
  int G = group_size(H);
  return (size_t)2 * B * (G > 0 ? G : 1) * H * 8;
}

MRG_API int mrg_lstm_supported_hidden(int H) { return group_size(H) > 0; }

// nprob independent same-shape recurrences in one persistent launch.
// Arrays are indexed by problem; strides in elements.  See lstm.hip header.
MRG_API int mrg_lstm_fwd(int nprob, int B, int T, int H,
                         const float* const* gx, const long* gx_bs, const long* gx_ts,
                         const float* const* w_hh, const float* const* b_hh,
                         const float* const* h0, const float* const* c0,
                         float* const* y, const long* y_bs, const long* y_ts,
                         float* const* gates, float* const* cs, float* const* hT, float* const* cT,
                         const int* reverse, void* const* xbuf, int* err, int cus, int force_bs,
                         hipStream_t stream) {
  MRG_REQUIRE(nprob >= 1 && nprob <= MAXP, "mrg_lstm_fwd: nprob %d out of range", nprob);
  int G = group_size(H);
  MRG_REQUIRE(G > 0, "mrg_lstm_fwd: unsupported hidden size %d", H);
  if (B == 0 || T == 0) return 0;
  LstmFwdArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = nprob; a.B = B; a.T = T; a.err = err;
  for (int i = 0; i < nprob; ++i) {
    LstmFwdProblem& p = a.p[i];
    p.gx = gx[i]; p.gx_bs = gx_bs[i]; p.gx_ts = gx_ts[i];
    p.w_hh = w_hh[i]; p.b_hh = b_hh[i]; p.h0 = h0 ? h0[i] : nullptr; p.c0 = c0 ? c0[i] : nullptr;
    p.y = y[i]; p.y_bs = y_bs[i]; p.y_ts = y_ts[i]; p.gates = gates[i]; p.cs = cs[i];
    p.hT = hT ? hT[i] : nullptr; p.cT = cT ? cT[i] : nullptr;
    p.xbuf = (unsigned long long*)xbuf[i]; p.reverse = reverse ? reverse[i] : 0;
    MRG_REQUIRE(((uintptr_t)p.w_hh & 15) == 0, "mrg_lstm_fwd: w_hh must be 16-byte aligned");
  }
  int BS = force_bs > 0 ? force_bs : pick_bs(nprob, B, G, cus > 0 ? cus : 256);
  int nblk = nprob * ((B + BS - 1) / BS) * G;
  switch (H) {
    case 256: return launch_fwd<256, 8>(a, BS, nblk, stream);
    case 128: return launch_fwd<128, 8>(a, BS, nblk, stream);
    case 64: return launch_fwd<64, 4>(a, BS, nblk, stream);
    case 32: return launch_fwd<32, 2>(a, BS, nblk, stream);
    case 16: return launch_fwd<16, 1>(a, BS, nblk, stream);
  }
  return 2;
}

MRG_API int mrg_lstm_bwd(int nprob, int B, int T, int H,
                         const float* const* w_hh, const float* const* gates, const float* const* cs,
                         const float* const* c0, const float* const* dy, const long* dy_bs,
                         const long* dy_ts, const float* const* dhT, const float* const* dcT,
                         float* const* dG, float* const* dh0, float* const* dc0, const int* reverse,
                         void* const* xbuf, int* err, int cus, int force_bs, hipStream_t stream) {
  MRG_REQUIRE(nprob >= 1 && nprob <= MAXP, "mrg_lstm_bwd: nprob %d out of range", nprob);
  int G = group_size(H);
  MRG_REQUIRE(G > 0, "mrg_lstm_bwd: unsupported hidden size %d", H);
  if (B == 0 || T == 0) return 0;
  LstmBwdArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = nprob; a.B = B; a.T = T; a.err = err;
  for (int i = 0; i < nprob; ++i) {
    LstmBwdProblem& p = a.p[i];
    p.w_hh = w_hh[i]; p.gates = gates[i]; p.cs = cs[i]; p.c0 = c0 ? c0[i] : nullptr;
    p.dy = dy ? dy[i] : nullptr; p.dy_bs = dy_bs ? dy_bs[i] : 0; p.dy_ts = dy_ts ? dy_ts[i] : 0;
    p.dhT = dhT ? dhT[i] : nullptr; p.dcT = dcT ? dcT[i] : nullptr; p.dG = dG[i];
    p.dh0 = dh0 ? dh0[i] : nullptr; p.dc0 = dc0 ? dc0[i] : nullptr;
    p.xbuf = (unsigned long long*)xbuf[i]; p.reverse = reverse ? reverse[i] : 0;
  }
  int BS = force_bs > 0 ? force_bs : pick_bs(nprob, B, G, cus > 0 ? cus : 256);
  int nblk = nprob * ((B + BS - 1) / BS) * G;
  switch (H) {
    case 256: return launch_bwd<256, 8>(a, BS, nblk, stream);
    case 128: return launch_bwd<128, 8>(a, BS, nblk, stream);
    case 64: return launch_bwd<64, 4>(a, BS, nblk, stream);
    case 32: return launch_bwd<32, 2>(a, BS, nblk, stream);
    case 16: return launch_bwd<16, 1>(a, BS, nblk, stream);
  }
  return 2;
}
