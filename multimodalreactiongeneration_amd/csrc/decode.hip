// Fused autoregressive decode of lstm_with_sampling's scheduled-sampling step (BASELINE configs[2]).
//
// Reference: LSTMwithSample.prediction -> head_motion_generation -> generate_one_step
// (mr_gen/model/lstm_with_sampling/lstm_with_sample.py:339-433): every frame t runs the whole
// forward on one frame; the sampler LSTM carries its state, the layered LSTM restarts from zero
// (SURVEY Q2), and the self-motion input is the previous prediction or, teacher-forced, motion_s
// one frame late (Q10):  ms_in(0) = ms[0],  ms_in(t+1) = mask[t] ? y(t) : ms[t].
//
// What is sequential across frames is only the chain feat(t) -> layered LSTMs -> FFN -> y(t) ->
// ms_in(t+1).  Everything else is hoisted out of the frame loop by the host (functional.py,
// _SSDecodeFn): the sampler over the whole audio sequence is one persistent LSTM per layer, the
// feature projection of [sampler output | partner motion] for all frames is one GEMM (P), and every
// weight gradient is one GEMM over all frames after the loop.  Per frame this file runs
//   fwd: ssd_gate_cell_fwd (layer 1: X = P(t) + ms_in(t) W_ms^T; layer l > 1: X = LN(h + x) of
//        layer l-1, the residual of LSTMBlock, lstm_block.py:88-103) -> zero-state LSTM cell,
//        then ssd_ffn_fwd (LN of the last layer, FFN 256->64->ReLU->6, the sampling select);
//   bwd: ssd_ln_cell_bwd (FFN backward for the last layer, LayerNorm backward, cell backward)
//        alternating with ssd_dx (dX = dG W_ih + the residual gradient), i.e. 1 + 3L launches
//        per frame.
// Arithmetic: fp32 FMA chains (parity 1e-4 with the reference's fp32 CPU path).
//
// Layouts: per-frame tensors are time-major [T][B][...] so a frame is one contiguous slab; the
// layer-1 input of frame t lives in the X_f buffer [T][B][F] = [sampler | partner | ms_in] whose
// last FM columns the FFN kernel of frame t-1 fills (the select).
#include "mrg_common.h"

namespace mrg {

// Guarded loads WITHOUT a branch, as range-checked buffer loads (cdna_hip_programming.md T8): a
// masked-off element gets an offset past the descriptor's range and the hardware returns 0.  A
// plain load under `if (ok)` (or a clamped address with a select after it, which hipcc turns back
// into a branch) is issued alone and waited for right behind it (cdna_hip_programming.md §5,
// "Projection GEMM", trap (c)): a tile of them then costs one L2 round trip PER LOAD instead of one
// for all of them.  `p` must be wave-uniform (a kernel argument): the descriptor lives in SGPRs.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
static constexpr int SSD_RANGE = 0x7fffff00;  // descriptor range; masked-off lanes load here (OOB)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ssd_rsrc(const float* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, SSD_RANGE, 0x00020000);
}
__device__ __forceinline__ float ld_or0(const float* p, long idx, bool ok) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ssd_rsrc(p), ok ? (int)(idx * 4) : SSD_RANGE,
                                                                         0, 0));
}
__device__ __forceinline__ float4 ld4_or0(const float* p, long idx, bool ok) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ssd_rsrc(p), ok ? (int)(idx * 4) : SSD_RANGE,
                                                                           0, 0));
}

struct SsdFwdArgs {
  int B, H;
  const float* xin;              // MODE 0: this layer's input [B][H]; MODE 2: P(t) [B][H]
  const float* hp;               // MODE 1: previous layer h [B][H]
  const float* rp;               // MODE 1: previous layer's residual input [B][H]
  const float* gamma;            // MODE 1: previous layer's LayerNorm
  const float* beta;
  float eps;
  float* xout;                   // this layer's input X [B][H], written by blockIdx.x == 0 (null: none)
  float* mean;                   // MODE 1: LN stats of the previous layer [B]
  float* rstd;
  const float* w_ih;             // [4H][H]
  const float* b_ih;
  const float* b_hh;
  float* gates;                  // [B][4H] post-activation i, f, g, o
  float* c;                      // [B][H]
  float* h;                      // [B][H]
  // MODE 2 (layer 1 of frame t): X = P(t) + ms_in(t) W_ms^T with ms_in(0) = ms[0] and
  // ms_in(t) = mask[t-1] ? y(t-1) : ms[t-1], y(t-1) = z(t-1) W2^T + b2 (the FFN's second Linear)
  int HB, FO, F, tm;             // tm = t - 1 (0 at t = 0)
  const float* z;                // z(t-1) [B][HB] (null at t = 0: ms_in = ms[0])
  const float* w2;               // [FO][HB]
  const float* b2;
  const unsigned char* mask;     // [T]
  const float* ms;               // ms[b * ms_bs + t * ms_ts + o]
  long ms_bs, ms_ts;
  const float* wms;              // W_ms^T [FO][H] (the ms columns of the feature projection)
  float* y;                      // y(t-1)[b * y_bs + o] (written when z is given)
  long y_bs;
  float* xf_ms;                  // ms_in(t) -> xf_ms[b * F + o] (the X_f row's ms columns)
};

// Zero-state LSTM layer of one frame (LSTMModule with h0 = c0 = 0, lstm_block.py:38-46):
// gates = X W_ih^T + b_ih + b_hh; c = sigmoid(i) tanh(g); h = sigmoid(o) tanh(c).
// Workgroup = 16 batch rows x 4 hidden units (16 gate columns, c = q * 4 + unit): the gate tile is
// one 16 x 16 exact-f32 MFMA tile (v_mfma_f32_16x16x4_f32), the K = H reduction split over the 4
// waves and summed in a fixed order.  Tiles are small on purpose: a CU streams ~11-28 B/cycle from
// L2 (MI355X_MICROARCH.md), so the bytes a workgroup loads (its 16 X rows + 16 W_ih rows,
// 32-48 KB) set the launch time, and 256 workgroups share the 1 MB of W_ih.
// The X tile is built in the prologue: MODE 0 reads it; MODE 1 is LayerNorm(hp + rp) of the
// previous layer on the registers (each wave holds whole rows: the statistics are lane-group
// reductions); MODE 2 is the frame's features with the previous frame's FFN output Linear and the
// sampling select folded in (every workgroup recomputes its 16 rows of y: 6 x 64 FMAs a row).
static constexpr int SSD_R = 16, SSD_U = 4;
typedef float ssd_f32x4 __attribute__((ext_vector_type(4)));

template <int EPL, int MODE, int DBG = 0>  // DBG (timing experiments only): 1 no X prologue, 2 no GEMM
__global__ __launch_bounds__(256) void ssd_gate_cell_fwd_kernel(SsdFwdArgs a) {
  constexpr int HMAX = EPL * 64, G = HMAX / 4;        // G lanes (x 4 columns) per row
  constexpr int LDK = HMAX + 2;                       // 2i + k banks: conflict-free fragment reads
  constexpr int NX = SSD_R * HMAX / 4 / 256 > 0 ? SSD_R * HMAX / 4 / 256 : 1;   // float4 per thread
  __shared__ __attribute__((aligned(16))) float Xs[SSD_R * LDK];
  __shared__ __attribute__((aligned(16))) float Ws[16 * LDK];
  __shared__ float red[4][16][17];
  __shared__ float bias[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, H4 = H / 4;
  const int r0 = blockIdx.y * SSD_R, u0 = blockIdx.x * SSD_U;
  const int c4 = tid % G;
  const bool cv = c4 < H4;
  // loads: the 16 W_ih rows of this tile, the X rows (MODE 1: h and x), biases, gamma / beta
  float4 wv[NX], xv[NX], rv[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int rr = (tid + i * 256) / G;             // tile column c = rr (< 16)
    const int q = rr >> 2, uu = rr & 3;
    wv[i] = ld4_or0(a.w_ih, (long)(q * H + u0 + uu) * H + 4 * c4, rr < 16 && u0 + uu < H && cv);
    const int b = r0 + rr;                          // tile row rr
    const bool ok = (DBG & 1) == 0 && rr < SSD_R && b < a.B && cv;
    xv[i] = ld4_or0(MODE == 1 ? a.hp : a.xin, (long)b * H + 4 * c4, ok);
    if (MODE == 1) rv[i] = ld4_or0(a.rp, (long)b * H + 4 * c4, ok);
  }
  if (tid < 16) {
    const int q = tid >> 2, uu = tid & 3;
    bias[tid] = ld_or0(a.b_ih, q * H + u0 + uu, u0 + uu < H) + ld_or0(a.b_hh, q * H + u0 + uu, u0 + uu < H);
  }
  if (MODE == 1 && (DBG & 1) == 0) {
    const float4 g = ld4_or0(a.gamma, 4 * c4, cv), bt = ld4_or0(a.beta, 4 * c4, cv);
    float s[NX], qv[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      xv[i].x += rv[i].x; xv[i].y += rv[i].y; xv[i].z += rv[i].z; xv[i].w += rv[i].w;
      s[i] = (xv[i].x + xv[i].y) + (xv[i].z + xv[i].w);
    }
#pragma unroll
    for (int o = 1; o < G; o <<= 1)
#pragma unroll
      for (int i = 0; i < NX; ++i) s[i] += __shfl_xor(s[i], o, 64);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      s[i] /= (float)H;
      const float d0 = xv[i].x - s[i], d1 = xv[i].y - s[i], d2 = xv[i].z - s[i], d3 = xv[i].w - s[i];
      qv[i] = cv ? (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3) : 0.0f;
    }
#pragma unroll
    for (int o = 1; o < G; o <<= 1)
#pragma unroll
      for (int i = 0; i < NX; ++i) qv[i] += __shfl_xor(qv[i], o, 64);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const float rs = rsqrtf(qv[i] / (float)H + a.eps);
      xv[i].x = (xv[i].x - s[i]) * rs * g.x + bt.x; xv[i].y = (xv[i].y - s[i]) * rs * g.y + bt.y;
      xv[i].z = (xv[i].z - s[i]) * rs * g.z + bt.z; xv[i].w = (xv[i].w - s[i]) * rs * g.w + bt.w;
      const int rr = (tid + i * 256) / G, b = r0 + rr;
      if (blockIdx.x == 0 && c4 == 0 && rr < SSD_R && b < a.B) {
        a.mean[b] = s[i];
        a.rstd[b] = rs;
      }
    }
  }
  if (MODE == 2) {
    // y(t-1) of the tile's rows from z(t-1), W2, b2; then X += ms_in W_ms^T
    __shared__ float zs[SSD_R][65];
    __shared__ float w2s[8][64];
    __shared__ float msin[SSD_R][8];
    const bool fed = a.z != nullptr;
    float zv[4], w2v[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = tid + i * 256, r = e >> 6, j = e & 63;
      zv[i] = ld_or0(a.z, (long)(r0 + r) * a.HB + j, fed && r0 + r < a.B && j < a.HB);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + i * 256, o = e >> 6, j = e & 63;
      w2v[i] = ld_or0(a.w2, (long)o * a.HB + j, fed && o < a.FO && j < a.HB);
    }
    float4 wm[8];
#pragma unroll
    for (int o = 0; o < 8; ++o) wm[o] = ld4_or0(a.wms, (long)o * H + 4 * c4, o < a.FO && cv);
    const int rs_ = tid >> 3, os_ = tid & 7, bs_ = r0 + rs_;
    const bool sv = tid < SSD_R * 8 && os_ < a.FO && bs_ < a.B;
    const float b2v = ld_or0(a.b2, os_, fed && sv);
    const float msv = ld_or0(a.ms, (long)bs_ * a.ms_bs + (long)a.tm * a.ms_ts + os_, sv);
    const bool sel = fed && a.mask[a.tm] != 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) zs[(tid + i * 256) >> 6][(tid + i * 256) & 63] = zv[i];
#pragma unroll
    for (int i = 0; i < 2; ++i) w2s[(tid + i * 256) >> 6][(tid + i * 256) & 63] = w2v[i];
    __syncthreads();
    if (tid < SSD_R * 8) {
      float m = 0.0f;
      if (sv) {
        float yv = b2v;
        if (fed) {
#pragma unroll 16
          for (int j = 0; j < 64; ++j) yv = fmaf(zs[rs_][j], w2s[os_][j], yv);
          if (blockIdx.x == 0) a.y[(long)bs_ * a.y_bs + os_] = yv;
        }
        m = sel ? yv : msv;
        if (blockIdx.x == 0) a.xf_ms[(long)bs_ * a.F + os_] = m;
      }
      msin[rs_][os_] = m;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int rr = (tid + i * 256) / G;
      if (rr >= SSD_R) continue;
#pragma unroll
      for (int o = 0; o < 8; ++o) {
        const float mo = msin[rr][o];
        xv[i].x = fmaf(mo, wm[o].x, xv[i].x); xv[i].y = fmaf(mo, wm[o].y, xv[i].y);
        xv[i].z = fmaf(mo, wm[o].z, xv[i].z); xv[i].w = fmaf(mo, wm[o].w, xv[i].w);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int rr = (tid + i * 256) / G, b = r0 + rr;
    if (rr >= 16) continue;
    float2* wd = reinterpret_cast<float2*>(&Ws[rr * LDK + 4 * c4]);
    wd[0] = make_float2(wv[i].x, wv[i].y);
    wd[1] = make_float2(wv[i].z, wv[i].w);
    float2* xd = reinterpret_cast<float2*>(&Xs[rr * LDK + 4 * c4]);
    xd[0] = make_float2(xv[i].x, xv[i].y);
    xd[1] = make_float2(xv[i].z, xv[i].w);
    if (a.xout && blockIdx.x == 0 && b < a.B && cv) *reinterpret_cast<float4*>(a.xout + (long)b * H + 4 * c4) = xv[i];
  }
  __syncthreads();
  // 16 x 16 gate tile over this wave's quarter of K: lane (l16, kg) feeds A[l16][k], B[k][l16]
  const int l16 = lane & 15, kg = lane >> 4;
  const int kq = HMAX / 4, kb = wave * kq;
  ssd_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if ((DBG & 2) == 0) {
#pragma unroll 8
    for (int k = kb; k < kb + kq; k += 8) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Xs[l16 * LDK + k + kg], Ws[l16 * LDK + k + kg], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(Xs[l16 * LDK + k + 4 + kg], Ws[l16 * LDK + k + 4 + kg], acc1, 0, 0, 0);
    }
  }
  // lane holds C[4 kg + i][l16] (rows = batch rows, columns = gate columns)
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][4 * kg + i][l16] = acc0[i] + acc1[i];
  __syncthreads();
  if (tid < SSD_R * SSD_U) {
    const int rr = tid >> 2, uu = tid & 3, b = r0 + rr, u = u0 + uu;
    if (b < a.B && u < H) {
      float z[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = q * 4 + uu;
        z[q] = ((red[0][rr][c] + red[1][rr][c]) + (red[2][rr][c] + red[3][rr][c])) + bias[c];
      }
      const float ig = sigmoidf_(z[0]), fg = sigmoidf_(z[1]), gg = tanhf_(z[2]), og = sigmoidf_(z[3]);
      const float cc = ig * gg;
      float* gs = a.gates + (long)b * 4 * H + u;
      gs[0] = ig; gs[H] = fg; gs[2 * H] = gg; gs[3 * H] = og;
      a.c[(long)b * H + u] = cc;
      a.h[(long)b * H + u] = og * tanhf_(cc);
    }
  }
}

// dX = dG W_ih + g for one frame: [B, 4H] x [4H, H] with W_ih given transposed (w_t [H][4H], so both
// operands are read k-contiguous).  The forget-gate block of dG is zero (zero state: c_prev = 0), so
// K runs over the i, g, o blocks only (3H).  Workgroup = 8 rows x 8 columns (256 workgroups at
// B = 64, H = 256, 48 KB loaded each); thread = (row, column, k phase of 4), float4 k-chunks
// interleaved by phase so the 4 phases hit different LDS banks; fixed-order shuffle reduction.
template <int KMAX>  // 3 * H rounded up
__global__ __launch_bounds__(256) void ssd_dx_kernel(int B, int H, const float* __restrict__ dG,
                                                     const float* __restrict__ w_t, const float* __restrict__ g,
                                                     float* __restrict__ dx) {
  constexpr int LDK = KMAX + 4, KC = KMAX / 4;  // KC float4 chunks a row
  constexpr int NL = (8 * KC + 255) / 256;      // float4 per thread per operand tile
  __shared__ __attribute__((aligned(16))) float As[8 * LDK];
  __shared__ __attribute__((aligned(16))) float Bs[8 * LDK];
  const int tid = threadIdx.x;
  const int K = 4 * H, H4 = H / 4;
  const int r0 = blockIdx.y * 8, n0 = blockIdx.x * 8;
  float4 av[NL], bv[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = tid + i * 256, rr = e / KC, k4 = e % KC;
    const int kg = k4 < H4 ? k4 : k4 + H4;  // skip the forget block [H, 2H)
    const bool kin = rr < 8 && k4 < 3 * H4;
    av[i] = ld4_or0(dG, (long)(r0 + rr) * K + 4 * kg, kin && r0 + rr < B);
    bv[i] = ld4_or0(w_t, (long)(n0 + rr) * K + 4 * kg, kin && n0 + rr < H);
  }
  const int r = tid >> 5, n = (tid >> 2) & 7, ph = tid & 3;
  const float gv = ld_or0(g, (long)(r0 + r) * H + n0 + n, r0 + r < B && n0 + n < H && ph == 0);
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int e = tid + i * 256, rr = e / KC, k4 = e % KC;
    if (rr < 8) {
      *reinterpret_cast<float4*>(&As[rr * LDK + 4 * k4]) = av[i];
      *reinterpret_cast<float4*>(&Bs[rr * LDK + 4 * k4]) = bv[i];
    }
  }
  __syncthreads();
  float acc = 0.0f;
#pragma unroll 8
  for (int j = ph; j < KC; j += 4) {
    const float4 x = *reinterpret_cast<const float4*>(&As[r * LDK + 4 * j]);
    const float4 w = *reinterpret_cast<const float4*>(&Bs[n * LDK + 4 * j]);
    acc = fmaf(x.x, w.x, acc);
    acc = fmaf(x.y, w.y, acc);
    acc = fmaf(x.z, w.z, acc);
    acc = fmaf(x.w, w.w, acc);
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  if (ph == 0 && r0 + r < B && n0 + n < H) dx[(long)(r0 + r) * H + n0 + n] = acc + gv;
}

// Last LayerNorm of the layered LSTM + the FFN's first Linear and ReLU (lstm_with_sample.py:123-130,
// 229-232): u = LN(h + x), z = relu(u W1^T + b1).  Workgroup = 8 rows x 8 outputs (64 workgroups at
// B = 64, HB = 64; 24 KB loaded each); the second Linear, the sampling select and the next frame's
// features are folded into the next frame's layer-1 gate kernel (MODE 2).
template <int EPL>
__global__ __launch_bounds__(256) void ssd_ffn_z_kernel(int B, int H, int HB, const float* __restrict__ hp,
                                                        const float* __restrict__ rp, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps, float* __restrict__ u,
                                                        float* __restrict__ mean, float* __restrict__ rstd,
                                                        const float* __restrict__ w1, const float* __restrict__ b1,
                                                        float* __restrict__ z) {
  constexpr int HMAX = EPL * 64, LDW = HMAX + 4, G = HMAX / 4;
  constexpr int RPP = 256 / G, NU = (8 + RPP - 1) / RPP;  // rows per pass, float4 per thread
  __shared__ __attribute__((aligned(16))) float us[8][LDW];
  __shared__ __attribute__((aligned(16))) float ws[8][LDW];
  const int tid = threadIdx.x, H4 = H / 4;
  const int r0 = blockIdx.y * 8, j0 = blockIdx.x * 8;
  const int c4 = tid % G;
  const bool cv = c4 < H4;
  float4 hv[NU], xv[NU], wv[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    const int r = (tid + i * 256) / G, b = r0 + r, j = j0 + r;
    const bool ok = r < 8 && b < B && cv;
    hv[i] = ld4_or0(hp, (long)b * H + 4 * c4, ok);
    xv[i] = ld4_or0(rp, (long)b * H + 4 * c4, ok);
    wv[i] = ld4_or0(w1, (long)j * H + 4 * c4, r < 8 && j < HB && cv);
  }
  const float4 g = ld4_or0(gamma, 4 * c4, cv), bt = ld4_or0(beta, 4 * c4, cv);
  const int r = tid >> 5, jj = (tid >> 2) & 7, ph = tid & 3;
  const float b1v = ld_or0(b1, j0 + jj, j0 + jj < HB);
  float s[NU], q[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    hv[i].x += xv[i].x; hv[i].y += xv[i].y; hv[i].z += xv[i].z; hv[i].w += xv[i].w;
    s[i] = (hv[i].x + hv[i].y) + (hv[i].z + hv[i].w);
  }
#pragma unroll
  for (int o = 1; o < G; o <<= 1)
#pragma unroll
    for (int i = 0; i < NU; ++i) s[i] += __shfl_xor(s[i], o, 64);
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    s[i] /= (float)H;
    const float d0 = hv[i].x - s[i], d1 = hv[i].y - s[i], d2 = hv[i].z - s[i], d3 = hv[i].w - s[i];
    q[i] = cv ? (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3) : 0.0f;
  }
#pragma unroll
  for (int o = 1; o < G; o <<= 1)
#pragma unroll
    for (int i = 0; i < NU; ++i) q[i] += __shfl_xor(q[i], o, 64);
#pragma unroll
  for (int i = 0; i < NU; ++i) {
    const int rr = (tid + i * 256) / G, b = r0 + rr;
    if (rr >= 8) continue;
    const float rs = rsqrtf(q[i] / (float)H + eps);
    float4 uv;
    uv.x = (hv[i].x - s[i]) * rs * g.x + bt.x; uv.y = (hv[i].y - s[i]) * rs * g.y + bt.y;
    uv.z = (hv[i].z - s[i]) * rs * g.z + bt.z; uv.w = (hv[i].w - s[i]) * rs * g.w + bt.w;
    *reinterpret_cast<float4*>(&us[rr][4 * c4]) = uv;
    *reinterpret_cast<float4*>(&ws[rr][4 * c4]) = wv[i];
    if (blockIdx.x == 0 && b < B) {
      if (cv) *reinterpret_cast<float4*>(u + (long)b * H + 4 * c4) = uv;
      if (c4 == 0) {
        mean[b] = s[i];
        rstd[b] = rs;
      }
    }
  }
  __syncthreads();
  float acc = 0.0f;
#pragma unroll 8
  for (int k = ph; k < G; k += 4) {
    const float4 x = *reinterpret_cast<const float4*>(&us[r][4 * k]);
    const float4 w = *reinterpret_cast<const float4*>(&ws[jj][4 * k]);
    acc = fmaf(x.x, w.x, acc);
    acc = fmaf(x.y, w.y, acc);
    acc = fmaf(x.z, w.z, acc);
    acc = fmaf(x.w, w.w, acc);
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  if (ph == 0 && r0 + r < B && j0 + jj < HB) z[(long)(r0 + r) * HB + j0 + jj] = fmaxf(acc + b1v, 0.0f);
}

// y = z W2^T + b2 of one frame (the last frame's: every earlier frame's y is written by the next
// frame's MODE 2 gate kernel, with the same FMA order).  Thread = (row, output).
__global__ __launch_bounds__(256) void ssd_y_kernel(int B, int HB, int FO, const float* __restrict__ z,
                                                    const float* __restrict__ w2, const float* __restrict__ b2,
                                                    float* __restrict__ y, long y_bs) {
  const int e = blockIdx.x * 256 + threadIdx.x, b = e >> 3, o = e & 7;
  if (b >= B || o >= FO) return;
  float yv = b2[o];
  for (int j = 0; j < 64; ++j) yv = fmaf(j < HB ? z[(long)b * HB + j] : 0.0f, j < HB ? w2[(long)o * HB + j] : 0.0f, yv);
  y[(long)b * y_bs + o] = yv;
}

// Backward of the last layer of one frame: FFN backward -> LayerNorm backward -> zero-state cell
// backward, tiled 8 rows x 8 hidden units (256 workgroups at B = 64, H = 256).
//   dy_total(t) = dy(t) + mask[t] * dfeat(t+1) W_ms   (the select fed y(t) to frame t + 1)
//   dz = relu'(z) * (dy_total W2);  du = dz W1        (this tile's 8 columns of du only)
// The LayerNorm backward needs two row sums of the full du row; they are taken through W1 instead:
//   sum_k du_k gamma_k      = dz . (W1 gamma)
//   sum_k du_k gamma_k xh_k = dz . (z - b1 - W1 beta)   (u = xh gamma + beta; relu'(z) = 0 where z = 0)
// with v = [W1 gamma | W1 beta] [HB][2] computed once per backward.  Every workgroup recomputes its
// rows' dy_total / dz (8 x 6 x H + 8 x 64 x 6 FMAs); blockIdx.x == 0 writes them (saved for dW2 / dW1).
struct SsdFfnBwdArgs {
  int B, H, HB, FO, t;
  const float* dy;          // dy(t)[b * dy_bs + o]
  long dy_bs;
  const float* dfeat_next;  // dfeat(t + 1) [B][H] (null at the last frame, or when dyx_next is given)
  const float* wms;         // W_ms^T [FO][H]
  const float* dyx_next;    // dfeat(t + 1) W_ms [B][FO], from frame t + 1's bottom layer (nullable)
  const unsigned char* mask;
  const float* w1;          // [HB][H]
  const float* w2;          // [FO][HB]
  const float* b1;
  const float* v;           // [HB][2]: W1 gamma, W1 beta
  const float* z;           // z(t) [B][HB]
  float* dyt;               // [B][FO]
  float* dz;                // [B][HB]
  float* du;                // [B][H] (saved: dgamma / dbeta)
  const float* h;
  const float* x;
  const float* gamma;
  const float* mean;
  const float* rstd;
  float* g;                 // d(h + x) [B][H]
  const float* gates;
  const float* c;
  float* dG;                // [B][4H]
};

__global__ __launch_bounds__(256) void ssd_ffn_bwd_kernel(SsdFfnBwdArgs a) {
  __shared__ float dys[8][8];
  __shared__ float dzs[8][64];
  __shared__ float msum[8][2];
  __shared__ float w1s[64][9];
  const int tid = threadIdx.x, H = a.H;
  const int r0 = blockIdx.y * 8, k0 = blockIdx.x * 8;
  // phase A: dy_total; thread = (row ra, part pa of 32), 8 columns each (2 float4)
  const int ra = tid >> 5, pa = tid & 31, ba = r0 + ra;
  const bool fed = a.dfeat_next != nullptr && a.mask[a.t] != 0;
  float4 df[2], wm[8][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int kk = 8 * pa + 4 * i;
    df[i] = ld4_or0(a.dfeat_next, (long)ba * H + kk, fed && ba < a.B && kk < H);
#pragma unroll
    for (int o = 0; o < 8; ++o) wm[o][i] = ld4_or0(a.wms, (long)o * H + kk, fed && o < a.FO && kk < H);
  }
  // loads of the later phases, issued now
  float zv[2], w2v[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = pa + 32 * i;
    zv[i] = ld_or0(a.z, (long)ba * a.HB + j, ba < a.B && j < a.HB);
#pragma unroll
    for (int o = 0; o < 8; ++o) w2v[i][o] = ld_or0(a.w2, (long)o * a.HB + j, o < a.FO && j < a.HB);
  }
  float v1[2], v2[2], b1v[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = pa + 32 * i;
    v1[i] = ld_or0(a.v, 2 * j, j < a.HB);
    v2[i] = ld_or0(a.v, 2 * j + 1, j < a.HB);
    b1v[i] = ld_or0(a.b1, j, j < a.HB);
  }
  const bool fed2 = a.dyx_next != nullptr && a.mask[a.t] != 0;
  const float dyv = ld_or0(a.dy, (long)ba * a.dy_bs + (pa & 7), pa < 8 && pa < a.FO && ba < a.B) +
                    ld_or0(a.dyx_next, (long)ba * a.FO + (pa & 7), fed2 && pa < 8 && pa < a.FO && ba < a.B);
  // W1 columns k0..k0+7 of all HB rows -> LDS (thread = (row j, half))
  {
    const int j = tid >> 1, hf = tid & 1;
    if (tid < 128) {
      const float4 w = ld4_or0(a.w1, (long)j * H + k0 + 4 * hf, j < a.HB && k0 + 4 * hf < H);
      w1s[j][4 * hf] = w.x; w1s[j][4 * hf + 1] = w.y; w1s[j][4 * hf + 2] = w.z; w1s[j][4 * hf + 3] = w.w;
    }
  }
  // this thread's (row, unit) of phase D: row rd, unit kd, j phase pd
  const int rd = tid >> 5, kd = (tid >> 2) & 7, pd = tid & 3, bd = r0 + rd, kc = k0 + kd;
  const bool dv = bd < a.B && kc < H && pd == 0;
  const float hx = ld_or0(a.h, (long)bd * H + kc, dv) + ld_or0(a.x, (long)bd * H + kc, dv);
  const float gam = ld_or0(a.gamma, kc, dv);
  const float mn = ld_or0(a.mean, bd, dv), rs = ld_or0(a.rstd, bd, dv);
  const float ig = ld_or0(a.gates, (long)bd * 4 * H + kc, dv);
  const float gg = ld_or0(a.gates, (long)bd * 4 * H + 2 * H + kc, dv);
  const float og = ld_or0(a.gates, (long)bd * 4 * H + 3 * H + kc, dv);
  const float cc = ld_or0(a.c, (long)bd * H + kc, dv);
  float p[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      s = fmaf(df[i].x, wm[o][i].x, s); s = fmaf(df[i].y, wm[o][i].y, s);
      s = fmaf(df[i].z, wm[o][i].z, s); s = fmaf(df[i].w, wm[o][i].w, s);
    }
    p[o] = s;
  }
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1)
#pragma unroll
    for (int o = 0; o < 8; ++o) p[o] += __shfl_xor(p[o], m, 64);
  if (pa < 8) {
    float v = 0.0f;
#pragma unroll
    for (int o = 0; o < 8; ++o) v = (pa == o) ? dyv + p[o] : v;
    if (pa >= a.FO) v = 0.0f;
    dys[ra][pa] = v;
    if (blockIdx.x == 0 && pa < a.FO && ba < a.B) a.dyt[(long)ba * a.FO + pa] = v;
  }
  __syncthreads();
  // phase B / C: dz (thread = (row ra, j = pa, pa + 32)) and the two row sums
  float m0 = 0.0f, m1 = 0.0f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = pa + 32 * i;
    float acc = 0.0f;
#pragma unroll
    for (int o = 0; o < 8; ++o) acc = fmaf(dys[ra][o], w2v[i][o], acc);
    const float d = zv[i] > 0.0f ? acc : 0.0f;
    dzs[ra][j] = d;
    if (blockIdx.x == 0 && ba < a.B && j < a.HB) a.dz[(long)ba * a.HB + j] = d;
    m0 = fmaf(d, v1[i], m0);
    m1 = fmaf(d, (zv[i] - b1v[i]) - v2[i], m1);
  }
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) {
    m0 += __shfl_xor(m0, m, 64);
    m1 += __shfl_xor(m1, m, 64);
  }
  if (pa == 0) {
    msum[ra][0] = m0;
    msum[ra][1] = m1;
  }
  __syncthreads();
  // phase D: du for (rd, kc) over j = pd, pd + 4, ... ; then LayerNorm and cell backward
  float du = 0.0f;
#pragma unroll
  for (int jj = 0; jj < 16; ++jj) du = fmaf(dzs[rd][pd + 4 * jj], w1s[pd + 4 * jj][kd], du);
  du += __shfl_xor(du, 1, 64);
  du += __shfl_xor(du, 2, 64);
  if (!dv) return;
  a.du[(long)bd * H + kc] = du;
  const float xh = (hx - mn) * rs;
  const float gd = du * gam;
  const float gv = rs * (gd - msum[rd][0] / (float)H - xh * (msum[rd][1] / (float)H));
  a.g[(long)bd * H + kc] = gv;
  const float tc = tanhf_(cc);
  const float dc = gv * og * (1.0f - tc * tc);
  float* d = a.dG + (long)bd * 4 * H + kc;
  d[0] = dc * gg * ig * (1.0f - ig);
  d[H] = 0.0f;
  d[2 * H] = dc * ig * (1.0f - gg * gg);
  d[3 * H] = gv * tc * og * (1.0f - og);
}

// Backward of a layer below the last one, one frame: LayerNorm backward (upstream du = dX of the
// layer above) -> zero-state cell backward.  One workgroup per row; thread k = hidden unit k.
// block-wide sums of N values at once (256 threads): one LDS round, fixed order
template <int N>
__device__ __forceinline__ void block_sums256(float (&v)[N], float (*sh)[4]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = wave_sum(v[i]);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) sh[i][wave] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = (sh[i][0] + sh[i][1]) + (sh[i][2] + sh[i][3]);
  __syncthreads();
}

// With dyx given (the bottom layer of a frame): also the frame's contribution to the previous
// frame's prediction gradient through the sampling select, dyx[b][o] = dfeat[b] . W_ms[:, o] with
// dfeat = dG W_ih + g, taken as dG . vt[o] + g . wms_t[o] (vt = W_ms^T W_ih, [FM][4H], formed once
// per backward), so the frame needs no dX product of its own (decode.py forms every frame's dfeat
// in one GEMM after the loop).
__global__ __launch_bounds__(256) void ssd_ln_cell_bwd_kernel(int H, const float* __restrict__ du_in,
                                                              const float* __restrict__ h, const float* __restrict__ x,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ rstd, float* __restrict__ g,
                                                              const float* __restrict__ gates,
                                                              const float* __restrict__ c, float* __restrict__ dG,
                                                              int FM, const float* __restrict__ vt,
                                                              const float* __restrict__ wms_t,
                                                              float* __restrict__ dyx) {
  __shared__ float sh[8][4];
  const int b = blockIdx.x, k = threadIdx.x;
  const bool kv = k < H;
  const float mn = ld_or0(mean, b, true), rs = ld_or0(rstd, b, true);
  const float hx = ld_or0(h, (long)b * H + k, kv) + ld_or0(x, (long)b * H + k, kv);
  const float gam = ld_or0(gamma, k, kv);
  const float cc = ld_or0(c, (long)b * H + k, kv);
  const float ig = ld_or0(gates, (long)b * 4 * H + k, kv);
  const float gg = ld_or0(gates, (long)b * 4 * H + 2 * H + k, kv);
  const float og = ld_or0(gates, (long)b * 4 * H + 3 * H + k, kv);
  const float du = ld_or0(du_in, (long)b * H + k, kv);
  const bool ext = dyx != nullptr;
  float vi[8], vg[8], vo[8], wm[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    const bool ok = ext && kv && o < FM;
    vi[o] = ld_or0(vt, (long)o * 4 * H + k, ok);
    vg[o] = ld_or0(vt, (long)o * 4 * H + 2 * H + k, ok);
    vo[o] = ld_or0(vt, (long)o * 4 * H + 3 * H + k, ok);
    wm[o] = ld_or0(wms_t, (long)o * H + k, ok);
  }
  // LayerNorm backward: g = rstd (gd - mean(gd) - xh mean(gd xh)), gd = du * gamma
  const float xh = kv ? (hx - mn) * rs : 0.0f;
  const float gd = du * gam;
  float m[2] = {gd, gd * xh};
  block_sums256<2>(m, sh);
  const float gv = rs * (gd - m[0] / (float)H - xh * (m[1] / (float)H));
  const float tc = tanhf_(cc);
  const float dc = gv * og * (1.0f - tc * tc);
  const float d_i = dc * gg * ig * (1.0f - ig);
  const float d_g = dc * ig * (1.0f - gg * gg);
  const float d_o = gv * tc * og * (1.0f - og);
  if (kv) {
    g[(long)b * H + k] = gv;
    float* d = dG + (long)b * 4 * H + k;
    d[0] = d_i;
    d[H] = 0.0f;
    d[2 * H] = d_g;
    d[3 * H] = d_o;
  }
  if (!ext) return;  // uniform
  float p[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    p[o] = kv ? fmaf(d_i, vi[o], fmaf(d_g, vg[o], fmaf(d_o, vo[o], gv * wm[o]))) : 0.0f;
  }
  block_sums256<8>(p, sh);
  if (k < FM) {
    float v = 0.0f;
#pragma unroll
    for (int o = 0; o < 8; ++o) v = (k == o) ? p[o] : v;
    dyx[(long)b * FM + k] = v;
  }
}

// One step (T = 1) of an LSTM with a carried state: the per-frame forward of the autoregressive
// generation loops (Metaformer.prediction's generate_one_step, lstmformer.py:466-521, whose mixer
// LSTMs carry (h, c) from frame to frame).  gates = [x | h0] [W_ih | W_hh]^T + b_ih + b_hh and the
// cell in ONE launch (it was two GEMMs and a cell kernel): the same 16 rows x 4 units MFMA tile as
// ssd_gate_cell_fwd_kernel over the concatenated K = In + H (zero-padded to KMAX), the operands
// loaded branch-free from both sources (the other source's lane reads out of range, i.e. 0).
struct LstmStepArgs {
  int B, H, In;
  const float* x;    // [B][In]
  const float* h0;   // [B][H] or null (zero state)
  const float* c0;   // [B][H] or null
  const float* w_ih;  // [4H][In]
  const float* w_hh;  // [4H][H]
  const float* b_ih;
  const float* b_hh;
  float* gates;      // [B][4H] i, f, g, o (post-activation)
  float* c;          // [B][H]
  float* y;          // y[b * ldy + u]
  long ldy;
  float* hT;         // [B][H] or null
};

template <int KMAX>
__global__ __launch_bounds__(256) void lstm_step_fwd_kernel(LstmStepArgs a) {
  constexpr int LDK = KMAX + 2;
  constexpr int C4 = KMAX / 4;                      // float4 slots a row
  constexpr int NX = SSD_R * C4 / 256;              // float4 per thread per operand
  __shared__ __attribute__((aligned(16))) float Xs[SSD_R * LDK];
  __shared__ __attribute__((aligned(16))) float Ws[16 * LDK];
  __shared__ float red[4][16][17];
  __shared__ float bias[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, In = a.In;
  const int KA = In, KT = In + (a.h0 ? H : 0);
  const int r0 = blockIdx.y * SSD_R, u0 = blockIdx.x * SSD_U;
  float4 xv[NX], wv[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int e = tid + i * 256, rr = e / C4, k = 4 * (e % C4);
    const int q = rr >> 2, uu = rr & 3, b = r0 + rr, wrow = q * H + u0 + uu;
    const bool inx = k < KA, inh = k >= KA && k < KT;
    const float4 x1 = ld4_or0(a.x, (long)b * In + k, inx && b < a.B);
    const float4 x2 = ld4_or0(a.h0, (long)b * H + (k - KA), inh && b < a.B);
    const float4 w1 = ld4_or0(a.w_ih, (long)wrow * In + k, inx);
    const float4 w2 = ld4_or0(a.w_hh, (long)wrow * H + (k - KA), inh);
    xv[i] = make_float4(x1.x + x2.x, x1.y + x2.y, x1.z + x2.z, x1.w + x2.w);
    wv[i] = make_float4(w1.x + w2.x, w1.y + w2.y, w1.z + w2.z, w1.w + w2.w);
  }
  float cprev = 0.0f;
  {
    const int rr = tid >> 2, uu = tid & 3, b = r0 + rr;
    if (tid < SSD_R * SSD_U) cprev = ld_or0(a.c0, (long)b * H + u0 + uu, a.c0 && b < a.B);
  }
  if (tid < 16) {
    const int q = tid >> 2, uu = tid & 3;
    bias[tid] = ld_or0(a.b_ih, q * H + u0 + uu, true) + ld_or0(a.b_hh, q * H + u0 + uu, true);
  }
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int e = tid + i * 256, rr = e / C4, k = 4 * (e % C4);
    float2* xd = reinterpret_cast<float2*>(&Xs[rr * LDK + k]);
    xd[0] = make_float2(xv[i].x, xv[i].y);
    xd[1] = make_float2(xv[i].z, xv[i].w);
    float2* wd = reinterpret_cast<float2*>(&Ws[rr * LDK + k]);
    wd[0] = make_float2(wv[i].x, wv[i].y);
    wd[1] = make_float2(wv[i].z, wv[i].w);
  }
  __syncthreads();
  // the 4 waves take K quarters of roundup(KT, 32)
  const int l16 = lane & 15, kg = lane >> 4;
  const int kq = ((KT + 31) / 32) * 8, kb = wave * kq;
  ssd_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int k = kb; k < kb + kq; k += 8) {
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Xs[l16 * LDK + k + kg], Ws[l16 * LDK + k + kg], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(Xs[l16 * LDK + k + 4 + kg], Ws[l16 * LDK + k + 4 + kg], acc1, 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][4 * kg + i][l16] = acc0[i] + acc1[i];
  __syncthreads();
  if (tid < SSD_R * SSD_U) {
    const int rr = tid >> 2, uu = tid & 3, b = r0 + rr, u = u0 + uu;
    if (b < a.B && u < H) {
      float z[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cc = q * 4 + uu;
        z[q] = ((red[0][rr][cc] + red[1][rr][cc]) + (red[2][rr][cc] + red[3][rr][cc])) + bias[cc];
      }
      const float ig = sigmoidf_(z[0]), fg = sigmoidf_(z[1]), gg = tanhf_(z[2]), og = sigmoidf_(z[3]);
      const float cn = fg * cprev + ig * gg;
      float* gs = a.gates + (long)b * 4 * H + u;
      gs[0] = ig; gs[H] = fg; gs[2 * H] = gg; gs[3 * H] = og;
      a.c[(long)b * H + u] = cn;
      const float hv = og * tanhf_(cn);
      a.y[(long)b * a.ldy + u] = hv;
      if (a.hT) a.hT[(long)b * H + u] = hv;
    }
  }
}

}  // namespace mrg

using namespace mrg;

template <int MODE, int DBG>
static void launch_gate(const SsdFwdArgs& a, hipStream_t stream) {
  const dim3 grid(a.H / SSD_U, (a.B + SSD_R - 1) / SSD_R);
  if (a.H <= 64) ssd_gate_cell_fwd_kernel<1, MODE, DBG><<<grid, 256, 0, stream>>>(a);
  else if (a.H <= 128) ssd_gate_cell_fwd_kernel<2, MODE, DBG><<<grid, 256, 0, stream>>>(a);
  else ssd_gate_cell_fwd_kernel<4, MODE, DBG><<<grid, 256, 0, stream>>>(a);
}

static SsdFwdArgs gate_args(int B, int H, const float* xin, const float* hp, const float* rp, const float* gamma,
                            const float* beta, float eps, float* xout, float* mean, float* rstd, const float* w_ih,
                            const float* b_ih, const float* b_hh, float* gates, float* c, float* h) {
  SsdFwdArgs a = {};
  a.B = B; a.H = H; a.xin = xin; a.hp = hp; a.rp = rp; a.gamma = gamma; a.beta = beta; a.eps = eps;
  a.xout = xout; a.mean = mean; a.rstd = rstd; a.w_ih = w_ih; a.b_ih = b_ih; a.b_hh = b_hh; a.gates = gates;
  a.c = c; a.h = h;
  return a;
}

MRG_API int mrg_ssd_gate_cell_fwd(int B, int H, int mode, const float* xin, const float* hp, const float* rp,
                                  const float* gamma, const float* beta, float eps, float* xout, float* mean,
                                  float* rstd, const float* w_ih, const float* b_ih, const float* b_hh, float* gates,
                                  float* c, float* h, hipStream_t stream) {
  MRG_REQUIRE(H >= 4 && H <= 256 && H % 4 == 0, "mrg_ssd_gate_cell_fwd: H=%d (4..256, %%4)", H);
  MRG_REQUIRE(mode == 0 || mode == 1, "mrg_ssd_gate_cell_fwd: mode=%d", mode);
  MRG_REQUIRE(((uintptr_t)w_ih & 15) == 0, "mrg_ssd_gate_cell_fwd: w_ih must be 16-B aligned");
  if (B == 0) return 0;
  SsdFwdArgs a = gate_args(B, H, xin, hp, rp, gamma, beta, eps, (mode == 0 && xout == xin) ? nullptr : xout, mean,
                           rstd, w_ih, b_ih, b_hh, gates, c, h);
  if (mode == 0) launch_gate<0, 0>(a, stream);
  else launch_gate<1, 0>(a, stream);
  return check_launch("ssd_gate_cell_fwd_kernel");
}

MRG_API int mrg_ssd_feat_gate_cell_fwd(int B, int H, int HB, int FO, int F, int t, const float* p, const float* z,
                                       const float* w2, const float* b2, const unsigned char* mask, const float* ms,
                                       long ms_bs, long ms_ts, const float* wms_t, float* y, long y_bs, float* xf_ms,
                                       float* xout, const float* w_ih, const float* b_ih, const float* b_hh,
                                       float* gates, float* c, float* h, hipStream_t stream) {
  MRG_REQUIRE(H >= 4 && H <= 256 && H % 4 == 0 && HB >= 1 && HB <= 64 && FO >= 1 && FO <= 8 && t >= 0,
              "mrg_ssd_feat_gate_cell_fwd: H=%d HB=%d FO=%d t=%d", H, HB, FO, t);
  MRG_REQUIRE(t == 0 || (z && y && mask), "mrg_ssd_feat_gate_cell_fwd: frame t > 0 needs z, y, mask");
  MRG_REQUIRE((((uintptr_t)w_ih | (uintptr_t)wms_t | (uintptr_t)p) & 15) == 0,
              "mrg_ssd_feat_gate_cell_fwd: w_ih, wms_t, p must be 16-B aligned");
  if (B == 0) return 0;
  SsdFwdArgs a = gate_args(B, H, p, nullptr, nullptr, nullptr, nullptr, 0.0f, xout, nullptr, nullptr, w_ih, b_ih,
                           b_hh, gates, c, h);
  a.HB = HB; a.FO = FO; a.F = F; a.tm = t > 0 ? t - 1 : 0; a.z = t > 0 ? z : nullptr; a.w2 = w2; a.b2 = b2;
  a.mask = mask; a.ms = ms; a.ms_bs = ms_bs; a.ms_ts = ms_ts; a.wms = wms_t; a.y = y; a.y_bs = y_bs; a.xf_ms = xf_ms;
  launch_gate<2, 0>(a, stream);
  return check_launch("ssd_gate_cell_fwd_kernel<MODE 2>");
}

// Timing experiments only (tools/tools_ssd_kernels.py): the MODE 1 gate/cell kernel with parts removed.
MRG_API int mrg_ssd_gate_cell_fwd_dbg(int dbg, int B, int H, int mode, const float* xin, const float* hp,
                                      const float* rp, const float* gamma, const float* beta, float eps, float* xout,
                                      float* mean, float* rstd, const float* w_ih, const float* b_ih,
                                      const float* b_hh, float* gates, float* c, float* h, hipStream_t stream) {
  MRG_REQUIRE(H == 256 && mode == 1, "dbg: H=256, mode 1 only");
  SsdFwdArgs a = gate_args(B, H, xin, hp, rp, gamma, beta, eps, xout, mean, rstd, w_ih, b_ih, b_hh, gates, c, h);
  switch (dbg) {
    case 1: launch_gate<1, 1>(a, stream); break;
    case 2: launch_gate<1, 2>(a, stream); break;
    case 3: launch_gate<1, 3>(a, stream); break;
    default: launch_gate<1, 0>(a, stream); break;
  }
  return check_launch("ssd_gate_cell_fwd_dbg");
}

MRG_API int mrg_ssd_dx(int B, int H, const float* dG, const float* w_t, const float* g, float* dx, hipStream_t stream) {
  MRG_REQUIRE(H >= 4 && H <= 256 && H % 4 == 0, "mrg_ssd_dx: H=%d (4..256, %%4)", H);
  MRG_REQUIRE((((uintptr_t)dG | (uintptr_t)w_t) & 15) == 0, "mrg_ssd_dx: dG and w_t must be 16-B aligned");
  if (B == 0) return 0;
  const dim3 grid((H + 7) / 8, (B + 7) / 8);
  if (H <= 64) ssd_dx_kernel<192><<<grid, 256, 0, stream>>>(B, H, dG, w_t, g, dx);
  else if (H <= 128) ssd_dx_kernel<384><<<grid, 256, 0, stream>>>(B, H, dG, w_t, g, dx);
  else ssd_dx_kernel<768><<<grid, 256, 0, stream>>>(B, H, dG, w_t, g, dx);
  return check_launch("ssd_dx_kernel");
}

MRG_API int mrg_ssd_ffn_z_fwd(int B, int H, int HB, const float* hp, const float* rp, const float* gamma,
                              const float* beta, float eps, float* u, float* mean, float* rstd, const float* w1,
                              const float* b1, float* z, hipStream_t stream) {
  MRG_REQUIRE(H >= 4 && H <= 256 && H % 4 == 0 && HB >= 1 && HB <= 64, "mrg_ssd_ffn_z_fwd: H=%d HB=%d", H, HB);
  MRG_REQUIRE((((uintptr_t)hp | (uintptr_t)rp | (uintptr_t)w1 | (uintptr_t)u) & 15) == 0,
              "mrg_ssd_ffn_z_fwd: hp, rp, w1, u must be 16-B aligned");
  if (B == 0) return 0;
  const dim3 grid((HB + 7) / 8, (B + 7) / 8);
  if (H <= 64) ssd_ffn_z_kernel<1><<<grid, 256, 0, stream>>>(B, H, HB, hp, rp, gamma, beta, eps, u, mean, rstd, w1, b1, z);
  else if (H <= 128) ssd_ffn_z_kernel<2><<<grid, 256, 0, stream>>>(B, H, HB, hp, rp, gamma, beta, eps, u, mean, rstd, w1, b1, z);
  else ssd_ffn_z_kernel<4><<<grid, 256, 0, stream>>>(B, H, HB, hp, rp, gamma, beta, eps, u, mean, rstd, w1, b1, z);
  return check_launch("ssd_ffn_z_kernel");
}

MRG_API int mrg_ssd_y_fwd(int B, int HB, int FO, const float* z, const float* w2, const float* b2, float* y, long y_bs,
                          hipStream_t stream) {
  MRG_REQUIRE(HB >= 1 && HB <= 64 && FO >= 1 && FO <= 8, "mrg_ssd_y_fwd: HB=%d FO=%d", HB, FO);
  if (B == 0) return 0;
  ssd_y_kernel<<<(B * 8 + 255) / 256, 256, 0, stream>>>(B, HB, FO, z, w2, b2, y, y_bs);
  return check_launch("ssd_y_kernel");
}

MRG_API int mrg_ssd_ffn_bwd(int B, int H, int HB, int FO, int t, const float* dy, long dy_bs, const float* dfeat_next,
                            const float* dyx_next, const float* wms_t, const unsigned char* mask, const float* w1,
                            const float* w2,
                            const float* b1, const float* v, const float* z, float* dyt, float* dz, float* du,
                            const float* h, const float* x, const float* gamma, const float* mean, const float* rstd,
                            float* g, const float* gates, const float* c, float* dG, hipStream_t stream) {
  MRG_REQUIRE(H >= 4 && H <= 256 && H % 4 == 0 && HB >= 1 && HB <= 64 && FO >= 1 && FO <= 8,
              "mrg_ssd_ffn_bwd: H=%d HB=%d FO=%d", H, HB, FO);
  MRG_REQUIRE((((uintptr_t)w1 | (uintptr_t)wms_t | (uintptr_t)(dfeat_next ? dfeat_next : w1)) & 15) == 0,
              "mrg_ssd_ffn_bwd: w1, wms_t, dfeat_next must be 16-B aligned");
  if (B == 0) return 0;
  SsdFfnBwdArgs a;
  MRG_REQUIRE(!(dfeat_next && dyx_next), "mrg_ssd_ffn_bwd: dfeat_next or dyx_next, not both");
  a.B = B; a.H = H; a.HB = HB; a.FO = FO; a.t = t; a.dy = dy; a.dy_bs = dy_bs; a.dfeat_next = dfeat_next;
  a.dyx_next = dyx_next;
  a.wms = wms_t; a.mask = mask; a.w1 = w1; a.w2 = w2; a.b1 = b1; a.v = v; a.z = z; a.dyt = dyt; a.dz = dz; a.du = du;
  a.h = h; a.x = x; a.gamma = gamma; a.mean = mean; a.rstd = rstd; a.g = g; a.gates = gates; a.c = c; a.dG = dG;
  ssd_ffn_bwd_kernel<<<dim3((H + 7) / 8, (B + 7) / 8), 256, 0, stream>>>(a);
  return check_launch("ssd_ffn_bwd_kernel");
}

MRG_API int mrg_ssd_ln_cell_bwd(int B, int H, const float* du, const float* h, const float* x, const float* gamma,
                                const float* mean, const float* rstd, float* g, const float* gates, const float* c,
                                float* dG, int FM, const float* vt, const float* wms_t, float* dyx,
                                hipStream_t stream) {
  MRG_REQUIRE(H >= 1 && H <= 256 && FM >= 0 && FM <= 8, "mrg_ssd_ln_cell_bwd: H=%d (1..256) FM=%d", H, FM);
  MRG_REQUIRE(!dyx || (vt && wms_t && FM > 0), "mrg_ssd_ln_cell_bwd: dyx needs vt, wms_t, FM");
  if (B == 0) return 0;
  ssd_ln_cell_bwd_kernel<<<B, 256, 0, stream>>>(H, du, h, x, gamma, mean, rstd, g, gates, c, dG, FM, vt, wms_t, dyx);
  return check_launch("ssd_ln_cell_bwd_kernel");
}

MRG_API int mrg_lstm_step_fwd(int B, int H, int In, const float* x, const float* h0, const float* c0,
                              const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh,
                              float* gates, float* c, float* y, long ldy, float* hT, hipStream_t stream) {
  MRG_REQUIRE(H >= 4 && H % 4 == 0 && In >= 4 && In % 4 == 0 && In + H <= 512,
              "mrg_lstm_step_fwd: H=%d In=%d (multiples of 4, In + H <= 512)", H, In);
  MRG_REQUIRE((((uintptr_t)x | (uintptr_t)w_ih | (uintptr_t)(h0 ? h0 : x) | (uintptr_t)w_hh) & 15) == 0,
              "mrg_lstm_step_fwd: x, h0, w_ih, w_hh must be 16-B aligned");
  if (B == 0) return 0;
  LstmStepArgs a;
  a.B = B; a.H = H; a.In = In; a.x = x; a.h0 = h0; a.c0 = c0; a.w_ih = w_ih; a.w_hh = w_hh; a.b_ih = b_ih;
  a.b_hh = b_hh; a.gates = gates; a.c = c; a.y = y; a.ldy = ldy; a.hT = hT;
  const dim3 grid(H / SSD_U, (B + SSD_R - 1) / SSD_R);
  const int kt = In + (h0 ? H : 0);
  if (kt <= 256) lstm_step_fwd_kernel<256><<<grid, 256, 0, stream>>>(a);
  else lstm_step_fwd_kernel<512><<<grid, 256, 0, stream>>>(a);
  return check_launch("lstm_step_fwd_kernel");
}
