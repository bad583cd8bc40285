// Fused per-frame kernels of lstmformer generation (Metaformer.prediction -> head_motion_generation
// -> generate_one_step, mr_gen/model/lstmformer/lstmformer.py:426-521).
//
// Every generated frame is a T = 1 forward with zero recurrent state and empty lead
// inputs (gen_dummy_input, :549-559).  What depends on the previous frame is only the MAIN chain
// (self motion -> feature_embedding.0 -> per block: LSTM mixer, two integrators, cat_linear,
// FeedForward -> output FeedForward -> y -> next frame's self motion).  The other modalities' block-0
// encoders and, at one audio frame per prediction frame, the integrators' whole attention output
// (one visible key: softmax weight exactly 1, so MHA(q, kv) = out_proj(V(kv)) whatever q is) are
// computed for all frames at once by the host (generate.py) as large GEMMs.  Per frame and block
// this file then runs five launches instead of ~30:
//
//   gen_lstm    X = LN(ffn(prev) + prev) (block 0: X = ms_in W_fe^T + b_fe), gates = X W_ih^T + b,
//               zero-state cell -> h                                    (mixer_block.py:237-252)
//   gen_linear  Y = LN(h + X), Z = Y W^T + b                           (mixer_block.py:479-507)
//   gen_linear  M = LN(Z + Y), Y_i = LN(a_i + M), Z_i = Y_i W_i^T + b_i  (both integrators,
//               mixer_block.py:567-603)
//   gen_linear  C = [LN(Z_0 + Y_0) | LN(Z_1 + Y_1)], M3 = C W_cat^T + b  (multi_modal_metaformer.py:128-217)
//   gen_ffn     Zf = relu(M3 W1^T + b1) W2^T + b2                       (multi_modal_metaformer.py:328)
//
// and one gen_ffn for the output FeedForward with the sampling select of :487-492 folded in
// (ms_in(t + 1) = mask[t] ? y(t) : motion_s[t]).  Each launch owns 16 batch rows x 16 output
// columns per workgroup; the LayerNorms a stage consumes are recomputed from their inputs in the
// workgroup's prologue (16 rows x 256, L2-resident) instead of a launch of their own, and each
// workgroup writes its share of the normalised rows the next stage needs as a residual.
// Products on v_mfma_f32_16x16x4_f32 (exact fp32 multiply-adds; the k order differs from the
// training kernels', fp32 class).  E = 256, FeedForward bottleneck 64 (the lstmformer config).
#include "gen_loop.h"

namespace mrg {

static constexpr int GR = 16;    // batch rows per workgroup

struct GenLstmArgs {
  int B, fm;
  const float* ms;               // PRO 0: self-motion input [B][fm]
  const float* fe_w;             // feature_embedding.0 [GE][fm], bias [GE]
  const float* fe_b;
  const float* a;                // PRO 1: X = LN(a + r) (the previous block's FeedForward)
  const float* r;
  const float* ga;
  const float* be;
  float eps;
  float* xw;                     // X [B][GE] (this block's residual input), each workgroup its share
  const float* w_ih;             // [4 GE][GE]
  const float* b_ih;
  const float* b_hh;
  float* h;                      // [B][GE]
};

struct GenLinArgs {
  int B;
  const float* a[2];             // first LayerNorm inputs (PRO 2: the two halves)
  const float* r[2];
  const float* ga[2];
  const float* be[2];
  long lda;                      // row stride of a / r / a2
  const float* a2[2];            // PRO 1: second LayerNorm: Y_i = LN(a2[i] + LN(a + r))
  const float* ga2[2];
  const float* be2[2];
  float eps;
  float* xw;                     // the normalised input rows (nullable), each workgroup its share
  long ldxw;
  const float* w[2];             // weight [n][K] of the column half (PRO 1: per integrator)
  const float* bias[2];
  float* out;
  long ldo;
};

struct GenFfnArgs {
  int B, N;                      // N output columns (256, or fm for the output FeedForward)
  const float* a;                // PRO 0: X = a; PRO 1: X = LN(a + r)
  const float* r;
  const float* ga;
  const float* be;
  float eps;
  const float* w1;               // [GHB][GE]
  const float* b1;
  const float* w2;               // [N][GHB]
  const float* b2;
  float* out;                    // OUT 0: [B][N]
  float* pred;                   // OUT 1: pred[b * pred_bs + t * N + n]
  long pred_bs;
  float* ms_next;                // OUT 1: [B][N] = mask[t] ? y : ms_src
  const float* ms_src;           // motion_s frame t [B][N]
  const unsigned char* mask;     // [T] on the device
  int t;
};


// acc[16 rows x 16 cols] += X[16][k0:k0+NK] W[n][k0:k0+NK]^T on v_mfma_f32_16x16x4_f32: lane l
// supplies row / column l & 15 at k = kb + 4 (l >> 4) + j for the j-th product of a 16-k group, so
// its four operands of a group are one float4 (A and B use the same k of each product pair).
// gen_wload issues the lane's weight loads (at kernel start: independent of the prologue)
template <int NK>
__device__ __forceinline__ void gen_wload(const float* __restrict__ wrow, int k0, int lane, float4 (&w)[NK / 16]) {
#pragma unroll
  for (int i = 0; i < NK / 16; ++i) w[i] = *reinterpret_cast<const float4*>(wrow + k0 + 16 * i + 4 * (lane >> 4));
}
template <int KP, int NK>
__device__ __forceinline__ gv4 gen_mfma(const float* xs, const float4 (&w)[NK / 16], int k0, int lane, gv4 acc) {
  const int m = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < NK / 16; ++i) {
    const float4 x = *reinterpret_cast<const float4*>(xs + m * KP + k0 + 16 * i + 4 * q);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, w[i].x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, w[i].y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, w[i].z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, w[i].w, acc, 0, 0, 0);
  }
  return acc;
}

// the four waves' k-quarter partial tiles into red[4][16][17]; accumulator register i of lane l is
// row 4 (l >> 4) + i, column l & 15
__device__ __forceinline__ void gen_park(float (*red)[GR][17], int wave, int lane, gv4 acc) {
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][4 * (lane >> 4) + i][lane & 15] = acc[i];
}
__device__ __forceinline__ float gen_sum(const float (*red)[GR][17], int m, int n) {
  return (red[0][m][n] + red[1][m][n]) + (red[2][m][n] + red[3][m][n]);
}

// Every launch below first issues the loads that do not depend on the previous launch (this lane's
// weight operands, the LayerNorm gamma / beta, the biases of its outputs), then the activation rows
// (clamped past B, zeroed after), so a kernel waits about one memory round trip before its products.

// ------------------------------------------------------------------ LSTM mixer gates + cell
// grid (GE / 4 unit groups, ceil(B / 16)); column n of the tile = gate n >> 2 of unit 4 bx + (n & 3)
template <int PRO>
__global__ __launch_bounds__(256) void gen_lstm_kernel(GenLstmArgs p) {
  constexpr int KP = GE + 4;
  __shared__ __attribute__((aligned(16))) float xs[GR][KP];
  __shared__ float red[4][GR][17];
  __shared__ float msl[GR][16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.y * GR, u0 = 4 * blockIdx.x;
  const int share = GE / gridDim.x;   // X columns this workgroup writes back
  const int n = lane & 15;
  float4 w[GE / 4 / 16];
  gen_wload<GE / 4>(p.w_ih + (long)((n >> 2) * GE + u0 + (n & 3)) * GE, wave * (GE / 4), lane, w);
  // cell thread (m, j): its unit's biases
  const int cm = tid >> 2, cj = tid & 3, cu = u0 + cj;
  float bi = 0.f, bg = 0.f, bo = 0.f;
  if (tid < 4 * GR) {
    bi = p.b_ih[cu] + p.b_hh[cu];
    bg = p.b_ih[2 * GE + cu] + p.b_hh[2 * GE + cu];
    bo = p.b_ih[3 * GE + cu] + p.b_hh[3 * GE + cu];
  }
  if (PRO == 0) {
    // X = ms W_fe^T + b_fe (K = fm <= 16): the 16 rows' inputs staged in LDS, thread = column
    const int k = tid;
    float wf[16];
#pragma unroll
    for (int f = 0; f < 16; ++f) wf[f] = f < p.fm ? p.fe_w[k * p.fm + f] : 0.0f;
    const float bk = p.fe_b[k];
    if (tid < GR * 16) {
      const int m = tid >> 4, f = tid & 15;
      msl[m][f] = (f < p.fm && row0 + m < p.B) ? p.ms[(long)(row0 + m) * p.fm + f] : 0.0f;
    }
    __syncthreads();
    const bool mine = k >= blockIdx.x * share && k < (blockIdx.x + 1) * share;
#pragma unroll
    for (int m = 0; m < GR; ++m) {
      float s = 0.0f;
#pragma unroll
      for (int f = 0; f < 16; ++f) s = fmaf(msl[m][f], wf[f], s);
      const float v = row0 + m < p.B ? s + bk : 0.0f;
      if (mine && row0 + m < p.B) p.xw[(long)(row0 + m) * GE + k] = v;
      xs[m][k] = v;
    }
  } else {
    const float4 gg = gen_ld4(p.ga + 4 * lane), bb = gen_ld4(p.be + 4 * lane);
    float4 va[GR / 4], vr[GR / 4];
#pragma unroll
    for (int i = 0; i < GR / 4; ++i) {
      const long b = min(row0 + wave + 4 * i, p.B - 1);
      va[i] = gen_ld4(p.a + b * GE + 4 * lane);
      vr[i] = gen_ld4(p.r + b * GE + 4 * lane);
    }
    const int k = 4 * lane;
    const bool mine = k >= blockIdx.x * share && k < (blockIdx.x + 1) * share;
#pragma unroll
    for (int i = 0; i < GR / 4; ++i) {
      const int m = wave + 4 * i, b = row0 + m;
      float4 v = gen_ln(gen_add4(va[i], vr[i]), gg, bb, p.eps);
      if (b >= p.B) v = gen_zero4();
      else if (mine) *reinterpret_cast<float4*>(p.xw + (long)b * GE + k) = v;
      *reinterpret_cast<float4*>(&xs[m][k]) = v;
    }
  }
  __syncthreads();
  gv4 acc = gv4{0.f, 0.f, 0.f, 0.f};
  acc = gen_mfma<KP, GE / 4>(&xs[0][0], w, wave * (GE / 4), lane, acc);
  gen_park(red, wave, lane, acc);
  __syncthreads();
  if (tid < 4 * GR && row0 + cm < p.B) {
    const float zi = gen_sum(red, cm, cj) + bi;
    const float zg = gen_sum(red, cm, 8 + cj) + bg;
    const float zo = gen_sum(red, cm, 12 + cj) + bo;
    const float c = sigmoidf_(zi) * tanhf_(zg);   // f c0 + i g with c0 = 0
    p.h[(long)(row0 + cm) * GE + cu] = sigmoidf_(zo) * tanhf_(c);
  }
}

// ------------------------------------------------------------------ Linear with LayerNorm prologue
// PRO 0: X = LN(a + r)                          K = 256, grid (N / 16, rows)
// PRO 1: X = LN(a2[i] + LN(a + r)), i = half     K = 256, N = 512 (two 256-column halves)
// PRO 2: X = [LN(a[0] + r[0]) | LN(a[1] + r[1])] K = 512
template <int PRO>
__global__ __launch_bounds__(256) void gen_linear_kernel(GenLinArgs p) {
  constexpr int K = PRO == 2 ? 2 * GE : GE;
  constexpr int KP = K + 4;
  constexpr int NH = PRO == 2 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) float xs[GR][KP];
  __shared__ float red[4][GR][17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.y * GR;
  const int n0 = 16 * blockIdx.x;
  const int half = PRO == 1 ? n0 / GE : 0;           // PRO 1: integrator of this column tile
  const int tiles = PRO == 1 ? gridDim.x / 2 : gridDim.x;
  const int share = GE / tiles, sh0 = (blockIdx.x % tiles) * share;
  const int nl = n0 - half * GE;                     // first row of this half's weight
  float4 w[K / 4 / 16];
  gen_wload<K / 4>(p.w[half] + (long)(nl + (lane & 15)) * K, wave * (K / 4), lane, w);
  const float bias = p.bias[half][nl + (tid & 15)];
  const int k = 4 * lane;
  float4 gg[NH], bb[NH], g2 = gen_zero4(), b2 = gen_zero4();
#pragma unroll
  for (int hh = 0; hh < NH; ++hh) {
    gg[hh] = gen_ld4(p.ga[hh] + k);
    bb[hh] = gen_ld4(p.be[hh] + k);
  }
  if (PRO == 1) {
    g2 = gen_ld4(p.ga2[half] + k);
    b2 = gen_ld4(p.be2[half] + k);
  }
  {
    float4 va[GR / 4][NH], vr[GR / 4][NH], v2[GR / 4];
#pragma unroll
    for (int i = 0; i < GR / 4; ++i) {
      const long b = min(row0 + wave + 4 * i, p.B - 1);
#pragma unroll
      for (int hh = 0; hh < NH; ++hh) {
        va[i][hh] = gen_ld4(p.a[hh] + b * p.lda + k);
        vr[i][hh] = gen_ld4(p.r[hh] + b * p.lda + k);
      }
      if (PRO == 1) v2[i] = gen_ld4(p.a2[half] + b * p.lda + k);
    }
    const bool mine = p.xw && k >= sh0 && k < sh0 + share;
#pragma unroll
    for (int i = 0; i < GR / 4; ++i) {
      const int m = wave + 4 * i, b = row0 + m;
#pragma unroll
      for (int hh = 0; hh < NH; ++hh) {
        float4 v = gen_ln(gen_add4(va[i][hh], vr[i][hh]), gg[hh], bb[hh], p.eps);
        if (PRO == 1) v = gen_ln(gen_add4(v2[i], v), g2, b2, p.eps);
        if (b >= p.B) v = gen_zero4();
        else if (mine) *reinterpret_cast<float4*>(p.xw + b * p.ldxw + half * GE + k) = v;
        *reinterpret_cast<float4*>(&xs[m][hh * GE + k]) = v;
      }
    }
  }
  __syncthreads();
  gv4 acc = gv4{0.f, 0.f, 0.f, 0.f};
  acc = gen_mfma<KP, K / 4>(&xs[0][0], w, wave * (K / 4), lane, acc);
  gen_park(red, wave, lane, acc);
  __syncthreads();
  const int m = tid >> 4, nn = tid & 15, b = row0 + m;
  if (b < p.B) p.out[b * p.ldo + n0 + nn] = gen_sum(red, m, nn) + bias;
}

// ------------------------------------------------------------------ FeedForward (Linear-ReLU-Linear)
// the 16 x 64 hidden rows computed per workgroup (wave w: hidden columns 16w..16w+15 over K = 256),
// then the output tile 16 x 16 over K = 64 (a k-quarter per wave).  grid (ceil(N / 16), rows).
// OUT 1: the output FeedForward's y written into pred[:, t] and the next frame's self motion
template <int PRO, int OUT>
__global__ __launch_bounds__(256) void gen_ffn_kernel(GenFfnArgs p) {
  constexpr int KP = GE + 4, HP = GHB + 4;
  __shared__ __attribute__((aligned(16))) float xs[GR][KP];
  __shared__ __attribute__((aligned(16))) float hs[GR][HP];
  __shared__ float red[4][GR][17];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.y * GR;
  const int n0 = 16 * blockIdx.x;
  const int hc = 16 * wave + (lane & 15);            // this lane's hidden column
  float4 w1[GE / 16];
  gen_wload<GE>(p.w1 + (long)hc * GE, 0, lane, w1);
  const float b1 = p.b1[hc];
  const int nw = n0 + (lane & 15);
  const bool nok = nw < p.N;
  // a column past N (the output FeedForward's 6 outputs) multiplies a zero row
  float4 w2 = *reinterpret_cast<const float4*>(p.w2 + (long)(nok ? nw : 0) * GHB + 16 * wave + 4 * (lane >> 4));
  if (!nok) w2 = gen_zero4();
  const int ocol = n0 + (tid & 15);
  const float b2 = ocol < p.N ? p.b2[ocol] : 0.0f;
  {
    float4 gg = gen_zero4(), bb = gen_zero4();
    if (PRO == 1) {
      gg = gen_ld4(p.ga + 4 * lane);
      bb = gen_ld4(p.be + 4 * lane);
    }
    float4 va[GR / 4], vr[GR / 4];
#pragma unroll
    for (int i = 0; i < GR / 4; ++i) {
      const long b = min(row0 + wave + 4 * i, p.B - 1);
      va[i] = gen_ld4(p.a + b * GE + 4 * lane);
      if (PRO == 1) vr[i] = gen_ld4(p.r + b * GE + 4 * lane);
    }
#pragma unroll
    for (int i = 0; i < GR / 4; ++i) {
      const int m = wave + 4 * i;
      float4 v = va[i];
      if (PRO == 1) v = gen_ln(gen_add4(v, vr[i]), gg, bb, p.eps);
      if (row0 + m >= p.B) v = gen_zero4();
      *reinterpret_cast<float4*>(&xs[m][4 * lane]) = v;
    }
  }
  __syncthreads();
  {
    gv4 acc = gv4{0.f, 0.f, 0.f, 0.f};
    acc = gen_mfma<KP, GE>(&xs[0][0], w1, 0, lane, acc);
#pragma unroll
    for (int i = 0; i < 4; ++i) hs[4 * (lane >> 4) + i][hc] = fmaxf(acc[i] + b1, 0.0f);
  }
  __syncthreads();
  gv4 acc = gv4{0.f, 0.f, 0.f, 0.f};
  {
    const int m = lane & 15, q = lane >> 4, k = 16 * wave;
    const float4 x = *reinterpret_cast<const float4*>(&hs[m][k + 4 * q]);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, w2.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, w2.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, w2.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, w2.w, acc, 0, 0, 0);
  }
  gen_park(red, wave, lane, acc);
  __syncthreads();
  const int m = tid >> 4, nn = tid & 15, b = row0 + m;
  if (b >= p.B || ocol >= p.N) return;
  const float y = gen_sum(red, m, nn) + b2;
  if (OUT == 0) {
    p.out[(long)b * p.N + ocol] = y;
  } else {
    p.pred[(long)b * p.pred_bs + (long)p.t * p.N + ocol] = y;
    const long i = (long)b * p.N + ocol;
    p.ms_next[i] = p.mask[p.t] ? y : p.ms_src[i];
  }
}


// ------------------------------------------------------------------ the whole frame loop, one launch
// gen_loop_kernel runs every frame of the generation in ONE persistent launch.  Rows are independent
// (every frame is a zero-state T = 1 forward per batch row), so the batch is cut into groups of 8
// rows and each group is served by 16 workgroups that own 1/16 of every stage's output columns;
// stage outputs travel as {tag, value} granules (the recurrences' hand-off, lstm_common.h) through a
// ring the launch zeroes first, and a member polls the full rows it needs instead of waiting at a
// kernel boundary.  Members of a group share blockIdx % 8 (one XCD under the round-robin dispatch,
// checked at launch start: then the granules stay in that XCD's L2).  Full-row intermediates a
// member needs again (the block input X, Y, Y_0 / Y_1, M3) stay in its LDS.  Per block:
//   S1 gather Zf -> X = LN(Zf + M3) (block 0: ms_in W_fe^T + b_fe) -> 4 x (4 units x 4 gates) ->
//      zero-state cell -> publish h
//   S2 gather h -> Y = LN(h + X) -> Z = Y W^T + b            -> publish Z
//   S3 gather Z -> M = LN(Z + Y), Y_i = LN(a_i[t] + M) -> Z_i -> publish Z_0 | Z_1
//   S4 gather Z_0 | Z_1 -> [LN(Z_0 + Y_0) | LN(Z_1 + Y_1)] W_cat^T + b -> publish M3
//   S5 gather M3 -> relu(M3 W1^T + b1) (all 64, per member) W2^T + b2 -> publish Zf
// and after the last block every member computes the output FeedForward of its rows itself
// (LN(Zf + M3) -> 64 -> fm), so the next frame's self motion (the sampling select) needs no exchange;
// member 0 writes the prediction.  Tag of block k's buffers in frame t: t * nb + k + 1.
static constexpr int GL_NBMAX = 5;
static constexpr int GL_PER_BLOCK = 31;

struct GenLoopBlock {
  const float* p[GL_PER_BLOCK];       // see mrg_gen_loop for the order
};
struct GenLoopArgs {
  GenLoopBlock blk[GL_NBMAX];
  const float *fe_w, *fe_b, *ow1, *ob1, *ow2, *ob2;
  const float* ms;                    // [T][B][fm]
  const unsigned char* mask;          // [T]
  float* pred;                        // [B][T][fm]
  unsigned long long* ring;           // h | z | z01 | m3 | zf granules, then the XCC slots
  int* err;
  int B, T, fm, nb, ngroups;
  float eps;
  unsigned long long* stamps;         // diagnostics (mrg_gen_loop_debug_stamps): [T][16][32] of group 0, or null
};

// thread 0 of each member of row group 0: 100 MHz real-time stamp (s_memrealtime, one clock for every
// CU) `slot` of frame t into stamps[t][member][slot] (slot 31 of frame 0: the local-hand-off flag)
#define GL_STAMP(slot)                                                                   \
  do {                                                                                   \
    if (p.stamps && g == 0 && threadIdx.x == 0) {                                        \
      unsigned long long _t;                                                             \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
      p.stamps[((long)t * GL_MEM + j) * 32 + (slot)] = _t;                               \
    }                                                                                    \
  } while (0)

enum { GL_WIH, GL_BIH, GL_BHH, GL_L1G, GL_L1B, GL_MW, GL_MB, GL_L2G, GL_L2B,
       GL_I0, GL_I1 = GL_I0 + 6, GL_CW = GL_I1 + 6, GL_CB, GL_FW1, GL_FB1, GL_FW2, GL_FB2, GL_FLG, GL_FLB,
       GL_ATT0, GL_ATT1 };   // integrator i: GL_Ii + {0 ln1 g, 1 ln1 b, 2 w, 3 b, 4 ln2 g, 5 ln2 b}
static_assert(GL_ATT1 + 1 == GL_PER_BLOCK, "gen loop pointer table");


__global__ __launch_bounds__(256) void gen_loop_kernel(GenLoopArgs p) {
  constexpr int XP = GE + 4, AP = 2 * GE + 4, HP = GHB + 4;
  __shared__ __attribute__((aligned(16))) float A[16][AP];      // the stage's product operand (rows 8..15 zero)
  __shared__ __attribute__((aligned(16))) float Xs[GL_ROWS][XP];
  __shared__ __attribute__((aligned(16))) float Ys[GL_ROWS][XP];
  __shared__ __attribute__((aligned(16))) float Y01[GL_ROWS][AP];
  __shared__ __attribute__((aligned(16))) float M3[GL_ROWS][XP];
  __shared__ __attribute__((aligned(16))) float hs[16][HP];
  __shared__ float red[4][4][16][17];
  __shared__ __attribute__((aligned(16))) float msin[GL_ROWS][16];
  __shared__ float fe_s[16][GE];   // feature_embedding.0 W^T (rows past fm zero) and its bias
  __shared__ float feb_s[GE];
  __shared__ int sdead, xflag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % p.ngroups, j = blockIdx.x / p.ngroups;   // group (8 rows), member (1/16 of columns)
  const int r0 = GL_ROWS * g, B = p.B, T = p.T, fm = p.fm;
  const float eps = p.eps;
  unsigned long long* bh = p.ring;
  unsigned long long* bz = bh + (long)B * GE;
  unsigned long long* bz01 = bz + (long)B * GE;
  unsigned long long* bm3 = bz01 + (long)B * 2 * GE;
  unsigned long long* bzf = bm3 + (long)B * GE;
  unsigned long long* slots = bzf + (long)B * GE;
  bool dead = false;
  for (int i = tid; i < 16 * AP; i += 256) (&A[0][0])[i] = 0.0f;
  for (int f = 0; f < 16; ++f) fe_s[f][tid] = f < p.fm ? p.fe_w[tid * p.fm + f] : 0.0f;
  feb_s[tid] = p.fe_b[tid];
  if (tid == 0) sdead = 0;
  const int local = group_on_one_xcd<GL_MEM>(slots + (long)g * GL_MEM, j, p.err, dead, &xflag);
  if (tid < GL_ROWS * 16) {   // frame 0's self motion
    const int m = tid >> 4, f = tid & 15;
    msin[m][f] = (f < fm && r0 + m < B) ? p.ms[(long)(r0 + m) * fm + f] : 0.0f;
  }
  __syncthreads();
  const int m8 = tid >> 4, n16 = tid & 15;   // epilogue thread -> (row, column of the tile), rows < 8 used
  const bool ep = tid < GL_ROWS * 16 && r0 + m8 < B;
  const int nl = lane & 15;                  // this lane's tile column (weight row) in the products
  if (p.stamps && g == 0 && threadIdx.x == 0) p.stamps[(long)j * 32 + 31] = (unsigned long long)local;
  for (int t = 0; t < T && !sdead; ++t) {
    GL_STAMP(0);
    for (int k = 0; k < p.nb; ++k) {
      const float* const* w = p.blk[k].p;
      const unsigned tag = (unsigned)(t * p.nb + k + 1);
      // ---- S1: X, gates of units 16 j .. 16 j + 15 (tile q: units 16 j + 4 q + (n & 3), gate n >> 2), cell
      {
        GlW<GE> f[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          gl_wload<GE>(f[q], w[GL_WIH] + (long)((nl >> 2) * GE + 16 * j + 4 * q + (nl & 3)) * GE, wave, lane);
        float bi = 0.f, bg = 0.f, bo = 0.f;
        const int u = 16 * j + n16;
        if (tid < GL_ROWS * 16) {
          bi = w[GL_BIH][u] + w[GL_BHH][u];
          bg = w[GL_BIH][2 * GE + u] + w[GL_BHH][2 * GE + u];
          bo = w[GL_BIH][3 * GE + u] + w[GL_BHH][3 * GE + u];
        }
        if (k == 0) {
          // all 16 self-motion columns from LDS, unrolled (msin and fe_s are zero past fm: the same
          // sums), so the reads issue back to back instead of one round trip per column
          const int c = tid;
          float wv[16];
#pragma unroll
          for (int f = 0; f < 16; ++f) wv[f] = fe_s[f][c];
          const float bc = feb_s[c];
#pragma unroll
          for (int m = 0; m < GL_ROWS; ++m) {
            float acc = 0.0f;
#pragma unroll
            for (int f4 = 0; f4 < 4; ++f4) {
              const float4 ms4 = *reinterpret_cast<const float4*>(&msin[m][4 * f4]);
              acc = fmaf(ms4.x, wv[4 * f4], acc);
              acc = fmaf(ms4.y, wv[4 * f4 + 1], acc);
              acc = fmaf(ms4.z, wv[4 * f4 + 2], acc);
              acc = fmaf(ms4.w, wv[4 * f4 + 3], acc);
            }
            const float v = r0 + m < B ? acc + bc : 0.0f;
            Xs[m][c] = v;
            A[m][c] = v;
          }
        } else {
          const float* const* wp = p.blk[k - 1].p;
          const GlLn ln = gl_lnp(wp[GL_FLG], wp[GL_FLB], lane);
          gl_gather<GE>(bzf, r0, B, tag - 1, &A[0][0], AP, p.err, dead, &sdead);
          __syncthreads();
          for (int m = wave; m < GL_ROWS; m += 4) gl_ln_row(A[m], M3[m], ln, eps, Xs[m], A[m], lane);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) gl_park(red, q, wave, lane, gl_mma<GE>(&A[0][0], AP, f[q], lane, wave));
        __syncthreads();
        if (ep) {
          const int q = n16 >> 2, jj = n16 & 3;
          const float zi = gl_sum(red, q, m8, jj) + bi;
          const float zg = gl_sum(red, q, m8, 8 + jj) + bg;
          const float zo = gl_sum(red, q, m8, 12 + jj) + bo;
          const float c = sigmoidf_(zi) * tanhf_(zg);   // f c0 + i g with c0 = 0
          put_granule(bh + (long)(r0 + m8) * GE + u, tag, sigmoidf_(zo) * tanhf_(c), local);
        }
        GL_STAMP(1 + 5 * k);
      }
      // ---- S2: Y = LN(h + X), Z = Y W_m^T + b
      {
        GlW<GE> f;
        gl_wload<GE>(f, w[GL_MW] + (long)(16 * j + nl) * GE, wave, lane);
        const GlLn ln = gl_lnp(w[GL_L1G], w[GL_L1B], lane);
        const float bias = w[GL_MB][16 * j + n16];
        gl_gather<GE>(bh, r0, B, tag, &A[0][0], AP, p.err, dead, &sdead);
        __syncthreads();
        for (int m = wave; m < GL_ROWS; m += 4) gl_ln_row(A[m], Xs[m], ln, eps, Ys[m], A[m], lane);
        __syncthreads();
        gl_park(red, 0, wave, lane, gl_mma<GE>(&A[0][0], AP, f, lane, wave));
        __syncthreads();
        if (ep) put_granule(bz + (long)(r0 + m8) * GE + 16 * j + n16, tag, gl_sum(red, 0, m8, n16) + bias, local);
        GL_STAMP(2 + 5 * k);
      }
      // ---- S3: M = LN(Z + Y), Y_i = LN(a_i + M), Z_i = Y_i W_i^T + b_i
      {
        GlW<GE> f[2];
        GlLn l1[2];
        float bias[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          gl_wload<GE>(f[i], w[GL_I0 + 6 * i + 2] + (long)(16 * j + nl) * GE, wave, lane);
          l1[i] = gl_lnp(w[GL_I0 + 6 * i + 0], w[GL_I0 + 6 * i + 1], lane);
          bias[i] = w[GL_I0 + 6 * i + 3][16 * j + n16];
        }
        const GlLn ln = gl_lnp(w[GL_L2G], w[GL_L2B], lane);
        float4 av[2][2];   // this wave's rows' attention outputs (frame t), loaded before the poll
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
          for (int i = 0; i < 2; ++i)
            av[rr][i] = gen_ld4(w[GL_ATT0 + i] + ((long)t * B + min(r0 + wave + 4 * rr, B - 1)) * GE + 4 * lane);
        gl_gather<GE>(bz, r0, B, tag, &A[0][0], AP, p.err, dead, &sdead);
        __syncthreads();
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
          const int m = wave + 4 * rr;
          const float4 mv = gen_ln(gen_add4(*reinterpret_cast<const float4*>(&A[m][4 * lane]),
                                            *reinterpret_cast<const float4*>(&Ys[m][4 * lane])),
                                   ln.g, ln.b, eps);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const float4 y = gen_ln(gen_add4(av[rr][i], mv), l1[i].g, l1[i].b, eps);
            *reinterpret_cast<float4*>(&Y01[m][GE * i + 4 * lane]) = y;
            *reinterpret_cast<float4*>(&A[m][GE * i + 4 * lane]) = y;
          }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 2; ++i) gl_park(red, i, wave, lane, gl_mma<GE>(&A[0][0] + GE * i, AP, f[i], lane, wave));
        __syncthreads();
        if (ep) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
            put_granule(bz01 + (long)(r0 + m8) * 2 * GE + GE * i + 16 * j + n16, tag, gl_sum(red, i, m8, n16) + bias[i],
                        local);
        }
        GL_STAMP(3 + 5 * k);
      }
      // ---- S4: M3 = [LN(Z_0 + Y_0) | LN(Z_1 + Y_1)] W_cat^T + b
      {
        GlW<2 * GE> f;
        gl_wload<2 * GE>(f, w[GL_CW] + (long)(16 * j + nl) * 2 * GE, wave, lane);
        GlLn l2[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) l2[i] = gl_lnp(w[GL_I0 + 6 * i + 4], w[GL_I0 + 6 * i + 5], lane);
        const float bias = w[GL_CB][16 * j + n16];
        gl_gather<2 * GE>(bz01, r0, B, tag, &A[0][0], AP, p.err, dead, &sdead);
        __syncthreads();
        for (int m = wave; m < GL_ROWS; m += 4)
#pragma unroll
          for (int i = 0; i < 2; ++i) gl_ln_row(A[m] + GE * i, Y01[m] + GE * i, l2[i], eps, A[m] + GE * i, nullptr, lane);
        __syncthreads();
        gl_park(red, 0, wave, lane, gl_mma<2 * GE>(&A[0][0], AP, f, lane, wave));
        __syncthreads();
        if (ep) put_granule(bm3 + (long)(r0 + m8) * GE + 16 * j + n16, tag, gl_sum(red, 0, m8, n16) + bias, local);
        GL_STAMP(4 + 5 * k);
      }
      // ---- S5: Zf = relu(M3 W1^T + b1) W2^T + b2 (all 64 hidden columns per member, wave w: 16 w ..)
      {
        GlW<4 * GE> f1;
        gl_wload<4 * GE>(f1, w[GL_FW1] + (long)(16 * wave + nl) * GE, 0, lane);
        GlW<GHB> f2;
        gl_wload<GHB>(f2, w[GL_FW2] + (long)(16 * j + nl) * GHB, wave, lane);
        const int hc = 16 * wave + nl;
        const float b1 = w[GL_FB1][hc];
        const float bias = w[GL_FB2][16 * j + n16];
        gl_gather<GE>(bm3, r0, B, tag, &A[0][0], AP, p.err, dead, &sdead);
        __syncthreads();
        for (int i = tid; i < GL_ROWS * GE; i += 256) M3[i / GE][i % GE] = A[i / GE][i % GE];
        {
          const gv4 acc = gl_mma<4 * GE>(&A[0][0], AP, f1, lane, 0);
#pragma unroll
          for (int i = 0; i < 4; ++i) hs[4 * (lane >> 4) + i][hc] = fmaxf(acc[i] + b1, 0.0f);
        }
        __syncthreads();
        gl_park(red, 0, wave, lane, gl_mma<GHB>(&hs[0][0], HP, f2, lane, wave));
        __syncthreads();
        if (ep) put_granule(bzf + (long)(r0 + m8) * GE + 16 * j + n16, tag, gl_sum(red, 0, m8, n16) + bias, local);
        GL_STAMP(5 + 5 * k);
      }
    }
    // ---- output FeedForward of this group's rows (every member), the sampling select
    {
      const float* const* wl = p.blk[p.nb - 1].p;
      GlW<4 * GE> f1;
      gl_wload<4 * GE>(f1, p.ow1 + (long)(16 * wave + nl) * GE, 0, lane);
      // columns past fm multiply zeroed fragments of a clamped (valid) weight row
      GlW<GHB> f2;
      gl_wload<GHB>(f2, p.ow2 + (long)(nl < fm ? nl : 0) * GHB, wave, lane);
      if (nl >= fm) f2.v[0] = make_float4(0.f, 0.f, 0.f, 0.f);
      const GlLn ln = gl_lnp(wl[GL_FLG], wl[GL_FLB], lane);
      const int hc = 16 * wave + nl;
      const float b1 = p.ob1[hc];
      const float b2 = n16 < fm ? p.ob2[n16] : 0.0f;
      gl_gather<GE>(bzf, r0, B, (unsigned)(t * p.nb + p.nb), &A[0][0], AP, p.err, dead, &sdead);
      __syncthreads();
      for (int m = wave; m < GL_ROWS; m += 4) gl_ln_row(A[m], M3[m], ln, eps, A[m], nullptr, lane);
      __syncthreads();
      {
        const gv4 acc = gl_mma<4 * GE>(&A[0][0], AP, f1, lane, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) hs[4 * (lane >> 4) + i][hc] = fmaxf(acc[i] + b1, 0.0f);
      }
      __syncthreads();
      gl_park(red, 0, wave, lane, gl_mma<GHB>(&hs[0][0], HP, f2, lane, wave));
      __syncthreads();
      if (tid < GL_ROWS * 16) {
        const int b = r0 + m8;
        float nxt = 0.0f;
        if (n16 < fm && b < B) {
          const float y = gl_sum(red, 0, m8, n16) + b2;
          if (j == 0) p.pred[((long)b * T + t) * fm + n16] = y;
          nxt = p.mask[t] ? y : p.ms[((long)t * B + b) * fm + n16];
        }
        msin[m8][n16] = nxt;
      }
      if (dead) sdead = 1;
      __syncthreads();
      GL_STAMP(30);
    }
  }
}

}  // namespace mrg

using namespace mrg;

static int gen_rows(int B) { return (B + GR - 1) / GR; }

// X [B][256] from the self-motion input (block 0: ms W_fe^T + b_fe, fm <= 16) or from the previous
// block's FeedForward (LN(a + r)); gates = X W_ih^T + b_ih + b_hh; zero-state cell -> h [B][256].
MRG_API int mrg_gen_lstm(int B, int fm, const float* ms, const float* fe_w, const float* fe_b, const float* a,
                         const float* r, const float* ga, const float* be, float eps, float* xw, const float* w_ih,
                         const float* b_ih, const float* b_hh, float* h, hipStream_t stream) {
  if (B == 0) return 0;
  MRG_REQUIRE(ms ? (fm >= 1 && fm <= 16 && fe_w && fe_b) : (a && r && ga && be),
              "mrg_gen_lstm: give ms + feature embedding (fm <= 16) or the LayerNorm inputs");
  GenLstmArgs p{B, fm, ms, fe_w, fe_b, a, r, ga, be, eps, xw, w_ih, b_ih, b_hh, h};
  const dim3 grid(GE / 4, gen_rows(B));
  if (ms) klaunch(gen_lstm_kernel<0>, grid, 256, 0, stream, p);
  else klaunch(gen_lstm_kernel<1>, grid, 256, 0, stream, p);
  return check_launch("gen_lstm_kernel");
}

// mode 0: out [B][256] = LN(a + r) W^T + b, the normalised rows into xw [B][256]
// mode 1: the two integrators: M = LN(a + r) (ga[0]), Y_i = LN(a2[i] + M) (ga2[i]) into xw[:, 256 i:],
//         out[:, 256 i:] = Y_i W_i^T + b_i   (out, xw [B][512])
// mode 2: out [B][256] = [LN(a[0] + r[0]) | LN(a[1] + r[1])] W^T + b   (W [256][512]; a, r of stride lda)
MRG_API int mrg_gen_linear(int mode, int B, const float* const* a, const float* const* r, const float* const* ga,
                           const float* const* be, long lda, const float* const* a2, const float* const* ga2,
                           const float* const* be2, float eps, float* xw, long ldxw, const float* const* w,
                           const float* const* bias, float* out, long ldo, hipStream_t stream) {
  if (B == 0) return 0;
  MRG_REQUIRE(mode >= 0 && mode <= 2 && a && r && ga && be && w && bias && out,
              "mrg_gen_linear: bad arguments (mode %d)", mode);
  GenLinArgs p{};
  p.B = B;
  const int nh = mode == 0 ? 1 : 2;
  for (int i = 0; i < 2; ++i) {
    const int s = (mode == 2 && i < nh) ? i : 0;
    p.a[i] = a[s]; p.r[i] = r[s]; p.ga[i] = ga[s]; p.be[i] = be[s];
    const int t = (mode == 1) ? i : 0;
    p.w[i] = w[t]; p.bias[i] = bias[t];
    if (mode == 1) {
      MRG_REQUIRE(a2 && ga2 && be2, "mrg_gen_linear: mode 1 needs the second LayerNorm's inputs");
      p.a2[i] = a2[i]; p.ga2[i] = ga2[i]; p.be2[i] = be2[i];
    }
  }
  p.lda = lda; p.eps = eps; p.xw = xw; p.ldxw = ldxw; p.out = out; p.ldo = ldo;
  const dim3 grid(mode == 1 ? 2 * GE / 16 : GE / 16, gen_rows(B));
  if (mode == 0) klaunch(gen_linear_kernel<0>, grid, 256, 0, stream, p);
  else if (mode == 1) klaunch(gen_linear_kernel<1>, grid, 256, 0, stream, p);
  else klaunch(gen_linear_kernel<2>, grid, 256, 0, stream, p);
  return check_launch("gen_linear_kernel");
}

// FeedForward 256 -> 64 -> ReLU -> N of X = a (r null) or LN(a + r).  pred null: out [B][N] (N = 256).
// pred given (the output FeedForward, N <= 16): y into pred[b * pred_bs + t * N + n] and
// ms_next [B][N] = mask[t] ? y : ms_src (the next frame's self motion, lstmformer.py:487-492).
MRG_API int mrg_gen_ffn(int B, int N, const float* a, const float* r, const float* ga, const float* be, float eps,
                        const float* w1, const float* b1, const float* w2, const float* b2, float* out, float* pred,
                        long pred_bs, float* ms_next, const float* ms_src, const unsigned char* mask, int t,
                        hipStream_t stream) {
  if (B == 0) return 0;
  MRG_REQUIRE(a && w1 && b1 && w2 && b2 && (r == nullptr || (ga && be)), "mrg_gen_ffn: bad arguments");
  MRG_REQUIRE(pred ? (N >= 1 && N <= 16 && ms_next && ms_src && mask) : (N == GE && out),
              "mrg_gen_ffn: N = 256 with out, or N <= 16 with pred / ms_next / ms_src / mask (N=%d)", N);
  GenFfnArgs p{B, N, a, r, ga, be, eps, w1, b1, w2, b2, out, pred, pred_bs, ms_next, ms_src, mask, t};
  const dim3 grid((N + 15) / 16, gen_rows(B));
  if (r && pred) klaunch(gen_ffn_kernel<1, 1>, grid, 256, 0, stream, p);
  else if (r) klaunch(gen_ffn_kernel<1, 0>, grid, 256, 0, stream, p);
  else if (pred) klaunch(gen_ffn_kernel<0, 1>, grid, 256, 0, stream, p);
  else klaunch(gen_ffn_kernel<0, 0>, grid, 256, 0, stream, p);
  return check_launch("gen_ffn_kernel");
}

static unsigned long long* g_gen_stamps = nullptr;
// Diagnostics (tools/gen_stamps.py): later mrg_gen_loop launches write row group 0's members' per-stage
// real-time (10 ns) stamps into buf ([T][16 members][32] u64; slot 31 of frame 0: the local hand-off
// flag); null = off.
MRG_API int mrg_gen_loop_debug_stamps(void* buf) {
  g_gen_stamps = static_cast<unsigned long long*>(buf);
  return 0;
}

// Bytes of the granule ring mrg_gen_loop needs (zeroed by the caller before every launch).
MRG_API long mrg_gen_loop_ring_bytes(int B) {
  const int ng = (B + GL_ROWS - 1) / GL_ROWS;
  return ((long)B * 6 * GE + (long)ng * GL_MEM) * 8;
}

// 1 when the whole persistent grid (16 workgroups per 8 batch rows) can be resident on `cus` CUs.
MRG_API int mrg_gen_loop_fits(int B, int cus) {
  const long nblk = (long)GL_MEM * ((B + GL_ROWS - 1) / GL_ROWS);
  return fits(gen_loop_kernel, 256, nblk, cus > 0 ? cus : device_cus()) ? 1 : 0;
}

// The whole generation frame loop in one persistent launch (gen_loop_kernel above): nb <= 5 blocks.
// ptrs (host array, 31 nb + 6 device pointers): per block w_ih, b_ih, b_hh, ln1 g / b (mixer
// LayerNorm), mixer Linear w / b, ln2 g / b (the mixer FeedForward's LayerNorm), per integrator i
// (ln1 g / b of the attention residual, FeedForward w / b, ln2 g / b), cat_linear w / b, block
// FeedForward w1 / b1 / w2 / b2, its LayerNorm g / b, the integrators' attention outputs a_0 / a_1
// [T][B][256]; then feature_embedding.0 w / b and the output FeedForward w1 / b1 / w2 / b2.
// ms [T][B][fm] (padding zeroed), mask [T] bytes, pred [B][T][fm]; ring: mrg_gen_loop_ring_bytes of
// zeroed memory; err: the recurrences' error flag (a hand-off poll that times out sets it).
MRG_API int mrg_gen_loop(int B, int T, int fm, int nb, float eps, const void* const* ptrs, int nptrs, const float* ms,
                         const unsigned char* mask, float* pred, void* ring, int* err, hipStream_t stream) {
  if (B == 0 || T == 0) return 0;
  MRG_REQUIRE(nb >= 1 && nb <= GL_NBMAX && nptrs == GL_PER_BLOCK * nb + 6 && fm >= 1 && fm <= 16 && ptrs && ms &&
                  mask && pred && ring && err,
              "mrg_gen_loop: bad arguments (B=%d nb=%d fm=%d nptrs=%d)", B, nb, fm, nptrs);
  MRG_REQUIRE(mrg_gen_loop_fits(B, 0) == 1, "mrg_gen_loop: %d workgroups cannot all be resident (B=%d)",
              GL_MEM * ((B + GL_ROWS - 1) / GL_ROWS), B);
  GenLoopArgs a{};
  for (int k = 0; k < nb; ++k)
    for (int i = 0; i < GL_PER_BLOCK; ++i) {
      a.blk[k].p[i] = static_cast<const float*>(ptrs[k * GL_PER_BLOCK + i]);
      MRG_REQUIRE(a.blk[k].p[i] != nullptr, "mrg_gen_loop: null pointer %d of block %d", i, k);
    }
  const float* const* gp = reinterpret_cast<const float* const*>(ptrs + GL_PER_BLOCK * nb);
  a.fe_w = gp[0]; a.fe_b = gp[1]; a.ow1 = gp[2]; a.ob1 = gp[3]; a.ow2 = gp[4]; a.ob2 = gp[5];
  a.ms = ms; a.mask = mask; a.pred = pred; a.ring = static_cast<unsigned long long*>(ring); a.err = err;
  a.B = B; a.T = T; a.fm = fm; a.nb = nb; a.ngroups = (B + GL_ROWS - 1) / GL_ROWS; a.eps = eps;
  a.stamps = g_gen_stamps;
  klaunch(gen_loop_kernel, dim3(GL_MEM * a.ngroups), 256, 0, stream, a);
  return check_launch("gen_loop_kernel");
}
