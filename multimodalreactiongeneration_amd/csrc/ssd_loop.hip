// The forward frame loop of lstm_with_sampling's scheduled-sampling decode (BASELINE configs[2]) in
// ONE persistent launch.
//
// Reference: LSTMwithSample.prediction -> head_motion_generation -> generate_one_step
// (mr_gen/model/lstm_with_sampling/lstm_with_sample.py:339-433).  decode.hip runs the same chain as
// L + 1 launches per frame (decode.py, _SSDecodeFn.forward); each launch costs a kernel boundary
// (~5 us at 64 rows) for ~1 us of work.  Here the batch is cut into groups of 8 rows served by 16
// workgroups each (gen_loop.h, the generation loop's layout), member j owning hidden units
// 16 j .. 16 j + 15 of every layer.  Per frame t:
//   L0  X_0 = P(t) + ms_in(t) W_ms^T (every member the full rows, in LDS) -> gates of its 16 units
//       (4 MFMA tiles of 4 units x 4 gates, v_mfma_f32_16x16x4_f32) -> zero-state cell -> publish h_0
//   Li  gather h_{i-1} -> X_i = LN(h_{i-1} + X_{i-1}) (full rows, LDS) -> gates -> cell -> publish h_i
//   F   gather h_{L-1} -> U = LN(h_{L-1} + X_{L-1}) -> Z = relu(U W1^T + b1) (all 64 hidden columns,
//       per member) -> y = Z W2^T + b2 -> ms_in(t + 1) = mask[t] ? y : ms[t]  (no exchange: every
//       member holds its rows' next input)
// so a frame is L hand-offs instead of L + 1 kernel boundaries.  The loop stores the post-activation
// gates, c and h of every layer and X_0 (member j its 16 units, the per-frame kernels' layout);
// everything else the backward reads is formed from those after the loop by decode.py (the
// LayerNorms X_i / U with their statistics, Z, y, X_f's ms columns: two LayerNorm launches, two
// products).  Storing the row-wide values inside the loop fell on one member, whose extra code held it
// ~1.2 us behind its group at every stage.  Hand-off buffers alternate by frame parity: a slot is
// rewritten two frames later, after every reader of it has passed the next frame's last gather.
#include "gen_loop.h"

namespace mrg {

static constexpr int SL_MAXL = 4;        // layered LSTM depth
static constexpr int SL_PER_LAYER = 9;   // see mrg_ssd_loop_fwd

struct SsdLoopLayer {
  const float *w_ih, *b_ih, *b_hh, *ln_g, *ln_b;   // ln: the LayerNorm after this layer
  float *X, *G, *C, *Hs;                          // [T][B][H] (layer 0 only), [T][B][4H], [T][B][H], [T][B][H]
};
struct SsdLoopArgs {
  SsdLoopLayer L[SL_MAXL];
  const float* P;                 // [T][B][H] feature projection of [sampler | partner] + b_f
  const float* wms;               // W_ms^T [FO][H]
  const float *w1, *b1, *w2, *b2; // FFN [HB][H], [HB], [FO][HB], [FO]
  const float* ms;                // ms[b * ms_bs + t * ms_ts + o]
  long ms_bs, ms_ts;
  const unsigned char* mask;      // [T]
  unsigned long long* ring;       // 2 x L x [B][H] granules, then the XCC slots
  int* err;
  int B, T, FO, nl, ngroups;
  float eps;
  unsigned long long* stamps;     // diagnostics (mrg_ssd_loop_debug_stamps): [T][16][16] of row group 0, or null
};

// thread 0 of each member of group 0: 100 MHz real-time stamp (s_memrealtime: one clock for every CU)
// `slot` of frame t into stamps[t][member][slot] (frame 0 of each member: slot 15 the local hand-off
// flag, slot 14 the hardware id register)
#define SL_STAMP(slot)                                                                   \
  do {                                                                                   \
    if (p.stamps && g == 0 && threadIdx.x == 0) {                                        \
      unsigned long long _t;                                                             \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
      p.stamps[((long)t * GL_MEM + j) * 16 + (slot)] = _t;                               \
    }                                                                                    \
  } while (0)
#define SL_STAMP_ID()                                                                    \
  do {                                                                                   \
    if (p.stamps && g == 0 && threadIdx.x == 0) {                                        \
      unsigned _id;                                                                      \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(_id));                  \
      p.stamps[(long)j * 16 + 15] = (unsigned long long)local;                           \
      p.stamps[(long)j * 16 + 14] = (unsigned long long)_id;                             \
    }                                                                                    \
  } while (0)

__global__ __launch_bounds__(256) void ssd_loop_kernel(SsdLoopArgs p) {
  constexpr int AP = GE + 4, HP = GHB + 4;
  __shared__ __attribute__((aligned(16))) float A[16][AP];     // the stage's product operand (rows 8..15 zero)
  __shared__ __attribute__((aligned(16))) float Xs[GL_ROWS][AP]; // the current layer's input rows
  __shared__ __attribute__((aligned(16))) float hs[16][HP];     // Z (rows 8..15 unused)
  __shared__ float red[4][4][16][17];
  __shared__ __attribute__((aligned(16))) float msin[GL_ROWS][16];
  __shared__ float wms_s[16][GE];                               // W_ms^T (rows past FO unused)
  __shared__ float bias_s[SL_MAXL][4][16];                      // b_ih + b_hh of this member's units
  // layer 0's 64 W_ih rows of this member (row 16 q + n: the tile-q column n of the products), resident:
  // layer 0 has no hand-off wait to hide a weight fetch under
  __shared__ __attribute__((aligned(16))) float W0s[64][AP];
  __shared__ float Ps[GL_ROWS][GE];                             // P rows of the next frame
  __shared__ int sdead, xflag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % p.ngroups, j = blockIdx.x / p.ngroups;   // group (8 rows), member (16 units)
  const int r0 = GL_ROWS * g, B = p.B, T = p.T, FO = p.FO, nl = p.nl;
  const long BH = (long)B * GE;
  const float eps = p.eps;
  unsigned long long* slots = p.ring + 2L * nl * BH;
  bool dead = false;
  for (int i = tid; i < 16 * AP; i += 256) (&A[0][0])[i] = 0.0f;
  for (int o = 0; o < 16; ++o) wms_s[o][tid] = o < FO ? p.wms[(long)o * GE + tid] : 0.0f;
  if (tid < 64 * nl) {
    const int i = tid >> 6, q = (tid >> 4) & 3, n = tid & 15;
    bias_s[i][q][n] = p.L[i].b_ih[q * GE + 16 * j + n] + p.L[i].b_hh[q * GE + 16 * j + n];
  }
  for (int e = tid; e < 64 * (GE / 4); e += 256) {
    const int rr = e / (GE / 4), k4 = e % (GE / 4), q = rr >> 4, n = rr & 15;
    *reinterpret_cast<float4*>(&W0s[rr][4 * k4]) = *reinterpret_cast<const float4*>(
        p.L[0].w_ih + (long)((n >> 2) * GE + 16 * j + 4 * q + (n & 3)) * GE + 4 * k4);
  }
  if (tid == 0) sdead = 0;
  const int local = group_on_one_xcd<GL_MEM>(slots + (long)g * GL_MEM, j, p.err, dead, &xflag);
  if (tid < GL_ROWS * 16) {   // ms_in(0) = ms[0]
    const int m = tid >> 4, o = tid & 15;
    msin[m][o] = (o < FO && r0 + m < B) ? p.ms[(long)(r0 + m) * p.ms_bs + o] : 0.0f;
  }
  __syncthreads();
  const int m8 = tid >> 4, n16 = tid & 15;   // epilogue thread -> (row, tile column), rows < 8 used
  const int b8 = r0 + m8;
  const bool ep = tid < GL_ROWS * 16 && b8 < B;
  const int c16 = lane & 15;                 // this lane's tile column (weight row) in the products
  const int u = 16 * j + n16;                // the epilogue thread's hidden unit
  SL_STAMP_ID();
  // The stores of a layer's gates, c and h (and X_0) are deferred to just after the NEXT hand-off poll:
  // on gfx9 a store holds a vmcnt slot until the memory acknowledges it, and the counter retires in
  // order, so stores issued before a poll would sit in front of the poll's loads.
  int pl = -1;                         // pending layer (-1: none)
  long prt = 0;                        // its frame's first row
  float pg[4] = {0.f, 0.f, 0.f, 0.f}, pc = 0.f, ph = 0.f, px = 0.f;
  auto flush = [&]() {
    if (pl >= 0 && ep) {
      const SsdLoopLayer& L = p.L[pl];
      const long row = prt + b8;
      float* gs = L.G + row * 4 * GE + u;
      gs[0] = pg[0]; gs[GE] = pg[1]; gs[2 * GE] = pg[2]; gs[3 * GE] = pg[3];
      L.C[row * GE + u] = pc;
      L.Hs[row * GE + u] = ph;
      if (pl == 0) L.X[row * GE + u] = px;
    }
    pl = -1;
  };
  // the gate tiles of layer i from A (4 tiles q: units 16 j + 4 q + (n & 3), gate n >> 2), the
  // zero-state cell, h published; the values saved for the backward become the pending set
  auto gates = [&](int i, const GlW<GE> (&f)[4], unsigned long long* hbuf, unsigned tag, long row_t) {
    __syncthreads();
    if (tid < GL_ROWS * 16) px = Xs[m8][u];
#pragma unroll
    for (int q = 0; q < 4; ++q) gl_park(red, q, wave, lane, gl_mma<GE>(&A[0][0], AP, f[q], lane, wave));
    __syncthreads();
    if (ep) {
      const int q = n16 >> 2, jj = n16 & 3;
      pg[0] = sigmoidf_(gl_sum(red, q, m8, jj) + bias_s[i][0][n16]);
      pg[1] = sigmoidf_(gl_sum(red, q, m8, 4 + jj) + bias_s[i][1][n16]);
      pg[2] = tanhf_(gl_sum(red, q, m8, 8 + jj) + bias_s[i][2][n16]);
      pg[3] = sigmoidf_(gl_sum(red, q, m8, 12 + jj) + bias_s[i][3][n16]);
      pc = pg[0] * pg[2];   // f c0 + i g with c0 = 0
      ph = pg[3] * tanhf_(pc);
      put_granule(hbuf + (long)b8 * GE + u, tag, ph, local);
    }
    pl = i;
    prt = row_t;
  };
  // the P rows of the next frame, loaded one frame ahead (after layer 1's hand-off poll, or the
  // FFN stage's with one layer; frame 0's here) and parked in LDS after the FFN stage's poll (which
  // waits for them anyway): layer 0 has no hand-off wait to hide an HBM fetch under, and a register
  // carried across the frame loop's back edge costs a full vmcnt(0) wait where it is used
  float pp[GL_ROWS];
  auto load_p = [&](int tn) {
#pragma unroll
    for (int m = 0; m < GL_ROWS; ++m) pp[m] = p.P[((long)tn * B + min(r0 + m, B - 1)) * GE + tid];
  };
  auto park_p = [&]() {
#pragma unroll
    for (int m = 0; m < GL_ROWS; ++m) Ps[m][tid] = pp[m];
  };
  load_p(0);
  park_p();
  for (int t = 0; t < T && !sdead; ++t) {
    SL_STAMP(0);
    unsigned long long* hb = p.ring + (long)(t & 1) * nl * BH;   // this frame's h_i buffers
    const unsigned tag = (unsigned)(t + 1);
    const long row_t = (long)t * B;   // frame t's first row in the [T][B][.] tensors
    // ---- layer 0: X_0 = P(t) + ms_in(t) W_ms^T (thread = column)
    {
      // all 16 ms columns, unrolled (msin and wms_s are zero past FO: the same sums), so the LDS
      // reads issue back to back instead of one round trip per column
      float wv[16];
#pragma unroll
      for (int o = 0; o < 16; ++o) wv[o] = wms_s[o][tid];
#pragma unroll
      for (int m = 0; m < GL_ROWS; ++m) {
        float v = Ps[m][tid];
#pragma unroll
        for (int o4 = 0; o4 < 4; ++o4) {
          const float4 ms4 = *reinterpret_cast<const float4*>(&msin[m][4 * o4]);
          v = fmaf(ms4.x, wv[4 * o4], v);
          v = fmaf(ms4.y, wv[4 * o4 + 1], v);
          v = fmaf(ms4.z, wv[4 * o4 + 2], v);
          v = fmaf(ms4.w, wv[4 * o4 + 3], v);
        }
        v = r0 + m < B ? v : 0.0f;
        Xs[m][tid] = v;
        A[m][tid] = v;
      }
      SL_STAMP(1);
      // the weight fragments after the build (a barrier keeps the compiler from hoisting them: held
      // through it they leave too few registers and the build's LDS reads serialise)
      __syncthreads();
      GlW<GE> f0[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) gl_wload<GE>(f0[q], W0s[16 * q + c16], wave, lane);
      gates(0, f0, hb, tag, row_t);
      SL_STAMP(2);
    }
    // ---- layer i > 0: X_i = LN(h_{i-1} + X_{i-1}) (the LayerNorm after layer i - 1)
    for (int i = 1; i < nl; ++i) {
      const SsdLoopLayer& Lp = p.L[i - 1];
      GlW<GE> f[4];   // weights first: their latency hides under the hand-off wait
#pragma unroll
      for (int q = 0; q < 4; ++q)
        gl_wload<GE>(f[q], p.L[i].w_ih + (long)((c16 >> 2) * GE + 16 * j + 4 * q + (c16 & 3)) * GE, wave, lane);
      const GlLn ln = gl_lnp(Lp.ln_g, Lp.ln_b, lane);
      gl_gather<GE>(hb + (long)(i - 1) * BH, r0, B, tag, &A[0][0], AP, p.err, dead, &sdead);
      __syncthreads();
      flush();
      if (i == 1 && t + 1 < T) load_p(t + 1);
      SL_STAMP(1 + 2 * i);
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int m = wave + 4 * rr;
        gl_ln_row(A[m], Xs[m], ln, eps, Xs[m], A[m], lane);
      }
      gates(i, f, hb + (long)i * BH, tag, row_t);
      SL_STAMP(2 + 2 * i);
    }
    // ---- F: U = LN(h + X) of the last layer, Z = relu(U W1^T + b1), y = Z W2^T + b2, the select
    {
      const SsdLoopLayer& Ll = p.L[nl - 1];
      GlW<4 * GE> f1;   // wave w: hidden columns 16 w .. 16 w + 15 over the whole k range
      gl_wload<4 * GE>(f1, p.w1 + (long)(16 * wave + c16) * GE, 0, lane);
      GlW<GHB> f2;      // output columns past FO multiply zeroed fragments of a valid weight row
      gl_wload<GHB>(f2, p.w2 + (long)(c16 < FO ? c16 : 0) * GHB, wave, lane);
      if (c16 >= FO) f2.v[0] = gen_zero4();
      const GlLn ln = gl_lnp(Ll.ln_g, Ll.ln_b, lane);
      const int hc = 16 * wave + c16;
      const float b1 = p.b1[hc];
      const bool yv_ok = tid < GL_ROWS * 16 && n16 < FO && b8 < B;
      const float b2 = yv_ok ? p.b2[n16] : 0.0f;
      const bool sel = p.mask[t] != 0;
      const float msv = yv_ok ? p.ms[(long)b8 * p.ms_bs + (long)t * p.ms_ts + n16] : 0.0f;
      gl_gather<GE>(hb + (long)(nl - 1) * BH, r0, B, tag, &A[0][0], AP, p.err, dead, &sdead);
      __syncthreads();
      flush();
      if (t + 1 < T) {
        if (nl == 1) load_p(t + 1);
        else park_p();   // Ps is free: layer 0 of this frame read it before its publish
      }
      SL_STAMP(1 + 2 * nl);
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int m = wave + 4 * rr;
        gl_ln_row(A[m], Xs[m], ln, eps, A[m], nullptr, lane);
      }
      __syncthreads();
      {
        const gv4 acc = gl_mma<4 * GE>(&A[0][0], AP, f1, lane, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          hs[4 * (lane >> 4) + i][hc] = fmaxf(acc[i] + b1, 0.0f);
        }
      }
      __syncthreads();
      gl_park(red, 0, wave, lane, gl_mma<GHB>(&hs[0][0], HP, f2, lane, wave));
      __syncthreads();
      if (tid < GL_ROWS * 16) {
        float nxt = 0.0f;
        if (yv_ok) {
          nxt = sel ? gl_sum(red, 0, m8, n16) + b2 : msv;
        }
        msin[m8][n16] = nxt;
      }
      if (nl == 1 && t + 1 < T) park_p();
      if (dead) sdead = 1;
      __syncthreads();
      SL_STAMP(2 + 2 * nl);
    }
  }
  flush();
}

// ------------------------------------------------------------------ the backward frame loop, one launch
// ssd_loop_bwd_kernel: the per-frame backward of decode.py (mrg_ssd_ffn_bwd, mrg_ssd_dx,
// mrg_ssd_ln_cell_bwd for L >= 2 layers) in ONE persistent launch over frames T-1 .. 0, with the
// same row groups and members as the forward (member j: hidden units 16 j .. 16 j + 15).  Per frame:
//   F  gather the 16 members' partial dyx(t+1) -> dy_total = dy(t) + mask[t] dyx(t+1) (every member
//      its rows) -> dz = relu'(z) (dy_total W2) (all 64, per member) -> du = dz W1 (own columns) and
//      the LayerNorm's two row sums through v = [W1 gamma | W1 beta] (no exchange, decode.hip's
//      identity) -> g, the zero-state cell backward -> dG of the last layer's own units
//   P  (after each dG of a layer l >= 1) this member's PARTIAL dX_l = dG[:, own gate columns] W_ih[own
//      rows, :] over all 256 columns (MFMA, K = 48), and its partial LayerNorm row sums of layer l-1's
//      backward over all columns: sum_k P[k] gamma[k] and sum_k P[k] (X_l[k] - beta[k]) (= gamma xh),
//      plus the own columns' g terms -> publish
//   B  gather the own columns of every member's partial and every member's row sums -> dX_l (own
//      columns) = the sum + g -> LayerNorm backward of layer l-1 -> cell backward -> P for l-1 > 0, or
//      at the bottom layer the partial dyx(t) = dfeat(t) W_ms over own units (dG vt^T + g wms^T,
//      vt = W_ms^T W_ih0), which frame t - 1's F stage sums
// so a frame is L hand-offs (2 at L = 2) instead of 2L launches.  The partial buffers alternate by
// level (a member writes one again only after a gather that needs every member past its last read).
static constexpr int SB_KP = 48;       // partial product K: the i, g, o gate columns of 16 units
static constexpr int SB_NP = 10;       // pending saved-tensor stores per thread
static constexpr int SB_PER_LAYER = 12;  // see mrg_ssd_loop_bwd

struct SsdBwdLayer {
  const float* w_ih;                   // W_ih [4H][H] (layers >= 1)
  const float *ln_g, *ln_b;            // the LayerNorm after this layer
  const float *X, *G, *C, *Hs, *mean, *rstd;   // the forward's saved tensors
  float *g, *dG, *dX;                  // d(h + x) [T][B][H], dG [T][B][4H], dX (layers >= 1) [T][B][H]
};
struct SsdBwdArgs {
  SsdBwdLayer L[SL_MAXL];
  const float* dy;                     // [B][T][FO]
  const unsigned char* mask;           // [T]
  const float *w1, *w2, *b1, *v;       // FFN W1 [HB][H], W2 [FO][HB], b1, v = [W1 gamma | W1 beta] [HB][2]
  const float* z;                      // Z [T][B][HB]
  const float *vt, *wms;               // vt = W_ms^T W_ih0 [FO][4H], W_ms^T [FO][H]
  float* du;                           // [T][B][H]
  unsigned long long* ring;            // 2 x (partials [B][16][256] | sums [B][16][2]) | dyx [B][256] granules, XCC slots
  int* err;
  int B, T, FO, nl, ngroups;
  unsigned long long* stamps;          // diagnostics (mrg_ssd_loop_bwd_debug_stamps): [T][16][16] of row group 0, or null
};

#define SB_STAMP(slot)                                                                   \
  do {                                                                                   \
    if (p.stamps && g == 0 && threadIdx.x == 0) {                                        \
      unsigned long long _t;                                                             \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
      p.stamps[((long)it * GL_MEM + j) * 16 + (slot)] = _t;                              \
    }                                                                                    \
  } while (0)

__global__ __launch_bounds__(256) void ssd_loop_bwd_kernel(SsdBwdArgs p) {
  constexpr int DP = SB_KP + 4;
  __shared__ __attribute__((aligned(16))) float A[GL_ROWS][GE + 4];   // gathered dyx partials
  __shared__ __attribute__((aligned(16))) float dgs[16][DP];          // own dG (rows 8..15 zero)
  __shared__ float ys[GL_ROWS][GE + 1];  // X_l - beta_{l-1} of the rows (the row sums' gamma xh)
  __shared__ float gam_f[GE], bet_f[GE]; // gamma / beta of LayerNorm l-1 (full width, this stage)
  __shared__ float parts[GL_ROWS][GL_MEM][17];   // gathered partials of the own columns
  __shared__ float sums[GL_ROWS][2 * GL_MEM];
  __shared__ float rsum[4][GL_ROWS][2];  // per-wave partial row sums
  __shared__ float w2s[16][GHB];        // W2 (rows past FO zero)
  __shared__ float w1c[GHB][16];        // W1 columns of this member's units
  __shared__ float hv1[GHB], hv2[GHB], hb1[GHB];
  __shared__ float gam_s[SL_MAXL][16];
  __shared__ float vts[3][16][16];      // vt[o][blk H + unit], blocks i, g, o (rows past FO zero)
  __shared__ float wmc[16][16];         // W_ms^T[o][unit]
  __shared__ float dys[GL_ROWS][16];
  __shared__ float dzs[GL_ROWS][GHB + 1];
  __shared__ float msum[GL_ROWS][2];
  __shared__ int sdead, xflag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % p.ngroups, j = blockIdx.x / p.ngroups;
  const int r0 = GL_ROWS * g, B = p.B, T = p.T, FO = p.FO, nl = p.nl;
  const long PB = (long)B * GL_MEM * GE, SBn = (long)B * GL_MEM * 2;
  unsigned long long* bpart = p.ring;                 // [2][B][16][256]
  unsigned long long* bsum = bpart + 2 * PB;          // [2][B][16][2]
  unsigned long long* bdyx = bsum + 2 * SBn;          // [B][256]
  unsigned long long* slots = bdyx + (long)B * 256;
  bool dead = false;
  for (int i = tid; i < 16 * DP; i += 256) (&dgs[0][0])[i] = 0.0f;
  {
    const int o = tid >> 4, n = tid & 15, u = 16 * j + n;
    const bool ov = o < FO;
    for (int i = tid; i < 16 * GHB; i += 256) w2s[i / GHB][i % GHB] = i / GHB < FO ? p.w2[i] : 0.0f;
    for (int i = tid; i < GHB * 16; i += 256) w1c[i >> 4][i & 15] = p.w1[(long)(i >> 4) * GE + 16 * j + (i & 15)];
    if (tid < GHB) {
      hv1[tid] = p.v[2 * tid];
      hv2[tid] = p.v[2 * tid + 1];
      hb1[tid] = p.b1[tid];
    }
    if (tid < 16 * nl) gam_s[tid >> 4][tid & 15] = p.L[tid >> 4].ln_g[16 * j + (tid & 15)];
    vts[0][o][n] = ov ? p.vt[(long)o * 4 * GE + u] : 0.0f;
    vts[1][o][n] = ov ? p.vt[(long)o * 4 * GE + 2 * GE + u] : 0.0f;
    vts[2][o][n] = ov ? p.vt[(long)o * 4 * GE + 3 * GE + u] : 0.0f;
    wmc[o][n] = ov ? p.wms[(long)o * GE + u] : 0.0f;
  }
  if (tid == 0) sdead = 0;
  const int local = group_on_one_xcd<GL_MEM>(slots + (long)g * GL_MEM, j, p.err, dead, &xflag);
  __syncthreads();
  const int m8 = tid >> 4, n16 = tid & 15;
  const int b8 = r0 + m8, bc = min(b8, B - 1);
  const bool ep = tid < GL_ROWS * 16 && b8 < B;
  const int u = 16 * j + n16;
  const int c16 = lane & 15, q4 = lane >> 4;
  SL_STAMP_ID();
  // pending saved-tensor stores, issued after the next hand-off poll (see the forward)
  float* pa[SB_NP];
  float pv[SB_NP];
#pragma unroll
  for (int s = 0; s < SB_NP; ++s) {
    pa[s] = nullptr;
    pv[s] = 0.0f;
  }
  auto flush = [&]() {
#pragma unroll
    for (int s = 0; s < SB_NP; ++s) {
      if (pa[s]) *pa[s] = pv[s];
      pa[s] = nullptr;
    }
  };
  auto defer = [&](int s, float* a, float v) {
    pa[s] = a;
    pv[s] = v;
  };
  // zero-state cell backward of unit u (c0 = 0: d f = 0), the four dG values pending from slot s
  auto cell_bwd = [&](const SsdBwdLayer& Ly, long row, float gv, float ig, float gg, float og, float cc, int s,
                      float& d_i, float& d_g, float& d_o) {
    const float tc = tanhf_(cc);
    const float dc = gv * og * (1.0f - tc * tc);
    d_i = dc * gg * ig * (1.0f - ig);
    d_g = dc * ig * (1.0f - gg * gg);
    d_o = gv * tc * og * (1.0f - og);
    float* d = Ly.dG + row * 4 * GE + u;
    defer(s, d, d_i);
    defer(s + 1, d + GE, 0.0f);
    defer(s + 2, d + 2 * GE, d_g);
    defer(s + 3, d + 3 * GE, d_o);
  };
  // P's operands of layer l, loaded ahead: W_ih rows of the own i, g, o gate columns (lane: k = 4 s +
  // q4, column 64 wave + 16 q + c16) and the rows' X_l into ys, gamma / beta of LayerNorm l-1
  float wf[SB_KP / 4][4];
  float xr[GL_ROWS];
  float gmv = 0.0f, btv = 0.0f;
  auto load_p = [&](int l, long rt) {
    const SsdBwdLayer& Ly = p.L[l];
#pragma unroll
    for (int s = 0; s < SB_KP / 4; ++s) {
      const int k = 4 * s + q4, blk = k >> 4;
      const float* wr = Ly.w_ih + (long)((blk == 0 ? 0 : blk + 1) * GE + 16 * j + (k & 15)) * GE + 64 * wave + c16;
#pragma unroll
      for (int q = 0; q < 4; ++q) wf[s][q] = wr[16 * q];
    }
#pragma unroll
    for (int m = 0; m < GL_ROWS; ++m) xr[m] = Ly.X[(rt + min(r0 + m, B - 1)) * GE + tid];
    gmv = p.L[l - 1].ln_g[tid];
    btv = p.L[l - 1].ln_b[tid];
  };
  // P of layer l: this member's partial dX_l and partial row sums, published at level `lv`; d_*, gv:
  // the epilogue threads' own dG / g of layer l
  auto partial = [&](int lv, float d_i, float d_g, float d_o, float gv) {
    if (ep) {
      dgs[m8][n16] = d_i;
      dgs[m8][16 + n16] = d_g;
      dgs[m8][32 + n16] = d_o;
    }
#pragma unroll
    for (int m = 0; m < GL_ROWS; ++m) ys[m][tid] = xr[m] - btv;
    gam_f[tid] = gmv;
    bet_f[tid] = btv;
    __syncthreads();
    gv4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = gv4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < SB_KP / 4; ++s) {
      const float av = dgs[c16][4 * s + q4];
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, wf[s][q], acc[q], 0, 0, 0);
    }
    // lane: rows 4 q4 + i (i < 4), column 64 wave + 16 q + c16; rows 8..15 (q4 >= 2) are padding
    const unsigned tag = (unsigned)(lv + 1);
    unsigned long long* pb = bpart + (long)(lv & 1) * PB;
    float s0[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f};
    if (q4 < 2) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int col = 64 * wave + 16 * q + c16;
        const float gm = gam_f[col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = 4 * q4 + i;
          s0[i] = fmaf(acc[q][i], gm, s0[i]);
          s1[i] = fmaf(acc[q][i], ys[m][col], s1[i]);
          if (r0 + m < B) put_granule(pb + ((long)(r0 + m) * GL_MEM + j) * GE + col, tag, acc[q][i], local);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s0[i] = group_sum<16>(s0[i]);
      s1[i] = group_sum<16>(s1[i]);
    }
    if (c16 == 0 && q4 < 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        rsum[wave][4 * q4 + i][0] = s0[i];
        rsum[wave][4 * q4 + i][1] = s1[i];
      }
    }
    // the own columns' g terms (g enters dX_l once, through its owner)
    float g0 = ep ? gv * gam_f[u] : 0.0f, g1 = ep ? gv * ys[m8][u] : 0.0f;
    g0 = group_sum<16>(g0);
    g1 = group_sum<16>(g1);
    __syncthreads();
    if (tid < GL_ROWS * 16 && n16 < 2 && b8 < B) {
      const float t0 = n16 ? g1 : g0;
      const float v = ((rsum[0][m8][n16] + rsum[1][m8][n16]) + (rsum[2][m8][n16] + rsum[3][m8][n16])) + t0;
      put_granule(bsum + (long)(lv & 1) * SBn + ((long)b8 * GL_MEM + j) * 2 + n16, tag, v, local);
    }
  };
  // B's gather: the own columns of every member's partial (8 a thread) and every member's sums (1)
  auto gather_p = [&](int lv) {
    if (sdead) dead = true;
    const unsigned tag = (unsigned)(lv + 1);
    const unsigned long long* pb = bpart + (long)(lv & 1) * PB;
    const unsigned long long* sb = bsum + (long)(lv & 1) * SBn;
    const int m = tid >> 5, jm = (tid >> 1) & 15, hf = tid & 1, rr = min(r0 + m, B - 1);
    int ip[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) ip[c] = (rr * GL_MEM + jm) * GE + 16 * j + 8 * hf + c;
    float v[8];
    get_granules_idx<8>(const_cast<unsigned long long*>(pb), ip, tag, v, p.err, dead);
    int is[1] = {rr * GL_MEM * 2 + (tid & 31)};
    float vs[1];
    get_granules_idx<1>(const_cast<unsigned long long*>(sb), is, tag, vs, p.err, dead);
    const bool ok = r0 + m < B;
#pragma unroll
    for (int c = 0; c < 8; ++c) parts[m][jm][8 * hf + c] = ok ? v[c] : 0.0f;
    sums[m][tid & 31] = ok ? vs[0] : 0.0f;
    if (dead) sdead = 1;
  };
  float gprev = 0.0f;   // g of layer l (own column), for dX_l
  for (int it = 0; it < T && !sdead; ++it) {
    const int t = T - 1 - it;
    const long rt = (long)t * B;
    SB_STAMP(0);
    // ---- F: the last layer, then its P
    {
      const SsdBwdLayer& Ly = p.L[nl - 1];
      const long row = rt + bc;
      const float hx = Ly.Hs[row * GE + u] + Ly.X[row * GE + u];
      const float mn = Ly.mean[row], rs = Ly.rstd[row];
      const float ig = Ly.G[row * 4 * GE + u], gg = Ly.G[row * 4 * GE + 2 * GE + u];
      const float og = Ly.G[row * 4 * GE + 3 * GE + u], cc = Ly.C[row * GE + u];
      const int mz = tid >> 5, jz = tid & 31, bz = min(r0 + mz, B - 1);
      const float z0 = p.z[(rt + bz) * GHB + jz], z1 = p.z[(rt + bz) * GHB + jz + 32];
      const bool dyv = tid < GL_ROWS * 16 && n16 < FO && b8 < B;
      const float dyin = dyv ? p.dy[((long)b8 * T + t) * FO + n16] : 0.0f;
      const bool fed = it > 0 && p.mask[t] != 0;
      if (it > 0) gl_gather<256>(bdyx, r0, B, (unsigned)it, &A[0][0], GE + 4, p.err, dead, &sdead);
      __syncthreads();
      flush();
      load_p(nl - 1, rt);
      SB_STAMP(1);
      if (tid < GL_ROWS * 16) {
        float dyx = 0.0f;
#pragma unroll
        for (int jm = 0; jm < GL_MEM; ++jm) dyx += A[m8][16 * jm + n16];
        const float v = dyv ? dyin + (fed ? dyx : 0.0f) : 0.0f;
        dys[m8][n16] = v;
      }
      __syncthreads();
      float m0 = 0.0f, m1 = 0.0f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int jh = jz + 32 * i;
        const float zv = i ? z1 : z0;
        float acc = 0.0f;
#pragma unroll
        for (int o = 0; o < 16; ++o) acc = fmaf(dys[mz][o], w2s[o][jh], acc);
        const float d = zv > 0.0f ? acc : 0.0f;
        dzs[mz][jh] = d;
        m0 = fmaf(d, hv1[jh], m0);
        m1 = fmaf(d, (zv - hb1[jh]) - hv2[jh], m1);
      }
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) {
        m0 += __shfl_xor(m0, o, 64);
        m1 += __shfl_xor(m1, o, 64);
      }
      if (jz == 0) {
        msum[mz][0] = m0;
        msum[mz][1] = m1;
      }
      __syncthreads();
      float d_i = 0.0f, d_g = 0.0f, d_o = 0.0f, gv = 0.0f;
      if (ep) {
        float du = 0.0f;
#pragma unroll 16
        for (int jh = 0; jh < GHB; ++jh) du = fmaf(dzs[m8][jh], w1c[jh][n16], du);
        defer(3, p.du + (rt + b8) * GE + u, du);
        const float xh = (hx - mn) * rs;
        const float gd = du * gam_s[nl - 1][n16];
        gv = rs * (gd - msum[m8][0] / (float)GE - xh * (msum[m8][1] / (float)GE));
        defer(4, Ly.g + (rt + b8) * GE + u, gv);
        cell_bwd(Ly, rt + b8, gv, ig, gg, og, cc, 5, d_i, d_g, d_o);
      }
      gprev = gv;
      partial(it * nl, d_i, d_g, d_o, gv);
      SB_STAMP(2);
    }
    for (int l = nl - 1; l >= 1; --l) {
      const SsdBwdLayer& Ly = p.L[l];
      const SsdBwdLayer& Lb = p.L[l - 1];
      const int lv = it * nl + (nl - 1 - l);
      // ---- B: dX_l (own columns), LayerNorm l-1 and cell backward; P of layer l-1, or the partial dyx
      const long row = rt + bc;
      const float hx = Lb.Hs[row * GE + u] + Lb.X[row * GE + u];
      const float mn = Lb.mean[row], rs = Lb.rstd[row];
      const float ig = Lb.G[row * 4 * GE + u], gg = Lb.G[row * 4 * GE + 2 * GE + u];
      const float og = Lb.G[row * 4 * GE + 3 * GE + u], cc = Lb.C[row * GE + u];
      gather_p(lv);
      __syncthreads();
      flush();
      if (l - 1 > 0) load_p(l - 1, rt);
      SB_STAMP(3 + 2 * (nl - 1 - l));
      float d_i = 0.0f, d_g = 0.0f, d_o = 0.0f, gv = 0.0f;
      if (ep) {
        float dx = 0.0f, q0 = 0.0f, q1 = 0.0f;
#pragma unroll
        for (int jm = 0; jm < GL_MEM; ++jm) {
          dx += parts[m8][jm][n16];
          q0 += sums[m8][2 * jm];
          q1 += sums[m8][2 * jm + 1];
        }
        dx += gprev;
        defer(0, Ly.dX + (rt + b8) * GE + u, dx);
        const float xh = (hx - mn) * rs;
        const float gd = dx * gam_s[l - 1][n16];
        gv = rs * (gd - q0 / (float)GE - xh * (q1 / (float)GE));
        defer(1, Lb.g + (rt + b8) * GE + u, gv);
        cell_bwd(Lb, rt + b8, gv, ig, gg, og, cc, 2, d_i, d_g, d_o);
      }
      if (l - 1 > 0) {
        gprev = gv;
        partial(lv + 1, d_i, d_g, d_o, gv);
      } else {
        // partial dyx(t)[b][o] = sum over own units of dG . vt[o] + g . W_ms^T[o] (lane n16: output o = n16)
        float mine = 0.0f;
#pragma unroll
        for (int o = 0; o < 16; ++o) {
          float q = fmaf(d_i, vts[0][o][n16], fmaf(d_g, vts[1][o][n16], fmaf(d_o, vts[2][o][n16], gv * wmc[o][n16])));
          q = group_sum<16>(q);
          mine = (n16 == o) ? q : mine;
        }
        if (ep) put_granule(bdyx + (long)b8 * 256 + 16 * j + n16, (unsigned)(it + 1), mine, local);
      }
      SB_STAMP(4 + 2 * (nl - 1 - l));
    }
  }
  flush();
}

}  // namespace mrg

using namespace mrg;

static unsigned long long* g_ssd_stamps = nullptr;
// Diagnostics (tools/ssd_stamps.py): later mrg_ssd_loop_fwd launches write group 0's members' per-stage
// real-time (10 ns) stamps into buf ([T][16 members][16] u64; frame 0: slot 15 the local hand-off flag,
// 14 the HW_ID register); null = off.
MRG_API int mrg_ssd_loop_debug_stamps(void* buf) {
  g_ssd_stamps = static_cast<unsigned long long*>(buf);
  return 0;
}

// Bytes of the granule ring mrg_ssd_loop_fwd needs for B rows and nl layers (zeroed by the caller
// before every launch).
MRG_API long mrg_ssd_loop_ring_bytes(int B, int nl) {
  const int ng = (B + GL_ROWS - 1) / GL_ROWS;
  return (2L * nl * B * GE + (long)ng * GL_MEM) * 8;
}

// 1 when the persistent grid (16 workgroups per 8 batch rows) can be resident on `cus` CUs (0: this device's).
MRG_API int mrg_ssd_loop_fits(int B, int cus) {
  const long nblk = (long)GL_MEM * ((B + GL_ROWS - 1) / GL_ROWS);
  return fits(ssd_loop_kernel, 256, nblk, cus > 0 ? cus : device_cus()) ? 1 : 0;
}

// The scheduled-sampling decode's forward frame loop in one persistent launch (ssd_loop_kernel;
// replaces the per-frame mrg_ssd_feat_gate_cell_fwd / mrg_ssd_gate_cell_fwd / mrg_ssd_ffn_z_fwd /
// mrg_ssd_y_fwd sequence of decode.py).  H = 256, HB = 64, FO <= 16, nl <= 4.  lptrs (host array, 9 per
// layer): w_ih [4H][H], b_ih, b_hh, the LayerNorm after the layer (gamma, beta), then the saved X
// [T][B][H] (layer 0's; ignored, may be null, for the others), gates [T][B][4H], c and h [T][B][H].
// P [T][B][H]; wms = W_ms^T [FO][H]; FFN w1 [HB][H], b1, w2 [FO][HB], b2; ms, mask as in
// mrg_ssd_feat_gate_cell_fwd; ring: mrg_ssd_loop_ring_bytes of zeroed memory; err: the recurrences'
// error flag.  The LayerNorm outputs and statistics, Z, y and the sampled self-motion inputs are not
// written: they follow from h, X_0 and ms after the loop (decode.py).
MRG_API int mrg_ssd_loop_fwd(int B, int T, int H, int HB, int FO, int nl, float eps, const void* const* lptrs,
                             int nptrs, const float* P, const float* wms, const float* w1, const float* b1,
                             const float* w2, const float* b2, const float* ms, long ms_bs, long ms_ts,
                             const unsigned char* mask, void* ring, int* err, hipStream_t stream) {
  if (B == 0 || T == 0) return 0;
  MRG_REQUIRE(H == GE && HB == GHB && FO >= 1 && FO <= 16 && nl >= 1 && nl <= SL_MAXL,
              "mrg_ssd_loop_fwd: needs H = %d, HB = %d, 1 <= FO <= 16, 1 <= nl <= %d (H=%d HB=%d FO=%d nl=%d)", GE,
              GHB, SL_MAXL, H, HB, FO, nl);
  MRG_REQUIRE(lptrs && nptrs == SL_PER_LAYER * nl && P && wms && w1 && b1 && w2 && b2 && ms && mask && ring && err,
              "mrg_ssd_loop_fwd: null argument or nptrs %d != %d", nptrs, SL_PER_LAYER * nl);
  MRG_REQUIRE(mrg_ssd_loop_fits(B, 0) == 1, "mrg_ssd_loop_fwd: %d workgroups cannot all be resident (B=%d)",
              GL_MEM * ((B + GL_ROWS - 1) / GL_ROWS), B);
  SsdLoopArgs a{};
  for (int i = 0; i < nl; ++i) {
    const void* const* q = lptrs + SL_PER_LAYER * i;
    for (int k = 0; k < SL_PER_LAYER; ++k)
      MRG_REQUIRE(q[k] != nullptr || (k == 5 && i > 0), "mrg_ssd_loop_fwd: null pointer %d of layer %d", k, i);
    SsdLoopLayer& L = a.L[i];
    L.w_ih = static_cast<const float*>(q[0]); L.b_ih = static_cast<const float*>(q[1]);
    L.b_hh = static_cast<const float*>(q[2]); L.ln_g = static_cast<const float*>(q[3]);
    L.ln_b = static_cast<const float*>(q[4]);
    L.X = (float*)q[5]; L.G = (float*)q[6]; L.C = (float*)q[7]; L.Hs = (float*)q[8];
  }
  a.P = P; a.wms = wms; a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2;
  a.ms = ms; a.ms_bs = ms_bs; a.ms_ts = ms_ts; a.mask = mask;
  a.ring = static_cast<unsigned long long*>(ring); a.err = err;
  a.B = B; a.T = T; a.FO = FO; a.nl = nl; a.ngroups = (B + GL_ROWS - 1) / GL_ROWS; a.eps = eps;
  a.stamps = g_ssd_stamps;
  klaunch(ssd_loop_kernel, dim3(GL_MEM * a.ngroups), 256, 0, stream, a);
  return check_launch("ssd_loop_kernel");
}

static unsigned long long* g_ssd_bwd_stamps = nullptr;
// Diagnostics (tools/ssd_stamps.py): later mrg_ssd_loop_bwd launches write group 0's members' per-stage
// real-time (10 ns) stamps into buf ([T][16 members][16] u64 by backward iteration, as the forward's); null = off.
MRG_API int mrg_ssd_loop_bwd_debug_stamps(void* buf) {
  g_ssd_bwd_stamps = static_cast<unsigned long long*>(buf);
  return 0;
}

// Bytes of the granule ring mrg_ssd_loop_bwd needs for B rows (zeroed by the caller before every launch).
MRG_API long mrg_ssd_loop_bwd_ring_bytes(int B) {
  const int ng = (B + GL_ROWS - 1) / GL_ROWS;
  return ((long)B * (2 * GL_MEM * (GE + 2) + 256) + (long)ng * GL_MEM) * 8;
}

MRG_API int mrg_ssd_loop_bwd_fits(int B, int cus) {
  const long nblk = (long)GL_MEM * ((B + GL_ROWS - 1) / GL_ROWS);
  return fits(ssd_loop_bwd_kernel, 256, nblk, cus > 0 ? cus : device_cus()) ? 1 : 0;
}

// The scheduled-sampling decode's backward frame loop (nl >= 2 layers) in one persistent launch
// (ssd_loop_bwd_kernel; replaces decode.py's per-frame mrg_ssd_ffn_bwd / mrg_ssd_dx /
// mrg_ssd_ln_cell_bwd sequence with the same outputs).  H = 256, HB = 64, FO <= 16, 2 <= nl <= 4.
// lptrs (host array, 12 per layer): W_ih [4H][H] (null for layer 0), the gamma and beta of the
// LayerNorm after the layer, the forward's saved X, gates, c, h and that LayerNorm's mean / rstd, then
// the outputs g = d(h + x) [T][B][H], dG [T][B][4H] and dX [T][B][H] (layers >= 1; null for layer 0).
// dy [B][T][FO]; mask [T] bytes; w1 [HB][H], w2 [FO][HB], b1, v = [W1 gamma | W1 beta] [HB][2] of the
// last LayerNorm; z [T][B][HB]; vt = W_ms^T W_ih0 [FO][4H]; wms_t [FO][H]; output du [T][B][H] (the
// last LayerNorm's upstream gradient, for its parameters); ring: mrg_ssd_loop_bwd_ring_bytes of zeroed
// memory; err as the forward's.  The prediction gradient through the select (dy_total) and dz are
// not written: they follow from dy, dfeat = dX_0 and z after the loop (decode.py).
MRG_API int mrg_ssd_loop_bwd(int B, int T, int H, int HB, int FO, int nl, const void* const* lptrs, int nptrs,
                             const float* dy, const unsigned char* mask, const float* w1, const float* w2,
                             const float* b1, const float* v, const float* z, const float* vt, const float* wms_t,
                             float* du, void* ring, int* err, hipStream_t stream) {
  if (B == 0 || T == 0) return 0;
  MRG_REQUIRE(H == GE && HB == GHB && FO >= 1 && FO <= 16 && nl >= 2 && nl <= SL_MAXL,
              "mrg_ssd_loop_bwd: needs H = %d, HB = %d, 1 <= FO <= 16, 2 <= nl <= %d (H=%d HB=%d FO=%d nl=%d)", GE,
              GHB, SL_MAXL, H, HB, FO, nl);
  MRG_REQUIRE(lptrs && nptrs == SB_PER_LAYER * nl && dy && mask && w1 && w2 && b1 && v && z && vt && wms_t && du &&
                  ring && err,
              "mrg_ssd_loop_bwd: null argument or nptrs %d != %d", nptrs, SB_PER_LAYER * nl);
  MRG_REQUIRE(mrg_ssd_loop_bwd_fits(B, 0) == 1, "mrg_ssd_loop_bwd: %d workgroups cannot all be resident (B=%d)",
              GL_MEM * ((B + GL_ROWS - 1) / GL_ROWS), B);
  SsdBwdArgs a{};
  for (int i = 0; i < nl; ++i) {
    const void* const* q = lptrs + SB_PER_LAYER * i;
    for (int k = 0; k < SB_PER_LAYER; ++k) {
      const bool optional = i == 0 && (k == 0 || k == 11);
      MRG_REQUIRE(optional || q[k] != nullptr, "mrg_ssd_loop_bwd: null pointer %d of layer %d", k, i);
    }
    SsdBwdLayer& L = a.L[i];
    L.w_ih = static_cast<const float*>(q[0]); L.ln_g = static_cast<const float*>(q[1]);
    L.ln_b = static_cast<const float*>(q[2]);
    L.X = static_cast<const float*>(q[3]); L.G = static_cast<const float*>(q[4]);
    L.C = static_cast<const float*>(q[5]); L.Hs = static_cast<const float*>(q[6]);
    L.mean = static_cast<const float*>(q[7]); L.rstd = static_cast<const float*>(q[8]);
    L.g = (float*)q[9]; L.dG = (float*)q[10]; L.dX = (float*)q[11];
  }
  a.dy = dy; a.mask = mask; a.w1 = w1; a.w2 = w2; a.b1 = b1; a.v = v; a.z = z; a.vt = vt; a.wms = wms_t;
  a.du = du; a.ring = static_cast<unsigned long long*>(ring); a.err = err;
  a.B = B; a.T = T; a.FO = FO; a.nl = nl; a.ngroups = (B + GL_ROWS - 1) / GL_ROWS;
  a.stamps = g_ssd_bwd_stamps;
  klaunch(ssd_loop_bwd_kernel, dim3(GL_MEM * a.ngroups), 256, 0, stream, a);
  return check_launch("ssd_loop_bwd_kernel");
}
