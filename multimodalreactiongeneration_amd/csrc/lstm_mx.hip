// Persistent LSTM recurrence, MFMA form, for batch tiles of 16 rows (H = 256, 8 workgroups per
// row group).  Same problem / argument blocks, hand-off protocol and results layout as lstm.hip
// (lstm_common.h); what changes is the per-step product of each member:
//
//   forward   pre[16 b][128 own gate rows] = h_{t-1}[16][256] W_slice^T      (K = 256)
//   backward  P  [16 b][256 h outputs]     = dG[16][128 own rows] W_slice    (K = 128)
//
// on v_mfma_f32_16x16x32_bf16 with the x6 split (each fp32 operand cut into three bf16 planes,
// the six products with i + j <= 2 accumulated in fp32: fp32-class error, gemm_glds.hip), W_slice's
// planes resident in VGPRs for the whole sequence (96 registers per lane) and h (or dG) split ONCE
// per step into three bf16 planes in LDS as it arrives (a split per wave cost 8x the VALU).  The
// VALU GEMV of lstm.hip reads every h value from LDS once per 2 FMAs, so at batch tiles >= 4 the
// step is bound by those LDS reads; here a wave reads the planes once per 16-column output tile and
// the product runs at the x6 MFMA rate (2.7x the fp32 VALU peak).  Used when a launch would need batch tiles >= 4 (several problems per launch: the
// encoder stacks' wavefront, encoder_stack.py), selected in lstm.hip's launchers.
#include "gemm_common.h"
#include "lstm_common.h"

namespace mrg {

typedef float f32x4mx __attribute__((ext_vector_type(4)));

static constexpr int MX_H = 256, MX_G = 8, MX_BS = 16, MX_NT = 512, MX_U = 32, MX_R = 128;
static constexpr int MX_HPB = MX_H + 8;  // LDS row pitch of an h plane (bf16): conflict-free b128 fragment reads
static constexpr int MX_RPB = MX_R + 8;  // LDS row pitch of a dG plane (bf16)
static constexpr int MX_RP = MX_R + 4;   // LDS row pitch of the gate rows (floats)

// 8 consecutive-k fp32 -> three bf16x8 planes (x6 split; gemm_glds.hip split8)
__device__ __forceinline__ void mx_split8(float4 v0, float4 v1, bf16x8 (&f)[3]) {
  unsigned a0, a1, a2, b0, b1, b2, c0, c1, c2, d0, d1, d2;
  split2(v0.x, v0.y, a0, a1, a2);
  split2(v0.z, v0.w, b0, b1, b2);
  split2(v1.x, v1.y, c0, c1, c2);
  split2(v1.z, v1.w, d0, d1, d2);
  typedef unsigned u32x4mx __attribute__((ext_vector_type(4)));
  const u32x4mx p0 = {a0, b0, c0, d0}, p1 = {a1, b1, c1, d1}, p2 = {a2, b2, c2, d2};
  f[0] = __builtin_bit_cast(bf16x8, p0);
  f[1] = __builtin_bit_cast(bf16x8, p1);
  f[2] = __builtin_bit_cast(bf16x8, p2);
}

// acc += A B over the x6 terms, small terms first (A: lane l holds A[l & 15][8 (l >> 4) + j],
// B: lane l holds B[8 (l >> 4) + j][l & 15]; D: lane l holds D[4 (l >> 4) + i][l & 15])
__device__ __forceinline__ f32x4mx mx_mfma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4mx acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
}

// global W_hh row of a member's local gate row r (gate-major: r = q * U + u)
__device__ __forceinline__ int mx_grow(int j, int r) { return (r / MX_U) * MX_H + j * MX_U + (r % MX_U); }

// ds_read_b128 outside the compiler's view: its waitcnt pass would put a vmcnt(0) (the LDS-DMA alias rule)
// before every LDS read that follows an LDS-DMA issue, stalling the product on the prefetch; the
// caller waits with lgkmcnt itself
__device__ __forceinline__ bf16x8 mx_lds_b128(const void* p) {
  typedef unsigned u32x4r __attribute__((ext_vector_type(4)));
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
  u32x4r v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ float mx_lds_f32(const void* p) {
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
  float v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
// the wait for those reads, tied to their results (a bare asm wait would let the compiler schedule
// the consumers above it)
__device__ __forceinline__ void mx_lds_wait3(bf16x8 (&f)[3]) {
  typedef unsigned u32x4r __attribute__((ext_vector_type(4)));
  u32x4r a = __builtin_bit_cast(u32x4r, f[0]), b = __builtin_bit_cast(u32x4r, f[1]),
         c = __builtin_bit_cast(u32x4r, f[2]);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c)::"memory");
  f[0] = __builtin_bit_cast(bf16x8, a); f[1] = __builtin_bit_cast(bf16x8, b); f[2] = __builtin_bit_cast(bf16x8, c);
}
__device__ __forceinline__ void mx_lds_wait8(float (&x)[4], float (&y)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3])::"memory");
}
// a step barrier with no fence: LDS writes complete (lgkmcnt), LDS-DMA in flight left in flight (a
// __syncthreads would wait vmcnt(0) for it)
__device__ __forceinline__ void mx_step_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__global__ __launch_bounds__(MX_NT, 1) void lstm_fwd_mx_kernel(LstmFwdArgs args) {
  constexpr int H = MX_H, G = MX_G, BS = MX_BS, U = MX_U;
  constexpr int WP = MX_HPB / 2;  // 32-bit words per plane row
  __shared__ __attribute__((aligned(16))) unsigned hp[3][BS][WP];
  __shared__ __attribute__((aligned(16))) float pre[BS][MX_RP];
  __shared__ __attribute__((aligned(16))) float gxs[3][4][BS * U];   // Gx of step mod 3, by LDS-DMA
  __shared__ int xcc_flag;
  int prob, grp, j;
  const int ngroups = (args.B + BS - 1) / BS;
  decompose(G, ngroups, args.nprob, prob, grp, j);
  const LstmFwdProblem& P = args.p[prob];
  const int B = args.B, T = args.T;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = grp * BS;
  bool dead = false;

  // W planes: wave w owns local gate rows 16 w .. 16 w + 15 (the MFMA B operand, B[k][r] = W[r][k])
  bf16x8 wf[8][3];
  {
    const float* wr = P.w_hh + (long)mx_grow(j, 16 * wave + (lane & 15)) * H + 8 * (lane >> 4);
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float4 v0 = *reinterpret_cast<const float4*>(wr + 32 * s);
      const float4 v1 = *reinterpret_cast<const float4*>(wr + 32 * s + 4);
      mx_split8(v0, v1, wf[s]);
    }
  }
  // cell role: every thread owns one (row, unit) cell
  const int cb = tid / U, cu = tid % U;
  const int bg = b0 + cb;
  const bool cvalid = bg < B;
  const int hcol = j * U + cu;
  float c = 0.0f, h = 0.0f, bh[4] = {0.f, 0.f, 0.f, 0.f};
  if (cvalid) {
#pragma unroll
    for (int q = 0; q < 4; ++q) bh[q] = P.b_hh[q * H + hcol];
    if (P.c0) c = P.c0[(long)bg * P.c0_bs + hcol];
  }
  // h lands in LDS as three bf16 planes (x6 split), one 32-bit word = the pair (k, k + 1) of a row
  auto put_planes = [&](int b, int k, float v0, float v1) {
    unsigned p0, p1, p2;
    split2(v0, v1, p0, p1, p2);
    hp[0][b][k >> 1] = p0; hp[1][b][k >> 1] = p1; hp[2][b][k >> 1] = p2;
  };
  for (int e = 2 * tid; e < BS * H; e += 2 * MX_NT) {
    const int b = e / H, k = e % H;
    const bool ok = P.h0 && b0 + b < B;
    put_planes(b, k, ok ? P.h0[(long)(b0 + b) * P.h0_bs + k] : 0.0f,
               ok ? P.h0[(long)(b0 + b) * P.h0_bs + k + 1] : 0.0f);
  }
  // Gx of processing step tt2 -> LDS slot tt2 % 3 by LDS-DMA (wave w moves its own 64 cells), issued
  // after the step's gather so the next gather's wait (vmcnt, in order on gfx9) finds it landed and
  // no Gx load sits in front of a hand-off poll; rows past B read row B - 1 (never used)
  auto gx_issue = [&](int tt2) {
    if (tt2 >= T) return;
    const int t2 = P.reverse ? T - 1 - tt2 : tt2;
    const float* g = P.gx + (long)min(bg, B - 1) * P.gx_bs + (long)t2 * P.gx_ts + hcol;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((const void*)(g + q * H),
                                       (__attribute__((address_space(3))) void*)&gxs[tt2 % 3][q][64 * wave], 4, 0, 0);
  };
  gx_issue(0);
  gx_issue(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // ring: [parity][B][H / 2] pair granules (units 2p, 2p + 1 of a row)
  unsigned long long* xb = P.xbuf;
  constexpr int HP = H / 2;
  const int local = args.local ? group_on_one_xcd<G>(xb + ((long)B + b0) * HP, j, args.err, dead, &xcc_flag) : 0;
  const int ar = lane & 15, ak = 8 * (lane >> 4);
  const int nvalidp = min(BS, B - b0) * HP;

  for (int tt = 0; tt < T; ++tt) {
    const int t = P.reverse ? T - 1 - tt : tt;
    MRG_STAMP(0);
    // 1. pre[b][r] = sum_k h[b][k] W[r][k] for this wave's 16 rows
    f32x4mx acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      bf16x8 fa[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) fa[p] = mx_lds_b128(&hp[p][ar][(32 * s + ak) >> 1]);
      mx_lds_wait3(fa);
      acc = mx_mfma6(fa, wf[s], acc);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) pre[4 * (lane >> 4) + i][16 * wave + ar] = acc[i];
    MRG_STAMP(1);
    mx_step_barrier();
    MRG_STAMP(2);
    // 2. gates + cell, 3. publish, store, prefetch
    const int par = tt & 1;
    float ig = 0.0f, fg = 0.0f, gg = 0.0f, og = 0.0f;
    if (cvalid) {
      const int sl = tt % 3;
      float pv[4], gv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        pv[q] = mx_lds_f32(&pre[cb][q * U + cu]);
        gv[q] = mx_lds_f32(&gxs[sl][q][tid]);
      }
      mx_lds_wait8(pv, gv);
      const float zi = pv[0] + gv[0] + bh[0];
      const float zf = pv[1] + gv[1] + bh[1];
      const float zg = pv[2] + gv[2] + bh[2];
      const float zo = pv[3] + gv[3] + bh[3];
      ig = sigmoidf_(zi); fg = sigmoidf_(zf); gg = tanhf_(zg); og = sigmoidf_(zo);
      c = fg * c + ig * gg;
      h = og * tanhf_(c);
    }
    {  // publish h of units (cu, cu + 1) from the even lane of each pair (lanes l, l ^ 1 hold cu, cu ^ 1)
      const float hn = dpp_f<0xB1>(h);
      if (cvalid && (cu & 1) == 0 && !(args.inject == 1 && j == 0 && tt == 0))
        put_pair(xb + ((long)par * B + bg) * HP + (hcol >> 1), (unsigned)(tt + 1) & 3u, h, hn, local);
    }
    if (cvalid) {
      P.y[(long)bg * P.y_bs + (long)t * P.y_ts + hcol] = h;
      float* gs = P.gates + (long)bg * P.g_bs + (long)t * P.g_ts + hcol;
      gs[0] = ig; gs[H] = fg; gs[2 * H] = gg; gs[3 * H] = og;
      P.cs[(long)bg * P.cs_bs + (long)t * P.cs_ts + hcol] = c;
    }
    MRG_STAMP(3);
    // 4. gather h_t of the group (BS x H / 2 pair granules, 4 per thread)
    if (tt + 1 < T) {
      constexpr int NG = BS * HP / MX_NT;  // 4 pair granules: units (k, k + 1) at 4 rows
      unsigned long long* rb = xb + ((long)par * B + b0) * HP;
      float g0[NG], g1[NG];
      int idx[NG];
#pragma unroll
      for (int i = 0; i < NG; ++i) idx[i] = min(tid + MX_NT * i, nvalidp - 1);
      get_pairs_idx<NG>(rb, idx, (unsigned)(tt + 1) & 3u, g0, g1, args.err, dead);
#pragma unroll
      for (int m = 0; m < NG; ++m) {
        const int e = tid + MX_NT * m, b = e / HP, k = 2 * (e % HP);
        const bool ok = b0 + b < B;
        put_planes(b, k, ok ? g0[m] : 0.0f, ok ? g1[m] : 0.0f);
      }
    }
    gx_issue(tt + 2);   // into the slot step tt - 1 used (this wave's own reads of it are done)
    MRG_STAMP(4);
    mx_step_barrier();
    MRG_STAMP(5);
  }
  if (cvalid) {
    if (P.hT) P.hT[(long)bg * H + hcol] = h;
    if (P.cT) P.cT[(long)bg * H + hcol] = c;
  }
}

__global__ __launch_bounds__(MX_NT, 1) void lstm_bwd_mx_kernel(LstmBwdArgs args) {
  constexpr int H = MX_H, G = MX_G, BS = MX_BS, U = MX_U;
  constexpr int RPB = MX_RPB;
  __shared__ __attribute__((aligned(16))) __bf16 dgp[3][BS][RPB];   // dG as three bf16 planes
  __shared__ __attribute__((aligned(16))) float sv[3][7][BS * U];  // saved i, f, g, o, c_t, c_{t-1}, dy: step mod 3
  __shared__ int xcc_flag;
  int prob, grp, j;
  const int ngroups = (args.B + BS - 1) / BS;
  decompose(G, ngroups, args.nprob, prob, grp, j);
  const LstmBwdProblem& P = args.p[prob];
  const int B = args.B, T = args.T;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = grp * BS;
  bool dead = false;

  // W planes: wave w owns output column tiles 2 w, 2 w + 1 (B[k][n] = W[grow(k)][n], k = own gate row)
  bf16x8 wf[2][4][3];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int n = 16 * (2 * wave + ct) + (lane & 15);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float v[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) v[jj] = P.w_hh[(long)mx_grow(j, 32 * s + 8 * (lane >> 4) + jj) * H + n];
      mx_split8(make_float4(v[0], v[1], v[2], v[3]), make_float4(v[4], v[5], v[6], v[7]), wf[ct][s]);
    }
  }
  const int cb = tid / U, cu = tid % U;
  const int bg = b0 + cb;
  const bool cvalid = bg < B;
  const int hcol = j * U + cu;
  float dcn = 0.0f, dhrec = 0.0f, dgv[4];
  if (cvalid) {
    if (P.dcT) dcn = P.dcT[(long)bg * H + hcol];
    if (P.dhT) dhrec = P.dhT[(long)bg * H + hcol];
  }
  float c0v = 0.0f;   // c_{t-1} at the sequence edge
  if (cvalid && P.c0) c0v = P.c0[(long)bg * P.c0_bs + hcol];
  // saved activations of processing step tt2 -> LDS slot tt2 % 3 by LDS-DMA (global_load_lds_dword: no
  // VGPRs held in flight); wave w moves its own 64 cells, issued right after the step's hand-off poll so
  // that the next poll (whose wait covers every older load: gfx9 counts in order) finds them landed —
  // with the loads issued at the end of the step, each poll waited for them.  Rows past B read row
  // B - 1 (never used); c_{t-1} at the sequence edge and a null dy are supplied by the cells.
  auto io_issue = [&](int tt2) {
    if (tt2 >= T) return;
    const int t = P.reverse ? tt2 : T - 1 - tt2;
    const int tp = P.reverse ? t + 1 : t - 1;
    const int tq = (tp >= 0 && tp < T) ? tp : t;
    const int eb = min(bg, B - 1);
    const float* gs = P.gates + (long)eb * P.g_bs + (long)t * P.g_ts + hcol;
    const float* src[7] = {gs, gs + H, gs + 2 * H, gs + 3 * H,
                           P.cs + (long)eb * P.cs_bs + (long)t * P.cs_ts + hcol,
                           P.cs + (long)eb * P.cs_bs + (long)tq * P.cs_ts + hcol,
                           P.dy ? P.dy + (long)eb * P.dy_bs + (long)t * P.dy_ts + hcol : gs};
#pragma unroll
    for (int q = 0; q < 7; ++q)
      __builtin_amdgcn_global_load_lds((const void*)src[q],
                                       (__attribute__((address_space(3))) void*)&sv[tt2 % 3][q][64 * wave], 4, 0, 0);
  };
  io_issue(0);
  io_issue(1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned long long* xb = P.xbuf;
  const long xstride_b = (long)G * H / 2;  // per batch row: [dest G][src G][U / 2] pair granules
  const int local = args.local ? group_on_one_xcd<G>(xb + ((long)B + b0) * xstride_b, j, args.err, dead, &xcc_flag)
                               : 0;
  const int ar = lane & 15, ak = 8 * (lane >> 4);
  // the step's barriers: mx_step_barrier (the DMA data is covered by the next hand-off poll's wait)
  auto step_barrier = mx_step_barrier;

  for (int tt = 0; tt < T; ++tt) {
    const int t = P.reverse ? tt : T - 1 - tt;
    MRG_STAMP(0);
    if (cvalid) {
      if (tt > 0) {
        const int par = (tt - 1) & 1;
        unsigned long long* g = xb + ((long)par * B + bg) * xstride_b + (long)j * (H / 2) + (cu >> 1);
        float gv[G];
        get_pair_halves<G>(g, U / 2, cu & 1, (unsigned)tt & 3u, gv, args.err, dead);
        float s = 0.0f;
#pragma unroll
        for (int src = 0; src < G; ++src) s += gv[src];
        dhrec = s;
      }
      MRG_STAMP(1);
      const int sl = tt % 3;
      const float ig = sv[sl][0][tid], fg = sv[sl][1][tid], gg = sv[sl][2][tid], og = sv[sl][3][tid];
      const float cc = sv[sl][4][tid];
      const float cp = tt + 1 < T ? sv[sl][5][tid] : c0v;
      const float dyv = P.dy ? sv[sl][6][tid] : 0.0f;
      const float dh = dhrec + dyv;
      const float tc = tanhf_(cc);
      const float dc = dh * og * (1.0f - tc * tc) + dcn;
      dgv[0] = dc * gg * ig * (1.0f - ig);
      dgv[1] = dc * cp * fg * (1.0f - fg);
      dgv[2] = dc * ig * (1.0f - gg * gg);
      dgv[3] = dh * tc * og * (1.0f - og);
      dcn = dc * fg;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) dgv[q] = 0.0f;
    }
    io_issue(tt + 2);   // into the slot step tt - 1 used (this wave's own reads of it are done)
#pragma unroll
    for (int q = 0; q < 4; q += 2) {  // planes of (dG_q, dG_{q+1}): one split of the pair
      unsigned p0, p1, p2;
      split2(dgv[q], dgv[q + 1], p0, p1, p2);
      const unsigned pw[3] = {p0, p1, p2};
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        dgp[p][cb][q * U + cu] = __builtin_bit_cast(__bf16, (unsigned short)(pw[p] & 0xffffu));
        dgp[p][cb][(q + 1) * U + cu] = __builtin_bit_cast(__bf16, (unsigned short)(pw[p] >> 16));
      }
    }
    MRG_STAMP(2);
    step_barrier();
    MRG_STAMP(3);
    // partial dh_{t-1}[b][n] = sum over this member's rows of dG[b][row] W[row][n], n in this wave's
    // two column tiles; lane holds rows 4 (lane >> 4) + i, column 16 ct' + (lane & 15)
    {
      const int par = tt & 1;
      f32x4mx acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 fa[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) fa[p] = mx_lds_b128(&dgp[p][ar][32 * s + ak]);
        mx_lds_wait3(fa);
        acc[0] = mx_mfma6(fa, wf[0][s], acc[0]);
        acc[1] = mx_mfma6(fa, wf[1][s], acc[1]);
      }
      MRG_STAMP(4);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {  // pairs (n, n + 1) from the even lane (lanes l, l ^ 1 hold n, n ^ 1)
        const int n = 16 * (2 * wave + ct) + ar;
        const int dest = n / U, du = n % U;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int b = 4 * (lane >> 4) + i;
          const float vn = dpp_f<0xB1>(acc[ct][i]);
          if (b0 + b < B && (ar & 1) == 0 && !(args.inject == 2 && j == 0 && tt == 0))
            put_pair(xb + ((long)par * B + b0 + b) * xstride_b + (long)dest * (H / 2) + (long)j * (U / 2) + (du >> 1),
                     (unsigned)(tt + 1) & 3u, acc[ct][i], vn, local);
        }
      }
    }
    if (cvalid) {   // dG of this step (fp32, from registers)
      float* dgo = P.dG + (long)bg * P.dG_bs + (long)t * P.dG_ts + hcol;
#pragma unroll
      for (int q = 0; q < 4; ++q) dgo[q * H] = dgv[q];
    }
    MRG_STAMP(5);
    step_barrier();
    MRG_STAMP(6);
  }
  if (cvalid) {
    if (P.dh0) {
      const int par = (T - 1) & 1;
      unsigned long long* g = xb + ((long)par * B + bg) * xstride_b + (long)j * (H / 2) + (cu >> 1);
      float gv[G];
      get_pair_halves<G>(g, U / 2, cu & 1, (unsigned)T & 3u, gv, args.err, dead);
      float s = 0.0f;
#pragma unroll
      for (int src = 0; src < G; ++src) s += gv[src];
      P.dh0[(long)bg * H + hcol] = s;
    }
    if (P.dc0) P.dc0[(long)bg * H + hcol] = dcn;
  }
}

// 0 when the MFMA form does not apply or its grid does not fit (the caller takes lstm.hip's kernels)
int launch_fwd_mx(const LstmFwdArgs& a, int cus, hipStream_t s) {
  const long nblk = (long)a.nprob * ((a.B + MX_BS - 1) / MX_BS) * MX_G;
  if (!fits(lstm_fwd_mx_kernel, MX_NT, nblk, cus)) return 0;
  klaunch(lstm_fwd_mx_kernel, (unsigned)nblk, MX_NT, 0, s, a);
  return check_launch("lstm_fwd_mx_kernel") ? -1 : 1;
}

int launch_bwd_mx(const LstmBwdArgs& a, int cus, hipStream_t s) {
  const long nblk = (long)a.nprob * ((a.B + MX_BS - 1) / MX_BS) * MX_G;
  if (!fits(lstm_bwd_mx_kernel, MX_NT, nblk, cus)) return 0;
  klaunch(lstm_bwd_mx_kernel, (unsigned)nblk, MX_NT, 0, s, a);
  return check_launch("lstm_bwd_mx_kernel") ? -1 : 1;
}

}  // namespace mrg
