// Row-parallel HBM-bound kernels: fused residual-add + LayerNorm (fwd/bwd),
// masked regression loss (Huber / MSE / L1 / SmoothL1, fwd/bwd) and the fused
// multi-tensor AdamW step.  One 64-lane wave owns one row; row reductions are
// wave shuffles (no LDS); parameter-gradient column sums go through per-block
// fp32 partials reduced in a fixed order (deterministic).
#include <atomic>
#include <mutex>
#include "mrg_common.h"

namespace mrg {

// ------------------------------------------------------------- residual + LayerNorm
// y = LN(a + b) * gamma + beta (ResidualConnection, residual_connection.py:20-37)
template <int EPL>  // elements per lane: E <= 64 * EPL (lanes past E idle)
__global__ __launch_bounds__(256) void resln_fwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                                        float* __restrict__ y, float* __restrict__ mean_out,
                                                        float* __restrict__ rstd_out, int rows, float eps, int E) {
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* pa = a + (long)row * E;
  const float* pb = b + (long)row * E;
  float x[EPL];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    int c = i * 64 + lane;
    x[i] = c < E ? pa[c] + pb[c] : 0.0f;
    s += x[i];
  }
  const float invE = 1.0f / (float)E;
  float mean = wave_sum(s) * invE;
  float v = 0.0f;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    float d = (i * 64 + lane) < E ? x[i] - mean : 0.0f;
    v += d * d;
  }
  float var = wave_sum(v) * invE;
  float rstd = rsqrtf(var + eps);
  float* py = y + (long)row * E;
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    int c = i * 64 + lane;
    if (c < E) py[c] = (x[i] - mean) * rstd * gamma[c] + beta[c];
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * gamma
// per-block partial column sums of dy*xhat and dy -> part[blk][2][E]
template <int EPL>
__global__ __launch_bounds__(256) void resln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ a,
                                                        const float* __restrict__ b, const float* __restrict__ gamma,
                                                        const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                        float* __restrict__ dx, float* __restrict__ part,
                                                        int rows, int rows_per_block, int E) {
  constexpr int EMAX = 64 * EPL;
  __shared__ float red[4][2][EMAX];
  int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float dg[EPL], db[EPL];
#pragma unroll
  for (int i = 0; i < EPL; ++i) { dg[i] = 0.0f; db[i] = 0.0f; }
  int r0 = blockIdx.x * rows_per_block;
  int r1 = min(rows, r0 + rows_per_block);
  for (int row = r0 + wave; row < r1; row += 4) {
    const float* pa = a + (long)row * E;
    const float* pb = b + (long)row * E;
    const float* pdy = dy + (long)row * E;
    float mean = mean_in[row], rstd = rstd_in[row];
    float xh[EPL], g[EPL];
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int i = 0; i < EPL; ++i) {
      int c = i * 64 + lane;
      bool ok = c < E;
      float d = ok ? pdy[c] : 0.0f;
      xh[i] = ok ? (pa[c] + pb[c] - mean) * rstd : 0.0f;
      g[i] = ok ? d * gamma[c] : 0.0f;
      s1 += g[i];
      s2 += g[i] * xh[i];
      dg[i] += d * xh[i];
      db[i] += d;
    }
    const float invE = 1.0f / (float)E;
    float m1 = wave_sum(s1) * invE;
    float m2 = wave_sum(s2) * invE;
    float* pdx = dx + (long)row * E;
#pragma unroll
    for (int i = 0; i < EPL; ++i)
      if (i * 64 + lane < E) pdx[i * 64 + lane] = rstd * (g[i] - m1 - xh[i] * m2);
  }
#pragma unroll
  for (int i = 0; i < EPL; ++i) {
    red[wave][0][i * 64 + lane] = dg[i];
    red[wave][1][i * 64 + lane] = db[i];
  }  // lanes past E hold zeros; only c < E is read below
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * E; c += 256) {
    int k = c / E, e = c % E;
    float s = red[0][k][e] + red[1][k][e] + red[2][k][e] + red[3][k][e];
    part[((long)blockIdx.x * 2 + k) * E + e] = s;
  }
}

// float4 forms for E % 4 == 0 (every LN of the benchmark: E = 256): a lane owns 4 consecutive
// columns per 256-column chunk, so a wave moves a whole 1-KB row per instruction; the backward
// keeps two rows in flight per wave to cover HBM latency.
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

template <int EPV>  // float4 chunks per lane: E <= 256 * EPV
__device__ __forceinline__ void resln_fwd_v4_rows(const float* __restrict__ a, const float* __restrict__ b,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  float* __restrict__ y, float* __restrict__ mean_out,
                                                  float* __restrict__ rstd_out, int rows, float eps, int E,
                                                  RowMap ymap) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* pa = a + (long)row * E;
  const float* pb = b + (long)row * E;
  float4 x[EPV];
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < EPV; ++i) {
    const int c = i * 256 + lane * 4;
    x[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < E) {
      float4 u = ld4(pa + c), v = ld4(pb + c);
      x[i] = make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
    }
    s += (x[i].x + x[i].y) + (x[i].z + x[i].w);
  }
  const float invE = 1.0f / (float)E;
  const float mean = wave_sum(s) * invE;
  float var = 0.0f;
#pragma unroll
  for (int i = 0; i < EPV; ++i) {
    if (i * 256 + lane * 4 < E) {
      float d0 = x[i].x - mean, d1 = x[i].y - mean, d2 = x[i].z - mean, d3 = x[i].w - mean;
      var += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    }
  }
  const float rstd = rsqrtf(wave_sum(var) * invE + eps);
  float* py = y + ymap.off(row);  // the output rows may be laid out differently (time-major -> [B, T, E])
#pragma unroll
  for (int i = 0; i < EPV; ++i) {
    const int c = i * 256 + lane * 4;
    if (c < E) {
      float4 g = ld4(gamma + c), bt = ld4(beta + c);
      st4(py + c, make_float4((x[i].x - mean) * rstd * g.x + bt.x, (x[i].y - mean) * rstd * g.y + bt.y,
                              (x[i].z - mean) * rstd * g.z + bt.z, (x[i].w - mean) * rstd * g.w + bt.w));
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

template <int EPV>
__global__ __launch_bounds__(256) void resln_fwd_v4_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* __restrict__ y,
                                                           float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                           int rows, float eps, int E, RowMap ymap) {
  resln_fwd_v4_rows<EPV>(a, b, gamma, beta, y, mean_out, rstd_out, rows, eps, E, ymap);
}

// Same-shape residual LayerNorms batched into one launch (blockIdx.y = problem): the encoder
// stack's per-diagonal chunks (encoder_stack.py), each with its own tensors, parameters and map.
static constexpr int MRG_LN_MAX = 16;
struct LnBatch {
  const float* a[MRG_LN_MAX];
  const float* b[MRG_LN_MAX];
  const float* gamma[MRG_LN_MAX];
  const float* beta[MRG_LN_MAX];  // backward: unused
  const float* dy[MRG_LN_MAX];    // backward only
  float* y[MRG_LN_MAX];           // forward: output; backward: dx
  float* mean[MRG_LN_MAX];
  float* rstd[MRG_LN_MAX];
  float* part[MRG_LN_MAX];        // backward: dgamma / dbeta partials
  RowMap map[MRG_LN_MAX];         // forward: output rows; backward: incoming-gradient rows
};

template <int EPV>
__global__ __launch_bounds__(256) void resln_fwd_v4_batched_kernel(LnBatch lb, int rows, float eps, int E) {
  const int p = blockIdx.y;
  resln_fwd_v4_rows<EPV>(lb.a[p], lb.b[p], lb.gamma[p], lb.beta[p], lb.y[p], lb.mean[p], lb.rstd[p], rows, eps, E,
                         lb.map[p]);
}

template <int EPV>
__device__ __forceinline__ void resln_bwd_v4_rows(const float* __restrict__ dy, const float* __restrict__ a,
                                                  const float* __restrict__ b, const float* __restrict__ gamma,
                                                  const float* __restrict__ mean_in,
                                                  const float* __restrict__ rstd_in, float* __restrict__ dx,
                                                  float* __restrict__ part, int rows, int rows_per_block, int E,
                                                  RowMap dmap) {
  constexpr int EMAX = 256 * EPV;
  __shared__ __attribute__((aligned(16))) float red[4][2][EMAX];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float4 dg[EPV], db[EPV], gm[EPV];
#pragma unroll
  for (int i = 0; i < EPV; ++i) {
    dg[i] = db[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int c = i * 256 + lane * 4;
    gm[i] = c < E ? ld4(gamma + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  const float invE = 1.0f / (float)E;
  for (int row = r0 + wave; row < r1; row += 8) {
    // two rows per pass (row, row + 4): all loads issued before any reduction
    const bool two = row + 4 < r1;
    float4 d[2][EPV], x[2][EPV];
    float mean[2], rstd[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int rr = q ? (two ? row + 4 : row) : row;
      mean[q] = mean_in[rr];
      rstd[q] = rstd_in[rr];
#pragma unroll
      for (int i = 0; i < EPV; ++i) {
        const int c = i * 256 + lane * 4;
        d[q][i] = x[q][i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c < E) {
          d[q][i] = ld4(dy + dmap.off(rr) + c);
          float4 u = ld4(a + (long)rr * E + c), v = ld4(b + (long)rr * E + c);
          x[q][i] = make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (q == 1 && !two) break;
      const int rr = row + 4 * q;
      float s1 = 0.0f, s2 = 0.0f;
      float4 xh[EPV], g[EPV];
#pragma unroll
      for (int i = 0; i < EPV; ++i) {
        const float m = mean[q], r = rstd[q];
        xh[i] = make_float4((x[q][i].x - m) * r, (x[q][i].y - m) * r, (x[q][i].z - m) * r, (x[q][i].w - m) * r);
        if (i * 256 + lane * 4 >= E) xh[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        g[i] = make_float4(d[q][i].x * gm[i].x, d[q][i].y * gm[i].y, d[q][i].z * gm[i].z, d[q][i].w * gm[i].w);
        s1 += (g[i].x + g[i].y) + (g[i].z + g[i].w);
        s2 += (g[i].x * xh[i].x + g[i].y * xh[i].y) + (g[i].z * xh[i].z + g[i].w * xh[i].w);
        dg[i].x += d[q][i].x * xh[i].x; dg[i].y += d[q][i].y * xh[i].y;
        dg[i].z += d[q][i].z * xh[i].z; dg[i].w += d[q][i].w * xh[i].w;
        db[i].x += d[q][i].x; db[i].y += d[q][i].y; db[i].z += d[q][i].z; db[i].w += d[q][i].w;
      }
      const float m1 = wave_sum(s1) * invE, m2 = wave_sum(s2) * invE, r = rstd[q];
#pragma unroll
      for (int i = 0; i < EPV; ++i) {
        const int c = i * 256 + lane * 4;
        if (c < E)
          st4(dx + (long)rr * E + c,
              make_float4(r * (g[i].x - m1 - xh[i].x * m2), r * (g[i].y - m1 - xh[i].y * m2),
                          r * (g[i].z - m1 - xh[i].z * m2), r * (g[i].w - m1 - xh[i].w * m2)));
      }
    }
  }
#pragma unroll
  for (int i = 0; i < EPV; ++i) {
    const int c = i * 256 + lane * 4;
    st4(&red[wave][0][c], dg[i]);
    st4(&red[wave][1][c], db[i]);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * E; c += 256) {
    const int k = c / E, e = c % E;
    part[((long)blockIdx.x * 2 + k) * E + e] = (red[0][k][e] + red[1][k][e]) + (red[2][k][e] + red[3][k][e]);
  }
}

template <int EPV>
__global__ __launch_bounds__(256) void resln_bwd_v4_kernel(const float* __restrict__ dy, const float* __restrict__ a,
                                                           const float* __restrict__ b,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ mean_in,
                                                           const float* __restrict__ rstd_in, float* __restrict__ dx,
                                                           float* __restrict__ part, int rows, int rows_per_block,
                                                           int E, RowMap dmap) {
  resln_bwd_v4_rows<EPV>(dy, a, b, gamma, mean_in, rstd_in, dx, part, rows, rows_per_block, E, dmap);
}

template <int EPV>
__global__ __launch_bounds__(256) void resln_bwd_v4_batched_kernel(LnBatch lb, int rows, int rows_per_block, int E) {
  const int p = blockIdx.y;
  resln_bwd_v4_rows<EPV>(lb.dy[p], lb.a[p], lb.b[p], lb.gamma[p], lb.mean[p], lb.rstd[p], lb.y[p], lb.part[p], rows,
                         rows_per_block, E, lb.map[p]);
}

// dgamma / dbeta: sum the per-block partials part[nblk][2][E] in ONE launch of (2E / 64 column
// blocks) x (R row groups) workgroups.  Group g sums its contiguous rows (one lane per column, 4
// waves interleaved over the rows, combined in LDS in fixed order) and stores the group sum over
// its own first row (only it reads that row, so the partials are consumed in place); then it draws
// a ticket for its column block, and the workgroup that draws the last one adds the R group sums in
// g order and writes the result.  Deterministic (every sum in a fixed order).  Round 3's form used
// 8 workgroups that each walked all 600 partial rows of a 19,200-row LayerNorm: 13.3 us per call,
// 1.2 % of HBM.  4-wave workgroups, so they still fit beside a persistent
// recurrence as deferred parameter-gradient products.
constexpr int RESLN_TSLOTS = 256;                // ticket sets: one per (device, stream, capture) (see launcher)
constexpr int RESLN_MAXCB = 32;                  // column blocks: 2E / 64 <= 32 (E <= 1024)
__device__ unsigned g_resln_tickets[RESLN_TSLOTS * RESLN_MAXCB];

__global__ __launch_bounds__(256) void resln_param_reduce_kernel(float* part, int nblk, int E, float* dgamma,
                                                                 float* dbeta, int accumulate, int R,
                                                                 unsigned* tick) {
  __shared__ float red[4][64];
  __shared__ int last_flag;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cb = blockIdx.x, g = blockIdx.y;
  const int c = cb * 64 + lane;
  const int E2 = 2 * E;
  const int r0 = (int)((long)nblk * g / R), r1 = (int)((long)nblk * (g + 1) / R);
  // wave w sums rows r0 + w + 4j: eight independent loads in flight per round of 32 rows
  float s = 0.0f;
  if (c < E2) {
    for (int i0 = r0 + wave; i0 < r1; i0 += 32) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + 4 * j;
        v[j] = i < r1 ? part[(long)i * E2 + c] : 0.0f;
      }
      s += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    }
  }
  red[wave][lane] = s;
  __syncthreads();
  const float v = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  if (R > 1) {
    if (wave == 0 && c < E2) part[(long)r0 * E2 + c] = v;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(tick + cb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == (unsigned)(R - 1);
      if (last) __hip_atomic_store(tick + cb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = last;
    }
    __syncthreads();
    if (!last_flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // every wave reads the other groups' rows
    // the group sums (each group's first row), wave w taking groups w + 4j, four loads in flight
    float t = 0.0f;
    if (c < E2) {
      for (int q0 = wave; q0 < R; q0 += 16) {
        float u[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = q0 + 4 * j;
          u[j] = q < R ? part[(long)((long)nblk * q / R) * E2 + c] : 0.0f;
        }
        t += (u[0] + u[1]) + (u[2] + u[3]);
      }
    }
    __syncthreads();   // every wave has read red[] above
    red[wave][lane] = t;
    __syncthreads();
  }
  if (wave == 0 && c < E2) {
    const float t = R > 1 ? (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]) : v;
    float* out = c < E ? dgamma + c : dbeta + (c - E);
    *out = accumulate ? *out + t : t;
  }
}

// ------------------------------------------------------------------ loss
// Masked regression loss over y viewed as [B, T, F] (batch stride ys, time stride F),
// target contiguous [B, T, F]; lossfun() of lstmformer.py:313-325 with the
// padding mask and delta scaler of training_step (lstmformer.py:372-380).
struct LossArgs {
  const float* y;
  long ys;
  const float* t;
  int B, T, F;
  int type;  // 0 huber, 1 mse, 2 l1, 3 smoothl1
  float delta, beta;
  int mask_padding;
  int delta_start;
  float dscale;  // sqrt(delta_loss_scale) for features >= delta_start
};

// elementwise loss l(d) and dl/dd of the four reference loss types
__device__ __forceinline__ void loss_fn(int type, float d, float delta, float beta, float& l, float& g) {
  const float z = fabsf(d);
  switch (type) {
    case 0:
      l = z < delta ? 0.5f * d * d : delta * (z - 0.5f * delta);
      g = d <= -delta ? -delta : (d >= delta ? delta : d);
      break;
    case 1:
      l = d * d;
      g = 2.0f * d;
      break;
    case 2:
      l = z;
      g = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
      break;
    default:
      l = z < beta ? 0.5f * d * d / beta : z - 0.5f * beta;
      g = z < beta ? d / beta : (d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f));
      break;
  }
}

__device__ __forceinline__ void loss_elem(const LossArgs& a, long i, float& l, float& g) {
  int f = i % a.F;
  long bt = i / a.F;
  int b = bt / a.T, tt = bt % a.T;
  float y = a.y[(long)b * a.ys + (long)tt * a.F + f];
  float t = a.t[i];
  float m = (a.mask_padding && t == -100.0f) ? 0.0f : 1.0f;
  float s = f >= a.delta_start ? a.dscale : 1.0f;
  float d = (y * m) * s - (t * m) * s;
  loss_fn(a.type, d, a.delta, a.beta, l, g);
  g *= s * m;
}

// ------------------------------------------------------------- broadcast-target loss
// Metaformer.prediction returns target [B,T,F] * motion_s_mask [Tm,B,1,F] = [Tm,B,T,F]
// (lstmformer.py:434-435); generation_step / scheduled-sampling training_step take the masked
// loss over that broadcast tensor (the [:, :, start:] scaler then indexes its T axis).  Per
// (b, t, f) the Tm copies collapse analytically: with c1 = #{t' : ms[b,t',f] != -100}, c0 = Tm - c1,
//   sum_t' l = c1 * (target pad ? 0 : l(s p - s tgt)) + c0 * l(s p)
// so nothing of size Tm*B*T*F is ever formed.  counts[b*F + f] = c1 (bcast_count_kernel).
struct BcastArgs {
  const float* y;
  long ys;
  const float* t;
  const float* counts;
  int B, T, F, Tm;
  int type;
  float delta, beta;
  int t_start;   // scaler applies to time index t >= t_start (T // (delta_order + 1); > T: none)
  float dscale;
};

__global__ __launch_bounds__(256) void bcast_count_kernel(const float* __restrict__ ms, long ms_bs, long ms_ts,
                                                          int B, int Tm, int F, float* __restrict__ counts) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * F) return;
  const int b = i / F, f = i % F;
  const float* p = ms + (long)b * ms_bs + f;
  int c = 0;
  for (int t = 0; t < Tm; ++t) c += p[(long)t * ms_ts] != -100.0f;
  counts[i] = (float)c;
}

__device__ __forceinline__ void bcast_elem(const BcastArgs& a, long i, float& l, float& g) {
  const int f = i % a.F;
  const long bt = i / a.F;
  const int b = bt / a.T, tt = bt % a.T;
  const float y = a.y[(long)b * a.ys + (long)tt * a.F + f];
  const float t = a.t[i];
  const float c1 = a.counts[b * a.F + f];
  const float c0 = (float)a.Tm - c1;
  const float s = tt >= a.t_start ? a.dscale : 1.0f;
  float l1 = 0.0f, g1 = 0.0f, l0, g0;
  if (t != -100.0f) loss_fn(a.type, y * s - t * s, a.delta, a.beta, l1, g1);
  loss_fn(a.type, y * s, a.delta, a.beta, l0, g0);
  l = c1 * l1 + c0 * l0;
  g = (c1 * g1 + c0 * g0) * s;
}

__global__ __launch_bounds__(256) void bcast_loss_partial_kernel(BcastArgs a, float* part) {
  const long n = (long)a.B * a.T * a.F;
  float acc = 0.0f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float l, g;
    bcast_elem(a, i, l, g);
    acc += l;
  }
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void bcast_loss_bwd_kernel(BcastArgs a, const float* grad_out, float inv_n,
                                                             float* dy) {
  const long n = (long)a.B * a.T * a.F;
  const float go = grad_out[0] * inv_n;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float l, g;
    bcast_elem(a, i, l, g);
    const int f = i % a.F;
    const long bt = i / a.F;
    const int b = bt / a.T, tt = bt % a.T;
    dy[(long)b * a.ys + (long)tt * a.F + f] = g * go;
  }
}

__global__ __launch_bounds__(256) void loss_fwd_partial_kernel(LossArgs a, float* part) {
  long n = (long)a.B * a.T * a.F;
  float acc = 0.0f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float l, g;
    loss_elem(a, i, l, g);
    acc += l;
  }
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void loss_fwd_final_kernel(const float* part, int nblk, float inv_n, float* out) {
  float acc = 0.0f;
  for (int i = threadIdx.x; i < nblk; i += 64) acc += part[i];
  acc = wave_sum(acc);
  if (threadIdx.x == 0) out[0] = acc * inv_n;
}

// dy (same strided layout as y) = grad_out * dloss/dy / N
__global__ __launch_bounds__(256) void loss_bwd_kernel(LossArgs a, const float* grad_out, float inv_n,
                                                       float* dy) {
  long n = (long)a.B * a.T * a.F;
  float go = grad_out[0] * inv_n;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float l, g;
    loss_elem(a, i, l, g);
    int f = i % a.F;
    long bt = i / a.F;
    int b = bt / a.T, tt = bt % a.T;
    dy[(long)b * a.ys + (long)tt * a.F + f] = g * go;
  }
}

// ------------------------------------------------------------------ AdamW
// torch.optim.AdamW (lstmformer.py:327-333), one launch over the flat buffers.
// step / lr live on the device so a captured graph replays correct bias corrections.
// err (nullable): the persistent-recurrence error flag; a set flag means this step's gradients
// are garbage (a hand-off timed out), so the update and the step count are skipped.
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, long n,
                                                    const float* __restrict__ step_lr, float wd, float b1,
                                                    float b2, float eps, const int* __restrict__ err) {
  if (err && *err) return;
  float t = step_lr[0] + 1.0f;
  float lr = step_lr[1];
  float bc1 = 1.0f - powf(b1, t);
  float bc2s = sqrtf(1.0f - powf(b2, t));
  float step_size = lr / bc1;
  float decay = 1.0f - lr * wd;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float gi = g[i];
    float pi = p[i] * decay;
    float mi = m[i] + (1.0f - b1) * (gi - m[i]);
    float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] = pi - step_size * mi / (sqrtf(vi) / bc2s + eps);
  }
}

__global__ void adamw_step_inc_kernel(float* step_lr, const int* err) {
  if (!(err && *err)) step_lr[0] += 1.0f;
}

}  // namespace mrg

using namespace mrg;

MRG_API int mrg_residual_layernorm_fwd(int rows, int E, const float* a, const float* b,
                                       const float* gamma, const float* beta, float eps, float* y,
                                       float* mean, float* rstd, hipStream_t stream) {
  if (rows == 0) return 0;
  dim3 grid((rows + 3) / 4);
  MRG_REQUIRE(E >= 1 && E <= 1024, "mrg_residual_layernorm_fwd: unsupported E=%d", E);
  const bool v4 = (E % 4) == 0 && (((uintptr_t)a | (uintptr_t)b | (uintptr_t)y | (uintptr_t)gamma |
                                       (uintptr_t)beta) & 15) == 0;
  if (v4) {
    const int epv = (E + 255) / 256;
    const RowMap plain{E, 0, 0};
    if (epv == 1) resln_fwd_v4_kernel<1><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E, plain);
    else if (epv == 2) resln_fwd_v4_kernel<2><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E, plain);
    else resln_fwd_v4_kernel<4><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E, plain);
    return check_launch("resln_fwd_v4_kernel");
  }
  const int epl = (E + 63) / 64;
  if (epl <= 1) resln_fwd_kernel<1><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E);
  else if (epl <= 2) resln_fwd_kernel<2><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E);
  else if (epl <= 4) resln_fwd_kernel<4><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E);
  else if (epl <= 8) resln_fwd_kernel<8><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E);
  else resln_fwd_kernel<16><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E);
  return check_launch("resln_fwd_kernel");
}

static constexpr int RESLN_RPB = 32;  // rows per backward block (600 blocks at B*T = 19200)

MRG_API size_t mrg_residual_layernorm_bwd_workspace_bytes(int rows, int E) {
  int nblk = (rows + RESLN_RPB - 1) / RESLN_RPB;
  return (size_t)nblk * 2 * E * sizeof(float);
}

MRG_API int mrg_residual_layernorm_param_reduce(int rows, int E, float* workspace, float* dgamma,
                                                float* dbeta, int accumulate, hipStream_t stream);

MRG_API int mrg_residual_layernorm_bwd(int rows, int E, const float* dy, const float* a,
                                       const float* b, const float* gamma, const float* mean,
                                       const float* rstd, float* dx, float* dgamma, float* dbeta,
                                       int accumulate, float* workspace, hipStream_t stream) {
  if (rows == 0) return 0;
  const int rpb = RESLN_RPB;
  int nblk = (rows + rpb - 1) / rpb;
  MRG_REQUIRE(E >= 1 && E <= 1024, "mrg_residual_layernorm_bwd: unsupported E=%d", E);
  const bool v4 = (E % 4) == 0 && (((uintptr_t)dy | (uintptr_t)a | (uintptr_t)b | (uintptr_t)dx |
                                       (uintptr_t)gamma) & 15) == 0;
  const int epl = (E + 63) / 64;
  if (v4) {
    const int epv = (E + 255) / 256;
    const RowMap plain{E, 0, 0};
    if (epv == 1) resln_bwd_v4_kernel<1><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, rpb, E, plain);
    else if (epv == 2) resln_bwd_v4_kernel<2><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, rpb, E, plain);
    else resln_bwd_v4_kernel<4><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, rpb, E, plain);
  } else if (epl <= 1) resln_bwd_kernel<1><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, rpb, E);
  else if (epl <= 2) resln_bwd_kernel<2><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, rpb, E);
  else if (epl <= 4) resln_bwd_kernel<4><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, rpb, E);
  else if (epl <= 8) resln_bwd_kernel<8><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, rpb, E);
  else resln_bwd_kernel<16><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, rpb, E);
  if (check_launch("resln_bwd_kernel")) return 1;
  if (!dgamma && !dbeta) return 0;  // partials stay in the workspace (mrg_residual_layernorm_param_reduce)
  MRG_REQUIRE(dgamma && dbeta, "mrg_residual_layernorm_bwd: dgamma and dbeta must both be given or both null");
  return mrg_residual_layernorm_param_reduce(rows, E, workspace, dgamma, dbeta, accumulate, stream);
}

// Row-mapped forms (E % 4 == 0, 16-B aligned rows): the output rows of the forward and the incoming
// gradient rows of the backward follow a RowMap, offset(r) = (r / div) * ld_hi + (r % div) * ld_lo
// (div = 0: r * ld_lo), so a time-major [T, B, E] chunk writes / reads a batch-major [B, T, E] tensor
// in place (the encoder stack's last LayerNorm, encoder_stack.py).  The backward writes the per-block
// dgamma / dbeta partials into the workspace for mrg_residual_layernorm_param_reduce.
MRG_API int mrg_residual_layernorm_fwd_map(int rows, int E, const float* a, const float* b, const float* gamma,
                                           const float* beta, float eps, float* y, long y_lo, long y_hi, int y_div,
                                           float* mean, float* rstd, hipStream_t stream) {
  if (rows == 0) return 0;
  MRG_REQUIRE(E % 4 == 0 && E <= 1024 && y_lo % 4 == 0 && y_hi % 4 == 0 &&
                  (((uintptr_t)a | (uintptr_t)b | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta) & 15) == 0,
              "mrg_residual_layernorm_fwd_map: E %% 4 == 0 and 16-byte aligned rows required (E=%d)", E);
  const RowMap m{y_lo, y_hi, y_div};
  dim3 grid((rows + 3) / 4);
  const int epv = (E + 255) / 256;
  if (epv == 1) resln_fwd_v4_kernel<1><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E, m);
  else if (epv == 2) resln_fwd_v4_kernel<2><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E, m);
  else resln_fwd_v4_kernel<4><<<grid, 256, 0, stream>>>(a, b, gamma, beta, y, mean, rstd, rows, eps, E, m);
  return check_launch("resln_fwd_v4_kernel");
}

MRG_API int mrg_residual_layernorm_bwd_map(int rows, int E, const float* dy, long dy_lo, long dy_hi, int dy_div,
                                           const float* a, const float* b, const float* gamma, const float* mean,
                                           const float* rstd, float* dx, float* workspace, hipStream_t stream) {
  if (rows == 0) return 0;
  MRG_REQUIRE(E % 4 == 0 && E <= 1024 && dy_lo % 4 == 0 && dy_hi % 4 == 0 &&
                  (((uintptr_t)dy | (uintptr_t)a | (uintptr_t)b | (uintptr_t)dx | (uintptr_t)gamma) & 15) == 0,
              "mrg_residual_layernorm_bwd_map: E %% 4 == 0 and 16-byte aligned rows required (E=%d)", E);
  const RowMap m{dy_lo, dy_hi, dy_div};
  const int nblk = (rows + RESLN_RPB - 1) / RESLN_RPB;
  const int epv = (E + 255) / 256;
  if (epv == 1) resln_bwd_v4_kernel<1><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, RESLN_RPB, E, m);
  else if (epv == 2) resln_bwd_v4_kernel<2><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, RESLN_RPB, E, m);
  else resln_bwd_v4_kernel<4><<<nblk, 256, 0, stream>>>(dy, a, b, gamma, mean, rstd, dx, workspace, rows, RESLN_RPB, E, m);
  return check_launch("resln_bwd_v4_kernel");
}

// n same-shape row-mapped residual LayerNorms in one launch (E % 4 == 0, E <= 1024, 16-B aligned
// rows): problem p reads a[p] + b[p] (rows of E) and writes y[p] through its own map (y_lo, y_hi,
// y_div), mean[p], rstd[p].
MRG_API int mrg_residual_layernorm_fwd_batched(int n, int rows, int E, const float* const* a, const float* const* b,
                                               const float* const* gamma, const float* const* beta, float eps,
                                               float* const* y, const long* y_lo, const long* y_hi,
                                               const int* y_div, float* const* mean, float* const* rstd,
                                               hipStream_t stream) {
  MRG_REQUIRE(n >= 0 && n <= MRG_LN_MAX, "mrg_residual_layernorm_fwd_batched: n %d out of range", n);
  if (n == 0 || rows == 0) return 0;
  MRG_REQUIRE(E % 4 == 0 && E <= 1024, "mrg_residual_layernorm_fwd_batched: E %d", E);
  LnBatch lb;
  memset(&lb, 0, sizeof(lb));
  for (int p = 0; p < n; ++p) {
    MRG_REQUIRE(y_lo[p] % 4 == 0 && y_hi[p] % 4 == 0 &&
                    (((uintptr_t)a[p] | (uintptr_t)b[p] | (uintptr_t)y[p] | (uintptr_t)gamma[p] |
                      (uintptr_t)beta[p]) & 15) == 0,
                "mrg_residual_layernorm_fwd_batched: 16-byte aligned rows required (problem %d)", p);
    lb.a[p] = a[p]; lb.b[p] = b[p]; lb.gamma[p] = gamma[p]; lb.beta[p] = beta[p];
    lb.y[p] = y[p]; lb.mean[p] = mean[p]; lb.rstd[p] = rstd[p];
    lb.map[p] = RowMap{y_lo[p], y_hi[p], y_div[p]};
  }
  dim3 grid((rows + 3) / 4, n);
  const int epv = (E + 255) / 256;
  if (epv == 1) resln_fwd_v4_batched_kernel<1><<<grid, 256, 0, stream>>>(lb, rows, eps, E);
  else if (epv == 2) resln_fwd_v4_batched_kernel<2><<<grid, 256, 0, stream>>>(lb, rows, eps, E);
  else resln_fwd_v4_batched_kernel<4><<<grid, 256, 0, stream>>>(lb, rows, eps, E);
  return check_launch("resln_fwd_v4_batched_kernel");
}

// Backward of n same-shape residual LayerNorms in one launch: problem p's incoming gradient rows
// through its map (dy_lo, dy_hi, dy_div), dx[p] rows of E, per-block dgamma / dbeta partials into
// ws[p] (mrg_residual_layernorm_param_reduce reduces them).
MRG_API int mrg_residual_layernorm_bwd_batched(int n, int rows, int E, const float* const* dy, const long* dy_lo,
                                               const long* dy_hi, const int* dy_div, const float* const* a,
                                               const float* const* b, const float* const* gamma,
                                               const float* const* mean, const float* const* rstd,
                                               float* const* dx, float* const* ws, hipStream_t stream) {
  MRG_REQUIRE(n >= 0 && n <= MRG_LN_MAX, "mrg_residual_layernorm_bwd_batched: n %d out of range", n);
  if (n == 0 || rows == 0) return 0;
  MRG_REQUIRE(E % 4 == 0 && E <= 1024, "mrg_residual_layernorm_bwd_batched: E %d", E);
  LnBatch lb;
  memset(&lb, 0, sizeof(lb));
  for (int p = 0; p < n; ++p) {
    MRG_REQUIRE(dy_lo[p] % 4 == 0 && dy_hi[p] % 4 == 0 &&
                    (((uintptr_t)dy[p] | (uintptr_t)a[p] | (uintptr_t)b[p] | (uintptr_t)dx[p] |
                      (uintptr_t)gamma[p]) & 15) == 0,
                "mrg_residual_layernorm_bwd_batched: 16-byte aligned rows required (problem %d)", p);
    lb.dy[p] = dy[p]; lb.a[p] = a[p]; lb.b[p] = b[p]; lb.gamma[p] = gamma[p];
    lb.mean[p] = const_cast<float*>(mean[p]); lb.rstd[p] = const_cast<float*>(rstd[p]);
    lb.y[p] = dx[p]; lb.part[p] = ws[p];
    lb.map[p] = RowMap{dy_lo[p], dy_hi[p], dy_div[p]};
  }
  dim3 grid((rows + RESLN_RPB - 1) / RESLN_RPB, n);
  const int epv = (E + 255) / 256;
  if (epv == 1) resln_bwd_v4_batched_kernel<1><<<grid, 256, 0, stream>>>(lb, rows, RESLN_RPB, E);
  else if (epv == 2) resln_bwd_v4_batched_kernel<2><<<grid, 256, 0, stream>>>(lb, rows, RESLN_RPB, E);
  else resln_bwd_v4_batched_kernel<4><<<grid, 256, 0, stream>>>(lb, rows, RESLN_RPB, E);
  return check_launch("resln_bwd_v4_batched_kernel");
}

// The ticket set of a launch belongs to its (device, stream, capture id): launches on one stream run
// one after the other (in a captured graph, nodes of one capture stream are chained), and every ticket
// is back at 0 before a launch ends, so one set per stream is never shared by two launches in flight,
// however far another stream lags (a rotation over a global pool could hand two
// overlapping launches on different streams the same set).  Under capture the capture id is part of
// the key: two graphs captured on the same capture stream (torch.cuda.graph's shared
// default one) hold different sets, so they may also be replayed concurrently.  Slots are never
// recycled (a graph's nodes keep their pointer for its lifetime); when the table is full the reduce
// runs ticket-free (R = 1: one workgroup per column block walks every partial row, slower, and its
// summation order differs from R > 1 in the last bits).
// The symbol is resolved per device.
static std::mutex g_tick_mu;
static struct { int dev; hipStream_t s; unsigned long long cap; } g_tick_owner[RESLN_TSLOTS];
static int g_tick_used = 0;
static void* g_tick_base[64];

// *tick = nullptr (and return 0) when the table is full: the caller then runs the ticket-free form.
static int resln_tickets(hipStream_t stream, unsigned** tick) {
  int dev = 0;
  MRG_HIP(hipGetDevice(&dev));
  MRG_REQUIRE(dev >= 0 && dev < 64, "mrg_residual_layernorm_param_reduce: device %d", dev);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long cap = 0;
  MRG_HIP(hipStreamGetCaptureInfo(stream, &st, &cap));
  if (st != hipStreamCaptureStatusActive) cap = 0;
  std::lock_guard<std::mutex> lk(g_tick_mu);
  if (!g_tick_base[dev]) MRG_HIP(hipGetSymbolAddress(&g_tick_base[dev], HIP_SYMBOL(g_resln_tickets)));
  int slot = -1;
  for (int i = 0; i < g_tick_used; ++i)
    if (g_tick_owner[i].dev == dev && g_tick_owner[i].s == stream && g_tick_owner[i].cap == cap) {
      slot = i;
      break;
    }
  if (slot < 0) {
    if (g_tick_used >= RESLN_TSLOTS) {
      *tick = nullptr;
      return 0;
    }
    slot = g_tick_used++;
    g_tick_owner[slot].dev = dev;
    g_tick_owner[slot].s = stream;
    g_tick_owner[slot].cap = cap;
  }
  *tick = static_cast<unsigned*>(g_tick_base[dev]) + slot * RESLN_MAXCB;
  return 0;
}

MRG_API int mrg_residual_layernorm_param_reduce(int rows, int E, float* workspace, float* dgamma,
                                                float* dbeta, int accumulate, hipStream_t stream) {
  if (rows == 0) return 0;
  MRG_REQUIRE(E >= 1 && E <= 1024 && dgamma && dbeta && workspace,
              "mrg_residual_layernorm_param_reduce: bad arguments (E=%d)", E);
  const int nblk = (rows + RESLN_RPB - 1) / RESLN_RPB;
  // row groups of ~32 partial rows (one round of loads per wave; distinct first rows), at most 64
  int R = nblk >= 64 ? ((nblk + 31) / 32 < 64 ? (nblk + 31) / 32 : 64) : 1;
  unsigned* tick = nullptr;
  if (R > 1 && resln_tickets(stream, &tick)) return 1;
  if (!tick) R = 1;   // ticket table full: one group per column block
  // the partials are consumed in place (each row group's sum overwrites its first row)
  resln_param_reduce_kernel<<<dim3((2 * E + 63) / 64, R), 256, 0, stream>>>(workspace, nblk, E, dgamma, dbeta,
                                                                            accumulate, R, tick);
  return check_launch("resln_param_reduce_kernel");
}

static LossArgs make_loss_args(int B, int T, int F, const float* y, long y_bstride, const float* t,
                               int type, float delta, float beta, int mask_padding, int delta_start,
                               float dscale) {
  LossArgs a;
  a.y = y; a.ys = y_bstride; a.t = t; a.B = B; a.T = T; a.F = F; a.type = type;
  a.delta = delta; a.beta = beta; a.mask_padding = mask_padding; a.delta_start = delta_start;
  a.dscale = dscale;
  return a;
}

static int loss_blocks(long n) {
  long b = (n + 255) / 256;
  return (int)(b < 1024 ? (b < 1 ? 1 : b) : 1024);
}

MRG_API size_t mrg_loss_workspace_bytes(int B, int T, int F) {
  return (size_t)loss_blocks((long)B * T * F) * sizeof(float);
}

MRG_API int mrg_masked_loss_fwd(int B, int T, int F, const float* y, long y_bstride, const float* target,
                                int type, float delta, float beta, int mask_padding, int delta_start,
                                float dscale, float* loss_out, float* workspace, hipStream_t stream) {
  MRG_REQUIRE(type >= 0 && type <= 3, "mrg_masked_loss_fwd: bad loss type %d", type);
  long n = (long)B * T * F;
  if (n == 0) return 0;
  LossArgs a = make_loss_args(B, T, F, y, y_bstride, target, type, delta, beta, mask_padding,
                              delta_start, dscale);
  int nb = loss_blocks(n);
  loss_fwd_partial_kernel<<<nb, 256, 0, stream>>>(a, workspace);
  if (check_launch("loss_fwd_partial_kernel")) return 1;
  loss_fwd_final_kernel<<<1, 64, 0, stream>>>(workspace, nb, 1.0f / (float)n, loss_out);
  return check_launch("loss_fwd_final_kernel");
}

MRG_API int mrg_masked_loss_bwd(int B, int T, int F, const float* y, long y_bstride, const float* target,
                                int type, float delta, float beta, int mask_padding, int delta_start,
                                float dscale, const float* grad_out, float* dy, hipStream_t stream) {
  long n = (long)B * T * F;
  if (n == 0) return 0;
  LossArgs a = make_loss_args(B, T, F, y, y_bstride, target, type, delta, beta, mask_padding,
                              delta_start, dscale);
  loss_bwd_kernel<<<loss_blocks(n), 256, 0, stream>>>(a, grad_out, 1.0f / (float)n, dy);
  return check_launch("loss_bwd_kernel");
}

static int bcast_setup(BcastArgs& a, int B, int T, int F, const float* y, long y_bstride, const float* target,
                       const float* ms, long ms_bs, long ms_ts, int Tm, int type, float delta, float beta,
                       int t_start, float dscale, float* workspace, hipStream_t stream) {
  MRG_REQUIRE(type >= 0 && type <= 3, "mrg_broadcast_loss: bad loss type %d", type);
  MRG_REQUIRE(B >= 0 && T >= 0 && F >= 1 && Tm >= 0 && ms && workspace,
              "mrg_broadcast_loss: bad arguments (B=%d T=%d F=%d Tm=%d)", B, T, F, Tm);
  a.y = y; a.ys = y_bstride; a.t = target; a.counts = workspace; a.B = B; a.T = T; a.F = F; a.Tm = Tm;
  a.type = type; a.delta = delta; a.beta = beta; a.t_start = t_start; a.dscale = dscale;
  if (B * F == 0) return 0;
  bcast_count_kernel<<<(B * F + 255) / 256, 256, 0, stream>>>(ms, ms_bs, ms_ts, B, Tm, F, workspace);
  return check_launch("bcast_count_kernel");
}

MRG_API size_t mrg_broadcast_loss_workspace_bytes(int B, int T, int F) {
  return ((size_t)B * F + (size_t)loss_blocks((long)B * T * F)) * sizeof(float);
}

MRG_API int mrg_broadcast_loss_fwd(int B, int T, int F, const float* y, long y_bstride, const float* target,
                                   const float* ms, long ms_bs, long ms_ts, int Tm, int type, float delta,
                                   float beta, int t_start, float dscale, float* loss_out, float* workspace,
                                   hipStream_t stream) {
  BcastArgs a;
  if (bcast_setup(a, B, T, F, y, y_bstride, target, ms, ms_bs, ms_ts, Tm, type, delta, beta, t_start, dscale,
                  workspace, stream))
    return 1;
  const long n = (long)B * T * F;
  const double nn = (double)n * (double)Tm;
  if (n == 0 || Tm == 0) {
    (void)hipMemsetAsync(loss_out, 0xff, sizeof(float), stream);  // mean over an empty tensor: NaN, as torch
    return check_launch("mrg_broadcast_loss_fwd");
  }
  float* part = workspace + (size_t)B * F;
  const int nb = loss_blocks(n);
  bcast_loss_partial_kernel<<<nb, 256, 0, stream>>>(a, part);
  if (check_launch("bcast_loss_partial_kernel")) return 1;
  loss_fwd_final_kernel<<<1, 64, 0, stream>>>(part, nb, (float)(1.0 / nn), loss_out);
  return check_launch("loss_fwd_final_kernel");
}

MRG_API int mrg_broadcast_loss_bwd(int B, int T, int F, const float* y, long y_bstride, const float* target,
                                   const float* ms, long ms_bs, long ms_ts, int Tm, int type, float delta,
                                   float beta, int t_start, float dscale, const float* grad_out, float* dy,
                                   float* workspace, hipStream_t stream) {
  BcastArgs a;
  if (bcast_setup(a, B, T, F, y, y_bstride, target, ms, ms_bs, ms_ts, Tm, type, delta, beta, t_start, dscale,
                  workspace, stream))
    return 1;
  const long n = (long)B * T * F;
  if (n == 0 || Tm == 0) return 0;
  bcast_loss_bwd_kernel<<<loss_blocks(n), 256, 0, stream>>>(a, grad_out, (float)(1.0 / ((double)n * Tm)), dy);
  return check_launch("bcast_loss_bwd_kernel");
}

// step_lr: device float[2] = {completed steps, lr}; incremented after the update.
// err: nullable device int; non-zero skips the update (see adamw_kernel).
MRG_API int mrg_adamw_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, long n,
                           float* step_lr, float weight_decay, float beta1, float beta2, float eps,
                           const int* err, hipStream_t stream) {
  if (n > 0) {
    long nb = (n + 255) / 256;
    int grid = (int)(nb < 4096 ? nb : 4096);
    adamw_kernel<<<grid, 256, 0, stream>>>(params, grads, exp_avg, exp_avg_sq, n, step_lr, weight_decay,
                                           beta1, beta2, eps, err);
    if (check_launch("adamw_kernel")) return 1;
  }
  adamw_step_inc_kernel<<<1, 1, 0, stream>>>(step_lr, err);
  return check_launch("adamw_step_inc_kernel");
}

// ------------------------------------------------------------------ padding helpers
// flags[b][t] = (x[b][t][0] == value): the padding test of gen_attention_mask
// (multi_modal_metaformer.py:67-73, `x[:, :, 0] == -100`), uint8; x rows at b * bs + t * ts.
namespace mrg {
__global__ __launch_bounds__(256) void padding_flags_kernel(int B, int T, const float* __restrict__ x, long bs,
                                                            long ts, float value, unsigned char* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * T) return;
  const long b = i / T, t = i - b * T;
  out[i] = x[b * bs + t * ts] == value ? 1 : 0;
}

// y = x * (x != value) elementwise: training_step's zeroing of padded motion_self frames
// (lstmformer.py:365-366, `batch[2] * (batch[2] != -100)`), float4 where aligned
__global__ __launch_bounds__(256) void zero_padding_kernel(long n, const float* __restrict__ x, float value,
                                                           float* __restrict__ y) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (4 * i + 3 < n) {
    float4 v = reinterpret_cast<const float4*>(x)[i];
    v.x = v.x != value ? v.x : 0.0f; v.y = v.y != value ? v.y : 0.0f;
    v.z = v.z != value ? v.z : 0.0f; v.w = v.w != value ? v.w : 0.0f;
    reinterpret_cast<float4*>(y)[i] = v;
  } else {
    for (long j = 4 * i; j < n; ++j) y[j] = x[j] != value ? x[j] : 0.0f;
  }
}
}  // namespace mrg

MRG_API int mrg_padding_flags(int B, int T, const float* x, long bs, long ts, float value, unsigned char* out,
                              hipStream_t stream) {
  if (B == 0 || T == 0) return 0;
  const long n = (long)B * T;
  padding_flags_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(B, T, x, bs, ts, value, out);
  return check_launch("padding_flags_kernel");
}

namespace mrg {

// bytes of zeros at p (16-B stores over the aligned body, byte stores at the ends): the step's
// buffer clears (gradient buffer, hand-off rings, loss-gradient lead frames) as a library kernel
__global__ __launch_bounds__(256) void fill_zero_kernel(unsigned char* p, long head, long nv, long bytes) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride)
    reinterpret_cast<float4*>(p + head)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  const long tail0 = head + nv * 16;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < head) p[t] = 0;
  if (t < bytes - tail0) p[tail0 + t] = 0;
}

// dst[j][i][:] = src[i][j][:] for an [n0][n1][E] tensor (E % 4 == 0, 16-B aligned): float4 rows,
// one thread per 16 B, rows in destination order (coalesced stores, 1-KB row reads)
__global__ __launch_bounds__(256) void swap01_kernel(const float* __restrict__ src, float* __restrict__ dst, int n0,
                                                     int n1, int E4, float beta) {
  const long total = (long)n0 * n1 * E4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const long row = e / E4;
    const int c = (int)(e - row * E4);
    const int j = (int)(row / n0), i = (int)(row - (long)j * n0);   // dst row (j, i)
    const float4 v = reinterpret_cast<const float4*>(src)[((long)i * n1 + j) * E4 + c];
    float4* d = reinterpret_cast<float4*>(dst) + e;
    if (beta != 0.0f) {
      const float4 o = *d;
      *d = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
    } else {
      *d = v;
    }
  }
}

}  // namespace mrg

// [n0][n1][E] -> [n1][n0][E] (batch-major <-> time-major activations at the block wavefront's
// boundaries); beta = 1 adds into dst (a gradient arriving from two consumers).
MRG_API int mrg_swap01(int n0, int n1, int E, const float* src, float* dst, float beta, hipStream_t stream) {
  MRG_REQUIRE(n0 >= 0 && n1 >= 0 && E > 0 && E % 4 == 0 && ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) &&
                  (beta == 0.0f || beta == 1.0f),
              "mrg_swap01: E %% 4 == 0, 16-B aligned buffers, beta 0 or 1 required");
  const long total = (long)n0 * n1 * (E / 4);
  if (total == 0) return 0;
  long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  klaunch(mrg::swap01_kernel, (unsigned)blocks, 256, 0, stream, src, dst, n0, n1, E / 4, beta);
  return check_launch("swap01_kernel");
}

MRG_API int mrg_fill_zero(void* p, long bytes, hipStream_t stream) {
  MRG_REQUIRE(bytes >= 0 && (bytes == 0 || p), "mrg_fill_zero: bad arguments");
  if (bytes == 0) return 0;
  unsigned char* b = reinterpret_cast<unsigned char*>(p);
  long head = (16 - (long)((uintptr_t)b & 15)) & 15;
  if (head > bytes) head = bytes;
  const long nv = (bytes - head) / 16;
  long blocks = (nv + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  klaunch(mrg::fill_zero_kernel, (unsigned)blocks, 256, 0, stream, b, head, nv, bytes);
  return check_launch("fill_zero_kernel");
}

MRG_API int mrg_zero_padding(long n, const float* x, float value, float* y, hipStream_t stream) {
  if (n == 0) return 0;
  MRG_REQUIRE((((uintptr_t)x | (uintptr_t)y) & 15) == 0, "mrg_zero_padding: 16-byte aligned buffers required");
  const long nv = (n + 3) / 4;
  zero_padding_kernel<<<(unsigned)((nv + 255) / 256), 256, 0, stream>>>(n, x, value, y);
  return check_launch("zero_padding_kernel");
}
