// Shared pieces of the persistent frame loops (gen.hip: lstmformer generation; ssd_loop.hip: the
// scheduled-sampling decode of lstm_with_sampling): 256-wide rows held 4 values per lane, the
// LayerNorm on them, exact-f32 16 x 16 MFMA tiles of 8 batch rows, and the {tag, value} granule
// gathers through which the members of a row group hand each stage's output to each other.
#pragma once
#include "lstm_common.h"

namespace mrg {

typedef float gv4 __attribute__((ext_vector_type(4)));
static constexpr int GE = 256;   // model width
static constexpr int GHB = 64;   // FeedForward bottleneck

// whole-wave sum: DPP within each 16-lane row (no LDS traffic), then the four row sums read out
__device__ __forceinline__ float gen_wave_sum(float v) {
  // (readlane moves 32-bit integers: the float travels as its bit pattern)
  const int u = __float_as_int(group_sum<16>(v));
  return (__int_as_float(__builtin_amdgcn_readlane(u, 0)) + __int_as_float(__builtin_amdgcn_readlane(u, 16))) +
         (__int_as_float(__builtin_amdgcn_readlane(u, 32)) + __int_as_float(__builtin_amdgcn_readlane(u, 48)));
}

// LayerNorm of a 256-wide row held as 4 consecutive values per lane, two-pass (torch.layer_norm:
// mean, then the mean of squared deviations, biased), eps inside the root; gg / bb: the lane's four
// gamma / beta values (loaded at kernel start, so their latency hides under the activation loads)
__device__ __forceinline__ float4 gen_ln(float4 v, float4 gg, float4 bb, float eps) {
  const float mean = gen_wave_sum((v.x + v.y) + (v.z + v.w)) * (1.0f / GE);
  const float dx = v.x - mean, dy = v.y - mean, dz = v.z - mean, dw = v.w - mean;
  const float var = gen_wave_sum((dx * dx + dy * dy) + (dz * dz + dw * dw)) * (1.0f / GE);
  const float rs = rsqrtf(var + eps);
  return make_float4(fmaf(dx * rs, gg.x, bb.x), fmaf(dy * rs, gg.y, bb.y), fmaf(dz * rs, gg.z, bb.z),
                     fmaf(dw * rs, gg.w, bb.w));
}

__device__ __forceinline__ float4 gen_ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 gen_add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 gen_zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

static constexpr int GL_ROWS = 8;     // rows per group (MFMA rows 8..15 are zero)
static constexpr int GL_MEM = 16;     // workgroups per group

// poll N granules per thread of `width`-wide rows: thread column c = tid + 256 q, rows 0..7; rows at
// or past B read a valid row's slot and are zeroed
// (sdead: the workgroup's shared flag, so after one timed-out poll every thread stops polling at its
// next gather and the launch drains within a frame)
template <int W>
__device__ __forceinline__ void gl_gather(unsigned long long* buf, int r0, int B, unsigned tag, float* dst, int ldd,
                                          int* err, bool& dead, int* sdead) {
  constexpr int N = GL_ROWS * W / 256;
  if (*sdead) dead = true;
  int idx[N];
  float v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int row = i / (W / 256), col = threadIdx.x + 256 * (i % (W / 256));
    idx[i] = min(r0 + row, B - 1) * W + col;
  }
  get_granules_idx<N>(buf, idx, tag, v, err, dead);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int row = i / (W / 256), col = threadIdx.x + 256 * (i % (W / 256));
    dst[row * ldd + col] = r0 + row < B ? v[i] : 0.0f;
  }
  if (dead) *sdead = 1;
}

// A wave's weight fragments of one 16-column tile over its k-quarter (K / 64 float4; with K = 4 E a
// wave takes the whole E-wide k range of its own tile).  Issued at the start of a stage, before the
// member polls its inputs, so the weights' memory latency hides under the hand-off wait.
template <int K>
struct GlW {
  float4 v[K / 64];
};
template <int K>
__device__ __forceinline__ void gl_wload(GlW<K>& f, const float* __restrict__ wrow, int wave, int lane) {
  const float* wr = wrow + wave * (K / 4) + 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < K / 64; ++i) f.v[i] = *reinterpret_cast<const float4*>(wr + 16 * i);
}
// acc = A[16][wave's k-quarter] x the fragments (lane l: row / column l & 15, k = 16 i + 4 (l >> 4) + j)
template <int K>
__device__ __forceinline__ gv4 gl_mma(const float* A, int lda, const GlW<K>& f, int lane, int wave) {
  const int m = lane & 15, q = lane >> 4;
  gv4 acc = gv4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < K / 64; ++i) {
    const float4 x = *reinterpret_cast<const float4*>(A + m * lda + wave * (K / 4) + 16 * i + 4 * q);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, f.v[i].x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, f.v[i].y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, f.v[i].z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, f.v[i].w, acc, 0, 0, 0);
  }
  return acc;
}

// a LayerNorm's gamma / beta for this lane's four columns
struct GlLn {
  float4 g, b;
};
__device__ __forceinline__ GlLn gl_lnp(const float* __restrict__ g, const float* __restrict__ b, int lane) {
  return GlLn{gen_ld4(g + 4 * lane), gen_ld4(b + 4 * lane)};
}
// LN(a[r] + b[r]) of one row (4 values per lane) into out (and out2 when given)
__device__ __forceinline__ void gl_ln_row(const float* a, const float* b, const GlLn& p, float eps, float* out,
                                          float* out2, int lane) {
  const float4 v = gen_ln(gen_add4(*reinterpret_cast<const float4*>(a + 4 * lane),
                                   *reinterpret_cast<const float4*>(b + 4 * lane)),
                          p.g, p.b, eps);
  *reinterpret_cast<float4*>(out + 4 * lane) = v;
  if (out2) *reinterpret_cast<float4*>(out2 + 4 * lane) = v;
}

// the four waves' partial tiles of tile q into red[.][q]
__device__ __forceinline__ void gl_park(float (*red)[4][16][17], int q, int wave, int lane, gv4 acc) {
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][q][4 * (lane >> 4) + i][lane & 15] = acc[i];
}
__device__ __forceinline__ float gl_sum(const float (*red)[4][16][17], int q, int m, int n) {
  return (red[0][q][m][n] + red[1][q][m][n]) + (red[2][q][m][n] + red[3][q][m][n]);
}

}  // namespace mrg
