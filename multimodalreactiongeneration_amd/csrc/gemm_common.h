// Shared definitions of the GEMM kernels (gemm.hip, gemm_glds.hip): argument block, epilogue,
// fp32 -> three bf16 planes split of the x6 arithmetic.
#pragma once
#include "mrg_common.h"

namespace mrg {

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct GemmArgs {
  int M, N, K;
  float alpha, beta;
  const float* A;
  RowMap amap;
  int transA;
  const float* B;
  RowMap bmap;
  int transB;
  float* C;
  long ldc;
  const float* bias;
  int epi;  // 0 none, 1 relu, 2 multiply by (aux > 0), 3 add aux (residual gradient)
  const float* aux;
  long ldaux;
  float* ws;  // split-K slabs [splits][M][N] (nullptr when splits == 1)
  int kchunk;
  int tiles_n, tiles_mn, ntiles;  // output tiles (x splits), walked by a persistent grid
  int nsplit;                     // K slices per tile (ntiles / tiles_mn)
  // in-launch split-K combine (x6 path, small outputs): per-tile tickets, zero between launches;
  // null -> the slabs are reduced by splitk_reduce*_kernel
  unsigned* cnt;
  int vec;                        // C / bias / aux / slab rows 16-B aligned: vector epilogue
  // fused row sums of op(A) (bias gradients of a weight-gradient GEMM, TA = 1, x6 path):
  // per-(split, m) partials in asum [splits][M], reduced in a fixed order into
  // asum_out[m] = asum_beta * asum_out[m] + sum (and asum_out2, nullable)
  float* asum;
  float* asum_out;
  float* asum_out2;
  float asum_beta;
  // few-row kernel: byte extent of A and B from their base pointers (buffer-load range checks)
  int a_bytes, b_bytes;
};

#ifndef MRG_GEMM_COUNTERS
#define MRG_GEMM_COUNTERS 4096  // tickets the caller provides (include/mrg.h)
#endif

static constexpr int BK = 32;  // K tile (64 measured no faster here: 2 blocks/CU instead of 3)
static constexpr int NT = 256;

__device__ __forceinline__ float apply_epi(const GemmArgs& a, float v, int m, int n) {
  v *= a.alpha;
  if (a.beta != 0.0f) v += a.beta * a.C[(long)m * a.ldc + n];
  if (a.bias) v += a.bias[n];
  if (a.epi == 1) v = fmaxf(v, 0.0f);
  else if (a.epi == 2) v = (a.aux[(long)m * a.ldaux + n] > 0.0f) ? v : 0.0f;
  else if (a.epi == 3) v += a.aux[(long)m * a.ldaux + n];
  return v;
}

// C[m, n..n+3] (or the split-K slab row) from four accumulators: one 16-B access per operand when
// the rows are 16-B aligned (a.vec), element-wise at the N edge or for unaligned operands.
__device__ __forceinline__ void store4(const GemmArgs& a, int z, int m, int n, float4 v) {
  if (a.ws) {
    float* p = a.ws + ((long)z * a.M + m) * a.N + n;
    if (a.vec && n + 3 < a.N) { *reinterpret_cast<float4*>(p) = v; return; }
    const float e[4] = {v.x, v.y, v.z, v.w};
    for (int q = 0; q < 4 && n + q < a.N; ++q) p[q] = e[q];
    return;
  }
  if (a.vec && n + 3 < a.N) {
    float* pc = a.C + (long)m * a.ldc + n;
    float4 o = make_float4(v.x * a.alpha, v.y * a.alpha, v.z * a.alpha, v.w * a.alpha);
    if (a.beta != 0.0f) {
      const float4 c = *reinterpret_cast<const float4*>(pc);
      o.x += a.beta * c.x; o.y += a.beta * c.y; o.z += a.beta * c.z; o.w += a.beta * c.w;
    }
    if (a.bias) {
      const float4 b = *reinterpret_cast<const float4*>(a.bias + n);
      o.x += b.x; o.y += b.y; o.z += b.z; o.w += b.w;
    }
    if (a.epi == 1) {
      o.x = fmaxf(o.x, 0.0f); o.y = fmaxf(o.y, 0.0f); o.z = fmaxf(o.z, 0.0f); o.w = fmaxf(o.w, 0.0f);
    } else if (a.epi == 2) {
      const float4 x = *reinterpret_cast<const float4*>(a.aux + (long)m * a.ldaux + n);
      o.x = x.x > 0.0f ? o.x : 0.0f; o.y = x.y > 0.0f ? o.y : 0.0f;
      o.z = x.z > 0.0f ? o.z : 0.0f; o.w = x.w > 0.0f ? o.w : 0.0f;
    } else if (a.epi == 3) {
      const float4 x = *reinterpret_cast<const float4*>(a.aux + (long)m * a.ldaux + n);
      o.x += x.x; o.y += x.y; o.z += x.z; o.w += x.w;
    }
    *reinterpret_cast<float4*>(pc) = o;
    return;
  }
  const float e[4] = {v.x, v.y, v.z, v.w};
  for (int q = 0; q < 4 && n + q < a.N; ++q) a.C[(long)m * a.ldc + n + q] = apply_epi(a, e[q], m, n + q);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// two floats -> packed bf16 pair (RNE), one v_cvt_pk_bf16_f32
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  const f32x2 v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
}

// two values -> three planes of 2 bf16: 3 cvt_pk + 2 x (and, shift, packed sub) per pair
__device__ __forceinline__ void split2(float a, float b, unsigned& p0, unsigned& p1, unsigned& p2) {
  p0 = pk_bf16(a, b);
  a -= __uint_as_float(p0 << 16);
  b -= __uint_as_float(p0 & 0xffff0000u);
  p1 = pk_bf16(a, b);
  a -= __uint_as_float(p1 << 16);
  b -= __uint_as_float(p1 & 0xffff0000u);
  p2 = pk_bf16(a, b);
}

// four consecutive-k values -> three planes of 4 bf16 (8 B each)
__device__ __forceinline__ void split4(float v0, float v1, float v2, float v3, uint2& p0, uint2& p1, uint2& p2) {
  split2(v0, v1, p0.x, p1.x, p2.x);
  split2(v2, v3, p0.y, p1.y, p2.y);
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Same-shape products batched into one launch (mrg_gemm_x6g_batched): per problem the operand,
// output, bias and aux pointers; everything else (shape, strides, epilogue) is GemmArgs'.
static constexpr int MRG_GB_MAX = 16;
struct GemmBatch {
  int n;  // 0 = not batched
  const float* A[MRG_GB_MAX];
  const float* B[MRG_GB_MAX];
  float* C[MRG_GB_MAX];
  const float* bias[MRG_GB_MAX];
  const float* aux[MRG_GB_MAX];
};

// LDS-DMA pipelined x6 kernel for k-contiguous products (gemm_glds.hip): ring depth ns, tile
// bm x bn (64 | 128 each); grid = one workgroup per output tile (x problems when batched);
// planes 3 = x6 split (fp32-class), 1 = bf16 operands (precision "bf16")
void launch_x6g(GemmArgs a, int ns, int bm, int bn, hipStream_t s, int planes = 3, const GemmBatch* gb = nullptr);
// its weight-gradient form (transA = 1, transB = 0, K % 32 == 0, M and N multiples of 4): split-K
// slabs in a.ws (splits > 1) and the fused row sums of A in a.asum, as gemm_x6_kernel leaves them
// max_grid > 0: at most that many workgroups (a multiple of 8), walking the items
void launch_x6g_wgrad(GemmArgs a, int splits, int bm, int bn, hipStream_t s, int planes = 3, int max_grid = 0);


// row-owning x6 kernel on pre-split B planes (gemm_wide.hip): 64-row tiles, bn in {64, 128, 256},
// ring depth ns in {2, 3}
void launch_x6w(GemmArgs a, int bn, int ns, long bplane, hipStream_t s, const GemmBatch* gb = nullptr);
// B-resident form (gemm_wide.hip) for K in {128, 256}: one workgroup of `waves` waves per CU; returns -1
// when K is not supported

static constexpr int MRG_TP_MAX = 32;
struct TransposeBatch {
  int n;
  const float* src[MRG_TP_MAX];
  float* dst[MRG_TP_MAX];
  int rows[MRG_TP_MAX], cols[MRG_TP_MAX];
  int first[MRG_TP_MAX + 1];  // first block of each matrix
};
__global__ void transpose_batched_kernel(TransposeBatch tb);

}  // namespace mrg
