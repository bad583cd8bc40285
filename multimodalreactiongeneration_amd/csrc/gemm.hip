// fp32 GEMM on the gfx950 f32-input matrix cores (v_mfma_f32_32x32x2_f32).
//
//   C[m, n] = epi( alpha * sum_k A(m, k) * B(k, n) + beta * C[m, n] + bias[n] )
//
// A(m, k) is A[row m][col k] (transA = 0) or A[row k][col m] (transA = 1); B
// likewise.  Rows go through a RowMap (see mrg_common.h), so the same kernel
// serves nn.Linear forward (X W^T), input-grad (dY W), weight-grad (dY^T X,
// reduction over B*T rows, split-K into fp32 slabs then an ordered reduce:
// deterministic), the LSTM input projection and the LSTM recurrent weight grad
// sum_t dG_t^T h_{t-1} (time-shifted rows, no copy).
//
// f32 MFMA is exact fp32 (a k-ordered fmaf chain), which keeps the 1e-4
// relative parity budget intact.  Tile: BM x BN x 16, 4 waves as 2 x 2, each
// wave (BM/2) x (BN/2) in 32x32 MFMA sub-tiles; A/B staged k-major in LDS so
// the per-lane fragment reads (lane -> row l&31, k-pair l>>5) are
// bank-conflict free; global loads for the next K tile are issued before the
// MFMAs of the current one (register prefetch).
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
  int epi;  // 0 none, 1 relu, 2 multiply by (aux > 0)
  const float* aux;
  long ldaux;
  float* ws;  // split-K slabs [splits][M][N] (nullptr when splits == 1)
  int kchunk;
};

static constexpr int BK = 16;
static constexpr int NT = 256;

__device__ __forceinline__ float apply_epi(const GemmArgs& a, float v, int m, int n) {
  v *= a.alpha;
  if (a.beta != 0.0f) v += a.beta * a.C[(long)m * a.ldc + n];
  if (a.bias) v += a.bias[n];
  if (a.epi == 1) v = fmaxf(v, 0.0f);
  else if (a.epi == 2) v = (a.aux[(long)m * a.ldaux + n] > 0.0f) ? v : 0.0f;
  return v;
}

template <int BM, int BN>
__global__ __launch_bounds__(NT) void gemm_f32_kernel(GemmArgs a) {
  constexpr int PAD = 1;
  constexpr int LA = BM * BK / NT;  // A elements per thread per tile
  constexpr int LB = BN * BK / NT;
  constexpr int TM = BM / 64, TN = BN / 64;
  __shared__ float As[BK][BM + PAD];
  __shared__ float Bs[BK][BN + PAD];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int m0 = blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;
  const int kbeg = blockIdx.z * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);

  float ra[LA], rb[LB];

  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      int e = tid + i * NT;
      int m, k;
      if (a.transA) { m = e % BM; k = e / BM; } else { m = e / BK; k = e % BK; }
      int gm = m0 + m, gk = k0 + k;
      float v = 0.0f;
      if (gm < a.M && gk < kend) {
        v = a.transA ? a.A[a.amap.off(gk) + gm] : a.A[a.amap.off(gm) + gk];
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      int e = tid + i * NT;
      int n, k;
      if (a.transB) { k = e % BK; n = e / BK; } else { n = e % BN; k = e / BN; }
      int gn = n0 + n, gk = k0 + k;
      float v = 0.0f;
      if (gn < a.N && gk < kend) {
        v = a.transB ? a.B[a.bmap.off(gn) + gk] : a.B[a.bmap.off(gk) + gn];
      }
      rb[i] = v;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      int e = tid + i * NT;
      int m, k;
      if (a.transA) { m = e % BM; k = e / BM; } else { m = e / BK; k = e % BK; }
      As[k][m] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      int e = tid + i * NT;
      int n, k;
      if (a.transB) { k = e % BK; n = e / BK; } else { n = e % BN; k = e / BN; }
      Bs[k][n] = rb[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  const int wm = (wave >> 1) * (BM / 2);
  const int wn = (wave & 1) * (BN / 2);
  const int lr = lane & 31, lk = lane >> 5;

  if (kbeg < kend) load_tile(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    store_tile();
    __syncthreads();
    if (k0 + BK < kend) load_tile(k0 + BK);
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      float fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = As[2 * kk + lk][wm + i * 32 + lr];
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = Bs[2 * kk + lk][wn + j * 32 + lr];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // epilogue: C/D map of the 32x32 f32 MFMA: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int m = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        int n = n0 + wn + j * 32 + lr;
        if (m < a.M && n < a.N) {
          if (a.ws) a.ws[((long)blockIdx.z * a.M + m) * a.N + n] = acc[i][j][r];
          else a.C[(long)m * a.ldc + n] = apply_epi(a, acc[i][j][r], m, n);
        }
      }
}

__global__ void splitk_reduce_kernel(GemmArgs a, int splits) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)a.M * a.N;
  if (idx >= total) return;
  int m = idx / a.N, n = idx % a.N;
  float s = 0.0f;
  for (int z = 0; z < splits; ++z) s += a.ws[(long)z * total + idx];
  a.C[(long)m * a.ldc + n] = apply_epi(a, s, m, n);
}

// column sums: part[s][n] = sum over rows [s*rows_per, ...) of X(row, n)
__global__ void colsum_partial_kernel(const float* X, RowMap map, int rows, int N,
                                      int rows_per, float* part) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  int s = blockIdx.y;
  if (n >= N) return;
  int r0 = s * rows_per, r1 = min(rows, r0 + rows_per);
  float acc = 0.0f;
  for (int r = r0; r < r1; ++r) acc += X[map.off(r) + n];
  part[(long)s * N + n] = acc;
}

__global__ void colsum_final_kernel(const float* part, int S, int N, float beta, float* out,
                                    float* out2) {
  int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float acc = 0.0f;
  for (int s = 0; s < S; ++s) acc += part[(long)s * N + n];
  float v = (beta != 0.0f ? beta * out[n] : 0.0f) + acc;
  out[n] = v;
  if (out2) out2[n] = (beta != 0.0f ? beta * out2[n] : 0.0f) + acc;
}

}  // namespace mrg

using namespace mrg;

MRG_API size_t mrg_gemm_workspace_bytes(int M, int N, int splits) {
  return splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
}

MRG_API int mrg_gemm_f32(int M, int N, int K, float alpha,
                         const float* A, int transA, long lda, long lda_hi, int a_rdiv,
                         const float* B, int transB, long ldb, long ldb_hi, int b_rdiv,
                         float beta, float* C, long ldc, const float* bias, int epilogue,
                         const float* aux, long ldaux, float* workspace, int splits,
                         hipStream_t stream) {
  MRG_REQUIRE(M >= 0 && N >= 0 && K >= 0, "mrg_gemm_f32: negative size");
  MRG_REQUIRE(epilogue >= 0 && epilogue <= 2, "mrg_gemm_f32: bad epilogue %d", epilogue);
  MRG_REQUIRE(epilogue != 2 || aux, "mrg_gemm_f32: epilogue 2 needs aux");
  if (M == 0 || N == 0) return 0;
  if (splits < 1) splits = 1;
  MRG_REQUIRE(splits == 1 || workspace, "mrg_gemm_f32: split-K needs workspace");
  GemmArgs a;
  a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta;
  a.A = A; a.amap = RowMap{lda, lda_hi, a_rdiv}; a.transA = transA;
  a.B = B; a.bmap = RowMap{ldb, ldb_hi, b_rdiv}; a.transB = transB;
  a.C = C; a.ldc = ldc; a.bias = bias; a.epi = epilogue; a.aux = aux; a.ldaux = ldaux;
  int kc = (K + splits - 1) / splits;
  kc = ((kc + BK - 1) / BK) * BK;
  if (kc == 0) kc = BK;
  splits = (K + kc - 1) / kc;
  if (splits < 1) splits = 1;
  a.kchunk = kc;
  a.ws = splits > 1 ? workspace : nullptr;
  const bool bigM = M >= 2048, bigN = N > 64;
  dim3 block(NT);
  if (bigM && bigN) {
    dim3 grid((N + 127) / 128, (M + 127) / 128, splits);
    gemm_f32_kernel<128, 128><<<grid, block, 0, stream>>>(a);
  } else if (bigM) {
    dim3 grid((N + 63) / 64, (M + 127) / 128, splits);
    gemm_f32_kernel<128, 64><<<grid, block, 0, stream>>>(a);
  } else {
    dim3 grid((N + 63) / 64, (M + 63) / 64, splits);
    gemm_f32_kernel<64, 64><<<grid, block, 0, stream>>>(a);
  }
  if (check_launch("gemm_f32_kernel")) return 1;
  if (splits > 1) {
    long total = (long)M * N;
    splitk_reduce_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(a, splits);
    if (check_launch("splitk_reduce_kernel")) return 1;
  }
  return 0;
}

MRG_API size_t mrg_colsum_workspace_bytes(int rows, int N) {
  int S = rows >= 4096 ? 64 : (rows >= 256 ? 16 : 1);
  return (size_t)S * N * sizeof(float);
}

// out[n] = beta*out[n] + sum_rows X(row, n)   (bias gradients; out2 optional mirror for b_hh)
MRG_API int mrg_colsum_f32(int rows, int N, const float* X, long ld, long ld_hi, int rdiv,
                           float beta, float* out, float* out2, float* workspace,
                           hipStream_t stream) {
  if (N == 0) return 0;
  int S = rows >= 4096 ? 64 : (rows >= 256 ? 16 : 1);
  int rows_per = (rows + S - 1) / S;
  if (rows_per == 0) rows_per = 1;
  dim3 grid((N + 255) / 256, S);
  colsum_partial_kernel<<<grid, 256, 0, stream>>>(X, RowMap{ld, ld_hi, rdiv}, rows, N, rows_per,
                                                  workspace);
  if (check_launch("colsum_partial_kernel")) return 1;
  colsum_final_kernel<<<(N + 255) / 256, 256, 0, stream>>>(workspace, S, N, beta, out, out2);
  return check_launch("colsum_final_kernel");
}
