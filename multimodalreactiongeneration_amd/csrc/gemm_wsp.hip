// Weight-gradient GEMM with warp specialization: C[m][n] = sum_k A[k][m] B[k][n] (dW = dY^T X over
// the B*T rows, the backward of nn.Linear / the LSTM input and recurrent products,
// mixer_block.py:63-74,237-252), fp32 through the x6 three-plane bf16 split.
//
// Round 3's LDS-DMA form (gemm_x6g_wgrad_kernel) runs each wave through the chain
//   8 k-strided ds_read_b32 per fragment -> split into three planes -> six MFMAs
// with one wave per SIMD, so the split's VALU work (about as many issue cycles as the MFMAs) and
// the LDS read latency serialise with the MFMAs (~2 us per 32-row k-tile and workgroup, VERDICT
// r03 weak #3); each fragment is also split by both waves that read it.
//
// Here a 512-thread workgroup holds two wave groups on every SIMD:
//   splitters (waves 4-7): global loads of the fp32 k-tile (two tiles in flight in registers),
//     one split per element (thread (x, kh) owns operand row x and the k-octets kh, kh + 2 of every
//     k-tile), three bf16 planes written to LDS in the x6 image (x6_off, conflict-free), and the
//     fused row sums of A (the bias gradient) in the round-3 summation order;
//   consumers (waves 0-3): each a 64 x 64 quarter of the 128 x 128 tile, fragments by ds_read_b128
//     from the planes, the six MFMAs per 32x32x16 block in the round-3 order.
// Plane buffers are double-buffered: while the consumers multiply k-tile kt the splitters fill
// k-tile kt + 1, one workgroup barrier per k-tile.  Every product and sum is taken in the order of
// gemm_x6g_wgrad_kernel, so the two kernels give bitwise the same gradients (tested).
#include "gemm_common.h"

namespace mrg {

namespace {

constexpr int WT = 512;                    // threads: 4 consumer + 4 splitter waves
constexpr int TBM = 128, TBN = 128;        // output tile
constexpr int PL = TBM * 64;               // bytes of one plane: 128 rows x 32 k x bf16
constexpr int PB = 6 * PL;                 // one plane buffer: A planes 0..2, B planes 0..2 (48 KB)

__device__ __forceinline__ int xo(int x, int c) {   // gemm.hip x6_off: the conflict-free plane image
  const int g = (x >> 2) & 3;
  return ((x >> 2) << 8) + (((x & 3) ^ g) << 6) + ((c ^ g) << 4);
}

typedef float f32x4w __attribute__((ext_vector_type(4)));
typedef unsigned u32x4w __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split8w(const float (&v)[8], u32x4w& p0, u32x4w& p1, u32x4w& p2) {
  unsigned a0, a1, a2, b0, b1, b2, c0, c1, c2, d0, d1, d2;
  split2(v[0], v[1], a0, a1, a2);
  split2(v[2], v[3], b0, b1, b2);
  split2(v[4], v[5], c0, c1, c2);
  split2(v[6], v[7], d0, d1, d2);
  p0 = u32x4w{a0, b0, c0, d0};
  p1 = u32x4w{a1, b1, c1, d1};
  p2 = u32x4w{a2, b2, c2, d2};
}

__device__ __forceinline__ f32x16 mfma6(const bf16x8 (&b)[3], const bf16x8 (&a)[3], f32x16 acc) {
  // the order of gemm_glds.hip mfma_planes<3>: small terms first; (B, A) operand order -> C^T per lane
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[2], a[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[1], a[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[0], a[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[1], a[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[0], a[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[0], a[0], acc, 0, 0, 0);
}

// One splitter thread's k-tile: two k-octets of operand row x of A and of B (16 values each).
struct Octets {
  float a[2][8], b[2][8];
};

__device__ __forceinline__ void load_tile(const GemmArgs& a, Octets& r, int kt0, int kh, int x, int m0, int n0) {
  const bool am = m0 + x < a.M, bn = n0 + x < a.N;
#pragma unroll
  for (int o = 0; o < 2; ++o) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kt0 + 8 * (kh + 2 * o) + j;
      r.a[o][j] = am ? a.A[a.amap.off(k) + m0 + x] : 0.0f;
      r.b[o][j] = bn ? a.B[a.bmap.off(k) + n0 + x] : 0.0f;
    }
  }
}

__device__ __forceinline__ void store_planes(unsigned char* buf, const Octets& r, int kh, int x) {
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const int off = xo(x, kh + 2 * o);
    u32x4w p0, p1, p2;
    split8w(r.a[o], p0, p1, p2);
    *reinterpret_cast<u32x4w*>(buf + 0 * PL + off) = p0;
    *reinterpret_cast<u32x4w*>(buf + 1 * PL + off) = p1;
    *reinterpret_cast<u32x4w*>(buf + 2 * PL + off) = p2;
    split8w(r.b[o], p0, p1, p2);
    *reinterpret_cast<u32x4w*>(buf + 3 * PL + off) = p0;
    *reinterpret_cast<u32x4w*>(buf + 4 * PL + off) = p1;
    *reinterpret_cast<u32x4w*>(buf + 5 * PL + off) = p2;
  }
}

__device__ __forceinline__ float octet_sum(const float (&v)[8]) {  // gemm_glds.hip's tree
  return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
}

}  // namespace

__global__ __launch_bounds__(WT, 1) void gemm_x6s_wgrad_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * PB];
  __shared__ float rsum[TBM];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const bool splitter = wave >= 4;
  const int total = a.ntiles, q8 = total >> 3, r8 = total & 7;
  for (int vb = blockIdx.x; vb < total; vb += gridDim.x) {
    const int xcd = vb & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (vb >> 3);
    const int z = t / a.tiles_mn, tr = t - z * a.tiles_mn;
    const int m0 = (tr / a.tiles_n) * TBM, n0 = (tr % a.tiles_n) * TBN;
    const int kbeg = z * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
    const int nk = (kend - kbeg) / 32;
    if (splitter) {
      const int s = tid - 256, x = s & 127, kh = s >> 7;
      const bool do_asum = a.asum && n0 == 0;
      float cs = 0.0f;
      Octets r0, r1;
      if (nk > 0) load_tile(a, r0, kbeg, kh, x, m0, n0);
      if (nk > 1) load_tile(a, r1, kbeg + 32, kh, x, m0, n0);
      if (nk > 0) {
        if (do_asum) { cs += octet_sum(r0.a[0]); cs += octet_sum(r0.a[1]); }
        store_planes(lds, r0, kh, x);
      }
      if (nk > 2) load_tile(a, r0, kbeg + 64, kh, x, m0, n0);
      __syncthreads();
      // k-tile kt + 1 into buffer (kt + 1) & 1 while the consumers multiply kt; two tiles in flight
      for (int kt = 0; kt < nk; kt += 2) {
        if (kt + 1 < nk) {
          if (do_asum) { cs += octet_sum(r1.a[0]); cs += octet_sum(r1.a[1]); }
          store_planes(lds + PB, r1, kh, x);
          if (kt + 3 < nk) load_tile(a, r1, kbeg + 32 * (kt + 3), kh, x, m0, n0);
        }
        __syncthreads();
        if (kt + 1 >= nk) break;
        if (kt + 2 < nk) {
          if (do_asum) { cs += octet_sum(r0.a[0]); cs += octet_sum(r0.a[1]); }
          store_planes(lds, r0, kh, x);
          if (kt + 4 < nk) load_tile(a, r0, kbeg + 32 * (kt + 4), kh, x, m0, n0);
        }
        __syncthreads();
      }
      // bias gradient partial: row x = (k-half 0 sum) + (k-half 1 sum), as lanes l and l + 32 combine
      if (do_asum && kh == 1) rsum[x] = cs;
      __syncthreads();
      if (do_asum && kh == 0 && m0 + x < a.M) a.asum[(long)z * a.M + m0 + x] = cs + rsum[x];
    } else {
      const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
      const int lr = lane & 31, lh = lane >> 5;
      f32x16 acc[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
      __syncthreads();
      for (int kt = 0; kt < nk; ++kt) {
        const unsigned char* buf = lds + (kt & 1) * PB;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 fa[2][3], fb[2][3];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int off = xo(wm + 32 * i + lr, 2 * s + lh);
#pragma unroll
            for (int p = 0; p < 3; ++p) fa[i][p] = *reinterpret_cast<const bf16x8*>(buf + p * PL + off);
          }
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int off = xo(wn + 32 * j + lr, 2 * s + lh);
#pragma unroll
            for (int p = 0; p < 3; ++p) fb[j][p] = *reinterpret_cast<const bf16x8*>(buf + (3 + p) * PL + off);
          }
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = mfma6(fb[j], fa[i], acc[i][j]);
        }
        __syncthreads();
      }
      __syncthreads();   // the splitters' row-sum exchange
      // epilogue (gemm_glds.hip's BN >= 128 form): each wave stages 32 rows of its quarter in LDS
      // (the plane buffers are free: every k-tile is consumed) and writes whole 256-B row runs
      constexpr int WC = 64, PITCH = WC + 4, C4 = WC / 4;
      float* stg = reinterpret_cast<float*>(lds) + wave * 32 * PITCH;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4)
            *reinterpret_cast<float4*>(stg + lr * PITCH + j * 32 + 8 * r4 + 4 * lh) =
                make_float4(acc[i][j][4 * r4], acc[i][j][4 * r4 + 1], acc[i][j][4 * r4 + 2], acc[i][j][4 * r4 + 3]);
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int it = 0; it < 32 * C4 / 64; ++it) {
          const int qq = lane + 64 * it, row = qq / C4, c4 = qq % C4;
          const float4 v = *reinterpret_cast<const float4*>(stg + row * PITCH + 4 * c4);
          const int m = m0 + wm + i * 32 + row;
          if (m < a.M) store4(a, z, m, n0 + wn + 4 * c4, v);
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();   // the staging area is the next item's plane buffer
  }
}

void launch_x6s_wgrad(GemmArgs a, int splits, hipStream_t s, int max_grid) {
  a.tiles_n = (a.N + TBN - 1) / TBN;
  a.tiles_mn = a.tiles_n * ((a.M + TBM - 1) / TBM);
  a.ntiles = a.tiles_mn * splits;
  a.nsplit = splits;
  unsigned grid = (unsigned)a.ntiles;
  if (max_grid > 0 && grid > (unsigned)max_grid) grid = (unsigned)max_grid & ~7u ? (unsigned)max_grid & ~7u : 8u;
  klaunch(gemm_x6s_wgrad_kernel, grid, WT, 0, s, a);
}

}  // namespace mrg
