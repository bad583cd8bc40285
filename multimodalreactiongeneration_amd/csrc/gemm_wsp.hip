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

// Rows past the edge load the last row (straight-line loads, no branches: the compiler then keeps
// every load of both tiles in flight); their products land in outputs that are never stored.
// MAPPED = 0: plain rows (off(k) = k ld); 1: two-level RowMaps (the time-shifted dW_hh operands),
// offsets stepped through the 8 k of an octet from one division, branch-free.
template <bool MAPPED>
__device__ __forceinline__ void octet_off(const RowMap& m, int k0, long (&off)[8]) {
  if constexpr (!MAPPED) {
#pragma unroll
    for (int j = 0; j < 8; ++j) off[j] = (long)(k0 + j) * m.ld_lo;
  } else {
    const int rd = m.rdiv > 0 ? m.rdiv : 0x7fffffff;
    int q = k0 / rd, r = k0 - q * rd;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      off[j] = (long)q * m.ld_hi + (long)r * m.ld_lo;
      const bool wrap = r + 1 == rd;
      r = wrap ? 0 : r + 1;
      q = wrap ? q + 1 : q;
    }
  }
}

template <bool MAPPED>
__device__ __forceinline__ void load_tile(const GemmArgs& a, Octets& r, int kt0, int kh, int x, int m0, int n0) {
  const float* pa = a.A + min(m0 + x, a.M - 1);
  const float* pb = a.B + min(n0 + x, a.N - 1);
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    const int k0 = kt0 + 8 * (kh + 2 * o);
    long oa[8], ob[8];
    octet_off<MAPPED>(a.amap, k0, oa);
    octet_off<MAPPED>(a.bmap, k0, ob);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      r.a[o][j] = pa[oa[j]];
      r.b[o][j] = pb[ob[j]];
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

// a workgroup barrier the compiler may not schedule work across (it otherwise hoists the next half's
// split above the barrier, which needs that half's loads: vmcnt(0) where vmcnt(4) would do)
__device__ __forceinline__ void fenced_sync() {
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ float octet_sum(const float (&v)[8]) {  // gemm_glds.hip's tree
  return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
}

}  // namespace

template <bool MAPPED>
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
    if (nk <= 0) continue;   // (uniform across the workgroup)
    if (splitter) {
      // branch-free k-tile pairs: loads past the last k-tile re-read it and stores past it fill the
      // buffer nobody reads that half, so the compiler keeps both tiles' loads in flight (counted
      // vmcnt waits instead of vmcnt(0) at every branch join)
      const int s = tid - 256, x = s & 127, kh = __builtin_amdgcn_readfirstlane(s >> 7);   // wave-uniform
      const bool do_asum = a.asum && n0 == 0;
      const int last = kbeg + 32 * (nk - 1);
      float cs = 0.0f;
      Octets r0, r1;
      load_tile<MAPPED>(a, r0, kbeg, kh, x, m0, n0);
      load_tile<MAPPED>(a, r1, min(kbeg + 32, last), kh, x, m0, n0);
      if (do_asum) { cs += octet_sum(r0.a[0]); cs += octet_sum(r0.a[1]); }
      store_planes(lds, r0, kh, x);
      load_tile<MAPPED>(a, r0, min(kbeg + 64, last), kh, x, m0, n0);
      fenced_sync();
      for (int kt = 0; kt < nk; kt += 2) {
        if (do_asum) {
          const float t0 = octet_sum(r1.a[0]), t1 = octet_sum(r1.a[1]);
          cs = kt + 1 < nk ? (cs + t0) + t1 : cs;
        }
        store_planes(lds + PB, r1, kh, x);
        load_tile<MAPPED>(a, r1, min(kbeg + 32 * (kt + 3), last), kh, x, m0, n0);
        fenced_sync();
        if (do_asum) {
          const float t0 = octet_sum(r0.a[0]), t1 = octet_sum(r0.a[1]);
          cs = kt + 2 < nk ? (cs + t0) + t1 : cs;
        }
        store_planes(lds, r0, kh, x);
        load_tile<MAPPED>(a, r0, min(kbeg + 32 * (kt + 4), last), kh, x, m0, n0);
        fenced_sync();
      }
      // bias gradient partial: row x = (k-half 0 sum) + (k-half 1 sum), as lanes l and l + 32 combine
      if (do_asum && kh == 1) rsum[x] = cs;
      fenced_sync();
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
      for (int kt = 0; kt < nk + (nk & 1); ++kt) {   // k-tile pairs, as the splitters
        if (kt < nk) {
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

// ----------------------------------------------------------------------------------------------
// The same specialization for the k-contiguous products C = A B^T (+ bias / epilogue): x W^T of
// nn.Linear / the LSTM input projection, and dY W through the transposed weight copies
// (mixer_block.py:63-74,237-252, for_sequential.py:42-51).  Splitter thread s owns the k-octet units
// u = s + 256 q of the (BM + BN) x 4 octets of a k-tile, 4 consecutive threads on one 128-B row
// piece (coalesced), loads two k-tiles ahead in registers; consumers are a 2 x 2 grid of
// (BM / 2) x (BN / 2) wave tiles, fragments and six-MFMA order of gemm_x6g_kernel (bitwise equal).
// One workgroup per output tile (grid = tiles x problems, problem-major like the batched form).
namespace {

template <int BM, int BN>
struct FwdUnits {
  static constexpr int U = (BM + BN) * 4 / 256;      // octet units per splitter thread per k-tile
  float v[U][8];
};

// the U operand rows' k-octet base pointers of splitter thread s (edge rows: the last row), once per tile
template <int BM, int BN>
__device__ __forceinline__ void fwd_rows(const GemmArgs& a, const float* (&rp)[FwdUnits<BM, BN>::U], int s, int m0,
                                         int n0) {
#pragma unroll
  for (int q = 0; q < FwdUnits<BM, BN>::U; ++q) {
    const int u = s + 256 * q, row = u >> 2, c = u & 3;
    const bool isa = row < BM;
    const int gr = isa ? min(m0 + row, a.M - 1) : min(n0 + row - BM, a.N - 1);
    rp[q] = (isa ? a.A + a.amap.off(gr) : a.B + a.bmap.off(gr)) + 8 * c;
  }
}

template <int BM, int BN>
__device__ __forceinline__ void fwd_load(const float* const (&rp)[FwdUnits<BM, BN>::U], FwdUnits<BM, BN>& r, int kt0) {
#pragma unroll
  for (int q = 0; q < FwdUnits<BM, BN>::U; ++q) {
    const float* p = rp[q] + kt0;
    const float4 x0 = *reinterpret_cast<const float4*>(p);
    const float4 x1 = *reinterpret_cast<const float4*>(p + 4);
    r.v[q][0] = x0.x; r.v[q][1] = x0.y; r.v[q][2] = x0.z; r.v[q][3] = x0.w;
    r.v[q][4] = x1.x; r.v[q][5] = x1.y; r.v[q][6] = x1.z; r.v[q][7] = x1.w;
  }
}

// plane buffer: A planes 0..2 ([BM][32 k] bf16 each) then B planes 0..2 ([BN][32 k])
template <int BM, int BN>
__device__ __forceinline__ void fwd_store(unsigned char* buf, const FwdUnits<BM, BN>& r, int s) {
#pragma unroll
  for (int q = 0; q < FwdUnits<BM, BN>::U; ++q) {
    const int u = s + 256 * q, row = u >> 2, c = u & 3;
    const bool isa = row < BM;
    const int x = isa ? row : row - BM;
    unsigned char* base = buf + (isa ? 0 : 3 * BM * 64);
    const int pl = (isa ? BM : BN) * 64;
    u32x4w p0, p1, p2;
    split8w(r.v[q], p0, p1, p2);
    const int off = xo(x, c);
    *reinterpret_cast<u32x4w*>(base + off) = p0;
    *reinterpret_cast<u32x4w*>(base + pl + off) = p1;
    *reinterpret_cast<u32x4w*>(base + 2 * pl + off) = p2;
  }
}

}  // namespace

template <int BM, int BN>
__global__ __launch_bounds__(WT, 1) void gemm_x6s_kernel(GemmArgs a_in, GemmBatch gb) {
  constexpr int FB = 3 * (BM + BN) * 64;   // one plane buffer
  constexpr int TM = BM / 64, TN = BN / 64;
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * FB > 4 * 32 * (TN * 32 + 4) * 4 ? 2 * FB
                                                                                               : 4 * 32 * (TN * 32 + 4) * 4];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  GemmArgs a = a_in;
  if (gb.n > 0) {
    const int p = t / a.tiles_mn;
    t -= p * a.tiles_mn;
    a.A = gb.A[p]; a.B = gb.B[p]; a.C = gb.C[p]; a.bias = gb.bias[p]; a.aux = gb.aux[p];
  }
  const int m0 = (t / a.tiles_n) * BM, n0 = (t % a.tiles_n) * BN;
  const int nk = a.K / 32;
  if (nk <= 0) return;
  if (wave >= 4) {   // branch-free k-tile pairs (see gemm_x6s_wgrad_kernel)
    const int s = tid - 256, last = 32 * (nk - 1);
    const float* rp[FwdUnits<BM, BN>::U];
    fwd_rows<BM, BN>(a, rp, s, m0, n0);
    FwdUnits<BM, BN> r0, r1;
    fwd_load<BM, BN>(rp, r0, 0);
    fwd_load<BM, BN>(rp, r1, min(32, last));
    fwd_store<BM, BN>(lds, r0, s);
    fwd_load<BM, BN>(rp, r0, min(64, last));
    fenced_sync();
    for (int kt = 0; kt < nk; kt += 2) {
      fwd_store<BM, BN>(lds + FB, r1, s);
      fwd_load<BM, BN>(rp, r1, min(32 * (kt + 3), last));
      fenced_sync();
      fwd_store<BM, BN>(lds, r0, s);
      fwd_load<BM, BN>(rp, r0, min(32 * (kt + 4), last));
      fenced_sync();
    }
    return;   // the consumers' epilogue needs no barrier with the splitters past the last k-tile
  }
  const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);
  const int lr = lane & 31, lh = lane >> 5;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
  __syncthreads();
  for (int kt = 0; kt < nk + (nk & 1); ++kt) {
    if (kt < nk) {
      const unsigned char* buf = lds + (kt & 1) * FB;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 fa[TM][3], fb[TN][3];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int off = xo(wm + 32 * i + lr, 2 * s + lh);
#pragma unroll
          for (int p = 0; p < 3; ++p) fa[i][p] = *reinterpret_cast<const bf16x8*>(buf + p * BM * 64 + off);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int off = xo(wn + 32 * j + lr, 2 * s + lh);
#pragma unroll
          for (int p = 0; p < 3; ++p)
            fb[j][p] = *reinterpret_cast<const bf16x8*>(buf + 3 * BM * 64 + p * BN * 64 + off);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma6(fb[j], fa[i], acc[i][j]);
      }
    }
    __syncthreads();
  }
  // epilogue: 128-wide wave tiles stage 32 rows in LDS (whole 256-B row runs); 64-wide ones store
  // straight from the accumulators (gemm_x6g_kernel's two forms).  The planes are free (every
  // splitter has passed the last barrier and writes no more).
  if constexpr (BN >= 128) {
    constexpr int WC = TN * 32, PITCH = WC + 4, C4 = WC / 4;
    float* stg = reinterpret_cast<float*>(lds) + wave * 32 * PITCH;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
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
        if (m < a.M) store4(a, 0, m, n0 + wn + 4 * c4, v);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm + i * 32 + lr;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          const int n = n0 + wn + j * 32 + 8 * r4 + 4 * lh;
          const float4 v = make_float4(acc[i][j][4 * r4], acc[i][j][4 * r4 + 1], acc[i][j][4 * r4 + 2],
                                       acc[i][j][4 * r4 + 3]);
          if (m < a.M) store4(a, 0, m, n, v);
        }
    }
  }
}

void launch_x6s(GemmArgs a, int bm, int bn, hipStream_t s, const GemmBatch* gbp) {
  GemmBatch none;
  none.n = 0;
  const GemmBatch& gb = gbp ? *gbp : none;
  auto go = [&](auto kern, int BM_, int BN_) {
    a.tiles_n = (a.N + BN_ - 1) / BN_;
    a.tiles_mn = a.tiles_n * ((a.M + BM_ - 1) / BM_);
    a.ntiles = a.tiles_mn;
    a.nsplit = 1;
    a.ws = nullptr;
    klaunch(kern, (unsigned)a.tiles_mn * (unsigned)(gb.n > 0 ? gb.n : 1), WT, 0, s, a, gb);
  };
  if (bm == 128 && bn == 128) go(gemm_x6s_kernel<128, 128>, 128, 128);
  else if (bm == 128) go(gemm_x6s_kernel<128, 64>, 128, 64);
  else if (bn == 128) go(gemm_x6s_kernel<64, 128>, 64, 128);
  else go(gemm_x6s_kernel<64, 64>, 64, 64);
}

void launch_x6s_wgrad(GemmArgs a, int splits, hipStream_t s, int max_grid) {
  a.tiles_n = (a.N + TBN - 1) / TBN;
  a.tiles_mn = a.tiles_n * ((a.M + TBM - 1) / TBM);
  a.ntiles = a.tiles_mn * splits;
  a.nsplit = splits;
  unsigned grid = (unsigned)a.ntiles;
  if (max_grid > 0 && grid > (unsigned)max_grid) grid = (unsigned)max_grid & ~7u ? (unsigned)max_grid & ~7u : 8u;
  if (a.amap.rdiv > 0 || a.bmap.rdiv > 0) klaunch(gemm_x6s_wgrad_kernel<true>, grid, WT, 0, s, a);
  else klaunch(gemm_x6s_wgrad_kernel<false>, grid, WT, 0, s, a);
}

}  // namespace mrg
