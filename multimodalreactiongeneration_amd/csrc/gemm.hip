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
#include "gemm_common.h"
#include <cstdlib>

namespace mrg {

// One operand tile (rows of the MFMA M or N dimension x BK) staged k-major in LDS:
// S[k][x], x = m (or n).  TR says which index is contiguous in memory:
//   TR = 1 : memory row = k, contiguous along x  -> float4 along x, ds_write_b128
//   TR = 0 : memory row = x, contiguous along k  -> float4 along k (8 lanes cover
//            one 128-B k-run of a row), four scalar LDS writes; row pitch X + 1
//            keeps those writes bank-conflict free.
template <int X, int TR, bool VEC, int BK>
struct TileIO {
  static constexpr int PAD = TR ? 4 : 1;
  static constexpr int LD = X + PAD;
  static constexpr int NV = X * BK / 4 / NT;  // float4 per thread per tile
  float4 r[NV];

  __device__ __forceinline__ void load(const float* base, const RowMap& map, int x0, int xlim, int k0,
                                       int kend) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int e = tid + i * NT;
      int x, k;
      if (TR) { x = (e % (X / 4)) * 4; k = e / (X / 4); } else { k = (e % (BK / 4)) * 4; x = e / (BK / 4); }
      int gx = x0 + x, gk = k0 + k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (TR) {
        if (gk < kend) {
          const float* p = base + map.off(gk) + gx;
          if (VEC && gx + 3 < xlim) v = *reinterpret_cast<const float4*>(p);
          else {
            if (gx < xlim) v.x = p[0];
            if (gx + 1 < xlim) v.y = p[1];
            if (gx + 2 < xlim) v.z = p[2];
            if (gx + 3 < xlim) v.w = p[3];
          }
        }
      } else {
        if (gx < xlim) {
          const float* p = base + map.off(gx) + gk;
          if (VEC && gk + 3 < kend) v = *reinterpret_cast<const float4*>(p);
          else {
            if (gk < kend) v.x = p[0];
            if (gk + 1 < kend) v.y = p[1];
            if (gk + 2 < kend) v.z = p[2];
            if (gk + 3 < kend) v.w = p[3];
          }
        }
      }
      r[i] = v;
    }
  }

  __device__ __forceinline__ void store(float* S) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int e = tid + i * NT;
      if (TR) {
        int x = (e % (X / 4)) * 4, k = e / (X / 4);
        *reinterpret_cast<float4*>(S + k * LD + x) = r[i];
      } else {
        int k = (e % (BK / 4)) * 4, x = e / (BK / 4);
        S[(k + 0) * LD + x] = r[i].x;
        S[(k + 1) * LD + x] = r[i].y;
        S[(k + 2) * LD + x] = r[i].z;
        S[(k + 3) * LD + x] = r[i].w;
      }
    }
  }
};

template <int BM, int BN, int BK, int TA, int TB, bool VA, bool VB>
__global__ __launch_bounds__(NT, (BK == 32 ? 3 : 2)) void gemm_f32_kernel(GemmArgs a) {
  using IA = TileIO<BM, TA, VA, BK>;
  using IB = TileIO<BN, !TB, VB, BK>;  // B(k, n): memory row k when TB == 0 (contiguous along n)
  constexpr int TM = BM / 64, TN = BN / 64;
  __shared__ __attribute__((aligned(16))) float As[BK * IA::LD];
  __shared__ __attribute__((aligned(16))) float Bs[BK * IB::LD];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * (BM / 2);
  const int wn = (wave & 1) * (BN / 2);
  const int lr = lane & 31, lk = lane >> 5;

  // Persistent walk over output tiles (n fastest, so co-running blocks share A rows in L2).
  // The first K tile of the NEXT output tile is loaded under the last MFMAs of this one, so
  // its HBM latency and this tile's epilogue stores overlap instead of adding up (K = 256
  // GEMMs are 8 K tiles long: the per-tile prologue was a third of their time).
  auto coords = [&](int t, int& m0, int& n0, int& kbeg, int& kend) {
    const int z = t / a.tiles_mn, r = t - z * a.tiles_mn;
    m0 = (r / a.tiles_n) * BM;
    n0 = (r % a.tiles_n) * BN;
    kbeg = z * a.kchunk;
    kend = min(a.K, kbeg + a.kchunk);
  };
  IA ia;
  IB ib;
  int t = blockIdx.x;
  int m0, n0, kbeg, kend;
  if (t < a.ntiles) {
    coords(t, m0, n0, kbeg, kend);
    if (kbeg < kend) {
      ia.load(a.A, a.amap, m0, a.M, kbeg, kend);
      ib.load(a.B, a.bmap, n0, a.N, kbeg, kend);
    }
  }
  for (; t < a.ntiles; t += gridDim.x) {
    const int tn = t + gridDim.x;
    int m1 = 0, n1 = 0, kb1 = 0, ke1 = 0;
    if (tn < a.ntiles) coords(tn, m1, n1, kb1, ke1);

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    for (int k0 = kbeg; k0 < kend; k0 += BK) {
      ia.store(As);
      ib.store(Bs);
      __syncthreads();
      {  // next K tile's global loads fly under this tile's MFMAs (or the next output tile's first)
        const bool more = k0 + BK < kend;
        const int lm = more ? m0 : m1, ln = more ? n0 : n1;
        const int lk = more ? k0 + BK : kb1, lke = more ? kend : ke1;
        if (more || (tn < a.ntiles && kb1 < ke1)) {
          ia.load(a.A, a.amap, lm, a.M, lk, lke);
          ib.load(a.B, a.bmap, ln, a.N, lk, lke);
        }
      }
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        float fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = As[(2 * kk + lk) * IA::LD + wm + i * 32 + lr];
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = Bs[(2 * kk + lk) * IB::LD + wn + j * 32 + lr];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
      __syncthreads();
    }

    // epilogue.  The MFMA computes C^T (B fragment as its first operand), so with its C/D map
    // (col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)) a lane holds, for ONE row m of C, four
    // consecutive columns per r>>2: every C access is a 16-B vector.
    const int z = t / a.tiles_mn;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm + i * 32 + lr;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          const int n = n0 + wn + j * 32 + 8 * r4 + 4 * lk;
          const float4 v = make_float4(acc[i][j][4 * r4], acc[i][j][4 * r4 + 1], acc[i][j][4 * r4 + 2],
                                       acc[i][j][4 * r4 + 3]);
          if (m < a.M) store4(a, z, m, n, v);
        }
    }
    m0 = m1; n0 = n1; kbeg = kb1; kend = ke1;
  }
}

// ----------------------------------------------------------------------------------------------
// fp32 GEMM on the bf16 matrix cores: "x6" split.  Every fp32 operand is cut into three bf16
// planes v = v0 + v1 + v2 + r (v0 = bf16(v), v1 = bf16(v - v0), v2 = bf16(v - v0 - v1),
// |r| <= 2^-24 |v|: 24 significand bits, the fp32 width) while it is staged into LDS, and the
// six products with i + j <= 2 (a0b0, a0b1, a1b0, a0b2, a1b1, a2b0) are accumulated in fp32 by
// v_mfma_f32_32x32x16_bf16.  bf16 x bf16 products are exact in fp32; the dropped terms and
// the residuals are <= ~2^-22 |a b| per product, the accuracy class of an fp32 fmaf chain
// (2^-24 per op), at 6 x 32 = 192 MFMA cycles per 32x32x16 block instead of 8 x 64 = 512 on
// v_mfma_f32_32x32x2_f32.  bf16 keeps the fp32 exponent range, so no scaling is needed.
//
// LDS image per plane: [x][32 k] bf16 (64-B rows), 16-B chunks c = k / 8.  Byte offset
//   off(x, c) = 256 (x >> 2) + 64 ((x & 3) ^ g) + 16 (c ^ g),  g = (x >> 2) & 3
// keeps the fragment reads (16 lanes = 16 consecutive rows, one chunk) and both staging
// patterns (4 rows x 64 B per 32 lanes, or 4 rows spaced 4 apart) bank-conflict free.
static constexpr int XBK = 32;

__device__ __forceinline__ int x6_off(int x, int c) {
  const int g = (x >> 2) & 3;
  return ((x >> 2) << 8) + (((x & 3) ^ g) << 6) + ((c ^ g) << 4);
}


// One operand tile (X rows of the MFMA M or N dimension x XBK) for the x6 kernel.
//   TR = 0 : memory row = x, contiguous along k: thread loads float4 (x, 4 k), 8 threads per row
//   TR = 1 : memory row = k, contiguous along x: thread loads a 4 k x 4 x block (4 float4) and
//            transposes it in registers (kg = tid % 8 fastest, so 32 lanes write 4 rows 4 apart)
template <int X, int TR, bool VEC, bool P0ONLY = false>
struct TileX6 {
  static constexpr int NV = TR ? 4 : X * XBK / 4 / NT;
  static constexpr int ACT = TR ? (X / 4) * (XBK / 4) : NT;  // active threads
  float4 r[NV];

  __device__ __forceinline__ void load(const float* base, const RowMap& map, int x0, int xlim, int k0, int kend) {
    const int tid = threadIdx.x;
    if (TR) {
      if (tid >= ACT) return;
      const int kg = tid & 7, mg = tid >> 3;
      const int gx = x0 + 4 * mg;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int gk = k0 + 4 * kg + i;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gk < kend) {
          const float* p = base + map.off(gk) + gx;
          if (VEC && gx + 3 < xlim) v = *reinterpret_cast<const float4*>(p);
          else {
            if (gx < xlim) v.x = p[0];
            if (gx + 1 < xlim) v.y = p[1];
            if (gx + 2 < xlim) v.z = p[2];
            if (gx + 3 < xlim) v.w = p[3];
          }
        }
        r[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int e = tid + i * NT;
        const int x = e >> 3, gk = k0 + 4 * (e & 7), gx = x0 + x;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gx < xlim) {
          const float* p = base + map.off(gx) + gk;
          if (VEC && gk + 3 < kend) v = *reinterpret_cast<const float4*>(p);
          else {
            if (gk < kend) v.x = p[0];
            if (gk + 1 < kend) v.y = p[1];
            if (gk + 2 < kend) v.z = p[2];
            if (gk + 3 < kend) v.w = p[3];
          }
        }
        r[i] = v;
      }
    }
  }

  // TR = 1: add this thread's 4 k-rows into per-x sums (column j = x offset 4 mg + j)
  __device__ __forceinline__ void accum(float (&cs)[4]) const {
    if (TR && (int)threadIdx.x < ACT) {
      cs[0] += (r[0].x + r[1].x) + (r[2].x + r[3].x);
      cs[1] += (r[0].y + r[1].y) + (r[2].y + r[3].y);
      cs[2] += (r[0].z + r[1].z) + (r[2].z + r[3].z);
      cs[3] += (r[0].w + r[1].w) + (r[2].w + r[3].w);
    }
  }

  __device__ __forceinline__ void store(unsigned char* S0, unsigned char* S1, unsigned char* S2) const {
    const int tid = threadIdx.x;
    if (TR) {
      if (tid >= ACT) return;
      const int kg = tid & 7, mg = tid >> 3;
      const float c0[4] = {r[0].x, r[0].y, r[0].z, r[0].w};
      const float c1[4] = {r[1].x, r[1].y, r[1].z, r[1].w};
      const float c2[4] = {r[2].x, r[2].y, r[2].z, r[2].w};
      const float c3[4] = {r[3].x, r[3].y, r[3].z, r[3].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = x6_off(4 * mg + j, kg >> 1) + 8 * (kg & 1);
        if (P0ONLY) {
          *reinterpret_cast<uint2*>(S0 + o) = make_uint2(pk_bf16(c0[j], c1[j]), pk_bf16(c2[j], c3[j]));
          continue;
        }
        uint2 p0, p1, p2;
        split4(c0[j], c1[j], c2[j], c3[j], p0, p1, p2);
        *reinterpret_cast<uint2*>(S0 + o) = p0;
        *reinterpret_cast<uint2*>(S1 + o) = p1;
        *reinterpret_cast<uint2*>(S2 + o) = p2;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int e = tid + i * NT;
        const int x = e >> 3, q = e & 7;
        const int o = x6_off(x, q >> 1) + 8 * (q & 1);
        if (P0ONLY) {
          *reinterpret_cast<uint2*>(S0 + o) = make_uint2(pk_bf16(r[i].x, r[i].y), pk_bf16(r[i].z, r[i].w));
          continue;
        }
        uint2 p0, p1, p2;
        split4(r[i].x, r[i].y, r[i].z, r[i].w, p0, p1, p2);
        *reinterpret_cast<uint2*>(S0 + o) = p0;
        *reinterpret_cast<uint2*>(S1 + o) = p1;
        *reinterpret_cast<uint2*>(S2 + o) = p2;
      }
    }
  }
};


// In-launch split-K combine (cdna_hip_programming.md, "Projection GEMM at M = 256", item 2):
// every K slice stores its fp32 slab and draws a ticket for its tile; the workgroup that draws
// the last one sums the tile's slabs in z order (deterministic, the order splitk_reduce uses)
// and runs the epilogue, then returns the ticket counter to 0 for the next launch.  Agent-scope
// release before the ticket, acquire after it, so slices on different XCDs are seen.
template <int BM, int BN>
__device__ __forceinline__ void splitk_fixup(const GemmArgs& a, int tile, int m0, int n0, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's slab stores
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(a.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (unsigned)(a.nsplit - 1);
    if (last) {
      __hip_atomic_store(a.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  const int last = *flag;
  __syncthreads();  // the flag lives in the staging array the next tile overwrites
  if (!last) return;
  GemmArgs b = a;
  b.ws = nullptr;  // store4 now writes C through the epilogue
  const long slab = (long)a.M * a.N;
  constexpr int C4 = BN / 4;
  for (int e = threadIdx.x; e < BM * C4; e += NT) {
    const int m = m0 + e / C4, n = n0 + 4 * (e % C4);
    if (m >= a.M || n >= a.N) continue;
    const float* p = a.ws + (long)m * a.N + n;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.vec && n + 3 < a.N) {
      for (int z = 0; z < a.nsplit; ++z) {
        const float4 v = *reinterpret_cast<const float4*>(p + z * slab);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
    } else {
      for (int z = 0; z < a.nsplit; ++z) {
        s.x += p[z * slab];
        if (n + 1 < a.N) s.y += p[z * slab + 1];
        if (n + 2 < a.N) s.z += p[z * slab + 2];
        if (n + 3 < a.N) s.w += p[z * slab + 3];
      }
    }
    store4(b, 0, m, n, s);
  }
}

// VAR (tuning experiments only, mrg_gemm_x6_variant): 0 = the product kernel; 1 = split but one
// MFMA (a0 b0) per block; 2 = plane 0 only (no residual split) with six MFMAs; 3 = plane 0 and one
// MFMA (a plain bf16 GEMM on the same structure)
template <int BM, int BN, int TA, int TB, bool VA, bool VB, int VAR = 0>
__global__ __launch_bounds__(NT, 2) void gemm_x6_kernel(GemmArgs a) {
  using IA = TileX6<BM, TA, VA, (VAR >= 2)>;
  using IB = TileX6<BN, !TB, VB, (VAR >= 2)>;  // B(k, n): memory row k when TB == 0 (contiguous along n)
  constexpr int TM = BM / 64, TN = BN / 64;
  // 64x64 tiles (small products) also finish unsplit bias sums and combine split-K slabs in-launch;
  // kept out of the 128-wide kernels, whose register budget sets 3 waves per SIMD
  constexpr bool SMALL = (BM == 64 && BN == 64);
  // one LDS array: the three bf16 planes of the A and B tiles, reused by the epilogue to
  // turn the accumulators into whole-row stores
  __shared__ __attribute__((aligned(16))) unsigned char lds[3 * (BM + BN) * 64];
  unsigned char* const sA[3] = {lds, lds + BM * 64, lds + 2 * BM * 64};
  unsigned char* const sB[3] = {lds + 3 * BM * 64, lds + 3 * BM * 64 + BN * 64, lds + 3 * BM * 64 + 2 * BN * 64};

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * (BM / 2);
  const int wn = (wave & 1) * (BN / 2);
  const int lr = lane & 31, lh = lane >> 5;

  auto coords = [&](int t, int& m0, int& n0, int& kbeg, int& kend) {
    const int z = t / a.tiles_mn, r = t - z * a.tiles_mn;
    m0 = (r / a.tiles_n) * BM;
    n0 = (r % a.tiles_n) * BN;
    kbeg = z * a.kchunk;
    kend = min(a.K, kbeg + a.kchunk);
  };
  IA ia;
  IB ib;
  int t = blockIdx.x;
  int m0, n0, kbeg, kend;
  if (t < a.ntiles) {
    coords(t, m0, n0, kbeg, kend);
    if (kbeg < kend) {
      ia.load(a.A, a.amap, m0, a.M, kbeg, kend);
      ib.load(a.B, a.bmap, n0, a.N, kbeg, kend);
    }
  }
  for (; t < a.ntiles; t += gridDim.x) {
    const int tn = t + gridDim.x;
    int m1 = 0, n1 = 0, kb1 = 0, ke1 = 0;
    if (tn < a.ntiles) coords(tn, m1, n1, kb1, ke1);

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    const bool do_asum = TA && a.asum && n0 == 0;
    float cs[4] = {0.f, 0.f, 0.f, 0.f};

    for (int k0 = kbeg; k0 < kend; k0 += XBK) {
      if (do_asum) ia.accum(cs);
      ia.store(sA[0], sA[1], sA[2]);
      ib.store(sB[0], sB[1], sB[2]);
      __syncthreads();
      {
        const bool more = k0 + XBK < kend;
        const int lm = more ? m0 : m1, ln = more ? n0 : n1;
        const int lk = more ? k0 + XBK : kb1, lke = more ? kend : ke1;
        if (more || (tn < a.ntiles && kb1 < ke1)) {
          ia.load(a.A, a.amap, lm, a.M, lk, lke);
          ib.load(a.B, a.bmap, ln, a.N, lk, lke);
        }
      }
#pragma unroll
      for (int s = 0; s < XBK / 16; ++s) {
        bf16x8 fa[TM][3], fb[TN][3];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int o = x6_off(wm + i * 32 + lr, 2 * s + lh);
#pragma unroll
          for (int p = 0; p < 3; ++p) fa[i][p] = *reinterpret_cast<const bf16x8*>(sA[p] + o);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int o = x6_off(wn + j * 32 + lr, 2 * s + lh);
#pragma unroll
          for (int p = 0; p < 3; ++p) fb[j][p] = *reinterpret_cast<const bf16x8*>(sB[p] + o);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            // small terms first; the MFMA operand order (B, A) yields C^T per lane (epilogue below)
            if (VAR == 1 || VAR == 3) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j][0], fa[i][0], acc[i][j], 0, 0, 0);
              continue;
            }
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j][2], fa[i][0], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j][1], fa[i][1], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j][0], fa[i][2], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j][1], fa[i][0], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j][0], fa[i][1], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j][0], fa[i][0], acc[i][j], 0, 0, 0);
          }
      }
      __syncthreads();
    }

    // epilogue: same C^T lane map as the f32 kernel (one row m, four consecutive n per r>>2)
    const int z = t / a.tiles_mn;
    if (do_asum) {  // the 8 k-group lanes of an m-group sum their partials; lane kg = 0 writes
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cs[j] += __shfl_xor(cs[j], 1, 64);
        cs[j] += __shfl_xor(cs[j], 2, 64);
        cs[j] += __shfl_xor(cs[j], 4, 64);
      }
      const int mg = threadIdx.x >> 3;
      if ((threadIdx.x & 7) == 0 && (int)threadIdx.x < IA::ACT) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int m = m0 + 4 * mg + j;
          if (m >= a.M) continue;
          if (!SMALL || a.ws) {
            a.asum[(long)z * a.M + m] = cs[j];
          } else {  // 64x64 tiles, no split: this tile holds the whole sum of row m; finish it here
            a.asum_out[m] = (a.asum_beta != 0.0f ? a.asum_beta * a.asum_out[m] : 0.0f) + cs[j];
            if (a.asum_out2)
              a.asum_out2[m] = (a.asum_beta != 0.0f ? a.asum_beta * a.asum_out2[m] : 0.0f) + cs[j];
          }
        }
      }
    }
    // Each wave stages one 32-row slab of its accumulators in LDS (C^T lane map: lane = row,
    // four consecutive n per register quad) and reads it back row-major, so every store
    // instruction writes whole 128-256-B row segments instead of 32 B in each of 32 rows.
    // (64-column tiles keep the direct per-lane stores: measured faster there)
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
          const int q = lane + 64 * it, row = q / C4, c4 = q % C4;
          const float4 v = *reinterpret_cast<const float4*>(stg + row * PITCH + 4 * c4);
          const int m = m0 + wm + i * 32 + row;
          if (m < a.M) store4(a, z, m, n0 + wn + 4 * c4, v);
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __syncthreads();  // the staging area is the next tile's A/B planes
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
            if (m < a.M) store4(a, z, m, n, v);
          }
      }
    }
    if constexpr (SMALL) {
      if (a.cnt) splitk_fixup<BM, BN>(a, t - z * a.tiles_mn, m0, n0, reinterpret_cast<int*>(lds));
    }
    m0 = m1; n0 = n1; kbeg = kb1; kend = ke1;
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

// Split-K slab reduce.  A block = 32 outputs x 8 z-groups: thread (o, g) sums slabs
// z = g, g + 8, ... (two loads in flight), then group 0 adds the 8 partials from LDS in a
// fixed order (deterministic).  Vector outputs (float4 of C) when a.vec and N % 4 == 0; the
// fused row sums of A (a.asum, [splits][M]) ride in trailing blocks of scalar outputs.
static constexpr int RZG = 8;   // z-groups per output
static constexpr int RPB = 32;  // outputs per block

template <typename V>
__device__ __forceinline__ V zsum(const V* base, long zs, int splits, int g) {
  V s0 = V{}, s1 = V{};
  int z = g;
  for (; z + RZG < splits; z += 2 * RZG) {
    const V v0 = base[(long)z * zs], v1 = base[(long)(z + RZG) * zs];
    s0 += v0;
    s1 += v1;
  }
  if (z < splits) s0 += base[(long)z * zs];
  return s0 + s1;
}

typedef float f32x4v __attribute__((ext_vector_type(4)));

// row sums of A for RPB rows per block (fused bias gradients)
__device__ __forceinline__ void asum_block(const GemmArgs& a, int splits, long blk) {
  __shared__ float rs[RZG][RPB];
  const int o = threadIdx.x % RPB, g = threadIdx.x / RPB;
  const long m = blk * RPB + o;
  rs[g][o] = m < a.M ? zsum(a.asum + m, (long)a.M, splits, g) : 0.0f;
  __syncthreads();
  if (g == 0 && m < a.M) {
    float r = rs[0][o];
#pragma unroll
    for (int i = 1; i < RZG; ++i) r += rs[i][o];
    a.asum_out[m] = (a.asum_beta != 0.0f ? a.asum_beta * a.asum_out[m] : 0.0f) + r;
    if (a.asum_out2) a.asum_out2[m] = (a.asum_beta != 0.0f ? a.asum_beta * a.asum_out2[m] : 0.0f) + r;
  }
}

__global__ __launch_bounds__(256) void asum_reduce_kernel(GemmArgs a, int splits) {
  asum_block(a, splits, blockIdx.x);
}

__global__ __launch_bounds__(256) void splitk_reduce4_kernel(GemmArgs a, int splits) {
  __shared__ f32x4v red[RZG][RPB];
  const int o = threadIdx.x % RPB, g = threadIdx.x / RPB;
  const long total = (long)a.M * a.N;
  const long cblocks = (total / 4 + RPB - 1) / RPB;
  if ((long)blockIdx.x >= cblocks) {  // trailing blocks: the fused bias-gradient sums
    asum_block(a, splits, (long)blockIdx.x - cblocks);
    return;
  }
  const long q = (long)blockIdx.x * RPB + o;  // float4 index into C
  f32x4v s = f32x4v{0.f, 0.f, 0.f, 0.f};
  if (q * 4 < total) s = zsum(reinterpret_cast<const f32x4v*>(a.ws) + q, total / 4, splits, g);
  red[g][o] = s;
  __syncthreads();
  if (g == 0 && q * 4 < total) {
    f32x4v r = red[0][o];
#pragma unroll
    for (int i = 1; i < RZG; ++i) r += red[i][o];
    const long idx = q * 4;
    const int m = idx / a.N, n = idx % a.N;
    GemmArgs b = a;
    b.ws = nullptr;  // store4 writes C (alpha / beta / bias / epilogue) instead of a slab
    store4(b, 0, m, n, make_float4(r.x, r.y, r.z, r.w));
  }
}

// column sums, stage 1: part[s][n] = sum of X(row, n) over rows [s*rows_per, (s+1)*rows_per).
// A block owns 64 columns (one per lane: 256-B coalesced row segments); its 4 waves
// interleave over the rows, then combine through LDS.
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* X, RowMap map, int rows, int N,
                                                             int rows_per, float* part) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + lane;
  const int s = blockIdx.y;
  const int r0 = s * rows_per, r1 = min(rows, r0 + rows_per);
  float acc = 0.0f;
  if (n < N) {
    int r = r0 + wave;
    for (; r + 12 < r1; r += 16) {  // 4 independent loads in flight per lane
      float a0 = X[map.off(r) + n], a1 = X[map.off(r + 4) + n];
      float a2 = X[map.off(r + 8) + n], a3 = X[map.off(r + 12) + n];
      acc += (a0 + a1) + (a2 + a3);
    }
    for (; r < r1; r += 4) acc += X[map.off(r) + n];
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && n < N) part[(long)s * N + n] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// stage 2: out[n] = beta*out[n] + sum_s part[s][n]; out2 (nullable) receives the same update.
// 16 waves per 64 columns, fixed combine order (deterministic).
__global__ __launch_bounds__(1024) void colsum_final_kernel(const float* part, int S, int N, float beta, float* out,
                                                            float* out2) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + lane;
  float acc = 0.0f;
  if (n < N) {
#pragma unroll 4
    for (int s = wave; s < S; s += 16) acc += part[(long)s * N + n];
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && n < N) {
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < 16; ++w) v += red[w][lane];
    out[n] = (beta != 0.0f ? beta * out[n] : 0.0f) + v;
    if (out2) out2[n] = (beta != 0.0f ? beta * out2[n] : 0.0f) + v;
  }
}

// blocks per CU the hardware admits for a kernel (cached per kernel FUNCTION: every instantiation
// has the same C++ type, so the cache is keyed by its address), x CUs of the current device
// Host-side cap on resident blocks per CU for the persistent tile walks (0 = the occupancy the HW
// reports).  The weight-gradient products issued beside a latency-bound recurrence run with 1, so
// they take the CU room the recurrence leaves instead of queueing whole waves of tiles ahead of it.
static int g_blocks_per_cu = 0;

template <typename K>
static int resident_blocks(K kernel) {
  static const void* keys[256];
  static int vals[256];
  static int nkeys = 0;
  static int cus[16] = {0};
  const void* key = reinterpret_cast<const void*>(kernel);
  int per_cu = -1;
  for (int i = 0; i < nkeys; ++i)
    if (keys[i] == key) { per_cu = vals[i]; break; }
  if (per_cu < 0) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, key, NT, 0) != hipSuccess || n < 1) n = 1;
    per_cu = n;
    if (nkeys < 256) { keys[nkeys] = key; vals[nkeys] = n; ++nkeys; }
  }
  if (g_blocks_per_cu > 0 && per_cu > g_blocks_per_cu) per_cu = g_blocks_per_cu;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 16) dev = 0;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
    cus[dev] = n;
  }
  return per_cu * cus[dev];
}

// CU count of the current device (cached per device)
static int resident_cus() {
  static int cus[16] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 16) dev = 0;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

template <int BM, int BN, int BK>
static void launch_tile(GemmArgs a, int ta, int tb, bool va, bool vb, int splits, hipStream_t s) {
  a.tiles_n = (a.N + BN - 1) / BN;
  a.tiles_mn = a.tiles_n * ((a.M + BM - 1) / BM);
  a.ntiles = a.tiles_mn * splits;
  a.nsplit = splits;
  const int code = (ta << 3) | (tb << 2) | ((int)va << 1) | (int)vb;
  switch (code) {
#define MRG_G(TA, TB, VA, VB)                                                                    \
    case (TA << 3) | (TB << 2) | (VA << 1) | VB: {                                               \
      auto k = gemm_f32_kernel<BM, BN, BK, TA, TB, (bool)VA, (bool)VB>;                              \
      const int grid = a.ntiles < resident_blocks(k) ? a.ntiles : resident_blocks(k);           \
      klaunch(k, grid, NT, 0, s, a);                                                                  \
    } break;
    MRG_G(0, 0, 0, 0) MRG_G(0, 0, 0, 1) MRG_G(0, 0, 1, 0) MRG_G(0, 0, 1, 1)
    MRG_G(0, 1, 0, 0) MRG_G(0, 1, 0, 1) MRG_G(0, 1, 1, 0) MRG_G(0, 1, 1, 1)
    MRG_G(1, 0, 0, 0) MRG_G(1, 0, 0, 1) MRG_G(1, 0, 1, 0) MRG_G(1, 0, 1, 1)
    MRG_G(1, 1, 0, 0) MRG_G(1, 1, 0, 1) MRG_G(1, 1, 1, 0) MRG_G(1, 1, 1, 1)
#undef MRG_G
  }
}

template <int BM, int BN, int VAR = 0>
static void launch_tile_x6(GemmArgs a, int ta, int tb, bool va, bool vb, int splits, hipStream_t s) {
  a.tiles_n = (a.N + BN - 1) / BN;
  a.tiles_mn = a.tiles_n * ((a.M + BM - 1) / BM);
  a.ntiles = a.tiles_mn * splits;
  a.nsplit = splits;
  const int code = (ta << 3) | (tb << 2) | ((int)va << 1) | (int)vb;
  switch (code) {
#define MRG_G(TA, TB, VA, VB)                                                                    \
    case (TA << 3) | (TB << 2) | (VA << 1) | VB: {                                               \
      auto k = gemm_x6_kernel<BM, BN, TA, TB, (bool)VA, (bool)VB, VAR>;                           \
      const int grid = a.ntiles < resident_blocks(k) ? a.ntiles : resident_blocks(k);           \
      klaunch(k, grid, NT, 0, s, a);                                                                  \
    } break;
    MRG_G(0, 0, 0, 0) MRG_G(0, 0, 0, 1) MRG_G(0, 0, 1, 0) MRG_G(0, 0, 1, 1)
    MRG_G(0, 1, 0, 0) MRG_G(0, 1, 0, 1) MRG_G(0, 1, 1, 0) MRG_G(0, 1, 1, 1)
    MRG_G(1, 0, 0, 0) MRG_G(1, 0, 0, 1) MRG_G(1, 0, 1, 0) MRG_G(1, 0, 1, 1)
    MRG_G(1, 1, 0, 0) MRG_G(1, 1, 0, 1) MRG_G(1, 1, 1, 0) MRG_G(1, 1, 1, 1)
#undef MRG_G
  }
}


// ----------------------------------------------------------------------------------------------
// Few-row products (M <= 64: the batch rows of a T = 1 decode step, lstm_with_sample.py:410-433,
// lstmformer.py:498-521).  Staging a 64x64 tile through LDS 32 k at a time leaves every k step
// waiting on a global round trip, so these run as exact f32 MFMA (v_mfma_f32_16x16x4_f32) straight
// from global/L2 into registers: a workgroup owns one 16 x 16 output block, its 4 waves take K
// quarters and each wave's 4 lane groups contiguous sub-ranges of those (operands load as runs),
// all loads of a chunk are in flight at once, and the 4 partial blocks are summed in LDS in a
// fixed order before the epilogue.  Arithmetic: fp32 FMA chains (no bf16 split needed).
typedef unsigned int u32x4r __attribute__((ext_vector_type(4)));
static constexpr int ROWS_OOB = 0x7fffff00;  // masked-off lanes load past every range (hardware zero)

// Operand loads are range-checked buffer loads with the out-of-range lanes pointed past the
// descriptor (cdna_hip_programming.md T8): no branch per load, so a lane's whole chunk of loads is
// in flight at once.  (Guarded plain loads compiled to a branch + vmcnt(0) per 4 elements: one L2
// round trip per load, 9 us for a 64 x 256 x 1024 product.)
template <int TA, int TB, int CH>
__global__ __launch_bounds__(256) void gemm_rows_kernel(GemmArgs a) {
  __shared__ float red[4][16][17];
  __shared__ float rsum[16][16];  // fused row sums of op(A) (TA: the bias gradient), per (wave, group)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, l16 = lane & 15;
  const int m0 = blockIdx.y * 16, n0 = blockIdx.x * 16;
  const int KQ = (a.K + 15) / 16;  // contiguous k per (wave, lane group)
  const int kb = (wave * 4 + g) * KQ;
  const int ke = min(a.K, kb + KQ);
  const int m = m0 + l16, n = n0 + l16;
  const bool mv = m < a.M, nv = n < a.N;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.A), (short)0, a.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.B), (short)0, a.b_bytes, 0x00020000);
  // element offsets of this lane's row (A, TA = 0) / column (B, TB = 1); the other forms walk rows of k
  const long arow = (!TA && mv) ? a.amap.off(m) : 0;
  const long bcol = (TB && nv) ? a.bmap.off(n) : 0;
  const bool sums = TA && a.asum_out && blockIdx.x == 0;
  f32x4v acc = f32x4v{0.f, 0.f, 0.f, 0.f};
  float rs = 0.0f;
  for (int k0 = kb; k0 < ke; k0 += CH) {
    float av[CH], bv[CH];
#pragma unroll
    for (int s = 0; s < CH; s += 4) {
      const int k = k0 + s;
      if (!TA) {  // 4 consecutive k of row m: one 16-B load, the k >= ke tail zeroed by select
        const int off = (mv && k < ke) ? (int)((arow + k) * 4) : ROWS_OOB;
        const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0));
        av[s] = v.x; av[s + 1] = k + 1 < ke ? v.y : 0.0f; av[s + 2] = k + 2 < ke ? v.z : 0.0f;
        av[s + 3] = k + 3 < ke ? v.w : 0.0f;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int off = (mv && k + e < ke) ? (int)((a.amap.off(k + e) + m) * 4) : ROWS_OOB;
          av[s + e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, off, 0, 0));
        }
      }
      if (TB) {
        const int off = (nv && k < ke) ? (int)((bcol + k) * 4) : ROWS_OOB;
        const float4 v = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 0));
        bv[s] = v.x; bv[s + 1] = k + 1 < ke ? v.y : 0.0f; bv[s + 2] = k + 2 < ke ? v.z : 0.0f;
        bv[s + 3] = k + 3 < ke ? v.w : 0.0f;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int off = (nv && k + e < ke) ? (int)((a.bmap.off(k + e) + n) * 4) : ROWS_OOB;
          bv[s + e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, off, 0, 0));
        }
      }
    }
#pragma unroll
    for (int s = 0; s < CH; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
    if (sums) {
#pragma unroll
      for (int s = 0; s < CH; ++s) rs += av[s];
    }
  }
  // lane holds C[4g + i][l16] of this wave's partial block
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][4 * g + i][l16] = acc[i];
  if (sums) rsum[wave * 4 + g][l16] = rs;
  __syncthreads();
  const int r = threadIdx.x >> 4, c = threadIdx.x & 15;
  const int mo = m0 + r, no = n0 + c;
  if (mo < a.M && no < a.N) {
    const float v = ((red[0][r][c] + red[1][r][c]) + red[2][r][c]) + red[3][r][c];
    a.C[(long)mo * a.ldc + no] = apply_epi(a, v, mo, no);
  }
  if (sums && threadIdx.x < 16 && m0 + (int)threadIdx.x < a.M) {  // bias gradient rows, fixed order
    const int mm = m0 + threadIdx.x;
    float t = 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += rsum[q][threadIdx.x];
    a.asum_out[mm] = (a.asum_beta != 0.0f ? a.asum_beta * a.asum_out[mm] : 0.0f) + t;
    if (a.asum_out2) a.asum_out2[mm] = (a.asum_beta != 0.0f ? a.asum_beta * a.asum_out2[mm] : 0.0f) + t;
  }
}

static void launch_rows(const GemmArgs& a, hipStream_t s) {
  const dim3 grid((a.N + 15) / 16, (a.M + 15) / 16);
  const bool big = (a.K + 15) / 16 > 16;
#define MRG_R(TA, TB)                                                                            \
  if (a.transA == TA && a.transB == TB) {                                                        \
    if (big) klaunch(gemm_rows_kernel<TA, TB, 64>, grid, 256, 0, s, a);                               \
    else klaunch(gemm_rows_kernel<TA, TB, 16>, grid, 256, 0, s, a);                                   \
    return;                                                                                      \
  }
  MRG_R(0, 0) MRG_R(0, 1) MRG_R(1, 0) MRG_R(1, 1)
#undef MRG_R
}

static int g_tile_override = -1;
// LDS-DMA x6 kernel for k-contiguous products (gemm_x6g_kernel): 0 = off, else ring depth (2..4);
// MRG_GEMM_GLDS overrides; g_glds_bn = column tile (128 or 64)
static int g_glds = [] {
  const char* e = getenv("MRG_GEMM_GLDS");
  return e ? atoi(e) : 2;
}();
static int g_glds_wg = [] {  // weight-gradient products on gemm_x6g_wgrad_kernel (MRG_GEMM_GLDS_WG=0: off)
  const char* e = getenv("MRG_GEMM_GLDS_WG");
  return e ? atoi(e) : 1;
}();
static int g_glds_bn = [] {  // 64 forces 64-wide column tiles (tuning); 128 = by shape
  const char* e = getenv("MRG_GEMM_GLDS_BN");
  return e ? atoi(e) : 128;
}();


// GEMM arithmetic: 1 = x6 bf16 split on the bf16 matrix cores (default), 0 = exact f32 MFMA
static int g_gemm_mode = [] {
  const char* e = getenv("MRG_GEMM_EXACT");
  return (e && atoi(e) != 0) ? 0 : 1;
}();

static int launch_gemm(int mode, const GemmArgs& a, int tile, int bk, int ta, int tb, bool va, bool vb,
                       int splits, hipStream_t s) {
  ta = ta ? 1 : 0;
  tb = tb ? 1 : 0;
  (void)bk;  // BK = 64 measured no faster on these shapes (short K): only BK = 32 is instantiated
  // bf16 operands (one plane, one MFMA per block), fp32 accumulate.  Measured (r02,
  // tools/tools_gemm_bench.py 2): faster than the x6 split only when both operands are k-contiguous
  // (NT: the forward products, 1.5-1.7x); with a transposed operand this staging structure runs
  // the one-plane form slower than the split (dX 35.7 -> 51.5 us, dW 36.9 -> 67.8 us), so those
  // products keep the split, which is at least as accurate as bf16 operands.
  if (mode == 2 && !(ta == 0 && tb == 1)) mode = 1;
  if (mode == 2) {
    if (tile == 0) launch_tile_x6<128, 128, 3>(a, ta, tb, va, vb, splits, s);
    else if (tile == 1) launch_tile_x6<128, 64, 3>(a, ta, tb, va, vb, splits, s);
    else launch_tile_x6<64, 64, 3>(a, ta, tb, va, vb, splits, s);
    return 0;
  }
  if (mode == 1) {
    if (tile == 0) launch_tile_x6<128, 128>(a, ta, tb, va, vb, splits, s);
    else if (tile == 1) launch_tile_x6<128, 64>(a, ta, tb, va, vb, splits, s);
    else launch_tile_x6<64, 64>(a, ta, tb, va, vb, splits, s);
    return 0;
  }
  if (tile == 0) launch_tile<128, 128, BK>(a, ta, tb, va, vb, splits, s);
  else if (tile == 1) launch_tile<128, 64, BK>(a, ta, tb, va, vb, splits, s);
  else launch_tile<64, 64, BK>(a, ta, tb, va, vb, splits, s);
  return 0;
}

}  // namespace mrg

using namespace mrg;

// GEMM arithmetic mode: 1 = fp32 via the x6 bf16 split (default), 0 = exact f32 MFMA
// (v_mfma_f32_32x32x2_f32, a k-ordered fmaf chain).  Env MRG_GEMM_EXACT=1 selects 0 at load.
MRG_API int mrg_gemm_set_mode(int mode) {
  MRG_REQUIRE(mode == 0 || mode == 1, "mrg_gemm_set_mode: mode must be 0 or 1");
  g_gemm_mode = mode;
  return 0;
}
MRG_API int mrg_gemm_get_mode(void) { return g_gemm_mode; }

// Weight-gradient products on the LDS-DMA kernel (1) or the register-staged one (0); returns the old value.
MRG_API int mrg_gemm_set_glds_wg(int on) {
  const int prev = g_glds_wg;
  g_glds_wg = on ? 1 : 0;
  return prev;
}

// LDS-DMA x6 kernel for k-contiguous products: ring depth 2..4 (0 = off) and column tile (64 forces
// 64-wide tiles; 128 = the shape heuristic).
MRG_API int mrg_gemm_set_glds(int depth, int bn) {
  MRG_REQUIRE(depth == 0 || (depth >= 2 && depth <= 4), "mrg_gemm_set_glds: depth must be 0 or 2..4");
  MRG_REQUIRE(bn == 64 || bn == 128, "mrg_gemm_set_glds: column tile must be 64 or 128");
  g_glds = depth;
  g_glds_bn = bn;
  return 0;
}

// Cap on resident blocks per CU of the following GEMM launches (0 = none); returns the previous cap.
// dst_i [cols_i][rows_i] = src_i [rows_i][cols_i]^T for n matrices, one launch per 32 of them.
MRG_API int mrg_transpose_batched(int n, const float* const* src, float* const* dst, const int* rows, const int* cols,
                                  hipStream_t stream) {
  MRG_REQUIRE(n >= 0 && (n == 0 || (src && dst && rows && cols)), "mrg_transpose_batched: bad arguments");
  for (int b0 = 0; b0 < n; b0 += MRG_TP_MAX) {
    TransposeBatch tb;
    memset(&tb, 0, sizeof(tb));
    tb.n = n - b0 < MRG_TP_MAX ? n - b0 : MRG_TP_MAX;
    int blocks = 0;
    for (int i = 0; i < tb.n; ++i) {
      MRG_REQUIRE(rows[b0 + i] >= 0 && cols[b0 + i] >= 0, "mrg_transpose_batched: negative size");
      tb.src[i] = src[b0 + i]; tb.dst[i] = dst[b0 + i]; tb.rows[i] = rows[b0 + i]; tb.cols[i] = cols[b0 + i];
      tb.first[i] = blocks;
      blocks += ((rows[b0 + i] + 31) / 32) * ((cols[b0 + i] + 31) / 32);
    }
    tb.first[tb.n] = blocks;
    if (blocks == 0) continue;
    klaunch(transpose_batched_kernel, blocks, 256, 0, stream, tb);
    if (check_launch("transpose_batched_kernel")) return 1;
  }
  return 0;
}

MRG_API int mrg_gemm_set_blocks_per_cu(int n) {
  const int prev = g_blocks_per_cu;
  g_blocks_per_cu = n > 0 ? n : 0;
  return prev;
}

// Tuning only: the x6 kernel's structural variants (see gemm_x6_kernel VAR) on C = A B^T,
// A [M][K], B [N][K] row-major, 128x128 tiles, no split-K.  Results are NOT C for var != 0.
MRG_API int mrg_gemm_x6_variant(int var, int M, int N, int K, const float* A, const float* B, float* C,
                                hipStream_t stream) {
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.M = M; a.N = N; a.K = K; a.alpha = 1.0f;
  a.A = A; a.amap = RowMap{K, 0, 0}; a.B = B; a.bmap = RowMap{K, 0, 0}; a.transB = 1;
  a.C = C; a.ldc = N; a.kchunk = ((K + 31) / 32) * 32; a.vec = 1;
  a.tiles_n = (N + 127) / 128;
  a.tiles_mn = a.tiles_n * ((M + 127) / 128);
  a.ntiles = a.tiles_mn;
  switch (var) {
#define MRG_V(V)                                                                            \
    case V: {                                                                               \
      auto k = gemm_x6_kernel<128, 128, 0, 1, true, true, V>;                               \
      const int grid = a.ntiles < resident_blocks(k) ? a.ntiles : resident_blocks(k);      \
      klaunch(k, grid, NT, 0, stream, a);                                                        \
    } break;
    MRG_V(0) MRG_V(1) MRG_V(2) MRG_V(3)
#undef MRG_V
    default: MRG_REQUIRE(false, "mrg_gemm_x6_variant: var 0..3");
  }
  return check_launch("gemm_x6_variant");
}

// Tuning only: force one tile shape (0: 128x128, 1: 128x64, 2: 64x64; -1 = heuristic).
MRG_API int mrg_gemm_force_tile(int tile) {
  MRG_REQUIRE(tile >= -1 && tile <= 2, "mrg_gemm_force_tile: tile must be -1..2");
  g_tile_override = tile;
  return 0;
}

// split-K slabs [splits][M][N] (splits > 1), then room for the fused row sums of A
// ([splits][M]) or, on the unfused path, the column-sum kernels' partials
MRG_API size_t mrg_gemm_workspace_bytes(int M, int N, int splits) {
  const size_t slabs = splits > 1 ? (size_t)splits * M * N : 0;
  const size_t rs = (size_t)(splits > 1 ? splits : 1) * M;
  const size_t cs = (size_t)512 * M;  // colsum_splits(K) <= 512 partial rows of M
  return (slabs + (rs > cs ? rs : cs)) * sizeof(float);
}

MRG_API int mrg_colsum_f32(int rows, int N, const float* X, long ld, long ld_hi, int rdiv,
                           float beta, float* out, float* out2, float* workspace,
                           hipStream_t stream);

static int gemm_ex(int mode, int M, int N, int K, float alpha,
                   const float* A, int transA, long lda, long lda_hi, int a_rdiv,
                   const float* B, int transB, long ldb, long ldb_hi, int b_rdiv,
                   float beta, float* C, long ldc, const float* bias, int epilogue,
                   const float* aux, long ldaux, float* workspace, int splits,
                   float* asum_out, float* asum_out2, float asum_beta,
                   unsigned* counters, hipStream_t stream) {
  const bool mx = mode >= 1;  // bf16 matrix-core paths (x6 split or plain bf16 operands)
  MRG_REQUIRE(M >= 0 && N >= 0 && K >= 0, "mrg_gemm_f32: negative size");
  MRG_REQUIRE(epilogue >= 0 && epilogue <= 3, "mrg_gemm_f32: bad epilogue %d", epilogue);
  MRG_REQUIRE(epilogue < 2 || aux, "mrg_gemm_f32: epilogue %d needs aux", epilogue);
  if (M == 0 || N == 0) return 0;
  if (splits < 1) splits = 1;
  MRG_REQUIRE(splits == 1 || workspace, "mrg_gemm_f32: split-K needs workspace");
  GemmArgs a;
  a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta;
  a.A = A; a.amap = RowMap{lda, lda_hi, a_rdiv}; a.transA = transA;
  a.B = B; a.bmap = RowMap{ldb, ldb_hi, b_rdiv}; a.transB = transB;
  a.C = C; a.ldc = ldc; a.bias = bias; a.epi = epilogue; a.aux = aux; a.ldaux = ldaux;
  const int bk = BK;
  int kc = (K + splits - 1) / splits;
  kc = ((kc + bk - 1) / bk) * bk;
  if (kc == 0) kc = bk;
  splits = (K + kc - 1) / kc;
  if (splits < 1) splits = 1;
  a.kchunk = kc;
  a.ws = splits > 1 ? workspace : nullptr;
  a.asum = nullptr; a.asum_out = asum_out; a.asum_out2 = asum_out2; a.asum_beta = asum_beta;
  a.cnt = nullptr; a.nsplit = splits;
  // fused bias-gradient row sums: x6 path with A = (memory rows k, contiguous along m)
  const bool fuse_asum = asum_out && mx && transA && workspace;
  if (fuse_asum) a.asum = workspace + (splits > 1 ? (long)splits * M * N : 0);
  // vector (float4) global loads need 16-B aligned rows along the contiguous index
  auto aligned = [](const float* p, const RowMap& m) {
    return ((uintptr_t)p & 15) == 0 && (m.ld_lo & 3) == 0 && (m.rdiv <= 0 || (m.ld_hi & 3) == 0);
  };
  const bool va = aligned(A, a.amap), vb = aligned(B, a.bmap);
  a.vec = ((((uintptr_t)C | (uintptr_t)bias | (uintptr_t)aux | (uintptr_t)workspace) & 15) == 0 && (ldc & 3) == 0 &&
           (!aux || (ldaux & 3) == 0) && (!a.ws || (N & 3) == 0)) ? 1 : 0;
  // few-row products (x6 mode): exact f32 MFMA from registers, no split, no LDS staging: M <= 64
  // rows of activations, or a weight gradient over <= 64 rows (K), its bias sums fused
  // (its buffer-load range checks need both operands' extents below 2 GB)
  const long a_ext = transA ? a.amap.off(K > 0 ? K - 1 : 0) + M : a.amap.off(M > 0 ? M - 1 : 0) + K;
  const long b_ext = transB ? a.bmap.off(N > 0 ? N - 1 : 0) + K : a.bmap.off(K > 0 ? K - 1 : 0) + N;
  const bool rows_ok = a_ext * 4 < ROWS_OOB && b_ext * 4 < ROWS_OOB && K > 0;
  if (mx && splits == 1 && rows_ok && ((!transA && M <= 64 && !asum_out) || (transA && K <= 64))) {
    a.transA = transA ? 1 : 0;
    a.transB = transB ? 1 : 0;
    a.a_bytes = (int)(a_ext * 4);
    a.b_bytes = (int)(b_ext * 4);
    launch_rows(a, stream);
    return check_launch("gemm_rows_kernel");
  }
  // LDS-DMA pipelined x6 kernel: k-contiguous A and B, whole 32-deep k-tiles, unsplit
  // (tile by shape, measured with tools/tools_gemm_bench.py: 128 x 128 for N >= 1024, 64 x 64 for
  // N = K = 256, else 64 x 128; ring depth 2 = two workgroups per CU)
  // (mode 2, bf16 operands: the same kernel with one plane and one MFMA per block)
  if (mx && g_glds > 0 && !transA && transB && splits == 1 && !asum_out && K > 0 && (K % 32) == 0 && va &&
      vb && M >= 2048 && N >= 256) {
    int bm = 64, bn = 128;
    if (N >= 1024) bm = 128;
    else if (N == 256 && K <= 256) bn = 64;
    if (g_glds_bn == 64) bn = 64;
    launch_x6g(a, g_glds, bm, bn, stream, mode == 2 ? 1 : 3);
    return check_launch("gemm_x6g_kernel");
  }
  int tile;  // 0: 128x128, 1: 128x64, 2: 64x64
  if (mx) {
    // x6 (measured on the step's shapes, tools_gemm_sweep.py): 128x128 for split-K weight
    // gradients and wide/deep products; 64x64 for narrow ones (N <= 128, or N = 256 at K <= 512
    // with K-contiguous B); small problems take the tile that gives the most workgroups
    const long t0 = (long)((M + 127) / 128) * ((N + 127) / 128) * splits;
    if (splits > 1) tile = transA ? 0 : 2;  // weight gradients / few-row activation products
    else if (t0 < 256) tile = 2;
    else if (N >= 512 || K >= 1024) tile = 0;
    else if (N <= 128) tile = 2;
    else tile = transB ? 2 : 0;
  } else if (M >= 2048 && N > 64) {
    tile = ((long)((M + 127) / 128) * ((N + 127) / 128) * splits >= 400) ? 0 : 1;
  } else if (M >= 2048) {
    tile = 1;
  } else {
    tile = 2;
  }
  if (g_tile_override >= 0 && g_tile_override <= 2) tile = g_tile_override;
  // small split outputs: the last K slice of each tile combines the slabs in-launch (no reduce
  // kernel) when the slabs it must read stay small (<= 64 KB per tile)
  if (splits > 1 && counters && mx && !a.asum && tile == 2) {
    const long tiles = (long)((M + 63) / 64) * ((N + 63) / 64);
    if (tiles <= MRG_GEMM_COUNTERS && (long)splits * 64 * 64 * 4 <= 65536) a.cnt = counters;
  }
  // weight gradients (dY^T X) on the LDS-DMA kernel: k-strided operands, split-K slabs, fused row sums
  const bool wg = mx && g_glds_wg && g_tile_override < 0 && transA && !transB && va && vb && K > 0 &&
                  (K % 32) == 0 && (M % 4) == 0 && (N % 4) == 0 && M >= 64 && N >= 64 && !a.cnt;
  if (wg) {
    tile = 0;
    const int cap = g_blocks_per_cu > 0 ? g_blocks_per_cu * resident_cus() : 0;
    launch_x6g_wgrad(a, splits, 128, 128, stream, mode == 2 ? 1 : 3, cap);
  } else if (launch_gemm(mode, a, tile, bk, transA, transB, va, vb, splits, stream)) {
    return 2;
  }
  if (check_launch("gemm_f32_kernel")) return 1;
  // unsplit 64x64-tile GEMM (x6): its n0 == 0 tiles wrote asum_out directly
  bool asum_done = splits == 1 && tile == 2 && mx;
  if (splits > 1 && !a.cnt) {
    long total = (long)M * N;
    if (a.vec && (N & 3) == 0) {
      const long cb = (total / 4 + RPB - 1) / RPB, ab = a.asum ? (M + RPB - 1) / RPB : 0;
      klaunch(splitk_reduce4_kernel, (unsigned)(cb + ab), 256, 0, stream, a, splits);
      asum_done = a.asum != nullptr;
    } else {
      klaunch(splitk_reduce_kernel, (unsigned)((total + 255) / 256), 256, 0, stream, a, splits);
    }
    if (check_launch("splitk_reduce_kernel")) return 1;
  }
  if (a.asum && !asum_done) {
    klaunch(asum_reduce_kernel, (unsigned)((M + RPB - 1) / RPB), 256, 0, stream, a, splits);
    if (check_launch("asum_reduce_kernel")) return 1;
  } else if (asum_out && !a.asum) {
    // not fusable here (exact-f32 mode or A not k-major): the two-pass column-sum kernels
    MRG_REQUIRE(workspace, "mrg_gemm_f32_ex: row sums need the workspace");
    float* cws = workspace + (splits > 1 ? (long)splits * M * N : 0);
    if (transA) {
      if (int e = mrg_colsum_f32(K, M, A, lda, lda_hi, a_rdiv, asum_beta, asum_out, asum_out2, cws, stream))
        return e;
    } else {
      MRG_REQUIRE(false, "mrg_gemm_f32_ex: row sums need transA = 1");
    }
  }
  return 0;
}

MRG_API int mrg_gemm_f32_ex(int M, int N, int K, float alpha,
                            const float* A, int transA, long lda, long lda_hi, int a_rdiv,
                            const float* B, int transB, long ldb, long ldb_hi, int b_rdiv,
                            float beta, float* C, long ldc, const float* bias, int epilogue,
                            const float* aux, long ldaux, float* workspace, int splits,
                            float* asum_out, float* asum_out2, float asum_beta,
                            unsigned* counters, hipStream_t stream) {
  return gemm_ex(g_gemm_mode, M, N, K, alpha, A, transA, lda, lda_hi, a_rdiv, B, transB, ldb, ldb_hi, b_rdiv, beta,
                 C, ldc, bias, epilogue, aux, ldaux, workspace, splits, asum_out, asum_out2, asum_beta, counters,
                 stream);
}

// bf16-operand arithmetic (mixed precision): every operand rounded to bf16 (RNE) as it is staged,
// one v_mfma_f32_32x32x16_bf16 per block, fp32 accumulation and fp32 output / epilogue.  Same
// arguments as mrg_gemm_f32_ex.  Few-row products (M <= 64) stay on the exact-f32 register kernel.
MRG_API int mrg_gemm_bf16_ex(int M, int N, int K, float alpha,
                             const float* A, int transA, long lda, long lda_hi, int a_rdiv,
                             const float* B, int transB, long ldb, long ldb_hi, int b_rdiv,
                             float beta, float* C, long ldc, const float* bias, int epilogue,
                             const float* aux, long ldaux, float* workspace, int splits,
                             float* asum_out, float* asum_out2, float asum_beta,
                             unsigned* counters, hipStream_t stream) {
  return gemm_ex(2, M, N, K, alpha, A, transA, lda, lda_hi, a_rdiv, B, transB, ldb, ldb_hi, b_rdiv, beta,
                 C, ldc, bias, epilogue, aux, ldaux, workspace, splits, asum_out, asum_out2, asum_beta, counters,
                 stream);
}

// n same-shape k-contiguous products in ONE launch (the encoder stack's per-diagonal chunk products,
// encoder_stack.py): C_p = alpha A_p B_p^T + beta C_p + bias_p (epilogue with aux_p), A_p [M][K] rows
// of stride lda, B_p [N][K] rows of stride ldb, p < n <= 16; bias / aux arrays nullable.  The
// LDS-DMA x6 kernel walks the n x tiles grid (bf16 = 1: one bf16 plane, the "bf16" precision);
// shapes or modes outside it run the products one by one through mrg_gemm_f32_ex's dispatch.
MRG_API int mrg_gemm_x6g_batched(int n, int M, int N, int K, float alpha, const float* const* A, long lda,
                                 const float* const* B, long ldb, float beta, float* const* C, long ldc,
                                 const float* const* bias, int epilogue, const float* const* aux, long ldaux,
                                 int bf16, hipStream_t stream) {
  MRG_REQUIRE(n >= 0 && n <= MRG_GB_MAX, "mrg_gemm_x6g_batched: n %d out of range", n);
  MRG_REQUIRE(epilogue >= 0 && epilogue <= 3 && (epilogue < 2 || aux), "mrg_gemm_x6g_batched: bad epilogue");
  if (n == 0 || M == 0 || N == 0) return 0;
  const int mode = bf16 ? 2 : g_gemm_mode;
  uintptr_t al = 0;
  for (int p = 0; p < n; ++p)
    al |= (uintptr_t)A[p] | (uintptr_t)B[p] | (uintptr_t)C[p] | (uintptr_t)(bias ? bias[p] : nullptr) |
          (uintptr_t)(aux ? aux[p] : nullptr);
  const bool ok = mode != 0 && g_glds > 0 && K > 0 && (K % 32) == 0 && (al & 15) == 0 && (lda & 3) == 0 &&
                  (ldb & 3) == 0 && (ldc & 3) == 0 && (!aux || (ldaux & 3) == 0) && M >= 2048 && N >= 256;
  if (!ok) {
    for (int p = 0; p < n; ++p)
      if (int e = gemm_ex(mode, M, N, K, alpha, A[p], 0, lda, 0, 0, B[p], 1, ldb, 0, 0, beta, C[p], ldc,
                          bias ? bias[p] : nullptr, epilogue, aux ? aux[p] : nullptr, ldaux, nullptr, 1, nullptr,
                          nullptr, 0.0f, nullptr, stream))
        return e;
    return 0;
  }
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta;
  a.A = A[0]; a.amap = RowMap{lda, 0, 0}; a.transA = 0;
  a.B = B[0]; a.bmap = RowMap{ldb, 0, 0}; a.transB = 1;
  a.C = C[0]; a.ldc = ldc; a.bias = bias ? bias[0] : nullptr; a.epi = epilogue;
  a.aux = aux ? aux[0] : nullptr; a.ldaux = ldaux;
  a.kchunk = K; a.nsplit = 1; a.vec = 1;
  GemmBatch gb;
  memset(&gb, 0, sizeof(gb));
  gb.n = n;
  for (int p = 0; p < n; ++p) {
    gb.A[p] = A[p]; gb.B[p] = B[p]; gb.C[p] = C[p];
    gb.bias[p] = bias ? bias[p] : nullptr;
    gb.aux[p] = aux ? aux[p] : nullptr;
  }
  int bm = 64, bn = 128;  // gemm_ex's shape rule for this kernel
  if (N >= 1024) bm = 128;
  else if (N == 256 && K <= 256) bn = 64;
  if (g_glds_bn == 64) bn = 64;
  launch_x6g(a, g_glds, bm, bn, stream, mode == 2 ? 1 : 3, &gb);
  return check_launch("gemm_x6g_kernel (batched)");
}

MRG_API int mrg_gemm_f32(int M, int N, int K, float alpha,
                         const float* A, int transA, long lda, long lda_hi, int a_rdiv,
                         const float* B, int transB, long ldb, long ldb_hi, int b_rdiv,
                         float beta, float* C, long ldc, const float* bias, int epilogue,
                         const float* aux, long ldaux, float* workspace, int splits,
                         hipStream_t stream) {
  return mrg_gemm_f32_ex(M, N, K, alpha, A, transA, lda, lda_hi, a_rdiv, B, transB, ldb, ldb_hi, b_rdiv, beta, C,
                         ldc, bias, epilogue, aux, ldaux, workspace, splits, nullptr, nullptr, 0.0f, nullptr,
                         stream);
}

static int colsum_splits(int rows) {
  int s = (rows + 63) / 64;  // 64 rows per stage-1 block
  return s < 1 ? 1 : (s > 512 ? 512 : s);
}

MRG_API size_t mrg_colsum_workspace_bytes(int rows, int N) {
  return (size_t)colsum_splits(rows) * N * sizeof(float);
}

// out[n] = beta*out[n] + sum_rows X(row, n)   (bias gradients; out2 optional mirror for b_hh)
MRG_API int mrg_colsum_f32(int rows, int N, const float* X, long ld, long ld_hi, int rdiv,
                           float beta, float* out, float* out2, float* workspace,
                           hipStream_t stream) {
  if (N == 0) return 0;
  int S = colsum_splits(rows);
  int rows_per = (rows + S - 1) / S;
  if (rows_per == 0) rows_per = 1;
  dim3 grid((N + 63) / 64, S);
  klaunch(colsum_partial_kernel, grid, 256, 0, stream, X, RowMap{ld, ld_hi, rdiv}, rows, N, rows_per, workspace);
  if (check_launch("colsum_partial_kernel")) return 1;
  klaunch(colsum_final_kernel, (N + 63) / 64, 1024, 0, stream, workspace, S, N, beta, out, out2);
  return check_launch("colsum_final_kernel");
}
