// x6 GEMM with LDS-DMA staging (gfx950 global_load_lds_dwordx4): see the comment below.
#include "gemm_common.h"
#include <cstdlib>

namespace mrg {


// ----------------------------------------------------------------------------------------------
// x6 GEMM with LDS-DMA staging for k-contiguous operands (transA = 0, transB = 1: X W^T, and dY W
// through a transposed weight copy).  The register-staged kernel above keeps ONE k-tile of loads
// in flight per workgroup; on the step's short-K products (K = 256..1024, 300..1200 tiles, about
// one workgroup per CU) each k-tile then waits out a full HBM round trip (33 us for a
// 19200 x 256 x 256 product whose MFMA work is ~6 us).  Here the fp32 tiles arrive by
// global_load_lds_dwordx4 into an NS-deep LDS ring (no VGPRs held by loads in flight), NS - 1
// k-tiles ahead, and each wave splits its own fragments into the three bf16 planes as it reads
// them (cdna_hip_programming.md §5, "Async global->LDS copy", "Pipelining across barriers").
//   ring slot: A [BM rows][32 k] fp32 then B [BN rows][32 k] fp32, 128-B rows in 1-KB groups of 8;
//   a DMA wave-instruction fills one group lane-linearly: lane L -> row 8g + L/8, 16-B slot L%8,
//   which holds k-chunk (L%8) ^ f(row), f(row) = (row >> 1) & 7 (source-address swizzle; the
//   fragment reads apply the same XOR: 16 lanes reading rows r0..r0+15 at one chunk hit 16
//   distinct 16-B bank groups).
//   per k-tile: counted s_waitcnt vmcnt (the later stages stay in flight) -> raw s_barrier ->
//   issue k-tile kt + NS - 1 into the slot read in the previous k-tile -> fragments, split, MFMAs.
__device__ __forceinline__ int glds_off(int row, int c) {
  return ((row >> 3) << 10) + ((row & 7) << 7) + ((c ^ ((row >> 1) & 7)) << 4);
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

typedef float f32x4v_ __attribute__((ext_vector_type(4)));

// 16-B LDS read the compiler does not track (see gemm_x6g_kernel); the caller waits lgkmcnt
__device__ __forceinline__ f32x4v_ lds_read16(unsigned addr) {
  f32x4v_ v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// 4-B LDS read the compiler does not track (see gemm_x6g_kernel); the caller waits lgkmcnt
__device__ __forceinline__ float lds_read4(unsigned addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// 8 ds_read_b32 at addr + (K0 + j) * ROWB, j = 0..7 (immediate offsets: one address register for the
// eight k-rows of a weight-gradient fragment); the caller waits lgkmcnt
template <int ROWB, int K0>
__device__ __forceinline__ void lds_read8k(unsigned addr, float (&v)[8]) {
  asm volatile(
      "ds_read_b32 %0, %8 offset:%9\n\t"
      "ds_read_b32 %1, %8 offset:%10\n\t"
      "ds_read_b32 %2, %8 offset:%11\n\t"
      "ds_read_b32 %3, %8 offset:%12\n\t"
      "ds_read_b32 %4, %8 offset:%13\n\t"
      "ds_read_b32 %5, %8 offset:%14\n\t"
      "ds_read_b32 %6, %8 offset:%15\n\t"
      "ds_read_b32 %7, %8 offset:%16"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(addr), "n"(K0 * ROWB), "n"((K0 + 1) * ROWB), "n"((K0 + 2) * ROWB), "n"((K0 + 3) * ROWB),
        "n"((K0 + 4) * ROWB), "n"((K0 + 5) * ROWB), "n"((K0 + 6) * ROWB), "n"((K0 + 7) * ROWB)
      : "memory");
}

// 8 consecutive-k fp32 -> three bf16x8 planes (v = p0 + p1 + p2 + r, |r| <= 2^-24 |v|)
__device__ __forceinline__ void split8(f32x4v_ v0, f32x4v_ v1, bf16x8 (&f)[3]) {
  unsigned a0, a1, a2, b0, b1, b2, c0, c1, c2, d0, d1, d2;
  split2(v0.x, v0.y, a0, a1, a2);
  split2(v0.z, v0.w, b0, b1, b2);
  split2(v1.x, v1.y, c0, c1, c2);
  split2(v1.z, v1.w, d0, d1, d2);
  const u32x4 p0 = {a0, b0, c0, d0}, p1 = {a1, b1, c1, d1}, p2 = {a2, b2, c2, d2};
  f[0] = __builtin_bit_cast(bf16x8, p0);
  f[1] = __builtin_bit_cast(bf16x8, p1);
  f[2] = __builtin_bit_cast(bf16x8, p2);
}

// one plane: 8 consecutive-k fp32 -> bf16x8 (RNE), the bf16-operand arithmetic (precision "bf16")
__device__ __forceinline__ bf16x8 cvt8(f32x4v_ v0, f32x4v_ v1) {
  const u32x4 p = {pk_bf16(v0.x, v0.y), pk_bf16(v0.z, v0.w), pk_bf16(v1.x, v1.y), pk_bf16(v1.z, v1.w)};
  return __builtin_bit_cast(bf16x8, p);
}

// NP = 3: the x6 split (fp32-class, six MFMAs per block); NP = 1: bf16 operands, one MFMA per block
template <int NP>
__device__ __forceinline__ void planes8(f32x4v_ v0, f32x4v_ v1, bf16x8 (&f)[NP]) {
  if constexpr (NP == 3) split8(v0, v1, f);
  else f[0] = cvt8(v0, v1);
}

template <int NP>
__device__ __forceinline__ f32x16 mfma_planes(const bf16x8 (&b)[NP], const bf16x8 (&a)[NP], f32x16 acc) {
  if constexpr (NP == 3) {  // small terms first; (B, A) operand order -> C^T per lane
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[2], a[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[1], a[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[0], a[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[1], a[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[0], a[1], acc, 0, 0, 0);
  }
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[0], a[0], acc, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// PB = 1: the B operand arrives pre-split, as three bf16 planes [3][N][ldb] (plane stride bplane
// elements; mrg_split_planes_batched makes them once per optimizer step for every weight), so only
// A is split in the loop (half the VALU of the split; the B fragments are three ds_read_b128).
// B plane rows are 64 B per k-tile: one DMA wave-instruction fills 16 rows (lane L -> row 16g + L/4,
// 16-B slot L%4 holding 8-k chunk (L%4) ^ ((row >> 2) & 3)).
template <int BM, int BN, int NS, int PB, int NP = 3>
__global__ __launch_bounds__(NT, 1) void gemm_x6g_kernel(GemmArgs a_in, long bplane, GemmBatch gb) {
  static_assert(NP == 3 || (NP == 1 && PB == 0), "gemm_x6g: one-plane form has no pre-split B");
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int SA = BM * 128;                                   // A: [BM][32] fp32
  constexpr int SBP = BN * 64;                                   // one B plane: [BN][32] bf16
  constexpr int SS = SA + (PB ? 3 * SBP : BN * 128);             // bytes of one ring slot
  constexpr int GA = BM / 32;                                    // DMA wave-instructions per wave per k-tile
  constexpr int GB = PB ? 3 * BN / 64 : BN / 32;
  constexpr int GT = GA + GB;
  static_assert(NS >= 2 && NS <= 4 && (BM == 64 || BM == 128) && (BN == 64 || BN == 128), "gemm_x6g tile");
  __shared__ __attribute__((aligned(16))) unsigned char lds[NS * SS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);
  const int lr = lane & 31, lh = lane >> 5;
  // XCD-aware bijective remap: the blocks that share an XCD (b % 8) take consecutive tiles, so the
  // column tiles of one row block (the same A rows) meet in one L2
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  // batched form (gb.n problems of one shape, mrg_gemm_x6g_batched): the grid covers n x tiles_mn
  // tiles, problem-major, so an XCD's consecutive tiles stay within one problem
  GemmArgs a = a_in;
  if (gb.n > 0) {
    const int p = t / a.tiles_mn;
    t -= p * a.tiles_mn;
    a.A = gb.A[p]; a.B = gb.B[p]; a.C = gb.C[p]; a.bias = gb.bias[p]; a.aux = gb.aux[p];
  }
  const int m0 = (t / a.tiles_n) * BM, n0 = (t % a.tiles_n) * BN;
  const int nk = a.K / 32;

  // per-lane DMA source (bytes) and LDS destination offset of each wave-instruction of a k-tile
  const unsigned char* src[GT];
  int dsto[GT];
#pragma unroll
  for (int g = 0; g < GT; ++g) {
    if (g < GA) {
      const int grp = wave * GA + g;
      const int row = 8 * grp + (lane >> 3);
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      src[g] = reinterpret_cast<const unsigned char*>(a.A + a.amap.off(min(m0 + row, a.M - 1)) + 4 * chunk);
      dsto[g] = grp << 10;
    } else if (!PB) {
      const int grp = wave * GB + (g - GA);
      const int row = 8 * grp + (lane >> 3);
      const int chunk = (lane & 7) ^ ((row >> 1) & 7);
      src[g] = reinterpret_cast<const unsigned char*>(a.B + a.bmap.off(min(n0 + row, a.N - 1)) + 4 * chunk);
      dsto[g] = SA + (grp << 10);
    } else {
      const int G = wave * GB + (g - GA), p = G / (BN / 16), grp = G % (BN / 16);
      const int row = 16 * grp + (lane >> 2);
      const int chunk = (lane & 3) ^ ((row >> 2) & 3);
      const __bf16* pb = reinterpret_cast<const __bf16*>(a.B) + p * bplane;
      src[g] = reinterpret_cast<const unsigned char*>(pb + (long)min(n0 + row, a.N - 1) * a.bmap.ld_lo + 8 * chunk);
      dsto[g] = SA + p * SBP + (grp << 10);
    }
  }
  const unsigned lds_base = (unsigned)(uintptr_t)((__attribute__((address_space(3))) unsigned char*)lds);
  auto issue = [&](int kt, int slot) {
#pragma unroll
    for (int g = 0; g < GT; ++g) {
      const int adv = (g < GA || !PB) ? 128 : 64;  // bytes per k-tile along a row
      __builtin_amdgcn_global_load_lds((const void*)(src[g] + (long)kt * adv),
                                       (__attribute__((address_space(3))) void*)(lds + slot * SS + dsto[g]), 16, 0,
                                       0);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

#pragma unroll
  for (int st = 0; st < NS - 1; ++st)
    if (st < nk) issue(st, st);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(NS - 2, nk - 1 - kt);  // k-tiles issued after kt, left in flight
    if (ahead >= 2) vm_wait<2 * GT>();
    else if (ahead == 1) vm_wait<GT>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + NS - 1 < nk) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const unsigned sa = lds_base + (kt % NS) * SS;
    const unsigned sb = sa + SA;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c0 = 4 * s + 2 * lh;
      // fragment reads in inline asm: hipcc would put s_waitcnt vmcnt(0) before any ds_read it
      // sees while an LDS-DMA is in flight (draining the ring every k-tile); the counted vmcnt and
      // the barrier above already order these reads after the DMA of this k-tile
      f32x4v_ ra[TM][2], rb[TN][2];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm + 32 * i + lr;
        ra[i][0] = lds_read16(sa + glds_off(row, c0));
        ra[i][1] = lds_read16(sa + glds_off(row, c0 + 1));
      }
      f32x4v_ rp[TN][3];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn + 32 * j + lr;
        if (PB) {
          const int c = 2 * s + lh;
#pragma unroll
          for (int p = 0; p < 3; ++p) rp[j][p] = lds_read16(sb + p * SBP + row * 64 + ((c ^ ((row >> 2) & 3)) << 4));
        } else {
          rb[j][0] = lds_read16(sb + glds_off(row, c0));
          rb[j][1] = lds_read16(sb + glds_off(row, c0 + 1));
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 fa[TM][NP], fb[TN][NP];
#pragma unroll
      for (int i = 0; i < TM; ++i) planes8<NP>(ra[i][0], ra[i][1], fa[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (PB) {
#pragma unroll
          for (int p = 0; p < 3; ++p) fb[j][p] = __builtin_bit_cast(bf16x8, rp[j][p]);
        } else {
          planes8<NP>(rb[j][0], rb[j][1], fb[j]);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_planes<NP>(fb[j], fa[i], acc[i][j]);
    }
  }
  __syncthreads();  // every wave's last fragment reads are done: the ring becomes the epilogue stage
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

template <int BM, int BN, int PB, int NP>
static void launch_tiles(GemmArgs a, int ns, long bplane, hipStream_t s, const GemmBatch& gb) {
  a.tiles_n = (a.N + BN - 1) / BN;
  a.tiles_mn = a.tiles_n * ((a.M + BM - 1) / BM);
  a.ntiles = a.tiles_mn;
  a.nsplit = 1;
  a.ws = nullptr;
  const unsigned grid = (unsigned)a.tiles_mn * (unsigned)(gb.n > 0 ? gb.n : 1);
  if constexpr (NP == 1) {  // one-plane form: ring depth 2 only
    klaunch(gemm_x6g_kernel<BM, BN, 2, 0, 1>, grid, NT, 0, s, a, bplane, gb);
    return;
  }
  switch (ns) {
    case 2: klaunch(gemm_x6g_kernel<BM, BN, 2, PB>, grid, NT, 0, s, a, bplane, gb); break;
    case 4: klaunch(gemm_x6g_kernel<BM, BN, 4, PB>, grid, NT, 0, s, a, bplane, gb); break;
    default: klaunch(gemm_x6g_kernel<BM, BN, 3, PB>, grid, NT, 0, s, a, bplane, gb); break;
  }
}

template <int PB, int NP = 3>
static void launch_shape(GemmArgs a, int ns, int bm, int bn, long bplane, hipStream_t s, const GemmBatch& gb) {
  if (bm == 64) {
    if (bn == 64) launch_tiles<64, 64, PB, NP>(a, ns, bplane, s, gb);
    else launch_tiles<64, 128, PB, NP>(a, ns, bplane, s, gb);
  } else if (bn == 64) {
    launch_tiles<128, 64, PB, NP>(a, ns, bplane, s, gb);
  } else {
    launch_tiles<128, 128, PB, NP>(a, ns, bplane, s, gb);
  }
}

void launch_x6g(GemmArgs a, int ns, int bm, int bn, hipStream_t s, int planes, const GemmBatch* gb) {
  GemmBatch none;
  none.n = 0;
  const GemmBatch& b = gb ? *gb : none;
  if (planes == 1) launch_shape<0, 1>(a, 2, bm, bn, 0, s, b);
  else launch_shape<0>(a, ns, bm, bn, 0, s, b);
}


// ----------------------------------------------------------------------------------------------
// Weight-gradient form (transA = 1, transB = 0): C[m][n] = sum_k A[k][m] B[k][n] over the B*T rows
// k (dW = dY^T X), split over K (fp32 slabs, ordered reduce) and with the bias gradient (row sums
// of A over k) fused.  Both operands are k-strided: a ring slot holds A [32 k][BM] and B [32 k][BN]
// fp32 rows as they lie in memory (one DMA wave-instruction = 1 KB = 1024 / (4 X) k-rows), and a
// fragment (8 consecutive k of one m) is 8 ds_read_b32; the 16-B chunk of row k sits at chunk
// c ^ 8 ((k >> 3) & 1) (source swizzle), so the two half-waves (rows k and k + 8) hit opposite
// bank halves.  K % 32 == 0 and M, N multiples of 4 (clamped chunk reads past the tile edge).
template <int X>
__device__ __forceinline__ int wg_off(int k, int c) {  // byte offset of chunk c of k-row k, X floats per row
  return k * X * 4 + ((c ^ (((k >> 3) & 1) << 3)) << 4);
}

// one (tile, K slice) of the weight-gradient product; lds = the kernel's ring
template <int BM, int BN, int NS, int NP>
__device__ __forceinline__ void wgrad_tile(const GemmArgs& a, int t, unsigned char* lds) {
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int SA = 32 * BM * 4, SS = SA + 32 * BN * 4;
  constexpr int GA = SA / 4096, GB = (32 * BN * 4) / 4096;  // 1-KB DMA instructions per wave per k-tile
  constexpr int GT = GA + GB;
  constexpr int RA = 1024 / (BM * 4), RB = 1024 / (BN * 4);  // k-rows per DMA instruction
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * (BM / 2), wn = (wave & 1) * (BN / 2);
  const int lr = lane & 31, lh = lane >> 5;
  const int z = t / a.tiles_mn, tr = t - z * a.tiles_mn;
  const int m0 = (tr / a.tiles_n) * BM, n0 = (tr % a.tiles_n) * BN;
  const int kbeg = z * a.kchunk, kend = min(a.K, kbeg + a.kchunk);
  const int nk = (kend - kbeg) / 32;

  const float* src[GT];
  long rstep[GT];  // not used: rows advance through the RowMap per k-tile
  int kk[GT], dsto[GT];
#pragma unroll
  for (int g = 0; g < GT; ++g) {
    if (g < GA) {
      const int grp = wave * GA + g, k = grp * RA + lane / (BM / 4), c = lane % (BM / 4);
      const int chunk = c ^ (((k >> 3) & 1) << 3);
      src[g] = a.A + min(m0 + 4 * chunk, a.M - 4);
      kk[g] = k;
      dsto[g] = grp << 10;
    } else {
      const int grp = wave * GB + (g - GA), k = grp * RB + lane / (BN / 4), c = lane % (BN / 4);
      const int chunk = c ^ (((k >> 3) & 1) << 3);
      src[g] = a.B + min(n0 + 4 * chunk, a.N - 4);
      kk[g] = k;
      dsto[g] = SA + (grp << 10);
    }
    rstep[g] = 0;
  }
  (void)rstep;
  auto issue = [&](int kt, int slot) {
#pragma unroll
    for (int g = 0; g < GT; ++g) {
      const int k = kbeg + kt * 32 + kk[g];
      const float* p = src[g] + (g < GA ? a.amap.off(k) : a.bmap.off(k));
      __builtin_amdgcn_global_load_lds((const void*)p, (__attribute__((address_space(3))) void*)(lds + slot * SS + dsto[g]),
                                       16, 0, 0);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  const bool do_asum = a.asum && n0 == 0 && (wave & 1) == 0;
  float cs[TM] = {};
  const unsigned lds_base = (unsigned)(uintptr_t)((__attribute__((address_space(3))) unsigned char*)lds);
  // a fragment's k-rows 16 s + 8 lh + j share the chunk swizzle of row 8 lh ((k >> 3) & 1 = lh), so
  // each fragment is one lane address (k-row 8 lh) plus immediate row offsets
  unsigned oa[TM], ob[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = wm + 32 * i + lr;
    oa[i] = wg_off<BM>(8 * lh, m >> 2) + 4 * (m & 3);
  }
#pragma unroll
  for (int jj = 0; jj < TN; ++jj) {
    const int n = wn + 32 * jj + lr;
    ob[jj] = SA + wg_off<BN>(8 * lh, n >> 2) + 4 * (n & 3);
  }

#pragma unroll
  for (int st = 0; st < NS - 1; ++st)
    if (st < nk) issue(st, st);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(NS - 2, nk - 1 - kt);
    if (ahead >= 2) vm_wait<2 * GT>();
    else if (ahead == 1) vm_wait<GT>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + NS - 1 < nk) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const unsigned sa = lds_base + (kt % NS) * SS;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float va[TM][8], vb[TN][8];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (s == 0) lds_read8k<BM * 4, 0>(sa + oa[i], va[i]);
        else lds_read8k<BM * 4, 16>(sa + oa[i], va[i]);
      }
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) {
        if (s == 0) lds_read8k<BN * 4, 0>(sa + ob[jj], vb[jj]);
        else lds_read8k<BN * 4, 16>(sa + ob[jj], vb[jj]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 fa[TM][NP], fb[TN][NP];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (do_asum)
          cs[i] += ((va[i][0] + va[i][1]) + (va[i][2] + va[i][3])) + ((va[i][4] + va[i][5]) + (va[i][6] + va[i][7]));
        planes8<NP>(f32x4v_{va[i][0], va[i][1], va[i][2], va[i][3]}, f32x4v_{va[i][4], va[i][5], va[i][6], va[i][7]},
                    fa[i]);
      }
#pragma unroll
      for (int jj = 0; jj < TN; ++jj)
        planes8<NP>(f32x4v_{vb[jj][0], vb[jj][1], vb[jj][2], vb[jj][3]},
                    f32x4v_{vb[jj][4], vb[jj][5], vb[jj][6], vb[jj][7]}, fb[jj]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_planes<NP>(fb[j], fa[i], acc[i][j]);
    }
  }
  if (do_asum) {  // lanes l and l + 32 hold the two k halves of row m = wm + 32 i + (l & 31)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float v = cs[i] + __shfl_xor(cs[i], 32, 64);
      const int m = m0 + wm + 32 * i + lr;
      if (lh == 0 && m < a.M) a.asum[(long)z * a.M + m] = v;
    }
  }
  __syncthreads();
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
        if (m < a.M) store4(a, z, m, n0 + wn + 4 * c4, v);
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
          if (m < a.M) store4(a, z, m, n, v);
        }
    }
  }
}

// Weight-gradient kernel: (tile, K slice) work items t < a.ntiles; grid = ntiles, or fewer blocks
// that walk the items in strides of the grid (a capped grid: one block per CU beside a recurrence,
// mrg_gemm_set_blocks_per_cu).  XCD-aware bijective item order either way (a multiple-of-8 grid keeps
// a block on one XCD's items).
template <int BM, int BN, int NS, int NP = 3>
__global__ __launch_bounds__(NT, 1) void gemm_x6g_wgrad_kernel(GemmArgs a) {
  constexpr int SS = 32 * BM * 4 + 32 * BN * 4;
  static_assert(NS >= 2 && NS <= 4 && (BM == 64 || BM == 128) && (BN == 64 || BN == 128), "wgrad tile");
  __shared__ __attribute__((aligned(16))) unsigned char lds[NS * SS];
  const int total = a.ntiles, q8 = total >> 3, r8 = total & 7;
  for (int vb = blockIdx.x; vb < total; vb += gridDim.x) {
    const int xcd = vb & 7;
    const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (vb >> 3);
    wgrad_tile<BM, BN, NS, NP>(a, t, lds);
    __syncthreads();  // the ring / epilogue stage is reused by the next item
  }
}

void launch_x6g_wgrad(GemmArgs a, int splits, int bm, int bn, hipStream_t s, int planes, int max_grid) {
  auto go = [&](auto kern, int BM_, int BN_) {
    a.tiles_n = (a.N + BN_ - 1) / BN_;
    a.tiles_mn = a.tiles_n * ((a.M + BM_ - 1) / BM_);
    a.ntiles = a.tiles_mn * splits;
    a.nsplit = splits;
    unsigned grid = (unsigned)a.ntiles;
    if (max_grid > 0 && grid > (unsigned)max_grid) grid = (unsigned)max_grid & ~7u ? (unsigned)max_grid & ~7u : 8u;
    klaunch(kern, grid, NT, 0, s, a);
  };
  if (planes == 1) go(gemm_x6g_wgrad_kernel<128, 128, 2, 1>, 128, 128);
  else if (bm == 64 && bn == 64) go(gemm_x6g_wgrad_kernel<64, 64, 2>, 64, 64);
  else if (bm == 64) go(gemm_x6g_wgrad_kernel<64, 128, 2>, 64, 128);
  else if (bn == 64) go(gemm_x6g_wgrad_kernel<128, 64, 2>, 128, 64);
  else go(gemm_x6g_wgrad_kernel<128, 128, 2>, 128, 128);
}

// ----------------------------------------------------------------------------------------------
// Batched transpose: dst_i [cols_i][rows_i] = src_i [rows_i][cols_i]^T for up to MRG_TP_MAX
// matrices in one launch (the weights' [in][out] copies that let the input-gradient products
// dY W run as k-contiguous products on the kernel above).  32 x 32 tiles through LDS.
__global__ __launch_bounds__(256) void transpose_batched_kernel(TransposeBatch tb) {
  __shared__ float tile[32][33];
  int blk = blockIdx.x, i = 0;
  while (i + 1 < tb.n && blk >= tb.first[i + 1]) ++i;
  const int local = blk - tb.first[i];
  const int R = tb.rows[i], C = tb.cols[i];
  const int tc = (C + 31) / 32;
  const int r0 = (local / tc) * 32, c0 = (local % tc) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const float* src = tb.src[i];
  float* dst = tb.dst[i];
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int r = r0 + ty + k, c = c0 + tx;
    if (r < R && c < C) tile[ty + k][tx] = src[(long)r * C + c];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int c = c0 + ty + k, r = r0 + tx;
    if (r < R && c < C) dst[(long)c * R + r] = tile[tx][ty + k];
  }
}

}  // namespace mrg

namespace mrg {

// ----------------------------------------------------------------------------------------------
// Three bf16 planes of a weight, once per optimizer step: dst [3][R'][C'] (plane stride R' C'),
// (R', C') = (rows, cols), or (cols, rows) for the transposed copy (the input-gradient products'
// k-contiguous operand).  32 x 32 tiles through LDS; the split is the x6 one (RNE, v - v0, ...).
struct PlaneBatch {
  int n;
  const float* src[MRG_TP_MAX];
  __bf16* dst[MRG_TP_MAX];
  int rows[MRG_TP_MAX], cols[MRG_TP_MAX], tr[MRG_TP_MAX];
  int first[MRG_TP_MAX + 1];
};

__global__ __launch_bounds__(256) void split_planes_kernel(PlaneBatch pb) {
  __shared__ float tile[32][33];
  int blk = blockIdx.x, i = 0;
  while (i + 1 < pb.n && blk >= pb.first[i + 1]) ++i;
  const int local = blk - pb.first[i];
  const int R = pb.rows[i], C = pb.cols[i];
  const int tc = (C + 31) / 32;
  const int r0 = (local / tc) * 32, c0 = (local % tc) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int r = r0 + ty + k, c = c0 + tx;
    tile[ty + k][tx] = (r < R && c < C) ? pb.src[i][(long)r * C + c] : 0.0f;
  }
  __syncthreads();
  const long plane = (long)R * C;
  unsigned short* d = reinterpret_cast<unsigned short*>(pb.dst[i]);
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    // output element (orow, ocol) of the [R'][C'] image
    const int orow = (pb.tr[i] ? c0 : r0) + ty + k, ocol = (pb.tr[i] ? r0 : c0) + tx;
    const float v = pb.tr[i] ? tile[tx][ty + k] : tile[ty + k][tx];
    const int OR = pb.tr[i] ? C : R, OC = pb.tr[i] ? R : C;
    if (orow < OR && ocol < OC) {
      unsigned p0, p1, p2;
      split2(v, 0.0f, p0, p1, p2);
      const long o = (long)orow * OC + ocol;
      d[o] = (unsigned short)(p0 & 0xffffu);
      d[plane + o] = (unsigned short)(p1 & 0xffffu);
      d[2 * plane + o] = (unsigned short)(p2 & 0xffffu);
    }
  }
}

}  // namespace mrg

using namespace mrg;

static int g_wide_cfg = [] {
  const char* e = getenv("MRG_GEMM_WIDE");
  const int v = e ? atoi(e) : 12;
  return (v == 0 || v == 22) ? v : 12;
}();

// planes of n weights (see split_planes_kernel): dst_i holds 3 x rows_i x cols_i bf16
MRG_API int mrg_split_planes_batched(int n, const float* const* src, void* const* dst, const int* rows, const int* cols,
                                     const int* transpose, hipStream_t stream) {
  MRG_REQUIRE(n >= 0 && (n == 0 || (src && dst && rows && cols && transpose)), "mrg_split_planes_batched: bad arguments");
  for (int b0 = 0; b0 < n; b0 += MRG_TP_MAX) {
    PlaneBatch pb;
    memset(&pb, 0, sizeof(pb));
    pb.n = n - b0 < MRG_TP_MAX ? n - b0 : MRG_TP_MAX;
    int blocks = 0;
    for (int i = 0; i < pb.n; ++i) {
      MRG_REQUIRE(rows[b0 + i] >= 0 && cols[b0 + i] >= 0, "mrg_split_planes_batched: negative size");
      pb.src[i] = src[b0 + i]; pb.dst[i] = reinterpret_cast<__bf16*>(dst[b0 + i]);
      pb.rows[i] = rows[b0 + i]; pb.cols[i] = cols[b0 + i]; pb.tr[i] = transpose[b0 + i] ? 1 : 0;
      pb.first[i] = blocks;
      blocks += ((rows[b0 + i] + 31) / 32) * ((cols[b0 + i] + 31) / 32);
    }
    pb.first[pb.n] = blocks;
    if (blocks == 0) continue;
    klaunch(split_planes_kernel, blocks, 256, 0, stream, pb);
    if (check_launch("split_planes_kernel")) return 1;
  }
  return 0;
}

// C = epi(alpha A B^T + beta C + bias) with B given as three bf16 planes (mrg_split_planes_batched):
// B plane p row n at Bplanes + p * bplane + n * ldb (bf16 elements).  A [M][K] rows through the
// RowMap (lda, lda_hi, a_rdiv).  K % 32 == 0; rows 16-B aligned.  The LDS-DMA x6 kernel with only
// A split in the loop.
MRG_API int mrg_gemm_x6_planes(int M, int N, int K, float alpha, const float* A, long lda, long lda_hi, int a_rdiv,
                               const void* Bplanes, long ldb, long bplane, float beta, float* C, long ldc,
                               const float* bias, int epilogue, const float* aux, long ldaux, hipStream_t stream) {
  MRG_REQUIRE(M >= 0 && N >= 0 && K >= 0, "mrg_gemm_x6_planes: negative size");
  MRG_REQUIRE(K % 32 == 0, "mrg_gemm_x6_planes: K %d not a multiple of 32", K);
  MRG_REQUIRE(epilogue >= 0 && epilogue <= 3 && (epilogue < 2 || aux), "mrg_gemm_x6_planes: bad epilogue");
  MRG_REQUIRE((((uintptr_t)A) & 15) == 0 && (lda & 3) == 0 && (a_rdiv <= 0 || (lda_hi & 3) == 0),
              "mrg_gemm_x6_planes: A rows must be 16-B aligned");
  MRG_REQUIRE((((uintptr_t)Bplanes) & 15) == 0 && (ldb & 7) == 0 && (bplane & 7) == 0,
              "mrg_gemm_x6_planes: B plane rows must be 16-B aligned");
  if (M == 0 || N == 0) return 0;
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta;
  a.A = A; a.amap = RowMap{lda, lda_hi, a_rdiv}; a.transA = 0;
  a.B = reinterpret_cast<const float*>(Bplanes); a.bmap = RowMap{ldb, 0, 0}; a.transB = 1;
  a.C = C; a.ldc = ldc; a.bias = bias; a.epi = epilogue; a.aux = aux; a.ldaux = ldaux;
  a.kchunk = K;
  a.vec = ((((uintptr_t)C | (uintptr_t)bias | (uintptr_t)aux) & 15) == 0 && (ldc & 3) == 0 &&
           (!aux || (ldaux & 3) == 0)) ? 1 : 0;
  if (g_wide_cfg > 8) {   // row-owning kernel (gemm_wide.hip); cfg = 10 * bn / 64 + ns, 0 = the kernel below
    const int bn = N <= 64 ? 64 : 64 * (g_wide_cfg / 10), ns = g_wide_cfg % 10;
    launch_x6w(a, bn, ns, bplane, stream);
    return check_launch("gemm_x6w_kernel");
  }
  int bm = 64, bn = 128;  // the fp32-operand kernel's shape rule (gemm.hip)
  if (N >= 1024) bm = 128;
  else if (N <= 256 && K <= 256) bn = 64;
  GemmBatch none;
  none.n = 0;
  launch_shape<1>(a, 2, bm, bn, bplane, stream, none);
  return check_launch("gemm_x6g_kernel");
}

// n same-shape products C_p = epi(alpha A_p B_p^T + beta C_p + bias_p) in one launch, B_p as the three
// bf16 planes of a weight (same ldb / plane stride for every p): the batched projections of the encoder
// stack and of the fused integrators (encoder_stack.py, integrate.py) on the row-owning kernel.
MRG_API int mrg_gemm_x6_planes_batched(int n, int M, int N, int K, float alpha, const float* const* A, long lda,
                                       const void* const* Bplanes, long ldb, long bplane, float beta,
                                       float* const* C, long ldc, const float* const* bias, int epilogue,
                                       const float* const* aux, long ldaux, hipStream_t stream) {
  MRG_REQUIRE(n >= 1 && n <= MRG_GB_MAX && M >= 0 && N >= 0 && K >= 0 && K % 32 == 0,
              "mrg_gemm_x6_planes_batched: bad shape (n=%d, K=%d)", n, K);
  MRG_REQUIRE(epilogue >= 0 && epilogue <= 3 && (epilogue < 2 || aux), "mrg_gemm_x6_planes_batched: bad epilogue");
  MRG_REQUIRE((lda & 3) == 0 && (ldb & 7) == 0 && (bplane & 7) == 0, "mrg_gemm_x6_planes_batched: alignment");
  if (M == 0 || N == 0) return 0;
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta;
  a.amap = RowMap{lda, 0, 0}; a.transA = 0;
  a.bmap = RowMap{ldb, 0, 0}; a.transB = 1;
  a.ldc = ldc; a.epi = epilogue; a.ldaux = ldaux;
  a.kchunk = K;
  GemmBatch gb;
  memset(&gb, 0, sizeof(gb));
  gb.n = n;
  int vec = (ldc & 3) == 0 && (!aux || (ldaux & 3) == 0);
  for (int p = 0; p < n; ++p) {
    MRG_REQUIRE((((uintptr_t)A[p] | (uintptr_t)Bplanes[p]) & 15) == 0, "mrg_gemm_x6_planes_batched: unaligned operand");
    gb.A[p] = A[p]; gb.B[p] = reinterpret_cast<const float*>(Bplanes[p]); gb.C[p] = C[p];
    gb.bias[p] = bias ? bias[p] : nullptr;
    gb.aux[p] = aux ? aux[p] : nullptr;
    if ((((uintptr_t)C[p] | (uintptr_t)gb.bias[p] | (uintptr_t)gb.aux[p]) & 15) != 0) vec = 0;
  }
  a.A = gb.A[0]; a.B = gb.B[0]; a.C = gb.C[0]; a.bias = gb.bias[0]; a.aux = gb.aux[0];
  a.vec = vec;
  const int cfg = g_wide_cfg > 8 ? g_wide_cfg : 12;
  launch_x6w(a, N <= 64 ? 64 : 64 * (cfg / 10), cfg % 10, bplane, stream, &gb);
  return check_launch("gemm_x6w_kernel (batched)");
}

// Tuning: which kernel mrg_gemm_x6_planes runs (0 = gemm_x6g_kernel with pre-split B; 12 / 22 =
// gemm_x6w_kernel with 64 / 128 columns); returns the previous setting.
MRG_API int mrg_gemm_set_wide(int cfg) {
  const int prev = g_wide_cfg;
  if (cfg == 0 || cfg == 12 || cfg == 22)
    g_wide_cfg = cfg;
  return prev;
}
