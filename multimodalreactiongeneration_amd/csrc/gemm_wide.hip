// x6 GEMM on pre-split weights, row-owning waves (gfx950): C = epi(A B^T) for the step's
// activation-times-weight products (nn.Linear / LSTM input / MultiheadAttention projections:
// mixer_block.py:63-74,237-252, for_sequential.py:42-51) and their input gradients dY W (B = the
// planes of W^T), A fp32 [M][K] through a RowMap, B as the three bf16 planes of the x6 split made
// once per optimizer step (mrg_split_planes_batched), K % 32 == 0.
//
// Why a second kernel (gemm_glds.hip's gemm_x6g_kernel keeps fp32 B and 32 x 32 MFMA blocks): with
// one 32 x 32 block per wave every fragment is split for ONE block, so the split's VALU (about six
// instructions per value) outweighs the six MFMAs it feeds.  Here a wave owns 16 rows and all BN
// columns of the tile (BN / 16 blocks of v_mfma_f32_16x16x32_bf16): its A fragment (16 x 32 fp32,
// 8 values per lane) is split once per k-tile and feeds BN / 16 x 6 MFMAs, and B needs no split at
// all (its planes come from LDS, 3 ds_read_b128 per block).  The tile's rows are owned by exactly one
// wave, so no value is split twice.
//
//   ring slot (one k-tile of 32): A [64 rows][32 k] fp32 (8 KB, 128-B rows), then the three B planes
//   [BN rows][32 k] bf16 (64-B rows).  Both arrive by LDS-DMA (global_load_lds_dwordx4, lane-linear
//   1-KB pieces) with the 16-B chunk order of each row XOR-swizzled at the source, so the fragment
//   reads (16 rows x 2 chunks for A, 16 rows x 1 chunk per plane for B) are bank-conflict free under
//   ds_read_b128's lane groups: A row r chunk c at slot c ^ ga(r), ga(r) = ((r >> 1) & 1) | (((r >> 3) & 1) << 2);
//   B row n chunk c at slot c ^ gb(n), gb(n) = ((n >> 3) & 1) << 1 (found by exhaustive search over
//   the 16-lane groups).
//   per k-tile: counted vmcnt (NS - 2 later k-tiles stay in flight) -> s_barrier -> issue k-tile
//   kt + NS - 1 into the slot read in the previous k-tile -> A fragment, split -> per block: its three
//   B plane fragments (issued one block ahead) and six MFMAs.
#include "gemm_common.h"

namespace mrg {

typedef float f32x4w __attribute__((ext_vector_type(4)));
typedef unsigned u32x4w __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int wa_off(int r, int c) {  // byte offset of 16-B chunk c of A row r (128-B rows)
  return (r << 7) + ((c ^ (((r >> 1) & 1) | (((r >> 3) & 1) << 2))) << 4);
}
__device__ __forceinline__ int wb_off(int n, int c) {  // byte offset of 16-B chunk c of a B plane row n (64-B rows)
  return (n << 6) + ((c ^ (((n >> 3) & 1) << 1)) << 4);
}

__device__ __forceinline__ f32x4w wlds16(unsigned addr) {
  f32x4w v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// 8 fp32 -> three bf16x8 planes (the x6 split of gemm_common.h, RNE)
__device__ __forceinline__ void wsplit8(f32x4w v0, f32x4w v1, bf16x8 (&f)[3]) {
  unsigned a0, a1, a2, b0, b1, b2, c0, c1, c2, d0, d1, d2;
  split2(v0.x, v0.y, a0, a1, a2);
  split2(v0.z, v0.w, b0, b1, b2);
  split2(v1.x, v1.y, c0, c1, c2);
  split2(v1.z, v1.w, d0, d1, d2);
  const u32x4w p0 = {a0, b0, c0, d0}, p1 = {a1, b1, c1, d1}, p2 = {a2, b2, c2, d2};
  f[0] = __builtin_bit_cast(bf16x8, p0);
  f[1] = __builtin_bit_cast(bf16x8, p1);
  f[2] = __builtin_bit_cast(bf16x8, p2);
}

template <int N>
__device__ __forceinline__ void wvm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// six products, small terms first (A: lane l holds A[l & 15][8 (l >> 4) + j]; B: lane l holds
// B[8 (l >> 4) + j][l & 15]; D: lane l holds D[4 (l >> 4) + i][l & 15])
__device__ __forceinline__ f32x4w wmfma6(const bf16x8 (&a)[3], bf16x8 b0, bf16x8 b1, bf16x8 b2, f32x4w acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b2, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b0, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b0, acc, 0, 0, 0);
}

template <int BN, int NS>
__global__ __launch_bounds__(256, 2) void gemm_x6w_kernel(GemmArgs a_in, long bplane, GemmBatch gb) {
  constexpr int BM = 64;
  constexpr int NB = BN / 16;                 // 16 x 16 blocks per wave
  constexpr int SA = BM * 128;                // A: [64][32] fp32
  constexpr int SBP = BN * 64;                // one B plane: [BN][32] bf16
  constexpr int SS = SA + 3 * SBP;            // bytes of one ring slot
  constexpr int PA = SA / 1024, PB = 3 * SBP / 1024;   // 1-KB DMA pieces per k-tile
  static_assert(PA % 4 == 0 && PB % 4 == 0, "pieces split over 4 waves");
  constexpr int GA = PA / 4, GB = PB / 4, GT = GA + GB;  // per wave
  __shared__ __attribute__((aligned(16))) unsigned char lds[NS * SS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
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

  const unsigned char* src[GT];
  int dsto[GT];
#pragma unroll
  for (int g = 0; g < GT; ++g) {
    if (g < GA) {   // A piece: 8 rows x 128 B; lane -> row 8 grp + lane / 8, LDS slot lane % 8
      const int grp = wave * GA + g;
      const int row = 8 * grp + (lane >> 3);
      const int chunk = (lane & 7) ^ (((row >> 1) & 1) | (((row >> 3) & 1) << 2));
      src[g] = reinterpret_cast<const unsigned char*>(a.A + a.amap.off(min(m0 + row, a.M - 1)) + 4 * chunk);
      dsto[g] = grp << 10;
    } else {        // B piece: one plane, 16 rows x 64 B; lane -> row 16 grp + lane / 4, slot lane % 4
      const int G = wave * GB + (g - GA), p = G / (BN / 16), grp = G % (BN / 16);
      const int row = 16 * grp + (lane >> 2);
      const int chunk = (lane & 3) ^ (((row >> 3) & 1) << 1);
      const __bf16* pb = reinterpret_cast<const __bf16*>(a.B) + p * bplane;
      src[g] = reinterpret_cast<const unsigned char*>(pb + (long)min(n0 + row, a.N - 1) * a.bmap.ld_lo + 8 * chunk);
      dsto[g] = SA + p * SBP + (grp << 10);
    }
  }
  auto issue = [&](int kt, int slot) {
#pragma unroll
    for (int g = 0; g < GT; ++g)
      __builtin_amdgcn_global_load_lds((const void*)(src[g] + (long)kt * (g < GA ? 128 : 64)),
                                       (__attribute__((address_space(3))) void*)(lds + slot * SS + dsto[g]), 16, 0, 0);
  };
  const unsigned lds_base = (unsigned)(uintptr_t)((__attribute__((address_space(3))) unsigned char*)lds);
  const int ar = 16 * wave + (lane & 15), ac = 2 * (lane >> 4);   // A fragment row, first chunk
  const int bc = lane >> 4;                                        // B fragment chunk

  f32x4w acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = f32x4w{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int st = 0; st < NS - 1; ++st)
    if (st < nk) issue(st, st);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(NS - 2, nk - 1 - kt);
    if (ahead >= 2) wvm_wait<2 * GT>();
    else if (ahead == 1) wvm_wait<GT>();
    else wvm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + NS - 1 < nk) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const unsigned sa = lds_base + (kt % NS) * SS;
    const unsigned sb = sa + SA;
    f32x4w va0 = wlds16(sa + wa_off(ar, ac)), va1 = wlds16(sa + wa_off(ar, ac + 1));
    f32x4w vb[2][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) vb[0][p] = wlds16(sb + p * SBP + wb_off(lane & 15, bc));
    asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(va0), "+v"(va1)::"memory");
    bf16x8 fa[3];
    wsplit8(va0, va1, fa);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int cur = j & 1, nxt = cur ^ 1;
      if (j + 1 < NB) {
#pragma unroll
        for (int p = 0; p < 3; ++p) vb[nxt][p] = wlds16(sb + p * SBP + wb_off(16 * (j + 1) + (lane & 15), bc));
        asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(vb[cur][0]), "+v"(vb[cur][1]), "+v"(vb[cur][2])::"memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vb[cur][0]), "+v"(vb[cur][1]), "+v"(vb[cur][2])::"memory");
      }
      acc[j] = wmfma6(fa, __builtin_bit_cast(bf16x8, vb[cur][0]), __builtin_bit_cast(bf16x8, vb[cur][1]),
                      __builtin_bit_cast(bf16x8, vb[cur][2]), acc[j]);
    }
  }
  __syncthreads();   // every wave's fragment reads are done: the ring becomes the epilogue stage
  // epilogue: the wave's 16 x BN tile through LDS (lane l, block j: rows 4 (l >> 4) + i, column l & 15),
  // then whole 16-B row pieces through store4 (bias / beta / epilogue / split-free)
  constexpr int PITCH = BN + 4;
  float* stg = reinterpret_cast<float*>(lds) + wave * 16 * PITCH;
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) stg[(4 * (lane >> 4) + i) * PITCH + 16 * j + (lane & 15)] = acc[j][i];
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  constexpr int C4 = BN / 4;
#pragma unroll
  for (int it = 0; it < 16 * C4 / 64; ++it) {
    const int qq = lane + 64 * it, row = qq / C4, c4 = qq % C4;
    const float4 v = *reinterpret_cast<const float4*>(stg + row * PITCH + 4 * c4);
    const int m = m0 + 16 * wave + row, n = n0 + 4 * c4;
    if (m < a.M && n < a.N) store4(a, 0, m, n, v);
  }
}

// ----------------------------------------------------------------------------------------------
// B-resident form for K <= 256 (most of the step's products: K = H = 256): the grid is one
// workgroup per CU; workgroup (slice, range) holds the planes of a 64-column slice of B for the whole
// K in LDS (3 x 64 x K bf16 = 96 KB at K = 256, loaded once by LDS-DMA) and walks the 16-row blocks
// of its row range; a wave owns whole row blocks, loads their A fragments straight from memory into
// registers (a lane's 8 consecutive k are 32 contiguous bytes; no LDS for A, the next block's loads in
// flight during this block's MFMAs), splits each once and multiplies it with the 4 column blocks'
// resident planes.  The LDS-DMA ring of gemm_x6w_kernel moved B (3 x BN x 64 B per k-tile per
// 64-row tile) on every tile: ~115 MB through LDS-DMA for a 19200 x 256 x 256 product, which bounds
// it; here B crosses once per workgroup (24 MB for the whole grid).
//   B plane row n (64 B per 32 k), 16-B chunk c at n * 2K + ((c ^ (n & 15)) << 4): a fragment read
//   (16 rows at chunks 4 kt + (l >> 4)) hits 16 distinct bank quads in every ds_read_b128 lane group
//   (rows' low 4 bits XORed into the chunk; needs >= 16 chunks per row, i.e. K >= 128).
__device__ unsigned long long* g_x6r_stamps = nullptr;   // diagnostics (mrg_gemm_debug_stamps)

template <int NK, int NW, int DBG = 0>
__global__ __launch_bounds__(64 * NW, 1) void gemm_x6r_kernel(GemmArgs a, long bplane, int nslice, int nrange) {
  unsigned long long* const stamps = (blockIdx.x == 0 && (threadIdx.x & 63) == 0) ? g_x6r_stamps : nullptr;
  int nst = 0;
  auto stamp = [&]() {
    if (stamps && nst < 16) stamps[(threadIdx.x >> 6) * 16 + nst++] = __builtin_amdgcn_s_memtime();
  };
  stamp();
  constexpr int SW = 64;                        // columns per slice
  constexpr int K = 32 * NK;
  constexpr int RP = 2 * K;                     // bytes per plane row
  constexpr int PL = SW * RP;                   // bytes per plane
  constexpr int CPR = K / 8;                    // 16-B chunks per plane row
  constexpr int RPP = 64 / CPR;                 // plane rows per 1-KB DMA piece
  constexpr int NPC = 3 * PL / 1024;            // pieces
  constexpr int PITCH = SW + 4;                 // epilogue staging row pitch (floats)
  static_assert(CPR >= 16 && NPC % NW == 0, "gemm_x6r: K in {128, 256}");
  __shared__ __attribute__((aligned(16))) unsigned char lds[3 * PL + NW * 16 * PITCH * 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int slice = t % nslice, range = t / nslice;
  if (range >= nrange) return;
  const int n0 = slice * SW;
  const int mb = (a.M + 15) / 16;                                  // 16-row blocks
  const int b0 = (int)((long)mb * range / nrange), b1 = (int)((long)mb * (range + 1) / nrange);

  const int lr = lane & 15, lq = lane >> 4;
  // A streams k-tile by k-tile through a 4-slot register ring (k-tile kt of any block sits in slot kt % 4):
  // k-tile kt + PD is requested while k-tile kt multiplies (and k-tile kt + 1 is split), so the A reads
  // spread over the kernel instead of bursting at its start
  constexpr int PD = 4;
  f32x4w ar[4][2];
  auto load_a = [&](int blk, int kt) {
    const float* ap = a.A + a.amap.off(min(16 * blk + lr, a.M - 1)) + 8 * lq + 32 * kt;
    ar[kt & 3][0] = *reinterpret_cast<const f32x4w*>(ap);
    ar[kt & 3][1] = *reinterpret_cast<const f32x4w*>(ap + 4);
  };
  if (b0 + wave < b1) {   // the first block's first k-tiles travel while the B slice loads
#pragma unroll
    for (int kt = 0; kt < PD; ++kt) load_a(b0 + wave, kt);
  }
  // B slice planes -> LDS (every wave its share of the pieces)
  {
    const __bf16* pb = reinterpret_cast<const __bf16*>(a.B);
#pragma unroll
    for (int i = 0; i < NPC / NW; ++i) {
      const int pc = wave * (NPC / NW) + i;
      const int p = pc / (PL / 1024), pr = pc % (PL / 1024);
      const int row = pr * RPP + lane / CPR, slot = lane % CPR, chunk = slot ^ (row & 15);
      const __bf16* s = pb + p * bplane + (long)min(n0 + row, a.N - 1) * a.bmap.ld_lo + 8 * chunk;
      __builtin_amdgcn_global_load_lds((const void*)s,
                                       (__attribute__((address_space(3))) void*)(lds + p * PL + pc % (PL / 1024) * 1024),
                                       16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp();

  float* stg = reinterpret_cast<float*>(lds + 3 * PL) + wave * 16 * PITCH;
  const unsigned lds_base = (unsigned)(uintptr_t)((__attribute__((address_space(3))) unsigned char*)lds);
  // B fragment addresses: lane row lr of column block j, chunk 4 kt + lq swizzled by lr; the plane and
  // column-block parts are constant offsets, so a k-tile's 12 reads share one per-lane address
  unsigned xo[NK];
#pragma unroll
  for (int kt = 0; kt < NK; ++kt) xo[kt] = lds_base + lr * RP + (((4 * kt + lq) ^ lr) << 4);
  // three plane fragments of column block j at k-tile kt (untracked reads: the caller waits)
  auto read_b = [&](int kt, int j, f32x4w (&r)[3]) {
    if constexpr (DBG == 3) {   // timing only: no B fragment reads
      r[0] = r[1] = r[2] = f32x4w{(float)kt, (float)j, 1.f, 2.f};
      return;
    }
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const unsigned addr = xo[kt] + p * PL + 16 * j * RP;
      asm volatile("ds_read_b128 %0, %1" : "=v"(r[p]) : "v"(addr) : "memory");
    }
  };
  auto block = [&](int blk, int nb) {
    stamp();
    f32x4w acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4w{0.f, 0.f, 0.f, 0.f};
    // reads run RD (k-tile, column block) steps ahead of the MFMAs through a ring of RD + 1 fragment sets;
    // the A split of k-tile kt + 1 is formed during k-tile kt's products
    constexpr int RD = 3, NSTEP = 4 * NK;
    f32x4w rb[RD + 1][3];
#pragma unroll
    for (int q = 0; q < RD; ++q) read_b(q >> 2, q & 3, rb[q]);
    bf16x8 fa[2][3];
    wsplit8(ar[0][0], ar[0][1], fa[0]);
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
      const int kt = st >> 2, j = st & 3;
      if (st + RD < NSTEP) {
        read_b((st + RD) >> 2, (st + RD) & 3, rb[(st + RD) % (RD + 1)]);
        asm volatile("s_waitcnt lgkmcnt(9)" : "+v"(rb[st % (RD + 1)][0]), "+v"(rb[st % (RD + 1)][1]),
                     "+v"(rb[st % (RD + 1)][2])::"memory");
      } else if (st + 2 < NSTEP) {
        asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(rb[st % (RD + 1)][0]), "+v"(rb[st % (RD + 1)][1]),
                     "+v"(rb[st % (RD + 1)][2])::"memory");
      } else if (st + 1 < NSTEP) {
        asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(rb[st % (RD + 1)][0]), "+v"(rb[st % (RD + 1)][1]),
                     "+v"(rb[st % (RD + 1)][2])::"memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rb[st % (RD + 1)][0]), "+v"(rb[st % (RD + 1)][1]),
                     "+v"(rb[st % (RD + 1)][2])::"memory");
      }
      if (j == 1) {   // next k-tile's A: prefetch PD + 1 ahead, split it while this k-tile multiplies
        const int kp = kt + PD;   // into the slot of k-tile kt, split one k-tile ago
        if (kp < NK) load_a(blk, kp);
        else if (nb >= 0) load_a(nb, kp - NK);
        if (kt + 1 < NK) {
          if constexpr (DBG == 2) {
            fa[(kt + 1) & 1][0] = __builtin_bit_cast(bf16x8, ar[(kt + 1) & 3][0]);
            fa[(kt + 1) & 1][1] = __builtin_bit_cast(bf16x8, ar[(kt + 1) & 3][1]);
            fa[(kt + 1) & 1][2] = fa[(kt + 1) & 1][0];
          } else {
            wsplit8(ar[(kt + 1) & 3][0], ar[(kt + 1) & 3][1], fa[(kt + 1) & 1]);
          }
        }
      }
      if constexpr (DBG == 4) {   // timing only: no MFMA
        acc[j] += rb[st % (RD + 1)][0] + rb[st % (RD + 1)][1] + rb[st % (RD + 1)][2];
        continue;
      }
      acc[j] = wmfma6(fa[kt & 1], __builtin_bit_cast(bf16x8, rb[st % (RD + 1)][0]),
                      __builtin_bit_cast(bf16x8, rb[st % (RD + 1)][1]), __builtin_bit_cast(bf16x8, rb[st % (RD + 1)][2]),
                      acc[j]);
    }
    // epilogue: 16 x 64 through the wave's staging rows, then 16-B row pieces through store4
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) stg[(4 * lq + i) * PITCH + 16 * j + lr] = acc[j][i];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int qq = lane + 64 * it, row = qq >> 4, c4 = qq & 15;
      const float4 o = *reinterpret_cast<const float4*>(stg + row * PITCH + 4 * c4);
      const int m = 16 * blk + row, n = n0 + 4 * c4;
      if (DBG == 1) {   // timing only: no epilogue stores
        if (o.x == 1.2345f) a.C[0] = o.y;
        continue;
      }
      if (m < a.M && n < a.N) store4(a, 0, m, n, o);
    }
    __builtin_amdgcn_wave_barrier();
  };
  for (int blk = b0 + wave; blk < b1; blk += NW) {
    const int nb = blk + NW < b1 ? blk + NW : -1;
    block(blk, nb);
  }
  stamp();
}

int x6r_debug_stamps(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_x6r_stamps), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}

int g_x6r_dbg = 0;   // timing-only structural variants (mrg_gemm_x6r_debug)

// B-resident launch: one workgroup per CU (grid = slices x ranges <= the CU count)
static int g_cu_count = 0;
int launch_x6r(GemmArgs a, long bplane, hipStream_t s, int waves) {
  if (!g_cu_count) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_cu_count, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      g_cu_count = 256;
  }
  const int nslice = (a.N + 63) / 64;
  int nrange = g_cu_count / nslice;
  if (nrange < 1) nrange = 1;
  const int mb = (a.M + 15) / 16;
  if (nrange > mb) nrange = mb;
  const unsigned grid = (unsigned)(nslice * nrange);
  if (a.K == 256 && g_x6r_dbg > 0) {
    switch (g_x6r_dbg) {
      case 1: klaunch(gemm_x6r_kernel<8, 8, 1>, grid, 512, 0, s, a, bplane, nslice, nrange); break;
      case 2: klaunch(gemm_x6r_kernel<8, 8, 2>, grid, 512, 0, s, a, bplane, nslice, nrange); break;
      case 3: klaunch(gemm_x6r_kernel<8, 8, 3>, grid, 512, 0, s, a, bplane, nslice, nrange); break;
      default: klaunch(gemm_x6r_kernel<8, 8, 4>, grid, 512, 0, s, a, bplane, nslice, nrange); break;
    }
    return 0;
  }
  if (a.K == 256) {
    if (waves == 8) klaunch(gemm_x6r_kernel<8, 8>, grid, 512, 0, s, a, bplane, nslice, nrange);
    else klaunch(gemm_x6r_kernel<8, 4>, grid, 256, 0, s, a, bplane, nslice, nrange);
  } else if (a.K == 128) {
    if (waves == 8) klaunch(gemm_x6r_kernel<4, 8>, grid, 512, 0, s, a, bplane, nslice, nrange);
    else klaunch(gemm_x6r_kernel<4, 4>, grid, 256, 0, s, a, bplane, nslice, nrange);
  } else {
    return -1;
  }
  return 0;
}

template <int BN, int NS>
static void launch_w(GemmArgs a, long bplane, hipStream_t s, const GemmBatch& gb) {
  a.tiles_n = (a.N + BN - 1) / BN;
  a.tiles_mn = a.tiles_n * ((a.M + 63) / 64);
  a.ntiles = a.tiles_mn;
  a.nsplit = 1;
  a.ws = nullptr;
  const unsigned grid = (unsigned)a.tiles_mn * (unsigned)(gb.n > 0 ? gb.n : 1);
  klaunch(gemm_x6w_kernel<BN, NS>, grid, NT, 0, s, a, bplane, gb);
}

// config: bn in {64, 128, 256}, ns in {2, 3}
void launch_x6w(GemmArgs a, int bn, int ns, long bplane, hipStream_t s, const GemmBatch* gbp) {
  GemmBatch none;
  none.n = 0;
  const GemmBatch& gb = gbp ? *gbp : none;
  if (bn == 64) {
    if (ns == 3) launch_w<64, 3>(a, bplane, s, gb);
    else launch_w<64, 2>(a, bplane, s, gb);
  } else if (bn == 256) {
    launch_w<256, 2>(a, bplane, s, gb);
  } else {
    if (ns == 3) launch_w<128, 3>(a, bplane, s, gb);
    else launch_w<128, 2>(a, bplane, s, gb);
  }
}

}  // namespace mrg
