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
#include <utility>

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

// the same read at addr + OFF (immediate offset: the fragment reads of one k-tile share one address)
template <int OFF>
__device__ __forceinline__ f32x4w wlds16o(unsigned addr) {
  f32x4w v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF) : "memory");
  return v;
}

// B plane P of block j (a constant once the block loop is unrolled): offset P SBP + 1024 j
template <int P, int SBP, int... J>
__device__ __forceinline__ f32x4w wlds16o_sel(unsigned addr, int j, std::integer_sequence<int, J...>) {
  f32x4w v{};
  ((j == J ? (void)(v = wlds16o<P * SBP + 1024 * J>(addr)) : (void)0), ...);
  return v;
}
template <int P, int SBP, int NB>
__device__ __forceinline__ f32x4w wlds16o_j(unsigned addr, int j) {
  return wlds16o_sel<P, SBP>(addr, j, std::make_integer_sequence<int, NB>{});
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
  // fragment offsets in a slot: A's two chunks; B block j plane p at ob + p SBP + 1024 j (wb_off's
  // swizzle bit (n >> 3) & 1 is the same for rows 16 j + (lane & 15) of every block)
  const unsigned oa0 = wa_off(ar, ac), oa1 = wa_off(ar, ac + 1), ob = SA + wb_off(lane & 15, bc);

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
    const unsigned sb = sa + ob;
    f32x4w va0 = wlds16(sa + oa0), va1 = wlds16(sa + oa1);
    f32x4w vb[2][3];
    vb[0][0] = wlds16o<0>(sb);
    vb[0][1] = wlds16o<SBP>(sb);
    vb[0][2] = wlds16o<2 * SBP>(sb);
    asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(va0), "+v"(va1)::"memory");
    bf16x8 fa[3];
    wsplit8(va0, va1, fa);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int cur = j & 1, nxt = cur ^ 1;
      if (j + 1 < NB) {
        vb[nxt][0] = wlds16o_j<0, SBP, NB>(sb, j + 1);
        vb[nxt][1] = wlds16o_j<1, SBP, NB>(sb, j + 1);
        vb[nxt][2] = wlds16o_j<2, SBP, NB>(sb, j + 1);
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

// config: bn in {64, 128}, ring depth 2 (depth 3 and 256-wide tiles measured slower in the step and
// were removed: profiles/r06_knobs_ab.txt)
void launch_x6w(GemmArgs a, int bn, int ns, long bplane, hipStream_t s, const GemmBatch* gbp) {
  (void)ns;
  GemmBatch none;
  none.n = 0;
  const GemmBatch& gb = gbp ? *gbp : none;
  if (bn == 64) launch_w<64, 2>(a, bplane, s, gb);
  else launch_w<128, 2>(a, bplane, s, gb);
}

}  // namespace mrg
