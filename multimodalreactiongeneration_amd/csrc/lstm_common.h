// Shared pieces of the persistent LSTM recurrences (lstm.hip: VALU GEMV form; lstm_mx.hip: MFMA
// form for batch tiles of 16 rows): problem / argument blocks, the {tag, value} granule hand-off,
// the block -> (problem, group, member) map and the co-residency check.
#pragma once
#include "mrg_common.h"

namespace mrg {

static constexpr int MAXP = 12;  // problems per launch (kernarg: 12 x 176 B)

struct LstmFwdProblem {
  const float* gx;  // pre-activations from the input GEMM (+ b_ih)
  long gx_bs, gx_ts;
  const float* w_hh;  // [4H, H]
  const float* b_hh;  // [4H]
  const float* h0;    // [B, H] or null
  const float* c0;    // [B, H] or null
  float* y;           // h_t
  long y_bs, y_ts;
  float* gates;  // [B, T, 4H] post-activation i, f, g, o (saved for backward)
  float* cs;     // [B, T, H] cell states (saved for backward)
  float* hT;     // [B, H] or null
  float* cT;     // [B, H] or null
  unsigned long long* xbuf;  // [2][B][H] granules
  long g_bs, g_ts, cs_bs, cs_ts, h0_bs, c0_bs;  // strides (elements) of gates / cs / h0 / c0: time chunks of a
                                                // longer sequence, time-major layouts
  int reverse;
};

struct LstmBwdProblem {
  const float* w_hh;
  const float* gates;
  const float* cs;
  const float* c0;  // nullable
  const float* dy;  // nullable
  long dy_bs, dy_ts;
  const float* dhT;  // nullable
  const float* dcT;  // nullable
  float* dG;         // [B, T, 4H]
  float* dh0;        // nullable
  float* dc0;        // nullable
  unsigned long long* xbuf;  // [2][B][G][H] granules
  long g_bs, g_ts, cs_bs, cs_ts, c0_bs, dG_bs, dG_ts;  // strides (elements) of gates / cs / c0 / dG
  int reverse;
};

struct LstmFwdArgs {
  LstmFwdProblem p[MAXP];
  int nprob, B, T;
  int inject;  // fault injection (mrg_lstm_debug_inject): 1 = member 0 drops its first hand-off
  int local;   // granule stores keep the line in L2 (put_granule)
  int* err;
  unsigned long long* stamps;  // diagnostics only (mrg_lstm_debug_stamps); null in normal use
};
struct LstmBwdArgs {
  LstmBwdProblem p[MAXP];
  int nprob, B, T;
  int inject;  // fault injection (mrg_lstm_debug_inject mode 2): member 0 drops its first hand-off
  int local;
  int* err;
  unsigned long long* stamps;
};

// Phase stamps of block 0 / thread 0 (shader-clock s_memtime), [T][8] per launch.
#define MRG_STAMP(ph)                                                                  \
  do {                                                                                 \
    if (args.stamps && blockIdx.x == 0 && threadIdx.x == 0) {                          \
      unsigned long long _t;                                                           \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");     \
      args.stamps[(long)tt * 8 + (ph)] = _t;                                           \
    }                                                                                  \
  } while (0)

static constexpr unsigned SPIN_LIMIT = 1u << 22;

__device__ __forceinline__ unsigned long long make_granule(unsigned tag, float v) {
  return ((unsigned long long)tag << 32) | (unsigned long long)__float_as_uint(v);
}

// local != 0: the granule is published with a workgroup-scope store, which (unlike the agent-scope
// one) keeps the line in the XCD's L2, so the group's pollers, which read with agent-scope loads
// (L1 bypassed, L2 served), find it there instead of reading it back from the memory side
// (MI355X_MICROARCH.md, "stores of each flavour"; measured: lstm fwd -14 %, bwd -12 %).  Only
// for groups whose members all run on one XCD (group_on_one_xcd, checked at launch start).
__device__ __forceinline__ void put_granule(unsigned long long* g, unsigned tag, float v, int local) {
  if (local) __hip_atomic_store(g, make_granule(tag, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else __hip_atomic_store(g, make_granule(tag, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum over aligned groups of N consecutive lanes with DPP (VALU, no LDS traffic):
// quad_perm xor1, xor2, then row_half_mirror and row_mirror pair the quads / octets.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int N>
__device__ __forceinline__ float group_sum(float v) {
  static_assert(N == 1 || N == 2 || N == 4 || N == 8 || N == 16, "group_sum");
  if (N >= 2) v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  if (N >= 4) v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  if (N >= 8) v += dpp_f<0x141>(v);  // row_half_mirror
  if (N >= 16) v += dpp_f<0x140>(v); // row_mirror
  return v;
}

// Poll N granules at once: all loads issued back-to-back (one round trip), then
// only the stale ones are re-polled.  Bounded like get_granule.
template <int N>
__device__ __forceinline__ void get_granules(unsigned long long* base, long stride, unsigned tag, float (&out)[N],
                                             int* err, bool& dead) {
  unsigned long long v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = __hip_atomic_load(base + i * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned spins = 0;
  while (!dead) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < N; ++i) ok &= (unsigned)(v[i] >> 32) == tag;
    if (ok) break;
    if (++spins > SPIN_LIMIT) {
      atomicOr(err, 1);
      dead = true;
      break;
    }
#pragma unroll
    for (int i = 0; i < N; ++i)
      if ((unsigned)(v[i] >> 32) != tag)
        v[i] = __hip_atomic_load(base + i * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = __uint_as_float((unsigned)v[i]);
}

// As get_granules, for N granules at arbitrary offsets from base.
template <int N>
__device__ __forceinline__ void get_granules_idx(unsigned long long* base, const int (&idx)[N], unsigned tag,
                                                 float (&out)[N], int* err, bool& dead) {
  unsigned long long v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = __hip_atomic_load(base + idx[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned spins = 0;
  while (!dead) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < N; ++i) ok &= (unsigned)(v[i] >> 32) == tag;
    if (ok) break;
    if (++spins > SPIN_LIMIT) {
      atomicOr(err, 1);
      dead = true;
      break;
    }
#pragma unroll
    for (int i = 0; i < N; ++i)
      if ((unsigned)(v[i] >> 32) != tag)
        v[i] = __hip_atomic_load(base + idx[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = __uint_as_float((unsigned)v[i]);
}

// Pair granules (the MFMA form, lstm_mx.hip): one 8-byte word carries TWO fp32 values, each with a
// 2-bit step tag in its two lowest mantissa bits ((step + 1) & 3; a ring slot is rewritten every
// second step, so the stale tag differs by 2).  Half the bytes of {tag, value} granules for the
// gathers that bound the MFMA form's step; a published value is off by at most 3 ulp (2^-21.4
// relative), far inside the fp32-class error of the x6 products it feeds.  A slot is fresh when both
// halves carry the tag (the word is written and read as one 64-bit access, single-copy atomic).
__device__ __forceinline__ unsigned long long make_pair(unsigned tag2, float v0, float v1) {
  const unsigned a = (__float_as_uint(v0) & ~3u) | tag2, b = (__float_as_uint(v1) & ~3u) | tag2;
  return ((unsigned long long)b << 32) | (unsigned long long)a;
}
__device__ __forceinline__ void put_pair(unsigned long long* g, unsigned tag2, float v0, float v1, int local) {
  if (local) __hip_atomic_store(g, make_pair(tag2, v0, v1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else __hip_atomic_store(g, make_pair(tag2, v0, v1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool pair_fresh(unsigned long long v, unsigned tag2) {
  return (((unsigned)v & 3u) == tag2) && (((unsigned)(v >> 32) & 3u) == tag2);
}
// Poll N pair granules at base + idx[i] (all loads in flight, then only the stale ones again).
template <int N>
__device__ __forceinline__ void get_pairs_idx(unsigned long long* base, const int (&idx)[N], unsigned tag2,
                                              float (&v0)[N], float (&v1)[N], int* err, bool& dead) {
  unsigned long long v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = __hip_atomic_load(base + idx[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned spins = 0;
  while (!dead) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < N; ++i) ok &= pair_fresh(v[i], tag2);
    if (ok) break;
    if (++spins > SPIN_LIMIT) {
      atomicOr(err, 1);
      dead = true;
      break;
    }
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (!pair_fresh(v[i], tag2)) v[i] = __hip_atomic_load(base + idx[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    v0[i] = __uint_as_float((unsigned)v[i]);
    v1[i] = __uint_as_float((unsigned)(v[i] >> 32));
  }
}
// N pair granules at base + i * stride; returns half `hi` (0: low value, 1: high value) of each.
template <int N>
__device__ __forceinline__ void get_pair_halves(unsigned long long* base, long stride, int hi, unsigned tag2,
                                                float (&out)[N], int* err, bool& dead) {
  int idx[N];
  float a[N], b[N];
#pragma unroll
  for (int i = 0; i < N; ++i) idx[i] = (int)(i * stride);
  get_pairs_idx<N>(base, idx, tag2, a, b, err, dead);
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = hi ? b[i] : a[i];
}

// Local hand-offs are used only where every member of a group verified, at launch start, that it
// runs on the same XCD as the others: each member publishes its HW_REG_XCC_ID with an agent-scope
// store into the ring slot `slots[member]` (parity-1 slots, first written with step data at step
// 1, after every member has finished this check) and reads the group's G ids back.  Every member
// sees the same G ids, so the group decides alike; a group split over XCDs keeps agent-scope
// stores.  Correctness never depends on placement; only the store flavour does.
static constexpr unsigned XCC_TAG = 0xFFFFFFFEu;

template <int G>
__device__ __forceinline__ int group_on_one_xcd(unsigned long long* slots, int member, int* err, bool& dead,
                                                int* flag) {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  // the id travels shifted left by 2: its low half's 2-bit tag is 0, so a pair-granule reader
  // (pair_fresh, the MFMA form's ring) never takes this word for step data (the high half,
  // XCC_TAG, carries tag 2); 32-bit-tag readers never match XCC_TAG
  const unsigned code = xcc << 2;
  if (threadIdx.x == 0) {
    __hip_atomic_store(slots + member, make_granule(XCC_TAG, __uint_as_float(code)), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    float ids[G];
    get_granules<G>(slots, 1, XCC_TAG, ids, err, dead);
    int same = 1;
#pragma unroll
    for (int m = 0; m < G; ++m) same &= __float_as_uint(ids[m]) == code;
    *flag = same;
  }
  __syncthreads();
  const int same = *flag;
  __syncthreads();
  return same;
}

// block -> (problem, group, member); members of a group share blockIdx % 8 (one XCD)
__device__ __forceinline__ void decompose(int G, int ngroups_per_prob, int nprob, int& prob, int& grp,
                                          int& member) {
  int b = blockIdx.x;
  int total_groups = ngroups_per_prob * nprob;
  int gid;
  if ((total_groups & 7) == 0) {
    int x = b & 7, idx = b >> 3;
    member = idx % G;
    gid = (idx / G) * 8 + x;
  } else {
    member = b % G;
    gid = b / G;
  }
  prob = gid / ngroups_per_prob;
  grp = gid % ngroups_per_prob;
}

// Persistent launches need every workgroup of a group resident: pick the smallest
// batch tile BS whose grid fits the occupancy the HW reports for that kernel, or fail.
template <typename K>
static bool fits(K kernel, int nt, long nblk, int cus) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kernel), nt, 0) !=
      hipSuccess)
    return false;
  return nblk <= (long)per_cu * cus;
}

// CU count of the current device (occupancy check of the persistent grids)
[[maybe_unused]] static int device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return n;
}

}  // namespace mrg
