// Block-causal cross-modal multi-head attention core, fp32, gfx950 f32 MFMA
// (v_mfma_f32_16x16x4_f32).  Replaces the SDPA call inside
// nn.MultiheadAttention as the reference uses it (MHAforSequentail,
// for_sequential.py:42-51; MultiModalAttentionBlockSequential,
// multi_modal_att.py:22-31).  The mask of gen_attention_mask
// (multi_modal_metaformer.py:32-79) is evaluated from indices, never
// materialised:
//   causal, Tk = r*Tq : query i sees key j  iff  j / r <= i
//   causal, Tq = r*Tk : query i sees key j  iff  j <= i / r
//   padding           : masked iff qpad[b][i] && kpad[b][j]   (the AND rule)
// A fully masked row yields NaN exactly like softmax over all -inf.
//
// Layouts: element (b, t, head, d) of q/k/v/o lives at
//   base + b*bs + t*ts + head*D + d      (the [B, T, E] projections, no copy)
// Forward: one workgroup = 4 waves = 64 queries of one (b, head); each wave
// keeps 16 queries' Q^T in registers and computes S^T = K Q^T so a query is a
// lane column: the online-softmax row max/sum is 4 registers + 2 shuffles,
// and P^T feeds the P.V MFMA straight from the accumulator (k-order permuted
// identically on both operands, no transpose).  Backward (deterministic, no
// atomics): one kernel per 64-key block for dK/dV, one per 64-query block for
// dQ, both recomputing P from the forward's log-sum-exp.
#include "mrg_common.h"

namespace mrg {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct AttnArgs {
  const float* q; long q_bs, q_ts;
  const float* k; long k_bs, k_ts;
  const float* v; long v_bs, v_ts;
  float* o; long o_bs, o_ts;
  float* lse;  // [B, Hh, Tq]
  const unsigned char* qpad;  // [B, Tq] nullable
  const unsigned char* kpad;  // [B, Tk] nullable
  const float* dout; long do_bs, do_ts;
  float* dlt;  // [B, Hh, Tq]
  float* dq; long dq_bs, dq_ts;
  float* dk; long dk_bs, dk_ts;
  float* dv; long dv_bs, dv_ts;
  int B, Hh, Tq, Tk;
  int causal;
  float scale;
};

__device__ __forceinline__ bool visible(const AttnArgs& a, int b, int i, int j) {
  if (i >= a.Tq || j >= a.Tk) return false;
  if (a.causal) {
    if (a.Tk % a.Tq == 0) {
      if (j / (a.Tk / a.Tq) > i) return false;
    } else {
      if (j > i / (a.Tq / a.Tk)) return false;
    }
  }
  if (a.qpad && a.kpad && a.qpad[(long)b * a.Tq + i] && a.kpad[(long)b * a.Tk + j]) return false;
  return true;
}

// exclusive upper bound of keys any query in [q_lo, q_hi] can see
__device__ __forceinline__ int key_limit(const AttnArgs& a, int q_hi) {
  if (!a.causal) return a.Tk;
  q_hi = min(q_hi, a.Tq - 1);
  int lim;
  if (a.Tk % a.Tq == 0) lim = (q_hi + 1) * (a.Tk / a.Tq);
  else lim = q_hi / (a.Tq / a.Tk) + 1;
  return min(lim, a.Tk);
}

// first query that can see key j_lo
__device__ __forceinline__ int query_start(const AttnArgs& a, int j_lo) {
  if (!a.causal) return 0;
  if (a.Tk % a.Tq == 0) return j_lo / (a.Tk / a.Tq);
  return j_lo * (a.Tq / a.Tk);
}

static constexpr int KT = 32;  // keys (or queries) per LDS tile

template <int D>
struct AttnCfg {
  static constexpr int DT = (D + 15) / 16;  // 16-wide d tiles
  static constexpr int DP = DT * 16;
  static constexpr int KS = D / 4;          // k-steps over d
  static constexpr int SA = DP + 2;         // row stride for [row = lane&15] reads
};

// load a [KT rows][D] tile (rows r0.., zero-filled past nrows) into LDS with row stride S
template <int D, int S>
__device__ __forceinline__ void load_rows(float* lds, const float* base, long bs_off, long ts, int hoff,
                                          int r0, int nrows) {
  constexpr int DP = AttnCfg<D>::DP;
  for (int e = threadIdx.x; e < KT * DP; e += 256) {
    int r = e / DP, d = e % DP;
    float v = 0.0f;
    if (d < D && r0 + r < nrows) v = base[bs_off + (long)(r0 + r) * ts + hoff + d];
    lds[r * S + d] = v;
  }
}

template <int D>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  using C = AttnCfg<D>;
  __shared__ float Ks[KT * C::SA];
  __shared__ float Vs[KT * (C::DP + 4)];
  constexpr int SV = C::DP + 4;
  const int b = blockIdx.z, h = blockIdx.y;
  const int q0 = blockIdx.x * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lq = lane & 15, lg = lane >> 4;
  const int qi = q0 + wave * 16 + lq;
  const int hoff = h * D;

  float qreg[C::KS];
#pragma unroll
  for (int s = 0; s < C::KS; ++s)
    qreg[s] = qi < a.Tq ? a.q[(long)b * a.q_bs + (long)qi * a.q_ts + hoff + 4 * s + lg] * a.scale : 0.0f;

  f32x4 o[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.0f;

  const int klim = key_limit(a, q0 + 63);
  for (int k0 = 0; k0 < klim; k0 += KT) {
    __syncthreads();
    load_rows<D, C::SA>(Ks, a.k, (long)b * a.k_bs, a.k_ts, hoff, k0, a.Tk);
    load_rows<D, SV>(Vs, a.v, (long)b * a.v_bs, a.v_ts, hoff, k0, a.Tk);
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < KT / 16; ++sub) {
      const int kb = k0 + sub * 16;
      if (kb >= klim) break;
      f32x4 s4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        float av = Ks[(sub * 16 + lq) * C::SA + 4 * s + lg];
        s4 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, qreg[s], s4, 0, 0, 0);
      }
      float sv[4];
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int kj = kb + lg * 4 + r;
        sv[r] = visible(a, b, qi, kj) ? s4[r] : -INFINITY;
        mx = fmaxf(mx, sv[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      float mn = fmaxf(m, mx);
      float alpha = (mn == -INFINITY) ? 1.0f : __expf(m - mn);
      float p[4];
      float ps = 0.0f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        p[r] = (sv[r] == -INFINITY) ? 0.0f : __expf(sv[r] - mn);
        ps += p[r];
      }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      l = l * alpha + ps;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt) {
        o[dt] *= alpha;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          float av = Vs[(sub * 16 + 4 * lg + s) * SV + dt * 16 + lq];
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, p[s], o[dt], 0, 0, 0);
        }
      }
    }
  }
  if (qi < a.Tq) {
    float inv = 1.0f / l;  // l == 0 (fully masked row) -> NaN like softmax(-inf row)
    float* op = a.o + (long)b * a.o_bs + (long)qi * a.o_ts + hoff;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int d = dt * 16 + lg * 4 + r;
        if (d < D) op[d] = (l == 0.0f) ? NAN : o[dt][r] * inv;
      }
    if (lg == 0) a.lse[((long)b * a.Hh + h) * a.Tq + qi] = (l == 0.0f) ? NAN : m + __logf(l);
  }
}

// dlt[b,h,q] = sum_d dO * O.  One wave per (b, q) row of all heads: float4 per
// lane (coalesced 1-KiB row segments), per-head sums by shuffles within the
// D/4 lanes that hold one head.
__global__ __launch_bounds__(256) void attn_dlt_kernel(AttnArgs a, int D) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= (long)a.B * a.Tq) return;
  const int b = row / a.Tq, qi = row % a.Tq;
  const int E = a.Hh * D;
  const float* po = a.o + (long)b * a.o_bs + (long)qi * a.o_ts;
  const float* pd = a.dout + (long)b * a.do_bs + (long)qi * a.do_ts;
  const int gl = D / 4;  // lanes per head
  for (int e0 = 0; e0 < E; e0 += 256) {
    const int e = e0 + lane * 4;
    float s = 0.0f;
    if (e < E) {
      float4 o4 = *reinterpret_cast<const float4*>(po + e);
      float4 d4 = *reinterpret_cast<const float4*>(pd + e);
      s = o4.x * d4.x + o4.y * d4.y + o4.z * d4.z + o4.w * d4.w;
    }
    for (int off = gl / 2; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    if (e < E && (lane % gl) == 0) a.dlt[((long)b * a.Hh + e / D) * a.Tq + qi] = s;
  }
}

// dQ for 64 queries of one (b, head): recompute P^T, dP^T = V dO^T, dS^T, dQ^T += K^T dS^T
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnArgs a) {
  using C = AttnCfg<D>;
  __shared__ float Ks[KT * C::SA];
  __shared__ float Vs[KT * C::SA];
  const int b = blockIdx.z, h = blockIdx.y;
  const int q0 = blockIdx.x * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lq = lane & 15, lg = lane >> 4;
  const int qi = q0 + wave * 16 + lq;
  const int hoff = h * D;
  const bool qv = qi < a.Tq;
  float qreg[C::KS], dreg[C::KS];
#pragma unroll
  for (int s = 0; s < C::KS; ++s) {
    qreg[s] = qv ? a.q[(long)b * a.q_bs + (long)qi * a.q_ts + hoff + 4 * s + lg] * a.scale : 0.0f;
    dreg[s] = qv ? a.dout[(long)b * a.do_bs + (long)qi * a.do_ts + hoff + 4 * s + lg] : 0.0f;
  }
  const long rowi = ((long)b * a.Hh + h) * a.Tq + qi;
  const float lse = qv ? a.lse[rowi] : 0.0f;
  const float dl = qv ? a.dlt[rowi] : 0.0f;
  f32x4 dq[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int klim = key_limit(a, q0 + 63);
  for (int k0 = 0; k0 < klim; k0 += KT) {
    __syncthreads();
    load_rows<D, C::SA>(Ks, a.k, (long)b * a.k_bs, a.k_ts, hoff, k0, a.Tk);
    load_rows<D, C::SA>(Vs, a.v, (long)b * a.v_bs, a.v_ts, hoff, k0, a.Tk);
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < KT / 16; ++sub) {
      const int kb = k0 + sub * 16;
      if (kb >= klim) break;
      f32x4 s4 = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 dp4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        float ka = Ks[(sub * 16 + lq) * C::SA + 4 * s + lg];
        float va = Vs[(sub * 16 + lq) * C::SA + 4 * s + lg];
        s4 = __builtin_amdgcn_mfma_f32_16x16x4f32(ka, qreg[s], s4, 0, 0, 0);
        dp4 = __builtin_amdgcn_mfma_f32_16x16x4f32(va, dreg[s], dp4, 0, 0, 0);
      }
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int kj = kb + lg * 4 + r;
        float p = (qv && visible(a, b, qi, kj)) ? __expf(s4[r] - lse) : 0.0f;
        ds[r] = p * (dp4[r] - dl);
      }
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          float ka = Ks[(sub * 16 + 4 * lg + s) * C::SA + dt * 16 + lq];
          dq[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ka, ds[s], dq[dt], 0, 0, 0);
        }
    }
  }
  if (qv) {
    float* op = a.dq + (long)b * a.dq_bs + (long)qi * a.dq_ts + hoff;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int d = dt * 16 + lg * 4 + r;
        if (d < D) op[d] = dq[dt][r] * a.scale;
      }
  }
}

// dK, dV for 64 keys of one (b, head): S = Q K^T (query rows), P, dP = dO V^T,
// dV^T += dO^T P, dK^T += Q^T dS
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(AttnArgs a) {
  using C = AttnCfg<D>;
  __shared__ float Qs[KT * C::SA];
  __shared__ float Ds[KT * C::SA];
  __shared__ float Ls[KT], Dl[KT];
  const int b = blockIdx.z, h = blockIdx.y;
  const int kb0 = blockIdx.x * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lk = lane & 15, lg = lane >> 4;
  const int kj = kb0 + wave * 16 + lk;
  const int hoff = h * D;
  const bool kv = kj < a.Tk;
  float kreg[C::KS], vreg[C::KS];
#pragma unroll
  for (int s = 0; s < C::KS; ++s) {
    kreg[s] = kv ? a.k[(long)b * a.k_bs + (long)kj * a.k_ts + hoff + 4 * s + lg] : 0.0f;
    vreg[s] = kv ? a.v[(long)b * a.v_bs + (long)kj * a.v_ts + hoff + 4 * s + lg] : 0.0f;
  }
  f32x4 dkT[C::DT], dvT[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt) {
    dkT[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    dvT[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int qs = (query_start(a, kb0) / KT) * KT;
  for (int qt0 = qs; qt0 < a.Tq; qt0 += KT) {
    __syncthreads();
    load_rows<D, C::SA>(Qs, a.q, (long)b * a.q_bs, a.q_ts, hoff, qt0, a.Tq);
    load_rows<D, C::SA>(Ds, a.dout, (long)b * a.do_bs, a.do_ts, hoff, qt0, a.Tq);
    if (threadIdx.x < KT) {
      int qq = qt0 + threadIdx.x;
      long ri = ((long)b * a.Hh + h) * a.Tq + qq;
      Ls[threadIdx.x] = qq < a.Tq ? a.lse[ri] : 0.0f;
      Dl[threadIdx.x] = qq < a.Tq ? a.dlt[ri] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int sub = 0; sub < KT / 16; ++sub) {
      const int qb = qt0 + sub * 16;
      if (qb >= a.Tq) break;
      f32x4 s4 = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 dp4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        float qa = Qs[(sub * 16 + lk) * C::SA + 4 * s + lg];
        float da = Ds[(sub * 16 + lk) * C::SA + 4 * s + lg];
        s4 = __builtin_amdgcn_mfma_f32_16x16x4f32(qa, kreg[s], s4, 0, 0, 0);
        dp4 = __builtin_amdgcn_mfma_f32_16x16x4f32(da, vreg[s], dp4, 0, 0, 0);
      }
      float p[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int ql = sub * 16 + lg * 4 + r;  // query row of this accumulator register
        int qq = qt0 + ql;
        bool vis = kv && visible(a, b, qq, kj);
        p[r] = vis ? __expf(s4[r] * a.scale - Ls[ql]) : 0.0f;
        ds[r] = p[r] * (dp4[r] - Dl[ql]);
      }
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          int row = (sub * 16 + 4 * lg + s) * C::SA + dt * 16 + lk;
          dvT[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ds[row], p[s], dvT[dt], 0, 0, 0);
          dkT[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Qs[row], ds[s], dkT[dt], 0, 0, 0);
        }
    }
  }
  if (kv) {
    float* pk = a.dk + (long)b * a.dk_bs + (long)kj * a.dk_ts + hoff;
    float* pv = a.dv + (long)b * a.dv_bs + (long)kj * a.dv_ts + hoff;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int d = dt * 16 + lg * 4 + r;
        if (d < D) {
          pk[d] = dkT[dt][r] * a.scale;
          pv[d] = dvT[dt][r];
        }
      }
  }
}

}  // namespace mrg

using namespace mrg;

static AttnArgs attn_base(int B, int Hh, int Tq, int Tk, const float* q, long q_bs, long q_ts,
                          const float* k, long k_bs, long k_ts, const float* v, long v_bs, long v_ts,
                          const float* o, long o_bs, long o_ts, const float* lse,
                          const unsigned char* qpad, const unsigned char* kpad, int causal, float scale) {
  AttnArgs a;
  memset(&a, 0, sizeof(a));
  a.q = q; a.q_bs = q_bs; a.q_ts = q_ts; a.k = k; a.k_bs = k_bs; a.k_ts = k_ts;
  a.v = v; a.v_bs = v_bs; a.v_ts = v_ts; a.o = const_cast<float*>(o); a.o_bs = o_bs; a.o_ts = o_ts;
  a.lse = const_cast<float*>(lse); a.qpad = qpad; a.kpad = kpad; a.B = B; a.Hh = Hh; a.Tq = Tq; a.Tk = Tk;
  a.causal = causal; a.scale = scale;
  return a;
}

static int attn_check(int D, int Tq, int Tk, int causal) {
  MRG_REQUIRE(D == 8 || D == 16 || D == 32 || D == 64, "attention: unsupported head dim %d", D);
  MRG_REQUIRE(!causal || Tq == 0 || Tk == 0 || Tk % Tq == 0 || Tq % Tk == 0,
              "attention: other_modal_len must be divisible by main_modal_len (Tq=%d Tk=%d)", Tq, Tk);
  return 0;
}

#define MRG_ATTN_DISPATCH(KERNEL, grid, args)                          \
  switch (D) {                                                         \
    case 8: KERNEL<8><<<grid, 256, 0, stream>>>(args); break;         \
    case 16: KERNEL<16><<<grid, 256, 0, stream>>>(args); break;       \
    case 32: KERNEL<32><<<grid, 256, 0, stream>>>(args); break;       \
    case 64: KERNEL<64><<<grid, 256, 0, stream>>>(args); break;       \
  }

MRG_API int mrg_attention_fwd(int B, int Hh, int Tq, int Tk, int D,
                              const float* q, long q_bs, long q_ts, const float* k, long k_bs, long k_ts,
                              const float* v, long v_bs, long v_ts, float* o, long o_bs, long o_ts,
                              float* lse, const unsigned char* qpad, const unsigned char* kpad,
                              int causal, float scale, hipStream_t stream) {
  if (int e = attn_check(D, Tq, Tk, causal)) return e;
  if (B == 0 || Tq == 0) return 0;
  AttnArgs a = attn_base(B, Hh, Tq, Tk, q, q_bs, q_ts, k, k_bs, k_ts, v, v_bs, v_ts, o, o_bs, o_ts, lse,
                         qpad, kpad, causal, scale);
  dim3 grid((Tq + 63) / 64, Hh, B);
  MRG_ATTN_DISPATCH(attn_fwd_kernel, grid, a);
  return check_launch("attn_fwd_kernel");
}

MRG_API size_t mrg_attention_bwd_workspace_bytes(int B, int Hh, int Tq) {
  return (size_t)B * Hh * Tq * sizeof(float);
}

MRG_API int mrg_attention_bwd(int B, int Hh, int Tq, int Tk, int D,
                              const float* q, long q_bs, long q_ts, const float* k, long k_bs, long k_ts,
                              const float* v, long v_bs, long v_ts, const float* o, long o_bs, long o_ts,
                              const float* lse, const unsigned char* qpad, const unsigned char* kpad,
                              int causal, float scale, const float* dout, long do_bs, long do_ts,
                              float* dq, long dq_bs, long dq_ts, float* dk, long dk_bs, long dk_ts,
                              float* dv, long dv_bs, long dv_ts, float* workspace, hipStream_t stream) {
  if (int e = attn_check(D, Tq, Tk, causal)) return e;
  if (B == 0 || Tq == 0 || Tk == 0) return 0;
  AttnArgs a = attn_base(B, Hh, Tq, Tk, q, q_bs, q_ts, k, k_bs, k_ts, v, v_bs, v_ts, o, o_bs, o_ts, lse,
                         qpad, kpad, causal, scale);
  a.dout = dout; a.do_bs = do_bs; a.do_ts = do_ts; a.dlt = workspace;
  a.dq = dq; a.dq_bs = dq_bs; a.dq_ts = dq_ts; a.dk = dk; a.dk_bs = dk_bs; a.dk_ts = dk_ts;
  a.dv = dv; a.dv_bs = dv_bs; a.dv_ts = dv_ts;
  MRG_REQUIRE((o_ts & 3) == 0 && (do_ts & 3) == 0 && (o_bs & 3) == 0 && (do_bs & 3) == 0 &&
              (((uintptr_t)o | (uintptr_t)dout) & 15) == 0, "attention bwd: O/dO rows must be 16-B aligned");
  long rows = (long)B * Tq;
  attn_dlt_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, stream>>>(a, D);
  if (check_launch("attn_dlt_kernel")) return 1;
  dim3 gq((Tq + 63) / 64, Hh, B);
  MRG_ATTN_DISPATCH(attn_bwd_dq_kernel, gq, a);
  if (check_launch("attn_bwd_dq_kernel")) return 1;
  dim3 gk((Tk + 63) / 64, Hh, B);
  MRG_ATTN_DISPATCH(attn_bwd_dkv_kernel, gk, a);
  return check_launch("attn_bwd_dkv_kernel");
}
