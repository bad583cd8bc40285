// Block-causal cross-modal multi-head attention core, fp32, gfx950 f32 MFMA
// (v_mfma_f32_16x16x4_f32).  Replaces the SDPA call inside
// nn.MultiheadAttention as the reference uses it (MHAforSequentail,
// for_sequential.py:42-51; MultiModalAttentionBlockSequential,
// multi_modal_att.py:22-31).  The mask of gen_attention_mask
// (multi_modal_metaformer.py:32-79) is evaluated from indices, never
// materialised:
//   causal, Tk = r*Tq : query i sees key j  iff  j / r <= i   (j < (i+1) r)
//   causal, Tq = r*Tk : query i sees key j  iff  j <= i / r
//   padding           : masked iff qpad[b][i] && kpad[b][j]   (the AND rule)
// A fully masked row yields NaN exactly like softmax over all -inf.
//
// Layouts: element (b, t, head, d) of q/k/v/o lives at
//   base + b*bs + t*ts + head*D + d      (the [B, T, E] projections, no copy;
//   rows 16-B aligned, loaded as float4)
// Forward: one workgroup = 4 waves = 64 queries of one (b, head); each wave
// keeps 16 queries' Q^T in registers and computes S^T = K Q^T so a query is a
// lane column: the online-softmax row max/sum is 4 registers + 2 shuffles,
// and P^T feeds the P.V MFMA straight from the accumulator (k-order permuted
// identically on both operands, no transpose).  K/V tiles of 64 keys go
// HBM -> registers (the next tile's loads fly under this tile's MFMAs) -> LDS.
// The causal limit is one compare per element against a per-lane bound, and
// the mask is skipped entirely for sub-tiles every query of the wave sees.
// Backward (deterministic, no atomics): a dQ kernel per 64-query block (which
// also forms delta = rowsum(dO * O) for its rows) and then a dK/dV kernel per
// 64-key block, both recomputing P from the forward's log-sum-exp.
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
  int qvec, ovec, dkvvec;  // rows of q / o / dk and dv 16-B aligned: float4 loads and stores
  // query chunk (mrg_attention_*_chunk): the Tq queries are rows [q_off, q_off + Tq) of a sequence of
  // Tqf queries (the causal rule uses global indices and Tk / Tqf); qpad rows have stride qp_bs;
  // kv_acc: the dK / dV pass adds into dk / dv (a chunk's share) instead of storing
  int q_off, Tqf;
  long qp_bs;
  int kv_acc;
  // lse / delta rows: [B, Hh, st_ld] arrays, this call's queries at column st_off (chunk calls hand in
  // the whole sequence's statistics: st_ld = Tqf, st_off = q_off)
  int st_ld, st_off;
};

__device__ __forceinline__ long stat_row(const AttnArgs& a, int b, int h, int qi) {
  return ((long)b * a.Hh + h) * a.st_ld + a.st_off + qi;
}

// exclusive upper bound of the keys query i may see (causal rule only; Tk when not causal)
__device__ __forceinline__ int key_bound(const AttnArgs& a, int i) {
  if (!a.causal) return a.Tk;
  i = min(i, a.Tq - 1) + a.q_off;
  int lim = (a.Tk >= a.Tqf) ? (i + 1) * (a.Tk / a.Tqf) : i / (a.Tqf / a.Tk) + 1;
  return min(lim, a.Tk);
}

// first query that may see key j (causal rule only)
__device__ __forceinline__ int query_start(const AttnArgs& a, int j) {
  if (!a.causal) return 0;
  const int g = (a.Tk >= a.Tqf) ? j / (a.Tk / a.Tqf) : j * (a.Tqf / a.Tk);
  return max(g - a.q_off, 0);   // chunk-local
}

static constexpr int TT = 64;  // keys (forward, dQ) or queries (dK/dV) per LDS tile

template <int D>
struct AttnCfg {
  static constexpr int DT = (D + 15) / 16;  // 16-wide d tiles of the output
  static constexpr int DP = DT * 16;
  static constexpr int KS = D / 4;          // k-steps over d
  // VEC (D >= 32): lane group lg takes the contiguous contraction indices d = KS*lg + s and the
  // output columns d = DT*i + dt, so LDS operands are read as float4 / float2 (4x fewer LDS
  // instructions than one ds_read_b32 per MFMA) and outputs are stored as contiguous runs; the
  // sums are the same, in a different order.  D < 32 keeps the interleaved map (d = 4s + lg).
  static constexpr bool VEC = D >= 32;
  static constexpr int SA = VEC ? DP + 4 : DP + 2;  // row stride for the [row = lane&15][d] operand reads
  static constexpr int SV = DP + 4;         // row stride for [row = 4(lane>>4)+s][16dt + lane&15] reads
  static constexpr int NV = TT * (D / 4) / 256;  // float4 per thread per tile (0 at D = 8: half the threads load)
  static constexpr int NVR = NV > 0 ? NV : 1;
};

// TT rows x D of a [T, ...] operand -> registers (float4, zero past nrows), then -> LDS.
template <int D>
struct TileRegs {
  float4 r[AttnCfg<D>::NVR];
  __device__ __forceinline__ void load(const float* base, long ts, int r0, int nrows) {
    constexpr int C4 = D / 4;
#pragma unroll
    for (int i = 0; i < AttnCfg<D>::NVR; ++i) {
      const int e = threadIdx.x + i * 256;
      const int row = e / C4, c = (e % C4) * 4;
      r[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < TT * C4 && r0 + row < nrows) r[i] = *reinterpret_cast<const float4*>(base + (long)(r0 + row) * ts + c);
    }
  }
  template <int S>
  __device__ __forceinline__ void store(float* lds) const {
    constexpr int C4 = D / 4;
#pragma unroll
    for (int i = 0; i < AttnCfg<D>::NVR; ++i) {
      const int e = threadIdx.x + i * 256;
      if (e < TT * C4) {
        const int row = e / C4, c = (e % C4) * 4;
        float* p = lds + row * S + c;
        if (S % 4 == 0) {
          *reinterpret_cast<float4*>(p) = r[i];
        } else {
          *reinterpret_cast<float2*>(p) = make_float2(r[i].x, r[i].y);
          *reinterpret_cast<float2*>(p + 2) = make_float2(r[i].z, r[i].w);
        }
      }
    }
  }
};

// contraction index d of k-step s for lane group lg (same map for every operand of a product)
template <int D>
__device__ __forceinline__ int dmap(int lg, int s) {
  return AttnCfg<D>::VEC ? AttnCfg<D>::KS * lg + s : 4 * s + lg;
}
// output d of accumulator register (dt, r) held by lane group lg
template <int D>
__device__ __forceinline__ int dout(int lg, int dt, int r) {
  return AttnCfg<D>::VEC ? AttnCfg<D>::DT * (4 * lg + r) + dt : dt * 16 + lg * 4 + r;
}
// the KS contraction operands of LDS row `row` for this lane: v[s] = S[row * STR + dmap(lg, s)]
template <int D, int STR>
__device__ __forceinline__ void row_operands(const float* S, int row, int lg, float (&v)[AttnCfg<D>::KS]) {
  using C = AttnCfg<D>;
  if constexpr (C::VEC) {
#pragma unroll
    for (int i = 0; i < C::KS; i += 4) {
      const float4 t = *reinterpret_cast<const float4*>(S + row * STR + C::KS * lg + i);
      v[i] = t.x; v[i + 1] = t.y; v[i + 2] = t.z; v[i + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int s = 0; s < C::KS; ++s) v[s] = S[row * STR + 4 * s + lg];
  }
}
// the DT output-side operands of LDS row `row` (A = X^T, MFMA row i = lane&15): v[dt] = X[row][col(i, dt)]
template <int D, int STR>
__device__ __forceinline__ void col_operands(const float* S, int row, int l16, float (&v)[AttnCfg<D>::DT]) {
  using C = AttnCfg<D>;
  if constexpr (C::VEC && C::DT == 4) {
    const float4 t = *reinterpret_cast<const float4*>(S + row * STR + 4 * l16);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else if constexpr (C::VEC && C::DT == 2) {
    const float2 t = *reinterpret_cast<const float2*>(S + row * STR + 2 * l16);
    v[0] = t.x; v[1] = t.y;
  } else {
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) v[dt] = S[row * STR + dt * 16 + l16];
  }
}

// this lane's KS contraction values of one row (row pointer p, 16-B aligned): v[s] = p[dmap(lg, s)]
// (float4 loads when the map is lane-contiguous), zero when !valid
template <int D>
__device__ __forceinline__ void row_values(const float* p, int lg, bool valid, float (&v)[AttnCfg<D>::KS]) {
  using C = AttnCfg<D>;
  if constexpr (C::VEC) {
#pragma unroll
    for (int i = 0; i < C::KS; i += 4) {
      const float4 t = valid ? *reinterpret_cast<const float4*>(p + C::KS * lg + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      v[i] = t.x; v[i + 1] = t.y; v[i + 2] = t.z; v[i + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int s = 0; s < C::KS; ++s) v[s] = valid ? p[4 * s + lg] : 0.0f;
  }
}

// store this lane's output values of one row: p[dout(lg, dt, r)] = v[dt][r] * mul (float4 per r
// when the map is lane-contiguous with DT = 4 and vec is set)
template <int D>
__device__ __forceinline__ void store_row(float* p, int lg, bool vec, const f32x4 (&v)[AttnCfg<D>::DT], float mul) {
  using C = AttnCfg<D>;
  if constexpr (C::VEC && C::DT == 4) {
    if (vec) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<float4*>(p + 4 * (4 * lg + r)) =
            make_float4(v[0][r] * mul, v[1][r] * mul, v[2][r] * mul, v[3][r] * mul);
      return;
    }
  }
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d = dout<D>(lg, dt, r);
      if (d < D) p[d] = v[dt][r] * mul;
    }
}

// as store_row, adding to what p holds
template <int D>
__device__ __forceinline__ void add_row(float* p, int lg, bool vec, const f32x4 (&v)[AttnCfg<D>::DT], float mul) {
  using C = AttnCfg<D>;
  if constexpr (C::VEC && C::DT == 4) {
    if (vec) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float4* q = reinterpret_cast<float4*>(p + 4 * (4 * lg + r));
        const float4 o = *q;
        *q = make_float4(o.x + v[0][r] * mul, o.y + v[1][r] * mul, o.z + v[2][r] * mul, o.w + v[3][r] * mul);
      }
      return;
    }
  }
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int d = dout<D>(lg, dt, r);
      if (d < D) p[d] += v[dt][r] * mul;
    }
}

// S^T tile (16 keys x 16 queries) = K rows [kr..kr+15] . Q^T, two accumulation chains
template <int D>
__device__ __forceinline__ f32x4 qk16(const float* Ks, int rowbase, const float (&qreg)[AttnCfg<D>::KS], int lq,
                                      int lg) {
  using C = AttnCfg<D>;
  f32x4 s0 = f32x4{0.f, 0.f, 0.f, 0.f}, s1 = f32x4{0.f, 0.f, 0.f, 0.f};
  float kv[C::KS];
  row_operands<D, C::SA>(Ks, rowbase + lq, lg, kv);
#pragma unroll
  for (int s = 0; s < C::KS; s += 2) {
    s0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kv[s], qreg[s], s0, 0, 0, 0);
    if (s + 1 < C::KS) s1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kv[s + 1], qreg[s + 1], s1, 0, 0, 0);
  }
  return s0 + s1;
}

template <int D>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
  using C = AttnCfg<D>;
  __shared__ __attribute__((aligned(16))) float Ks[TT * C::SA];
  __shared__ __attribute__((aligned(16))) float Vs[TT * C::SV];
  // grid (heads, B, query blocks), the last (most keys under the causal mask) dispatched first
  const int h = blockIdx.x, b = blockIdx.y;
  const int q0 = (gridDim.z - 1 - blockIdx.z) * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lq = lane & 15, lg = lane >> 4;
  const int qi = q0 + wave * 16 + lq;
  const int hoff = h * D;
  const bool pad = a.qpad && a.kpad;
  const bool qp = pad && qi < a.Tq && a.qpad[(long)b * a.qp_bs + qi];
  const int kmax = key_bound(a, qi);                    // this lane's query
  const int wmin = key_bound(a, q0 + wave * 16);        // smallest bound in the wave (monotone in i)
  const int wlim = key_bound(a, q0 + wave * 16 + 15);   // largest: sub-tiles from here on are masked

  float qreg[C::KS];
  if (a.qvec) {
    row_values<D>(a.q + (long)b * a.q_bs + (long)min(qi, a.Tq - 1) * a.q_ts + hoff, lg, qi < a.Tq, qreg);
#pragma unroll
    for (int s = 0; s < C::KS; ++s) qreg[s] *= a.scale;
  } else {
#pragma unroll
    for (int s = 0; s < C::KS; ++s)
      qreg[s] = qi < a.Tq ? a.q[(long)b * a.q_bs + (long)qi * a.q_ts + hoff + dmap<D>(lg, s)] * a.scale : 0.0f;
  }

  f32x4 o[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.0f;

  const int klim = key_bound(a, q0 + 63);
  const float* kb_ = a.k + (long)b * a.k_bs + hoff;
  const float* vb_ = a.v + (long)b * a.v_bs + hoff;
  const unsigned char* kpb = pad ? a.kpad + (long)b * a.Tk : nullptr;
  TileRegs<D> tk, tv;
  tk.load(kb_, a.k_ts, 0, a.Tk);
  tv.load(vb_, a.v_ts, 0, a.Tk);
  unsigned char kpn = (pad && lane < a.Tk) ? kpb[lane] : 0;  // padding flag of key k0 + lane
  for (int k0 = 0; k0 < klim; k0 += TT) {
    __syncthreads();
    tk.template store<C::SA>(Ks);
    tv.template store<C::SV>(Vs);
    const unsigned long long kbits = __ballot(kpn != 0);
    const unsigned long long qmask = qp ? kbits : 0ull;  // keys of this tile padding hides from query qi
    __syncthreads();
    if (k0 + TT < klim) {
      tk.load(kb_, a.k_ts, k0 + TT, a.Tk);
      tv.load(vb_, a.v_ts, k0 + TT, a.Tk);
      kpn = (pad && k0 + TT + lane < a.Tk) ? kpb[k0 + TT + lane] : 0;
    }
    // 32 keys per online-softmax update: two independent S^T sub-tiles (four MFMA chains), one
    // max / sum reduction and one rescale of O per pair
#pragma unroll
    for (int sp = 0; sp < TT / 16; sp += 2) {
      const int kb = k0 + sp * 16;
      if (kb >= wlim) break;            // every query of this wave masks these keys (no contribution)
      const bool two = kb + 16 < wlim;  // wave-uniform: the second sub-tile has visible keys
      f32x4 s4[2];
      s4[0] = qk16<D>(Ks, sp * 16, qreg, lq, lg);
      s4[1] = two ? qk16<D>(Ks, sp * 16 + 16, qreg, lq, lg) : f32x4{0.f, 0.f, 0.f, 0.f};
      float sv[8];
      float mx = -INFINITY;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int kh = kb + 16 * h;
        if (!pad && kh + 16 <= wmin) {  // every query of the wave sees all 16 keys
#pragma unroll
          for (int r = 0; r < 4; ++r) { sv[4 * h + r] = s4[h][r]; mx = fmaxf(mx, sv[4 * h + r]); }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int kl = (sp + h) * 16 + lg * 4 + r;
            const bool vis = (k0 + kl < kmax) && !((qmask >> kl) & 1ull);
            sv[4 * h + r] = vis ? s4[h][r] : -INFINITY;
            mx = fmaxf(mx, sv[4 * h + r]);
          }
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float alpha = (mn == -INFINITY) ? 1.0f : __expf(m - mn);
      float p[8];
      float ps = 0.0f;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        p[r] = (sv[r] == -INFINITY) ? 0.0f : __expf(sv[r] - mn);
        ps += p[r];
      }
      ps += __shfl_xor(ps, 16, 64);
      ps += __shfl_xor(ps, 32, 64);
      l = l * alpha + ps;
      m = mn;
#pragma unroll
      for (int dt = 0; dt < C::DT; ++dt) o[dt] *= alpha;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !two) break;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          float vv[C::DT];
          col_operands<D, C::SV>(Vs, (sp + h) * 16 + 4 * lg + s, lq, vv);
#pragma unroll
          for (int dt = 0; dt < C::DT; ++dt)
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[dt], p[4 * h + s], o[dt], 0, 0, 0);
        }
      }
    }
  }
  if (qi < a.Tq) {
    const float inv = (l == 0.0f) ? NAN : 1.0f / l;  // l == 0 (fully masked row) -> NaN like softmax(-inf row)
    store_row<D>(a.o + (long)b * a.o_bs + (long)qi * a.o_ts + hoff, lg, a.ovec, o, inv);
    if (lg == 0) a.lse[stat_row(a, b, h, qi)] = (l == 0.0f) ? NAN : m + __logf(l);
  }
}

// Backward.  The padding flags of a 64-row tile are one wave-uniform 64-bit mask (a ballot over
// the lanes' prefetched flag bytes), the visibility test is a select (no divergent branches around
// exp), and the log-sum-exp / delta rows of the dK/dV pass are float4 LDS reads.
//
// dQ for 64 queries of one (b, head): recompute P^T, dP^T = V dO^T, dS^T, dQ^T += K^T dS^T.
// Also forms delta = rowsum(dO * O) for these rows (the dK/dV kernel reads it from a.dlt).
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnArgs a) {
  using C = AttnCfg<D>;
  constexpr int ST = 1;  // 16-row sub-tiles per step (2 measured no faster)
  __shared__ __attribute__((aligned(16))) float Ks[TT * C::SA];
  __shared__ __attribute__((aligned(16))) float Vs[TT * C::SA];
  const int h = blockIdx.x, b = blockIdx.y;
  const int q0 = (gridDim.z - 1 - blockIdx.z) * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lq = lane & 15, lg = lane >> 4;
  const int qi = q0 + wave * 16 + lq;
  const int hoff = h * D;
  const bool qv = qi < a.Tq;
  const bool pad = a.qpad && a.kpad;
  const bool qp = pad && qv && a.qpad[(long)b * a.qp_bs + qi];
  const int kmax = key_bound(a, qi);
  const int wlim = key_bound(a, q0 + wave * 16 + 15);
  float qreg[C::KS], dreg[C::KS];
  float dsum = 0.0f;
  row_values<D>(a.q + (long)b * a.q_bs + (long)min(qi, a.Tq - 1) * a.q_ts + hoff, lg, qv, qreg);
  row_values<D>(a.dout + (long)b * a.do_bs + (long)min(qi, a.Tq - 1) * a.do_ts + hoff, lg, qv, dreg);
  float oreg[C::KS];
  if (a.ovec) {
    row_values<D>(a.o + (long)b * a.o_bs + (long)min(qi, a.Tq - 1) * a.o_ts + hoff, lg, qv, oreg);
  } else {
#pragma unroll
    for (int s = 0; s < C::KS; ++s) oreg[s] = qv ? a.o[(long)b * a.o_bs + (long)qi * a.o_ts + hoff + dmap<D>(lg, s)] : 0.0f;
  }
#pragma unroll
  for (int s = 0; s < C::KS; ++s) {
    qreg[s] *= a.scale;
    dsum = fmaf(dreg[s], oreg[s], dsum);
  }
  dsum += __shfl_xor(dsum, 16, 64);
  dsum += __shfl_xor(dsum, 32, 64);
  const long rowi = stat_row(a, b, h, qi);
  const float lse = qv ? a.lse[rowi] : 0.0f;
  const float dl = dsum;
  if (qv && lg == 0) a.dlt[rowi] = dsum;
  f32x4 dq[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int klim = key_bound(a, q0 + 63);
  const float* kb_ = a.k + (long)b * a.k_bs + hoff;
  const float* vb_ = a.v + (long)b * a.v_bs + hoff;
  const unsigned char* kpb = pad ? a.kpad + (long)b * a.Tk : nullptr;
  TileRegs<D> tk, tv;
  tk.load(kb_, a.k_ts, 0, a.Tk);
  tv.load(vb_, a.v_ts, 0, a.Tk);
  unsigned char kpn = (pad && lane < a.Tk) ? kpb[lane] : 0;  // padding flag of key k0 + lane
  for (int k0 = 0; k0 < klim; k0 += TT) {
    __syncthreads();
    tk.template store<C::SA>(Ks);
    tv.template store<C::SA>(Vs);
    const unsigned long long kbits = __ballot(kpn != 0);
    const unsigned long long qmask = qp ? kbits : 0ull;  // keys of this tile padding hides from query qi
    __syncthreads();
    if (k0 + TT < klim) {
      tk.load(kb_, a.k_ts, k0 + TT, a.Tk);
      tv.load(vb_, a.v_ts, k0 + TT, a.Tk);
      kpn = (pad && k0 + TT + lane < a.Tk) ? kpb[k0 + TT + lane] : 0;
    }
#pragma unroll
    for (int sub = 0; sub < TT / 16; sub += ST) {
      const int kb = k0 + sub * 16;
      if (kb >= wlim) break;
      const bool two = ST == 2 && kb + 16 < wlim;
      f32x4 s4[ST], dp4[ST];
#pragma unroll
      for (int u = 0; u < ST; ++u) {
        s4[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp4[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      {
        float kk[ST][C::KS], vv[ST][C::KS];
#pragma unroll
        for (int u = 0; u < ST; ++u) {
          row_operands<D, C::SA>(Ks, (sub + u) * 16 + lq, lg, kk[u]);
          row_operands<D, C::SA>(Vs, (sub + u) * 16 + lq, lg, vv[u]);
        }
#pragma unroll
        for (int s = 0; s < C::KS; ++s)
#pragma unroll
          for (int u = 0; u < ST; ++u) {
            s4[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(kk[u][s], qreg[s], s4[u], 0, 0, 0);
            dp4[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(vv[u][s], dreg[s], dp4[u], 0, 0, 0);
          }
      }
      float ds[ST][4];
#pragma unroll
      for (int u = 0; u < ST; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kl = (sub + u) * 16 + lg * 4 + r;
          const bool vis = qv && (k0 + kl < kmax) && !((qmask >> kl) & 1ull);
          const float e = __expf(s4[u][r] - lse);
          ds[u][r] = (vis ? e : 0.0f) * (dp4[u][r] - dl);
        }
#pragma unroll
      for (int u = 0; u < ST; ++u) {
        if (u == 1 && !two) break;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          float kk[C::DT];
          col_operands<D, C::SA>(Ks, (sub + u) * 16 + 4 * lg + s, lq, kk);
#pragma unroll
          for (int dt = 0; dt < C::DT; ++dt)
            dq[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(kk[dt], ds[u][s], dq[dt], 0, 0, 0);
        }
      }
    }
  }
  if (qv) {
    float* op = a.dq + (long)b * a.dq_bs + (long)qi * a.dq_ts + hoff;
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = dout<D>(lg, dt, r);
        if (d < D) op[d] = dq[dt][r] * a.scale;
      }
  }
}

// dK, dV for 64 keys of one (b, head): S = Q K^T (query rows), P, dP = dO V^T,
// dV^T += dO^T P, dK^T += Q^T dS
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(AttnArgs a) {
  using C = AttnCfg<D>;
  constexpr int ST = 1;
  __shared__ __attribute__((aligned(16))) float Qs[TT * C::SA];
  __shared__ __attribute__((aligned(16))) float Ds[TT * C::SA];
  __shared__ __attribute__((aligned(16))) float Ls[TT];
  __shared__ __attribute__((aligned(16))) float Dl[TT];
  const int h = blockIdx.x, b = blockIdx.y;
  const int kb0 = blockIdx.z * 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lk = lane & 15, lg = lane >> 4;
  const int kj = kb0 + wave * 16 + lk;
  const int hoff = h * D;
  const bool kv = kj < a.Tk;
  const bool pad = a.qpad && a.kpad;
  const bool kp = pad && kv && a.kpad[(long)b * a.Tk + kj];
  const int qmin = query_start(a, kj);
  const int wq0 = query_start(a, min(kb0 + wave * 16, a.Tk - 1));
  float kreg[C::KS], vreg[C::KS];
  row_values<D>(a.k + (long)b * a.k_bs + (long)min(kj, a.Tk - 1) * a.k_ts + hoff, lg, kv, kreg);
  row_values<D>(a.v + (long)b * a.v_bs + (long)min(kj, a.Tk - 1) * a.v_ts + hoff, lg, kv, vreg);
  f32x4 dkT[C::DT], dvT[C::DT];
#pragma unroll
  for (int dt = 0; dt < C::DT; ++dt) {
    dkT[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    dvT[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int qs = (query_start(a, kb0) / 16) * 16;
  const float* qb_ = a.q + (long)b * a.q_bs + hoff;
  const float* db_ = a.dout + (long)b * a.do_bs + hoff;
  const unsigned char* qpb = pad ? a.qpad + (long)b * a.qp_bs : nullptr;
  TileRegs<D> tq, td;
  unsigned char qpn = 0;  // padding flag of query qt0 + lane
  if (qs < a.Tq) {
    tq.load(qb_, a.q_ts, qs, a.Tq);
    td.load(db_, a.do_ts, qs, a.Tq);
    qpn = (pad && qs + lane < a.Tq) ? qpb[qs + lane] : 0;
  }
  for (int qt0 = qs; qt0 < a.Tq; qt0 += TT) {
    __syncthreads();
    tq.template store<C::SA>(Qs);
    td.template store<C::SA>(Ds);
    if (threadIdx.x < TT) {
      const int qq = qt0 + threadIdx.x;
      const long ri = stat_row(a, b, h, qq);
      Ls[threadIdx.x] = qq < a.Tq ? a.lse[ri] : 0.0f;
      Dl[threadIdx.x] = qq < a.Tq ? a.dlt[ri] : 0.0f;
    }
    const unsigned long long qbits = __ballot(qpn != 0);
    const unsigned long long kmask = kp ? qbits : 0ull;  // queries of this tile padding hides from key kj
    __syncthreads();
    if (qt0 + TT < a.Tq) {
      tq.load(qb_, a.q_ts, qt0 + TT, a.Tq);
      td.load(db_, a.do_ts, qt0 + TT, a.Tq);
      qpn = (pad && qt0 + TT + lane < a.Tq) ? qpb[qt0 + TT + lane] : 0;
    }
#pragma unroll
    for (int sub = 0; sub < TT / 16; sub += ST) {
      const int qb = qt0 + sub * 16;
      if (qb >= a.Tq) break;
      if (qb + 16 * ST <= wq0) continue;  // no query of these sub-tiles sees a key of this wave
      const bool two = ST == 2 && qb + 16 < a.Tq;
      f32x4 s4[ST], dp4[ST];
#pragma unroll
      for (int u = 0; u < ST; ++u) {
        s4[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp4[u] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      {
        float qq[ST][C::KS], dd[ST][C::KS];
#pragma unroll
        for (int u = 0; u < ST; ++u) {
          row_operands<D, C::SA>(Qs, (sub + u) * 16 + lk, lg, qq[u]);
          row_operands<D, C::SA>(Ds, (sub + u) * 16 + lk, lg, dd[u]);
        }
#pragma unroll
        for (int s = 0; s < C::KS; ++s)
#pragma unroll
          for (int u = 0; u < ST; ++u) {
            s4[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(qq[u][s], kreg[s], s4[u], 0, 0, 0);
            dp4[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(dd[u][s], vreg[s], dp4[u], 0, 0, 0);
          }
      }
      float p[ST][4], ds[ST][4];
#pragma unroll
      for (int u = 0; u < ST; ++u) {
        const int qr = (sub + u) * 16 + lg * 4;  // query row of accumulator register 0
        const float4 L4 = *reinterpret_cast<const float4*>(Ls + qr);
        const float4 D4 = *reinterpret_cast<const float4*>(Dl + qr);
        const float lv[4] = {L4.x, L4.y, L4.z, L4.w}, dv[4] = {D4.x, D4.y, D4.z, D4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qq = qt0 + qr + r;
          const bool vis = kv && qq >= qmin && qq < a.Tq && !((kmask >> (qr + r)) & 1ull);
          const float e = __expf(s4[u][r] * a.scale - lv[r]);
          p[u][r] = vis ? e : 0.0f;
          ds[u][r] = p[u][r] * (dp4[u][r] - dv[r]);
        }
      }
#pragma unroll
      for (int u = 0; u < ST; ++u) {
        if (u == 1 && !two) break;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          float dd[C::DT], qq[C::DT];
          col_operands<D, C::SA>(Ds, (sub + u) * 16 + 4 * lg + s, lk, dd);
          col_operands<D, C::SA>(Qs, (sub + u) * 16 + 4 * lg + s, lk, qq);
#pragma unroll
          for (int dt = 0; dt < C::DT; ++dt) {
            dvT[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(dd[dt], p[u][s], dvT[dt], 0, 0, 0);
            dkT[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(qq[dt], ds[u][s], dkT[dt], 0, 0, 0);
          }
        }
      }
    }
  }
  if (kv) {
    if (a.kv_acc) {   // a query chunk's share: add (the chunks run in a fixed order: deterministic)
      add_row<D>(a.dk + (long)b * a.dk_bs + (long)kj * a.dk_ts + hoff, lg, a.dkvvec, dkT, a.scale);
      add_row<D>(a.dv + (long)b * a.dv_bs + (long)kj * a.dv_ts + hoff, lg, a.dkvvec, dvT, 1.0f);
    } else {
      store_row<D>(a.dk + (long)b * a.dk_bs + (long)kj * a.dk_ts + hoff, lg, a.dkvvec, dkT, a.scale);
      store_row<D>(a.dv + (long)b * a.dv_bs + (long)kj * a.dv_ts + hoff, lg, a.dkvvec, dvT, 1.0f);
    }
  }
}

// Single-pass backward (D = 64, Tq <= 320 queries): ONE workgroup of 8 waves per (b, head) walks the
// key blocks of 128 keys (wave w keeps keys 16w..16w+15 of the block and their dK / dV accumulators in
// VGPRs, exactly as attn_bwd_dkv_kernel does) and, inside, the query tiles of 64 that see them; the
// dS tile of a (key block, query tile) pair goes to LDS and the eight waves turn it into that tile's
// dQ share at once (dQ += dS K over the block's keys; wave w holds the block's K columns of its d tile
// in VGPRs), accumulated in LDS for all Tq queries and written once at the end.  So Q, K, V, O and dO
// are read from HBM once and dQ, dK, dV written once (the two-pass form reads Q, dO, K and V twice and
// recomputes S and dP), with no atomics: the dQ shares add in key-block order, deterministic.
// delta = rowsum(dO * O) and lse of every query are formed in a prologue (LDS).  dK / dV sum the same
// products in the same order as the two-pass form (bitwise equal); dQ sums over keys in another order.
static constexpr int FKB = 128;          // keys per block (8 waves x 16)
static constexpr int FQT = 64;           // queries per tile
static constexpr int FTQ = 320;          // most queries per (b, head): the dQ accumulators live in LDS
static constexpr int FSQ = FKB + 4;      // dS tile row stride
template <int D>
struct FusedLds {
  static constexpr int SA = AttnCfg<D>::SA;
  static constexpr int QS = 0, DS = QS + FQT * SA, SS = DS + FQT * SA;
  // lse / delta rows: FTQ + FQT, so a tile's reads stay inside the arrays for any tile start
  // (they reach ceil16(Tq) - 1 < FTQ today, through the wave-uniform qb < Tq guard)
  static constexpr int QA = SS + FQT * FSQ, LS = QA + FTQ * SA, DL = LS + FTQ + FQT;
  static constexpr int FLOATS = DL + FTQ + FQT;
};

template <int D>
__global__ __launch_bounds__(512) void attn_bwd_fused_kernel(AttnArgs a) {
  static_assert(D == 64, "fused attention backward: D = 64 only");
  using C = AttnCfg<D>;
  using L = FusedLds<D>;
  constexpr int NT = FQT * (D / 4) / 512;   // float4 of a query tile per thread
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Qs = lds + L::QS;    // query tile rows [FQT][SA]
  float* Ds = lds + L::DS;    // dO tile rows
  float* Ss = lds + L::SS;    // dS of the pair [FQT query][FSQ key]
  float* Qa = lds + L::QA;    // dQ accumulators [FTQ][SA]
  float* Ls = lds + L::LS;    // lse of every query
  float* Dl = lds + L::DL;    // delta of every query
  const int h = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lk = lane & 15, lg = lane >> 4;
  const int hoff = h * D;
  const int Tq = a.Tq, Tk = a.Tk;
  const bool pad = a.qpad && a.kpad;
  const float* qb_ = a.q + (long)b * a.q_bs + hoff;
  const float* db_ = a.dout + (long)b * a.do_bs + hoff;
  const float* kb_ = a.k + (long)b * a.k_bs + hoff;
  const unsigned char* qpb = pad ? a.qpad + (long)b * a.qp_bs : nullptr;

  // prologue: 4 lanes per query (16 consecutive d each: the dQ kernel's lane-group split, so delta
  // sums in its order), 128 queries per pass
  for (int q0 = 0; q0 < Tq; q0 += 128) {
    const int q = q0 + (tid >> 2), g = tid & 3;
    float dsum = 0.0f;
    if (q < Tq) {
      const float* op = a.o + (long)b * a.o_bs + (long)q * a.o_ts + hoff + 16 * g;
      const float* dp = db_ + (long)q * a.do_ts + 16 * g;
#pragma unroll
      for (int i = 0; i < 16; i += 4) {
        const float4 o4 = *reinterpret_cast<const float4*>(op + i), d4 = *reinterpret_cast<const float4*>(dp + i);
        dsum = fmaf(d4.x, o4.x, dsum);
        dsum = fmaf(d4.y, o4.y, dsum);
        dsum = fmaf(d4.z, o4.z, dsum);
        dsum = fmaf(d4.w, o4.w, dsum);
      }
    }
    dsum += __shfl_xor(dsum, 1, 64);
    dsum += __shfl_xor(dsum, 2, 64);
    if (q < Tq && g == 0) {
      Dl[q] = dsum;
      Ls[q] = a.lse[stat_row(a, b, h, q)];
    }
  }
  for (int q = Tq + tid; q < FTQ + FQT; q += 512) {   // zeros past Tq: a sub-tile's rows beyond it read them (p = 0)
    Dl[q] = 0.0f;
    Ls[q] = 0.0f;
  }
  for (int i = tid; i < FTQ * C::SA / 4; i += 512)
    reinterpret_cast<float4*>(Qa)[i] = make_float4(0.f, 0.f, 0.f, 0.f);

  const int dtl = wave & 3;   // this wave's d tile of the dQ products
  for (int kb0 = 0; kb0 < Tk; kb0 += FKB) {
    const int kj = kb0 + wave * 16 + lk;
    const bool kv = kj < Tk;
    const bool wact = kb0 + wave * 16 < Tk;            // the wave holds some key
    const bool kp = pad && kv && a.kpad[(long)b * Tk + kj];
    const int qmin = query_start(a, kj);
    const int wq0 = query_start(a, min(kb0 + wave * 16, Tk - 1));
    float kreg[C::KS], vreg[C::KS];
    row_values<D>(kb_ + (long)min(kj, Tk - 1) * a.k_ts, lg, kv, kreg);
    row_values<D>(a.v + (long)b * a.v_bs + (long)min(kj, Tk - 1) * a.v_ts + hoff, lg, kv, vreg);
    // the dQ products' K operand: K[kb0 + 16m + 4lg + i][16 dtl + lk], m < 8, i < 4
    float kd[FKB / 4];
#pragma unroll
    for (int m = 0; m < FKB / 16; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kb0 + 16 * m + 4 * lg + i;
        kd[4 * m + i] = key < Tk ? kb_[(long)key * a.k_ts + 16 * dtl + lk] : 0.0f;
      }
    f32x4 dkT[C::DT], dvT[C::DT];
#pragma unroll
    for (int dt = 0; dt < C::DT; ++dt) {
      dkT[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
      dvT[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int qs = (query_start(a, kb0) / 16) * 16;
    float4 rq[NT], rd[NT];
    unsigned char qpn = 0;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int e = tid + 512 * j, q = qs + (e >> 4), c = (e & 15) * 4;
      rq[j] = rd[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q < Tq) {
        rq[j] = *reinterpret_cast<const float4*>(qb_ + (long)q * a.q_ts + c);
        rd[j] = *reinterpret_cast<const float4*>(db_ + (long)q * a.do_ts + c);
      }
    }
    qpn = (pad && qs + lane < Tq) ? qpb[qs + lane] : 0;
    for (int qt0 = qs; qt0 < Tq; qt0 += FQT) {
      __syncthreads();   // the previous tile's dS / dQ products are done
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int e = tid + 512 * j, row = e >> 4, c = (e & 15) * 4;
        *reinterpret_cast<float4*>(Qs + row * C::SA + c) = rq[j];
        *reinterpret_cast<float4*>(Ds + row * C::SA + c) = rd[j];
      }
      const unsigned long long qbits = __ballot(qpn != 0);
      const unsigned long long kmask = kp ? qbits : 0ull;   // queries of this tile padding hides from key kj
      __syncthreads();
      if (qt0 + FQT < Tq) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int e = tid + 512 * j, q = qt0 + FQT + (e >> 4), c = (e & 15) * 4;
          rq[j] = rd[j] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (q < Tq) {
            rq[j] = *reinterpret_cast<const float4*>(qb_ + (long)q * a.q_ts + c);
            rd[j] = *reinterpret_cast<const float4*>(db_ + (long)q * a.do_ts + c);
          }
        }
        qpn = (pad && qt0 + FQT + lane < Tq) ? qpb[qt0 + FQT + lane] : 0;
      }
#pragma unroll
      for (int u = 0; u < FQT / 16; ++u) {
        const int qb = qt0 + u * 16;
        float ds[4] = {0.f, 0.f, 0.f, 0.f};
        if (wact && qb < Tq && qb + 16 > wq0) {   // wave-uniform: some query of the sub-tile sees a key of the wave
          f32x4 s4 = f32x4{0.f, 0.f, 0.f, 0.f}, dp4 = s4;
          {
            float qq[C::KS], dd[C::KS];
            row_operands<D, C::SA>(Qs, u * 16 + lk, lg, qq);
            row_operands<D, C::SA>(Ds, u * 16 + lk, lg, dd);
#pragma unroll
            for (int s = 0; s < C::KS; ++s) {
              s4 = __builtin_amdgcn_mfma_f32_16x16x4f32(qq[s], kreg[s], s4, 0, 0, 0);
              dp4 = __builtin_amdgcn_mfma_f32_16x16x4f32(dd[s], vreg[s], dp4, 0, 0, 0);
            }
          }
          const int ql = u * 16 + lg * 4;   // tile-local query of accumulator register 0
          const float4 L4 = *reinterpret_cast<const float4*>(Ls + qt0 + ql);
          const float4 D4 = *reinterpret_cast<const float4*>(Dl + qt0 + ql);
          const float lv[4] = {L4.x, L4.y, L4.z, L4.w}, dv[4] = {D4.x, D4.y, D4.z, D4.w};
          float p[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int qq = qt0 + ql + r;
            const bool vis = kv && qq >= qmin && qq < Tq && !((kmask >> (ql + r)) & 1ull);
            const float e = __expf(s4[r] * a.scale - lv[r]);
            p[r] = vis ? e : 0.0f;
            ds[r] = p[r] * (dp4[r] - dv[r]);
          }
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            float dd[C::DT], qq[C::DT];
            col_operands<D, C::SA>(Ds, u * 16 + 4 * lg + s, lk, dd);
            col_operands<D, C::SA>(Qs, u * 16 + 4 * lg + s, lk, qq);
#pragma unroll
            for (int dt = 0; dt < C::DT; ++dt) {
              dvT[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(dd[dt], p[s], dvT[dt], 0, 0, 0);
              dkT[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(qq[dt], ds[s], dkT[dt], 0, 0, 0);
            }
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Ss[(u * 16 + lg * 4 + r) * FSQ + wave * 16 + lk] = ds[r];
      }
      __syncthreads();
      // dQ shares of the tile: wave w -> d tile w & 3 of query sub-tiles (w >> 2) and (w >> 2) + 2;
      // C[d][q] = K^T dS^T over the keys any of the sub-tile's queries sees (k-step 4m + i of lane
      // group lg: key 16m + 4lg + i)
#pragma unroll
      for (int hq = 0; hq < 2; ++hq) {
        const int qu = (wave >> 2) + 2 * hq;
        const int qr0 = qt0 + qu * 16;
        if (qr0 < Tq) {
          const int kend = min(key_bound(a, min(qr0 + 15, Tq - 1)) - kb0, FKB);
          const int nm = (kend + 15) / 16;
          f32x4 c0 = f32x4{0.f, 0.f, 0.f, 0.f}, c1 = c0;
          const float* srow = Ss + (qu * 16 + lk) * FSQ + 4 * lg;
#pragma unroll
          for (int m = 0; m < FKB / 16; ++m) {
            if (m < nm) {
              const float4 sv = *reinterpret_cast<const float4*>(srow + 16 * m);
              c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kd[4 * m], sv.x, c0, 0, 0, 0);
              c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kd[4 * m + 1], sv.y, c1, 0, 0, 0);
              c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(kd[4 * m + 2], sv.z, c0, 0, 0, 0);
              c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(kd[4 * m + 3], sv.w, c1, 0, 0, 0);
            }
          }
          if (nm > 0) {
            float4* qa = reinterpret_cast<float4*>(Qa + (qr0 + lk) * C::SA + dtl * 16 + 4 * lg);
            const float4 o = *qa;
            *qa = make_float4(o.x + (c0[0] + c1[0]), o.y + (c0[1] + c1[1]), o.z + (c0[2] + c1[2]),
                              o.w + (c0[3] + c1[3]));
          }
        }
      }
    }
    if (kv) {
      store_row<D>(a.dk + (long)b * a.dk_bs + (long)kj * a.dk_ts + hoff, lg, 1, dkT, a.scale);
      store_row<D>(a.dv + (long)b * a.dv_bs + (long)kj * a.dv_ts + hoff, lg, 1, dvT, 1.0f);
    }
  }
  __syncthreads();
  float* dqb = a.dq + (long)b * a.dq_bs + hoff;
  for (int e = tid; e < Tq * (D / 4); e += 512) {
    const int q = e >> 4, c = (e & 15) * 4;
    const float4 v4 = *reinterpret_cast<const float4*>(Qa + q * C::SA + c);
    *reinterpret_cast<float4*>(dqb + (long)q * a.dq_ts + c) =
        make_float4(v4.x * a.scale, v4.y * a.scale, v4.z * a.scale, v4.w * a.scale);
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
  a.q_off = 0; a.Tqf = Tq; a.qp_bs = Tq; a.kv_acc = 0; a.st_ld = Tq; a.st_off = 0;
  return a;
}

// single-pass backward (attn_bwd_fused_kernel) where it applies: 1 (default) or 0 (MRG_ATTN_FUSED,
// mrg_attention_set_fused: the two-pass form always)
static int g_attn_fused = [] {
  const char* e = getenv("MRG_ATTN_FUSED");
  return e ? atoi(e) : 1;
}();

MRG_API int mrg_attention_set_fused(int on) {
  const int prev = g_attn_fused;
  g_attn_fused = on ? 1 : 0;
  return prev;
}

static bool rows16(const float* p, long bs, long ts) {
  return p == nullptr || ((((uintptr_t)p) & 15) == 0 && (bs & 3) == 0 && (ts & 3) == 0);
}

static int attn_check(int D, int Tq, int Tk, int causal) {
  MRG_REQUIRE(D == 8 || D == 16 || D == 32 || D == 64, "attention: unsupported head dim %d", D);
  MRG_REQUIRE(!causal || Tq == 0 || Tk == 0 || Tk % Tq == 0 || Tq % Tk == 0,
              "attention: other_modal_len must be divisible by main_modal_len (Tq=%d Tk=%d)", Tq, Tk);
  return 0;
}

#define MRG_ATTN_DISPATCH(KERNEL, grid, args)                          \
  switch (D) {                                                         \
    case 8: klaunch(KERNEL<8>, grid, 256, 0, stream, args); break;         \
    case 16: klaunch(KERNEL<16>, grid, 256, 0, stream, args); break;       \
    case 32: klaunch(KERNEL<32>, grid, 256, 0, stream, args); break;       \
    case 64: klaunch(KERNEL<64>, grid, 256, 0, stream, args); break;       \
  }

MRG_API int mrg_attention_fwd(int B, int Hh, int Tq, int Tk, int D,
                              const float* q, long q_bs, long q_ts, const float* k, long k_bs, long k_ts,
                              const float* v, long v_bs, long v_ts, float* o, long o_bs, long o_ts,
                              float* lse, const unsigned char* qpad, const unsigned char* kpad,
                              int causal, float scale, hipStream_t stream) {
  if (int e = attn_check(D, Tq, Tk, causal)) return e;
  if (B == 0 || Tq == 0) return 0;
  MRG_REQUIRE(rows16(k, k_bs, k_ts) && rows16(v, v_bs, v_ts),
              "attention fwd: K/V rows must be 16-B aligned (strides multiple of 4 floats)");
  AttnArgs a = attn_base(B, Hh, Tq, Tk, q, q_bs, q_ts, k, k_bs, k_ts, v, v_bs, v_ts, o, o_bs, o_ts, lse,
                         qpad, kpad, causal, scale);
  a.qvec = rows16(q, q_bs, q_ts) && (D % 4) == 0;
  a.ovec = rows16(o, o_bs, o_ts) && (D % 4) == 0;
  dim3 grid(Hh, B, (Tq + 63) / 64);
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
  MRG_REQUIRE(rows16(q, q_bs, q_ts) && rows16(k, k_bs, k_ts) && rows16(v, v_bs, v_ts) &&
              rows16(dout, do_bs, do_ts), "attention bwd: Q/K/V/dO rows must be 16-B aligned");
  MRG_REQUIRE(workspace != nullptr, "attention bwd: workspace (B*heads*Tq floats) required");
  AttnArgs a = attn_base(B, Hh, Tq, Tk, q, q_bs, q_ts, k, k_bs, k_ts, v, v_bs, v_ts, o, o_bs, o_ts, lse,
                         qpad, kpad, causal, scale);
  a.dout = dout; a.do_bs = do_bs; a.do_ts = do_ts; a.dlt = workspace;
  a.dq = dq; a.dq_bs = dq_bs; a.dq_ts = dq_ts; a.dk = dk; a.dk_bs = dk_bs; a.dk_ts = dk_ts;
  a.dv = dv; a.dv_bs = dv_bs; a.dv_ts = dv_ts;
  a.qvec = 1;  // required above
  a.ovec = rows16(o, o_bs, o_ts);
  a.dkvvec = rows16(dk, dk_bs, dk_ts) && rows16(dv, dv_bs, dv_ts);
  if (g_attn_fused && D == 64 && Tq <= FTQ && rows16(o, o_bs, o_ts) && a.dkvvec && rows16(dq, dq_bs, dq_ts)) {
    static bool attr[64] = {};   // the LDS size attribute, set once per device
    constexpr int bytes = FusedLds<64>::FLOATS * (int)sizeof(float);
    static_assert(bytes <= 160 * 1024, "fused attention backward: LDS layout exceeds a CU's 160 KB");
    int dev = 0;
    MRG_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64 || !attr[dev]) {
      MRG_HIP(hipFuncSetAttribute((const void*)attn_bwd_fused_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  bytes));
      if (dev >= 0 && dev < 64) attr[dev] = true;
    }
    klaunch(attn_bwd_fused_kernel<64>, dim3(Hh, B), 512, bytes, stream, a);
    return check_launch("attn_bwd_fused_kernel");
  }
  dim3 gq(Hh, B, (Tq + 63) / 64);
  MRG_ATTN_DISPATCH(attn_bwd_dq_kernel, gq, a);  // also writes delta = rowsum(dO * O) to the workspace
  if (check_launch("attn_bwd_dq_kernel")) return 1;
  dim3 gk(Hh, B, (Tk + 63) / 64);
  MRG_ATTN_DISPATCH(attn_bwd_dkv_kernel, gk, a);
  return check_launch("attn_bwd_dkv_kernel");
}

// Query-chunk forms (the block-level (block, time-chunk) wavefront, block_stack.py): the Tq query
// rows handed in (q, o, dout, dq: pointers to the chunk's first row) are rows [q_off, q_off + Tq) of
// a Tq_full-query sequence; lse, the workspace (delta) and qpad are the whole sequence's
// [B, heads, Tq_full] / [B, Tq_full] arrays (the chunk's columns at q_off).  bwd passes: 1 = dQ (+ the
// chunk's delta into the workspace), 2 = dK / dV from the lse / delta already there (a later call
// over q_off = 0, Tq = Tq_full: the whole sequence's dK / dV once every chunk's dQ pass has run), 3 =
// both; with kv_accumulate = 1 the dK / dV pass ADDS the chunk's share (only the key blocks some
// query of the chunk sees are touched).
MRG_API int mrg_attention_fwd_chunk(int B, int Hh, int Tq, int Tk, int D, int q_off, int Tq_full,
                                    const float* q, long q_bs, long q_ts, const float* k, long k_bs, long k_ts,
                                    const float* v, long v_bs, long v_ts, float* o, long o_bs, long o_ts,
                                    float* lse, const unsigned char* qpad, const unsigned char* kpad,
                                    int causal, float scale, hipStream_t stream) {
  if (int e = attn_check(D, Tq_full, Tk, causal)) return e;
  MRG_REQUIRE(q_off >= 0 && Tq >= 0 && q_off + Tq <= Tq_full, "attention fwd chunk: rows [%d, %d) outside %d",
              q_off, q_off + Tq, Tq_full);
  if (B == 0 || Tq == 0) return 0;
  MRG_REQUIRE(rows16(k, k_bs, k_ts) && rows16(v, v_bs, v_ts),
              "attention fwd: K/V rows must be 16-B aligned (strides multiple of 4 floats)");
  AttnArgs a = attn_base(B, Hh, Tq, Tk, q, q_bs, q_ts, k, k_bs, k_ts, v, v_bs, v_ts, o, o_bs, o_ts, lse,
                         qpad ? qpad + q_off : nullptr, kpad, causal, scale);
  a.q_off = q_off; a.Tqf = Tq_full; a.qp_bs = Tq_full; a.st_ld = Tq_full; a.st_off = q_off;
  a.qvec = rows16(q, q_bs, q_ts) && (D % 4) == 0;
  a.ovec = rows16(o, o_bs, o_ts) && (D % 4) == 0;
  dim3 grid(Hh, B, (Tq + 63) / 64);
  MRG_ATTN_DISPATCH(attn_fwd_kernel, grid, a);
  return check_launch("attn_fwd_kernel");
}

MRG_API int mrg_attention_bwd_chunk(int B, int Hh, int Tq, int Tk, int D, int q_off, int Tq_full,
                                    const float* q, long q_bs, long q_ts, const float* k, long k_bs, long k_ts,
                                    const float* v, long v_bs, long v_ts, const float* o, long o_bs, long o_ts,
                                    const float* lse, const unsigned char* qpad, const unsigned char* kpad,
                                    int causal, float scale, const float* dout, long do_bs, long do_ts,
                                    float* dq, long dq_bs, long dq_ts, float* dk, long dk_bs, long dk_ts,
                                    float* dv, long dv_bs, long dv_ts, int passes, int kv_accumulate,
                                    float* workspace, hipStream_t stream) {
  if (int e = attn_check(D, Tq_full, Tk, causal)) return e;
  MRG_REQUIRE(q_off >= 0 && Tq >= 0 && q_off + Tq <= Tq_full, "attention bwd chunk: rows [%d, %d) outside %d",
              q_off, q_off + Tq, Tq_full);
  if (B == 0 || Tq == 0 || Tk == 0) return 0;
  MRG_REQUIRE(rows16(q, q_bs, q_ts) && rows16(k, k_bs, k_ts) && rows16(v, v_bs, v_ts) &&
              rows16(dout, do_bs, do_ts), "attention bwd: Q/K/V/dO rows must be 16-B aligned");
  MRG_REQUIRE(workspace != nullptr, "attention bwd: workspace (B*heads*Tq_full floats) required");
  MRG_REQUIRE(passes >= 1 && passes <= 3, "attention bwd chunk: passes %d (1 dQ, 2 dK/dV, 3 both)", passes);
  AttnArgs a = attn_base(B, Hh, Tq, Tk, q, q_bs, q_ts, k, k_bs, k_ts, v, v_bs, v_ts, o, o_bs, o_ts, lse,
                         qpad ? qpad + q_off : nullptr, kpad, causal, scale);
  a.q_off = q_off; a.Tqf = Tq_full; a.qp_bs = Tq_full; a.kv_acc = kv_accumulate ? 1 : 0;
  a.st_ld = Tq_full; a.st_off = q_off;
  a.dout = dout; a.do_bs = do_bs; a.do_ts = do_ts; a.dlt = workspace;
  a.dq = dq; a.dq_bs = dq_bs; a.dq_ts = dq_ts; a.dk = dk; a.dk_bs = dk_bs; a.dk_ts = dk_ts;
  a.dv = dv; a.dv_bs = dv_bs; a.dv_ts = dv_ts;
  a.qvec = 1;
  a.ovec = rows16(o, o_bs, o_ts);
  a.dkvvec = rows16(dk, dk_bs, dk_ts) && rows16(dv, dv_bs, dv_ts);
  if (passes & 1) {   // dQ and delta (the dK / dV pass reads delta from the workspace)
    dim3 gq(Hh, B, (Tq + 63) / 64);
    MRG_ATTN_DISPATCH(attn_bwd_dq_kernel, gq, a);
    if (check_launch("attn_bwd_dq_kernel")) return 1;
  }
  if (!(passes & 2)) return 0;
  // accumulating: only the key blocks the chunk's last query can see (the rest get nothing)
  int tk = Tk;
  if (a.kv_acc && causal) {
    const int gl = q_off + Tq - 1;
    tk = (Tk >= Tq_full) ? (gl + 1) * (Tk / Tq_full) : gl / (Tq_full / Tk) + 1;
    tk = tk < Tk ? tk : Tk;
  }
  dim3 gk(Hh, B, (tk + 63) / 64);
  MRG_ATTN_DISPATCH(attn_bwd_dkv_kernel, gk, a);
  return check_launch("attn_bwd_dkv_kernel");
}
