// Persistent scheduled-sampling decode forward of lstm_with_sampling (BASELINE configs[2]): the whole
// frame loop of decode.hip's per-frame launches (layer-1 gate/cell with the features, the sampling
// select and the previous frame's FFN output; layer l > 1 gate/cell on LayerNorm(h + x) of layer l-1;
// last LayerNorm + FFN first Linear) in ONE launch.
//
// Reference: LSTMwithSample.prediction -> head_motion_generation -> generate_one_step
// (mr_gen/model/lstm_with_sampling/lstm_with_sample.py:339-433), the same chain as decode.hip.
//
// Decomposition.  Every op of a frame is row-wise in the batch, so the batch is cut into row tiles of
// 16 (one 16 x 16 exact-f32 MFMA tile, as decode.hip) and each tile is served by G = H / 4 workgroups
// ("members"); member j owns hidden units 4j .. 4j+3 of every layer (its 16 gate rows of each W_ih
// live in LDS for the whole launch, read from HBM once) and FFN outputs j, j + G, ...  Per frame a
// member: builds its tile's layer input (every member recomputes the 16 x H rows it needs: P(t) plus
// the ms columns through W_ms, or the LayerNorm of the layer below), runs its 16 x 16 gate tile and
// the zero-state cells, publishes its 16 x 4 h values as {tag, value} granules (lstm_common.h), and
// gathers the full 16 x H rows of the layer below from all members before the next layer; the FFN's
// z columns are handed off the same way to the next frame's layer 1.  Tags are frame + 1, the rings
// 2-deep by frame parity (a member publishes frame t + 2 only after gathering frame t + 1 from every
// member, which each produced after finishing its reads of frame t).  A tile whose members all run on
// one XCD (checked at launch start) publishes with workgroup-scope stores that keep the lines in that
// XCD's L2; otherwise agent-scope.  Every spin is bounded and reports through *err.
//
// Arithmetic: the same per-element operation order as decode.hip's per-frame kernels (f32 MFMA tile,
// fixed-order wave reduction, LayerNorm lane-group sums, FFN lane-phase sums), so both forms agree to
// fp32 rounding of identical expressions (tests/test_gpu_models.py checks them against each other).
#include "lstm_common.h"

namespace mrg {

static constexpr int SSDP_R = 16;     // batch rows per tile
static constexpr int SSDP_MAXL = 4;   // layers
typedef float ssdp_f32x4 __attribute__((ext_vector_type(4)));

struct SsdPersistLayer {
  const float* w_ih;   // [4H][H]
  const float* b_ih;
  const float* b_hh;
  const float* ln_w;   // this layer's LayerNorm (applied to h + x by the next stage)
  const float* ln_b;
  float* x;            // saved layer input X [T][B][H]
  float* gates;        // [T][B][4H]
  float* c;            // [T][B][H]
  float* h;            // [T][B][H]
  float* mean;         // [T][B] LayerNorm statistics of this layer's output
  float* rstd;
};

struct SsdPersistArgs {
  int B, H, HB, FO, F, T, nl;
  float eps;
  const float* p;                 // P [T][B][H] (features through W_a, W_mp, bias)
  const float* ms;                // ms[b * ms_bs + t * ms_ts + o]
  long ms_bs, ms_ts;
  const unsigned char* mask;      // [T]
  const float* wms;               // W_ms^T [FO][H]
  const float* w1;                // [HB][H]
  const float* b1;
  const float* w2;                // [FO][HB]
  const float* b2;
  float* u;                       // [T][B][H] last LayerNorm output
  float* z;                       // [T][B][HB]
  float* y;                       // y(t)[b * y_bs + t * FO + o] for t < T - 1 (the last by ssd_y_kernel)
  long y_bs;
  float* xf_ms;                   // ms_in(t) -> xf_ms[t * B * F + b * F + o]
  unsigned long long* ring_h;     // [nl][2][B][H] granules
  unsigned long long* ring_z;     // [2][B][HB] granules
  unsigned long long* xcc_slots;  // [NR][G]: each member's XCC id (the launch-start placement check)
  int* err;
  unsigned long long* stamps;     // diagnostics: block 0's phase wall clocks [T][8] (null in normal use)
  SsdPersistLayer L[SSDP_MAXL];
};

#define SSDP_STAMP(ph)                                                                 \
  do {                                                                                 \
    if (a.stamps && blockIdx.x == 0 && threadIdx.x == 0) a.stamps[(long)t * 8 + (ph)] = wall_clock64(); \
  } while (0)

__device__ __forceinline__ float4 ssdp_ld4(const float* p, long idx, bool ok) {
  return ok ? *reinterpret_cast<const float4*>(p + idx) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Block -> (row tile, member): a tile's members share blockIdx % 8 (one XCD under the observed round-robin
// dispatch; checked at launch start, placement never decides correctness) -- tiles are dealt over
// NR8 = 8 ceil(NR / 8) slots and the blocks of the slots past NR return at once.  With two workgroups
// per CU a tile's 64 members fit one XCD's 32 CUs, so their hand-offs stay in that XCD's L2
// (workgroup-scope granule stores, as lstm.hip's groups): agent-scope ones sent every poll of the
// 64 x 16 x H gathers per stage to the memory side (C3 13.4 ms vs 12.2 with per-frame launches).
template <int EPL, int MAXL>
__global__ __launch_bounds__(256, 2) void ssd_fwd_persist_kernel(SsdPersistArgs a) {
  constexpr int HMAX = EPL * 64, GL = HMAX / 4;           // GL lanes (x 4 columns) per row
  constexpr int LDK = HMAX + 2;
  constexpr int NX = SSDP_R * GL / 256 > 0 ? SSDP_R * GL / 256 : 1;   // float4 per thread of a tile
  __shared__ __attribute__((aligned(16))) float Ws[MAXL][16 * LDK];
  // the stage's input tile; the gathers of the layer below land here first (each thread then reads
  // and rewrites only its own elements: LayerNorm(h + x) -> X)
  __shared__ __attribute__((aligned(16))) float Xs[SSDP_R * LDK];
  __shared__ float red[4][16][17];
  __shared__ float bias[MAXL][16];
  __shared__ int xcc_flag;
  __shared__ float zs[SSDP_R][65];
  __shared__ float w2s[8][64];
  __shared__ float msin[SSDP_R][8];
  __shared__ __attribute__((aligned(16))) float w1s[4][HMAX];        // this member's FFN rows (<= 4)
  __shared__ float4 wms[8][GL];                                      // W_ms^T (LDS: registers are short)
  __shared__ float4 lnp[MAXL][2][GL];                                // every LayerNorm's gamma / beta
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, H4 = H / 4, B = a.B, T = a.T, nl = a.nl, HB = a.HB, FO = a.FO;
  const int G = H / 4;                                     // members per row tile
  const int NR = (B + SSDP_R - 1) / SSDP_R, NR8 = 8 * ((NR + 7) / 8);
  const int rt = blockIdx.x % NR8, j = blockIdx.x / NR8;
  if (rt >= NR) return;
  const int r0 = rt * SSDP_R, u0 = 4 * j;
  const int c4 = tid % GL;
  const bool cv = c4 < H4;
  const int nz = (HB - j + G - 1) / G;                      // FFN outputs j, j + G, ... of this member
  bool dead = false;
  // local (workgroup-scope) granule stores when every member of the tile runs on this XCD
  int local;
  {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long* slots = a.xcc_slots + (long)rt * G;
    if (tid == 0) {
      xcc_flag = 1;
      __hip_atomic_store(slots + j, make_granule(XCC_TAG, __uint_as_float(xcc)), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (tid < G) {
      float id[1];
      get_granules<1>(slots + tid, 1, XCC_TAG, id, a.err, dead);
      if (__float_as_uint(id[0]) != xcc) xcc_flag = 0;
    }
    __syncthreads();
    local = xcc_flag;
  }

  // ---- resident operands
  for (int l = 0; l < nl; ++l) {
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int rr = (tid + i * 256) / GL, q = rr >> 2, uu = rr & 3;
      const float4 w = ssdp_ld4(a.L[l].w_ih, (long)(q * H + u0 + uu) * H + 4 * c4, rr < 16 && cv);
      if (rr < 16) {
        float2* wd = reinterpret_cast<float2*>(&Ws[l][rr * LDK + 4 * c4]);
        wd[0] = make_float2(w.x, w.y);
        wd[1] = make_float2(w.z, w.w);
      }
    }
    if (tid < 16) {
      const int q = tid >> 2, uu = tid & 3;
      bias[l][tid] = a.L[l].b_ih[q * H + u0 + uu] + a.L[l].b_hh[q * H + u0 + uu];
    }
  }
  for (int e = tid; e < 4 * HMAX; e += 256) {
    const int zi = e / HMAX, k = e % HMAX, jj = j + zi * G;
    w1s[zi][k] = (zi < nz && k < H) ? a.w1[(long)jj * H + k] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + i * 256, o = e >> 6, jj = e & 63;
    w2s[o][jj] = (o < FO && jj < HB) ? a.w2[(long)o * HB + jj] : 0.0f;
  }
  for (int e = tid; e < 8 * GL; e += 256) {
    const int o = e / GL, cc = e % GL;
    wms[o][cc] = ssdp_ld4(a.wms, (long)o * H + 4 * cc, o < FO && cc < H4);
  }
  for (int e = tid; e < nl * 2 * GL; e += 256) {
    const int l = e / (2 * GL), w = (e / GL) & 1, cc = e % GL;
    lnp[l][w][cc] = ssdp_ld4(w ? a.L[l].ln_b : a.L[l].ln_w, 4 * cc, cc < H4);
  }
  const int rs_ = tid >> 3, os_ = tid & 7, bs_ = r0 + rs_;
  const bool svalid = tid < SSDP_R * 8 && os_ < FO && bs_ < B;
  const float b2v = svalid ? a.b2[os_] : 0.0f;
  // per-frame scalars off the chain: frame t's ms[.][t - 1] and mask[t - 1] are loaded during frame t - 1
  float msv_next = svalid ? a.ms[(long)bs_ * a.ms_bs + os_] : 0.0f;   // frame 0: ms[.][0]
  bool sel_next = false;
  // the FFN thread roles: output zi of this member, row r, k phase ph (decode.hip's ssd_ffn_z order)
  const int fr = (tid >> 2) & 15, fph = tid & 3, fzi = tid >> 6;
  const float b1v = (fzi < nz) ? a.b1[j + fzi * G] : 0.0f;
  // P(t) of this tile, prefetched a frame ahead
  float4 pv[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int rr = (tid + i * 256) / GL, b = r0 + rr;
    pv[i] = ssdp_ld4(a.p, (long)b * H + 4 * c4, rr < SSDP_R && b < B && cv);
  }
  __syncthreads();

  float4 xv[NX];   // this thread's part of the current layer input
  for (int t = 0; t < T; ++t) {
    const int par = t & 1;
    SSDP_STAMP(0);
    // ================= layer 1 input: X = P(t) + ms_in(t) W_ms^T
    {
      const bool fed = t > 0;
      const int tm = t > 0 ? t - 1 : 0;
      if (fed && !dead) {   // z(t-1) of the tile's rows from every member's FFN columns
        constexpr int NZ = (SSDP_R * 64 + 255) / 256;
        int idx[NZ];
        float gv[NZ];
        const int nvalid = min(SSDP_R, B - r0) * HB;
#pragma unroll
        for (int i = 0; i < NZ; ++i) idx[i] = min(tid + i * 256, nvalid - 1);
        unsigned long long* rz = a.ring_z + ((long)(tm & 1) * B + r0) * HB;
        get_granules_idx<NZ>(rz, idx, (unsigned)t, gv, a.err, dead);
#pragma unroll
        for (int i = 0; i < NZ; ++i) {
          const int e = tid + i * 256;
          if (e < SSDP_R * 64) {
            const int r = e / HB, jj = e % HB;
            if (e < nvalid) zs[r][jj] = gv[i];
          }
        }
      }
      SSDP_STAMP(1);
      const float msv = msv_next;
      const bool sel = fed && sel_next;
      if (t + 1 < T) {   // for frame t + 1: ms[.][t] and mask[t]
        msv_next = svalid ? a.ms[(long)bs_ * a.ms_bs + (long)t * a.ms_ts + os_] : 0.0f;
        sel_next = a.mask[t] != 0;
      }
      __syncthreads();
      if (tid < SSDP_R * 8) {
        float m = 0.0f;
        if (svalid) {
          float yv = b2v;
          if (fed) {
#pragma unroll 16
            for (int jj = 0; jj < 64; ++jj) yv = fmaf(jj < HB ? zs[rs_][jj] : 0.0f, w2s[os_][jj], yv);
            if (j == 0) a.y[(long)bs_ * a.y_bs + (long)tm * FO + os_] = yv;
          }
          m = sel ? yv : msv;
          if (j == 0) a.xf_ms[(long)t * B * a.F + (long)bs_ * a.F + os_] = m;
        }
        msin[rs_][os_] = m;
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        const int rr = (tid + i * 256) / GL;
        xv[i] = pv[i];
        if (rr >= SSDP_R) continue;
#pragma unroll
        for (int o = 0; o < 8; ++o) {
          const float mo = msin[rr][o];
          const float4 w = wms[o][c4];
          xv[i].x = fmaf(mo, w.x, xv[i].x); xv[i].y = fmaf(mo, w.y, xv[i].y);
          xv[i].z = fmaf(mo, w.z, xv[i].z); xv[i].w = fmaf(mo, w.w, xv[i].w);
        }
      }
      if (t + 1 < T) {   // next frame's P rows, off the chain
#pragma unroll
        for (int i = 0; i < NX; ++i) {
          const int rr = (tid + i * 256) / GL, b = r0 + rr;
          pv[i] = ssdp_ld4(a.p, (long)(t + 1) * B * H + (long)b * H + 4 * c4, rr < SSDP_R && b < B && cv);
        }
      }
    }
    for (int l = 0; l < nl; ++l) {
      const SsdPersistLayer& L = a.L[l];
      if (l > 0) {
        // gather h of layer l-1 (all H units of the tile's rows), then X = LayerNorm(h + x)
        const SsdPersistLayer& P = a.L[l - 1];
        if (!dead) {
          constexpr int NGH = SSDP_R * HMAX / 256;
          int idx[NGH];
          float gv[NGH];
          const int nvalid = min(SSDP_R, B - r0) * H;
#pragma unroll
          for (int i = 0; i < NGH; ++i) idx[i] = min(tid + i * 256, nvalid - 1);
          unsigned long long* rh = a.ring_h + (((long)(l - 1) * 2 + par) * B + r0) * H;
          get_granules_idx<NGH>(rh, idx, (unsigned)(t + 1), gv, a.err, dead);
#pragma unroll
          for (int i = 0; i < NGH; ++i) {
            const int e = tid + i * 256;
            if (e < nvalid) Xs[(e / H) * LDK + e % H] = gv[i];
          }
        }
        SSDP_STAMP(3);
        __syncthreads();
        const float4 g = lnp[l - 1][0][c4], bt = lnp[l - 1][1][c4];
        float s[NX], qv[NX];
#pragma unroll
        for (int i = 0; i < NX; ++i) {
          const int rr = (tid + i * 256) / GL;
          float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
          if (rr < SSDP_R && cv) {
            const float2* hs = reinterpret_cast<const float2*>(&Xs[rr * LDK + 4 * c4]);
            const float2 h0 = hs[0], h1 = hs[1];
            hv = make_float4(h0.x, h0.y, h1.x, h1.y);
          }
          xv[i].x = hv.x + xv[i].x; xv[i].y = hv.y + xv[i].y; xv[i].z = hv.z + xv[i].z; xv[i].w = hv.w + xv[i].w;
          s[i] = (xv[i].x + xv[i].y) + (xv[i].z + xv[i].w);
        }
#pragma unroll
        for (int o = 1; o < GL; o <<= 1)
#pragma unroll
          for (int i = 0; i < NX; ++i) s[i] += __shfl_xor(s[i], o, 64);
#pragma unroll
        for (int i = 0; i < NX; ++i) {
          s[i] /= (float)H;
          const float d0 = xv[i].x - s[i], d1 = xv[i].y - s[i], d2 = xv[i].z - s[i], d3 = xv[i].w - s[i];
          qv[i] = cv ? (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3) : 0.0f;
        }
#pragma unroll
        for (int o = 1; o < GL; o <<= 1)
#pragma unroll
          for (int i = 0; i < NX; ++i) qv[i] += __shfl_xor(qv[i], o, 64);
#pragma unroll
        for (int i = 0; i < NX; ++i) {
          const float rs = rsqrtf(qv[i] / (float)H + a.eps);
          xv[i].x = (xv[i].x - s[i]) * rs * g.x + bt.x; xv[i].y = (xv[i].y - s[i]) * rs * g.y + bt.y;
          xv[i].z = (xv[i].z - s[i]) * rs * g.z + bt.z; xv[i].w = (xv[i].w - s[i]) * rs * g.w + bt.w;
          const int rr = (tid + i * 256) / GL, b = r0 + rr;
          if (j == 0 && c4 == 0 && rr < SSDP_R && b < B) {
            P.mean[(long)t * B + b] = s[i];
            P.rstd[(long)t * B + b] = rs;
          }
        }
      }
      // ---- the layer input tile -> LDS (member 0 saves it)
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        const int rr = (tid + i * 256) / GL, b = r0 + rr;
        if (rr >= SSDP_R) continue;
        float2* xd = reinterpret_cast<float2*>(&Xs[rr * LDK + 4 * c4]);
        xd[0] = make_float2(xv[i].x, xv[i].y);
        xd[1] = make_float2(xv[i].z, xv[i].w);
        if (j == 0 && b < B && cv) *reinterpret_cast<float4*>(L.x + (long)t * B * H + (long)b * H + 4 * c4) = xv[i];
      }
      __syncthreads();
      if (l == 0) SSDP_STAMP(2);
      // ---- 16 x 16 gate tile over this wave's quarter of K (decode.hip's order)
      const int l16 = lane & 15, kg = lane >> 4;
      const int kq = HMAX / 4, kb = wave * kq;
      ssdp_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const float* wsl = Ws[l];
#pragma unroll 8
      for (int k = kb; k < kb + kq; k += 8) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(Xs[l16 * LDK + k + kg], wsl[l16 * LDK + k + kg], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(Xs[l16 * LDK + k + 4 + kg], wsl[l16 * LDK + k + 4 + kg], acc1, 0,
                                                    0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wave][4 * kg + i][l16] = acc0[i] + acc1[i];
      __syncthreads();
      if (tid < SSDP_R * 4) {
        const int rr = tid >> 2, uu = tid & 3, b = r0 + rr, uo = u0 + uu;
        if (b < B && uo < H) {
          float zz[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = q * 4 + uu;
            zz[q] = ((red[0][rr][c] + red[1][rr][c]) + (red[2][rr][c] + red[3][rr][c])) + bias[l][c];
          }
          const float ig = sigmoidf_(zz[0]), fg = sigmoidf_(zz[1]), gg = tanhf_(zz[2]), og = sigmoidf_(zz[3]);
          const float cc = ig * gg;
          const float hh = og * tanhf_(cc);
          put_granule(a.ring_h + (((long)l * 2 + par) * B + b) * H + uo, (unsigned)(t + 1), hh, local);
          float* gs = L.gates + (long)t * B * 4 * H + (long)b * 4 * H + uo;
          gs[0] = ig; gs[H] = fg; gs[2 * H] = gg; gs[3 * H] = og;
          L.c[(long)t * B * H + (long)b * H + uo] = cc;
          L.h[(long)t * B * H + (long)b * H + uo] = hh;
        }
      }
    }
    // ================= last LayerNorm + the FFN's first Linear and ReLU: z columns of this member
    {
      const SsdPersistLayer& P = a.L[nl - 1];
      if (!dead) {
        constexpr int NGH = SSDP_R * HMAX / 256;
        int idx[NGH];
        float gv[NGH];
        const int nvalid = min(SSDP_R, B - r0) * H;
#pragma unroll
        for (int i = 0; i < NGH; ++i) idx[i] = min(tid + i * 256, nvalid - 1);
        unsigned long long* rh = a.ring_h + (((long)(nl - 1) * 2 + par) * B + r0) * H;
        get_granules_idx<NGH>(rh, idx, (unsigned)(t + 1), gv, a.err, dead);
#pragma unroll
        for (int i = 0; i < NGH; ++i) {
          const int e = tid + i * 256;
          if (e < nvalid) Xs[(e / H) * LDK + e % H] = gv[i];
        }
      }
      SSDP_STAMP(4);
      __syncthreads();
      const float4 g = lnp[nl - 1][0][c4], bt = lnp[nl - 1][1][c4];
      float s[NX], qv[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        const int rr = (tid + i * 256) / GL;
        float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (rr < SSDP_R && cv) {
          const float2* hs = reinterpret_cast<const float2*>(&Xs[rr * LDK + 4 * c4]);
          const float2 h0 = hs[0], h1 = hs[1];
          hv = make_float4(h0.x, h0.y, h1.x, h1.y);
        }
        hv.x += xv[i].x; hv.y += xv[i].y; hv.z += xv[i].z; hv.w += xv[i].w;
        xv[i] = hv;
        s[i] = (hv.x + hv.y) + (hv.z + hv.w);
      }
#pragma unroll
      for (int o = 1; o < GL; o <<= 1)
#pragma unroll
        for (int i = 0; i < NX; ++i) s[i] += __shfl_xor(s[i], o, 64);
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        s[i] /= (float)H;
        const float d0 = xv[i].x - s[i], d1 = xv[i].y - s[i], d2 = xv[i].z - s[i], d3 = xv[i].w - s[i];
        qv[i] = cv ? (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3) : 0.0f;
      }
#pragma unroll
      for (int o = 1; o < GL; o <<= 1)
#pragma unroll
        for (int i = 0; i < NX; ++i) qv[i] += __shfl_xor(qv[i], o, 64);
      __syncthreads();   // every wave is done reading the gathered h in Xs
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        const int rr = (tid + i * 256) / GL, b = r0 + rr;
        if (rr >= SSDP_R) continue;
        const float rs = rsqrtf(qv[i] / (float)H + a.eps);
        float4 uv;
        uv.x = (xv[i].x - s[i]) * rs * g.x + bt.x; uv.y = (xv[i].y - s[i]) * rs * g.y + bt.y;
        uv.z = (xv[i].z - s[i]) * rs * g.z + bt.z; uv.w = (xv[i].w - s[i]) * rs * g.w + bt.w;
        float2* ud = reinterpret_cast<float2*>(&Xs[rr * LDK + 4 * c4]);
        ud[0] = make_float2(uv.x, uv.y);
        ud[1] = make_float2(uv.z, uv.w);
        if (j == 0 && b < B) {
          if (cv) *reinterpret_cast<float4*>(a.u + (long)t * B * H + (long)b * H + 4 * c4) = uv;
          if (c4 == 0) {
            P.mean[(long)t * B + b] = s[i];
            P.rstd[(long)t * B + b] = rs;
          }
        }
      }
      __syncthreads();
      // z[r][jj] = relu(u[r] . W1[jj] + b1[jj]): 4 lanes (k phases) per (output, row), decode.hip's order
      if (fzi < nz) {
        float acc = 0.0f;
#pragma unroll 8
        for (int k = fph; k < GL; k += 4) {
          const float2* xp = reinterpret_cast<const float2*>(&Xs[fr * LDK + 4 * k]);
          const float2 x0 = xp[0], x1 = xp[1];
          const float4 w = *reinterpret_cast<const float4*>(&w1s[fzi][4 * k]);
          acc = fmaf(x0.x, w.x, acc);
          acc = fmaf(x0.y, w.y, acc);
          acc = fmaf(x1.x, w.z, acc);
          acc = fmaf(x1.y, w.w, acc);
        }
        acc += __shfl_xor(acc, 1, 64);
        acc += __shfl_xor(acc, 2, 64);
        const int b = r0 + fr, jj = j + fzi * G;
        if (fph == 0 && b < B) {
          const float zv = fmaxf(acc + b1v, 0.0f);
          a.z[(long)t * B * HB + (long)b * HB + jj] = zv;
          put_granule(a.ring_z + ((long)par * B + b) * HB + jj, (unsigned)(t + 1), zv, local);
        }
      }
      SSDP_STAMP(5);
      __syncthreads();   // Xs is rebuilt by the next frame
    }
  }
}

}  // namespace mrg

using namespace mrg;

static unsigned long long* g_ssdp_stamps = nullptr;
// Diagnostics: block 0 of the next persistent decode forwards records per-frame phase wall clocks
// (100 MHz) into buf ([T][8]: frame start, z gathered, layer-1 input built, layer-2 h gathered, last h
// gathered, z published); null disables.  Never in timed runs.
MRG_API int mrg_ssd_persist_debug_stamps(void* buf) {
  g_ssdp_stamps = static_cast<unsigned long long*>(buf);
  return 0;
}

// Bytes of the hand-off rings (zeroed by the caller before each launch).
MRG_API long mrg_ssd_persist_ring_bytes(int B, int H, int HB, int nl) {
  return 8L * (2L * B * ((long)nl * H + HB) + (long)((B + SSDP_R - 1) / SSDP_R) * (H / 4));
}

// Whether the persistent decode forward fits this GPU resident (every member of every row tile at once).
MRG_API int mrg_ssd_persist_fits(int B, int H, int cus) {
  if (B <= 0 || H < 4 || H > 256 || H % 4) return 0;
  const long blocks = (long)((B + SSDP_R - 1) / SSDP_R) * (H / 4);
  int per = 0;
  const void* k = H <= 64 ? (const void*)ssd_fwd_persist_kernel<1, 4>
                : H <= 128 ? (const void*)ssd_fwd_persist_kernel<2, 4> : (const void*)ssd_fwd_persist_kernel<4, 2>;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 256, 0) != hipSuccess) return 0;
  const long launched = 8L * ((((B + SSDP_R - 1) / SSDP_R) + 7) / 8) * (H / 4);   // incl. the idle slots
  return (blocks <= (long)per * cus && launched <= 2L * per * cus) ? 1 : 0;
}

// The scheduled-sampling decode forward over all T frames in one launch (see the file comment).
// Layer l: w_ih[l] [4H][H], b_ih, b_hh, LayerNorm ln_w / ln_b; outputs as decode.py's per-frame path.
MRG_API int mrg_ssd_fwd_persist(int B, int H, int HB, int FO, int F, int T, int nl, float eps, const float* p,
                                const float* ms, long ms_bs, long ms_ts, const unsigned char* mask, const float* wms_t,
                                const float* w1, const float* b1, const float* w2, const float* b2,
                                const float* const* w_ih, const float* const* b_ih, const float* const* b_hh,
                                const float* const* ln_w, const float* const* ln_b, float* const* x,
                                float* const* gates, float* const* c, float* const* h, float* const* mean,
                                float* const* rstd, float* u, float* z, float* y, long y_bs, float* xf_ms,
                                void* rings, int* err, hipStream_t stream) {
  MRG_REQUIRE(H >= 4 && H <= 256 && H % 4 == 0 && HB >= 1 && HB <= 64 && FO >= 1 && FO <= 8 && T >= 1 &&
              nl >= 1 && nl <= SSDP_MAXL, "mrg_ssd_fwd_persist: H=%d HB=%d FO=%d T=%d nl=%d", H, HB, FO, T, nl);
  MRG_REQUIRE(HB <= 4 * (H / 4), "mrg_ssd_fwd_persist: HB=%d > 4 outputs per member", HB);
  MRG_REQUIRE(H <= 128 || nl <= 2, "mrg_ssd_fwd_persist: H=%d supports nl <= 2 (nl=%d)", H, nl);
  MRG_REQUIRE((((uintptr_t)p | (uintptr_t)wms_t | (uintptr_t)u) & 15) == 0, "mrg_ssd_fwd_persist: alignment");
  MRG_REQUIRE(rings && err && mask && ms, "mrg_ssd_fwd_persist: rings, err, mask, ms required");
  if (B == 0) return 0;
  SsdPersistArgs a;
  memset(&a, 0, sizeof(a));
  a.B = B; a.H = H; a.HB = HB; a.FO = FO; a.F = F; a.T = T; a.nl = nl; a.eps = eps;
  a.p = p; a.ms = ms; a.ms_bs = ms_bs; a.ms_ts = ms_ts; a.mask = mask; a.wms = wms_t;
  a.w1 = w1; a.b1 = b1; a.w2 = w2; a.b2 = b2; a.u = u; a.z = z; a.y = y; a.y_bs = y_bs; a.xf_ms = xf_ms;
  a.ring_h = static_cast<unsigned long long*>(rings);
  a.ring_z = a.ring_h + 2L * B * nl * H;
  a.xcc_slots = a.ring_z + 2L * B * HB;
  a.err = err;
  a.stamps = g_ssdp_stamps;
  for (int l = 0; l < nl; ++l) {
    MRG_REQUIRE((((uintptr_t)w_ih[l] | (uintptr_t)x[l]) & 15) == 0, "mrg_ssd_fwd_persist: layer %d alignment", l);
    a.L[l] = SsdPersistLayer{w_ih[l], b_ih[l], b_hh[l], ln_w[l], ln_b[l], x[l], gates[l], c[l], h[l], mean[l], rstd[l]};
  }
  const int NR = (B + SSDP_R - 1) / SSDP_R;
  const unsigned blocks = (unsigned)(8 * ((NR + 7) / 8) * (H / 4));
  if (H <= 64) ssd_fwd_persist_kernel<1, 4><<<blocks, 256, 0, stream>>>(a);
  else if (H <= 128) ssd_fwd_persist_kernel<2, 4><<<blocks, 256, 0, stream>>>(a);
  else if (nl <= 2) ssd_fwd_persist_kernel<4, 2><<<blocks, 256, 0, stream>>>(a);
  else ssd_fwd_persist_kernel<4, 4><<<blocks, 256, 0, stream>>>(a);
  return check_launch("ssd_fwd_persist_kernel");
}
