// GRU mixer (mixer_block.py:169-208 GRUMixer = torch.nn.GRU, gate order r, z, n):
// the element-wise step of the recurrence.  The step's products run as GEMMs (functional.py):
//   gx = X W_ih^T + b_ih for all B*T rows once; per step gh = h_{t-1} W_hh^T (few-row GEMM kernel),
//   then THIS cell:  r = s(gx_r + gh_r + b_hr), z = s(gx_z + gh_z + b_hz),
//                    ghn = gh_n + b_hn, n = tanh(gx_n + r * ghn), h = (1 - z) n + z h_{t-1}.
// Backward per step: this cell's derivative, then dh_{t-1} = dh z + dGH W_hh (few-row GEMM, beta 1);
// dW_ih / dW_hh / biases / dX are GEMMs over all steps afterwards.
#include "mrg_common.h"

namespace mrg {

// gx rows of stride gx_ld ([B, 3H] slice of step t), gh [B, 3H] dense, hp rows of stride hp_ld
// (nullable: zero state); writes h (stride h_ld), gates [B, 3H] (r, z, n) and ghn [B, H] (stride sv_ld
// rows for both, i.e. the step-t slices of [B, T, .] buffers)
__global__ __launch_bounds__(256) void gru_cell_fwd_kernel(int B, int H, const float* __restrict__ gx, long gx_ld,
                                                           const float* __restrict__ gh, const float* __restrict__ b_hh,
                                                           const float* __restrict__ hp, long hp_ld,
                                                           float* __restrict__ h, long h_ld,
                                                           float* __restrict__ gates, long g_ld,
                                                           float* __restrict__ ghn, long n_ld) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * H) return;
  const int b = i / H, u = i % H;
  const float* x = gx + (long)b * gx_ld;
  const float* g = gh + (long)b * 3 * H;
  const float r = sigmoidf_(x[u] + g[u] + b_hh[u]);
  const float z = sigmoidf_(x[H + u] + g[H + u] + b_hh[H + u]);
  const float hn = g[2 * H + u] + b_hh[2 * H + u];
  const float n = tanhf_(x[2 * H + u] + r * hn);
  const float hprev = hp ? hp[(long)b * hp_ld + u] : 0.0f;
  h[(long)b * h_ld + u] = (1.0f - z) * n + z * hprev;
  float* gs = gates + (long)b * g_ld + u;
  gs[0] = r; gs[H] = z; gs[2 * H] = n;
  ghn[(long)b * n_ld + u] = hn;
}

// dh = dy (rows of stride dy_ld, nullable) + dhn (dense [B, H], nullable); writes dgx / dgh rows
// (stride d_ld: step-t slices of [B, T, 3H]) and dhp = dh * z (dense [B, H], the direct part of
// dh_{t-1}; the GEMM adds dgh W_hh)
__global__ __launch_bounds__(256) void gru_cell_bwd_kernel(int B, int H, const float* __restrict__ gates, long g_ld,
                                                           const float* __restrict__ ghn, long n_ld,
                                                           const float* __restrict__ hp, long hp_ld,
                                                           const float* __restrict__ dy, long dy_ld,
                                                           const float* __restrict__ dhn,
                                                           float* __restrict__ dgx, float* __restrict__ dgh,
                                                           long d_ld, float* __restrict__ dhp) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * H) return;
  const int b = i / H, u = i % H;
  const float* gs = gates + (long)b * g_ld + u;
  const float r = gs[0], z = gs[H], n = gs[2 * H];
  const float hn = ghn[(long)b * n_ld + u];
  const float hprev = hp ? hp[(long)b * hp_ld + u] : 0.0f;
  const float dh = (dy ? dy[(long)b * dy_ld + u] : 0.0f) + (dhn ? dhn[i] : 0.0f);
  const float dn = dh * (1.0f - z);
  const float dz = dh * (hprev - n);
  const float dpn = dn * (1.0f - n * n);
  const float dr = dpn * hn;
  const float dpr = dr * r * (1.0f - r);
  const float dpz = dz * z * (1.0f - z);
  float* ox = dgx + (long)b * d_ld + u;
  float* oh = dgh + (long)b * d_ld + u;
  ox[0] = dpr; ox[H] = dpz; ox[2 * H] = dpn;
  oh[0] = dpr; oh[H] = dpz; oh[2 * H] = dpn * r;
  dhp[i] = dh * z;
}

}  // namespace mrg

using namespace mrg;

MRG_API int mrg_gru_cell_fwd(int B, int H, const float* gx, long gx_ld, const float* gh, const float* b_hh,
                             const float* hp, long hp_ld, float* h, long h_ld, float* gates, long g_ld, float* ghn,
                             long n_ld, hipStream_t stream) {
  MRG_REQUIRE(B >= 0 && H > 0, "mrg_gru_cell_fwd: bad sizes");
  if (B == 0) return 0;
  const long n = (long)B * H;
  gru_cell_fwd_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(B, H, gx, gx_ld, gh, b_hh, hp, hp_ld, h, h_ld,
                                                                       gates, g_ld, ghn, n_ld);
  return check_launch("gru_cell_fwd_kernel");
}

MRG_API int mrg_gru_cell_bwd(int B, int H, const float* gates, long g_ld, const float* ghn, long n_ld, const float* hp,
                             long hp_ld, const float* dy, long dy_ld, const float* dhn, float* dgx, float* dgh,
                             long d_ld, float* dhp, hipStream_t stream) {
  MRG_REQUIRE(B >= 0 && H > 0, "mrg_gru_cell_bwd: bad sizes");
  if (B == 0) return 0;
  const long n = (long)B * H;
  gru_cell_bwd_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(B, H, gates, g_ld, ghn, n_ld, hp, hp_ld, dy,
                                                                       dy_ld, dhn, dgx, dgh, d_ld, dhp);
  return check_launch("gru_cell_bwd_kernel");
}
