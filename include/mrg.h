/*
 * mrg.h — C-ABI of libmrg.so, the MI355X (gfx950) kernels of the mr_gen
 * training path.  Plain pointers, sizes and hipStream_t only; no torch types.
 *
 * The reference (TUT-SLP-lab/MultimodalReactionGeneration) has no FFI of its
 * own: its GPU work is stock PyTorch ops.  Each entry point below replaces the
 * torch op the reference calls at the cited line; the Python drop-in layer
 * (multimodalreactiongeneration_amd/functional.py) binds them with ctypes.
 *
 * Conventions
 *   - every function returns 0 on success; on failure a non-zero code and a
 *     message via mrg_last_error() (thread-local);
 *   - the caller owns every buffer, including workspaces sized by the
 *     *_bytes() helpers; nothing here allocates device memory or synchronises,
 *     so calls are legal inside hipGraph capture;
 *   - all tensors are fp32, row-major; strides are in elements;
 *   - RowMap operands (lda/lda_hi/a_rdiv): row r lives at
 *       (r / rdiv) * ld_hi + (r % rdiv) * ld   (rdiv <= 0: r * ld)
 *     which lets one call walk a [B, T, F] tensor with a time shift or a
 *     [:, lead:] slice without a copy.
 */
#ifndef MRG_H_
#define MRG_H_

#include <stddef.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* mrg_last_error(void);
int mrg_version(void);
int mrg_device_cu_count(int device, int* out);

/* ---------------------------------------------------------------- GEMM
 * C = epi(alpha * op(A) op(B) + beta * C + bias[n]); epi 0 none, 1 relu,
 * 2 multiply by (aux[m, n] > 0) (relu backward), 3 add aux[m, n] (the residual
 * branch of LN(f(x) + x): dx = g W + g without a separate add).  split-K > 1 writes fp32
 * slabs to `workspace` and reduces them in a fixed order (deterministic).
 * Replaces nn.Linear / addmm (mixer_block.py:63-74, multi_modal_metaformer.py:
 * 433-435,474,504, lstm_with_sample.py:92-130) and the x W_ih^T / weight-grad
 * GEMMs inside cuDNN's LSTM (mixer_block.py:237-252).                      */
size_t mrg_gemm_workspace_bytes(int M, int N, int splits);
/* Arithmetic of every GEMM: 1 (default) = fp32 via a three-plane bf16 split
 * (v = v0 + v1 + v2, |residual| <= 2^-24 |v|; the six products with i+j <= 2
 * accumulated in fp32 on the bf16 matrix cores, <= ~2^-22 |ab| per product);
 * 0 = exact f32 MFMA (a k-ordered fmaf chain).  Env MRG_GEMM_EXACT=1 -> 0.  */
int mrg_gemm_set_mode(int mode);
int mrg_gemm_get_mode(void);
/* Cap on resident blocks per CU of the following GEMM launches (0 = HW occupancy); returns the
 * previous cap.  Host-side state read at launch (and graph-capture) time.                       */
int mrg_gemm_set_blocks_per_cu(int n);
/* dst_i [cols_i][rows_i] = src_i [rows_i][cols_i]^T for n row-major fp32 matrices (host arrays of
 * device pointers and sizes), one launch per 32 matrices: the [in][out] weight copies that let the
 * input-gradient products dY W run k-contiguous (nn.Linear / LSTM backward, mixer_block.py:63-74).*/
int mrg_transpose_batched(int n, const float* const* src, float* const* dst, const int* rows, const int* cols,
                          hipStream_t stream);
int mrg_gemm_f32(int M, int N, int K, float alpha,
                 const float* A, int transA, long lda, long lda_hi, int a_rdiv,
                 const float* B, int transB, long ldb, long ldb_hi, int b_rdiv,
                 float beta, float* C, long ldc, const float* bias, int epilogue,
                 const float* aux, long ldaux, float* workspace, int splits,
                 hipStream_t stream);
/* As mrg_gemm_f32, plus the row sums of op(A) folded into asum_out (and
 * asum_out2, nullable): asum_out[m] = asum_beta * asum_out[m] + sum_k A(m, k).
 * With transA = 1 (A stored k-major, e.g. dY of a weight gradient dY^T X) this
 * is the bias gradient of the same Linear, computed inside the GEMM's A-tile
 * staging instead of by a separate column-sum pass; needs `workspace`
 * (mrg_gemm_workspace_bytes).
 * counters (nullable): MRG_GEMM_COUNTERS u32 tickets, zero-filled once by the caller and kept
 * across calls on one stream.  With it, a split-K GEMM with a small output lets the last K slice
 * of each tile combine the slabs in the same launch (fixed z order, like the reduce kernel) and
 * return the tickets to zero, instead of a separate reduce launch.                            */
#define MRG_GEMM_COUNTERS 4096
int mrg_gemm_f32_ex(int M, int N, int K, float alpha,
                    const float* A, int transA, long lda, long lda_hi, int a_rdiv,
                    const float* B, int transB, long ldb, long ldb_hi, int b_rdiv,
                    float beta, float* C, long ldc, const float* bias, int epilogue,
                    const float* aux, long ldaux, float* workspace, int splits,
                    float* asum_out, float* asum_out2, float asum_beta,
                    unsigned* counters, hipStream_t stream);

/* Mixed precision (bf16 configs, BASELINE configs[1]): the same GEMM with every operand rounded to
 * bf16 (RNE) as it is staged and ONE v_mfma_f32_32x32x16_bf16 per block, fp32 accumulation,
 * fp32 output and epilogue.  Arguments as mrg_gemm_f32_ex.                                  */
int mrg_gemm_bf16_ex(int M, int N, int K, float alpha,
                     const float* A, int transA, long lda, long lda_hi, int a_rdiv,
                     const float* B, int transB, long ldb, long ldb_hi, int b_rdiv,
                     float beta, float* C, long ldc, const float* bias, int epilogue,
                     const float* aux, long ldaux, float* workspace, int splits,
                     float* asum_out, float* asum_out2, float asum_beta,
                     unsigned* counters, hipStream_t stream);

/* n <= 16 same-shape k-contiguous products in ONE launch: C_p = alpha A_p B_p^T + beta C_p + bias_p
 * (+ epilogue with aux_p), A_p [M][K] rows of stride lda, B_p [N][K] rows of stride ldb (a Linear's
 * weight); bias / aux arrays nullable; bf16 = 1 for bf16 operands.  The layer-wavefront encoder
 * stack's per-diagonal chunk products (the input projection and FeedForward Linear of every
 * LSTMMixerBlock in flight, mixer_block.py:237-252,63-74, lstmformer.py:165-170).  Products the
 * LDS-DMA kernel cannot take run one by one through mrg_gemm_f32_ex.                         */
int mrg_gemm_x6g_batched(int n, int M, int N, int K, float alpha, const float* const* A, long lda,
                         const float* const* B, long ldb, float beta, float* const* C, long ldc,
                         const float* const* bias, int epilogue, const float* const* aux, long ldaux,
                         int bf16, hipStream_t stream);
/* Three bf16 planes (the x6 split: v ~ p0 + p1 + p2) of n row-major fp32 weights, once per optimizer
 * step: dst_i [3][R'][C'] with (R', C') = (rows_i, cols_i), or (cols_i, rows_i) when transpose_i.   */
int mrg_split_planes_batched(int n, const float* const* src, void* const* dst, const int* rows, const int* cols,
                             const int* transpose, hipStream_t stream);
/* C = epi(alpha A B^T + beta C + bias), B as three bf16 planes (row n of plane p at
 * Bplanes + p * bplane + n * ldb, bf16 elements), A [M][K] through the RowMap; K % 32 == 0.  The
 * forward products x W^T and the input-gradient products dY W (B = planes of W^T) of the nn.Linear /
 * LSTM / MultiheadAttention layers (mixer_block.py:63-74,237-252, for_sequential.py:42-51).      */
int mrg_gemm_x6_planes(int M, int N, int K, float alpha, const float* A, long lda, long lda_hi, int a_rdiv,
                       const void* Bplanes, long ldb, long bplane, float beta, float* C, long ldc,
                       const float* bias, int epilogue, const float* aux, long ldaux, hipStream_t stream);
/* n same-shape products on pre-split weight planes (three bf16 planes per weight, as made by
 * mrg_split_planes_batched; plane p row r at Bplanes[i] + p * bplane + r * ldb bf16): the batched
 * activation-times-weight products of the encoder stack and the fused integrators, fp32-class x6
 * arithmetic.  K % 32 == 0, 16-byte aligned rows, n <= 16.                                         */
int mrg_gemm_x6_planes_batched(int n, int M, int N, int K, float alpha, const float* const* A, long lda,
                               const void* const* Bplanes, long ldb, long bplane, float beta,
                               float* const* C, long ldc, const float* const* bias, int epilogue,
                               const float* const* aux, long ldaux, hipStream_t stream);

/* out[n] = beta*out[n] + sum_rows X(row, n); out2 (nullable) receives the same
 * sum (b_ih and b_hh share one gradient).  Bias gradients of every Linear.  */
size_t mrg_colsum_workspace_bytes(int rows, int N);
int mrg_colsum_f32(int rows, int N, const float* X, long ld, long ld_hi, int rdiv,
                   float beta, float* out, float* out2, float* workspace, hipStream_t stream);

/* ---------------------------------------------------------------- LSTM
 * Persistent recurrence of torch.nn.LSTM (gate order i, f, g, o) given the
 * input projection gx = x W_ih^T + b_ih.  Replaces the cuDNN RNN behind
 * LSTMMixer.forward (mixer_block.py:248-252), LSTMModule.forward
 * (lstm_block.py:38-46) and LSTMSampler.forward (lstm_sampler.py:26-34).
 * `nprob` (1..12) independent same-shape recurrences share one launch
 * (e.g. the audio and partner encoders of block 0).  Arrays are indexed by
 * problem.  xbuf[i] must be zeroed before every call
 * (mrg_lstm_fwd_xbuf_bytes / mrg_lstm_bwd_xbuf_bytes); *err is OR-ed with 1
 * if a hand-off spin times out; cus = CU count (<= 0: query the current device).
 * H in {16, 32, 64, 128, 256}.             */
int mrg_lstm_supported_hidden(int H);
size_t mrg_lstm_fwd_xbuf_bytes(int B, int H);
size_t mrg_lstm_bwd_xbuf_bytes(int B, int H);
int mrg_lstm_fwd(int nprob, int B, int T, int H,
                 const float* const* gx, const long* gx_bs, const long* gx_ts,
                 const float* const* w_hh, const float* const* b_hh,
                 const float* const* h0, const float* const* c0,
                 float* const* y, const long* y_bs, const long* y_ts,
                 float* const* gates, float* const* cs, float* const* hT, float* const* cT,
                 const int* reverse, void* const* xbuf, const long* lay, int* err, int cus,
                 int force_bs, hipStream_t stream);
/* Backward: dG[B, T, 4H] = d(pre-activation gates); dh0 / dc0 optional.
 * lay (nullable = dense [B, T, .] / [B, H]): 8 strides (elements) per problem, so a problem can be
 * a time chunk of a longer (e.g. time-major) sequence, its state carried through h0/c0 = the
 * previous chunk's last y / c:  fwd {gates bs, gates ts, cs bs, cs ts, h0 bs, c0 bs, -, -},
 * bwd {gates bs, gates ts, cs bs, cs ts, c0 bs, dG bs, dG ts, -}.                              */
int mrg_lstm_bwd(int nprob, int B, int T, int H,
                 const float* const* w_hh, const float* const* gates, const float* const* cs,
                 const float* const* c0, const float* const* dy, const long* dy_bs,
                 const long* dy_ts, const float* const* dhT, const float* const* dcT,
                 float* const* dG, float* const* dh0, float* const* dc0, const int* reverse,
                 void* const* xbuf, const long* lay, int* err, int cus, int force_bs,
                 hipStream_t stream);

/* MFMA form of the H = 256 recurrences (batch tiles of 16 rows, x6 bf16 split on
 * v_mfma_f32_16x16x32_bf16, fp32-class): mode 0 never, 1 (default) when the VALU form would need
 * batch tiles >= min_bs (several problems per launch), 2 whenever its grid fits; min_bs <= 0 keeps
 * the current threshold.  Returns the previous mode.  Process-wide.  */
int mrg_lstm_set_mx(int mode, int min_bs);
/* Backward recurrences pick the smallest batch tile whose grid fits n workgroups per CU (0 = HW
 * occupancy), leaving CU room for weight-gradient GEMMs issued beside them; returns the old cap. */
int mrg_lstm_set_blocks_per_cu(int n);
/* Single-step cell (T = 1), e.g. the per-frame decode of lstm_with_sampling's scheduled-sampling
 * training (lstm_with_sample.py:410-433): pre [B, 4H] = x W_ih^T + b_ih (+ h0 W_hh^T) from the
 * GEMMs; fwd adds b_hh and writes gates [B, 4H], c [B, H], h (row stride h_ld) and a dense copy
 * h2 [B, H] (nullable; the step's output and its final state); bwd takes the h gradient as
 * dh (row stride dh_ld) + dh2 (dense) and writes dG and dc0 (nullable).  c0 / dh / dh2 / dc
 * nullable (zero).                                                                            */
int mrg_lstm_cell_fwd(int B, int H, const float* pre, long pre_ld, const float* b_hh, const float* c0,
                      float* gates, float* c, float* h, long h_ld, float* h2, hipStream_t stream);
int mrg_lstm_cell_bwd(int B, int H, const float* gates, const float* c, const float* c0, const float* dh,
                      long dh_ld, const float* dh2, const float* dc, float* dG, float* dc0,
                      hipStream_t stream);

/* GRU mixer (mixer_block.py:169-208, torch.nn.GRU gate order r, z, n), one time step: the step's
 * products are GEMMs (gx = x W_ih^T + b_ih for all steps, gh = h_{t-1} W_hh^T per step), the cell
 * fuses the rest.  fwd: h = (1-z) n + z h_{t-1}, saves gates (r, z, n) and ghn = gh_n + b_hn.
 * bwd: dh = dy + dh_next; writes dgx, dgh (= dgx with the n column times r) and dhp = dh z (the
 * caller's GEMM adds dgh W_hh).  hp / dy / dh_next nullable (zero).                          */
int mrg_gru_cell_fwd(int B, int H, const float* gx, long gx_ld, const float* gh, const float* b_hh,
                     const float* hp, long hp_ld, float* h, long h_ld, float* gates, long g_ld, float* ghn,
                     long n_ld, hipStream_t stream);
int mrg_gru_cell_bwd(int B, int H, const float* gates, long g_ld, const float* ghn, long n_ld, const float* hp,
                     long hp_ld, const float* dy, long dy_ld, const float* dh_next, float* dgx, float* dgh,
                     long d_ld, float* dhp, hipStream_t stream);

/* Persistent GRU recurrence (one launch per layer direction; replaces the per-step products + cells
 * above for torch.nn.GRU at H = 256 / 128 / 64 / 32, mixer_block.py:169-208).  Same tensors as the
 * per-step path: gx [B, T, 3H] (strides bs / ts), y, gates (r, z, n), ghn; bwd writes dgx / dgh (the
 * input / weight gradient GEMMs' operands) and dh0.  xbuf: mrg_gru_xbuf_bytes(B, H) zeroed bytes per
 * launch; err: the device flag a hand-off timeout sets (as mrg_lstm_fwd's).  h0 / dy / dhT / dh0
 * nullable.  */
int mrg_gru_supported_hidden(int H);
size_t mrg_gru_xbuf_bytes(int B, int H);
int mrg_gru_fwd(int B, int T, int H, const float* gx, long gx_bs, long gx_ts, const float* w_hh,
                const float* b_hh, const float* h0, float* y, long y_bs, long y_ts, float* gates, long g_bs,
                long g_ts, float* ghn, long n_bs, long n_ts, int reverse, void* xbuf, int* err, int cus,
                hipStream_t stream);
int mrg_gru_bwd(int B, int T, int H, const float* w_hh, const float* gates, long g_bs, long g_ts,
                const float* ghn, long n_bs, long n_ts, const float* y, long y_bs, long y_ts, const float* h0,
                const float* dy, long dy_bs, long dy_ts, const float* dhT, float* dgx, float* dgh, long d_bs,
                long d_ts, float* dh0, int reverse, void* xbuf, int* err, int cus, hipStream_t stream);

/* ---------------------------------------------------------------- scheduled-sampling decode
 * The per-frame kernels of lstm_with_sampling's autoregressive training step
 * (LSTMwithSample.head_motion_generation / generate_one_step, lstm_with_sample.py:379-433), whose
 * layered LSTM restarts from zero state every frame.  Host side: decode.py.  All
 * per-frame tensors are [B, ...] row-major slabs; H <= 256 and H % 4 == 0, HB <= 64, FO <= 8.
 * mrg_ssd_gate_cell_fwd: one zero-state LSTM layer of one frame for B rows; its input X [B, H]
 *   is mode 0: xin, mode 1: LayerNorm(hp + rp) of the previous layer (gamma, beta; its mean /
 *   rstd written).  X goes to xout (unless it is xin); gates [B, 4H] (i, f, g, o), c, h [B, H].
 * mrg_ssd_feat_gate_cell_fwd: the same for layer 1 of frame t, whose input is the frame's features
 *   X = p + ms_in W_ms^T (p = P(t): the projection of the sampler / partner columns; wms_t =
 *   W_ms^T [FO, H]) with ms_in = ms[:, 0] at t = 0 and, for t > 0, ms_in = mask[t-1] ? y(t-1) :
 *   ms[:, t-1] where y(t-1) = z(t-1) W2^T + b2 is written to y[b * y_bs + o]; ms_in goes to
 *   xf_ms[b * F + o] and X to xout.
 * mrg_ssd_ffn_z_fwd: u = LayerNorm(hp + rp) of the last layer (mean / rstd written),
 *   z = relu(u W1^T + b1) [B, HB].
 * mrg_ssd_y_fwd: y = z W2^T + b2 -> y[b * y_bs + o] (the last frame's; earlier frames' come from
 *   mrg_ssd_feat_gate_cell_fwd of the next frame).
 * mrg_ssd_ffn_bwd: last layer of frame t: dy_total = dy(t) + mask[t] (dfeat_next W_ms, or dyx_next
 *   when the next frame's bottom layer formed that product already) -> dyt
 *   [B, FO]; dz [B, HB]; du = dz W1 [B, H]; LayerNorm backward g = d(h + x) (its row sums through
 *   v = [W1 gamma | W1 beta] [HB, 2]); zero-state cell backward -> dG [B, 4H].
 * mrg_ssd_ln_cell_bwd: a lower layer: LayerNorm backward of upstream du, then the cell -> g, dG;
 *   with dyx (the bottom layer): dyx [B, FM] = (dG W_ih + g) W_ms as dG vt^T + g wms_t^T
 *   (vt = W_ms^T W_ih [FM, 4H]), the prediction gradient the select passes to frame t - 1.
 * mrg_ssd_dx: dx [B, H] = dG [B, 4H] W_ih + g, with W_ih given transposed (w_t [H, 4H]).       */
int mrg_ssd_gate_cell_fwd(int B, int H, int mode, const float* xin, const float* hp, const float* rp,
                          const float* gamma, const float* beta, float eps, float* xout, float* mean,
                          float* rstd, const float* w_ih, const float* b_ih, const float* b_hh, float* gates,
                          float* c, float* h, hipStream_t stream);
int mrg_ssd_feat_gate_cell_fwd(int B, int H, int HB, int FO, int F, int t, const float* p, const float* z,
                               const float* w2, const float* b2, const unsigned char* mask, const float* ms,
                               long ms_bs, long ms_ts, const float* wms_t, float* y, long y_bs, float* xf_ms,
                               float* xout, const float* w_ih, const float* b_ih, const float* b_hh,
                               float* gates, float* c, float* h, hipStream_t stream);
int mrg_ssd_ffn_z_fwd(int B, int H, int HB, const float* hp, const float* rp, const float* gamma,
                      const float* beta, float eps, float* u, float* mean, float* rstd, const float* w1,
                      const float* b1, float* z, hipStream_t stream);
int mrg_ssd_y_fwd(int B, int HB, int FO, const float* z, const float* w2, const float* b2, float* y, long y_bs,
                  hipStream_t stream);
/* The forward frame loop above (every frame's gate / cell / FFN kernels) in ONE persistent launch
 * (ssd_loop.hip ssd_loop_kernel; decode.py uses it when H = 256, HB = 64, FO <= 16, nl <= 4 and the
 * grid fits): groups of 8 batch rows x 16 workgroups, each layer's h handed to the group's members
 * as {tag, value} granules.  lptrs: 9 device pointers per layer (w_ih, b_ih, b_hh, the LayerNorm
 * after the layer gamma / beta, then the saved X [T][B][H] (layer 0's; null for the others), gates
 * [T][B][4H], c and h [T][B][H]); P [T][B][H] = the sampler / partner projection + b_f; wms_t;
 * w1 / b1 / w2 / b2; ms, mask as above.  The LayerNorm outputs / statistics, z, y and the sampled
 * self-motion inputs are not written (they follow from h, X_0 and ms: decode.py forms them after the
 * launch).  ring: mrg_ssd_loop_ring_bytes(B, nl) of zeroed device memory per launch; err: set when a
 * hand-off poll times out.  Replaces the per-frame launches of lstm_with_sample.py:379-433's loop.   */
long mrg_ssd_loop_ring_bytes(int B, int nl);
int mrg_ssd_loop_fits(int B, int cus);
int mrg_ssd_loop_fwd(int B, int T, int H, int HB, int FO, int nl, float eps, const void* const* lptrs,
                     int nptrs, const float* P, const float* wms_t, const float* w1, const float* b1,
                     const float* w2, const float* b2, const float* ms, long ms_bs, long ms_ts,
                     const unsigned char* mask, void* ring, int* err, hipStream_t stream);
/* The backward frame loop (mrg_ssd_ffn_bwd / mrg_ssd_dx / mrg_ssd_ln_cell_bwd of every frame, nl >= 2)
 * in ONE persistent launch (ssd_loop.hip ssd_loop_bwd_kernel; decode.py uses it under the same
 * conditions as the forward loop): per frame the last layer's FFN / LayerNorm / cell backward needs no
 * exchange (the row sums through v), then per lower layer one hand-off of dG rows (dX = dG W_ih + g
 * on MFMA) and one of partial LayerNorm row sums, and the bottom layer's partial dyx feeds the
 * previous frame.  lptrs: 12 per layer (W_ih [4H][H] or null for layer 0, the LayerNorm gamma and
 * beta, the forward's X, gates, c, h, mean, rstd, then g, dG and dX (null for layer 0)); dy [B][T][FO]; v =
 * [W1 gamma | W1 beta] [HB][2]; z [T][B][HB]; vt = W_ms^T W_ih0 [FO][4H]; output du [T][B][H] (dy_total
 * and dz follow from dy, dX_0 and z after the launch); ring: mrg_ssd_loop_bwd_ring_bytes(B) of zeroed
 * memory per launch.                                                                                  */
long mrg_ssd_loop_bwd_ring_bytes(int B);
int mrg_ssd_loop_bwd_fits(int B, int cus);
int mrg_ssd_loop_bwd(int B, int T, int H, int HB, int FO, int nl, const void* const* lptrs, int nptrs,
                     const float* dy, const unsigned char* mask, const float* w1, const float* w2, const float* b1,
                     const float* v, const float* z, const float* vt, const float* wms_t, float* du, void* ring,
                     int* err, hipStream_t stream);
int mrg_ssd_ffn_bwd(int B, int H, int HB, int FO, int t, const float* dy, long dy_bs, const float* dfeat_next,
                    const float* dyx_next, const float* wms_t, const unsigned char* mask, const float* w1,
                    const float* w2,
                    const float* b1, const float* v, const float* z, float* dyt, float* dz, float* du,
                    const float* h, const float* x, const float* gamma, const float* mean, const float* rstd,
                    float* g, const float* gates, const float* c, float* dG, hipStream_t stream);
int mrg_ssd_ln_cell_bwd(int B, int H, const float* du, const float* h, const float* x, const float* gamma,
                        const float* mean, const float* rstd, float* g, const float* gates, const float* c,
                        float* dG, int FM, const float* vt, const float* wms_t, float* dyx, hipStream_t stream);
int mrg_ssd_dx(int B, int H, const float* dG, const float* w_t, const float* g, float* dx, hipStream_t stream);
/* One step (T = 1) of an LSTM direction with a carried state (the generation loops' mixers,
 * lstmformer.py:466-521): gates = [x | h0] [W_ih | W_hh]^T + b_ih + b_hh (i, f, g, o) -> gates
 * [B, 4H], c = f c0 + i g [B, H], h -> y[b * ldy + u] and hT [B, H] (nullable); h0 / c0 nullable
 * (zero state).  In, H multiples of 4, In + H <= 512.  Replaces two GEMMs + mrg_lstm_cell_fwd. */
int mrg_lstm_step_fwd(int B, int H, int In, const float* x, const float* h0, const float* c0,
                      const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh,
                      float* gates, float* c, float* y, long ldy, float* hT, hipStream_t stream);

/* Per-frame main chain of lstmformer generation (gen.hip; Metaformer.prediction, lstmformer.py:466-521,
 * every frame a T = 1 forward with zero state): E = 256, FeedForward bottleneck 64, 16 batch rows x
 * 16 output columns per workgroup, the LayerNorms a stage consumes recomputed in its prologue.
 * mrg_gen_lstm: X = ms W_fe^T + b_fe (ms [B][fm], fm <= 16; feature_embedding.0) or X = LN(a + r)
 *   (the previous block's FeedForward residual LayerNorm), written to xw [B][256]; gates =
 *   X W_ih^T + b_ih + b_hh, zero-state cell (LSTMMixer, mixer_block.py:237-252) -> h [B][256].
 * mrg_gen_linear mode 0: out = LN(a + r) W^T + b, LN rows to xw (LSTMMixerBlock, mixer_block.py:479-507);
 *   mode 1: M = LN(a + r), Y_i = LN(a2[i] + M) to xw[:, 256 i:], out[:, 256 i:] = Y_i W_i^T + b_i
 *   (both integrators' MHAMixerBlocks, mixer_block.py:567-603, with their attention output a2[i]);
 *   mode 2: out = [LN(a[0] + r[0]) | LN(a[1] + r[1])] W^T + b (cat_linear over the integrators'
 *   FeedForward LayerNorms, multi_modal_metaformer.py:128-217).  Host arrays of device pointers.
 * mrg_gen_ffn: Linear(256 -> 64) -> ReLU -> Linear(64 -> N) of X = a or LN(a + r): out [B][256]; or,
 *   with pred (the output FeedForward, N <= 16), y into pred[b * pred_bs + t * N + n] and the next
 *   frame's self motion ms_next = mask[t] ? y : ms_src (lstmformer.py:487-492).                      */
int mrg_gen_lstm(int B, int fm, const float* ms, const float* fe_w, const float* fe_b, const float* a,
                 const float* r, const float* ga, const float* be, float eps, float* xw, const float* w_ih,
                 const float* b_ih, const float* b_hh, float* h, hipStream_t stream);
int mrg_gen_linear(int mode, int B, const float* const* a, const float* const* r, const float* const* ga,
                   const float* const* be, long lda, const float* const* a2, const float* const* ga2,
                   const float* const* be2, float eps, float* xw, long ldxw, const float* const* w,
                   const float* const* bias, float* out, long ldo, hipStream_t stream);
int mrg_gen_ffn(int B, int N, const float* a, const float* r, const float* ga, const float* be, float eps,
                const float* w1, const float* b1, const float* w2, const float* b2, float* out, float* pred,
                long pred_bs, float* ms_next, const float* ms_src, const unsigned char* mask, int t,
                hipStream_t stream);
/* The whole frame loop in ONE persistent launch (gen.hip gen_loop_kernel): groups of 8 batch rows,
 * 16 workgroups per group exchanging each stage's outputs as {tag, value} granules; the same stages
 * as the three entries above.  ptrs: host array of 31 nb + 6 device pointers -- per block w_ih,
 * b_ih, b_hh, mixer LayerNorm g / b, mixer Linear w / b, mixer FeedForward LayerNorm g / b, per
 * integrator i = 0, 1 (attention residual LayerNorm g / b, FeedForward w / b, its LayerNorm g / b),
 * cat_linear w / b, block FeedForward w1 / b1 / w2 / b2, its LayerNorm g / b, the integrators'
 * attention outputs a_0 / a_1 [T][B][256]; then feature_embedding.0 w / b and the output FeedForward
 * w1 / b1 / w2 / b2.  ms [T][B][fm], mask [T] bytes, pred [B][T][fm]; ring: mrg_gen_loop_ring_bytes
 * of zeroed device memory per launch; err: set when a hand-off poll times out.  mrg_gen_loop_fits:
 * 1 when the grid (16 ceil(B / 8) workgroups) can be resident on `cus` CUs (0: the device's).   */
long mrg_gen_loop_ring_bytes(int B);
int mrg_gen_loop_fits(int B, int cus);
int mrg_gen_loop(int B, int T, int fm, int nb, float eps, const void* const* ptrs, int nptrs, const float* ms,
                 const unsigned char* mask, float* pred, void* ring, int* err, hipStream_t stream);

/* ---------------------------------------------------------------- attention
 * Scaled-dot-product core of nn.MultiheadAttention as the reference calls it
 * (MHAforSequentail.forward, for_sequential.py:42-51;
 * MultiModalAttentionBlockSequential.forward, multi_modal_att.py:22-31) with
 * the gen_attention_mask rules (multi_modal_metaformer.py:32-79) evaluated
 * from indices: causal != 0 selects the block-causal rectangular mask;
 * qpad/kpad (uint8 [B,Tq]/[B,Tk], nullable) give the padding AND rule.
 * Element (b, t, head, d) lives at base + b*bs + t*ts + head*D + d.
 * lse: [B, heads, Tq] log-sum-exp saved for the backward.  D in {8,16,32,64}.
 * Backward: deterministic (no atomics).  D = 64 with Tq <= 320 and 16-B rows everywhere runs a single
 * pass (one workgroup per (sample, head); the workspace is then unused); other shapes run a dQ pass
 * (delta = rowsum(dO * O) into the workspace) and a dK / dV pass. */
int mrg_attention_fwd(int B, int heads, int Tq, int Tk, int D,
                      const float* q, long q_bs, long q_ts, const float* k, long k_bs, long k_ts,
                      const float* v, long v_bs, long v_ts, float* o, long o_bs, long o_ts,
                      float* lse, const unsigned char* qpad, const unsigned char* kpad,
                      int causal, float scale, hipStream_t stream);
size_t mrg_attention_bwd_workspace_bytes(int B, int heads, int Tq);
int mrg_attention_bwd(int B, int heads, int Tq, int Tk, int D,
                      const float* q, long q_bs, long q_ts, const float* k, long k_bs, long k_ts,
                      const float* v, long v_bs, long v_ts, const float* o, long o_bs, long o_ts,
                      const float* lse, const unsigned char* qpad, const unsigned char* kpad,
                      int causal, float scale, const float* dout, long do_bs, long do_ts,
                      float* dq, long dq_bs, long dq_ts, float* dk, long dk_bs, long dk_ts,
                      float* dv, long dv_bs, long dv_ts, float* workspace, hipStream_t stream);

/* Query-chunk forms (the metaformer blocks' (block, time-chunk) wavefront): q / o / dout / dq point at
 * the chunk's first query row; the Tq queries are rows [q_off, q_off + Tq) of a Tq_full-query
 * sequence (the mask rule uses global indices and Tk / Tq_full); lse, the workspace and qpad are the
 * whole sequence's [B, heads, Tq_full] / [B, Tq_full] arrays.  bwd passes: 1 = dQ (and the chunk's
 * delta into the workspace), 2 = dK / dV from the lse / delta already there, 3 = both; a pass-2 call
 * over q_off = 0, Tq = Tq_full after every chunk's pass-1 call gives the whole sequence's dK / dV.
 * kv_accumulate = 1 adds a chunk's dK / dV share into dk / dv (key blocks no query of the chunk sees
 * are not touched).  */
int mrg_attention_fwd_chunk(int B, int heads, int Tq, int Tk, int D, int q_off, int Tq_full,
                            const float* q, long q_bs, long q_ts, const float* k, long k_bs, long k_ts,
                            const float* v, long v_bs, long v_ts, float* o, long o_bs, long o_ts,
                            float* lse, const unsigned char* qpad, const unsigned char* kpad,
                            int causal, float scale, hipStream_t stream);
int mrg_attention_bwd_chunk(int B, int heads, int Tq, int Tk, int D, int q_off, int Tq_full,
                            const float* q, long q_bs, long q_ts, const float* k, long k_bs, long k_ts,
                            const float* v, long v_bs, long v_ts, const float* o, long o_bs, long o_ts,
                            const float* lse, const unsigned char* qpad, const unsigned char* kpad,
                            int causal, float scale, const float* dout, long do_bs, long do_ts,
                            float* dq, long dq_bs, long dq_ts, float* dk, long dk_bs, long dk_ts,
                            float* dv, long dv_bs, long dv_ts, int passes, int kv_accumulate,
                            float* workspace, hipStream_t stream);

/* ---------------------------------------------------------------- LayerNorm
 * y = LayerNorm(a + b) (ResidualConnection.forward, residual_connection.py:
 * 20-37), rows x E, 1 <= E <= 1024; mean/rstd saved per row.     */
int mrg_residual_layernorm_fwd(int rows, int E, const float* a, const float* b,
                               const float* gamma, const float* beta, float eps, float* y,
                               float* mean, float* rstd, hipStream_t stream);
size_t mrg_residual_layernorm_bwd_workspace_bytes(int rows, int E);
int mrg_residual_layernorm_bwd(int rows, int E, const float* dy, const float* a, const float* b,
                               const float* gamma, const float* mean, const float* rstd,
                               float* dx, float* dgamma, float* dbeta, int accumulate,
                               float* workspace, hipStream_t stream);
/* dgamma = dbeta = NULL in mrg_residual_layernorm_bwd leaves the per-block partials in the
 * workspace; this reduces them (dgamma/dbeta += or = their sums) — e.g. on another stream, since
 * only the optimizer reads parameter gradients.  The reduce CONSUMES the workspace: each row
 * group's sum overwrites that group's first partial row, so a second reduce of the same partials
 * gives wrong sums (re-run the backward first).  Any number of streams may reduce concurrently
 * (each (device, stream) has its own completion tickets, up to 64 pairs per process).          */
int mrg_residual_layernorm_param_reduce(int rows, int E, float* workspace, float* dgamma,
                                        float* dbeta, int accumulate, hipStream_t stream);
/* Row-mapped forms (E % 4 == 0, 16-byte aligned rows) for the time-major encoder stack
 * (mixer_block.py:479-507 per layer, run as time chunks): the forward's output rows y and the
 * backward's incoming gradient rows dy sit at (r / div) * hi + (r % div) * lo (div = 0: r * lo), so
 * time-major rows [T, B, E] write / read a batch-major [B, T, E] tensor in place.  The backward
 * leaves dgamma / dbeta partials in workspace (one 32-row block each; a chunk passes its offset). */
int mrg_residual_layernorm_fwd_map(int rows, int E, const float* a, const float* b, const float* gamma,
                                   const float* beta, float eps, float* y, long y_lo, long y_hi, int y_div,
                                   float* mean, float* rstd, hipStream_t stream);
int mrg_residual_layernorm_bwd_map(int rows, int E, const float* dy, long dy_lo, long dy_hi, int dy_div,
                                   const float* a, const float* b, const float* gamma, const float* mean,
                                   const float* rstd, float* dx, float* workspace, hipStream_t stream);
/* n <= 16 same-shape row-mapped residual LayerNorms (ResidualConnection, residual_connection.py:20-37)
 * in one launch, each with its own tensors, parameters and map: the encoder stack's per-diagonal
 * chunks.  Backward partials go to ws[p] (reduce with mrg_residual_layernorm_param_reduce).      */
int mrg_residual_layernorm_fwd_batched(int n, int rows, int E, const float* const* a, const float* const* b,
                                       const float* const* gamma, const float* const* beta, float eps,
                                       float* const* y, const long* y_lo, const long* y_hi, const int* y_div,
                                       float* const* mean, float* const* rstd, hipStream_t stream);
int mrg_residual_layernorm_bwd_batched(int n, int rows, int E, const float* const* dy, const long* dy_lo,
                                       const long* dy_hi, const int* dy_div, const float* const* a,
                                       const float* const* b, const float* const* gamma,
                                       const float* const* mean, const float* const* rstd, float* const* dx,
                                       float* const* ws, hipStream_t stream);

/* Padding helpers: flags[b][t] = (x[b][t][0] == value) as uint8 (gen_attention_mask's padding test,
 * multi_modal_metaformer.py:67-73; x rows at b * bs + t * ts); y = x * (x != value) (training_step's
 * zeroing of padded motion_self frames, lstmformer.py:365-366). */
int mrg_padding_flags(int B, int T, const float* x, long bs, long ts, float value, unsigned char* out,
                      hipStream_t stream);
int mrg_zero_padding(long n, const float* x, float value, float* y, hipStream_t stream);
/* bytes of zeros at p (any alignment): the training step's buffer clears (gradient buffer, hand-off
 * rings, loss-gradient lead frames) without a torch fill kernel.  Replaces the `zero_grad` /
 * `torch.zeros` of the reference's step (lstmformer.py:313-322 loss, Lightning's optimizer zero_grad). */
int mrg_fill_zero(void* p, long bytes, hipStream_t stream);
/* dst [n1][n0][E] = src [n0][n1][E] (beta = 1: dst +=): the batch-major [B, T, E] <-> time-major
 * [T, B, E] activations and gradients at the metaformer blocks' wavefront boundaries
 * (multi_modal_metaformer.py:501-502 feeds block outputs forward batch-major).  E % 4 == 0.     */
int mrg_swap01(int n0, int n1, int E, const float* src, float* dst, float beta, hipStream_t stream);

/* ---------------------------------------------------------------- loss
 * Masked regression loss of training_step (lstmformer.py:372-380,
 * lossfun :313-325): mask = target != -100, feature scaler from
 * delta_start; type 0 huber, 1 mse, 2 l1, 3 smoothl1; mean reduction.
 * y is viewed [B, T, F] with batch stride y_bstride (y[:, lead:] slices). */
size_t mrg_loss_workspace_bytes(int B, int T, int F);
int mrg_masked_loss_fwd(int B, int T, int F, const float* y, long y_bstride, const float* target,
                        int type, float delta, float beta, int mask_padding, int delta_start,
                        float dscale, float* loss_out, float* workspace, hipStream_t stream);
int mrg_masked_loss_bwd(int B, int T, int F, const float* y, long y_bstride, const float* target,
                        int type, float delta, float beta, int mask_padding, int delta_start,
                        float dscale, const float* grad_out, float* dy, hipStream_t stream);

/* Broadcast-target loss of the lstmformer AR path: Metaformer.prediction returns
 * target [B,T,F] * motion_s_mask [Tm,B,1,F] -> [Tm,B,T,F] (lstmformer.py:434-435, mask from
 * :540-547), and generation_step (:410-424) / the scheduled-sampling training_step (:357-385)
 * take the padding-masked mean loss over that broadcast tensor, the training scaler
 * sqrt(delta_loss_scale) applying to time indices t >= t_start (its [:, :, start:] slice lands on
 * the T axis; pass t_start > T for none).  Computed analytically from per-(b, f) counts of
 * non-padded motion_s frames: ms is the raw self motion [B, Tm, F] (batch / time strides), y the
 * prediction [B, T, F] (batch stride y_bstride), target contiguous.  workspace:
 * mrg_broadcast_loss_workspace_bytes.  Mean over Tm*B*T*F elements.                        */
size_t mrg_broadcast_loss_workspace_bytes(int B, int T, int F);
int mrg_broadcast_loss_fwd(int B, int T, int F, const float* y, long y_bstride, const float* target,
                           const float* ms, long ms_bs, long ms_ts, int Tm, int type, float delta,
                           float beta, int t_start, float dscale, float* loss_out, float* workspace,
                           hipStream_t stream);
int mrg_broadcast_loss_bwd(int B, int T, int F, const float* y, long y_bstride, const float* target,
                           const float* ms, long ms_bs, long ms_ts, int Tm, int type, float delta,
                           float beta, int t_start, float dscale, const float* grad_out, float* dy,
                           float* workspace, hipStream_t stream);

/* ---------------------------------------------------------------- AdamW
 * torch.optim.AdamW step over flat buffers (configure_optimizers,
 * lstmformer.py:327-333).  step_lr = device float[2] {steps done, lr}.
 * err (nullable): the device error flag the persistent LSTM kernels OR into on a hand-off
 * timeout; when it is set the update and the step count are skipped (garbage gradients never
 * reach the weights, even inside a replayed graph).                                       */
int mrg_adamw_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, long n,
                   float* step_lr, float weight_decay, float beta1, float beta2, float eps,
                   const int* err, hipStream_t stream);

/* ---------------------------------------------------------------- features (data loader)
 * AudioPreprocessor (mr_gen/utils/preprocess/audio.py:6-67).  The power spectrum comes from one
 * GEMM of the frames (read in place from the waveform, row stride `hop`) with the windowed DFT
 * basis [2*NF, nfft] (cos rows then sin rows); mrg_fbank_finish turns spec [F][spec_ld] into
 * out[f] = [log(max(mel_j, 1e-6)) for j < NM, log(max(sum_n frame_f[n]^2, 1e-10))]
 * (MelSpectrogram + log, audio.py:33-35; compute_log_power, :43-56), melfb [NF][NM], where
 * frame f starts at wave + (f / frames_per_clip) * clip_len + (f % frames_per_clip) * hop
 * (equal-length clips stacked: one launch for a batch; one clip: frames_per_clip = F).
 * mrg_feature_delta stacks [x[d:], delta1[d-1:], delta2] (compute_delta, audio.py:58-67,
 * motion_nx.py:49-58) for order d in 0..2 over nclip sequences x [nclip][T][C] (row stride
 * ldx): out [nclip][T-d][C*(d+1)].                                                           */
int mrg_fbank_finish(int F, int NF, int NM, const float* spec, long spec_ld, const float* melfb,
                     const float* wave, long hop, int nfft, int frames_per_clip, long clip_len,
                     float* out, long out_ld, hipStream_t stream);
int mrg_feature_delta(int nclip, int T, int C, const float* x, long ldx, int order, float* out,
                      hipStream_t stream);
/* collate_fn (lstmformer/dataloader.py:114-121): pack_sequence + pad_packed_sequence with
 * padding_value -100.  seqs: device table of B pointers to contiguous [lens[b], F] rows; lens:
 * device int[B]; out [B, Tmax, F].                                                            */
int mrg_pad_sequences(int B, int Tmax, int F, const float* const* seqs, const int* lens, float pad,
                      float* out, hipStream_t stream);

/* ---------------------------------------------------------------- RCCL gradient exchange
 * The data-parallel step's one exchange: Lightning `strategy: ddp`
 * (mr_gen/model/lstmformer/config.yaml:127) averages the gradients across ranks after backward;
 * here an in-place fp32 all-reduce of spans of the flat gradient buffer over RCCL (xGMI).
 * librccl.so.1 is resolved at run time (the copy torch already mapped); mrg_comm_available()
 * says whether one was found.  Rank 0 calls mrg_comm_unique_id, the host moves the
 * mrg_comm_id_bytes() bytes to every rank, each rank (its GPU already selected) calls
 * mrg_comm_init.  mrg_comm_allreduce_f32 issues the spans [offsets[i], offsets[i] + counts[i])
 * of buf as one RCCL group on `stream`; op 0 = sum, 1 = mean.                               */
int mrg_comm_available(void);
size_t mrg_comm_id_bytes(void);
int mrg_comm_unique_id(void* id_out);
int mrg_comm_init(void** comm_out, int nranks, const void* id, int rank);
int mrg_comm_allreduce_f32(void* comm, float* buf, const long* offsets, const long* counts, int nbuckets,
                           int op, hipStream_t stream);
int mrg_comm_destroy(void* comm);

#ifdef __cplusplus
}
#endif
#endif /* MRG_H_ */
