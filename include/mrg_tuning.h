/*
 * mrg_tuning.h — tuning, measurement and test hooks of libmrg.so (not part of the drop-in
 * boundary in mrg.h): knobs the measured A/Bs in DESIGN.md used, the kernel-bound probes
 * bench.py times the families with, fault injection / CU-occupying stand-ins for the tests, and
 * the structural-variant GEMM entry points.
 * Same conventions as mrg.h (0 = success, mrg_last_error()).
 */
#ifndef MRG_TUNING_H_
#define MRG_TUNING_H_

#include "mrg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* LDS-DMA pipelined x6 kernel for k-contiguous products (transA 0, transB 1, K % 32 == 0, unsplit,
 * >= 2048 rows, >= 256 columns): ring depth 2..4 (0 = off; default 2, MRG_GEMM_GLDS) and column
 * tile (64 forces 64-wide tiles, 128 = by shape).                                               */
int mrg_gemm_set_glds(int depth, int bn);
/* Weight-gradient products (transA 1, transB 0) on the LDS-DMA kernel (1, default) or the
 * register-staged one (0); returns the previous setting.                                        */
int mrg_gemm_set_glds_wg(int on);
/* Kernel of mrg_gemm_x6_planes: 0 = gemm_x6g_kernel (pre-split B, 32 x 32 blocks), 12 / 22 =
 * gemm_x6w_kernel (gemm_wide.hip: row-owning waves, 64 / 128 columns per tile, ring depth 2); env
 * MRG_GEMM_WIDE; other values are ignored; returns the previous setting.                            */
int mrg_gemm_set_wide(int cfg);
/* Attention backward form: 1 (default, MRG_ATTN_FUSED) = the single-pass kernel (one workgroup per
 * (sample, head); D = 64, Tq <= 320, 16-B rows) where it applies, 0 = always the two-pass dQ, dK / dV
 * kernels; returns the previous setting.                                                           */
int mrg_attention_set_fused(int on);
/* Tuning only: force the tile shape (0: 128x128, 1: 128x64, 2: 64x64), -1 = heuristic. */
int mrg_gemm_force_tile(int tile);
/* Tuning only: structural variants of the x6 kernel (0 product, 1 split + one MFMA, 2 plane-0 +
 * six MFMAs, 3 plane-0 + one MFMA) on C = A B^T, A [M][K], B [N][K]; var != 0 gives no valid C. */
int mrg_gemm_x6_variant(int var, int M, int N, int K, const float* A, const float* B, float* C,
                        hipStream_t stream);
/* Fault injection (tests only): mode 1 makes the NEXT mrg_lstm_fwd launch (mode 2: the next
 * mrg_lstm_bwd launch) drop member 0's first hand-off, VALU or MFMA form, so the recurrence times
 * out and reports through *err; 0 disarms.  Process-wide.  */
int mrg_lstm_debug_inject(int mode);
/* Tests only: keep `blocks` workgroups of `threads` lanes and `lds` bytes of LDS resident for `usec`
 * microseconds on `stream` (a stand-in for a CU-occupying kernel, e.g. an RCCL collective, beside a
 * persistent recurrence, which must then wait for CUs without timing out its hand-offs).        */
int mrg_debug_busy(int blocks, int threads, int lds, double usec, hipStream_t stream);
/* Diagnostics: a 1-thread kernel writing the 100 MHz wall clock into ((uint64*)buf)[slot] in `stream`'s
 * order (tools/side_timing.py: when a replayed graph reaches a point). */
int mrg_debug_stamp(void* buf, int slot, hipStream_t stream);
/* Diagnostics: per-stage 100 MHz real-time stamps of row group 0's 16 members in later mrg_gen_loop
 * launches ([T][16 members][32] u64; slot 31 of frame 0: the local hand-off flag); null turns them off
 * (tools/gen_stamps.py). */
int mrg_gen_loop_debug_stamps(void* buf);
/* Diagnostics: per-stage 100 MHz real-time stamps (s_memrealtime, one clock for all CUs) of the 16
 * members of row group 0 in later mrg_ssd_loop_fwd launches ([T][16 members][16] u64: frame start, then
 * per layer after its input / after its publish, then the FFN stage; frame 0: slot 15 the local
 * hand-off flag, slot 14 the HW_ID register) (tools/ssd_stamps.py). */
int mrg_ssd_loop_debug_stamps(void* buf);
/* Diagnostics: the same for mrg_ssd_loop_bwd (by backward iteration). */
int mrg_ssd_loop_bwd_debug_stamps(void* buf);
/* Measurement (bench.py): while on, every kernel launched for a tagged library call (tag >= 0) is
 * timed by start / stop events bound to that kernel (hipExtLaunchKernelGGL): its own execution,
 * as rocprofv3 reports it.  stop waits, writes (ms, tag) per launch and returns the count. */
int mrg_probe_start(int cap);
int mrg_probe_tag(int tag);
int mrg_probe_stop(float* ms, int* tags, int cap);

/* Tuning knob: number of workgroups that share one batch row group at H = 256
 * (4, 8 or 16; default 8; 4 measured 2 ms slower on the headline step, r04).  Process-wide; set before capture, not during. */
int mrg_lstm_config(int group256);
/* Tuning knob: members of a persistent GRU ring at H = 256 (4, default, or 8); returns the previous
 * setting.  Process-wide; set before capture, not during. */
int mrg_gru_config(int group256);
/* Solo (one-workgroup, LDS-exchange) recurrence groups at H <= 128: 1 on (default), 0 off; returns the
 * previous setting. */
int mrg_lstm_set_solo(int on);
/* Diagnostics only: record per-step phase clocks (s_memtime) of block 0 of the next
 * LSTM launches into buf ([T][8] u64); null disables.  Never in timed runs. */
int mrg_lstm_debug_stamps(void* buf);
/* Hand-off granule stores at workgroup scope (1, default; the line stays in the XCD's L2 where the
 * group's agent-scope polls read it) or agent scope (0).  Env MRG_LSTM_LOCAL=0 starts with 0. */
int mrg_lstm_set_local_handoff(int on);

/* Timing experiments only: mrg_ssd_gate_cell_fwd (mode 1) with parts removed (dbg 1: no input
 * prologue, 2: no gate GEMM, 3: neither); H = 256.  Outputs are not meaningful for dbg != 0. */
int mrg_ssd_gate_cell_fwd_dbg(int dbg, int B, int H, int mode, const float* xin, const float* hp,
                              const float* rp, const float* gamma, const float* beta, float eps, float* xout,
                              float* mean, float* rstd, const float* w_ih, const float* b_ih,
                              const float* b_hh, float* gates, float* c, float* h, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MRG_TUNING_H_ */
