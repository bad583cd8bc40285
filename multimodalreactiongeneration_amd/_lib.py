"""ctypes binding of libmrg.so (declared in include/mrg.h).

The library is built in-tree by ``__graft_entry__.build()`` /
``make -C multimodalreactiongeneration_amd/csrc``.  There is deliberately no
fallback: every op of the MI355X path goes through this library and raises if
it is missing or if no HIP device is present.  ``torch`` is imported first so
the library binds to the HIP runtime torch already loaded
(``libamdhip64.so.7``).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (load torch's HIP runtime before libmrg.so)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MRG_LIB_PATH", os.path.join(_HERE, "libmrg.so"))

c_int, c_long, c_float, c_size, c_void = (ctypes.c_int, ctypes.c_long, ctypes.c_float,
                                          ctypes.c_size_t, ctypes.c_void_p)
P = ctypes.c_void_p
PP = ctypes.POINTER(ctypes.c_void_p)
PL = ctypes.POINTER(ctypes.c_long)
PI = ctypes.POINTER(ctypes.c_int)

# name -> (restype, argtypes)
SIGNATURES = {
    "mrg_last_error": (ctypes.c_char_p, []),
    "mrg_version": (c_int, []),
    "mrg_device_cu_count": (c_int, [c_int, PI]),
    "mrg_gemm_workspace_bytes": (c_size, [c_int, c_int, c_int]),
    "mrg_gemm_set_mode": (c_int, [c_int]),
    "mrg_gemm_get_mode": (c_int, []),
    "mrg_gemm_force_tile": (c_int, [c_int]),
    "mrg_gemm_set_blocks_per_cu": (c_int, [c_int]),
    "mrg_attention_set_fused": (c_int, [c_int]),
    "mrg_gemm_set_glds": (c_int, [c_int, c_int]),
    "mrg_gemm_set_glds_wg": (c_int, [c_int]),
    "mrg_transpose_batched": (c_int, [c_int, PP, PP, PI, PI, P]),
    "mrg_split_planes_batched": (c_int, [c_int, PP, PP, PI, PI, PI, P]),
    "mrg_gemm_set_wide": (c_int, [c_int]),
    "mrg_gemm_x6_planes_batched": (c_int, [c_int, c_int, c_int, c_int, c_float, P, c_long, P, c_long, c_long, c_float,
                                           P, c_long, P, c_int, P, c_long, P]),
    "mrg_gemm_x6_planes": (c_int, [c_int, c_int, c_int, c_float, P, c_long, c_long, c_int, P, c_long, c_long,
                                   c_float, P, c_long, P, c_int, P, c_long, P]),
    "mrg_lstm_set_blocks_per_cu": (c_int, [c_int]),
    "mrg_gemm_x6_variant": (c_int, [c_int, c_int, c_int, c_int, P, P, P, P]),
    "mrg_gemm_f32": (c_int, [c_int, c_int, c_int, c_float,
                             P, c_int, c_long, c_long, c_int,
                             P, c_int, c_long, c_long, c_int,
                             c_float, P, c_long, P, c_int, P, c_long, P, c_int, P]),
    "mrg_gemm_f32_ex": (c_int, [c_int, c_int, c_int, c_float,
                                P, c_int, c_long, c_long, c_int,
                                P, c_int, c_long, c_long, c_int,
                                c_float, P, c_long, P, c_int, P, c_long, P, c_int,
                                P, P, c_float, P, P]),
    "mrg_gemm_bf16_ex": (c_int, [c_int, c_int, c_int, c_float,
                                 P, c_int, c_long, c_long, c_int,
                                 P, c_int, c_long, c_long, c_int,
                                 c_float, P, c_long, P, c_int, P, c_long, P, c_int,
                                 P, P, c_float, P, P]),
    "mrg_gemm_x6g_batched": (c_int, [c_int, c_int, c_int, c_int, c_float, PP, c_long, PP, c_long, c_float, PP,
                                     c_long, PP, c_int, PP, c_long, c_int, P]),
    "mrg_colsum_workspace_bytes": (c_size, [c_int, c_int]),
    "mrg_colsum_f32": (c_int, [c_int, c_int, P, c_long, c_long, c_int, c_float, P, P, P, P]),
    "mrg_lstm_supported_hidden": (c_int, [c_int]),
    "mrg_lstm_fwd_xbuf_bytes": (c_size, [c_int, c_int]),
    "mrg_lstm_bwd_xbuf_bytes": (c_size, [c_int, c_int]),
    "mrg_lstm_fwd": (c_int, [c_int, c_int, c_int, c_int,
                             PP, PL, PL, PP, PP, PP, PP,
                             PP, PL, PL, PP, PP, PP, PP,
                             PI, PP, PL, P, c_int, c_int, P]),
    "mrg_lstm_bwd": (c_int, [c_int, c_int, c_int, c_int,
                             PP, PP, PP, PP, PP, PL, PL, PP, PP,
                             PP, PP, PP, PI, PP, PL, P, c_int, c_int, P]),
    "mrg_lstm_config": (c_int, [c_int]),
    "mrg_lstm_set_solo": (c_int, [c_int]),
    "mrg_gru_config": (c_int, [c_int]),
    "mrg_lstm_set_mx": (c_int, [c_int, c_int]),
    "mrg_lstm_cell_fwd": (c_int, [c_int, c_int, P, c_long, P, P, P, P, P, c_long, P, P]),
    "mrg_lstm_cell_bwd": (c_int, [c_int, c_int, P, P, P, P, c_long, P, P, P, P, P]),
    "mrg_gru_cell_fwd": (c_int, [c_int, c_int, P, c_long, P, P, P, c_long, P, c_long, P, c_long, P, c_long, P]),
    "mrg_gru_cell_bwd": (c_int, [c_int, c_int, P, c_long, P, c_long, P, c_long, P, c_long, P, P, P, c_long, P, P]),
    "mrg_gru_supported_hidden": (c_int, [c_int]),
    "mrg_gru_xbuf_bytes": (c_size, [c_int, c_int]),
    "mrg_gru_fwd": (c_int, [c_int, c_int, c_int, P, c_long, c_long, P, P, P, P, c_long, c_long, P, c_long, c_long,
                            P, c_long, c_long, c_int, P, P, c_int, P]),
    "mrg_gru_bwd": (c_int, [c_int, c_int, c_int, P, P, c_long, c_long, P, c_long, c_long, P, c_long, c_long, P,
                            P, c_long, c_long, P, P, P, c_long, c_long, P, c_int, P, P, c_int, P]),
    "mrg_fbank_finish": (c_int, [c_int, c_int, c_int, P, c_long, P, P, c_long, c_int, c_int, c_long, P, c_long, P]),
    "mrg_feature_delta": (c_int, [c_int, c_int, c_int, P, c_long, c_int, P, P]),
    "mrg_pad_sequences": (c_int, [c_int, c_int, c_int, P, P, c_float, P, P]),
    "mrg_lstm_debug_stamps": (c_int, [P]),
    "mrg_lstm_set_local_handoff": (c_int, [c_int]),
    "mrg_attention_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int,
                                  P, c_long, c_long, P, c_long, c_long, P, c_long, c_long,
                                  P, c_long, c_long, P, P, P, c_int, c_float, P]),
    "mrg_attention_bwd_workspace_bytes": (c_size, [c_int, c_int, c_int]),
    "mrg_attention_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int,
                                  P, c_long, c_long, P, c_long, c_long, P, c_long, c_long,
                                  P, c_long, c_long, P, P, P, c_int, c_float,
                                  P, c_long, c_long, P, c_long, c_long, P, c_long, c_long,
                                  P, c_long, c_long, P, P]),
    "mrg_attention_fwd_chunk": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                        P, c_long, c_long, P, c_long, c_long, P, c_long, c_long,
                                        P, c_long, c_long, P, P, P, c_int, c_float, P]),
    "mrg_attention_bwd_chunk": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                        P, c_long, c_long, P, c_long, c_long, P, c_long, c_long,
                                        P, c_long, c_long, P, P, P, c_int, c_float,
                                        P, c_long, c_long, P, c_long, c_long, P, c_long, c_long,
                                        P, c_long, c_long, c_int, c_int, P, P]),
    "mrg_residual_layernorm_fwd": (c_int, [c_int, c_int, P, P, P, P, c_float, P, P, P, P]),
    "mrg_residual_layernorm_bwd_workspace_bytes": (c_size, [c_int, c_int]),
    "mrg_residual_layernorm_bwd": (c_int, [c_int, c_int, P, P, P, P, P, P, P, P, P, c_int, P, P]),
    "mrg_residual_layernorm_param_reduce": (c_int, [c_int, c_int, P, P, P, c_int, P]),
    "mrg_residual_layernorm_fwd_map": (c_int, [c_int, c_int, P, P, P, P, c_float, P, c_long, c_long, c_int,
                                               P, P, P]),
    "mrg_residual_layernorm_bwd_map": (c_int, [c_int, c_int, P, c_long, c_long, c_int, P, P, P, P, P, P, P, P]),
    "mrg_residual_layernorm_fwd_batched": (c_int, [c_int, c_int, c_int, PP, PP, PP, PP, c_float, PP, PL, PL, PI,
                                                   PP, PP, P]),
    "mrg_residual_layernorm_bwd_batched": (c_int, [c_int, c_int, c_int, PP, PL, PL, PI, PP, PP, PP, PP, PP, PP,
                                                   PP, P]),
    "mrg_debug_busy": (c_int, [c_int, c_int, c_int, ctypes.c_double, P]),
    "mrg_debug_stamp": (c_int, [P, c_int, P]),
    "mrg_padding_flags": (c_int, [c_int, c_int, P, c_long, c_long, c_float, P, P]),
    "mrg_zero_padding": (c_int, [c_long, P, c_float, P, P]),
    "mrg_swap01": (c_int, [c_int, c_int, c_int, P, P, c_float, P]),
    "mrg_fill_zero": (c_int, [P, c_long, P]),
    "mrg_probe_start": (c_int, [c_int]),
    "mrg_probe_tag": (c_int, [c_int]),
    "mrg_probe_stop": (c_int, [ctypes.POINTER(ctypes.c_float), PI, c_int]),
    "mrg_loss_workspace_bytes": (c_size, [c_int, c_int, c_int]),
    "mrg_masked_loss_fwd": (c_int, [c_int, c_int, c_int, P, c_long, P, c_int, c_float, c_float,
                                    c_int, c_int, c_float, P, P, P]),
    "mrg_masked_loss_bwd": (c_int, [c_int, c_int, c_int, P, c_long, P, c_int, c_float, c_float,
                                    c_int, c_int, c_float, P, P, P]),
    "mrg_broadcast_loss_workspace_bytes": (c_size, [c_int, c_int, c_int]),
    "mrg_broadcast_loss_fwd": (c_int, [c_int, c_int, c_int, P, c_long, P, P, c_long, c_long, c_int, c_int,
                                       c_float, c_float, c_int, c_float, P, P, P]),
    "mrg_broadcast_loss_bwd": (c_int, [c_int, c_int, c_int, P, c_long, P, P, c_long, c_long, c_int, c_int,
                                       c_float, c_float, c_int, c_float, P, P, P, P]),
    "mrg_ssd_gate_cell_fwd": (c_int, [c_int, c_int, c_int, P, P, P, P, P, c_float, P, P, P, P, P, P, P, P, P, P]),
    "mrg_ssd_gate_cell_fwd_dbg": (c_int, [c_int, c_int, c_int, c_int, P, P, P, P, P, c_float, P, P, P, P, P, P, P,
                                          P, P, P]),
    "mrg_ssd_feat_gate_cell_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, P, P, P, c_long, c_long,
                                           P, P, c_long, P, P, P, P, P, P, P, P, P]),
    "mrg_ssd_dx": (c_int, [c_int, c_int, P, P, P, P, P]),
    "mrg_lstm_step_fwd": (c_int, [c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, c_long, P, P]),
    "mrg_gen_lstm": (c_int, [c_int, c_int, P, P, P, P, P, P, P, c_float, P, P, P, P, P, P]),
    "mrg_gen_linear": (c_int, [c_int, c_int, PP, PP, PP, PP, c_long, PP, PP, PP, c_float, P, c_long, PP, PP, P,
                               c_long, P]),
    "mrg_gen_ffn": (c_int, [c_int, c_int, P, P, P, P, c_float, P, P, P, P, P, P, c_long, P, P, P, c_int, P]),
    "mrg_gen_loop_ring_bytes": (c_long, [c_int]),
    "mrg_gen_loop_fits": (c_int, [c_int, c_int]),
    "mrg_gen_loop_debug_stamps": (c_int, [P]),
    "mrg_ssd_loop_debug_stamps": (c_int, [P]),
    "mrg_ssd_loop_bwd_debug_stamps": (c_int, [P]),
    "mrg_gen_loop": (c_int, [c_int, c_int, c_int, c_int, c_float, PP, c_int, P, P, P, P, P, P]),
    "mrg_ssd_loop_ring_bytes": (c_long, [c_int, c_int]),
    "mrg_ssd_loop_fits": (c_int, [c_int, c_int]),
    "mrg_ssd_loop_fwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_float, PP, c_int, P, P, P, P, P, P,
                                 P, c_long, c_long, P, P, P, P]),
    "mrg_ssd_loop_bwd_ring_bytes": (c_long, [c_int]),
    "mrg_ssd_loop_bwd_fits": (c_int, [c_int, c_int]),
    "mrg_ssd_loop_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, PP, c_int, P, P, P, P, P, P, P, P, P, P, P,
                                 P, P]),
    "mrg_ssd_ffn_z_fwd": (c_int, [c_int, c_int, c_int, P, P, P, P, c_float, P, P, P, P, P, P, P]),
    "mrg_ssd_y_fwd": (c_int, [c_int, c_int, c_int, P, P, P, P, c_long, P]),
    "mrg_ssd_ffn_bwd": (c_int, [c_int, c_int, c_int, c_int, c_int, P, c_long, P, P, P, P, P, P, P, P, P, P, P,
                                P, P, P, P, P, P, P, P, P, P, P]),
    "mrg_ssd_ln_cell_bwd": (c_int, [c_int, c_int, P, P, P, P, P, P, P, P, P, P, c_int, P, P, P, P]),
    "mrg_adamw_step": (c_int, [P, P, P, P, c_long, P, c_float, c_float, c_float, c_float, P, P]),
    "mrg_lstm_debug_inject": (c_int, [c_int]),
    "mrg_comm_available": (c_int, []),
    "mrg_comm_id_bytes": (c_size, []),
    "mrg_comm_unique_id": (c_int, [P]),
    "mrg_comm_init": (c_int, [ctypes.POINTER(ctypes.c_void_p), c_int, P, c_int]),
    "mrg_comm_allreduce_f32": (c_int, [P, P, PL, PL, c_int, c_int, P]),
    "mrg_comm_destroy": (c_int, [P]),
}

_lock = threading.Lock()
_lib = None


def load(path: str = LIB_PATH):
    """Load libmrg.so (cached).  Raises with a clear message if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(
                f"libmrg.so not found at {path}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` "
                "(or make -C multimodalreactiongeneration_amd/csrc). "
                "There is no CPU / PyTorch fallback for the MI355X path.")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def exported_symbols():
    return list(SIGNATURES.keys())


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = load().mrg_last_error().decode(errors="replace")
        raise RuntimeError(f"libmrg {what} failed (code {rc}): {msg}")


def require_device(t: torch.Tensor):
    if not t.is_cuda:
        raise RuntimeError("the MI355X path needs HIP device tensors (got a CPU tensor); "
                           "there is no CPU fallback — use oracle/ for CPU reference math")


_cu_cache = {}


def cu_count(device: int) -> int:
    if device not in _cu_cache:
        out = ctypes.c_int(0)
        check(load().mrg_device_cu_count(device, ctypes.byref(out)), "device query")
        _cu_cache[device] = out.value
    return _cu_cache[device]
