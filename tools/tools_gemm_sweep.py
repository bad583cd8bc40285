"""Sweep GEMM arithmetic mode x tile shape (x split-K for weight gradients) on the step's shapes.

    python tools/tools_gemm_sweep.py            (on a GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import _lib  # noqa: E402
from tools_gemm_bench import SHAPES, run_shape  # noqa: E402
import tools_gemm_bench as TB  # noqa: E402
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402


def main():
    lib = _lib.load()
    for name, M, N, K, ta, tb, calls, wgrad in SHAPES:
        best = None
        for mode in (0, 1):
            _lib.check(lib.mrg_gemm_set_mode(mode), "mode")
            for tile in (0, 1, 2):
                _lib.check(lib.mrg_gemm_force_tile(tile), "tile")
                for splits in ((4, 8, 16, 32, 64) if wgrad else (1,)):
                    orig = Fn.wgrad_splits
                    Fn.wgrad_splits = lambda *a, s=splits: s
                    try:
                        ms, _, err = run_shape(M, N, K, ta, tb, wgrad, iters=10)
                    finally:
                        Fn.wgrad_splits = orig
                    tf = 2.0 * M * N * K / (ms / 1e3) / 1e12
                    line = f"{name:18s} mode={mode} tile={tile} splits={splits:3d} {ms*1e3:8.1f} us {tf:6.1f} TF/s err={err:.1e}"
                    print(line, flush=True)
                    if best is None or ms < best[0]:
                        best = (ms, line)
        print("BEST", best[1], flush=True)
    _lib.check(lib.mrg_gemm_force_tile(-1), "tile")


if __name__ == "__main__":
    main()
