"""Run ONE planes GEMM shape repeatedly (for rocprofv3 passes): python tools/gemm_one.py M N K cfg [iters]."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import _lib, functional as Fn  # noqa: E402

M, N, K, cfg = (int(x) for x in sys.argv[1:5])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
lib = _lib.load()
VP, CI = ctypes.c_void_p, ctypes.c_int
dev = "cuda:0"
A = torch.randn(M, K, device=dev)
B = torch.randn(N, K, device=dev)
C = torch.zeros(M, N, device=dev)
planes = torch.empty(3, N, K, dtype=torch.int16, device=dev)
st = VP(torch.cuda.current_stream().cuda_stream)
_lib.check(lib.mrg_split_planes_batched(1, (VP * 1)(Fn._ptr(B)), (VP * 1)(VP(planes.data_ptr())), (CI * 1)(N),
                                        (CI * 1)(K), (CI * 1)(0), st), "split")
lib.mrg_gemm_set_wide(cfg)
for _ in range(iters):
    _lib.check(lib.mrg_gemm_x6_planes(M, N, K, 1.0, Fn._ptr(A), K, 0, 0, VP(planes.data_ptr()), K, N * K, 0.0,
                                      Fn._ptr(C), N, None, 0, None, 0, st), "planes")
torch.cuda.synchronize()
print("ok")
if os.environ.get("STAMPS"):
    st_buf = torch.zeros(8 * 16, dtype=torch.int64, device=dev)
    lib.mrg_gemm_debug_stamps(VP(st_buf.data_ptr()))
    for _ in range(3):
        _lib.check(lib.mrg_gemm_x6_planes(M, N, K, 1.0, Fn._ptr(A), K, 0, 0, VP(planes.data_ptr()), K, N * K, 0.0,
                                          Fn._ptr(C), N, None, 0, None, 0, st), "planes")
    torch.cuda.synchronize()
    lib.mrg_gemm_debug_stamps(None)
    v = st_buf.view(8, 16).cpu()
    t0 = v[:, 0][v[:, 0] > 0].min().item()
    for w in range(8):
        row = [x - t0 for x in v[w].tolist() if x > 0]
        print(f"wave {w}: " + " ".join(str(x) for x in row) + "   deltas " + " ".join(str(b - a) for a, b in zip(row, row[1:])))
