// Shared helpers for the mr_gen MI355X (gfx950 / CDNA4) kernels.
// C-ABI entry points return 0 on success, non-zero on failure; the message is
// available from mrg_last_error() (thread-local).  No entry point allocates
// device memory or synchronises: every launch is stream-ordered on the
// hipStream_t the caller passes (torch's current stream), so calls are safe
// inside hipGraph capture.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cmath>

#include <hip/hip_ext.h>

#define MRG_API extern "C" __attribute__((visibility("default")))

namespace mrg {

void set_error(const char* fmt, ...);

// Live kernel timing for bench.py (mrg_probe_*): while a probe is on and the host has tagged the
// current library call (tag >= 0), every launch of the probed kernels goes through
// hipExtLaunchKernelGGL with a start / stop event pair that the runtime ties to THAT kernel's own
// execution, so the time per launch is the kernel's, as rocprofv3 reports it (an event recorded on
// the stream before / after a launch also holds the dispatch of the next packet).
struct ProbeState {
  int on = 0, tag = -1, n = 0, cap = 0;
  hipEvent_t* ev = nullptr;  // [cap][2]
  int* tags = nullptr;       // [cap]
};
extern ProbeState g_probe;

template <typename K, typename... A>
inline void klaunch(K kernel, dim3 grid, dim3 block, unsigned shmem, hipStream_t s, A... args) {
  if (g_probe.on && g_probe.tag >= 0 && g_probe.n < g_probe.cap) {
    const int i = g_probe.n++;
    g_probe.tags[i] = g_probe.tag;
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, g_probe.ev[2 * i], g_probe.ev[2 * i + 1], 0, args...);
    return;
  }
  kernel<<<grid, block, shmem, s>>>(args...);
}

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return 1;
  }
  return 0;
}

#define MRG_REQUIRE(cond, ...)            \
  do {                                    \
    if (!(cond)) {                        \
      ::mrg::set_error(__VA_ARGS__);      \
      return 2;                           \
    }                                     \
  } while (0)

#define MRG_HIP(call)                                                        \
  do {                                                                       \
    hipError_t _e = (call);                                                  \
    if (_e != hipSuccess) {                                                  \
      ::mrg::set_error("%s failed: %s", #call, hipGetErrorString(_e));       \
      return 3;                                                              \
    }                                                                        \
  } while (0)

// Gate nonlinearities on the native v_exp_f32 / v_rcp_f32 (1-ulp class; absolute error ~1e-7,
// far inside the 1e-4 parity budget).  exp overflow saturates correctly: rcp(inf) = 0.
__device__ __forceinline__ float sigmoidf_(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __expf(-x));
}
__device__ __forceinline__ float tanhf_(float x) {
  return fmaf(2.0f, __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * x)), -1.0f);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// A row-major operand view with an optional 2-level row map:
//   offset(row, col) = (row / rdiv) * ld_hi + (row % rdiv) * ld_lo + col
// rdiv == 0 means "plain": offset = row * ld_lo + col.  The 2-level form lets
// one GEMM walk [B, T, F] tensors with a time shift (e.g. h_{t-1} for dW_hh)
// or a [:, lead:] slice without a copy.
struct RowMap {
  long ld_lo;
  long ld_hi;
  int rdiv;
  __host__ __device__ __forceinline__ long off(long row) const {
    if (rdiv <= 0) return row * ld_lo;
    long q = row / rdiv;
    return q * ld_hi + (row - q * rdiv) * ld_lo;
  }
};

}  // namespace mrg
