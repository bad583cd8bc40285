// Error plumbing + library identity for libmrg.so.
#include "mrg_common.h"
#include <cstdarg>

namespace mrg {
static thread_local char g_err[1024] = "";
ProbeState g_probe;

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace mrg

MRG_API const char* mrg_last_error(void) { return mrg::g_err; }

MRG_API int mrg_version(void) { return 100; }

// Device query used by the host side to size persistent grids.
MRG_API int mrg_device_cu_count(int device, int* out) {
  hipDeviceProp_t p;
  MRG_HIP(hipGetDeviceProperties(&p, device));
  *out = p.multiProcessorCount;
  return 0;
}

// Tests only: a kernel that keeps `blocks` workgroups of `threads` lanes (and `lds` bytes of LDS
// each) resident for `usec` microseconds of wall clock, standing in for a CU-occupying kernel on
// another stream (an RCCL collective beside the backward): a persistent recurrence launched
// behind it must wait for CUs, not time out its hand-offs.
namespace mrg {
__global__ void busy_kernel(unsigned long long ticks, float* sink) {
  extern __shared__ float scratch[];
  const unsigned long long t0 = wall_clock64();
  float acc = 0.0f;
  while (wall_clock64() - t0 < ticks) acc += 1.0f;
  scratch[threadIdx.x] = acc;
  __syncthreads();
  if (sink && threadIdx.x == 0 && scratch[0] < 0.0f) sink[blockIdx.x] = scratch[0];   // never taken
}
// one wall-clock stamp (100 MHz, the same clock on every XCD) into buf[slot], by a 1-thread kernel
// placed in a stream's order: diagnostics of when a point of a replayed graph was reached
__global__ void stamp_kernel(unsigned long long* buf, int slot) { buf[slot] = wall_clock64(); }
}  // namespace mrg

MRG_API int mrg_debug_stamp(void* buf, int slot, hipStream_t stream) {
  MRG_REQUIRE(buf && slot >= 0, "mrg_debug_stamp: bad slot");
  mrg::stamp_kernel<<<1, 1, 0, stream>>>(static_cast<unsigned long long*>(buf), slot);
  return mrg::check_launch("stamp_kernel");
}

MRG_API int mrg_debug_busy(int blocks, int threads, int lds, double usec, hipStream_t stream) {
  MRG_REQUIRE(blocks > 0 && threads > 0 && threads <= 1024 && lds >= threads * 4 && lds <= 160 * 1024,
              "mrg_debug_busy: bad shape");
  MRG_REQUIRE(usec >= 0.0 && usec <= 2e6, "mrg_debug_busy: usec out of range");
  int dev = 0, khz = 0;
  MRG_HIP(hipGetDevice(&dev));
  MRG_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  const unsigned long long ticks = (unsigned long long)(usec * 1e-3 * (khz > 0 ? khz : 100000));
  if (lds > 64 * 1024) MRG_HIP(hipFuncSetAttribute((const void*)mrg::busy_kernel,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  mrg::busy_kernel<<<blocks, threads, lds, stream>>>(ticks, nullptr);
  return mrg::check_launch("busy_kernel");
}

using mrg::g_probe;

// Live per-kernel timing (bench.py): up to `cap` launches of the tagged library calls are timed
// with kernel-bound events (klaunch, mrg_common.h).  Not for graph capture.
MRG_API int mrg_probe_start(int cap) {
  MRG_REQUIRE(cap > 0 && cap <= (1 << 16), "mrg_probe_start: cap %d out of range", cap);
  if (g_probe.cap < cap) {
    for (int i = 0; i < 2 * g_probe.cap; ++i) (void)hipEventDestroy(g_probe.ev[i]);
    delete[] g_probe.ev;
    delete[] g_probe.tags;
    g_probe.ev = new hipEvent_t[2 * cap];
    g_probe.tags = new int[cap];
    for (int i = 0; i < 2 * cap; ++i) MRG_HIP(hipEventCreate(&g_probe.ev[i]));
    g_probe.cap = cap;
  }
  g_probe.n = 0;
  g_probe.tag = -1;
  g_probe.on = 1;
  return 0;
}

// Tag of the following launches (the host's library-call index), -1 = not timed.
MRG_API int mrg_probe_tag(int tag) {
  g_probe.tag = tag;
  return 0;
}

// Stop; waits for the timed launches and writes (kernel ms, tag) per launch; returns the count.
MRG_API int mrg_probe_stop(float* ms, int* tags, int cap) {
  g_probe.on = 0;
  g_probe.tag = -1;
  const int n = g_probe.n < cap ? g_probe.n : cap;
  for (int i = 0; i < n; ++i) {
    if (hipEventSynchronize(g_probe.ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&ms[i], g_probe.ev[2 * i], g_probe.ev[2 * i + 1]) != hipSuccess) {
      mrg::set_error("mrg_probe_stop: event %d failed", i);
      return -1;
    }
    tags[i] = g_probe.tags[i];
  }
  g_probe.n = 0;
  return n;
}
