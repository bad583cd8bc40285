// FETCH_SIZE / WRITE_SIZE calibration for the access patterns of the LSTM recurrences (the guide
// calibrates only 16-B-per-lane streaming reads and stores, MI355X_MICROARCH.md "HBM"):
//   read16 : float4 per lane, coalesced (the guide's case: FETCH_SIZE = 1/2 of the bytes)
//   read4  : one float per lane, 64 lanes on 256 contiguous bytes (the LSTM gx / gates loads)
//   poll8  : one 8-B agent-scope relaxed atomic load per lane (the {tag, value} granule polls),
//            of a ring another kernel has just written
//   store4 / store8 : one float / one agent-scope 8-B atomic store per lane (y / gates, granules)
// Each kernel moves N bytes over a 512 MiB buffer (past the 256 MiB Infinity Cache).
//   hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
//   rocprofv3 --pmc FETCH_SIZE -- tools/pmc_calib      (then WRITE_SIZE in its own pass)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void read16(const float4* __restrict__ p, long n, float* out) {
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float4 v = p[i];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  if (s.x + s.y + s.z + s.w == 1234.5f) out[0] = s.x;
}

__global__ void read4(const float* __restrict__ p, long n, float* out) {
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) s += p[i];
  if (s == 1234.5f) out[0] = s;
}

__global__ void poll8(unsigned long long* p, long n, float* out) {
  unsigned long long s = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (s == 12345ull) out[0] = 1.f;
}

__global__ void store4(float* p, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    p[i] = (float)i;
}

__global__ void store8(unsigned long long* p, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    __hip_atomic_store(p + i, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int main() {
  const long bytes = 512l << 20;
  void* buf = nullptr;
  float* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  const dim3 grid(2048), blk(256);
  for (int rep = 0; rep < 2; ++rep) {
    store4<<<grid, blk>>>((float*)buf, bytes / 4);
    read16<<<grid, blk>>>((const float4*)buf, bytes / 16, out);
    store4<<<grid, blk>>>((float*)buf, bytes / 4);
    read4<<<grid, blk>>>((const float*)buf, bytes / 4, out);
    store8<<<grid, blk>>>((unsigned long long*)buf, bytes / 8);
    poll8<<<grid, blk>>>((unsigned long long*)buf, bytes / 8, out);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("pmc_calib: %ld bytes per kernel (read16, read4, poll8, store4, store8)\n", bytes);
  hipFree(buf);
  hipFree(out);
  return 0;
}
