// pmc_calib — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the access
// widths the tick kernels use (4-byte and 8-byte per lane, fully coalesced),
// per MI355X_MICROARCH.md §HBM ("other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").
// Each kernel moves exactly BYTES bytes over a 1 GiB buffer (beyond the
// 256 MiB Infinity Cache); tools/pmc_summary.py divides the counters by it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr size_t BYTES = size_t(1) << 30;

__global__ void read_u32(const unsigned* __restrict__ in, unsigned* __restrict__ sink, size_t n) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    acc += in[i];
  if (acc == 0x9E3779B9u) sink[0] = acc;   // keeps the loads live, practically never stores
}
__global__ void write_u32(unsigned* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    out[i] = unsigned(i);
}
__global__ void read_u64(const unsigned long long* __restrict__ in, unsigned long long* __restrict__ sink, size_t n) {
  unsigned long long acc = 0;
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    acc += in[i];
  if (acc == 0x9E3779B97F4A7C15ull) sink[0] = acc;
}
__global__ void write_u64(unsigned long long* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    out[i] = i;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  void *a = nullptr, *b = nullptr, *sink = nullptr;
  CK(hipMalloc(&a, BYTES));
  CK(hipMalloc(&b, BYTES));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 1, BYTES));
  const dim3 grid(256 * 16), block(256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read_u32, grid, block, 0, 0, (const unsigned*)a, (unsigned*)sink, BYTES / 4);
    hipLaunchKernelGGL(write_u32, grid, block, 0, 0, (unsigned*)b, BYTES / 4);
    hipLaunchKernelGGL(read_u64, grid, block, 0, 0, (const unsigned long long*)b, (unsigned long long*)sink, BYTES / 8);
    hipLaunchKernelGGL(write_u64, grid, block, 0, 0, (unsigned long long*)a, BYTES / 8);
  }
  CK(hipDeviceSynchronize());
  printf("pmc_calib: %zu bytes per kernel\n", BYTES);
  return 0;
}
