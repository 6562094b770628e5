// Queue-ordering probe (diagnostics, not product): does a kernel launched
// with hipExtAnyOrderLaunch start before the previous kernel of its stream
// ends, and what does a wait on an already-completed event of another stream
// cost at a kernel boundary? Kernels stamp the device's constant 100-MHz
// clock into a buffer; the host prints the gaps in microseconds.
//
//   order_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

// every block spins for `ticks` of the 100-MHz clock; block 0 lane 0 stamps start / end
__global__ __launch_bounds__(64) void spin(unsigned long long* out, int slot, unsigned long long ticks) {
  const unsigned long long t0 = now();
  if (blockIdx.x == 0 && threadIdx.x == 0) out[2 * slot] = t0;
  while (now() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) out[2 * slot + 1] = now();
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

static void report(const char* what, const unsigned long long* h, int a, int b) {
  // gap from the end of kernel a to the start of kernel b (negative: overlap)
  printf("%-58s end(a) -> start(b) %8.1f us  (a %6.1f us, b %6.1f us)\n", what,
         (double(h[2 * b]) - double(h[2 * a + 1])) / 100.0, (h[2 * a + 1] - h[2 * a]) / 100.0,
         (h[2 * b + 1] - h[2 * b]) / 100.0);
}

int main() {
  unsigned long long* d = nullptr;
  unsigned long long h[64];
  CK(hipMalloc(&d, sizeof h));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t ev, evt;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreate(&evt));
  const unsigned long long T100 = 10000, T20 = 2000;   // 100 us, 20 us
  auto K = [&](hipStream_t st, int slot, unsigned long long ticks, hipEvent_t stop, uint32_t fl = 0) {
    hipExtLaunchKernelGGL(spin, dim3(256), dim3(64), 0, st, nullptr, stop, fl, d, slot, ticks);
  };
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemset(d, 0, sizeof h));
    CK(hipDeviceSynchronize());
    printf("-- repeat %d\n", rep);
    // same stream, plain and with hipExtAnyOrderLaunch
    K(s0, 0, T100, nullptr); K(s0, 1, T20, nullptr);
    K(s0, 2, T100, nullptr); K(s0, 3, T20, nullptr, hipExtAnyOrderLaunch);
    CK(hipDeviceSynchronize());
    // A: wait for a running kernel of another stream that ends after this stream's kernel (marker event)
    K(s1, 4, T100 + 3000, nullptr); CK(hipEventRecord(ev, s1));
    K(s0, 5, T100, nullptr); CK(hipStreamWaitEvent(s0, ev, 0)); K(s0, 6, T20, nullptr);
    CK(hipDeviceSynchronize());
    // A': the same with the kernel's own stop event
    K(s1, 7, T100 + 3000, evt);
    K(s0, 8, T100, nullptr); CK(hipStreamWaitEvent(s0, evt, 0)); K(s0, 9, T20, nullptr);
    CK(hipDeviceSynchronize());
    // B: the other stream's kernel ends long before this stream's kernel (stop event)
    K(s1, 10, T20, evt);
    K(s0, 11, T100, nullptr); CK(hipStreamWaitEvent(s0, evt, 0)); K(s0, 12, T20, nullptr);
    CK(hipDeviceSynchronize());
    // D: an idle stream waits for a running kernel of another (stop event)
    K(s0, 13, T100, evt); CK(hipStreamWaitEvent(s1, evt, 0)); K(s1, 14, T20, nullptr);
    CK(hipDeviceSynchronize());
    // E: a busy stream (its kernel ends first) waits for a running kernel of another (stop event)
    K(s0, 15, T100, evt); K(s1, 16, T100 - 4000, nullptr); CK(hipStreamWaitEvent(s1, evt, 0)); K(s1, 17, T20, nullptr);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
    report("same stream, plain", h, 0, 1);
    report("same stream, second with hipExtAnyOrderLaunch", h, 2, 3);
    report("A: after another stream's running kernel (marker event)", h, 4, 6);
    report("A: ... this stream's kernel end", h, 5, 6);
    report("A': after another stream's running kernel (stop event)", h, 7, 9);
    report("A': ... this stream's kernel end", h, 8, 9);
    report("B: other stream's kernel done early: this stream's end", h, 11, 12);
    report("D: idle stream after another's running kernel", h, 13, 14);
    report("E: busy stream after another's running kernel", h, 15, 17);
    report("E: ... this stream's kernel end", h, 16, 17);
  }
  return 0;
}
