// Kernel-boundary latency probe (diagnostics, not product): how long after a
// kernel's last wave the next kernel of the same stream (or of another stream
// waiting on an event) starts, as a function of how many dirty L2 lines the
// first kernel leaves behind. Run under `rocprofv3 --kernel-trace` and read
// the gaps with tools/gap_summary.py.
//
//   gap_probe <mode>   mode 0: same stream, 1: second stream after an event
//
// Each round: `dirty` (one 4-B store into each of `lines` distinct 128-B lines
// of a 2 GiB buffer, plain or non-temporal, or one whole line per 32 lanes),
// then `tiny`. The kernel names carry the variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int KIND>   // 0: plain partial lines, 1: non-temporal partial lines, 2: plain whole lines
__global__ __launch_bounds__(256) void dirty(int* p, unsigned long long lines, unsigned long long span, int v) {
  const unsigned long long i = blockIdx.x * 256ull + threadIdx.x;
  if (KIND == 2) {
    const unsigned long long line = i / 32ull;
    if (line >= lines) return;
    const unsigned long long l = (line * 2654435761ull) % span;
    p[l * 32ull + (i & 31ull)] = v;
    return;
  }
  if (i >= lines) return;
  const unsigned long long l = (i * 2654435761ull) % span;   // scattered lines
  if (KIND == 1) __builtin_nontemporal_store(v, p + l * 32ull);
  else p[l * 32ull] = v;
}

__global__ void tiny(int* q) {
  if (threadIdx.x == 0 && blockIdx.x == 0) q[0] += 1;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const unsigned long long span = (2ull << 30) / 128ull;   // lines in 2 GiB
  int* p = nullptr;
  int* q = nullptr;
  CK(hipMalloc(&p, span * 128ull));
  CK(hipMalloc(&q, 256));
  CK(hipMemset(p, 0, span * 128ull));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const unsigned long long sizes[] = {0ull, 1ull << 14, 1ull << 16, 1ull << 18, 1ull << 20, 1ull << 22};
  for (int kind = 0; kind < 3; ++kind)
    for (unsigned long long lines : sizes) {
      const unsigned long long thr = kind == 2 ? lines * 32ull : lines;
      const unsigned blocks = unsigned(thr / 256ull) + 1u;
      for (int r = 0; r < 12; ++r) {
        if (kind == 0) hipLaunchKernelGGL(dirty<0>, dim3(blocks), dim3(256), 0, s0, p, lines, span, r);
        if (kind == 1) hipLaunchKernelGGL(dirty<1>, dim3(blocks), dim3(256), 0, s0, p, lines, span, r);
        if (kind == 2) hipLaunchKernelGGL(dirty<2>, dim3(blocks), dim3(256), 0, s0, p, lines, span, r);
        if (mode == 1) {
          CK(hipEventRecord(ev, s0));
          CK(hipStreamWaitEvent(s1, ev, 0));
          hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s1, q);
          CK(hipEventRecord(ev, s1));
          CK(hipStreamWaitEvent(s0, ev, 0));
        } else {
          hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s0, q);
        }
      }
      CK(hipDeviceSynchronize());
      printf("kind %d lines %llu done\n", kind, lines);
      fflush(stdout);
    }
  CK(hipDeviceSynchronize());
  return 0;
}
