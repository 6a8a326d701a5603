// Dev probe (GPU box): device-time cost of the stream-ordering primitives the pipeline's ingest
// can use between two kernels of the compute stream. Each variant enqueues N x [kernel, op] and
// reports the mean per-iteration time from two events around the loop, minus the kernel-only loop.
// Build: hipcc -O2 --offload-arch=gfx950 tools/probe/probe_sync.hip -o tools/probe/probe_sync
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);   \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ void k_work(double* a, int n) {  // ~5-10 us of trivial streaming work
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = a[i] * 1.0000001 + 1e-9;
}

int main() {
  const int n = 1 << 22, N = 400;
  double* a;
  CK(hipMalloc(&a, n * sizeof(double)));
  CK(hipMemset(a, 0, n * sizeof(double)));
  unsigned* flag;
  CK(hipMalloc((void**)&flag, 64));
  CK(hipMemset(flag, 0, 64));
  hipStream_t s, c;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  hipEvent_t t0, t1, e_def, e_nt, e_nsf, e_dev, e_other;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  CK(hipEventCreate(&e_def));
  CK(hipEventCreateWithFlags(&e_nt, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&e_nsf, hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventCreateWithFlags(&e_dev, hipEventDisableTiming | hipEventReleaseToDevice));
  CK(hipEventCreateWithFlags(&e_other, hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventRecord(e_other, c));  // recorded (complete) on the other stream
  CK(hipStreamSynchronize(c));
  const char* names[] = {"kernel only", "eventRecord default", "eventRecord disableTiming",
                         "eventRecord disableSystemFence", "eventRecord releaseToDevice",
                         "streamWaitEvent (done, default-fence event)", "streamWaitEvent (done, no-fence event)",
                         "streamWriteValue32", "streamWaitValue32 (satisfied)"};
  hipEvent_t e_other_def;
  CK(hipEventCreateWithFlags(&e_other_def, hipEventDisableTiming));
  CK(hipEventRecord(e_other_def, c));
  CK(hipStreamSynchronize(c));
  double base = 0.0;
  for (int rep = 0; rep < 2; ++rep) {
    for (int v = 0; v < 9; ++v) {
      for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k_work, dim3(n / 256), dim3(256), 0, s, a, n);
      CK(hipEventRecord(t0, s));
      for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(k_work, dim3(n / 256), dim3(256), 0, s, a, n);
        switch (v) {
          case 1: CK(hipEventRecord(e_def, s)); break;
          case 2: CK(hipEventRecord(e_nt, s)); break;
          case 3: CK(hipEventRecord(e_nsf, s)); break;
          case 4: CK(hipEventRecord(e_dev, s)); break;
          case 5: CK(hipStreamWaitEvent(s, e_other_def, 0)); break;
          case 6: CK(hipStreamWaitEvent(s, e_other, 0)); break;
          case 7: CK(hipStreamWriteValue32(s, flag, (uint32_t)i, 0)); break;
          case 8: CK(hipStreamWaitValue32(s, flag, 0, hipStreamWaitValueGte, 0xFFFFFFFFu)); break;
          default: break;
        }
      }
      CK(hipEventRecord(t1, s));
      CK(hipEventSynchronize(t1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, t0, t1));
      const double us = 1e3 * ms / N;
      if (v == 0) base = us;
      if (rep == 1) std::printf("%-48s %8.2f us/iter  (+%.2f)\n", names[v], us, us - base);
    }
  }
  return 0;
}
