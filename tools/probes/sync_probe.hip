// host-sync latency probe: a tiny kernel, then (a) hipStreamSynchronize, (b) a synchronous
// 16-byte hipMemcpy D2H, (c) an async D2H into pinned memory + event spin (hipEventQuery),
// (d) hipEventSynchronize; per variant the mean wall time of kernel + sync over 2000 reps
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
__global__ void k_tiny(int* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1; }
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
int main() {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* d; CK(hipMalloc(&d, 4096)); CK(hipMemset(d, 0, 4096));
  int* hp; CK(hipHostMalloc(&hp, 4096, hipHostMallocDefault));
  int hv[4];
  hipEvent_t ev; CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const int N = 2000;
  for (int v = 0; v < 5; ++v) {
    for (int w = 0; w < 2; ++w) {
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s, d);
        if (v == 0) CK(hipStreamSynchronize(s));
        else if (v == 1) CK(hipMemcpy(hv, d, 16, hipMemcpyDeviceToHost));  // legacy null stream: waits for s? no: copy on null stream
        else if (v == 2) { CK(hipMemcpyAsync(hp, d, 16, hipMemcpyDeviceToHost, s)); CK(hipEventRecord(ev, s)); while (hipEventQuery(ev) == hipErrorNotReady) {} }
        else if (v == 3) { CK(hipEventRecord(ev, s)); CK(hipEventSynchronize(ev)); }
        else { CK(hipMemcpyAsync(hp, d, 16, hipMemcpyDeviceToHost, s)); CK(hipStreamSynchronize(s)); }
      }
      if (v == 1) CK(hipStreamSynchronize(s));
      auto t1 = std::chrono::steady_clock::now();
      if (w == 1) {
        const char* nm[] = {"kernel+StreamSynchronize", "kernel+hipMemcpy D2H (sync)", "kernel+async D2H pinned+event spin",
                            "kernel+EventSynchronize", "kernel+async D2H pinned+StreamSynchronize"};
        printf("%-44s %8.2f us\n", nm[v], std::chrono::duration<double, std::micro>(t1 - t0).count() / N);
      }
    }
  }
  return 0;
}
