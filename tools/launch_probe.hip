// launch_probe.hip — host cost of one kernel launch on this ROCm stack: an empty kernel with
// a small and with a 2 KB argument struct (the GEMM descriptor size), hipLaunchKernelGGL vs
// hipExtLaunchKernel, plus hipEventRecord / hipStreamWaitEvent pairs.  Host-side timing only.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

struct Small { int a[4]; };
struct Big { int a[512]; };
__global__ void k_small(Small s) { if (s.a[0] == 12345) asm volatile("s_nop 0"); }
__global__ void k_big(Big s) { if (s.a[0] == 12345) asm volatile("s_nop 0"); }

template <typename F>
double per_call_us(F f, int n) {
  for (int i = 0; i < 200; ++i) f();
  (void)hipDeviceSynchronize();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  (void)hipDeviceSynchronize();
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
  hipStream_t st, sd;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&sd, hipStreamNonBlocking);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  Small s{};
  Big b{};
  const int n = 2000;
  printf("launch small args   %.2f us\n", per_call_us([&] { hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, st, s); }, n));
  printf("launch 2KB args     %.2f us\n", per_call_us([&] { hipLaunchKernelGGL(k_big, dim3(256), dim3(256), 0, st, b); }, n));
  printf("ext launch small    %.2f us\n", per_call_us([&] {
    void* args[] = {&s};
    (void)hipExtLaunchKernel((const void*)k_small, dim3(256), dim3(256), args, 0, st, nullptr, nullptr, 0);
  }, n));
  printf("event record+wait   %.2f us\n", per_call_us([&] {
    (void)hipEventRecord(ev, st);
    (void)hipStreamWaitEvent(sd, ev, 0);
  }, n));
  printf("launch alt streams  %.2f us\n", per_call_us([&] {
    hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, st, s);
    hipLaunchKernelGGL(k_small, dim3(256), dim3(256), 0, sd, s);
  }, n / 2) / 2);
  float* p;
  (void)hipMalloc(&p, 1 << 20);
  printf("memsetAsync 1MB     %.2f us\n", per_call_us([&] { (void)hipMemsetAsync(p, 0, 1 << 20, st); }, n));
  printf("getLastError        %.3f us\n", per_call_us([&] { (void)hipGetLastError(); }, n));
  int dev;
  printf("getDevice           %.3f us\n", per_call_us([&] { (void)hipGetDevice(&dev); }, n));
  return 0;
}
