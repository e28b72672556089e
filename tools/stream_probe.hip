// Host cost of launches on one stream vs alternating streams, and of event fork/join.
//   hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o build/stream_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty(float* p) {
  if (threadIdx.x == 0 && p[0] == 12345.f) p[1] = 1.f;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  float* d;
  hipMalloc(&d, 1024);
  hipMemset(d, 0, 1024);
  hipStream_t a, b;
  hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
  int lo, hi;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  hipStreamCreateWithPriority(&b, hipStreamNonBlocking, lo);
  hipEvent_t ev[64];
  for (auto& e : ev) hipEventCreateWithFlags(&e, hipEventDisableTiming);
  const int n = 2000;
  for (int rep = 0; rep < 2; ++rep) {
    hipDeviceSynchronize();
    double t0 = now_us();
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, a, d);
    double t1 = now_us();
    hipDeviceSynchronize();
    double t2 = now_us();
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, (i & 1) ? b : a, d);
    double t3 = now_us();
    hipDeviceSynchronize();
    double t4 = now_us();
    for (int i = 0; i < n; ++i) {
      hipEventRecord(ev[i & 63], a);
      hipStreamWaitEvent(b, ev[i & 63], 0);
    }
    double t5 = now_us();
    hipDeviceSynchronize();
    double t6 = now_us();
    for (int i = 0; i < n; ++i) {
      hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, a, d);
      hipEventRecord(ev[i & 63], a);
      hipStreamWaitEvent(b, ev[i & 63], 0);
      hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, b, d);
    }
    double t7 = now_us();
    hipDeviceSynchronize();
    double t8 = now_us();
    printf("rep %d: launch same stream %.2f us | alternating streams %.2f us | record+wait %.2f us | "
           "launch,fork,launch %.2f us per iter; gpu drain same-stream %.1f us/launch\n",
           rep, (t1 - t0) / n, (t3 - t2) / n, (t5 - t4) / n, (t7 - t6) / n, (t2 - t0) / n);
    (void)t8;
  }
  return 0;
}
