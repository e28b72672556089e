// fork_probe.hip — device-side cost of cross-stream synchronisation on gfx950 / ROCm 7.2:
// the idle gap the main stream shows between two back-to-back kernels when, between them,
//   0: nothing             1: hipEventRecord (disable-timing) on main (a fork's producer side)
//   2: main waits an event recorded long ago on the side (a join that is already satisfied)
//   3: hipStreamWriteValue32 on main      4: hipStreamWaitValue32 on main (already satisfied)
// Each pattern runs 200 times; the gaps come from rocprofv3 --kernel-trace (tools/fork_probe.py).
//   hipcc -O3 --offload-arch=gfx950 tools/fork_probe.hip -o tools/fork_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_busy(float* p, int iters, int tag) {
  float v = p[threadIdx.x];
  for (int i = 0; i < iters; ++i) v = v * 0.999f + 0.001f;
  if (v == 12345.f) p[threadIdx.x + tag] = v;
}

int main() {
  float* d;
  (void)hipMalloc(&d, 1 << 20);
  (void)hipMemset(d, 0, 1 << 20);
  uint32_t* flag;
  (void)hipExtMallocWithFlags((void**)&flag, 4096, hipMallocSignalMemory);
  (void)hipMemset(flag, 0, 4096);
  hipStream_t a, b;
  (void)hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
  hipEvent_t ev, old;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&old, hipEventDisableTiming);
  (void)hipEventRecord(old, b);
  (void)hipDeviceSynchronize();
  const int iters = 4000;  // ~10 us per kernel
  for (int mode = 0; mode < 5; ++mode) {
    for (int r = 0; r < 200; ++r) {
      hipLaunchKernelGGL(k_busy, dim3(1024), dim3(256), 0, a, d, iters, mode * 1000 + 1);
      if (mode == 1) (void)hipEventRecord(ev, a);
      if (mode == 2) (void)hipStreamWaitEvent(a, old, 0);
      if (mode == 3) (void)hipStreamWriteValue32(a, flag, (uint32_t)r, 0);
      if (mode == 4) (void)hipStreamWaitValue32(a, flag + 16, 0, hipStreamWaitValueGte, 0xffffffffu);
      hipLaunchKernelGGL(k_busy, dim3(1024), dim3(256), 0, a, d, iters, mode * 1000 + 2);
    }
    (void)hipDeviceSynchronize();
  }
  printf("done\n");
  return 0;
}
