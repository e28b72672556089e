// flag_sync_probe.hip — is hipStreamWriteValue32 on the producer stream + hipStreamWaitValue32
// on the consumer stream a correct cross-stream dependency for kernel data (gfx950, ROCm 7.2)?
// Producer kernel (all XCDs) computes ~20 us, then writes X[i] = tag; the flag write follows
// on its stream; the consumer stream waits for flag >= tag and its kernel checks every X[i]
// (all XCDs) and counts mismatches.  Both directions, 300 rounds each, and the same with the
// event pair for reference.  Prints the mismatch counts (must be 0) and the wall time.
// argv[1] = s: the flag words in hipMallocSignalMemory (else hipMalloc).
// Modes 4 / 5: the flag is written by the NEXT kernel on the producer stream (workgroup 0,
// thread 0, at its start: a system-scope release store) instead of a hipStreamWriteValue32 —
// the block's kernel-prologue signal (block.hip Streams::fork) — the producer's data being
// complete once any later kernel of its stream runs.
//   hipcc -O3 --offload-arch=gfx950 tools/flag_sync_probe.hip -o tools/flag_sync_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

constexpr int kN = 1 << 20;

__global__ void produce(float* x, int iters, float tag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float v = (float)(i & 7);
  for (int k = 0; k < iters; ++k) v = v * 0.999f + 0.001f;
  x[i] = v == 12345.f ? v : tag;
}
__global__ void signal_then_work(unsigned* flag, unsigned v, float* z, int iters) {
  if (blockIdx.x == 0 && threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float w = (float)(i & 3);
  for (int k = 0; k < iters; ++k) w = w * 0.999f + 0.001f;
  z[i] = w;
}
__global__ void consume(const float* x, float tag, unsigned* err, float* y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const float v = x[i];
  if (v != tag) atomicAdd(err, 1u);
  y[i] = v;
}

int main(int argc, char** argv) {
  const bool sig = argc > 1 && argv[1][0] == 's';  // flags in hipMallocSignalMemory
  float *x, *y, *z;
  unsigned* err;
  uint32_t* flag;
  (void)hipMalloc(&x, kN * 4);
  (void)hipMalloc(&y, kN * 4);
  (void)hipMalloc(&z, kN * 4);
  (void)hipMalloc(&err, 64);
  if (sig) (void)hipExtMallocWithFlags((void**)&flag, 4096, hipMallocSignalMemory);
  else (void)hipMalloc(&flag, 4096);
  (void)hipMemset(x, 0, kN * 4);
  (void)hipMemset(err, 0, 64);
  (void)hipMemset(flag, 0, 4096);
  hipStream_t a, b;
  int lo, hi;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
  (void)hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
  (void)hipStreamCreateWithPriority(&b, hipStreamNonBlocking, lo);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  (void)hipDeviceSynchronize();
  uint32_t seq = 0;
  // 0: flags a->b, 1: flags b->a, 2: events a->b, 3: events b->a, 4 / 5: kernel-written flags a->b / b->a
  for (int mode = 0; mode < 6; ++mode) {
    hipStream_t p = (mode & 1) ? b : a, c = (mode & 1) ? a : b;
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 300; ++r) {
      const float tag = (float)(mode * 1000 + r + 1);
      hipLaunchKernelGGL(produce, dim3(kN / 256), dim3(256), 0, p, x, 8000, tag);
      if (mode >= 4) {
        ++seq;
        (void)hipStreamWaitValue32(c, flag, seq, hipStreamWaitValueGte, 0xffffffffu);
        hipLaunchKernelGGL(signal_then_work, dim3(kN / 256), dim3(256), 0, p, flag, seq, z, 2000);
      } else if (mode < 2) {
        ++seq;
        (void)hipStreamWriteValue32(p, flag, seq, 0);
        (void)hipStreamWaitValue32(c, flag, seq, hipStreamWaitValueGte, 0xffffffffu);
      } else {
        (void)hipEventRecord(ev, p);
        (void)hipStreamWaitEvent(c, ev, 0);
      }
      hipLaunchKernelGGL(consume, dim3(kN / 256), dim3(256), 0, c, x, tag, err + mode, y);
      // the next round's producer must not overwrite x before this consumer read it
      if (mode < 2 || mode >= 4) {
        ++seq;
        (void)hipStreamWriteValue32(c, flag + 32, seq, 0);
        (void)hipStreamWaitValue32(p, flag + 32, seq, hipStreamWaitValueGte, 0xffffffffu);
      } else {
        (void)hipEventRecord(ev, c);
        (void)hipStreamWaitEvent(p, ev, 0);
      }
    }
    (void)hipDeviceSynchronize();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    unsigned h[6];
    (void)hipMemcpy(h, err, 24, hipMemcpyDeviceToHost);
    printf("%s mode %d (%s %s): mismatches %u, %.3f ms per round\n", sig ? "signal-mem" : "device-mem", mode, mode < 2 ? "flags" : (mode < 4 ? "events" : "kernel-flags"),
           (mode & 1) ? "side->main" : "main->side", h[mode], ms / 300);
  }
  return 0;
}
