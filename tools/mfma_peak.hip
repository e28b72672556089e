// Achievable fp32-MFMA rate on this part (v_mfma_f32_32x32x2_f32), as a calibration for
// the GEMM roofline: NACC independent accumulators per wave, WPB waves per workgroup.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_peak.hip -o build/mfma_peak && build/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ void mfma_loop(float* out, int iters, float a, float b) {
  floatx16 acc[NACC];
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  float av = a + threadIdx.x * 1e-7f, bv = b;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i], 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  if (s == 12345.f) out[threadIdx.x] = s;
}

template <int NACC>
void run(int blocks, int threads, int iters) {
  float* d;
  hipMalloc(&d, 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  mfma_loop<NACC><<<blocks, threads>>>(d, iters, 1.f, 1.f);
  hipEventRecord(e0);
  mfma_loop<NACC><<<blocks, threads>>>(d, iters, 1.f, 1.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)blocks * (threads / 64) * iters * NACC * 32.0 * 32 * 2 * 2;
  printf("NACC=%d blocks=%d threads=%d: %.3f ms, %.1f TFLOP/s\n", NACC, blocks, threads, ms, flops / ms / 1e9);
  hipFree(d);
}

int main() {
  run<1>(256, 256, 20000);
  run<1>(768, 256, 20000);
  run<2>(256, 256, 20000);
  run<4>(256, 256, 20000);
  run<4>(512, 256, 20000);
  run<4>(1024, 256, 20000);
  return 0;
}
