// Probe of global_load_lds_dword on gfx950 (calibration for the GEMM's DMA staging):
//  1. semantics: does the instruction offset move the LDS destination as well as the
//     global source?  (LDS slot written by lane l of an instruction with offset 1024)
//  2. issue cost: cycles per DMA instruction for (a) M0 save/set/restore around every
//     instruction, (b) one M0 per batch of 4 with the LDS step carried by the offset.
//   hipcc -O3 --offload-arch=gfx950 tools/glds_probe.hip -o build/glds_probe && build/glds_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void semantics(const float* src, float* out) {
  __shared__ float s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = -1.f;
  __syncthreads();
  const uint32_t lds = (uint32_t)reinterpret_cast<uintptr_t>(&s[0]);
  const uint32_t voff = threadIdx.x * 4;
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2 offset:1024\n\t"
      "s_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
      : "=&s"(keep)
      : "v"(voff), "s"(src), "s"(lds)
      : "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 64) out[i] = s[i];
}

template <int MODE>
__global__ void cost(const float* src, unsigned long long* cyc, int iters) {
  __shared__ float s[4][4096];
  const uint32_t lds = (uint32_t)reinterpret_cast<uintptr_t>(&s[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)][0]);
  const uint32_t v = (threadIdx.x & 63) * 4;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    uint32_t keep;
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(v + 256 * j), "s"(src), "s"(lds + 1024 * j)
            : "memory");
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
            "global_load_lds_dword %1, %2\n\t"
            "global_load_lds_dword %1, %2 offset:1024\n\t"
            "global_load_lds_dword %1, %2 offset:2048\n\t"
            "global_load_lds_dword %1, %2 offset:3072\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(v + 4096 * b), "s"(src), "s"(lds + 4096 * b)
            : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  float *src, *out;
  unsigned long long* cyc;
  hipMalloc(&src, 1 << 20);
  hipMalloc(&out, 4096);
  hipMalloc(&cyc, 256 * 4 * 8);
  std::vector<float> h(1 << 18);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)i;
  hipMemcpy(src, h.data(), 1 << 20, hipMemcpyHostToDevice);
  semantics<<<1, 64>>>(src, out);
  std::vector<float> o(1024);
  hipMemcpy(o.data(), out, 4096, hipMemcpyDeviceToHost);
  int first = -1;
  for (int i = 0; i < 1024; ++i)
    if (o[i] != -1.f) { first = i; break; }
  printf("semantics: first written LDS slot %d (value %.0f = src element), slot 256 holds %.0f\n", first,
         first >= 0 ? o[first] : -1.f, o[256]);
  const int iters = 2000;
  for (int mode = 0; mode < 2; ++mode) {
    if (mode == 0) cost<0><<<256, 256>>>(src, cyc, iters);
    else cost<1><<<256, 256>>>(src, cyc, iters);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(1024);
    hipMemcpy(c.data(), cyc, 1024 * 8, hipMemcpyDeviceToHost);
    double m = 0;
    for (auto x : c) m += (double)x;
    m /= 1024;
    printf("mode %d (%s): %.1f cycles per 16-DMA batch + vmcnt(0), %.1f per DMA\n", mode,
           mode == 0 ? "M0 per instruction" : "M0 per 4, offset steps", m / iters, m / iters / 16);
  }
  return 0;
}
