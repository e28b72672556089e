// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the block's kernels use
// (MI355X_MICROARCH.md: FETCH_SIZE reads exactly 1/2 of a 16-B-per-lane streaming read; other
// widths are uncalibrated).  Each kernel moves a known byte count once:
//   k0 read_x4    global_load_dwordx4, 16 B per lane      (64 MiB)
//   k1 read_x1    global_load_dword,    4 B per lane      (64 MiB)
//   k2 read_glds  global_load_lds_dword, 4 B per lane DMA  (64 MiB, the GEMM's staging)
//   k3 write_x4   global_store_dwordx4                    (64 MiB)
//   k4 write_x1   global_store_dword                      (64 MiB)
// Run:  rocprofv3 --pmc FETCH_SIZE -- tools/fetch_calib ; rocprofv3 --pmc WRITE_SIZE -- tools/fetch_calib
// and divide the known bytes by the counter (KiB) to get the per-width correction factor
// (tools/pmc_step_summary.py applies them).
//   hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t kBytes = size_t(64) << 20;

__global__ __launch_bounds__(256) void read_x4(const float4* __restrict__ src, size_t n4, float* sink) {
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 v = src[i];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  if (a.x + a.y + a.z + a.w == 12345.f) sink[0] = a.x;  // keeps the loads alive
}

__global__ __launch_bounds__(256) void read_x1(const float* __restrict__ src, size_t n, float* sink) {
  float a = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a += src[i];
  if (a == 12345.f) sink[0] = a;
}

// every wave DMAs 64 consecutive dwords (256 B) per instruction into its own LDS slot
__global__ __launch_bounds__(256) void read_glds(const float* __restrict__ src, size_t n, float* sink) {
  __shared__ float s[4][64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  const uint32_t lds = (uint32_t)reinterpret_cast<uintptr_t>(&s[w][0]);
  for (size_t base = ((size_t)blockIdx.x * 4 + w) * 64; base < n; base += (size_t)gridDim.x * 256) {
    const float* p = src + base + l;
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(p), "s"(lds)
                 : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (s[w][l] == 12345.f) sink[0] = 1.f;
}

__global__ __launch_bounds__(256) void write_x4(float4* __restrict__ dst, size_t n4) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    dst[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

__global__ __launch_bounds__(256) void write_x1(float* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = (float)i;
}

int main() {
  float *buf, *sink;
  if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&sink, 256) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, kBytes);
  const size_t n = kBytes / 4;
  const dim3 grid(2048), block(256);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(read_x4, grid, block, 0, 0, (const float4*)buf, n / 4, sink);
    hipLaunchKernelGGL(read_x1, grid, block, 0, 0, (const float*)buf, n, sink);
    hipLaunchKernelGGL(read_glds, grid, block, 0, 0, (const float*)buf, n, sink);
    hipLaunchKernelGGL(write_x4, grid, block, 0, 0, (float4*)buf, n / 4);
    hipLaunchKernelGGL(write_x1, grid, block, 0, 0, buf, n);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("fetch_calib: each kernel moved %zu bytes (%.1f KiB)\n", kBytes, kBytes / 1024.0);
  return 0;
}
