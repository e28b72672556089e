// optim.hip — the training driver's optimiser step on the GPU (gfx950): torch.optim.Adam
// (train_DSTAGNN_my.py:126, `optim.Adam(net.parameters(), lr=learning_rate)`, default betas /
// eps, no weight decay) over every parameter tensor of the model in ONE launch.
//
// torch's fused multi-tensor Adam splits a model's ~150 tensors over four launches of ~43 us
// each at PEMS08 (nb_block = 4: 2.6 M parameters, ~70 MB moved — ~10 us of HBM time), and
// its Python-side grouping leaves the GPU idle for ~0.2 ms before them
// (profiles/r04_model_step_*.txt).  Here the host hands over a table of (param, grad,
// exp_avg, exp_avg_sq, n) segments plus a chunk table ((segment, offset) per 4096 elements);
// a workgroup updates one chunk: every load of its 16 elements per thread first, then the
// update, then the stores.  Per element the arithmetic of torch's fused Adam
// (ATen/native/cuda/fused_adam_utils.cuh, ADAM_MODE::ORIGINAL) in fp32:
//   m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g g;
//   p -= step_size * m / (sqrt(v) / sqrt(1 - b2^t) + eps),  step_size = lr / (1 - b1^t)
#include "common.hpp"

namespace {

constexpr int kAdamThreads = 256, kAdamPer = 16, kAdamChunk = kAdamThreads * kAdamPer;

__global__ __launch_bounds__(kAdamThreads) void adam_kernel(const dstagnn_adam_seg* __restrict__ segs,
                                                            const int64_t* __restrict__ chunks, float b1, float b2,
                                                            float eps, float step_size, float bc2_sqrt) {
  const int64_t si = chunks[2 * (int64_t)blockIdx.x], off = chunks[2 * (int64_t)blockIdx.x + 1];
  const dstagnn_adam_seg s = segs[si];
  const int64_t end = min(off + (int64_t)kAdamChunk, s.n);
  float* __restrict__ p = s.p;
  const float* __restrict__ g = s.g;
  float* __restrict__ m = s.m;
  float* __restrict__ v = s.v;
  float gv[kAdamPer], mv[kAdamPer], vv[kAdamPer], pv[kAdamPer];
#pragma unroll
  for (int u = 0; u < kAdamPer; ++u) {
    const int64_t i = off + threadIdx.x + (int64_t)kAdamThreads * u;
    const bool ok = i < end;
    gv[u] = ok ? g[i] : 0.f;
    mv[u] = ok ? m[i] : 0.f;
    vv[u] = ok ? v[i] : 0.f;
    pv[u] = ok ? p[i] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < kAdamPer; ++u) {
    const int64_t i = off + threadIdx.x + (int64_t)kAdamThreads * u;
    if (i >= end) continue;
    const float mm = b1 * mv[u] + (1.f - b1) * gv[u];
    const float vw = b2 * vv[u] + (1.f - b2) * gv[u] * gv[u];
    const float denom = sqrtf(vw) / bc2_sqrt + eps;
    m[i] = mm;
    v[i] = vw;
    p[i] = pv[u] - step_size * mm / denom;
  }
}

}  // namespace

int dstagnn_adam_chunk_elems(void) { return kAdamChunk; }

int dstagnn_adam_step(const dstagnn_adam_seg* segs, const int64_t* chunks, int nchunk, float beta1,
                        float beta2, float eps, float step_size, float bc2_sqrt, dstagnn_stream_t stream) {
  if (nchunk < 0 || (nchunk > 0 && (!segs || !chunks))) {
    set_last_error("adam_step: null segment / chunk table");
    return DSTAGNN_E_ARG;
  }
  if (nchunk == 0) return 0;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)nchunk), dim3(kAdamThreads), 0, (hipStream_t)stream, segs, chunks,
                     beta1, beta2, eps, step_size, bc2_sqrt);
  DS_CHECK_LAUNCH();
  return 0;
}
