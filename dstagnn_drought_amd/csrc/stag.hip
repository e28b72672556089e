// stag.hip — the two graph builders of the reference on gfx950.
//
//  STAG_gen (data/STAG_gen.py:17-59): exact EMD per node pair.
//    stag_prep_kernel   per node: unit rows xhat_t = x_t / |x_t| (zero rows -> 1e-12 guard, so
//                       xhat = 0) and marginals p_t = |x_t| / (sum |x| + 1e-12)   (:47-54)
//    stag_emd_kernel    one wave per pair: network simplex (emd_simplex.hpp) with the whole
//                       workspace in LDS, costs recomputed from xhat (:56-58); the reference's
//                       1.0 failure value when HiGHS would call the LP infeasible (:37).
//    emd_dense_kernel   same solver on caller-given dense costs = wasserstein_distance(p,q,D).
//  fast_STAG_gen (data/fast_STAG_gen.py:16-35, 55-74):
//    fast_stag_dist_kernel  windowed cosine distance, symmetric, zero diagonal, fp64
//    topk_rows_kernel       per row the k smallest keys (ties: lower index), bitonic sort of
//                           (key, index) in LDS -> A (0/1), R, neighbour list
#include <cstring>

#include "common.hpp"
#include "emd_simplex.hpp"

namespace {

constexpr int kPrepThreads = 256;
constexpr int kLdsMax = 160 * 1024;

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

struct WaveMin {
  __device__ emd::Cand operator()(emd::Cand c) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double orc = __shfl_xor(c.rc, o, 64);
      const int ooff = __shfl_xor(c.off, o, 64);
      const bool take = ooff >= 0 && (c.off < 0 || orc < c.rc || (orc == c.rc && ooff < c.off));
      if (take) { c.rc = orc; c.off = ooff; }
    }
    return c;
  }
};

struct WaveSync {
  __device__ void operator()() const { __syncthreads(); }
};

// block reduction over kPrepThreads threads (double)
__device__ double block_sum(double v, double* red) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kPrepThreads / 64; ++i) s += red[i];
  return s;
}

// data (T, N, F) -> xhat (N, T, F), p (N, T), psum (N)
__global__ __launch_bounds__(kPrepThreads) void stag_prep_kernel(const double* __restrict__ data, int T, int N, int F,
                                                                 double* __restrict__ xhat, double* __restrict__ p,
                                                                 double* __restrict__ psum) {
  __shared__ double red[kPrepThreads / 64];
  const int n = blockIdx.x;
  double part = 0.0;
  for (int t = threadIdx.x; t < T; t += kPrepThreads) {
    const double* x = data + ((int64_t)t * N + n) * F;
    double s = 0.0;
    for (int f = 0; f < F; ++f) s += x[f] * x[f];
    double nr = sqrt(s);
    if (nr == 0.0) nr = 1e-12;
    part += nr;
    double* xh = xhat + ((int64_t)n * T + t) * F;
    for (int f = 0; f < F; ++f) xh[f] = x[f] / nr;
    p[(int64_t)n * T + t] = nr;   // norms for now
  }
  const double S = block_sum(part, red) + 1e-12;
  double ps = 0.0;
  for (int t = threadIdx.x; t < T; t += kPrepThreads) {
    const double v = p[(int64_t)n * T + t] / S;
    p[(int64_t)n * T + t] = v;
    ps += v;
  }
  const double tot = block_sum(ps, red);
  if (threadIdx.x == 0) psum[n] = tot;
}

// one wave per pair (grid-stride over pairs); dynamic LDS = emd::work_bytes(T, GX ? 0 : F).
// GX: the pair's unit rows stay in global memory (read through L1 / L2 by the pricing scan; a
// node's rows serve all N - 1 of its pairs) instead of an LDS copy — at the GAMBIA shape the copy
// is 18 of the 39 KB of a pair's workspace, so LDS admits 4 pairs per CU with it and 7 without:
// the solver's serial tree walks are LDS-latency chains of one wave, so more resident pairs
// per CU is the throughput lever (tools/bench_stag.py).
template <bool GX>
__global__ __launch_bounds__(64) void stag_emd_kernel(const double* __restrict__ xhat, const double* __restrict__ p,
                                                      const double* __restrict__ psum, int T, int F,
                                                      const int32_t* __restrict__ pairs, int64_t P,
                                                      double* __restrict__ out, int32_t* __restrict__ status,
                                                      int64_t* __restrict__ pivots) {
  extern __shared__ double smem[];
  const int lane = threadIdx.x;
  emd::Work w;
  emd::carve(w, (char*)smem, T, GX ? 0 : F);
  w.F = F;
  for (int64_t k = blockIdx.x; k < P; k += gridDim.x) {
    const int i = pairs[2 * k], j = pairs[2 * k + 1];
    if (!emd::balanced(psum[i], psum[j])) {
      if (lane == 0) { out[k] = 1.0; status[k] = 1; if (pivots) pivots[k] = 0; }
      continue;
    }
    const int64_t tf = (int64_t)T * F;
    if (GX) {
      w.xh = xhat + (int64_t)i * tf;
      w.yh = xhat + (int64_t)j * tf;
    } else {
      for (int64_t e = lane; e < tf; e += 64) {
        ((double*)w.xh)[e] = xhat[(int64_t)i * tf + e];
        ((double*)w.yh)[e] = xhat[(int64_t)j * tf + e];
      }
    }
    for (int t = lane; t < T; t += 64) {
      ((double*)w.p)[t] = p[(int64_t)i * T + t];
      ((double*)w.q)[t] = p[(int64_t)j * T + t];
    }
    __syncthreads();
    int st = 0;
    int64_t piv = 0;
    double obj = emd::solve<64>(w, lane, WaveMin(), WaveSync(), 1.0, &st, &piv);
    obj = wave_sum_d(obj);
    if (lane == 0) { out[k] = obj; status[k] = st; if (pivots) pivots[k] = piv; }
    __syncthreads();
  }
}

// batched wasserstein_distance(p, q, D): p, q (B, T), D (B, T, T)
__global__ __launch_bounds__(64) void emd_dense_kernel(const double* __restrict__ p, const double* __restrict__ q,
                                                       const double* __restrict__ D, int T, int64_t B,
                                                       double* __restrict__ out, int32_t* __restrict__ status) {
  extern __shared__ double smem[];
  const int lane = threadIdx.x;
  emd::Work w;
  emd::carve(w, (char*)smem, T, 0);
  for (int64_t k = blockIdx.x; k < B; k += gridDim.x) {
    double sp = 0.0, sq = 0.0, neg = 0.0;
    for (int t = lane; t < T; t += 64) {
      const double a = p[k * T + t], b = q[k * T + t];
      ((double*)w.p)[t] = a;
      ((double*)w.q)[t] = b;
      sp += a; sq += b;
      if (a < 0.0 || b < 0.0) neg = 1.0;
    }
    sp = wave_sum_d(sp); sq = wave_sum_d(sq); neg = wave_max_d(neg);
    if (neg > 0.0 || !emd::balanced(sp, sq)) {
      if (lane == 0) { out[k] = 1.0; status[k] = 1; }
      continue;
    }
    w.Dm = D + k * (int64_t)T * T;
    double cm = 0.0;
    for (int64_t e = lane; e < (int64_t)T * T; e += 64) cm = fmax(cm, fabs(emd::clean_cost(w.Dm[e])));
    cm = wave_max_d(cm);
    __syncthreads();
    int st = 0;
    int64_t piv = 0;
    double obj = emd::solve<64>(w, lane, WaveMin(), WaveSync(), cm, &st, &piv);
    obj = wave_sum_d(obj);
    if (lane == 0) { out[k] = obj; status[k] = st; }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// fast_STAG_gen
// ---------------------------------------------------------------------------------------
constexpr int kDistThreads = 256;

// sta[i][j] = 1 - x_i.x_j / ((|x_i| + 1e-12)(|x_j| + 1e-12)) if |c_i - c_j| <= maxd, i != j
__global__ __launch_bounds__(kDistThreads) void fast_stag_dist_kernel(const double* __restrict__ coords, int N, int Dc,
                                                                      const double* __restrict__ feats, int Fp,
                                                                      double maxd, double* __restrict__ sta) {
  const int i = blockIdx.y;
  const int j = blockIdx.x * kDistThreads + threadIdx.x;
  if (j >= N) return;
  double v = 0.0;
  if (j != i) {
    double d2 = 0.0;
    for (int c = 0; c < Dc; ++c) {
      const double d = coords[(int64_t)i * Dc + c] - coords[(int64_t)j * Dc + c];
      d2 += d * d;
    }
    if (sqrt(d2) <= maxd) {
      const double* x = feats + (int64_t)i * Fp;
      const double* y = feats + (int64_t)j * Fp;
      double sx = 0.0, sy = 0.0, dot = 0.0;
      for (int f = 0; f < Fp; ++f) {
        sx += x[f] * x[f];
        sy += y[f] * y[f];
        dot += x[f] * y[f];
      }
      const double nx = sqrt(sx) + 1e-12, ny = sqrt(sy) + 1e-12;
      v = 1.0 - dot / (nx * ny);
    }
  }
  sta[(int64_t)i * N + j] = v;
}

// total order of doubles as unsigned keys (numpy sort order: -0 == +0, nan last)
__device__ __forceinline__ uint64_t order_key(double v) {
  if (v != v) return ~0ull;
  if (v == 0.0) v = 0.0;
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

constexpr int kTopkThreads = 1024;

// mode 0 (fast_STAG_gen :71-74):  key = sta, R = 1 - sta
// mode 1 (STAG_gen :105-116):     key = adj = 1 - sta + I, R = adj
__global__ __launch_bounds__(kTopkThreads) void topk_rows_kernel(const double* __restrict__ sta, int N, int k,
                                                                 int mode, int npow, double* __restrict__ A,
                                                                 double* __restrict__ R, int32_t* __restrict__ nbr) {
  extern __shared__ uint64_t keys[];
  uint32_t* idx = (uint32_t*)(keys + npow);
  uint8_t* sel = (uint8_t*)(idx + npow);
  const int i = blockIdx.x;
  const double* row = sta + (int64_t)i * N;
  for (int j = threadIdx.x; j < npow; j += kTopkThreads) {
    if (j < N) {
      double v = row[j];
      if (mode == 1) v = 1.0 - v + (j == i ? 1.0 : 0.0);
      keys[j] = order_key(v);
      idx[j] = (uint32_t)j;
      sel[j] = 0;
    } else {
      keys[j] = ~0ull;
      idx[j] = 0xffffffffu;
    }
  }
  __syncthreads();
  // bitonic sort ascending by (key, idx)
  for (int size = 2; size <= npow; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < npow / 2; t += kTopkThreads) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t ka = keys[lo], kb = keys[hi];
        const uint32_t ia = idx[lo], ib = idx[hi];
        const bool gt = ka > kb || (ka == kb && ia > ib);
        if (gt == up) { keys[lo] = kb; keys[hi] = ka; idx[lo] = ib; idx[hi] = ia; }
      }
      __syncthreads();
    }
  }
  for (int r = threadIdx.x; r < k; r += kTopkThreads) {
    sel[idx[r]] = 1;
    if (nbr) nbr[(int64_t)i * k + r] = (int32_t)idx[r];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < N; j += kTopkThreads) {
    const double s = row[j];
    const double key = mode == 1 ? 1.0 - s + (j == i ? 1.0 : 0.0) : s;
    const bool on = sel[j] != 0;
    A[(int64_t)i * N + j] = on ? 1.0 : 0.0;
    R[(int64_t)i * N + j] = on ? (mode == 1 ? key : 1.0 - s) : 0.0;
  }
}

int set_lds(const void* fn, int64_t lds) {
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) { set_last_error(std::string("LDS attribute: ") + hipGetErrorString(e)); return (int)e; }
  }
  return 0;
}

int emd_grid(int64_t P, int64_t lds) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
  const int per_cu = (int)std::max<int64_t>(1, std::min<int64_t>(8, kLdsMax / std::max<int64_t>(lds, 1)));
  return (int)std::max<int64_t>(1, std::min<int64_t>(P, (int64_t)cus * per_cu));
}

}  // namespace

extern "C" {

int64_t dstagnn_stag_emd_lds_bytes(int T, int F) { return emd::work_bytes(T, F); }

int dstagnn_stag_prep(const double* data, int T, int N, int F, double* xhat, double* p, double* psum,
                      dstagnn_stream_t stream) {
  if (!data || !xhat || !p || !psum) { set_last_error("stag_prep: null argument"); return DSTAGNN_E_ARG; }
  if (T <= 0 || N <= 0 || F <= 0) { set_last_error("stag_prep: non-positive dimension"); return DSTAGNN_E_SHAPE; }
  hipLaunchKernelGGL(stag_prep_kernel, dim3(N), dim3(kPrepThreads), 0, (hipStream_t)stream, data, T, N, F, xhat, p,
                     psum);
  DS_CHECK_LAUNCH();
  return 0;
}

int dstagnn_stag_emd_pairs(const double* xhat, const double* p, const double* psum, int T, int N, int F,
                           const int32_t* pairs, int64_t P, double* out, int32_t* status, int64_t* pivots,
                           dstagnn_stream_t stream) {
  if (!xhat || !p || !psum || !pairs || !out || !status) { set_last_error("stag_emd: null argument"); return DSTAGNN_E_ARG; }
  if (T <= 0 || N <= 0 || F <= 0 || P < 0) { set_last_error("stag_emd: bad dimension"); return DSTAGNN_E_SHAPE; }
  if (2 * (int64_t)T + 1 > 32767) { set_last_error("stag_emd: T too large (node ids are int16)"); return DSTAGNN_E_SHAPE; }
  // DSTAGNN_STAG_XH=lds keeps the unit rows in LDS (the round-1 layout); default: global
  static const bool gx = !getenv("DSTAGNN_STAG_XH") || strcmp(getenv("DSTAGNN_STAG_XH"), "lds") != 0;
  const int64_t lds = emd::work_bytes(T, gx ? 0 : F);
  if (lds > kLdsMax) { set_last_error("stag_emd: T*F too large for LDS"); return DSTAGNN_E_SHAPE; }
  if (P == 0) return 0;
  const void* kern = gx ? (const void*)stag_emd_kernel<true> : (const void*)stag_emd_kernel<false>;
  if (int rc = set_lds(kern, lds)) return rc;
  if (gx)
    hipLaunchKernelGGL(stag_emd_kernel<true>, dim3(emd_grid(P, lds)), dim3(64), lds, (hipStream_t)stream, xhat, p, psum,
                       T, F, pairs, P, out, status, pivots);
  else
    hipLaunchKernelGGL(stag_emd_kernel<false>, dim3(emd_grid(P, lds)), dim3(64), lds, (hipStream_t)stream, xhat, p,
                       psum, T, F, pairs, P, out, status, pivots);
  DS_CHECK_LAUNCH();
  return 0;
}

int dstagnn_emd_dense(const double* p, const double* q, const double* D, int T, int64_t B, double* out,
                      int32_t* status, dstagnn_stream_t stream) {
  if (!p || !q || !D || !out || !status) { set_last_error("emd_dense: null argument"); return DSTAGNN_E_ARG; }
  if (T <= 0 || B < 0) { set_last_error("emd_dense: bad dimension"); return DSTAGNN_E_SHAPE; }
  if (2 * (int64_t)T + 1 > 32767) { set_last_error("emd_dense: T too large (node ids are int16)"); return DSTAGNN_E_SHAPE; }
  const int64_t lds = emd::work_bytes(T, 0);
  if (lds > kLdsMax) { set_last_error("emd_dense: T too large for LDS"); return DSTAGNN_E_SHAPE; }
  if (B == 0) return 0;
  if (int rc = set_lds((const void*)emd_dense_kernel, lds)) return rc;
  hipLaunchKernelGGL(emd_dense_kernel, dim3(emd_grid(B, lds)), dim3(64), lds, (hipStream_t)stream, p, q, D, T, B, out,
                     status);
  DS_CHECK_LAUNCH();
  return 0;
}

int dstagnn_fast_stag_distances(const double* coords, int N, int Dc, const double* feats, int Fp, double max_distance,
                                double* sta, dstagnn_stream_t stream) {
  if (!coords || !feats || !sta) { set_last_error("fast_stag: null argument"); return DSTAGNN_E_ARG; }
  if (N <= 0 || Dc <= 0 || Fp <= 0) { set_last_error("fast_stag: non-positive dimension"); return DSTAGNN_E_SHAPE; }
  if (N > 65535) { set_last_error("fast_stag: N > 65535"); return DSTAGNN_E_SHAPE; }
  dim3 grid((N + kDistThreads - 1) / kDistThreads, N);
  hipLaunchKernelGGL(fast_stag_dist_kernel, grid, dim3(kDistThreads), 0, (hipStream_t)stream, coords, N, Dc, feats, Fp,
                     max_distance, sta);
  DS_CHECK_LAUNCH();
  return 0;
}

int dstagnn_graph_topk(const double* sta, int N, int k, int mode, double* A, double* R, int32_t* nbr,
                       dstagnn_stream_t stream) {
  if (!sta || !A || !R) { set_last_error("graph_topk: null argument"); return DSTAGNN_E_ARG; }
  if (N <= 0 || k <= 0 || k > N || (mode != 0 && mode != 1)) { set_last_error("graph_topk: bad argument"); return DSTAGNN_E_SHAPE; }
  int npow = 1;
  while (npow < N) npow <<= 1;
  const int64_t lds = (int64_t)npow * (8 + 4 + 1);
  if (lds > kLdsMax) { set_last_error("graph_topk: N too large for the in-LDS row sort (N <= 8192)"); return DSTAGNN_E_SHAPE; }
  if (int rc = set_lds((const void*)topk_rows_kernel, lds)) return rc;
  hipLaunchKernelGGL(topk_rows_kernel, dim3(N), dim3(kTopkThreads), lds, (hipStream_t)stream, sta, N, k, mode, npow, A,
                     R, nbr);
  DS_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
