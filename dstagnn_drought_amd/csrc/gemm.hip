// gemm.hip — generic strided fp32 contraction on the CDNA4 f32 matrix cores.
//
// Every dense contraction of the DSTAGNN block (TAt / SAt projections, pre_conv,
// SAt scores, Chebyshev aggregation, GTU temporal convolutions as implicit im2col,
// and all their weight / input gradients) is one call of this kernel with a
// different set of two-level affine index maps — no permute / im2col copies in HBM.
//
// Math: v_mfma_f32_32x32x2_f32 (exact fp32 FMA chain, 64 FLOP/clk/SIMD = the fp32
// peak; gfx950 has no xf32).  A workgroup is 4 waves arranged WGM x WGN; each wave
// owns WM x WN 32x32 accumulators, so the block tile is (32*WM*WGM) x (32*WN*WGN) x 16
// (64x64, 128x64, 128x128, 128x32, 256x32 are instantiated; a cost model picks one).
// Global loads of full k-tiles are issued UNCONDITIONALLY (out-of-range rows/columns are
// clamped to a valid address; their products land only in unstored C entries): a
// predicated load makes hipcc branch and wait vmcnt(0) per element, serialising the
// k-tile prefetch.  The next k-tile is
// prefetched into registers while the MFMAs consume the current LDS buffer (2 LDS
// buffers, one barrier per k-tile).  Long reductions are split over workgroups into
// fp32 partial slabs summed by a deterministic second pass (no float atomics).
#include <cstdlib>

#include "common.hpp"

namespace {

constexpr int BKMAX = 32;  // k-tile depth (16 or 32, template parameter)

struct GemmK {
  int M, N, K, batch, splitk, kchunk;
  const float* A; Idx2 am, az; KIdx ak;
  const float* B; Idx2 bn, bz; KIdx bk;
  float* C; Idx2 cm, cn, cz;
  float alpha, beta;
  const float* bias; int64_t bias_stride;
  int relu;
  float* ws;  // split partials [batch][splitk][M][N]
};

__device__ __forceinline__ void epilogue_store(const GemmK& g, int zb, int m, int n, float v) {
  float* C = g.C + ioff(g.cz, zb);
  int64_t o = ioff(g.cm, m) + ioff(g.cn, n);
  v *= g.alpha;
  if (g.beta != 0.f) v += g.beta * C[o];
  if (g.bias) v += g.bias[(int64_t)n * g.bias_stride];
  if (g.relu) v = fmaxf(v, 0.f);
  C[o] = v;
}

// A_KC: A is contiguous along k (16 lanes read one row's k-tile).  Otherwise lanes run
// along m.  B_NC: B contiguous along n (lanes along n), otherwise lanes along k.
template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, int BK>
__device__ __forceinline__ void gemm_f32_body(const GemmK& g) {
  constexpr int BM = 32 * WM * WGM, BN = 32 * WN * WGN;
  constexpr int LA = BM * BK / 256, LB = BN * BK / 256;  // elements per thread per k-tile
  __shared__ float As[2][BK][BM + 1];
  __shared__ float Bs[2][BK][BN + 1];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WGN, wc = wid % WGN;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int zb = blockIdx.z / g.splitk, sp = blockIdx.z % g.splitk;
  const int kbeg = sp * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);

  const float* A = g.A + ioff(g.az, zb);
  const float* Bp = g.B + ioff(g.bz, zb);

  // --- per-thread element coordinates inside a tile (fixed over the k loop)
  int a_ml[LA], a_kl[LA], b_kl[LB], b_nl[LB];
#pragma unroll
  for (int j = 0; j < LA; ++j) {
    int e = tid + 256 * j;
    if (A_KC) { a_kl[j] = e % BK; a_ml[j] = e / BK; }
    else      { a_ml[j] = e % BM; a_kl[j] = e / BM; }
  }
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    int e = tid + 256 * j;
    if (B_NC) { b_nl[j] = e % BN; b_kl[j] = e / BN; }
    else      { b_kl[j] = e % BK; b_nl[j] = e / BK; }
  }
  // per-element row / column offsets as int32 from the (wave-uniform) operand bases:
  // the host guarantees every offset fits (check_span), halving the pointer registers
  int32_t ao[LA], bo[LB];
#pragma unroll
  for (int j = 0; j < LA; ++j) {
    const int m = m0 + a_ml[j];
    ao[j] = m < g.M ? (int32_t)ioff(g.am, m) : 0;  // clamped: row 0 is always valid
  }
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    const int n = n0 + b_nl[j];
    bo[j] = n < g.N ? (int32_t)ioff(g.bn, n) : 0;
  }

  float ra[LA], rb[LB];
  // Rows m >= M / columns n >= N read row/column 0 (valid memory): they only feed C
  // rows/columns the epilogue never stores, so they need no masking.  k >= kend must
  // read as 0; that happens only in the last k-tile, handled by a uniform branch so the
  // full tiles issue all their loads back to back with no per-element predicate (a
  // predicated load is sunk into an exec-masked region and waited on alone).
  auto load_tile = [&](int k0) {
    if (k0 + BK <= kend) {
#pragma unroll
      for (int j = 0; j < LA; ++j) ra[j] = A[ao[j] + koff(g.ak, k0 + a_kl[j])];
#pragma unroll
      for (int j = 0; j < LB; ++j) rb[j] = Bp[bo[j] + koff(g.bk, k0 + b_kl[j])];
    } else {
#pragma unroll
      for (int j = 0; j < LA; ++j) {
        const int k = k0 + a_kl[j];
        ra[j] = k < kend ? A[ao[j] + koff(g.ak, k)] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const int k = k0 + b_kl[j];
        rb[j] = k < kend ? Bp[bo[j] + koff(g.bk, k)] : 0.f;
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int j = 0; j < LA; ++j) As[buf][a_kl[j]][a_ml[j]] = ra[j];
#pragma unroll
    for (int j = 0; j < LB; ++j) Bs[buf][b_kl[j]][b_nl[j]] = rb[j];
  };

  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int ntiles = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (ntiles > 0) {
    load_tile(kbeg);
    store_tile(0);
    __syncthreads();
  }
  const int lr = lane & 31, lk = lane >> 5;
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
#ifndef DSTAGNN_ABLATE_LOADS
    if (t + 1 < ntiles) load_tile(kbeg + (t + 1) * BK);
#endif
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a[WM], b[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i) a[i] = As[cur][kk + lk][wr * 32 * WM + i * 32 + lr];
#pragma unroll
      for (int j = 0; j < WN; ++j) b[j] = Bs[cur][kk + lk][wc * 32 * WN + j * 32 + lr];
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
#ifdef DSTAGNN_ABLATE_MFMA
          { acc[i][j][0] += a[i] * b[j]; }
#else
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
#endif
    }
    if (t + 1 < ntiles) store_tile(cur ^ 1);
    __syncthreads();
  }

  // --- epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int n = n0 + wc * 32 * WN + j * 32 + lr;
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wr * 32 * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (m >= g.M) continue;
        if (g.splitk > 1) {
          g.ws[(((int64_t)zb * g.splitk + sp) * g.M + m) * g.N + n] = acc[i][j][r];
        } else {
          epilogue_store(g, zb, m, n, acc[i][j][r]);
        }
      }
    }
}

template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, int BK>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmK g) {
  gemm_f32_body<WGM, WGN, WM, WN, A_KC, B_NC, BK>(g);
}
// identical body under its own symbol: the call site the benchmark reports as the
// dominant kernel (rocprofv3 then lists exactly that call site's launches)
template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, int BK>
__global__ __launch_bounds__(256) void gemm_f32_hot_kernel(GemmK g) {
  gemm_f32_body<WGM, WGN, WM, WN, A_KC, B_NC, BK>(g);
}

// out[zb][m][n] = epilogue( sum_s ws[zb][s][m][n] ).  A workgroup takes 256/G outputs and
// G split groups per output (G = power of two ~ splitk/8), combined by an LDS tree.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmK g, int G) {
  __shared__ float red[256];
  const int64_t MN = (int64_t)g.M * g.N;
  const int64_t total = (int64_t)g.batch * MN;
  const int per = 256 / G;
  const int c = threadIdx.x / G, q = threadIdx.x % G;
  const int64_t idx = (int64_t)blockIdx.x * per + c;
  float s = 0.f;
  if (idx < total) {
    const int zb = (int)(idx / MN);
    const int64_t mn = idx % MN;
    const float* p = g.ws + (int64_t)zb * g.splitk * MN + mn;
    for (int sp = q; sp < g.splitk; sp += G) s += p[(int64_t)sp * MN];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = G / 2; w > 0; w >>= 1) {
    if (q < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (q == 0 && idx < total) {
    const int zb = (int)(idx / MN);
    const int64_t mn = idx % MN;
    epilogue_store(g, zb, (int)(mn / g.N), (int)(mn % g.N), red[threadIdx.x]);
  }
}

struct Cfg {
  int wgm, wgn, wm, wn;
  int bm() const { return 32 * wm * wgm; }
  int bn() const { return 32 * wn * wgn; }
};
constexpr Cfg kCfgs[] = {{2, 2, 1, 1}, {2, 2, 2, 1}, {2, 2, 2, 2}, {4, 1, 1, 1}, {4, 1, 2, 1}};

template <int WGM, int WGN, int WM, int WN, int BK>
void launch_cfg(const GemmK& k, bool akc, bool bnc, bool hot, hipStream_t st) {
  constexpr int BM = 32 * WM * WGM, BN = 32 * WN * WGN;
  dim3 grid((unsigned)cdiv64(k.M, BM), (unsigned)cdiv64(k.N, BN), (unsigned)(k.batch * k.splitk));
#define DS_GEMM_LAUNCH(KER)                                                                                  \
  if (akc && bnc) hipLaunchKernelGGL((KER<WGM, WGN, WM, WN, true, true, BK>), grid, dim3(256), 0, st, k);       \
  else if (akc)   hipLaunchKernelGGL((KER<WGM, WGN, WM, WN, true, false, BK>), grid, dim3(256), 0, st, k);      \
  else if (bnc)   hipLaunchKernelGGL((KER<WGM, WGN, WM, WN, false, true, BK>), grid, dim3(256), 0, st, k);      \
  else            hipLaunchKernelGGL((KER<WGM, WGN, WM, WN, false, false, BK>), grid, dim3(256), 0, st, k);
  if (hot) { DS_GEMM_LAUNCH(gemm_f32_hot_kernel) } else { DS_GEMM_LAUNCH(gemm_f32_kernel) }
#undef DS_GEMM_LAUNCH
}

}  // namespace

int run_gemm(const Gemm& g, float* ws, size_t ws_floats, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0 || g.batch <= 0) return 0;
  if (!g.A || !g.B || !g.C) { set_last_error("gemm: null operand"); return DSTAGNN_E_ARG; }
  GemmK k;
  k.M = g.M; k.N = g.N; k.K = g.K; k.batch = g.batch;
  k.A = g.A + g.a_off; k.am = g.am; k.az = g.az;
  k.B = g.B + g.b_off; k.bn = g.bn; k.bz = g.bz;
  if (!make_kidx(g.ak, g.K, &k.ak) || !make_kidx(g.bk, g.K, &k.bk) ||
      idx_span(g.am, g.M) + idx_span(g.ak, g.K) >= (1ll << 31) ||
      idx_span(g.bn, g.N) + idx_span(g.bk, g.K) >= (1ll << 31)) {
    set_last_error("gemm: operand offsets exceed int32 (split the batch)");
    return DSTAGNN_E_SHAPE;
  }
  k.C = g.C + g.c_off; k.cm = g.cm; k.cn = g.cn; k.cz = g.cz;
  k.alpha = g.alpha; k.beta = g.beta; k.bias = g.bias; k.bias_stride = g.bias_stride; k.relu = g.relu;
  k.ws = ws;

  // optional overrides for tuning sweeps (scripts/gemm_sweep.py)
  static const int env_cfg = getenv("DSTAGNN_GEMM_CFG") ? atoi(getenv("DSTAGNN_GEMM_CFG")) : -1;
  static const int env_bk = getenv("DSTAGNN_GEMM_BK") ? atoi(getenv("DSTAGNN_GEMM_BK")) : 0;
  static const int env_split = getenv("DSTAGNN_GEMM_SPLITK") ? atoi(getenv("DSTAGNN_GEMM_SPLITK")) : 0;
  const int BK = env_bk == 16 ? 16 : 32;
  // tile choice by a small cost model: waves of ~2 workgroups per CU, each costing its
  // MFMA area plus a per-edge load overhead
  int best = 0;
  double best_cost = 1e300;
  for (int c = 0; c < (int)(sizeof(kCfgs) / sizeof(kCfgs[0])); ++c) {
    const int bm = kCfgs[c].bm(), bn = kCfgs[c].bn();
    const int64_t blocks = cdiv64(g.M, bm) * cdiv64(g.N, bn) * g.batch;
    const double waves = (double)cdiv64(blocks, 512);
    const double cost = waves * bm * bn * (1.0 + 48.0 / bm + 48.0 / bn);
    if (cost < best_cost - 1e-9) { best_cost = cost; best = c; }
  }
  if (env_cfg >= 0 && env_cfg < (int)(sizeof(kCfgs) / sizeof(kCfgs[0]))) best = env_cfg;
  Cfg cfg = kCfgs[best];
  int64_t blocks = cdiv64(g.M, cfg.bm()) * cdiv64(g.N, cfg.bn()) * g.batch;

  // split-K when the grid leaves CUs idle and the reduction is long
  int splitk = 1;
  if (g.K > 0 && blocks < 256 && g.K >= 512 && ws) {
    int want = (int)std::min<int64_t>(512, cdiv64(512, blocks));
    int maxk = g.K / 128;  // keep >= 128 k per split
    splitk = std::max(1, std::min(want, maxk));
    if (env_split > 0) splitk = std::min(env_split, std::max(1, g.K / 64));
    while (splitk > 1 && (size_t)g.batch * splitk * g.M * g.N > ws_floats) --splitk;
  }
  int kchunk = g.K;
  if (splitk > 1) {
    kchunk = (int)cdiv64(cdiv64(g.K, splitk), BKMAX) * BKMAX;
    splitk = (int)cdiv64(g.K, kchunk);
  }
  if (g.K <= 0) { splitk = 1; kchunk = 0; }
  k.splitk = splitk; k.kchunk = kchunk;

  const bool akc = !g.ak.two && g.ak.s0 == 1;
  const bool bnc = !g.bn.two && g.bn.s0 == 1;
  const bool hot = g.hot != 0;
#define DS_CFG_SWITCH(BKV)                                          \
  switch (best) {                                                   \
    case 0: launch_cfg<2, 2, 1, 1, BKV>(k, akc, bnc, hot, st); break; \
    case 1: launch_cfg<2, 2, 2, 1, BKV>(k, akc, bnc, hot, st); break; \
    case 2: launch_cfg<2, 2, 2, 2, BKV>(k, akc, bnc, hot, st); break; \
    case 3: launch_cfg<4, 1, 1, 1, BKV>(k, akc, bnc, hot, st); break; \
    default: launch_cfg<4, 1, 2, 1, BKV>(k, akc, bnc, hot, st); break; \
  }
  if (BK == 16) { DS_CFG_SWITCH(16) } else { DS_CFG_SWITCH(32) }
#undef DS_CFG_SWITCH
  DS_CHECK_LAUNCH();
  if (splitk > 1) {
    int64_t total = (int64_t)g.batch * g.M * g.N;
    int G = 1;
    while (G < 64 && G * 8 < splitk) G *= 2;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)cdiv64(total, 256 / G)), dim3(256), 0, st, k, G);
    DS_CHECK_LAUNCH();
  }
  return 0;
}
