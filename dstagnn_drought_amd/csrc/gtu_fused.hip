// gtu_fused.hip — the block's GTU stage forward as ONE kernel.
//
// GTU.forward x3 + cat + fcmy + dropout + residual + ReLUs + LN over C (model/DSTAGNN_my.py:184-197,
// 239-252).  Was two launches on the main stream: the grouped implicit-im2col GEMM writing the
// three convolution outputs conv_k (B*N*(T-k+1), 2C) — 33 MB at PEMS08 — and gtu_tail_fwd_ct
// reading them back for the gates.  Here a workgroup owns NB = 22 consecutive nodes (B*N/22 ~
// one workgroup per CU at PEMS08) and keeps everything between X and the block output on chip:
//   1. the nodes' X rows (t, c) staged in LDS (rows padded to 36 floats: conflict-free float4
//      fragments), plus every activation the tail reads, issued in the same round;
//   2. per GTU, conv = X (*) W + b on the f32 matrix cores (v_mfma_f32_16x16x4_f32): output row
//      (node, t') reads the contiguous window X[node][t'..t'+k-1][:] — the implicit im2col is just
//      a row offset into the staged tile; a wave owns one channel half (16 of the C tanh columns
//      and the same 16 sigmoid columns) for every second row tile, so the P and Q of a gate sit in
//      the same lane: the gate tanh(P) * sigmoid(Q) is formed in registers and stored into the
//      node's concat tile G (LDS) — conv_k still goes to HBM (the backward's gate derivative);
//   3. fcmy + dropout + residual + ReLUs from LDS, the LayerNorm over C per (node, t).
// Weights: the GTU weights re-laid (o, j, c) (param_prep kind 3, rows of k C floats: a lane's B
// fragment is one float4), streamed from L2 with double-buffered fragments.
// Outputs and saved tensors are exactly the two-launch path's (conv_k, G, tco, r, mu, rs, out),
// so the backward is unchanged.  C = 32, T = 12 (PEMS04/07/08); elsewhere the two launches.
#include <mutex>
#include <set>

#include "common.hpp"
#include "ops.hpp"

namespace {

constexpr int kGC = 32, kGT = 12, kGS = 3 * kGT - 12, kGCT = kGC * kGT;  // C, T, S = 3T - 12
constexpr int kGNB = 22;        // nodes per workgroup
constexpr int kGXS = kGC + 4;   // LDS row stride of the X tile
constexpr int kGSP = kGS + 1;   // ... of a node channel's concat row in G
constexpr int kGMT = (kGNB * (kGT - 2) + 15) / 16;  // row tiles of the widest output (k = 3): 14
constexpr int kGMTW = (kGMT + 1) / 2;                // per wave (two waves per channel half): 7

__device__ __forceinline__ floatx4 gmf16(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float g4at(const float4& v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}
__device__ __forceinline__ float gf_sigmoid(float x) { return __frcp_rn(1.f + __expf(-x)); }
__device__ __forceinline__ float gf_tanh(float x) {  // gtu_tail.hip's fast_tanh (same arithmetic)
  const float e = __expf(2.f * fminf(fmaxf(x, -15.f), 15.f));
  return 1.f - 2.f * __frcp_rn(e + 1.f);
}

// one GTU (kernel width KS): conv rows m = node * Tg + t' of this workgroup, channel half h of
// wave w, row tiles mt = w/2, w/2 + 2, ...; gates into Gs, conv_k (+ bias) to HBM
template <int KS>
__device__ __forceinline__ void gf_gtu(const GtuFusedArgs& a, int q, int s_off, int64_t bn0, int nn, const float* Xs,
                                       float* Gs, int w, int i, int lq) {
  constexpr int Tg = kGT - KS + 1, KK = KS * kGC, NCH = KK / 16;
  const int M = nn * Tg, MT = (M + 15) / 16;
  const int h = w & 1, mt0 = w >> 1;
  floatx4 accp[kGMTW], accq[kGMTW];
  int rowoff[kGMTW];
#pragma unroll
  for (int u = 0; u < kGMTW; ++u) {
    accp[u] = accq[u] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int m = min((mt0 + 2 * u) * 16 + i, M - 1);  // (clamped rows: computed, never stored)
    const int n = m / Tg, tp = m - n * Tg;
    rowoff[u] = (n * kGT + tp) * kGXS;
  }
  const float* wt = a.wt[q];  // (2C, KS C): row o = output channel, column j C + c
  const float* wpp = wt + (int64_t)(h * 16 + i) * KK + 4 * lq;          // tanh half, channel h*16 + i
  const float* wpq = wt + (int64_t)(kGC + h * 16 + i) * KK + 4 * lq;    // sigmoid half
  auto step = [&](int ch, const float4& bp, const float4& bq) {
    const int j = ch >> 1, c0 = (ch & 1) * 16;  // contraction index 16 ch + 4 lq + s = j C + c
#pragma unroll
    for (int u = 0; u < kGMTW; ++u) {
      if (mt0 + 2 * u >= MT) continue;  // (wave-uniform)
      const float4 av = *reinterpret_cast<const float4*>(Xs + rowoff[u] + j * kGXS + c0 + 4 * lq);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        accp[u] = gmf16(g4at(av, s), g4at(bp, s), accp[u]);
        accq[u] = gmf16(g4at(av, s), g4at(bq, s), accq[u]);
      }
    }
  };
  float4 p0 = *reinterpret_cast<const float4*>(wpp), q0 = *reinterpret_cast<const float4*>(wpq), p1, q1;
  int ch = 0;
  for (; ch + 1 < NCH; ch += 2) {
    p1 = *reinterpret_cast<const float4*>(wpp + 16 * (ch + 1));
    q1 = *reinterpret_cast<const float4*>(wpq + 16 * (ch + 1));
    __builtin_amdgcn_sched_barrier(0);
    step(ch, p0, q0);
    __builtin_amdgcn_sched_barrier(0);
    const int cn = min(ch + 2, NCH - 1);
    p0 = *reinterpret_cast<const float4*>(wpp + 16 * cn);
    q0 = *reinterpret_cast<const float4*>(wpq + 16 * cn);
    __builtin_amdgcn_sched_barrier(0);
    step(ch + 1, p1, q1);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (ch < NCH) step(ch, p0, q0);
  // epilogue: D[4 lq + r][i] of row tile mt -> row m, channel c = h 16 + i
  const int c = h * 16 + i;
  const float bp_ = a.bias[q][c], bq_ = a.bias[q][kGC + c];
  float* conv = a.conv[q];
#pragma unroll
  for (int u = 0; u < kGMTW; ++u) {
    if (mt0 + 2 * u >= MT) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = (mt0 + 2 * u) * 16 + 4 * lq + r;
      if (m >= M) continue;
      const int n = m / Tg, tp = m - n * Tg;
      const float P = accp[u][r] + bp_, Q = accq[u][r] + bq_;
      float* row = conv + ((bn0 + n) * Tg + tp) * (2 * kGC);
      row[c] = P;
      row[kGC + c] = Q;
      Gs[(n * kGC + c) * kGSP + s_off + tp] = gf_tanh(P) * gf_sigmoid(Q);
    }
  }
}

template <bool FIRST>
__global__ __launch_bounds__(256, 1) void gtu_fwd_fused_kernel(GtuFusedArgs a) {
  constexpr int NE = (kGNB * kGCT + 255) / 256;  // tail elements per thread (33)
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  float* Xs = lds;                                  // [NB T][36]
  float* Gs = Xs + kGNB * kGT * kGXS;               // [NB C][25]
  float* Rl = Gs + kGNB * kGC * kGSP;               // [NB][C T] r for the LayerNorm
  float* Wl = Rl + kGNB * kGCT;                     // [T][25] fcmy weight
  float* mus = Wl + kGT * kGSP;                     // [NB T]
  float* rss = mus + kGNB * kGT;                    // [NB T]
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, i = l & 15, lq = l >> 4;
  const int64_t bn0 = (int64_t)blockIdx.x * kGNB;
  const int nn = (int)min<int64_t>(kGNB, a.BN - bn0);
  const int ne = nn * kGCT;

  // ---- 1. one round of loads: X tile, the fcmy weight, this thread's tail operands ----------
  {
    const float4* gx = reinterpret_cast<const float4*>(a.X + bn0 * kGCT);
    constexpr int XV = (kGNB * kGCT / 4 + 255) / 256;  // 9
    float4 xv[XV];
#pragma unroll
    for (int u = 0; u < XV; ++u) xv[u] = gx[min(u * 256 + tid, ne / 4 - 1)];
    float wv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) wv[u] = a.fcmy_w[min(tid + 256 * u, kGT * kGS - 1)];
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int e4 = u * 256 + tid;
      if (e4 < ne / 4) {
        const int e = 4 * e4, row = e / kGC, c = e - row * kGC;  // X rows (n t, c)
        *reinterpret_cast<float4*>(Xs + row * kGXS + c) = xv[u];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + 256 * u;
      if (e < kGT * kGS) Wl[(e / kGS) * kGSP + e % kGS] = wv[u];
    }
  }
  float xr[NE];  // the residual source of this thread's tail elements e = (n, c, t)
#pragma unroll
  for (int u = 0; u < NE; ++u) {
    const int e = min(tid + 256 * u, ne - 1), n = e / kGCT, t = e % kGT;
    xr[u] = FIRST ? a.x[(bn0 + n) * kGT + t] : a.x[bn0 * kGCT + e];
  }
  __syncthreads();

  // ---- 2. the three convolutions and their gates --------------------------------------------
  gf_gtu<3>(a, 0, 0, bn0, nn, Xs, Gs, w, i, lq);
  gf_gtu<5>(a, 1, kGT - 2, bn0, nn, Xs, Gs, w, i, lq);
  gf_gtu<7>(a, 2, 2 * kGT - 6, bn0, nn, Xs, Gs, w, i, lq);
  __syncthreads();

  // ---- 3. fcmy + dropout + residual + ReLUs (gtu_tail_fwd_ct's arithmetic) -----------------
  float rv[NE];
#pragma unroll
  for (int u = 0; u < NE; ++u) {
    const int e = tid + 256 * u;
    rv[u] = 0.f;
    if (e >= ne) continue;
    const int n = e / kGCT, ct = e - n * kGCT, c = ct / kGT, t = ct - c * kGT;
    float tc = a.fcmy_b[t];
    const float* gr = Gs + (n * kGC + c) * kGSP;
    const float* wr = Wl + t * kGSP;
#pragma unroll 8
    for (int s = 0; s < kGS; ++s) tc = fmaf(gr[s], wr[s], tc);
    const int64_t ge = bn0 * kGCT + e;  // global (b, n, c, t) index
    if (a.drop_p > 0.f) tc *= drop_scale(a.seed, 1, (uint64_t)ge + a.drop_off, a.drop_p);
    float tco, xres;
    if (FIRST) {
      tco = fmaxf(tc, 0.f);
      xres = a.res_w[c] * xr[u] + a.res_b[c];
    } else {
      tco = fmaxf(Xs[(n * kGT + t) * kGXS + c] + tc, 0.f);
      xres = xr[u];
    }
    const float r = fmaxf(xres + tco, 0.f);
    a.tco[ge] = tco;
    a.r[ge] = r;
    Rl[e] = r;
    rv[u] = r;
  }
  __syncthreads();
  // G out (the fcmy weight gradient's operand): the nodes' [c][s] rows are one contiguous block
  for (int e = tid; e < nn * kGC * kGS; e += 256) {
    const int nc = e / kGS, s = e - nc * kGS;
    a.G[bn0 * kGC * kGS + e] = Gs[nc * kGSP + s];
  }
  // ---- 4. LayerNorm over C per (node, t): two fixed-order passes -----------------------------
  for (int row = tid; row < nn * kGT; row += 256) {
    const int n = row / kGT, t = row - n * kGT;
    const float* rr = Rl + n * kGCT + t;
    float sum = 0.f;
#pragma unroll 8
    for (int c = 0; c < kGC; ++c) sum += rr[c * kGT];
    const float mean = sum * (1.f / kGC);
    float var = 0.f;
#pragma unroll 8
    for (int c = 0; c < kGC; ++c) {
      const float d = rr[c * kGT] - mean;
      var += d * d;
    }
    const float rs = rsqrtf(var * (1.f / kGC) + 1e-5f);
    mus[row] = mean;
    rss[row] = rs;
    a.mu[(bn0 + n) * kGT + t] = mean;
    a.rs[(bn0 + n) * kGT + t] = rs;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < NE; ++u) {
    const int e = tid + 256 * u;
    if (e >= ne) continue;
    const int n = e / kGCT, ct = e - n * kGCT, c = ct / kGT, t = ct - c * kGT;
    a.out[bn0 * kGCT + e] = (rv[u] - mus[n * kGT + t]) * rss[n * kGT + t] * a.ln_g[c] + a.ln_b[c];
  }
}

size_t gtu_fused_lds() {
  return sizeof(float) * ((size_t)kGNB * kGT * kGXS + (size_t)kGNB * kGC * kGSP + (size_t)kGNB * kGCT +
                          (size_t)kGT * kGSP + 2 * (size_t)kGNB * kGT);
}

}  // namespace

bool gtu_fused_fwd_ok(int C, int T) {
  static const bool on = getenv("DSTAGNN_GTU_FUSED") && atoi(getenv("DSTAGNN_GTU_FUSED")) != 0;
  return on && C == kGC && T == kGT;
}

int op_gtu_fused_fwd(const GtuFusedArgs& a, hipStream_t st) {
  if (!gtu_fused_fwd_ok(a.C, a.T) || a.BN <= 0 || a.BN * kGCT >= (1ll << 31)) {
    set_last_error("gtu_fused_fwd: unsupported shape");
    return DSTAGNN_E_SHAPE;
  }
  using Kern = void (*)(GtuFusedArgs);
  const Kern k = a.first ? gtu_fwd_fused_kernel<true> : gtu_fwd_fused_kernel<false>;
  const size_t lds = gtu_fused_lds();
  {
    static std::mutex mu;
    static std::set<Kern> done;
    std::lock_guard<std::mutex> lock(mu);
    if (!done.count(k)) {
      const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) { set_last_error(std::string("gtu_fused_fwd: ") + hipGetErrorString(e)); return (int)e; }
      done.insert(k);
    }
  }
  // the three convolutions' algorithmic FLOP (the GEMM family's accounting)
  const double flops = 2.0 * a.BN * (2.0 * kGC) * kGC * ((kGT - 2) * 3 + (kGT - 4) * 5 + (kGT - 6) * 7);
  const double bytes = 4.0 * a.BN * (kGCT * 6.0 + 2 * kGC * 24.0 + kGC * kGS);
  void* rec = gemm_prof_begin(flops, bytes, st);
  hipLaunchKernelGGL(k, dim3((unsigned)cdiv64(a.BN, kGNB)), dim3(256), lds, st, a);
  DS_CHECK_LAUNCH();
  gemm_prof_end(rec, st);
  return 0;
}
