// gtu_fused.hip — the block's GTU stage forward as ONE kernel.
//
// GTU.forward x3 + cat + fcmy + dropout + residual + ReLUs + LN over C (model/DSTAGNN_my.py:184-197,
// 239-252).  Was two launches on the main stream: the grouped implicit-im2col GEMM writing the
// three convolution outputs conv_k (B*N*(T-k+1), 2C) — 33 MB at PEMS08 — and gtu_tail_fwd_ct
// reading them back for the gates.  Here a workgroup of 8 waves owns NB = 22 consecutive nodes
// (B*N/22 ~ one workgroup per CU at PEMS08, two waves per SIMD) and keeps everything between X
// and the block output on chip:
//   1. the nodes' X rows (t, c) staged in LDS (rows padded to 36 floats: conflict-free float4
//      fragments) with the residual source, plus the tail's per-lane parameters, in one round;
//   2. per GTU, conv = X (*) W + b on the f32 matrix cores (v_mfma_f32_16x16x4_f32): output row
//      (node, t') reads the contiguous window X[node][t'..t'+k-1][:] — the implicit im2col is just
//      a row offset into the staged tile; a wave owns one channel half (16 of the C tanh columns
//      and the same 16 sigmoid columns) for every fourth row tile, so the P and Q of a gate sit in
//      the same lane: the gate tanh(P) * sigmoid(Q) is formed in registers and stored into the
//      node's concat tile G (LDS) — conv_k still goes to HBM (the backward's gate derivative);
//   3. per node (one wave each): fcmy as a 32 x 12 x 24 product on the matrix cores, + bias,
//      dropout, residual and ReLUs in the accumulator registers, and the LayerNorm over C per
//      (node, t) by two cross-lane sums — no LDS round trip.
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
constexpr int kGW = 8;          // waves per workgroup (two per SIMD)
constexpr int kGXS = kGC + 4;   // LDS row stride of the X tile
constexpr int kGSP = kGS + 1;   // ... of a node channel's concat row in G
constexpr int kGMT = (kGNB * (kGT - 2) + 15) / 16;  // row tiles of the widest output (k = 3): 14
constexpr int kGMTW = (kGMT + 3) / 4;                // per wave (four waves per channel half): 4

__device__ __forceinline__ floatx4 gmf16(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float g4at(const float4& v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}
// the gates with the hardware reciprocal (v_rcp_f32, 1 ulp): gtu_tail.hip's fast_tanh /
// fast_sigmoid up to the last bit of the reciprocal
__device__ __forceinline__ float gf_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float gf_tanh(float x) {
  const float e = __expf(2.f * fminf(fmaxf(x, -15.f), 15.f));
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

// sum over the 16 lanes of a DPP row, the same value in every lane (quad swaps, then the half-row
// and row mirrors)
__device__ __forceinline__ float gf_row16_sum(float x) {
  x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x141, 0xF, 0xF, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x140, 0xF, 0xF, true));
  return x;
}

// one GTU (kernel width KS): conv rows m = node * Tg + t' of this workgroup; wave w owns channel
// half h = w & 1 (16 tanh columns and the same 16 sigmoid columns) for row tiles w/2 + 4u; the
// gates go to Gs, conv_k (+ bias) to HBM.  p0 / q0 hold the first B fragments on entry (issued
// by the caller ahead of the previous GTU's stores); on exit they hold the next GTU's (KN = 0:
// none).
template <int KS, int KN>
__device__ __forceinline__ void gf_gtu(const GtuFusedArgs& a, int q, int s_off, int64_t bn0, int nn, const float* Xs,
                                       float* Gs, int w, int i, int lq, float4& p0, float4& q0) {
  constexpr int Tg = kGT - KS + 1, KK = KS * kGC, NCH = KK / 16;
  const int M = nn * Tg, MT = (M + 15) / 16;
  const int h = w & 1, mt0 = w >> 1;
  floatx4 accp[kGMTW], accq[kGMTW];
  int rowoff[kGMTW];
#pragma unroll
  for (int u = 0; u < kGMTW; ++u) {
    accp[u] = accq[u] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int m = min((mt0 + 4 * u) * 16 + i, M - 1);  // (clamped rows: computed, never stored)
    const int n = m / Tg, tp = m - n * Tg;
    rowoff[u] = (n * kGT + tp) * kGXS;
  }
  const float* wt = a.wt[q];  // (2C, KS C): row o = output channel, column j C + c
  const float* wpp = wt + (h * 16 + i) * KK + 4 * lq;          // tanh half, channel h*16 + i
  const float* wpq = wt + (kGC + h * 16 + i) * KK + 4 * lq;    // sigmoid half
  auto step = [&](int ch, const float4& bp, const float4& bq) {
    const int j = ch >> 1, c0 = (ch & 1) * 16;  // contraction index 16 ch + 4 lq + s = j C + c
    float4 av[kGMTW];
#pragma unroll
    for (int u = 0; u < kGMTW; ++u)
      if (mt0 + 4 * u < MT) av[u] = *reinterpret_cast<const float4*>(Xs + rowoff[u] + j * kGXS + c0 + 4 * lq);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int u = 0; u < kGMTW; ++u) {
        if (mt0 + 4 * u >= MT) continue;  // (wave-uniform)
        accp[u] = gmf16(g4at(bp, s), g4at(av[u], s), accp[u]);
        accq[u] = gmf16(g4at(bq, s), g4at(av[u], s), accq[u]);
      }
  };
  float4 p1, q1;
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
  // the next GTU's first fragments, issued before this epilogue's stores (a later wait on them
  // then does not wait for the stores: gfx9 counts both in vmcnt, in order)
  if (KN > 0) {
    constexpr int KKN = KN * kGC;
    p0 = *reinterpret_cast<const float4*>(a.wt[q + 1] + (h * 16 + i) * KKN + 4 * lq);
    q0 = *reinterpret_cast<const float4*>(a.wt[q + 1] + (kGC + h * 16 + i) * KKN + 4 * lq);
  }
  __builtin_amdgcn_sched_barrier(0);
  // epilogue: the weights are the A operand, so D[4 lq + r][i] of row tile mt is channel
  // c0 + r = h 16 + 4 lq + r of row m = 16 mt + i: a lane's P and Q are float4 runs of a conv row
  const int c0 = h * 16 + 4 * lq;
  const float4 bp4 = *reinterpret_cast<const float4*>(a.bias[q] + c0);
  const float4 bq4 = *reinterpret_cast<const float4*>(a.bias[q] + kGC + c0);
  float* conv = a.conv[q];
#pragma unroll
  for (int u = 0; u < kGMTW; ++u) {
    if (mt0 + 4 * u >= MT) continue;
    const int m = (mt0 + 4 * u) * 16 + i;
    if (m >= M) continue;
    const int n = m / Tg, tp = m - n * Tg;
    const float4 P = make_float4(accp[u][0] + bp4.x, accp[u][1] + bp4.y, accp[u][2] + bp4.z, accp[u][3] + bp4.w);
    const float4 Q = make_float4(accq[u][0] + bq4.x, accq[u][1] + bq4.y, accq[u][2] + bq4.z, accq[u][3] + bq4.w);
    float* row = conv + ((bn0 + n) * Tg + tp) * (2 * kGC);
    *reinterpret_cast<float4*>(row + c0) = P;
    *reinterpret_cast<float4*>(row + kGC + c0) = Q;
    float* g = Gs + (n * kGC + c0) * kGSP + s_off + tp;
#pragma unroll
    for (int r = 0; r < 4; ++r) g[r * kGSP] = gf_tanh(g4at(P, r)) * gf_sigmoid(g4at(Q, r));
  }
}

template <bool FIRST>
__global__ __launch_bounds__(kGW * 64, 1) void gtu_fwd_fused_kernel(GtuFusedArgs a) {
  constexpr int NT = kGW * 64;
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  float* Xs = lds;                                  // [NB T][36]
  float* Gs = Xs + kGNB * kGT * kGXS;               // [NB C][25]
  float* Rl = Gs + kGNB * kGC * kGSP;               // the residual source: [NB][C T] (FIRST: [NB][T])
  // (the wave index in an SGPR: every per-wave tile condition below is a scalar branch)
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63, i = l & 15, lq = l >> 4;
  const int64_t bn0 = (int64_t)blockIdx.x * kGNB;
  const int nn = (int)min<int64_t>(kGNB, a.BN - bn0);
  const int ne = nn * kGCT;
  TF_DECL;
  TF_MARK(0);

  // ---- 1. one round of loads: X tile, the residual source, the first GTU's B fragments, the
  //         fcmy A fragments and the per-channel parameters of the tail ---------------------
  constexpr int XV = (kGNB * kGCT / 4 + NT - 1) / NT;  // 5
  float4 p0, q0;
  {
    const int h = w & 1;
    p0 = *reinterpret_cast<const float4*>(a.wt[0] + (h * 16 + i) * 3 * kGC + 4 * lq);
    q0 = *reinterpret_cast<const float4*>(a.wt[0] + (kGC + h * 16 + i) * 3 * kGC + 4 * lq);
  }
  {
    const float4* gx = reinterpret_cast<const float4*>(a.X + bn0 * kGCT);
    float4 xv[XV];
#pragma unroll
    for (int u = 0; u < XV; ++u) xv[u] = gx[min(u * NT + tid, ne / 4 - 1)];
    if (FIRST) {
      if (tid < nn * kGT) Rl[tid] = a.x[bn0 * kGT + tid];
    } else {
      const float4* gr = reinterpret_cast<const float4*>(a.x + bn0 * kGCT);
      float4 rv4[XV];
#pragma unroll
      for (int u = 0; u < XV; ++u) rv4[u] = gr[min(u * NT + tid, ne / 4 - 1)];
#pragma unroll
      for (int u = 0; u < XV; ++u)
        if (u * NT + tid < ne / 4) reinterpret_cast<float4*>(Rl)[u * NT + tid] = rv4[u];
    }
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int e4 = u * NT + tid;
      if (e4 < ne / 4) {
        const int e = 4 * e4, row = e / kGC, c = e - row * kGC;  // X rows (n t, c)
        *reinterpret_cast<float4*>(Xs + row * kGXS + c) = xv[u];
      }
    }
  }
  // tail operands of this lane: fcmy weight rows t = i (the A operand; lanes i >= T zero) and
  // the per-channel parameters of channels c = i and 16 + i
  float aw[kGS / 4];  // A[m = t][k = s = 4 kk + lq] = fcmy_w[t][s]
#pragma unroll
  for (int kk = 0; kk < kGS / 4; ++kk) aw[kk] = i < kGT ? a.fcmy_w[min(i, kGT - 1) * kGS + 4 * kk + lq] : 0.f;
  const int t0 = min(4 * lq, kGT - 4);  // this lane's 4 output columns t0..t0+3 (lq = 3: a copy, not stored)
  const float4 fb = *reinterpret_cast<const float4*>(a.fcmy_b + t0);
  float lg[2], lb[2], rw[2], rb[2];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    lg[v] = a.ln_g[16 * v + i];
    lb[v] = a.ln_b[16 * v + i];
    rw[v] = FIRST ? a.res_w[16 * v + i] : 0.f;
    rb[v] = FIRST ? a.res_b[16 * v + i] : 0.f;
  }
  __syncthreads();
  TF_MARK(1);

  // ---- 2. the three convolutions and their gates --------------------------------------------
  gf_gtu<3, 5>(a, 0, 0, bn0, nn, Xs, Gs, w, i, lq, p0, q0);
  TF_MARK(2);
  gf_gtu<5, 7>(a, 1, kGT - 2, bn0, nn, Xs, Gs, w, i, lq, p0, q0);
  TF_MARK(3);
  gf_gtu<7, 0>(a, 2, 2 * kGT - 6, bn0, nn, Xs, Gs, w, i, lq, p0, q0);
  TF_MARK(4);
  __syncthreads();
  TF_MARK(5);

  // ---- 3. per node (one wave each): fcmy on the matrix cores (tc[t][c] = sum_s W[t][s] G[c][s],
  //         two 16-channel tiles), + bias, dropout, residual, ReLUs (gtu_tail_fwd_ct's
  //         arithmetic), then the LayerNorm over C per (node, t) in registers: lane (i, lq) holds
  //         columns t0..t0+3 of channels i and 16 + i, the channel sums are DPP row sums ---------
  const bool tv = lq < kGT / 4;
#pragma unroll
  for (int j = 0; j < (kGNB + kGW - 1) / kGW; ++j) {
    const int n = w + kGW * j;
    if (n >= nn) continue;
    floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
    const float* g0 = Gs + (n * kGC + i) * kGSP + lq;
#pragma unroll
    for (int kk = 0; kk < kGS / 4; ++kk) {
      acc[0] = gmf16(aw[kk], g0[4 * kk], acc[0]);
      acc[1] = gmf16(aw[kk], g0[16 * kGSP + 4 * kk], acc[1]);
    }
    float rv[2][4];
    float sum[4];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int c = 16 * v + i;
      const int e0 = n * kGCT + c * kGT + t0;
      const int64_t ge0 = bn0 * kGCT + e0;  // global (b, n, c, t0) index
      float4 xres4;
      if (!FIRST) xres4 = *reinterpret_cast<const float4*>(Rl + e0);
      float tco[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float tc = acc[v][r] + g4at(fb, r);
        if (a.drop_p > 0.f) tc *= drop_scale(a.seed, 1, (uint64_t)(ge0 + r) + a.drop_off, a.drop_p);
        float xres;
        if (FIRST) {
          tco[r] = fmaxf(tc, 0.f);
          xres = rw[v] * Rl[n * kGT + t0 + r] + rb[v];
        } else {
          tco[r] = fmaxf(Xs[(n * kGT + t0 + r) * kGXS + c] + tc, 0.f);
          xres = g4at(xres4, r);
        }
        rv[v][r] = fmaxf(xres + tco[r], 0.f);
      }
      if (tv) {
        *reinterpret_cast<float4*>(a.tco + ge0) = make_float4(tco[0], tco[1], tco[2], tco[3]);
        *reinterpret_cast<float4*>(a.r + ge0) = make_float4(rv[v][0], rv[v][1], rv[v][2], rv[v][3]);
      }
    }
    float mean[4], rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) sum[r] = gf_row16_sum(rv[0][r] + rv[1][r]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      mean[r] = sum[r] * (1.f / kGC);
      const float d0 = rv[0][r] - mean[r], d1 = rv[1][r] - mean[r];
      rs[r] = d0 * d0 + d1 * d1;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) rs[r] = rsqrtf(gf_row16_sum(rs[r]) * (1.f / kGC) + 1e-5f);
    if (tv) {
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (rv[v][r] - mean[r]) * rs[r] * lg[v] + lb[v];
        *reinterpret_cast<float4*>(a.out + bn0 * kGCT + n * kGCT + (16 * v + i) * kGT + t0) =
            make_float4(o[0], o[1], o[2], o[3]);
      }
      if (i == 0) {
        *reinterpret_cast<float4*>(a.mu + (bn0 + n) * kGT + t0) = make_float4(mean[0], mean[1], mean[2], mean[3]);
        *reinterpret_cast<float4*>(a.rs + (bn0 + n) * kGT + t0) = make_float4(rs[0], rs[1], rs[2], rs[3]);
      }
    }
  }
  TF_MARK(6);
  // G out (the fcmy weight gradient's operand): the nodes' [c][s] rows are one contiguous block
  {
    float4* gout = reinterpret_cast<float4*>(a.G + bn0 * kGC * kGS);
    for (int e4 = tid; e4 < nn * kGC * (kGS / 4); e4 += NT) {
      const int nc = e4 / (kGS / 4), s = 4 * (e4 - nc * (kGS / 4));
      const float* g = Gs + nc * kGSP + s;
      gout[e4] = make_float4(g[0], g[1], g[2], g[3]);
    }
  }
  TF_MARK(7);
  TF_PRINT("gtu_fused", 8);
}

__device__ __forceinline__ float gf_ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gf_st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

bool gf_al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

size_t gtu_fused_lds() {
  return sizeof(float) * ((size_t)kGNB * kGT * kGXS + (size_t)kGNB * kGC * kGSP + (size_t)kGNB * kGCT);
}


// ---------------------------------------------------------------------------------------------
// Backward: the GTU stage's backward as ONE kernel (model/DSTAGNN_my.py:184-197, 239-252 by
// autograd).  Was gtu_tail_bwd_ct (LN / ReLU / residual / dropout backward, dG = dtc W, the gate
// derivatives into zero-padded 2C-wide rows, 50 MB at PEMS08) + gtu_tconv (the transposed
// convolutions over the padded rows, 60 % of its MACs on zeros).  Here a workgroup of 8 waves
// owns the same NB = 22 nodes as the forward:
//   A. per node (one wave each), in the forward tail's register layout (lane (i, lq): channels
//      i and 16 + i, columns t0..t0+3): the LayerNorm backward with DPP row sums, the ReLU /
//      dropout / residual backward, dtc and dx out; dG = dtc W as 2 x 2 matrix-core tiles whose
//      k steps contract t = 4 lq + r — the lane's own dtc values ARE the A fragments, and the
//      result holds 4 consecutive channels of one s: the gate derivatives read P / Q and write
//      dconv as float4 runs, compact (BN Tg, 2C) — the weight gradients' operand, no zero rows;
//   B. per GTU, its gate-gradient rows staged in LDS (read back from L2: one workgroup's rows),
//      then dX[n][t' + j][c] += sum_o dconv[(n, t')][o] W[o][c][j] input-stationary: a wave owns
//      16-row tiles of (node, t') rows x 16-channel halves and computes all k taps against the
//      same B fragments, then the workgroup adds tap by tap into the LDS accumulator rows
//      shifted by j (float4 read-modify-write, a barrier between taps: a fixed summation order
//      per output row) — exactly the convolution's MACs, none on padding;
//   C. gpre = (X > 0) ? dX : 0 (the Chebyshev output's ReLU backward), float4 rows.
// LN gamma / beta (and first-block residual_conv) partial sums: one row per workgroup.
// ---------------------------------------------------------------------------------------------
constexpr int kGBS = 2 * kGC + 4;            // LDS row stride of a staged gate-gradient / weight row
constexpr int kGBX = kGC + 4;                // ... of a dX accumulator row
// per GTU q: its row tiles' gate-gradient rows, then its weights (j, c) rows of 2C
constexpr int gb_rows(int q) { return (kGNB * (kGT - 2 - 2 * q) + 15) / 16 * 16; }
constexpr int gb_stage(int q) { return (gb_rows(q) + (3 + 2 * q) * kGC) * kGBS; }
constexpr int gb_cmax(int a, int b) { return a > b ? a : b; }
constexpr int kGBStage = gb_cmax(gb_stage(0), gb_cmax(gb_stage(1), gb_stage(2)));

constexpr int kGBTT = kGC * 13;                     // a wave's dtc transpose buffer [c][13]
constexpr int kGBF = kGT * (kGS + 1);                // fcmy weight + bias gradient entries (t, s <= S)
static_assert(kGW * kGBTT <= kGBStage, "dtc transpose buffers live in the staging region");
constexpr int kGBP = 4 * kGC + kGBF;                 // a workgroup's partial row: gamma, beta, res w, res b, fcmy
constexpr int kGBG1 = 16;                            // workgroups per level-1 group of the ticket tree

size_t gtu_fused_bwd_lds() {
  return sizeof(float) * ((size_t)kGBStage + (size_t)kGNB * kGT * kGBX + 4 * kGW * kGC + (size_t)kGW * kGBF);
}

// step B for GTU KQ (kernel width KS): the staged operands — its rows (rows M..16 MT zero) and
// its weights (j, c, o) as rows j C + c — are loaded into registers one GTU ahead (GbStage)
template <int KQ>
struct GbStage {
  static constexpr int KS = 3 + 2 * KQ, RX = gb_rows(KQ), NT = kGW * 64;
  static constexpr int NV = (RX * 16 + NT - 1) / NT, NW = (KS * kGC * 16 + NT - 1) / NT;
  float4 v[NV], wv[NW];
};
template <int KQ>
__device__ __forceinline__ void gb_load(const GtuFusedBwdArgs& a, int64_t bn0, int nn, GbStage<KQ>& g) {
  using S = GbStage<KQ>;
  constexpr int Tg = kGT - S::KS + 1;
  const int M = nn * Tg;
  const float4* src = reinterpret_cast<const float4*>(a.dconv[KQ] + bn0 * Tg * 2 * kGC);
  const float4* wsrc = reinterpret_cast<const float4*>(a.wf[KQ]);
#pragma unroll
  for (int u = 0; u < S::NV; ++u) {
    const int e4 = u * S::NT + (int)threadIdx.x;
    g.v[u] = e4 < M * 16 ? src[e4] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int u = 0; u < S::NW; ++u) g.wv[u] = wsrc[min(u * S::NT + (int)threadIdx.x, S::KS * kGC * 16 - 1)];
}
template <int KQ>
__device__ __forceinline__ void gb_store(float* Ds, const GbStage<KQ>& g) {
  using S = GbStage<KQ>;
  float* Ws = Ds + S::RX * kGBS;
#pragma unroll
  for (int u = 0; u < S::NV; ++u) {
    const int e4 = u * S::NT + (int)threadIdx.x, row = e4 >> 4;
    if (row < S::RX) *reinterpret_cast<float4*>(Ds + row * kGBS + (e4 & 15) * 4) = g.v[u];
  }
#pragma unroll
  for (int u = 0; u < S::NW; ++u) {
    const int e4 = u * S::NT + (int)threadIdx.x, row = e4 >> 4;
    if (row < S::KS * kGC) *reinterpret_cast<float4*>(Ws + row * kGBS + (e4 & 15) * 4) = g.wv[u];
  }
}
// the staged operands in LDS on entry; next() issues the next GTU's loads between this GTU's
// matrix-core work and its accumulator taps; Ds is free on exit
template <int KQ, class NX>
__device__ __forceinline__ void gb_tconv(int nn, float* Ds, float* dXs, int w, int i, int lq, NX&& next) {
  constexpr int KS = 3 + 2 * KQ, Tg = kGT - KS + 1;
  const int M = nn * Tg, MT = (M + 15) / 16;
  float* Ws = Ds + gb_rows(KQ) * kGBS;
  // every unit's k taps first (unit u = (tile u / 2, channel half u % 2), wave w: u = w + 8 uu) ...
  constexpr int MTX = (kGNB * Tg + 15) / 16, UPW = (2 * MTX + kGW - 1) / kGW;
  const int units = 2 * MT;
  floatx4 acc[UPW][KS];
#pragma unroll
  for (int uu = 0; uu < UPW; ++uu) {
    const int u = w + kGW * uu;
    if (u >= units) continue;  // (wave-uniform)
    const int mt = u >> 1, ct = u & 1;
#pragma unroll
    for (int j = 0; j < KS; ++j) acc[uu][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* brow = Ds + (mt * 16 + i) * kGBS + 4 * lq;             // B[k = o][n = row]
    const float* wrow = Ws + (16 * ct + i) * kGBS + 4 * lq;             // A[m = c][k = o], tap j at + j C rows
    // fragments of chunk ch + 1 loaded while chunk ch multiplies; within a chunk the k taps'
    // independent accumulators interleave (no back-to-back dependent MFMA)
    float4 bq[2], aq[2][KS];
    auto frag = [&](int ch, int buf) {
      bq[buf] = *reinterpret_cast<const float4*>(brow + 16 * ch);
#pragma unroll
      for (int j = 0; j < KS; ++j) aq[buf][j] = *reinterpret_cast<const float4*>(wrow + j * kGC * kGBS + 16 * ch);
    };
    frag(0, 0);
#pragma unroll
    for (int ch = 0; ch < 2 * kGC / 16; ++ch) {
      if (ch + 1 < 2 * kGC / 16) frag(ch + 1, (ch + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < KS; ++j) acc[uu][j] = gmf16(g4at(aq[ch & 1][j], s), g4at(bq[ch & 1], s), acc[uu][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  next();
  // ... then tap by tap into the accumulator rows: D[4 lq + r][i] is channel 16 ct + 4 lq + r of
  // input row m = 16 mt + i, and tap j sends it to row t' + j.  For one tap the input -> output
  // row map is one-to-one (no two writers of a row); the taps go in order with a barrier
  // between them, so every output row sums its contributions in the fixed order (GTU, tap) —
  // the same bits wherever the node sits in its workgroup's tiles
#pragma unroll
  for (int j = 0; j < KS; ++j) {
#pragma unroll
    for (int uu = 0; uu < UPW; ++uu) {
      const int u = w + kGW * uu;
      if (u >= units) continue;
      const int mt = u >> 1, ct = u & 1, m = mt * 16 + i;
      if (m >= M) continue;
      const int n = m / Tg, tp = m - n * Tg;
      float* d = dXs + (n * kGT + tp + j) * kGBX + 16 * ct + 4 * lq;
      float4 o = *reinterpret_cast<const float4*>(d);
      o.x += acc[uu][j][0];
      o.y += acc[uu][j][1];
      o.z += acc[uu][j][2];
      o.w += acc[uu][j][3];
      *reinterpret_cast<float4*>(d) = o;
    }
    __syncthreads();
  }
}

template <bool FIRST>
__global__ __launch_bounds__(kGW * 64, 1) void gtu_bwd_fused_kernel(GtuFusedBwdArgs a) {
  constexpr int NT = kGW * 64, NS = FIRST ? 4 : 2;
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  float* Ds = lds;                          // [16 MT][68] the current GTU's gate-gradient rows, its weights
  float* dXs = Ds + kGBStage;               // [NB T][36] the dX accumulator
  float* red = dXs + kGNB * kGT * kGBX;     // [NS][8 waves][C] partial sums
  float* redf = red + 4 * kGW * kGC;        // [8 waves][T][S + 1] fcmy gradient partial sums
  constexpr bool fw = true;
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63, i = l & 15, lq = l >> 4;
  const int64_t bn0 = (int64_t)blockIdx.x * kGNB;
  const int nn = (int)min<int64_t>(kGNB, a.BN - bn0);
  const int t0 = min(4 * lq, kGT - 4);  // lq = 3: a copy of lq = 2's columns, never stored
  const bool tv = lq < kGT / 4;
  TF_DECL;
  TF_MARK(0);

  // fcmy weight B fragments: B[k][n = s] at k step r = W[t = 4 lq + r][s = 16 st + i]
  float aw[2][4];
#pragma unroll
  for (int st = 0; st < 2; ++st)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = 4 * lq + r, sidx = 16 * st + i;
      aw[st][r] = (t < kGT && sidx < kGS) ? a.fcmy_w[t * kGS + sidx] : 0.f;
    }
  float lg[2], rw[2];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    lg[v] = a.ln_g[16 * v + i];
    rw[v] = FIRST ? a.res_w[16 * v + i] : 0.f;
  }
  float acc_s[NS][2];
#pragma unroll
  for (int q = 0; q < NS; ++q) acc_s[q][0] = acc_s[q][1] = 0.f;
  floatx4 accf[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};  // dW_fcmy[t][s]
  float* tt = Ds + w * kGBTT;  // this wave's dtc transpose buffer (the staging region is free in A)

  // ---- A. per node (the next node's operands loaded while this one is processed) -----------
  struct NodeIn {
    float4 dy[2], r[2], tc[2], mu, rs, x;
    float4 p[2][2], q[2][2];  // the conv rows behind the lane's dG entries (s = 16 st + i,
                              // c = 16 ct + 4 lq + 0..3): float4 runs of P and of Q
  };
  auto load_node = [&](int n, NodeIn& d) {
    const int64_t nb = bn0 + n;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int64_t e0 = nb * kGCT + (16 * v + i) * kGT + t0;
      d.dy[v] = *reinterpret_cast<const float4*>(a.dout + e0);
      d.r[v] = *reinterpret_cast<const float4*>(a.r + e0);
      d.tc[v] = *reinterpret_cast<const float4*>(a.tco + e0);
    }
    d.mu = *reinterpret_cast<const float4*>(a.mu + nb * kGT + t0);
    d.rs = *reinterpret_cast<const float4*>(a.rs + nb * kGT + t0);
    d.x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (FIRST) d.x = *reinterpret_cast<const float4*>(a.x + nb * kGT + t0);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int sidx = 16 * st + i;
      const int kq = sidx < kGT - 2 ? 0 : (sidx < 2 * kGT - 6 ? 1 : 2);
      const int tp = sidx - (kq == 0 ? 0 : (kq == 1 ? kGT - 2 : 2 * kGT - 6)), Tg = kGT - 2 - 2 * kq;
      const float* cb = kq == 0 ? a.conv[0] : (kq == 1 ? a.conv[1] : a.conv[2]);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        d.p[st][ct] = d.q[st][ct] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (sidx < kGS) {
          const float* row = cb + (nb * Tg + tp) * (2 * kGC) + 16 * ct + 4 * lq;
          d.p[st][ct] = *reinterpret_cast<const float4*>(row);
          d.q[st][ct] = *reinterpret_cast<const float4*>(row + kGC);
        }
      }
    }
  };
  NodeIn nx;
  if (w < nn) load_node(w, nx);
#pragma unroll
  for (int jn = 0; jn < (kGNB + kGW - 1) / kGW; ++jn) {
    const int n = w + kGW * jn;
    if (n >= nn) continue;
    const int64_t nb = bn0 + n;
    const NodeIn cur = nx;
    if (jn + 1 < (kGNB + kGW - 1) / kGW && n + kGW < nn) load_node(n + kGW, nx);
    const float4 *dy4 = cur.dy, *r4 = cur.r, *tc4 = cur.tc;
    const float4 mu4 = cur.mu, rs4 = cur.rs, x4 = cur.x;
    const float4(&pv)[2][2] = cur.p;
    const float4(&qv)[2][2] = cur.q;
    // LayerNorm over C backward (the channel sums: DPP row sums over i, two channels a lane)
    float xh[2][4], dxh[2][4], s1[4], s2[4];
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        xh[v][r] = (g4at(r4[v], r) - g4at(mu4, r)) * g4at(rs4, r);
        dxh[v][r] = g4at(dy4[v], r) * lg[v];
      }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s1[r] = gf_row16_sum(dxh[0][r] + dxh[1][r]) * (1.f / kGC);
      s2[r] = gf_row16_sum(dxh[0][r] * xh[0][r] + dxh[1][r] * xh[1][r]) * (1.f / kGC);
    }
    float dtc[2][4], dr[2][4];
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int64_t e0 = nb * kGCT + (16 * v + i) * kGT + t0;
      float dtco[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float d = g4at(rs4, r) * (dxh[v][r] - s1[r] - xh[v][r] * s2[r]);
        d = g4at(r4[v], r) > 0.f ? d : 0.f;             // relu(xres + tco)
        dr[v][r] = d;
        dtco[r] = g4at(tc4[v], r) > 0.f ? d : 0.f;      // tco = relu(...)
        float dt = dtco[r];
        if (a.drop_p > 0.f) dt *= drop_scale(a.seed, 1, (uint64_t)(e0 + r) + a.drop_off, a.drop_p);
        dtc[v][r] = tv ? dt : 0.f;
        if (tv) {
          acc_s[0][v] += g4at(dy4[v], r) * xh[v][r];
          acc_s[1][v] += g4at(dy4[v], r);
          if (FIRST) {
            acc_s[NS > 2 ? 2 : 0][v] += FIRST ? d * g4at(x4, r) : 0.f;
            acc_s[NS > 3 ? 3 : 0][v] += FIRST ? d : 0.f;
          }
        }
      }
      if (tv) {
#pragma unroll
        for (int r = 0; r < 4; ++r) tt[(16 * v + i) * 13 + t0 + r] = dtc[v][r];
        if (!FIRST) *reinterpret_cast<float4*>(a.dx + e0) = make_float4(dr[v][0], dr[v][1], dr[v][2], dr[v][3]);
#pragma unroll
        for (int r = 0; r < 4; ++r) dXs[(n * kGT + t0 + r) * kGBX + 16 * v + i] = FIRST ? 0.f : dtco[r];
      }
    }
    if (FIRST) {  // dx[n][t] = sum_c res_w[c] dr[c][t]
      float dxs[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) dxs[r] = gf_row16_sum(rw[0] * dr[0][r] + rw[1] * dr[1][r]);
      if (tv && i == 0) *reinterpret_cast<float4*>(a.dx + nb * kGT + t0) = make_float4(dxs[0], dxs[1], dxs[2], dxs[3]);
    }
    // dG[c][s] = sum_t dtc[c][t] W[t][s] (k step r contracts t = 4 lq + r: the A fragment of
    // lane (i, lq) is its own dtc[ct][r]); D[4 lq + r'][i] = dG[c = 16 ct + 4 lq + r'][s = 16 st + i]
    floatx4 g[2][2];
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        g[st][ct] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 4; ++r) g[st][ct] = gmf16(dtc[ct][r], aw[st][r], g[st][ct]);
      }
    // the gate derivatives: o = c (tanh side) and o = C + c (sigmoid side) of conv row (n, t');
    // the gates themselves are the fcmy weight gradient's B fragments (below): G is not re-read
    float gbv[2][2][4];  // [st][ct][r]: G[c = 16 ct + 4 lq + r][s = 16 st + i]; s = S: ones (bias)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int sidx = 16 * st + i;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) gbv[st][ct][r] = sidx == kGS ? 1.f : 0.f;
      if (sidx >= kGS) continue;
      const int kq = sidx < kGT - 2 ? 0 : (sidx < 2 * kGT - 6 ? 1 : 2);
      const int tp = sidx - (kq == 0 ? 0 : (kq == 1 ? kGT - 2 : 2 * kGT - 6)), Tg = kGT - 2 - 2 * kq;
      float* db = kq == 0 ? a.dconv[0] : (kq == 1 ? a.dconv[1] : a.dconv[2]);
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        float dp[4], dq[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dg = g[st][ct][r];
          const float th = gf_tanh(g4at(pv[st][ct], r)), sg = gf_sigmoid(g4at(qv[st][ct], r));
          dp[r] = dg * (1.f - th * th) * sg;
          dq[r] = dg * th * sg * (1.f - sg);
          gbv[st][ct][r] = th * sg;
        }
        float* row = db + (nb * Tg + tp) * (2 * kGC) + 16 * ct + 4 * lq;
        *reinterpret_cast<float4*>(row) = make_float4(dp[0], dp[1], dp[2], dp[3]);
        *reinterpret_cast<float4*>(row + kGC) = make_float4(dq[0], dq[1], dq[2], dq[3]);
      }
    }
    // dW_fcmy[t][s] += sum_c dtc[c][t] G[c][s]: k step kk = 4 ct + r contracts c = 16 ct + 4 lq + r
    // (the channels whose gates the lane holds); A[m = t][k = c] from the wave's transpose buffer
    // (its own LDS ops run in order; the fences keep the compiler from moving them)
    if (fw) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float av = i < kGT ? tt[(16 * ct + 4 * lq + r) * 13 + i] : 0.f;
#pragma unroll
          for (int st = 0; st < 2; ++st) accf[st] = gmf16(av, gbv[st][ct][r], accf[st]);
        }
      asm volatile("" ::: "memory");
    }
  }
  // the partial sums: over lq (xor 16, 32), then over the waves
#pragma unroll
  for (int q = 0; q < NS; ++q)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      float x = acc_s[q][v];
      x += __shfl_xor(x, 16, 64);
      x += __shfl_xor(x, 32, 64);
      if (lq == 0) red[(q * kGW + w) * kGC + 16 * v + i] = x;
    }
  if (fw) {  // D[4 lq + r][i] = dW_fcmy[t = 4 lq + r][s = 16 st + i]
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = 4 * lq + r, sidx = 16 * st + i;
        if (t < kGT && sidx <= kGS) redf[w * kGBF + t * (kGS + 1) + sidx] = accf[st][r];
      }
  }
  TF_MARK(1);
  __syncthreads();  // (also: every wave's gate-gradient rows are visible to the workgroup)
  TF_MARK(2);
  if (tid < NS * kGC) {
    const int q = tid / kGC, c = tid - q * kGC;
    float x = 0.f;
#pragma unroll
    for (int ww = 0; ww < kGW; ++ww) x += red[(q * kGW + ww) * kGC + c];
    gf_st_agent(a.part + (int64_t)blockIdx.x * kGBP + q * kGC + c, x);
  }
  if (tid < kGBF) {
    float x = 0.f;
#pragma unroll
    for (int ww = 0; ww < kGW; ++ww) x += redf[ww * kGBF + tid];
    gf_st_agent(a.part + (int64_t)blockIdx.x * kGBP + 4 * kGC + tid, x);
  }

  // ---- B. the transposed convolutions (each GTU's operands loaded during the previous one) ---
  {
    GbStage<0> st0;
    gb_load<0>(a, bn0, nn, st0);
    gb_store<0>(Ds, st0);
  }
  __syncthreads();
  GbStage<1> st1;
  gb_tconv<0>(nn, Ds, dXs, w, i, lq, [&]() { gb_load<1>(a, bn0, nn, st1); });
  gb_store<1>(Ds, st1);
  __syncthreads();
  TF_MARK(3);
  GbStage<2> st2;
  gb_tconv<1>(nn, Ds, dXs, w, i, lq, [&]() { gb_load<2>(a, bn0, nn, st2); });
  gb_store<2>(Ds, st2);
  __syncthreads();
  TF_MARK(4);
  // (the X rows of step C ride on the last GTU)
  constexpr int XV = (kGNB * kGCT / 4 + NT - 1) / NT;
  const int ne4 = nn * kGCT / 4;
  float4 xv[XV];
  gb_tconv<2>(nn, Ds, dXs, w, i, lq, [&]() {
    const float4* gx = reinterpret_cast<const float4*>(a.X + bn0 * kGCT);
#pragma unroll
    for (int u = 0; u < XV; ++u) xv[u] = gx[min(u * NT + tid, ne4 - 1)];
  });
  TF_MARK(5);

  // ---- C. gpre = (X > 0) ? dX : 0 -----------------------------------------------------------
  {
    float4* go = reinterpret_cast<float4*>(a.gpre + bn0 * kGCT);
#pragma unroll
    for (int u = 0; u < XV; ++u) {
      const int e4 = u * NT + tid;
      if (e4 >= ne4) continue;
      const int row = e4 / (kGC / 4), c = (e4 - row * (kGC / 4)) * 4;  // (n t, c)
      const float4 d = *reinterpret_cast<const float4*>(dXs + row * kGBX + c);
      go[e4] = make_float4(xv[u].x > 0.f ? d.x : 0.f, xv[u].y > 0.f ? d.y : 0.f, xv[u].z > 0.f ? d.z : 0.f,
                           xv[u].w > 0.f ? d.w : 0.f);
    }
  }
  TF_MARK(6);
  TF_PRINT("gtu_fused_bwd", 7);

  // ---- D. the parameter gradients: the last of each group of 16 workgroups sums the group's
  //         partial rows (agent-scope stores above, agent acquire here) into a level-2 row, the
  //         last group sums the level-2 rows in order: deterministic, no column-sum launches ---
  int* flag = reinterpret_cast<int*>(red);  // (red is free after step A)
  const int nwg = (int)gridDim.x, ng = (nwg + kGBG1 - 1) / kGBG1, g1 = (int)blockIdx.x / kGBG1;
  const int gsz = min(kGBG1, nwg - g1 * kGBG1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int lg = atomicAdd(a.cnt + g1, 1) == gsz - 1;
    if (lg) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.cnt + g1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
    flag[0] = lg;
  }
  __syncthreads();
  if (!flag[0]) return;
  float* l2 = a.part + (int64_t)nwg * kGBP;  // level-2 rows [ng][P]
  for (int e = tid; e < kGBP; e += NT) {
    const float* src = a.part + (int64_t)g1 * kGBG1 * kGBP + e;
    float u[kGBG1];
#pragma unroll
    for (int k = 0; k < kGBG1; ++k) u[k] = k < gsz ? gf_ld_agent(src + (int64_t)k * kGBP) : 0.f;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < kGBG1; ++k) v += u[k];
    gf_st_agent(l2 + (int64_t)g1 * kGBP + e, v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int last2 = atomicAdd(a.cnt + ng, 1) == ng - 1;
    if (last2) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.cnt + ng, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    flag[1] = last2;
  }
  __syncthreads();
  if (!flag[1]) return;
  for (int e = tid; e < kGBP; e += NT) {
    float* out;
    int o;
    if (e < 4 * kGC) {
      const int q = e / kGC;
      out = q == 0 ? a.gout : (q == 1 ? a.bout : (q == 2 ? a.rwout : a.rbout));
      o = e - q * kGC;
    } else {
      const int f = e - 4 * kGC, t = f / (kGS + 1), sidx = f - t * (kGS + 1);
      out = sidx < kGS ? a.fwout : a.fbout;
      o = sidx < kGS ? t * kGS + sidx : t;
    }
    if (!out) continue;
    float v = 0.f;
    for (int k0 = 0; k0 < ng; k0 += kGBG1) {
      float u[kGBG1];
#pragma unroll
      for (int k = 0; k < kGBG1; ++k) u[k] = k0 + k < ng ? gf_ld_agent(l2 + (int64_t)(k0 + k) * kGBP + e) : 0.f;
#pragma unroll
      for (int k = 0; k < kGBG1; ++k) v += u[k];
    }
    out[o] = v;
  }
}

}  // namespace

bool gtu_fused_fwd_ok(int C, int T) {
  static const bool on = !getenv("DSTAGNN_GTU_FUSED") || atoi(getenv("DSTAGNN_GTU_FUSED")) != 0;  // default on
  return on && C == kGC && T == kGT;
}

int op_gtu_fused_fwd(const GtuFusedArgs& a, hipStream_t st) {
  if (!gtu_fused_fwd_ok(a.C, a.T) || a.BN <= 0 || a.BN * kGCT >= (1ll << 31)) {
    set_last_error("gtu_fused_fwd: unsupported shape");
    return DSTAGNN_E_SHAPE;
  }
  bool al = gf_al16(a.X) && gf_al16(a.x) && gf_al16(a.G) && gf_al16(a.tco) && gf_al16(a.r) && gf_al16(a.mu) &&
            gf_al16(a.rs) && gf_al16(a.out) && gf_al16(a.fcmy_b);
  for (int q = 0; q < 3; ++q) al = al && gf_al16(a.conv[q]) && gf_al16(a.wt[q]) && gf_al16(a.bias[q]);
  if (!al) {
    set_last_error("gtu_fused_fwd: operands must be 16-B aligned");
    return DSTAGNN_E_ARG;
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
  void* rec = gemm_prof_begin(flops, bytes, st, DSTAGNN_PROF_GTU_FUSED_FWD);
  hipLaunchKernelGGL(k, dim3((unsigned)cdiv64(a.BN, kGNB)), dim3(kGW * 64), lds, st, a);
  DS_CHECK_LAUNCH();
  gemm_prof_end(rec, st);
  return 0;
}

bool gtu_fused_bwd_ok(int C, int T) {
  static const bool on = !getenv("DSTAGNN_GTU_FUSED_BWD") || atoi(getenv("DSTAGNN_GTU_FUSED_BWD")) != 0;  // default on
  return on && C == kGC && T == kGT;
}
int64_t gtu_fused_bwd_part_floats(int64_t BN) {
  const int64_t nwg = cdiv64(BN, kGNB);
  return (nwg + cdiv64(nwg, kGBG1)) * kGBP;
}

int op_gtu_fused_bwd(const GtuFusedBwdArgs& a, hipStream_t st) {
  if (!gtu_fused_bwd_ok(a.C, a.T) || a.BN <= 0 || a.BN * kGCT >= (1ll << 31) || !a.part) {
    set_last_error("gtu_fused_bwd: unsupported shape or no partial-row workspace");
    return DSTAGNN_E_SHAPE;
  }
  bool al = gf_al16(a.dout) && gf_al16(a.r) && gf_al16(a.tco) && gf_al16(a.mu) && gf_al16(a.rs) && gf_al16(a.x) &&
            gf_al16(a.X) && gf_al16(a.dx) && gf_al16(a.gpre);
  for (int q = 0; q < 3; ++q) al = al && gf_al16(a.dconv[q]) && gf_al16(a.wf[q]);
  if (!al) {
    set_last_error("gtu_fused_bwd: operands must be 16-B aligned");
    return DSTAGNN_E_ARG;
  }
  using Kern = void (*)(GtuFusedBwdArgs);
  const Kern k = a.first ? gtu_bwd_fused_kernel<true> : gtu_bwd_fused_kernel<false>;
  const size_t lds = gtu_fused_bwd_lds();
  {
    static std::mutex mu;
    static std::set<Kern> done;
    std::lock_guard<std::mutex> lock(mu);
    if (!done.count(k)) {
      const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) { set_last_error(std::string("gtu_fused_bwd: ") + hipGetErrorString(e)); return (int)e; }
      done.insert(k);
    }
  }
  // the transposed convolutions' algorithmic FLOP (the GEMM family's accounting)
  const double flops = 2.0 * a.BN * (2.0 * kGC) * kGC * ((kGT - 2) * 3 + (kGT - 4) * 5 + (kGT - 6) * 7);
  const double bytes = 4.0 * a.BN * (kGCT * 7.0 + 2 * kGC * 24.0 * 3);
  GtuFusedBwdArgs b = a;
  const int64_t nwg = cdiv64(a.BN, kGNB);
  b.cnt = stream_counters(st, (int)(cdiv64(nwg, kGBG1) + 1));  // [ng] level-1 tickets, one level-2 ticket
  if (!b.cnt) {
    set_last_error("gtu_fused_bwd: no ticket counters");
    return DSTAGNN_E_ARG;
  }
  void* rec = gemm_prof_begin(flops, bytes, st, DSTAGNN_PROF_GTU_FUSED_BWD);
  hipLaunchKernelGGL(k, dim3((unsigned)nwg), dim3(kGW * 64), lds, st, b);
  DS_CHECK_LAUNCH();
  gemm_prof_end(rec, st);
  return 0;
}
