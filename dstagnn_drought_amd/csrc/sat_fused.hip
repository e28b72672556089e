// sat_fused.hip — the spatial-attention projection backward and the EmbedS LayerNorm backward
// as ONE kernel (model/DSTAGNN_my.py:62-63 W_Q' / W_K' and :233-234 EmbedS LN_D + dropout, by
// autograd).  Was two launches on the main stream: the dZd GEMM (dZd = dqk [W_Q'; W_K'],
// 5440 x 512 x 192 at PEMS08, 20 us) writing the (B N, D) gradient, and ln_bwd reading it back
// with u (16 us) — 22 MB of round trip and a second launch.  Here a workgroup of 8 waves owns 32
// rows (b, n) (two 16-row tiles: each weight fragment feeds both):
//   1. its 32 dqk rows staged in LDS (float4), the LayerNorm operands (u, gamma, mu, rstd) of
//      the wave's columns issued in the same round;
//   2. dZd = dqk W on the f32 matrix cores with the transposed weights (D, 2 KD) as the A
//      operand (param_prep kind 9): lane (i, lq) of d-tile dt ends with 4 consecutive columns
//      16 dt + 4 lq + r of rows i and 16 + i — wave w owns columns [64 w, 64 w + 64) of every row;
//   3. the LayerNorm backward in those registers (ln_bwd_kernel's arithmetic, the dropout keep
//      mask re-derived from the seed): the two row sums over D through lq shuffles + one LDS
//      round over the 8 waves; dY out as float4 runs;
//   4. per-workgroup partial rows of the gamma / beta / pre_conv-bias column sums (sum over the
//      32 rows by DPP row sums), reduced by the caller's column sums.
#include "common.hpp"
#include "ops.hpp"

namespace {

constexpr int kSbRT = 2, kSbRows = 16 * kSbRT, kSbW = 8, kSbD = 512, kSbK = 192;  // rows per workgroup, waves, D, 2 KD
constexpr int kSbDT = kSbD / 16 / kSbW;                          // d-tiles per wave (4)
constexpr int kSbKS = kSbK + 4;                                  // LDS row stride of the dqk tile

__device__ __forceinline__ floatx4 smf16(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float s4at(const float4& v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}
__device__ __forceinline__ float sb_row16_sum(float x) {  // sum over a DPP row of 16 lanes
  x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x4E, 0xF, 0xF, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x141, 0xF, 0xF, true));
  x += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0x140, 0xF, 0xF, true));
  return x;
}

__global__ __launch_bounds__(kSbW * 64, 1) void sat_ln_bwd_fused_kernel(SatLnBwdArgs a) {
  constexpr int NT = kSbW * 64;
  __shared__ float4 Qs4[kSbRows * kSbKS / 4];
  __shared__ float red[2][kSbW][kSbRows];
  float* Qs = reinterpret_cast<float*>(Qs4);
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), l = tid & 63, i = l & 15, lq = l >> 4;
  const int64_t r0 = (int64_t)blockIdx.x * kSbRows;
  const int nr = (int)min<int64_t>(kSbRows, a.R - r0);
  int64_t row[kSbRT];  // the lane's rows 16 rt + i (clamped rows: computed, never stored)
#pragma unroll
  for (int rt = 0; rt < kSbRT; ++rt) row[rt] = r0 + min(16 * rt + i, nr - 1);
  TF_DECL;
  TF_MARK(0);

  // ---- 1. one round of loads ------------------------------------------------------------------
  {
    constexpr int QV = kSbRows * kSbK / 4 / NT;  // 3 (+1: a guarded spare)
    float4 qv[QV + 1];
    const float4* src = reinterpret_cast<const float4*>(a.dqk + r0 * kSbK);
#pragma unroll
    for (int u = 0; u <= QV; ++u) qv[u] = src[min(u * NT + tid, nr * kSbK / 4 - 1)];
#pragma unroll
    for (int u = 0; u <= QV; ++u) {
      const int e4 = u * NT + tid, rr = e4 / (kSbK / 4), c4 = e4 - rr * (kSbK / 4);
      if (e4 < kSbRows * kSbK / 4) *reinterpret_cast<float4*>(Qs + rr * kSbKS + 4 * c4) = qv[u];
    }
  }
  float4 uv[kSbRT][kSbDT], gv[kSbDT];
  float mean[kSbRT], rs[kSbRT];
#pragma unroll
  for (int t = 0; t < kSbDT; ++t) {
    const int d0 = 16 * (kSbDT * w + t) + 4 * lq;
    gv[t] = *reinterpret_cast<const float4*>(a.g + d0);
#pragma unroll
    for (int rt = 0; rt < kSbRT; ++rt) uv[rt][t] = *reinterpret_cast<const float4*>(a.u + row[rt] * kSbD + d0);
  }
#pragma unroll
  for (int rt = 0; rt < kSbRT; ++rt) {
    mean[rt] = a.mu[row[rt]];
    rs[rt] = a.rs[row[rt]];
  }
  __syncthreads();
  TF_MARK(1);

  // ---- 2. dZd[row i][d] = sum_k dqk[i][k] W[k][d]: A[m = d][k] = WT[d][k], B[k][n = i] --------
  floatx4 acc[kSbRT][kSbDT];
#pragma unroll
  for (int rt = 0; rt < kSbRT; ++rt)
#pragma unroll
    for (int t = 0; t < kSbDT; ++t) acc[rt][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float* brow = Qs + i * kSbKS + 4 * lq;  // + 16 rt rows per row tile
  const float* wrow = a.wT + (int64_t)(16 * kSbDT * w + i) * kSbK + 4 * lq;  // + 16 t rows per d-tile
  float4 ap[2][kSbDT], bp[2][kSbRT];
  auto frag = [&](int ch, int buf) {
#pragma unroll
    for (int rt = 0; rt < kSbRT; ++rt) bp[buf][rt] = *reinterpret_cast<const float4*>(brow + 16 * rt * kSbKS + 16 * ch);
#pragma unroll
    for (int t = 0; t < kSbDT; ++t) ap[buf][t] = *reinterpret_cast<const float4*>(wrow + 16 * t * kSbK + 16 * ch);
  };
  // the dropout keep bits of the lane's 32 elements (bit 16 rt + 4 t + r), hashed between the
  // matrix-core instructions of the k loop (drop_scale's hash and threshold; its multiplies
  // are quarter rate: after the loop they cost more than the product itself)
  constexpr int NE = kSbRT * kSbDT * 4, NCH = kSbK / 16, PER = (NE + NCH - 1) / NCH;
  uint32_t keep = 0;
  const bool drop = a.drop_p > 0.f;
  const DropKey dk = drop_key(a.seed, 0);  // which = 0
  auto hash = [&](int k) {
    const int rt = k >> 4, t = (k >> 2) & 3, r = k & 3;
    const uint64_t idx = (uint64_t)row[rt] * kSbD + 16 * (kSbDT * w + t) + 4 * lq + r + a.drop_off;
    keep |= (drop_u(dk, idx) >= a.drop_p ? 1u : 0u) << k;
  };
  frag(0, 0);
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    if (ch + 1 < NCH) frag(ch + 1, (ch + 1) & 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int rt = 0; rt < kSbRT; ++rt)
#pragma unroll
        for (int t = 0; t < kSbDT; ++t)
          acc[rt][t] = smf16(s4at(ap[ch & 1][t], s), s4at(bp[ch & 1][rt], s), acc[rt][t]);
    if (drop)
#pragma unroll
      for (int k = ch * PER; k < (ch + 1) * PER && k < NE; ++k) hash(k);
    __builtin_amdgcn_sched_barrier(0);
  }
  const float dscale = 1.0f / (1.0f - a.drop_p);
  TF_MARK(2);

  // ---- 3. LayerNorm(D) backward of rows i and 16 + i over the lane's 16 columns ---------------
  float dy[kSbRT][kSbDT][4], xh[kSbRT][kSbDT][4];
  float s1[kSbRT], s2[kSbRT];
#pragma unroll
  for (int rt = 0; rt < kSbRT; ++rt) {
    s1[rt] = s2[rt] = 0.f;
#pragma unroll
    for (int t = 0; t < kSbDT; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[rt][t][r];
        if (drop) v *= (keep >> (16 * rt + 4 * t + r)) & 1u ? dscale : 0.0f;
        dy[rt][t][r] = v;
        xh[rt][t][r] = (s4at(uv[rt][t], r) - mean[rt]) * rs[rt];
        const float dxh = v * s4at(gv[t], r);
        s1[rt] += dxh;
        s2[rt] += dxh * xh[rt][t][r];
      }
    }
    s1[rt] += __shfl_xor(s1[rt], 16, 64);
    s1[rt] += __shfl_xor(s1[rt], 32, 64);
    s2[rt] += __shfl_xor(s2[rt], 16, 64);
    s2[rt] += __shfl_xor(s2[rt], 32, 64);
    if (lq == 0) {
      red[0][w][16 * rt + i] = s1[rt];
      red[1][w][16 * rt + i] = s2[rt];
    }
  }
  TF_MARK(3);
  __syncthreads();
  TF_MARK(4);
#pragma unroll
  for (int rt = 0; rt < kSbRT; ++rt) {
    s1[rt] = 0.f;
    s2[rt] = 0.f;
#pragma unroll
    for (int ww = 0; ww < kSbW; ++ww) {  // (waves in order: every lane of the row, the same sums)
      s1[rt] += red[0][ww][16 * rt + i];
      s2[rt] += red[1][ww][16 * rt + i];
    }
    s1[rt] *= 1.f / kSbD;
    s2[rt] *= 1.f / kSbD;
  }
#pragma unroll
  for (int t = 0; t < kSbDT; ++t) {
    const int d0 = 16 * (kSbDT * w + t) + 4 * lq;
    float gp[4] = {0.f, 0.f, 0.f, 0.f}, bq[4] = {0.f, 0.f, 0.f, 0.f}, xp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int rt = 0; rt < kSbRT; ++rt) {
      const bool live = 16 * rt + i < nr;
      float dx[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dx[r] = rs[rt] * (dy[rt][t][r] * s4at(gv[t], r) - s1[rt] - xh[rt][t][r] * s2[rt]);
        if (live) {  // column partials over the workgroup's rows
          gp[r] += dy[rt][t][r] * xh[rt][t][r];
          bq[r] += dy[rt][t][r];
          xp[r] += dx[r];
        }
      }
      if (live) *reinterpret_cast<float4*>(a.dx + row[rt] * kSbD + d0) = make_float4(dx[0], dx[1], dx[2], dx[3]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      gp[r] = sb_row16_sum(gp[r]);
      bq[r] = sb_row16_sum(bq[r]);
      xp[r] = sb_row16_sum(xp[r]);
    }
    if (i == 0) {
      const int64_t po = (int64_t)blockIdx.x * kSbD + d0;
      *reinterpret_cast<float4*>(a.gpart + po) = make_float4(gp[0], gp[1], gp[2], gp[3]);
      *reinterpret_cast<float4*>(a.bpart + po) = make_float4(bq[0], bq[1], bq[2], bq[3]);
      if (a.xpart) *reinterpret_cast<float4*>(a.xpart + po) = make_float4(xp[0], xp[1], xp[2], xp[3]);
    }
  }
  TF_MARK(5);
  TF_PRINT("sat_ln_bwd", 6);
}

bool sb_al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

bool sat_ln_bwd_fused_ok(int64_t D, int64_t K2) {
  static const bool on = getenv("DSTAGNN_SATLN_FUSED") && atoi(getenv("DSTAGNN_SATLN_FUSED")) != 0;
  return on && D == kSbD && K2 == kSbK;
}
int64_t sat_ln_bwd_fused_wgs(int64_t R) { return cdiv64(R, kSbRows); }

int op_sat_ln_bwd_fused(const SatLnBwdArgs& a, hipStream_t st) {
  if (!sat_ln_bwd_fused_ok(a.D, a.K2) || a.R <= 0 || !a.dqk || !a.wT || !a.u || !a.mu || !a.rs || !a.g || !a.dx ||
      !a.gpart || !a.bpart) {
    set_last_error("sat_ln_bwd_fused: unsupported shape or missing operand");
    return DSTAGNN_E_SHAPE;
  }
  if (!(sb_al16(a.dqk) && sb_al16(a.wT) && sb_al16(a.u) && sb_al16(a.g) && sb_al16(a.dx) && sb_al16(a.gpart) &&
        sb_al16(a.bpart) && sb_al16(a.xpart))) {
    set_last_error("sat_ln_bwd_fused: operands must be 16-B aligned");
    return DSTAGNN_E_ARG;
  }
  const double flops = 2.0 * a.R * kSbD * kSbK;
  const double bytes = 4.0 * ((double)a.R * (kSbK + 2.0 * kSbD) + (double)kSbD * kSbK);
  void* rec = gemm_prof_begin(flops, bytes, st, DSTAGNN_PROF_SAT_FUSED);
  hipLaunchKernelGGL(sat_ln_bwd_fused_kernel, dim3((unsigned)cdiv64(a.R, kSbRows)), dim3(kSbW * 64), 0, st, a);
  DS_CHECK_LAUNCH();
  gemm_prof_end(rec, st);
  return 0;
}
