// tat_fused.hip — the temporal-attention stage as ONE kernel per direction.
//
// MultiHeadAttention.forward + the block's LN over N (model/DSTAGNN_my.py:84-100 with :30-42):
//   Q | K | V = E W_{Q,K,V}^T        (rows (b,f,t), contraction over the N nodes)
//   S = Q K^T / sqrt(dk) + res_att   -> re_At;  A = softmax over the query axis (quirk 1)
//   ctx = A V;  O = LN_N(ctx W_fc^T + E)
// was five launches (x transpose, Q|K|V GEMM, tat_fwd_mfma, fc GEMM, LayerNorm) with the
// (B,F,T,3h dk), (B,F,T,N) tensors round-tripping HBM between them and a ~9.6 us fixed cost per
// GEMM call on the main chain.  Here a workgroup owns 48 consecutive rows (b,f,t) — 48/T whole
// (b,f) problems — and keeps every intermediate in LDS:
//   1. E tile (48 x N, zero-padded to NP = 16 ceil(N/16)) from x (B,N,F,T) in place (inner
//      block: the rows of one node are 48 contiguous floats) or from the EmbedT output E;
//   2. Q | K | V = E Wqkv^T on the f32 matrix cores (v_mfma_f32_16x16x4_f32, 3 row tiles x the
//      wave's 16-column tiles, contraction index 16 c + 4 q + s: one float4 per lane per operand
//      and chunk; Wqkv re-laid (QW, NP) zero-padded by param_prep, streamed from L2);
//   3. per (problem, head): tat_fwd_mfma's register-resident attention on the LDS tile;
//   4. u = ctx W_fc^T + E accumulated in the E tile in place;
//   5. LayerNorm over N per row, writing u / mu / rs (saved for the backward) and O in its
//      [(f,t)][(b,n)] order.
// The saved tensors are the unfused path's (qkv, att, ctx, u, mu, rs; re_At and O are outputs),
// so the backward is unchanged — except that the inner block's x transpose E is never written
// (the Q|K|V weight gradient reads x through its index maps instead).
#include <mutex>
#include <set>

#include "common.hpp"
#include "ops.hpp"

namespace {

constexpr int kTfRows = 48;   // rows (b,f,t) per workgroup
constexpr int kTfD = 32;      // d_k = d_v
constexpr int kTfH = 3;       // heads (PEMS04 / PEMS08)
constexpr int kTfQW = 3 * kTfH * kTfD;  // 288
constexpr int kTfHV = kTfH * kTfD;      // 96
constexpr int kTfLQ = kTfQW + 4;        // LDS row stride of the Q|K|V tile
constexpr int kTfLC = kTfHV + 4;        // ... of the ctx tile
constexpr int kTfQT = kTfQW / 16;       // 18 column tiles of Q|K|V
constexpr int kTfQTW = (kTfQT + 3) / 4; // 5 per wave (the last of waves 2, 3 is a discarded duplicate)
constexpr int kTfNmax = 320;            // N <= 320 (LDS: E tile + Q|K|V tile + ctx tile <= 133 KB)

__device__ __forceinline__ floatx4 mf16(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float xmax16(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  v = fmaxf(v, __shfl_xor(v, 4, 64));
  return fmaxf(v, __shfl_xor(v, 8, 64));
}
__device__ __forceinline__ float xsum16(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v + __shfl_xor(v, 8, 64);
}
__device__ __forceinline__ float f4at(const float4& v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}

// row R of the (B F T) x N input E: src[(R % FT) s0 + (R / FT) s1 + n sN]  (R, FT < 2^31: the
// host checks; 32-bit division — a 64-bit one is a ~200-instruction software routine)
__device__ __forceinline__ int64_t tf_row(const TatFusedArgs& a, int64_t R) {
  const uint32_t r = (uint32_t)R, ft = (uint32_t)a.FT, b = r / ft;
  return (int64_t)(r - b * ft) * a.s0 + (int64_t)b * a.s1;
}
// the Q|K|V product's k loop step: A fragments of chunk c from the E tile, B fragments bq
template <int NJ>
__device__ __forceinline__ void tf_qkv_step(floatx4 (&acc)[3][NJ], const float* Es, int LE, int c, int i, int q,
                                            const float4 (&bq)[NJ]) {
  float4 av[3];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) av[mt] = *reinterpret_cast<const float4*>(Es + (mt * 16 + i) * LE + 16 * c + 4 * q);
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[mt][j] = mf16(f4at(av[mt], s), f4at(bq[j], s), acc[mt][j]);
}
template <int NJ>
__device__ __forceinline__ void tf_load_b(float4 (&b)[NJ], const float* const (&wp)[NJ], int off) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const float4*>(wp[j] + off);
}
// 3 x NJ tiles of (48 x 16 NJ) += A (48 x 16 NC, LDS, row stride LA) B (16 NC x 16 NJ, global
// rows wp[j] + 16 c), the B fragments double-buffered (ping-pong: no register copies, so the
// loads of chunk c + 1 stay in flight while chunk c is multiplied)
template <int NJ>
__device__ __forceinline__ void tf_gemm_rows48(floatx4 (&acc)[3][NJ], const float* A, int LA, int NC, int i, int q,
                                               const float* const (&wp)[NJ]) {
  // (sched_barrier: the scheduler otherwise sinks each chunk's loads to just before their use)
  float4 b0[NJ], b1[NJ];
  tf_load_b(b0, wp, 0);
  int c = 0;
  for (; c + 1 < NC; c += 2) {
    tf_load_b(b1, wp, 16 * (c + 1));
    __builtin_amdgcn_sched_barrier(0);
    tf_qkv_step(acc, A, LA, c, i, q, b0);
    __builtin_amdgcn_sched_barrier(0);
    tf_load_b(b0, wp, 16 * min(c + 2, NC - 1));
    __builtin_amdgcn_sched_barrier(0);
    tf_qkv_step(acc, A, LA, c + 1, i, q, b1);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (c < NC) tf_qkv_step(acc, A, LA, c, i, q, b0);
}

// E tile (48 x NP, zero-padded) into LDS.  Every load of a thread is issued before its first
// LDS store (one memory round trip, not one per element).  x (B,N,F,T) with the workgroup's 48
// rows inside one sample: a node's 48 values are contiguous — float4 per lane; otherwise (E
// row-major, first block) scalar loads along the nodes.
__device__ __forceinline__ void tf_load_e_tile(const float* src, const TatFusedArgs& a, int64_t R0, int nrows,
                                               float* Es, int LE, int NP, int N, int tid) {
  const uint32_t ft0 = (uint32_t)(R0 % a.FT);
  if (a.sN != 1 && a.s0 == 1 && nrows == kTfRows && ft0 + kTfRows <= (uint32_t)a.FT) {
    const float* base = src + tf_row(a, R0);
    constexpr int Q4 = kTfRows / 4;  // 12 float4 per node
    const int total = N * Q4;
    for (int e0 = 0; e0 < total; e0 += 256 * 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = min(e0 + u * 256 + tid, total - 1);
        const int n = e / Q4, c4 = e - n * Q4;
        v[u] = *reinterpret_cast<const float4*>(base + (int64_t)n * a.sN + 4 * c4);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * 256 + tid;
        if (e < total) {
          const int n = e / Q4, r = 4 * (e - n * Q4);
          Es[r * LE + n] = v[u].x;
          Es[(r + 1) * LE + n] = v[u].y;
          Es[(r + 2) * LE + n] = v[u].z;
          Es[(r + 3) * LE + n] = v[u].w;
        }
      }
    }
    for (int e = tid; e < kTfRows * (NP - N); e += 256) {  // pad columns
      const int r = e / (NP - N), n = N + e - r * (NP - N);
      Es[r * LE + n] = 0.f;
    }
    return;
  }
  int64_t* roff = reinterpret_cast<int64_t*>(Es + kTfRows * LE) ;  // (scratch: the Q|K|V tile region)
  if (tid < kTfRows) roff[tid] = tf_row(a, R0 + min(tid, max(nrows - 1, 0)));
  __syncthreads();
  const int total = kTfRows * NP;
  for (int e0 = 0; e0 < total; e0 += 256 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * 256 + tid;
      int r, n;
      if (a.sN == 1) { r = e / NP; n = e - r * NP; }
      else { n = e / kTfRows; r = e - n * kTfRows; }
      const bool ok = e < total && r < nrows && n < N;
      v[u] = ok ? src[roff[min(r, kTfRows - 1)] + (int64_t)min(n, N - 1) * a.sN] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * 256 + tid;
      if (e < total) {
        int r, n;
        if (a.sN == 1) { r = e / NP; n = e - r * NP; }
        else { n = e / kTfRows; r = e - n * kTfRows; }
        Es[r * LE + n] = v[u];
      }
    }
  }
  __syncthreads();  // (roff is overwritten by the Q|K|V tile later)
}

template <int T, int NTW>
__global__ __launch_bounds__(256, 1) void tat_fused_fwd_kernel(TatFusedArgs a) {
  static_assert(T % 4 == 0 && T <= 16 && kTfRows % T == 0, "whole problems per workgroup, one 16 x 16 tile");
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int NP = a.NP, LE = NP + 4, N = a.N;
  float* Es = lds;                       // [48][LE]   E, then u = fc + E
  float* Qs = Es + kTfRows * LE;         // [48][kTfLQ] Q | K | V
  float* Cs = Qs + kTfRows * kTfLQ;      // [48][kTfLC] ctx
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, i = l & 15, q = l >> 4;
  const int64_t R0 = (int64_t)blockIdx.x * kTfRows;
  const int nrows = (int)min<int64_t>(kTfRows, a.BFT - R0);
  stream_sig_store(a.sig, a.sig_v);

  // ---- 1. E tile --------------------------------------------------------------------------
  tf_load_e_tile(a.src, a, R0, nrows, Es, LE, NP, N, tid);
  __syncthreads();

  // ---- 2. Q | K | V = E Wqkv^T ------------------------------------------------------------
  {
    floatx4 acc[3][kTfQTW];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int j = 0; j < kTfQTW; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* wp[kTfQTW];
#pragma unroll
    for (int j = 0; j < kTfQTW; ++j) wp[j] = a.wqkv + (int64_t)(min(w + 4 * j, kTfQT - 1) * 16 + i) * NP + 4 * q;
    tf_gemm_rows48(acc, Es, LE, NP / 16, i, q, wp);
    // D[4q + r][i] of tile (mt, nt)
#pragma unroll
    for (int j = 0; j < kTfQTW; ++j) {
      const int nt = w + 4 * j;
      if (nt < kTfQT) {
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) Qs[(mt * 16 + 4 * q + r) * kTfLQ + nt * 16 + i] = acc[mt][j][r];
      }
    }
  }
  __syncthreads();

  // ---- 3. attention per (problem, head) (tat_fwd_mfma_kernel's math, operands from LDS) ----
  constexpr int PW = kTfRows / T;  // problems per workgroup
  for (int task = w; task < PW * kTfH; task += 4) {
    const int p = task / kTfH, hd = task - p * kTfH;
    const int rb = p * T;
    if (rb >= nrows) continue;  // (wave-uniform)
    const int64_t P = R0 / T + p;  // global problem (b, f)
    const int64_t b = P / a.F;
    const float* Qp = Qs + rb * kTfLQ + hd * kTfD;
    const float* Kp = Qp + kTfHV;
    const float* Vp = Qp + 2 * kTfHV;
    const int c = i;
    const bool vi = c < T, vj = q < T / 4;
    float vv[2][4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) vv[t][s] = (4 * q + s < T) ? Vp[(4 * q + s) * kTfLQ + c + 16 * t] : 0.f;
    float4 k0 = {0.f, 0.f, 0.f, 0.f}, k1 = k0, q0 = k0, q1 = k0;
    if (vi) {
      k0 = *reinterpret_cast<const float4*>(Kp + c * kTfLQ + 8 * q);
      k1 = *reinterpret_cast<const float4*>(Kp + c * kTfLQ + 8 * q + 4);
      q0 = *reinterpret_cast<const float4*>(Qp + c * kTfLQ + 8 * q);
      q1 = *reinterpret_cast<const float4*>(Qp + c * kTfLQ + 8 * q + 4);
    }
    const int64_t sbase = (P * kTfH + hd) * T * T;
    const float* rp = nullptr;
    if (a.res_mode == DSTAGNN_RES_BCAST) rp = a.res + (b * kTfH + hd) * T * T;
    else if (a.res_mode == DSTAGNN_RES_FULL) rp = a.res + sbase;
    float4 rr = {0.f, 0.f, 0.f, 0.f};
    if (rp && vi && vj) rr = *reinterpret_cast<const float4*>(rp + c * T + 4 * q);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = mf16(k0.x, q0.x, acc);
    acc = mf16(k0.y, q0.y, acc);
    acc = mf16(k0.z, q0.z, acc);
    acc = mf16(k0.w, q0.w, acc);
    acc = mf16(k1.x, q1.x, acc);
    acc = mf16(k1.y, q1.y, acc);
    acc = mf16(k1.z, q1.z, acc);
    acc = mf16(k1.w, q1.w, acc);
    const float rv[4] = {rr.x, rr.y, rr.z, rr.w};
    float sc[4], pr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sc[r] = acc[r] * a.scale;
      sc[r] += rv[r];
    }
    if (vi && vj) *reinterpret_cast<float4*>(a.re_at + sbase + c * T + 4 * q) = make_float4(sc[0], sc[1], sc[2], sc[3]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float m = xmax16(vi ? sc[r] : -INFINITY);
      const float e = vi ? __expf(sc[r] - m) : 0.f;
      const float inv = 1.f / xsum16(e);
      pr[r] = vj ? e * inv : 0.f;
    }
    if (vi && vj) *reinterpret_cast<float4*>(a.att + sbase + c * T + 4 * q) = make_float4(pr[0], pr[1], pr[2], pr[3]);
    floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      c0 = mf16(pr[s], vv[0][s], c0);
      c1 = mf16(pr[s], vv[1][s], c1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = 4 * q + r;
      if (ii < T) {
        Cs[(rb + ii) * kTfLC + hd * kTfD + c] = c0[r];
        Cs[(rb + ii) * kTfLC + hd * kTfD + c + 16] = c1[r];
      }
    }
  }
  __syncthreads();

  // saved Q | K | V and ctx: the workgroup's rows are contiguous in both (coalesced float4)
  {
    float4* gq = reinterpret_cast<float4*>(a.qkv + R0 * kTfQW);
    for (int e = tid; e < nrows * (kTfQW / 4); e += 256) {
      const int r = e / (kTfQW / 4), c4 = e - r * (kTfQW / 4);
      gq[e] = *reinterpret_cast<const float4*>(Qs + r * kTfLQ + 4 * c4);
    }
    float4* gc = reinterpret_cast<float4*>(a.ctx + R0 * kTfHV);
    for (int e = tid; e < nrows * (kTfHV / 4); e += 256) {
      const int r = e / (kTfHV / 4), c4 = e - r * (kTfHV / 4);
      gc[e] = *reinterpret_cast<const float4*>(Cs + r * kTfLC + 4 * c4);
    }
  }

  // ---- 4. u = ctx W_fc^T + E, in the E tile -------------------------------------------------
  {
    const int NT = NP / 16;
    floatx4 acc[3][NTW];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* wp[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) wp[j] = a.wfc + (int64_t)min(min(w + 4 * j, NT - 1) * 16 + i, N - 1) * kTfHV + 4 * q;
    tf_gemm_rows48(acc, Cs, kTfLC, kTfHV / 16, i, q, wp);
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int nt = w + 4 * j;
      if (nt < NT) {
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* e = Es + (mt * 16 + 4 * q + r) * LE + nt * 16 + i;
            *e = acc[mt][j][r] + *e;  // (pad columns: garbage + 0, never read)
          }
      }
    }
  }
  __syncthreads();

  // ---- 5. LayerNorm over N per row (ln_fwd_kernel's two-pass statistics) ---------------------
  constexpr int VPT = (kTfNmax + 63) / 64;
  for (int r = w; r < nrows; r += 4) {
    const int64_t R = R0 + r;
    const float* row = Es + r * LE;
    float v[VPT];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int n = l + 64 * k;
      v[k] = n < N ? row[n] : 0.f;
      sum += v[k];
    }
    const float mean = wave_sum(sum) / N;
    float var = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int n = l + 64 * k;
      if (n < N) {
        const float d = v[k] - mean;
        var += d * d;
      }
    }
    var = wave_sum(var) / N;
    const float rs = rsqrtf(var + a.eps);
    if (l == 0) {
      a.mu[R] = mean;
      a.rs[R] = rs;
    }
    const uint32_t bb = (uint32_t)R / (uint32_t)a.FT, ft = (uint32_t)R - bb * (uint32_t)a.FT;
    float* orow = a.O + (int64_t)ft * a.BN + (int64_t)bb * N;
    float* urow = a.u + R * N;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int n = l + 64 * k;
      if (n < N) {
        urow[n] = v[k];
        orow[n] = (v[k] - mean) * rs * a.g[n] + a.bta[n];
      }
    }
  }
}

// =====================================================================================
// Backward: LN_N backward -> dctx = dU W_fc -> attention backward -> dE = dU + dqkv Wqkv,
// accumulated straight into dx (inner block: dx[b, n, ft] is x's layout, so the four rows a
// lane's accumulator holds for one node are one float4) or written as dE (first block: the
// EmbedT LayerNorm backward follows).  Was: ln_bwd, dctx GEMM, tat_bwd_mfma, dE GEMM, transpose.
// Saved for the weight gradients (issued after it): dU (fc) and dqkv (Q|K|V); the LayerNorm's
// gamma / beta as one partial row per workgroup; the broadcast res_att gradient sum_f dS folded
// in-kernel (fixed chunk order, tat_bwd_mfma's ticket hand-off).
// =====================================================================================
__device__ __forceinline__ float tf_ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void tf_st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void tf_wave_sync() {  // LDS hand-off inside one wave
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
constexpr int kTfDsMax = 2304;  // (48 / T) * h * T * T floats at T = 16, h = 3

template <int T, int NTW>
__global__ __launch_bounds__(256, 1) void tat_fused_bwd_kernel(TatFusedBwdArgs a) {
  static_assert(T % 4 == 0 && T <= 16 && kTfRows % T == 0, "whole problems per workgroup, one 16 x 16 tile");
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int NP = a.NP, LE = NP + 4, N = a.N;
  float* DUs = lds;                        // [48][LE]    dU
  float* Qs = DUs + kTfRows * LE;          // [48][kTfLQ] Q | K | V, then dQ | dK | dV in place
  float* Cs = Qs + kTfRows * kTfLQ;        // [48][kTfLC] dctx (phase A: gamma / beta partials)
  float* TRs = Cs + kTfRows * kTfLC;       // [4][16][17] per-wave dS transpose
  float* DSs = TRs + 4 * 16 * 17;          // [48/T][h][T*T] dS tiles (broadcast res_att)
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, i = l & 15, q = l >> 4;
  const int64_t R0 = (int64_t)blockIdx.x * kTfRows;
  const int nrows = (int)min<int64_t>(kTfRows, a.BFT - R0);
  stream_sig_store(a.sig, a.sig_v);

  // ---- A0. saved Q | K | V rows (contiguous) -> LDS -----------------------------------------
  {
    const float4* gq = reinterpret_cast<const float4*>(a.qkv + R0 * kTfQW);
    for (int e = tid; e < nrows * (kTfQW / 4); e += 256) {
      const int r = e / (kTfQW / 4), c4 = e - r * (kTfQW / 4);
      *reinterpret_cast<float4*>(Qs + r * kTfLQ + 4 * c4) = gq[e];
    }
  }
  // ---- A1. LayerNorm(N) backward (ln_bwd_kernel's arithmetic), wave per row ----------------
  constexpr int VPT = (kTfNmax + 63) / 64;
  float gp[VPT], bp[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) { gp[k] = 0.f; bp[k] = 0.f; }
  for (int r = w; r < kTfRows; r += 4) {
    float* dur = DUs + r * LE;
    if (r >= nrows) {  // rows past the end: zeros (they only feed discarded output rows)
      for (int n = l; n < NP; n += 64) dur[n] = 0.f;
      continue;
    }
    const int64_t R = R0 + r;
    const uint32_t bb = (uint32_t)R / (uint32_t)a.FT, ft = (uint32_t)R - bb * (uint32_t)a.FT;
    const float* dyr = a.dO + (int64_t)ft * a.BN + (int64_t)bb * N;
    const float* ur = a.u + R * N;
    const float mean = a.mu[R], rsv = a.rs[R];
    float dyv[VPT], xh[VPT], gl[VPT];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int n = l + 64 * k;
      const int e = min(n, N - 1);
      const float dy = dyr[e], uu = ur[e], gg = a.g[e];
      const bool ok = n < N;
      dyv[k] = ok ? dy : 0.f;
      xh[k] = ok ? (uu - mean) * rsv : 0.f;
      gl[k] = ok ? gg : 0.f;
      const float dxh = dyv[k] * gl[k];
      s1 += dxh;
      s2 += dxh * xh[k];
      gp[k] += dyv[k] * xh[k];
      bp[k] += dyv[k];
    }
    s1 = wave_sum(s1) / N;
    s2 = wave_sum(s2) / N;
    float* gdu = a.dU + R * N;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int n = l + 64 * k;
      if (n < N) {
        const float du = rsv * (dyv[k] * gl[k] - s1 - xh[k] * s2);
        dur[n] = du;
        gdu[n] = du;
      } else if (n < NP) {
        dur[n] = 0.f;
      }
    }
  }
  {  // gamma / beta: one partial row per workgroup (four wave rows summed in wave order)
    float* red = Cs;  // [2][4][NP] (Cs is free until phase B's epilogue)
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int n = l + 64 * k;
      if (n < NP) {
        red[(0 * 4 + w) * NP + n] = gp[k];
        red[(1 * 4 + w) * NP + n] = bp[k];
      }
    }
    __syncthreads();
    for (int n = tid; n < N; n += 256) {
      if (a.gpart) a.gpart[(int64_t)blockIdx.x * N + n] = ((red[0 * NP + n] + red[1 * NP + n]) + red[2 * NP + n]) + red[3 * NP + n];
      if (a.bpart) a.bpart[(int64_t)blockIdx.x * N + n] = ((red[4 * NP + n] + red[5 * NP + n]) + red[6 * NP + n]) + red[7 * NP + n];
    }
    __syncthreads();
  }

  // ---- B. dctx = dU W_fc  (48 x h dv, contraction over the NP nodes) -----------------------
  {
    constexpr int CT = kTfHV / 16;          // 6 column tiles
    constexpr int NTL = 3 * CT;             // 18 (row, column) tiles
    constexpr int TPW = (NTL + 3) / 4;      // 5 per wave (the last of waves 2, 3: a duplicate)
    floatx4 acc[TPW];
    const float* wp[TPW];
    int arow[TPW];
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
      const int t = min(w + 4 * j, NTL - 1), mt = t / CT, nt = t - mt * CT;
      arow[j] = (mt * 16 + i) * LE + 4 * q;
      wp[j] = a.wfcT + (int64_t)(nt * 16 + i) * NP + 4 * q;
    }
    const int NC = NP / 16;
    auto step = [&](int c, const float4 (&bv)[TPW]) {
      float4 av[TPW];
#pragma unroll
      for (int j = 0; j < TPW; ++j) av[j] = *reinterpret_cast<const float4*>(DUs + arow[j] + 16 * c);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < TPW; ++j) acc[j] = mf16(f4at(av[j], s), f4at(bv[j], s), acc[j]);
    };
    float4 b0[TPW], b1[TPW];
    tf_load_b(b0, wp, 0);
    int c = 0;
    for (; c + 1 < NC; c += 2) {
      tf_load_b(b1, wp, 16 * (c + 1));
      __builtin_amdgcn_sched_barrier(0);
      step(c, b0);
      __builtin_amdgcn_sched_barrier(0);
      tf_load_b(b0, wp, 16 * min(c + 2, NC - 1));
      __builtin_amdgcn_sched_barrier(0);
      step(c + 1, b1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c < NC) step(c, b0);
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int t = w + 4 * j;
      if (t < NTL) {
        const int mt = t / CT, nt = t - mt * CT;
#pragma unroll
        for (int r = 0; r < 4; ++r) Cs[(mt * 16 + 4 * q + r) * kTfLC + nt * 16 + i] = acc[j][r];
      }
    }
  }
  __syncthreads();

  // ---- C. attention backward per (problem, head) (tat_bwd_mfma_kernel's math) ---------------
  constexpr int PW = kTfRows / T;
  for (int task = w; task < PW * kTfH; task += 4) {
    const int p = task / kTfH, hd = task - p * kTfH;
    const int rb = p * T;
    if (rb >= nrows) continue;  // (wave-uniform)
    const int64_t P = R0 / T + p;
    float* Qp = Qs + rb * kTfLQ + hd * kTfD;
    float* Kp = Qp + kTfHV;
    float* Vp = Qp + 2 * kTfHV;
    const float* Cp = Cs + rb * kTfLC + hd * kTfD;
    const int64_t sbase = (P * kTfH + hd) * T * T;
    const int c = i;
    const bool vj = c < T;
    float4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = d0, v0 = d0, v1 = d0;
    float cb[2][4], qb[2][4], kb[2][4], at[4], dr[4];
    if (vj) {
      d0 = *reinterpret_cast<const float4*>(Cp + c * kTfLC + 8 * q);
      d1 = *reinterpret_cast<const float4*>(Cp + c * kTfLC + 8 * q + 4);
      v0 = *reinterpret_cast<const float4*>(Vp + c * kTfLQ + 8 * q);
      v1 = *reinterpret_cast<const float4*>(Vp + c * kTfLQ + 8 * q + 4);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ii = 4 * q + s;
      const bool ok = ii < T;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        cb[t][s] = ok ? Cp[ii * kTfLC + c + 16 * t] : 0.f;
        qb[t][s] = ok ? Qp[ii * kTfLQ + c + 16 * t] : 0.f;
        kb[t][s] = ok ? Kp[ii * kTfLQ + c + 16 * t] : 0.f;
      }
      at[s] = ok && vj ? a.att[sbase + ii * T + c] : 0.f;
      dr[s] = ok && vj && a.dre ? a.dre[sbase + ii * T + c] : 0.f;
    }
    floatx4 dA = {0.f, 0.f, 0.f, 0.f};
    dA = mf16(d0.x, v0.x, dA);
    dA = mf16(d0.y, v0.y, dA);
    dA = mf16(d0.z, v0.z, dA);
    dA = mf16(d0.w, v0.w, dA);
    dA = mf16(d1.x, v1.x, dA);
    dA = mf16(d1.y, v1.y, dA);
    dA = mf16(d1.z, v1.z, dA);
    dA = mf16(d1.w, v1.w, dA);
    float cs = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) cs = fmaf(at[r], dA[r], cs);
    cs += __shfl_xor(cs, 16, 64);
    cs += __shfl_xor(cs, 32, 64);
    float ds[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ds[r] = at[r] * (dA[r] - cs) + dr[r];
    if (vj) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (4 * q + r >= T) continue;
        if (a.res_mode == DSTAGNN_RES_FULL && a.dres) a.dres[sbase + (4 * q + r) * T + c] = ds[r];
        else if (a.res_mode == DSTAGNN_RES_BCAST) DSs[(p * kTfH + hd) * T * T + (4 * q + r) * T + c] = ds[r];
      }
    }
    floatx4 z = {0.f, 0.f, 0.f, 0.f};
    floatx4 gv0 = z, gv1 = z, gk0 = z, gk1 = z, gq0 = z, gq1 = z;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      gv0 = mf16(at[s], cb[0][s], gv0);
      gv1 = mf16(at[s], cb[1][s], gv1);
      gk0 = mf16(ds[s], qb[0][s], gk0);
      gk1 = mf16(ds[s], qb[1][s], gk1);
    }
    float* tr = TRs + w * 16 * 17;
#pragma unroll
    for (int r = 0; r < 4; ++r) tr[(4 * q + r) * 17 + c] = ds[r];
    tf_wave_sync();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float xv = tr[c * 17 + 4 * q + s];
      gq0 = mf16(xv, kb[0][s], gq0);
      gq1 = mf16(xv, kb[1][s], gq1);
    }
    tf_wave_sync();  // (every lane's Q/K/V reads of this task precede the in-place writes below)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = 4 * q + r;
      if (ii >= T) continue;
      float* row = Qp + ii * kTfLQ + c;
      row[0] = gq0[r] * a.scale;
      row[16] = gq1[r] * a.scale;
      row[kTfHV] = gk0[r] * a.scale;
      row[kTfHV + 16] = gk1[r] * a.scale;
      row[2 * kTfHV] = gv0[r];
      row[2 * kTfHV + 16] = gv1[r];
    }
  }
  __syncthreads();

  // ---- D0. dqkv out (the Q|K|V weight gradient's operand); res_att partial per (b, chunk) ----
  {
    float4* gq = reinterpret_cast<float4*>(a.dqkv + R0 * kTfQW);
    for (int e = tid; e < nrows * (kTfQW / 4); e += 256) {
      const int r = e / (kTfQW / 4), c4 = e - r * (kTfQW / 4);
      gq[e] = *reinterpret_cast<const float4*>(Qs + r * kTfLQ + 4 * c4);
    }
  }
  const int nch = (int)(a.FT / kTfRows);
  const int64_t bwg = (uint32_t)R0 / (uint32_t)a.FT, chw = ((uint32_t)R0 - (uint32_t)bwg * (uint32_t)a.FT) / kTfRows;
  if (a.res_mode == DSTAGNN_RES_BCAST) {
    for (int e = tid; e < kTfH * T * T; e += 256) {
      float v = 0.f;
      for (int p = 0; p < PW; ++p) v += DSs[p * kTfH * T * T + e];  // problems in order
      tf_st_agent(a.dpart + (bwg * nch + chw) * kTfH * T * T + e, v);
    }
  }

  // ---- D1. dE = dU + dqkv [Wq; Wk; Wv] ---------------------------------------------------
  {
    const int NT = NP / 16;
    floatx4 acc[3][NTW];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int j = 0; j < NTW; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* wp[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) wp[j] = a.wqT + (int64_t)(min(w + 4 * j, NT - 1) * 16 + i) * kTfQW + 4 * q;
    tf_gemm_rows48(acc, Qs, kTfLQ, kTfQW / 16, i, q, wp);
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = (w + 4 * j) * 16 + i;
      if (w + 4 * j >= NT || n >= N) continue;
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) {
        const int r0 = mt * 16 + 4 * q;  // this lane's four consecutive rows
        if (r0 >= nrows) continue;       // (nrows is a multiple of T, so of 4)
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[mt][j][r] + DUs[(r0 + r) * LE + n];
        const int64_t R = R0 + r0;
        if (a.dx) {  // inner block: rows R..R+3 are four consecutive ft of one b (FT % 4 == 0)
          const uint32_t bb = (uint32_t)R / (uint32_t)a.FT, ft = (uint32_t)R - bb * (uint32_t)a.FT;
          float4* dp = reinterpret_cast<float4*>(a.dx + (int64_t)bb * a.dxb + (int64_t)n * a.FT + ft);
          float4 o = *dp;
          o.x += v[0]; o.y += v[1]; o.z += v[2]; o.w += v[3];
          *dp = o;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) a.dE[(R + r) * N + n] = v[r];
        }
      }
    }
  }

  // ---- D2. broadcast res_att gradient: the last workgroup of each b sums the chunks in order --
  if (a.res_mode == DSTAGNN_RES_BCAST) {
    int& last = *reinterpret_cast<int*>(DSs + kTfDsMax);  // (no static __shared__: it would shift the dynamic base)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      last = atomicAdd(a.cnt + bwg, 1) == nch - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(a.cnt + bwg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
      }
    }
    __syncthreads();
    if (!last) return;
    for (int e = tid; e < kTfH * T * T; e += 256) {
      float v = 0.f;
      for (int ch = 0; ch < nch; ++ch) v += tf_ld_agent(a.dpart + (bwg * nch + ch) * kTfH * T * T + e);
      a.dres[bwg * kTfH * T * T + e] = v;
    }
  }
}

size_t tat_fused_bwd_lds(int NP) {
  return sizeof(float) * ((size_t)kTfRows * (NP + 4) + (size_t)kTfRows * kTfLQ + (size_t)kTfRows * kTfLC + 4 * 16 * 17 +
                          kTfDsMax + 4);
}

size_t tat_fused_lds(int NP) {
  return sizeof(float) * ((size_t)kTfRows * (NP + 4) + (size_t)kTfRows * kTfLQ + (size_t)kTfRows * kTfLC);
}

}  // namespace

bool tat_fused_fwd_ok(int N, int T, int h, int dk, int dv) {
  // DSTAGNN_TAT_FUSED=0 (or DSTAGNN_TAT_MFMA=0, the VALU attention A/B): the unfused launches
  static const bool env = (!getenv("DSTAGNN_TAT_FUSED") || atoi(getenv("DSTAGNN_TAT_FUSED")) != 0) &&
                          (!getenv("DSTAGNN_TAT_MFMA") || atoi(getenv("DSTAGNN_TAT_MFMA")) != 0);
  return env && h == kTfH && dk == kTfD && dv == kTfD && N >= 1 && N <= kTfNmax &&
         (T == 4 || T == 8 || T == 12 || T == 16);
}

int tat_fused_np(int N) { return (N + 15) / 16 * 16; }

int op_tat_fused_fwd(const TatFusedArgs& a0, hipStream_t st) {
  if (!tat_fused_fwd_ok(a0.N, a0.T, a0.h, kTfD, kTfD) || a0.NP != tat_fused_np(a0.N) || a0.BFT % a0.T != 0) {
    set_last_error("tat_fused_fwd: unsupported shape");
    return DSTAGNN_E_SHAPE;
  }
  TatFusedArgs a = a0;
  const StreamSig sg = peek_stream_sig(st);
  a.sig = sg.p;
  a.sig_v = sg.v;
  const int64_t grid = cdiv64(a.BFT, kTfRows);
  const size_t lds = tat_fused_lds(a.NP);
  const int ntw = (a.NP / 16 + 3) / 4;  // fc column tiles per wave
  // algorithmic FLOP of the two products (the GEMM family's accounting) + the attention
  const double flops = 2.0 * a.BFT * (double)kTfQW * a.N + 2.0 * a.BFT * (double)a.N * kTfHV +
                       4.0 * (a.BFT / a.T) * kTfH * (double)a.T * a.T * kTfD;
  const double bytes = 4.0 * a.BFT * (a.N + kTfQW + kTfHV + 2.0 * a.N + 2.0 * kTfH * a.T) + 4.0 * kTfQW * a.NP;
  using Kern = void (*)(TatFusedArgs);
  Kern k = nullptr;
#define TF_T(TT)                                          \
  switch (ntw) {                                          \
    case 1: k = tat_fused_fwd_kernel<TT, 1>; break;       \
    case 2: k = tat_fused_fwd_kernel<TT, 2>; break;       \
    case 3: k = tat_fused_fwd_kernel<TT, 3>; break;       \
    case 4: k = tat_fused_fwd_kernel<TT, 4>; break;       \
    default: k = tat_fused_fwd_kernel<TT, 5>; break;      \
  }                                                       \
  break;
  switch (a.T) {
    case 4: TF_T(4)
    case 8: TF_T(8)
    case 12: TF_T(12)
    default: TF_T(16)
  }
#undef TF_T
  if (lds > 64 * 1024) {  // once per instantiation: dynamic LDS above 64 KB needs the opt-in
    static std::mutex mu;
    static std::set<Kern> done;
    std::lock_guard<std::mutex> lock(mu);
    if (!done.count(k)) {
      const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) { set_last_error(std::string("tat_fused_fwd: ") + hipGetErrorString(e)); return (int)e; }
      done.insert(k);
    }
  }
  void* rec = gemm_prof_begin(flops, bytes, st);
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), lds, st, a);
  DS_CHECK_LAUNCH();
  if (sg.p) DS_TRY(stream_sig_sent(st, sg));
  gemm_prof_end(rec, st);
  return 0;
}

bool tat_fused_bwd_ok(int N, int T, int h, int dk, int dv, int F, int res_mode) {
  static const bool env = !getenv("DSTAGNN_TAT_FUSED_BWD") || atoi(getenv("DSTAGNN_TAT_FUSED_BWD")) != 0;
  if (!env || !tat_fused_fwd_ok(N, T, h, dk, dv)) return false;
  // the in-kernel res_att fold needs whole workgroups per sample
  return res_mode != DSTAGNN_RES_BCAST || ((int64_t)F * T) % kTfRows == 0;
}

int op_tat_fused_bwd(const TatFusedBwdArgs& a0, hipStream_t st) {
  if (!tat_fused_bwd_ok(a0.N, a0.T, a0.h, kTfD, kTfD, a0.F, a0.res_mode) || a0.NP != tat_fused_np(a0.N) ||
      a0.BFT % a0.T != 0 || a0.FT % 4 != 0 || (!a0.dx && !a0.dE)) {
    set_last_error("tat_fused_bwd: unsupported shape");
    return DSTAGNN_E_SHAPE;
  }
  TatFusedBwdArgs a = a0;
  if (a.res_mode == DSTAGNN_RES_BCAST) {
    if (!a.dres) {
      a.res_mode = DSTAGNN_RES_NONE;  // nothing to fold
    } else {
      a.cnt = stream_counters(st, (int)(a.BFT / a.FT));
      if (!a.cnt || !a.dpart) { set_last_error("tat_fused_bwd: no ticket counters"); return DSTAGNN_E_ARG; }
    }
  }
  const StreamSig sg = peek_stream_sig(st);
  a.sig = sg.p;
  a.sig_v = sg.v;
  const int64_t grid = cdiv64(a.BFT, kTfRows);
  const size_t lds = tat_fused_bwd_lds(a.NP);
  const int ntw = (a.NP / 16 + 3) / 4;
  const double flops = 2.0 * a.BFT * (double)a.N * kTfHV + 2.0 * a.BFT * (double)kTfQW * a.N +
                       8.0 * (a.BFT / a.T) * kTfH * (double)a.T * a.T * kTfD;
  const double bytes = 4.0 * a.BFT * (4.0 * a.N + 2.0 * kTfQW + 2.0 * kTfH * a.T) + 8.0 * kTfQW * a.NP;
  using Kern = void (*)(TatFusedBwdArgs);
  Kern k = nullptr;
#define TB_T(TT)                                          \
  switch (ntw) {                                          \
    case 1: k = tat_fused_bwd_kernel<TT, 1>; break;       \
    case 2: k = tat_fused_bwd_kernel<TT, 2>; break;       \
    case 3: k = tat_fused_bwd_kernel<TT, 3>; break;       \
    case 4: k = tat_fused_bwd_kernel<TT, 4>; break;       \
    default: k = tat_fused_bwd_kernel<TT, 5>; break;      \
  }                                                       \
  break;
  switch (a.T) {
    case 4: TB_T(4)
    case 8: TB_T(8)
    case 12: TB_T(12)
    default: TB_T(16)
  }
#undef TB_T
  if (lds > 64 * 1024) {
    static std::mutex mu;
    static std::set<Kern> done;
    std::lock_guard<std::mutex> lock(mu);
    if (!done.count(k)) {
      const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) { set_last_error(std::string("tat_fused_bwd: ") + hipGetErrorString(e)); return (int)e; }
      done.insert(k);
    }
  }
  void* rec = gemm_prof_begin(flops, bytes, st);
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(256), lds, st, a);
  DS_CHECK_LAUNCH();
  if (sg.p) DS_TRY(stream_sig_sent(st, sg));
  gemm_prof_end(rec, st);
  return 0;
}
