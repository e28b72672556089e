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
constexpr int kTfQTW = (kTfQT + 3) / 4; // 5 per GEMM wave (the last of waves 2, 3 is a discarded duplicate)
constexpr int kTfNmax = 320;            // N <= 320 (LDS: <= 156 KB)
constexpr int kTfDsMax = 2304;          // (48 / T) h T^2 at T = 16
constexpr int kTfG1 = 16;               // workgroups per level-1 group of the gamma / beta ticket tree


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
// NV independent full-wave sums, every lane ending with every total: the xor butterfly run
// level by level over all NV values, so each level's NV shuffles are independent (one shuffle
// latency per level, not per value).  Fixed order, and lanes agree bitwise (each level adds two
// values in either order: commutative).  (common.hpp's wave_sum_many selects between halves of
// its register array by lane; the compiler turned that into lane-indexed array accesses with
// compare chains whose masks spilled ~600 SGPRs here: the forward LayerNorm phase took 16 us.)
template <int NV>
__device__ __forceinline__ void tf_wave_sums(float (&v)[NV]) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += __shfl_xor(v[k], o, 64);
}
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
// a contiguous block of n floats from LDS (row stride ls, row length rl, both multiples of 4)
// to global memory, float4 per lane (the stores of a kernel go out at its end: stores count in
// vmcnt on gfx9, so a store issued before a k loop would hold up that loop's operand waits)
template <int NTH = 256>  // threads of the workgroup
__device__ __forceinline__ void tf_copy_out(float* g, const float* l, int rows, int rl, int ls, int tid) {
  const int q4 = rl / 4;
  float4* g4 = reinterpret_cast<float4*>(g);
  for (int e = tid; e < rows * q4; e += NTH) {
    const int r = e / q4, c4 = e - r * q4;
    g4[e] = *reinterpret_cast<const float4*>(l + r * ls + 4 * c4);
  }
}

// row R of the (B F T) x N input E: src[(R % FT) s0 + (R / FT) s1 + n sN]  (R, FT < 2^31: the
// host checks; 32-bit division — a 64-bit one is a ~200-instruction software routine)
__device__ __forceinline__ int64_t tf_row(const TatFusedArgs& a, int64_t R) {
  const uint32_t r = (uint32_t)R, ft = (uint32_t)a.FT, b = r / ft;
  return (int64_t)(r - b * ft) * a.s0 + (int64_t)b * a.s1;
}

// ---- the 48-row products on the matrix cores -------------------------------------------------
// 3 x NJ tiles (48 x 16 NJ) += A (48 x 16 NC, LDS rows of stride LA) B (16 NC x 16 NJ: lane
// (i, q) of tile j reads the float4 at wp[j] + 16 c: B row 16 c + 4 q + s, column i).
// Contraction index of step s of chunk c: 16 c + 4 q + s in both operands.  A and B fragments
// are double-buffered (ping-pong, no register copies), so chunk c + 1's global and LDS loads are
// in flight while chunk c is multiplied; sched_barrier keeps the scheduler from sinking them.
template <int NJ>
__device__ __forceinline__ void tf_ld_b(float4 (&b)[NJ], const float* const (&wp)[NJ], int off) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const float4*>(wp[j] + off);
}
__device__ __forceinline__ void tf_ld_a(float4 (&av)[3], const float* A, int LA, int c, int i, int q) {
#pragma unroll
  for (int mt = 0; mt < 3; ++mt) av[mt] = *reinterpret_cast<const float4*>(A + (mt * 16 + i) * LA + 16 * c + 4 * q);
}
template <int NJ>
__device__ __forceinline__ void tf_mma(floatx4 (&acc)[3][NJ], const float4 (&av)[3], const float4 (&bq)[NJ]) {
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[mt][j] = mf16(f4at(av[mt], s), f4at(bq[j], s), acc[mt][j]);
}
// B fragments come from L2 (the re-laid weights): with one chunk of look-ahead every chunk waited
// a full L2 round trip (the products ran at ~1/3 of the CU's MFMA rate, -DDSTAGNN_TF_TIMING).  A
// ring of DB chunks keeps DB - 1 chunks of B loads in flight; A (LDS) is double-buffered.  Chunk
// indices past NC are clamped (the redundant loads hit L2) and their products skipped.
#ifndef DSTAGNN_TF_DB
#define DSTAGNN_TF_DB 4  // (-DDSTAGNN_TF_DB=2: one chunk of look-ahead, the round-5 pipeline; A/B builds)
#endif
template <int NJ, int DB = DSTAGNN_TF_DB>
__device__ __forceinline__ void tf_gemm_rows48(floatx4 (&acc)[3][NJ], const float* A, int LA, int NC, int i, int q,
                                               const float* const (&wp)[NJ]) {
  static_assert(DB % 2 == 0 && DB >= 2, "even ring: the A ping-pong slot is d % 2");
  float4 b[DB][NJ], av[2][3];
#pragma unroll
  for (int d = 0; d < DB - 1; ++d) tf_ld_b(b[d], wp, 16 * min(d, NC - 1));
  tf_ld_a(av[0], A, LA, 0, i, q);
  for (int c0 = 0; c0 < NC; c0 += DB) {
#pragma unroll
    for (int d = 0; d < DB; ++d) {
      const int c = c0 + d;
      tf_ld_b(b[(d + DB - 1) % DB], wp, 16 * min(c + DB - 1, NC - 1));
      tf_ld_a(av[(d + 1) % 2], A, LA, min(c + 1, NC - 1), i, q);
      __builtin_amdgcn_sched_barrier(0);
      if (c < NC) tf_mma(acc, av[d % 2], b[d]);  // (wave-uniform)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// E tile (48 x NP, zero-padded) into LDS, every load of a thread issued before its first LDS
// store.  x (B,N,F,T) with the 48 rows inside one sample: a node's 48 values are contiguous —
// float4 per lane; otherwise (E row-major, first block) scalar loads along the nodes.
template <int NTH = 256>  // threads of the workgroup
__device__ __forceinline__ void tf_load_e_tile(const TatFusedArgs& a, int64_t R0, int nrows, float* Es, int LE,
                                               int NP, int N, int tid, int64_t* roff) {
  constexpr int UE = 2048 / NTH;  // loads in flight per thread (2048 per workgroup round)
  const uint32_t ft0 = (uint32_t)R0 % (uint32_t)a.FT;
  if (a.sN != 1 && a.s0 == 1 && nrows == kTfRows && ft0 + kTfRows <= (uint32_t)a.FT) {
    const float* base = a.src + tf_row(a, R0);
    constexpr int Q4 = kTfRows / 4;  // 12 float4 per node
    const int total = N * Q4;
    for (int e0 = 0; e0 < total; e0 += NTH * UE) {
      float4 v[UE];
#pragma unroll
      for (int u = 0; u < UE; ++u) {
        const int e = min(e0 + u * NTH + tid, total - 1);
        const int n = e / Q4, c4 = e - n * Q4;
        v[u] = *reinterpret_cast<const float4*>(base + (int64_t)n * a.sN + 4 * c4);
      }
#pragma unroll
      for (int u = 0; u < UE; ++u) {
        const int e = e0 + u * NTH + tid;
        if (e < total) {
          const int n = e / Q4, r = 4 * (e - n * Q4);
          Es[r * LE + n] = v[u].x;
          Es[(r + 1) * LE + n] = v[u].y;
          Es[(r + 2) * LE + n] = v[u].z;
          Es[(r + 3) * LE + n] = v[u].w;
        }
      }
    }
    for (int e = tid; e < kTfRows * (NP - N); e += NTH) {  // pad columns
      const int r = e / (NP - N), n = N + e - r * (NP - N);
      Es[r * LE + n] = 0.f;
    }
    return;
  }
  if (tid < kTfRows) roff[tid] = tf_row(a, R0 + min(tid, max(nrows - 1, 0)));
  __syncthreads();
  const int total = kTfRows * NP;
  for (int e0 = 0; e0 < total; e0 += NTH * UE) {
    float v[UE];
#pragma unroll
    for (int u = 0; u < UE; ++u) {
      const int e = e0 + u * NTH + tid;
      int r, n;
      if (a.sN == 1) { r = e / NP; n = e - r * NP; }
      else { n = e / kTfRows; r = e - n * kTfRows; }
      const bool ok = e < total && r < nrows && n < N;
      v[u] = ok ? a.src[roff[min(r, kTfRows - 1)] + (int64_t)min(n, N - 1) * a.sN] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UE; ++u) {
      const int e = e0 + u * NTH + tid;
      if (e < total) {
        int r, n;
        if (a.sN == 1) { r = e / NP; n = e - r * NP; }
        else { n = e / kTfRows; r = e - n * kTfRows; }
        Es[r * LE + n] = v[u];
      }
    }
  }
  __syncthreads();  // (roff lives in a region written later)
}

// =====================================================================================
// Forward
// =====================================================================================
// LDS (floats): Es [48][NP+4] (E, then u = fc + E) | Qs [48][292] Q|K|V | Cs [48][100] ctx |
// RA [PW h T^2] re_At | AT [PW h T^2] softmax — re_At / A / Q|K|V / ctx go out at the end
// W waves (4: one per SIMD; 8: two per SIMD — each phase's work split over twice the waves, so
// one wave's latency (LDS fragment loads, L2 weight loads, shuffles) hides behind its SIMD twin's)
template <int T, int NTW, int W>  // NTW: LayerNorm values per lane (ceil(NP / 64))
__global__ __launch_bounds__(64 * W, 1) void tat_fused_fwd_kernel(TatFusedArgs a) {
  static_assert(T % 4 == 0 && T <= 16 && kTfRows % T == 0, "whole problems per workgroup, one 16 x 16 tile");
  static_assert(W == 4 || W == 8, "four or eight waves");
  constexpr int NTH = 64 * W;
  constexpr int PW = kTfRows / T;                  // problems per workgroup
  constexpr int NTASK = PW * kTfH;                 // (problem, head) attention tasks
  constexpr int TPW = (NTASK + W - 1) / W;         // per wave
  // the two products run on waves 0-3 only (the 4-wave column tiling, one wave per SIMD): with
  // 8 waves on them both an 8-way column split (a third of the Q|K|V tiles duplicates) and a
  // contraction split (partials added through LDS) measured slower — 15 / 19 us for the Q|K|V
  // product against 12.5 on four waves (-DDSTAGNN_TF_TIMING); the latency-bound phases
  // (E tile, attention, LayerNorm, stores) use all W waves
  constexpr int QTW = kTfQTW;                      // Q|K|V column tiles per wave
  constexpr int NFC = NTW;                         // fc column tiles per wave (NP / 16 <= 4 NTW tiles)
  constexpr int RPW = kTfRows / W;                 // LayerNorm rows per wave
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int NP = a.NP, LE = NP + 4, N = a.N;
  float* Es = lds;
  float* Qs = Es + kTfRows * LE;
  float* Cs = Qs + kTfRows * kTfLQ;
  float* RA = Cs + kTfRows * kTfLC;
  float* AT = RA + kTfDsMax;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, i = l & 15, q = l >> 4;
  const int64_t R0 = (int64_t)blockIdx.x * kTfRows;
  const int nrows = (int)min<int64_t>(kTfRows, a.BFT - R0);
  const int64_t P0 = R0 / T;  // first problem (b, f)
  stream_sig_store(a.sig, a.sig_v);
  TF_DECL;
  TF_MARK(0);

  // res_att operands of this wave's attention tasks, issued first (they land during the GEMM)
  float4 rr[TPW];
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    rr[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int task = w + W * k, p = task / kTfH, hd = task - p * kTfH;
    if (task < NTASK && p * T < nrows && i < T && q < T / 4 && a.res_mode != DSTAGNN_RES_NONE) {
      const int64_t P = P0 + p;
      const int64_t bP = (uint32_t)P / (uint32_t)a.F;
      const float* rp = a.res_mode == DSTAGNN_RES_BCAST ? a.res + (bP * kTfH + hd) * T * T
                                                        : a.res + (P * kTfH + hd) * T * T;
      rr[k] = *reinterpret_cast<const float4*>(rp + i * T + 4 * q);
    }
  }
  // the LayerNorm's gamma / beta for this lane's nodes (used at the end; loaded now)
  float gv[NTW], bv[NTW];
#pragma unroll
  for (int j = 0; j < NTW; ++j) {
    const int n = min(l + 64 * j, N - 1);
    gv[j] = a.g[n];
    bv[j] = a.bta[n];
  }
  // ---- 1. E tile --------------------------------------------------------------------------
  tf_load_e_tile<NTH>(a, R0, nrows, Es, LE, NP, N, tid, reinterpret_cast<int64_t*>(Qs));
  __syncthreads();
  TF_MARK(1);

  // ---- 2. Q | K | V = E Wqkv^T ------------------------------------------------------------
  {
    floatx4 acc[3][QTW];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int j = 0; j < QTW; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (w < 4) {  // (wave-uniform)
      const float* wp[QTW];
#pragma unroll
      for (int j = 0; j < QTW; ++j) wp[j] = a.wqkv + (int64_t)(min(w + 4 * j, kTfQT - 1) * 16 + i) * NP + 4 * q;
      tf_gemm_rows48(acc, Es, LE, NP / 16, i, q, wp);
#pragma unroll
      for (int j = 0; j < QTW; ++j) {
        const int nt = w + 4 * j;
        if (nt < kTfQT) {
#pragma unroll
          for (int mt = 0; mt < 3; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) Qs[(mt * 16 + 4 * q + r) * kTfLQ + nt * 16 + i] = acc[mt][j][r];
        }
      }
    }
  }
  __syncthreads();
  TF_MARK(2);

  // ---- 3. attention per (problem, head) (tat_fwd_mfma_kernel's math, operands from LDS) ----
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int task = w + W * k;
    // (continue, not break: a break leaves the loop not fully unrolled and the per-task register
    // arrays rr / at / dr dynamically indexed — readlane / cndmask chains, measured 2x slower)
    if (task >= NTASK || (task / kTfH) * T >= nrows) continue;  // (wave-uniform)
    const int p = task / kTfH, hd = task - p * kTfH;
    const int rb = p * T;
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
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = mf16(k0.x, q0.x, acc);
    acc = mf16(k0.y, q0.y, acc);
    acc = mf16(k0.z, q0.z, acc);
    acc = mf16(k0.w, q0.w, acc);
    acc = mf16(k1.x, q1.x, acc);
    acc = mf16(k1.y, q1.y, acc);
    acc = mf16(k1.z, q1.z, acc);
    acc = mf16(k1.w, q1.w, acc);
    const float rv[4] = {rr[k].x, rr[k].y, rr[k].z, rr[k].w};
    float sc[4], pr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sc[r] = acc[r] * a.scale;
      sc[r] += rv[r];
    }
    const int tb = task * T * T;  // this task's tile in RA / AT ([p][hd] order = the global order)
    if (vi && vj) *reinterpret_cast<float4*>(RA + tb + c * T + 4 * q) = make_float4(sc[0], sc[1], sc[2], sc[3]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float m = xmax16(vi ? sc[r] : -INFINITY);
      const float e = vi ? __expf(sc[r] - m) : 0.f;
      const float inv = 1.f / xsum16(e);
      pr[r] = vj ? e * inv : 0.f;
    }
    if (vi && vj) *reinterpret_cast<float4*>(AT + tb + c * T + 4 * q) = make_float4(pr[0], pr[1], pr[2], pr[3]);
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
  TF_MARK(3);

  // ---- 4. u = ctx W_fc^T + E, in the E tile -------------------------------------------------
  {
    const int NT = NP / 16;
    floatx4 acc[3][NFC];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt)
#pragma unroll
      for (int j = 0; j < NFC; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    if (w < 4) {  // (wave-uniform)
    const float* wp[NFC];
#pragma unroll
    for (int j = 0; j < NFC; ++j) wp[j] = a.wfc + (int64_t)min(min(w + 4 * j, NT - 1) * 16 + i, N - 1) * kTfHV + 4 * q;
    tf_gemm_rows48(acc, Cs, kTfLC, kTfHV / 16, i, q, wp);
#pragma unroll
    for (int j = 0; j < NFC; ++j) {
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
  }
  __syncthreads();
  TF_MARK(4);

  // ---- 5. LayerNorm over N, the wave's 12 rows at once (ln_fwd_kernel's two-pass statistics;
  // the row sums of all 12 rows in one multi-value reduction instead of 12 dependent chains) ----
  {
    float v[RPW][NTW];
    float s16[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const float* row = Es + (w + W * k) * LE;
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int n = l + 64 * j;
        v[k][j] = n < N ? row[n] : 0.f;
        sum += v[k][j];
      }
      s16[k] = sum;
    }
    tf_wave_sums(s16);
    float mean[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) mean[k] = s16[k] / N;
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      float var = 0.f;
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int n = l + 64 * j;
        if (n < N) {
          const float d = v[k][j] - mean[k];
          var += d * d;
        }
      }
      s16[k] = var;
    }
    tf_wave_sums(s16);
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const int r = w + W * k;
      if (r >= nrows) continue;
      const int64_t R = R0 + r;
      const float rs = rsqrtf(s16[k] / N + a.eps);
      if (l == 0) {
        a.mu[R] = mean[k];
        a.rs[R] = rs;
      }
      const uint32_t bb = (uint32_t)R / (uint32_t)a.FT, ft = (uint32_t)R - bb * (uint32_t)a.FT;
      float* orow = a.O + (int64_t)ft * a.BN + (int64_t)bb * N;
      float* urow = a.u + R * N;
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int n = l + 64 * j;
        if (n < N) {
          urow[n] = v[k][j];
          orow[n] = (v[k][j] - mean[k]) * rs * gv[j] + bv[j];
        }
      }
    }
  }
  TF_MARK(5);
  // ---- 6. the saved tiles: Q|K|V, ctx, re_At, A (contiguous blocks for the workgroup) --------
  tf_copy_out<NTH>(a.qkv + R0 * kTfQW, Qs, nrows, kTfQW, kTfLQ, tid);
  tf_copy_out<NTH>(a.ctx + R0 * kTfHV, Cs, nrows, kTfHV, kTfLC, tid);
  const int np = nrows / T;
  tf_copy_out<NTH>(a.re_at + P0 * kTfH * T * T, RA, 1, np * kTfH * T * T, 0, tid);
  tf_copy_out<NTH>(a.att + P0 * kTfH * T * T, AT, 1, np * kTfH * T * T, 0, tid);
  TF_MARK(6);
  TF_PRINT("tat_fused_fwd", 7);
}

size_t tat_fused_lds(int NP) {
  return sizeof(float) * ((size_t)kTfRows * (NP + 4) + (size_t)kTfRows * kTfLQ + (size_t)kTfRows * kTfLC +
                          2 * (size_t)kTfDsMax);
}

// =====================================================================================
// Backward: LN_N backward -> dctx = dU W_fc -> attention backward -> dE = dU + dqkv Wqkv,
// accumulated straight into dx (inner block: dx[b, n, ft] is x's layout, so the four rows a
// lane's accumulator holds for one node are one float4) or written as dE (first block: the
// EmbedT LayerNorm backward follows).  Was: ln_bwd, dctx GEMM, tat_bwd_mfma, dE GEMM, transpose.
// Saved for the weight gradients (issued after it): dU (fc) and dqkv (Q|K|V); the LayerNorm's
// gamma / beta as one partial row per workgroup; the broadcast res_att gradient sum_f dS folded
// in-kernel (fixed chunk order, tat_bwd_mfma's ticket hand-off).
// LDS (floats): DUs [48][NP+4] | Qs [48][292] u, then the gamma / beta wave partials, then Q|K|V,
// then dQ|dK|dV | Cs [48][100] dctx | TRs [W][16][17] | DSs [PW h T^2] dS (+ one int)
// =====================================================================================
// W waves as in the forward: the two products (dctx, dE) on waves 0-3 (one per SIMD), the load,
// LayerNorm, attention and store phases on all W
template <int T, int NTW, int W>
__global__ __launch_bounds__(64 * W, 1) void tat_fused_bwd_kernel(TatFusedBwdArgs a) {
  static_assert(T % 4 == 0 && T <= 16 && kTfRows % T == 0, "whole problems per workgroup, one 16 x 16 tile");
  static_assert(W == 4 || W == 8, "four or eight waves");
  constexpr int NTH = 64 * W;
  constexpr int PW = kTfRows / T;
  constexpr int NTASK = PW * kTfH;
  constexpr int TPW = (NTASK + W - 1) / W;
  constexpr int RPW = kTfRows / W;            // LayerNorm rows per wave
  constexpr int GJ = (512 + NTH - 1) / NTH;   // gamma / beta columns per thread (N <= 320 < 512)
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int NP = a.NP, LE = NP + 4, N = a.N;
  float* DUs = lds;
  float* Qs = DUs + kTfRows * LE;
  float* Cs = Qs + kTfRows * kTfLQ;
  float* TRs = Cs + kTfRows * kTfLC;
  float* DSs = TRs + W * 16 * 17;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, i = l & 15, q = l >> 4;
  const int64_t R0 = (int64_t)blockIdx.x * kTfRows;
  const int nrows = (int)min<int64_t>(kTfRows, a.BFT - R0);
  const int64_t P0 = R0 / T;
  stream_sig_store(a.sig, a.sig_v);
  TF_DECL;
  TF_MARK(0);

  // ---- A0. every load of the first phases in ONE round, before any LDS store — the LayerNorm's
  // u block (contiguous: float4) and dO rows (float2), the LayerNorm statistics, the softmax and
  // d re_At of the wave's attention tasks, the Q|K|V rows (to LDS after the LayerNorm).  (With
  // each group's LDS stores between the groups, the scheduler kept the program order and the
  // phase paid three HBM round trips: 15-20 us of the kernel's ~50, -DDSTAGNN_TF_TIMING.)
  // Native vector types throughout: HIP's float4 struct copies become memcpys that pin a
  // staging array in scratch.
  typedef float tf_f2 __attribute__((ext_vector_type(2)));
  float* Us = Qs;  // [48][LE] u (the Q|K|V + ctx regions, free until after the LayerNorm)
  constexpr int UV = (12 * NTW + W - 1) / W;  // float4 of u per thread: 48 N / 4 / NTH (one round)
  constexpr int DV = (24 * NTW + W - 1) / W;  // float2 of dO per thread: 48 N / 2 / NTH
  const int tot = nrows * N, h2 = N / 2, tot2 = nrows * h2;
  const bool vec = (tot & 3) == 0 && (N & 1) == 0;  // else: dword loads (odd N), the slow path below
  const float* gu = a.u + R0 * N;
  floatx4 uv[UV];
  tf_f2 dv[DV];
  if (vec) {
#pragma unroll
    for (int u = 0; u < UV; ++u) uv[u] = reinterpret_cast<const floatx4*>(gu)[min(u * NTH + tid, tot / 4 - 1)];
#pragma unroll
    for (int u = 0; u < DV; ++u) {  // (magic divisions: runtime-divisor ones cost ~40 VALU each)
      const int e = min(u * NTH + tid, tot2 - 1), r = (int)fdiv((uint32_t)e, a.fdH2), c2 = e - r * h2;
      const uint32_t R = (uint32_t)(R0 + r);
      const uint32_t bb = fdiv(R, a.fdFT), ft = R - bb * (uint32_t)a.FT;
      dv[u] = *reinterpret_cast<const tf_f2*>(a.dO + (int64_t)ft * a.BN + (int64_t)bb * N + 2 * c2);
    }
  }
  // the LayerNorm statistics of the wave's rows (lane k < RPW: row w + W k) and gamma
  float mu_l, rs_l, gl[NTW];
  {
    const int64_t R = R0 + min(w + W * min(l, RPW - 1), nrows - 1);
    mu_l = a.mu[R];
    rs_l = a.rs[R];
#pragma unroll
    for (int j = 0; j < NTW; ++j) gl[j] = a.g[min(l + 64 * j, N - 1)];
  }
  float at[TPW][4], dr[TPW][4];
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int task = w + W * k, p = task / kTfH, hd = task - p * kTfH;
    const bool live = task < NTASK && p * T < nrows;
    const int64_t sbase = ((P0 + p) * kTfH + hd) * T * T;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ii = 4 * q + s;
      const bool ok = live && ii < T && i < T;
      at[k][s] = ok ? a.att[sbase + ii * T + i] : 0.f;
      dr[k][s] = ok && a.dre ? a.dre[sbase + ii * T + i] : 0.f;
    }
  }
  constexpr int QV4 = kTfRows * kTfQW / 4 / NTH;  // 13.5 -> 14 (6.75 -> 7) float4 per thread
  floatx4 qv[QV4 + 1];
  {
    const floatx4* gq = reinterpret_cast<const floatx4*>(a.qkv + R0 * kTfQW);
    const int totq = nrows * (kTfQW / 4);
#pragma unroll
    for (int u = 0; u <= QV4; ++u) qv[u] = gq[min(u * NTH + tid, totq - 1)];
  }
  __builtin_amdgcn_sched_barrier(0);  // (every load above is issued before the first LDS store)
  if (vec) {
#pragma unroll
    for (int u = 0; u < UV; ++u) {
      const int e4 = u * NTH + tid;
      if (e4 >= tot / 4) continue;
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        const int e = 4 * e4 + z, r = (int)fdiv((uint32_t)e, a.fdN), n = e - r * N;
        Us[r * LE + n] = uv[u][z];
      }
    }
#pragma unroll
    for (int u = 0; u < DV; ++u) {
      const int e = u * NTH + tid;
      if (e >= tot2) continue;
      const int r = (int)fdiv((uint32_t)e, a.fdH2), c2 = e - r * h2;
      DUs[r * LE + 2 * c2] = dv[u][0];
      DUs[r * LE + 2 * c2 + 1] = dv[u][1];
    }
  } else {
    for (int e = tid; e < tot; e += NTH) {
      const int r = e / N, n = e - r * N;
      Us[r * LE + n] = gu[e];
      const int64_t R = R0 + r;
      const uint32_t bb = (uint32_t)R / (uint32_t)a.FT, ft = (uint32_t)R - bb * (uint32_t)a.FT;
      DUs[r * LE + n] = a.dO[(int64_t)ft * a.BN + (int64_t)bb * N + n];
    }
  }
  // the u / dO tiles: a raw barrier behind the LDS stores only — __syncthreads() would also
  // drain vmcnt, i.e. wait here for the 55 KB of Q|K|V rows (and the softmax / d re_At
  // operands) that are first used after the LayerNorm phase; they stay in flight through it
#ifdef DSTAGNN_TF_SYNC_A0
  __syncthreads();  // (A/B builds: the round-5 barrier)
#else
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#endif
  TF_MARK(1);
  TF_MARK(2);
  // ---- A1. LayerNorm(N) backward of the wave's RPW rows at once (ln_bwd_kernel's arithmetic) --
  float gp[NTW], bp[NTW], gsum[GJ], bsum[GJ];
  {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      gp[j] = 0.f;
      bp[j] = 0.f;
      if (l + 64 * j >= N) gl[j] = 0.f;
    }
    float s32[2 * RPW], xh[RPW][NTW], dyv[RPW][NTW];
    float mean[RPW], rsv[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const int r = w + W * k;
      mean[k] = __shfl(mu_l, k, 64);
      rsv[k] = __shfl(rs_l, k, 64);
      const bool live = r < nrows;
      float uu[NTW];
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int n = min(l + 64 * j, N - 1);
        dyv[k][j] = DUs[min(r, kTfRows - 1) * LE + n];
        uu[j] = Us[min(r, kTfRows - 1) * LE + n];
      }
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const bool ok = live && l + 64 * j < N;
        if (!ok) dyv[k][j] = 0.f;
        xh[k][j] = ok ? (uu[j] - mean[k]) * rsv[k] : 0.f;
        const float dxh = dyv[k][j] * gl[j];
        s1 += dxh;
        s2 += dxh * xh[k][j];
        gp[j] += dyv[k][j] * xh[k][j];
        bp[j] += dyv[k][j];
      }
      s32[k] = s1;
      s32[RPW + k] = s2;
    }
    tf_wave_sums(s32);
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
      const int r = w + W * k;
      float* dur = DUs + r * LE;
      const float s1 = s32[k] / N, s2 = s32[RPW + k] / N;
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        const int n = l + 64 * j;
        if (n < NP) dur[n] = (r < nrows && n < N) ? rsv[k] * (dyv[k][j] * gl[j] - s1 - xh[k][j] * s2) : 0.f;
      }
    }
  }
  __syncthreads();  // (every wave's reads of the u tile: its region takes the partials, then Q|K|V)
  {  // gamma / beta: the W waves' partials summed in wave order (kept for the end)
    float* red = Us;  // [2][W][NP] in the u tile's region (free now; <= 5 120 of its 14 016 floats)
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = l + 64 * j;
      if (n < NP) {
        red[(0 * W + w) * NP + n] = gp[j];
        red[(1 * W + w) * NP + n] = bp[j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < GJ; ++j) {  // n = tid + NTH j (N <= 320 < 512)
      const int n = min(tid + NTH * j, NP - 1);
      float g = red[n], b = red[W * NP + n];
#pragma unroll
      for (int v = 1; v < W; ++v) {
        g += red[v * NP + n];
        b += red[(W + v) * NP + n];
      }
      gsum[j] = g;
      bsum[j] = b;
    }
    __syncthreads();
  }
  {
    const int tot = nrows * (kTfQW / 4);
#pragma unroll
    for (int u = 0; u <= QV4; ++u) {
      const int e = u * NTH + tid;
      if (e < tot) {
        const int r = e / (kTfQW / 4), c4 = e - r * (kTfQW / 4);
        *reinterpret_cast<floatx4*>(Qs + r * kTfLQ + 4 * c4) = qv[u];
      }
    }
  }
  TF_MARK(3);
  TF_MARK(4);

  // ---- B. dctx = dU W_fc  (48 x h dv, contraction over the NP nodes) -----------------------
  if (w < 4) {  // (wave-uniform)
    constexpr int CT = kTfHV / 16;          // 6 column tiles x 3 row tiles
    floatx4 acc[3][2];                      // wave w: columns {w, w + 4} (waves 2, 3: one + a duplicate)
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) acc[mt][0] = acc[mt][1] = floatx4{0.f, 0.f, 0.f, 0.f};
    const float* wp[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) wp[j] = a.wfcT + (int64_t)(min(w + 4 * j, CT - 1) * 16 + i) * NP + 4 * q;
    tf_gemm_rows48(acc, DUs, LE, NP / 16, i, q, wp);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nt = w + 4 * j;
      if (nt < CT) {
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) Cs[(mt * 16 + 4 * q + r) * kTfLC + nt * 16 + i] = acc[mt][j][r];
      }
    }
  }
  __syncthreads();
  TF_MARK(5);

  // the dx tile of D1's epilogue (inner block), issued now: it lands during C and D1
  float4 dxo[3][NTW];
  if (a.dx && w < 4) {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = min((w + 4 * j) * 16 + i, N - 1);
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) {
        const int64_t R = R0 + min(mt * 16 + 4 * q, nrows - 4);
        const uint32_t bb = fdiv((uint32_t)R, a.fdFT), ft = (uint32_t)R - bb * (uint32_t)a.FT;
        dxo[mt][j] = *reinterpret_cast<const float4*>(a.dx + (int64_t)bb * a.dxb + (int64_t)n * a.FT + ft);
      }
    }
  }

  // ---- C. attention backward per (problem, head) (tat_bwd_mfma_kernel's math) ---------------
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int task = w + W * k;
    // (continue, not break: a break leaves the loop not fully unrolled and the per-task register
    // arrays rr / at / dr dynamically indexed — readlane / cndmask chains, measured 2x slower)
    if (task >= NTASK || (task / kTfH) * T >= nrows) continue;  // (wave-uniform)
    const int p = task / kTfH, hd = task - p * kTfH;
    const int rb = p * T;
    float* Qp = Qs + rb * kTfLQ + hd * kTfD;
    float* Kp = Qp + kTfHV;
    float* Vp = Qp + 2 * kTfHV;
    const float* Cp = Cs + rb * kTfLC + hd * kTfD;
    const int c = i;
    const bool vj = c < T;
    float4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = d0, v0 = d0, v1 = d0;
    float cb[2][4], qb[2][4], kb[2][4];
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
    for (int r = 0; r < 4; ++r) cs = fmaf(at[k][r], dA[r], cs);
    cs += __shfl_xor(cs, 16, 64);
    cs += __shfl_xor(cs, 32, 64);
    float ds[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) ds[r] = at[k][r] * (dA[r] - cs) + dr[k][r];
    if (vj) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * q + r < T) DSs[task * T * T + (4 * q + r) * T + c] = ds[r];
    }
    floatx4 z = {0.f, 0.f, 0.f, 0.f};
    floatx4 gv0 = z, gv1 = z, gk0 = z, gk1 = z, gq0 = z, gq1 = z;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      gv0 = mf16(at[k][s], cb[0][s], gv0);
      gv1 = mf16(at[k][s], cb[1][s], gv1);
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
      // the row offset made opaque to the compiler: at T = 16 (no predicate on these stores) the
      // AMDGPU backend (ROCm 7.2 clang 22) merged the four rows' stores into rebased ds_write2
      // pairs and encoded the dQ column-c store of row 4q+2 at +61 floats instead of +292 —
      // writing into another head's Q columns (tests/test_gpu_parity.py t16h3 cases).  With an
      // opaque per-row base every store's offset is <= 208 floats from it: no rebasing.
      int off = ii * kTfLQ + c;
      asm volatile("" : "+v"(off));
      float* row = Qp + off;
      row[0] = gq0[r] * a.scale;
      row[16] = gq1[r] * a.scale;
      row[kTfHV] = gk0[r] * a.scale;
      row[kTfHV + 16] = gk1[r] * a.scale;
      row[2 * kTfHV] = gv0[r];
      row[2 * kTfHV + 16] = gv1[r];
    }
  }
  __syncthreads();
  TF_MARK(6);

  // ---- D1. dE = dU + dqkv [Wq; Wk; Wv] ---------------------------------------------------
  if (w < 4) {  // (wave-uniform)
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
    TF_MARK(7);
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
          const uint32_t bb = fdiv((uint32_t)R, a.fdFT), ft = (uint32_t)R - bb * (uint32_t)a.FT;
          float4* dp = reinterpret_cast<float4*>(a.dx + (int64_t)bb * a.dxb + (int64_t)n * a.FT + ft);
          const float4 o = dxo[mt][j];
          *dp = make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) a.dE[(R + r) * N + n] = v[r];
        }
      }
    }
  }

  TF_MARK(8);
  // ---- E. the saved tiles and partials (stores last: see tf_copy_out) ----------------------
  tf_copy_out<NTH>(a.dqkv + R0 * kTfQW, Qs, nrows, kTfQW, kTfLQ, tid);
  if (((nrows * N) & 3) == 0) {  // dU: the workgroup's rows are one contiguous block (float4)
    float4* g4 = reinterpret_cast<float4*>(a.dU + R0 * N);
    for (int e4 = tid; e4 < nrows * N / 4; e4 += NTH) {
      float vv[4];
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        const int e = 4 * e4 + z, r = (int)fdiv((uint32_t)e, a.fdN), n = e - r * N;
        vv[z] = DUs[r * LE + n];
      }
      g4[e4] = make_float4(vv[0], vv[1], vv[2], vv[3]);
    }
  } else {
    for (int e = tid; e < nrows * N; e += NTH) {
      const int r = e / N, n = e - r * N;
      a.dU[R0 * N + e] = DUs[r * LE + n];
    }
  }
  const bool lnf = a.ln_fold != 0;  // gamma / beta summed in-kernel by a two-level ticket tree
#pragma unroll
  for (int j = 0; j < GJ; ++j) {
    const int n = tid + NTH * j;
    if (n < N) {
      if (lnf) {
        tf_st_agent(a.gpart + (int64_t)blockIdx.x * N + n, gsum[j]);
        tf_st_agent(a.bpart + (int64_t)blockIdx.x * N + n, bsum[j]);
      } else {
        if (a.gpart) a.gpart[(int64_t)blockIdx.x * N + n] = gsum[j];
        if (a.bpart) a.bpart[(int64_t)blockIdx.x * N + n] = bsum[j];
      }
    }
  }
  const int np = nrows / T;
  if (a.res_mode == DSTAGNN_RES_FULL && a.dres) tf_copy_out<NTH>(a.dres + P0 * kTfH * T * T, DSs, 1, np * kTfH * T * T, 0, tid);
  const int nch = (int)(a.FT / kTfRows);
  const int64_t bwg = (uint32_t)R0 / (uint32_t)a.FT, chw = ((uint32_t)R0 - (uint32_t)bwg * (uint32_t)a.FT) / kTfRows;
  if (a.res_mode == DSTAGNN_RES_BCAST) {
    for (int e = tid; e < kTfH * T * T; e += NTH) {
      float v = 0.f;
      for (int p = 0; p < PW; ++p) v += DSs[p * kTfH * T * T + e];  // problems in order
      tf_st_agent(a.dpart + (bwg * nch + chw) * kTfH * T * T + e, v);
    }
  }
  TF_MARK(9);
  TF_PRINT("tat_fused_bwd", 10);

  // ---- F. ticket folds (the partials above went out with agent-scope stores; the last arrival
  // takes an agent acquire and sums in a fixed order: deterministic) ---------------------------
  //   res_att (broadcast): the last workgroup of each sample b sums its nch chunks;
  //   LayerNorm gamma / beta: the last of each group of kTfG1 workgroups sums the group's rows
  //   into a level-2 row, the last group sums the level-2 rows into the parameter gradients
  //   (this replaced a colsum2d launch at the end of the main stream)
  if (a.res_mode != DSTAGNN_RES_BCAST && !lnf) return;
  int* flag = reinterpret_cast<int*>(DSs + kTfDsMax);  // (no static __shared__: it would shift the dynamic base)
  const int nwg = (int)gridDim.x, ng = (nwg + kTfG1 - 1) / kTfG1, g1 = (int)blockIdx.x / kTfG1;
  const int gsz = min(kTfG1, nwg - g1 * kTfG1);
  int* cnt_ln = a.cnt + a.B;  // [ng] level-1 tickets, then one level-2 ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int lb = a.res_mode == DSTAGNN_RES_BCAST && atomicAdd(a.cnt + bwg, 1) == nch - 1;
    const int lg = lnf && atomicAdd(cnt_ln + g1, 1) == gsz - 1;
    if (lb || lg) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (lb) __hip_atomic_store(a.cnt + bwg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    if (lg) __hip_atomic_store(cnt_ln + g1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = lb;
    flag[1] = lg;
  }
  __syncthreads();
  const bool lb = flag[0] != 0, lg = flag[1] != 0;
  if (lb) {
    for (int e = tid; e < kTfH * T * T; e += NTH) {
      float v = 0.f;
      for (int ch = 0; ch < nch; ++ch) v += tf_ld_agent(a.dpart + (bwg * nch + ch) * kTfH * T * T + e);
      a.dres[bwg * kTfH * T * T + e] = v;
    }
  }
  if (!lg) return;
  float* l2g = a.gpart + (int64_t)nwg * N;  // level-2 rows [ng][N] after the level-1 rows (slab of BFT x N)
  float* l2b = a.bpart + (int64_t)nwg * N;
  for (int e = tid; e < 2 * N; e += NTH) {  // (column, gamma | beta): the group's rows in order
    const int n = e % N, wh = e / N;
    const float* src = (wh ? a.bpart : a.gpart) + (int64_t)g1 * kTfG1 * N + n;
    float u[kTfG1];
#pragma unroll
    for (int k = 0; k < kTfG1; ++k) u[k] = k < gsz ? tf_ld_agent(src + (int64_t)k * N) : 0.f;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < kTfG1; ++k) v += u[k];
    tf_st_agent((wh ? l2b : l2g) + (int64_t)g1 * N + n, v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int last2 = atomicAdd(cnt_ln + ng, 1) == ng - 1;
    if (last2) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(cnt_ln + ng, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    flag[2] = last2;
  }
  __syncthreads();
  if (!flag[2]) return;
  for (int e = tid; e < 2 * N; e += NTH) {
    const int n = e % N, wh = e / N;
    float* out = wh ? a.bout : a.gout;
    if (!out) continue;
    const float* src = (wh ? l2b : l2g) + n;
    float v = 0.f;
    for (int k0 = 0; k0 < ng; k0 += kTfG1) {
      float u[kTfG1];
#pragma unroll
      for (int k = 0; k < kTfG1; ++k) u[k] = k0 + k < ng ? tf_ld_agent(src + (int64_t)(k0 + k) * N) : 0.f;
#pragma unroll
      for (int k = 0; k < kTfG1; ++k) v += u[k];
    }
    out[n] = v;
  }
}

size_t tat_fused_bwd_lds(int NP, int W) {
  return sizeof(float) * ((size_t)kTfRows * (NP + 4) + (size_t)kTfRows * kTfLQ + (size_t)kTfRows * kTfLC +
                          (size_t)W * 16 * 17 + kTfDsMax + 4);
}

}  // namespace

bool tat_fused_fwd_ok(int N, int T, int h, int dk, int dv) {
  // DSTAGNN_TAT_FUSED=0 (or DSTAGNN_TAT_MFMA=0, the VALU attention A/B): the unfused launches
  static const bool env = (!getenv("DSTAGNN_TAT_FUSED") || atoi(getenv("DSTAGNN_TAT_FUSED")) != 0) &&
                          (!getenv("DSTAGNN_TAT_MFMA") || atoi(getenv("DSTAGNN_TAT_MFMA")) != 0);
  // (T >= 7 for any block — check_dims — so of the 48-row tilings only T = 8, 12, 16 occur)
  return env && h == kTfH && dk == kTfD && dv == kTfD && N >= 1 && N <= kTfNmax && (T == 8 || T == 12 || T == 16);
}

int tat_fused_np(int N) { return (N + 15) / 16 * 16; }

// the backward's grid (one gamma / beta partial row per workgroup) and the rows of its two-level
// ticket tree (level-1 rows, then one level-2 row per kTfG1 workgroups): the caller's slab layout
int64_t tat_fused_bwd_wgs(int64_t BFT) { return cdiv64(BFT, kTfRows); }
int64_t tat_fused_bwd_part_rows(int64_t BFT) {
  const int64_t nwg = tat_fused_bwd_wgs(BFT);
  return nwg + cdiv64(nwg, kTfG1);
}

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
  // DSTAGNN_TF_WAVES=4|8: the forward's workgroup size (A/B)
  static const int waves = getenv("DSTAGNN_TF_WAVES") && atoi(getenv("DSTAGNN_TF_WAVES")) == 4 ? 4 : 8;
#define TF_NTW(TT, WW)                                        \
  switch (ntw) {                                              \
    case 1: k = tat_fused_fwd_kernel<TT, 1, WW>; break;       \
    case 2: k = tat_fused_fwd_kernel<TT, 2, WW>; break;       \
    case 3: k = tat_fused_fwd_kernel<TT, 3, WW>; break;       \
    case 4: k = tat_fused_fwd_kernel<TT, 4, WW>; break;       \
    default: k = tat_fused_fwd_kernel<TT, 5, WW>; break;      \
  }
#define TF_T(TT)                                              \
  if (waves == 8) { TF_NTW(TT, 8) } else { TF_NTW(TT, 4) }   \
  break;
  switch (a.T) {
    case 8: TF_T(8)
    case 12: TF_T(12)
    default: TF_T(16)
  }
#undef TF_T
#undef TF_NTW
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
  void* rec = gemm_prof_begin(flops, bytes, st, DSTAGNN_PROF_TAT_FUSED_FWD);
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * waves), lds, st, a);
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
  if (a.res_mode == DSTAGNN_RES_BCAST && !a.dres) a.res_mode = DSTAGNN_RES_NONE;  // nothing to fold
  const int64_t nwg = tat_fused_bwd_wgs(a.BFT);
  a.B = (int)(a.BFT / a.FT);
  a.fdN = make_fastdiv((uint32_t)a.N);
  a.fdH2 = make_fastdiv((uint32_t)std::max(1, a.N / 2));
  a.fdFT = make_fastdiv((uint32_t)a.FT);
  a.ln_fold = a.ln_fold && a.gpart && a.bpart && (a.gout || a.bout);
  if (a.res_mode == DSTAGNN_RES_BCAST || a.ln_fold) {
    // [B] res_att tickets, then the gamma / beta tree's [ng] level-1 tickets and one level-2 ticket
    a.cnt = stream_counters(st, (int)(a.B + cdiv64(nwg, kTfG1) + 1));
    if (!a.cnt || (a.res_mode == DSTAGNN_RES_BCAST && !a.dpart)) {
      set_last_error("tat_fused_bwd: no ticket counters");
      return DSTAGNN_E_ARG;
    }
  }
  const StreamSig sg = peek_stream_sig(st);
  a.sig = sg.p;
  a.sig_v = sg.v;
  const int64_t grid = cdiv64(a.BFT, kTfRows);
  // DSTAGNN_TF_BWD_WAVES=4|8: the backward's workgroup size (A/B)
  static const int waves = getenv("DSTAGNN_TF_BWD_WAVES") && atoi(getenv("DSTAGNN_TF_BWD_WAVES")) == 4 ? 4 : 8;
  // (NP > 256 stays on four waves: eight would spill — 256 VGPRs each at two waves per SIMD)
  const int wv = waves == 8 && (a.NP / 16 + 3) / 4 < 5 ? 8 : 4;
  const size_t lds = tat_fused_bwd_lds(a.NP, wv);
  const int ntw = (a.NP / 16 + 3) / 4;
  const double flops = 2.0 * a.BFT * (double)a.N * kTfHV + 2.0 * a.BFT * (double)kTfQW * a.N +
                       8.0 * (a.BFT / a.T) * kTfH * (double)a.T * a.T * kTfD;
  const double bytes = 4.0 * a.BFT * (4.0 * a.N + 2.0 * kTfQW + 2.0 * kTfH * a.T) + 8.0 * kTfQW * a.NP;
  using Kern = void (*)(TatFusedBwdArgs);
  Kern k = nullptr;
#define TB_NTW(TT, WW)                                        \
  switch (ntw) {                                              \
    case 1: k = tat_fused_bwd_kernel<TT, 1, WW>; break;       \
    case 2: k = tat_fused_bwd_kernel<TT, 2, WW>; break;       \
    case 3: k = tat_fused_bwd_kernel<TT, 3, WW>; break;       \
    case 4: k = tat_fused_bwd_kernel<TT, 4, WW>; break;       \
    default: k = tat_fused_bwd_kernel<TT, 5, WW>; break;      \
  }
#define TB_T(TT)                                              \
  if (wv == 8) { TB_NTW(TT, 8) } else { TB_NTW(TT, 4) }   \
  break;
  switch (a.T) {
    case 8: TB_T(8)
    case 12: TB_T(12)
    default: TB_T(16)
  }
#undef TB_T
#undef TB_NTW
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
  void* rec = gemm_prof_begin(flops, bytes, st, DSTAGNN_PROF_TAT_FUSED_BWD);
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * wv), lds, st, a);
  DS_CHECK_LAUNCH();
  if (sg.p) DS_TRY(stream_sig_sent(st, sg));
  gemm_prof_end(rec, st);
  return 0;
}
