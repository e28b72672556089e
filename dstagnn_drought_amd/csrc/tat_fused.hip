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

// row R of the (B F T) x N input E: src[(R % FT) s0 + (R / FT) s1 + n sN]
__device__ __forceinline__ int64_t tf_row(const TatFusedArgs& a, int64_t R) {
  const int64_t b = R / a.FT;
  return (R - b * a.FT) * a.s0 + b * a.s1;
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
  if (a.sN != 1) {  // x (B,N,F,T): lanes along the rows (contiguous for one node)
    for (int e = tid; e < kTfRows * NP; e += 256) {
      const int n = e / kTfRows, r = e - n * kTfRows;
      float v = 0.f;
      if (r < nrows && n < N) v = a.src[tf_row(a, R0 + r) + (int64_t)n * a.sN];
      Es[r * LE + n] = v;
    }
  } else {          // E (B F T, N) row-major: lanes along the nodes
    for (int e = tid; e < kTfRows * NP; e += 256) {
      const int r = e / NP, n = e - r * NP;
      float v = 0.f;
      if (r < nrows && n < N) v = a.src[tf_row(a, R0 + r) + n];
      Es[r * LE + n] = v;
    }
  }
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
    const int NC = NP / 16;
    float4 bq[kTfQTW];
#pragma unroll
    for (int j = 0; j < kTfQTW; ++j) bq[j] = *reinterpret_cast<const float4*>(wp[j]);
    for (int c = 0; c < NC; ++c) {
      float4 bn[kTfQTW];
      const int cn = min(c + 1, NC - 1);
#pragma unroll
      for (int j = 0; j < kTfQTW; ++j) bn[j] = *reinterpret_cast<const float4*>(wp[j] + 16 * cn);
      float4 av[3];
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) av[mt] = *reinterpret_cast<const float4*>(Es + (mt * 16 + i) * LE + 16 * c + 4 * q);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int j = 0; j < kTfQTW; ++j) acc[mt][j] = mf16(f4at(av[mt], s), f4at(bq[j], s), acc[mt][j]);
#pragma unroll
      for (int j = 0; j < kTfQTW; ++j) bq[j] = bn[j];
    }
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
#pragma unroll
    for (int c = 0; c < kTfHV / 16; ++c) {
      float4 bw[NTW], av[3];
#pragma unroll
      for (int j = 0; j < NTW; ++j) bw[j] = *reinterpret_cast<const float4*>(wp[j] + 16 * c);
#pragma unroll
      for (int mt = 0; mt < 3; ++mt) av[mt] = *reinterpret_cast<const float4*>(Cs + (mt * 16 + i) * kTfLC + 16 * c + 4 * q);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int mt = 0; mt < 3; ++mt)
#pragma unroll
          for (int j = 0; j < NTW; ++j) acc[mt][j] = mf16(f4at(av[mt], s), f4at(bw[j], s), acc[mt][j]);
    }
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
    const int64_t ft = R % a.FT, bb = R / a.FT;
    float* orow = a.O + ft * a.BN + bb * N;
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
