// cheb_agg.hip — the block's sparse Chebyshev convolution in aggregate-first order (gfx950).
//
// cheb_conv_withSAt (model/DSTAGNN_my.py:117-133) computes, per timestep t and order k,
//   out_t += (T_k o P_k)^T x_t Theta_k        then ReLU           (W_k := T_k o P_k)
// The Theta-first order (cheb_sparse.hip) multiplies x by all K Thetas first — a GEMM that
// writes K*C*T floats per node (25 MB at PEMS08 B=32) — and then gathers those rows.  Here the
// gather comes first, on x itself (F*T floats per source node, gathered ONCE for all K orders:
// K times fewer bytes), and the K small (T x F)(F x C) products per destination node run on
// the wave's own matrix cores:
//
//   fwd      agg_k[j] = sum_{i in supp(j)} W_k[i,j] x_i          (F x T, saved for dTheta)
//            X[j]     = ReLU( sum_k agg_k[j]^T Theta_k )          (T x C)
//   sddmm    dagg_k[j] = Theta_k g_j^T                             (F x T per k, wave-local LDS)
//            dW_k[i,j] = < x_i, dagg_k[j] >  on the support      (the softmax backward's input)
//   spmm_t   dx_i    += sum_k Theta_k ( sum_{j in supp_row(i)} W_k[i,j] g_j )^T
//   dTheta_k = sum_{b,j,t} agg_k[b,j,:,t] g[b,j,t,:]  — one GEMM (block.hip)
//
// so the Theta GEMM of the forward and the dx GEMM of the backward disappear together with
// the (B,N,K,C,T) tensor and its gradient.  g = d(pre-ReLU X), layout (B,N,T,C); x (B,N,F,T).
// MFMA v_mfma_f32_32x32x2_f32: lane l supplies A[m = l&31][kk] and B[kk][n = l&31] with the
// lane half h = l>>5 giving the contraction index kk(s, h) at step s (any bijection works if A
// and B agree: kk = 2s + h where the operands come from LDS, kk = 16h + s where each lane
// reads 16 consecutive floats of a row, four 16-B loads); the accumulator holds
// D[m = (r&3) + 8(r>>2) + 4h][n = l&31] in register r.  Time chunks of <= 32 steps (m = t).
// The kernels are templated on KM >= K (the K aggregates live in registers together).
#include "common.hpp"
#include "ops.hpp"

namespace {

__device__ __forceinline__ int frow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ floatx16 zero16() {
  floatx16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// 16 consecutive floats of a row (4 x 16-B loads); zeros when !ok
__device__ __forceinline__ void row16(const float* p, bool ok, float (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 t = ok ? *reinterpret_cast<const float4*>(p + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// XCD-aware row-block order (cheb_sparse.hip): each XCD walks one contiguous eighth of the rows
__device__ __forceinline__ int64_t xcd_block(int on) {
  const int64_t p = blockIdx.x;
  if (!on) return p;
  const int64_t per = gridDim.x >> 3;
  return (p & 7) * per + (p >> 3);
}

constexpr int kE = 4;      // support entries per batch
// Support walks: a chunk of up to 64 entries is loaded ONE per lane (indices and the K weights),
// entry e's values then come back by v_readlane (wave-uniform e: the gathered row's base is an
// SGPR), and the gathered rows of batch e0 + kE are issued before batch e0 is multiplied (two
// batches in flight instead of three dependent round trips per batch).
__device__ __forceinline__ int rl_i(int v, int i) { return __builtin_amdgcn_readlane(v, i); }
__device__ __forceinline__ float rl_f(float v, int i) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), i));
}
// occupancy the register allocator targets (waves per SIMD) from an estimate of the VGPRs a
// variant needs (two batches of gathered rows, the K accumulators / dot products, addresses):
// as many resident waves as fit without spills (PEMS08: fwd / spmm_t 4, sddmm 3)
// (thresholds fitted to the compiler's allocation of every instantiated variant: no spills)
template <int kNQ>
constexpr bool agg_prefetch() { return kNQ <= 8; }  // wider rows: one batch in flight
template <int kNQ, int KM>
constexpr int gather_wpe() {
  return kNQ >= 12 ? 2 : (agg_prefetch<kNQ>() ? 2 : 1) * kE * kNQ + KM * kNQ + 40 <= 110 ? 4
       : ((agg_prefetch<kNQ>() ? 2 : 1) * kE * kNQ + KM * kNQ + 40 <= 125 ? 3 : 2);
}
template <int kNQ, int KM, bool PF = agg_prefetch<kNQ>()>
constexpr int sddmm_wpe() {
  // without the batch prefetch (PF false, DSTAGNN_SDDMM_NOPF=1): one batch of rows fewer in
  // registers -> PEMS08's <6, 3> fits 4 waves (more resident waves instead of the prefetch)
  return !PF && kNQ <= 6 && KM <= 3 ? 4
       : (KM <= 3 && (PF ? 2 : 1) * kE * kNQ + 16 + KM * kNQ + 64 <= 150 ? 3 : 2);
}
constexpr int kAs = 33;    // LDS row stride of a 32 x 32 operand tile

// ---------------------------------------------------------------------------------------
// forward: one wave per (b, j, time chunk)
// ---------------------------------------------------------------------------------------
template <int kNQ, int KM>  // kNQ >= F * Tc / 64, KM >= K
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(gather_wpe<kNQ, KM>(), 8))) void cheb_agg_fwd_kernel(ChebAg a) {
  __shared__ float As[4][32 * kAs];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int64_t wv = xcd_block(a.xcd_order) * 4 + w;
  if (wv >= (int64_t)a.B * a.N) return;
  const int b = (int)(wv / a.N), j = (int)(wv % a.N);
  const int t0 = blockIdx.y * 32, Tc = min(32, a.T - t0), FT = a.F * a.T, nel = a.F * Tc;
  const int64_t NN = (int64_t)a.N * a.N;
  float* at = As[w];
  // this lane's elements e = lane + 64 q of the (F x Tc) chunk: (f, t') and their x offset
  int xo[kNQ], lo[kNQ];
#pragma unroll
  for (int q = 0; q < kNQ; ++q) {
    const int e = min(lane + 64 * q, nel - 1), f = e / Tc, tl = e - f * Tc;
    xo[q] = f * a.T + t0 + tl;
    lo[q] = f * kAs + tl;  // LDS tile [f][t']
  }
  const int p0 = a.csc_ptr[j], p1 = a.csc_ptr[j + 1];
  const float* xb = a.x + (int64_t)b * a.N * FT;
  float ag[KM][kNQ];
#pragma unroll
  for (int k = 0; k < KM; ++k)
#pragma unroll
    for (int q = 0; q < kNQ; ++q) ag[k][q] = 0.f;
  for (int c0 = p0; c0 < p1; c0 += 64) {
    const int nc = min(64, p1 - c0), pl = c0 + min(lane, nc - 1);
    const int rowl = a.csc_row[pl];
    float wl[KM];  // W_k[row, j] of this lane's entry (0 past the chunk)
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      float ww = 0.f;
      if (k < a.K) {
        const int64_t o = (int64_t)rowl * a.N + j;
        ww = a.wsupp ? a.wsupp[((int64_t)b * a.K + k) * a.nnz + pl]
                     : a.cheb[(int64_t)k * NN + o] * a.P[((int64_t)b * a.K + k) * NN + o];
      }
      wl[k] = lane < nc ? ww : 0.f;
    }
    auto gather = [&](int e0, float (&dst)[kE][kNQ]) {
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const float* xr = xb + (int64_t)rl_i(rowl, min(e0 + e, nc - 1)) * FT;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) dst[e][q] = xr[xo[q]];
      }
    };
    float v[kE][kNQ];
    if constexpr (agg_prefetch<kNQ>()) gather(0, v);
    for (int e0 = 0; e0 < nc; e0 += kE) {
      float vn[kE][kNQ];
      if constexpr (agg_prefetch<kNQ>()) gather(e0 + kE, vn);  // the next batch (clamped: harmless re-reads past the chunk)
      else gather(e0, v);
#pragma unroll
      for (int k = 0; k < KM; ++k)
#pragma unroll
        for (int e = 0; e < kE; ++e) {
          const float wk = rl_f(wl[k], e0 + e);  // e0 + e <= 63; lanes >= nc hold 0
#pragma unroll
          for (int q = 0; q < kNQ; ++q) ag[k][q] = fmaf(wk, v[e][q], ag[k][q]);
        }
      if constexpr (agg_prefetch<kNQ>()) {
#pragma unroll
        for (int e = 0; e < kE; ++e)
#pragma unroll
          for (int q = 0; q < kNQ; ++q) v[e][q] = vn[e][q];
      }
    }
  }
  floatx16 acc = zero16();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k >= a.K) break;
    // Theta_k as the B operand: B[kk = f][n = c], f = 2s + h (zero past F / C)
    float bt[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int f = 2 * s + h;
      bt[s] = (f < a.F && l32 < a.C) ? a.thcat[(int64_t)f * a.KC + k * a.C + l32] : 0.f;
    }
    // agg_k[j] saved for the Theta gradient, and staged as the MFMA A operand [f][t'] (the
    // previous k's reads of the tile precede these writes in the wave's LDS order)
    float* sv = a.agg + (((int64_t)b * a.N + j) * a.K + k) * FT;
#pragma unroll
    for (int q = 0; q < kNQ; ++q)
      if (lane + 64 * q < nel) {
        sv[xo[q]] = ag[k][q];
        at[lo[q]] = ag[k][q];
      }
    wave_lds_sync();
    // D[m = t'][n = c] += sum_f agg_k[f][t'] Theta_k[f][c]
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int f = 2 * s + h;
      const float av = (f < a.F && l32 < Tc) ? at[f * kAs + l32] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bt[s], acc, 0, 0, 0);
    }
    wave_lds_sync();
  }
  if (l32 >= a.C) return;
  float* orow = a.X + ((int64_t)b * a.N + j) * a.T * a.C;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int tl = frow(r, h);
    if (tl < Tc) orow[(int64_t)(t0 + tl) * a.C + l32] = fmaxf(acc[r], 0.f);
  }
}

// ---------------------------------------------------------------------------------------
// forward for T <= 16 (F T <= 512): one wave per (sample PAIR, j), as the pair SDDMM below.  The
// support walk runs over virtual entries v = 2 e + bsel (sample bsel of entry e), accumulating
// sample bsel's aggregates ag[bsel]; the two samples' agg_k then stack into one MFMA A operand
// (m = bsel T + t), so the Theta_k chain of 16 MFMAs serves both.  Per sample the same sums in
// the same order as cheb_agg_fwd_kernel (entries in support order, orders k separately).
// ---------------------------------------------------------------------------------------
template <int kNQ, int KM>  // kNQ >= F * T / 64 (<= 8), KM >= K
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(gather_wpe<kNQ, 2 * KM>(), 8))) void cheb_agg_fwd2_kernel(ChebAg a) {
  static_assert(kNQ <= 8, "F T <= 512");
  __shared__ float As[4][32 * kAs];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int64_t wv = xcd_block(a.xcd_order) * 4 + w;
  const int npair = (a.B + 1) >> 1;
  if (wv >= (int64_t)npair * a.N) return;
  const int bp = (int)(wv / a.N), j = (int)(wv % a.N), b0 = 2 * bp, nb = min(2, a.B - b0);
  const int T = a.T, FT = a.F * T;
  const int64_t NN = (int64_t)a.N * a.N;
  float* at = As[w];
  // this lane's elements e = lane + 64 q of a sample's (F x T) block: (f, t), x offset = e
  int lo[kNQ];
#pragma unroll
  for (int q = 0; q < kNQ; ++q) {
    const int e = min(lane + 64 * q, FT - 1), f = e / T, tl = e - f * T;
    lo[q] = f * kAs + tl;  // LDS tile [f][m], m = bsel T + t (+ T for sample 1)
  }
  const int p0 = a.csc_ptr[j], p1 = a.csc_ptr[j + 1];
  const float* xb0 = a.x + (int64_t)b0 * a.N * FT;
  const float* xb1 = a.x + (int64_t)(b0 + nb - 1) * a.N * FT;
  float ag[2][KM][kNQ];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int k = 0; k < KM; ++k)
#pragma unroll
      for (int q = 0; q < kNQ; ++q) ag[s][k][q] = 0.f;
  for (int c0 = p0; c0 < p1; c0 += 32) {  // 32 entries = 64 virtual entries per chunk
    const int nc = min(32, p1 - c0), nv = 2 * nc, pl = c0 + min(lane, nc - 1);
    const int rowl = a.csc_row[pl];
    float wl[2][KM];  // W_k[row, j] of this lane's entry for each sample (0 past the chunk)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        float ww = 0.f;
        if (k < a.K) {
          const int b = b0 + min(s, nb - 1);
          const int64_t o = (int64_t)rowl * a.N + j;
          ww = a.wsupp ? a.wsupp[((int64_t)b * a.K + k) * a.nnz + pl]
                       : a.cheb[(int64_t)k * NN + o] * a.P[((int64_t)b * a.K + k) * NN + o];
        }
        wl[s][k] = lane < nc ? ww : 0.f;
      }
    auto gather = [&](int e0, float (&dst)[kE][kNQ]) {
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const int ve = min(e0 + e, nv - 1);  // (e0 even: ve & 1 == e & 1 unless clamped)
        const float* xr = ((e & 1) ? xb1 : xb0) + (int64_t)rl_i(rowl, ve >> 1) * FT;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) dst[e][q] = xr[min(lane + 64 * q, FT - 1)];
      }
    };
    float v[kE][kNQ];
    gather(0, v);
    for (int e0 = 0; e0 < nv; e0 += kE) {
      float vn[kE][kNQ];
      gather(e0 + kE, vn);  // the next batch (clamped: harmless re-reads past the chunk)
#pragma unroll
      for (int k = 0; k < KM; ++k)
#pragma unroll
        for (int e = 0; e < kE; ++e) {
          // entry (e0 + e) / 2 of sample e & 1; past the chunk: lane >= nc holds 0 (e0 + e <= 63)
          const float wk = rl_f(wl[e & 1][k], min((e0 + e) >> 1, 31));
          const float wz = e0 + e < nv ? wk : 0.f;
#pragma unroll
          for (int q = 0; q < kNQ; ++q) ag[e & 1][k][q] = fmaf(wz, v[e][q], ag[e & 1][k][q]);
        }
#pragma unroll
      for (int e = 0; e < kE; ++e)
#pragma unroll
        for (int q = 0; q < kNQ; ++q) v[e][q] = vn[e][q];
    }
  }
  floatx16 acc = zero16();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k >= a.K) break;
    float bt[16];  // Theta_k as the B operand: B[kk = f][n = c], f = 2s + h (zero past F / C)
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int f = 2 * s + h;
      bt[s] = (f < a.F && l32 < a.C) ? a.thcat[(int64_t)f * a.KC + k * a.C + l32] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s >= nb) break;
      float* sv = a.agg + (((int64_t)(b0 + s) * a.N + j) * a.K + k) * FT;  // agg_k[j], saved for dTheta
#pragma unroll
      for (int q = 0; q < kNQ; ++q)
        if (lane + 64 * q < FT) {
          sv[lane + 64 * q] = ag[s][k][q];
          at[lo[q] + s * T] = ag[s][k][q];
        }
    }
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < 16; ++s) {  // D[m][n = c] += sum_f agg_k[f][m] Theta_k[f][c]
      const int f = 2 * s + h;
      const float av = (f < a.F && l32 < nb * T) ? at[f * kAs + l32] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bt[s], acc, 0, 0, 0);
    }
    wave_lds_sync();
  }
  if (l32 >= a.C) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = frow(r, h), ms = m >= T ? 1 : 0, mt = m - ms * T;
    if (m < nb * T) a.X[(((int64_t)(b0 + ms) * a.N + j) * T + mt) * a.C + l32] = fmaxf(acc[r], 0.f);
  }
}

// ---------------------------------------------------------------------------------------
// backward SDDMM: one wave per (b, j).  dagg_k = Theta_k g_j^T (F x T) for every k on the
// wave's matrix cores into LDS, then the column's support rows x_i gathered ONCE and dotted
// with all K: dW_k[i, j] = <x_i, dagg_k> (flash path: the softmax backward's support terms
// dzs = P T dW and c_j instead, as cheb_sparse.hip).
// ---------------------------------------------------------------------------------------
template <int kNQ, int KM, bool PF = agg_prefetch<kNQ>()>  // kNQ >= min(F*T, 1024) / 64
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sddmm_wpe<kNQ, KM, PF>(), 8))) void cheb_agg_sddmm_kernel(ChebAg a) {
  extern __shared__ float Dg[];  // [waves][K][F * T]
  stream_sig_store(a.sig, a.sig_v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int64_t wv = xcd_block(a.xcd_order) * 4 + w;
  if (wv >= (int64_t)a.B * a.N) return;
  const int b = (int)(wv / a.N), j = (int)(wv % a.N);
  const int FT = a.F * a.T;
  float* dg = Dg + (int64_t)w * a.K * FT;
  const int64_t NN = (int64_t)a.N * a.N;
  const float* gj = a.g + ((int64_t)b * a.N + j) * a.T * a.C;
  const int p0 = a.csc_ptr[j], p1 = a.csc_ptr[j + 1];
  for (int t0 = 0; t0 < a.T; t0 += 32) {
    const int Tc = min(32, a.T - t0);
    // A[m = t'][kk = c] = g[t'][c], kk = 16h + s: the lane's 16 consecutive floats of row t'
    float gv[16];
    row16(gj + (int64_t)(t0 + min(l32, Tc - 1)) * a.C + 16 * h, l32 < Tc && 16 * h < a.C, gv);
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k >= a.K) break;
      float bt[16];  // B[kk = c][n = f] = Theta_k[f][c]
      row16(a.thcat + (int64_t)min(l32, a.F - 1) * a.KC + k * a.C + 16 * h, l32 < a.F && 16 * h < a.C, bt);
      floatx16 acc = zero16();
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(gv[s], bt[s], acc, 0, 0, 0);
      if (l32 < a.F) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int tl = frow(r, h);
          if (tl < Tc) dg[(int64_t)k * FT + l32 * a.T + t0 + tl] = acc[r];  // [k][f][t], the x row's order
        }
      }
    }
  }
  wave_lds_sync();
  const float* xb = a.x + (int64_t)b * a.N * FT;
  // the KM x kE dot products of a batch reduce across the wave together (wave_sum_many):
  // lane owns value j = k kE + e, one lane of each 64 / NV does the stores
  constexpr int NV0 = KM * kE, NV = NV0 <= 16 ? 16 : (NV0 <= 32 ? 32 : 64);
  constexpr int LG = NV == 16 ? 4 : (NV == 32 ? 5 : 6);
  const int jl = (lane >> (6 - LG)) & (NV - 1), kl = jl / kE, el = jl - kl * kE;
  const bool owner = (lane & ((64 >> LG) - 1)) == 0 && jl < NV0 && kl < a.K;
  float csum = 0.f;  // this lane's share of c_j for order kl
  for (int c0 = p0; c0 < p1; c0 += 64) {
    const int nc = min(64, p1 - c0);
    const int rowl = a.csc_row[c0 + min(lane, nc - 1)];
    // rows of entries e0.. (elements e1 + lane + 64 q of each x row)
    auto gather = [&](int e0, int e1, float (&dst)[kE][kNQ]) {
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const float* xr = xb + (int64_t)rl_i(rowl, min(e0 + e, nc - 1)) * FT;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) dst[e][q] = xr[min(e1 + lane + 64 * q, FT - 1)];
      }
    };
    auto accum = [&](int e1, const float (&v)[kE][kNQ], float (&sf)[NV]) {
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        if (k >= a.K) break;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) {
          const int el2 = e1 + lane + 64 * q;
          const float d = el2 < FT ? dg[(int64_t)k * FT + el2] : 0.f;
#pragma unroll
          for (int e = 0; e < kE; ++e) sf[k * kE + e] = fmaf(v[e][q], d, sf[k * kE + e]);
        }
      }
    };
    float v[kE][kNQ];
    if constexpr (PF) gather(0, 0, v);
    for (int e0 = 0; e0 < nc; e0 += kE) {
      float vn[kE][kNQ];
      if constexpr (PF) gather(e0 + kE, 0, vn);  // the next batch's first element range, in flight meanwhile
      else gather(e0, 0, v);
      float sf[NV];  // dot products, value k kE + e (zero padded to NV: reduced in place)
#pragma unroll
      for (int jj = 0; jj < NV; ++jj) sf[jj] = 0.f;
      accum(0, v, sf);
      if constexpr (kNQ == 16) {  // F*T > 1024 (long series; nq_of gives 16): the rest of the rows
        for (int e1 = 64 * kNQ; e1 < FT; e1 += 64 * kNQ) {
          float vx[kE][kNQ];
          gather(e0, e1, vx);
          accum(e1, vx, sf);
        }
      }
      // the support weights of the owned entry, loaded before the reduction (independent of it)
      const int p = c0 + e0 + el;
      const bool mine = owner && e0 + el < nc;
      const int64_t zk = ((int64_t)b * a.K + kl) * a.nnz;
      float ps = 0.f, ts = 0.f;
      if (mine && a.dzs) {
        ps = a.psupp[zk + p];
        ts = a.tsupp[(int64_t)kl * a.nnz + p];
      }
      const float sv = wave_sum_many<NV>(sf);
      if (mine) {
        if (a.dzs) {
          const float dd = ps * (ts * sv);
          csum += dd;
          a.dzs[zk + p] = dd;
          if (a.dzs_r) a.dzs_r[zk + a.csc2csr[p]] = dd;
        } else {
          a.dW[((int64_t)b * a.K + kl) * NN + (int64_t)a.csc_row[p] * a.N + j] = sv;
        }
      }
      if constexpr (PF) {
#pragma unroll
        for (int e = 0; e < kE; ++e)
#pragma unroll
          for (int q = 0; q < kNQ; ++q) v[e][q] = vn[e][q];
      }
    }
  }
  if (a.dzs) {
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k >= a.K) break;
      const float c = wave_sum(owner && kl == k ? csum : 0.f);
      if (lane == 0) a.cc[((int64_t)b * a.K + k) * a.N + j] = c;
    }
  }
}

// ---------------------------------------------------------------------------------------
// backward SDDMM for T <= 16 (F T <= 512): one wave per (sample PAIR, j).  The two samples' g_j
// rows stack into one 32-row MFMA operand (m = bsel T + t: 2 T <= 32 rows of the 32 x 32 tile,
// where a single sample used T of them), so one chain of 16 MFMAs per order makes both samples'
// dagg_k; the column's support indices and weights are loaded once for both.  The support walk
// runs over virtual entries v = 2 e + bsel (sample bsel of entry e; batches of kE = 4 start at
// multiples of 4, so a value's sample is e & 1 at compile time).  Half the waves of the one-
// sample kernel, each with the same dependent load chain: PEMS08 B = 32 gives 2 720 waves, one
// round at 3 waves per SIMD, where 5 440 took two.  Same arithmetic per entry and order as the
// one-sample kernel (same dot-product order, same reduction): results bit-identical.
// ---------------------------------------------------------------------------------------
template <int kNQ, int KM>  // kNQ >= F * T / 64 (<= 8)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sddmm_wpe<kNQ, KM, true>(), 8))) void cheb_agg_sddmm2_kernel(ChebAg a) {
  static_assert(kNQ <= 8, "F T <= 512");
  extern __shared__ float Dg[];  // [waves][2][K][F * T]
  stream_sig_store(a.sig, a.sig_v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int64_t wv = xcd_block(a.xcd_order) * 4 + w;
  const int npair = (a.B + 1) >> 1;
  if (wv >= (int64_t)npair * a.N) return;
  const int bp = (int)(wv / a.N), j = (int)(wv % a.N), b0 = 2 * bp, nb = min(2, a.B - b0);
  const int T = a.T, FT = a.F * T;
  float* dg = Dg + (int64_t)w * 2 * a.K * FT;
  const int64_t NN = (int64_t)a.N * a.N;
  const int p0 = a.csc_ptr[j], p1 = a.csc_ptr[j + 1];
  {
    // A[m][kk = c] = g_{b0 + bsel}[t][c], m = bsel T + t, kk = 16h + s
    const int bs = l32 >= T ? 1 : 0, tl = l32 - bs * T;
    const bool mv = l32 < nb * T;
    float gv[16];
    row16(a.g + (((int64_t)(b0 + (mv ? bs : 0)) * a.N + j) * T + (mv ? tl : 0)) * a.C + 16 * h, mv && 16 * h < a.C, gv);
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k >= a.K) break;
      float bt[16];  // B[kk = c][n = f] = Theta_k[f][c]
      row16(a.thcat + (int64_t)min(l32, a.F - 1) * a.KC + k * a.C + 16 * h, l32 < a.F && 16 * h < a.C, bt);
      floatx16 acc = zero16();
#pragma unroll
      for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(gv[s], bt[s], acc, 0, 0, 0);
      if (l32 < a.F) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = frow(r, h), ms = m >= T ? 1 : 0, mt = m - ms * T;
          if (m < nb * T) dg[(int64_t)(ms * a.K + k) * FT + l32 * T + mt] = acc[r];  // [bsel][k][f][t]
        }
      }
    }
  }
  wave_lds_sync();
  const float* xb0 = a.x + (int64_t)b0 * a.N * FT;
  const float* xb1 = a.x + (int64_t)(b0 + nb - 1) * a.N * FT;
  constexpr int NV0 = KM * kE, NV = NV0 <= 16 ? 16 : (NV0 <= 32 ? 32 : 64);
  constexpr int LG = NV == 16 ? 4 : (NV == 32 ? 5 : 6);
  const int jl = (lane >> (6 - LG)) & (NV - 1), kl = jl / kE, el = jl - kl * kE, bsl = el & 1;
  const bool owner = (lane & ((64 >> LG) - 1)) == 0 && jl < NV0 && kl < a.K && bsl < nb;
  float csum = 0.f;  // this lane's share of c_j for (order kl, sample b0 + bsl)
  for (int c0 = p0; c0 < p1; c0 += 32) {  // 32 entries = 64 virtual entries per chunk
    const int nc = min(32, p1 - c0), nv = 2 * nc;
    const int rowl = a.csc_row[c0 + min(lane, nc - 1)];
    auto gather = [&](int e0, float (&dst)[kE][kNQ]) {
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const int ve = min(e0 + e, nv - 1);  // (e0 even: ve & 1 == e & 1 unless clamped)
        const float* xr = ((e & 1) ? xb1 : xb0) + (int64_t)rl_i(rowl, ve >> 1) * FT;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) dst[e][q] = xr[min(lane + 64 * q, FT - 1)];
      }
    };
    float v[kE][kNQ];
    gather(0, v);
    for (int e0 = 0; e0 < nv; e0 += kE) {
      float vn[kE][kNQ];
      gather(e0 + kE, vn);  // the next batch, in flight meanwhile
      float sf[NV];
#pragma unroll
      for (int jj = 0; jj < NV; ++jj) sf[jj] = 0.f;
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        if (k >= a.K) break;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) {
          const int el2 = lane + 64 * q;
          const float d0 = el2 < FT ? dg[(int64_t)k * FT + el2] : 0.f;
          const float d1 = el2 < FT ? dg[(int64_t)(a.K + k) * FT + el2] : 0.f;
#pragma unroll
          for (int e = 0; e < kE; ++e) sf[k * kE + e] = fmaf(v[e][q], (e & 1) ? d1 : d0, sf[k * kE + e]);
        }
      }
      const int ve = e0 + el, p = c0 + (ve >> 1);
      const bool mine = owner && ve < nv;
      const int64_t zk = ((int64_t)(b0 + bsl) * a.K + kl) * a.nnz;
      float ps = 0.f, ts = 0.f;
      if (mine && a.dzs) {
        ps = a.psupp[zk + p];
        ts = a.tsupp[(int64_t)kl * a.nnz + p];
      }
      const float sv = wave_sum_many<NV>(sf);
      if (mine) {
        if (a.dzs) {
          const float dd = ps * (ts * sv);
          csum += dd;
          a.dzs[zk + p] = dd;
          if (a.dzs_r) a.dzs_r[zk + a.csc2csr[p]] = dd;
        } else {
          a.dW[((int64_t)(b0 + bsl) * a.K + kl) * NN + (int64_t)a.csc_row[p] * a.N + j] = sv;
        }
      }
#pragma unroll
      for (int e = 0; e < kE; ++e)
#pragma unroll
        for (int q = 0; q < kNQ; ++q) v[e][q] = vn[e][q];
    }
  }
  if (a.dzs) {
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k >= a.K) break;
#pragma unroll
      for (int bs = 0; bs < 2; ++bs) {
        const float c = wave_sum(owner && kl == k && bsl == bs ? csum : 0.f);
        if (lane == 0 && bs < nb) a.cc[((int64_t)(b0 + bs) * a.K + k) * a.N + j] = c;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// backward transposed SpMM: one wave per (b, i, time chunk).  The row's neighbours g_j are
// gathered once: h_k = sum_{j in supp_row(i)} W_k[i,j] g_j (Tc x C) for every k, then
// dx_i[f, t'] += sum_k sum_c Theta_k[f][c] h_k[t'][c] on the matrix cores.
// ---------------------------------------------------------------------------------------
template <int kNQ, int KM>  // kNQ >= Tc * C / 64
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(gather_wpe<kNQ, KM>(), 8))) void cheb_agg_spmm_t_kernel(ChebAg a) {
  __shared__ float Hs[4][32 * kAs];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int64_t wv = xcd_block(a.xcd_order) * 4 + w;
  if (wv >= (int64_t)a.B * a.N) return;
  const int b = (int)(wv / a.N), i = (int)(wv % a.N);
  const int t0 = blockIdx.y * 32, Tc = min(32, a.T - t0), nel = Tc * a.C;
  const int64_t NN = (int64_t)a.N * a.N;
  float* hs = Hs[w];
  // elements e = lane + 64 q of the (Tc x C) chunk of a g row: offset and LDS slot [t'][c]
  int go[kNQ], lo[kNQ];
#pragma unroll
  for (int q = 0; q < kNQ; ++q) {
    const int e = min(lane + 64 * q, nel - 1), tl = e / a.C, c = e - tl * a.C;
    go[q] = (t0 + tl) * a.C + c;
    lo[q] = tl * kAs + c;
  }
  const int q0 = a.csr_ptr[i], q1 = a.csr_ptr[i + 1];
  const float* gb = a.g + (int64_t)b * a.N * a.T * a.C;
  float hv[KM][kNQ];
#pragma unroll
  for (int k = 0; k < KM; ++k)
#pragma unroll
    for (int q = 0; q < kNQ; ++q) hv[k][q] = 0.f;
  for (int c0 = q0; c0 < q1; c0 += 64) {
    const int nc = min(64, q1 - c0), pl = c0 + min(lane, nc - 1);
    const int coll = a.csr_col[pl];
    float wl[KM];  // W_k[i, col] of this lane's entry (0 past the chunk)
    {
      const int ci = a.wsupp ? a.csr2csc[pl] : 0;
      const int64_t o = (int64_t)i * a.N + coll;
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        float ww = 0.f;
        if (k < a.K)
          ww = a.wsupp ? a.wsupp[((int64_t)b * a.K + k) * a.nnz + ci]
                       : a.cheb[(int64_t)k * NN + o] * a.P[((int64_t)b * a.K + k) * NN + o];
        wl[k] = lane < nc ? ww : 0.f;
      }
    }
    auto gather = [&](int e0, float (&dst)[kE][kNQ]) {
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const float* gr = gb + (int64_t)rl_i(coll, min(e0 + e, nc - 1)) * a.T * a.C;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) dst[e][q] = gr[go[q]];
      }
    };
    float v[kE][kNQ];
    if constexpr (agg_prefetch<kNQ>()) gather(0, v);
    for (int e0 = 0; e0 < nc; e0 += kE) {
      float vn[kE][kNQ];
      if constexpr (agg_prefetch<kNQ>()) gather(e0 + kE, vn);  // the next batch, in flight meanwhile
      else gather(e0, v);
#pragma unroll
      for (int k = 0; k < KM; ++k)
#pragma unroll
        for (int e = 0; e < kE; ++e) {
          const float wk = rl_f(wl[k], e0 + e);  // e0 + e <= 63; lanes >= nc hold 0
#pragma unroll
          for (int q = 0; q < kNQ; ++q) hv[k][q] = fmaf(wk, v[e][q], hv[k][q]);
        }
      if constexpr (agg_prefetch<kNQ>()) {
#pragma unroll
        for (int e = 0; e < kE; ++e)
#pragma unroll
          for (int q = 0; q < kNQ; ++q) v[e][q] = vn[e][q];
      }
    }
  }
  floatx16 acc = zero16();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k >= a.K) break;
    float bt[16];  // B[kk = c][n = f] = Theta_k[f][c], kk = 16h + s
    row16(a.thcat + (int64_t)min(l32, a.F - 1) * a.KC + k * a.C + 16 * h, l32 < a.F && 16 * h < a.C, bt);
#pragma unroll
    for (int q = 0; q < kNQ; ++q)
      if (lane + 64 * q < nel) hs[lo[q]] = hv[k][q];
    wave_lds_sync();
    // D[m = t'][n = f] += sum_c h_k[t'][c] Theta_k[f][c]
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int c = 16 * h + s;
      const float av = (c < a.C && l32 < Tc) ? hs[l32 * kAs + c] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bt[s], acc, 0, 0, 0);
    }
    wave_lds_sync();
  }
  if (l32 >= a.F) return;
  float* dxr = a.dx + ((int64_t)b * a.N + i) * a.F * a.T + (int64_t)l32 * a.T + t0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int tl = frow(r, h);
    if (tl < Tc) dxr[tl] = a.dx_beta * dxr[tl] + acc[r];
  }
}

// ---------------------------------------------------------------------------------------
// transposed SpMM for T <= 16 (T C <= 512): one wave per (sample PAIR, i), as the pair forward:
// h_k of sample bsel accumulated over virtual entries v = 2 e + bsel of the row's support, the
// two samples' h_k stacked into one MFMA A operand (m = bsel T + t) for the Theta_k chain.
// ---------------------------------------------------------------------------------------
template <int kNQ, int KM>  // kNQ >= T * C / 64 (<= 8)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(gather_wpe<kNQ, 2 * KM>(), 8))) void cheb_agg_spmm_t2_kernel(ChebAg a) {
  static_assert(kNQ <= 8, "T C <= 512");
  __shared__ float Hs[4][32 * kAs];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int64_t wv = xcd_block(a.xcd_order) * 4 + w;
  const int npair = (a.B + 1) >> 1;
  if (wv >= (int64_t)npair * a.N) return;
  const int bp = (int)(wv / a.N), i = (int)(wv % a.N), b0 = 2 * bp, nb = min(2, a.B - b0);
  const int T = a.T, TC = T * a.C;
  const int64_t NN = (int64_t)a.N * a.N;
  float* hs = Hs[w];
  int lo[kNQ];  // element e = lane + 64 q of a g row (t, c): LDS slot [m = t][c] (+ T rows for sample 1)
#pragma unroll
  for (int q = 0; q < kNQ; ++q) {
    const int e = min(lane + 64 * q, TC - 1), tl = e / a.C, c = e - tl * a.C;
    lo[q] = tl * kAs + c;
  }
  const int q0 = a.csr_ptr[i], q1 = a.csr_ptr[i + 1];
  const float* gb0 = a.g + (int64_t)b0 * a.N * TC;
  const float* gb1 = a.g + (int64_t)(b0 + nb - 1) * a.N * TC;
  float hv[2][KM][kNQ];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int k = 0; k < KM; ++k)
#pragma unroll
      for (int q = 0; q < kNQ; ++q) hv[s][k][q] = 0.f;
  for (int c0 = q0; c0 < q1; c0 += 32) {
    const int nc = min(32, q1 - c0), nv = 2 * nc, pl = c0 + min(lane, nc - 1);
    const int coll = a.csr_col[pl];
    float wl[2][KM];
    {
      const int ci = a.wsupp ? a.csr2csc[pl] : 0;
      const int64_t o = (int64_t)i * a.N + coll;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int k = 0; k < KM; ++k) {
          float ww = 0.f;
          if (k < a.K) {
            const int b = b0 + min(s, nb - 1);
            ww = a.wsupp ? a.wsupp[((int64_t)b * a.K + k) * a.nnz + ci]
                         : a.cheb[(int64_t)k * NN + o] * a.P[((int64_t)b * a.K + k) * NN + o];
          }
          wl[s][k] = lane < nc ? ww : 0.f;
        }
    }
    auto gather = [&](int e0, float (&dst)[kE][kNQ]) {
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const int ve = min(e0 + e, nv - 1);
        const float* gr = ((e & 1) ? gb1 : gb0) + (int64_t)rl_i(coll, ve >> 1) * TC;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) dst[e][q] = gr[min(lane + 64 * q, TC - 1)];
      }
    };
    float v[kE][kNQ];
    gather(0, v);
    for (int e0 = 0; e0 < nv; e0 += kE) {
      float vn[kE][kNQ];
      gather(e0 + kE, vn);
#pragma unroll
      for (int k = 0; k < KM; ++k)
#pragma unroll
        for (int e = 0; e < kE; ++e) {
          const float wk = rl_f(wl[e & 1][k], min((e0 + e) >> 1, 31));
          const float wz = e0 + e < nv ? wk : 0.f;
#pragma unroll
          for (int q = 0; q < kNQ; ++q) hv[e & 1][k][q] = fmaf(wz, v[e][q], hv[e & 1][k][q]);
        }
#pragma unroll
      for (int e = 0; e < kE; ++e)
#pragma unroll
        for (int q = 0; q < kNQ; ++q) v[e][q] = vn[e][q];
    }
  }
  floatx16 acc = zero16();
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    if (k >= a.K) break;
    float bt[16];  // B[kk = c][n = f] = Theta_k[f][c], kk = 16h + s
    row16(a.thcat + (int64_t)min(l32, a.F - 1) * a.KC + k * a.C + 16 * h, l32 < a.F && 16 * h < a.C, bt);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (s >= nb) break;
#pragma unroll
      for (int q = 0; q < kNQ; ++q)
        if (lane + 64 * q < TC) hs[lo[q] + s * T * kAs] = hv[s][k][q];
    }
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < 16; ++s) {  // D[m][n = f] += sum_c h_k[m][c] Theta_k[f][c]
      const int c = 16 * h + s;
      const float av = (c < a.C && l32 < nb * T) ? hs[l32 * kAs + c] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bt[s], acc, 0, 0, 0);
    }
    wave_lds_sync();
  }
  if (l32 >= a.F) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = frow(r, h), ms = m >= T ? 1 : 0, mt = m - ms * T;
    if (m < nb * T) {
      float* d = a.dx + ((int64_t)(b0 + ms) * a.N + i) * a.F * T + (int64_t)l32 * T + mt;
      *d = a.dx_beta * *d + acc[r];
    }
  }
}

int nq_of(int n) { return n <= 64 ? 1 : n <= 128 ? 2 : n <= 256 ? 4 : n <= 384 ? 6 : n <= 512 ? 8 : n <= 768 ? 12 : 16; }
int km_of(int K) { return K <= 2 ? 2 : K <= 3 ? 3 : K <= 5 ? 5 : 8; }

ChebAg with_order(const ChebAg& a0) {
  ChebAg a = a0;
  // XCD-aware order when one batch's gathered slice (x: N*F*T floats) fits a 4 MB L2
  a.xcd_order = (int64_t)a.N * a.F * a.T * (int64_t)sizeof(float) <= (int64_t(4) << 20) ? 1 : 0;
  return a;
}

unsigned grid_rows(int64_t waves) { return (unsigned)(cdiv64(cdiv64(waves, 4), 8) * 8); }

// kernel<kNQ, KM> for the runtime (nq, km)
struct Launch {
  const ChebAg& a;
  dim3 grid;
  size_t lds;
  hipStream_t st;
};

template <template <int, int> class Fn>
void dispatch(int nq, int km, const Launch& l) {
#define DS_KM(NQ)                                   \
  switch (km) {                                     \
    case 2: Fn<NQ, 2>::run(l); return;              \
    case 3: Fn<NQ, 3>::run(l); return;              \
    case 5: Fn<NQ, 5>::run(l); return;              \
    default: Fn<NQ, 8>::run(l); return;             \
  }
  switch (nq) {
    case 1: DS_KM(1)
    case 2: DS_KM(2)
    case 4: DS_KM(4)
    case 6: DS_KM(6)
    case 8: DS_KM(8)
    case 12: DS_KM(12)
    default: DS_KM(16)
  }
#undef DS_KM
}

template <int NQ, int KM>
struct FwdL {
  static void run(const Launch& l) {
    hipLaunchKernelGGL((cheb_agg_fwd_kernel<NQ, KM>), l.grid, dim3(256), 0, l.st, l.a);
  }
};
template <int NQ, int KM>
struct Fwd2L {
  static void run(const Launch& l) {
    if constexpr (NQ <= 8) hipLaunchKernelGGL((cheb_agg_fwd2_kernel<NQ, KM>), l.grid, dim3(256), 0, l.st, l.a);
  }
};
template <int NQ, int KM>
struct SddmmL {
  static void run(const Launch& l) {
    if (l.lds > (64u << 10)) {
      static bool done = false;  // raise the kernel's dynamic-LDS limit once
      if (!done) {
        (void)hipFuncSetAttribute((const void*)cheb_agg_sddmm_kernel<NQ, KM>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10);
        done = true;
      }
    }
    static const bool nopf = getenv("DSTAGNN_SDDMM_NOPF") && atoi(getenv("DSTAGNN_SDDMM_NOPF")) != 0;
    if constexpr (NQ <= 6 && KM <= 3) {
      if (nopf) {
        if (l.lds > (64u << 10)) {
          static bool done2 = false;
          if (!done2) {
            (void)hipFuncSetAttribute((const void*)cheb_agg_sddmm_kernel<NQ, KM, false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10);
            done2 = true;
          }
        }
        hipLaunchKernelGGL((cheb_agg_sddmm_kernel<NQ, KM, false>), l.grid, dim3(256), l.lds, l.st, l.a);
        return;
      }
    }
    hipLaunchKernelGGL((cheb_agg_sddmm_kernel<NQ, KM>), l.grid, dim3(256), l.lds, l.st, l.a);
  }
};
template <int NQ, int KM>
struct Sddmm2L {
  static void run(const Launch& l) {
    if constexpr (NQ <= 8) {
      if (l.lds > (64u << 10)) {
        static bool done = false;
        if (!done) {
          (void)hipFuncSetAttribute((const void*)cheb_agg_sddmm2_kernel<NQ, KM>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10);
          done = true;
        }
      }
      hipLaunchKernelGGL((cheb_agg_sddmm2_kernel<NQ, KM>), l.grid, dim3(256), l.lds, l.st, l.a);
    }
  }
};
template <int NQ, int KM>
struct SpmmT2L {
  static void run(const Launch& l) {
    if constexpr (NQ <= 8) hipLaunchKernelGGL((cheb_agg_spmm_t2_kernel<NQ, KM>), l.grid, dim3(256), 0, l.st, l.a);
  }
};
template <int NQ, int KM>
struct SpmmTL {
  static void run(const Launch& l) {
    hipLaunchKernelGGL((cheb_agg_spmm_t_kernel<NQ, KM>), l.grid, dim3(256), 0, l.st, l.a);
  }
};

int check(const ChebAg& a) {
  if (!cheb_agg_ok(a.F, a.C, a.K, a.T)) {
    set_last_error("cheb_agg: F in 1..32, C in {16, 32}, K in 1..8, SDDMM LDS 16*K*F*T <= 160 KB");
    return DSTAGNN_E_SHAPE;
  }
  return 0;
}

size_t sddmm_lds_bytes(int K, int F, int T) { return (size_t)4 * K * F * T * sizeof(float); }

}  // namespace

// F <= 32 (one MFMA contraction / tile side), C = 16 or 32 (16-float operand rows), K <= 8
// (the kernels' order templates), and the backward SDDMM's per-workgroup LDS image of the K
// dagg_k = Theta_k g_j^T tiles (4 waves x K x F x T floats) within the CU's 160 KB — checked
// here, where the block picks its path, so a shape the backward cannot run (e.g. K = 3, F = 32,
// T = 144) takes the Theta-first sparse path from the forward on
bool cheb_agg_ok(int F, int C, int K, int T) {
  return F >= 1 && F <= 32 && (C == 16 || C == 32) && K >= 1 && K <= 8 && T >= 1 &&
         sddmm_lds_bytes(K, F, T) <= (160u << 10);
}

int op_cheb_agg_fwd(const ChebAg& a0, hipStream_t st) {
  DS_TRY(check(a0));
  const ChebAg a = with_order(a0);
  // T <= 16: sample pairs per wave (cheb_agg_fwd2_kernel; DSTAGNN_AGG_PAIR=0: one sample)
  static const bool pair_env = !getenv("DSTAGNN_AGG_PAIR") || atoi(getenv("DSTAGNN_AGG_PAIR")) != 0;
  if (pair_env && a.T <= 16 && a.F * a.T <= 512)
    dispatch<Fwd2L>(nq_of(a.F * a.T), km_of(a.K), Launch{a, dim3(grid_rows((int64_t)((a.B + 1) / 2) * a.N)), 0, st});
  else
    dispatch<FwdL>(nq_of(a.F * std::min(32, a.T)), km_of(a.K),
                   Launch{a, dim3(grid_rows((int64_t)a.B * a.N), (unsigned)cdiv64(a.T, 32)), 0, st});
  DS_CHECK_LAUNCH();
  return 0;
}

int op_cheb_agg_sddmm(const ChebAg& a0, hipStream_t st) {
  DS_TRY(check(a0));
  ChebAg a = with_order(a0);
  const StreamSig sg = peek_stream_sig(st);  // carries a pending stream signal (common.hpp)
  a.sig = sg.p;
  a.sig_v = sg.v;
  const int FT = a.F * a.T;
  // T <= 16: sample pairs per wave (cheb_agg_sddmm2_kernel; DSTAGNN_SDDMM_PAIR=0: one sample)
  // (DSTAGNN_SDDMM_NOPF=1 names a variant of the one-sample kernel: it implies PAIR=0)
  static const bool pair_env = (!getenv("DSTAGNN_SDDMM_PAIR") || atoi(getenv("DSTAGNN_SDDMM_PAIR")) != 0) &&
                               !(getenv("DSTAGNN_SDDMM_NOPF") && atoi(getenv("DSTAGNN_SDDMM_NOPF")) != 0);
  const bool pair = pair_env && a.T <= 16 && FT <= 512 && 2 * sddmm_lds_bytes(a.K, a.F, a.T) <= (160u << 10);
  if (pair) {
    dispatch<Sddmm2L>(nq_of(FT), km_of(a.K),
                      Launch{a, dim3(grid_rows((int64_t)((a.B + 1) / 2) * a.N)), 2 * sddmm_lds_bytes(a.K, a.F, a.T), st});
  } else {
    const size_t lds = sddmm_lds_bytes(a.K, a.F, a.T);
    dispatch<SddmmL>(nq_of(std::min(FT, 1024)), km_of(a.K), Launch{a, dim3(grid_rows((int64_t)a.B * a.N)), lds, st});
  }
  DS_CHECK_LAUNCH();
  if (sg.p) DS_TRY(stream_sig_sent(st, sg));
  return 0;
}

int op_cheb_agg_spmm_t(const ChebAg& a0, hipStream_t st) {
  DS_TRY(check(a0));
  const ChebAg a = with_order(a0);
  static const bool pair_env = !getenv("DSTAGNN_AGG_PAIR") || atoi(getenv("DSTAGNN_AGG_PAIR")) != 0;
  if (pair_env && a.T <= 16 && a.T * a.C <= 512) {  // sample pairs per wave (cheb_agg_spmm_t2_kernel)
    dispatch<SpmmT2L>(nq_of(a.T * a.C), km_of(a.K), Launch{a, dim3(grid_rows((int64_t)((a.B + 1) / 2) * a.N)), 0, st});
    DS_CHECK_LAUNCH();
    return 0;
  }
  dispatch<SpmmTL>(nq_of(std::min(32, a.T) * a.C), km_of(a.K),
                   Launch{a, dim3(grid_rows((int64_t)a.B * a.N), (unsigned)cdiv64(a.T, 32)), 0, st});
  DS_CHECK_LAUNCH();
  return 0;
}
