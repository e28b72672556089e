// cheb_agg.hip — the block's sparse Chebyshev convolution in aggregate-first order (gfx950).
//
// cheb_conv_withSAt (model/DSTAGNN_my.py:117-133) computes, per timestep t and order k,
//   out_t += (T_k o P_k)^T x_t Theta_k        then ReLU           (W_k := T_k o P_k)
// The Theta-first order (cheb_sparse.hip) multiplies x by all K Thetas first — a GEMM that
// writes K*C*T floats per node (25 MB at PEMS08 B=32) — and then gathers those rows.  Here the
// gather comes first, on x itself (F*T floats per source node: K times fewer bytes), and the
// K small (T x F)(F x C) products per destination node run on the wave's own matrix cores:
//
//   fwd      agg_k[j] = sum_{i in supp(j)} W_k[i,j] x_i          (F x T, saved for dTheta)
//            X[j]     = ReLU( sum_k agg_k[j]^T Theta_k )          (T x C)
//   sddmm    dagg_k[j] = Theta_k g_j^T                             (F x T, wave-local, LDS)
//            dW_k[i,j] = < x_i, dagg_k[j] >  on the support      (the softmax backward's input)
//   spmm_t   dx_i    += sum_k Theta_k ( sum_{j in supp_row(i)} W_k[i,j] g_j )^T
//   dTheta_k = sum_{b,j,t} agg_k[b,j,:,t] g[b,j,t,:]  — one GEMM (block.hip)
//
// so the Theta GEMM of the forward and the dx GEMM of the backward disappear together with
// the (B,N,K,C,T) tensor and its gradient.  g = d(pre-ReLU X), layout (B,N,T,C); x (B,N,F,T).
// MFMA v_mfma_f32_32x32x2_f32: lane l supplies A[m = l&31][kk] and B[kk][n = l&31], lane half
// h = l>>5 taking the contraction index kk = 2s + h at step s; the accumulator holds
// D[m = (r&3) + 8(r>>2) + 4h][n = l&31] in register r.  Time chunks of <= 32 steps (m = t).
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

// XCD-aware row-block order (cheb_sparse.hip): each XCD walks one contiguous eighth of the rows
__device__ __forceinline__ int64_t xcd_block(int on) {
  const int64_t p = blockIdx.x;
  if (!on) return p;
  const int64_t per = gridDim.x >> 3;
  return (p & 7) * per + (p >> 3);
}

constexpr int kE = 4;      // support entries per batch (one memory round per batch)
constexpr int kAs = 33;    // LDS row stride of a 32 x 32 operand tile

// the weight of support entry p of column j (CSC position), order k
__device__ __forceinline__ float wgt(const ChebAg& a, int b, int k, int p, int i, int j) {
  if (a.wsupp) return a.wsupp[((int64_t)b * a.K + k) * a.nnz + p];
  const int64_t o = (int64_t)i * a.N + j, NN = (int64_t)a.N * a.N;
  return a.cheb[(int64_t)k * NN + o] * a.P[((int64_t)b * a.K + k) * NN + o];
}

// ---------------------------------------------------------------------------------------
// forward: one wave per (b, j, time chunk)
// ---------------------------------------------------------------------------------------
template <int kNQ>  // >= F * Tc / 64
__global__ __launch_bounds__(256) void cheb_agg_fwd_kernel(ChebAg a) {
  __shared__ float As[4][32 * kAs];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int64_t wv = xcd_block(a.xcd_order) * 4 + w;
  if (wv >= (int64_t)a.B * a.N) return;
  const int b = (int)(wv / a.N), j = (int)(wv % a.N);
  const int t0 = blockIdx.y * 32, Tc = min(32, a.T - t0), FT = a.F * a.T, nel = a.F * Tc;
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
  floatx16 acc = zero16();
  for (int k = 0; k < a.K; ++k) {
    // Theta_k as the B operand: B[kk = f][n = c], f = 2s + h (zero past F / C)
    float bt[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int f = 2 * s + h;
      bt[s] = (f < a.F && l32 < a.C) ? a.thcat[(int64_t)f * a.KC + k * a.C + l32] : 0.f;
    }
    float ag[kNQ];
#pragma unroll
    for (int q = 0; q < kNQ; ++q) ag[q] = 0.f;
    for (int pb = p0; pb < p1; pb += kE) {
      int rows[kE];
#pragma unroll
      for (int e = 0; e < kE; ++e) rows[e] = a.csc_row[min(pb + e, p1 - 1)];
      float wv_[kE], v[kE][kNQ];
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const float ww = wgt(a, b, k, min(pb + e, p1 - 1), rows[e], j);
        wv_[e] = pb + e < p1 ? ww : 0.f;
        const float* xr = xb + (int64_t)rows[e] * FT;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) v[e][q] = xr[xo[q]];
      }
#pragma unroll
      for (int e = 0; e < kE; ++e)
#pragma unroll
        for (int q = 0; q < kNQ; ++q) ag[q] = fmaf(wv_[e], v[e][q], ag[q]);
    }
    // agg_k[j] saved for the Theta gradient, and staged as the MFMA A operand [f][t']
    float* sv = a.agg + (((int64_t)b * a.N + j) * a.K + k) * FT;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < kNQ; ++q)
      if (lane + 64 * q < nel) {
        sv[xo[q]] = ag[q];
        at[lo[q]] = ag[q];
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // D[m = t'][n = c] += sum_f agg_k[f][t'] Theta_k[f][c]
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int f = 2 * s + h;
      const float av = (f < a.F && l32 < Tc) ? at[f * kAs + l32] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bt[s], acc, 0, 0, 0);
    }
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
// backward SDDMM: one wave per (b, j, k).  dagg = Theta_k g_j^T (F x T) on the wave's matrix
// cores into LDS, then dW_k[i, j] = <x_i, dagg> for the column's support (flash path: the
// softmax backward's support terms dzs = P T dW and c_j instead, as cheb_sparse.hip).
// ---------------------------------------------------------------------------------------
template <int kNQ>  // >= min(F*T, 1024) / 64
__global__ __launch_bounds__(256) void cheb_agg_sddmm_kernel(ChebAg a) {
  extern __shared__ float Dg[];  // [4 waves][F * T]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int64_t wv0 = xcd_block(a.xcd_order) * 4 + w;
  if (wv0 >= (int64_t)a.B * a.N * a.K) return;
  const int k = (int)(wv0 % a.K);
  const int64_t wv = wv0 / a.K;
  const int b = (int)(wv / a.N), j = (int)(wv % a.N);
  const int FT = a.F * a.T;
  float* dg = Dg + (int64_t)w * FT;
  const int64_t NN = (int64_t)a.N * a.N;
  // Theta_k as the B operand of D[m = t'][n = f] = sum_c g[t'][c] Theta_k[f][c]: kk = c = 2s + h
  float bt[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int c = 2 * s + h;
    bt[s] = (c < a.C && l32 < a.F) ? a.thcat[(int64_t)l32 * a.KC + k * a.C + c] : 0.f;
  }
  const float* gj = a.g + ((int64_t)b * a.N + j) * a.T * a.C;
  for (int t0 = 0; t0 < a.T; t0 += 32) {
    const int Tc = min(32, a.T - t0);
    floatx16 acc = zero16();
    const float* gr = gj + (int64_t)(t0 + min(l32, Tc - 1)) * a.C;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int c = 2 * s + h;
      const float av = (c < a.C && l32 < Tc) ? gr[c] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bt[s], acc, 0, 0, 0);
    }
    if (l32 < a.F) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int tl = frow(r, h);
        if (tl < Tc) dg[l32 * a.T + t0 + tl] = acc[r];  // [f][t], the x row's own order
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int p0 = a.csc_ptr[j], p1 = a.csc_ptr[j + 1];
  const int64_t zk = ((int64_t)b * a.K + k) * a.nnz;
  const float* xb = a.x + (int64_t)b * a.N * FT;
  float csum = 0.f;
  for (int pb = p0; pb < p1; pb += kE) {
    int rows[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) rows[e] = a.csc_row[min(pb + e, p1 - 1)];
    float pv[kE] = {}, tv[kE] = {};
    int rp[kE] = {};
    if (a.dzs) {
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const int p = min(pb + e, p1 - 1);
        pv[e] = a.psupp[zk + p];
        tv[e] = a.tsupp[(int64_t)k * a.nnz + p];
        rp[e] = a.dzs_r ? a.csc2csr[p] : 0;
      }
    }
    float s4[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) s4[e] = 0.f;
    for (int e0 = 0; e0 < FT; e0 += 64 * kNQ) {  // one pass unless F*T > 64 kNQ (long series)
      float v[kE][kNQ], d[kNQ];
#pragma unroll
      for (int q = 0; q < kNQ; ++q) d[q] = e0 + lane + 64 * q < FT ? dg[e0 + lane + 64 * q] : 0.f;
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const float* xr = xb + (int64_t)rows[e] * FT;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) v[e][q] = xr[min(e0 + lane + 64 * q, FT - 1)];
      }
#pragma unroll
      for (int e = 0; e < kE; ++e)
#pragma unroll
        for (int q = 0; q < kNQ; ++q) s4[e] = fmaf(v[e][q], d[q], s4[e]);
    }
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const float s = wave_sum(s4[e]);
      const int p = pb + e;
      if (p >= p1) break;
      if (a.dzs) {
        const float dd = pv[e] * (tv[e] * s);
        csum += dd;
        if (lane == 0) {
          a.dzs[zk + p] = dd;
          if (a.dzs_r) a.dzs_r[zk + rp[e]] = dd;
        }
      } else if (lane == 0) {
        a.dW[((int64_t)b * a.K + k) * NN + (int64_t)rows[e] * a.N + j] = s;
      }
    }
  }
  if (a.dzs && lane == 0) a.cc[((int64_t)b * a.K + k) * a.N + j] = csum;
}

// ---------------------------------------------------------------------------------------
// backward transposed SpMM: one wave per (b, i, time chunk).  h_k = sum_{j in supp_row(i)}
// W_k[i,j] g_j (Tc x C, LDS), then dx_i[f, t'] += sum_k sum_c Theta_k[f][c] h_k[t'][c].
// ---------------------------------------------------------------------------------------
template <int kNQ>  // >= Tc * C / 64
__global__ __launch_bounds__(256) void cheb_agg_spmm_t_kernel(ChebAg a) {
  __shared__ float Hs[4][32 * kAs];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
  const int64_t wv = xcd_block(a.xcd_order) * 4 + w;
  if (wv >= (int64_t)a.B * a.N) return;
  const int b = (int)(wv / a.N), i = (int)(wv % a.N);
  const int t0 = blockIdx.y * 32, Tc = min(32, a.T - t0), nel = Tc * a.C;
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
  floatx16 acc = zero16();
  for (int k = 0; k < a.K; ++k) {
    float bt[16];  // B[kk = c][n = f] = Theta_k[f][c], c = 2s + h
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int c = 2 * s + h;
      bt[s] = (c < a.C && l32 < a.F) ? a.thcat[(int64_t)l32 * a.KC + k * a.C + c] : 0.f;
    }
    float hv[kNQ];
#pragma unroll
    for (int q = 0; q < kNQ; ++q) hv[q] = 0.f;
    for (int pb = q0; pb < q1; pb += kE) {
      int cols[kE], ci[kE];
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const int p = min(pb + e, q1 - 1);
        cols[e] = a.csr_col[p];
        ci[e] = a.wsupp ? a.csr2csc[p] : 0;
      }
      float wv_[kE], v[kE][kNQ];
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        float ww;
        if (a.wsupp) {
          ww = a.wsupp[((int64_t)b * a.K + k) * a.nnz + ci[e]];
        } else {
          const int64_t o = (int64_t)i * a.N + cols[e], NN = (int64_t)a.N * a.N;
          ww = a.cheb[(int64_t)k * NN + o] * a.P[((int64_t)b * a.K + k) * NN + o];
        }
        wv_[e] = pb + e < q1 ? ww : 0.f;
        const float* gr = gb + (int64_t)cols[e] * a.T * a.C;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) v[e][q] = gr[go[q]];
      }
#pragma unroll
      for (int e = 0; e < kE; ++e)
#pragma unroll
        for (int q = 0; q < kNQ; ++q) hv[q] = fmaf(wv_[e], v[e][q], hv[q]);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < kNQ; ++q)
      if (lane + 64 * q < nel) hs[lo[q]] = hv[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // D[m = t'][n = f] += sum_c h_k[t'][c] Theta_k[f][c]
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int c = 2 * s + h;
      const float av = (c < a.C && l32 < Tc) ? hs[l32 * kAs + c] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bt[s], acc, 0, 0, 0);
    }
  }
  if (l32 >= a.F) return;
  float* dxr = a.dx + ((int64_t)b * a.N + i) * a.F * a.T + (int64_t)l32 * a.T + t0;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int tl = frow(r, h);
    if (tl < Tc) dxr[tl] = a.dx_beta * dxr[tl] + acc[r];
  }
}

int nq_of(int n) { return n <= 64 ? 1 : n <= 128 ? 2 : n <= 256 ? 4 : n <= 384 ? 6 : n <= 512 ? 8 : n <= 768 ? 12 : 16; }

ChebAg with_order(const ChebAg& a0) {
  ChebAg a = a0;
  // XCD-aware order when one batch's gathered slice (x: N*F*T floats) fits a 4 MB L2
  a.xcd_order = (int64_t)a.N * a.F * a.T * (int64_t)sizeof(float) <= (int64_t(4) << 20) ? 1 : 0;
  return a;
}

unsigned grid_rows(int64_t waves) { return (unsigned)(cdiv64(cdiv64(waves, 4), 8) * 8); }

}  // namespace

bool cheb_agg_ok(int F, int C) { return F >= 1 && F <= 32 && C >= 1 && C <= 32; }

#define DS_AGG_NQ(KER, nq, grid, lds, st, a)                                                          \
  switch (nq) {                                                                                       \
    case 1: hipLaunchKernelGGL(KER<1>, grid, dim3(256), lds, st, a); break;                           \
    case 2: hipLaunchKernelGGL(KER<2>, grid, dim3(256), lds, st, a); break;                           \
    case 4: hipLaunchKernelGGL(KER<4>, grid, dim3(256), lds, st, a); break;                           \
    case 6: hipLaunchKernelGGL(KER<6>, grid, dim3(256), lds, st, a); break;                           \
    case 8: hipLaunchKernelGGL(KER<8>, grid, dim3(256), lds, st, a); break;                           \
    case 12: hipLaunchKernelGGL(KER<12>, grid, dim3(256), lds, st, a); break;                         \
    default: hipLaunchKernelGGL(KER<16>, grid, dim3(256), lds, st, a); break;                         \
  }

int op_cheb_agg_fwd(const ChebAg& a0, hipStream_t st) {
  if (!cheb_agg_ok(a0.F, a0.C)) { set_last_error("cheb_agg: F, C must be in 1..32"); return DSTAGNN_E_SHAPE; }
  const ChebAg a = with_order(a0);
  const int nq = nq_of(a.F * std::min(32, a.T));
  const dim3 grid(grid_rows((int64_t)a.B * a.N), (unsigned)cdiv64(a.T, 32));
  DS_AGG_NQ(cheb_agg_fwd_kernel, nq, grid, 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

int op_cheb_agg_sddmm(const ChebAg& a0, hipStream_t st) {
  if (!cheb_agg_ok(a0.F, a0.C)) { set_last_error("cheb_agg: F, C must be in 1..32"); return DSTAGNN_E_SHAPE; }
  const ChebAg a = with_order(a0);
  const int FT = a.F * a.T;
  const int nq = nq_of(std::min(FT, 1024));
  const size_t lds = (size_t)4 * FT * sizeof(float);
  if (lds > (160u << 10)) { set_last_error("cheb_agg: F*T too large for the LDS"); return DSTAGNN_E_SHAPE; }
  if (lds > (64u << 10)) {
#define DS_ATTR(n) (void)hipFuncSetAttribute((const void*)cheb_agg_sddmm_kernel<n>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    DS_ATTR(1) DS_ATTR(2) DS_ATTR(4) DS_ATTR(6) DS_ATTR(8) DS_ATTR(12) DS_ATTR(16)
#undef DS_ATTR
  }
  const dim3 grid(grid_rows((int64_t)a.B * a.N * a.K));
  DS_AGG_NQ(cheb_agg_sddmm_kernel, nq, grid, lds, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

int op_cheb_agg_spmm_t(const ChebAg& a0, hipStream_t st) {
  if (!cheb_agg_ok(a0.F, a0.C)) { set_last_error("cheb_agg: F, C must be in 1..32"); return DSTAGNN_E_SHAPE; }
  const ChebAg a = with_order(a0);
  const int nq = nq_of(std::min(32, a.T) * a.C);
  const dim3 grid(grid_rows((int64_t)a.B * a.N), (unsigned)cdiv64(a.T, 32));
  DS_AGG_NQ(cheb_agg_spmm_t_kernel, nq, grid, 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}
