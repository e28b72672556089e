// cheb_sparse.hip — sparse-T_k Chebyshev aggregation of cheb_conv_withSAt (gfx950).
//
// The reference's Chebyshev recurrence is ELEMENTWISE (lib/utils.py:201, quirk 4), so
// every T_k has the support of L~ u I (~3-4 nnz per column on real graphs).  The
// product (T_k o P_k)^T x of model/DSTAGNN_my.py:128-130 therefore only touches those
// entries: instead of a dense (N x N) . (N x C*T) GEMM per (b,k) we gather the C*T-long
// rows xTheta[b,i,k,:] of the supporting source nodes (contiguous 1.5 KB rows at the
// PEMS08 shape: coalesced, L2/MALL-resident).  One wave64 per destination node; each
// lane owns C*T/64 output channels-times-steps.  The softmax statistics stay dense
// (they normalise over all N source nodes); only the aggregation and its two backward
// products are sparse.
//
//   spmm_fwd    out[b,j,:]   = ReLU( sum_k sum_{i in supp(j)} T_k[i,j] P[b,k,i,j] xth[b,i,:,k,:] )
//   sddmm_bwd   dW[b,k,i,j]  = <xth[b,i,:,k,:], g[b,j,:]>          for (i,j) in supp
//   spmm_t_bwd  dxth[b,i,:,k,:] = sum_{j in supp_row(i)} T_k[i,j] P[b,k,i,j] g[b,j,:]
// On the fused (flash) path T o P and dW are compact (B,K,nnz) arrays in CSC order
// (ChebSp::wsupp / dws; the CSR walk maps through csr2csc) and P is never dense.
// Layouts: xth (B,N,T,K,C) (the Theta GEMM's plain row-major output), out / g (B,N,T,C).
// Element e = t*C + c of a node's C*T vector sits at e + t*(K-1)*C inside the node's
// xth block, plus k*C.
#include "common.hpp"
#include "ops.hpp"

namespace {

constexpr int kMaxNQ = 16;  // a wave covers 64*16 = 1024 elements of a row per pass
constexpr int kChunk = 64 * kMaxNQ;
// Rows longer than 1024 (C*T: GAMBIA 32 x 144 = 4608) are cut into 1024-element chunks:
// grid.y = chunk for the two SpMMs (independent outputs), a loop over chunks inside the
// SDDMM (its dot product spans the whole row).

// Lanes past C*T read a clamped (valid) address and are never stored / are zeroed in
// the one operand loaded outside the hot loop: no predicated loads in the inner loops.

// per-lane offsets of elements e = lane + 64 q (clamped to the last one) in a node's xth block
template <int kNQ>
__device__ __forceinline__ void xth_offsets(const ChebSp& a, int e0, int lane, int (&xo)[kNQ]) {
  const int skip = (a.K - 1) * a.C;
#pragma unroll
  for (int q = 0; q < kNQ; ++q) {
    const int e = min(e0 + lane + 64 * q, a.CT - 1);
    xo[q] = e + (e / a.C) * skip;
  }
}

// XCD-aware row-block order: blocks are dealt round-robin over the 8 XCDs (linear block id
// % 8), so physical block p runs logical row block (p % 8) * (gridDim.x / 8) + p / 8 and each
// XCD walks one contiguous eighth of the (b, j) rows.  The rows of one batch b then share an
// XCD, and the neighbour gathers of xth / g (b's K*N*C*T slice, ~0.8 MB at PEMS08) hit that
// XCD's 4 MB L2 instead of every XCD streaming the whole 25 MB tensor.  gridDim.x is a
// multiple of 8 (the launcher pads; padded rows exit at the wv bound).  Only when one batch's
// slice fits an L2 (xcd_order, set by the launcher): at GAMBIA / SYN sizes (63-79 MB per b)
// eight XCDs on eight different batches would overflow the 256 MB Infinity Cache that the
// plain order (all XCDs on one batch) stays inside.
__device__ __forceinline__ int64_t xcd_row_block(int on) {
  const int64_t p = blockIdx.x;
  if (!on) return p;
  const int64_t per = gridDim.x >> 3;
  return (p & 7) * per + (p >> 3);
}

// The support walks below go kE entries at a time: the batch's row indices in one memory
// round, then every gathered element of the batch in the next (one round trip per batch and
// k instead of two per entry — at ~3.6 entries per column the per-entry chain was the cost).
// Entries past the end of the support repeat the batch's last valid one with weight 0.
constexpr int kE = 4;

template <int kNQ>
__global__ __launch_bounds__(256) void cheb_spmm_fwd_kernel(ChebSp a) {
  const int lane = threadIdx.x & 63;
  const int64_t wv = xcd_row_block(a.xcd_order) * 4 + (threadIdx.x >> 6);
  if (wv >= (int64_t)a.B * a.N) return;
  const int b = (int)(wv / a.N), j = (int)(wv % a.N);
  const int e0 = blockIdx.y * kChunk;
  const int64_t NN = (int64_t)a.N * a.N;
  float acc[kNQ];
#pragma unroll
  for (int q = 0; q < kNQ; ++q) acc[q] = 0.f;
  int xo[kNQ];
  xth_offsets<kNQ>(a, e0, lane, xo);
  const int64_t KCT = (int64_t)a.K * a.CT;
  const int p0 = a.csc_ptr[j], p1 = a.csc_ptr[j + 1];
  for (int pb = p0; pb < p1; pb += kE) {
    int rows[kE];
#pragma unroll
    for (int e = 0; e < kE; ++e) rows[e] = a.csc_row[min(pb + e, p1 - 1)];
    for (int k = 0; k < a.K; ++k) {
      const float* Pk = a.P + ((int64_t)b * a.K + k) * NN;
      const float* Tk = a.cheb + (int64_t)k * NN;
      const float* Wk = a.wsupp ? a.wsupp + ((int64_t)b * a.K + k) * a.nnz : nullptr;
      float w[kE], v[kE][kNQ];
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const int64_t o = (int64_t)rows[e] * a.N + j;
        const float wv = Wk ? Wk[min(pb + e, p1 - 1)] : Tk[o] * Pk[o];
        w[e] = pb + e < p1 ? wv : 0.f;
        const float* xr = a.xth + ((int64_t)b * a.N + rows[e]) * KCT + k * a.C;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) v[e][q] = xr[xo[q]];
      }
#pragma unroll
      for (int e = 0; e < kE; ++e)
#pragma unroll
        for (int q = 0; q < kNQ; ++q) acc[q] = fmaf(w[e], v[e][q], acc[q]);
    }
  }
  float* orow = a.out + ((int64_t)b * a.N + j) * a.CT;
#pragma unroll
  for (int q = 0; q < kNQ; ++q) {
    const int e = e0 + lane + 64 * q;
    if (e < a.CT) orow[e] = fmaxf(acc[q], 0.f);
  }
}

// SDDMM dW_ij = <xth_i, g_j> on the support.  On the flash path the softmax backward's
// support terms ride along: dzs_ij = P_ij T_ij dW_ij (also in CSR order for the small-graph
// kernels) and c_j = sum_i dzs_ij, instead of dW.
// One wave per (b, j, k) on the one-pass path (K x the waves of a (b, j) walk: the walk is a
// latency chain, so more, shorter chains in flight); per (b, j) on the chunked path.
template <int kNQ>
__global__ __launch_bounds__(256) void cheb_sddmm_bwd_kernel(ChebSp a) {
  const int lane = threadIdx.x & 63;
  const int64_t wv0 = xcd_row_block(a.xcd_order) * 4 + (threadIdx.x >> 6);
  const bool per_k = a.CT <= kChunk;
  if (wv0 >= (int64_t)a.B * a.N * (per_k ? a.K : 1)) return;
  const int kk = per_k ? (int)(wv0 % a.K) : 0;
  const int64_t wv = per_k ? wv0 / a.K : wv0;
  const int b = (int)(wv / a.N), j = (int)(wv % a.N);
  const int64_t NN = (int64_t)a.N * a.N;
  const float* grow = a.g + ((int64_t)b * a.N + j) * a.CT;
  const int64_t KCT = (int64_t)a.K * a.CT;
  const int p0 = a.csc_ptr[j], p1 = a.csc_ptr[j + 1];
  if (a.CT <= kChunk) {  // one pass: the row of g stays in registers
    float g[kNQ];
#pragma unroll
    for (int q = 0; q < kNQ; ++q) {
      const int e = lane + 64 * q;
      g[q] = e < a.CT ? grow[e] : 0.f;
    }
    int xo[kNQ];
    xth_offsets<kNQ>(a, 0, lane, xo);
    {
      const int k = kk;
      float* dWk = a.dW + ((int64_t)b * a.K + k) * NN;
      float* dSk = a.dws ? a.dws + ((int64_t)b * a.K + k) * a.nnz : nullptr;
      const int64_t zk = ((int64_t)b * a.K + k) * a.nnz;
      float csum = 0.f;
      for (int pb = p0; pb < p1; pb += kE) {
        int rows[kE];
#pragma unroll
        for (int e = 0; e < kE; ++e) rows[e] = a.csc_row[min(pb + e, p1 - 1)];
        // the flash path's softmax-backward operands of the batch, in the same round
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
        float v[kE][kNQ];
#pragma unroll
        for (int e = 0; e < kE; ++e) {
          const float* xr = a.xth + ((int64_t)b * a.N + rows[e]) * KCT + k * a.C;
#pragma unroll
          for (int q = 0; q < kNQ; ++q) v[e][q] = xr[xo[q]];
        }
#pragma unroll
        for (int e = 0; e < kE; ++e) {
          float s = 0.f;
#pragma unroll
          for (int q = 0; q < kNQ; ++q) s = fmaf(g[q], v[e][q], s);
          s = wave_sum(s);
          const int p = pb + e;
          if (p >= p1) break;
          if (a.dzs) {
            const float d = pv[e] * (tv[e] * s);
            csum += d;
            if (lane == 0) {
              a.dzs[zk + p] = d;
              if (a.dzs_r) a.dzs_r[zk + rp[e]] = d;
            }
          } else if (lane == 0) {
            if (dSk) dSk[p] = s;
            else dWk[(int64_t)rows[e] * a.N + j] = s;
          }
        }
      }
      if (a.dzs && lane == 0) a.cc[((int64_t)b * a.K + k) * a.N + j] = csum;
    }
    return;
  }
  for (int k = 0; k < a.K; ++k) {  // long rows: the dot product walks the chunks
    float* dWk = a.dW + ((int64_t)b * a.K + k) * NN;
    float* dSk = a.dws ? a.dws + ((int64_t)b * a.K + k) * a.nnz : nullptr;
    const int64_t zk = ((int64_t)b * a.K + k) * a.nnz;
    float csum = 0.f;
    for (int p = p0; p < p1; ++p) {
      const int i = a.csc_row[p];
      const float* xr = a.xth + ((int64_t)b * a.N + i) * KCT + k * a.C;
      float s = 0.f;
      for (int e0 = 0; e0 < a.CT; e0 += kChunk) {
        int xo[kNQ];
        xth_offsets<kNQ>(a, e0, lane, xo);
#pragma unroll
        for (int q = 0; q < kNQ; ++q) {
          const int e = e0 + lane + 64 * q;
          s = fmaf(e < a.CT ? grow[e] : 0.f, xr[xo[q]], s);
        }
      }
      s = wave_sum(s);
      if (a.dzs) {
        const float d = a.psupp[zk + p] * (a.tsupp[(int64_t)k * a.nnz + p] * s);
        csum += d;
        if (lane == 0) {
          a.dzs[zk + p] = d;
          if (a.dzs_r) a.dzs_r[zk + a.csc2csr[p]] = d;
        }
      } else if (lane == 0) {
        if (dSk) dSk[p] = s;
        else dWk[(int64_t)i * a.N + j] = s;
      }
    }
    if (a.dzs && lane == 0) a.cc[((int64_t)b * a.K + k) * a.N + j] = csum;
  }
}

// one wave per (b, i, k): every k writes its own slice of dxth
template <int kNQ>
__global__ __launch_bounds__(256) void cheb_spmm_t_bwd_kernel(ChebSp a) {
  const int lane = threadIdx.x & 63;
  const int64_t wv0 = xcd_row_block(a.xcd_order) * 4 + (threadIdx.x >> 6);
  if (wv0 >= (int64_t)a.B * a.N * a.K) return;
  const int kk = (int)(wv0 % a.K);
  const int64_t wv = wv0 / a.K;
  const int b = (int)(wv / a.N), i = (int)(wv % a.N);
  const int e0 = blockIdx.y * kChunk;
  const int64_t NN = (int64_t)a.N * a.N;
  int xo[kNQ];
  xth_offsets<kNQ>(a, e0, lane, xo);
  const int64_t KCT = (int64_t)a.K * a.CT;
  const int p0 = a.csr_ptr[i], p1 = a.csr_ptr[i + 1];
  {
    const int k = kk;
    const float* Pk = a.P + ((int64_t)b * a.K + k) * NN;
    const float* Tk = a.cheb + (int64_t)k * NN;
    const float* Wk = a.wsupp ? a.wsupp + ((int64_t)b * a.K + k) * a.nnz : nullptr;
    float acc[kNQ];
#pragma unroll
    for (int q = 0; q < kNQ; ++q) acc[q] = 0.f;
    for (int pb = p0; pb < p1; pb += kE) {
      int cols[kE], ci[kE];
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const int p = min(pb + e, p1 - 1);
        cols[e] = a.csr_col[p];
        ci[e] = Wk ? a.csr2csc[p] : 0;
      }
      float w[kE], v[kE][kNQ];
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        const int64_t o = (int64_t)i * a.N + cols[e];
        const float wv = Wk ? Wk[ci[e]] : Tk[o] * Pk[o];
        w[e] = pb + e < p1 ? wv : 0.f;
        const float* gr = a.g + ((int64_t)b * a.N + cols[e]) * a.CT;
#pragma unroll
        for (int q = 0; q < kNQ; ++q) v[e][q] = gr[min(e0 + lane + 64 * q, a.CT - 1)];
      }
#pragma unroll
      for (int e = 0; e < kE; ++e)
#pragma unroll
        for (int q = 0; q < kNQ; ++q) acc[q] = fmaf(w[e], v[e][q], acc[q]);
    }
    float* dr = a.dxth + ((int64_t)b * a.N + i) * KCT + k * a.C;
#pragma unroll
    for (int q = 0; q < kNQ; ++q) {
      const int e = e0 + lane + 64 * q;
      if (e < a.CT) dr[xo[q]] = acc[q];
    }
  }
}

}  // namespace

bool cheb_sparse_ok(int CT) { return CT > 0 && CT <= (1 << 20); }

namespace {
#define DS_NQ_DISPATCH(KER, a, st, CHUNKED, WPR)                                                   \
  do {                                                                                             \
    const int nq = (int)cdiv64(std::min((a).CT, kChunk), 64);                                      \
    const dim3 grid((unsigned)(cdiv64(cdiv64((int64_t)(a).B * (a).N * (WPR), 4), 8) * 8),           \
                    (CHUNKED) ? (unsigned)cdiv64((a).CT, kChunk) : 1u);                            \
    if (nq <= 1) hipLaunchKernelGGL(KER<1>, grid, dim3(256), 0, st, a);                            \
    else if (nq <= 2) hipLaunchKernelGGL(KER<2>, grid, dim3(256), 0, st, a);                       \
    else if (nq <= 3) hipLaunchKernelGGL(KER<3>, grid, dim3(256), 0, st, a);                       \
    else if (nq <= 4) hipLaunchKernelGGL(KER<4>, grid, dim3(256), 0, st, a);                       \
    else if (nq <= 6) hipLaunchKernelGGL(KER<6>, grid, dim3(256), 0, st, a);                       \
    else if (nq <= 8) hipLaunchKernelGGL(KER<8>, grid, dim3(256), 0, st, a);                       \
    else if (nq <= 12) hipLaunchKernelGGL(KER<12>, grid, dim3(256), 0, st, a);                     \
    else if (nq <= 16) hipLaunchKernelGGL(KER<16>, grid, dim3(256), 0, st, a);                     \
    else { set_last_error("cheb sparse: bad row length"); return DSTAGNN_E_SHAPE; }               \
  } while (0)
// XCD-aware order when one batch's gathered slice (xth: N*K*C*T floats) fits a 4 MB L2
ChebSp with_xcd_order(const ChebSp& a0) {
  ChebSp a = a0;
  a.xcd_order = (int64_t)a.N * a.K * a.CT * (int64_t)sizeof(float) <= (int64_t(4) << 20) ? 1 : 0;
  return a;
}
}  // namespace

int op_cheb_spmm_fwd(const ChebSp& a0, hipStream_t st) {
  const ChebSp a = with_xcd_order(a0);
  DS_NQ_DISPATCH(cheb_spmm_fwd_kernel, a, st, true, 1);
  DS_CHECK_LAUNCH();
  return 0;
}
int op_cheb_sddmm_bwd(const ChebSp& a0, hipStream_t st) {
  const ChebSp a = with_xcd_order(a0);
  DS_NQ_DISPATCH(cheb_sddmm_bwd_kernel, a, st, false, (a.CT <= kChunk ? a.K : 1));
  DS_CHECK_LAUNCH();
  return 0;
}
int op_cheb_spmm_t_bwd(const ChebSp& a0, hipStream_t st) {
  const ChebSp a = with_xcd_order(a0);
  DS_NQ_DISPATCH(cheb_spmm_t_bwd_kernel, a, st, true, a.K);
  DS_CHECK_LAUNCH();
  return 0;
}
