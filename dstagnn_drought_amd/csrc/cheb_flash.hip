// cheb_flash.hip — fused (flash-style) Chebyshev spatial attention for large graphs (gfx950).
//
// cheb_conv_withSAt (model/DSTAGNN_my.py:117-133) normalises, for every destination node j,
//   z_ij = Q'_i . K'_j / sqrt(dk) + A_pa[i,j] M_k[i,j]        (SAt scores :19 + the mask term :122)
//   P_ij = softmax over the source node i of z_ij             (dim=1, quirk 2)
// and aggregates only over the T_k support (cheb_sparse.hip).  The unfused path writes the
// (B,K,N,N) scores, reads them twice for the softmax and writes P, then writes the dense
// score gradient dz for the dQ'/dK' GEMMs — 4 x 10.7 GB per step at N = 4096, B = 32.  Here
// none of those is written:
//
//   forward   stats   per (b,k, 32 columns j): S tiles from Q', K' on the f32 matrix cores
//                     (dk = 32: 16 MFMAs per 32x32 tile), the A_pa o M_k term added where
//                     the A_pa bit row says so, online column max / exp-sum -> lse_j
//             psupp   P and W = T o P on the T_k support only (CSC order, compact)
//   backward  colc    dP = T o dW on the support (dW from the sparse SDDMM, compact):
//                     c_j = sum_i P_ij dP_ij, dzs_ij = P_ij dP_ij          (dz = dzs - P c)
//             dq      dQ'_i = s (sum_{j in supp} dzs_ij K'_j - sum_j P_ij c_j K'_j): the dense
//                     term recomputes P tiles (S^T tile: the P fragment lands in the MFMA
//                     A-operand layout for P . (c K'), no transpose)
//             dk      dK'_j = s (sum_{i in supp} dzs_ij Q'_i - c_j sum_i P_ij Q'_i)
//             mask    dM_k = A_pa o sum_b dz, on the A_pa support only
// The MFMA is v_mfma_f32_32x32x2_f32 (exact fp32): lane l supplies A[m = l&31][k = l>>5] and
// B[k = l>>5][n = l&31]; at step s the lane half h carries element d = 16h + s of the 32-long
// Q'/K' rows; the accumulator holds D[m = (r&3) + 8(r>>2) + 4h][n = l&31] in register r.
#include "common.hpp"
#include "ops.hpp"

namespace {

__device__ __forceinline__ void load16(const float* p, float (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 t = *reinterpret_cast<const float4*>(p + 4 * q);
    v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
  }
}

__device__ __forceinline__ int frag_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Each wave stages its tile in its own LDS slice and only its own lanes read it back, so the
// hand-off needs no workgroup barrier: a wavefront-scope release/acquire orders the LDS
// accesses (the compiler may not move a read of another lane's element above this lane's
// writes) and waves run independently.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ floatx16 zero16() {
  floatx16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// the A_pa o M_k term of z_ij (A_pa is a weight matrix; read only where its bit is set)
__device__ __forceinline__ float apa_term(const ChebFl& a, const float* Mk, int i, int j) {
  const int64_t o = (int64_t)i * a.N + j;
  return a.apa[o] * Mk[o];
}

// The A_pa o M_k term of a tile is a dependent global load wherever the tile's bit word has a
// bit in the lane's 16 fragment rows (at SYN, N = 4096 with 4 A_pa entries per row: ~60 % of
// the tiles have one in some lane, so the whole wave waited on it).  The large-graph kernels
// therefore carry it one tile ahead: the next tile's bit word and the term of its FIRST set bit
// in the lane's rows are loaded while the current tile is multiplied; further set bits (rare:
// ~2 % of the lanes' tiles) still load in place.  Same additions in the same order: identical
// results.  Lane half h holds fragment rows (r & 3) + 8 (r >> 2) + 4 h.
__device__ __forceinline__ uint32_t half_rows(int h) { return h ? 0xF0F0F0F0u : 0x0F0F0F0Fu; }
struct ApaNext {
  int f = -1;      // the first set fragment row of the lane's half, or -1
  float v = 0.f;   // its A_pa o M_k term
};
// row-major walk (flash_dq): fixed row i, tile columns j0 + [0, 32)
__device__ __forceinline__ ApaNext apa_first_row(const ChebFl& a, const float* Mk, uint32_t bits, int h, int i, int j0) {
  ApaNext n;
  const uint32_t b = bits & half_rows(h);
  if (b) {
    n.f = __builtin_ctz(b);
    n.v = apa_term(a, Mk, i, j0 + n.f);
  }
  return n;
}
// column walk (flash_stats / flash_dk): fixed column j, tile rows i0 + [0, 32)
__device__ __forceinline__ ApaNext apa_first_col(const ChebFl& a, const float* Mk, uint32_t bits, int h, int i0, int j) {
  ApaNext n;
  const uint32_t b = bits & half_rows(h);
  if (b) {
    n.f = __builtin_ctz(b);
    n.v = apa_term(a, Mk, i0 + n.f, j);
  }
  return n;
}

// ---------------------------------------------------------------------------------------
// forward: column statistics.  One wave per (b, k, 32 columns); waves independent.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void flash_stats_kernel(ChebFl a) {
  const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int nt = (a.N + 31) >> 5;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= (int64_t)a.B * a.K * nt) return;
  const int jt = (int)(wid % nt), bk = (int)(wid / nt), k = bk % a.K, b = bk / a.K;
  const float* Q = a.qk + (int64_t)b * a.N * a.ld + k * 32;
  const float* Kp = Q + a.kd;
  const int j = jt * 32 + l32, jc = min(j, a.N - 1);
  float bkv[16];
  load16(Kp + (int64_t)jc * a.ld + h * 16, bkv);
  const int32_t* bt = a.bits_t + (int64_t)jc * a.nw;
  const float* Mk = a.mask[k];
  float m = -INFINITY, l = 0.f;
  float aq[16];
  load16(Q + (int64_t)min(l32, a.N - 1) * a.ld + h * 16, aq);
  uint32_t bits = (uint32_t)bt[0];
  ApaNext cur = apa_first_col(a, Mk, bits, h, 0, jc);
  uint32_t bnext = nt > 1 ? (uint32_t)bt[1] : 0u;
  for (int it = 0; it < nt; ++it) {
    floatx16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(aq[s], bkv[s], acc, 0, 0, 0);
    if (it + 1 < nt) load16(Q + (int64_t)min((it + 1) * 32 + l32, a.N - 1) * a.ld + h * 16, aq);
    const ApaNext nxt = it + 1 < nt ? apa_first_col(a, Mk, bnext, h, (it + 1) * 32, jc) : ApaNext{};
    const uint32_t bnn = it + 2 < nt ? (uint32_t)bt[it + 2] : 0u;
    const int i0 = it * 32;
    float z[16], tmax = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int il = frag_row(r, h), i = i0 + il;
      float v = acc[r] * a.scale;
      if ((bits >> il) & 1u) v += il == cur.f ? cur.v : apa_term(a, Mk, i, jc);
      v = i < a.N ? v : -INFINITY;
      z[r] = v;
      tmax = fmaxf(tmax, v);
    }
    if (tmax > -INFINITY) {
      const float mn = fmaxf(m, tmax);
      float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 16; ++r) s4[r & 3] += __expf(z[r] - mn);
      l = l * __expf(m - mn) + ((s4[0] + s4[1]) + (s4[2] + s4[3]));
      m = mn;
    }
    bits = bnext;
    cur = nxt;
    bnext = bnn;
  }
  const float m2 = __shfl_xor(m, 32, 64), l2 = __shfl_xor(l, 32, 64);
  const float M = fmaxf(m, m2);
  const float L = (m == -INFINITY ? 0.f : l * __expf(m - M)) + (m2 == -INFINITY ? 0.f : l2 * __expf(m2 - M));
  if (h == 0 && j < a.N) a.lse[(int64_t)bk * a.N + j] = M + __logf(L);
}

__device__ __forceinline__ float dot32(const float* x, const float (&y)[32]) {
  float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 t = *reinterpret_cast<const float4*>(x + 4 * q);
    s4[0] = fmaf(t.x, y[4 * q], s4[0]);
    s4[1] = fmaf(t.y, y[4 * q + 1], s4[1]);
    s4[2] = fmaf(t.z, y[4 * q + 2], s4[2]);
    s4[3] = fmaf(t.w, y[4 * q + 3], s4[3]);
  }
  return (s4[0] + s4[1]) + (s4[2] + s4[3]);
}

// forward: P and W = T o P on the support of column j (CSC order).  One thread per (b,k,j).
__global__ __launch_bounds__(256) void flash_psupp_kernel(ChebFl a) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)a.B * a.K * a.N) return;
  const int j = (int)(t % a.N), bk = (int)(t / a.N), k = bk % a.K, b = bk / a.K;
  const float* Q = a.qk + (int64_t)b * a.N * a.ld + k * 32;
  float kv[32];
  const float* kr = Q + a.kd + (int64_t)j * a.ld;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 v = *reinterpret_cast<const float4*>(kr + 4 * q);
    kv[4 * q] = v.x; kv[4 * q + 1] = v.y; kv[4 * q + 2] = v.z; kv[4 * q + 3] = v.w;
  }
  const float lse = a.lse[t];
  const float* Mk = a.mask[k];
  const int64_t base = (int64_t)bk * a.nnz;
  for (int p = a.csc_ptr[j]; p < a.csc_ptr[j + 1]; ++p) {
    const int i = a.csc_row[p];
    const int64_t o = (int64_t)i * a.N + j;
    const float w = a.apa[o];
    const float z = dot32(Q + (int64_t)i * a.ld, kv) * a.scale + (w != 0.f ? w * Mk[o] : 0.f);
    const float P = __expf(z - lse);
    a.psupp[base + p] = P;
    a.wsupp[base + p] = a.tsupp[(int64_t)k * a.nnz + p] * P;
  }
}

// backward: c_j = sum_i P_ij T_ij dW_ij and dzs_ij = P_ij T_ij dW_ij on the support
__global__ __launch_bounds__(256) void flash_colc_kernel(ChebFl a) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)a.B * a.K * a.N) return;
  const int j = (int)(t % a.N), bk = (int)(t / a.N), k = bk % a.K;
  const int64_t base = (int64_t)bk * a.nnz;
  float c = 0.f;
  for (int p = a.csc_ptr[j]; p < a.csc_ptr[j + 1]; ++p) {
    const float d = a.psupp[base + p] * (a.tsupp[(int64_t)k * a.nnz + p] * a.dws[base + p]);
    a.dzs[base + p] = d;
    c += d;
  }
  a.cc[t] = c;
}

// backward: dQ'.  One wave per (b, k, 32 rows i), independent (own LDS slice).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void flash_dq_kernel(ChebFl a) {
  stream_sig_store(a.sig, a.sig_v);
  __shared__ float Kt[4][32][33];
  __shared__ float lse_t[4][32], c_t[4][32];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int nt = (a.N + 31) >> 5;
  const int64_t wid = (int64_t)blockIdx.x * 4 + w;
  if (wid >= (int64_t)a.B * a.K * nt) return;
  const int itl = (int)(wid % nt), bk = (int)(wid / nt), k = bk % a.K, b = bk / a.K;
  const float* Q = a.qk + (int64_t)b * a.N * a.ld + k * 32;
  const float* Kp = Q + a.kd;
  const int ic = min(itl * 32 + l32, a.N - 1);
  float bq[16];
  load16(Q + (int64_t)ic * a.ld + h * 16, bq);
  const int32_t* br = a.bits + (int64_t)ic * a.nw;
  const float* Mk = a.mask[k];
  const float* lseb = a.lse + (int64_t)bk * a.N;
  const float* cb = a.cc + (int64_t)bk * a.N;
  floatx16 O = zero16();
  float ak[16];
  load16(Kp + (int64_t)min(l32, a.N - 1) * a.ld + h * 16, ak);
  uint32_t bits = (uint32_t)br[0];
  ApaNext cur = apa_first_row(a, Mk, bits, h, ic, 0);
  uint32_t bnext = nt > 1 ? (uint32_t)br[1] : 0u;
  for (int jt = 0; jt < nt; ++jt) {
    const int j0 = jt * 32;
#pragma unroll
    for (int s = 0; s < 16; ++s) Kt[w][l32][h * 16 + s] = ak[s];
    if (h == 0) {
      const int jj = j0 + l32;
      lse_t[w][l32] = jj < a.N ? lseb[jj] : INFINITY;
      c_t[w][l32] = jj < a.N ? cb[jj] : 0.f;
    }
    floatx16 S = zero16();  // S^T tile: D[m = j][n = i]
#pragma unroll
    for (int s = 0; s < 16; ++s) S = __builtin_amdgcn_mfma_f32_32x32x2f32(ak[s], bq[s], S, 0, 0, 0);
    if (jt + 1 < nt) load16(Kp + (int64_t)min(j0 + 32 + l32, a.N - 1) * a.ld + h * 16, ak);
    const ApaNext nxt = jt + 1 < nt ? apa_first_row(a, Mk, bnext, h, ic, j0 + 32) : ApaNext{};
    const uint32_t bnn = jt + 2 < nt ? (uint32_t)br[jt + 2] : 0u;
    wave_lds_sync();
    float pa[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jl = frag_row(r, h);
      float v = S[r] * a.scale;
      if ((bits >> jl) & 1u) v += jl == cur.f ? cur.v : apa_term(a, Mk, ic, j0 + jl);
      pa[r] = __expf(v - lse_t[w][jl]) * c_t[w][jl];  // P_ij c_j (0 past N: lse = +inf)
    }
#pragma unroll
    for (int s = 0; s < 16; ++s)
      O = __builtin_amdgcn_mfma_f32_32x32x2f32(pa[s], Kt[w][frag_row(s, h)][l32], O, 0, 0, 0);
    wave_lds_sync();
    bits = bnext;
    cur = nxt;
    bnext = bnn;
  }
  const int64_t zb = (int64_t)bk * a.nnz;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = itl * 32 + frag_row(r, h);
    if (i >= a.N) continue;
    float sp = 0.f;
    for (int q = a.csr_ptr[i]; q < a.csr_ptr[i + 1]; ++q)
      sp = fmaf(a.dzs[zb + a.csr2csc[q]], Kp[(int64_t)a.csr_col[q] * a.ld + l32], sp);
    a.dqk[((int64_t)b * a.N + i) * a.ld + k * 32 + l32] = (sp - O[r]) * a.scale;
  }
}

// backward: dK'.  One wave per (b, k, 32 columns j), same structure as flash_dq_kernel with
// the S tile (D[m = i][n = j]) whose P fragment is the A operand of P^T . Q'.
__global__ __launch_bounds__(256) void flash_dk_kernel(ChebFl a) {
  __shared__ float Qt[4][32][33];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int nt = (a.N + 31) >> 5;
  const int64_t wid = (int64_t)blockIdx.x * 4 + w;
  if (wid >= (int64_t)a.B * a.K * nt) return;
  const int jtl = (int)(wid % nt), bk = (int)(wid / nt), k = bk % a.K, b = bk / a.K;
  const float* Q = a.qk + (int64_t)b * a.N * a.ld + k * 32;
  const float* Kp = Q + a.kd;
  const int jc = min(jtl * 32 + l32, a.N - 1);
  float bkv[16];
  load16(Kp + (int64_t)jc * a.ld + h * 16, bkv);
  const float lse = a.lse[(int64_t)bk * a.N + jc];
  const int32_t* bt = a.bits_t + (int64_t)jc * a.nw;
  const float* Mk = a.mask[k];
  floatx16 U = zero16();
  float aq[16];
  load16(Q + (int64_t)min(l32, a.N - 1) * a.ld + h * 16, aq);
  uint32_t bits = (uint32_t)bt[0];
  ApaNext cur = apa_first_col(a, Mk, bits, h, 0, jc);
  uint32_t bnext = nt > 1 ? (uint32_t)bt[1] : 0u;
  for (int it = 0; it < nt; ++it) {
    const int i0 = it * 32;
#pragma unroll
    for (int s = 0; s < 16; ++s) Qt[w][l32][h * 16 + s] = aq[s];
    floatx16 S = zero16();  // D[m = i][n = j]
#pragma unroll
    for (int s = 0; s < 16; ++s) S = __builtin_amdgcn_mfma_f32_32x32x2f32(aq[s], bkv[s], S, 0, 0, 0);
    if (it + 1 < nt) load16(Q + (int64_t)min(i0 + 32 + l32, a.N - 1) * a.ld + h * 16, aq);
    const ApaNext nxt = it + 1 < nt ? apa_first_col(a, Mk, bnext, h, i0 + 32, jc) : ApaNext{};
    const uint32_t bnn = it + 2 < nt ? (uint32_t)bt[it + 2] : 0u;
    wave_lds_sync();
    float pr[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int il = frag_row(r, h), i = i0 + il;
      float v = S[r] * a.scale;
      if ((bits >> il) & 1u) v += il == cur.f ? cur.v : apa_term(a, Mk, i, jc);
      pr[r] = i < a.N ? __expf(v - lse) : 0.f;
    }
#pragma unroll
    for (int s = 0; s < 16; ++s)
      U = __builtin_amdgcn_mfma_f32_32x32x2f32(pr[s], Qt[w][frag_row(s, h)][l32], U, 0, 0, 0);
    wave_lds_sync();
    bits = bnext;
    cur = nxt;
    bnext = bnn;
  }
  const int64_t zb = (int64_t)bk * a.nnz;
  const float* cb = a.cc + (int64_t)bk * a.N;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = jtl * 32 + frag_row(r, h);
    if (j >= a.N) continue;
    float sp = 0.f;
    for (int p = a.csc_ptr[j]; p < a.csc_ptr[j + 1]; ++p)
      sp = fmaf(a.dzs[zb + p], Q[(int64_t)a.csc_row[p] * a.ld + l32], sp);
    a.dqk[((int64_t)b * a.N + j) * a.ld + a.kd + k * 32 + l32] = (sp - cb[j] * U[r]) * a.scale;
  }
}

// backward: dM_k[i,j] = A_pa[i,j] sum_b dz_b[i,j] on the A_pa support.  One wave per (k, j),
// lanes over the batch (B <= 128); P recomputed by a 32-long dot product per (b, i, j).
__global__ __launch_bounds__(256) void flash_mask_grad_kernel(ChebFl a) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= (int64_t)a.K * a.N) return;
  const int j = (int)(wid % a.N), k = (int)(wid / a.N);
  const float* Mk = a.mask[k];
  float* dM = a.dmask[k];
  if (!dM) return;
  // per lane: K'_j, lse_j and c_j of its batch elements b = lane + 64 bb (loaded once per column)
  constexpr int kMaxBB = 2;
  const int nb = min(kMaxBB, (a.B + 63) / 64);
  float kv[kMaxBB][32], lse[kMaxBB], cj[kMaxBB];
#pragma unroll
  for (int bb = 0; bb < kMaxBB; ++bb) {
    const int b = min(lane + 64 * bb, a.B - 1);
    const int bk = b * a.K + k;
    const float* kr = a.qk + (int64_t)b * a.N * a.ld + k * 32 + a.kd + (int64_t)j * a.ld;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float4 v = *reinterpret_cast<const float4*>(kr + 4 * u);
      kv[bb][4 * u] = v.x; kv[bb][4 * u + 1] = v.y; kv[bb][4 * u + 2] = v.z; kv[bb][4 * u + 3] = v.w;
    }
    lse[bb] = a.lse[(int64_t)bk * a.N + j];
    cj[bb] = a.cc[(int64_t)bk * a.N + j];
  }
  for (int q = a.apa_ptr[j]; q < a.apa_ptr[j + 1]; ++q) {
    const int i = a.apa_row[q];
    const int64_t o = (int64_t)i * a.N + j;
    const float w = a.apa[o];
    int pt = -1;  // the T-support entry (i, j), if any
    for (int p = a.csc_ptr[j]; p < a.csc_ptr[j + 1]; ++p)
      if (a.csc_row[p] == i) pt = p;
    float s = 0.f;
    for (int bb = 0; bb < nb; ++bb) {
      const int b = lane + 64 * bb;
      if (b >= a.B) break;
      const int bk = b * a.K + k;
      const float* Q = a.qk + (int64_t)b * a.N * a.ld + k * 32;
      const float z = dot32(Q + (int64_t)i * a.ld, kv[bb]) * a.scale + w * Mk[o];
      const float P = __expf(z - lse[bb]);
      const float dzs = pt >= 0 ? a.dzs[(int64_t)bk * a.nnz + pt] : 0.f;
      s += dzs - P * cj[bb];
    }
    s = wave_sum(s);
    if (lane == 0) dM[o] = w * s;
  }
}

// dM_k = 0 off the A_pa support: every (N,N) mask gradient in one launch (hipMemsetAsync ran at
// ~0.2 TB/s here, 0.4 ms per 67 MB mask at N = 4096)
__global__ __launch_bounds__(256) void flash_zero_kernel(ChebFl a) {
  float* d = a.dmask[blockIdx.y];
  if (!d) return;
  const int64_t NN = (int64_t)a.N * a.N;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < NN; e += (int64_t)gridDim.x * 256) d[e] = 0.f;
}

unsigned grid_waves(int64_t waves) { return (unsigned)cdiv64(waves, 4); }

// ---------------------------------------------------------------------------------------
// Small graphs (N <= kSmallN: PEMS08 170, PEMS04 307).  The kernels above give one wave a
// whole 32-column strip and walk its row tiles with a global round trip per tile (Q' rows,
// bit words, the A_pa term) behind a serial MFMA chain: at N = 170 that is ~6 latency-bound
// iterations on < 1 wave per SIMD.  Here a 4-wave workgroup owns the strip, each wave takes
// every 4th tile, and every operand is fetched in ONE round at kernel entry: the score
// operands, the dense A_pa o M_k strip (AM, formed once per forward by param_prep: no bit
// tests and no dependent loads; AM = 0 off the support, and z + 0 = z exactly), and the
// strip's support pointers.  The forward also keeps P on the A_pa support (papa), so the mask
// gradient needs no score recomputation at all.
// ---------------------------------------------------------------------------------------
constexpr int kSmallN = 512;         // <= 16 tiles: <= kSmallTPW per wave
// a staged (N, 32) operand sits in LDS as dense 128-B rows whose 16-B quads are XOR-swizzled by
// (row & 7): a row-quad read by 8 consecutive rows (the S operand) and a column read of 32
// lanes in one row (the P X product, the sparse term) are both conflict-free without a pad
// column (36-float rows took 12 % more LDS: 3 workgroups per CU instead of 5)
__device__ __forceinline__ int xo(int row, int col) { return row * 32 + ((((col >> 2) ^ row) & 7) << 2) + (col & 3); }
constexpr int kRedF = 4 * 32 * 33;   // the waves' 32 x 32 partials, aliased on the staged rows after use
constexpr int kStripE = 512;         // sparse entries of one strip staged in LDS (else read from HBM); 512: the
                                     // PEMS08 backward fits 5 workgroups per CU (30 KB of LDS each)

// forward: lse_j, P and W = T o P on the T support, P on the A_pa support, for one
// (b, k, 32-column strip).  The strip's P tile goes through LDS ((32 nt) x 33 floats, dynamic).
template <int kSmallTiles>
__global__ __launch_bounds__(256) void flash_small_fwd_kernel(ChebFl a) {
  extern __shared__ float Pt[];  // [(32 nt)][33]
  __shared__ float red_m[4][32], red_l[4][32];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int nt = (a.N + 31) >> 5;
  const int jt = (int)(blockIdx.x % nt), bk = (int)(blockIdx.x / nt), k = bk % a.K, b = bk / a.K;
  const float* Q = a.qk + (int64_t)b * a.N * a.ld + k * 32;
  const float* Kp = Q + a.kd;
  const float* AM = a.am + (int64_t)k * a.N * a.N;
  const int j = jt * 32 + l32, jc = min(j, a.N - 1);
  // the strip's support walk (8 threads per column): pointers now, first entries below
  const int jl = threadIdx.x >> 3, sub = threadIdx.x & 7, jj = min(jt * 32 + jl, a.N - 1);
  const bool jok = jt * 32 + jl < a.N;
  const int p0 = a.csc_ptr[jj], p1 = a.csc_ptr[jj + 1], q0 = a.apa_ptr[jj], q1 = a.apa_ptr[jj + 1];
  // every operand of this wave's tiles in the same round
  float bkv[16], aq[kSmallTiles][16], am[kSmallTiles][16];
  load16(Kp + (int64_t)jc * a.ld + h * 16, bkv);
#pragma unroll
  for (int q = 0; q < kSmallTiles; ++q) {
    const int it = w + 4 * q;
    if (it < nt) {
      load16(Q + (int64_t)min(it * 32 + l32, a.N - 1) * a.ld + h * 16, aq[q]);
#pragma unroll
      for (int r = 0; r < 16; ++r) am[q][r] = AM[(int64_t)min(it * 32 + frag_row(r, h), a.N - 1) * a.N + jc];
    }
  }
  const int pf = p0 + sub, qf = q0 + sub;  // first support entries of this thread
  const int row_p = pf < p1 ? a.csc_row[pf] : 0, row_q = qf < q1 ? a.apa_row[qf] : 0;
  const float t_p = pf < p1 ? a.tsupp[(int64_t)k * a.nnz + pf] : 0.f;
  float z[kSmallTiles][16];
  float mx = -INFINITY;
#pragma unroll
  for (int q = 0; q < kSmallTiles; ++q) {
    const int it = w + 4 * q;
    if (it >= nt) break;
    floatx16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(aq[q][s], bkv[s], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = it * 32 + frag_row(r, h) < a.N ? acc[r] * a.scale + am[q][r] : -INFINITY;
      z[q][r] = v;
      mx = fmaxf(mx, v);
    }
  }
  // column max, then column sum of exp over the four waves (two-pass softmax statistics)
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  if (h == 0) red_m[w][l32] = mx;
  __syncthreads();
  const float M = fmaxf(fmaxf(red_m[0][l32], red_m[1][l32]), fmaxf(red_m[2][l32], red_m[3][l32]));
  float l = 0.f;
#pragma unroll
  for (int q = 0; q < kSmallTiles; ++q) {
    if (w + 4 * q >= nt) break;
#pragma unroll
    for (int r = 0; r < 16; ++r) l += __expf(z[q][r] - M);
  }
  l += __shfl_xor(l, 32, 64);
  if (h == 0) red_l[w][l32] = l;
  __syncthreads();
  const float lse = M + __logf((red_l[0][l32] + red_l[1][l32]) + (red_l[2][l32] + red_l[3][l32]));
  if (w == 0 && h == 0 && j < a.N) a.lse[(int64_t)bk * a.N + j] = lse;
#pragma unroll
  for (int q = 0; q < kSmallTiles; ++q) {
    const int it = w + 4 * q;
    if (it >= nt) break;
#pragma unroll
    for (int r = 0; r < 16; ++r) Pt[(it * 32 + frag_row(r, h)) * 33 + l32] = __expf(z[q][r] - lse);
  }
  __syncthreads();
  if (!jok) return;
  const int64_t base = (int64_t)bk * a.nnz;
  for (int p = pf; p < p1; p += 8) {
    const int i = p == pf ? row_p : a.csc_row[p];
    const float P = Pt[i * 33 + jl];
    a.psupp[base + p] = P;
    a.wsupp[base + p] = (p == pf ? t_p : a.tsupp[(int64_t)k * a.nnz + p]) * P;
  }
  const int64_t abase = (int64_t)bk * a.apa_nnz;
  for (int q = qf; q < q1; q += 8) a.papa[abase + q] = Pt[(q == qf ? row_q : a.apa_row[q]) * 33 + jl];
}

// stage rows [0, N) of one (b, k) 32-float block of qk (Q' or K') into LDS X[(32 nt)][kXs]
// (rows past N zero) — one cooperative round of 16-B loads: every load is issued before the
// first LDS store (a load-store loop would wait out one memory round trip per iteration)
template <int kIt>  // >= NP * 8 / 256
__device__ __forceinline__ void stage_rows(const float* src, int64_t ld, int N, int NP, float* X) {
  float4 v[kIt];
#pragma unroll
  for (int u = 0; u < kIt; ++u) {
    const int e = threadIdx.x + 256 * u, row = e >> 3, c4 = (e & 7) * 4;
    v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < N) v[u] = *reinterpret_cast<const float4*>(src + (int64_t)row * ld + c4);
  }
#pragma unroll
  for (int u = 0; u < kIt; ++u) {
    const int e = threadIdx.x + 256 * u, row = e >> 3, c4 = (e & 7) * 4;
    if (row < NP) *reinterpret_cast<float4*>(X + xo(row, c4)) = v[u];
  }
}

// 16 floats of staged row `row` from column c0 (a multiple of 16)
__device__ __forceinline__ void lds16(const float* X, int row, int c0, float (&v)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 t = *reinterpret_cast<const float4*>(X + xo(row, c0 + 4 * q));
    v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
  }
}

// backward: dK' (workgroups [0, B K nt): one 32-column strip each) and dQ' (the next B K nt:
// one 32-row strip each) in one launch.  The strip's own operand sits in registers, the other
// (all N rows of Q' resp. K') is staged in LDS once; the waves split the contraction's tiles
// and their 32 x 32 partial products are summed through LDS.  The sparse terms walk the
// strip's support (CSC for dK', CSR with the CSR-ordered dzs_r for dQ').
//   dK'_j = s (sum_{i in supp(j)} dzs_ij Q'_i - c_j sum_i P_ij Q'_i)
//   dQ'_i = s (sum_{j in supp_row(i)} dzs_ij K'_j - sum_j P_ij c_j K'_j)
// WPE: the register budget as waves per SIMD (4: no spill; 5: 5 workgroups per CU — the PEMS08
// grid of 1 152 workgroups in one round — at ~22 spilled dwords per lane; DSTAGNN_FLASH_DQK_WPE);
// 1 (no constraint) for 3 / 4 tiles per wave
template <int kSmallTiles, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void flash_small_dqk_kernel(ChebFl a) {
  stream_sig_store(a.sig, a.sig_v);
  extern __shared__ float X[];  // [(32 nt)][32] operand rows (>= kRedF floats), then lse [32 nt], c [32 nt] (dQ)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int nt = (a.N + 31) >> 5, NP = nt * 32;
  const int64_t half = (int64_t)a.B * a.K * nt;
  const bool dq = blockIdx.x >= half;
  const int64_t wg = dq ? blockIdx.x - half : blockIdx.x;
  const int st = (int)(wg % nt), bk = (int)(wg / nt), k = bk % a.K, b = bk / a.K;
  const float* Q = a.qk + (int64_t)b * a.N * a.ld + k * 32;
  const float* Kp = Q + a.kd;
  const float* AM = a.am + (int64_t)k * a.N * a.N;
  const float* AMT = a.amt + (int64_t)k * a.N * a.N;  // transposed: the dQ role's strip is a row strip
  const float* lseb = a.lse + (int64_t)bk * a.N;
  const float* cb = a.cc + (int64_t)bk * a.N;
  const int64_t zb = (int64_t)bk * a.nnz;
  float* Ls = X + max(NP * 32, kRedF);
  float (*red)[32][33] = reinterpret_cast<float (*)[32][33]>(X);  // after the last read of the rows
  float* Cs = Ls + NP;
  float* Ed = Cs + NP;                            // the strip's sparse entries: dzs values ...
  int* Ec = reinterpret_cast<int*>(Ed + kStripE);  // ... and their staged-row indices
  const int own = min(st * 32 + l32, a.N - 1);  // this lane's row (dQ) / column (dK) of the strip
  // final phase: thread -> (4 strip rows, d); their support pointers fetched now.  The strip's
  // entries are contiguous in CSR (dQ) / CSC (dK) order: staged in LDS when they fit
  const int d = threadIdx.x & 31;
  const int* ptr = dq ? a.csr_ptr : a.csc_ptr;
  const int* eidx = dq ? a.csr_col : a.csc_row;
  const float* edz = (dq ? a.dzs_r : a.dzs) + zb;
  int pb[4], pe[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = min(st * 32 + (threadIdx.x >> 5) + 8 * u, a.N - 1);
    pb[u] = ptr[row];
    pe[u] = ptr[row + 1];
  }
  const int sbeg = ptr[st * 32], send = ptr[min(st * 32 + 32, a.N)];
  const bool staged = send - sbeg <= kStripE;
  int ec[kStripE / 256] = {};
  float ed[kStripE / 256] = {};
  if (staged && send > sbeg) {
#pragma unroll
    for (int u = 0; u < kStripE / 256; ++u) {
      const int p = min(sbeg + (int)threadIdx.x + 256 * u, send - 1);
      ec[u] = eidx[p];
      ed[u] = edz[p];
    }
  }
  float bv[16], am[kSmallTiles][16];
  float lse_own = 0.f, c_own = 0.f;
  if (dq) {
    load16(Q + (int64_t)own * a.ld + h * 16, bv);
#pragma unroll
    for (int q = 0; q < kSmallTiles; ++q)
      if (w + 4 * q < nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) am[q][r] = AMT[(int64_t)min((w + 4 * q) * 32 + frag_row(r, h), a.N - 1) * a.N + own];
    stage_rows<kSmallTiles * 4>(Kp, a.ld, a.N, NP, X);
    float lv[kSmallTiles / 2 + 1], cv[kSmallTiles / 2 + 1];  // NP <= 128 kSmallTiles
#pragma unroll
    for (int u = 0; u <= kSmallTiles / 2; ++u) {
      const int e = threadIdx.x + 256 * u;
      lv[u] = e < a.N ? lseb[e] : INFINITY;
      cv[u] = e < a.N ? cb[e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u <= kSmallTiles / 2; ++u) {
      const int e = threadIdx.x + 256 * u;
      if (e < NP) { Ls[e] = lv[u]; Cs[e] = cv[u]; }
    }
  } else {
    load16(Kp + (int64_t)own * a.ld + h * 16, bv);
#pragma unroll
    for (int q = 0; q < kSmallTiles; ++q)
      if (w + 4 * q < nt)
#pragma unroll
        for (int r = 0; r < 16; ++r) am[q][r] = AM[(int64_t)min((w + 4 * q) * 32 + frag_row(r, h), a.N - 1) * a.N + own];
    lse_own = lseb[own];
    stage_rows<kSmallTiles * 4>(Q, a.ld, a.N, NP, X);
  }
  (void)c_own;
  if (staged) {
#pragma unroll
    for (int u = 0; u < kStripE / 256; ++u) {
      const int p = sbeg + (int)threadIdx.x + 256 * u;
      if (p < send) { Ec[p - sbeg] = ec[u]; Ed[p - sbeg] = ed[u]; }
    }
  }
  __syncthreads();
  floatx16 O = zero16();
#pragma unroll
  for (int q = 0; q < kSmallTiles; ++q) {
    const int tt = w + 4 * q;  // the contraction's tile: columns j (dQ) / rows i (dK)
    if (tt >= nt) break;
    float av[16];
    lds16(X, tt * 32 + l32, h * 16, av);
    floatx16 S = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) S = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], S, 0, 0, 0);
    float pv[16];
    if (dq) {  // S^T tile D[m = j][n = i]: lane (i = l32) holds P_ij c_j for j = frag_row(r, h)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int jj = tt * 32 + frag_row(r, h);
        pv[r] = __expf(S[r] * a.scale + am[q][r] - Ls[jj]) * Cs[jj];  // 0 past N (lse = +inf, c = 0)
      }
    } else {   // S tile D[m = i][n = j]: lane (j = l32) holds P_ij for i = frag_row(r, h)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        pv[r] = tt * 32 + frag_row(r, h) < a.N ? __expf(S[r] * a.scale + am[q][r] - lse_own) : 0.f;
    }
    // O[m = strip row][n = d] += sum over the tile's 32 entries of pv x (staged row)[d]
#pragma unroll
    for (int s = 0; s < 16; ++s)
      O = __builtin_amdgcn_mfma_f32_32x32x2f32(pv[s], X[xo(tt * 32 + frag_row(s, h), l32)], O, 0, 0, 0);
  }
  // the sparse term (the last reads of the staged rows), then the partials over the rows
  float sp[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = st * 32 + (threadIdx.x >> 5) + 8 * u;
    float v = 0.f;
    if (row < a.N) {
      if (staged) {
        for (int p = pb[u] - sbeg; p < pe[u] - sbeg; ++p) v = fmaf(Ed[p], X[xo(Ec[p], d)], v);
      } else {
        for (int p = pb[u]; p < pe[u]; ++p) v = fmaf(edz[p], X[xo(eidx[p], d)], v);
      }
    }
    sp[u] = v;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][frag_row(r, h)][l32] = O[r];
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int rl = (threadIdx.x >> 5) + 8 * u, row = st * 32 + rl;
    if (row >= a.N) continue;
    const float dense = (red[0][rl][d] + red[1][rl][d]) + (red[2][rl][d] + red[3][rl][d]);
    if (dq) a.dqk[((int64_t)b * a.N + row) * a.ld + k * 32 + d] = (sp[u] - dense) * a.scale;
    else a.dqk[((int64_t)b * a.N + row) * a.ld + a.kd + k * 32 + d] = (sp[u] - cb[row] * dense) * a.scale;
  }
}

// the same dK' / dQ' for N <= 192 (nt <= 6) with TWO strips per workgroup: waves 2 hw + s take
// strip s's tiles hw, hw + 2, ... (nt / 2 each at nt = 6: 3 tile units per wave, where one strip
// over four waves left two waves with 2 tiles and two with 1).  The staged rows (all N rows of
// Q' resp. K' of the (b, k)) serve both strips.  Half the workgroups: PEMS08's 576 fit one
// wave round (3 per CU) where 1 152 took two.  Per strip the same products and the same
// summation order as flash_small_dqk_kernel except the dense partials, summed over the strip's
// two waves instead of four (tile order hw, hw + 2, ... per wave).
constexpr int kStripE2 = 1024;  // sparse entries of a strip pair staged in LDS
template <int TPW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void flash_small_dqk2_kernel(ChebFl a) {
  stream_sig_store(a.sig, a.sig_v);
  extern __shared__ float X[];  // [(32 nt)][32] operand rows (>= kRedF floats), lse [32 nt], c [32 nt],
                                // the pair's sparse entries, the pair's 65 row pointers
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
  const int s = w & 1, hw = w >> 1;  // this wave's strip of the pair and its half of the tiles
  const int nt = (a.N + 31) >> 5, NP = nt * 32, ns = (nt + 1) >> 1;
  const int64_t half = (int64_t)a.B * a.K * ns;
  const bool dq = blockIdx.x >= half;
  const int64_t wg = dq ? blockIdx.x - half : blockIdx.x;
  const int sp = (int)(wg % ns), bk = (int)(wg / ns), k = bk % a.K, b = bk / a.K;
  const int r0 = sp * 64;                      // the pair's first row (dQ) / column (dK)
  const int nr = min(64, a.N - r0);            // its rows
  const bool live = s * 32 < nr;               // (wave-uniform: the pair's second strip may not exist)
  const float* Q = a.qk + (int64_t)b * a.N * a.ld + k * 32;
  const float* Kp = Q + a.kd;
  const float* AM = a.am + (int64_t)k * a.N * a.N;
  const float* AMT = a.amt + (int64_t)k * a.N * a.N;
  const float* lseb = a.lse + (int64_t)bk * a.N;
  const float* cb = a.cc + (int64_t)bk * a.N;
  const int64_t zb = (int64_t)bk * a.nnz;
  float* Ls = X + max(NP * 32, kRedF);
  float (*red)[32][33] = reinterpret_cast<float (*)[32][33]>(X);  // [w]: after the last read of the rows
  float* Cs = Ls + NP;
  float* Ed = Cs + NP;
  int* Ec = reinterpret_cast<int*>(Ed + kStripE2);
  int* Pp = Ec + kStripE2;                     // row pointers r0 .. r0 + nr
  const int own = min(r0 + 32 * s + l32, a.N - 1);
  const int d = threadIdx.x & 31;
  const int* ptr = dq ? a.csr_ptr : a.csc_ptr;
  const int* eidx = dq ? a.csr_col : a.csc_row;
  const float* edz = (dq ? a.dzs_r : a.dzs) + zb;
  const int sbeg = ptr[r0], send = ptr[r0 + nr];
  const bool staged = send - sbeg <= kStripE2;
  int ec[kStripE2 / 256] = {};
  float ed[kStripE2 / 256] = {};
  if (staged && send > sbeg) {
#pragma unroll
    for (int u = 0; u < kStripE2 / 256; ++u) {
      const int p = min(sbeg + (int)threadIdx.x + 256 * u, send - 1);
      ec[u] = eidx[p];
      ed[u] = edz[p];
    }
  }
  const int pv0 = threadIdx.x <= nr ? ptr[r0 + (int)threadIdx.x] : 0;
  float bv[16], am[TPW][16];
  float lse_own = 0.f;
  load16((dq ? Q : Kp) + (int64_t)own * a.ld + h * 16, bv);
#pragma unroll
  for (int q = 0; q < TPW; ++q) {
    const int tt = hw + 2 * q;
    if (tt < nt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t o = (int64_t)min(tt * 32 + frag_row(r, h), a.N - 1) * a.N + own;
        am[q][r] = dq ? AMT[o] : AM[o];
      }
  }
  if (dq) {
    stage_rows<2 * TPW>(Kp, a.ld, a.N, NP, X);  // (kIt >= NP 8 / 256 = nt; TPW = nt / 2 rounded up)
    constexpr int LV = (TPW * 64 + 255) / 256;
    float lv[LV], cv[LV];
#pragma unroll
    for (int u = 0; u < LV; ++u) {
      const int e = threadIdx.x + 256 * u;
      lv[u] = e < a.N ? lseb[e] : INFINITY;
      cv[u] = e < a.N ? cb[e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < LV; ++u) {
      const int e = threadIdx.x + 256 * u;
      if (e < NP) { Ls[e] = lv[u]; Cs[e] = cv[u]; }
    }
  } else {
    lse_own = lseb[own];
    stage_rows<2 * TPW>(Q, a.ld, a.N, NP, X);
  }
  if (staged) {
#pragma unroll
    for (int u = 0; u < kStripE2 / 256; ++u) {
      const int p = sbeg + (int)threadIdx.x + 256 * u;
      if (p < send) { Ec[p - sbeg] = ec[u]; Ed[p - sbeg] = ed[u]; }
    }
  }
  if (threadIdx.x <= nr) Pp[threadIdx.x] = pv0;
  __syncthreads();
  floatx16 O = zero16();
  if (live) {
#pragma unroll
    for (int q = 0; q < TPW; ++q) {
      const int tt = hw + 2 * q;
      if (tt >= nt) break;
      float av[16];
      lds16(X, tt * 32 + l32, h * 16, av);
      floatx16 S = zero16();
#pragma unroll
      for (int st = 0; st < 16; ++st) S = __builtin_amdgcn_mfma_f32_32x32x2f32(av[st], bv[st], S, 0, 0, 0);
      float pv[16];
      if (dq) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int jj = tt * 32 + frag_row(r, h);
          pv[r] = __expf(S[r] * a.scale + am[q][r] - Ls[jj]) * Cs[jj];
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          pv[r] = tt * 32 + frag_row(r, h) < a.N ? __expf(S[r] * a.scale + am[q][r] - lse_own) : 0.f;
      }
#pragma unroll
      for (int st = 0; st < 16; ++st)
        O = __builtin_amdgcn_mfma_f32_32x32x2f32(pv[st], X[xo(tt * 32 + frag_row(st, h), l32)], O, 0, 0, 0);
    }
  }
  // the sparse term (the last reads of the staged rows): thread -> rows (tid >> 5) + 8 u of the pair
  // staged: the first kSpB entries of every row in one batch of independent LDS reads (the
  // index, then the row element) instead of two dependent LDS round trips per entry; the rest
  // (rows longer than kSpB) in order after them — the same summation order either way
  constexpr int RU = 8, kSpB = 4;
  float spv[RU];
  int pr0[RU], pr1[RU];
#pragma unroll
  for (int u = 0; u < RU; ++u) {
    const int rl = (threadIdx.x >> 5) + 8 * u;
    pr0[u] = rl < nr ? Pp[rl] : 0;
    pr1[u] = rl < nr ? Pp[rl + 1] : 0;
  }
  if (staged) {
    int ci[RU][kSpB];
    float cw[RU][kSpB];
#pragma unroll
    for (int u = 0; u < RU; ++u)
#pragma unroll
      for (int t = 0; t < kSpB; ++t) {
        const int p = pr0[u] + t;
        const bool ok = p < pr1[u];
        ci[u][t] = ok ? Ec[p - sbeg] : 0;
        cw[u][t] = ok ? Ed[p - sbeg] : 0.f;
      }
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      float xv[kSpB];
#pragma unroll
      for (int t = 0; t < kSpB; ++t) xv[t] = X[xo(ci[u][t], d)];
      float v = 0.f;
#pragma unroll
      for (int t = 0; t < kSpB; ++t) v = fmaf(cw[u][t], xv[t], v);  // (0 x row 0 past the row's end)
      for (int p = pr0[u] + kSpB; p < pr1[u]; ++p) v = fmaf(Ed[p - sbeg], X[xo(Ec[p - sbeg], d)], v);
      spv[u] = v;
    }
  } else {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      float v = 0.f;
      for (int p = pr0[u]; p < pr1[u]; ++p) v = fmaf(edz[p], X[xo(eidx[p], d)], v);
      spv[u] = v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][frag_row(r, h)][l32] = O[r];
  __syncthreads();
#pragma unroll
  for (int u = 0; u < RU; ++u) {
    const int rl = (threadIdx.x >> 5) + 8 * u, row = r0 + rl;
    if (rl >= nr) continue;
    const int ss = rl >> 5, rr = rl & 31;
    const float dense = red[ss][rr][d] + red[2 + ss][rr][d];  // the strip's waves, hw = 0 then 1
    if (dq) a.dqk[((int64_t)b * a.N + row) * a.ld + k * 32 + d] = (spv[u] - dense) * a.scale;
    else a.dqk[((int64_t)b * a.N + row) * a.ld + a.kd + k * 32 + d] = (spv[u] - cb[row] * dense) * a.scale;
  }
}

// backward, small graphs: dM_k[i,j] = A_pa[i,j] sum_b (dzs_b[i,j] - P_b[i,j] c_b[j]), every
// element of the K (N,N) gradients written by one thread (0 off the A_pa support), P on the
// support kept by the forward (papa), the T-support position of the entry from apa2t.
__global__ __launch_bounds__(256) void flash_small_mask_kernel(ChebFl a) {
  const int64_t NN = (int64_t)a.N * a.N;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)a.K * NN) return;
  const int k = (int)(e / NN);
  const int64_t o = e - (int64_t)k * NN;
  float* dM = a.dmask[k];
  if (!dM) return;
  const int q = a.apa_idx[o];
  if (q < 0) {
    dM[o] = 0.f;
    return;
  }
  const int j = (int)(o % a.N), pt = a.apa2t[q];
  float s = 0.f;
  constexpr int kBB = 8;  // batch elements per round of loads (fixed summation order; 32 measured no faster)
  for (int b0 = 0; b0 < a.B; b0 += kBB) {
    float dz[kBB], pp[kBB], cv[kBB];
#pragma unroll
    for (int u = 0; u < kBB; ++u) {
      const int64_t bk = (int64_t)min(b0 + u, a.B - 1) * a.K + k;
      dz[u] = pt >= 0 ? a.dzs[bk * a.nnz + pt] : 0.f;
      pp[u] = a.papa[bk * a.apa_nnz + q];
      cv[u] = a.cc[bk * a.N + j];
    }
#pragma unroll
    for (int u = 0; u < kBB; ++u)
      if (b0 + u < a.B) s += dz[u] - pp[u] * cv[u];
  }
  dM[o] = a.apa[o] * s;
}

// the same gradient with the batch sum spread over the wave's lanes: the elements stay one per
// lane (zeros off the support, coalesced), and the wave walks its own support entries (a ballot
// over its 64 elements; ~1.5 per wave at PEMS08) one at a time, lane b loading sample b's
// (dzs, P, c) — one load round per entry and a wave sum, where the per-thread loop paid B / 8
// dependent rounds in its slowest lane.  B <= 128 (two samples per lane).  A fixed reduction
// tree: deterministic, but not flash_small_mask_kernel's sequential order.
__global__ __launch_bounds__(256) void flash_small_mask2_kernel(ChebFl a) {
  const int64_t NN = (int64_t)a.N * a.N;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool in = e < (int64_t)a.K * NN;
  const int k = in ? (int)(e / NN) : 0;
  const int64_t o = in ? e - (int64_t)k * NN : 0;
  float* dM = in ? a.dmask[k] : nullptr;
  const int q = in ? a.apa_idx[o] : -1;
  if (dM && q < 0) dM[o] = 0.f;
  uint64_t mine = __ballot(dM != nullptr && q >= 0);
  while (mine) {  // (wave-uniform)
    const int src = __builtin_ctzll(mine);
    mine &= mine - 1;
    const int qs = __shfl(q, src, 64), ks = __shfl(k, src, 64);
    const int64_t os = ((int64_t)__shfl((int)(o >> 32), src, 64) << 32) | (uint32_t)__shfl((int)o, src, 64);
    const int j = (int)(os % a.N), pt = a.apa2t[qs];
    float s = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int b = lane + 64 * h;
      if (b < a.B) {
        const int64_t bk = (int64_t)b * a.K + ks;
        const float dz = pt >= 0 ? a.dzs[bk * a.nnz + pt] : 0.f;
        s += dz - a.papa[bk * a.apa_nnz + qs] * a.cc[bk * a.N + j];
      }
    }
    s = wave_sum(s);
    if (lane == src) dM[o] = a.apa[o] * s;
  }
}

// backward: dM_k[i, :] for one (k, row i) per wave, every N entries written: zeros off the A_pa
// support (coalesced row stores — no separate zeroing pass), A_pa[i,j] sum_b dz_b[i,j] on it.
// Lanes over the batch (B <= 128); P recomputed by a 32-long dot product per (b, j); the
// T-support position of (i, j) from the CSR row (no search over a CSC column).
__global__ __launch_bounds__(256) void flash_mask_grad_rows_kernel(ChebFl a) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= (int64_t)a.K * a.N) return;
  const int i = (int)(wid % a.N), k = (int)(wid / a.N);
  float* dM = a.dmask[k];
  if (!dM) return;
  const float* Mk = a.mask[k];
  const int32_t* br = a.bits + (int64_t)i * a.nw;
  float* drow = dM + (int64_t)i * a.N;
  for (int j = lane; j < a.N; j += 64)
    if (!((br[j >> 5] >> (j & 31)) & 1)) drow[j] = 0.f;
  constexpr int kMaxBB = 2;
  const int nb = min(kMaxBB, (a.B + 63) / 64);
  float qv[kMaxBB][32];
#pragma unroll
  for (int bb = 0; bb < kMaxBB; ++bb) {
    const int b = min(lane + 64 * bb, a.B - 1);
    const float* qr = a.qk + ((int64_t)b * a.N + i) * a.ld + k * 32;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float4 v = *reinterpret_cast<const float4*>(qr + 4 * u);
      qv[bb][4 * u] = v.x; qv[bb][4 * u + 1] = v.y; qv[bb][4 * u + 2] = v.z; qv[bb][4 * u + 3] = v.w;
    }
  }
  const int q0 = a.csr_ptr[i], q1 = a.csr_ptr[i + 1];
  for (int w0 = 0; w0 < a.nw; w0 += 64) {
    const uint32_t wl = w0 + lane < a.nw ? (uint32_t)br[w0 + lane] : 0u;
    const int nwc = min(64, a.nw - w0);
    for (int wi = 0; wi < nwc; ++wi) {
      uint32_t word = (uint32_t)__builtin_amdgcn_readlane((int)wl, wi);
      while (word) {
        const int bit = __builtin_ctz(word);
        word &= word - 1u;
        const int j = (w0 + wi) * 32 + bit;
        const float av = a.apa[(int64_t)i * a.N + j];
        const float mterm = av * Mk[(int64_t)i * a.N + j];
        int pt = -1;  // the T-support entry (i, j), if any (CSC position)
        for (int q = q0; q < q1; ++q)
          if (a.csr_col[q] == j) pt = a.csr2csc[q];
        float s = 0.f;
        for (int bb = 0; bb < nb; ++bb) {
          const int b = lane + 64 * bb;
          if (b >= a.B) break;
          const int bk = b * a.K + k;
          const float* kr = a.qk + ((int64_t)b * a.N + j) * a.ld + a.kd + k * 32;
          const float z = dot32(kr, qv[bb]) * a.scale + mterm;
          const float P = __expf(z - a.lse[(int64_t)bk * a.N + j]);
          const float dzs = pt >= 0 ? a.dzs[(int64_t)bk * a.nnz + pt] : 0.f;
          s += dzs - P * a.cc[(int64_t)bk * a.N + j];
        }
        s = wave_sum(s);
        if (lane == 0) drow[j] = av * s;
      }
    }
  }
}

}  // namespace

bool flash_small(int N) { return N <= kSmallN; }

namespace {
// dynamic LDS beyond the default 64 KB needs the kernel's limit raised once
template <typename Kern>
int allow_lds(Kern k, size_t bytes) {
  if (bytes <= (64u << 10)) return 0;
  const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) { set_last_error(std::string("flash: LDS attribute: ") + hipGetErrorString(e)); return (int)e; }
  return 0;
}
}  // namespace

int op_flash_forward(const ChebFl& a, hipStream_t st) {
  const int nt = (a.N + 31) >> 5;
  if (a.am) {  // small graphs (flash_small): statistics and the support P from the same score tiles
    const size_t lds = (size_t)nt * 32 * 33 * sizeof(float);
    const dim3 grid((unsigned)((int64_t)a.B * a.K * nt));
    switch ((nt + 3) / 4) {  // tiles per wave
#define DS_FWD(T) case T: DS_TRY(allow_lds(flash_small_fwd_kernel<T>, lds)); \
      hipLaunchKernelGGL(flash_small_fwd_kernel<T>, grid, dim3(256), lds, st, a); break;
      DS_FWD(1) DS_FWD(2) DS_FWD(3) DS_FWD(4)
#undef DS_FWD
      default: set_last_error("flash: graph too large for the small-graph kernels"); return DSTAGNN_E_SHAPE;
    }
    DS_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(flash_stats_kernel, dim3(grid_waves((int64_t)a.B * a.K * nt)), dim3(256), 0, st, a);
  DS_CHECK_LAUNCH();
  hipLaunchKernelGGL(flash_psupp_kernel, dim3((unsigned)cdiv64((int64_t)a.B * a.K * a.N, 256)), dim3(256), 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

int op_flash_colc(const ChebFl& a, hipStream_t st) {
  hipLaunchKernelGGL(flash_colc_kernel, dim3((unsigned)cdiv64((int64_t)a.B * a.K * a.N, 256)), dim3(256), 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

int op_flash_dqk(const ChebFl& a0, hipStream_t st) {
  ChebFl a = a0;  // the first launch carries a pending stream signal (common.hpp)
  const StreamSig sg = peek_stream_sig(st);
  a.sig = sg.p;
  a.sig_v = sg.v;
  const int nt = (a.N + 31) >> 5;
  // N <= 192: two strips per workgroup (flash_small_dqk2_kernel; DSTAGNN_FLASH_DQK2=0: one)
  static const bool dqk2 = !getenv("DSTAGNN_FLASH_DQK2") || atoi(getenv("DSTAGNN_FLASH_DQK2")) != 0;
  if (a.am && dqk2 && nt <= 6) {
    const int ns = (nt + 1) / 2;
    const size_t lds = (std::max<size_t>((size_t)nt * 32 * 32, kRedF) + 2 * (size_t)nt * 32 + 2 * (size_t)kStripE2 + 65) *
                       sizeof(float);
    const dim3 grid((unsigned)(2 * (int64_t)a.B * a.K * ns));
    switch (ns) {
#define DS_DQK2(T) case T: DS_TRY(allow_lds(flash_small_dqk2_kernel<T>, lds)); \
      hipLaunchKernelGGL((flash_small_dqk2_kernel<T>), grid, dim3(256), lds, st, a); break;
      DS_DQK2(1) DS_DQK2(2) DS_DQK2(3)
#undef DS_DQK2
    }
    DS_CHECK_LAUNCH();
    if (sg.p) DS_TRY(stream_sig_sent(st, sg));
    return 0;
  }
  if (a.am) {  // small graphs (flash_small): dK' and dQ' strips in one launch
    const size_t lds = (std::max<size_t>((size_t)nt * 32 * 32, kRedF) + 2 * (size_t)nt * 32 + 2 * (size_t)kStripE) *
                       sizeof(float);
    const dim3 grid((unsigned)(2 * (int64_t)a.B * a.K * nt));
    static const bool wpe5 = getenv("DSTAGNN_FLASH_DQK_WPE") && atoi(getenv("DSTAGNN_FLASH_DQK_WPE")) == 5;
    switch ((nt + 3) / 4) {  // tiles per wave
#define DS_DQK(T) case T: \
      if (wpe5) { DS_TRY(allow_lds(flash_small_dqk_kernel<T, 5>, lds)); \
                  hipLaunchKernelGGL((flash_small_dqk_kernel<T, 5>), grid, dim3(256), lds, st, a); } \
      else { DS_TRY(allow_lds(flash_small_dqk_kernel<T, 4>, lds)); \
             hipLaunchKernelGGL((flash_small_dqk_kernel<T, 4>), grid, dim3(256), lds, st, a); } \
      break;
      DS_DQK(1) DS_DQK(2)
#undef DS_DQK
      // 3 / 4 tiles per wave (N > 256): the register budget of 4 or 5 waves would spill
      case 3: DS_TRY(allow_lds(flash_small_dqk_kernel<3, 1>, lds));
        hipLaunchKernelGGL((flash_small_dqk_kernel<3, 1>), grid, dim3(256), lds, st, a); break;
      case 4: DS_TRY(allow_lds(flash_small_dqk_kernel<4, 1>, lds));
        hipLaunchKernelGGL((flash_small_dqk_kernel<4, 1>), grid, dim3(256), lds, st, a); break;
      default: set_last_error("flash: graph too large for the small-graph kernels"); return DSTAGNN_E_SHAPE;
    }
    DS_CHECK_LAUNCH();
    if (sg.p) DS_TRY(stream_sig_sent(st, sg));
    return 0;
  }
  hipLaunchKernelGGL(flash_dq_kernel, dim3(grid_waves((int64_t)a.B * a.K * nt)), dim3(256), 0, st, a);
  DS_CHECK_LAUNCH();
  if (sg.p) DS_TRY(stream_sig_sent(st, sg));
  hipLaunchKernelGGL(flash_dk_kernel, dim3(grid_waves((int64_t)a.B * a.K * nt)), dim3(256), 0, st, a0);
  DS_CHECK_LAUNCH();
  return 0;
}

int op_flash_mask_grad(const ChebFl& a, hipStream_t st) {
  // row-wise: every row of dM_k written by one wave (zeros off the A_pa support included);
  // DSTAGNN_FLASH_MASK_COLS=1 keeps the column-wise kernel + zeroing pass (A/B)
  static const bool cols = getenv("DSTAGNN_FLASH_MASK_COLS") && atoi(getenv("DSTAGNN_FLASH_MASK_COLS")) != 0;
  if (a.papa && a.apa_idx && !cols) {  // small graphs: one thread per element, P from the forward
    // the batch sum over the wave's lanes (B <= 128; DSTAGNN_FLASH_MASK2=0: one thread per sum)
    static const bool m2 = !getenv("DSTAGNN_FLASH_MASK2") || atoi(getenv("DSTAGNN_FLASH_MASK2")) != 0;
    if (m2 && a.B <= 128)
      hipLaunchKernelGGL(flash_small_mask2_kernel, dim3((unsigned)cdiv64((int64_t)a.K * a.N * a.N, 256)), dim3(256), 0,
                         st, a);
    else
      hipLaunchKernelGGL(flash_small_mask_kernel, dim3((unsigned)cdiv64((int64_t)a.K * a.N * a.N, 256)), dim3(256), 0,
                         st, a);
    DS_CHECK_LAUNCH();
    return 0;
  }
  if (!cols) {
    hipLaunchKernelGGL(flash_mask_grad_rows_kernel, dim3(grid_waves((int64_t)a.K * a.N)), dim3(256), 0, st, a);
    DS_CHECK_LAUNCH();
    return 0;
  }
  const int64_t NN = (int64_t)a.N * a.N;
  hipLaunchKernelGGL(flash_zero_kernel, dim3((unsigned)std::min<int64_t>(cdiv64(NN, 256), 4096), (unsigned)a.K),
                     dim3(256), 0, st, a);
  DS_CHECK_LAUNCH();
  hipLaunchKernelGGL(flash_mask_grad_kernel, dim3(grid_waves((int64_t)a.K * a.N)), dim3(256), 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}
