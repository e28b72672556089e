// gtu_tconv.hip — the backward of the three GTU convolutions with respect to their input
// (model/DSTAGNN_my.py:184-197, the Conv2d(C, 2C, (1, k)) of GTU(C, 1, k) for k = 3, 5, 7),
// as ONE sliding-window kernel on the f32 matrix cores (gfx950).
//
// For node row m = (bn, t) of the (B·N·T, C) result,
//   gpre[m][c] = (X[m][c] > 0) · ( dX[m][c] + Σ_q Σ_{j<k_q} Σ_{o<2C} dconv_q[m + j][o] · Wflip_q[j][o][c] )
// where dconv_q is the gate gradient in the zero-padded row layout of block.hip (node n's
// rows [nT, nT + T): k_q − 1 zero rows then its T − k_q + 1 gate rows, k_q − 1 trailing rows)
// and Wflip_q the flipped weight (param_prep kind 4).  As a GEMM (run_gemm_kcat) every output
// row reads its own k_q·2C-long window, so the tiles' LDS-DMA moves k_q× the bytes of the
// window rows they actually cover (250 MB per PEMS08 step, 5 GB at SYN) and the kernel ran at
// ~45–65 TF/s, bound by that traffic.  Here a 128-row tile stages the UNION of its windows —
// 128 + k_q − 1 rows of 2C floats, once per GTU — into LDS, and the A fragment of tap j is the
// staged row r + j: the same products, k_q× less operand traffic, MFMA-bound.
//
// MFMA v_mfma_f32_32x32x2_f32, wave w owns rows [32w, 32w + 32) of the tile and all C = 32
// columns; step s of tap j contracts o = s + 32h (lane half h: the two halves read columns 32
// apart, so the 64 lanes of an A-fragment read hit 64 distinct banks with the 65-float rows) —
// the same products as the K-concatenated GEMM, summed in this fixed order.
// The weight fragments (≤ 57 KB per GTU, L2-resident) come from global memory one tap ahead.
#include <algorithm>

#include "common.hpp"
#include "ops.hpp"

namespace {

constexpr int kTcBM = 128;                 // output rows per workgroup (4 waves x 32)
constexpr int kTcC = 32;                   // output channels (C)
constexpr int kTcCin = 64;                 // window row width (2C)
constexpr int kTcKmax = 7;                 // widest GTU
constexpr int kTcRow = kTcCin + 1;         // LDS row stride: conflict-free column reads
constexpr int kTcRowsMax = kTcBM + kTcKmax - 1;
constexpr int kTcStageF4 = (kTcRowsMax * kTcCin / 4 + 255) / 256;  // float4 loads per thread

__device__ __forceinline__ int tc_frow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// the 15 taps of the three GTUs as one flat sequence: tap i -> (GTU, offset j)
struct TcTap {
  int q, j;
};
__device__ __forceinline__ TcTap tc_tap(const TconvArgs& a, int i) {
  const int k0 = a.ks[0], k1 = a.ks[1];
  if (i < k0) return {0, i};
  if (i < k0 + k1) return {1, i - k0};
  return {2, i - k0 - k1};
}
// B fragments of a tap: B[kk = s + 32h][n = l32] = Wflip[(j 2C + s + 32h) C + l32]
__device__ __forceinline__ void tc_load_b(const TconvArgs& a, TcTap t, int h, int l32, float (&b)[32]) {
  const float* wq = a.wflip[t.q] + ((int64_t)t.j * kTcCin + 32 * h) * kTcC + l32;
#pragma unroll
  for (int s = 0; s < 32; ++s) b[s] = wq[s * kTcC];
}
// the tile's window rows of GTU q, one round of 16-B loads into registers
__device__ __forceinline__ void tc_load_a(const TconvArgs& a, int q, int64_t m0, float4 (&v)[kTcStageF4]) {
  const int ks = a.ks[q], rows = kTcBM + ks - 1;
  const int64_t avail = a.M + ks - 1 - m0;
  const float* src = a.dconv[q] + m0 * kTcCin;
#pragma unroll
  for (int u = 0; u < kTcStageF4; ++u) {
    const int e4 = threadIdx.x + 256 * u, row = e4 >> 4;
    v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < rows && row < avail) v[u] = *reinterpret_cast<const float4*>(src + (int64_t)e4 * 4);
  }
}

// One workgroup per 128 output rows; the taps of all three GTUs run as one sequence with the
// weight fragments loaded two taps ahead and the next GTU's window rows loaded during the
// current GTU's last tap (the grid gives ~2 waves per SIMD at PEMS08, so the registers are
// spent on keeping loads in flight instead of on occupancy).
__global__ __launch_bounds__(256) void gtu_tconv_kernel(TconvArgs a) {
  stream_sig_store(a.sig, a.sig_v);
  __shared__ float As[kTcRowsMax * kTcRow];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int64_t m0 = (int64_t)blockIdx.x * kTcBM;
  const int ntap = a.ks[0] + a.ks[1] + a.ks[2];
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float4 v[kTcStageF4];
  tc_load_a(a, 0, m0, v);
  float b0[32], b1[32];
  tc_load_b(a, tc_tap(a, 0), h, l32, b0);
  tc_load_b(a, tc_tap(a, min(1, ntap - 1)), h, l32, b1);
  const float* arow = As + (32 * w + l32) * kTcRow + 32 * h;
  for (int i = 0; i < ntap; ++i) {
    const TcTap t = tc_tap(a, i);
    if (t.j == 0) {  // a GTU's first tap: its window rows (loaded earlier) into LDS
      const int rows = kTcBM + a.ks[t.q] - 1;
      __syncthreads();  // the previous GTU's reads of As are done
#pragma unroll
      for (int u = 0; u < kTcStageF4; ++u) {
        const int e4 = tid + 256 * u, row = e4 >> 4, c = (e4 & 15) * 4;
        if (row < rows) {
          float* d = As + row * kTcRow + c;
          d[0] = v[u].x; d[1] = v[u].y; d[2] = v[u].z; d[3] = v[u].w;
        }
      }
      __syncthreads();
    }
    float b2[32];  // two taps ahead
    if (i + 2 < ntap) tc_load_b(a, tc_tap(a, i + 2), h, l32, b2);
    if (t.j == a.ks[t.q] - 1 && t.q < 2) tc_load_a(a, t.q + 1, m0, v);  // the next GTU's rows
    const float* ar = arow + t.j * kTcRow;
#pragma unroll
    for (int s = 0; s < 32; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[s], b0[s], acc, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      b0[s] = b1[s];
      b1[s] = b2[s];
    }
  }
  // epilogue: gpre = (X > 0) ? dX + acc : 0, row m = m0 + 32 w + frow(r, h), column l32;
  // every load before the first store
  float dx[16], xm[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t m = min(m0 + 32 * w + tc_frow(r, h), a.M - 1);
    dx[r] = a.dX[m * kTcC + l32];
    xm[r] = a.X[m * kTcC + l32];
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t m = m0 + 32 * w + tc_frow(r, h);
    if (m >= a.M) continue;
    const float v2 = acc[r] * 1.f + 1.f * dx[r];
    a.gpre[m * kTcC + l32] = xm[r] > 0.f ? v2 : 0.f;
  }
}

// ---------------------------------------------------------------------------------------
// Forward: the three GTU convolutions (model/DSTAGNN_my.py:190, Conv2d(C, 2C, (1, k))) by the
// same sliding window.  Output row m = (bn, t') of GTU q (t' < Tg = T - k + 1) reads the X rows
// (bn, t' + j), j < k — in X's (BN, T, C) layout the rows bn T + t' + j.  A 64-row output tile
// of one GTU needs the X rows from in(m0) to in(m0 + 63) + k - 1 (in(m) = (m / Tg) T + m % Tg):
// ONE contiguous range (a node's last rows are followed by the next node's first), staged once
// into LDS; the A fragment of tap j for row m is staged row in(m) - in(m0) + j.  Wave w owns
// rows 32 (w & 1) and output channels 32 (w >> 1) of the tile; step s of tap j contracts
// c = s + 16h (the halves read columns 16 apart: fewer bank conflicts than c = 2s + h).  Output: conv_q[m][o] = bias[o] + sum.
// ---------------------------------------------------------------------------------------
constexpr int kGcBM = 64, kGcRowsMax = 320, kGcRow = kTcC + 1;
constexpr int kGcStageF4 = kGcRowsMax * kTcC / 4 / 256;  // float4 loads per thread (10)

__global__ __launch_bounds__(256) void gtu_conv_fwd_kernel(GconvArgs a) {
  extern __shared__ float Xs[];  // [rows][kGcRow], rows <= the launch's bound (gconv_rows_max)
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int b = (int)blockIdx.x;
  const int q = b >= a.start[2] ? 2 : (b >= a.start[1] ? 1 : 0);
  const int ks = a.ks[q], Tg = a.Tg[q], T = a.T;
  const int64_t Mq = a.BN * Tg;
  const int64_t m0 = (int64_t)(b - a.start[q]) * kGcBM;
  const int64_t mlast = min(m0 + kGcBM, Mq) - 1;
  auto in_row = [&](int64_t m) -> int64_t { const int64_t bn = m / Tg; return bn * T + (m - bn * Tg); };
  const int64_t r0 = in_row(m0);
  const int rows = (int)(in_row(mlast) - r0) + ks;  // <= kGcRowsMax (host-checked)
  const float* src = a.X + r0 * kTcC;
  float4 v[kGcStageF4];
#pragma unroll
  for (int u = 0; u < kGcStageF4; ++u) {
    const int e4 = tid + 256 * u, row = e4 >> 3;
    v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < rows) v[u] = *reinterpret_cast<const float4*>(src + (int64_t)e4 * 4);
  }
  // this lane's output row / channel and its first tap's weight fragments
  const int64_t m = min(m0 + 32 * (w & 1) + l32, mlast);
  const int ar = (int)(in_row(m) - r0);
  const int o = 32 * (w >> 1) + l32;
  const float* wo = a.wf[q] + o;  // (j, c, o): B[kk = j C + c][n = o], lanes along o (coalesced)
  float bc[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) bc[s] = wo[(s + 16 * h) * (2 * kTcC)];
#pragma unroll
  for (int u = 0; u < kGcStageF4; ++u) {
    const int e4 = tid + 256 * u, row = e4 >> 3, c = (e4 & 7) * 4;
    if (row < rows) {
      float* d = Xs + row * kGcRow + c;
      d[0] = v[u].x; d[1] = v[u].y; d[2] = v[u].z; d[3] = v[u].w;
    }
  }
  __syncthreads();
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int j = 0; j < ks; ++j) {
    float bn[16];
    if (j + 1 < ks) {
#pragma unroll
      for (int s = 0; s < 16; ++s) bn[s] = wo[((j + 1) * kTcC + s + 16 * h) * (2 * kTcC)];
    }
    const float* xr = Xs + (ar + j) * kGcRow + 16 * h;
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xr[s], bc[s], acc, 0, 0, 0);
    if (j + 1 < ks) {
#pragma unroll
      for (int s = 0; s < 16; ++s) bc[s] = bn[s];
    }
  }
  // D[m = row frow(r, h)][n = channel l32] of the wave's 32 x 32 block
  const int on = 32 * (w >> 1) + l32;
  const float bias = a.bias[q] ? a.bias[q][on] : 0.f;
  float* out = a.conv[q];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t mr = m0 + 32 * (w & 1) + tc_frow(r, h);
    if (mr < Mq) out[mr * (2 * kTcC) + on] = acc[r] + bias;
  }
}

}  // namespace

// the largest staged X range of any 64-row tile of GTU width ks (tile rows m0..m0+63)
static int gconv_rows_max(int T, int Tg, int ks) {
  return (kGcBM - 1) / Tg * T + std::min(kGcBM - 1, Tg - 1) + ks + T;
}

bool gtu_conv_fwd_ok(int C, int T, const int* ks, int n) {
  if (C != kTcC || n != 3) return false;
  for (int q = 0; q < n; ++q) {
    const int Tg = T - ks[q] + 1;
    if (ks[q] < 1 || ks[q] > kTcKmax || Tg < 1 || gconv_rows_max(T, Tg, ks[q]) > kGcRowsMax) return false;
  }
  return true;
}

int op_gtu_conv_fwd(GconvArgs a, hipStream_t st) {
  if (a.BN <= 0) return 0;
  if (!gtu_conv_fwd_ok(kTcC, a.T, a.ks, 3)) {
    set_last_error("gtu_conv_fwd: C = 32, widths 1..7, staged window <= 320 rows");
    return DSTAGNN_E_SHAPE;
  }
  if ((reinterpret_cast<uintptr_t>(a.X) & 15) != 0) {
    set_last_error("gtu_conv_fwd: X must be 16-B aligned");
    return DSTAGNN_E_ARG;
  }
  double flops = 0, bytes = 4.0 * a.BN * a.T * kTcC;
  int at = 0;
  for (int q = 0; q < 3; ++q) {
    a.Tg[q] = a.T - a.ks[q] + 1;
    a.start[q] = at;
    const int64_t Mq = a.BN * a.Tg[q];
    at += (int)cdiv64(Mq, kGcBM);
    flops += 2.0 * Mq * (2 * kTcC) * (double)(kTcC * a.ks[q]);
    bytes += 4.0 * ((double)Mq * 2 * kTcC + 2.0 * kTcC * kTcC * a.ks[q]);
  }
  a.start[3] = at;
  int rmax = 0;
  for (int q = 0; q < 3; ++q) rmax = std::max(rmax, gconv_rows_max(a.T, a.Tg[q], a.ks[q]));
  const size_t lds = (size_t)rmax * kGcRow * sizeof(float);  // <= 42 KB
  void* rec = gemm_prof_begin(flops, bytes, st, DSTAGNN_PROF_GTU_TCONV);
  hipLaunchKernelGGL(gtu_conv_fwd_kernel, dim3((unsigned)at), dim3(256), lds, st, a);
  DS_CHECK_LAUNCH();
  gemm_prof_end(rec, st);
  return 0;
}

bool gtu_tconv_ok(int C, const int* ks, int n) {
  if (C != kTcC || n != 3) return false;
  for (int q = 0; q < n; ++q)
    if (ks[q] < 1 || ks[q] > kTcKmax) return false;
  return true;
}

int op_gtu_tconv(const TconvArgs& a, hipStream_t st) {
  if (a.M <= 0) return 0;
  if (!gtu_tconv_ok(kTcC, a.ks, 3)) {
    set_last_error("gtu_tconv: C = 32 and GTU widths 1..7 only");
    return DSTAGNN_E_SHAPE;
  }
  for (int q = 0; q < 3; ++q)
    if ((reinterpret_cast<uintptr_t>(a.dconv[q]) & 15) != 0) {
      set_last_error("gtu_tconv: dconv rows must be 16-B aligned");
      return DSTAGNN_E_ARG;
    }
  // GEMM-family accounting (bench roofline): the K-concatenated product's FLOP and operand bytes
  double flops = 0, bytes = 4.0 * 3 * (double)a.M * kTcC;  // dX, X in; gpre out
  for (int q = 0; q < 3; ++q) {
    flops += 2.0 * a.M * kTcC * (double)(kTcCin * a.ks[q]);
    bytes += 4.0 * ((double)(a.M + a.ks[q] - 1) * kTcCin + (double)kTcCin * a.ks[q] * kTcC);
  }
  TconvArgs b = a;  // carries a pending stream signal (common.hpp)
  const StreamSig sg = peek_stream_sig(st);
  b.sig = sg.p;
  b.sig_v = sg.v;
  void* rec = gemm_prof_begin(flops, bytes, st, DSTAGNN_PROF_GTU_TCONV);
  hipLaunchKernelGGL(gtu_tconv_kernel, dim3((unsigned)cdiv64(a.M, kTcBM)), dim3(256), 0, st, b);
  DS_CHECK_LAUNCH();
  if (sg.p) DS_TRY(stream_sig_sent(st, sg));
  gemm_prof_end(rec, st);
  return 0;
}
