// ops.hip — the non-GEMM kernels of the DSTAGNN block (gfx950, wave64).
//
//   tat_fwd / tat_bwd     temporal attention core per (b,f,head): T x T scores,
//                         softmax over the QUERY axis (model/DSTAGNN_my.py:37-41)
//   ln_fwd / ln_bwd       row LayerNorm over strided multi-source sums (TAt LN_N :100,
//                         EmbedT LN_N :176-181, EmbedS LN_D :180-181) + fused dropout
//   cheb_softmax_fwd/bwd  column softmax over source node i of S'+A_pa*M_k, times T_k
//                         (cheb_conv_withSAt :126-128), and its backward
//   gate_fwd / gate_bwd   GTU gates tanh(p)*sigmoid(q) + concat (:192-197, :242)
//   tail_fwd / tail_bwd   fcmy dropout + residual + ReLU + LN_C (:243-252)
//   reductions            deterministic two-stage column sums (bias / gamma / beta grads)
#include <initializer_list>
#include <map>
#include <mutex>

#include "common.hpp"
#include "ops.hpp"

namespace {

// =====================================================================================
// generic batched transpose  out[b][c][r] = in[b][r][c] (+ beta * out)
// =====================================================================================
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                        int R, int Cc, int64_t in_bs, int64_t out_bs, float beta) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const float* ip = in + (int64_t)b * in_bs;
  float* op = out + (int64_t)b * out_bs;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  // the accumulated output's old values are loaded in the same round as the input tile (they do
  // not depend on it): one memory round trip per workgroup instead of two
  float old[4] = {0.f, 0.f, 0.f, 0.f};
  if (beta != 0.f) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + ty + 8 * u, r = r0 + tx;
      if (r < R && c < Cc) old[u] = op[(int64_t)c * R + r];
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int y = ty + 8 * u, r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < R && c < Cc) ? ip[(int64_t)r * Cc + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int y = ty + 8 * u, c = c0 + y, r = r0 + tx;
    if (r < R && c < Cc) {
      const int64_t o = (int64_t)c * R + r;
      float v = tile[tx][y];
      if (beta != 0.f) v += beta * old[u];
      op[o] = v;
    }
  }
}

// =====================================================================================
// temporal attention core (one workgroup per (b, f, head))
// =====================================================================================
struct TatArgs {
  int B, F, T, h, dk, dv;
  const float* qkv;      // (B*F*T, 2*h*dk + h*dv): [Q | K | V]
  const float* res;      // res_att or null
  int res_mode;
  float scale;
  float* re_at;          // (B,F,h,T,T) scores
  float* att;            // (B,F,h,T,T) softmax (saved)
  float* ctx;            // (B*F*T, h*dv)
  // bwd
  const float* dctx;     // (B*F*T, h*dv)
  const float* dre;      // (B,F,h,T,T) or null
  float* dqkv;           // (B*F*T, 3 cols blocks)
  float* dscore;         // (B,F,h,T,T) dS (== d res_att before f-reduction); scratch when !keep_ds
  // matrix-core backward only: dres_sum = sum_f dS ((B,1,h,T,T), the broadcast res_att's
  // gradient) folded in-kernel by tickets cnt[b*h + hd] over partials in dscore
  float* dres_sum;
  int* cnt;
  int keep_ds;           // write the full dS to dscore
};

// -------------------------------------------------------------------------------------
// Wave-per-problem variants for short series (T <= 16): one 64-lane wave owns one
// (b, f, head) problem, four per workgroup, so no lane idles through the T-wide softmax
// phases: the column softmax over the query axis runs on lanes (j = lane % 16, part =
// lane / 16) with the part sums combined by xor-shuffles over lane bits 4 and 5.  All
// global accesses are row-contiguous (coalesced).
// -------------------------------------------------------------------------------------
constexpr int kTatW = 4;  // problems (waves) per workgroup

__device__ __forceinline__ float xor_max_1632(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ float xor_sum_1632(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

__host__ __device__ inline int tat_wave_fwd_floats(int T, int dk, int dv) {
  return 2 * T * (dk + 1) + T * (dv + 1) + T * T;
}
__host__ __device__ inline int tat_wave_bwd_floats(int T, int dk, int dv) {
  return 2 * T * (dk + 1) + 2 * T * (dv + 1) + 2 * T * T;
}

__global__ __launch_bounds__(256) void tat_fwd_wave_kernel(TatArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int T = a.T, dk = a.dk, dv = a.dv, dkp = dk + 1, dvp = dv + 1;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int id = blockIdx.x * kTatW + w;  // ((b*F + f)*h + hd)
  const bool live = id < a.B * a.F * a.h;
  float* Qs = sm + w * tat_wave_fwd_floats(T, dk, dv);
  float* Ks = Qs + T * dkp;
  float* Vs = Ks + T * dkp;
  float* Ss = Vs + T * dvp;
  const int hd = id % a.h, bf = id / a.h, b = bf / a.F;
  const int ld = 2 * a.h * dk + a.h * dv;
  const float* base = a.qkv + (int64_t)bf * T * ld;
  if (live) {
    for (int e = lane; e < T * dk; e += 64) {
      const int i = e / dk, d = e - i * dk;
      Qs[i * dkp + d] = base[(int64_t)i * ld + hd * dk + d];
      Ks[i * dkp + d] = base[(int64_t)i * ld + a.h * dk + hd * dk + d];
    }
    for (int e = lane; e < T * dv; e += 64) {
      const int i = e / dv, d = e - i * dv;
      Vs[i * dvp + d] = base[(int64_t)i * ld + 2 * a.h * dk + hd * dv + d];
    }
  }
  __syncthreads();
  const int64_t sbase = (int64_t)id * T * T;
  if (live) {
    const float* rp = nullptr;
    if (a.res_mode == DSTAGNN_RES_BCAST) rp = a.res + ((int64_t)b * a.h + hd) * T * T;
    else if (a.res_mode == DSTAGNN_RES_FULL) rp = a.res + sbase;
    for (int e = lane; e < T * T; e += 64) {
      const int i = e / T, j = e - i * T;
      float sc = 0.f;
      for (int d = 0; d < dk; ++d) sc = fmaf(Qs[i * dkp + d], Ks[j * dkp + d], sc);
      sc *= a.scale;
      if (rp) sc += rp[e];
      Ss[e] = sc;
      a.re_at[sbase + e] = sc;
    }
  }
  __syncthreads();
  if (live) {  // softmax over i for column j
    const int j = lane & 15, part = lane >> 4;
    float m = -INFINITY;
    if (j < T)
      for (int i = part; i < T; i += 4) m = fmaxf(m, Ss[i * T + j]);
    m = xor_max_1632(m);
    float l = 0.f;
    if (j < T)
      for (int i = part; i < T; i += 4) l += __expf(Ss[i * T + j] - m);
    l = xor_sum_1632(l);
    const float inv = 1.f / l;
    if (j < T)
      for (int i = part; i < T; i += 4) Ss[i * T + j] = __expf(Ss[i * T + j] - m) * inv;
  }
  __syncthreads();
  if (live) {
    for (int e = lane; e < T * T; e += 64) a.att[sbase + e] = Ss[e];
    const int ldc = a.h * dv;
    float* cbase = a.ctx + (int64_t)bf * T * ldc;
    for (int e = lane; e < T * dv; e += 64) {
      const int i = e / dv, d = e - i * dv;
      float acc = 0.f;
      for (int j = 0; j < T; ++j) acc = fmaf(Ss[i * T + j], Vs[j * dvp + d], acc);
      cbase[(int64_t)i * ldc + hd * dv + d] = acc;
    }
  }
}

__global__ __launch_bounds__(256) void tat_bwd_wave_kernel(TatArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int T = a.T, dk = a.dk, dv = a.dv, dkp = dk + 1, dvp = dv + 1;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int id = blockIdx.x * kTatW + w;
  const bool live = id < a.B * a.F * a.h;
  float* Qs = sm + w * tat_wave_bwd_floats(T, dk, dv);
  float* Ks = Qs + T * dkp;
  float* Vs = Ks + T * dkp;
  float* dCs = Vs + T * dvp;
  float* As = dCs + T * dvp;
  float* dAs = As + T * T;
  const int hd = id % a.h, bf = id / a.h;
  const int ld = 2 * a.h * dk + a.h * dv, ldc = a.h * dv;
  const float* base = a.qkv + (int64_t)bf * T * ld;
  const float* cb = a.dctx + (int64_t)bf * T * ldc;
  const int64_t sbase = (int64_t)id * T * T;
  if (live) {
    for (int e = lane; e < T * dk; e += 64) {
      const int i = e / dk, d = e - i * dk;
      Qs[i * dkp + d] = base[(int64_t)i * ld + hd * dk + d];
      Ks[i * dkp + d] = base[(int64_t)i * ld + a.h * dk + hd * dk + d];
    }
    for (int e = lane; e < T * dv; e += 64) {
      const int i = e / dv, d = e - i * dv;
      Vs[i * dvp + d] = base[(int64_t)i * ld + 2 * a.h * dk + hd * dv + d];
      dCs[i * dvp + d] = cb[(int64_t)i * ldc + hd * dv + d];
    }
    for (int e = lane; e < T * T; e += 64) As[e] = a.att[sbase + e];
  }
  __syncthreads();
  float* dbase = a.dqkv + (int64_t)bf * T * ld;
  if (live) {
    for (int e = lane; e < T * T; e += 64) {  // dA[i][j] = sum_d dctx[i][d] V[j][d]
      const int i = e / T, j = e - i * T;
      float acc = 0.f;
      for (int d = 0; d < dv; ++d) acc = fmaf(dCs[i * dvp + d], Vs[j * dvp + d], acc);
      dAs[e] = acc;
    }
    for (int e = lane; e < T * dv; e += 64) {  // dV[j][d] = sum_i A[i][j] dctx[i][d]
      const int j = e / dv, d = e - j * dv;
      float acc = 0.f;
      for (int i = 0; i < T; ++i) acc = fmaf(As[i * T + j], dCs[i * dvp + d], acc);
      dbase[(int64_t)j * ld + 2 * a.h * dk + hd * dv + d] = acc;
    }
  }
  __syncthreads();
  if (live) {  // column softmax backward: dS = A (dA - sum_i A dA) + d re_At
    const int j = lane & 15, part = lane >> 4;
    float c = 0.f;
    if (j < T)
      for (int i = part; i < T; i += 4) c = fmaf(As[i * T + j], dAs[i * T + j], c);
    c = xor_sum_1632(c);
    if (j < T)
      for (int i = part; i < T; i += 4) {
        float v = As[i * T + j] * (dAs[i * T + j] - c);
        if (a.dre) v += a.dre[sbase + i * T + j];
        dAs[i * T + j] = v;
      }
  }
  __syncthreads();
  if (live) {
    for (int e = lane; e < T * T; e += 64) a.dscore[sbase + e] = dAs[e];
    for (int e = lane; e < T * dk; e += 64) {
      const int i = e / dk, d = e - i * dk;
      float sq = 0.f, sk = 0.f;
      for (int j = 0; j < T; ++j) {
        sq = fmaf(dAs[i * T + j], Ks[j * dkp + d], sq);
        sk = fmaf(dAs[j * T + i], Qs[j * dkp + d], sk);
      }
      dbase[(int64_t)i * ld + hd * dk + d] = sq * a.scale;
      dbase[(int64_t)i * ld + a.h * dk + hd * dk + d] = sk * a.scale;
    }
  }
}

__global__ __launch_bounds__(256) void tat_fwd_kernel(TatArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int T = a.T, dk = a.dk, dv = a.dv;
  const int dkp = dk + 1, dvp = dv + 1;
  float* Qs = sm;
  float* Ks = Qs + T * dkp;
  float* Vs = Ks + T * dkp;
  float* Ss = Vs + T * dvp;  // T*T
  const int id = blockIdx.x;  // ((b*F + f)*h + hd)
  const int hd = id % a.h;
  const int bf = id / a.h;
  const int b = bf / a.F;
  const int ld = 2 * a.h * dk + a.h * dv;
  const float* base = a.qkv + (int64_t)bf * T * ld;
  for (int e = threadIdx.x; e < T * dk; e += blockDim.x) {
    int i = e / dk, d = e % dk;
    Qs[i * dkp + d] = base[(int64_t)i * ld + hd * dk + d];
    Ks[i * dkp + d] = base[(int64_t)i * ld + a.h * dk + hd * dk + d];
  }
  for (int e = threadIdx.x; e < T * dv; e += blockDim.x) {
    int i = e / dv, d = e % dv;
    Vs[i * dvp + d] = base[(int64_t)i * ld + 2 * a.h * dk + hd * dv + d];
  }
  __syncthreads();
  const int64_t sbase = (int64_t)id * T * T;
  const float* rp = nullptr;
  if (a.res_mode == DSTAGNN_RES_BCAST) rp = a.res + ((int64_t)b * a.h + hd) * T * T;
  else if (a.res_mode == DSTAGNN_RES_FULL) rp = a.res + sbase;
  for (int e = threadIdx.x; e < T * T; e += blockDim.x) {
    int i = e / T, j = e % T;
    float s = 0.f;
    for (int d = 0; d < dk; ++d) s = fmaf(Qs[i * dkp + d], Ks[j * dkp + d], s);
    s = s * a.scale;
    if (rp) s += rp[e];
    Ss[e] = s;
    a.re_at[sbase + e] = s;
  }
  __syncthreads();
  // softmax over i (query axis) for each column j
  for (int j = threadIdx.x; j < T; j += blockDim.x) {
    float m = -INFINITY;
    for (int i = 0; i < T; ++i) m = fmaxf(m, Ss[i * T + j]);
    float l = 0.f;
    for (int i = 0; i < T; ++i) l += expf(Ss[i * T + j] - m);
    float inv = 1.f / l;
    for (int i = 0; i < T; ++i) Ss[i * T + j] = expf(Ss[i * T + j] - m) * inv;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * T; e += blockDim.x) a.att[sbase + e] = Ss[e];
  const int ldc = a.h * dv;
  float* cbase = a.ctx + (int64_t)bf * T * ldc;
  for (int e = threadIdx.x; e < T * dv; e += blockDim.x) {
    int i = e / dv, d = e % dv;
    float s = 0.f;
    for (int j = 0; j < T; ++j) s = fmaf(Ss[i * T + j], Vs[j * dvp + d], s);
    cbase[(int64_t)i * ldc + hd * dv + d] = s;
  }
}

__global__ __launch_bounds__(256) void tat_bwd_kernel(TatArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int T = a.T, dk = a.dk, dv = a.dv;
  const int dkp = dk + 1, dvp = dv + 1;
  float* Qs = sm;
  float* Ks = Qs + T * dkp;
  float* Vs = Ks + T * dkp;
  float* dCs = Vs + T * dvp;    // T*dvp
  float* As = dCs + T * dvp;    // T*T
  float* dAs = As + T * T;      // T*T  (becomes dS)
  const int id = blockIdx.x;
  const int hd = id % a.h;
  const int bf = id / a.h;
  const int ld = 2 * a.h * dk + a.h * dv;
  const int ldc = a.h * dv;
  const float* base = a.qkv + (int64_t)bf * T * ld;
  const float* cb = a.dctx + (int64_t)bf * T * ldc;
  const int64_t sbase = (int64_t)id * T * T;
  for (int e = threadIdx.x; e < T * dk; e += blockDim.x) {
    int i = e / dk, d = e % dk;
    Qs[i * dkp + d] = base[(int64_t)i * ld + hd * dk + d];
    Ks[i * dkp + d] = base[(int64_t)i * ld + a.h * dk + hd * dk + d];
  }
  for (int e = threadIdx.x; e < T * dv; e += blockDim.x) {
    int i = e / dv, d = e % dv;
    Vs[i * dvp + d] = base[(int64_t)i * ld + 2 * a.h * dk + hd * dv + d];
    dCs[i * dvp + d] = cb[(int64_t)i * ldc + hd * dv + d];
  }
  for (int e = threadIdx.x; e < T * T; e += blockDim.x) As[e] = a.att[sbase + e];
  __syncthreads();
  // dA[i][j] = sum_d dctx[i][d] V[j][d]
  for (int e = threadIdx.x; e < T * T; e += blockDim.x) {
    int i = e / T, j = e % T;
    float s = 0.f;
    for (int d = 0; d < dv; ++d) s = fmaf(dCs[i * dvp + d], Vs[j * dvp + d], s);
    dAs[e] = s;
  }
  // dV[j][d] = sum_i A[i][j] dctx[i][d]
  float* dbase = a.dqkv + (int64_t)bf * T * ld;
  for (int e = threadIdx.x; e < T * dv; e += blockDim.x) {
    int j = e / dv, d = e % dv;
    float s = 0.f;
    for (int i = 0; i < T; ++i) s = fmaf(As[i * T + j], dCs[i * dvp + d], s);
    dbase[(int64_t)j * ld + 2 * a.h * dk + hd * dv + d] = s;
  }
  __syncthreads();
  // column softmax backward: dS = A * (dA - sum_i A dA) + d re_At
  for (int j = threadIdx.x; j < T; j += blockDim.x) {
    float c = 0.f;
    for (int i = 0; i < T; ++i) c = fmaf(As[i * T + j], dAs[i * T + j], c);
    for (int i = 0; i < T; ++i) {
      float v = As[i * T + j] * (dAs[i * T + j] - c);
      if (a.dre) v += a.dre[sbase + i * T + j];
      dAs[i * T + j] = v;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < T * T; e += blockDim.x) a.dscore[sbase + e] = dAs[e];
  // dQ[i][d] = scale * sum_j dS[i][j] K[j][d];  dK[j][d] = scale * sum_i dS[i][j] Q[i][d]
  for (int e = threadIdx.x; e < T * dk; e += blockDim.x) {
    int i = e / dk, d = e % dk;
    float sq = 0.f, sk = 0.f;
    for (int j = 0; j < T; ++j) {
      sq = fmaf(dAs[i * T + j], Ks[j * dkp + d], sq);
      sk = fmaf(dAs[j * T + i], Qs[j * dkp + d], sk);
    }
    dbase[(int64_t)i * ld + hd * dk + d] = sq * a.scale;
    dbase[(int64_t)i * ld + a.h * dk + hd * dk + d] = sk * a.scale;
  }
}

// Long-series variants (GAMBIA T = 144: one workgroup per (b,f,head) problem would hold
// 140-160 KB of LDS and leave most of its threads idle in the column phases).  The query-axis
// softmax normalises each COLUMN j over the rows i, so a problem splits into column chunks of
// kTatCW columns, one workgroup each (B*F*h*ceil(T/kTatCW) workgroups):
//   fwd  S[:, chunk] -> re_At, softmax -> att; then ctx = att . V as one batched GEMM
//   bwd  dA[:, chunk] = dctx . V_chunk^T, dV_chunk = A_chunk^T dctx, dS[:, chunk] (-> d score),
//        dK_chunk = s dS_chunk^T Q; then dQ = s dS . K as one batched GEMM
constexpr int kTatCW = 16;

__host__ __device__ inline int tat_cols_fwd_floats(int T, int dk) {
  return T * (dk + 1) + kTatCW * (dk + 1) + T * kTatCW + 2 * 16 * 16;
}
__host__ __device__ inline int tat_cols_bwd_floats(int T, int dk, int dv) {
  return T * (dk + 1) + T * (dv + 1) + kTatCW * (dv + 1) + 2 * T * kTatCW + 16 * 16;
}

// column reduction helper: 256 threads = 16 columns x 16 row groups (tid = g * 16 + jj)
__device__ __forceinline__ float col_reduce16(float v, float* red, bool is_max) {
  const int jj = threadIdx.x & 15, g = threadIdx.x >> 4;
  red[g * 16 + jj] = v;
  __syncthreads();
  float r = red[jj];
#pragma unroll
  for (int q = 1; q < 16; ++q) r = is_max ? fmaxf(r, red[q * 16 + jj]) : r + red[q * 16 + jj];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(256) void tat_fwd_cols_kernel(TatArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int T = a.T, dk = a.dk, dkp = dk + 1;
  const int nch = (T + kTatCW - 1) / kTatCW;
  const int id = blockIdx.x / nch, j0 = (blockIdx.x % nch) * kTatCW, cw = min(kTatCW, T - j0);
  float* Qs = sm;
  float* Ks = Qs + T * dkp;
  float* Ss = Ks + kTatCW * dkp;   // [i][jj]
  float* red = Ss + T * kTatCW;
  const int hd = id % a.h, bf = id / a.h, b = bf / a.F;
  const int ld = 2 * a.h * dk + a.h * a.dv;
  const float* base = a.qkv + (int64_t)bf * T * ld;
  for (int e = threadIdx.x; e < T * dk; e += 256) {
    const int i = e / dk, d = e - i * dk;
    Qs[i * dkp + d] = base[(int64_t)i * ld + hd * dk + d];
  }
  for (int e = threadIdx.x; e < cw * dk; e += 256) {
    const int jj = e / dk, d = e - jj * dk;
    Ks[jj * dkp + d] = base[(int64_t)(j0 + jj) * ld + a.h * dk + hd * dk + d];
  }
  __syncthreads();
  const int64_t sbase = (int64_t)id * T * T;
  const float* rp = nullptr;
  if (a.res_mode == DSTAGNN_RES_BCAST) rp = a.res + ((int64_t)b * a.h + hd) * T * T;
  else if (a.res_mode == DSTAGNN_RES_FULL) rp = a.res + sbase;
  for (int e = threadIdx.x; e < T * kTatCW; e += 256) {
    const int i = e / kTatCW, jj = e - i * kTatCW;
    float sc = 0.f;
    if (jj < cw) {
      for (int d = 0; d < dk; ++d) sc = fmaf(Qs[i * dkp + d], Ks[jj * dkp + d], sc);
      sc *= a.scale;
      if (rp) sc += rp[(int64_t)i * T + j0 + jj];
      a.re_at[sbase + (int64_t)i * T + j0 + jj] = sc;
    }
    Ss[e] = sc;
  }
  __syncthreads();
  const int jj = threadIdx.x & 15, g = threadIdx.x >> 4;
  float m = -INFINITY;
  for (int i = g; i < T; i += 16) m = fmaxf(m, Ss[i * kTatCW + jj]);
  m = col_reduce16(m, red, true);
  float l = 0.f;
  for (int i = g; i < T; i += 16) l += __expf(Ss[i * kTatCW + jj] - m);
  l = col_reduce16(l, red, false);
  const float inv = 1.f / l;
  if (jj < cw)
    for (int i = g; i < T; i += 16) a.att[sbase + (int64_t)i * T + j0 + jj] = __expf(Ss[i * kTatCW + jj] - m) * inv;
}

__global__ __launch_bounds__(256) void tat_bwd_cols_kernel(TatArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int T = a.T, dk = a.dk, dv = a.dv, dkp = dk + 1, dvp = dv + 1;
  const int nch = (T + kTatCW - 1) / kTatCW;
  const int id = blockIdx.x / nch, j0 = (blockIdx.x % nch) * kTatCW, cw = min(kTatCW, T - j0);
  float* Qs = sm;                       // T x dkp
  float* dCs = Qs + T * dkp;            // T x dvp
  float* Vs = dCs + T * dvp;            // kTatCW x dvp
  float* As = Vs + kTatCW * dvp;        // [i][jj]
  float* dAs = As + T * kTatCW;         // [i][jj] -> dS
  float* red = dAs + T * kTatCW;
  const int hd = id % a.h, bf = id / a.h;
  const int ld = 2 * a.h * dk + a.h * dv, ldc = a.h * dv;
  const float* base = a.qkv + (int64_t)bf * T * ld;
  const float* cb = a.dctx + (int64_t)bf * T * ldc;
  const int64_t sbase = (int64_t)id * T * T;
  for (int e = threadIdx.x; e < T * dk; e += 256) {
    const int i = e / dk, d = e - i * dk;
    Qs[i * dkp + d] = base[(int64_t)i * ld + hd * dk + d];
  }
  for (int e = threadIdx.x; e < T * dv; e += 256) {
    const int i = e / dv, d = e - i * dv;
    dCs[i * dvp + d] = cb[(int64_t)i * ldc + hd * dv + d];
  }
  for (int e = threadIdx.x; e < cw * dv; e += 256) {
    const int jj = e / dv, d = e - jj * dv;
    Vs[jj * dvp + d] = base[(int64_t)(j0 + jj) * ld + 2 * a.h * dk + hd * dv + d];
  }
  for (int e = threadIdx.x; e < T * kTatCW; e += 256) {
    const int i = e / kTatCW, jj = e - i * kTatCW;
    As[e] = jj < cw ? a.att[sbase + (int64_t)i * T + j0 + jj] : 0.f;
  }
  __syncthreads();
  float* dbase = a.dqkv + (int64_t)bf * T * ld;
  for (int e = threadIdx.x; e < T * kTatCW; e += 256) {  // dA[i][j] = sum_d dctx[i][d] V[j][d]
    const int i = e / kTatCW, jj = e - i * kTatCW;
    float acc = 0.f;
    if (jj < cw)
      for (int d = 0; d < dv; ++d) acc = fmaf(dCs[i * dvp + d], Vs[jj * dvp + d], acc);
    dAs[e] = acc;
  }
  for (int e = threadIdx.x; e < cw * dv; e += 256) {  // dV[j][d] = sum_i A[i][j] dctx[i][d]
    const int jj = e / dv, d = e - jj * dv;
    float acc = 0.f;
    for (int i = 0; i < T; ++i) acc = fmaf(As[i * kTatCW + jj], dCs[i * dvp + d], acc);
    dbase[(int64_t)(j0 + jj) * ld + 2 * a.h * dk + hd * dv + d] = acc;
  }
  __syncthreads();
  // column softmax backward: dS = A (dA - sum_i A dA) + d re_At
  const int jj = threadIdx.x & 15, g = threadIdx.x >> 4;
  float c = 0.f;
  for (int i = g; i < T; i += 16) c = fmaf(As[i * kTatCW + jj], dAs[i * kTatCW + jj], c);
  c = col_reduce16(c, red, false);
  for (int i = g; i < T; i += 16) {
    float v = As[i * kTatCW + jj] * (dAs[i * kTatCW + jj] - c);
    if (jj < cw) {
      if (a.dre) v += a.dre[sbase + (int64_t)i * T + j0 + jj];
      a.dscore[sbase + (int64_t)i * T + j0 + jj] = v;
    }
    dAs[i * kTatCW + jj] = v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < cw * dk; e += 256) {  // dK[j][d] = s sum_i dS[i][j] Q[i][d]
    const int jj2 = e / dk, d = e - jj2 * dk;
    float acc = 0.f;
    for (int i = 0; i < T; ++i) acc = fmaf(dAs[i * kTatCW + jj2], Qs[i * dkp + d], acc);
    dbase[(int64_t)(j0 + jj2) * ld + a.h * dk + hd * dk + d] = acc * a.scale;
  }
}

// =====================================================================================
// LayerNorm over rows of length L; one wave per row, values kept in registers.
// Every global load of a row (all sources, gamma / beta) is issued in one round, branch-free
// (out-of-row lanes load the row's last element and are masked after): a per-element
// `if (e < L)` around a load, or a runtime loop over the sources, made the compiler wait
// vmcnt(0) after every load — 16 dependent round trips per row for the EmbedS LN (L = 512, two
// sources), ~1.3 TB/s.
// =====================================================================================
template <int VPT, int NSRC>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LnFwd a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.R) return;
  const int L = a.L;
  const float* sp[NSRC];
  int64_t o[NSRC], es[NSRC];
#pragma unroll
  for (int s = 0; s < NSRC; ++s) {
    sp[s] = a.src[s].p;
    o[s] = ioff(a.src[s].row, row);
    es[s] = a.src[s].es;
  }
  // long rows (VPT > 16: GAMBIA's N = 2139) keep one value per element in registers and read
  // gamma / beta at the store (register budget); short ones preload everything
  constexpr bool PRE = VPT <= 16;
  float v[VPT], gv[PRE ? VPT : 1], bv[PRE ? VPT : 1];
  float sum = 0.f;
  if constexpr (PRE) {
    float xs[NSRC][VPT];
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const int e = min(lane + 64 * q, L - 1);
#pragma unroll
      for (int s = 0; s < NSRC; ++s) xs[s][q] = sp[s][o[s] + (int64_t)e * es[s]];
      gv[q] = a.g[e];
      bv[q] = a.b[e];
    }
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      float u = 0.f;
#pragma unroll
      for (int s = 0; s < NSRC; ++s) u += xs[s][q];
      v[q] = lane + 64 * q < L ? u : 0.f;
    }
  } else {
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const int e = min(lane + 64 * q, L - 1);
      float u = 0.f;
#pragma unroll
      for (int s = 0; s < NSRC; ++s) u += sp[s][o[s] + (int64_t)e * es[s]];
      v[q] = lane + 64 * q < L ? u : 0.f;
    }
  }
#pragma unroll
  for (int q = 0; q < VPT; ++q) sum += v[q];
  const float mean = wave_sum(sum) / L;
  float var = 0.f;
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    int e = lane + 64 * q;
    if (e < L) { float d = v[q] - mean; var += d * d; }
  }
  var = wave_sum(var) / L;
  const float rs = rsqrtf(var + a.eps);
  if (lane == 0) { a.mu[row] = mean; a.rs[row] = rs; }
  const int64_t yo = ioff(a.yrow, row);
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    int e = lane + 64 * q;
    if (e < L) {
      if (a.u) a.u[(int64_t)row * L + e] = v[q];
      float y = (v[q] - mean) * rs * (PRE ? gv[PRE ? q : 0] : a.g[e]) + (PRE ? bv[PRE ? q : 0] : a.b[e]);
      if (a.drop_p > 0.f) y *= drop_scale(a.seed, a.which, (uint64_t)row * L + e + a.drop_off, a.drop_p);
      a.y[yo + (int64_t)e * a.yes] = y;
    }
  }
}

// Rows of L = 256 V4 contiguous floats (the EmbedS LayerNorm over D = 512): the same
// arithmetic with every load and store a float4 — lane l holds elements 4 (l + 64 q) .. + 3 —
// so a row is V4 16-B loads per source per lane instead of 4 V4 dword loads (the wave-per-row
// kernel above at L = 512 issued 32 loads and 16 stores per lane).  The row sums go over a
// different partition of the row (within the fp32 rounding of the other kernel).
__device__ __forceinline__ float l4at(const float4& v, int c) { return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w; }
__device__ __forceinline__ void l4set(float4& v, int c, float x) {
  if (c == 0) v.x = x; else if (c == 1) v.y = x; else if (c == 2) v.z = x; else v.w = x;
}
template <int V4, int NSRC>
__global__ __launch_bounds__(256) void ln_fwd_v4_kernel(LnFwd a) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.R) return;
  constexpr int L = 256 * V4;
  float4 xs[NSRC][V4], gv[V4], bv[V4], v[V4];
#pragma unroll
  for (int q = 0; q < V4; ++q) {
    const int e4 = lane + 64 * q;
#pragma unroll
    for (int s = 0; s < NSRC; ++s)
      xs[s][q] = reinterpret_cast<const float4*>(a.src[s].p + ioff(a.src[s].row, row))[e4];
    gv[q] = reinterpret_cast<const float4*>(a.g)[e4];
    bv[q] = reinterpret_cast<const float4*>(a.b)[e4];
  }
  float sum = 0.f;
#pragma unroll
  for (int q = 0; q < V4; ++q) {
    v[q] = xs[0][q];
#pragma unroll
    for (int s = 1; s < NSRC; ++s) {
      v[q].x += xs[s][q].x; v[q].y += xs[s][q].y; v[q].z += xs[s][q].z; v[q].w += xs[s][q].w;
    }
    sum += (v[q].x + v[q].y) + (v[q].z + v[q].w);
  }
  const float mean = wave_sum(sum) / L;
  float var = 0.f;
#pragma unroll
  for (int q = 0; q < V4; ++q)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float d = l4at(v[q], c) - mean;
      var += d * d;
    }
  var = wave_sum(var) / L;
  const float rs = rsqrtf(var + a.eps);
  if (lane == 0) { a.mu[row] = mean; a.rs[row] = rs; }
  const int64_t yo = ioff(a.yrow, row);
  const DropKey dk = drop_key(a.seed, a.which);
  const float dscale = 1.0f / (1.0f - a.drop_p);
#pragma unroll
  for (int q = 0; q < V4; ++q) {
    const int e4 = lane + 64 * q;
    if (a.u) reinterpret_cast<float4*>(a.u + (int64_t)row * L)[e4] = v[q];
    float4 y;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float t = (l4at(v[q], c) - mean) * rs * l4at(gv[q], c) + l4at(bv[q], c);
      if (a.drop_p > 0.f) t *= drop_u(dk, (uint64_t)row * L + 4 * e4 + c + a.drop_off) >= a.drop_p ? dscale : 0.0f;
      l4set(y, c, t);
    }
    reinterpret_cast<float4*>(a.y + yo)[e4] = y;
  }
}

// the backward of the same rows (ln_bwd_kernel's arithmetic; PART: per-workgroup partial slabs)
template <int V4, bool PART>
__global__ __launch_bounds__(256) void ln_bwd_v4_kernel(LnBwd a) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int L = 256 * V4;
  const int row = blockIdx.x * 4 + wv;
  float4 gp[V4], bp[V4], xp[V4];
#pragma unroll
  for (int q = 0; q < V4; ++q) gp[q] = bp[q] = xp[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (row < a.R) {
    const int64_t yo = ioff(a.dyrow, row), xo = ioff(a.dxrow, row);
    float4 dyl[V4], ul[V4], gl[V4], xin[V4];
#pragma unroll
    for (int q = 0; q < V4; ++q) {
      const int e4 = lane + 64 * q;
      dyl[q] = reinterpret_cast<const float4*>(a.dy + yo)[e4];
      ul[q] = reinterpret_cast<const float4*>(a.u + (int64_t)row * L)[e4];
      gl[q] = reinterpret_cast<const float4*>(a.g)[e4];
      if (a.beta != 0.f) xin[q] = reinterpret_cast<const float4*>(a.dx + xo)[e4];
    }
    const float mean = a.mu[row], rs = a.rs[row];
    const DropKey dk = drop_key(a.seed, a.which);
    const float dscale = 1.0f / (1.0f - a.drop_p);
    float4 dyv[V4], xh[V4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < V4; ++q) {
      const int e4 = lane + 64 * q;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float dy = l4at(dyl[q], c);
        if (a.drop_p > 0.f) dy *= drop_u(dk, (uint64_t)row * L + 4 * e4 + c + a.drop_off) >= a.drop_p ? dscale : 0.0f;
        const float x = (l4at(ul[q], c) - mean) * rs;
        l4set(dyv[q], c, dy);
        l4set(xh[q], c, x);
        const float dxh = dy * l4at(gl[q], c);
        s1 += dxh;
        s2 += dxh * x;
        if (PART) {
          l4set(gp[q], c, dy * x);
          l4set(bp[q], c, dy);
        } else {
          if (a.gcontrib) a.gcontrib[(int64_t)row * L + 4 * e4 + c] = dy * x;
          if (a.bcontrib) a.bcontrib[(int64_t)row * L + 4 * e4 + c] = dy;
        }
      }
    }
    s1 = wave_sum(s1) / L;
    s2 = wave_sum(s2) / L;
#pragma unroll
    for (int q = 0; q < V4; ++q) {
      float4 d;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float t = rs * (l4at(dyv[q], c) * l4at(gl[q], c) - s1 - l4at(xh[q], c) * s2);
        if (a.beta != 0.f) t += a.beta * l4at(xin[q], c);
        l4set(d, c, t);
      }
      reinterpret_cast<float4*>(a.dx + xo)[lane + 64 * q] = d;
      if (PART) xp[q] = d;
    }
  }
  if constexpr (PART) {
    __shared__ float4 red[2][4][64 * V4];
#pragma unroll
    for (int q = 0; q < V4; ++q) {
      red[0][wv][lane + 64 * q] = gp[q];
      red[1][wv][lane + 64 * q] = bp[q];
    }
    __syncthreads();
    for (int e4 = threadIdx.x; e4 < L / 4; e4 += 256) {
      float4 g = red[0][0][e4], b = red[1][0][e4];
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const float4 g2 = red[0][k][e4], b2 = red[1][k][e4];
        g.x += g2.x; g.y += g2.y; g.z += g2.z; g.w += g2.w;
        b.x += b2.x; b.y += b2.y; b.z += b2.z; b.w += b2.w;
      }
      if (a.gpart) reinterpret_cast<float4*>(a.gpart + (int64_t)blockIdx.x * L)[e4] = g;
      if (a.bpart) reinterpret_cast<float4*>(a.bpart + (int64_t)blockIdx.x * L)[e4] = b;
    }
    if (a.xpart) {  // the dx sums through the same LDS rows (workgroup-uniform branch)
      __syncthreads();
#pragma unroll
      for (int q = 0; q < V4; ++q) red[0][wv][lane + 64 * q] = xp[q];
      __syncthreads();
      for (int e4 = threadIdx.x; e4 < L / 4; e4 += 256) {
        float4 x = red[0][0][e4];
#pragma unroll
        for (int k = 1; k < 4; ++k) {
          const float4 x2 = red[0][k][e4];
          x.x += x2.x; x.y += x2.y; x.z += x2.z; x.w += x2.w;
        }
        reinterpret_cast<float4*>(a.xpart + (int64_t)blockIdx.x * L)[e4] = x;
      }
    }
  }
}

// the float4 kernels' preconditions: L = 256 or 512 or 1024, unit element strides, every row
// base and pointer 16-B aligned (row maps with strides that are multiples of 4 floats)
static bool al16p(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
static bool map4(const Idx2& m) { return m.s0 % 4 == 0 && m.s1 % 4 == 0; }
static bool ln_v4_env() {
  static const bool on = !getenv("DSTAGNN_LN_V4") || atoi(getenv("DSTAGNN_LN_V4")) != 0;  // default on
  return on;
}
static bool ln_fwd_v4_ok(const LnFwd& a) {
  if (!ln_v4_env() || (a.L != 256 && a.L != 512 && a.L != 1024) || a.yes != 1 || !map4(a.yrow)) return false;
  for (int s = 0; s < a.nsrc; ++s)
    if (a.src[s].es != 1 || !map4(a.src[s].row) || !al16p(a.src[s].p)) return false;
  return al16p(a.g) && al16p(a.b) && al16p(a.y) && al16p(a.u);
}
static bool ln_bwd_v4_ok(const LnBwd& a) {
  return ln_v4_env() && (a.L == 256 || a.L == 512 || a.L == 1024) && a.dyes == 1 && a.dxes == 1 && map4(a.dyrow) &&
         map4(a.dxrow) && al16p(a.dy) && al16p(a.u) && al16p(a.g) && al16p(a.dx) && al16p(a.gpart) &&
         al16p(a.bpart) && al16p(a.xpart);
}

// Long rows (L > 1024: the TAt / EmbedT LayerNorm over N nodes at GAMBIA N = 2139 and SYN
// N = 4096): a 256-thread WORKGROUP per row, element e = tid + 256 q (VPT <= 16 values per
// thread, all loads in one round as above), the sums over the row by a wave reduction and the
// four waves' partials through LDS in a fixed order.  The wave-per-row kernel needed 64 values
// per lane there (~210-256 VGPRs + AGPR spills of the gradient: one wave per SIMD, ~25 % of
// HBM bandwidth).
__device__ __forceinline__ float wg_sum4(float v, float* red4) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red4[w] = v;
  __syncthreads();
  const float t = (red4[0] + red4[1]) + (red4[2] + red4[3]);
  __syncthreads();  // red4 reused by the next reduction
  return t;
}

template <int VPT, int NSRC>
__global__ __launch_bounds__(256) void ln_fwd_wg_kernel(LnFwd a) {
  __shared__ float red4[4];
  const int tid = threadIdx.x, row = blockIdx.x, L = a.L;
  float xs[NSRC][VPT], gv[VPT], bv[VPT], v[VPT];
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    const int e = min(tid + 256 * q, L - 1);
#pragma unroll
    for (int s = 0; s < NSRC; ++s) xs[s][q] = a.src[s].p[ioff(a.src[s].row, row) + (int64_t)e * a.src[s].es];
    gv[q] = a.g[e];
    bv[q] = a.b[e];
  }
  float sum = 0.f;
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    float u = 0.f;
#pragma unroll
    for (int s = 0; s < NSRC; ++s) u += xs[s][q];
    v[q] = tid + 256 * q < L ? u : 0.f;
    sum += v[q];
  }
  const float mean = wg_sum4(sum, red4) / L;
  float var = 0.f;
#pragma unroll
  for (int q = 0; q < VPT; ++q)
    if (tid + 256 * q < L) { const float d = v[q] - mean; var += d * d; }
  var = wg_sum4(var, red4) / L;
  const float rs = rsqrtf(var + a.eps);
  if (tid == 0) { a.mu[row] = mean; a.rs[row] = rs; }
  const int64_t yo = ioff(a.yrow, row);
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    const int e = tid + 256 * q;
    if (e >= L) continue;
    if (a.u) a.u[(int64_t)row * L + e] = v[q];
    float y = (v[q] - mean) * rs * gv[q] + bv[q];
    if (a.drop_p > 0.f) y *= drop_scale(a.seed, a.which, (uint64_t)row * L + e + a.drop_off, a.drop_p);
    a.y[yo + (int64_t)e * a.yes] = y;
  }
}

// backward of the above (per-element gamma / beta contributions: the partial-slab form needs
// L <= 1024)
template <int VPT>
__global__ __launch_bounds__(256) void ln_bwd_wg_kernel(LnBwd a) {
  __shared__ float red4[4];
  const int tid = threadIdx.x, row = blockIdx.x, L = a.L;
  const int64_t yo = ioff(a.dyrow, row), xo = ioff(a.dxrow, row);
  float dyl[VPT], ul[VPT], gl[VPT], xin[VPT];
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    const int e = min(tid + 256 * q, L - 1);
    dyl[q] = a.dy[yo + (int64_t)e * a.dyes];
    ul[q] = a.u[(int64_t)row * L + e];
    gl[q] = a.g[e];
    xin[q] = a.beta != 0.f ? a.dx[xo + (int64_t)e * a.dxes] : 0.f;
  }
  const float mean = a.mu[row], rs = a.rs[row];
  float dyv[VPT], xh[VPT], s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    const int e = tid + 256 * q;
    dyv[q] = 0.f; xh[q] = 0.f;
    if (e < L) {
      float dy = dyl[q];
      if (a.drop_p > 0.f) dy *= drop_scale(a.seed, a.which, (uint64_t)row * L + e + a.drop_off, a.drop_p);
      const float x = (ul[q] - mean) * rs;
      dyv[q] = dy; xh[q] = x;
      const float dxh = dy * gl[q];
      s1 += dxh; s2 += dxh * x;
      if (a.gcontrib) a.gcontrib[(int64_t)row * L + e] = dy * x;
      if (a.bcontrib) a.bcontrib[(int64_t)row * L + e] = dy;
    }
  }
  s1 = wg_sum4(s1, red4) / L;
  s2 = wg_sum4(s2, red4) / L;
#pragma unroll
  for (int q = 0; q < VPT; ++q) {
    const int e = tid + 256 * q;
    if (e >= L) continue;
    float dx = rs * (dyv[q] * gl[q] - s1 - xh[q] * s2);
    if (a.beta != 0.f) dx += a.beta * xin[q];
    a.dx[xo + (int64_t)e * a.dxes] = dx;
  }
}

// PART: gamma / beta gradient partial sums per workgroup instead of per-element contribution
// tensors: a wave takes kLnRowsPerWave consecutive rows, keeps the sums over them in
// registers, and the 4 waves combine through LDS into one row of the (blocks, L) slabs
// gpart / bpart (reduced over blocks by a column sum afterwards).  Cuts the (R, L) contribution
// write and its re-read.  Loads: one branch-free round per row, as ln_fwd_kernel.
template <int VPT, bool PART>
__global__ __launch_bounds__(256) void ln_bwd_kernel(LnBwd a) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int RPW = PART ? kLnRowsPerWave : 1;
  const int L = a.L;
  float gp[VPT], bp[VPT], xp[VPT];
#pragma unroll
  for (int q = 0; q < VPT; ++q) { gp[q] = 0.f; bp[q] = 0.f; xp[q] = 0.f; }
  for (int i = 0; i < RPW; ++i) {
    const int row = (blockIdx.x * 4 + wv) * RPW + i;
    if (row >= a.R) break;  // wave-uniform
    const int64_t yo = ioff(a.dyrow, row);
    constexpr bool PRE = VPT <= 16;  // long rows: gamma read at its use (register budget)
    float dyl[VPT], ul[VPT], gl[PRE ? VPT : 1], xin[VPT];
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const int e = min(lane + 64 * q, L - 1);
      dyl[q] = a.dy[yo + (int64_t)e * a.dyes];
      ul[q] = a.u[(int64_t)row * L + e];
      if constexpr (PRE) gl[q] = a.g[e];
    }
    const int64_t xo = ioff(a.dxrow, row);
    if (a.beta != 0.f) {
#pragma unroll
      for (int q = 0; q < VPT; ++q) xin[q] = a.dx[xo + (int64_t)min(lane + 64 * q, L - 1) * a.dxes];
    }
    const float mean = a.mu[row], rs = a.rs[row];
    float dyv[VPT], xh[VPT];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      int e = lane + 64 * q;
      dyv[q] = 0.f; xh[q] = 0.f;
      if (e < L) {
        float dy = dyl[q];
        if (a.drop_p > 0.f) dy *= drop_scale(a.seed, a.which, (uint64_t)row * L + e + a.drop_off, a.drop_p);
        float x = (ul[q] - mean) * rs;
        dyv[q] = dy; xh[q] = x;
        float dxh = dy * (PRE ? gl[PRE ? q : 0] : a.g[e]);
        s1 += dxh; s2 += dxh * x;
        if (PART) {
          gp[q] += dy * x;
          bp[q] += dy;
        } else {
          if (a.gcontrib) a.gcontrib[(int64_t)row * L + e] = dy * x;
          if (a.bcontrib) a.bcontrib[(int64_t)row * L + e] = dy;
        }
      }
    }
    s1 = wave_sum(s1) / L;
    s2 = wave_sum(s2) / L;
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      int e = lane + 64 * q;
      if (e < L) {
        float dx = rs * (dyv[q] * (PRE ? gl[PRE ? q : 0] : a.g[e]) - s1 - xh[q] * s2);
        int64_t oo = xo + (int64_t)e * a.dxes;
        if (a.beta != 0.f) dx += a.beta * xin[q];
        a.dx[oo] = dx;
        if (PART) xp[q] += dx;
      }
    }
  }
  if constexpr (PART) {
    __shared__ float red[2][4][64 * VPT];
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      red[0][wv][lane + 64 * q] = gp[q];
      red[1][wv][lane + 64 * q] = bp[q];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < L; e += 256) {
      const float g = red[0][0][e] + red[0][1][e] + red[0][2][e] + red[0][3][e];
      const float b = red[1][0][e] + red[1][1][e] + red[1][2][e] + red[1][3][e];
      if (a.gpart) a.gpart[(int64_t)blockIdx.x * L + e] = g;
      if (a.bpart) a.bpart[(int64_t)blockIdx.x * L + e] = b;
    }
    if (a.xpart) {  // the dx sums through the same LDS rows (workgroup-uniform branch)
      __syncthreads();
#pragma unroll
      for (int q = 0; q < VPT; ++q) red[0][wv][lane + 64 * q] = xp[q];
      __syncthreads();
      for (int e = threadIdx.x; e < L; e += 256)
        a.xpart[(int64_t)blockIdx.x * L + e] = red[0][0][e] + red[0][1][e] + red[0][2][e] + red[0][3][e];
    }
  }
}

// =====================================================================================
// per-(device, stream) zero-armed ticket counters for single-launch reductions: kernels
// that take tickets re-arm them (write 0) before they finish, so consecutive launches on
// one stream can share them; different streams never do.
// =====================================================================================
}  // namespace

int* stream_counters(hipStream_t st, int n) {
  constexpr int kCounters = 1 << 16;
  if (n > kCounters) return nullptr;
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, int*> table;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(mu);
  auto key = std::make_pair(dev, st);
  auto it = table.find(key);
  if (it != table.end()) return it->second;
  if (table.size() >= 256) return nullptr;
  int* p = nullptr;
  if (hipMalloc(&p, sizeof(int) * kCounters) != hipSuccess) return nullptr;
  if (hipMemsetAsync(p, 0, sizeof(int) * kCounters, st) != hipSuccess) {
    (void)hipFree(p);
    return nullptr;
  }
  table[key] = p;
  return p;
}

namespace {

// =====================================================================================
// reductions
// =====================================================================================
// Column sums of up to 4 same-shape sources in one launch pair (deterministic: fixed
// reduction order, no atomics).
// stage 1: each source viewed as (A, E) rows, E = O*I contiguous per row a.
// part[p][s*O + o] = sum over the p-th chunk of rows, sum_i in_s[a][o*I+i].
// Column sums land in LDS (colv[E], dynamic), then each output folds its I columns, so
// stage 2 reads a compact (P, nsrc*O) slab.  E <= 256: the block is R' = 256/E row-lanes x
// E columns (consecutive threads read consecutive addresses); E > 256: threads stride e.
__global__ __launch_bounds__(256) void colsum_stage1(ColsumArgs a) {
  extern __shared__ float colv[];
  __shared__ float red[256];
  const int E = a.O * a.I, OT = a.nsrc * a.O;
  const int p = blockIdx.x;
  const int64_t a0 = (int64_t)p * a.achunk, a1 = min(a.A, a0 + a.achunk);
  const int t = threadIdx.x;
  for (int src = 0; src < a.nsrc; ++src) {
    const float* __restrict__ in = a.in[src];
    if (E <= 256) {
      const int R = 256 / E;
      const int r = t / E, e = t % E;
      float sum = 0.f;
      if (r < R) {
#pragma unroll 8
        for (int64_t aa = a0 + r; aa < a1; aa += R) sum += in[aa * E + e];
      }
      red[t] = sum;
      __syncthreads();
      if (t < E) {
        float tot = 0.f;
        for (int q = 0; q < R; ++q) tot += red[q * E + t];
        colv[t] = tot;
      }
    } else {
      for (int e = t; e < E; e += 256) {
        float sum = 0.f;
#pragma unroll 8
        for (int64_t aa = a0; aa < a1; ++aa) sum += in[aa * E + e];
        colv[e] = sum;
      }
    }
    __syncthreads();
    for (int o = t; o < a.O; o += 256) {
      float sum = 0.f;
      for (int i = 0; i < a.I; ++i) sum += colv[o * a.I + i];
      a.part[(int64_t)p * OT + src * a.O + o] = sum;
    }
    __syncthreads();
  }
}
// stage 2: out_s[o] = beta*out_s[o] + sum_p part[p][s*O + o].  1024 threads = OL output
// lanes x PG row groups (coalesced along o), LDS tree over the groups (fixed order).
__global__ __launch_bounds__(1024) void colsum_stage2(ColsumArgs a) {
  __shared__ float red[1024];
  const int OT = a.nsrc * a.O;
  const int t = threadIdx.x;
  const int PG = 1024 / a.OL, g = t / a.OL, l = t % a.OL;
  const int o = blockIdx.x * a.OL + l;
  float sum = 0.f;
  if (o < OT) {
#pragma unroll 8
    for (int pp = g; pp < a.P; pp += PG) sum += a.part[(int64_t)pp * OT + o];
  }
  red[t] = sum;
  __syncthreads();
  for (int w = PG >> 1; w > 0; w >>= 1) {
    if (g < w) red[t] += red[t + w * a.OL];
    __syncthreads();
  }
  if (g == 0 && o < OT) {
    const int src = o / a.O, oo = o - src * a.O;
    float* d = a.out[src] + (int64_t)oo * a.ostride;
    *d = (a.beta != 0.f ? a.beta * *d : 0.f) + red[l];
  }
}

// -------------------------------------------------------------------------------------
// Single-launch column sums (deterministic).  Each source is an (A, E) row-major matrix.
// Columns: E <= 256 -> one group, RP = 256/E rows per block pass (thread t: column t % E,
// row lane t / E, so a pass reads RP*E consecutive floats); E > 256 -> groups of
// W = I*floor(256/I) columns, one row per pass.  Rows: R chunks (grid.x), ~1K blocks in
// total, 8 independent loads in flight per thread.  The cross-block sum is a two-level
// ticket tree: the last block of each run of 32 row chunks adds their partials (fixed
// order) into a level-2 partial; the last of those adds the <= 32 level-2 partials, folds
// each output's I columns and stores.  Tickets are re-armed (0) by the blocks that drew the
// last one, so the next launch on this stream finds them zero.  One launch, no float atomics.
// -------------------------------------------------------------------------------------
constexpr int kCsW = 256;   // partial width (columns)
constexpr int kCsL1 = 32;   // row chunks per level-1 ticket

struct Colsum2dArgs {
  const float* in[4] = {};
  float* out[4] = {};
  int nsrc = 1;
  int64_t A = 0; int O = 0, I = 1, E = 0;
  int W = 256, G = 1, RP = 1, R = 1, R2 = 1;  // group width, groups/source, rows per pass, chunks, level-2 count
  int64_t achunk = 1;
  int64_t ostride = 1; float beta = 0.f;
  float* part = nullptr;   // level 1: [nsrc*G][R][256], then level 2: [nsrc*G][R2][256]
  int* cnt = nullptr;      // [nsrc*G][R2] level-1 tickets, then [nsrc*G] level-2 tickets
};

__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// consumer side of the hand-off: agent acquire, then wait for the invalidate to complete
// (the caller's workgroup barrier holds the other waves behind it)
__device__ __forceinline__ void colsum_acquire() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// sum of n <= 32 partial rows p[q*256 + t] in fixed order; all loads issued before the
// first add (one memory round trip: the sc1 loads are served beyond the XCD's L2)
__device__ __forceinline__ float sum_partials(const float* p, int n, int t) {
  float u[kCsL1];
#pragma unroll
  for (int k = 0; k < kCsL1; ++k) u[k] = k < n ? ld_agent(p + (int64_t)k * kCsW + t) : 0.f;
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < kCsL1; ++k) v += u[k];
  return v;
}

__global__ __launch_bounds__(256) void colsum2d_kernel(Colsum2dArgs a) {
  __shared__ float red[kCsW];
  __shared__ int last;
  const int t = threadIdx.x;
  const int r = blockIdx.x, gidx = blockIdx.y;  // gidx = src * G + group
  const int src = gidx / a.G, grp = gidx - src * a.G;
  const float* __restrict__ in = a.in[src];
  const int64_t a0 = (int64_t)r * a.achunk, a1 = min(a.A, a0 + a.achunk);
  // thread -> (column, row lane)
  int col, lane;
  bool act;
  if (a.G == 1 && a.E <= kCsW) { col = t % a.E; lane = t / a.E; act = lane < a.RP; }
  else { col = grp * a.W + t; lane = 0; act = t < a.W && col < a.E; }
  float s0 = 0.f, s1 = 0.f;
  if (act) {
    const int RP = a.RP;
    int64_t aa = a0 + lane;
    for (; aa + 15 * RP < a1; aa += 16 * RP) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = in[(aa + (int64_t)u * RP) * a.E + col];
#pragma unroll
      for (int u = 0; u < 16; u += 2) { s0 += v[u]; s1 += v[u + 1]; }
    }
    for (; aa < a1; aa += RP) s0 += in[aa * a.E + col];
  }
  // fold the row lanes in fixed order: thread t holds column t % E of lane t / E (E <= 256)
  red[t] = act ? s0 + s1 : 0.f;
  __syncthreads();
  float colv = red[t];
  if (a.G == 1 && a.E <= kCsW) {
    colv = 0.f;
    if (t < a.E)
      for (int l = 0; l < a.RP; ++l) colv += red[l * a.E + t];
  }
  // hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, "valid forms"): producers
  // store sc1 (agent-scope relaxed atomics), every storing wave drains them (vmcnt(0)), a
  // barrier, then ONE lane's agent-scope ticket add.  The block whose add came last issues
  // an agent-scope ACQUIRE (L1 invalidate, only the winning blocks pay it) before any read
  // of the partials, so the hand-off does not rest on the measured sc1-load table (whose
  // row assumes one workgroup per CU).  No release fence on the producers (it would write
  // back the XCD's whole L2): sc1 stores already bypass it.
  float* p1 = a.part + ((int64_t)gidx * a.R + r) * kCsW;
  if (t < a.W) st_agent(p1 + t, colv);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int c1 = r / kCsL1;
  const int n1 = min(kCsL1, a.R - c1 * kCsL1);
  if (t == 0) {
    last = atomicAdd(a.cnt + (int64_t)gidx * a.R2 + c1, 1) == n1 - 1;
    if (last) colsum_acquire();
  }
  __syncthreads();
  if (!last) return;
  float* p2 = a.part + ((int64_t)a.nsrc * a.G * a.R + (int64_t)gidx * a.R2 + c1) * kCsW;
  if (t < a.W) st_agent(p2 + t, sum_partials(a.part + ((int64_t)gidx * a.R + (int64_t)c1 * kCsL1) * kCsW, n1, t));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* cnt2 = a.cnt + (int64_t)a.nsrc * a.G * a.R2 + gidx;
  if (t == 0) {
    __hip_atomic_store(a.cnt + (int64_t)gidx * a.R2 + c1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = atomicAdd(cnt2, 1) == a.R2 - 1;
    if (last) colsum_acquire();
  }
  __syncthreads();
  if (!last) return;
  red[t] = t < a.W ? sum_partials(a.part + ((int64_t)a.nsrc * a.G * a.R + (int64_t)gidx * a.R2) * kCsW, a.R2, t)
                   : 0.f;
  __syncthreads();
  const int opg = a.W / a.I;
  if (t < opg) {
    const int o = grp * opg + t;
    if (o < a.O) {
      float v = 0.f;
      for (int i = 0; i < a.I; ++i) v += red[t * a.I + i];
      float* d = a.out[src] + (int64_t)o * a.ostride;
      *d = (a.beta != 0.f ? a.beta * *d : 0.f) + v;
    }
  }
  if (t == 0) __hip_atomic_store(cnt2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// =====================================================================================
// Temporal attention on the matrix cores: T <= 16 with T % 4 == 0, d_k = d_v = 32 — the
// production TAt (model/DSTAGNN_my.py:27-67 at T = 12, d_k = d_v = 32).  One wave per
// (b, f, head) problem (four per workgroup); the T x T tile is padded to 16 x 16 and every
// product is a v_mfma_f32_16x16x4_f32 chain (fragments: A[l&15][k = l>>4], B[k = l>>4][l&15],
// D[4(l>>4) + r][l&15]) whose operands come from global memory straight into registers.
// Each product's contraction index is assigned to (k slot q = l>>4, step s) as 4q + s, so an
// accumulator tile whose ROW index is that contraction index is, register s for register s,
// the next product's A operand: scores -> P -> ctx in the forward, dA -> dS -> dK / dV in the
// backward, with one 16 x 16 LDS transpose of dS for dQ.  (The VALU wave kernels above spend
// ~2 400 VALU and ~700 LDS instructions per problem on index arithmetic and LDS operands.)
// =====================================================================================
constexpr int kTmD = 32;  // d_k = d_v of the matrix-core variant

__device__ __forceinline__ float xor_max_16(float v) {
  v = fmaxf(v, __shfl_xor(v, 1, 64));
  v = fmaxf(v, __shfl_xor(v, 2, 64));
  v = fmaxf(v, __shfl_xor(v, 4, 64));
  return fmaxf(v, __shfl_xor(v, 8, 64));
}
__device__ __forceinline__ float xor_sum_16(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v + __shfl_xor(v, 8, 64);
}
__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int T>
__global__ __launch_bounds__(256) void tat_fwd_mfma_kernel(TatArgs a) {
  static_assert(T % 4 == 0 && T <= 16, "one 16 x 16 tile, float4 rows");
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, c = l & 15, q = l >> 4;
  const int id = blockIdx.x * kTatW + w;
  if (id >= a.B * a.F * a.h) return;  // no barrier in this kernel
  const int h = a.h, hd = id % h, bf = id / h, b = bf / a.F;
  const int ld = 3 * h * kTmD;
  const float* Qp = a.qkv + (int64_t)bf * T * ld + hd * kTmD;
  const float* Kp = Qp + h * kTmD;
  const float* Vp = Qp + 2 * h * kTmD;
  const bool vi = c < T, vj = q < T / 4;
  // ctx's B operand V[j = 4q + s][d = c + 16t] first: it does not depend on the scores
  float vv[2][4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int t = 0; t < 2; ++t) vv[t][s] = (4 * q + s < T) ? Vp[(int64_t)(4 * q + s) * ld + c + 16 * t] : 0.f;
  // S^T = K Q^T: A[m = j][k = d] = K[j = c][8q + s], B[k = d][n = i] = Q[i = c][8q + s]
  float4 k0 = {0.f, 0.f, 0.f, 0.f}, k1 = k0, q0 = k0, q1 = k0;
  if (vi) {
    k0 = *reinterpret_cast<const float4*>(Kp + (int64_t)c * ld + 8 * q);
    k1 = *reinterpret_cast<const float4*>(Kp + (int64_t)c * ld + 8 * q + 4);
    q0 = *reinterpret_cast<const float4*>(Qp + (int64_t)c * ld + 8 * q);
    q1 = *reinterpret_cast<const float4*>(Qp + (int64_t)c * ld + 8 * q + 4);
  }
  const int64_t sbase = (int64_t)id * T * T;
  const float* rp = nullptr;
  if (a.res_mode == DSTAGNN_RES_BCAST) rp = a.res + ((int64_t)b * h + hd) * T * T;
  else if (a.res_mode == DSTAGNN_RES_FULL) rp = a.res + sbase;
  float4 rr = {0.f, 0.f, 0.f, 0.f};
  if (rp && vi && vj) rr = *reinterpret_cast<const float4*>(rp + c * T + 4 * q);
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = mfma16(k0.x, q0.x, acc);
  acc = mfma16(k0.y, q0.y, acc);
  acc = mfma16(k0.z, q0.z, acc);
  acc = mfma16(k0.w, q0.w, acc);
  acc = mfma16(k1.x, q1.x, acc);
  acc = mfma16(k1.y, q1.y, acc);
  acc = mfma16(k1.z, q1.z, acc);
  acc = mfma16(k1.w, q1.w, acc);
  // lane (c, q) holds S[i = c][j = 4q + r]
  const float rv[4] = {rr.x, rr.y, rr.z, rr.w};
  float sc[4], p[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    sc[r] = acc[r] * a.scale;
    sc[r] += rv[r];
  }
  if (vi && vj) *reinterpret_cast<float4*>(a.re_at + sbase + c * T + 4 * q) = make_float4(sc[0], sc[1], sc[2], sc[3]);
  // softmax over the query axis i = the 16 lanes c of this quarter (column j = 4q + r)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float m = xor_max_16(vi ? sc[r] : -INFINITY);
    const float e = vi ? __expf(sc[r] - m) : 0.f;
    const float inv = 1.f / xor_sum_16(e);
    p[r] = vj ? e * inv : 0.f;
  }
  if (vi && vj) *reinterpret_cast<float4*>(a.att + sbase + c * T + 4 * q) = make_float4(p[0], p[1], p[2], p[3]);
  // ctx = P V: A[m = i][k = j] = P[i = c][j = 4q + s] = p[s], B = vv
  floatx4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    c0 = mfma16(p[s], vv[0][s], c0);
    c1 = mfma16(p[s], vv[1][s], c1);
  }
  const int ldc = h * kTmD;
  float* cb = a.ctx + (int64_t)bf * T * ldc + hd * kTmD + c;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 4 * q + r;
    if (i < T) {
      cb[(int64_t)i * ldc] = c0[r];
      cb[(int64_t)i * ldc + 16] = c1[r];
    }
  }
}

template <int T>
__global__ __launch_bounds__(256) void tat_bwd_mfma_kernel(TatArgs a) {
  static_assert(T % 4 == 0 && T <= 16, "one 16 x 16 tile");
  __shared__ float tr[kTatW][16][17];  // per-wave dS transpose (dQ's A operand)
  __shared__ float red[kTatW][T * T];  // F-sum: the workgroup's four dS tiles
  __shared__ int last;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, c = l & 15, q = l >> 4;
  const int h = a.h, P = a.B * a.F * h;
  const int nch = a.F / kTatW;
  int id;
  if (a.dres_sum) {  // workgroup = (b, head, four consecutive f): wave w takes f = 4 ch + w
    const int bh = blockIdx.x / nch, ch = blockIdx.x - bh * nch;
    id = ((bh / h) * a.F + ch * kTatW + w) * h + bh % h;
  } else {
    id = blockIdx.x * kTatW + w;
  }
  const bool live = id < P;
  const int hd = id % h, bf = id / h;
  const int ld = 3 * h * kTmD, ldc = h * kTmD;
  const float* Qp = a.qkv + (int64_t)bf * T * ld + hd * kTmD;
  const float* Kp = Qp + h * kTmD;
  const float* Vp = Qp + 2 * h * kTmD;
  const float* Cp = a.dctx + (int64_t)bf * T * ldc + hd * kTmD;
  const int64_t sbase = (int64_t)id * T * T;
  const bool vj = c < T;  // lane column j = c; rows i = 4q + r
  // every load up front: dA's operands dC[i = c][8q + s] / V[j = c][8q + s]; the B operands
  // [4q + s][c + 16t] of dV (dC), dK (Q) and dQ (K); A[i = 4q + r][j = c] and d re_At
  float4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = d0, v0 = d0, v1 = d0;
  float cb[2][4], qb[2][4], kb[2][4], at[4], dr[4];
  if (live && vj) {
    d0 = *reinterpret_cast<const float4*>(Cp + (int64_t)c * ldc + 8 * q);
    d1 = *reinterpret_cast<const float4*>(Cp + (int64_t)c * ldc + 8 * q + 4);
    v0 = *reinterpret_cast<const float4*>(Vp + (int64_t)c * ld + 8 * q);
    v1 = *reinterpret_cast<const float4*>(Vp + (int64_t)c * ld + 8 * q + 4);
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int i = 4 * q + s;
    const bool ok = live && i < T;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      cb[t][s] = ok ? Cp[(int64_t)i * ldc + c + 16 * t] : 0.f;
      qb[t][s] = ok ? Qp[(int64_t)i * ld + c + 16 * t] : 0.f;
      kb[t][s] = ok ? Kp[(int64_t)i * ld + c + 16 * t] : 0.f;
    }
    at[s] = ok && vj ? a.att[sbase + i * T + c] : 0.f;
    dr[s] = ok && vj && a.dre ? a.dre[sbase + i * T + c] : 0.f;
  }
  // dA = dC V^T: D[m = i][n = j], A[m = i][k = d] = dC[i = c][8q + s], B[k = d][n = j] = V[j = c][8q + s]
  floatx4 dA = {0.f, 0.f, 0.f, 0.f};
  dA = mfma16(d0.x, v0.x, dA);
  dA = mfma16(d0.y, v0.y, dA);
  dA = mfma16(d0.z, v0.z, dA);
  dA = mfma16(d0.w, v0.w, dA);
  dA = mfma16(d1.x, v1.x, dA);
  dA = mfma16(d1.y, v1.y, dA);
  dA = mfma16(d1.z, v1.z, dA);
  dA = mfma16(d1.w, v1.w, dA);
  // column softmax backward over i (this lane's four rows, then the quarters): dS = A (dA - sum_i A dA) + d re_At
  float cs = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) cs = fmaf(at[r], dA[r], cs);
  cs = xor_sum_1632(cs);
  float ds[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) ds[r] = at[r] * (dA[r] - cs) + dr[r];
  if (a.keep_ds && live && vj) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * q + r < T) a.dscore[sbase + (4 * q + r) * T + c] = ds[r];
  }
  // dV = A^T dC and dK = dS^T Q: A operand [m = j = c][k = i = 4q + s] = at[s] / ds[s]
  floatx4 z = {0.f, 0.f, 0.f, 0.f};
  floatx4 gv0 = z, gv1 = z, gk0 = z, gk1 = z, gq0 = z, gq1 = z;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    gv0 = mfma16(at[s], cb[0][s], gv0);
    gv1 = mfma16(at[s], cb[1][s], gv1);
    gk0 = mfma16(ds[s], qb[0][s], gk0);
    gk1 = mfma16(ds[s], qb[1][s], gk1);
  }
  // dQ = dS K: A operand [m = i = c][k = j = 4q + s] = dS[c][4q + s], through LDS
#pragma unroll
  for (int r = 0; r < 4; ++r) tr[w][4 * q + r][c] = ds[r];
  if (a.dres_sum && vj) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * q + r < T) red[w][(4 * q + r) * T + c] = ds[r];
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float x = tr[w][c][4 * q + s];
    gq0 = mfma16(x, kb[0][s], gq0);
    gq1 = mfma16(x, kb[1][s], gq1);
  }
  if (live) {
    float* db = a.dqkv + (int64_t)bf * T * ld + hd * kTmD + c;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * q + r;
      if (i >= T) continue;
      float* row = db + (int64_t)i * ld;
      row[0] = gq0[r] * a.scale;
      row[16] = gq1[r] * a.scale;
      row[h * kTmD] = gk0[r] * a.scale;
      row[h * kTmD + 16] = gk1[r] * a.scale;
      row[2 * h * kTmD] = gv0[r];
      row[2 * h * kTmD + 16] = gv1[r];
    }
  }
  if (!a.dres_sum) return;
  // res_att gradient sum_f dS (deterministic): the four tiles in wave order, one partial per
  // workgroup (sc1 stores, drained, barrier), a ticket per (b, head); the last of its nch
  // workgroups acquires and adds the partials in chunk order (colsum2d's hand-off)
  const int t = threadIdx.x, bh = blockIdx.x / nch, ch = blockIdx.x - bh * nch;
  float* part = a.dscore + (int64_t)bh * nch * T * T;
  if (t < T * T) st_agent(part + (int64_t)ch * T * T + t, ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    last = atomicAdd(a.cnt + bh, 1) == nch - 1;
    if (last) {
      colsum_acquire();
      __hip_atomic_store(a.cnt + bh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
  }
  __syncthreads();
  if (!last || t >= T * T) return;
  float v = 0.f;
  for (int k = 0; k < nch; ++k) v += ld_agent(part + (int64_t)k * T * T + t);
  a.dres_sum[(int64_t)bh * T * T + t] = v;
}

// out[a][i] = beta*out + sum_m in[a][m][i]; grid (i blocks, a)
// out[a][i] = beta*out[a][i] + sum_m in[a][m][i]: a workgroup owns 32 consecutive i of one a;
// its 8 wave-quarters sum interleaved m (8-way parallel chains per output instead of one
// Mm-long chain), combined through LDS in a fixed order.
__global__ __launch_bounds__(256) void sum_middle_kernel(const float* __restrict__ in, int64_t A, int Mm, int64_t I,
                                                         float* __restrict__ out, float beta) {
  __shared__ float red[8][33];
  const int64_t a = blockIdx.y;
  const int il = threadIdx.x & 31, mg = threadIdx.x >> 5;
  const int64_t i = (int64_t)blockIdx.x * 32 + il;
  const float* src = in + a * Mm * I;
  float s = 0.f;
  if (i < I) {
#pragma unroll 4
    for (int m = mg; m < Mm; m += 8) s += src[(int64_t)m * I + i];
  }
  red[mg][il] = s;
  __syncthreads();
  if (mg == 0 && i < I) {
    float t = red[0][il];
#pragma unroll
    for (int g = 1; g < 8; ++g) t += red[g][il];
    float* d = out + a * I + i;
    *d = (beta != 0.f ? beta * *d : 0.f) + t;
  }
}

// the same sums with float4 columns (I % 4 == 0, 16-B aligned rows): a workgroup takes 256
// consecutive columns (64 lanes x 4), its 4 waves split the Mm rows, 8 row loads in flight per
// lane (the scalar kernel's 128-B row pieces ran at ~2 TB/s: sum_middle 5-6 us at PEMS08)
__global__ __launch_bounds__(256) void sum_middle4_kernel(const float* __restrict__ in, int64_t A, int Mm, int64_t I,
                                                          float* __restrict__ out, float beta) {
  __shared__ floatx4 red[4][64];
  const int64_t a = blockIdx.y;
  const int il = threadIdx.x & 63, mg = threadIdx.x >> 6;
  const int64_t i4 = (int64_t)blockIdx.x * 64 + il;  // float4 column
  const floatx4* src = reinterpret_cast<const floatx4*>(in + a * Mm * I);
  const int64_t I4 = I / 4;
  floatx4 s = {0.f, 0.f, 0.f, 0.f};
  if (i4 < I4) {
    int m = mg;
    for (; m + 28 < Mm; m += 32) {
      floatx4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)(m + 4 * u) * I4 + i4];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; m < Mm; m += 4) s += src[(int64_t)m * I4 + i4];
  }
  red[mg][il] = s;
  __syncthreads();
  if (mg == 0 && i4 < I4) {
    floatx4 t = ((red[0][il] + red[1][il]) + red[2][il]) + red[3][il];
    floatx4* d = reinterpret_cast<floatx4*>(out + a * I) + i4;
    if (beta != 0.f) t += beta * *d;
    *d = t;
  }
}

__global__ __launch_bounds__(256) void relu_mask_kernel(const float* __restrict__ g, const float* __restrict__ y,
                                                        float* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = y[i] > 0.f ? g[i] : 0.f;
}

// =====================================================================================
// Chebyshev spatial-attention softmax (column softmax over source node i)
// grid ceil(N/64)*B*K (see sm_tile), block 512 = 64 columns x 8 row groups
// =====================================================================================
constexpr int kSmG = 8;  // row groups per workgroup (64 columns x 8 groups = 512 threads)
constexpr int kSmCondN = 1024;  // N from which the softmax kernels load under the support only

// workgroup -> (column group, b, k) with b fastest: the B workgroups that share one
// (k, column group) tile of A_pa, M_k and T_k are dispatched together (round-robin over the
// XCDs, B/8 per XCD), so those tiles come from L2 instead of HBM once per batch element
__device__ __forceinline__ void sm_tile(const ChebSm& a, int* b, int* k, int* cg) {
  const int ncg = (a.N + 63) / 64;
  int id = blockIdx.x;
  *b = id % a.B; id /= a.B;
  *cg = id % ncg;
  *k = id / ncg;
}

// CL ("conditional loads"): read M_k (fwd) and P / dW (bwd) only under the A_pa / T_k
// support.  Pays at large N (HBM-bound passes over N^2 tiles); at small N (PEMS08, 170) the
// passes are latency chains and the dependent load costs more than the bytes it saves.
template <bool CL>
__global__ __launch_bounds__(512) void cheb_softmax_fwd_kernel(ChebSm a) {
  __shared__ float sm_m[kSmG][64], sm_l[kSmG][64];
  const int N = a.N;
  int b, k, cg;
  sm_tile(a, &b, &k, &cg);
  const int bk = b * a.K + k;
  const int cj = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int j = cg * 64 + cj;
  const float* S = a.S + (int64_t)bk * N * N;
  const float* Mk = a.mask[k];
  const float* Tk = a.cheb + (int64_t)k * N * N;
  // one pass: online column max and sum of exp (4 independent chains, loads batched)
  float m = -INFINITY, l = 0.f;
  if (j < N) {
    float m4[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, l4[4] = {0.f, 0.f, 0.f, 0.f};
    int i = g;
    for (; i + 3 * kSmG < N; i += 4 * kSmG) {
      float z[4], w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = (int64_t)(i + u * kSmG) * N + j;
        z[u] = S[o];
        w[u] = a.apa[o];
      }
      float mv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) mv[u] = CL ? 0.f : Mk[(int64_t)(i + u * kSmG) * N + j];
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // CL: M_k read only under the A_pa support
        if (CL) {
          if (w[u] != 0.f) z[u] += w[u] * Mk[(int64_t)(i + u * kSmG) * N + j];
        } else {
          z[u] += w[u] * mv[u];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float mn = fmaxf(m4[u], z[u]);
        l4[u] = l4[u] * __expf(m4[u] - mn) + __expf(z[u] - mn);
        m4[u] = mn;
      }
    }
    for (; i < N; i += kSmG) {
      const int64_t o = (int64_t)i * N + j;
      const float w = a.apa[o];
      const float z = S[o] + (CL ? (w != 0.f ? w * Mk[o] : 0.f) : w * Mk[o]);
      const float mn = fmaxf(m4[0], z);
      l4[0] = l4[0] * __expf(m4[0] - mn) + __expf(z - mn);
      m4[0] = mn;
    }
    m = fmaxf(fmaxf(m4[0], m4[1]), fmaxf(m4[2], m4[3]));
#pragma unroll
    for (int u = 0; u < 4; ++u) l += m4[u] == -INFINITY ? 0.f : l4[u] * __expf(m4[u] - m);
  }
  sm_m[g][cj] = m; sm_l[g][cj] = l;
  __syncthreads();
  float M = sm_m[0][cj];
#pragma unroll
  for (int q = 1; q < kSmG; ++q) M = fmaxf(M, sm_m[q][cj]);
  float L = 0.f;
#pragma unroll
  for (int q = 0; q < kSmG; ++q) L += sm_m[q][cj] == -INFINITY ? 0.f : sm_l[q][cj] * __expf(sm_m[q][cj] - M);
  const float inv = 1.f / L;
  if (j < N) {
    float* P = a.P + (int64_t)bk * N * N;
    float* W = a.W ? a.W + (int64_t)bk * N * N : nullptr;
#pragma unroll 2
    for (int i = g; i < N; i += kSmG) {
      const int64_t o = (int64_t)i * N + j;
      const float w = a.apa[o];
      const float z = S[o] + (CL ? (w != 0.f ? w * Mk[o] : 0.f) : w * Mk[o]);
      const float p = __expf(z - M) * inv;
      P[o] = p;
      if (W) W[o] = Tk[o] * p;
    }
  }
}

// dz = P * (T*dW - sum_i P*T*dW)   written to dz (may alias dW)
template <bool CL>
__global__ __launch_bounds__(512) void cheb_softmax_bwd_kernel(ChebSm a) {
  __shared__ float sm_c[kSmG][64];
  const int N = a.N;
  int b, k, cg;
  sm_tile(a, &b, &k, &cg);
  const int bk = b * a.K + k;
  const int cj = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int j = cg * 64 + cj;
  const float* P = a.P + (int64_t)bk * N * N;
  const float* dW = a.dW + (int64_t)bk * N * N;
  const float* Tk = a.cheb + (int64_t)k * N * N;
  float c = 0.f;
  if (j < N) {
    // dW is only defined where T_k is non-zero (the sparse path writes the support only,
    // no memset) and only needed there: T_k (shared by the batch, from L2) is read first and
    // P / dW only under its support, so a sparse graph costs one dense pass over P, not
    // three over P, T_k and dW.  Off-support garbage in dW never propagates.
    float c4[4] = {0.f, 0.f, 0.f, 0.f};
    int i = g;
    for (; i + 3 * kSmG < N; i += 4 * kSmG) {
      float tv[4], pv[4], dv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = (int64_t)(i + u * kSmG) * N + j;
        tv[u] = Tk[o];
        if (!CL) { pv[u] = P[o]; dv[u] = dW[o]; }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t o = (int64_t)(i + u * kSmG) * N + j;
        if (CL) {
          if (tv[u] != 0.f) c4[u] += P[o] * (tv[u] * dW[o]);
        } else {
          c4[u] += pv[u] * (tv[u] != 0.f ? tv[u] * dv[u] : 0.f);
        }
      }
    }
    for (; i < N; i += kSmG) {
      const int64_t o = (int64_t)i * N + j;
      const float t = Tk[o];
      if (t != 0.f) c4[0] += P[o] * (t * dW[o]);
    }
    c = (c4[0] + c4[1]) + (c4[2] + c4[3]);
  }
  sm_c[g][cj] = c;
  __syncthreads();
  c = 0.f;
#pragma unroll
  for (int q = 0; q < kSmG; ++q) c += sm_c[q][cj];
  if (j < N) {
    float* dz = a.dz + (int64_t)bk * N * N;
    int i = g;
    for (; i + kSmG < N; i += 2 * kSmG) {
      const int64_t o0 = (int64_t)i * N + j, o1 = o0 + (int64_t)kSmG * N;
      const float t0 = Tk[o0], t1 = Tk[o1], p0 = P[o0], p1 = P[o1];
      float w0, w1;
      if (CL) {
        w0 = t0 != 0.f ? t0 * dW[o0] : 0.f;
        w1 = t1 != 0.f ? t1 * dW[o1] : 0.f;
      } else {
        const float d0 = dW[o0], d1 = dW[o1];
        w0 = t0 != 0.f ? t0 * d0 : 0.f;
        w1 = t1 != 0.f ? t1 * d1 : 0.f;
      }
      dz[o0] = p0 * (w0 - c);
      dz[o1] = p1 * (w1 - c);
    }
    for (; i < N; i += kSmG) {
      const int64_t o = (int64_t)i * N + j;
      const float t = Tk[o];
      dz[o] = P[o] * ((t != 0.f ? t * dW[o] : 0.f) - c);
    }
  }
}

// dM_k[i][j] = A_pa[i][j] * sum_b dz[b][k][i][j]
__global__ __launch_bounds__(256) void cheb_mask_grad_kernel(ChebSm a) {
  const int64_t NN = (int64_t)a.N * a.N;
  const int k = blockIdx.y;
  float* out = a.dmask[k];
  for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < NN; o += (int64_t)gridDim.x * blockDim.x) {
    const float w = a.apa[o];
    float s = 0.f;
    if (w != 0.f) {  // dz is read only under the A_pa support (dM_k is 0 elsewhere)
#pragma unroll 8
      for (int b = 0; b < a.B; ++b) s += a.dz[((int64_t)b * a.K + k) * NN + o];
    }
    out[o] = w * s;
  }
}


__global__ __launch_bounds__(256) void pack_rows_kernel(PackRows a) {
  int r0 = 0;
  for (int q = 0; q < a.n; ++q) {
    const int64_t n = (int64_t)a.rows[q] * a.cols;
    const float* src = a.unpack ? a.src[0] + (int64_t)r0 * a.cols : a.src[q];
    float* dst = a.unpack ? a.dst[q] : a.dst[0] + (int64_t)r0 * a.cols;
    if (dst)
      for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = src[i];
    r0 += a.rows[q];
  }
}

// blockIdx.y = segment; grid-stride over the segment's source elements
__global__ __launch_bounds__(256) void param_prep_kernel(ParamPrepK a) {
  const PrepSeg& g = a.seg[blockIdx.y];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < g.n; i += (int64_t)gridDim.x * 256) {
    if (g.kind == 8) {  // DESTINATION-indexed: src (R, p0) -> dst (R, p1) rows zero-padded to p1 >= p0
      const int64_t r = i / g.p1, c = i - r * g.p1;
      g.dst[g.dst_off + i] = c < g.p0 ? g.src[r * g.p0 + c] : 0.f;
      continue;
    }
    if (g.kind == 9) {  // DESTINATION-indexed zero-padded transpose: src (p3, p1) row-major;
      // dst row a, column b < p0 (row stride p2): src[b][a] where b < p3 and a < p1, else 0
      const int64_t ra = i / g.p0, cb = i - ra * g.p0;
      g.dst[g.dst_off + ra * g.p2 + cb] = (cb < g.p3 && ra < g.p1) ? g.src[cb * g.p1 + ra] : 0.f;
      continue;
    }
    const float v = g.src[i];
    int64_t o;
    switch (g.kind) {
      case 0: o = g.dst_off + i; break;
      case 1: {  // src (d, t, f) -> dst (d, f, t)
        const int64_t f = i % g.p0, r = i / g.p0, t = r % g.p1, d = r / g.p1;
        o = (d * g.p0 + f) * g.p1 + t;
        break;
      }
      case 2: {  // src (f, c) -> dst (f, k*C + c)
        const int64_t c = i % g.p0, f = i / g.p0;
        o = f * g.p1 + (int64_t)g.p2 * g.p0 + c;
        break;
      }
      case 3: {  // src (o, c, j) -> dst (o, j, c)
        const int64_t j = i % g.p1, r = i / g.p1, c = r % g.p0, oc = r / g.p0;
        o = (oc * g.p1 + j) * g.p0 + c;
        break;
      }
      case 7: {  // src (o, c, j) -> dst (j, c, o): the forward convolution's B operand, o fastest
        const int64_t j = i % g.p1, r = i / g.p1, c = r % g.p0, oc = r / g.p0;
        o = (j * g.p0 + c) * 2 * g.p0 + oc;
        break;
      }
      case 4: {  // src (o, c, j) -> dst (ks-1-j, o, c)
        const int64_t j = i % g.p1, r = i / g.p1, c = r % g.p0, oc = r / g.p0;
        o = ((g.p1 - 1 - j) * 2 * g.p0 + oc) * g.p0 + c;
        break;
      }
      case 5:  // elementwise product (A_pa o M_k: the reference's adj_pa.mul(mask[k]), :122)
        g.dst[i] = v * g.src2[i];
        continue;
      default:  // its transpose: (i, j) -> (j, i), N = p0
        o = (i % g.p0) * g.p0 + i / g.p0;
        g.dst[o] = v * g.src2[i];
        continue;
    }
    g.dst[o] = v;
  }
}


// =====================================================================================
// block tail: fcmy dropout, residual, ReLUs and LN over C (one thread per (b,n,t) row)
// =====================================================================================
// one workgroup per node (b,n): its C*T elements are contiguous in (B,N,C,T), so every
// pass is a coalesced sweep; the LN over C (stride T) goes through LDS.



// thcat[f][k*C + c] = theta_k[f][c]   (and the inverse for the gradients)
__global__ __launch_bounds__(256) void pack_theta_kernel(PackTheta a) {
  const int total = a.K * a.F * a.C;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i % a.C, r = i / a.C, f = r % a.F, k = r / a.F;
    const int64_t cat = (int64_t)f * a.K * a.C + (int64_t)k * a.C + c;
    if (a.unpack) {
      if (a.dst[k]) a.dst[k][(int64_t)f * a.C + c] = a.cat_in[cat];
    } else {
      a.cat_out[cat] = a.src[k][(int64_t)f * a.C + c];
    }
  }
}

__global__ void dropout_mask_kernel(float* out, int64_t n, uint64_t seed, uint32_t which, float p, uint64_t off) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = drop_scale(seed, which, (uint64_t)i + off, p);
}

inline unsigned grid1d(int64_t n, int64_t cap = 8192) {
  int64_t b = cdiv64(n, 256);
  return (unsigned)std::max<int64_t>(1, std::min(b, cap));
}

}  // namespace

// =====================================================================================
// launchers
// =====================================================================================
int op_transpose(const float* in, float* out, int R, int Cc, int batch, int64_t in_bs, int64_t out_bs, float beta,
                 hipStream_t st) {
  dim3 grid((unsigned)cdiv64(Cc, 32), (unsigned)cdiv64(R, 32), (unsigned)batch);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, st, in, out, R, Cc, in_bs, out_bs, beta);
  DS_CHECK_LAUNCH();
  return 0;
}

// dynamic LDS above 64 KB must be opted into per kernel (gfx950 has 160 KB per workgroup)
static int allow_lds(const void* kernel, size_t bytes) {
  hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) { set_last_error(std::string("LDS attribute: ") + hipGetErrorString(e)); return (int)e; }
  return 0;
}

// the matrix-core TAt kernels: T in {4, 8, 12, 16}, d_k = d_v = 32, 16-B aligned operands
// (float4 rows); DSTAGNN_TAT_MFMA=0 keeps the VALU wave kernels (A/B switch)
static bool tat_mfma_ok(int T, int dk, int dv, std::initializer_list<const float*> ptrs) {
  static const bool off = getenv("DSTAGNN_TAT_MFMA") && atoi(getenv("DSTAGNN_TAT_MFMA")) == 0;
  if (off || dk != kTmD || dv != kTmD || T % 4 != 0 || T < 4 || T > 16) return false;
  for (const float* p : ptrs)
    if (reinterpret_cast<uintptr_t>(p) % 16 != 0) return false;
  return true;
}
static void launch_tat_bwd_mfma(const TatArgs& a, dim3 grid, hipStream_t st) {
  const dim3 blk(64 * kTatW);
  switch (a.T) {
    case 4: hipLaunchKernelGGL(tat_bwd_mfma_kernel<4>, grid, blk, 0, st, a); break;
    case 8: hipLaunchKernelGGL(tat_bwd_mfma_kernel<8>, grid, blk, 0, st, a); break;
    case 12: hipLaunchKernelGGL(tat_bwd_mfma_kernel<12>, grid, blk, 0, st, a); break;
    default: hipLaunchKernelGGL(tat_bwd_mfma_kernel<16>, grid, blk, 0, st, a); break;
  }
}

static size_t tat_fwd_lds(int T, int dk, int dv) {
  return sizeof(float) * (size_t)(2 * T * (dk + 1) + T * (dv + 1) + T * T);
}
static size_t tat_bwd_lds(int T, int dk, int dv) {
  return sizeof(float) * (size_t)(2 * T * (dk + 1) + 2 * T * (dv + 1) + 2 * T * T);
}

int op_tat_fwd(int B, int F, int T, int h, int dk, int dv, const float* qkv, const float* res, int res_mode,
               float* re_at, float* att, float* ctx, hipStream_t st) {
  TatArgs a{};
  a.B = B; a.F = F; a.T = T; a.h = h; a.dk = dk; a.dv = dv;
  a.qkv = qkv; a.res = res; a.res_mode = res ? res_mode : 0; a.scale = 1.f / sqrtf((float)dk);
  a.re_at = re_at; a.att = att; a.ctx = ctx;
  const int P = B * F * h;
  if (tat_mfma_ok(T, dk, dv, {qkv, res, re_at, att})) {
    const dim3 grid((unsigned)cdiv64(P, kTatW)), blk(64 * kTatW);
    switch (T) {
      case 4: hipLaunchKernelGGL(tat_fwd_mfma_kernel<4>, grid, blk, 0, st, a); break;
      case 8: hipLaunchKernelGGL(tat_fwd_mfma_kernel<8>, grid, blk, 0, st, a); break;
      case 12: hipLaunchKernelGGL(tat_fwd_mfma_kernel<12>, grid, blk, 0, st, a); break;
      default: hipLaunchKernelGGL(tat_fwd_mfma_kernel<16>, grid, blk, 0, st, a); break;
    }
    DS_CHECK_LAUNCH();
    return 0;
  }
  if (T <= 16 && (size_t)kTatW * tat_wave_fwd_floats(T, dk, dv) * sizeof(float) <= 64 * 1024) {
    hipLaunchKernelGGL(tat_fwd_wave_kernel, dim3((unsigned)cdiv64(P, kTatW)), dim3(64 * kTatW),
                       (size_t)kTatW * tat_wave_fwd_floats(T, dk, dv) * sizeof(float), st, a);
    DS_CHECK_LAUNCH();
    return 0;
  }
  size_t lds = tat_fwd_lds(T, dk, dv);
  if (lds > 64 * 1024) {  // long series: column chunks, then ctx = att . V as one batched GEMM
    const size_t lc = sizeof(float) * (size_t)tat_cols_fwd_floats(T, dk);
    if (lc > 160 * 1024) { set_last_error("tat_fwd: T too large for LDS"); return DSTAGNN_E_SHAPE; }
    if (lc > 64 * 1024) DS_TRY(allow_lds((const void*)tat_fwd_cols_kernel, lc));
    const int nch = (T + kTatCW - 1) / kTatCW;
    hipLaunchKernelGGL(tat_fwd_cols_kernel, dim3((unsigned)(P * nch)), dim3(256), lc, st, a);
    DS_CHECK_LAUNCH();
    const int64_t ld = 2 * (int64_t)h * dk + (int64_t)h * dv, ldc = (int64_t)h * dv;
    Gemm g;  // ctx[bf,i,hd,:] = sum_j att[bf,hd,i,j] V[bf,j,hd,:]
    g.M = T; g.N = dv; g.K = T; g.batch = P;
    g.A = att; g.am = idx1(T); g.ak = idx1(1); g.az = idx1((int64_t)T * T);
    g.B = qkv; g.b_off = 2 * (int64_t)h * dk; g.bk = idx1(ld); g.bn = idx1(1); g.bz = idx2(h, dv, (int64_t)T * ld);
    g.C = ctx; g.cm = idx1(ldc); g.cn = idx1(1); g.cz = idx2(h, dv, (int64_t)T * ldc);
    return run_gemm(g, nullptr, 0, st);
  }
  hipLaunchKernelGGL(tat_fwd_kernel, dim3((unsigned)(B * F * h)), dim3(256), lds, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

int op_tat_bwd(int B, int F, int T, int h, int dk, int dv, const float* qkv, const float* att, const float* dctx,
               const float* dre, float* dqkv, float* dscore, float* dres_sum, hipStream_t st) {
  if (dres_sum) {  // the full dS is scratch; the output is its sum over f
    if (tat_mfma_ok(T, dk, dv, {qkv, att, dctx, dre}) && F % kTatW == 0) {
      int* cnt = stream_counters(st, B * h);
      if (cnt) {
        TatArgs a{};
        a.B = B; a.F = F; a.T = T; a.h = h; a.dk = dk; a.dv = dv;
        a.qkv = qkv; a.att = const_cast<float*>(att); a.scale = 1.f / sqrtf((float)dk);
        a.dctx = dctx; a.dre = dre; a.dqkv = dqkv; a.dscore = dscore;
        a.dres_sum = dres_sum; a.cnt = cnt; a.keep_ds = 0;
        launch_tat_bwd_mfma(a, dim3((unsigned)(B * h * (F / kTatW))), st);
        DS_CHECK_LAUNCH();
        return 0;
      }
    }
    DS_TRY(op_tat_bwd(B, F, T, h, dk, dv, qkv, att, dctx, dre, dqkv, dscore, nullptr, st));
    return op_sum_middle(dscore, B, F, (int64_t)h * T * T, dres_sum, 0.f, st);
  }
  TatArgs a{};
  a.B = B; a.F = F; a.T = T; a.h = h; a.dk = dk; a.dv = dv;
  a.qkv = qkv; a.att = const_cast<float*>(att); a.scale = 1.f / sqrtf((float)dk);
  a.dctx = dctx; a.dre = dre; a.dqkv = dqkv; a.dscore = dscore;
  a.keep_ds = 1;
  const int P = B * F * h;
  if (tat_mfma_ok(T, dk, dv, {qkv, att, dctx, dre})) {
    launch_tat_bwd_mfma(a, dim3((unsigned)cdiv64(P, kTatW)), st);
    DS_CHECK_LAUNCH();
    return 0;
  }
  if (T <= 16 && (size_t)kTatW * tat_wave_bwd_floats(T, dk, dv) * sizeof(float) <= 64 * 1024) {
    hipLaunchKernelGGL(tat_bwd_wave_kernel, dim3((unsigned)cdiv64(P, kTatW)), dim3(64 * kTatW),
                       (size_t)kTatW * tat_wave_bwd_floats(T, dk, dv) * sizeof(float), st, a);
    DS_CHECK_LAUNCH();
    return 0;
  }
  size_t lds = tat_bwd_lds(T, dk, dv);
  if (lds > 64 * 1024) {  // long series: column chunks, then dQ = s dS . K as one batched GEMM
    const size_t lc = sizeof(float) * (size_t)tat_cols_bwd_floats(T, dk, dv);
    if (lc > 160 * 1024) { set_last_error("tat_bwd: T too large for LDS"); return DSTAGNN_E_SHAPE; }
    if (lc > 64 * 1024) DS_TRY(allow_lds((const void*)tat_bwd_cols_kernel, lc));
    const int nch = (T + kTatCW - 1) / kTatCW;
    hipLaunchKernelGGL(tat_bwd_cols_kernel, dim3((unsigned)(P * nch)), dim3(256), lc, st, a);
    DS_CHECK_LAUNCH();
    const int64_t ld = 2 * (int64_t)h * dk + (int64_t)h * dv;
    Gemm g;  // dQ[bf,i,hd,:] = s sum_j dS[bf,hd,i,j] K[bf,j,hd,:]
    g.M = T; g.N = dk; g.K = T; g.batch = P;
    g.A = dscore; g.am = idx1(T); g.ak = idx1(1); g.az = idx1((int64_t)T * T);
    g.B = qkv; g.b_off = (int64_t)h * dk; g.bk = idx1(ld); g.bn = idx1(1); g.bz = idx2(h, dk, (int64_t)T * ld);
    g.C = dqkv; g.cm = idx1(ld); g.cn = idx1(1); g.cz = idx2(h, dk, (int64_t)T * ld);
    g.alpha = a.scale;
    return run_gemm(g, nullptr, 0, st);
  }
  hipLaunchKernelGGL(tat_bwd_kernel, dim3((unsigned)(B * F * h)), dim3(256), lds, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

template <int VPT>
static void launch_ln_fwd(const LnFwd& a, dim3 grid, hipStream_t st) {
  if (a.nsrc == 1) hipLaunchKernelGGL((ln_fwd_kernel<VPT, 1>), grid, dim3(256), 0, st, a);
  else if (a.nsrc == 2) hipLaunchKernelGGL((ln_fwd_kernel<VPT, 2>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((ln_fwd_kernel<VPT, 3>), grid, dim3(256), 0, st, a);
}

// DSTAGNN_LN_WG=0: long rows keep the wave-per-row kernels (A/B)
static bool ln_wg_rows() {
  static const bool on = !getenv("DSTAGNN_LN_WG") || atoi(getenv("DSTAGNN_LN_WG")) != 0;
  return on;
}

int op_ln_fwd(const LnFwd& a, hipStream_t st) {
  if (a.nsrc < 1 || a.nsrc > 3 || a.L < 1) { set_last_error("ln_fwd: 1..3 sources, L >= 1"); return DSTAGNN_E_ARG; }
  dim3 grid((unsigned)cdiv64(a.R, 4));
  if (ln_fwd_v4_ok(a)) {  // float4 rows
#define DS_LN4(V) \
    if (a.nsrc == 1) hipLaunchKernelGGL((ln_fwd_v4_kernel<V, 1>), grid, dim3(256), 0, st, a); \
    else if (a.nsrc == 2) hipLaunchKernelGGL((ln_fwd_v4_kernel<V, 2>), grid, dim3(256), 0, st, a); \
    else hipLaunchKernelGGL((ln_fwd_v4_kernel<V, 3>), grid, dim3(256), 0, st, a);
    if (a.L == 256) { DS_LN4(1) } else if (a.L == 512) { DS_LN4(2) } else { DS_LN4(4) }
#undef DS_LN4
    DS_CHECK_LAUNCH();
    return 0;
  }
  int vpt = (int)cdiv64(a.L, 64);
  if (vpt <= 1) launch_ln_fwd<1>(a, grid, st);
  else if (vpt <= 2) launch_ln_fwd<2>(a, grid, st);
  else if (vpt <= 4) launch_ln_fwd<4>(a, grid, st);
  else if (vpt <= 8) launch_ln_fwd<8>(a, grid, st);
  else if (vpt <= 16) launch_ln_fwd<16>(a, grid, st);
  else if (ln_wg_rows() && a.L <= 4096) {  // a workgroup per row (ln_fwd_wg_kernel)
    const dim3 g((unsigned)a.R);
    const int v = (int)cdiv64(a.L, 256);
#define DS_LNW(V) \
  if (a.nsrc == 1) hipLaunchKernelGGL((ln_fwd_wg_kernel<V, 1>), g, dim3(256), 0, st, a); \
  else if (a.nsrc == 2) hipLaunchKernelGGL((ln_fwd_wg_kernel<V, 2>), g, dim3(256), 0, st, a); \
  else hipLaunchKernelGGL((ln_fwd_wg_kernel<V, 3>), g, dim3(256), 0, st, a);
    if (v <= 8) { DS_LNW(8) } else { DS_LNW(16) }
#undef DS_LNW
  }
  else if (vpt <= 64) launch_ln_fwd<64>(a, grid, st);
  else { set_last_error("ln_fwd: row too long"); return DSTAGNN_E_SHAPE; }
  DS_CHECK_LAUNCH();
  return 0;
}

int op_ln_bwd(const LnBwd& a, hipStream_t st) {
  int vpt = (int)cdiv64(a.L, 64);
  if (a.gpart || a.bpart || a.xpart) {
    if (!ln_bwd_partials_ok(a.L)) { set_last_error("ln_bwd: partial slabs need L <= 1024"); return DSTAGNN_E_SHAPE; }
    dim3 grid((unsigned)ln_bwd_part_blocks(a.R));
    if (kLnRowsPerWave == 1 && ln_bwd_v4_ok(a)) {  // float4 rows (one row per wave, as below)
      if (a.L == 256) hipLaunchKernelGGL((ln_bwd_v4_kernel<1, true>), grid, dim3(256), 0, st, a);
      else if (a.L == 512) hipLaunchKernelGGL((ln_bwd_v4_kernel<2, true>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((ln_bwd_v4_kernel<4, true>), grid, dim3(256), 0, st, a);
      DS_CHECK_LAUNCH();
      return 0;
    }
    if (vpt <= 1) hipLaunchKernelGGL((ln_bwd_kernel<1, true>), grid, dim3(256), 0, st, a);
    else if (vpt <= 2) hipLaunchKernelGGL((ln_bwd_kernel<2, true>), grid, dim3(256), 0, st, a);
    else if (vpt <= 4) hipLaunchKernelGGL((ln_bwd_kernel<4, true>), grid, dim3(256), 0, st, a);
    else if (vpt <= 8) hipLaunchKernelGGL((ln_bwd_kernel<8, true>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((ln_bwd_kernel<16, true>), grid, dim3(256), 0, st, a);
    DS_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid((unsigned)cdiv64(a.R, 4));
  if (vpt <= 1) hipLaunchKernelGGL((ln_bwd_kernel<1, false>), grid, dim3(256), 0, st, a);
  else if (vpt <= 2) hipLaunchKernelGGL((ln_bwd_kernel<2, false>), grid, dim3(256), 0, st, a);
  else if (vpt <= 4) hipLaunchKernelGGL((ln_bwd_kernel<4, false>), grid, dim3(256), 0, st, a);
  else if (vpt <= 8) hipLaunchKernelGGL((ln_bwd_kernel<8, false>), grid, dim3(256), 0, st, a);
  else if (vpt <= 16) hipLaunchKernelGGL((ln_bwd_kernel<16, false>), grid, dim3(256), 0, st, a);
  else if (ln_wg_rows() && a.L <= 4096) {
    if (a.L <= 2048) hipLaunchKernelGGL((ln_bwd_wg_kernel<8>), dim3((unsigned)a.R), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((ln_bwd_wg_kernel<16>), dim3((unsigned)a.R), dim3(256), 0, st, a);
  }
  else if (vpt <= 64) hipLaunchKernelGGL((ln_bwd_kernel<64, false>), grid, dim3(256), 0, st, a);
  else { set_last_error("ln_bwd: row too long"); return DSTAGNN_E_SHAPE; }
  DS_CHECK_LAUNCH();
  return 0;
}

// out_s[o*ostride] = beta*out_s + sum_{a<A, i<I} in_s[a][o][i],  s < nsrc <= 4
int op_colsum_multi(const float* const* ins, float* const* outs, int nsrc, int64_t A, int O, int I,
                    int64_t ostride, float beta, float* part, size_t part_floats, hipStream_t st) {
  const int E = O * I;
  if (nsrc < 1 || nsrc > 4) { set_last_error("colsum: 1..4 sources"); return DSTAGNN_E_ARG; }
  if (E > 16384) { set_last_error("colsum: O*I > 16384"); return DSTAGNN_E_SHAPE; }
  if (A <= 0 || O <= 0) return 0;
  static const int kCsBlocks = getenv("DSTAGNN_COLSUM_BLOCKS") ? atoi(getenv("DSTAGNN_COLSUM_BLOCKS")) : 256;
  static const bool two_stage = getenv("DSTAGNN_COLSUM_2STAGE") && atoi(getenv("DSTAGNN_COLSUM_2STAGE")) != 0;
  if (I <= kCsW && !two_stage) {
    Colsum2dArgs c;
    for (int q = 0; q < nsrc; ++q) { c.in[q] = ins[q]; c.out[q] = outs[q]; }
    c.nsrc = nsrc; c.A = A; c.O = O; c.I = I; c.E = E;
    if (E <= kCsW) { c.W = E; c.G = 1; c.RP = kCsW / E; }
    else { c.W = I * (kCsW / I); c.G = (int)cdiv64(E, c.W); c.RP = 1; }
    const int64_t groups = (int64_t)nsrc * c.G;
    // ~512 blocks in total, >= 16 row passes per block, <= 1024 chunks (two ticket levels of 32)
    int64_t R = std::max<int64_t>(1, std::min<int64_t>(1024, cdiv64(kCsBlocks, groups)));
    R = std::min<int64_t>(R, std::max<int64_t>(1, A / (16 * c.RP)));
    c.achunk = cdiv64(A, R);
    c.R = (int)cdiv64(A, c.achunk);
    c.R2 = (int)cdiv64(c.R, kCsL1);
    c.ostride = ostride; c.beta = beta; c.part = part;
    int* cnt = stream_counters(st, (int)(groups * (c.R2 + 1)));
    if (cnt && (size_t)groups * (c.R + c.R2) * kCsW <= part_floats) {
      c.cnt = cnt;
      hipLaunchKernelGGL(colsum2d_kernel, dim3((unsigned)c.R, (unsigned)groups), dim3(256), 0, st, c);
      DS_CHECK_LAUNCH();
      return 0;
    }
  }
  ColsumArgs a;
  for (int q = 0; q < nsrc; ++q) { a.in[q] = ins[q]; a.out[q] = outs[q]; }
  a.nsrc = nsrc; a.A = A; a.O = O; a.I = I; a.ostride = ostride; a.beta = beta; a.part = part;
  // ~4K elements per stage-1 workgroup, at most 256 partial rows (stage 2's loop over
  // the partials is latency-bound: keep it short)
  int64_t P = std::max<int64_t>(1, std::min<int64_t>(256, cdiv64(A * E, 4096)));
  P = std::min<int64_t>(P, A);
  while (P > 1 && (size_t)P * nsrc * O > part_floats) P /= 2;
  if ((size_t)P * nsrc * O > part_floats) { set_last_error("colsum: scratch too small"); return DSTAGNN_E_SPACE; }
  a.achunk = cdiv64(A, P);
  a.P = (int)cdiv64(A, a.achunk);
  hipLaunchKernelGGL(colsum_stage1, dim3((unsigned)a.P), dim3(256), (size_t)E * sizeof(float), st, a);
  DS_CHECK_LAUNCH();
  const int OT = nsrc * O;
  a.OL = 1;
  while (a.OL < OT && a.OL < 64) a.OL <<= 1;
  hipLaunchKernelGGL(colsum_stage2, dim3((unsigned)cdiv64(OT, a.OL)), dim3(1024), 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}
int op_colsum(const float* in, int64_t A, int O, int I, float* out, int64_t ostride, float beta, float* part,
              size_t part_floats, hipStream_t st) {
  return op_colsum_multi(&in, &out, 1, A, O, I, ostride, beta, part, part_floats, st);
}

int op_sum_middle(const float* in, int64_t A, int Mm, int64_t I, float* out, float beta, hipStream_t st) {
  if (A <= 0 || I <= 0) return 0;
  if (A > 65535) { set_last_error("sum_middle: A > 65535"); return DSTAGNN_E_SHAPE; }
  if (cdiv64(I, 32) > 0x7fffffff) { set_last_error("sum_middle: I too large"); return DSTAGNN_E_SHAPE; }
  if (I % 4 == 0 && reinterpret_cast<uintptr_t>(in) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0)
    hipLaunchKernelGGL(sum_middle4_kernel, dim3((unsigned)cdiv64(I / 4, 64), (unsigned)A), dim3(256), 0, st, in, A, Mm,
                       I, out, beta);
  else
    hipLaunchKernelGGL(sum_middle_kernel, dim3((unsigned)cdiv64(I, 32), (unsigned)A), dim3(256), 0, st, in, A, Mm, I,
                       out, beta);
  DS_CHECK_LAUNCH();
  return 0;
}

int op_relu_mask(const float* g, const float* y, float* out, int64_t n, hipStream_t st) {
  hipLaunchKernelGGL(relu_mask_kernel, dim3(grid1d(n)), dim3(256), 0, st, g, y, out, n);
  DS_CHECK_LAUNCH();
  return 0;
}

int op_cheb_softmax_fwd(const ChebSm& a, hipStream_t st) {
  dim3 grid((unsigned)(cdiv64(a.N, 64) * a.B * a.K));
  if (a.N >= kSmCondN) hipLaunchKernelGGL(cheb_softmax_fwd_kernel<true>, grid, dim3(64 * kSmG), 0, st, a);
  else hipLaunchKernelGGL(cheb_softmax_fwd_kernel<false>, grid, dim3(64 * kSmG), 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}
int op_cheb_softmax_bwd(const ChebSm& a, hipStream_t st) {
  dim3 grid((unsigned)(cdiv64(a.N, 64) * a.B * a.K));
  if (a.N >= kSmCondN) hipLaunchKernelGGL(cheb_softmax_bwd_kernel<true>, grid, dim3(64 * kSmG), 0, st, a);
  else hipLaunchKernelGGL(cheb_softmax_bwd_kernel<false>, grid, dim3(64 * kSmG), 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}
int op_cheb_mask_grad(const ChebSm& a, hipStream_t st) {
  dim3 grid(grid1d((int64_t)a.N * a.N, 1024), (unsigned)a.K);
  hipLaunchKernelGGL(cheb_mask_grad_kernel, grid, dim3(256), 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

int op_param_prep(const ParamPrep& a, hipStream_t st) {
  if (a.nseg <= 0) return 0;
  if (a.nseg > kPrepSegsHost) { set_last_error("param_prep: too many segments"); return DSTAGNN_E_ARG; }
  // chunks of kPrepSegs segments per launch (K >= 4 on the small-graph attention path needs
  // more: 2 K mask re-layouts + K Theta blocks beside the fixed ones)
  for (int q0 = 0; q0 < a.nseg; q0 += kPrepSegs) {
    ParamPrepK k;
    k.nseg = std::min(kPrepSegs, a.nseg - q0);
    int64_t mx = 1;
    for (int q = 0; q < k.nseg; ++q) {
      k.seg[q] = a.seg[q0 + q];
      mx = std::max<int64_t>(mx, k.seg[q].n);
    }
    hipLaunchKernelGGL(param_prep_kernel, dim3((unsigned)std::min<int64_t>(cdiv64(mx, 256), 256), (unsigned)k.nseg),
                       dim3(256), 0, st, k);
    DS_CHECK_LAUNCH();
  }
  return 0;
}
int op_pack_rows(const PackRows& a, hipStream_t st) {
  if (a.n < 1 || a.n > 8) { set_last_error("pack_rows: 1..8 matrices"); return DSTAGNN_E_ARG; }
  int64_t mx = 1;
  for (int q = 0; q < a.n; ++q) mx = std::max<int64_t>(mx, (int64_t)a.rows[q] * a.cols);
  hipLaunchKernelGGL(pack_rows_kernel, dim3((unsigned)std::min<int64_t>(cdiv64(mx, 256), 1024)), dim3(256), 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}


int op_dropout_mask(float* out, int64_t n, uint64_t seed, uint32_t which, float p, uint64_t off, hipStream_t st) {
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(grid1d(n)), dim3(256), 0, st, out, n, seed, which, p, off);
  DS_CHECK_LAUNCH();
  return 0;
}

int op_pack_theta(const PackTheta& a, hipStream_t st) {
  hipLaunchKernelGGL(pack_theta_kernel, dim3(grid1d((int64_t)a.K * a.F * a.C, 256)), dim3(256), 0, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}
