// ops.hpp — argument structs and launchers of the non-GEMM kernels (ops.hip).
#pragma once
#include "common.hpp"

struct LnSrc {
  const float* p = nullptr;
  Idx2 row;          // row r -> base offset
  int64_t es = 1;    // element stride
};

struct LnFwd {
  int R = 0, L = 0;
  LnSrc src[3];
  int nsrc = 0;
  const float* g = nullptr;
  const float* b = nullptr;
  float eps = 1e-5f;
  float* y = nullptr; Idx2 yrow; int64_t yes = 1;
  float* u = nullptr;           // optional (R, L) copy of the LN input sum
  float* mu = nullptr; float* rs = nullptr;
  float drop_p = 0.f; uint64_t seed = 0; uint32_t which = 0;  // dropout on the output
  uint64_t drop_off = 0;  // added to the mask index (row * L + e): the shard's first global sample
};

struct LnBwd {
  int R = 0, L = 0;
  const float* dy = nullptr; Idx2 dyrow; int64_t dyes = 1;
  const float* u = nullptr; const float* mu = nullptr; const float* rs = nullptr; const float* g = nullptr;
  float drop_p = 0.f; uint64_t seed = 0; uint32_t which = 0;  // mask applied to dy
  uint64_t drop_off = 0;  // as LnFwd::drop_off
  float* dx = nullptr; Idx2 dxrow; int64_t dxes = 1; float beta = 0.f;
  float* gcontrib = nullptr;    // optional (R, L): dy' * xhat  (gamma grad contributions)
  float* bcontrib = nullptr;    // optional (R, L): dy'         (beta grad contributions)
  // or (instead of the contribution tensors) per-workgroup partial sums over its rows:
  // (ln_bwd_part_blocks(R), L) slabs, L <= 1024 (ln_bwd_partials_ok)
  float* gpart = nullptr;
  float* bpart = nullptr;
  // optional with the slabs: per-workgroup sums of the written dx rows (a following linear
  // layer's bias gradient: the column sum of dx, with no re-read of dx)
  float* xpart = nullptr;
};
constexpr int kLnRowsPerWave = 1;  // rows per wave of the partial-slab LN backward (measured: 4 is slower)
inline int64_t ln_bwd_part_blocks(int64_t R) { return (R + 4 * kLnRowsPerWave - 1) / (4 * kLnRowsPerWave); }
inline bool ln_bwd_partials_ok(int L) { return L <= 1024; }

struct ChebSm {
  int B = 0, K = 0, N = 0;
  const float* S = nullptr;       // (B,K,N,N) scores
  const float* apa = nullptr;     // (N,N)
  const float* mask[DSTAGNN_MAX_K] = {};
  const float* cheb = nullptr;    // (K,N,N)
  float* P = nullptr;             // (B,K,N,N)
  float* W = nullptr;             // (B,K,N,N)
  // bwd
  const float* dW = nullptr;
  float* dz = nullptr;
  float* dmask[DSTAGNN_MAX_K] = {};
};

struct ColsumArgs {
  const float* in[4] = {};
  float* out[4] = {};
  int nsrc = 1;
  int64_t A = 0; int O = 0, I = 1;
  int64_t achunk = 1;
  int64_t ostride = 1; float beta = 0.f;
  float* part = nullptr; int P = 1; int OL = 1;
};

// Stack up to 8 row-major matrices (rows_i x cols) into one (sum rows_i) x cols matrix
// (unpack = 1: the inverse, null destinations skipped) — fuses same-input projections.
struct PackRows {
  int n = 0, cols = 0, unpack = 0;
  int rows[8] = {};
  const float* src[8] = {};   // pack sources / unpack: src[0] = packed
  float* dst[8] = {};         // pack: dst[0] = packed / unpack destinations
};

// Every per-forward parameter re-layout of the block in ONE launch: a list of segments,
// each a copy with one of a few index maps (element i of the destination):
//   0 copy           dst[i] = src[i]                                   (stacked projections)
//   1 pre_conv       Wp[d][f][t] = W[d][t][0][f]        p0 = F, p1 = T
//   2 theta          thcat[f][k*C + c] = theta_k[f][c]  p0 = C, p1 = K*C, p2 = k
//   3 gtu fwd        perm[o][j][c] = w[o][c][j]         p0 = C, p1 = ks
//   4 gtu bwd        perm[j'][o][c] = w[o][c][ks-1-j']  p0 = C, p1 = ks
//   5 product        dst[i] = src[i] * src2[i]                          (A_pa o M_k)
//   6 product^T      dst[(i % p0) * p0 + i / p0] = src[i] * src2[i]     (its transpose, N = p0)
struct PrepSeg {
  int kind = 0, p0 = 0, p1 = 0, p2 = 0, p3 = 0;
  int64_t n = 0;        // source elements (kind 8: destination elements)
  int64_t dst_off = 0;  // kind 0: element offset into dst
  const float* src = nullptr;
  const float* src2 = nullptr;  // kind 5
  float* dst = nullptr;
};
constexpr int kPrepSegs = 32;      // segments per launch (the kernel argument)
constexpr int kPrepSegsHost = 96;  // segments per call (op_param_prep launches them in chunks)
struct ParamPrepK {
  int nseg = 0;
  PrepSeg seg[kPrepSegs];
};
struct ParamPrep {
  int nseg = 0;
  PrepSeg seg[kPrepSegsHost];
};

// fused per-node GTU gates + fcmy + dropout + residual + LayerNorm (gtu_tail.hip)
struct GtuTailArgs {
  int64_t BN = 0; int C = 0, T = 0; int first = 0;
  const float* conv[3] = {};      // GTU conv outputs [bn][T-ks+1][2C] (bias included)
  const float* fcmy_w = nullptr;  // (T, 3T-12)
  const float* fcmy_b = nullptr;  // (T)
  const float* X = nullptr;       // cheb output (B,N,T,C)
  const float* x = nullptr;       // block input (B,N,F,T)
  const float* res_w = nullptr; const float* res_b = nullptr;
  const float* ln_g = nullptr; const float* ln_b = nullptr;
  float drop_p = 0.f; uint64_t seed = 0;
  uint64_t drop_off = 0;  // added to the mask index (bn * C * T + e): the shard's first global sample
  // fwd outputs
  float* G = nullptr;             // [bn][C][3T-12] (saved for the fcmy weight gradient)
  float* tco = nullptr; float* r = nullptr; float* mu = nullptr; float* rs = nullptr; float* out = nullptr;
  // bwd
  const float* dout = nullptr;
  float* gcontrib = nullptr;      // dout * xhat (LN gamma grad contributions)
  float* dtc = nullptr;           // d fcmy output (B,N,C,T)
  float* dX = nullptr;            // residual part of d cheb output (B,N,T,C)
  float* dx = nullptr;            // d block input
  float* rcontrib = nullptr; float* dres = nullptr;  // first block residual_conv grads
  // per-node partial sums over t instead of the contribution tensors above ([bn][C] each;
  // gpart: sum dout*xhat, bpart: sum dout; first block rpart: sum dr*x, dpart: sum dr)
  float* gpart = nullptr; float* bpart = nullptr; float* rpart = nullptr; float* dpart = nullptr;
  float* dconv_pad[3] = {};       // rows [bn*T + t'][2C]: ks-1 zero rows + T-ks+1 gate rows per node, ks-1 zero rows after the last
  float* dG = nullptr;            // [bn][C][3T-12] scratch of the split (long-series) backward
  // in-kernel column sums of the four partial arrays above (compile-time C / T backward, one node
  // per workgroup; gtu_tail_bwd_folds): fold_out[q] = sum over bn of {gpart, bpart, rpart, dpart}
  // (null: skipped) by a two-level ticket tree, level-2 rows in fold_ws (4 x ceil(BN / 64) x C)
  int fold = 0; float* fold_out[4] = {}; float* fold_ws = nullptr;
  int* fold_cnt = nullptr;        // (set by the launcher)
};
bool gtu_tail_bwd_folds(const GtuTailArgs& a);  // the launcher will fold (a.fold honoured)



struct PackTheta {
  int K = 0, F = 0, C = 0, unpack = 0;
  const float* src[DSTAGNN_MAX_K] = {};   // pack: K x (F,C)
  float* cat_out = nullptr;               // pack: (F, K*C)
  const float* cat_in = nullptr;          // unpack: (F, K*C)
  float* dst[DSTAGNN_MAX_K] = {};         // unpack: K x (F,C) (null entries skipped)
};

// sparse Chebyshev aggregation over the union support of T_0..T_{K-1} (cheb_sparse.hip)
struct ChebSp {
  int B = 0, N = 0, K = 0, CT = 0, C = 0;   // element e of a C*T row = (t, c), e = t*C + c
  const int* csc_ptr = nullptr; const int* csc_row = nullptr;  // column j -> source rows i
  const int* csr_ptr = nullptr; const int* csr_col = nullptr;  // row i -> destination columns j
  const float* cheb = nullptr;   // (K,N,N)
  const float* P = nullptr;      // (B,K,N,N) column softmax
  const float* xth = nullptr;    // (B,N,T,K,C)
  float* out = nullptr;          // (B,N,T,C)  fwd (ReLU applied)
  const float* g = nullptr;      // (B,N,T,C)  bwd: d(pre-ReLU out)
  float* dW = nullptr;           // (B,K,N,N) bwd: written on the support only
  float* dxth = nullptr;         // (B,N,T,K,C) bwd
  // fused (flash) path: W = T o P and dW kept compact on the support, (B,K,nnz) in CSC order
  int nnz = 0;
  const float* wsupp = nullptr;  // fwd / spmm_t: replaces T_k[i,j] P[b,k,i,j]
  float* dws = nullptr;          // sddmm: written instead of dW
  // sddmm with the softmax-backward column terms fused (flash path): with dzs set, instead
  // of dW it writes dzs = P o T o dW on the support and cc[b,k,j] = sum_i dzs_ij
  const float* psupp = nullptr;  // (B,K,nnz) P on the support
  const float* tsupp = nullptr;  // (K,nnz) T_k on the support
  float* dzs = nullptr;          // (B,K,nnz)
  float* cc = nullptr;           // (B,K,N)
  const int* csc2csr = nullptr;  // with dzs_r: dzs also stored in CSR order (small-graph flash)
  float* dzs_r = nullptr;        // (B,K,nnz)
  const int* csr2csc = nullptr;  // CSR position -> CSC position
  int xcd_order = 0;             // set by the launcher: XCD-aware row-block order (cheb_sparse.hip)
};
bool cheb_sparse_ok(int CT);

// the block's sparse Chebyshev convolution in aggregate-first order (cheb_agg.hip): the
// support gather runs on x (F*T per node) and the Theta products on each wave's matrix cores
struct ChebAg {
  int B = 0, N = 0, K = 0, F = 0, C = 0, T = 0, KC = 0, nnz = 0;
  const float* x = nullptr;        // (B,N,F,T)
  const float* thcat = nullptr;    // (F, K*C)
  const int *csc_ptr = nullptr, *csc_row = nullptr, *csr_ptr = nullptr, *csr_col = nullptr, *csr2csc = nullptr;
  const float* cheb = nullptr;     // (K,N,N)   } unfused path: W = T o P
  const float* P = nullptr;        // (B,K,N,N) }
  const float* wsupp = nullptr;    // (B,K,nnz) flash path: W on the support (CSC order)
  float* agg = nullptr;            // (B,N,K,F,T) fwd output, saved for dTheta
  float* X = nullptr;              // (B,N,T,C) fwd output (ReLU applied)
  const float* g = nullptr;        // (B,N,T,C) bwd: d(pre-ReLU X)
  float* dW = nullptr;             // (B,K,N,N) sddmm, unfused path (support entries only)
  const float* psupp = nullptr; const float* tsupp = nullptr;  // flash path: the softmax backward's
  float* dzs = nullptr; float* dzs_r = nullptr; const int* csc2csr = nullptr; float* cc = nullptr;  // support terms
  float* dx = nullptr; float dx_beta = 1.f;  // spmm_t: dx = dx_beta dx + (the Chebyshev path's gradient)
  int xcd_order = 0;
  uint32_t* sig = nullptr; uint32_t sig_v = 0;  // kernel-written stream signal (SDDMM; common.hpp)
};
bool cheb_agg_ok(int F, int C, int K, int T);
int op_cheb_agg_fwd(const ChebAg& a, hipStream_t st);
int op_cheb_agg_sddmm(const ChebAg& a, hipStream_t st);
int op_cheb_agg_spmm_t(const ChebAg& a, hipStream_t st);

// fused (flash-style) Chebyshev attention (cheb_flash.hip); dk == 32
struct ChebFl {
  int B = 0, N = 0, K = 0, nnz = 0, nw = 0;  // nw = 32-bit words per A_pa bit row
  float scale = 1.f;                       // 1/sqrt(dk)
  const float* qk = nullptr; int64_t ld = 0; int kd = 0;  // (B*N, ld) rows [Q'_0..Q'_{K-1} | K'_0..]
  const float* apa = nullptr;              // (N,N)
  const float* mask[DSTAGNN_MAX_K] = {};   // (N,N) each
  const int32_t* bits = nullptr;           // (N, nw): bit j of row i = A_pa[i,j] != 0
  const int32_t* bits_t = nullptr;         // (N, nw): bit i of row j
  const int *csc_ptr = nullptr, *csc_row = nullptr, *csr_ptr = nullptr, *csr_col = nullptr, *csr2csc = nullptr;
  const int *apa_ptr = nullptr, *apa_row = nullptr;  // CSC of the A_pa support
  const float* tsupp = nullptr;            // (K, nnz) T_k on the union support, CSC order
  float* lse = nullptr;                    // (B,K,N) column log-sum-exp
  float* psupp = nullptr; float* wsupp = nullptr;  // (B,K,nnz)
  const float* dws = nullptr; float* dzs = nullptr; float* cc = nullptr;  // (B,K,nnz) x2, (B,K,N)
  float* dqk = nullptr;                    // (B*N, ld) dQ' | dK'
  float* dmask[DSTAGNN_MAX_K] = {};        // (N,N) each, fully written
  // small graphs (flash_small(N)): the dense A_pa o M_k, P on the A_pa support, the index maps
  const float* am = nullptr;               // (K,N,N) A_pa o M_k (param_prep, every forward)
  const float* amt = nullptr;              // (K,N,N) its transpose (the dQ' kernel's row strips)
  float* papa = nullptr; int apa_nnz = 0;  // (B,K,apa_nnz) P on the A_pa support (A_pa CSC order)
  const int* apa_idx = nullptr;            // (N,N) A_pa-CSC index or -1
  const int* apa2t = nullptr;              // (apa_nnz) union-support CSC position or -1
  float* dzs_r = nullptr;                  // (B,K,nnz) dzs in CSR order (the SDDMM writes it)
  uint32_t* sig = nullptr; uint32_t sig_v = 0;  // kernel-written stream signal (common.hpp)
};
bool flash_small(int N);  // the LDS-staged small-graph kernels (N <= 512)
int op_flash_forward(const ChebFl& a, hipStream_t st);   // lse, psupp, wsupp
int op_flash_colc(const ChebFl& a, hipStream_t st);      // cc, dzs
int op_flash_dqk(const ChebFl& a, hipStream_t st);       // dqk
int op_flash_mask_grad(const ChebFl& a, hipStream_t st); // dmask
int op_cheb_spmm_fwd(const ChebSp& a, hipStream_t st);
int op_cheb_sddmm_bwd(const ChebSp& a, hipStream_t st);
int op_cheb_spmm_t_bwd(const ChebSp& a, hipStream_t st);

int op_pack_theta(const PackTheta& a, hipStream_t st);
int op_transpose(const float* in, float* out, int R, int Cc, int batch, int64_t in_bs, int64_t out_bs, float beta,
                 hipStream_t st);
// the GTU convolutions' input gradient as one sliding-window kernel (gtu_tconv.hip)
struct TconvArgs {
  const float* dconv[3];  // zero-padded gate-gradient rows (M + ks - 1, 2C) per GTU
  const float* wflip[3];  // flipped weights (ks, 2C, C) per GTU
  int ks[3];
  const float* dX;        // (M, C) the tail's gradient of the GTU block input (beta input)
  const float* X;         // (M, C) the Chebyshev output (ReLU mask)
  float* gpre;            // (M, C) result
  int64_t M;              // rows B*N*T
  uint32_t* sig = nullptr; uint32_t sig_v = 0;  // kernel-written stream signal (common.hpp)
};
bool gtu_tconv_ok(int C, const int* ks, int n);
// the three GTU convolutions (forward) by the same sliding window (gtu_tconv.hip)
struct GconvArgs {
  const float* X;        // (BN, T, C) Chebyshev output
  const float* wf[3];    // (ks, C, 2C) re-laid weights (j, c, o)
  const float* bias[3];  // (2C) or null
  float* conv[3];        // (BN * Tg, 2C)
  int ks[3];
  int Tg[3];             // set by the launcher
  int start[4];          // first workgroup of each GTU (set by the launcher)
  int64_t BN;
  int T;
};
bool gtu_conv_fwd_ok(int C, int T, const int* ks, int n);
int op_gtu_conv_fwd(GconvArgs a, hipStream_t st);
int op_gtu_tconv(const TconvArgs& a, hipStream_t st);
// the temporal-attention stage as one kernel (tat_fused.hip): Q|K|V projection, attention, fc,
// residual and the LayerNorm over N; E(R, n) = src[(R % FT) s0 + (R / FT) s1 + n sN]
struct TatFusedArgs {
  const float* src = nullptr; int64_t s0 = 0, s1 = 0, sN = 0;
  const float* wqkv = nullptr;  // (3 h dk, NP) zero-padded re-layout of [Wq; Wk; Wv]
  const float* wfc = nullptr;   // (N, h dv) TAt.fc.weight
  const float* res = nullptr; int res_mode = 0;
  const float* g = nullptr; const float* bta = nullptr;  // LayerNorm(N) gamma / beta
  float *qkv = nullptr, *re_at = nullptr, *att = nullptr, *ctx = nullptr;
  float *u = nullptr, *mu = nullptr, *rs = nullptr, *O = nullptr;  // O[(R % FT) BN + (R / FT) N + n]
  int64_t FT = 0, BFT = 0, BN = 0;
  int F = 0, T = 0, N = 0, NP = 0, h = 0;
  float scale = 1.f, eps = 1e-5f;
  uint32_t* sig = nullptr; uint32_t sig_v = 0;  // kernel-written stream signal (common.hpp)
};
bool tat_fused_fwd_ok(int N, int T, int h, int dk, int dv);
int tat_fused_np(int N);  // the padded node count of the re-laid Q|K|V weights
int64_t tat_fused_bwd_wgs(int64_t BFT);        // the fused backward's workgroups (partial rows)
int64_t tat_fused_bwd_part_rows(int64_t BFT);  // ... + its level-2 ticket-tree rows: one slab's rows
int op_tat_fused_fwd(const TatFusedArgs& a, hipStream_t st);
struct TatFusedBwdArgs {
  const float* dO = nullptr;  // O's [(f,t)][(b,n)] order
  const float *u = nullptr, *mu = nullptr, *rs = nullptr, *g = nullptr;
  float *gpart = nullptr, *bpart = nullptr;  // (ceil(BFT / 48), N) gamma / beta partial rows (+ level-2 rows)
  int ln_fold = 0; float *gout = nullptr, *bout = nullptr;  // ln_fold: the column sums in-kernel -> gout / bout
  float* dU = nullptr;                       // (BFT, N)
  const float* wfcT = nullptr;               // (h dv, NP) zero-padded transpose of TAt.fc.weight
  const float *qkv = nullptr, *att = nullptr, *dre = nullptr;
  float* dqkv = nullptr;                     // (BFT, 3 h dk)
  int res_mode = 0;
  float* dres = nullptr;                     // FULL: (B,F,h,T,T); BCAST: (B,h,T,T)
  float* dpart = nullptr; int* cnt = nullptr;  // BCAST: (B, FT/48, h, T, T) partials, per-b tickets
  const float* wqT = nullptr;                // (NP, 3 h dk) zero-padded transpose of [Wq; Wk; Wv]
  float* dx = nullptr; int64_t dxb = 0;      // inner block: dx[b dxb + n FT + ft] += dE
  float* dE = nullptr;                       // first block: (BFT, N)
  int64_t FT = 0, BFT = 0, BN = 0;
  int F = 0, T = 0, N = 0, NP = 0, h = 0;
  int B = 0;  // (set by the launcher)
  float scale = 1.f;
  uint32_t* sig = nullptr; uint32_t sig_v = 0;
  FastDiv fdN, fdH2, fdFT;  // (set by the launcher) magic divisions by N, N / 2, FT
};
bool tat_fused_bwd_ok(int N, int T, int h, int dk, int dv, int F, int res_mode);
int op_tat_fused_bwd(const TatFusedBwdArgs& a, hipStream_t st);
// the GTU stage forward as one kernel (gtu_fused.hip): the three convolutions, gates, fcmy,
// dropout, residual, ReLUs, LN over C; C = 32, T = 12
struct GtuFusedArgs {
  int64_t BN = 0; int C = 0, T = 0; int first = 0;
  const float* X = nullptr;        // (BN, T, C) Chebyshev output
  const float* x = nullptr;        // block input (B,N,F,T)
  const float* wt[3] = {};         // GTU weights re-laid (2C, k, C) (param_prep kind 3)
  const float* bias[3] = {};       // (2C)
  const float* fcmy_w = nullptr; const float* fcmy_b = nullptr;
  const float* res_w = nullptr; const float* res_b = nullptr;
  const float* ln_g = nullptr; const float* ln_b = nullptr;
  float drop_p = 0.f; uint64_t seed = 0; uint64_t drop_off = 0;
  float* conv[3] = {};             // (BN (T - k + 1), 2C), bias included (saved)
  float *G = nullptr, *tco = nullptr, *r = nullptr, *mu = nullptr, *rs = nullptr, *out = nullptr;
};
struct SatLnBwdArgs {  // sat_fused.hip: dZd = dqk [W_Q'; W_K'] + EmbedS LayerNorm(D) backward
  int64_t R = 0, D = 0, K2 = 0;    // rows B N, d_model, 2 K d_k
  const float* dqk = nullptr;      // (R, K2)
  const float* wT = nullptr;       // (D, K2) = [W_Q'; W_K']^T (param_prep kind 9)
  const float *u = nullptr, *mu = nullptr, *rs = nullptr, *g = nullptr;
  float drop_p = 0.f; uint64_t seed = 0; uint64_t drop_off = 0;  // the EmbedS dropout (which = 0)
  float* dx = nullptr;             // dY (R, D)
  float *gpart = nullptr, *bpart = nullptr, *xpart = nullptr;  // [workgroup][D] partial rows (xpart optional)
};
bool sat_ln_bwd_fused_ok(int64_t D, int64_t K2);
int64_t sat_ln_bwd_fused_wgs(int64_t R);
int op_sat_ln_bwd_fused(const SatLnBwdArgs& a, hipStream_t st);
bool gtu_fused_fwd_ok(int C, int T);
int op_gtu_fused_fwd(const GtuFusedArgs& a, hipStream_t st);
struct GtuFusedBwdArgs {
  int64_t BN = 0; int C = 0, T = 0; int first = 0;
  const float *dout = nullptr, *r = nullptr, *tco = nullptr, *mu = nullptr, *rs = nullptr;
  const float* x = nullptr;        // first block: the block input (BN, T)
  const float* X = nullptr;        // (BN, T, C) Chebyshev output (the ReLU mask of gpre)
  const float* conv[3] = {};       // (BN Tg, 2C) saved by the forward
  const float* wf[3] = {};         // GTU weights re-laid (j, c, o) (param_prep kind 7)
  const float *fcmy_w = nullptr, *ln_g = nullptr, *res_w = nullptr;
  float drop_p = 0.f; uint64_t seed = 0; uint64_t drop_off = 0;
  float *dx = nullptr, *gpre = nullptr;
  float* dconv[3] = {};            // (BN Tg, 2C) compact gate gradients (the weight gradients' operand)
  // the parameter gradients reduced in-kernel (two-level ticket tree over per-workgroup rows of
  // gtu_fused_bwd_row() floats in part, level-2 rows after them; null outputs skipped):
  // LayerNorm gamma / beta, residual_conv weight / bias (first block), fcmy weight / bias
  float *gout = nullptr, *bout = nullptr, *rwout = nullptr, *rbout = nullptr, *fwout = nullptr, *fbout = nullptr;
  float* part = nullptr;           // gtu_fused_bwd_part_floats(BN) floats
  int* cnt = nullptr;              // (set by op_gtu_fused_bwd: the stream's ticket counters)
};
bool gtu_fused_bwd_ok(int C, int T);
int64_t gtu_fused_bwd_part_floats(int64_t BN);
int op_gtu_fused_bwd(const GtuFusedBwdArgs& a, hipStream_t st);
int op_tat_fwd(int B, int F, int T, int h, int dk, int dv, const float* qkv, const float* res, int res_mode,
               float* re_at, float* att, float* ctx, hipStream_t st);
int op_tat_bwd(int B, int F, int T, int h, int dk, int dv, const float* qkv, const float* att, const float* dctx,
               const float* dre, float* dqkv, float* dscore, float* dres_sum, hipStream_t st);
int op_ln_fwd(const LnFwd& a, hipStream_t st);
int op_ln_bwd(const LnBwd& a, hipStream_t st);
// zero-armed int tickets private to (current device, stream); nullptr if unavailable
int* stream_counters(hipStream_t st, int n);
int op_colsum(const float* in, int64_t A, int O, int I, float* out, int64_t ostride, float beta, float* part,
              size_t part_floats, hipStream_t st);
int op_colsum_multi(const float* const* ins, float* const* outs, int nsrc, int64_t A, int O, int I,
                    int64_t ostride, float beta, float* part, size_t part_floats, hipStream_t st);
int op_sum_middle(const float* in, int64_t A, int Mm, int64_t I, float* out, float beta, hipStream_t st);
int op_relu_mask(const float* g, const float* y, float* out, int64_t n, hipStream_t st);
int op_cheb_softmax_fwd(const ChebSm& a, hipStream_t st);
int op_cheb_softmax_bwd(const ChebSm& a, hipStream_t st);
int op_cheb_mask_grad(const ChebSm& a, hipStream_t st);
int op_pack_rows(const PackRows& a, hipStream_t st);
int op_gtu_tail_fwd(const GtuTailArgs& a, hipStream_t st);
int op_gtu_tail_bwd(const GtuTailArgs& a, hipStream_t st);
// true when the backward runs split (LN | dG GEMM | gates) and needs GtuTailArgs::dG
bool gtu_tail_bwd_split(int C, int T);
int op_param_prep(const ParamPrep& a, hipStream_t st);
int op_dropout_mask(float* out, int64_t n, uint64_t seed, uint32_t which, float p, uint64_t off, hipStream_t st);
