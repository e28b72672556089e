// head.hip — the model head of DSTAGNN_submodule (model/DSTAGNN_my.py:265-280):
//   final_x = cat_j(out_j, dim=-1)                      (B,N,C,nb*T)
//   h       = final_conv(final_x.permute(0,3,1,2))[..., -1].permute(0,2,1)   (B,N,O)
//   y       = final_fc(h)                                (B,N,P)
// The conv's kernel (1,C) spans the whole C axis (width 1 output), so it is a contraction
// over (t,c) of every block output: h[m,o] = b1[o] + sum_j sum_{c,t} W1[o, jT+t, 0, c]
// out_j[m,c,t] with m = (b,n).  The cat is never materialised: one GEMM per block output
// accumulates into h (k = c*T + t is the block output's contiguous order; W1 is read
// through a two-level k map).  Backward mirrors it (d out_j, dW1 slices, dW2, biases).
#include "common.hpp"
#include "ops.hpp"

namespace {

constexpr size_t kHeadWs = size_t(4) << 20;   // floats: split-K slabs
constexpr size_t kHeadPart = size_t(1) << 20; // floats: column-sum partials

int check_head(int B, int N, int C, int T, int nb, int O, int P) {
  if (B <= 0 || N <= 0 || C <= 0 || T <= 0 || nb <= 0 || nb > DSTAGNN_HEAD_MAX_BLOCKS || O <= 0 || P <= 0) {
    set_last_error("head: bad dims");
    return DSTAGNN_E_ARG;
  }
  if ((int64_t)B * N * (int64_t)std::max(O, C * T) >= (1ll << 31)) {
    set_last_error("head: B*N*max(O,C*T) must be < 2^31");
    return DSTAGNN_E_SHAPE;
  }
  return 0;
}

}  // namespace

extern "C" {

int64_t dstagnn_head_scratch_bytes(void) { return (int64_t)(kHeadWs + kHeadPart) * sizeof(float) + 512; }

int dstagnn_head_forward(int B, int N, int C, int T, int nb, int O, int P, const float* const* outs,
                         const float* w1, const float* b1, const float* w2, const float* b2, float* h, float* y,
                         void* scratch, size_t scratch_bytes, dstagnn_stream_t stream) {
  DS_TRY(check_head(B, N, C, T, nb, O, P));
  if (scratch_bytes < (size_t)dstagnn_head_scratch_bytes()) {
    set_last_error("head: scratch too small");
    return DSTAGNN_E_SPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)(((uintptr_t)scratch + 255) & ~uintptr_t(255));
  const int64_t M = (int64_t)B * N, CT = (int64_t)C * T, W1row = (int64_t)nb * T * C;
  for (int j = 0; j < nb; ++j) {
    if (!outs[j]) { set_last_error("head: null block output"); return DSTAGNN_E_ARG; }
    Gemm g;
    g.M = (int)M; g.N = O; g.K = (int)CT;
    g.A = outs[j]; g.am = idx1(CT); g.ak = idx1(1);
    // W1[o][jT + t][0][c] at k = c*T + t
    g.B = w1; g.b_off = (int64_t)j * T * C; g.bk = idx2(T, C, 1); g.bn = idx1(W1row);
    g.C = h; g.cm = idx1(O); g.cn = idx1(1);
    g.beta = j ? 1.f : 0.f;
    g.bias = j ? nullptr : b1;
    DS_TRY(run_gemm(g, ws, kHeadWs, st));
  }
  Gemm g;
  g.M = (int)M; g.N = P; g.K = O;
  g.A = h; g.am = idx1(O); g.ak = idx1(1);
  g.B = w2; g.bk = idx1(1); g.bn = idx1(O);
  g.C = y; g.cm = idx1(P); g.cn = idx1(1);
  g.bias = b2;
  return run_gemm(g, ws, kHeadWs, st);
}

int dstagnn_head_backward(int B, int N, int C, int T, int nb, int O, int P, const float* const* outs,
                          const float* w1, const float* w2, const float* h, const float* dy, float* dh,
                          float* const* douts, float* dw1, float* db1, float* dw2, float* db2, void* scratch,
                          size_t scratch_bytes, dstagnn_stream_t stream) {
  DS_TRY(check_head(B, N, C, T, nb, O, P));
  if (scratch_bytes < (size_t)dstagnn_head_scratch_bytes()) {
    set_last_error("head: scratch too small");
    return DSTAGNN_E_SPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)(((uintptr_t)scratch + 255) & ~uintptr_t(255));
  float* part = ws + kHeadWs;
  const int64_t M = (int64_t)B * N, CT = (int64_t)C * T, W1row = (int64_t)nb * T * C;
  // dh[m,o] = sum_p dy[m,p] W2[p,o]
  {
    Gemm g;
    g.M = (int)M; g.N = O; g.K = P;
    g.A = dy; g.am = idx1(P); g.ak = idx1(1);
    g.B = w2; g.bk = idx1(O); g.bn = idx1(1);
    g.C = dh; g.cm = idx1(O); g.cn = idx1(1);
    DS_TRY(run_gemm(g, ws, kHeadWs, st));
  }
  // dW2[p,o] = sum_m dy[m,p] h[m,o]
  if (dw2) {
    Gemm g;
    g.M = P; g.N = O; g.K = (int)M;
    g.A = dy; g.am = idx1(1); g.ak = idx1(P);
    g.B = h; g.bk = idx1(O); g.bn = idx1(1);
    g.C = dw2; g.cm = idx1(O); g.cn = idx1(1);
    DS_TRY(run_gemm(g, ws, kHeadWs, st));
  }
  // bias gradients: column sums of dy and dh over the M rows
  {
    const float* ins[2] = {dy, dh};
    float* outs_b[2] = {db2, db1};
    if (db2) DS_TRY(op_colsum_multi(&ins[0], &outs_b[0], 1, M, P, 1, 1, 0.f, part, kHeadPart, st));
    if (db1) DS_TRY(op_colsum_multi(&ins[1], &outs_b[1], 1, M, O, 1, 1, 0.f, part, kHeadPart, st));
  }
  for (int j = 0; j < nb; ++j) {
    // dW1[o][jT+t][0][c] = sum_m dh[m,o] out_j[m, c*T + t]
    if (dw1) {
      Gemm g;
      g.M = O; g.N = (int)CT; g.K = (int)M;
      g.A = dh; g.am = idx1(1); g.ak = idx1(O);
      g.B = outs[j]; g.bk = idx1(CT); g.bn = idx1(1);
      g.C = dw1; g.c_off = (int64_t)j * T * C; g.cm = idx1(W1row); g.cn = idx2(T, C, 1);
      DS_TRY(run_gemm(g, ws, kHeadWs, st));
    }
    // d out_j[m, c*T + t] = sum_o dh[m,o] W1[o][jT+t][0][c]
    if (douts[j]) {
      Gemm g;
      g.M = (int)M; g.N = (int)CT; g.K = O;
      g.A = dh; g.am = idx1(O); g.ak = idx1(1);
      g.B = w1; g.b_off = (int64_t)j * T * C; g.bk = idx1(W1row); g.bn = idx2(T, C, 1);
      g.C = douts[j]; g.cm = idx1(CT); g.cn = idx1(1);
      DS_TRY(run_gemm(g, ws, kHeadWs, st));
    }
  }
  return 0;
}

}  // extern "C"
