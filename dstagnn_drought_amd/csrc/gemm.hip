// gemm.hip — generic strided fp32 contraction on the CDNA4 f32 matrix cores.
//
// Every dense contraction of the DSTAGNN block (TAt / SAt projections, pre_conv,
// SAt scores, Chebyshev aggregation, GTU temporal convolutions as implicit im2col,
// and all their weight / input gradients) is one call of this kernel with a
// different set of two-level affine index maps — no permute / im2col copies in HBM.
//
// Math: v_mfma_f32_32x32x2_f32 (exact fp32 FMA chain, 64 FLOP/clk/SIMD = the fp32
// peak; gfx950 has no xf32).  A workgroup is 4 waves arranged WGM x WGN; each wave
// owns WM x WN 32x32 accumulators, so the block tile is (32*WM*WGM) x (32*WN*WGN) x 16
// (64x64, 128x128, 128x32 are instantiated; a cost model picks one).
// Operands are staged global -> LDS by LDS-DMA (global_load_lds_dwordx4 where every quad is
// contiguous and aligned, global_load_lds_dword otherwise) in a 2- or 3-stage
// pipeline (see gemm_glds_body); out-of-range rows/columns are clamped to a valid address
// (their products land only in unstored C entries), so full k-tiles issue with no
// per-element predicate.  Long reductions are split over workgroups into fp32 partial
// slabs summed by a deterministic second pass (no float atomics).
#include <cstdio>
#include <cstdlib>

#include "common.hpp"

#include "gemm_kern.hpp"

using namespace dsgemm;

namespace {


// out[zb][m][n] = epilogue( sum_s ws[zb][s][m][n] ).  A workgroup takes 256/G outputs and
// G split groups per output (G = power of two ~ splitk/8, per problem), combined by an LDS
// tree.  Grouped like the GEMM: problem p owns workgroups [start[p], start[p+1]).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmG gin) {
  __shared__ float red[256];
  uint32_t lbid, lnwg;
  const GemmK g = load_group(gin, lbid, lnwg);
  const int G = g.red_g;
  const int64_t MN = (int64_t)g.M * g.N;
  const int64_t total = (int64_t)g.batch * MN;
  const int per = 256 / G;
  const int c = threadIdx.x / G, q = threadIdx.x % G;
  const int64_t idx = (int64_t)lbid * per + c;
  float s = 0.f;
  if (idx < total) {
    const int zb = (int)(idx / MN);
    const int64_t mn = idx % MN;
    const float* p = g.ws + (int64_t)zb * g.splitk * MN + mn;
    // four independent chains so the loads of one thread overlap (fixed order: deterministic)
    float s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int sp = q;
    for (; sp + 3 * G < g.splitk; sp += 4 * G) {
      s += p[(int64_t)sp * MN];
      s1 += p[(int64_t)(sp + G) * MN];
      s2 += p[(int64_t)(sp + 2 * G) * MN];
      s3 += p[(int64_t)(sp + 3 * G) * MN];
    }
    for (; sp < g.splitk; sp += G) s += p[(int64_t)sp * MN];
    s = (s + s1) + (s2 + s3);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = G / 2; w > 0; w >>= 1) {
    if (q < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (q == 0 && idx < total) {
    const int zb = (int)(idx / MN);
    const int64_t mn = idx % MN;
    epilogue_store(g, zb, (int)(mn / g.N), (int)(mn % g.N), red[threadIdx.x]);
  }
}

struct Cfg {
  int wgm, wgn, wm, wn;
  int bm() const { return 32 * wm * wgm; }
  int bn() const { return 32 * wn * wgn; }
};
constexpr Cfg kCfgs[] = {{2, 2, 1, 1}, {2, 2, 2, 2}, {4, 1, 1, 1}};  // 64x64, 128x128, 128x32


// 16-B DMA eligibility of one operand (see gemm_glds_body): every quad of elements one lane
// moves must be 4 consecutive floats at a 16-B aligned address.  kmaj: the image is
// [rows][BK] (quads along k, which needs a unit-stride single-level k map); otherwise
// [BK][rows] (quads along rows: a unit-stride row map whose quads never straddle a level
// and a row count that is a multiple of 4).  All remaining offsets must be multiples of 4.
bool quad_ok(const Idx2& x) { return x.s0 % 4 == 0 && (!x.two || x.s1 % 4 == 0); }
bool rows_quad(const Idx2& x) { return x.s0 == 1 && (!x.two || (x.f.d % 4 == 0 && x.s1 % 4 == 0)); }
int dma_width(const float* base, const Idx2& rowmap, int rows, const Idx2& kmap, const Idx2& zmap, bool kmaj) {
  if ((reinterpret_cast<uintptr_t>(base) & 15) != 0 || !quad_ok(zmap)) return 1;
  if (kmaj) return (!kmap.two && kmap.s0 == 1 && quad_ok(rowmap)) ? 4 : 1;
  return (rows_quad(rowmap) && rows % 4 == 0 && quad_ok(kmap)) ? 4 : 1;
}

// ---------------------------------------------------------------------------------
// GEMM-family profiling (dstagnn_prof_start / _stop): a timing event pair around every
// run_gemm call (kernel + split-K fold) on the stream it is issued on, with its algorithmic
// FLOP and minimum bytes, so the benchmark reports the family's achieved rate from HIP
// events of the same run.  Off by default (one branch per call).
// ---------------------------------------------------------------------------------
struct ProfRec {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  double flops = 0, bytes = 0;
};
struct Prof {
  bool on = false;
  int n = 0, cap = 0, dropped = 0;
  ProfRec* rec = nullptr;
};
Prof g_prof;
// split-K target grid (workgroups): a GEMM whose grid is below 128 workgroups splits its K
// range to about this many (320: best of a same-box sweep over 128..1024, tools/knob_sweep.sh,
// DESIGN §5; 1 = never split: every reduction in one fixed order, so a per-sample result is
// bit-identical at any batch size); DSTAGNN_SPLITK_TARGET overrides
int g_splitk_target = getenv("DSTAGNN_SPLITK_TARGET") ? atoi(getenv("DSTAGNN_SPLITK_TARGET")) : 320;
// operand precision of every GEMM: 0 = fp32 (v_mfma_f32_32x32x2_f32, the reference's
// arithmetic), 1 = bf16 operands rounded to nearest even with fp32 accumulation
// (v_mfma_f32_32x32x16_bf16) — an opt-in variant, see gemm_set_bf16
int g_bf16 = 0;

}  // namespace

bool gemm_prof_on() { return g_prof.on; }

int gemm_set_splitk_target(int target) {
  const int prev = g_splitk_target;
  if (target > 0) g_splitk_target = target;
  return prev;
}

int gemm_set_bf16(int on) {
  const int prev = g_bf16;
  if (on >= 0) g_bf16 = on ? 1 : 0;
  return prev;
}

int gemm_prof_start(int capacity) {
  if (capacity <= 0) return DSTAGNN_E_ARG;
  if (capacity > g_prof.cap) {
    ProfRec* r = new ProfRec[capacity];
    for (int i = 0; i < g_prof.cap; ++i) r[i] = g_prof.rec[i];
    for (int i = g_prof.cap; i < capacity; ++i) {
      if (hipEventCreate(&r[i].e0) != hipSuccess || hipEventCreate(&r[i].e1) != hipSuccess) {
        set_last_error("prof: hipEventCreate failed");
        delete[] r;
        return DSTAGNN_E_ARG;
      }
    }
    delete[] g_prof.rec;
    g_prof.rec = r;
    g_prof.cap = capacity;
  }
  g_prof.n = 0;
  g_prof.dropped = 0;
  g_prof.on = true;
  return 0;
}

int gemm_prof_stop(dstagnn_prof_stats* out) {
  g_prof.on = false;
  dstagnn_prof_stats s{};
  for (int i = 0; i < g_prof.n; ++i) {
    ProfRec& r = g_prof.rec[i];
    if (hipEventSynchronize(r.e1) != hipSuccess) { set_last_error("prof: event sync failed"); return DSTAGNN_E_ARG; }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.e0, r.e1) != hipSuccess) { set_last_error("prof: elapsed failed"); return DSTAGNN_E_ARG; }
    s.launches += 1;
    s.flops += r.flops;
    s.bytes += r.bytes;
    s.ms += ms;
    s.max_ms = std::max(s.max_ms, (double)ms);
  }
  s.dropped = g_prof.dropped;
  g_prof.n = 0;
  if (out) *out = s;
  return 0;
}

namespace {

// one problem's launch plan: its kernel descriptor and the kernel configuration it needs
bool gemm_log_on() {
  static const bool on = getenv("DSTAGNN_GEMM_LOG") != nullptr;
  return on;
}

struct Plan {
  GemmK k;
  char log[220];
  int best, va, vb, ns;
  bool akc, bnc, ktwo, hot, acc2;
  bool same_kernel(const Plan& o) const {
    return best == o.best && va == o.va && vb == o.vb && ns == o.ns && akc == o.akc && bnc == o.bnc &&
           ktwo == o.ktwo && hot == o.hot && acc2 == o.acc2;
  }
};

// a split-K workgroup reducing more than this many k in one fp32 chain takes the two-level
// accumulation (gemm_kern.hpp ACC2); DSTAGNN_GEMM_ACC2_MINK overrides
int acc2_min_k() {
  static const int v = getenv("DSTAGNN_GEMM_ACC2_MINK") ? atoi(getenv("DSTAGNN_GEMM_ACC2_MINK")) : 1024;
  return v;
}

// Plan one problem (tile shape, split-K, DMA widths, stages); ws: its split-K slab space.
int plan_gemm(const Gemm& g, float* ws, size_t ws_floats, Plan* out) {
  if (!g.A || !g.B || !g.C) { set_last_error("gemm: null operand"); return DSTAGNN_E_ARG; }
  if (g.ones_out && (g.cm.two || g.beta != 0.f || g.emask || g.bias || g.relu)) {
    set_last_error("gemm: column-sum output only with a plain epilogue");
    return DSTAGNN_E_ARG;
  }
  Plan& pl = *out;
  GemmK& k = pl.k;
  k = GemmK{};
  const int Nk = g.N + (g.ones_out ? 1 : 0);  // kernel columns (the column-sum column last)
  k.M = g.M; k.N = Nk; k.K = g.K; k.batch = g.batch;
  k.nload = g.N; k.ones_out = g.ones_out; k.ones_stride = (int32_t)g.ones_stride;
  // negative strides (the flipped-kernel convolution gradient): rebase the operand
  // pointer so every per-element offset the kernel forms is >= 0 and fits uint32
  k.abias = (int32_t)-(idx_min(g.am, g.M) + idx_min(g.ak, g.K));
  k.bbias = (int32_t)-(idx_min(g.bn, g.N) + idx_min(g.bk, g.K));
  k.A = g.A + g.a_off - k.abias; k.az = make_zidx(g.az);
  k.B = g.B + g.b_off - k.bbias; k.bz = make_zidx(g.bz);
  k.C = g.C + g.c_off; k.cz = make_zidx(g.cz);
  if (!make_kidx(g.am, g.M, &k.am) || !make_kidx(g.ak, g.K, &k.ak) || !make_kidx(g.bn, g.N, &k.bn) ||
      !make_kidx(g.bk, g.K, &k.bk) || !make_kidx(g.cm, g.M, &k.cm) || !make_kidx(g.cn, g.N, &k.cn) ||
      idx_span(g.am, g.M) + idx_span(g.ak, g.K) >= (1ll << 30) - 2048 ||
      idx_span(g.bn, g.N) + idx_span(g.bk, g.K) >= (1ll << 30) - 2048 ||
      idx_span(g.cm, g.M) + idx_span(g.cn, g.N) >= (1ll << 31) ||
      (int64_t)g.M * g.ones_stride >= (1ll << 31) ||
      g.bias_stride >= (1ll << 31) || (int64_t)g.N * g.bias_stride >= (1ll << 31)) {
    set_last_error("gemm: operand offsets exceed int32 (split the batch)");
    return DSTAGNN_E_SHAPE;
  }
  k.alpha = g.alpha; k.beta = g.beta; k.bias = g.bias; k.bias_stride = (int32_t)g.bias_stride; k.relu = g.relu;
  k.emask = g.emask ? g.emask + g.c_off : nullptr;
  k.Cout = g.Cout ? g.Cout + g.c_off : nullptr;
  k.ws = ws;

  // optional overrides for tuning sweeps (tools/gemm_sweep.py)
  static const int env_cfg = getenv("DSTAGNN_GEMM_CFG") ? atoi(getenv("DSTAGNN_GEMM_CFG")) : -1;
  static const int env_split = getenv("DSTAGNN_GEMM_SPLITK") ? atoi(getenv("DSTAGNN_GEMM_SPLITK")) : 0;
  // Tile choice, from the measured sweep (tools/gemm_sweep.py, profiles/): at these
  // sizes a block's latency (setup, first-tile load, epilogue) dominates, so the small
  // 64x64 tile (most blocks, 4 resident per CU) wins unless N is skinny (<= 32: 128x32)
  // or the grid is large enough for 128x128 tiles to fill the chip several times over.
  int best = 0;
  {
    const int64_t b64 = cdiv64(g.M, 64) * cdiv64(Nk, 64) * g.batch;
    if (Nk <= 32) best = 2;
    else if (b64 >= 4096 && g.K >= 1024) best = 1;
    else best = 0;
  }
  if (env_cfg >= 0 && env_cfg < (int)(sizeof(kCfgs) / sizeof(kCfgs[0]))) best = env_cfg;
  const Cfg cfg = kCfgs[best];
  const int64_t blocks = cdiv64(g.M, cfg.bm()) * cdiv64(Nk, cfg.bn()) * g.batch;

  // split-K when the grid leaves CUs idle and the reduction is long
  int splitk = 1;
  static const int min_grid = getenv("DSTAGNN_SPLITK_MINGRID") ? atoi(getenv("DSTAGNN_SPLITK_MINGRID")) : 128;
  static const int min_k = getenv("DSTAGNN_SPLITK_MINK") ? atoi(getenv("DSTAGNN_SPLITK_MINK")) : 512;
  if (g.K > 0 && blocks < min_grid && g.K >= min_k && ws) {
    int want = (int)std::min<int64_t>(512, cdiv64(g_splitk_target, blocks));
    int maxk = g.K / 128;  // keep >= 128 k per split
    splitk = std::max(1, std::min(want, maxk));
    if (env_split > 0) splitk = std::min(env_split, std::max(1, g.K / 64));
    while (splitk > 1 && (size_t)g.batch * splitk * g.M * Nk > ws_floats) --splitk;
  }
  int kchunk = g.K;
  if (splitk > 1) {
    kchunk = (int)cdiv64(cdiv64(g.K, splitk), BKMAX) * BKMAX;
    splitk = (int)cdiv64(g.K, kchunk);
  }
  if (g.K <= 0) { splitk = 1; kchunk = 0; }
  k.splitk = splitk; k.kchunk = kchunk;
  k.tiles_m = (uint32_t)cdiv64(g.M, cfg.bm());
  k.tiles_n = (uint32_t)cdiv64(Nk, cfg.bn());
  k.n_fast = (int64_t)g.M >= (int64_t)Nk ? 1u : 0u;  // A (M x K) is the bigger operand
  k.count = (uint32_t)(blocks * splitk);
  k.red_g = 1;
  while (k.red_g < 64 && k.red_g * 8 < splitk) k.red_g *= 2;

  pl.best = best;
  // split-K launches only: their K slices are the long chains (weight gradients), and a GEMM
  // that does not split keeps one summation order under every tile configuration (a B=1 and a
  // B=32 call may pick different tiles: per-sample results stay bit-identical, test_batch_consistency)
  pl.acc2 = !g_bf16 && (best == 0 || best == 2) && splitk > 1 && kchunk > acc2_min_k();
  pl.akc = !g.ak.two && g.ak.s0 == 1;
  pl.bnc = !g.bn.two && g.bn.s0 == 1;
  pl.ktwo = g.ak.two || g.bk.two;
  pl.hot = g.hot != 0;
  // DSTAGNN_GEMM_DMA16: bit 0 allows the 16-B DMA for A, bit 1 for B (default both)
  static const int env_v = getenv("DSTAGNN_GEMM_DMA16") ? atoi(getenv("DSTAGNN_GEMM_DMA16")) : 3;
  pl.va = (env_v & 1) ? dma_width(g.A + g.a_off, g.am, g.M, g.ak, g.az, pl.akc) : 1;
  pl.vb = (env_v & 2) ? dma_width(g.B + g.b_off, g.bn, g.N, g.bk, g.bz, !pl.bnc) : 1;
  // LDS pipeline depth: two stages, compile-time (gemm_glds_body)
  pl.ns = 2;
  k.nstage = pl.ns;
  if (gemm_log_on()) {
    // one "[gemm]" line per kernel launch (run_gemm_group joins a group's problems with " | ")
    snprintf(pl.log, sizeof(pl.log), "M=%d N=%d K=%d batch=%d cfg=%d splitk=%d akc=%d bnc=%d ktwo=%d blocks=%lld ns=%d va=%d vb=%d bf=%d ones=%d acc2=%d",
             g.M, Nk, g.K, g.batch, best, splitk, (int)pl.akc, (int)pl.bnc, (int)pl.ktwo, (long long)blocks * splitk,
             pl.ns, pl.va, pl.vb, g_bf16, g.ones_out ? 1 : 0, (int)pl.acc2);
  }
  return 0;
}

// one grouped argument: slices padded to multiples of 8 workgroups; returns the grid size
uint32_t make_group(const GemmK* const* ks, const uint32_t* counts, int n, GemmG* gg) {
  *gg = GemmG{};
  uint32_t at = 0;
  for (int p = 0; p < n; ++p) {
    gg->start[p] = at;
    gg->k[p] = *ks[p];
    at += (counts[p] + 7u) & ~7u;
  }
  for (int p = n; p < 4; ++p) gg->start[p] = at;
  return at;
}

void launch_plans(Plan* const* ps, int n, hipStream_t st) {
  const GemmK* ks[kGroupMax];
  uint32_t counts[kGroupMax];
  for (int p = 0; p < n; ++p) { ks[p] = &ps[p]->k; counts[p] = ps[p]->k.count; }
  GemmG gg;
  const uint32_t grid = make_group(ks, counts, n, &gg);
  using Unit = void (*)(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
  static const Unit units[3][3][2] = {
      {{gemm_c0_k0, gemm_c0_k1}, {gemm_c1_k0, gemm_c1_k1}, {gemm_c2_k0, gemm_c2_k1}},
      {{gemm_c0_k0_bf, gemm_c0_k1_bf}, {gemm_c1_k0_bf, gemm_c1_k1_bf}, {gemm_c2_k0_bf, gemm_c2_k1_bf}},
      {{gemm_c0_k0_a2, gemm_c0_k1_a2}, {nullptr, nullptr}, {gemm_c2_k0_a2, gemm_c2_k1_a2}}};
  const Plan& pl = *ps[0];
  const int var = pl.acc2 ? 2 : (g_bf16 ? 1 : 0);
  units[var][pl.best][pl.ktwo ? 1 : 0](gg, dim3(grid), pl.akc, pl.bnc, pl.va, pl.vb, pl.hot, st);
}

}  // namespace

// Up to kGroupMax independent problems: planned one by one (each its own slice of the
// split-K slab space), launched as ONE grouped kernel when their kernel configurations agree
// (else one launch per run of equal configurations), their split-K folds as one grouped
// reduce.  The problems must not write overlapping outputs.
int run_gemm_group(const Gemm* gs, int n, float* ws, size_t ws_floats, hipStream_t st) {
  if (n < 1 || n > 3) { set_last_error("gemm: 1..3 problems per group"); return DSTAGNN_E_ARG; }
  ProfRec* prec = nullptr;
  Plan plans[3];
  Plan* live[3];
  int nl = 0;
  size_t ws_used = 0;
  double flops = 0, bytes = 0;
  for (int i = 0; i < n; ++i) {
    const Gemm& g = gs[i];
    if (g.M <= 0 || g.N <= 0 || g.batch <= 0) continue;
    DS_TRY(plan_gemm(g, ws ? ws + ws_used : nullptr, ws_floats - ws_used, &plans[i]));
    const GemmK& k = plans[i].k;
    if (k.splitk > 1) ws_used += (size_t)k.batch * k.splitk * k.M * k.N;
    flops += 2.0 * g.M * g.N * (double)g.K * g.batch;
    bytes += 4.0 * g.batch * ((double)g.M * g.K + (double)g.K * g.N + (double)g.M * g.N * (g.beta != 0.f ? 2 : 1));
    live[nl++] = &plans[i];
  }
  if (!nl) return 0;
  if (g_prof.on) {
    if (g_prof.n < g_prof.cap) {
      prec = &g_prof.rec[g_prof.n++];
      prec->flops = flops;
      prec->bytes = bytes;
      (void)hipEventRecord(prec->e0, st);
    } else {
      ++g_prof.dropped;
    }
  }
  for (int i = 0; i < nl;) {
    int j = i + 1;
    while (j < nl && j - i < kGroupMax && live[j]->same_kernel(*live[i])) ++j;
    launch_plans(live + i, j - i, st);
    DS_CHECK_LAUNCH();
    if (gemm_log_on()) {
      fprintf(stderr, "[gemm] %s", live[i]->log);
      for (int q = i + 1; q < j; ++q) fprintf(stderr, " | %s", live[q]->log);
      fprintf(stderr, "\n");
    }
    i = j;
  }
  // split-K folds of every problem that split, as one grouped launch
  const GemmK* rk[3];
  uint32_t rc[3];
  int nr = 0;
  for (int i = 0; i < nl; ++i) {
    const GemmK& k = live[i]->k;
    if (k.splitk <= 1) continue;
    rk[nr] = &k;
    rc[nr] = (uint32_t)cdiv64((int64_t)k.batch * k.M * k.N, 256 / k.red_g);
    ++nr;
  }
  for (int i = 0; i < nr; i += kGroupMax) {
    GemmG gg;
    const uint32_t grid = make_group(rk + i, rc + i, std::min(kGroupMax, nr - i), &gg);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, st, gg);
    DS_CHECK_LAUNCH();
  }
  if (prec) (void)hipEventRecord(prec->e1, st);
  return 0;
}

// ONE product over the concatenation of the problems' K ranges:
//   C = epilogue_0( sum_p A_p B_p )
// (same M, N, batch and kernel configuration; each A_p / B_p with its own pointer and maps;
// the epilogue, C and its maps are problem 0's).  One launch, no split-K, no intermediate C
// round trips: the GTU transposed convolutions of widths 3, 5, 7 accumulating into one dX.
int run_gemm_kcat(const Gemm* gs, int n, hipStream_t st) {
  if (n < 1 || n > 3) { set_last_error("gemm: 1..3 K segments"); return DSTAGNN_E_ARG; }
  const Gemm& g0 = gs[0];
  if (g0.M <= 0 || g0.N <= 0 || g0.batch <= 0) return 0;
  Plan plans[3];
  double flops = 0, bytes = 0;
  for (int p = 0; p < n; ++p) {
    const Gemm& g = gs[p];
    if (g.M != g0.M || g.N != g0.N || g.batch != g0.batch || g.ones_out || g.hot) {
      set_last_error("gemm kcat: segments must share M, N, batch (no column sums)");
      return DSTAGNN_E_ARG;
    }
    DS_TRY(plan_gemm(g, nullptr, 0, &plans[p]));
    const Plan& q0 = plans[0];
    const bool kcat_ok = n <= kGroupMax && q0.best == 2 && !q0.ktwo && q0.akc && q0.bnc && q0.va == 4 &&
                         q0.vb == 4;  // kcat_supported
    if (!kcat_ok || (p && !plans[p].same_kernel(plans[0]))) {
      // different kernels (DMA widths / map kinds): fall back to a chain of launches
      Gemm first = g0, next;
      first.Cout = nullptr; first.emask = nullptr;
      DS_TRY(run_gemm(first, nullptr, 0, st));
      for (int q = 1; q < n; ++q) {
        next = gs[q];
        next.C = g0.C; next.cm = g0.cm; next.cn = g0.cn; next.cz = g0.cz; next.c_off = g0.c_off;
        next.beta = 1.f; next.bias = nullptr; next.relu = 0;
        next.Cout = q == n - 1 ? g0.Cout : nullptr;
        next.emask = q == n - 1 ? g0.emask : nullptr;
        DS_TRY(run_gemm(next, nullptr, 0, st));
      }
      return 0;
    }
    flops += 2.0 * g.M * g.N * (double)g.K * g.batch;
    bytes += 4.0 * g.batch * ((double)g.M * g.K + (double)g.K * g.N);
  }
  bytes += 4.0 * g0.batch * (double)g0.M * g0.N * (g0.beta != 0.f ? 2 : 1);
  ProfRec* prec = nullptr;
  if (g_prof.on) {
    if (g_prof.n < g_prof.cap) {
      prec = &g_prof.rec[g_prof.n++];
      prec->flops = flops;
      prec->bytes = bytes;
      (void)hipEventRecord(prec->e0, st);
    } else {
      ++g_prof.dropped;
    }
  }
  GemmG gg{};
  const uint32_t grid = (plans[0].k.count + 7u) & ~7u;
  gg.start[0] = (uint32_t)n;  // K-concatenated
  for (int p = 1; p < 4; ++p) gg.start[p] = grid;
  for (int p = 0; p < n; ++p) gg.k[p] = plans[p].k;
  using Unit = void (*)(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
  static const Unit units[2][3][2] = {
      {{gemm_c0_k0, gemm_c0_k1}, {gemm_c1_k0, gemm_c1_k1}, {gemm_c2_k0, gemm_c2_k1}},
      {{gemm_c0_k0_bf, gemm_c0_k1_bf}, {gemm_c1_k0_bf, gemm_c1_k1_bf}, {gemm_c2_k0_bf, gemm_c2_k1_bf}}};
  const Plan& pl = plans[0];
  units[g_bf16 ? 1 : 0][pl.best][pl.ktwo ? 1 : 0](gg, dim3(grid), pl.akc, pl.bnc, pl.va, pl.vb, false, st);
  DS_CHECK_LAUNCH();
  if (gemm_log_on()) {
    fprintf(stderr, "[gemm] kcat %s", plans[0].log);
    for (int q = 1; q < n; ++q) fprintf(stderr, " + %s", plans[q].log);
    fprintf(stderr, "\n");
  }
  if (prec) (void)hipEventRecord(prec->e1, st);
  return 0;
}

int run_gemm(const Gemm& g, float* ws, size_t ws_floats, hipStream_t st) { return run_gemm_group(&g, 1, ws, ws_floats, st); }

