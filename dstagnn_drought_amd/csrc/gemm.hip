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
#include <cstring>

#include "common.hpp"
#include "ops.hpp"

#include "gemm_kern.hpp"

using namespace dsgemm;

namespace {


// out[zb][m][n] = epilogue( sum_s ws[zb][s][m][n] ).  A workgroup takes 256/G outputs and
// G split groups per output (G = power of two ~ splitk/8, per problem), combined by an LDS
// tree.  Consecutive threads take consecutive outputs of one split group (thread = q per + c),
// so one load instruction of a wave touches 64 / per slab rows (per contiguous floats each)
// instead of G slab rows of 64 / G floats.  Same sums in the same order.  Grouped like the GEMM: problem p owns workgroups [start[p], start[p+1]).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmG gin) {
  __shared__ float red[256];
  uint32_t lbid, lnwg;
  const GemmK g = load_group(gin, lbid, lnwg);
  const int G = g.red_g;
  const int64_t MN = (int64_t)g.M * g.N;
  const int64_t total = (int64_t)g.batch * MN;
  const int per = 256 / G;
  const int c = threadIdx.x % per, q = threadIdx.x / per;
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
  red[threadIdx.x] = s;  // = red[q per + c]
  __syncthreads();
  for (int w = G / 2; w > 0; w >>= 1) {
    if (q < w) red[threadIdx.x] += red[threadIdx.x + w * per];
    __syncthreads();
  }
  if (q == 0 && idx < total) {
    const int zb = (int)(idx / MN);
    const int64_t mn = idx % MN;
    epilogue_store(g, zb, (int)(mn / g.N), (int)(mn % g.N), red[threadIdx.x]);
  }
}

// ---------------------------------------------------------------------------------
// Skinny long reductions: M <= 96 and the kernel's N (with the column-sum column) <= 32,
// batch 1, K >= kSkinnyMinK — the fcmy weight gradient (12 x 25 over B*N*C = 174K rows at
// PEMS08) and the aggregate-first Chebyshev weight gradient dTheta (K*F x C = 96 x 32 over
// B*N*T = 65K rows).  The tiled kernel leaves most of its tile clamped (or splits K into
// hundreds of slabs and a fold launch) and spends its time in per-k-tile DMA round trips.
// Here every wave owns kpw consecutive k and loads a round of U k-quads at once
// (v_mfma_f32_16x16x4_f32, lane (q = l>>4, i = l&15): A[mt*16 + i][k + q] and
// B[k + q][nt*16 + i]), then MT x NT MFMAs per quad into 16x16 accumulators.  One
// 1024-thread workgroup per CU (<= 256 of them): its 16 accumulators fold in LDS in a fixed
// order, and the workgroups' partials fold by tickets (colsum2d's hand-off: sc1 stores drained
// by every storing wave, a barrier, one agent-scope ticket per workgroup; the last arrival
// acquires, then all its 1024 threads sum the partials in a fixed order).  Small outputs
// (fcmy: 300 floats) fold in ONE level — the acquire's price grows with the workgroups per CU
// (MI355X_MICROARCH.md), so one per CU pays it once; large ones (dTheta: 3 072 floats x 256
// partials = 3 MB would take one CU ~20 us to read) fold in two: the last of each group of
// kSkGroup workgroups sums its group's partials, the last group sums the group sums.  Either
// way the summation order is fixed: deterministic.
// ---------------------------------------------------------------------------------
constexpr int kSkWaves = 16;       // waves per workgroup
constexpr int kSkMaxWg = 256;      // workgroups (partials) at most
constexpr int kSkGroup = 16;       // workgroups per first-level fold group (two-level fold)
constexpr int kSkinnyMinK = 4096;  // shorter reductions stay on the tiled kernel
constexpr int kSkMaxM = 96;
struct SkinnyK {
  GemmK g;
  float* part;  // [nwg][P4] partials, then [ngrp][P4] group sums (two-level fold)
  int* cnt;     // tickets: [0] the final fold, [1 + grp] the groups
  int kpw;      // k per wave (multiple of 4)
  int nwg, P;   // P = M * N (kernel columns, the column-sum column included)
  int P4;       // partial row stride: P rounded up to 4 (16-B rows)
  int ngrp;     // 0: one-level fold; else first-level groups of kSkGroup workgroups
  int stop;     // profiling probe (DSTAGNN_SKINNY_STOP): 1 = after the loads + MFMAs, 2 = after the ticket
};

__device__ __forceinline__ float sk_ld(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sk_st(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ticket of one workgroup on *c among n arrivals (call after every storing wave drained its
// sc1 stores and a barrier): true in every thread of the last arrival, which has acquired
__device__ __forceinline__ bool sk_ticket(int* c, int n, int* last) {
  if (threadIdx.x == 0) {
    *last = atomicAdd(c, 1) == n - 1;
    if (*last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
  }
  __syncthreads();
  return *last != 0;
}

// sum of rows [0, nrows) of src (rows of P4 floats, 16-B aligned) in a fixed order: thread t
// < C4 = P4/4 gets column quad t.  S = 1024 / C4 subsets of the rows per quad (sub, sub + S,
// ...), sixteen 16-B loads in flight per round, then the subsets in order via LDS (sums:
// >= 1024 float4).  relaxed: agent-scope loads (the rows came from other workgroups' sc1
// stores and are read without this workgroup having acquired them at load time)
template <bool RELAXED>
__device__ __forceinline__ float4 sk_fold_rows(const float* src, int nrows, int P4, float4* sums) {
  const int t = threadIdx.x;
  const int C4 = P4 / 4, S = max(1, 1024 / C4);
  const int sub = t / C4, c = t % C4;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (sub < S) {
    const float4* p = reinterpret_cast<const float4*>(src) + c;
    for (int q = sub; q < nrows; q += 16 * S) {
      float4 u[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if (q + j * S < nrows) {
          const float4* a = p + (int64_t)(q + j * S) * C4;
          if (RELAXED) {
            const float* f = reinterpret_cast<const float*>(a);
            u[j] = make_float4(sk_ld(f), sk_ld(f + 1), sk_ld(f + 2), sk_ld(f + 3));
          } else {
            u[j] = *a;
          }
        } else {
          u[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) { v.x += u[j].x; v.y += u[j].y; v.z += u[j].z; v.w += u[j].w; }
    }
  }
  __syncthreads();
  if (sub < S) sums[t] = v;
  __syncthreads();
  float4 tot = make_float4(0.f, 0.f, 0.f, 0.f);
  if (t < C4) {
    tot = sums[t];
    for (int j = 1; j < S; ++j) {
      const float4 x = sums[j * C4 + t];
      tot.x += x.x; tot.y += x.y; tot.z += x.z; tot.w += x.w;
    }
  }
  return tot;
}

// A4: A's k map takes every aligned quad of k to 4 contiguous, 16-B aligned floats (the
// aggregate-first dTheta: A = agg[b,j,k,f,t], k = (b,j,t), T % 4 == 0) — each lane then loads
// a float4 of A per 4 MFMA steps (contraction index 16 v + 4 q + s of round v, step s, lane
// group q) instead of one dword per step: 4x fewer A load instructions and 16-B row pieces
// instead of 4-B ones (was 26 us for the PEMS08 dTheta, ~1.3 TB/s).
template <int MT, int NT, int U, bool A4 = false>  // 16-row / 16-column accumulator tiles, MFMA steps per load round
__global__ __launch_bounds__(1024) void skinny_dw_kernel(SkinnyK s) {
  constexpr int kS = MT > 2 ? 4 : 8;  // LDS fold slots (waves fold in 16 / kS rounds)
  static_assert(kS * MT * 16 * 33 >= 4096, "the final fold's 1024 float4 sums live in red");
  __shared__ __attribute__((aligned(16))) float red[kS][MT * 16 * 33];
  __shared__ int last;
  const GemmK& g = s.g;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, q4 = lane >> 4, i16 = lane & 15;
  const int k0 = (blockIdx.x * kSkWaves + w) * s.kpw, k1 = min(g.K, k0 + s.kpw);
  uint32_t ao[MT], bo[NT];
  bool arow[MT], bcol[NT], ones[NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + i16;
    arow[mt] = m < g.M;
    ao[mt] = (uint32_t)g.abias + (arow[mt] ? (uint32_t)koff(g.am, m) : 0u);
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int n = nt * 16 + i16;
    bcol[nt] = n < g.nload;
    ones[nt] = n == g.nload && g.nload < g.N;
    bo[nt] = (uint32_t)g.bbias + (bcol[nt] ? (uint32_t)koff(g.bn, n) : 0u);
  }
  floatx4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int kb = k0; kb < k1; kb += 4 * U) {
    float av[U][MT], bv[U][NT];
    if constexpr (A4) {
      static_assert(U % 4 == 0, "rounds of 16 k");
#pragma unroll
      for (int v = 0; v < U / 4; ++v) {
        const int kq = kb + 16 * v + 4 * q4;  // this lane's k quad (all valid or all past k1)
        const bool ok = kq < k1;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const floatx4 x = ok && arow[mt] ? *reinterpret_cast<const floatx4*>(g.A + ao[mt] + (uint32_t)koff(g.ak, kq))
                                           : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int sq = 0; sq < 4; ++sq) av[4 * v + sq][mt] = x[sq];
        }
#pragma unroll
        for (int sq = 0; sq < 4; ++sq)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            bv[4 * v + sq][nt] = ok && bcol[nt] ? g.B[bo[nt] + (uint32_t)koff(g.bk, kq + sq)] : (ok && ones[nt] ? 1.f : 0.f);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int k = kb + 4 * u + q4;
        const bool ok = k < k1;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) av[u][mt] = ok && arow[mt] ? g.A[ao[mt] + (uint32_t)koff(g.ak, k)] : 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          bv[u][nt] = ok && bcol[nt] ? g.B[bo[nt] + (uint32_t)koff(g.bk, k)] : (ok && ones[nt] ? 1.f : 0.f);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u][mt], bv[u][nt], acc[mt][nt], 0, 0, 0);
  }
  // fold the 16 waves: D[m = mt*16 + 4 (l>>4) + r][n = nt*16 + (l&15)]; in rounds from the
  // last kS waves down, each round adding its accumulators into the kS slots, then the slots
  // in order
  auto slot = [&](int mt, int nt, int r) { return (mt * 16 + 4 * q4 + r) * 33 + nt * 16 + i16; };
  constexpr int kRounds = kSkWaves / kS;
#pragma unroll
  for (int rd = kRounds - 1; rd >= 0; --rd) {
    if (w / kS == rd) {
      float* sl = red[w % kS];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sl[slot(mt, nt, r)] = rd == kRounds - 1 ? acc[mt][nt][r] : acc[mt][nt][r] + sl[slot(mt, nt, r)];
    }
    __syncthreads();
  }
  if (s.stop == 1) return;
  float* p1 = s.part + (int64_t)blockIdx.x * s.P4;
  for (int e = t; e < s.P; e += 1024) {
    const int m = e / g.N, o = m * 33 + (e - m * g.N);
    float v = red[0][o];
#pragma unroll
    for (int q = 1; q < kS; ++q) v += red[q][o];
    sk_st(p1 + e, v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float4* sums = reinterpret_cast<float4*>(&red[0][0]);
  const int C4 = s.P4 / 4;
  const float* rows = s.part;
  int nrows = s.nwg;
  if (s.ngrp > 0) {
    // first level: the last arrival of this workgroup's group sums the group's partials
    const int grp = blockIdx.x / kSkGroup, g0 = grp * kSkGroup, gn = min(kSkGroup, s.nwg - g0);
    if (!sk_ticket(s.cnt + 1 + grp, gn, &last) || s.stop == 2) return;
    const float4 tot = sk_fold_rows<false>(s.part + (int64_t)g0 * s.P4, gn, s.P4, sums);
    float* gs = s.part + ((int64_t)s.nwg + grp) * s.P4;
    if (t < C4) {
      sk_st(gs + 4 * t, tot.x); sk_st(gs + 4 * t + 1, tot.y); sk_st(gs + 4 * t + 2, tot.z); sk_st(gs + 4 * t + 3, tot.w);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    rows = s.part + (int64_t)s.nwg * s.P4;
    nrows = s.ngrp;
  }
  if (!sk_ticket(s.cnt, nrows, &last) || (s.stop == 2 && s.ngrp == 0)) return;
  // the last arrival (plain loads behind its acquire)
  const float4 tot = sk_fold_rows<false>(rows, nrows, s.P4, sums);
  if (t < C4) {
    const float tv[4] = {tot.x, tot.y, tot.z, tot.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = 4 * t + i;
      if (e < s.P) epilogue_store(g, 0, e / g.N, e % g.N, tv[i]);
    }
  }
}

// A's k map sends every aligned k quad to 4 contiguous, 16-B aligned floats (skinny_dw_kernel A4)
bool skinny_a4(const SkinnyK& s) {
  static const bool on = !getenv("DSTAGNN_SKINNY_A4") || atoi(getenv("DSTAGNN_SKINNY_A4")) != 0;
  const GemmK& g = s.g;
  const bool quads = g.ak.s0 == 1 && (g.ak.d == 0x80000000u || g.ak.d % 4 == 0) && g.ak.s1 % 4 == 0;
  bool rows = reinterpret_cast<uintptr_t>(g.A) % 16 == 0 && g.abias % 4 == 0 && g.K % 4 == 0 && s.kpw % 4 == 0;
  for (int m = 0; m < g.M && rows; ++m) {  // every row's offset a multiple of 4 (host-side koff)
    const uint32_t q = g.am.d == 0x80000000u ? 0u : (uint32_t)m / g.am.d, r = (uint32_t)m - q * g.am.d;
    rows = ((int64_t)r * g.am.s0 + (int64_t)q * g.am.s1) % 4 == 0;
  }
  return on && quads && rows;
}

void launch_skinny(const SkinnyK& s, hipStream_t st) {
  const dim3 grid((unsigned)s.nwg), blk(64 * kSkWaves);
  const int mt = (s.g.M + 15) / 16, nt = s.g.N > 16 ? 2 : 1;
  const bool a4 = skinny_a4(s);
#define SK_L(MT_, U_)                                                                                       \
  if (a4) {                                                                                                 \
    if (nt == 1) hipLaunchKernelGGL((skinny_dw_kernel<MT_, 1, U_, true>), grid, blk, 0, st, s);          \
    else hipLaunchKernelGGL((skinny_dw_kernel<MT_, 2, U_, true>), grid, blk, 0, st, s);                  \
  } else if (nt == 1) hipLaunchKernelGGL((skinny_dw_kernel<MT_, 1, U_>), grid, blk, 0, st, s);            \
  else hipLaunchKernelGGL((skinny_dw_kernel<MT_, 2, U_>), grid, blk, 0, st, s);
  if (mt == 1) { SK_L(1, 16) }
  else if (mt == 2) { SK_L(2, 16) }
  else if (mt == 3) { SK_L(3, 8) }
  else if (mt == 4) { SK_L(4, 8) }
  else { SK_L(6, 4) }
#undef SK_L
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
  int kind = DSTAGNN_PROF_GEMM;  // DSTAGNN_PROF_* (include/dstagnn.h)
  float ms = 0.f;                // set by gemm_prof_stop
};
struct Prof {
  bool on = false;
  int n = 0, cap = 0, dropped = 0, last = 0;
  ProfRec* rec = nullptr;
};
Prof g_prof;
// split-K target grid (workgroups): a GEMM whose grid is below 128 workgroups splits its K
// range to about this many (448: best of the round-3-end same-box sweep over 256 / 320 / 448,
// tools/knob_sweep.sh; 1 = never split: every tiled reduction in one fixed order, so
// a per-sample result is bit-identical at any batch size — the skinny weight-gradient kernel
// splits regardless, see plan_skinny); DSTAGNN_SPLITK_TARGET overrides
int g_splitk_target = getenv("DSTAGNN_SPLITK_TARGET") ? atoi(getenv("DSTAGNN_SPLITK_TARGET")) : 448;
// operand precision of every GEMM: 0 = fp32 (v_mfma_f32_32x32x2_f32, the reference's
// arithmetic), 1 = bf16 operands rounded to nearest even with fp32 accumulation
// (v_mfma_f32_32x32x16_bf16) — an opt-in variant, see gemm_set_bf16
int g_bf16 = 0;

}  // namespace

namespace { bool gemm_log_on(); }
bool gemm_prof_on() { return g_prof.on; }

// the same event pair around a non-GEMM kernel that computes a GEMM-family product (the
// sliding-window GTU input gradient, gtu_tconv.hip): counted with its algorithmic FLOP / bytes
void* gemm_prof_begin(double flops, double bytes, hipStream_t st, int kind) {
  if (gemm_log_on() && kind != DSTAGNN_PROF_GEMM)  // (tools/step_kernels.py pairs these with the trace)
    fprintf(stderr, "[fused] kind=%d flops=%.0f bytes=%.0f\n", kind, flops, bytes);
  if (!g_prof.on) return nullptr;
  if (g_prof.n >= g_prof.cap) {
    ++g_prof.dropped;
    return nullptr;
  }
  ProfRec* r = &g_prof.rec[g_prof.n++];
  r->flops = flops;
  r->bytes = bytes;
  r->kind = kind;
  (void)hipEventRecord(r->e0, st);
  return r;
}
void gemm_prof_end(void* rec, hipStream_t st) {
  if (rec) (void)hipEventRecord(static_cast<ProfRec*>(rec)->e1, st);
}

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
    r.ms = ms;
    s.launches += 1;
    s.flops += r.flops;
    s.bytes += r.bytes;
    s.ms += ms;
    s.max_ms = std::max(s.max_ms, (double)ms);
  }
  s.dropped = g_prof.dropped;
  g_prof.last = g_prof.n;  // the window's records stay readable (gemm_prof_records) until the next start
  g_prof.n = 0;
  if (out) *out = s;
  return 0;
}

int gemm_prof_records(dstagnn_prof_record* out, int cap) {
  const int n = std::min(cap, g_prof.last);
  for (int i = 0; i < n && out; ++i) {
    const ProfRec& r = g_prof.rec[i];
    out[i].flops = r.flops;
    out[i].bytes = r.bytes;
    out[i].ms = r.ms;
    out[i].kind = r.kind;
  }
  return g_prof.last;
}

namespace {

// persistent tile loop knobs: DSTAGNN_GEMM_PERSIST=1 turns it on; _MIN = fewest tiles that take
// it; _WPC = workgroups per CU of its grid
bool gemm_persist_on() {
  static const bool on = getenv("DSTAGNN_GEMM_PERSIST") && atoi(getenv("DSTAGNN_GEMM_PERSIST")) != 0;
  return on;
}
int64_t gemm_persist_min_tiles() {
  static const int64_t v = getenv("DSTAGNN_GEMM_PERSIST_MIN") ? atoll(getenv("DSTAGNN_GEMM_PERSIST_MIN")) : 384;
  return v;
}
int gemm_persist_wpc() {
  static const int v = getenv("DSTAGNN_GEMM_PERSIST_WPC") ? std::max(1, atoi(getenv("DSTAGNN_GEMM_PERSIST_WPC"))) : 1;
  return v;
}
constexpr int kCUs = 256;  // MI355X compute units

// one problem's launch plan: its kernel descriptor and the kernel configuration it needs
bool gemm_log_on() {
  static const bool on = getenv("DSTAGNN_GEMM_LOG") != nullptr;
  return on;
}

struct Plan {
  GemmK k;
  char log[240];
  int best, va, vb, ns;
  bool akc, bnc, ktwo, hot, acc2;
  bool skinny;  // runs as skinny_dw_kernel (sk), never grouped
  bool persist; // runs as gemm_f32_persist_kernel: k.count tiles over `wgs` workgroups
  uint32_t wgs;
  SkinnyK sk;
  bool same_kernel(const Plan& o) const {
    return !skinny && !o.skinny && best == o.best && va == o.va && vb == o.vb && ns == o.ns && akc == o.akc &&
           bnc == o.bnc && ktwo == o.ktwo && hot == o.hot && acc2 == o.acc2 && persist == o.persist;
  }
  // workgroups of this problem's grid slice (before the padding to a multiple of 8)
  uint32_t slice() const { return persist ? wgs : k.count; }
  // split-K slab floats this plan takes from the workspace
  size_t ws_floats() const {
    if (skinny) return (size_t)(sk.nwg + sk.ngrp) * sk.P4;
    return k.splitk > 1 ? (size_t)k.batch * k.splitk * k.M * k.N : 0;
  }
};

// the skinny kernel's plan (plan_gemm has filled pl.k); false: keep the tiled kernel
bool plan_skinny(Plan& pl, float* ws, size_t ws_floats, hipStream_t st) {
  static const bool on = !getenv("DSTAGNN_GEMM_SKINNY") || atoi(getenv("DSTAGNN_GEMM_SKINNY")) != 0;
  const GemmK& k = pl.k;
  if (!on || g_bf16 || !ws || k.batch != 1 || k.M > kSkMaxM || k.N > 32 || k.K < kSkinnyMinK) return false;
  SkinnyK& s = pl.sk;
  s = SkinnyK{};
  // <= kSkMaxWg workgroups of kSkWaves waves, a multiple of 4 k per wave
  static const int env_kpw = getenv("DSTAGNN_SKINNY_KPW") ? atoi(getenv("DSTAGNN_SKINNY_KPW")) : 0;
  s.kpw = (int)std::max<int64_t>(4, cdiv64(cdiv64(k.K, (int64_t)kSkMaxWg * kSkWaves), 4) * 4);
  if (env_kpw > 0) s.kpw = (int)std::max<int64_t>(s.kpw, cdiv64(env_kpw, 4) * 4);
  s.nwg = (int)cdiv64(k.K, (int64_t)kSkWaves * s.kpw);
  s.P = k.M * k.N;
  s.P4 = (s.P + 3) / 4 * 4;
  // one fold level while the last workgroup reads <= DSTAGNN_SKINNY_FOLD1_KB of partials (one
  // CU pulls ~150 GB/s: 512 KB ~ 3.5 us), else groups of kSkGroup first
  static const int fold1_kb = getenv("DSTAGNN_SKINNY_FOLD1_KB") ? atoi(getenv("DSTAGNN_SKINNY_FOLD1_KB")) : 512;
  s.ngrp = (int64_t)s.nwg * s.P4 * 4 > (int64_t)fold1_kb * 1024 ? (int)cdiv64(s.nwg, kSkGroup) : 0;
  if ((size_t)(s.nwg + s.ngrp) * s.P4 > ws_floats || (reinterpret_cast<uintptr_t>(ws) & 15) != 0) return false;
  s.cnt = stream_counters(st, 1 + s.ngrp);
  if (!s.cnt) return false;
  s.stop = getenv("DSTAGNN_SKINNY_STOP") ? atoi(getenv("DSTAGNN_SKINNY_STOP")) : 0;
  pl.k.splitk = 1;
  pl.k.kchunk = k.K;
  s.g = pl.k;
  s.part = ws;
  pl.skinny = true;
  if (gemm_log_on()) {
    const size_t n = strlen(pl.log);
    snprintf(pl.log + n, sizeof(pl.log) - n, " skinny kpw=%d nwg=%d ngrp=%d", s.kpw, s.nwg, s.ngrp);
  }
  return true;
}

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
  pl.skinny = false;
  pl.persist = false;
  pl.wgs = 0;
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
  if (g.omap) {  // Cout's own maps (no c_off: an independent tensor)
    if (!g.Cout || g.relu || g.emask || g.ones_out) {
      set_last_error("gemm: an output map needs Cout and no ReLU / mask / column-sum epilogue");
      return DSTAGNN_E_ARG;
    }
    if (g.om.two && g.om.f.d % 32 != 0) {  // gemm_epilogue: 32-row fragments in one map period
      set_last_error("gemm: a two-level output row map needs a period that is a multiple of 32");
      return DSTAGNN_E_ARG;
    }
    if (!make_kidx(g.om, g.M, &k.om) || !make_kidx(g.on, g.N, &k.on) ||
        idx_span(g.om, g.M) + idx_span(g.on, g.N) >= (1ll << 31) || idx_min(g.om, g.M) < 0 || idx_min(g.on, g.N) < 0) {
      set_last_error("gemm: output map offsets exceed int32");
      return DSTAGNN_E_SHAPE;
    }
    k.Cout = g.Cout;
    k.oz = make_zidx(g.oz);
    k.omap = 1;
    k.obeta = g.obeta;
  }
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
  if (g.omap) best = 0;  // the output-map epilogue exists in the 64x64 tile's kernels only
  const Cfg cfg = kCfgs[best];
  const int64_t blocks = cdiv64(g.M, cfg.bm()) * cdiv64(Nk, cfg.bn()) * g.batch;

  // split-K when the grid leaves CUs idle and the reduction is long
  int splitk = 1;
  static const int min_grid = getenv("DSTAGNN_SPLITK_MINGRID") ? atoi(getenv("DSTAGNN_SPLITK_MINGRID")) : 128;
  static const int min_k = getenv("DSTAGNN_SPLITK_MINK") ? atoi(getenv("DSTAGNN_SPLITK_MINK")) : 512;
  if (g.K > 0 && blocks < min_grid && g.K >= min_k && ws) {
    // (a per-call target yields to the global "split-K off" = 1 of the deterministic tests)
    const int target = (g.splitk_target > 0 && g_splitk_target != 1) ? g.splitk_target : g_splitk_target;
    int want = (int)std::min<int64_t>(512, cdiv64(target, blocks));
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
  // persistent tile loop (gemm_persist_body): no split-K, no column-sum column, fp32, the 64x64 /
  // 128x32 tiles, enough tiles that a workgroup walks several; the workgroup count is set per
  // launch (persist_slices)
  pl.persist = gemm_persist_on() && splitk == 1 && !g.ones_out && !g.omap && !g_bf16 && (best == 0 || best == 2) && g.K > 0 &&
               (int64_t)blocks >= gemm_persist_min_tiles();
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
    snprintf(pl.log, sizeof(pl.log), "M=%d N=%d K=%d batch=%d cfg=%d splitk=%d akc=%d bnc=%d ktwo=%d blocks=%lld ns=%d va=%d vb=%d bf=%d ones=%d acc2=%d persist=%d",
             g.M, Nk, g.K, g.batch, best, splitk, (int)pl.akc, (int)pl.bnc, (int)pl.ktwo, (long long)blocks * splitk,
             pl.ns, pl.va, pl.vb, g_bf16, g.ones_out ? 1 : 0, (int)pl.acc2, (int)pl.persist);
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

// the workgroups of each persistent problem of one launch: about kCUs * wpc in all, shared in
// proportion to the problems' k-tile work, each a multiple of 8 (every XCD walks its eighth of
// the tile order) and at most the problem's tile count rounded up to 8
void persist_slices(Plan* const* ps, int n, int ktiles_per_tile0 = -1) {
  double work[kGroupMax], tot = 0;
  for (int p = 0; p < n; ++p) {
    const GemmK& k = ps[p]->k;
    const int kt = ktiles_per_tile0 > 0 ? ktiles_per_tile0 : (k.K + BKMAX - 1) / BKMAX;
    work[p] = (double)k.count * std::max(1, kt);
    tot += work[p];
  }
  const double slots = (double)kCUs * gemm_persist_wpc();
  for (int p = 0; p < n; ++p) {
    const GemmK& k = ps[p]->k;
    uint32_t w = (uint32_t)std::max(8.0, slots * work[p] / std::max(tot, 1.0));
    w = std::min<uint32_t>((w + 7u) & ~7u, (k.count + 7u) & ~7u);
    ps[p]->wgs = std::max<uint32_t>(8u, w & ~7u);
  }
}

int launch_plans(Plan* const* ps, int n, hipStream_t st) {
  const GemmK* ks[kGroupMax];
  uint32_t counts[kGroupMax];
  if (ps[0]->persist) persist_slices(ps, n);
  for (int p = 0; p < n; ++p) { ks[p] = &ps[p]->k; counts[p] = ps[p]->slice(); }
  GemmG gg;
  const uint32_t grid = make_group(ks, counts, n, &gg);
  const StreamSig sg = peek_stream_sig(st);
  gg.sig = sg.p;
  gg.sig_v = sg.v;
  using Unit = void (*)(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
  static const Unit units[3][3][2] = {
      {{gemm_c0_k0, gemm_c0_k1}, {gemm_c1_k0, gemm_c1_k1}, {gemm_c2_k0, gemm_c2_k1}},
      {{gemm_c0_k0_bf, gemm_c0_k1_bf}, {gemm_c1_k0_bf, gemm_c1_k1_bf}, {gemm_c2_k0_bf, gemm_c2_k1_bf}},
      {{gemm_c0_k0_a2, gemm_c0_k1_a2}, {nullptr, nullptr}, {gemm_c2_k0_a2, gemm_c2_k1_a2}}};
  const Plan& pl = *ps[0];
  if (pl.persist) {
    static const Unit punits[3][2] = {{gemm_p0_k0, gemm_p0_k1}, {nullptr, nullptr}, {gemm_p2_k0, gemm_p2_k1}};
    punits[pl.best][pl.ktwo ? 1 : 0](gg, dim3(grid), pl.akc, pl.bnc, pl.va, pl.vb, false, st);
  } else {
    const int var = pl.acc2 ? 2 : (g_bf16 ? 1 : 0);
    units[var][pl.best][pl.ktwo ? 1 : 0](gg, dim3(grid), pl.akc, pl.bnc, pl.va, pl.vb, pl.hot, st);
  }
  DS_CHECK_LAUNCH();
  if (sg.p) DS_TRY(stream_sig_sent(st, sg));
  return 0;
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
    plan_skinny(plans[i], ws ? ws + ws_used : nullptr, ws_floats - ws_used, st);
    ws_used += plans[i].ws_floats();
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
      prec->kind = nl == 1 && live[0]->skinny ? DSTAGNN_PROF_SKINNY : DSTAGNN_PROF_GEMM;
      (void)hipEventRecord(prec->e0, st);
    } else {
      ++g_prof.dropped;
    }
  }
  for (int i = 0; i < nl;) {
    int j = i + 1;
    while (j < nl && j - i < kGroupMax && live[j]->same_kernel(*live[i])) ++j;
    if (live[i]->skinny) launch_skinny(live[i]->sk, st);
    else DS_TRY(launch_plans(live + i, j - i, st));
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
    if (k.splitk <= 1 || live[i]->skinny) continue;
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
    if (g.M != g0.M || g.N != g0.N || g.batch != g0.batch || g.ones_out || g.hot || g.omap) {
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
      prec->kind = DSTAGNN_PROF_GEMM;
      (void)hipEventRecord(prec->e0, st);
    } else {
      ++g_prof.dropped;
    }
  }
  GemmG gg{};
  Plan* p0 = &plans[0];
  int kts = 0;
  for (int p = 0; p < n; ++p) kts += (gs[p].K + BKMAX - 1) / BKMAX;
  if (p0->persist) persist_slices(&p0, 1, kts);
  const uint32_t grid = (p0->slice() + 7u) & ~7u;
  gg.start[0] = (uint32_t)n;  // K-concatenated
  for (int p = 1; p < 4; ++p) gg.start[p] = grid;
  for (int p = 0; p < n; ++p) gg.k[p] = plans[p].k;
  const StreamSig sg = peek_stream_sig(st);
  gg.sig = sg.p;
  gg.sig_v = sg.v;
  using Unit = void (*)(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
  static const Unit units[2][3][2] = {
      {{gemm_c0_k0, gemm_c0_k1}, {gemm_c1_k0, gemm_c1_k1}, {gemm_c2_k0, gemm_c2_k1}},
      {{gemm_c0_k0_bf, gemm_c0_k1_bf}, {gemm_c1_k0_bf, gemm_c1_k1_bf}, {gemm_c2_k0_bf, gemm_c2_k1_bf}}};
  const Plan& pl = plans[0];
  if (pl.persist)
    gemm_p2_k0(gg, dim3(grid), pl.akc, pl.bnc, pl.va, pl.vb, false, st);
  else
    units[g_bf16 ? 1 : 0][pl.best][pl.ktwo ? 1 : 0](gg, dim3(grid), pl.akc, pl.bnc, pl.va, pl.vb, false, st);
  DS_CHECK_LAUNCH();
  if (sg.p) DS_TRY(stream_sig_sent(st, sg));
  if (gemm_log_on()) {
    fprintf(stderr, "[gemm] kcat %s", plans[0].log);
    for (int q = 1; q < n; ++q) fprintf(stderr, " + %s", plans[q].log);
    fprintf(stderr, "\n");
  }
  if (prec) (void)hipEventRecord(prec->e1, st);
  return 0;
}

int run_gemm(const Gemm& g, float* ws, size_t ws_floats, hipStream_t st) { return run_gemm_group(&g, 1, ws, ws_floats, st); }

