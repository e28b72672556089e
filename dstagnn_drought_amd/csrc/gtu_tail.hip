// gtu_tail.hip — the block's per-node epilogue, fused (gfx950).
//
// After the three GTU convolution GEMMs (conv[q] rows (t, o), bias included) everything up
// to the block output is per node (b, n) and tiny (C*T = 384 values at PEMS08):
//   gates       G[c, s]  = tanh(P) * sigmoid(Q)          (GTU :190-197, concat over q)
//   fcmy        tc[c, t] = b[t] + sum_s G[c, s] W[t, s]   (:243, Linear(3T-12 -> T))
//   dropout, residual, ReLUs, LayerNorm over C            (:244-253)
// One workgroup per node does all of it from LDS: G is written once (the backward's fcmy
// weight gradient needs it) and never re-read, tc never leaves the workgroup.  The
// backward fuses the mirror image: LN / residual backward -> dtc -> dG = dtc W (fcmy) ->
// the gates' backward into the zero-padded (t', o) rows the transposed-convolution GEMMs
// read.  Replaces gate_fwd + fcmy GEMM + tail_fwd (3 launches, 2 HBM round trips of G and
// tc) and tail_bwd + dG GEMM + gate_bwd.
//
// Long series (GAMBIA T=144: S = 420, the fcmy weight is 242 KB and a node's G tile 54 KB)
// do not fit that mould: one wave per node would run the 2*C*T*S = 3.9 MFLOP fcmy product
// per node as scalar FMAs out of cache (measured 0.37 TFLOP/s, 93 % of the step).  There
// the tail splits around the product (also from T >= 20, measured faster): gates -> G
// (gtu_gates_kernel, LDS transpose), the fcmy product as one MFMA GEMM over all B*N*C rows
// (bias in its epilogue, written into tco), residual / ReLUs / LayerNorm reading it back
// (node kernel, PH 2); backward: LN / residual -> dtc (node kernel, PH 1), dG = dtc W as
// one GEMM, the gates backward from dG (gtu_gates_bwd_kernel).
#include "common.hpp"
#include "ops.hpp"

namespace {

// agent-scope stores / loads of the in-kernel partial hand-off (colsum2d's protocol)
__device__ __forceinline__ void gt_st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float gt_ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int kGtG1 = 64;  // workgroups (nodes) per level-1 group of the partial-sum ticket tree

// the last workgroup of each kGtG1 group sums the group's rows of the NS partial arrays (fixed
// order) into level-2 rows; the last group sums those into fold_out.  Called by every
// workgroup after its partial rows went out with agent-scope stores.
template <int C, int NT, int NS>
__device__ __forceinline__ void tail_fold(const GtuTailArgs& a, float* red, int* flag) {
  const int tid = threadIdx.x;
  const float* part[4] = {a.gpart, a.bpart, a.rpart, a.dpart};
  const int nwg = (int)gridDim.x, ng = (nwg + kGtG1 - 1) / kGtG1, g1 = (int)blockIdx.x / kGtG1;
  const int gsz = min(kGtG1, nwg - g1 * kGtG1);
  constexpr int ITEMS = NS * C, SPL = NT / ITEMS > 0 ? NT / ITEMS : 1;  // (item, row-split) per thread
  static_assert(NT % ITEMS == 0 || ITEMS % NT == 0, "thread layout");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int last = atomicAdd(a.fold_cnt + g1, 1) == gsz - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.fold_cnt + g1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  for (int e = tid; e < ITEMS * SPL; e += NT) {  // level 1: rows [g1 * kGtG1, + gsz) of each array
    const int it = e % ITEMS, sp = e / ITEMS, q = it / C, c = it - q * C;
    const float* src = part[q] + (int64_t)g1 * kGtG1 * C + c;
    float v = 0.f;
    for (int r = sp; r < gsz; r += SPL) v += gt_ld_agent(src + (int64_t)r * C);
    red[e] = v;
  }
  __syncthreads();
  for (int it = tid; it < ITEMS; it += NT) {
    float v = 0.f;
    for (int sp = 0; sp < SPL; ++sp) v += red[sp * ITEMS + it];
    gt_st_agent(a.fold_ws + ((int64_t)(it / C) * ng + g1) * C + it % C, v);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int last = atomicAdd(a.fold_cnt + ng, 1) == ng - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.fold_cnt + ng, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return;
  for (int e = tid; e < ITEMS * SPL; e += NT) {  // level 2: the ng group rows
    const int it = e % ITEMS, sp = e / ITEMS, q = it / C, c = it - q * C;
    const float* src = a.fold_ws + (int64_t)q * ng * C + c;
    float v = 0.f;
    for (int r = sp; r < ng; r += SPL) v += gt_ld_agent(src + (int64_t)r * C);
    red[e] = v;
  }
  __syncthreads();
  for (int it = tid; it < ITEMS; it += NT) {
    float v = 0.f;
    for (int sp = 0; sp < SPL; ++sp) v += red[sp * ITEMS + it];
    float* o = a.fold_out[it / C];
    if (o) o[it % C] = v;
  }
}


__device__ __forceinline__ void gate_index(int s, int T, int* gi, int* t) {
  const int T0 = T - 2, T1 = T - 4;
  *gi = s < T0 ? 0 : (s < T0 + T1 ? 1 : 2);
  *t = *gi == 0 ? s : (*gi == 1 ? s - T0 : s - T0 - T1);
}

// tanh / sigmoid from one v_exp + one v_rcp each (absolute error ~1e-7, far inside the
// 1e-4 parity bound) instead of the branchy libm tanhf and an IEEE division
__device__ __forceinline__ float fast_sigmoid(float x) { return __frcp_rn(1.f + __expf(-x)); }
__device__ __forceinline__ float fast_tanh(float x) {
  const float e = __expf(2.f * fminf(fmaxf(x, -15.f), 15.f));
  return 1.f - 2.f * __frcp_rn(e + 1.f);
}

// One wave (64 threads) per node: a node's work is a chain of short dependent phases, so
// what pays is many nodes in flight per CU (up to ~27 single-wave workgroups by LDS), not
// wide workgroups with block-wide barriers.  Every phase first issues all of a lane's global
// loads (clamped addresses, chunks of kU elements), then computes and stores: with a global
// store between two loads the compiler cannot prove they don't alias and would serialise one
// memory round trip per element.
constexpr int kNT = 64;
constexpr int kU = 8;

// KC / KT: compile-time C and T (0 = runtime) so the index divisions fold.  WL: the fcmy
// weight (T x 3T-12) staged in LDS; false for long series (GAMBIA T=144: 242 KB), where
// it is read through L1/L2 instead.
//
// Access patterns: the conv outputs are read with c fastest (rows (t', o) are contiguous
// in o), the X tile (t, c) is staged in LDS coalesced, G goes to HBM from LDS in its
// [c][s] order; LDS rows of G / W / X are padded to an odd stride (S+1, C+1) so the
// column walks are bank-conflict free; the LayerNorm statistics over C use P = 64/T lane
// groups per t (a fixed-order two-level sum) instead of T lanes walking all of C.

// LDS layout (floats), shared by the kernel and the host size computation
struct TailFwdLds {
  int SP, CP, P, gs, rl, xs, red, mus, rss, wl, total;
  __host__ __device__ TailFwdLds(int C, int T, bool stage_w, bool has_g = true, int nt = kNT) {
    const int S = 3 * T - 12;
    SP = S + 1; CP = C + 1; P = T < nt ? nt / T : 1;
    gs = 0; rl = gs + (has_g ? C * SP : 0); xs = rl + C * T; red = xs + T * CP;
    mus = red + (P * T > nt ? P * T : nt); rss = mus + T; wl = rss + T;
    total = wl + (stage_w ? T * SP : 0);
  }
};

// sum over c of v[c*T + t] for every t, into out[t] (lanes: t = l % T, part = l / T)
template <int NT>
__device__ __forceinline__ void col_sums_over_c(const float* v, int C, int T, int P, float* red, float* out,
                                                int tid) {
  for (int l = tid; l < P * T; l += NT) {
    const int t = l % T, part = l / T;
    float acc = 0.f;
    for (int c = part; c < C; c += P) acc += v[c * T + t];
    red[l] = acc;
  }
  __syncthreads();
  for (int t = tid; t < T; t += NT) {
    float acc = 0.f;
    for (int q = 0; q < P; ++q) acc += red[q * T + t];
    out[t] = acc;
  }
  __syncthreads();
}

// PH: 0 = fused, 2 = split path: from the GEMM's tc (in tco) to the output (the gates run
// in gtu_gates_kernel)
template <int KC, int KT, bool WL, int PH = 0, int NT = kNT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(6, 8))) void gtu_tail_fwd_kernel(GtuTailArgs a) {
  extern __shared__ float lds[];
  const int C = KC ? KC : a.C, T = KT ? KT : a.T, S = 3 * T - 12, CT = C * T, C2 = 2 * C, CS = C * S;
  const TailFwdLds L(C, T, WL, PH != 2, NT);
  const int SP = L.SP, CP = L.CP;
  float* Gs = lds + L.gs;    // [c][SP]
  float* rl = lds + L.rl;    // [c][t]
  float* Xs = lds + L.xs;    // [t][CP]
  float* red = lds + L.red;
  float* mus = lds + L.mus;
  float* rss = lds + L.rss;
  float* Wl = lds + L.wl;    // [t][SP] (WL only)
  const float* Ws = WL ? Wl : a.fcmy_w;
  const int WS = WL ? SP : S;
  const int tid = threadIdx.x;
  if (WL)
    for (int e = tid; e < T * S; e += NT) Wl[(e / S) * SP + e % S] = a.fcmy_w[e];
  for (int64_t bn = blockIdx.x; bn < a.BN; bn += gridDim.x) {
    const int64_t base = bn * CT;
    // gates, element (s, c) with c fastest: coalesced conv-row reads
    #pragma unroll 1
    for (int e0 = 0; e0 < (PH == 2 ? 0 : CS); e0 += NT * kU) {
      float pv[kU], qv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = min(e0 + tid + NT * u, CS - 1);
        const int sidx = e / C, c = e - sidx * C;
        int gi, t;
        gate_index(sidx, T, &gi, &t);
        const int Tg = T - 2 - 2 * gi;
        // select, not index: a per-lane index into the kernel-argument array would copy it
        // to scratch memory
        const float* cg = gi == 0 ? a.conv[0] : (gi == 1 ? a.conv[1] : a.conv[2]);
        const float* cv = cg + (bn * Tg + t) * C2;
        pv[u] = cv[c];
        qv[u] = cv[C + c];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + tid + NT * u;
        if (e < CS) {
          const int sidx = e / C, c = e - sidx * C;
          Gs[c * SP + sidx] = fast_tanh(pv[u]) * fast_sigmoid(qv[u]);
        }
      }
    }
    if (!a.first)
      for (int e = tid; e < CT; e += NT) Xs[(e / C) * CP + e % C] = a.X[base + e];  // X rows (t, c)
    __syncthreads();
    if (PH != 2)
      for (int e = tid; e < CS; e += NT) a.G[bn * CS + e] = Gs[(e / S) * SP + e % S];  // [c][s], coalesced
    // fcmy + dropout + residual + ReLUs; element e = (c, t) of the (C, T) output
    #pragma unroll 1
    for (int e0 = 0; e0 < CT; e0 += NT * kU) {
      float xv[kU], tcv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = min(e0 + tid + NT * u, CT - 1);
        xv[u] = a.first ? a.x[bn * T + e % T] : a.x[base + e];
        if (PH == 2) tcv[u] = a.tco[base + e];  // fcmy output (bias included) from the GEMM
      }
#pragma unroll 1
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + tid + NT * u;
        if (e >= CT) continue;
        const int c = e / T, t = e - c * T;
        float tc;
        if (PH == 2) {
          tc = tcv[u];
        } else {
          tc = a.fcmy_b[t];
          const float* gr = Gs + c * SP;
          const float* wr = Ws + t * WS;
          for (int sidx = 0; sidx < S; ++sidx) tc = fmaf(gr[sidx], wr[sidx], tc);
        }
        if (a.drop_p > 0.f) tc *= drop_scale(a.seed, 1, (uint64_t)(base + e) + a.drop_off, a.drop_p);
        float tco, xres;
        if (a.first) {
          tco = fmaxf(tc, 0.f);
          xres = a.res_w[c] * xv[u] + a.res_b[c];
        } else {
          tco = fmaxf(Xs[t * CP + c] + tc, 0.f);
          xres = xv[u];
        }
        const float r = fmaxf(xres + tco, 0.f);
        a.tco[base + e] = tco;
        a.r[base + e] = r;
        rl[e] = r;
      }
    }
    __syncthreads();
    // LayerNorm over C: mean, then the centred second moment (two fixed-order passes)
    col_sums_over_c<NT>(rl, C, T, L.P, red, mus, tid);
    for (int t = tid; t < T; t += NT) mus[t] *= 1.f / C;
    __syncthreads();
    for (int l = tid; l < L.P * T; l += NT) {
      const int t = l % T, part = l / T;
      const float mean = mus[t];
      float acc = 0.f;
      for (int c = part; c < C; c += L.P) { const float d = rl[c * T + t] - mean; acc += d * d; }
      red[l] = acc;
    }
    __syncthreads();
    for (int t = tid; t < T; t += NT) {
      float var = 0.f;
      for (int q = 0; q < L.P; ++q) var += red[q * T + t];
      const float rs = rsqrtf(var * (1.f / C) + 1e-5f);
      rss[t] = rs;
      a.mu[bn * T + t] = mus[t];
      a.rs[bn * T + t] = rs;
    }
    __syncthreads();
    for (int e = tid; e < CT; e += NT) {
      const int c = e / T, t = e - c * T;
      a.out[base + e] = (rl[e] - mus[t]) * rss[t] * a.ln_g[c] + a.ln_b[c];
    }
    __syncthreads();  // LDS reuse by the next node
  }
}

// Split path, gates only: G[bn][c][s] = tanh(P) * sigmoid(Q) for one (node, 64-wide s
// chunk) per 256-thread workgroup.  Conv rows are read with c fastest (coalesced), the tile
// is transposed through LDS ([c][s], odd stride) and written as 64-float G row segments.
// Small LDS (C*65 floats), so many workgroups per CU: this is an HBM stream, not a chain.
constexpr int kGsW = 64;
__global__ __launch_bounds__(256) void gtu_gates_kernel(GtuTailArgs a, int nchunk) {
  extern __shared__ float lds[];
  const int C = a.C, T = a.T, S = 3 * T - 12, C2 = 2 * C;
  const int64_t bn = blockIdx.x / nchunk;
  const int s0 = (int)(blockIdx.x % nchunk) * kGsW;
  const int tid = threadIdx.x;
  for (int e = tid; e < kGsW * C; e += 256) {
    const int sl = e / C, c = e - sl * C, sidx = s0 + sl;
    if (sidx < S) {
      int gi, t;
      gate_index(sidx, T, &gi, &t);
      const int Tg = T - 2 - 2 * gi;
      const float* cg = gi == 0 ? a.conv[0] : (gi == 1 ? a.conv[1] : a.conv[2]);
      const float* cv = cg + (bn * Tg + t) * C2;
      lds[c * (kGsW + 1) + sl] = fast_tanh(cv[c]) * fast_sigmoid(cv[C + c]);
    }
  }
  __syncthreads();
  float* G = a.G + bn * (int64_t)C * S;
  for (int e = tid; e < C * kGsW; e += 256) {
    const int c = e / kGsW, sl = e - c * kGsW;
    if (s0 + sl < S) G[(int64_t)c * S + s0 + sl] = lds[c * (kGsW + 1) + sl];
  }
}

// Split path, gates backward: one (node, gate, 64-row chunk of the node's zero-padded (t', o)
// rows, the shared-pad layout of the fused kernel) per 256-thread workgroup.  The dG slice is read along s (coalesced), transposed
// through LDS to [t][c]; conv rows and the output rows are walked with o fastest.  vec (C % 4
// == 0, 16-B aligned rows): a thread takes 4 channels c of one row and produces both halves
// (dP | dQ) from one 16-B load of P and of Q — tanh / sigmoid once per (t, c), 16-B loads and
// stores — instead of one output element per thread (each (P, Q) pair loaded and its
// activations computed twice, 4-B accesses).
__global__ __launch_bounds__(256) void gtu_gates_bwd_kernel(GtuTailArgs a, int nchunk, int vec) {
  extern __shared__ float lds[];
  const int C = a.C, T = a.T, S = 3 * T - 12, C2 = 2 * C, CP = C + 1;
  int id = blockIdx.x;
  const int chunk = id % nchunk; id /= nchunk;
  const int gi = id % 3;
  const int64_t bn = id / 3;
  const int ks = 3 + 2 * gi, Tg = T - ks + 1, Lp = T + (bn == a.BN - 1 ? ks - 1 : 0);  // rows of this node
  const int off = gi == 0 ? 0 : (gi == 1 ? T - 2 : 2 * T - 6);
  const int tp0 = chunk * kGsW;
  if (tp0 >= Lp) return;
  const int tid = threadIdx.x;
  const float* dG = a.dG + bn * (int64_t)C * S + off;
  for (int e = tid; e < kGsW * C; e += 256) {
    const int c = e / kGsW, tl = e - c * kGsW, t = tp0 + tl - (ks - 1);
    lds[tl * CP + c] = (t >= 0 && t < Tg) ? dG[(int64_t)c * S + t] : 0.f;
  }
  __syncthreads();
  const float* cv = (gi == 0 ? a.conv[0] : (gi == 1 ? a.conv[1] : a.conv[2])) + bn * C2 * Tg;
  float* orow = (gi == 0 ? a.dconv_pad[0] : (gi == 1 ? a.dconv_pad[1] : a.dconv_pad[2])) + bn * (int64_t)C2 * T;
  if (vec) {
    const int C4 = C >> 2;
    for (int e = tid; e < kGsW * C4; e += 256) {
      const int tl = e / C4, c = (e - tl * C4) * 4, tp = tp0 + tl;
      if (tp >= Lp) continue;
      const int t = tp - (ks - 1);
      float4 vp = make_float4(0.f, 0.f, 0.f, 0.f), vq = vp;
      if (t >= 0 && t < Tg) {
        const float4 p4 = *reinterpret_cast<const float4*>(cv + (int64_t)t * C2 + c);
        const float4 q4 = *reinterpret_cast<const float4*>(cv + (int64_t)t * C2 + C + c);
        const float* dl = lds + tl * CP + c;
        const float pv[4] = {p4.x, p4.y, p4.z, p4.w}, qv[4] = {q4.x, q4.y, q4.z, q4.w};
        float op[4], oq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float th = fast_tanh(pv[j]), sg = fast_sigmoid(qv[j]), dg = dl[j];
          op[j] = dg * (1.f - th * th) * sg;
          oq[j] = dg * th * sg * (1.f - sg);
        }
        vp = make_float4(op[0], op[1], op[2], op[3]);
        vq = make_float4(oq[0], oq[1], oq[2], oq[3]);
      }
      *reinterpret_cast<float4*>(orow + (int64_t)tp * C2 + c) = vp;
      *reinterpret_cast<float4*>(orow + (int64_t)tp * C2 + C + c) = vq;
    }
    return;
  }
  for (int e = tid; e < kGsW * C2; e += 256) {
    const int tl = e / C2, o = e - tl * C2, tp = tp0 + tl;
    if (tp >= Lp) continue;
    const int t = tp - (ks - 1);
    float v = 0.f;
    if (t >= 0 && t < Tg) {
      const int c = o < C ? o : o - C;
      const float pv = cv[t * C2 + c], qv = cv[t * C2 + C + c];
      const float dg = lds[tl * CP + c];
      const float th = fast_tanh(pv), sg = fast_sigmoid(qv);
      v = o < C ? dg * (1.f - th * th) * sg : dg * th * sg * (1.f - sg);
    }
    orow[(int64_t)tp * C2 + o] = v;
  }
}

// dG, the dX tile and the LN reduction scratch share one region (disjoint phases)
struct TailBwdLds {
  int SP, CP, P, dxh, xhl, rr, dg, dxs, red, s1, s2, wl, total;
  __host__ __device__ TailBwdLds(int C, int T, bool stage_w, bool has_g = true, int nt = kNT) {
    const int S = 3 * T - 12, CT = C * T;
    SP = S + 1; CP = C + 1; P = T < nt ? nt / T : 1;
    const int nred = 2 * (P * T > nt ? P * T : nt);
    int shared = has_g ? C * SP : 0;
    if (T * CP > shared) shared = T * CP;
    if (nred > shared) shared = nred;
    dxh = 0; xhl = dxh + CT; rr = xhl + CT; dg = rr + CT; dxs = dg; red = dg; s1 = dg + shared; s2 = s1 + T; wl = s2 + T;
    total = wl + (stage_w ? T * S : 0);
  }
};



// PH: 0 = fused, 1 = split path: LN / residual backward to dtc only (dG by a GEMM, the
// gates backward in gtu_gates_bwd_kernel)
template <int KC, int KT, bool WL, int PH = 0, int NT = kNT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4, 8))) void gtu_tail_bwd_kernel(GtuTailArgs a) {
  extern __shared__ float lds[];
  const int C = KC ? KC : a.C, T = KT ? KT : a.T, S = 3 * T - 12, CT = C * T, C2 = 2 * C;
  const TailBwdLds L(C, T, WL, PH == 0, NT);
  const int SP = L.SP, CP = L.CP;
  float* dxh = lds + L.dxh;   // CT  (LN dxhat, then dtc)
  float* xhl = lds + L.xhl;   // CT
  float* rr = lds + L.rr;     // CT  (r, kept for the ReLU masks)
  float* dGs = lds + L.dg;    // [c][SP]
  float* s1s = lds + L.s1;    // T
  float* s2s = lds + L.s2;    // T
  float* dXs = lds + L.dxs;   // [t][CP] (dX tile, written to HBM coalesced)
  float* red = lds + L.red;
  float* Wl = lds + L.wl;     // T*S (WL only)
  const float* Ws = WL ? Wl : a.fcmy_w;
  const int tid = threadIdx.x;
  if (WL)
    for (int e = tid; e < T * S; e += NT) Wl[e] = a.fcmy_w[e];
  for (int64_t bn = blockIdx.x; bn < a.BN; bn += gridDim.x) {
    const int64_t base = bn * CT;
    const float* mu = a.mu + bn * T;
    const float* rsv = a.rs + bn * T;
    // LayerNorm over C backward
    #pragma unroll 1
    for (int e0 = 0; e0 < CT; e0 += NT * kU) {
      float dyv[kU], rv[kU], muv[kU], rsw[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = min(e0 + tid + NT * u, CT - 1);
        const int t = e % T;
        dyv[u] = a.dout[base + e];
        rv[u] = a.r[base + e];
        muv[u] = mu[t];
        rsw[u] = rsv[t];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + tid + NT * u;
        if (e >= CT) continue;
        const int c = e / T;
        const float xh = (rv[u] - muv[u]) * rsw[u];
        xhl[e] = xh;
        rr[e] = rv[u];
        dxh[e] = dyv[u] * a.ln_g[c];
        if (!a.gpart) a.gcontrib[base + e] = dyv[u] * xh;
      }
    }
    __syncthreads();
    if (a.gpart) {  // LN gamma / beta: sum_t dout * xhat and sum_t dout per channel of this node
      // (dout re-read from L1 / L2: the node's 4*C*T bytes were just loaded)
      for (int c = tid; c < C; c += NT) {
        float g = 0.f, b = 0.f;
        for (int t = 0; t < T; ++t) {
          const float dy = a.dout[base + c * T + t];
          g = fmaf(dy, xhl[c * T + t], g);
          b += dy;
        }
        a.gpart[bn * C + c] = g;
        a.bpart[bn * C + c] = b;
      }
    }
    for (int l = tid; l < L.P * T; l += NT) {  // sum_c dxhat and dxhat*xhat per t, P lane groups
      const int t = l % T, part = l / T;
      float s1 = 0.f, s2 = 0.f;
      for (int c = part; c < C; c += L.P) { s1 += dxh[c * T + t]; s2 += dxh[c * T + t] * xhl[c * T + t]; }
      red[l] = s1;
      red[L.P * T + l] = s2;
    }
    __syncthreads();
    for (int t = tid; t < T; t += NT) {
      float s1 = 0.f, s2 = 0.f;
      for (int q = 0; q < L.P; ++q) { s1 += red[q * T + t]; s2 += red[L.P * T + q * T + t]; }
      s1s[t] = s1 * (1.f / C); s2s[t] = s2 * (1.f / C);
    }
    __syncthreads();
    // ReLUs, residual, dropout: dtc (kept in LDS, dxh reused) and the direct grads
    #pragma unroll 1
    for (int e0 = 0; e0 < CT; e0 += NT * kU) {
      float tcov[kU], xv[kU], rsw[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = min(e0 + tid + NT * u, CT - 1);
        const int t = e % T;
        tcov[u] = a.tco[base + e];

        xv[u] = a.first ? a.x[bn * T + t] : 0.f;
        rsw[u] = rsv[t];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int e = e0 + tid + NT * u;
        if (e >= CT) continue;
        const int c = e / T, t = e - c * T;
        float dr = rsw[u] * (dxh[e] - s1s[t] - xhl[e] * s2s[t]);
        dr = rr[e] > 0.f ? dr : 0.f;                 // relu(xres + tco)
        const float dtco = tcov[u] > 0.f ? dr : 0.f;  // tco = relu(...)
        float dtc = dtco;
        if (a.drop_p > 0.f) dtc *= drop_scale(a.seed, 1, (uint64_t)(base + e) + a.drop_off, a.drop_p);
        a.dtc[base + e] = dtc;
        if (a.first) {
          dXs[t * CP + c] = 0.f;
          if (!a.rpart) {
            a.rcontrib[base + e] = dr * xv[u];
            a.dres[base + e] = dr;
          }
          xhl[e] = dr;  // for the residual_conv channel reduction below (and its partial sums)
        } else {
          dXs[t * CP + c] = dtco;  // dX rows are (t, c), like X
          a.dx[base + e] = dr;
        }
        dxh[e] = dtc;
      }
    }
    __syncthreads();
    for (int e = tid; e < CT; e += NT) a.dX[base + e] = dXs[(e / C) * CP + e % C];  // coalesced
    __syncthreads();  // dXs shares its LDS with dGs
    if (a.first) {
      for (int t = tid; t < T; t += NT) {
        float sum = 0.f;
        for (int c = 0; c < C; ++c) sum += a.res_w[c] * xhl[c * T + t];
        a.dx[bn * T + t] = sum;
      }
      if (a.rpart) {  // residual_conv weight / bias: sum_t dr * x and sum_t dr per channel
        for (int c = tid; c < C; c += NT) {
          float rw = 0.f, rb = 0.f;
          for (int t = 0; t < T; ++t) {
            rw = fmaf(xhl[c * T + t], a.x[bn * T + t], rw);
            rb += xhl[c * T + t];
          }
          a.rpart[bn * C + c] = rw;
          a.dpart[bn * C + c] = rb;
        }
      }
    }
    if (PH == 1) {
      __syncthreads();  // LDS reuse by the next node
      continue;
    }
    // fcmy backward: dG[c, s] = sum_t dtc[c, t] W[t, s]
    #pragma unroll 1
    for (int e = tid; e < (PH == 0 ? C * S : 0); e += NT) {
      const int c = e / S, s = e - c * S;
      float g = 0.f;
      for (int t = 0; t < T; ++t) g = fmaf(dxh[c * T + t], Ws[t * S + s], g);
      dGs[c * SP + s] = g;
    }
    __syncthreads();
    // gates backward into the zero-padded (t', o) rows of each GTU: node bn owns rows
    // [bn*T, bn*T + T) = ks-1 zero rows, then its Tg gate rows; a transposed-convolution
    // window of node bn reaches ks-1 rows into node bn+1, i.e. exactly its zero rows (the
    // last node writes ks-1 trailing zero rows): half the zeros of a per-node [ks-1 | Tg |
    // ks-1] layout
#pragma unroll 1
    for (int gi = 0; gi < 3; ++gi) {
      const int ks = 3 + 2 * gi;
      const int Tg = T - ks + 1;
      const int off = gi == 0 ? 0 : (gi == 1 ? T - 2 : 2 * T - 6);
      const int E = C2 * (T + (bn == a.BN - 1 ? ks - 1 : 0));
      float* orow = (gi == 0 ? a.dconv_pad[0] : (gi == 1 ? a.dconv_pad[1] : a.dconv_pad[2])) + bn * C2 * T;
      const float* cv = (gi == 0 ? a.conv[0] : (gi == 1 ? a.conv[1] : a.conv[2])) + bn * C2 * Tg;
      #pragma unroll 1
      for (int e0 = 0; e0 < E; e0 += NT * kU) {
        float pv[kU], qv[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int e = min(e0 + tid + NT * u, E - 1);
          const int tp = e / C2, o = e - tp * C2;
          const int t = min(max(tp - (ks - 1), 0), Tg - 1);
          const int c = o < C ? o : o - C;
          pv[u] = cv[t * C2 + c];
          qv[u] = cv[t * C2 + C + c];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int e = e0 + tid + NT * u;
          if (e >= E) continue;
          const int tp = e / C2, o = e - tp * C2;
          const int t = tp - (ks - 1);
          float v = 0.f;
          if (t >= 0 && t < Tg) {
            const int c = o < C ? o : o - C;
            const float dg = dGs[c * SP + off + t];
            const float th = fast_tanh(pv[u]), sg = fast_sigmoid(qv[u]);
            v = o < C ? dg * (1.f - th * th) * sg : dg * th * sg * (1.f - sg);
          }
          orow[e] = v;
        }
      }
    }
    __syncthreads();  // LDS reuse by the next node
  }
}

// ---------------------------------------------------------------------------------------
// Compile-time C / T fused tail (the C = 32, T = 12 blocks of PEMS04/07/08): the arithmetic of
// gtu_tail_{fwd,bwd}_kernel<C, T, true, 0, NT> element for element (bit-identical outputs),
// restructured for latency.  The per-node kernels above walk a node in phases that each
// start with their own global loads (fwd: conv rows, then X, then x; bwd: dout / r / mu / rs,
// dout again for the LN partials, tco, then the conv rows of each GTU), and a node's lifetime
// is ~5 dependent memory round trips (46 us for the PEMS08 backward at ~7 resident nodes per
// CU).  Here every global load of a node — activations, conv rows of all three GTUs (one
// thread per (row, channel) pair: its P and Q values feed both output halves), the small
// parameter vectors — is issued in ONE round at the node's start, into registers; everything
// after that reads LDS and registers only and ends in stores.
// ---------------------------------------------------------------------------------------
// FIRST (compile-time a.first): no uniform branch among the node's loads — a branch there made
// the compiler wait for every load issued before it (vmcnt(0) at the join), splitting the one
// round into three dependent ones
template <int C, int T, int NT, int W, bool FIRST>  // W: occupancy floor for the register allocator (waves / SIMD)
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(W, 8))) void gtu_tail_fwd_ct_kernel(GtuTailArgs a) {
  constexpr int S = 3 * T - 12, CT = C * T, C2 = 2 * C, CS = C * S, SP = S + 1, CP = C + 1;
  constexpr int P = T < NT ? NT / T : 1, NRED = P * T > NT ? P * T : NT;
  constexpr int NG = (CS + NT - 1) / NT, NE = (CT + NT - 1) / NT;
  __shared__ float Gs[C * SP], rl[CT], Xs[T * CP], red[NRED], mus[T], rss[T], Wl[T * SP];
  const int tid = threadIdx.x;
  constexpr int NW = (T * S + NT - 1) / NT;
  {  // the fcmy weight: every load first, then the LDS stores (one memory round)
    float wv[NW];
#pragma unroll
    for (int u = 0; u < NW; ++u) wv[u] = a.fcmy_w[min(tid + NT * u, T * S - 1)];
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int e = tid + NT * u;
      if (e < T * S) Wl[(e / S) * SP + e % S] = wv[u];
    }
  }
  for (int64_t bn = blockIdx.x; bn < a.BN; bn += gridDim.x) {
    const int64_t base = bn * CT;
    // every load of the node, one round
    float pv[NG], qv[NG], Xv[NE], xv[NE], fb[NE], rw[NE], rb[NE], lg[NE], lb[NE];
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      const int e = min(tid + NT * u, CS - 1);
      const int sidx = e / C, c = e - sidx * C;
      int gi, t;
      gate_index(sidx, T, &gi, &t);
      const int Tg = T - 2 - 2 * gi;
      const float* cg = gi == 0 ? a.conv[0] : (gi == 1 ? a.conv[1] : a.conv[2]);
      const float* cv = cg + (bn * Tg + t) * C2;
      pv[u] = cv[c];
      qv[u] = cv[C + c];
    }
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = min(tid + NT * u, CT - 1);
      const int c = e / T, t = e - c * T;
      Xv[u] = FIRST ? 0.f : a.X[base + e];  // (t, c) order, staged below
      xv[u] = FIRST ? a.x[bn * T + t] : a.x[base + e];
      fb[u] = a.fcmy_b[t];
      rw[u] = FIRST ? a.res_w[c] : 0.f;
      rb[u] = FIRST ? a.res_b[c] : 0.f;
      lg[u] = a.ln_g[c];
      lb[u] = a.ln_b[c];
    }
    // gates, element (s, c) with c fastest
#pragma unroll
    for (int u = 0; u < NG; ++u) {
      const int e = tid + NT * u;
      if (e < CS) {
        const int sidx = e / C, c = e - sidx * C;
        Gs[c * SP + sidx] = fast_tanh(pv[u]) * fast_sigmoid(qv[u]);
      }
    }
    if (!FIRST) {
#pragma unroll
      for (int u = 0; u < NE; ++u) {
        const int e = tid + NT * u;
        if (e < CT) Xs[(e / C) * CP + e % C] = Xv[u];  // X rows (t, c)
      }
    }
    __syncthreads();
    for (int e = tid; e < CS; e += NT) a.G[bn * CS + e] = Gs[(e / S) * SP + e % S];  // [c][s], coalesced
    // fcmy + dropout + residual + ReLUs; element e = (c, t) of the (C, T) output
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + NT * u;
      if (e >= CT) continue;
      const int c = e / T, t = e - c * T;
      float tc = fb[u];
      const float* gr = Gs + c * SP;
      const float* wr = Wl + t * SP;
      for (int sidx = 0; sidx < S; ++sidx) tc = fmaf(gr[sidx], wr[sidx], tc);
      if (a.drop_p > 0.f) tc *= drop_scale(a.seed, 1, (uint64_t)(base + e) + a.drop_off, a.drop_p);
      float tco, xres;
      if (FIRST) {
        tco = fmaxf(tc, 0.f);
        xres = rw[u] * xv[u] + rb[u];
      } else {
        tco = fmaxf(Xs[t * CP + c] + tc, 0.f);
        xres = xv[u];
      }
      const float r = fmaxf(xres + tco, 0.f);
      a.tco[base + e] = tco;
      a.r[base + e] = r;
      rl[e] = r;
    }
    __syncthreads();
    // LayerNorm over C: mean, then the centred second moment (two fixed-order passes)
    col_sums_over_c<NT>(rl, C, T, P, red, mus, tid);
    for (int t = tid; t < T; t += NT) mus[t] *= 1.f / C;
    __syncthreads();
    for (int l = tid; l < P * T; l += NT) {
      const int t = l % T, part = l / T;
      const float mean = mus[t];
      float acc = 0.f;
      for (int c = part; c < C; c += P) { const float d = rl[c * T + t] - mean; acc += d * d; }
      red[l] = acc;
    }
    __syncthreads();
    for (int t = tid; t < T; t += NT) {
      float var = 0.f;
      for (int q = 0; q < P; ++q) var += red[q * T + t];
      const float rs = rsqrtf(var * (1.f / C) + 1e-5f);
      rss[t] = rs;
      a.mu[bn * T + t] = mus[t];
      a.rs[bn * T + t] = rs;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + NT * u;
      if (e >= CT) continue;
      const int t = e % T;
      a.out[base + e] = (rl[e] - mus[t]) * rss[t] * lg[u] + lb[u];
    }
    __syncthreads();  // LDS reuse by the next node
  }
}

// the conv rows of GTU gi (kernel width ks) this thread's gate items need: item i = (tp, c)
// of the node's zero-padded output rows, tp < T (+ ks - 1 trailing rows on the last node);
// clamped addresses (always inside the node's rows), zeroed where the item is not a gate row
template <int C, int T, int NT, int NQ>
__device__ __forceinline__ void tail_gate_loads(const float* conv, int ks, int64_t bn, float (&p)[NQ], float (&q)[NQ]) {
  constexpr int C2 = 2 * C;
  const int Tg = T - ks + 1;
  const float* cv = conv + bn * C2 * Tg;
#pragma unroll
  for (int u = 0; u < NQ; ++u) {
    const int i = threadIdx.x + NT * u, tp = i / C, c = i - tp * C;
    const int t = min(max(tp - (ks - 1), 0), Tg - 1);
    p[u] = cv[t * C2 + c];
    q[u] = cv[t * C2 + C + c];
  }
}
// the gates' backward into the node's zero-padded rows: both halves (o = c: tanh side,
// o = C + c: sigmoid side) of item (tp, c) from the preloaded P / Q values
template <int C, int T, int NT, int NQ>
__device__ __forceinline__ void tail_gate_bwd(float* dconv, int ks, int off, int64_t bn, bool last, const float* dGs,
                                              int SP, const float (&p)[NQ], const float (&q)[NQ]) {
  constexpr int C2 = 2 * C;
  const int Tg = T - ks + 1, items = (T + (last ? ks - 1 : 0)) * C;
  float* orow = dconv + bn * C2 * T;
#pragma unroll
  for (int u = 0; u < NQ; ++u) {
    const int i = threadIdx.x + NT * u;
    if (i >= items) continue;
    const int tp = i / C, c = i - tp * C, t = tp - (ks - 1);
    float v0 = 0.f, v1 = 0.f;
    if (t >= 0 && t < Tg) {
      const float dg = dGs[c * SP + off + t];
      const float th = fast_tanh(p[u]), sg = fast_sigmoid(q[u]);
      v0 = dg * (1.f - th * th) * sg;
      v1 = dg * th * sg * (1.f - sg);
    }
    orow[tp * C2 + c] = v0;
    orow[tp * C2 + C + c] = v1;
  }
}

template <int C, int T, int NT, int W, bool FIRST>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(W, 8))) void gtu_tail_bwd_ct_kernel(GtuTailArgs a) {
  constexpr int S = 3 * T - 12, CT = C * T, SP = S + 1, CP = C + 1;
  constexpr int P = T < NT ? NT / T : 1, NRED2 = 2 * (P * T > NT ? P * T : NT);
  constexpr int SH0 = C * SP > T * CP ? C * SP : T * CP, SH = SH0 > NRED2 ? SH0 : NRED2;
  constexpr int NE = (CT + NT - 1) / NT;
  constexpr int NQ3 = ((T + 2) * C + NT - 1) / NT, NQ5 = ((T + 4) * C + NT - 1) / NT, NQ7 = ((T + 6) * C + NT - 1) / NT;
  __shared__ float dxh[CT], xhl[CT], rr[CT], dys[CT], sh[SH], s1s[T], s2s[T], Wl[T * S];
  float* dGs = sh;  // [c][SP]
  float* dXs = sh;  // [t][CP] (dX tile, written to HBM coalesced)
  float* red = sh;
  const int tid = threadIdx.x;
  constexpr int NW = (T * S + NT - 1) / NT;
  {  // the fcmy weight: every load first, then the LDS stores (one memory round)
    float wv[NW];
#pragma unroll
    for (int u = 0; u < NW; ++u) wv[u] = a.fcmy_w[min(tid + NT * u, T * S - 1)];
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      const int e = tid + NT * u;
      if (e < T * S) Wl[e] = wv[u];
    }
  }
  float facc[4] = {0.f, 0.f, 0.f, 0.f};  // fold: this workgroup's partial sums (thread c < C)
  for (int64_t bn = blockIdx.x; bn < a.BN; bn += gridDim.x) {
    const int64_t base = bn * CT;
    const bool last = bn == a.BN - 1;
    // every load of the node, one round
    float dyv[NE], rv[NE], muv[NE], rsw[NE], tcov[NE], xv[NE], lg[NE];
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = min(tid + NT * u, CT - 1);
      const int c = e / T, t = e - c * T;
      dyv[u] = a.dout[base + e];
      rv[u] = a.r[base + e];
      muv[u] = a.mu[bn * T + t];
      rsw[u] = a.rs[bn * T + t];
      tcov[u] = a.tco[base + e];
      xv[u] = FIRST ? a.x[bn * T + t] : 0.f;
      lg[u] = a.ln_g[c];
    }
    float p3[NQ3], q3[NQ3], p5[NQ5], q5[NQ5], p7[NQ7], q7[NQ7];
    tail_gate_loads<C, T, NT, NQ3>(a.conv[0], 3, bn, p3, q3);
    tail_gate_loads<C, T, NT, NQ5>(a.conv[1], 5, bn, p5, q5);
    tail_gate_loads<C, T, NT, NQ7>(a.conv[2], 7, bn, p7, q7);
    // LayerNorm over C backward
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + NT * u;
      if (e >= CT) continue;
      const float xh = (rv[u] - muv[u]) * rsw[u];
      xhl[e] = xh;
      rr[e] = rv[u];
      dxh[e] = dyv[u] * lg[u];
      dys[e] = dyv[u];
      if (!a.gpart) a.gcontrib[base + e] = dyv[u] * xh;
    }
    __syncthreads();
    if (a.gpart) {  // LN gamma / beta: sum_t dout * xhat and sum_t dout per channel of this node
      for (int c = tid; c < C; c += NT) {
        float g = 0.f, b = 0.f;
        for (int t = 0; t < T; ++t) {
          const float dy = dys[c * T + t];
          g = fmaf(dy, xhl[c * T + t], g);
          b += dy;
        }
        if (a.fold) {  // (tid == c < C: this workgroup's sums over its nodes)
          facc[0] += g;
          facc[1] += b;
        } else {
          a.gpart[bn * C + c] = g;
          a.bpart[bn * C + c] = b;
        }
      }
    }
    for (int l = tid; l < P * T; l += NT) {  // sum_c dxhat and dxhat*xhat per t, P lane groups
      const int t = l % T, part = l / T;
      float s1 = 0.f, s2 = 0.f;
      for (int c = part; c < C; c += P) { s1 += dxh[c * T + t]; s2 += dxh[c * T + t] * xhl[c * T + t]; }
      red[l] = s1;
      red[P * T + l] = s2;
    }
    __syncthreads();
    for (int t = tid; t < T; t += NT) {
      float s1 = 0.f, s2 = 0.f;
      for (int q = 0; q < P; ++q) { s1 += red[q * T + t]; s2 += red[P * T + q * T + t]; }
      s1s[t] = s1 * (1.f / C); s2s[t] = s2 * (1.f / C);
    }
    __syncthreads();
    // ReLUs, residual, dropout: dtc (kept in LDS, dxh reused) and the direct grads
#pragma unroll
    for (int u = 0; u < NE; ++u) {
      const int e = tid + NT * u;
      if (e >= CT) continue;
      const int c = e / T, t = e - c * T;
      float dr = rsw[u] * (dxh[e] - s1s[t] - xhl[e] * s2s[t]);
      dr = rr[e] > 0.f ? dr : 0.f;                 // relu(xres + tco)
      const float dtco = tcov[u] > 0.f ? dr : 0.f;  // tco = relu(...)
      float dtc = dtco;
      if (a.drop_p > 0.f) dtc *= drop_scale(a.seed, 1, (uint64_t)(base + e) + a.drop_off, a.drop_p);
      a.dtc[base + e] = dtc;
      if (FIRST) {
        dXs[t * CP + c] = 0.f;
        if (!a.rpart) {
          a.rcontrib[base + e] = dr * xv[u];
          a.dres[base + e] = dr;
        }
        xhl[e] = dr;  // for the residual_conv channel reduction below (and its partial sums)
      } else {
        dXs[t * CP + c] = dtco;  // dX rows are (t, c), like X
        a.dx[base + e] = dr;
      }
      dxh[e] = dtc;
    }
    __syncthreads();
    for (int e = tid; e < CT; e += NT) a.dX[base + e] = dXs[(e / C) * CP + e % C];  // coalesced
    __syncthreads();  // dXs shares its LDS with dGs
    if (FIRST) {
      for (int t = tid; t < T; t += NT) {
        float sum = 0.f;
        for (int c = 0; c < C; ++c) sum += a.res_w[c] * xhl[c * T + t];
        a.dx[bn * T + t] = sum;
      }
      if (a.rpart) {  // residual_conv weight / bias: sum_t dr * x and sum_t dr per channel
        for (int c = tid; c < C; c += NT) {
          float rw = 0.f, rb = 0.f;
          for (int t = 0; t < T; ++t) {
            rw = fmaf(xhl[c * T + t], a.x[bn * T + t], rw);
            rb += xhl[c * T + t];
          }
          if (a.fold) {
            facc[2] += rw;
            facc[3] += rb;
          } else {
            a.rpart[bn * C + c] = rw;
            a.dpart[bn * C + c] = rb;
          }
        }
      }
    }
    // fcmy backward: dG[c, s] = sum_t dtc[c, t] W[t, s]
    for (int e = tid; e < C * S; e += NT) {
      const int c = e / S, s = e - c * S;
      float g = 0.f;
      for (int t = 0; t < T; ++t) g = fmaf(dxh[c * T + t], Wl[t * S + s], g);
      dGs[c * SP + s] = g;
    }
    __syncthreads();
    // gates backward into the zero-padded (t', o) rows of each GTU (layout: gtu_tail_bwd_kernel)
    tail_gate_bwd<C, T, NT, NQ3>(a.dconv_pad[0], 3, 0, bn, last, dGs, SP, p3, q3);
    tail_gate_bwd<C, T, NT, NQ5>(a.dconv_pad[1], 5, T - 2, bn, last, dGs, SP, p5, q5);
    tail_gate_bwd<C, T, NT, NQ7>(a.dconv_pad[2], 7, 2 * T - 6, bn, last, dGs, SP, p7, q7);
    __syncthreads();  // LDS reuse by the next node
  }
  if (a.fold) {  // one partial row per workgroup (its grid-stride nodes), then the ticket tree
    if (tid < C) {
      gt_st_agent(a.gpart + (int64_t)blockIdx.x * C + tid, facc[0]);
      gt_st_agent(a.bpart + (int64_t)blockIdx.x * C + tid, facc[1]);
      if (FIRST) {
        gt_st_agent(a.rpart + (int64_t)blockIdx.x * C + tid, facc[2]);
        gt_st_agent(a.dpart + (int64_t)blockIdx.x * C + tid, facc[3]);
      }
    }
    __shared__ int flag;
    tail_fold<C, NT, FIRST ? 4 : 2>(a, sh, &flag);
  }
}

size_t fwd_lds(const GtuTailArgs& a, bool wl, bool has_g = true, int nt = kNT) {
  return sizeof(float) * (size_t)TailFwdLds(a.C, a.T, wl, has_g, nt).total;
}
size_t bwd_lds(const GtuTailArgs& a, bool wl, bool has_g = true, int nt = kNT) {
  return sizeof(float) * (size_t)TailBwdLds(a.C, a.T, wl, has_g, nt).total;
}

unsigned node_grid(int64_t BN) { return (unsigned)std::min<int64_t>(BN, 65536); }

constexpr size_t kLdsMax = 160 * 1024;  // gfx950 LDS per workgroup

template <typename K>
int launch_node_kernel(K kernel, size_t lds, const GtuTailArgs& a, hipStream_t st, int nt = kNT) {
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) { set_last_error(std::string("gtu_tail LDS: ") + hipGetErrorString(e)); return (int)e; }
  }
  hipLaunchKernelGGL(kernel, dim3(node_grid(a.BN)), dim3(nt), lds, st, a);
  DS_CHECK_LAUNCH();
  return 0;
}

// rows [r0, r0+M) of C[r, n] = sum_k A[r, k] B[k, n] (+ bias[n]); row chunks keep every
// operand offset inside the GEMM's int32 index range
int rows_gemm(const float* A, int lda, const float* B, Idx2 bk, Idx2 bn, float* Cm, int ldc, int64_t M, int N,
              int K, const float* bias, hipStream_t st) {
  const int64_t chunk = std::max<int64_t>(64, ((int64_t)1 << 28) / std::max(lda, ldc)) / 64 * 64;
  for (int64_t r0 = 0; r0 < M; r0 += chunk) {
    Gemm g;
    g.M = (int)std::min(chunk, M - r0); g.N = N; g.K = K;
    g.A = A + r0 * lda; g.am = idx1(lda); g.ak = idx1(1);
    g.B = B; g.bk = bk; g.bn = bn;
    g.C = Cm + r0 * ldc; g.cm = idx1(ldc); g.cn = idx1(1);
    g.bias = bias;
    DS_TRY(run_gemm(g, nullptr, 0, st));
  }
  return 0;
}

}  // namespace

// split (gates | GEMM | tail) when the weight does not fit LDS, or from T >= 20 on
// (measured: SYN T=24 step 60.9 -> 57.7 ms split; PEMS08 T=12 0.91 fused vs 0.99 split);
// DSTAGNN_TAIL_SPLIT_T overrides the threshold (0 = always split, used by the parity runs)
constexpr int kTailSplitT = 20;
// The compile-time tail kernels also at C = 32, T = 24 (the synthetic N = 4096 config) instead
// of the split path: SYN B=32 40.2 -> 37.4-37.7 ms/step same box (2 x 2 runs,
// tools/gpu_check.sh cfgab); DSTAGNN_TAIL_CT24=0 keeps the split path (A/B)
static bool tail_ct24(const GtuTailArgs& a) {
  static const bool on = !getenv("DSTAGNN_TAIL_CT24") || atoi(getenv("DSTAGNN_TAIL_CT24")) != 0;
  return on && a.C == 32 && a.T == 24;
}
bool tail_split_fwd(const GtuTailArgs& a) {
  static const int split_t = getenv("DSTAGNN_TAIL_SPLIT_T") ? atoi(getenv("DSTAGNN_TAIL_SPLIT_T")) : kTailSplitT;
  if (tail_ct24(a) && split_t > 0) return false;
  return fwd_lds(a, true) > 32 * 1024 || a.T >= split_t;
}
bool tail_split_bwd(const GtuTailArgs& a) {
  static const int split_t = getenv("DSTAGNN_TAIL_SPLIT_T") ? atoi(getenv("DSTAGNN_TAIL_SPLIT_T")) : kTailSplitT;
  if (tail_ct24(a) && split_t > 0) return false;
  return bwd_lds(a, true) > 32 * 1024 || a.T >= split_t;
}

// threads per node in the split path's residual / LayerNorm kernels: a long series' node
// tile (C*T = 4608 at GAMBIA) holds ~74 KB of LDS, so only two workgroups fit a CU; 256
// threads each keep 8 waves per CU in flight instead of 2 (DSTAGNN_TAIL_NT=64 for A/B)
int split_nt() {
  static const int nt = getenv("DSTAGNN_TAIL_NT") ? atoi(getenv("DSTAGNN_TAIL_NT")) : 256;
  return nt == 64 ? 64 : 256;
}

// threads per node of the fused C=32/T=12 kernels (DSTAGNN_TAIL_FUSED_NT = 64 | 128 | 256):
// 256 measured 0.868 vs 0.873 ms/step for 64 (PEMS08 block, 2 x 200 steps each)
int fused_nt() {
  static const int nt = getenv("DSTAGNN_TAIL_FUSED_NT") ? atoi(getenv("DSTAGNN_TAIL_FUSED_NT")) : 256;
  return nt;
}

// the one-round-of-loads C = 32 / T = 12 kernels (DSTAGNN_TAIL_CT=0: the phase-by-phase ones;
// 2: register cap for 5 waves / SIMD)
int tail_ct() {
  static const int v = getenv("DSTAGNN_TAIL_CT") ? atoi(getenv("DSTAGNN_TAIL_CT")) : 1;
  return v;
}

bool gtu_tail_bwd_split(int C, int T) {
  GtuTailArgs a;
  a.C = C; a.T = T;
  return tail_split_bwd(a);
}

int op_gtu_tail_fwd(const GtuTailArgs& a, hipStream_t st) {
  if (tail_split_fwd(a)) {  // long series: gates | fcmy GEMM | tail
    const int S = 3 * a.T - 12;
    if (fwd_lds(a, false, false) > kLdsMax) { set_last_error("gtu_tail: C*T too large for LDS"); return DSTAGNN_E_SHAPE; }
    {
      const int nchunk = (S + kGsW - 1) / kGsW;
      const int64_t nwg = a.BN * nchunk;
      if (nwg >= (1ll << 31)) { set_last_error("gtu_gates: grid too large"); return DSTAGNN_E_SHAPE; }
      hipLaunchKernelGGL(gtu_gates_kernel, dim3((unsigned)nwg), dim3(256), sizeof(float) * a.C * (kGsW + 1), st, a,
                         nchunk);
      DS_CHECK_LAUNCH();
    }
    DS_TRY(rows_gemm(a.G, S, a.fcmy_w, idx1(1), idx1(S), a.tco, a.T, a.BN * a.C, a.T, S, a.fcmy_b, st));
    if (split_nt() == 64)
      return launch_node_kernel(gtu_tail_fwd_kernel<0, 0, false, 2, 64>, fwd_lds(a, false, false, 64), a, st, 64);
    return launch_node_kernel(gtu_tail_fwd_kernel<0, 0, false, 2, 256>, fwd_lds(a, false, false, 256), a, st, 256);
  }
  const size_t lds = fwd_lds(a, true);
  if (tail_ct24(a)) {
    const dim3 g(node_grid(a.BN));
    if (a.first) hipLaunchKernelGGL((gtu_tail_fwd_ct_kernel<32, 24, 256, 1, true>), g, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((gtu_tail_fwd_ct_kernel<32, 24, 256, 1, false>), g, dim3(256), 0, st, a);
    DS_CHECK_LAUNCH();
    return 0;
  }
  if (a.C == 32 && a.T == 12 && tail_ct()) {
    const dim3 g(node_grid(a.BN));
    if (tail_ct() == 2) {
      if (a.first) hipLaunchKernelGGL((gtu_tail_fwd_ct_kernel<32, 12, 256, 5, true>), g, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((gtu_tail_fwd_ct_kernel<32, 12, 256, 5, false>), g, dim3(256), 0, st, a);
    } else {
      if (a.first) hipLaunchKernelGGL((gtu_tail_fwd_ct_kernel<32, 12, 256, 1, true>), g, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((gtu_tail_fwd_ct_kernel<32, 12, 256, 1, false>), g, dim3(256), 0, st, a);
    }
    DS_CHECK_LAUNCH();
    return 0;
  }
  if (a.C == 32 && a.T == 12) {
    switch (fused_nt()) {
      case 128: return launch_node_kernel(gtu_tail_fwd_kernel<32, 12, true, 0, 128>, fwd_lds(a, true, true, 128), a, st, 128);
      case 256: return launch_node_kernel(gtu_tail_fwd_kernel<32, 12, true, 0, 256>, fwd_lds(a, true, true, 256), a, st, 256);
      default: return launch_node_kernel(gtu_tail_fwd_kernel<32, 12, true>, lds, a, st);
    }
  }
  return launch_node_kernel(gtu_tail_fwd_kernel<0, 0, true>, lds, a, st);
}

static int64_t fold_wgs() {
  static const int v = getenv("DSTAGNN_TAIL_FOLD_WGS") ? atoi(getenv("DSTAGNN_TAIL_FOLD_WGS")) : 2048;
  return v > 0 ? v : 2048;
}
static bool tail_generic() {
  static const bool generic = getenv("DSTAGNN_TAIL_GENERIC") && atoi(getenv("DSTAGNN_TAIL_GENERIC")) != 0;
  return generic;
}
// the compile-time C / T backward with one node per workgroup, which folds its partial sums
// in-kernel (DSTAGNN_TAIL_FOLD=0: colsum2d launches instead)
bool gtu_tail_bwd_folds(const GtuTailArgs& a) {
  static const bool on = getenv("DSTAGNN_TAIL_FOLD") && atoi(getenv("DSTAGNN_TAIL_FOLD")) != 0;
  if (!on || tail_split_bwd(a) || tail_generic() || !a.gpart) return false;
  return tail_ct24(a) || (a.C == 32 && a.T == 12 && tail_ct());
}

int op_gtu_tail_bwd(const GtuTailArgs& a0, hipStream_t st) {
  const bool generic = tail_generic();
  GtuTailArgs a = a0;
  a.fold = a0.fold && gtu_tail_bwd_folds(a0) && a0.fold_ws;
  if (a.fold) {
    a.fold_cnt = stream_counters(st, (int)cdiv64(std::min<int64_t>(a.BN, fold_wgs()), 64) + 1);
    if (!a.fold_cnt) a.fold = 0;
  }
  if (tail_split_bwd(a)) {  // long series: LN / residual | dG GEMM | gates
    if (!a.dG) { set_last_error("gtu_tail: split backward needs the dG scratch"); return DSTAGNN_E_ARG; }
    const int S = 3 * a.T - 12;
    if (bwd_lds(a, false, false) > kLdsMax) { set_last_error("gtu_tail: C*T too large for LDS"); return DSTAGNN_E_SHAPE; }
    if (split_nt() == 64)
      DS_TRY(launch_node_kernel(gtu_tail_bwd_kernel<0, 0, false, 1, 64>, bwd_lds(a, false, false, 64), a, st, 64));
    else
      DS_TRY(launch_node_kernel(gtu_tail_bwd_kernel<0, 0, false, 1, 256>, bwd_lds(a, false, false, 256), a, st, 256));
    DS_TRY(rows_gemm(a.dtc, a.T, a.fcmy_w, idx1(S), idx1(1), a.dG, S, a.BN * a.C, S, a.T, nullptr, st));
    const int nchunk = (a.T + 6 + kGsW - 1) / kGsW;  // rows of the longest padded output (ks = 7)
    const int64_t nwg = a.BN * 3 * nchunk;
    if (nwg >= (1ll << 31)) { set_last_error("gtu_gates_bwd: grid too large"); return DSTAGNN_E_SHAPE; }
    bool vec = a.C % 4 == 0 && !(getenv("DSTAGNN_GATES_BWD_SCALAR") && atoi(getenv("DSTAGNN_GATES_BWD_SCALAR")));
    for (int q = 0; q < 3; ++q)
      vec = vec && (reinterpret_cast<uintptr_t>(a.conv[q]) & 15) == 0 && (reinterpret_cast<uintptr_t>(a.dconv_pad[q]) & 15) == 0;
    hipLaunchKernelGGL(gtu_gates_bwd_kernel, dim3((unsigned)nwg), dim3(256), sizeof(float) * kGsW * (a.C + 1), st, a,
                       nchunk, vec ? 1 : 0);
    DS_CHECK_LAUNCH();
    return 0;
  }
  const size_t lds = bwd_lds(a, true);
  // folding: fewer workgroups, each walking several nodes, so the per-workgroup hand-off (store
  // drain, barrier, ticket) is paid once per ~3 nodes (one node per workgroup: 36 -> 72 us)
  const unsigned fold_grid = (unsigned)std::min<int64_t>(a.BN, fold_wgs());
  if (tail_ct24(a) && !generic) {
    const dim3 g(a.fold ? fold_grid : node_grid(a.BN));
    if (a.first) hipLaunchKernelGGL((gtu_tail_bwd_ct_kernel<32, 24, 256, 1, true>), g, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((gtu_tail_bwd_ct_kernel<32, 24, 256, 1, false>), g, dim3(256), 0, st, a);
    DS_CHECK_LAUNCH();
    return 0;
  }
  if (a.C == 32 && a.T == 12 && !generic && tail_ct()) {
    const dim3 g(a.fold ? fold_grid : node_grid(a.BN));
    if (tail_ct() == 2) {
      if (a.first) hipLaunchKernelGGL((gtu_tail_bwd_ct_kernel<32, 12, 256, 5, true>), g, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((gtu_tail_bwd_ct_kernel<32, 12, 256, 5, false>), g, dim3(256), 0, st, a);
    } else {
      if (a.first) hipLaunchKernelGGL((gtu_tail_bwd_ct_kernel<32, 12, 256, 1, true>), g, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((gtu_tail_bwd_ct_kernel<32, 12, 256, 1, false>), g, dim3(256), 0, st, a);
    }
    DS_CHECK_LAUNCH();
    return 0;
  }
  if (a.C == 32 && a.T == 12 && !generic) {
    switch (fused_nt()) {
      case 128: return launch_node_kernel(gtu_tail_bwd_kernel<32, 12, true, 0, 128>, bwd_lds(a, true, true, 128), a, st, 128);
      case 256: return launch_node_kernel(gtu_tail_bwd_kernel<32, 12, true, 0, 256>, bwd_lds(a, true, true, 256), a, st, 256);
      default: return launch_node_kernel(gtu_tail_bwd_kernel<32, 12, true>, lds, a, st);
    }
  }
  return launch_node_kernel(gtu_tail_bwd_kernel<0, 0, true>, lds, a, st);
}
