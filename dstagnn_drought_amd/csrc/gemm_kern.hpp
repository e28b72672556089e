// gemm_kern.hpp — the GEMM kernel (gemm_glds_body) and its launchers, shared by the
// instantiation units gemm_c<cfg>_k<ktwo>.hip (one tile shape x one k-map kind each, so the
// 32 kernels of a unit compile in parallel with the others) and gemm.hip (host dispatch,
// split-K fold, profiling).  See gemm.hip for the design.
#pragma once
#include <cstddef>
#include <cstdio>
#include <cstdlib>

#include "common.hpp"

namespace dsgemm {

struct GemmK {
  int M, N, K, batch, splitk, kchunk;
  int32_t abias, bbias;  // added to every A / B element offset (see run_gemm)
  uint32_t tiles_m, tiles_n, n_fast;
  // every map is branch-free (single-level ones encoded with d = 2^31): no control flow
  // between the kernel-argument loads, so they all issue in one round at entry
  const float* A; KIdx am, ak; ZIdx az;
  const float* B; KIdx bn, bk; ZIdx bz;
  float* C; KIdx cm, cn; ZIdx cz;
  float alpha, beta;
  const float* bias; int32_t bias_stride;
  int relu;
  float* ws;  // split partials [batch][splitk][M][N]
  const float* emask;  // optional: zero where emask <= 0 (same maps as C, offset c_off)
  float* Cout;         // optional: destination instead of C (beta still reads C)
  int omap;            // Cout has its own maps om / on / oz (Gemm::omap), obeta * old Cout added
  float obeta;
  KIdx om, on; ZIdx oz;
  int nstage;          // LDS pipeline stages (2 or 3; dynamic LDS)
  // optional column-sum column: N = nload + 1 and column nload of B reads as 1.0, so
  // C[m][nload] = sum_k A[m][k] (a bias gradient folded into its weight-gradient GEMM);
  // it is stored to ones_out[m * ones_stride], never into C.  Without it nload = N.
  int nload;
  float* ones_out;
  int32_t ones_stride;
  uint32_t count;      // workgroups of this problem (tiles x batch x splitk; the grid slice is padded to 8)
  int red_g;           // split-K fold: split groups per output (splitk_reduce_kernel)
};

// One launch runs up to kGroupMax independent problems of the same kernel configuration
// (the three GTU convolutions, their three weight gradients): problem p owns workgroups
// [start[p], start[p+1]); each slice starts at a multiple of 8, so a workgroup's XCD (id % 8)
// is the same in the slice as in the grid and the XCD-aware tile order holds per problem.
#ifndef DSTAGNN_GEMM_GROUP_MAX
#define DSTAGNN_GEMM_GROUP_MAX 3
#endif
constexpr int kGroupMax = DSTAGNN_GEMM_GROUP_MAX;
struct GemmG {
  // start[p] (p = 1..3): first workgroup of problem p (the grid size for p >= n).
  // start[0] = 0 for independent problems; = n >= 2 for ONE K-concatenated problem
  // (run_gemm_kcat): every workgroup runs its tile over the K ranges of problems 0..n-1 in
  // turn (same M, N, tiles; own A / B operands and maps) into one accumulator and stores it
  // with problem 0's epilogue.
  uint32_t start[4];
  GemmK k[kGroupMax];
  uint32_t* sig;  // kernel-written stream signal (common.hpp), read by workgroup 0 only
  uint32_t sig_v, sig_pad;
};

namespace {

constexpr int BKMAX = 32;  // k-tile depth

__device__ __forceinline__ floatx16 zero_acc() {
  floatx16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// The problem of this workgroup and its descriptor, in one memory round: every lane loads
// dwords lane, lane+64, ... of the whole group argument, the slice starts come back by
// readlane, and the selected problem's dwords by readlane from compile-time positions (one
// uniform branch per problem index).  See load_args.
template <int P, int NV>
__device__ __forceinline__ void pick_problem(const uint32_t (&v)[NV], uint32_t* w) {
  constexpr int NK = (int)(sizeof(GemmK) / 4);
#pragma unroll
  for (int i = 0; i < NK; ++i) {
    constexpr int H = 4;  // start[4]
    const int x = H + P * NK + i;
    w[i] = (uint32_t)__builtin_amdgcn_readlane((int)v[x >> 6], x & 63);
  }
}
constexpr int kGroupWords = (int)(sizeof(GemmG) / 4), kGroupVregs = (kGroupWords + 63) / 64;
__device__ __forceinline__ void load_group_words(const GemmG& in, uint32_t (&v)[kGroupVregs]) {
  static_assert(sizeof(GemmK) % 4 == 0 && sizeof(GemmG) % 4 == 0, "dword structs");
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&in);
  const int lane = (int)(threadIdx.x & 63);
#pragma unroll
  for (int r = 0; r < kGroupVregs; ++r)
    v[r] = src[lane + 64 * r < kGroupWords ? lane + 64 * r : kGroupWords - 1];
}
__device__ __forceinline__ uint32_t group_word(const uint32_t (&v)[kGroupVregs], int i) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v[0], i);
}
// problem p's descriptor (p wave-uniform)
__device__ __forceinline__ GemmK pick(const uint32_t (&v)[kGroupVregs], int p) {
  constexpr int NK = (int)(sizeof(GemmK) / 4);
  union U {
    GemmK t;
    uint32_t w[NK];
    __device__ U() {}
  } u;
  if constexpr (kGroupMax >= 3) {
    if (p == 2) { pick_problem<2>(v, u.w); return u.t; }
  }
  if constexpr (kGroupMax >= 2) {
    if (p == 1) { pick_problem<1>(v, u.w); return u.t; }
  }
  pick_problem<0>(v, u.w);
  return u.t;
}
// this workgroup's problem, its workgroup index within the problem's slice and the slice size
__device__ __forceinline__ int group_slot(const uint32_t (&v)[kGroupVregs], uint32_t& lbid, uint32_t& lnwg) {
  const uint32_t s1 = group_word(v, 1), s2 = group_word(v, 2), s3 = group_word(v, 3);
  const uint32_t bid = blockIdx.x;
  if (bid >= s2) { lbid = bid - s2; lnwg = s3 - s2; return 2; }
  if (bid >= s1) { lbid = bid - s1; lnwg = s2 - s1; return 1; }
  lbid = bid; lnwg = s1;
  return 0;
}
__device__ __forceinline__ GemmK load_group(const GemmG& in, uint32_t& lbid, uint32_t& lnwg) {
  uint32_t v[kGroupVregs];
  load_group_words(in, v);
  return pick(v, group_slot(v, lbid, lnwg));
}


__device__ __forceinline__ void epilogue_store(const GemmK& g, int zb, int m, int n, float v) {
  if (n == g.nload) {  // the column-sum column (only exists with ones_out)
    g.ones_out[(int64_t)m * g.ones_stride] = v * g.alpha;
    return;
  }
  const int64_t zo = zoff(g.cz, zb);
  const int32_t o = koff(g.cm, m) + koff(g.cn, n);
  v *= g.alpha;
  if (g.beta != 0.f) v += g.beta * g.C[zo + o];
  if (g.bias) v += g.bias[n * g.bias_stride];
  if (g.relu) v = fmaxf(v, 0.f);
  if (g.emask) v = g.emask[zo + o] > 0.f ? v : 0.f;
  if (g.omap) {
    float* d = g.Cout + zoff(g.oz, zb) + koff(g.om, m) + koff(g.on, n);
    *d = g.obeta != 0.f ? v + g.obeta * *d : v;
    return;
  }
  (g.Cout ? g.Cout : g.C)[zo + o] = v;
}

struct TileCoord {
  int m0, n0, zb, sp;
};
// XCD-aware tile order (1-D grid): the dispatcher deals consecutive workgroup ids
// round-robin over the 8 XCDs, so id%8 labels the blocks sharing one L2.  Give each
// such group a contiguous run of tiles, the small operand's index fastest, so the
// blocks that re-read one panel of the big operand sit behind the same L2.
// Bijective for any count.
template <int BM, int BN>
__device__ __forceinline__ TileCoord decode_tile(const GemmK& g, uint32_t bid, uint32_t nwg, bool& idle) {
  const uint32_t q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const uint32_t t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  idle = t >= g.count;  // padding of the problem's grid slice
  const uint32_t gn = g.tiles_n, gm = g.tiles_m;
  const uint32_t tf = g.n_fast ? gn : gm, ts = g.n_fast ? gm : gn;
  const uint32_t f = t % tf, tr = t / tf, sl = tr % ts;
  TileCoord c;
  c.n0 = (int)(g.n_fast ? f : sl) * BN;
  c.m0 = (int)(g.n_fast ? sl : f) * BM;
  const int zz = (int)(tr / ts);
  c.zb = zz / g.splitk;
  c.sp = zz % g.splitk;
  return c;
}

// --- epilogue: C/D layout col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
// Row offsets: a single-level row map (d = 2^31, the common case) gives row r's offset as the
// lane's base row offset plus a compile-time multiple of the uniform stride (one scalar
// multiply, one add), instead of a full koff (three 32-bit vector multiplies and a high
// multiply) per row; split-K slab offsets likewise from one 64-bit base per accumulator.
__device__ __forceinline__ int rrow(int r) { return (r & 3) + 8 * (r >> 2); }
// OMAP: the output-map epilogue is compiled into the 64x64 tile's kernels only (the host plans
// every omap product on that tile): elsewhere its registers would cost occupancy
template <int WM, int WN, bool OMAP = false>
__device__ __forceinline__ void gemm_epilogue(const GemmK& g, const TileCoord& c, int wrow0, int wcol0, int lane,
                                              floatx16 (&acc)[WM][WN]) {
  const int lr = lane & 31, lk = lane >> 5;
  const bool reads = g.splitk == 1 && (g.beta != 0.f || g.emask);
  const bool cm1 = g.cm.d == 0x80000000u;  // single-level row map (uniform)
  const int64_t zo = zoff(g.cz, c.zb);
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int n = c.n0 + wcol0 + j * 32 + lr;
      if (n >= g.N) continue;
      const int mb = c.m0 + wrow0 + i * 32 + 4 * lk;  // row of r = 0
      if (n == g.nload) {  // column-sum column
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mb + rrow(r);
          if (m >= g.M) continue;
          if (g.splitk > 1) g.ws[(((int64_t)c.zb * g.splitk + c.sp) * g.M + m) * g.N + n] = acc[i][j][r];
          else epilogue_store(g, c.zb, m, n, acc[i][j][r]);
        }
        continue;
      }
      if (g.splitk > 1) {
        float* wsp = g.ws + (((int64_t)c.zb * g.splitk + c.sp) * g.M + mb) * g.N + n;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (mb + rrow(r) < g.M) wsp[(int64_t)rrow(r) * g.N] = acc[i][j][r];
        continue;
      }
      const int32_t no = koff(g.cn, n);
      const int32_t mob = cm1 ? mb * g.cm.s0 : 0;
      auto mo = [&](int r) -> int32_t { return cm1 ? mob + rrow(r) * g.cm.s0 : koff(g.cm, mb + rrow(r)); };
      if (OMAP && g.omap) {
        // Cout with its own maps (no ReLU / mask here; the host keeps every 32-row fragment
        // inside one period of a two-level row map, so row r sits at a fixed stride from the
        // fragment's first row): beta * C and obeta * the old Cout, all loads before the
        // first store, as below
        const int64_t ozo = zoff(g.oz, c.zb) + koff(g.on, n) + koff(g.om, c.m0 + wrow0 + i * 32) + 4 * lk * g.om.s0;
        float cin[16], ob[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = min(mb + rrow(r), g.M - 1);
          cin[r] = g.beta != 0.f ? g.C[zo + (cm1 ? mob + (m - mb) * g.cm.s0 : koff(g.cm, m)) + no] : 0.f;
          ob[r] = g.obeta != 0.f && mb + rrow(r) < g.M ? g.Cout[ozo + rrow(r) * g.om.s0] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (mb + rrow(r) >= g.M) continue;
          float v = acc[i][j][r] * g.alpha + g.beta * cin[r];
          if (g.bias) v += g.bias[n * g.bias_stride];
          g.Cout[ozo + rrow(r) * g.om.s0] = v + g.obeta * ob[r];
        }
        continue;
      }
      float* dst = g.Cout ? g.Cout : g.C;
      if (reads) {
        // beta * C and the ReLU mask: all 16 loads issued before the first store (the
        // stores may alias C, so element-wise load/store pairs would serialise 16 memory
        // round trips per lane)
        float cin[16], em[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = min(mb + rrow(r), g.M - 1);
          const int64_t o = zo + (cm1 ? mob + (m - mb) * g.cm.s0 : koff(g.cm, m)) + no;
          cin[r] = g.beta != 0.f ? g.C[o] : 0.f;
          em[r] = g.emask ? g.emask[o] : 1.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (mb + rrow(r) >= g.M) continue;
          float v = acc[i][j][r] * g.alpha + g.beta * cin[r];
          if (g.bias) v += g.bias[n * g.bias_stride];
          if (g.relu) v = fmaxf(v, 0.f);
          if (em[r] <= 0.f) v = 0.f;
          dst[zo + mo(r) + no] = v;
        }
        continue;
      }
      const float bv = g.bias ? g.bias[n * g.bias_stride] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (mb + rrow(r) >= g.M) continue;
        float v = acc[i][j][r] * g.alpha;
        if (g.bias) v += bv;
        if (g.relu) v = fmaxf(v, 0.f);
        dst[zo + mo(r) + no] = v;
      }
    }
}

// ---------------------------------------------------------------------------------
// LDS-DMA pipeline (global_load_lds_dword / _dwordx4): the operands go global -> LDS with
// no VGPR staging and no ds_write pass, two or three LDS stages deep (the next tile(s) in
// flight while tile t is multiplied).  The DMA image is lane-linear per wave instruction,
// so the layouts are chosen per operand orientation:
//   m-contiguous operand (A not A_KC, B B_NC): image [BK][BM] (k rows of BM floats); a
//     wave instruction reads 64 consecutive m at one k (coalesced); fragments are
//     ds_read_b32 at (k, m = lane&31), conflict-free.
//   k-contiguous operand: image [BM][BK] with the 4-float quads of row m XOR-swizzled by
//     (m>>1)&7; the swizzle is applied on the SOURCE address (lane l of an instruction
//     fetches the k that belongs in slot l), fragments are ds_read_b128, conflict-free.
// Ordering: tile t's DMAs are retired by a counted vmcnt (tile t+1 stays in flight), then a
// raw s_barrier makes them visible to every wave and proves every wave has finished
// reading the stage that tile t+2 will overwrite.  No __syncthreads in the loop: its
// fence would drain the in-flight DMAs (vmcnt(0)).
// ---------------------------------------------------------------------------------
__device__ float g_zero_page[64];  // k >= K lanes of the last tile fetch zeros from here

// The DMA is issued from inline asm, not __builtin_amdgcn_global_load_lds: with the
// builtin, hipcc's waitcnt pass cannot tell the fragment ds_reads of stage t from the DMA
// in flight into stage t+2 and drains it (vmcnt(0)) before every read.  The asm saves and
// restores M0 (compiler-owned); all ordering is by the explicit waits + barrier below.
// four DMAs into consecutive 1 KiB LDS slots under one M0: the instruction offset moves
// both the LDS destination and the global source (probed: tools/glds_probe.hip), so the
// VGPR offsets carry -1024*i and the SGPR base is pre-lowered by 4 KiB to keep them >= 0.
// wave-uniform values for the SGPR operands of the DMA asm (the compiler may keep a uniform
// value in a VGPR after the per-problem branch of load_group; readfirstlane is free when not)
__device__ __forceinline__ const float* sgpr_ptr(const float* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return reinterpret_cast<const float*>(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t sgpr_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

__device__ __forceinline__ void glds4_saddr(const float* base_m4k, uint32_t o0, uint32_t o1, uint32_t o2,
                                            uint32_t o3, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, %5\n\t"
      "global_load_lds_dword %2, %5 offset:1024\n\t"
      "global_load_lds_dword %3, %5 offset:2048\n\t"
      "global_load_lds_dword %4, %5 offset:3072\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"((o0 << 2) + 4096u), "v"((o1 << 2) + 3072u), "v"((o2 << 2) + 2048u), "v"((o3 << 2) + 1024u),
        "s"(sgpr_ptr(base_m4k)), "s"(sgpr_u32(lds_addr))
      : "memory");
}
__device__ __forceinline__ void glds_vaddr(const void* p, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(p), "s"(sgpr_u32(lds_addr))
      : "memory");
}
__device__ __forceinline__ uint32_t lds_addr_of(const float* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>(p);  // low 32 bits of a shared-aperture address
}

template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  // gfx9 s_waitcnt: vmcnt[3:0] | expcnt[6:4] (7 = no wait) | lgkmcnt[11:8] | vmcnt[5:4] << 14
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (0 << 8) | ((N >> 4) << 14));
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// one 16-B-per-lane DMA: 1 KiB per wave instruction into LDS at M0 (wave-uniform) + 16*lane
__device__ __forceinline__ void glds16_saddr(const float* base, uint32_t off_bytes, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(off_bytes), "s"(sgpr_ptr(base)), "s"(sgpr_u32(lds_addr))
      : "memory");
}

// Operand images (per stage): A [BM][BK] (A_KC, quads XOR-swizzled) or [BK][BM]; B [BN][BK]
// (!B_NC, swizzled) or [BK][BN].  Image position p <-> (row, k) by the same formula for both
// DMA widths, so the MFMA side never knows which width filled a stage.
//   V = 1: thread tid, instruction j fills position 256 j + 64 wave + lane (4 B per lane);
//   V = 4: instruction J fills positions 1024 J + 256 wave + 4 lane .. +3 (16 B per lane):
//          4x fewer DMA instructions per k-tile (the per-lane address rate of the
//          load path, not the bytes, bounds the 4-B form).  The host picks V = 4 where the
//          four elements of every quad are contiguous and 16-B aligned (dma_width).
// The last, partial k-tile always goes element by element (V = 1 form, zeros past K).
template <int ROWS, bool KMAJ>
__device__ __forceinline__ void img_rk(int p, int& row, int& k) {
  constexpr int BK = 32;
  if (KMAJ) {  // [row][BK], quads swizzled by (row >> 1) & 7
    row = p / BK;
    const int sl = p % BK;
    k = ((((sl >> 2) ^ ((row >> 1) & 7)) << 2) | (sl & 3));
  } else {     // [BK][ROWS]
    k = p / ROWS;
    row = p % ROWS;
  }
}

// ACC2: two-level fp32 accumulation for long reductions — each k-tile's 32 products go into a
// fresh tile accumulator, which is then added to the running one, so no fp32 chain is longer
// than 32 + K/32 additions (a single MFMA chain over K = 5.8K lost 1e-3 of a cancelling weight
// gradient against the fp64 oracle).  +16 VGPRs per accumulator: only for long K per workgroup.
template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, bool KTWO, int VA, int VB, bool BF, bool KCAT = false,
          bool ACC2 = false>
__device__ __forceinline__ void gemm_glds_body(const GemmG& gin) {
  constexpr int BK = 32;
  stream_sig_store(gin.sig, gin.sig_v);
  constexpr int BM = 32 * WM * WGM, BN = 32 * WN * WGN;
  constexpr int NA = BM * BK / (256 * VA), NB = BN * BK / (256 * VB);  // DMA instructions per thread per k-tile
  constexpr int LA1 = BM * BK / 256, LB1 = BN * BK / 256;              // element DMAs of the partial tile
  static_assert(NA + NB < 64 && LA1 % 4 == 0 && LB1 % 4 == 0, "vmcnt range / DMA batches");

  uint32_t gv[kGroupVregs];
  load_group_words(gin, gv);
  uint32_t lbid, lnwg;
  const GemmK g = pick(gv, group_slot(gv, lbid, lnwg));
  bool idle;
  const TileCoord tc = decode_tile<BM, BN>(g, lbid, lnwg, idle);
  if (idle) return;  // uniform over the workgroup, before any barrier
  // two LDS stages, compile-time (static LDS: the stage addresses fold into the ds_read /
  // M0 immediates; a runtime stage count cost ~10 % of the GEMM family, measured)
#ifndef DSTAGNN_GEMM_NS
#define DSTAGNN_GEMM_NS 2
#endif
  // LDS stages (compile-time: the stage addresses fold into immediates); deeper rings for the
  // tiles whose ring still fits 64 KB
  constexpr int NS = (BM + BN) * BK * 4 * DSTAGNN_GEMM_NS <= 65536 ? DSTAGNN_GEMM_NS : 2;
  // the pipelined K loop (three stages, barrier before the last MFMA step; DSTAGNN_GEMM_PIPE=1)
#ifndef DSTAGNN_GEMM_PIPE
#define DSTAGNN_GEMM_PIPE 0
#endif
  constexpr bool PIPE = DSTAGNN_GEMM_PIPE && NS == 3 && !BF;
  constexpr int FT = NA + NB, PT = LA1 + LB1;  // DMA instructions of a full / the partial k-tile
  static_assert(NS >= 2 && NS <= 4, "LDS ring of 2..4 stages");
  __shared__ __attribute__((aligned(16))) float Asm[NS * BM * BK];
  __shared__ __attribute__((aligned(16))) float Bsm[NS * BN * BK];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WGN, wc = wid % WGN;
  // lane half h (lane >> 5) supplies k = 16 h + s at MFMA step s (A and B agree)
  const int lr = lane & 31, lk = lane >> 5;
  const int arow0 = wr * 32 * WM, bcol0 = wc * 32 * WN;
  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // the K loop of one problem (of one K segment) into acc
  auto kseg = [&](const GemmK& g) {
  const int kbeg = tc.sp * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const float* A = g.A + zoff(g.az, tc.zb);
  const float* Bp = g.B + zoff(g.bz, tc.zb);

  // per-instruction element coordinates and offsets (row part + the in-tile k part for
  // single-level k maps: one add per instruction per k-tile)
  int a_kl[NA], b_kl[NB];
  uint32_t ao[NA], bo[NB];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    int row, k;
    img_rk<BM, A_KC>(VA == 4 ? 1024 * j + 256 * wid + 4 * lane : 256 * j + 64 * wid + lane, row, k);
    a_kl[j] = k;
    const int m = tc.m0 + row;
    ao[j] = (uint32_t)g.abias + (m < g.M ? (uint32_t)koff(g.am, m) : 0u);  // clamped rows are never stored
    if (!KTWO) ao[j] += (uint32_t)(k * g.ak.s0);
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    int col, k;
    img_rk<BN, !B_NC>(VB == 4 ? 1024 * j + 256 * wid + 4 * lane : 256 * j + 64 * wid + lane, col, k);
    b_kl[j] = k;
    const int n = tc.n0 + col;
    bo[j] = (uint32_t)g.bbias + (n < g.nload ? (uint32_t)koff(g.bn, n) : 0u);
    if (!KTWO) bo[j] += (uint32_t)(k * g.bk.s0);
  }
  auto aoff = [&](int j, int k0) -> uint32_t {
    return KTWO ? ao[j] + (uint32_t)koff(g.ak, k0 + a_kl[j]) : ao[j] + (uint32_t)(k0 * g.ak.s0);
  };
  auto boff = [&](int j, int k0) -> uint32_t {
    return KTWO ? bo[j] + (uint32_t)koff(g.bk, k0 + b_kl[j]) : bo[j] + (uint32_t)(k0 * g.bk.s0);
  };
  auto gp = [](const float* base, uint32_t off) -> const void* {
    return reinterpret_cast<const char*>(base) + (size_t)(off << 2);
  };
  auto issue = [&](int k0, int st) {
    const uint32_t sa = lds_addr_of(Asm + st * BM * BK);
    const uint32_t sb = lds_addr_of(Bsm + st * BN * BK);
    if (k0 + BK <= kend) {
      if constexpr (VA == 4) {
#pragma unroll
        for (int j = 0; j < NA; ++j) glds16_saddr(A, aoff(j, k0) << 2, sa + 4 * (1024 * j + 256 * wid));
      } else {
#pragma unroll
        for (int j = 0; j < NA; j += 4)
          glds4_saddr(A - 1024, aoff(j, k0), aoff(j + 1, k0), aoff(j + 2, k0), aoff(j + 3, k0),
                      sa + 4 * (256 * j + 64 * wid));
      }
      if constexpr (VB == 4) {
#pragma unroll
        for (int j = 0; j < NB; ++j) glds16_saddr(Bp, boff(j, k0) << 2, sb + 4 * (1024 * j + 256 * wid));
      } else {
#pragma unroll
        for (int j = 0; j < NB; j += 4)
          glds4_saddr(Bp - 1024, boff(j, k0), boff(j + 1, k0), boff(j + 2, k0), boff(j + 3, k0),
                      sb + 4 * (256 * j + 64 * wid));
      }
    } else {  // partial tile: element by element, zeros past kend
      // (from the loop-invariant start of the last tile, not k0: with k0 the compiler keeps
      // every element's k as an induction variable, +32 VALU adds per k-tile iteration)
      int kt = kbeg + (kend - kbeg - 1) / BK * BK;
      // opaque here, so the partial tile's ~32 index-map evaluations (about a hundred 32-bit
      // vector multiplies) are not hoisted into every workgroup's prologue by LICM: only the
      // workgroups that reach a partial tile pay them
      asm volatile("" : "+s"(kt));
#pragma unroll
      for (int j = 0; j < LA1; ++j) {
        int row, k;
        img_rk<BM, A_KC>(256 * j + 64 * wid + lane, row, k);
        const int m = tc.m0 + row;
        const uint32_t o = (uint32_t)g.abias + (m < g.M ? (uint32_t)koff(g.am, m) : 0u) + (uint32_t)koff(g.ak, kt + k);
        glds_vaddr(kt + k < kend ? gp(A, o) : (const void*)g_zero_page, sa + 4 * (256 * j + 64 * wid));
      }
#pragma unroll
      for (int j = 0; j < LB1; ++j) {
        int col, k;
        img_rk<BN, !B_NC>(256 * j + 64 * wid + lane, col, k);
        const int n = tc.n0 + col;
        const uint32_t o = (uint32_t)g.bbias + (n < g.nload ? (uint32_t)koff(g.bn, n) : 0u) + (uint32_t)koff(g.bk, kt + k);
        glds_vaddr(kt + k < kend ? gp(Bp, o) : (const void*)g_zero_page, sb + 4 * (256 * j + 64 * wid));
      }
    }
  };

  const int ntiles = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const bool ones_tile = g.nload < g.N && tc.n0 + BN > g.nload;  // uniform
  // fragments: lane half lk supplies k = 16 lk + 4 q + c (c = 0..3) at step q (A and B agree)
  auto read_a_st = [&](const float* as, int i, int q, float* v4) {
    const int m = arow0 + i * 32 + lr;
    if (A_KC) {
      const int pq = (lk * 4 + q) ^ ((m >> 1) & 7);
      const float4 v = *reinterpret_cast<const float4*>(as + m * BK + pq * 4);
      v4[0] = v.x; v4[1] = v.y; v4[2] = v.z; v4[3] = v.w;
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) v4[c] = as[(lk * 16 + q * 4 + c) * BM + m];
    }
  };
  auto read_b_st = [&](const float* bs, int j, int q, float* v4) {
    const int n = bcol0 + j * 32 + lr;
    if (!B_NC) {
      const int pq = (lk * 4 + q) ^ ((n >> 1) & 7);
      const float4 v = *reinterpret_cast<const float4*>(bs + n * BK + pq * 4);
      v4[0] = v.x; v4[1] = v.y; v4[2] = v.z; v4[3] = v.w;
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) v4[c] = bs[(lk * 16 + q * 4 + c) * BN + n];
    }
  };
  if constexpr (PIPE) {
    // Pipelined K loop (three LDS stages, two tiles in flight): the wait + barrier that
    // publishes tile t+1 sits BEFORE tile t's last MFMA step, and tile t+1's first two
    // fragment steps are read behind it, so the LDS-read latency at a tile start and the
    // barrier skew overlap tile t's last four MFMAs instead of idling the matrix pipe.
    //   iteration t: issue tile t+2 -> stage (t+2)%3 (last read in iteration t-1, whose
    //   fragments were all read and waited for before that iteration's barrier); MFMA steps
    //   0..2 of tile t beside the reads of its steps 2, 3; lgkmcnt(0); vmcnt(tile t+2's DMAs)
    //   + s_barrier; reads of tile t+1 steps 0, 1; MFMA step 3 of tile t.
    static_assert(NS == 3 && !BF, "pipelined loop: three stages, fp32");
    if (ntiles == 0) return;
    const bool lastp = (kend - kbeg) % BK != 0;
    // retire every DMA but those of tile `younger` (which may still be in flight), then barrier
    auto retire = [&](int younger) {
      if (younger >= ntiles) wait_vm_barrier<0>();
      else if (younger == ntiles - 1 && lastp) wait_vm_barrier<PT>();
      else wait_vm_barrier<FT>();
    };
    auto ones_fix = [&](int stg) {
      if (ones_tile) {  // column-sum column: B = 1 in this stage's image (see the plain loop)
        float* bst = Bsm + stg * BN * BK;
        const int c = g.nload - tc.n0;
        if (tid < BK) bst[B_NC ? tid * BN + c : c * BK + tid] = 1.f;
        __syncthreads();
      }
    };
    float fa[4][WM][4], fb[4][WN][4];
    auto read_step = [&](int stg, int q) {
      const float* as = Asm + stg * BM * BK;
      const float* bs = Bsm + stg * BN * BK;
#pragma unroll
      for (int i = 0; i < WM; ++i) read_a_st(as, i, q, fa[q][i]);
#pragma unroll
      for (int j = 0; j < WN; ++j) read_b_st(bs, j, q, fb[q][j]);
    };
    floatx16 tacc[WM][WN];
    auto mfma_step = [&](int q) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) {
            if constexpr (ACC2)
              tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q][i][c], fb[q][j][c], (q | c) ? tacc[i][j] : zero_acc(),
                                                               0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q][i][c], fb[q][j][c], acc[i][j], 0, 0, 0);
          }
    };
    issue(kbeg, 0);
    if (ntiles > 1) issue(kbeg + BK, 1);
    retire(1);
    ones_fix(0);
    read_step(0, 0);
    read_step(0, 1);
    int st = 0;
    for (int t = 0; t < ntiles; ++t) {
      const int st1 = st == 2 ? 0 : st + 1, st2 = st1 == 2 ? 0 : st1 + 1;
      if (t + 2 < ntiles) issue(kbeg + (t + 2) * BK, st2);
      read_step(st, 2);
      mfma_step(0);
      read_step(st, 3);
      mfma_step(1);
      mfma_step(2);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < ntiles) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this stage's reads are complete
        retire(t + 2);
        ones_fix(st1);
        read_step(st1, 0);
        read_step(st1, 1);
        __builtin_amdgcn_sched_barrier(0);
      }
      mfma_step(3);
      if constexpr (ACC2) {
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) acc[i][j] += tacc[i][j];
      }
      st = st1;
    }
    return;
  }
  for (int s0 = 0; s0 < NS - 1; ++s0)
    if (s0 < ntiles) issue(kbeg + s0 * BK, s0);
  int st = 0;
  for (int t = 0; t < ntiles; ++t) {
    // retire tile t: the DMAs of the (up to NS - 2) younger tiles issued so far stay in flight
    if constexpr (NS == 2) {
      wait_vm_barrier<0>();
    } else {
      const int young = min(NS - 2, ntiles - 1 - t);
      const bool lastp = (kend - kbeg) % BK != 0;  // the last k-tile is the partial one
      if (young <= 0) wait_vm_barrier<0>();
      else if (young == 1) {
        if (t + 1 == ntiles - 1 && lastp) wait_vm_barrier<PT>();
        else wait_vm_barrier<FT>();
      } else {
        if constexpr (NS >= 4) {
          if (t + 2 == ntiles - 1 && lastp) wait_vm_barrier<FT + PT>();
          else wait_vm_barrier<2 * FT>();
        }
      }
    }
    if (ones_tile) {
      // column-sum column: B = 1 in this stage's image (A is 0 past K); written after the
      // DMA landed, read after one more barrier (only the tile column that holds it pays)
      float* bst = Bsm + st * BN * BK;
      const int c = g.nload - tc.n0;
      if (tid < BK) bst[B_NC ? tid * BN + c : c * BK + tid] = 1.f;
      __syncthreads();
    }
    if (t + NS - 1 < ntiles) issue(kbeg + (t + NS - 1) * BK, st == 0 ? NS - 1 : st - 1);
    const float* as = Asm + st * BM * BK;
    const float* bs = Bsm + st * BN * BK;
    // fragments: lane half lk supplies k = 16 lk + 4 q + c (c = 0..3) at step q (A and B agree)
    auto read_a = [&](int i, int q, float* v4) {
      const int m = arow0 + i * 32 + lr;
      if (A_KC) {
        const int pq = (lk * 4 + q) ^ ((m >> 1) & 7);
        const float4 v = *reinterpret_cast<const float4*>(as + m * BK + pq * 4);
        v4[0] = v.x; v4[1] = v.y; v4[2] = v.z; v4[3] = v.w;
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) v4[c] = as[(lk * 16 + q * 4 + c) * BM + m];
      }
    };
    auto read_b = [&](int j, int q, float* v4) {
      const int n = bcol0 + j * 32 + lr;
      if (!B_NC) {
        const int pq = (lk * 4 + q) ^ ((n >> 1) & 7);
        const float4 v = *reinterpret_cast<const float4*>(bs + n * BK + pq * 4);
        v4[0] = v.x; v4[1] = v.y; v4[2] = v.z; v4[3] = v.w;
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) v4[c] = bs[(lk * 16 + q * 4 + c) * BN + n];
      }
    };
    if constexpr (BF) {
      // bf16 operands (rounded to nearest even), fp32 accumulate: steps q, q+1 form the 8
      // elements of one v_mfma_f32_32x32x16_bf16 (element e of lane half lk <-> the same k
      // in A and B, so the k permutation cancels)
#pragma unroll
      for (int q = 0; q < BK / 8; q += 2) {
        bf16x8 af[WM], bfr[WN];
#pragma unroll
        for (int i = 0; i < WM; ++i) {
          float v[8];
          read_a(i, q, v);
          read_a(i, q + 1, v + 4);
#pragma unroll
          for (int e = 0; e < 8; ++e) af[i][e] = (__bf16)v[e];
        }
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          float v[8];
          read_b(j, q, v);
          read_b(j, q + 1, v + 4);
#pragma unroll
          for (int e = 0; e < 8; ++e) bfr[j][e] = (__bf16)v[e];
        }
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
      // every fragment of the k-tile first (ds_reads complete in order: the MFMAs of step q
      // wait only for step q's reads), then the 16 MFMAs per accumulator
      float av[BK / 8][WM][4], bv[BK / 8][WN][4];
#pragma unroll
      for (int q = 0; q < BK / 8; ++q) {
#pragma unroll
        for (int i = 0; i < WM; ++i) read_a(i, q, av[q][i]);
#pragma unroll
        for (int j = 0; j < WN; ++j) read_b(j, q, bv[q][j]);
      }
      if constexpr (ACC2) {
        floatx16 tacc[WM][WN];
#pragma unroll
        for (int q = 0; q < BK / 8; ++q)
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
              for (int j = 0; j < WN; ++j)
                tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q][i][c], bv[q][j][c],
                                                                 (q | c) ? tacc[i][j] : zero_acc(), 0, 0, 0);
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) acc[i][j] += tacc[i][j];
      } else {
#pragma unroll
      for (int q = 0; q < BK / 8; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int i = 0; i < WM; ++i)
#pragma unroll
            for (int j = 0; j < WN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q][i][c], bv[q][j][c], acc[i][j], 0, 0, 0);
      }
      // software-pipeline the k-tile by one step: the reads of steps 0 and 1, then the MFMAs of
      // step q beside the reads of step q + 2 (DS reads per step: b128 per row-major operand,
      // two read2 pairs per column-major one)
      constexpr int DSQ = (A_KC ? WM : 2 * WM) + (!B_NC ? WN : 2 * WN);
      constexpr int MFQ = 4 * WM * WN;
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * DSQ, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, MFQ, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, DSQ, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, MFQ, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, DSQ, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * MFQ, 0);
    }
    st = st == NS - 1 ? 0 : st + 1;
  }
  };
  if constexpr (KCAT) {
    // K-concatenated segments (a separate instantiation: the runtime descriptor choice costs
    // the plain kernel about twice the VGPRs)
    const int nseg = (int)group_word(gv, 0);
    for (int p = 0; p < nseg; ++p) {
      if (p) __syncthreads();  // every wave is done with the LDS stages before the next segment's DMA
      kseg(p ? pick(gv, p) : g);
    }
  } else {
    kseg(g);
  }
  gemm_epilogue<WM, WN, WGM == 2 && WGN == 2 && WM == 1 && WN == 1 && !KCAT>(g, tc, arow0, bcol0, lane, acc);
}

// ---------------------------------------------------------------------------------
// Persistent tile loop (gemm_persist_body).  For GEMMs that do not split K, every output tile
// of the plain kernel pays a fixed cost the 6-30 k-tiles behind it do not amortise: the
// argument fetch and tile decode, the first DMA round trip (~1 us under load) with the matrix
// pipe idle, and the epilogue's stores.  Here a grid of about one workgroup per CU walks the
// problem's tiles instead: workgroup (XCD x, index r) takes a contiguous run of the XCD's
// eighth of the tile order (the same XCD-local order as decode_tile), and ONE three-stage
// DMA / MFMA stream runs over the flattened (tile, k-tile) sequence of the run — the next
// tile's first k-tiles are in flight while the current tile finishes, and its epilogue stores
// drain behind the next tile's MFMAs.  The k loop is the pipelined one of gemm_glds_body
// (PIPE: the barrier that publishes k-tile i+1 sits before k-tile i's last MFMA step, i+1's
// first fragment steps are read behind it).  K-concatenated problems (run_gemm_kcat) walk
// their segments in turn inside every tile.  No split-K, no column-sum column, fp32.
// ---------------------------------------------------------------------------------
template <int I>
__device__ __forceinline__ uint32_t gword(const uint32_t (&v)[kGroupVregs]) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v[I >> 6], I & 63);
}
// K of problem / segment p (wave-uniform p <= 2)
__device__ __forceinline__ int seg_k(const uint32_t (&v)[kGroupVregs], int p) {
  constexpr int NK = (int)(sizeof(GemmK) / 4), OK = (int)(offsetof(GemmK, K) / 4);
  if constexpr (kGroupMax >= 3) {
    if (p == 2) return (int)gword<4 + 2 * NK + OK>(v);
  }
  if constexpr (kGroupMax >= 2) {
    if (p == 1) return (int)gword<4 + NK + OK>(v);
  }
  return (int)gword<4 + OK>(v);
}

// retire every DMA but the newest n (a runtime count from a small set of sums of FT / PT)
template <int FT, int PT>
__device__ __forceinline__ void wait_vm_barrier_rt(int n) {
  if (n == 0) wait_vm_barrier<0>();
  else if (n == FT) wait_vm_barrier<FT>();
  else if (n == PT) wait_vm_barrier<PT>();
  else if (n == 2 * FT) wait_vm_barrier<(2 * FT < 64 ? 2 * FT : 0)>();
  else if (n == FT + PT) wait_vm_barrier<(FT + PT < 64 ? FT + PT : 0)>();
  else if (n == 2 * PT) wait_vm_barrier<(2 * PT < 64 ? 2 * PT : 0)>();
  else wait_vm_barrier<0>();  // (never: n is one of the above) the safe over-wait
}

// PNS: LDS stages (PNS - 1 k-tiles in flight); the stage ring lives in ONE dynamic LDS array
template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, bool KTWO, int VA, int VB, bool KCAT, int PNS>
__device__ __forceinline__ void gemm_persist_body(const GemmG& gin) {
  constexpr int BK = 32, NS = PNS;
  stream_sig_store(gin.sig, gin.sig_v);
  constexpr int BM = 32 * WM * WGM, BN = 32 * WN * WGN;
  constexpr int NA = BM * BK / (256 * VA), NB = BN * BK / (256 * VB);
  constexpr int LA1 = BM * BK / 256, LB1 = BN * BK / 256;
  constexpr int FT = NA + NB, PT = LA1 + LB1;
  static_assert(NA + NB < 64 && LA1 % 4 == 0 && LB1 % 4 == 0, "vmcnt range / DMA batches");
  static_assert(NS >= 3 && NS <= 4 && (NS - 2) * (FT > PT ? FT : PT) < 64, "two or three stages in flight");
  static_assert((BM + BN) * BK * 4 * NS <= 160 * 1024, "persistent loop: the ring within the CU's LDS");
  extern __shared__ __attribute__((aligned(16))) float psmem[];
  float* const Asm = psmem;
  float* const Bsm = psmem + NS * BM * BK;

  uint32_t gv[kGroupVregs];
  load_group_words(gin, gv);
  uint32_t lbid, lnwg;
  const GemmK g = pick(gv, group_slot(gv, lbid, lnwg));  // tile geometry + epilogue (problem 0's for kcat)
  // this workgroup's run [u0, u1) of the tile order
  const uint32_t T = g.count, xcd = lbid & 7, nx = lnwg >> 3, r = lbid >> 3;
  const uint32_t X0 = (uint32_t)((uint64_t)T * xcd / 8), X1 = (uint32_t)((uint64_t)T * (xcd + 1) / 8);
  const uint32_t u0 = X0 + (uint32_t)((uint64_t)(X1 - X0) * r / nx);
  const uint32_t u1 = X0 + (uint32_t)((uint64_t)(X1 - X0) * (r + 1) / nx);
  if (u0 >= u1) return;  // uniform, before any barrier
  const int ntl = (int)(u1 - u0);
  auto coords = [&](int tl) {
    const uint32_t u = u0 + (uint32_t)tl;
    const uint32_t gn = g.tiles_n, gm = g.tiles_m;
    const uint32_t tf = g.n_fast ? gn : gm, ts = g.n_fast ? gm : gn;
    const uint32_t f = u % tf, tr = u / tf, sl = tr % ts;
    TileCoord c;
    c.n0 = (int)(g.n_fast ? f : sl) * BN;
    c.m0 = (int)(g.n_fast ? sl : f) * BM;
    c.zb = (int)(tr / ts);
    c.sp = 0;
    return c;
  };
  // k-tiles per segment (one segment unless K-concatenated)
  const int nseg = KCAT ? (int)group_word(gv, 0) : 1;
  int segk[3] = {0, 0, 0}, skt[3] = {0, 0, 0};
  segk[0] = KCAT ? seg_k(gv, 0) : g.K;
  if (KCAT) {
    if (nseg > 1) segk[1] = seg_k(gv, 1);
    if (nseg > 2) segk[2] = seg_k(gv, 2);
  }
#pragma unroll
  for (int p = 0; p < 3; ++p) skt[p] = (segk[p] + BK - 1) / BK;
  const int kts = skt[0] + skt[1] + skt[2];
  const int total = ntl * kts;
  if (kts == 0) return;  // K = 0 never reaches here (the host keeps such problems on the plain kernel)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WGN, wc = wid % WGN;
  const int lr = lane & 31, lk = lane >> 5;
  const int arow0 = wr * 32 * WM, bcol0 = wc * 32 * WN;

  // ---- DMA side: the descriptor, tile and row offsets of the k-tile being issued
  int dtl = -1, dp = -1;
  GemmK dg = g;
  TileCoord dtc = coords(0);
  const float* dA = nullptr;
  const float* dB = nullptr;
  int a_kl[NA], b_kl[NB];
  uint32_t ao[NA], bo[NB];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    int row, k;
    img_rk<BM, A_KC>(VA == 4 ? 1024 * j + 256 * wid + 4 * lane : 256 * j + 64 * wid + lane, row, k);
    a_kl[j] = k;
    ao[j] = 0;
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    int col, k;
    img_rk<BN, !B_NC>(VB == 4 ? 1024 * j + 256 * wid + 4 * lane : 256 * j + 64 * wid + lane, col, k);
    b_kl[j] = k;
    bo[j] = 0;
  }
  auto set_dma = [&](int tl, int p) {
    if (tl != dtl) dtc = coords(tl);
    if (KCAT && p != dp) dg = pick(gv, p);
    dtl = tl;
    dp = p;
    dA = dg.A + zoff(dg.az, dtc.zb);
    dB = dg.B + zoff(dg.bz, dtc.zb);
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      int row, k;
      img_rk<BM, A_KC>(VA == 4 ? 1024 * j + 256 * wid + 4 * lane : 256 * j + 64 * wid + lane, row, k);
      const int m = dtc.m0 + row;
      ao[j] = (uint32_t)dg.abias + (m < dg.M ? (uint32_t)koff(dg.am, m) : 0u);
      if (!KTWO) ao[j] += (uint32_t)(k * dg.ak.s0);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      int col, k;
      img_rk<BN, !B_NC>(VB == 4 ? 1024 * j + 256 * wid + 4 * lane : 256 * j + 64 * wid + lane, col, k);
      const int n = dtc.n0 + col;
      bo[j] = (uint32_t)dg.bbias + (n < dg.nload ? (uint32_t)koff(dg.bn, n) : 0u);
      if (!KTWO) bo[j] += (uint32_t)(k * dg.bk.s0);
    }
  };
  // segment / k-tile of flattened iteration it (within its tile)
  auto split_it = [&](int it, int& tl, int& p, int& kt) {
    tl = it / kts;
    int rr = it - tl * kts;
    p = 0;
    if (KCAT) {
      if (rr >= skt[0]) { rr -= skt[0]; p = 1; if (rr >= skt[1]) { rr -= skt[1]; p = 2; } }
    }
    kt = rr;
  };
  auto is_partial = [&](int it) {
    int tl, p, kt;
    split_it(it, tl, p, kt);
    const int K = p == 0 ? segk[0] : (p == 1 ? segk[1] : segk[2]);
    return kt == (K - 1) / BK && K % BK != 0;
  };
  auto issue_it = [&](int it, int st) {
    int tl, p, kt;
    split_it(it, tl, p, kt);
    if (tl != dtl || p != dp) set_dma(tl, p);
    const int kend = dg.K, k0 = kt * BK;
    const uint32_t sa = lds_addr_of(Asm + st * BM * BK);
    const uint32_t sb = lds_addr_of(Bsm + st * BN * BK);
    auto aoff = [&](int j) -> uint32_t {
      return KTWO ? ao[j] + (uint32_t)koff(dg.ak, k0 + a_kl[j]) : ao[j] + (uint32_t)(k0 * dg.ak.s0);
    };
    auto boff = [&](int j) -> uint32_t {
      return KTWO ? bo[j] + (uint32_t)koff(dg.bk, k0 + b_kl[j]) : bo[j] + (uint32_t)(k0 * dg.bk.s0);
    };
    if (k0 + BK <= kend) {
      if constexpr (VA == 4) {
#pragma unroll
        for (int j = 0; j < NA; ++j) glds16_saddr(dA, aoff(j) << 2, sa + 4 * (1024 * j + 256 * wid));
      } else {
#pragma unroll
        for (int j = 0; j < NA; j += 4)
          glds4_saddr(dA - 1024, aoff(j), aoff(j + 1), aoff(j + 2), aoff(j + 3), sa + 4 * (256 * j + 64 * wid));
      }
      if constexpr (VB == 4) {
#pragma unroll
        for (int j = 0; j < NB; ++j) glds16_saddr(dB, boff(j) << 2, sb + 4 * (1024 * j + 256 * wid));
      } else {
#pragma unroll
        for (int j = 0; j < NB; j += 4)
          glds4_saddr(dB - 1024, boff(j), boff(j + 1), boff(j + 2), boff(j + 3), sb + 4 * (256 * j + 64 * wid));
      }
    } else {  // partial k-tile: element by element, zeros past K (as gemm_glds_body)
      int kt0 = (kend - 1) / BK * BK;
      asm volatile("" : "+s"(kt0));
#pragma unroll
      for (int j = 0; j < LA1; ++j) {
        int row, k;
        img_rk<BM, A_KC>(256 * j + 64 * wid + lane, row, k);
        const int m = dtc.m0 + row;
        const uint32_t o = (uint32_t)dg.abias + (m < dg.M ? (uint32_t)koff(dg.am, m) : 0u) + (uint32_t)koff(dg.ak, kt0 + k);
        glds_vaddr(kt0 + k < kend ? reinterpret_cast<const char*>(dA) + (size_t)(o << 2) : (const void*)g_zero_page,
                   sa + 4 * (256 * j + 64 * wid));
      }
#pragma unroll
      for (int j = 0; j < LB1; ++j) {
        int col, k;
        img_rk<BN, !B_NC>(256 * j + 64 * wid + lane, col, k);
        const int n = dtc.n0 + col;
        const uint32_t o = (uint32_t)dg.bbias + (n < dg.nload ? (uint32_t)koff(dg.bn, n) : 0u) + (uint32_t)koff(dg.bk, kt0 + k);
        glds_vaddr(kt0 + k < kend ? reinterpret_cast<const char*>(dB) + (size_t)(o << 2) : (const void*)g_zero_page,
                   sb + 4 * (256 * j + 64 * wid));
      }
    }
  };
  // retire every DMA but those of iterations [first, first + NS - 2) (still in flight), then barrier
  auto dmas_of = [&](int it) { return it >= total ? 0 : (is_partial(it) ? PT : FT); };
  auto retire = [&](int first) {
    int n = dmas_of(first);
    if constexpr (NS >= 4) n += dmas_of(first + 1);
    wait_vm_barrier_rt<FT, PT>(n);
  };

  // ---- MFMA side
  floatx16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = zero_acc();
  float fa[4][WM][4], fb[4][WN][4];
  auto read_step = [&](int stg, int q) {
    const float* as = Asm + stg * BM * BK;
    const float* bs = Bsm + stg * BN * BK;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      const int m = arow0 + i * 32 + lr;
      if (A_KC) {
        const int pq = (lk * 4 + q) ^ ((m >> 1) & 7);
        const float4 v = *reinterpret_cast<const float4*>(as + m * BK + pq * 4);
        fa[q][i][0] = v.x; fa[q][i][1] = v.y; fa[q][i][2] = v.z; fa[q][i][3] = v.w;
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) fa[q][i][c] = as[(lk * 16 + q * 4 + c) * BM + m];
      }
    }
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int n = bcol0 + j * 32 + lr;
      if (!B_NC) {
        const int pq = (lk * 4 + q) ^ ((n >> 1) & 7);
        const float4 v = *reinterpret_cast<const float4*>(bs + n * BK + pq * 4);
        fb[q][j][0] = v.x; fb[q][j][1] = v.y; fb[q][j][2] = v.z; fb[q][j][3] = v.w;
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) fb[q][j][c] = bs[(lk * 16 + q * 4 + c) * BN + n];
      }
    }
  };
  auto mfma_step = [&](int q) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q][i][c], fb[q][j][c], acc[i][j], 0, 0, 0);
  };

#pragma unroll
  for (int q = 0; q < NS - 1; ++q)
    if (q < total) issue_it(q, q);
  retire(1);
  read_step(0, 0);
  read_step(0, 1);
  TileCoord ctc = coords(0);
  int st = 0, tl = 0, kin = 0;  // compute side: stage, tile of the run, iteration within the tile
  for (int it = 0; it < total; ++it) {
    const int st1 = st == NS - 1 ? 0 : st + 1;
    const int stn = st == 0 ? NS - 1 : st - 1;  // the stage of iteration it - 1 = it + NS - 1
    if (it + NS - 1 < total) issue_it(it + NS - 1, stn);
    read_step(st, 2);
    mfma_step(0);
    read_step(st, 3);
    mfma_step(1);
    mfma_step(2);
    __builtin_amdgcn_sched_barrier(0);
    if (it + 1 < total) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this stage's fragment reads are complete
      retire(it + 2);
      read_step(st1, 0);
      read_step(st1, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    mfma_step(3);
    st = st1;
    if (++kin == kts) {  // the tile is complete: its epilogue, then the next tile
      gemm_epilogue<WM, WN>(g, ctc, arow0, bcol0, lane, acc);
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) acc[i][j] = zero_acc();
      kin = 0;
      if (++tl < ntl) ctc = coords(tl);
    }
  }
}

// occupancy target (waves per SIMD) the register allocator works to
#ifndef DSTAGNN_GEMM_WPE
#define DSTAGNN_GEMM_WPE 4
#endif
template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, bool KTWO, int VA, int VB, bool BF, bool KCAT = false,
          bool ACC2 = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, DSTAGNN_GEMM_WPE))) void gemm_f32_kernel(GemmG g) {
  gemm_glds_body<WGM, WGN, WM, WN, A_KC, B_NC, KTWO, VA, VB, BF, KCAT, ACC2>(g);
}
// same code under a second name: the GEMM a profile reports as "the hot kernel" (Gemm::hot)
template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, bool KTWO, int VA, int VB, bool BF, bool KCAT = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, DSTAGNN_GEMM_WPE))) void gemm_f32_hot_kernel(GemmG g) {
  gemm_glds_body<WGM, WGN, WM, WN, A_KC, B_NC, KTWO, VA, VB, BF, KCAT>(g);
}
template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, bool KTWO, int VA, int VB, bool KCAT, int PNS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void gemm_f32_persist_kernel(GemmG g) {
  gemm_persist_body<WGM, WGN, WM, WN, A_KC, B_NC, KTWO, VA, VB, KCAT, PNS>(g);
}
}  // namespace

// LDS stages of the persistent kernel (DSTAGNN_GEMM_PERSIST_NS = 3 or 4)
inline int persist_ns() {
  static const int v = getenv("DSTAGNN_GEMM_PERSIST_NS") && atoi(getenv("DSTAGNN_GEMM_PERSIST_NS")) == 4 ? 4 : 3;
  return v;
}
template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, bool KTWO, int VA, int VB, bool KCAT, int PNS>
void persist_launch(const GemmG& kk, dim3 grid, hipStream_t st) {
  constexpr size_t lds = (size_t)(32 * WM * WGM + 32 * WN * WGN) * 32 * 4 * PNS;
  auto ker = gemm_f32_persist_kernel<WGM, WGN, WM, WN, A_KC, B_NC, KTWO, VA, VB, KCAT, PNS>;
  if constexpr (lds > 65536) {
    static bool done = false;  // raise the kernel's dynamic-LDS limit once
    if (!done) {
      (void)hipFuncSetAttribute((const void*)ker, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      done = true;
    }
  }
  hipLaunchKernelGGL(ker, grid, dim3(256), lds, st, kk);
}
template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, bool KTWO, int VA, int VB, bool KCAT>
void persist_launch_ns(const GemmG& kk, dim3 grid, hipStream_t st) {
  if (persist_ns() == 4) persist_launch<WGM, WGN, WM, WN, A_KC, B_NC, KTWO, VA, VB, KCAT, 4>(kk, grid, st);
  else persist_launch<WGM, WGN, WM, WN, A_KC, B_NC, KTWO, VA, VB, KCAT, 3>(kk, grid, st);
}

// the persistent kernel for one configuration; grid = the sum of the problems' padded slices
template <int WGM, int WGN, int WM, int WN, bool KTWO>
void persist_cfg(const GemmG& kk, dim3 grid, bool akc, bool bnc, int va, int vb, hipStream_t st) {
  if (kk.start[0] > 0) {  // K-concatenated (run_gemm_kcat checked kcat_ok)
    if constexpr (WGM == 4 && WGN == 1 && WM == 1 && WN == 1 && !KTWO)
      persist_launch_ns<WGM, WGN, WM, WN, true, true, KTWO, 4, 4, true>(kk, grid, st);
    return;
  }
#define DS_PV(AK, BN_)                                                                             \
  if (va == 4 && vb == 4)  persist_launch_ns<WGM, WGN, WM, WN, AK, BN_, KTWO, 4, 4, false>(kk, grid, st); \
  else if (va == 4)        persist_launch_ns<WGM, WGN, WM, WN, AK, BN_, KTWO, 4, 1, false>(kk, grid, st); \
  else if (vb == 4)        persist_launch_ns<WGM, WGN, WM, WN, AK, BN_, KTWO, 1, 4, false>(kk, grid, st); \
  else                     persist_launch_ns<WGM, WGN, WM, WN, AK, BN_, KTWO, 1, 1, false>(kk, grid, st);
  if (akc && bnc) { DS_PV(true, true) }
  else if (akc)   { DS_PV(true, false) }
  else if (bnc)   { DS_PV(false, true) }
  else            { DS_PV(false, false) }
#undef DS_PV
}
#define DS_GEMM_PUNIT(NAME, WGM, WGN, WM, WN, KTWO)                                                    \
  void NAME(const GemmG& k, dim3 grid, bool akc, bool bnc, int va, int vb, bool, hipStream_t st) {    \
    persist_cfg<WGM, WGN, WM, WN, KTWO>(k, grid, akc, bnc, va, vb, st);                               \
  }

template <int WGM, int WGN, int WM, int WN, bool A_KC, bool B_NC, bool KTWO, int VA, int VB, bool BF, bool KCAT = false,
          bool ACC2 = false>
void launch_one(const GemmG& k, dim3 grid, bool hot, hipStream_t st) {
  // the "hot" name exists for the one GEMM it tags (pre_conv forward: 64x64, single-level k, fp32)
  constexpr bool HOT_OK = WGM == 2 && WGN == 2 && WM == 1 && WN == 1 && !KTWO && !BF && !KCAT && !ACC2;
  auto ker = gemm_f32_kernel<WGM, WGN, WM, WN, A_KC, B_NC, KTWO, VA, VB, BF, KCAT, ACC2>;
  if constexpr (HOT_OK) {
    if (hot) ker = gemm_f32_hot_kernel<WGM, WGN, WM, WN, A_KC, B_NC, KTWO, VA, VB, BF, KCAT>;
  }
  hipLaunchKernelGGL(ker, grid, dim3(256), 0, st, k);
}

// the K-concatenated form exists for one configuration (the GTU transposed convolutions:
// 128x32 tiles, single-level k maps, both operands k-/n-contiguous with 16-B DMA)
constexpr bool kcat_supported(int wgm, int wgn, int wm, int wn, bool ktwo) {
  return wgm == 4 && wgn == 1 && wm == 1 && wn == 1 && !ktwo;
}
template <int WGM, int WGN, int WM, int WN, bool KTWO, bool BF, bool ACC2 = false>
void launch_cfg(const GemmG& kk, dim3 grid, bool akc, bool bnc, int va, int vb, bool hot, hipStream_t st) {
  if (kk.start[0] > 0) {  // K-concatenated (run_gemm_kcat checked kcat_ok)
    if constexpr (kcat_supported(WGM, WGN, WM, WN, KTWO) && !ACC2)
      launch_one<WGM, WGN, WM, WN, true, true, KTWO, 4, 4, BF, true>(kk, grid, false, st);
    return;
  }
#define DS_V(AK, BN_)                                                                                        \
  if (va == 4 && vb == 4)  launch_one<WGM, WGN, WM, WN, AK, BN_, KTWO, 4, 4, BF, false, ACC2>(kk, grid, hot, st); \
  else if (va == 4)        launch_one<WGM, WGN, WM, WN, AK, BN_, KTWO, 4, 1, BF, false, ACC2>(kk, grid, hot, st); \
  else if (vb == 4)        launch_one<WGM, WGN, WM, WN, AK, BN_, KTWO, 1, 4, BF, false, ACC2>(kk, grid, hot, st); \
  else                     launch_one<WGM, WGN, WM, WN, AK, BN_, KTWO, 1, 1, BF, false, ACC2>(kk, grid, hot, st);
  if (akc && bnc) { DS_V(true, true) }
  else if (akc)   { DS_V(true, false) }
  else if (bnc)   { DS_V(false, true) }
  else            { DS_V(false, false) }
#undef DS_V
}

// one explicit instantiation per unit (gemm_c*_k*.hip)
#define DS_GEMM_UNIT(NAME, WGM, WGN, WM, WN, KTWO, BF)                                                   \
  void NAME(const GemmG& k, dim3 grid, bool akc, bool bnc, int va, int vb, bool hot, hipStream_t st) {  \
    launch_cfg<WGM, WGN, WM, WN, KTWO, BF>(k, grid, akc, bnc, va, vb, hot, st);                          \
  }
// the two-level-accumulation variants (fp32, the tiles split-K uses: 64x64 and 128x32)
#define DS_GEMM_UNIT_ACC2(NAME, WGM, WGN, WM, WN, KTWO)                                                  \
  void NAME(const GemmG& k, dim3 grid, bool akc, bool bnc, int va, int vb, bool hot, hipStream_t st) {  \
    launch_cfg<WGM, WGN, WM, WN, KTWO, false, true>(k, grid, akc, bnc, va, vb, hot, st);                 \
  }
void gemm_c0_k0(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c0_k1(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c1_k0(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c1_k1(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c2_k0(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c2_k1(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c0_k0_bf(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c0_k1_bf(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c1_k0_bf(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c1_k1_bf(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c2_k0_bf(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c2_k1_bf(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c0_k0_a2(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c0_k1_a2(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c2_k0_a2(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_c2_k1_a2(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_p0_k0(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_p0_k1(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_p2_k0(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);
void gemm_p2_k1(const GemmG&, dim3, bool, bool, int, int, bool, hipStream_t);

}  // namespace dsgemm
