// common.hpp — shared device/host helpers for the gfx950 (CDNA4) DSTAGNN kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <cstdlib>
#include <string>

#include "../../include/dstagnn.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------
// Unsigned fast division by a runtime constant (round-up magic, valid for n < 2^31).
// q = (umulhi(n, m) + n) >> s   with s = ceil(log2 d), m = 2^32 (2^s - d) / d + 1.
// ---------------------------------------------------------------------------------
struct FastDiv {
  uint32_t d = 1, m = 1, s = 0;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d ? d : 1;
  uint32_t s = 0;
  while ((1ull << s) < f.d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - f.d)) / f.d + 1);
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

// Two-level affine index map:  off(i) = (i % d) * s0 + (i / d) * s1   (d == 0: i * s0)
struct Idx2 {
  FastDiv f;
  int32_t two = 0;  // 0: single level
  int64_t s0 = 0, s1 = 0;
};

inline Idx2 make_idx(const dstagnn_idx& x) {
  Idx2 r;
  r.two = x.div > 0 ? 1 : 0;
  r.f = make_fastdiv(x.div > 0 ? (uint32_t)x.div : 1u);
  r.s0 = x.s0;
  r.s1 = x.s1;
  return r;
}
inline Idx2 idx1(int64_t s0) {
  dstagnn_idx x{0, s0, 0};
  return make_idx(x);
}
inline Idx2 idx2(int64_t div, int64_t s0, int64_t s1) {
  dstagnn_idx x{div, s0, s1};
  return make_idx(x);
}

__device__ __forceinline__ int64_t ioff(const Idx2& m, uint32_t i) {
  if (!m.two) return (int64_t)i * m.s0;
  uint32_t q = fdiv(i, m.f);
  uint32_t r = i - q * m.f.d;
  return (int64_t)r * m.s0 + (int64_t)q * m.s1;
}

// Branch-free 32-bit variant for the inner (k) loop of the GEMM: a single-level map is
// encoded with d = 2^31 so q = 0 for every valid index; offsets are int32 (the host
// checks the range), so no 64-bit multiplies and no control flow between the loads.
struct KIdx {
  uint32_t d = 0x80000000u, m = 1, s = 31;
  int32_t s0 = 0, s1 = 0;
};

// largest |offset| an index map produces over [0, count)
inline int64_t idx_span(const Idx2& x, int64_t count) {
  if (count <= 0) return 0;
  if (!x.two) return std::llabs(x.s0) * (count - 1);
  const int64_t d = x.f.d;
  return std::llabs(x.s0) * (std::min<int64_t>(d, count) - 1) + std::llabs(x.s1) * ((count - 1) / d);
}

// most negative offset of the map over [0, count) (0 when all strides are >= 0)
inline int64_t idx_min(const Idx2& x, int64_t count) {
  if (count <= 0) return 0;
  if (!x.two) return std::min<int64_t>(0, x.s0 * (count - 1));
  const int64_t d = x.f.d;
  return std::min<int64_t>(0, x.s0 * (std::min<int64_t>(d, count) - 1)) +
         std::min<int64_t>(0, x.s1 * ((count - 1) / d));
}

inline bool make_kidx(const Idx2& x, int64_t K, KIdx* out) {
  KIdx k;
  int64_t maxoff;
  if (x.two) {
    k.d = x.f.d; k.m = x.f.m; k.s = x.f.s;
    int64_t nq = K > 0 ? (K - 1) / x.f.d + 1 : 1;
    maxoff = std::llabs(x.s0) * (int64_t)(std::min<int64_t>(x.f.d, K)) + std::llabs(x.s1) * nq;
  } else {
    maxoff = std::llabs(x.s0) * K;
  }
  if (maxoff >= (1ll << 31) || std::llabs(x.s0) >= (1ll << 31) || std::llabs(x.s1) >= (1ll << 31)) return false;
  k.s0 = (int32_t)x.s0;
  k.s1 = (int32_t)x.s1;
  *out = k;
  return true;
}

__device__ __forceinline__ int32_t koff(const KIdx& m, uint32_t i) {
  const uint32_t q = (__umulhi(i, m.m) + i) >> m.s;
  const uint32_t r = i - q * m.d;
  return (int32_t)r * m.s0 + (int32_t)q * m.s1;
}

// Branch-free 64-bit variant for batch (z) maps, same encoding as KIdx.
struct ZIdx {
  uint32_t d = 0x80000000u, m = 1, s = 31;
  int64_t s0 = 0, s1 = 0;
};
inline ZIdx make_zidx(const Idx2& x) {
  ZIdx z;
  if (x.two) { z.d = x.f.d; z.m = x.f.m; z.s = x.f.s; }
  z.s0 = x.s0;
  z.s1 = x.s1;
  return z;
}
__device__ __forceinline__ int64_t zoff(const ZIdx& m, uint32_t i) {
  const uint32_t q = (__umulhi(i, m.m) + i) >> m.s;
  const uint32_t r = i - q * m.d;
  return (int64_t)r * m.s0 + (int64_t)q * m.s1;
}

// ---------------------------------------------------------------------------------
// Kernel-argument fetch in ONE memory round.  The kernarg segment is cold at every
// launch (~1000 cycles per access round) and hipcc issues a large struct's s_loads in
// several dependent rounds (7 for the GEMM descriptor).  Instead every lane loads one
// dword of the struct (one or two vector loads, a single round) and v_readlane puts each
// dword back into an SGPR, so the compiler still sees wave-uniform values.  Call it first
// thing in the kernel, with every lane active (block sizes are multiples of 64).
// ---------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T load_args(const T& in) {
  constexpr int NW = (int)((sizeof(T) + 3) / 4);
  static_assert(NW <= 128, "load_args: struct larger than 512 bytes");
  static_assert(sizeof(T) % 4 == 0, "load_args: struct size must be a multiple of 4");
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&in);
  const int lane = (int)(threadIdx.x & 63);
  const uint32_t v0 = src[lane < NW ? lane : NW - 1];
  uint32_t v1 = 0;
  if (NW > 64) v1 = src[lane + 64 < NW ? lane + 64 : NW - 1];
  union U {
    T t;
    uint32_t w[NW];
    __device__ U() {}
  } u;
#pragma unroll
  for (int i = 0; i < NW; ++i) u.w[i] = (uint32_t)__builtin_amdgcn_readlane((int)(i < 64 ? v0 : v1), i & 63);
  return u.t;
}

// ---------------------------------------------------------------------------------
// Wave64 reductions (CDNA: 64 lanes; __shfl_xor spans the whole wave).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// NV independent full-wave sums at once (NV = 2^L <= 64): L halving exchange steps (offsets
// 32, 16, ...: each lane keeps the half of its values its offset bit selects and adds the
// partner's copy of that half), then plain butterflies; NV - 1 + 6 - L shuffles instead of 6 NV.
// Returns the total of value j = (lane >> (6 - L)) & (NV - 1) (held by 64 / NV lanes).  Fixed
// order: deterministic.
template <int NV>
__device__ __forceinline__ float wave_sum_many(float (&v)[NV]) {
  static_assert(NV >= 1 && NV <= 64 && (NV & (NV - 1)) == 0, "power of two <= 64");
  const int lane = (int)(threadIdx.x & 63);
  int o = 32;
#pragma unroll
  for (int n = NV; n > 1; n >>= 1, o >>= 1) {
    const bool hi = (lane & o) != 0;
#pragma unroll
    for (int i = 0; i < n / 2; ++i) {
      const float keep = hi ? v[i + n / 2] : v[i];
      const float send = hi ? v[i] : v[i + n / 2];
      v[i] = keep + __shfl_xor(send, o, 64);
    }
  }
  float r = v[0];
#pragma unroll
  for (; o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
  return r;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------------------------
// Counter-based dropout RNG: a splitmix64 key per (seed, mask), two 32-bit finalisers per element.
// ---------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// 32-bit finaliser (two 32-bit multiplies; "lowbias32")
__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// the per-(seed, mask) key: one 64-bit finaliser of uniform values (hoisted out of the loops)
struct DropKey {
  uint32_t lo, hi;
};
__host__ __device__ __forceinline__ DropKey drop_key(uint64_t seed, uint32_t which) {
  const uint64_t z = mix64(seed * 0x9E3779B97F4A7C15ull + ((uint64_t)which << 56) + 1);
  return DropKey{(uint32_t)z, (uint32_t)(z >> 32)};
}
// the uniform draw of element idx: two 32-bit finalisers (the element index's high word first,
// its low word through a bijection: distinct indices of one high word never collide) — the
// 64-bit multiplies of a 64-bit finaliser per element are quarter rate on the vector ALU
__host__ __device__ __forceinline__ float drop_u(DropKey k, uint64_t idx) {
  const uint32_t h = mix32((uint32_t)idx ^ k.lo ^ mix32((uint32_t)(idx >> 32) ^ k.hi));
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}
// scale = 1/(1-p) when kept, 0 when dropped
__device__ __forceinline__ float drop_scale(uint64_t seed, uint32_t which, uint64_t idx, float p) {
  return drop_u(drop_key(seed, which), idx) >= p ? 1.0f / (1.0f - p) : 0.0f;
}

// ---------------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------------
void set_last_error(const std::string& s);

#define DS_CHECK_LAUNCH()                                            \
  do {                                                               \
    hipError_t _e = hipGetLastError();                               \
    if (_e != hipSuccess) {                                          \
      set_last_error(std::string("launch: ") + hipGetErrorString(_e)); \
      return (int)_e;                                                \
    }                                                                \
  } while (0)

#define DS_TRY(x)                 \
  do {                            \
    int _r = (x);                 \
    if (_r != 0) return _r;       \
  } while (0)

static inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------------
// kernel-written stream signals (block.hip Streams::fork_k): a fork from the block's main
// stream to its side stream leaves the flag write PENDING for the next kernel launched on the
// main stream that can carry it (the GEMMs, the GTU input-gradient kernel, the aggregate-first
// SDDMM, the flash dQ / dK kernels): that kernel's workgroup 0 stores the flag as it starts —
// every earlier kernel of the stream has completed by then — instead of a
// hipStreamWriteValue32 (a ~4.5 us ROCclr kernel plus its dispatch gap on the critical path).
// A launcher reads the pending signal (peek_stream_sig), passes it to its kernel and, once the
// launch succeeded, calls stream_sig_sent, which queues the side stream's wait for the flag —
// so the writer is always queued BEFORE the wait (no dependence on how streams map to hardware
// queues, nor on whether a wait can block the host).  A signal nobody consumed is written by
// flush_stream_sig() (write on main, then the side's wait), which runs before the main stream
// waits for the side stream and when the block's op returns (also on its error paths).  The
// block issues no side-stream work between a fork_k and the launch that carries its signal.
// ---------------------------------------------------------------------------------
struct StreamSig {
  uint32_t* p = nullptr;
  uint32_t v = 0;
};
StreamSig peek_stream_sig(hipStream_t st);  // the pending signal for st, or {}
int stream_sig_sent(hipStream_t st, const StreamSig& s);  // a launch on st carried s: queue the wait
int flush_stream_sig();  // a pending signal nobody consumed: hipStreamWriteValue32, then the wait

// workgroup 0, thread 0: a vector store (system scope, release) of the signal, if any
__device__ __forceinline__ void stream_sig_store(uint32_t* p, uint32_t v) {
  if (p != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0)
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------------
// internal GEMM entry (gemm.hip)
// ---------------------------------------------------------------------------------
struct Gemm {
  int M = 0, N = 0, K = 0, batch = 1;
  const float* A = nullptr; Idx2 am, ak, az; int64_t a_off = 0;
  const float* B = nullptr; Idx2 bk, bn, bz; int64_t b_off = 0;
  float* C = nullptr;       Idx2 cm, cn, cz; int64_t c_off = 0;
  float alpha = 1.f, beta = 0.f;
  const float* bias = nullptr; int64_t bias_stride = 1;
  int relu = 0;
  // optional epilogue extras (same C index maps): write to Cout instead of C, and zero
  // where emask <= 0 (a fused ReLU backward: d_pre = d_out * (out > 0))
  const float* emask = nullptr;
  float* Cout = nullptr;
  // optional: Cout with its OWN index maps (omap; else C's), plus obeta * the old Cout value:
  // out[om(m) + on(n)] = obeta * out[...] + (alpha AB + beta C[cm(m) + cn(n)]) — e.g. a product
  // whose beta input is row-major but whose result accumulates into a transposed tensor
  bool omap = false; Idx2 om, on, oz; float obeta = 0.f;
  int hot = 0;  // 1: launch under the separately named gemm_f32_hot_kernel (profiling tag)
  // optional column sums of A over k: ones_out[m * ones_stride] = alpha * sum_k A[m][k] (a bias
  // gradient folded into its weight-gradient GEMM); plain epilogue only (no beta/bias/relu/emask)
  float* ones_out = nullptr; int64_t ones_stride = 1;
  int splitk_target = 0;  // split-K workgroup target for this call (0: the global target)
  Gemm() { am = ak = az = bk = bn = bz = cm = cn = cz = om = on = oz = idx1(0); }
};
// ws: split-K partial slab scratch (may be null -> no split)
int run_gemm(const Gemm& g, float* ws, size_t ws_floats, hipStream_t st);
// 1..3 independent problems (disjoint outputs) as one grouped launch where their kernel
// configurations agree; each takes its own slice of the split-K slab space ws
int run_gemm_group(const Gemm* gs, int n, float* ws, size_t ws_floats, hipStream_t st);
// 1..3 products summed over their concatenated K ranges into problem 0's output and
// epilogue (same M, N, batch): C = epilogue_0(sum_p A_p B_p), one launch, no split-K
int run_gemm_kcat(const Gemm* gs, int n, hipStream_t st);
// GEMM-family profiling (gemm.hip): while on, the block runs on ONE stream (no side-stream
// overlap) so every recorded GEMM duration is its own
bool gemm_prof_on();
// a GEMM-family product computed by another kernel, timed into the same records (or null)
void* gemm_prof_begin(double flops, double bytes, hipStream_t st, int kind = DSTAGNN_PROF_GEMM);
int gemm_prof_records(dstagnn_prof_record* out, int cap);
void gemm_prof_end(void* rec, hipStream_t st);
int gemm_prof_start(int capacity);
int gemm_prof_stop(dstagnn_prof_stats* out);
int gemm_set_splitk_target(int target);
int gemm_set_bf16(int on);

// fused-kernel phase timestamps (a variant build with -DDSTAGNN_TF_TIMING, e.g. into
// abtest/tftime): thread 0 of workgroups 0 and 100 prints the wall-clock (100 MHz) deltas between the marks
#ifdef DSTAGNN_TF_TIMING
#define TF_MARK(k) do { if (threadIdx.x == 0) tmark[k] = wall_clock64(); } while (0)
#define TF_DECL uint64_t tmark[12] = {}
#define TF_PRINT(tag, n)                                                                          \
  do {                                                                                          \
    if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == 100)) {                           \
      double d_[12];                                                                            \
      for (int k_ = 1; k_ < (n); ++k_) d_[k_] = (double)(tmark[k_] - tmark[k_ - 1]) / 100.0;    \
      for (int k_ = (n); k_ < 12; ++k_) d_[k_] = 0.0;                                          \
      printf("%s wg %d: %.2f %.2f %.2f %.2f %.2f %.2f %.2f %.2f %.2f us\n", tag, (int)blockIdx.x, \
             d_[1], d_[2], d_[3], d_[4], d_[5], d_[6], d_[7], d_[8], d_[9]);                    \
    }                                                                                           \
  } while (0)
#else
#define TF_MARK(k) do {} while (0)
#define TF_DECL
#define TF_PRINT(tag, n) do {} while (0)
#endif
