// torch_ops.cpp — the PyTorch-ROCm operator boundary: TORCH_LIBRARY(dstagnn, ...) over the
// C-ABI of libdstagnn.so (include/dstagnn.h).  Built as dstagnn_drought_amd/_C.so (links
// libdstagnn.so; loaded with torch.ops.load_library).
//
// What each op replaces in the reference (model/DSTAGNN_my.py, data/*.py):
//   dstagnn::block          DSTAGNN_block.forward (:225-253) + its autograd backward, as ONE
//                           C++ autograd node (torch::autograd::Function): forward = one
//                           dstagnn_block_forward call, backward = one dstagnn_block_backward
//   dstagnn::block_fwd/bwd  the same two calls as plain ops (tests, tools)
//   dstagnn::cheb_sat_fwd/bwd  cheb_conv_withSAt.forward (:117-133) and its gradient
//   dstagnn::head_fwd/bwd   DSTAGNN_submodule's cat + final_conv + final_fc (:272-280)
//   dstagnn::gemm_f32       the strided f32-MFMA GEMM (tests / tools)
//   dstagnn::colsum         the fixed-order column-sum reduction (bias / LayerNorm affine grads; tests)
//   dstagnn::stag_* / emd_dense / fast_stag_distances / graph_topk   the graph builders
//                           (data/STAG_gen.py:17-129, data/fast_STAG_gen.py:16-74)
//
// Conventions: inputs are borrowed (contiguous, on the HIP device, fp32 —
// fp64 / int32 for the graph builders), outputs and saved-for-backward buffers are allocated
// here with at::empty (PyTorch's caching allocator), every launch is asynchronous on the
// current HIP stream of the input's device, shape / dtype errors and library error codes
// raise RuntimeError through TORCH_CHECK (with dstagnn_last_error()'s text).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/autograd.h>
#include <torch/library.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/dstagnn.h"

using at::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

namespace {

// -------------------------------------------------------------------------------------
// helpers
// -------------------------------------------------------------------------------------
dstagnn_stream_t stream_of(const Tensor& t) {
  return (dstagnn_stream_t)c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed (code ", rc, "): ", dstagnn_last_error());
}

void check_dev(const Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.defined(), name, ": undefined tensor");
  TORCH_CHECK(t.is_cuda(), name, ": must be a HIP device tensor (there is no CPU path)");
  TORCH_CHECK(t.scalar_type() == dt, name, ": expected ", c10::toString(dt), ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), name, ": must be contiguous");
}

template <typename T>
T* ptr_or_null(const c10::optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<T>() : nullptr;
}

at::TensorOptions f32(const Tensor& like) { return like.options().dtype(at::kFloat); }

// ---- block parameters: the dstagnn_block_params struct is an array of 44 pointers ----
constexpr int kSlots = 16 + 2 * DSTAGNN_MAX_K + 3 + 3 + 6;
static_assert(sizeof(dstagnn_block_params) == kSlots * sizeof(void*), "params struct layout");
static_assert(sizeof(dstagnn_block_grads) == kSlots * sizeof(void*), "grads struct layout");
// slots of the parameters an INNER block (F != 1) never uses (EmbedT, residual_conv:
// quirk 11, their .grad stays None)
bool unused_inner(int64_t slot) { return slot == 2 || slot == 3 || slot == 4 || slot == 38 || slot == 39; }

// cfg = [n_heads, d_k, d_v, d_model, K, C]; flags: 1 train, 2 sparse, 4 direct grads, 8 poison,
// 16 fused (flash) Chebyshev attention; bits 32.. carry the call's first global sample index
// (dstagnn_block_dims::sample_base: a data-parallel shard's offset, keys the dropout masks)
enum { kTrain = 1, kSparse = 2, kDirect = 4, kPoison = 8, kFlash = 16 };
constexpr int kSampleShift = 32;

int res_mode_of(const c10::optional<Tensor>& res, int64_t F) {
  if (!res.has_value() || !res->defined()) return DSTAGNN_RES_NONE;
  const Tensor& r = *res;
  TORCH_CHECK(r.dim() == 5, "res_att must be 5-D (B,F|1,h,T,T), got ", r.sizes());
  if (r.size(1) == F) return DSTAGNN_RES_FULL;
  if (r.size(1) == 1) return DSTAGNN_RES_BCAST;
  TORCH_CHECK(false, "The size of tensor a (", F, ") must match the size of tensor b (", r.size(1),
              ") at non-singleton dimension 1");
  return 0;
}

struct BlockCall {
  dstagnn_block_dims d{};
  dstagnn_block_params p{};
  dstagnn_graph g{};
  int mode = 0;
  int64_t flags = 0;
};

dstagnn_graph graph_of(at::TensorList graph, bool sparse, int64_t K, int64_t N);

BlockCall make_call(const Tensor& x, const c10::optional<Tensor>& res, at::TensorList params, at::IntArrayRef slots,
                    at::TensorList graph, at::IntArrayRef cfg, double drop_p, int64_t seed, int64_t flags) {
  check_dev(x, at::kFloat, "x");
  TORCH_CHECK(x.dim() == 4, "x must be (B,N,F,T), got ", x.sizes());
  TORCH_CHECK(cfg.size() == 6, "cfg must be [n_heads, d_k, d_v, d_model, K, C]");
  TORCH_CHECK(params.size() == slots.size(), "params / slots length mismatch");
  TORCH_CHECK(graph.size() == 2 || graph.size() == 6 || graph.size() == 15,
              "graph = [cheb, adj_pa] (+ csc_ptr, csc_row, csr_ptr, csr_col (+ csr2csc, apa_bits, apa_bits_t, "
              "apa_ptr, apa_row, tsupp, csc2csr, apa_idx, apa2t))");
  BlockCall c;
  c.flags = flags;
  c.mode = res_mode_of(res, x.size(2));
  if (c.mode != DSTAGNN_RES_NONE) check_dev(*res, at::kFloat, "res_att");
  auto& d = c.d;
  d.B = (int)x.size(0); d.N = (int)x.size(1); d.F = (int)x.size(2); d.T = (int)x.size(3);
  d.n_heads = (int)cfg[0]; d.d_k = (int)cfg[1]; d.d_v = (int)cfg[2]; d.d_model = (int)cfg[3]; d.K = (int)cfg[4];
  d.C = (int)cfg[5];
  d.res_mode = c.mode;
  d.train = (flags & kTrain) ? 1 : 0;
  d.drop_p = (float)drop_p;
  d.seed = (uint64_t)seed;
  TORCH_CHECK(flags >= 0, "flags: negative sample base");
  d.sample_base = flags >> kSampleShift;
  d.cheb_sparse = (flags & kSparse) ? 1 : 0;
  const float** arr = reinterpret_cast<const float**>(&c.p);
  for (size_t i = 0; i < params.size(); ++i) {
    TORCH_CHECK(slots[i] >= 0 && slots[i] < kSlots, "bad parameter slot ", slots[i]);
    if (!params[i].defined()) continue;
    check_dev(params[i], at::kFloat, "parameter");
    arr[slots[i]] = params[i].data_ptr<float>();
  }
  c.g = graph_of(graph, d.cheb_sparse != 0, d.K, d.N);
  d.cheb_flash = (flags & kFlash) ? 1 : 0;
  TORCH_CHECK(!d.cheb_flash || graph.size() == 15, "flash Chebyshev path requested without its graph data");
  d.cheb_nnz = d.cheb_flash ? c.g.nnz : 0;
  d.cheb_apa_nnz = d.cheb_flash ? c.g.apa_nnz : 0;
  return c;
}

std::pair<size_t, size_t> block_sizes(const BlockCall& c) {
  size_t sv = 0, sc = 0;
  check_rc(dstagnn_block_sizes(&c.d, &sv, &sc), "dstagnn_block_sizes");
  return {sv, sc};
}

Tensor bytes(size_t n, const Tensor& like) { return at::empty({(int64_t)n}, like.options().dtype(at::kByte)); }

// forward: (out, re_at, save)
std::tuple<Tensor, Tensor, Tensor> run_forward(const BlockCall& c, const Tensor& x,
                                               const c10::optional<Tensor>& res) {
  c10::DeviceGuard guard(x.device());
  auto [sv, sc] = block_sizes(c);
  const auto& d = c.d;
  Tensor save = bytes(sv, x), scratch = bytes(sc, x);
  Tensor out = at::empty({d.B, d.N, d.C, d.T}, f32(x));
  Tensor re_at = at::empty({d.B, d.F, d.n_heads, d.T, d.T}, f32(x));
  if (c.flags & kPoison) {  // every library-written buffer starts as NaN (all-ones bytes)
    for (Tensor* t : {&save, &scratch}) t->fill_(255);
    out.fill_(NAN);
    re_at.fill_(NAN);
  }
  const float* ra = c.mode != DSTAGNN_RES_NONE ? res->data_ptr<float>() : nullptr;
  check_rc(dstagnn_block_forward(&c.d, &c.p, &c.g, x.data_ptr<float>(), ra, out.data_ptr<float>(),
                                 re_at.data_ptr<float>(), save.data_ptr(), sv, scratch.data_ptr(), sc, stream_of(x)),
           "dstagnn_block_forward");
  return {out, re_at, save};
}

// backward: d_x, d_res (undefined for mode 0), the flat gradient buffer, per-parameter
// views of it (undefined for parameters this block kind does not use)
struct BwdResult {
  Tensor dx, dres, flat;
  std::vector<Tensor> grads;
};

BwdResult run_backward(const BlockCall& c, const Tensor& x, const c10::optional<Tensor>& res, Tensor d_out,
                       const c10::optional<Tensor>& d_re_at, const Tensor& save, at::TensorList params,
                       at::IntArrayRef slots) {
  c10::DeviceGuard guard(x.device());
  const auto& d = c.d;
  TORCH_CHECK(save.defined() && save.numel() > 0,
              "dstagnn::block backward: the saved forward state is gone (backward called twice? "
              "use retain_graph only with a fresh forward)");
  auto [sv, sc] = block_sizes(c);
  TORCH_CHECK((size_t)save.numel() >= sv, "save buffer smaller than dstagnn_block_sizes()");
  if (!d_out.defined()) d_out = at::zeros({d.B, d.N, d.C, d.T}, f32(x));
  d_out = d_out.contiguous();
  Tensor dre;
  if (d_re_at.has_value() && d_re_at->defined()) dre = d_re_at->contiguous();
  const bool first = d.F == 1;
  // every used parameter's gradient is a view of ONE flat buffer, packed in parameter
  // order (the library writes the stacked Q|K|V, Q'|K', Theta_k gradients in place)
  int64_t total = 0;
  std::vector<char> used(params.size());
  for (size_t i = 0; i < params.size(); ++i) {
    used[i] = params[i].defined() && (first || !unused_inner(slots[i]));
    if (used[i]) total += params[i].numel();
  }
  BwdResult r;
  r.flat = at::empty({total}, f32(x));
  r.grads.resize(params.size());
  dstagnn_block_grads gs{};
  float** garr = reinterpret_cast<float**>(&gs);
  int64_t off = 0;
  for (size_t i = 0; i < params.size(); ++i) {
    if (!used[i]) continue;
    const int64_t n = params[i].numel();
    r.grads[i] = r.flat.narrow(0, off, n).view(params[i].sizes());
    garr[slots[i]] = r.flat.data_ptr<float>() + off;
    off += n;
  }
  r.dx = at::empty_like(x);
  if (c.mode != DSTAGNN_RES_NONE) r.dres = at::empty_like(*res);
  Tensor scratch = bytes(sc, x);
  if (c.flags & kPoison) {
    scratch.fill_(255);
    r.flat.fill_(NAN);
    r.dx.fill_(NAN);
    if (r.dres.defined()) r.dres.fill_(NAN);
  }
  const float* ra = c.mode != DSTAGNN_RES_NONE ? res->data_ptr<float>() : nullptr;
  check_rc(dstagnn_block_backward(&c.d, &c.p, &c.g, x.data_ptr<float>(), ra, d_out.data_ptr<float>(),
                                  dre.defined() ? dre.data_ptr<float>() : nullptr, r.dx.data_ptr<float>(),
                                  r.dres.defined() ? r.dres.data_ptr<float>() : nullptr, &gs,
                                  const_cast<void*>(save.data_ptr()), (size_t)save.numel(), scratch.data_ptr(), sc,
                                  stream_of(x)),
           "dstagnn_block_backward");
  return r;
}

// -------------------------------------------------------------------------------------
// dstagnn::block — one autograd node per DSTAGNN_block
// -------------------------------------------------------------------------------------
class BlockFunction : public torch::autograd::Function<BlockFunction> {
 public:
  static variable_list forward(AutogradContext* ctx, const Tensor& x, const c10::optional<Tensor>& res,
                               at::TensorList params, at::IntArrayRef slots, at::TensorList graph,
                               at::IntArrayRef cfg, double drop_p, int64_t seed, int64_t flags) {
    ctx->set_materialize_grads(false);
    BlockCall c = make_call(x, res, params, slots, graph, cfg, drop_p, seed, flags);
    auto [out, re_at, save] = run_forward(c, x, res);
    ctx->save_for_backward({x, c.mode != DSTAGNN_RES_NONE ? *res : Tensor()});
    // parameters and graph constants: strong references (they are leaves / buffers, no
    // reference cycle through this node); the save buffer is dropped after the backward
    ctx->saved_data["params"] = params.vec();
    ctx->saved_data["graph"] = graph.vec();
    ctx->saved_data["slots"] = slots.vec();
    ctx->saved_data["cfg"] = cfg.vec();
    ctx->saved_data["drop_p"] = drop_p;
    ctx->saved_data["seed"] = seed;
    ctx->saved_data["flags"] = flags;
    ctx->saved_data["save"] = save;
    return {out, re_at};
  }

  static variable_list backward(AutogradContext* ctx, variable_list gout) {
    auto saved = ctx->get_saved_variables();
    const Tensor x = saved[0];
    c10::optional<Tensor> res;
    if (saved[1].defined()) res = saved[1];
    const auto params = ctx->saved_data["params"].toTensorVector();
    const auto graph = ctx->saved_data["graph"].toTensorVector();
    const auto slots = ctx->saved_data["slots"].toIntVector();
    const auto cfg = ctx->saved_data["cfg"].toIntVector();
    const int64_t flags = ctx->saved_data["flags"].toInt();
    BlockCall c = make_call(x, res, params, slots, graph, cfg, ctx->saved_data["drop_p"].toDouble(),
                            ctx->saved_data["seed"].toInt(), flags);
    Tensor save = ctx->saved_data["save"].toTensor();
    ctx->saved_data["save"] = Tensor();  // release the forward state with the backward
    c10::optional<Tensor> dre;
    if (gout.size() > 1 && gout[1].defined()) dre = gout[1];
    BwdResult r = run_backward(c, x, res, gout[0], dre, save, params, slots);
    // gradient list: x, res_att, params..., slots, graph..., cfg, drop_p, seed, flags
    variable_list g;
    g.reserve(2 + params.size() + 1 + graph.size() + 4);
    g.push_back(r.dx);
    g.push_back(r.dres);
    if (flags & kDirect) {
      // direct-grad mode (model.set_direct_grads): .grad is set here (or accumulated) instead
      // of through one AccumulateGrad node per parameter
      for (size_t i = 0; i < params.size(); ++i) {
        Tensor p = params[i];
        if (r.grads[i].defined() && p.requires_grad()) {
          Tensor& pg = p.mutable_grad();
          if (!pg.defined()) pg = r.grads[i];
          else pg.add_(r.grads[i]);
        }
        g.push_back(Tensor());
      }
    } else {
      for (auto& t : r.grads) g.push_back(t);
    }
    g.push_back(Tensor());  // slots
    for (size_t i = 0; i < graph.size(); ++i) g.push_back(Tensor());
    for (int i = 0; i < 4; ++i) g.push_back(Tensor());
    return g;
  }
};

// -------------------------------------------------------------------------------------
// dstagnn::block_planned — the same node for direct-gradient mode with the block's constant
// arguments (parameters, slots, graph, cfg) held in ONE cached BlockPlan object instead of
// being boxed, edge-linked and saved per call: the parameters are not autograd inputs (their
// gradients are written by the backward itself), so the node has three inputs (x, res_att and
// an anchor parameter that keeps the node in the graph when x needs no gradient) instead of
// ~50.  Host cost, not arithmetic: the kernels and their results are the same as dstagnn::block.
// -------------------------------------------------------------------------------------
struct BlockPlan : torch::CustomClassHolder {
  std::vector<Tensor> params, graph;
  std::vector<int64_t> slots, cfg;
  BlockPlan(std::vector<Tensor> p, std::vector<int64_t> s, std::vector<Tensor> g, std::vector<int64_t> c)
      : params(std::move(p)), graph(std::move(g)), slots(std::move(s)), cfg(std::move(c)) {
    TORCH_CHECK(params.size() == slots.size(), "BlockPlan: params / slots length mismatch");
  }
};

class BlockPlanFunction : public torch::autograd::Function<BlockPlanFunction> {
 public:
  static variable_list forward(AutogradContext* ctx, const Tensor& x, const c10::optional<Tensor>& res,
                               const c10::intrusive_ptr<BlockPlan>& plan, const Tensor& anchor, double drop_p,
                               int64_t seed, int64_t flags) {
    (void)anchor;
    ctx->set_materialize_grads(false);
    TORCH_CHECK(flags & kDirect, "block_planned: direct-gradient mode only");
    BlockCall c = make_call(x, res, plan->params, plan->slots, plan->graph, plan->cfg, drop_p, seed, flags);
    auto [out, re_at, save] = run_forward(c, x, res);
    ctx->save_for_backward({x, c.mode != DSTAGNN_RES_NONE ? *res : Tensor()});
    ctx->saved_data["plan"] = plan;
    ctx->saved_data["drop_p"] = drop_p;
    ctx->saved_data["seed"] = seed;
    ctx->saved_data["flags"] = flags;
    ctx->saved_data["save"] = save;
    return {out, re_at};
  }

  static variable_list backward(AutogradContext* ctx, variable_list gout) {
    auto saved = ctx->get_saved_variables();
    const Tensor x = saved[0];
    c10::optional<Tensor> res;
    if (saved[1].defined()) res = saved[1];
    auto plan = ctx->saved_data["plan"].toCustomClass<BlockPlan>();
    const int64_t flags = ctx->saved_data["flags"].toInt();
    BlockCall c = make_call(x, res, plan->params, plan->slots, plan->graph, plan->cfg, ctx->saved_data["drop_p"].toDouble(),
                            ctx->saved_data["seed"].toInt(), flags);
    Tensor save = ctx->saved_data["save"].toTensor();
    ctx->saved_data["save"] = Tensor();  // release the forward state with the backward
    c10::optional<Tensor> dre;
    if (gout.size() > 1 && gout[1].defined()) dre = gout[1];
    BwdResult r = run_backward(c, x, res, gout[0], dre, save, plan->params, plan->slots);
    for (size_t i = 0; i < plan->params.size(); ++i) {
      Tensor p = plan->params[i];
      if (r.grads[i].defined() && p.requires_grad()) {
        Tensor& pg = p.mutable_grad();
        if (!pg.defined()) pg = r.grads[i];
        else pg.add_(r.grads[i]);
      }
    }
    // gradient list: x, res_att, plan, anchor, drop_p, seed, flags
    return {r.dx, r.dres, Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

std::tuple<Tensor, Tensor> block_planned_autograd(const Tensor& x, const c10::optional<Tensor>& res,
                                                  const c10::intrusive_ptr<BlockPlan>& plan, const Tensor& anchor,
                                                  double drop_p, int64_t seed, int64_t flags) {
  auto o = BlockPlanFunction::apply(x, res, plan, anchor, drop_p, seed, flags);
  return {o[0], o[1]};
}

std::tuple<Tensor, Tensor> block_planned_infer(const Tensor& x, const c10::optional<Tensor>& res,
                                               const c10::intrusive_ptr<BlockPlan>& plan, const Tensor& anchor,
                                               double drop_p, int64_t seed, int64_t flags) {
  (void)anchor;
  BlockCall c = make_call(x, res, plan->params, plan->slots, plan->graph, plan->cfg, drop_p, seed, flags);
  auto [out, re_at, save] = run_forward(c, x, res);
  return {out, re_at};
}

std::tuple<Tensor, Tensor> block_autograd(const Tensor& x, const c10::optional<Tensor>& res, at::TensorList params,
                                          at::IntArrayRef slots, at::TensorList graph, at::IntArrayRef cfg,
                                          double drop_p, int64_t seed, int64_t flags) {
  auto o = BlockFunction::apply(x, res, params, slots, graph, cfg, drop_p, seed, flags);
  return {o[0], o[1]};
}

// inference (no autograd key): forward only
std::tuple<Tensor, Tensor> block_infer(const Tensor& x, const c10::optional<Tensor>& res, at::TensorList params,
                                       at::IntArrayRef slots, at::TensorList graph, at::IntArrayRef cfg, double drop_p,
                                       int64_t seed, int64_t flags) {
  BlockCall c = make_call(x, res, params, slots, graph, cfg, drop_p, seed, flags);
  auto [out, re_at, save] = run_forward(c, x, res);
  return {out, re_at};
}

std::tuple<Tensor, Tensor, Tensor> block_fwd(const Tensor& x, const c10::optional<Tensor>& res,
                                             at::TensorList params, at::IntArrayRef slots, at::TensorList graph,
                                             at::IntArrayRef cfg, double drop_p, int64_t seed, int64_t flags) {
  BlockCall c = make_call(x, res, params, slots, graph, cfg, drop_p, seed, flags);
  return run_forward(c, x, res);
}

// -> (d_x, d_res_att (empty for res_att None), flat gradient buffer); the flat buffer holds
// the used parameters' gradients back to back in parameter order
std::tuple<Tensor, Tensor, Tensor> block_bwd(const Tensor& x, const c10::optional<Tensor>& res, const Tensor& d_out,
                                             const c10::optional<Tensor>& d_re_at, const Tensor& save,
                                             at::TensorList params, at::IntArrayRef slots, at::TensorList graph,
                                             at::IntArrayRef cfg, double drop_p, int64_t seed, int64_t flags) {
  BlockCall c = make_call(x, res, params, slots, graph, cfg, drop_p, seed, flags);
  BwdResult r = run_backward(c, x, res, d_out, d_re_at, save, params, slots);
  return {r.dx, r.dres.defined() ? r.dres : at::empty({0}, f32(x)), r.flat};
}

// a ReLU output the forward keeps in `save` (parity tests: its sign pattern is that ReLU's
// decision): which 0 = the Chebyshev output X (B,N,T,C) (model/DSTAGNN_my.py:133), 1 = tco
// (B,N,C,T) (:245/:247), 2 = ReLU(residual + tco) (B,N,C,T) (:252)
Tensor block_relu_out(const Tensor& x, const c10::optional<Tensor>& res, at::TensorList params, at::IntArrayRef slots,
                      at::TensorList graph, at::IntArrayRef cfg, double drop_p, int64_t seed, int64_t flags,
                      int64_t which) {
  BlockCall c = make_call(x, res, params, slots, graph, cfg, drop_p, seed, flags);
  auto [out, re_at, save] = run_forward(c, x, res);
  size_t off = 0, n = 0;
  check_rc(dstagnn_block_save_offset(&c.d, (int)which, &off, &n), "dstagnn_block_save_offset");
  const int64_t base = (int64_t)((256 - ((uintptr_t)save.data_ptr() & 255)) & 255);  // the library's align256
  Tensor t = save.narrow(0, base + (int64_t)off, (int64_t)n * 4).view(at::kFloat);
  return (which == 0 ? t.view({c.d.B, c.d.N, c.d.T, c.d.C}) : t.view({c.d.B, c.d.N, c.d.C, c.d.T})).clone();
}
Tensor block_cheb_out(const Tensor& x, const c10::optional<Tensor>& res, at::TensorList params, at::IntArrayRef slots,
                      at::TensorList graph, at::IntArrayRef cfg, double drop_p, int64_t seed, int64_t flags) {
  return block_relu_out(x, res, params, slots, graph, cfg, drop_p, seed, flags, 0);
}

// the kernel path (DSTAGNN_PATH_* bits) the block takes for this call's dims: launches nothing
int64_t block_paths(const Tensor& x, const c10::optional<Tensor>& res, at::TensorList params, at::IntArrayRef slots,
                    at::TensorList graph, at::IntArrayRef cfg, double drop_p, int64_t seed, int64_t flags) {
  BlockCall c = make_call(x, res, params, slots, graph, cfg, drop_p, seed, flags);
  uint32_t bits = 0;
  check_rc(dstagnn_block_paths(&c.d, &bits), "dstagnn_block_paths");
  return (int64_t)bits;
}

// HIP-event timing of one block stage (dstagnn_block_time_stage) after one forward:
// mean milliseconds per launch on the current stream
double block_time_stage(const Tensor& x, const c10::optional<Tensor>& res, at::TensorList params,
                        at::IntArrayRef slots, at::TensorList graph, at::IntArrayRef cfg, double drop_p, int64_t seed,
                        int64_t flags, int64_t stage, int64_t iters) {
  BlockCall c = make_call(x, res, params, slots, graph, cfg, drop_p, seed, flags);
  c10::DeviceGuard guard(x.device());
  auto [sv, sc] = block_sizes(c);
  Tensor save = bytes(sv, x), scratch = bytes(sc, x);
  Tensor out = at::empty({c.d.B, c.d.N, c.d.C, c.d.T}, f32(x));
  Tensor re_at = at::empty({c.d.B, c.d.F, c.d.n_heads, c.d.T, c.d.T}, f32(x));
  const float* ra = c.mode != DSTAGNN_RES_NONE ? res->data_ptr<float>() : nullptr;
  check_rc(dstagnn_block_forward(&c.d, &c.p, &c.g, x.data_ptr<float>(), ra, out.data_ptr<float>(),
                                 re_at.data_ptr<float>(), save.data_ptr(), sv, scratch.data_ptr(), sc, stream_of(x)),
           "dstagnn_block_forward");
  float ms = 0.f;
  check_rc(dstagnn_block_time_stage(&c.d, &c.p, &c.g, x.data_ptr<float>(), ra, out.data_ptr<float>(),
                                    re_at.data_ptr<float>(), save.data_ptr(), sv, scratch.data_ptr(), sc, (int)stage,
                                    (int)iters, &ms, stream_of(x)),
           "dstagnn_block_time_stage");
  return ms;
}

// the dropout keep-masks (1/(1-p) or 0) the block draws for `seed` on samples sample_base ..
// sample_base + B - 1 of the global batch: (after EmbedS (B,N,D), after fcmy (B,N,C,T))
std::tuple<Tensor, Tensor> dropout_masks(const Tensor& like, at::IntArrayRef shape, at::IntArrayRef cfg, double drop_p,
                                         int64_t seed, int64_t sample_base) {
  TORCH_CHECK(shape.size() == 4 && cfg.size() == 6, "dropout_masks: shape (B,N,F,T), cfg[6]");
  c10::DeviceGuard guard(like.device());
  dstagnn_block_dims d{};
  d.B = (int)shape[0]; d.N = (int)shape[1]; d.F = (int)shape[2]; d.T = (int)shape[3];
  d.n_heads = (int)cfg[0]; d.d_k = (int)cfg[1]; d.d_v = (int)cfg[2]; d.d_model = (int)cfg[3]; d.K = (int)cfg[4];
  d.C = (int)cfg[5];
  d.train = 1; d.drop_p = (float)drop_p; d.seed = (uint64_t)seed;
  TORCH_CHECK(sample_base >= 0, "dropout_masks: sample_base must be >= 0");
  d.sample_base = sample_base;
  Tensor m0 = at::empty({d.B, d.N, d.d_model}, f32(like));
  Tensor m1 = at::empty({d.B, d.N, d.C, d.T}, f32(like));
  check_rc(dstagnn_dropout_mask(&d, 0, m0.data_ptr<float>(), stream_of(like)), "dstagnn_dropout_mask");
  check_rc(dstagnn_dropout_mask(&d, 1, m1.data_ptr<float>(), stream_of(like)), "dstagnn_dropout_mask");
  return {m0, m1};
}

// -------------------------------------------------------------------------------------
// cheb_conv_withSAt operator pair
// -------------------------------------------------------------------------------------
constexpr int64_t kGemmWsBytes = int64_t(8) << 22;  // the library's split-K slab (8M floats)

// every size a kernel indexes by is checked here: the kernels trust them (an undersized
// support array would be an out-of-bounds device read)
dstagnn_graph graph_of(at::TensorList graph, bool sparse, int64_t K, int64_t N) {
  TORCH_CHECK(graph.size() == 2 || graph.size() == 6 || graph.size() == 15, "graph: 2, 6 or 15 tensors");
  dstagnn_graph g{};
  check_dev(graph[0], at::kFloat, "cheb");
  check_dev(graph[1], at::kFloat, "adj_pa");
  TORCH_CHECK(graph[0].numel() >= K * N * N, "cheb must hold K (N,N) polynomials: ", graph[0].sizes(), " for K=", K,
              " N=", N);
  TORCH_CHECK(graph[1].numel() == N * N, "adj_pa must be (N,N) for N=", N, ", got ", graph[1].sizes());
  g.cheb = graph[0].data_ptr<float>();
  g.adj_pa = graph[1].data_ptr<float>();
  if (graph.size() >= 6) {
    for (int i = 2; i < 6; ++i) check_dev(graph[i], at::kInt, "graph support");
    g.nnz = (int)graph[3].numel();
    TORCH_CHECK(graph[2].numel() == N + 1 && graph[4].numel() == N + 1, "graph support: csc_ptr / csr_ptr must have N+1 entries");
    TORCH_CHECK(graph[5].numel() == g.nnz, "graph support: csr_col and csc_row lengths differ");
    g.csc_ptr = graph[2].data_ptr<int>(); g.csc_row = graph[3].data_ptr<int>();
    g.csr_ptr = graph[4].data_ptr<int>(); g.csr_col = graph[5].data_ptr<int>();
  }
  if (graph.size() == 15) {  // csr2csc, apa_bits, apa_bits_t, apa_ptr, apa_row, tsupp, csc2csr, apa_idx, apa2t
    for (int i = 6; i < 11; ++i) check_dev(graph[i], at::kInt, "flash graph data");
    for (int i = 12; i < 15; ++i) check_dev(graph[i], at::kInt, "flash graph data");
    check_dev(graph[11], at::kFloat, "tsupp");
    const int64_t nw = (N + 31) / 32;
    TORCH_CHECK(graph[6].numel() == g.nnz, "flash graph data: csr2csc must have nnz entries");
    TORCH_CHECK(graph[7].numel() == N * nw && graph[8].numel() == N * nw,
                "flash graph data: apa_bits / apa_bits_t must be (N, ceil(N/32)) words");
    TORCH_CHECK(graph[9].numel() == N + 1, "flash graph data: apa_ptr must have N+1 entries");
    TORCH_CHECK(graph[11].numel() == K * (int64_t)g.nnz, "flash graph data: tsupp must be (K, nnz) for K=", K);
    g.csr2csc = graph[6].data_ptr<int>();
    g.apa_bits = graph[7].data_ptr<int32_t>();
    g.apa_bits_t = graph[8].data_ptr<int32_t>();
    g.apa_ptr = graph[9].data_ptr<int>();
    g.apa_row = graph[10].data_ptr<int>();
    g.apa_nnz = (int)graph[10].numel();
    g.tsupp = graph[11].data_ptr<float>();
    // the small-graph arrays (empty for larger graphs: the library then takes the streamed kernels)
    const bool small = graph[13].numel() > 0;
    if (small) {
      TORCH_CHECK(graph[12].numel() == g.nnz && graph[13].numel() == N * N && graph[14].numel() == g.apa_nnz,
                  "flash graph data: csc2csr (nnz), apa_idx (N,N), apa2t (apa_nnz)");
      g.csc2csr = graph[12].data_ptr<int>();
      g.apa_idx = graph[13].data_ptr<int>();
      g.apa2t = graph[14].data_ptr<int>();
    }
  }
  TORCH_CHECK(!sparse || g.nnz > 0, "sparse path requested without a CSC/CSR support");
  return g;
}

// x (B,N,F,T), sat (B,K,N,N), theta_cat (F,K*C), mask_cat (K,N,N) -> (out (B,N,C,T), P, W, xth)
std::tuple<Tensor, Tensor, Tensor, Tensor> cheb_sat_fwd(const Tensor& x, const Tensor& sat, const Tensor& theta_cat,
                                                        const Tensor& mask_cat, at::TensorList graph, int64_t C,
                                                        bool sparse) {
  for (auto [t, n] : {std::pair<const Tensor&, const char*>{x, "x"}, {sat, "sat"}, {theta_cat, "theta_cat"},
                      {mask_cat, "mask_cat"}})
    check_dev(t, at::kFloat, n);
  const int64_t B = x.size(0), N = x.size(1), F = x.size(2), T = x.size(3), K = sat.size(1);
  TORCH_CHECK(sat.sizes() == at::IntArrayRef({B, K, N, N}), "sat must be (B,K,N,N)");
  TORCH_CHECK(theta_cat.sizes() == at::IntArrayRef({F, K * C}), "theta_cat must be (F,K*C)");
  TORCH_CHECK(mask_cat.sizes() == at::IntArrayRef({K, N, N}), "mask_cat must be (K,N,N)");
  c10::DeviceGuard guard(x.device());
  dstagnn_graph g = graph_of(graph, sparse, K, N);
  Tensor out = at::empty({B, N, C, T}, f32(x));
  Tensor P = at::empty({B, K, N, N}, f32(x));
  Tensor W = sparse ? at::empty({0}, f32(x)) : at::empty({B, K, N, N}, f32(x));
  Tensor xth = at::empty({B, N, K, C, T}, f32(x));
  const int64_t ws = kGemmWsBytes + B * N * C * T * 4 + 1024;
  Tensor scratch = bytes(ws, x);
  check_rc(dstagnn_cheb_sat_forward((int)B, (int)N, (int)F, (int)T, (int)K, (int)C, sparse ? 1 : 0,
                                    x.data_ptr<float>(), sat.data_ptr<float>(), theta_cat.data_ptr<float>(),
                                    mask_cat.data_ptr<float>(), &g, out.data_ptr<float>(), P.data_ptr<float>(),
                                    sparse ? nullptr : W.data_ptr<float>(), xth.data_ptr<float>(), scratch.data_ptr(),
                                    ws, stream_of(x)),
           "dstagnn_cheb_sat_forward");
  return {out, P, W, xth};
}

// -> (d_x, d_sat, d_theta_cat, d_mask_cat)
std::tuple<Tensor, Tensor, Tensor, Tensor> cheb_sat_bwd(const Tensor& x, const Tensor& theta_cat, at::TensorList graph,
                                                        const Tensor& out, const Tensor& P, const Tensor& W,
                                                        const Tensor& xth, const Tensor& d_out, int64_t C,
                                                        bool sparse) {
  for (auto [t, n] : {std::pair<const Tensor&, const char*>{x, "x"}, {theta_cat, "theta_cat"}, {out, "out"},
                      {P, "P"}, {xth, "xth"}, {d_out, "d_out"}})
    check_dev(t, at::kFloat, n);
  const int64_t B = x.size(0), N = x.size(1), F = x.size(2), T = x.size(3), K = P.size(1);
  c10::DeviceGuard guard(x.device());
  dstagnn_graph g = graph_of(graph, sparse, K, N);
  Tensor dx = at::empty_like(x), dsat = at::empty({B, K, N, N}, f32(x));
  Tensor dth = at::empty({F, K * C}, f32(x)), dmask = at::empty({K, N, N}, f32(x));
  const int64_t nbig = B * N * C * T, nxth = B * N * K * C * T;
  const int64_t ws = kGemmWsBytes + (2 * nbig + nxth) * 4 + 2048;
  Tensor scratch = bytes(ws, x);
  check_rc(dstagnn_cheb_sat_backward((int)B, (int)N, (int)F, (int)T, (int)K, (int)C, sparse ? 1 : 0,
                                     x.data_ptr<float>(), theta_cat.data_ptr<float>(), &g, out.data_ptr<float>(),
                                     P.data_ptr<float>(), sparse ? nullptr : W.data_ptr<float>(),
                                     xth.data_ptr<float>(), d_out.data_ptr<float>(), dx.data_ptr<float>(),
                                     dsat.data_ptr<float>(), dth.data_ptr<float>(), dmask.data_ptr<float>(),
                                     scratch.data_ptr(), ws, stream_of(x)),
           "dstagnn_cheb_sat_backward");
  return {dx, dsat, dth, dmask};
}

// -------------------------------------------------------------------------------------
// strided GEMM: C = alpha A B + beta C (+ bias, ReLU); maps = 9 x (div, s0, s1) for
// a_m a_k a_z b_k b_n b_z c_m c_n c_z; offsets in elements from each tensor's data pointer
// -------------------------------------------------------------------------------------
void gemm_f32(const Tensor& A, const Tensor& B, const Tensor& C, at::IntArrayRef mnkb, at::IntArrayRef maps,
              at::IntArrayRef offs, double alpha, double beta, const c10::optional<Tensor>& bias, int64_t bias_stride,
              bool relu) {
  check_dev(A, at::kFloat, "A");
  check_dev(B, at::kFloat, "B");
  check_dev(C, at::kFloat, "C");
  TORCH_CHECK(mnkb.size() == 4 && maps.size() == 27 && offs.size() == 3, "gemm_f32: mnkb[4], maps[27], offs[3]");
  c10::DeviceGuard guard(C.device());
  dstagnn_gemm_desc d{};
  d.M = (int)mnkb[0]; d.N = (int)mnkb[1]; d.K = (int)mnkb[2]; d.batch = (int)mnkb[3];
  dstagnn_idx* ix[9] = {&d.a_m, &d.a_k, &d.a_z, &d.b_k, &d.b_n, &d.b_z, &d.c_m, &d.c_n, &d.c_z};
  for (int i = 0; i < 9; ++i) *ix[i] = dstagnn_idx{maps[3 * i], maps[3 * i + 1], maps[3 * i + 2]};
  d.A = A.data_ptr<float>(); d.a_off = offs[0];
  d.B = B.data_ptr<float>(); d.b_off = offs[1];
  d.C = C.data_ptr<float>(); d.c_off = offs[2];
  d.alpha = (float)alpha; d.beta = (float)beta;
  d.bias = ptr_or_null<float>(bias); d.bias_stride = bias_stride;
  d.relu = relu ? 1 : 0;
  Tensor ws = bytes(kGemmWsBytes + 256, C);
  check_rc(dstagnn_gemm_f32(&d, ws.data_ptr(), (size_t)ws.numel(), stream_of(C)), "dstagnn_gemm_f32");
}

// column sums: out[o] = sum_{a, i} in[a][o][i] over in viewed as (A, O, I), fixed order
Tensor colsum(const Tensor& in, int64_t O, int64_t I) {
  check_dev(in, at::kFloat, "in");
  TORCH_CHECK(O > 0 && I > 0 && in.numel() % (O * I) == 0, "colsum: numel must be a multiple of O*I");
  c10::DeviceGuard guard(in.device());
  Tensor out = at::zeros({O}, in.options());  // A = 0 sums to zero (the launcher writes nothing)
  Tensor ws = bytes((size_t(8) << 20) + 256, in);
  check_rc(dstagnn_colsum(in.data_ptr<float>(), in.numel() / (O * I), (int)O, (int)I, out.data_ptr<float>(), 1, 0.f,
                          ws.data_ptr(), (size_t)ws.numel(), stream_of(in)),
           "dstagnn_colsum");
  return out;
}

// -------------------------------------------------------------------------------------
// model head
// -------------------------------------------------------------------------------------
std::tuple<Tensor, Tensor> head_fwd(at::TensorList outs, const Tensor& w1, const Tensor& b1, const Tensor& w2,
                                    const Tensor& b2) {
  TORCH_CHECK(!outs.empty() && outs.size() <= DSTAGNN_HEAD_MAX_BLOCKS, "head: 1..16 block outputs");
  const Tensor& o0 = outs[0];
  const int64_t B = o0.size(0), N = o0.size(1), C = o0.size(2), T = o0.size(3), nb = outs.size();
  std::vector<const float*> op(nb);
  for (int64_t j = 0; j < nb; ++j) {
    check_dev(outs[j], at::kFloat, "block output");
    TORCH_CHECK(outs[j].sizes() == o0.sizes(), "head: block outputs differ in shape: ", outs[j].sizes(), " vs ",
                o0.sizes());
    op[j] = outs[j].data_ptr<float>();
  }
  for (auto [t, n] : {std::pair<const Tensor&, const char*>{w1, "final_conv.weight"}, {b1, "final_conv.bias"},
                      {w2, "final_fc.weight"}, {b2, "final_fc.bias"}})
    check_dev(t, at::kFloat, n);
  const int64_t O = w1.size(0), P = w2.size(0);
  TORCH_CHECK(w1.sizes() == at::IntArrayRef({O, nb * T, 1, C}), "Given weight of size ", w1.sizes(),
              ", expected input[", B, ", ", nb * T, ", ", N, ", ", C, "] to match final_conv (model/DSTAGNN_my.py:265)");
  TORCH_CHECK(w2.size(1) == O, "mat1 and mat2 shapes cannot be multiplied (", B * N, "x", O, " and ", w2.size(1), "x",
              P, ")");
  c10::DeviceGuard guard(o0.device());
  Tensor h = at::empty({B, N, O}, f32(o0)), y = at::empty({B, N, P}, f32(o0));
  const int64_t sb = dstagnn_head_scratch_bytes();
  Tensor sc = bytes(sb, o0);
  check_rc(dstagnn_head_forward((int)B, (int)N, (int)C, (int)T, (int)nb, (int)O, (int)P, op.data(),
                                w1.data_ptr<float>(), b1.data_ptr<float>(), w2.data_ptr<float>(), b2.data_ptr<float>(),
                                h.data_ptr<float>(), y.data_ptr<float>(), sc.data_ptr(), sb, stream_of(o0)),
           "dstagnn_head_forward");
  return {h, y};
}

// -> [dw1, db1, dw2, db2, d_out_0 .. d_out_{nb-1}]; entries whose `need` flag is 0 come back
// as empty (numel 0) tensors
std::vector<Tensor> head_bwd(at::TensorList outs, const Tensor& w1, const Tensor& w2, const Tensor& h,
                             const Tensor& dy_in, at::IntArrayRef need) {
  const Tensor& o0 = outs[0];
  const int64_t B = o0.size(0), N = o0.size(1), C = o0.size(2), T = o0.size(3), nb = outs.size();
  const int64_t O = w1.size(0), P = w2.size(0);
  TORCH_CHECK((int64_t)need.size() == 4 + nb, "head_bwd: need[4 + nb]");
  c10::DeviceGuard guard(o0.device());
  Tensor dy = dy_in.contiguous();
  check_dev(dy, at::kFloat, "dy");
  std::vector<const float*> op(nb);
  for (int64_t j = 0; j < nb; ++j) op[j] = outs[j].data_ptr<float>();
  auto maybe = [&](bool on, at::IntArrayRef shape) { return at::empty(on ? shape : at::IntArrayRef({0}), f32(o0)); };
  Tensor dh = at::empty({B, N, O}, f32(o0));
  std::vector<Tensor> r = {maybe(need[0], w1.sizes()), maybe(need[1], {O}), maybe(need[2], w2.sizes()),
                           maybe(need[3], {P})};
  std::vector<float*> dop(nb);
  for (int64_t j = 0; j < nb; ++j) {
    r.push_back(maybe(need[4 + j], o0.sizes()));
    dop[j] = need[4 + j] ? r.back().data_ptr<float>() : nullptr;
  }
  auto p = [&](int i) { return need[i] ? r[i].data_ptr<float>() : nullptr; };
  const int64_t sb = dstagnn_head_scratch_bytes();
  Tensor sc = bytes(sb, o0);
  check_rc(dstagnn_head_backward((int)B, (int)N, (int)C, (int)T, (int)nb, (int)O, (int)P, op.data(),
                                 w1.data_ptr<float>(), w2.data_ptr<float>(), h.data_ptr<float>(), dy.data_ptr<float>(),
                                 dh.data_ptr<float>(), dop.data(), p(0), p(1), p(2), p(3), sc.data_ptr(), sb,
                                 stream_of(o0)),
           "dstagnn_head_backward");
  return r;
}

// -------------------------------------------------------------------------------------
// optimiser: one Adam step over the listed tensors (optim.hip); the segment / chunk tables
// go through a pinned host buffer and an asynchronous copy on the current stream (the
// caching host allocator keeps the buffer alive until the copy has run)
// -------------------------------------------------------------------------------------
void adam_step(at::TensorList params, at::TensorList grads, at::TensorList exp_avgs, at::TensorList exp_avg_sqs,
               double beta1, double beta2, double eps, double step_size, double bc2_sqrt) {
  const size_t n = params.size();
  TORCH_CHECK(grads.size() == n && exp_avgs.size() == n && exp_avg_sqs.size() == n, "adam_step: list lengths differ");
  if (n == 0) return;
  c10::DeviceGuard guard(params[0].device());
  const int64_t ce = dstagnn_adam_chunk_elems();
  std::vector<dstagnn_adam_seg> segs(n);
  std::vector<Tensor> gcopy;  // contiguous copies of strided gradients, alive until the launch is queued
  gcopy.reserve(n);
  int64_t nchunk = 0;
  for (size_t i = 0; i < n; ++i) {
    const Tensor* g = &grads[i];
    if (g->defined() && g->is_cuda() && !g->is_contiguous()) {
      gcopy.push_back(g->contiguous());
      g = &gcopy.back();
    }
    for (const Tensor* t : {&params[i], g, &exp_avgs[i], &exp_avg_sqs[i]}) {
      check_dev(*t, at::kFloat, "adam_step tensor");
      TORCH_CHECK(t->device() == params[0].device(), "adam_step: tensors on different devices");
      TORCH_CHECK(t->numel() == params[i].numel(), "adam_step: param / grad / state sizes differ");
    }
    segs[i] = {params[i].data_ptr<float>(), g->data_ptr<float>(), exp_avgs[i].data_ptr<float>(),
               exp_avg_sqs[i].data_ptr<float>(), params[i].numel()};
    nchunk += (params[i].numel() + ce - 1) / ce;
  }
  TORCH_CHECK(nchunk < (1ll << 31), "adam_step: too many chunks");
  const size_t sb = n * sizeof(dstagnn_adam_seg), cb = (size_t)nchunk * 2 * sizeof(int64_t);
  Tensor host = at::empty({(int64_t)(sb + cb)}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
  uint8_t* hp = host.data_ptr<uint8_t>();
  std::memcpy(hp, segs.data(), sb);
  int64_t* ch = reinterpret_cast<int64_t*>(hp + sb);
  int64_t k = 0;
  for (size_t i = 0; i < n; ++i)
    for (int64_t off = 0; off < segs[i].n; off += ce) {
      ch[2 * k] = (int64_t)i;
      ch[2 * k + 1] = off;
      ++k;
    }
  Tensor dev = host.to(params[0].device(), /*non_blocking=*/true);
  const uint8_t* dp = dev.data_ptr<uint8_t>();
  check_rc(dstagnn_adam_step(reinterpret_cast<const dstagnn_adam_seg*>(dp), reinterpret_cast<const int64_t*>(dp + sb),
                             (int)nchunk, (float)beta1, (float)beta2, (float)eps, (float)step_size, (float)bc2_sqrt,
                             stream_of(params[0])),
           "dstagnn_adam_step");
}

// -------------------------------------------------------------------------------------
// graph builders (fp64)
// -------------------------------------------------------------------------------------
// data (T,N,F) -> (xhat (N,T,F), p (N,T), psum (N))
std::tuple<Tensor, Tensor, Tensor> stag_prep(const Tensor& data) {
  check_dev(data, at::kDouble, "data");
  TORCH_CHECK(data.dim() == 3, "data must be (T, N, F)");
  const int64_t T = data.size(0), N = data.size(1), F = data.size(2);
  c10::DeviceGuard guard(data.device());
  auto o = data.options();
  Tensor xhat = at::empty({N, T, F}, o), p = at::empty({N, T}, o), psum = at::empty({N}, o);
  check_rc(dstagnn_stag_prep(data.data_ptr<double>(), (int)T, (int)N, (int)F, xhat.data_ptr<double>(),
                             p.data_ptr<double>(), psum.data_ptr<double>(), stream_of(data)),
           "dstagnn_stag_prep");
  return {xhat, p, psum};
}

// pairs (P,2) int32 -> (emd (P) fp64, status (P) int32, pivots (P) int64 or empty)
std::tuple<Tensor, Tensor, Tensor> stag_emd_pairs(const Tensor& xhat, const Tensor& p, const Tensor& psum,
                                                  const Tensor& pairs, bool with_pivots) {
  check_dev(xhat, at::kDouble, "xhat");
  check_dev(p, at::kDouble, "p");
  check_dev(psum, at::kDouble, "psum");
  check_dev(pairs, at::kInt, "pairs");
  const int64_t N = xhat.size(0), T = xhat.size(1), F = xhat.size(2), P = pairs.size(0);
  c10::DeviceGuard guard(xhat.device());
  Tensor out = at::empty({P}, xhat.options());
  Tensor st = at::empty({P}, pairs.options());
  Tensor piv = at::empty({with_pivots ? P : 0}, pairs.options().dtype(at::kLong));
  check_rc(dstagnn_stag_emd_pairs(xhat.data_ptr<double>(), p.data_ptr<double>(), psum.data_ptr<double>(), (int)T,
                                  (int)N, (int)F, pairs.data_ptr<int32_t>(), P, out.data_ptr<double>(),
                                  st.data_ptr<int32_t>(), with_pivots ? piv.data_ptr<int64_t>() : nullptr,
                                  stream_of(xhat)),
           "dstagnn_stag_emd_pairs");
  return {out, st, piv};
}

int64_t stag_emd_lds_bytes(int64_t T, int64_t F) { return dstagnn_stag_emd_lds_bytes((int)T, (int)F); }

// p, q (B,T), D (B,T,T) -> (emd (B), status (B))
std::tuple<Tensor, Tensor> emd_dense(const Tensor& p, const Tensor& q, const Tensor& D) {
  check_dev(p, at::kDouble, "p");
  check_dev(q, at::kDouble, "q");
  check_dev(D, at::kDouble, "D");
  const int64_t B = p.size(0), T = p.size(1);
  TORCH_CHECK(q.sizes() == p.sizes() && D.numel() == B * T * T, "wasserstein_distance: p, q must be (B,T) and D (B,T,T)");
  c10::DeviceGuard guard(p.device());
  Tensor out = at::empty({B}, p.options()), st = at::empty({B}, p.options().dtype(at::kInt));
  check_rc(dstagnn_emd_dense(p.data_ptr<double>(), q.data_ptr<double>(), D.data_ptr<double>(), (int)T, B,
                             out.data_ptr<double>(), st.data_ptr<int32_t>(), stream_of(p)),
           "dstagnn_emd_dense");
  return {out, st};
}

// coords (N,Dc), feats (N,Fp) -> sta (N,N)
Tensor fast_stag_distances(const Tensor& coords, const Tensor& feats, double max_distance) {
  check_dev(coords, at::kDouble, "coords");
  check_dev(feats, at::kDouble, "feats");
  const int64_t N = coords.size(0);
  TORCH_CHECK(feats.size(0) == N, "coords and features disagree on the node count");
  c10::DeviceGuard guard(coords.device());
  Tensor sta = at::empty({N, N}, coords.options());
  check_rc(dstagnn_fast_stag_distances(coords.data_ptr<double>(), (int)N, (int)coords.size(1),
                                       feats.data_ptr<double>(), (int)feats.size(1), max_distance,
                                       sta.data_ptr<double>(), stream_of(coords)),
           "dstagnn_fast_stag_distances");
  return sta;
}

// sta (N,N) -> (A, R, nbr (N,k) int32)
std::tuple<Tensor, Tensor, Tensor> graph_topk(const Tensor& sta, int64_t k, int64_t mode) {
  check_dev(sta, at::kDouble, "sta");
  const int64_t N = sta.size(0);
  c10::DeviceGuard guard(sta.device());
  Tensor A = at::empty({N, N}, sta.options()), R = at::empty({N, N}, sta.options());
  Tensor nbr = at::empty({N, k}, sta.options().dtype(at::kInt));
  check_rc(dstagnn_graph_topk(sta.data_ptr<double>(), (int)N, (int)k, (int)mode, A.data_ptr<double>(),
                              R.data_ptr<double>(), nbr.data_ptr<int32_t>(), stream_of(sta)),
           "dstagnn_graph_topk");
  return {A, R, nbr};
}

int64_t library_version() { return dstagnn_version(); }

int64_t set_splitk_target(int64_t target) { return dstagnn_set_splitk_target((int)target); }
int64_t set_gemm_bf16(int64_t on) { return dstagnn_set_gemm_bf16((int)on); }

// GEMM-family profiling: prof_start(capacity); ...; prof_stop() ->
// [launches, flops, bytes, ms, max_ms, dropped]
void prof_start(int64_t capacity) { check_rc(dstagnn_prof_start((int)capacity), "dstagnn_prof_start"); }
std::vector<double> prof_stop() {
  dstagnn_prof_stats s{};
  check_rc(dstagnn_prof_stop(&s), "dstagnn_prof_stop");
  return {s.launches, s.flops, s.bytes, s.ms, s.max_ms, s.dropped};
}
// the last window's records one by one: [kind, flops, bytes, ms] * n
std::vector<double> prof_records() {
  const int n = dstagnn_prof_records(nullptr, 0);
  std::vector<dstagnn_prof_record> r((size_t)std::max(n, 0));
  if (n > 0) dstagnn_prof_records(r.data(), n);
  std::vector<double> out;
  out.reserve(4 * r.size());
  for (const auto& x : r) {
    out.push_back((double)x.kind);
    out.push_back(x.flops);
    out.push_back(x.bytes);
    out.push_back(x.ms);
  }
  return out;
}

}  // namespace

TORCH_LIBRARY(dstagnn, m) {
  m.class_<BlockPlan>("BlockPlan")
      .def(torch::init<std::vector<Tensor>, std::vector<int64_t>, std::vector<Tensor>, std::vector<int64_t>>());
  m.def("block_planned(Tensor x, Tensor? res_att, __torch__.torch.classes.dstagnn.BlockPlan plan, Tensor anchor, "
        "float drop_p, int seed, int flags) -> (Tensor, Tensor)");
#define DSTAGNN_BLK_ARGS \
  "Tensor x, Tensor? res_att, Tensor[] params, int[] slots, Tensor[] graph, int[] cfg, float drop_p, int seed, int flags"
  m.def("block(" DSTAGNN_BLK_ARGS ") -> (Tensor, Tensor)");
  m.def("block_fwd(" DSTAGNN_BLK_ARGS ") -> (Tensor, Tensor, Tensor)");
  m.def("block_bwd(Tensor x, Tensor? res_att, Tensor d_out, Tensor? d_re_at, Tensor save, Tensor[] params, "
        "int[] slots, Tensor[] graph, int[] cfg, float drop_p, int seed, int flags) -> (Tensor, Tensor, Tensor)");
  m.def("block_time_stage(" DSTAGNN_BLK_ARGS ", int stage, int iters) -> float");
  m.def("block_cheb_out(" DSTAGNN_BLK_ARGS ") -> Tensor");
  m.def("block_relu_out(" DSTAGNN_BLK_ARGS ", int which) -> Tensor");
  m.def("block_paths(" DSTAGNN_BLK_ARGS ") -> int");
#undef DSTAGNN_BLK_ARGS
  m.def("dropout_masks(Tensor like, int[] shape, int[] cfg, float drop_p, int seed, int sample_base=0) -> (Tensor, Tensor)");
  m.def("cheb_sat_fwd(Tensor x, Tensor sat, Tensor theta_cat, Tensor mask_cat, Tensor[] graph, int C, bool sparse) "
        "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def("cheb_sat_bwd(Tensor x, Tensor theta_cat, Tensor[] graph, Tensor out, Tensor P, Tensor W, Tensor xth, "
        "Tensor d_out, int C, bool sparse) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("gemm_f32(Tensor A, Tensor B, Tensor(a!) C, int[] mnkb, int[] maps, int[] offs, float alpha, float beta, "
        "Tensor? bias, int bias_stride, bool relu) -> ()");
  m.def("colsum(Tensor x, int O, int I) -> Tensor");
  m.def("head_fwd(Tensor[] outs, Tensor w1, Tensor b1, Tensor w2, Tensor b2) -> (Tensor, Tensor)");
  m.def("head_bwd(Tensor[] outs, Tensor w1, Tensor w2, Tensor h, Tensor dy, int[] need) -> Tensor[]");
  m.def("adam_step(Tensor(a!)[] params, Tensor[] grads, Tensor(b!)[] exp_avgs, Tensor(c!)[] exp_avg_sqs, "
        "float beta1, float beta2, float eps, float step_size, float bc2_sqrt) -> ()");
  m.def("stag_prep(Tensor data) -> (Tensor, Tensor, Tensor)");
  m.def("stag_emd_pairs(Tensor xhat, Tensor p, Tensor psum, Tensor pairs, bool with_pivots) -> (Tensor, Tensor, Tensor)");
  m.def("stag_emd_lds_bytes(int T, int F) -> int", stag_emd_lds_bytes);
  m.def("emd_dense(Tensor p, Tensor q, Tensor D) -> (Tensor, Tensor)");
  m.def("fast_stag_distances(Tensor coords, Tensor feats, float max_distance) -> Tensor");
  m.def("graph_topk(Tensor sta, int k, int mode) -> (Tensor, Tensor, Tensor)");
  m.def("version() -> int", library_version);
  m.def("prof_start(int capacity) -> ()", prof_start);
  m.def("set_splitk_target(int target) -> int", set_splitk_target);
  m.def("set_gemm_bf16(int on) -> int", set_gemm_bf16);
  m.def("prof_stop() -> float[]", prof_stop);
  m.def("prof_records() -> float[]", prof_records);
}

// PyTorch-ROCm dispatches HIP device tensors under the CUDA key
TORCH_LIBRARY_IMPL(dstagnn, CUDA, m) {
  m.impl("block", block_infer);
  m.impl("block_planned", block_planned_infer);
  m.impl("block_fwd", block_fwd);
  m.impl("block_bwd", block_bwd);
  m.impl("block_time_stage", block_time_stage);
  m.impl("dropout_masks", dropout_masks);
  m.impl("block_cheb_out", block_cheb_out);
  m.impl("block_relu_out", block_relu_out);
  m.impl("block_paths", block_paths);
  m.impl("cheb_sat_fwd", cheb_sat_fwd);
  m.impl("cheb_sat_bwd", cheb_sat_bwd);
  m.impl("gemm_f32", gemm_f32);
  m.impl("colsum", colsum);
  m.impl("head_fwd", head_fwd);
  m.impl("head_bwd", head_bwd);
  m.impl("adam_step", adam_step);
  m.impl("stag_prep", stag_prep);
  m.impl("stag_emd_pairs", stag_emd_pairs);
  m.impl("emd_dense", emd_dense);
  m.impl("fast_stag_distances", fast_stag_distances);
  m.impl("graph_topk", graph_topk);
}

TORCH_LIBRARY_IMPL(dstagnn, Autograd, m) {
  m.impl("block", block_autograd);
  m.impl("block_planned", block_planned_autograd);
}
