"""Data parallelism for DSTAGNN: one process per GPU, batch sharded
across ranks, ONE exchange step per iteration — the gradient all-reduce that
`xm.optimizer_step` performs in the reference (train_DSTAGNN_my.py:148,158) — done
with torch.distributed over RCCL (backend "nccl" on ROCm) across xGMI.

Design for MI355X / xGMI:
  * gradients are packed into a few large flat fp32 buckets (default 32 MB) so each
    RCCL call is bandwidth-bound on the point-to-point xGMI links, not latency-bound;
  * parameters whose .grad is None (inner blocks' EmbedT / residual_conv, quirk 11)
    are skipped identically on every rank (the set is fixed by the module structure);
  * cheb_conv_SAt.mask.k gradients are non-zero only on adj_pa's support
    (dM_k = A_pa o sum_b dz), so only those nnz values travel (92 % of the bytes at
    the SYN config); the off-support zeros are restored locally;
  * overlap: with attach(), each block's flat gradient buffer is all-reduced asynchronously
    the moment that block's backward finishes, beside the remaining blocks' backward;
  * the reference shards nothing (all replicas see the same batch, quirk 15): here each
    rank takes a disjoint slice of the global batch (shard_batch).
"""
import torch
import torch.distributed as dist


def shard_start(B, rank, world):
    """Global index of the first sample of `rank`'s shard of a B-sample batch (shard_batch)."""
    per = (B + world - 1) // world
    return min(B, rank * per)


def shard_batch(t, rank, world, model=None):
    """Disjoint contiguous slice of the leading (batch) dim for `rank` (ceil(B/world) samples per
    rank, the last shard shorter).  With `model`, its blocks' dropout sample base is set to the
    shard's true global offset (model.set_sample_base): the default base, rank * local_B, is
    right only for equal shards (B=5 over 2 ranks: rank 1 starts at 3, not 2).  That base is
    STICKY: it holds for every later call of the model until reset — pass `model` on every
    sharded call, or use `sharded(...)` below, which restores the previous base on exit."""
    B = t.shape[0]
    per = (B + world - 1) // world
    start = shard_start(B, rank, world)
    if model is not None:
        from .model import set_sample_base
        set_sample_base(model, start)
    return t[start:min(B, (rank + 1) * per)]


class sharded:
    """``with dp.sharded(x, rank, world, model) as xs:`` — shard_batch with the model's dropout
    sample base set to the shard's global offset for the block only; on exit every block's
    previous base comes back (None: the default rank * B), so a later full-batch or differently
    sharded call cannot key its masks from a stale offset."""

    def __init__(self, t, rank, world, model):
        self.t, self.rank, self.world, self.model = t, rank, world, model

    def __enter__(self):
        from .model import DSTAGNN_block
        self._saved = [(m, m.sample_base) for m in self.model.modules() if isinstance(m, DSTAGNN_block)]
        return shard_batch(self.t, self.rank, self.world, model=self.model)

    def __exit__(self, *exc):
        for m, base in self._saved:
            m.sample_base = base
        return False


class GradAllReducer:
    """Bucketed mean all-reduce of parameter gradients with sparse mask payloads."""

    def __init__(self, named_params, mask_support=None, bucket_bytes=32 << 20, group=None,
                 dense_limit=256 << 20):
        """named_params: iterable of (name, Parameter).  mask_support: dict name -> bool (N,N)
        tensor (adj_pa > 0) for cheb mask params whose grads are supported there only.
        dense_limit: a block's flat gradient buffer up to this size is all-reduced whole
        (mask grads included, dense); larger ones (N = 4096: the masks are 1.3 GB) go through
        the bucketed path that sends the masks as their support only."""
        self.group = group
        self.dense_limit = dense_limit
        self.items = []  # (param, index or None)
        sup = mask_support or {}
        for n, p in named_params:
            idx = None
            if n in sup:
                idx = torch.nonzero(sup[n].reshape(-1).to(p.device), as_tuple=False).reshape(-1)
            self.items.append((n, p, idx))
        self.bucket_elems = max(1, bucket_bytes // 4)
        self._inflight = []  # (flat gradient buffer, async work) started during the backward
        self._avg = None     # RCCL averages in the collective itself (ncclAvg): no scale kernel

    def _mean_op(self):
        """(op, scale-after?) of a mean all-reduce: AVG on the nccl (RCCL) backend, SUM and a
        division elsewhere (gloo has no AVG)."""
        if self._avg is None:
            self._avg = dist.get_backend(self.group) == "nccl"
        return (dist.ReduceOp.AVG, False) if self._avg else (dist.ReduceOp.SUM, True)

    def _mean(self, t, world, async_op=False):
        op, scale = self._mean_op()
        work = dist.all_reduce(t, op=op, group=self.group, async_op=async_op)
        if not async_op and scale and world > 1:
            t.div_(world)
        return work

    def attach(self, model):
        """Overlap the exchange with the backward: every DSTAGNN_block of `model` in
        direct-grad mode hands its gradients over the moment its backward node has run (a
        post-hook on the dstagnn::block node, model.DSTAGNN_block.grads_ready); their flat
        buffer's all-reduce is issued asynchronously there (RCCL runs it on its own stream
        beside the next block's backward kernels).  all_reduce() then waits for those and
        reduces what is left (the head's grads)."""
        from .model import DSTAGNN_block
        for m in model.modules():
            if isinstance(m, DSTAGNN_block):
                m.grads_ready = self.on_grads_ready
        return self

    @staticmethod
    def block_flat_grad(block):
        """The one flat buffer the HIP backward packed this block's gradients into (their
        common ``_base``), or None when the gradients are not exactly that (accumulated into
        pre-existing tensors, or not written directly)."""
        if not block.direct_grads:
            return None  # AccumulateGrad has not run yet when the node's post-hook fires
        base, n = None, 0
        for p in block.parameters():
            g = p.grad
            if g is None:
                continue
            b = g._base
            if b is None or (base is not None and b is not base):
                return None
            base, n = b, n + g.numel()
        if base is None or n != base.numel() or not base.is_contiguous():
            return None
        return base

    def on_grads_ready(self, block):
        flat = self.block_flat_grad(block)
        if flat is None or flat.numel() * 4 > self.dense_limit:
            return  # reduced by all_reduce() (masks as their support only on the large graphs)
        if any(f.data_ptr() == flat.data_ptr() for f, _ in self._inflight):
            return
        work = self._mean(flat, dist.get_world_size(self.group), async_op=True)
        self._inflight.append((flat, work))

    def _payload(self, p, idx):
        g = p.grad.reshape(-1)
        return g if idx is None else g.index_select(0, idx)

    def _flat_groups(self, live):
        """Gradients that exactly tile one flat base tensor (the HIP block's backward packs a
        block's parameter gradients back to back into one buffer): reduce the base itself —
        one collective and one scale, no pack / unpack kernels."""
        by_base = {}
        for it in live:
            g = it[1].grad
            b = g._base
            if b is None or not b.is_contiguous() or not g.is_contiguous():
                continue
            by_base.setdefault(id(b), (b, []))[1].append(it)
        groups, taken = [], set()
        for b, its in by_base.values():
            if sum(it[1].grad.numel() for it in its) != b.numel() or b.numel() * 4 > self.dense_limit:
                continue
            groups.append(b)
            taken.update(id(it[1]) for it in its)
        return groups, taken

    def all_reduce(self):
        world = dist.get_world_size(self.group)
        done = set()
        for flat, work in self._inflight:  # started during the backward (attach)
            work.wait()
            if self._mean_op()[1] and world > 1:
                flat.div_(world)
            done.add(flat.data_ptr())
        self._inflight.clear()
        live = [(n, p, idx) for n, p, idx in self.items if p.grad is not None]
        bases, taken = self._flat_groups(live)
        for b in bases:
            if b.data_ptr() in done:
                continue
            self._mean(b, world)
        live = [it for it in live if id(it[1]) not in taken]
        buckets, cur, size = [], [], 0
        for it in live:
            k = it[1].numel() if it[2] is None else it[2].numel()
            if cur and size + k > self.bucket_elems:
                buckets.append(cur)
                cur, size = [], 0
            cur.append(it)
            size += k
        if cur:
            buckets.append(cur)
        for b in buckets:
            flat = torch.cat([self._payload(p, idx) for _, p, idx in b])
            self._mean(flat, world)
            off = 0
            for _, p, idx in b:
                g = p.grad.view(-1)
                if idx is None:
                    k = g.numel()
                    g.copy_(flat[off:off + k])
                else:
                    k = idx.numel()
                    g.zero_()
                    g.index_copy_(0, idx, flat[off:off + k])
                off += k
        return len(buckets) + len(bases)

    def payload_bytes(self):
        return 4 * sum((p.numel() if idx is None else idx.numel()) for _, p, idx in self.items)


def mask_support_of(model):
    """{param name: adj_pa > 0} for every cheb_conv_SAt.mask.k of a DSTAGNN model/block."""
    sup = {}
    for mn, mod in model.named_modules():
        if hasattr(mod, "cheb_conv_SAt") and hasattr(mod, "adj_pa"):
            s = (mod.adj_pa > 0)
            for k in range(len(mod.cheb_conv_SAt.mask)):
                name = (mn + "." if mn else "") + f"cheb_conv_SAt.mask.{k}"
                sup[name] = s
    return sup
