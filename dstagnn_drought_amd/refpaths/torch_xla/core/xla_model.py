"""torch_xla.core.xla_model over the HIP device and torch.distributed (see torch_xla/__init__.py).

Calls of train_DSTAGNN_my.py served here (file:line of the reference script):
  xrt_world_size   :25      xla_device        :33     is_master_ordinal :127, :161, :173, :183
  optimizer_step   :148, :158 (the gradient all-reduce + Adam step; quirk 14: called twice)
  master_print     :151     get_memory_info   :153    save              :180
"""
import os

import torch
import torch.distributed as dist

_reducers = {}  # id(optimizer) -> (param ids, GradAllReducer)


def _dist_on():
    return dist.is_available() and dist.is_initialized()


def xrt_world_size():
    """Number of replicas: the torch.distributed world (or WORLD_SIZE before initialisation)."""
    if _dist_on():
        return dist.get_world_size()
    return int(os.environ.get("WORLD_SIZE", "1"))


def get_ordinal():
    if _dist_on():
        return dist.get_rank()
    return int(os.environ.get("RANK", "0"))


def get_local_ordinal():
    return int(os.environ.get("LOCAL_RANK", "0"))


def is_master_ordinal(local=True):
    return (get_local_ordinal() if local else get_ordinal()) == 0


def xla_device(n=None, devkind=None):
    """The HIP device of this process (cuda:LOCAL_RANK, or cuda:n).  Under a multi-process launch
    (WORLD_SIZE > 1: xmp.spawn below or torch.distributed.run) the process group is initialised
    here on RCCL ("nccl", device_id bound, as bench.py does); DSTAGNN_DIST_BACKEND=gloo for tests.
    There is no CPU fallback: without a HIP device this raises."""
    if not torch.cuda.is_available():
        raise RuntimeError("xla_device: no HIP device (the MI355X build has no CPU path)")
    idx = get_local_ordinal() if n is None else int(n)
    dev = torch.device("cuda", idx)
    torch.cuda.set_device(dev)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not _dist_on():
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        backend = os.environ.get("DSTAGNN_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return dev


def _reducer_for(optimizer):
    """One GradAllReducer per optimiser, over its parameters (built on first use; the cheb mask
    gradients travel as their A_pa support only on large graphs, dp.py)."""
    params = [p for g in optimizer.param_groups for p in g["params"]]
    key = id(optimizer)
    ids = tuple(id(p) for p in params)
    hit = _reducers.get(key)
    if hit is not None and hit[0] == ids:
        return hit[1]
    from dstagnn_drought_amd.dp import GradAllReducer
    named = [(f"p{i}", p) for i, p in enumerate(params)]
    red = GradAllReducer(named)
    _reducers[key] = (ids, red)
    return red


def reduce_gradients(optimizer, groups=None, pin_layout=True):
    """Mean all-reduce of the optimiser's gradients over the replicas (no-op at world 1).  With
    WORLD_SIZE > 1 but no process group (xla_device() not called first, or called before the
    launcher's environment was set) this raises: the replicas would otherwise step on their own
    unreduced gradients and drift apart silently."""
    if xrt_world_size() > 1:
        if not _dist_on():
            raise RuntimeError("xm.optimizer_step / reduce_gradients: WORLD_SIZE > 1 but the process group is not "
                               "initialised (call xm.xla_device() first, as train_DSTAGNN_my.py:33 does)")
        _reducer_for(optimizer).all_reduce()


def optimizer_step(optimizer, barrier=False, optimizer_args=None, groups=None, pin_layout=True):
    """xm.optimizer_step: reduce_gradients + optimizer.step(**optimizer_args).  `barrier` cuts an
    XLA graph (mark_step) there; the HIP ops run eagerly and asynchronously on the stream, so
    there is nothing to cut.  Returns what optimizer.step returns."""
    reduce_gradients(optimizer, groups=groups)
    return optimizer.step(**(optimizer_args or {}))


def mark_step(wait=False):
    """Graph cut in XLA; nothing to do on the eager HIP path (wait=True synchronises)."""
    if wait and torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


def wait_device_ops(devices=None):
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


def rendezvous(tag, payload=b"", replicas=None):
    if _dist_on():
        dist.barrier()
    return [payload]


def master_print(*args, fd=None, finalize=False, **kw):
    if is_master_ordinal(local=False):
        print(*args, file=fd, **kw)


def get_memory_info(device):
    """{'kb_free', 'kb_total'} of the device, as torch_xla reports it (hipMemGetInfo)."""
    free, total = torch.cuda.mem_get_info(device)
    return {"kb_free": free // 1024, "kb_total": total // 1024}


def _to_cpu(data):
    if torch.is_tensor(data):
        return data.detach().cpu()
    if isinstance(data, dict):
        return type(data)((k, _to_cpu(v)) for k, v in data.items())
    if isinstance(data, (list, tuple)):
        return type(data)(_to_cpu(v) for v in data)
    return data


def save(data, file_or_path, master_only=True, global_master=False):
    """xm.save: tensors moved to the CPU, written by the master ordinal only (torch.save format;
    the reference reloads it with torch.load, :184).  No collective: the reference calls save
    from inside `if xm.is_master_ordinal():` (train_DSTAGNN_my.py:173-180), so a barrier here
    would pair the master's barrier with the other ranks' next gradient all-reduce (a hang, or a
    mismatched RCCL collective).  Callers that need the file visible to every rank
    synchronise themselves (xm.rendezvous)."""
    master = is_master_ordinal(local=not global_master)
    if master or not master_only:
        torch.save(_to_cpu(data), file_or_path)
