"""torch_xla.distributed.xla_multiprocessing.spawn (train_DSTAGNN_my.py:195-197): one process per
GPU with the torch.distributed environment set (MASTER_ADDR 127.0.0.1, a free port, RANK =
LOCAL_RANK = index, WORLD_SIZE = nprocs); xm.xla_device() in the child then binds its GPU and
initialises the process group on RCCL.  fn(index, *args) as torch_xla calls it (a zero-argument
fn, like the reference's main, is called without the index)."""
import inspect
import os
import socket

import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(index, fn, args, nprocs, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(index), LOCAL_RANK=str(index),
                      WORLD_SIZE=str(nprocs), HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        takes_index = len(inspect.signature(fn).parameters) > len(args)
    except (TypeError, ValueError):
        takes_index = True
    try:
        fn(index, *args) if takes_index else fn(*args)
    finally:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.destroy_process_group()


def spawn(fn, args=(), nprocs=None, join=True, daemon=False, start_method="spawn"):
    """nprocs=None: every visible GPU.  A 'fork' start method is honoured only while this process
    has not initialised the GPU (a forked child cannot use the parent's HIP context)."""
    if nprocs is None:
        nprocs = max(1, torch.cuda.device_count())
    if start_method == "fork" and torch.cuda.is_initialized():
        start_method = "spawn"
    return mp.start_processes(_entry, args=(fn, tuple(args), nprocs, _free_port()), nprocs=nprocs, join=join,
                              daemon=daemon, start_method=start_method)
