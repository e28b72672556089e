"""torch_xla.distributed.parallel_loader.MpDeviceLoader (train_DSTAGNN_my.py:113-115): the wrapped
loader's batches copied to the device (non-blocking from pinned memory when the loader pins).
Like the reference under xmp.spawn, every replica iterates its own loader over the same data
(quirk 15); train.fit / dp.shard_batch are the sharded path."""
import torch


def _to(x, device):
    if torch.is_tensor(x):
        return x.to(device, non_blocking=True)
    if isinstance(x, (list, tuple)):
        return type(x)(_to(v, device) for v in x)
    if isinstance(x, dict):
        return {k: _to(v, device) for k, v in x.items()}
    return x


class MpDeviceLoader:
    def __init__(self, loader, device, **kwargs):
        self._loader = loader
        self._device = device

    def __iter__(self):
        for batch in self._loader:
            yield _to(batch, self._device)

    def __len__(self):
        return len(self._loader)


class ParallelLoader:
    def __init__(self, loader, devices, **kwargs):
        self._loader = loader
        self._devices = list(devices)

    def per_device_loader(self, device):
        return MpDeviceLoader(self._loader, device)
