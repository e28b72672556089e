"""tensorboardX.SummaryWriter for train_DSTAGNN_my.py:16, which imports it and never uses it: a no-op
writer (TensorBoard logging is out of scope)."""


class SummaryWriter:
    def __init__(self, logdir=None, *args, **kwargs):
        self.logdir = logdir

    def __getattr__(self, name):  # add_scalar, add_histogram, flush, ...: accepted and ignored
        if name.startswith("add_") or name in ("flush", "close"):
            return lambda *a, **k: None
        raise AttributeError(name)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False
