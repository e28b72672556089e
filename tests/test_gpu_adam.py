"""GPU: HipAdam (one launch of csrc/optim.hip over every parameter) against torch.optim.Adam
with the reference's construction (train_DSTAGNN_my.py:126: lr only, default betas / eps) on
the same parameters and gradients: odd tensor sizes (chunk tails), gradients that are views at
unaligned offsets of one flat buffer (how the block's direct gradients arrive), a parameter
whose gradient is None for a step (its step count then lags: a second launch), six steps.
Bound: |p_hip - p_torch| <= 1e-6 * max(1, |p|) elementwise (the same fp32 formula; torch's
default implementation orders the bias corrections differently, a few ulp apart)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_hip_adam_matches_torch_adam():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from dstagnn_drought_amd.train import HipAdam
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    shapes = [(7,), (4096,), (4097,), (33, 65), (3, 170, 170), (512, 384), (1,)]
    base = [torch.randn(s, device=dev, generator=g) for s in shapes]
    pa = [torch.nn.Parameter(t.clone()) for t in base]
    pb = [torch.nn.Parameter(t.clone()) for t in base]
    oa = HipAdam(pa, lr=1e-3)
    ob = torch.optim.Adam(pb, lr=1e-3, foreach=False)
    total = sum(t.numel() for t in base)
    for step in range(6):
        flat = torch.randn(total + 3, device=dev, generator=g)  # views at offsets not multiples of 4
        off = 3
        for i, (a, b) in enumerate(zip(pa, pb)):
            n = a.numel()
            gr = flat[off:off + n].view(a.shape)
            off += n
            if step == 2 and i == 3:
                a.grad = None
                b.grad = None
            else:
                a.grad = gr
                b.grad = gr.clone()
        oa.step()
        ob.step()
    for a, b in zip(pa, pb):
        err = (a.detach() - b.detach()).abs()
        bound = 1e-6 * torch.clamp(b.detach().abs(), min=1.0)
        assert bool((err <= bound).all()), float(err.max())
    assert oa.state[pa[3]]["step"] == 5 and oa.state[pa[0]]["step"] == 6
