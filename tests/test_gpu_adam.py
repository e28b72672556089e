"""GPU: HipAdam (one launch of csrc/optim.hip over every parameter) against torch.optim.Adam
with the reference's construction (train_DSTAGNN_my.py:126: lr only, default betas / eps) on
the same parameters and gradients: odd tensor sizes (chunk tails), gradients that are views at
unaligned offsets of one flat buffer (how the block's direct gradients arrive), a parameter
whose gradient is None for a step (its step count then lags: a second launch), a strided
(transposed) gradient, six steps; then the cached one-launch path (every parameter with a
gradient, one shared step count) over further steps, and after a load_state_dict.
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
            if step == 4 and i == 3:
                gr = flat[off:off + n].view(a.shape[1], a.shape[0]).t()
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


def test_hip_adam_cached_path_matches_torch_adam():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from dstagnn_drought_amd.train import HipAdam
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(4)
    shapes = [(5,), (4099,), (31, 17), (2, 64, 64)]
    base = [torch.randn(s, device=dev, generator=g) for s in shapes]
    pa = [torch.nn.Parameter(t.clone()) for t in base]
    pb = [torch.nn.Parameter(t.clone()) for t in base]
    oa = HipAdam(pa, lr=1e-3)
    ob = torch.optim.Adam(pb, lr=1e-3, foreach=False)

    def run(steps, strided_at=-1):
        for step in range(steps):
            for i, (a, b) in enumerate(zip(pa, pb)):
                gr = torch.randn(a.shape, device=dev, generator=g)
                if step == strided_at and i == 2:
                    gr = torch.randn(a.shape[1], a.shape[0], device=dev, generator=g).t()
                a.grad = gr
                b.grad = gr.clone()
            oa.step()
            ob.step()

    run(5, strided_at=3)
    assert oa._plans, "cached path not taken"
    oa.load_state_dict(oa.state_dict())
    assert not oa._plans
    run(4)
    for a, b in zip(pa, pb):
        err = (a.detach() - b.detach()).abs()
        bound = 1e-6 * torch.clamp(b.detach().abs(), min=1.0)
        assert bool((err <= bound).all()), float(err.max())
    assert all(oa.state[p]["step"] == 9 for p in pa)
    assert all(torch.equal(oa.state[a]["exp_avg"], ob.state[b]["exp_avg"]) or
               bool(torch.allclose(oa.state[a]["exp_avg"], ob.state[b]["exp_avg"], rtol=1e-6, atol=1e-7))
               for a, b in zip(pa, pb))
