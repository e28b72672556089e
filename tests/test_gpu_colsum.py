"""Stress test of the column-sum reduction behind every bias / LayerNorm gamma-beta gradient
of the block (model/DSTAGNN_my.py:207,220,252: the reductions autograd does for nn.Linear /
nn.Conv2d biases and nn.LayerNorm's affine parameters), called through dstagnn_colsum.

The one-launch path hands partial sums between workgroups through an in-kernel ticket
(ops.hip colsum2d_kernel): a stale read would show up as a wrong or
launch-to-launch varying sum.  Every shape is launched many times back to back on one
stream and each result must be (1) bit-identical to the first launch (fixed summation
order) and (2) within fp32 rounding of an fp64 sum: |err| <= 1e-6 * sum|x| per column.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (A, O, I): the block's shapes (PEMS08 B=32: LN over N=170 rows of B*T*F, bias over C,
# fcmy bias over T) plus ragged / single-row / wide-group / two-stage (I > 256) edge cases
SHAPES = [
    (32 * 12 * 32, 170, 1), (32 * 170 * 32, 12, 1), (5440, 64, 1), (12288, 96, 1), (1, 170, 1),
    (7, 3, 5), (100003, 17, 1), (4096, 1000, 1), (333, 40, 16), (2048, 8, 300), (65280, 32, 1),
    (0, 5, 1),
]


@pytest.mark.parametrize("A,O,I", SHAPES)
def test_colsum_repeated_launches(A, O, I):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from dstagnn_drought_amd import _lib
    ops = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(A * 131 + O * 7 + I)
    x = torch.randn(A, O, I, generator=g).cuda()
    ref = x.double().sum(dim=(0, 2)).cpu()
    bound = 1e-6 * x.double().abs().sum(dim=(0, 2)).cpu() + 1e-30
    outs = [ops.colsum(x, O, I) for _ in range(40)]
    torch.cuda.synchronize()
    first = outs[0].cpu()
    assert ((first.double() - ref).abs() <= bound).all(), float((first.double() - ref).abs().max())
    for k, o in enumerate(outs[1:], 1):
        assert torch.equal(o.cpu(), first), f"launch {k} differs from launch 0"


def test_colsum_interleaved_shapes():
    """Different shapes back to back reuse the stream's ticket counters: every launch must
    leave them zero for the next one."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from dstagnn_drought_amd import _lib
    ops = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(5)
    xs = [torch.randn(a, o, i, generator=g).cuda() for a, o, i in SHAPES[:6]]
    want = [ops.colsum(x, x.shape[1], x.shape[2]).cpu() for x in xs]
    for _ in range(10):
        got = [ops.colsum(x, x.shape[1], x.shape[2]) for x in xs]
        for w, o in zip(want, got):
            assert torch.equal(o.cpu(), w)
