"""CPU: the index data of the sparse and fused (flash) Chebyshev paths (model.support_index,
model.flash_support) against brute-force definitions."""
import torch

from dstagnn_drought_amd.model import flash_support, support_index


def _case(N=50, seed=0):
    g = torch.Generator().manual_seed(seed)
    cs = (torch.rand(3, N, N, generator=g) < 0.05).float() * torch.rand(3, N, N, generator=g)
    cs[0] += torch.eye(N)  # T_0 = I, as cheb_polynomial builds it
    apa = (torch.rand(N, N, generator=g) < 0.08).float() * 2.0
    return cs, apa


def test_support_index_is_the_union_support():
    cs, _ = _case()
    N = cs.shape[1]
    cp, cr, rp, rc = support_index(cs)
    nz = (cs != 0).any(0)
    for j in range(N):
        assert torch.equal(cr[cp[j]:cp[j + 1]].long(), torch.nonzero(nz[:, j]).reshape(-1))
        assert torch.equal(rc[rp[j]:rp[j + 1]].long(), torch.nonzero(nz[j, :]).reshape(-1))
    assert int(cp[-1]) == int(rp[-1]) == int(nz.sum())


def test_flash_support_maps_and_bits():
    cs, apa = _case(N=70, seed=3)  # N not a multiple of 32: partial last bit word
    N = cs.shape[1]
    cp, cr, rp, rc = support_index(cs)
    f = flash_support(cs, cp, cr, rp, rc, apa)
    for i in range(N):  # csr2csc: CSR entry (i, j) -> its CSC position in column j
        for q in range(int(rp[i]), int(rp[i + 1])):
            j, p = int(rc[q]), int(f["csr2csc"][q])
            assert int(cp[j]) <= p < int(cp[j + 1]) and int(cr[p]) == i
    ccol = torch.repeat_interleave(torch.arange(N), (cp[1:] - cp[:-1]).long())
    assert torch.equal(f["tsupp"], cs[:, cr.long(), ccol])
    bits, bt = f["apa_bits"], f["apa_bits_t"]
    assert bits.dtype == torch.int32 and bits.shape == (N, (N + 31) // 32)
    for i in range(N):
        for j in range(N):
            assert ((int(bits[i, j // 32]) >> (j % 32)) & 1) == int(apa[i, j] != 0)
            assert ((int(bt[j, i // 32]) >> (i % 32)) & 1) == int(apa[i, j] != 0)
    ap, ar = f["apa_ptr"], f["apa_row"]
    for j in range(N):
        assert torch.equal(ar[ap[j]:ap[j + 1]].long(), torch.nonzero(apa[:, j] != 0).reshape(-1))
