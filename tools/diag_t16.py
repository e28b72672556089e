import os, sys
ROOT = "/root/repo" if os.path.exists("/root/repo/tests") else os.getcwd()
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch, numpy as np
import test_gpu_parity as T
import dstagnn_drought_amd as D_
name, first, B, rk = sys.argv[1], sys.argv[2] == "1", int(sys.argv[3]), int(sys.argv[4])
N, Tt, K, h, D, dk, C = T.CONFIGS[name]
ref, p, x, res, cheb, apa, dims, gen = T._oracle_case(B, N, Tt, K, h, D, dk, C, first, rk, seed=3)
g_out = torch.randn(B, N, C, Tt, generator=gen)
g_re = torch.randn(B, x.shape[2], h, Tt, Tt, generator=gen)
F = x.shape[2]
blk = D_.DSTAGNN_block("cpu", F, F, K, C, C, 1, cheb, apa, apa, N, Tt, D, dk, dk, h)
blk.load_state_dict(p); blk = blk.cuda().eval()
xg = x.cuda().requires_grad_(True)
rg = res.cuda().requires_grad_(True) if torch.is_tensor(res) else 0
masks = T.hip_relu_masks(blk, xg, rg)
d64 = lambda t: t.double() if torch.is_tensor(t) else t
o = ref.block_forward_backward({k: d64(v) for k, v in p.items()}, d64(x), d64(res), [d64(c) for c in cheb], d64(apa), dims, d64(g_out), d64(g_re), relu_mask=masks[0], tail_masks=masks[1:])
out, re_at = blk(xg, rg)
((out * g_out.cuda()).sum() + (re_at * g_re.cuda()).sum()).backward()
gr = o[4]
for n in ("TAt.W_Q.weight", "TAt.W_K.weight", "TAt.W_V.weight"):
    a = dict(blk.named_parameters())[n].grad.double().cpu(); b = gr[n]
    e = (a - b).abs()
    print(n, "per head:", [f"{float(e[hh*dk:(hh+1)*dk].max()):.2e}" for hh in range(h)], "scale", f"{float(b.abs().max()):.2e}")
    # per d within head 0
    print("   per d (head0..2, max over n):", " ".join(f"{float(e[dd].max()):.0e}" for dd in range(h*dk)))
ex = (xg.grad.double().cpu() - o[2]).abs()  # (B,N,F,T)
print("grad_x err per t:", [f"{float(ex[..., t].max()):.1e}" for t in range(Tt)])
print("grad_x err per b:", [f"{float(ex[b].max()):.1e}" for b in range(B)])
if F > 1:
    print("grad_x err per f (first 8):", [f"{float(ex[:, :, f].max()):.1e}" for f in range(8)])
