"""Per-tensor RELATIVE gradient error of the HIP model vs the reference golden g4 (debug)."""
import json, os, sys
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import dstagnn_drought_amd as D
g = dict(np.load("tests/golden/g4_model.npz"))
m = json.loads(str(g["meta"]))
model = D.make_model("cpu", 1, m["nb_block"], 1, m["K"], m["C"], m["C"], 1, torch.FloatTensor(g["adj_tmd"]),
                     torch.FloatTensor(g["adj_pa"]), torch.FloatTensor(g["adj_tmd"]), m["num_for_predict"],
                     m["T"], m["N"], m["D"], m["d_k"], m["d_k"], m["n_heads"])
model.load_state_dict({k[6:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("param/")})
cheb = torch.from_numpy(np.stack([g[f"cheb_{k}"] for k in range(m["K"])]))
for b in model.BlockList:
    b.cheb_conv_SAt.cheb_stack.copy_(cheb)
model = model.cuda().eval()
x = torch.from_numpy(g["x"]).cuda().requires_grad_(True)
out = model(x)
loss = torch.nn.SmoothL1Loss()(out, torch.from_numpy(g["target"]).cuda())
loss.backward()
rows = []
for n, p in model.named_parameters():
    if bool(g["hasgrad/" + n]):
        r = g["grad/" + n]
        e = float(np.abs(p.grad.cpu().numpy() - r).max())
        rows.append((e / max(1e-30, float(np.abs(r).max())), e, n))
rows.sort(reverse=True)
for r in rows[:15]:
    print("rel %.2e abs %.2e %s" % r)
