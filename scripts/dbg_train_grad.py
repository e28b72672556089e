"""Debug: one train-mode (dropout 0) gradient of the g12 model, HIP vs oracle, per tensor."""
import os, sys, tempfile, configparser
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from dstagnn_drought_amd import train as TR, set_dropout  # noqa
from dstagnn_drought_amd.data import read_and_generate_dataset
from oracle import dstagnn_ref as ref
g = dict(np.load("tests/golden/g12_train.npz"))
td = tempfile.mkdtemp()
for k in ("adj.csv", "stag.csv", "strg.csv"):
    open(os.path.join(td, k), "w").write(str(g[k + "_text"]))
np.savez(os.path.join(td, "SYN.npz"), data=g["series"])
a = read_and_generate_dataset(os.path.join(td, "SYN.npz"), 0, 0, 1, 12, points_per_hour=12, save=False)
conf = configparser.ConfigParser(); conf.read_string(str(g["config_text"]).replace("@DIR@", td))
torch.manual_seed(1)
net = TR.build(conf, torch.device("cuda", 0))
TR.set_dropout(net, 0.0)
net.train()
x = torch.from_numpy(a["train"]["x"][:8]).float()
y = torch.from_numpy(a["train"]["target"][:8]).float()
loss = torch.nn.SmoothL1Loss()(net(x.cuda()), y.cuda())
loss.backward()
sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
tc = conf["Training"]
blocks, final = ref.split_state_dict(sd, int(tc["nb_block"]))
pb = [{k: v.clone().requires_grad_(True) for k, v in b.items()} for b in blocks]
pf = {k: v.clone().requires_grad_(True) for k, v in final.items()}
b0 = net.BlockList[0]
cheb = [c for c in b0.cheb_conv_SAt.cheb_stack.cpu()]
apa = b0.adj_pa.cpu()
dims = dict(n_heads=int(tc["n_heads"]), d_k=int(tc["d_k"]), d_v=int(tc["d_k"]), K=int(tc["K"]))
out = ref.model_forward(pb, pf, x, cheb, apa, dims, hoist=True)
lr_ = torch.nn.SmoothL1Loss()(out, y)
lr_.backward()
print("loss", loss.item(), lr_.item())
rows = []
for n, p in net.named_parameters():
    if n.startswith("BlockList."):
        _, i, rest = n.split(".", 2)
        r = pb[int(i)][rest].grad
    else:
        r = pf[n].grad
    if p.grad is None or r is None:
        continue
    e = float((p.grad.cpu() - r).abs().max())
    rows.append((e / max(1e-30, float(r.abs().max())), e, float(r.abs().max()), n))
rows.sort(reverse=True)
for r in rows[:10]:
    print("rel %.2e abs %.2e max %.2e %s" % r)
