import os, sys, numpy as np, torch, tempfile
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from dstagnn_drought_amd import train as TR
from dstagnn_drought_amd.data import read_and_generate_dataset
g = dict(np.load("tests/golden/g12_train.npz"))
td = tempfile.mkdtemp()
for k in ("adj.csv", "stag.csv", "strg.csv"):
    open(os.path.join(td, k), "w").write(str(g[k + "_text"]))
np.savez(os.path.join(td, "SYN.npz"), data=g["series"])
read_and_generate_dataset(os.path.join(td, "SYN.npz"), 0, 0, 1, 12, points_per_hour=12, save=True)
conf = os.path.join(td, "train.conf"); open(conf, "w").write(str(g["config_text"]).replace("@DIR@", td))
res = TR.run(conf, dropout=0.0, root=os.path.join(td, "m"), log=print)
print([h["val_loss"] for h in res["history"]], g["val_losses"])
for e in [0, 3]:
    sd = torch.load(os.path.join(res["params_path"], f"epoch_{e}.params"), weights_only=True)
    errs = []
    for k, v in sd.items():
        ref = g[f"ep{e}/{k}"]
        errs.append((float(np.abs(v.numpy() - ref).max()), k, float(np.abs(ref).max())))
    errs.sort(reverse=True)
    print("epoch", e, "n", len(errs))
    for x in errs[:12]: print("  %.2e %s (max %.3f)" % x)
    print("  median", np.median([x[0] for x in errs]))
