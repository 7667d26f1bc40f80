import os, sys, torch, numpy as np
sys.path.insert(0, os.getcwd())
from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.ops import kernels as K
dev = torch.device("cuda", 0)
spec = ArchSpec.aggregating(4, 10, 3)
n = 2000
uid = torch.arange(n, dtype=torch.int64, device=dev)
W = torch.zeros(n, spec.PP, device=dev); K.init_rows(spec, W, uid, 4)
idx = torch.roll(torch.arange(n, device=dev), 3).contiguous()
for ep in (1, 3):
    outs = {}
    for mode in ("wave", "row"):
        if mode == "wave": os.environ["SRNN_BIG_WAVE"] = "1"
        else: os.environ.pop("SRNN_BIG_WAVE", None)
        Wt = W.clone(); lt = K.train(spec, Wt, epochs=ep, uid=uid, seed=5)
        Wl = W.clone(); ll = K.learn_from(spec, Wl, W, idx_t=idx, epochs=ep, uid=uid, seed=5)
        outs[mode] = (Wt.cpu().numpy(), lt.cpu().numpy(), Wl.cpu().numpy(), ll.cpu().numpy())
    for nm, i in (("train", 0), ("learn", 2)):
        a, b = outs["wave"][i][:, :spec.P], outs["row"][i][:, :spec.P]
        d = np.abs(a - b).max(axis=1) / (np.abs(a).max(axis=1) + 1e-6)
        bad = np.argsort(-d)[:3]
        print(ep, nm, "max rel", d.max(), "rows", bad, "n>1e-5", int((d > 1e-5).sum()), "loss rel",
              np.nanmax(np.abs(outs["wave"][i+1] - outs["row"][i+1]) / (np.abs(outs["wave"][i+1]) + 1e-9)))
        r = bad[0]
        print("   wave", a[r, :6], "\n   row ", b[r, :6], "\n   W0  ", W[r, :6].cpu().numpy())
