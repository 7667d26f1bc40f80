"""Debug: fp16 WW(2,2) run_fixpoint, group kernel vs lane kernel vs rounded fp32 steps."""
import os
import torch
from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.ops import kernels as K

cuda = torch.device("cuda", 0)
spec = ArchSpec.weightwise(2, 2)
n = 5000
uid = torch.arange(n, dtype=torch.int64, device=cuda)
for dtype in (torch.float16, torch.bfloat16):
    W = torch.zeros(n, spec.PP, dtype=dtype, device=cuda)
    K.init_rows(spec, W, uid, 2)
    res = {}
    for mode in ("0", "1"):
        os.environ["SRNN_FIX_GROUP"] = mode
        Wk = W.clone()
        K.run_fixpoint(spec, Wk, 4, 1e-4, early_exit=False)
        ref = W.clone()
        for _ in range(4):
            r = ref.float()
            K.run_fixpoint(spec, r, 1, 1e-4, early_exit=False)
            ref = r.to(dtype)
        res[mode] = (Wk, ref)
    nan = lambda t: t.float().nan_to_num(7.0, 9.0, -9.0)
    for name, x in (("lane4", res["0"][0]), ("lane_ref", res["0"][1]), ("group4", res["1"][0]), ("group_ref", res["1"][1])):
        d = (nan(x) != nan(res["0"][1])).any(1).nonzero().flatten()
        print(dtype, name, "rows differing from lane_ref:", d.numel(), d[:5].tolist())
        for i in d[:2].tolist():
            print("   ", x[i, :spec.P].tolist())
            print("   ref", res["0"][1][i, :spec.P].tolist())
