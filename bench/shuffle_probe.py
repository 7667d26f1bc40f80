import torch, json, sys, os
sys.path.insert(0, os.getcwd())
from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.ops import kernels as K
spec = ArchSpec.weightwise(2, 2); dev = torch.device("cuda", 0)
for n in (65536, 100000):
    uid = torch.arange(n, dtype=torch.int64, device=dev)
    W0 = torch.zeros(n, spec.PP, device=dev); K.init_rows(spec, W0, uid, 1); W = W0.clone()
    for shuf in (True, False):
        def f():
            W.copy_(W0); K.train(spec, W, epochs=20, uid=uid, seed=2, shuffle=shuf)
        f(); torch.cuda.synchronize()
        ts=[]
        for _ in range(7):
            a,b=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
            a.record(); f(); b.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
        print(json.dumps(dict(n=n, shuffle=shuf, ms=sorted(ts)[3])), flush=True)
