import sys, torch
sys.path.insert(0, ".")
from self_replicating_neural_networks_amd.arch import ArchSpec
from self_replicating_neural_networks_amd.population import Population
from self_replicating_neural_networks_amd.ops import kernels as K
spec = ArchSpec.recurrent(16, 2)
pop = Population(spec, 4096, device="cuda", seed=1)
out = torch.zeros_like(pop.W)
K.apply(spec, pop.W, out)
pop.train(1)
torch.cuda.synchronize()
