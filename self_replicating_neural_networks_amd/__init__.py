"""MI355X-native engine for self-replicating neural networks.

A re-design of illiumst/self-replicating-neural-networks for AMD Instinct MI355X (gfx950):
particles are rows of device-resident population tensors, their self-application,
attacks, self-training, learn-from and fixpoint classification run as hand-written HIP
kernels (csrc/, lane-per-particle with weights in VGPRs), populations are sharded over
the GPUs of a node with RCCL collectives, and the reference's Experiment / Soup /
network API is re-exposed on top (``self_replicating_neural_networks_amd.compat``).
"""
from .arch import ArchSpec  # noqa: F401
from .population import Population  # noqa: F401

__version__ = "0.1.0"
