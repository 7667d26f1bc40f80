"""``from network import *`` compatibility (reference code/network.py)."""
import copy  # noqa: F401  (the reference leaks these names through star imports)
import os  # noqa: F401

import numpy as np  # noqa: F401
from tqdm import tqdm  # noqa: F401

from self_replicating_neural_networks_amd.models.network import (  # noqa: F401
    AggregatingNeuralNetwork, FFTNeuralNetwork, NeuralNetwork, ParticleDecorator, RecurrentNeuralNetwork,
    REFERENCE_QUIRKS, SaveStateCallback, TrainingNeuralNetworkDecorator, WeightwiseNeuralNetwork)
from self_replicating_neural_networks_amd.experiment import (  # noqa: F401
    Experiment, FixpointExperiment, IdentLearningExperiment, MixedFixpointExperiment, SoupExperiment)
from self_replicating_neural_networks_amd.utils.printing import PrintingObject  # noqa: F401
