"""``from experiment import *`` compatibility (reference code/experiment.py)."""
import copy  # noqa: F401
import os  # noqa: F401
import time  # noqa: F401

from tqdm import tqdm  # noqa: F401

from self_replicating_neural_networks_amd.experiment import (  # noqa: F401
    Experiment, FixpointExperiment, IdentLearningExperiment, MixedFixpointExperiment, SoupExperiment)
