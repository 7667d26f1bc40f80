"""Experiment drivers of the reference (code/setups/*.py) at population scale.

    python -m self_replicating_neural_networks_amd.setups <name> [--key value ...]

names: applying_fixpoints, training_fixpoints, fixpoint_density, known_fixpoint_variation,
learn_from_soup, mixed_self_fixpoints, mixed_soup, network_trajectorys, soup_trajectorys,
soup_demo, network_demo.
"""
from .experiments import REGISTRY  # noqa: F401
