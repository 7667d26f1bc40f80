"""Reference module ``methods`` (code/methods.py): the functional prototype API."""
from self_replicating_neural_networks_amd.models.prototypes import (  # noqa: F401
    FeedForwardNetwork, Network, RecurrentNetwork, _BaseNetwork)
