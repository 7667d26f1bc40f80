"""``from soup import *`` compatibility (reference code/soup.py)."""
try:
    from network import *  # noqa: F401,F403  (reference star-import chain, compat dir on sys.path)
except ImportError:  # imported as a package module
    from .network import *  # noqa: F401,F403
from self_replicating_neural_networks_amd.soup import Soup, prng  # noqa: F401
