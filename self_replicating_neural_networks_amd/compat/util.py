"""``from util import *`` compatibility (reference code/util.py)."""
from self_replicating_neural_networks_amd.utils.printing import PrintingObject  # noqa: F401
