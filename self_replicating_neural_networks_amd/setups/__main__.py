"""CLI: python -m self_replicating_neural_networks_amd.setups <name> [--trials N] [--device cuda] ..."""
import argparse
import inspect
import json
import sys

from .experiments import REGISTRY


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in REGISTRY:
        print("usage: python -m self_replicating_neural_networks_amd.setups <name> [--param value ...]")
        print("names: " + ", ".join(sorted(REGISTRY)))
        return 2
    fn = REGISTRY[argv[0]]
    ap = argparse.ArgumentParser(prog=argv[0])
    for name, p in inspect.signature(fn).parameters.items():
        if name in ("specs", "spec"):
            continue
        d = p.default
        typ = type(d) if d not in (None, inspect.Parameter.empty) and not isinstance(d, (list, tuple)) else str
        ap.add_argument("--" + name.replace("_", "-"), dest=name, type=typ, default=d)
    ns = ap.parse_args(argv[1:])
    out = fn(**{k: v for k, v in vars(ns).items()})
    out = {k: v for k, v in out.items() if k != "soup"}
    print(json.dumps(out, default=str))
    return 0


if __name__ == "__main__":
    sys.exit(main())
