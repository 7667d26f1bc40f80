"""CLI mirroring the reference's plotting scripts:

    python -m self_replicating_neural_networks_amd.analysis {trajectories,tsne,bars,lines,box} -i <file-or-dir>

trajectories: trajectorys.dill / soup.dill -> 3-D PCA trajectories (visualization.py)
tsne:         same inputs -> 2-D t-SNE
bars:         all_counters.dill (+ all_names.dill) -> stacked outcome bars (bar_plot.py)
lines:        all_data.dill (+ all_names.dill) -> lines (line_plots.py)
box:          experiment.dill of known-fixpoint-variation -> boxes (box_plots.py)
"""
import argparse
import sys

from . import plots as P


def main(argv=None):
    ap = argparse.ArgumentParser(prog="srnn-analysis")
    ap.add_argument("kind", choices=["trajectories", "tsne", "bars", "lines", "box"])
    ap.add_argument("-i", "--in_file", required=True)
    ap.add_argument("-o", "--out_file", default="out")
    ap.add_argument("--overwrite", action="store_true")
    a = ap.parse_args(argv)
    if a.kind == "trajectories":
        done = P.search_and_apply(a.in_file, P.plot_latent_trajectories_3D, ["trajectorys.dill", "soup.dill"],
                                  overwrite=a.overwrite)
    elif a.kind == "tsne":
        done = P.search_and_apply(a.in_file, P.plot_latent_trajectories, ["trajectorys.dill", "soup.dill"],
                                  overwrite=a.overwrite)
    elif a.kind == "bars":
        done = P.search_and_apply(a.in_file, P.plot_bars, ["all_counters.dill"], loader=P._with_names,
                                  overwrite=a.overwrite)
    elif a.kind == "lines":
        done = P.search_and_apply(a.in_file, P.plot_lines, ["all_data.dill"], loader=P._with_names,
                                  overwrite=a.overwrite)
    else:
        done = P.search_and_apply(a.in_file, P.plot_box, ["experiment.dill"], overwrite=a.overwrite)
    print("\n".join(done))
    return 0


if __name__ == "__main__":
    sys.exit(main())
