"""Trajectory embeddings and outcome plots (reference L6: code/visualization.py,
code/bar_plot.py, code/line_plots.py, code/box_plots.py)."""
from .plots import (build_from_soup_or_exp, line_plot, plot_bars, plot_box, plot_histogram,  # noqa: F401
                    plot_latent_trajectories, plot_latent_trajectories_3D, plot_lines, search_and_apply)
