"""Analysis of recorded experiments: trajectory embeddings and outcome plots.

Re-implements the reference's plotting CLIs (code/visualization.py, code/bar_plot.py,
code/line_plots.py, code/box_plots.py) on top of the restricted reader, so both our
pickles and the reference's ``*.dill`` artifacts can be plotted without executing code
from them.  Figures are written as self-contained plotly HTML next to the input file
(as the reference does); ``auto_open`` defaults to False for headless use.

Embeddings: PCA (numpy SVD, or ``torch.pca_lowrank`` on the GPU for large state sets)
and t-SNE (``sklearn.manifold.TSNE``; the reference used a removed private path).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

from ..io import refpickle

CLASS_ORDER = ("divergent", "fix_zero", "fix_other", "fix_sec", "other")


def _go():
    import plotly.graph_objs as go
    return go


def color_scale(n: int) -> List[str]:
    """n colours interpolated red -> yellow -> green (the reference's RdYlGn scale)."""
    stops = np.array([[215, 48, 39], [254, 224, 139], [26, 152, 80]], dtype=float)
    out = []
    for k in range(max(n, 1)):
        t = k / max(n - 1, 1) * 2
        i = min(int(t), 1)
        c = stops[i] + (stops[i + 1] - stops[i]) * (t - i)
        out.append("rgb({},{},{})".format(*[int(round(v)) for v in c]))
    return out


def _write(fig, filename, auto_open=False):
    import plotly.offline as po
    po.plot(fig, auto_open=auto_open, filename=filename, validate=True)
    return filename


# ------------------------------------------------------------------------------ trajectories
def build_from_soup_or_exp(obj) -> List[Dict]:
    """Per-particle trajectories of a soup / experiment (reference visualization.py:27-40)."""
    hp = obj.historical_particles if hasattr(obj, "historical_particles") else obj
    out = []
    for states in hp.values():
        states = states.states if hasattr(states, "states") else states
        states = [s for s in states if isinstance(s, dict) and isinstance(s.get("weights"), np.ndarray)]
        if not states:
            continue
        out.append(dict(
            trajectory=np.stack([np.asarray(s["weights"], dtype=np.float32).reshape(-1) for s in states]),
            time=[s.get("time", k) for k, s in enumerate(states)],
            action=[s.get("action", None) for s in states],
            counterpart=[s.get("counterpart", None) for s in states],
        ))
    return out


def pca_2d(x: np.ndarray, use_torch: bool = False) -> Callable[[np.ndarray], np.ndarray]:
    """Fit a 2-component PCA; returns the projection function."""
    mu = x.mean(axis=0, keepdims=True)
    if use_torch:
        import torch
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        _, _, v = torch.pca_lowrank(torch.as_tensor(x - mu, device=dev), q=2, center=False)
        comps = v.T.cpu().numpy()
    else:
        _, _, vt = np.linalg.svd(x - mu, full_matrices=False)
        comps = vt[:2]
    return lambda y: (np.asarray(y) - mu) @ comps.T


def plot_latent_trajectories_3D(obj, filename="plot.html", auto_open=False, use_torch=None):
    """PCA(2) of every recorded state, z = time; start red, end black (visualization.py:96-180)."""
    go = _go()
    data_list = build_from_soup_or_exp(obj)
    if not data_list:
        return None
    allx = np.vstack([d["trajectory"] for d in data_list])
    proj = pca_2d(allx, use_torch=(allx.shape[0] > 200_000) if use_torch is None else use_torch)
    scale = color_scale(len(data_list) + 1)
    data = []
    for pid, d in enumerate(data_list):
        t = proj(d["trajectory"])
        z = np.asarray(d["time"], dtype=float)
        data.append(go.Scatter3d(x=t[:, 0], y=t[:, 1], z=z, mode="lines", showlegend=False, hoverinfo="text",
                                 text="Particle: {}<br> It had {} lifes.".format(pid, len(t)),
                                 line=dict(color=scale[pid], width=4), name="Particle -{}".format(pid)))
        data.append(go.Scatter3d(mode="markers", x=[t[0, 0]], y=[t[0, 1]], z=[z[0]], showlegend=False,
                                 marker=dict(color="rgb(255, 0, 0)", size=4)))
        data.append(go.Scatter3d(mode="markers", x=[t[-1, 0]], y=[t[-1, 1]], z=[z[-1]], showlegend=False,
                                 marker=dict(color="rgb(0, 0, 0)", size=4)))
    axis = dict(gridcolor="rgb(255, 255, 255)", gridwidth=3, zerolinecolor="rgb(255, 255, 255)",
                showbackground=True, backgroundcolor="rgb(230, 230,230)")
    layout = go.Layout(scene=dict(xaxis=dict(title="Transformed X", **axis), yaxis=dict(title="Transformed Y", **axis),
                                  zaxis=dict(title="Epoch", **axis)),
                       width=1024, height=1024, margin=dict(l=0, r=0, b=0, t=0))
    return _write(go.Figure(data=data, layout=layout), filename, auto_open)


def plot_latent_trajectories(obj, filename="latent_trajectory_plot.html", auto_open=False, perplexity=30.0):
    """t-SNE 2-D embedding of all states (visualization.py:43-93)."""
    from sklearn.manifold import TSNE
    go = _go()
    data_list = build_from_soup_or_exp(obj)
    if not data_list:
        return None
    allx = np.vstack([d["trajectory"] for d in data_list])
    emb = TSNE(n_components=2, perplexity=min(perplexity, max(2.0, (allx.shape[0] - 1) / 3.0)),
               init="pca", random_state=0).fit_transform(allx)
    scale = color_scale(len(data_list) + 1)
    data, o = [], 0
    for pid, d in enumerate(data_list):
        t = emb[o:o + len(d["trajectory"])]
        o += len(d["trajectory"])
        data.append(go.Scatter(x=t[:, 0], y=t[:, 1], mode="lines", line=dict(color=scale[pid]),
                               name="Particle - {}".format(pid)))
        data.append(go.Scatter(mode="markers", x=[t[0, 0]], y=[t[0, 1]], showlegend=False,
                               marker=dict(color="rgb(255, 0, 0)", size=4)))
        data.append(go.Scatter(mode="markers", x=[t[-1, 0]], y=[t[-1, 1]], showlegend=False,
                               marker=dict(color="rgb(0, 0, 0)", size=4)))
    layout = dict(title="Latent Trajectory Movement", height=800, width=800)
    return _write(go.Figure(data=data, layout=layout), filename, auto_open)


def plot_histogram(bars_dict_list, filename="histogram_plot.html", auto_open=False):
    go = _go()
    scale = color_scale(len(bars_dict_list) + 1)
    data = [go.Histogram(histfunc="count", y=d.get("value", []), x=d.get("name", []), showlegend=False,
                         marker=dict(color=scale[i])) for i, d in enumerate(bars_dict_list)]
    return _write(go.Figure(data=data, layout=dict(title="Histogram Plot", height=400, width=400)), filename, auto_open)


def line_plot(line_dict_list, filename="lineplot.html", auto_open=False):
    """Lines with a shaded band (visualization.py:209-252): dicts with x, main_y, upper_y, lower_y."""
    go = _go()
    scale = color_scale(len(line_dict_list) + 1)
    data = []
    for i, d in enumerate(line_dict_list):
        band = scale[i].replace("rgb", "rgba").replace(")", ",0.4)")
        data.append(go.Scatter(name="Upper Bound", x=d["x"], y=d["upper_y"], mode="lines", line=dict(width=0),
                               fillcolor=band, showlegend=False))
        data.append(go.Scatter(x=d["x"], y=d["main_y"], mode="lines", name=d.get("name", "line"),
                               line=dict(color=scale[i]), fillcolor=band, fill="tonexty"))
        data.append(go.Scatter(name="Lower Bound", x=d["x"], y=d["lower_y"], mode="lines", line=dict(width=0),
                               showlegend=False))
    return _write(go.Figure(data=data, layout=dict(title="Line Plot", height=800, width=800)), filename, auto_open)


# ------------------------------------------------------------------------------ outcome plots
def short_names(names: Sequence[str]) -> List[str]:
    out = []
    for n in names:
        base = str(n).split(" ")[0].replace("NeuralNetwork", "")
        out.append(base or str(n))
    return out


def plot_bars(names_bars_tuple, filename="histogram_plot.html", auto_open=False):
    """Stacked bars of the 5 outcome classes per network (code/bar_plot.py:28-59)."""
    go = _go()
    names, bars = names_bars_tuple
    names = short_names(names)
    situations = [k for k in CLASS_ORDER if k in bars[0]] + [k for k in bars[0] if k not in CLASS_ORDER]
    data = [go.Bar(y=[b.get(s, 0) for b in bars], x=names, name=s, showlegend=True) for s in situations]
    layout = dict(xaxis=dict(title="Networks"), barmode="stack", legend=dict(orientation="h", x=0.05))
    return _write(go.Figure(data=data, layout=layout), filename, auto_open)


def plot_lines(names_data_tuple, filename="lineplot.html", auto_open=False, y_key="ys",
               xlabel="Trains per self-application", ylabel="Average amount of fixpoints found"):
    """Lines of all_data.dill ``xs``/``ys`` per network (code/line_plots.py:27-81)."""
    go = _go()
    names, line_dicts = names_data_tuple
    names = short_names(names)
    data = [go.Scatter(x=d["xs"], y=d[y_key], name=names[i] if i < len(names) else str(i), line=dict(width=5))
            for i, d in enumerate(line_dicts)]
    layout = dict(xaxis=dict(title=xlabel), yaxis=dict(title=ylabel), legend=dict(orientation="h", x=0.3, y=-0.3))
    return _write(go.Figure(data=data, layout=layout), filename, auto_open)


def plot_box(exp, filename="box_plot.html", auto_open=False):
    """Time-to-vergence / time-as-fixpoint boxes per perturbation scale (code/box_plots.py:28-94)."""
    go = _go()
    cats = []
    for d in range(exp.depth):
        cats.extend(["D 10e-{}".format(d)] * exp.trials)
    data = [go.Box(y=exp.ys, x=cats, name="Time to Vergence", boxpoints=False, marker=dict(color="rgb(253,174,97)")),
            go.Box(y=exp.zs, x=cats, name="Time as Fixpoint", boxpoints=False, marker=dict(color="rgb(49,54,149)"))]
    layout = dict(title="Known Fixpoint Variation", boxmode="group", boxgap=0, yaxis=dict(title="Steps"),
                  legend=dict(orientation="h", x=0.1, y=-0.1))
    return _write(go.Figure(data=data, layout=layout), filename, auto_open)


# ------------------------------------------------------------------------------ walking
def search_and_apply(path, plotting_function, files_to_look_for=(), loader=None, overwrite=False):
    """Recursively apply ``plotting_function`` to matching ``*.dill`` files without an
    existing ``.html`` next to them (reference visualization.py:255-275)."""
    loader = loader or (lambda p: refpickle.load(p))
    done = []
    if os.path.isdir(path):
        for entry in sorted(os.scandir(path), key=lambda e: e.path):
            done += search_and_apply(entry.path, plotting_function, files_to_look_for, loader, overwrite)
    elif path.endswith(".dill") and os.path.basename(path) in files_to_look_for:
        html = path[:-5] + ".html"
        if overwrite or not os.path.exists(html):
            print('Apply Plotting function "{}" on file "{}"'.format(plotting_function.__name__, path))
            try:
                plotting_function(loader(path), filename=html)
                done.append(html)
            except (ValueError, AttributeError, KeyError, IndexError) as e:  # reference: skip broken files
                print("  skipped: {}".format(e))
    return done


def _with_names(path):
    names = refpickle.load(os.path.join(os.path.dirname(path), "all_names.dill"))
    return names, refpickle.load(path)
