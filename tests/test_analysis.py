"""Analysis CLIs on our own experiment outputs and on the reference's artifacts."""
import os
import shutil

import numpy as np
import pytest

from self_replicating_neural_networks_amd.analysis import plots as P
from self_replicating_neural_networks_amd.analysis.__main__ import main as cli
from self_replicating_neural_networks_amd.setups import experiments as E

REF = "/root/reference/code/results"


def test_pca_projection_recovers_plane():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(200, 2)) @ np.array([[1.0, 0, 0, 0], [0, 0.5, 0, 0]]) + 3.0
    proj = P.pca_2d(x)
    y = proj(x)
    assert y.shape == (200, 2)
    assert abs(np.corrcoef(y[:, 0], x[:, 0])[0, 1]) > 0.97  # first component ~ the high-variance axis


def test_all_plots_on_our_experiments(tmp_path):
    r1 = E.applying_fixpoints(trials=30, device="cpu", seed=1, root=str(tmp_path))
    r2 = E.mixed_soup(trials=4, device="cpu", seed=2, root=str(tmp_path), trains=[0, 10])
    r3 = E.known_fixpoint_variation(trials=10, depth=3, device="cpu", seed=3, root=str(tmp_path))
    r4 = E.network_trajectorys(trials=5, device="cpu", seed=4, root=str(tmp_path))
    assert cli(["bars", "-i", r1["dir"]]) == 0
    assert os.path.exists(os.path.join(r1["dir"], "all_counters.html"))
    assert cli(["lines", "-i", r2["dir"]]) == 0
    assert os.path.exists(os.path.join(r2["dir"], "all_data.html"))
    assert cli(["box", "-i", r3["dir"]]) == 0
    assert os.path.exists(os.path.join(r3["dir"], "experiment.html"))
    assert cli(["trajectories", "-i", r4["dir"]]) == 0
    assert os.path.exists(os.path.join(r4["dir"], "trajectorys.html"))


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not mounted")
def test_plots_reference_artifacts(tmp_path):
    src = os.path.join(REF, "Soup", "soup.dill")
    dst = tmp_path / "soup.dill"
    shutil.copy(src, dst)
    out = P.plot_latent_trajectories_3D(P.refpickle.load(str(dst)), filename=str(tmp_path / "soup.html"))
    assert os.path.getsize(out) > 10000
    kfv = os.path.join(REF, "known_fixpoint_variation", "experiment.dill")
    out = P.plot_box(P.refpickle.load(kfv), filename=str(tmp_path / "box.html"))
    assert os.path.exists(out)
