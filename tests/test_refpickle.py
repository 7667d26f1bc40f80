"""Reference-schema pickles: restricted reader on the reference's own artifacts and the
writer's global set."""
import glob
import os
import pickle

import numpy as np
import pytest

from self_replicating_neural_networks_amd.compat import network as N
from self_replicating_neural_networks_amd.experiment import Experiment, FixpointExperiment
from self_replicating_neural_networks_amd.io import refpickle as R
from self_replicating_neural_networks_amd.soup import Soup

REF = "/root/reference/code/results"
needs_ref = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not mounted")


@needs_ref
def test_reads_reference_soup_without_executing_code():
    s = R.load(os.path.join(REF, "Soup", "soup.dill"))
    assert isinstance(s, R.SoupRecord)
    assert len(s.historical_particles) == 20
    states = next(iter(s.historical_particles.values()))
    assert len(states) == 100 and states[0]["weights"].dtype == np.float32 and states[0]["weights"].shape == (14,)
    assert isinstance(s.generator, R.Opaque)  # the pickled lambda stays inert


@needs_ref
def test_reads_learn_from_soup_uids():
    s = R.load(glob.glob(os.path.join(REF, "exp-learn-from-soup-*", "soup.dill"))[0])
    assert sorted(s.historical_particles) == list(range(1090, 1100))  # process-global uids (S13)
    acts = [st.get("action") for v in s.historical_particles.values() for st in v]
    assert acts.count("init") == 10 and acts.count("learn_from") == 98


@needs_ref
def test_reads_every_reference_artifact():
    files = glob.glob(os.path.join(REF, "**", "*.dill"), recursive=True)
    assert len(files) >= 20
    for f in files:
        R.load(f)
    e = R.load(os.path.join(REF, "known_fixpoint_variation", "experiment.dill"))
    assert len(e.ys) == 1000 and e.trials == 100


def test_restricted_reader_refuses_code():
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned > /tmp/srnn_pwned",))
    data = pickle.dumps(Evil(), protocol=3)
    if os.path.exists("/tmp/srnn_pwned"):
        os.remove("/tmp/srnn_pwned")
    obj = R.loads(data)
    assert isinstance(obj, R.Opaque)
    assert not os.path.exists("/tmp/srnn_pwned")


def test_writer_uses_reference_globals(tmp_path):
    gen = lambda: N.TrainingNeuralNetworkDecorator(N.WeightwiseNeuralNetwork(2, 2))  # noqa: E731
    s = Soup(4, gen, mode="sequential").with_params(train=1)
    s.seed()
    s.evolve(2)
    data = R.dumps(s.without_particles())
    assert R.globals_of(data) <= {("soup", "Soup"), ("numpy", "ndarray"), ("numpy", "dtype"),
                                  ("numpy.core.multiarray", "_reconstruct"),
                                  ("numpy._core.multiarray", "_reconstruct"),
                                  ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar")}
    back = R.loads(data)
    assert back.size == 4 and back.time == 2 and back.params["train"] == 1
    assert back.generator["arch"]["kind"] == "weightwise"
    states = next(iter(back.historical_particles.values()))
    assert states[0]["action"] == "init"


def test_experiment_context_manager_contract(tmp_path):
    with FixpointExperiment(root=str(tmp_path)) as exp:
        for i in range(3):
            n = N.ParticleDecorator(N.WeightwiseNeuralNetwork(2, 2))
            exp.run_net(n, 20, run_id=i + 1)
            exp.historical_particles[i] = n
        exp.log(exp.counters)
        exp.save(all_counters=[exp.counters], all_names=["ww"])
        d = exp.dir
    assert os.path.basename(d).startswith("exp-FixpointExperiment-_") and d.endswith("-0")
    files = sorted(os.listdir(d))
    assert files == ["all_counters.dill", "all_names.dill", "experiment.dill", "log.txt"]
    e = Experiment.from_dill(os.path.join(d, "experiment.dill"))
    assert isinstance(e, R.ExperimentRecord)
    assert sum(e.counters.values()) == 3 and len(e.historical_particles) == 3
    assert R.globals_of(open(os.path.join(d, "experiment.dill"), "rb").read()) >= {("experiment", "Experiment")}
    assert open(os.path.join(d, "log.txt")).read().startswith("{'divergent'")
    assert R.load(os.path.join(d, "all_names.dill")) == ["ww"]
