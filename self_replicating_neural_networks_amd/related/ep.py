"""The bundled sibling project "EP" (reference related/EP/src): networks that learn the
identity on a *feature-reduced vector of their own weights*.

Reference components and their equivalents here:

==========================  ==================================================  ======================
reference                   behaviour                                           here
==========================  ==================================================  ======================
FeatureReduction.py         fft / rfft / fractional-bin mean / shuffled mean    ``FeatureReduction``
Functions.py                MSE, scale, N(0, sd) random layers, file checks     module functions
LossHistory.py              per-batch loss recorder                             ``LossHistory``
NeuralNetwork.py            Keras MLP + Adadelta self-fit loop, stochastic      ``ReductionLearner``
                            hill climbers V1/V2/V3, local-maximum analytics
PltData.py                  matplotlib loss curves, network graph plots         ``plot_*`` functions
testSomething.py drivers    checkLM / searchForThreshold / checkScale sweeps    ``ReductionLearner.fit``
==========================  ==================================================  ======================

``ReductionLearner`` is population-batched: N independent learners (each its own MLP
with biases and Keras-style activations) are stepped together with batched matmuls on
the device, so the reference's serial per-configuration sweeps become one run.  Every
feature reduction of the reference is linear in the weight vector (the fft variants
after the implicit real cast Keras applied to complex inputs), so the batched path uses a
precomputed reduction matrix; the scalar reference algorithms are kept for single
vectors and pinned by the reference's own unit-test values (tests/test_ep.py).
"""
from __future__ import annotations

import glob
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

# ====================================================================================
# Functions.py
# ====================================================================================


def check_file_exists(file_name: str):
    """Path of the first file matching ``file_name`` (glob) or False (Functions.py:5-16)."""
    found = glob.glob(file_name)
    return found[0] if found else False


def calc_mean_squared_error(a, b) -> float:
    """MSE of two arrays, string arrays accepted (Functions.py:18-29)."""
    a = np.asarray(a).astype(float)
    b = np.asarray(b).astype(float)
    return float(((a - b) ** 2).mean())


def calc_scale(array) -> float:
    return float(abs(max(array) - min(array)))


def get_random_gaus_number(standard_deviation: float, rng: Optional[np.random.Generator] = None) -> float:
    rng = rng or np.random.default_rng()
    return float(rng.normal(0.0, standard_deviation))


def get_random_layer(shape, standard_deviation=0.01, rng: Optional[np.random.Generator] = None):
    """Keras-format random layer [kernel (in, out) ~ N(0, sd), zero bias] (Functions.py:39-58)."""
    rng = rng or np.random.default_rng()
    return [rng.normal(0.0, standard_deviation, size=tuple(shape)), np.zeros(shape[1])]


# reference-name aliases
checkFileExists = check_file_exists
calcMeanSquaredError = calc_mean_squared_error
calcScale = calc_scale
getRandomGausNumber = get_random_gaus_number
getRandomLayer = get_random_layer


# ====================================================================================
# FeatureReduction.py
# ====================================================================================
class FeatureReduction:
    TYPES = ("fft", "rfft", "mean", "meanShuffled")

    def __init__(self, type: str):
        if type not in self.TYPES:
            raise ValueError(f"unknown feature reduction {type!r}")
        self.type = type
        self.VecFromWeigths = None

    # -------------------------------------------------------------- scalar reference semantics
    def calc(self, vec, n):
        """Reduce a weight list (kernels only) or a flat vector to the network input."""
        self.weigthsToVec(vec)
        v = self.VecFromWeigths
        if self.type == "fft":
            return self.fft(v, n)
        if self.type == "rfft":
            return self.rfftn(v, n)
        if self.type == "mean":
            return self.mean(v, n)
        return self.mean(self.shuffelVec(v, 3), n)

    @staticmethod
    def fft(vec, n):
        return np.fft.fft(vec, n)

    @staticmethod
    def rfftn(vec, n):
        return np.fft.rfft(vec, n)

    @staticmethod
    def shuffelVec(vec, mod):
        """Every mod-th element first, then the rest shuffled the same way, recursively
        (FeatureReduction.py:24-36)."""
        vec = np.asarray(vec, dtype=float)
        if len(vec) == 0:
            return vec
        picked = vec[::mod]
        rest = np.array([v for i, v in enumerate(vec) if i % mod != 0])
        if len(picked) == len(vec):
            return picked
        return np.concatenate([picked, FeatureReduction.shuffelVec(rest, mod)])

    @staticmethod
    def mean(vec, n):
        """Split ``vec`` into ``n`` equal (fractional) parts and average each one, rounded
        to 6 decimals (FeatureReduction.py:38-70).  Values at a part boundary are split
        between the two parts in proportion to the overlap."""
        vec = np.asarray(vec, dtype=float)
        L = len(vec)
        width = L / n
        out = []
        # exact interval overlap of element [i, i+1) with part [k*width, (k+1)*width)
        acc = 0.0
        k = 0
        edge = width
        for i, v in enumerate(vec):
            lo, hi = float(i), float(i + 1)
            while k < n and round(edge, 5) <= hi - 1e-12 + 1e-5 and round(edge, 5) < round(hi, 5) + 1e-9:
                part = edge - lo
                if round(part, 5) <= 0:
                    break
                acc += part * v
                out.append(round(acc / width, 6))
                acc = 0.0
                lo = edge
                k += 1
                edge = (k + 1) * width
            frac = hi - lo
            if round(frac, 5) > 0:
                acc += frac * v
            if round(edge, 5) <= round(hi, 5) and k < n:
                out.append(round(acc / width, 6))
                acc = 0.0
                k += 1
                edge = (k + 1) * width
        return np.array(out[:n])

    def weigthsToVec(self, weights, vec=None):
        """Flatten the kernels of a Keras weight list, dropping bias vectors
        (FeatureReduction.py:72-95)."""
        if isinstance(weights, np.ndarray) and weights.ndim == 1 and weights.dtype != object:
            self.VecFromWeigths = weights.astype(float)
            return
        parts = []
        for w in weights:
            a = np.asarray(w)
            if a.ndim >= 2:
                parts.append(a.reshape(-1))
        self.VecFromWeigths = np.concatenate(parts).astype(float) if parts else np.array([])

    # -------------------------------------------------------------- batched (linear map)
    def matrix(self, length: int, n: int) -> np.ndarray:
        """(out, length) matrix R with reduce(v) == R @ v for every v (before rounding)."""
        cols = []
        for i in range(length):
            e = np.zeros(length)
            e[i] = 1.0
            if self.type == "fft":
                r = np.real(np.fft.fft(e, n))
            elif self.type == "rfft":
                r = np.real(np.fft.rfft(e, n))
            elif self.type == "mean":
                r = self._mean_linear(e, n)
            else:
                r = self._mean_linear(self.shuffelVec(e, 3), n)
            cols.append(r)
        return np.stack(cols, axis=1)

    @staticmethod
    def _mean_linear(vec, n):
        L = len(vec)
        width = L / n
        out = np.zeros(n)
        for k in range(n):
            a, b = k * width, (k + 1) * width
            for i in range(L):
                ov = max(0.0, min(b, i + 1) - max(a, i))
                out[k] += ov * vec[i]
        return out / width


# ====================================================================================
# LossHistory.py
# ====================================================================================
class LossHistory:
    def __init__(self):
        self.losses: List = []

    def on_train_begin(self, logs=None):
        self.losses = []

    def on_batch_end(self, batch, logs=None):
        self.losses.append((logs or {}).get("loss"))

    def addLoss(self, loss):
        self.losses.append(loss)


# ====================================================================================
# NeuralNetwork.py -> population-batched ReductionLearner
# ====================================================================================
_ACT = {
    "linear": lambda x: x,
    "sigmoid": torch.sigmoid,
    "tanh": torch.tanh,
    "relu": torch.relu,
    "elu": torch.nn.functional.elu,
    "softplus": torch.nn.functional.softplus,
    "hard_sigmoid": lambda x: torch.clamp(0.2 * x + 0.5, 0.0, 1.0),
}


def check_growing(m_array: Sequence[float], rng: int, check_same: bool = True) -> bool:
    """Is the mean of the last ``rng`` values >= that of the ``rng`` before
    (NeuralNetwork.py:296-306)?"""
    if len(m_array) < rng * 2:
        return False
    v = np.asarray(m_array[-rng * 2:], dtype=float).reshape(2, rng)
    if v[0].sum() == v[1].sum() and check_same:
        return False
    return not v[0].sum() > v[1].sum()


class ReductionLearner:
    """N independent EP networks learning f(R(w)) = R(w), trained together.

    ``number_of_neurons`` = [n0, n1, ..., nk] (n0 = reduced input size), one activation
    per layer, Keras "uniform" kernel init U(-0.05, 0.05), zero biases, Adadelta
    (lr 1.0, rho 0.95, eps 1e-7: Keras 2.2.4 defaults) or the stochastic hill climber."""

    def __init__(self, number_of_neurons: Sequence[int], activation_functions: Sequence[str],
                 feature_reduction: str = "mean", number_loops: int = 1000, population: int = 1,
                 device="cpu", seed: int = 0, fit_by_hill_climber: bool = False, standard_deviation: float = 0.01,
                 number_of_random_shots: int = 20, check_new_weights_is_really_better: bool = False,
                 hill_climber_version: int = 3, lr: float = 1.0, rho: float = 0.95, eps: float = 1e-7):
        if len(activation_functions) != len(number_of_neurons) - 1:
            raise ValueError("one activation per layer")
        self.sizes = list(number_of_neurons)
        self.acts = list(activation_functions)
        self.reduction = FeatureReduction(feature_reduction)
        self.number_loops = number_loops
        self.n = population
        self.device = torch.device(device)
        self.gen = torch.Generator(device="cpu").manual_seed(seed)
        self.hill = fit_by_hill_climber
        self.sd = standard_deviation
        self.shots = number_of_random_shots
        self.check_better = check_new_weights_is_really_better
        self.hc_version = hill_climber_version
        self.lr, self.rho, self.eps = lr, rho, eps
        self.kernels, self.biases = [], []
        for a, b in zip(self.sizes[:-1], self.sizes[1:]):
            k = (torch.rand((population, a, b), generator=self.gen) * 0.1 - 0.05).to(self.device)
            self.kernels.append(k)
            self.biases.append(torch.zeros((population, b), device=self.device))
        L = sum(a * b for a, b in zip(self.sizes[:-1], self.sizes[1:]))
        self.R = torch.as_tensor(self.reduction.matrix(L, self.sizes[0]), dtype=torch.float32, device=self.device)
        if self.R.shape[0] != self.sizes[0]:
            raise ValueError(f"{feature_reduction} reduction gives {self.R.shape[0]} features, "
                             f"input layer has {self.sizes[0]}")
        self._acc_g = [torch.zeros_like(p) for p in self.kernels + self.biases]
        self._acc_dx = [torch.zeros_like(p) for p in self.kernels + self.biases]
        self.result: List[torch.Tensor] = []
        self.begin_growing = 0
        self.stop_growing = 0
        self.lm = 0.0

    # -------------------------------------------------------------- model
    def flat_kernels(self) -> torch.Tensor:
        return torch.cat([k.reshape(self.n, -1) for k in self.kernels], dim=1)

    def features(self) -> torch.Tensor:
        x = self.flat_kernels() @ self.R.T
        if self.reduction.type in ("mean", "meanShuffled"):
            x = torch.round(x * 1e6) / 1e6  # the reference rounds every part mean to 6 decimals
        return x

    def forward(self, x, kernels=None, biases=None) -> torch.Tensor:
        kernels = kernels or self.kernels
        biases = biases or self.biases
        h = x
        for k, b, a in zip(kernels, biases, self.acts):
            h = _ACT[a](torch.bmm(h.unsqueeze(1), k).squeeze(1) + b)
        return h

    def loss(self, kernels=None, biases=None, x=None) -> torch.Tensor:
        if x is None:
            x = self.features() if kernels is None else \
                torch.cat([k.reshape(self.n, -1) for k in kernels], 1) @ self.R.T
        y = self.forward(x, kernels, biases)
        return ((y - x) ** 2).mean(dim=1)

    # -------------------------------------------------------------- optimisers
    def adadelta_step(self) -> torch.Tensor:
        x = self.features().detach()
        params = [p.detach().requires_grad_(True) for p in self.kernels + self.biases]
        ks, bs = params[:len(self.kernels)], params[len(self.kernels):]
        lvec = self.loss(ks, bs, x)
        lvec.sum().backward()  # per-learner gradients (learners are independent)
        with torch.no_grad():
            for i, p in enumerate(params):
                g = p.grad
                self._acc_g[i].mul_(self.rho).addcmul_(g, g, value=1 - self.rho)
                upd = g * torch.sqrt(self._acc_dx[i] + self.eps) / torch.sqrt(self._acc_g[i] + self.eps)
                p.sub_(self.lr * upd)
                self._acc_dx[i].mul_(self.rho).addcmul_(upd, upd, value=1 - self.rho)
        self.kernels = [p.detach() for p in ks]
        self.biases = [p.detach() for p in bs]
        return lvec.detach()

    def hill_climber_step(self) -> torch.Tensor:
        """Stochastic hill climber: perturb the kernels with N(0, sd) ``shots`` times and keep
        the best (V3: every candidate judged on its own reduced vector; V1: judged on the
        current vector; V2: V1 plus a re-check against the old weights)."""
        with torch.no_grad():
            x0 = self.features()
            best_loss = self.loss(x=x0)
            first = best_loss.clone()
            best_k = [k.clone() for k in self.kernels]
            cur = [k.clone() for k in self.kernels]
            for _ in range(self.shots):
                cur = [k + torch.randn(k.shape, generator=self.gen).to(self.device) * self.sd for k in cur]
                if self.hc_version == 3:
                    lv = self.loss(cur, self.biases)
                else:
                    lv = self.loss(cur, self.biases, x0)
                better = lv < best_loss
                best_loss = torch.where(better, lv, best_loss)
                best_k = [torch.where(better[:, None, None], c, b) for c, b in zip(cur, best_k)]
            if self.hc_version == 2 and self.check_better:
                xn = torch.cat([k.reshape(self.n, -1) for k in best_k], 1) @ self.R.T
                new_err = self.loss(best_k, self.biases, xn)
                old_err = self.loss(self.kernels, self.biases, xn)
                keep = new_err < old_err
                best_k = [torch.where(keep[:, None, None], b, k) for b, k in zip(best_k, self.kernels)]
            self.kernels = best_k
            return first

    # -------------------------------------------------------------- training loop
    def fit(self, check_lm: bool = False, search_for_threshold: bool = False, check_scale: bool = False,
            history: Optional[LossHistory] = None) -> Dict:
        """The reference's self-fit loop (NeuralNetwork.py:218-286) for every learner at once.
        Early-exit criteria are evaluated on the population-mean loss curve."""
        hist = history or LossHistory()
        for i in range(self.number_loops):
            l = self.hill_climber_step() if self.hill else self.adadelta_step()
            self.result.append(l.cpu())
            hist.addLoss(float(l.mean()))
            curve = [float(r.mean()) for r in self.result]
            if check_scale and (check_growing(curve, 10) or curve[-1] == 0.0 or i > 2500):
                break
            if search_for_threshold:
                if check_growing(curve, 100):
                    return dict(first=float(self.result[0].mean()), growing=True, loops=i + 1)
                if i > 1000:
                    return dict(first=float(self.result[0].mean()), growing=False, loops=i + 1)
            if check_lm:
                if len(curve) > 1000 and sum(curve[-1000:]) == 0.0:
                    self.begin_growing = 0
                    break
                if check_growing(curve, 10) and self.begin_growing == 0:
                    self.begin_growing = i
                if self.begin_growing > 0 and not check_growing(curve, 10, check_same=False) \
                        and i - self.begin_growing > 500:
                    self.stop_growing = i
                    self.lm = curve[-1]
                    break
        return dict(losses=torch.stack(self.result).numpy(), begin_growing=self.begin_growing,
                    stop_growing=self.stop_growing, lm=self.lm)

    def evaluate(self, inputs) -> np.ndarray:
        """Model outputs for scalar inputs (input layer of size 1), per learner."""
        x = torch.as_tensor(np.asarray(inputs, dtype=np.float32), device=self.device).reshape(1, -1, 1)
        outs = []
        for j in range(x.shape[1]):
            outs.append(self.forward(x[:, j].expand(self.n, 1)))
        return torch.stack(outs, 1).squeeze(-1).cpu().numpy()

    def save(self, path: str):
        np.savez(path, sizes=np.asarray(self.sizes), acts=np.asarray(self.acts),
                 **{f"k{i}": k.cpu().numpy() for i, k in enumerate(self.kernels)},
                 **{f"b{i}": b.cpu().numpy() for i, b in enumerate(self.biases)})

    def load(self, path: str):
        d = np.load(path, allow_pickle=False)
        self.kernels = [torch.as_tensor(d[f"k{i}"], device=self.device) for i in range(len(self.kernels))]
        self.biases = [torch.as_tensor(d[f"b{i}"], device=self.device) for i in range(len(self.biases))]
        return self

    def file_name(self, loops=None) -> str:
        loops = self.number_loops if loops is None else loops
        name = "nOL_{}inputDim_{}_nLoops_{}_fR_{}".format(len(self.acts), "_".join(
            [str(self.sizes[0])] + [f"{a}_{s}" for a, s in zip(self.acts, self.sizes[1:])]), loops, self.reduction.type)
        if self.hill:
            name += f"_standardDeviation_{self.sd}_numberOtRandomShots_{self.shots}"
        return name


# ====================================================================================
# PltData.py
# ====================================================================================
def plot_line(data, file_name, x=None, legend=(), text="", y_label="MSE", x_label="loops", width=1600, height=800):
    """Loss curve(s) as PNG (PltData.linePlot)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    data = np.asarray(data, dtype=float)
    plt.figure(figsize=(width / 96, height / 96))
    rows = data if data.ndim == 2 else data[None]
    for i, r in enumerate(rows):
        plt.plot(r if x is None else x, r if x is not None else None, label=legend[i] if i < len(legend) else None) \
            if x is not None else plt.plot(r, label=legend[i] if i < len(legend) else None)
    if text:
        plt.gcf().text(0.01, 0.01, text, fontsize=8)
    plt.xlabel(x_label)
    plt.ylabel(y_label)
    plt.grid(True)
    if legend:
        plt.legend()
    os.makedirs(os.path.dirname(os.path.abspath(file_name)), exist_ok=True)
    plt.savefig(file_name)
    plt.close()
    return file_name


def plot_nn_model(weights, file_name):
    """Network graph with weighted edges (PltData.plotNNModel, networkx)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    import networkx as nx
    g = nx.DiGraph()
    kernels = [np.asarray(w) for w in weights if np.asarray(w).ndim == 2]
    pos = {}
    for l, k in enumerate(kernels):
        for i in range(k.shape[0]):
            pos[(l, i)] = (l, -i)
            for j in range(k.shape[1]):
                pos[(l + 1, j)] = (l + 1, -j)
                g.add_edge((l, i), (l + 1, j), weight=float(k[i, j]))
    plt.figure(figsize=(8, 6))
    nx.draw(g, pos, node_size=80, width=[0.5 + 2 * abs(d["weight"]) for _, _, d in g.edges(data=True)])
    plt.savefig(file_name)
    plt.close()
    return file_name
