"""The reference's prototype and scratch particle APIs, population-batched.

* ``code/methods.py``: an alternate functional-Keras design.  ``Network``
  describes a stack (features, cells, layers, recurrent) with an analytic parameter count
  (:17-60); ``RecurrentNetwork.fit`` (:99-129) iterates self-application of a SimpleRNN
  stack that reads its own flat weights as a (P/features, features) sequence;
  ``FeedForwardNetwork.fit`` (:132-174) maps every weight with the input
  ``(weight, index / num_cells)`` through a dense stack.  Both record
  ``mean_sqrd_error(new, old)`` -- the self-application loss -- per step.
* ``code/test.py``: the deprecated ``LearningNeuralNetwork`` (its constructor
  raises ``DeprecationWarning``, :28) with the mean / fft / random weight reductions
  (:10-25), and ``vary(e, f)`` (:84-89), the perturbed identity fixpoint.

Here a prototype is a *population* of such nets: weights are batched tensors
``[N, ...]`` (any torch device), every step is a batched matmul chain, and ``fit`` returns
the per-step losses of every particle (``[epochs, N]``).  These are not hot paths of the
reference (they are prototypes), so they are plain PyTorch rather than HIP kernels.
Initialisation follows Keras: glorot-uniform kernels, orthogonal recurrent kernels.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch


class Network:
    """Stack description with the reference's analytic parameter count
    (code/methods.py:17-60).  ``parameters`` is the reference formula; ``layer_shapes``
    / ``actual_parameters`` describe the stack that is actually built (for the
    feed-forward stack the formula counts a ``features x cells`` output layer while the
    built model ends in ``Dense(1)``; the reference only asserts the recurrent count)."""

    def __init__(self, features: int, cells: int, layers: int, bias: bool = False, recurrent: bool = False):
        if bias:
            raise NotImplementedError("the prototypes were only built without biases (code/methods.py:44-49)")
        self.features, self.cells, self.num_layer, self.recurrent = features, cells, layers, recurrent
        if recurrent:
            p1 = features * cells + cells ** 2
            pn = (cells * cells + cells ** 2) * (layers - 1)
        else:
            p1 = features * cells
            pn = cells * cells * (layers - 1)
        self.parameters = int(p1 + pn + features * cells)

    def layer_shapes(self) -> List[tuple]:
        f, c, L = self.features, self.cells, self.num_layer
        shapes = []
        for l in range(L):
            shapes.append((f if l == 0 else c, c))
            if self.recurrent:
                shapes.append((c, c))
        shapes.append((c, f if self.recurrent else 1))
        return shapes

    @property
    def actual_parameters(self) -> int:
        return int(sum(a * b for a, b in self.layer_shapes()))


def _glorot(n, a, b, g, device):
    lim = (6.0 / (a + b)) ** 0.5
    return (torch.rand((n, a, b), generator=g, dtype=torch.float64) * 2 - 1).mul_(lim).float().to(device)


def _orthogonal(n, k, g, device):
    q, r = torch.linalg.qr(torch.randn((n, k, k), generator=g, dtype=torch.float64))
    d = torch.sign(torch.diagonal(r, dim1=-2, dim2=-1))
    d[d == 0] = 1
    return (q * d[:, None, :]).float().to(device)


class _BaseNetwork:
    """Population of prototype nets (code/methods.py:63-96)."""

    def __init__(self, network: Network, n: int = 1, device="cpu", seed: int = 0):
        self.network = network
        self.features = network.features
        self.n = int(n)
        self.device = torch.device(device)
        g = torch.Generator().manual_seed(int(seed))
        self.weights: List[torch.Tensor] = []
        shapes = network.layer_shapes()
        for idx, (a, b) in enumerate(shapes):
            recurrent_kernel = network.recurrent and idx < len(shapes) - 1 and idx % 2 == 1
            self.weights.append(_orthogonal(self.n, a, g, self.device) if recurrent_kernel
                                else _glorot(self.n, a, b, g, self.device))

    def get_weights(self) -> List[torch.Tensor]:
        return [w.clone() for w in self.weights]

    def set_weights(self, ws):
        self.weights = [torch.as_tensor(w, dtype=torch.float32, device=self.device).reshape(self.weights[i].shape)
                        for i, w in enumerate(ws)]

    def get_weights_flat(self) -> torch.Tensor:
        """[N, P] in Keras get_weights() order (row-major kernels)."""
        return torch.cat([w.reshape(self.n, -1) for w in self.weights], dim=1)

    def _set_flat(self, flat: torch.Tensor):
        out, o = [], 0
        for w in self.weights:
            k = w[0].numel()
            out.append(flat[:, o:o + k].reshape(w.shape).contiguous())
            o += k
        self.weights = out

    def get_parameter_count(self) -> int:
        return int(sum(w[0].numel() for w in self.weights))

    @staticmethod
    def mean_abs_error(labels, predictions):
        return (predictions - labels).abs().mean(dim=-1)

    @staticmethod
    def mean_sqrd_error(labels, predictions):
        return (predictions - labels).square().mean(dim=-1)

    def step(self, x):
        raise NotImplementedError

    def fit(self, epochs: int = 500) -> torch.Tensor:
        """Iterated self-application; returns the losses MSE(new, old), [epochs, N]."""
        losses = []
        for _ in range(int(epochs)):
            old = self.get_weights_flat()
            y = self.step(old)
            losses.append(self.mean_sqrd_error(y, old))
            self._set_flat(y)
        return torch.stack(losses) if losses else torch.zeros((0, self.n))


class RecurrentNetwork(_BaseNetwork):
    """Linear SimpleRNN stack reading its own weights as a sequence of ``features``-vectors
    (code/methods.py:99-129)."""

    def __init__(self, network: Network, n: int = 1, device="cpu", seed: int = 0):
        if not network.recurrent:
            raise ValueError("RecurrentNetwork needs Network(..., recurrent=True)")
        super().__init__(network, n, device, seed)
        self.parameters = network.parameters
        if self.get_parameter_count() != self.parameters:
            raise AssertionError("parameter count differs from the analytic formula")
        if self.parameters % self.features:
            raise ValueError("parameters must be a multiple of features")

    def step(self, x: torch.Tensor) -> torch.Tensor:
        n, L = self.n, self.network.num_layer
        seq = x.reshape(n, -1, self.features)  # [N, T, features]
        for l in range(L):
            K, U = self.weights[2 * l], self.weights[2 * l + 1]
            h = torch.zeros((n, U.shape[1]), dtype=x.dtype, device=x.device)
            outs = []
            for t in range(seq.shape[1]):
                h = torch.bmm(seq[:, t:t + 1, :], K)[:, 0] + torch.bmm(h[:, None, :], U)[:, 0]
                outs.append(h)
            seq = torch.stack(outs, dim=1)
        return torch.bmm(seq, self.weights[-1]).reshape(n, -1)


class FeedForwardNetwork(_BaseNetwork):
    """Dense stack applied to every weight with the input (weight, index / num_cells)
    (code/methods.py:132-174)."""

    def __init__(self, network: Network, n: int = 1, device="cpu", seed: int = 0):
        if network.recurrent:
            raise ValueError("FeedForwardNetwork needs Network(..., recurrent=False)")
        if network.features != 2:
            raise ValueError("the feed-forward prototype feeds (weight, index / num_cells): features must be 2")
        super().__init__(network, n, device, seed)
        self.parameters = network.parameters
        self.num_layer = network.num_layer
        self.num_cells = network.cells

    def step(self, x: torch.Tensor) -> torch.Tensor:
        P = x.shape[1]
        cell_idx = torch.arange(P, dtype=x.dtype, device=x.device) / self.num_cells  # reference quirk: / cells
        h = torch.stack([x, cell_idx.expand_as(x)], dim=2)  # [N, P, 2]
        for w in self.weights:
            h = torch.bmm(h, w)
        return h[:, :, 0]


# ------------------------------------------------------------------ code/test.py (C31)
class LearningNeuralNetwork:
    """Deprecated in the reference: the constructor raises ``DeprecationWarning``
    (code/test.py:28).  Its weight reductions stay available as static helpers."""

    @staticmethod
    def mean_reduction(weights, features):
        flat = np.hstack([np.asarray(w).flatten() for w in weights])
        return np.mean(np.reshape(flat, (1, features, -1)), axis=-1)

    @staticmethod
    def fft_reduction(weights, features):
        flat = np.hstack([np.asarray(w).flatten() for w in weights])
        return np.fft.fft(flat, n=features)[None, ...]

    @staticmethod
    def random_reduction(_, features, rng: Optional[np.random.Generator] = None):
        rng = rng or np.random.default_rng()
        return rng.random(features)[None, ...]

    def __init__(self, *args, **kwargs):
        raise DeprecationWarning


def vary(e: float = 0.0, f: float = 0.0):
    """The Weightwise(2, 2) identity fixpoint with the identity entries shifted by ``e``
    and every other entry set to ``f`` (code/test.py:84-89)."""
    return [
        np.array([[1.0 + e, 0.0 + f], [0.0 + f, 0.0 + f], [0.0 + f, 0.0 + f], [0.0 + f, 0.0 + f]], dtype=np.float32),
        np.array([[1.0 + e, 0.0 + f], [0.0 + f, 0.0 + f]], dtype=np.float32),
        np.array([[1.0 + e], [0.0 + f]], dtype=np.float32),
    ]
