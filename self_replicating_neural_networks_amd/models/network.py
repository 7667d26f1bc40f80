"""Reference-compatible particle networks (facades over one population row).

Re-exposes the API of the reference's ``code/network.py`` — ``NeuralNetwork`` and its
Weightwise / Aggregating / FFT / Recurrent subclasses, ``ParticleDecorator``,
``TrainingNeuralNetworkDecorator`` and ``SaveStateCallback`` — without Keras.  A net owns a
1-row CPU weight table ``[1, spec.PP]``; every dynamic operation (self-application,
attack, SGD epoch, fixpoint predicates) is executed by the native library's host path
(the same C++ per-particle code as the HIP kernels), so single-net results match
population results on the GPU.  Large experiments should use ``Population`` /
``SoupEngine`` directly; these facades exist so reference-shaped scripts keep working.

Behavioural decisions:
* networks are linear and bias-free; ``with_keras_params`` is recorded but does not
  change the model, exactly as in the reference (S1);
* ``fuck`` (reverse attack) is kept under its reference name and aliased as
  ``reverse_attack``;
* ``meet`` returns ``self`` like the reference (the attacked copy is discarded) unless
  ``return_copy=True``;
* the verbose ``print_all_weight_updates`` path prints instead of crashing
  (code/network.py:275-278 called ``.format`` on ``print``'s return value);
* the FFT net uses the defined real-valued semantics of csrc FFTNet (S6).
"""
from __future__ import annotations

import copy
from typing import Callable, List, Optional

import numpy as np
import torch

from ..arch import ArchSpec, normalize_id as _normalize_id
from ..ops import _lib
from ..ops import kernels as K
from ..oracle import core as O
from ..utils import rng as _rng
from ..utils.printing import PrintingObject

# Reference quirks that change *recorded data*, reproducible on demand
REFERENCE_QUIRKS = {"savestate_time_doubling": False}


class _ModelView:
    """Minimal stand-in for the Keras model of a net (``net.model`` / ``get_model()``)."""

    def __init__(self, net):
        self._net = net

    def get_weights(self):
        return self._net.get_weights()

    def set_weights(self, w):
        return self._net.set_weights(w)

    def count_params(self):
        return self._net.spec.P

    @property
    def layers(self):
        return [tuple(s) for s in self._net.spec.layer_shapes]


class NeuralNetwork(PrintingObject):
    """Abstract particle (reference code/network.py:29-163)."""

    # ---------------------------------------------------------------- statics
    @staticmethod
    def weights_to_string(weights):
        s = ""
        for layer in weights:
            for cell in np.atleast_2d(layer):
                s += "[ " + "".join(str(w) + " " for w in cell) + "]"
            s += "\n"
        return s

    @staticmethod
    def are_weights_diverged(network_weights):
        return any(not np.all(np.isfinite(np.asarray(l, dtype=np.float64))) for l in network_weights)

    @staticmethod
    def are_weights_within(network_weights, lower_bound, upper_bound):
        for layer in network_weights:
            a = np.asarray(layer, dtype=np.float64)
            with np.errstate(invalid="ignore"):
                if not np.all((lower_bound <= a) & (a <= upper_bound)):
                    return False
        return True

    @staticmethod
    def fill_weights(old_weights, new_weights_list):
        new = copy.deepcopy(old_weights)
        k = 0
        for li, layer in enumerate(new):
            flat = layer.reshape(-1)
            for j in range(flat.shape[0]):
                flat[j] = new_weights_list[k]
                k += 1
            new[li] = flat.reshape(layer.shape)
        return new

    # ---------------------------------------------------------------- construction
    def __init__(self, spec: ArchSpec, **params):
        super().__init__()
        self.params = dict(epsilon=0.00000000000001)
        self.params.update(params)
        self.keras_params = dict(activation="linear", use_bias=False)
        self.states = []
        self._base_spec = spec
        self._key = _rng.next_init_key()
        self._table = torch.zeros((1, spec.PP), dtype=torch.float32)
        uid = torch.tensor([self._key], dtype=torch.int64)
        K.init_rows(spec, self._table, uid, _rng.get_seed())
        self.model = _ModelView(self)

    # spec may change through params (aggregator / shuffler functions)
    @property
    def spec(self) -> ArchSpec:
        return self._base_spec

    def get_model(self):
        return self.model

    def get_params(self):
        return self.params

    def get_keras_params(self):
        return self.keras_params

    def with_params(self, **kwargs):
        self.params.update(kwargs)
        return self

    def with_keras_params(self, **kwargs):
        # recorded only: the reference builds its model before this call
        self.keras_params.update(kwargs)
        return self

    def __deepcopy__(self, memo):
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            if k == "model":
                continue
            setattr(new, k, copy.deepcopy(v, memo))
        new.model = _ModelView(new)
        return new

    # ---------------------------------------------------------------- weights
    def get_weights(self) -> List[np.ndarray]:
        return self.spec.unflatten(self._table[0, : self.spec.P].numpy())

    def get_weights_flat(self) -> np.ndarray:
        return self._table[0, : self.spec.P].numpy().copy()

    def set_weights(self, new_weights):
        flat = self.spec.flatten(new_weights) if isinstance(new_weights, (list, tuple)) else \
            np.asarray(new_weights, dtype=np.float32).reshape(-1)
        if flat.shape[0] != self.spec.P:
            raise ValueError(f"expected {self.spec.P} weights, got {flat.shape[0]}")
        self._table[0, : self.spec.P] = torch.from_numpy(flat)

    def get_amount_of_weights(self):
        return self.spec.P

    # ---------------------------------------------------------------- application
    def _native(self) -> bool:
        return _lib.has_config(self.spec)

    def _apply_flat(self, target_flat: np.ndarray, target_spec: Optional[ArchSpec] = None) -> np.ndarray:
        """f_self(target) as a flat vector."""
        target_spec = target_spec or self.spec
        if target_spec == self.spec and self._native():
            t = torch.zeros((2, self.spec.PP), dtype=torch.float32)
            t[0] = self._table[0]
            t[1, : self.spec.P] = torch.from_numpy(np.asarray(target_flat, dtype=np.float32))
            out = torch.zeros((1, self.spec.PP), dtype=torch.float32)
            K.apply(self.spec, t, out, idx_f=torch.tensor([0]), idx_t=torch.tensor([1]), idx_o=torch.tensor([0]), n=1,
                    uid=torch.tensor([self._key, self._key], dtype=torch.int64), seed=_rng.get_seed(), ctr=_rng.next_op())
            return out[0, : self.spec.P].numpy().copy()
        return self._apply_flat_python(np.asarray(target_flat, dtype=np.float32), target_spec)

    def _apply_flat_python(self, target_flat, target_spec):
        raise NotImplementedError

    def apply_to_weights(self, old_weights):
        tspec = self._spec_of_weights(old_weights)
        new_flat = self._apply_flat(tspec.flatten(old_weights) if tspec is not None else
                                    np.hstack([np.asarray(w).reshape(-1) for w in old_weights]), tspec)
        if self.params.get("print_all_weight_updates", False) and not self.is_silent():
            print("updated weights:\n" + self.weights_to_string(self._unflatten_like(old_weights, new_flat)))
        return self._unflatten_like(old_weights, new_flat)

    def _spec_of_weights(self, weights) -> Optional[ArchSpec]:
        shapes = [tuple(np.asarray(w).shape) for w in weights]
        return self.spec if shapes == [tuple(s) for s in self.spec.layer_shapes] else None

    @staticmethod
    def _unflatten_like(like, flat):
        out, k = [], 0
        for w in like:
            a = np.asarray(w)
            out.append(np.asarray(flat[k:k + a.size], dtype=np.float32).reshape(a.shape))
            k += a.size
        return out

    def apply_to_network(self, other_network):
        return self.apply_to_weights(other_network.get_weights())

    def attack(self, other_network):
        other_network.set_weights(self.apply_to_network(other_network))
        return self

    def fuck(self, other_network):
        """Reverse attack: self <- f_self(other) (reference name, code/network.py:120-122)."""
        self.set_weights(self.apply_to_network(other_network))
        return self

    reverse_attack = fuck

    def self_attack(self, iterations=1):
        if iterations > 1 and self._native():
            K.run_fixpoint(self.spec, self._table, iterations, 1e-14, early_exit=False, with_sec=False,
                           uid=torch.tensor([self._key], dtype=torch.int64), seed=_rng.get_seed(),
                           ctr=_rng.next_op())
            return self
        for _ in range(iterations):
            self.attack(self)
        return self

    def meet(self, other_network, return_copy=False):
        new_other = copy.deepcopy(other_network)
        self.attack(new_other)
        return new_other if return_copy else self

    # ---------------------------------------------------------------- predicates
    def _eps(self, epsilon):
        return epsilon or self.get_params().get("epsilon")

    def is_diverged(self):
        return self.are_weights_diverged(self.get_weights())

    def is_zero(self, epsilon=None):
        e = self._eps(epsilon)
        return self.are_weights_within(self.get_weights(), -e, e)

    def is_fixpoint(self, degree=1, epsilon=None):
        assert degree >= 1, "degree must be >= 1"
        e = self._eps(epsilon)
        old = self.get_weights_flat()
        new = old
        for _ in range(degree):
            new = self._apply_flat(new)
        if not np.all(np.isfinite(new)):
            return False
        with np.errstate(invalid="ignore"):
            return not np.any(np.abs(new.astype(np.float64) - old.astype(np.float64)) >= e)

    def repr_weights(self, weights=None):
        return self.weights_to_string(weights or self.get_weights())

    def print_weights(self, weights=None):
        print(self.repr_weights(weights))

    # ---------------------------------------------------------------- training hooks
    def compute_samples(self):
        raise NotImplementedError

    def _train_epoch(self, samples_flat: np.ndarray, lr: float) -> float:
        """One SGD epoch on the samples generated from ``samples_flat``; returns the epoch loss."""
        spec = self.spec
        if not self._native():
            w, loss = O.train_epoch(spec, self._table[:, : spec.P].numpy(), samples_flat[None], lr, True,
                                    _rng.get_seed(), np.array([self._key], dtype=np.uint64), _rng.next_op())
            self._table[0, : spec.P] = torch.from_numpy(w[0])
            return float(loss[0])
        teach = torch.zeros((1, spec.PP), dtype=torch.float32)
        teach[0, : spec.P] = torch.from_numpy(np.asarray(samples_flat, dtype=np.float32))
        loss = K.learn_from(spec, self._table, teach, None, 1, lr, True,
                            uid=torch.tensor([self._key], dtype=torch.int64), seed=_rng.get_seed(), ctr=_rng.next_op())
        return float(loss[0])


# ====================================================================================
class WeightwiseNeuralNetwork(NeuralNetwork):
    """MLP 4 -> width ... -> 1 applied at every weight point (code/network.py:213-289)."""

    @staticmethod
    def normalize_id(value, norm):
        return _normalize_id(value, norm)

    def __init__(self, width, depth, **kwargs):
        self.width = width
        self.depth = depth
        super().__init__(ArchSpec.weightwise(width, depth), **kwargs)

    def apply(self, *inputs):
        """Net output at one (weight, layer, cell, position) point."""
        x = np.asarray(inputs[:4], dtype=np.float32)[None]
        mats = [m for m in self.spec.unflatten(self.get_weights_flat())]
        h = x
        for m in mats:
            h = (h @ m).astype(np.float32)
        return np.float32(h[0, 0])

    @classmethod
    def compute_all_duplex_weight_points(cls, old_weights):
        points, normal_points = [], []
        max_layer_id = len(old_weights) - 1
        for layer_id, layer in enumerate(old_weights):
            layer = np.atleast_2d(layer)
            max_cell_id = len(layer) - 1
            for cell_id, cell in enumerate(layer):
                max_weight_id = len(cell) - 1
                for weight_id, weight in enumerate(cell):
                    points.append([weight, layer_id, cell_id, weight_id])
                    normal_points.append([weight, cls.normalize_id(layer_id, max_layer_id),
                                          cls.normalize_id(cell_id, max_cell_id),
                                          cls.normalize_id(weight_id, max_weight_id)])
        return points, normal_points

    @classmethod
    def compute_all_weight_points(cls, all_weights):
        return cls.compute_all_duplex_weight_points(all_weights)[0]

    @classmethod
    def compute_all_normal_weight_points(cls, all_weights):
        return cls.compute_all_duplex_weight_points(all_weights)[1]

    def _apply_flat_python(self, target_flat, target_spec):
        # weightwise application to an arbitrary target shape: coordinates of the target
        if target_spec is None:
            raise ValueError("weightwise attack on weights without a known layout")
        co = target_spec.coords()
        x = np.concatenate([target_flat[:, None], co], axis=1).astype(np.float32)
        h = x
        for m in self.spec.unflatten(self.get_weights_flat()):
            h = (h @ m).astype(np.float32)
        return h[:, 0]

    def apply_to_weights(self, old_weights):
        tspec = self._spec_of_weights(old_weights)
        if tspec is None:
            # foreign target layout: coordinates from the target's own shapes
            _, normal = self.compute_all_duplex_weight_points(old_weights)
            x = np.asarray(normal, dtype=np.float32)
            h = x
            for m in self.spec.unflatten(self.get_weights_flat()):
                h = (h @ m).astype(np.float32)
            return self._unflatten_like(old_weights, h[:, 0])
        return super().apply_to_weights(old_weights)

    def compute_samples(self):
        x, y = O.samples(self.spec, self.get_weights_flat()[None])
        return x[0], y[0]


# ====================================================================================
class AggregatingNeuralNetwork(NeuralNetwork):
    """Chunk-aggregate -> MLP a->...->a -> broadcast back (code/network.py:292-439)."""

    @staticmethod
    def aggregate_average(weights):
        total, count = 0.0, 0
        for w in weights:
            total += float(w)
            count += 1
        return total / float(count)

    @staticmethod
    def aggregate_max(weights):
        max_found = weights[0]
        for w in weights:
            max_found = w if w > max_found else max_found
        return max_found

    @staticmethod
    def deaggregate_identically(aggregate, amount):
        return [aggregate for _ in range(amount)]

    @staticmethod
    def shuffle_not(weights_list):
        return weights_list

    @staticmethod
    def shuffle_random(weights_list):
        _rng.py_random().shuffle(weights_list)
        return weights_list

    def __init__(self, aggregates, width, depth, **kwargs):
        self.aggregates = aggregates
        self.width = width
        self.depth = depth
        super().__init__(ArchSpec.aggregating(aggregates, width, depth), **kwargs)

    def get_aggregator(self):
        return self.params.get("aggregator", self.aggregate_average)

    def get_deaggregator(self):
        return self.params.get("deaggregator", self.deaggregate_identically)

    def get_shuffler(self):
        return self.params.get("shuffler", self.shuffle_not)

    @property
    def spec(self) -> ArchSpec:
        agg = self.params.get("aggregator", None)
        shf = self.params.get("shuffler", None)
        aggregator = {None: "mean", AggregatingNeuralNetwork.aggregate_average: "mean",
                      AggregatingNeuralNetwork.aggregate_max: "max"}.get(agg, "custom")
        shuffler = {None: "none", AggregatingNeuralNetwork.shuffle_not: "none",
                    AggregatingNeuralNetwork.shuffle_random: "random"}.get(shf, "custom")
        b = self._base_spec
        if aggregator == "custom" or shuffler == "custom" or "deaggregator" in self.params:
            return b  # custom python callables: handled by the python path (_native() is False)
        return ArchSpec(b.kind, b.width, b.depth, b.aggregates, aggregator, shuffler)

    def _custom(self):
        return any(k in self.params and self.params[k] not in (AggregatingNeuralNetwork.aggregate_average,
                                                                 AggregatingNeuralNetwork.aggregate_max,
                                                                 AggregatingNeuralNetwork.shuffle_not,
                                                                 AggregatingNeuralNetwork.shuffle_random)
                   for k in ("aggregator", "shuffler")) or "deaggregator" in self.params

    def _native(self):
        return not self._custom() and _lib.has_config(self.spec)

    def apply(self, *inputs):
        g = np.asarray(inputs[: self.aggregates], dtype=np.float32)[None]
        h = g
        for m in self.spec.unflatten(self.get_weights_flat()):
            h = (h @ m).astype(np.float32)
        return h[0]

    @staticmethod
    def collect_weights(all_weights, collection_size):
        collections, nxt = [], []
        k = 0
        for layer in all_weights:
            for w in np.asarray(layer).reshape(-1):
                nxt.append(w)
                if (k + 1) % collection_size == 0:
                    collections.append(nxt)
                    nxt = []
                k += 1
        collections[-1] += nxt
        return collections, len(nxt)

    def get_collected_weights(self):
        return self.collect_weights(self.get_weights(), self.get_amount_of_weights() // self.aggregates)

    def get_aggregated_weights(self):
        collections, leftovers = self.get_collected_weights()
        return [self.get_aggregator()(c) for c in collections], leftovers

    def _apply_flat_python(self, target_flat, target_spec):
        cs = self.get_amount_of_weights() // self.aggregates
        collections, leftovers = self.collect_weights([target_flat], cs)
        old_aggs = [self.get_aggregator()(c) for c in collections]
        new_aggs = self.apply(*old_aggs)
        lst = []
        for k, agg in enumerate(new_aggs):
            lst += self.get_deaggregator()(agg, cs + leftovers if k == self.aggregates - 1 else cs)
        lst = self.get_shuffler()(lst)
        return np.asarray(lst, dtype=np.float32)

    def compute_samples(self):
        aggs, _ = self.get_aggregated_weights()
        s = np.asarray(aggs, dtype=np.float32)[None]
        return [s], [s]

    def is_fixpoint_after_aggregation(self, degree=1, epsilon=None):
        assert degree >= 1, "degree must be >= 1"
        e = self._eps(epsilon)
        old_aggs, _ = self.get_aggregated_weights()
        new = self.get_weights_flat()
        for _ in range(degree):
            new = self._apply_flat(new)
        if not np.all(np.isfinite(new)):
            return False
        cs = self.get_amount_of_weights() // self.aggregates
        collections, _ = self.collect_weights([new], cs)
        new_aggs = [self.get_aggregator()(c) for c in collections]
        for o, n in zip(old_aggs, new_aggs):
            if abs(n - o) >= e:
                return False, new_aggs
        return True, new_aggs


# ====================================================================================
class FFTNeuralNetwork(NeuralNetwork):
    """FFT-reduction net with defined real-valued semantics (see csrc FFTNet; S6)."""

    @staticmethod
    def aggregate_fft(weights, dims):
        flat = np.hstack([np.asarray(w).reshape(-1) for w in weights])
        return np.real(np.fft.fftn(flat, (dims,))).astype(np.float32)[None, ...]

    @staticmethod
    def deaggregate_identically(aggregate, dims):
        return np.real(np.fft.ifftn(np.asarray(aggregate).reshape(-1), (dims,))).astype(np.float32)

    shuffle_not = AggregatingNeuralNetwork.shuffle_not
    shuffle_random = AggregatingNeuralNetwork.shuffle_random

    def __init__(self, aggregates, width, depth, **kwargs):
        self.aggregates = aggregates
        self.width = width
        self.depth = depth
        super().__init__(ArchSpec.fft(aggregates, width, depth), **kwargs)

    def get_shuffler(self):
        return self.params.get("shuffler", self.shuffle_not)

    @property
    def spec(self) -> ArchSpec:
        shf = self.params.get("shuffler", None)
        b = self._base_spec
        s = "random" if shf is FFTNeuralNetwork.shuffle_random or shf is AggregatingNeuralNetwork.shuffle_random else "none"
        return ArchSpec(b.kind, b.width, b.depth, b.aggregates, "mean", s)

    def apply(self, inputs):
        h = np.asarray(inputs, dtype=np.float32).reshape(1, -1)
        for m in self.spec.unflatten(self.get_weights_flat()):
            h = (h @ m).astype(np.float32)
        return h[0]

    def _apply_flat_python(self, target_flat, target_spec):
        out = O.apply(self.spec, self.get_weights_flat()[None], np.asarray(target_flat, np.float32)[None])
        return out[0]

    def compute_samples(self):
        g = O.fft_reduce(self.spec, self.get_weights_flat()[None])
        return [g], [g]


# ====================================================================================
class RecurrentNeuralNetwork(NeuralNetwork):
    """Stacked linear SimpleRNN over the flat weight sequence (code/network.py:524-574)."""

    def __init__(self, width, depth, **kwargs):
        self.features = 1
        self.width = width
        self.depth = depth
        super().__init__(ArchSpec.recurrent(width, depth), **kwargs)

    def apply(self, *inputs):
        seq = np.asarray(inputs, dtype=np.float32)[None]
        return O.apply(self.spec, self.get_weights_flat()[None], seq)[0] if seq.shape[1] == self.spec.P else \
            O._rnn_forward(self.spec, O._mats(self.spec, self.get_weights_flat()[None]), seq)[0][0]

    def _apply_flat_python(self, target_flat, target_spec):
        seq = np.asarray(target_flat, dtype=np.float32)[None]
        return O._rnn_forward(self.spec, O._mats(self.spec, self.get_weights_flat()[None]), seq)[0][0]

    def compute_samples(self):
        s = self.get_weights_flat()[None, :, None]
        return s, s


# ====================================================================================
class ParticleDecorator:
    """Gives a net a process-global uid and a state trajectory (code/network.py:166-210)."""

    next_uid = 0

    def __init__(self, net):
        self.uid = self.__class__.next_uid
        self.__class__.next_uid += 1
        self.net = net
        self.states = []
        self.save_state(time=0, action="init", counterpart=None)

    def __getattr__(self, name):
        if name in ("net", "__deepcopy__", "__getstate__", "__setstate__"):
            raise AttributeError(name)
        return getattr(self.net, name)

    def get_uid(self):
        return self.uid

    def make_state(self, **kwargs):
        weights = self.net.get_weights_flat()
        if np.any(np.isinf(weights)) or np.any(np.isnan(weights)):
            return None
        state = {"class": self.net.__class__.__name__, "weights": weights}
        state.update(kwargs)
        return state

    def save_state(self, **kwargs):
        state = self.make_state(**kwargs)
        if state is not None:
            self.states.append(state)

    def update_state(self, number, **kwargs):
        raise NotImplementedError("Result is vague")

    def get_states(self):
        return self.states


class SaveStateCallback:
    """Epoch-end hook recording a 'train_self' state (code/network.py:15-26)."""

    def __init__(self, net, epoch=0):
        self.net = net
        self.init_epoch = epoch

    def on_epoch_end(self, epoch, logs=None):
        t = epoch + self.init_epoch if REFERENCE_QUIRKS["savestate_time_doubling"] else epoch
        if hasattr(self.net, "save_state"):
            self.net.save_state(time=t, action="train_self", counterpart=None)


class TrainingNeuralNetworkDecorator:
    """Self-training (SGD, MSE, batch 1, shuffled) and learn_from (code/network.py:577-626)."""

    def __init__(self, net, **kwargs):
        self.net = net
        self.compile_params = dict(loss="mse", optimizer="sgd")
        self.model_compiled = False

    def __getattr__(self, name):
        if name in ("net", "__deepcopy__", "__getstate__", "__setstate__"):
            raise AttributeError(name)
        return getattr(self.net, name)

    def with_params(self, **kwargs):
        self.net.with_params(**kwargs)
        return self

    def with_keras_params(self, **kwargs):
        self.net.with_keras_params(**kwargs)
        return self

    def get_compile_params(self):
        return self.compile_params

    def with_compile_params(self, **kwargs):
        self.compile_params.update(kwargs)
        return self

    def _lr(self) -> float:
        cp = self.compile_params
        if "lr" in cp:
            return float(cp["lr"])
        opt = cp.get("optimizer", "sgd")
        if isinstance(opt, str):
            if opt.lower() != "sgd":
                raise NotImplementedError(f"optimizer {opt!r}: only SGD (the reference's) is implemented")
            return 0.01
        return float(getattr(opt, "lr", getattr(opt, "learning_rate", 0.01)))

    def compile_model(self, **kwargs):
        self.compile_params.update(kwargs)
        if self.compile_params.get("loss", "mse") not in ("mse", "mean_squared_error"):
            raise NotImplementedError("only the MSE loss of the reference is implemented")
        return None

    def compiled(self, **kwargs):
        if not self.model_compiled:
            self.compile_model(**kwargs)
            self.model_compiled = True
        return self

    def _inner(self) -> NeuralNetwork:
        n = self.net
        while not isinstance(n, NeuralNetwork):
            n = n.net
        return n

    def train(self, batchsize=1, store_states=True, epoch=0):
        if batchsize != 1:
            raise NotImplementedError("batch size 1 only (reference default)")
        self.compiled()
        inner = self._inner()
        loss = inner._train_epoch(inner.get_weights_flat(), self._lr())
        if store_states:
            SaveStateCallback(net=self, epoch=epoch).on_epoch_end(epoch)
        return loss

    def learn_from(self, other_network, batchsize=1):
        self.compiled()
        inner = self._inner()
        other = other_network
        while not isinstance(other, NeuralNetwork):
            other = other.net
        return inner._train_epoch(other.get_weights_flat(), self._lr())

    def save_state(self, **kwargs):
        n = self.net
        if hasattr(n, "save_state"):
            return n.save_state(**kwargs)

    def __deepcopy__(self, memo):
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            setattr(new, k, copy.deepcopy(v, memo))
        return new


def net_spec(net) -> ArchSpec:
    """ArchSpec of a (possibly decorated) network facade."""
    while not isinstance(net, NeuralNetwork):
        net = net.net
    return net.spec


def inner_net(net) -> NeuralNetwork:
    while not isinstance(net, NeuralNetwork):
        net = net.net
    return net
