"""Per-generation metrics as a JSONL stream.

The reference logs the counters dict of ``Soup.count`` / ``FixpointExperiment.count`` to
``log.txt`` (code/experiment.py:35-42, code/soup.py:89-103) and shows losses in tqdm
postfixes.  :class:`MetricsWriter` records, per sampled generation: the global census and
its fractions, the respawn count, the mean self-train loss, the uid counter and the
throughput since the previous record -- one JSON object per line, rank 0 only.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional

CLASSES = ("divergent", "fix_zero", "fix_other", "fix_sec", "other")


class MetricsWriter:
    def __init__(self, path: Optional[str], every: int = 1, rank: int = 0, extra: Optional[Dict] = None):
        self.path = path
        self.every = max(int(every), 1)
        self.rank = rank
        self.extra = dict(extra or {})
        self._f = None
        self._t = None
        self._gen = None
        self.records = []  # kept in memory too (tests / in-process consumers)
        if path and rank == 0:
            d = os.path.dirname(os.path.abspath(path))
            os.makedirs(d, exist_ok=True)
            self._f = open(path, "a", buffering=1)

    def due(self, generation: int) -> bool:
        return generation % self.every == 0

    def log(self, generation: int, census: Dict[str, int], n_total: int, respawns: Optional[int] = None,
            mean_loss: Optional[float] = None, next_uid: Optional[int] = None, **kw) -> Dict:
        now = time.perf_counter()
        rec = dict(generation=int(generation), time=time.time(), census={k: int(census.get(k, 0)) for k in CLASSES})
        tot = max(sum(rec["census"].values()), 1)
        rec["fractions"] = {k: v / tot for k, v in rec["census"].items()}
        rec["fixpoint_fraction"] = (rec["census"]["fix_zero"] + rec["census"]["fix_other"]
                                    + rec["census"]["fix_sec"]) / tot
        if respawns is not None:
            rec["respawns"] = int(respawns)
        if mean_loss is not None:
            rec["mean_loss"] = float(mean_loss)
        if next_uid is not None:
            rec["next_uid"] = int(next_uid)
        if self._t is not None and self._gen is not None and generation > self._gen:
            dt = now - self._t
            rec["ms_per_generation"] = dt / (generation - self._gen) * 1e3
            rec["particle_generations_per_s"] = n_total * (generation - self._gen) / dt if dt > 0 else None
        rec.update(self.extra)
        rec.update(kw)
        self._t, self._gen = now, generation
        self.records.append(rec)
        if self._f is not None:
            self._f.write(json.dumps(rec) + "\n")
        return rec

    def close(self):
        if self._f is not None:
            self._f.close()
            self._f = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_metrics(path: str):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]
