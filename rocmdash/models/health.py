"""Per-source sampler health of every GPU of the node.

Reference counterpart: the reference has one failure signal, the ``st.error`` banner
of a failed Prometheus fetch (``app.py:225-227``); a GPU whose exporter stopped
updating is invisible to it. Here every rank appends its sources' health rows
(``schema.HEALTH_FIELDS``) to the stats tensor it all-gathers, so rank 0 knows, per
GPU and per source, how many samples and failures there were and how old the newest
sample is - and exports ``rocmdash_source_stale`` / ``rocmdash_sample_age_seconds`` /
``rocmdash_sampler_*_total`` for every GPU, and degrades ``/healthz`` when any is stale.
"""

from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from .schema import HEALTH_INDEX, HEALTH_SOURCES, HEALTH_SPLIT


@dataclass
class SourceStatus:
    gpu: int  # row in the node tensor
    kind: str  # "smi" | "counter"
    backend: str
    samples: int
    failures: int
    overruns: int
    age_s: float  # NaN: no sample yet
    hz: float
    stale: bool


class SourceHealth:
    """``rows`` [N, len(HEALTH_SOURCES), 8] float32 as gathered; ``backends`` per GPU
    (smi_backend, counter_backend); a source is stale when its newest sample is older
    than ``stale_periods`` of its sampling periods, or it has none."""

    def __init__(self, rows: np.ndarray, backends: list, stale_periods: float = 5.0):
        self.rows = np.asarray(rows, dtype=np.float64)
        if self.rows.ndim != 3 or self.rows.shape[1] != len(HEALTH_SOURCES):
            raise ValueError(f"health rows must be [N, {len(HEALTH_SOURCES)}, 8], got {self.rows.shape}")
        self.backends = list(backends)
        self.stale_periods = float(stale_periods)

    def statuses(self) -> list:
        H = HEALTH_INDEX
        out = []
        for g in range(self.rows.shape[0]):
            for i, kind in enumerate(HEALTH_SOURCES):
                r = self.rows[g, i]
                if not r[H["present"]] == 1.0:
                    continue
                age, hz = float(r[H["age_s"]]), float(r[H["hz"]])
                limit = self.stale_periods / hz if hz > 0 else math.inf
                stale = math.isnan(age) or age > limit
                backend = self.backends[g][i] if g < len(self.backends) and i < len(self.backends[g]) else ""
                out.append(SourceStatus(
                    g, kind, backend,
                    int(r[H["samples_hi"]] * HEALTH_SPLIT + r[H["samples_lo"]]),
                    int(r[H["failures_hi"]] * HEALTH_SPLIT + r[H["failures_lo"]]),
                    int(r[H["overruns"]]), age, hz, stale))
        return out

    def stale_gpus(self) -> list:
        """Rows of the GPUs with at least one stale source."""
        return sorted({s.gpu for s in self.statuses() if s.stale})
