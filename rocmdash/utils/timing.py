"""Latency recording: percentiles for benchmarks and Prometheus histograms for the
exporter / service (refresh, scrape and sampling durations).

Reference counterpart: none - the reference measures nothing about itself; its only
self-report is the "Last updated" footer (app.py:484).
"""

from __future__ import annotations

import bisect
import math
import threading
import time
from contextlib import contextmanager

# seconds; spans a 10 us device refresh up to a multi-second Prometheus stall
DEFAULT_BUCKETS = (1e-5, 2.5e-5, 5e-5, 1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2, 2.5e-2, 5e-2, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0)


def percentile(sorted_values, q: float) -> float:
    """Linear-interpolated percentile (numpy's default) of an ascending sequence."""
    n = len(sorted_values)
    if n == 0:
        return math.nan
    pos = q / 100.0 * (n - 1)
    lo = int(math.floor(pos))
    hi = min(lo + 1, n - 1)
    f = pos - lo
    return sorted_values[lo] + (sorted_values[hi] - sorted_values[lo]) * f


class LatencyHistogram:
    """Thread-safe cumulative histogram in Prometheus' bucket layout."""

    def __init__(self, name: str, help: str = "", buckets=DEFAULT_BUCKETS):
        self.name = name
        self.help = help
        self.buckets = tuple(sorted(buckets))
        self._counts = [0] * (len(self.buckets) + 1)
        self._sum = 0.0
        self._n = 0
        self._lock = threading.Lock()

    def observe(self, seconds: float) -> None:
        i = bisect.bisect_left(self.buckets, seconds)
        with self._lock:
            self._counts[i] += 1
            self._sum += seconds
            self._n += 1

    @contextmanager
    def time(self):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.observe(time.perf_counter() - t0)

    @property
    def count(self) -> int:
        return self._n

    def add_to(self, exposition, labels: dict | None = None) -> None:
        """Append ``<name>_bucket{le}``, ``_sum`` and ``_count`` to an Exposition."""
        labels = dict(labels or {})
        with self._lock:
            counts = list(self._counts)
            total, n = self._sum, self._n
        cum = 0
        for b, c in zip(self.buckets, counts):
            cum += c
            exposition.add(self.name + "_bucket", cum, {**labels, "le": repr(float(b))}, self.help, "histogram", self.name)
        exposition.add(self.name + "_bucket", n, {**labels, "le": "+Inf"}, self.help, "histogram", self.name)
        exposition.add(self.name + "_sum", total, labels, self.help, "histogram", self.name)
        exposition.add(self.name + "_count", n, labels, self.help, "histogram", self.name)


class Stopwatch:
    """Collects durations (ms) and summarises them."""

    def __init__(self):
        self.ms = []

    @contextmanager
    def lap(self):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.ms.append((time.perf_counter() - t0) * 1e3)

    def summary(self, drop: int = 0) -> dict:
        v = sorted(self.ms[drop:])
        return {
            "n": len(v),
            "p50_ms": percentile(v, 50),
            "p90_ms": percentile(v, 90),
            "p99_ms": percentile(v, 99),
            "min_ms": v[0] if v else math.nan,
            "max_ms": v[-1] if v else math.nan,
        }
