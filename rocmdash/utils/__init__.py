"""Small shared utilities: latency histograms / percentiles, natural sort."""

from .timing import LatencyHistogram, Stopwatch, percentile  # noqa: F401
from ..viz.panels import natural_key  # noqa: F401
