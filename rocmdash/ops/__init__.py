"""Device ops: the CDNA4 windowed-statistics kernel and its CPU/PyTorch references."""

from .window_stats import (  # noqa: F401
    DEFAULT_PCT,
    window_stats,
    window_stats_reference,
    window_stats_torch,
)
