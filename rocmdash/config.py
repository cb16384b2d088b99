"""Configuration: environment variables and module constants.

Reference: ``app.py:21-24`` reads two env vars once at import and hard-codes the
5 s refresh period. The same two variables and defaults are kept verbatim so a
deployment of the reference can point this framework at the same Prometheus.
Everything new is env-overridable with a ``ROCMDASH_`` prefix and has a default
sized for one 8x MI355X node (288 GB HBM3E per GPU, 10 Hz amd-smi, 100 Hz HW
counters).
"""

from __future__ import annotations

import os
from dataclasses import dataclass, field


def _env_float(name: str, default: float) -> float:
    raw = os.environ.get(name)
    if raw is None or raw == "":
        return default
    try:
        return float(raw)
    except ValueError as exc:  # fail loudly: a typo in a DaemonSet env must not be silent
        raise ValueError(f"{name}={raw!r} is not a number") from exc


def _env_int(name: str, default: int) -> int:
    return int(_env_float(name, float(default)))


# --- reference-compatible names (app.py:22-24) ------------------------------------
PROMETHEUS_METRICS_ENDPOINT = os.environ.get(
    "PROMETHEUS_METRICS_ENDPOINT", "http://localhost:9090/api/v1/query"
)
PROMETHEUS_METRICS_PODNAME = os.environ.get("PROMETHEUS_METRICS_PODNAME", "prometheus")
# The reference hard-codes 5 s (app.py:24); same default, but env-overridable.
REFRESH_INTERVAL = _env_float("ROCMDASH_REFRESH_INTERVAL", 5.0)

# --- new knobs --------------------------------------------------------------------
# requests to Prometheus had no timeout in the reference (app.py:158,173).
HTTP_TIMEOUT_S = _env_float("ROCMDASH_HTTP_TIMEOUT", 5.0)


MAX_LDS_WINDOW = 32768  # csrc/window_stats.hip: sorted in LDS, updated incrementally
MAX_LONG_WINDOW = 1 << 26  # csrc/long_window.hip: HBM-resident, radix select per refresh


@dataclass
class SamplerConfig:
    """Rates and window sizes of the native sampling pipeline.

    ``window`` is the per-series sample window W the HIP stats kernel reduces
    (the analogue of a sequence length here); it must be a power of two.
    ``ring_capacity`` is the host ring's depth in rows (multiple of ``2 * window``).
    """

    smi_hz: float = field(default_factory=lambda: _env_float("ROCMDASH_SMI_HZ", 10.0))
    counter_hz: float = field(default_factory=lambda: _env_float("ROCMDASH_COUNTER_HZ", 100.0))
    window: int = field(default_factory=lambda: _env_int("ROCMDASH_WINDOW", 4096))
    ring_capacity: int = field(default_factory=lambda: _env_int("ROCMDASH_RING_CAPACITY", 16384))
    percentiles: tuple = (50.0, 90.0, 99.0)
    # A sample older than this many periods of its source marks the GPU "stale".
    stale_periods: float = field(default_factory=lambda: _env_float("ROCMDASH_STALE_PERIODS", 5.0))
    # request()/wait() hand-off with the sampler worker threads spins this long before
    # sleeping (closed-loop refreshes back to back); 0 = always sleep on the futex
    spin_us: float = field(default_factory=lambda: _env_float("ROCMDASH_SAMPLER_SPIN_US", 200.0))
    # "numa": sampler threads on the CPUs local to the GPU's PCIe root; "init": on the NUMA
    # node the runtime was started on (placement.py); "off": anywhere
    pin_samplers: str = field(default_factory=lambda: os.environ.get("ROCMDASH_PIN_SAMPLERS", "numa"))

    def __post_init__(self) -> None:
        if self.window <= 0 or self.window & (self.window - 1):
            raise ValueError(f"window must be a power of two, got {self.window}")
        if self.window > MAX_LONG_WINDOW:
            raise ValueError(f"window must be <= {MAX_LONG_WINDOW}")
        if self.ring_capacity <= 0 or self.ring_capacity & (self.ring_capacity - 1):
            raise ValueError("ring_capacity must be a power of two")
        if not self.long_window and self.ring_capacity % (2 * self.window):
            raise ValueError("ring_capacity must be a multiple of 2 x window (the device ring depth)")
        if self.smi_hz <= 0 or self.counter_hz <= 0:
            raise ValueError("sampling rates must be positive")

    @property
    def long_window(self) -> bool:
        """Windows beyond one workgroup's LDS live only in HBM (csrc/long_window.h); the
        host ring is then just the staging queue in front of them."""
        return self.window > MAX_LDS_WINDOW


EXPORTER_PORT = _env_int("ROCMDASH_EXPORTER_PORT", 9400)
MOCK_PROMETHEUS_PORT = _env_int("ROCMDASH_MOCK_PROMETHEUS_PORT", 9090)


def reload() -> None:
    """Re-read the environment (the reference reads it once at import)."""
    global PROMETHEUS_METRICS_ENDPOINT, PROMETHEUS_METRICS_PODNAME, REFRESH_INTERVAL
    global HTTP_TIMEOUT_S, EXPORTER_PORT, MOCK_PROMETHEUS_PORT
    PROMETHEUS_METRICS_ENDPOINT = os.environ.get(
        "PROMETHEUS_METRICS_ENDPOINT", "http://localhost:9090/api/v1/query"
    )
    PROMETHEUS_METRICS_PODNAME = os.environ.get("PROMETHEUS_METRICS_PODNAME", "prometheus")
    REFRESH_INTERVAL = _env_float("ROCMDASH_REFRESH_INTERVAL", 5.0)
    HTTP_TIMEOUT_S = _env_float("ROCMDASH_HTTP_TIMEOUT", 5.0)
    EXPORTER_PORT = _env_int("ROCMDASH_EXPORTER_PORT", 9400)
    MOCK_PROMETHEUS_PORT = _env_int("ROCMDASH_MOCK_PROMETHEUS_PORT", 9090)
