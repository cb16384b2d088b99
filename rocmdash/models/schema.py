"""Metric schema shared by the native runtime, the exporter, the query layer and the UI.

Reference anchors:
  * the five series the reference asks Prometheus for (``app.py:168-170``) and the
    ``card_model`` label it reads (``app.py:192``) -> :data:`COMPAT_METRICS`;
  * the derived ``vram_usage_ratio`` column (``app.py:210-212``);
  * the mean/max/min statistics (``app.py:216-221``).

The native row layouts (``csrc/sources.h`` ``SmiField`` / ``CtrField``) are mirrored
here so pure-Python code (tests, the mock Prometheus, the CPU reference of the stats
kernel) does not need the extension; :func:`check_native_layout` asserts they agree.
"""

from __future__ import annotations

from dataclasses import dataclass

# app.py:169-170, in the reference's query order.
COMPAT_METRICS = (
    "amd_gpu_edge_temperature",
    "amd_gpu_gfx_activity",
    "amd_gpu_average_package_power",
    "amd_gpu_used_vram",
    "amd_gpu_total_vram",
)

# Row layout of the amd-smi source ring (csrc/sources.h SmiField).
SMI_FIELDS = (
    "amd_gpu_edge_temperature",
    "amd_gpu_gfx_activity",
    "amd_gpu_average_package_power",
    "amd_gpu_used_vram",
    "amd_gpu_total_vram",
    "amd_gpu_junction_temperature",
    "amd_gpu_memory_temperature",
    "amd_gpu_umc_activity",
    "amd_gpu_xgmi_read_bandwidth",
    "amd_gpu_xgmi_write_bandwidth",
    "amd_gpu_pcie_bandwidth",
)

# Row layout of the hardware-counter source ring (csrc/sources.h CtrField).
CTR_FIELDS = (
    "amd_gpu_mfma_utilization",
    "amd_gpu_hbm_read_bandwidth",
    "amd_gpu_hbm_write_bandwidth",
    "amd_gpu_gfx_busy",
    "amd_gpu_cu_active",
)

# How often each amd-smi column carries NEW data (bench.py's fresh-sample count):
#   * the SMU gpu_metrics table columns change only when the firmware publishes a new
#     table (tens of times per second; csrc/sources.cpp counts raw_table_changes);
#   * used VRAM is read live from its own sysfs attribute on every sample;
#   * total VRAM is a constant of the board.
SMI_LIVE_FIELDS = ("amd_gpu_used_vram",)
SMI_STATIC_FIELDS = ("amd_gpu_total_vram",)
SMI_TABLE_FIELDS = tuple(f for f in SMI_FIELDS if f not in SMI_LIVE_FIELDS + SMI_STATIC_FIELDS)

# Per-rank source health, appended to each rank's gathered stats tensor as one row of
# 8 floats per source (smi, counter), so rank 0 sees every rank's sampler health with
# no extra collective (rocmdash/runtime/pipeline.py). Counts are split into exact
# float32 halves: total = hi * 2**24 + lo.
HEALTH_SOURCES = ("smi", "counter")
HEALTH_FIELDS = ("samples_hi", "samples_lo", "failures_hi", "failures_lo", "overruns", "age_s", "hz", "present")
HEALTH_INDEX = {n: i for i, n in enumerate(HEALTH_FIELDS)}
HEALTH_SPLIT = float(1 << 24)

# Output slots of the window-stats kernel (csrc/window_stats.h StatSlot). The three
# percentile slots default to p50 / p90 / p99.
STAT_NAMES = ("min", "max", "mean", "p50", "p90", "p99", "last", "count")
STAT_INDEX = {n: i for i, n in enumerate(STAT_NAMES)}
NUM_STATS = len(STAT_NAMES)

# Accelerator complex dies (XCDs) per MI355X: the SMU table reports busy and gfx clock
# per XCD (csrc/sources.h kMaxXcds); exported as amd_gpu_xcd_activity / _gfx_clock
XCDS = 8

# Rows a node-service rank appends to its gathered [S, 8] statistics besides the
# health rows, so ONE all-gather per refresh carries everything rank 0 exports and
# every rank's stop vote (rocmdash/runtime/pipeline.py, rocmdash/serve.py):
#   XCD_ROWS    per-XCD busy (%) and gfx clock (MHz) of the latest SMU sample
#   CONTROL_ROW the rank's stop vote (1: stop after this refresh), its own footprint -
#               process HBM (MB), resident host memory (MB), CPU time in ms and the part
#               of it spent by SCHED_IDLE threads (rocmdash.runtime.threads), both split
#               into exact float32 halves (hi * 2**24 + lo: the exported counters stay
#               exact and monotone for years, where float32 seconds would round to
#               0.25 s after a month) - and its gather state: gathers validated bit for
#               bit so far on the native RCCL gather, -1 on the host fallback
XCD_ROWS = 2
CONTROL_FIELDS = ("stop", "self_hbm_mb", "self_rss_mb", "self_cpu_ms_hi", "self_cpu_ms_lo", "self_cpu_idle_ms_hi",
                  "self_cpu_idle_ms_lo", "gather_validated")
CONTROL_INDEX = {n: i for i, n in enumerate(CONTROL_FIELDS)}
# The rank's SOURCE row (after the control row): how its amd-smi source reads the SMU
# table - 1 raw sysfs table / 0 amd-smi, the calibration attempts (start-up + retries),
# the last attempt's matched raw / amd-smi / raw triples (of 8; -1 none), the retries
# that promoted it to the raw path, 1 when the table can never calibrate - so rank 0
# exports every GPU's fast-path state (rocmdash_smi_raw_path{gpu_id}, rocmdash.serve).
SOURCE_FIELDS = ("smi_raw_path", "smi_calibration_attempts", "smi_calibration_matched", "smi_calibration_promotions",
                 "smi_calibration_final", "reserved0", "reserved1", "reserved2")
SOURCE_INDEX = {n: i for i, n in enumerate(SOURCE_FIELDS)}
CONTROL_ROWS = 2  # the control row and the source row


@dataclass(frozen=True)
class MetricSpec:
    name: str
    unit: str
    help: str
    axis_max: float | None = None  # default gauge axis max (None = per-GPU / derived)


METRIC_SPECS = {
    s.name: s
    for s in (
        MetricSpec("amd_gpu_edge_temperature", "C", "GPU edge temperature (hotspot where the edge sensor is absent)", 100),
        MetricSpec("amd_gpu_gfx_activity", "%", "Graphics/compute engine activity", 100),
        MetricSpec("amd_gpu_average_package_power", "W", "Socket power (current_socket_power on MI300+)", None),
        MetricSpec("amd_gpu_used_vram", "MB", "Used VRAM (HBM)", None),
        MetricSpec("amd_gpu_total_vram", "MB", "Total VRAM (HBM)", None),
        MetricSpec("amd_gpu_junction_temperature", "C", "Junction (hotspot) temperature", 110),
        MetricSpec("amd_gpu_memory_temperature", "C", "HBM temperature", 105),
        MetricSpec("amd_gpu_umc_activity", "%", "Memory controller activity", 100),
        MetricSpec("amd_gpu_xgmi_read_bandwidth", "GB/s", "xGMI receive bandwidth, all links (SMU accumulators)", 600),
        MetricSpec("amd_gpu_xgmi_write_bandwidth", "GB/s", "xGMI send bandwidth, all links (SMU accumulators)", 600),
        MetricSpec("amd_gpu_pcie_bandwidth", "GB/s", "PCIe bandwidth (SMU instantaneous figure)", 128),
        MetricSpec("amd_gpu_mfma_utilization", "%", "Matrix-core (MFMA) busy share of SIMD cycles", 100),
        # memory-side traffic (csrc/counters.cpp): L2 misses / write-backs the memory
        # fabric served - HBM or the Infinity Cache (MALL) in front of it - exact for every
        # request size; the 8000 GB/s axis is the HBM peak, a MALL-resident loop can pass it
        MetricSpec("amd_gpu_hbm_read_bandwidth", "GB/s",
                   "Memory-side read bandwidth: L2 misses served by HBM or the Infinity Cache (MALL)", 8000),
        MetricSpec("amd_gpu_hbm_write_bandwidth", "GB/s",
                   "Memory-side write bandwidth: L2 write-backs to HBM or the Infinity Cache (MALL)", 8000),
        MetricSpec("amd_gpu_gfx_busy", "%", "GRBM GUI-active share of cycles", 100),
        MetricSpec("amd_gpu_cu_active", "%", "Share of CU-cycles with at least one wave resident", 100),
    )
}


def series_names(with_counters: bool = True) -> tuple:
    """Series order of one rank's stats tensor: smi ring columns, then counter ring."""
    return SMI_FIELDS + (CTR_FIELDS if with_counters else ())


def check_native_layout(native) -> None:
    """Fail loudly if the compiled row layouts drifted from this schema."""
    if tuple(native.SMI_FIELDS) != SMI_FIELDS or tuple(native.CTR_FIELDS) != CTR_FIELDS:
        raise RuntimeError(
            "rocmdash._native row layout differs from rocmdash.models.schema: "
            f"{native.SMI_FIELDS} / {native.CTR_FIELDS}"
        )
