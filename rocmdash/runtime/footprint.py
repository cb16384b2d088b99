"""The exporter's own cost on the node it watches: HBM, host memory and CPU per rank.

The reference is a read-only HTTP client with no GPU footprint at all
(``/root/reference/app.py:153-178``). rocmdash puts a process on every GPU of the node
(HIP context, RCCL communicator, device rings and resident sorted windows, pinned host
rings, sampler threads), so it measures and exports what that costs:

* **HBM** - the process's device memory as the amdgpu driver accounts it
  (``/sys/class/kfd/kfd/proc/<pid>/vram_<gpu>``: exact, per process, whatever allocated
  it - HIP runtime, RCCL, rocprofiler, torch); where that file is absent, the drop of the
  device's free memory since :meth:`Footprint.mark` was first called (``hipMemGetInfo``).
* **RSS** - ``/proc/self/statm`` resident pages.
* **CPU** - ``time.process_time()``: CPU seconds of every thread of the process (sampler
  threads, RCCL proxy, HTTP server).

Every rank samples its own numbers once per service refresh into the control row of
its gathered block (schema.CONTROL_FIELDS), so rank 0 exports all of them:
``rocmdash_self_hbm_bytes``, ``rocmdash_self_rss_bytes``,
``rocmdash_self_cpu_seconds_total`` per ``gpu_id``. ``stages`` keeps the HBM after
each start-up stage (agent, communicator, node-window buffers) for the bound test.
"""

from __future__ import annotations

import glob
import os
import time

from ..models.schema import CONTROL_INDEX, HEALTH_SPLIT

_PAGE = os.sysconf("SC_PAGE_SIZE") if hasattr(os, "sysconf") else 4096


def kfd_vram_bytes(pid: int | None = None) -> int | None:
    """Device memory of process ``pid`` summed over its GPUs (KFD sysfs), or None."""
    pid = os.getpid() if pid is None else pid
    files = glob.glob(f"/sys/class/kfd/kfd/proc/{pid}/vram_*")
    if not files:
        return None
    total = 0
    for f in files:
        try:
            with open(f) as fh:
                total += int(fh.read().strip() or 0)
        except (OSError, ValueError):
            continue
    return total


def rss_bytes() -> int:
    try:
        with open("/proc/self/statm") as f:
            return int(f.read().split()[1]) * _PAGE
    except (OSError, ValueError, IndexError):
        return 0


def device_used_bytes(device) -> int | None:
    """Used memory of the whole device (hipMemGetInfo: total - free), or None."""
    if device is None or getattr(device, "type", "cpu") != "cuda":
        return None
    try:
        import torch

        free, total = torch.cuda.mem_get_info(device)
        return int(total - free)
    except Exception:  # noqa: BLE001 - no device / runtime error: unknown
        return None


class Footprint:
    """This process's HBM / RSS / CPU, sampled on demand."""

    def __init__(self, device=None):
        self.device = device
        self.pid = os.getpid()
        self._base_used = None  # device-wide used bytes at the first mark() (fallback)
        self.stages = {}  # stage -> {"hbm": bytes, "device_used": bytes, "rss": bytes}

    def hbm_bytes(self) -> int | None:
        v = kfd_vram_bytes(self.pid)
        if v is not None:
            return v
        used = device_used_bytes(self.device)
        if used is None or self._base_used is None:
            return None
        return max(0, used - self._base_used)

    def mark(self, stage: str) -> dict:
        """Record the footprint after a start-up stage (the first call sets the
        baseline of the hipMemGetInfo fallback)."""
        used = device_used_bytes(self.device)
        if self._base_used is None:
            self._base_used = used
        rec = {"hbm": self.hbm_bytes(), "device_used": used, "rss": rss_bytes()}
        self.stages[stage] = rec
        return rec

    def sample(self) -> dict:
        return {"hbm_bytes": self.hbm_bytes(), "rss_bytes": rss_bytes(), "cpu_seconds": time.process_time()}

    def fill(self, ctl) -> None:
        """Write this rank's numbers into its control row (float32, exact halves)."""
        s = self.sample()
        nan = float("nan")
        ctl[CONTROL_INDEX["self_hbm_mb"]] = s["hbm_bytes"] / 2**20 if s["hbm_bytes"] is not None else nan
        ctl[CONTROL_INDEX["self_rss_mb"]] = s["rss_bytes"] / 2**20
        hi, lo = divmod(int(s["cpu_seconds"] * 1e3), int(HEALTH_SPLIT))
        ctl[CONTROL_INDEX["self_cpu_ms_hi"]] = hi
        ctl[CONTROL_INDEX["self_cpu_ms_lo"]] = lo


def decode_control(ctl) -> dict:
    """One gathered control row -> {"hbm_bytes", "rss_bytes", "cpu_seconds",
    "native_gather", "gather_validated"} (None where the rank sent NaN)."""
    import math

    def g(name):
        v = float(ctl[CONTROL_INDEX[name]])
        return None if math.isnan(v) else v

    hbm, rss, hi, lo = g("self_hbm_mb"), g("self_rss_mb"), g("self_cpu_ms_hi"), g("self_cpu_ms_lo")
    return {
        "hbm_bytes": None if hbm is None else hbm * 2**20,
        "rss_bytes": None if rss is None else rss * 2**20,
        "cpu_seconds": None if hi is None or lo is None else (hi * HEALTH_SPLIT + lo) * 1e-3,
        "native_gather": g("native_gather"),
        "gather_validated": g("gather_validated"),
    }
