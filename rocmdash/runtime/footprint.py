"""The exporter's own cost on the node it watches: HBM, host memory and CPU per rank.

The reference is a read-only HTTP client with no GPU footprint at all
(``/root/reference/app.py:153-178``). rocmdash puts a process on every GPU of the node
(HIP context, RCCL communicator, device rings and resident sorted windows, pinned host
rings, sampler threads), so it measures and exports what that costs:

* **HBM** - the process's device memory as the amdgpu driver accounts it
  (``/sys/class/kfd/kfd/proc/<pid>/vram_<gpu>``: exact, per process, whatever allocated
  it - HIP runtime, RCCL, rocprofiler, torch) where the kernel exposes it; elsewhere (the
  pool's boxes) the growth of the device's used VRAM across rocmdash's OWN start-up
  stages - from before the HIP runtime starts (sysfs ``mem_info_vram_used``, no HIP
  needed) to the last stage: rocmdash allocates nothing after start-up (rings, resident
  windows, RCCL buffers are sized once), so that delta is its footprint, and later
  allocations of the node's workloads are not counted. (With oversubscribed ranks the
  delta also holds the other ranks' concurrent start-up.)
  The device-wide counter also moves with OTHER processes on the device (seen on a pool
  box: 280 -> 257 GB used while rocmdash started). The sysfs delta is trusted only when
  every stage's step is plausible next to HIP's own view (``hipMemGetInfo``, which misses
  driver-side allocations such as rocprofiler's); otherwise the footprint is the HIP-view
  growth from the HIP start on, plus the HIP context's sysfs step when that alone is
  plausible (``startup_delta``).
* **RSS** - ``/proc/self/statm`` resident pages.
* **CPU** - ``time.process_time()``: CPU seconds of every thread of the process (sampler
  threads, RCCL proxy, HTTP server), and the part of it used by ``SCHED_IDLE`` threads -
  the runtime's busy-polling thread rocmdash demotes (rocmdash.runtime.threads).

Every rank copies its own numbers into the control row of its gathered block once per
service refresh (schema.CONTROL_FIELDS), so rank 0 exports all of them. The numbers
themselves are sampled OFF the refresh path: :meth:`Footprint.start` runs a <= 1 Hz
background thread (the per-thread ``/proc/self/task/*/stat`` walk behind the CPU split,
the KFD glob, the RSS read), and :meth:`Footprint.fill` only copies its latest sample -
no ``/proc`` walk delays any rank's stats launch or ``ncclAllGather``. Series:
``rocmdash_self_hbm_bytes``, ``rocmdash_self_rss_bytes``,
``rocmdash_self_cpu_seconds_total`` per ``gpu_id``. ``stages`` keeps the HBM after
each start-up stage (agent, communicator, node-window buffers) for the bound test.
"""

from __future__ import annotations

import glob
import os
import threading
import time

from ..models.schema import CONTROL_INDEX, HEALTH_SPLIT

_PAGE = os.sysconf("SC_PAGE_SIZE") if hasattr(os, "sysconf") else 4096


def kfd_vram_bytes(pid: int | None = None, root: str = "/sys/class/kfd/kfd/proc") -> int | None:
    """Device memory of process ``pid`` summed over its GPUs (KFD sysfs), or None. A
    total of 0 counts as unavailable: some kernels list the per-process ``vram_*`` files
    but never fill them (seen on a pool box: 0 for a process holding a HIP context and
    its rings), and 0 is not a footprint any rocmdash rank can have."""
    pid = os.getpid() if pid is None else pid
    files = glob.glob(f"{root}/{pid}/vram_*")
    if not files:
        return None
    total = 0
    for f in files:
        try:
            with open(f) as fh:
                total += int(fh.read().strip() or 0)
        except (OSError, ValueError):
            continue
    return total or None


def pdev_bdf(pdev: str) -> int | None:
    """``"0000:75:00.0"`` (DRM fdinfo ``drm-pdev``, sysfs) -> amd-smi bdf id."""
    try:
        dom, bus, rest = pdev.strip().split(":")
        dev, fn = rest.split(".")
        return (int(dom, 16) << 32) | (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn, 16)
    except (ValueError, AttributeError):
        return None


def drm_vram_by_bdf(pid: int, root: str = "/proc") -> dict:
    """{bdf: bytes} of VRAM process ``pid``'s own buffer objects hold on each GPU, from
    its DRM clients' fdinfo (``drm-memory-vram``, one client per open render node, deduped
    by ``drm-client-id``). Exact and per process on every box - KFD's per-process sysfs
    reads 0 on the pool's - but it counts only the buffers the process allocated: the
    driver's per-process / per-queue state (~170 MiB per process per GPU plus ~177 MiB per
    hardware queue on MI355X, profiles/r06/footprint/) belongs to no DRM client. Empty
    when the process has no GPU open (or is gone)."""
    out: dict = {}
    seen = set()
    for f in glob.glob(f"{root}/{pid}/fdinfo/*"):
        try:
            with open(f) as fh:
                txt = fh.read()
        except OSError:
            continue
        if "drm-driver" not in txt:
            continue
        client = pdev = vram = None
        for line in txt.splitlines():
            k, _, v = line.partition(":")
            v = v.strip()
            if k == "drm-client-id":
                client = v
            elif k == "drm-pdev":
                pdev = v
            elif k == "drm-memory-vram":
                try:
                    num, _, unit = v.partition(" ")
                    vram = int(num) * {"KiB": 1024, "MiB": 1 << 20, "GiB": 1 << 30, "": 1}.get(unit.strip(), 1)
                except ValueError:
                    vram = None
        if vram is None or (client, pdev) in seen:
            continue
        seen.add((client, pdev))
        b = pdev_bdf(pdev) if pdev else None
        out[b] = out.get(b, 0) + vram
    return out


def rss_bytes() -> int:
    try:
        with open("/proc/self/statm") as f:
            return int(f.read().split()[1]) * _PAGE
    except (OSError, ValueError, IndexError):
        return 0


def sysfs_vram_used(bdf: int | None) -> int | None:
    """Used VRAM of the whole device from amdgpu's sysfs (no HIP call), or None."""
    if not bdf:
        return None
    from .agent import bdf_path

    try:
        with open(bdf_path(bdf) + "/mem_info_vram_used") as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return None


def device_used_bytes(device, bdf: int | None = None) -> int | None:
    """Used memory of the whole device: amdgpu sysfs when the bdf is known (works before
    HIP starts), else hipMemGetInfo (total - free); None when neither is available."""
    v = sysfs_vram_used(bdf)
    if v is not None:
        return v
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

    _AGREE = 64 << 20  # sysfs vs HIP view of rocmdash's own growth
    _CTX_MAX = 2 << 30  # a plausible HIP context (+ rocprofiler) step

    def __init__(self, device=None, bdf: int | None = None):
        self.device = device
        self.bdf = bdf
        self.pid = os.getpid()
        self._marks = []  # (stage, device-wide used bytes from sysfs, used bytes in HIP's view)
        self.stages = {}  # stage -> {"hbm": bytes, "device_used": bytes, "rss": bytes}
        self.method = "kfd" if kfd_vram_bytes(self.pid) is not None else "start-up delta"
        self._latest = None  # the background thread's newest sample()
        self._lock = threading.Lock()
        self._stop = None
        self._thread = None
        self.samples_taken = 0  # sample() calls (tests: none on the refresh path)

    def hbm_bytes(self) -> int | None:
        v = kfd_vram_bytes(self.pid)
        if v is not None:
            return v
        return startup_delta(self._marks, self._AGREE, self._CTX_MAX)

    def mark(self, stage: str) -> dict:
        """Record the footprint after a start-up stage. The first call (before the HIP
        runtime starts, when a bdf is known) sets the baseline."""
        used = sysfs_vram_used(self.bdf)
        hip = device_used_bytes(self.device, None)  # HIP's view (None before HIP / on CPU)
        self._marks.append((stage, used, hip))
        rec = {"hbm": self.hbm_bytes(), "device_used": used if used is not None else hip, "rss": rss_bytes()}
        self.stages[stage] = rec
        return rec

    def sample(self) -> dict:
        from .threads import cpu_by_class

        self.samples_taken += 1
        return {"hbm_bytes": self.hbm_bytes(), "rss_bytes": rss_bytes(), "cpu_seconds": time.process_time(),
                "cpu_idle_seconds": cpu_by_class()["idle"]}

    def start(self, period_s: float = 1.0) -> None:
        """Sample every ``period_s`` seconds on a daemon thread (``rd-footprint``); from
        now on :meth:`fill` copies the newest sample instead of taking one."""
        if self._thread is not None:
            return
        self._refresh_latest()
        self._stop = threading.Event()

        def loop():
            while not self._stop.wait(period_s):
                self._refresh_latest()

        self._thread = threading.Thread(target=loop, name="rd-footprint", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        if self._thread is not None:
            self._stop.set()
            self._thread.join(timeout=5.0)
            self._thread = None

    def _refresh_latest(self) -> None:
        s = self.sample()
        with self._lock:
            self._latest = s

    def latest(self) -> dict:
        """The background thread's newest sample (one taken now when none runs)."""
        with self._lock:
            s = self._latest
        return s if s is not None and self._thread is not None else self.sample()

    def fill(self, ctl) -> None:
        """Write this rank's numbers into its control row (float32, exact halves): the
        background sample when :meth:`start` runs (a copy, no I/O), else one taken now."""
        s = self.latest()
        nan = float("nan")
        ctl[CONTROL_INDEX["self_hbm_mb"]] = s["hbm_bytes"] / 2**20 if s["hbm_bytes"] is not None else nan
        ctl[CONTROL_INDEX["self_rss_mb"]] = s["rss_bytes"] / 2**20
        for key, sec in (("self_cpu_ms", s["cpu_seconds"]), ("self_cpu_idle_ms", s["cpu_idle_seconds"])):
            hi, lo = divmod(int(sec * 1e3), int(HEALTH_SPLIT))
            ctl[CONTROL_INDEX[key + "_hi"]] = hi
            ctl[CONTROL_INDEX[key + "_lo"]] = lo


def startup_delta(marks, agree: int = 64 << 20, ctx_max: int = 2 << 30, extra: int = 512 << 20) -> int | None:
    """rocmdash's HBM from its start-up marks [(stage, sysfs used, HIP-view used)] (see
    the module docstring). The device-wide sysfs growth is trusted when every stage's
    step is plausible: the step that starts HIP in (0, ``ctx_max``), and every later step
    at least HIP's own step (- ``agree``) and at most HIP's step + ``extra`` (allocations
    HIP does not see: rocprofiler's counting context and code objects took ~170 MiB that
    ``hipMemGetInfo`` never showed). Otherwise - another process allocated or freed
    memory on the device meanwhile - HIP's growth plus the context step when that alone
    is plausible, else None."""
    sysv = [u for _, u, _ in marks if u is not None]
    hip = [(u, h) for _, u, h in marks if h is not None]
    hip_growth = hip[-1][1] - hip[0][1] if len(hip) >= 2 and hip[-1][1] >= hip[0][1] else None
    before = [u for _, u, h in marks if h is None and u is not None]  # sysfs before HIP started
    ctx = hip[0][0] - before[-1] if before and hip and hip[0][0] is not None else None
    ok = len(sysv) >= 2 and sysv[-1] > sysv[0]
    if ok and ctx is not None:
        ok = 0 < ctx < ctx_max
    if ok and all(u is not None for u, _ in hip):
        for (u0, h0), (u1, h1) in zip(hip, hip[1:]):
            if not (h1 - h0 - agree <= u1 - u0 <= h1 - h0 + extra):
                ok = False
                break
    if ok:
        return sysv[-1] - sysv[0]
    if hip_growth is None:
        return None
    return (ctx if ctx is not None and 0 < ctx < ctx_max else 0) + hip_growth


def decode_control(ctl) -> dict:
    """One gathered control row -> {"hbm_bytes", "rss_bytes", "cpu_seconds",
    "cpu_idle_seconds", "native_gather", "gather_validated"} (None where the rank sent
    NaN)."""
    import math

    def g(name):
        v = float(ctl[CONTROL_INDEX[name]])
        return None if math.isnan(v) else v

    def ms_pair(key):
        hi, lo = g(key + "_hi"), g(key + "_lo")
        return None if hi is None or lo is None else (hi * HEALTH_SPLIT + lo) * 1e-3

    hbm, rss, val = g("self_hbm_mb"), g("self_rss_mb"), g("gather_validated")
    return {
        "hbm_bytes": None if hbm is None else hbm * 2**20,
        "rss_bytes": None if rss is None else rss * 2**20,
        "cpu_seconds": ms_pair("self_cpu_ms"),
        "cpu_idle_seconds": ms_pair("self_cpu_idle_ms"),
        "native_gather": None if val is None else float(val >= 0),
        "gather_validated": None if val is None else max(val, 0.0),
    }
