"""The runtime's busy-polling thread, and what rocmdash does about it.

Measured on the MI355X box (tools/probes/probe_cpu_spin.py, profiles/r03/footprint/):
once the rocprofiler-sdk device-counting context is started, one thread that the HSA
runtime created at start-up - not one of rocmdash's (those are named ``rd-*``) - runs
at 1.0 CPU-second per second, at any counter rate (10 or 100 Hz), idle or sampling. The
SDK registers an asynchronous completion handler on its counting signal
(``hsa_amd_signal_async_handler`` in librocprofiler-sdk); ROCr's async-events thread
then busy-polls. With counters off the process uses 0.004 CPU-s/s.

That polling is also what makes a counter read fast: the read's completion reaches the
SDK through that thread. Demoted to ``SCHED_IDLE`` on the box, the reads took 130-155 us
instead of 80 us (and the bench's fresh rate halved: 34-38k vs 52-66k samples/s,
alternating A/B, profiles/r03/demote_ab/). Hence:

* the node service (``rocmdash.serve``, counters at 100 Hz: reads 10 ms apart, the read
  time irrelevant) demotes that one thread: it keeps polling on CPUs that are otherwise
  idle and yields to every other runnable thread on the node - the GPU workloads the
  dashboard watches first. Measured at the production rates: 0.023 CPU-s/s at normal
  priority (rocmdash's threads and the rest of the runtime), 0.99 CPU-s/s of idle-class
  polling (profiles/r03/demote_ab/footprint_w1.json);
* ``bench.py`` (closed loop at the read floor) leaves it alone (``--demote-spin 1`` to
  A/B it).

The service exports its CPU use split by scheduling class
(``rocmdash_self_cpu_seconds_total{class="normal"|"idle"}``), so the cost taken from
workloads and the idle-time polling are reported apart. ``ROCMDASH_DEMOTE_SPIN=0``
leaves the thread alone.
"""

from __future__ import annotations

import os
import time

_TCK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100
_demoted: set = set()


def thread_cpu(pid: int | None = None) -> dict:
    """{tid: (name, cpu_seconds, policy)} of every thread of ``pid`` (default: self)."""
    pid = os.getpid() if pid is None else pid
    out = {}
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for t in tids:
        try:
            with open(f"/proc/{pid}/task/{t}/stat") as f:
                st = f.read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        fields = st[st.rindex(")") + 2:].split()
        # fields[38] = policy (stat field 41); utime / stime = fields 11 / 12
        out[int(t)] = (name, (int(fields[11]) + int(fields[12])) / _TCK, int(fields[38]) if len(fields) > 38 else 0)
    return out


def busy_foreign_threads(window_s: float = 0.25, threshold: float = 0.5) -> list:
    """Threads of this process that used more than ``threshold`` CPU-s/s over
    ``window_s`` and are neither the main thread nor rocmdash's own (``rd-*``)."""
    me = os.getpid()
    a = thread_cpu()
    time.sleep(window_s)
    b = thread_cpu()
    out = []
    for tid, (name, cpu, _) in b.items():
        if tid == me or name.startswith("rd-"):
            continue
        rate = (cpu - a.get(tid, (name, cpu, 0))[1]) / window_s
        if rate > threshold:
            out.append((tid, name, rate))
    return out


def demote_runtime_spinners(window_s: float = 0.25) -> list:
    """Put the runtime's busy-polling thread(s) on SCHED_IDLE. Returns the demoted
    [(tid, name, cpu_per_s)] (empty when none, on non-Linux, or when disabled)."""
    if os.environ.get("ROCMDASH_DEMOTE_SPIN", "1") in ("0", "off", "false") or not hasattr(os, "SCHED_IDLE"):
        return []
    done = []
    for tid, name, rate in busy_foreign_threads(window_s):
        try:
            os.sched_setscheduler(tid, os.SCHED_IDLE, os.sched_param(0))
        except OSError:
            continue
        _demoted.add(tid)
        done.append((tid, name, round(rate, 3)))
    return done


def cpu_by_class() -> dict:
    """{"normal": s, "idle": s}: CPU seconds of this process's threads by scheduling
    class (SCHED_IDLE threads vs everything else)."""
    out = {"normal": 0.0, "idle": 0.0}
    idle = getattr(os, "SCHED_IDLE", 5)
    for tid, (_, cpu, policy) in thread_cpu().items():
        out["idle" if (policy == idle or tid in _demoted) else "normal"] += cpu
    return out
