"""The production node service, measured from outside (what a node pays for rocmdash).

Starts the DaemonSet's entrypoint - ``python -m rocmdash.launch --nproc N ... -m
rocmdash.serve`` (the node supervisor, one rank per GPU, the node counter process) - at
the production sampling rates (amd-smi 10 Hz, device counters 100 Hz, 1 Hz node
refresh), waits until every GPU is on /metrics with fresh counter rows, and reads the
supervisor's own accounting twice ``seconds`` apart:

* ``rocmdash_node_cpu_seconds_total{process}``: CPU-s/s of the supervisor, the counter
  process and the ranks - the node total VERDICT r04 item 3 asks for;
* ``rocmdash_sampler_samples_total{source="counter"}``: each GPU's counter rows per
  second (the 100 Hz counters still fresh on every GPU);
* ``rocmdash_node_process_memory_bytes``: every process's PSS / anonymous PSS / RSS
  (smaps_rollup) - what the pod's memory limit must hold;
* ``rocmdash_self_hbm_bytes``: each rank's own HBM.

Used by ``bench.py`` (its ``production_node`` field, after the measurement's ranks have
exited) and ``tools/node_cpu_probe.py``.

Reference anchor: the reference's sampling is an external exporter that costs the node
nothing it accounts for (``/root/reference/app.py:167-176``).
"""

from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
import urllib.error
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def get(url: str, timeout: float = 2.0):
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return r.status, r.read().decode()
    except urllib.error.HTTPError as e:
        return e.code, e.read().decode()
    except (urllib.error.URLError, ConnectionError, OSError):
        return None, ""


def start_node(n: int, port: int, *, serve_args=(), env=None, restart_base_s: float = 1.0, cpu: bool = True,
               log_path: str | None = None, counter_daemon: str = "auto"):
    """``python -m rocmdash.launch --nproc n ... -m rocmdash.serve`` in a session of its own."""
    cmd = [sys.executable, "-m", "rocmdash.launch", "--nproc", str(n), "--restart-base-s", str(restart_base_s),
           "--counter-daemon", counter_daemon,
           "--restart-max-s", "30", "--start-timeout", "120", f"--master-port={free_port()}",
           "-m", "rocmdash.serve", "--host", "127.0.0.1", "--port", str(port), *(("--cpu",) if cpu else ()),
           *serve_args]
    out = open(log_path, "w") if log_path else subprocess.DEVNULL
    try:
        return subprocess.Popen(cmd, cwd=ROOT, stdout=out, stderr=subprocess.STDOUT, start_new_session=True,
                                env=dict(os.environ, PYTHONPATH=ROOT, **(env or {})))
    finally:
        if log_path:
            out.close()  # the child holds its own descriptor


def stop_node(p, timeout: float = 60.0):
    if p.poll() is None:
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
    return p.returncode


def read_node(port: int) -> dict | None:
    """The accounting series of one /metrics body, or None while it is not served."""
    from ..prom.exposition import parse_text

    code, body = get(f"http://127.0.0.1:{port}/metrics", timeout=5.0)
    if code != 200:
        return None
    out = {"cpu": {}, "ctr": {}, "age": {}, "backend": {}, "gpus": set(), "rss": {}, "hbm": {}, "mem": {},
           "node_pss": None, "dev": {}, "dev_procs": {}}
    for s in parse_text(body):
        d = s.label_dict()
        if s.name == "rocmdash_node_cpu_seconds_total":
            out["cpu"][d["process"]] = s.value
        elif s.name == "rocmdash_sampler_samples_total" and d.get("source") == "counter":
            out["ctr"][d["gpu_id"]] = s.value
            out["backend"][d["gpu_id"]] = d.get("backend")
        elif s.name == "rocmdash_sample_age_seconds" and d.get("source") == "counter":
            out["age"][d["gpu_id"]] = s.value
        elif s.name == "amd_gpu_gfx_activity":
            out["gpus"].add(d["gpu_id"])
        elif s.name == "rocmdash_self_rss_bytes":
            out["rss"][d["gpu_id"]] = s.value
        elif s.name == "rocmdash_self_hbm_bytes":
            out["hbm"][d["gpu_id"]] = s.value
        elif s.name == "rocmdash_node_process_memory_bytes":
            key = d["process"] + (f":{d['gpu_id']}" if d.get("gpu_id") else "")
            out["mem"].setdefault(key, {})[d["kind"]] = s.value
        elif s.name == "rocmdash_node_pss_bytes":
            out["node_pss"] = s.value
        elif s.name == "rocmdash_node_process_device_memory_bytes":
            out["dev"].setdefault(d.get("bdf", ""), {})
            kind = d["process"]
            out["dev"][d.get("bdf", "")][kind] = out["dev"][d.get("bdf", "")].get(kind, 0.0) + s.value
            out["dev_procs"].setdefault(d.get("bdf", ""), set()).add((kind, d.get("gpu_id", "")))
    return out


def _descendants(pid: int) -> list:
    """Every process below ``pid`` (from /proc's parent links)."""
    kids = {}
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open(f"/proc/{d}/stat") as f:
                ppid = int(f.read().rsplit(")", 1)[1].split()[1])
        except (OSError, IndexError, ValueError):
            continue
        kids.setdefault(ppid, []).append(int(d))
    out, todo = [], [pid]
    while todo:
        p = todo.pop()
        for c in kids.get(p, []):
            out.append(c)
            todo.append(c)
    return out


def thread_cpu(pids) -> dict:
    """(pid, tid) -> (process name, thread name, CPU seconds) of every thread of ``pids``."""
    tck = os.sysconf("SC_CLK_TCK")
    out = {}
    for pid in pids:
        try:
            with open(f"/proc/{pid}/comm") as f:
                pname = f.read().strip()
            tids = os.listdir(f"/proc/{pid}/task")
        except OSError:
            continue
        for tid in tids:
            try:
                with open(f"/proc/{pid}/task/{tid}/stat") as f:
                    txt = f.read()
                name = txt[txt.index("(") + 1:txt.rindex(")")]
                parts = txt.rsplit(")", 1)[1].split()
                out[(pid, int(tid))] = (pname, name, (int(parts[11]) + int(parts[12])) / tck)
            except (OSError, ValueError, IndexError):
                continue
    return out


def busiest_threads(a: dict, b: dict, dt: float, top: int = 12) -> list:
    """The threads that used the most CPU between two thread_cpu() readings, by CPU-s/s,
    summed over threads of the same (process name, thread name)."""
    agg = {}
    for k, (pname, tname, c) in b.items():
        c0 = a.get(k, (pname, tname, c))[2]
        key = f"{pname}/{tname}"
        agg[key] = agg.get(key, 0.0) + max(0.0, c - c0) / dt
    return [[k, round(v, 4)] for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:top] if v > 0]


def _vram_used_by_gpu() -> dict:
    """Used VRAM of every GPU of the node plan (amdgpu sysfs, no HIP), by bdf hex."""
    from .footprint import sysfs_vram_used
    from .topology import node_plan

    plan = node_plan()
    if not plan:
        return {}
    return {"%x" % g["bdf"]: sysfs_vram_used(g["bdf"]) for g in plan["gpus"]}


def _settled_vram_used(timeout_s: float = 20.0, tol: int = 2 << 20) -> tuple:
    """Used VRAM of every GPU once it stopped moving (two reads 0.5 s apart within 2 MiB
    on every GPU): processes that just exited (the bench's own measurement children) free
    their device memory asynchronously, and a baseline read before that ends made round
    5's node growth NEGATIVE. Returns (reading, seconds waited)."""
    t0 = time.monotonic()
    a = _vram_used_by_gpu()
    while time.monotonic() - t0 < timeout_s:
        time.sleep(0.5)
        b = _vram_used_by_gpu()
        if all(a.get(k) is not None and b.get(k) is not None and abs(b[k] - a[k]) <= tol for k in b):
            return b, round(time.monotonic() - t0, 2)
        a = b
    return a, round(time.monotonic() - t0, 2)


def device_memory_report(vram0: dict, vram1: dict, dev: dict, dev_procs: dict) -> dict:
    """Per GPU (bdf hex): the device memory of the node's processes, by process kind, from
    per-process accounting (DRM fdinfo - never negative), the device's used-VRAM growth
    across the service's start (settled baseline) and the part of that growth no process's
    buffers explain: the driver's per-process and per-queue state (CWSR save areas,
    queue rings; profiles/r06/footprint/), shown per process that opened the GPU."""
    out = {}
    for g in sorted(set(vram1) | set(dev)):
        by_kind = {k: _mib(v) for k, v in sorted((dev.get(g) or {}).items())}
        attributed = sum((dev.get(g) or {}).values())
        growth = None
        if vram0.get(g) is not None and vram1.get(g) is not None:
            growth = vram1[g] - vram0[g]
        procs = len(dev_procs.get(g) or ())
        rec = {"process_buffers_mib": by_kind, "attributed_mib": _mib(attributed), "processes": procs}
        if growth is not None and growth >= attributed:
            rest = growth - attributed
            rec.update(device_used_growth_mib=_mib(growth), driver_state_mib=_mib(rest),
                       driver_state_mib_per_process=_mib(rest / procs) if procs else None)
        elif growth is not None:
            # another process freed memory during the measurement: no device-wide figure
            # (never a negative one); the per-process buffers above stand
            rec["note"] = (f"device usage grew {_mib(growth)} MiB, less than the processes' own buffers: "
                           "another process freed memory meanwhile")
        out[g] = rec
    return out


def _mib(v):
    return None if v is None else round(v / 2**20, 1)


def measure_production(nproc: int, *, seconds: float = 10.0, counter_daemon: str = "on", counters: str = "auto",
                       start_budget_s: float = 240.0, log_path: str | None = None, cpu: bool = False,
                       extra_serve_args=()) -> dict:
    """Run the production node service on ``nproc`` GPUs and measure it (module docstring).
    Never raises for a service that does not come up: the result's ``error`` says why."""
    port = free_port()
    serve_args = ("--refresh-hz", "1", "--node-window", "--collective-timeout", "30", "--counters", counters,
                  *extra_serve_args)
    vram0, settle_s = _settled_vram_used()  # before anything of the service starts (no HIP in this process)
    p = start_node(nproc, port, cpu=cpu, counter_daemon=counter_daemon, log_path=log_path, serve_args=serve_args,
                   env={"ROCMDASH_SMI_HZ": "10", "ROCMDASH_COUNTER_HZ": "100"}, restart_base_s=5.0)
    res = {"nproc": nproc, "counter_daemon": counter_daemon,
           "config": "rocmdash.launch (supervisor) -> rocmdash.serve --refresh-hz 1 --node-window; amd-smi 10 Hz, "
                     "counters 100 Hz", "error": None}
    t_start = time.monotonic()
    try:
        a = None
        while time.monotonic() < t_start + start_budget_s:
            if p.poll() is not None:
                res["error"] = f"the service exited with {p.returncode} before every GPU was up"
                return res
            a = read_node(port)
            if a and len(a["gpus"]) == nproc and len(a["ctr"]) == nproc and min(a["ctr"].values()) > 200:
                break
            time.sleep(1.0)
        else:
            res["error"] = f"not every GPU up with counter rows within {start_budget_s:.0f} s"
            return res
        res["startup_s"] = round(time.monotonic() - t_start, 1)
        time.sleep(6.0)  # one memory accounting period after every rank is up
        a = read_node(port)
        pids = _descendants(p.pid)
        th_a = thread_cpu(pids)
        ta = time.monotonic()
        time.sleep(seconds)
        b = read_node(port)
        dt = time.monotonic() - ta
        th_b = thread_cpu(pids)
        res["busiest_threads_cpu_seconds_per_s"] = busiest_threads(th_a, th_b, dt, top=64)
        # RCCL's proxy progress threads: busy only on the network transport (sockets - the
        # oversubscribed rehearsal, where every rank is its own "host"); on an xGMI node the
        # peers are P2P and the proxy has no network operations to progress
        proxy = sum(v for k, v in res["busiest_threads_cpu_seconds_per_s"] if "/NCCL Progress" in k)
        res["rccl_proxy_cpu_seconds_per_s"] = round(proxy, 4)
        res["busiest_threads_cpu_seconds_per_s"] = res["busiest_threads_cpu_seconds_per_s"][:12]
        # the single busiest threads, with their process (pid) and position in it (the n-th
        # thread started: ROCr / RCCL threads carry the interpreter's name)
        order = {}
        for pid, tid in sorted(th_b):
            order.setdefault(pid, []).append(tid)
        top = sorted(((max(0.0, c - th_a.get(k, (0, 0, c))[2]) / dt, k, n) for k, (_, n, c) in th_b.items()),
                     reverse=True)[:16]
        res["top_threads"] = [[round(r, 4), k[0], order[k[0]].index(k[1]), n] for r, k, n in top if r > 0.005]
        if a is None or b is None:
            res["error"] = "/metrics stopped answering during the measurement"
            return res
        rate = {k: round((b["cpu"][k] - a["cpu"].get(k, 0.0)) / dt, 4) for k in b["cpu"]}
        vram1 = _vram_used_by_gpu()
        # every process of the service together (ranks, counter process, supervisor) on
        # each GPU: the device's used VRAM growth across the service's start (a box that
        # runs nothing else; with oversubscribed ranks all of them land on the one GPU)
        res["baseline_settle_s"] = settle_s
        # per GPU and process kind, from per-process accounting
        res["device_memory_by_gpu"] = device_memory_report(vram0, vram1, b["dev"], b["dev_procs"])
        ranks = {k: v for k, v in b["mem"].items() if k.startswith("rank:")}
        res.update({
            "seconds": round(dt, 2),
            "node_cpu_seconds_per_s": rate,
            "node_cpu_seconds_per_s_total": round(sum(rate.values()), 4),
            "node_cpu_seconds_per_s_without_rccl_proxy": round(sum(rate.values()) - res["rccl_proxy_cpu_seconds_per_s"], 4),
            "counter_rows_per_s_by_gpu": {g: round((b["ctr"][g] - a["ctr"].get(g, 0.0)) / dt, 1) for g in sorted(b["ctr"])},
            "counter_age_s_by_gpu": b["age"],
            "counter_backend": sorted({v for v in b["backend"].values() if v}),
            # each rank's own start-up estimate (rocmdash.runtime.footprint: the device's
            # growth across its start, which with oversubscribed ranks also holds the other
            # ranks' concurrent starts); device_memory_by_gpu is the per-process accounting
            "rank_hbm_startup_delta_mib": {g: _mib(v) for g, v in sorted(b["hbm"].items())},
            "rank_rss_mib": {g: _mib(v) for g, v in sorted(b["rss"].items())},
            "process_pss_mib": {k: _mib(v.get("pss")) for k, v in sorted(b["mem"].items())},
            "process_pss_anon_mib": {k: _mib(v.get("pss_anon")) for k, v in sorted(b["mem"].items())},
            "rank_pss_mib_max": max((_mib(v.get("pss")) for v in ranks.values()), default=None),
            "node_pss_mib": _mib(b["node_pss"]),
        })
        return res
    finally:
        res["rc"] = stop_node(p)
