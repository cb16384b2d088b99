"""Where the process initialises the HSA runtime: the NUMA node that makes the
device-counter read fast.

The rocprofiler-sdk device-counter read costs ~70 us or ~140 us depending on the
NUMA node of the CPUs the process ran on when it brought the HSA runtime up, and the
cost then holds for the life of the process. It does not depend on the core that
later issues the reads, on the counting context, or on ROCr's signal wait mode. On
the test box, starting on the GPU's *own* node (sysfs ``numa_node``) was the slow case,
every time. The evidence is in profiles/r01/:

- ``numa_ab.txt``: probe_counter_ctx pinned with taskset, 5 runs per node.
- ``numa_bench.txt``: bench.py, 75-84k versus 179-190k samples/s.
- ``probe_counter_ctx.txt`` and ``interrupt_ab.txt``.

The rule is not written down anywhere, so it is measured instead:

1. Before the runtime starts, this module runs a small probe once per NUMA node FOR
   THE WHOLE NODE: each probe is a short child process pinned to that NUMA node; it
   starts HIP, configures the same counters on every GPU, and times 200 reads of each.
2. The parent thread is pinned to the fastest NUMA node for its GPU before HSA starts.
   The runtime's threads inherit that. The sampler threads later pin themselves as
   configured.
3. The results of every GPU are cached by bdf, per boot, in one file in ``$TMPDIR``: the
   first of 8 ranks starting together calibrates the node with 2 children (2 sockets),
   the 7 others and every later start (bench N = 1, 2, 4, 8; restarts) read the cache.
   Round 2 probed each GPU on its own: 16 children in series, ~35 s before the last
   rank of a node could start.
4. Probes are serialised node-wide by an ``fcntl`` lock next to the cache: the read
   cost is sensitive to contention (profiles/r01/probe_overlap.txt), so concurrent
   probes would measure each other. A rank re-reads the cache once it holds the lock.
5. Once the runtime is up (``restore_affinity()``, called by ``GpuAgent``) the thread
   gets its original CPU mask back: the state is fixed at HSA start, and threads the
   process creates later (RCCL proxies, torch pools, HTTP servers) must not inherit
   the init pin.

``ROCMDASH_INIT_PLACEMENT=0`` turns this off, and ``=<node>`` forces a node.
"""

from __future__ import annotations

import fcntl
import json
import os
import subprocess
import sys
import tempfile
import time
from contextlib import contextmanager

_original_mask: set | None = None  # the thread's CPUs before pin_for_init()
_choice: dict | None = None


def process_cpus() -> set:
    """The CPUs this process may use: the mask from before ``pin_for_init()``."""
    return set(_original_mask) if _original_mask is not None else set(os.sched_getaffinity(0))


def choice() -> dict | None:
    """What ``pin_for_init()`` decided (for reports): node, calibration, source."""
    return _choice


def _cpulist(text: str) -> list:
    out = []
    for part in text.strip().split(","):
        if part:
            lo, _, hi = part.partition("-")
            out.extend(range(int(lo), int(hi or lo) + 1))
    return out


def numa_nodes() -> dict:
    """{node: [cpus this process may use]} over the NUMA nodes that have any."""
    allowed = process_cpus()
    root = "/sys/devices/system/node"
    nodes = {}
    try:
        names = sorted(n for n in os.listdir(root) if n.startswith("node") and n[4:].isdigit())
    except OSError:
        return {}
    for n in names:
        try:
            with open(os.path.join(root, n, "cpulist")) as f:
                cpus = [c for c in _cpulist(f.read()) if c in allowed]
        except (OSError, ValueError):
            continue
        if cpus:
            nodes[int(n[4:])] = cpus
    return nodes


def _boot_id() -> str:
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            return f.read().strip()[:8]
    except OSError:
        return "noboot"


def _cache_path() -> str:
    """The node's calibration (every GPU, by bdf), per boot and user."""
    return os.path.join(tempfile.gettempdir(), f"rocmdash-placement-node-{_boot_id()}-u{os.getuid()}.json")


def _lock_path() -> str:
    return os.path.join(tempfile.gettempdir(), f"rocmdash-placement-{_boot_id()}-u{os.getuid()}.lock")


@contextmanager
def node_lock(timeout_s: float = 600.0, path: str | None = None):
    """Exclusive node-wide lock (``fcntl.flock``) held while probing. Yields True when
    held; after ``timeout_s`` without it, yields False and the caller goes on (a
    stuck holder must not keep a rank from starting at all)."""
    path = path or _lock_path()
    fd = None
    held = False
    try:
        fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
        deadline = time.monotonic() + timeout_s
        while True:
            try:
                fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
                held = True
                break
            except BlockingIOError:
                if time.monotonic() >= deadline:
                    break
                time.sleep(0.05)
    except OSError:
        pass
    try:
        yield held
    finally:
        if fd is not None:
            if held:
                fcntl.flock(fd, fcntl.LOCK_UN)
            os.close(fd)


# Whether a probe round decided anything is judged RELATIVELY - no absolute microseconds,
# which were tied to one counter set (the 7-counter set read ~105 us
# on the fast node and every calibration looked "slow"). The NUMA effect makes one node's
# reads 1.7-1.9x the other's on every box seen, whatever the counter set (profiles/r01,
# BENCH_r01..r05, profiles/r06/counter_ab/*placement.json: 73/137, 84/152, 79/145,
# 81/150, 113/195, 106/201 us). Right after a box comes up BOTH nodes can read alike and
# slow for some seconds (profiles/r02/head/bench_reps_s4.txt), and a decision taken then -
# and cached for the boot - would be a coin flip. So a round is conclusive when, for
# every GPU, the slowest node reads at least NUMA_RATIO x the fastest; an inconclusive
# round is probed again after a pause. If no round is conclusive but the rounds agree
# with one another (within STABLE_TOL), the box simply has no NUMA effect: cached like a
# decision ("uniform"). Rounds that neither separate the nodes nor agree are a transient
# phase: kept only briefly ("slow", re-probed after SLOW_CACHE_S).
NUMA_RATIO = float(os.environ.get("ROCMDASH_PLACEMENT_NUMA_RATIO", "1.35"))
STABLE_TOL = 0.15
PROBE_ROUNDS = 3
RETRY_PAUSE_S = 1.0
SLOW_CACHE_S = 60.0  # an inconclusive (all-slow) calibration is re-probed after this
PROBE_TIMEOUT_S = 90.0  # one probe child (HIP start + counters on every GPU + reads)


def _read_cache(path: str, nodes: dict, bdf: int) -> dict | None:
    """This GPU's entry of the node-wide calibration, or None (absent, taken on another
    set of NUMA nodes, or an all-slow calibration older than SLOW_CACHE_S)."""
    try:
        with open(path) as f:
            cached = json.load(f)
    except (OSError, ValueError):
        return None
    if set(map(int, cached.get("nodes", []))) != set(nodes):
        return None
    if cached.get("slow") and time.time() - float(cached.get("t", 0.0)) > SLOW_CACHE_S:
        return None
    entry = cached.get("gpus", {}).get(f"{bdf:x}")
    if entry is None:
        return None
    out = dict(entry)
    out.update(source="cache", gpus_calibrated=len(cached.get("gpus", {})),
               calibration_s=cached.get("calibration_s"))
    return out


def _probe_node(cpus: list, timeout_s: float = PROBE_TIMEOUT_S) -> dict | None:
    """{bdf hex: p50 µs} of a device-counter read of EVERY GPU, from one child process
    started on these CPUs (None if the child failed)."""
    cmd = [sys.executable, "-m", "rocmdash.runtime.placement", "--probe-all", ",".join(map(str, cpus))]
    env = dict(os.environ, ROCMDASH_INIT_PLACEMENT="0")
    # the child configures counters on EVERY GPU of the node: not only this rank's (a
    # launcher that gives each rank its own visibility would otherwise leave each probe
    # seeing one GPU, and the node-wide cache would hold one entry per start)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
              "ROCR_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"):
        env.pop(k, None)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    try:
        res = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s, env=env)
    except (subprocess.TimeoutExpired, OSError):
        return None
    for line in res.stdout.splitlines():
        if line.startswith("{"):
            try:
                got = json.loads(line)["p50_us"]
                return {str(k): float(v) for k, v in got.items() if v is not None}
            except (ValueError, KeyError, TypeError, AttributeError):
                return None
    return None


def calibrate(device: int, bdf: int, use_cache: bool = True) -> dict:
    """{"node": n | None, "p50_us": {node: µs}, "source": "probe" | "cache" | ...} for
    the GPU ``bdf``. ONE calibration serves the whole node: the first rank to take the
    node-wide lock starts one probe child per NUMA node, each timing EVERY GPU's counter
    read, and caches all GPUs' results by bdf for the boot - 2 probe children for an
    8-GPU, 2-socket node instead of 16, so 8 ranks starting together wait for one
    calibration (~2 child start-ups), not eight in series. The other ranks (and every
    later start) read the cache."""
    path = _cache_path()
    nodes = numa_nodes()
    if use_cache:
        cached = _read_cache(path, nodes, bdf)
        if cached is not None:
            return cached
    if len(nodes) < 2:
        return {"node": None, "p50_us": {}, "source": "single node"}
    t_wait = time.perf_counter()
    with node_lock() as held:
        waited = time.perf_counter() - t_wait
        if use_cache:  # another rank may have calibrated the node while we waited
            cached = _read_cache(path, nodes, bdf)
            if cached is not None:
                cached["lock_wait_s"] = round(waited, 2)
                return cached
        table = _probe_all(nodes, path)
        entry = dict(table["gpus"].get(f"{bdf:x}") or {"node": None, "p50_us": {}})
        entry.update(source="probe", calibration_s=table["calibration_s"], gpus_calibrated=len(table["gpus"]),
                     lock_wait_s=round(waited, 2), lock_held=held)
        if table.get("slow_rounds"):
            entry["slow_rounds"] = table["slow_rounds"]
        return entry


def fast_reference_us(dec: dict | None) -> float | None:
    """The counter read this process should see: its GPU's calibrated read on the chosen
    node - measured with the SAME counter set the service configures (the probe child
    uses the defaults), so thresholds derived from it follow the set. None when there is
    no calibration (one NUMA node, placement off)."""
    if not dec or dec.get("node") is None:
        return None
    v = (dec.get("p50_us") or {}).get(str(dec.get("node")))
    return float(v) if v else None


def _conclusive(per_node: dict) -> bool:
    """Every GPU of the round separates the nodes by NUMA_RATIO (one node: nothing to
    separate, conclusive)."""
    bdfs = sorted({b for r in per_node.values() if r for b in r})
    if not bdfs:
        return True
    for b in bdfs:
        vals = [r[b] for r in per_node.values() if r and r.get(b)]
        if len(vals) >= 2 and max(vals) < NUMA_RATIO * min(vals):
            return False
    return True


def _stable(rounds: list) -> bool:
    """The inconclusive rounds agree with one another: every (node, GPU) read within
    STABLE_TOL of its mean over the rounds."""
    if len(rounds) < 2:
        return False
    keys = {(n, b) for r in rounds for n, v in r.items() if v for b in v}
    for n, b in keys:
        vals = [(r.get(n) or {}).get(b) for r in rounds]
        if any(v is None for v in vals):
            return False
        m = sum(vals) / len(vals)
        if any(abs(v - m) > STABLE_TOL * m for v in vals):
            return False
    return True


def _probe_all(nodes: dict, path: str) -> dict:
    """Probe every GPU from every NUMA node (one child per node per round, up to
    PROBE_ROUNDS rounds while a round does not separate the nodes); cache and return
    {"nodes", "gpus": {bdf hex: {"node", "p50_us": {node: µs}, "slow"?}}, ...}."""
    t0 = time.perf_counter()
    slow_rounds = []
    per_node = {}
    conclusive = False
    for rnd in range(PROBE_ROUNDS):
        per_node = {n: _probe_node(cpus) for n, cpus in nodes.items()}
        if not any(per_node.values()) or _conclusive(per_node):
            conclusive = True
            break
        slow_rounds.append({str(n): r for n, r in per_node.items()})  # nodes alike: again
        if rnd + 1 < PROBE_ROUNDS:
            time.sleep(RETRY_PAUSE_S)
    uniform = not conclusive and _stable(slow_rounds)
    gpus = {}
    for b in sorted({b for r in per_node.values() if r for b in r}):
        p50 = {str(n): (r or {}).get(b) for n, r in per_node.items()}
        good = {n: v for n, v in p50.items() if v is not None}
        node = int(min(good, key=good.get)) if good else None
        e = {"node": node, "p50_us": p50}
        if not conclusive:
            e["uniform" if uniform else "slow"] = True
        gpus[b] = e
    out = {"nodes": sorted(nodes), "gpus": gpus, "calibration_s": round(time.perf_counter() - t0, 2), "t": time.time(),
           "probe_children": len(nodes) * (len(slow_rounds) + (0 if len(slow_rounds) == PROBE_ROUNDS else 1)),
           "numa_ratio": NUMA_RATIO}
    if slow_rounds:
        out["slow_rounds"] = slow_rounds
    if any(e.get("slow") for e in gpus.values()):
        out["slow"] = True  # a transient phase, no decision: cached for SLOW_CACHE_S only
    if gpus:
        # merge: entries of GPUs this probe did not see (a device the child could not
        # open) stay in the node-wide cache instead of being erased
        try:
            with open(path) as f:
                prev = json.load(f)
            if set(map(int, prev.get("nodes", []))) == set(nodes):
                for b, e in prev.get("gpus", {}).items():
                    out["gpus"].setdefault(b, e)
        except (OSError, ValueError, AttributeError, TypeError):
            pass
        try:
            tmp = path + f".{os.getpid()}"
            with open(tmp, "w") as f:
                json.dump(out, f)
            os.replace(tmp, path)
        except OSError:
            pass
    return out


def _runtime_started() -> bool:
    """True once this process has opened the KFD device (the HSA runtime is up): too
    late to choose where it starts, and no probe children are spawned then."""
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                if os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd":
                    return True
            except OSError:
                continue
    except OSError:
        pass
    return False


def restore_affinity() -> bool:
    """Give the calling thread back the CPU mask it had before ``pin_for_init()``
    (call once the HSA runtime is up). True if a pin was undone.
    ``ROCMDASH_RESTORE_AFFINITY=0`` keeps the pin."""
    if _original_mask is None or os.environ.get("ROCMDASH_RESTORE_AFFINITY", "1") in ("0", "off", "false"):
        return False
    try:
        if set(os.sched_getaffinity(0)) != _original_mask:
            os.sched_setaffinity(0, _original_mask)
            return True
    except OSError:
        pass
    return False


def pin_for_init(device: int, bdf: int) -> dict | None:
    """Pin the calling thread to the fastest node for this GPU's counter reads, before
    HSA starts. Threads the runtime creates afterwards inherit the mask. Returns the
    decision, or None when there is nothing to decide."""
    global _original_mask, _choice
    mode = os.environ.get("ROCMDASH_INIT_PLACEMENT", "auto").strip().lower()
    if mode in ("0", "off", "false", "no") or not bdf or _runtime_started():
        return None
    if _original_mask is None:
        _original_mask = set(os.sched_getaffinity(0))
    nodes = numa_nodes()
    if mode.isdigit():
        dec = {"node": int(mode), "p50_us": {}, "source": "ROCMDASH_INIT_PLACEMENT"}
    else:
        dec = calibrate(device, bdf)
    node = dec.get("node")
    if node is None or node not in nodes:
        _choice = dec
        return dec
    os.sched_setaffinity(0, nodes[node])
    _choice = dec
    return dec


def _probe_main(cpus: list) -> None:
    """Probe child: started on ``cpus``, bring HIP up with device counting on EVERY GPU
    and time 200 counter reads of each (after 30 warm-up reads)."""
    os.sched_setaffinity(0, cpus)
    import ctypes

    from . import native

    nat = native.load()
    ok, status = native.enable_counters()
    if not ok:
        print(json.dumps({"error": status}))
        return
    hip = ctypes.CDLL("libamdhip64.so")
    if hip.hipInit(0) != 0:
        print(json.dumps({"error": "hipInit failed"}))
        return
    out = {}
    for dev in range(int(nat.hip_device_count())):
        bdf = int(nat.hip_device_bdf(dev))
        try:
            src = nat.make_counter_source(bdf, dev)
            for _ in range(30):
                src.sample()
            ts = []
            for _ in range(200):
                t0 = time.perf_counter()
                src.sample()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            out[f"{bdf:x}"] = round(ts[len(ts) // 2] * 1e6, 1)
        except RuntimeError:
            out[f"{bdf:x}"] = None
    print(json.dumps({"p50_us": out, "cpus": len(cpus)}))


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--probe-all":
        _probe_main([int(c) for c in sys.argv[2].split(",")])
    else:
        print(json.dumps(calibrate(int(sys.argv[1]) if len(sys.argv) > 1 else 0,
                                   int(sys.argv[2]) if len(sys.argv) > 2 else 0, use_cache=False)))
