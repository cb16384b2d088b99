"""Node supervisor: one rank process per physical GPU, re-formed around the GPUs that work.

The DaemonSet's entrypoint (``python -m rocmdash.launch ... -m rocmdash.serve ...``).
It never touches a GPU. It

  * starts one rank process per GPU *slot* (the KFD node plan: one per physical GPU),
    each in a session of its own, and hosts the store the ranks rendezvous on;
  * decides **epochs** - numbered member lists of slots - and publishes them on that
    store (``rocmdash.parallel.membership``). The members of an epoch run the node
    refresh together: a gloo control plane of their own and a fresh native RCCL
    communicator (``ncclCommInitRank`` with a new unique id) over xGMI;
  * when a member is lost - its process exits, or it stops answering so that the other
    members' collectives fail and they report it (``decide_culprits``) - forms the next
    epoch from the members that are left. They keep their agents (sources, rings, the
    resident W-sample windows): only the process group and the communicator are new;
  * restarts a lost slot in a FRESH process after an exponential backoff (``--restart-
    base-s`` doubling to ``--restart-max-s``). The new process builds its GPU agent first
    (the probe: HIP device, SMU table, counters) and is re-admitted by the next epoch only
    once it announced itself ready;
  * serves ``/metrics`` and ``/healthz`` itself: each epoch's root pushes its refresh's
    snapshot here (``SnapshotPusher``), so the endpoint outlives any rank. ``/metrics`` adds
    ``rocmdash_gpu_up{gpu_id}`` (0 for a GPU outside the epoch) with the reason it is down,
    its restarts and the node epoch; ``/healthz`` answers from refresh-loop progress only
    (a stale GPU source is a metric, ``rocmdash_source_stale``, never a restart).

A GPU that keeps failing therefore costs the node one regroup per restart attempt
(seconds, or one collective timeout if it hangs), backed off to one attempt per
``--restart-max-s``, while the other GPUs stay on the dashboard.

Reference anchor: the reference shows whatever GPUs the exporter reports and drops the
rest (``/root/reference/app.py:183-201, 262-313, 335``).
"""

from __future__ import annotations

import json
import logging
import os
import secrets
import signal
import subprocess
import sys
import tempfile
import threading
import time
from dataclasses import dataclass, field

from ..parallel.membership import (
    ENV_ADDR,
    ENV_INCARNATION,
    ENV_PUSH,
    ENV_PUSH_KEY,
    ENV_SLOT,
    ENV_SLOTS,
    format_members,
)

log = logging.getLogger("rocmdash.supervisor")


# The node's collectives are small (a ~1 KB stats all-gather per rank, <= 150 KB
# node-window records, <= 96 KB histogram all-reduces): RCCL's default 4 MiB buffers on
# every channel of every peer connection held ~1 GB per rank at 8 ranks
# (profiles/r05/nodecpu/), two 1 MiB channels carry them
# (NCCL_SET_THREAD_NAME: RCCL's threads carry their role - "NCCL Progress" is the proxy
# thread the node measurement accounts separately)
LEAN_RUNTIME_ENV = {"GPU_MAX_HW_QUEUES": "1", "HSA_SCRATCH_SINGLE_LIMIT": "1048576", "NCCL_BUFFSIZE": "1048576",
                    "NCCL_MAX_NCHANNELS": "2", "NCCL_SET_THREAD_NAME": "1"}


def decide_culprits(members, reported, dead=()) -> list:
    """Who left epoch ``members``: every member whose process is ``dead``, and - once some
    member reported a failed collective - every live member that did NOT report (it
    stopped answering: its peers' collectives timed out waiting for it, it never saw a
    failure of its own). With every live member reporting, nobody is excluded (a
    transient failure: the same members re-form)."""
    dead = set(dead)
    reported = set(reported)
    out = [m for m in members if m in dead]
    if reported:
        out += [m for m in members if m not in dead and m not in reported]
    return sorted(set(out))


def restart_delay(failures: int, base_s: float, max_s: float) -> float:
    """Backoff before starting a slot again after its ``failures``-th consecutive
    failure: base, 2 base, 4 base, ... capped at max."""
    if failures <= 0:
        return 0.0
    return float(min(max_s, base_s * (2 ** min(failures - 1, 30))))


@dataclass
class Slot:
    index: int
    device: int | None = None
    proc: subprocess.Popen | None = None
    incarnation: int = -1
    state: str = "down"  # starting | ready | member | down | stopped (left on a stop vote)
    info: dict | None = None  # the rank's announcement (AgentInfo + slot)
    failures: int = 0  # consecutive (reset after healthy_reset_s as a member)
    restarts: int = 0
    last_error: str = ""
    next_start: float = 0.0
    t_start: float = 0.0
    t_member: float | None = None
    history: list = field(default_factory=list)  # (monotonic time, event)

    @property
    def own_id(self) -> str | None:
        """The gpu_id the slot's rank announced (amd-smi's index), if any."""
        if self.info and self.info.get("gpu_id") not in (None, "", "-1"):
            return str(self.info["gpu_id"])
        return None


class SupervisedSource:
    """The exporter's source in the supervisor: the newest snapshot an epoch root pushed,
    plus the node's membership as metrics. ``health()`` is refresh-loop progress."""

    def __init__(self, sup: "NodeSupervisor", stall_s: float, regroup_budget_s: float):
        self.sup = sup
        self.stall_s = float(stall_s)
        self.regroup_budget_s = float(regroup_budget_s)
        self._lock = threading.Lock()
        self.snapshot = None
        self.extra = None
        self.epoch = 0
        self.t_snapshot = None
        self.snapshots = 0
        self._combined = None  # (key, extra) cache: same objects while nothing changed

    def push(self, epoch: int, snap, extra) -> None:
        with self._lock:
            if epoch < self.sup.epoch:
                return  # an old epoch's root, after the node moved on
            self.snapshot, self.extra, self.epoch = snap, extra, epoch
            self.t_snapshot = time.monotonic()
            self.snapshots += 1

    def collect(self):
        from ..prom.exposition import Exposition

        with self._lock:
            if self.snapshot is None:
                raise RuntimeError("no refresh yet")
            snap, extra, n = self.snapshot, self.extra, self.snapshots
        key = (n, self.sup.version)
        if self._combined is not None and self._combined[0] == key:
            return snap, self._combined[1]
        exp = Exposition()
        if extra is not None:
            exp._fams.update({k: (h, t, list(s)) for k, (h, t, s) in extra._fams.items()})
        self.sup.export_membership(exp, shown=set(snap.gpu_ids))
        self._combined = (key, exp)
        return snap, exp

    def health(self):
        """(ok, message): ok while the node refresh loop makes progress - a snapshot
        within ``stall_s``, or a regroup under way for less than ``regroup_budget_s`` (a
        member was lost and the others are re-forming). Stale sources do not count."""
        now = time.monotonic()
        with self._lock:
            t = self.t_snapshot
        sup = self.sup
        if t is not None and now - t < self.stall_s:
            return True, f"last refresh {now - t:.2f} s ago (epoch {sup.epoch}, {len(sup.members)} GPUs)"
        since = now - sup.t_change
        if since < self.regroup_budget_s:
            what = "starting" if t is None else f"regrouping (last refresh {now - t:.1f} s ago)"
            return True, f"{what}: epoch {sup.epoch} formed {since:.1f} s ago"
        if t is None:
            return False, f"no refresh {since:.1f} s after the last membership change"
        return False, f"last refresh {now - t:.2f} s ago"

    def close(self) -> None:
        pass


class NodeSupervisor:
    """Starts and supervises the rank processes of one node (see the module docstring).
    ``rank_cmd`` is the rank's argv; each rank gets ``ROCMDASH_SLOT`` / ``LOCAL_RANK`` =
    its slot, its HIP device in ``ROCMDASH_RANK_DEVICES``, the store address and the
    snapshot socket."""

    def __init__(self, rank_cmd: list, slots: int, devices=None, *, env: dict | None = None,
                 store_port: int = 0, collective_timeout_s: float = 60.0, start_timeout_s: float = 300.0,
                 restart_base_s: float = 5.0, restart_max_s: float = 300.0, healthy_reset_s: float = 600.0,
                 report_grace_s: float = 2.0, stall_s: float = 10.0, join_budget_s: float | None = None,
                 http: tuple | None = None, hostname: str | None = None, counter_daemon: dict | None = None):
        import torch.distributed as dist
        from datetime import timedelta

        if slots < 1:
            raise ValueError("no GPU slot to supervise")
        self.rank_cmd = list(rank_cmd)
        self.env = dict(os.environ if env is None else env)
        # the node's processes hold the least HBM the HIP runtime allows (a caller's own
        # settings win): every stream on ONE hardware queue - each extra queue costs ~177 MiB
        # of device memory on MI355X - a 1 MiB scratch preallocation instead of ~139 MiB
        # (rocmdash's kernels use no scratch: tests/test_kernel_resources.py), measured with
        # a bare HIP process (tools/probes/probe_hip_init.hip, profiles/r05/footprint/); and
        # RCCL buffers sized for the node's small collectives
        for k, v in LEAN_RUNTIME_ENV.items():
            self.env.setdefault(k, v)
        self.slots = [Slot(i, None if devices is None else int(devices[i])) for i in range(slots)]
        self.collective_timeout_s = float(collective_timeout_s)
        self.start_timeout_s = float(start_timeout_s)
        self.restart_base_s = float(restart_base_s)
        self.restart_max_s = float(restart_max_s)
        self.healthy_reset_s = float(healthy_reset_s)
        self.report_grace_s = float(report_grace_s)
        # an epoch that produced no snapshot this long after it formed, with no member
        # reporting anything, is wedged (every member hung): restart them all
        self.join_budget_s = float(join_budget_s if join_budget_s is not None
                                   else 3 * self.collective_timeout_s + float(os.environ.get(
                                       "ROCMDASH_RCCL_INIT_TIMEOUT", "120")))
        self.store = dist.TCPStore("127.0.0.1", int(store_port), None, True, timeout=timedelta(seconds=60),
                                   wait_for_workers=False)
        self.store_port = int(self.store.port)
        self.store.add("epoch", 0)
        self.epoch = 0
        self.members: list = []
        self.t_change = time.monotonic()
        self.version = 0  # bumped on every membership / slot-state change (exposition cache)
        self._fail_first = None  # monotonic time of the first failure report of this epoch
        self.events: list = []  # (wall time, text): the membership log (tests, /metrics info)
        self.stopping = threading.Event()
        self.source = SupervisedSource(self, stall_s, regroup_budget_s=self.collective_timeout_s * 2 + 60.0)
        self._dir = tempfile.mkdtemp(prefix="rocmdash-sup-")
        self.push_path = os.path.join(self._dir, "push.sock")
        self.push_key = secrets.token_bytes(16)
        self._listener = None
        self.exporter = None
        self._http = http
        self._hostname = hostname
        # the node's one device-counter process (rocmdash.runtime.counterd): {"devices",
        # "hz", "source"}; its rings live in a tmpfs directory the ranks get in
        # ROCMDASH_COUNTER_SHM
        self.daemon = None
        if counter_daemon:
            base = "/dev/shm" if os.path.isdir("/dev/shm") else self._dir
            shm = tempfile.mkdtemp(prefix=f"rocmdash-ctr-{self.store_port}-", dir=base)
            self.daemon = Slot(-1)
            self.daemon.info = {"dir": shm, **counter_daemon}
        # per-GPU lanes of the counter process: heartbeat watch (rocmdash.runtime.lanes)
        self.lanes = None
        if counter_daemon:
            from .lanes import LaneWatch

            self.lanes = LaneWatch(counter_daemon["devices"], float(counter_daemon.get("hz", 100.0)),
                                   base_s=restart_base_s, max_s=restart_max_s, healthy_reset_s=healthy_reset_s)
        # a counter process whose every lane stopped beating this long is wedged: restarted
        self.daemon_hang_s = float(os.environ.get("ROCMDASH_COUNTERD_HANG_S", "10"))
        self._t_lanes = -1e9
        self._cpu_last = {}  # pid -> cpu seconds at the last accounting
        self.cpu_total = {"supervisor": 0.0, "counterd": 0.0, "rank": 0.0}
        self._t_cpu = 0.0
        self.mem = {}  # (kind, gpu label) -> {"pss", "pss_anon", "rss"} bytes, every ~5 s
        self.dev_mem = {}  # (kind, gpu label, bdf hex) -> bytes of the process's own VRAM buffers there
        self._t_mem = -1e9

    # ------------------------------------------------------------------ infrastructure
    def _start_listener(self) -> None:
        from multiprocessing.connection import Listener

        self._listener = Listener(self.push_path, family="AF_UNIX", authkey=self.push_key)

        def serve_conn(conn):
            try:
                while not self.stopping.is_set():
                    epoch, snap, extra = conn.recv()
                    self.source.push(epoch, snap, extra)
            except (EOFError, OSError):
                pass
            finally:
                conn.close()

        def accept_loop():
            while not self.stopping.is_set():
                try:
                    conn = self._listener.accept()
                except (OSError, EOFError):
                    if self.stopping.is_set():
                        return
                    continue
                except Exception:  # noqa: BLE001 - a bad handshake must not end the loop
                    continue
                threading.Thread(target=serve_conn, args=(conn,), name="rocmdash-sup-push", daemon=True).start()

        threading.Thread(target=accept_loop, name="rocmdash-sup-accept", daemon=True).start()

    def _start_http(self) -> None:
        if self._http is None:
            return
        from ..prom.exporter import Exporter

        self.exporter = Exporter(self.source, hostname=self._hostname)
        self.exporter.serve(*self._http)
        log.info("supervisor serving /metrics on %s:%d for %d GPU slot(s)", self._http[0], self.exporter.port,
                 len(self.slots))

    def label(self, s: Slot) -> str:
        """The ``gpu_id`` label of a slot: its GPU's own id, unless two slots announced the
        same one (synthetic sources, several ranks on one GPU) - then the slot number, as
        the ranks' NodePipeline labels them (``rank_labels``)."""
        own = s.own_id
        if own is None:
            return str(s.index)
        ids = [x.own_id for x in self.slots if x.own_id is not None]
        return own if ids.count(own) == 1 else str(s.index)

    def _event(self, text: str) -> None:
        self.events.append((time.time(), text))
        del self.events[:-200]
        self.version += 1
        log.info("%s", text)

    # ------------------------------------------------------------------ slots
    def _spawn(self, s: Slot) -> None:
        s.incarnation += 1
        env = dict(self.env)
        for k in ("RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "TORCHELASTIC_RESTART_COUNT",
                  "TORCHELASTIC_USE_AGENT_STORE"):
            env.pop(k, None)
        env.update({ENV_ADDR: f"127.0.0.1:{self.store_port}", ENV_SLOT: str(s.index), ENV_SLOTS: str(len(self.slots)),
                    ENV_INCARNATION: str(s.incarnation), ENV_PUSH: self.push_path, ENV_PUSH_KEY: self.push_key.hex(),
                    "LOCAL_RANK": str(s.index), "MASTER_ADDR": "127.0.0.1"})
        if s.device is not None:
            devs = [str(x.device if x.device is not None else x.index) for x in self.slots]
            env["ROCMDASH_RANK_DEVICES"] = ",".join(devs)
        if self.daemon is not None:
            env["ROCMDASH_COUNTER_SHM"] = self.daemon.info["dir"]
        s.proc = subprocess.Popen(self.rank_cmd, env=env, start_new_session=True)
        s.state = "starting"
        s.t_start = time.monotonic()
        if s.incarnation > 0:
            s.restarts += 1
        s.history.append((time.monotonic(), f"start #{s.incarnation}"))
        self._event(f"slot {s.index}: started incarnation {s.incarnation} (pid {s.proc.pid})")

    def _spawn_daemon(self) -> None:
        d = self.daemon
        d.incarnation += 1
        inf = d.info
        cmd = [sys.executable, "-m", "rocmdash.runtime.counterd", "--dir", inf["dir"],
               "--devices", ",".join(str(x) for x in inf["devices"]), "--hz", str(inf.get("hz", 100.0)),
               "--source", inf.get("source", "hw")]
        env = dict(self.env)
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", ENV_ADDR):
            env.pop(k, None)
        d.proc = subprocess.Popen(cmd, env=env, start_new_session=True)
        d.state = "member"
        d.t_start = time.monotonic()
        if d.incarnation > 0:
            d.restarts += 1
        self._event(f"counter process: started incarnation {d.incarnation} (pid {d.proc.pid}) for devices "
                    f"{inf['devices']}")

    def _watch_daemon(self, now: float) -> None:
        d = self.daemon
        if d is None or self.stopping.is_set():
            return
        if d.proc is not None:
            rc = d.proc.poll()
            if rc is None:
                if d.failures and now - d.t_start > self.healthy_reset_s:
                    d.failures = 0
                if self._watch_lanes(now):
                    return
                self._kill(d)  # every lane stopped beating: the process is wedged
                try:
                    d.proc.wait(timeout=5.0)
                except subprocess.TimeoutExpired:
                    pass
                rc = f"killed: no lane beat for {self.daemon_hang_s:.0f} s"
            d.proc = None
            d.state = "down"
            d.failures += 1
            d.last_error = f"counter process exited with code {rc}"
            d.next_start = now + restart_delay(d.failures, self.restart_base_s, self.restart_max_s)
            self._event(f"{d.last_error}; restart in {d.next_start - now:.1f} s (the ranks' counter series go stale)")
        if d.proc is None and now >= d.next_start:
            self._spawn_daemon()

    def _lane_headers(self) -> dict:
        from .counterd import ring_path
        from .lanes import read_ring_header

        return {dev: read_ring_header(ring_path(self.daemon.info["dir"], dev)) for dev in self.lanes.lanes}

    def _watch_lanes(self, now: float) -> bool:
        """Per-GPU heartbeat watch of the counter process (every ~0.1 s): a GPU whose lane
        stalled while the others advance is reported down and, after a backoff, given a
        fresh lane; False when the whole process stopped beating (restart it)."""
        if self.lanes is None or now - self._t_lanes < 0.1:
            return True
        self._t_lanes = now
        headers = self._lane_headers()
        n_events = len(self.lanes.events)
        ask = self.lanes.update(now, headers)
        for _, text in self.lanes.events[n_events:]:
            self._event(text)
        if ask is not None:
            from .lanes import write_control

            try:
                write_control(self.daemon.info["dir"], ask)
            except OSError as exc:
                log.error("counter lanes: cannot write the control file: %s", exc)
        if now - self.daemon.t_start > self.daemon_hang_s and \
                self.lanes.whole_process_stalled(now, headers, self.daemon_hang_s):
            return False
        return True

    @staticmethod
    def _proc_cpu(pid: int) -> float | None:
        """utime + stime of a process (all its threads), seconds."""
        try:
            with open(f"/proc/{pid}/stat") as f:
                parts = f.read().rsplit(")", 1)[1].split()
            return (int(parts[11]) + int(parts[12])) / os.sysconf("SC_CLK_TCK")
        except (OSError, IndexError, ValueError):
            return None

    @staticmethod
    def proc_mem(pid: int) -> dict | None:
        """Proportional set size (shared pages split between the processes that map them,
        e.g. the torch / HIP libraries every rank maps), its anonymous part and RSS, bytes,
        from /proc/<pid>/smaps_rollup (one kernel-aggregated read)."""
        keys = {"Rss:": "rss", "Pss:": "pss", "Pss_Anon:": "pss_anon"}
        out = {}
        try:
            with open(f"/proc/{pid}/smaps_rollup") as f:
                for line in f:
                    k = line.split(None, 1)[0]
                    if k in keys:
                        out[keys[k]] = int(line.split()[1]) * 1024
        except (OSError, IndexError, ValueError):
            return None
        return out or None

    def account_mem(self) -> None:
        """Host memory of every node process, and the device memory each one's own
        buffers hold on each GPU (DRM fdinfo: per process, never a difference of device
        totals - ``footprint.drm_vram_by_bdf``)."""
        from .footprint import drm_vram_by_bdf

        mem = {}
        dev = {}
        procs = [("supervisor", "", os.getpid())]
        if self.daemon is not None and self.daemon.proc is not None:
            procs.append(("counterd", "", self.daemon.proc.pid))
        procs += [("rank", self.label(s), s.proc.pid) for s in self.slots if s.proc is not None]
        for kind, lab, pid in procs:
            m = self.proc_mem(pid)
            if m is not None:
                mem[(kind, lab)] = m
            for bdf, v in drm_vram_by_bdf(pid).items():
                dev[(kind, lab, "%x" % bdf if bdf else "")] = v
        self.mem = mem
        self.dev_mem = dev

    def account_cpu(self) -> None:
        """Add every node process's CPU time since the last call to ``cpu_total`` (by
        process kind; a process that exited keeps what it used up to the last call)."""
        procs = [("supervisor", os.getpid())]
        if self.daemon is not None and self.daemon.proc is not None:
            procs.append(("counterd", self.daemon.proc.pid))
        procs += [("rank", s.proc.pid) for s in self.slots if s.proc is not None]
        for kind, pid in procs:
            c = self._proc_cpu(pid)
            if c is None:
                continue
            last = self._cpu_last.get(pid, 0.0)
            if c >= last:
                self.cpu_total[kind] += c - last
            self._cpu_last[pid] = c

    def _kill(self, s: Slot, sig=signal.SIGKILL) -> None:
        if s.proc is not None and s.proc.poll() is None:
            try:
                os.killpg(s.proc.pid, sig)
            except (ProcessLookupError, PermissionError):
                pass

    def _down(self, s: Slot, why: str, kill: bool = True) -> None:
        """Slot ``s`` failed: out of service, restarted after the backoff."""
        if kill:
            self._kill(s)
        s.state = "down"
        s.t_member = None
        s.failures += 1
        s.last_error = why
        s.next_start = time.monotonic() + restart_delay(s.failures, self.restart_base_s, self.restart_max_s)
        s.history.append((time.monotonic(), "down: " + why))
        self._event(f"slot {s.index} (gpu {self.label(s)}) down: {why}; restart in "
                    f"{s.next_start - time.monotonic():.1f} s (failure {s.failures})")

    def _form(self, members: list, why: str) -> None:
        members = sorted(set(members))
        if not members:  # every member lost and none ready: the next ready slot forms one
            self.members = []
            self.t_change = time.monotonic()
            self._event(f"epoch {self.epoch}: no member left ({why})")
            return
        e = self.epoch + 1
        self.store.set(f"members/{e}", format_members(members))
        got = int(self.store.add("epoch", 1))
        if got != e:  # nothing else writes it
            raise RuntimeError(f"epoch counter {got}, expected {e}")
        self.epoch = e
        self.members = members
        self.t_change = time.monotonic()
        self._fail_first = None
        now = time.monotonic()
        for s in self.slots:
            if s.index in members:
                if s.state != "member":
                    s.t_member = now
                s.state = "member"
        self._event(f"epoch {e}: members {members} ({why})")

    # ------------------------------------------------------------------ the loop
    def step(self) -> None:
        """One pass of the supervision loop (also driven directly by tests)."""
        now = time.monotonic()
        dead = []
        for s in self.slots:
            if s.proc is None:
                continue
            rc = s.proc.poll()
            if rc is None:
                continue
            s.proc = None
            if self.stopping.is_set():
                continue
            if self.store.check([f"stopped/{s.index}/{s.incarnation}"]):  # left on a stop vote
                was_member = s.state == "member"
                s.state = "stopped"
                self._event(f"slot {s.index} stopped (exit {rc})")
                if was_member:
                    dead.append(s.index)
                continue
            if s.state == "member":
                dead.append(s.index)
            if s.state in ("member", "starting", "ready"):
                where = "in epoch %d" % self.epoch if s.state == "member" else "before it was ready"
                self._down(s, f"rank process exited with code {rc} {where}", kill=False)
        # announcements of started slots
        for s in self.slots:
            if s.state != "starting":
                continue
            key = f"ready/{s.index}/{s.incarnation}"
            if self.store.check([key]):
                try:
                    s.info = json.loads(self.store.get(key).decode())
                except ValueError:
                    s.info = {}
                s.state = "ready"
                self._event(f"slot {s.index} (gpu {self.label(s)}) ready (incarnation {s.incarnation})")
            elif now - s.t_start > self.start_timeout_s:
                self._down(s, f"not ready within {self.start_timeout_s:.0f} s of its start")
        # members that left on a stop vote while the supervisor itself is not stopping and
        # some slot is not stopped (a stray SIGTERM to one rank; the others were down or
        # ready and never voted): start them again, or the node would never re-form
        # (ADVICE r05). Every slot stopped = the node was told to stop: run() exits.
        if not self.stopping.is_set() and not all(s.state == "stopped" for s in self.slots) and \
                not any(s.state == "member" for s in self.slots):  # every voter has left
            for s in self.slots:
                if s.state == "stopped" and s.proc is None:
                    s.state = "down"
                    s.next_start = now
                    s.last_error = "left on a stop vote the node did not take"
                    self._event(f"slot {s.index}: stopped while the node runs on; starting it again")
        # backoff expired: start again (the new process probes its GPU)
        if not self.stopping.is_set():
            for s in self.slots:
                if s.state == "down" and s.proc is None and now >= s.next_start:
                    self._spawn(s)
            for s in self.slots:  # a member that stayed healthy long enough: forget its failures
                if s.state == "member" and s.failures and s.t_member is not None and \
                        now - s.t_member >= self.healthy_reset_s:
                    s.failures = 0
        self._membership(dead, now)
        self._watch_daemon(now)
        if now - self._t_cpu >= 1.0:
            self._t_cpu = now
            self.account_cpu()
        if now - self._t_mem >= 5.0:
            self._t_mem = now
            self.account_mem()

    def _membership(self, dead: list, now: float) -> None:
        ready = [s.index for s in self.slots if s.state == "ready"]
        if self.epoch == 0 or not self.members:
            # the first epoch: once every slot is ready or down (a slot that is still
            # starting holds it back, bounded by start_timeout_s)
            if ready and all(s.state in ("ready", "down") for s in self.slots):
                self._form(ready, "start-up" if self.epoch == 0 else "re-forming after every member was lost")
            return
        members = [m for m in self.members]
        if dead:
            keep = [m for m in members if m not in dead]
            self._form(keep + ready, f"lost {dead}: process exited")
            return
        # failure reports of the current epoch
        reported = [m for m in members if self.store.check([f"fail/{self.epoch}/{m}"])]
        if reported:
            if self._fail_first is None:
                self._fail_first = now
                reasons = {m: self.store.get(f"fail/{self.epoch}/{m}").decode()[:200] for m in reported}
                log.info("epoch %d: failure reports %s", self.epoch, reasons)
            if now - self._fail_first >= self.report_grace_s or len(reported) == len(members):
                culprits = decide_culprits(members, reported)
                for m in culprits:
                    self._down(self.slots[m], f"stopped answering in epoch {self.epoch} "
                                              f"(members {sorted(reported)} reported failed collectives)")
                keep = [m for m in members if m not in culprits]
                self._form(keep + ready, f"failed collectives in epoch {self.epoch}; excluded {culprits}")
            return
        if ready:
            self._form(members + ready, f"re-admitting {ready}")
            return
        # wedged: no snapshot of this epoch long after it formed and nobody reports
        src = self.source
        last = src.t_snapshot if src.epoch == self.epoch else None
        ref = last if last is not None else self.t_change
        if now - ref > self.join_budget_s:
            for m in members:
                self._down(self.slots[m], f"epoch {self.epoch} made no progress for {now - ref:.0f} s")
            self.members = []
            self.version += 1

    def start(self) -> None:
        self._start_listener()
        self._start_http()
        if self.daemon is not None:
            self._spawn_daemon()  # before the ranks: their counter sources wait for its rings
        for s in self.slots:
            self._spawn(s)

    def run(self, poll_s: float = 0.1) -> int:
        self.start()
        try:
            while not self.stopping.is_set():
                self.step()
                if all(s.state == "stopped" for s in self.slots):  # every rank voted to stop
                    log.info("every rank stopped on purpose: the supervisor exits")
                    break
                self.stopping.wait(poll_s)
        finally:
            self.shutdown()
        return 0

    def shutdown(self, grace_s: float = 15.0) -> None:
        """SIGTERM every rank (they vote to stop and leave together), then SIGKILL what
        is left after ``grace_s``."""
        self.stopping.set()
        for s in self.slots:
            self._kill(s, signal.SIGTERM)
        t_end = time.monotonic() + grace_s
        for s in self.slots + ([self.daemon] if self.daemon is not None else []):
            if s is self.daemon and s.proc is not None:
                self._kill(s, signal.SIGTERM)  # after the ranks were told to stop
            if s.proc is None:
                continue
            try:
                s.proc.wait(timeout=max(0.1, t_end - time.monotonic()))
            except subprocess.TimeoutExpired:
                self._kill(s, signal.SIGKILL)
                s.proc.wait()
        if self.exporter is not None:
            self.exporter.close()
            self.exporter = None
        if self._listener is not None:
            try:
                self._listener.close()
            except OSError:
                pass
        try:
            os.unlink(self.push_path)
            os.rmdir(self._dir)
        except OSError:
            pass
        if self.daemon is not None:
            import shutil

            shutil.rmtree(self.daemon.info["dir"], ignore_errors=True)

    # ------------------------------------------------------------------ exposition
    def export_membership(self, exp, shown: set) -> None:
        """The node's membership as metrics (added to every /metrics body)."""
        now = time.monotonic()
        for s in self.slots:
            lab = {"gpu_id": self.label(s)}
            up = 1.0 if (s.state == "member" and self.label(s) in shown) else 0.0
            exp.add("rocmdash_gpu_up", up, lab,
                    "1 while this GPU is a member of the node's current epoch and on the dashboard; 0 while it is "
                    "out (lost, restarting, or not re-admitted yet: rocmdash.runtime.supervisor)")
            exp.add("rocmdash_gpu_state", 1.0, dict(lab, state=s.state),
                    "The supervisor's state of this GPU's rank: member, ready (waiting for the next epoch), starting, "
                    "down (restart pending)")
            exp.add("rocmdash_gpu_restarts_total", s.restarts, lab, "Rank processes started again for this GPU", "counter")
            exp.add("rocmdash_gpu_consecutive_failures", s.failures, lab,
                    "Failures since this GPU was last a healthy member (sets the restart backoff)")
            if s.state != "member" and s.last_error:
                exp.add("rocmdash_gpu_down_info", 1.0, dict(lab, reason=s.last_error[:200]),
                        "Why this GPU is out of the node's epoch")
                if s.state == "down":
                    exp.add("rocmdash_gpu_restart_in_seconds", max(0.0, s.next_start - now), lab,
                            "Seconds until the supervisor starts this GPU's rank again")
        exp.add("rocmdash_node_epoch", self.epoch, {}, "Membership epochs the supervisor formed (one per regroup)",
                "counter")
        for kind, sec in self.cpu_total.items():
            exp.add("rocmdash_node_cpu_seconds_total", sec, {"process": kind},
                    "CPU seconds used by the node's rocmdash processes (all threads), by kind: supervisor, counterd "
                    "(the one device-counter process), rank (every GPU's rank process)", "counter")
        for (kind, lab), m in sorted(self.mem.items()):
            for k, v in m.items():
                exp.add("rocmdash_node_process_memory_bytes", v, {"process": kind, "gpu_id": lab, "kind": k},
                        "Host memory of the node's rocmdash processes (smaps_rollup, every ~5 s): pss (shared "
                        "pages split between the processes mapping them - sums to the node's share), pss_anon, rss")
        if self.mem:
            exp.add("rocmdash_node_pss_bytes", sum(m.get("pss", 0) for m in self.mem.values()), {},
                    "Proportional set size of every rocmdash process of the node, summed (the pod's memory)")
        for (kind, lab, bdf), v in sorted(self.dev_mem.items()):
            exp.add("rocmdash_node_process_device_memory_bytes", v, {"process": kind, "gpu_id": lab, "bdf": bdf},
                    "VRAM of the buffers each rocmdash process allocated on each GPU (DRM fdinfo drm-memory-vram, "
                    "every ~5 s; the driver's per-process and per-queue state is not in it)")
        if self.daemon is not None:
            d = self.daemon
            exp.add("rocmdash_counter_daemon_up", 1.0 if d.proc is not None else 0.0, {},
                    "1 while the node's device-counter process runs (rocmdash.runtime.counterd)")
            exp.add("rocmdash_counter_daemon_restarts_total", d.restarts, {}, "Counter process restarts", "counter")
            if d.proc is not None:
                exp.add("rocmdash_counter_daemon_pid", d.proc.pid, {"dir": d.info["dir"]},
                        "Process id of the node's counter process and its ring directory")
            if self.lanes is not None:
                by_dev = {}
                for s in self.slots:
                    by_dev.setdefault(s.device if s.device is not None else s.index, self.label(s))
                for dev, st in sorted(self.lanes.lanes.items()):
                    lab = {"gpu_id": by_dev.get(dev, str(dev))}
                    up = st.up and d.proc is not None
                    reason = st.reason if not st.up else ("" if up else d.last_error or "counter process down")
                    exp.add("rocmdash_counter_source_up", 1.0 if up else 0.0, lab,
                            "1 while this GPU's lane of the node counter process publishes counter rows; 0 while "
                            "its reads are stalled (the other GPUs' lanes go on; rocmdash.runtime.lanes) or the "
                            "process is down")
                    if not up:
                        exp.add("rocmdash_counter_source_down_info", 1.0, dict(lab, reason=reason[:200]),
                                "Why this GPU's device-counter source is down")
                    if st.age_s is not None:
                        exp.add("rocmdash_counter_source_beat_age_seconds", st.age_s, lab,
                                "Seconds since this GPU's counter lane finished its last read")
                    exp.add("rocmdash_counter_source_lane", st.lane, lab,
                            "Generation of this GPU's counter lane (a fresh lane replaces a stalled one)")
                    exp.add("rocmdash_counter_source_stalls_total", st.stalls, lab,
                            "Times this GPU's counter lane stalled", "counter")
        exp.add("rocmdash_node_members", len(self.members), {}, "GPUs in the current epoch")
        exp.add("rocmdash_node_slots", len(self.slots), {}, "GPU slots the supervisor runs (physical GPUs of the node)")
        t = self.source.t_snapshot
        if t is not None:
            exp.add("rocmdash_supervisor_snapshot_age_seconds", now - t, {},
                    "Seconds since the epoch root pushed its last refresh")


def serve_args(module_args: list) -> dict:
    """The options of ``rocmdash.serve`` the supervisor needs (HTTP address, refresh rate,
    collective timeout, stall budget, where the counters come from), from the rank command
    line."""
    import argparse

    from .. import config

    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=config.EXPORTER_PORT)
    ap.add_argument("--refresh-hz", type=float, default=1.0)
    ap.add_argument("--collective-timeout", type=float,
                    default=float(os.environ.get("ROCMDASH_COLLECTIVE_TIMEOUT", "60")))
    ap.add_argument("--stall-seconds", type=float, default=0.0)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--source", default="auto")
    ap.add_argument("--counters", default="auto")
    known, _ = ap.parse_known_args(module_args)
    period = 1.0 / known.refresh_hz
    return {"host": known.host, "port": known.port, "period": period, "collective_timeout": known.collective_timeout,
            "stall_s": known.stall_seconds or max(10.0, 5 * period), "cpu": known.cpu, "source": known.source,
            "counters": known.counters}


def counter_daemon_plan(mode: str, sa: dict, slots: int, devices=None) -> dict | None:
    """Whether the node's counter process runs, and for which devices: ``mode`` "on",
    "off" or "auto" (on for live hardware counters: not ``--cpu``, counters auto / hw, a
    live source). Its source is synthetic when the ranks' counters are synthetic (CPU
    tests of the same path). Devices: the HIP device of every slot (one ring each)."""
    live = not sa["cpu"] and sa["counters"] in ("auto", "hw") and sa["source"] != "synthetic"
    if mode == "off" or sa["counters"] == "off" or (mode == "auto" and not live):
        return None
    if sa["cpu"]:
        devs = list(range(slots))
    elif devices is not None:
        devs = [int(d) for d in devices]
    else:
        from ..parallel.node import device_index_for

        devs = [device_index_for(i) for i in range(slots)]
    return {"devices": sorted(set(devs)), "hz": float(os.environ.get("ROCMDASH_COUNTER_HZ", "100")),
            "source": "hw" if live else "synthetic"}


def run_supervisor(module: str, module_args: list, slots: int, devices=None, *, store_port: int = 0,
                   restart_base_s: float = 5.0, restart_max_s: float = 300.0, start_timeout_s: float = 300.0,
                   counter_daemon: str = "auto") -> int:
    """Entry of ``rocmdash.launch`` (default mode): supervise ``slots`` ranks of
    ``python -m <module> <module_args>``. SIGTERM / SIGINT stop the node (every rank
    votes to stop and leaves after the same refresh)."""
    if not logging.getLogger().handlers:
        logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(message)s")
    sa = serve_args(module_args)
    sup = NodeSupervisor([sys.executable, "-m", module, *module_args], slots, devices, store_port=store_port,
                         collective_timeout_s=sa["collective_timeout"], start_timeout_s=start_timeout_s,
                         restart_base_s=restart_base_s, restart_max_s=restart_max_s,
                         report_grace_s=min(max(2.0, 3 * sa["period"]), max(2.0, sa["collective_timeout"] / 2)),
                         stall_s=sa["stall_s"], http=(sa["host"], sa["port"]),
                         counter_daemon=counter_daemon_plan(counter_daemon, sa, slots, devices))

    def on_signal(*_):
        sup.stopping.set()

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, on_signal)
    return sup.run()
