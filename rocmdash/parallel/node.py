"""Whole-node aggregation: one process per GPU, RCCL all-gather over xGMI.

Reference counterpart: the cross-GPU mean over the selected GPUs (``app.py:338-345``)
and the mean/max/min over all GPUs (``app.py:216-221``), computed on one pandas
DataFrame that an external Prometheus filled. Here each rank owns its GPU's sampler,
rings and window-stats kernel output ``[S, 8]`` float32 on its device, and ONE
all-gather per refresh builds the ``[N, rows, 8]`` node tensor.

Two planes:

* **Data plane** - the refresh's gathers of device tensors: ONE RCCL communicator per
  process, created by rocmdash itself (``RcclTransport``, csrc/rccl_comm.cpp), driven
  with ``ncclAllGather`` on the caller's stream right behind the stats kernel. At N > 1
  that is the ring over xGMI; the publish kernel behind it hands rank 0 the node tensor
  (``NativeNodeGather``).
* **Control plane** - ``torch.distributed`` on gloo: rendezvous, the start-up facts
  (``all_gather_object``), barriers, the bench's reductions, the bit-for-bit validation
  of the first native gathers and the agreed fallback gather through host memory. No
  ``ProcessGroupNCCL`` is ever created, so each rank holds one RCCL communicator, not two
  (``ROCMDASH_PG_BACKEND=nccl`` restores torch's RCCL group, e.g. for A/B runs).

Sizing for MI355X xGMI: a rank contributes (S + side rows) * 8 * 4 B - 512 B for the 16
series, ~900 B with the service's health, XCD and control rows - so the collective is
latency-bound (alpha term), not bandwidth-bound; the communicator is created once and
reused every refresh, with no host synchronisation between the stats kernel and the
gather. Static per-GPU facts (part number, power cap, bdf) travel once, at start-up,
through ``all_gather_object``.

On CPU (tests, a CPU-only dashboard) the same code runs over ``gloo``.
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int
    world_size: int
    local_rank: int
    backend: str
    device: torch.device
    initialized_here: bool = False


def _truthy(name: str, default: str = "0") -> bool:
    return os.environ.get(name, default).strip().lower() not in ("0", "", "false", "off", "no")


def control_backend() -> str:
    """torch.distributed backend of the control plane: ``gloo`` unless
    ``ROCMDASH_PG_BACKEND`` says otherwise (the data plane is rocmdash's own RCCL
    communicator either way)."""
    return os.environ.get("ROCMDASH_PG_BACKEND", "gloo").strip().lower() or "gloo"


def oversubscribed() -> bool:
    """``ROCMDASH_OVERSUBSCRIBE=1``: rehearsal mode for a box with fewer GPUs than ranks.
    Rank r drives GPU ``local_rank % device_count`` and announces its own host id to RCCL
    (``NCCL_HOSTID``): RCCL refuses two ranks of one communicator on one device of one
    host, so the ranks pose as separate hosts and RCCL connects them with its network
    transport (sockets on ``lo``) instead of xGMI. The collective - RCCL's kernels, proxy
    threads, rank order, rocmdash's publish / validation / fallback - runs for real with
    N ranks on one MI355X; the xGMI links do not (profiles/r03/multirank/)."""
    return _truthy("ROCMDASH_OVERSUBSCRIBE")


def device_index_for(local_rank: int) -> int:
    """The HIP device a rank drives (``torch.cuda.device_count()`` and the topology
    walk do not initialise HIP):
      * ``ROCMDASH_RANK_DEVICES`` (set by ``python -m rocmdash.launch``): its entry;
      * a node whose GPUs are compute-partitioned (several HIP devices per physical
        GPU, rocmdash.runtime.topology.node_plan): the first partition of the rank's
        physical GPU - one rank per physical GPU;
      * oversubscribed: ``local_rank % GPUs``;
      * else its local rank."""
    spec = os.environ.get("ROCMDASH_RANK_DEVICES", "").strip()
    if spec:
        devs = [int(x) for x in spec.split(",") if x.strip()]
        if local_rank < len(devs):
            return devs[local_rank]
    if oversubscribed():
        n = torch.cuda.device_count()
        return local_rank % n if n > 0 else local_rank
    from ..runtime.topology import node_plan

    plan = node_plan()
    if (plan is not None and plan["logical_devices"] > len(plan["gpus"]) and local_rank < len(plan["gpus"])
            and plan["logical_devices"] <= torch.cuda.device_count()):
        return plan["gpus"][local_rank]["hip_device"]
    return local_rank


def dist_env_from_environ(prefer_gpu: bool = True, backend: str | None = None,
                          timeout_s: float | None = None, world1_group: bool = False) -> DistEnv:
    """Initialise ``torch.distributed`` from torchrun's env (RANK/WORLD_SIZE/
    LOCAL_RANK/MASTER_*) if needed. World size 1 without env vars stays
    non-distributed, unless ``world1_group``: then a one-rank group is created on an
    in-process store (no rendezvous, no port), so the collective path - the native RCCL
    communicator, ``ncclAllGather``, the publish kernel - runs for real on a single GPU
    (GPU tests, the bench's N = 1 gather measurement).

    ``backend`` defaults to :func:`control_backend` (gloo): the process group is the
    control plane only. ``timeout_s`` bounds every control-plane collective: a rank that
    stops answering (dead process, hung driver call) makes the others fail after that
    long instead of blocking forever, so the service exits and its launcher (torchrun
    ``--max-restarts``) re-creates the whole group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    device, local_rank = local_device(prefer_gpu)
    use_gpu = device.type == "cuda"
    if backend is None:
        backend = control_backend()
        if backend == "nccl" and not use_gpu:
            backend = "gloo"
    created = False
    if world == 1 and world1_group and not dist.is_initialized():
        kw = {"backend": backend, "rank": 0, "world_size": 1, "store": dist.HashStore()}
        if backend == "nccl" and nccl_eager():
            kw["device_id"] = device
        dist.init_process_group(**kw)
        created = True
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = {"backend": backend, "rank": rank, "world_size": world}
        if timeout_s:
            from datetime import timedelta

            kw["timeout"] = timedelta(seconds=float(timeout_s))
        store = _restart_store(rank, world)
        if store is not None:
            kw["store"] = store
        if backend == "nccl" and nccl_eager():
            kw["device_id"] = device
        dist.init_process_group(**kw)
        created = True
    if dist.is_initialized():
        backend = dist.get_backend()
        rank = dist.get_rank()
        world = dist.get_world_size()
    return DistEnv(rank, world, local_rank, backend, device, created)


def local_device(prefer_gpu: bool = True) -> tuple:
    """(torch device, local rank) of this rank from the launcher's env, WITHOUT creating
    the process group: the bench builds its GPU agent and takes its start-up verdict
    before any group or communicator exists (so one rank can be restarted alone). Sets the
    current device, and for an oversubscribed rehearsal the rank's own RCCL host id
    (before anything loads RCCL)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    if oversubscribed() and world > 1:
        # before anything loads RCCL: every rank its own "host" (see oversubscribed())
        os.environ["NCCL_HOSTID"] = f"rocmdash-virt-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    device = torch.device("cuda", device_index_for(local_rank)) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    return device, local_rank


def nccl_eager() -> bool:
    """(``ROCMDASH_PG_BACKEND=nccl`` only) create torch's RCCL communicator inside
    ``init_process_group`` (``device_id``) or at the first collective (default). Lazy
    creation is a measured choice: a communicator created BEFORE the GPU agent (pinned
    rings, counter contexts, device windows) left every later device-counter read at
    ~109 us instead of ~75 us and the stats launch + sync at ~105 us instead of ~31 us
    for the life of the process, while the same communicator created after the agent
    costs nothing (profiles/r02/rccl_order_ab.txt). rocmdash's own communicator is
    likewise created after the agent (``NodePipeline``). ``ROCMDASH_NCCL_EAGER=1``
    forces eager creation."""
    return _truthy("ROCMDASH_NCCL_EAGER")


def _restart_store(rank: int, world: int):
    """After a torchrun restart (TORCHELASTIC_RESTART_COUNT > 0) the rendezvous store
    still holds the previous attempt's process-group keys (peer addresses of ranks
    that are gone), and a fast rank can read a stale one before its peer rewrites it.
    Key the group by attempt instead: same store, prefix ``rocmdash/attempt<k>/``.
    bench.py's per-rank measurement children (``ROCMDASH_BENCH_CHILD``) are keyed by
    the start-up round their parents agreed on: all their starts share the launcher's
    store."""
    attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or "0"
    if os.environ.get("ROCMDASH_BENCH_CHILD"):
        # the round the rank processes agreed on when they let their children go (ranks
        # may have restarted their children a different number of times)
        attempt += ".b" + os.environ.get("ROCMDASH_BENCH_ROUND", os.environ.get("ROCMDASH_BENCH_ATTEMPT", "0"))
    elif attempt == "0":
        return None
    from datetime import timedelta

    agent_store = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
    base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                         is_master=(rank == 0 and not agent_store), timeout=timedelta(seconds=300),
                         wait_for_workers=False)
    return dist.PrefixStore(f"rocmdash/attempt{attempt}/", base)


class NativeGatherUnavailable(RuntimeError):
    """Some rank could not set up the native RCCL gather; raised on every rank alike."""


class PublicationSuperseded(RuntimeError):
    """A newer publication overwrote the one being waited for before it was read out: a
    hand-off ordering error on this rank, not a lost peer (the communicator is left
    alone)."""


def await_publication(pub, seq: int, transport, timeout_s: float, what: str = "native RCCL gather",
                      abandon=None) -> None:
    """Wait until publication ``seq`` of ``pub`` (a HostPublisher enqueued behind a
    collective) is out, bounded. RCCL's kernels wait on the device for peers that may be
    gone (a dead or hung rank never arrives, and a stream synchronisation would block
    forever), so: past ``timeout_s`` - or as soon as ``transport`` reports an error, or
    ``abandon()`` (checked every 0.25 s once the wait has lasted 1 s) says the node has
    moved on without this collective (the supervisor formed a newer epoch:
    rocmdash.parallel.membership) - the communicator is aborted (its stuck kernels exit)
    and this raises RuntimeError. A superseded publication raises
    :class:`PublicationSuperseded` at once instead of being mistaken for a slow peer
    (ADVICE r03)."""
    if not seq:
        raise RuntimeError(f"{what}: nothing was published")
    sup0 = int(getattr(pub, "superseded", 0))
    if pub.wait(seq, 1.0):
        return
    deadline = time.monotonic() + timeout_s
    while True:
        if int(getattr(pub, "superseded", 0)) != sup0:
            raise PublicationSuperseded(f"{what}: publication {seq} was superseded before it was read")
        if pub.wait(seq, 0.25):
            return
        broken = transport is not None and hasattr(transport, "healthy") and not transport.healthy()
        gone = not broken and abandon is not None and bool(abandon())
        if broken or gone or time.monotonic() >= deadline:
            if transport is not None:
                transport.close()  # ncclCommAbort
            raise RuntimeError(f"{what} " + ("reported an error" if broken else
                               "abandoned: the node supervisor formed a newer epoch" if gone else
                               f"not complete after {timeout_s:.0f} s: a rank is gone or hung"))


def _rccl_lib() -> str:
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


class RcclTransport:
    """The process's ONE RCCL communicator (csrc/rccl_comm.cpp): ``ncclAllGather`` of
    device tensors on the caller's stream, and the publishers (csrc/publish.hip) that
    hand gathered tensors to the host.

    Created collectively (every rank, after its GPU agent: see ``nccl_eager``), in three
    agreed steps so that no rank is ever left blocked in a collective its peers skipped
    (ADVICE r02):
      1. every rank loads RCCL (``rccl_load``) and the ranks share the outcome;
      2. rank 0's unique id travels through ``all_gather_object``;
      3. every rank creates its communicator non-blocking with a deadline
         (``ROCMDASH_RCCL_INIT_TIMEOUT``, default 120 s: a peer that failed inside its
         init turns into an error here, not a hang), then the ranks share the outcome.
    Any failure in any step raises ``NativeGatherUnavailable`` on EVERY rank."""

    kind = "rccl"

    def __init__(self, comm, device: torch.device, nat, version: int, log_path: str | None = None):
        self.comm = comm
        self.device = device
        self.nat = nat
        self.version = version
        self.log_path = log_path  # RCCL's INIT log of this rank (rccl_log.configure_debug_log)
        self._detail = None

    @classmethod
    def create(cls, aggregator: "NodeAggregator", device: torch.device, timeout_s: float | None = None):
        from ..runtime import native

        from .rccl_log import configure_debug_log

        nat = native.load()
        lib = _rccl_lib()
        timeout_s = float(os.environ.get("ROCMDASH_RCCL_INIT_TIMEOUT", "120")) if timeout_s is None else timeout_s
        # RCCL's own record of the transport it picks per peer (P2P over xGMI, SHM, NET):
        # its INIT log, pointed at a per-rank file before RCCL's first logging call
        log_path = configure_debug_log(aggregator.rank)

        def agree(err):
            errs = [e for e in aggregator.all_gather_object(err) if e]
            if errs:
                raise NativeGatherUnavailable("; ".join(errs))

        version, err = 0, None
        try:
            version = int(nat.rccl_load(lib))
        except Exception as e:  # noqa: BLE001 - reported to every rank
            err = f"rank {aggregator.rank}: {e}"
        agree(err)
        uid, err = None, None
        if aggregator.rank == 0:
            try:
                uid = nat.rccl_unique_id(lib)
            except Exception as e:  # noqa: BLE001
                err = f"rank 0: {e}"
        got = aggregator.all_gather_object((uid, err))
        uid, err = got[0]
        if err:
            raise NativeGatherUnavailable(err)
        comm, err = None, None
        try:
            comm = nat.RcclComm(device.index, aggregator.world_size, aggregator.rank, uid, lib, timeout_s)
        except Exception as e:  # noqa: BLE001
            err = f"rank {aggregator.rank}: {e}"
        try:
            agree(err)
        except NativeGatherUnavailable:
            if comm is not None:
                comm.abort()  # a communicator whose peers failed is never used
            raise
        return cls(comm, device, nat, version, log_path)

    def all_gather(self, local: torch.Tensor, out: torch.Tensor, stream: int) -> None:
        self.comm.all_gather(local.data_ptr(), out.data_ptr(), local.numel(), stream)

    def view(self) -> dict:
        """RCCL's own view of the communicator: {"nranks", "rank", "device"}
        (ncclCommCount / ncclCommUserRank / ncclCommCuDevice)."""
        if self.comm is None:
            return {"nranks": -1, "rank": -1, "device": -1}
        return dict(self.comm.view())

    def transport_detail(self) -> dict | None:
        """The transports RCCL logged for this rank's peer connections
        (rccl_log.parse_transport_log), or None without a log. Channels connect at the
        first collective, so call it after a gather; the answer is kept once it names a
        peer."""
        if self._detail is not None:
            return self._detail
        from .rccl_log import read_transport_log

        d = read_transport_log(self.log_path, self.comm.rank if self.comm is not None else None)
        if d is not None and d["kinds"]:
            self._detail = d
        return d

    def publisher(self, tagged: bool):
        return self.nat.HostPublisher(self.device.index, tagged=tagged)

    def healthy(self) -> bool:
        return self.comm is not None and self.comm.async_error() == 0

    def describe(self) -> str:
        return f"RCCL {self.version} ncclAllGather (native communicator)"

    def close(self) -> None:
        if self.comm is not None:
            self.comm.abort()
            self.comm = None


class NodeAggregator:
    """All-gathers each rank's stats tensor into the node tensor.

    At world size 1 the gather is the identity and no collective is issued, unless
    ``force_collective`` (default: ``ROCMDASH_FORCE_COLLECTIVE=1``) and a process group
    exists: then every call below runs the real collective on the one-rank group, so
    RCCL's communicator and kernels are exercised and timed on a single GPU.

    Device tensors go through the native RCCL communicator once :meth:`enable_native`
    succeeded (collectively); without it, through torch's collective on an nccl group,
    or through host memory on the gloo control plane (the agreed fallback)."""

    def __init__(self, group=None, force_collective: bool | None = None):
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world_size = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.backend = dist.get_backend(group) if self.distributed else "none"
        if force_collective is None:
            force_collective = _truthy("ROCMDASH_FORCE_COLLECTIVE")
        if force_collective and not self.distributed:
            raise RuntimeError("force_collective needs a process group (dist_env_from_environ(world1_group=True))")
        self.force_collective = bool(force_collective)
        # True when every call issues a collective (world > 1, or forced at world 1)
        self.collective = self.world_size > 1 or self.force_collective
        self._outs = {}
        self.calls = 0
        self.collectives = 0  # collectives actually issued (tests assert on it)
        self.native = None  # the data-plane transport (RcclTransport), enable_native()
        self.native_error = None  # why enable_native() failed (every rank alike)
        # supervised service (rocmdash.parallel.membership): a callable that is true once
        # the node moved on to a newer epoch - bounded waits give up at once then
        self.abandon = None

    # ------------------------------------------------------------------ data plane
    def enable_native(self, device: torch.device, factory=None) -> bool:
        """Collective (every rank, once its GPU agent exists): create the data-plane
        transport - ``RcclTransport`` unless ``factory(aggregator, device)`` builds
        another (tests: a gloo stand-in). True when every rank has it; False on every
        rank (``native_error`` says why) when any rank could not. ``ROCMDASH_NATIVE_GATHER=0``
        turns it off everywhere (the setting must agree across ranks)."""
        if self.native is not None:
            return True
        if not self.collective or not _truthy("ROCMDASH_NATIVE_GATHER", "1"):
            return False
        try:
            self.native = (factory or RcclTransport.create)(self, device)
        except NativeGatherUnavailable as e:
            self.native_error = str(e)
            self.native = None
            return False
        return True

    def disable_native(self, reason: str) -> None:
        """Drop the data-plane transport on this rank (callers agree first: every rank
        calls it after the same collective outcome)."""
        if self.native is not None:
            self.native.close()
        self.native = None
        self.native_error = reason

    def _buffer(self, shape, dtype, device):
        key = (tuple(shape), dtype, device)
        out = self._outs.get(key)
        if out is None:
            pin = device.type == "cpu" and torch.cuda.is_available()
            out = self._outs[key] = torch.empty(shape, dtype=dtype, device=device, pin_memory=pin)
        return out

    def all_gather(self, local: torch.Tensor) -> torch.Tensor:
        """``local`` [*shape] -> [world, *shape] on the same device. One output buffer
        per (shape, dtype, device) is allocated once and reused (stable address for
        graph capture / no allocator churn per refresh, also when the stats, window and
        per-XCD gathers of a service refresh alternate). The result is overwritten by
        the next gather of the same shape."""
        self.calls += 1
        if not self.collective:
            return local.unsqueeze(0)
        self.collectives += 1
        local = local.contiguous()
        out = self._buffer((self.world_size,) + tuple(local.shape), local.dtype, local.device)
        if self.native is not None and local.device == self.native.device and local.dtype == torch.float32:
            self.native.all_gather(local, out, torch.cuda.current_stream(local.device).cuda_stream)
        elif self.backend == "nccl":
            dist.all_gather_into_tensor(out, local, group=self.group)
        elif local.is_cuda:  # gloo control plane without the native transport: via the host
            out.copy_(self._host_gather(local), non_blocking=True)
        else:
            dist.all_gather(list(out.unbind(0)), local, group=self.group)
        return out

    def host_all_gather(self, local: torch.Tensor) -> torch.Tensor:
        """``local`` (any device) -> [world, *shape] in host memory, over the control
        plane (the native gather's validation reference and its agreed fallback).
        Synchronises ``local``'s stream (the D2H copy). Counted as a collective."""
        self.calls += 1
        if not self.collective:
            return local.detach().to("cpu").unsqueeze(0)
        self.collectives += 1
        return self._host_gather(local)

    def _host_gather(self, local: torch.Tensor) -> torch.Tensor:
        h = local.detach().contiguous().to("cpu")
        out = self._buffer((self.world_size,) + tuple(h.shape), h.dtype, torch.device("cpu"))
        if self.backend == "nccl":  # torch's RCCL group carries no host tensors
            for r, blk in enumerate(self.all_gather_object(h.numpy())):
                out[r].copy_(torch.from_numpy(blk))
        else:
            dist.all_gather(list(out.unbind(0)), h, group=self.group)
        return out

    # ------------------------------------------------------------------ control plane
    def all_gather_object(self, obj) -> list:
        if self.world_size == 1:  # start-up only: nothing to measure, never forced
            return [obj]
        res = [None] * self.world_size
        dist.all_gather_object(res, obj, group=self.group)
        return res

    def barrier(self) -> None:
        if self.collective:
            self.collectives += 1
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)

    def max_over_ranks(self, value: float, device=None) -> float:
        return self._reduce(value, dist.ReduceOp.MAX, device)

    def min_over_ranks(self, value: float, device=None) -> float:
        return self._reduce(value, dist.ReduceOp.MIN, device)

    def sum_over_ranks(self, value: float, device=None) -> float:
        return self._reduce(value, dist.ReduceOp.SUM, device)

    def _reduce(self, value: float, op, device=None) -> float:
        if not self.collective:
            return float(value)
        if self.backend == "nccl":
            device = device or torch.device("cuda", torch.cuda.current_device())
        else:
            device = None  # gloo: host tensors
        self.collectives += 1
        t = torch.tensor([float(value)], dtype=torch.float64, device=device or "cpu")
        dist.all_reduce(t, op=op, group=self.group)
        return float(t.item())


class NativeNodeGather:
    """The refresh's node all-gather as ONE ``ncclAllGather`` on the caller's stream,
    on the aggregator's data-plane transport, followed by the publish kernel
    (csrc/publish.hip): rank 0's pinned buffer receives the node tensor (tagged words
    by default) and every rank gets a completion signal in mapped host memory to spin on.
    Replaces torch's ``all_gather_into_tensor`` (~14 us of host time per call, plus
    stream hand-offs) + D2H copy + stream synchronisation on the N > 1 hot path.

    ``validated`` counts gathers that matched the control plane's host gather bit for
    bit (``NodePipeline`` checks the first ``ROCMDASH_GATHER_VALIDATE`` of them)."""

    def __init__(self, aggregator: "NodeAggregator", device: torch.device, block_shape: tuple,
                 root_host: torch.Tensor | None = None, tagged: bool | None = None):
        if aggregator.native is None:
            raise NativeGatherUnavailable(aggregator.native_error or "native transport not enabled")
        self.transport = aggregator.native
        self.world_size = aggregator.world_size
        self.out = torch.empty((aggregator.world_size,) + tuple(block_shape), dtype=torch.float32, device=device)
        if tagged is None:  # ROCMDASH_TAGGED_OUT=0: copy + completion flag
            tagged = _truthy("ROCMDASH_TAGGED_OUT", "1")
        self.pub = self.transport.publisher(tagged)
        if root_host is not None and (root_host.numel() != self.out.numel()
                                      or (self.out.is_cuda and not root_host.is_pinned())):
            raise ValueError("root_host must be a pinned tensor with the node tensor's size")
        self.host = root_host
        self.seq = 0
        self.validated = 0

    def all_gather(self, local: torch.Tensor, stream: int) -> torch.Tensor:
        """Enqueue the gather of ``local`` (contiguous float32 of ``block_shape``);
        returns the device node tensor (valid in stream order)."""
        if not local.is_contiguous() or local.numel() * self.world_size != self.out.numel():
            raise ValueError("local block does not match the node tensor")
        self.transport.all_gather(local, self.out, stream)
        return self.out

    def publish(self, stream: int) -> int:
        """Enqueue the publication of the gathered tensor (rank 0: into ``host``; other
        ranks: the completion signal only)."""
        if self.host is not None:
            self.seq = self.pub.publish(self.out.data_ptr(), self.host.data_ptr(), self.out.numel(), stream)
        else:
            self.seq = self.pub.publish(0, 0, 0, stream)
        return self.seq

    def gather(self, local: torch.Tensor, stream: int) -> torch.Tensor:
        self.all_gather(local, stream)
        self.publish(stream)
        return self.out

    def wait(self, timeout_s: float = 1.0) -> bool:
        """Spin until the last gather is published (rank 0: its node tensor is in the
        pinned buffer); False on timeout (or a superseded publication)."""
        return bool(self.seq) and bool(self.pub.wait(self.seq, timeout_s))
