"""Whole-node aggregation: one process per GPU, RCCL all-gather over xGMI.

Reference counterpart: the cross-GPU mean over the selected GPUs (``app.py:338-345``)
and the mean/max/min over all GPUs (``app.py:216-221``), computed on one pandas
DataFrame that an external Prometheus filled. Here each rank owns its GPU's sampler,
rings and window-stats kernel output ``[S, 8]`` float32 on its device, and ONE
``all_gather_into_tensor`` per refresh builds the ``[N, S, 8]`` node tensor on every
rank (backend ``"nccl"`` is RCCL on ROCm).

Sizing for MI355X xGMI: a rank contributes S * 8 * 4 B = 480 B (S = 15 series), so
the collective is latency-bound (alpha term), not bandwidth-bound; the communicator is
created once and reused every refresh, and the gather is issued on the current
stream right behind the stats kernel with no host synchronisation in between. Static
per-GPU facts (part number, power cap, bdf) travel once, at start-up, through
``all_gather_object``.

On CPU (tests, a CPU-only dashboard) the same code runs over ``gloo``.
"""

from __future__ import annotations

import os
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


def dist_env_from_environ(prefer_gpu: bool = True, backend: str | None = None,
                          timeout_s: float | None = None, world1_group: bool = False) -> DistEnv:
    """Initialise ``torch.distributed`` from torchrun's env (RANK/WORLD_SIZE/
    LOCAL_RANK/MASTER_*) if needed. World size 1 without env vars stays
    non-distributed, unless ``world1_group``: then a one-rank group is created on an
    in-process store (no rendezvous, no port), so the collective path - RCCL
    communicator, ``all_gather_into_tensor``, barrier, all-reduce - runs for real on a
    single GPU (GPU tests, the bench's N = 1 gather measurement).

    ``timeout_s`` bounds every collective: a rank that stops answering (dead process,
    hung driver call) makes the others' all-gather fail after that long instead of
    blocking forever, so the service exits and its launcher (torchrun
    ``--max-restarts``) re-creates the whole communicator."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = prefer_gpu and torch.cuda.is_available()
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    device = torch.device("cuda", local_rank) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
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


def nccl_eager() -> bool:
    """Create the RCCL communicator inside ``init_process_group`` (``device_id``) or at
    the first collective (default). Lazy creation is a measured choice: a communicator
    created BEFORE the GPU agent (pinned rings, counter contexts, device windows) left
    every later device-counter read at ~109 us instead of ~75 us and the stats launch +
    sync at ~105 us instead of ~31 us for the life of the process, while the same
    communicator created after the agent costs nothing (profiles/r02/rccl_order_ab.txt).
    The first collective of every entry point (``NodePipeline``'s start-up
    ``all_gather_object``) runs after its agent exists. ``ROCMDASH_NCCL_EAGER=1`` forces
    eager creation."""
    return os.environ.get("ROCMDASH_NCCL_EAGER", "0") not in ("0", "", "false", "off")


def _restart_store(rank: int, world: int):
    """After a torchrun restart (TORCHELASTIC_RESTART_COUNT > 0) the rendezvous store
    still holds the previous attempt's process-group keys (peer addresses of ranks
    that are gone), and a fast rank can read a stale one before its peer rewrites it.
    Key the group by attempt instead: same store, prefix ``rocmdash/attempt<k>/``.
    bench.py's per-rank measurement children (``ROCMDASH_BENCH_CHILD``) are keyed by
    their own attempt too: all their starts share the launcher's store."""
    attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or "0"
    if os.environ.get("ROCMDASH_BENCH_CHILD"):
        attempt += ".b" + os.environ.get("ROCMDASH_BENCH_ATTEMPT", "0")
    elif attempt == "0":
        return None
    from datetime import timedelta

    agent_store = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
    base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                         is_master=(rank == 0 and not agent_store), timeout=timedelta(seconds=300),
                         wait_for_workers=False)
    return dist.PrefixStore(f"rocmdash/attempt{attempt}/", base)


class NodeAggregator:
    """All-gathers each rank's stats tensor into the node tensor.

    At world size 1 the gather is the identity and no collective is issued, unless
    ``force_collective`` (default: ``ROCMDASH_FORCE_COLLECTIVE=1``) and a process group
    exists: then every call below runs the real collective on the one-rank group, so
    RCCL's communicator and kernels are exercised and timed on a single GPU."""

    def __init__(self, group=None, force_collective: bool | None = None):
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world_size = dist.get_world_size(group) if self.distributed else 1
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.backend = dist.get_backend(group) if self.distributed else "none"
        if force_collective is None:
            force_collective = os.environ.get("ROCMDASH_FORCE_COLLECTIVE", "0") not in ("0", "", "false", "off")
        if force_collective and not self.distributed:
            raise RuntimeError("force_collective needs a process group (dist_env_from_environ(world1_group=True))")
        self.force_collective = bool(force_collective)
        # True when every call issues a collective (world > 1, or forced at world 1)
        self.collective = self.world_size > 1 or self.force_collective
        self._outs = {}
        self.calls = 0
        self.collectives = 0  # collectives actually issued (tests assert on it)

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
        shape = (self.world_size,) + tuple(local.shape)
        key = (shape, local.dtype, local.device)
        out = self._outs.get(key)
        if out is None:
            out = self._outs[key] = torch.empty(shape, dtype=local.dtype, device=local.device)
        if self.backend == "nccl":
            dist.all_gather_into_tensor(out, local, group=self.group)
        else:
            dist.all_gather(list(out.unbind(0)), local, group=self.group)
        return out

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

    def sum_over_ranks(self, value: float, device=None) -> float:
        return self._reduce(value, dist.ReduceOp.SUM, device)

    def _reduce(self, value: float, op, device=None) -> float:
        if not self.collective:
            return float(value)
        if device is None and self.backend == "nccl":
            device = torch.device("cuda", torch.cuda.current_device())
        self.collectives += 1
        t = torch.tensor([float(value)], dtype=torch.float64, device=device or "cpu")
        dist.all_reduce(t, op=op, group=self.group)
        return float(t.item())


class NativeGatherUnavailable(RuntimeError):
    """Some rank could not set up the native RCCL gather; raised on every rank alike."""


class NativeNodeGather:
    """The refresh's node all-gather as ONE ``ncclAllGather`` on the caller's stream,
    on a communicator of its own (csrc/rccl_comm.cpp), followed by the publish kernel
    (csrc/publish.hip): rank 0's pinned buffer receives the node tensor and every rank
    gets a completion flag in mapped host memory to spin on. Replaces torch's
    ``all_gather_into_tensor`` (~14 us of host time per call, plus stream hand-offs)
    + D2H copy + stream synchronisation on the N > 1 hot path.

    Created collectively (every rank, after its GPU agent: see ``nccl_eager``); the
    unique id travels through ``all_gather_object`` once. The ranks then agree on the
    outcome: if any rank could not load RCCL or create its communicator, every rank
    raises ``NativeGatherUnavailable`` (the caller keeps torch's collective) instead of
    some ranks gathering on a communicator their peers do not have."""

    def __init__(self, aggregator: "NodeAggregator", device: torch.device, block_shape: tuple,
                 root_host: torch.Tensor | None = None):
        from ..runtime import native

        nat = native.load()
        lib = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        uid, err = None, None
        if aggregator.rank == 0:
            try:
                uid = nat.rccl_unique_id(lib)
            except Exception as e:  # noqa: BLE001 - reported to every rank below
                err = f"rank 0: {e}"
        uid = aggregator.all_gather_object(uid)[0]
        self.world_size = aggregator.world_size
        self.comm = None
        if uid is not None:
            try:
                self.comm = nat.RcclComm(device.index, aggregator.world_size, aggregator.rank, uid, lib)
            except Exception as e:  # noqa: BLE001
                err = f"rank {aggregator.rank}: {e}"
        errs = [e for e in aggregator.all_gather_object(err) if e]
        if errs:
            self.comm = None  # a communicator whose peers failed is never used
            raise NativeGatherUnavailable("; ".join(errs))
        self.out = torch.empty((aggregator.world_size,) + tuple(block_shape), dtype=torch.float32, device=device)
        # rank 0's node tensor as tagged words (the host copies the values out in wait());
        # ROCMDASH_TAGGED_OUT=0: copy + completion flag
        self.pub = nat.HostPublisher(device.index,
                                     tagged=os.environ.get("ROCMDASH_TAGGED_OUT", "1") not in ("0", "off", "false"))
        if root_host is not None and (root_host.numel() != self.out.numel() or not root_host.is_pinned()):
            raise ValueError("root_host must be a pinned tensor with the node tensor's size")
        self.host = root_host
        self.seq = 0

    def gather(self, local: torch.Tensor, stream: int) -> torch.Tensor:
        """Enqueue the gather of ``local`` (contiguous float32 of ``block_shape``) and
        the publication; returns the device node tensor (valid in stream order)."""
        if not local.is_contiguous() or local.numel() * self.world_size != self.out.numel():
            raise ValueError("local block does not match the node tensor")
        self.comm.all_gather(local.data_ptr(), self.out.data_ptr(), local.numel(), stream)
        if self.host is not None:
            self.seq = self.pub.publish(self.out.data_ptr(), self.host.data_ptr(), self.out.numel(), stream)
        else:
            self.seq = self.pub.publish(0, 0, 0, stream)
        return self.out

    def wait(self, timeout_s: float = 1.0) -> bool:
        """Spin until the last gather is published (rank 0: its node tensor is in the
        pinned buffer); False on timeout."""
        return bool(self.seq) and self.pub.wait(self.seq, timeout_s)
