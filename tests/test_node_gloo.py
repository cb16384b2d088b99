"""Multi-rank node aggregation on the CPU (gloo): the same NodeAggregator /
NodePipeline code the GPUs run over RCCL, at world sizes 2, 4 and 8, plus bench.py
under torch.distributed.run with 2 ranks."""

import json
import os
import socket
import subprocess
import sys

import pytest

from rocmdash.viz.panels import EXTENDED_PANELS
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import numpy as np
        import torch

        from rocmdash.config import SamplerConfig
        from rocmdash.parallel.node import NodeAggregator, dist_env_from_environ
        from rocmdash.runtime.agent import GpuAgent
        from rocmdash.runtime.pipeline import NodePipeline

        env = dist_env_from_environ(prefer_gpu=False)
        assert env.world_size == world and env.backend == "gloo"
        agg = NodeAggregator()
        x = torch.full((12, 8), float(rank))
        out = agg.all_gather(x)
        assert out.shape == (world, 12, 8)
        assert all(float(out[r, 0, 0]) == r for r in range(world))
        objs = agg.all_gather_object({"rank": rank})
        assert [o["rank"] for o in objs] == list(range(world))
        assert agg.max_over_ranks(rank) == world - 1

        agent = GpuAgent(rank, source="synthetic", counters="synthetic",
                         cfg=SamplerConfig(window=64, ring_capacity=256), use_gpu=False)
        agent.prefill(64)
        pipe = NodePipeline(agent, agg, extended=True)
        payload, _ = pipe.step()
        res = None
        if rank == 0:
            d = json.loads(payload)
            res = {"figures": len(d["figures"]), "gpus": sorted(d["window"]["gpus"])}
            # rank r's own stats arrive at rank 0 unchanged
            node = pipe.gather()
            local = agent.refresh()
            np.testing.assert_allclose(node[0].numpy(), local.numpy())
        else:
            assert payload is None
            pipe.gather()
        # per-rank health rows ride in the same gather: rank 0 sees every rank's sources
        hp = NodePipeline(agent, agg, health=True)
        snap = hp.latest_snapshot()
        if rank == 0:
            st = snap.source_health.statuses()
            assert sorted({s.gpu for s in st}) == list(range(world))
            assert all(s.samples >= 64 for s in st), [(s.gpu, s.kind, s.samples) for s in st]
            assert snap.window.shape == (world, len(agent.series), 8)
        else:
            assert snap is None
        # ... and so do the per-XCD detail and the stop votes: every rank learns from the
        # one gather that the last rank wants to stop
        hp.stop_vote = 1.0 if rank == world - 1 else 0.0
        snap = hp.latest_snapshot()
        votes = hp.stop_votes()
        assert votes.tolist() == [0.0] * (world - 1) + [1.0], votes
        if rank == 0:
            assert snap.xcd is not None and snap.xcd.shape == (world, 2, 8)
            assert np.isfinite(snap.xcd[:, 0, 0]).all()  # the synthetic SMU source models XCDs
        # stage timing (serve.py exports it): both stages timed on every rank
        timed = NodePipeline(agent, agg, device_timing=True)
        timed.gather()
        st = timed.stage_seconds()
        assert set(st) == {"stats_kernel", "allgather"} and min(st.values()) >= 0, st
        # node-wide window statistics: rank 0's result is the statistics of the union of
        # every rank's window
        from rocmdash.parallel.node_window import NodeWindowStats, node_window_reference

        nws = NodeWindowStats(agent, agg)
        agent.refresh()
        got = nws.refresh()
        blocks = agg.all_gather_object(agent.export_window().numpy())
        if rank == 0:
            ref = node_window_reference(np.stack(blocks))
            np.testing.assert_allclose(got.numpy(), ref, rtol=1e-6, atol=1e-5)
            assert got[0, 7] == sum(b[0, 0] for b in blocks)
        else:
            assert got is None
        agg.barrier()
        import torch.distributed as dist

        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, "err", traceback.format_exc() + repr(e)))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_node_pipeline_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    errs = [r for r in results if r[1] != "ok"]
    assert not errs, errs
    root = [r for r in results if r[0] == 0][0][2]
    assert root["figures"] == 4 + (4 + len(EXTENDED_PANELS)) * world  # extended: + MFMA, HBM r/w, xGMI r/w per GPU
    assert root["gpus"] == [str(r) for r in range(world)]


@pytest.mark.parametrize("world", [2, 4])
def test_bench_cpu_torchrun(world):
    """bench.py's driver contract under torch.distributed.run (gloo on CPU): one JSON
    line from rank 0, n_gpus = world size, 4 + 4N figures per refresh."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world), "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", str(world), "--steps", "20", "--warmup", "2",
           "--cpu", "--window", "256", "--e2e-s", "2"]
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout  # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == 20 and d["config"]["figures_per_refresh"] == 4 + 4 * world
    assert d["config"]["parallelism"].startswith(f"rank-per-GPU x{world}")
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert 0 < d["value"] <= d["hardware_reads_per_s"] * 1.05  # fresh <= raw (+1 prefetched row of slack)
    dev = d["device_us_p50"]  # the side run: stats + gloo all-gather on every rank
    assert dev["stats_kernel"] > 0 and dev["allgather"] > 0 and "gloo all_gather" in dev["gather"], dev
    assert f"gloo all_gather x{world}" in d["config"]["model"]
    # the deployed path ran on every rank: rank 0's page saw every GPU through Prometheus
    dep = d["deployed_path"]
    assert dep["error"] is None and dep["gpus"] == world and d["prometheus_page_p50_ms"] > 0, dep
    assert set(d["display_age_p50_ms"]) == {"smi", "counter"}, d["display_age_p50_ms"]


@pytest.mark.parametrize("fault,world,extra", [("exit", 2, ()), ("hang", 2, ()), ("exit", 8, ("--node-window",))])
def test_serve_recovers_from_rank_loss(fault, world, extra):
    """Fault injection: rank 1 dies (or stops answering) after 3 refreshes. The
    collective timeout ends rank 0's all-gather, the service exits for a restart and
    torchrun (--max-restarts) re-creates the group - the second attempt runs its 8
    refreshes to completion. The 8-rank case runs the DaemonSet's shape: one rank per
    GPU of a full node, node-wide window statistics on."""
    port = _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--max-restarts", "1",
           "--monitor-interval", "0.5", "--master-addr", "127.0.0.1", "--master-port", str(port),
           "-m", "rocmdash.serve", "--cpu", "--source", "synthetic", "--counters", "synthetic", "--port", "0",
           "--refresh-hz", "20", "--max-refreshes", "8", "--collective-timeout", "8" if world == 2 else "20",
           *extra]
    env = dict(os.environ, ROCMDASH_FAULT=f"{fault}:1:3", PYTHONPATH=ROOT)
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-4000:]
    assert "fault injection: rank 1" in out
    assert "rank 0 stopped after 8 refreshes (exit 0)" in out, out[-4000:]


def _world1_worker(port, q):
    """World 1 with a forced collective: every call issues the real gloo collective."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    try:
        import torch

        from rocmdash.parallel.node import NodeAggregator, dist_env_from_environ

        env = dist_env_from_environ(prefer_gpu=False, world1_group=True)
        assert env.initialized_here and env.world_size == 1
        agg = NodeAggregator(force_collective=True)
        x = torch.arange(16.0).view(2, 8)
        out = agg.all_gather(x)
        assert out.shape == (1, 2, 8) and torch.equal(out[0], x) and out.data_ptr() != x.data_ptr()
        agg.barrier()
        assert agg.max_over_ranks(3.5) == 3.5 and agg.sum_over_ranks(2.0) == 2.0
        assert agg.collectives == 4
        plain = NodeAggregator(force_collective=False)
        assert plain.all_gather(x).data_ptr() == x.data_ptr() and plain.collectives == 0
        import torch.distributed as dist

        dist.destroy_process_group()
        q.put("ok")
    except Exception as e:  # pragma: no cover
        import traceback

        q.put(traceback.format_exc() + repr(e))


def test_forced_collective_world1_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_world1_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=120)
    p.join(timeout=60)
    assert res == "ok", res


def test_force_collective_needs_a_group():
    from rocmdash.parallel.node import NodeAggregator

    with pytest.raises(RuntimeError):
        NodeAggregator(force_collective=True)


def _native_gather_worker(rank, world, port, fail, q):
    """The native transport's set-up agreement over gloo, RCCL replaced by a fake. Three
    agreed steps (load, unique id, init): when one rank cannot load RCCL, NO rank enters
    the (collective) communicator init; when the unique id (rank 0) or one rank's
    communicator fails, EVERY rank gives up and aborts what it created; when all
    succeed, every rank keeps its communicator."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import torch

        from rocmdash.parallel import node as node_mod
        from rocmdash.runtime import native

        inits, aborts = [], []

        class FakeNative:
            @staticmethod
            def rccl_load(lib):
                if fail == "load" and rank == 1:
                    raise RuntimeError("RCCL not loadable (librccl.so.1)")
                return 22606

            @staticmethod
            def rccl_unique_id(lib):
                if fail == "uid":
                    raise RuntimeError("ncclGetUniqueId: unhandled system error")
                return b"\x01" * 128

            class RcclComm:
                def __init__(self, dev, n, r, uid, lib, timeout_s):
                    assert n == world and r == rank and len(uid) == 128 and timeout_s > 0
                    inits.append(r)
                    if fail == "comm" and r == world - 1:
                        raise RuntimeError("ncclCommInitRank: not every rank joined within 120 s")

                def abort(self):
                    aborts.append(rank)

        native.load = lambda: FakeNative  # this spawned process only
        node_mod.dist_env_from_environ(prefer_gpu=False)
        agg = node_mod.NodeAggregator()
        ok = agg.enable_native(torch.device("cpu", 0))
        res = ("ok", ok and agg.native is not None) if ok else ("unavailable", agg.native_error)
        import torch.distributed as dist

        dist.destroy_process_group()
        q.put((rank, "ok", res, inits, aborts))
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, "err", traceback.format_exc() + repr(e), [], []))


@pytest.mark.parametrize("fail", ["none", "load", "uid", "comm"])
def test_native_gather_setup_agreement(fail):
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_gather_worker, args=(r, world, port, fail, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in results), results
    outcomes = [r[2] for r in results]
    if fail == "none":
        assert outcomes == [("ok", True)] * world
        return
    assert all(o[0] == "unavailable" for o in outcomes), outcomes
    want = {"load": "rank 1: RCCL not loadable", "uid": "rank 0: ncclGetUniqueId",
            "comm": f"rank {world - 1}: ncclCommInitRank"}[fail]
    assert all(want in o[1] for o in outcomes), outcomes
    inits = [r[3] for r in results]
    aborts = [r[4] for r in results]
    if fail in ("load", "uid"):
        assert inits == [[]] * world  # nobody entered the collective init
    else:  # every rank that created a communicator aborts it
        assert inits == [[r] for r in range(world)] and aborts == [[r] for r in range(world - 1)] + [[]]


class _GlooStandInTransport:
    """Stand-in for RcclTransport on the CPU: the data plane's all-gather over gloo, and
    a publisher that copies the gathered tensor into the root's host buffer (ctypes
    memmove) - so NativeNodeGather.gather/wait and NodePipeline._to_host /
    _sync_gathered / _validate run their multi-rank bookkeeping for real."""

    kind = "gloo-stand-in"

    def __init__(self, device, corrupt_rank=None):
        self.device = device
        self.corrupt_rank = corrupt_rank
        self.closed = False
        self.gathers = 0
        self.publishers = []

    def all_gather(self, local, out, stream):
        import torch.distributed as dist

        dist.all_gather(list(out.unbind(0)), local)
        self.gathers += 1
        if self.corrupt_rank is not None and dist.get_rank() == self.corrupt_rank and self.gathers == 3:
            out.view(-1)[5] += 1.0  # one flipped value on one rank, third gather

    def publisher(self, tagged):
        import ctypes

        class Pub:
            def __init__(self):
                self.seq = 0
                self.copied = []  # n of every publication

            def publish(self, src, dst, n, stream):
                if n:
                    ctypes.memmove(dst, src, 4 * n)
                self.copied.append(n)
                self.seq += 1
                return self.seq

            def wait(self, seq, timeout_s=1.0):
                return 0 < seq <= self.seq

        p = Pub()
        self.publishers.append(p)
        return p

    def healthy(self):
        return not self.closed

    def describe(self):
        return "gloo stand-in"

    def close(self):
        self.closed = True


def _native_bookkeeping_worker(rank, world, port, corrupt, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), ROCMDASH_GATHER_VALIDATE="4")
    try:
        import numpy as np
        import torch

        from rocmdash.config import SamplerConfig
        from rocmdash.parallel.node import NodeAggregator, dist_env_from_environ
        from rocmdash.runtime import pipeline as pl
        from rocmdash.runtime.agent import GpuAgent

        pl._VALIDATE = 4
        dist_env_from_environ(prefer_gpu=False)
        agg = NodeAggregator()
        tr = _GlooStandInTransport(torch.device("cpu"), corrupt_rank=(world - 1) if corrupt else None)
        assert agg.enable_native(torch.device("cpu"), factory=lambda a, d: tr)
        agent = GpuAgent(rank, source="synthetic", counters="synthetic",
                         cfg=SamplerConfig(window=64, ring_capacity=256), use_gpu=False, seed=100 + rank)
        agent.prefill(64)
        # the root's pinned buffer stand-in: NodePipeline keeps _host only on GPUs
        pipe = pl.NodePipeline(agent, agg, health=True, native_gather=True)
        assert pipe._ng is not None and pipe.gather_status == "native"
        root_host = torch.empty((world, pipe.rows, 8), dtype=torch.float32) if rank == 0 else None
        pipe._host = root_host
        pipe._ng.host = root_host
        S = len(agent.series)
        statuses = []
        for i in range(8):
            agent.sample()
            snap = pipe.latest_snapshot()
            own = agent.refresh().numpy()  # same window: this rank's own stats again
            blocks = agg.all_gather_object(own)
            if rank == 0:
                # rank order: block r of the node tensor is rank r's own statistics
                np.testing.assert_array_equal(snap.window, np.stack(blocks), err_msg=f"refresh {i}")
                assert snap.source_health is not None and len(snap.source_health.statuses()) == 2 * world
            else:
                assert snap is None
            assert pipe.stop_votes().tolist() == [0.0] * world
            statuses.append(pipe.gather_status)
        pubs = tr.publishers[0].copied
        # the root publishes the node tensor every native gather, the others only signal
        if rank == 0:
            assert all(n == world * pipe.rows * 8 for n in pubs), pubs
        else:
            assert all(n == 0 for n in pubs), pubs
        res = {"statuses": statuses, "validated": pipe._ng.validated if pipe._ng is not None else None,
               "closed": tr.closed, "publications": len(pubs)}
        import torch.distributed as dist

        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, "err", traceback.format_exc() + repr(e)))


@pytest.mark.parametrize("world,corrupt", [(2, False), (4, False), (8, False), (4, True)])
def test_native_gather_bookkeeping_gloo(world, corrupt):
    """NativeNodeGather's multi-rank bookkeeping on a gloo stand-in of the RCCL
    transport, at 2/4/8 ranks: rank order of the node tensor, the root-only
    publication, the non-root completion waits, the stop votes, and the start-up
    validation (4 gathers checked bit for bit against the control plane). With one
    value flipped on the last rank's third gather, EVERY rank drops the native path at
    that refresh together and the node tensor stays right."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_bookkeeping_worker, args=(r, world, port, corrupt, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in results), results
    res = [r[2] for r in results]
    if not corrupt:
        assert all(r["statuses"] == ["native"] * 8 and r["validated"] == 4 and not r["closed"] for r in res), res
        assert all(r["publications"] == 8 for r in res), res
    else:
        want = ["native"] * 2 + ["host (native gather failed validation)"] * 6
        assert all(r["statuses"] == want and r["validated"] is None and r["closed"] for r in res), res
        assert all(r["publications"] == 3 for r in res), res


def test_superseded_publication_fails_fast():
    """A publication a newer one overwrote before it was read is a hand-off error, not a
    slow peer: the bounded wait raises at once, without aborting the communicator
    (ADVICE r03); a publication that never arrives still times out and aborts."""
    import time

    import pytest

    from rocmdash.parallel.node import PublicationSuperseded, await_publication

    class Pub:
        superseded = 0

        def wait(self, seq, timeout_s):
            self.superseded = 1  # a newer publication overwrote the tagged words
            return False

    class Tr:
        closed = False

        def healthy(self):
            return True

        def close(self):
            self.closed = True

    tr = Tr()
    t0 = time.monotonic()
    with pytest.raises(PublicationSuperseded):
        await_publication(Pub(), 3, tr, timeout_s=30.0)
    assert time.monotonic() - t0 < 5.0 and not tr.closed

    class Never:
        def wait(self, seq, timeout_s):
            time.sleep(min(timeout_s, 0.01))
            return False

    with pytest.raises(RuntimeError, match="not complete"):
        await_publication(Never(), 3, tr, timeout_s=0.1)
    assert tr.closed
