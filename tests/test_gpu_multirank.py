"""The N > 1 native gather with several ranks on real MI355X hardware.

The pool's boxes have one GPU, so the ranks oversubscribe it (``ROCMDASH_OVERSUBSCRIBE``,
rocmdash.parallel.node.oversubscribed): every rank is its own process with its own HIP
context, sampler, device window and RCCL communicator, and RCCL connects the ranks
with its network transport instead of xGMI. What runs for real: ncclCommInitRank over N
ranks (non-blocking, bounded), RCCL's multi-rank all-gather kernels and proxies, the
publish kernel's root-only tagged hand-off and the non-root completion flags, the
start-up validation against the gloo control plane, the rank order of the node tensor,
the node-window gather, the bench's N > 1 code path (restart protocol, validated native
gather, deployed path), and the service's bounded failure path when a rank dies.
What does not: the xGMI links (the driver's 8-GPU SCALE run measures those)."""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    # NCCL_DEBUG unset: rocmdash points RCCL's INFO log at its own file to read the
    # transports (a caller's quieter NCCL_DEBUG would be respected: no transport record)
    env = dict(os.environ, ROCMDASH_OVERSUBSCRIBE="1", PYTHONPATH=ROOT)
    env.pop("NCCL_DEBUG", None)
    return env


def _torchrun(world, *args, max_restarts=0):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
            "--max-restarts", str(max_restarts), "--monitor-interval", "0.5",
            "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *args]


@pytest.mark.parametrize("world", [2, 4])
def test_native_gather_multirank_one_gpu(world):
    res = subprocess.run(_torchrun(world, "tools/multirank_check.py", "--refreshes", "30"), cwd=ROOT,
                         capture_output=True, text=True, timeout=240, env=_env())
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert res.returncode == 0 and lines, (res.stdout[-3000:], res.stderr[-4000:])
    d = json.loads(lines[-1])
    assert d["ok"] and d["world"] == world and d["oversubscribed"], d
    assert "ncclAllGather" in d["transport"] and d["gather_validated"] == 8, d
    assert d["node_window_ok"] is True, d
    # RCCL's own view: a communicator of `world` ranks, this rank's index, and the NET
    # transport (sockets) the oversubscribed ranks must use - on a real node it is P2P
    for r, v in enumerate(d["rccl_views"]):
        assert v["rccl_nranks"] == world and v["rccl_rank"] == r, d["rccl_views"]
        assert v["kinds"] and set(v["kinds"]) == {"NET"}, d["rccl_views"]
    st = d["stage_us_p50"]
    assert st["allgather"] > 0 and st["publish"] > 0 and st["stats_kernel"] > 0, st


def test_bench_multirank_one_gpu():
    """bench.py's N > 1 path with 2 ranks: parents' gloo group + restart protocol, the
    timed region on the validated native gather, the side run's HIP events, the deployed
    path run by both ranks; the line says it is a rehearsal, not a 2-GPU number."""
    res = subprocess.run(_torchrun(2, "bench.py", "--gpus", "2", "--steps", "100", "--warmup", "10", "--source",
                                   "synthetic", "--counters", "synthetic", "--timing-steps", "20", "--e2e-s", "2"),
                         cwd=ROOT, capture_output=True, text=True, timeout=300, env=_env())
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert res.returncode == 0 and len(lines) == 1, (res.stdout[-3000:], res.stderr[-4000:])
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and "NOT an 2-GPU measurement" in d["rehearsal"], d.get("rehearsal")
    assert d["gather"]["status"] == "native" and d["gather"]["validated"] == 8, d["gather"]
    assert "RCCL ncclAllGather (native) x2" in d["config"]["model"]
    assert d["device_us_p50"]["gather_validated"] == 8 and d["device_us_p50"]["allgather"] > 0
    assert d["deployed_path"]["error"] is None and d["deployed_path"]["gpus"] == 2, d["deployed_path"]
    assert d["value"] > 0 and d["p50_refresh_ms"] < 50


@pytest.mark.parametrize("world,window,full_cap", [(2, 1 << 20, False), (4, 1 << 20, False), (8, 1 << 18, True)])
def test_node_long_window_multirank_one_gpu(world, window, full_cap):
    """Node-wide statistics of long windows on every rank by the distributed radix select
    (LongWindowSet.refresh_node: predictions / partials all-gathered, digit histograms
    all-reduced over the native communicator) and node bracket mode, exact against the
    fp64 reference of the union of the ranks' windows on every rank, every node refresh.
    At 8 ranks (kNodeBrkRanks) the check ends with a node reset and a
    bracket refresh in which every rank keeps exactly kNodeCap = 1024 keys of each of one
    series' brackets: scan B selects among 8 x 1024 = 8192 keys, its LDS bound, and the
    records travel at the full cap."""
    args = ["tools/node_long_window_check.py", "--window", str(window)] + (["--full-cap", "--steady", "12"]
                                                                          if full_cap else [])
    res = subprocess.run(_torchrun(world, *args), cwd=ROOT, capture_output=True, text=True, timeout=420, env=_env())
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert res.returncode == 0 and lines, (res.stdout[-3000:], res.stderr[-4000:])
    d = json.loads(lines[-1])
    print(json.dumps({k: d[k] for k in ("world", "node_refreshes", "steady_node_refresh_ms_p50", "full_cap",
                                        "record_bytes_first_last")}))
    assert d["ok"] and d["world"] == world and d["window"] == window and d["node_refreshes"] >= 8, d
    assert all(v > 0 for v in d["collective_us_p50"].values()), d
    # after a bracket refresh the records all-gather ~2x the kept keys (lw_node_cap_next),
    # not kNodeCap per bracket: 12 series x (96 + 3 x 4 x cap) bytes
    first, last = d["record_bytes_first_last"]
    assert first == 12 * (96 + 12 * 1024), d
    if not full_cap:
        assert 0 < last <= 12 * (96 + 12 * 512), d
    else:
        fc = d["full_cap"]
        assert fc["node_cap"] == 1024 and fc["maxmid"] == 1024 and fc["hit"], fc
        assert fc["record_bytes"] == 12 * (96 + 12 * 1024) and fc["union_keys_per_bracket"] == world * 1024, fc


def test_bench_self_launches_ranks_one_gpu():
    """``--gpus 2`` with no launcher (the driver's N > 1 form without torchrun): the bench
    starts both ranks itself; the timed region gathers natively (validated 8/8) and every
    rank's record carries RCCL's view (2 ranks) and its transport (NET: oversubscribed)."""
    env = _env()
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "100", "--warmup", "10", "--source",
                          "synthetic", "--counters", "synthetic", "--timing-steps", "20", "--e2e-s", "1"],
                         cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert res.returncode == 0 and len(lines) == 1, (res.stdout[-3000:], res.stderr[-4000:])
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and len(d["ranks"]) == 2 and "rehearsal" in d, d.get("rehearsal")
    assert d["gather"]["status"] == "native" and d["gather"]["validated"] == 8, d["gather"]
    for r in d["ranks"]:
        assert r["rccl_nranks"] == 2 and r["rccl_rank"] == r["rank"], r
        assert r["transport_kinds"] and set(r["transport_kinds"]) == {"NET"}, r
    assert d["rccl"]["nranks_by_rank"] == [2, 2] and d["rccl"]["all_p2p"] is False, d["rccl"]
    assert d["cpu_seconds_per_s"] > 0 and d["production_fresh_per_s_per_gpu"] > 0


def test_bench_eight_ranks_one_gpu():
    """``--gpus 8`` with no launcher, 8 oversubscribed ranks: one JSON
    line, the timed region on the validated native gather, every rank's RCCL communicator
    of 8 ranks."""
    env = _env()
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--steps", "50", "--warmup", "5", "--source",
                          "synthetic", "--counters", "synthetic", "--timing-steps", "10", "--e2e-s", "1"],
                         cwd=ROOT, capture_output=True, text=True, timeout=420, env=env)
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert res.returncode == 0 and len(lines) == 1, (res.stdout[-3000:], res.stderr[-4000:])
    d = json.loads(lines[0])
    print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step", "p50_refresh_ms", "rccl", "gather")}))
    assert d["n_gpus"] == 8 and len(d["ranks"]) == 8 and "rehearsal" in d, d.get("rehearsal")
    assert d["gather"]["status"] == "native" and d["gather"]["validated"] == 8, d["gather"]
    assert d["rccl"]["nranks_by_rank"] == [8] * 8, d["rccl"]
    assert d["deployed_path"]["error"] is None and d["deployed_path"]["gpus"] == 8, d["deployed_path"]


def test_bench_slow_ranks_restart_alone_one_gpu():
    """4 oversubscribed ranks, no launcher: ranks 1 and 3 report the slow driver state on
    their first attempt. Only those two children start again - before any process group
    or RCCL communicator exists - and the 4-rank line gathers natively (validated 8/8)."""
    env = _env()
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR"):
        env.pop(k, None)
    env["ROCMDASH_BENCH_FAKE_SLOW"] = "1:0,3:0"
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "50", "--warmup", "5", "--source",
                          "synthetic", "--counters", "synthetic", "--timing-steps", "10", "--e2e-s", "0"],
                         cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert res.returncode == 0 and len(lines) == 1, (res.stdout[-3000:], res.stderr[-4000:])
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["startup_restarts_by_rank"] == [0, 1, 0, 1], d["startup_restarts_by_rank"]
    assert d["gather"]["status"] == "native" and d["gather"]["validated"] == 8, d["gather"]
    restarted = sorted({ln.split(":")[0] for ln in res.stderr.splitlines() if "starting attempt" in ln})
    assert restarted == ["[bench] rank 1", "[bench] rank 3"], restarted


def test_bench_refuses_more_gpus_than_visible():
    """``--gpus 8`` on a one-GPU box (not oversubscribed): non-zero exit, no JSON line."""
    env = {k: v for k, v in os.environ.items() if k not in ("ROCMDASH_OVERSUBSCRIBE", "WORLD_SIZE", "RANK")}
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--steps", "5"], cwd=ROOT, capture_output=True,
                         text=True, timeout=120, env=env)
    assert res.returncode != 0 and "GPU(s) visible" in res.stderr, (res.returncode, res.stderr[-2000:])
    assert not [ln for ln in res.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("fault", ["exit", "hang"])
def test_serve_native_gather_recovers_from_rank_loss(fault):
    """The service on the native gather, 2 ranks: rank 1 exits (or stops answering while
    staying alive) after 3 refreshes. Rank 0's ncclAllGather can never complete; the
    bounded wait (collective timeout) aborts its communicator and the service exits for
    a restart; torchrun starts both ranks again, which re-creates the communicator, and
    the second attempt finishes."""
    cmd = _torchrun(2, "-m", "rocmdash.serve", "--source", "synthetic", "--counters", "synthetic", "--port", "0",
                    "--refresh-hz", "20", "--max-refreshes", "8", "--collective-timeout", "10", "--node-window",
                    max_restarts=1)
    env = dict(_env(), ROCMDASH_FAULT=f"{fault}:1:3")
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-5000:]
    assert "fault injection: rank 1" in out
    assert "'status': 'native'" in out  # both attempts gathered natively
    assert "rank 0 stopped after 8 refreshes (exit 0)" in out, out[-5000:]


def test_launch_entrypoint_on_the_box():
    """The DaemonSet's entrypoint on the box: ``rocmdash.launch`` reads the node plan (one
    physical GPU here), supervises that many service ranks on live sources, and the
    service runs its refreshes and exits 0."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT",
                                                             "ROCMDASH_OVERSUBSCRIBE")}
    res = subprocess.run([sys.executable, "-m", "rocmdash.launch", f"--master-port={_free_port()}",
                          "-m", "rocmdash.serve", "--port", "0", "--refresh-hz", "10",
                          "--max-refreshes", "5", "--node-window"],
                         cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    out = res.stdout + res.stderr
    assert res.returncode == 0, out[-4000:]
    assert "[rocmdash.launch] supervising 1 rank(s) (partition mode SPX" in out, out[-3000:]
    assert "slot 0 stopped after 5 refreshes" in out, out[-3000:]


@pytest.mark.parametrize("fault,slots,window", [("exit", 3, 4096), ("hang", 3, 4096), ("hang", 8, 4096),
                                                  ("exit", 3, 1 << 16)])
def test_supervised_node_keeps_serving_on_native_gather(fault, slots, window, tmp_path):
    """Partial-node operation on the native RCCL gather: supervised ranks on the GPU
    (oversubscribed), GPU slot 1 dies / stops answering 30 refreshes into every attempt.
    The others are back on /metrics within 2 collective timeouts, on a fresh RCCL
    communicator without it; slot 1 is restarted, re-admitted (a full communicator again)
    and lost again, and the node never stops serving. 8 slots: the node's design size
    (VERDICT r05 item 3). A 2^16 window: node bracket mode of the long window
    (--node-window), whose node state every member resets at each epoch - a restarted
    rank and the survivors take the same collectives."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _supervisor_helpers import free_port, max_gap_s, outage_s, start_node, stop_node, watch

    T = 10.0
    port = free_port()
    env = {"ROCMDASH_OVERSUBSCRIBE": "1", "NCCL_DEBUG": "WARN", "ROCMDASH_FAULT": f"{fault}:1:30:always",
           "ROCMDASH_WINDOW": str(window)}
    p = start_node(slots, port, cpu=False, env=env, log_path=str(tmp_path / "node.log"),
                   serve_args=("--source", "synthetic", "--counters", "synthetic", "--refresh-hz", "10",
                               "--collective-timeout", str(T), "--node-window"))
    full = {str(i) for i in range(slots)}
    partial = full - {"1"}
    try:
        hist, codes = watch(port, lambda h: any(s["gpus"] == full for _, s in h)
                            and h[-1][1]["restarts"].get("1", 0) >= 2 and h[-1][1]["gpus"] == partial,
                            timeout=200 if slots <= 3 else 360)
    finally:
        rc = stop_node(p)
    log = (tmp_path / "node.log").read_text()
    gap = outage_s(hist, full, partial)
    assert gap is not None and gap < 2 * T, (gap, log[-4000:])
    assert max_gap_s(hist) < 2 * T, (max_gap_s(hist), log[-4000:])
    assert hist[-1][1]["up"] == {g: (0.0 if g == "1" else 1.0) for g in full}, hist[-1][1]
    assert set(codes) <= {200}, codes
    assert "gather native" in log, log[-4000:]  # every epoch re-created the RCCL communicator
    assert rc == 0, log[-4000:]
