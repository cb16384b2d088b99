#!/usr/bin/env python3
"""Headline benchmark: metric samples/s + p50 dashboard refresh latency, 1..8 MI355X.

BASELINE.json metric: "metric samples/sec/GPU + p50 dashboard refresh latency at
1/2/4/8 MI355X". One *step* is one full dashboard refresh of the node, the same work
BASELINE.md times on the reference (fetch + aggregate + build all 4 + 4N figures +
serialise), minus the reference's 5 s sleep:

  every rank (one process per GPU):
    its GPU's sources (amd-smi: 11 series, rocprofiler-sdk device counters: 5 series)
      read back to back on their own native threads (--sampling free, the default) into
      pinned SPSC rings; the refresh waits until every source has at least one new row
      -> window-stats kernel over the last W = 4096 samples of every series
      (min/max/mean/p50/p90/p99/last/count) including every row that arrived, pulling
      the entering rows straight from the mapped ring. No rank's reads wait for the
      node's refresh, so at N > 1 the node does not run at the pace of its slowest
      rank's read tail (tools/probes/probe_lockstep_tail.py: a lockstep 8-rank refresh
      would lose 10 % on a quiet box, half in a tail phase); --sampling closed takes
      exactly one (prefetched) read per source per refresh instead
    -> N > 1: ONE native ncclAllGather (RCCL over xGMI, rocmdash's own communicator; the
       gloo process group is the control plane only) of the [S, 8] stats -> [N, S, 8]
       node tensor, and the publish kernel hands it to rank 0's pinned buffer; the first
       gathers are validated bit for bit against the control plane (``gather``);
       N = 1 (default --gather auto): the gather is the identity and the stats kernel
       writes rank 0's pinned host buffer directly (--gather rccl runs the one-rank
       native RCCL all-gather instead)
  rank 0: node snapshot, averages, 4 + 4N gauge figures + stats/window tables, JSON
    payload (what the browser receives).

``value`` = FRESH metric samples per second that went through the whole pipeline onto
the dashboard, summed over all N GPUs. A value counts when it carries new data
(``GpuAgent.fresh_samples``): every device-counter row (each a new counter delta) x 5
series, every amd-smi row's live used-VRAM column, and the 9 SMU-table series once per
table the firmware actually published (most back-to-back reads return the previous
table); failed reads push no row and count nothing. ``hardware_reads_per_s`` keeps
the raw count (every series of every completed read). The reference ingests 5 series
per GPU per 5 s refresh (<= 1.0 sample/s/GPU), so ``vs_baseline`` =
value / (N * 1.0). ``p50_refresh_ms`` (from the start of the oldest source's newest read
to the frame payload) is compared with the reference's measured p50 full-refresh latency
at the same N. After the timed region an untimed
side run of ``--timing-steps`` refreshes records HIP events around the stats kernel,
the native ncclAllGather and the publish kernel - the same native path the timed region
runs at N > 1 and the node service runs (one-rank communicator at N = 1):
``device_us_p50``. Then ``--e2e-s`` seconds of the DEPLOYED path, run collectively by the
job's own ranks at production sampling rates (rocmdash/runtime/deployed.py): service
refresh -> /metrics -> mini-Prometheus -> the page's queries -> frame, reported as
``prometheus_page_p50_ms`` and ``display_age_p50_ms`` (the path users see).

Process layout: the process the launcher starts for a rank never touches the GPU; it
runs the measurement in a child process. A child that finds its device-counter reads
in the slow driver state after prefill (~140 instead of ~80 us: fixed for a process's
life when its HSA runtime starts) reports it BEFORE any process group or communicator
exists; the rank processes (a gloo group at N > 1) agree, and only the slow ranks start a
fresh child, at most --restarts times each, while the others wait with their agents up:
the node refresh is paced by its slowest GPU, and at 8 ranks restarting every rank would
rarely end all fast. The JSON line reports ``startup_restarts`` (per rank in
``startup_restarts_by_rank`` / ``ranks[].attempt``).

Run: python bench.py [--gpus N --steps K --warmup W]. For N > 1 either under
torch.distributed.run (one rank per GPU, RCCL), or without a launcher: the process then
starts the N rank processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT, as the launcher would set them; it never touches the GPU) and exits with the
first failing rank's code. Fewer than N visible GPUs is an error (unless
ROCMDASH_OVERSUBSCRIBE=1, a labelled rehearsal), and so is a --gpus that disagrees with
the launcher's WORLD_SIZE: the line never reports a node size it did not run.
At N > 1 every rank's record carries RCCL's own view of the communicator
(ncclCommCount / ncclCommUserRank) and the transport RCCL logged per peer; on a real node
(not oversubscribed) a peer connection that is not P2P (xGMI) fails the run.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

# reference p50 / p90 full-refresh latency (ms) at N = 1, 2, 4, 8
REF_P50_MS = {1: 39.95, 2: 56.04, 4: 85.97, 8: 154.53}
REF_SAMPLES_PER_S_PER_GPU = 1.0
METRIC = "metric samples/sec/GPU + p50 dashboard refresh latency at 1/2/4/8 MI355X"


def _interp_ref(n: int) -> float:
    if n in REF_P50_MS:
        return REF_P50_MS[n]
    ks = sorted(REF_P50_MS)
    lo = max([k for k in ks if k <= n], default=ks[0])
    hi = min([k for k in ks if k >= n], default=ks[-1])
    if lo == hi:
        return REF_P50_MS[lo]
    return REF_P50_MS[lo] + (REF_P50_MS[hi] - REF_P50_MS[lo]) * (n - lo) / (hi - lo)


def _placement_report():
    """NUMA node the runtime was started on and the per-node counter-read calibration
    (rocmdash/runtime/placement.py), or None."""
    from rocmdash.runtime.placement import choice

    c = choice()
    return None if c is None else {k: c.get(k) for k in ("node", "p50_us", "source", "calibration_s", "gpus_calibrated",
                                                         "lock_wait_s", "slow_rounds", "slow") if k in c}


def agg_possible() -> bool:
    import torch.distributed as dist

    return dist.is_available() and dist.is_initialized()


def _series_read(c0: dict, c1: dict) -> int:
    """Series values in the rows the sources pushed between two ``sample_counts()``."""
    from rocmdash.models.schema import CTR_FIELDS, SMI_FIELDS

    return int((c1.get("counter_rows", 0) - c0.get("counter_rows", 0)) * len(CTR_FIELDS)
               + (c1.get("smi_rows", 0) - c0.get("smi_rows", 0)) * len(SMI_FIELDS))


def _values_read(agent, c0: dict, c1: dict, s0: dict, s1: dict) -> int:
    """Values the sources read from the hardware between two snapshots (bench JSON)."""
    from rocmdash.models.schema import CTR_FIELDS, SMI_LIVE_FIELDS, SMI_TABLE_FIELDS

    n = (c1.get("counter_rows", 0) - c0.get("counter_rows", 0)) * len(CTR_FIELDS)
    smi_rows = c1.get("smi_rows", 0) - c0.get("smi_rows", 0)
    n += smi_rows * len(SMI_LIVE_FIELDS)
    table = s1.get("raw_reads", 0) - s0.get("raw_reads", 0) if "raw_reads" in s1 and s1.get("raw_reads") else smi_rows
    return int(n + table * len(SMI_TABLE_FIELDS))


def _gather_desc(pipe, agg) -> str:
    if pipe.host_out:
        return "identity gather (world 1: stats kernel writes pinned host memory, no collective)"
    if getattr(pipe, "_ng", None) is not None:
        kind = getattr(agg.native, "kind", "rccl")
        if kind != "rccl":
            return f"{kind} all_gather x{agg.world_size} (stand-in transport) + publish"
        return f"RCCL ncclAllGather (native) x{agg.world_size} on the stats stream + publish kernel"
    if agg.collective:
        if agg.backend == "nccl":
            return f"RCCL all_gather_into_tensor x{agg.world_size} (torch)"
        return f"{agg.backend} all_gather x{agg.world_size} through host memory (control plane)"
    return "identity gather (world 1)"


def _device_timing(agent, env, agg0, args):
    """Untimed side run: HIP events around the stats kernel, the native ncclAllGather
    and the publish kernel of ``--timing-steps`` refreshes (same agent, same 16-series
    window, counters live) - the node service's path. At N > 1 it reuses the timed
    region's aggregator (its one RCCL communicator); at N = 1 the gather is a one-rank
    native RCCL all-gather (the timed region's identity gather has nothing to time).
    Returns (rank 0's p50 in µs per stage - host clocks on the CPU path -, the
    aggregator used)."""
    import statistics

    import torch

    from rocmdash.parallel.node import NodeAggregator
    from rocmdash.runtime.pipeline import NodePipeline

    agent.wait_sample()  # the timed pipeline's prefetched sample, if one is pending
    agg = agg0 if agg0.collective else NodeAggregator(force_collective=agg_possible())
    pipe = NodePipeline(agent, agg, device_timing=True, allow_host_out=False)
    pipe.prevalidate()
    st = {}
    for _ in range(args.timing_steps):
        pipe.step(render=False)
        if env.device.type == "cuda":
            torch.cuda.synchronize(env.device)
        for k, v in pipe.stage_seconds().items():
            st.setdefault(k, []).append(v * 1e6)
    out = {k: round(statistics.median(v), 2) for k, v in st.items()}
    out["gather"] = _gather_desc(pipe, agg)
    out["gather_validated"] = pipe.gather_report()["validated"]
    out["collectives_issued"] = agg.collectives
    return out, agg


EXIT_SLOW_STATE = 75  # child: the device-counter reads came up in the slow driver state


SMI_FAST_US = 65.0  # SMU table read: 45-53 us steady on every box, 78-97 us in the start-up slow phase


def _settle(agent, args) -> float:
    """Right after a box comes up its driver reads can all run slow for some seconds
    (SMU table ~80-100 us, counters ~100-120 us; profiles/r02/fresh_box/): a monitoring
    service runs for days, so the measurement should not start inside that transient.
    Keep sampling (more prefill rows) while the last 1024 reads of either source are
    slow, at most --settle-s seconds; returns the time spent (reported as settle_s)."""
    if args.settle_s <= 0 or agent.ctr_sampler is None or agent.info.counter_backend != "rocprofiler":
        return 0.0
    from rocmdash.runtime.placement import choice, fast_reference_us

    # relative to this GPU's calibrated read of the configured counter set (placement.py);
    # without a calibration only the SMU-table read is waited for
    fast = fast_reference_us(choice())
    ctr_ref = 1.15 * fast if fast else float("inf")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.settle_s:
        smi, ctr = (s["p50_us"] for s in agent.sampler_stats()[:2])
        if ctr <= ctr_ref and smi <= SMI_FAST_US:
            break
        agent.prefill(1024)
    return time.perf_counter() - t0


def _node_window_mode(nws, lw_set) -> str:
    if not nws.long:
        return "sorted windows all-gathered + rank selection"
    if lw_set is not None and lw_set.brackets and lw_set.incremental:
        return ("node bracket mode (one all-gather of every rank's bracket records per refresh), "
                "distributed radix select for the series a bracket misses")
    return "distributed radix select"


def _node_window_tail(ms: list, kinds: list) -> dict | None:
    """p50 / p90 / p99 of the node refreshes, and the same for hits and misses apart."""
    if not ms:
        return None

    def pct(v):
        v = sorted(v)
        if not v:
            return None
        at = lambda q: v[min(len(v) - 1, int(q * len(v)))]  # noqa: E731
        return {"n": len(v), "p50": round(statistics.median(v), 4), "p90": round(at(0.9), 4),
                "p99": round(at(0.99), 4), "max": round(v[-1], 4)}

    out = {"all": pct(ms)}
    if kinds:
        for k in ("hit", "chain", "other"):
            sel = [m for m, kk in zip(ms, kinds) if kk == k]
            if sel:
                out[k] = pct(sel)
        out["chain_refreshes"] = sum(1 for k in kinds if k == "chain")
        out["chain_at"] = [i for i, k in enumerate(kinds) if k == "chain"][:50]
    return out


def _fake_slow(rank: int, attempt: str) -> bool:
    """``ROCMDASH_BENCH_FAKE_SLOW=<rank>:<attempt>[,<rank>:<attempt>...]`` (tests): these
    (rank, attempt) children report the slow state on purpose."""
    spec = os.environ.get("ROCMDASH_BENCH_FAKE_SLOW", "")
    pairs = {tuple(p.strip().split(":")) for p in spec.split(",") if p.strip()}
    return (str(rank), str(attempt)) in pairs


def _slow_state(agent, args) -> dict | None:
    """After prefill: the counter reads' p50 against the placement calibration's fast
    node (rocmdash/runtime/placement.py). A process keeps the read cost it got when the
    HSA runtime started, and a start can land in the slow state (~140 vs ~78 us,
    profiles/r01/probe_state.txt, profiles/r02/bench_restart_reps.txt) despite the NUMA
    placement. Returns {"counter_p50_us", "fast_p50_us"} when this one did, else None.
    ``ROCMDASH_BENCH_FAKE_SLOW`` reports it on purpose (tests, ``_fake_slow``)."""
    if os.environ.get("ROCMDASH_BENCH_FAKE_SLOW", ""):
        if _fake_slow(int(os.environ.get("RANK", "0")), os.environ.get("ROCMDASH_BENCH_ATTEMPT", "0")):
            return {"counter_p50_us": None, "fast_p50_us": None, "fake": True}
        return None
    from rocmdash.runtime.placement import choice, fast_reference_us

    c = choice() or {}
    fast = fast_reference_us(c)
    if not fast or c.get("slow") or agent.ctr_sampler is None or agent.info.counter_backend != "rocprofiler":
        # no reference, or one taken in a transient phase (placement.py: no round separated
        # the NUMA nodes) - a restart decision against it would be a coin flip
        return None
    # relative: the slow start reads ~1.7-1.9x this GPU's calibrated read of the same
    # counter set, the fast one ~1.0x (profiles/r06/counter_ab/)
    p50 = agent.ctr_sampler.stats()["p50_us"]
    return {"counter_p50_us": round(p50, 1), "fast_p50_us": fast} if p50 > args.slow_factor * fast else None


def _parents_group(world: int, rank: int):
    """World > 1: the launcher's processes (which never touch the GPU) form a gloo group
    of their own on the launcher's store, to agree on restarting their children."""
    if world == 1:
        return None
    from datetime import timedelta

    import torch.distributed as dist

    agent_store = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
    base = dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ.get("MASTER_PORT", "29500")), world,
                         is_master=rank == 0 and not agent_store, timeout=timedelta(seconds=600),
                         wait_for_workers=False)
    dist.init_process_group("gloo", store=dist.PrefixStore("rocmdash/bench-parents/", base), rank=rank,
                            world_size=world, timeout=timedelta(seconds=600))
    # the children use the same store as clients (keys prefixed per attempt,
    # rocmdash.parallel.node._restart_store), whoever hosts it
    return base


def _start_child(args_list, attempt: int, last: bool, store):
    """One measurement child of this rank: (Popen, verdict reader, decision writer)."""
    import subprocess

    r_v, w_v = os.pipe()  # child -> parent: verdict
    r_d, w_d = os.pipe()  # parent -> child: decision
    env = dict(os.environ, ROCMDASH_BENCH_CHILD="1", ROCMDASH_BENCH_ATTEMPT=str(attempt),
               ROCMDASH_BENCH_LAST="1" if last else "0", ROCMDASH_BENCH_VERDICT_FD=str(w_v),
               ROCMDASH_BENCH_DECISION_FD=str(r_d))
    if store is not None:
        env["TORCHELASTIC_USE_AGENT_STORE"] = "True"  # rank 0's parent or the launcher hosts it
    p = subprocess.Popen([sys.executable, os.path.abspath(__file__), *args_list], env=env, pass_fds=(w_v, r_d))
    os.close(w_v)
    os.close(r_d)
    return p, os.fdopen(r_v, "r"), os.fdopen(w_d, "w")


def restart_plan(codes: list, attempts: list, budget: int) -> tuple:
    """The parents' decision for one start-up round, from every rank's verdict code (0 ok,
    1 slow state, 2 died before its verdict) and restarts so far: ("abort", []) when any
    child died; ("restart", ranks) - ONLY the slow ranks that still have restarts left -
    while there are any; else ("go", []) (a slow rank out of restarts measures slow, and
    the line says so)."""
    if any(c == 2 for c in codes):
        return "abort", []
    again = [r for r, c in enumerate(codes) if c == 1 and attempts[r] < budget]
    return ("restart", again) if again else ("go", [])


def _run_with_restarts(argv) -> int:
    """Run the measurement in a child process per rank and start a rank's child again
    (at most --restarts times per rank) when ITS counter reads came up in the slow driver
    state: the node refresh is paced by its slowest GPU, so one slow rank would slow all
    of them. Only the slow ranks' children start again - the other children wait with
    their agents up - and the verdict is taken after prefill, BEFORE any child forms the
    process group or the RCCL communicator, so no group has to be torn down (VERDICT r04
    weak 4: at 8 ranks P(all fast) per whole-node attempt is ~0.8^8). This process never
    touches the GPU, so starting children is safe.

    Protocol: each child writes "ok" / "slow" to a pipe after its prefill; the parents
    all-gather the codes (gloo, world > 1) and decide (``restart_plan``); a child to
    restart reads "restart" and exits, its parent starts the next attempt; when nobody is
    left to restart every child reads "go <round>" (the round keys the children's
    process group on the launcher's store) or "abort". Rank 0's child hands its line to
    this process (ROCMDASH_BENCH_LINE_FILE), which prints it once every child has exited
    (``_print_final_line``)."""
    args_list = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--restarts", type=int, default=2)
    ap.add_argument("--production-s", type=float, default=10.0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--cpu", action="store_true")
    known, _ = ap.parse_known_args(args_list)
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    store = _parents_group(world, rank)
    line_file = None
    if rank == 0:
        import tempfile

        fd, line_file = tempfile.mkstemp(prefix="rocmdash-bench-line-", suffix=".json")
        os.close(fd)
        os.environ["ROCMDASH_BENCH_LINE_FILE"] = line_file  # every child attempt of rank 0 inherits it
    try:
        rc = _restart_rounds(args_list, known, world, rank, store)
        if store is not None:
            import torch.distributed as dist

            dist.barrier()  # every rank's child has exited: the GPUs are free
        if rank == 0:
            _print_final_line(line_file, rc, known, world)
        return rc
    finally:
        if line_file:
            try:
                os.unlink(line_file)
            except OSError:
                pass


def _print_final_line(line_file, rc: int, known, world: int) -> None:
    """Rank 0's parent: the measurement's line, plus (GPU runs, --production-s > 0) the
    production node service measured on the same GPUs after every measurement child has
    exited (``production_node``: node-total CPU-s/s with the node counter process, counter
    rows per GPU, per-process PSS, per-rank HBM; rocmdash.runtime.nodemeasure)."""
    try:
        with open(line_file) as f:
            line = f.read().strip()
    except OSError:
        line = ""
    if not line:
        return
    if rc == 0 and known.production_s > 0 and not known.cpu:
        from rocmdash.runtime.nodemeasure import measure_production

        out = json.loads(line)
        print(f"[bench] production node service on {world} GPU(s) for {known.production_s:g} s", file=sys.stderr,
              flush=True)
        prod = measure_production(world, seconds=known.production_s, counter_daemon="on")
        out["production_node"] = prod
        out["production_node_cpu_seconds_per_s"] = prod.get("node_cpu_seconds_per_s_total")
        print("[bench] side run + deployed path under the production runtime environment", file=sys.stderr, flush=True)
        out["lean_env"] = _lean_env_block()
        line = json.dumps(out)
        if known.json_out:
            with open(known.json_out, "w") as f:
                f.write(line + "\n")
    print(line, flush=True)


def _lean_env_block(timeout_s: float = 240.0) -> dict:
    """the driver's line measures the default HIP / RCCL environment,
    but the supervisor starts every node process with LEAN_RUNTIME_ENV (one hardware queue,
    1 MiB scratch, 2 RCCL channels of 1 MiB; rocmdash.runtime.supervisor). A fresh one-rank
    bench process (the same driver shape, on rank 0's GPU) under that environment reports
    the side run's device timing and the deployed path's service stages, next to the
    default-environment fields of the same line (device_us_p50,
    deployed_path.service_stage_us_p50)."""
    import subprocess
    import tempfile

    from rocmdash.runtime.supervisor import LEAN_RUNTIME_ENV

    drop = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR", "MASTER_PORT",
            "TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_RESTART_COUNT", "ROCMDASH_BENCH_LINE_FILE",
            "ROCMDASH_BENCH_CHILD", "ROCMDASH_BENCH_LAUNCHED", "ROCMDASH_OVERSUBSCRIBE")
    env = {k: v for k, v in os.environ.items() if k not in drop and not k.startswith("ROCMDASH_BENCH_")}
    env.update(LEAN_RUNTIME_ENV)
    env["ROCMDASH_BENCH_RESTARTS"] = "0"  # measured in this process, no restart parent
    fd, path = tempfile.mkstemp(prefix="rocmdash-bench-lean-", suffix=".json")
    os.close(fd)
    block = {"env": dict(LEAN_RUNTIME_ENV), "config": "python bench.py --gpus 1 --steps 20 --warmup 5 --e2e-s 3 "
             "(rank 0's GPU), one process under the supervisor's runtime environment", "error": None}
    try:
        res = subprocess.run([sys.executable, os.path.abspath(__file__), "--gpus", "1", "--steps", "20", "--warmup",
                              "5", "--e2e-s", "3", "--production-s", "0", "--json-out", path], env=env,
                             capture_output=True, text=True, timeout=timeout_s)
        with open(path) as f:
            txt = f.read().strip()
        if res.returncode != 0 or not txt:
            block["error"] = f"exit {res.returncode}: {res.stderr.strip()[-400:]}"
            return block
        d = json.loads(txt.splitlines()[-1])
        dep = d.get("deployed_path") or {}
        block.update(device_us_p50=d.get("device_us_p50"), service_stage_us_p50=dep.get("service_stage_us_p50"),
                     value=d.get("value"), sampler_p50_us=d.get("sampler_p50_us"),
                     prometheus_page_p50_ms=d.get("prometheus_page_p50_ms"))
    except (subprocess.TimeoutExpired, OSError, ValueError) as e:
        block["error"] = f"{type(e).__name__}: {e}"
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass
    return block


def _restart_rounds(args_list, known, world: int, rank: int, store) -> int:
    """The start-up rounds of _run_with_restarts; returns the measurement child's code."""
    import torch

    attempt = 0
    p, verdict_r, decision_w = _start_child(args_list, attempt, known.restarts == 0, store)
    code = None
    rnd = 0
    while True:
        if code is None:
            verdict = verdict_r.readline().strip()  # "" if the child died before its prefill ended
            verdict_r.close()
            code = {"ok": 0, "slow": 1}.get(verdict, 2)
        codes, attempts = [code], [attempt]
        if store is not None:
            import torch.distributed as dist

            t = torch.tensor([code, attempt], dtype=torch.int64)
            out = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(out, t)
            codes, attempts = [int(x[0]) for x in out], [int(x[1]) for x in out]
        decision, again = restart_plan(codes, attempts, known.restarts)
        rnd += 1
        if decision == "restart":
            if rank not in again:
                continue  # this rank's child keeps waiting with its verdict
            try:
                decision_w.write("restart\n")
                decision_w.close()
            except BrokenPipeError:
                pass
            p.wait()
            print(f"[bench] rank {rank}: attempt {attempt} came up in the slow state; starting attempt {attempt + 1} "
                  f"(ranks restarting this round: {again})", file=sys.stderr, flush=True)
            attempt += 1
            p, verdict_r, decision_w = _start_child(args_list, attempt, attempt >= known.restarts, store)
            code = None
            continue
        try:
            decision_w.write(("go %d" % rnd if decision == "go" else "abort") + "\n")
            decision_w.close()
        except BrokenPipeError:
            pass
        return p.wait()


def _child_verdict(agent, args, rank: int) -> int | None:
    """Child side of the restart protocol (see _run_with_restarts): report this
    process's state, then follow the parents' decision. On "go <round>" the round keys
    the process group this child forms next. Returns an exit code when the measurement
    must not go on, else None."""
    vfd = os.environ.get("ROCMDASH_BENCH_VERDICT_FD")
    if not vfd:
        return None
    slow = _slow_state(agent, args)
    with os.fdopen(int(vfd), "w") as f:
        f.write("slow\n" if slow else "ok\n")
    with os.fdopen(int(os.environ["ROCMDASH_BENCH_DECISION_FD"]), "r") as f:
        decision = f.readline().strip()
    if decision.startswith("go"):
        os.environ["ROCMDASH_BENCH_ROUND"] = decision.split()[1] if len(decision.split()) > 1 else "0"
        return None
    if slow:
        print(f"[bench] rank {rank} attempt {os.environ.get('ROCMDASH_BENCH_ATTEMPT')}: counter reads in the slow "
              f"driver state ({slow['counter_p50_us']} us p50 vs {slow['fast_p50_us']} us calibrated); this rank "
              "starts a fresh process", file=sys.stderr, flush=True)
    agent.close()
    return EXIT_SLOW_STATE if decision == "restart" else 1


def _rccl_summary(ranks: list) -> dict | None:
    """Every rank's RCCL view (ncclCommCount / ncclCommUserRank) and transport kinds."""
    if not any("rccl_nranks" in r for r in ranks):
        return None
    from rocmdash.parallel.rccl_log import all_p2p

    kinds: dict = {}
    for r in ranks:
        for k, v in (r.get("transport_kinds") or {}).items():
            kinds[k] = kinds.get(k, 0) + v
    return {"nranks_by_rank": [r.get("rccl_nranks") for r in ranks], "rank_by_rank": [r.get("rccl_rank") for r in ranks],
            "transport_connections": kinds, "all_p2p": all_p2p({"kinds": kinds}),
            "via": sorted({v for r in ranks for v in (r.get("transport_via") or [])})}


EXIT_USAGE = 2  # the requested node size cannot be run as asked
EXIT_TRANSPORT = 4  # N > 1 on a real node, but RCCL connected a peer without P2P (xGMI)


def _requested_gpus(argv_list) -> int | None:
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=None)
    known, _ = ap.parse_known_args(argv_list)
    return known.gpus


def _visible_gpus() -> int:
    """PHYSICAL GPUs this process may use, counted without starting the HIP runtime: the
    KFD topology's node plan (a compute-partitioned MI355X is several HIP devices but one
    GPU, one rank: rocmdash.runtime.topology), else ``torch.cuda.device_count()`` (which
    does not initialise HIP on this image)."""
    import torch

    from rocmdash.runtime.topology import node_plan

    hip_n = int(torch.cuda.device_count())
    plan = node_plan()
    # the plan only when HIP sees every device it lists (a container may show KFD nodes
    # of GPUs it cannot use)
    if plan is not None and plan["gpus"] and plan["logical_devices"] <= hip_n:
        return len(plan["gpus"])
    return hip_n


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def _launch_ranks(argv_list, n: int) -> int:
    """``--gpus N > 1`` without a launcher: start the N rank processes the launcher would
    (one per GPU, each then running its own measurement child as under torchrun) and
    wait. The first rank that fails ends the others (their process groups, started
    here) and its exit code is returned. This process never touches the GPU."""
    import signal
    import subprocess

    port = _free_port()
    drop = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR", "MASTER_PORT",
            "TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_RESTART_COUNT")
    base = {k: v for k, v in os.environ.items() if k not in drop}
    procs = []
    stopping = []

    def on_signal(sig, _frame):
        # before the first rank starts: a SIGTERM / SIGINT to this process
        # ends every rank's session instead of orphaning ranks that hold GPUs
        stopping.append(sig)
        for q in procs:
            try:
                os.killpg(q.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, on_signal)
    for r in range(n):
        if stopping:
            break
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ROCMDASH_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv_list], env=env,
                                      start_new_session=True))
    print(f"[bench] no launcher: started {n} rank processes (master 127.0.0.1:{port})", file=sys.stderr, flush=True)
    rc = 128 + int(stopping[0]) if stopping else 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    print(f"[bench] rank {procs.index(p)} exited with {code}; stopping the other ranks", file=sys.stderr,
                          flush=True)
                    for q in live:
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            time.sleep(0.1)
    finally:
        for q in procs:
            if q.poll() is None:
                try:
                    q.wait(timeout=15)
                except subprocess.TimeoutExpired:
                    os.killpg(q.pid, signal.SIGKILL)
                    q.wait()
    return rc


def _check_node_size(argv_list) -> int | None:
    """The node size the line will report must be the one that runs: returns an exit
    code to stop with, or None to go on. Under a launcher --gpus must equal WORLD_SIZE;
    without one, N > 1 needs N visible GPUs (or ROCMDASH_OVERSUBSCRIBE=1)."""
    want = _requested_gpus(argv_list)
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if want is not None and want != int(world):
            print(f"[bench] error: --gpus {want} but the launcher started WORLD_SIZE {world} ranks", file=sys.stderr)
            return EXIT_USAGE
        return None
    n = 1 if want is None else want
    if n < 1:
        print(f"[bench] error: --gpus {n}", file=sys.stderr)
        return EXIT_USAGE
    if "--cpu" in argv_list:
        return None
    from rocmdash.parallel.node import oversubscribed

    have = _visible_gpus()
    if have < n and not oversubscribed():
        print(f"[bench] error: --gpus {n} but {have} GPU(s) visible; a {n}-GPU number needs {n} GPUs "
              "(ROCMDASH_OVERSUBSCRIBE=1 runs a labelled rehearsal on fewer)", file=sys.stderr)
        return EXIT_USAGE
    if have == 0:
        print("[bench] error: no GPU visible (--cpu runs the CPU reference path)", file=sys.stderr)
        return EXIT_USAGE
    return None


def main(argv=None) -> int:
    argv_list = sys.argv[1:] if argv is None else argv
    if os.environ.get("ROCMDASH_BENCH_CHILD") is None and os.environ.get("ROCMDASH_BENCH_LAUNCHED") is None:
        stop = _check_node_size(argv_list)
        if stop is not None:
            return stop
        n = _requested_gpus(argv_list) or 1
        if os.environ.get("WORLD_SIZE") is None and n > 1:
            return _launch_ranks(argv_list, n)
    if (os.environ.get("ROCMDASH_BENCH_CHILD") is None and os.environ.get("ROCMDASH_BENCH_RESTARTS", "1") != "0"
            and ("--cpu" not in argv_list or os.environ.get("ROCMDASH_BENCH_FAKE_SLOW"))):
        return _run_with_restarts(argv)
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--window", type=int, default=4096, help="samples per series reduced each refresh")
    ap.add_argument("--source", default="auto", choices=["auto", "hw", "synthetic"])
    ap.add_argument("--counters", default="auto", choices=["auto", "hw", "synthetic", "off"])
    ap.add_argument("--gauge", type=int, default=1, help="1 = gauges (reference default), 0 = bars")
    ap.add_argument("--extended", action="store_true", help="add MFMA/HBM-bandwidth panels")
    ap.add_argument("--prefill", type=int, default=-1, help="rows sampled before timing (-1 = one window)")
    ap.add_argument("--prefill-generated", type=int, default=0,
                    help="long windows: first fill this many GENERATED rows per ring (numpy, telemetry-like) so a "
                    "2^24-sample window is full for its kernel cost; reported as window_prefill")
    ap.add_argument("--prefill-generated-from", default="live", choices=["live", "normal"],
                    help="the generated rows: resampled from the live rows of the --prefill phase (the window holds "
                    "the node's own distribution) or drawn from N(50, 10)")
    ap.add_argument("--cpu", action="store_true", help="CPU reference path (no GPU)")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="1 = rank 0 renders refresh i on a render thread while refresh i+1 samples and gathers "
                    "(PipelinedRefresher); 0 = render inline (default: the native render of an 8-GPU frame "
                    "takes ~20 us, less than the thread hand-off saves; profiles/r01/rehearse8_*.json)")
    ap.add_argument("--prefetch", type=int, default=1,
                    help="1 = each refresh requests the next refresh's sample on the native sampler threads "
                    "(overlaps sampling with stats/gather/render); 0 = sample inline")
    ap.add_argument("--sampling", default="auto", choices=["auto", "closed", "free"],
                    help="closed = one read per source per refresh (prefetched); free = every source reads back to "
                    "back on its own thread and each refresh waits for at least one new row per source, so at N > 1 "
                    "no rank waits for another rank's read tail (auto = free: +13 % fresh samples/s at N = 1 on "
                    "MI355X for +2 us p50, profiles/r03/sampling_ab/)")
    ap.add_argument("--node-window", action="store_true",
                    help="each refresh also computes node-wide window statistics (every GPU's sorted window "
                    "all-gathered, rank selection on rank 0)")
    ap.add_argument("--gather", default="auto", choices=["auto", "identity", "rccl"],
                    help="N = 1: identity (kernel writes pinned host memory, default) or a real one-rank RCCL "
                    "all-gather; N > 1 always gathers")
    ap.add_argument("--world1-group", type=int, default=1,
                    help="N = 1: create the one-rank RCCL group (for --gather rccl and the side run's gather timing)")
    ap.add_argument("--timing-steps", type=int, default=100,
                    help="untimed side run after the timed region with HIP events around the stats kernel and the "
                    "all-gather (0 = skip)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--production-s", type=float, default=10.0,
                    help="after every measurement rank has exited: seconds of the PRODUCTION node service (the "
                    "DaemonSet's supervisor + ranks + node counter process at amd-smi 10 Hz / counters 100 Hz) on "
                    "the same GPUs, measured from outside - node-total CPU-s/s, counter rows per GPU, per-process "
                    "PSS, per-rank HBM (production_node; 0 = skip; needs the restart parent)")
    ap.add_argument("--restarts", type=int, default=2,
                    help="N = 1: start the measurement again (in a fresh child process) at most this many times when "
                    "its device-counter reads came up in the slow driver state (ROCMDASH_BENCH_RESTARTS=0: never)")
    ap.add_argument("--settle-s", type=float, default=5.0,
                    help="after prefill, keep sampling at most this long while the recent driver reads are in the "
                    "start-up slow phase (reported as settle_s; 0 = off)")
    ap.add_argument("--slow-factor", type=float, default=1.4,
                    help="slow state = counter-read p50 above this multiple of the placement calibration's fast node "
                    "(the slow state reads 1.7-1.9x, a normal start ~1.0x)")
    ap.add_argument("--cpu-window-s", type=float, default=1.0,
                    help="after the timed region, the same refreshes continue untimed this long to measure the mode's "
                    "CPU-s/s (cpu_seconds_per_s; 0 = over the timed region only)")
    ap.add_argument("--e2e-s", type=float, default=5.0,
                    help="after the timed region: seconds of the deployed path (service refresh 10 Hz -> /metrics -> "
                    "mini-Prometheus scrape 0.25 s -> page queries -> frame), run by every rank (0 = skip)")
    ap.add_argument("--collective-timeout", type=float,
                    default=float(os.environ.get("ROCMDASH_COLLECTIVE_TIMEOUT", "120")),
                    help="seconds a native gather may wait for the slowest rank before the job fails")
    ap.add_argument("--demote-spin", type=int, default=int(os.environ.get("ROCMDASH_BENCH_DEMOTE_SPIN", "0")),
                    help="1 = put the runtime's busy-polling thread on SCHED_IDLE as the node service does "
                    "(rocmdash/runtime/threads.py)")
    ap.add_argument("--rehearse-gpus", type=int, default=0,
                    help="experiment only: rank 0 renders a frame for this many GPUs (repeating the gathered ones); "
                    "the JSON line is marked 'rehearsal' and is not a measurement of that node size")
    args = ap.parse_args(argv)

    # Counters must be registered before the HIP runtime initialises.
    from rocmdash.runtime import native

    native.load()
    if not args.cpu and args.counters in ("auto", "hw") and args.source != "synthetic":
        native.enable_counters()

    import torch

    from rocmdash.config import SamplerConfig
    from rocmdash.parallel.node import NodeAggregator, dist_env_from_environ, local_device, oversubscribed
    from rocmdash.runtime.agent import GpuAgent
    from rocmdash.runtime.pipeline import NodePipeline, PipelinedRefresher
    from rocmdash.viz.panels import EXTENDED_PANELS

    # the GPU agent first, with no process group or communicator yet: the start-up
    # verdict (slow driver state) is taken after prefill, so a slow rank's child can be
    # replaced alone before the node's group forms (_run_with_restarts)
    device, local_rank = local_device(prefer_gpu=not args.cpu)
    use_gpu = device.type == "cuda"
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world_env:  # _check_node_size ran first: only a launcher that changed size
        print(f"[bench] error: --gpus {args.gpus} but the launcher started {world_env} ranks", file=sys.stderr)
        return EXIT_USAGE
    if args.window > 32768:  # HBM-resident long window: the host ring is only a staging queue
        cfg = SamplerConfig(window=args.window, ring_capacity=65536)
    else:
        cfg = SamplerConfig(window=args.window, ring_capacity=max(4 * args.window, 16384))
    agent = GpuAgent(device.index if use_gpu else local_rank, source=args.source, counters=args.counters,
                     cfg=cfg, use_gpu=use_gpu)
    demoted = []
    spin_pin = os.environ.get("ROCMDASH_PIN_SPINNER", "0")  # experiment: move the runtime's poller too
    if spin_pin not in ("0", "") and agent.info.counter_backend == "rocprofiler" and agent.sampler_cpus:
        from rocmdash.runtime.threads import busy_foreign_threads

        for tid, name, rate in busy_foreign_threads():
            os.sched_setaffinity(tid, agent.sampler_cpus)
            demoted.append([tid, name, round(rate, 3), "pinned to the sampler CPUs"])
    if args.demote_spin and agent.info.counter_backend == "rocprofiler":
        from rocmdash.runtime.threads import demote_runtime_spinners

        demoted = demote_runtime_spinners()
    prefill = min(args.window, 65536) if args.prefill < 0 else args.prefill
    generated = 0
    if args.prefill_generated > 0 and args.prefill_generated_from == "normal":
        generated = agent.prefill_bulk(args.prefill_generated)
    t_pf = time.perf_counter()
    agent.prefill(prefill)
    prefill_s = time.perf_counter() - t_pf
    if args.prefill_generated > 0 and args.prefill_generated_from == "live":
        # the bulk resampled from the live rows just read, then live rows on top again
        generated = agent.prefill_bulk(args.prefill_generated, like="live")
        agent.prefill(prefill)
    settle_s = _settle(agent, args)
    stop = _child_verdict(agent, args, int(os.environ.get("RANK", "0")))
    if stop is not None:
        return stop  # no group exists yet: this child just leaves
    # N = 1 on a GPU: a one-rank process group, so the RCCL all-gather can run (and be
    # timed) even though the default N = 1 refresh needs no collective
    # the control plane's collectives are bounded too: a rank that never arrives fails the
    # job after this long instead of hanging it (ranks start seconds apart: calibration)
    env = dist_env_from_environ(prefer_gpu=not args.cpu, timeout_s=max(300.0, args.collective_timeout),
                                world1_group=not args.cpu and torch.cuda.is_available() and args.world1_group)
    if args.gpus != env.world_size:
        print(f"[bench] error: --gpus {args.gpus} but the process group has {env.world_size} ranks", file=sys.stderr)
        return EXIT_USAGE
    n = env.world_size
    agg = NodeAggregator(force_collective=args.gather == "rccl" and n == 1 and agg_possible())
    if args.pipeline < 0:
        args.pipeline = int(n > 1 or args.rehearse_gpus > 1)
    if args.sampling == "auto":
        args.sampling = "free"
    pipe = NodePipeline(agent, agg, use_gauge=bool(args.gauge), extended=args.extended, prefetch=bool(args.prefetch),
                        render_gpus=args.rehearse_gpus, allow_host_out=not args.pipeline,
                        collective_timeout_s=args.collective_timeout, sampling=args.sampling)
    pipe.prevalidate()  # N > 1: the native gather's start-up validation, before any timing
    slow = _slow_state(agent, args) if os.environ.get("ROCMDASH_BENCH_CHILD") else None

    def sync():
        if use_gpu:
            torch.cuda.synchronize(env.device)

    refresher = PipelinedRefresher(pipe) if args.pipeline else None
    nws = None
    if args.node_window:
        from rocmdash.parallel.node_window import NodeWindowStats

        if refresher is not None:
            raise SystemExit("--node-window runs with the inline refresh (--pipeline 0)")
        nws = NodeWindowStats(agent, agg, collective_timeout_s=args.collective_timeout)
        nws.timing = nws.long  # long windows: HIP events around the per-pass collectives
    nw_coll, nw_times, nw_kind = [], [], []
    lw_set = getattr(agent, "dws", None) if nws is not None and nws.long else None
    nw_st0 = None

    def node_window():
        c0 = lw_set.stats() if lw_set is not None else None
        t = time.perf_counter()
        st = nws.refresh()
        if st is not None:
            st.cpu()  # rank 0: the node statistics are on the host
        elif use_gpu:
            torch.cuda.synchronize(env.device)
        ms = (time.perf_counter() - t) * 1e3
        if nws.last_collective_us:
            nw_coll.append(nws.last_collective_us)
        nw_times.append(ms)
        if c0 is not None:  # what this node refresh ran: a bracket hit, or the radix chain (a miss)
            c1 = lw_set.stats()
            nw_kind.append("chain" if c1["chain_refreshes"] > c0["chain_refreshes"] else
                           "hit" if c1["bracket_refreshes"] > c0["bracket_refreshes"] else "other")
        return ms

    if args.sampling == "free":
        pipe.start_sampling()  # the sources read back to back from here to the end of the timed region
    for _ in range(args.warmup):
        if refresher is not None:
            refresher.step()
        else:
            pipe.step()
            if nws is not None:
                node_window()
    if refresher is not None:
        refresher.flush()
        refresher.latencies_ms.clear()
        refresher.parts_ms.clear()
    nw_coll.clear()
    nw_times.clear()
    nw_kind.clear()
    if lw_set is not None:
        nw_st0 = lw_set.stats()
        nw_series0 = lw_set.bracket_stats(1)
    agg.barrier()
    sync()

    lat = []
    parts = []
    payload_bytes = 0
    # exactly K reads per source are counted for K steps, and all K lie inside the timed
    # window: the warm-up's prefetched read lands before it (step 1 renders it), and the
    # read the last step requests is waited for before the window closes - without the
    # drains a short run (the driver's K = 20) counted K + 1
    # (free-running sampling: the counts are taken right at t0 and t1, so exactly the rows
    # that completed inside the timed window are counted)
    agent.wait_sample()
    agg.barrier()
    sync()
    t0 = time.perf_counter()
    cpu_t0 = time.process_time()  # every thread of this rank: samplers, runtime poller, RCCL proxy
    smi_c0 = agent.smi_source.counts()
    counts0 = agent.sample_counts()
    if refresher is not None:
        for _ in range(args.steps):
            refresher.step()
        refresher.flush()  # the last refresh's frame is rendered inside the timed region
    else:
        for _ in range(args.steps):
            _, tm = pipe.step()
            nw_ms = node_window() if nws is not None else 0.0
            lat.append(tm.total_ms + nw_ms)
            parts.append((tm.sample_ms, tm.device_ms + nw_ms, tm.render_ms))
            payload_bytes = max(payload_bytes, tm.payload_bytes)
    agent.wait_sample()  # the K-th read (requested by the last step): counted, so timed
    sync()
    agg.barrier()
    t1 = time.perf_counter()
    cpu_t1 = time.process_time()
    counts1 = agent.sample_counts()
    smi_c1 = agent.smi_source.counts()
    smp = agent.sampler_stats()  # read durations of the timed region (before the side runs)
    elapsed = agg.max_over_ranks(t1 - t0, device=env.device if agg.backend == "nccl" else None)
    # what the timed region's mode costs in CPU: the driver's K = 20 steps last ~1.5 ms,
    # shorter than the kernel's per-thread CPU accounting resolves for the OTHER threads
    # (samplers, the runtime's poller), so the same refreshes continue untimed for >= 1 s
    # (the same step count on every rank: from the all-reduced elapsed time) and the
    # process's CPU-s/s is taken over that window
    cpu_rate = (cpu_t1 - cpu_t0) / (t1 - t0)
    if refresher is None and args.cpu_window_s > 0:
        extra = min(200000, int(args.cpu_window_s / max(elapsed / args.steps, 1e-6)) + 1)
        c_w0, t_w0 = time.process_time(), time.perf_counter()
        for _ in range(extra):
            pipe.step()
        sync()
        cpu_rate = (time.process_time() - c_w0) / (time.perf_counter() - t_w0)
        agg.barrier()
    pipe.stop_sampling()
    if refresher is not None:
        lat = list(refresher.latencies_ms) if env.rank == 0 else [a + b for a, b in refresher.parts_ms]
        parts = [(a, b, max(0.0, l - a - b)) for (a, b), l in zip(refresher.parts_ms, lat)] if env.rank == 0 else [
            (a, b, 0.0) for a, b in refresher.parts_ms]
        payload_bytes = refresher.payload_bytes
        refresher.close()
    fresh = agg.sum_over_ranks(agent.fresh_samples(counts0, counts1),
                               device=env.device if agg.backend == "nccl" else None)

    # per-rank detail for the scaling curve (N > 1: which rank paced the node, and why)
    my = {"rank": env.rank, "device": env.device.index if use_gpu else None,
          "fresh_samples": int(agent.fresh_samples(counts0, counts1)), "timed_s": round(t1 - t0, 4),
          "sampler_p50_us": [round(x["p50_us"], 1) for x in agent.sampler_stats()],
          "init_node": (_placement_report() or {}).get("node"), "slow_state": bool(slow),
          # fresh processes this rank started before this one (slow driver state)
          "attempt": int(os.environ.get("ROCMDASH_BENCH_ATTEMPT", "0")),
          "cpu_seconds_per_s": round(cpu_rate, 4),
          "cpu_seconds_per_s_timed_region": round((cpu_t1 - cpu_t0) / (t1 - t0), 4)}
    grep = pipe.gather_report()
    if "rccl_nranks" in grep:  # RCCL's own view of this rank's communicator, and its transports
        td = grep.get("transport_detail") or {}
        my.update(rccl_nranks=grep["rccl_nranks"], rccl_rank=grep["rccl_rank"], rccl_device=grep["rccl_device"],
                  transport_kinds=td.get("kinds"), transport_via=td.get("via"))
    ranks = agg.all_gather_object(my)
    if n > 1 and use_gpu:
        from rocmdash.parallel.rccl_log import all_p2p

        bad = [r for r in ranks if r.get("rccl_nranks") not in (None, n)]
        if bad:
            print(f"[bench] error: RCCL reports communicators of {[r['rccl_nranks'] for r in bad]} ranks, not {n}",
                  file=sys.stderr, flush=True)
            agent.close()
            return EXIT_TRANSPORT
        not_p2p = [r["rank"] for r in ranks if all_p2p({"kinds": r.get("transport_kinds")}) is False]
        if not_p2p and not oversubscribed() and os.environ.get("ROCMDASH_REQUIRE_P2P", "1") != "0":
            print(f"[bench] error: RCCL connected rank(s) {not_p2p} to a peer without P2P "
                  f"({[r.get('transport_via') for r in ranks if r['rank'] in not_p2p]}): not an xGMI measurement "
                  "(ROCMDASH_REQUIRE_P2P=0 measures anyway)", file=sys.stderr, flush=True)
            agent.close()
            return EXIT_TRANSPORT
    S = len(agent.series)
    reads_per_s = agg.sum_over_ranks(_series_read(counts0, counts1)) / elapsed
    value = fresh / elapsed
    device_us, tagg = _device_timing(agent, env, agg, args) if args.timing_steps > 0 else (None, agg)
    deployed = None
    if args.e2e_s > 0:
        from rocmdash.runtime.deployed import run_deployed_path

        agent.wait_sample()
        deployed = run_deployed_path(agent, tagg if tagg.collective else agg, seconds=args.e2e_s,
                                     collective_timeout_s=args.collective_timeout)
    dep = deployed or {}
    ms_per_step = elapsed / args.steps * 1e3
    lat_sorted = sorted(lat)
    p50 = statistics.median(lat_sorted)
    p90 = lat_sorted[min(len(lat_sorted) - 1, int(0.9 * len(lat_sorted)))]
    ref_p50 = _interp_ref(n)

    n_render = max(n, args.rehearse_gpus)
    if env.rank == 0:
        med = lambda i: statistics.median(p[i] for p in parts)  # noqa: E731
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "fresh metric samples/s (whole job; a series value counts only when it carries new data: "
                    "counter deltas and live used-VRAM every read, SMU-table series once per firmware publication)",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (n * REF_SAMPLES_PER_S_PER_GPU), 2),
            "dtype": "fp32 samples, fp64 accumulation",
            "data": (
                f"live telemetry: smi={agent.info.smi_backend}, counters={agent.info.counter_backend}"
                if agent.info.smi_backend != "synthetic"
                else "synthetic counter streams (native synthetic sources)"
            ),
            "config": {
                "model": "rocmdash node refresh: amd-smi + rocprofiler-sdk -> pinned ring -> HIP window stats "
                f"(W={args.window}) -> {_gather_desc(pipe, agg)} -> 4+4N {'gauge' if args.gauge else 'bar'} "
                "figures + tables",
                "global_batch": n,
                "seq_len": args.window,
                "parallelism": f"rank-per-GPU x{n} ({_gather_desc(pipe, agg)})"
                + (", rank-0 render pipelined with the next refresh" if args.pipeline else "")
                + (", sources free-running on native threads (each refresh waits for >= 1 new row per source)"
                   if args.sampling == "free" else
                   ", next sample prefetched on native sampler threads" if args.prefetch else "")
                + ((", node-wide window statistics (distributed radix select: digit histograms all-reduced)"
                    if nws.long else ", node-wide window statistics (sorted windows all-gathered)")
                   if args.node_window else ""),
                "series_per_gpu": S,
                "figures_per_refresh": 4 + 4 * n_render + (len(EXTENDED_PANELS) * n_render if args.extended else 0),
            },
            "samples_per_s_per_gpu": round(value / n, 2),
            "hardware_reads_per_s": round(reads_per_s, 2),
            "sampling": args.sampling,
            "fresh_samples": int(fresh),
            # rank 0's fresh values per second by origin (the value sums these over ranks)
            "fresh_per_s_by_source": {k: round(v / (t1 - t0), 1)
                                      for k, v in agent.fresh_breakdown(counts0, counts1).items()},
            "device_us_p50": device_us,
            # --node-window: the node statistics' own time per refresh and (long windows,
            # N > 1 or --gather rccl) the per-pass collective µs (HIP events, rank 0)
            "node_window": None if nws is None else {
                "mode": _node_window_mode(nws, lw_set),
                "ms_p50": round(statistics.median(nw_times), 4) if nw_times else None,
                # the timed node refreshes' tail, and the misses (radix chain) on their own
                "timed": _node_window_tail(nw_times[:args.steps], nw_kind[:args.steps]),
                # per series over the timed region: node refreshes that used its brackets, and
                # those the brackets resolved (a series' misses = used - hits)
                "series_bracket_refreshes_hits": None if lw_set is None else [
                    [int(b[0] - a[0]), int(b[1] - a[1])] for a, b in zip(nw_series0, lw_set.bracket_stats(1))],
                # the steps that ran (a bracket hit: the record all-gather only)
                "collective_us_p50": {k: round(statistics.median(c[k] for c in nw_coll if k in c), 2)
                                      for k in sorted({k for c in nw_coll for k in c})} if nw_coll else None,
                # long windows: the node refreshes' bracket hits and radix chains, pass-B
                # chunks streamed (incremental), over the timed region and the runs after it
                "long_window": None if lw_set is None or nw_st0 is None else {
                    k: lw_set.stats()[k] - nw_st0[k]
                    for k in ("node_refreshes", "bracket_refreshes", "chain_refreshes", "passb_chunks", "refreshes",
                              "fused_refreshes", "single_kernel_refreshes")}},
            # how the timed region gathered: native RCCL (validated bit for bit at start-up
            # against the gloo control plane), the host fallback, or the identity (N = 1)
            "gather": pipe.gather_report(),
            # N > 1 (or --gather rccl): RCCL's own view of every rank's communicator and
            # the transports it logged for the rank's peers (P2P = xGMI on a real node)
            "rccl": _rccl_summary(ranks),
            # the DEPLOYED path (what users see), measured by this job's ranks after the
            # timed region: service refresh -> /metrics -> Prometheus -> page -> frame
            "prometheus_page_p50_ms": (dep.get("prometheus_page_ms") or {}).get("p50"),
            # the number comparable with the reference's 39.95 ms, which
            # includes its Prometheus HTTP fetch: the deployed page refresh (fetch over
            # real sockets + snapshot + frame); p50_refresh_ms has no HTTP fetch in it
            "comparable_refresh_ms": {
                "value": (dep.get("prometheus_page_ms") or {}).get("p50"),
                "field": "prometheus_page_p50_ms",
                "reference_ms": ref_p50,
                "why": "includes the Prometheus HTTP fetch + snapshot + frame, as the reference's full refresh does; "
                       "p50_refresh_ms is the in-process refresh without HTTP"},
            # the cost of the timed region's sampling mode: CPU seconds per second of
            # every rank process (all threads) over >= --cpu-window-s of the same
            # refreshes right after the timed region, summed over the job (per rank in
            # ranks[], with the timed region's own figure)
            "cpu_seconds_per_s": round(sum(r["cpu_seconds_per_s"] for r in ranks), 4),
            # what the production rates (amd-smi 10 Hz, counters 100 Hz) deliver per GPU,
            # measured in the deployed-path run (the headline runs free-running sources)
            "production_fresh_per_s_per_gpu": dep.get("production_fresh_per_s_per_gpu"),
            "production_cpu_seconds_per_s": (round(sum(dep["cpu_seconds_per_s_by_rank"]), 4)
                                             if dep.get("cpu_seconds_per_s_by_rank") else None),
            "display_age_p50_ms": {k: v["p50"] for k, v in (dep.get("display_age_ms") or {}).items() if v},
            "deployed_path": deployed,
            "p50_refresh_ms": round(p50, 4),
            "p90_refresh_ms": round(p90, 4),
            "reference_p50_refresh_ms": ref_p50,
            "refresh_speedup_vs_reference_p50": round(ref_p50 / p50, 2),
            "refresh_rate_hz": round(1e3 / ms_per_step, 1),
            "window_samples_reduced_per_s": round(n * S * args.window * args.steps / elapsed, 1),
            "p50_breakdown_ms": {"sample": round(med(0), 4), "device+gather": round(med(1), 4), "render": round(med(2), 4)},
            "payload_bytes": payload_bytes,
            "prefill_rows": prefill,
            # rows per ring generated (not sampled) before the live prefill: only to make a
            # long window full for its kernel cost (--prefill-generated)
            "window_prefill": {"generated_rows": generated, "live_rows": prefill,
                               "generated_from": args.prefill_generated_from if generated else None},
            "prefill_s": round(prefill_s, 3),
            "settle_s": round(settle_s, 3),
            "sampler_mean_us": [round(s["mean_us"], 2) for s in smp],
            "sampler_p50_us": [round(s["p50_us"], 2) for s in smp],
            "sampler_p99_us": [round(s["p99_us"], 2) for s in smp],
            "sampler_threads": {"spin_us": cfg.spin_us, "cpus": len(agent.sampler_cpus) or "unpinned"},
            "sched_idle_threads": demoted,
            "init_placement": _placement_report(),
            "ranks": ranks,
            # fresh processes started because counter reads came up in the slow driver
            # state (--restarts): summed over ranks, and per rank (only the slow ranks
            # restart, before the node's group forms)
            "startup_restarts": int(sum(r.get("attempt", 0) for r in ranks)),
            "startup_restarts_by_rank": [int(r.get("attempt", 0)) for r in ranks],
            "slow_state": slow,
            # how often the SMU actually published a new metrics table during the timed
            # steps (rank 0's GPU): every read is real, most repeat the last table
            "smi_table_refreshes_per_s": round((smi_c1.get("raw_table_changes", 0) - smi_c0.get("raw_table_changes", 0))
                                               / (t1 - t0), 1) if "raw_table_changes" in smi_c1 else None,
            # SMU table reads actually issued (ROCMDASH_SMU_TABLE_MIN_US throttles them; the
            # rows in between repeat the table, used VRAM is read live on every row)
            "smu_table_reads_per_s": round((smi_c1.get("raw_reads", 0) - smi_c0.get("raw_reads", 0)) / (t1 - t0), 1)
            if "raw_reads" in smi_c1 else None,
            # values the hardware was actually asked for on rank 0 (each counter row: its
            # series; each amd-smi row: the live used-VRAM column; each SMU table read:
            # the table's series); hardware_reads_per_s counts every series of every row
            "hardware_values_read_per_s": round(_values_read(agent, counts0, counts1, smi_c0, smi_c1) / (t1 - t0), 1),
            "smu_table_min_us": smi_c1.get("table_min_us"),
            "device": torch.cuda.get_device_name(env.device) if use_gpu else "cpu",
        }
        if args.rehearse_gpus:
            out["rehearsal"] = (f"rank 0 rendered {n_render} GPUs from {n} gathered; NOT a {n_render}-GPU measurement")
        if oversubscribed() and n > 1:
            ngpu = torch.cuda.device_count() if use_gpu else 0
            out["rehearsal"] = (f"{n} ranks on {ngpu} GPU(s) (ROCMDASH_OVERSUBSCRIBE: RCCL between the ranks over "
                                f"sockets, not xGMI); NOT an {n}-GPU measurement")
        line = json.dumps(out)
        line_file = os.environ.get("ROCMDASH_BENCH_LINE_FILE")
        if line_file:  # the restart parent prints it, with the production node's figures added
            with open(line_file, "w") as f:
                f.write(line + "\n")
        else:
            print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    agent.close()
    if env.initialized_here:
        import torch.distributed as dist

        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
