"""Node entrypoint: one rank per physical GPU, supervised.

    python -m rocmdash.launch [--nproc auto|N] [--print-plan] [--torchrun] [options] -m rocmdash.serve ...

The DaemonSet runs this (deploy/k8s/exporter-daemonset.yaml). It reads the KFD topology
WITHOUT starting the HIP runtime (rocmdash.runtime.topology.node_plan): one rank per
physical GPU, whatever the GPU count (1-8) and compute-partition mode (SPX, or DPX / QPX
/ CPX where one MI355X is several HIP devices), and passes each rank its HIP device in
``ROCMDASH_RANK_DEVICES`` (rank r drives the first partition of physical GPU r; its
amd-smi source reads that GPU's SMU table once, its counter source combines every
partition of the GPU).

By default it then SUPERVISES the ranks itself (rocmdash.runtime.supervisor): the ranks
run the node refresh in membership epochs, a lost or failing GPU is left out of the next
epoch while the others keep exporting (``rocmdash_gpu_up{gpu_id}`` = 0 for it), and it is
restarted in a fresh process with a backoff and re-admitted once it works; this process
serves ``/metrics`` and ``/healthz``. ``--torchrun`` keeps the old form: ``torch.
distributed.run --nnodes=1 --nproc-per-node=<ranks> <the rest>`` as a CHILD process
(every rank restarts together on any failure).

Signal handlers are installed before the first child starts, so a SIGTERM never leaves
orphaned ranks holding GPUs.

Reference anchor: the reference shows whatever GPUs the exporter of the node reports
(``/root/reference/app.py:183-201, 262-313``); this makes the exporter follow the node.
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys


def plan_ranks(nproc: str = "auto", root: str | None = None):
    """(ranks, rank devices or None, plan or None). ``nproc`` "auto": one rank per
    physical GPU of the KFD topology (``torch.cuda.device_count()`` - no HIP start -
    when the topology cannot be read); a number: that many ranks on devices 0..n-1."""
    from .runtime.topology import KFD_NODES, node_plan, rank_devices

    import torch

    plan = node_plan(root or KFD_NODES)
    if nproc != "auto":
        return int(nproc), None, plan
    hip_n = int(torch.cuda.device_count())  # no HIP start
    # the plan only when HIP sees every device it lists (a container can show KFD nodes
    # of GPUs it cannot use): else one rank per HIP device
    if plan is not None and plan["gpus"] and plan["logical_devices"] <= hip_n:
        return len(plan["gpus"]), rank_devices(plan), plan
    return hip_n, None, plan


def _split_module(rest: list) -> tuple:
    """``[opts..., -m, module, module args...]`` -> (opts, module, module args)."""
    if "-m" not in rest:
        return rest, None, []
    i = rest.index("-m")
    if i + 1 >= len(rest):
        raise SystemExit("rocmdash.launch: -m needs a module")
    return rest[:i], rest[i + 1], rest[i + 2:]


def store_port_from(opts: list, ignored: list | None = None) -> int:
    """The store port among torchrun options of older manifests (``--master-port=N``,
    ``--master-port N``, ``--master_port ...``); 0 when none. Other options land in
    ``ignored``. A port that is not a number is an error, never silently a random port
    (ADVICE r05)."""
    port = 0
    i = 0
    while i < len(opts):
        o = opts[i]
        key, eq, val = o.partition("=")
        if key in ("--master-port", "--master_port"):
            if not eq:
                if i + 1 >= len(opts):
                    raise SystemExit(f"rocmdash.launch: {key} needs a port number")
                val = opts[i + 1]
                i += 1
            try:
                port = int(val)
            except ValueError:
                raise SystemExit(f"rocmdash.launch: {key}: not a port number: {val!r}") from None
        elif ignored is not None:
            ignored.append(o)
        i += 1
    return port


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter,
                                 allow_abbrev=False)
    ap.add_argument("--nproc", default=os.environ.get("ROCMDASH_NPROC", "auto"),
                    help="ranks: 'auto' (one per physical GPU of the KFD topology) or a number")
    ap.add_argument("--print-plan", action="store_true", help="print the node plan as JSON and exit")
    ap.add_argument("--torchrun", action="store_true",
                    help="run the ranks under torch.distributed.run (all restart together) instead of supervising them")
    ap.add_argument("--restart-base-s", type=float, default=float(os.environ.get("ROCMDASH_RESTART_BASE_S", "5")),
                    help="supervised: first backoff before a failed GPU's rank starts again (doubles per failure)")
    ap.add_argument("--restart-max-s", type=float, default=float(os.environ.get("ROCMDASH_RESTART_MAX_S", "300")),
                    help="supervised: longest backoff between restart attempts of a failing GPU")
    ap.add_argument("--start-timeout", type=float, default=float(os.environ.get("ROCMDASH_START_TIMEOUT", "240")),
                    help="supervised: a rank not ready (GPU agent up) this long after its start is restarted")
    ap.add_argument("--counter-daemon", default=os.environ.get("ROCMDASH_COUNTER_DAEMON", "auto"),
                    choices=["auto", "on", "off"],
                    help="supervised: read every GPU's device counters in ONE node process (rocmdash.runtime.counterd) "
                    "instead of one counting context - and one busy runtime thread - per rank (auto: with live "
                    "counters)")
    args, rest = ap.parse_known_args(argv)
    n, devices, plan = plan_ranks(args.nproc)
    if args.print_plan:
        print(json.dumps({"ranks": n, "rank_devices": devices, "plan": plan}))
        return 0
    if n < 1:
        print("[rocmdash.launch] no GPU found in the KFD topology: nothing to launch", file=sys.stderr)
        return 2
    mode = plan["mode"] if plan else "unknown"
    if not args.torchrun:
        opts, module, module_args = _split_module(rest)
        if module is None:
            raise SystemExit("rocmdash.launch: supervised mode needs -m <module> (e.g. -m rocmdash.serve)")
        store_port = 0
        ignored = []
        store_port = store_port_from(opts, ignored)
        print(f"[rocmdash.launch] supervising {n} rank(s) (partition mode {mode}, rank devices {devices}): "
              f"-m {module} {' '.join(module_args)}" + (f" (ignored: {' '.join(ignored)})" if ignored else ""),
              file=sys.stderr, flush=True)
        from .runtime.supervisor import run_supervisor

        return run_supervisor(module, module_args, n, devices, store_port=store_port,
                              restart_base_s=args.restart_base_s, restart_max_s=args.restart_max_s,
                              start_timeout_s=args.start_timeout, counter_daemon=args.counter_daemon)
    env = dict(os.environ)
    if devices is not None:
        env["ROCMDASH_RANK_DEVICES"] = ",".join(map(str, devices))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", *rest]
    print(f"[rocmdash.launch] {n} rank(s) (partition mode {mode}, rank devices {devices}): {' '.join(cmd[1:])}",
          file=sys.stderr, flush=True)
    child = None
    pending = []

    def forward(sig, _frame):
        if child is None:  # a signal before the child exists: delivered right after Popen
            pending.append(sig)
            return
        try:
            child.send_signal(sig)
        except ProcessLookupError:
            pass

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    child = subprocess.Popen(cmd, env=env)
    for sig in pending:
        forward(sig, None)
    return child.wait()


if __name__ == "__main__":
    raise SystemExit(main())
