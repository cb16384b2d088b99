"""Node entrypoint: as many ranks as the node has physical GPUs, then torchrun.

    python -m rocmdash.launch [--nproc auto|N] [--print-plan] <torchrun options> -m rocmdash.serve ...

The DaemonSet runs this instead of a torchrun with a fixed ``--nproc-per-node``
(deploy/k8s/exporter-daemonset.yaml). It reads the KFD topology WITHOUT starting the HIP
runtime (rocmdash.runtime.topology.node_plan): one rank per physical GPU, whatever the
GPU count (1-8) and compute-partition mode (SPX, or DPX / QPX / CPX where one MI355X is
several HIP devices), and passes each rank its HIP device in ``ROCMDASH_RANK_DEVICES``
(rank r drives the first partition of physical GPU r; its amd-smi source reads that
GPU's SMU table once, its counter source combines every partition of the GPU). Then it
starts ``torch.distributed.run --nnodes=1 --nproc-per-node=<ranks> <the rest>`` as a
CHILD process (no exec), forwards SIGTERM / SIGINT to it and exits with its code.

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


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter,
                                 allow_abbrev=False)
    ap.add_argument("--nproc", default=os.environ.get("ROCMDASH_NPROC", "auto"),
                    help="ranks: 'auto' (one per physical GPU of the KFD topology) or a number")
    ap.add_argument("--print-plan", action="store_true", help="print the node plan as JSON and exit")
    args, rest = ap.parse_known_args(argv)
    n, devices, plan = plan_ranks(args.nproc)
    if args.print_plan:
        print(json.dumps({"ranks": n, "rank_devices": devices, "plan": plan}))
        return 0
    if n < 1:
        print("[rocmdash.launch] no GPU found in the KFD topology: nothing to launch", file=sys.stderr)
        return 2
    env = dict(os.environ)
    if devices is not None:
        env["ROCMDASH_RANK_DEVICES"] = ",".join(map(str, devices))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", *rest]
    mode = plan["mode"] if plan else "unknown"
    print(f"[rocmdash.launch] {n} rank(s) (partition mode {mode}, rank devices {devices}): {' '.join(cmd[1:])}",
          file=sys.stderr, flush=True)
    child = subprocess.Popen(cmd, env=env)

    def forward(sig, _frame):
        try:
            child.send_signal(sig)
        except ProcessLookupError:
            pass

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    return child.wait()


if __name__ == "__main__":
    raise SystemExit(main())
