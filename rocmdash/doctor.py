"""``python -m rocmdash doctor``: what a node service needs, checked on this machine.

For the operator of the exporter DaemonSet (and for bug reports): each check prints one
line ``[ok|warn|FAIL] name: detail`` (``--json`` for one JSON object) and the exit code
is 1 when an essential check fails. Order matters - the device counters must be
registered before the HIP runtime starts (rocmdash/runtime/native.py), so the checks
that need no HIP run first:

  native      the in-tree extension imports and was built from the current csrc/
  topology    GPUs in the KFD topology (PCI addresses, HIP order) - no HIP call
  numa        NUMA nodes this process may use, and the node-wide placement calibration
              cached for this boot (rocmdash/runtime/placement.py)
  sysfs       the SMU gpu_metrics table and the VRAM counter of every GPU are readable
  amdsmi      amd-smi sees the GPUs; how GPU 0's SMU table is read (raw sysfs after the
              start-up calibration against amd-smi, or through amd-smi) and why
  counters    rocprofiler-sdk device counting configured for the GPUs
  hip         HIP devices, names, and the extension's view of each one's PCI address
  rccl        RCCL loads (the library torch ships) and reports its version
  kfd-proc    per-process VRAM accounting (/sys/class/kfd/kfd/proc) - else footprints
              fall back to start-up deltas (rocmdash/runtime/footprint.py)
"""

from __future__ import annotations

import argparse
import json
import os
import sys


def _check(results, name, fn, essential=True):
    try:
        status, detail = fn()
    except Exception as e:  # noqa: BLE001 - a check that raises failed
        status, detail = "FAIL", f"{type(e).__name__}: {e}"
    if status == "FAIL" and not essential:
        status = "warn"
    results.append({"check": name, "status": status, "detail": detail, "essential": essential})
    return status


def run(counters: bool = True) -> list:
    res = []

    def native_check():
        from ._build import built_from_current_sources
        from .runtime import native

        native.load()
        cur = built_from_current_sources()
        return ("ok" if cur is not False else "warn"), f"rocmdash._native loaded; built from current csrc/: {cur}"

    _check(res, "native", native_check)
    from .runtime import topology

    bdfs = []

    def topo():
        nonlocal bdfs
        bdfs = topology.hip_order_bdfs() or []
        if not bdfs:
            return "FAIL", "no GPU in the KFD topology (/sys/class/kfd/kfd/topology/nodes)"
        return "ok", f"{len(bdfs)} GPU(s): " + ", ".join(f"{b:x}" for b in bdfs)

    _check(res, "topology", topo)

    def numa():
        from .runtime import placement

        nodes = placement.numa_nodes()
        path = placement._cache_path()
        cal = None
        if os.path.exists(path):
            with open(path) as f:
                cal = json.load(f)
        gpus = (cal or {}).get("gpus", {})
        detail = f"nodes {sorted(nodes)} ({', '.join(str(len(c)) + ' cpus' for c in nodes.values())}); "
        detail += (f"calibration cached for {len(gpus)} GPU(s): " + ", ".join(f"{b}->node {e.get('node')}" for b, e in gpus.items())
                   if gpus else "no calibration cached for this boot yet (the first service start probes)")
        return "ok", detail

    _check(res, "numa", numa, essential=False)

    def sysfs():
        from .runtime.agent import bdf_path

        bad = []
        for b in bdfs:
            for f in ("gpu_metrics", "mem_info_vram_used"):
                try:
                    with open(os.path.join(bdf_path(b), f), "rb") as fh:
                        fh.read(8)
                except OSError as e:
                    bad.append(f"{b:x}/{f}: {e.strerror}")
        if not bdfs:
            return "FAIL", "no GPU to read"
        return ("FAIL", "; ".join(bad)) if bad else ("ok", f"gpu_metrics + mem_info_vram_used readable on {len(bdfs)} GPU(s)")

    _check(res, "sysfs", sysfs)

    def amdsmi():
        from .runtime import native

        nat = native.load()
        n = int(nat.amdsmi_gpu_count())
        detail = f"amd-smi sees {max(n, 0)} GPU(s)"
        if n > 0:  # how the SMU table will be read: raw sysfs (calibrated) or through amd-smi
            try:
                info = nat.make_smi_source(0, 0).info()
                detail += (f"; GPU 0 metrics table {info.get('metrics_table')} read via {info.get('metrics_path')}"
                           f" ({info.get('metrics_calibration') or 'no calibration'})")
            except Exception as e:  # noqa: BLE001 - informational only
                detail += f"; SMI source: {type(e).__name__}: {e}"
        return ("ok" if n > 0 else "FAIL"), detail

    _check(res, "amdsmi", amdsmi, essential=False)

    if counters:
        def ctr():
            from .runtime import native

            ok, status = native.enable_counters()
            return ("ok" if ok else "FAIL"), f"rocprofiler-sdk tool registered before HIP start: {status}"

        _check(res, "counters", ctr, essential=False)

    def hip():
        import torch

        from .runtime import native

        if not torch.cuda.is_available():
            return "FAIL", "torch.cuda.is_available() is False"
        nat = native.load()
        devs = []
        for i in range(torch.cuda.device_count()):
            devs.append(f"{i}: {torch.cuda.get_device_name(i)} ({int(nat.hip_device_bdf(i)):x})")
        return "ok", "; ".join(devs)

    _check(res, "hip", hip)

    if counters:
        def ctr_ready():
            from .runtime import native

            return ("ok" if native.counters_ready() else "FAIL"), "after HIP start: " + native.counters_status()

        _check(res, "counters-ready", ctr_ready, essential=False)

    def rccl():
        from .parallel.node import _rccl_lib
        from .runtime import native

        v = int(native.load().rccl_load(_rccl_lib()))
        return "ok", f"RCCL {v // 10000}.{v // 100 % 100}.{v % 100} ({_rccl_lib()})"

    _check(res, "rccl", rccl)

    def kfd_proc():
        from .runtime.footprint import kfd_vram_bytes

        v = kfd_vram_bytes()
        if v is None:
            return "warn", "no /sys/class/kfd/kfd/proc/<pid>: footprints use start-up VRAM deltas"
        return "ok", f"per-process VRAM accounting available ({v / 2**20:.0f} MiB for this process)"

    _check(res, "kfd-proc", kfd_proc, essential=False)
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--no-counters", action="store_true", help="skip the device-counter checks")
    args = ap.parse_args(argv)
    res = run(counters=not args.no_counters)
    failed = [r for r in res if r["status"] == "FAIL" and r["essential"]]
    if args.json:
        print(json.dumps({"ok": not failed, "checks": res}))
    else:
        for r in res:
            print(f"[{r['status']:>4}] {r['check']}: {r['detail']}")
        print("essential checks passed" if not failed else f"{len(failed)} essential check(s) failed", file=sys.stderr)
    return 1 if failed else 0


if __name__ == "__main__":
    raise SystemExit(main())
