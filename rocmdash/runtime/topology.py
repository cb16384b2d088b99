"""GPU order of the HIP runtime, worked out from the KFD topology in sysfs WITHOUT
initialising HIP.

A rank-per-GPU process must configure the rocprofiler-sdk device-counting service for
ITS GPU before the HIP runtime starts (rocmdash/runtime/native.py), i.e. before it can
ask HIP which PCI device ``cuda:LOCAL_RANK`` is. The HIP runtime lists GPUs in the
order the ROCr runtime finds them: the KFD topology nodes with SIMDs, by node id, that
this process can open (its ``/dev/dri/renderD<minor>``), filtered by
``ROCR_VISIBLE_DEVICES`` and then by ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``
(index lists). This module repeats that walk and maps LOCAL_RANK to the GPU's PCI
address (amd-smi bdf id: domain<<32 | bus<<8 | dev<<3 | fn, what the counters and
amd-smi sources key on). Anything it cannot decide (UUID visibility lists, no sysfs)
returns None, and the caller falls back to the agent ordinal.

The node's GPU layout for the rank-per-GPU service (:func:`node_plan`): one rank per
PHYSICAL GPU, whatever the compute-partition mode. An MI355X in CPX (or DPX / QPX) mode
shows up as several KFD nodes - one per partition, each its own HIP device - that share
the physical GPU's PCI address and ``unique_id``. Grouping them gives one SMU-table
reader per physical GPU (the table is the GPU's, every partition would read the same
one) and the GPU's device counters summed / averaged over all its partitions (csrc/
counters.cpp ``make_counter_source_all``); the rank drives its GPU's first partition in
HIP order for the stats kernel and the RCCL communicator. ``python -m rocmdash.launch``
starts ``len(plan["gpus"])`` ranks and tells each its HIP device
(``ROCMDASH_RANK_DEVICES``), so a node with 4 GPUs, or 8 GPUs in CPX mode (64 HIP
devices), gets 4 or 8 ranks - never a hardcoded 8.

Reference counterpart: the reference renders whatever ``gpu_id`` rows the exporter
reports (``/root/reference/app.py:183-201, 262-313``).
"""

from __future__ import annotations

import os
from dataclasses import dataclass

KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _props(path: str) -> dict:
    out = {}
    try:
        with open(path) as f:
            for line in f:
                k, _, v = line.strip().partition(" ")
                if v.lstrip("-").isdigit():
                    out[k] = int(v)
    except OSError:
        pass
    return out


def _index_filter(items: list, env: str):
    spec = os.environ.get(env)
    if spec is None:
        return items
    spec = spec.strip()
    if spec == "":
        return []
    picked = []
    for tok in spec.split(","):
        tok = tok.strip()
        if not tok.isdigit():  # a UUID list: not decidable here
            return None
        i = int(tok)
        if i >= len(items):
            break  # HIP stops at the first invalid index
        picked.append(items[i])
    return picked


def kfd_gpus(root: str = KFD_NODES, check_access: bool = True) -> list:
    """[(node_id, bdf_id)] of the GPU nodes this process can open, by node id."""
    try:
        nodes = sorted(int(n) for n in os.listdir(root) if n.isdigit())
    except OSError:
        return []
    gpus = []
    for n in nodes:
        p = _props(os.path.join(root, str(n), "properties"))
        if p.get("simd_count", 0) <= 0:
            continue  # CPU node
        if check_access and "drm_render_minor" in p:
            dev = f"/dev/dri/renderD{p['drm_render_minor']}"
            if os.path.exists("/dev/dri") and not os.access(dev, os.R_OK | os.W_OK):
                continue
        bdf = (p.get("domain", 0) << 32) | p.get("location_id", 0)
        gpus.append((n, bdf))
    return gpus


def hip_order_bdfs(root: str = KFD_NODES, check_access: bool = True):
    """bdf ids in HIP device order, or None if that order cannot be decided."""
    gpus = [bdf for _, bdf in kfd_gpus(root, check_access)]
    if not gpus:
        return None
    for env in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        gpus = _index_filter(gpus, env)
        if gpus is None:
            return None
    return gpus


def bdf_of_hip_device(index: int, root: str = KFD_NODES, check_access: bool = True):
    order = hip_order_bdfs(root, check_access)
    if order is None or not 0 <= index < len(order):
        return None
    return order[index]


@dataclass
class KfdGpu:
    """One GPU node of the KFD topology (a physical GPU, or one partition of one)."""

    node: int
    bdf: int
    unique_id: int
    num_xcc: int
    simd_count: int
    hip_index: int = -1  # HIP device index (after the visibility filters)


def kfd_gpu_nodes(root: str = KFD_NODES, check_access: bool = True):
    """Every GPU node this process can use, in HIP device order (visibility filters
    applied, ``hip_index`` set), or None when that order cannot be decided."""
    try:
        nodes = sorted(int(n) for n in os.listdir(root) if n.isdigit())
    except OSError:
        return None
    gpus = []
    for n in nodes:
        p = _props(os.path.join(root, str(n), "properties"))
        if p.get("simd_count", 0) <= 0:
            continue
        if check_access and "drm_render_minor" in p:
            dev = f"/dev/dri/renderD{p['drm_render_minor']}"
            if os.path.exists("/dev/dri") and not os.access(dev, os.R_OK | os.W_OK):
                continue
        gpus.append(KfdGpu(n, (p.get("domain", 0) << 32) | p.get("location_id", 0), p.get("unique_id", 0),
                           p.get("num_xcc", 1), p["simd_count"]))
    for env in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        gpus = _index_filter(gpus, env)
        if gpus is None:
            return None
    for i, g in enumerate(gpus):
        g.hip_index = i
    return gpus


_MODES = {1: "SPX", 2: "DPX", 3: "TPX", 4: "QPX", 8: "CPX"}


def physical_gpus(gpus) -> list:
    """Group partition nodes by physical GPU (``unique_id`` when the driver reports
    one, else the PCI address), in order of each GPU's first HIP device."""
    groups: dict = {}
    for g in gpus:
        key = ("uid", g.unique_id) if g.unique_id else ("bdf", g.bdf)
        groups.setdefault(key, []).append(g)
    return sorted(groups.values(), key=lambda parts: parts[0].hip_index)


def node_plan(root: str = KFD_NODES, check_access: bool = True) -> dict | None:
    """The rank layout of this node: {"mode", "logical_devices", "gpus": [{"rank",
    "hip_device", "bdf", "partitions" (HIP indices), "kfd_nodes", "num_xcc"}]}, one
    entry per physical GPU (rank order = HIP order of their first partitions), or None
    when the HIP order cannot be decided (no sysfs, UUID visibility lists)."""
    gpus = kfd_gpu_nodes(root, check_access)
    if gpus is None:
        return None
    phys = physical_gpus(gpus)
    sizes = {len(p) for p in phys}
    mode = "none" if not phys else (_MODES.get(sizes.pop(), "mixed") if len(sizes) == 1 else "mixed")
    return {
        "mode": mode,
        "logical_devices": len(gpus),
        "gpus": [{"rank": r, "hip_device": parts[0].hip_index, "bdf": parts[0].bdf,
                  "partitions": [g.hip_index for g in parts], "kfd_nodes": [g.node for g in parts],
                  "num_xcc": sum(g.num_xcc for g in parts)} for r, parts in enumerate(phys)],
    }


def rank_devices(plan: dict | None) -> list | None:
    """HIP device of each rank (the first partition of its physical GPU)."""
    return None if plan is None else [g["hip_device"] for g in plan["gpus"]]
