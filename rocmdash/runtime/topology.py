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

Reference counterpart: none (the reference reads metrics through Prometheus only).
"""

from __future__ import annotations

import os

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
