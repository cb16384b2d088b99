"""ROCTx ranges around the refresh phases (sample -> window stats -> all-gather ->
D2H -> render), enabled with ``ROCMDASH_TRACE=1``.

PyTorch-ROCm routes ``torch.cuda.nvtx`` to roctx, so ``rocprofv3 --marker-trace``
(or ``--sys-trace``) shows the phases on the same timeline as the kernels and
copies. Disabled, a range costs one attribute check.
"""

from __future__ import annotations

import os
from contextlib import contextmanager

_enabled = os.environ.get("ROCMDASH_TRACE", "0") not in ("0", "", "false", "off")
_nvtx = None


def enabled() -> bool:
    return _enabled


def set_enabled(on: bool) -> None:
    global _enabled
    _enabled = bool(on)


def _backend():
    global _nvtx
    if _nvtx is None:
        try:
            import torch.cuda.nvtx as nvtx

            _nvtx = nvtx
        except Exception:  # pragma: no cover - torch without nvtx/roctx
            _nvtx = False
    return _nvtx


@contextmanager
def trace_range(name: str):
    if not _enabled:
        yield
        return
    b = _backend()
    if b:
        b.range_push(name)
    try:
        yield
    finally:
        if b:
            b.range_pop()
