"""Windowed statistics over metric series: HIP/CDNA4 kernel entry + fp64 references.

Kernel: ``csrc/window_stats.hip`` (one workgroup per series, register/shuffle/LDS
bitonic sort, wave64 reductions). Per series it returns, in this order
(``rocmdash.models.schema.STAT_NAMES``):

    min, max, mean, p<a>, p<b>, p<c>, last, count

over the valid (non-NaN) samples of the window; ``last`` is the newest raw sample
(NaN if that read failed) and ``count`` the number of valid samples. Percentiles use
numpy's default ('linear') definition. With no valid sample every statistic except
``last``/``count`` is NaN.

Reference counterpart: ``app.py:216-221`` (mean/max/min across GPUs of one instant
sample) - here per series over time, for every series of the node.
"""

from __future__ import annotations

import numpy as np

from ..models.schema import NUM_STATS

DEFAULT_PCT = (50.0, 90.0, 99.0)
MAX_WINDOW = 32768


def window_stats_reference(x, pct=DEFAULT_PCT) -> np.ndarray:
    """fp64 numpy reference. ``x``: [S, n] samples, oldest first. Returns [S, 8]."""
    x = np.asarray(x, dtype=np.float64)
    if x.ndim != 2:
        raise ValueError("x must be [series, samples]")
    S, n = x.shape
    out = np.full((S, NUM_STATS), np.nan)
    for s in range(S):
        row = x[s]
        v = row[~np.isnan(row)]
        out[s, 7] = v.size
        out[s, 6] = row[-1] if n else np.nan
        if v.size:
            out[s, 0] = v.min()
            out[s, 1] = v.max()
            out[s, 2] = v.mean()
            out[s, 3:6] = np.percentile(v, pct)
    return out


def window_stats_torch(x, pct=DEFAULT_PCT):
    """Plain PyTorch fp32-input reference (computed in fp64) of the same op, for
    comparing the HIP kernel on the device. ``x``: [S, n] tensor."""
    import torch

    xd = x.to(torch.float64)
    S, n = xd.shape
    valid = ~torch.isnan(xd)
    cnt = valid.sum(dim=1)
    inf = torch.tensor(float("inf"), dtype=xd.dtype, device=xd.device)
    mn = torch.where(valid, xd, inf).amin(dim=1)
    mx = torch.where(valid, xd, -inf).amax(dim=1)
    mean = torch.where(valid, xd, torch.zeros_like(xd)).sum(dim=1) / cnt.clamp(min=1)
    q = torch.tensor([p / 100.0 for p in pct], dtype=xd.dtype, device=xd.device)
    qs = torch.nanquantile(xd, q, dim=1).T  # [S, 3]
    out = torch.stack([mn, mx, mean], dim=1)
    out = torch.cat([out, qs, xd[:, -1:], cnt.to(xd.dtype)[:, None]], dim=1)
    empty = cnt == 0
    if bool(empty.any()):
        out[empty, :6] = float("nan")
    return out


def sort_width(n: int) -> int:
    p = 64
    while p < n:
        p <<= 1
    return p


def window_stats(x, pct=DEFAULT_PCT, out=None):
    """Run the HIP kernel on a device tensor ``x`` [S, n] (float32, oldest sample first).

    The samples are laid out time-major ([P, S], P = next power of two >= n, the
    layout of the device rings the runtime mirrors) and the kernel is launched on the
    current stream, one workgroup per series (chunks of 96 series per launch).
    """
    import torch

    from ..runtime.native import load

    if not x.is_cuda:
        raise ValueError("window_stats runs on a GPU tensor; use window_stats_reference on the CPU")
    if x.ndim != 2:
        raise ValueError("x must be [series, samples]")
    S, n = x.shape
    if n < 1 or n > MAX_WINDOW:
        raise ValueError(f"window length must be in [1, {MAX_WINDOW}], got {n}")
    nat = load()
    P = 1
    while P < n:
        P <<= 1
    ring = torch.empty((P, S), dtype=torch.float32, device=x.device)
    ring[:n].copy_(x.t())
    if out is None:
        out = torch.empty((S, NUM_STATS), dtype=torch.float32, device=x.device)
    if out.shape != (S, NUM_STATS) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("out must be a contiguous float32 [S, 8] tensor")
    stream = torch.cuda.current_stream(x.device).cuda_stream
    base = ring.data_ptr()
    per = int(nat.MAX_SERIES_PER_LAUNCH)
    for s0 in range(0, S, per):
        cols = list(range(s0, min(S, s0 + per)))
        nat.window_stats_raw(base, n, S, P - 1, n, cols, out[s0:].data_ptr(), stream,
                             float(pct[0]), float(pct[1]), float(pct[2]))
    return out
