"""Node-wide long-window statistics by a distributed radix select: the host model.

The GPUs run it natively (``LongWindowSet.refresh_node``, csrc/long_window.hip): every
rank streams ITS OWN HBM-resident window (2^15..2^26 samples per series), and only digit
histograms, per-series partials and pass-0 predictions cross the node - the windows
never do. Per refresh, on every rank, in the same order:

  1. predict the key bits that vary (previous min / max / lowest varying bit and the
     rows that entered since; 0 / ~0 / 0 when there is no prediction) and all-gather the
     predictions; every rank combines them in rank order - min / max, the lowest varying
     bit including where the ranks' reference keys differ, the first holding rank's
     newest sample as the common reference key - and so picks the SAME pass-0 digit;
  2. pass 0 over the local window: a 8- or 10-bit digit histogram + partials (count,
     fp64 sum, min / max key, OR of key ^ reference); all-gather the partials,
     all-reduce (sum) the histogram - exact integers;
  3. scan 0 (identical inputs on every rank -> identical state): node count, mean (the
     ranks' sums added in rank order), min, max, the lowest varying bit; six sorted
     positions (lo / hi of three percentiles, numpy 'linear') -> digit + residual rank;
  4. passes 1..3: <= 8-bit digits below, counting only samples whose found bits match a
     rank's prefix, histograms all-reduced, down to the lowest varying bit.

Cost on the node: 2 small all-gathers (S x 32 B per rank) and 4 all-reduces of at most
S x 1024 x 4 B = 64 KB (pass 0) / S x 6 x 256 x 4 B = 96 KB (passes 1-3) for S = 16
series - independent of W, where all-gathering a 2^24-sample window would move 64 MB per
series per rank.

This module is the same algorithm in numpy over any ``allgather`` / ``allreduce``
(gloo on CPU: the multi-rank tests, a CPU-only node) and the fp64 oracle's partner:
``node_window_reference`` of the union must equal it exactly for order statistics.

Reference anchor: the statistics over ALL GPUs (``/root/reference/app.py:216-221``).
"""

from __future__ import annotations

import numpy as np

from ..models.schema import NUM_STATS

KD0 = 10  # pass 0: at most 10 key bits (1024 bins)
RANKS = 6  # lo / hi sorted positions of the three percentiles
NO_PRED = (0, 0xFFFFFFFF, 0)  # (pmin, pmax, lo): the top-byte fallback


def fkey(x: np.ndarray) -> np.ndarray:
    """Order-preserving float32 -> uint32 key (as csrc/long_window.hip ``fkey``)."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000).astype(np.uint64)


def kfloat(k: int) -> float:
    u = (k & 0x7FFFFFFF) if (k & 0x80000000) else (~k & 0xFFFFFFFF)
    return float(np.array([u], np.uint32).view(np.float32)[0])


def _ctz(v: int) -> int:
    return (v & -v).bit_length() - 1 if v else 32


def _next_width(shift: int, lo: int) -> int:
    return min(8, shift - lo) if shift > lo else 0


def pass0_digit(pmin: int, pmax: int, lo: int) -> tuple[int, int]:
    """(shift, width) of pass 0's digit for a predicted range (lw_pass<0>)."""
    d = pmin ^ pmax
    top = d.bit_length() - 1 if d else 0
    span = top - lo + 1 if top >= lo else 1

    def passes(dw):
        return (span - dw + 7) // 8 if span > dw else 0

    dw = KD0 if passes(KD0) < passes(8) else 8
    return (top - (dw - 1) if top >= dw - 1 else 0), dw


def combine_predictions(preds) -> tuple[int, int, int, int]:
    """Every rank's (pmin, pmax, lo, ref, has) of one series, in rank order -> the node's
    (pmin, pmax, lo, ref): what every rank's pass 0 computes from the all-gather."""
    mn, mx, lo, ref, anyh = 0xFFFFFFFF, 0, 32, 0, False
    for pmin, pmax, plo, pref, has in preds:
        mn, mx, lo = min(mn, pmin), max(mx, pmax), min(lo, plo)
        if has:
            if not anyh:
                ref, anyh = pref, True
            elif pref != ref:
                lo = min(lo, _ctz(pref ^ ref))
    return mn, mx, lo, ref


def positions(nv: int, pct) -> tuple[list, list]:
    """Sorted positions [lo0, hi0, lo1, hi1, lo2, hi2] and float32 weights (lw_positions)."""
    last = nv - 1 if nv else 0
    pos, frac = [], []
    for p in pct:
        x = float(p) / 100.0 * float(last)
        lo = min(int(np.floor(x)), last)
        pos += [lo, lo + 1 if lo + 1 < nv else last]
        frac.append(float(np.float32(x - lo)))
    return pos, frac


def node_radix_select(x: np.ndarray, pct, allgather, allreduce_sum, pred=None) -> np.ndarray:
    """Collective over the callables: ``x`` [S, n] float32 - THIS rank's window of every
    series (NaN = no sample) - -> the node's [S, 8] statistics over the union of every
    rank's window (min, max, mean, 3 percentiles, last = NaN, count). ``allgather(obj)``
    returns every rank's object in rank order; ``allreduce_sum(uint32 array)`` returns
    the element-wise sum. ``pred``: this rank's (pmin, pmax, lo) per series - a superset
    of the varying bits (default: none, the top-byte digit)."""
    x = np.asarray(x, np.float32)
    S = x.shape[0]
    keys = [fkey(x[s][~np.isnan(x[s])]) for s in range(S)]
    # 1. predictions -> the common pass-0 digit
    mine = []
    for s in range(S):
        pmin, pmax, lo = (pred[s] if pred is not None else NO_PRED)
        k = keys[s]
        has = len(k) > 0
        mine.append((int(pmin), int(pmax), int(lo), int(k[-1]) if has else 0, has))
    preds = allgather(mine)
    dig = []
    for s in range(S):
        pmin, pmax, lo, ref = combine_predictions([p[s] for p in preds])
        shift, dw = pass0_digit(pmin, pmax, lo)
        dig.append((shift, dw, ref))
    # 2. pass 0: histogram + partials
    hist0 = np.zeros((S, 1 << KD0), np.uint32)
    part = []
    for s in range(S):
        k = keys[s]
        shift, dw, ref = dig[s]
        if len(k):
            hist0[s, : 1 << dw] = np.bincount(((k >> np.uint64(shift)) & np.uint64((1 << dw) - 1)).astype(np.int64),
                                              minlength=1 << dw)
            orx = int(np.bitwise_or.reduce(k ^ np.uint64(ref)))
            part.append((float(np.sum(x[s][~np.isnan(x[s])], dtype=np.float64)), len(k), int(k.min()), int(k.max()),
                         orx))
        else:
            part.append((0.0, 0, 0xFFFFFFFF, 0, 0))
    parts = allgather(part)
    hist0 = allreduce_sum(hist0)
    # 3. scan 0 (the same inputs on every rank)
    out = np.full((S, NUM_STATS), np.nan)
    state = []
    for s in range(S):
        sm, nv, mn, mx, orx = 0.0, 0, 0xFFFFFFFF, 0, 0
        for p in parts:  # rank order: the same sum on every rank
            sm += p[s][0]
            nv += p[s][1]
            mn, mx, orx = min(mn, p[s][2]), max(mx, p[s][3]), orx | p[s][4]
        shift, dw, _ = dig[s]
        lo = _ctz(orx)
        pos, frac = positions(nv, pct)
        hb = shift + dw
        high = 0 if hb >= 32 else (mn >> hb) << hb
        pre, res = [high] * RANKS, list(pos)
        if nv and dw:
            c = np.cumsum(hist0[s, : 1 << dw].astype(np.int64))
            for q in range(RANKS):
                d = int(np.searchsorted(c, res[q], side="right"))
                res[q] -= int(c[d - 1]) if d else 0
                pre[q] |= d << shift
        state.append({"nv": nv, "sum": sm, "min": mn, "max": mx, "lo": lo, "shift": shift, "pre": pre, "res": res,
                      "width": _next_width(shift, lo) if nv else 0, "frac": frac})
    # 4. passes 1..3
    for _ in range(3):
        histk = np.zeros((S, RANKS, 256), np.uint32)
        for s in range(S):
            st, k = state[s], keys[s]
            w = st["width"]
            if not w or not len(k):
                continue
            fsh, ns = st["shift"], st["shift"] - w
            digit = ((k >> np.uint64(ns)) & np.uint64((1 << w) - 1)).astype(np.int64)
            for q in range(RANKS):
                m = (k >> np.uint64(fsh)) == np.uint64(st["pre"][q] >> fsh)
                histk[s, q, : 1 << w] = np.bincount(digit[m], minlength=1 << w)
        histk = allreduce_sum(histk)
        for s in range(S):
            st = state[s]
            w = st["width"]
            if w:
                ns = st["shift"] - w
                for q in range(RANKS):
                    c = np.cumsum(histk[s, q, : 1 << w].astype(np.int64))
                    d = int(np.searchsorted(c, st["res"][q], side="right"))
                    st["res"][q] -= int(c[d - 1]) if d else 0
                    st["pre"][q] |= d << ns
                st["shift"] = ns
            st["width"] = _next_width(st["shift"], st["lo"]) if st["nv"] else 0
    for s in range(S):
        st = state[s]
        out[s, 7] = st["nv"]
        if not st["nv"]:
            continue
        assert st["width"] == 0, "every varying bit resolved within 4 passes"
        low = st["min"] & ~((0xFFFFFFFF << st["shift"]) & 0xFFFFFFFF)
        out[s, 0], out[s, 1] = kfloat(st["min"]), kfloat(st["max"])
        out[s, 2] = np.float32(st["sum"] / st["nv"])
        for q in range(3):
            x0, x1 = kfloat(st["pre"][2 * q] | low), kfloat(st["pre"][2 * q + 1] | low)
            f = st["frac"][q]
            out[s, 3 + q] = np.float32(x1 - (x1 - x0) * (1.0 - f) if f >= 0.5 else x0 + (x1 - x0) * f)
    return out
