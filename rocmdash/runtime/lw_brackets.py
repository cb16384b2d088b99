"""Bracket mode of the long-window statistics: the host model of ``lw_pass_brk`` +
``lw_scan_brk`` (csrc/long_window.hip "Bracket mode").

A window of W samples per series changes by the few rows that entered and left since the
previous refresh, so each percentile moves by a few ranks. The previous refresh's
percentile keys, widened by an adaptive half-width, bracket the new ones. One streaming
pass counts, per percentile q, the samples below the bracket (``lt``) and inside it
(``inn``) and keeps the keys inside; when both sorted positions of every percentile fall
inside their brackets (``lt <= pos < lt + inn``), the percentiles are order statistics of
the kept keys. Otherwise the exact radix chain resolves the series in the same refresh -
here ``np.partition``, which gives the same keys.

The half-width adapts so a bracket holds about ``target`` samples (2048, or 1/16 of a
small window); a bracket of one key (ties: integer telemetry) keeps holding while the
ties cover the rank. Brackets are only wanted where the radix chain needs more than one
streaming pass (the varying key bits span more than pass 0's 10-bit digit).

``BracketModel.refresh(x)`` returns the same [8] statistics as ``window_stats_reference``
(min, max, mean, p50 / p90 / p99 by numpy's 'linear' rule, last, count) and whether the
brackets resolved the refresh; ``tests/test_lw_brackets.py`` checks both against numpy
over stationary, drifting, jumping and tied data.

Reference anchor: the statistics table over a window (``/root/reference/app.py:216-221``).
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

TARGET = 2048  # kBrkTarget
CAP = 8192  # kBrkCap: kept keys scan B selects among
KD0 = 10  # pass 0's widest digit
PCT = (50.0, 90.0, 99.0)


def fkey(x: np.ndarray) -> np.ndarray:
    """Order-preserving float32 -> uint32 key (csrc/long_window.hip ``fkey``)."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000).astype(np.uint64)


def kfloat(k: int) -> float:
    u = (k & 0x7FFFFFFF) if (k & 0x80000000) else (~k & 0xFFFFFFFF)
    return float(np.array([u], np.uint32).view(np.float32)[0])


def positions(nv: int, pct=PCT):
    """Sorted positions (lo, hi) and float32 weights of each percentile (lw_positions)."""
    last = nv - 1 if nv else 0
    out = []
    for p in pct:
        x = float(p) / 100.0 * float(last)
        lo = min(int(np.floor(x)), last)
        out.append((lo, lo + 1 if lo + 1 < nv else last, float(np.float32(x - lo))))
    return out


def target(nv: int) -> int:
    return max(64, min(TARGET, nv // 16))


def wanted(nv: int, minkey: int, maxkey: int, lo: int) -> bool:
    """Brackets pay when the radix chain needs more than one pass (lw_brk_wanted)."""
    d = minkey ^ maxkey
    top = d.bit_length() - 1 if d else 0
    span = top - lo + 1 if top >= lo else 1
    return bool(nv) and span > KD0


def next_bracket(delta: int, cin: int, klo: int, khi: int, est: int, had: bool, tgt: int):
    """(delta, lo, hi) of the next refresh's bracket (lw_next_bracket)."""
    if not had:
        d = est
    elif delta == 0:
        d = 0 if cin >= tgt // 8 else est
    else:
        d = int(float(delta) * min(8.0, float(tgt) / float(max(cin, 1))))
    d = min(d, 0x7FFFFFFF)
    return d, (klo - d if klo > d else 0), min(0xFFFFFFFF, khi + d)


@dataclass
class BracketModel:
    """One series' bracket state across refreshes."""

    lo: list = field(default_factory=lambda: [0, 0, 0])
    hi: list = field(default_factory=lambda: [0, 0, 0])
    delta: list = field(default_factory=lambda: [0, 0, 0])
    cin: list = field(default_factory=lambda: [0, 0, 0])
    valid: bool = False
    refreshes: int = 0
    hits: int = 0

    def refresh(self, window: np.ndarray, pct=PCT):
        """Statistics of ``window`` (float32 samples, NaN = none) and whether the brackets
        resolved them (else the radix chain did)."""
        x = np.asarray(window, np.float32)
        x = x[~np.isnan(x)]
        nv = int(x.size)
        out = np.full(8, np.nan)
        out[7] = nv
        if not nv:
            self.valid = False
            return out, False
        k = fkey(x)
        minkey, maxkey = int(k.min()), int(k.max())
        newest = np.float32(np.asarray(window, np.float32)[-1])
        ref = 0 if np.isnan(newest) else int(fkey(np.array([newest]))[0])  # orx's reference: the newest row
        orx = int(np.bitwise_or.reduce(k ^ np.uint64(ref)))
        lov = (orx & -orx).bit_length() - 1 if orx else 32
        pos = positions(nv, pct)
        tgt, est = target(nv), max(1, (maxkey - minkey) * target(nv) // (2 * nv))
        hit = False
        keys = [None] * 3
        if self.valid:  # pass B + scan B
            self.refreshes += 1
            lt = [int(np.count_nonzero(k < np.uint64(self.lo[q]))) for q in range(3)]
            inside = [k[(k >= np.uint64(self.lo[q])) & (k <= np.uint64(self.hi[q]))] for q in range(3)]
            inn = [int(v.size) for v in inside]
            hit = all(lt[q] <= pos[q][0] and pos[q][1] < lt[q] + inn[q]
                      and (self.lo[q] == self.hi[q] or inn[q] <= CAP) for q in range(3))
            self.cin = inn
            if hit:
                for q in range(3):
                    s = np.sort(inside[q])
                    keys[q] = (int(s[pos[q][0] - lt[q]]), int(s[pos[q][1] - lt[q]]))
                self.hits += 1
        if not hit:  # the radix chain: exact keys at the sorted positions
            ks = np.sort(k)
            keys = [(int(ks[lo]), int(ks[hi])) for lo, hi, _ in pos]
        had = self.valid
        for q in range(3):
            self.delta[q], self.lo[q], self.hi[q] = next_bracket(self.delta[q], self.cin[q], keys[q][0], keys[q][1],
                                                                 est, had, tgt)
        self.valid = wanted(nv, minkey, maxkey, lov)
        out[0], out[1] = kfloat(minkey), kfloat(maxkey)
        out[2] = np.float32(np.sum(x, dtype=np.float64) / nv)
        for q, (lo, hi, f) in enumerate(pos):
            x0, x1 = kfloat(keys[q][0]), kfloat(keys[q][1])
            out[3 + q] = np.float32(x1 - (x1 - x0) * (1.0 - f) if f >= 0.5 else x0 + (x1 - x0) * f)
        out[6] = float(newest)
        return out, hit
