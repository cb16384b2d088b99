"""CPU model of the long-window kernel's adaptive digit schedule (csrc/long_window.hip).

The kernel resolves only the key bits that vary over the window: pass 0 histograms a
digit of 8 or 10 bits just below the top bit of a PREDICTED range (a superset of the true
range), later passes take <= 8-bit digits down to the lowest bit any key differs in from a
reference key, and the bits below that are filled from min's. This model repeats that
arithmetic in numpy - same key transform, same prefix / shift / width bookkeeping as
``lw_scan`` - and checks every selected rank against ``np.sort``, for predictions that are
exact, wider than needed or absent, reference keys that are or are not window members,
and data from one distinct value to all 32 key bits. The GPU tests
(tests/test_gpu_long_window.py) check the kernel itself against the fp64 reference."""

import numpy as np
import pytest


def _keys(x: np.ndarray) -> np.ndarray:
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000).astype(np.uint64)


def _kfloat(k: int) -> np.float32:
    u = (k & 0x7FFFFFFF) if (k & 0x80000000) else (~k & 0xFFFFFFFF)
    return np.array([u], np.uint32).view(np.float32)[0]


def _next_width(shift: int, lo: int) -> int:
    return min(8, shift - lo) if shift > lo else 0


def _pass0_digit(pmin: int, pmax: int, plo: int) -> tuple[int, int]:
    d = pmin ^ pmax
    top = d.bit_length() - 1 if d else 0
    span = top - plo + 1 if top >= plo else 1
    passes = lambda dw: (span - dw + 7) // 8 if span > dw else 0  # noqa: E731
    dw = 10 if passes(10) < passes(8) else 8
    return (top - (dw - 1) if top >= dw - 1 else 0), dw


def _select(x: np.ndarray, ranks, pmin: int, pmax: int, plo: int, ref: int):
    k = _keys(x[~np.isnan(x)])
    shift, dw = _pass0_digit(pmin, pmax, plo)
    mn = int(k.min())
    orx = int(np.bitwise_or.reduce(k ^ np.uint64(ref)))
    lo = (orx & -orx).bit_length() - 1 if orx else 32
    hb = shift + dw
    high = 0 if hb >= 32 else (mn >> hb) << hb
    out, passes = [], 1
    for r in ranks:
        pre, res = high, r
        h = np.bincount(((k >> np.uint64(shift)) & np.uint64((1 << dw) - 1)).astype(np.int64), minlength=1 << dw)
        c = np.cumsum(h)
        dg = int(np.searchsorted(c, res, side="right"))
        res -= int(c[dg - 1]) if dg else 0
        pre |= dg << shift
        sh, width, n = shift, _next_width(shift, lo), 1
        for _ in range(3):
            if width:
                m = (k >> np.uint64(sh)) == np.uint64(pre >> sh)
                ns = sh - width
                h = np.bincount(((k[m] >> np.uint64(ns)) & np.uint64((1 << width) - 1)).astype(np.int64), minlength=256)
                c = np.cumsum(h)
                dg = int(np.searchsorted(c, res, side="right"))
                res -= int(c[dg - 1]) if dg else 0
                pre |= dg << ns
                sh, n = ns, n + 1
            width = _next_width(sh, lo)
        assert width == 0, "every varying bit resolved within 4 passes"
        out.append(_kfloat(pre | (mn & ~((0xFFFFFFFF << sh) & 0xFFFFFFFF))))
        passes = max(passes, n)
    return out, passes


_GENS = {
    "continuous": lambda rng, n: rng.normal(50, 10, n),
    "telemetry": lambda rng, n: rng.integers(40, 56, n).astype(float),
    "tiny": lambda rng, n: rng.normal(0, 1e-3, n),
    "signed_zeros": lambda rng, n: rng.choice([-0.0, 0.0, -1.5, 3.25], n),
    "constant": lambda rng, n: np.full(n, 42.0),
    "heavy_tail": lambda rng, n: rng.standard_cauchy(n) * 1e6,
    "decades": lambda rng, n: rng.integers(-5, 5, n) * 2.0 ** rng.integers(-30, 30, n),
}


@pytest.mark.parametrize("shape", sorted(_GENS))
def test_adaptive_digits_select_exact_ranks(shape):
    rng = np.random.default_rng(7)
    for trial in range(30):
        n = int(rng.integers(1, 3000))
        x = _GENS[shape](rng, n).astype(np.float32)
        x[rng.random(n) < 0.05] = np.nan
        v = x[~np.isnan(x)]
        if len(v) == 0:
            continue
        k = _keys(v)
        mode = trial % 3
        if mode == 0:  # no prediction: the top byte
            pmin, pmax, plo = 0, 0xFFFFFFFF, 0
        elif mode == 1:  # exact
            pmin, pmax = int(k.min()), int(k.max())
            o = int(np.bitwise_or.reduce(k ^ k[0]))
            plo = (o & -o).bit_length() - 1 if o else 32
        else:  # a superset: wider range, lower bit
            pmin = max(0, int(k.min()) - int(rng.integers(0, 1 << 20)))
            pmax = min(0xFFFFFFFF, int(k.max()) + int(rng.integers(0, 1 << 20)))
            plo = 0
        ref = int(k[rng.integers(0, len(k))]) if trial % 2 else int(rng.integers(0, 1 << 32))
        ranks = sorted({0, len(v) - 1, len(v) // 2, int(rng.integers(0, len(v)))})
        got, _ = _select(x, ranks, pmin, pmax, plo, ref)
        s = np.sort(v)
        assert [float(g) for g in got] == [float(s[r]) for r in ranks], (shape, trial)


def test_integer_telemetry_takes_one_pass_continuous_takes_four():
    """What the schedule buys: an integer band with an exact prediction resolves in pass 0;
    mixed-sign continuous data keeps four passes."""
    rng = np.random.default_rng(1)
    tele = rng.integers(700, 760, 5000).astype(np.float32)
    k = _keys(tele)
    o = int(np.bitwise_or.reduce(k ^ k[0]))
    _, p = _select(tele, [2500], int(k.min()), int(k.max()), (o & -o).bit_length() - 1, int(k[0]))
    assert p == 1
    cont = rng.normal(0, 1, 5000).astype(np.float32)
    k = _keys(cont)
    _, p = _select(cont, [2500], int(k.min()), int(k.max()), 0, int(k[0]))
    assert p == 4
