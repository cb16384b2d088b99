"""Bracket mode of the long-window statistics, host model (rocmdash/runtime/lw_brackets.py
mirrors lw_pass_brk + lw_scan_brk): every refresh exact against numpy, brackets resolving
the steady state of continuous data, missing - and the radix chain taking over - on a
jump, and never asked for by integer telemetry that pass 0 resolves in one pass."""

import numpy as np
import pytest

from rocmdash.runtime.lw_brackets import BracketModel, wanted, fkey


def _ref(w):
    from rocmdash.ops.window_stats import window_stats_reference

    return window_stats_reference(np.asarray(w, np.float32)[None, :])[0]


def _run(stream, W, steps):
    m = BracketModel()
    hits = []
    t = 0
    for k in steps:
        t += k
        w = stream[max(0, t - W):t]
        got, hit = m.refresh(w)
        np.testing.assert_allclose(got, _ref(w), rtol=1e-6, atol=1e-6, equal_nan=True)
        hits.append(hit)
    return m, hits


def test_steady_state_continuous_hits():
    rng = np.random.default_rng(1)
    W = 1 << 16
    x = rng.normal(50, 10, 3 * W).astype(np.float32)
    m, hits = _run(x, W, [W] + [1, 3, 0, 100, 1, 7, 1, 1, 50, 1] * 2)
    assert not hits[0] and all(hits[4:]), hits  # a few refreshes size the brackets
    assert m.valid and max(m.cin) <= 4 * 2048


def test_jump_misses_then_recovers():
    rng = np.random.default_rng(2)
    W = 1 << 14
    x = rng.normal(50, 10, 4 * W).astype(np.float32)
    x[2 * W:] += 1000.0  # the level jumps: the old brackets hold no percentile
    steps = [W] + [64] * 8 + [W] + [64] * 12  # the 10th refresh brings 512 jumped rows: p99 leaves
    _, hits = _run(x, W, steps)
    assert any(hits[:9]) and not hits[9] and hits[-1], hits


def test_integer_telemetry_stays_on_the_one_pass_radix_chain():
    rng = np.random.default_rng(3)
    W = 1 << 14
    x = rng.integers(40, 56, 2 * W).astype(np.float32)
    m, hits = _run(x, W, [W] + [10] * 10)
    assert not any(hits) and not m.valid
    k = fkey(x[:W])
    assert not wanted(W, int(k.min()), int(k.max()), 18)  # 5 varying bits


@pytest.mark.parametrize("seed", [4, 5])
def test_nan_stretches_and_spikes_stay_exact(seed):
    rng = np.random.default_rng(seed)
    W = 4096
    x = rng.normal(0, 1, 6 * W).astype(np.float32)
    x[rng.random(x.size) < 0.01] = -1e6
    x[W:W + 700] = np.nan
    _run(x, W, [W] + list(rng.choice([0, 1, 5, 64, 257, 700], size=30)))
