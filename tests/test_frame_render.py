"""The native frame renderer (csrc/frame_render.cpp) against the Python frame
(rocmdash/viz/panels.py): byte-identical refresh payloads over randomised node
snapshots - NaN readings, idle (zero-power) GPUs, missing metrics, unknown models,
natural-sorted ids, partial / vanished selections, gauge and bar styles, the
extended panels and the window table."""

import json
from datetime import datetime

import numpy as np
import pytest

from rocmdash.models.schema import CTR_FIELDS, SMI_FIELDS, STAT_NAMES
from rocmdash.viz.panels import NodeSnapshot, build_frame, render_frame_json

NOW = datetime(2026, 10, 15, 23, 59, 58, 123456)


def _snapshot(rng, g, cols, models=None, window=True, nan_frac=0.1, zero_power=True, ids=None):
    vals = rng.uniform(0, 1000, size=(g, len(cols)))
    vals[rng.random(vals.shape) < nan_frac] = np.nan
    if "amd_gpu_total_vram" in cols:
        vals[:, cols.index("amd_gpu_total_vram")] = 294896.0
    if zero_power and g and "amd_gpu_average_package_power" in cols:
        vals[rng.integers(0, g), cols.index("amd_gpu_average_package_power")] = 0.0
    vals = np.round(vals, int(rng.integers(0, 4)))
    w = rng.uniform(-5, 500, size=(g, len(cols), len(STAT_NAMES))).astype(np.float32) if window else None
    if w is not None and g:
        w[0, 0, :] = np.nan
    return NodeSnapshot(
        gpu_ids=ids if ids is not None else [str(i) for i in range(g)],
        card_models=models or (["102-G36237-0C"] * g),
        columns=tuple(cols),
        values=vals,
        power_limits=[1400.0 if i % 3 else None for i in range(g)],
        window=w,
        window_series=tuple(cols) if window else (),
    )


@pytest.fixture(scope="module")
def nat():
    from rocmdash.runtime import native

    return native.load(build=True)


@pytest.mark.parametrize("seed", range(40))
def test_native_render_is_byte_identical(nat, seed):
    rng = np.random.default_rng(seed)
    g = int(rng.choice([0, 1, 2, 3, 5, 8, 12]))
    cols = list(SMI_FIELDS + (CTR_FIELDS if seed % 2 else ()))
    if seed % 5 == 0:
        cols.remove("amd_gpu_gfx_activity")  # a metric the node does not report -> literal 0
    models = [["102-G36237-0C", "102-G30211-0C", "999-UNKNOWN", "102-D65209-00"][i % 4] for i in range(g)]
    snap = _snapshot(rng, g, cols, models=models, window=seed % 3 != 0, ids=[str(i) for i in rng.permutation(g)])
    selected = [str(i) for i in range(g) if rng.random() < 0.7] + (["77"] if seed % 4 == 0 else [])
    for use_gauge in (True, False):
        for extended in (False, True):
            ref = build_frame(snap, selected, use_gauge=use_gauge, extended=extended, now=NOW).to_json()
            got = render_frame_json(snap, selected, use_gauge=use_gauge, extended=extended, now=NOW, native=True)
            assert got == ref, (seed, use_gauge, extended)
            json.loads(got)


def test_native_render_all_nan_and_single_gpu(nat):
    cols = list(SMI_FIELDS)
    snap = NodeSnapshot(["0"], ["102-G36237-0C"], tuple(cols), np.full((1, len(cols)), np.nan),
                        window=np.full((1, len(cols), 8), np.nan, np.float32), window_series=tuple(cols))
    for ext in (False, True):
        assert render_frame_json(snap, ["0"], extended=ext, now=NOW, native=True) == build_frame(
            snap, ["0"], extended=ext, now=NOW).to_json()


def test_native_render_is_faster(nat):
    import time

    rng = np.random.default_rng(1)
    snap = _snapshot(rng, 8, list(SMI_FIELDS + CTR_FIELDS))
    for _ in range(20):
        render_frame_json(snap, snap.gpu_ids, native=True)
        build_frame(snap, snap.gpu_ids).to_json()
    t0 = time.perf_counter()
    for _ in range(200):
        render_frame_json(snap, snap.gpu_ids, native=True)
    t_nat = time.perf_counter() - t0
    t0 = time.perf_counter()
    for _ in range(200):
        build_frame(snap, snap.gpu_ids).to_json()
    t_py = time.perf_counter() - t0
    assert t_nat * 2 < t_py, (t_nat, t_py)


def test_py_float_repr_matches_python(nat):
    rng = np.random.default_rng(3)
    vals = np.concatenate([rng.normal(size=2000) * 10.0 ** rng.integers(-20, 20, 2000), [0.0, -0.0, 1e16, 1e-4, 2.5e-5]])
    for x in vals.tolist():
        assert nat.py_float_repr(x) == repr(x)


def test_round2_repr_matches_numpy_round_then_json(nat):
    rng = np.random.default_rng(5)
    vals = np.concatenate([
        rng.normal(size=3000) * 10.0 ** rng.integers(-4, 13, 3000),
        rng.integers(-10**6, 10**6, 500) / 100.0 + 0.005,  # half-way cases
        [0.0, -0.0, -0.001, 0.004999, 0.005, 0.015, 2.675, -2.675, 1e13, 9.99e12, 1e16, -1e14, 123456789.125],
        np.float32(rng.uniform(-5, 500, 500)).astype(np.float64),
    ])
    for x in vals.tolist():
        want = json.dumps(float(np.round(x, 2)))
        assert nat.py_round2_repr(x) == want, (x, want)
    assert nat.py_round2_repr(float("nan")) == "null"


def test_compiled_frame_matches_render_frame_json(nat):
    """CompiledFrame (the refresh loop's renderer) == render_frame_json of the same
    snapshot, for fresh values each refresh, incl. a zero VRAM total."""
    from rocmdash.viz.panels import CompiledFrame

    rng = np.random.default_rng(11)
    cols = SMI_FIELDS + CTR_FIELDS
    for g, ext, gauge in [(1, False, True), (3, True, False), (8, True, True)]:
        first = _snapshot(rng, g, list(cols), window=True)
        cf = CompiledFrame(first, first.gpu_ids, use_gauge=gauge, extended=ext)
        for it in range(5):
            node = rng.uniform(0, 900, size=(g, len(cols), len(STAT_NAMES))).astype(np.float32)
            node[:, cols.index("amd_gpu_total_vram"), 6] = 0.0 if it == 3 else 294896.0
            snap = NodeSnapshot(first.gpu_ids, first.card_models, tuple(cols), node[:, :, 6],
                                power_limits=first.power_limits, window=node, window_series=tuple(cols))
            want = render_frame_json(snap, snap.gpu_ids, use_gauge=gauge, extended=ext, now=NOW, native=True)
            assert cf.render(node[:, :, 6], node, now=NOW) == want, (g, ext, it)
