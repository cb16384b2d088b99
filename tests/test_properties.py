"""Property-based tests (hypothesis): the exposition text format round-trips arbitrary
label values and floats, the query layer's long->wide step agrees with a pandas pivot
(the reference's app.py:204-207) on arbitrary instant vectors, and the fp64 window
statistics agree with the PyTorch reference on arbitrary windows (NaN included)."""

import math

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from rocmdash.ops.window_stats import window_stats_reference, window_stats_torch
from rocmdash.prom.exposition import Exposition, parse_text
from rocmdash.prom.query import _long_to_wide

FAST = settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])

label_text = st.text(alphabet=st.characters(blacklist_categories=("Cs",)), max_size=12)
finite = st.floats(allow_nan=False, allow_infinity=False, width=64)
any_float = st.floats(allow_nan=True, allow_infinity=True, width=64)


@FAST
@given(values=st.lists(st.tuples(label_text, any_float), min_size=1, max_size=8))
def test_exposition_round_trip(values):
    exp = Exposition()
    for i, (lab, v) in enumerate(values):
        exp.add("rocmdash_prop", v, {"k": lab, "i": str(i)}, "property test")
    parsed = {s.label_dict()["i"]: s for s in parse_text(exp.text()) if s.name == "rocmdash_prop"}
    assert len(parsed) == len(values)
    for i, (lab, v) in enumerate(values):
        s = parsed[str(i)]
        assert s.label_dict()["k"] == lab
        if math.isnan(v):
            assert math.isnan(s.value)
        else:
            assert s.value == v


@FAST
@given(rows=st.lists(st.tuples(st.integers(0, 11), st.sampled_from(
    ["amd_gpu_edge_temperature", "amd_gpu_gfx_activity", "amd_gpu_used_vram", "amd_gpu_total_vram"]), finite),
    min_size=1, max_size=40))
def test_long_to_wide_matches_pandas_pivot(rows):
    pd = pytest.importorskip("pandas")
    result = [{"metric": {"__name__": m, "gpu_id": str(g), "card_model": "102-G36236-0C"}, "value": [0, repr(v)]}
              for g, m, v in rows]
    df = pd.DataFrame([{"gpu_id": str(g), "metric_name": m, "value": v} for g, m, v in rows])
    try:
        ref = df.pivot(index="gpu_id", columns="metric_name", values="value")
    except ValueError:
        with pytest.raises(ValueError):
            _long_to_wide(result)
        return
    names = set(df["metric_name"])
    if not {"amd_gpu_used_vram", "amd_gpu_total_vram"} <= names:
        with pytest.raises(KeyError):
            _long_to_wide(result)
        return
    gpu_ids, models, columns, table = _long_to_wide(result)
    assert gpu_ids == list(ref.index) and list(columns) == list(ref.columns)
    np.testing.assert_array_equal(np.array(table, dtype=float), ref.to_numpy(dtype=float))


@FAST
@given(x=st.lists(st.lists(st.one_of(st.floats(-1e6, 1e6, width=32), st.just(float("nan"))), min_size=1, max_size=60),
                  min_size=1, max_size=4),
       pct=st.tuples(st.floats(0, 100), st.floats(0, 100), st.floats(0, 100)))
def test_window_stats_reference_matches_torch(x, pct):
    torch = pytest.importorskip("torch")
    n = min(len(r) for r in x)
    a = np.array([r[:n] for r in x], dtype=np.float32)
    ref = window_stats_reference(a, pct)
    got = window_stats_torch(torch.from_numpy(a), pct).numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-6, equal_nan=True)


def _promql_quote(v: str) -> str:
    return '"' + v.replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n") + '"'


@FAST
@given(value=label_text, other=label_text)
def test_promql_string_literals_round_trip(value, other):
    """An equality matcher on any label value (quotes, backslashes, newlines, Unicode)
    selects exactly the series carrying that value."""
    from rocmdash.prom.promql import parse

    sel = parse("{__name__=\"amd_gpu_gfx_activity\", gpu_id=" + _promql_quote(value) + "}")
    assert sel.matches({"__name__": "amd_gpu_gfx_activity", "gpu_id": value})
    assert sel.matches({"__name__": "amd_gpu_gfx_activity", "gpu_id": other}) == (other == value)


@settings(max_examples=40, deadline=None)
@given(ops=st.lists(st.one_of(st.tuples(st.just("push"), st.integers(0, 70)),
                              st.tuples(st.just("read"), st.integers(0, 80))), min_size=1, max_size=30))
def test_series_ring_matches_a_list_model(native, ops):
    """SeriesRing (csrc/ring.h) against a plain list: after any sequence of pushes,
    window(n) returns the newest min(n, pushed, capacity) rows, oldest first."""
    cap, width = 32, 3
    ring = native.SeriesRing(width, cap)
    model = []
    t = 0
    for op, k in ops:
        if op == "push":
            rows = np.arange(t * width, (t + k) * width, dtype=np.float32).reshape(k, width)
            if k:
                ring.push_many(rows, np.arange(t, t + k, dtype=np.uint64))
            model.extend(rows.tolist())
            t += k
        else:
            got, ts = ring.window(k)
            want = model[-min(k, cap, len(model)):] if k and model else []
            assert got.shape == (len(want), width)
            np.testing.assert_array_equal(got, np.array(want, dtype=np.float32).reshape(-1, width))
            np.testing.assert_array_equal(ts, np.arange(t - len(want), t, dtype=np.uint64))
    assert ring.head == t
