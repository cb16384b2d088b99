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


def _run(stream, W, steps, incremental=False):
    m = BracketModel(incremental=incremental)
    hits = []
    t = 0
    for i, k in enumerate(steps):
        t += k
        w = stream[max(0, t - W):t]
        got, hit = m.refresh(w, entered=k if i else None)
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


@pytest.mark.parametrize("shape", ["continuous", "mixed", "telemetry"])
def test_incremental_brackets_stay_put(shape):
    """Incremental mode (the kernels' default): 100 rows per refresh into a full window,
    every refresh exact; after the brackets are sized they resolve every refresh and are
    hardly ever re-centred - so pass B streams only the chunks the new rows landed in.
    Integer telemetry takes brackets too (one-key brackets on tied values)."""
    rng = np.random.default_rng(9)
    W = 1 << 15
    if shape == "telemetry":
        x = rng.integers(40, 56, 3 * W).astype(np.float32)
    elif shape == "mixed":
        x = rng.normal(0, 10, 3 * W).astype(np.float32)
    else:
        x = rng.normal(50, 10, 3 * W).astype(np.float32)
    steps = [W] + [100] * 150
    m, hits = _run(x, W, steps, incremental=True)
    assert all(hits[12:]), [i for i, h in enumerate(hits) if not h]
    moves_late = m.moves
    m2, _ = _run(x, W, steps[:40], incremental=True)
    # after sizing, re-centring is rare: the percentiles drift by ~sqrt(100) ranks a refresh
    assert moves_late - m2.moves <= 6, (moves_late, m2.moves)


def test_incremental_recentres_on_a_jump():
    """A level jump moves every percentile out of its bracket: a miss (the radix chain),
    then new brackets that resolve again."""
    rng = np.random.default_rng(6)
    W = 1 << 13
    x = rng.normal(50, 10, 5 * W).astype(np.float32)
    x[2 * W:] += 1000.0  # rows from 2W on jumped: the p99 leaves its bracket first
    steps = [W] + [256] * 100  # ends with a window of jumped rows only
    m, hits = _run(x, W, steps, incremental=True)
    ends = np.cumsum(steps)
    first_jumped = int(np.argmax(ends > 2 * W))
    assert all(hits[3:first_jumped]), hits  # steady before the jump
    assert not all(hits[first_jumped:first_jumped + 8]), hits  # the jump takes the radix chain
    assert all(hits[-5:]), hits  # re-centred brackets resolve again


# ---- node bracket mode (the host model of refresh_node's bracket path) ----------------


class _Group:
    """Collectives between threads: all-gather (rank order) and a summing all-reduce."""

    def __init__(self, n):
        import threading

        self.n = n
        self.bar = threading.Barrier(n)
        self.slots = [None] * n
        self.gathers = [0] * n

    def allgather(self, rank, obj):
        self.gathers[rank] += 1
        self.slots[rank] = obj
        self.bar.wait()
        out = list(self.slots)
        self.bar.wait()
        return out

    def allreduce(self, rank, a):
        got = self.allgather(rank, a)
        return np.sum(np.stack(got).astype(np.uint64), axis=0).astype(np.uint32)


def _node_stream(nranks, shape, steps, W, seed):
    """Every rank's window after each step (sliding, W samples per rank)."""
    rng = np.random.default_rng(seed)
    wins = [np.zeros(0, np.float32) for _ in range(nranks)]
    out = []
    for k in steps:
        for r in range(nranks):
            if shape == "telemetry":
                x = rng.integers(40 + r, 56 + r, k).astype(np.float32)
            elif shape == "cauchy":  # heavy tails: the first estimate's bracket overflows
                x = (rng.standard_cauchy(k) * 1e5 + r).astype(np.float32)
            elif shape == "drift":
                x = rng.normal(100 + 10 * r + 0.01 * len(out), 15, k).astype(np.float32)
            else:
                x = rng.normal(100 + 10 * r, 20, k).astype(np.float32)
            x[rng.random(k) < 0.02] = np.nan
            wins[r] = np.concatenate([wins[r], x])[-W:]
        out.append([w.copy() for w in wins])
    return out


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
@pytest.mark.parametrize("shape", ["continuous", "telemetry", "drift", "cauchy"])
def test_node_brackets_exact_and_hit(nranks, shape):
    """Every rank ends each refresh with the SAME statistics (the union's, exactly) and the
    SAME next brackets; after the sizing refreshes the steady 100-row pushes resolve from
    the brackets - one all-gather per refresh instead of the radix chain's collectives."""
    from rocmdash.ops.window_stats import window_stats_reference
    from rocmdash.runtime.lw_brackets import NODE_CAP, NodeBracketModel, node_cap_next

    W = 1 << 14
    steps = [W] + [100] * 30
    stream = _node_stream(nranks, shape, steps, W, seed=nranks * 7 + len(shape))
    g = _Group(nranks)
    models = [NodeBracketModel() for _ in range(nranks)]
    outs = [[None] * len(steps) for _ in range(nranks)]
    caps = [[] for _ in range(nranks)]
    errs = []

    def work(r):
        try:
            cap = NODE_CAP  # the record cap: kNodeCap until a bracket refresh measured the kept keys
            for i, wins in enumerate(stream):
                n0 = models[r].refreshes
                outs[r][i] = models[r].refresh_node(wins[r], lambda o: g.allgather(r, o),
                                                    lambda a: g.allreduce(r, a), entered=steps[i], cap=cap)
                if models[r].refreshes > n0:  # a bracket refresh: the next cap from its counts
                    cap = node_cap_next(models[r].maxmid, nranks)
                caps[r].append(cap)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            g.bar.abort()

    import threading

    th = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert not errs, errs
    for i, wins in enumerate(stream):
        union = np.concatenate(wins)
        exp = window_stats_reference(union[None, :])[0]
        for r in range(nranks):
            got, _ = outs[r][i]
            assert np.array_equal(np.float32(got[[0, 1, 7]]), np.float32(exp[[0, 1, 7]]), equal_nan=True), (i, r)
            # percentiles: two exact order statistics, lerped in fp64 and rounded to float32
            # (numpy's lerp may round a midpoint the other way: 1 ulp)
            g32, e32 = np.float32(got[3:6]), np.float32(exp[3:6])
            assert np.all(np.abs(g32 - e32) <= np.spacing(np.abs(e32))), (i, r, g32, e32)
            assert np.isclose(got[2], exp[2], rtol=1e-6) and np.isnan(got[6])
            assert np.array_equal(got, outs[0][i][0], equal_nan=True)  # the same bits on every rank
    for m in models[1:]:
        assert (m.lo, m.hi, m.delta, m.valid) == (models[0].lo, models[0].hi, models[0].delta, models[0].valid)
    m = models[0]
    hits = [outs[0][i][1] for i in range(len(steps))]
    assert sum(hits[10:]) >= 18, (shape, hits, m.moves, caps[0])
    # the records shrink to ~2x the kept keys, the same size on every rank
    assert all(c == caps[0] for c in caps)
    if nranks > 1 and shape != "cauchy":
        assert caps[0][-1] <= NODE_CAP // 2, caps[0]


def test_node_cap_next():
    """The record cap mirrors csrc/long_window.hip lw_node_cap_next: 64-key steps, a floor
    of 4x a rank's share of the node target, 2x headroom, at most kNodeCap."""
    from rocmdash.runtime.lw_brackets import NODE_CAP, node_cap_next

    assert node_cap_next(0, 1) == NODE_CAP
    assert node_cap_next(0, 8) == 128 and node_cap_next(0, 4) == 256 and node_cap_next(0, 3) == 384
    assert node_cap_next(100, 8) == 256 and node_cap_next(65, 8) == 192
    assert node_cap_next(5000, 2) == NODE_CAP
    assert all(node_cap_next(m, n) % 64 == 0 for m in range(0, 2000, 7) for n in range(1, 9))
    try:
        from rocmdash.runtime import native

        nat = native.load(with_torch=False)
    except Exception:  # noqa: BLE001 - the native build is checked by its own tests
        return
    # the kernels' host code computes the same caps (every rank's collective size)
    assert all(nat.long_window_node_cap(m, n) == node_cap_next(m, n) for m in range(0, 3000, 5) for n in range(1, 9))


def test_percentile_between_two_tied_values_holds():
    """Integer telemetry whose median sits on the boundary between two readings (16
    equally likely integers: p50 between the 8th and 9th): every sample of both values is
    inside the bracket - far more than the kept-key cap. The bracket narrows to exactly
    the tied key (an overflow reads as ties), the first flip to the neighbouring reading
    joins both keys into one exact bracket, whose ties are COUNTED on its bounds (not
    kept), and then it holds: one miss after sizing, no re-centring."""
    W = 1 << 18
    rng = np.random.default_rng(3)
    x = rng.integers(40, 56, W + 100 * 80).astype(np.float32)
    m = BracketModel(incremental=True)
    hits = []
    for i in range(81):
        win = x[100 * i: 100 * i + W]
        out, hit = m.refresh(win, entered=W if i == 0 else 100)
        ref = _ref(win)
        assert np.array_equal(np.float32(out[[0, 1, 3, 4, 5, 7]]), np.float32(ref[[0, 1, 3, 4, 5, 7]])), (i, out, ref)
        hits.append(hit)
    assert hits[2:].count(False) <= 1 and all(hits[20:]), [i for i, h in enumerate(hits) if not h]
    assert m.delta[0] == 0.0 and m.lo[0] != m.hi[0], (m.lo, m.hi, m.delta)  # two tied keys, counted
    assert m.moves == 0
