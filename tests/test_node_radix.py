"""Node-wide long-window statistics by a distributed radix select
(rocmdash.parallel.node_radix, the host model of ``LongWindowSet.refresh_node``): only
predictions, partials and digit histograms cross the ranks, and every rank ends with the
same exact order statistics of the UNION of the ranks' windows - checked against the fp64
reference on the union, for 1..8 ranks (threads with an in-process collective), and for
8 gloo ranks through ``NodeWindowStats`` with long-window agents."""

import os
import socket
import threading

import numpy as np
import pytest
import torch.multiprocessing as mp

from rocmdash.ops.window_stats import window_stats_reference
from rocmdash.parallel.node_radix import combine_predictions, fkey, node_radix_select, pass0_digit

PCT = (50.0, 90.0, 99.0)


class _Group:
    """Collectives between threads: all-gather (rank order) and a summing all-reduce."""

    def __init__(self, n):
        self.n = n
        self.bar = threading.Barrier(n)
        self.slots = [None] * n

    def allgather(self, rank, obj):
        self.slots[rank] = obj
        self.bar.wait()
        out = list(self.slots)
        self.bar.wait()
        return out

    def allreduce(self, rank, a):
        got = self.allgather(rank, a)
        return np.sum(np.stack(got).astype(np.uint64), axis=0).astype(np.uint32)


def _run(xs, pct=PCT, preds=None):
    n = len(xs)
    g = _Group(n)
    outs = [None] * n
    errs = []

    def work(r):
        try:
            outs[r] = node_radix_select(xs[r], pct, lambda o: g.allgather(r, o), lambda a: g.allreduce(r, a),
                                        None if preds is None else preds[r])
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            g.bar.abort()

    th = [threading.Thread(target=work, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return outs


def _reference(xs, pct=PCT):
    S = xs[0].shape[0]
    ref = np.full((S, 8), np.nan)
    for s in range(S):
        v = np.concatenate([x[s][~np.isnan(x[s])] for x in xs]).astype(np.float64)
        st = window_stats_reference(v[None, :] if len(v) else np.full((1, 1), np.nan), pct)[0]
        st[6] = np.nan
        st[7] = len(v)
        ref[s] = st
    return ref


def _data(rng, ranks, n):
    xs = []
    for r in range(ranks):
        x = np.empty((7, n), np.float32)
        x[0] = rng.normal(50 + 5 * r, 10, n)  # continuous, shifted per rank
        x[1] = rng.integers(40, 56, n)  # integer telemetry
        x[2] = 42.0 if r % 2 else 43.0  # a constant per rank, different across ranks
        x[3] = rng.choice(np.array([-0.0, 0.0, -1.5, 3.25], np.float32), n)  # signed zeros
        x[4] = rng.standard_cauchy(n) * 1e6  # heavy tail, both signs
        x[5] = np.nan if r == 0 else rng.normal(0, 1e-3, n)  # a rank with no samples
        x[6] = rng.normal(1e-30, 1e-31, n)  # tiny magnitudes
        x[rng.random((7, n)) < 0.05] = np.nan
        xs.append(x)
    return xs


@pytest.mark.parametrize("ranks", [1, 2, 3, 8])
def test_matches_the_union_reference(ranks):
    rng = np.random.default_rng(ranks)
    xs = _data(rng, ranks, 3000)
    outs = _run(xs)
    ref = _reference(xs)
    for o in outs:  # every rank holds the same statistics
        np.testing.assert_array_equal(np.nan_to_num(o, nan=-7.0), np.nan_to_num(outs[0], nan=-7.0))
    order = [0, 1, 3, 4, 5, 7]  # order statistics and count: exact
    np.testing.assert_array_equal(outs[0][:, order], np.float32(ref[:, order]).astype(np.float64))
    np.testing.assert_allclose(outs[0][:, 2], ref[:, 2], rtol=1e-5, atol=1e-30)
    assert np.isnan(outs[0][:, 6]).all()  # no node-wide "last"


def test_other_percentiles_and_uneven_ranks():
    rng = np.random.default_rng(9)
    xs = [rng.normal(0, 1, (2, n)).astype(np.float32) for n in (1, 17, 4096, 250)]
    pct = (5.0, 25.0, 75.0)
    outs = _run(xs, pct)
    ref = _reference(xs, pct)
    np.testing.assert_array_equal(outs[0][:, [0, 1, 3, 4, 5, 7]], np.float32(ref[:, [0, 1, 3, 4, 5, 7]]))


def test_predictions_exact_or_wider_give_the_same_result():
    """Each rank's pass-0 prediction only has to be a superset of its varying bits: an
    exact one (10-bit digit on integer telemetry: one pass fewer), a wider one or none
    give the same bits."""
    rng = np.random.default_rng(5)
    xs = [rng.integers(40, 56, (1, 2000)).astype(np.float32) for _ in range(4)]
    exact = []
    for x in xs:
        k = fkey(x[0])
        orx = int(np.bitwise_or.reduce(k ^ k[-1]))
        exact.append([(int(k.min()), int(k.max()), (orx & -orx).bit_length() - 1 if orx else 32)])
    wide = [[(p[0][0] - 1000, p[0][1] + 1000, 0)] for p in exact]
    a, b, c = _run(xs, preds=exact)[0], _run(xs, preds=wide)[0], _run(xs)[0]
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(a, c)
    # the combined exact prediction of telemetry in [40, 56) is resolved by pass 0 alone:
    # its digit reaches down to the lowest varying bit
    pm = combine_predictions([(p[0][0], p[0][1], p[0][2], int(fkey(x[0])[-1]), True) for p, x in zip(exact, xs)])
    shift, width = pass0_digit(pm[0], pm[1], pm[2])
    assert shift <= pm[2] < shift + width


def test_combine_predictions_counts_reference_differences():
    """Ranks whose reference keys differ add the differing bits to the varying range;
    a rank without samples contributes no reference."""
    a = (100, 200, 32, 0x80000010, True)
    b = (150, 180, 32, 0x80000011, True)
    empty = (0, 0xFFFFFFFF, 0, 0, False)
    assert combine_predictions([a, b]) == (100, 200, 0, 0x80000010)
    assert combine_predictions([a, (150, 180, 32, 0x80000018, True)])[2] == 3
    assert combine_predictions([empty, b]) == (0, 0xFFFFFFFF, 0, 0x80000011)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import torch.distributed as dist

        from rocmdash.config import SamplerConfig
        from rocmdash.parallel.node import NodeAggregator, dist_env_from_environ
        from rocmdash.parallel.node_window import NodeWindowStats
        from rocmdash.runtime.agent import GpuAgent

        env = dist_env_from_environ(prefer_gpu=False)
        agg = NodeAggregator()
        cfg = SamplerConfig(window=1 << 15 << 1, ring_capacity=1 << 16)  # 65536: a long window
        assert cfg.long_window
        agent = GpuAgent(rank, source="synthetic", counters="synthetic", cfg=cfg, use_gpu=False, seed=100 + rank)
        agent.prefill(300 + 97 * rank)  # uneven windows
        nws = NodeWindowStats(agent, agg)
        got = nws.refresh()
        x = nws._local_rows()
        xs = agg.all_gather_object(x)
        res = None
        if rank == 0:
            ref = _reference(xs, tuple(agent.pct))
            g = got.numpy().astype(np.float64)
            order = [0, 1, 3, 4, 5, 7]
            res = (np.array_equal(np.float32(g[:, order]), np.float32(ref[:, order]), equal_nan=True),
                   bool(np.allclose(g[:, 2], ref[:, 2], rtol=1e-5, equal_nan=True)), int(g[0, 7]))
        else:
            res = got is None
        agent.close()
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, None, traceback.format_exc()))


@pytest.mark.slow
def test_node_window_long_gloo_8_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world, port = 8, _free_port()
    ps = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    errs = [e for _, _, e in got if e]
    assert not errs, errs[0]
    res = dict((r, v) for r, v, _ in got)
    assert res[0][0] and res[0][1], res[0]
    assert res[0][2] == sum(300 + 97 * r for r in range(world))  # every rank's window counted
    assert all(res[r] is True for r in range(1, world))
