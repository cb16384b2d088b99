"""Node-wide window statistics: exact order statistics over every GPU's window at once.

Reference counterpart: the statistics over ALL GPUs of ``app.py:216-221`` (mean / max /
min over the GPUs' instant samples). Here, per series, over the union of the last W
samples of all N GPUs: min, max, mean, three percentiles and the sample count - e.g.
the node's p99 junction temperature or p50 xGMI bandwidth over the window.

Per refresh (after every rank's ``GpuAgent.refresh()``):
  1. each rank exports its series' sorted windows as one ``[S, 1 + W]`` block straight
     from the resident sorted state on its GPU (``GpuAgent.export_window``);
  2. ONE all-gather over RCCL / xGMI (the aggregator's native ``ncclAllGather``, the same
     communicator as the stats gather) builds ``[N, S, 1 + W]`` - at N = 8,
     S = 15, W = 4096 that is 246 KB per rank, 1.97 MB per rank received: unlike the
     400-byte stats gather this one is sized by the links, not by latency;
  3. rank 0 selects the order statistics of the union with the rank-selection kernel
     (csrc/node_window.hip), which never re-sorts: each sample finds its merged rank by
     binary searches in the other ranks' sorted lists staged in LDS.
Other ranks take part in the collective and get ``None``.

Windows beyond LDS (W > 32768: HBM-resident ``LongWindowSet``, up to 2^26 samples per
series) are never moved: the node statistics come from a distributed radix select
(``LongWindowSet.refresh_node``, rocmdash.parallel.node_radix) in which only per-series
predictions, partials and digit histograms cross the node - ~0.3 MB per refresh for 16
series at any W, instead of the windows themselves (64 MB per series per rank at 2^24).
Every rank computes the same statistics; rank 0's are returned.
"""

from __future__ import annotations

import numpy as np
import torch

from ..models.schema import NUM_STATS
from ..ops.window_stats import DEFAULT_PCT, window_stats_reference


def node_window_reference(node: np.ndarray, pct=DEFAULT_PCT) -> np.ndarray:
    """fp64 reference: ``node`` [N, S, 1 + W] export blocks -> [S, 8] statistics over
    the union of every rank's valid samples (``last`` is NaN: there is no node-wide
    newest sample)."""
    node = np.asarray(node, dtype=np.float64)
    N, S, _ = node.shape
    out = np.full((S, NUM_STATS), np.nan)
    for s in range(S):
        vals = np.concatenate([node[i, s, 1 : 1 + int(node[i, s, 0])] for i in range(N)])
        st = window_stats_reference(vals[None, :] if len(vals) else np.full((1, 1), np.nan), pct)[0]
        st[6] = np.nan
        st[7] = len(vals)
        if not len(vals):
            st[:6] = np.nan
        out[s] = st
    return out


class NodeWindowStats:
    """Node-wide statistics of every series over all ranks' windows (one collective)."""

    def __init__(self, agent, aggregator, pct=None, collective_timeout_s: float = 60.0):
        self.agent = agent
        self.aggregator = aggregator
        self.pct = tuple(float(p) for p in (pct or agent.pct))
        self.is_root = aggregator.rank == 0
        self.collective_timeout_s = float(collective_timeout_s)
        self._out = None
        self._nat = agent.nat
        self._pub = None  # completion signal behind the native gather (bounded wait)
        self.long = bool(getattr(agent.cfg, "long_window", False))
        # long windows: HIP events around the collective steps of each node refresh
        # (``last_collective_us`` after the refresh; a few µs of events, off by default)
        self.timing = False
        self.last_collective_us = None
        # a NodeWindowStats lives for one membership epoch: every member starts it with
        # the same (empty) node bracket state, whatever the previous epochs left on this
        # rank - a restarted rank and the survivors must take the same branch and size
        # their records alike
        dws = getattr(agent, "dws", None)
        if self.long and dws is not None and hasattr(dws, "reset_node"):
            dws.reset_node()

    def refresh(self):
        """Collective: every rank calls it after its ``agent.refresh()``. Returns the
        ``[S, 8]`` node statistics on rank 0 (a device tensor on GPUs, complete: the
        gather was waited for), ``None`` elsewhere.

        On the native transport the gather (+ rank 0's selection) is followed by a
        completion signal that every rank waits for with a deadline
        (``await_publication``): a peer that died or hung between the stats gather and
        this one makes the refresh raise (communicator aborted) instead of blocking rank
        0's copy of the statistics forever."""
        if self.long:
            return self._refresh_long()
        local = self.agent.export_window()
        node = self.aggregator.all_gather(local)
        out = None
        if self.is_root and node.is_cuda:
            N, S, Wp1 = node.shape
            out = self._out
            if out is None or out.device != node.device or out.shape[0] != S:
                out = self._out = torch.empty((S, NUM_STATS), dtype=torch.float32, device=node.device)
            node = node.contiguous()
            self._nat.node_select(node.data_ptr(), N, S, Wp1 - 1, out.data_ptr(),
                                  torch.cuda.current_stream(node.device).cuda_stream, *self.pct)
        self._await(node)
        if not self.is_root:
            return None
        if out is not None:
            return out
        return torch.from_numpy(node_window_reference(node.numpy(), self.pct).astype(np.float32))

    # csrc/long_window.h LongWindowSet::node_collective_us: a bracket hit runs only the
    # first step, a miss (or no brackets) the radix chain's five
    COLLECTIVE_STEPS = ("bracket_records_allgather", "predictions_allgather",
                        "pass0_partials_allgather+hist_allreduce", "pass1_hist_allreduce", "pass2_hist_allreduce",
                        "pass3_hist_allreduce")

    def _refresh_long(self):
        """Distributed radix select over every rank's long window (see the module
        docstring): on GPUs ``LongWindowSet.refresh_node`` with the collectives on the
        native RCCL communicator, on the CPU the numpy model over the control plane."""
        agg = self.aggregator
        dws = self.agent.dws
        if dws is None:  # CPU: the same algorithm over gloo
            import torch.distributed as dist

            from .node_radix import node_radix_select

            x = self._local_rows()

            def allreduce(a):
                if not agg.collective:
                    return a
                t = torch.from_numpy(a.astype(np.int64))
                dist.all_reduce(t, group=agg.group)
                return t.numpy().astype(np.uint32)

            st = node_radix_select(x, self.pct, agg.all_gather_object, allreduce)
            return torch.from_numpy(st.astype(np.float32)) if self.is_root else None
        tr = agg.native
        comm = getattr(tr, "comm", None) if tr is not None else None
        if agg.collective and comm is None:
            raise RuntimeError("node-wide long-window statistics need the native RCCL communicator "
                               f"({agg.native_error or 'not enabled'})")
        out = self._out
        if out is None:
            out = self._out = torch.empty((len(self.agent.series), NUM_STATS), dtype=torch.float32,
                                          device=self.agent.device)
        stream = torch.cuda.current_stream(self.agent.device).cuda_stream
        try:
            # node bracket mode waits on the host for the brackets' outcome (it decides
            # whether the radix chain's collectives follow): bounded like every gather
            dws.refresh_node(out.data_ptr(), stream, *self.pct, comm if agg.collective else None,
                             bool(self.timing and agg.collective), timeout_s=self.collective_timeout_s,
                             abandon=agg.abandon if agg.collective else None)
        except RuntimeError:
            tr = agg.native
            if tr is not None and agg.collective:  # a peer is gone mid-refresh: abort the communicator
                tr.close()
                agg.native = None
            raise
        self._await(out)
        if self.timing and agg.collective:
            self.last_collective_us = {k: v for k, v in zip(self.COLLECTIVE_STEPS, dws.node_collective_us())
                                       if v == v}  # NaN: the step did not run this refresh
        return out if self.is_root else None

    def _local_rows(self) -> np.ndarray:
        """CPU: this rank's window of every series as [S, W] (NaN-padded)."""
        W = self.agent.window
        blocks = []
        for r in self.agent.rings:
            rows, _ = r.window(W)
            b = np.full((r.width, W), np.nan, np.float32)
            if len(rows):
                b[:, W - len(rows):] = rows.T
            blocks.append(b)
        return np.concatenate(blocks, axis=0)

    def _await(self, node) -> None:
        tr = self.aggregator.native
        if tr is None or not node.is_cuda or not hasattr(tr, "publisher"):
            return  # identity / host gathers are synchronous already
        from .node import await_publication

        if self._pub is None:
            self._pub = tr.publisher(False)
        seq = self._pub.publish(0, 0, 0, torch.cuda.current_stream(node.device).cuda_stream)
        try:
            await_publication(self._pub, seq, tr, self.collective_timeout_s, what="node-window gather",
                              abandon=self.aggregator.abandon)
        except RuntimeError:
            if not tr.healthy():
                self.aggregator.native = None
            raise
