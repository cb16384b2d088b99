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

    def refresh(self):
        """Collective: every rank calls it after its ``agent.refresh()``. Returns the
        ``[S, 8]`` node statistics on rank 0 (a device tensor on GPUs, complete: the
        gather was waited for), ``None`` elsewhere.

        On the native transport the gather (+ rank 0's selection) is followed by a
        completion signal that every rank waits for with a deadline
        (``await_publication``): a peer that died or hung between the stats gather and
        this one makes the refresh raise (communicator aborted) instead of blocking rank
        0's copy of the statistics forever."""
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

    def _await(self, node) -> None:
        tr = self.aggregator.native
        if tr is None or not node.is_cuda or not hasattr(tr, "publisher"):
            return  # identity / host gathers are synchronous already
        from .node import await_publication

        if self._pub is None:
            self._pub = tr.publisher(False)
        seq = self._pub.publish(0, 0, 0, torch.cuda.current_stream(node.device).cuda_stream)
        try:
            await_publication(self._pub, seq, tr, self.collective_timeout_s, what="node-window gather")
        except RuntimeError:
            if not tr.healthy():
                self.aggregator.native = None
            raise
