"""Rank side of the node supervisor's membership protocol (partial-node operation).

The reference shows whatever ``gpu_id``s its exporter reports and keeps drawing the
others (``/root/reference/app.py:183-201, 262-313``); a vanished GPU just drops out of
the next fetch (``app.py:335``). rocmdash's node service is a collective, so the same
property needs a protocol: the node supervisor (``rocmdash.runtime.supervisor``, the
DaemonSet's entrypoint) hosts a TCP store and decides *epochs* - numbered member lists
of GPU slots - and every rank process runs the node refresh only inside the epoch it
is a member of:

  * ``ready/<slot>/<incarnation>``: a rank whose GPU agent came up (sources, device
    window) announces it, with its GPU's identity;
  * ``epoch`` (an add-counter) and ``members/<E>``: the supervisor's decisions. The ranks
    of epoch E form a gloo control plane on the store prefix ``e<E>/`` (rank = position in
    the member list) and a fresh native RCCL communicator (new unique id) on top;
  * ``fail/<E>/<slot>``: a rank whose collective failed in epoch E says so, drops its
    communicator and process group, and waits for the next epoch. It keeps its agent: its
    sources, rings and device window (the W-sample history) survive the regroup.

A member that stops answering never reports; the members that do report tell the
supervisor who is gone (``rocmdash.runtime.supervisor.decide_culprits``). A rank that
sees a newer epoch while it waits on a native collective gives up at once
(``newer_epoch``), so a member whose process died costs its peers no collective timeout.
"""

from __future__ import annotations

import json
import os
import time
from datetime import timedelta

ENV_ADDR = "ROCMDASH_SUPERVISOR"  # host:port of the supervisor's store
ENV_SLOT = "ROCMDASH_SLOT"
ENV_SLOTS = "ROCMDASH_SLOTS"
ENV_INCARNATION = "ROCMDASH_INCARNATION"
ENV_PUSH = "ROCMDASH_PUSH"  # unix socket of the supervisor's snapshot listener
ENV_PUSH_KEY = "ROCMDASH_PUSH_KEY"


def parse_members(text: str) -> list:
    return [int(x) for x in text.split(",") if x.strip()]


def format_members(members) -> str:
    return ",".join(str(int(m)) for m in members)


class Membership:
    """One rank's view of the supervisor: its slot, its incarnation (how many times the
    supervisor started this slot before) and a store client."""

    def __init__(self, addr: str, slot: int, slots: int, incarnation: int = 0, timeout_s: float = 60.0):
        import torch.distributed as dist

        host, _, port = addr.rpartition(":")
        self.addr = addr
        self.slot = int(slot)
        self.slots = int(slots)
        self.incarnation = int(incarnation)
        self.timeout_s = float(timeout_s)
        self.store = dist.TCPStore(host or "127.0.0.1", int(port), is_master=False,
                                   timeout=timedelta(seconds=max(30.0, self.timeout_s)))
        self.epoch = 0  # the epoch this rank last joined (0: none)
        self.members: list = []

    @classmethod
    def from_environ(cls, timeout_s: float = 60.0) -> "Membership | None":
        addr = os.environ.get(ENV_ADDR, "").strip()
        if not addr:
            return None
        return cls(addr, int(os.environ[ENV_SLOT]), int(os.environ.get(ENV_SLOTS, "0") or 0),
                   int(os.environ.get(ENV_INCARNATION, "0") or 0), timeout_s)

    # ------------------------------------------------------------------ announcements
    def announce_ready(self, info: dict) -> None:
        """The agent is up: the supervisor may put this slot into the next epoch."""
        self.store.set(f"ready/{self.slot}/{self.incarnation}", json.dumps(info, default=str))

    def report_failure(self, epoch: int, reason: str) -> None:
        """A collective of ``epoch`` failed on this rank (it is alive and answering)."""
        self.store.set(f"fail/{epoch}/{self.slot}", reason[:500])

    def announce_stopped(self) -> None:
        """This rank leaves on purpose (a stop vote): its exit is not a failure."""
        self.store.set(f"stopped/{self.slot}/{self.incarnation}", "1")

    # ------------------------------------------------------------------ epochs
    def current_epoch(self) -> int:
        return int(self.store.add("epoch", 0))

    def newer_epoch(self) -> bool:
        """True once the supervisor decided an epoch after the one this rank joined."""
        return self.current_epoch() > self.epoch

    def members_of(self, epoch: int) -> list:
        return parse_members(self.store.get(f"members/{epoch}").decode())

    def wait_epoch(self, stop=None, poll_s: float = 0.05):
        """Block until an epoch newer than the last joined one lists this slot; returns
        (epoch, members), or None when ``stop`` (a threading.Event) is set first. Epochs
        that leave this slot out are skipped (a re-admitted slot waits for the one that
        takes it back)."""
        seen = self.epoch
        while stop is None or not stop.is_set():
            e = self.current_epoch()
            if e > seen:
                members = self.members_of(e)
                if self.slot in members:
                    self.epoch, self.members = e, members
                    return e, members
                seen = e
            time.sleep(poll_s)
        return None

    def rank_in_epoch(self) -> int:
        return self.members.index(self.slot)

    def pg_store(self, epoch: int | None = None):
        """The control plane's store of an epoch: the supervisor's store under a prefix
        of its own, so no key of an earlier epoch (peer addresses of ranks that are gone)
        is ever read."""
        import torch.distributed as dist

        return dist.PrefixStore(f"e{self.epoch if epoch is None else epoch}/", self.store)


class SnapshotPusher:
    """The epoch root's hand-off of each refresh's snapshot to the supervisor, which
    serves ``/metrics`` and ``/healthz`` (so the HTTP endpoint outlives any rank)."""

    def __init__(self, address: str | None = None, authkey: bytes | None = None):
        self.address = address or os.environ.get(ENV_PUSH)
        key = authkey if authkey is not None else bytes.fromhex(os.environ.get(ENV_PUSH_KEY, ""))
        self.authkey = key
        self._conn = None
        self.errors = 0

    def push(self, epoch: int, snapshot, extra) -> bool:
        from multiprocessing.connection import Client

        if not self.address:
            return False
        try:
            if self._conn is None:
                self._conn = Client(self.address, family="AF_UNIX", authkey=self.authkey)
            self._conn.send((int(epoch), snapshot, extra))
            return True
        except (OSError, EOFError, ValueError) as e:  # supervisor restarting: retried next refresh
            self.errors += 1
            self.close()
            if self.errors in (1, 10, 100):
                import logging

                logging.getLogger("rocmdash.membership").warning("snapshot push failed (%s)", e)
            return False

    def close(self) -> None:
        if self._conn is not None:
            try:
                self._conn.close()
            except OSError:
                pass
            self._conn = None
