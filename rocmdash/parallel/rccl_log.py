"""What RCCL itself says about the communicator: rank count and the transport per peer.

A node's record must prove that the gather ran over N ranks and over xGMI, not that some
communicator existed. Two sources, both RCCL's own:

* ``ncclCommCount`` / ``ncclCommUserRank`` / ``ncclCommCuDevice`` (csrc/rccl_comm.cpp,
  ``RcclComm.view()``): the rank count, this rank and the HIP device RCCL bound;
* RCCL's INIT log. Before the communicator is created, :func:`configure_debug_log`
  points ``NCCL_DEBUG=INFO`` / ``NCCL_DEBUG_SUBSYS=INIT,GRAPH`` at a per-rank
  ``NCCL_DEBUG_FILE``; when RCCL connects a channel to a peer it logs the transport it
  chose (``... 0[0] -> 1[1] via P2P/IPC`` for xGMI peer access, ``via SHM/...`` through
  host shared memory, ``[send] via NET/Socket/0`` over the network stack).
  :func:`parse_transport_log` turns those lines into per-peer transport kinds.

On a real node every peer of an N > 1 communicator must be P2P (xGMI); the oversubscribed
rehearsal on one GPU (rocmdash.parallel.node.oversubscribed) shows NET, by design.

Reference anchor: the reference pins one node by its IP (``/root/reference/app.py:164,
171``); this is the GPU-side proof of what "one node" meant for the collective.
"""

from __future__ import annotations

import os
import re
import tempfile

# "Channel 00/0 : 0[0] -> 1[1] via P2P/IPC", "Channel 01/0 : 1[0] -> 0[0] [send] via
# NET/Socket/0", "Channel 00 : 0[5000] -> 1[6000] via SHM/direct/direct" (the bracket
# holds the device or bus id, depending on the RCCL version)
_CHANNEL = re.compile(r"Channel\s+(\d+)(?:/\d+)?\s*:\s*(\d+)\[[^\]]*\]\s*->\s*(\d+)\[[^\]]*\]"
                      r"(?:\s*\[(send|receive)\])?\s*via\s+(\S+)")
_INIT_DONE = re.compile(r"rank\s+(\d+)\s+nranks\s+(\d+).*Init COMPLETE")
_WARN = re.compile(r"NCCL WARN (.*)")

KINDS = ("P2P", "SHM", "NET", "COLLNET")


def transport_kind(via: str) -> str:
    """``P2P/IPC/read`` -> ``P2P``; ``NET/Socket/0`` -> ``NET``; unknown prefixes kept."""
    head = via.split("/", 1)[0].upper()
    return head if head else "UNKNOWN"


def parse_transport_log(text: str, rank: int | None = None) -> dict:
    """RCCL INFO log text -> {"kinds": {kind: connections}, "peers": {peer: [kinds]},
    "via": [distinct transport strings], "init_complete", "nranks_logged", "warnings",
    "lines"}. Only connections made BY ``rank`` (``rank -> peer``) count when ``rank`` is
    given; a line that names neither end as this rank is ignored."""
    kinds: dict = {}
    peers: dict = {}
    via_seen: list = []
    lines = []
    init_complete = False
    nranks = None
    warnings = []
    for ln in text.splitlines():
        m = _CHANNEL.search(ln)
        if m:
            src, dst, via = int(m.group(2)), int(m.group(3)), m.group(5)
            if rank is not None and rank not in (src, dst):
                continue
            peer = dst if rank is None or src == rank else src
            k = transport_kind(via)
            kinds[k] = kinds.get(k, 0) + 1
            peers.setdefault(str(peer), set()).add(k)
            if via not in via_seen:
                via_seen.append(via)
            if len(lines) < 4:
                lines.append(ln.strip()[-160:])
            continue
        m = _INIT_DONE.search(ln)
        if m and (rank is None or int(m.group(1)) == rank):
            init_complete = True
            nranks = int(m.group(2))
            continue
        m = _WARN.search(ln)
        if m and len(warnings) < 4:
            warnings.append(m.group(1).strip()[-200:])
    return {"kinds": kinds, "peers": {p: sorted(v) for p, v in sorted(peers.items(), key=lambda kv: int(kv[0]))},
            "via": via_seen, "init_complete": init_complete, "nranks_logged": nranks, "warnings": warnings,
            "lines": lines}


def all_p2p(detail: dict | None) -> bool | None:
    """True when every logged peer connection is P2P, False when one is not, None when
    nothing was logged (RCCL's log was not ours to read: an earlier debug init, or
    ``ROCMDASH_RCCL_TRANSPORT_LOG=0``)."""
    if not detail or not detail.get("kinds"):
        return None
    return set(detail["kinds"]) == {"P2P"}


_CREATED: list = []  # log files this process created (removed at exit)


def _remove_created() -> None:
    for p in _CREATED:
        try:
            os.unlink(p)
        except OSError:
            pass


def _expand(pattern: str) -> str:
    """RCCL's NCCL_DEBUG_FILE patterns: %h = host name, %p = process id."""
    import socket

    return pattern.replace("%h", socket.gethostname()).replace("%p", str(os.getpid()))


def configure_debug_log(rank: int, directory: str | None = None) -> str | None:
    """Point RCCL's INFO log (INIT + GRAPH subsystems: communicator set-up and channel
    connections only, nothing per collective) at a per-rank file; returns its path, or
    None when there is none to read. Must run before the process's first RCCL call that
    logs (RCCL reads these once).

    A caller's own settings win: ``NCCL_DEBUG`` set to anything is kept (below
    INFO there are no channel lines to read: None); ``NCCL_DEBUG_FILE`` is kept and read -
    its ``%h`` / ``%p`` expanded as RCCL does; ``NCCL_DEBUG_SUBSYS`` is left alone when the
    caller chose the debug level. A file this function creates is removed at process exit,
    so restarts leave no logs behind. ``ROCMDASH_RCCL_TRANSPORT_LOG=0`` turns it off."""
    if os.environ.get("ROCMDASH_RCCL_TRANSPORT_LOG", "1").strip().lower() in ("0", "off", "false", "no"):
        return None
    level = os.environ.get("NCCL_DEBUG")
    if level is not None and level.strip().upper() not in ("INFO", "TRACE"):
        return None  # the caller's level logs no channel lines
    own = os.environ.get("NCCL_DEBUG_FILE")
    if own:
        path = _expand(own)
    else:
        d = directory or os.environ.get("ROCMDASH_RCCL_LOG_DIR") or tempfile.gettempdir()
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, f"rocmdash-rccl.{rank}.{os.getpid()}.log")
        os.environ["NCCL_DEBUG_FILE"] = path
        if not _CREATED:
            import atexit

            atexit.register(_remove_created)
        _CREATED.append(path)
    if level is None:
        os.environ["NCCL_DEBUG"] = "INFO"
        subsys = {s.strip().upper() for s in os.environ.get("NCCL_DEBUG_SUBSYS", "").split(",") if s.strip()}
        os.environ["NCCL_DEBUG_SUBSYS"] = ",".join(sorted(subsys | {"INIT", "GRAPH"}))
    return path


def read_transport_log(path: str | None, rank: int | None = None) -> dict | None:
    if not path:
        return None
    try:
        with open(path, errors="replace") as f:
            return parse_transport_log(f.read(), rank)
    except OSError:
        return None
