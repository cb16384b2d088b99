"""RCCL's own record of a communicator: the INIT-log parser that turns channel lines into
per-peer transports (rocmdash.parallel.rccl_log), on lines in the formats RCCL logs for
its three intra-node transports."""

import os

from rocmdash.parallel.rccl_log import all_p2p, configure_debug_log, parse_transport_log, transport_kind

P2P = """node:1234:1240 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC
node:1234:1240 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC/read
node:1234:1240 [0] NCCL INFO Channel 00/0 : 7[7] -> 0[0] via P2P/IPC
node:1234:1240 [0] NCCL INFO comm 0x55d1c0 rank 0 nranks 8 cudaDev 0 busId 5000 commId 0x9f - Init COMPLETE
"""
SHM = """node:1:2 [1] NCCL INFO Channel 00 : 1[6000] -> 2[7000] via SHM/direct/direct
node:1:2 [1] NCCL INFO Channel 00 : 0[5000] -> 1[6000] via SHM/direct/direct
node:1:2 [1] NCCL INFO Channel 00 : 2[7000] -> 3[8000] via SHM/direct/direct
"""
NET = """box:77:80 [0] NCCL INFO Channel 00/0 : 1[0] -> 0[0] [receive] via NET/Socket/0
box:77:80 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[0] [send] via NET/Socket/0
box:77:80 [0] NCCL WARN NET/Socket : no interface found, using lo
box:77:80 [0] NCCL INFO comm 0xabc rank 0 nranks 2 cudaDev 0 busId 5000 commId 0x1 - Init COMPLETE
"""


def test_p2p_lines():
    d = parse_transport_log(P2P, rank=0)
    assert d["kinds"] == {"P2P": 3} and d["peers"] == {"1": ["P2P"], "7": ["P2P"]}
    assert d["via"] == ["P2P/IPC", "P2P/IPC/read"]
    assert d["init_complete"] and d["nranks_logged"] == 8
    assert all_p2p(d) is True


def test_shm_lines_only_this_ranks_connections():
    d = parse_transport_log(SHM, rank=1)
    assert d["kinds"] == {"SHM": 2} and d["peers"] == {"0": ["SHM"], "2": ["SHM"]}
    assert all_p2p(d) is False


def test_net_lines_and_warnings():
    d = parse_transport_log(NET, rank=0)
    assert d["kinds"] == {"NET": 2} and d["peers"] == {"1": ["NET"]}
    assert d["warnings"] and "no interface" in d["warnings"][0]
    assert all_p2p(d) is False


def test_nothing_logged_is_unknown_not_a_failure():
    assert all_p2p(parse_transport_log("", rank=0)) is None
    assert all_p2p(None) is None
    assert transport_kind("NET/IB/0") == "NET" and transport_kind("COLLNET/x") == "COLLNET"


def test_configure_debug_log(tmp_path, monkeypatch):
    for k in ("NCCL_DEBUG", "NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS", "ROCMDASH_RCCL_TRANSPORT_LOG"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("NCCL_DEBUG_SUBSYS", "NET")
    path = configure_debug_log(3, str(tmp_path))
    assert path.startswith(str(tmp_path)) and ".3." in os.path.basename(path)
    assert os.environ["NCCL_DEBUG"] == "INFO" and os.environ["NCCL_DEBUG_FILE"] == path
    assert set(os.environ["NCCL_DEBUG_SUBSYS"].split(",")) == {"GRAPH", "INIT", "NET"}
    monkeypatch.setenv("ROCMDASH_RCCL_TRANSPORT_LOG", "0")
    assert configure_debug_log(3, str(tmp_path)) is None
    # a caller's own settings win: a quieter level means no log to read, and
    # the levels / subsystems it chose are left alone
    monkeypatch.delenv("ROCMDASH_RCCL_TRANSPORT_LOG")
    for k in ("NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("NCCL_DEBUG", "WARN")
    assert configure_debug_log(3, str(tmp_path)) is None and os.environ["NCCL_DEBUG"] == "WARN"
    assert "NCCL_DEBUG_FILE" not in os.environ and "NCCL_DEBUG_SUBSYS" not in os.environ
    # the caller's file pattern is kept and read where RCCL writes it (%h / %p expanded)
    monkeypatch.setenv("NCCL_DEBUG", "INFO")
    monkeypatch.setenv("NCCL_DEBUG_SUBSYS", "COLL")
    monkeypatch.setenv("NCCL_DEBUG_FILE", str(tmp_path / "rccl.%p.log"))
    got = configure_debug_log(1, str(tmp_path))
    assert got == str(tmp_path / f"rccl.{os.getpid()}.log") and os.environ["NCCL_DEBUG_SUBSYS"] == "COLL"


def test_created_debug_log_is_removed_at_exit(tmp_path):
    """A log file rocmdash created for its own reading does not outlive the process."""
    import subprocess
    import sys

    code = ("import os; from rocmdash.parallel.rccl_log import configure_debug_log as c; "
            f"p = c(0, {str(tmp_path)!r}); open(p, 'w').write('x'); print(p)")
    env = {k: v for k, v in os.environ.items() if not k.startswith("NCCL_")}
    res = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    path = res.stdout.strip().splitlines()[-1]
    assert res.returncode == 0 and path.startswith(str(tmp_path)) and not os.path.exists(path), res.stderr


def test_rccl_2_26_line_formats():
    """The exact formats in the RCCL 2.26 this image ships (librccl.so strings): the
    channel lines end with `comm 0x... nRanks NN`, and P2P may go through an
    intermediate GPU (`P2P/indirect/...`) - still P2P (xGMI)."""
    text = """h:1:2 [0] NCCL INFO Channel 00/0 : 0[5000] -> 1[6000] via P2P/IPC comm 0x55aa nRanks 08
h:1:2 [0] NCCL INFO Channel 01/0 : 0[5000] -> 2[7000] via P2P/indirect/1[6000] comm 0x55aa nRanks 08
h:1:2 [0] NCCL INFO Channel 02/0 : 7[c000] -> 0[5000] via P2P/CUMEM/read comm 0x55aa nRanks 08
h:1:2 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[0] [send] via NET/Socket/0(0)/GDRDMA comm 0x55ab nRanks 02
h:1:2 [0] NCCL INFO ncclCommInitRankConfig comm 0x55aa rank 0 nranks 8 cudaDev 0 nvmlDev 0 busId 5000 commId 0x1f - Init COMPLETE
"""
    d = parse_transport_log(text, rank=0)
    assert d["kinds"] == {"P2P": 3, "NET": 1} and d["init_complete"] and d["nranks_logged"] == 8
    assert d["peers"] == {"1": ["NET", "P2P"], "2": ["P2P"], "7": ["P2P"]}
    assert "P2P/indirect/1[6000]" in d["via"] and all_p2p(d) is False
    p2p_only = "\n".join(text.splitlines()[:3])
    assert all_p2p(parse_transport_log(p2p_only, rank=0)) is True
