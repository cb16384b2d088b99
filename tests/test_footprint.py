"""The exporter's own footprint travels in each rank's control row (float32 slots of the
gathered block, rocmdash.models.schema.CONTROL_FIELDS) and comes out as Prometheus
counters on rank 0 (rocmdash/serve.py). Counters must stay exact and monotone for the
life of a DaemonSet pod: CPU seconds - all threads and the SCHED_IDLE part - are carried
as exact millisecond halves, not float32 seconds (0.25 s resolution after a month)."""

import numpy as np

from rocmdash.models.schema import CONTROL_FIELDS
from rocmdash.runtime.footprint import Footprint, decode_control


def _row(fp, sample):
    fp.sample = lambda: sample
    ctl = np.full(len(CONTROL_FIELDS), np.nan, np.float32)
    fp.fill(ctl)
    return ctl


def test_cpu_counters_exact_after_months():
    fp = Footprint()
    day = 86400.0
    prev_normal = -1.0
    for t in range(5):
        total = 180 * day * 1.02 + t * 1.017  # 180 days at ~1 CPU-s/s, then 1 s refreshes
        idle = 180 * day + t * 1.0
        ctl = _row(fp, {"hbm_bytes": 667 << 20, "rss_bytes": 1 << 30, "cpu_seconds": total, "cpu_idle_seconds": idle})
        d = decode_control(ctl)
        assert abs(d["cpu_seconds"] - total) < 1e-3 and abs(d["cpu_idle_seconds"] - idle) < 1e-3
        normal = d["cpu_seconds"] - d["cpu_idle_seconds"]
        assert normal > prev_normal  # the normal-class counter never steps back
        prev_normal = normal
    assert d["hbm_bytes"] == 667 << 20 and d["rss_bytes"] == 1 << 30
    # what float32 seconds would have carried after a month: a refresh's 17 ms of normal
    # CPU time rounds away (0.25 s steps)
    month = 30 * 86400.0
    assert float(np.float32(month + 0.017)) == float(np.float32(month))


def test_gather_state_encoding():
    ctl = np.full(len(CONTROL_FIELDS), np.nan, np.float32)
    ctl[CONTROL_FIELDS.index("gather_validated")] = -1.0  # host fallback
    d = decode_control(ctl)
    assert d["native_gather"] == 0.0 and d["gather_validated"] == 0.0
    ctl[CONTROL_FIELDS.index("gather_validated")] = 8.0  # native, 8 gathers validated
    d = decode_control(ctl)
    assert d["native_gather"] == 1.0 and d["gather_validated"] == 8.0
    assert decode_control(np.full(len(CONTROL_FIELDS), np.nan, np.float32))["native_gather"] is None


def test_kfd_vram_zero_counts_as_unavailable(tmp_path):
    from rocmdash.runtime.footprint import kfd_vram_bytes

    d = tmp_path / "4242"
    d.mkdir()
    assert kfd_vram_bytes(4242, root=str(tmp_path)) is None  # no files
    (d / "vram_1234").write_text("0\n")
    assert kfd_vram_bytes(4242, root=str(tmp_path)) is None  # listed, never filled
    (d / "vram_5678").write_text(str(667 << 20) + "\n")
    assert kfd_vram_bytes(4242, root=str(tmp_path)) == 667 << 20


def test_startup_delta_survives_other_processes_on_the_device():
    """The device-wide sysfs counter also moves with other processes on the GPU: trusted
    only when it rose at every stage and agrees with HIP's view, else HIP's growth."""
    from rocmdash.runtime.footprint import startup_delta

    MiB = 1 << 20
    # quiet device: sysfs rose 487 (HIP context) + 180 MiB; HIP saw the 180
    quiet = [("start", 1000 * MiB, None), ("hip", 1487 * MiB, 300 * MiB), ("agent", 1667 * MiB, 480 * MiB)]
    assert startup_delta(quiet) == 667 * MiB
    # ... HIP saw only 10 of the 180 (rocprofiler's context allocates past HIP): still sysfs
    quiet2 = [("start", 1000 * MiB, None), ("hip", 1487 * MiB, 300 * MiB), ("agent", 1667 * MiB, 310 * MiB)]
    assert startup_delta(quiet2) == 667 * MiB
    # another process freed 23 GB while rocmdash started (pool box): HIP growth + context step
    busy = [("start", 280_000 * MiB, None), ("hip", 280_487 * MiB, 300 * MiB), ("agent", 257_000 * MiB, 480 * MiB)]
    assert startup_delta(busy) == 487 * MiB + 180 * MiB
    # another process allocated 4 GB after the HIP start: sysfs rose but disagrees with HIP
    grew = [("start", 1000 * MiB, None), ("hip", 1487 * MiB, 300 * MiB), ("agent", 5667 * MiB, 480 * MiB)]
    assert startup_delta(grew) == 667 * MiB
    # the context step itself polluted: HIP growth alone
    both = [("start", 9000 * MiB, None), ("hip", 1487 * MiB, 300 * MiB), ("agent", 5667 * MiB, 480 * MiB)]
    assert startup_delta(both) == 180 * MiB
    # no sysfs (bdf unknown): HIP growth
    assert startup_delta([("hip", None, 300 * MiB), ("agent", None, 480 * MiB)]) == 180 * MiB
    assert startup_delta([("start", None, None)]) is None


def test_refresh_path_does_no_proc_walk(monkeypatch):
    """The service's side rows copy the footprint from a background sample (VERDICT r03
    item 3): after the first refresh starts the ``rd-footprint`` thread, refreshes walk
    no ``/proc/self/task`` and read no KFD file on the refresh path."""
    import threading

    from rocmdash.config import SamplerConfig
    from rocmdash.parallel.node import NodeAggregator
    from rocmdash.runtime import threads
    from rocmdash.runtime.agent import GpuAgent
    from rocmdash.runtime.pipeline import NodePipeline

    agent = GpuAgent(0, source="synthetic", counters="synthetic", cfg=SamplerConfig(window=64, ring_capacity=256),
                     use_gpu=False)
    agent.prefill(8)
    pipe = NodePipeline(agent, NodeAggregator(), health=True, device_timing=True)
    on_refresh_thread = []
    real = threads.thread_cpu

    def counted(*a, **k):
        on_refresh_thread.append(threading.current_thread() is threading.main_thread())
        return real(*a, **k)

    monkeypatch.setattr(threads, "thread_cpu", counted)
    pipe.step()  # starts the background sampler (one sample taken on start)
    first = pipe.footprint.samples_taken
    assert pipe.footprint._thread is not None and pipe.footprint._thread.name == "rd-footprint"
    on_refresh_thread.clear()
    for _ in range(20):
        agent.sample()
        pipe.step()
    assert not any(on_refresh_thread), "a refresh walked /proc on the refresh thread"
    assert pipe.footprint.samples_taken - first <= 2  # only the <= 1 Hz thread samples
    assert set(pipe.stage_seconds()) == {"stats_kernel", "allgather"}
    ctl = pipe.last_control
    assert ctl is not None and decode_control(ctl[0])["cpu_seconds"] is not None
    pipe.close()
    assert pipe.footprint._thread is None
    agent.close()


def _fdinfo(client, pdev, vram_kib):
    return (f"pos:\t0\nflags:\t02100002\ndrm-driver:\tamdgpu\ndrm-client-id:\t{client}\ndrm-pdev:\t{pdev}\n"
            f"drm-total-vram:\t{vram_kib} KiB\ndrm-memory-vram:\t{vram_kib} KiB\ndrm-memory-gtt:\t2100 KiB\n")


def test_drm_fdinfo_per_process_vram(tmp_path):
    """Per-process device memory from DRM fdinfo: summed per GPU
    (pdev -> amd-smi bdf), one count per DRM client (a client's fd dup'ed twice counts
    once), non-DRM fds ignored; a process without the GPU open has none."""
    from rocmdash.runtime.footprint import drm_vram_by_bdf, pdev_bdf

    d = tmp_path / "123" / "fdinfo"
    d.mkdir(parents=True)
    (d / "3").write_text("pos:\t0\nflags:\t0100002\nmnt_id:\t22\n")
    (d / "7").write_text(_fdinfo(51, "0000:75:00.0", 48316))
    (d / "8").write_text(_fdinfo(51, "0000:75:00.0", 48316))  # the same client again
    (d / "9").write_text(_fdinfo(52, "0001:05:00.0", 1108))
    got = drm_vram_by_bdf(123, root=str(tmp_path))
    assert pdev_bdf("0000:75:00.0") == 0x7500 and pdev_bdf("0001:05:00.0") == (1 << 32) | 0x500
    assert got == {0x7500: 48316 * 1024, (1 << 32) | 0x500: 1108 * 1024}
    assert drm_vram_by_bdf(999, root=str(tmp_path)) == {}


def test_node_device_memory_report_is_never_negative():
    from rocmdash.runtime.nodemeasure import device_memory_report

    M = 1 << 20
    dev = {"7500": {"rank": 48 * M, "counterd": 1 * M}}
    procs = {"7500": {("rank", "0"), ("counterd", "")}}
    r = device_memory_report({"7500": 1000 * M}, {"7500": 1742 * M}, dev, procs)["7500"]
    assert r["process_buffers_mib"] == {"counterd": 1.0, "rank": 48.0} and r["attributed_mib"] == 49.0
    assert r["device_used_growth_mib"] == 742.0 and r["driver_state_mib"] == 693.0
    assert r["driver_state_mib_per_process"] == 346.5
    # another process freed memory meanwhile: no device-wide figure, no negative one
    r = device_memory_report({"7500": 1000 * M}, {"7500": 800 * M}, dev, procs)["7500"]
    assert "device_used_growth_mib" not in r and "note" in r
    assert all(v is None or not isinstance(v, (int, float)) or v >= 0 for v in r.values())
