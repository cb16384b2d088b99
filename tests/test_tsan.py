"""Race detection on the host side of the native runtime: the SPSC ring, the sampler
thread, its request()/wait() worker and concurrent readers, built with
-fsanitize=thread (host code only; GPU sanitizers are not available on this pool)."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def test_ring_and_sampler_are_tsan_clean(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "ring_stress"
    cmd = [
        gxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", f"-I{ROOT}/csrc", "-I/opt/rocm/include",
        f"{ROOT}/tools/tsan/ring_stress.cpp", f"{ROOT}/csrc/sampler.cpp", f"{ROOT}/csrc/sources.cpp",
        "-L/opt/rocm/lib", "-lamd_smi", "-lpthread", "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe),
    ]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    for spin_us in ("0", "50"):  # futex hand-off, spin hand-off
        run = subprocess.run([str(exe), "1.0", spin_us], capture_output=True, text=True, timeout=120, env=env)
        assert "ThreadSanitizer" not in run.stderr, run.stderr[-4000:]
        assert run.returncode == 0, (run.stdout, run.stderr[-2000:])
        assert "bad=0" in run.stdout


def test_tagged_word_handoff_is_tsan_clean(tmp_path):
    """csrc/tagged.h, the host side of the tagged outputs (stats kernel) and the tagged
    N > 1 publication: a writer thread publishes {value, seq} words in shuffled order,
    up to two publications ahead of the reader. wait_tagged() must return a publication
    only when EVERY word is of it (never a mix of two), report a partly overwritten one
    as superseded, and never return one that does not come. The deterministic case
    shows the round-2 rule (accept a newer tag) returned exactly such a mix."""
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "tagged_stress"
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", f"-I{ROOT}/csrc", f"{ROOT}/tools/tsan/tagged_stress.cpp",
           "-lpthread", "-o", str(exe)]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    run = subprocess.run([str(exe), "2000", "128"], capture_output=True, text=True, timeout=120, env=env)
    assert "ThreadSanitizer" not in run.stderr, run.stderr[-4000:]
    assert run.returncode == 0, (run.stdout, run.stderr[-2000:])
    assert "bad=0" in run.stdout and "mixed=0" in run.stdout
    assert "legacy_returns_mix=1 current=superseded" in run.stdout, run.stdout


def test_counter_lanes_are_tsan_clean(tmp_path):
    """csrc/node_counters.cpp's per-GPU lanes under ThreadSanitizer:
    three lanes at 5 kHz, one hanging; readers on every ring, stats() polled, the hung
    lane replaced twice (the second replacement hangs too), stop() leaving the blocked
    lane behind within its grace period."""
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "lanes_stress"
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", f"-I{ROOT}/csrc", "-I/opt/rocm/include",
           f"{ROOT}/tools/tsan/lanes_stress.cpp", f"{ROOT}/csrc/node_counters.cpp", f"{ROOT}/csrc/sources.cpp",
           "-L/opt/rocm/lib", "-lamd_smi", "-lpthread", "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    run = subprocess.run([str(exe), "1.0", str(tmp_path)], capture_output=True, text=True, timeout=120, env=env)
    assert "ThreadSanitizer" not in run.stderr, run.stderr[-4000:]
    assert run.returncode == 0, (run.stdout, run.stderr[-2000:])
    assert "bad=0" in run.stdout and "replaced=2" in run.stdout, run.stdout
