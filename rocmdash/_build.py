"""Build the native runtime extension ``rocmdash._native`` in-tree with hipcc (gfx950).

Sources live in ``csrc/``: the SPSC ring, amd-smi / rocprofiler-sdk / synthetic
sources, the sampler thread, the device-ring mirror and the CDNA4 window-stats
kernel, plus pybind11 bindings. The .so is written next to this file so it travels
with ``gpurun`` snapshots (``*.so`` is git-ignored, not gpurun-ignored).

    python -m rocmdash._build          # incremental
    python -m rocmdash._build --force  # rebuild everything
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
PKG = ROOT / "rocmdash"
ARCH = os.environ.get("ROCMDASH_OFFLOAD_ARCH", "gfx950")

SOURCES = [
    "window_stats.hip",
    "long_window.hip",
    "node_window.hip",
    "calib.hip",
    "publish.hip",
    "device_window.cpp",
    "rccl_comm.cpp",
    "sources.cpp",
    "counters.cpp",
    "node_counters.cpp",
    "sampler.cpp",
    "frame_render.cpp",
    "bindings.cpp",
]


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the native runtime needs ROCm's hipcc")


def output_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return PKG / f"_native{suffix}"


def _flags() -> list[str]:
    import pybind11

    return [
        "-O3",
        "-std=c++17",
        "-fPIC",
        f"--offload-arch={ARCH}",
        "-Wall",
        "-Wno-unused-result",
        "-Wno-unused-function",
        f"-I{CSRC}",
        "-I/opt/rocm/include",
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
        "-fvisibility=hidden",
    ]


def _compile(src: Path, obj: Path, flags: list[str]) -> None:
    obj.parent.mkdir(parents=True, exist_ok=True)
    cmd = [_hipcc(), *flags, "-c", str(src), "-o", str(obj)]
    if src.suffix == ".cpp":
        cmd[1:1] = ["-x", "hip"]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")


def source_hash() -> str:
    """Digest of every native source and header (and this build script): what the
    built extension must have been compiled from."""
    import hashlib

    h = hashlib.sha256()
    for f in sorted([CSRC / s for s in SOURCES] + list(CSRC.glob("*.h")) + [Path(__file__)]):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def stamp_path() -> Path:
    return PKG / "_native.srchash"


def built_from_current_sources() -> bool | None:
    """True / False if the in-tree extension was / was not built from the sources in
    csrc/ now; None when there is no stamp (an extension built before stamps)."""
    try:
        return stamp_path().read_text().strip() == source_hash()
    except OSError:
        return None


def _stale(out: Path, deps: list[Path]) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> Path:
    out = output_path()
    headers = sorted(CSRC.glob("*.h"))
    srcs = [CSRC / s for s in SOURCES]
    flags = _flags()
    objs = []
    todo = []
    for s in srcs:
        obj = BUILD / (s.name + ".o")
        objs.append(obj)
        if force or _stale(obj, [s, *headers, Path(__file__)]):
            todo.append((s, obj))
    jobs = jobs or min(len(todo) or 1, max(1, min(8, os.cpu_count() or 1)))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda so: _compile(so[0], so[1], flags), todo))
            if verbose:
                for s, _ in todo:
                    print(f"[rocmdash._build] compiled {s.name}", file=sys.stderr)
    if force or todo or _stale(out, objs):
        cmd = [
            _hipcc(),
            "-shared",
            "-fPIC",
            f"--offload-arch={ARCH}",
            *map(str, objs),
            "-o",
            str(out),
            "-L/opt/rocm/lib",
            "-lamd_smi",
            "-ldl",
            "-lpthread",
            "-Wl,-rpath,/opt/rocm/lib",
        ]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
        if verbose:
            print(f"[rocmdash._build] linked {out}", file=sys.stderr)
    stamp_path().write_text(source_hash() + "\n")
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--check", action="store_true", help="exit 1 if the extension is not built from csrc/ as it is now")
    args = ap.parse_args(argv)
    if args.check:
        ok = built_from_current_sources()
        print(f"native extension built from current sources: {ok}")
        return 0 if ok else 1
    print(build(force=args.force, verbose=args.verbose))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
