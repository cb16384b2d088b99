"""Loader for the compiled runtime ``rocmdash._native`` (csrc/, built by rocmdash._build).

GPU code paths never fall back silently: if the extension is missing on a machine
with a GPU, :func:`load` raises (or builds it in-tree first when ``build=True``).

Hardware-counter sampling (rocprofiler-sdk device counting) must be configured
before the HIP/HSA runtime initialises in this process, so :func:`enable_counters`
has to run before the first ``torch.cuda`` call that touches a device; it is
idempotent and returns whether counters are usable.
"""

from __future__ import annotations

import importlib
import os

from ..models.schema import check_native_layout

DEFAULT_COUNTERS = (
    "GRBM_COUNT",
    "GRBM_GUI_ACTIVE",
    "SQ_VALU_MFMA_BUSY_CYCLES",
    # memory-side read and write bytes in 32 B units, any request size, one counter each
    # (csrc/counters.cpp). The write pair WRREQ + WRREQ_64B (rocprofiler's WRITE_SIZE) costs
    # +24..27 us on every read for the same bytes (profiles/r06/counter_ab/): on gfx950 the
    # request-count counters below are skipped and only stand in where an agent lacks the
    # 32 B-unit ones
    "TCC_EA0_RDREQ_DRAM_32B_sum",
    "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum",
    "TCC_EA0_RDREQ_sum",
    "TCC_EA0_WRREQ_sum",
    "TCC_EA0_WRREQ_64B_sum",
    "SQ_BUSY_CU_CYCLES",  # CU active; +3..8 us per read (profiles/r02/counter_sets.jsonl)
)

_mod = None
_counters_state = None  # None = not attempted, else (ok: bool, status: str)


def available() -> bool:
    try:
        load(build=False)
        return True
    except Exception:
        return False


def load(build: bool = False, with_torch: bool = True):
    """Import the native extension (optionally building it in-tree first).

    ``with_torch=False``: a process that never touches torch (the node counter process,
    rocmdash.runtime.counterd) loads the extension alone - its HIP runtime is then
    /opt/rocm's (the extension's RUNPATH) and the process saves torch's ~250 MiB of
    anonymous memory. Importing torch later in such a process is refused by the
    two-runtime check below on the next load()."""
    global _mod
    if _mod is not None:
        return _mod
    # PyTorch-ROCm bundles its own HIP runtime (torch/lib/libamdhip64.so, soname
    # libamdhip64.so.7). Loading torch first makes the extension's NEEDED
    # libamdhip64.so.7 bind to THAT copy instead of /opt/rocm's, so the extension
    # and torch share one HIP runtime (one device table, one stream namespace).
    # Loading the extension first would put two HIP runtimes in the process and
    # every launch on a torch stream would fail (hipErrorNoDevice).
    if with_torch:
        import torch  # noqa: F401

    try:
        mod = importlib.import_module("rocmdash._native")
    except ImportError as exc:
        if not build:
            raise RuntimeError(
                "rocmdash._native is not built: run `python -m rocmdash._build` "
                "(or __graft_entry__.build()) to compile csrc/ for gfx950"
            ) from exc
        from .. import _build

        _build.build()
        importlib.invalidate_caches()
        mod = importlib.import_module("rocmdash._native")
    try:  # a stale in-tree build runs yesterday's kernels silently: say so
        from .._build import built_from_current_sources

        if built_from_current_sources() is False:
            import warnings

            warnings.warn("rocmdash._native was built from different csrc/ sources: run `python -m rocmdash._build`",
                          RuntimeWarning, stacklevel=2)
    except Exception:  # noqa: BLE001 - sources not shipped (installed package)
        pass
    check_native_layout(mod)
    libs = hip_runtimes_loaded()
    if len(libs) > 1:
        raise RuntimeError(f"two HIP runtimes are loaded in this process: {sorted(libs)}")
    _mod = mod
    return mod


def hip_runtimes_loaded() -> set:
    """Distinct libamdhip64 files mapped into this process (Linux)."""
    found = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    found.add(os.path.realpath(line.split()[-1]))
    except OSError:
        pass
    return found


def enable_counters(names=DEFAULT_COUNTERS, only_device: int | None = None) -> tuple:
    """Register the rocprofiler-sdk device-counting tool (before HIP init).

    ``only_device``: configure just that GPU (a rank-per-GPU process); default: the
    LOCAL_RANK of a multi-process job (WORLD_SIZE > 1), else every GPU.
    Returns ``(ok, status)``. ``ROCMDASH_COUNTERS=0`` disables counters (e.g. when
    the process runs under ``rocprofv3 --pmc``, which owns the counter hardware).
    """
    global _counters_state
    if _counters_state is not None:
        return _counters_state
    if os.environ.get("ROCMDASH_COUNTERS", "1") in ("0", "false", "off"):
        _counters_state = (False, "disabled by ROCMDASH_COUNTERS")
        return _counters_state
    mod = load()
    if only_device is None and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from ..parallel.node import device_index_for

        only_device = device_index_for(int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0"))))
    only_bdf = 0
    if only_device is not None:
        # the GPU's PCI address in HIP order (no HIP init): robust to agent orderings
        from .topology import bdf_of_hip_device

        only_bdf = bdf_of_hip_device(int(only_device)) or 0
    # start the runtime on the NUMA node where this GPU's counter reads are fast
    # (placement.py: a per-process 2x, measured per GPU, cached per boot)
    from .placement import pin_for_init
    from .topology import bdf_of_hip_device as _bdf

    try:
        pin_for_init(int(only_device or 0), int(only_bdf or _bdf(int(only_device or 0)) or 0))
    except OSError:
        pass
    rc = mod.counters_preinit(list(names), -1 if only_device is None else int(only_device), int(only_bdf))
    _counters_state = (rc == 0, mod.counters_status())
    return _counters_state


def counters_requested() -> bool:
    """True when enable_counters() ran and was not disabled by the environment."""
    return _counters_state is not None and _counters_state[1] != "disabled by ROCMDASH_COUNTERS"


def counters_ready() -> bool:
    if _counters_state is None or not _counters_state[0]:
        return False
    return bool(load().counters_ready())


def counters_status() -> str:
    if _counters_state is None:
        return "not requested"
    return load().counters_status() if _counters_state[0] else _counters_state[1]
