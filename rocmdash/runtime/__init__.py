"""Native telemetry runtime: samplers, pinned rings, device windows, refresh pipeline."""

from . import native  # noqa: F401
