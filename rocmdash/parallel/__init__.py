"""Rank-per-GPU node aggregation (RCCL all-gather on GPUs, gloo on CPU)."""

from .node import DistEnv, NodeAggregator, dist_env_from_environ  # noqa: F401
