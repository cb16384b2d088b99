"""Prometheus layer: query client (reference-compatible), exposition, exporter, mini-Prometheus."""
