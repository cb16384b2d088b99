"""rocmdash — an MI355X-native GPU metrics dashboard framework.

Capability parity target: ontheklaud/k8s-rocm-metrics-dashboard (a single-file
Streamlit app, reference ``app.py``). The reference only *reads* Prometheus; this
framework owns the whole chain for an 8x MI355X node:

    amd-smi / rocprofiler-sdk samplers (C++)      rocmdash.runtime  (csrc/sources.cpp, csrc/counters.cpp,
                                                                     csrc/sampler.cpp)
      -> pinned host SPSC ring (mapped)             csrc/ring.h
      -> HIP/CDNA4 windowed min/mean/max/pXX kernel rocmdash.ops.window_stats, csrc/window_stats.hip
         (pulls the entering rows straight from the
         mapped ring; resident sorted windows)
      -> native RCCL ncclAllGather over xGMI        rocmdash.parallel.node, csrc/rccl_comm.cpp,
         (rank per GPU, one communicator each)     csrc/publish.hip
      -> Prometheus exposition / query API          rocmdash.prom
      -> Plotly panel specs + Streamlit app.py      rocmdash.viz, rocmdash.ui

Subpackages:
    models    metric schema + GPU SKU tables (the "data model" of the dashboard)
    ops       device kernels (window statistics) and their CPU references
    parallel  rank-per-GPU node aggregation (RCCL all-gather; gloo on CPU)
    runtime   native samplers, rings and the refresh pipeline
    prom      Prometheus query layer, exposition, exporter and mock server
    viz       colour bands, gauge/bar factories and the fast panel-spec builder
    ui        the Streamlit page (reference app.py:247-486)
    utils     timing, logging, natural sort
"""

__version__ = "0.1.0"
