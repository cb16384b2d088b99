"""Data model of the dashboard: metric schema, statistic slots, GPU SKU tables."""

from .gpu_models import (  # noqa: F401
    GPU_NAME_RESOLVE,
    GPU_POWER_LIMITS,
    get_power_limit,
    normalize_power_limit_w,
    resolve_model,
)
from .schema import (  # noqa: F401
    COMPAT_METRICS,
    CTR_FIELDS,
    SMI_FIELDS,
    STAT_NAMES,
    STAT_INDEX,
    MetricSpec,
    METRIC_SPECS,
    series_names,
)
