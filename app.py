"""Streamlit entry point: ``streamlit run app.py`` (same as the reference's).

API-compatible with the reference ``app.py``: the page config runs at import time
(``app.py:14-19``) and the module-level names the reference defines stay importable
(``PROMETHEUS_METRICS_ENDPOINT``, ``PROMETHEUS_METRICS_PODNAME``, ``REFRESH_INTERVAL``,
``GPU_NAME_RESOLVE``, ``GPU_POWER_LIMITS``, ``GAUGE_COLORS``, ``get_color_for_value``,
``create_gauge``, ``create_horizontal_bar``, ``fetch_gpu_metrics``,
``get_power_limit``, ``create_visualization``, ``main``). The implementation lives in
the ``rocmdash`` package.
"""

import streamlit as st

from rocmdash.ui.page import PAGE_CONFIG

st.set_page_config(**PAGE_CONFIG)

from rocmdash.config import (  # noqa: E402,F401
    PROMETHEUS_METRICS_ENDPOINT,
    PROMETHEUS_METRICS_PODNAME,
    REFRESH_INTERVAL,
)
from rocmdash.models.gpu_models import GPU_NAME_RESOLVE, GPU_POWER_LIMITS  # noqa: E402,F401
from rocmdash.ui.page import (  # noqa: E402,F401
    create_visualization,
    fetch_gpu_metrics,
    get_power_limit,
    main,
)
from rocmdash.viz.figures import (  # noqa: E402,F401
    GAUGE_COLORS,
    create_gauge,
    create_horizontal_bar,
    get_color_for_value,
)

if __name__ == "__main__":
    main()
