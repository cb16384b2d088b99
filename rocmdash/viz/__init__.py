"""Visualisation: colour bands, gauge/bar figure factories, dashboard frame builder."""

from .figures import (  # noqa: F401
    GAUGE_COLORS,
    Figure,
    create_chart,
    create_gauge,
    create_horizontal_bar,
    get_color_for_value,
    template_json,
)
from .panels import Frame, NodeSnapshot, build_frame, selected_averages  # noqa: F401
