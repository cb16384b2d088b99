"""GPU SKU tables: board part number -> marketing name -> power-axis maximum.

Reference: ``app.py:26-38`` (``GPU_NAME_RESOLVE``, ``GPU_POWER_LIMITS``) and the
dead helper ``get_power_limit`` at ``app.py:229-232``. The reference has no
MI350-series rows, so an MI355X shows ``(None)`` and a 300 W power axis there.
The MI355 OAM board part number below was read from amd-smi on the MI355X test
box (``amdsmi_get_gpu_board_info().model_number``, see
``profiles/probe_amdsmi.txt``); the power limit comes from
``amdsmi_power_info_t.power_limit`` on the same box (1400 W).
"""

from __future__ import annotations

# Reference rows kept verbatim (app.py:26-30), MI3xx/MI35x rows added.
GPU_NAME_RESOLVE = {
    "102-D65209-00": "MI250",
    "102-G30211-0C": "MI300",
    "102-G30219-00": "MI308X",
    "102-G36236-0C": "MI355X",  # "AMD Instinct MI355 OAM" (amd-smi on a test box)
    "102-G36237-0C": "MI355X",  # "AMD Instinct MI355 OAM" (amd-smi on another test box)
    "102-G36216-0C": "MI355X",  # "AMD Instinct MI355 OAM" (tests/fixtures/mi355x_capture.npz)
}

# Reference rows kept verbatim (app.py:33-38).
GPU_POWER_LIMITS = {
    "MI250": 560,
    "MI300": 750,
    "MI308X": 650,
    "MI325X": 1000,
    "MI350X": 1000,
    "MI355X": 1400,
    "default": 300,
}

# product_name substrings -> model, used when the part number is unknown
# (amd-smi product names look like "AMD Instinct MI355 OAM").
_PRODUCT_HINTS = (
    ("MI355", "MI355X"),
    ("MI350", "MI350X"),
    ("MI325", "MI325X"),
    ("MI308", "MI308X"),
    ("MI300", "MI300"),
    ("MI250", "MI250"),
)


def resolve_model(card_model, product_name: str | None = None):
    """Part number -> marketing name. Unknown part numbers fall back to a
    product-name hint, else ``None`` (reference behaviour: ``GPU_NAME_RESOLVE.get``)."""
    name = GPU_NAME_RESOLVE.get(card_model)
    if name is not None:
        return name
    for text in (product_name, card_model):
        if isinstance(text, str):
            for hint, model in _PRODUCT_HINTS:
                if hint in text:
                    return model
    return None


def get_power_limit(card_model):
    """Power-axis max for a part number (reference ``app.py:229-232``, same lookup
    chain: part number -> name -> limit, default 300 W)."""
    resolved_model = GPU_NAME_RESOLVE.get(card_model, card_model)
    return GPU_POWER_LIMITS.get(resolved_model, GPU_POWER_LIMITS["default"])


def normalize_power_limit_w(raw) -> float | None:
    """amd-smi reports ``power_limit`` in W on some ASICs and uW on others
    (1_400_000_000 on the MI355X box). Returns watts or None if unsupported."""
    if raw is None:
        return None
    raw = float(raw)
    if raw <= 0 or raw >= 0xFFFFFFFF:
        return None
    if raw > 100_000:  # no accelerator draws 100 kW: this is micro-watts
        return raw / 1e6
    return raw
