"""Recording test double of the Streamlit API surface the dashboard uses.

Streamlit is not installable in this environment (no network).
Every call is appended to ``CALLS`` as ``(name, args, kwargs)``; widgets return their
``value`` argument (or a value forced through ``WIDGET_VALUES[key-or-label]``).
"""

from contextlib import contextmanager

CALLS = []
WIDGET_VALUES = {}


class _SessionState(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


session_state = _SessionState()


def reset():
    CALLS.clear()
    WIDGET_VALUES.clear()
    session_state.clear()


def _rec(name):
    def f(*args, **kwargs):
        CALLS.append((name, args, kwargs))
    return f


for _n in ("set_page_config", "title", "markdown", "header", "subheader", "text", "error", "warning",
           "info", "dataframe", "plotly_chart", "write", "caption", "json"):
    globals()[_n] = _rec(_n)


def toggle(label, value=False, key=None, **kw):
    CALLS.append(("toggle", (label,), dict(value=value, key=key, **kw)))
    return WIDGET_VALUES.get(key or label, value)


def checkbox(label, value=False, key=None, **kw):
    CALLS.append(("checkbox", (label,), dict(value=value, key=key, **kw)))
    return WIDGET_VALUES.get(key or label, value)


class _Ctx:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        CALLS.append(("enter", (self.name,), {}))
        return self

    def __exit__(self, *a):
        return False

    def container(self):
        return _Ctx(self.name + ".container")


def columns(n, **kw):
    CALLS.append(("columns", (n,), kw))
    k = n if isinstance(n, int) else len(n)
    return [_Ctx(f"col{i}") for i in range(k)]


def empty():
    CALLS.append(("empty", (), {}))
    return _Ctx("empty")


@contextmanager
def spinner(*a, **k):
    yield


class _Sidebar:
    def write(self, *args, **kwargs):
        CALLS.append(("sidebar.write", args, kwargs))


sidebar = _Sidebar()


def calls(name):
    return [c for c in CALLS if c[0] == name]
