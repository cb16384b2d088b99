"""A PromQL subset: instant-vector selectors and simple aggregations.

Enough for every query the reference issues (``app.py:157`` node discovery:
``kube_pod_info{pod=~".*<pod>.*"}``; ``app.py:167-172`` metric fetch:
``{__name__=~"a|b|c", instance=~"<ip>:.+"}``) plus what the new panels and the
K8s deployment's recording rules use:

    selector   := [metric_name] ['{' matcher (',' matcher)* [','] '}']
    matcher    := label ('=' | '!=' | '=~' | '!~') string
    aggregate  := ('sum'|'avg'|'min'|'max'|'count') [('by'|'without') '(' labels ')']
                  '(' selector ')' [('by'|'without') '(' labels ')']

Regex matchers are fully anchored, as in Prometheus. A selector must contain at
least one matcher that does not match the empty string (Prometheus' rule).
"""

from __future__ import annotations

import math
import re
from dataclasses import dataclass, field

_IDENT = re.compile(r"[a-zA-Z_:][a-zA-Z0-9_:]*")
_LABEL = re.compile(r"[a-zA-Z_][a-zA-Z0-9_]*")
_AGGS = ("sum", "avg", "min", "max", "count")


class PromQLError(ValueError):
    pass


@dataclass(frozen=True)
class Matcher:
    label: str
    op: str
    value: str
    _re: object = field(default=None, compare=False, repr=False)

    @staticmethod
    def make(label: str, op: str, value: str) -> "Matcher":
        rx = None
        if op in ("=~", "!~"):
            try:
                rx = re.compile(f"(?:{value})\\Z", re.DOTALL)
            except re.error as exc:
                raise PromQLError(f"invalid regex {value!r}: {exc}") from exc
        return Matcher(label, op, value, rx)

    def matches(self, v: str) -> bool:
        if self.op == "=":
            return v == self.value
        if self.op == "!=":
            return v != self.value
        hit = self._re.match(v) is not None
        return hit if self.op == "=~" else not hit


@dataclass(frozen=True)
class Selector:
    matchers: tuple

    def matches(self, labels: dict) -> bool:
        for m in self.matchers:
            if not m.matches(labels.get(m.label, "")):
                return False
        return True

    @property
    def metric_name(self):
        for m in self.matchers:
            if m.label == "__name__" and m.op == "=":
                return m.value
        return None


@dataclass(frozen=True)
class Aggregate:
    op: str
    selector: Selector
    by: tuple | None = None
    without: tuple | None = None


class _Lexer:
    def __init__(self, s: str):
        self.s = s
        self.i = 0

    def ws(self):
        while self.i < len(self.s) and self.s[self.i].isspace():
            self.i += 1

    def peek(self, tok: str) -> bool:
        self.ws()
        return self.s.startswith(tok, self.i)

    def eat(self, tok: str) -> bool:
        if self.peek(tok):
            self.i += len(tok)
            return True
        return False

    def expect(self, tok: str):
        if not self.eat(tok):
            raise PromQLError(f"expected {tok!r} at position {self.i} in {self.s!r}")

    def ident(self, rx=_IDENT):
        self.ws()
        m = rx.match(self.s, self.i)
        if not m:
            return None
        self.i = m.end()
        return m.group(0)

    def string(self) -> str:
        self.ws()
        if self.i >= len(self.s) or self.s[self.i] not in "\"'`":
            raise PromQLError(f"expected a string at position {self.i} in {self.s!r}")
        q = self.s[self.i]
        self.i += 1
        out = []
        while self.i < len(self.s):
            c = self.s[self.i]
            if c == q:
                self.i += 1
                return "".join(out)
            if c == "\\" and q != "`" and self.i + 1 < len(self.s):
                n = self.s[self.i + 1]
                out.append({"n": "\n", "t": "\t", "\\": "\\", '"': '"', "'": "'"}.get(n, "\\" + n))
                self.i += 2
                continue
            out.append(c)
            self.i += 1
        raise PromQLError("unterminated string")

    def done(self) -> bool:
        self.ws()
        return self.i >= len(self.s)


def _parse_selector(lx: _Lexer) -> Selector:
    name = lx.ident()
    matchers = []
    if name is not None:
        if name in _AGGS or name in ("by", "without"):
            raise PromQLError(f"unexpected keyword {name!r}")
        matchers.append(Matcher.make("__name__", "=", name))
    if lx.eat("{"):
        while not lx.eat("}"):
            label = lx.ident(_LABEL)
            if label is None:
                raise PromQLError(f"expected a label name at position {lx.i}")
            for op in ("=~", "!~", "!=", "="):
                if lx.eat(op):
                    break
            else:
                raise PromQLError(f"expected a matcher operator at position {lx.i}")
            matchers.append(Matcher.make(label, op, lx.string()))
            if not lx.eat(","):
                lx.expect("}")
                break
    if not matchers:
        raise PromQLError("empty selector")
    if all(m.matches("") for m in matchers):
        raise PromQLError("vector selector must contain at least one non-empty matcher")
    return Selector(tuple(matchers))


def _parse_grouping(lx: _Lexer):
    for kw in ("by", "without"):
        save = lx.i
        if lx.ident() == kw:
            lx.expect("(")
            labels = []
            while not lx.eat(")"):
                lab = lx.ident(_LABEL)
                if lab is None:
                    raise PromQLError("expected a label in grouping")
                labels.append(lab)
                if not lx.eat(","):
                    lx.expect(")")
                    break
            return kw, tuple(labels)
        lx.i = save
    return None, None


def parse(query: str):
    """Parse a query into a ``Selector`` or an ``Aggregate``."""
    lx = _Lexer(query.strip())
    save = lx.i
    word = lx.ident()
    if word in _AGGS:
        kw, labels = _parse_grouping(lx)
        lx.expect("(")
        sel = _parse_selector(lx)
        lx.expect(")")
        if kw is None:
            kw, labels = _parse_grouping(lx)
        if not lx.done():
            raise PromQLError(f"unexpected trailing input at position {lx.i}")
        return Aggregate(word, sel, labels if kw == "by" else None, labels if kw == "without" else None)
    lx.i = save
    sel = _parse_selector(lx)
    if not lx.done():
        raise PromQLError(f"unexpected trailing input at position {lx.i}")
    return sel


def aggregate(expr: Aggregate, series: list) -> list:
    """``series``: [(labels_dict, value)] matched by the selector -> aggregated list."""
    groups: dict = {}
    for labels, v in series:
        if expr.by is not None:
            key = tuple((k, labels[k]) for k in expr.by if k in labels)
        elif expr.without is None:  # plain `sum(x)`: one group, no labels
            key = ()
        else:
            drop = set(expr.without or ()) | {"__name__"}
            key = tuple(sorted((k, x) for k, x in labels.items() if k not in drop))
        groups.setdefault(key, []).append(v)
    out = []
    for key, vals in groups.items():
        finite = [x for x in vals if not math.isnan(x)]
        if expr.op == "count":
            r = float(len(vals))
        elif expr.op == "sum":
            r = float(sum(vals))
        elif expr.op == "avg":
            r = float(sum(vals)) / len(vals)
        elif expr.op == "min":
            r = min(finite) if finite else float("nan")
        else:
            r = max(finite) if finite else float("nan")
        out.append((dict(key), r))
    return out
