"""String orderings of dimension values (query/ordering/StringComparators.java) as sort keys.

A dimension-ordered topN (DimensionTopNMetricSpec / LexicographicTopNMetricSpec /
AlphaNumericTopNMetricSpec, optionally inside InvertedTopNMetricSpec) ranks dictionary values by a
StringComparator. The engine does not compare strings on the device: the host hands it, once per
segment and ordering, the rank of every dictionary id (``dg_segment_set_dim_order``), exactly what a
JNI shim would compute by sorting the dictionary with the Java comparator itself. Here each
comparator is restated as a key function whose tuple order equals the comparator's order
(comparator-equal values get equal keys):

* LEXICOGRAPHIC (:48-70): nulls first, then unsigned UTF-8 bytes.
* NUMERIC (:346-392): nulls first; values neither GuavaUtils.tryParseLong nor new BigDecimal can
  parse come next in LEXICOGRAPHIC order; every parseable value after them by decimal value.
* STRLEN (:281-300): nulls first, UTF-16 length, then String.compareTo (UTF-16 units).
* ALPHANUMERIC (:99-279): nulls first, "" next, then the sequence of chunks the comparator walks:
  a digit chunk (smaller than any non-digit chunk) is keyed by the digits compareNumbers visits
  (count, then values; the first significant digit is visited twice and a run of zeros that ends
  the string visits its last zero, as the Java loop does), then its leading-zero count; a non-digit
  chunk by its UTF-16 units folded as String.CASE_INSENSITIVE_ORDER folds them.

InvertedTopNMetricSpec.getComparator (InvertedTopNMetricSpec.java:62-84) is
inverse(nulls-last delegate): nulls first, then the delegate order reversed.
"""
from __future__ import annotations

import bisect
import functools
from decimal import Decimal
from typing import List, Optional, Sequence, Tuple

import numpy as np

ORDER_IDS = {"lexicographic": 0, "numeric": 1, "alphanumeric": 2, "strlen": 3}


def order_slot(ordering: str, inverted: bool) -> int:
    """dg_segment_set_dim_order slot: 2 * DG_ORDER_* + inverted."""
    return 2 * ORDER_IDS[ordering] + int(bool(inverted))


# ---- LEXICOGRAPHIC ---------------------------------------------------------------------------
def _utf8(s: str) -> bytes:
    return s.encode("utf-8", "replace")


def lexicographic_key(s: Optional[str]):
    return (0,) if s is None else (1, _utf8(s))


# ---- NUMERIC ---------------------------------------------------------------------------------
def parse_long(s: str) -> Optional[int]:
    """GuavaUtils.tryParseLong (common/.../guava/GuavaUtils.java:37-42) -> Longs.tryParse."""
    if not s:
        return None
    t = s[1:] if s[0] == "+" else s
    body = t[1:] if t[:1] == "-" else t
    if not body or not body.isascii() or not body.isdigit():
        return None
    v = int(t)
    return v if -(1 << 63) <= v < (1 << 63) else None


def parse_big_decimal(s: str) -> Optional[Decimal]:
    """new BigDecimal(String): sign, Character.isDigit digits with at most one '.', optional
    [eE][sign]digits exponent that fits an int; None where Java throws NumberFormatException."""
    n = len(s)
    i = 1 if n and s[0] in "+-" else 0
    digits, frac, seen_dot = [], 0, False
    while i < n:
        ch = s[i]
        if ch == "." and not seen_dot:
            seen_dot = True
        elif ch.isdecimal():
            digits.append(int(ch))
            frac += seen_dot
        else:
            break
        i += 1
    if not digits:
        return None
    exp = 0
    if i < n:
        if s[i] not in "eE" or i + 1 >= n:
            return None
        j = i + 1
        sign = -1 if s[j] == "-" else 1
        if s[j] in "+-":
            j += 1
        if j >= n or not all(c.isdecimal() for c in s[j:]):
            return None
        exp = sign * int("".join(str(int(c)) for c in s[j:]))
        if not -(1 << 31) <= exp < (1 << 31):
            return None
    mant = int("".join(map(str, digits)))
    if s[:1] == "-":
        mant = -mant
    return Decimal(mant).scaleb(exp - frac)


def numeric_key(s: Optional[str]):
    if s is None:
        return (0,)
    v = parse_long(s)
    d = Decimal(v) if v is not None else parse_big_decimal(s)
    if d is None:
        return (1, _utf8(s))
    return (2, d)


# ---- STRLEN ----------------------------------------------------------------------------------
def _utf16(s: str) -> Tuple[int, ...]:
    b = s.encode("utf-16-le", "surrogatepass")
    return tuple(b[i] | (b[i + 1] << 8) for i in range(0, len(b), 2))


def strlen_key(s: Optional[str]):
    if s is None:
        return (0,)
    u = _utf16(s)
    return (1, len(u), u)


# ---- ALPHANUMERIC ----------------------------------------------------------------------------
_DIGIT_ZEROS = (0x30, 0x660, 0x6F0, 0x966, 0xFF10)


def _digit_value(cp: int) -> int:
    """-1 for a non-digit (AlphanumericComparator.isDigit), else valueOf(digit)."""
    for z in _DIGIT_ZEROS:
        if z <= cp <= z + 9:
            return cp - z
    return -1


def _cp_at(u: Sequence[int], i: int) -> int:
    c = u[i]
    if 0xD800 <= c <= 0xDBFF and i + 1 < len(u) and 0xDC00 <= u[i + 1] <= 0xDFFF:
        return 0x10000 + ((c - 0xD800) << 10) + (u[i + 1] - 0xDC00)
    return c


def _fold(c: int) -> int:
    """Character.toLowerCase(Character.toUpperCase(c)) on one UTF-16 unit."""
    u = chr(c).upper()
    c2 = ord(u) if len(u) == 1 else c
    lo = chr(c2).lower()
    return ord(lo) if len(lo) == 1 else c2


def alphanumeric_key(s: Optional[str]):
    if s is None:
        return (0,)
    u = _utf16(s)
    n = len(u)
    chunks = []
    pos = 0
    while pos < n:
        cp = _cp_at(u, pos)
        if _digit_value(cp) >= 0:
            zeros, ch = 0, -1
            while pos < n:
                ch = _cp_at(u, pos)
                if ch not in _DIGIT_ZEROS:
                    break
                zeros += 1
                pos += 2 if ch >= 0x10000 else 1
            visited = []
            while ch >= 0 and _digit_value(ch) >= 0:
                visited.append(_digit_value(ch))
                if pos < n:
                    ch = _cp_at(u, pos)
                    if _digit_value(ch) >= 0:
                        pos += 2 if ch >= 0x10000 else 1
                    else:
                        ch = -1
                else:
                    ch = -1
            chunks.append((0, len(visited), tuple(visited), zeros))
        else:
            start = pos
            pos += 2 if cp >= 0x10000 else 1
            while pos < n:
                ch = _cp_at(u, pos)
                if _digit_value(ch) >= 0:
                    break
                pos += 2 if ch >= 0x10000 else 1
            chunks.append((1, tuple(_fold(c) for c in u[start:pos])))
    return (1, tuple(chunks))


KEY_FUNCTIONS = {"lexicographic": lexicographic_key, "numeric": numeric_key, "alphanumeric": alphanumeric_key,
                 "strlen": strlen_key}


class _Desc:
    """Reverses a key's order (inverted orderings)."""
    __slots__ = ("k",)

    def __init__(self, k):
        self.k = k

    def __lt__(self, o):
        return o.k < self.k

    def __eq__(self, o):
        return self.k == o.k

    def __hash__(self):
        return hash(self.k)


_SORT_KEYS: dict = {}


def sort_key(ordering: str, inverted: bool = False):
    """Key function of the topN comparator: StringComparator, or InvertedTopNMetricSpec over it
    (memoized: merges rank the same head values query after query)."""
    fn = _SORT_KEYS.get((ordering, inverted))
    if fn is None:
        base = KEY_FUNCTIONS[ordering]
        raw = base if not inverted else (lambda s: (0,) if s is None else (1, _Desc(base(s))))
        fn = _SORT_KEYS[(ordering, inverted)] = functools.lru_cache(maxsize=1 << 16)(raw)
    return fn


class DictionaryOrder:
    """Rank of every id of one sorted dictionary under a topN comparator (dense: comparator-equal
    values share a rank), plus the previousStop cut (`min_rank`)."""

    def __init__(self, dictionary: Sequence[Optional[str]], ordering: str, inverted: bool = False):
        self.key = sort_key(ordering, inverted)
        keys = [self.key(v) for v in dictionary]
        order = sorted(range(len(keys)), key=keys.__getitem__)
        rank = np.zeros(len(keys), dtype=np.int32)
        self.distinct: List = []
        r = -1
        for i in order:
            if not self.distinct or self.distinct[-1] != keys[i]:
                self.distinct.append(keys[i])
                r += 1
            rank[i] = r
        self.rank = rank
        self.has_ties = len(self.distinct) < len(keys)

    def min_rank(self, previous_stop: Optional[str]) -> int:
        """Smallest rank a value needs to be after previousStop (comparator.compare(v, stop) > 0,
        TopNLexicographicResultBuilder.shouldAdd :166-174); 0 without a previousStop."""
        if previous_stop is None:
            return 0
        return bisect.bisect_right(self.distinct, self.key(previous_stop))
