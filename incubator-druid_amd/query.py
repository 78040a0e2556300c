"""Native query model: the JSON query specs of Druid's timeseries / topN / groupBy (v2) path.

Mirrors the reference's query objects closely enough that a Druid native query JSON can be
fed in unchanged (``Query.from_json``):

* granularities: java-util/.../granularity/{Granularity,AllGranularity,PeriodGranularity}.java
  (bucketStart / increment / getIterable, PeriodGranularity.java:222-230,411-428)
* filters: query/filter/{SelectorDimFilter,InDimFilter,BoundDimFilter,AndDimFilter,OrDimFilter,
  NotDimFilter}.java (``toFilter`` / ``optimize``, e.g. InDimFilter.java:132-139)
* aggregators: query/aggregation/{Count,LongSum,DoubleSum,FloatSum,LongMin,LongMax,DoubleMin,
  DoubleMax,FloatMin,FloatMax}AggregatorFactory.java (combine / comparator / initial values)
* queries: query/timeseries/TimeseriesQuery.java, query/topn/TopNQuery.java,
  query/groupby/GroupByQuery.java; topN metric specs NumericTopNMetricSpec / InvertedTopNMetricSpec
  / DimensionTopNMetricSpec.

Only the null-handling mode the reference defaults to is modelled
(``druid.generic.useDefaultValueForNull=true``, common/config/NullHandling.java:34,54):
null string == "" and numeric nulls read as 0.
"""
from __future__ import annotations

import datetime as _dt
import functools
import math
import re
import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

# ----------------------------------------------------------------------------------------------
# time helpers
# ----------------------------------------------------------------------------------------------
MIN_INSTANT = -(2 ** 62)   # JodaUtils.MIN_INSTANT (Long.MIN_VALUE / 2)
MAX_INSTANT = 2 ** 62 - 1  # JodaUtils.MAX_INSTANT
_EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)


def parse_time(s) -> int:
    """ISO-8601 instant (or epoch millis) -> epoch millis (UTC)."""
    if isinstance(s, (int,)):
        return int(s)
    s = str(s).strip()
    if re.fullmatch(r"-?\d+", s) and len(s) > 8:
        return int(s)
    m = re.fullmatch(r"(\d{4})(?:-(\d{2})(?:-(\d{2}))?)?(?:T(\d{2})(?::(\d{2})(?::(\d{2})(?:\.(\d{1,3}))?)?)?)?(Z|[+-]\d{2}:?\d{2})?", s)
    if not m:
        raise ValueError(f"unparseable time {s!r}")
    y, mo, d, h, mi, se, ms, tz = m.groups()
    t = _dt.datetime(int(y), int(mo or 1), int(d or 1), int(h or 0), int(mi or 0), int(se or 0),
                     tzinfo=_dt.timezone.utc)
    millis = int((t - _EPOCH) // _dt.timedelta(milliseconds=1)) + int((ms or "0").ljust(3, "0"))
    if tz and tz != "Z":
        sign = 1 if tz[0] == "+" else -1
        hh, mm = int(tz[1:3]), int(tz[-2:])
        millis -= sign * (hh * 3600 + mm * 60) * 1000
    return millis


def format_time(ms: int) -> str:
    t = _EPOCH + _dt.timedelta(milliseconds=int(ms))
    return t.strftime("%Y-%m-%dT%H:%M:%S.") + f"{int(ms) % 1000:03d}Z"


def parse_interval(s) -> Tuple[int, int]:
    if isinstance(s, (tuple, list)):
        return int(s[0]), int(s[1])
    a, b = str(s).split("/")
    return parse_time(a), parse_time(b)


# ----------------------------------------------------------------------------------------------
# granularity
# ----------------------------------------------------------------------------------------------
_PERIOD_MS = {
    "none": 1, "second": 1000, "minute": 60_000, "five_minute": 300_000, "ten_minute": 600_000,
    "fifteen_minute": 900_000, "thirty_minute": 1_800_000, "hour": 3_600_000, "six_hour": 21_600_000,
    "day": 86_400_000, "week": 604_800_000,
}
_ISO_PERIOD = re.compile(r"P(?:(\d+)W)?(?:(\d+)D)?(?:T(?:(\d+)H)?(?:(\d+)M)?(?:(\d+)S)?)?")


@dataclass(frozen=True)
class Granularity:
    """ALL (period_ms == 0), a fixed-length UTC period with an origin, or a calendar granularity.

    Fixed: bucketStart(t) = t - floorMod(t - origin, period) (PeriodGranularity.truncateMillisPeriod,
    PeriodGranularity.java:411-428, UTC so fixed-length days/hours/weeks); Joda weeks start on
    Monday, so WEEK carries origin 1969-12-29 (Monday) = -3 days.
    Calendar (name "calendar"): any other PeriodGranularity — months / years, a time zone, compound
    periods with calendar fields — bucketed through the Joda restatement of granularity.py; the
    engine receives its bucket starts (dg_scan.bucket_starts).
    """
    period_ms: int = 0
    origin_ms: int = 0
    name: str = "all"
    iso: str = ""                   # calendar: ISO-8601 period
    tz: str = ""                    # calendar: time zone id ("" = UTC)
    origin: Optional[int] = None    # calendar: the spec's origin (None = the zone's local epoch)
    exact_from: Optional[int] = None  # fixed grid of a period spec: exact only for t >= this (None: always)

    @property
    def is_all(self) -> bool:
        return self.period_ms == 0 and self.name != "calendar"

    @property
    def is_calendar(self) -> bool:
        return self.name == "calendar"

    @property
    def calendar(self):
        return _calendar(self.iso, self.origin, self.tz or None)

    def bucket_start(self, t: int) -> int:
        if self.is_calendar:
            return self.calendar.truncate(t)
        if self.is_all:
            return MIN_INSTANT
        return t - ((t - self.origin_ms) % self.period_ms)

    def increment(self, t: int) -> int:
        if self.is_calendar:
            return self.calendar.increment(t)
        if self.is_all:
            return MAX_INSTANT
        return t + self.period_ms

    def bucket_end(self, t: int) -> int:
        return self.increment(self.bucket_start(t))

    def iterable(self, interval: Tuple[int, int]) -> List[Tuple[int, int]]:
        """Granularity.getIterable (Granularity.java:176-240); AllGranularity yields the input."""
        s, e = interval
        if self.is_all:
            return [(s, e)]
        if self.is_calendar:
            b = self.calendar.iterable_starts(s, e)
            return list(zip(b[:-1], b[1:]))
        out = []
        cur = self.bucket_start(s)
        while cur < e:
            out.append((cur, cur + self.period_ms))
            cur += self.period_ms
        return out

    def bucket_starts(self, interval: Tuple[int, int]) -> List[int]:
        """Calendar: starts of the buckets getIterable(interval) yields, then the end of the last."""
        return self.calendar.iterable_starts(*interval)

    def to_json(self):
        if self.is_all:
            return "all"
        if self.is_calendar:
            js = {"type": "period", "period": self.iso}
            if self.tz:
                js["timeZone"] = self.tz
            if self.origin is not None:
                js["origin"] = format_time(self.origin)
            return js
        if self.name in _PERIOD_MS:
            return self.name
        if self.iso:  # a period spec bucketed on its fixed grid
            js = {"type": "period", "period": self.iso}
            if self.tz:
                js["timeZone"] = self.tz
            if self.origin is not None:
                js["origin"] = format_time(self.origin)
            return js
        return {"type": "duration", "duration": self.period_ms, "origin": self.origin_ms}

    @staticmethod
    def period(iso: str, tz: Optional[str] = None, origin=None) -> "Granularity":
        """PeriodGranularity(period, origin, timeZone): the fixed grid when it is exact, else calendar.
        Exact: a period without months / years in UTC or a fixed-offset zone ("+05:30"), where every
        truncate branch (PeriodGranularity.java:222-330) is a floor on the grid of the period from the
        origin (default: the zone's local epoch, 0 - offset; P1W: its Monday). Two quirks of the hours
        branch (:313-326) are not: an origin < 0 off the local hour rounds to the hour (calendar), and
        with an origin <= 0 a timestamp before the origin gets the aligned point AFTER it — exact on the
        grid only at or after the origin, so the grid records `exact_from` and the runners switch to
        the calendar restatement when the data reaches before it (compound periods likewise before 0)."""
        from .granularity import Zone, parse_period
        y, mo, w, d, h, mi, s, ms = parse_period(iso)
        utc = tz in (None, "", "UTC", "Etc/UTC")
        off = 0 if utc else Zone(tz).fixed  # fixed offset in ms, None for a zone with rules
        o = parse_time(origin) if origin is not None else None
        single = sum(1 for v in (y, mo, w, d, h, mi, s, ms) if v) == 1
        hours_branch = bool(h) and single and (h > 1 or o is not None)
        # hours with an origin before 1970 not on the (local) hour: PeriodGranularity.java:313-315 floors to the hour
        quirk = bool(h) and single and o is not None and o < 0 and (o + (off or 0)) % 3_600_000 != 0
        if off is not None and not (y or mo) and not quirk:
            P = ((((w * 7 + d) * 24 + h) * 60 + mi) * 60 + s) * 1000 + ms
            default_origin = (-3 * 86_400_000 if (w == 1 and single) else 0) - off  # P1W: Mondays
            org = o if o is not None else default_origin
            exact_from = None
            if not single:
                # compound: truncateMillisPeriod (PeriodGranularity.java:411-428) = t - (t % P - origin % P,
                # + P once if negative) with Java remainders: the grid's floor only for t >= 0 and a
                # non-negative origin remainder
                if math.fmod(org, P) < 0:
                    return Granularity(0, 0, "calendar", iso.upper(), "" if utc else tz, o)
                exact_from = 0
            elif hours_branch and org <= 0:
                exact_from = org
            return Granularity(P, org, "period", iso.upper(), "" if utc else tz, o, exact_from)
        return Granularity(0, 0, "calendar", iso.upper(), "" if utc else tz, o)

    def calendar_form(self) -> "Granularity":
        """The same PeriodGranularity bucketed through the calendar restatement."""
        return Granularity(0, 0, "calendar", self.iso, self.tz, self.origin)

    @staticmethod
    def of(spec) -> "Granularity":
        if isinstance(spec, Granularity):
            return spec
        if spec is None:
            return ALL
        if isinstance(spec, str):
            k = spec.lower()
            if k == "all":
                return ALL
            if k in _PERIOD_MS:
                return Granularity(_PERIOD_MS[k], -3 * 86_400_000 if k == "week" else 0, k)
            if k in _CALENDAR:  # Granularities.MONTH / QUARTER / YEAR (GranularityType.java)
                return Granularity.period(_CALENDAR[k])
            raise ValueError(f"unsupported granularity {spec!r}")
        t = spec.get("type")
        if t == "all":
            return ALL
        if t == "duration":
            origin = parse_time(spec["origin"]) if spec.get("origin") is not None else 0
            return Granularity(int(spec["duration"]), origin, "duration")
        if t == "period":
            return Granularity.period(spec["period"], spec.get("timeZone"), spec.get("origin"))
        raise ValueError(f"unsupported granularity {spec!r}")


_CALENDAR = {"month": "P1M", "quarter": "P3M", "year": "P1Y"}


@functools.lru_cache(maxsize=64)
def _calendar(iso: str, origin: Optional[int], tz: Optional[str]):
    from .granularity import PeriodGranularity
    return PeriodGranularity(iso, origin, tz)


ALL = Granularity(0, 0, "all")
HOUR = Granularity.of("hour")
DAY = Granularity.of("day")


# ----------------------------------------------------------------------------------------------
# filters
# ----------------------------------------------------------------------------------------------
class DimFilter:
    def to_json(self) -> Dict[str, Any]:
        raise NotImplementedError

    def optimize(self) -> "DimFilter":
        return self

    @staticmethod
    def from_json(js) -> Optional["DimFilter"]:
        if js is None:
            return None
        if isinstance(js, DimFilter):
            return js
        t = js["type"]
        if t == "selector":
            return SelectorDimFilter(js["dimension"], js.get("value"))
        if t == "in":
            return InDimFilter(js["dimension"], list(js["values"]))
        if t == "bound":
            return BoundDimFilter(js["dimension"], js.get("lower"), js.get("upper"),
                                  bool(js.get("lowerStrict", False)), bool(js.get("upperStrict", False)),
                                  _ordering_name(js.get("ordering"), js.get("alphaNumeric", False)))
        if t == "and":
            return AndDimFilter([DimFilter.from_json(f) for f in js["fields"]])
        if t == "or":
            return OrDimFilter([DimFilter.from_json(f) for f in js["fields"]])
        if t == "not":
            return NotDimFilter(DimFilter.from_json(js["field"]))
        if t == "regex":
            return RegexDimFilter(js["dimension"], js["pattern"])
        if t == "search":
            return SearchQueryDimFilter(js["dimension"], dict(js["query"]))
        if t == "like":
            return LikeDimFilter(js["dimension"], js["pattern"], js.get("escape"))
        raise ValueError(f"unsupported filter type {t!r}")


def _ordering_name(o, alpha_numeric=False) -> str:
    if o is None:
        return "alphanumeric" if alpha_numeric else "lexicographic"
    if isinstance(o, dict):
        o = o.get("type")
    return str(o).lower()


def _empty_to_null(v):
    return None if v is None or v == "" else str(v)


@dataclass
class SelectorDimFilter(DimFilter):
    dimension: str
    value: Optional[str]

    def to_json(self):
        return {"type": "selector", "dimension": self.dimension, "value": self.value}


@dataclass
class InDimFilter(DimFilter):
    dimension: str
    values: List[Optional[str]]

    def optimize(self):
        # InDimFilter.optimize (InDimFilter.java:132-139): single value -> selector
        vals = sorted({_empty_to_null(v) or "" for v in self.values})
        if len(vals) == 1:
            return SelectorDimFilter(self.dimension, _empty_to_null(vals[0]))
        return InDimFilter(self.dimension, [_empty_to_null(v) for v in vals])

    def to_json(self):
        return {"type": "in", "dimension": self.dimension, "values": list(self.values)}


@dataclass
class BoundDimFilter(DimFilter):
    dimension: str
    lower: Optional[str] = None
    upper: Optional[str] = None
    lowerStrict: bool = False
    upperStrict: bool = False
    ordering: str = "lexicographic"

    def to_json(self):
        return {"type": "bound", "dimension": self.dimension, "lower": self.lower, "upper": self.upper,
                "lowerStrict": self.lowerStrict, "upperStrict": self.upperStrict, "ordering": self.ordering}


@dataclass
class AndDimFilter(DimFilter):
    fields: List[DimFilter]

    def optimize(self):
        fs = [f.optimize() for f in self.fields]
        return fs[0] if len(fs) == 1 else AndDimFilter(fs)

    def to_json(self):
        return {"type": "and", "fields": [f.to_json() for f in self.fields]}


@dataclass
class OrDimFilter(DimFilter):
    fields: List[DimFilter]

    def optimize(self):
        fs = [f.optimize() for f in self.fields]
        return fs[0] if len(fs) == 1 else OrDimFilter(fs)

    def to_json(self):
        return {"type": "or", "fields": [f.to_json() for f in self.fields]}


@dataclass
class NotDimFilter(DimFilter):
    field: DimFilter

    def optimize(self):
        return NotDimFilter(self.field.optimize())

    def to_json(self):
        return {"type": "not", "field": self.field.to_json()}


# ---- predicate filters: evaluated over dictionary values (DimensionPredicateFilter ->
# Filters.matchPredicate, segment/filter/Filters.java:239-290), i.e. the union of the bitmaps of every
# value the predicate accepts; a missing column is all-true iff the predicate accepts null ----
def _java_regex(pattern: str) -> "re.Pattern":
    """java.util.regex.Pattern.compile for the common syntax (Python re; \\p{..} classes and
    possessive quantifiers are not translated)."""
    return re.compile(pattern)


def _region_matches_ignore_case(s: str, i: int, sub: str) -> bool:
    """String.regionMatches(true, i, sub, 0, len): per UTF-16 char, equal after toUpperCase or
    toLowerCase (BMP characters; Python's case tables)."""
    def up(c):
        u = c.upper()
        return u if len(u) == 1 else c

    def low(c):
        u = c.lower()
        return u if len(u) == 1 else c

    for a, b in zip(s[i:i + len(sub)], sub):
        if a == b:
            continue
        ua, ub = up(a), up(b)
        if ua == ub or low(ua) == low(ub):
            continue
        return False
    return True


def contains_ignore_case(s: Optional[str], sub: Optional[str]) -> bool:
    """commons-lang StringUtils.containsIgnoreCase."""
    if s is None or sub is None:
        return False
    return any(_region_matches_ignore_case(s, i, sub) for i in range(len(s) - len(sub) + 1))


@dataclass
class RegexDimFilter(DimFilter):
    """RegexDimFilter -> RegexFilter (segment/filter/RegexFilter.java:44-48): non-null and find()."""
    dimension: str
    pattern: str

    def predicate(self, v: Optional[str]) -> bool:
        return v is not None and _java_regex(self.pattern).search(v) is not None

    def to_json(self):
        return {"type": "regex", "dimension": self.dimension, "pattern": self.pattern}


@dataclass
class SearchQueryDimFilter(DimFilter):
    """SearchQueryDimFilter with a SearchQuerySpec (query/search/*SearchQuerySpec.java accept()):
    contains / insensitive_contains (StringUtils.containsIgnoreCase), fragment (every value
    contained), regex (find), all."""
    dimension: str
    query: Dict[str, Any]

    def predicate(self, v: Optional[str]) -> bool:
        q, t = self.query, self.query.get("type")
        if t == "all":
            return True
        if v is None:
            return False
        if t in ("contains", "insensitive_contains"):
            val = q.get("value")
            if val is None:
                return False
            if t == "contains" and q.get("caseSensitive", False):
                return val in v
            return contains_ignore_case(v, val)
        if t == "fragment":
            vals = q.get("values")
            if vals is None:
                return False
            if q.get("caseSensitive", False):
                return all(x in v for x in set(vals))
            return all(contains_ignore_case(v, x) for x in set(vals))
        if t == "regex":
            return _java_regex(q["pattern"]).search(v) is not None
        raise ValueError(f"unsupported search query spec {t!r}")

    def to_json(self):
        return {"type": "search", "dimension": self.dimension, "query": dict(self.query)}


@dataclass
class LikeDimFilter(DimFilter):
    """LikeDimFilter.LikeMatcher (query/filter/LikeDimFilter.java:75-158): % -> .*, _ -> ., the escape
    character quotes the next one, other characters outside [\\w\\d\\s-] as \\uXXXX; matches()
    over nullToEmpty(value) in default null mode."""
    dimension: str
    pattern: str
    escape: Optional[str] = None

    def _regex(self) -> "re.Pattern":
        esc = self.escape[0] if self.escape else None
        out, escaping = [], False
        for c in self.pattern:
            if esc is not None and c == esc and not escaping:
                escaping = True
            elif c == "%" and not escaping:
                out.append(".*")
            elif c == "_" and not escaping:
                out.append(".")
            else:
                out.append(c if re.fullmatch(r"[A-Za-z0-9_\s-]", c) else "\\u%04x" % ord(c) if ord(c) < 0x10000
                           else re.escape(c))
                escaping = False
        return re.compile("".join(out))

    def predicate(self, v: Optional[str]) -> bool:
        return self._regex().fullmatch("" if v is None else v) is not None

    def to_json(self):
        js = {"type": "like", "dimension": self.dimension, "pattern": self.pattern}
        if self.escape is not None:
            js["escape"] = self.escape
        return js


PREDICATE_FILTERS = (RegexDimFilter, SearchQueryDimFilter, LikeDimFilter)


# ----------------------------------------------------------------------------------------------
# aggregators
# ----------------------------------------------------------------------------------------------
AGG_KINDS = {
    "count": 0, "longSum": 1, "doubleSum": 2, "floatSum": 3, "longMin": 4, "longMax": 5,
    "doubleMin": 6, "doubleMax": 7, "floatMin": 8, "floatMax": 9,
}
AGG_OUTPUT = {0: "long", 1: "long", 4: "long", 5: "long", 2: "double", 6: "double", 7: "double",
              3: "float", 8: "float", 9: "float"}


def _f32(x: float) -> float:
    return struct.unpack("<f", struct.pack("<f", x))[0]


def java_min(a, b):
    """java.lang.Math.min for doubles/floats (NaN-propagating, -0.0 < +0.0)."""
    if a != a:
        return a
    if a == 0.0 and b == 0.0 and math.copysign(1.0, b) < 0:
        return b
    return a if a <= b else b


def java_max(a, b):
    if a != a:
        return a
    if a == 0.0 and b == 0.0 and math.copysign(1.0, a) < 0:
        return b
    return a if a >= b else b


def _wrap64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


@dataclass
class AggregatorFactory:
    """An aggregator factory; `filter` set = FilteredAggregatorFactory around it
    (query/aggregation/FilteredAggregatorFactory.java:40-73: the delegate aggregates a row only when
    the filter's ValueMatcher matches it; name, combine and comparator are the delegate's)."""
    type: str
    name: str
    fieldName: Optional[str] = None
    filter: Optional["DimFilter"] = None

    def __post_init__(self):
        if self.type not in AGG_KINDS:
            raise ValueError(f"unsupported aggregator type {self.type!r}")

    @property
    def kind(self) -> int:
        return AGG_KINDS[self.type]

    @property
    def output_type(self) -> str:
        return AGG_OUTPUT[self.kind]

    def initial(self):
        """Aggregator reset / BufferAggregator.init values."""
        k = self.kind
        if k in (0, 1):
            return 0
        if k == 4:
            return (1 << 63) - 1
        if k == 5:
            return -(1 << 63)
        if k in (2, 3):
            return 0.0
        if k in (6, 8):
            return math.inf
        return -math.inf

    def combine(self, a, b):
        """AggregatorFactory.combine (e.g. LongSumAggregator.combineValues, FloatSumAggregator.java:40-43)."""
        k = self.kind
        if k in (0, 1):
            return _wrap64(int(a) + int(b))
        if k == 4:
            return min(int(a), int(b))
        if k == 5:
            return max(int(a), int(b))
        if k == 2:
            return float(a) + float(b)
        if k == 3:
            return _f32(_f32(a) + _f32(b))
        if k in (6, 8):
            r = java_min(float(a), float(b))
            return _f32(r) if k == 8 else r
        r = java_max(float(a), float(b))
        return _f32(r) if k == 9 else r

    def compare_key(self, v):
        """Sort key realising the factory comparator (Long.compare / Doubles.compare)."""
        if self.output_type == "long":
            return (0, int(v))
        v = float(v)
        if v != v:
            return (1, 0.0)  # Double.compare: NaN is greatest
        if v == 0.0:
            return (0, -0.0 if math.copysign(1.0, v) < 0 else 0.0, 1 if math.copysign(1.0, v) > 0 else 0)
        return (0, v, 0)

    def to_json(self):
        js = {"type": self.type, "name": self.name}
        if self.fieldName is not None:
            js["fieldName"] = self.fieldName
        if self.filter is not None:
            return {"type": "filtered", "filter": self.filter.to_json(), "aggregator": js}
        return js

    @staticmethod
    def from_json(js) -> "AggregatorFactory":
        if isinstance(js, AggregatorFactory):
            return js
        if js["type"] == "filtered":
            inner = AggregatorFactory.from_json(js["aggregator"])
            f = DimFilter.from_json(js["filter"])
            if f is None:
                raise ValueError("filtered aggregator without a filter")
            # FilteredAggregatorFactory(FilteredAggregatorFactory(x, f1), f2) matches f2 and then f1
            both = f if inner.filter is None else AndDimFilter([f, inner.filter])
            return AggregatorFactory(inner.type, inner.name, inner.fieldName, both)
        return AggregatorFactory(js["type"], js["name"], js.get("fieldName"))


def filtered(agg: AggregatorFactory, flt) -> AggregatorFactory:
    """FilteredAggregatorFactory(agg, filter)."""
    return AggregatorFactory.from_json({"type": "filtered", "filter": flt, "aggregator": agg})


def count(name="count"):
    return AggregatorFactory("count", name)


def long_sum(name, field_name=None):
    return AggregatorFactory("longSum", name, field_name or name)


def double_sum(name, field_name=None):
    return AggregatorFactory("doubleSum", name, field_name or name)


def float_sum(name, field_name=None):
    return AggregatorFactory("floatSum", name, field_name or name)


def long_min(name, field_name=None):
    return AggregatorFactory("longMin", name, field_name or name)


def long_max(name, field_name=None):
    return AggregatorFactory("longMax", name, field_name or name)


def double_min(name, field_name=None):
    return AggregatorFactory("doubleMin", name, field_name or name)


def double_max(name, field_name=None):
    return AggregatorFactory("doubleMax", name, field_name or name)


def float_min(name, field_name=None):
    return AggregatorFactory("floatMin", name, field_name or name)


def float_max(name, field_name=None):
    return AggregatorFactory("floatMax", name, field_name or name)


# ----------------------------------------------------------------------------------------------
# topN metric specs
# ----------------------------------------------------------------------------------------------
@dataclass
class TopNMetricSpec:
    """numeric (metric name), inverted(numeric), or dimension ordering (DimensionTopNMetricSpec,
    LexicographicTopNMetricSpec, AlphaNumericTopNMetricSpec; `inverted` = InvertedTopNMetricSpec
    around it)."""
    type: str = "numeric"
    metric: Optional[str] = None
    ordering: str = "lexicographic"
    previous_stop: Optional[str] = None
    inverted: bool = False

    @staticmethod
    def of(spec) -> "TopNMetricSpec":
        if isinstance(spec, TopNMetricSpec):
            return spec
        if isinstance(spec, str):
            return TopNMetricSpec("numeric", spec)
        t = spec.get("type")
        if t == "numeric":
            return TopNMetricSpec("numeric", spec["metric"])
        if t == "inverted":
            inner = TopNMetricSpec.of(spec["metric"])
            if inner.type == "dimension":
                return TopNMetricSpec("dimension", None, inner.ordering, inner.previous_stop, not inner.inverted)
            if inner.type != "numeric":
                raise ValueError("only inverted numeric or dimension metric specs are supported")
            return TopNMetricSpec("inverted", inner.metric)
        if t in ("dimension", "lexicographic", "alphaNumeric"):
            ordering = _ordering_name(spec.get("ordering"), t == "alphaNumeric")
            return TopNMetricSpec("dimension", None, ordering, spec.get("previousStop"))
        raise ValueError(f"unsupported topN metric spec {spec!r}")

    def to_json(self):
        if self.type == "numeric":
            return {"type": "numeric", "metric": self.metric}
        if self.type == "inverted":
            return {"type": "inverted", "metric": {"type": "numeric", "metric": self.metric}}
        js = {"type": "dimension", "ordering": self.ordering, "previousStop": self.previous_stop}
        return {"type": "inverted", "metric": js} if self.inverted else js


# ----------------------------------------------------------------------------------------------
# queries
# ----------------------------------------------------------------------------------------------
@dataclass
class BaseQuery:
    dataSource: str = "ds"
    intervals: List[Tuple[int, int]] = field(default_factory=lambda: [(MIN_INSTANT, MAX_INSTANT)])
    granularity: Granularity = ALL
    filter: Optional[DimFilter] = None
    aggregations: List[AggregatorFactory] = field(default_factory=list)
    context: Dict[str, Any] = field(default_factory=dict)

    def __post_init__(self):
        self.intervals = [parse_interval(i) for i in self.intervals]
        if len(self.intervals) != 1:
            raise ValueError("exactly one query interval is supported (TopNQueryEngine.java:75-77)")
        self.granularity = Granularity.of(self.granularity)
        self.filter = DimFilter.from_json(self.filter)
        self.aggregations = [AggregatorFactory.from_json(a) for a in self.aggregations]
        names = [a.name for a in self.aggregations]
        if len(set(names)) != len(names):
            raise ValueError("duplicate aggregator names")

    @property
    def interval(self) -> Tuple[int, int]:
        return self.intervals[0]

    def effective_filter(self) -> Optional[DimFilter]:
        return self.filter.optimize() if self.filter is not None else None

    def _base_json(self, qtype):
        js = {"queryType": qtype, "dataSource": self.dataSource,
              "intervals": [f"{format_time(s)}/{format_time(e)}" for s, e in self.intervals],
              "granularity": self.granularity.to_json(),
              "aggregations": [a.to_json() for a in self.aggregations]}
        if self.filter is not None:
            js["filter"] = self.filter.to_json()
        if self.context:
            js["context"] = dict(self.context)
        return js


@dataclass
class TimeseriesQuery(BaseQuery):
    descending: bool = False

    @property
    def skip_empty_buckets(self) -> bool:
        return bool(self.context.get("skipEmptyBuckets", False))

    def to_json(self):
        js = self._base_json("timeseries")
        js["descending"] = self.descending
        return js


@dataclass
class TopNQuery(BaseQuery):
    dimension: str = ""
    metric: Any = None
    threshold: int = 10

    def __post_init__(self):
        super().__post_init__()
        if isinstance(self.dimension, dict):
            if self.dimension.get("extractionFn") is not None:
                raise ValueError("extraction functions are out of scope")
            self.dimension = self.dimension["dimension"]
        self.metric = TopNMetricSpec.of(self.metric)
        if self.metric.type in ("numeric", "inverted") and self.metric.metric not in {a.name for a in self.aggregations}:
            raise ValueError("topN metric must name an aggregator")

    @property
    def min_topn_threshold(self) -> int:
        # TopNQueryConfig.minTopNThreshold = 1000 (TopNQueryConfig.java:32), context override
        return int(self.context.get("minTopNThreshold", 1000))

    @property
    def segment_threshold(self) -> int:
        """Per-segment threshold after TopNQueryQueryToolChest.preMergeQueryDecoration (:553-561)."""
        return max(self.threshold, self.min_topn_threshold)

    def to_json(self):
        js = self._base_json("topN")
        js.update({"dimension": self.dimension, "metric": self.metric.to_json(), "threshold": self.threshold})
        return js


@dataclass
class OrderByColumnSpec:
    """groupby/orderby/OrderByColumnSpec.java: column, direction, dimensionOrder (StringComparator)."""
    dimension: str
    direction: str = "ascending"
    dimensionOrder: str = "lexicographic"

    @staticmethod
    def from_json(js) -> "OrderByColumnSpec":
        if isinstance(js, str):
            return OrderByColumnSpec(js)
        d = str(js.get("direction", "ascending")).lower()
        if d in ("asc", "ascending"):
            d = "ascending"
        elif d in ("desc", "descending"):
            d = "descending"
        else:
            raise ValueError(f"Unknown direction[{d}]")
        order = js.get("dimensionOrder", "lexicographic") or "lexicographic"
        if isinstance(order, dict):
            order = order.get("type", "lexicographic")
        order = str(order).lower()
        if order not in ("lexicographic", "alphanumeric", "numeric", "strlen"):
            raise ValueError(f"unsupported dimensionOrder {order!r}")
        return OrderByColumnSpec(js["dimension"], d, order)

    def to_json(self):
        return {"dimension": self.dimension, "direction": self.direction, "dimensionOrder": self.dimensionOrder}


@dataclass
class DefaultLimitSpec:
    """groupby/orderby/DefaultLimitSpec.java: ORDER BY columns + LIMIT (None = Integer.MAX_VALUE)."""
    columns: List[OrderByColumnSpec] = field(default_factory=list)
    limit: Optional[int] = None

    @staticmethod
    def from_json(js) -> Optional["DefaultLimitSpec"]:
        if js is None:
            return None
        t = js.get("type", "default")
        if t == "noop":
            return None
        if t != "default":
            raise ValueError(f"unsupported limitSpec {t!r}")
        limit = js.get("limit")
        if limit is not None and int(limit) <= 0:
            raise ValueError(f"limit[{limit}] must be >0")
        return DefaultLimitSpec([OrderByColumnSpec.from_json(c) for c in js.get("columns") or []],
                                None if limit is None else int(limit))

    def to_json(self):
        js = {"type": "default", "columns": [c.to_json() for c in self.columns]}
        if self.limit is not None:
            js["limit"] = self.limit
        return js


@dataclass
class HavingSpec:
    """groupby/having/*HavingSpec.java as a tree: type in greaterThan / lessThan / equalTo
    (aggregation, value), dimSelector (dimension, value), and / or (specs), not (specs[0]), always,
    never."""
    type: str
    aggregation: Optional[str] = None
    value: Any = None
    dimension: Optional[str] = None
    specs: List["HavingSpec"] = field(default_factory=list)

    @staticmethod
    def from_json(js) -> Optional["HavingSpec"]:
        if js is None:
            return None
        t = js["type"]
        if t in ("greaterThan", "lessThan", "equalTo"):
            return HavingSpec(t, aggregation=js["aggregation"], value=js["value"])
        if t == "dimSelector":
            if js.get("extractionFn") is not None:
                raise ValueError("extraction functions are out of scope")
            return HavingSpec(t, dimension=js["dimension"], value=js.get("value"))
        if t in ("and", "or"):
            return HavingSpec(t, specs=[HavingSpec.from_json(x) for x in js["havingSpecs"]])
        if t == "not":
            return HavingSpec(t, specs=[HavingSpec.from_json(js["havingSpec"])])
        if t in ("always", "never"):
            return HavingSpec(t)
        raise ValueError(f"unsupported having {t!r}")

    def to_json(self):
        if self.type in ("greaterThan", "lessThan", "equalTo"):
            return {"type": self.type, "aggregation": self.aggregation, "value": self.value}
        if self.type == "dimSelector":
            return {"type": self.type, "dimension": self.dimension, "value": self.value}
        if self.type in ("and", "or"):
            return {"type": self.type, "havingSpecs": [x.to_json() for x in self.specs]}
        if self.type == "not":
            return {"type": "not", "havingSpec": self.specs[0].to_json()}
        return {"type": self.type}


@dataclass
class GroupByQuery(BaseQuery):
    dimensions: List[str] = field(default_factory=list)
    limitSpec: Optional[DefaultLimitSpec] = None
    having: Optional[HavingSpec] = None

    def __post_init__(self):
        super().__post_init__()
        if isinstance(self.limitSpec, dict):
            self.limitSpec = DefaultLimitSpec.from_json(self.limitSpec)
        if isinstance(self.having, dict):
            self.having = HavingSpec.from_json(self.having)
        dims = []
        for d in self.dimensions:
            if isinstance(d, dict):
                if d.get("extractionFn") is not None:
                    raise ValueError("extraction functions are out of scope")
                dims.append(d["dimension"])
            else:
                dims.append(d)
        self.dimensions = dims

    def _ctx_bool(self, key: str, default: bool) -> bool:
        v = (self.context or {}).get(key, default)
        if isinstance(v, str):  # QueryContexts.parseBoolean: Boolean.parseBoolean of a string
            return v.strip().lower() == "true"
        return bool(v)

    def order_by_dims(self) -> Optional[List[int]]:
        """Dimension index of every ORDER BY column (OrderByColumnSpec.getDimIndexForOrderBy), or None
        when one sorts on a non-grouping field (DefaultLimitSpec.sortingOrderHasNonGroupingFields)."""
        idx = []
        for c in (self.limitSpec.columns if self.limitSpec else []):
            if c.dimension not in self.dimensions:
                return None
            idx.append(self.dimensions.index(c.dimension))
        return idx

    def apply_limit_push_down(self) -> bool:
        """GroupByQuery.determineApplyLimitPushDown / validateAndGetForceLimitPushDown
        (query/groupby/GroupByQuery.java:352-416): a limited DefaultLimitSpec ordered by grouping
        dimensions only, no having spec, applyLimitPushDown not switched off in the context. A forced
        push-down (forceLimitPushDown) that sorts on aggregators is not pushed here: the reference
        then truncates every segment's grouper by partial aggregates (approximate); this engine
        returns the exact ordering instead."""
        ls = self.limitSpec
        force = self._ctx_bool("forceLimitPushDown", False)
        if force:
            if ls is None:
                raise ValueError("When forcing limit push down, a limit spec must be provided.")
            if ls.limit is None:
                raise ValueError("When forcing limit push down, the provided limit spec must have a limit.")
            if self.having is not None:
                raise ValueError("Cannot force limit push down when a having spec is present.")
        if ls is None or ls.limit is None:
            return False
        if not force and (not self._ctx_bool("applyLimitPushDown", True) or self.having is not None):
            return False
        return self.order_by_dims() is not None

    def to_json(self):
        js = self._base_json("groupBy")
        js["dimensions"] = list(self.dimensions)
        if self.limitSpec is not None:
            js["limitSpec"] = self.limitSpec.to_json()
        if self.having is not None:
            js["having"] = self.having.to_json()
        return js


def query_from_json(js: Dict[str, Any]):
    qt = js["queryType"]
    common = dict(dataSource=js.get("dataSource", "ds"), intervals=js["intervals"],
                  granularity=js.get("granularity", "all"), filter=js.get("filter"),
                  aggregations=js.get("aggregations", []), context=js.get("context", {}) or {})
    if qt == "timeseries":
        return TimeseriesQuery(descending=bool(js.get("descending", False)), **common)
    if qt == "topN":
        return TopNQuery(dimension=js["dimension"], metric=js["metric"], threshold=int(js["threshold"]), **common)
    if qt == "groupBy":
        return GroupByQuery(dimensions=js.get("dimensions", []), limitSpec=js.get("limitSpec"),
                            having=js.get("having"), **common)
    raise ValueError(f"unsupported queryType {qt!r}")


@dataclass
class Result:
    """Result<T> (query/Result.java): timestamp + value (dict for timeseries, list for topN)."""
    timestamp: int
    value: Any

    def to_json(self):
        return {"timestamp": format_time(self.timestamp), "result": self.value}


@dataclass
class Row:
    """groupBy MapBasedRow: timestamp + event."""
    timestamp: int
    event: Dict[str, Any]

    def to_json(self):
        return {"version": "v1", "timestamp": format_time(self.timestamp), "event": self.event}
