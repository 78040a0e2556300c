"""PeriodGranularity over Joda's ISO chronology in a time zone (host side of the calendar path).

Druid buckets rows by ``Granularity.getIterable(interval)`` (java-util/.../granularity/
Granularity.java:176-240): the first bucket starts at ``bucketStart(interval.start)`` and every next
one at ``increment(previous start)``. For periods the engine cannot express as a fixed-length UTC
grid (months, years, any period in a zone with daylight-saving or historical offset changes,
compound periods with calendar fields) the host computes that bucket list with the restatement
below and hands the bucket starts to the engine (``dg_scan.bucket_starts``); the kernels find a
row's bucket by binary search over them.

Restated from the reference (paths under java-util/src/main/java/org/apache/druid/java/util/common/):
* ``granularity/PeriodGranularity.java:58-74`` constructor (default origin = local 1970-01-01T00:00
  of the zone, ``withZoneRetainFields``), ``:212-221`` increment = ``chronology.add(period, t, 1)``,
  ``:222-410`` truncate (per-field roundFloor / set, origin-aligned multiples, compound periods via
  ``truncateMillisPeriod`` or ``truncateCompoundPeriod``), ``:432-445`` isCompoundPeriod.
* Joda-Time 2.9 semantics the above relies on (a pom dependency, not vendored): ZonedChronology's
  ZonedDateTimeField (roundFloor / set through ``convertLocalToUTC(local, false, original)``; time
  fields shorter than 12 h keep the instant's offset) and ZonedDurationField (add / getDifference
  on local millis for days and longer, on elapsed millis for time fields),
  ``DateTimeZone.getOffsetFromLocal`` (overlaps take the earlier instant, gaps move forward),
  BasicMonthOfYearDateTimeField.add / getDifferenceAsLong and BasicGJChronology.getYearDifference.

Pinned by the reference's QueryGranularityTest.java:318-866 vectors (tests/golden/granularity_kats.json).
"""
from __future__ import annotations

import datetime as _dt
import re
from functools import lru_cache
from typing import List, Optional, Tuple

DAY_MS = 86_400_000
_FIELD_MS = [None, None, 7 * DAY_MS, DAY_MS, 3_600_000, 60_000, 1000, 1]  # years..millis (precise ones)
_ISO = re.compile(r"P(?:(\d+)Y)?(?:(\d+)M)?(?:(\d+)W)?(?:(\d+)D)?(?:T(?:(\d+)H)?(?:(\d+)M)?(?:(\d+)(?:\.(\d{1,3}))?S)?)?")
_EPOCH_DATE = _dt.date(1970, 1, 1)
_FEB_29 = (31 + 29 - 1) * DAY_MS


def parse_period(s: str) -> Tuple[int, ...]:
    """ISO-8601 period -> (years, months, weeks, days, hours, minutes, seconds, millis)
    (org.joda.time.Period(String), PeriodType.standard field order)."""
    m = _ISO.fullmatch(s.strip().upper())
    if not m or not any(g is not None for g in m.groups()):
        raise ValueError(f"unparseable period {s!r}")
    y, mo, w, d, h, mi, se, frac = m.groups()
    vals = tuple(int(x or 0) for x in (y, mo, w, d, h, mi, se)) + (int((frac or "0").ljust(3, "0")),)
    if not any(vals):
        raise ValueError("zero period is not acceptable in QueryGranularity")
    return vals


def _jdiv(a: int, b: int) -> int:
    """Java long division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def _jrem(a: int, b: int) -> int:
    return a - _jdiv(a, b) * b


# ---- ISO calendar on local millis (proleptic Gregorian, as Joda's ISOChronology UTC) ----
def _split(ms: int):
    days, mod = divmod(ms, DAY_MS)
    return _EPOCH_DATE + _dt.timedelta(days=days), mod


def _date_ms(d: _dt.date) -> int:
    return (d - _EPOCH_DATE).days * DAY_MS


def _days_in_month(y: int, m: int) -> int:
    if m == 12:
        return 31
    return (_dt.date(y, m + 1, 1) - _dt.date(y, m, 1)).days


def _is_leap(y: int) -> bool:
    return y % 4 == 0 and (y % 100 != 0 or y % 400 == 0)


def _add_months(ms: int, months: int) -> int:
    """BasicMonthOfYearDateTimeField.add: month arithmetic, day of month clamped, time of day kept."""
    d, tod = _split(ms)
    z = d.year * 12 + (d.month - 1) + months
    y, m = divmod(z, 12)
    m += 1
    day = min(d.day, _days_in_month(y, m))
    return _date_ms(_dt.date(y, m, day)) + tod


def _month_diff(a: int, b: int) -> int:
    """BasicMonthOfYearDateTimeField.getDifferenceAsLong(minuend a, subtrahend b)."""
    if a < b:
        return -_month_diff(b, a)
    da, _ = _split(a)
    db, tb = _split(b)
    diff = (da.year - db.year) * 12 + da.month - db.month
    if da.day == _days_in_month(da.year, da.month) and db.day > da.day:
        b = _date_ms(db.replace(day=da.day)) + tb  # dayOfMonth().set(subtrahend, minuendDom)
        db, tb = _split(b)
    rem_a = a - _date_ms(_dt.date(da.year, da.month, 1))
    rem_b = b - _date_ms(_dt.date(db.year, db.month, 1))
    return diff - 1 if rem_a < rem_b else diff


def _year_diff(a: int, b: int) -> int:
    """BasicYearDateTimeField.getDifferenceAsLong -> BasicGJChronology.getYearDifference."""
    if a < b:
        return -_year_diff(b, a)
    ya, yb = _split(a)[0].year, _split(b)[0].year
    rem_a = a - _date_ms(_dt.date(ya, 1, 1))
    rem_b = b - _date_ms(_dt.date(yb, 1, 1))
    if rem_b >= _FEB_29:
        if _is_leap(yb):
            if not _is_leap(ya):
                rem_b -= DAY_MS
        elif rem_a >= _FEB_29 and _is_leap(ya):
            rem_a -= DAY_MS
    return ya - yb - 1 if rem_a < rem_b else ya - yb


# ---- zones ----
class Zone:
    """DateTimeZone: UTC, a fixed offset ("+05:30") or an IANA id (zoneinfo database)."""

    def __init__(self, name: Optional[str]):
        self.name = name or "UTC"
        self.fixed: Optional[int] = None
        n = self.name
        if n.upper() in ("UTC", "Z", "ETC/UTC", "GMT", "ETC/GMT"):
            self.fixed = 0
        elif re.fullmatch(r"[+-]\d{2}(:?\d{2})?", n):
            sign = 1 if n[0] == "+" else -1
            self.fixed = sign * (int(n[1:3]) * 60 + (int(n[-2:]) if len(n) > 3 else 0)) * 60_000
        else:
            from zoneinfo import ZoneInfo
            self.tz = ZoneInfo(n)

    @property
    def is_utc(self) -> bool:
        return self.fixed == 0

    def offset(self, t: int) -> int:
        """getOffset(instant)."""
        if self.fixed is not None:
            return self.fixed
        return _zone_offset(self.tz, t // 1000)

    def offset_from_local(self, local: int) -> int:
        """getOffsetFromLocal: a local time in an overlap maps to the earlier instant, one in a gap
        moves forward past it (zoneinfo fold=0 has exactly these semantics)."""
        if self.fixed is not None:
            return self.fixed
        d, tod = _split(local)
        naive = _dt.datetime(d.year, d.month, d.day) + _dt.timedelta(milliseconds=tod)
        off = naive.replace(tzinfo=self.tz, fold=0).utcoffset()
        return int(off // _dt.timedelta(milliseconds=1))

    def local(self, t: int) -> int:
        return t + self.offset(t)

    def to_utc(self, local: int, original: int) -> int:
        """convertLocalToUTC(local, strict=false, originalInstantUTC): keep the original instant's
        offset when it is valid at the result."""
        off = self.offset(original)
        u = local - off
        if self.offset(u) == off:
            return u
        return local - self.offset_from_local(local)


@lru_cache(maxsize=1 << 16)
def _zone_offset(tz, secs: int) -> int:
    dt = _dt.datetime.fromtimestamp(secs, tz) if -62135596800 < secs < 253402300799 else None
    if dt is None:
        return 0
    return int(dt.utcoffset() // _dt.timedelta(milliseconds=1))


class PeriodGranularity:
    """PeriodGranularity(period, origin, timeZone) restated (see the module docstring)."""

    def __init__(self, period: str, origin: Optional[int] = None, tz: Optional[str] = None):
        self.period_str = period
        self.p = parse_period(period)
        self.zone = Zone(tz)
        if origin is None:
            # new DateTime(0, UTC).withZoneRetainFields(zone).getMillis()
            self.origin = 0 - self.zone.offset_from_local(0)
            self.has_origin = False
        else:
            self.origin = int(origin)
            self.has_origin = True
        self.is_compound = sum(1 for v in self.p if v > 0) > 1

    # -- fixed-length UTC form (what the engine can bucket by arithmetic alone) --
    def standard_ms(self) -> Optional[int]:
        """Period.toStandardDuration() when the period has no months / years."""
        y, mo, w, d, h, mi, s, ms = self.p
        if y or mo:
            return None
        return ((((w * 7 + d) * 24 + h) * 60 + mi) * 60 + s) * 1000 + ms

    # -- Joda field operations in this chronology --
    def _add_field(self, i: int, t: int, v: int) -> int:
        if v == 0:
            return t
        z = self.zone
        if i >= 4:  # hours / minutes / seconds / millis: time fields (elapsed arithmetic)
            return t + v * _FIELD_MS[i]
        off = z.offset(t)
        loc = t + off
        if i == 0:
            loc = _add_months(loc, 12 * v)
        elif i == 1:
            loc = _add_months(loc, v)
        else:
            loc = loc + v * _FIELD_MS[i]
        return loc - z.offset_from_local(loc)

    def _diff_field(self, i: int, t: int, origin: int) -> int:
        z = self.zone
        off_o = z.offset(origin)
        if i >= 4:
            return _jdiv(t - origin, _FIELD_MS[i])
        a, b = t + z.offset(t), origin + off_o
        if i == 0:
            return _year_diff(a, b)
        if i == 1:
            return _month_diff(a, b)
        return _jdiv(a - b, _FIELD_MS[i])

    def add(self, t: int, scalar: int) -> int:
        """chronology.add(period, t, scalar): field by field, years first."""
        for i, v in enumerate(self.p):
            if v:
                t = self._add_field(i, t, v * scalar)
        return t

    def increment(self, t: int) -> int:
        return self.add(t, 1)

    # roundFloor / set of the calendar fields (not time fields: through local time)
    def _floor_local(self, t: int, fn) -> int:
        z = self.zone
        return z.to_utc(fn(z.local(t)), t)

    def _floor_time(self, t: int, unit: int) -> int:
        off = self.zone.offset(t)
        return (t + off) // unit * unit - off

    def _set_time(self, t: int, unit: int, span: int) -> int:
        """set(t, 0) of a time field whose value runs over `span` (e.g. hourOfDay: unit 1 h, span 1 d)."""
        z = self.zone
        loc = z.local(t)
        loc = loc - (loc % span) // unit * unit
        return z.to_utc(loc, t)

    def _aligned(self, i: int, t: int, n: int) -> int:
        """The origin-aligned multiple branch: difference in whole units from the origin (toward
        zero), rounded down to a multiple of n, one period back for timestamps before it."""
        k = self._diff_field(i, t, self.origin)
        k -= _jrem(k, n)
        tt = self._add_field(i, self.origin, k)
        return self._add_field(i, tt, -n) if t < tt else tt

    def truncate(self, t: int) -> int:
        if self.is_compound:
            std = self.standard_ms()
            if std is not None and self.zone.fixed is not None:  # truncateMillisPeriod
                off = _jrem(t, std) - _jrem(self.origin, std)
                if off < 0:
                    off += std
                return t - off
            return self._truncate_compound(t)
        y, mo, w, d, h, mi, s, ms = self.p
        if y:
            if y > 1 or self.has_origin:
                return self._aligned(0, t, y)
            return self._floor_local(t, lambda L: _date_ms(_dt.date(_split(L)[0].year, 1, 1)))
        if mo:
            if mo > 1 or self.has_origin:
                return self._aligned(1, t, mo)
            return self._floor_local(t, lambda L: _date_ms(_split(L)[0].replace(day=1)))
        if w:
            if w > 1 or self.has_origin:
                return self._aligned(2, t, w)
            t = self._floor_local(t, lambda L: L - L % DAY_MS)  # dayOfWeek().roundFloor
            # dayOfWeek().set(t, 1): Monday of the week (ISO day of week)
            return self._floor_local(t, lambda L: L - (_split(L)[0].isoweekday() - 1) * DAY_MS)
        if d:
            if d > 1 or self.has_origin:
                return self._aligned(3, t, d)
            t = self._floor_time(t, 3_600_000)  # hourOfDay().roundFloor
            return self._set_time(t, 3_600_000, DAY_MS)  # hourOfDay().set(t, 0)
        if h:
            if h > 1 or self.has_origin:
                k = self._diff_field(4, t, self.origin)
                k -= _jrem(k, h)
                tt = self._add_field(4, self.origin, k)
                if t < tt and self.origin > 0:
                    return self._add_field(4, tt, -h)
                if t > tt and self.origin < 0:
                    tt = self._floor_time(tt, 60_000)  # minuteOfHour().roundFloor
                    return self._set_time(tt, 60_000, 3_600_000)  # minuteOfHour().set(t, 0)
                return tt
            t = self._floor_time(t, 60_000)
            return self._set_time(t, 60_000, 3_600_000)
        if mi:
            if mi > 1 or self.has_origin:
                return self._aligned(5, t, mi)
            t = self._floor_time(t, 1000)
            return self._set_time(t, 1000, 60_000)
        if s:
            if s > 1 or self.has_origin:
                return self._aligned(6, t, s)
            return self._set_time(t, 1, 1000)  # millisOfSecond().set(t, 0)
        if ms:
            if ms > 1:
                return self._aligned(7, t, ms)
            return t
        return t

    def _truncate_compound(self, t: int) -> int:
        if t >= self.origin:
            nxt = self.origin
            while True:
                cur = nxt
                nxt = self.add(cur, 1)
                if not t >= nxt:
                    return cur
        cur = self.origin
        while True:
            cur = self.add(cur, -1)
            if not t < cur:
                return cur

    bucket_start = truncate

    def iterable_starts(self, start: int, end: int, limit: int = 1 << 22) -> List[int]:
        """Granularity.getIterable([start, end)): bucket starts, plus the end of the last bucket."""
        out = []
        cur = self.truncate(start)
        while cur < end:
            out.append(cur)
            if len(out) > limit:
                raise ValueError("too many granularity buckets")
            cur = self.increment(cur)
        out.append(cur)
        return out
