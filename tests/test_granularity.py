"""Calendar / zoned granularities: the host restatement that computes the engine's
bucket starts (incubator-druid_amd/granularity.py) and the oracle's own restatement, both pinned by
the reference's QueryGranularityTest vectors (tests/golden/granularity_kats.json, transcribed by
tests/golden/make_granularity_kats.py), then cross-checked against each other on random instants."""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def gkats():
    with open(os.path.join(GOLDEN, "granularity_kats.json")) as f:
        return json.load(f)["cases"]


def _run(Q, case, bucket_start, iterable):
    g = Q.Granularity.of(case["granularity"])
    if case["kind"] == "iterable":
        s, e = (Q.parse_time(x) for x in case["input"])
        got = [b for b, _ in iterable(g, (s, e))]
    else:
        got = [bucket_start(g, Q.parse_time(x)) for x in case["input"]]
    return g, got, [Q.parse_time(x) for x in case["expected"]]


def test_host_restatement_matches_reference_kats(Q, gkats):
    assert len(gkats) == 37
    for case in gkats:
        g, got, exp = _run(Q, case, lambda g, t: g.bucket_start(t), lambda g, iv: g.iterable(iv))
        assert got == exp, (case["name"], [Q.format_time(x) for x in got])


def test_oracle_restatement_matches_reference_kats(Q, O, gkats):
    for case in gkats:
        g, got, exp = _run(Q, case, O.o_bucket_start, O.o_iterable)
        assert got == exp, (case["name"], [Q.format_time(x) for x in got])


def test_calendar_mode_selection(Q):
    G = Q.Granularity
    assert G.of("month").is_calendar and G.of("year").is_calendar and G.of("quarter").is_calendar
    assert not G.of("day").is_calendar and not G.of("day").is_all
    assert G.of({"type": "period", "period": "P1D", "timeZone": "America/Los_Angeles"}).is_calendar
    assert not G.of({"type": "period", "period": "PT6H"}).is_calendar
    # P2W without an origin aligns on the zone's local epoch (a Thursday), P1W on Mondays
    assert G.of({"type": "period", "period": "P2W"}).origin_ms == 0
    assert G.of({"type": "period", "period": "P1W"}).origin_ms == -3 * 86_400_000
    js = G.of({"type": "period", "period": "P1M", "timeZone": "Asia/Kathmandu"}).to_json()
    assert G.of(js) == G.of({"type": "period", "period": "P1M", "timeZone": "Asia/Kathmandu"})


SPECS = [
    {"type": "period", "period": "P1M"},
    {"type": "period", "period": "P3M", "timeZone": "Europe/Berlin"},
    {"type": "period", "period": "P1Y", "timeZone": "Asia/Kathmandu"},
    {"type": "period", "period": "P1D", "timeZone": "America/Los_Angeles"},
    {"type": "period", "period": "P1W", "timeZone": "America/Sao_Paulo"},
    {"type": "period", "period": "PT1H", "timeZone": "Australia/Lord_Howe"},
    {"type": "period", "period": "PT2H", "timeZone": "Asia/Kolkata"},
    {"type": "period", "period": "P2D", "timeZone": "America/New_York", "origin": "2012-03-10T03:00:00Z"},
    {"type": "period", "period": "P1M2D", "timeZone": "America/Los_Angeles"},
    {"type": "period", "period": "P1M", "origin": "2011-01-31T00:00:00Z"},
    {"type": "period", "period": "PT12H5M", "timeZone": "Europe/London", "origin": "2012-01-02T05:00:00Z"},
    {"type": "period", "period": "P1DT12H", "timeZone": "+05:30"},
]


@pytest.mark.parametrize("spec", SPECS, ids=lambda s: s["period"] + "@" + s.get("timeZone", "UTC"))
def test_host_and_oracle_restatements_agree(Q, O, spec):
    """Two independent restatements of PeriodGranularity (Joda local-millis arithmetic vs Python
    wall-clock datetimes) on random instants around DST transitions and month ends."""
    g = Q.Granularity.of(spec)
    rng = np.random.default_rng(7)
    lo, hi = Q.parse_time("2010-01-01"), Q.parse_time("2014-01-01")
    ts = rng.integers(lo, hi, size=150).tolist() + [Q.parse_time(x) for x in (
        "2012-03-11T10:00:00Z", "2012-11-04T08:30:00Z", "2012-11-04T09:30:00Z", "2012-02-29T12:00:00Z",
        "2013-01-31T23:59:59.999Z", "2012-10-28T01:30:00Z", "2012-04-01T15:45:00Z")]
    for t in ts:
        b = g.bucket_start(t)
        assert b == O.o_bucket_start(g, t), (spec, Q.format_time(t))
        # (b <= t < increment(b) need not hold: month arithmetic clamps days, P1M from a 31st origin
        # truncates 2010-03-28T13:35 to 2010-02-28 whose increment is 2010-03-28T00:00 — in Joda too)
        assert b <= t, (spec, Q.format_time(t))
        assert g.increment(b) == O.o_increment(g, b)
    starts = g.bucket_starts((lo, lo + 200 * 86_400_000))
    assert starts == [b for b, _ in O.o_iterable(g, (lo, lo + 200 * 86_400_000))] + [starts[-1]]
    assert all(x < y for x, y in zip(starts, starts[1:]))


def test_segment_bucket_chains_diverge_only_for_clamped_origins(Q):
    """makeCursors buckets each segment on gran.getIterable(its actual interval): bucketStart of its
    first row, then increments. With an origin on a day that clamps (P1M from Jan 31) that chain is
    not the query interval's, and runners.segment_queries sends every segment down on its own."""
    import importlib
    R = importlib.import_module("incubator-druid_amd.runners")

    class Seg:
        def __init__(self, a, b):
            self.min_time, self.max_time, self.num_rows = Q.parse_time(a), Q.parse_time(b), 10

    segs = [Seg("2012-09-15", "2012-11-14"), Seg("2012-11-16", "2013-01-14"), Seg("2013-01-16", "2013-03-19")]
    iv = ["2012-09-20T05:00:00Z/2013-03-15T00:00:00Z"]
    for gran in ("month", "day", {"type": "period", "period": "P3M", "timeZone": "Europe/Berlin"}):
        assert R.segment_queries(Q.TimeseriesQuery(intervals=iv, granularity=gran), segs) is None
    q = Q.TimeseriesQuery(intervals=iv, granularity={"type": "period", "period": "P1M", "origin": "2000-01-31T00:00:00Z"})
    split = R.segment_queries(q, segs)
    assert [s.interval[0] for s in split] == [Q.parse_time(iv[0].split("/")[0]), segs[1].min_time, segs[2].min_time]
    g = q.granularity
    # segment 2's chain starts at Oct 31 (Jan 31 + 9 months), the query's has Oct 30 there
    assert g.bucket_start(segs[1].min_time) == Q.parse_time("2012-10-31")
    assert Q.parse_time("2012-10-30") in g.bucket_starts(q.interval)


def test_fixed_offset_zones_bucket_on_a_fixed_grid(Q):
    """A fixed-offset zone ("+05:30") with a period without months / years is an exact fixed grid
    (origin = the zone's local epoch), the same buckets as the calendar restatement, with no
    per-query bucket list (whose size is capped)."""
    rng = np.random.default_rng(3)
    ts = rng.integers(-3 * 10**12, 3 * 10**12, 400)
    for iso, tz, origin in (("P1D", "+05:30", None), ("PT1H", "-03:30", None), ("P1W", "+01:00", None),
                            ("PT6H", "+05:45", None), ("P2D", "-08:00", "2012-03-04T05:06:07Z"),
                            ("PT15M", "+05:30", None), ("PT1H30M", "-02:00", None)):
        g = Q.Granularity.period(iso, tz, origin)
        assert not g.is_calendar, (iso, tz)
        cal = g.calendar_form()
        for t in ts:
            if g.exact_from is not None and t < g.exact_from:
                continue
            assert g.bucket_start(int(t)) == cal.bucket_start(int(t)), (iso, tz, int(t))
    # a compound period whose origin has a negative Java remainder: truncateMillisPeriod is not the
    # grid's floor, so it stays on the calendar restatement
    assert Q.Granularity.period("PT1H30M", "+02:00").is_calendar


def test_hours_branch_before_the_origin(Q):
    """PeriodGranularity.truncate's hours branch (PeriodGranularity.java:313-326) with an origin <= 0:
    a timestamp before the origin gets the aligned point AFTER it (PT2H, default origin 0: -1.5 h ->
    0); after the origin it is the grid's floor. The fixed grid records this and the runners switch
    to the calendar restatement when the data reaches before the origin."""
    import importlib
    R = importlib.import_module("incubator-druid_amd.runners")
    g = Q.Granularity.period("PT2H")
    assert g.exact_from == 0 and g.origin_ms == 0
    cal = g.calendar_form()
    assert cal.bucket_start(-5_400_000) == 0  # the quirk
    assert cal.bucket_start(-7_200_000) == -7_200_000  # on the grid: itself
    assert cal.bucket_start(5_400_000) == 0 == g.bucket_start(5_400_000)
    assert Q.Granularity.period("PT1H").exact_from is None  # roundFloor branch

    class Seg:
        def __init__(self, a, b):
            self.min_time, self.max_time, self.num_rows = a, b, 10

    q = Q.TimeseriesQuery(intervals=["1960-01-01/1980-01-01"], granularity={"type": "period", "period": "PT2H"})
    assert R.exact_granularity(q, [Seg(0, 10**9)]) is q  # data after the origin: the grid is exact
    q2 = R.exact_granularity(q, [Seg(-10**9, 10**9)])
    assert q2.granularity.is_calendar and q2.interval == (-10**9, 10**9 + 1)
