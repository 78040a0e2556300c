"""Result comparison with the tolerances north_star states: longs / row selections / min / max
bit-exact, doubleSum within 1e-9 relative, floatSum within 1e-5 relative."""
import math

TOL = {"long": 0.0, "double": 1e-9, "float": 1e-5}


def _close(a, b, rel):
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    if rel == 0.0:  # exact: for floats also the sign of zero (Math.min/max order -0.0 < 0.0)
        if isinstance(a, float) or isinstance(b, float):
            return a == b and math.copysign(1.0, a) == math.copysign(1.0, b)
        return a == b
    if a == b:
        return True
    return abs(a - b) <= rel * max(abs(a), abs(b), 1e-300)


def agg_tolerance(agg):
    # sums reorder under parallel accumulation; min/max/count/longSum are exact
    if agg.type == "doubleSum":
        return TOL["double"]
    if agg.type == "floatSum":
        return TOL["float"]
    return 0.0


def assert_values(query, got: dict, exp: dict, ctx=""):
    assert set(got) == set(exp), f"{ctx}: keys {sorted(got)} != {sorted(exp)}"
    aggs = {a.name: a for a in query.aggregations}
    for k, v in exp.items():
        if k in aggs:
            assert _close(got[k], v, agg_tolerance(aggs[k])), f"{ctx}: {k}: got {got[k]!r} expected {v!r}"
        else:
            assert got[k] == v, f"{ctx}: {k}: got {got[k]!r} expected {v!r}"


def assert_results(query, got, exp):
    assert len(got) == len(exp), f"{len(got)} results vs {len(exp)}: {got[:3]} / {exp[:3]}"
    for i, (g, e) in enumerate(zip(got, exp)):
        assert g.timestamp == e.timestamp, f"result {i}: ts {g.timestamp} != {e.timestamp}"
        gv = getattr(g, "value", None)
        if gv is None:  # groupBy Row
            assert_values(query, g.event, e.event, f"row {i}")
        elif isinstance(gv, list):
            assert len(gv) == len(e.value), f"result {i}: {len(gv)} entries vs {len(e.value)}"
            for j, (a, b) in enumerate(zip(gv, e.value)):
                assert_values(query, a, b, f"result {i} entry {j}")
        else:
            assert_values(query, gv, e.value, f"result {i}")


def assert_kat(query, got, expected_json, rel=1e-6):
    """Against the reference's KATs: doubles at the reference's own 1e-6 relative tolerance."""
    import importlib
    Q = importlib.import_module("incubator-druid_amd.query")
    assert len(got) == len(expected_json), f"{got} vs {expected_json}"
    for g, e in zip(got, expected_json):
        assert g.timestamp == Q.parse_time(e["timestamp"]), (g.timestamp, e["timestamp"])
        exp = e["result"]
        rows = g.value if isinstance(exp, list) else [g.value]
        exps = exp if isinstance(exp, list) else [exp]
        assert len(rows) == len(exps), f"{rows} vs {exps}"
        for r, x in zip(rows, exps):
            for k, v in x.items():
                if isinstance(v, float):
                    assert abs(r[k] - v) <= rel * abs(v) + 1e-12, f"{k}: {r[k]} vs {v}"
                else:
                    assert r[k] == v, f"{k}: {r[k]} vs {v}"
