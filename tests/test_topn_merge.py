"""dg_topn_merge (the engine's TopNBinaryFn fold, host code of the C-ABI) against the oracle's
restatement of TopNBinaryFn.apply / TopNNumericResultBuilder (oracle/oracle.py merge_topn), on
randomized per-segment lists with heavy metric ties, every metric type, inverted ordering, empty
and no-cursor lists. No GPU needed: the merge is host code."""
import importlib

import numpy as np
import pytest

from compare import assert_results


def _encode(a, v):
    if a.output_type == "long":
        return np.int64(v).view(np.uint64)
    if a.output_type == "double":
        return np.float64(v).view(np.uint64)
    return np.uint64(np.float32(v).view(np.uint32))


def _rand_value(rng, a, ties):
    if a.output_type == "long":
        return int(rng.integers(-ties, ties))
    if a.output_type == "double":
        return float(rng.integers(-ties, ties)) * 0.5
    return float(np.float32(rng.integers(-ties, ties) * 0.25))


CASES = [
    ("longSum", "numeric", 3), ("doubleSum", "numeric", 4), ("floatSum", "numeric", 5),
    ("longMax", "inverted", 3), ("doubleMin", "numeric", 1000), ("count", "inverted", 6),
]


@pytest.mark.parametrize("metric_type,order,ties", CASES)
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_topn_merge_matches_oracle(Q, O, metric_type, order, ties, seed):
    R = importlib.import_module("incubator-druid_amd.runners")
    rng = np.random.default_rng(seed)
    values = [None] + sorted({f"v{rng.integers(0, 10**6)}" for _ in range(300)})  # Java order (ASCII)
    aggs = [Q.AggregatorFactory(metric_type, "m", "x"), Q.long_sum("ls", "y"), Q.double_sum("ds", "z"),
            Q.AggregatorFactory("floatMin", "fm", "w")]
    metric = {"numeric": Q.TopNMetricSpec("numeric", "m"),
              "inverted": Q.TopNMetricSpec("inverted", "m")}[order]
    q = Q.TopNQuery(intervals=["1970-01-01/2020-01-01"], dimension="d", metric=metric, threshold=7,
                    aggregations=aggs)
    K = 40
    nl = 6
    na = len(aggs)
    cnt = np.zeros(nl, dtype=np.int32)
    keys = np.zeros(nl * K, dtype=np.int64)
    vals = np.zeros(nl * K * na, dtype=np.uint64)
    ts = rng.integers(0, 3, size=nl).astype(np.int64) * 1000
    per = []
    for l in range(nl):
        if l == 2:
            cnt[l] = -1  # no cursor
            per.append([])
            continue
        n = 0 if l == 4 else int(rng.integers(1, K + 1))
        cnt[l] = n
        ids = np.sort(rng.choice(len(values), size=n, replace=False))
        entries = []
        for j, k in enumerate(ids):
            e = {"d": values[k]}
            keys[l * K + j] = k
            for a_i, a in enumerate(aggs):
                v = _rand_value(rng, a, ties) if a.type != "count" else int(rng.integers(0, ties))
                if a.type == "count":
                    v = abs(v)
                e[a.name] = v
                vals[(l * K + j) * na + a_i] = _encode(a, v)
            entries.append(e)
        # a per-segment list is already in builder order
        bob = O.NumericResultBuilder(O._metric_key_fn(q), K)
        for e in entries:
            bob.add(e["d"], e["m"], e)
        built = bob.build()
        order_ids = [values.index(e["d"]) for e in built]
        for j, e in enumerate(built):
            keys[l * K + j] = order_ids[j]
            for a_i, a in enumerate(aggs):
                vals[(l * K + j) * na + a_i] = _encode(a, e[a.name])
        per.append([Q.Result(int(ts[l]), built)])
    exp = O.merge_topn(q, per)
    res = R.topn_merge_raw(q, cnt, keys, vals, K, ts, handles=None)
    assert res is not None
    t0, _lists, out_keys, slots = res
    got = [Q.Result(t0, R._topn_entries(q, [values[int(k)] for k in out_keys], slots))]
    assert_results(q, got, exp)


def test_topn_merge_no_cursor_anywhere(Q):
    R = importlib.import_module("incubator-druid_amd.runners")
    q = Q.TopNQuery(intervals=["1970-01-01/2020-01-01"], dimension="d", metric="m", threshold=3,
                    aggregations=[Q.long_sum("m", "x")])
    cnt = np.full(3, -1, dtype=np.int32)
    assert R.topn_merge_raw(q, cnt, np.zeros(3 * 4, np.int64), np.zeros(3 * 4, np.uint64), 4,
                            np.zeros(3, np.int64)) is None


@pytest.mark.parametrize("ordering", ["lexicographic", "numeric", "alphanumeric", "strlen"])
@pytest.mark.parametrize("inverted", [False, True])
def test_dimension_order_merge_matches_oracle(O, Q, ordering, inverted):
    """runners.merge_dimension_lists (head-only fold when tie-free, literal fold otherwise) against
    the oracle's TopNBinaryFn fold with TopNLexicographicResultBuilder and the literal comparators;
    lists hold nulls (dropped when they reach a full queue) and comparator-equal values."""
    import random
    R = importlib.import_module("incubator-druid_amd.runners")
    rng = random.Random(hash((ordering, inverted)) & 0xffff)
    tie_pool = ["1", "1.0", "01", "a", "A", "x1", "X01", "ab", "AB"]
    plain_pool = [str(i) for i in range(15)] + list("bcdefg")
    for trial in range(150):
        ties = trial % 3 == 0
        pool = [None] + plain_pool + (tie_pool if ties else [])
        T, min_t = rng.randint(1, 5), rng.randint(1, 9)
        stop = rng.choice([None, "3", "c", ""])
        m = {"type": "dimension", "ordering": ordering, "previousStop": stop}
        q = Q.TopNQuery(intervals=["1970-01-01/2020-01-01"], dimension="v", threshold=T,
                        aggregations=[Q.count("rows"), Q.double_sum("d", "d")],
                        metric={"type": "inverted", "metric": m} if inverted else m,
                        context={"minTopNThreshold": min_t})
        cmp = O.topn_comparator(q.metric)
        per, lists = [], []
        for seg in range(rng.randint(1, 5)):
            vals = [v for v in rng.sample(pool, rng.randint(0, len(pool))) if stop is None or cmp(v, stop) > 0]
            b = O.LexicographicResultBuilder(cmp, q.segment_threshold, stop)
            for v in sorted(vals, key=lambda x: (x is not None, x or "")):  # any deterministic order
                b.add(v, {"v": v, "rows": rng.randint(1, 9), "d": rng.random()})
            entries = b.build()
            ts = rng.choice([0, 0, 5])
            per.append([Q.Result(ts, entries)] if entries or rng.random() < 0.8 else [])
            if per[-1]:
                slots = np.array([[_encode(q.aggregations[0], e["rows"]), _encode(q.aggregations[1], e["d"])]
                                  for e in entries], dtype=np.uint64).reshape(-1, 2)
                lists.append((ts, len(entries), (lambda j, en=entries: en[j]["v"]), slots))
        order = sorted(range(len(lists)), key=lambda i: (lists[i][0], i))
        tie_free = not ties
        got = R.merge_dimension_lists(q, [lists[i] for i in order], tie_free)
        exp = O.merge_topn(q, [p for p in per if p])
        assert_results(q, got, exp)
