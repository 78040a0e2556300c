"""CPU: the N-rank bench's result checks (bench.rank_groupby_summary / evaluate_dist_groupby). Two ranks'
CPU-engine groups (rank-local merged ids, re-keyed to cluster ids with the exchange's maps) are merged
by key in rank order the way dg_merge combines them (GroupByMergingQueryRunnerV2.java:170-290) and cut
into two key ranges; the evaluation passes on that answer and fails when a group is lost, a group is
duplicated across ranges, the ranges are swapped or a value is off."""
import copy
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

CARD = 40
UNIVERSAL = 1_000


def _rank_data(rng, nvals):
    """A rank's merged dictionaries (as cluster ids, ascending) and its CPU groups."""
    maps = [np.sort(rng.choice(CARD, nvals, replace=False)).astype(np.int32) for _ in range(2)]
    pairs = {(int(a), int(b)) for a, b in zip(rng.integers(0, nvals, 400), rng.integers(0, nvals, 400))}
    pairs = sorted(pairs)
    m1 = np.array([p[0] for p in pairs], np.uint64)
    m2 = np.array([p[1] for p in pairs], np.uint64)
    groups = {"key": (m1 << np.uint64(32)) | m2,  # ALL granularity: bucket 0
              "lsum": rng.integers(-1000, 1000, len(pairs)).astype(np.int64),
              "dsum": rng.normal(0, 10, len(pairs))}
    dicts = [[f"v{int(c):03d}" for c in m] for m in maps]
    return maps, groups, dicts


def _merge(ranks):
    """Expected final result: every rank's groups in cluster ids, combined by key in rank order."""
    acc = {}
    for maps, g, _ in ranks:
        key = g["key"]
        m1 = (key >> np.uint64(32)).astype(np.int64)
        m2 = (key & np.uint64(0xFFFFFFFF)).astype(np.int64)
        for a, b, l, d in zip(maps[0][m1], maps[1][m2], g["lsum"], g["dsum"]):
            k = (UNIVERSAL, int(a), int(b))
            if k in acc:
                acc[k] = (acc[k][0] + int(l), acc[k][1] + float(d))
            else:
                acc[k] = (int(l), float(d))
    keys = sorted(acc)
    return keys, acc


def _final(keys, acc, lo, hi):
    ks = keys[lo:hi]
    return {"times": np.array([k[0] for k in ks], np.int64), "c1": np.array([k[1] for k in ks], np.int64),
            "c2": np.array([k[2] for k in ks], np.int64), "lsum": np.array([acc[k][0] for k in ks], np.int64),
            "dsum": np.array([acc[k][1] for k in ks], np.float64)}


def _summaries(ranks, finals):
    out = []
    for (maps, g, dicts), f in zip(ranks, finals):
        out.append(bench.rank_groupby_summary(f, g, dicts, (0, 0, 0, len(maps[0])), maps, dicts, UNIVERSAL,
                                              len(g["key"])))
    return out


def test_dist_groupby_checks(monkeypatch):
    monkeypatch.setattr(bench, "SAMPLE_BITS", 1)  # sample half of the groups (small data)
    rng = np.random.default_rng(7)
    ranks = [_rank_data(rng, 30), _rank_data(rng, 30)]
    keys, acc = _merge(ranks)
    cut = len(keys) // 2
    finals = [_final(keys, acc, 0, cut), _final(keys, acc, cut, len(keys))]
    good = bench.evaluate_dist_groupby(_summaries(ranks, finals))
    assert good["all_equal"], good
    assert good["groups"] == len(keys) and good["sample_groups"] > 0

    # a lost group
    lost = copy.deepcopy(finals)
    for k in lost[1]:
        lost[1][k] = lost[1][k][1:]
    r = bench.evaluate_dist_groupby(_summaries(ranks, lost))
    assert not r["all_equal"]
    # a group in both ranges (misrouted boundary)
    dup = [_final(keys, acc, 0, cut + 1), _final(keys, acc, cut, len(keys))]
    r = bench.evaluate_dist_groupby(_summaries(ranks, dup))
    assert not r["ranges_disjoint_ascending"] and not r["all_equal"]
    # ranges held by the wrong ranks
    r = bench.evaluate_dist_groupby(_summaries(ranks[::-1], finals[::-1]))
    assert not r["ranges_disjoint_ascending"] and not r["all_equal"]
    # a double off by more than 1e-9 relative (the totals can hide it; the sampled groups cannot)
    off = copy.deepcopy(finals)
    sel = np.flatnonzero(bench.sample_mask(off[0]["times"], off[0]["c1"], off[0]["c2"]))
    off[0]["dsum"][sel[0]] += 1e-3 * max(abs(off[0]["dsum"][sel[0]]), 1.0)
    r = bench.evaluate_dist_groupby(_summaries(ranks, off))
    assert not r["sample_equal"] and not r["all_equal"]
    # a wrong long sum on a sampled group
    off = copy.deepcopy(finals)
    off[1]["lsum"][np.flatnonzero(bench.sample_mask(off[1]["times"], off[1]["c1"], off[1]["c2"]))[0]] += 1
    r = bench.evaluate_dist_groupby(_summaries(ranks, off))
    assert not r["long_sum_equal"] and not r["sample_long_sums_equal"] and not r["all_equal"]


def test_sample_mask_is_deterministic_and_sparse():
    rng = np.random.default_rng(1)
    t = np.zeros(200_000, np.int64)
    a, b = rng.integers(0, 1 << 17, 200_000), rng.integers(0, 1 << 17, 200_000)
    m = bench.sample_mask(t, a, b)
    assert np.array_equal(m, bench.sample_mask(t, a, b))
    assert 0.5 / 1024 < m.mean() < 2.0 / 1024
