"""Builds the TestIndex fixture segment from druid.sample.numeric.tsv (test fixture builder).

Rows and metrics follow processing/src/test/java/org/apache/druid/segment/TestIndex.java:70-137,
252-330: dimensions market, quality, qualityNumericString, placement, partial_null_column (string),
qualityLong / qualityFloat / qualityDouble (numeric dimensions stored as numeric columns), metrics
index (doubleSum), indexFloat (floatSum), indexMin (doubleMin), indexMinFloat (floatMin),
indexMaxFloat (floatMax), indexMaxPlusTen (doubleMax over the FLOAT expression index + 10). The
TSV has no duplicate (timestamp, dimensions) rows, so rollup leaves every row as is. The
multi-value 'placementish' dimension and the hyperUnique metric are not written (out of scope).
"""
import os
import sys

import numpy as np


def build(out_dir, repo_root, bitmap="concise", compression="lz4"):
    sys.path.insert(0, repo_root)
    import importlib
    W = importlib.import_module("incubator-druid_amd.writer")
    Q = importlib.import_module("incubator-druid_amd.query")
    tsv = os.path.join(os.path.dirname(os.path.abspath(__file__)), "druid.sample.numeric.tsv")
    rows = [line.rstrip("\n").split("\t") for line in open(tsv, encoding="utf-8")]
    rows = [r + [""] * (11 - len(r)) for r in rows]
    rows.sort(key=lambda r: (Q.parse_time(r[0]), r[1], r[2]))
    ts = np.array([Q.parse_time(r[0]) for r in rows], dtype=np.int64)
    index = np.array([float(r[9]) for r in rows], dtype=np.float64)
    dims = {}
    for name, col in (("market", 1), ("quality", 2), ("qualityNumericString", 6), ("placement", 7),
                      ("partial_null_column", 10)):
        dims[name] = W.encode_strings([r[col] or None for r in rows])
    metrics = {
        "qualityLong": ("long", np.array([int(r[3]) for r in rows], dtype=np.int64)),
        "qualityFloat": ("float", np.array([float(r[4]) for r in rows], dtype=np.float32)),
        "qualityDouble": ("double", np.array([float(r[5]) for r in rows], dtype=np.float64)),
        "index": ("double", index),
        "indexFloat": ("float", index.astype(np.float32)),
        "indexMin": ("double", index),
        "indexMinFloat": ("float", index.astype(np.float32)),
        "indexMaxFloat": ("float", index.astype(np.float32)),
        "indexMaxPlusTen": ("double", (index + 10).astype(np.float32).astype(np.float64)),
    }
    spec = W.SegmentSpec(timestamps=ts, dims=dims, metrics=metrics,
                         interval=(Q.parse_time("2011-01-12"), Q.parse_time("2011-05-01")))
    return W.write_segment(out_dir, spec, bitmap=bitmap, compression=compression)


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    print(build(sys.argv[1], os.path.dirname(os.path.dirname(here))))
