"""Synthetic segments of the reference benchmarks' ``basic`` schema.

Column distributions follow benchmarks/.../datagen/BenchmarkSchemas.java:44-97 and the generator
conventions of BenchmarkDataGenerator.java:75-145 (timestamps spread evenly over the schema's
interval [0, 1,000,000) ms, one seed per segment = 9999 + segment index). Values are drawn from a
seeded numpy generator, not Java's commons-math streams: parity is checked on the same segment
bytes between the CPU oracle and the GPU, so the streams need not match.

Single-value dimensions and numeric metrics are written; the schema's multi-value dimensions and the
hyperUnique complex metric are out of scope for the scan path and are not written.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import numpy as np

from .writer import SegmentSpec, encode_int_strings, write_segment

BASIC_INTERVAL = (0, 1_000_000)
BASIC_DIMS = ["dimSequential", "dimZipf", "dimUniform", "dimSequentialHalfNull", "dimHyperUnique", "dimNull"]
BASIC_METRICS = ["rows", "sumLongSequential", "maxLongUniform", "sumFloatNormal", "minFloatZipf"]


def _zipf(rng, n: int, lo: int, hi: int, s: float) -> np.ndarray:
    ks = np.arange(lo, hi + 1)
    ranks = np.arange(1, len(ks) + 1, dtype=np.float64)
    p = 1.0 / ranks ** s
    p /= p.sum()
    return rng.choice(ks, size=n, p=p)


def basic_columns(num_rows: int, seed: int, interval=BASIC_INTERVAL, row_offset: int = 0,
                  total_rows: Optional[int] = None, dims: Optional[Sequence[str]] = None,
                  metrics: Optional[Sequence[str]] = None):
    """Column arrays of one segment of the basic schema.

    row_offset/total_rows place this segment's rows inside a larger time-ordered stream (multi-segment
    datasets split one interval into consecutive time chunks).
    """
    rng = np.random.default_rng(seed)
    total = total_rows or num_rows
    start, end = interval
    step = (end - 1 - start) / total
    idx = np.arange(row_offset, row_offset + num_rows, dtype=np.float64)
    ts = np.minimum(np.round(start + (idx + 1) * step).astype(np.int64), end - 1)
    seq = np.arange(row_offset, row_offset + num_rows, dtype=np.int64)
    want_d = set(dims) if dims is not None else set(BASIC_DIMS)
    want_m = set(metrics) if metrics is not None else set(BASIC_METRICS)
    out_dims: Dict = {}
    if "dimSequential" in want_d:
        out_dims["dimSequential"] = encode_int_strings(seq % 1000)
    if "dimZipf" in want_d:
        out_dims["dimZipf"] = encode_int_strings(_zipf(rng, num_rows, 1, 101, 1.0))
    if "dimUniform" in want_d:
        out_dims["dimUniform"] = encode_int_strings(rng.integers(1, 100001, size=num_rows))
    if "dimSequentialHalfNull" in want_d:
        out_dims["dimSequentialHalfNull"] = encode_int_strings(seq % 1000, rng.random(num_rows) < 0.5)
    if "dimHyperUnique" in want_d:
        out_dims["dimHyperUnique"] = encode_int_strings(seq % 100000)
    if "dimNull" in want_d:
        out_dims["dimNull"] = ([""], np.zeros(num_rows, dtype=np.int32))
    out_m: Dict = {}
    if "rows" in want_m:
        out_m["rows"] = ("long", np.ones(num_rows, dtype=np.int64))
    if "sumLongSequential" in want_m:
        out_m["sumLongSequential"] = ("long", seq % 10000)
    if "maxLongUniform" in want_m:
        out_m["maxLongUniform"] = ("long", rng.integers(0, 501, size=num_rows).astype(np.int64))
    if "sumFloatNormal" in want_m:
        out_m["sumFloatNormal"] = ("double", rng.normal(5000.0, 1.0, size=num_rows))
    if "minFloatZipf" in want_m:
        out_m["minFloatZipf"] = ("double", _zipf(rng, num_rows, 0, 1000, 1.0).astype(np.float64))
    return SegmentSpec(timestamps=ts, dims=out_dims, metrics=out_m, interval=interval)


def write_basic_segment(out_dir: str, num_rows: int, seed: int = 9999, bitmap: str = "concise",
                        compression: str = "lz4", lz4_mode: str = "hc", long_encoding: str = "longs", **kw) -> str:
    spec = basic_columns(num_rows, seed, **kw)
    return write_segment(out_dir, spec, bitmap=bitmap, compression=compression, lz4_mode=lz4_mode,
                         long_encoding=long_encoding)


def write_basic_dataset(root: str, num_segments: int, rows_per_segment: int, base_seed: int = 9999,
                        bitmap: str = "concise", compression: str = "lz4", lz4_mode: str = "hc",
                        time_partitioned: bool = False, **kw) -> List[str]:
    """num_segments segments (seed 9999 + i, like TimeseriesBenchmark.java:260-266).

    time_partitioned=True splits the interval into consecutive chunks (one per segment), as a
    time-partitioned datasource would be; otherwise every segment spans the whole interval like the
    JMH benchmarks' segments do.
    """
    paths = []
    for i in range(num_segments):
        p = os.path.join(root, f"seg{i:04d}")
        if time_partitioned:
            spec = basic_columns(rows_per_segment, base_seed + i, row_offset=i * rows_per_segment,
                                 total_rows=num_segments * rows_per_segment, **kw)
        else:
            spec = basic_columns(rows_per_segment, base_seed + i, **kw)
        write_segment(p, spec, bitmap=bitmap, compression=compression, lz4_mode=lz4_mode)
        paths.append(p)
    return paths
