"""Multi-GPU merging: one process per GPU, partials exchanged with torch.distributed.

Segments shard naturally over GPUs (ChainedExecutionQueryRunner.java:103-144 runs every segment
independently); each rank runs its segments through the GPU engine and the per-rank partials are
merged with one collective per query — backend "nccl" (= RCCL over xGMI) on MI355X, "gloo" on CPU:

* timeseries: per-bucket partial aggregates -> all_reduce (SUM for count/long/double sums, MIN/MAX
  for min/max aggregators on order-preserving integer keys; float sums are reduced in float32 like
  FloatSumAggregator.combine), then TimeseriesBinaryFn semantics per bucket.
* topN: per-segment top-K lists (dictionary values mapped to a cluster-wide id space) ->
  all_gather of fixed-size [segments, K, 1 + aggs] tensors; rank 0 folds them with TopNBinaryFn in
  global segment order inside the engine (dg_topn_merge) — the reference's approximation
  (per-segment top max(K, 1000), pairwise merge to the query threshold) is kept exactly.
* groupBy: per-rank merged groups -> all_gather of row counts + padded (time, ids, aggs) tensors;
  rank 0 merges by key (GroupByMergingQueryRunnerV2.java:170-290).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import query as Q
from . import runners as R


def _torch():
    import torch
    import torch.distributed as dist
    return torch, dist


def init_from_env(prefer_nccl: bool = True):
    """Initialise the default process group from torchrun's env (MASTER_ADDR=127.0.0.1)."""
    torch, dist = _torch()
    if dist.is_initialized():
        return dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    backend = "nccl" if (prefer_nccl and torch.cuda.is_available()) else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return dist


def _device(dist):
    torch, _ = _torch()
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class GlobalDictionary:
    """Cluster-wide id space of one dimension: the union of every rank's segment dictionaries in
    Java String order (nulls first), built once per datasource at segment-load time."""

    def __init__(self, values: Sequence[Optional[str]]):
        self.values = list(values)
        self.index = {v: i for i, v in enumerate(self.values)}

    def translate(self, local_values: Sequence[Optional[str]]) -> np.ndarray:
        """segment-local dictionary id -> cluster-wide id (computed once per segment at load time)"""
        return np.fromiter((self.index[v] for v in local_values), dtype=np.int64, count=len(local_values))

    @staticmethod
    def build(dist, local_dicts: Sequence[Sequence[Optional[str]]]) -> "GlobalDictionary":
        local = set()
        for d in local_dicts:
            local.update(d)
        gathered: List = [None] * dist.get_world_size()
        dist.all_gather_object(gathered, sorted(local, key=R._java_key))
        allv = set()
        for g in gathered:
            allv.update(g)
        return GlobalDictionary(sorted(allv, key=R._java_key))


# ----------------------------------------------------------------------------------------------
# timeseries
# ----------------------------------------------------------------------------------------------
def allreduce_timeseries(dist, query: Q.TimeseriesQuery, local: List[Q.Result],
                         buckets: Optional[Sequence[int]] = None):
    """Reduce this rank's merged timeseries results over all ranks (every rank gets the result).

    `buckets` is the cluster-wide, identical-on-every-rank list of bucket keys (bucket starts; [0] for
    ALL granularity); None derives it with one all_gather_object of the local keys. Ranks without
    data for a bucket contribute identities."""
    torch, _ = _torch()
    dev = _device(dist)
    gran = query.granularity
    if buckets is None:
        mine = sorted({0 if gran.is_all else gran.bucket_start(r.timestamp) for r in local})
        gathered: List = [None] * dist.get_world_size()
        dist.all_gather_object(gathered, mine)
        buckets = sorted({b for g in gathered for b in g})
    nb, aggs = len(buckets), query.aggregations
    pos = {b: i for i, b in enumerate(buckets)}
    present = np.zeros(nb, dtype=np.int64)
    ts = np.full(nb, Q.MAX_INSTANT, dtype=np.int64)
    cols = {a.name: np.full(nb, a.initial(), dtype=_np_type(a)) for a in aggs}
    for r in local:
        i = pos[0 if gran.is_all else gran.bucket_start(r.timestamp)]
        present[i] = 1
        ts[i] = r.timestamp
        for a in aggs:
            cols[a.name][i] = r.value[a.name]
    t_present = torch.from_numpy(present).to(dev)
    dist.all_reduce(t_present, op=dist.ReduceOp.MAX)
    t_ts = torch.from_numpy(ts).to(dev)
    dist.all_reduce(t_ts, op=dist.ReduceOp.MIN)
    out_cols = {}
    for a in aggs:
        t = torch.from_numpy(cols[a.name].copy()).to(dev)
        op = dist.ReduceOp.SUM if a.kind in (0, 1, 2, 3) else (dist.ReduceOp.MIN if a.kind in (4, 6, 8) else dist.ReduceOp.MAX)
        dist.all_reduce(t, op=op)
        out_cols[a.name] = t.cpu().numpy()
    present = t_present.cpu().numpy()
    ts = t_ts.cpu().numpy()
    out = []
    for i, b in enumerate(buckets):
        if not present[i]:
            continue
        out.append(Q.Result(int(ts[i]) if gran.is_all else int(b),
                            {a.name: R._py(out_cols[a.name][i], a.output_type) for a in aggs}))
    if query.descending:
        out.reverse()
    return out


def _np_type(a):
    return {"long": np.int64, "double": np.float64, "float": np.float32}[a.output_type]


# ----------------------------------------------------------------------------------------------
# topN
# ----------------------------------------------------------------------------------------------
def gather_topn(dist, query: Q.TopNQuery, raw: "R.TopNRaw", gdict: GlobalDictionary,
                translations: Sequence[np.ndarray], segments: Optional[Sequence] = None) -> Optional[List[Q.Result]]:
    """all_gather every rank's per-segment top-K lists (ids mapped to the cluster-wide dictionary);
    rank 0 folds them with TopNBinaryFn in global segment order (rank-major) inside the engine
    (dg_topn_merge, global-id mode) and returns the result; other ranks return None.

    The reference's approximation is kept exactly: each segment contributes its own top
    max(threshold, 1000) list and the fold truncates to the query threshold after every step."""
    torch, _ = _torch()
    dev = _device(dist)
    K = raw.K
    na = len(query.aggregations)
    if not query.granularity.is_all:
        # one list per (segment, cursor): ranks hold different cursor counts, so the lists travel as
        # objects; rank 0 folds them per bucket (merge_topn) in global segment order
        local = []
        for s in range(len(raw.cnt) // raw.bcap):
            res = []
            for b in range(raw.bcap):
                L = s * raw.bcap + b
                c = int(raw.cnt[L])
                if c < 0:
                    continue
                values = [gdict.values[int(g)] for g in translations[s][raw.ids[L * K:L * K + c]]]
                slots = raw.vals.reshape(-1, max(na, 1))[L * K:L * K + c, :na]
                res.append(Q.Result(int(raw.ts[L]), R._topn_entries(query, values, slots)))
            local.append(res)
        gathered: List = [None] * dist.get_world_size()
        dist.all_gather_object(gathered, local)
        if dist.get_rank() != 0:
            return None
        return R.merge_topn(query, [lst for g in gathered for lst in g])
    S = len(raw.cnt)
    cnt = raw.cnt.astype(np.int64)
    gids = np.full((S, K), -1, dtype=np.int64)
    for s in range(S):
        c = int(cnt[s])
        if c > 0:
            gids[s, :c] = translations[s][raw.ids[s * K:s * K + c]]
    vals = raw.vals.reshape(S, K, max(na, 1)).view(np.int64)
    dim_spec = query.metric if query.metric.type == "dimension" else None
    ties = np.zeros(S, dtype=np.int64)  # dimension orders: does the segment's order have ties
    if dim_spec is not None:
        for s in range(S):
            o = segments[s].dim_order(query.dimension, dim_spec.ordering, dim_spec.inverted) if segments else None
            ties[s] = int(o is not None and o.has_ties)
    payload = torch.from_numpy(np.concatenate([raw.ts.astype(np.int64), cnt, gids.ravel(), vals.ravel(),
                                               ties])).to(dev)
    world = dist.get_world_size()
    bufs = [torch.empty_like(payload) for _ in range(world)]
    dist.all_gather(bufs, payload)
    if dist.get_rank() != 0:
        return None
    arrs = [b.cpu().numpy() for b in bufs]
    ts = np.concatenate([a[:S] for a in arrs])
    cn = np.concatenate([a[S:2 * S] for a in arrs]).astype(np.int32)
    keys = np.concatenate([a[2 * S:2 * S + S * K] for a in arrs])
    vv = np.concatenate([a[2 * S + S * K:len(a) - S] for a in arrs]).view(np.uint64)
    if dim_spec is not None:  # TopNLexicographicResultBuilder fold over the gathered lists
        tie_free = not any(int(a[len(a) - S + s]) for a in arrs for s in range(S))
        slots = vv.reshape(-1, max(na, 1))
        order = sorted((i for i in range(len(cn)) if cn[i] >= 0), key=lambda i: (int(ts[i]), i))
        lists = [(int(ts[i]), int(cn[i]), (lambda j, i=i: gdict.values[int(keys[i * K + j])]),
                  slots[i * K:i * K + int(cn[i])]) for i in order]
        return R.merge_dimension_lists(query, lists, tie_free)
    res = R.topn_merge_raw(query, cn, keys, vv, K, ts, handles=None)
    if res is None:
        return []
    t0, _lists, out_keys, slots = res
    values = [gdict.values[int(k)] for k in out_keys]
    return [Q.Result(t0, R._topn_entries(query, values, slots))]


def _to_bits(a, v) -> int:
    if a.output_type == "long":
        return int(v)
    if a.output_type == "double":
        return int(np.float64(v).view(np.int64))
    return int(np.float32(v).view(np.int32))


def _from_bits(a, b):
    if a.output_type == "long":
        return int(b)
    if a.output_type == "double":
        return float(np.int64(b).view(np.float64))
    return float(np.int32(b).view(np.float32))


# ----------------------------------------------------------------------------------------------
# groupBy
# ----------------------------------------------------------------------------------------------
def gather_groupby(dist, query: Q.GroupByQuery, partial: R.GroupByPartial,
                   gdicts: Dict[str, GlobalDictionary]):
    """all_gather this rank's (already device-merged) groups; rank 0 returns merged columns."""
    torch, _ = _torch()
    dev = _device(dist)
    nd, na = len(query.dimensions), len(query.aggregations)
    n = len(partial)
    cnt = torch.tensor([n], dtype=torch.int64, device=dev)
    world = dist.get_world_size()
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    mx = int(max(int(c.item()) for c in counts))
    width = 1 + nd + na
    mat = np.zeros((max(mx, 1), width), dtype=np.int64)
    if n:
        mat[:n, 0] = partial.times
        for d, dn in enumerate(query.dimensions):
            idx = gdicts[dn].index
            mat[:n, 1 + d] = np.fromiter((idx[v] for v in partial.dims[d]), dtype=np.int64, count=n)
        for a_i, a in enumerate(query.aggregations):
            col = partial.aggs[a_i]
            if a.output_type == "long":
                mat[:n, 1 + nd + a_i] = col.astype(np.int64)
            elif a.output_type == "double":
                mat[:n, 1 + nd + a_i] = col.astype(np.float64).view(np.int64)
            else:
                mat[:n, 1 + nd + a_i] = col.astype(np.float32).view(np.int32).astype(np.int64)
    t = torch.from_numpy(mat).to(dev)
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(bufs, t)
    if dist.get_rank() != 0:
        return None
    parts = []
    for c, b in zip(counts, bufs):
        k = int(c.item())
        arr = b.cpu().numpy()[:k]
        dims = [np.array(gdicts[dn].values, dtype=object)[arr[:, 1 + d]] if k else np.zeros(0, object)
                for d, dn in enumerate(query.dimensions)]
        aggs = []
        for a_i, a in enumerate(query.aggregations):
            col = arr[:, 1 + nd + a_i]
            if a.output_type == "long":
                aggs.append(col.astype(np.int64))
            elif a.output_type == "double":
                aggs.append(col.astype(np.int64).view(np.float64))
            else:
                aggs.append(col.astype(np.int32).view(np.float32))
        parts.append(R.GroupByPartial(arr[:, 0].astype(np.int64), dims, aggs))
    return R.merge_groupby_columnar(query, parts)
