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
* groupBy: every rank's merged groups (in HBM, dg_groupby_run) are re-keyed into one cluster-wide
  key space (dg_result_export), cut into key ranges at sampled splitters (dg_keys_partition), sent
  to the rank owning each range with one all_to_all (RCCL over xGMI) and merged there
  (dg_merge, GroupByMergingQueryRunnerV2.java:170-290 semantics): every rank ends with its key range
  of the final, ordered result, no rank holds the whole table (GroupByExchange).
"""
from __future__ import annotations

import ctypes
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
    # DG_DIST_BACKEND=gloo: the collectives on the host (rehearsal of the multi-rank path with several
    # ranks on one GPU, which RCCL refuses: "Duplicate GPU detected")
    backend = os.environ.get("DG_DIST_BACKEND", backend)
    if backend == "nccl":
        torch.cuda.set_device(device_index())
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return dist


def device_index() -> int:
    """This rank's GPU: LOCAL_RANK, or DG_BENCH_DEVICE when set (every rank on that one device: a
    rehearsal with DG_DIST_BACKEND=gloo on a one-GPU box)."""
    forced = os.environ.get("DG_BENCH_DEVICE")
    return int(forced) if forced not in (None, "") else int(os.environ.get("LOCAL_RANK", "0"))


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
        is_min = a.kind in (4, 6, 8)
        fp_minmax = a.kind in (6, 7, 8, 9)
        col = cols[a.name]
        # double/float min/max reduce on order-preserving int64 keys (Math.min/max: NaN wins, -0.0 < 0.0)
        t = torch.from_numpy(_ord_keys(col, is_min) if fp_minmax else col.copy()).to(dev)
        op = dist.ReduceOp.SUM if a.kind in (0, 1, 2, 3) else (dist.ReduceOp.MIN if is_min else dist.ReduceOp.MAX)
        dist.all_reduce(t, op=op)
        out = t.cpu().numpy()
        out_cols[a.name] = _from_ord_keys(out, is_min, col.dtype) if fp_minmax else out
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


_SIGN = np.uint64(1 << 63)


def _ord_keys(col: np.ndarray, is_min: bool) -> np.ndarray:
    """float64/float32 values -> int64 keys whose signed order is Java's Math.min/Math.max order:
    -0.0 < 0.0, and NaN is the extreme the operator picks (the smallest key for min, largest for max),
    so an integer MIN/MAX all_reduce reproduces DoubleMinAggregator.combine / DoubleMaxAggregator.combine."""
    d = col.astype(np.float64)
    u = d.view(np.uint64)
    k = np.where((u & _SIGN) != 0, ~u, u | _SIGN)
    s = (k ^ _SIGN).view(np.int64)
    nan = np.isnan(d)
    s = np.where(nan, np.iinfo(np.int64).min if is_min else np.iinfo(np.int64).max, s)
    return s.astype(np.int64)


def _from_ord_keys(s: np.ndarray, is_min: bool, dtype) -> np.ndarray:
    nan = s == (np.iinfo(np.int64).min if is_min else np.iinfo(np.int64).max)
    k = s.astype(np.int64).view(np.uint64) ^ _SIGN
    u = np.where((k & _SIGN) != 0, k & ~_SIGN, ~k)
    d = u.view(np.float64)
    d = np.where(nan, np.nan, d)
    return d.astype(dtype)


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


# ----------------------------------------------------------------------------------------------
# groupBy: key-range exchange + device merge
# ----------------------------------------------------------------------------------------------
class NativeMerge:
    """The device side of the exchange through the C-ABI (dg_result_export / dg_keys_partition /
    dg_merge) on one context; records travel as torch tensors on that device."""

    def __init__(self, context):
        self.context = context

    def export(self, res, ks, maps, rec):
        torch, _ = _torch()
        from . import _native as N
        n = res.groups
        dev = torch.device("cuda", self.context.device)
        keys = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        slots = torch.empty(max(n, 1) * rec, dtype=torch.int64, device=dev)
        arr = (ctypes.c_void_p * max(len(maps), 1))(*[m.ctypes.data for m in maps])
        torch.cuda.current_stream(dev).synchronize()  # allocations are ordered on torch's stream
        N.check(N.lib().dg_result_export(res.handle, ctypes.byref(ks.struct), arr, keys.data_ptr(), slots.data_ptr()))
        return keys[:n], slots[:n * rec]

    def partition(self, keys, splits):
        from . import _native as N
        pos = np.zeros(len(splits), dtype=np.int64)
        if len(splits):
            sp = np.ascontiguousarray(splits, dtype=np.uint64)
            N.check(N.lib().dg_keys_partition(self.context.handle, keys.data_ptr() if keys.numel() else None,
                                              keys.numel(), sp.ctypes.data, len(sp), pos.ctypes.data))
        return pos

    def sample(self, keys, idx):
        torch, _ = _torch()
        return keys[torch.from_numpy(idx).to(keys.device)].cpu().numpy()

    def merge(self, ks, keys, slots, query, dictionaries):
        torch, _ = _torch()
        from . import _native as N
        torch.cuda.current_stream(keys.device).synchronize()  # the received records have landed
        out = ctypes.c_void_p()
        m = N.dg_metrics()
        n = keys.numel()
        N.check(N.lib().dg_merge(self.context.handle, ctypes.byref(ks.struct), keys.data_ptr() if n else None,
                                 slots.data_ptr() if n else None, n, ctypes.byref(out), ctypes.byref(m)))
        return R.GroupByResult(out, query, dictionaries=dictionaries)


class KeySpace:
    """dg_keyspace of one groupBy query over the cluster (kept alive with its arrays)."""

    def __init__(self, cards, period_ms, bucket0, n_buckets, universal, agg_kinds):
        from . import _native as N
        self.cards = np.ascontiguousarray(cards, dtype=np.int32)
        self.kinds = np.ascontiguousarray(agg_kinds, dtype=np.int32)
        self.period_ms, self.bucket0, self.n_buckets, self.universal = period_ms, bucket0, n_buckets, universal
        st = N.dg_keyspace()
        st.n_dims = len(self.cards)
        st.card = self.cards.ctypes.data if len(self.cards) else None
        st.period_ms, st.bucket0, st.n_buckets, st.universal_time = period_ms, bucket0, n_buckets, universal
        st.n_aggs = len(self.kinds)
        st.agg_kinds = self.kinds.ctypes.data if len(self.kinds) else None
        self.struct = st
        # key = [bucket | d0 | d1 | ...], the last dimension least significant (dg_groupby_run's layout)
        self.dim_bits = [max(int(c) - 1, 0).bit_length() for c in self.cards]
        self.bucket_bits = max(n_buckets - 1, 0).bit_length() if period_ms else 0
        self.bits = sum(self.dim_bits) + self.bucket_bits


class GroupByExchange:
    """Cluster-wide merge of one groupBy query's per-rank results (built once per query shape:
    cluster dictionaries, id maps, bucket grid; then one `exchange` per run).

    Key-range partitioning: each rank samples its sorted keys, the samples (weighted by the rank's
    group count) give world - 1 splitters identical on every rank, dg_keys_partition cuts the
    rank's keys at them, one all_to_all moves every range to its owner, dg_merge combines equal
    keys (sources in rank order). Rank r ends with range r of the ordered result."""

    SAMPLES = 256

    def __init__(self, dist, query: Q.GroupByQuery, segments, engine=None):
        self.dist, self.query = dist, query
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.engine = engine if engine is not None else NativeMerge(segments[0].context)
        nd = len(query.dimensions)
        # this rank's merged dictionaries: the union of its segments' dictionaries (a segment without
        # the column contributes null), exactly as dg_groupby_run builds them
        local = []
        for d in query.dimensions:
            vals = set()
            for s in segments:
                vals.update(s.dictionary(d))
            local.append(sorted(vals, key=R._java_key))
        gran = query.granularity
        span = None
        # calendar granularity: the engines bucket on the query's bucket list (identical on every rank),
        # keys carry bucket indices into it (dg_keyspace period 1)
        self.starts = np.asarray(gran.bucket_starts(tuple(query.interval)), np.int64) if gran.is_calendar else None
        if self.starts is not None:
            coord = lambda t: int(np.searchsorted(self.starts, t, side="right")) - 1  # noqa: E731
            bend = lambda t: int(self.starts[coord(t) + 1]) if coord(t) + 1 < len(self.starts) else Q.MAX_INSTANT  # noqa: E731
            period = 1
        else:
            coord = lambda t: gran.bucket_start(t)  # noqa: E731
            bend = lambda t: gran.bucket_start(t) + gran.period_ms  # noqa: E731
            period = gran.period_ms
        if not gran.is_all:  # the grid of bucket indices every rank's result is re-keyed onto
            q0, q1 = query.interval
            for s in segments:
                if s.num_rows == 0:
                    continue
                data_e = bend(s.max_time)
                if not (q0 < data_e and s.min_time < q1):
                    continue
                lo = coord(max(q0, s.min_time))
                hi = coord(min(q1, data_e) - 1)
                span = (lo, hi) if span is None else (min(span[0], lo), max(span[1], hi))
        gathered: List = [None] * self.world
        dist.all_gather_object(gathered, {"dicts": local, "span": span})
        self.dicts = []
        for i in range(nd):
            allv = set()
            for g in gathered:
                allv.update(g["dicts"][i])
            self.dicts.append(sorted(allv, key=R._java_key))
        index = [{v: k for k, v in enumerate(gd)} for gd in self.dicts]
        self.local = local
        self.maps = [np.array([index[i][v] for v in local[i]], dtype=np.int32) for i in range(nd)]
        spans = [g["span"] for g in gathered if g["span"] is not None]
        if gran.is_all or not spans:
            bucket0, nb = 0, 1
        else:
            bucket0 = min(s[0] for s in spans)
            nb = (max(s[1] for s in spans) - bucket0) // period + 1
        self.ks = KeySpace([len(d) for d in self.dicts], 0 if gran.is_all else period, bucket0, nb, query.interval[0],
                           [a.kind for a in query.aggregations])
        if self.ks.bits > 63:
            raise R.N.UnsupportedQuery(2, f"cluster groupBy key of {self.ks.bits} bits")
        self.rec = 1 + len(query.aggregations)
        self._checked = False

    def _splitters(self, keys) -> np.ndarray:
        """world - 1 ascending splitters from every rank's evenly spaced key samples, each weighted by
        the share of its rank's groups it stands for (identical on every rank)."""
        torch, _ = _torch()
        n = keys.numel()
        S = self.SAMPLES
        k = min(S, n)
        idx = (np.arange(k, dtype=np.int64) * n) // max(k, 1)
        samp = np.full(S, -1, dtype=np.int64)
        if k:
            samp[:k] = self.engine.sample(keys, idx)
        payload = torch.from_numpy(np.concatenate([[n, k], samp]).astype(np.int64)).to(_device(self.dist))
        bufs = [torch.empty_like(payload) for _ in range(self.world)]
        self.dist.all_gather(bufs, payload)
        pts, wts = [], []
        for b in bufs:
            a = b.cpu().numpy()
            nn, kk = int(a[0]), int(a[1])
            if kk:
                pts.append(a[2:2 + kk])
                wts.append(np.full(kk, nn / kk))
        if not pts:
            return np.zeros(self.world - 1, dtype=np.uint64)
        pts = np.concatenate(pts)
        wts = np.concatenate(wts)
        order = np.argsort(pts, kind="stable")
        pts, cum = pts[order], np.cumsum(wts[order])
        total = cum[-1]
        out = []
        for r in range(1, self.world):
            j = int(np.searchsorted(cum, total * r / self.world, side="left"))
            out.append(int(pts[min(j, len(pts) - 1)]))
        return np.maximum.accumulate(np.array(out, dtype=np.int64)).astype(np.uint64)

    def exchange(self, res):
        """This rank's key range of the cluster-wide merged result (a device-resident result whose
        dimension ids index `self.dicts`)."""
        torch, _ = _torch()
        if not self._checked:  # the engine's merged dictionaries are the ones the maps were built for
            for d in range(len(self.query.dimensions)):
                if res.dictionary(d) != self.local[d]:
                    raise RuntimeError(f"merged dictionary of {self.query.dimensions[d]} differs from the segments'")
            self._checked = True
        keys, slots = self.engine.export(res, self.ks, self.maps, self.rec)
        n = keys.numel()
        splits = self._splitters(keys)
        pos = self.engine.partition(keys, splits)
        bounds = np.concatenate([[0], pos, [n]]).astype(np.int64)
        send = np.diff(bounds)
        dev = keys.device
        cdev = _device(self.dist)  # where the collective's tensors live (the GPU under RCCL)
        cnt_in = torch.from_numpy(send.astype(np.int64)).to(cdev)
        cnt_out = torch.empty_like(cnt_in)
        self.dist.all_to_all_single(cnt_out, cnt_in)
        recv = cnt_out.cpu().numpy().astype(np.int64)
        rkeys = torch.empty(int(recv.sum()), dtype=torch.int64, device=cdev)
        rslots = torch.empty(int(recv.sum()) * self.rec, dtype=torch.int64, device=cdev)
        self.dist.all_to_all_single(rkeys, keys.contiguous().to(cdev), [int(x) for x in recv], [int(x) for x in send])
        self.dist.all_to_all_single(rslots, slots.contiguous().to(cdev), [int(x) * self.rec for x in recv],
                                    [int(x) * self.rec for x in send])
        rkeys, rslots = rkeys.to(dev), rslots.to(dev)  # (no copies when the collective ran on the GPU)
        res = self.engine.merge(self.ks, rkeys, rslots, self.query, self.dicts)
        if self.starts is not None:
            res.time_map = self.starts  # dg_merge times are bucket indices into the query's bucket list
        # limit push-down: this rank's key range holds whole groups, and the ordering is on grouping
        # fields only, so the cluster's first `limit` groups are among the ranks' first `limit`
        if hasattr(res, "apply_limit_push_down"):  # (the CPU tests' host engine returns its rows whole)
            res.apply_limit_push_down()
        return res


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
