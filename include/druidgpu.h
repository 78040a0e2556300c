/*
 * druidgpu.h — C-ABI of the MI355X segment scan-and-aggregate engine.
 *
 * This is the drop-in boundary a JNI shim binds. Every entry point replaces
 * one reference interface on the historical's per-segment query path (paths relative to the
 * reference root; processing/... = processing/src/main/java/org/apache/druid/...):
 *
 *   dg_segment_attach        <- IndexIO.loadIndex / V9IndexLoader.load (processing/.../segment/IndexIO.java:569-663)
 *                               + Segment.asQueryableIndex/asStorageAdapter (processing/.../segment/Segment.java:30-35)
 *   dg_segment_release       <- QueryableIndex.close / ReferenceCountingSegment (SmooshedFileMapper.close)
 *   dg_segment_time_bounds   <- StorageAdapter.getMinTime / getMaxTime (processing/.../segment/StorageAdapter.java:33-80)
 *   dg_segment_dim_*         <- StorageAdapter.getDimensionCardinality, DimensionSelector.lookupName,
 *                               GenericIndexed.get (processing/.../segment/data/GenericIndexed.java:479-492)
 *   dg_filter_bitmap         <- Filter.getBitmapResult over BitmapIndexSelector
 *                               (processing/.../query/filter/Filter.java:28-110; segment/filter/{Selector,In,Bound,
 *                               And,Or,Not}Filter.java) as used by QueryableIndexStorageAdapter.makeCursors (:244-299)
 *   dg_timeseries_run        <- TimeseriesQueryRunnerFactory.createRunner(segment).run
 *                               (processing/.../query/timeseries/TimeseriesQueryRunnerFactory.java:93-105,
 *                               TimeseriesQueryEngine.java:40-111)
 *   dg_topn_run              <- TopNQueryRunnerFactory.createRunner(segment).run (query/topn/TopNQueryRunnerFactory.java:61-90,
 *                               TopNQueryEngine.java:60-160 -> PooledTopNAlgorithm + TopNNumericResultBuilder)
 *   dg_segment_set_dim_order <- StringComparator.compare over one dictionary (query/ordering/StringComparators.java),
 *                               the order DimensionTopNMetricSpec / TopNLexicographicResultBuilder ranks values by
 *   dg_topn_merge            <- TopNBinaryFn.apply fold of QueryRunnerFactory.mergeRunners (query/topn/TopNBinaryFn.java:75-135)
 *   dg_groupby_run           <- GroupByStrategyV2.process -> GroupByQueryEngineV2.process per segment
 *                               (query/groupby/strategy/GroupByStrategyV2.java:472-477, epinephelinae/GroupByQueryEngineV2.java:91-187)
 *                               + GroupByStrategyV2.mergeRunners -> GroupByMergingQueryRunnerV2.run (:170-290)
 *   dg_result_*              <- the merged grouper's sorted iterator (ConcurrentGrouper.iterator(true))
 *   dg_result_export / dg_keys_partition / dg_merge
 *                            <- QueryRunnerFactory.mergeRunners across devices (query/QueryRunnerFactory.java:62):
 *                               GroupByMergingQueryRunnerV2 semantics over the devices' merged groups
 *   dg_groupby_merge_devices <- the same within one process: the library moves key ranges between devices itself
 *   dg_timeseries_merge      <- TimeseriesBinaryFn fold of runners' results (query/timeseries/TimeseriesBinaryFn.java:67-70)
 *   dg_records_pack          <- BufferAggregator.get* record layout (query/aggregation/BufferAggregator.java:35-199)
 *
 * Segment arrays: every *_run takes n_segs segments that are attached to the SAME context (device)
 * and runs them as one batched launch sequence; results stay per segment, exactly as the
 * reference's per-segment runners return them (cross-segment merging is QueryRunnerFactory.mergeRunners,
 * done by the host layer / RCCL, see incubator-druid_amd/runners.py and distributed.py).
 *
 * Conventions: 0 = DG_OK, otherwise a DG_ERR_* code and dg_last_error() (thread-local) describes it.
 * All output buffers are caller-allocated host memory. No callbacks into the caller. Every entry
 * point is safe to call concurrently for different segments; calls on one context serialize on
 * that context's HIP stream. Only the reference's default null mode is implemented
 * (druid.generic.useDefaultValueForNull=true, common/config/NullHandling.java:34,54): anything else
 * is the caller's problem (the Java shim keeps its CPU path, DG_ERR_UNSUPPORTED).
 */
#ifndef DRUIDGPU_H
#define DRUIDGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DG_ABI_VERSION 16

/* status codes (the JNI shim maps them to the reference's exceptions) */
#define DG_OK 0
#define DG_ERR_FORMAT 1      /* IAE / ISE on malformed segment bytes (GenericIndexed.java:131-149) */
#define DG_ERR_UNSUPPORTED 2 /* shape not implemented on GPU: caller keeps its CPU engine */
#define DG_ERR_OOM 3         /* device allocation failed */
#define DG_ERR_INTERRUPTED 4 /* QueryInterruptedException (BaseQuery.checkInterrupted, BaseQuery.java:46-51) */
#define DG_ERR_TABLE_FULL 5  /* Groupers.HASH_TABLE_FULL (Groupers.java:36-40) */
#define DG_ERR_ARG 6         /* IllegalArgumentException */
#define DG_ERR_DEVICE 7      /* HIP runtime failure */
#define DG_ERR_NOT_FOUND 8   /* SegmentMissingException (TimeseriesQueryEngine.java:42-46) */
#define DG_ERR_TIMEOUT 9     /* QueryInterruptedException(TimeoutException): "Query timeout" (ChainedExecutionQueryRunner.java:164-167,
                                QueryInterruptedException.java:46) */

/* column types (ValueType, processing/.../segment/column/ValueType.java) */
#define DG_COL_MISSING 0
#define DG_COL_LONG 1
#define DG_COL_FLOAT 2
#define DG_COL_DOUBLE 3
#define DG_COL_STRING 4      /* single- or multi-value (V3, legacy compressed or uncompressed multi-value:
                                filters, topN per value and groupBy explode all run on it) */
#define DG_COL_UNSUPPORTED 5 /* complex column / unsupported codec */

/* aggregator kinds (query/aggregation/...AggregatorFactory.java) */
#define DG_AGG_COUNT 0
#define DG_AGG_LONG_SUM 1
#define DG_AGG_DOUBLE_SUM 2
#define DG_AGG_FLOAT_SUM 3
#define DG_AGG_LONG_MIN 4
#define DG_AGG_LONG_MAX 5
#define DG_AGG_DOUBLE_MIN 6
#define DG_AGG_DOUBLE_MAX 7
#define DG_AGG_FLOAT_MIN 8
#define DG_AGG_FLOAT_MAX 9

/* filter node kinds (query/filter/...DimFilter.java -> segment/filter/...Filter.java) */
#define DG_F_AND 1
#define DG_F_OR 2
#define DG_F_NOT 3
#define DG_F_SELECTOR 4
#define DG_F_IN 5
#define DG_F_BOUND 6

/* string orderings (query/ordering/StringComparators.java): bound filters use LEXICOGRAPHIC / NUMERIC,
 * dimension-ordered topN all four */
#define DG_ORDER_LEXICOGRAPHIC 0
#define DG_ORDER_NUMERIC 1
#define DG_ORDER_ALPHANUMERIC 2
#define DG_ORDER_STRLEN 3

typedef struct dg_context dg_context;
typedef struct dg_segment dg_segment;
typedef struct dg_result dg_result;

/*
 * One filter node. A filter is an array of nodes in prefix order: an AND/OR node is followed by
 * its n_children subtrees, a NOT node by exactly one subtree. Strings are NUL-terminated UTF-8;
 * a NULL value pointer means the null value ("" in default null mode). A leaf on a string column
 * runs on its bitmap index; a leaf on a long / float / double column (no bitmap index) is the
 * reference's row post-filter (QueryableIndexStorageAdapter.java:244-260, FilteredOffset.java:40-105)
 * with its ValueMatcher semantics: selector / in values parsed as getExactLongFromDecimalString or
 * Floats/Doubles.tryParse, NUMERIC bounds as BoundDimFilter's long / float / double predicates,
 * LEXICOGRAPHIC bounds on long columns over String.valueOf(value); other orderings on numeric
 * columns -> DG_ERR_UNSUPPORTED.
 */
typedef struct {
  int32_t kind;
  int32_t n_children;
  const char* dimension;
  const char* const* values; /* SELECTOR: values[0]; IN: values[0..n_values) */
  int32_t n_values;
  const char* lower;         /* BOUND: NULL = no bound */
  const char* upper;
  int32_t lower_strict;
  int32_t upper_strict;
  int32_t ordering;          /* DG_ORDER_* */
} dg_filter;

/* AggregatorFactory (name is the caller's business; field is the input column, NULL for count).
 * filter / n_filter: FilteredAggregatorFactory (query/aggregation/FilteredAggregatorFactory.java:56-73,
 * FilteredBufferAggregator.java:45-50): the aggregator takes a cursor row only when the filter
 * (same node encoding as dg_scan.filter) matches it; NULL / 0 = unfiltered. */
typedef struct {
  int32_t kind;
  const char* field;
  const dg_filter* filter;
  int32_t n_filter;
} dg_agg;

/*
 * The scan common to all three query types (what makeCursors receives:
 * CursorFactory.makeCursors(filter, interval, virtualColumns, gran, descending, metrics),
 * processing/.../segment/CursorFactory.java:32-42).
 * Granularity: period_ms == 0 is ALL; otherwise a fixed-length UTC period with bucket starts at
 * origin_ms + k * period_ms (PeriodGranularity.truncateMillisPeriod, PeriodGranularity.java:411-428).
 * Calendar granularities (months, years, periods in a time zone, compound periods: PeriodGranularity
 * with Joda chronology arithmetic, PeriodGranularity.java:212-410) are given as the bucket list
 * gran.getIterable(interval) yields (Granularity.java:176-240): bucket_starts[0..n_bucket_starts)
 * = the starts followed by the end of the last bucket (strictly ascending, the last end at or past the
 * interval end; the first start may lie after the interval start, rows before it are in no bucket),
 * period_ms = 0; bucket k = [bucket_starts[k], bucket_starts[k + 1]). The Java shim computes it
 * with the query's own Granularity object. In dg_keyspace / dg_merge such a granularity is the
 * grid period_ms = 1 over bucket indices into that list.
 * seg_bounds (calendar only, optional): per segment of the call two instants, {gran.bucketStart(s),
 * gran.bucketEnd(maxTime)} with s = max(interval start, minTime): where the segment's iterable starts
 * and where its dataInterval ends (QueryableIndexStorageAdapter.java:367-372). Both truncate from
 * the origin, so they can leave the listed buckets: bucketEnd past the end of the listed bucket that
 * holds maxTime (an origin whose day clamps: P1M from Jan 31), bucketStart after s (the hours branch
 * before its origin, PeriodGranularity.java:313-326: rows in [s, bucketStart(s)) are in no cursor).
 * NULL = the listed bucket ends and no clipping at the start.
 * descending: CursorFactory.makeCursors(..., descending) (QueryableIndexStorageAdapter.java:378-424):
 * cursors in descending time order and each cursor's rows last to first (order-dependent floatSum);
 * timeseries / topN write their per-segment buckets in that order. groupBy ignores it (its engine
 * always asks for ascending cursors, GroupByQueryEngineV2.java:108-115).
 */
typedef struct {
  int64_t interval_start; /* [start, end) epoch millis */
  int64_t interval_end;
  int64_t period_ms;
  int64_t origin_ms;
  const dg_filter* filter; /* NULL / n_filter == 0: no filter */
  int32_t n_filter;
  const dg_agg* aggs;
  int32_t n_aggs;
  /* optional cancellation flag (Thread.interrupt / QueryWatcher cancel, BaseQuery.checkInterrupted,
     BaseQuery.java:46-51): polled between every launch group and while the call waits for the device;
     non-zero => DG_ERR_INTERRUPTED. Work already queued on the device finishes before the call
     returns, so the context is ready for its next call. */
  const volatile int32_t* cancel;
  const int64_t* bucket_starts;   /* calendar granularity (see above); NULL = period_ms grid */
  int32_t n_bucket_starts;
  int32_t descending;
  const int64_t* seg_bounds;      /* calendar granularity: 2 per segment (see above), or NULL */
  /* since ABI 14: the query context's "timeout" in ms (QueryContexts.getTimeout, ChainedExecutionQueryRunner
     futures.get(timeout), ChainedExecutionQueryRunner.java:150-167), measured from the call's start and
     checked where `cancel` is; <= 0: none. Past it => DG_ERR_TIMEOUT. */
  int64_t timeout_ms;
} dg_scan;

/* QueryMetrics counters (query/QueryMetrics.java:295-306) + device timings */
typedef struct {
  int64_t segment_rows;      /* reportSegmentRows */
  int64_t pre_filtered_rows; /* reportPreFilteredRows: rows passing the bitmap filter */
  int64_t selected_rows;     /* rows aggregated (filter AND interval) */
  int64_t bytes_read;        /* algorithmic HBM bytes of the column blocks / bitmaps scanned */
  double bitmap_ms;          /* reportBitmapConstructionTime (device time) */
  double decode_ms;          /* column decode kernels */
  double aggregate_ms;       /* aggregation kernels (all of them, groupBy: keygen + sort + reduce) */
  double total_ms;           /* whole call, host wall */
  /* groupBy phases (device time) and their element counts */
  double keygen_ms;          /* selected rows -> (key, row ref) */
  double sort_ms;            /* radix passes */
  double reduce_ms;          /* run heads + segmented reduce + floatSum pass + finalize */
  int32_t sort_passes;
  int32_t key_bits;
  int64_t groups;            /* merged groups */
  /* groupBy: payload columns decoded in place on the side stream, overlapping the key build + sort */
  double decode_side_ms;     /* device time of those decodes (their own stream) */
  int64_t bytes_side;        /* their algorithmic bytes (part of bytes_read) */
  /* the general LZ4 decoder (token-dense blocks: 8-byte value runs, noisy doubles), both streams: device
     time of its launches, the stored bytes and number of the blocks it decoded, and its launches */
  double lz4_general_ms;
  int64_t lz4_general_bytes;
  int32_t lz4_general_blocks;
  int32_t lz4_general_launches;
  /* filter bitmaps: serialized bitmap bytes read + row bitsets written and read (since ABI 11) */
  int64_t bitmap_bytes;
  /* since ABI 12: the groupBy reduce kernels alone (reduce_ms also holds the wait for the side-stream
     payload decode) */
  double reduce_kernel_ms;
  /* since ABI 13: timeseries LZ4 blocks whose decode was fused with their aggregator (the decoder
     folded the block's values into its bucket's slot and wrote no decoded image) */
  int64_t lz4_fused_blocks;
  /* the wall time the general decoder ran on either stream (the union of its main- and side-stream
     spans; lz4_general_ms is their sum) */
  double lz4_general_wall_ms;
  /* since ABI 16: of the general decoder's blocks, those decoded by its flow kernel (k_lz4_decode_flow)
     and their stored bytes; the rest went to k_lz4_decode */
  int64_t lz4_flow_blocks;
  int64_t lz4_flow_bytes;
} dg_metrics;

/* Aggregate values are returned in 8-byte slots: int64 for count/long*, double for double*,
 * and for float* a float32 in the first 4 bytes of the slot (rest zero). */

/* ---- library / context ---- */
const char* dg_last_error(void);
int dg_abi_version(void);
int dg_device_count(int* out);
int dg_context_create(int device, dg_context** out);
void dg_context_release(dg_context* ctx);
/* Bind the context's work to an existing HIP stream (e.g. torch's current stream); NULL resets. */
int dg_context_set_stream(dg_context* ctx, void* hip_stream);
/* Resource limits of the context's calls (the processing-buffer budget a historical configures,
 * DruidProcessingConfig / GroupByQueryConfig; exceeding one is answered DG_ERR_UNSUPPORTED before any
 * buffer is sized, so the Java factory keeps its CPU engine). value <= 0 restores the default.
 *   DG_LIMIT_GROUP_ELEMENTS: sort elements of one groupBy call (rows, or for multi-value dimensions
 *   rows x the product of their value-list lengths, GroupByQueryEngineV2.java:480-540); never more
 *   than 2^32 - 64 (element indices are 32-bit). */
#define DG_LIMIT_GROUP_ELEMENTS 1
int dg_context_set_limit(dg_context* ctx, int32_t which, int64_t value);

/* ---- segments ---- */
int dg_segment_attach(dg_context* ctx, const char* segment_dir, dg_segment** out);
void dg_segment_release(dg_segment* seg);
/* In-memory (realtime) segment: the rows of an IncrementalIndex queried like a persisted segment
 * (IncrementalIndexStorageAdapter, processing/.../segment/incremental/IncrementalIndexStorageAdapter.java:
 * the index's facts in its iteration order, TimeAndDims order: time ascending). Rows are copied into
 * HBM as flat columns (__time from `timestamps`); a string dimension comes as the index's
 * DimensionDictionary (values by id in insertion order, NULL or "" = null) plus one id per row and is
 * re-sorted into the sorted-dictionary form (SortedDimensionDictionary) the engines use. Such a
 * segment has no bitmap index: string filters run as row predicates on the ids (the adapter's
 * ValueMatchers; a multi-value row matches when one of its values does, an empty row as null).
 * Multi-value dimension: offsets[n_rows + 1] into ids (StringDimensionIndexer's encoded rows, values
 * in the row's order; an empty row = no values). Released with dg_segment_release. */
typedef struct {
  const char* name;
  int32_t type;            /* DG_COL_LONG / DG_COL_FLOAT / DG_COL_DOUBLE / DG_COL_STRING */
  int32_t card;            /* STRING: dictionary size */
  const char* const* dict; /* STRING: value of every id */
  const int32_t* ids;      /* STRING: [n_rows] ids into dict (multi-value: [offsets[n_rows]]) */
  const void* values;      /* numeric: [n_rows] int64 / float / double */
  const int32_t* offsets;  /* STRING multi-value: [n_rows + 1] row starts into ids; NULL = one id per row */
} dg_row_column;
int dg_segment_from_rows(dg_context* ctx, int64_t n_rows, const int64_t* timestamps, int64_t interval_start,
                         int64_t interval_end, const dg_row_column* columns, int32_t n_columns, dg_segment** out);
int64_t dg_segment_num_rows(const dg_segment* seg);
int dg_segment_interval(const dg_segment* seg, int64_t* start, int64_t* end);
int dg_segment_time_bounds(const dg_segment* seg, int64_t* min_time, int64_t* max_time);
int dg_segment_num_columns(const dg_segment* seg);
const char* dg_segment_column_name(const dg_segment* seg, int index);
int dg_segment_column_type(const dg_segment* seg, const char* column);
int64_t dg_segment_device_bytes(const dg_segment* seg);
int32_t dg_segment_dim_cardinality(const dg_segment* seg, const char* dim);
/* lookupName: *len = -1 for null (empty) values */
int dg_segment_dim_value(const dg_segment* seg, const char* dim, int32_t id, const char** out, int32_t* len);
/* Bulk dictionary export: offsets[card + 1] (byte offsets into bytes), bytes (size offsets[card]).
 * Call with bytes == NULL to get *total_bytes first. */
int dg_segment_dim_dictionary(const dg_segment* seg, const char* dim, int64_t* offsets, char* bytes,
                              int64_t* total_bytes);
/* Hand the engine one dictionary order (kept in HBM with the segment, set once per segment):
 * slot = 2 * DG_ORDER_* + inverted (InvertedTopNMetricSpec over DimensionTopNMetricSpec);
 * rank[id] for every dictionary id (card of them): position of the value under the comparator,
 * comparator-equal values share a rank (has_ties != 0 then). The ordering is the caller's
 * StringComparator (the JNI shim sorts the dictionary with the Java comparator itself). */
int dg_segment_set_dim_order(dg_segment* seg, const char* dim, int32_t slot, const int32_t* rank, int32_t card,
                             int32_t has_ties);

/* ---- scan pieces ---- */
/* Filter.getBitmapResult: row bitset (uint32 words, bit r = row r) of the filter, into out_words
 * (ceil(num_rows / 32) words); *out_count = cardinality of the result. */
int dg_filter_bitmap(dg_segment* seg, const dg_filter* filter, int32_t n_filter, uint32_t* out_words,
                     int64_t* out_count);

/* ---- timeseries ---- */
/* Per segment i: out_n_buckets[i] cursors (one per granularity bucket of the segment's actual
 * interval, TimeseriesQueryEngine emits each even when empty); bucket k of segment i is at
 * index i * bucket_cap + k of out_bucket_time / out_bucket_rows, and its aggregate slots at
 * (i * bucket_cap + k) * n_aggs. out_bucket_rows = rows aggregated (skipEmptyBuckets decision). */
int dg_timeseries_run(dg_segment* const* segs, int32_t n_segs, const dg_scan* scan, int32_t bucket_cap,
                      int32_t* out_n_buckets, int64_t* out_bucket_time, int64_t* out_bucket_rows,
                      uint64_t* out_values, dg_metrics* metrics);

/* ---- topN ---- */
typedef struct {
  const char* dimension;
  int32_t metric_agg; /* index into scan->aggs of the NumericTopNMetricSpec metric */
  int32_t inverted;   /* InvertedTopNMetricSpec */
  int32_t threshold;  /* per-segment threshold, i.e. max(query threshold, minTopNThreshold) */
  /* DimensionTopNMetricSpec / LexicographicTopNMetricSpec / AlphaNumericTopNMetricSpec
   * (query/topn/DimensionTopNMetricSpec.java): dim_order = order slot set with
   * dg_segment_set_dim_order (metric_agg / inverted ignored), -1 = metric ordering. */
  int32_t dim_order;
  const char* previous_stop;  /* NULL = none; LEXICOGRAPHIC skips to it (computeStartEnd) */
  const int32_t* min_rank;    /* per segment: values need rank >= min_rank[i], i.e. after previousStop
                                 under the comparator (NULL = no previousStop) */
  /* non-ALL granularity (scan->period_ms != 0): one result list per cursor (granularity bucket) */
  int32_t bucket_cap;         /* list slots per segment (>= its bucket count) */
  int64_t* out_bucket_time;   /* [n_segs * bucket_cap] bucket start of every list */
} dg_topn;

/* Per segment i and cursor b (b = 0 for ALL granularity, where bucket_cap counts as 1): list
 * L = i * bucket_cap + b holds out_n[L] entries (-1: no cursor), ordered as
 * TopNNumericResultBuilder.build() (or, for a dimension order, TopNLexicographicResultBuilder.build())
 * returns them; entry j at index L * threshold + j: dictionary id (segment-local) and n_aggs slots. */
int dg_topn_run(dg_segment* const* segs, int32_t n_segs, const dg_scan* scan, const dg_topn* topn,
                int32_t* out_n, int32_t* out_ids, uint64_t* out_values, dg_metrics* metrics);

/* TopNBinaryFn fold (query/topn/TopNBinaryFn.java:75-135) of per-segment topN lists, as
 * TopNQueryQueryToolChest.mergeResults applies it over the per-segment runners' results
 * (QueryRunnerFactory.mergeRunners): lists in merge order (result timestamp, then segment index),
 * pairwise: union by dimension value with AggregatorFactory.combine, then TopNNumericResultBuilder with
 * the query threshold; the final list is truncated to the query threshold. ALL granularity.
 *   keys: segment mode (segs != NULL, one per list): segment-local dictionary ids, values compared by
 *         string through segs[i]'s dictionary; global mode (segs == NULL): ids of one cluster-wide
 *         dictionary whose order is Java String order, nulls first.
 * Output: out_n entries (<= topn->threshold), entry j taken from list out_list[j] with key out_keys[j]
 * and n_aggs slots in dg_topn_run's encoding. topn->threshold here is the QUERY threshold. */
typedef struct {
  int32_t n_lists;
  const int32_t* list_n;   /* entries of list i; <= 0: empty (no cursor) */
  int32_t stride;          /* entry j of list i is at index i * stride + j */
  const int64_t* keys;
  const uint64_t* values;  /* n_aggs slots per entry */
} dg_topn_lists;

int dg_topn_merge(dg_segment* const* segs, const dg_scan* scan, const dg_topn* topn, const dg_topn_lists* in,
                  int32_t* out_n, int32_t* out_list, int64_t* out_keys, uint64_t* out_values);

/* ---- groupBy (v2) ---- */
/* GroupByStrategyV2.mergeRunners over the call's segments: every segment's rows grouped
 * (GroupByQueryEngineV2.process, epinephelinae/GroupByQueryEngineV2.java:91-187) and merged by
 * (bucket, dimension values) like GroupByMergingQueryRunnerV2 (:170-290), in that order. A call
 * with one segment is that segment's runner (createRunner(segment).run). The groups stay in HBM in
 * the dg_result until fetched (page by page for large results). */
typedef struct {
  const char* const* dimensions;
  int32_t n_dims;
} dg_groupby;

int dg_groupby_run(dg_segment* const* segs, int32_t n_segs, const dg_scan* scan, const dg_groupby* g,
                   dg_result** out, dg_metrics* metrics);
/* ---- groupBy limit push-down ----
 * GroupByQuery.isApplyLimitPushDown (query/groupby/GroupByQuery.java:377-416: a limited DefaultLimitSpec
 * whose ORDER BY columns are all grouping dimensions, no having spec, no subtotals) orders rows by
 * getRowOrderingForPushDown (:423-528): the bucket time first (last with the sortByDimsFirst context
 * flag on a non-ALL granularity), then the ORDER BY dimensions in their order, each under its
 * StringComparator and direction (compareDimsForLimitPushDown :600-633), then the other dimensions
 * ascending; the grouper keeps the first `limit` rows (LimitedBufferHashGrouper.java). dg_result_limit
 * applies that to a dg_groupby_run / dg_merge result on the device: afterwards the result holds
 * min(limit, groups) groups in that order (comparator-equal groups keep the result's natural order),
 * fetched as before; dg_result_export refuses a limited result. */
typedef struct {
  int32_t dim;         /* index into dg_groupby.dimensions */
  int32_t descending;  /* OrderByColumnSpec.Direction.DESCENDING */
  const int32_t* rank; /* rank of every id of the result's dictionary of `dim` under the column's
                          StringComparator (0 <= rank < cardinality, nulls first, comparator-equal
                          values share a rank); NULL = LEXICOGRAPHIC, the id order itself */
} dg_order_column;

typedef struct {
  const dg_order_column* columns;
  int32_t n_columns;
  int32_t limit;              /* > 0 */
  int32_t sort_by_dims_first; /* query context sortByDimsFirst */
} dg_limit;

int dg_result_limit(dg_result* res, const dg_limit* spec);
/* number of merged groups */
int64_t dg_result_groups(const dg_result* res);
/* groups [start, start + count), in result order (bucket time, then dimension values in Java
 * String order, nulls first): bucket_time[count] (ALL granularity: the universal timestamp = the
 * query interval's start, GroupByStrategyV2.getUniversalTimestamp :125-138), ids[count * n_dims]
 * = indices into the result's merged dictionary of each dimension, values[count * n_aggs] in the
 * slot encoding of dg_timeseries_run. Any output pointer may be NULL (under ALL granularity the
 * caller knows every bucket time and passes NULL). Destinations in pinned host memory (dg_host_alloc,
 * or memory the caller registered with HIP) receive the columns by DMA straight from the device;
 * others through the library's pinned staging. */
int dg_result_fetch_groups(dg_result* res, int64_t start, int64_t count, int64_t* bucket_time, int32_t* ids,
                           uint64_t* values);
/* Pinned host memory for result delivery (since ABI 14): the shim allocates its result buffers once
 * and wraps them as direct ByteBuffers (JNI NewDirectByteBuffer), the way the processing pool's
 * buffers are allocated once at startup (OffheapBufferGenerator.java:53 allocateDirect). */
int dg_host_alloc(int64_t bytes, void** out);
void dg_host_free(void* p);
/* Phase timing (since ABI 15, process-wide, on by default): the dg_metrics *_ms phase times come from
 * GPU timestamps the calls record between their launch groups. A small query pays ~25 us for them
 * (configs[0]), so a caller timing queries end to end turns them off and samples phases in separate
 * calls (the phase fields then read 0). No reference counterpart: the reference's per-query metrics
 * (QueryMetrics reportSegmentTime etc.) are host wall times. */
int dg_set_phase_timing(int32_t on);
/* rows aggregated into each group of [start, start + count) */
int dg_result_fetch_rows(dg_result* res, int64_t start, int64_t count, int64_t* rows);
/* merged dictionary of dimension `dim` (the union of the segments' dictionaries, Java String
 * order, null first when present): cardinality, and a bulk export like dg_segment_dim_dictionary
 * (a null value has length 0) */
int32_t dg_result_dim_cardinality(const dg_result* res, int32_t dim);
int dg_result_dim_dictionary(const dg_result* res, int32_t dim, int64_t* offsets, char* bytes, int64_t* total_bytes);
void dg_result_release(dg_result* res);

/* ---- cross-device groupBy merge (QueryRunnerFactory.mergeRunners over devices, processing/.../query/
 * QueryRunnerFactory.java:62; GroupByMergingQueryRunnerV2.java:170-290 semantics) ----
 * Every device runs dg_groupby_run over its segments; the devices' groups are then re-keyed into one
 * cluster-wide key space (dg_result_export), cut into key ranges (dg_keys_partition), exchanged
 * (RCCL all-to-all over xGMI — the transport is the caller's: torch.distributed in
 * incubator-druid_amd/distributed.py, or the JNI shim's own communicator) and merged on the receiving
 * device (dg_merge), which combines equal keys with the combining aggregators in partial order. */
typedef struct {
  int32_t n_dims;
  const int32_t* card;      /* [n_dims] cardinality of the cluster-wide dictionary of each dimension
                               (the union of every device's merged dictionary, Java String order,
                               nulls first) */
  int64_t period_ms;        /* 0 = ALL granularity */
  int64_t bucket0;          /* non-ALL: epoch ms of bucket index 0 (on the query's period grid) */
  int64_t n_buckets;        /* non-ALL: bucket indices [0, n_buckets) */
  int64_t universal_time;   /* ALL: the result timestamp (GroupByStrategyV2.getUniversalTimestamp) */
  int32_t n_aggs;
  const int32_t* agg_kinds; /* [n_aggs] DG_AGG_* (combine semantics of each aggregator) */
} dg_keyspace;

/* total bits of a key of the key space; DG_ERR_UNSUPPORTED above 64 */
int dg_keyspace_bits(const dg_keyspace* ks, int32_t* bits);
/* Re-key res into the key space: maps[d][merged id of res] = cluster-wide id, strictly increasing
 * (so the ascending order is kept). Writes dg_result_groups(res) records into caller-allocated
 * DEVICE buffers of res's device: d_keys[n], d_slots[n * (1 + n_aggs)] (rows aggregated, then the
 * values in the slot encoding of dg_timeseries_run). Completes before returning. */
int dg_result_export(dg_result* res, const dg_keyspace* ks, const int32_t* const* maps, uint64_t* d_keys,
                     uint64_t* d_slots);
/* Key ranges of ascending device keys d_keys[n]: out_pos[i] = first index with key >= splits[i]
 * (splits ascending, host array), i.e. range i = [out_pos[i - 1], out_pos[i]). */
int dg_keys_partition(dg_context* ctx, const uint64_t* d_keys, int64_t n, const uint64_t* splits, int32_t n_splits,
                      int64_t* out_pos);
/* Merge n records (device buffers of ctx's device: keys, slots as written by dg_result_export),
 * the concatenation of partials that are each ascending, into a dg_result in the key space. Equal
 * keys combine in input order. The result's dimension ids are cluster-wide ids: its
 * dg_result_dim_cardinality is ks->card[d], and the dictionary is the caller's. */
int dg_merge(dg_context* ctx, const dg_keyspace* ks, const uint64_t* d_keys, const uint64_t* d_slots, int64_t n,
             dg_result** out, dg_metrics* metrics);

/* ---- in-process cross-device merge (QueryRunnerFactory.mergeRunners over the devices of ONE process,
 * query/QueryRunnerFactory.java:62: a historical is one JVM whose processing pool drives every
 * segment, ChainedExecutionQueryRunner.java:89-180; GroupByMergingQueryRunnerV2.java:170-290
 * semantics) ----
 * parts: n_parts dg_groupby_run results of one query, each on its own context (device), in merge
 * order. The library builds the union of their merged dictionaries, re-keys every part into that key
 * space on its own device (as dg_result_export), cuts the keys into n_targets ranges at splitters
 * sampled from all parts (dg_keys_partition), moves every range to its target's device with peer
 * copies over xGMI (hipMemcpyPeerAsync; a device copy when part and target share a device) and
 * merges it there (dg_merge: equal keys combine in part order with the combining aggregators).
 * outs[t] = key range t of the merged result, resident on targets[t]; concatenated in t order they
 * are the whole merged, ordered result. The outputs fetch like dg_groupby_run results: their
 * dg_result_dim_dictionary is the union dictionary. n_targets == 1: the whole merge on one device.
 * Parts stay valid (the caller releases them). No transport from the caller is needed. */
int dg_groupby_merge_devices(dg_result* const* parts, int32_t n_parts, dg_context* const* targets, int32_t n_targets,
                             dg_result** outs, dg_metrics* metrics);

/* TimeseriesBinaryFn fold (query/timeseries/TimeseriesBinaryFn.java:67-70) as the toolchest's
 * mergeResults applies it over runners' results (ResultMergeQueryRunner: by time, then runner
 * order): n_lists lists in dg_timeseries_run's output layout (list i holds n[i] buckets: times[i * cap
 * + k], rows[...], values[(i * cap + k) * n_aggs ...]) — the segments of one call, or the lists of
 * several devices' calls concatenated. Results of one granularity bucket combine with
 * AggregatorFactory.combine (long wrap, float adds in float, Math.min/max with NaN and -0.0); ALL
 * granularity keeps the earliest result's timestamp. skip_empty: skipEmptyBuckets drops buckets with
 * zero rows before merging. Output: out_n merged buckets, ascending (descending when scan->descending),
 * out_rows = rows aggregated per bucket. Host memory only. */
int dg_timeseries_merge(const dg_scan* scan, int32_t n_lists, const int32_t* n, int32_t cap, const int64_t* times,
                        const int64_t* rows, const uint64_t* values, int32_t skip_empty, int32_t out_cap, int32_t* out_n,
                        int64_t* out_time, int64_t* out_rows, uint64_t* out_values);

/* ---- BufferAggregator record layout (query/aggregation/BufferAggregator.java:35-199) ----
 * Writes n records of aggregate slots (n_aggs per record, the dg_*_run slot encoding) into Druid's
 * buffer layout so a JNI shim can fill a processing-pool direct ByteBuffer in place
 * (GetDirectBufferAddress): aggregator a at byte offsets[a] of each record_size-byte record, the
 * value as its BufferAggregator stores it — count / long* as an 8-byte long (LongSumBufferAggregator
 * buf.putLong), double* as an 8-byte double, float* as a 4-byte float (FloatSumBufferAggregator
 * buf.putFloat) — big-endian (java.nio.ByteBuffer's default order, big_endian != 0) or little-endian.
 * Host memory only; no device work. */
typedef struct {
  int32_t n_aggs;
  const int32_t* kinds;   /* DG_AGG_* */
  const int32_t* offsets; /* byte offset of each aggregator inside a record */
  int32_t record_size;
  int32_t big_endian;
} dg_record_layout;

int dg_records_pack(const uint64_t* slots, int64_t n, const dg_record_layout* layout, void* out);

/* ---- diagnostics (test harness; no reference counterpart) ----
 * Decode n raw LZ4 blocks (host buffers, <= 64 KiB decoded each) through the same attach-time
 * checkpoint index and HIP decoder the segment path uses. out: n * 65536 bytes, block i at
 * i * 65536; out_lens[i] = decoded length, or -1 when the block fails validation (not decoded).
 * *ms = device time of the decode kernel; prof (optional, NULL = off): 12 words per decoded block,
 * s_memtime stamps of the decoder's phases + counters (tools/lz4_profile.py prints them). */
int dg_debug_lz4_decode(dg_context* ctx, const uint8_t* const* blocks, const int32_t* lens, int32_t n, uint8_t* out,
                        int32_t* out_lens, double* ms, uint64_t* prof);

/* Which HIP decoder the attach-time classification routes one raw LZ4 block to (host only, no
 * device work): *kind = -1 malformed (fails validation), 0 general (k_lz4_decode), 1 general with
 * wide checkpoints, 2 light (k_lz4_light). Since ABI 11. */
int dg_debug_lz4_classify(const uint8_t* block, int32_t len, int32_t* kind);

/* Measurement probes (since ABI 16): what the device and its host link deliver to plain kernels and
 * copies, timed with HIP events over `iters` repetitions after one warm-up; *ms = average per
 * repetition. Buffers are allocated and freed inside the call.
 *   DG_PROBE_COPY      n bytes read and n bytes written by a grid-stride 16-byte copy kernel (HBM)
 *   DG_PROBE_D2H       n bytes device -> pinned host memory (hipMemcpyAsync, DMA)
 *   DG_PROBE_H2D       n bytes pinned host memory -> device
 *   DG_PROBE_GATHER    n elements: an 8-byte word read in order, a 16-byte record gathered at a pseudo-random
 *                      row (a permutation), four 8-byte stores in order (the groupBy reduce's memory floor)
 *   DG_PROBE_ZC_WRITE  n bytes written by a kernel straight into pinned host memory (zero-copy over the link,
 *                      the dg_result_fetch_groups path)
 *   DG_PROBE_SORT      the groupBy sort alone: n packed [key | element index] words with the headline's key
 *                      shape (two uniform 17-bit dictionary ids below 100000), sorted by the engine's radix
 *                      passes (timed alone; the input is rewritten before each repetition) and checked
 *                      ascending afterwards (DG_ERR_DEVICE when not).
 *   DG_PROBE_CHAIN     n dependent one-workgroup kernels in a row on one stream (each reads the word its
 *                      predecessor wrote): the per-launch cost of a chain of small kernels
 *   DG_PROBE_CHAIN_GRAPH  the same chain captured once into a hipGraph and replayed with hipGraphLaunch
 *                      (capture and instantiation outside the timing)
 *   DG_PROBE_HOST_LAUNCH  host time per kernel launch call (n launches of the chain's kernel, timed on the
 *                      host without waiting for them)
 *   DG_PROBE_HOST_H2D  host time per hipMemcpyAsync of n bytes pinned host -> device (the staged upload)
 *   DG_PROBE_HOST_JOIN host time per cross-stream join (hipEventRecord on one stream + hipStreamWaitEvent
 *                      on another) */
#define DG_PROBE_COPY 0
#define DG_PROBE_D2H 1
#define DG_PROBE_H2D 2
#define DG_PROBE_GATHER 3
#define DG_PROBE_ZC_WRITE 4
#define DG_PROBE_SORT 5
#define DG_PROBE_CHAIN 6
#define DG_PROBE_CHAIN_GRAPH 7
#define DG_PROBE_HOST_LAUNCH 8
#define DG_PROBE_HOST_H2D 9
#define DG_PROBE_HOST_JOIN 10
int dg_debug_probe(int32_t device, int32_t kind, int64_t n, int32_t iters, double* ms);

#ifdef __cplusplus
}
#endif
#endif /* DRUIDGPU_H */
