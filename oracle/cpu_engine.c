/*
 * cpu_engine.c — multi-threaded native CPU restatement of the benchmarked query paths, timed as
 * bench.py's cpu_baseline. TEST / MEASUREMENT INFRASTRUCTURE ONLY (same rule as druid_oracle.c:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it).
 *
 * The reference's JMH harness cannot run here (no JVM). SURVEY §8(d) prescribes this
 * stand-in: the reference's per-segment loops in C, compiled -O3 -march=native, on all host cores
 * the caller passes, as ChainedExecutionQueryRunner / GroupByMergingQueryRunnerV2 spread segments
 * over the processing pool (query/ChainedExecutionQueryRunner.java:89-180,
 * druid.processing.numThreads) — here segments are further cut into row chunks so that every core
 * has work when there are fewer segments than cores.
 * It is linked with druid_oracle.c's segment reader and block decoders (LZ4 decoded per block
 * inside the timed call, as the reference decompresses per query).
 *
 * cpu_groupby2 — GroupByV2 over two string dimensions, ALL granularity, no filter,
 * count / longSum / doubleSum (BASELINE config 3), on every host core the caller gives it:
 *   per scan unit (a segment's rows in 1 M-row chunks, so a box with more cores than segments is
 *   used whole; one thread per unit at a time): decode the blocks of the id and metric columns
 *   holding the unit's rows; group rows with an
 *   open-addressing table on the (id1, id2) key (BufferHashGrouper / ByteBufferHashTable.findBucket,
 *   epinephelinae/ByteBufferHashTable.java:286-327, linear probing); the segment's groups are mapped
 *   to merged dictionary ids (the caller's per-segment maps: GroupByMergingQueryRunnerV2 merges by
 *   value, :188-246) and scattered into nthreads ranges of the first dimension;
 *   merge (one thread per range): fold equal keys across segments (AggregatorFactory.combine) in a
 *   hash table, then sort the range by key = the merged grouper's sorted iterator. The ranges'
 *   concatenation is the ordered merged result.
 * Returns the number of merged groups; sums[0..2] = total count, long sum, double sum (checks).
 * With a period (granularity), the key leads with the row's bucket index (GroupByQueryEngineV2 keys
 * rows by the cursor's bucket; the result orders by time, then dimensions).
 *
 * cpu_timeseries — TimeseriesQueryEngine (query/timeseries/TimeseriesQueryEngine.java:40-111) over
 *   every segment: the filter's bitmap (Filter.getBitmapResult: And/Or/Not over selector / in / bound
 *   leaves, each leaf the union of its dictionary ids' bitmaps, decoded from the segment's Concise or
 *   Roaring bytes) as a row bitset per segment, then per scan unit (1 M-row chunk) the rows of the
 *   interval, bucketed by the period's granularity, aggregated with Java semantics (long sums wrap,
 *   Math.min/max on doubles); units combine in order (TimeseriesBinaryFn).
 * cpu_topn — PooledTopNAlgorithm per segment (dense aggregation per dictionary id, top
 *   max(threshold, 1000) by the metric, TopNQueryQueryToolChest.java:553-561) and the TopNBinaryFn
 *   fold over the segments in order with the query's threshold (TopNBinaryFn.java:75-135), by merged
 *   (value-ordered) ids; the metric is a numeric aggregator (descending, ties by value), or with
 *   `merged_rank` the dimension's own order (DimensionTopNMetricSpec, TopNLexicographicResultBuilder:
 *   ascending rank of the value under the LEXICOGRAPHIC / ALPHANUMERIC / NUMERIC comparator, computed by
 *   the caller; equal ranks by value order) and `id_limit` > 0 the LEXICOGRAPHIC optimizer's cut: only
 *   local ids below it aggregate (BaseTopNAlgorithm.java:296-326 after
 *   DimensionTopNMetricSpec.configureOptimizer, DimensionTopNMetricSpec.java:117-124).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define OR_LONG 1
#define OR_DOUBLE 3

#include <math.h>

int or_read_column(void* h, const char* name, int as_kind, void* out);
int or_dim_ids(void* h, const char* name, int32_t* out);
int64_t or_num_rows(void* h);

typedef struct {
  uint64_t key;
  int64_t cnt, lsum;
  double dsum;
} grp;

typedef struct {
  grp* g;
  int64_t n, cap;
} grp_vec;

static void vec_push(grp_vec* v, const grp* x) {
  if (v->n == v->cap) {
    v->cap = v->cap ? 2 * v->cap : 1024;
    v->g = (grp*)realloc(v->g, (size_t)v->cap * sizeof(grp));
  }
  v->g[v->n++] = *x;
}

static inline uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

#define EMPTY (~0ull)

/* open-addressing grouper over the keys of `n` entries (rows or partial groups) */
static grp* group_table(int64_t n, uint64_t* mask_out) {
  uint64_t cap = 1024;
  while (cap < 2 * (uint64_t)n) cap <<= 1;
  grp* t = (grp*)malloc(cap * sizeof(grp));
  for (uint64_t i = 0; i < cap; ++i) t[i].key = EMPTY;
  *mask_out = cap - 1;
  return t;
}

static inline grp* find_bucket(grp* t, uint64_t mask, uint64_t key) {
  uint64_t h = mix64(key) & mask;
  for (;;) {
    grp* b = &t[h];
    if (b->key == key) return b;
    if (b->key == EMPTY) {
      b->key = key;
      b->cnt = 0;
      b->lsum = 0;
      b->dsum = 0.0;
      return b;
    }
    h = (h + 1) & mask;
  }
}

typedef struct {
  int64_t groups, cnt, lsum;
  double dsum;
  grp* out; /* the range's groups in key order (kept when the caller wants the rows) */
} part_res;

/* the scan units: a segment's rows in chunks of kChunkRows (a multiple of every block size: 8192
 * longs / doubles, 16384-65536 ids), so every host core has work even with fewer segments than
 * cores; each chunk groups its rows in its own table (a partial, folded by the merge in unit
 * order = segment, then row order) */
#define kChunkRows (1 << 20)

typedef struct {
  void** segs;
  int nseg;
  const char *d1, *d2, *lcol, *dcol;
  const int32_t* const* remap1;
  const int32_t* const* remap2;
  int32_t card1;
  int64_t origin, period, bucket0; /* period > 0: key hi = bucket index * card1 + merged id 1 */
  int32_t nbuckets;
  int nthreads;
  int nunits;
  int* unit_seg;
  int64_t* unit_row0;
  int64_t* unit_rows;
  grp_vec* parts; /* [nunits][nthreads]: a unit's groups, by range of the first merged id */
  part_res* res;  /* [nthreads] */
  int keep;
  int64_t next_unit;
  int64_t next_part;
  int err;
} gb_ctx;

int or_read_rows(void* h, const char* name, int kind, int64_t row0, int64_t n, void* out);
#define OR_STRING 4

static int64_t floor_div(int64_t a, int64_t b) { return a / b - ((a % b != 0) && ((a < 0) != (b < 0))); }

static void* gb_segment_worker(void* arg) {
  gb_ctx* c = (gb_ctx*)arg;
  int64_t* tt = c->period > 0 ? (int64_t*)malloc((size_t)kChunkRows * 8 + 16) : NULL;
  int32_t* a = (int32_t*)malloc((size_t)kChunkRows * 4 + 16);
  int32_t* b = (int32_t*)malloc((size_t)kChunkRows * 4 + 16);
  int64_t* l = (int64_t*)malloc((size_t)kChunkRows * 8 + 16);
  double* d = (double*)malloc((size_t)kChunkRows * 8 + 16);
  for (;;) {
    const int u = (int)__atomic_fetch_add(&c->next_unit, 1, __ATOMIC_RELAXED);
    if (u >= c->nunits) break;
    const int s = c->unit_seg[u];
    void* h = c->segs[s];
    const int64_t r0 = c->unit_row0[u], n = c->unit_rows[u];
    if (or_read_rows(h, c->d1, OR_STRING, r0, n, a) || or_read_rows(h, c->d2, OR_STRING, r0, n, b) ||
        or_read_rows(h, c->lcol, OR_LONG, r0, n, l) || or_read_rows(h, c->dcol, OR_DOUBLE, r0, n, d) ||
        (tt && or_read_rows(h, "__time", OR_LONG, r0, n, tt))) {
      c->err = 1;
      continue;
    }
    uint64_t mask;
    grp* t = group_table(n, &mask);
    for (int64_t r = 0; r < n; ++r) {
      /* local key: bucket index (20 bits) | local id 1 (22 bits) | local id 2 (22 bits) */
      const uint64_t bk = tt ? (uint64_t)(floor_div(tt[r] - c->origin, c->period) - c->bucket0) : 0;
      grp* g = find_bucket(t, mask, (bk << 44) | ((uint64_t)(uint32_t)a[r] << 22) | (uint32_t)b[r]);
      g->cnt += 1;
      g->lsum += l[r];
      g->dsum += d[r];
    }
    const int T = c->nthreads;
    for (uint64_t i = 0; i <= mask; ++i) {
      if (t[i].key == EMPTY) continue;
      grp x = t[i];
      const uint64_t bk = x.key >> 44;
      const uint32_t m1 = (uint32_t)c->remap1[s][(x.key >> 22) & 0x3FFFFF], m2 = (uint32_t)c->remap2[s][x.key & 0x3FFFFF];
      const uint64_t hi = bk * (uint64_t)(c->card1 > 0 ? c->card1 : 1) + m1;
      x.key = (hi << 32) | m2;
      const uint64_t span = (uint64_t)(c->nbuckets > 0 ? c->nbuckets : 1) * (uint64_t)(c->card1 > 0 ? c->card1 : 1);
      const int p = (int)((hi * (uint64_t)T) / span);
      vec_push(&c->parts[(size_t)u * T + p], &x);
    }
    free(t);
  }
  free(tt);
  free(a);
  free(b);
  free(l);
  free(d);
  return NULL;
}

static int cmp_key(const void* x, const void* y) {
  const uint64_t a = ((const grp*)x)->key, b = ((const grp*)y)->key;
  return (a > b) - (a < b);
}

static void* gb_merge_worker(void* arg) {
  gb_ctx* c = (gb_ctx*)arg;
  const int T = c->nthreads;
  for (;;) {
    const int p = (int)__atomic_fetch_add(&c->next_part, 1, __ATOMIC_RELAXED);
    if (p >= T) break;
    int64_t total = 0;
    for (int u = 0; u < c->nunits; ++u) total += c->parts[(size_t)u * T + p].n;
    uint64_t mask;
    grp* t = group_table(total, &mask);
    int64_t ng = 0;
    for (int u = 0; u < c->nunits; ++u) {  /* unit order: segment, then row order */
      const grp_vec* v = &c->parts[(size_t)u * T + p];
      for (int64_t i = 0; i < v->n; ++i) {
        grp* g = find_bucket(t, mask, v->g[i].key);
        ng += g->cnt == 0;
        g->cnt += v->g[i].cnt;
        g->lsum += v->g[i].lsum;
        g->dsum += v->g[i].dsum;
      }
    }
    grp* out = (grp*)malloc((size_t)(ng > 0 ? ng : 1) * sizeof(grp));
    int64_t k = 0;
    for (uint64_t i = 0; i <= mask; ++i)
      if (t[i].key != EMPTY) out[k++] = t[i];
    free(t);
    qsort(out, (size_t)k, sizeof(grp), cmp_key); /* the range in merged-key (= value) order */
    part_res r = {k, 0, 0, 0.0, NULL};
    for (int64_t i = 0; i < k; ++i) {
      r.cnt += out[i].cnt;
      r.lsum += out[i].lsum;
      r.dsum += out[i].dsum;
    }
    if (c->keep) r.out = out;
    else free(out);
    c->res[p] = r;
  }
  return NULL;
}

static void run_threads(int nthreads, void* (*fn)(void*), void* arg) {
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, fn, arg);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* out_key / out_lsum / out_dsum (optional, capacity = total rows): the merged groups in result
 * order, key = merged id 1 << 32 | merged id 2 (written after the timed part); *seconds = the
 * query's wall time (scan + merge + ordered result), excluding that copy-out */
int64_t cpu_groupby2(void** segs, int nseg, const char* d1, const char* d2, const char* lcol, const char* dcol,
                     const int32_t* const* remap1, const int32_t* const* remap2, int32_t card1, int nthreads,
                     int64_t origin, int64_t period, int64_t bucket0, int32_t nbuckets,
                     double* sums, uint64_t* out_key, int64_t* out_cnt, int64_t* out_lsum, double* out_dsum,
                     double* seconds) {
  if (nthreads < 1) nthreads = 1;
  if (period > 0 && (nbuckets <= 0 || nbuckets >= (1 << 20))) return -1;
  const double t0 = now_s();
  gb_ctx c;
  memset(&c, 0, sizeof c);
  c.segs = segs;
  c.nseg = nseg;
  c.d1 = d1;
  c.d2 = d2;
  c.lcol = lcol;
  c.dcol = dcol;
  c.remap1 = remap1;
  c.remap2 = remap2;
  c.card1 = card1;
  c.origin = origin;
  c.period = period;
  c.bucket0 = bucket0;
  c.nbuckets = period > 0 ? nbuckets : 1;
  c.nthreads = nthreads;
  c.keep = out_key != NULL;
  for (int s = 0; s < nseg; ++s) c.nunits += (int)((or_num_rows(segs[s]) + kChunkRows - 1) / kChunkRows);
  c.unit_seg = (int*)malloc(sizeof(int) * (size_t)(c.nunits + 1));
  c.unit_row0 = (int64_t*)malloc(sizeof(int64_t) * (size_t)(c.nunits + 1));
  c.unit_rows = (int64_t*)malloc(sizeof(int64_t) * (size_t)(c.nunits + 1));
  for (int s = 0, u = 0; s < nseg; ++s)
    for (int64_t r = 0, n = or_num_rows(segs[s]); r < n; r += kChunkRows, ++u) {
      c.unit_seg[u] = s;
      c.unit_row0[u] = r;
      c.unit_rows[u] = n - r < kChunkRows ? n - r : kChunkRows;
    }
  c.parts = (grp_vec*)calloc((size_t)c.nunits * nthreads, sizeof(grp_vec));
  c.res = (part_res*)calloc((size_t)nthreads, sizeof(part_res));
  run_threads(nthreads < c.nunits ? nthreads : (c.nunits > 0 ? c.nunits : 1), gb_segment_worker, &c);
  int64_t ng = -1;
  if (!c.err) {
    run_threads(nthreads, gb_merge_worker, &c);
    if (seconds) *seconds = now_s() - t0;
    ng = 0;
    double cnt = 0, ls = 0, ds = 0;
    for (int p = 0; p < nthreads; ++p) {
      if (c.keep)
        for (int64_t i = 0; i < c.res[p].groups; ++i) {
          const grp* g = &c.res[p].out[i];
          out_key[ng + i] = g->key;
          if (out_cnt) out_cnt[ng + i] = g->cnt;
          out_lsum[ng + i] = g->lsum;
          out_dsum[ng + i] = g->dsum;
        }
      free(c.res[p].out);
      ng += c.res[p].groups;
      cnt += (double)c.res[p].cnt;
      ls += (double)c.res[p].lsum;
      ds += c.res[p].dsum;
    }
    if (sums) {
      sums[0] = cnt;
      sums[1] = ls;
      sums[2] = ds;
    }
  }
  for (int64_t i = 0; i < (int64_t)c.nunits * nthreads; ++i) free(c.parts[i].g);
  free(c.parts);
  free(c.res);
  free(c.unit_seg);
  free(c.unit_row0);
  free(c.unit_rows);
  return ng;
}

/* ------------------------------------------------------------------------------------------------
 * filter programs: postfix over leaves (op >= 0: push leaf op; -1: AND of the top two, -2: OR of the
 * top two, -3: NOT of the top) -> a row bitset per segment (NULL: no filter, every row)
 * ------------------------------------------------------------------------------------------------ */
int64_t or_dim_bitmap(void* h, const char* name, int32_t id, int32_t* out, int64_t cap);

typedef struct {
  const int32_t* prog;
  int nprog;
  const char* const* leaf_dims;
  const int32_t* const* leaf_ids; /* [nseg * nleaf], each -1 terminated */
  int nleaf;
} fprog;

static uint64_t* eval_filter(void* h, int seg, int64_t nrows, const fprog* f, int* err) {
  if (!f->nprog) return NULL;
  const int64_t W = (nrows + 63) / 64;
  uint64_t* st[16];
  int sp = 0;
  int32_t* rows = (int32_t*)malloc((size_t)(nrows > 0 ? nrows : 1) * 4);
  for (int i = 0; i < f->nprog; ++i) {
    const int op = f->prog[i];
    if (op >= 0) {
      if (sp >= 16) {
        *err = 1;
        break;
      }
      uint64_t* b = (uint64_t*)calloc((size_t)(W > 0 ? W : 1), 8);
      const int32_t* ids = f->leaf_ids[(size_t)seg * f->nleaf + op];
      for (int k = 0; ids && ids[k] >= 0; ++k) {
        const int64_t m = or_dim_bitmap(h, f->leaf_dims[op], ids[k], rows, nrows);
        for (int64_t j = 0; j < m; ++j) b[rows[j] >> 6] |= 1ull << (rows[j] & 63);
      }
      st[sp++] = b;
    } else if (op == -3) {
      if (sp < 1) {
        *err = 1;
        break;
      }
      uint64_t* b = st[sp - 1];
      for (int64_t w = 0; w < W; ++w) b[w] = ~b[w];
      if (nrows & 63) b[W - 1] &= (1ull << (nrows & 63)) - 1;
    } else {
      if (sp < 2) {
        *err = 1;
        break;
      }
      uint64_t *a = st[sp - 2], *b = st[sp - 1];
      if (op == -1)
        for (int64_t w = 0; w < W; ++w) a[w] &= b[w];
      else
        for (int64_t w = 0; w < W; ++w) a[w] |= b[w];
      free(b);
      --sp;
    }
  }
  free(rows);
  if (*err || sp != 1) {
    *err = 1;
    while (sp > 0) free(st[--sp]);
    return NULL;
  }
  return st[0];
}

/* aggregator kinds (druid_oracle.c AGG_*) with 8-byte states */
enum { K_COUNT = 0, K_LONG_SUM = 1, K_DOUBLE_SUM = 2, K_LONG_MIN = 4, K_LONG_MAX = 5, K_DOUBLE_MIN = 6, K_DOUBLE_MAX = 7 };
void or_agg_init(int kind, int32_t ngroups, void* state);
void or_agg_combine(int kind, int32_t n, void* acc, const void* other);

static int is_negzero(double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  return u == 0x8000000000000000ull;
}
static inline double jmin(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && is_negzero(b)) return b;
  return a <= b ? a : b;
}
static inline double jmax(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && is_negzero(a)) return b;
  return a >= b ? a : b;
}
static int kind_is_long(int k) { return k == K_LONG_SUM || k == K_LONG_MIN || k == K_LONG_MAX; }

typedef struct {
  void** segs;
  int nseg, nthreads;
  fprog f;
  uint64_t** bits; /* per segment (NULL: every row) */
  int64_t t_lo, t_hi, origin, period, bucket0;
  int32_t nbuckets;
  int nagg;
  const int32_t* kinds;
  const char* const* cols;
  int nunits;
  int* unit_seg;
  int64_t *unit_row0, *unit_rows;
  int64_t* unit_cnt;    /* [nunits][nbuckets] */
  uint64_t* unit_state; /* [nunits][nagg][nbuckets] */
  int64_t next;
  int err;
} ts_ctx;

static void* ts_filter_worker(void* arg) {
  ts_ctx* c = (ts_ctx*)arg;
  for (;;) {
    const int s = (int)__atomic_fetch_add(&c->next, 1, __ATOMIC_RELAXED);
    if (s >= c->nseg) break;
    int err = 0;
    c->bits[s] = eval_filter(c->segs[s], s, or_num_rows(c->segs[s]), &c->f, &err);
    if (err) c->err = 1;
  }
  return NULL;
}

static void* ts_unit_worker(void* arg) {
  ts_ctx* c = (ts_ctx*)arg;
  int64_t* tt = (int64_t*)malloc((size_t)kChunkRows * 8 + 16);
  void* vals = malloc((size_t)kChunkRows * 8 * (size_t)(c->nagg > 0 ? c->nagg : 1) + 16);
  int32_t* bk = (int32_t*)malloc((size_t)kChunkRows * 4 + 16);
  for (;;) {
    const int u = (int)__atomic_fetch_add(&c->next, 1, __ATOMIC_RELAXED);
    if (u >= c->nunits) break;
    const int s = c->unit_seg[u];
    void* h = c->segs[s];
    const int64_t r0 = c->unit_row0[u], n = c->unit_rows[u], NB = c->nbuckets;
    int64_t* cnt = c->unit_cnt + (size_t)u * NB;
    uint64_t* st = c->unit_state + (size_t)u * c->nagg * NB;
    for (int a = 0; a < c->nagg; ++a) or_agg_init(c->kinds[a], (int32_t)NB, st + (size_t)a * NB);
    if (or_read_rows(h, "__time", OR_LONG, r0, n, tt)) {
      c->err = 1;
      continue;
    }
    for (int a = 0; a < c->nagg; ++a)
      if (c->kinds[a] != K_COUNT &&
          or_read_rows(h, c->cols[a], kind_is_long(c->kinds[a]) ? OR_LONG : OR_DOUBLE, r0, n, (uint8_t*)vals + (size_t)a * kChunkRows * 8))
        c->err = 1;
    const uint64_t* bits = c->bits[s];
    /* the selected rows' buckets (-1: not selected) */
    for (int64_t r = 0; r < n; ++r) {
      const int64_t row = r0 + r, t = tt[r];
      int32_t b = -1;
      if ((!bits || ((bits[row >> 6] >> (row & 63)) & 1)) && t >= c->t_lo && t < c->t_hi)
        b = c->period > 0 ? (int32_t)(floor_div(t - c->origin, c->period) - c->bucket0) : 0;
      if (b >= NB) b = -1;
      bk[r] = b;
      if (b >= 0) cnt[b] += 1;
    }
    for (int a = 0; a < c->nagg; ++a) {
      uint64_t* sa = st + (size_t)a * NB;
      const int64_t* lv = (const int64_t*)((uint8_t*)vals + (size_t)a * kChunkRows * 8);
      const double* dv = (const double*)lv;
      switch (c->kinds[a]) {
        case K_COUNT:
          for (int64_t r = 0; r < n; ++r)
            if (bk[r] >= 0) sa[bk[r]] += 1;
          break;
        case K_LONG_SUM:
          for (int64_t r = 0; r < n; ++r)
            if (bk[r] >= 0) sa[bk[r]] += (uint64_t)lv[r];
          break;
        case K_LONG_MIN:
          for (int64_t r = 0; r < n; ++r)
            if (bk[r] >= 0 && lv[r] < (int64_t)sa[bk[r]]) sa[bk[r]] = (uint64_t)lv[r];
          break;
        case K_LONG_MAX:
          for (int64_t r = 0; r < n; ++r)
            if (bk[r] >= 0 && lv[r] > (int64_t)sa[bk[r]]) sa[bk[r]] = (uint64_t)lv[r];
          break;
        case K_DOUBLE_SUM:
          for (int64_t r = 0; r < n; ++r)
            if (bk[r] >= 0) ((double*)sa)[bk[r]] += dv[r];
          break;
        case K_DOUBLE_MIN:
          for (int64_t r = 0; r < n; ++r)
            if (bk[r] >= 0) ((double*)sa)[bk[r]] = jmin(((double*)sa)[bk[r]], dv[r]);
          break;
        case K_DOUBLE_MAX:
          for (int64_t r = 0; r < n; ++r)
            if (bk[r] >= 0) ((double*)sa)[bk[r]] = jmax(((double*)sa)[bk[r]], dv[r]);
          break;
        default:
          c->err = 1;
      }
    }
  }
  free(tt);
  free(vals);
  free(bk);
  return NULL;
}

static void make_units(void** segs, int nseg, int64_t chunk, int* nunits, int** useg, int64_t** ur0, int64_t** urows) {
  int nu = 0;
  for (int s = 0; s < nseg; ++s) nu += (int)((or_num_rows(segs[s]) + chunk - 1) / chunk);
  *useg = (int*)malloc(sizeof(int) * (size_t)(nu + 1));
  *ur0 = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nu + 1));
  *urows = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nu + 1));
  for (int s = 0, u = 0; s < nseg; ++s)
    for (int64_t r = 0, n = or_num_rows(segs[s]); r < n; r += chunk, ++u) {
      (*useg)[u] = s;
      (*ur0)[u] = r;
      (*urows)[u] = n - r < chunk ? n - r : chunk;
    }
  *nunits = nu;
}

/* Timeseries over the segments; out_rows[b] = selected rows of bucket b, out_state[a * nbuckets + b] =
 * aggregator a's 8-byte state (int64 / double). Returns 0, or -1 on an error. *seconds = wall time. */
int cpu_timeseries(void** segs, int nseg, int nthreads, const int32_t* prog, int nprog, const char* const* leaf_dims,
                   const int32_t* const* leaf_ids, int nleaf, int64_t t_lo, int64_t t_hi, int64_t origin,
                   int64_t period, int64_t bucket0, int32_t nbuckets, int nagg, const int32_t* kinds,
                   const char* const* cols, int64_t* out_rows, uint64_t* out_state, double* seconds) {
  if (nthreads < 1) nthreads = 1;
  if (nbuckets < 1) return -1;
  const double t0 = now_s();
  ts_ctx c;
  memset(&c, 0, sizeof c);
  c.segs = segs;
  c.nseg = nseg;
  c.nthreads = nthreads;
  c.f.prog = prog;
  c.f.nprog = nprog;
  c.f.leaf_dims = leaf_dims;
  c.f.leaf_ids = leaf_ids;
  c.f.nleaf = nleaf;
  c.t_lo = t_lo;
  c.t_hi = t_hi;
  c.origin = origin;
  c.period = period;
  c.bucket0 = bucket0;
  c.nbuckets = nbuckets;
  c.nagg = nagg;
  c.kinds = kinds;
  c.cols = cols;
  c.bits = (uint64_t**)calloc((size_t)(nseg > 0 ? nseg : 1), sizeof(uint64_t*));
  run_threads(nthreads < nseg ? nthreads : (nseg > 0 ? nseg : 1), ts_filter_worker, &c);
  make_units(segs, nseg, kChunkRows, &c.nunits, &c.unit_seg, &c.unit_row0, &c.unit_rows);
  c.unit_cnt = (int64_t*)calloc((size_t)c.nunits * nbuckets + 1, 8);
  c.unit_state = (uint64_t*)calloc((size_t)c.nunits * nagg * nbuckets + 1, 8);
  c.next = 0;
  if (!c.err) run_threads(nthreads < c.nunits ? nthreads : (c.nunits > 0 ? c.nunits : 1), ts_unit_worker, &c);
  /* units combine in order (segment, then rows): AggregatorFactory.combine */
  memset(out_rows, 0, sizeof(int64_t) * (size_t)nbuckets);
  for (int a = 0; a < nagg; ++a) or_agg_init(kinds[a], nbuckets, out_state + (size_t)a * nbuckets);
  for (int u = 0; u < c.nunits && !c.err; ++u) {
    for (int b = 0; b < nbuckets; ++b) out_rows[b] += c.unit_cnt[(size_t)u * nbuckets + b];
    for (int a = 0; a < nagg; ++a)
      or_agg_combine(kinds[a], nbuckets, out_state + (size_t)a * nbuckets, c.unit_state + ((size_t)u * nagg + a) * nbuckets);
  }
  if (seconds) *seconds = now_s() - t0;
  for (int s = 0; s < nseg; ++s) free(c.bits[s]);
  free(c.bits);
  free(c.unit_cnt);
  free(c.unit_state);
  free(c.unit_seg);
  free(c.unit_row0);
  free(c.unit_rows);
  return c.err ? -1 : 0;
}

/* ---- topN ---- */
typedef struct {
  int32_t id; /* merged id */
  double metric;
  uint64_t v[8];
} tn_ent;

typedef struct {
  void** segs;
  int nseg, nthreads;
  fprog f;
  const char* dim;
  const int32_t* const* remap; /* per segment: local id -> merged id (value order) */
  int nagg, metric;
  const int32_t* kinds;
  const char* const* cols;
  int32_t seg_threshold;
  const int32_t* merged_rank; /* dimension order: rank of every merged id (NULL: the numeric metric) */
  int32_t id_limit;           /* > 0: local ids at or above it do not aggregate */
  tn_ent** lists;
  int32_t* nlist;
  int64_t next;
  int err;
} tn_ctx;

static int tn_cmp(const void* x, const void* y) { /* metric descending (Double.compare), ties by value */
  const tn_ent *a = (const tn_ent*)x, *b = (const tn_ent*)y;
  const double ma = a->metric, mb = b->metric;
  const int an = ma != ma, bn = mb != mb;
  if (an != bn) return an ? -1 : 1; /* NaN is the largest */
  if (!an && ma != mb) return ma > mb ? -1 : 1;
  return (a->id > b->id) - (a->id < b->id);
}

static double tn_metric(int kind, uint64_t v) {
  if (kind_is_long(kind) || kind == K_COUNT) return (double)(int64_t)v;
  double d;
  memcpy(&d, &v, 8);
  return d;
}

static void* tn_seg_worker(void* arg) {
  tn_ctx* c = (tn_ctx*)arg;
  for (;;) {
    const int s = (int)__atomic_fetch_add(&c->next, 1, __ATOMIC_RELAXED);
    if (s >= c->nseg) break;
    void* h = c->segs[s];
    const int64_t n = or_num_rows(h);
    int err = 0;
    uint64_t* bits = eval_filter(h, s, n, &c->f, &err);
    int32_t* ids = (int32_t*)malloc((size_t)(n > 0 ? n : 1) * 4);
    void* vals = malloc((size_t)(n > 0 ? n : 1) * 8 * (size_t)(c->nagg > 0 ? c->nagg : 1));
    int32_t card = 0;
    if (err || or_read_rows(h, c->dim, OR_STRING, 0, n, ids)) err = 1;
    for (int64_t r = 0; r < n && !err; ++r)
      if (ids[r] + 1 > card) card = ids[r] + 1;
    for (int a = 0; a < c->nagg && !err; ++a)
      if (c->kinds[a] != K_COUNT &&
          or_read_rows(h, c->cols[a], kind_is_long(c->kinds[a]) ? OR_LONG : OR_DOUBLE, 0, n, (uint8_t*)vals + (size_t)a * n * 8))
        err = 1;
    /* PooledTopNAlgorithm: one record per dictionary id */
    uint64_t* st = (uint64_t*)calloc((size_t)(card > 0 ? card : 1) * c->nagg + 1, 8);
    uint8_t* touched = (uint8_t*)calloc((size_t)(card > 0 ? card : 1), 1);
    for (int a = 0; a < c->nagg && !err; ++a) or_agg_init(c->kinds[a], card, st + (size_t)a * card);
    for (int64_t r = 0; r < n && !err; ++r) {
      if (bits && !((bits[r >> 6] >> (r & 63)) & 1)) continue;
      const int32_t g = ids[r];
      if (c->id_limit > 0 && g >= c->id_limit) continue;
      touched[g] = 1;
      for (int a = 0; a < c->nagg; ++a) {
        uint64_t* sa = st + (size_t)a * card + g;
        const int64_t lv = ((const int64_t*)((uint8_t*)vals + (size_t)a * n * 8))[r];
        double dv;
        memcpy(&dv, &lv, 8);
        switch (c->kinds[a]) {
          case K_COUNT: *sa += 1; break;
          case K_LONG_SUM: *sa += (uint64_t)lv; break;
          case K_LONG_MIN: if (lv < (int64_t)*sa) *sa = (uint64_t)lv; break;
          case K_LONG_MAX: if (lv > (int64_t)*sa) *sa = (uint64_t)lv; break;
          case K_DOUBLE_SUM: *(double*)sa += dv; break;
          case K_DOUBLE_MIN: *(double*)sa = jmin(*(double*)sa, dv); break;
          case K_DOUBLE_MAX: *(double*)sa = jmax(*(double*)sa, dv); break;
          default: err = 1;
        }
      }
    }
    int32_t m = 0;
    tn_ent* all = (tn_ent*)malloc(sizeof(tn_ent) * (size_t)(card > 0 ? card : 1));
    for (int32_t g = 0; g < card && !err; ++g) {
      if (!touched[g]) continue;
      tn_ent e;
      memset(&e, 0, sizeof e);
      e.id = c->remap[s][g];
      for (int a = 0; a < c->nagg; ++a) e.v[a] = st[(size_t)a * card + g];
      e.metric = c->merged_rank ? -(double)c->merged_rank[e.id] : tn_metric(c->kinds[c->metric], e.v[c->metric]);
      all[m++] = e;
    }
    qsort(all, (size_t)m, sizeof(tn_ent), tn_cmp);
    c->nlist[s] = m < c->seg_threshold ? m : c->seg_threshold;
    c->lists[s] = all;
    if (err) c->err = 1;
    free(bits);
    free(ids);
    free(vals);
    free(st);
    free(touched);
  }
  return NULL;
}

/* out: up to `threshold` entries: merged id and the aggregators' 8-byte states [threshold][nagg].
 * Returns the entry count, or -1 on an error. */
int cpu_topn(void** segs, int nseg, int nthreads, const int32_t* prog, int nprog, const char* const* leaf_dims,
             const int32_t* const* leaf_ids, int nleaf, const char* dim, const int32_t* const* remap, int nagg,
             const int32_t* kinds, const char* const* cols, int metric, int32_t threshold, int32_t min_threshold,
             const int32_t* merged_rank, int32_t id_limit, int32_t* out_ids, uint64_t* out_vals, double* seconds) {
  if (nagg > 8 || (!merged_rank && (metric < 0 || metric >= nagg)) || threshold < 1) return -1;
  if (nthreads < 1) nthreads = 1;
  const double t0 = now_s();
  tn_ctx c;
  memset(&c, 0, sizeof c);
  c.segs = segs;
  c.nseg = nseg;
  c.nthreads = nthreads;
  c.f.prog = prog;
  c.f.nprog = nprog;
  c.f.leaf_dims = leaf_dims;
  c.f.leaf_ids = leaf_ids;
  c.f.nleaf = nleaf;
  c.dim = dim;
  c.remap = remap;
  c.nagg = nagg;
  c.metric = metric;
  c.kinds = kinds;
  c.cols = cols;
  c.seg_threshold = threshold > min_threshold ? threshold : min_threshold;
  c.merged_rank = merged_rank;
  c.id_limit = id_limit;
  c.lists = (tn_ent**)calloc((size_t)(nseg > 0 ? nseg : 1), sizeof(tn_ent*));
  c.nlist = (int32_t*)calloc((size_t)(nseg > 0 ? nseg : 1), sizeof(int32_t));
  run_threads(nthreads < nseg ? nthreads : (nseg > 0 ? nseg : 1), tn_seg_worker, &c);
  /* TopNBinaryFn fold in segment order: combine equal values, keep the query's threshold */
  tn_ent* acc = (tn_ent*)malloc(sizeof(tn_ent) * (size_t)(2 * c.seg_threshold + threshold + 1));  /* (a list + the next) */
  int32_t na = 0;
  for (int s = 0; s < nseg && !c.err; ++s) {
    tn_ent* l = c.lists[s];
    const int32_t nl = c.nlist[s];
    if (s == 0) {
      memcpy(acc, l, sizeof(tn_ent) * (size_t)nl);
      na = nl;
      /* (a lone first result keeps its per-segment list; the fold truncates at the next merge) */
      continue;
    }
    int32_t n0 = na;
    for (int32_t i = 0; i < nl; ++i) {
      int32_t j = 0;
      while (j < n0 && acc[j].id != l[i].id) ++j;
      if (j < n0) {
        for (int a = 0; a < nagg; ++a) or_agg_combine(kinds[a], 1, &acc[j].v[a], &l[i].v[a]);
        if (!merged_rank) acc[j].metric = tn_metric(kinds[metric], acc[j].v[metric]);
      } else {
        acc[na++] = l[i];
      }
    }
    qsort(acc, (size_t)na, sizeof(tn_ent), tn_cmp);
    if (na > threshold) na = threshold;
  }
  if (na > threshold) na = threshold; /* the toolchest's final Iterables.limit */
  if (seconds) *seconds = now_s() - t0;
  for (int32_t i = 0; i < na; ++i) {
    out_ids[i] = acc[i].id;
    for (int a = 0; a < nagg; ++a) out_vals[(size_t)i * nagg + a] = acc[i].v[a];
  }
  for (int s = 0; s < nseg; ++s) free(c.lists[s]);
  free(c.lists);
  free(c.nlist);
  free(acc);
  return c.err ? -1 : na;
}
