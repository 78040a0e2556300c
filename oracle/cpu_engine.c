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
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define OR_LONG 1
#define OR_DOUBLE 3

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

static void* gb_segment_worker(void* arg) {
  gb_ctx* c = (gb_ctx*)arg;
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
        or_read_rows(h, c->lcol, OR_LONG, r0, n, l) || or_read_rows(h, c->dcol, OR_DOUBLE, r0, n, d)) {
      c->err = 1;
      continue;
    }
    uint64_t mask;
    grp* t = group_table(n, &mask);
    for (int64_t r = 0; r < n; ++r) {
      grp* g = find_bucket(t, mask, ((uint64_t)(uint32_t)a[r] << 32) | (uint32_t)b[r]);
      g->cnt += 1;
      g->lsum += l[r];
      g->dsum += d[r];
    }
    const int T = c->nthreads;
    for (uint64_t i = 0; i <= mask; ++i) {
      if (t[i].key == EMPTY) continue;
      grp x = t[i];
      const uint32_t m1 = (uint32_t)c->remap1[s][x.key >> 32], m2 = (uint32_t)c->remap2[s][x.key & 0xffffffffu];
      x.key = ((uint64_t)m1 << 32) | m2;
      const int p = (int)(((int64_t)m1 * T) / (c->card1 > 0 ? c->card1 : 1));
      vec_push(&c->parts[(size_t)u * T + p], &x);
    }
    free(t);
  }
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
                     double* sums, uint64_t* out_key, int64_t* out_cnt, int64_t* out_lsum, double* out_dsum,
                     double* seconds) {
  if (nthreads < 1) nthreads = 1;
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
