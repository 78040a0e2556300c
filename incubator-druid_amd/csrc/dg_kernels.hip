// dg_kernels.hip — HIP kernels (gfx950 / CDNA4) of the segment scan-and-aggregate path.
//
// Every kernel here replaces a Java hot loop of the reference:
//   k_lz4_decode      LZ4 block decompression          CompressionStrategy.LZ4Decompressor (data/CompressionStrategy.java:284-305)
//                                                      -> lz4-java LZ4SafeDecompressor (LZ4 block format)
//   k_concise_or      Concise word expansion + union   ImmutableConciseSet.union / BitIterator (extendedset/.../BitIterator.java:145-281)
//   k_roaring_or      Roaring container expansion      ImmutableRoaringBitmap.or (RoaringBitmapFactory.java:145-179)
//   k_filter_eval     AND/OR/NOT over row bitsets       AndFilter/OrFilter/NotFilter.getBitmapResult (segment/filter/*.java)
//   k_scan_agg        masked per-bucket aggregation     TimeseriesQueryEngine.java:86-92 (Aggregator.aggregate per cursor row),
//                     / per-dictionary-id aggregation   PooledTopNAlgorithm.aggregateDimValue (query/topn/PooledTopNAlgorithm.java:661-719)
//   k_topn_select     K-th largest metric + candidates  TopNNumericResultBuilder priority queue (TopNNumericResultBuilder.java:94-191)
//   (groupBy: dg_sort.hip — keygen + radix sort + segmented reduce replace BufferHashGrouper and the merge)
//
// Nothing here is a dense contraction, so there is no MFMA: every kernel is HBM/L2-bound integer and
// byte work, written for 64-wide wavefronts (ballot masks are 64-bit) with coalesced row tiles.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dg_device.h"

namespace dg {

// block-wide (256 threads = 4 waves) exclusive scan of int64; returns total via *total
__device__ int64_t block_exclusive_scan(int64_t v, int64_t* total, int64_t* s_tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_tmp[wave] = x;
  __syncthreads();
  int64_t wave_off = 0, tot = 0;
  const int nw = blockDim.x >> 6;
  for (int w = 0; w < nw; ++w) {
    if (w < wave) wave_off += s_tmp[w];
    tot += s_tmp[w];
  }
  __syncthreads();
  *total = tot;
  return wave_off + x - v;
}


// ------------------------------------------------------------------------------------------------
// Concise -> dense row bitset (OR). One workgroup per bitmap; 256 words per step: each thread
// decodes one big-endian word, a block scan turns word spans (31 or 31*(n+1) rows) into row
// offsets, then the word's bits are OR-ed into the dense uint32 bitset.
// Word format: ConciseSetUtils.java:45-75,149-281 (literal = MSB 1 + 31 bits; fill = bit30 fill
// value, bits25-29 flipped bit+1, bits0-24 blocks-1; flipped bit is in the first block).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void or_bits(uint32_t* set, int64_t bit, uint32_t bits31, int64_t limit) {
  if (!bits31 || bit < 0 || bit >= limit) return;
  const int64_t w = bit >> 5;
  const int sh = (int)(bit & 31);
  const uint32_t lo = bits31 << sh;
  if (lo) atomicOr(set + w, lo);
  if (sh > 1 && ((w + 1) << 5) < limit) {
    const uint32_t hi = bits31 >> (32 - sh);
    if (hi) atomicOr(set + w + 1, hi);
  }
}

__device__ void or_range(uint32_t* set, int64_t lo, int64_t hi, int64_t skip, int64_t limit) {
  // set bits [lo, hi) except `skip`; bits at or beyond `limit` (the bitset capacity) are dropped
  if (hi > limit) hi = limit;
  if (lo < 0) lo = 0;
  if (hi <= lo) return;
  for (int64_t w = lo >> 5; w <= ((hi - 1) >> 5); ++w) {
    int64_t b0 = w << 5;
    uint32_t m = 0xFFFFFFFFu;
    if (lo > b0) m &= 0xFFFFFFFFu << (lo - b0);
    if (hi < b0 + 32) m &= 0xFFFFFFFFu >> (b0 + 32 - hi);
    if (skip >= b0 && skip < b0 + 32) m &= ~(1u << (skip - b0));
    if (m == 0xFFFFFFFFu) set[w] = m;  // idempotent with concurrent ORs
    else if (m) atomicOr(set + w, m);
  }
}

__global__ __launch_bounds__(256) void k_concise_or(const uint8_t* __restrict__ base, const int64_t* __restrict__ off,
                                                    const int32_t* __restrict__ len, const int32_t* __restrict__ target,
                                                    const int64_t* __restrict__ row0, uint32_t* const* __restrict__ sets,
                                                    int64_t limit) {
  __shared__ int64_t s_tmp[8];
  const int b = blockIdx.x;
  const uint32_t* words = reinterpret_cast<const uint32_t*>(base + off[b]);
  const int nw = len[b] >> 2;
  uint32_t* set = sets[target[b]];
  int64_t carry = row0 ? row0[b] : 0;  // a piece of a split bitmap starts mid-way
  for (int basew = 0; basew < nw; basew += 256) {
    const int i = basew + threadIdx.x;
    uint32_t w = 0;
    int64_t span = 0;
    if (i < nw) {
      w = __builtin_bswap32(words[i]);
      span = (w & 0x80000000u) ? 31 : 31ll * ((int64_t)(w & 0x01FFFFFFu) + 1);
    }
    int64_t total;
    const int64_t o = carry + block_exclusive_scan(span, &total, s_tmp);
    if (i < nw) {
      if (w & 0x80000000u) {
        or_bits(set, o, w & 0x7FFFFFFFu, limit);
      } else {
        const int flip = (int)((w >> 25) & 0x1Fu) - 1;
        if ((w & 0x40000000u) == 0) {
          if (flip >= 0) or_bits(set, o + flip, 1u, limit);
        } else {
          or_range(set, o, o + span, flip >= 0 ? o + flip : -1, limit);
        }
      }
    }
    carry += total;
  }
}

void launch_concise_or(const uint8_t* bm_base, const int64_t* d_off, const int32_t* d_len, const int32_t* d_target,
                       const int64_t* d_row0, int nbitmaps, uint32_t* const* d_sets, int64_t limit, hipStream_t s) {
  if (nbitmaps <= 0) return;
  hipLaunchKernelGGL(k_concise_or, dim3(nbitmaps), dim3(256), 0, s, bm_base, d_off, d_len, d_target, d_row0, d_sets,
                     limit);
}

// ------------------------------------------------------------------------------------------------
// Roaring (portable format, RoaringFormatSpec) -> dense row bitset (OR). One workgroup per bitmap;
// thread 0 walks the headers into LDS, then waves take containers round-robin.
// ------------------------------------------------------------------------------------------------
constexpr int kMaxContainers = 4096;

__device__ __forceinline__ uint32_t rd16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
__device__ __forceinline__ uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__global__ __launch_bounds__(256) void k_roaring_or(const uint8_t* __restrict__ base, const int64_t* __restrict__ off,
                                                    const int32_t* __restrict__ len, const int32_t* __restrict__ target,
                                                    uint32_t* const* __restrict__ sets, int32_t* __restrict__ err,
                                                    int64_t limit) {
  __shared__ int32_t s_key[kMaxContainers];
  __shared__ int32_t s_card[kMaxContainers];
  __shared__ int32_t s_off[kMaxContainers];
  __shared__ uint8_t s_run[kMaxContainers];
  __shared__ int32_t s_n;
  const int b = blockIdx.x;
  const uint8_t* p = base + off[b];
  const int nbytes = len[b];
  uint32_t* set = sets[target[b]];
  if (threadIdx.x == 0) {
    int n = 0;
    if (nbytes >= 4) {
      const uint32_t cookie = rd32(p);
      int pos = 4;
      const uint8_t* runbits = nullptr;
      bool has_off = true;
      bool ok = true;
      if ((cookie & 0xFFFFu) == 12347u) {
        n = (int)(cookie >> 16) + 1;
        runbits = p + pos;
        pos += (n + 7) / 8;
        has_off = n >= 4;
      } else if (cookie == 12346u) {
        n = (int)rd32(p + 4);
        pos = 8;
      } else {
        ok = false;
      }
      if (!ok || n > kMaxContainers || n < 0) {
        atomicOr(err, 2);
        n = 0;
      } else {
        const uint8_t* desc = p + pos;
        pos += 4 * n;
        const uint8_t* offs = has_off ? p + pos : nullptr;
        if (has_off) pos += 4 * n;
        int cur = pos;
        for (int c = 0; c < n; ++c) {
          s_key[c] = (int)rd16(desc + 4 * c);
          s_card[c] = (int)rd16(desc + 4 * c + 2) + 1;
          s_run[c] = runbits ? ((runbits[c >> 3] >> (c & 7)) & 1) : 0;
          const int start = offs ? (int)rd32(offs + 4 * c) : cur;
          s_off[c] = start;
          int sz;
          if (s_run[c]) sz = 2 + 4 * (int)rd16(p + start);
          else if (s_card[c] <= 4096) sz = 2 * s_card[c];
          else sz = 8192;
          cur = start + sz;
        }
      }
    }
    s_n = n;
  }
  __syncthreads();
  const int n = s_n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int c = wave; c < n; c += 4) {
    const int64_t row0 = (int64_t)s_key[c] << 16;
    const uint8_t* d = p + s_off[c];
    if (s_run[c]) {
      const int nruns = (int)rd16(d);
      for (int r = lane; r < nruns; r += 64) {
        const int64_t st = row0 + rd16(d + 2 + 4 * r);
        const int64_t ln = (int64_t)rd16(d + 4 + 4 * r) + 1;
        or_range(set, st, st + ln, -1, limit);
      }
    } else if (s_card[c] <= 4096) {
      for (int k = lane; k < s_card[c]; k += 64) {
        const int64_t row = row0 + rd16(d + 2 * k);
        if (row < limit) atomicOr(set + (row >> 5), 1u << (row & 31));
      }
    } else {
      uint32_t* dst = set + (row0 >> 5);
      for (int k = lane; k < 2048; k += 64) {
        const uint32_t w = rd32(d + 4 * k);
        if (w && row0 + 32ll * k < limit) atomicOr(dst + k, w);
      }
    }
  }
}

void launch_roaring_or(const uint8_t* bm_base, const int64_t* d_off, const int32_t* d_len, const int32_t* d_target,
                       int nbitmaps, uint32_t* const* d_sets, int32_t* d_err, int64_t limit, hipStream_t s) {
  if (nbitmaps <= 0) return;
  hipLaunchKernelGGL(k_roaring_or, dim3(nbitmaps), dim3(256), 0, s, bm_base, d_off, d_len, d_target, d_sets, d_err,
                     limit);
}

// ------------------------------------------------------------------------------------------------
// Filter program over dense bitsets (postfix): >= 0 push set i; -1 all; -2 none; -3 AND; -4 OR; -5 NOT.
// Rows >= nrows are kept clear (complement is within numRows, NotFilter.java:44-50).
// ------------------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_filter_eval(const int32_t* __restrict__ prog, int prog_len,
                                                     uint32_t* const* __restrict__ sets, uint32_t* __restrict__ out,
                                                     int64_t nrows, unsigned long long* __restrict__ count) {
  const int64_t nwords = (nrows + 31) >> 5;
  unsigned long long local = 0;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * blockDim.x) {
    uint32_t st[16];
    int sp = 0;
    const uint32_t valid = (w == nwords - 1 && (nrows & 31)) ? ((1u << (nrows & 31)) - 1u) : 0xFFFFFFFFu;
    for (int i = 0; i < prog_len; ++i) {
      const int c = prog[i];
      if (c >= 0) st[sp++] = sets[c][w];
      else if (c == -1) st[sp++] = valid;
      else if (c == -2) st[sp++] = 0u;
      else if (c == -3) { sp--; st[sp - 1] &= st[sp]; }
      else if (c == -4) { sp--; st[sp - 1] |= st[sp]; }
      else st[sp - 1] = ~st[sp - 1] & valid;
    }
    const uint32_t r = st[0] & valid;
    out[w] = r;
    local += __popc(r);
  }
  // wave reduce, the workgroup's waves in LDS, then one atomic per workgroup (a grid of at most 512:
  // thousands of atomics on one word serialise)
  __shared__ unsigned long long s_c[4];
  for (int o = 32; o > 0; o >>= 1) local += __shfl_down(local, o, 64);
  if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = local;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long c = s_c[0] + s_c[1] + s_c[2] + s_c[3];
    if (c) atomicAdd(count, c);
  }
}

// one Roaring container per wave (pieces of long bitmaps, split at attach): the container's rows are
// OR-ed exactly as k_roaring_or does for a whole bitmap
__global__ __launch_bounds__(256) void k_roaring_pieces(const uint8_t* __restrict__ base, const int64_t* __restrict__ off,
                                                        const int64_t* __restrict__ row0s, const int32_t* __restrict__ info,
                                                        const int32_t* __restrict__ target, int npieces,
                                                        uint32_t* const* __restrict__ sets, int64_t limit) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= npieces) return;
  const uint8_t* d = base + off[c];
  const int64_t row0 = row0s[c];
  const bool run = info[c] < 0;
  const int card = (info[c] & 0x7FFFFFFF) + 1;
  uint32_t* set = sets[target[c]];
  if (run) {
    const int nruns = (int)rd16(d);
    for (int r = lane; r < nruns; r += 64) {
      const int64_t st = row0 + rd16(d + 2 + 4 * r);
      const int64_t ln = (int64_t)rd16(d + 4 + 4 * r) + 1;
      or_range(set, st, st + ln, -1, limit);
    }
  } else if (card <= 4096) {
    for (int k = lane; k < card; k += 64) {
      const int64_t row = row0 + rd16(d + 2 * k);
      if (row < limit) atomicOr(set + (row >> 5), 1u << (row & 31));
    }
  } else {
    uint32_t* dst = set + (row0 >> 5);
    for (int k = lane; k < 2048; k += 64) {
      const uint32_t w = rd32(d + 4 * k);
      if (w && row0 + 32ll * k < limit) atomicOr(dst + k, w);
    }
  }
}

void launch_roaring_pieces(const uint8_t* bm_base, const int64_t* d_off, const int64_t* d_row0, const int32_t* d_info,
                           const int32_t* d_target, int npieces, uint32_t* const* d_sets, int64_t limit_bits,
                           hipStream_t s) {
  if (npieces <= 0) return;
  hipLaunchKernelGGL(k_roaring_pieces, dim3((npieces + 3) / 4), dim3(256), 0, s, bm_base, d_off, d_row0, d_info,
                     d_target, npieces, d_sets, limit_bits);
}

// ------------------------------------------------------------------------------------------------
// numeric post-filters: per-row predicate -> bitset words (FilteredOffset + ValueMatcher, see NumPred)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool in_sorted(const int64_t* set, int n, int64_t x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (set[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && set[lo] == x;
}

// Double.compare order as unsigned keys: -0.0 < 0.0, every NaN equal and greatest
__device__ __forceinline__ uint64_t dcmp_key(double d) { return d != d ? ~0ull : ord_key(d); }

// UnsignedBytes.lexicographicalComparator of String.valueOf(x) (ASCII) against a UTF-8 string
__device__ __forceinline__ int lex_cmp_long(int64_t x, const uint8_t* b, int blen) {
  char buf[20];
  int n = 0;
  uint64_t u = x < 0 ? (uint64_t)0 - (uint64_t)x : (uint64_t)x;
  do {
    buf[n++] = (char)('0' + (int)(u % 10));
    u /= 10;
  } while (u);
  const int len = n + (x < 0 ? 1 : 0);
  for (int i = 0; i < len && i < blen; ++i) {
    const int c = x < 0 ? (i == 0 ? '-' : buf[n - i]) : buf[n - 1 - i];
    if (c != b[i]) return c < (int)b[i] ? -1 : 1;
  }
  return (len > blen) - (len < blen);
}

__device__ __forceinline__ bool range_ok(int lc, int uc, const NumPred& p) {
  // lc = compare(value, lower), uc = compare(upper, value)
  const bool lok = !p.has_lo || (p.lo_strict ? lc > 0 : lc >= 0);
  const bool uok = !p.has_hi || (p.hi_strict ? uc > 0 : uc >= 0);
  return lok && uok;
}

__global__ __launch_bounds__(256) void k_num_pred(ColView v, ColView voff, int64_t nrows, NumPred p, uint32_t* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool m = false;
  if (r < nrows && p.kind != PRED_FALSE) {
    const uint8_t* ptr = cv_ptr(v, r);
    if (v.kind == VIEW_IDS && voff.kind != VIEW_ABSENT) {
      // a multi-value row matches when any of its values does; an empty row as the null value
      // (DimensionSelector value matchers over IndexedInts: size 0 -> predicate(null))
      const uint32_t b = load_id(voff, r), e = load_id(voff, r + 1);
      if (b == e) m = p.has_lo != 0;
      for (uint32_t k = b; k < e && !m; ++k) {
        const uint32_t id = load_id(v, k);
        m = ((uint64_t)p.set[id >> 6] >> (id & 63)) & 1ull;
      }
    } else if (v.kind == VIEW_IDS) {
      const uint32_t id = load_id(v, r);
      m = p.kind == PRED_ID_SET && ((uint64_t)p.set[id >> 6] >> (id & 63)) & 1ull;
    } else if (v.kind == VIEW_LONG) {
      const int64_t x = *reinterpret_cast<const int64_t*>(ptr);
      if (p.kind == PRED_LONG_RANGE) m = range_ok((x > p.lo) - (x < p.lo), (p.hi > x) - (p.hi < x), p);
      else if (p.kind == PRED_LONG_SET) m = in_sorted(p.set, p.nset, x);
      else if (p.kind == PRED_LONG_LEX) {
        const int lc = p.has_lo ? lex_cmp_long(x, p.lo_str, p.lo_len) : 1;
        const int uc = p.has_hi ? -lex_cmp_long(x, p.hi_str, p.hi_len) : 1;
        m = range_ok(lc, uc, p);
      }
    } else {
      int64_t bits;
      double d;
      if (v.kind == VIEW_FLOAT) {
        const float f = *reinterpret_cast<const float*>(ptr);
        bits = f != f ? 0x7fc00000ll : (int64_t)__float_as_uint(f);  // Float.floatToIntBits
        d = (double)f;
      } else {
        d = *reinterpret_cast<const double*>(ptr);
        bits = d != d ? 0x7ff8000000000000ll : (int64_t)__double_as_longlong(d);  // Double.doubleToLongBits
      }
      if (p.kind == PRED_BITS_SET) {
        m = in_sorted(p.set, p.nset, bits);
      } else if (p.kind == PRED_ORD_RANGE) {
        const uint64_t k = dcmp_key(d), klo = (uint64_t)p.lo, khi = (uint64_t)p.hi;
        m = range_ok((k > klo) - (k < klo), (khi > k) - (khi < k), p);
      }
    }
  }
  const uint64_t b = __ballot(m);
  const int lane = threadIdx.x & 63;
  const int64_t w = (r - lane) >> 5;  // first word of this wave's 64 rows
  if (r - lane < nrows) {
    if (lane == 0) out[w] = (uint32_t)b;
    if (lane == 32 && r < nrows) out[w + 1] = (uint32_t)(b >> 32);
  }
}

void launch_num_pred(ColView v, ColView voff, int64_t nrows, NumPred p, uint32_t* out, hipStream_t s) {
  if (nrows <= 0) return;
  hipLaunchKernelGGL(k_num_pred, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, s, v, voff, nrows, p, out);
}

void launch_filter_eval(const int32_t* d_prog, int prog_len, uint32_t* const* d_sets, uint32_t* out, int64_t nrows,
                        unsigned long long* d_count, hipStream_t s) {
  const int64_t nwords = (nrows + 31) >> 5;
  int grid = (int)((nwords + 255) / 256);
  if (grid > 512) grid = 512;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(k_filter_eval, dim3(grid), dim3(256), 0, s, d_prog, prog_len, d_sets, out, nrows, d_count);
}

// ------------------------------------------------------------------------------------------------
// accumulator init
// ------------------------------------------------------------------------------------------------
__global__ void k_fill_u64(uint64_t* __restrict__ p, int64_t rows, int slots, SlotInit init) {
  const int64_t n = rows * slots;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = init.v[i % slots];
}

void launch_fill_u64(uint64_t* p, int64_t rows, int slots, const SlotInit& init, hipStream_t s) {
  const int64_t n = rows * slots;
  if (n <= 0) return;
  int grid = (int)((n + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(k_fill_u64, dim3(grid), dim3(256), 0, s, p, rows, slots, init);
}

// ------------------------------------------------------------------------------------------------
// Scan + aggregate. One workgroup per tile of kTileRows rows of one segment; row r of the tile is
// handled by thread (r % 256) so every column read is coalesced.
//   TOPN == false: timeseries. Rows are time-sorted, so a tile touches few granularity buckets:
//     each thread keeps register partials for its current bucket and flushes them into LDS bins
//     (one bin per bucket touched by the tile), then the bins go to HBM with one atomic per
//     (bucket, aggregator) per tile.
//   TOPN == true: aggregate by dictionary id into the segment's dense [card][1 + naggs] table.
// Slot 0 of every record counts aggregated rows (skipEmptyBuckets / topN "touched" position).
// ------------------------------------------------------------------------------------------------
constexpr int kBins = 32;

__device__ __forceinline__ bool row_selected(const ScanJob& j, int64_t r, int64_t* bucket) {
  if (j.bitset && !((j.bitset[r >> 5] >> (r & 31)) & 1u)) return false;
  if (j.time.kind != VIEW_ABSENT) {
    const int64_t t = load_time(j.time, r);
    if (t < j.t_lo || t >= j.t_hi) return false;
    *bucket = j.period ? (bucket_coord(j.bounds, j.nbounds, t) - j.bucket0) / j.period : 0;
  } else {
    *bucket = 0;
  }
  return true;
}

template <bool TOPN>
__global__ __launch_bounds__(256) void k_scan_agg(const ScanJob* __restrict__ jobs, const int32_t* __restrict__ tile_job,
                                                  AggPlan plan) {
  __shared__ uint64_t s_bins[kBins][kMaxAggs + 1];
  __shared__ int64_t s_b0;
  const int tile = blockIdx.x;
  const ScanJob& j = jobs[tile_job[tile]];
  const int64_t row0 = (int64_t)(tile - j.tile_begin) * kTileRows;
  const int64_t row_end = min((int64_t)j.nrows, row0 + kTileRows);
  const int na = plan.n;
  // a tile whose filter bitset is empty selects nothing: one load of its 64 words, then done (a
  // selective filter leaves most tiles empty; the bits past the segment's last row only keep it)
  static_assert(kTileRows == 32 * 64 && kTileRows % 32 == 0, "one bitset word per thread of the first wave");
  if (j.bitset) {
    const int nw = (int)((row_end - row0 + 31) >> 5);
    const uint32_t w = (int)threadIdx.x < nw ? j.bitset[(row0 >> 5) + threadIdx.x] : 0u;
    if (!__syncthreads_or(w != 0u)) {
      if (!TOPN && j.part && (int)threadIdx.x <= na) {  // (an empty tile's record: identities)
        const int s = threadIdx.x;
        j.part[(size_t)(tile - j.tile_begin) * (na + 1) + s] = s == 0 ? 0ull : identity_of(plan.op[s - 1], plan.kind[s - 1]);
      }
      return;
    }
  }

  if (TOPN) {
    // topN over a multi-value dimension (PooledTopNAlgorithm.scanAndAggregate: every value of the
    // row's list aggregates the row, an empty list none): atomics into the [keys][1 + naggs] table
    const bool mv = j.key_off.kind != VIEW_ABSENT;
    for (int64_t r = row0 + threadIdx.x; r < row_end; r += 256) {
      int64_t b;
      if (!row_selected(j, r, &b)) continue;
      const uint32_t k0 = mv ? load_id(j.key_off, r) : 0u, k1 = mv ? load_id(j.key_off, r + 1) : 1u;
      for (uint32_t k = k0; k < k1; ++k) {
        const uint32_t id = mv ? load_id(j.key, k) : (j.key.kind == VIEW_IDS ? load_id(j.key, r) : 0u);
        const uint32_t key = j.key_card ? (uint32_t)b * (uint32_t)j.key_card + id : id;
        uint64_t* rec = j.out + (size_t)key * (na + 1);
        atomicAdd(reinterpret_cast<unsigned long long*>(rec), 1ull);
#pragma unroll
        for (int a = 0; a < kMaxAggs; ++a) {
          if (a < na) atomic_op(plan.op[a], rec + 1 + a, agg_in(j, plan, a, r));
        }
      }
    }
    return;
  }

  // timeseries
  // A tile of an unfiltered scan whose rows share one verdict and one bucket (no time needed, or a
  // uniform __time block: time_view) and whose every aggregator is folded by the decoders for the
  // tile's block (a tagged kViewFused block) or a plain count adds only its row count: no row is read.
  if (!j.bitset) {
    bool fast = j.time.kind == VIEW_ABSENT;
    if (!fast) {
      const int64_t tk = row0 >> j.time.log2_per;
      fast = (reinterpret_cast<uintptr_t>(j.time.blocks[tk]) & 1u) && tk == ((row_end - 1) >> j.time.log2_per);
    }
    for (int a = 0; a < na && fast; ++a) {
      if (plan.kind[a] == DG_AGG_COUNT && !j.agg_bits[a]) continue;
      const ColView& v = j.vals[a];
      const int64_t bk = row0 >> v.log2_per;
      fast = (v.pad & kViewFused) && (reinterpret_cast<uintptr_t>(v.blocks[bk]) & 1u) && bk == ((row_end - 1) >> v.log2_per);
    }
    if (fast) {
      if (threadIdx.x <= na) {
        int64_t b = 0;
        const bool sel = row_selected(j, row0, &b);  // (the whole tile's verdict and bucket)
        const int s = threadIdx.x;
        const uint64_t cnt = sel ? (uint64_t)(row_end - row0) : 0ull;
        const bool counts = s == 0 || plan.kind[s - 1] == DG_AGG_COUNT;
        if (j.part) {
          j.part[(size_t)(tile - j.tile_begin) * (na + 1) + s] =
              counts ? cnt : identity_of(plan.op[s - 1], plan.kind[s - 1]);
        } else if (sel && counts && b >= 0 && b < j.nbuckets) {
          atomicAdd(reinterpret_cast<unsigned long long*>(j.out + (size_t)b * (na + 1) + s), (unsigned long long)cnt);
        }
      }
      return;
    }
  }
  if (threadIdx.x == 0) {
    int64_t b0 = 0;
    if (j.period && j.time.kind != VIEW_ABSENT) {
      const int64_t t = load_time(j.time, row0);
      const int64_t v = bucket_coord(j.bounds, j.nbounds, t);
      b0 = v >= j.bucket0 ? (v - j.bucket0) / j.period : 0;
    }
    s_b0 = b0;
  }
  for (int i = threadIdx.x; i < kBins * (kMaxAggs + 1); i += 256) {
    const int bin = i / (kMaxAggs + 1), s = i % (kMaxAggs + 1);
    (void)bin;
    s_bins[i / (kMaxAggs + 1)][s] = s == 0 ? 0ull : (s - 1 < na ? identity_of(plan.op[s - 1], plan.kind[s - 1]) : 0ull);
  }
  __syncthreads();
  const int64_t b0 = s_b0;

  uint64_t acc[kMaxAggs];
  uint64_t cnt = 0;
  int64_t cur = -1;
  auto flush = [&](int64_t bucket) {
    if (bucket < 0 || cnt == 0) return;
    const int64_t lb = bucket - b0;
    if (lb >= 0 && lb < kBins) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&s_bins[lb][0]), (unsigned long long)cnt);
#pragma unroll
      for (int a = 0; a < kMaxAggs; ++a) {
        if (a < na) atomic_op(plan.op[a], &s_bins[lb][1 + a], acc[a]);
      }
    } else {
      uint64_t* rec = j.out + (size_t)bucket * (na + 1);
      atomicAdd(reinterpret_cast<unsigned long long*>(rec), (unsigned long long)cnt);
#pragma unroll
      for (int a = 0; a < kMaxAggs; ++a) {
        if (a < na) atomic_op(plan.op[a], rec + 1 + a, acc[a]);
      }
    }
  };
  for (int64_t r = row0 + threadIdx.x; r < row_end; r += 256) {
    int64_t b;
    if (!row_selected(j, r, &b)) continue;
    if (b != cur) {
      flush(cur);
      cur = b;
      cnt = 0;
#pragma unroll
      for (int a = 0; a < kMaxAggs; ++a) acc[a] = a < na ? identity_of(plan.op[a], plan.kind[a]) : 0ull;
    }
    cnt++;
#pragma unroll
    for (int a = 0; a < kMaxAggs; ++a) {
      if (a < na) acc[a] = combine_op(plan.op[a], acc[a], agg_in_scan(j, plan, a, r));
    }
  }
  flush(cur);
  __syncthreads();
  if (j.part) {  // one bucket: the tile's record, plain stores (k_scan_combine folds the tiles)
    if ((int)threadIdx.x <= na) j.part[(size_t)(tile - j.tile_begin) * (na + 1) + threadIdx.x] = s_bins[0][threadIdx.x];
    return;
  }
  for (int i = threadIdx.x; i < kBins * (na + 1); i += 256) {
    const int bin = i / (na + 1), s = i % (na + 1);
    const int64_t bucket = b0 + bin;
    if (bucket >= j.nbuckets || s_bins[bin][0] == 0) continue;
    uint64_t* rec = j.out + (size_t)bucket * (na + 1);
    if (s == 0) atomicAdd(reinterpret_cast<unsigned long long*>(rec), (unsigned long long)s_bins[bin][0]);
    else atomic_op(plan.op[s - 1], rec + s, s_bins[bin][s]);
  }
}

void launch_scan_agg(const ScanJob* d_jobs, const int32_t* d_tile_job, int ntiles, AggPlan plan, int topn, hipStream_t s) {
  if (ntiles <= 0) return;
  if (topn) hipLaunchKernelGGL(k_scan_agg<true>, dim3(ntiles), dim3(256), 0, s, d_jobs, d_tile_job, plan);
  else hipLaunchKernelGGL(k_scan_agg<false>, dim3(ntiles), dim3(256), 0, s, d_jobs, d_tile_job, plan);
}

// A one-bucket job's tile records folded slot by slot (each thread a strided run of tiles, then a wave
// tree, then the four waves in order) and combined into the record that may already hold the fused
// decoders' folds (TimeseriesBinaryFn / AggregatorFactory.combine: the slot's own combine op).
__global__ __launch_bounds__(256) void k_scan_combine(const ScanJob* __restrict__ jobs, AggPlan plan) {
  __shared__ uint64_t s_w[4];
  const ScanJob& j = jobs[blockIdx.x];
  if (!j.part) return;
  const int na = plan.n, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nt = (int)((j.nrows + kTileRows - 1) / kTileRows);
  for (int s = 0; s <= na; ++s) {
    const int op = s == 0 ? OP_ADD_I64 : plan.op[s - 1];
    const uint64_t id = s == 0 ? 0ull : identity_of(op, plan.kind[s - 1]);
    uint64_t acc = id;
    for (int t = threadIdx.x; t < nt; t += 256) acc = combine_op(op, acc, j.part[(size_t)t * (na + 1) + s]);
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t y = __shfl_down(acc, o, 64);
      acc = lane + o < 64 ? combine_op(op, acc, y) : acc;
    }
    if (lane == 0) s_w[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t v = s_w[0];
      for (int w = 1; w < 4; ++w) v = combine_op(op, v, s_w[w]);
      j.out[s] = combine_op(op, j.out[s], v);
    }
    __syncthreads();
  }
}

void launch_scan_combine(const ScanJob* d_jobs, int njobs, AggPlan plan, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(k_scan_combine, dim3(njobs), dim3(256), 0, s, d_jobs, plan);
}

// ------------------------------------------------------------------------------------------------
// topN aggregation, LDS-privatised by dictionary-id range (PooledTopNAlgorithm's per-id records,
// PooledTopNAlgorithm.java:661-719, held in LDS instead of a 1 GiB ByteBuffer). ScanJob.nbuckets
// carries the segment's cardinality.
// ------------------------------------------------------------------------------------------------
constexpr int kPartThreads = 1024;
constexpr int kPartUnroll = 4;

// rows of the quad that pass the bitset and the interval (bit k = row r + k)
__device__ __forceinline__ unsigned quad_selected(const ScanJob& j, int64_t r) {
  unsigned m = 0xF;
  if (j.bitset) m = (j.bitset[r >> 5] >> (r & 31)) & 0xF;
  if (m && j.time.kind != VIEW_ABSENT) {
    uint64_t t[4];
    load_time4(j.time, r, t);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((int64_t)t[k] < j.t_lo || (int64_t)t[k] >= j.t_hi) m &= ~(1u << k);
  }
  return m;
}

// workgroup (x = range * splits + split, y = segment): ids [range_lo, range_hi) of the segment,
// rows of one split; the range goes to partial table `split` with plain stores
__global__ __launch_bounds__(kPartThreads) void k_topn_part(const ScanJob* __restrict__ jobs, AggPlan plan, int64_t range,
                                                            int splits) {
  extern __shared__ uint64_t s_tab[];
  const ScanJob& j = jobs[blockIdx.y];
  const int64_t card = j.nbuckets;
  const int split = (int)(blockIdx.x % splits);
  const int64_t lo = (int64_t)(blockIdx.x / splits) * range;
  if (lo >= card) return;
  const int64_t hi = min(card, lo + range);
  const int na = plan.n, rec = na + 1;
  const int64_t nslots = (hi - lo) * rec;
  for (int64_t x = threadIdx.x; x < nslots; x += kPartThreads) {
    const int s = (int)(x % rec);
    s_tab[x] = s == 0 ? 0ull : identity_of(plan.op[s - 1], plan.kind[s - 1]);
  }
  __syncthreads();
  // rows of this split, in whole quads; kPartUnroll quads per thread are in flight at once
  const int64_t nrows = j.nrows;
  const int64_t nfull = nrows >> 2;  // quads without a ragged tail
  const int64_t nquads = (nrows + 3) >> 2;
  const int64_t qper = (nquads + splits - 1) / splits;
  const int64_t q0 = split * qper, q1 = min(nquads, q0 + qper), q1f = min(q1, nfull);
  for (int64_t qb = q0 + threadIdx.x; qb < q1f; qb += kPartThreads * kPartUnroll) {
    uint32_t id[kPartUnroll][4];
    unsigned m[kPartUnroll];
#pragma unroll
    for (int u = 0; u < kPartUnroll; ++u) {
      const int64_t q = qb + (int64_t)u * kPartThreads;
      m[u] = 0;
      if (q < q1f) {
        m[u] = quad_selected(j, q << 2);
        load_ids4(j.key, q << 2, id[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < kPartUnroll; ++u) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if ((int64_t)id[u][k] < lo || (int64_t)id[u][k] >= hi) m[u] &= ~(1u << k);
    }
#pragma unroll
    for (int u = 0; u < kPartUnroll; ++u) {
      if (!m[u]) continue;
      const int64_t r = (qb + (int64_t)u * kPartThreads) << 2;
      uint64_t* e[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        e[k] = s_tab + ((int64_t)id[u][k] - lo) * rec;
        if ((m[u] >> k) & 1) atomicAdd(reinterpret_cast<unsigned long long*>(e[k]), 1ull);
      }
      for (int a = 0; a < na; ++a) {  // one column at a time keeps four lanes of it in registers
        uint64_t raw[4] = {0, 0, 0, 0};
        const int vk = j.vals[a].kind;
        if (plan.kind[a] != DG_AGG_COUNT && vk != VIEW_ABSENT) load_raw4(j.vals[a], r, raw);
        const unsigned fm = agg_quad(j.agg_bits[a], r);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((m[u] >> k) & 1)
            atomic_op(plan.op[a], e[k] + 1 + a,
                      (fm >> k) & 1 ? agg_input_raw(plan.kind[a], vk, raw[k]) : identity_of(plan.op[a], plan.kind[a]));
      }
    }
  }
  if (q1 > nfull && threadIdx.x == 0) {  // the segment's ragged last quad
    for (int64_t rr = nfull << 2; rr < nrows; ++rr) {
      int64_t b;
      if (!row_selected(j, rr, &b)) continue;
      const int64_t id = (int64_t)load_id(j.key, rr);
      if (id < lo || id >= hi) continue;
      uint64_t* e = s_tab + (id - lo) * rec;
      atomicAdd(reinterpret_cast<unsigned long long*>(e), 1ull);
      for (int a = 0; a < na; ++a) atomic_op(plan.op[a], e + 1 + a, agg_in(j, plan, a, rr));
    }
  }
  __syncthreads();
  uint64_t* out = j.out + (size_t)split * (size_t)card * rec + lo * rec;
  for (int64_t x = threadIdx.x; x < nslots; x += kPartThreads) out[x] = s_tab[x];
}

// fold the split partial tables into table 0
__global__ __launch_bounds__(256) void k_topn_combine(const ScanJob* __restrict__ jobs, AggPlan plan, int splits) {
  const ScanJob& j = jobs[blockIdx.y];
  const int64_t card = j.nbuckets;
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (id >= card) return;
  const int rec = plan.n + 1;
  uint64_t* e = j.out + id * rec;
  uint64_t acc[kMaxAggs + 1];
#pragma unroll
  for (int a = 0; a <= kMaxAggs; ++a)
    if (a < rec) acc[a] = e[a];
  for (int s = 1; s < splits; ++s) {
    const uint64_t* f = j.out + ((size_t)s * card + id) * rec;
    acc[0] += f[0];
#pragma unroll
    for (int a = 0; a < kMaxAggs; ++a)
      if (a < plan.n) acc[1 + a] = combine_op(plan.op[a], acc[1 + a], f[1 + a]);
  }
#pragma unroll
  for (int a = 0; a <= kMaxAggs; ++a)
    if (a < rec) e[a] = acc[a];
}

int topn_part_splits(int64_t max_card, int naggs, int njobs) {
  const int64_t ranges = (max_card + topn_part_range(naggs) - 1) / topn_part_range(naggs);
  const int64_t groups = std::max<int64_t>(1, ranges * njobs);
  return (int)std::max<int64_t>(1, std::min<int64_t>(16, kPartTargetGroups / groups));
}

void launch_topn_part(const ScanJob* d_jobs, int njobs, int64_t max_card, AggPlan plan, int splits, hipStream_t s) {
  if (njobs <= 0 || max_card <= 0) return;
  const int64_t range = topn_part_range(plan.n);
  const int64_t ranges = (max_card + range - 1) / range;
  const dim3 grid((unsigned)(ranges * splits), (unsigned)njobs);
  const size_t lds = (size_t)std::min<int64_t>(range, max_card) * (plan.n + 1) * 8;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_topn_part),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, kPartLdsBytes);
  (void)attr;
  hipLaunchKernelGGL(k_topn_part, grid, dim3(kPartThreads), lds, s, d_jobs, plan, range, splits);
  if (splits > 1)
    hipLaunchKernelGGL(k_topn_combine, dim3((unsigned)((max_card + 255) / 256), (unsigned)njobs), dim3(256), 0, s,
                       d_jobs, plan, splits);
}

// ------------------------------------------------------------------------------------------------
// topN aggregation by dictionary-id bins (PooledTopNAlgorithm.scanAndAggregate,
// PooledTopNAlgorithm.java:438-719: one record per dictionary id). With ~7 rows per id (dimUniform)
// a workgroup's rows hit almost only distinct ids, so privatising per row tile buys nothing and
// per-row HBM atomics are slow. The rows are radix-partitioned once by id >> shift instead:
//   k_topn_bin_count    per tile: LDS histogram of selected rows per bin -> global bin counts
//   k_topn_bin_scan     exclusive scan of all bins (every segment's bins are consecutive)
//   k_topn_bin_scatter  per tile: recount, reserve one chunk per (tile, bin), write (id, inputs)
//   k_topn_bin_reduce   per bin: LDS table of its 2^shift records, streamed rows, plain stores
// Traffic per selected row: id read twice + inputs read once + (2 + 8 * naggs) B written and read.
// ScanJob.nbuckets carries the segment's cardinality.
// ------------------------------------------------------------------------------------------------
constexpr int kBinThreads = 256;
constexpr int kMaxTileBins = 4096;  // bins of one segment counted in LDS; above that, global atomics

// topN over granularity buckets (one cursor per bucket, TopNQueryEngine.java:80-104): the table key of
// a row is bucket * cardinality + dictionary id, so every bucket has its own per-id records
__device__ __forceinline__ uint32_t row_key(const ScanJob& j, int64_t r, int64_t b) {
  const uint32_t id = load_id(j.key, r);
  return j.key_card ? (uint32_t)b * (uint32_t)j.key_card + id : id;
}
// keys of rows r .. r + 3 (r % 4 == 0); rows outside the interval get garbage keys and stay masked
__device__ __forceinline__ void quad_keys(const ScanJob& j, int64_t r, uint32_t id[4]) {
  load_ids4(j.key, r, id);
  if (j.key_card) {
    uint64_t t[4];
    load_time4(j.time, r, t);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      id[k] += (uint32_t)((bucket_coord(j.bounds, j.nbounds, (int64_t)t[k]) - j.bucket0) / j.period) * (uint32_t)j.key_card;
  }
}

__device__ __forceinline__ bool tile_rows(const ScanJob& j, int t, int64_t* r0, int64_t* r1) {
  *r0 = (int64_t)(t - j.tile_begin) * kTileRows;
  *r1 = min((int64_t)j.nrows, *r0 + kTileRows);
  return *r0 < *r1;
}

__global__ __launch_bounds__(kBinThreads) void k_topn_bin_count(const ScanJob* __restrict__ jobs,
                                                                const int32_t* __restrict__ tile_job,
                                                                const int32_t* __restrict__ bin_first, int shift,
                                                                uint32_t* __restrict__ hist) {
  __shared__ uint32_t s_cnt[kMaxTileBins];
  const int seg = tile_job[blockIdx.x];
  const ScanJob& j = jobs[seg];
  const int nb = (int)((j.nbuckets + (1ll << shift) - 1) >> shift);
  const bool lds = nb <= kMaxTileBins;
  if (lds)
    for (int b = threadIdx.x; b < nb; b += kBinThreads) s_cnt[b] = 0;
  __syncthreads();
  uint32_t* h = hist + bin_first[seg];
  int64_t r0, r1;
  tile_rows(j, blockIdx.x, &r0, &r1);
  const int64_t full = r0 + ((r1 - r0) & ~3ll);
  for (int64_t r = r0 + 4 * threadIdx.x; r < full; r += 4 * kBinThreads) {
    const unsigned m = quad_selected(j, r);
    if (!m) continue;
    uint32_t id[4];
    quad_keys(j, r, id);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((m >> k) & 1) atomicAdd(lds ? &s_cnt[id[k] >> shift] : &h[id[k] >> shift], 1u);
  }
  if (threadIdx.x == 0)
    for (int64_t r = full; r < r1; ++r) {
      int64_t b;
      if (row_selected(j, r, &b)) {
        const uint32_t key = row_key(j, r, b);
        atomicAdd(lds ? &s_cnt[key >> shift] : &h[key >> shift], 1u);
      }
    }
  __syncthreads();
  if (lds)
    for (int b = threadIdx.x; b < nb; b += kBinThreads)
      if (s_cnt[b]) atomicAdd(&h[b], s_cnt[b]);
}

// one workgroup: base[b] = exclusive prefix of hist over all bins, cursor[b] = base[b]
__global__ __launch_bounds__(1024) void k_topn_bin_scan(const uint32_t* __restrict__ hist, uint32_t* __restrict__ base,
                                                        uint32_t* __restrict__ cursor, int nbins) {
  __shared__ int64_t s_tmp[16];
  __shared__ uint32_t s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (int c = 0; c < nbins; c += 1024) {
    const int b = c + threadIdx.x;
    const uint32_t v = b < nbins ? hist[b] : 0;
    int64_t tot;
    const uint32_t pre = (uint32_t)block_exclusive_scan(v, &tot, s_tmp) + s_carry;
    if (b < nbins) {
      base[b] = pre;
      cursor[b] = pre;
    }
    __syncthreads();
    if (threadIdx.x == 0) s_carry += (uint32_t)tot;
    __syncthreads();
  }
}

// Rows of one tile are counting-sorted by bin in LDS first, so that every bin's chunk of this tile
// goes out as consecutive lanes writing consecutive slots (coalesced), not as scattered 2- and
// 8-byte stores. Segments with more than kMaxSortBins bins take per-row global reservations.
constexpr int kMaxSortBins = 2048;
constexpr int kRowsPerThread = kTileRows / kBinThreads;  // 8 = two quads
static_assert(kRowsPerThread == 8, "tile = two quads per thread");

__global__ __launch_bounds__(kBinThreads) void k_topn_bin_scatter(const ScanJob* __restrict__ jobs,
                                                                  const int32_t* __restrict__ tile_job,
                                                                  const int32_t* __restrict__ bin_first, int shift,
                                                                  uint32_t* __restrict__ cursor, AggPlan plan,
                                                                  uint16_t* __restrict__ lid, uint64_t* __restrict__ vals,
                                                                  int64_t cap) {
  __shared__ uint32_t s_cnt[kMaxSortBins];   // counts, then tile-local starts
  __shared__ uint32_t s_goff[kMaxSortBins];  // reserved global offsets
  __shared__ uint32_t s_gpos[kTileRows];     // global slot of the k-th sorted row
  __shared__ uint64_t s_val[kTileRows];
  __shared__ uint16_t s_lid[kTileRows];
  __shared__ int64_t s_tmp[kBinThreads / 64];
  const int seg = tile_job[blockIdx.x];
  const ScanJob& j = jobs[seg];
  const int nb = (int)((j.nbuckets + (1ll << shift) - 1) >> shift);
  const uint32_t lmask = (1u << shift) - 1;
  uint32_t* cur = cursor + bin_first[seg];
  const int na = plan.n;
  int64_t r0, r1;
  tile_rows(j, blockIdx.x, &r0, &r1);
  const int64_t full = r0 + ((r1 - r0) & ~3ll);
  if (nb > kMaxSortBins) {  // huge dictionaries: per-row reservation
    for (int64_t r = r0 + threadIdx.x; r < r1; r += kBinThreads) {
      int64_t bb;
      if (!row_selected(j, r, &bb)) continue;
      const uint32_t id = row_key(j, r, bb);
      const uint32_t pos = atomicAdd(&cur[id >> shift], 1u);
      lid[pos] = (uint16_t)(id & lmask);
      for (int a = 0; a < na; ++a) vals[(size_t)a * cap + pos] = agg_in(j, plan, a, r);
    }
    return;
  }
  for (int b = threadIdx.x; b < nb; b += kBinThreads) s_cnt[b] = 0;
  __syncthreads();
  // pass 1: my two quads (rows r0 + 4 * (tid + 256 * u) ..): bin and rank within the tile's bin
  uint32_t id[2][4], rk[2][4];
  unsigned m[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int64_t r = r0 + 4 * (threadIdx.x + (int64_t)u * kBinThreads);
    m[u] = 0;
    if (r < full) {
      m[u] = quad_selected(j, r);
      if (m[u]) quad_keys(j, r, id[u]);
    } else if (r < r1) {  // the segment's ragged last quad
      for (int k = 0; k < 4 && r + k < r1; ++k) {
        int64_t bb;
        if (row_selected(j, r + k, &bb)) {
          m[u] |= 1u << k;
          id[u][k] = row_key(j, r + k, bb);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((m[u] >> k) & 1) rk[u][k] = atomicAdd(&s_cnt[id[u][k] >> shift], 1u);
  }
  __syncthreads();
  // tile-local starts (exclusive scan of the counts) + one global reservation per non-empty bin
  {
    const int per = (nb + kBinThreads - 1) / kBinThreads;
    const int b0 = threadIdx.x * per;
    uint32_t sum = 0;
    for (int q = 0; q < per; ++q)
      if (b0 + q < nb) sum += s_cnt[b0 + q];
    int64_t tot;
    uint32_t run = (uint32_t)block_exclusive_scan(sum, &tot, s_tmp);
    for (int q = 0; q < per; ++q) {
      const int b = b0 + q;
      if (b >= nb) break;
      const uint32_t c = s_cnt[b];
      s_goff[b] = c ? atomicAdd(&cur[b], c) : 0u;
      s_cnt[b] = run;
      run += c;
    }
  }
  __syncthreads();
  // pass 2: global slots and local ids into sorted order
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if ((m[u] >> k) & 1) {
        const uint32_t b = id[u][k] >> shift;
        const uint32_t p = s_cnt[b] + rk[u][k];
        s_gpos[p] = s_goff[b] + rk[u][k];
        s_lid[p] = (uint16_t)(id[u][k] & lmask);
      }
  __syncthreads();
  int ntile = 0;
#pragma unroll
  for (int u = 0; u < 2; ++u) ntile += __popc(m[u]);
  int64_t tot_sel;
  {
    int64_t t;
    block_exclusive_scan(ntile, &t, s_tmp);
    tot_sel = t;
  }
  for (int p = threadIdx.x; p < tot_sel; p += kBinThreads) lid[s_gpos[p]] = s_lid[p];
  // pass 3, per aggregator: inputs into sorted order, then coalesced stores
  for (int a = 0; a < na; ++a) {
    const int vk = j.vals[a].kind;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!m[u]) continue;
      const int64_t r = r0 + 4 * (threadIdx.x + (int64_t)u * kBinThreads);
      uint64_t in[4];
      if (r + 4 <= full) {
        uint64_t raw[4] = {0, 0, 0, 0};
        if (plan.kind[a] != DG_AGG_COUNT && vk != VIEW_ABSENT) load_raw4(j.vals[a], r, raw);
        const unsigned fm = agg_quad(j.agg_bits[a], r);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          in[k] = (fm >> k) & 1 ? agg_input_raw(plan.kind[a], vk, raw[k]) : identity_of(plan.op[a], plan.kind[a]);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) in[k] = ((m[u] >> k) & 1) ? agg_in(j, plan, a, r + k) : 0;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if ((m[u] >> k) & 1) s_val[s_cnt[id[u][k] >> shift] + rk[u][k]] = in[k];
    }
    __syncthreads();
    for (int p = threadIdx.x; p < tot_sel; p += kBinThreads) vals[(size_t)a * cap + s_gpos[p]] = s_val[p];
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBinThreads) void k_topn_bin_reduce(const ScanJob* __restrict__ jobs,
                                                                 const int32_t* __restrict__ bin_seg,
                                                                 const int32_t* __restrict__ bin_first, int shift,
                                                                 const uint32_t* __restrict__ base,
                                                                 const uint32_t* __restrict__ hist, AggPlan plan,
                                                                 const uint16_t* __restrict__ lid,
                                                                 const uint64_t* __restrict__ vals, int64_t cap) {
  extern __shared__ uint64_t s_tab[];
  const int gb = blockIdx.x, seg = bin_seg[gb];
  const ScanJob& j = jobs[seg];
  const int na = plan.n, rec = na + 1;
  const int64_t id0 = (int64_t)(gb - bin_first[seg]) << shift;
  const int64_t nid = min((int64_t)j.nbuckets - id0, 1ll << shift);
  const int nslots = (int)nid * rec;
  for (int x = threadIdx.x; x < nslots; x += kBinThreads) {
    const int sl = x % rec;
    s_tab[x] = sl == 0 ? 0ull : identity_of(plan.op[sl - 1], plan.kind[sl - 1]);
  }
  __syncthreads();
  const int64_t p0 = base[gb], p1 = p0 + hist[gb];
  for (int64_t p = p0 + threadIdx.x; p < p1; p += kBinThreads) {
    uint64_t* e = s_tab + (int)lid[p] * rec;
    atomicAdd(reinterpret_cast<unsigned long long*>(e), 1ull);
    for (int a = 0; a < na; ++a) atomic_op(plan.op[a], e + 1 + a, vals[(size_t)a * cap + p]);
  }
  __syncthreads();
  uint64_t* out = j.out + id0 * rec;
  for (int x = threadIdx.x; x < nslots; x += kBinThreads) out[x] = s_tab[x];
}

int topn_bin_shift(int naggs) {
  const int rec = naggs + 1;
  int shift = 10;
  while (shift > 6 && ((size_t)rec << shift) * 8 > 48 * 1024) shift--;
  return shift;
}

void launch_topn_bins(const ScanJob* d_jobs, const int32_t* d_tile_job, int ntiles, const int32_t* d_bin_first,
                      const int32_t* d_bin_seg, int nbins, int shift, uint32_t* d_hist, uint32_t* d_base,
                      uint32_t* d_cursor, AggPlan plan, uint16_t* d_lid, uint64_t* d_vals, int64_t cap, hipStream_t s) {
  if (ntiles <= 0 || nbins <= 0) return;
  hipLaunchKernelGGL(k_topn_bin_count, dim3(ntiles), dim3(kBinThreads), 0, s, d_jobs, d_tile_job, d_bin_first, shift,
                     d_hist);
  hipLaunchKernelGGL(k_topn_bin_scan, dim3(1), dim3(1024), 0, s, d_hist, d_base, d_cursor, nbins);
  hipLaunchKernelGGL(k_topn_bin_scatter, dim3(ntiles), dim3(kBinThreads), 0, s, d_jobs, d_tile_job, d_bin_first, shift,
                     d_cursor, plan, d_lid, d_vals, cap);
  const size_t lds = ((size_t)(plan.n + 1) << shift) * 8;
  hipLaunchKernelGGL(k_topn_bin_reduce, dim3(nbins), dim3(kBinThreads), lds, s, d_jobs, d_bin_seg, d_bin_first, shift,
                     d_base, d_hist, plan, d_lid, d_vals, cap);
}

// topN by a cached bin index (the dimension column's rows grouped by dictionary-id bin, built by the
// first topN over the column and kept with it): a query's bin reduce walks its bin's rows through the
// index instead of counting, scanning and scattering the rows again, and the dictionary ids need no
// decode. Same records as k_topn_bin_reduce (count + the aggregators' slots, identity-initialised,
// every id of the bin written); the inputs are gathered per row from the decoded metric columns.
//   k_tix_count / k_topn_bin_scan / k_tix_scatter   build: rows per bin, bin starts, rows by bin
//   k_topn_ix_reduce                                per bin: LDS table of its 2^shift ids, its rows
__global__ __launch_bounds__(256) void k_tix_count(const ScanJob* __restrict__ jobs, int seg, int shift, int nbins,
                                                   uint32_t* __restrict__ cnt) {
  const ScanJob& j = jobs[seg];
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < j.nrows; r += (int64_t)gridDim.x * 256) {
    const uint32_t b = load_id(j.key, r) >> shift;
    if (b < (uint32_t)nbins) atomicAdd(&cnt[b], 1u);  // (an id past the dictionary: not indexed)
  }
}
__global__ __launch_bounds__(256) void k_tix_scatter(const ScanJob* __restrict__ jobs, int seg, int shift, int nbins,
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ perm,
                                                     uint16_t* __restrict__ lid) {
  const ScanJob& j = jobs[seg];
  const uint32_t lmask = (1u << shift) - 1;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < j.nrows; r += (int64_t)gridDim.x * 256) {
    const uint32_t id = load_id(j.key, r);
    if ((id >> shift) >= (uint32_t)nbins) continue;
    const uint32_t pos = atomicAdd(&cursor[id >> shift], 1u);
    perm[pos] = (uint32_t)r;
    lid[pos] = (uint16_t)(id & lmask);
  }
}

// (dictionaries of at most kTixLdsBins bins: per workgroup of kTixRows rows, counts and ranks in LDS and
// one global atomic per (workgroup, bin) — the per-row global atomics above contend on a few hundred
// counters)
constexpr int kTixLdsBins = 4096;
constexpr int kTixPer = 16;                // rows per thread
constexpr int kTixRows = 256 * kTixPer;   // rows per workgroup
__global__ __launch_bounds__(256) void k_tix_count_lds(const ScanJob* __restrict__ jobs, int seg, int shift, int nbins,
                                                       uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s_cnt[kTixLdsBins];
  const ScanJob& j = jobs[seg];
  for (int b = threadIdx.x; b < nbins; b += 256) s_cnt[b] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kTixRows;
  for (int u = 0; u < kTixPer; ++u) {
    const int64_t r = r0 + u * 256 + threadIdx.x;
    if (r >= j.nrows) continue;
    const uint32_t b = load_id(j.key, r) >> shift;
    if (b < (uint32_t)nbins) atomicAdd(&s_cnt[b], 1u);  // (an id past the dictionary: not indexed)
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += 256)
    if (s_cnt[b]) atomicAdd(&cnt[b], s_cnt[b]);
}
__global__ __launch_bounds__(256) void k_tix_scatter_lds(const ScanJob* __restrict__ jobs, int seg, int shift, int nbins,
                                                         uint32_t* __restrict__ cursor, uint32_t* __restrict__ perm,
                                                         uint16_t* __restrict__ lid) {
  __shared__ uint32_t s_cnt[kTixLdsBins];  // counts, then this workgroup's first slot per bin
  const ScanJob& j = jobs[seg];
  const uint32_t lmask = (1u << shift) - 1;
  for (int b = threadIdx.x; b < nbins; b += 256) s_cnt[b] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kTixRows;
  uint32_t id[kTixPer], rk[kTixPer];
#pragma unroll
  for (int u = 0; u < kTixPer; ++u) {
    const int64_t r = r0 + u * 256 + threadIdx.x;
    id[u] = r < j.nrows ? load_id(j.key, r) : ~0u;
    rk[u] = (id[u] >> shift) < (uint32_t)nbins ? atomicAdd(&s_cnt[id[u] >> shift], 1u) : 0u;
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += 256)
    s_cnt[b] = s_cnt[b] ? atomicAdd(&cursor[b], s_cnt[b]) : 0u;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kTixPer; ++u) {
    const int64_t r = r0 + u * 256 + threadIdx.x;
    if (r >= j.nrows || (id[u] >> shift) >= (uint32_t)nbins) continue;
    const uint32_t pos = s_cnt[id[u] >> shift] + rk[u];
    perm[pos] = (uint32_t)r;
    lid[pos] = (uint16_t)(id[u] & lmask);
  }
}

void launch_topn_ix_build(const ScanJob* d_jobs, int seg, int64_t nrows, int shift, int nbins, uint32_t* d_cnt,
                          uint32_t* d_cursor, uint32_t* base, uint32_t* perm, uint16_t* lid, hipStream_t s) {
  if (nrows <= 0 || nbins <= 0) return;
  // (the scan runs over nbins + 1 counts, the last one zero: base[nbins] = the indexed rows, the end
  // of the last bin)
  if (nbins <= kTixLdsBins) {
    const unsigned grid = (unsigned)((nrows + kTixRows - 1) / kTixRows);
    hipLaunchKernelGGL(k_tix_count_lds, dim3(grid), dim3(256), 0, s, d_jobs, seg, shift, nbins, d_cnt);
    hipLaunchKernelGGL(k_topn_bin_scan, dim3(1), dim3(1024), 0, s, d_cnt, base, d_cursor, nbins + 1);
    hipLaunchKernelGGL(k_tix_scatter_lds, dim3(grid), dim3(256), 0, s, d_jobs, seg, shift, nbins, d_cursor, perm, lid);
    return;
  }
  const unsigned grid = (unsigned)std::min<int64_t>((nrows + 255) / 256, 2048);
  hipLaunchKernelGGL(k_tix_count, dim3(grid), dim3(256), 0, s, d_jobs, seg, shift, nbins, d_cnt);
  hipLaunchKernelGGL(k_topn_bin_scan, dim3(1), dim3(1024), 0, s, d_cnt, base, d_cursor, nbins + 1);
  hipLaunchKernelGGL(k_tix_scatter, dim3(grid), dim3(256), 0, s, d_jobs, seg, shift, nbins, d_cursor, perm, lid);
}

__global__ __launch_bounds__(kBinThreads) void k_topn_ix_reduce(const ScanJob* __restrict__ jobs,
                                                                const TopnIx* __restrict__ ixs,
                                                                const int32_t* __restrict__ bin_seg,
                                                                const int32_t* __restrict__ bin_first, int shift,
                                                                AggPlan plan) {
  extern __shared__ uint64_t s_tab[];
  const int gb = blockIdx.x, seg = bin_seg[gb];
  const ScanJob& j = jobs[seg];
  const TopnIx ix = ixs[seg];
  const int na = plan.n, rec = na + 1;
  const int b = gb - bin_first[seg];
  const int64_t id0 = (int64_t)b << shift;
  const int64_t nid = min((int64_t)j.nbuckets - id0, 1ll << shift);
  const int nslots = (int)nid * rec;
  for (int x = threadIdx.x; x < nslots; x += kBinThreads) {
    const int sl = x % rec;
    s_tab[x] = sl == 0 ? 0ull : identity_of(plan.op[sl - 1], plan.kind[sl - 1]);
  }
  __syncthreads();
  const int64_t p0 = ix.base[b], p1 = ix.base[b + 1];
  // kIxU rows per thread per round: their index entries, then their inputs, loaded together (each row's
  // gather waits on its index load; one round trip of each per round instead of per row)
  constexpr int kIxU = 4;
  for (int64_t pb = p0 + threadIdx.x; pb < p1; pb += kBinThreads * kIxU) {
    int64_t r[kIxU];
    int e_at[kIxU];
    bool ok[kIxU];
#pragma unroll
    for (int u = 0; u < kIxU; ++u) {
      const int64_t p = pb + u * kBinThreads;
      ok[u] = p < p1;
      r[u] = ok[u] ? (int64_t)ix.perm[p] : 0;
      e_at[u] = ok[u] ? (int)ix.lid[p] * rec : 0;
    }
#pragma unroll
    for (int u = 0; u < kIxU; ++u) {
      int64_t bb;
      ok[u] = ok[u] && row_selected(j, r[u], &bb);
      if (ok[u]) atomicAdd(reinterpret_cast<unsigned long long*>(s_tab + e_at[u]), 1ull);
    }
    for (int a = 0; a < na; ++a) {
      uint64_t v[kIxU];
#pragma unroll
      for (int u = 0; u < kIxU; ++u) v[u] = ok[u] ? agg_in(j, plan, a, r[u]) : 0ull;
#pragma unroll
      for (int u = 0; u < kIxU; ++u)
        if (ok[u]) atomic_op(plan.op[a], s_tab + e_at[u] + 1 + a, v[u]);
    }
  }
  __syncthreads();
  uint64_t* out = j.out + id0 * rec;
  for (int x = threadIdx.x; x < nslots; x += kBinThreads) out[x] = s_tab[x];
}

void launch_topn_ix_reduce(const ScanJob* d_jobs, const TopnIx* d_ix, const int32_t* d_bin_first,
                           const int32_t* d_bin_seg, int nbins, int shift, AggPlan plan, hipStream_t s) {
  if (nbins <= 0) return;
  const size_t lds = ((size_t)(plan.n + 1) << shift) * 8;
  hipLaunchKernelGGL(k_topn_ix_reduce, dim3(nbins), dim3(kBinThreads), lds, s, d_jobs, d_ix, d_bin_seg, d_bin_first,
                     shift, plan);
}

// ------------------------------------------------------------------------------------------------
// topN selection for one segment: the K-th largest metric key among touched ids (8-bit radix
// select over the ordered key), then the ids whose key >= that K-th key, compacted in id order.
// The host replays TopNNumericResultBuilder's priority queue over those candidates only (ids with a
// smaller key can never survive it, whatever the insertion order).
// Metric keys realise the factory comparators: Long.compare, Double.compare / Float.compare
// (NaN greatest, -0.0 < 0.0); inverted flips them.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t metric_key(uint64_t slot, int op, int kind, int inverted) {
  uint64_t k;
  if (op == OP_ADD_I64) {
    k = slot ^ kSign;
  } else if (op == OP_ADD_F64) {
    double d = __longlong_as_double((long long)slot);
    if (kind == DG_AGG_FLOAT_SUM) d = (double)(float)d;
    k = d != d ? ~0ull : ord_key(d);
  } else if (kind == DG_AGG_LONG_MIN || kind == DG_AGG_LONG_MAX) {
    k = slot;  // biased signed already ordered
  } else {
    // min/max key: decode (NaN encodings 0 / ~0) and re-key with NaN greatest
    bool nan = (op == OP_MIN_U64) ? slot == 0 : slot == ~0ull;
    if (nan) k = ~0ull;
    else {
      double d = unord_key(slot);
      if (kind == DG_AGG_FLOAT_MIN || kind == DG_AGG_FLOAT_MAX) d = (double)(float)d;
      k = ord_key(d);
    }
  }
  return inverted ? ~k : k;
}

// One level of the radix digit choice from its histogram (wave-parallel: 64 lanes x 4 bins, descending
// digit order) on a running choice (prefix, mask, keys still to take); returns whether the chosen
// bucket is needed whole (its count = the keys still to take: exactly `threshold` keys are then >= the
// prefix with zero low bits, so that is the K-th key bound and the deeper levels are not needed).
// Called by one full wave.
__device__ bool replay_one(const uint32_t* __restrict__ hist, int q, uint64_t* prefix, uint64_t* mask, int64_t* krem) {
  const int lane = threadIdx.x & 63;
  const int shift = 56 - 8 * q;
  int64_t h[4], sum = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = hist[q * 256 + 255 - (lane * 4 + j)];
    sum += h[j];
  }
  int64_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  const int64_t excl = incl - sum;
  const bool hit = excl < *krem && incl >= *krem;
  const unsigned long long bm = __ballot(hit);
  int digit = 0, whole = 0;
  int64_t nk = *krem;
  if (hit) {
    int64_t cum = excl;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (cum + h[j] >= *krem) {
        digit = 255 - (lane * 4 + j);
        nk = *krem - cum;
        whole = h[j] == nk;
        break;
      }
      cum += h[j];
    }
  }
  if (bm) {
    const int src = __ffsll((long long)bm) - 1;
    digit = __shfl(digit, src, 64);
    nk = __shfl(nk, src, 64);
    whole = __shfl(whole, src, 64);
  }
  *prefix |= (uint64_t)digit << shift;
  *mask |= 255ull << shift;
  *krem = nk;
  return whole != 0;
}

// the radix choice after `level` levels: entry level - 1 of jb.rstate (written by the previous level's
// kernel) plus one replayed histogram; workgroup 0 stores it as entry `level` for the next kernel.
// Called by one full wave; returns whether the choice is final.
__device__ bool radix_state(const TopnSelJob& jb, int level, int threshold, uint64_t* p_out, uint64_t* m_out) {
  uint64_t p = 0, m = 0;
  int64_t krem = threshold;
  bool done = false;
  if (level > 1) {
    const uint64_t* sa = jb.rstate + 4 * (level - 1);
    p = sa[0];
    m = sa[1];
    krem = (int64_t)sa[2];
    done = sa[3] != 0;
  }
  if (!done) done = replay_one(jb.hist, level - 1, &p, &m, &krem);
  if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && level < 8) {
    uint64_t* sb = jb.rstate + 4 * level;
    sb[0] = p;
    sb[1] = m;
    sb[2] = (uint64_t)krem;
    sb[3] = done ? 1ull : 0ull;
  }
  *p_out = p;
  *m_out = m;
  return done;
}

// DimensionTopNMetricSpec key of a touched id: smaller dictionary rank = larger key; 0 = not eligible
// (outside the computeStartEnd id range, BaseTopNAlgorithm.java:296-326, or not after previousStop,
// TopNLexicographicResultBuilder.shouldAdd :166-174)
__device__ __forceinline__ uint64_t dim_key(const TopnSelJob& jb, int64_t id) {
  const int32_t r = jb.rank ? jb.rank[id] : 0;
  if (id < jb.lo || id >= jb.hi || r < jb.min_rank) return 0;
  return (uint64_t)(0xFFFFFFFFu - (uint32_t)r) + 1ull;
}

// pass 0: metric keys, touched / row counts, histogram of the top byte
__global__ __launch_bounds__(kSelBlock) void k_topn_keys(const TopnSelJob* __restrict__ jobs, int naggs, int metric,
                                                         int op, int kind, int inverted) {
  __shared__ unsigned int s_hist[256];
  __shared__ unsigned long long s_c, s_rows;
  const TopnSelJob& jb = jobs[blockIdx.y];
  const int64_t i = (int64_t)blockIdx.x * kSelBlock + threadIdx.x;
  if ((int64_t)blockIdx.x * kSelBlock >= jb.card) return;
  if (threadIdx.x < 256) s_hist[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    s_c = 0;
    s_rows = 0;
  }
  __syncthreads();
  const int rec = naggs + 1;
  unsigned long long c = 0, rows = 0;
  if (i < jb.card) {
    const uint64_t n = jb.table[i * rec];
    uint64_t k = 0;
    if (n) {
      if (jb.dim_mode) {
        k = dim_key(jb, i);
      } else {
        k = metric_key(jb.table[i * rec + 1 + metric], op, kind, inverted);
        k = k ? k : 1;  // 0 marks untouched ids; a touched key of 0 becomes 1 (only widens the candidates)
      }
      if (k) atomicAdd(&s_hist[k >> 56], 1u);
    }
    jb.keys[i] = k;
    c = k != 0;
    rows = n;
  }
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_down(c, o, 64);
    rows += __shfl_down(rows, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&s_c, c);
    atomicAdd(&s_rows, rows);
  }
  __syncthreads();
  if (threadIdx.x < 256 && s_hist[threadIdx.x]) atomicAdd(&jb.hist[threadIdx.x], s_hist[threadIdx.x]);
  if (threadIdx.x == 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(&jb.state[2]), s_c);
    atomicAdd(reinterpret_cast<unsigned long long*>(&jb.state[1]), s_rows);
  }
}

// pass `level` (1..7): histogram of byte (56 - 8 level) among keys matching the chosen prefix
__global__ __launch_bounds__(kSelBlock) void k_topn_radix(const TopnSelJob* __restrict__ jobs, int level, int threshold) {
  __shared__ unsigned int s_hist[256];
  __shared__ uint64_t s_prefix, s_mask;
  __shared__ int s_used;
  const TopnSelJob& jb = jobs[blockIdx.y];
  if ((int64_t)blockIdx.x * kSelBlock >= jb.card) return;
  if ((int64_t)jb.state[2] <= threshold) return;  // everything touched is a candidate
  if (threadIdx.x < 64) {
    uint64_t p, m;
    const bool done = radix_state(jb, level, threshold, &p, &m);
    if (threadIdx.x == 0) {
      s_prefix = p;
      s_mask = m;
      s_used = done ? 0 : level;
    }
  }
  if (threadIdx.x < 256) s_hist[threadIdx.x] = 0;
  __syncthreads();
  if (s_used < level) return;  // the bound is final (a bucket taken whole): no deeper histogram
  const int64_t i = (int64_t)blockIdx.x * kSelBlock + threadIdx.x;
  const int shift = 56 - 8 * level;
  if (i < jb.card) {
    const uint64_t k = jb.keys[i];
    if (k && (k & s_mask) == s_prefix) atomicAdd(&s_hist[(k >> shift) & 255], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 256 && s_hist[threadIdx.x]) atomicAdd(&jb.hist[level * 256 + threadIdx.x], s_hist[threadIdx.x]);
}

__device__ __forceinline__ uint64_t sel_kth(const TopnSelJob& jb, int threshold, uint64_t* s_kth) {
  if (threadIdx.x < 64) {
    uint64_t p = 0, m = 0;
    if ((int64_t)jb.state[2] > threshold) radix_state(jb, 8, threshold, &p, &m);  // levels 0..6 stored, 7 replayed
    if (threadIdx.x == 0) *s_kth = p;
  }
  __syncthreads();
  return *s_kth;
}

// candidates per workgroup
__global__ __launch_bounds__(kSelBlock) void k_topn_count(const TopnSelJob* __restrict__ jobs, int threshold) {
  __shared__ uint64_t s_kth;
  __shared__ int s_n;
  const TopnSelJob& jb = jobs[blockIdx.y];
  if ((int64_t)blockIdx.x * kSelBlock >= jb.card) return;
  const uint64_t kth = sel_kth(jb, threshold, &s_kth);
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kSelBlock + threadIdx.x;
  int f = 0;
  if (i < jb.card) {
    const uint64_t k = jb.keys[i];
    f = k != 0 && k >= kth;
  }
  const unsigned long long m = __ballot(f);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(&s_n, __popcll(m));
  __syncthreads();
  if (threadIdx.x == 0) jb.blkcnt[blockIdx.x] = s_n;
}

// ordered compaction of the candidates + gather of their records
__global__ __launch_bounds__(kSelBlock) void k_topn_compact(const TopnSelJob* __restrict__ jobs, int naggs, int threshold) {
  __shared__ uint64_t s_kth;
  __shared__ int s_wave[kSelBlock / 64];
  __shared__ long long s_base, s_total;
  const TopnSelJob& jb = jobs[blockIdx.y];
  if ((int64_t)blockIdx.x * kSelBlock >= jb.card) return;
  const uint64_t kth = sel_kth(jb, threshold, &s_kth);
  const int nblk = (int)((jb.card + kSelBlock - 1) / kSelBlock);
  if (threadIdx.x < 64) {
    long long before = 0, total = 0;
    for (int b = threadIdx.x; b < nblk; b += 64) {
      const int c = jb.blkcnt[b];
      total += c;
      before += b < (int)blockIdx.x ? c : 0;
    }
    for (int o = 32; o > 0; o >>= 1) {
      before += __shfl_down(before, o, 64);
      total += __shfl_down(total, o, 64);
    }
    if (threadIdx.x == 0) {
      s_base = before;
      s_total = total;
    }
  }
  const int64_t i = (int64_t)blockIdx.x * kSelBlock + threadIdx.x;
  int f = 0;
  if (i < jb.card) {
    const uint64_t k = jb.keys[i];
    f = k != 0 && k >= kth;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long m = __ballot(f);
  if (lane == 0) s_wave[wave] = __popcll(m);
  __syncthreads();
  if (f) {
    long long pos = s_base + __popcll(m & ((1ull << lane) - 1ull));
    for (int w = 0; w < wave; ++w) pos += s_wave[w];
    jb.cand[pos] = (int32_t)i;
    if (pos < jb.gather_cap) {  // read-back record: [id, rec slots]
      const int rec = naggs + 1;
      jb.gathered[pos * (rec + 1)] = (uint64_t)i;
      for (int c = 0; c < rec; ++c) jb.gathered[pos * (rec + 1) + 1 + c] = jb.table[i * rec + c];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *jb.ncand = (int32_t)(s_total < 0x7fffffff ? s_total : 0x7fffffff);
    jb.state[0] = kth;
  }
}

// Final ordering of one segment's gathered candidates (TopNNumericResultBuilder.build order:
// metric descending, then dimension value = dictionary id ascending), one workgroup per segment:
// order[k] = gather position of the k-th entry. Bitonic sort in LDS; skipped (order untouched)
// when the candidates exceed kOrderCap (the host sorts then).
constexpr int kOrderCap = 4096;
__global__ __launch_bounds__(1024) void k_topn_order(const TopnSelJob* __restrict__ jobs, int naggs, int metric, int op,
                                                     int kind, int inverted) {
  __shared__ uint64_t s_key[kOrderCap];
  __shared__ uint16_t s_pos[kOrderCap];
  const TopnSelJob& jb = jobs[blockIdx.x];
  const int n = *jb.ncand;
  if (n > kOrderCap || n > jb.gather_cap || n <= 0) return;  // the host replays in id order then
  int P = 1;
  while (P < n) P <<= 1;
  const int rec = naggs + 1;
  auto key_of = [&](int c) {
    const uint64_t* g = jb.gathered + (size_t)c * (rec + 1);
    return c >= n ? 0ull : jb.dim_mode ? dim_key(jb, (int64_t)g[0]) : metric_key(g[1 + 1 + metric], op, kind, inverted);
  };
  if (P <= 1024) {
    // one element per thread: the compare-exchange stages of stride < 64 between the lanes of a
    // wave (shuffles, no barrier), the wider ones through LDS (45 of the 55 stages of P = 1024 stay
    // in registers). Threads >= P pair among themselves (c ^ stride >= P) and are never written.
    const int c = threadIdx.x;
    uint64_t k = c < P ? key_of(c) : 0ull;
    int pos = c;
    for (int size = 2; size <= P; size <<= 1) {
      const bool up = (c & size) == 0;
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        uint64_t ko;
        int po;
        if (stride >= 64) {
          s_key[c] = k;
          s_pos[c] = (uint16_t)pos;
          __syncthreads();
          ko = s_key[c ^ stride];
          po = s_pos[c ^ stride];
          __syncthreads();
        } else {
          ko = __shfl_xor((unsigned long long)k, stride, 64);
          po = __shfl_xor(pos, stride, 64);
        }
        // the same network as below: the lower index of a pair keeps the element that comes first
        // (larger key, or equal key and smaller position) when `up`, the other one otherwise
        const bool lower = (c & stride) == 0;
        const bool mine_first = k != ko ? k > ko : pos < po;
        if (mine_first != (lower == up)) {
          k = ko;
          pos = po;
        }
      }
    }
    s_pos[c] = (uint16_t)pos;
    __syncthreads();
  } else {
  for (int c = threadIdx.x; c < P; c += 1024) {
    s_key[c] = key_of(c);
    s_pos[c] = (uint16_t)c;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int c = threadIdx.x; c < P; c += 1024) {
        const int o = c ^ stride;
        if (o > c) {
          const uint64_t ka = s_key[c], kb = s_key[o];
          const uint16_t pa = s_pos[c], pb = s_pos[o];
          // a precedes b: larger key, or equal key and smaller position (a padding slot has key 0
          // and position >= n, so it sorts last)
          const bool a_first = ka != kb ? ka > kb : pa < pb;
          const bool up = (c & size) == 0;
          if (a_first != up) {
            s_key[c] = kb;
            s_key[o] = ka;
            s_pos[c] = pb;
            s_pos[o] = pa;
          }
        }
      }
      __syncthreads();
    }
  }
  }
  for (int c = threadIdx.x; c < n; c += 1024) jb.order[c] = s_pos[c];
  // the gathered records permuted into that order, in place, one record word at a time (every
  // read of the word before the barrier, every write after it): the host reads its lists in order
  const int rw = rec + 1;
  for (int w = 0; w < rw; ++w) {
    uint64_t v[kOrderCap / 1024];
#pragma unroll
    for (int j = 0; j < kOrderCap / 1024; ++j) {
      const int c = threadIdx.x + j * 1024;
      v[j] = c < n ? jb.gathered[(size_t)s_pos[c] * rw + w] : 0ull;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kOrderCap / 1024; ++j) {
      const int c = threadIdx.x + j * 1024;
      if (c < n) jb.gathered[(size_t)c * rw + w] = v[j];
    }
  }
}

void launch_topn_select(const TopnSelJob* d_jobs, int njobs, int64_t max_card, int naggs, int metric, int metric_op,
                        int inverted, int threshold, hipStream_t s) {
  if (njobs <= 0 || max_card <= 0) return;
  const dim3 grid((unsigned)((max_card + kSelBlock - 1) / kSelBlock), (unsigned)njobs);
  // metric_op encodes (op << 8) | kind
  hipLaunchKernelGGL(k_topn_keys, grid, dim3(kSelBlock), 0, s, d_jobs, naggs, metric, metric_op >> 8, metric_op & 255,
                     inverted);
  for (int level = 1; level < 8; ++level)
    hipLaunchKernelGGL(k_topn_radix, grid, dim3(kSelBlock), 0, s, d_jobs, level, threshold);
  hipLaunchKernelGGL(k_topn_count, grid, dim3(kSelBlock), 0, s, d_jobs, threshold);
  hipLaunchKernelGGL(k_topn_compact, grid, dim3(kSelBlock), 0, s, d_jobs, naggs, threshold);
  hipLaunchKernelGGL(k_topn_order, dim3((unsigned)njobs), dim3(1024), 0, s, d_jobs, naggs, metric, metric_op >> 8,
                     metric_op & 255, inverted);
}

// ------------------------------------------------------------------------------------------------
// DELTA / TABLE long blocks -> int64 (CompressionFactory.LongEncodingFormat, CompressionFactory.java:153-188)
// Values are packed MSB-first at `bits` bits (VSizeLongSerde.java:416-657: Size1Des..Size64Des all read
// the same big-endian bit stream). One 256-thread workgroup expands a chunk of 2048 rows: the chunk's
// 256 * bits packed bytes are staged into LDS with coalesced dword loads, every thread then cuts its
// values out of a 96-bit big-endian window and stores int64 rows with consecutive lanes on
// consecutive rows. DELTA adds the base (DeltaLongEncodingReader.read, :63-66); TABLE looks the id up
// in the LDS copy of the table (TableLongEncodingReader.read, :69-72; an id past the table is a
// malformed segment -> error word).
// ------------------------------------------------------------------------------------------------
constexpr int kVsRows = 2048;

__global__ __launch_bounds__(256) void k_vsize_expand(const VsJob* __restrict__ jobs, int32_t* __restrict__ err) {
  __shared__ uint32_t lds[kVsRows * 64 / 32 + 4];
  __shared__ int64_t tab[256];
  const VsJob j = jobs[blockIdx.y];
  const int64_t r0 = (int64_t)blockIdx.x * kVsRows;
  if (r0 >= j.rows) return;
  const int n = (int)min<int64_t>(kVsRows, j.rows - r0);
  const int bits = j.bits;
  const int tid = threadIdx.x;
  // chunk start is r0 * bits / 8 = blockIdx.x * 256 * bits bytes: dword aligned
  const uint32_t* src = reinterpret_cast<const uint32_t*>(j.src + (size_t)blockIdx.x * 256 * bits);
  const int nbytes = (n * bits + 7) >> 3;  // packed bytes of this chunk (the 4 closing bytes follow)
  const int ndw = (nbytes + 3) >> 2;
  for (int q = tid; q < ndw; q += 256) lds[q] = src[q];
  if (tid < 4) lds[ndw + tid] = 0;
  const bool is_table = j.table != nullptr;
  if (is_table)
    for (int t = tid; t < j.table_n; t += 256) tab[t] = j.table[t];
  __syncthreads();
  int64_t* dst = j.dst + r0;
  bool bad = false;
  for (int i = tid; i < n; i += 256) {
    const int64_t o = (int64_t)i * bits;
    const int byte = (int)(o >> 3);
    const int q = byte >> 2;
    const int start = ((byte & 3) << 3) + (int)(o & 7);  // <= 31
    const uint64_t hi = ((uint64_t)__builtin_bswap32(lds[q]) << 32) | __builtin_bswap32(lds[q + 1]);
    const uint32_t lo = __builtin_bswap32(lds[q + 2]);
    const unsigned __int128 w = (((unsigned __int128)hi << 32) | lo) << (32 + start);
    const uint64_t v = (uint64_t)(w >> (128 - bits));
    int64_t out;
    if (is_table) {
      if (v >= (uint64_t)j.table_n) {
        bad = true;
        out = 0;
      } else {
        out = tab[v];
      }
    } else {
      out = (int64_t)((uint64_t)j.base + v);
    }
    dst[i] = out;
  }
  if (bad) atomicOr(err, 1);
}

void launch_vsize_expand(const VsJob* d_jobs, int njobs, int32_t max_rows, int32_t* d_err, hipStream_t s) {
  if (njobs <= 0 || max_rows <= 0) return;
  const unsigned gx = (unsigned)((max_rows + kVsRows - 1) / kVsRows);
  hipLaunchKernelGGL(k_vsize_expand, dim3(gx, (unsigned)njobs), dim3(256), 0, s, d_jobs, d_err);
}

// ------------------------------------------------------------------------------------------------
// Multi-value row lists, checked once decoded (the reference would fail on them with an
// IndexOutOfBounds from SliceIndexedInts / the dictionary): offsets[0] == 0, non-decreasing,
// offsets[rows] <= values, and every value id < the dictionary's cardinality. A bad list sets bit 2
// of the call's error word (DG_ERR_FORMAT at the call's synchronisation) before any kernel reads it.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_mv_check(const MvCheck* __restrict__ jobs, int32_t* __restrict__ err) {
  const MvCheck j = jobs[blockIdx.y];
  bool bad = false;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < j.rows; r += stride) {
    const uint32_t a = load_id(j.offs, r), b = load_id(j.offs, r + 1);
    bad |= b < a || (r == 0 && a != 0) || (r + 1 == j.rows && (int64_t)b > j.nvals);
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < j.nvals; i += stride)
    bad |= (int64_t)load_id(j.vals, i) >= (int64_t)j.card;
  if (__syncthreads_or(bad) && threadIdx.x == 0) atomicOr(err, 4);
}

void launch_mv_check(const MvCheck* d_jobs, int njobs, int32_t* d_err, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(k_mv_check, dim3(256, (unsigned)njobs), dim3(256), 0, s, d_jobs, d_err);
}

// ------------------------------------------------------------------------------------------------
// LZF blocks (CompressionStrategy.LZF, id 0x00 / LZF_VERSION columns): compress-lzf 1.0.4's chunk
// stream ("ZV" + type 0 raw | type 1 liblzf, ChunkDecoder.decodeChunk). One wave per block: the
// compressed block is staged into LDS with coalesced dword loads, the wave walks the tokens in
// lockstep (every lane reads the same LDS token bytes, so control flow stays uniform; the input is
// staged through an 8 KiB LDS window so two workgroups fit a CU) and copies
// literal runs and back-references lane-parallel into an LDS output image (an overlapping reference
// is the periodic extension of its last `dist` bytes, copied in one pass), which is then
// written out with 16-byte stores. A malformed stream sets the error word.
// ------------------------------------------------------------------------------------------------
constexpr int kLzfWin = 8192;  // staged input window: 64 KiB output + 8 KiB input -> two workgroups per CU

__global__ __launch_bounds__(64) void k_lzf_decode(const LzfJob* __restrict__ jobs, int32_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) uint8_t outb[kBlockBytes + 16];
  __shared__ __attribute__((aligned(16))) uint32_t win[kLzfWin / 4 + 4];
  const LzfJob j = jobs[blockIdx.x];
  const int lane = threadIdx.x;
  const int n = j.src_len;
  const uint8_t* winb = reinterpret_cast<const uint8_t*>(win);
  int wb = 0, we = 0;  // window = input bytes [wb, we), wb 4-byte aligned (src is 16-byte aligned)
  // (re)stage the window at ip when fewer than 48 bytes (chunk header, longest token + literals) remain
  auto refill = [&](int ip) {
    if (ip + 48 <= we || we >= n) return;
    __syncthreads();
    wb = ip & ~3;
    we = min(n, wb + kLzfWin);
    const int ndw = (we - wb + 3) >> 2;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(j.src + wb);
    const int full = (n - wb) >> 2;  // whole dwords inside the block
    for (int q = lane; q < ndw; q += 64) {
      uint32_t v;
      if (q < full) {
        v = src[q];
      } else {
        v = 0;
        for (int b = 0; b < 4 && wb + 4 * q + b < n; ++b) v |= (uint32_t)j.src[wb + 4 * q + b] << (8 * b);
      }
      win[q] = v;
    }
    if (lane < 4) win[ndw + lane] = 0;
    __syncthreads();
  };
  auto in8 = [&](int x) -> int { return winb[x - wb]; };
  int ip = 0, op = 0;
  bool bad = false;
  while (ip < n && !bad) {
    refill(ip);
    if (ip + 5 > n || in8(ip) != 'Z' || in8(ip + 1) != 'V') {
      bad = true;
      break;
    }
    const int type = __builtin_amdgcn_readfirstlane(in8(ip + 2));
    const int len = __builtin_amdgcn_readfirstlane((in8(ip + 3) << 8) | in8(ip + 4));
    if (type == 0) {  // raw chunk: straight from global memory
      ip += 5;
      if (ip + len > n || op + len > kBlockBytes) {
        bad = true;
        break;
      }
      for (int k = lane; k < len; k += 64) outb[op + k] = j.src[ip + k];
      ip += len;
      op += len;
      __syncthreads();
      continue;
    }
    if (type != 1 || ip + 7 > n) {
      bad = true;
      break;
    }
    const int ulen = __builtin_amdgcn_readfirstlane((in8(ip + 5) << 8) | in8(ip + 6));
    ip += 7;
    const int end = ip + len, oend = op + ulen;
    if (end > n || oend > kBlockBytes) {
      bad = true;
      break;
    }
    while (ip < end) {
      refill(ip);
      // one 4-byte peek (two aligned LDS dwords) yields ctrl and both back-reference bytes
      const int x = ip - wb;
      const uint64_t pw = (uint64_t)win[x >> 2] | ((uint64_t)win[(x >> 2) + 1] << 32);
      // every lane holds the same token: make it wave-uniform so the token branches are scalar
      const uint32_t tok = __builtin_amdgcn_readfirstlane((uint32_t)(pw >> ((x & 3) * 8)));
      const int ctrl = tok & 0xFF;
      ip++;
      if (ctrl < 32) {
        const int run = ctrl + 1;
        if (ip + run > end || op + run > oend) {
          bad = true;
          break;
        }
        if (lane < run) outb[op + lane] = winb[ip - wb + lane];
        ip += run;
        op += run;
      } else {
        int l = ctrl >> 5;
        int offb;
        if (l == 7) {
          l += (tok >> 8) & 0xFF;
          offb = (tok >> 16) & 0xFF;
          ip += 2;
        } else {
          offb = (tok >> 8) & 0xFF;
          ip += 1;
        }
        if (ip > end) {
          bad = true;
          break;
        }
        const int dist = ((ctrl & 31) << 8) + 1 + offb;
        l += 2;
        if (dist > op || op + l > oend) {
          bad = true;
          break;
        }
        // an overlapping reference repeats its last `dist` bytes: byte k of the copy is
        // out[op - dist + k % dist], all of which precede op, so one lane-parallel pass suffices
        __syncthreads();
        if (dist >= l) {
          for (int k = lane; k < l; k += 64) outb[op + k] = outb[op - dist + k];
        } else {
          for (int k = lane; k < l; k += 64) outb[op + k] = outb[op - dist + k % dist];
        }
        op += l;
      }
      __syncthreads();
    }
    if (!bad && op != oend) bad = true;
  }
  __syncthreads();
  if (bad || op < j.expect_len) {
    if (lane == 0) atomicOr(err, 1);
    return;
  }
  const int o16 = op >> 4;
  for (int q = lane; q < o16; q += 64)
    reinterpret_cast<uint4*>(j.dst)[q] = reinterpret_cast<const uint4*>(outb)[q];
  for (int b = (o16 << 4) + lane; b < op; b += 64) j.dst[b] = outb[b];
}

void launch_lzf_decode(const LzfJob* d_jobs, int njobs, int32_t* d_err, hipStream_t s) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(k_lzf_decode, dim3((unsigned)njobs), dim3(64), 0, s, d_jobs, d_err);
}

}  // namespace dg

// ------------------------------------------------------------------------------------------------
// measurement probes (dg_debug_probe): what this box's HBM and host link deliver to plain kernels and
// copies, for bench.py's roofline ("also report vs a measured device copy-bandwidth")
// ------------------------------------------------------------------------------------------------
namespace dg {

// stream copy: every byte read once and written once, 16-byte accesses, grid-stride
__global__ __launch_bounds__(256) void k_probe_copy(const uint4* __restrict__ in, uint4* __restrict__ out, int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

// the groupBy reduce's memory floor: per element one sequential 8-byte word (a sorted [key | row]
// word), one 16-byte record gathered at its row, four sequential 8-byte stores (key + the three slots
// of a group, slot-major) — k_gb_reduce's loads and stores without its segmented scan
__global__ __launch_bounds__(256) void k_probe_gather(const uint64_t* __restrict__ words, const uint4* __restrict__ rec,
                                                     int64_t n, uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t w = words[i];
    const uint4 r = rec[w & ((1ull << 32) - 1)];
    out[i] = w >> 32;
    out[n + i] = 1;
    out[2 * n + i] = ((uint64_t)r.y << 32) | r.x;
    out[3 * n + i] = ((uint64_t)r.w << 32) | r.z;
  }
}

// words[i] = (i << 32) | (i * m mod n): a permutation of the rows (m odd and prime to n), so the
// gathers land on pseudo-random records like the reduce's sorted row references
__global__ void k_probe_fill(uint64_t* __restrict__ words, uint4* __restrict__ rec, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t r = ((uint64_t)i * 2654435761ull) % (uint64_t)n;  // (i < 2^32: no overflow)
    words[i] = ((uint64_t)i << 32) | r;
    rec[i] = make_uint4((uint32_t)i, 1u, (uint32_t)(i * 3), 2u);
  }
}

// DG_PROBE_CHAIN: one 64-thread workgroup; lane 0 reads the word its predecessor wrote and writes it + 1
__global__ __launch_bounds__(64) void k_probe_step(uint32_t* __restrict__ word) {
  if (threadIdx.x == 0) word[0] = word[0] + 1u;
}
void launch_probe_chain(uint32_t* word, int n, hipStream_t s) {
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_probe_step, dim3(1), dim3(64), 0, s, word);
}

void launch_probe_copy(const void* in, void* out, int64_t bytes, hipStream_t s) {
  const int64_t n16 = bytes / 16;
  hipLaunchKernelGGL(k_probe_copy, dim3(256 * 16), dim3(256), 0, s, static_cast<const uint4*>(in), static_cast<uint4*>(out), n16);
}

void launch_probe_gather(const uint64_t* words, const void* rec, int64_t n, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_probe_gather, dim3(256 * 16), dim3(256), 0, s, words, static_cast<const uint4*>(rec), n, out);
}

void launch_probe_fill(uint64_t* words, void* rec, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_probe_fill, dim3(256 * 16), dim3(256), 0, s, words, static_cast<uint4*>(rec), n);
}

}  // namespace dg
