// dg_sort.hip — groupBy v2 as a device-wide sort, and the floatSum row-order pass (gfx950).
//
// Replaces, for the merged result of the segments of one call:
//   GroupByQueryEngineV2.HashAggregateIterator.aggregateSingleValueDims + BufferHashGrouper per
//     segment (query/groupby/epinephelinae/GroupByQueryEngineV2.java:413-475,
//     ByteBufferHashTable.java:286-327, AbstractBufferHashGrouper.java:119-171), and
//   GroupByMergingQueryRunnerV2.run (epinephelinae/GroupByMergingQueryRunnerV2.java:170-290): the
//     ConcurrentGrouper merge of the segments' rows keyed by dimension values and its sorted iterator.
// A hash grouper pays one random CAS + one random atomic per aggregator per row (memory-side
// atomics on gfx950, ~17x slower than coalesced ones when every lane hits another row) and still
// has to sort its groups for the merged, ordered result. At Druid's high-cardinality shapes
// (config 3: ~1 group per row) sorting the rows is the whole job, so it is done directly:
//   keygen   selected rows -> (key, row ref): key = [segment slot | bucket | merged dictionary id of
//            each dimension] (ids of the call's merged dictionaries, Java String order, nulls first),
//            written in (segment, row) order with a deterministic per-tile compaction;
//   sort     stable LSD radix sort over the key's used bits (<= 8-bit digits: per-tile histograms,
//            per-digit scans, a ballot match-any ranking per wave, one scatter per pass);
//   runs     run heads of the sorted keys = the groups, in output order;
//   reduce   one record per group: 16 consecutive sorted rows per thread, inputs gathered by row
//            ref, the record written by the thread that owns the group's head with plain stores;
//            the partial of a group that started in an earlier thread goes to a carry slot that a
//            second kernel folds in with one atomic per (wave, group);
//   floatSum the reference adds float32 values one row at a time in row order per segment
//            (FloatSumBufferAggregator.java:38-46) and combines segments with float adds
//            (FloatSumAggregator.java:40-43); fp32 addition is not associative, so a floatSum slot
//            is computed by one thread per group walking its rows in (segment, row) order — exact
//            parity with the reference's recurrence instead of a tree sum.
// Integer results are exact; doubleSum partials combine in a different order than the reference's
// row loop (within the 1e-9 relative tolerance north_star states).
#include <hip/hip_runtime.h>
#include <cstring>

#include "dg_device.h"

namespace dg {

// Zero a device range before a kernel that reads it as look-back status / counters; on failure the
// dependent kernel is not launched (un-zeroed status words could make a look-back wait forever) and
// the error surfaces at the call's finish_call (take_launch_error).
static bool zero_async(void* p, size_t n, hipStream_t s) {
  const hipError_t e = hipMemsetAsync(p, 0, n, s);
  if (e != hipSuccess) note_launch_error(e);
  return e == hipSuccess;
}

constexpr int kST = 256;                 // threads of the sort / run kernels
constexpr int kSPT = kSortTile / kST;    // 16 elements per thread
// radix scatter tiles: DG_RS_TILE_MUL sort tiles each (A/B builds; 1 = the sort tile)
#ifndef DG_RS_TILE_MUL
#define DG_RS_TILE_MUL 1
#endif
// radix scatter threads (A/B builds; 256 = the sort kernels' kST)
#ifndef DG_RS_THREADS
#define DG_RS_THREADS 256
#endif
constexpr int kRsTile = kSortTile * DG_RS_TILE_MUL;
constexpr int kRsT = DG_RS_THREADS;
constexpr int kRsW = kRsT / 64;  // waves of a scatter tile
constexpr int kRsSPT = kRsTile / kRsT;

// exclusive scan of one u32 per thread over an NT-thread workgroup; *total = workgroup sum
template <int NT>
__device__ __forceinline__ uint32_t block_scan_u32(uint32_t v, uint32_t* total, uint32_t* s_tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_tmp[wave] = x;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const uint32_t y = s_tmp[w];
    off += w < wave ? y : 0u;
    tot += y;
  }
  __syncthreads();
  *total = tot;
  return off + x - v;
}

template <int NT>
__device__ __forceinline__ uint64_t block_scan_u64(uint64_t v, uint64_t* total, uint64_t* s_tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_tmp[wave] = x;
  __syncthreads();
  uint64_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const uint64_t y = s_tmp[w];
    off += w < wave ? y : 0ull;
    tot += y;
  }
  __syncthreads();
  *total = tot;
  return off + x - v;
}

template <int NT>
__device__ __forceinline__ uint32_t block_sum_u32(uint32_t v, uint32_t* s_tmp) {
  uint32_t t;
  block_scan_u32<NT>(v, &t, s_tmp);
  return t;
}

// one workgroup: exclusive scan of a[0..n) in place, *total = sum
__global__ __launch_bounds__(1024) void k_scan_u32(uint32_t* __restrict__ a, int n, uint32_t* __restrict__ total) {
  __shared__ uint32_t s_tmp[16];
  uint32_t carry = 0;
  for (int base = 0; base < n; base += 1024) {
    const int i = base + threadIdx.x;
    const uint32_t v = i < n ? a[i] : 0u;
    uint32_t t;
    const uint32_t ex = block_scan_u32<1024>(v, &t, s_tmp);
    if (i < n) a[i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) *total = carry;
}

// payload word a of the element with reference i ([i][pw] words: i = the element index, or in
// row-ref mode the row's index over the call's segments). Records, not columns: the reduce gathers one
// 16-byte record per element (payload columns: two random 8-byte reads, measured slower)
__device__ __forceinline__ size_t pay_at(int pw, size_t i, int a) { return i * (size_t)pw + (size_t)a; }

// segment of an element index (or row ref): the last job whose base <= it (bases ascend)
__device__ __forceinline__ int locate_seg(const uint32_t* s_base, int njobs, uint32_t ref) {
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s_base[mid] <= ref) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// ------------------------------------------------------------------------------------------------
// keygen: the cursor's rows (bitmap offset + interval, QueryableIndexStorageAdapter.makeCursors
// :190-316, CursorSequenceBuilder.build :367-456) -> grouping keys
// (GroupByQueryEngineV2.aggregateSingleValueDims :457-475 writes the row's dictionary ids as the key)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool gb_select(const GbJob& j, int64_t r, int64_t* bucket) {
  if (j.bitset && !((j.bitset[r >> 5] >> (r & 31)) & 1u)) return false;
  *bucket = 0;
  if (j.time.kind != VIEW_ABSENT) {
    const int64_t t = load_time(j.time, r);
    if (t < j.t_lo || t >= j.t_hi) return false;
    if (j.period) *bucket = (bucket_coord(j.bounds, j.nbounds, t) - j.bucket0) / j.period;
  }
  return true;
}

__device__ __forceinline__ uint64_t gb_key(const GbJob& j, int64_t r, int64_t bucket) {
  uint64_t k = ((uint64_t)j.seg_slot << j.seg_shift) | ((uint64_t)bucket << j.bucket_shift);
  for (int d = 0; d < j.ndims; ++d) {
    uint32_t g;
    if (j.dims[d].kind == VIEW_IDS) {
      const uint32_t id = load_id(j.dims[d], r);
      g = j.remap[d] ? (uint32_t)j.remap[d][id] : id;
    } else {
      g = (uint32_t)j.null_gid[d];  // missing dimension: every row has the null value
    }
    k |= (uint64_t)g << j.dim_shift[d];
  }
  return k;
}

// Multi-value dimensions: a row groups under every combination of its dimensions' values (an empty
// list = GROUP_BY_MISSING_VALUE, reported as null), the last dimension varying fastest
// (GroupByQueryEngineV2.HashAggregateIterator.aggregateMultiValueDims :480-540,
// StringGroupByColumnSelectorStrategy :47-57, :94-141). Row r's list of dimension d is
// dims[d][moff[d][r] .. moff[d][r + 1]).
// The product is formed in 64 bits and saturates at 0xFFFFFFFF: a row (or tile) that reaches it
// makes the element total >= 2^32, which the host rejects before sizing the sort.
__device__ __forceinline__ uint32_t gb_fanout(const GbJob& j, int64_t r) {
  uint64_t n = 1;
  for (int d = 0; d < j.ndims; ++d)
    if (j.moff[d].kind != VIEW_ABSENT) {
      const uint32_t a = load_id(j.moff[d], r), b = load_id(j.moff[d], r + 1);
      n *= b > a ? (uint64_t)(b - a) : (j.skip_empty ? 0ull : 1ull);
      n = n > 0xFFFFFFFFull ? 0xFFFFFFFFull : n;
    }
  return (uint32_t)n;
}

// key of grouping c (0 <= c < gb_fanout) of row r
__device__ __forceinline__ uint64_t gb_key_multi(const GbJob& j, int64_t r, int64_t bucket, uint32_t c) {
  uint64_t k = ((uint64_t)j.seg_slot << j.seg_shift) | ((uint64_t)bucket << j.bucket_shift);
  for (int d = j.ndims - 1; d >= 0; --d) {
    uint32_t g = (uint32_t)j.null_gid[d];
    if (j.moff[d].kind != VIEW_ABSENT) {
      const uint32_t a = load_id(j.moff[d], r), b = load_id(j.moff[d], r + 1);
      if (b > a) {
        const uint32_t m = b - a, i = c % m;
        c /= m;
        const uint32_t id = load_id(j.dims[d], (int64_t)a + i);
        g = j.remap[d] ? (uint32_t)j.remap[d][id] : id;
      }
    } else if (j.dims[d].kind == VIEW_IDS) {
      const uint32_t id = load_id(j.dims[d], r);
      g = j.remap[d] ? (uint32_t)j.remap[d][id] : id;
    }
    k |= (uint64_t)g << j.dim_shift[d];
  }
  return k;
}

template <bool MULTI>
__global__ __launch_bounds__(256) void k_gb_count(const GbJob* __restrict__ jobs, const int32_t* __restrict__ tile_job,
                                                  uint32_t* __restrict__ cnt) {
  __shared__ uint32_t s_tmp[4];
  const GbJob& j = jobs[tile_job[blockIdx.x]];
  const int64_t r0 = (int64_t)(blockIdx.x - j.tile_begin) * kTileRows;
  const int64_t r1 = min((int64_t)j.nrows, r0 + kTileRows);
  uint64_t c = 0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
    int64_t b;
    if (gb_select(j, r, &b)) c += MULTI ? gb_fanout(j, r) : 1u;
  }
  // the tile's sum in 64 bits (a row's fan-out is the product of its value-list lengths: a few rows can
  // pass 2^32 between them); only the stored 32-bit count saturates, which marks >= 2^32 elements
  __shared__ unsigned long long s_sum[4];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long t = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
    cnt[blockIdx.x] = t >= 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)t;
  }
  (void)s_tmp;
}

// total of n u32 counts in 64 bits (the element count of a multi-value keygen, checked against 2^32)
__global__ __launch_bounds__(1024) void k_sum_u64(const uint32_t* __restrict__ a, int n, unsigned long long* __restrict__ total) {
  __shared__ unsigned long long s[16];
  unsigned long long c = 0;
  for (int i = threadIdx.x; i < n; i += 1024) c += a[i];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < 16; ++w) t += s[w];
    *total = t;
  }
}

void launch_gb_count_total(const GbJob* d_jobs, const int32_t* d_tile_job, int ntiles, uint32_t* tile_cnt,
                           unsigned long long* total, hipStream_t s) {
  if (ntiles <= 0) {
    zero_async(total, 8, s);
    return;
  }
  hipLaunchKernelGGL(k_gb_count<true>, dim3(ntiles), dim3(256), 0, s, d_jobs, d_tile_job, tile_cnt);
  hipLaunchKernelGGL(k_sum_u64, dim3(1), dim3(1024), 0, s, tile_cnt, ntiles, total);
}

// element of the sort: packed = one word [key | row ref] (ref in the low sb->ref_bits bits, so equal
// keys stay in row-ref order without a second array), otherwise key words + a u32 ref array
__device__ __forceinline__ uint32_t elem_ref(uint64_t w, const uint32_t* refs, int64_t i, int kshift) {
  return refs ? refs[i] : (uint32_t)(w & ((1ull << kshift) - 1ull));
}

// Selected rows in (segment, row) order get consecutive element indices; the element's sort word
// carries its reference (packed) or the ref array does. The reference is the element index, or in
// row-ref mode (`rowref`: no multi-value dimension, one element per row) the row's index over the
// call's segments (row_base + r). The aggregators' inputs of the element are written at
// payload[ref * pw] in the device slot encoding, in row order (coalesced column reads), so the
// reduce after the sort gathers one payload record per element instead of one random read per
// column. In row-ref mode the payload columns in `j.inplace` were written by the LZ4 decoder
// itself (payload_view: the decoded value is the aggregator's input) and are left alone.
template <bool MULTI>
__global__ __launch_bounds__(256) void k_gb_keygen(const GbJob* __restrict__ jobs, const int32_t* __restrict__ tile_job,
                                                   const uint32_t* __restrict__ offs, uint64_t* __restrict__ keys,
                                                   uint32_t* __restrict__ refs, int kshift, AggPlan plan,
                                                   uint64_t* __restrict__ payload, int pw, int rowref, int rows_elems) {
  __shared__ uint32_t s_tmp[4];
  const GbJob& j = jobs[tile_job[blockIdx.x]];
  const int64_t r0 = (int64_t)(blockIdx.x - j.tile_begin) * kTileRows;
  const int64_t r1 = min((int64_t)j.nrows, r0 + kTileRows);
  // rows_elems: every row of the call is an element, in row order (no filter, every row's time inside
  // the interval, one element per row): the tile's first element is its first row's index over the
  // call, no count pass
  uint32_t base = rows_elems ? j.row_base + (uint32_t)r0 : offs[blockIdx.x];
  const uint32_t inplace = rowref ? j.inplace : 0u;
  const bool all_inplace = pw > 0 && inplace == (pw >= 32 ? 0xFFFFFFFFu : (1u << pw) - 1u);
  // the element's sort word(s) and payload record
  auto emit = [&](uint32_t idx, uint32_t ref, uint64_t key, auto&& val) {
    if (refs) {
      keys[idx] = key;
      refs[idx] = ref;
    } else {
      keys[idx] = (key << kshift) | ref;
    }
    if (all_inplace) return;
    if (pw == 2 && !inplace) {
      *reinterpret_cast<ulonglong2*>(payload + (size_t)ref * 2) = make_ulonglong2(val(0), val(1));
    } else {
      for (int a = 0; a < pw; ++a)
        if (!((inplace >> a) & 1u)) payload[pay_at(pw, ref, a)] = val(a);
    }
  };
  // every row of the tile selected: no filter, and the interval covers the segment or the tile's
  // __time block is a uniform one (time_view: its rows all inside the interval, in one bucket)
  bool all_rows = !MULTI && !j.bitset;
  int64_t tbucket = 0;
  if (all_rows && j.time.kind != VIEW_ABSENT) {
    const int64_t tk = r0 >> j.time.log2_per;
    all_rows = (reinterpret_cast<uintptr_t>(j.time.blocks[tk]) & 1u) && tk == ((r1 - 1) >> j.time.log2_per);
    if (all_rows) all_rows = gb_select(j, r0, &tbucket);
  }
  if (all_rows) {
    // element index = tile base + row offset, no per-block scan.
    // A tile (kTileRows, aligned) lies inside one block of every view (blocks hold >= 8192 rows):
    // each column's block pointer is then read once per tile (a scalar load) instead of per row, and
    // 3-byte ids are two aligned dword loads instead of three byte loads.
    bool direct = pw <= kMaxAggs;
    for (int d = 0; d < j.ndims; ++d)
      direct &= j.dims[d].kind != VIEW_IDS ||
                (!(j.dims[d].pad & kViewBigEndian) && (r0 >> j.dims[d].log2_per) == ((r1 - 1) >> j.dims[d].log2_per));
    for (int a = 0; a < pw; ++a)
      direct &= ((inplace >> a) & 1u) || j.vals[a].kind == VIEW_ABSENT ||
                (r0 >> j.vals[a].log2_per) == ((r1 - 1) >> j.vals[a].log2_per);
    if (direct) {
      // kB rows per thread (one batch: the whole tile), each dimension's id loads of the batch in flight
      // together, then its dictionary-map lookups together
      constexpr int kB = kTileRows / 256;
      static_assert(kTileRows % 256 == 0, "whole batches per tile");
      uint64_t key[kB];
#pragma unroll
      for (int u = 0; u < kB; ++u) key[u] = ((uint64_t)j.seg_slot << j.seg_shift) | ((uint64_t)tbucket << j.bucket_shift);
      // dimension d's ids of the batch, then their merged ids (rows past r1: id 0, a valid index)
      auto load_ids = [&](int d, uint32_t* id) {
        const ColView& v = j.dims[d];
        if (v.kind != VIEW_IDS) return;
        const int64_t blk = r0 >> v.log2_per;
        const uint8_t* bp = v.blocks[blk];
#pragma unroll
        for (int u = 0; u < kB; ++u) {
          const int64_t r = r0 + threadIdx.x + 256 * u;
          id[u] = 0;
          if (r < r1) {
            const uint32_t off = (uint32_t)(r - (blk << v.log2_per)) * (uint32_t)v.width;
            if (v.width == 3) {  // the slot / flat allocation extends past the last id's dword
              const uint32_t* w = reinterpret_cast<const uint32_t*>(bp + (off & ~3u));
              id[u] = __builtin_amdgcn_alignbyte(w[1], w[0], off & 3u) & 0xFFFFFFu;
            } else if (v.width == 1) {
              id[u] = bp[off];
            } else if (v.width == 2) {
              id[u] = *reinterpret_cast<const uint16_t*>(bp + off);
            } else {
              id[u] = *reinterpret_cast<const uint32_t*>(bp + off);
            }
          }
        }
      };
      auto merge_ids = [&](int d, uint32_t* id) {
        const int32_t* rm = j.remap[d];
        if (j.dims[d].kind != VIEW_IDS) {
#pragma unroll
          for (int u = 0; u < kB; ++u) key[u] |= (uint64_t)(uint32_t)j.null_gid[d] << j.dim_shift[d];
          return;
        }
#pragma unroll
        for (int u = 0; u < kB; ++u) key[u] |= (uint64_t)(rm ? (uint32_t)rm[id[u]] : id[u]) << j.dim_shift[d];
      };
      if (j.ndims == 2) {  // (the common two-dimension key: both columns' loads in flight, then both maps)
        uint32_t id0[kB], id1[kB];
        load_ids(0, id0);
        load_ids(1, id1);
        merge_ids(0, id0);
        merge_ids(1, id1);
      } else {
        for (int d = 0; d < j.ndims; ++d) {
          uint32_t id[kB];
          load_ids(d, id);
          merge_ids(d, id);
        }
      }
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        const int64_t r = r0 + threadIdx.x + 256 * u;
        if (r >= r1) continue;
        const uint32_t idx = base + (uint32_t)(r - r0);
        emit(idx, rowref ? j.row_base + (uint32_t)r : idx, key[u], [&](int a) -> uint64_t {
          const ColView& v = j.vals[a];
          if (!agg_row(j.agg_bits[a], r)) return identity_of(plan.op[a], plan.kind[a]);
          if (plan.kind[a] == DG_AGG_COUNT || v.kind == VIEW_ABSENT) return agg_input_at(plan.kind[a], v.kind, nullptr);
          const int64_t blk = r0 >> v.log2_per;
          return agg_input_at(plan.kind[a], v.kind, v.blocks[blk] + (size_t)(r - (blk << v.log2_per)) * (size_t)v.width);
        });
      }
      return;
    }
    for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
      const uint32_t idx = base + (uint32_t)(r - r0);
      emit(idx, rowref ? j.row_base + (uint32_t)r : idx, gb_key(j, r, tbucket), [&](int a) { return agg_in(j, plan, a, r); });
    }
    return;
  }
  for (int64_t rb = r0; rb < r1; rb += 256) {
    const int64_t r = rb + threadIdx.x;
    int64_t b = 0;
    const bool sel = r < r1 && gb_select(j, r, &b);
    uint32_t tot;
    if (MULTI) {  // every grouping of the row is an element with the row's aggregator inputs
      const uint32_t nf = sel ? gb_fanout(j, r) : 0u;
      const uint32_t ex = block_scan_u32<256>(nf, &tot, s_tmp);
      for (uint32_t e = 0; e < nf; ++e)
        emit(base + ex + e, base + ex + e, gb_key_multi(j, r, b, e), [&](int a) { return agg_in(j, plan, a, r); });
      base += tot;
      continue;
    }
    const uint32_t ex = block_scan_u32<256>(sel ? 1u : 0u, &tot, s_tmp);
    if (sel)
      emit(base + ex, rowref ? j.row_base + (uint32_t)r : base + ex, gb_key(j, r, b),
           [&](int a) { return agg_in(j, plan, a, r); });
    base += tot;
  }
}

void launch_gb_count(const GbJob* d_jobs, const int32_t* d_tile_job, int ntiles, uint32_t* tile_cnt, uint32_t* total,
                     bool multi, hipStream_t s) {
  if (ntiles <= 0) {
    zero_async(total, 4, s);
    return;
  }
  if (multi) hipLaunchKernelGGL(k_gb_count<true>, dim3(ntiles), dim3(256), 0, s, d_jobs, d_tile_job, tile_cnt);
  else hipLaunchKernelGGL(k_gb_count<false>, dim3(ntiles), dim3(256), 0, s, d_jobs, d_tile_job, tile_cnt);
  hipLaunchKernelGGL(k_scan_u32, dim3(1), dim3(1024), 0, s, tile_cnt, ntiles, total);
}

void launch_gb_keygen(const GbJob* d_jobs, const int32_t* d_tile_job, int ntiles, SortBufs* sb, AggPlan plan,
                      hipStream_t s, bool multi, int64_t all_rows) {
  if (ntiles <= 0) {
    zero_async(sb->n, 4, s);
    return;
  }
  const bool rows_elems = !multi && all_rows >= 0;
  if (rows_elems) {  // the element count is the call's row count (no per-tile count + scan)
    const hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(sb->n), (int)(uint32_t)all_rows, 1, s);
    if (e != hipSuccess) note_launch_error(e);
  } else {
    launch_gb_count(d_jobs, d_tile_job, ntiles, sb->tile_cnt, sb->n, multi, s);
  }
  if (multi)
    hipLaunchKernelGGL(k_gb_keygen<true>, dim3(ntiles), dim3(256), 0, s, d_jobs, d_tile_job, sb->tile_cnt,
                       sb->keys[sb->cur], sb->refs[sb->cur], sb->ref_bits, plan, sb->payload, sb->pw, 0, 0);
  else
    hipLaunchKernelGGL(k_gb_keygen<false>, dim3(ntiles), dim3(256), 0, s, d_jobs, d_tile_job, sb->tile_cnt,
                       sb->keys[sb->cur], sb->refs[sb->cur], sb->ref_bits, plan, sb->payload, sb->pw, sb->row_refs,
                       rows_elems ? 1 : 0);
}

// ------------------------------------------------------------------------------------------------
// stable LSD radix sort (key words [+ u32 refs]), tiles of kSortTile consecutive elements, one sweep
// per pass: a pass is a single kernel whose tiles find their digits' global offsets by decoupled
// look-back over the earlier tiles' published counts, and which counts the next pass's digits of the
// keys it stores; only the first pass's digit totals need a read of the keys of their own
// (k_rs_hist0). No per-pass histogram read, no separate scan.
// ------------------------------------------------------------------------------------------------
// look-back status words: a flag in the top two bits (the tile's own count / the inclusive prefix up
// to the tile) and a count below. An inclusive prefix counts every earlier element of the digit, up to
// n: 32-bit words (30-bit counts) when the call's capacity is below 2^30 elements, 64-bit words
// otherwise (n < 2^32) — the narrow words halve the look-back traffic of every pass
template <class W>
struct Lb {
  static constexpr int kShift = 8 * sizeof(W) - 2;
  static constexpr W kAgg = (W)1 << kShift;
  static constexpr W kPre = (W)2 << kShift;
  static constexpr W kVal = ((W)1 << kShift) - 1;
};
constexpr uint64_t kLbAgg = Lb<uint64_t>::kAgg;  // (the groupBy reduce's per-tile look-back)
constexpr uint64_t kLbPre = Lb<uint64_t>::kPre;
constexpr uint64_t kLbVal = Lb<uint64_t>::kVal;

// the first pass's digit totals: totals[d] += elements whose digit (bits above shift) is d
__global__ __launch_bounds__(kST) void k_rs_hist0(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ n_ptr,
                                                  int shift, int bits, uint32_t* __restrict__ totals) {
  __shared__ uint32_t s_h[4][kMaxBins];  // one histogram per wave (fewer same-address LDS atomics)
  const int tid = threadIdx.x, wave = tid >> 6;
  for (int i = tid; i < 4 * kMaxBins; i += kST) (&s_h[0][0])[i] = 0;
  __syncthreads();
  const uint32_t n = *n_ptr;
  const uint64_t mask = (1ull << bits) - 1;
  // four independent loads in flight per thread (one per iteration left the read latency-bound)
  constexpr int kU = 4;
  const int64_t stride = (int64_t)gridDim.x * kST;
  int64_t i = (int64_t)blockIdx.x * kST + tid;
  for (; i + (kU - 1) * stride < (int64_t)n; i += kU * stride) {
    uint64_t w[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) w[u] = keys[i + u * stride];
#pragma unroll
    for (int u = 0; u < kU; ++u) atomicAdd(&s_h[wave][(int)((w[u] >> shift) & mask)], 1u);
  }
  for (; i < (int64_t)n; i += stride) atomicAdd(&s_h[wave][(int)((keys[i] >> shift) & mask)], 1u);
  __syncthreads();
  for (int d = tid; d < (1 << bits); d += kST) {
    const uint32_t c = s_h[0][d] + s_h[1][d] + s_h[2][d] + s_h[3][d];
    if (c) atomicAdd(&totals[d], c);
  }
}

// lanes of the wave whose digit equals mine (ballot per digit bit), restricted to valid lanes
__device__ __forceinline__ uint64_t match_digit(uint32_t d, int bits, bool valid) {
  uint64_t m = __ballot(valid);
  for (int b = 0; b < bits; ++b) {
    const bool x = (d >> b) & 1u;
    const uint64_t bb = __ballot(x);
    m &= x ? bb : ~bb;
  }
  return m;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// One LSD pass. Tiles take their index from a counter as they start, so a tile only waits for tiles
// that are running or done. Wave w of a tile owns its elements [w * 1024, (w + 1) * 1024) in 16 chunks
// of 64. Each element is ranked among the earlier elements of its wave with the same digit (chunk
// order, then lane order = element order). Thread d publishes the tile's count of digit d, adds the
// earlier tiles' counts walking back until one has published its inclusive prefix, and publishes its
// own. The tile is then reordered by digit in LDS, so the global stores of a wave run along each
// digit's contiguous output range (coalesced) instead of scattering lane by lane.
template <bool REFS, class W>
__global__ __launch_bounds__(kRsT) void k_rs_scatter(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                    uint64_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                    const uint32_t* __restrict__ n_ptr, int shift, int bits,
                                                    const uint32_t* __restrict__ totals, W* __restrict__ status,
                                                    uint32_t* __restrict__ tile_ctr, int nshift, int nbits,
                                                    uint32_t* __restrict__ ntotals) {
  __shared__ uint64_t s_k[kRsTile];
  __shared__ uint32_t s_v[REFS ? kRsTile : 1];
  __shared__ uint32_t s_cnt[kRsW * kMaxBins];
  __shared__ uint32_t s_next[kMaxBins];  // the next pass's digit counts of the tile
  __shared__ int64_t s_delta[kMaxBins];  // global position of tile-sorted element i of digit d = s_delta[d] + i
  __shared__ uint64_t s_tmp64[kRsW];
  __shared__ int s_tile;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t n = *n_ptr;  // (in flight with the tile counter: one round trip before the key loads)
  if (tid == 0) s_tile = (int)atomicAdd(tile_ctr, 1u);
  // during the ranking the tile buffer is free: per wave and digit, the mask of the chunk's lanes
  // holding that digit (one LDS OR per chunk instead of a ballot per digit bit)
  uint64_t* s_peer = reinterpret_cast<uint64_t*>(s_k);
  static_assert(kRsW * kMaxBins <= kRsTile, "peer masks fit the tile buffer");
  for (int i = tid; i < kRsW * kMaxBins; i += kRsT) {
    s_cnt[i] = 0;
    s_peer[i] = 0;
  }
  for (int i = tid; i < kMaxBins; i += kRsT) s_next[i] = 0;
  __syncthreads();
  const int tile = s_tile;
  const int64_t base = (int64_t)tile * kRsTile;
  if (base >= n) return;  // (every later tile is past the end too: none waits for this one)
  const int tile_n = (int)min<int64_t>(kRsTile, (int64_t)n - base);
  const int nb = 1 << bits;
  const uint64_t dmask = (uint64_t)(nb - 1);
  const uint64_t nmask = (1ull << nbits) - 1;
  const int wbase = wave * (kRsTile / kRsW);
  uint64_t k[kRsSPT];
  uint32_t v[kRsSPT], rank[kRsSPT];
#pragma unroll
  for (int c = 0; c < kRsSPT; ++c) {
    const int x = wbase + c * 64 + lane;
    const bool ok = x < tile_n;
    k[c] = ok ? kin[base + x] : 0ull;
    if (REFS) v[c] = ok ? vin[base + x] : 0u;
  }
  uint32_t* cnt = s_cnt + wave * kMaxBins;
  uint64_t* peer = s_peer + wave * kMaxBins;
#pragma unroll
  for (int c = 0; c < kRsSPT; ++c) {
    const bool ok = wbase + c * 64 + lane < tile_n;
    const uint32_t d = (uint32_t)((k[c] >> shift) & dmask);
    // every lane ORs its bit into its digit's mask, then reads the mask back: the lanes with my digit
    // (a wave's LDS operations complete in issue order: every OR lands before the read)
    if (ok) __hip_atomic_fetch_or(peer + d, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    uint64_t peers = 0;
    uint32_t prior = 0;
    if (ok) {
      peers = peer[d];
      prior = cnt[d];
    }
    rank[c] = prior + lanes_below(peers);
    // the highest lane of each digit group advances the wave's count and clears the mask (every lane
    // above read both before these writes)
    if (ok && 63 - __clzll((long long)peers) == lane) {
      cnt[d] = prior + (uint32_t)__popcll(peers);
      peer[d] = 0;
    }
  }
  __syncthreads();
  // thread t: digits t * kDPT .. + kDPT: each one's count in the tile, its wave offsets, the earlier
  // tiles' counts (look-back) and the digit's global base (the earlier digits' totals)
  {
    constexpr int kDPT = kMaxBins > kRsT ? kMaxBins / kRsT : 1;
    static_assert(kMaxBins <= kRsT || kMaxBins % kRsT == 0, "digits per thread");
    uint32_t cw[kDPT][kRsW], ct[kDPT];
    uint64_t excl[kDPT];
    uint32_t csum = 0, gsum = 0;
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {
      const int d = tid * kDPT + j;
      ct[j] = 0;
      excl[j] = 0;
#pragma unroll
      for (int w = 0; w < kRsW; ++w) {
        cw[j][w] = d < nb ? s_cnt[w * kMaxBins + d] : 0u;
        ct[j] += cw[j][w];
      }
      csum += ct[j];
      gsum += d < nb ? totals[d] : 0u;
      if (d >= nb) continue;
      W* st = status + (size_t)tile * nb + d;
      if (tile == 0) {
        __hip_atomic_store(st, Lb<W>::kPre | (W)ct[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      __hip_atomic_store(st, Lb<W>::kAgg | (W)ct[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // eight earlier tiles at a time (independent loads), newest first, up to the first one with its
      // inclusive prefix; a tile not published yet (it has started: it publishes its count without
      // waiting) is loaded again
#ifndef DG_RS_LB
#define DG_RS_LB 8
#endif
      constexpr int kLb = DG_RS_LB;
      uint64_t ex = 0;
#ifdef DG_RS_NO_LOOKBACK  // (timing probe builds only: every tile takes offset 0 — the sort is wrong)
      for (int jt = -1; jt >= 0;) {
#else
      for (int jt = tile - 1; jt >= 0;) {
#endif
        W sv[kLb];
#pragma unroll
        for (int q = 0; q < kLb; ++q)
          sv[q] = jt - q >= 0 ? __hip_atomic_load(status + (size_t)(jt - q) * nb + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                              : Lb<W>::kPre;
        int q = 0;
        bool prefix = false;
        for (; q < kLb; ++q) {
          if ((sv[q] >> Lb<W>::kShift) == 0) break;
          ex += sv[q] & Lb<W>::kVal;
          if (sv[q] & Lb<W>::kPre) {
            prefix = true;
            break;
          }
        }
        if (prefix) break;
        jt -= q;
        if (q < kLb) __builtin_amdgcn_s_sleep(1);
      }
      excl[j] = ex;
      __hip_atomic_store(st, Lb<W>::kPre | (W)(ex + ct[j]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // both exclusive scans in one (the tile's counts in the low word: at most kRsTile, no carry)
    uint64_t tot;
    const uint64_t both = block_scan_u64<kRsT>(((uint64_t)gsum << 32) | csum, &tot, s_tmp64);
    uint32_t toff = (uint32_t)both, gex = (uint32_t)(both >> 32);
#pragma unroll
    for (int j = 0; j < kDPT; ++j) {
      const int d = tid * kDPT + j;
      if (d < nb) {
        uint32_t wo = toff;
#pragma unroll
        for (int w = 0; w < kRsW; ++w) {
          s_cnt[w * kMaxBins + d] = wo;
          wo += cw[j][w];
        }
        s_delta[d] = (int64_t)gex + (int64_t)excl[j] - (int64_t)toff;
        toff += ct[j];
        gex += totals[d];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < kRsSPT; ++c) {
    if (wbase + c * 64 + lane >= tile_n) continue;
    const uint32_t d = (uint32_t)((k[c] >> shift) & dmask);
    const uint32_t lp = cnt[d] + rank[c];
    s_k[lp] = k[c];
    if (REFS) s_v[lp] = v[c];
  }
  __syncthreads();
  // (unrolled: the LDS reads of every store are independent)
#pragma unroll
  for (int c = 0; c < kRsSPT; ++c) {
    const int i = c * kRsT + tid;
    if (i < tile_n) {
      const uint64_t kk = s_k[i];
      const int64_t pos = s_delta[(kk >> shift) & dmask] + i;
      kout[pos] = kk;
      if (REFS) vout[pos] = s_v[i];
      if (ntotals) atomicAdd(&s_next[(kk >> nshift) & nmask], 1u);
    }
  }
  if (ntotals) {  // the next pass's digit totals (complete once this pass's kernel is)
    __syncthreads();
    for (int dd = tid; dd < (1 << nbits); dd += kRsT)
      if (s_next[dd]) atomicAdd(&ntotals[dd], s_next[dd]);
  }
}

// LSD passes over key bits [lo, hi) of the key field (above the element index bits)
static void radix_passes(SortBufs* sb, int lo, int hi, hipStream_t s) {
  const int kb = hi - lo;
  if (kb <= 0) return;
  const int npass = (kb + kMaxDigitBits - 1) / kMaxDigitBits;
  const int w = (kb + npass - 1) / npass;
  const int nt = (sb->ntiles_sort + DG_RS_TILE_MUL - 1) / DG_RS_TILE_MUL;  // scatter tiles
  uint32_t* totals = sb->bin_total;                            // [npass][kMaxBins]
  uint32_t* ctr = sb->bin_total + kRsMaxPasses * kMaxBins;     // [npass] tile counters
  if (!zero_async(sb->bin_total, ((size_t)kRsMaxPasses * kMaxBins + kRsMaxPasses) * sizeof(uint32_t), s)) return;
  // the first pass's digit totals from one read of the keys; every pass's scatter counts the next
  // pass's digits of the keys it stores
  hipLaunchKernelGGL(k_rs_hist0, dim3(std::min(nt, 4096)), dim3(kST), 0, s, sb->keys[sb->cur], sb->n,
                     sb->ref_bits + lo, std::min(kb, w), totals);
  for (int p = 0, off = lo; p < npass; ++p, off += w) {
    const int bits = std::min(w, hi - off);
    const int shift = sb->ref_bits + off;
    const int nbits = p + 1 < npass ? std::min(w, hi - off - w) : 0;
    uint32_t* nt_tot = p + 1 < npass ? totals + (size_t)(p + 1) * kMaxBins : nullptr;
    const int in = sb->cur, out = sb->cur ^ 1;
    // 30-bit counts hold every prefix (n <= cap); DG_SORT_WIDE_STATUS=1: 64-bit words regardless (tests)
    const char* wide = getenv("DG_SORT_WIDE_STATUS");
    const bool narrow = sb->cap < ((int64_t)1 << 30) && !(wide && *wide && *wide != '0');
    if (!zero_async(sb->lb_status, (size_t)(1 << bits) * nt * (narrow ? 4 : 8), s)) return;  // look-back status
    uint32_t* st32 = reinterpret_cast<uint32_t*>(sb->lb_status);
    uint64_t* st64 = sb->lb_status;
    const uint32_t* tp = totals + (size_t)p * kMaxBins;
    if (sb->refs[in] && narrow)
      hipLaunchKernelGGL((k_rs_scatter<true, uint32_t>), dim3(nt), dim3(kRsT), 0, s, sb->keys[in], sb->refs[in], sb->keys[out],
                         sb->refs[out], sb->n, shift, bits, tp, st32, ctr + p, shift + w, nbits, nt_tot);
    else if (sb->refs[in])
      hipLaunchKernelGGL((k_rs_scatter<true, uint64_t>), dim3(nt), dim3(kRsT), 0, s, sb->keys[in], sb->refs[in], sb->keys[out],
                         sb->refs[out], sb->n, shift, bits, tp, st64, ctr + p, shift + w, nbits, nt_tot);
    else if (narrow)
      hipLaunchKernelGGL((k_rs_scatter<false, uint32_t>), dim3(nt), dim3(kRsT), 0, s, sb->keys[in], nullptr, sb->keys[out],
                         nullptr, sb->n, shift, bits, tp, st32, ctr + p, shift + w, nbits, nt_tot);
    else
      hipLaunchKernelGGL((k_rs_scatter<false, uint64_t>), dim3(nt), dim3(kRsT), 0, s, sb->keys[in], nullptr, sb->keys[out],
                         nullptr, sb->n, shift, bits, tp, st64, ctr + p, shift + w, nbits, nt_tot);
    sb->cur = out;
  }
}

void launch_radix_sort(SortBufs* sb, int key_bits, hipStream_t s) {
  if (key_bits <= 0) return;
  static_assert(64 / kMaxDigitBits <= kRsMaxPasses, "passes of a 64-bit key");
  radix_passes(sb, 0, key_bits, s);
}

// DG_PROBE_SORT: the headline's sort words — [id0 (17 bits) | id1 (17 bits) | element index], the ids
// uniform below 100000 (splitmix64 of the index) — and a check that the sorted words ascend
__global__ void k_probe_sort_fill(uint64_t* __restrict__ keys, int64_t n, int ref_bits) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const uint64_t key = (((z & 0xFFFFFFFFull) % 100000ull) << 17) | ((z >> 32) % 100000ull);
    keys[i] = (key << ref_bits) | (uint64_t)i;
  }
}
__global__ void k_probe_sort_check(const uint64_t* __restrict__ keys, int64_t n, uint32_t* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += (int64_t)gridDim.x * blockDim.x)
    if (keys[i] >= keys[i + 1]) atomicAdd(bad, 1u);
}

int probe_sort(int64_t n, int iters, double* ms, hipStream_t st) {
  if (n <= 0 || n >= (1ll << 30)) return set_error(DG_ERR_ARG, "probe: sort of %lld elements", (long long)n);
  SortBufs sb;
  memset(&sb, 0, sizeof sb);
  sb.cap = n;
  sb.ntiles_sort = sort_tiles(n);
  int rb = 1;
  while ((1ll << rb) < n) ++rb;
  sb.ref_bits = rb;
  const int key_bits = 34;
  void* mem[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  const size_t sz[5] = {((size_t)n + 16) * 8, ((size_t)n + 16) * 8, (size_t)kMaxBins * sb.ntiles_sort * 8,
                        ((size_t)kMaxBins * kRsMaxPasses + kRsMaxPasses + 1) * 4, 16};
  int rc = DG_OK;
  for (int i = 0; i < 5 && rc == DG_OK; ++i)
    if (hipMalloc(&mem[i], sz[i]) != hipSuccess) rc = set_error(DG_ERR_OOM, "probe: sort buffers of %lld", (long long)n);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (rc == DG_OK) {
    sb.keys[0] = static_cast<uint64_t*>(mem[0]);
    sb.keys[1] = static_cast<uint64_t*>(mem[1]);
    sb.lb_status = static_cast<uint64_t*>(mem[2]);
    sb.bin_total = static_cast<uint32_t*>(mem[3]);
    sb.n = static_cast<uint32_t*>(mem[4]);
    const uint32_t nn[4] = {(uint32_t)n, 0u, 0u, 0u};
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    double tot = 0;
    for (int it = 0; it <= iters && rc == DG_OK; ++it) {  // (repetition 0: warm-up)
      sb.cur = 0;
      (void)hipMemcpyAsync(sb.n, nn, 16, hipMemcpyHostToDevice, st);
      hipLaunchKernelGGL(k_probe_sort_fill, dim3(4096), dim3(256), 0, st, sb.keys[0], n, rb);
      (void)hipEventRecord(e0, st);
      launch_radix_sort(&sb, key_bits, st);
      (void)hipEventRecord(e1, st);
      (void)hipMemsetAsync(sb.n + 1, 0, 4, st);
      hipLaunchKernelGGL(k_probe_sort_check, dim3(4096), dim3(256), 0, st, sb.keys[sb.cur], n, sb.n + 1);
      uint32_t bad = 0;
      (void)hipMemcpyAsync(&bad, sb.n + 1, 4, hipMemcpyDeviceToHost, st);
      if (hipStreamSynchronize(st) != hipSuccess || hipGetLastError() != hipSuccess) {
        rc = set_error(DG_ERR_DEVICE, "probe: sort failed");
#ifndef DG_RS_NO_LOOKBACK
      } else if (bad) {
        rc = set_error(DG_ERR_DEVICE, "probe: %u sorted words out of order", bad);
#endif
      } else if (it > 0) {
        float f = 0;
        (void)hipEventElapsedTime(&f, e0, e1);
        tot += f;
      }
    }
    if (rc == DG_OK) *ms = tot / iters;
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  for (void* m : mem)
    if (m) (void)hipFree(m);
  return rc;
}

// ------------------------------------------------------------------------------------------------
// runs of equal keys (= groups, in output order)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kST) void k_run_count(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ n_ptr,
                                                   int kshift, uint32_t* __restrict__ run_cnt) {
  __shared__ uint32_t s_tmp[4];
  const uint32_t n = *n_ptr;
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
  uint32_t c = 0;
  if (base < n) {
#pragma unroll 4
    for (int q = 0; q < kSPT; ++q) {
      const int64_t i = base + q * kST + threadIdx.x;
      if (i < n) c += (i == 0 || (keys[i] >> kshift) != (keys[i - 1] >> kshift)) ? 1u : 0u;
    }
  }
  const uint32_t t = block_sum_u32<kST>(c, s_tmp);
  if (threadIdx.x == 0) run_cnt[blockIdx.x] = t;
}

void launch_run_heads(SortBufs* sb, hipStream_t s) {
  hipLaunchKernelGGL(k_run_count, dim3(sb->ntiles_sort), dim3(kST), 0, s, sb->keys[sb->cur], sb->n, sb->ref_bits,
                     sb->run_cnt);
  hipLaunchKernelGGL(k_scan_u32, dim3(1), dim3(1024), 0, s, sb->run_cnt, sb->ntiles_sort, sb->n + 1);
}

// head_pos[g] = first element of run g (per-segment engines; the groupBy reduce writes its own)
__global__ __launch_bounds__(kST) void k_run_mark(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ n_ptr,
                                                  int kshift, const uint32_t* __restrict__ run_off,
                                                  uint32_t* __restrict__ head_pos) {
  __shared__ uint32_t s_tmp[4];
  const uint32_t n = *n_ptr;
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
  if (base >= n) return;
  const int64_t x0 = base + (int64_t)threadIdx.x * kSPT;
  uint32_t h = 0;
  for (int q = 0; q < kSPT; ++q) {
    const int64_t i = x0 + q;
    if (i < n && (i == 0 || (keys[i] >> kshift) != (keys[i - 1] >> kshift))) h |= 1u << q;
  }
  uint32_t tot;
  uint32_t g = run_off[blockIdx.x] + block_scan_u32<kST>((uint32_t)__popc(h), &tot, s_tmp);
  for (int q = 0; q < kSPT; ++q)
    if ((h >> q) & 1u) head_pos[g++] = (uint32_t)(x0 + q);
}

void launch_run_mark(SortBufs* sb, uint32_t* head_pos, hipStream_t s) {
  hipLaunchKernelGGL(k_run_mark, dim3(sb->ntiles_sort), dim3(kST), 0, s, sb->keys[sb->cur], sb->n, sb->ref_bits,
                     sb->run_cnt, head_pos);
}

// ------------------------------------------------------------------------------------------------
// finalize: device slot encoding -> the ABI's (int64 / double / float32 in the low 4 bytes)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t finalize_dev(int kind, uint64_t s) {
  switch (kind) {
    case DG_AGG_COUNT:
    case DG_AGG_LONG_SUM:
    case DG_AGG_DOUBLE_SUM: return s;
    case DG_AGG_FLOAT_SUM: return (uint64_t)__float_as_uint((float)__longlong_as_double((long long)s));
    case DG_AGG_LONG_MIN:
    case DG_AGG_LONG_MAX: return s ^ kSign;
    case DG_AGG_DOUBLE_MIN:
    case DG_AGG_DOUBLE_MAX: {
      const bool nan = kind == DG_AGG_DOUBLE_MIN ? s == 0 : s == ~0ull;
      const double d = nan ? __longlong_as_double(0x7ff8000000000000ll) : unord_key(s);
      return (uint64_t)__double_as_longlong(d);
    }
    default: {
      const bool nan = kind == DG_AGG_FLOAT_MIN ? s == 0 : s == ~0ull;
      const float f = nan ? __uint_as_float(0x7fc00000u) : (float)unord_key(s);
      return (uint64_t)__float_as_uint(f);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// groupBy reduce: the merged grouper's records (AggregatorFactory.combine semantics across segments
// = the per-row aggregate ops, both exact for counts / long sums / min / max)
// ------------------------------------------------------------------------------------------------
// Reduce-by-key over a tile of kSortTile sorted elements, processed as 16 chunks of 256 consecutive
// elements (lane = element): a segmented scan per chunk (wave shuffles, then the 4 waves' carries
// through LDS, then the chunk's open run carried into the next chunk). The element that ends a run
// writes its group's slot, so a wave's stores go to consecutive groups. A group that starts in the
// tile and ends there is written finalized (ABI encoding); the tile's last group, if it continues,
// is written in the device encoding and listed in open_g; the tile's leading part of a group that
// started in an earlier tile goes to the tile's carry slot. k_gb_carry folds the carries in,
// k_gb_open_finalize finalizes the open groups. floatSum slots are left to k_fsum_runs.
__device__ __forceinline__ uint64_t seg_scan_wave(int op, uint64_t v, bool head, bool* any_head) {
  const int lane = threadIdx.x & 63;
  bool f = head;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(v, o, 64);
    const int fy = __shfl_up((int)f, o, 64);
    if (lane >= o) {
      if (!f) v = combine_op(op, y, v);
      f = f || fy;
    }
  }
  *any_head = f;
  return v;
}

constexpr int kRedMinW = 4;  // waves per EU the reduce is compiled for (87 VGPRs)
constexpr int kRT = 64 * kRedWaves;             // reduce threads per tile
constexpr int kRSPT = kSortTile / kRT;          // elements per lane
// A workgroup barrier for LDS only: waits for this wave's LDS operations, not its global loads, so the
// reduce's random payload gathers stay in flight across the head count and the look-back (a
// __syncthreads would wait for them: s_waitcnt vmcnt(0) before s_barrier; measured equal or slower).
__device__ __forceinline__ void red_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool REFS>
__global__ __launch_bounds__(kRT, kRedMinW) void k_gb_reduce(const uint64_t* __restrict__ payload, int pw,
                                                   const uint64_t* __restrict__ keys, const uint32_t* __restrict__ refs,
                                                   int kshift, uint32_t* __restrict__ n_ptr,
                                                   uint64_t* __restrict__ status, uint32_t* __restrict__ tile_ctr,
                                                   AggPlan plan,
                                                   uint64_t* __restrict__ out_keys, uint64_t* __restrict__ out_slots,
                                                   int64_t cap, uint32_t* __restrict__ head_pos,
                                                   int64_t* __restrict__ carry_g, uint64_t* __restrict__ carry_slots,
                                                   int64_t* __restrict__ open_g) {
  // Each wave reduces its own contiguous share of the tile (kWSeg elements, kRSPT chunks of 64): a
  // segmented wave scan per chunk with the open run carried in registers, no barriers. A run that
  // crosses a share boundary is finished like one crossing a tile boundary: the share holding
  // its head writes it open (device encoding, listed in open_g), every later share's share goes to
  // that share's carry slot (k_gb_carry folds it in, k_gb_open_finalize finalizes).
  // The groups before a tile are counted by decoupled look-back over the earlier tiles' run-head
  // counts (tiles take their index from a counter as they start, so a tile only waits on running
  // ones); the last tile publishes the group count (n_ptr[1]). No separate run-count pass over the
  // keys, no host read-back before the reduce: the result is laid out for `cap` (>= groups) records.
  constexpr int kWSeg = kSortTile / kRedWaves;
  __shared__ uint64_t s_key[kSortTile + 2];  // [0] = element before the tile, [1 + x] = element x
  __shared__ uint32_t s_heads[kRedWaves];
  __shared__ int s_tile;
  __shared__ int64_t s_gbase;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t n = n_ptr[0];  // (in flight with the tile counter)
  if (tid == 0) s_tile = (int)atomicAdd(tile_ctr, 1u);
  __syncthreads();
  const int tile = s_tile;
  const int64_t base = (int64_t)tile * kSortTile;
  const int64_t wt = (int64_t)tile * kRedWaves + wave;  // wave tile (carry / open slot)
  if (lane == 0) {
    carry_g[wt] = -1;
    open_g[wt] = -1;
  }
  if (base >= n) return;
  const int tile_n = (int)min<int64_t>(kSortTile, (int64_t)n - base);
  const uint64_t kmask = kshift ? ((1ull << kshift) - 1ull) : 0ull;
  const int wbase = wave * kWSeg;
  uint32_t idx_of[kRSPT];
  uint64_t kw[kRSPT];
#pragma unroll
  for (int c = 0; c < kRSPT; ++c) {  // every key load in flight before the first LDS store
    const int x = wbase + c * 64 + lane;
    kw[c] = x < tile_n ? keys[base + x] : 0ull;
    idx_of[c] = REFS ? (x < tile_n ? refs[base + x] : 0u) : 0u;
  }
#pragma unroll
  for (int c = 0; c < kRSPT; ++c) {
    const int x = wbase + c * 64 + lane;
    s_key[1 + x] = kw[c] >> kshift;
    if (!REFS) idx_of[c] = (uint32_t)(kw[c] & kmask);
  }
  const bool has_next = base + kSortTile < n;
  if (tid == 0) {
    s_key[0] = base > 0 ? keys[base - 1] >> kshift : ~(keys[0] >> kshift);
    if (has_next) s_key[1 + kSortTile] = keys[base + kSortTile] >> kshift;
  }
  // up to two payload slots per element, gathered once and together (random record reads in flight)
  constexpr int kRegSlots = 2;
  uint64_t xr[kRSPT][kRegSlots];
  if (pw <= kRegSlots) {
#pragma unroll
    for (int c = 0; c < kRSPT; ++c) {
      const bool valid = wbase + c * 64 + lane < tile_n;
      const uint64_t* pr = payload + (size_t)idx_of[c] * pw;
      if (pw == 2 && valid) {
        const ulonglong2 w = *reinterpret_cast<const ulonglong2*>(pr);  // 16-byte aligned: pw == 2
        xr[c][0] = w.x;
        xr[c][1] = w.y;
      } else {
        xr[c][0] = valid && pw >= 1 ? pr[0] : 0ull;
        xr[c][1] = 0ull;
      }
    }
  }
  red_barrier();  // the tile's keys are in LDS (the payload gathers stay in flight)
  // run heads / ends of my elements, and the groups whose head lies before my share
  uint32_t hm = 0, tm = 0;
  uint32_t nh = 0;  // heads in my share
#pragma unroll
  for (int c = 0; c < kRSPT; ++c) {
    const int x = wbase + c * 64 + lane;
    const bool valid = x < tile_n;
    const uint64_t k = s_key[1 + x];
    const bool h = valid && k != s_key[x];
    bool t = false;
    if (valid) t = x + 1 < tile_n ? s_key[2 + x] != k : (!has_next || s_key[1 + kSortTile] != k);
    hm |= (uint32_t)h << c;
    tm |= (uint32_t)t << c;
    nh += (uint32_t)__popcll(__ballot(h));
  }
  if (lane == 0) s_heads[wave] = nh;
  red_barrier();
  if (tid == 0) {  // look-back: the groups headed in earlier tiles
    uint64_t cnt = 0;
    for (int w = 0; w < kRedWaves; ++w) cnt += s_heads[w];
    uint64_t excl = 0;
    uint64_t* st = status + tile;
    if (tile == 0) {
      __hip_atomic_store(st, kLbPre | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(st, kLbAgg | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      constexpr int kLb = 8;
      for (int j = tile - 1; j >= 0;) {
        uint64_t sv[kLb];
#pragma unroll
        for (int q = 0; q < kLb; ++q)
          sv[q] = j - q >= 0 ? __hip_atomic_load(status + (j - q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbPre;
        int q = 0;
        bool prefix = false;
        for (; q < kLb; ++q) {
          if ((sv[q] >> 62) == 0) break;
          excl += sv[q] & kLbVal;
          if (sv[q] & kLbPre) {
            prefix = true;
            break;
          }
        }
        if (prefix) break;
        j -= q;
        if (q < kLb) __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(st, kLbPre | (excl + cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (base + kSortTile >= (int64_t)n) n_ptr[1] = (uint32_t)(excl + cnt);  // the last tile: the group count
    s_gbase = (int64_t)excl;
  }
  red_barrier();
  int64_t G = s_gbase;  // groups with a head before my share
  for (int w = 0; w < wave; ++w) G += s_heads[w];
  const int64_t Gq = G;
  int32_t grel[kRSPT];  // group of each element relative to Gq (-1: the group open before my share)
  {
    int heads = 0;
#pragma unroll
    for (int c = 0; c < kRSPT; ++c) {
      const bool h = (hm >> c) & 1u;
      const uint64_t bal = __ballot(h);
      const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
      grel[c] = heads + below + (h ? 1 : 0) - 1;
      heads += __popcll(bal);
      if (h) {
        const int x = wbase + c * 64 + lane;
        out_keys[Gq + grel[c]] = s_key[1 + x];
        if (head_pos) head_pos[Gq + grel[c]] = (uint32_t)(base + x);
      }
    }
  }
  const int na = plan.n, rec = na + 1;
  const int wend = min(tile_n, wbase + kWSeg) - 1;  // my share's last element
  for (int a = -1; a < na; ++a) {
    const int kind = a < 0 ? DG_AGG_COUNT : plan.kind[a];
    if (kind == DG_AGG_FLOAT_SUM) continue;  // k_fsum_runs: float32 in row order
    const int op = a < 0 ? (int)OP_ADD_I64 : plan.op[a];
    const uint64_t ident = a < 0 ? 0ull : identity_of(op, kind);
    uint64_t run = ident;  // the run open at the end of the previous chunk
#pragma unroll
    for (int c = 0; c < kRSPT; ++c) {
      const int x = wbase + c * 64 + lane;
      const bool valid = x < tile_n;
      uint64_t xv;
      if (!valid) xv = ident;
      else if (a < 0) xv = 1ull;
      else if (pw <= kRegSlots) xv = a == 0 ? xr[c][0] : xr[c][1];
      else xv = payload[pay_at(pw, idx_of[c], a)];
      uint64_t v = xv;
      // a chunk of singleton groups (every element a run head and end: ~3 in 4 chunks at one group per
      // row) needs no scan; otherwise the segmented scan with the open run carried in
      const bool single = !valid || ((hm >> c) & (tm >> c) & 1u);
      if (__ballot(!single)) {
        bool f;
        v = seg_scan_wave(op, xv, (hm >> c) & 1u, &f);
        if (!f) v = combine_op(op, run, v);
        run = __shfl(v, 63, 64);
      }
      if (valid) {
        const bool t = (tm >> c) & 1u;
        if (t || x == wend) {
          const int32_t gr = grel[c];
          if (gr >= 0) {  // a group headed in my share: complete, or open at the share's end
            out_slots[(1 + a) * cap + Gq + gr] = t ? finalize_dev(kind, v) : v;
            if (!t) open_g[wt] = Gq + gr;
          } else {  // my share's share of a group headed earlier
            carry_slots[wt * rec + 1 + a] = v;
            carry_g[wt] = Gq - 1;
          }
        }
      }
    }
  }
}

// carried partials (one per tile) -> their group's record: equal groups are consecutive, so one
// segmented combine per wave and one atomic per (wave, group, slot)
__global__ __launch_bounds__(256) void k_gb_carry(const int64_t* __restrict__ carry_g, const uint64_t* __restrict__ carry_slots,
                                                  int64_t ncarry, AggPlan plan, uint64_t* __restrict__ out_slots,
                                                  int64_t cap) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int64_t g = t < ncarry ? carry_g[t] : -1;
  if (__ballot(g >= 0) == 0) return;
  const int64_t gnext = __shfl_down(g, 1, 64);
  const bool tail = lane == 63 || gnext != g;
  const int rec = plan.n + 1;
  for (int s = 0; s < rec; ++s) {
    const int op = s == 0 ? (int)OP_ADD_I64 : plan.op[s - 1];
    if (s > 0 && plan.kind[s - 1] == DG_AGG_FLOAT_SUM) continue;
    uint64_t v = g >= 0 ? carry_slots[t * rec + s] : 0ull;
    // inclusive scan restricted to the run of equal g ending at this lane (runs are contiguous)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(v, o, 64);
      const int64_t gy = __shfl_up(g, o, 64);
      if (lane >= o && gy == g) v = combine_op(op, y, v);
    }
    if (g >= 0 && tail) atomic_op(op, out_slots + s * cap + g, v);
  }
}

__global__ __launch_bounds__(256) void k_gb_open_finalize(const int64_t* __restrict__ open_g, int64_t nopen, AggPlan plan,
                                                          uint64_t* __restrict__ out_slots, int64_t cap) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t g = t < nopen ? open_g[t] : -1;
  if (g < 0) return;
  for (int a = 0; a < plan.n; ++a)
    if (plan.kind[a] != DG_AGG_FLOAT_SUM) out_slots[(1 + a) * cap + g] = finalize_dev(plan.kind[a], out_slots[(1 + a) * cap + g]);
}

void launch_gb_reduce(SortBufs* sb, AggPlan plan, uint64_t* out_keys, uint64_t* out_slots, int64_t cap,
                      uint32_t* head_pos, int64_t* carry_g, uint64_t* carry_slots, int64_t* open_g, hipStream_t s) {
  const int nt = sb->ntiles_sort;
  const uint32_t* refs = sb->refs[sb->cur];
  // the look-back status (the sort's, free again) and the tile counter; the group count starts at 0
  // (a separate k_run_count pass + scan for the tile offsets measured the same, same box: 14.17-14.29
  // vs 14.22-14.25 ms per headline step)
  uint32_t* ctr = sb->bin_total + (size_t)kRsMaxPasses * kMaxBins + kRsMaxPasses;
  if (!zero_async(sb->lb_status, (size_t)nt * sizeof(uint64_t), s)) return;
  if (!zero_async(ctr, sizeof(uint32_t), s)) return;
  if (!zero_async(sb->n + 1, sizeof(uint32_t), s)) return;
  if (refs)
    hipLaunchKernelGGL(k_gb_reduce<true>, dim3(nt), dim3(kRT), 0, s, sb->payload, sb->pw, sb->keys[sb->cur], refs,
                       sb->ref_bits, sb->n, sb->lb_status, ctr, plan, out_keys, out_slots, cap, head_pos,
                       carry_g, carry_slots, open_g);
  else
    hipLaunchKernelGGL(k_gb_reduce<false>, dim3(nt), dim3(kRT), 0, s, sb->payload, sb->pw, sb->keys[sb->cur], refs,
                       sb->ref_bits, sb->n, sb->lb_status, ctr, plan, out_keys, out_slots, cap, head_pos,
                       carry_g, carry_slots, open_g);
  const int64_t nw = (int64_t)nt * kRedWaves;  // carry / open slots: one per wave share of a tile
  const unsigned g = (unsigned)((nw + 255) / 256);
  hipLaunchKernelGGL(k_gb_carry, dim3(g), dim3(256), 0, s, carry_g, carry_slots, nw, plan, out_slots, cap);
  hipLaunchKernelGGL(k_gb_open_finalize, dim3(g), dim3(256), 0, s, open_g, nw, plan, out_slots, cap);
}

// ------------------------------------------------------------------------------------------------
// floatSum in row order (FloatSumBufferAggregator.aggregate: buf.putFloat(pos, buf.getFloat(pos) +
// selector.getFloat()), FloatSumAggregator.combine across segments)
// ------------------------------------------------------------------------------------------------
// FloatColumnSelector.getFloat of the aggregator's input (segment/*ColumnSelector coercions)
__device__ __forceinline__ float agg_float(const ColView& v, int64_t r) {
  if (v.kind == VIEW_ABSENT) return 0.0f;
  const uint8_t* p = cv_ptr(v, r);
  if (v.kind == VIEW_FLOAT) return *reinterpret_cast<const float*>(p);
  if (v.kind == VIEW_LONG) return (float)*reinterpret_cast<const int64_t*>(p);
  return (float)*reinterpret_cast<const double*>(p);
}

// Element index -> segment: the last job whose first element index (its first keygen tile's offset)
// is <= the index. Rows in an element's payload keep (segment, row) order, so the run's elements of
// one segment are consecutive in it.
__global__ __launch_bounds__(256) void k_fsum_runs(const GbJob* __restrict__ jobs, int njobs,
                                                   const uint32_t* __restrict__ tile_off, int ntiles,
                                                   const uint64_t* __restrict__ keys, const uint32_t* __restrict__ refs,
                                                   int kshift, const uint32_t* __restrict__ n_ptr,
                                                   const uint32_t* __restrict__ head_pos, const uint64_t* __restrict__ payload,
                                                   int pw, int rowref, int agg, uint64_t* __restrict__ out_slots, int64_t cap,
                                                   int rec, int desc) {
  __shared__ uint32_t s_base[kMaxCallSegs];
  const uint32_t n = n_ptr[0], ng = n_ptr[1];
  // first reference of every segment: its row base (row-ref mode) or its first element index
  for (int x = threadIdx.x; x < njobs; x += 256)
    s_base[x] = rowref ? jobs[x].row_base : jobs[x].tile_begin < ntiles ? tile_off[jobs[x].tile_begin] : n;
  __syncthreads();
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < ng; g += (int64_t)gridDim.x * 256) {
    const uint32_t i0 = head_pos[g], i1 = g + 1 < ng ? head_pos[g + 1] : n;
    float total = 0.0f, sum = 0.0f;
    int cur = -1;
    bool first = true;
    // a descending cursor adds its rows last to first (QueryableIndexStorageAdapter.java:397-403)
    for (uint32_t k = i0; k < i1; ++k) {
      const uint32_t i = desc ? i1 - 1 - (k - i0) : k;
      const uint32_t idx = elem_ref(keys[i], refs, i, kshift);
      const int seg = locate_seg(s_base, njobs, idx);
      if (seg != cur) {
        if (cur >= 0) {
          total = first ? sum : total + sum;
          first = false;
        }
        sum = 0.0f;
        cur = seg;
      }
      // the row's float input (identity 0.0f for a row its FilteredAggregator rejects: x + 0.0f == x
      // for every partial sum, which starts at +0.0f)
      sum = sum + (float)__longlong_as_double((long long)payload[pay_at(pw, idx, agg)]);
    }
    if (cur >= 0) total = first ? sum : total + sum;
    if (out_slots) {  // groupBy: the final ABI value
      out_slots[(1 + agg) * cap + g] = (uint64_t)__float_as_uint(total);
    } else if (cur >= 0) {  // per-segment engines: the run is one (segment, bucket, id) cell (device encoding)
      const GbJob& j = jobs[cur];
      const uint64_t key = keys[i0] >> kshift;
      const int64_t bucket = j.bucket_bits ? (int64_t)((key >> j.bucket_shift) & ((1ull << j.bucket_bits) - 1)) : 0;
      const int64_t id = j.ndims ? (int64_t)((key >> j.dim_shift[0]) & ((1ull << j.dim_bits[0]) - 1)) : 0;
      j.fs_out[(bucket * j.fs_mul + id) * rec + 1 + agg] = (uint64_t)__double_as_longlong((double)total);
    }
  }
}

void launch_fsum_runs(const GbJob* d_jobs, int njobs, int ntiles, SortBufs* sb, AggPlan plan, int agg,
                      const uint32_t* head_pos, uint64_t* out_slots, int64_t cap, hipStream_t s, int desc) {
  const int64_t blocks = std::min<int64_t>(8192, std::max<int64_t>(1, (sb->cap + 255) / 256));
  hipLaunchKernelGGL(k_fsum_runs, dim3((unsigned)blocks), dim3(256), 0, s, d_jobs, njobs, sb->tile_cnt, ntiles,
                     sb->keys[sb->cur], sb->refs[sb->cur], sb->ref_bits, sb->n, head_pos, sb->payload, sb->pw, sb->row_refs, agg,
                     out_slots, cap, plan.n + 1, desc);
}

// ------------------------------------------------------------------------------------------------
// finalize (for slots written in the device encoding) and unpack
// ------------------------------------------------------------------------------------------------
// slots [rec][cap] (SoA), groups n_ptr[0]
__global__ void k_slots_finalize(uint64_t* __restrict__ slots, const uint32_t* __restrict__ n_ptr, AggPlan plan, int64_t cap) {
  const int64_t ng = n_ptr[0];
  for (int a = 0; a < plan.n; ++a) {
    uint64_t* col = slots + (1 + a) * cap;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ng; i += (int64_t)gridDim.x * blockDim.x)
      col[i] = finalize_dev(plan.kind[a], col[i]);
  }
}

void launch_slots_finalize(uint64_t* slots, const uint32_t* n_ptr, int64_t cap, AggPlan plan, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>(16384, std::max<int64_t>(1, (cap + 255) / 256));
  hipLaunchKernelGGL(k_slots_finalize, dim3((unsigned)blocks), dim3(256), 0, s, slots, n_ptr, plan, cap);
}

// SoA result slots [rec][cap] -> AoS records [n][rec] (the exchange format of dg_result_export)
__global__ void k_soa_to_aos(const uint64_t* __restrict__ soa, int64_t cap, int64_t n, int rec, uint64_t* __restrict__ aos) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * rec; i += (int64_t)gridDim.x * blockDim.x)
    aos[i] = soa[(i % rec) * cap + i / rec];
}

// keys [n] and the rec slot rows [rec][cap] -> [rec][n]: row r (r = 0: the keys) is copied in 16-byte
// pieces where both rows are 16-byte aligned, else word by word (an odd n shifts every later row by 8)
__global__ __launch_bounds__(256) void k_result_compact(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ slots,
                                                        int64_t cap, int64_t n, int rec, uint64_t* __restrict__ keys2,
                                                        uint64_t* __restrict__ slots2) {
  const int r = blockIdx.y;  // 0: keys, 1 + s: slot row s
  const uint64_t* src = r == 0 ? keys : slots + (size_t)(r - 1) * cap;
  uint64_t* dst = r == 0 ? keys2 : slots2 + (size_t)(r - 1) * n;
  const int64_t stride = (int64_t)gridDim.x * 256;
  if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
    const int64_t n2 = n >> 1;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride)
      reinterpret_cast<ulonglong2*>(dst)[i] = reinterpret_cast<const ulonglong2*>(src)[i];
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) dst[n - 1] = src[n - 1];
  } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) dst[i] = src[i];
  }
}

void launch_result_compact(const uint64_t* keys, const uint64_t* slots, int64_t cap, int64_t n, int rec, uint64_t* keys2,
                           uint64_t* slots2, hipStream_t s) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n / 2 + 255) / 256 + 1, 2048);
  hipLaunchKernelGGL(k_result_compact, dim3((unsigned)blocks, (unsigned)(rec + 1)), dim3(256), 0, s, keys, slots, cap, n, rec,
                     keys2, slots2);
}

void launch_soa_to_aos(const uint64_t* soa, int64_t cap, int64_t n, int rec, uint64_t* aos, hipStream_t s) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>(16384, (n * rec + 255) / 256);
  hipLaunchKernelGGL(k_soa_to_aos, dim3((unsigned)blocks), dim3(256), 0, s, soa, cap, n, rec, aos);
}

__global__ void k_gb_unpack(const uint64_t* __restrict__ keys, int64_t start, int64_t count, KeyLayout lay,
                            int64_t* __restrict__ bucket, int32_t* __restrict__ ids) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[start + i];
    bucket[i] = lay.bucket_bits ? (int64_t)((k >> lay.bucket_shift) & ((1ull << lay.bucket_bits) - 1)) : 0;
    for (int d = 0; d < lay.ndims; ++d)
      ids[i * lay.ndims + d] = lay.dim_bits[d] ? (int32_t)((k >> lay.dim_shift[d]) & ((1ull << lay.dim_bits[d]) - 1)) : 0;
  }
}

void launch_gb_unpack(const uint64_t* keys, int64_t start, int64_t count, KeyLayout lay, int64_t* bucket, int32_t* ids,
                      hipStream_t s) {
  if (count <= 0) return;
  const int64_t blocks = std::min<int64_t>(16384, (count + 255) / 256);
  hipLaunchKernelGGL(k_gb_unpack, dim3((unsigned)blocks), dim3(256), 0, s, keys, start, count, lay, bucket, ids);
}

// groups [start, start + count) of a result packed for one host copy: bucket times [count] (ALL: the
// universal time; grid: bucket0 + index * period; calendar: bounds[bucket0 + index]), dimension ids
// [count][ndims], then the ABI values [count][naggs] (the slot-major rows of `slots` transposed);
// a null region pointer skips it
__global__ void k_gb_fetch_pack(const uint64_t* __restrict__ keys, const uint64_t* __restrict__ slots, int64_t cap,
                                int64_t start, int64_t count, KeyLayout lay, int naggs, int64_t universal,
                                int64_t bucket0, int64_t period, const int64_t* __restrict__ bounds,
                                int64_t* __restrict__ times, int32_t* __restrict__ ids, uint64_t* __restrict__ vals) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[start + i];
    if (times) {
      const int64_t b = lay.bucket_bits ? (int64_t)((k >> lay.bucket_shift) & ((1ull << lay.bucket_bits) - 1)) : 0;
      times[i] = !period ? universal : bounds ? bounds[bucket0 + b] : bucket0 + b * period;
    }
    if (ids)
      for (int d = 0; d < lay.ndims; ++d)
        ids[i * lay.ndims + d] = lay.dim_bits[d] ? (int32_t)((k >> lay.dim_shift[d]) & ((1ull << lay.dim_bits[d]) - 1)) : 0;
    if (vals)
      for (int a = 0; a < naggs; ++a) vals[i * naggs + a] = slots[(size_t)(1 + a) * cap + start + i];
  }
}

void launch_gb_fetch_pack(const uint64_t* keys, const uint64_t* slots, int64_t cap, int64_t start, int64_t count,
                          KeyLayout lay, int naggs, int64_t universal, int64_t bucket0, int64_t period,
                          const int64_t* bounds, int64_t* times, int32_t* ids, uint64_t* vals, hipStream_t s) {
  if (count <= 0) return;
  const int64_t blocks = std::min<int64_t>(16384, (count + 255) / 256);
  hipLaunchKernelGGL(k_gb_fetch_pack, dim3((unsigned)blocks), dim3(256), 0, s, keys, slots, cap, start, count, lay, naggs,
                     universal, bucket0, period, bounds, times, ids, vals);
}

// ------------------------------------------------------------------------------------------------
// cross-device merge (QueryRunnerFactory.mergeRunners over the devices' merged groups): re-key a
// result into the cluster key space, split it by key range, merge the received partials
// ------------------------------------------------------------------------------------------------
__global__ void k_gb_rekey(const uint64_t* __restrict__ in, int64_t n, KeyLayout lin, KeyLayout lout,
                           int64_t bucket_delta, RekeyMaps maps, uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = in[i];
    uint64_t o = 0;
    if (lout.bucket_bits) {
      const int64_t b = lin.bucket_bits ? (int64_t)((k >> lin.bucket_shift) & ((1ull << lin.bucket_bits) - 1)) : 0;
      o |= (uint64_t)(b + bucket_delta) << lout.bucket_shift;
    }
    for (int d = 0; d < lout.ndims; ++d) {
      const uint32_t id = lin.dim_bits[d] ? (uint32_t)((k >> lin.dim_shift[d]) & ((1ull << lin.dim_bits[d]) - 1)) : 0u;
      o |= (uint64_t)(uint32_t)maps.m[d][id] << lout.dim_shift[d];
    }
    out[i] = o;
  }
}

void launch_gb_rekey(const uint64_t* in, int64_t n, KeyLayout lin, KeyLayout lout, int64_t bucket_delta,
                     RekeyMaps maps, uint64_t* out, hipStream_t s) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>(16384, (n + 255) / 256);
  hipLaunchKernelGGL(k_gb_rekey, dim3((unsigned)blocks), dim3(256), 0, s, in, n, lin, lout, bucket_delta, maps, out);
}

// pos[i] = first index of the ascending keys[0, n) whose key >= split[i]
__global__ void k_lower_bound(const uint64_t* __restrict__ keys, int64_t n, const uint64_t* __restrict__ split, int nsplit,
                              int64_t* __restrict__ pos) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsplit) return;
  const uint64_t x = split[i];
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  pos[i] = lo;
}

void launch_lower_bound(const uint64_t* keys, int64_t n, const uint64_t* split, int nsplit, int64_t* pos, hipStream_t s) {
  if (nsplit <= 0) return;
  hipLaunchKernelGGL(k_lower_bound, dim3((nsplit + 255) / 256), dim3(256), 0, s, keys, n, split, nsplit, pos);
}

// sort input of a merge: the concatenated partials' keys, row refs = record index; n[0] = n
__global__ void k_merge_load(const uint64_t* __restrict__ keys, int64_t n, uint64_t* __restrict__ kout,
                             uint32_t* __restrict__ rout, int kshift, uint32_t* __restrict__ n_out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) n_out[0] = (uint32_t)n;
  for (int64_t i = t; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (rout) {
      kout[i] = keys[i];
      rout[i] = (uint32_t)i;
    } else {
      kout[i] = (keys[i] << kshift) | (uint64_t)i;
    }
  }
}

void launch_merge_load(const uint64_t* keys, int64_t n, SortBufs* sb, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>(16384, std::max<int64_t>(1, (n + 255) / 256));
  hipLaunchKernelGGL(k_merge_load, dim3((unsigned)blocks), dim3(256), 0, s, keys, n, sb->keys[sb->cur], sb->refs[sb->cur],
                     sb->ref_bits, sb->n);
}

// ------------------------------------------------------------------------------------------------
// limit push-down (GroupByQuery.getRowOrderingForPushDown, GroupByQuery.java:423-528): a result's
// keys re-packed with their fields in the push-down order (comparator ranks, descending columns
// complemented), sorted, and the first `limit` groups gathered in that order
// ------------------------------------------------------------------------------------------------
__global__ void k_limit_load(const uint64_t* __restrict__ keys, int64_t n, LimitOrder o, uint64_t* __restrict__ kout,
                             uint32_t* __restrict__ rout, int kshift, uint32_t* __restrict__ n_out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) n_out[0] = (uint32_t)n;
  for (int64_t i = t; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    uint64_t ord = 0;
    for (int f = 0; f < o.nfields; ++f) {
      const uint64_t m = (1ull << o.bits[f]) - 1ull;
      uint64_t v = (k >> o.in_shift[f]) & m;
      if (o.rank[f]) v = (uint64_t)(uint32_t)o.rank[f][v];
      if (o.desc[f]) v = m - v;
      ord |= v << o.out_shift[f];
    }
    if (rout) {
      kout[i] = ord;
      rout[i] = (uint32_t)i;
    } else {
      kout[i] = (ord << kshift) | (uint64_t)i;
    }
  }
}

void launch_limit_load(const uint64_t* keys, int64_t n, const LimitOrder& o, SortBufs* sb, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>(16384, std::max<int64_t>(1, (n + 255) / 256));
  hipLaunchKernelGGL(k_limit_load, dim3((unsigned)blocks), dim3(256), 0, s, keys, n, o, sb->keys[sb->cur],
                     sb->refs[sb->cur], sb->ref_bits, sb->n);
}

__global__ void k_limit_gather(const uint64_t* __restrict__ skeys, const uint32_t* __restrict__ srefs, int kshift,
                               int64_t m, const uint64_t* __restrict__ keys, const uint64_t* __restrict__ slots,
                               int64_t cap, int rec, uint64_t* __restrict__ okeys, uint64_t* __restrict__ oslots,
                               int64_t ocap) {
  const uint64_t rmask = kshift ? (1ull << kshift) - 1ull : 0ull;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t src = srefs ? (int64_t)srefs[i] : (int64_t)(skeys[i] & rmask);
    okeys[i] = keys[src];
    for (int s = 0; s < rec; ++s) oslots[(size_t)s * ocap + i] = slots[(size_t)s * cap + src];
  }
}

void launch_limit_gather(const SortBufs* sb, int64_t m, const uint64_t* keys, const uint64_t* slots, int64_t cap,
                         int rec, uint64_t* okeys, uint64_t* oslots, int64_t ocap, hipStream_t s) {
  if (m <= 0) return;
  const int64_t blocks = std::min<int64_t>(16384, (m + 255) / 256);
  hipLaunchKernelGGL(k_limit_gather, dim3((unsigned)blocks), dim3(256), 0, s, sb->keys[sb->cur], sb->refs[sb->cur],
                     sb->ref_bits, m, keys, slots, cap, rec, okeys, oslots, ocap);
}

// AggregatorFactory.getCombiningFactory semantics on ABI-encoded partial values: the combining
// aggregator starts from its identity and folds the partials in order (sums: LongSumAggregator /
// DoubleSumAggregator / FloatSumAggregator.combine with float adds; min / max: Math.min / Math.max,
// NaN-propagating with -0.0 < 0.0, DoubleMinAggregator.combine etc.)
__device__ __forceinline__ uint64_t abi_to_dev(int kind, uint64_t v) {
  switch (kind) {
    case DG_AGG_COUNT:
    case DG_AGG_LONG_SUM:
    case DG_AGG_DOUBLE_SUM: return v;
    case DG_AGG_FLOAT_SUM: return (uint64_t)__double_as_longlong((double)__uint_as_float((uint32_t)v));
    case DG_AGG_LONG_MIN:
    case DG_AGG_LONG_MAX: return v ^ kSign;
    case DG_AGG_DOUBLE_MIN:
    case DG_AGG_DOUBLE_MAX: {
      const double d = __longlong_as_double((long long)v);
      return d != d ? (kind == DG_AGG_DOUBLE_MIN ? 0ull : ~0ull) : ord_key(d);
    }
    default: {
      const float f = __uint_as_float((uint32_t)v);
      return f != f ? (kind == DG_AGG_FLOAT_MIN ? 0ull : ~0ull) : ord_key((double)f);
    }
  }
}

__global__ __launch_bounds__(256) void k_merge_reduce(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ refs,
                                                      int kshift, const uint32_t* __restrict__ n_ptr,
                                                      const uint32_t* __restrict__ head_pos,
                                                      const uint64_t* __restrict__ in_slots, AggPlan plan,
                                                      uint64_t* __restrict__ out_keys, uint64_t* __restrict__ out_slots,
                                                      int64_t cap) {
  const uint32_t n = n_ptr[0], ng = n_ptr[1];
  const int na = plan.n, rec = na + 1;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < ng; g += (int64_t)gridDim.x * 256) {
    const uint32_t i0 = head_pos[g], i1 = g + 1 < ng ? head_pos[g + 1] : n;
    out_keys[g] = keys[i0] >> kshift;
    uint64_t rows = 0;
    for (uint32_t i = i0; i < i1; ++i) rows += in_slots[(size_t)elem_ref(keys[i], refs, i, kshift) * rec];
    out_slots[g] = rows;
    for (int a = 0; a < na; ++a) {
      const int kind = plan.kind[a];
      if (kind == DG_AGG_FLOAT_SUM) {  // float adds in partial order
        float acc = 0.0f;
        for (uint32_t i = i0; i < i1; ++i)
          acc = acc + __uint_as_float((uint32_t)in_slots[(size_t)elem_ref(keys[i], refs, i, kshift) * rec + 1 + a]);
        out_slots[(1 + a) * cap + g] = (uint64_t)__double_as_longlong((double)acc);  // finalized later
        continue;
      }
      uint64_t acc = identity_of(plan.op[a], kind);
      for (uint32_t i = i0; i < i1; ++i)
        acc = combine_op(plan.op[a], acc, abi_to_dev(kind, in_slots[(size_t)elem_ref(keys[i], refs, i, kshift) * rec + 1 + a]));
      out_slots[(1 + a) * cap + g] = acc;
    }
  }
}

void launch_merge_reduce(SortBufs* sb, const uint32_t* head_pos, const uint64_t* in_slots, AggPlan plan, int64_t cap,
                         uint64_t* out_keys, uint64_t* out_slots, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>(8192, std::max<int64_t>(1, (cap + 255) / 256));
  hipLaunchKernelGGL(k_merge_reduce, dim3((unsigned)blocks), dim3(256), 0, s, sb->keys[sb->cur], sb->refs[sb->cur],
                     sb->ref_bits, sb->n, head_pos, in_slots, plan, out_keys, out_slots, cap);
}

}  // namespace dg
