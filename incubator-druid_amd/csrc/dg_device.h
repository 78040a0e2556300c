// dg_device.h — device helpers shared by the HIP translation units (dg_kernels.hip, dg_sort.hip):
// column views, dictionary-id loads, Java-semantics aggregator inputs and slot operations.
#pragma once

#include <hip/hip_runtime.h>

#include "dg_internal.h"

namespace dg {

constexpr uint64_t kSign = 0x8000000000000000ull;

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t ord_key(double d) {
  uint64_t u = __double_as_longlong(d);
  return (u & kSign) ? ~u : (u | kSign);
}
__device__ __forceinline__ double unord_key(uint64_t k) {
  uint64_t u = (k & kSign) ? (k & ~kSign) : ~k;
  return __longlong_as_double((long long)u);
}
// java (long) double: NaN -> 0, saturating
__device__ __forceinline__ int64_t java_d2l(double d) {
  if (d != d) return 0;
  if (d >= 9223372036854775807.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}

// bucket coordinate of timestamp t: t itself on a period grid, or (calendar granularity, caller-given
// bucket starts b[0..n)) the index of the last start <= t (-1 before the first)
__device__ __forceinline__ int64_t bucket_coord(const int64_t* __restrict__ b, int32_t n, int64_t t) {
  if (!b) return t;
  int lo = 0, len = n;
  while (len > 0) {
    const int h = len >> 1;
    if (b[lo + h] <= t) {
      lo += h + 1;
      len -= h + 1;
    } else {
      len = h;
    }
  }
  return (int64_t)lo - 1;
}

__device__ __forceinline__ const uint8_t* cv_ptr(const ColView& v, int64_t r) {
  const uint8_t* base = v.blocks[r >> v.log2_per];
  return base + (size_t)(r & ((1ll << v.log2_per) - 1)) * (size_t)v.width;
}

// The cursor time of row r (the scan's __time view): a block whose rows all share one bucket and lie
// inside the interval is not decoded; its pointer is tagged (low bit) and points at one representative
// timestamp (the block's first row time), which gives every row of the block the same bucket and
// interval verdict as its own time would.
__device__ __forceinline__ int64_t load_time(const ColView& v, int64_t r) {
  const uintptr_t b = reinterpret_cast<uintptr_t>(v.blocks[r >> v.log2_per]);
  if (b & 1u) return *reinterpret_cast<const int64_t*>(b & ~(uintptr_t)1);
  return *reinterpret_cast<const int64_t*>(reinterpret_cast<const uint8_t*>(b) +
                                           (size_t)(r & ((1ll << v.log2_per) - 1)) * 8);
}

// a width-byte big-endian id read as little-endian -> its value (VSizeColumnarInts.get, :124-127)
__device__ __forceinline__ uint32_t id_bswap(uint32_t x, int width) {
  const uint32_t b = __builtin_bswap32(x);
  return width >= 4 ? b : b >> (32 - 8 * width);
}

__device__ __forceinline__ uint32_t load_id(const ColView& v, int64_t r) {
  const uint8_t* p = cv_ptr(v, r);
  if (v.pad & kViewBigEndian) {  // uncompressed VSizeColumnarInts: big-endian, byte aligned
    uint32_t x = 0;
    for (int k = 0; k < v.width; ++k) x = (x << 8) | p[k];
    return x;
  }
  switch (v.width) {
    case 1: return p[0];
    case 2: return *reinterpret_cast<const uint16_t*>(p);
    case 3: return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16);
    default: return *reinterpret_cast<const uint32_t*>(p);
  }
}

// Input of one aggregator for row r, encoded for its slot op.
// Selector coercions follow LongColumnSelector / DoubleColumnSelector / FloatColumnSelector
// (segment/DoubleColumnSelector.java:40-55): getLong of a double = (long) d, getFloat = (float) x, ...
// the aggregator input of a value at p (a view of kind vkind; p unused for VIEW_ABSENT)
__device__ __forceinline__ uint64_t agg_input_at(int kind, int vkind, const uint8_t* p) {
  int64_t l = 0;
  double d = 0.0;
  float f = 0.0f;
  if (kind != DG_AGG_COUNT && vkind != VIEW_ABSENT) {
    if (vkind == VIEW_LONG) {
      l = *reinterpret_cast<const int64_t*>(p);
      d = (double)l;
      f = (float)l;
    } else if (vkind == VIEW_DOUBLE) {
      d = *reinterpret_cast<const double*>(p);
      l = java_d2l(d);
      f = (float)d;
    } else {
      f = *reinterpret_cast<const float*>(p);
      d = (double)f;
      l = java_d2l(d);
    }
  }
  switch (kind) {
    case DG_AGG_COUNT: return 1;
    case DG_AGG_LONG_SUM: return (uint64_t)l;
    case DG_AGG_DOUBLE_SUM: return (uint64_t)__double_as_longlong(d);
    case DG_AGG_FLOAT_SUM: return (uint64_t)__double_as_longlong((double)f);
    case DG_AGG_LONG_MIN:
    case DG_AGG_LONG_MAX: return (uint64_t)l ^ kSign;
    case DG_AGG_DOUBLE_MIN: return d != d ? 0ull : ord_key(d);
    case DG_AGG_DOUBLE_MAX: return d != d ? ~0ull : ord_key(d);
    case DG_AGG_FLOAT_MIN: return f != f ? 0ull : ord_key((double)f);
    default: return f != f ? ~0ull : ord_key((double)f);  // FLOAT_MAX
  }
}

__device__ __forceinline__ uint64_t agg_input(int kind, const ColView& v, int64_t r) {
  return agg_input_at(kind, v.kind, kind != DG_AGG_COUNT && v.kind != VIEW_ABSENT ? cv_ptr(v, r) : nullptr);
}

// ---- four consecutive rows r .. r + 3 (r % 4 == 0, all inside the view's block): one or a few
// wide loads per column instead of four scalar ones; consecutive threads read consecutive quads, so
// every load instruction of a wave is one contiguous span ----
__device__ __forceinline__ void load_ids4_le(const ColView& v, int64_t r, uint32_t id[4]) {
  const uint8_t* p = cv_ptr(v, r);
  switch (v.width) {
    case 1: {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
#pragma unroll
      for (int k = 0; k < 4; ++k) id[k] = (w >> (8 * k)) & 0xFF;
      break;
    }
    case 2: {
      const uint2 w = *reinterpret_cast<const uint2*>(p);
      id[0] = w.x & 0xFFFF;
      id[1] = w.x >> 16;
      id[2] = w.y & 0xFFFF;
      id[3] = w.y >> 16;
      break;
    }
    case 3: {
      const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
      const uint32_t a = q[0], b = q[1], c = q[2];
      id[0] = a & 0xFFFFFF;
      id[1] = (a >> 24) | ((b & 0xFFFF) << 8);
      id[2] = (b >> 16) | ((c & 0xFF) << 16);
      id[3] = c >> 8;
      break;
    }
    default: {
      const uint4 w = *reinterpret_cast<const uint4*>(p);
      id[0] = w.x;
      id[1] = w.y;
      id[2] = w.z;
      id[3] = w.w;
    }
  }
}

__device__ __forceinline__ void load_ids4(const ColView& v, int64_t r, uint32_t id[4]) {
  load_ids4_le(v, r, id);
  if (v.pad & kViewBigEndian) {
#pragma unroll
    for (int k = 0; k < 4; ++k) id[k] = id_bswap(id[k], v.width);
  }
}

// cursor times of rows r .. r + 3 (r % 4 == 0, inside one block; see load_time)
__device__ __forceinline__ void load_time4(const ColView& v, int64_t r, uint64_t t[4]) {
  const uintptr_t b = reinterpret_cast<uintptr_t>(v.blocks[r >> v.log2_per]);
  if (b & 1u) {
    const uint64_t x = *reinterpret_cast<const uint64_t*>(b & ~(uintptr_t)1);
    t[0] = t[1] = t[2] = t[3] = x;
    return;
  }
  const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(b) + (size_t)(r & ((1ll << v.log2_per) - 1)) * 8);
  const uint4 a = p[0], c = p[1];
  t[0] = (uint64_t)a.x | ((uint64_t)a.y << 32);
  t[1] = (uint64_t)a.z | ((uint64_t)a.w << 32);
  t[2] = (uint64_t)c.x | ((uint64_t)c.y << 32);
  t[3] = (uint64_t)c.z | ((uint64_t)c.w << 32);
}

// raw 8-byte lanes of a numeric view for rows r .. r + 3 (float views: 4-byte values in the low half)
__device__ __forceinline__ void load_raw4(const ColView& v, int64_t r, uint64_t x[4]) {
  const uint8_t* p = cv_ptr(v, r);
  if (v.kind == VIEW_FLOAT) {
    const uint4 w = *reinterpret_cast<const uint4*>(p);
    x[0] = w.x;
    x[1] = w.y;
    x[2] = w.z;
    x[3] = w.w;
  } else {
    const uint4 a = reinterpret_cast<const uint4*>(p)[0], b = reinterpret_cast<const uint4*>(p)[1];
    x[0] = (uint64_t)a.x | ((uint64_t)a.y << 32);
    x[1] = (uint64_t)a.z | ((uint64_t)a.w << 32);
    x[2] = (uint64_t)b.x | ((uint64_t)b.y << 32);
    x[3] = (uint64_t)b.z | ((uint64_t)b.w << 32);
  }
}

// agg_input on an already loaded raw lane (same coercions)
__device__ __forceinline__ uint64_t agg_input_raw(int kind, int view_kind, uint64_t raw) {
  int64_t l = 0;
  double d = 0.0;
  float f = 0.0f;
  if (kind != DG_AGG_COUNT && view_kind != VIEW_ABSENT) {
    if (view_kind == VIEW_LONG) {
      l = (int64_t)raw;
      d = (double)l;
      f = (float)l;
    } else if (view_kind == VIEW_DOUBLE) {
      d = __longlong_as_double((long long)raw);
      l = java_d2l(d);
      f = (float)d;
    } else {
      f = __uint_as_float((uint32_t)raw);
      d = (double)f;
      l = java_d2l(d);
    }
  }
  switch (kind) {
    case DG_AGG_COUNT: return 1;
    case DG_AGG_LONG_SUM: return (uint64_t)l;
    case DG_AGG_DOUBLE_SUM: return (uint64_t)__double_as_longlong(d);
    case DG_AGG_FLOAT_SUM: return (uint64_t)__double_as_longlong((double)f);
    case DG_AGG_LONG_MIN:
    case DG_AGG_LONG_MAX: return (uint64_t)l ^ kSign;
    case DG_AGG_DOUBLE_MIN: return d != d ? 0ull : ord_key(d);
    case DG_AGG_DOUBLE_MAX: return d != d ? ~0ull : ord_key(d);
    case DG_AGG_FLOAT_MIN: return f != f ? 0ull : ord_key((double)f);
    default: return f != f ? ~0ull : ord_key((double)f);  // FLOAT_MAX
  }
}

__device__ __forceinline__ uint64_t combine_op(int op, uint64_t a, uint64_t b) {
  switch (op) {
    case OP_ADD_I64: return a + b;
    case OP_ADD_F64: return (uint64_t)__double_as_longlong(__longlong_as_double((long long)a) + __longlong_as_double((long long)b));
    case OP_MIN_U64: return a < b ? a : b;
    default: return a > b ? a : b;
  }
}

__device__ __forceinline__ void atomic_op(int op, uint64_t* p, uint64_t v) {
  switch (op) {
    case OP_ADD_I64: atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v); break;
    case OP_ADD_F64: atomicAdd(reinterpret_cast<double*>(p), __longlong_as_double((long long)v)); break;
    case OP_MIN_U64: atomicMin(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v); break;
    default: atomicMax(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v); break;
  }
}

__device__ __forceinline__ uint64_t identity_of(int op, int kind) {
  switch (op) {
    case OP_ADD_I64: return 0;
    case OP_ADD_F64: return 0;  // +0.0
    case OP_MIN_U64:
      if (kind == DG_AGG_LONG_MIN) return (uint64_t)INT64_MAX ^ kSign;
      return 0xFFF0000000000000ull;  // ord_key(+inf)
    default:
      if (kind == DG_AGG_LONG_MAX) return (uint64_t)INT64_MIN ^ kSign;
      return 0x000FFFFFFFFFFFFFull;  // ord_key(-inf)
  }
}

// FilteredAggregatorFactory: a row the aggregator's matcher rejects contributes the slot identity
// (FilteredBufferAggregator.aggregate skips the delegate; the record keeps its init value)
__device__ __forceinline__ bool agg_row(const uint32_t* bits, int64_t r) {
  return !bits || ((bits[r >> 5] >> (r & 31)) & 1u);
}
__device__ __forceinline__ unsigned agg_quad(const uint32_t* bits, int64_t r) {  // r % 4 == 0
  return bits ? (bits[r >> 5] >> (r & 31)) & 0xFu : 0xFu;
}
template <class Job>
__device__ __forceinline__ uint64_t agg_in(const Job& j, const AggPlan& plan, int a, int64_t r) {
  return agg_row(j.agg_bits[a], r) ? agg_input(plan.kind[a], j.vals[a], r) : identity_of(plan.op[a], plan.kind[a]);
}

// agg_in for the timeseries scan: rows of a block the decoder already aggregated (kViewFused view,
// tagged block pointer) contribute the identity
template <class Job>
__device__ __forceinline__ uint64_t agg_in_scan(const Job& j, const AggPlan& plan, int a, int64_t r) {
  const ColView& v = j.vals[a];
  if ((v.pad & kViewFused) && (reinterpret_cast<uintptr_t>(v.blocks[r >> v.log2_per]) & 1u))
    return identity_of(plan.op[a], plan.kind[a]);
  return agg_in(j, plan, a, r);
}

}  // namespace dg
