// dg_engine.cpp — C-ABI entry points and query execution on one device.
//
// Host side of the per-segment runners (reference: TimeseriesQueryEngine.process, TopNQueryEngine.query +
// PooledTopNAlgorithm, GroupByQueryEngineV2.process). The host resolves filters against the segment
// dictionaries (BitmapIndexSelector semantics), computes granularity buckets from the segment time
// bounds (QueryableIndexStorageAdapter.makeCursors:190-316 + CursorSequenceBuilder.build:367-456),
// builds the kernel job tables and launches; every row-level operation runs on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <functional>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <queue>
#include <unordered_map>
#include <string>
#include <string_view>
#include <vector>

#include "dg_internal.h"

namespace dg {

// ------------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------------
static thread_local char g_err[1024] = "";
static thread_local uint64_t g_err_count = 0;  // set_error calls on this thread (CallGuard: did the call fail?)

static thread_local hipError_t g_launch_err = hipSuccess;
void note_launch_error(hipError_t e) {
  if (g_launch_err == hipSuccess) g_launch_err = e;
}
hipError_t take_launch_error() {
  const hipError_t e = g_launch_err;
  g_launch_err = hipSuccess;
  return e;
}

int set_error(int code, const char* fmt, ...) {
  ++g_err_count;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}

void DevBuf::reset() {
  if (p) hipFree(p);
  p = nullptr;
  n = 0;
}

bool DevBuf::alloc(size_t bytes) {
  reset();
  if (bytes == 0) bytes = 16;
  if (hipMalloc(&p, bytes) != hipSuccess) {
    p = nullptr;
    return false;
  }
  n = bytes;
  return true;
}

// ------------------------------------------------------------------------------------------------
// per-call device/pinned scratch
// ------------------------------------------------------------------------------------------------
struct Pool {
  struct Chunk {
    void* p;
    size_t n;
  };
  std::vector<Chunk> chunks;
  size_t cur = 0, off = 0;
  bool pinned = false;
  ~Pool() {
    for (auto& c : chunks) {
      if (pinned) hipHostFree(c.p);
      else hipFree(c.p);
    }
  }
  void reset() {
    cur = 0;
    off = 0;
  }
  void* take(size_t n) {
    n = (n + 255) & ~(size_t)255;
    while (cur < chunks.size()) {
      if (off + n <= chunks[cur].n) {
        void* r = (char*)chunks[cur].p + off;
        off += n;
        return r;
      }
      cur++;
      off = 0;
    }
    size_t sz = std::max(n, (size_t)64 << 20);
    void* p = nullptr;
    hipError_t e = pinned ? hipHostMalloc(&p, sz, hipHostMallocDefault) : hipMalloc(&p, sz);
    if (e != hipSuccess) return nullptr;
    chunks.push_back({p, sz});
    cur = chunks.size() - 1;
    off = n;
    return p;
  }
};

// Host->device staging: tables built on the host go into a pinned chunk mirrored by a device chunk
// and leave in ONE copy per launch group (up_flush), instead of one hipMemcpyAsync per table.
struct UpPool {
  struct Chunk {
    void* h;
    void* d;
    size_t n;
  };
  std::vector<Chunk> chunks;
  size_t cur = 0, off = 0, flushed = 0;
  ~UpPool() {
    for (auto& c : chunks) {
      hipHostFree(c.h);
      hipFree(c.d);
    }
  }
  void reset() {
    cur = 0;
    off = 0;
    flushed = 0;
  }
  bool flush(hipStream_t st) {
    if (cur < chunks.size() && off > flushed) {
      const Chunk& c = chunks[cur];
      if (hipMemcpyAsync((char*)c.d + flushed, (char*)c.h + flushed, off - flushed, hipMemcpyHostToDevice, st) !=
          hipSuccess)
        return false;
    }
    flushed = off;
    return true;
  }
  // do device addresses [lo, hi) lie in one chunk
  bool one_chunk(const void* lo, const void* hi) const {
    for (const auto& c : chunks) {
      const char* d = static_cast<const char*>(c.d);
      if (static_cast<const char*>(lo) >= d && static_cast<const char*>(hi) <= d + c.n) return true;
    }
    return false;
  }
  void* take(size_t n, void** dev, hipStream_t st) {
    n = (n + 255) & ~(size_t)255;
    if (cur >= chunks.size() || off + n > chunks[cur].n) {
      if (!flush(st)) return nullptr;
      size_t next = cur < chunks.size() ? cur + 1 : 0;
      while (next < chunks.size() && chunks[next].n < n) next++;
      if (next >= chunks.size()) {
        Chunk c{nullptr, nullptr, std::max(n, (size_t)8 << 20)};
        if (hipHostMalloc(&c.h, c.n, hipHostMallocDefault) != hipSuccess) return nullptr;
        if (hipMalloc(&c.d, c.n) != hipSuccess) {
          hipHostFree(c.h);
          return nullptr;
        }
        chunks.push_back(c);
        next = chunks.size() - 1;
      }
      cur = next;
      off = 0;
      flushed = 0;
    }
    void* h = (char*)chunks[cur].h + off;
    *dev = (char*)chunks[cur].d + off;
    off += n;
    return h;
  }
};

// Interruption of a query call: the scan's cancel flag (Thread.interrupt / QueryWatcher.cancel,
// BaseQuery.checkInterrupted, BaseQuery.java:46-51) and the context's timeout measured from the call's
// start (ChainedExecutionQueryRunner.java:150-167: futures.get(timeout) -> QueryInterruptedException(
// TimeoutException)). Checked between launch groups and while finish_call waits for the device.
struct Interrupt {
  const volatile int32_t* cancel = nullptr;
  bool timed = false;
  int64_t timeout_ms = 0;
  std::chrono::steady_clock::time_point deadline;
  // DG_DEBUG_CANCEL_AT=k (tests): the call's k-th check finds its cancel flag set — written here, as
  // another thread would, at a fixed point of the call (k = 2: after its first launch group)
  int cancel_at = 0;
  mutable int checks = 0;
  Interrupt(const dg_scan* q, std::chrono::steady_clock::time_point t0) {
    if (!q) return;
    cancel = q->cancel;
    if (cancel) {
      const char* v = getenv("DG_DEBUG_CANCEL_AT");
      cancel_at = v ? atoi(v) : 0;
    }
    if (q->timeout_ms > 0) {
      timed = true;
      timeout_ms = q->timeout_ms;
      deadline = t0 + std::chrono::milliseconds(q->timeout_ms);
    }
  }
  bool active() const { return cancel || timed; }
  int check() const {
    if (cancel_at > 0 && ++checks >= cancel_at) *const_cast<volatile int32_t*>(cancel) = 1;
    if (cancel && *cancel) return set_error(DG_ERR_INTERRUPTED, "query cancelled");
    if (timed && std::chrono::steady_clock::now() >= deadline)
      return set_error(DG_ERR_TIMEOUT, "query timeout (%lld ms)", (long long)timeout_ms);
    return DG_OK;
  }
};
#define DG_CHECK_INTERRUPT(intr)       \
  do {                                 \
    const int _irc = (intr).check();   \
    if (_irc) return _irc;             \
  } while (0)

struct CallScratch {
  const Interrupt* intr = nullptr;  // the running query call's (null outside query calls)
  Pool dev;
  Pool host;
  UpPool up;
  // per-call device error word (bit 0: corrupt LZ4 block, bit 1: corrupt Roaring bitmap, bit 2:
  // corrupt multi-value row lists), read once
  // at the call's final synchronisation instead of after every kernel
  int32_t* d_err = nullptr;
  int32_t* h_err = nullptr;
  // the call's filtered-row counts (build_bitset): one zeroed staged block, read back once with the
  // error word at the call's final synchronisation instead of one copy per filter
  unsigned long long* cnt_d = nullptr;
  unsigned long long* cnt_h = nullptr;
  int cnt_used = 0;
  // device -> host reads of staged (upload-pool) words due at the call's final synchronisation:
  // finish_call moves them with one copy of the span holding them all
  struct LateRead {
    void* h;
    const void* d;
    size_t n;
  };
  std::vector<LateRead> late;
  Context* ctx = nullptr;
  // algorithmic bytes of the call's filter bitmaps (dg_metrics.bitmap_bytes): serialized bitmaps
  // read + every row bitset written and read once
  int64_t bitmap_bytes = 0;
  CallScratch() { host.pinned = true; }
  void reset() {
    dev.reset();
    host.reset();
    up.reset();
    d_err = nullptr;
    h_err = nullptr;
    cnt_d = nullptr;
    cnt_h = nullptr;
    cnt_used = 0;
    late.clear();
    bitmap_bytes = 0;
    intr = nullptr;
  }
};

static CallScratch* scratch_of(Context* ctx) {
  static std::mutex m;
  static std::map<Context*, CallScratch*> s;
  std::lock_guard<std::mutex> g(m);
  auto it = s.find(ctx);
  if (it != s.end()) return it->second;
  CallScratch* c = new CallScratch();
  c->ctx = ctx;
  s[ctx] = c;
  return c;
}

template <class T>
static T* dev_take(CallScratch* cs, size_t count) {
  return static_cast<T*>(cs->dev.take(count * sizeof(T)));
}
template <class T>
static T* host_take(CallScratch* cs, size_t count) {
  return static_cast<T*>(cs->host.take(count * sizeof(T)));
}
// staged upload of `count` T: returns the host view to fill, *dev = its device address (valid for
// kernels after the next up_flush)
template <class T>
static T* up_take(CallScratch* cs, size_t count, T** dev, hipStream_t st) {
  void* d = nullptr;
  T* h = static_cast<T*>(cs->up.take(std::max<size_t>(count, 1) * sizeof(T), &d, st));
  *dev = static_cast<T*>(d);
  return h;
}
#define DG_FLUSH(cs, st)                                                                   \
  do {                                                                                     \
    if (!(cs)->up.flush(st)) return ::dg::set_error(DG_ERR_DEVICE, "staged upload failed"); \
  } while (0)

// A phase-timing event (dg_metrics' *_ms fields). dg_set_phase_timing(0) or DG_NO_PHASE_EVENTS=1 leaves
// them out (the phase times then read 0): a small query pays ~25 us for the timestamps. Only timing
// events go through phase_event: an event another stream waits on is always recorded (hipEventRecord).
// The switch is read once per call (CallGuard sets t_phase_on), so a toggle from another thread while a
// call runs cannot make it read elapsed times of events it never recorded.
static std::atomic<bool> g_phase_timing{true};
static thread_local bool t_phase_on = true;
// an engine switch (environment, read per call so tests can flip it): set and not "0"
static bool env_on(const char* name) {
  const char* v = getenv(name);
  return v && *v && *v != '0';
}
static bool phase_events_off() {
  return env_on("DG_NO_PHASE_EVENTS") || !g_phase_timing.load(std::memory_order_relaxed);
}
static void phase_event(hipEvent_t e, hipStream_t st) {
  if (t_phase_on) hipEventRecord(e, st);
}
static hipError_t phase_elapsed(float* ms, hipEvent_t a, hipEvent_t b) {
  if (!t_phase_on) {
    *ms = 0.f;
    return hipSuccess;
  }
  return hipEventElapsedTime(ms, a, b);
}

// a zeroed device word for a filter's row count and its host copy (valid after finish_call); null when
// the call's count block is full (the caller then reads its count itself)
static unsigned long long* count_slot(CallScratch* cs, hipStream_t st, unsigned long long** host) {
  constexpr int kCountSlots = 64;
  if (!cs->cnt_d) {
    unsigned long long* z = up_take<unsigned long long>(cs, kCountSlots, &cs->cnt_d, st);
    cs->cnt_h = host_take<unsigned long long>(cs, kCountSlots);
    if (!z || !cs->cnt_h) {
      cs->cnt_d = nullptr;
      return nullptr;
    }
    memset(z, 0, 8 * kCountSlots);
  }
  if (cs->cnt_used >= kCountSlots) return nullptr;
  *host = cs->cnt_h + cs->cnt_used;
  return cs->cnt_d + cs->cnt_used++;
}

constexpr size_t kStagedAccBytes = 64 << 10;  // accumulator tables up to this start in the call's upload

static int32_t* call_err(CallScratch* cs, hipStream_t st) {
  if (!cs->d_err) {
    int32_t* z = up_take<int32_t>(cs, 1, &cs->d_err, st);  // zeroed by the next flush
    cs->h_err = host_take<int32_t>(cs, 1);
    if (!z || !cs->h_err) return nullptr;
    *z = 0;
    *cs->h_err = 0;
  }
  return cs->d_err;
}

// Enqueue the error-word read-back, wait for the stream, and turn device-side errors into codes. In a
// query call with a cancel flag or a timeout the wait polls them: once one fires, the queued work still
// drains (it owns the context's scratch) and the call then returns the interruption.
static int finish_call(CallScratch* cs, hipStream_t st) {
  DG_FLUSH(cs, st);
  auto& late = cs->late;
  if (cs->cnt_used) late.push_back({cs->cnt_h, cs->cnt_d, 8 * (size_t)cs->cnt_used});
  if (cs->d_err) late.push_back({cs->h_err, cs->d_err, 4});
  // the late reads with one copy of the span holding them, when it is compact (they are staged words of
  // one upload chunk, a few KiB apart); else one copy each
  uint8_t* span_h = nullptr;
  const uint8_t* lo = nullptr;
  size_t span = 0, sum = 0;
  if (late.size() > 1) {
    const uint8_t* hi = nullptr;
    for (const auto& r : late) {
      const uint8_t* d = static_cast<const uint8_t*>(r.d);
      lo = !lo || d < lo ? d : lo;
      hi = !hi || d + r.n > hi ? d + r.n : hi;
      sum += r.n;
    }
    span = (size_t)(hi - lo);
    if (span <= 2 * sum + (64 << 10) && cs->up.one_chunk(lo, hi)) span_h = host_take<uint8_t>(cs, span);
  }
  if (span_h) {
    DG_HIP(hipMemcpyAsync(span_h, lo, span, hipMemcpyDeviceToHost, st));
  } else {
    for (const auto& r : late) DG_HIP(hipMemcpyAsync(r.h, r.d, r.n, hipMemcpyDeviceToHost, st));
  }
  if (cs->intr && cs->intr->active()) {
    int irc = DG_OK;
    for (int spin = 0;; ++spin) {
      const hipError_t e = hipStreamQuery(st);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) return set_error(DG_ERR_DEVICE, "hipStreamQuery: %s", hipGetErrorString(e));
      if (!irc) irc = cs->intr->check();
      if (spin < 256) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    if (irc) return irc;
  } else {
    DG_HIP(hipStreamSynchronize(st));
  }
  if (span_h)
    for (const auto& r : late) memcpy(r.h, span_h + (static_cast<const uint8_t*>(r.d) - lo), r.n);
  late.clear();
  DG_HIP(hipGetLastError());
  DG_HIP(take_launch_error());
  if (cs->d_err && *cs->h_err)
    return set_error(DG_ERR_FORMAT, (*cs->h_err & 1)   ? "corrupt LZ4 block"
                                    : (*cs->h_err & 4) ? "corrupt multi-value row lists"
                                                       : "corrupt Roaring bitmap");
  return DG_OK;
}

// ------------------------------------------------------------------------------------------------
// Java string ordering (String.compareTo = UTF-16 code units; GenericIndexed.STRING_STRATEGY is
// naturalNullsFirst) and dictionary search (GenericIndexed.indexOf, GenericIndexed.java:308-333)
// ------------------------------------------------------------------------------------------------
static void to_utf16(const std::string& s, std::vector<uint16_t>* out) {
  out->clear();
  for (size_t i = 0; i < s.size();) {
    uint32_t c = (uint8_t)s[i];
    int n = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
    if (n == 2) c &= 0x1F;
    else if (n == 3) c &= 0x0F;
    else if (n == 4) c &= 0x07;
    for (int k = 1; k < n && i + k < s.size(); ++k) c = (c << 6) | ((uint8_t)s[i + k] & 0x3F);
    i += n;
    if (c >= 0x10000) {
      c -= 0x10000;
      out->push_back((uint16_t)(0xD800 + (c >> 10)));
      out->push_back((uint16_t)(0xDC00 + (c & 0x3FF)));
    } else {
      out->push_back((uint16_t)c);
    }
  }
}

static int java_compare(const std::string& a, const std::string& b) {
  bool ascii = true;
  for (unsigned char ch : a) ascii &= ch < 0x80;
  for (unsigned char ch : b) ascii &= ch < 0x80;
  if (ascii) {
    int c = a.compare(b);
    return (c > 0) - (c < 0);
  }
  std::vector<uint16_t> ua, ub;
  to_utf16(a, &ua);
  to_utf16(b, &ub);
  size_t n = std::min(ua.size(), ub.size());
  for (size_t i = 0; i < n; ++i)
    if (ua[i] != ub[i]) return ua[i] < ub[i] ? -1 : 1;
  return ua.size() == ub.size() ? 0 : (ua.size() < ub.size() ? -1 : 1);
}

int java_compare_str(const char* a, const char* b) { return java_compare(std::string(a), std::string(b)); }

// null-aware compare: null < anything
static int cmp_nullable(bool an, const std::string& a, bool bn, const std::string& b) {
  if (an || bn) return an == bn ? 0 : (an ? -1 : 1);
  return java_compare(a, b);
}

static int index_of(const Column* c, const char* value) {
  const bool vnull = value == nullptr || value[0] == 0;  // NullHandling.emptyToNullIfNeeded
  const std::string v = vnull ? std::string() : std::string(value);
  int lo = 0, hi = (int)c->dict.size() - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    int r = cmp_nullable(c->dict_null[mid], c->dict[mid], vnull, v);
    if (r == 0) return mid;
    if (r < 0) lo = mid + 1;
    else hi = mid - 1;
  }
  return -(lo + 1);
}

// StringComparators.NumericComparator (query/ordering/StringComparators.java:346-392)
static bool try_long(const char* s, long long* out) {
  if (!s || !*s) return false;
  const char* p = s;
  if (*p == '-') p++;
  if (!*p) return false;
  for (const char* q = p; *q; ++q)
    if (*q < '0' || *q > '9') return false;
  errno = 0;
  char* end;
  long long v = strtoll(s, &end, 10);
  if (errno || *end) return false;
  *out = v;
  return true;
}

static bool try_decimal(const char* s, long double* out) {
  if (!s || !*s) return false;
  // BigDecimal grammar: [+-]digits[.digits][(e|E)[+-]digits] or [+-].digits...
  const char* p = s;
  if (*p == '+' || *p == '-') p++;
  bool digits = false;
  while (*p >= '0' && *p <= '9') p++, digits = true;
  if (*p == '.') {
    p++;
    while (*p >= '0' && *p <= '9') p++, digits = true;
  }
  if (!digits) return false;
  if (*p == 'e' || *p == 'E') {
    p++;
    if (*p == '+' || *p == '-') p++;
    if (!(*p >= '0' && *p <= '9')) return false;
    while (*p >= '0' && *p <= '9') p++;
  }
  if (*p) return false;
  *out = strtold(s, nullptr);
  return true;
}

static int numeric_compare(const char* a, const char* b) {
  if (a == b) return 0;
  if (!a) return -1;
  if (!b) return 1;
  long long la, lb;
  bool ha = try_long(a, &la), hb = try_long(b, &lb);
  if (ha && hb) return (la > lb) - (la < lb);
  long double da = ha ? (long double)la : 0, db = hb ? (long double)lb : 0;
  bool pa = ha || try_decimal(a, &da), pb = hb || try_decimal(b, &db);
  if (pa && pb) return (da > db) - (da < db);
  if (!pa && !pb) return java_compare(a, b);
  return pa ? 1 : -1;
}

// BoundFilter.doesMatch (BoundFilter.java:249-275), default null mode
static bool bound_matches(const dg_filter& f, const char* value /* NULL = null */) {
  const bool has_lower = f.lower != nullptr, has_upper = f.upper != nullptr;
  if (!value) {
    const bool lower_null = !has_lower || f.lower[0] == 0;
    const bool upper_null = !has_upper || f.upper[0] == 0;
    return (!has_lower || (lower_null && !f.lower_strict)) && (!has_upper || !upper_null || !f.upper_strict);
  }
  auto cmp = [&](const char* x, const char* y) {
    if (f.ordering == DG_ORDER_NUMERIC) return numeric_compare(x, y);
    return cmp_nullable(x == nullptr, x ? x : "", y == nullptr, y ? y : "");
  };
  const int lc = has_lower ? cmp(value, f.lower) : 1;
  const int uc = has_upper ? cmp(f.upper, value) : 1;
  if (f.lower_strict && f.upper_strict) return lc > 0 && uc > 0;
  if (f.lower_strict) return lc > 0 && uc >= 0;
  if (f.upper_strict) return lc >= 0 && uc > 0;
  return lc >= 0 && uc >= 0;
}

static bool leaf_matches_null(const dg_filter& f) {
  if (f.kind == DG_F_SELECTOR) return f.n_values < 1 || !f.values || !f.values[0] || !f.values[0][0];
  if (f.kind == DG_F_IN) {
    for (int i = 0; i < f.n_values; ++i)
      if (!f.values[i] || !f.values[i][0]) return true;
    return false;
  }
  return bound_matches(f, nullptr);
}

struct DecodeBatch {
  std::vector<Lz4Job> jobs;
  std::vector<LzfJob> lzf_jobs;  // LZF blocks, decoded one wave per block
  std::vector<VsJob> expands;  // DELTA / TABLE blocks, expanded after the LZ4 decodes
  std::vector<MvCheck> mv_checks;  // multi-value row lists, validated after the decodes
  int32_t expand_rows = 0;     // largest block of `expands` (grid width)
  int64_t* last_expanded = nullptr;
  uint8_t* last_slots = nullptr;  // decode slots of the last viewed LZ4 / LZF column
  int64_t bytes = 0;  // algorithmic bytes read
  // the general decoder's launches bracketed by these events (when set), and its blocks' stored bytes
  hipEvent_t gen_a = nullptr, gen_b = nullptr;
  int64_t gen_bytes = 0;
  int32_t gen_blocks = 0;
  int32_t gen_launches = 0;
  int64_t flow_blocks = 0, flow_bytes = 0;  // of the general blocks, those of k_lz4_decode_flow
  // blocks planned as tasks (add_tasks), per decoder kind, and their stored bytes
  std::vector<Lz4Task> tasks[kKinds];
  int64_t task_bytes[kKinds] = {0, 0, 0, 0, 0, 0};
  int64_t fused_blocks = 0;  // blocks whose decode was fused with their aggregator (fused_agg_view)
};
// device time of the general decoder's launches of a batch (0 if it launched none)
static double gen_ms(const DecodeBatch& db) {
  if (!db.gen_blocks || !db.gen_a) return 0;
  float f = 0;
  phase_elapsed(&f, db.gen_a, db.gen_b);
  return f;
}
// the decode-timing events of a call's main (side = false) or side batch
static void decode_events(Context* ctx, DecodeBatch* db, bool side) {
  db->gen_a = ctx->gen_ev[side ? 2 : 0];
  db->gen_b = ctx->gen_ev[side ? 3 : 1];
}
// a call's decode metrics from its main and side batches
static void decode_metrics(const DecodeBatch& db, const DecodeBatch& side, dg_metrics* m, hipEvent_t base) {
  m->lz4_general_ms = gen_ms(db) + gen_ms(side);
  // the wall time the general decoder ran on either stream: the union of the two spans (from the
  // call's first event)
  m->lz4_general_wall_ms = m->lz4_general_ms;
  if (db.gen_blocks && side.gen_blocks && db.gen_a && side.gen_a && base) {
    float s1 = 0, e1 = 0, s2 = 0, e2 = 0;
    phase_elapsed(&s1, base, db.gen_a);
    phase_elapsed(&e1, base, db.gen_b);
    phase_elapsed(&s2, base, side.gen_a);
    phase_elapsed(&e2, base, side.gen_b);
    const double overlap = std::max(0.0, (double)std::min(e1, e2) - (double)std::max(s1, s2));
    m->lz4_general_wall_ms = (double)(e1 - s1) + (double)(e2 - s2) - overlap;
  }
  m->lz4_general_bytes = db.gen_bytes + side.gen_bytes;
  m->lz4_general_blocks = db.gen_blocks + side.gen_blocks;
  m->lz4_general_launches = db.gen_launches + side.gen_launches;
  m->lz4_fused_blocks = db.fused_blocks + side.fused_blocks;
  m->lz4_flow_blocks = db.flow_blocks + side.flow_blocks;
  m->lz4_flow_bytes = db.flow_bytes + side.flow_bytes;
}
static int column_view(const Column* c, CallScratch* cs, DecodeBatch* db, ColView* v, hipStream_t st);
static int multi_view(const Column* c, CallScratch* cs, DecodeBatch* db, ColView* vals, ColView* offs, hipStream_t st);
static int run_decodes(CallScratch* cs, DecodeBatch* db, hipStream_t st, uint64_t* d_prof = nullptr, bool overlap = false);
static int run_decodes_only(CallScratch* cs, DecodeBatch* db, hipStream_t st, uint64_t* d_prof, bool overlap = false);

// ------------------------------------------------------------------------------------------------
// numeric post-filters: Java's parsing of the filter's strings (host side, once per call)
// ------------------------------------------------------------------------------------------------
// java.math.BigDecimal(String) (sign, digits with one optional '.', optional [eE][+-]digits; no
// whitespace): value = (neg ? -1 : 1) * digits * 10^exp, digits without leading zeros
struct Decimal {
  bool neg = false;
  std::string digits;  // "" = zero
  long long exp = 0;
};

static bool parse_big_decimal(const char* s, Decimal* d) {
  if (!s || !*s) return false;
  const char* p = s;
  d->neg = false;
  if (*p == '+' || *p == '-') d->neg = *p++ == '-';
  std::string all;
  long long frac = 0;
  bool dot = false, any = false;
  for (; *p; ++p) {
    if (*p >= '0' && *p <= '9') {
      all.push_back(*p);
      any = true;
      if (dot) frac++;
    } else if (*p == '.' && !dot) {
      dot = true;
    } else {
      break;
    }
  }
  if (!any) return false;
  long long e = 0;
  if (*p == 'e' || *p == 'E') {
    p++;
    bool eneg = false;
    if (*p == '+' || *p == '-') eneg = *p++ == '-';
    if (!(*p >= '0' && *p <= '9')) return false;
    for (; *p >= '0' && *p <= '9'; ++p) {
      e = e * 10 + (*p - '0');
      if (e > 1000000000ll) return false;  // BigDecimal: the exponent must fit an int
    }
    if (eneg) e = -e;
  }
  if (*p) return false;
  size_t z = 0;
  while (z < all.size() && all[z] == '0') z++;
  d->digits = all.substr(z);
  d->exp = e - frac;
  if (d->digits.empty()) d->neg = false;
  return true;
}

// setScale(0, FLOOR / CEILING) (or exact: integral only) then longValueExact. Returns 1 = fits
// *out, 0 = not integral (exact mode), +2 / -2 = beyond Long.MAX / Long.MIN
static int decimal_to_long(const Decimal& d, int mode /* 0 exact, 1 floor, 2 ceiling */, long long* out) {
  std::string ip;  // integer part digits
  bool frac_nonzero = false;
  if (d.exp >= 0) {
    if (!d.digits.empty()) {
      if (d.digits.size() + (size_t)d.exp > 40) return d.neg ? -2 : 2;
      ip = d.digits + std::string((size_t)d.exp, '0');
    }
  } else {
    const long long k = -d.exp;
    if ((long long)d.digits.size() > k) ip = d.digits.substr(0, d.digits.size() - (size_t)k);
    const std::string fr = (long long)d.digits.size() > k ? d.digits.substr(d.digits.size() - (size_t)k) : d.digits;
    for (char c : fr) frac_nonzero |= c != '0';
  }
  if (mode == 0 && frac_nonzero) return 0;
  if (ip.size() > 20) return d.neg ? -2 : 2;
  unsigned __int128 m = 0;
  for (char c : ip) m = m * 10 + (unsigned)(c - '0');
  __int128 v = d.neg ? -(__int128)m : (__int128)m;
  if (frac_nonzero) {
    if (mode == 1 && d.neg) v -= 1;   // floor of a negative non-integer
    if (mode == 2 && !d.neg) v += 1;  // ceiling of a positive non-integer
  }
  if (v > (__int128)INT64_MAX) return 2;
  if (v < (__int128)INT64_MIN) return -2;
  *out = (long long)v;
  return 1;
}

// GuavaUtils.tryParseLong (a leading '+' stripped) -> Longs.tryParse: [-]digits within range
static bool guava_try_parse_long(const char* s, long long* out) {
  if (!s || !*s) return false;
  if (*s == '+') s++;
  return try_long(s, out);
}

// DimensionHandlerUtils.getExactLongFromDecimalString (DimensionHandlerUtils.java:404-426)
static bool exact_long(const char* s, long long* out) {
  if (guava_try_parse_long(s, out)) return true;
  Decimal d;
  if (!parse_big_decimal(s, &d)) return false;
  return decimal_to_long(d, 0, out) == 1;
}

// Guava Floats/Doubles.tryParse: [+-]?(NaN|Infinity|decimal[eE..]?[fFdD]?|0[xX]hex[pP]exp[fFdD]?)
// validated like FLOATING_POINT_PATTERN, then Float.parseFloat / Double.parseDouble (correctly rounded)
static bool guava_float_syntax(const char* s, std::string* body) {
  if (!s || !*s) return false;
  const char* p = s;
  std::string out;
  if (*p == '+' || *p == '-') out.push_back(*p++);
  if (!strcmp(p, "NaN") || !strcmp(p, "Infinity")) {
    *body = out + p;
    return true;
  }
  auto isx = [](char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); };
  const char* q = p;
  if (q[0] == '0' && (q[1] == 'x' || q[1] == 'X')) {
    q += 2;
    bool any = false;
    while (isx(*q)) q++, any = true;
    if (*q == '.') {
      q++;
      while (isx(*q)) q++, any = true;
    }
    if (!any || (*q != 'p' && *q != 'P')) return false;
    q++;
    if (*q == '+' || *q == '-') q++;
    if (!(*q >= '0' && *q <= '9')) return false;
    while (*q >= '0' && *q <= '9') q++;
  } else {
    bool any = false;
    while (*q >= '0' && *q <= '9') q++, any = true;
    if (*q == '.') {
      q++;
      while (*q >= '0' && *q <= '9') q++, any = true;
    }
    if (!any) return false;
    if (*q == 'e' || *q == 'E') {
      q++;
      if (*q == '+' || *q == '-') q++;
      if (!(*q >= '0' && *q <= '9')) return false;
      while (*q >= '0' && *q <= '9') q++;
    }
  }
  out.append(p, q);
  if (*q == 'f' || *q == 'F' || *q == 'd' || *q == 'D') q++;
  if (*q) return false;
  *body = out;
  return true;
}

static bool guava_try_parse_double(const char* s, double* out) {
  std::string b;
  if (!guava_float_syntax(s, &b)) return false;
  *out = strtod(b.c_str(), nullptr);
  return true;
}

static bool guava_try_parse_float(const char* s, float* out) {
  std::string b;
  if (!guava_float_syntax(s, &b)) return false;
  *out = strtof(b.c_str(), nullptr);
  return true;
}

static int64_t float_bits(float f) {  // Float.floatToIntBits
  if (f != f) return 0x7fc00000ll;
  uint32_t u;
  memcpy(&u, &f, 4);
  return (int64_t)u;
}

static int64_t double_bits(double d) {  // Double.doubleToLongBits
  if (d != d) return 0x7ff8000000000000ll;
  int64_t u;
  memcpy(&u, &d, 8);
  return u;
}

static uint64_t dcmp_key_host(double d) {  // Double.compare order as unsigned keys
  if (d != d) return ~0ull;
  uint64_t u;
  memcpy(&u, &d, 8);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

struct PredLeaf {
  NumPred p;
  std::vector<int64_t> set;
  std::string lo, hi;
  const Column* col;
};

// The row predicate of a selector / in / bound filter on a numeric column, as the reference builds
// its ValueMatcher. Default null mode: a numeric row is never null, so null-matching predicates
// (nullValueMatcher) select nothing.
static int plan_numeric_leaf(const dg_filter& f, const Column* c, PredLeaf* L) {
  memset(&L->p, 0, sizeof L->p);
  L->col = c;
  NumPred& p = L->p;
  p.kind = PRED_FALSE;
  const bool is_long = c->type == DG_COL_LONG, is_float = c->type == DG_COL_FLOAT;
  auto add_value = [&](const char* v) {  // one selector / IN value
    if (!v || !*v) return;  // emptyToNullIfNeeded -> null: no numeric row matches
    if (is_long) {
      long long x;
      if (exact_long(v, &x)) L->set.push_back(x);
    } else if (is_float) {
      float x;
      if (guava_try_parse_float(v, &x)) L->set.push_back(float_bits(x));
    } else {
      double x;
      if (guava_try_parse_double(v, &x)) L->set.push_back(double_bits(x));
    }
  };
  if (f.kind == DG_F_SELECTOR || f.kind == DG_F_IN) {
    // SelectorFilter -> {Long,Float,Double}ValueMatcherColumnSelectorStrategy.makeValueMatcher(value)
    // (convertObjectToLong = getExactLongFromDecimalString, Floats/Doubles.tryParse + *ToIntBits);
    // InFilter -> InDimFilter.get{Long,Float,Double}PredicateSupplier (the same parsing, a set)
    const int nv = f.kind == DG_F_SELECTOR ? std::min(f.n_values, 1) : f.n_values;
    for (int k = 0; k < nv; ++k) add_value(f.values ? f.values[k] : nullptr);
    std::sort(L->set.begin(), L->set.end());
    L->set.erase(std::unique(L->set.begin(), L->set.end()), L->set.end());
    if (!L->set.empty()) p.kind = is_long ? PRED_LONG_SET : PRED_BITS_SET;
    return DG_OK;
  }
  // BoundFilter: NUMERIC ordering -> BoundDimFilter.{long,float,double}PredicateSupplier
  // (BoundDimFilter.java:341-652); other orderings compare String.valueOf(value) (BoundFilter
  // makeLongPredicate etc.: doesMatch) — for long columns under LEXICOGRAPHIC (UTF-8 bytes)
  // the bounds are kept as given (BoundDimFilter.java:73-76; hasLowerBound = lower != null): "" is a
  // bound, unparseable as a number
  const char* lo = f.lower;
  const char* hi = f.upper;
  p.lo_strict = f.lower_strict;
  p.hi_strict = f.upper_strict;
  if (f.ordering != DG_ORDER_NUMERIC) {
    if (!is_long || f.ordering != DG_ORDER_LEXICOGRAPHIC)
      return set_error(DG_ERR_UNSUPPORTED, "bound ordering %d on numeric column %s (String.valueOf formatting)",
                       f.ordering, c->name.c_str());
    p.kind = PRED_LONG_LEX;
    p.has_lo = lo != nullptr;
    p.has_hi = hi != nullptr;
    L->lo = lo ? lo : "";
    L->hi = hi ? hi : "";
    return DG_OK;
  }
  if (is_long) {
    bool nothing = false;
    long long lv = 0, hv = 0;
    if (lo) {
      if (guava_try_parse_long(lo, &lv)) {
        p.has_lo = 1;
      } else {
        Decimal d;
        if (!parse_big_decimal(lo, &d)) {
          p.has_lo = 0;  // unparseable: below every number
        } else {
          const int r = decimal_to_long(d, f.lower_strict ? 1 : 2, &lv);
          if (r == 1) p.has_lo = 1;
          else if (r == 2) nothing = true;  // positive lower bound above every long
        }
      }
    }
    if (hi) {
      if (guava_try_parse_long(hi, &hv)) {
        p.has_hi = 1;
      } else {
        Decimal d;
        if (!parse_big_decimal(hi, &d)) {
          nothing = true;  // unparseable upper bound: below every number
        } else {
          const int r = decimal_to_long(d, f.upper_strict ? 2 : 1, &hv);
          if (r == 1) p.has_hi = 1;
          else if (r == -2) nothing = true;
        }
      }
    }
    p.kind = nothing ? PRED_FALSE : PRED_LONG_RANGE;
    p.lo = lv;
    p.hi = hv;
    return DG_OK;
  }
  bool nothing = false;
  double lv = 0, hv = 0;
  if (lo) {
    if (is_float) {
      float x;
      p.has_lo = guava_try_parse_float(lo, &x);
      lv = x;
    } else {
      p.has_lo = guava_try_parse_double(lo, &lv);
    }
  }
  if (hi) {
    bool ok;
    if (is_float) {
      float x;
      ok = guava_try_parse_float(hi, &x);
      hv = x;
    } else {
      ok = guava_try_parse_double(hi, &hv);
    }
    p.has_hi = ok;
    nothing = !ok;
  }
  p.kind = nothing ? PRED_FALSE : PRED_ORD_RANGE;
  p.lo = (int64_t)dcmp_key_host(lv);
  p.hi = (int64_t)dcmp_key_host(hv);
  return DG_OK;
}

// ------------------------------------------------------------------------------------------------
// filter planning: prefix nodes -> postfix program over leaf bitsets
// ------------------------------------------------------------------------------------------------
struct FilterPlan {
  std::vector<int32_t> prog;
  std::vector<std::vector<int32_t>> leaf_ids;  // dictionary ids whose bitmaps are OR-ed
  std::vector<const Column*> leaf_col;         // null: a row-predicate leaf (leaf_pred)
  std::vector<int32_t> leaf_pred;              // index into preds, -1 for bitmap leaves
  std::vector<PredLeaf> preds;
};

static int plan_node(const Segment* seg, const dg_filter* nodes, int n, int* pos, FilterPlan* fp) {
  if (*pos >= n) return set_error(DG_ERR_ARG, "truncated filter");
  const dg_filter& f = nodes[(*pos)++];
  switch (f.kind) {
    case DG_F_AND:
    case DG_F_OR: {
      if (f.n_children < 1) return set_error(DG_ERR_ARG, "empty and/or filter");
      for (int c = 0; c < f.n_children; ++c) {
        int rc = plan_node(seg, nodes, n, pos, fp);
        if (rc) return rc;
        if (c > 0) fp->prog.push_back(f.kind == DG_F_AND ? -3 : -4);
      }
      return DG_OK;
    }
    case DG_F_NOT: {
      int rc = plan_node(seg, nodes, n, pos, fp);
      if (rc) return rc;
      fp->prog.push_back(-5);
      return DG_OK;
    }
    case DG_F_SELECTOR:
    case DG_F_IN:
    case DG_F_BOUND: {
      if (!f.dimension) return set_error(DG_ERR_ARG, "filter without dimension");
      const Column* c = seg->find(f.dimension);
      if (!c) {
        // missing column: allTrue iff the filter matches null (ColumnSelectorBitmapIndexSelector.java:212-218)
        fp->prog.push_back(leaf_matches_null(f) ? -1 : -2);
        return DG_OK;
      }
      if (c->type == DG_COL_LONG || c->type == DG_COL_FLOAT || c->type == DG_COL_DOUBLE) {
        // no bitmap index: a row post-filter (QueryableIndexStorageAdapter.java:244-260, FilteredOffset)
        PredLeaf L;
        int rc = plan_numeric_leaf(f, c, &L);
        if (rc) return rc;
        if (L.p.kind == PRED_FALSE) {
          fp->prog.push_back(-2);
          return DG_OK;
        }
        fp->prog.push_back((int32_t)fp->leaf_ids.size());
        fp->leaf_ids.emplace_back();
        fp->leaf_col.push_back(nullptr);
        fp->leaf_pred.push_back((int32_t)fp->preds.size());
        fp->preds.push_back(std::move(L));
        return DG_OK;
      }
      if (c->type != DG_COL_STRING)
        return set_error(DG_ERR_UNSUPPORTED, "filter on %s needs a bitmap index", f.dimension);
      std::vector<int32_t> ids;
      if (f.kind == DG_F_SELECTOR) {
        int i = index_of(c, f.n_values > 0 && f.values ? f.values[0] : nullptr);
        if (i >= 0) ids.push_back(i);
      } else if (f.kind == DG_F_IN) {
        for (int k = 0; k < f.n_values; ++k) {
          int i = index_of(c, f.values[k]);
          if (i >= 0) ids.push_back(i);
        }
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
      } else if (f.ordering == DG_ORDER_LEXICOGRAPHIC) {
        // BoundFilter.getStartEndIndexes (BoundFilter.java:141-174)
        const int card = (int)c->dict.size();
        int start, end;
        if (!f.lower) start = 0;
        else {
          int found = index_of(c, f.lower);
          start = found >= 0 ? (f.lower_strict ? found + 1 : found) : -(found + 1);
        }
        if (!f.upper) end = card;
        else {
          int found = index_of(c, f.upper);
          end = found >= 0 ? (f.upper_strict ? found : found + 1) : -(found + 1);
        }
        if (end < start) end = start;
        for (int i = start; i < end; ++i) ids.push_back(i);
      } else if (f.ordering == DG_ORDER_NUMERIC) {
        // predicate over every dictionary value (Filters.matchPredicate, Filters.java:239-290)
        for (int i = 0; i < (int)c->dict.size(); ++i)
          if (bound_matches(f, c->dict_null[i] ? nullptr : c->dict[i].c_str())) ids.push_back(i);
      } else {
        return set_error(DG_ERR_UNSUPPORTED, "bound ordering %d", f.ordering);
      }
      if (ids.empty()) {
        fp->prog.push_back(-2);
        return DG_OK;
      }
      if (!c->has_bitmaps) {
        // no bitmap index (an in-memory segment): the matching ids become a row predicate, as
        // IncrementalIndexStorageAdapter's cursors evaluate filter.makeMatcher per row
        PredLeaf L;
        memset(&L.p, 0, sizeof L.p);
        L.p.kind = PRED_ID_SET;
        L.col = c;
        L.set.assign((c->dict.size() + 63) / 64, 0);
        for (int32_t i : ids) L.set[i >> 6] |= (int64_t)(1ull << (i & 63));
        L.p.has_lo = c->multi_value && !c->dict.empty() && c->dict_null[0] && !ids.empty() && ids[0] == 0;
        fp->prog.push_back((int32_t)fp->leaf_ids.size());
        fp->leaf_ids.emplace_back();
        fp->leaf_col.push_back(nullptr);
        fp->leaf_pred.push_back((int32_t)fp->preds.size());
        fp->preds.push_back(std::move(L));
        return DG_OK;
      }
      fp->prog.push_back((int32_t)fp->leaf_ids.size());
      fp->leaf_ids.push_back(std::move(ids));
      fp->leaf_col.push_back(c);
      fp->leaf_pred.push_back(-1);
      return DG_OK;
    }
    default:
      return set_error(DG_ERR_ARG, "unknown filter kind %d", f.kind);
  }
}

// Build the row bitset of `filter` for segment `seg` on the device. *out = nullptr means "all rows".
// The bitset's cardinality lands in the pinned word *count once finish_call has synchronised
// (nullptr when there is no filter: every row). Nothing here synchronises.
static int build_bitset(Segment* seg, CallScratch* cs, const dg_filter* filter, int n_filter, uint32_t** out,
                        const unsigned long long** count, hipStream_t st) {
  *out = nullptr;
  *count = nullptr;
  if (!filter || n_filter <= 0) return DG_OK;
  FilterPlan fp;
  int pos = 0;
  int rc = plan_node(seg, filter, n_filter, &pos, &fp);
  if (rc) return rc;
  if (pos != n_filter) return set_error(DG_ERR_ARG, "filter has %d trailing nodes", n_filter - pos);
  if (fp.prog.size() > 64) return set_error(DG_ERR_UNSUPPORTED, "filter program too long");
  // stack depth check (kernel stack of 16)
  int depth = 0, maxd = 0;
  for (int op : fp.prog) {
    if (op >= -2) depth++;
    else if (op != -5) depth--;
    maxd = std::max(maxd, depth);
  }
  if (maxd > 16) return set_error(DG_ERR_UNSUPPORTED, "filter nesting too deep");
  const int64_t nwords = (seg->nrows + 31) / 32;
  const int nleaves = (int)fp.leaf_ids.size();
  // the program and the row count staged first: the leaves' upload carries them
  const int plen = (int)fp.prog.size();
  int32_t* d_prog;
  int32_t* h_prog = up_take<int32_t>(cs, plen + 2, &d_prog, st);  // (+ a zeroed count word when no slot)
  if (!h_prog) return set_error(DG_ERR_OOM, "filter program");
  memcpy(h_prog, fp.prog.data(), plen * 4);
  unsigned long long* h_count = nullptr;
  unsigned long long* d_count = count_slot(cs, st, &h_count);
  const bool own_count = d_count == nullptr;
  if (own_count) {
    d_count = reinterpret_cast<unsigned long long*>(d_prog + ((plen + 1) & ~1));
    memset(h_prog + ((plen + 1) & ~1), 0, 8);
  }
  uint32_t** d_sets;
  uint32_t** h_sets = up_take<uint32_t*>(cs, std::max(nleaves, 1), &d_sets, st);
  uint32_t* leaf_mem = dev_take<uint32_t>(cs, (size_t)std::max(nleaves, 1) * (nwords + 2));
  if (!h_sets || !leaf_mem) return set_error(DG_ERR_OOM, "bitset scratch");
  for (int l = 0; l < nleaves; ++l) h_sets[l] = leaf_mem + (size_t)l * (nwords + 2);
  DG_HIP(hipMemsetAsync(leaf_mem, 0, (size_t)std::max(nleaves, 1) * (nwords + 2) * 4, st));
  // one launch per (column, codec): group leaves by column
  for (int l = 0; l < nleaves; ++l) {
    const Column* c = fp.leaf_col[l];
    if (!c) continue;  // row-predicate leaf, below
    // gather all leaves on the same column into this launch
    bool first = true;
    for (int k = 0; k < l; ++k)
      if (fp.leaf_col[k] == c) first = false;
    if (!first) continue;
    std::vector<int64_t> offs, row0s, p_off, p_row0;
    std::vector<int32_t> lens, tgts, p_info, p_tgt;
    const bool split = !c->bm_piece_first.empty();
    for (int k = l; k < nleaves; ++k) {
      if (fp.leaf_col[k] != c) continue;
      for (int32_t id : fp.leaf_ids[k]) {
        if (c->bm_len[id] == 0) continue;
        cs->bitmap_bytes += c->bm_len[id];
        if (split && c->bm_piece_first[id + 1] > c->bm_piece_first[id]) {  // a long bitmap: its pieces
          for (int32_t q = c->bm_piece_first[id]; q < c->bm_piece_first[id + 1]; ++q) {
            const BmPiece& pc = c->bm_pieces[q];
            if (c->bitmap_roaring) {
              p_off.push_back(pc.off);
              p_row0.push_back(pc.row0);
              p_info.push_back(pc.info);
              p_tgt.push_back(k);
            } else {
              offs.push_back(pc.off);
              lens.push_back(pc.len);
              row0s.push_back(pc.row0);
              tgts.push_back(k);
            }
          }
          continue;
        }
        offs.push_back(c->bm_off[id]);
        lens.push_back(c->bm_len[id]);
        row0s.push_back(0);
        tgts.push_back(k);
      }
    }
    if (!p_off.empty()) {  // Roaring containers of split bitmaps
      const int np = (int)p_off.size();
      int64_t *d_poff, *d_prow;
      int32_t *d_pinfo, *d_ptgt;
      int64_t* h_poff = up_take<int64_t>(cs, np, &d_poff, st);
      int64_t* h_prow = up_take<int64_t>(cs, np, &d_prow, st);
      int32_t* h_pinfo = up_take<int32_t>(cs, np, &d_pinfo, st);
      int32_t* h_ptgt = up_take<int32_t>(cs, np, &d_ptgt, st);
      if (!h_poff || !h_prow || !h_pinfo || !h_ptgt) return set_error(DG_ERR_OOM, "bitmap piece tables");
      memcpy(h_poff, p_off.data(), np * 8);
      memcpy(h_prow, p_row0.data(), np * 8);
      memcpy(h_pinfo, p_info.data(), np * 4);
      memcpy(h_ptgt, p_tgt.data(), np * 4);
      DG_FLUSH(cs, st);
      launch_roaring_pieces(c->bm_bytes.as<uint8_t>(), d_poff, d_prow, d_pinfo, d_ptgt, np, d_sets, (nwords + 2) * 32, st);
    }
    if (offs.empty()) continue;
    const int nb = (int)offs.size();
    int64_t *d_off, *d_row0;
    int32_t *d_len, *d_tgt;
    int64_t* h_off = up_take<int64_t>(cs, nb, &d_off, st);
    int64_t* h_row0 = up_take<int64_t>(cs, nb, &d_row0, st);
    int32_t* h_len = up_take<int32_t>(cs, nb, &d_len, st);
    int32_t* h_tgt = up_take<int32_t>(cs, nb, &d_tgt, st);
    if (!h_off || !h_row0 || !h_len || !h_tgt) return set_error(DG_ERR_OOM, "bitmap tables");
    memcpy(h_off, offs.data(), nb * 8);
    memcpy(h_row0, row0s.data(), nb * 8);
    memcpy(h_len, lens.data(), nb * 4);
    memcpy(h_tgt, tgts.data(), nb * 4);
    if (c->bitmap_roaring) {
      int32_t* d_err = call_err(cs, st);
      if (!d_err) return set_error(DG_ERR_OOM, "error word");
      DG_FLUSH(cs, st);
      launch_roaring_or(c->bm_bytes.as<uint8_t>(), d_off, d_len, d_tgt, nb, d_sets, d_err, (nwords + 2) * 32, st);
    } else {
      DG_FLUSH(cs, st);
      launch_concise_or(c->bm_bytes.as<uint8_t>(), d_off, d_len, d_tgt, d_row0, nb, d_sets, (nwords + 2) * 32, st);
    }
  }
  // row-predicate leaves: decode the column (its blocks, as the reference's post-filter reads them
  // through the column selector) and evaluate the predicate per row into the leaf's bitset
  for (int l = 0; l < nleaves; ++l) {
    if (fp.leaf_pred[l] < 0) continue;
    PredLeaf& L = fp.preds[fp.leaf_pred[l]];
    DecodeBatch db;
    ColView v, voff;
    memset(&v, 0, sizeof v);
    memset(&voff, 0, sizeof voff);
    int rc2 = L.col->multi_value ? multi_view(L.col, cs, &db, &v, &voff, st) : column_view(L.col, cs, &db, &v, st);
    if (rc2) return rc2;
    if (!L.set.empty()) {
      int64_t* d_set;
      int64_t* h_set = up_take<int64_t>(cs, L.set.size(), &d_set, st);
      if (!h_set) return set_error(DG_ERR_OOM, "predicate set");
      memcpy(h_set, L.set.data(), 8 * L.set.size());
      L.p.set = d_set;
      L.p.nset = (int32_t)L.set.size();
    }
    if (L.p.kind == PRED_LONG_LEX) {
      uint8_t *d_lo, *d_hi;
      uint8_t* h_lo = up_take<uint8_t>(cs, L.lo.size() + 1, &d_lo, st);
      uint8_t* h_hi = up_take<uint8_t>(cs, L.hi.size() + 1, &d_hi, st);
      if (!h_lo || !h_hi) return set_error(DG_ERR_OOM, "predicate bounds");
      memcpy(h_lo, L.lo.data(), L.lo.size());
      memcpy(h_hi, L.hi.data(), L.hi.size());
      L.p.lo_str = d_lo;
      L.p.hi_str = d_hi;
      L.p.lo_len = (int32_t)L.lo.size();
      L.p.hi_len = (int32_t)L.hi.size();
    }
    rc2 = run_decodes(cs, &db, st);
    if (rc2) return rc2;
    DG_FLUSH(cs, st);
    launch_num_pred(v, voff, seg->nrows, L.p, h_sets[l], st);
    cs->bitmap_bytes += seg->nrows * (int64_t)std::max(v.width, 1);  // the predicate's column
  }
  cs->bitmap_bytes += (2 * (int64_t)nleaves + 1) * nwords * 4;  // leaf bitsets written + read, the result
  uint32_t* result = dev_take<uint32_t>(cs, (size_t)nwords + 2);
  DG_FLUSH(cs, st);
  launch_filter_eval(d_prog, plen, d_sets, result, seg->nrows, d_count, st);
  if (own_count) {
    h_count = host_take<unsigned long long>(cs, 1);
    if (!h_count) return set_error(DG_ERR_OOM, "filter count");
    DG_HIP(hipMemcpyAsync(h_count, d_count, 8, hipMemcpyDeviceToHost, st));
  }
  *count = h_count;
  *out = result;
  return DG_OK;
}

// ------------------------------------------------------------------------------------------------
// column decode: returns a ColView, scheduling LZ4 block decodes into scratch when needed
// ------------------------------------------------------------------------------------------------

// A literal-only LZ4 block is its own decoded image (lz4_literal_start): the view points at its literal
// bytes in HBM (16-byte aligned at attach) and no decoder runs for it; null for other blocks.
static const uint8_t* literal_block(const BlockColumn& b, int32_t k) {
  return (!b.lit_off.empty() && b.lit_off[k] >= 0) ? b.comp.as<uint8_t>() + b.lit_off[k] : nullptr;
}

// Whether a column's LZ4 blocks can be planned as tasks (its attach-time tables hold the default routes).
static bool taskable(const BlockColumn& b, int routes) {
  return b.codec == CODEC_LZ4 && routes == (kRouteRun | kRouteFlow) && b.job_desc.p && b.kind_dev.p;
}

// The column's LZ4 blocks k in [k0, k1) of every decoder kind (literal-only and empty blocks are in no
// list) as one task per kind: block k decodes to dst_base + k * dst_step (vstride: into records), or
// folds into *red (fused) when red is given. O(kinds * log blocks) host work.
struct FoldSpec {
  uint64_t* dst;
  int32_t op, kind, vkind, code;
  const uint32_t* bits;  // a filtered scan's row bitset (null: every row folds)
  int32_t rpb;           // rows per block
};
static void add_tasks(DecodeBatch* db, const BlockColumn& b, int32_t k0, int32_t k1, uint8_t* dst_base, int64_t dst_step,
                      int32_t vstride, const FoldSpec* red, bool with_light = true) {
  for (int kd = 0; kd < kKinds; ++kd) {
    if (kd == kKindLight && !with_light) continue;
    // (the column's blocks of the kind below k0 / k1: attach-time prefix counts, O(1))
    const int32_t i0 = b.kind_pos[kd][k0], i1 = b.kind_pos[kd][k1];
    if (i1 <= i0) continue;
    Lz4Task t;
    memset(&t, 0, sizeof t);
    t.desc = b.job_desc.as<Lz4Job>();
    t.list = b.kind_dev.as<int32_t>() + b.kind_at[kd];
    t.i0 = i0;
    t.n = i1 - i0;
    t.dst_base = dst_base;
    t.dst_step = dst_step;
    t.vstride = vstride;
    if (red) {
      t.red_dst = red->dst;
      t.red_op = red->op;
      t.red_kind = red->kind;
      t.red_vkind = red->vkind;
      t.red_code = red->code;
      t.red_bits = red->bits;
      t.red_rpb = red->rpb;
    }
    db->tasks[kd].push_back(t);
    db->task_bytes[kd] += b.kind_bytes[kd][i1] - b.kind_bytes[kd][i0];
  }
}

static int block_view(const BlockColumn& b, int kind, const char* name, CallScratch* cs, DecodeBatch* db, ColView* v,
                      hipStream_t st);

static int column_view(const Column* c, CallScratch* cs, DecodeBatch* db, ColView* v, hipStream_t st) {
  if (c->multi_value)
    return set_error(DG_ERR_UNSUPPORTED, "%s: multi-value dimension", c->name.c_str());
  const int kind = c->type == DG_COL_LONG ? VIEW_LONG : c->type == DG_COL_DOUBLE ? VIEW_DOUBLE
                   : c->type == DG_COL_FLOAT ? VIEW_FLOAT : VIEW_IDS;
  return block_view(c->data, kind, c->name.c_str(), cs, db, v, st);
}

// a multi-value dimension: its value ids and the rows' value offsets
static int multi_view(const Column* c, CallScratch* cs, DecodeBatch* db, ColView* vals, ColView* offs, hipStream_t st) {
  int rc = block_view(c->data, VIEW_IDS, c->name.c_str(), cs, db, vals, st);
  if (rc) return rc;
  rc = block_view(c->mv_off, VIEW_IDS, c->name.c_str(), cs, db, offs, st);
  if (rc) return rc;
  MvCheck m;
  m.vals = *vals;
  m.offs = *offs;
  m.rows = (int64_t)c->mv_off.total - 1;
  m.nvals = c->data.total;
  m.card = (int64_t)c->dict.size();
  db->mv_checks.push_back(m);
  return DG_OK;
}

static int block_view(const BlockColumn& b, int kind, const char* name, CallScratch* cs, DecodeBatch* db, ColView* v,
                      hipStream_t st) {
  v->log2_per = b.log2_per;
  v->width = b.width;
  v->pad = b.big_endian ? kViewBigEndian : 0;
  v->kind = kind;
  db->bytes += b.stored_bytes + b.index_bytes;
  if (b.codec != CODEC_LZ4 && b.codec != CODEC_LZF && b.codec != CODEC_UNCOMPRESSED && b.codec != CODEC_NONE)
    return set_error(DG_ERR_UNSUPPORTED, "codec 0x%02x of %s", b.codec, name);
  uint8_t* slots = nullptr;
  const int routes = b.codec == CODEC_LZ4 ? decode_routes() : 0;
  if (b.codec == CODEC_LZ4 || b.codec == CODEC_LZF) {
    slots = dev_take<uint8_t>(cs, (size_t)b.nblocks * kBlockBytes + 64);
    if (!slots) return set_error(DG_ERR_OOM, "decode scratch");
    db->last_slots = slots;
  }
  int64_t* expanded = nullptr;
  if (b.vbits) {
    expanded = dev_take<int64_t>(cs, (size_t)b.nblocks * b.size_per + 8);
    if (!expanded) return set_error(DG_ERR_OOM, "expand scratch");
    db->last_expanded = expanded;
  }
  if (!slots && !expanded) {
    v->blocks = b.block_ptrs.as<const uint8_t*>();
    return DG_OK;
  }
  const uint8_t** d_ptrs;
  const uint8_t** h_ptrs = up_take<const uint8_t*>(cs, std::max(b.nblocks, 1), &d_ptrs, st);
  if (!h_ptrs || !d_ptrs) return set_error(DG_ERR_OOM, "decode scratch");
  const bool tasks = taskable(b, routes);  // every LZ4 block decodes to its slot k: one task per kind
  if (tasks) add_tasks(db, b, 0, b.nblocks, slots, kBlockBytes, 0, nullptr);
  for (int32_t k = 0; k < b.nblocks; ++k) {
    const int64_t rows = std::min<int64_t>(b.size_per, (int64_t)b.total - (int64_t)k * b.size_per);
    // the packed (or plain) bytes of block k: an LZ4 slot, an uncompressed slot or a NONE range
    const uint8_t* src;
    const uint8_t* lit = literal_block(b, k);
    if (lit) src = lit;
    else if (slots) src = slots + (size_t)k * kBlockBytes;
    else if (b.codec == CODEC_UNCOMPRESSED) src = b.raw.as<uint8_t>() + (size_t)k * kBlockBytes;
    else src = b.raw.as<uint8_t>() + (size_t)k * (size_t)b.size_per * b.vbits / 8;
    h_ptrs[k] = expanded ? reinterpret_cast<const uint8_t*>(expanded + (size_t)k * b.size_per) : src;
    if (rows <= 0) continue;
    if (slots && !lit && !tasks) {
      const int64_t expect = b.vbits ? (b.vbits * rows + 7) / 8 : rows * b.width;
      if (b.codec == CODEC_LZ4) {
        db->jobs.push_back(lz4_job(b, k, const_cast<uint8_t*>(src), (int32_t)expect, routes));
      } else {
        LzfJob lj;
        lj.src = b.comp.as<uint8_t>() + b.comp_off[k];
        lj.dst = const_cast<uint8_t*>(src);
        lj.src_len = b.comp_len[k];
        lj.expect_len = (int32_t)expect;
        db->lzf_jobs.push_back(lj);
      }
    }
    if (expanded) {
      VsJob e;
      e.src = src;
      e.dst = expanded + (size_t)k * b.size_per;
      e.table = b.table.p ? b.table.as<int64_t>() : nullptr;
      e.base = b.delta_base;
      e.rows = (int32_t)rows;
      e.bits = b.vbits;
      e.table_n = b.table_n;
      e.pad = 0;
      db->expands.push_back(e);
      db->expand_rows = std::max(db->expand_rows, (int32_t)rows);
    }
  }
  v->blocks = d_ptrs;
  return DG_OK;
}

// A plain 8-byte LZ4 value column decoded straight into column `a` of the groupBy payload records
// ([rows][pw] words, row ref row_base + r): the value is its aggregator's input as is (longSum of a
// long column, doubleSum of a double column), so the decoded block needs no second pass (the keygen
// leaves that column alone). Returns false when the column is not of that form (the caller then
// takes the ordinary view).
static bool payload_view(const Column* c, int agg_kind, uint64_t* payload, int pw, int a, uint32_t row_base,
                         DecodeBatch* db) {
  const BlockColumn& b = c->data;
  const bool ident = (agg_kind == DG_AGG_LONG_SUM && c->type == DG_COL_LONG) ||
                     (agg_kind == DG_AGG_DOUBLE_SUM && c->type == DG_COL_DOUBLE);
  if (!ident || c->multi_value || b.codec != CODEC_LZ4 || b.vbits || b.width != 8 || !payload) return false;
  if (!b.lit_off.empty()) return false;  // (literal-only blocks are viewed in place: the keygen copies them)
  db->bytes += b.stored_bytes + b.index_bytes;
  const int routes = decode_routes();
  if (taskable(b, routes)) {  // block k's values go to the records of rows row_base + k * size_per ..
    add_tasks(db, b, 0, b.nblocks, reinterpret_cast<uint8_t*>(payload + (size_t)row_base * pw + a),
              (int64_t)b.size_per * pw * 8, pw * 8, nullptr);
    return true;
  }
  for (int32_t k = 0; k < b.nblocks; ++k) {
    const int64_t rows = std::min<int64_t>(b.size_per, (int64_t)b.total - (int64_t)k * b.size_per);
    if (rows <= 0) continue;
    const int64_t r0 = (int64_t)row_base + (int64_t)k * b.size_per;
    Lz4Job j = lz4_job(b, k, reinterpret_cast<uint8_t*>(payload + (size_t)r0 * pw + a), (int32_t)(rows * 8), routes);
    j.vstride = pw * 8;
    db->jobs.push_back(j);
  }
  return true;
}

static int run_expands(CallScratch* cs, DecodeBatch* db, hipStream_t st) {
  if (db->expands.empty()) return DG_OK;
  const int n = (int)db->expands.size();
  VsJob* d;
  VsJob* h = up_take<VsJob>(cs, n, &d, st);
  int32_t* d_err = call_err(cs, st);
  if (!h || !d_err) return set_error(DG_ERR_OOM, "expand jobs");
  memcpy(h, db->expands.data(), sizeof(VsJob) * n);
  DG_FLUSH(cs, st);
  launch_vsize_expand(d, n, db->expand_rows, d_err, st);
  return DG_OK;
}

static int run_lzf(CallScratch* cs, DecodeBatch* db, hipStream_t st) {
  if (db->lzf_jobs.empty()) return DG_OK;
  const int n = (int)db->lzf_jobs.size();
  LzfJob* d;
  LzfJob* h = up_take<LzfJob>(cs, n, &d, st);
  int32_t* d_err = call_err(cs, st);
  if (!h || !d_err) return set_error(DG_ERR_OOM, "lzf jobs");
  memcpy(h, db->lzf_jobs.data(), sizeof(LzfJob) * n);
  DG_FLUSH(cs, st);
  launch_lzf_decode(d, n, d_err, st);
  return DG_OK;
}

static int run_mv_checks(CallScratch* cs, DecodeBatch* db, hipStream_t st) {
  if (db->mv_checks.empty()) return DG_OK;
  const int n = (int)db->mv_checks.size();
  MvCheck* d;
  MvCheck* h = up_take<MvCheck>(cs, n, &d, st);
  int32_t* d_err = call_err(cs, st);
  if (!h || !d_err) return set_error(DG_ERR_OOM, "multi-value checks");
  memcpy(h, db->mv_checks.data(), sizeof(MvCheck) * n);
  DG_FLUSH(cs, st);
  launch_mv_check(d, n, d_err, st);
  db->mv_checks.clear();
  // wait for the verdict before any kernel follows the row lists (an offset past the values would
  // send the consumers' loads out of their buffers); multi-value scans are rare, one sync is cheap
  return finish_call(cs, st);
}

static int run_decodes(CallScratch* cs, DecodeBatch* db, hipStream_t st, uint64_t* d_prof, bool overlap) {
  int rcl = run_decodes_only(cs, db, st, d_prof, overlap);
  if (rcl) return rcl;
  return run_mv_checks(cs, db, st);
}

// overlap (a call whose side stream is otherwise idle: timeseries, topN): the short decoders (run, light)
// go to the side stream beside the general decoder's launch on `st`, joined before `st` continues
static int run_decodes_only(CallScratch* cs, DecodeBatch* db, hipStream_t st, uint64_t* d_prof, bool overlap) {
  int rcl = run_lzf(cs, db, st);
  if (rcl) return rcl;
  int tb[kKinds], nt = 0;  // task blocks per kind, tasks
  int64_t ttb = 0;
  for (int kd = 0; kd < kKinds; ++kd) {
    tb[kd] = 0;
    for (const Lz4Task& t : db->tasks[kd]) tb[kd] += t.n;
    nt += (int)db->tasks[kd].size();
    ttb += tb[kd];
  }
  if (db->jobs.empty() && !ttb) return run_expands(cs, db, st);
  const int n = (int)db->jobs.size();
  // per-block jobs (the few blocks a call plans one by one: skipped / fused time buckets, other
  // routes), partitioned by decoder the way the tasks are kinded:
  // run blocks (value runs with a run index) first, to k_lz4_run;
  // then the general blocks, each kind narrow then wide, flow blocks (k_lz4_decode_flow) after the
  // others; wide blocks (more than 8192 sequences) go to their own launch (twice the per-thread
  // sequence registers); longest first (token-dense blocks cost the most; workgroups dispatch in order,
  // so this is greedy LPT scheduling of the blocks over the CUs and shortens the ragged last wave), for
  // a few waves of blocks only: with hundreds of waves the tail is noise and the host sort is not;
  // light blocks (literal-heavy, short chains) last, to the light decoder (many blocks per CU).
  auto& J = db->jobs;
  const int nr = (int)(std::stable_partition(J.begin(), J.end(), [](const Lz4Job& j) { return j.rx != nullptr; }) - J.begin());
  const int nh = (int)(std::stable_partition(J.begin() + nr, J.end(), [](const Lz4Job& j) { return !j.light; }) - J.begin());
  auto by_kind = [](const Lz4Job& a, const Lz4Job& b) { return a.wide < b.wide; };  // wide: bit 0 | kLzFlow
  std::stable_sort(J.begin() + nr, J.begin() + nh, by_kind);
  int kb[5] = {nr, nr, nr, nr, nh};  // kb[w] .. kb[w + 1]: the general blocks of wide == w
  for (int w = 1; w < 4; ++w)
    kb[w] = (int)(std::lower_bound(J.begin() + nr, J.begin() + nh, w, [](const Lz4Job& j, int v) { return j.wide < v; }) -
                  J.begin());
  auto by_ncp = [](const Lz4Job& a, const Lz4Job& b) { return a.ncp > b.ncp; };
  for (int w = 0; w < 4; ++w)
    if (kb[w + 1] - kb[w] <= 16 * 256) std::stable_sort(J.begin() + kb[w], J.begin() + kb[w + 1], by_ncp);
  int jb[kKinds], jn[kKinds];  // per kind: its per-block jobs J[jb .. jb + jn)
  jb[kKindRun] = 0;
  jn[kKindRun] = nr;
  for (int w = 0; w < 4; ++w) {
    jb[kKindGen0 + w] = kb[w];
    jn[kKindGen0 + w] = kb[w + 1] - kb[w];
  }
  jb[kKindLight] = nh;
  jn[kKindLight] = n - nh;
  // one staged upload: the jobs, the tasks, and per kind the launch blocks' task map + each task's
  // first launch block
  Lz4Job* d;
  Lz4Job* h = up_take<Lz4Job>(cs, n, &d, st);
  Lz4Task* d_tasks = nullptr;
  Lz4Task* h_tasks = nt ? up_take<Lz4Task>(cs, nt, &d_tasks, st) : nullptr;
  int32_t* d_first = nullptr;
  int32_t* h_first = nt ? up_take<int32_t>(cs, nt, &d_first, st) : nullptr;
  int32_t* d_of = nullptr;
  int32_t* h_of = ttb ? up_take<int32_t>(cs, (size_t)ttb, &d_of, st) : nullptr;
  int32_t* d_err = call_err(cs, st);
  if (!h || !d_err || (nt && (!h_tasks || !h_first)) || (ttb && !h_of)) return set_error(DG_ERR_OOM, "lz4 jobs");
  memcpy(h, J.data(), sizeof(Lz4Job) * n);
  Lz4Launch L[kKinds];
  int t_at = 0;
  int64_t of_at = 0;
  for (int kd = 0; kd < kKinds; ++kd) {
    L[kd].jobs = d + jb[kd];
    L[kd].tasks = d_tasks;
    L[kd].task_of = d_of ? d_of + of_at : nullptr;
    L[kd].task_first = d_first;
    L[kd].njobs = jn[kd];
    L[kd].pad = 0;
    int first = jn[kd];
    for (const Lz4Task& t : db->tasks[kd]) {
      h_tasks[t_at] = t;
      h_first[t_at] = first;
      std::fill(h_of + of_at, h_of + of_at + t.n, t_at);
      of_at += t.n;
      first += t.n;
      t_at++;
    }
  }
  DG_FLUSH(cs, st);
  int cnt[kKinds];  // launch blocks per kind
  for (int kd = 0; kd < kKinds; ++kd) cnt[kd] = jn[kd] + tb[kd];
  const int n_run = cnt[kKindRun], n_light = cnt[kKindLight];
  int ng = 0;
  for (int w = 0; w < 4; ++w) ng += cnt[kKindGen0 + w];
  Context* ctx = cs->ctx;
  const bool no_ovl = env_on("DG_NO_OVERLAP");  // (same-box A/B and tests: every decoder on the call's stream)
  const bool ovl = overlap && !no_ovl && ctx && ctx->side && st == ctx->stream && ng > 0 && (n_run > 0 || n_light > 0) && !d_prof;
  hipStream_t ss = st;
  if (ovl) {
    hipEventRecord(ctx->ovl_ev[0], st);
    DG_HIP(hipStreamWaitEvent(ctx->side, ctx->ovl_ev[0], 0));
    ss = ctx->side;
  }
  // staging the input in LDS (104 KiB per block) pays where the run decoder has the CUs to itself: a
  // main-stream launch with nothing beside it stages always, a launch on the side stream next to the main
  // stream's general decoder only when it is small (latency), and a call decoding on the side stream
  // beside the main stream's sort never (it would wait for whole CUs)
  const int stage = ctx && st == ctx->side ? 0 : ss == st ? 2 : 1;
  // with the run blocks beside it, the light blocks follow the general decoder on `st` (the run
  // decoder alone is the longer leg: topN's side stream was run + light while `st` idled)
  const int light_env = [] {
    const char* v = getenv("DG_LIGHT_MAIN");  // (same-box A/B and tests: 1 = light blocks on `st`, 0 = beside)
    return v && *v ? (*v != '0' ? 1 : 0) : -1;
  }();
  const bool light_main = ovl && n_run > 0 && light_env != 0;
  // A groupBy's payload decode on the side stream, beside the main stream's key decode, keygen and sort
  // (round 6): the general decoder first, as kFlowSideWgs persistent workgroups. A flow workgroup
  // needs a whole CU (139 KiB of LDS, every VGPR), which frees only when every smaller workgroup of
  // the other stream on it has finished: one workgroup per block waits for whole CUs again and again
  // (decoder 5.3 ms beside the sort, 1.5 ms alone); launched first, the persistent grid takes its
  // CUs once and keeps them, and the other stream runs on the rest (same box: 10.27-10.32 ->
  // 9.93-9.97 ms per headline step, profiles/r06_v16_ab_gen_first.log).
  // DG_GEN_FIRST=0/1 and DG_FLOW_WGS=k (0: one workgroup per block) override (same-box A/B, tests).
  const bool beside_sort = ctx && st == ctx->side;
  const char* gf = getenv("DG_GEN_FIRST");
  const bool gen_first = ss == st && (gf && *gf ? *gf != '0' : beside_sort);
  const char* fw = getenv("DG_FLOW_WGS");
  const int flow_wgs = fw && *fw ? atoi(fw) : beside_sort ? kFlowSideWgs : 0;
  if (gen_first) {
    if (db->gen_a && ng) phase_event(db->gen_a, st);
    for (int w = 0; w < 4; ++w)
      launch_lz4_decode(L[kKindGen0 + w], cnt[kKindGen0 + w], w, d_err, st,
                        d_prof ? d_prof + (size_t)kb[w] * kLz4ProfWords : nullptr, flow_wgs);
    if (db->gen_a && ng) phase_event(db->gen_b, st);
  }
  launch_lz4_run(L[kKindRun], n_run, stage, d_err, ss);
  if (!light_main)
    launch_lz4_light(L[kKindLight], n_light, d_err, ss, d_prof ? d_prof + (size_t)nh * kLz4ProfWords : nullptr);
  if (ovl) hipEventRecord(ctx->ovl_ev[1], ss);
  for (int i = nr; i < nh; ++i) {
    db->gen_bytes += J[i].src_len;
    if (J[i].wide & kLzFlow) {
      db->flow_blocks++;
      db->flow_bytes += J[i].src_len;
    }
  }
  for (int w = 0; w < 4; ++w) {
    db->gen_bytes += db->task_bytes[kKindGen0 + w];
    if (w & kLzFlow) {
      db->flow_blocks += tb[kKindGen0 + w];
      db->flow_bytes += db->task_bytes[kKindGen0 + w];
    }
  }
  db->gen_blocks += ng;
  for (int w = 0; w < 4; ++w) db->gen_launches += cnt[kKindGen0 + w] > 0;
  if (!gen_first) {
    if (db->gen_a && ng) phase_event(db->gen_a, st);
    for (int w = 0; w < 4; ++w)
      launch_lz4_decode(L[kKindGen0 + w], cnt[kKindGen0 + w], w, d_err, st,
                        d_prof ? d_prof + (size_t)kb[w] * kLz4ProfWords : nullptr, flow_wgs);
    if (db->gen_a && ng) phase_event(db->gen_b, st);
  }
  if (light_main) launch_lz4_light(L[kKindLight], n_light, d_err, st, nullptr);
  if (ovl) DG_HIP(hipStreamWaitEvent(st, ctx->ovl_ev[1], 0));
  return run_expands(cs, db, st);  // errors surface at finish_call
}

// ------------------------------------------------------------------------------------------------
// aggregator plan
// ------------------------------------------------------------------------------------------------
static int slot_op(int kind) {
  switch (kind) {
    case DG_AGG_COUNT:
    case DG_AGG_LONG_SUM: return OP_ADD_I64;
    case DG_AGG_DOUBLE_SUM:
    case DG_AGG_FLOAT_SUM: return OP_ADD_F64;
    case DG_AGG_LONG_MIN:
    case DG_AGG_DOUBLE_MIN:
    case DG_AGG_FLOAT_MIN: return OP_MIN_U64;
    default: return OP_MAX_U64;
  }
}

static uint64_t identity_host(int kind) {
  switch (kind) {
    case DG_AGG_LONG_MIN: return (uint64_t)INT64_MAX ^ 0x8000000000000000ull;
    case DG_AGG_LONG_MAX: return (uint64_t)INT64_MIN ^ 0x8000000000000000ull;
    case DG_AGG_DOUBLE_MIN:
    case DG_AGG_FLOAT_MIN: return 0xFFF0000000000000ull;
    case DG_AGG_DOUBLE_MAX:
    case DG_AGG_FLOAT_MAX: return 0x000FFFFFFFFFFFFFull;
    default: return 0;
  }
}

static double unord_host(uint64_t k) {
  uint64_t u = (k & 0x8000000000000000ull) ? (k & ~0x8000000000000000ull) : ~k;
  double d;
  memcpy(&d, &u, 8);
  return d;
}

// device slot -> ABI slot (int64 / double / float-in-low-bytes)
static uint64_t finalize_slot(int kind, uint64_t s) {
  uint64_t out = 0;
  switch (kind) {
    case DG_AGG_COUNT:
    case DG_AGG_LONG_SUM:
    case DG_AGG_DOUBLE_SUM: return s;
    case DG_AGG_FLOAT_SUM: {
      double d;
      memcpy(&d, &s, 8);
      float f = (float)d;
      memcpy(&out, &f, 4);
      return out;
    }
    case DG_AGG_LONG_MIN:
    case DG_AGG_LONG_MAX: return s ^ 0x8000000000000000ull;
    case DG_AGG_DOUBLE_MIN:
    case DG_AGG_DOUBLE_MAX: {
      bool nan = kind == DG_AGG_DOUBLE_MIN ? s == 0 : s == ~0ull;
      double d = nan ? NAN : unord_host(s);
      memcpy(&out, &d, 8);
      return out;
    }
    default: {
      bool nan = kind == DG_AGG_FLOAT_MIN ? s == 0 : s == ~0ull;
      float f = nan ? NAN : (float)unord_host(s);
      memcpy(&out, &f, 4);
      return out;
    }
  }
}

static int make_plan(const dg_scan* q, AggPlan* plan) {
  if (q->n_aggs < 0 || q->n_aggs > kMaxAggs) return set_error(DG_ERR_UNSUPPORTED, "%d aggregators (max %d)", q->n_aggs, kMaxAggs);
  memset(plan, 0, sizeof *plan);
  plan->n = q->n_aggs;
  for (int a = 0; a < q->n_aggs; ++a) {
    int k = q->aggs[a].kind;
    if (k < DG_AGG_COUNT || k > DG_AGG_FLOAT_MAX) return set_error(DG_ERR_ARG, "aggregator kind %d", k);
    plan->kind[a] = k;
    plan->op[a] = slot_op(k);
  }
  return DG_OK;
}

// ------------------------------------------------------------------------------------------------
// cursors: granularity buckets of one segment (makeCursors / CursorSequenceBuilder.build)
// ------------------------------------------------------------------------------------------------
static const int64_t kMinInstant = -(1ll << 62);
static const int64_t kMaxInstant = (1ll << 62) - 1;

static int64_t floor_mod(int64_t a, int64_t b) {
  int64_t m = a % b;
  return m < 0 ? m + b : m;
}

struct Cursors {
  bool any = false;       // interval overlaps the data interval
  int64_t t_lo = 0, t_hi = 0;  // actual interval
  int64_t bucket0 = 0;    // first bucket start (period) / bucket time (ALL) / first bucket index (calendar)
  int64_t nbuckets = 0;
  bool need_time = false;
};

// Calendar granularity (months, years, zoned or compound periods): the caller's bucket starts
// (Granularity.getIterable of the query interval, Granularity.java:176-240), b[0..nb] with bucket k
// = [b[k], b[k + 1]). The scan is then run on a virtual grid of period 1 whose coordinates are bucket
// indices; the kernels map a timestamp to its index by binary search (bucket_coord).
struct Grain {
  const int64_t* hb = nullptr;  // host bucket starts (nb + 1), null on a period grid
  int32_t nb = 0;
  const int64_t* db = nullptr;  // device copy (uploaded per call)
  bool desc = false;            // descending cursors
  int64_t coord(int64_t t) const {
    return (int64_t)(std::upper_bound(hb, hb + nb + 1, t) - hb) - 1;
  }
  int64_t time_of(int64_t v) const { return hb ? hb[v] : v; }
};

// Validates the scan's granularity and returns the scan the engines run (calendar: period 1 over
// bucket indices).
static int prepare_scan(const dg_scan* in, dg_scan* out, Grain* g) {
  *out = *in;
  *g = Grain();
  g->desc = in->descending != 0;
  if (!in->bucket_starts) {
    if (in->n_bucket_starts) return set_error(DG_ERR_ARG, "n_bucket_starts without bucket_starts");
    if (in->period_ms < 0) return set_error(DG_ERR_ARG, "negative period");
    return DG_OK;
  }
  const int64_t* b = in->bucket_starts;
  const int32_t n = in->n_bucket_starts;
  if (in->period_ms != 0) return set_error(DG_ERR_ARG, "bucket_starts with a period");
  if (n < 2) return set_error(DG_ERR_ARG, "bucket_starts needs at least one bucket (start and end)");
  for (int32_t k = 1; k < n; ++k)
    if (b[k] <= b[k - 1]) return set_error(DG_ERR_ARG, "bucket_starts not strictly ascending at %d", k);
  // the list may start after the interval (bucketStart of the interval start can lie after it:
  // the hours branch before its origin, PeriodGranularity.java:313-326): rows before b[0] are in
  // no cursor (makeCursors clips each cursor to its bucket)
  if (b[n - 1] < in->interval_end) return set_error(DG_ERR_ARG, "bucket_starts do not cover the interval");
  g->hb = b;
  g->nb = n - 1;
  out->period_ms = 1;
  out->origin_ms = 0;
  return DG_OK;
}

static int upload_grain(CallScratch* cs, Grain* g, hipStream_t st) {
  if (!g->hb) return DG_OK;
  int64_t* d;
  int64_t* h = up_take<int64_t>(cs, (size_t)g->nb + 1, &d, st);
  if (!h) return set_error(DG_ERR_OOM, "bucket starts");
  memcpy(h, g->hb, sizeof(int64_t) * ((size_t)g->nb + 1));
  g->db = d;
  return DG_OK;
}

static Cursors plan_cursors(const Segment* seg, int seg_index, const dg_scan* q, const Grain& g) {
  Cursors c;
  if (seg->nrows == 0) return c;
  const int64_t P = q->period_ms;
  const int64_t data_s = seg->min_time;
  if (g.hb) {
    // dataInterval = [minTime, gran.bucketEnd(maxTime)) (QueryableIndexStorageAdapter.makeCursors):
    // the caller's bucketEnd when given, else the end of the listed bucket holding maxTime
    const int64_t km = g.coord(seg->max_time);
    const int64_t data_e = q->seg_bounds ? q->seg_bounds[2 * seg_index + 1]
                                         : (km < 0 ? g.hb[0] : (km >= g.nb ? kMaxInstant : g.hb[km + 1]));
    if (!(q->interval_start < data_e && data_s < q->interval_end)) return c;
    // the segment's cursors start at its iterable's first bucket (gran.bucketStart of the actual start)
    const int64_t it0 = q->seg_bounds ? q->seg_bounds[2 * seg_index] : g.hb[0];
    c.t_lo = std::max(std::max(q->interval_start, data_s), std::max(it0, g.hb[0]));
    c.t_hi = std::min(q->interval_end, data_e);
    if (c.t_lo >= c.t_hi) return c;
    c.any = true;
    c.bucket0 = g.coord(c.t_lo);
    c.nbuckets = g.coord(c.t_hi - 1) - c.bucket0 + 1;
    c.need_time = true;
    return c;
  }
  auto bucket_start = [&](int64_t t) { return P ? t - floor_mod(t - q->origin_ms, P) : kMinInstant; };
  const int64_t data_e = P ? bucket_start(seg->max_time) + P : kMaxInstant;
  if (!(q->interval_start < data_e && data_s < q->interval_end)) return c;
  c.any = true;
  c.t_lo = std::max(q->interval_start, data_s);
  c.t_hi = std::min(q->interval_end, data_e);
  if (P == 0) {
    c.bucket0 = c.t_lo;
    c.nbuckets = 1;
    c.need_time = !(c.t_lo <= seg->min_time && seg->max_time < c.t_hi);
  } else {
    c.bucket0 = bucket_start(c.t_lo);
    c.nbuckets = (c.t_hi - c.bucket0 + P - 1) / P;
    c.need_time = true;
  }
  return c;
}

// The cursor's __time view of a scan (ScanJob / GbJob .time: bucket and interval of every row). An
// LZ4 LONGS block whose rows all fall in one bucket and inside [t_lo, t_hi) is not decoded: its block
// pointer is tagged and points at one representative time (load_time), which gives each of its rows
// the verdict its own time would. Block k's rows lie in [min8[k], max8[k]] (its smallest and largest
// row time, from the attach-time host decode of __time), so no assumption on the row order is needed.
// g: calendar buckets. Per __time block: the bucket (the scan's index, row_selected's formula) its rows
// share inside the interval, or -1 when they may span buckets or leave it. Empty when the blocks' time
// ranges are unknown (not plain LZ4 LONGS, a segment from rows, or DG_NO_TIME_SKIP).
static std::vector<int64_t> time_block_buckets(const Segment* seg, const Column* c, const Cursors& cu, int64_t period,
                                               const Grain& g) {
  std::vector<int64_t> tb;
  if (!c) return tb;
  const BlockColumn& b = c->data;
  (void)seg;
  const bool plain = b.codec == CODEC_LZ4 && !b.vbits && b.width == 8 && (int32_t)b.min8.size() == b.nblocks &&
                     (int32_t)b.max8.size() == b.nblocks && b.nblocks > 0 && !c->multi_value;
  const char* off = getenv("DG_NO_TIME_SKIP");  // (same-box A/B and tests: decode every block)
  if (!plain || (off && *off && *off != '0')) return tb;
  auto bucket = [&](int64_t t) -> int64_t {
    const int64_t v = g.hb ? g.coord(t) : t;
    return period ? (v - cu.bucket0) / period : 0;
  };
  tb.assign(b.nblocks, -1);
  for (int32_t k = 0; k < b.nblocks; ++k) {
    const int64_t lo = b.min8[k], hi = b.max8[k];
    if (lo >= cu.t_lo && hi < cu.t_hi && bucket(lo) == bucket(hi)) tb[k] = bucket(lo);
  }
  return tb;
}

static int time_view(const Column* c, const std::vector<int64_t>& tb, CallScratch* cs,
                     DecodeBatch* db, ColView* v, hipStream_t st) {
  if (tb.empty()) return column_view(c, cs, db, v, st);
  const BlockColumn& b = c->data;
  std::vector<uint8_t> uni(b.nblocks, 0);
  int32_t ndec = 0;
  for (int32_t k = 0; k < b.nblocks; ++k) {
    uni[k] = tb[k] >= 0;
    ndec += !uni[k];
  }
  v->log2_per = b.log2_per;
  v->width = b.width;
  v->pad = 0;
  v->kind = VIEW_LONG;
  uint8_t* slots = ndec ? dev_take<uint8_t>(cs, (size_t)ndec * kBlockBytes + 64) : nullptr;
  int64_t* d_const;
  int64_t* h_const = up_take<int64_t>(cs, std::max(b.nblocks, 1), &d_const, st);
  const uint8_t** d_ptrs;
  const uint8_t** h_ptrs = up_take<const uint8_t*>(cs, std::max(b.nblocks, 1), &d_ptrs, st);
  if ((ndec && !slots) || !h_const || !h_ptrs) return set_error(DG_ERR_OOM, "time view");
  if (ndec) db->last_slots = slots;
  int32_t at = 0;
  const int routes = decode_routes();
  for (int32_t k = 0; k < b.nblocks; ++k) {
    const int64_t rows = std::min<int64_t>(b.size_per, (int64_t)b.total - (int64_t)k * b.size_per);
    if (uni[k]) {
      h_const[k] = b.min8[k];  // (any time of the block's rows: they share the bucket and the interval verdict)
      h_ptrs[k] = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(d_const + k) | 1u);
      continue;
    }
    if (const uint8_t* lit = literal_block(b, k)) {  // its own decoded image
      h_ptrs[k] = lit;
      db->bytes += b.comp_len[k];
      continue;
    }
    uint8_t* slot = slots + (size_t)at++ * kBlockBytes;
    h_ptrs[k] = slot;
    if (rows > 0) {
      db->jobs.push_back(lz4_job(b, k, slot, (int32_t)(rows * 8), routes));
      const Lz4Job& j = db->jobs.back();
      db->bytes += b.comp_len[k] + (j.rx ? run_index_bytes(j.run_n, j.run_far) : 4 * (int64_t)(j.ncp + j.nfine));
    }
  }
  v->blocks = d_ptrs;
  return DG_OK;
}


// ------------------------------------------------------------------------------------------------
// ABI: library & context
// ------------------------------------------------------------------------------------------------
extern "C" {

const char* dg_last_error(void) { return g_err; }
int dg_abi_version(void) { return DG_ABI_VERSION; }

int dg_device_count(int* out) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *out = n;
  return DG_OK;
}

int dg_context_create(int device, dg_context** out) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return set_error(DG_ERR_DEVICE, "no HIP device visible");
  if (device < 0 || device >= n) return set_error(DG_ERR_ARG, "device %d of %d", device, n);
  DG_HIP(hipSetDevice(device));
  Context* ctx = new Context();
  ctx->device = device;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return set_error(DG_ERR_DEVICE, "stream create failed");
  }
  ctx->own_stream = true;
  for (auto& e : ctx->ev) hipEventCreate(&e);
  if (hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking) != hipSuccess) ctx->side = nullptr;
  for (auto& e : ctx->side_ev) hipEventCreate(&e);
  for (auto& e : ctx->gen_ev) hipEventCreate(&e);
  for (auto& e : ctx->ovl_ev) hipEventCreateWithFlags(&e, hipEventDisableTiming);
  *out = reinterpret_cast<dg_context*>(ctx);
  return DG_OK;
}

void dg_context_release(dg_context* c) {
  Context* ctx = reinterpret_cast<Context*>(c);
  if (!ctx) return;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  if (ctx->side) {
    hipStreamSynchronize(ctx->side);
    hipStreamDestroy(ctx->side);
  }
  for (auto& e : ctx->ev) hipEventDestroy(e);
  for (auto& e : ctx->side_ev) hipEventDestroy(e);
  for (auto& e : ctx->gen_ev) hipEventDestroy(e);
  for (auto& e : ctx->ovl_ev) hipEventDestroy(e);
  for (auto& b : ctx->free_blocks) hipFree(b.first);
  if (ctx->own_stream) hipStreamDestroy(ctx->stream);
  delete ctx;
}

int dg_context_set_stream(dg_context* c, void* stream) {
  Context* ctx = reinterpret_cast<Context*>(c);
  std::lock_guard<std::mutex> g(ctx->mu);
  if (ctx->own_stream) hipStreamDestroy(ctx->stream);
  if (stream) {
    ctx->stream = (hipStream_t)stream;
    ctx->own_stream = false;
  } else {
    hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    ctx->own_stream = true;
  }
  return DG_OK;
}

int dg_context_set_limit(dg_context* c, int32_t which, int64_t value) {
  Context* ctx = reinterpret_cast<Context*>(c);
  if (!ctx) return set_error(DG_ERR_ARG, "null context");
  std::lock_guard<std::mutex> g(ctx->mu);
  switch (which) {
    case DG_LIMIT_GROUP_ELEMENTS:
      ctx->max_elements = value <= 0 ? ~0ull : (uint64_t)value;
      return DG_OK;
    default: return set_error(DG_ERR_ARG, "unknown limit %d", which);
  }
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// time bounds (getMinTime / getMaxTime read the first / last __time row)
// ------------------------------------------------------------------------------------------------
int read_time_bounds(Segment* seg) {
  if (seg->nrows == 0) return DG_OK;
  Context* ctx = seg->ctx;
  Column* t = seg->find("__time");
  CallScratch* cs = scratch_of(ctx);
  cs->reset();
  DecodeBatch db;
  ColView v;
  hipStream_t st = ctx->stream;
  const BlockColumn& b = t->data;
  int64_t* h = host_take<int64_t>(cs, 2);
  if (b.vbits || b.codec == CODEC_LZF) {
    // DELTA / TABLE or LZF __time: decode the column once and read its first and last row
    int rc0 = column_view(t, cs, &db, &v, st);
    if (!rc0) rc0 = run_decodes(cs, &db, st);
    if (rc0) return rc0;
    const int64_t last = seg->nrows - 1;
    const uint8_t* first_p = b.vbits ? reinterpret_cast<const uint8_t*>(db.last_expanded) : db.last_slots;
    const uint8_t* last_p = b.vbits ? reinterpret_cast<const uint8_t*>(db.last_expanded + last)
                                    : db.last_slots + (size_t)(last >> b.log2_per) * kBlockBytes +
                                          (size_t)(last & ((1ll << b.log2_per) - 1)) * 8;
    DG_HIP(hipMemcpyAsync(h, first_p, 8, hipMemcpyDeviceToHost, st));
    DG_HIP(hipMemcpyAsync(h + 1, last_p, 8, hipMemcpyDeviceToHost, st));
  } else if (b.codec == CODEC_LZ4) {
    // decode only the first and last block
    uint8_t* slots = dev_take<uint8_t>(cs, 2 * (size_t)kBlockBytes + 64);
    int32_t last = (int32_t)((seg->nrows - 1) >> b.log2_per);
    const uint8_t* img[2];
    for (int k = 0; k < 2; ++k) {
      int32_t blk = k == 0 ? 0 : last;
      int64_t rows = std::min<int64_t>(b.size_per, (int64_t)b.total - (int64_t)blk * b.size_per);
      img[k] = literal_block(b, blk);
      if (!img[k]) {
        img[k] = slots + (size_t)k * kBlockBytes;
        db.jobs.push_back(lz4_job(b, blk, slots + (size_t)k * kBlockBytes, (int32_t)(rows * 8), decode_routes()));
      }
    }
    int rc0 = run_decodes(cs, &db, st);
    if (rc0) return rc0;
    int64_t idx_last = (seg->nrows - 1) & ((1ll << b.log2_per) - 1);
    DG_HIP(hipMemcpyAsync(h, img[0], 8, hipMemcpyDeviceToHost, st));
    DG_HIP(hipMemcpyAsync(h + 1, img[1] + idx_last * 8, 8, hipMemcpyDeviceToHost, st));
  } else {
    std::vector<const uint8_t*> ptrs(b.nblocks);
    DG_HIP(hipMemcpy(ptrs.data(), b.block_ptrs.p, sizeof(void*) * b.nblocks, hipMemcpyDeviceToHost));
    int64_t last = seg->nrows - 1;
    DG_HIP(hipMemcpyAsync(h, ptrs[0], 8, hipMemcpyDeviceToHost, st));
    DG_HIP(hipMemcpyAsync(h + 1, ptrs[last >> b.log2_per] + (last & ((1ll << b.log2_per) - 1)) * 8, 8,
                          hipMemcpyDeviceToHost, st));
  }
  (void)v;
  int rc = finish_call(cs, st);
  if (rc) return rc;
  seg->min_time = h[0];
  seg->max_time = h[1];
  return DG_OK;
}

// ------------------------------------------------------------------------------------------------
// common per-call setup
// ------------------------------------------------------------------------------------------------
// joins the side stream on every exit of a call that launched work on it (its kernels write into the
// call's scratch, which the next call reuses)
struct SideJoin {
  hipStream_t s = nullptr;
  ~SideJoin() {
    if (s) hipStreamSynchronize(s);
  }
};

// memcpy of several (dst, src, bytes) ranges over a few host threads (large result fetches: the
// destination pages fault in on first touch, which one thread alone does slowly)
static void par_copy(const std::vector<std::pair<void*, std::pair<const void*, size_t>>>& parts) {
  size_t total = 0;
  for (auto& p : parts) total += p.second.second;
  const int nt = (int)std::min<size_t>(8, std::max<size_t>(1, total >> 23));
  auto run = [&](int t) {
    for (auto& p : parts) {
      const size_t b = p.second.second, lo = b * t / nt, hi = b * (t + 1) / nt;
      if (hi > lo) memcpy((char*)p.first + lo, (const char*)p.second.first + lo, hi - lo);
    }
  };
  if (nt == 1) {
    run(0);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(run, t);
  run(0);
  for (auto& x : th) x.join();
}

struct CallGuard {
  Context* ctx;
  std::unique_lock<std::mutex> lock;
  CallScratch* cs;
  uint64_t errs0;
  explicit CallGuard(Context* c) : ctx(c), lock(c->mu), cs(scratch_of(c)), errs0(g_err_count) {
    hipSetDevice(c->device);
    cs->reset();
    t_phase_on = !phase_events_off();
    (void)take_launch_error();  // (a previous call's, already reported or abandoned)
  }
  // a call that fails (interrupted, timed out, or any error after launches) drains both streams before
  // it returns: queued kernels and copies still use the call's scratch and staging, which the next call
  // of the context reuses
  ~CallGuard() {
    if (g_err_count != errs0) {
      hipStreamSynchronize(ctx->stream);
      if (ctx->side) hipStreamSynchronize(ctx->side);
    }
    cs->intr = nullptr;
  }
};

// DG_HOST_TRACE=1: per-call host wall stamps (diagnostic) printed to stderr
struct HostTrace {
  bool on;
  std::chrono::steady_clock::time_point t0;
  std::vector<std::pair<const char*, double>> pts;
  HostTrace() : on(getenv("DG_HOST_TRACE") != nullptr), t0(std::chrono::steady_clock::now()) {}
  void mark(const char* what) {
    if (on)
      pts.emplace_back(what, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
  ~HostTrace() {
    if (!on || pts.empty()) return;
    fprintf(stderr, "[dg host]");
    for (auto& p : pts) fprintf(stderr, " %s=%.3f", p.first, p.second);
    fprintf(stderr, "\n");
  }
};

static double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

static int check_segments(dg_segment* const* segs, int32_t n, Context** ctx) {
  if (n <= 0 || !segs) return set_error(DG_ERR_ARG, "no segments");
  Context* c = nullptr;
  for (int i = 0; i < n; ++i) {
    Segment* s = reinterpret_cast<Segment*>(segs[i]);
    if (!s) return set_error(DG_ERR_NOT_FOUND, "null segment");
    if (c && s->ctx != c) return set_error(DG_ERR_ARG, "segments of one call must share a context");
    c = s->ctx;
  }
  *ctx = c;
  return DG_OK;
}


// resolve an aggregator's input column into a view (absent column reads 0) and, for a
// FilteredAggregatorFactory, its filter into a row bitset (the ValueMatcher of
// FilteredBufferAggregator.aggregate, FilteredBufferAggregator.java:45-50: for the supported filters
// the row matcher and the bitmap index select the same rows)
static int agg_view(Segment* seg, const dg_agg& a, CallScratch* cs, DecodeBatch* db, ColView* v, const uint32_t** bits,
                    hipStream_t st) {
  memset(v, 0, sizeof *v);
  v->kind = VIEW_ABSENT;
  *bits = nullptr;
  if (a.filter && a.n_filter > 0) {
    uint32_t* b = nullptr;
    const unsigned long long* cnt = nullptr;
    int rc = build_bitset(seg, cs, a.filter, a.n_filter, &b, &cnt, st);
    if (rc) return rc;
    *bits = b;
  }
  if (a.kind == DG_AGG_COUNT || !a.field) return DG_OK;
  Column* c = seg->find(a.field);
  if (!c) return DG_OK;
  if (c->type == DG_COL_STRING || c->type == DG_COL_UNSUPPORTED)
    return set_error(DG_ERR_UNSUPPORTED, "aggregating non-numeric column %s", a.field);
  return column_view(c, cs, db, v, st);
}

// Timeseries decode fused with aggregation (BlockLayoutColumnarLongsSupplier.java:64-90 reads each
// decompressed block in the loop that consumes it): the LZ4 blocks of an 8-byte long / double input
// whose rows share one bucket inside the interval (time_block_buckets; every block when the cursor
// needs no time) are reduced by the decoder itself into the bucket's slot (Lz4Job.red_*), nothing is
// written; their view pointers are tagged (kViewFused) so the scan takes the identity for those rows.
// Other blocks (light blocks, blocks straddling a bucket edge) are decoded into slots as usual. For an
// unfiltered aggregator other than floatSum (its row-order fp32 recurrence) and count; a filtered scan
// (round 6) folds only the rows of its row bitset `bits`. `out` = the segment's [buckets][rec]
// accumulators, initialised before the decoders run. *whole: every block of the column folds (the
// scan then reads nothing of it). Returns 1 when the aggregator does not qualify (the caller builds
// the plain view).
static int fused_agg_view(Segment* seg, const dg_agg& a, int slot, const std::vector<int64_t>& tb, bool one_bucket,
                          uint64_t* out, int rec, const uint32_t* bits, bool* whole, CallScratch* cs, DecodeBatch* db,
                          ColView* v, hipStream_t st) {
  *whole = false;
  const char* off = getenv("DG_NO_FUSE");  // (same-box A/B and tests: decode every block)
  if ((off && *off && *off != '0') || (a.filter && a.n_filter > 0) || a.kind == DG_AGG_COUNT ||
      a.kind == DG_AGG_FLOAT_SUM || !a.field)
    return 1;
  const Column* c = seg->find(a.field);
  const Column* tc = seg->find("__time");
  if (!c || c->multi_value || (c->type != DG_COL_LONG && c->type != DG_COL_DOUBLE)) return 1;
  const BlockColumn& b = c->data;
  if (b.codec != CODEC_LZ4 || b.vbits || b.width != 8 || b.nblocks <= 0) return 1;
  if (!one_bucket && (tb.empty() || !tc)) return 1;
  const int64_t ts = one_bucket ? 1 : tc->data.size_per;
  std::vector<int64_t> bk(b.nblocks, -1);
  int32_t nfused = 0;
  const int routes = decode_routes();
  for (int32_t k = 0; k < b.nblocks; ++k) {
    const int64_t r0 = (int64_t)k * b.size_per, r1 = std::min<int64_t>((int64_t)b.total, r0 + b.size_per);
    // (light blocks are decoded by k_lz4_light, which does not fold; a run block folds in k_lz4_run)
    const bool run = (routes & kRouteRun) && !b.run_off.empty() && b.run_off[k] >= 0;
    if (r1 <= r0 || literal_block(b, k) || (!run && !b.cp_light.empty() && b.cp_light[k])) continue;
    if (one_bucket) {
      bk[k] = 0;
    } else {
      const int64_t t0 = r0 / ts, t1 = (r1 - 1) / ts;
      if (t1 >= (int64_t)tb.size()) continue;
      int64_t bu = tb[t0];
      for (int64_t t = t0 + 1; t <= t1 && bu >= 0; ++t)
        if (tb[t] != bu) bu = -1;
      bk[k] = bu;
    }
    nfused += bk[k] >= 0;
  }
  if (!nfused) return 1;
  *whole = nfused == b.nblocks;
  v->log2_per = b.log2_per;
  v->width = b.width;
  v->pad = kViewFused;
  v->kind = c->type == DG_COL_LONG ? VIEW_LONG : VIEW_DOUBLE;
  db->bytes += b.stored_bytes + b.index_bytes;
  const int32_t ndec = b.nblocks - nfused;
  uint8_t* slots = ndec ? dev_take<uint8_t>(cs, (size_t)ndec * kBlockBytes + 64) : nullptr;
  const uint8_t** d_ptrs;
  const uint8_t** h_ptrs = up_take<const uint8_t*>(cs, b.nblocks, &d_ptrs, st);
  if ((ndec && !slots) || !h_ptrs) return set_error(DG_ERR_OOM, "fused view");
  if (ndec) db->last_slots = slots;
  int32_t at = 0;
  FoldSpec fold;
  fold.op = slot_op(a.kind);
  fold.kind = a.kind;
  fold.vkind = v->kind;
  fold.code = v->kind == VIEW_LONG ? (a.kind == DG_AGG_LONG_SUM ? kRedLongSum : a.kind == DG_AGG_LONG_MAX ? kRedLongMax
                                      : a.kind == DG_AGG_LONG_MIN ? kRedLongMin : kRedGeneric)
                                   : (a.kind == DG_AGG_DOUBLE_SUM ? kRedDoubleSum : kRedGeneric);
  fold.bits = bits;
  fold.rpb = (int32_t)b.size_per;
  const bool tasks = taskable(b, routes);
  for (int32_t k = 0; k < b.nblocks; ++k) {
    const int64_t rows = std::min<int64_t>(b.size_per, (int64_t)b.total - (int64_t)k * b.size_per);
    if (bk[k] >= 0) {
      h_ptrs[k] = reinterpret_cast<const uint8_t*>((uintptr_t)1);  // tagged: never dereferenced
      fold.dst = out + (size_t)bk[k] * rec + 1 + slot;
      if (tasks) {  // the run of blocks folding into this bucket: one task per kind (light blocks never fold)
        int32_t k1 = k + 1;
        while (k1 < b.nblocks && bk[k1] == bk[k]) h_ptrs[k1++] = reinterpret_cast<const uint8_t*>((uintptr_t)1);
        add_tasks(db, b, k, k1, nullptr, 0, 0, &fold, false);
        db->fused_blocks += k1 - k;
        k = k1 - 1;
        continue;
      }
      Lz4Job j = lz4_job(b, k, nullptr, (int32_t)(rows * 8), routes);
      j.red_dst = fold.dst;
      j.red_op = fold.op;
      j.red_kind = fold.kind;
      j.red_vkind = fold.vkind;
      j.red_code = fold.code;
      j.red_bits = bits;
      j.red_row0 = (int64_t)k * b.size_per;
      db->jobs.push_back(j);
      db->fused_blocks++;
      continue;
    }
    if (const uint8_t* lit = literal_block(b, k)) {  // its own decoded image
      h_ptrs[k] = lit;
      continue;
    }
    uint8_t* dst = slots + (size_t)at++ * kBlockBytes;
    h_ptrs[k] = dst;
    if (rows > 0) db->jobs.push_back(lz4_job(b, k, dst, (int32_t)(rows * 8), routes));
  }
  v->blocks = d_ptrs;
  return DG_OK;
}

// per-segment tile assignment
static int32_t* tile_table(CallScratch* cs, const std::vector<int64_t>& nrows, std::vector<int32_t>* begin, int* ntiles,
                           hipStream_t st) {
  int total = 0;
  begin->resize(nrows.size());
  for (size_t i = 0; i < nrows.size(); ++i) {
    (*begin)[i] = total;
    total += (int)((nrows[i] + kTileRows - 1) / kTileRows);
  }
  *ntiles = total;
  int32_t* d;
  int32_t* h = up_take<int32_t>(cs, std::max(total, 1), &d, st);
  if (!h) return nullptr;
  for (size_t i = 0; i < nrows.size(); ++i) {
    int nt = (int)((nrows[i] + kTileRows - 1) / kTileRows);
    for (int k = 0; k < nt; ++k) h[(*begin)[i] + k] = (int32_t)i;
  }
  return d;
}

static int bits_for(int64_t card) {
  int b = 0;
  while ((1ll << b) < card) b++;
  return b;
}

static bool has_float_sum(const AggPlan& plan) {
  for (int a = 0; a < plan.n; ++a)
    if (plan.kind[a] == DG_AGG_FLOAT_SUM) return true;
  return false;
}

// device buffers of a sort-based grouping of at most `cap` rows with keys of key_bits bits (call
// scratch): one 8-byte word per element [key | row ref] when both fit, else keys + a u32 ref array
static int sort_bufs(CallScratch* cs, int64_t cap, int ntiles_keygen, int key_bits, int pw, SortBufs* sb) {
  memset(sb, 0, sizeof *sb);
  sb->cap = cap;
  sb->ntiles_sort = sort_tiles(cap);
  const int rb = bits_for(std::max<int64_t>(cap, 1));
  const bool packed = key_bits + rb <= 64;
  sb->ref_bits = packed ? rb : 0;
  const size_t c = (size_t)std::max<int64_t>(cap, 1) + 16;
  for (int k = 0; k < 2; ++k) {
    sb->keys[k] = dev_take<uint64_t>(cs, c);
    sb->refs[k] = packed ? nullptr : dev_take<uint32_t>(cs, c);
    if (!sb->keys[k] || (!packed && !sb->refs[k])) return set_error(DG_ERR_OOM, "sort buffers of %lld rows", (long long)cap);
  }
  sb->pw = pw;
  if (pw > 0) {
    sb->payload = dev_take<uint64_t>(cs, c * (size_t)pw);
    if (!sb->payload) return set_error(DG_ERR_OOM, "payload of %lld rows", (long long)cap);
  }
  sb->tile_cnt = dev_take<uint32_t>(cs, (size_t)std::max(ntiles_keygen, 1));
  sb->n = dev_take<uint32_t>(cs, 4);
  sb->lb_status = dev_take<uint64_t>(cs, (size_t)kMaxBins * sb->ntiles_sort);
  // per-pass digit totals + tile counters (radix_passes)
  // + one tile counter for the groupBy reduce's look-back
  sb->bin_total = dev_take<uint32_t>(cs, (size_t)kMaxBins * kRsMaxPasses + kRsMaxPasses + 1);
  sb->run_cnt = dev_take<uint32_t>(cs, (size_t)sb->ntiles_sort);
  if (!sb->tile_cnt || !sb->n || !sb->lb_status || !sb->bin_total || !sb->run_cnt) return set_error(DG_ERR_OOM, "sort tables");
  return DG_OK;
}

// keygen tiles + row refs of the call's jobs, and the job table in HBM
static int upload_gb_jobs(CallScratch* cs, std::vector<GbJob>& gj, const std::vector<int64_t>& rows, GbJob** d_jobs,
                          int32_t** d_tile, int* ntiles, int64_t* total, hipStream_t st) {
  if (gj.size() > (size_t)kMaxCallSegs) return set_error(DG_ERR_UNSUPPORTED, "%zu segments in one call (max %d)", gj.size(), kMaxCallSegs);
  std::vector<int32_t> begin;
  *d_tile = tile_table(cs, rows, &begin, ntiles, st);
  if (!*d_tile) return set_error(DG_ERR_OOM, "tile table");
  int64_t t = 0;
  for (size_t i = 0; i < gj.size(); ++i) {
    gj[i].tile_begin = begin[i];
    gj[i].row_base = (uint32_t)t;
    gj[i].nrows = (int32_t)rows[i];
    t += rows[i];
  }
  if (t >= (1ll << 32)) return set_error(DG_ERR_UNSUPPORTED, "%lld rows in one call (row refs are 32-bit)", (long long)t);
  *total = t;
  GbJob* h = up_take<GbJob>(cs, gj.size(), d_jobs, st);
  if (!h) return set_error(DG_ERR_OOM, "job table");
  memcpy(h, gj.data(), sizeof(GbJob) * gj.size());
  return DG_OK;
}

// elements of a keygen over rows with multi-value dimensions (one per grouping), counted on the
// device before the sort buffers are sized
// (counted in 64 bits: rows x the product of their value-list lengths can pass 2^32, and element
// indices / sort offsets are 32-bit, so such a call is refused before anything is sized from it)
static int count_elements(CallScratch* cs, GbJob* d_jobs, int32_t* d_tile, int ntiles, int64_t* total,
                          hipStream_t st) {
  const int nt = std::max(ntiles, 1);
  uint32_t* d_cnt = dev_take<uint32_t>(cs, (size_t)nt + 4);
  unsigned long long* d_tot = dev_take<unsigned long long>(cs, 1);
  unsigned long long* h_tot = host_take<unsigned long long>(cs, 1);
  if (!d_cnt || !d_tot || !h_tot) return set_error(DG_ERR_OOM, "element count");
  DG_FLUSH(cs, st);
  launch_gb_count_total(d_jobs, d_tile, ntiles, d_cnt, d_tot, st);
  DG_HIP(hipMemcpyAsync(h_tot, d_tot, 8, hipMemcpyDeviceToHost, st));
  int rc = finish_call(cs, st);
  if (rc) return rc;
  const unsigned long long cap = std::min<unsigned long long>(cs->ctx->max_elements, (1ull << 32) - 64);
  if (*h_tot > cap)
    return set_error(DG_ERR_UNSUPPORTED, "multi-value grouping explodes into %llu elements (limit %llu)", *h_tot, cap);
  *total = (int64_t)*h_tot;
  return DG_OK;
}

// floatSum of the per-segment engines (timeseries, topN), as the reference computes it: every
// (segment, bucket[, id]) cell's float32 sum in row order, written over the cell's slot in the
// accumulator tables (the scan kernels accumulate floatSum in fp64 first; this pass replaces it).
// Keys are already in (segment, bucket) order unless `sort`.
static int fsum_pass(CallScratch* cs, std::vector<GbJob>& gj, const std::vector<int64_t>& rows, int key_bits, bool sort,
                     const AggPlan& plan, hipStream_t st, bool desc) {
  if (key_bits > 64) return set_error(DG_ERR_UNSUPPORTED, "floatSum cell key of %d bits", key_bits);
  GbJob* d_jobs;
  int32_t* d_tile;
  int ntiles = 0;
  int64_t total = 0;
  int rc = upload_gb_jobs(cs, gj, rows, &d_jobs, &d_tile, &ntiles, &total, st);
  if (rc) return rc;
  bool multi = false;
  for (const GbJob& g : gj) multi |= g.multi != 0;
  if (multi) {
    rc = count_elements(cs, d_jobs, d_tile, ntiles, &total, st);
    if (rc) return rc;
  }
  SortBufs sb;
  rc = sort_bufs(cs, total, ntiles, key_bits, plan.n, &sb);
  if (rc) return rc;
  uint32_t* head_pos = dev_take<uint32_t>(cs, (size_t)total + 16);
  if (!head_pos) return set_error(DG_ERR_OOM, "floatSum runs");
  DG_FLUSH(cs, st);
  launch_gb_keygen(d_jobs, d_tile, ntiles, &sb, plan, st, multi);
  if (sort) launch_radix_sort(&sb, key_bits, st);
  launch_run_heads(&sb, st);
  launch_run_mark(&sb, head_pos, st);
  for (int a = 0; a < plan.n; ++a)
    if (plan.kind[a] == DG_AGG_FLOAT_SUM)
      launch_fsum_runs(d_jobs, (int)gj.size(), ntiles, &sb, plan, a, head_pos, nullptr, 0, st, desc ? 1 : 0);
  return DG_OK;
}

static void gb_copy_aggs(GbJob* g, const ScanJob& j) {
  memcpy(g->vals, j.vals, sizeof g->vals);
  memcpy(g->agg_bits, j.agg_bits, sizeof g->agg_bits);
}

}  // namespace dg

using namespace dg;

extern "C" {

// ------------------------------------------------------------------------------------------------
// segments
// ------------------------------------------------------------------------------------------------
int dg_segment_attach(dg_context* c, const char* dir, dg_segment** out) {
  Context* ctx = reinterpret_cast<Context*>(c);
  if (!ctx || !dir || !out) return set_error(DG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  Segment* seg = nullptr;
  int rc = load_segment(ctx, dir, &seg);
  if (rc) return rc;
  *out = reinterpret_cast<dg_segment*>(seg);
  return DG_OK;
}

int dg_segment_from_rows(dg_context* c, int64_t n_rows, const int64_t* timestamps, int64_t interval_start,
                         int64_t interval_end, const dg_row_column* columns, int32_t n_columns, dg_segment** out) {
  Context* ctx = reinterpret_cast<Context*>(c);
  if (!ctx || !out) return set_error(DG_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> g(ctx->mu);
  hipSetDevice(ctx->device);
  Segment* seg = nullptr;
  int rc = segment_from_rows(ctx, n_rows, timestamps, interval_start, interval_end, columns, n_columns, &seg);
  if (rc) return rc;
  *out = reinterpret_cast<dg_segment*>(seg);
  return DG_OK;
}

void dg_segment_release(dg_segment* s) {
  Segment* seg = reinterpret_cast<Segment*>(s);
  if (!seg) return;
  std::lock_guard<std::mutex> g(seg->ctx->mu);
  hipSetDevice(seg->ctx->device);
  delete seg;
}

int64_t dg_segment_num_rows(const dg_segment* s) { return reinterpret_cast<const Segment*>(s)->nrows; }

int dg_segment_interval(const dg_segment* s, int64_t* st, int64_t* en) {
  const Segment* seg = reinterpret_cast<const Segment*>(s);
  *st = seg->istart;
  *en = seg->iend;
  return DG_OK;
}

int dg_segment_time_bounds(const dg_segment* s, int64_t* mn, int64_t* mx) {
  const Segment* seg = reinterpret_cast<const Segment*>(s);
  *mn = seg->min_time;
  *mx = seg->max_time;
  return DG_OK;
}

int dg_segment_num_columns(const dg_segment* s) { return (int)reinterpret_cast<const Segment*>(s)->columns.size(); }

const char* dg_segment_column_name(const dg_segment* s, int i) {
  const Segment* seg = reinterpret_cast<const Segment*>(s);
  if (i < 0 || i >= (int)seg->columns.size()) return nullptr;
  return seg->columns[i]->name.c_str();
}

int dg_segment_column_type(const dg_segment* s, const char* col) {
  const Column* c = reinterpret_cast<const Segment*>(s)->find(col ? col : "");
  return c ? c->type : DG_COL_MISSING;
}

int64_t dg_segment_device_bytes(const dg_segment* s) { return reinterpret_cast<const Segment*>(s)->device_bytes; }

int32_t dg_segment_dim_cardinality(const dg_segment* s, const char* dim) {
  const Column* c = reinterpret_cast<const Segment*>(s)->find(dim ? dim : "");
  if (!c || c->type != DG_COL_STRING) return -1;
  return (int32_t)c->dict.size();
}

int dg_segment_dim_value(const dg_segment* s, const char* dim, int32_t id, const char** out, int32_t* len) {
  const Column* c = reinterpret_cast<const Segment*>(s)->find(dim ? dim : "");
  if (!c || c->type != DG_COL_STRING) return set_error(DG_ERR_NOT_FOUND, "no string column %s", dim ? dim : "");
  if (id < 0 || id >= (int32_t)c->dict.size()) return set_error(DG_ERR_ARG, "id %d out of range", id);
  *out = c->dict[id].c_str();
  *len = c->dict_null[id] ? -1 : (int32_t)c->dict[id].size();
  return DG_OK;
}

int dg_segment_dim_dictionary(const dg_segment* s, const char* dim, int64_t* offsets, char* bytes, int64_t* total) {
  const Column* c = reinterpret_cast<const Segment*>(s)->find(dim ? dim : "");
  if (!c || c->type != DG_COL_STRING) return set_error(DG_ERR_NOT_FOUND, "no string column %s", dim ? dim : "");
  int64_t t = 0;
  for (size_t i = 0; i < c->dict.size(); ++i) {
    if (offsets) offsets[i] = t;
    if (bytes) memcpy(bytes + t, c->dict[i].data(), c->dict[i].size());
    t += (int64_t)c->dict[i].size();
  }
  if (offsets) offsets[c->dict.size()] = t;
  if (total) *total = t;
  return DG_OK;
}

int dg_segment_set_dim_order(dg_segment* s, const char* dim, int32_t slot, const int32_t* rank, int32_t card,
                             int32_t has_ties) {
  Segment* seg = reinterpret_cast<Segment*>(s);
  if (!seg || !dim || !rank) return set_error(DG_ERR_ARG, "null argument");
  if (slot < 0 || slot >= kOrderSlots) return set_error(DG_ERR_ARG, "order slot %d", slot);
  Column* c = seg->find(dim);
  if (!c || c->type != DG_COL_STRING) return set_error(DG_ERR_NOT_FOUND, "no string column %s", dim);
  if (card != (int32_t)c->dict.size()) return set_error(DG_ERR_ARG, "rank of %d ids for cardinality %zu", card, c->dict.size());
  for (int32_t i = 0; i < card; ++i)
    if (rank[i] < 0 || rank[i] >= card) return set_error(DG_ERR_ARG, "rank[%d] = %d out of range", i, rank[i]);
  std::lock_guard<std::mutex> g(seg->ctx->mu);
  hipSetDevice(seg->ctx->device);
  DevBuf& b = c->order_rank[slot];
  if (!b.alloc(sizeof(int32_t) * (size_t)std::max(card, 1))) return set_error(DG_ERR_OOM, "hipMalloc order");
  if (card) DG_HIP(hipMemcpy(b.p, rank, sizeof(int32_t) * (size_t)card, hipMemcpyHostToDevice));
  c->order_host[slot].assign(rank, rank + card);
  c->order_ties[slot] = has_ties != 0;
  c->order_set[slot] = true;
  return DG_OK;
}

int dg_filter_bitmap(dg_segment* s, const dg_filter* filter, int32_t n_filter, uint32_t* out_words, int64_t* out_count) {
  Segment* seg = reinterpret_cast<Segment*>(s);
  if (!seg || !out_words) return set_error(DG_ERR_ARG, "null argument");
  CallGuard g(seg->ctx);
  hipStream_t st = seg->ctx->stream;
  uint32_t* bits = nullptr;
  const unsigned long long* count = nullptr;
  int rc = build_bitset(seg, g.cs, filter, n_filter, &bits, &count, st);
  if (rc) return rc;
  const int64_t nwords = (seg->nrows + 31) / 32;
  if (!bits) {
    for (int64_t w = 0; w < nwords; ++w) out_words[w] = 0xFFFFFFFFu;
    if (seg->nrows & 31) out_words[nwords - 1] = (1u << (seg->nrows & 31)) - 1u;
  } else {
    DG_HIP(hipMemcpyAsync(out_words, bits, nwords * 4, hipMemcpyDeviceToHost, st));
  }
  rc = finish_call(g.cs, st);
  if (rc) return rc;
  if (out_count) *out_count = count ? (int64_t)*count : seg->nrows;
  return DG_OK;
}

// ------------------------------------------------------------------------------------------------
// timeseries
// ------------------------------------------------------------------------------------------------
int dg_timeseries_run(dg_segment* const* segs, int32_t n, const dg_scan* q, int32_t bucket_cap, int32_t* out_nb,
                      int64_t* out_time, int64_t* out_rows, uint64_t* out_values, dg_metrics* metrics) {
  auto t0 = std::chrono::steady_clock::now();
  HostTrace ht;
  Context* ctx;
  int rc = check_segments(segs, n, &ctx);
  if (rc) return rc;
  if (!q) return set_error(DG_ERR_ARG, "null scan");
  dg_scan qs;
  Grain gr;
  rc = prepare_scan(q, &qs, &gr);
  if (rc) return rc;
  q = &qs;
  AggPlan plan;
  rc = make_plan(q, &plan);
  if (rc) return rc;
  CallGuard g(ctx);
  CallScratch* cs = g.cs;
  Interrupt intr(q, t0);
  cs->intr = &intr;
  hipStream_t st = ctx->stream;
  rc = upload_grain(cs, &gr, st);
  if (rc) return rc;
  dg_metrics m;
  memset(&m, 0, sizeof m);
  const int na = plan.n, rec = na + 1;
  std::vector<Cursors> cur(n);
  std::vector<ScanJob> jobs(n);
  std::vector<int64_t> tiles_rows(n, 0);
  std::vector<const unsigned long long*> counts(n, nullptr);
  const bool fsum = has_float_sum(plan);
  std::vector<char> staged_acc(n, 0), skip_scan(n, 0);
  bool any_part = false;
  DecodeBatch db, db0;  // db0: the first segment's decodes, launched while the host plans the others
  decode_events(ctx, &db, false);
  decode_events(ctx, &db0, true);
  bool early = false;
  phase_event(ctx->ev[0], st);
  ht.mark("setup");
  for (int i = 0; i < n; ++i) {
    if (i == 1) ht.mark("segment0");
    Segment* seg = reinterpret_cast<Segment*>(segs[i]);
    cur[i] = plan_cursors(seg, i, q, gr);
    out_nb[i] = (int32_t)(cur[i].any ? cur[i].nbuckets : 0);
    m.segment_rows += seg->nrows;
    if (!cur[i].any) continue;
    if (cur[i].nbuckets > bucket_cap) return set_error(DG_ERR_ARG, "%lld buckets > cap %d", (long long)cur[i].nbuckets, bucket_cap);
    uint32_t* bits = nullptr;
    rc = build_bitset(seg, cs, q->filter, q->n_filter, &bits, &counts[i], st);
    if (rc) return rc;
    ScanJob& j = jobs[i];
    memset(&j, 0, sizeof j);
    j.nrows = (int32_t)seg->nrows;
    j.bitset = bits;
    j.t_lo = cur[i].t_lo;
    j.t_hi = cur[i].t_hi;
    j.bucket0 = cur[i].bucket0;
    j.period = q->period_ms;
    j.bounds = gr.db;
    j.nbounds = gr.nb + 1;
    j.nbuckets = (int32_t)cur[i].nbuckets;
    j.time.kind = VIEW_ABSENT;
    const Column* tcol = seg->find("__time");
    std::vector<int64_t> tb;
    if (cur[i].need_time) {
      tb = time_block_buckets(seg, tcol, cur[i], q->period_ms, gr);
      if (i == 0) ht.mark("seg0_buckets");
      rc = time_view(tcol, tb, cs, &db, &j.time, st);
      if (rc) return rc;
      if (i == 0) ht.mark("seg0_time_view");
    }
    // the accumulators: a small table starts as identities in the call's upload (no fill kernel)
    const size_t outn = (size_t)cur[i].nbuckets * rec;
    if (outn * 8 <= kStagedAccBytes) {
      uint64_t* h = up_take<uint64_t>(cs, outn, &j.out, st);
      if (!h) return set_error(DG_ERR_OOM, "accumulators");
      for (int64_t b = 0; b < cur[i].nbuckets; ++b)
        for (int k = 0; k < rec; ++k) h[b * rec + k] = k == 0 ? 0ull : identity_host(plan.kind[k - 1]);
      staged_acc[i] = 1;
    } else {
      j.out = dev_take<uint64_t>(cs, outn);
    }
    if (!j.out) return set_error(DG_ERR_OOM, "accumulators");
    // A one-bucket scan that needs no row time and whose every aggregator is a plain count or folded
    // whole by the decoders reads nothing row by row: no scan tiles; its rows and counts are the
    // filter's row count (the interval covers the segment) or the segment's rows, set after the call.
    bool no_rows = cur[i].nbuckets == 1 && !cur[i].need_time && !fsum;
    for (int a = 0; a < na; ++a) {
      rc = 1;
      bool whole = false;
      if (!fsum)
        rc = fused_agg_view(seg, q->aggs[a], a, tb, !cur[i].need_time, j.out, rec, bits, &whole, cs, &db, &j.vals[a], st);
      if (rc == 1) rc = agg_view(seg, q->aggs[a], cs, &db, &j.vals[a], &j.agg_bits[a], st);
      if (rc) return rc;
      no_rows &= whole || (q->aggs[a].kind == DG_AGG_COUNT && !(q->aggs[a].filter && q->aggs[a].n_filter > 0));
    }
    skip_scan[i] = no_rows ? 1 : 0;
    if (!no_rows && cur[i].nbuckets == 1) {  // one bucket: per-tile records + one fold (k_scan_combine)
      j.part = dev_take<uint64_t>(cs, (size_t)std::max<int64_t>((seg->nrows + kTileRows - 1) / kTileRows, 1) * rec);
      if (!j.part) return set_error(DG_ERR_OOM, "scan partials");
      any_part = true;
    }
    tiles_rows[i] = no_rows ? 0 : seg->nrows;
    // A call over several segments launches the first segment's decodes as soon as they are planned
    // (its accumulators initialised first: fused blocks fold into them), so the device works while
    // the host plans the rest (configs[4]a: ≈ 40 µs per segment of host planning).
    bool work = !db.jobs.empty();
    for (const auto& t : db.tasks) work |= !t.empty();
    if (i == 0 && n > 1 && work) {
      std::swap(db, db0);
      std::swap(db.gen_a, db0.gen_a);
      std::swap(db.gen_b, db0.gen_b);
      if (cur[0].any && !staged_acc[0]) {
        SlotInit init0{};
        for (int a = 0; a < na; ++a) init0.v[1 + a] = identity_host(plan.kind[a]);
        launch_fill_u64(jobs[0].out, cur[0].nbuckets, rec, init0, st);
      }
      phase_event(ctx->ev[1], st);
      rc = run_decodes(cs, &db0, st, nullptr, true);
      if (rc) return rc;
      early = true;
      ht.mark("seg0_decode_launched");
    }
  }
  DG_CHECK_INTERRUPT(intr);
  ht.mark("planned");
  // init accumulators (before the decoders: fused blocks combine into them)
  SlotInit init{};
  for (int a = 0; a < na; ++a) init.v[1 + a] = identity_host(plan.kind[a]);
  for (int i = early ? 1 : 0; i < n; ++i)
    if (cur[i].any && !staged_acc[i]) launch_fill_u64(jobs[i].out, cur[i].nbuckets, rec, init, st);
  // the scan's tile table and jobs staged before the decode: one upload carries them with its jobs
  std::vector<int32_t> begin;
  int ntiles = 0;
  for (int i = 0; i < n; ++i)
    if (!cur[i].any) tiles_rows[i] = 0;
  int32_t* d_tile = tile_table(cs, tiles_rows, &begin, &ntiles, st);
  if (!d_tile) return set_error(DG_ERR_DEVICE, "tile table");
  for (int i = 0; i < n; ++i) jobs[i].tile_begin = begin[i];
  ScanJob* d_jobs;
  ScanJob* h_jobs = up_take<ScanJob>(cs, n, &d_jobs, st);
  if (!h_jobs) return set_error(DG_ERR_OOM, "scan jobs");
  memcpy(h_jobs, jobs.data(), sizeof(ScanJob) * n);
  if (!early) phase_event(ctx->ev[1], st);
  rc = run_decodes(cs, &db, st, nullptr, true);
  if (rc) return rc;
  phase_event(ctx->ev[2], st);
  ht.mark("decode_launched");
  m.bytes_read = db.bytes + db0.bytes;
  DG_CHECK_INTERRUPT(intr);
  DG_FLUSH(cs, st);  // (a no-op unless the decode staged nothing)
  phase_event(ctx->ev[3], st);
  launch_scan_agg(d_jobs, d_tile, ntiles, plan, 0, st);
  if (any_part) launch_scan_combine(d_jobs, n, plan, st);
  DG_CHECK_INTERRUPT(intr);
  if (fsum) {
    // floatSum as the reference adds it: float32, one row at a time per cursor (bucket)
    std::vector<GbJob> gj(n);
    std::vector<int64_t> frows(n, 0);
    int64_t maxb = 1;
    for (int i = 0; i < n; ++i)
      if (cur[i].any) maxb = std::max<int64_t>(maxb, cur[i].nbuckets);
    const int bb = bits_for(maxb);
    for (int i = 0; i < n; ++i) {
      GbJob& f = gj[i];
      memset(&f, 0, sizeof f);
      if (!cur[i].any) continue;
      f.bitset = jobs[i].bitset;
      f.time = jobs[i].time;
      f.t_lo = jobs[i].t_lo;
      f.t_hi = jobs[i].t_hi;
      f.bucket0 = cur[i].bucket0;
      f.period = q->period_ms;
      f.bounds = gr.db;
      f.nbounds = gr.nb + 1;
      f.seg_slot = i;
      f.seg_shift = bb;
      f.bucket_bits = bb;
      gb_copy_aggs(&f, jobs[i]);
      f.fs_out = jobs[i].out;
      f.fs_mul = 1;
      frows[i] = jobs[i].nrows;
    }
    rc = fsum_pass(cs, gj, frows, bb + bits_for(n), false, plan, st, gr.desc);
    if (rc) return rc;
  }
  phase_event(ctx->ev[4], st);
  // results
  std::vector<uint64_t*> h_out(n, nullptr);
  for (int i = 0; i < n; ++i) {
    if (!cur[i].any) continue;
    h_out[i] = host_take<uint64_t>(cs, (size_t)cur[i].nbuckets * rec);
    if (!h_out[i]) return set_error(DG_ERR_OOM, "results");
    if (staged_acc[i]) cs->late.push_back({h_out[i], jobs[i].out, (size_t)cur[i].nbuckets * rec * 8});
    else DG_HIP(hipMemcpyAsync(h_out[i], jobs[i].out, (size_t)cur[i].nbuckets * rec * 8, hipMemcpyDeviceToHost, st));
  }
  ht.mark("agg_launched");
  rc = finish_call(cs, st);
  ht.mark("synced");
  if (rc) return rc;
  for (int i = 0; i < n; ++i) {
    if (!cur[i].any) continue;
    const int64_t pre = counts[i] ? (int64_t)*counts[i] : reinterpret_cast<Segment*>(segs[i])->nrows;
    m.pre_filtered_rows += pre;
    if (skip_scan[i]) {  // no scan: the bucket's rows and plain counts are the selected rows
      h_out[i][0] = (uint64_t)pre;
      for (int a = 0; a < na; ++a)
        if (plan.kind[a] == DG_AGG_COUNT) h_out[i][1 + a] = (uint64_t)pre;
    }
    for (int64_t b = 0; b < cur[i].nbuckets; ++b) {
      // cursor order: a descending query emits the buckets last to first (:378-381)
      const int64_t o = (int64_t)i * bucket_cap + (gr.desc ? cur[i].nbuckets - 1 - b : b);
      out_time[o] = q->period_ms ? gr.time_of(cur[i].bucket0 + b * q->period_ms) : cur[i].t_lo;
      out_rows[o] = (int64_t)h_out[i][b * rec];
      m.selected_rows += out_rows[o];
      for (int a = 0; a < na; ++a) out_values[o * na + a] = finalize_slot(plan.kind[a], h_out[i][b * rec + 1 + a]);
    }
  }
  float f1 = 0, f2 = 0, f3 = 0;
  phase_elapsed(&f1, ctx->ev[0], ctx->ev[1]);
  phase_elapsed(&f2, ctx->ev[1], ctx->ev[2]);
  phase_elapsed(&f3, ctx->ev[3], ctx->ev[4]);
  m.bitmap_ms = f1;
  m.bitmap_bytes = cs->bitmap_bytes;
  m.decode_ms = f2;
  decode_metrics(db, db0, &m, early ? ctx->ev[0] : nullptr);
  m.aggregate_ms = f3;
  m.total_ms = ms_since(t0);
  if (metrics) *metrics = m;
  return DG_OK;
}

// ------------------------------------------------------------------------------------------------
// topN
// ------------------------------------------------------------------------------------------------
static uint64_t metric_key_host(uint64_t slot, int kind, int inverted) {
  uint64_t k;
  auto ord = [](double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
  };
  int op = slot_op(kind);
  if (op == OP_ADD_I64) {
    k = slot ^ 0x8000000000000000ull;
  } else if (op == OP_ADD_F64) {
    double d;
    memcpy(&d, &slot, 8);
    if (kind == DG_AGG_FLOAT_SUM) d = (double)(float)d;
    k = std::isnan(d) ? ~0ull : ord(d);
  } else if (kind == DG_AGG_LONG_MIN || kind == DG_AGG_LONG_MAX) {
    k = slot;
  } else {
    bool nan = op == OP_MIN_U64 ? slot == 0 : slot == ~0ull;
    if (nan) k = ~0ull;
    else {
      double d = unord_host(slot);
      if (kind == DG_AGG_FLOAT_MIN || kind == DG_AGG_FLOAT_MAX) d = (double)(float)d;
      k = ord(d);
    }
  }
  return inverted ? ~k : k;
}

int dg_topn_run(dg_segment* const* segs, int32_t n, const dg_scan* q, const dg_topn* t, int32_t* out_n, int32_t* out_ids,
                uint64_t* out_values, dg_metrics* metrics) {
  auto t0 = std::chrono::steady_clock::now();
  HostTrace ht;
  Context* ctx;
  int rc = check_segments(segs, n, &ctx);
  if (rc) return rc;
  if (!q || !t || !t->dimension) return set_error(DG_ERR_ARG, "null argument");
  dg_scan qs;
  Grain gr;
  rc = prepare_scan(q, &qs, &gr);
  if (rc) return rc;
  q = &qs;
  // non-ALL granularity: one cursor (and result list) per bucket, TopNQueryEngine.java:80-104
  const int bcap = q->period_ms ? t->bucket_cap : 1;
  if (bcap <= 0) return set_error(DG_ERR_ARG, "bucket_cap");
  if (q->period_ms && !t->out_bucket_time) return set_error(DG_ERR_ARG, "out_bucket_time");
  const bool dim = t->dim_order >= 0;
  if (dim && t->dim_order >= kOrderSlots) return set_error(DG_ERR_ARG, "order slot %d", t->dim_order);
  if (!dim && (t->metric_agg < 0 || t->metric_agg >= q->n_aggs)) return set_error(DG_ERR_ARG, "metric index");
  if (t->threshold <= 0) return set_error(DG_ERR_ARG, "threshold");
  AggPlan plan;
  rc = make_plan(q, &plan);
  if (rc) return rc;
  CallGuard g(ctx);
  CallScratch* cs = g.cs;
  Interrupt intr(q, t0);
  cs->intr = &intr;
  hipStream_t st = ctx->stream;
  rc = upload_grain(cs, &gr, st);
  if (rc) return rc;
  dg_metrics m;
  memset(&m, 0, sizeof m);
  const int na = plan.n, rec = na + 1;
  // topN bin index (Column::tix_*): used when every segment's dimension is a present single-value
  // column, over ALL granularity, with no floatSum pass and the bin's table within LDS; the first
  // topN over a column builds it from the decoded ids, later ones skip the id decode and the per-call
  // row partition (DG_NO_TOPN_INDEX=1: the per-call bins, k_topn_bin_*)
  bool use_ix = q->period_ms == 0 && !has_float_sum(plan) && ((size_t)rec << kTopnIxShift) * 8 <= 48 * 1024 &&
                !env_on("DG_NO_TOPN_INDEX");
  for (int i = 0; i < n && use_ix; ++i) {
    const Column* c = reinterpret_cast<Segment*>(segs[i])->find(t->dimension);
    use_ix = c && c->type == DG_COL_STRING && !c->multi_value;
  }
  std::vector<char> ix_skip(n, 0);  // segment i's ids are not decoded (its index is built)
  std::vector<Cursors> cur(n);
  std::vector<ScanJob> jobs(n);
  std::vector<int64_t> card(n, 1), tiles_rows(n, 0);
  std::vector<const unsigned long long*> counts(n, nullptr);
  DecodeBatch db;
  decode_events(ctx, &db, false);
  bool any_multi = false;
  phase_event(ctx->ev[0], st);
  for (int i = 0; i < n; ++i) {
    Segment* seg = reinterpret_cast<Segment*>(segs[i]);
    cur[i] = plan_cursors(seg, i, q, gr);
    m.segment_rows += seg->nrows;
    for (int b = 0; b < bcap; ++b) out_n[(int64_t)i * bcap + b] = -1;
    if (!cur[i].any) continue;
    if (cur[i].nbuckets > bcap) return set_error(DG_ERR_ARG, "segment %d has %lld buckets > bucket_cap %d", i,
                                                 (long long)cur[i].nbuckets, bcap);
    ScanJob& j = jobs[i];
    memset(&j, 0, sizeof j);
    Column* dc = seg->find(t->dimension);
    if (dc && dc->type != DG_COL_STRING) return set_error(DG_ERR_UNSUPPORTED, "topN on non-string dimension %s", t->dimension);
    uint32_t* bits = nullptr;
    rc = build_bitset(seg, cs, q->filter, q->n_filter, &bits, &counts[i], st);
    if (rc) return rc;
    j.nrows = (int32_t)seg->nrows;
    j.bitset = bits;
    j.t_lo = cur[i].t_lo;
    j.t_hi = cur[i].t_hi;
    j.time.kind = VIEW_ABSENT;
    if (cur[i].need_time) {
      rc = time_view(seg->find("__time"), time_block_buckets(seg, seg->find("__time"), cur[i], q->period_ms, gr), cs, &db, &j.time, st);
      if (rc) return rc;
    }
    if (dc) {
      if (dim && !dc->order_set[t->dim_order])
        return set_error(DG_ERR_ARG, "order slot %d of %s not set (dg_segment_set_dim_order)", t->dim_order, t->dimension);
      if (dc->multi_value) {  // every value of a row's list aggregates the row
        rc = multi_view(dc, cs, &db, &j.key, &j.key_off, st);
        any_multi = true;
      } else if (use_ix && dc->tix_ready) {
        ix_skip[i] = 1;
      } else {
        rc = column_view(dc, cs, &db, &j.key, st);
      }
      if (rc) return rc;
      card[i] = std::max<int64_t>((int64_t)dc->dict.size(), 1);
    } else {
      // missing dimension: every row has the null value -> one group (id 0)
      static_assert(sizeof(ColView) == 24, "ColView layout");
      memset(&j.key, 0, sizeof j.key);
      j.key.kind = VIEW_ABSENT;
      card[i] = 1;
    }
    for (int a = 0; a < na; ++a) {
      rc = agg_view(seg, q->aggs[a], cs, &db, &j.vals[a], &j.agg_bits[a], st);
      if (rc) return rc;
    }
    j.out = nullptr;  // allocated below with the bins
    tiles_rows[i] = seg->nrows;
  }
  DG_CHECK_INTERRUPT(intr);
  phase_event(ctx->ev[1], st);
  ht.mark("planned");
  // dictionary-id bins: every segment's table [card][rec] is written whole by the bin reduce
  const int shift = use_ix ? kTopnIxShift : topn_bin_shift(na);
  std::vector<int32_t> bin_first(n, 0), bin_seg;
  int64_t cap = 0;
  for (int i = 0; i < n; ++i) {
    bin_first[i] = (int32_t)bin_seg.size();
    if (!cur[i].any) continue;
    // table keys: dictionary ids, or bucket * cardinality + id over granularity buckets
    const int64_t nkeys = card[i] * (q->period_ms ? cur[i].nbuckets : 1);
    if (nkeys > (1ll << 31) - 1 || (double)nkeys * rec * 8 > 16e9)
      return set_error(DG_ERR_UNSUPPORTED, "topN table of %lld keys", (long long)nkeys);
    jobs[i].nbuckets = (int32_t)nkeys;
    jobs[i].key_card = q->period_ms ? (int32_t)card[i] : 0;
    jobs[i].bucket0 = cur[i].bucket0;
    jobs[i].period = q->period_ms;
    jobs[i].bounds = gr.db;
    jobs[i].nbounds = gr.nb + 1;
    jobs[i].out = dev_take<uint64_t>(cs, (size_t)nkeys * rec);
    if (!jobs[i].out) return set_error(DG_ERR_OOM, "topN table");
    const int64_t nb = (nkeys + (1ll << shift) - 1) >> shift;
    for (int64_t k = 0; k < nb; ++k) bin_seg.push_back(i);
    cap += tiles_rows[i];
  }
  const int nbins = (int)bin_seg.size();
  // staged: bin_first[n] | bin_seg[nbins] | hist[nbins] (zero) | base | cursor
  const size_t nbw = (size_t)std::max(nbins, 1);
  int32_t* d_bin_first;
  int32_t* h_bins = up_take<int32_t>(cs, (size_t)n + 4 * nbw, &d_bin_first, st);
  uint16_t* d_lid = use_ix ? nullptr : dev_take<uint16_t>(cs, (size_t)std::max<int64_t>(cap, 1) + 8);
  uint64_t* d_bvals = use_ix ? nullptr : dev_take<uint64_t>(cs, (size_t)std::max<int64_t>(cap, 1) * std::max(na, 1));
  if (!h_bins || (!use_ix && (!d_lid || !d_bvals))) return set_error(DG_ERR_OOM, "topN bins");
  memcpy(h_bins, bin_first.data(), sizeof(int32_t) * n);
  if (nbins) memcpy(h_bins + n, bin_seg.data(), sizeof(int32_t) * nbins);
  memset(h_bins + n + nbw, 0, 4 * nbw);
  int32_t* d_bin_seg = d_bin_first + n;
  uint32_t* d_bins = reinterpret_cast<uint32_t*>(d_bin_first + n + nbw);  // hist | base | cursor
  std::vector<int32_t> begin;
  int ntiles = 0;
  int32_t* d_tile = tile_table(cs, tiles_rows, &begin, &ntiles, st);
  if (!d_tile) return set_error(DG_ERR_DEVICE, "tile table");
  for (int i = 0; i < n; ++i) jobs[i].tile_begin = begin[i];
  ScanJob* d_jobs;
  ScanJob* h_jobs = up_take<ScanJob>(cs, n, &d_jobs, st);
  if (!h_jobs) return set_error(DG_ERR_OOM, "scan jobs");
  memcpy(h_jobs, jobs.data(), sizeof(ScanJob) * n);
  // the segments' bin indexes; those not built yet are built by this call from its decoded ids
  TopnIx* d_ix = nullptr;
  std::vector<int> ix_build;
  if (use_ix) {
    TopnIx* h_ix = up_take<TopnIx>(cs, n, &d_ix, st);
    if (!h_ix) return set_error(DG_ERR_OOM, "topN index table");
    for (int i = 0; i < n; ++i) {
      memset(&h_ix[i], 0, sizeof(TopnIx));
      if (!cur[i].any) continue;
      Column* dc = reinterpret_cast<Segment*>(segs[i])->find(t->dimension);
      bool queued = false;  // (a segment listed twice: one build)
      for (int k : ix_build) queued |= reinterpret_cast<Segment*>(segs[k])->find(t->dimension) == dc;
      if (!dc->tix_ready && !queued) {
        const int64_t nb = (card[i] + (1ll << shift) - 1) >> shift;
        const size_t rows = (size_t)std::max<int64_t>(jobs[i].nrows, 1);
        if (!dc->tix_perm.alloc(4 * rows) || !dc->tix_lid.alloc(2 * rows) || !dc->tix_base.alloc(4 * (size_t)(nb + 1)))
          return set_error(DG_ERR_OOM, "topN index of %s", t->dimension);
        ix_build.push_back(i);
      }
      h_ix[i] = TopnIx{dc->tix_perm.as<uint32_t>(), dc->tix_lid.as<uint16_t>(), dc->tix_base.as<uint32_t>()};
    }
  }
  // missing-dimension segments: the key view is absent; load_id would fault, so route them
  // through a 1-entry table with a zero id view
  for (int i = 0; i < n; ++i) {
    if (cur[i].any && !ix_skip[i] && jobs[i].key.kind == VIEW_ABSENT) {
      // a constant-zero id column: block pointer table pointing at a zeroed 64 KiB slot
      uint8_t* zero = dev_take<uint8_t>(cs, kBlockBytes);
      DG_HIP(hipMemsetAsync(zero, 0, kBlockBytes, st));
      const int nb = (int)((jobs[i].nrows + 65535) / 65536) + 1;
      const uint8_t** dp;
      const uint8_t** hp = up_take<const uint8_t*>(cs, nb, &dp, st);
      if (!hp) return set_error(DG_ERR_OOM, "zero id view");
      for (int k = 0; k < nb; ++k) hp[k] = zero;
      ScanJob fixed = jobs[i];
      fixed.key.blocks = dp;
      fixed.key.log2_per = 16;
      fixed.key.width = 1;
      fixed.key.pad = 0;
      fixed.key.kind = VIEW_IDS;
      h_jobs[i] = fixed;
    }
  }
  // selection + gather of the candidates' records, all segments in one launch (staged before the
  // decode: its upload carries the bins', the scan's and the selection's tables)
  const int mk = dim ? DG_AGG_COUNT : plan.kind[t->metric_agg];
  const int metric_agg = dim ? 0 : t->metric_agg;
  const int metric_op = (slot_op(mk) << 8) | mk;
  std::vector<TopnSelJob> sel;
  std::vector<int> sel_seg, sel_bucket;  // one selection per (segment, bucket)
  std::vector<int64_t> jgcap, jgoff, out_base;
  int64_t max_card = 0, gtotal = 0;
  // DimensionTopNMetricSpec: per segment the dictionary order, the computeStartEnd id range
  // (BaseTopNAlgorithm.java:296-326; only LEXICOGRAPHIC is optimized, DimensionTopNMetricSpec.java:117-124)
  // and whether the order has comparator-equal values (then the builder's queue is replayed literally)
  std::vector<const int32_t*> dim_rank(n, nullptr), dim_rank_host(n, nullptr);
  std::vector<int32_t> dim_lo(n, 0), dim_hi(n, 0);
  std::vector<char> dim_ties(n, 0);
  bool any_ties = false;
  if (dim) {
    for (int i = 0; i < n; ++i) {
      if (!cur[i].any) continue;
      Segment* seg = reinterpret_cast<Segment*>(segs[i]);
      const Column* dc = seg->find(t->dimension);
      const int32_t cd = (int32_t)card[i];
      if (dc) {
        dim_rank[i] = dc->order_rank[t->dim_order].as<int32_t>();
        dim_rank_host[i] = dc->order_host[t->dim_order].data();
        dim_ties[i] = (char)dc->order_ties[t->dim_order];
        any_ties |= dim_ties[i] != 0;
      }
      int32_t lo = 0, hi = cd;
      if (t->dim_order == 2 * DG_ORDER_LEXICOGRAPHIC) {
        if (t->previous_stop) {
          // lookupId(previousStop) + 1, negated when missing; a missing dimension's selector
          // resolves only null / "" (to id 0)
          int64_t look;
          if (dc) look = (int64_t)index_of(dc, t->previous_stop) + 1;
          else look = t->previous_stop[0] == 0 ? 1 : 0;
          if (look < 0) look = -look;
          lo = look > cd ? cd : (int32_t)look;
        }
        const bool covers = q->interval_start <= seg->istart && seg->iend <= q->interval_end && seg->istart < q->interval_end;
        if (q->n_filter == 0 && covers) hi = (int32_t)std::min<int64_t>(hi, (int64_t)lo + t->threshold);
      }
      dim_lo[i] = lo;
      dim_hi[i] = hi;
    }
  }
  // with comparator-equal values every eligible id is a candidate (the queue is replayed in id order)
  const int sel_threshold = any_ties ? 0x3fffffff : t->threshold;
  for (int i = 0; i < n; ++i) {
    if (!cur[i].any) continue;
    for (int64_t b = 0; b < (q->period_ms ? cur[i].nbuckets : 1); ++b) {
      // candidates = ids whose key >= the K-th key: the threshold plus ties, rarely more
      int64_t gc = std::min<int64_t>(card[i], 2 * (int64_t)t->threshold + 64);
      if (any_ties) gc = card[i];
      sel_seg.push_back(i);
      sel_bucket.push_back((int)b);
      // cursor order: a descending query emits the buckets last to first
      const int64_t L = (int64_t)i * bcap + (q->period_ms && gr.desc ? cur[i].nbuckets - 1 - b : b);
      out_base.push_back(L);
      if (q->period_ms) t->out_bucket_time[L] = gr.time_of(cur[i].bucket0 + b * q->period_ms);
      jgcap.push_back(gc);
      jgoff.push_back(gtotal);
      gtotal += gc * (rec + 1) + (gc + 3) / 4;  // records + u16 builder order
    }
  }
  // read-back block (one D2H copy): gathered records of every (segment, bucket)
  uint64_t* d_gath = dev_take<uint64_t>(cs, (size_t)std::max<int64_t>(gtotal, 1));
  if (!d_gath) return set_error(DG_ERR_OOM, "topN gather");
  for (size_t k = 0; k < sel_seg.size(); ++k) {
    const int i = sel_seg[k];
    TopnSelJob sj;
    memset(&sj, 0, sizeof sj);
    sj.table = jobs[i].out + (size_t)sel_bucket[k] * (size_t)card[i] * rec;
    sj.card = card[i];
    sj.cand = dev_take<int32_t>(cs, (size_t)card[i]);
    sj.keys = dev_take<uint64_t>(cs, (size_t)card[i]);
    sj.blkcnt = dev_take<int32_t>(cs, (size_t)((card[i] + kSelBlock - 1) / kSelBlock));
    sj.gather_cap = (int32_t)jgcap[k];
    if (dim) {
      sj.dim_mode = 1;
      sj.rank = dim_rank[i];
      sj.lo = dim_lo[i];
      sj.hi = dim_hi[i];
      sj.min_rank = t->min_rank ? t->min_rank[i] : 0;
    }
    sj.gathered = d_gath + jgoff[k];
    sj.order = reinterpret_cast<uint16_t*>(d_gath + jgoff[k] + jgcap[k] * (rec + 1));
    if (!sj.cand || !sj.keys || !sj.blkcnt) return set_error(DG_ERR_OOM, "topN candidates");
    max_card = std::max(max_card, card[i]);
    sel.push_back(sj);
  }
  const int ns = (int)sel.size();
  // staged zero block: per selection state[4] | ncand (+pad) | radix state[9][4] | hist[8][256] words
  const size_t sel_words = 4 + 1 + 36 + 8 * 256 / 2;
  uint64_t* d_selmem;
  uint64_t* h_selz = up_take<uint64_t>(cs, sel_words * std::max(ns, 1), &d_selmem, st);
  TopnSelJob* d_sel;
  TopnSelJob* h_sel = up_take<TopnSelJob>(cs, std::max(ns, 1), &d_sel, st);
  if (!h_selz || !h_sel) return set_error(DG_ERR_OOM, "topN selection");
  memset(h_selz, 0, 8 * sel_words * std::max(ns, 1));
  for (int k = 0; k < ns; ++k) {
    sel[k].state = d_selmem + sel_words * k;
    sel[k].ncand = reinterpret_cast<int32_t*>(d_selmem + sel_words * k + 4);
    sel[k].rstate = d_selmem + sel_words * k + 5;
    sel[k].hist = reinterpret_cast<uint32_t*>(d_selmem + sel_words * k + 41);
  }
  if (ns) memcpy(h_sel, sel.data(), sizeof(TopnSelJob) * ns);
  rc = run_decodes(cs, &db, st, nullptr, true);
  ht.mark("decode_launched");
  if (rc) return rc;
  phase_event(ctx->ev[2], st);
  m.bytes_read = db.bytes;
  phase_event(ctx->ev[3], st);
  if (any_multi) {
    // multi-value dimension: per-(row, value) atomics into identity-initialised tables
    SlotInit init{};
    for (int a = 0; a < na; ++a) init.v[1 + a] = identity_host(plan.kind[a]);
    DG_FLUSH(cs, st);
    for (int i = 0; i < n; ++i)
      if (cur[i].any) launch_fill_u64(jobs[i].out, jobs[i].nbuckets, rec, init, st);
    launch_scan_agg(d_jobs, d_tile, ntiles, plan, 1, st);
  } else {
    DG_FLUSH(cs, st);
    if (use_ix) {
      for (int i : ix_build) {
        const int nb = (int)((card[i] + (1ll << shift) - 1) >> shift);
        uint32_t* d_cnt = dev_take<uint32_t>(cs, 2 * (size_t)(nb + 1));  // counts (+ a zero) | cursors
        if (!d_cnt) return set_error(DG_ERR_OOM, "topN index build");
        DG_HIP(hipMemsetAsync(d_cnt, 0, 4 * (size_t)(nb + 1), st));
        Column* dc = reinterpret_cast<Segment*>(segs[i])->find(t->dimension);
        launch_topn_ix_build(d_jobs, i, jobs[i].nrows, shift, nb, d_cnt, d_cnt + nb + 1, dc->tix_base.as<uint32_t>(),
                             dc->tix_perm.as<uint32_t>(), dc->tix_lid.as<uint16_t>(), st);
      }
      launch_topn_ix_reduce(d_jobs, d_ix, d_bin_first, d_bin_seg, nbins, shift, plan, st);
    } else {
      launch_topn_bins(d_jobs, d_tile, ntiles, d_bin_first, d_bin_seg, nbins, shift, d_bins, d_bins + nbins,
                       d_bins + 2 * (size_t)nbins, plan, d_lid, d_bvals, std::max<int64_t>(cap, 1), st);
    }
  }
  ht.mark("bins_launched");
  if (has_float_sum(plan)) {
    // floatSum as the reference adds it: float32, one row at a time per (cursor, dictionary id)
    // position of the pooled buffer (PooledTopNAlgorithm.aggregateDimValue -> FloatSumBufferAggregator)
    std::vector<GbJob> gj(n);
    std::vector<int64_t> frows(n, 0);
    int64_t maxb = 1, maxc = 1;
    for (int i = 0; i < n; ++i)
      if (cur[i].any) {
        maxb = std::max<int64_t>(maxb, q->period_ms ? cur[i].nbuckets : 1);
        maxc = std::max<int64_t>(maxc, card[i]);
      }
    const int bb = q->period_ms ? bits_for(maxb) : 0, ib = bits_for(maxc);
    for (int i = 0; i < n; ++i) {
      GbJob& f = gj[i];
      memset(&f, 0, sizeof f);
      if (!cur[i].any) continue;
      f.bitset = jobs[i].bitset;
      f.time = jobs[i].time;
      f.t_lo = jobs[i].t_lo;
      f.t_hi = jobs[i].t_hi;
      f.bucket0 = cur[i].bucket0;
      f.period = q->period_ms;
      f.bounds = gr.db;
      f.nbounds = gr.nb + 1;
      f.ndims = 1;
      f.dims[0] = jobs[i].key;  // VIEW_ABSENT for a missing dimension: id 0 (its null value)
      f.moff[0] = jobs[i].key_off;
      f.multi = any_multi;
      f.skip_empty = 1;
      f.dim_bits[0] = ib;
      f.bucket_shift = ib;
      f.bucket_bits = bb;
      f.seg_slot = i;
      f.seg_shift = ib + bb;
      gb_copy_aggs(&f, jobs[i]);
      f.fs_out = jobs[i].out;
      f.fs_mul = jobs[i].key_card;
      frows[i] = jobs[i].nrows;
    }
    rc = fsum_pass(cs, gj, frows, bits_for(n) + bb + ib, true, plan, st, gr.desc);
    if (rc) return rc;
  }
  if (ns) {
    DG_FLUSH(cs, st);
    launch_topn_select(d_sel, ns, max_card, na, metric_agg, metric_op, t->inverted, sel_threshold, st);
    ht.mark("select_launched");
  }
  phase_event(ctx->ev[4], st);
  uint64_t* h_selmem = host_take<uint64_t>(cs, sel_words * (size_t)std::max(ns, 1));
  uint64_t* h_gath = host_take<uint64_t>(cs, (size_t)std::max<int64_t>(gtotal, 1));
  if (!h_selmem || !h_gath) return set_error(DG_ERR_OOM, "topN read-back");
  if (ns) {
    // (state + ncand of each selection, not its histograms)
    DG_HIP(hipMemcpy2DAsync(h_selmem, 8 * sel_words, d_selmem, 8 * sel_words, 8 * 5, (size_t)ns, hipMemcpyDeviceToHost, st));
    DG_HIP(hipMemcpyAsync(h_gath, d_gath, 8 * (size_t)gtotal, hipMemcpyDeviceToHost, st));
  }
  std::vector<int32_t> h_ncand_v(std::max(ns, 1));
  int32_t* h_ncand = h_ncand_v.data();
  uint64_t* h_state = h_selmem;
  std::vector<int32_t*> h_cand(ns, nullptr);
  std::vector<uint64_t*> h_tab(ns, nullptr);
  rc = finish_call(cs, st);
  ht.mark("synced");
  if (rc) return rc;
  for (int i : ix_build) {  // (the index's HBM counts toward the segment's footprint from now on)
    Segment* seg = reinterpret_cast<Segment*>(segs[i]);
    Column* dc = seg->find(t->dimension);
    dc->tix_ready = true;
    seg->device_bytes += (int64_t)(dc->tix_perm.n + dc->tix_lid.n + dc->tix_base.n);
  }
  for (int k = 0; k < ns; ++k) h_ncand[k] = *reinterpret_cast<const int32_t*>(h_selmem + sel_words * k + 4);
  // k_topn_order left a list's records in output order (`sorted_at`); the replays that walk the
  // candidates in id order unpack them first (ids + rec-strided slots, back in id order)
  auto ordered = [&](int k) { return h_ncand[k] > 0 && h_ncand[k] <= jgcap[k] && h_ncand[k] <= kTopnOrderCap; };
  auto order_of = [&](int k) { return reinterpret_cast<const uint16_t*>(h_gath + jgoff[k] + jgcap[k] * (rec + 1)); };
  auto sorted_at = [&](int k, int e) { return h_gath + jgoff[k] + (int64_t)e * (rec + 1); };  // [id, rec slots]
  auto unpack = [&](int k) -> int {
    if (h_cand[k]) return DG_OK;
    const int64_t g = std::min<int64_t>(jgcap[k], h_ncand[k]);
    h_cand[k] = host_take<int32_t>(cs, (size_t)std::max<int64_t>(jgcap[k], 1));
    h_tab[k] = host_take<uint64_t>(cs, (size_t)std::max<int64_t>(jgcap[k], 1) * rec);
    if (!h_cand[k] || !h_tab[k]) return set_error(DG_ERR_OOM, "topN read-back");
    const uint64_t* src = h_gath + jgoff[k];
    const uint16_t* ord = ordered(k) ? order_of(k) : nullptr;
    for (int64_t e = 0; e < g; ++e) {
      const int64_t c = ord ? ord[e] : e;
      h_cand[k][c] = (int32_t)src[e * (rec + 1)];
      memcpy(h_tab[k] + c * rec, src + e * (rec + 1) + 1, 8 * (size_t)rec);
    }
    return DG_OK;
  };
  ht.mark("unpacked");
  // rare: more candidates than the speculative read-back held (many ties at the K-th key)
  bool again = false;
  for (int k = 0; k < ns; ++k) {
    const int nc = h_ncand[k];
    if (nc <= jgcap[k]) continue;
    again = true;
    h_cand[k] = host_take<int32_t>(cs, (size_t)nc);
    h_tab[k] = host_take<uint64_t>(cs, (size_t)nc * rec);
    if (!h_cand[k] || !h_tab[k]) return set_error(DG_ERR_OOM, "topN read-back");
    DG_HIP(hipMemcpyAsync(h_cand[k], sel[k].cand, 4 * (size_t)nc, hipMemcpyDeviceToHost, st));
  }
  if (again) {
    DG_HIP(hipStreamSynchronize(st));
    for (int k = 0; k < ns; ++k) {
      const int nc = h_ncand[k];
      if (nc <= jgcap[k]) continue;
      for (int c = 0; c < nc;) {  // candidates ascend: copy contiguous id runs
        int e = c + 1;
        while (e < nc && h_cand[k][e] == h_cand[k][e - 1] + 1) e++;
        DG_HIP(hipMemcpyAsync(h_tab[k] + (size_t)c * rec, sel[k].table + (size_t)h_cand[k][c] * rec,
                              (size_t)(e - c) * rec * 8, hipMemcpyDeviceToHost, st));
        c = e;
      }
    }
    DG_HIP(hipStreamSynchronize(st));
  }
  for (int i = 0; i < n; ++i)
    if (cur[i].any) m.pre_filtered_rows += counts[i] ? (int64_t)*counts[i] : reinterpret_cast<Segment*>(segs[i])->nrows;
  ht.mark("overflow_checked");
  // replay TopNNumericResultBuilder over the candidates in id (= dimension value) order
  for (int k = 0; k < ns; ++k) {
    if (k == 1) ht.mark("replayed_seg0");
    const int i = sel_seg[k];
    m.selected_rows += (int64_t)h_state[sel_words * k + 1];
    const int nc = h_ncand[k];
    struct E {
      uint64_t key;
      int32_t id;
      int32_t idx;
    };
    const int K = t->threshold;
    if (dim) {
      // TopNLexicographicResultBuilder (TopNLexicographicResultBuilder.java:40-176) over the eligible
      // ids in id order: every non-null value is offered (shouldAdd compares the head's unset metric
      // value, null, with it), the queue's head is the largest value under the comparator and is
      // polled past the threshold; build() sorts the queue's array by the comparator (stable).
      const int32_t* hr = dim_rank_host[i];
      auto rank_of = [&](int c) { return hr ? hr[h_cand[k][c]] : 0; };
      std::vector<int> res;
      if (!dim_ties[i] && ordered(k)) {  // distinct ranks: the K smallest, ascending = the first K in order
        const int nout = std::min(nc, K);
        out_n[out_base[k]] = nout;
        for (int e = 0; e < nout; ++e) {
          const int64_t o = out_base[k] * t->threshold + (int64_t)e;
          const uint64_t* r = sorted_at(k, e);
          out_ids[o] = (int32_t)r[0];
          for (int a = 0; a < na; ++a) out_values[o * na + a] = finalize_slot(plan.kind[a], r[2 + a]);
        }
        continue;
      }
      if ((rc = unpack(k))) return rc;
      if (!dim_ties[i]) {
        res.resize(nc);
        for (int c = 0; c < nc; ++c) res[c] = c;
        std::sort(res.begin(), res.end(), [&](int a, int b) { return rank_of(a) < rank_of(b); });
        if ((int)res.size() > K) res.resize(K);
      } else {  // java.util.PriorityQueue, literally (OpenJDK 8 siftUp / siftDown)
        const Column* dc = reinterpret_cast<Segment*>(segs[i])->find(t->dimension);
        auto is_null = [&](int c) { return !dc || dc->dict_null[h_cand[k][c]]; };
        auto pq_cmp = [&](int a, int b) { return (rank_of(b) > rank_of(a)) - (rank_of(b) < rank_of(a)); };
        std::vector<int> q;
        for (int c = 0; c < nc; ++c) {
          if ((int)q.size() >= K && is_null(c)) continue;
          int x = c, at = (int)q.size();
          q.push_back(c);
          while (at > 0) {
            const int parent = (at - 1) >> 1;
            if (pq_cmp(x, q[parent]) >= 0) break;
            q[at] = q[parent];
            at = parent;
          }
          q[at] = x;
          if ((int)q.size() > K) {  // poll
            const int last = q.back();
            q.pop_back();
            const int size = (int)q.size();
            if (size) {
              int a = 0;
              const int half = size >> 1;
              while (a < half) {
                int child = 2 * a + 1;
                const int right = child + 1;
                if (right < size && pq_cmp(q[child], q[right]) > 0) child = right;
                if (pq_cmp(last, q[child]) <= 0) break;
                q[a] = q[child];
                a = child;
              }
              q[a] = last;
            }
          }
        }
        res = q;
        std::stable_sort(res.begin(), res.end(), [&](int a, int b) { return rank_of(a) < rank_of(b); });
      }
      out_n[out_base[k]] = (int32_t)res.size();
      for (size_t e = 0; e < res.size(); ++e) {
        const int64_t o = out_base[k] * t->threshold + (int64_t)e;
        out_ids[o] = h_cand[k][res[e]];
        for (int a = 0; a < na; ++a) out_values[o * na + a] = finalize_slot(plan.kind[a], h_tab[k][(size_t)res[e] * rec + 1 + a]);
      }
      continue;
    }
    std::vector<E> v;
    if (ordered(k)) {
      // k_topn_order sorted the candidates by (key desc, id asc) and left their records in that
      // order; keep every key > kth and, of the kth ties, those the builder's queue keeps (see
      // below), already in output order
      const uint16_t* ord = order_of(k);
      auto key_at = [&](int e) { return metric_key_host(sorted_at(k, e)[2 + t->metric_agg], mk, t->inverted); };
      const int r = std::min(nc, K) - 1;
      const uint64_t kth = key_at(r);
      bool exact = key_at(nc - 1) >= kth;  // nothing below the K-th key
      if (exact) {
        int g = 0, gF = 0;
        while (g < nc && key_at(g) > kth) gF += ord[g++] < K;
        int skip = g - gF;  // ties popped by later pushes into the full queue, oldest first
        int nout = 0;
        auto emit = [&](int e) {
          const int64_t o = out_base[k] * t->threshold + (int64_t)nout++;
          const uint64_t* rr = sorted_at(k, e);
          out_ids[o] = (int32_t)rr[0];
          for (int a = 0; a < na; ++a) out_values[o * na + a] = finalize_slot(plan.kind[a], rr[2 + a]);
        };
        for (int e = 0; e < g; ++e) emit(e);
        for (int e = g; e < nc && nout < K; ++e) {
          if (ord[e] >= K) continue;  // a tie after the queue filled is never pushed
          if (skip > 0) {
            skip--;
            continue;
          }
          emit(e);
        }
        out_n[out_base[k]] = (int32_t)nout;
        continue;
      }
    }
    if ((rc = unpack(k))) return rc;
    std::vector<E> all(nc);
    for (int c = 0; c < nc; ++c)
      all[c] = E{metric_key_host(h_tab[k][(size_t)c * rec + 1 + t->metric_agg], mk, t->inverted), h_cand[k][c], c};
    // The candidates are the ids whose key >= the K-th largest key (kth), in id order. The builder's
    // priority queue (min-heap on (key, id), push when not full or top.key < key, pop the minimum
    // when over K) then keeps every key > kth and, of the kth ties, those pushed while it was not
    // full minus one per later push into a full queue, oldest (= smallest id) first: linear time.
    uint64_t kth = 0;
    if (nc > 0) {
      std::vector<uint64_t> keys(nc);
      for (int c = 0; c < nc; ++c) keys[c] = all[c].key;
      const int r = std::min(nc, K) - 1;
      std::nth_element(keys.begin(), keys.begin() + r, keys.end(), std::greater<uint64_t>());
      kth = keys[r];
    }
    bool fifo = true;
    for (int c = 0; c < nc && fifo; ++c) fifo = all[c].key >= kth;
    if (fifo) {
      std::vector<int> ties;
      int count = 0;
      size_t popped = 0;
      for (int c = 0; c < nc; ++c) {
        if (all[c].key > kth) {
          v.push_back(all[c]);
          if (count < K) count++;
          else popped++;
        } else if (count < K) {
          ties.push_back(c);
          count++;
        }
      }
      for (size_t q = popped; q < ties.size(); ++q) v.push_back(all[ties[q]]);
    } else {  // not reached for an exact K-th key; the builder's queue, literally
      auto less = [](const E& a, const E& b) { return a.key != b.key ? a.key < b.key : a.id < b.id; };
      auto gt = [&](const E& a, const E& b) { return less(b, a); };
      std::priority_queue<E, std::vector<E>, decltype(gt)> pq(gt);  // min-heap on (key, id)
      for (int c = 0; c < nc; ++c) {
        if ((int)pq.size() < K || pq.top().key < all[c].key) pq.push(all[c]);
        if ((int)pq.size() > K) pq.pop();
      }
      while (!pq.empty()) {
        v.push_back(pq.top());
        pq.pop();
      }
    }
    std::sort(v.begin(), v.end(), [](const E& a, const E& b) { return a.key != b.key ? a.key > b.key : a.id < b.id; });
    out_n[out_base[k]] = (int32_t)v.size();
    for (size_t e = 0; e < v.size(); ++e) {
      const int64_t o = out_base[k] * t->threshold + (int64_t)e;
      out_ids[o] = v[e].id;
      for (int a = 0; a < na; ++a) out_values[o * na + a] = finalize_slot(plan.kind[a], h_tab[k][(size_t)v[e].idx * rec + 1 + a]);
    }
  }
  ht.mark("replayed");
  float f1 = 0, f2 = 0, f3 = 0;
  phase_elapsed(&f1, ctx->ev[0], ctx->ev[1]);
  phase_elapsed(&f2, ctx->ev[1], ctx->ev[2]);
  phase_elapsed(&f3, ctx->ev[3], ctx->ev[4]);
  m.bitmap_ms = f1;
  m.bitmap_bytes = cs->bitmap_bytes;
  m.decode_ms = f2;
  decode_metrics(db, DecodeBatch(), &m, nullptr);
  m.aggregate_ms = f3;
  m.total_ms = ms_since(t0);
  ht.mark("done");
  if (metrics) *metrics = m;
  return DG_OK;
}

// ------------------------------------------------------------------------------------------------
// topN merge (TopNBinaryFn fold)
// ------------------------------------------------------------------------------------------------
}  // extern "C"

namespace dg {

// AggregatorFactory.combine on ABI-encoded values (Java semantics: long wrap, float adds in float,
// Math.min / Math.max with NaN propagation and -0.0 < 0.0)
template <class F>
static F java_min(F a, F b) {
  if (a != a) return a;
  if (a == 0 && b == 0 && std::signbit(b)) return b;
  return a <= b ? a : b;
}
template <class F>
static F java_max(F a, F b) {
  if (a != a) return a;
  if (a == 0 && b == 0 && std::signbit(a)) return b;
  return a >= b ? a : b;
}
static uint64_t combine_abi(int kind, uint64_t a, uint64_t b) {
  uint64_t out = 0;
  switch (kind) {
    case DG_AGG_COUNT:
    case DG_AGG_LONG_SUM: return (uint64_t)((int64_t)a + (int64_t)b);
    case DG_AGG_LONG_MIN: return (uint64_t)std::min((int64_t)a, (int64_t)b);
    case DG_AGG_LONG_MAX: return (uint64_t)std::max((int64_t)a, (int64_t)b);
    case DG_AGG_DOUBLE_SUM:
    case DG_AGG_DOUBLE_MIN:
    case DG_AGG_DOUBLE_MAX: {
      double x, y, r;
      memcpy(&x, &a, 8);
      memcpy(&y, &b, 8);
      r = kind == DG_AGG_DOUBLE_SUM ? x + y : kind == DG_AGG_DOUBLE_MIN ? java_min(x, y) : java_max(x, y);
      memcpy(&out, &r, 8);
      return out;
    }
    default: {
      float x, y, r;
      memcpy(&x, &a, 4);
      memcpy(&y, &b, 4);
      r = kind == DG_AGG_FLOAT_SUM ? x + y : kind == DG_AGG_FLOAT_MIN ? java_min(x, y) : java_max(x, y);
      memcpy(&out, &r, 4);
      return out;
    }
  }
}

// comparator key of an ABI-encoded metric value (Long.compare / Double.compare / Float.compare)
static uint64_t abi_metric_key(int kind, uint64_t v, int inverted) {
  uint64_t k;
  if (kind == DG_AGG_COUNT || kind == DG_AGG_LONG_SUM || kind == DG_AGG_LONG_MIN || kind == DG_AGG_LONG_MAX) {
    k = v ^ 0x8000000000000000ull;
  } else {
    double d;
    if (kind == DG_AGG_DOUBLE_SUM || kind == DG_AGG_DOUBLE_MIN || kind == DG_AGG_DOUBLE_MAX) {
      memcpy(&d, &v, 8);
    } else {
      float f;
      memcpy(&f, &v, 4);
      d = f;
    }
    if (d != d) {
      k = ~0ull;
    } else {
      uint64_t u;
      memcpy(&u, &d, 8);
      k = (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
    }
  }
  return inverted ? ~k : k;
}

}  // namespace dg

extern "C" {

int dg_topn_merge(dg_segment* const* segs, const dg_scan* q, const dg_topn* t, const dg_topn_lists* in, int32_t* out_n,
                  int32_t* out_list, int64_t* out_keys, uint64_t* out_values) {
  if (!q || !t || !in || !out_n || (in->n_lists > 0 && (!in->list_n || !in->keys || !in->values)))
    return set_error(DG_ERR_ARG, "null argument");
  AggPlan plan;
  int rc = make_plan(q, &plan);
  if (rc) return rc;
  if (t->metric_agg < 0 || t->metric_agg >= plan.n) return set_error(DG_ERR_ARG, "metric index");
  if (t->threshold <= 0) return set_error(DG_ERR_ARG, "threshold");
  const int na = plan.n, mk = plan.kind[t->metric_agg], nl = in->n_lists;
  // the dimension column of every list's segment, resolved once (segment mode)
  std::vector<const Column*> lcol(nl > 0 ? nl : 1, nullptr);
  if (segs) {
    const std::string dim = t->dimension ? t->dimension : "";
    for (int l = 0; l < nl; ++l) {
      const Column* c = reinterpret_cast<const Segment*>(segs[l])->find(dim);
      lcol[l] = (c && c->type == DG_COL_STRING) ? c : nullptr;
    }
  }
  struct Ent {
    int32_t list;
    int64_t key;
    uint64_t mkey;       // comparator key of the metric (Long/Double/Float.compare, inverted)
    uint64_t h;          // identity hash of the dimension value (see ident)
    const uint64_t* v;   // value slots: the caller's list row until combined, then a row of `vals`
  };
  int64_t total = 0;
  for (int l = 0; l < nl; ++l) total += std::max(in->list_n[l], 0);
  // rows of combined values (copy on first combine; at most one per entry)
  std::vector<uint64_t> vals((size_t)std::max<int64_t>(total, 1) * std::max(na, 1));
  size_t vo = 0;
  auto owned = [&](const uint64_t* v) { return v >= vals.data() && v < vals.data() + vals.size(); };
  // dimension value of an entry: (is null, bytes)
  auto value_of = [&](const Ent& e, std::string_view* sv) -> bool {
    const Column* c = lcol[e.list];
    if (!c || e.key < 0 || e.key >= (int64_t)c->dict.size() || c->dict_null[e.key]) return true;
    *sv = c->dict[e.key];
    return false;
  };
  auto dim_cmp = [&](const Ent& a, const Ent& b) -> int {
    if (!segs) return a.key < b.key ? -1 : (a.key > b.key ? 1 : 0);
    std::string_view sa, sb;
    const bool an = value_of(a, &sa), bn = value_of(b, &sb);
    if (an || bn) return an == bn ? 0 : (an ? -1 : 1);
    return java_compare(std::string(sa), std::string(sb));
  };
  // TopNNumericResultBuilder over `ents` (insertion order matters for ties at the minimum)
  std::vector<size_t> keep;
  auto build = [&](std::vector<Ent>& ents, int threshold) {
    auto less = [&](size_t a, size_t b) {
      if (ents[a].mkey != ents[b].mkey) return ents[a].mkey < ents[b].mkey;
      return dim_cmp(ents[a], ents[b]) < 0;
    };
    auto gt = [&](size_t a, size_t b) { return less(b, a); };
    std::vector<size_t> heap;
    heap.reserve(threshold + 1);
    for (size_t e = 0; e < ents.size(); ++e) {
      if ((int)heap.size() < threshold || ents[heap.front()].mkey < ents[e].mkey) {
        heap.push_back(e);
        std::push_heap(heap.begin(), heap.end(), gt);
      }
      if ((int)heap.size() > threshold) {
        std::pop_heap(heap.begin(), heap.end(), gt);
        heap.pop_back();
      }
    }
    keep.assign(heap.begin(), heap.end());
    std::sort(keep.begin(), keep.end(), [&](size_t a, size_t b) {
      if (ents[a].mkey != ents[b].mkey) return ents[a].mkey > ents[b].mkey;
      return dim_cmp(ents[a], ents[b]) < 0;
    });
    std::vector<Ent> out;
    out.reserve(keep.size());
    for (size_t k : keep) out.push_back(ents[k]);
    ents.swap(out);
  };
  // identity of a dimension value across segments (TopNBinaryFn keys results by value): the
  // attach-time value hash (segment mode) or the global id, in a flat open-addressing table; a hash
  // hit is confirmed on the bytes
  auto ident = [&](const Ent& e) -> uint64_t {
    if (!segs) return (uint64_t)e.key * 0x9e3779b97f4a7c15ull;
    const Column* c = lcol[e.list];
    if (!c || e.key < 0 || e.key >= (int64_t)c->dict.size()) return kNullValueHash;
    return c->dict_hash[e.key];
  };
  auto same = [&](const Ent& a, const Ent& b) -> bool {
    if (!segs) return a.key == b.key;
    std::string_view sa, sb;
    const bool an = value_of(a, &sa), bn = value_of(b, &sb);
    return an == bn && (an || sa == sb);
  };
  std::vector<int32_t> slot_of;
  std::vector<uint64_t> slot_hash;
  size_t tmask = 0;
  auto table_reset = [&](size_t n) {
    size_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    slot_of.assign(cap, -1);
    slot_hash.resize(cap);
    tmask = cap - 1;
  };
  std::vector<Ent> acc, cur;
  bool have = false;
  const int ma = t->metric_agg, inv = t->inverted;
  for (int l = 0; l < nl; ++l) {
    const int cnt = in->list_n[l];
    if (cnt < 0) continue;  // no cursor: no result from this segment
    cur.resize(cnt);
    const int64_t* ks = in->keys + (int64_t)l * in->stride;
    const uint64_t* vs = in->values + (int64_t)l * in->stride * na;
    for (int e = 0; e < cnt; ++e) {  // the entries reference the caller's rows (no copy)
      const uint64_t* v = vs + (int64_t)e * na;
      cur[e] = Ent{l, ks[e], abi_metric_key(mk, v[ma], inv), 0, v};
    }
    // the value hashes in a pass of their own: independent dictionary reads the core overlaps (one
    // random read per entry; interleaved with the table probes they were serialized)
    for (int e = 0; e < cnt; ++e) cur[e].h = ident(cur[e]);
    if (!have) {
      acc.swap(cur);
      have = true;
      continue;
    }
    // retVals (LinkedHashMap): r1's entries, then r2's new values; shared values combined in place
    table_reset(acc.size() + cur.size());
    auto find_or_insert = [&](const Ent& e, int32_t idx) -> int32_t {
      const uint64_t h = e.h;
      for (size_t q = h & tmask;; q = (q + 1) & tmask) {
        if (slot_of[q] < 0) {
          slot_of[q] = idx;
          slot_hash[q] = h;
          return -1;
        }
        if (slot_hash[q] == h && same(acc[slot_of[q]], e)) return slot_of[q];
      }
    };
    for (size_t e = 0; e < acc.size(); ++e) find_or_insert(acc[e], (int32_t)e);
    for (auto& e : cur) {
      const int32_t hit = find_or_insert(e, (int32_t)acc.size());
      if (hit >= 0) {
        Ent& a = acc[hit];
        if (!owned(a.v)) {
          memcpy(vals.data() + vo, a.v, 8 * (size_t)na);
          a.v = vals.data() + vo;
          vo += na;
        }
        uint64_t* w = const_cast<uint64_t*>(a.v);
        for (int k = 0; k < na; ++k) w[k] = combine_abi(plan.kind[k], w[k], e.v[k]);
        a.mkey = abi_metric_key(mk, w[ma], inv);
      } else {
        acc.push_back(e);
      }
    }
    build(acc, t->threshold);
  }
  const int nout = std::min<int>((int)acc.size(), t->threshold);
  *out_n = have ? nout : -1;
  for (int e = 0; e < nout; ++e) {
    if (out_list) out_list[e] = acc[e].list;
    if (out_keys) out_keys[e] = acc[e].key;
    if (out_values) memcpy(out_values + (size_t)e * na, acc[e].v, 8 * (size_t)na);
  }
  return DG_OK;
}

// ------------------------------------------------------------------------------------------------
// groupBy (v2): per-segment grouping + GroupByMergingQueryRunnerV2 merge, as one device-wide sort
// ------------------------------------------------------------------------------------------------
}  // extern "C"

namespace dg {

// Merged dictionary of `dim` over the call's segments: k-way merge of their sorted dictionaries
// (GenericIndexed STRING_STRATEGY = Java String.compareTo with nulls first), plus each segment's
// local id -> merged id table in HBM. A segment without the column contributes the null value.
static int merged_dict(Context* ctx, Segment* const* segs, int n, const std::string& dim, std::shared_ptr<MergedDict>* out) {
  std::vector<uint64_t> uids(n);
  for (int i = 0; i < n; ++i) uids[i] = segs[i]->uid;
  for (auto it = ctx->dict_cache.rbegin(); it != ctx->dict_cache.rend(); ++it)
    if ((*it)->dim == dim && (*it)->uids == uids) {
      *out = *it;
      return DG_OK;
    }
  auto md = std::make_shared<MergedDict>();
  md->uids = uids;
  md->dim = dim;
  md->remap.resize(n);
  std::vector<const Column*> cols(n, nullptr);
  bool need_null = false;
  for (int i = 0; i < n; ++i) {
    const Column* c = segs[i]->find(dim);
    if (c && c->type != DG_COL_STRING) return set_error(DG_ERR_UNSUPPORTED, "groupBy on non-string column %s", dim.c_str());
    cols[i] = c;
    need_null |= c == nullptr;
  }
  bool same = cols[0] != nullptr;
  for (int i = 1; i < n && same; ++i)
    same = cols[i] && (cols[i] == cols[0] || (cols[i]->dict == cols[0]->dict && cols[i]->dict_null == cols[0]->dict_null));
  if (same) {  // identical dictionaries (one segment, or segments of one generator): identity maps
    md->values = cols[0]->dict;
    md->is_null = cols[0]->dict_null;
  } else {
    if (need_null) {
      md->values.emplace_back();
      md->is_null.push_back(1);
    }
    struct Cur {
      int seg, pos;
    };
    auto entry_cmp = [&](const Cur& a, const Cur& b) {
      return cmp_nullable(cols[a.seg]->dict_null[a.pos], cols[a.seg]->dict[a.pos], cols[b.seg]->dict_null[b.pos],
                          cols[b.seg]->dict[b.pos]);
    };
    auto later = [&](const Cur& a, const Cur& b) {  // min-heap on (value, segment)
      const int c = entry_cmp(a, b);
      return c != 0 ? c > 0 : a.seg > b.seg;
    };
    std::priority_queue<Cur, std::vector<Cur>, decltype(later)> pq(later);
    std::vector<std::vector<int32_t>> host(n);
    for (int i = 0; i < n; ++i) {
      if (!cols[i] || cols[i]->dict.empty()) continue;
      host[i].resize(cols[i]->dict.size());
      pq.push(Cur{i, 0});
    }
    while (!pq.empty()) {
      Cur c = pq.top();
      pq.pop();
      const Column* col = cols[c.seg];
      const bool nul = col->dict_null[c.pos] != 0;
      const std::string& v = col->dict[c.pos];
      if (md->values.empty() || cmp_nullable(md->is_null.back() != 0, md->values.back(), nul, v) != 0) {
        md->values.push_back(nul ? std::string() : v);
        md->is_null.push_back(nul ? 1 : 0);
      }
      host[c.seg][c.pos] = (int32_t)md->values.size() - 1;
      if (++c.pos < (int)col->dict.size()) pq.push(c);
    }
    for (int i = 0; i < n; ++i) {
      if (host[i].empty()) continue;
      // a segment whose dictionary is the merged one keeps its ids: no table (no lookup per row)
      bool identity = true;
      for (size_t k = 0; identity && k < host[i].size(); ++k) identity = host[i][k] == (int32_t)k;
      if (identity) continue;
      md->remap[i].reset(new DevBuf());
      if (!md->remap[i]->alloc(host[i].size() * 4)) return set_error(DG_ERR_OOM, "hipMalloc dictionary map");
      DG_HIP(hipMemcpy(md->remap[i]->p, host[i].data(), host[i].size() * 4, hipMemcpyHostToDevice));
    }
  }
  md->null_gid = (!md->values.empty() && md->is_null[0]) ? 0 : -1;
  if (need_null && md->null_gid != 0) return set_error(DG_ERR_ARG, "merged dictionary of %s lacks null", dim.c_str());
  ctx->dict_cache.push_back(md);
  if (ctx->dict_cache.size() > 32) ctx->dict_cache.erase(ctx->dict_cache.begin());
  *out = md;
  return DG_OK;
}

// Result buffers outlive the call. They come from a per-context cache of device blocks: a released
// result's blocks are kept for the next result (every call ends with a stream synchronisation, so a
// cached block is idle) instead of a hipMalloc / hipFree (device-synchronising) per query.
static void* result_alloc(Context* ctx, size_t bytes) {
  bytes = (std::max<size_t>(bytes, 256) + 255) & ~(size_t)255;
  size_t best = (size_t)-1;
  for (size_t i = 0; i < ctx->free_blocks.size(); ++i) {
    const size_t sz = ctx->free_blocks[i].second;
    if (sz >= bytes && sz <= 2 * bytes + (64 << 20) && (best == (size_t)-1 || sz < ctx->free_blocks[best].second)) best = i;
  }
  if (best != (size_t)-1) {
    void* p = ctx->free_blocks[best].first;
    ctx->block_size[p] = ctx->free_blocks[best].second;
    ctx->free_blocks.erase(ctx->free_blocks.begin() + best);
    return p;
  }
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) {
    // give the cached blocks back and retry once
    for (auto& b : ctx->free_blocks) hipFree(b.first);
    ctx->free_blocks.clear();
    (void)hipGetLastError();
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  }
  ctx->block_size[p] = bytes;
  return p;
}

static void result_free(Context* ctx, void* p) {
  if (!p) return;
  auto it = ctx->block_size.find(p);
  if (it == ctx->block_size.end()) return;
  ctx->free_blocks.emplace_back(p, it->second);
  ctx->block_size.erase(it);
}

}  // namespace dg

struct dg_result {
  dg::Context* ctx = nullptr;
  int ndims = 0, naggs = 0;
  int64_t ngroups = 0;
  uint64_t* keys = nullptr;   // [ngroups] packed keys, ascending
  uint64_t* slots = nullptr;  // [1 + naggs][cap] (slot-major): rows, then the ABI-encoded aggregate values
  int64_t cap = 0;
  dg::KeyLayout lay{};
  int64_t bucket0 = 0, period = 0, universal = 0;
  std::vector<int64_t> bounds;  // calendar granularity: the call's bucket starts (bucket index -> time)
  std::vector<std::shared_ptr<dg::MergedDict>> dicts;  // empty for a dg_merge result (cluster ids)
  std::vector<int32_t> cards;                         // dg_merge result: cluster dictionary sizes
  bool limited = false;                               // dg_result_limit: groups in the push-down order
  std::vector<int32_t> kinds;                         // DG_AGG_* of every aggregator (combine semantics)
  ~dg_result() {
    if (!ctx) return;
    std::lock_guard<std::mutex> g(ctx->mu);
    hipSetDevice(ctx->device);
    dg::result_free(ctx, keys);
    dg::result_free(ctx, slots);
  }
};

// A result under construction inside a call, whose CallGuard holds the context's lock: on an error
// return its blocks go back to the cache here (~dg_result would take the lock again).
struct ResultDrop {
  void operator()(dg_result* r) const {
    if (!r) return;
    if (r->ctx) {
      dg::result_free(r->ctx, r->keys);
      dg::result_free(r->ctx, r->slots);
    }
    r->ctx = nullptr;
    delete r;
  }
};
using PendingResult = std::unique_ptr<dg_result, ResultDrop>;

extern "C" {

int dg_groupby_run(dg_segment* const* segs, int32_t n, const dg_scan* q, const dg_groupby* gb, dg_result** out,
                   dg_metrics* metrics) {
  auto t0 = std::chrono::steady_clock::now();
  HostTrace ht;
  Context* ctx;
  int rc = check_segments(segs, n, &ctx);
  if (rc) return rc;
  if (!q || !gb || !out) return set_error(DG_ERR_ARG, "null argument");
  dg_scan qs;
  Grain gr;
  rc = prepare_scan(q, &qs, &gr);
  if (rc) return rc;
  q = &qs;  // (groupBy cursors are always ascending: GroupByQueryEngineV2.java:108-115)
  const int nd = gb->n_dims;
  if (nd < 0 || nd > kMaxGroupDims) return set_error(DG_ERR_UNSUPPORTED, "%d groupBy dimensions (max %d)", nd, kMaxGroupDims);
  if (n > kMaxCallSegs) return set_error(DG_ERR_UNSUPPORTED, "%d segments in one call (max %d)", n, kMaxCallSegs);
  AggPlan plan;
  rc = make_plan(q, &plan);
  if (rc) return rc;
  CallGuard g(ctx);
  CallScratch* cs = g.cs;
  Interrupt intr(q, t0);
  cs->intr = &intr;
  hipStream_t st = ctx->stream;
  rc = upload_grain(cs, &gr, st);
  if (rc) return rc;
  dg_metrics m;
  memset(&m, 0, sizeof m);
  const int na = plan.n, rec = na + 1;
  std::vector<Segment*> sv(n);
  for (int i = 0; i < n; ++i) sv[i] = reinterpret_cast<Segment*>(segs[i]);
  std::vector<Cursors> cur(n);
  for (int i = 0; i < n; ++i) {
    cur[i] = plan_cursors(sv[i], i, q, gr);
    m.segment_rows += sv[i]->nrows;
  }
  // merged dictionaries (GroupByMergingQueryRunnerV2 merges by value; merged ids order like values)
  std::vector<std::shared_ptr<MergedDict>> md(nd);
  for (int d = 0; d < nd; ++d) {
    if (!gb->dimensions || !gb->dimensions[d]) return set_error(DG_ERR_ARG, "null dimension %d", d);
    rc = merged_dict(ctx, sv.data(), n, gb->dimensions[d], &md[d]);
    if (rc) return rc;
  }
  // buckets shared by the segments: one index origin (bucket starts are on one period grid)
  int64_t gb0 = 0, gend = 0;
  bool anyc = false;
  for (int i = 0; i < n; ++i) {
    if (!cur[i].any || !q->period_ms) continue;
    const int64_t b0 = cur[i].bucket0, e = b0 + cur[i].nbuckets * q->period_ms;
    gb0 = anyc ? std::min(gb0, b0) : b0;
    gend = anyc ? std::max(gend, e) : e;
    anyc = true;
  }
  // key = [bucket | d0 | d1 | ... ], the last dimension least significant
  KeyLayout lay{};
  lay.ndims = nd;
  int shift = 0;
  for (int d = nd - 1; d >= 0; --d) {
    lay.dim_shift[d] = shift;
    lay.dim_bits[d] = bits_for(std::max<int64_t>((int64_t)md[d]->values.size(), 1));
    shift += lay.dim_bits[d];
  }
  lay.bucket_shift = shift;
  lay.bucket_bits = (q->period_ms && anyc) ? bits_for((gend - gb0) / q->period_ms) : 0;
  const int key_bits = shift + lay.bucket_bits;
  if (key_bits > 64) return set_error(DG_ERR_UNSUPPORTED, "groupBy key of %d bits", key_bits);
  ht.mark("dicts");
  phase_event(ctx->ev[0], st);
  std::vector<GbJob> gj(n);
  std::vector<int64_t> rows(n, 0);
  // one element per row unless a grouping dimension is multi-value: then the payload is indexed by
  // the row (row-ref mode) and sized before the decodes, so plain LZ4 value columns decode straight
  // into it (payload_view)
  bool any_multi = false;
  int64_t row_total = 0;
  int ntiles_rows = 0;
  std::vector<uint32_t> row_base(n, 0);
  for (int i = 0; i < n; ++i) {
    if (!cur[i].any) continue;
    for (int d = 0; d < nd; ++d) {
      const Column* c = sv[i]->find(gb->dimensions[d]);
      any_multi |= c && c->multi_value;
    }
    row_base[i] = (uint32_t)row_total;
    row_total += sv[i]->nrows;
    ntiles_rows += (int)((sv[i]->nrows + kTileRows - 1) / kTileRows);
  }
  if (row_total >= (1ll << 32)) return set_error(DG_ERR_UNSUPPORTED, "%lld rows in one call (row refs are 32-bit)", (long long)row_total);
  SortBufs sb;
  if (!any_multi) {
    rc = sort_bufs(cs, row_total, std::max(ntiles_rows, 1), key_bits, na, &sb);
    if (rc) return rc;
    sb.row_refs = 1;
  }
  std::vector<const unsigned long long*> counts(n, nullptr);
  DecodeBatch db, db_side;  // db_side: payload columns decoded in place (side stream)
  decode_events(ctx, &db, false);
  decode_events(ctx, &db_side, true);
  for (int i = 0; i < n; ++i) {
    GbJob& j = gj[i];
    memset(&j, 0, sizeof j);
    if (!cur[i].any) continue;
    Segment* seg = sv[i];
    uint32_t* bits = nullptr;
    rc = build_bitset(seg, cs, q->filter, q->n_filter, &bits, &counts[i], st);
    if (rc) return rc;
    j.bitset = bits;
    j.time.kind = VIEW_ABSENT;
    if (cur[i].need_time) {
      rc = time_view(seg->find("__time"), time_block_buckets(seg, seg->find("__time"), cur[i], q->period_ms, gr), cs, &db, &j.time, st);
      if (rc) return rc;
    }
    j.t_lo = cur[i].t_lo;
    j.t_hi = cur[i].t_hi;
    j.bucket0 = gb0;
    j.period = q->period_ms;
    j.bounds = gr.db;
    j.nbounds = gr.nb + 1;
    j.bucket_shift = lay.bucket_shift;
    j.bucket_bits = lay.bucket_bits;
    j.ndims = nd;
    for (int d = 0; d < nd; ++d) {
      Column* c = seg->find(gb->dimensions[d]);
      if (c && c->multi_value) {  // row value lists: every row groups under each of its values
        rc = multi_view(c, cs, &db, &j.dims[d], &j.moff[d], st);
        if (rc) return rc;
        j.multi = 1;
        j.remap[d] = md[d]->remap[i] ? md[d]->remap[i]->as<int32_t>() : nullptr;
      } else if (c) {
        rc = column_view(c, cs, &db, &j.dims[d], st);
        if (rc) return rc;
        j.remap[d] = md[d]->remap[i] ? md[d]->remap[i]->as<int32_t>() : nullptr;
      } else {
        j.dims[d].kind = VIEW_ABSENT;
      }
      j.null_gid[d] = std::max(md[d]->null_gid, 0);
      j.dim_shift[d] = lay.dim_shift[d];
      j.dim_bits[d] = lay.dim_bits[d];
    }
    for (int a = 0; a < na; ++a) {
      const Column* ac = q->aggs[a].field ? seg->find(q->aggs[a].field) : nullptr;
      if (!any_multi && ac && !(q->aggs[a].filter && q->aggs[a].n_filter > 0) &&
          payload_view(ac, q->aggs[a].kind, sb.payload, na, a, row_base[i], &db_side)) {
        j.inplace |= 1u << a;
        j.vals[a].kind = VIEW_ABSENT;
        continue;
      }
      rc = agg_view(seg, q->aggs[a], cs, &db, &j.vals[a], &j.agg_bits[a], st);
      if (rc) return rc;
    }
    rows[i] = seg->nrows;
  }
  ht.mark("views");
  DG_CHECK_INTERRUPT(intr);
  // The payload columns only meet the keys at the reduce: they decode on the side stream while the
  // main stream decodes the key columns, builds the keys and sorts them (the general LZ4 decoder is
  // LDS / latency bound, the sort HBM bound, so the two overlap on the CUs).
  SideJoin side_join;
  const bool no_side = env_on("DG_NO_SIDE");  // everything on the main stream (same-box A/B and tests)
  bool side_work = !db_side.jobs.empty();
  for (const auto& t : db_side.tasks) side_work |= !t.empty();
  const bool side = ctx->side && side_work && !no_side;
  if (side) {
    if (!call_err(cs, st)) return set_error(DG_ERR_OOM, "error word");
    DG_FLUSH(cs, st);  // everything staged so far leaves on the main stream first
    // side_ev[0] (side waits for the flush and the zeroed error word) and side_ev[2] (the reduce waits
    // for the payload) order the streams: recorded on every call, phase timing or not
    DG_HIP(hipEventRecord(ctx->side_ev[0], st));
    DG_HIP(hipStreamWaitEvent(ctx->side, ctx->side_ev[0], 0));
    side_join.s = ctx->side;
    phase_event(ctx->side_ev[1], ctx->side);
    rc = run_decodes_only(cs, &db_side, ctx->side, nullptr);
    if (rc) return rc;
    DG_HIP(hipEventRecord(ctx->side_ev[2], ctx->side));
  } else {
    db.jobs.insert(db.jobs.end(), db_side.jobs.begin(), db_side.jobs.end());
    for (int kd = 0; kd < kKinds; ++kd) {
      db.tasks[kd].insert(db.tasks[kd].end(), db_side.tasks[kd].begin(), db_side.tasks[kd].end());
      db.task_bytes[kd] += db_side.task_bytes[kd];
    }
    db.bytes += db_side.bytes;
    db_side.bytes = 0;
  }
  ht.mark("side_launched");
  phase_event(ctx->ev[1], st);
  rc = run_decodes(cs, &db, st);
  if (rc) return rc;
  phase_event(ctx->ev[2], st);
  ht.mark("main_decode_launched");
  DG_CHECK_INTERRUPT(intr);
  m.bytes_read = db.bytes + db_side.bytes;
  m.bytes_side = db_side.bytes;
  GbJob* d_jobs;
  int32_t* d_tile;
  int ntiles = 0;
  int64_t total = 0;
  rc = upload_gb_jobs(cs, gj, rows, &d_jobs, &d_tile, &ntiles, &total, st);
  if (rc) return rc;
  if (any_multi) {  // rows explode into one element per grouping: count them first to size the sort
    rc = count_elements(cs, d_jobs, d_tile, ntiles, &total, st);
    if (rc) return rc;
    rc = sort_bufs(cs, total, ntiles, key_bits, na, &sb);
    if (rc) return rc;
  }
  uint32_t* h_n = host_take<uint32_t>(cs, 4);
  if (!h_n) return set_error(DG_ERR_OOM, "groupBy counters");
  DG_FLUSH(cs, st);
  phase_event(ctx->ev[3], st);
  // every row an element (no filter, no multi-value dimension, every row's time inside the cursor's
  // interval — no time view, or the attach-time block bounds of __time inside it — and no floatSum
  // pass, which reads the per-tile counts): the keygen needs no count pass (DG_GB_COUNT=1: count anyway)
  auto all_rows_in = [&](int i) {
    if (gj[i].bitset || gj[i].multi) return false;
    if (gj[i].time.kind == VIEW_ABSENT) return true;
    const Column* tc = sv[i]->find("__time");
    if (!tc || !tc->data.time_col || tc->data.nblocks <= 0 || tc->data.min8.size() != (size_t)tc->data.nblocks ||
        tc->data.max8.size() != (size_t)tc->data.nblocks)
      return false;
    const int64_t lo = *std::min_element(tc->data.min8.begin(), tc->data.min8.end());
    const int64_t hi = *std::max_element(tc->data.max8.begin(), tc->data.max8.end());
    return lo >= gj[i].t_lo && hi < gj[i].t_hi;
  };
  bool rows_elems = !any_multi && !has_float_sum(plan) && !env_on("DG_GB_COUNT");
  for (int i = 0; i < n && rows_elems; ++i) rows_elems = !cur[i].any || all_rows_in(i);
  launch_gb_keygen(d_jobs, d_tile, ntiles, &sb, plan, st, any_multi, rows_elems ? total : -1);
  phase_event(ctx->ev[5], st);
  launch_radix_sort(&sb, key_bits, st);
  phase_event(ctx->ev[6], st);
  DG_CHECK_INTERRUPT(intr);
  // the result is laid out for the sort's capacity (>= the groups): the reduce counts the groups itself
  // (look-back over tiles), so there is no host read-back between the sort and the reduce
  const int64_t cap = std::max<int64_t>(sb.cap, 1);
  PendingResult res(new dg_result());
  res->ctx = ctx;
  res->ndims = nd;
  res->naggs = na;
  res->lay = lay;
  res->bucket0 = gb0;
  res->period = q->period_ms;
  if (gr.hb) res->bounds.assign(gr.hb, gr.hb + gr.nb + 1);
  res->universal = q->interval_start;  // GroupByStrategyV2.getUniversalTimestamp (ALL granularity)
  res->kinds.assign(plan.kind, plan.kind + na);
  res->dicts = md;
  res->keys = static_cast<uint64_t*>(result_alloc(ctx, (size_t)cap * 8));
  res->slots = static_cast<uint64_t*>(result_alloc(ctx, (size_t)cap * rec * 8));
  res->cap = cap;
  if (!res->keys || !res->slots) return set_error(DG_ERR_OOM, "groupBy result of %lld records", (long long)cap);
  bool reduce_timed = false;
  {
    // run heads are only needed by the floatSum row-order pass
    uint32_t* head_pos = has_float_sum(plan) ? dev_take<uint32_t>(cs, (size_t)cap + 16) : nullptr;
    const size_t nt = (size_t)sb.ntiles_sort;  // one carry / open group per tile
    int64_t* carry_g = dev_take<int64_t>(cs, (size_t)kRedWaves * nt);  // one carry / open slot per wave share of a tile
    int64_t* open_g = dev_take<int64_t>(cs, (size_t)kRedWaves * nt);
    uint64_t* carry_slots = dev_take<uint64_t>(cs, (size_t)kRedWaves * nt * rec);
    if ((has_float_sum(plan) && !head_pos) || !carry_g || !open_g || !carry_slots)
      return set_error(DG_ERR_OOM, "groupBy reduce scratch");
    if (side) DG_HIP(hipStreamWaitEvent(st, ctx->side_ev[2], 0));  // the payload is decoded
    phase_event(ctx->ev[7], st);
    reduce_timed = true;
    launch_gb_reduce(&sb, plan, res->keys, res->slots, cap, head_pos, carry_g, carry_slots, open_g, st);
    for (int a = 0; a < na; ++a)
      if (plan.kind[a] == DG_AGG_FLOAT_SUM) launch_fsum_runs(d_jobs, n, ntiles, &sb, plan, a, head_pos, res->slots, cap, st);
  }
  phase_event(ctx->ev[4], st);
  DG_HIP(hipMemcpyAsync(h_n, sb.n, 8, hipMemcpyDeviceToHost, st));  // selected rows, groups
  ht.mark("reduce_launched");
  rc = finish_call(cs, st);  // (polls the cancel flag / timeout while the device works)
  if (rc) return rc;
  ht.mark("synced");
  const int64_t nsel = h_n[0], ng = h_n[1];
  res->ngroups = ng;
  // The result was laid out for the call's rows; when the groups are far fewer (filtered or few-group
  // queries) it is compacted to them and the row-sized blocks go back to the context's cache.
  if (ng * 2 < cap && (size_t)cap * rec * 8 >= ((size_t)1 << 20)) {
    const int64_t c2 = std::max<int64_t>(ng, 1);
    uint64_t* k2 = static_cast<uint64_t*>(result_alloc(ctx, (size_t)c2 * 8));
    uint64_t* s2 = static_cast<uint64_t*>(result_alloc(ctx, (size_t)c2 * rec * 8));
    if (k2 && s2) {
      if (ng > 0) {  // (one copy kernel: the runtime's 2-D copy moved these at ≈ 0.8 TB/s)
        launch_result_compact(res->keys, res->slots, cap, ng, rec, k2, s2, st);
        DG_HIP(hipStreamSynchronize(st));
        DG_HIP(hipGetLastError());
      }
      result_free(ctx, res->keys);
      result_free(ctx, res->slots);
      res->keys = k2;
      res->slots = s2;
      res->cap = c2;
    } else {  // no room for the compact copy: keep the row-sized result
      result_free(ctx, k2);
      result_free(ctx, s2);
    }
  }
  if (side) {
    float fs = 0;
    phase_elapsed(&fs, ctx->side_ev[1], ctx->side_ev[2]);
    m.decode_side_ms = fs;
  }
  for (int i = 0; i < n; ++i)
    if (cur[i].any) m.pre_filtered_rows += counts[i] ? (int64_t)*counts[i] : sv[i]->nrows;
  m.selected_rows = nsel;
  float f1 = 0, f2 = 0, f3 = 0, f4 = 0, f5 = 0, f6 = 0;
  phase_elapsed(&f1, ctx->ev[0], ctx->ev[1]);
  phase_elapsed(&f2, ctx->ev[1], ctx->ev[2]);
  phase_elapsed(&f3, ctx->ev[3], ctx->ev[4]);
  phase_elapsed(&f4, ctx->ev[3], ctx->ev[5]);
  phase_elapsed(&f5, ctx->ev[5], ctx->ev[6]);
  phase_elapsed(&f6, ctx->ev[6], ctx->ev[4]);
  m.bitmap_ms = f1;
  m.bitmap_bytes = cs->bitmap_bytes;
  m.decode_ms = f2;
  decode_metrics(db, db_side, &m, ctx->ev[0]);
  m.aggregate_ms = f3;
  m.keygen_ms = f4;
  m.sort_ms = f5;
  m.reduce_ms = f6;  // includes the wait for the side-stream payload decode
  if (reduce_timed) {
    float fr = 0;
    phase_elapsed(&fr, ctx->ev[7], ctx->ev[4]);
    m.reduce_kernel_ms = fr;
  }
  m.sort_passes = key_bits > 0 ? (key_bits + 7) / 8 : 0;
  m.key_bits = key_bits;
  m.groups = ng;
  m.total_ms = ms_since(t0);
  if (metrics) *metrics = m;
  *out = res.release();
  return DG_OK;
}

int64_t dg_result_groups(const dg_result* r) { return r ? r->ngroups : -1; }

int dg_result_fetch_groups(dg_result* r, int64_t start, int64_t count, int64_t* bucket_time, int32_t* ids,
                           uint64_t* values) {
  if (!r || start < 0 || count < 0 || start + count > r->ngroups) return set_error(DG_ERR_ARG, "bad result range");
  if (count == 0) return DG_OK;
  CallGuard g(r->ctx);
  CallScratch* cs = g.cs;
  hipStream_t st = r->ctx->stream;
  const int nd = r->ndims, na = r->naggs;
  // per group: time 8 B, ids 4 B each, values 8 B each, packed on the device and copied through two
  // pinned staging chunks; the host copies chunk i into the caller's arrays (several threads) while
  // chunk i + 1 crosses PCIe. Pinned destinations take each chunk's columns by DMA instead.
  const int64_t per = (bucket_time ? 8 : 0) + (ids ? 4 * (int64_t)nd : 0) + (values ? 8 * (int64_t)na : 0);
  if (per == 0) return DG_OK;
  auto pinned = [](const void* p) {
    if (!p) return true;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return a.type == hipMemoryTypeHost;
  };
  // pinned destinations the device can address: the pack kernel writes the columns straight into them
  // over PCIe (posted writes from every CU; no staging, no DMA copy). DG_FETCH_ZC=0: the staged DMA path.
  auto dev_ptr = [](void* h) -> void* {
    if (!h) return nullptr;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    return d;
  };
  const bool zc_off = [] {  // (same-box A/B and tests)
    const char* v = getenv("DG_FETCH_ZC");
    return v && *v == '0';
  }();
  if (!zc_off && pinned(bucket_time) && pinned(ids) && pinned(values)) {
    int64_t* dt = static_cast<int64_t*>(dev_ptr(bucket_time));
    int32_t* di = static_cast<int32_t*>(dev_ptr(ids));
    uint64_t* dv = static_cast<uint64_t*>(dev_ptr(values));
    if ((!bucket_time || dt) && (!ids || di) && (!values || dv)) {
      const int64_t* d_bounds = nullptr;
      if (r->period && !r->bounds.empty()) {
        int64_t* db;
        int64_t* hb = up_take<int64_t>(cs, r->bounds.size(), &db, st);
        if (!hb) return set_error(DG_ERR_OOM, "bucket table");
        memcpy(hb, r->bounds.data(), r->bounds.size() * 8);
        d_bounds = db;
      }
      DG_FLUSH(cs, st);
      launch_gb_fetch_pack(r->keys, r->slots, r->cap, start, count, r->lay, na, r->universal, r->bucket0, r->period, d_bounds,
                           dt, nd ? di : nullptr, na ? dv : nullptr, st);
      return finish_call(cs, st);
    }
  }
  if (pinned(bucket_time) && pinned(ids) && pinned(values)) {
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(count, ((int64_t)256 << 20) / per));
    uint8_t* d_stage = dev_take<uint8_t>(cs, (size_t)(chunk * per + 64));
    if (!d_stage) return set_error(DG_ERR_OOM, "fetch staging");
    const int64_t* d_bounds = nullptr;
    if (r->period && !r->bounds.empty()) {
      int64_t* db;
      int64_t* hb = up_take<int64_t>(cs, r->bounds.size(), &db, st);
      if (!hb) return set_error(DG_ERR_OOM, "bucket table");
      memcpy(hb, r->bounds.data(), r->bounds.size() * 8);
      d_bounds = db;
    }
    DG_FLUSH(cs, st);
    for (int64_t c0 = start; c0 < start + count; c0 += chunk) {
      const int64_t n = std::min<int64_t>(chunk, start + count - c0);
      uint8_t* p = d_stage;
      int64_t* t = bucket_time ? reinterpret_cast<int64_t*>(p) : nullptr;
      p += bucket_time ? 8 * n : 0;
      uint64_t* v = values && na ? reinterpret_cast<uint64_t*>(p) : nullptr;
      p += v ? 8 * n * na : 0;
      int32_t* i = ids && nd ? reinterpret_cast<int32_t*>(p) : nullptr;
      launch_gb_fetch_pack(r->keys, r->slots, r->cap, c0, n, r->lay, na, r->universal, r->bucket0, r->period, d_bounds, t,
                           i, v, st);
      const int64_t o = c0 - start;
      if (t) DG_HIP(hipMemcpyAsync(bucket_time + o, t, (size_t)n * 8, hipMemcpyDeviceToHost, st));
      if (v) DG_HIP(hipMemcpyAsync(values + o * na, v, (size_t)(n * na) * 8, hipMemcpyDeviceToHost, st));
      if (i) DG_HIP(hipMemcpyAsync(ids + o * nd, i, (size_t)(n * nd) * 4, hipMemcpyDeviceToHost, st));
    }
    return finish_call(cs, st);
  }
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(count, ((int64_t)64 << 20) / per));
  const size_t cbytes = (size_t)(chunk * per + 64);
  uint8_t* d_stage = dev_take<uint8_t>(cs, cbytes);
  uint8_t* h_stage[2] = {host_take<uint8_t>(cs, cbytes), host_take<uint8_t>(cs, cbytes)};
  if (!d_stage || !h_stage[0] || !h_stage[1]) return set_error(DG_ERR_OOM, "fetch staging");
  const int64_t* d_bounds = nullptr;
  if (r->period && !r->bounds.empty()) {
    int64_t* db;
    int64_t* hb = up_take<int64_t>(cs, r->bounds.size(), &db, st);
    if (!hb) return set_error(DG_ERR_OOM, "bucket table");
    memcpy(hb, r->bounds.data(), r->bounds.size() * 8);
    d_bounds = db;
  }
  DG_FLUSH(cs, st);
  hipEvent_t done[2] = {r->ctx->ev[6], r->ctx->ev[7]};
  auto layout = [&](uint8_t* base, int64_t n, int64_t** t, int32_t** i, uint64_t** v) {
    uint8_t* p = base;
    *t = bucket_time ? reinterpret_cast<int64_t*>(p) : nullptr;
    p += bucket_time ? 8 * n : 0;
    *v = values ? reinterpret_cast<uint64_t*>(p) : nullptr;
    p += values ? 8 * n * na : 0;
    *i = ids ? reinterpret_cast<int32_t*>(p) : nullptr;
  };
  auto drain = [&](int k, int64_t c0, int64_t n) {  // chunk in h_stage[k] -> the caller's arrays
    int64_t* t;
    int32_t* i;
    uint64_t* v;
    layout(h_stage[k], n, &t, &i, &v);
    std::vector<std::pair<void*, std::pair<const void*, size_t>>> parts;
    if (t) parts.push_back({bucket_time + (c0 - start), {t, (size_t)n * 8}});
    if (v && na) parts.push_back({values + (c0 - start) * na, {v, (size_t)n * na * 8}});
    if (i && nd) parts.push_back({ids + (c0 - start) * nd, {i, (size_t)n * nd * 4}});
    par_copy(parts);
  };
  int64_t prev0 = -1, prevn = 0;
  int k = 0;
  for (int64_t c0 = start; c0 < start + count; c0 += chunk, k ^= 1) {
    const int64_t n = std::min<int64_t>(chunk, start + count - c0);
    int64_t* t;
    int32_t* i;
    uint64_t* v;
    layout(d_stage, n, &t, &i, &v);
    launch_gb_fetch_pack(r->keys, r->slots, r->cap, c0, n, r->lay, na, r->universal, r->bucket0, r->period, d_bounds, t,
                         nd ? i : nullptr, na ? v : nullptr, st);
    DG_HIP(hipMemcpyAsync(h_stage[k], d_stage, (size_t)(n * per), hipMemcpyDeviceToHost, st));
    DG_HIP(hipEventRecord(done[k], st));
    if (prev0 >= 0) {
      DG_HIP(hipEventSynchronize(done[k ^ 1]));
      drain(k ^ 1, prev0, prevn);
    }
    prev0 = c0;
    prevn = n;
  }
  DG_HIP(hipEventSynchronize(done[k ^ 1]));
  drain(k ^ 1, prev0, prevn);
  return finish_call(cs, st);
}

int dg_host_alloc(int64_t bytes, void** out) {
  if (!out || bytes < 0) return set_error(DG_ERR_ARG, "bad arguments");
  *out = nullptr;
  if (hipHostMalloc(out, (size_t)std::max<int64_t>(bytes, 64), hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return set_error(DG_ERR_OOM, "hipHostMalloc %lld", (long long)bytes);
  }
  return DG_OK;
}

void dg_host_free(void* p) {
  if (p) hipHostFree(p);
}

int dg_result_fetch_rows(dg_result* r, int64_t start, int64_t count, int64_t* rows) {
  if (!r || !rows || start < 0 || count < 0 || start + count > r->ngroups) return set_error(DG_ERR_ARG, "bad result range");
  if (count == 0) return DG_OK;
  CallGuard g(r->ctx);
  DG_HIP(hipMemcpyAsync(rows, r->slots + start, (size_t)count * 8, hipMemcpyDeviceToHost, r->ctx->stream));
  return finish_call(g.cs, r->ctx->stream);
}

int dg_result_dim_dictionary(const dg_result* r, int32_t dim, int64_t* offsets, char* bytes, int64_t* total) {
  if (!r || dim < 0 || dim >= r->ndims) return set_error(DG_ERR_ARG, "dimension index %d", dim);
  if (r->dicts.empty()) return set_error(DG_ERR_ARG, "a merged result's dictionary is the caller's cluster dictionary");
  const MergedDict& d = *r->dicts[dim];
  int64_t t = 0;
  for (size_t i = 0; i < d.values.size(); ++i) {
    if (offsets) offsets[i] = t;
    if (bytes && !d.is_null[i]) memcpy(bytes + t, d.values[i].data(), d.values[i].size());
    t += d.is_null[i] ? 0 : (int64_t)d.values[i].size();
  }
  if (offsets) offsets[d.values.size()] = t;
  if (total) *total = t;
  return DG_OK;
}

int dg_result_limit(dg_result* r, const dg_limit* spec) {
  if (!r || !spec || spec->limit <= 0 || spec->n_columns < 0 || (spec->n_columns > 0 && !spec->columns))
    return set_error(DG_ERR_ARG, "bad limit spec");
  Context* ctx = r->ctx;
  const KeyLayout& lay = r->lay;
  // the push-down field order: time, ORDER BY dimensions (first mention), the other dimensions
  // ascending; time last with sortByDimsFirst
  LimitOrder o;
  memset(&o, 0, sizeof o);
  std::vector<int> field_dim;  // -1 = bucket
  const bool time_last = spec->sort_by_dims_first != 0;
  if (lay.bucket_bits && !time_last) field_dim.push_back(-1);
  std::vector<int> desc(r->ndims, 0);
  std::vector<const int32_t*> rank(r->ndims, nullptr);
  std::vector<bool> used(r->ndims, false);
  for (int c = 0; c < spec->n_columns; ++c) {
    const dg_order_column& oc = spec->columns[c];
    if (oc.dim < 0 || oc.dim >= r->ndims) return set_error(DG_ERR_ARG, "ORDER BY dimension %d of %d", oc.dim, r->ndims);
    if (used[oc.dim]) continue;  // a later mention never decides (the first already compared equal)
    used[oc.dim] = true;
    desc[oc.dim] = oc.descending != 0;
    rank[oc.dim] = oc.rank;
    field_dim.push_back(oc.dim);
  }
  for (int d = 0; d < r->ndims; ++d)
    if (!used[d]) field_dim.push_back(d);
  if (lay.bucket_bits && time_last) field_dim.push_back(-1);
  int key_bits = 0;
  for (int f : field_dim) key_bits += f < 0 ? lay.bucket_bits : lay.dim_bits[f];
  CallGuard g(ctx);
  CallScratch* cs = g.cs;
  hipStream_t st = ctx->stream;
  int out = key_bits;
  for (size_t f = 0; f < field_dim.size(); ++f) {
    const int d = field_dim[f];
    o.bits[o.nfields] = d < 0 ? lay.bucket_bits : lay.dim_bits[d];
    o.in_shift[o.nfields] = d < 0 ? lay.bucket_shift : lay.dim_shift[d];
    out -= o.bits[o.nfields];
    o.out_shift[o.nfields] = out;
    if (d >= 0) {
      o.desc[o.nfields] = desc[d];
      if (rank[d]) {  // caller's comparator ranks over the result's dictionary ids, checked and uploaded
        const int32_t card = dg_result_dim_cardinality(r, d);
        const int64_t top = o.bits[o.nfields] >= 31 ? INT32_MAX : (1ll << o.bits[o.nfields]);
        for (int32_t i = 0; i < card; ++i)
          if (rank[d][i] < 0 || rank[d][i] >= card || rank[d][i] >= top)
            return set_error(DG_ERR_ARG, "rank %d of id %d of dimension %d outside [0, %d)", rank[d][i], i, d, card);
        int32_t* dr;
        int32_t* h = up_take<int32_t>(cs, (size_t)std::max(card, 1), &dr, st);
        if (!h) return set_error(DG_ERR_OOM, "rank table");
        memcpy(h, rank[d], sizeof(int32_t) * (size_t)card);
        o.rank[o.nfields] = dr;
      }
    }
    if (o.bits[o.nfields] > 0) o.nfields++;
  }
  const int64_t n = r->ngroups;
  const int64_t m = std::min<int64_t>(spec->limit, n);
  // the push-down order is the result's own key order (no ORDER BY beyond an ascending LEXICOGRAPHIC
  // prefix of the dimensions, time first): the first `limit` groups already are the answer
  bool natural = true;
  for (int f = 0, d = 0; f < (int)field_dim.size(); ++f) {
    if (field_dim[f] < 0) {
      natural &= f == 0;
      continue;
    }
    natural &= field_dim[f] == d++ && !desc[field_dim[f]] && !rank[field_dim[f]];
  }
  if (n == 0 || natural) {
    r->ngroups = m;
    r->limited = true;
    return DG_OK;
  }
  SortBufs sb;
  int rc = sort_bufs(cs, n, 1, key_bits, 0, &sb);
  if (rc) return rc;
  const int rec = r->naggs + 1;
  DG_FLUSH(cs, st);
  uint64_t* nk = static_cast<uint64_t*>(result_alloc(ctx, (size_t)m * 8));
  uint64_t* ns = static_cast<uint64_t*>(result_alloc(ctx, (size_t)m * rec * 8));
  if (!nk || !ns) {
    result_free(ctx, nk);
    result_free(ctx, ns);
    return set_error(DG_ERR_OOM, "limited result of %lld groups", (long long)m);
  }
  launch_limit_load(r->keys, n, o, &sb, st);
  launch_radix_sort(&sb, key_bits, st);
  launch_limit_gather(&sb, m, r->keys, r->slots, r->cap, rec, nk, ns, m, st);
  rc = finish_call(cs, st);
  if (rc) {
    result_free(ctx, nk);
    result_free(ctx, ns);
    return rc;
  }
  result_free(ctx, r->keys);
  result_free(ctx, r->slots);
  r->keys = nk;
  r->slots = ns;
  r->cap = m;
  r->ngroups = m;
  r->limited = true;
  return DG_OK;
}

int32_t dg_result_dim_cardinality(const dg_result* r, int32_t dim) {
  if (!r || dim < 0 || dim >= r->ndims) return -1;
  if (r->dicts.empty()) return r->cards[dim];
  return (int32_t)r->dicts[dim]->values.size();
}

void dg_result_release(dg_result* r) { delete r; }

// ---- BufferAggregator records ----
int dg_records_pack(const uint64_t* slots, int64_t n, const dg_record_layout* lay, void* out) {
  if (n < 0 || !lay || (n > 0 && (!slots || !out)) || lay->n_aggs < 0 || (lay->n_aggs && (!lay->kinds || !lay->offsets)))
    return set_error(DG_ERR_ARG, "bad record layout");
  const int na = lay->n_aggs;
  for (int a = 0; a < na; ++a) {
    const int k = lay->kinds[a];
    if (k < DG_AGG_COUNT || k > DG_AGG_FLOAT_MAX) return set_error(DG_ERR_ARG, "aggregator kind %d", k);
    const int w = (k == DG_AGG_FLOAT_SUM || k == DG_AGG_FLOAT_MIN || k == DG_AGG_FLOAT_MAX) ? 4 : 8;
    if (lay->offsets[a] < 0 || lay->offsets[a] + w > lay->record_size)
      return set_error(DG_ERR_ARG, "aggregator %d at offset %d does not fit a %d-byte record", a, lay->offsets[a], lay->record_size);
  }
  uint8_t* o = static_cast<uint8_t*>(out);
  for (int64_t i = 0; i < n; ++i) {
    uint8_t* rec = o + i * (int64_t)lay->record_size;
    for (int a = 0; a < na; ++a) {
      const int k = lay->kinds[a];
      const uint64_t v = slots[i * na + a];
      uint8_t* p = rec + lay->offsets[a];
      if (k == DG_AGG_FLOAT_SUM || k == DG_AGG_FLOAT_MIN || k == DG_AGG_FLOAT_MAX) {
        const uint32_t f = (uint32_t)v;  // the float's bits ride in the slot's low 4 bytes
        for (int b = 0; b < 4; ++b) p[b] = (uint8_t)(f >> (8 * (lay->big_endian ? 3 - b : b)));
      } else {
        for (int b = 0; b < 8; ++b) p[b] = (uint8_t)(v >> (8 * (lay->big_endian ? 7 - b : b)));
      }
    }
  }
  return DG_OK;
}

// ---- cross-device merge ----
static int keyspace_layout(const dg_keyspace* ks, KeyLayout* lay, AggPlan* plan) {
  if (!ks || ks->n_dims < 0 || ks->n_dims > kMaxGroupDims || (ks->n_dims && !ks->card))
    return set_error(DG_ERR_ARG, "bad key space");
  if (ks->n_aggs < 0 || ks->n_aggs > kMaxAggs || (ks->n_aggs && !ks->agg_kinds)) return set_error(DG_ERR_ARG, "bad key space aggregators");
  memset(lay, 0, sizeof *lay);
  lay->ndims = ks->n_dims;
  int shift = 0;
  for (int d = ks->n_dims - 1; d >= 0; --d) {
    if (ks->card[d] < 0) return set_error(DG_ERR_ARG, "cardinality of dimension %d", d);
    lay->dim_shift[d] = shift;
    lay->dim_bits[d] = bits_for(std::max<int64_t>(ks->card[d], 1));
    shift += lay->dim_bits[d];
  }
  lay->bucket_shift = shift;
  if (ks->period_ms < 0 || (ks->period_ms && ks->n_buckets <= 0)) return set_error(DG_ERR_ARG, "bad key space buckets");
  lay->bucket_bits = ks->period_ms ? bits_for(ks->n_buckets) : 0;
  if (shift + lay->bucket_bits > 64) return set_error(DG_ERR_UNSUPPORTED, "cluster groupBy key of %d bits", shift + lay->bucket_bits);
  if (plan) {
    memset(plan, 0, sizeof *plan);
    plan->n = ks->n_aggs;
    for (int a = 0; a < ks->n_aggs; ++a) {
      const int k = ks->agg_kinds[a];
      if (k < DG_AGG_COUNT || k > DG_AGG_FLOAT_MAX) return set_error(DG_ERR_ARG, "aggregator kind %d", k);
      plan->kind[a] = k;
      plan->op[a] = slot_op(k);
    }
  }
  return DG_OK;
}

int dg_keyspace_bits(const dg_keyspace* ks, int32_t* bits) {
  KeyLayout lay;
  int rc = keyspace_layout(ks, &lay, nullptr);
  if (rc) return rc;
  if (bits) *bits = lay.bucket_shift + lay.bucket_bits;
  return DG_OK;
}

int dg_result_export(dg_result* r, const dg_keyspace* ks, const int32_t* const* maps, uint64_t* d_keys, uint64_t* d_slots) {
  if (!r) return set_error(DG_ERR_ARG, "null result");
  if (r->limited) return set_error(DG_ERR_ARG, "a limited result is not in key order");
  KeyLayout lay;
  AggPlan plan;
  int rc = keyspace_layout(ks, &lay, &plan);
  if (rc) return rc;
  if (ks->n_dims != r->ndims || ks->n_aggs != r->naggs) return set_error(DG_ERR_ARG, "key space does not match the result");
  if (r->ngroups > 0 && (!d_keys || !d_slots)) return set_error(DG_ERR_ARG, "null output buffer");
  int64_t bucket_delta = 0;
  if (ks->period_ms) {
    if (r->period != ks->period_ms) return set_error(DG_ERR_ARG, "granularity differs from the key space");
    const int64_t off = r->bucket0 - ks->bucket0;
    if (off < 0 || off % ks->period_ms) return set_error(DG_ERR_ARG, "result buckets off the key space grid");
    bucket_delta = off / ks->period_ms;  // the extent is checked on the last key below
  } else if (r->period) {
    return set_error(DG_ERR_ARG, "granularity differs from the key space");
  }
  for (int d = 0; d < r->ndims; ++d) {
    const int32_t card = dg_result_dim_cardinality(r, d);
    if (card > 0 && (!maps || !maps[d])) return set_error(DG_ERR_ARG, "null id map of dimension %d", d);
    for (int32_t i = 0; i < card; ++i) {
      const int32_t v = maps[d][i];
      if (v < 0 || v >= ks->card[d] || (i > 0 && v <= maps[d][i - 1]))
        return set_error(DG_ERR_ARG, "id map of dimension %d is not strictly increasing into [0, %d)", d, ks->card[d]);
    }
  }
  if (r->ngroups == 0) return DG_OK;
  CallGuard g(r->ctx);
  CallScratch* cs = g.cs;
  hipStream_t st = r->ctx->stream;
  RekeyMaps rm;
  memset(&rm, 0, sizeof rm);
  for (int d = 0; d < r->ndims; ++d) {
    const int32_t card = std::max(dg_result_dim_cardinality(r, d), 1);
    int32_t* dev;
    int32_t* h = up_take<int32_t>(cs, (size_t)card, &dev, st);
    if (!h) return set_error(DG_ERR_OOM, "id maps");
    if (dg_result_dim_cardinality(r, d) > 0) memcpy(h, maps[d], 4 * (size_t)card);
    else h[0] = 0;
    rm.m[d] = dev;
  }
  DG_FLUSH(cs, st);
  launch_gb_rekey(r->keys, r->ngroups, r->lay, lay, bucket_delta, rm, d_keys, st);
  launch_soa_to_aos(r->slots, r->cap, r->ngroups, r->naggs + 1, d_slots, st);
  if (ks->period_ms) {  // the last group holds the largest bucket index
    uint64_t last = 0;
    DG_HIP(hipMemcpyAsync(&last, r->keys + r->ngroups - 1, 8, hipMemcpyDeviceToHost, st));
    rc = finish_call(cs, st);
    if (rc) return rc;
    const int64_t b = r->lay.bucket_bits ? (int64_t)((last >> r->lay.bucket_shift) & ((1ull << r->lay.bucket_bits) - 1)) : 0;
    if (b + bucket_delta >= ks->n_buckets) return set_error(DG_ERR_ARG, "result bucket beyond the key space");
    return DG_OK;
  }
  return finish_call(cs, st);
}

int dg_keys_partition(dg_context* c, const uint64_t* d_keys, int64_t n, const uint64_t* splits, int32_t nsplit,
                      int64_t* out_pos) {
  Context* ctx = reinterpret_cast<Context*>(c);
  if (!ctx || n < 0 || nsplit < 0 || (nsplit && (!splits || !out_pos)) || (n > 0 && !d_keys))
    return set_error(DG_ERR_ARG, "bad arguments");
  if (nsplit == 0) return DG_OK;
  CallGuard g(ctx);
  CallScratch* cs = g.cs;
  hipStream_t st = ctx->stream;
  uint64_t* d_split;
  uint64_t* h = up_take<uint64_t>(cs, (size_t)nsplit, &d_split, st);
  int64_t* d_pos = dev_take<int64_t>(cs, (size_t)nsplit);
  int64_t* h_pos = host_take<int64_t>(cs, (size_t)nsplit);
  if (!h || !d_pos || !h_pos) return set_error(DG_ERR_OOM, "partition tables");
  memcpy(h, splits, 8 * (size_t)nsplit);
  DG_FLUSH(cs, st);
  launch_lower_bound(d_keys, n, d_split, nsplit, d_pos, st);
  DG_HIP(hipMemcpyAsync(h_pos, d_pos, 8 * (size_t)nsplit, hipMemcpyDeviceToHost, st));
  int rc = finish_call(cs, st);
  if (rc) return rc;
  memcpy(out_pos, h_pos, 8 * (size_t)nsplit);
  return DG_OK;
}

int dg_merge(dg_context* c, const dg_keyspace* ks, const uint64_t* d_keys, const uint64_t* d_slots, int64_t n,
             dg_result** out, dg_metrics* metrics) {
  auto t0 = std::chrono::steady_clock::now();
  Context* ctx = reinterpret_cast<Context*>(c);
  if (!ctx || !out || n < 0 || (n > 0 && (!d_keys || !d_slots))) return set_error(DG_ERR_ARG, "bad arguments");
  if (n >= (1ll << 32) - 16) return set_error(DG_ERR_UNSUPPORTED, "%lld records in one merge", (long long)n);
  KeyLayout lay;
  AggPlan plan;
  int rc = keyspace_layout(ks, &lay, &plan);
  if (rc) return rc;
  const int key_bits = lay.bucket_shift + lay.bucket_bits;
  const int rec = plan.n + 1;
  CallGuard g(ctx);
  CallScratch* cs = g.cs;
  hipStream_t st = ctx->stream;
  PendingResult res(new dg_result());
  res->ctx = ctx;
  res->ndims = ks->n_dims;
  res->naggs = plan.n;
  res->lay = lay;
  res->bucket0 = ks->bucket0;
  res->period = ks->period_ms;
  res->universal = ks->universal_time;
  res->kinds.assign(plan.kind, plan.kind + plan.n);
  res->cards.assign(ks->card, ks->card + ks->n_dims);
  dg_metrics m;
  memset(&m, 0, sizeof m);
  int64_t ng = 0;
  if (n > 0) {
    SortBufs sb;
    rc = sort_bufs(cs, n, 1, key_bits, 0, &sb);
    if (rc) return rc;
    uint32_t* head_pos = dev_take<uint32_t>(cs, (size_t)n + 16);
    uint32_t* h_n = host_take<uint32_t>(cs, 4);
    if (!head_pos || !h_n) return set_error(DG_ERR_OOM, "merge scratch of %lld records", (long long)n);
    // groups <= records: the result is sized by the input (no second pass over the groups)
    res->keys = static_cast<uint64_t*>(result_alloc(ctx, (size_t)n * 8));
    res->slots = static_cast<uint64_t*>(result_alloc(ctx, (size_t)n * rec * 8));
    res->cap = n;
    if (!res->keys || !res->slots) return set_error(DG_ERR_OOM, "merged result of %lld records", (long long)n);
    phase_event(ctx->ev[3], st);
    launch_merge_load(d_keys, n, &sb, st);
    launch_radix_sort(&sb, key_bits, st);
    phase_event(ctx->ev[5], st);
    launch_run_heads(&sb, st);
    launch_run_mark(&sb, head_pos, st);
    launch_merge_reduce(&sb, head_pos, d_slots, plan, n, res->keys, res->slots, st);
    launch_slots_finalize(res->slots, sb.n + 1, n, plan, st);
    DG_HIP(hipMemcpyAsync(h_n, sb.n, 8, hipMemcpyDeviceToHost, st));
    phase_event(ctx->ev[4], st);
    rc = finish_call(cs, st);
    if (rc) return rc;
    ng = h_n[1];
    float fs = 0, fr = 0;
    phase_elapsed(&fs, ctx->ev[3], ctx->ev[5]);
    phase_elapsed(&fr, ctx->ev[5], ctx->ev[4]);
    m.sort_ms = fs;
    m.reduce_ms = fr;
    m.aggregate_ms = fs + fr;
    m.sort_passes = key_bits > 0 ? (key_bits + 7) / 8 : 0;
    m.key_bits = key_bits;
  }
  res->ngroups = ng;
  m.selected_rows = n;
  m.groups = ng;
  m.total_ms = ms_since(t0);
  if (metrics) *metrics = m;
  *out = res.release();
  return DG_OK;
}

// ---- in-process cross-device merge (one process, several devices / contexts) ----
}  // extern "C"

namespace dg {

// Union of the parts' merged dictionaries of one dimension (each sorted, Java String order, nulls
// first) + for every part the map of its ids into the union (strictly increasing).
static void union_dictionary(const std::vector<const MergedDict*>& ds, MergedDict* out, std::vector<std::vector<int32_t>>* maps) {
  const size_t n = ds.size();
  maps->assign(n, {});
  std::vector<size_t> pos(n, 0);
  for (size_t p = 0; p < n; ++p) (*maps)[p].resize(ds[p]->values.size());
  for (;;) {
    int best = -1;
    for (size_t p = 0; p < n; ++p) {
      if (pos[p] >= ds[p]->values.size()) continue;
      if (best < 0 || cmp_nullable(ds[p]->is_null[pos[p]] != 0, ds[p]->values[pos[p]], ds[best]->is_null[pos[best]] != 0,
                                   ds[best]->values[pos[best]]) < 0)
        best = (int)p;
    }
    if (best < 0) break;
    const bool nul = ds[best]->is_null[pos[best]] != 0;
    const std::string v = ds[best]->values[pos[best]];
    out->values.push_back(nul ? std::string() : v);
    out->is_null.push_back(nul ? 1 : 0);
    const int32_t id = (int32_t)out->values.size() - 1;
    for (size_t p = 0; p < n; ++p)
      while (pos[p] < ds[p]->values.size() &&
             cmp_nullable(ds[p]->is_null[pos[p]] != 0, ds[p]->values[pos[p]], nul, v) == 0)
        (*maps)[p][pos[p]++] = id;
  }
  out->null_gid = (!out->values.empty() && out->is_null[0]) ? 0 : -1;
}

struct CtxBlock {  // a device block from a context's result cache, returned on scope exit
  Context* ctx = nullptr;
  void* p = nullptr;
  CtxBlock() = default;
  CtxBlock(const CtxBlock&) = delete;
  CtxBlock& operator=(const CtxBlock&) = delete;
  bool take(Context* c, size_t bytes) {
    ctx = c;
    std::lock_guard<std::mutex> g(c->mu);
    hipSetDevice(c->device);
    p = result_alloc(c, bytes);
    return p != nullptr;
  }
  ~CtxBlock() {
    if (!ctx || !p) return;
    std::lock_guard<std::mutex> g(ctx->mu);
    result_free(ctx, p);
  }
};

}  // namespace dg

extern "C" {

int dg_groupby_merge_devices(dg_result* const* parts, int32_t n_parts, dg_context* const* targets, int32_t n_targets,
                             dg_result** outs, dg_metrics* metrics) {
  auto t0 = std::chrono::steady_clock::now();
  if (!parts || n_parts <= 0 || !targets || n_targets <= 0 || !outs) return set_error(DG_ERR_ARG, "bad arguments");
  for (int32_t t = 0; t < n_targets; ++t) {
    if (!targets[t]) return set_error(DG_ERR_ARG, "null target %d", t);
    outs[t] = nullptr;
  }
  // every error return after the targets' merges have started releases what they produced
  struct OutsGuard {
    dg_result** outs;
    int32_t n;
    bool ok = false;
    ~OutsGuard() {
      if (ok) return;
      for (int32_t t = 0; t < n; ++t) {
        dg_result_release(outs[t]);
        outs[t] = nullptr;
      }
    }
  } guard{outs, n_targets};
  const dg_result* r0 = parts[0];
  for (int32_t p = 0; p < n_parts; ++p) {
    const dg_result* r = parts[p];
    if (!r) return set_error(DG_ERR_ARG, "null part %d", p);
    if (r->limited) return set_error(DG_ERR_ARG, "part %d is a limited result (not in key order)", p);
    if (r->dicts.empty() || (int)r->dicts.size() != r->ndims)
      return set_error(DG_ERR_ARG, "part %d is not a dg_groupby_run result", p);
    if (r->ndims != r0->ndims || r->naggs != r0->naggs || r->kinds != r0->kinds || r->period != r0->period ||
        r->bounds != r0->bounds || (!r->period && r->universal != r0->universal))
      return set_error(DG_ERR_ARG, "part %d is not a result of the same query", p);
  }
  const int nd = r0->ndims, na = r0->naggs, rec = na + 1;
  // one cluster key space: union dictionaries, bucket indices from the earliest part's origin
  std::vector<std::shared_ptr<MergedDict>> udicts(nd);
  std::vector<std::vector<std::vector<int32_t>>> maps(nd);  // [dim][part][id]
  std::vector<int32_t> card(nd);
  for (int d = 0; d < nd; ++d) {
    std::vector<const MergedDict*> ds;
    for (int32_t p = 0; p < n_parts; ++p) ds.push_back(parts[p]->dicts[d].get());
    udicts[d] = std::make_shared<MergedDict>();
    udicts[d]->dim = ds[0]->dim;
    union_dictionary(ds, udicts[d].get(), &maps[d]);
    card[d] = (int32_t)udicts[d]->values.size();
  }
  dg_keyspace ks;
  memset(&ks, 0, sizeof ks);
  ks.n_dims = nd;
  ks.card = card.data();
  ks.period_ms = r0->period;
  ks.universal_time = r0->universal;
  ks.n_aggs = na;
  ks.agg_kinds = r0->kinds.data();
  if (r0->period) {
    int64_t b0 = INT64_MAX, end = INT64_MIN;
    for (int32_t p = 0; p < n_parts; ++p) b0 = std::min(b0, parts[p]->bucket0);
    for (int32_t p = 0; p < n_parts; ++p) {
      const int64_t delta = (parts[p]->bucket0 - b0) / r0->period;
      if ((parts[p]->bucket0 - b0) % r0->period) return set_error(DG_ERR_ARG, "part %d buckets off the grid", p);
      end = std::max(end, delta + ((int64_t)1 << parts[p]->lay.bucket_bits));
    }
    ks.bucket0 = b0;
    ks.n_buckets = std::max<int64_t>(end, 1);
  }
  int32_t kbits = 0;
  int rc = dg_keyspace_bits(&ks, &kbits);
  if (rc) return rc;
  // Work items of the phases below run concurrently, one host thread each (ChainedExecutionQueryRunner
  // runs the segment runners on the processing pool; here every device's work goes out at once and
  // each context's own mutex serialises calls that share a device). An item's error (code and the
  // thread's dg_last_error text) is handed back to the calling thread.
  struct ItemErr {
    int rc = DG_OK;
    std::string msg;
  };
  auto run_items = [](int n, const std::function<int(int)>& fn, std::vector<ItemErr>* errs) -> int {
    errs->assign(n, ItemErr());
    std::vector<std::thread> th;
    for (int i = 1; i < n; ++i)
      th.emplace_back([&, i] {
        (*errs)[i].rc = fn(i);
        if ((*errs)[i].rc) (*errs)[i].msg = dg_last_error();
      });
    if (n > 0) {
      (*errs)[0].rc = fn(0);
      if ((*errs)[0].rc) (*errs)[0].msg = dg_last_error();
    }
    for (auto& x : th) x.join();
    for (auto& e : *errs)
      if (e.rc) return set_error(e.rc, "%s", e.msg.c_str());
    return DG_OK;
  };
  std::vector<ItemErr> errs;
  // every part re-keyed into the key space on its own device
  std::vector<CtxBlock> xkeys(n_parts), xslots(n_parts);
  std::vector<int64_t> np(n_parts);
  rc = run_items(n_parts, [&](int p) -> int {
    dg_result* r = parts[p];
    np[p] = r->ngroups;
    if (!np[p]) return DG_OK;
    if (!xkeys[p].take(r->ctx, (size_t)np[p] * 8) || !xslots[p].take(r->ctx, (size_t)np[p] * rec * 8))
      return set_error(DG_ERR_OOM, "export buffers of part %d (%lld groups)", p, (long long)np[p]);
    std::vector<const int32_t*> mp(nd);
    for (int d = 0; d < nd; ++d) mp[d] = maps[d][p].data();
    return dg_result_export(r, &ks, mp.data(), static_cast<uint64_t*>(xkeys[p].p), static_cast<uint64_t*>(xslots[p].p));
  }, &errs);
  if (rc) return rc;
  // key ranges: n_targets - 1 splitters from evenly spaced samples of every part (weighted by the
  // part's size), identical cuts on every part, so equal keys meet on one target
  std::vector<uint64_t> splits;
  if (n_targets > 1) {
    struct Smp {
      uint64_t key;
      double w;
    };
    std::vector<Smp> smp;
    double total = 0;
    for (int32_t p = 0; p < n_parts; ++p) {
      if (!np[p]) continue;
      const int64_t s = std::min<int64_t>(np[p], 4096), stride = np[p] / s;
      std::vector<uint64_t> h((size_t)s);
      Context* c = parts[p]->ctx;
      {
        std::lock_guard<std::mutex> g(c->mu);
        hipSetDevice(c->device);
        DG_HIP(hipMemcpy2D(h.data(), 8, xkeys[p].p, (size_t)stride * 8, 8, (size_t)s, hipMemcpyDeviceToHost));
      }
      for (uint64_t k : h) smp.push_back({k, (double)np[p] / (double)s});
      total += (double)np[p];
    }
    std::sort(smp.begin(), smp.end(), [](const Smp& a, const Smp& b) { return a.key < b.key; });
    double acc = 0;
    size_t i = 0;
    for (int32_t t = 1; t < n_targets; ++t) {
      const double want = total * t / n_targets;
      while (i < smp.size() && acc + smp[i].w <= want) acc += smp[i++].w;
      splits.push_back(i < smp.size() ? smp[i].key : ~0ull);
    }
  }
  std::vector<std::vector<int64_t>> cut(n_parts, std::vector<int64_t>(n_targets + 1, 0));
  rc = run_items(n_parts, [&](int p) -> int {
    cut[p][n_targets] = np[p];
    if (n_targets > 1 && np[p])
      return dg_keys_partition(reinterpret_cast<dg_context*>(parts[p]->ctx), static_cast<uint64_t*>(xkeys[p].p), np[p],
                               splits.data(), n_targets - 1, cut[p].data() + 1);
    return DG_OK;
  }, &errs);
  if (rc) return rc;
  // every range moves to its target (peer copies over xGMI; a device copy on the same device) and is
  // merged there in part order (equal keys combine in that order); the targets work concurrently
  std::vector<dg_metrics> tm(n_targets);
  rc = run_items(n_targets, [&](int t) -> int {
    Context* tc = reinterpret_cast<Context*>(targets[t]);
    int64_t n = 0;
    for (int32_t p = 0; p < n_parts; ++p) n += cut[p][t + 1] - cut[p][t];
    CtxBlock rk, rs;
    if (n > 0 && (!rk.take(tc, (size_t)n * 8) || !rs.take(tc, (size_t)n * rec * 8)))
      return set_error(DG_ERR_OOM, "receive buffers of target %d (%lld records)", t, (long long)n);
    {
      std::lock_guard<std::mutex> g(tc->mu);
      hipSetDevice(tc->device);
      int64_t at = 0;
      for (int32_t p = 0; p < n_parts; ++p) {
        const int64_t a = cut[p][t], m = cut[p][t + 1] - a;
        if (m <= 0) continue;
        const int sdev = parts[p]->ctx->device;
        if (sdev != tc->device) {
          int can = 0;
          if (hipDeviceCanAccessPeer(&can, tc->device, sdev) == hipSuccess && can) {
            hipError_t e = hipDeviceEnablePeerAccess(sdev, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
              return set_error(DG_ERR_DEVICE, "peer access %d -> %d", tc->device, sdev);
            (void)hipGetLastError();
          }
        }
        DG_HIP(hipMemcpyPeerAsync(static_cast<uint64_t*>(rk.p) + at, tc->device, static_cast<uint64_t*>(xkeys[p].p) + a,
                                  sdev, (size_t)m * 8, tc->stream));
        DG_HIP(hipMemcpyPeerAsync(static_cast<uint64_t*>(rs.p) + at * rec, tc->device,
                                  static_cast<uint64_t*>(xslots[p].p) + a * rec, sdev, (size_t)m * rec * 8, tc->stream));
        at += m;
      }
      DG_HIP(hipStreamSynchronize(tc->stream));
    }
    const int mrc = dg_merge(targets[t], &ks, static_cast<uint64_t*>(rk.p), static_cast<uint64_t*>(rs.p), n, &outs[t], &tm[t]);
    if (mrc) return mrc;
    outs[t]->dicts = udicts;  // the union dictionaries: the merged result fetches like a groupBy result
    outs[t]->bounds = r0->bounds;
    return DG_OK;
  }, &errs);
  if (rc) return rc;
  dg_metrics tot;
  memset(&tot, 0, sizeof tot);
  for (int32_t t = 0; t < n_targets; ++t) {
    tot.sort_ms += tm[t].sort_ms;
    tot.reduce_ms += tm[t].reduce_ms;
    tot.aggregate_ms += tm[t].aggregate_ms;
    tot.selected_rows += tm[t].selected_rows;
    tot.groups += tm[t].groups;
    tot.sort_passes = tm[t].sort_passes;
    tot.key_bits = tm[t].key_bits;
  }
  tot.total_ms = ms_since(t0);
  if (metrics) *metrics = tot;
  guard.ok = true;
  return DG_OK;
}

// ---- timeseries merge (TimeseriesBinaryFn fold, host) ----
int dg_timeseries_merge(const dg_scan* scan, int32_t n_lists, const int32_t* n, int32_t cap, const int64_t* times,
                        const int64_t* rows, const uint64_t* values, int32_t skip_empty, int32_t out_cap,
                        int32_t* out_n, int64_t* out_time, int64_t* out_rows, uint64_t* out_values) {
  if (!scan || n_lists < 0 || cap < 0 || (n_lists && (!n || !times || !rows)) || !out_n || out_cap < 0)
    return set_error(DG_ERR_ARG, "bad arguments");
  const int na = scan->n_aggs;
  if (na < 0 || na > kMaxAggs || (na && (!scan->aggs || (n_lists && !values)))) return set_error(DG_ERR_ARG, "bad aggregators");
  for (int a = 0; a < na; ++a)
    if (scan->aggs[a].kind < DG_AGG_COUNT || scan->aggs[a].kind > DG_AGG_FLOAT_MAX)
      return set_error(DG_ERR_ARG, "aggregator kind %d", scan->aggs[a].kind);
  const bool all = scan->period_ms == 0 && !scan->bucket_starts;
  struct E {
    int64_t t;
    int32_t list, k;
  };
  std::vector<E> es;
  for (int32_t i = 0; i < n_lists; ++i) {
    if (n[i] > cap) return set_error(DG_ERR_ARG, "list %d holds %d > cap %d buckets", i, n[i], cap);
    for (int32_t k = 0; k < n[i]; ++k) {
      const int64_t at = (int64_t)i * cap + k;
      if (skip_empty && rows[at] == 0) continue;
      es.push_back({times[at], i, k});
    }
  }
  // ResultMergeQueryRunner order: time, then the runners' order
  std::stable_sort(es.begin(), es.end(), [](const E& a, const E& b) { return a.t != b.t ? a.t < b.t : a.list < b.list; });
  std::vector<int64_t> mt, mr;
  std::vector<uint64_t> mv;
  for (size_t e = 0; e < es.size(); ++e) {
    const int64_t at = (int64_t)es[e].list * cap + es[e].k;
    const bool same = !mt.empty() && (all || mt.back() == es[e].t);
    if (!same) {
      mt.push_back(es[e].t);  // ALL: the earliest result's timestamp
      mr.push_back(0);
      for (int a = 0; a < na; ++a) mv.push_back(values[at * na + a]);
    } else {
      uint64_t* acc = mv.data() + (mt.size() - 1) * na;
      for (int a = 0; a < na; ++a) acc[a] = combine_abi(scan->aggs[a].kind, acc[a], values[at * na + a]);
    }
    mr.back() += rows[at];
  }
  const int32_t m = (int32_t)mt.size();
  if (m > out_cap) return set_error(DG_ERR_ARG, "%d merged buckets > out_cap %d", m, out_cap);
  for (int32_t i = 0; i < m; ++i) {
    const int32_t j = scan->descending ? m - 1 - i : i;  // descending queries list buckets latest first
    if (out_time) out_time[i] = mt[j];
    if (out_rows) out_rows[i] = mr[j];
    if (out_values)
      for (int a = 0; a < na; ++a) out_values[(int64_t)i * na + a] = mv[(size_t)j * na + a];
  }
  *out_n = m;
  return DG_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// diagnostics: decode arbitrary LZ4 blocks through the engine's attach-time index + HIP decoder
// ------------------------------------------------------------------------------------------------
extern "C" int dg_set_phase_timing(int32_t on) {
  g_phase_timing.store(on != 0, std::memory_order_relaxed);
  return DG_OK;
}

// DG_PROBE_CHAIN / _GRAPH: n dependent tiny kernels per repetition, launched one by one or replayed
// from one captured graph; checks that every step ran (the word counts the launches)
static int probe_chain(int n, int iters, bool graph, double* ms, hipStream_t st) {
  uint32_t* w = nullptr;
  if (hipMalloc(&w, 4) != hipSuccess) return set_error(DG_ERR_OOM, "probe word");
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = DG_OK;
  hipMemsetAsync(w, 0, 4, st);
  if (graph) {
    bool ok = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) == hipSuccess;
    if (ok) launch_probe_chain(w, n, st);
    ok = hipStreamEndCapture(st, &g) == hipSuccess && ok;
    ok = ok && hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) == hipSuccess;
    if (!ok) rc = set_error(DG_ERR_DEVICE, "probe: graph capture");
  }
  auto once = [&] {
    if (graph) hipGraphLaunch(ge, st);
    else launch_probe_chain(w, n, st);
  };
  if (rc == DG_OK) {
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    once();  // warm-up
    hipEventRecord(e0, st);
    for (int i = 0; i < iters; ++i) once();
    hipEventRecord(e1, st);
    uint32_t got = 0;
    if (hipStreamSynchronize(st) != hipSuccess || hipGetLastError() != hipSuccess ||
        hipMemcpy(&got, w, 4, hipMemcpyDeviceToHost) != hipSuccess) {
      rc = set_error(DG_ERR_DEVICE, "probe failed");
    } else if (got != (uint32_t)n * (uint32_t)(iters + 1)) {
      rc = set_error(DG_ERR_DEVICE, "probe: chain counted %u of %lld steps", got, (long long)n * (iters + 1));
    } else {
      float f = 0;
      hipEventElapsedTime(&f, e0, e1);
      *ms = (double)f / iters;
    }
  }
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  if (ge) hipGraphExecDestroy(ge);
  if (g) hipGraphDestroy(g);
  hipFree(w);
  return rc;
}

// DG_PROBE_HOST_*: host-side cost of the enqueue calls a small query makes (ms per call, host clock)
static int probe_host(int kind, int64_t n, int iters, double* ms, hipStream_t st) {
  uint32_t* w = nullptr;
  void* h = nullptr;
  hipStream_t s2 = nullptr;
  hipEvent_t ev = nullptr;
  int rc = DG_OK;
  const size_t bytes = kind == DG_PROBE_HOST_H2D ? (size_t)std::max<int64_t>(n, 4) : 4;
  bool ok = hipMalloc(&w, bytes) == hipSuccess && hipHostMalloc(&h, bytes, hipHostMallocDefault) == hipSuccess &&
            hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess;
  if (!ok) rc = set_error(DG_ERR_OOM, "probe buffers");
  const int reps = kind == DG_PROBE_HOST_LAUNCH ? (int)std::min<int64_t>(n, 4096) : 1;
  auto once = [&] {
    if (kind == DG_PROBE_HOST_LAUNCH) {
      launch_probe_chain(w, reps, st);
    } else if (kind == DG_PROBE_HOST_H2D) {
      hipMemcpyAsync(w, h, bytes, hipMemcpyHostToDevice, st);
    } else {
      hipEventRecord(ev, st);
      hipStreamWaitEvent(s2, ev, 0);
    }
  };
  if (rc == DG_OK) {
    hipMemsetAsync(w, 0, bytes, st);
    for (int i = 0; i < 8; ++i) once();  // warm-up
    if (hipStreamSynchronize(st) != hipSuccess || hipStreamSynchronize(s2) != hipSuccess) rc = set_error(DG_ERR_DEVICE, "probe failed");
  }
  if (rc == DG_OK) {
    double total = 0;
    for (int i = 0; i < iters; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      once();
      total += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (hipStreamSynchronize(st) != hipSuccess || hipStreamSynchronize(s2) != hipSuccess) {
        rc = set_error(DG_ERR_DEVICE, "probe failed");
        break;
      }
    }
    if (rc == DG_OK) *ms = total / iters / reps;
  }
  if (ev) hipEventDestroy(ev);
  if (s2) hipStreamDestroy(s2);
  if (h) hipHostFree(h);
  if (w) hipFree(w);
  return rc;
}

extern "C" int dg_debug_probe(int32_t device, int32_t kind, int64_t n, int32_t iters, double* ms) {
  if (!ms || n <= 0 || iters <= 0 || kind < DG_PROBE_COPY || kind > DG_PROBE_HOST_JOIN)
    return set_error(DG_ERR_ARG, "bad probe arguments");
  DG_HIP(hipSetDevice(device));
  hipStream_t st;
  DG_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  if (kind == DG_PROBE_SORT) {
    const int rcs = probe_sort(n, iters, ms, st);
    hipStreamDestroy(st);
    return rcs;
  }
  if (kind >= DG_PROBE_HOST_LAUNCH) {
    const int rch = probe_host(kind, n, iters, ms, st);
    hipStreamDestroy(st);
    return rch;
  }
  if (kind == DG_PROBE_CHAIN || kind == DG_PROBE_CHAIN_GRAPH) {
    const int rcc = probe_chain((int)std::min<int64_t>(n, 4096), iters, kind == DG_PROBE_CHAIN_GRAPH, ms, st);
    hipStreamDestroy(st);
    return rcc;
  }
  void *a = nullptr, *b = nullptr, *h = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = DG_OK;
  auto dev_alloc = [&](void** p, size_t bytes) { return hipMalloc(p, bytes) == hipSuccess; };
  const bool gather = kind == DG_PROBE_GATHER;
  if (gather && n >= (1ll << 32)) rc = set_error(DG_ERR_ARG, "probe: gather of %lld rows (32-bit rows)", (long long)n);
  const size_t bytes = gather ? 0 : (size_t)((n + 15) & ~15ll);
  bool ok = rc == DG_OK;
  if (ok && gather) ok = dev_alloc(&a, (size_t)n * 8) && dev_alloc(&b, (size_t)n * 16) && dev_alloc(&h, (size_t)n * 32);
  else if (ok && kind == DG_PROBE_COPY) ok = dev_alloc(&a, bytes) && dev_alloc(&b, bytes);
  else if (ok) ok = dev_alloc(&a, bytes) && hipHostMalloc(&h, bytes, hipHostMallocDefault) == hipSuccess;
  if (ok && kind == DG_PROBE_ZC_WRITE) ok = hipHostGetDevicePointer(&b, h, 0) == hipSuccess;
  if (!ok && rc == DG_OK) rc = set_error(DG_ERR_OOM, "probe buffers of %lld", (long long)n);
  if (rc == DG_OK) {
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    if (gather) launch_probe_fill(static_cast<uint64_t*>(a), b, n, st);
    else if (kind != DG_PROBE_H2D) hipMemsetAsync(a, 1, bytes, st);
    auto once = [&] {
      switch (kind) {
        case DG_PROBE_COPY: launch_probe_copy(a, b, (int64_t)bytes, st); break;
        case DG_PROBE_D2H: hipMemcpyAsync(h, a, bytes, hipMemcpyDeviceToHost, st); break;
        case DG_PROBE_H2D: hipMemcpyAsync(a, h, bytes, hipMemcpyHostToDevice, st); break;
        case DG_PROBE_GATHER: launch_probe_gather(static_cast<const uint64_t*>(a), b, n, static_cast<uint64_t*>(h), st); break;
        default: launch_probe_copy(a, b, (int64_t)bytes, st); break;  // (a -> pinned host memory, mapped)
      }
    };
    once();  // warm-up
    hipEventRecord(e0, st);
    for (int i = 0; i < iters; ++i) once();
    hipEventRecord(e1, st);
    if (hipStreamSynchronize(st) != hipSuccess || hipGetLastError() != hipSuccess) {
      rc = set_error(DG_ERR_DEVICE, "probe failed");
    } else {
      float f = 0;
      hipEventElapsedTime(&f, e0, e1);
      *ms = (double)f / iters;
    }
  }
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  if (a) hipFree(a);
  if (gather || kind == DG_PROBE_COPY) {
    if (b) hipFree(b);
    if (h && gather) hipFree(h);
  } else if (h) {
    hipHostFree(h);
  }
  hipStreamDestroy(st);
  return rc;
}

extern "C" int dg_debug_lz4_classify(const uint8_t* block, int32_t len, int32_t* kind) {
  if (!block || len <= 0 || len > kBlockBytes + 2048 || !kind) return set_error(DG_ERR_ARG, "bad arguments");
  std::vector<uint32_t> one;
  int wide = 0, light = 0, nfine = 0;
  std::vector<uint8_t> lv;
  const int d = lz4_index_block(block, len, &one, &wide, &light, &nfine, &lv);
  std::vector<uint8_t> rx;
  int nint = 0, nfar = 0;
  const bool run = d > 0 && lz4_run_index(block, len, d, &rx, &nint, &nfar);
  // -1 malformed, 0 general, 1 general (wide), 2 light, 3 run, 4 flow (narrow or wide)
  *kind = d < 0 ? -1 : run ? 3 : light ? 2 : (wide & kLzFlow) ? 4 : wide ? 1 : 0;
  return DG_OK;
}

extern "C" int dg_debug_lz4_decode(dg_context* c, const uint8_t* const* blocks, const int32_t* lens, int32_t n,
                                   uint8_t* out, int32_t* out_lens, double* ms, uint64_t* prof) {
  Context* ctx = reinterpret_cast<Context*>(c);
  if (!ctx || n <= 0 || !blocks || !lens || !out || !out_lens) return set_error(DG_ERR_ARG, "bad arguments");
  BlockColumn b;
  b.codec = CODEC_LZ4;
  b.nblocks = n;
  b.comp_off.resize(n);
  b.comp_len.resize(n);
  b.cp_off.resize(n);
  b.cp_n.resize(n);
  b.cp_wide.assign(n, 0);
  b.cp_light.assign(n, 0);
  b.cp_fine.assign(n, 0);
  b.dec_len.resize(n);
  b.run_off.assign(n, -1);
  b.run_n.assign(n, 0);
  b.run_far.assign(n, 0);
  b.lvl_off.assign(n, -1);
  b.lvl_n.assign(n, 0);
  std::vector<uint8_t> rall, lall;
  int64_t total = kCompSlack;
  for (int i = 0; i < n; ++i) {
    if (lens[i] <= 0 || lens[i] > kBlockBytes + 2048) return set_error(DG_ERR_ARG, "block %d length %d", i, lens[i]);
    b.comp_off[i] = total;
    b.comp_len[i] = lens[i];
    total += (lens[i] + 15) & ~15;
  }
  std::vector<uint8_t> host((size_t)total + kCompSlack, 0);
  std::vector<uint32_t> cps;
  for (int i = 0; i < n; ++i) {
    memcpy(host.data() + b.comp_off[i], blocks[i], (size_t)lens[i]);
    std::vector<uint32_t> one;
    int wide = 0, light = 0, nfine = 0, nlvl = 0;
    const size_t lat = lall.size();
    const int d = lz4_index_block(blocks[i], lens[i], &one, &wide, &light, &nfine, &lall, &nlvl);
    if (lall.size() > lat) {
      b.lvl_off[i] = (int64_t)lat;
      b.lvl_n[i] = nlvl;
    }
    b.cp_wide[i] = (uint8_t)wide;
    b.cp_light[i] = (uint8_t)light;
    b.cp_fine[i] = nfine;
    b.cp_off[i] = (int64_t)cps.size();
    b.cp_n[i] = d < 0 ? -1 : (int32_t)one.size() - nfine;
    b.dec_len[i] = d < 0 ? 0 : d;
    out_lens[i] = d;
    if (d >= 0) cps.insert(cps.end(), one.begin(), one.end());
    const size_t at = rall.size();
    if (d > 0 && lz4_run_index(blocks[i], lens[i], d, &rall, &b.run_n[i], &b.run_far[i])) b.run_off[i] = (int64_t)at;
  }
  if (cps.empty()) cps.push_back(0);
  if (!rall.empty()) rall.resize(rall.size() + 16, 0);  // (k_lz4_run reads 12 bytes at a time)
  CallGuard g(ctx);
  hipStream_t st = ctx->stream;
  if (!b.comp.alloc(host.size()) || !b.cps.alloc(cps.size() * 4)) return set_error(DG_ERR_OOM, "debug decode");
  if (!rall.empty() && !b.runx.alloc(rall.size())) return set_error(DG_ERR_OOM, "debug decode");
  if (!lall.empty() && !b.lvls.alloc(lall.size())) return set_error(DG_ERR_OOM, "debug decode");
  DG_HIP(hipMemcpy(b.comp.p, host.data(), host.size(), hipMemcpyHostToDevice));
  DG_HIP(hipMemcpy(b.cps.p, cps.data(), cps.size() * 4, hipMemcpyHostToDevice));
  if (!rall.empty()) DG_HIP(hipMemcpy(b.runx.p, rall.data(), rall.size(), hipMemcpyHostToDevice));
  if (!lall.empty()) DG_HIP(hipMemcpy(b.lvls.p, lall.data(), lall.size(), hipMemcpyHostToDevice));
  const int routes = decode_routes();
  DecodeBatch db;
  uint8_t* slots = dev_take<uint8_t>(g.cs, (size_t)n * kBlockBytes + 64);
  if (!slots) return set_error(DG_ERR_OOM, "debug decode slots");
  for (int i = 0; i < n; ++i)
    if (out_lens[i] >= 0) db.jobs.push_back(lz4_job(b, i, slots + (size_t)i * kBlockBytes, out_lens[i], routes));
  uint64_t* d_prof = nullptr;
  if (prof) {
    d_prof = dev_take<uint64_t>(g.cs, (size_t)n * kLz4ProfWords);
    if (!d_prof) return set_error(DG_ERR_OOM, "debug decode profile");
    DG_HIP(hipMemsetAsync(d_prof, 0, (size_t)n * kLz4ProfWords * 8, st));
  }
  phase_event(ctx->ev[0], st);
  int rc = run_decodes(g.cs, &db, st, d_prof);
  if (rc) return rc;
  phase_event(ctx->ev[1], st);
  rc = finish_call(g.cs, st);
  if (rc) return rc;
  float f = 0;
  phase_elapsed(&f, ctx->ev[0], ctx->ev[1]);
  if (ms) *ms = f;
  DG_HIP(hipMemcpy(out, slots, (size_t)n * kBlockBytes, hipMemcpyDeviceToHost));
  if (prof) DG_HIP(hipMemcpy(prof, d_prof, (size_t)db.jobs.size() * kLz4ProfWords * 8, hipMemcpyDeviceToHost));
  return DG_OK;
}
