// dg_lz4.hip — LZ4 block decompression on gfx950 (Druid's per-block column codec).
//
// Replaces CompressionStrategy.LZ4Decompressor.decompress (processing/.../segment/data/
// CompressionStrategy.java:284-305 -> lz4-java 1.4.0 LZ4SafeDecompressor): one 64 KiB Druid block
// (CompressedPools.BUFFER_SIZE, segment/CompressedPools.java:39) per 1024-thread workgroup.
//
// Druid's numeric blocks are token-dense: a block of sequential longs is ~8,160 sequences of
// [1 literal byte, 7-byte match] whose matches copy bytes earlier matches produced (copy chains up
// to ~300 deep), so neither a lane walking the token stream nor match-by-match copying is fast. The
// block is decoded in four data-parallel phases, all in LDS:
//   1. parse: the attach-time checkpoint index (lz4_index_block: the token offset of every 8th
//      sequence, every 16th in blocks of more than 8192, every ceil(n / 1024)th in blocks of n <
//      8192) gives every thread its own interval; it parses those sequences from the staged input
//      into registers (literal start or bytes, literal length, distance, match length);
//   2. a block scan of the threads' output lengths places every sequence; each output byte x gets a
//      16-bit entry E[x] in LDS: a literal is 0xFF00 | byte, a match byte the distance to the byte
//      it copies (LZ4 overlap semantics: src = start - dist + (k mod dist));
//   3. resolution: E[x] += E[x - E[x]] until x - E[x] is a literal (updates are asynchronous, any
//      value read is a valid ancestor distance) — a carry scan over residue classes for blocks of
//      distance-8 chains, position-ordered stages (then pointer-jumping rounds) otherwise;
//   4. out[x] = low byte of the literal at x - E[x], written as 16-byte stores.
// The staged input and E share one 128 KiB LDS array (the parse finishes before E is written;
// literals are re-read from the compressed block in HBM/L2). Entries >= 0xFF00 are literals, so a
// distance must stay below 0xFF00: the last 256 output positions, whose distances can exceed it,
// are moved into a small tail table of absolute sources and resolved by a short chase.
#include <hip/hip_runtime.h>


#include "dg_internal.h"
#include "dg_device.h"

namespace dg {

// Global-memory accesses through address-space-1 pointers: the pointers of a job are generic, and a
// generic (flat) access also counts as an LDS operation, so every later wait for an LDS result
// would wait for it too (the decoders interleave their output stores and L2 literal reads with LDS).
typedef __attribute__((ext_vector_type(4))) unsigned int v4u32;
typedef __attribute__((address_space(1))) v4u32 g_v4u32;
typedef __attribute__((address_space(1))) uint64_t g_u64;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint8_t g_u8;
__device__ __forceinline__ uint4 gld16(const void* p) {
  const v4u32 v = *(const g_v4u32*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t gld4(const void* p) { return *(const g_u32*)p; }
__device__ __forceinline__ uint32_t gld1(const void* p) { return *(const g_u8*)p; }
__device__ __forceinline__ void gst16(void* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  v4u32 v;
  v.x = a;
  v.y = b;
  v.z = c;
  v.w = d;
  *(g_v4u32*)p = v;
}
__device__ __forceinline__ void gst8(void* p, uint32_t lo, uint32_t hi) { *(g_u64*)p = ((uint64_t)hi << 32) | lo; }
__device__ __forceinline__ void gst4(void* p, uint32_t v) { *(g_u32*)p = v; }

constexpr int kLzThreads = 1024;               // 16 waves: 4 per SIMD hide LDS latency
constexpr int kLzWaves = kLzThreads / 64;
constexpr int kLz4InCap = kBlockBytes + 2048;  // >= LZ4_compressBound(65536) = 65809
constexpr int kTail = 0xFF00;                  // E codes >= kTail are literals; positions >= kTail use the tail table
constexpr int kTailN = kBlockBytes - kTail;    // 256
constexpr uint32_t kTailLit = 0x10000u;        // tail table word: a literal byte (else an absolute source)
constexpr int kShortLit = 4;                   // literal runs up to this ride in the parse registers
static_assert(kShortLit <= 4, "Tok::lv holds four literal bytes");
constexpr int kLongFill = 48;                  // matches above this are filled cooperatively
constexpr int kMaxJobs = 2048;
constexpr int kPairs = 32;                     // E pairs per thread: 2 * 32 * 1024 = 65536 positions
#ifndef DG_LZ_STAGE_K
#define DG_LZ_STAGE_K 1  // pairs per thread in a resolution stage (1 measured faster than 2 and 4)
#endif
#ifndef DG_LZ_STAGE_STEPS
#define DG_LZ_STAGE_STEPS 24  // extra jumps inside a stage before an entry is left to the rounds (3 / 6 / 12 / 24: 24 fastest)
#endif
#ifndef DG_LZ_JUMP_BATCH
#define DG_LZ_JUMP_BATCH 4
#endif
constexpr int kJumpBatch = DG_LZ_JUMP_BATCH;  // steps of a jump sweep whose reads are issued together
constexpr int kMaxRounds = 20;                 // > log2(65536) + 1: pointer jumping always converges before
constexpr int kClass = 8;                      // the value width whose distance-8 copy chains are scanned
static_assert(kLz4InCap + 32 <= kBlockBytes * 2, "staged input must fit in the E array");
static_assert(kLzMaxCps == kLzThreads, "one checkpoint interval per thread");
static_assert(kLzThreads * kLzMaxSeqPerCp >= kBlockBytes / 4, "a block can hold 16384 sequences");

struct Tok {
  int lit;   // literal start (input offset)
  int L;     // literal length
  uint32_t lv;  // the first min(L, 4) literal bytes, little-endian
  int off;   // match distance (0 for the last sequence)
  int M;     // match length (0 for the last sequence)
  int next;  // next token start
};

// LZ4 extended length: sum of bytes up to and including the first byte != 255. Runs of 255 (long
// zero runs in dictionary-id blocks: a 64 KiB match is 256 of them) are skipped 16 bytes at a time.
__device__ __forceinline__ bool ext_len(const uint8_t* __restrict__ in, int n, int& q, int& len) {
  for (;;) {
    if ((q & 15) == 0 && q + 16 <= n) {
      const uint4 w = *reinterpret_cast<const uint4*>(in + q);
      if ((w.x & w.y & w.z & w.w) == 0xFFFFFFFFu) {
        len += 16 * 255;
        q += 16;
        continue;
      }
    }
    if (q >= n) return false;
    const int b = in[q++];
    len += b;
    if (b != 255) return true;
  }
}

// Byte-wise parse (long lengths / windows that do not hold the offset); out of line: rare, and the
// decoder's per-sequence loops are unrolled.
__device__ __forceinline__ bool parse_tok_slow(const uint8_t* __restrict__ in, int n, int p, Tok& t) {
  if (p >= n) return false;
  const int tk = in[p];
  int q = p + 1;
  int L = tk >> 4;
  if (L == 15 && !ext_len(in, n, q, L)) return false;
  t.lit = q;
  t.L = L;
  t.lv = 0;
  if (L <= 4 && q + L <= n)
    for (int k = 0; k < L; ++k) t.lv |= (uint32_t)in[q + k] << (8 * k);
  q += L;
  if (q > n) return false;
  if (q == n) {  // last sequence: literals only
    t.off = 0;
    t.M = 0;
    t.next = n;
    return true;
  }
  if (q + 2 > n) return false;
  t.off = (int)in[q] | ((int)in[q + 1] << 8);
  q += 2;
  int M = tk & 15;
  if (M == 15 && !ext_len(in, n, q, M)) return false;
  t.M = M + 4;
  t.next = q;
  return t.off != 0;
}

// Parse the token at p from one 8-byte window (three aligned dword reads, one LDS round trip) when
// the token, its literals and its distance fit in it; false = not a valid token here.
__device__ __forceinline__ bool parse_tok(const uint8_t* __restrict__ in, int n, int p, Tok& t) {
  if (p >= n) return false;
  const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in);
  const int a = p >> 2, sh = (p & 3) << 3;
  const uint64_t w01 = (uint64_t)in32[a] | ((uint64_t)in32[a + 1] << 32);
  const uint32_t w2 = in32[a + 2];
  const uint64_t win = sh ? ((w01 >> sh) | ((uint64_t)w2 << (64 - sh))) : w01;
  const int tk = (int)(win & 0xFF);
  const int L = tk >> 4, M = tk & 15;
  if (L > 5 || M == 15) return parse_tok_slow(in, n, p, t);
  const int q = p + 1 + L;
  t.lit = p + 1;
  t.L = L;
  t.lv = (uint32_t)(win >> 8);
  if (q > n) return false;
  if (q == n) {
    t.off = 0;
    t.M = 0;
    t.next = n;
    return true;
  }
  if (q + 2 > n) return false;
  t.off = (int)((win >> (8 * (1 + L))) & 0xFFFF);
  t.M = M + 4;
  t.next = q + 2;
  return t.off != 0;
}

// inclusive add-scan over the 64 lanes of a wave: row shifts 1/2/4/8, then the row broadcasts of
// lanes 15 and 31 (DPP: no LDS round trips, unlike a __shfl_up ladder)
template <int CTRL, int RMASK>
__device__ __forceinline__ int dpp_add_step(int v) {
  return v + __builtin_amdgcn_update_dpp(0, v, CTRL, RMASK, 0xf, false);
}
__device__ __forceinline__ int wave_add_scan(int v) {
  v = dpp_add_step<0x111, 0xf>(v);  // row_shr:1
  v = dpp_add_step<0x112, 0xf>(v);  // row_shr:2
  v = dpp_add_step<0x114, 0xf>(v);  // row_shr:4
  v = dpp_add_step<0x118, 0xf>(v);  // row_shr:8
  v = dpp_add_step<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v = dpp_add_step<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
  return v;
}

// block-wide (1024 threads) exclusive scan; total via *total
__device__ int block_scan_lz(int v, int* total, int* s_tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int x = wave_add_scan(v);
  if (lane == 63) s_tmp[wave] = x;
  __syncthreads();
  int wave_off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kLzWaves; ++w) {
    const int y = s_tmp[w];
    wave_off += w < wave ? y : 0;
    tot += y;
  }
  __syncthreads();
  *total = tot;
  return wave_off + x - v;
}

// E is skewed by one dword every 128 entries so that the threads of a wave, whose intervals start
// ~128 output bytes apart in token-dense blocks, write different LDS banks.
constexpr int kESkewShift = 7;
constexpr int kEWords = kBlockBytes + (kBlockBytes >> kESkewShift) * 2;  // u16 entries incl. skew
__device__ __forceinline__ int eph(int x) { return x + ((x >> kESkewShift) << 1); }

// The fill writes E at every position, the tail's too: a literal code, or the distance when it is
// below kTail. A tail position whose distance is not (a match reaching the block's first bytes) gets
// E = 0 and its absolute source in the tail table. Before the tail's rounds its wave turns the tail's
// E entries into tail-table words (absolute sources, or kTailLit | byte), so the fill's common path
// serves the tail's sequences too.
struct LzState {
  uint16_t* e;
  uint32_t* tsrc;  // tail positions: absolute source, or kTailLit | the literal byte
};

__device__ __forceinline__ void put_lit(const LzState& S, int x, int v) { S.e[eph(x)] = (uint16_t)(0xFF00 | v); }

__device__ __forceinline__ void put_ptr(const LzState& S, int x, int src) {
  if (x - src < kTail) {
    S.e[eph(x)] = (uint16_t)(x - src);
  } else {
    S.e[eph(x)] = 0;
    S.tsrc[x - kTail] = (uint32_t)src;
  }
}

// value of output byte x once E and the tail table have converged (literal codes, or in E one hop
// from one)
__device__ __forceinline__ uint32_t lz_value(const LzState& S, int x) {
  if (x < kTail) {
    uint32_t e = S.e[eph(x)];
    if (e < (uint32_t)kTail) e = S.e[eph(x - (int)e)];  // class mode: one hop from the code
    return e & 0xFF;
  }
  return S.tsrc[x - kTail] & 0xFF;
}

// E entries of one sequence in the general form (out of line: the rare cases): literals that did not
// get a job (table full; read from the compressed block in HBM, `lit` = input offset) or whose
// bytes ride in `lv`, matches without a job, and tail matches at distances >= kTail.
__device__ __noinline__
void fill_general(uint16_t* e, uint32_t* tsrc, const uint8_t* __restrict__ gin, int o, int L, int M, int d,
                                          uint32_t lv, bool lit_inline, bool lit_here, bool match_here) {
  const LzState S{e, tsrc};
  if (lit_inline) {
    for (int k = 0; k < L; ++k) put_lit(S, o + k, (int)gld1(gin + lv + k));
  } else if (lit_here) {
    for (int k = 0; k < L; ++k) put_lit(S, o + k, (lv >> (8 * k)) & 0xFF);
  }
  if (match_here) {
    const int om = o + L;
    int r = 0;
    for (int k = 0; k < M; ++k) {
      put_ptr(S, om + k, (d >= M || d == kClass) ? om + k - d : om - d + r);
      if (++r == d) r = 0;
    }
  }
}

// max(v, v of the lane DPP control `ctrl` names), rows outside `rmask` and invalid lanes unchanged
template <int CTRL, int RMASK>
__device__ __forceinline__ uint32_t dpp_max_step(uint32_t old, uint32_t v) {
  return max(old, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RMASK, 0xf, false));
}

// inclusive max-scan over the 64 lanes of a wave: row shifts 1/2/4/8, then the row broadcasts of
// lanes 15 and 31 (no LDS round trips)
__device__ __forceinline__ uint32_t wave_max_scan(uint32_t v) {
  v = dpp_max_step<0x111, 0xf>(v, v);  // row_shr:1
  v = dpp_max_step<0x112, 0xf>(v, v);  // row_shr:2
  v = dpp_max_step<0x114, 0xf>(v, v);  // row_shr:4
  v = dpp_max_step<0x118, 0xf>(v, v);  // row_shr:8
  v = dpp_max_step<0x142, 0xa>(v, v);  // row_bcast:15 into rows 1, 3
  v = dpp_max_step<0x143, 0xc>(v, v);  // row_bcast:31 into rows 2, 3
  return v;
}

// Wave-aggregated slot allocation: each lane asking for n slots gets its first slot index.
__device__ __forceinline__ int wave_alloc(int* counter, int n) {
  const int incl = wave_add_scan(n);  // inclusive prefix of n over the lanes
  const int total = __builtin_amdgcn_readlane(incl, 63);
  int base = 0;
  if ((threadIdx.x & 63) == 63 && total) base = atomicAdd(counter, total);
  return __builtin_amdgcn_readlane(base, 63) + incl - n;
}

#ifndef DG_LZ_WAVE_STAMP
#define DG_LZ_WAVE_STAMP 3  // (diagnostic builds: the point whose per-wave times fill prof[16..31])
#endif
#define LZ_WAVE_STAMP(k)                                                                                  \
  do {                                                                                                    \
    if (PROF && DG_LZ_WAVE_STAMP == (k) && (tid & 63) == 0)                                               \
      prof[(size_t)blockIdx.x * kLz4ProfWords + 16 + (tid >> 6)] = __builtin_amdgcn_s_memtime();          \
  } while (0)

#define LZ_STAMP(k)                                                                           \
  do {                                                                                        \
    if (PROF && tid == 0) prof[(size_t)blockIdx.x * kLz4ProfWords + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// cooperative-copy job: x = output start | (len - 1) << 16, y = literal input offset (kind 0) or
// match distance | 1 << 31 (kind 1)
__device__ __forceinline__ int job_len(uint2 j) { return (int)(j.x >> 16) + 1; }

// Output of decoded bytes [16c, 16c + 16): a 16-byte store into a slot, or with job.vstride the two
// 8-byte values to their payload records (only values inside the block's expect_len), or with
// job.red_dst the two values folded into the thread's aggregate `acc` (nothing written)
// whether value v of a fused block folds: every row, or (a filtered scan) the row's bit in red_bits
__device__ __forceinline__ bool red_row(const Lz4Job& job, int v) {
  if (!job.red_bits) return true;
  const int64_t r = job.red_row0 + v;
  return (job.red_bits[r >> 5] >> (r & 31)) & 1u;
}

__device__ __forceinline__ void out16(const Lz4Job& job, int c, const uint32_t w[4], uint64_t& acc) {
  if (job.red_dst) {
    const int v = 2 * c;
    const bool has0 = (v + 1) * 8 <= job.expect_len && red_row(job, v),
               has1 = (v + 2) * 8 <= job.expect_len && red_row(job, v + 1);
    const uint64_t x0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), x1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
    switch (job.red_code) {
      case kRedLongSum:
        acc += (has0 ? x0 : 0) + (has1 ? x1 : 0);
        break;
      case kRedDoubleSum: {
        double a = __longlong_as_double((long long)acc);
        if (has0) a += __longlong_as_double((long long)x0);
        if (has1) a += __longlong_as_double((long long)x1);
        acc = (uint64_t)__double_as_longlong(a);
        break;
      }
      case kRedLongMax: {
        long long a = (long long)acc;
        if (has0) a = max(a, (long long)x0);
        if (has1) a = max(a, (long long)x1);
        acc = (uint64_t)a;
        break;
      }
      case kRedLongMin: {
        long long a = (long long)acc;
        if (has0) a = min(a, (long long)x0);
        if (has1) a = min(a, (long long)x1);
        acc = (uint64_t)a;
        break;
      }
      default:
        if (has0) acc = combine_op(job.red_op, acc, agg_input_raw(job.red_kind, job.red_vkind, x0));
        if (has1) acc = combine_op(job.red_op, acc, agg_input_raw(job.red_kind, job.red_vkind, x1));
    }
    return;
  }
  if (!job.vstride) {
    gst16(job.dst + 16 * (size_t)c, w[0], w[1], w[2], w[3]);
    return;
  }
  const int v = 2 * c;
  if ((v + 1) * 8 <= job.expect_len) gst8(job.dst + (size_t)v * job.vstride, w[0], w[1]);
  if ((v + 2) * 8 <= job.expect_len) gst8(job.dst + (size_t)(v + 1) * job.vstride, w[2], w[3]);
}

// decoded bytes [x, x + 4) (x % 4 == 0) as one dword store (same placement rules as out16)
__device__ __forceinline__ void out4(const Lz4Job& job, int x, uint32_t w) {
  if (!job.vstride) {
    gst4(job.dst + x, w);
    return;
  }
  if (((x >> 3) + 1) * 8 <= job.expect_len) gst4(job.dst + (size_t)(x >> 3) * job.vstride + (x & 7), w);
}

// the fold's starting value in the encoding out16 accumulates in (red_code)
__device__ __forceinline__ uint64_t red_identity(const Lz4Job& job) {
  switch (job.red_code) {
    case kRedLongSum:
    case kRedDoubleSum: return 0;
    case kRedLongMax: return (uint64_t)INT64_MIN;
    case kRedLongMin: return (uint64_t)INT64_MAX;
    default: return identity_of(job.red_op, job.red_kind);
  }
}

// The fused block's aggregate: the workgroup's per-thread values folded (wave shuffles, then one
// slot per wave in s_red) and combined into the bucket's slot with one atomic. Every thread calls it.
__device__ __forceinline__ void red_finish(const Lz4Job& job, uint64_t acc, uint64_t* s_red, int nwaves) {
  if (job.red_code == kRedLongMax || job.red_code == kRedLongMin) acc ^= kSign;  // -> the slot encoding
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
    acc = combine_op(job.red_op, acc, (uint64_t)__shfl_xor((unsigned long long)acc, o, 64));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s_red[w] = acc;
  __syncthreads();
  if (w == 0) {  // the waves' results folded by the first wave's lanes, one atomic
    const int l = threadIdx.x;
    // lanes past the waves: a copy of wave 0's value for min / max (idempotent), +0 for the sums (the
    // sums' identity in the slot encoding, like identity_of)
    uint64_t t = l < nwaves ? s_red[l] : (job.red_op == OP_ADD_I64 || job.red_op == OP_ADD_F64 ? 0ull : s_red[0]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
      t = combine_op(job.red_op, t, (uint64_t)__shfl_xor((unsigned long long)t, o, 64));
    if (l == 0) atomic_op(job.red_op, job.red_dst, t);
  }
}

// the job of launch block b: a per-block job, or its task's block with the task's destination and fold
__device__ __forceinline__ Lz4Job fetch_job(const Lz4Launch& L, int b) {
  if (b < L.njobs) return L.jobs[b];
  const int t = L.task_of[b - L.njobs];
  const Lz4Task& T = L.tasks[t];
  const int k = T.list[T.i0 + (b - L.task_first[t])];
  Lz4Job j = T.desc[k];
  j.dst = T.dst_base ? T.dst_base + (int64_t)k * T.dst_step : nullptr;
  j.vstride = T.vstride;
  j.red_dst = T.red_dst;
  j.red_op = T.red_op;
  j.red_kind = T.red_kind;
  j.red_vkind = T.red_vkind;
  j.red_code = T.red_code;
  j.red_bits = T.red_bits;
  j.red_row0 = (int64_t)k * T.red_rpb;
  return j;
}

template <bool PROF, int SEQ>
__global__ __launch_bounds__(kLzThreads) void k_lz4_decode(const Lz4Launch L, int32_t* __restrict__ err,
                                                           uint64_t* __restrict__ prof) {
  __shared__ __attribute__((aligned(16))) uint16_t s_e[kEWords];  // 130 KiB: staged input, then E
  __shared__ uint32_t s_tsrc[kTailN];
  __shared__ uint2 s_jobs_buf[kMaxJobs + kMaxJobs / 2];  // jobs, then their prefix sums; later the open list
  uint2* s_job = s_jobs_buf;
  int* s_jpre = reinterpret_cast<int*>(s_jobs_buf + kMaxJobs);
  __shared__ int s_njob, s_bad, s_c8, s_nopen;
  __shared__ int s_tmp[kLzWaves];
  __shared__ uint64_t s_red[kLzWaves];

  const Lz4Job job = fetch_job(L, blockIdx.x);
  const int tid = threadIdx.x;
  const int n = job.src_len, ncp = job.ncp;
  if (n <= 0 || n > kLz4InCap || ncp <= 0 || ncp > kLzMaxCps || job.dec_len > kBlockBytes ||
      job.dec_len < job.expect_len) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  LZ_STAMP(0);
  // my interval's token offsets, loaded with the staging (not after it)
  const int cp0 = tid < ncp ? (int)gld4(job.cp + tid) : 0;
  const int cp1 = tid + 1 < ncp ? (int)gld4(job.cp + tid + 1) : n;
  uint8_t* s_in = reinterpret_cast<uint8_t*>(s_e);
  uint32_t* s_e32 = reinterpret_cast<uint32_t*>(s_e);
  const LzState S{s_e, s_tsrc};
  // ---- stage the compressed block (16-byte aligned and padded in the device image) ----
  {
    uint4* dst = reinterpret_cast<uint4*>(s_in);
    const int n16 = (n + 15) >> 4;
    for (int i = tid; i < n16; i += kLzThreads) dst[i] = gld16(job.src + 16 * (size_t)i);
    if (tid == 0) {
      dst[n16] = make_uint4(0, 0, 0, 0);
      s_njob = 0;
      s_bad = 0;
      s_c8 = 0;
    }
  }
  __syncthreads();
  LZ_STAMP(1);
  // ---- 1. parse my interval (<= SEQ sequences: kLzSeqPerCp, or 2 * kLzSeqPerCp in a wide block)
  // into registers ----
  uint32_t r_L[SEQ], r_DM[SEQ], r_lv[SEQ];  // r_lv: literal bytes (L <= 4) or offset
  int cnt = 0, out_rel = 0;
  if (tid < ncp) {
    int pos = cp0;
    const int end = cp1;
#pragma unroll
    for (int s = 0; s < SEQ; ++s) {
      if (pos < end) {
        Tok t;
        if (parse_tok(s_in, n, pos, t)) {
          r_L[s] = (uint32_t)t.L;
          r_DM[s] = (uint32_t)t.off | ((uint32_t)t.M << 16);
          r_lv[s] = t.L <= kShortLit ? t.lv : (uint32_t)t.lit;
          out_rel += t.L + t.M;
          pos = t.next;
          cnt = s + 1;
        } else {
          pos = -1;
        }
      }
    }
    if (pos != end) s_bad = 1;
  }
  LZ_WAVE_STAMP(0);
  int total;
  const int base = block_scan_lz(out_rel, &total, s_tmp);  // its barriers end every read of s_in
  LZ_STAMP(2);
  if (s_bad || total != job.dec_len) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  // ---- 2. long runs (literals > kShortLit bytes, matches > kLongFill) become jobs; the jobs'
  // bytes form one flat range split evenly over the threads, and each thread reads the literal
  // bytes of its range from the staged input into registers before any E entry is written over it.
  // Then every thread writes the E entries of its own short runs (literal codes from the parse
  // registers, distances) and of its job range. ----
  const uint8_t* __restrict__ gin = job.src;
  constexpr uint32_t kInlineLit = 0x80000000u, kInlineMatch = 0x40000000u;  // r_L flags: job table full
  int c8 = 0;  // match bytes at distance 8 (class chains of 8-byte values, resolved by a scan below)
  {  // (every lane of the wave takes part: slot allocation is wave-aggregated)
    // my job slots: one wave-aggregated allocation for all my sequences (one LDS atomic per wave)
    int need = 0;
#pragma unroll
    for (int s = 0; s < SEQ; ++s)
      if (s < cnt) need += ((int)r_L[s] > kShortLit) + ((int)(r_DM[s] >> 16) > kLongFill);
    int j = __ballot(need) ? wave_alloc(&s_njob, need) : 0;
    int o = base;
#pragma unroll
    for (int s = 0; s < SEQ; ++s) {
      const bool act = s < cnt;  // (cnt = 0 beyond the checkpoints)
      const int L = act ? (int)r_L[s] : 0;
      const int d = (int)(r_DM[s] & 0xFFFF), M = act ? (int)(r_DM[s] >> 16) : 0;
      if (L > kShortLit) {
        if (j < kMaxJobs) s_job[j] = make_uint2((uint32_t)o | ((uint32_t)(L - 1) << 16), r_lv[s]);
        else r_L[s] |= kInlineLit;
        ++j;
      }
      if (M > kLongFill) {
        if (j < kMaxJobs) s_job[j] = make_uint2((uint32_t)(o + L) | ((uint32_t)(M - 1) << 16), (uint32_t)d | 0x80000000u);
        else r_L[s] |= kInlineMatch;
        ++j;
      }
      c8 += d == kClass ? M : 0;
      o += L + M;
    }
    for (int off = 32; off > 0; off >>= 1) c8 += __shfl_xor(c8, off, 64);  // wave sum, one LDS atomic
    if ((tid & 63) == 0 && c8) atomicAdd(&s_c8, c8);
  }
  LZ_WAVE_STAMP(1);
  __syncthreads();
  const int nj = min(s_njob, kMaxJobs);
  int tot = 0;
  if (nj > 0) {
    int l0 = 0, l1 = 0;
    if (2 * tid < nj) l0 = job_len(s_job[2 * tid]);
    if (2 * tid + 1 < nj) l1 = job_len(s_job[2 * tid + 1]);
    const int pre = block_scan_lz(l0 + l1, &tot, s_tmp);
    if (2 * tid < nj) s_jpre[2 * tid] = pre;
    if (2 * tid + 1 < nj) s_jpre[2 * tid + 1] = pre + l0;
    __syncthreads();
  }
  // my contiguous range of the flat job bytes (<= 64: jobs cover distinct output positions)
  const int per = (tot + kLzThreads - 1) / kLzThreads;
  const int g0 = tid * per, gend = min(g0 + per, tot);
  int j0 = 0;
  if (g0 < gend) {  // last job with s_jpre <= g0
    int lo = 0, hi = nj - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_jpre[mid] <= g0) lo = mid;
      else hi = mid - 1;
    }
    j0 = lo;
  }
  uint32_t lit4[16];  // the literal bytes of my range, four per register
#pragma unroll
  for (int q = 0; q < 16; ++q) lit4[q] = 0;
  // walk of my range over the jobs (jobs hold >= 5 bytes: at most one step per 4 positions)
  int wj = j0, wjs = 0, wje = 0;
  uint2 wjb = make_uint2(0, 0);
  auto walk_reset = [&]() {
    wj = j0;
    wjs = s_jpre[wj];
    wjb = s_job[wj];
    wje = wjs + job_len(wjb);
  };
  auto walk_to = [&](int pos) {
    if (pos >= wje) {
      ++wj;
      wjs = s_jpre[wj];
      wjb = s_job[wj];
      wje = wjs + job_len(wjb);
    }
  };
  if (g0 < gend) {
    walk_reset();
    const uint32_t* in32 = reinterpret_cast<const uint32_t*>(s_in);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int pq = g0 + 4 * q;
      if (pq < gend) {
        walk_to(pq);
        uint32_t w = 0;
        if (pq + 4 <= wje && pq + 4 <= gend) {  // four bytes of one job: one unaligned read
          if (!(wjb.y & 0x80000000u)) {
            const int src = (int)wjb.y + (pq - wjs);
            w = __builtin_amdgcn_alignbyte(in32[(src >> 2) + 1], in32[src >> 2], src & 3);
          }
        } else {
#pragma unroll 1
          for (int i = 0; i < 4; ++i) {
            if (pq + i < gend) {
              walk_to(pq + i);
              if (!(wjb.y & 0x80000000u)) w |= (uint32_t)s_in[wjb.y + (pq + i - wjs)] << (8 * i);
            }
          }
        }
        lit4[q] = w;
      }
    }
  }
  LZ_WAVE_STAMP(2);
  __syncthreads();  // every read of the staged input is done
  // class mode (mostly distance-8 matches): E starts as all 8, and the fill skips distance-8 matches
  const bool cls = s_c8 * 4 > total;
  if (cls) {
    uint4* e4 = reinterpret_cast<uint4*>(s_e);
    const uint4 eight = make_uint4(0x00080008u, 0x00080008u, 0x00080008u, 0x00080008u);
    for (int i = tid; i < kEWords / 8; i += kLzThreads) e4[i] = eight;
    __syncthreads();
  }
  LZ_STAMP(3);
  uint64_t tfg = 0;  // (PROF: cycles in fill_general)
  if (tid < ncp) {
    int o = base;
#pragma unroll
    for (int s = 0; s < SEQ; ++s) {
      if (s < cnt) {
        const uint32_t lf = r_L[s];
        const int L = (int)(lf & 0x3FFFFFFFu);
        const int d = (int)(r_DM[s] & 0xFFFF), M = (int)(r_DM[s] >> 16);
        // (a tail sequence's entries stay below kTail when d + M does: d * (1 + k / d) <= d + k)
        const bool fast = !(lf & (kInlineLit | kInlineMatch)) && (o + L + M <= kTail || d + M < kTail);
        if (fast) {  // the common case: plain E entries, no tail table
          if (L <= kShortLit) {
            const uint32_t lv = r_lv[s];
#pragma unroll
            for (int k = 0; k < kShortLit; ++k)
              if (k < L) S.e[eph(o + k)] = (uint16_t)(0xFF00u | ((lv >> (8 * k)) & 0xFFu));
          }
          if (M > 0 && M <= kLongFill && !(cls && d == kClass)) {
            const int om = o + L;
            if (d >= M || d == kClass) {  // one distance for the whole match (distance 8: class chains), by pairs
              int x = om;
              const int xe = om + M;
              if (x & 1) S.e[eph(x++)] = (uint16_t)d;
              const uint32_t dd = (uint32_t)d * 0x10001u;
              for (; x + 2 <= xe; x += 2) s_e32[eph(x) >> 1] = dd;
              if (x < xe) S.e[eph(x)] = (uint16_t)d;
            } else {  // overlapping: byte k copies the first period, distance d * (1 + k / d)
              int r = 0, dk = d;
              for (int k = 0; k < M; ++k) {
                S.e[eph(om + k)] = (uint16_t)dk;
                if (++r == d) { r = 0; dk += d; }
              }
            }
          }
        } else {
          const uint64_t tf0 = PROF ? __builtin_amdgcn_s_memtime() : 0;
          fill_general(s_e, s_tsrc, gin, o, L, M, d, r_lv[s], (lf & kInlineLit) != 0, L <= kShortLit,
                       (lf & kInlineMatch) != 0 || (M > 0 && M <= kLongFill));
          if (PROF) tfg += __builtin_amdgcn_s_memtime() - tf0;
        }
        o += L;
        if (M > 0) {
          if (d > o) s_bad = 1;
          o += M;
        }
      }
    }
  }
  LZ_WAVE_STAMP(3);
  if (PROF && tid == ncp - 1) prof[(size_t)blockIdx.x * kLz4ProfWords + 14] = tfg;
  if (g0 < gend) {  // my job range: literal codes from lit4, distances for long matches
    walk_reset();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int pq = g0 + 4 * q;
      if (pq < gend) {
        walk_to(pq);
        const int o = (int)(wjb.x & 0xFFFF), x = o + (pq - wjs);
        const bool lit = !(wjb.y & 0x80000000u);
        const int d = (int)(wjb.y & 0xFFFF), M = job_len(wjb);
        const bool flat = pq + 4 <= wje && pq + 4 <= gend && x + 4 <= kTail && (x & 127) <= 124;
        if (flat && lit) {  // four literal codes in one 128-entry skew span
          const uint32_t w = lit4[q];
          const uint32_t c01 = 0xFF00FF00u | (w & 0xFFu) | ((w & 0xFF00u) << 8);
          const uint32_t c23 = 0xFF00FF00u | ((w >> 16) & 0xFFu) | ((w >> 8) & 0xFF0000u);
          if (!(x & 1)) {
            s_e32[eph(x) >> 1] = c01;
            s_e32[(eph(x) >> 1) + 1] = c23;
          } else {
            S.e[eph(x)] = (uint16_t)c01;
            s_e32[(eph(x) + 1) >> 1] = (c01 >> 16) | (c23 << 16);
            S.e[eph(x) + 3] = (uint16_t)(c23 >> 16);
          }
        } else if (flat && (d >= M || d == kClass)) {  // four entries of one distance
          if (!(cls && d == kClass)) {
            const uint32_t dd = (uint32_t)d * 0x10001u;
            if (!(x & 1)) {
              s_e32[eph(x) >> 1] = dd;
              s_e32[(eph(x) >> 1) + 1] = dd;
            } else {
              S.e[eph(x)] = (uint16_t)d;
              s_e32[(eph(x) + 1) >> 1] = dd;
              S.e[eph(x) + 3] = (uint16_t)d;
            }
          }
        } else {
#pragma unroll 1
          for (int i = 0; i < 4; ++i) {
            if (pq + i < gend) {
              walk_to(pq + i);
              const int k = pq + i - wjs, oo = (int)(wjb.x & 0xFFFF);
              if (wjb.y & 0x80000000u) {
                const int dj = (int)(wjb.y & 0xFFFF);
                put_ptr(S, oo + k, (dj >= job_len(wjb) || dj == kClass) ? oo + k - dj : oo - dj + k % dj);
              } else {
                put_lit(S, oo + k, (lit4[q] >> (8 * i)) & 0xFF);
              }
            }
          }
        }
      }
    }
  }
  __syncthreads();
  if (s_bad) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  LZ_STAMP(4);
  // ---- 3. resolution over positions [0, min(total, kTail)). Every E entry is a literal code or a
  // distance to an earlier byte of the same value; jumping (E[x] += E[x - E[x]], or the target's
  // code once it is a literal) rewrites distances until only literal codes remain.
  //
  // Class mode: a byte copied from 8 back (E == 8) has the value of the last byte before it in its
  // residue class mod 8 whose entry is not 8 (its "terminal"). Value columns of 8-byte values
  // (sequential longs, timestamps) are ~99 % distance-8 matches chaining through the whole block; in
  // such blocks a carry scan gives every E == 8 entry the distance to its terminal and lists the
  // terminals that are still distances (the few matches at other distances). Jumping over that list
  // resolves the terminals (through the scanned entries, one hop per class chain), and one final
  // sweep gives every scanned entry its terminal's code.
  //
  // Otherwise: wave w sweeps its own 4 KiB of positions in increasing order, so a position sees the
  // updates of the earlier batches of its wave (LDS ops of one wave complete in order); the pairs
  // still open after that first sweep are listed and later rounds only visit the list. Both lists
  // live in the job tables' space; on overflow the rounds fall back to full sweeps. ----
  const int lim = min(total, kTail);
  // positions in [lim, kTail) act as resolved literals
  if (lim < kTail) {
    for (int x = lim + tid; x < kTail; x += kLzThreads) s_e[eph(x)] = 0xFF00;
  }
  uint16_t* s_open = reinterpret_cast<uint16_t*>(s_job);  // pair indices, or positions in class mode
  constexpr int kOpenCap = (kMaxJobs + kMaxJobs / 2) * (int)sizeof(uint2) / 2;
  __shared__ uint32_t s_scan[kLzWaves * kClass];
  if (tid == 0) s_nopen = 0;
  __syncthreads();
  const int wv = tid >> 6, ln = tid & 63;
  auto is_open = [](uint32_t v) { return (v & 0xFFFF) < (uint32_t)kTail || (v >> 16) < (uint32_t)kTail; };
  // one jump step for an entry d whose target holds e
  auto jstep = [](uint32_t d, uint32_t e) -> uint32_t {
    return d >= (uint32_t)kTail ? d : (e >= (uint32_t)kTail ? e : d + e);
  };
  // full sweep of my wave's region, one step per open entry (the class scan's fallback when its list of
  // open terminals overflows). Returns whether any of my entries is still open.
  uint32_t* s_obits = reinterpret_cast<uint32_t*>(s_jobs_buf);  // kBlockBytes / 2 bits (non-class mode)
  auto sweep = [&]() -> bool {
    bool any = false;
#pragma unroll 1
    for (int b = 0; b < kPairs / kJumpBatch; ++b) {
      const int j0 = b * kJumpBatch;
      uint32_t dv[kJumpBatch], ta[kJumpBatch], tb[kJumpBatch];
      bool need = false;
#pragma unroll
      for (int k = 0; k < kJumpBatch; ++k) {
        const int x = 2 * (wv * (kPairs * 64) + (j0 + k) * 64 + ln);
        dv[k] = x < kTail ? s_e32[eph(x) >> 1] : 0xFF00FF00u;
        need |= is_open(dv[k]);
      }
      if (__ballot(need) == 0) continue;
#pragma unroll
      for (int k = 0; k < kJumpBatch; ++k) {
        const int x = 2 * (wv * (kPairs * 64) + (j0 + k) * 64 + ln);
        const uint32_t d0 = dv[k] & 0xFFFF, d1 = dv[k] >> 16;
        ta[k] = d0 < (uint32_t)kTail ? s_e[eph(x - (int)d0)] : 0xFF00u;
        tb[k] = d1 < (uint32_t)kTail ? s_e[eph(x + 1 - (int)d1)] : 0xFF00u;
      }
#pragma unroll
      for (int k = 0; k < kJumpBatch; ++k) {
        const int x = 2 * (wv * (kPairs * 64) + (j0 + k) * 64 + ln);
        const uint32_t nv = jstep(dv[k] & 0xFFFF, ta[k]) | (jstep(dv[k] >> 16, tb[k]) << 16);
        if (nv != dv[k]) s_e32[eph(x) >> 1] = nv;
        any |= is_open(nv);
      }
    }
    return any;
  };
  // Staged resolution in position order: stage s takes the kLzThreads pairs after stage s - 1, all
  // of whose entries are literal codes by then, so a target before the stage is one read from its
  // code. A target inside the stage (distance < the stage) is followed for up to kStageSteps more
  // jumps (no barrier: entries only ever get closer to their code, so any value read is valid); pairs
  // still open are set in the open-pair bitmap for the rounds below. One barrier per stage.
  auto staged = [&]() -> bool {
    constexpr int kSK = DG_LZ_STAGE_K;  // pairs per thread per stage
    constexpr int kStage = kSK * kLzThreads;  // pairs per stage
    constexpr int kStageSteps = DG_LZ_STAGE_STEPS;
    const int npairs = (lim + 1) >> 1;
    bool any = false;
#pragma unroll 1
    for (int p0 = 0; p0 < npairs; p0 += kStage) {
      uint32_t v[kSK], nv[kSK];
#pragma unroll
      for (int k = 0; k < kSK; ++k) {
        const int x = 2 * (p0 + k * kLzThreads + tid);
        v[k] = x < kTail ? s_e32[eph(x) >> 1] : 0xFF00FF00u;
        nv[k] = v[k];
      }
#pragma unroll 1
      for (int it = 0; it <= kStageSteps; ++it) {
        uint32_t ta[kSK], tb[kSK];
#pragma unroll
        for (int k = 0; k < kSK; ++k) {
          const int x = 2 * (p0 + k * kLzThreads + tid);
          const uint32_t d0 = nv[k] & 0xFFFF, d1 = nv[k] >> 16;
          ta[k] = d0 < (uint32_t)kTail ? s_e[eph(x - (int)d0)] : 0xFF00u;
          tb[k] = d1 < (uint32_t)kTail ? s_e[eph(x + 1 - (int)d1)] : 0xFF00u;
        }
        bool open = false;
#pragma unroll
        for (int k = 0; k < kSK; ++k) {
          nv[k] = jstep(nv[k] & 0xFFFF, ta[k]) | (jstep(nv[k] >> 16, tb[k]) << 16);
          open |= is_open(nv[k]);
        }
        if (!__ballot(open)) break;
      }
#pragma unroll
      for (int k = 0; k < kSK; ++k) {
        const int x = 2 * (p0 + k * kLzThreads + tid);
        if (nv[k] != v[k]) s_e32[eph(x) >> 1] = nv[k];  // (x < kTail whenever an entry changes)
        const bool op = is_open(nv[k]);
        any |= op;
        const uint64_t bal = __ballot(op);  // 64 consecutive pairs: two bitmap words
        const int w0 = (p0 + k * kLzThreads + wv * 64) >> 5;
        if (ln == 0) s_obits[w0] = (uint32_t)bal;
        if (ln == 32) s_obits[w0 + 1] = (uint32_t)(bal >> 32);
      }
      __syncthreads();
    }
    // bitmap words past the last stage: nothing open
    for (int w = ((npairs + kStage - 1) / kStage) * (kStage / 32) + tid; w < kLzThreads; w += kLzThreads) s_obits[w] = 0u;
    return any;
  };
  int jump_rounds = 0;
  if (cls) {
    // carry scan over my 64 positions [tid * 64, tid * 64 + 64). A terminal travels as key
    // (position + 1) << 16 | its entry (0 = none yet); an E == 8 entry takes the terminal's literal
    // code, or the distance to the terminal while that is still open.
    const int x0 = tid * 64;
    // my 64 positions lie in one skew span (64 | 128): pair q is dword eb + q of E
    const int eb = (x0 >> 1) + (x0 >> kESkewShift);
    auto pair_at = [&](int q) { return x0 + 2 * q < lim ? s_e32[eb + q] : 0xFF00FF00u; };
    uint32_t last[kClass];
#pragma unroll
    for (int c = 0; c < kClass; ++c) last[c] = 0;
#pragma unroll 1
    for (int q0 = 0; q0 < 32; q0 += 4) {  // 4 pairs (one residue-class period) per step
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = q0 + j, c = 2 * j;
        const uint32_t v = pair_at(q);
        if ((v & 0xFFFF) != (uint32_t)kClass) last[c] = ((uint32_t)(x0 + 2 * q + 1) << 16) | (v & 0xFFFF);
        if ((v >> 16) != (uint32_t)kClass) last[c + 1] = ((uint32_t)(x0 + 2 * q + 2) << 16) | (v >> 16);
      }
    }
    uint32_t carry[kClass];
#pragma unroll
    for (int c = 0; c < kClass; ++c) {  // exclusive max-scan over the threads (positions grow with tid)
      const uint32_t v = wave_max_scan(last[c]);
      carry[c] = dpp_max_step<0x138, 0xf>(0u, v);  // wave_shr:1 (lane 0 gets 0)
      if (ln == 63) s_scan[wv * kClass + c] = v;
    }
    __syncthreads();
    LZ_STAMP(12);
    {  // the earlier waves' totals: lane l reads class l % 8 of waves l / 8 and 8 + l / 8, then a
       // max over the lanes of one class; no loop of dependent LDS reads
      static_assert(kLzWaves == 16 && kClass == 8, "s_scan = two entries per lane");
      uint32_t v = max((ln >> 3) < wv ? s_scan[ln] : 0u, 8 + (ln >> 3) < wv ? s_scan[64 + ln] : 0u);
      v = max(v, (uint32_t)__shfl_xor((int)v, 8, 64));
      v = max(v, (uint32_t)__shfl_xor((int)v, 16, 64));
      v = max(v, (uint32_t)__shfl_xor((int)v, 32, 64));
#pragma unroll
      for (int c = 0; c < kClass; ++c) carry[c] = max(carry[c], (uint32_t)__builtin_amdgcn_readlane((int)v, c));
    }
    uint64_t omask = 0;  // my open terminals (bit = position - x0)
    auto take = [](uint32_t key, int x) -> uint32_t {  // new entry of a distance-8 byte at x
      const uint32_t tv = key & 0xFFFF;
      return tv >= (uint32_t)kTail ? tv : (uint32_t)(x + 1) - (key >> 16);
    };
#pragma unroll 1
    for (int q0 = 0; q0 < 32; q0 += 4)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = q0 + j, c = 2 * j, x = x0 + 2 * q;
      const uint32_t v = pair_at(q);
      uint32_t lo = v & 0xFFFF, hi = v >> 16;
      const bool t0 = lo != (uint32_t)kClass, t1 = hi != (uint32_t)kClass;
      if (!t0) {
        if (carry[c]) lo = take(carry[c], x);
      } else {
        carry[c] = ((uint32_t)(x + 1) << 16) | lo;
      }
      if (!t1) {
        if (carry[c + 1]) hi = take(carry[c + 1], x + 1);
      } else {
        carry[c + 1] = ((uint32_t)(x + 2) << 16) | hi;
      }
      const uint32_t nv = lo | (hi << 16);
      if (nv != v) s_e32[eb + q] = nv;  // x < lim whenever an entry changes
      omask |= (uint64_t)(t0 && lo < (uint32_t)kTail) << (2 * q);  // open terminals
      omask |= (uint64_t)(t1 && hi < (uint32_t)kTail) << (2 * q + 1);
    }
    {
      const int nm = __popcll(omask);
      if (__ballot(nm)) {
        int at = wave_alloc(&s_nopen, nm);
        for (; omask; omask &= omask - 1, ++at)
          if (at < kOpenCap) s_open[at] = (uint16_t)(x0 + __builtin_ctzll(omask));
      }
    }
    LZ_WAVE_STAMP(4);
    __syncthreads();
    LZ_STAMP(13);
    const int no = s_nopen;
    if (no <= kOpenCap) {
      // terminal rounds over the list, then one sweep: every scanned entry reads its terminal's code
      for (int round = 0;; ++round) {
        if (round > kMaxRounds) {  // unreachable for a valid block
          if (tid == 0) atomicOr(err, 1);
          return;
        }
        jump_rounds++;
        bool any = false;
        for (int i = tid; i < no; i += kLzThreads) {
          const int x = s_open[i];
          const uint32_t d = s_e[eph(x)];
          if (d < (uint32_t)kTail) {
            const uint32_t nd = jstep(d, s_e[eph(x - (int)d)]);
            s_e[eph(x)] = (uint16_t)nd;
            any |= nd < (uint32_t)kTail;
          }
        }
        if (!__syncthreads_or(any)) break;
      }
      // every scanned entry now holds a code or the distance to a terminal that holds one: the tail
      // and the output take that last hop themselves (final_code)
    } else {
      for (int round = 0; __syncthreads_or(sweep()); ++round) {
        jump_rounds++;
        if (round > kMaxRounds) {
          if (tid == 0) atomicOr(err, 1);
          return;
        }
      }
    }
  } else {
    jump_rounds = 1;
    const bool open1 = __syncthreads_or(staged());
    LZ_STAMP(12);
    LZ_STAMP(13);
    if (open1) {
      // later rounds: thread t takes bitmap word t (pairs 32t .. 32t + 31) and steps its open pairs
      uint32_t m = s_obits[tid];
      int cnt_open = __popc(m);
      for (int round = 1;; ++round) {
        if (round > kMaxRounds) {  // unreachable for a valid block
          if (tid == 0) atomicOr(err, 1);
          return;
        }
        jump_rounds++;
        // four open pairs per step, their reads issued together (a step may read a pair another
        // step of this round already advanced: jumping only converges faster)
        uint32_t keep = 0, mm = m;
        const int xb = 64 * tid, eb = eph(xb) >> 1;  // my 64 positions lie in one skew span
        while (mm) {
          int bit[4];
          uint32_t v[4], e0[4], e1[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            bit[k] = mm ? __builtin_ctz(mm) : -1;
            mm &= mm - 1;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] = bit[k] >= 0 ? s_e32[eb + bit[k]] : 0xFF00FF00u;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int x = xb + 2 * bit[k];
            const uint32_t d0 = v[k] & 0xFFFF, d1 = v[k] >> 16;
            e0[k] = d0 < (uint32_t)kTail ? s_e[eph(x - (int)d0)] : 0xFF00u;
            e1[k] = d1 < (uint32_t)kTail ? s_e[eph(x + 1 - (int)d1)] : 0xFF00u;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t nv = jstep(v[k] & 0xFFFF, e0[k]) | (jstep(v[k] >> 16, e1[k]) << 16);
            if (nv != v[k]) s_e32[eb + bit[k]] = nv;  // (bit < 0: v is two codes, unchanged)
            if (bit[k] >= 0 && is_open(nv)) keep |= 1u << bit[k];
          }
        }
        m = keep;
        if (!__syncthreads_or(m != 0)) break;
      }
      if (PROF && cnt_open) atomicAdd(&s_nopen, cnt_open);  // (unused otherwise in this mode)
    }
  }
  __syncthreads();
  if (PROF && tid == 0) prof[(size_t)blockIdx.x * kLz4ProfWords + 7] = (uint64_t)s_nopen;
  LZ_STAMP(5);
  if (PROF && tid == 0) {
    prof[(size_t)blockIdx.x * kLz4ProfWords + 8] = (uint64_t)jump_rounds;
    prof[(size_t)blockIdx.x * kLz4ProfWords + 9] = (uint64_t)n;
    prof[(size_t)blockIdx.x * kLz4ProfWords + 10] = (uint64_t)nj;
    prof[(size_t)blockIdx.x * kLz4ProfWords + 11] = (uint64_t)ncp;
  }
  // the literal code of position y < kTail: E holds it, or (class mode) the distance to a byte that does
  auto final_code = [&](int y) -> uint32_t {
    uint32_t e = s_e[eph(y)];
    if (e < (uint32_t)kTail) e = s_e[eph(y - (int)e)];
    return e;
  };
  // ---- tail: positions [kTail, total) hold absolute sources. The last wave alone jumps over the
  // table (its LDS ops complete in order, so a round's reads precede its writes without a barrier)
  // while the other waves write the chunks below kTail; the tail's chunks follow one barrier. ----
  const int nchunks = (total + 15) >> 4;
  const bool has_tail = total > kTail;
  const int nbody = has_tail ? (kTail >> 4) : nchunks;  // chunks below kTail (kTail % 16 == 0)
  uint64_t racc = job.red_dst ? red_identity(job) : 0ull;
  auto out_chunk = [&](int c) {
    const int x0 = c << 4;
    uint32_t w[4];
    if (x0 + 16 <= lim) {
      const uint32_t* ep = s_e32 + (eph(x0) >> 1);
      uint32_t e[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) e[q] = ep[q];
      const uint32_t all = e[0] & e[1] & e[2] & e[3] & e[4] & e[5] & e[6] & e[7];
      if ((all & 0xFF00FF00u) != 0xFF00FF00u) {  // class mode: entries one hop from their code
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          uint32_t lo = e[q] & 0xFFFF, hi = e[q] >> 16;
          if (lo < (uint32_t)kTail) lo = s_e[eph(x0 + 2 * q - (int)lo)];
          if (hi < (uint32_t)kTail) hi = s_e[eph(x0 + 2 * q + 1 - (int)hi)];
          e[q] = lo | (hi << 16);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t e0 = e[2 * q], e1 = e[2 * q + 1];
        w[q] = (e0 & 0xFF) | ((e0 >> 8) & 0xFF00) | ((e1 & 0xFF) << 16) | ((e1 & 0xFF0000) << 8);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t acc = 0;
        for (int i = 0; i < 4; ++i) {
          const int x = x0 + 4 * q + i;
          if (x < total) acc |= lz_value(S, x) << (8 * i);
        }
        w[q] = acc;
      }
    }
    out16(job, c, w, racc);
  };
  if (has_tail && wv == kLzWaves - 1) {
    const int nt = total - kTail;
    auto lit_at = [&](int i) { return s_tsrc[i] >> 16; };
    uint32_t act = 0;  // bit k: position ln + 64 k still a source
#pragma unroll
    for (int k = 0; k < kTailN / 64; ++k) {  // the tail's E entries -> tail-table words
      const int i = ln + 64 * k;
      if (i < nt) {
        const uint32_t e = s_e[eph(kTail + i)];
        if (e >= (uint32_t)kTail) s_tsrc[i] = kTailLit | (e & 0xFFu);
        else if (e) s_tsrc[i] = (uint32_t)(kTail + i - (int)e);
      }
    }
#pragma unroll
    for (int k = 0; k < kTailN / 64; ++k) {
      const int i = ln + 64 * k;
      if (i < nt && !lit_at(i)) act |= 1u << k;
    }
    for (int round = 0; __ballot(act != 0); ++round) {
      if (round > 10) {  // 256 positions: 9 rounds suffice
        s_bad = 1;
        break;
      }
      uint32_t nsrc[kTailN / 64], res = 0;
#pragma unroll
      for (int k = 0; k < kTailN / 64; ++k) {
        nsrc[k] = 0;
        if ((act >> k) & 1u) {
          const int src = s_tsrc[ln + 64 * k];
          if (src < kTail) {
            nsrc[k] = kTailLit | (final_code(src) & 0xFFu);
            res |= 1u << k;
          } else {
            nsrc[k] = s_tsrc[src - kTail];  // a flagged literal, or its source
            res |= (nsrc[k] >> 16) << k;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < kTailN / 64; ++k) {
        if ((act >> k) & 1u) s_tsrc[ln + 64 * k] = nsrc[k];
      }
      act &= ~res;
    }
  }
  if (!(has_tail && wv == kLzWaves - 1)) {
    // ---- 4. output: every entry is a literal code or one hop from one; 16 bytes per 16-byte store ----
    const int nthr = has_tail ? kLzThreads - 64 : kLzThreads;
    for (int c = tid; c < nbody; c += nthr) out_chunk(c);
  }
  LZ_WAVE_STAMP(5);
  if (has_tail) {
    __syncthreads();
    if (s_bad) {
      if (tid == 0) atomicOr(err, 1);
      return;
    }
    for (int c = nbody + tid; c < nchunks; c += kLzThreads) out_chunk(c);
  }
  if (job.red_dst) red_finish(job, racc, s_red, kLzWaves);
  if (PROF) {
    __syncthreads();
    LZ_STAMP(6);
  }
}

// ------------------------------------------------------------------------------------------------
// Flow decoder: general blocks of at most 8,192 sequences that are not distance-8 class chains and
// whose copy chains are at most kFlowMaxDepth hops deep (attach-time classification, lz4_index_block):
// the literal-heavy, short-match blocks of noisy doubles (~7,500 sequences of ~5 literal bytes and a
// 4-byte copy from ~5 KiB back), zipfian doubles and uniform longs. k_lz4_decode spends most of its time
// on per-byte entries (write 64 K of them, then resolve them all in position-ordered stages); here the
// workgroup decodes straight into the block's byte image in LDS, in the order of the attach-time
// schedule (lz4_flow_schedule: a match whose source lies inside one earlier match's output copies from
// that match's source instead — forwarded distance; its level is one more than the highest level among
// the bytes it copies, literal bytes are level 0; every match has its rank in (level, position) order):
//   1. stage + parse + scan as in k_lz4_decode (every thread: one checkpoint interval in registers) and
//      zero the image;
//   2. level 0: every thread ORs its literal runs of up to 8 bytes into the image from its parse
//      registers; every 16-byte piece of a longer run is a job, and thread t then copies job t from the
//      staged input;
//   3. the staged input is dead: every thread writes its matches (start, forwarded distance, length)
//      into a table over it, at their ranks — each level's matches are then one contiguous range;
//   4. levels 1 .. nlvl, one barrier each: thread t copies matches t, t + 1024, ... of the level's range
//      (their sources are complete);
//   5. output: 16-byte chunks of the image, coalesced stores (or out16's payload / fused paths).
// A copy reads its source dwords (one more than the destination dwords it covers) and funnels them to
// the destination's alignment; whole destination dwords are plain stores, the partial ones at its ends
// LDS atomic ORs into the zeroed image (a neighbouring run owns the other bytes). LDS: staged input
// (later the match table) 66 KiB + image 64 KiB + literal jobs 8 KiB: one block per CU, like
// k_lz4_decode.
// ------------------------------------------------------------------------------------------------
constexpr int kFlowJobs = 1024;     // literal-run jobs per block (one per thread)
constexpr int kFlowRegLit = 8;      // literal runs up to this ride in the parse registers; longer ones are jobs
constexpr int kFlowPad = 4;         // dwords before the staged input and the image: a copy's first
                                    // source dword may start up to 3 bytes before its source
constexpr int kFlowInWords = kFlowPad + (kLz4InCap + 32) / 4 + 8;  // (+ the unconditional reads past a copy)
constexpr int kFlowOutWords = kFlowPad + kBlockBytes / 4 + 8;
constexpr int kFlowMaxMatches = kLzMaxCps * kLzSeqPerCp;  // the match table's rows (over the staged input)
static_assert(kFlowMaxMatches * 8 <= kFlowInWords * 4, "the match table fits the staged input");

__device__ __forceinline__ void lds_or(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t lds_ld8(const uint32_t* a, int p) {
  return reinterpret_cast<const uint8_t*>(a + kFlowPad)[p];
}

// the byte mask of destination dword t (0 .. NJ - 1) of a run [dst, dst + len) whose first dword is
// dst >> 2: its bytes below the run's end (k = the run's end - 4t, clamped to 0 .. 4), and in dword 0 from
// the run's start
__device__ __forceinline__ uint32_t run_mask(int t, int dst, int len) {
  const int k = min(max((dst & 3) + len - 4 * t, 0), 4);
  const uint32_t m = (uint32_t)((1ull << (8 * k)) - 1ull);
  return t == 0 ? m & (0xFFFFFFFFu << (8 * (dst & 3))) : m;
}

// bytes [dst, dst + len) of the image o32 <- bytes [src, src + len) of i32 (padded LDS byte arrays,
// 1 <= len <= 4 * (NJ - 1) + 1): NJ + 1 source dwords, then NJ masked ORs into the destination dwords
// (nothing past the copy's end), all unconditional — one LDS round trip. Inside one array the source
// must end before the destination starts (it is read before anything is written).
template <int NJ>
__device__ __forceinline__ void flow_copyn(uint32_t* o32, int dst, const uint32_t* i32, int src, int len) {
  const int j0 = dst >> 2;
  const int q0 = 4 * j0 + (src - dst) + 4 * kFlowPad;  // padded offset of dword j0's first source byte
  const int k0 = q0 >> 2, sh = q0 & 3;
  uint32_t sw[NJ + 1];
#pragma unroll
  for (int t = 0; t <= NJ; ++t) sw[t] = i32[k0 + t];
#pragma unroll
  for (int t = 0; t < NJ; ++t)
    lds_or(o32 + kFlowPad + j0 + t, __builtin_amdgcn_alignbyte(sw[t + 1], sw[t], sh) & run_mask(t, dst, len));
}

// the first min(M, 16) bytes of an overlapping match (d < 16, d < M): out[om + k] = out[om - d + k mod d].
// A period dividing 8 (the common ones: byte runs, repeated 8-byte values) is read as 8 bytes and
// doubled in a register; other periods are gathered byte by byte.
__device__ __forceinline__ void flow_head(uint32_t* o32, int om, int d, int M) {
  const int h = min(M, 16);
  uint32_t v[4];  // the head's bytes, little-endian
  if (d <= 8 && (d & (d - 1)) == 0) {
    const int q = om - d + 4 * kFlowPad, k = q >> 2, sh = q & 3;
    const uint32_t w0 = o32[k], w1 = o32[k + 1], w2 = o32[k + 2];
    uint64_t x = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    x = d == 8 ? x : (x & ((1ull << (8 * d)) - 1));
    for (int per = d; per < 8; per <<= 1) x |= x << (8 * per);
    v[0] = v[2] = (uint32_t)x;
    v[1] = v[3] = (uint32_t)(x >> 32);
  } else {
    v[0] = v[1] = v[2] = v[3] = 0u;
    int r = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      v[k >> 2] |= lds_ld8(o32, om - d + r) << (8 * (k & 3));
      if (++r == d) r = 0;
    }
  }
  const int a = om & 3, j0 = om >> 2;
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const uint32_t lo = t > 0 ? v[t - 1] : 0u, hi = t < 4 ? v[t] : 0u;
    const uint32_t w = a == 0 ? hi : __builtin_amdgcn_alignbyte(hi, lo, 4 - a);  // bytes 4t - a ..
    lds_or(o32 + kFlowPad + j0 + t, w & run_mask(t, om, h));
  }
}

// one match (its source complete) in 16-byte pieces: the first piece a plain copy from d back (or, when
// it overlaps itself, the gathered head), every later piece a plain copy from D back, D the first
// multiple of d of at least 16 bytes (the bytes repeat with period d, and a piece's source ends before
// it starts). Pieces in order: a piece may read what the earlier ones wrote.
__device__ __forceinline__ void flow_match(uint32_t* o32, int om, int d, int M) {
  if (d >= min(M, 16)) flow_copyn<5>(o32, om, o32, om - d, min(M, 16));
  else flow_head(o32, om, d, M);
  if (M > 16) {
    int D = d;
    while (D < 16) D += d;
#pragma unroll 1
    for (int k = 16; k < M; k += 16) flow_copyn<5>(o32, om + k, o32, om + k - D, min(16, M - k));
  }
}

// a copy of any length from the staged input (16-byte pieces)
__device__ __forceinline__ void flow_copy(uint32_t* o32, int dst, const uint32_t* i32, int src, int len) {
#pragma unroll 1
  for (int k = 0; k < len; k += 16) flow_copyn<5>(o32, dst + k, i32, src + k, min(16, len - k));
}

// The flow decoder's parse: one 20-byte window (five aligned dword reads, one LDS round trip) holds a
// token, its literal length extension byte, up to 8 literal bytes (they ride along in lv / lv_hi) and,
// for runs of up to 14 bytes, the distance; a distance or match length extension byte past the window
// is one more read. Only an extension of 255 or more (a run or match of 270+ bytes) takes the byte-wise
// parse_tok_slow.
__device__ __forceinline__ uint32_t lds_byte(const uint32_t* in32, int q) { return (in32[q >> 2] >> (8 * (q & 3))) & 0xFFu; }

__device__ __forceinline__ bool parse_tok8(const uint8_t* __restrict__ in, int n, int p, Tok& t, uint32_t& lv_hi) {
  if (p >= n) return false;
  const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in);
  auto word = [&](int i) -> uint32_t { return in32[i]; };
  auto byte = [&](int q) -> uint32_t { return lds_byte(in32, q); };
  const int a = p >> 2, sh = p & 3;
  const uint32_t d0 = word(a), d1 = word(a + 1), d2 = word(a + 2), d3 = word(a + 3), d4 = word(a + 4);
  const uint32_t b0 = __builtin_amdgcn_alignbyte(d1, d0, sh), b1 = __builtin_amdgcn_alignbyte(d2, d1, sh),
                 b2 = __builtin_amdgcn_alignbyte(d3, d2, sh), b3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
  // bytes p .. p + 15 as b0..b3 (the 17th byte, p + 16, is not needed from the window)
  const int tk = (int)(b0 & 0xFF);
  int L = tk >> 4, M = tk & 15;
  lv_hi = __builtin_amdgcn_alignbyte(b2, b1, 1);  // bytes 5 .. 8
  t.lv = __builtin_amdgcn_alignbyte(b1, b0, 1);   // bytes 1 .. 4
  int q = p + 1;
  if (L == 15) {
    const int e = (int)((b0 >> 8) & 0xFF);
    if (e == 255) return parse_tok_slow(in, n, p, t);
    L += e;
    q = p + 2;
  }
  t.lit = q;
  t.L = L;
  q += L;
  if (q > n) return false;
  if (q == n) {
    t.off = 0;
    t.M = 0;
    t.next = n;
    return true;
  }
  if (q + 2 > n) return false;
  const int k = q - p;  // the distance: window bytes k, k + 1
  int off;
  if (k <= 14) {
    const uint64_t lo = (uint64_t)b0 | ((uint64_t)b1 << 32), hi = (uint64_t)b2 | ((uint64_t)b3 << 32);
    off = (int)((k <= 6 ? lo >> (8 * k) : k < 8 ? (lo >> (8 * k)) | (hi << (64 - 8 * k)) : hi >> (8 * (k - 8))) & 0xFFFF);
  } else {
    off = (int)(byte(q) | (byte(q + 1) << 8));
  }
  q += 2;
  if (M == 15) {
    if (q >= n) return false;
    const int e = (int)byte(q);
    if (e == 255) {
      const uint32_t lv = t.lv;
      const bool ok = parse_tok_slow(in, n, p, t);
      t.lv = lv;  // (parse_tok_slow keeps only runs of <= 4 literal bytes)
      return ok;
    }
    M += e;
    q += 1;
  }
  t.off = off;
  t.M = M + 4;
  t.next = q;
  return off != 0;
}

template <bool PROF>
__global__ __launch_bounds__(kLzThreads) void k_lz4_decode_flow(const Lz4Launch L, int32_t* __restrict__ err,
                                                                uint64_t* __restrict__ prof, int nblocks) {
  constexpr int SEQ = kLzSeqPerCp;
  __shared__ __attribute__((aligned(16))) uint32_t s_in32[kFlowInWords];    // staged input (after the pad)
  __shared__ __attribute__((aligned(16))) uint32_t s_out32[kFlowOutWords];  // the decoded image (after the pad)
  __shared__ uint2 s_job[kFlowJobs];  // literal runs past the registers: output start | (L - 1) << 16, input offset
  __shared__ int s_lvl[kFlowMaxDepth + 1];  // s_lvl[k - 1] .. s_lvl[k]: the table rows of level k
  __shared__ int s_njob, s_bad;
  __shared__ int s_tmp[kLzWaves];
  __shared__ uint64_t s_red[kLzWaves];
  uint2* s_tab = reinterpret_cast<uint2*>(s_in32);  // the match table, after the literals

  // a grid smaller than the launch's blocks is persistent: workgroup w decodes blocks w, w + grid, ...
  // and keeps its CU (and its 139 KiB of LDS) for the whole launch
#pragma unroll 1
  for (int blk = blockIdx.x; blk < nblocks; blk += gridDim.x) {
  if (blk != (int)blockIdx.x) __syncthreads();  // the previous block's output has left the image
  const Lz4Job job = fetch_job(L, blk);
  const int tid = threadIdx.x;
  const int n = job.src_len, ncp = job.ncp;
  if (n <= 0 || n > kLz4InCap || ncp <= 0 || ncp > kLzMaxCps || job.dec_len > kBlockBytes ||
      job.dec_len < job.expect_len || !job.lvl || job.nlvl < 0 || job.nlvl > kFlowMaxDepth) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  LZ_STAMP(0);
  const uint8_t* s_in = reinterpret_cast<const uint8_t*>(s_in32 + kFlowPad);
  // my matches' table rows (u16 each, 0xFFFF: none) and the levels' row ranges
  // my interval's schedule (match ranks, forwarded distances, token offsets) and checkpoints, loaded
  // with the staging (not after it)
  const uint8_t* my = job.lvl + (size_t)tid * kFlowRecBytes;
  const uint4 rk4 = tid < ncp ? gld16(my) : make_uint4(~0u, ~0u, ~0u, ~0u);
  const uint4 fd4 = tid < ncp ? gld16(my + 2 * SEQ) : make_uint4(0u, 0u, 0u, 0u);
  const uint4 tk4 = tid < ncp ? gld16(my + 4 * SEQ) : make_uint4(~0u, ~0u, ~0u, ~0u);
  const int cp0 = tid < ncp ? (int)gld4(job.cp + tid) : 0;
  const int cp1 = tid + 1 < ncp ? (int)gld4(job.cp + tid + 1) : n;
  if (tid <= job.nlvl) {
    const uint8_t* st = job.lvl + kFlowRecBytes * (size_t)ncp;
    s_lvl[tid] = (int)(gld4(st + 2 * tid - 2 * (tid & 1)) >> (16 * (tid & 1))) & 0xFFFF;
  }
  {
    uint4* dst = reinterpret_cast<uint4*>(s_in32 + kFlowPad);
    const int n16 = (n + 15) >> 4;
    for (int i = tid; i < n16; i += kLzThreads) dst[i] = gld16(job.src + 16 * (size_t)i);
    uint4* img = reinterpret_cast<uint4*>(s_out32 + kFlowPad);
    for (int i = tid; i < kBlockBytes / 16; i += kLzThreads) img[i] = make_uint4(0, 0, 0, 0);
    if (tid == 0) {
      dst[n16] = make_uint4(0, 0, 0, 0);
      s_njob = 0;
      s_bad = 0;
    }
  }
  __syncthreads();
  LZ_STAMP(1);
  // ---- 1. parse my interval into registers (as k_lz4_decode) ----
  // r_lv / r_lvh: the literal bytes (L <= kFlowRegLit), or in r_lv the literal input offset
  uint32_t r_L[SEQ], r_DM[SEQ], r_lv[SEQ], r_lvh[SEQ];
#pragma unroll
  for (int s = 0; s < SEQ; ++s) r_L[s] = r_DM[s] = r_lv[s] = r_lvh[s] = 0;
  // the interval's tokens parsed independently (token offsets from the schedule), then checked to
  // chain: each token ends where the next begins, the last where the next interval does
  int cnt = 0, out_rel = 0;
  if (tid < ncp) {
    const uint32_t tkw[4] = {tk4.x, tk4.y, tk4.z, tk4.w};
    bool ok = true;
    int prev_next = cp0;
#pragma unroll
    for (int s = 0; s < SEQ; ++s) {
      const uint32_t dlt = (tkw[s >> 1] >> (16 * (s & 1))) & 0xFFFFu;
      if (dlt != 0xFFFFu) {
        const int pos = cp0 + (int)dlt;
        Tok t{};
        uint32_t hi = 0;
        const bool parsed = parse_tok8(s_in, n, pos, t, hi);  // (independent of the previous token)
        ok &= parsed & (pos == prev_next);
        r_L[s] = (uint32_t)t.L;
        r_DM[s] = (uint32_t)t.off | ((uint32_t)t.M << 16);
        r_lv[s] = t.L <= kFlowRegLit ? t.lv : (uint32_t)t.lit;
        r_lvh[s] = hi;
        out_rel += t.L + t.M;
        prev_next = t.next;
        cnt = s + 1;
      }
    }
    if (!ok || prev_next != cp1) s_bad = 1;
  }
  int total;
  const int base = block_scan_lz(out_rel, &total, s_tmp);
  LZ_STAMP(2);
  if (s_bad || total != job.dec_len) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  const uint32_t rkw[4] = {rk4.x, rk4.y, rk4.z, rk4.w}, fdw[4] = {fd4.x, fd4.y, fd4.z, fd4.w};
  auto rank = [&](int s) { return (int)((rkw[s >> 1] >> (16 * (s & 1))) & 0xFFFFu); };
  auto fdist = [&](int s) { return (fdw[s >> 1] >> (16 * (s & 1))) & 0xFFFFu; };  // the forwarded distance
  // ---- 2. level 0: literals into the image; long runs become jobs split evenly over the threads ----
  constexpr uint32_t kOwnLit = 0x80000000u;  // r_L flag: a long run the job table had no room for
  {
    // a run past the registers: one job per 16 bytes of it
    auto pieces = [](int L) { return L > kFlowRegLit ? (L + 15) >> 4 : 0; };
    int need = 0;
#pragma unroll
    for (int s = 0; s < SEQ; ++s)
      if (s < cnt) need += pieces((int)r_L[s]);
    int j = __ballot(need) ? wave_alloc(&s_njob, need) : 0;
    int o = base;
#pragma unroll
    for (int s = 0; s < SEQ; ++s) {
      if (s < cnt) {
        const int L = (int)r_L[s], d = (int)(r_DM[s] & 0xFFFF), M = (int)(r_DM[s] >> 16);
        if (L > kFlowRegLit) {
          const int nq = pieces(L);
          // (every slot below the table's end is written — the job threads read slots 0 .. min(jobs,
          // table) - 1 — and a run that does not fit whole is also copied by its own thread: its
          // pieces that got a slot write the same bytes again, an OR of equal values)
#pragma unroll 1
          for (int q = 0; q < nq && j + q < kFlowJobs; ++q)
            s_job[j + q] = make_uint2((uint32_t)(o + 16 * q) | ((uint32_t)(min(16, L - 16 * q) - 1) << 16),
                                      r_lv[s] + 16u * (uint32_t)q);
          if (j + nq > kFlowJobs) r_L[s] |= kOwnLit;
          j += nq;
        } else if (L > 0) {  // the literal bytes ride in r_lv / r_lvh: cut to L bytes, up to three ORs, no reads
          const int a = o & 3;
          const uint64_t x = ((uint64_t)r_lv[s] | ((uint64_t)r_lvh[s] << 32)) & (~0ull >> (64 - 8 * L));
          const uint64_t xs = x << (8 * a);
          lds_or(s_out32 + kFlowPad + (o >> 2), (uint32_t)xs);
          if (a + L > 4) lds_or(s_out32 + kFlowPad + (o >> 2) + 1, (uint32_t)(xs >> 32));
          if (a + L > 8) lds_or(s_out32 + kFlowPad + (o >> 2) + 2, (uint32_t)(x >> (64 - 8 * a)));
        }
        // a match's (forwarded) source inside the block, its table row inside the table (the attach-time
        // parse validated the stream; these keep a damaged index from reaching outside the image)
        if (M > 0 && ((unsigned)(d - 1) >= (unsigned)(o + L) || (unsigned)(fdist(s) - 1) >= (unsigned)(o + L) ||
                      rank(s) >= kFlowMaxMatches))
          s_bad = 1;
        o += L + M;
      }
    }
  }
  LZ_STAMP(13);
  __syncthreads();
  // every 16-byte piece of a literal run longer than the registers hold is one job: thread t copies job t
  const int nj = min(s_njob, kFlowJobs);
  LZ_STAMP(14);
  if (tid < nj) {
    const uint2 jb = s_job[tid];
    flow_copyn<5>(s_out32, (int)(jb.x & 0xFFFF), s_in32, (int)jb.y, job_len(jb));
  }
  LZ_STAMP(15);
  if (tid < ncp) {  // long runs the job table had no room for: their own thread copies them. From
                    // here on r_L holds the sequence's match start.
    int o = base;
#pragma unroll
    for (int s = 0; s < SEQ; ++s) {
      if (s < cnt) {
        const int L = (int)(r_L[s] & ~kOwnLit);
        if (r_L[s] & kOwnLit) flow_copy(s_out32, o, s_in32, (int)r_lv[s], L);
        r_L[s] = (uint32_t)(o + L);
        o += L + (int)(r_DM[s] >> 16);
      }
    }
  }
  LZ_STAMP(3);
  __syncthreads();  // every literal is in the image; the staged input is dead
  if (s_bad || s_lvl[job.nlvl] > kFlowMaxMatches) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  // ---- 3. my matches into the table at their ranks: start | distance << 16, length ----
#pragma unroll
  for (int s = 0; s < SEQ; ++s)
    if (s < cnt && (r_DM[s] >> 16) > 0) s_tab[rank(s)] = make_uint2(r_L[s] | (fdist(s) << 16), r_DM[s] >> 16);
  __syncthreads();
  LZ_STAMP(4);
  // ---- 4. matches level by level (every source byte is of a lower level: complete) ----
  uint64_t t_busy = 0, t_wait = 0;  // (PROF: this wave's cycles copying / waiting at the level barriers)
#pragma unroll 1
  for (int k = 1; k <= job.nlvl; ++k) {
    const uint64_t t0 = PROF ? __builtin_amdgcn_s_memtime() : 0;
    const int r1 = s_lvl[k];
#pragma unroll 1
    for (int r = s_lvl[k - 1] + tid; r < r1; r += kLzThreads) {
      const uint2 m = s_tab[r];
      flow_match(s_out32, (int)(m.x & 0xFFFF), (int)(m.x >> 16), (int)m.y);
    }
    if (PROF) {
      __builtin_amdgcn_s_waitcnt(0);
      const uint64_t t1 = __builtin_amdgcn_s_memtime();
      t_busy += t1 - t0;
      __syncthreads();
      t_wait += __builtin_amdgcn_s_memtime() - t1;
    } else {
      __syncthreads();
    }
  }
  if (PROF && (tid & 63) == 0) {
    prof[(size_t)blockIdx.x * kLz4ProfWords + 16 + (tid >> 6)] = t_busy;
    if (tid == 0) prof[(size_t)blockIdx.x * kLz4ProfWords + 12] = t_wait;
  }
  LZ_STAMP(5);
  if (PROF && tid == 0) {
    prof[(size_t)blockIdx.x * kLz4ProfWords + 8] = (uint64_t)job.nlvl;
    prof[(size_t)blockIdx.x * kLz4ProfWords + 9] = (uint64_t)n;
    prof[(size_t)blockIdx.x * kLz4ProfWords + 10] = (uint64_t)nj;
    prof[(size_t)blockIdx.x * kLz4ProfWords + 11] = (uint64_t)ncp;
  }
  // ---- 4. output: 16 bytes per 16-byte store (bytes past the block's end are zero) ----
  uint64_t racc = job.red_dst ? red_identity(job) : 0ull;
  const int nchunks = (total + 15) >> 4;
  for (int c = tid; c < nchunks; c += kLzThreads) {
    const uint4 v = reinterpret_cast<const uint4*>(s_out32 + kFlowPad)[c];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    out16(job, c, w, racc);
  }
  if (job.red_dst) red_finish(job, racc, s_red, kLzWaves);
  if (PROF) {
    __syncthreads();
    LZ_STAMP(6);
  }
  }
}

// ------------------------------------------------------------------------------------------------
// Light decoder: blocks of at most kLtMaxCps checkpoint intervals (<= 2048 sequences) whose copy
// chains are at most kLtMaxDepth hops long (attach-time classification, lz4_index_block). These are
// the literal-heavy blocks of high-entropy columns (random dictionary ids, noisy doubles: one long
// literal run, or ~700 sequences of ~90 literal bytes and a short match). Instead of a per-byte
// entry image (the general decoder's 128 KiB of LDS, one block per CU) the workgroup keeps only the
// staged input, then the sequence table in the same LDS (68 KiB: two blocks per CU), and resolves
// every output byte directly: a byte inside a literal run is read from the compressed block (L2,
// just staged), a match byte hops to its source position (at most kLtMaxDepth hops).
//   1. stage the compressed block in LDS; thread t parses checkpoint interval t (<= 8 sequences);
//   2. a block scan of the intervals' output lengths places every sequence: start, match start,
//      literal input offset, distance (written over the staged input); a 64-byte-granular LUT maps a
//      position to its first sequence;
//   3. output: 16-byte chunks, one per thread per step (coalesced 16-byte stores). A chunk inside one
//      literal run is five dword loads from the input; otherwise each byte is resolved hop by hop.
// ------------------------------------------------------------------------------------------------
constexpr int kLtMaxSeq = kLtMaxCps * kLzSeqPerCp;  // 2048
constexpr int kLtLut = kBlockBytes / 64;
constexpr int kLtBufWords = (kLz4InCap + 32) / 4;  // staged input (+ zero pad), later the sequence table
static_assert(kLtMaxCps <= kLtThreads, "one checkpoint interval per light-decoder thread");
static_assert((kLtMaxSeq + 1 + 3 * kLtMaxSeq) * 4 + kLtMaxSeq * 2 <= kLtBufWords * 4, "table fits the input buffer");

template <bool PROF>
__global__ __launch_bounds__(kLtThreads) void k_lz4_light(const Lz4Launch L, int32_t* __restrict__ err,
                                                          uint64_t* __restrict__ prof) {
  __shared__ __attribute__((aligned(16))) uint32_t s_buf[kLtBufWords];
  __shared__ uint16_t s_lut[kLtLut];  // first sequence covering position 64 * i
  __shared__ int s_tmp[kLtThreads / 64];
  __shared__ int s_bad;
  const Lz4Job job = fetch_job(L, blockIdx.x);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the light checkpoints: one interval of g sequences per thread
  const int n = job.src_len, ncp = job.nfine, g = job.light;
  const uint32_t* cpl = job.cp + job.ncp;
  if (n <= 0 || n > kLz4InCap || ncp <= 0 || ncp > kLtThreads || g < 1 || g > kLzSeqPerCp || ncp * g > kLtMaxSeq + g ||
      job.dec_len > kBlockBytes || job.dec_len < job.expect_len) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  // sequence table (sequence i = thread * g + s): right after the staged input when both fit, so the
  // output reads literals from LDS; otherwise over the input (literals from L2)
  const int nsq = ncp * g;
  const int in_words = ((n + 15) >> 4) * 4 + 4;  // staged input + one zero uint4
  const bool keep_in = in_words + (nsq + 1) + 3 * nsq + (nsq + 1) / 2 <= kLtBufWords;
  uint32_t* s_start = s_buf + (keep_in ? in_words : 0);  // [nsq + 1] output start of every sequence, then the total
  uint32_t* s_mst = s_start + nsq + 1;                    // [nsq] output start of its match
  uint32_t* s_lit = s_mst + nsq;                          // [nsq] input offset of its literals
  int32_t* s_mb = reinterpret_cast<int32_t*>(s_lit + nsq);  // [nsq] input base of a resolved match, -1
  uint16_t* s_dist = reinterpret_cast<uint16_t*>(s_mb + nsq);  // [nsq] match distance
  LZ_STAMP(0);
  // ---- stage the compressed block (16-byte aligned and padded in the device image) ----
  {
    uint4* dst = reinterpret_cast<uint4*>(s_buf);
    const int n16 = (n + 15) >> 4;
    for (int i = tid; i < n16; i += kLtThreads) dst[i] = gld16(job.src + 16 * (size_t)i);
    if (tid == 0) {
      dst[n16] = make_uint4(0, 0, 0, 0);
      s_bad = 0;
    }
  }
  __syncthreads();
  LZ_STAMP(1);
  const uint8_t* s_in = reinterpret_cast<const uint8_t*>(s_buf);
  // ---- 1. parse my interval ----
  int r_L[kLzSeqPerCp], r_M[kLzSeqPerCp], r_off[kLzSeqPerCp], r_lit[kLzSeqPerCp];
  int cnt = 0, out_rel = 0;
  bool bad = false;
  if (tid < ncp) {
    int pos = (int)gld4(cpl + tid);
    const int end = tid + 1 < ncp ? (int)gld4(cpl + tid + 1) : n;
#pragma unroll
    for (int s = 0; s < kLzSeqPerCp; ++s) {
      r_L[s] = r_M[s] = r_off[s] = r_lit[s] = 0;
      if (s < g && pos < end) {
        Tok t;
        if (parse_tok(s_in, n, pos, t)) {
          r_L[s] = t.L;
          r_M[s] = t.M;
          r_off[s] = t.off;
          r_lit[s] = t.lit;
          out_rel += t.L + t.M;
          pos = t.next;
          cnt = s + 1;
        } else {
          pos = -1;
        }
      }
    }
    bad = pos != end || (tid + 1 < ncp && cnt != g);
  }
  // ---- 2. block scan of the intervals' output lengths -> sequence table (over the staged input) ----
  const int x = wave_add_scan(out_rel);
  if (lane == 63) s_tmp[wave] = x;
  if (bad) s_bad = 1;
  __syncthreads();  // also the end of every read of the staged input
  LZ_STAMP(2);
  int base = x - out_rel, total = 0;
#pragma unroll
  for (int w = 0; w < kLtThreads / 64; ++w) {
    const int y = s_tmp[w];
    base += w < wave ? y : 0;
    total += y;
  }
  if (s_bad || total != job.dec_len) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  {
    int o = base;
#pragma unroll
    for (int s = 0; s < kLzSeqPerCp; ++s) {
      if (s < cnt) {
        const int i = tid * g + s;
        s_start[i] = (uint32_t)o;
        s_mst[i] = (uint32_t)(o + r_L[s]);
        s_lit[i] = (uint32_t)r_lit[s];
        s_dist[i] = (uint16_t)r_off[s];
        s_mb[i] = -1;
        if (r_M[s] > 0 && r_off[s] > o + r_L[s]) s_bad = 1;  // distance before the block start
        // LUT entries of the 64-byte boundaries inside [o, o + L + M)
        const int e = o + r_L[s] + r_M[s];
        for (int k = (o + 63) >> 6; (k << 6) < e; ++k) s_lut[k] = (uint16_t)i;
        o = e;
      }
    }
    if (tid == ncp - 1) s_start[tid * g + cnt] = (uint32_t)total;
  }
  __syncthreads();
  if (s_bad) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  auto seq_of = [&](int pos) {
    int s = s_lut[pos >> 6];
    while ((int)s_start[s + 1] <= pos) ++s;
    return s;
  };
  // ---- match resolution by sequence: a match whose first period (its source [ms - d, ms - d +
  // min(M, d))) lies inside one literal run, or inside one resolved non-periodic match, copies
  // input bytes base + (k mod d): record base (rounds, one per chain level; the rest stay per byte) ----
  {
    uint32_t todo = 0;  // my sequences with a match still to resolve
#pragma unroll
    for (int s = 0; s < kLzSeqPerCp; ++s) todo |= (s < cnt && r_M[s] > 0) ? 1u << s : 0u;
    for (int round = 0; round < kLtMaxDepth; ++round) {
      bool progress = false;
#pragma unroll
      for (int s = 0; s < kLzSeqPerCp; ++s) {
        if (!((todo >> s) & 1u)) continue;
        const int i = tid * g + s;
        const int ms = (int)s_mst[i], d = r_off[s], a = ms - d, len = min(r_M[s], d);
        const int t = seq_of(a);
        const int tst = (int)s_start[t], tms = (int)s_mst[t], ten = (int)s_start[t + 1];
        int base = -1;
        if (a + len <= tms) {
          base = (int)s_lit[t] + (a - tst);
        } else if (a >= tms && a + len <= ten) {
          const int tb = s_mb[t], td = s_dist[t];
          if (tb >= 0 && td >= ten - tms) base = tb + (a - tms);  // (a resolved, non-periodic match)
          else if (tb < 0) continue;                             // (its source may resolve next round)
        }
        if (base >= 0) {
          s_mb[i] = base;
          progress = true;
        }
        todo &= ~(1u << s);  // resolved, or left to the per-byte path
      }
      if (!__syncthreads_or(progress)) break;  // (another thread's match may unlock one of mine)
    }
  }
  __syncthreads();
  LZ_STAMP(3);
  // ---- 3. output: 16-byte chunks ----
  const uint8_t* __restrict__ in = job.src;
  const int nchunks = (total + 15) >> 4;
  bool fail = false;
  uint64_t lt_acc = 0;  // (unused: the engine fuses only blocks of the general decoder)
  // the source of output byte x: its literal position (a literal byte, a resolved match byte, or
  // hop by hop back to one); -1 = longer chain than the light limit (malformed classification)
  auto resolve = [&](int x, int s) -> int {  // s: a sequence starting at or before x
    while ((int)s_start[s + 1] <= x) ++s;
    const int st = (int)s_start[s], ms = (int)s_mst[s];
    if (x < ms) return (int)s_lit[s] + (x - st);
    const int dd = s_dist[s], mb = s_mb[s], k = x - ms;
    if (mb >= 0) return mb + (k < dd ? k : k % dd);
    const int M = (int)s_start[s + 1] - ms;
    int y = dd >= M ? x - dd : ms - dd + k % dd;
    int sy = s;
#pragma unroll 1
    for (int hop = 0; hop <= kLtMaxDepth && y >= 0; ++hop) {
      if (y < (int)s_start[sy] || y >= (int)s_start[sy + 1]) sy = seq_of(y);
      const int yst = (int)s_start[sy], yms = (int)s_mst[sy];
      if (y < yms) return (int)s_lit[sy] + (y - yst);
      const int yd = s_dist[sy], yM = (int)s_start[sy + 1] - yms, yk = y - yms;
      const int yb = s_mb[sy];
      if (yb >= 0) return yb + (yk < yd ? yk : yk % yd);
      y = yd >= yM ? y - yd : yms - yd + yk % yd;
    }
    return -1;
  };
  const int nsteps = (nchunks + 2 * kLtThreads - 1) / (2 * kLtThreads);
  for (int it = 0; it < nsteps; ++it) {  // (wave-uniform trip count: the per-byte pass shuffles)
    // two chunks per step: their literal loads are issued together
    const int c0 = it * 2 * kLtThreads + tid;
    int cs[2], src[2];
    bool lit[2];
    uint32_t v[2][5];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = c0 + u * kLtThreads;
      cs[u] = c < nchunks ? seq_of(c << 4) : 0;
      lit[u] = c < nchunks && (c << 4) + 16 <= (int)s_mst[cs[u]];
      src[u] = lit[u] ? (int)s_lit[cs[u]] + ((c << 4) - (int)s_start[cs[u]]) : 0;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q = 0; q < 5; ++q)
        v[u][q] = !lit[u] ? 0u : keep_in ? reinterpret_cast<const uint32_t*>(s_in)[(src[u] >> 2) + q] : gld4(in + 4 * ((src[u] >> 2) + q));
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!lit[u]) continue;  // inside one literal run: one 16-byte store
      const int sh = src[u] & 3;
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = sh ? __builtin_amdgcn_alignbyte(v[u][q + 1], v[u][q], sh) : v[u][q];
      out16(job, c0 + u * kLtThreads, w, lt_acc);
    }
    // the wave's other chunks, four at a time with one lane per byte: every byte resolves on its own
    // (no per-byte serial walk in one lane), bytes pack into dwords across lanes
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int mine = c0 + u * kLtThreads;
      uint64_t pend = __ballot(mine < nchunks && !lit[u]);
      while (pend) {
        int own[4] = {0, 0, 0, 0}, k = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (pend) {
            own[q] = __builtin_ctzll(pend);
            pend &= pend - 1;
            k = q + 1;
          }
        const int sub = lane >> 4, bi = lane & 15;
        const int ol = sub == 0 ? own[0] : sub == 1 ? own[1] : sub == 2 ? own[2] : own[3];
        const int cc = __shfl(mine, ol, 64);
        const int s0 = __shfl(cs[u], ol, 64);  // the chunk's first sequence
        const int x = (cc << 4) + bi;
        uint32_t b = 0;
        if (sub < k && x < total) {
          const int sp = resolve(x, s0);
          if (sp < 0) fail = true;
          else b = keep_in ? (uint32_t)s_in[sp] : gld1(in + sp);
        }
        const uint32_t b1 = __shfl_down(b, 1, 64), b2 = __shfl_down(b, 2, 64), b3 = __shfl_down(b, 3, 64);
        if (sub < k && (bi & 3) == 0) out4(job, cc * 16 + bi, b | (b1 << 8) | (b2 << 16) | (b3 << 24));
      }
    }
  }
  if (fail) atomicOr(err, 1);
  if (PROF) {
    __syncthreads();
    LZ_STAMP(4);
    if (tid == 0) prof[(size_t)blockIdx.x * kLz4ProfWords + 11] = (uint64_t)ncp;
  }
}

// ------------------------------------------------------------------------------------------------
// Run decoder: blocks of 8-byte value runs with a run index (lz4_run_index, dg_internal.h). Columns of
// sequential longs and timestamps are ~8 K sequences of [1-2 literal bytes, a 6-7-byte copy from 8
// bytes back] whose copy chains run through the whole block: the general decoder resolves them with a
// 128 KiB per-byte entry image, one block per CU. Here the attach-time index gives every interval of
// >= kRunTarget output bytes the 8 bytes before it, so each thread decodes its interval alone: the
// last 8 output bytes live in one 64-bit register (`win`, oldest byte lowest), a literal or far-copy
// chunk is shifted in from the compressed block (L1/L2: a thread reads its own interval's bytes),
// a copy from d <= 8 bytes back is the window's last d bytes repeated, and every 8-byte-aligned value is
// complete the moment it is emitted. Values go to the block's image in LDS (64 KiB: two blocks per CU)
// and leave in coalesced stores after one barrier (a slot, or the payload records' 8-byte field: 64 lanes
// fill 64 consecutive records), or are folded into the fused aggregator (no image).
// ------------------------------------------------------------------------------------------------
// 8 bytes of global memory at byte offset p of a 4-byte aligned buffer (three aligned dword loads)
__device__ __forceinline__ uint64_t g_rd8(const uint8_t* __restrict__ base, int p) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(base) + (p >> 2);
  const int sh = (p & 3) << 3;
  const uint64_t w01 = (uint64_t)gld4(q) | ((uint64_t)gld4(q + 1) << 32);
  const uint32_t w2 = gld4(q + 2);
  return sh ? ((w01 >> sh) | ((uint64_t)w2 << (64 - sh))) : w01;
}

// fold of one 8-byte value into a fused decode's accumulator (red_code)
__device__ __forceinline__ void run_fold(const Lz4Job& job, uint64_t x, uint64_t& acc) {
  switch (job.red_code) {
    case kRedLongSum: acc += x; break;
    case kRedDoubleSum:
      acc = (uint64_t)__double_as_longlong(__longlong_as_double((long long)acc) + __longlong_as_double((long long)x));
      break;
    case kRedLongMax: acc = (uint64_t)max((long long)acc, (long long)x); break;
    case kRedLongMin: acc = (uint64_t)min((long long)acc, (long long)x); break;
    default: acc = combine_op(job.red_op, acc, agg_input_raw(job.red_kind, job.red_vkind, x));
  }
}

constexpr int kRunVals = kBlockBytes / 8;
constexpr int kRunStageBlocks = 512;  // launches up to this many blocks stage their input (latency mode)

// 8 bytes of an LDS byte array at byte offset p (three aligned dword reads)
__device__ __forceinline__ uint64_t l_rd8(const uint32_t* __restrict__ a, int p) {
  const uint32_t* q = a + (p >> 2);
  const int sh = p & 3;
  const uint32_t w0 = q[0], w1 = q[1], w2 = q[2];
  return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
}

// STAGE (launches of at most kRunStageBlocks blocks, which leave most CUs idle): the compressed block and
// its far table are staged in LDS first, so each interval's serial chain waits on LDS instead of L2/HBM
// (a block's latency, not the launch's throughput, is the cost there); 104 KiB of LDS, one block per
// CU. Otherwise the thread reads its ~128 contiguous input bytes from L1/L2 and two blocks share a CU.
template <bool STAGE>
__global__ __launch_bounds__(kRunThreads) void k_lz4_run(const Lz4Launch L, int32_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) uint64_t s_val[kRunVals];  // the block's decoded image
  __shared__ __attribute__((aligned(16))) uint32_t s_in[STAGE ? kRunLdsMax / 4 + 8 : 4];  // staged input, far table
  __shared__ uint64_t s_red[kRunThreads / 64];
  const Lz4Job job = fetch_job(L, blockIdx.x);
  const int tid = threadIdx.x;
  const int n = job.src_len, ni = job.run_n, nfar = job.run_far;
  if (n <= 0 || ni <= 0 || ni > kRunThreads || nfar < 0 || nfar > kRunFarMax ||
      16 * (((n + 15) >> 4) + ((nfar + 15) >> 4) + 2) > kRunLdsMax || job.dec_len <= 0 || (job.dec_len & 7) ||
      job.dec_len > kBlockBytes || job.dec_len < job.expect_len) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  const uint8_t* __restrict__ in = job.src;                          // 16-byte aligned, zero padded
  const uint8_t* __restrict__ far = job.rx + ((14 * ni + 15) & ~15);  // 16-byte aligned, zero padded
  const int n16 = (n + 15) >> 4;
  if constexpr (STAGE) {
    const int f16 = (nfar + 15) >> 4;
    uint4* st = reinterpret_cast<uint4*>(s_in);
    for (int i = tid; i < n16 + f16 + 1; i += kRunThreads)
      st[i] = i < n16 ? gld16(in + 16 * (size_t)i) : i < n16 + f16 ? gld16(far + 16 * (size_t)(i - n16)) : make_uint4(0, 0, 0, 0);
  }
  auto rd8_in = [&](int q) -> uint64_t {
    if constexpr (STAGE) return l_rd8(s_in, q);
    else return g_rd8(in, q);
  };
  auto rd8_far = [&](int q) -> uint64_t {
    if constexpr (STAGE) return l_rd8(s_in + 4 * n16, q);
    else return g_rd8(far, q);
  };
  auto rd1_in = [&](int q) -> int {
    if constexpr (STAGE) return (int)((s_in[q >> 2] >> (8 * (q & 3))) & 0xFF);
    else return (int)gld1(in + q);
  };
  const bool fold = job.red_dst != nullptr;
  uint64_t acc = fold ? red_identity(job) : 0ull;
  bool bad = false;
  uint64_t win = 0;
  uint32_t tf = 0;
  int o = 0, oend = 0;
  if (tid < ni) {  // (loaded beside the staging)
    win = (uint64_t)gld4(job.rx + 8 * (size_t)tid) | ((uint64_t)gld4(job.rx + 8 * (size_t)tid + 4) << 32);
    tf = gld4(job.rx + 8 * (size_t)ni + 4 * (size_t)tid);
    const uint16_t* ost = reinterpret_cast<const uint16_t*>(job.rx + 12 * (size_t)ni);
    o = ost[tid];
    oend = tid + 1 < ni ? (int)ost[tid + 1] : job.dec_len;
  }
  if constexpr (STAGE) __syncthreads();
  if (tid < ni) {
    int p = (int)(tf & 0x1FFFFu), fp = (int)(tf >> 17);
    // shift k (1..8) bytes, the low bytes of x, into the window; a completed aligned value is emitted
    auto push = [&](uint64_t x, int k) {
      win = k == 8 ? x : ((win >> (8 * k)) | (x << (64 - 8 * k)));
      o += k;
      if ((o & 7) == 0) {
        if (fold) {
          if (o <= job.expect_len && red_row(job, (o >> 3) - 1)) run_fold(job, win, acc);
        } else {
          s_val[(o >> 3) - 1] = win;
        }
      }
    };
    auto ext = [&](int& q, int& len) {  // LZ4 extended length (bytes up to the first != 255)
      for (int b = 255; b == 255;) {
        if (q >= n) {
          bad = true;
          return;
        }
        b = rd1_in(q++);
        len += b;
      }
    };
#pragma unroll 1
    while (o < oend && !bad) {
      const uint64_t w = rd8_in(p);
      const int tk = (int)(w & 0xFF);
      int L = tk >> 4, M = tk & 15, q = p + 1;
      if (L == 15) ext(q, L);
      if (L > oend - o) {
        bad = true;
        break;
      }
      // literals: from the token's window when they and the distance fit in it, else from the block
      if (L > 0) {
        if (tk < 0x60) {  // L <= 5: the token window holds them
          const uint64_t lv = w >> 8;
          const int k1 = min(L, 8 - (o & 7));
          push(lv, k1);
          if (L > k1) push(lv >> (8 * k1), L - k1);
        } else {
          int lp = q, rem = L;
#pragma unroll 1
          while (rem > 0) {
            const int k = min(rem, 8 - (o & 7));
            push(rd8_in(lp), k);
            lp += k;
            rem -= k;
          }
        }
      }
      q += L;
      if (q >= n) {  // the last sequence: literals only
        if (q > n || o != job.dec_len) bad = true;
        break;
      }
      const int d = tk < 0x60 ? (int)((w >> (8 * (1 + L))) & 0xFFFF) : (int)(rd8_in(q) & 0xFFFF);
      q += 2;
      if (M == 15) ext(q, M);
      M += 4;
      if (d == 0 || d > o || M > oend - o) {
        bad = true;
        break;
      }
      if (d <= 8) {  // near copy: the window's last d bytes, repeated
#pragma unroll 1
        while (M > 0) {
          const int k = min(M, 8 - (o & 7));
          uint64_t r = win >> (64 - 8 * d);
          for (int per = d; per < 8; per <<= 1) r |= r << (8 * per);
          push(r, k);
          M -= k;
        }
      } else {  // far copy: its bytes from the far table
#pragma unroll 1
        while (M > 0) {
          const int k = min(M, 8 - (o & 7));
          push(rd8_far(fp), k);
          fp += k;
          M -= k;
        }
      }
      p = q;
    }
    if (o != oend) bad = true;
  }
  if (bad) atomicOr(err, 1);
  if (fold) {
    red_finish(job, acc, s_red, kRunThreads / 64);
    return;
  }
  __syncthreads();
  // the block's values out: a slot takes every value of the block, payload records only its rows
  if (!job.vstride) {
    const int nq = job.dec_len >> 4;  // 16-byte stores (dec_len % 8 == 0)
    const uint4* s16 = reinterpret_cast<const uint4*>(s_val);
    for (int c = tid; c < nq; c += kRunThreads) {
      const uint4 v = s16[c];
      gst16(job.dst + 16 * (size_t)c, v.x, v.y, v.z, v.w);
    }
    if ((job.dec_len & 8) && tid == 0) {
      const uint64_t v = s_val[(job.dec_len >> 3) - 1];
      gst8(job.dst + (size_t)job.dec_len - 8, (uint32_t)v, (uint32_t)(v >> 32));
    }
  } else {
    const int nv = job.expect_len >> 3;
    for (int v = tid; v < nv; v += kRunThreads) {
      const uint64_t x = s_val[v];
      gst8(job.dst + (size_t)v * job.vstride, (uint32_t)x, (uint32_t)(x >> 32));
    }
  }
}

void launch_lz4_run(const Lz4Launch& L, int njobs, int stage_mode, int32_t* d_err, hipStream_t s) {
  if (njobs <= 0) return;
  // DG_RUN_STAGE=0 / 1 forces the mode (tests run every run block through both)
  const char* force = getenv("DG_RUN_STAGE");
  const bool stage = force && *force ? *force != '0' : stage_mode == 2 || (stage_mode == 1 && njobs <= kRunStageBlocks);
  if (stage) hipLaunchKernelGGL(k_lz4_run<true>, dim3(njobs), dim3(kRunThreads), 0, s, L, d_err);
  else hipLaunchKernelGGL(k_lz4_run<false>, dim3(njobs), dim3(kRunThreads), 0, s, L, d_err);
}

void launch_lz4_light(const Lz4Launch& L, int njobs, int32_t* d_err, hipStream_t s, uint64_t* d_prof) {
  if (njobs <= 0) return;
  if (d_prof) hipLaunchKernelGGL(k_lz4_light<true>, dim3(njobs), dim3(kLtThreads), 0, s, L, d_err, d_prof);
  else hipLaunchKernelGGL(k_lz4_light<false>, dim3(njobs), dim3(kLtThreads), 0, s, L, d_err, nullptr);
}

void launch_lz4_decode(const Lz4Launch& L, int njobs, int wide, int32_t* d_err, hipStream_t s, uint64_t* d_prof,
                       int flow_wgs) {
  if (njobs <= 0) return;
  if (wide & kLzFlow) {  // (flow blocks are never wide)
    const int grid = flow_wgs > 0 && !d_prof ? std::min(njobs, flow_wgs) : njobs;
    if (d_prof) hipLaunchKernelGGL(k_lz4_decode_flow<true>, dim3(njobs), dim3(kLzThreads), 0, s, L, d_err, d_prof, njobs);
    else hipLaunchKernelGGL(k_lz4_decode_flow<false>, dim3(grid), dim3(kLzThreads), 0, s, L, d_err, nullptr, njobs);
    return;
  }
  if (wide) {
    if (d_prof) hipLaunchKernelGGL((k_lz4_decode<true, kLzMaxSeqPerCp>), dim3(njobs), dim3(kLzThreads), 0, s, L, d_err, d_prof);
    else hipLaunchKernelGGL((k_lz4_decode<false, kLzMaxSeqPerCp>), dim3(njobs), dim3(kLzThreads), 0, s, L, d_err, nullptr);
  } else {
    if (d_prof) hipLaunchKernelGGL((k_lz4_decode<true, kLzSeqPerCp>), dim3(njobs), dim3(kLzThreads), 0, s, L, d_err, d_prof);
    else hipLaunchKernelGGL((k_lz4_decode<false, kLzSeqPerCp>), dim3(njobs), dim3(kLzThreads), 0, s, L, d_err, nullptr);
  }
}

}  // namespace dg
