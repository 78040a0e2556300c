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
//   1. parse: the attach-time checkpoint index (lz4_index_block: the token offset of every 16th
//      sequence) gives every thread its own 16 sequences; it parses them from the staged input into
//      registers (literal start, literal length, distance, match length);
//   2. a block scan of the threads' output lengths places every sequence; each output byte x gets a
//      16-bit entry E[x] in LDS: a literal is 0xFF00 | byte, a match byte the distance to the byte
//      it copies (LZ4 overlap semantics: src = start - dist + (k mod dist));
//   3. pointer jumping: E[x] += E[x - E[x]] until x - E[x] is a literal (log2(chain depth) rounds;
//      updates are asynchronous, any value read is a valid ancestor distance);
//   4. out[x] = low byte of the literal at x - E[x], written as 16-byte stores.
// The staged input and E share one 128 KiB LDS array (the parse finishes before E is written;
// literals are re-read from the compressed block in HBM/L2). Entries >= 0xFF00 are literals, so a
// distance must stay below 0xFF00: the last 256 output positions, whose distances can exceed it,
// keep absolute source positions in a small tail table and are resolved by a short chase.
// The sequential one-wave decoder (k_lz4_decode_seq) stays as a differential reference, DG_LZ4_SEQ=1.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "dg_internal.h"

namespace dg {

constexpr int kLzThreads = 1024;               // 16 waves: 4 per SIMD hide LDS latency
constexpr int kLzWaves = kLzThreads / 64;
constexpr int kLz4InCap = kBlockBytes + 2048;  // >= LZ4_compressBound(65536) = 65809
constexpr int kTail = 0xFF00;                  // E codes >= kTail are literals; positions >= kTail use the tail table
constexpr int kTailN = kBlockBytes - kTail;    // 256
constexpr int kShortLit = 4;                   // literal runs up to this ride in the parse registers
static_assert(kShortLit <= 4, "Tok::lv holds four literal bytes");
constexpr int kLongFill = 48;                  // matches above this are filled cooperatively
constexpr int kMaxJobs = 2048;
constexpr int kPairs = 32;                     // E pairs per thread: 2 * 32 * 1024 = 65536 positions
constexpr int kJumpBatch = 8;                 // steps of a jump sweep whose reads are issued together
constexpr int kMaxRounds = 20;                 // > log2(65536) + 1: pointer jumping always converges before
constexpr int kClass = 8;                      // the value width whose distance-8 copy chains are scanned
static_assert(kLz4InCap + 32 <= kBlockBytes * 2, "staged input must fit in the E array");
static_assert(kLzThreads * kLzSeqPerCp >= kBlockBytes / 4, "a block can hold 16384 sequences");

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

// Byte-wise parse (long lengths / windows that do not hold the offset).
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

// block-wide (1024 threads) exclusive scan; total via *total
__device__ int block_scan_lz(int v, int* total, int* s_tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
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
#ifndef DG_LZ_NOSKEW
constexpr int kESkewShift = 7;
constexpr int kEWords = kBlockBytes + (kBlockBytes >> kESkewShift) * 2;  // u16 entries incl. skew
__device__ __forceinline__ int eph(int x) { return x + ((x >> kESkewShift) << 1); }
#else
constexpr int kESkewShift = 16;
constexpr int kEWords = kBlockBytes;
__device__ __forceinline__ int eph(int x) { return x; }
#endif

struct LzState {
  uint16_t* e;
  uint16_t* tsrc;
  uint32_t* tlit;
};

__device__ __forceinline__ void put_lit(const LzState& S, int x, int v) {
  if (x < kTail) {
    S.e[eph(x)] = (uint16_t)(0xFF00 | v);
  } else {
    S.tsrc[x - kTail] = (uint16_t)v;
    atomicOr(&S.tlit[(x - kTail) >> 5], 1u << ((x - kTail) & 31));
  }
}

__device__ __forceinline__ void put_ptr(const LzState& S, int x, int src) {
  if (x < kTail) S.e[eph(x)] = (uint16_t)(x - src);
  else S.tsrc[x - kTail] = (uint16_t)src;
}

// value of output byte x once E and the tail table have converged (both hold literal codes)
__device__ __forceinline__ uint32_t lz_value(const LzState& S, int x) {
  if (x < kTail) return S.e[eph(x)] & 0xFF;
  return S.tsrc[x - kTail] & 0xFF;
}

#define LZ_STAMP(k)                                                                           \
  do {                                                                                        \
    if (PROF && tid == 0) prof[(size_t)blockIdx.x * kLz4ProfWords + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// cooperative-copy job: x = output start | (len - 1) << 16, y = literal input offset (kind 0) or
// match distance | 1 << 31 (kind 1)
__device__ __forceinline__ int job_len(uint2 j) { return (int)(j.x >> 16) + 1; }

template <bool PROF>
__global__ __launch_bounds__(kLzThreads) void k_lz4_decode(const Lz4Job* __restrict__ jobs, int32_t* __restrict__ err,
                                                           uint64_t* __restrict__ prof) {
  __shared__ __attribute__((aligned(16))) uint16_t s_e[kEWords];  // 130 KiB: staged input, then E
  __shared__ uint16_t s_tsrc[kTailN];
  __shared__ uint32_t s_tlit[kTailN / 32];
  __shared__ uint2 s_job[kMaxJobs];
  __shared__ int s_jpre[kMaxJobs];
  __shared__ int s_njob, s_bad, s_c8;
  __shared__ int s_tmp[kLzWaves];

  const Lz4Job job = jobs[blockIdx.x];
  const int tid = threadIdx.x;
  const int n = job.src_len, ncp = job.ncp;
  if (n <= 0 || n > kLz4InCap || ncp <= 0 || ncp > kLzThreads || job.dec_len > kBlockBytes ||
      job.dec_len < job.expect_len) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  LZ_STAMP(0);
  uint8_t* s_in = reinterpret_cast<uint8_t*>(s_e);
  const LzState S{s_e, s_tsrc, s_tlit};
  // ---- stage the compressed block (16-byte aligned and padded in the device image) ----
  {
    const uint4* src = reinterpret_cast<const uint4*>(job.src);
    uint4* dst = reinterpret_cast<uint4*>(s_in);
    const int n16 = (n + 15) >> 4;
    for (int i = tid; i < n16; i += kLzThreads) dst[i] = src[i];
    if (tid == 0) {
      dst[n16] = make_uint4(0, 0, 0, 0);
      s_njob = 0;
      s_bad = 0;
      s_c8 = 0;
    }
    if (tid < kTailN / 32) s_tlit[tid] = 0;
  }
  __syncthreads();
  LZ_STAMP(1);
  // ---- 1. parse my interval of kLzSeqPerCp sequences into registers ----
  uint32_t r_L[kLzSeqPerCp], r_DM[kLzSeqPerCp], r_lv[kLzSeqPerCp];  // r_lv: literal bytes (L <= 4) or offset
  int cnt = 0, out_rel = 0;
  if (tid < ncp) {
    int pos = (int)job.cp[tid];
    const int end = tid + 1 < ncp ? (int)job.cp[tid + 1] : n;
#pragma unroll
    for (int s = 0; s < kLzSeqPerCp; ++s) {
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
  int total;
  const int base = block_scan_lz(out_rel, &total, s_tmp);  // its barriers end every read of s_in
  LZ_STAMP(2);
  if (s_bad || total != job.dec_len) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  // ---- 2. E entries: short literals from registers, short matches as distances; longer runs
  // become jobs for the cooperative pass (their literals come from the compressed block in HBM) ----
  const uint8_t* __restrict__ gin = job.src;
  int c8 = 0;  // my match bytes at distance 8 (class chains of 8-byte values, resolved by a scan below)
  if (tid < ncp) {
    int o = base;
#pragma unroll
    for (int s = 0; s < kLzSeqPerCp; ++s) {
      if (s < cnt) {
        const int L = (int)r_L[s];
        const int d = (int)(r_DM[s] & 0xFFFF), M = (int)(r_DM[s] >> 16);
        if (L <= kShortLit) {
          const uint32_t lv = r_lv[s];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (k < L) put_lit(S, o + k, (lv >> (8 * k)) & 0xFF);
        } else {
          const int j = atomicAdd(&s_njob, 1);
          if (j < kMaxJobs) {
            s_job[j] = make_uint2((uint32_t)o | ((uint32_t)(L - 1) << 16), r_lv[s]);
          } else {
            for (int k = 0; k < L; ++k) put_lit(S, o + k, gin[r_lv[s] + k]);
          }
        }
        o += L;
        if (M > 0) {
          if (d > o) s_bad = 1;
          c8 += d == 8 ? M : 0;
          int j = kMaxJobs;
          if (M > kLongFill) {
            j = atomicAdd(&s_njob, 1);
            if (j < kMaxJobs) s_job[j] = make_uint2((uint32_t)o | ((uint32_t)(M - 1) << 16), (uint32_t)d | 0x80000000u);
          }
          if (j >= kMaxJobs) {
            if (d >= M || d == kClass) {  // distance 8: plain x - 8 (same value, same class chain)
              for (int k = 0; k < M; ++k) put_ptr(S, o + k, o + k - d);
            } else {
              int r = 0;
              for (int k = 0; k < M; ++k) {
                put_ptr(S, o + k, o - d + r);
                if (++r == d) r = 0;
              }
            }
          }
          o += M;
        }
      }
    }
  }
  if (c8) atomicAdd(&s_c8, c8);
  __syncthreads();
  LZ_STAMP(3);
  // ---- cooperative pass: the jobs' bytes as one flat range, split evenly over the threads ----
  const int nj = min(s_njob, kMaxJobs);
  if (nj > 0) {
    int l0 = 0, l1 = 0;
    if (2 * tid < nj) l0 = job_len(s_job[2 * tid]);
    if (2 * tid + 1 < nj) l1 = job_len(s_job[2 * tid + 1]);
    int tot;
    const int pre = block_scan_lz(l0 + l1, &tot, s_tmp);
    if (2 * tid < nj) s_jpre[2 * tid] = pre;
    if (2 * tid + 1 < nj) s_jpre[2 * tid + 1] = pre + l0;
    __syncthreads();
    // flat positions interleaved over the threads (f = tid, tid + 1024, ...): a wave's 64 lanes take
    // 64 consecutive positions, so the literal byte loads of a long run are one cache line per wave
    // instruction and the E stores consecutive; each lane's job index only moves forward
    auto find_job = [&](int f, int lo) {  // last job with s_jpre <= f, searching from lo
      int hi = nj - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_jpre[mid] <= f) lo = mid;
        else hi = mid - 1;
      }
      return lo;
    };
    int j = 0;
    for (int fb = tid; fb < tot; fb += 8 * kLzThreads) {
      int xs[8], srcs[8];
      uint32_t vals[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        xs[u] = -1;
        const int g = fb + u * kLzThreads;
        if (g < tot) {
          if (g >= s_jpre[j] + job_len(s_job[j])) j = find_job(g, j);
          const uint2 jb = s_job[j];
          const int k = g - s_jpre[j], o = (int)(jb.x & 0xFFFF);
          xs[u] = o + k;
          if (jb.y & 0x80000000u) {
            const int d = (int)(jb.y & 0xFFFF);
            srcs[u] = (d >= job_len(jb) || d == kClass) ? o + k - d : o - d + k % d;
          } else {
            srcs[u] = -1 - ((int)jb.y + k);  // literal: input offset, encoded negative
          }
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (xs[u] >= 0 && srcs[u] < 0) vals[u] = gin[-1 - srcs[u]];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (xs[u] < 0) continue;
        if (srcs[u] < 0) put_lit(S, xs[u], vals[u]);
        else put_ptr(S, xs[u], srcs[u]);
      }
    }
  }
  __syncthreads();
  if (s_bad) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  LZ_STAMP(4);
  // ---- 3. pointer jumping with value propagation over positions [0, min(total, kTail)):
  // E[x] += E[x - E[x]] while that target holds a distance; once it holds a literal code, x takes
  // the code itself, so later readers of x resolve in one step. My pairs stay in registers. ----
  const int lim = min(total, kTail);
  uint32_t* s_e32 = reinterpret_cast<uint32_t*>(s_e);
  // positions in [lim, 2 * kPairs * kLzThreads) act as resolved literals
  if (lim < kTail) {
    for (int x = lim + tid; x < kTail; x += kLzThreads) s_e[eph(x)] = 0xFF00;
  }
#ifndef DG_LZ_NOSCAN8
  // ---- 2b. class chains: a byte copied from 8 back holds the value of the last "terminal" (a
  // literal, or a byte of a match at another distance) of its residue class mod 8 before it. A
  // carry scan over the block turns every distance-8 entry into the distance to that terminal, so
  // the jumping below only has to chase the few other matches (8-byte value columns: sequential
  // longs and timestamps are ~99.5 % distance-8 matches chaining through the whole block). ----
  if (s_c8 * 4 > total) {
    __syncthreads();
    const int x0 = tid * 64;
    // my 64 entries as pairs (read twice: keeping them in registers spills); positions >= lim read
    // as literals
    auto pair_at = [&](int q) { return x0 + 2 * q < lim ? s_e32[eph(x0 + 2 * q) >> 1] : 0xFF00FF00u; };
    int last[kClass];
#pragma unroll
    for (int c = 0; c < kClass; ++c) last[c] = -1;
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int c = (2 * q) & 7;
      const uint32_t v = pair_at(q);
      if ((v & 0xFFFF) != (uint32_t)kClass) last[c] = x0 + 2 * q;
      if ((v >> 16) != (uint32_t)kClass) last[c + 1] = x0 + 2 * q + 1;
    }
    // exclusive max-scan of the per-class last terminal over the threads (positions grow with tid)
    const int lane = tid & 63, wave = tid >> 6;
    int carry[kClass];
    int* s_scan = s_jpre;  // free after the cooperative pass: [kLzWaves][kClass]
#pragma unroll
    for (int c = 0; c < kClass; ++c) {
      int v = last[c];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o, 64);
        if (lane >= o) v = max(v, y);
      }
      const int ex = __shfl_up(v, 1, 64);
      carry[c] = lane ? ex : -1;
      if (lane == 63) s_scan[wave * kClass + c] = v;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < kClass; ++c)
      for (int w = 0; w < wave; ++w) carry[c] = max(carry[c], s_scan[w * kClass + c]);
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int c = (2 * q) & 7, x = x0 + 2 * q;
      const uint32_t v = pair_at(q);
      uint32_t lo = v & 0xFFFF, hi = v >> 16;
      if (lo == (uint32_t)kClass) {
        if (carry[c] >= 0) lo = (uint32_t)(x - carry[c]);
      } else {
        carry[c] = x;
      }
      if (hi == (uint32_t)kClass) {
        if (carry[c + 1] >= 0) hi = (uint32_t)(x + 1 - carry[c + 1]);
      } else {
        carry[c + 1] = x + 1;
      }
      const uint32_t nv = lo | (hi << 16);
      if (nv != v && x < lim) s_e32[eph(x) >> 1] = nv;
    }
  }
#endif
  bool any = true;
  int jump_rounds = 0;
  // Rounds of jumping. Wave w sweeps its own 4 KiB of positions in increasing order, 64 pairs per
  // step, so within a round a position already sees the updates of the earlier steps of its wave
  // (LDS ops of one wave complete in order): chains collapse to the region start in one round, and
  // the rounds only have to jump across the 16 regions. A batch of kJumpBatch steps issues its
  // reads back to back; a resolved position reads itself; only changed pairs are written.
  const int wv = tid >> 6, ln = tid & 63;
  uint32_t done = 0;  // wave-uniform: batch b of my wave's region is fully resolved
  for (int round = 0; __syncthreads_or(any); ++round) {
    if (round > kMaxRounds) {  // unreachable for a valid block
      if (tid == 0) atomicOr(err, 1);
      return;
    }
    jump_rounds++;
    any = false;
#pragma unroll 1
    for (int b = 0; b < kPairs / kJumpBatch; ++b) {
      if ((done >> b) & 1u) continue;
      const int j0 = b * kJumpBatch;
      uint32_t dv[kJumpBatch], ta[kJumpBatch], tb[kJumpBatch];
#pragma unroll
      for (int k = 0; k < kJumpBatch; ++k) {
        const int x = 2 * (wv * (kPairs * 64) + (j0 + k) * 64 + ln);
        dv[k] = x < kTail ? s_e32[eph(x) >> 1] : 0xFF00FF00u;
      }
#pragma unroll
      for (int k = 0; k < kJumpBatch; ++k) {
        const int x = 2 * (wv * (kPairs * 64) + (j0 + k) * 64 + ln);
        const uint32_t v = dv[k], d0 = v & 0xFFFF, d1 = v >> 16;
        const int a0 = x - (d0 < (uint32_t)kTail ? (int)d0 : 0);
        const int a1 = x + 1 - (d1 < (uint32_t)kTail ? (int)d1 : 0);
        // a resolved entry (literal code) needs no target read
        ta[k] = (x < kTail && d0 < (uint32_t)kTail) ? s_e[eph(a0)] : 0xFF00u;
        tb[k] = (x < kTail && d1 < (uint32_t)kTail) ? s_e[eph(a1)] : 0xFF00u;
      }
      bool open = false;
#pragma unroll
      for (int k = 0; k < kJumpBatch; ++k) {
        const int x = 2 * (wv * (kPairs * 64) + (j0 + k) * 64 + ln);
        const uint32_t v = dv[k], d0 = v & 0xFFFF, d1 = v >> 16;
        const uint32_t e0 = ta[k], e1 = tb[k];
        const uint32_t n0 = d0 >= (uint32_t)kTail ? d0 : (e0 >= (uint32_t)kTail ? e0 : d0 + e0);
        const uint32_t n1 = d1 >= (uint32_t)kTail ? d1 : (e1 >= (uint32_t)kTail ? e1 : d1 + e1);
        const uint32_t nv = n0 | (n1 << 16);
        if (nv != v) s_e32[eph(x) >> 1] = nv;
        open |= n0 < (uint32_t)kTail || n1 < (uint32_t)kTail;
      }
      if (__ballot(open) == 0) done |= 1u << b;
      any |= open;
    }
  }
  LZ_STAMP(5);
  if (PROF && tid == 0) {
    prof[(size_t)blockIdx.x * kLz4ProfWords + 8] = (uint64_t)jump_rounds;
    prof[(size_t)blockIdx.x * kLz4ProfWords + 9] = (uint64_t)n;
    prof[(size_t)blockIdx.x * kLz4ProfWords + 10] = (uint64_t)nj;
    prof[(size_t)blockIdx.x * kLz4ProfWords + 11] = (uint64_t)ncp;
  }
  // ---- tail: positions [kTail, total) hold absolute sources; rounds of jumping over the table ----
  if (total > kTail) {
    const int nt = total - kTail;
    bool tact = tid < nt && !((s_tlit[tid >> 5] >> (tid & 31)) & 1u);
    for (int round = 0;; ++round) {
      uint32_t nsrc = 0;
      bool res = false;
      if (tact) {
        const int src = s_tsrc[tid];
        if (src < kTail) {
          nsrc = s_e[eph(src)];  // a literal code: E has converged
          res = true;
        } else {
          const int i2 = src - kTail;
          nsrc = s_tsrc[i2];
          res = (s_tlit[i2 >> 5] >> (i2 & 31)) & 1u;
        }
      }
      __syncthreads();
      if (tact) {
        s_tsrc[tid] = (uint16_t)nsrc;
        if (res) {
          atomicOr(&s_tlit[tid >> 5], 1u << (tid & 31));
          tact = false;
        }
      }
      if (!__syncthreads_or(tact)) break;
      if (round > 10) {  // 256 positions: 9 rounds suffice
        if (tid == 0) atomicOr(err, 1);
        return;
      }
    }
  }
  // ---- 4. output: every entry is now a literal code; 16 bytes per 16-byte store ----
  uint4* dst = reinterpret_cast<uint4*>(job.dst);
  const int nchunks = (total + 15) >> 4;
  for (int c = tid; c < nchunks; c += kLzThreads) {
    const int x0 = c << 4;
    uint32_t w[4];
    if (x0 + 16 <= lim) {
      const uint32_t* ep = s_e32 + (eph(x0) >> 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t e0 = ep[2 * q], e1 = ep[2 * q + 1];
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
    dst[c] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  if (PROF) {
    __syncthreads();
    LZ_STAMP(6);
  }
}

// Sequential reference decoder (DG_LZ4_SEQ=1): one wave per block, compressed input and decoded output staged in LDS.
// Tokens are parsed in order (the format is sequential); literal and match copies are spread over
// the 64 lanes. Overlapping matches (offset < length) use the periodic form
// out[op + k] = out[op - off + k % off], which only reads bytes before op, so the lanes never race.
// ------------------------------------------------------------------------------------------------

__global__ __launch_bounds__(64) void k_lz4_decode_seq(const Lz4Job* __restrict__ jobs, int32_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kLz4InCap + 16];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kBlockBytes + 64];
  const Lz4Job job = jobs[blockIdx.x];
  const int lane = threadIdx.x;
  const int iend = job.src_len;
  if (iend <= 0 || iend > kLz4InCap) {
    if (lane == 0) atomicOr(err, 1);
    return;
  }
  {
    const uint4* src = reinterpret_cast<const uint4*>(job.src);
    uint4* dst = reinterpret_cast<uint4*>(s_in);
    const int n16 = (iend + 15) >> 4;
    for (int i = lane; i < n16; i += 64) dst[i] = src[i];
  }
  __syncthreads();
  int ip = 0, op = 0;
  bool bad = false;
  for (;;) {
    if (ip >= iend) {
      bad = true;
      break;
    }
    const int tok = __builtin_amdgcn_readfirstlane(s_in[ip]);
    ip++;
    int lit = tok >> 4;
    if (lit == 15) {
      int b;
      do {
        if (ip >= iend) {
          bad = true;
          break;
        }
        b = __builtin_amdgcn_readfirstlane(s_in[ip]);
        ip++;
        lit += b;
      } while (b == 255);
      if (bad) break;
    }
    if (lit > iend - ip || lit > kBlockBytes - op) {
      bad = true;
      break;
    }
    for (int k = lane; k < lit; k += 64) s_out[op + k] = s_in[ip + k];
    ip += lit;
    op += lit;
    if (ip == iend) break;  // last sequence: literals only
    if (iend - ip < 2) {
      bad = true;
      break;
    }
    const int off = __builtin_amdgcn_readfirstlane((int)s_in[ip] | ((int)s_in[ip + 1] << 8));
    ip += 2;
    int ml = tok & 15;
    if (ml == 15) {
      int b;
      do {
        if (ip >= iend) {
          bad = true;
          break;
        }
        b = __builtin_amdgcn_readfirstlane(s_in[ip]);
        ip++;
        ml += b;
      } while (b == 255);
      if (bad) break;
    }
    ml += 4;
    if (off == 0 || off > op || ml > kBlockBytes - op) {
      bad = true;
      break;
    }
    __syncthreads();
    if (off >= ml) {
      for (int k = lane; k < ml; k += 64) s_out[op + k] = s_out[op - off + k];
    } else {
      for (int k = lane; k < ml; k += 64) s_out[op + k] = s_out[op - off + (k % off)];
    }
    op += ml;
    __syncthreads();
  }
  __syncthreads();
  if (bad || op < job.expect_len) {
    if (lane == 0) atomicOr(err, 1);
    return;
  }
  uint4* dst = reinterpret_cast<uint4*>(job.dst);
  const uint4* src = reinterpret_cast<const uint4*>(s_out);
  const int n16 = (op + 15) >> 4;
  for (int i = lane; i < n16; i += 64) dst[i] = src[i];
}


void launch_lz4_decode(const Lz4Job* d_jobs, int njobs, int32_t* d_err, hipStream_t s, uint64_t* d_prof) {
  if (njobs <= 0) return;
  static const bool seq = getenv("DG_LZ4_SEQ") && getenv("DG_LZ4_SEQ")[0] == '1';
  if (seq) hipLaunchKernelGGL(k_lz4_decode_seq, dim3(njobs), dim3(64), 0, s, d_jobs, d_err);
  else if (d_prof) hipLaunchKernelGGL(k_lz4_decode<true>, dim3(njobs), dim3(kLzThreads), 0, s, d_jobs, d_err, d_prof);
  else hipLaunchKernelGGL(k_lz4_decode<false>, dim3(njobs), dim3(kLzThreads), 0, s, d_jobs, d_err, nullptr);
}

}  // namespace dg
