// dg_lz4.hip — LZ4 block decompression on gfx950 (Druid's per-block column codec).
//
// Replaces CompressionStrategy.LZ4Decompressor.decompress (processing/.../segment/data/
// CompressionStrategy.java:284-305 -> lz4-java 1.4.0 LZ4SafeDecompressor): one 64 KiB Druid block
// (CompressedPools.BUFFER_SIZE) per 256-thread workgroup, compressed input and decoded output in LDS.
//
// LZ4's token stream is sequential and Druid's numeric blocks are token-dense: a block of sequential
// longs is ~8k tokens of [1 literal byte, 7-byte match at offset 8], i.e. ONE dependency chain
// through the whole block (every match copies bytes the previous match produced). Neither a lane
// walking the stream (~2 ms/block measured) nor match-by-match rounds (one round per chunk) scale.
// This kernel decodes in five data-parallel phases:
//   1. parse, speculatively: the compressed block is cut into 256 chunks; thread i walks the token
//      chain from the start of its chunk as if a token started there, marking visited positions;
//   2. the true chain enters chunk i at the exit of chunk i-1 and meets the speculative chain within
//      a few tokens (chains are functions of position, so they merge): exits are computed in
//      parallel for the assumed entry and for the likely correction, wave 0 stitches them together;
//   3. each chunk's true tokens give output sizes and match counts -> block scans -> offsets;
//   4. literals are copied into the output (long runs cooperatively) and every match is recorded
//      as (output offset, distance, length) in a per-block table in global memory;
//   5. matches are resolved by pointer jumping instead of by copying in order: for each output
//      byte, P[x] = x for a literal byte and P[x] = src + (x - start) mod distance for a match byte
//      (LZ4 overlap semantics); repeated P[x] <- P[P[x]] converges in log2(chain depth) rounds, then
//      out[x] = out[P[x]]. P is 16 bits per byte and lives in the (dead) input buffer, one 32 KiB
//      half of the output at a time (the second half's pointers into the first half are final).
// The sequential one-wave decoder (k_lz4_decode_seq) stays as a differential reference, DG_LZ4_SEQ=1.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "dg_internal.h"

namespace dg {

constexpr int kLzThreads = 1024;               // 16 waves: 4 per SIMD hide LDS latency
constexpr int kLzWaves = kLzThreads / 64;
constexpr int kMinChunk = 32;                  // bytes of compressed input per speculative chunk (min)
constexpr int kLz4InCap = kBlockBytes + 2048;  // >= LZ4_compressBound(65536) = 65809
constexpr int kLongLit = 32;                   // literal runs above this are copied cooperatively
constexpr int kLongFill = 64;                  // match spans above this fill P cooperatively
constexpr int kMaxJobs = 512;
constexpr int kHalf = kBlockBytes / 2;
constexpr int kMaxJumpRounds = 40;
constexpr int kFixRounds = 8;                  // parallel entry fix-point rounds before the serial stitch
constexpr int kSeqFraction = 4;                // > 1/4 of chunks inconsistent after one round and a
                                               // compression ratio < 1.05: walk the tokens serially
constexpr int kJumpBatch = 8;                  // independent pointer chases in flight per thread
// per-chunk arrays live in the output buffer while it is free (phases 1-3), after the visited bitmap
constexpr int kChunkArrOff = 16384;
static_assert(kChunkArrOff >= (kLz4InCap + 64) / 8, "visited bitmap overlaps the chunk arrays");
static_assert(kChunkArrOff + 4 * kLzThreads * 4 <= kBlockBytes, "chunk arrays exceed the output buffer");

struct Tok {
  int lit;   // literal start (input offset)
  int L;     // literal length
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

// walk from `pos` inside [.., ce): stop on a position the speculative chain of this chunk visited
// (then the exit is that chain's exit `spec_exit`) or at the first token start >= ce
__device__ __forceinline__ int walk_to_exit(const uint8_t* __restrict__ in, int n, int pos, int ce,
                                            const uint32_t* __restrict__ vb, int spec_exit) {
  while (pos < ce) {
    if ((vb[pos >> 5] >> (pos & 31)) & 1u) return spec_exit;
    Tok t;
    if (!parse_tok(in, n, pos, t)) return n;
    pos = t.next;
  }
  return pos;
}

// block-wide exclusive scan; total via *total
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

#define LZ_STAMP(k)                                                                                   \
  do {                                                                                                \
    if (prof && tid == 0) prof[(size_t)blockIdx.x * kLz4ProfWords + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

__global__ __launch_bounds__(kLzThreads) void k_lz4_decode(const Lz4Job* __restrict__ jobs, int32_t* __restrict__ err,
                                                           uint64_t* __restrict__ mtab_all, uint64_t* __restrict__ prof) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kLz4InCap + 16];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kBlockBytes + 64];
  __shared__ int s_job[kMaxJobs][3];
  __shared__ int s_njob, s_bad, s_slow, s_e2hit;
  __shared__ int s_tmp[kLzWaves];

  const Lz4Job job = jobs[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  LZ_STAMP(0);
  const int n = job.src_len;
  if (n <= 0 || n > kLz4InCap) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  uint64_t* mtab = mtab_all + (size_t)blockIdx.x * kLz4MatchTable;
  uint32_t* vb = reinterpret_cast<uint32_t*>(s_out);  // visited bitmap (phases 1-2)
  int* s_x = reinterpret_cast<int*>(s_out + kChunkArrOff);  // speculative exit of each chunk
  int* s_E = s_x + kLzThreads;                              // entry guess of each chunk
  int* s_P = s_E + kLzThreads;                              // exit of each chunk from its entry guess
  int* s_t = s_P + kLzThreads;                              // true entry
  // ---- stage input; clear the visited bitmap ----
  {
    const uint4* src = reinterpret_cast<const uint4*>(job.src);
    uint4* dst = reinterpret_cast<uint4*>(s_in);
    const int n16 = (n + 15) >> 4;
    for (int i = tid; i < n16; i += kLzThreads) dst[i] = src[i];
    if (tid == 0) *reinterpret_cast<uint4*>(s_in + (n16 << 4)) = make_uint4(0, 0, 0, 0);
    const int nw = (n + 32) >> 5;
    for (int i = tid; i < nw; i += kLzThreads) vb[i] = 0;
    if (tid == 0) {
      s_njob = 0;
      s_bad = 0;
      s_slow = 0;
      s_e2hit = 0;
    }
  }
  __syncthreads();
  LZ_STAMP(1);
  // chunking: NC chunks of CH bytes (threads >= NC only help in the cooperative phases)
  const int NC = max(1, min(kLzThreads, n / kMinChunk));
  const int CH = (n + NC - 1) / NC;
  const bool has_chunk = tid < NC;
  const int cs = has_chunk ? min(tid * CH, n) : n, ce = has_chunk ? min(cs + CH, n) : n;

  // ---- 1. speculative walk of my chunk ----
  if (has_chunk) {
    int pos = cs;
    while (pos < ce) {
      atomicOr(&vb[pos >> 5], 1u << (pos & 31));
      Tok t;
      if (!parse_tok(s_in, n, pos, t)) {
        pos = n;
        break;
      }
      pos = t.next;
    }
    s_x[tid] = pos;
  }
  __syncthreads();
  LZ_STAMP(2);
  // ---- 2. entry fix-point: chunk i's entry guess E_i starts as the speculative exit of chunk i-1,
  // P_i = exit of chunk i from E_i; then rounds of E_i <- P_{i-1} (in parallel, re-walking only chunks
  // whose guess changed) until nothing changes or kFixRounds. Chains are functions of position and
  // merge quickly, so a few rounds make nearly every chunk consistent (P_i == E_{i+1}); wave 0 then
  // stitches the true chain from chunk 0, 64 consistent chunks per ballot. ----
  const int x_me = has_chunk ? s_x[tid] : n;
  int myE = n, myP = n;
  if (has_chunk) {
    myE = tid == 0 ? 0 : s_x[tid - 1];
    myP = myE >= ce ? myE : walk_to_exit(s_in, n, myE, ce, vb, x_me);
    s_E[tid] = myE;
    s_P[tid] = myP;
  }
  // Literal-heavy blocks (near-incompressible data: few, long tokens) give speculative chains that
  // rarely merge (a wrong parse lands on a true token start about once per token length); there one
  // lane simply walks the true tokens and records every chunk's entry. Dense blocks with the same
  // first-round inconsistency converge in a few fix-point rounds instead.
  const int inconsistent = __syncthreads_count(has_chunk && tid + 1 < NC && myP != s_E[tid + 1]);
  const bool sequential = inconsistent * kSeqFraction > NC && n * 20 > job.expect_len * 19;
  int fix_rounds = 0;
  if (sequential) {
    if (tid == 0) {
      int pos = 0, k = 0, bad = 0;
      while (pos < n) {
        while (k < NC && k * CH <= pos) s_t[k++] = pos;
        Tok t;
        if (!parse_tok(s_in, n, pos, t)) {
          bad = 1;
          break;
        }
        pos = t.next;
      }
      while (k < NC) s_t[k++] = n;
      s_bad = bad;
      s_slow = 0;
      s_e2hit = -1;
    }
    __syncthreads();
  }
  for (int r = 0; r < kFixRounds && !sequential; ++r) {
    const int newE = (has_chunk && tid > 0) ? s_P[tid - 1] : myE;
    const bool changed = newE != myE;
    __syncthreads();  // every read of s_P precedes this round's writes
    if (changed) {
      myE = newE;
      myP = myE >= ce ? myE : walk_to_exit(s_in, n, myE, ce, vb, x_me);
      s_E[tid] = myE;
      s_P[tid] = myP;
    }
    fix_rounds++;
    if (!__syncthreads_or(changed)) break;
  }
  LZ_STAMP(3);
  if (wave == 0 && !sequential) {
    int cur = 0, i = 0, slow = 0;
    while (i < NC) {
      if (cur == s_E[i]) {
        // a run of consistent chunks: one ballot
        const int idx = i + lane;
        const bool valid = idx < NC;
        const bool ok = valid && (idx == NC - 1 || s_P[idx] == s_E[idx + 1]);
        const unsigned long long badm = __ballot(valid && !ok);
        const int first_bad = badm ? (__ffsll((long long)badm) - 1) : 64;
        const int upto = min(first_bad + 1, NC - i);
        if (lane < upto) s_t[idx] = s_E[idx];
        if (first_bad < 64 && i + first_bad < NC) {
          cur = s_P[i + first_bad];
          i = i + first_bad + 1;
        } else {
          i = min(i + 64, NC);
          cur = s_P[i - 1];
        }
      } else {
        int next_i = i + 1, next_cur = cur;
        if (lane == 0) {
          const int ci_s = min(i * CH, n), ci_e = min(ci_s + CH, n);
          if (cur >= ci_e) {
            // a long token covers whole chunks: they contain no token start
            int j = cur / CH;
            if (j > NC) j = NC;
            if (j <= i) j = i + 1;
            for (int k = i; k < j; ++k) s_t[k] = cur;
            next_i = j;
          } else {
            s_t[i] = cur;
            next_cur = walk_to_exit(s_in, n, cur, ci_e, vb, s_x[i]);
          }
        }
        i = __shfl(next_i, 0, 64);
        cur = __shfl(next_cur, 0, 64);
        slow++;
      }
    }
    if (tid == 0) {
      s_slow = slow;
      s_e2hit = fix_rounds;
    }
  }
  __syncthreads();
  LZ_STAMP(4);
  // ---- 3. sizes of my chunk's true tokens -> output offsets, match-table offsets ----
  const int my_t = has_chunk ? s_t[tid] : n;
  int my_out = 0, my_nm = 0;
  {
    int pos = my_t;
    while (pos < ce) {
      Tok t;
      if (!parse_tok(s_in, n, pos, t)) {
        s_bad = 1;
        break;
      }
      my_out += t.L + t.M;
      my_nm += t.M > 0;
      pos = t.next;
    }
  }
  int total, nmatch;
  const int my_ostart = block_scan_lz(my_out, &total, s_tmp);
  const int my_mstart = block_scan_lz(my_nm, &nmatch, s_tmp);
  if (tid == 0 && (total > kBlockBytes || total < job.expect_len || nmatch > (int)kLz4MatchTable)) s_bad = 1;
  __syncthreads();
  LZ_STAMP(5);
  if (s_bad) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  // ---- 4. literals -> output; matches -> table (the chunk arrays in s_out are dead) ----
  {
    int pos = my_t, o = my_ostart, m = my_mstart;
    while (pos < ce) {
      Tok t;
      parse_tok(s_in, n, pos, t);
      if (t.L <= kLongLit) {
        for (int k = 0; k < t.L; ++k) s_out[o + k] = s_in[t.lit + k];
      } else {
        const int j = atomicAdd(&s_njob, 1);
        if (j < kMaxJobs) {
          s_job[j][0] = t.lit;
          s_job[j][1] = o;
          s_job[j][2] = t.L;
        } else {
          for (int k = 0; k < t.L; ++k) s_out[o + k] = s_in[t.lit + k];
        }
      }
      o += t.L;
      if (t.M > 0) {
        if (t.off > o) s_bad = 1;  // distance before the block start
        mtab[m++] = (uint64_t)o | ((uint64_t)t.off << 16) | ((uint64_t)t.M << 32);
      }
      o += t.M;
      pos = t.next;
    }
  }
  __syncthreads();
  {
    const int nj = min(s_njob, kMaxJobs);
    for (int j = 0; j < nj; ++j) {
      const int li = s_job[j][0], lo = s_job[j][1], ll = s_job[j][2];
      for (int k = tid; k < ll; k += kLzThreads) s_out[lo + k] = s_in[li + k];
    }
  }
  __syncthreads();
  LZ_STAMP(6);
  if (s_bad) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  // ---- 5. matches by pointer jumping, one 32 KiB half of the output at a time ----
  uint16_t* P = reinterpret_cast<uint16_t*>(s_in);  // input is dead; 32 Ki x u16 = 64 KiB
  int jump_rounds = 0;
  for (int lo = 0; lo < total; lo += kHalf) {
    const int hi = min(lo + kHalf, total);
    for (int x = lo + tid; x < hi; x += kLzThreads) P[x - lo] = (uint16_t)x;
    if (tid == 0) s_njob = 0;
    __syncthreads();
    for (int m = my_mstart; m < my_mstart + my_nm; ++m) {
      const uint64_t e = mtab[m];
      const int om = (int)(e & 0xFFFF), off = (int)((e >> 16) & 0xFFFF), M = (int)(e >> 32);
      const int a = max(om, lo), b = min(om + M, hi);
      if (a >= b) continue;
      if (b - a > kLongFill) {
        const int j = atomicAdd(&s_njob, 1);
        if (j < kMaxJobs) {
          s_job[j][0] = om;
          s_job[j][1] = off;
          s_job[j][2] = M;
          continue;
        }
      }
      const int src = om - off;
      if (off >= M) {
        for (int x = a; x < b; ++x) P[x - lo] = (uint16_t)(src + (x - om));
      } else {
        int r = (a - om) % off;
        for (int x = a; x < b; ++x) {
          P[x - lo] = (uint16_t)(src + r);
          if (++r == off) r = 0;
        }
      }
    }
    __syncthreads();
    {
      const int nj = min(s_njob, kMaxJobs);
      for (int j = 0; j < nj; ++j) {
        const int om = s_job[j][0], off = s_job[j][1], M = s_job[j][2];
        const int a = max(om, lo), b = min(om + M, hi), src = om - off;
        if (off >= M) {
          for (int x = a + tid; x < b; x += kLzThreads) P[x - lo] = (uint16_t)(src + (x - om));
        } else {
          const int step = kLzThreads % off;
          int r = (a + tid - om) % off;
          for (int x = a + tid; x < b; x += kLzThreads) {
            P[x - lo] = (uint16_t)(src + r);
            r += step;
            if (r >= off) r -= off;
          }
        }
      }
    }
    __syncthreads();
    // P[x] <- P[P[x]] until every pointer is a root (a literal byte of this half, or a byte of an
    // earlier half, which is final); asynchronous updates only make pointers jump further.
    // kJumpBatch chases per thread are issued together so their LDS latencies overlap.
    for (int r = 0;; ++r) {
      int changed = 0;
      for (int x0 = lo + tid; x0 < hi; x0 += kLzThreads * kJumpBatch) {
        int p[kJumpBatch], pp[kJumpBatch];
#pragma unroll
        for (int k = 0; k < kJumpBatch; ++k) {
          const int x = x0 + k * kLzThreads;
          p[k] = x < hi ? (int)P[x - lo] : x;
        }
#pragma unroll
        for (int k = 0; k < kJumpBatch; ++k) {
          const int x = x0 + k * kLzThreads;
          pp[k] = (p[k] >= lo && p[k] != x) ? (int)P[p[k] - lo] : p[k];
        }
#pragma unroll
        for (int k = 0; k < kJumpBatch; ++k) {
          const int x = x0 + k * kLzThreads;
          if (pp[k] != p[k]) {
            P[x - lo] = (uint16_t)pp[k];
            changed = 1;
          }
        }
      }
      jump_rounds++;
      if (!__syncthreads_or(changed)) break;
      if (r >= kMaxJumpRounds) {
        if (tid == 0) atomicOr(err, 1);
        return;
      }
    }
    for (int x = lo + tid; x < hi; x += kLzThreads) {
      const int p = P[x - lo];
      if (p != x) s_out[x] = s_out[p];
    }
    __syncthreads();
  }
  LZ_STAMP(7);
  if (prof && tid == 0) {
    uint64_t* pr = prof + (size_t)blockIdx.x * kLz4ProfWords;
    pr[8] = (uint64_t)jump_rounds;
    pr[9] = (uint64_t)n;
    pr[10] = (uint64_t)s_slow;
    pr[11] = (uint64_t)s_e2hit;
  }
  // ---- 6. write the decoded block ----
  uint4* dst = reinterpret_cast<uint4*>(job.dst);
  const uint4* srco = reinterpret_cast<const uint4*>(s_out);
  const int n16 = (total + 15) >> 4;
  for (int i = tid; i < n16; i += kLzThreads) dst[i] = srco[i];
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


void launch_lz4_decode(const Lz4Job* d_jobs, int njobs, int32_t* d_err, uint64_t* d_mtab, hipStream_t s,
                       uint64_t* d_prof) {
  if (njobs <= 0) return;
  static const bool seq = getenv("DG_LZ4_SEQ") && getenv("DG_LZ4_SEQ")[0] == '1';
  if (seq) hipLaunchKernelGGL(k_lz4_decode_seq, dim3(njobs), dim3(64), 0, s, d_jobs, d_err);
  else hipLaunchKernelGGL(k_lz4_decode, dim3(njobs), dim3(kLzThreads), 0, s, d_jobs, d_err, d_mtab, d_prof);
}

}  // namespace dg
