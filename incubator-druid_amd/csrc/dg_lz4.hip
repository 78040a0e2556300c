// dg_lz4.hip — LZ4 block decompression on gfx950 (Druid's per-block column codec).
//
// Replaces CompressionStrategy.LZ4Decompressor.decompress (processing/.../segment/data/
// CompressionStrategy.java:284-305 -> lz4-java 1.4.0 LZ4SafeDecompressor): one 64 KiB Druid block
// (CompressedPools.BUFFER_SIZE) per workgroup, compressed input and decoded output both in LDS.
//
// LZ4's token stream is sequential (a token's position depends on every earlier token) and Druid's
// numeric blocks are token-dense (~8k tokens / block for sequential longs), so one lane walking the
// stream is latency-bound (measured: ~2 ms per block). This kernel parses speculatively in parallel:
//   1. the compressed block is cut into 256 chunks; thread i walks the token chain from the start of
//      chunk i as if a token started there, marking the positions it visits (LDS bitmap);
//   2. the true chain enters chunk i at the exit of chunk i-1; walking from there, it meets the
//      speculative chain within a few tokens (chains are functions of position, so they merge) —
//      checked in parallel, with a wave-level fix-up where an entry guess was wrong (long tokens);
//   3. each thread re-walks its chunk's true tokens: output sizes -> block scan -> output offsets;
//   4. literals are copied (long runs cooperatively);
//   5. matches are resolved in rounds: a match runs once every byte it copies from is final
//      (per-chunk "done" frontiers); matches longer than kLongMatch are copied by the whole block.
// The sequential one-wave decoder is kept (k_lz4_decode_seq) as a differential reference and
// selected with DG_LZ4_SEQ=1.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "dg_internal.h"

namespace dg {

constexpr int kLzThreads = 256;
constexpr int kLz4InCap = kBlockBytes + 2048;  // LZ4_compressBound(65536) = 65809
constexpr int kLongLit = 48;                   // literal runs above this are copied cooperatively
constexpr int kLongMatch = 48;                 // matches above this are copied cooperatively
constexpr int kMaxLitJobs = 512;
constexpr int kMaxRounds = 1 << 16;

struct Tok {
  int lit;   // literal start (input offset)
  int L;     // literal length
  int off;   // match offset (0 for the last sequence)
  int M;     // match length (0 for the last sequence)
  int next;  // next token start
};

// Parse the token starting at p. false = not a valid token here (speculative walks just stop).
__device__ __forceinline__ bool parse_tok(const uint8_t* __restrict__ in, int n, int p, Tok& t) {
  if (p >= n) return false;
  const int tk = in[p];
  int q = p + 1;
  int L = tk >> 4;
  if (L == 15) {
    int b;
    do {
      if (q >= n) return false;
      b = in[q++];
      L += b;
    } while (b == 255);
  }
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
  if (M == 15) {
    int b;
    do {
      if (q >= n) return false;
      b = in[q++];
      M += b;
    } while (b == 255);
  }
  t.M = M + 4;
  t.next = q;
  return t.off != 0;
}

// block-wide (256 threads) exclusive scan of int; total via *total
__device__ int64_t block_exclusive_scan_lz(int v, int64_t* total, int64_t* s_tmp) {
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
  for (int w = 0; w < (kLzThreads >> 6); ++w) {
    if (w < wave) wave_off += s_tmp[w];
    tot += s_tmp[w];
  }
  __syncthreads();
  *total = tot;
  return wave_off + x - v;
}

__global__ __launch_bounds__(kLzThreads) void k_lz4_decode(const Lz4Job* __restrict__ jobs, int32_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kLz4InCap];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kBlockBytes + 64];
  __shared__ int s_x[kLzThreads];       // speculative exit of each chunk
  __shared__ int s_pexit[kLzThreads];   // true exit assuming entry = s_x[i-1]
  __shared__ int s_t[kLzThreads];       // true entry
  __shared__ int s_ostart[kLzThreads + 1];
  __shared__ int s_done[kLzThreads];    // output bytes of chunk i below this are final
  __shared__ uint16_t s_chunk_at[kBlockBytes / 64 + 1];
  __shared__ int s_lit_job[kMaxLitJobs][3];
  __shared__ int s_m_job[kLzThreads][3];
  __shared__ int s_nlit, s_nm, s_bad;
  __shared__ int64_t s_scan_tmp[8];

  const Lz4Job job = jobs[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = job.src_len;
  if (n <= 0 || n > kLz4InCap) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  // ---- stage input, clear the visited bitmap (aliases the output buffer) ----
  {
    const uint4* src = reinterpret_cast<const uint4*>(job.src);
    uint4* dst = reinterpret_cast<uint4*>(s_in);
    const int n16 = (n + 15) >> 4;
    for (int i = tid; i < n16; i += kLzThreads) dst[i] = src[i];
    uint32_t* vb = reinterpret_cast<uint32_t*>(s_out);
    const int nw = (n + 32) >> 5;
    for (int i = tid; i < nw; i += kLzThreads) vb[i] = 0;
    if (tid == 0) {
      s_nlit = 0;
      s_nm = 0;
      s_bad = 0;
    }
  }
  __syncthreads();
  uint32_t* vb = reinterpret_cast<uint32_t*>(s_out);
  const int CH = (n + kLzThreads - 1) / kLzThreads;
  const int cs = min(tid * CH, n), ce = min(cs + CH, n);

  // ---- 1. speculative walk of my chunk ----
  {
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
  // ---- 2a. walk from the assumed entry until the speculative chain is met ----
  {
    const int a = tid == 0 ? 0 : s_x[tid - 1];
    int pos = a;
    if (pos < ce) {
      while (pos < ce) {
        if ((vb[pos >> 5] >> (pos & 31)) & 1u) {
          pos = s_x[tid];
          break;
        }
        Tok t;
        if (!parse_tok(s_in, n, pos, t)) {
          pos = n;
          break;
        }
        pos = t.next;
      }
    }
    s_pexit[tid] = pos;
  }
  __syncthreads();
  // ---- 2b. resolve true entries (wave 0; a run of consistent chunks is one ballot) ----
  if (wave == 0) {
    int cur = 0, i = 0;
    while (i < kLzThreads) {
      const int assumed = i == 0 ? 0 : s_x[i - 1];
      if (cur == assumed) {
        const int idx = i + lane;
        const bool valid = idx < kLzThreads;
        const bool ok = valid && s_pexit[idx] == s_x[idx];
        const unsigned long long badm = __ballot(valid && !ok);
        const int first_bad = badm ? (__ffsll((long long)badm) - 1) : 64;
        const int upto = min(first_bad + 1, kLzThreads - i);  // chunks i .. i+upto-1 get t = assumed
        if (lane < upto) s_t[idx] = idx == 0 ? 0 : s_x[idx - 1];
        if (first_bad < 64 && i + first_bad < kLzThreads) {
          cur = s_pexit[i + first_bad];
          i = i + first_bad + 1;
        } else {
          i = min(i + 64, kLzThreads);
          cur = s_x[i - 1];
        }
      } else {
        int next_i = i + 1, next_cur = cur;
        if (lane == 0) {
          const int ci_s = min(i * CH, n), ci_e = min(ci_s + CH, n);
          if (cur >= ci_e) {
            // a token spans the whole chunk: every chunk ending at or before cur has no token start
            int j = CH > 0 ? cur / CH : kLzThreads;
            if (j > kLzThreads) j = kLzThreads;
            if (j <= i) j = i + 1;
            for (int k = i; k < j; ++k) s_t[k] = cur;
            next_i = j;
          } else {
            s_t[i] = cur;
            int pos = cur;
            while (pos < ci_e) {
              if ((vb[pos >> 5] >> (pos & 31)) & 1u) {
                pos = s_x[i];
                break;
              }
              Tok t;
              if (!parse_tok(s_in, n, pos, t)) {
                pos = n;
                break;
              }
              pos = t.next;
            }
            next_cur = pos;
          }
        }
        i = __shfl(next_i, 0, 64);
        cur = __shfl(next_cur, 0, 64);
      }
    }
  }
  __syncthreads();
  // ---- 3. output size of my chunk's true tokens -> block scan ----
  const int my_t = s_t[tid];
  int my_out = 0;
  {
    int pos = my_t;
    while (pos < ce) {
      Tok t;
      if (!parse_tok(s_in, n, pos, t)) {
        s_bad = 1;
        break;
      }
      my_out += t.L + t.M;
      pos = t.next;
    }
  }
  int64_t total64;
  const int my_ostart = (int)block_exclusive_scan_lz(my_out, &total64, s_scan_tmp);
  const int total = (int)total64;
  s_ostart[tid] = my_ostart;
  if (tid == 0) s_ostart[kLzThreads] = total;
  if (total > kBlockBytes || total < job.expect_len) s_bad = 1;
  __syncthreads();
  if (s_bad) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  // chunk lookup table over 64-byte output granules (output ranges partition [0, total))
  for (int g = (my_ostart + 63) >> 6; (g << 6) < my_ostart + my_out; ++g) s_chunk_at[g] = (uint16_t)tid;
  // ---- 4. literals (the visited bitmap in s_out is dead from here) ----
  int first_match_out = my_ostart + my_out;
  {
    int pos = my_t, o = my_ostart;
    bool seen_match = false;
    while (pos < ce) {
      Tok t;
      parse_tok(s_in, n, pos, t);
      if (t.L <= kLongLit) {
        for (int k = 0; k < t.L; ++k) s_out[o + k] = s_in[t.lit + k];
      } else {
        const int j = atomicAdd(&s_nlit, 1);
        if (j < kMaxLitJobs) {
          s_lit_job[j][0] = t.lit;
          s_lit_job[j][1] = o;
          s_lit_job[j][2] = t.L;
        } else {
          for (int k = 0; k < t.L; ++k) s_out[o + k] = s_in[t.lit + k];
        }
      }
      if (!seen_match && t.M > 0) {
        first_match_out = o + t.L;
        seen_match = true;
      }
      o += t.L + t.M;
      pos = t.next;
    }
  }
  __syncthreads();
  {
    const int nj = min(s_nlit, kMaxLitJobs);
    for (int j = 0; j < nj; ++j) {
      const int li = s_lit_job[j][0], lo = s_lit_job[j][1], ll = s_lit_job[j][2];
      for (int k = tid; k < ll; k += kLzThreads) s_out[lo + k] = s_in[li + k];
    }
  }
  s_done[tid] = first_match_out;
  __syncthreads();
  // ---- 5. matches in rounds ----
  volatile int* vdone = s_done;
  int pos = my_t, o = my_ostart;
  bool have = false, waiting = false, finished = pos >= ce;
  Tok t;
  int rounds = 0;
  for (;;) {
    while (!finished && !waiting) {
      if (!have) {
        parse_tok(s_in, n, pos, t);
        have = true;
      }
      if (t.M == 0) {  // last sequence
        o += t.L;
        pos = t.next;
        have = false;
        if (pos >= ce) finished = true;
        continue;
      }
      const int om = o + t.L;
      const int src = om - t.off;
      if (src < 0) {
        s_bad = 1;
        finished = true;
        break;
      }
      // bytes [src, src + min(off, M)) must be final; those of my own chunk are (in-order processing)
      const int need_end = min(src + min(t.off, t.M), my_ostart);
      bool ready = true;
      int xq = src;
      while (xq < need_end) {
        int c = s_chunk_at[xq >> 6];
        while (s_ostart[c + 1] <= xq) c++;
        const int cend = s_ostart[c + 1];
        const int want = min(need_end, cend);
        if (vdone[c] < want) {
          ready = false;
          break;
        }
        xq = cend;
      }
      if (!ready) break;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      if (t.M > kLongMatch) {
        const int j = atomicAdd(&s_nm, 1);
        s_m_job[j][0] = om;
        s_m_job[j][1] = t.off;
        s_m_job[j][2] = t.M;
        waiting = true;
        break;
      }
      if (t.off >= t.M) {
        for (int k = 0; k < t.M; ++k) s_out[om + k] = s_out[src + k];
      } else {
        for (int k = 0; k < t.M; ++k) s_out[om + k] = s_out[src + (k % t.off)];
      }
      o = om + t.M;
      pos = t.next;
      have = false;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      vdone[tid] = o;
      if (pos >= ce) finished = true;
    }
    __syncthreads();
    const int nm = s_nm;
    for (int j = 0; j < nm; ++j) {
      const int mo = s_m_job[j][0], moff = s_m_job[j][1], mlen = s_m_job[j][2];
      const int msrc = mo - moff;
      if (moff >= mlen) {
        for (int k = tid; k < mlen; k += kLzThreads) s_out[mo + k] = s_out[msrc + k];
      } else {
        for (int k = tid; k < mlen; k += kLzThreads) s_out[mo + k] = s_out[msrc + (k % moff)];
      }
    }
    __syncthreads();
    if (waiting) {
      o = o + t.L + t.M;
      pos = t.next;
      have = false;
      waiting = false;
      vdone[tid] = o;
      if (pos >= ce) finished = true;
    }
    if (tid == 0) s_nm = 0;
    if (finished) vdone[tid] = my_ostart + my_out;
    const int pending = __syncthreads_count(!finished);
    if (pending == 0) break;
    if (++rounds > kMaxRounds) {
      if (tid == 0) atomicOr(err, 1);
      return;
    }
  }
  if (s_bad) {
    if (tid == 0) atomicOr(err, 1);
    return;
  }
  // ---- 6. write the decoded block ----
  uint4* dst = reinterpret_cast<uint4*>(job.dst);
  const uint4* srco = reinterpret_cast<const uint4*>(s_out);
  const int n16 = (total + 15) >> 4;
  for (int i = tid; i < n16; i += kLzThreads) dst[i] = srco[i];
}

// ------------------------------------------------------------------------------------------------
// Sequential reference decoder (DG_LZ4_SEQ=1): one wave per block, compressed input and decoded output staged in LDS.
// Tokens are parsed in order (the format is sequential); literal and match copies are spread over
// the 64 lanes. Overlapping matches (offset < length) use the periodic form
// out[op + k] = out[op - off + k % off], which only reads bytes before op, so the lanes never race.
// ------------------------------------------------------------------------------------------------

__global__ __launch_bounds__(64) void k_lz4_decode_seq(const Lz4Job* __restrict__ jobs, int32_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) uint8_t s_in[kLz4InCap];
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


void launch_lz4_decode(const Lz4Job* d_jobs, int njobs, int32_t* d_err, hipStream_t s) {
  if (njobs <= 0) return;
  static const bool seq = getenv("DG_LZ4_SEQ") && getenv("DG_LZ4_SEQ")[0] == '1';
  if (seq) hipLaunchKernelGGL(k_lz4_decode_seq, dim3(njobs), dim3(64), 0, s, d_jobs, d_err);
  else hipLaunchKernelGGL(k_lz4_decode, dim3(njobs), dim3(kLzThreads), 0, s, d_jobs, d_err);
}

}  // namespace dg
