// dg_segment.cpp — v9 segment loader: parses the on-disk format on the host and builds the
// device-resident columnar image in HBM.
//
// Format followed (reference paths, processing/... = processing/src/main/java/org/apache/druid/...):
//   version.bin / meta.smoosh / NNNNN.smoosh   IndexIO.V9IndexLoader.load (segment/IndexIO.java:569-663),
//                                              SmooshedFileMapper (java-util/.../io/smoosh/SmooshedFileMapper.java)
//   index.drd                                  cols, dims (GenericIndexed<String>), interval, bitmap serde JSON
//   column = int32 BE json length + ColumnDescriptor JSON + part (IndexIO.java:665-672)
//   GenericIndexed v1                          data/GenericIndexed.java:52-77, 479-492
//   long/float/double part                     data/CompressedColumnar{Longs,Floats}Supplier.fromByteBuffer,
//                                              CompressedColumnarDoublesSuppliers (+ CompressionFactory flag logic
//                                              data/CompressionFactory.java:64-116); V2 serdes skip their int offset +
//                                              null bitmap (serde/DoubleGenericColumnPartSerdeV2.java:140-162)
//   stringDictionary part                      serde/DictionaryEncodedColumnPartSerde.java:283-345,
//                                              data/CompressedVSizeColumnarIntsSupplier.java:143-168
//
// Device image (all HBM, built once at attach; queries never touch the files again):
//   LZ4 blocks        packed, each block 16-byte aligned, + host offset/length tables
//   UNCOMPRESSED      one 64 KiB-aligned slot per block (so every value is naturally aligned)
//   NONE              the flat value array
//   bitmaps           every dictionary value's serialized Concise/Roaring bytes, 4-byte aligned
//   dictionaries      host-side (filters resolve on the host like BitmapIndexSelector does)
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

#include "dg_internal.h"

namespace dg {


namespace {

int32_t be32(const uint8_t* p) {
  return (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
}
int64_t be64(const uint8_t* p) { return ((int64_t)(uint32_t)be32(p) << 32) | (uint32_t)be32(p + 4); }

struct MappedFile {
  void* base = nullptr;
  size_t size = 0;
  ~MappedFile() {
    if (base && base != MAP_FAILED) munmap(base, size);
  }
  bool open(const std::string& path) {
    int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) {
      ::close(fd);
      return false;
    }
    size = (size_t)st.st_size;
    if (size == 0) {
      ::close(fd);
      base = nullptr;
      return true;
    }
    base = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    return base != MAP_FAILED;
  }
  const uint8_t* data() const { return static_cast<const uint8_t*>(base); }
};

struct Slice {
  const uint8_t* p = nullptr;
  const uint8_t* end = nullptr;
  int64_t left() const { return end - p; }
};

// GenericIndexed v1 view
// Element i occupies [end[i-1] + 4, end[i]) of the values region (the 4 bytes skipped are the
// element's length prefix, GenericIndexed.java:479-492); offsets read from the file are checked
// against the region the header declares (numBytesUsed), so a truncated or corrupt segment is a
// format error (the reference's IAE/ISE), never an out-of-bounds read.
struct GI {
  int32_t n = 0;
  int64_t size = 0;  // bytes of the values region
  const uint8_t* header = nullptr;
  const uint8_t* values = nullptr;
  // length of element i (0 = null / empty), or -1 when its offsets are outside the region
  int32_t get(int32_t i, const uint8_t** ptr) const {
    *ptr = values;
    if (i < 0 || i >= n) return -1;
    const int64_t start = i == 0 ? 4 : (int64_t)be32(header + 4 * (i - 1)) + 4;
    const int64_t end = be32(header + 4 * i);
    if (start < 4 || start > size || end < start - 4 || end > size) return -1;
    if (end < start) return 0;  // an empty element directly after a length prefix of 0
    *ptr = values + start;
    return (int32_t)(end - start);
  }
};

bool gi_read(Slice& s, GI* g) {
  if (s.left() < 6) return false;
  if (s.p[0] != 0x01) return false;  // version 2 (multi-file, > 2 GiB columns) not supported
  int32_t used = be32(s.p + 2);
  const uint8_t* body = s.p + 6;
  if (used < 4 || s.end - body < used) return false;
  g->n = be32(body);
  if (g->n < 0 || 4 + 4 * (int64_t)g->n > used) return false;
  g->header = body + 4;
  g->values = body + 4 + 4 * (int64_t)g->n;
  g->size = (int64_t)used - 4 - 4 * (int64_t)g->n;
  s.p = body + used;
  return true;
}

// tiny JSON probe: value of "key" at/after `from`
std::string json_get(const std::string& js, const char* key, size_t from = 0) {
  std::string pat = std::string("\"") + key + "\":";
  size_t k = js.find(pat, from);
  if (k == std::string::npos) return "";
  k += pat.size();
  while (k < js.size() && js[k] == ' ') k++;
  if (k < js.size() && js[k] == '"') {
    size_t e = js.find('"', k + 1);
    return js.substr(k + 1, e - k - 1);
  }
  size_t e = k;
  while (e < js.size() && js[e] != ',' && js[e] != '}') e++;
  return js.substr(k, e - k);
}

int log2i(int32_t v) {
  int l = 0;
  while ((1 << l) < v) l++;
  return (1 << l) == v ? l : -1;
}

}  // namespace

// Validating parse of one LZ4 block (the checks of lz4-java's LZ4SafeDecompressor / liblz4's
// LZ4_decompress_safe: lengths inside the input, match distance inside the output produced so far,
// output within one 64 KiB Druid block, CompressedPools.java:39). Records the token offset of every
// kLzSeqPerCp-th sequence; a block with more than kLzMaxCps such checkpoints keeps every other one
// (intervals of 2 * kLzSeqPerCp sequences), and one that still has more is rejected. A general
// (not light) block with fewer sequences gets intervals of ceil(sequences / kLzMaxCps) instead.
// Longest copy chain of a validated block: a literal byte has depth 0, a match byte one more than the
// byte it copies (overlapping matches copy from the match's first period). Stops above `cap`.
static int lz4_max_depth(const uint8_t* in, int n, int cap) {
  thread_local std::vector<uint8_t> dep(kBlockBytes);
  int pos = 0, out = 0, mx = 0;
  auto ext = [&](int* len) {
    for (int b = 255; b == 255 && pos < n;) {
      b = in[pos++];
      *len += b;
    }
  };
  for (;;) {
    const int tok = in[pos++];
    int L = tok >> 4;
    if (L == 15) ext(&L);
    memset(dep.data() + out, 0, (size_t)L);
    out += L;
    pos += L;
    if (pos >= n) return mx;
    const int off = in[pos] | (in[pos + 1] << 8);
    pos += 2;
    int M = tok & 15;
    if (M == 15) ext(&M);
    M += 4;
    for (int k = 0, r = 0; k < M; ++k) {
      const int src = off >= M ? out + k - off : out - off + r;
      const int v = dep[src] + 1;
      if (v > cap) return v;
      dep[out + k] = (uint8_t)v;
      mx = std::max(mx, v);
      if (++r == off) r = 0;
    }
    out += M;
  }
}

// The flow decoder's schedule of a validated block (kLzSeqPerCp sequences per checkpoint interval, g of
// them used). Source forwarding: a match (not overlapping itself) whose source lies entirely inside the
// output of one earlier such match copies the same bytes from that match's source, repeatedly — LZ4 HC
// chains a 4-byte pattern through every earlier occurrence, so this shortens the chains (noisy doubles:
// 24 -> 8 levels). Every match then gets its copy-chain level — one more than the highest level among
// the bytes of its (forwarded) source; literal bytes are level 0 — and its rank in the block's matches
// ordered by (level, position). Appended per interval (kFlowRecBytes): kLzSeqPerCp u16 ranks (0xFFFF: no
// match), kLzSeqPerCp u16 forwarded distances and kLzSeqPerCp u16 token offsets from the interval's
// first token (0xFFFF: no such sequence; the decoder parses an interval's tokens independently); then the u16
// start of every level's ranks (nlvl + 1 of them, zero padded to 16 bytes). Returns the highest level,
// or -1 above `cap` or when a token lies 64 KiB or more past its interval's first (nothing appended).
static int lz4_flow_schedule(const uint8_t* in, int n, int64_t g, int cap, std::vector<uint8_t>* lv) {
  struct Mt {
    int om, M, fsrc, d;
  };
  thread_local std::vector<uint8_t> lev(kBlockBytes);
  thread_local std::vector<int32_t> owner(kBlockBytes);  // the match that produced a byte, -1: a literal
  thread_local std::vector<Mt> ms;
  thread_local std::vector<int32_t> seqm;  // per sequence: its match's index in ms, -1: none
  thread_local std::vector<int32_t> seqp;  // per sequence: its token's offset
  ms.clear();
  seqm.clear();
  seqp.clear();
  int pos = 0, out = 0, mx = 0;
  auto ext = [&](int* len) {
    for (int b = 255; b == 255 && pos < n;) {
      b = in[pos++];
      *len += b;
    }
  };
  for (;;) {
    seqp.push_back(pos);
    const int tok = in[pos++];
    int L = tok >> 4;
    if (L == 15) ext(&L);
    memset(lev.data() + out, 0, (size_t)L);
    std::fill(owner.begin() + out, owner.begin() + out + L, -1);
    out += L;
    pos += L;
    if (pos >= n) {
      seqm.push_back(-1);
      break;
    }
    const int off = in[pos] | (in[pos + 1] << 8);
    pos += 2;
    int M = tok & 15;
    if (M == 15) ext(&M);
    M += 4;
    int src = out - off;
    if (off >= M) {  // forward through earlier non-overlapping matches holding the whole source
      for (;;) {
        const int j = owner[src];
        if (j < 0 || ms[j].d < ms[j].M || src + M > ms[j].om + ms[j].M) break;
        src = ms[j].fsrc + (src - ms[j].om);
      }
    }
    const int span = std::min(out - src, M);
    int v = 0;
    for (int k = 0; k < span; ++k) v = std::max(v, (int)lev[src + k]);
    if (++v > cap) return -1;
    memset(lev.data() + out, v, (size_t)M);
    std::fill(owner.begin() + out, owner.begin() + out + M, (int32_t)ms.size());
    seqm.push_back((int32_t)ms.size());
    ms.push_back(Mt{out, M, src, off});
    mx = std::max(mx, v);
    out += M;
  }
  std::vector<int> cnt(mx + 2, 0);
  for (const Mt& m : ms) cnt[lev[m.om]]++;
  std::vector<uint16_t> next(mx + 2, 0), st(mx + 1, 0);
  for (int k = 1, acc = 0; k <= mx; ++k) {
    next[k] = (uint16_t)acc;
    acc += cnt[k];
    st[k] = (uint16_t)acc;  // st[k - 1] .. st[k]: the ranks of level k
  }
  const int64_t m = ((int64_t)seqm.size() + g - 1) / g;
  for (int64_t i = 0; i < m; ++i)  // token offsets as u16 deltas from the interval's first token
    for (int64_t q = 1; q < g && i * g + q < (int64_t)seqp.size(); ++q)
      if (seqp[i * g + q] - seqp[i * g] >= 0xFFFF) return -1;
  const size_t at = lv->size(), rec = kFlowRecBytes;  // per interval: ranks, distances, token deltas, levels
  lv->resize(at + (size_t)m * rec + (((size_t)(mx + 1) * 2 + 15) & ~(size_t)15), 0);
  for (int64_t i = 0; i < m; ++i)
    for (int q = 0; q < kLzSeqPerCp; ++q) {
      uint16_t* r = reinterpret_cast<uint16_t*>(lv->data() + at + (size_t)i * rec);
      const int64_t sq = i * g + q;
      const bool here = q < g && sq < (int64_t)seqm.size();
      const int j = here ? seqm[sq] : -1;
      r[q] = j < 0 ? (uint16_t)0xFFFF : next[lev[ms[j].om]]++;
      r[kLzSeqPerCp + q] = j < 0 ? (uint16_t)0 : (uint16_t)(ms[j].om - ms[j].fsrc);
      r[2 * kLzSeqPerCp + q] = here ? (uint16_t)(seqp[sq] - seqp[i * g]) : (uint16_t)0xFFFF;
    }
  memcpy(lv->data() + at + (size_t)m * rec, st.data(), (size_t)(mx + 1) * 2);
  return mx;
}

int lz4_index_block(const uint8_t* in, int n, std::vector<uint32_t>* cps, int* wide, int* light, int* nfine,
                    std::vector<uint8_t>* levels, int* nlvl) {
  if (nlvl) *nlvl = 0;
  const size_t first = cps->size();
  if (light) *light = 0;
  if (nfine) *nfine = 0;
  int pos = 0, out = 0;
  int64_t seq = 0, c8 = 0;  // c8: bytes copied from 8 back (distance-8 class chains)
  auto ext = [&](int* len) {
    for (;;) {
      if (pos >= n) return false;
      const int b = in[pos++];
      *len += b;
      if (b != 255) return true;
    }
  };
  *wide = 0;
  // checkpoints every g sequences from the block's start (appended after cps[first + ...])
  auto push_every = [&](int64_t g) {
    int p = 0, m = 0;
    for (int64_t k = 0; k < seq; ++k) {
      if (k % g == 0) {
        cps->push_back((uint32_t)p);
        ++m;
      }
      const int tok = in[p++];
      int L = tok >> 4;
      if (L == 15) for (int b = 255; b == 255;) L += (b = in[p++]);
      p += L;
      if (p >= n) break;
      p += 2;
      if ((tok & 15) == 15) for (int b = 255; b == 255;) b = in[p++];
    }
    return m;
  };
  auto finish = [&](int dec) {
    size_t m = cps->size() - first;
    if (m > (size_t)kLzMaxCps) {
      *wide = 1;
      for (size_t i = 0; 2 * i < m; ++i) (*cps)[first + i] = (*cps)[first + 2 * i];
      m = (m + 1) / 2;
      cps->resize(first + m);
    }
    if (m > (size_t)kLzMaxCps) return -1;
    if (light && !*wide && m <= (size_t)kLtMaxCps && lz4_max_depth(in, n, kLtMaxDepth) <= kLtMaxDepth) {
      // light checkpoints: every g sequences, the fewest that fit one per light-decoder thread
      const int g = (int)std::max<int64_t>(1, (seq + kLtThreads - 1) / kLtThreads);
      if (nfine && g <= kLzSeqPerCp) {
        *nfine = push_every(g);
        *light = g;
      } else if (!nfine) {
        *light = 1;
      }
    }
    int64_t gi = *wide ? kLzMaxSeqPerCp : kLzSeqPerCp;  // sequences per checkpoint interval
    if (!*wide && !(light && *light)) {
      // a general block of fewer than kLzMaxCps * kLzSeqPerCp sequences: intervals of the fewest
      // sequences that still give one per decoder thread, so every wave parses and fills
      const int64_t g = std::max<int64_t>(1, (seq + kLzMaxCps - 1) / kLzMaxCps);
      if (g < kLzSeqPerCp) {
        cps->resize(first);
        push_every(g);
        gi = g;
      }
    }
    // a general block (not wide) that is not a class chain and whose copy chains are short: the flow
    // decoder, with its schedule
    if (levels && !*wide && !(light && *light) && c8 * 4 <= dec) {
      const int mx = lz4_flow_schedule(in, n, gi, kFlowMaxDepth, levels);
      if (mx >= 0) {
        *wide |= kLzFlow;
        if (nlvl) *nlvl = mx;
      }
    }
    return dec;
  };
  for (;;) {
    if (seq % kLzSeqPerCp == 0) cps->push_back((uint32_t)pos);
    seq++;
    if (pos >= n) return -1;
    const int tok = in[pos++];
    int L = tok >> 4;
    if (L == 15 && !ext(&L)) return -1;
    if (L > n - pos || L > kBlockBytes - out) return -1;
    pos += L;
    out += L;
    if (pos == n) return finish(out);  // last sequence: literals only
    if (n - pos < 2) return -1;
    const int off = in[pos] | (in[pos + 1] << 8);
    pos += 2;
    int M = tok & 15;
    if (M == 15 && !ext(&M)) return -1;
    M += 4;
    if (off == 0 || off > out || M > kBlockBytes - out) return -1;
    out += M;
    if (off == 8) c8 += M;
  }
}

int lz4_decode_host(const uint8_t* in, int n, uint8_t* out) {
  int pos = 0, o = 0;
  auto ext = [&](int* len) {
    for (;;) {
      if (pos >= n) return false;
      const int b = in[pos++];
      *len += b;
      if (b != 255) return true;
    }
  };
  for (;;) {
    if (pos >= n) return -1;
    const int t = in[pos++];
    int L = t >> 4;
    if (L == 15 && !ext(&L)) return -1;
    if (L > n - pos || L > kBlockBytes - o) return -1;
    memcpy(out + o, in + pos, (size_t)L);
    pos += L;
    o += L;
    if (pos == n) return o;
    if (n - pos < 2) return -1;
    const int d = in[pos] | (in[pos + 1] << 8);
    pos += 2;
    int M = t & 15;
    if (M == 15 && !ext(&M)) return -1;
    M += 4;
    if (d == 0 || d > o || M > kBlockBytes - o) return -1;
    for (int k = 0; k < M; ++k) out[o + k] = out[o + k - d];
    o += M;
  }
}

int lz4_literal_start(const uint8_t* in, int n) {
  if (n < 2) return -1;
  int q = 1, L = in[0] >> 4;
  if (in[0] & 15) return -1;  // (a match length: not the block's only, last sequence)
  if (L == 15) {
    for (int b = 255; b == 255;) {
      if (q >= n) return -1;
      b = in[q++];
      L += b;
    }
  }
  return L > 0 && L <= kBlockBytes && q + L == n ? q : -1;
}

int decode_routes() {
  auto off = [](const char* v) {
    const char* e = getenv(v);
    return e && *e && *e != '0';
  };
  return (off("DG_NO_RUN_DECODE") ? 0 : kRouteRun) | (off("DG_NO_FLOW_DECODE") ? 0 : kRouteFlow);
}

// The run index of a validated block (layout: dg_internal.h, kRunThreads): the block is decoded once
// on the host, cut into intervals of at least kRunTarget output bytes at sequence starts, and every
// interval records its token offset, its output start and the 8 output bytes before it; the bytes
// of matches reaching further back than 8 bytes (far copies) are listed in sequence order.
bool lz4_run_index(const uint8_t* in, int n, int dec_len, std::vector<uint8_t>* idx, int* nint, int* nfar) {
  *nint = 0;
  *nfar = 0;
  if (dec_len <= 0 || dec_len % 8 || dec_len > kBlockBytes || run_lds_bytes(n, 0) > kRunLdsMax) return false;
  thread_local std::vector<uint8_t> out(kBlockBytes);
  std::vector<uint64_t> win;
  std::vector<uint32_t> tok;
  std::vector<uint16_t> ost;
  std::vector<uint8_t> far;
  int pos = 0, o = 0, cur = 0;
  auto ext = [&](int* len) {
    for (;;) {
      if (pos >= n) return false;
      const int b = in[pos++];
      *len += b;
      if (b != 255) return true;
    }
  };
  for (bool first = true;; first = false) {
    if (first || o - cur >= kRunTarget) {  // a new interval at this sequence
      cur = o;
      uint64_t w = 0;
      if (o >= 8) memcpy(&w, out.data() + o - 8, 8);
      win.push_back(w);
      tok.push_back((uint32_t)pos | ((uint32_t)far.size() << 17));
      ost.push_back((uint16_t)o);
    }
    if (pos >= n) return false;
    const int t = in[pos++];
    int L = t >> 4;
    if (L == 15 && !ext(&L)) return false;
    if (L > kRunMaxRun || L > n - pos || L > dec_len - o) return false;
    memcpy(out.data() + o, in + pos, (size_t)L);
    pos += L;
    o += L;
    if (pos == n) break;  // last sequence: literals only
    if (n - pos < 2) return false;
    const int d = in[pos] | (in[pos + 1] << 8);
    pos += 2;
    int M = t & 15;
    if (M == 15 && !ext(&M)) return false;
    M += 4;
    if (d == 0 || d > o || M > kRunMaxRun || M > dec_len - o) return false;
    for (int k = 0; k < M; ++k) out[o + k] = out[o + k - d];
    if (d > 8) {
      far.insert(far.end(), out.begin() + o, out.begin() + o + M);
      if ((int)far.size() > kRunFarMax) return false;
    }
    o += M;
  }
  const int ni = (int)tok.size();
  if (o != dec_len || ni > kRunThreads || run_lds_bytes(n, (int)far.size()) > kRunLdsMax) return false;
  const size_t at = idx->size();
  idx->resize(at + (size_t)run_index_bytes(ni, (int)far.size()), 0);
  uint8_t* p = idx->data() + at;
  memcpy(p, win.data(), 8 * (size_t)ni);
  memcpy(p + 8 * (size_t)ni, tok.data(), 4 * (size_t)ni);
  memcpy(p + 12 * (size_t)ni, ost.data(), 2 * (size_t)ni);
  if (!far.empty()) memcpy(p + ((14 * (size_t)ni + 15) & ~(size_t)15), far.data(), far.size());
  *nint = ni;
  *nfar = (int)far.size();
  return true;
}

// routes: decode_routes(), read once per column by the caller (run blocks to k_lz4_run, flow blocks to
// k_lz4_decode_flow)
Lz4Job lz4_job(const BlockColumn& b, int32_t k, uint8_t* dst, int32_t expect, int routes) {
  Lz4Job j;
  j.src = b.comp.as<uint8_t>() + b.comp_off[k];
  j.dst = dst;
  j.cp = b.cps.as<uint32_t>() + b.cp_off[k];
  j.src_len = b.comp_len[k];
  j.expect_len = expect;
  j.ncp = b.cp_n[k];
  j.dec_len = b.dec_len[k];
  const bool flow = (routes & kRouteFlow) && !b.lvl_off.empty() && b.lvl_off[k] >= 0 && (b.cp_wide[k] & kLzFlow);
  j.wide = (b.cp_wide[k] & 1) | (flow ? kLzFlow : 0);
  j.lvl = flow ? b.lvls.as<uint8_t>() + b.lvl_off[k] : nullptr;
  j.nlvl = flow ? b.lvl_n[k] : 0;
  j.light = b.cp_light.empty() ? 0 : b.cp_light[k];
  j.nfine = b.cp_fine.empty() ? 0 : b.cp_fine[k];
  j.vstride = 0;
  const bool run = (routes & kRouteRun) && !b.run_off.empty() && b.run_off[k] >= 0;
  j.rx = run ? b.runx.as<uint8_t>() + b.run_off[k] : nullptr;
  j.run_n = run ? b.run_n[k] : 0;
  j.run_far = run ? b.run_far[k] : 0;
  j.red_dst = nullptr;
  j.red_op = j.red_kind = j.red_vkind = j.red_code = 0;
  j.red_bits = nullptr;
  j.red_row0 = 0;
  return j;
}

namespace {
static void index_bitmap_pieces(Column* c, const std::vector<uint8_t>& host);


// The column's attach-time decode tables (BlockColumn.job_desc / kind_list): a query then plans its
// LZ4 decodes as a few Lz4Tasks per column instead of one job per block.
static int decode_tables(BlockColumn* col) {
  const int32_t nb = col->nblocks;
  std::vector<Lz4Job> desc((size_t)std::max(nb, 1));
  memset(desc.data(), 0, desc.size() * sizeof(Lz4Job));
  for (auto& l : col->kind_list) l.clear();
  for (int32_t k = 0; k < nb; ++k) {
    const int64_t rows = std::min<int64_t>(col->size_per, (int64_t)col->total - (int64_t)k * col->size_per);
    const int64_t expect = col->vbits ? (col->vbits * rows + 7) / 8 : rows * col->width;
    desc[k] = lz4_job(*col, k, nullptr, (int32_t)std::max<int64_t>(expect, 0), kRouteRun | kRouteFlow);
    if (rows <= 0 || (!col->lit_off.empty() && col->lit_off[k] >= 0)) continue;
    const Lz4Job& j = desc[k];
    const int kind = j.rx ? kKindRun : j.light ? kKindLight : kKindGen0 + j.wide;
    col->kind_list[kind].push_back(k);
  }
  std::vector<int32_t> all;
  for (int kd = 0; kd < kKinds; ++kd) {
    auto& pos = col->kind_pos[kd];
    pos.assign((size_t)nb + 1, 0);
    size_t at = 0;
    for (int32_t k = 0; k < nb; ++k) {
      pos[k] = (int32_t)at;
      if (at < col->kind_list[kd].size() && col->kind_list[kd][at] == k) ++at;
    }
    pos[nb] = (int32_t)at;
    col->kind_at[kd] = (int64_t)all.size();
    all.insert(all.end(), col->kind_list[kd].begin(), col->kind_list[kd].end());
    auto& pb = col->kind_bytes[kd];
    pb.assign(col->kind_list[kd].size() + 1, 0);
    for (size_t i = 0; i < col->kind_list[kd].size(); ++i) pb[i + 1] = pb[i] + col->comp_len[col->kind_list[kd][i]];
  }
  if (all.empty()) all.push_back(0);
  if (!col->job_desc.alloc(desc.size() * sizeof(Lz4Job)) || !col->kind_dev.alloc(all.size() * 4))
    return set_error(DG_ERR_OOM, "hipMalloc lz4 decode tables");
  DG_HIP(hipMemcpy(col->job_desc.p, desc.data(), desc.size() * sizeof(Lz4Job), hipMemcpyHostToDevice));
  DG_HIP(hipMemcpy(col->kind_dev.p, all.data(), all.size() * 4, hipMemcpyHostToDevice));
  return DG_OK;
}

// Upload the blocks of a GenericIndexed of (compressed or raw) blocks.
int upload_blocks(Context* ctx, BlockColumn* col, const GI& blocks) {
  col->nblocks = blocks.n;
  if (col->codec == CODEC_LZ4 || col->codec == CODEC_LZF) {
    col->comp_off.resize(blocks.n);
    col->comp_len.resize(blocks.n);
    int64_t total = kCompSlack;  // (slack before the first block and after the last: the decoders read
                                 // whole dwords around a token or a literal run, from global memory too)
    col->lit_off.clear();
    for (int32_t b = 0; b < blocks.n; ++b) {
      const uint8_t* p;
      int32_t len = blocks.get(b, &p);
      if (len <= 0) return set_error(DG_ERR_FORMAT, "empty or out-of-range compressed block %d", b);
      // a literal-only LZ4 block (one sequence of literals: incompressible data) is placed so that its
      // literal bytes, its decoded image, start 16-byte aligned: views point at them, nothing decodes
      const int ls = col->codec == CODEC_LZ4 ? lz4_literal_start(p, len) : -1;
      if (ls >= 0) {
        if (col->lit_off.empty()) col->lit_off.assign(blocks.n, -1);
        col->comp_off[b] = ((total + ls + 15) & ~(int64_t)15) - ls;
        col->lit_off[b] = col->comp_off[b] + ls;
      } else {
        col->comp_off[b] = total;
      }
      col->comp_len[b] = len;
      total = (col->comp_off[b] + len + 15) & ~(int64_t)15;
    }
    std::vector<uint8_t> host((size_t)total + kCompSlack, 0);
    for (int32_t b = 0; b < blocks.n; ++b) {
      const uint8_t* p;
      int32_t len = blocks.get(b, &p);
      memcpy(host.data() + col->comp_off[b], p, (size_t)len);
      col->stored_bytes += len;
    }
    if (!col->comp.alloc(host.size())) return set_error(DG_ERR_OOM, "hipMalloc %zu", host.size());
    DG_HIP(hipMemcpy(col->comp.p, host.data(), host.size(), hipMemcpyHostToDevice));
    if (col->codec == CODEC_LZF) return DG_OK;  // decoded sequentially per block: no index
    // sequence checkpoints of every block (host threads over blocks; validated parse)
    col->cp_off.assign(blocks.n, 0);
    col->cp_n.assign(blocks.n, -1);
    col->cp_wide.assign(blocks.n, 0);
    col->cp_light.assign(blocks.n, 0);
    col->cp_fine.assign(blocks.n, 0);
    col->dec_len.assign(blocks.n, 0);
    std::vector<std::vector<uint32_t>> per(blocks.n);
    std::vector<std::vector<uint8_t>> runs(blocks.n), lvls(blocks.n);
    col->lvl_off.assign(blocks.n, -1);
    col->lvl_n.assign(blocks.n, 0);
    col->run_n.assign(blocks.n, 0);
    col->run_far.assign(blocks.n, 0);
    col->run_off.assign(blocks.n, -1);
    const bool minmax = col->time_col && col->width == 8 && !col->vbits;
    if (minmax) {
      col->min8.assign(blocks.n, 0);
      col->max8.assign(blocks.n, 0);
    }
    std::vector<uint8_t> has_mm(blocks.n, 0);
    const int nth = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const int nt = blocks.n >= 64 ? nth : 1;
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        for (int32_t b = t; b < blocks.n; b += nt) {
          int wide = 0, light = 0, nfine = 0, nlvl = 0;
          const int d = lz4_index_block(host.data() + col->comp_off[b], col->comp_len[b], &per[b], &wide, &light, &nfine,
                                        &lvls[b], &nlvl);
          col->cp_wide[b] = (uint8_t)wide;
          col->lvl_n[b] = nlvl;
          col->cp_light[b] = (uint8_t)light;
          col->cp_fine[b] = nfine;
          col->dec_len[b] = d;
          col->cp_n[b] = d < 0 ? -1 : (int32_t)per[b].size() - nfine;
          if (d > 0 && lz4_run_index(host.data() + col->comp_off[b], col->comp_len[b], d, &runs[b], &col->run_n[b],
                                     &col->run_far[b]))
            col->run_off[b] = 0;
          if (minmax && d >= 8) {  // the block's smallest and largest row time (its rows only)
            thread_local std::vector<uint8_t> dec(kBlockBytes);
            const int64_t rows = std::min<int64_t>(col->size_per, (int64_t)col->total - (int64_t)b * col->size_per);
            if (rows > 0 && lz4_decode_host(host.data() + col->comp_off[b], col->comp_len[b], dec.data()) >= rows * 8) {
              int64_t mn = INT64_MAX, mx = INT64_MIN;
              for (int64_t r = 0; r < rows; ++r) {
                int64_t v;
                memcpy(&v, dec.data() + 8 * r, 8);
                mn = std::min(mn, v);
                mx = std::max(mx, v);
              }
              col->min8[b] = mn;
              col->max8[b] = mx;
              has_mm[b] = 1;
            }
          }
        }
      });
    for (auto& x : th) x.join();
    // a literal-only block is read in place (no decoder, so no device check of its decoded length):
    // its literals must cover its rows (packed vbits columns are checked by parse_numeric)
    for (int32_t b = 0; !col->lit_off.empty() && !col->vbits && b < blocks.n; ++b) {
      if (col->lit_off[b] < 0) continue;
      const int64_t rows = std::min<int64_t>(col->size_per, (int64_t)col->total - (int64_t)b * col->size_per);
      if (rows > 0 && (int64_t)col->dec_len[b] < rows * col->width)
        return set_error(DG_ERR_FORMAT, "literal-only block %d holds %d of %lld bytes", b, col->dec_len[b],
                         (long long)(rows * col->width));
    }
    for (int32_t b = 0; minmax && b < blocks.n; ++b)
      if (!has_mm[b]) {  // (then no block's time range is known: every block is decoded)
        col->min8.clear();
        col->max8.clear();
      }
    std::vector<uint32_t> all;
    std::vector<uint8_t> rall, lall;
    col->index_bytes = 0;
    for (int32_t b = 0; b < blocks.n; ++b) {
      col->cp_off[b] = (int64_t)all.size();
      if (col->cp_n[b] > 0) all.insert(all.end(), per[b].begin(), per[b].end());
      if (col->run_off[b] >= 0) {  // a query reads the run index of a run block, not its checkpoints
        col->run_off[b] = (int64_t)rall.size();
        rall.insert(rall.end(), runs[b].begin(), runs[b].end());
        col->index_bytes += (int64_t)runs[b].size();
      } else if (col->cp_n[b] > 0) {
        col->index_bytes += 4 * (int64_t)per[b].size();
        if (!lvls[b].empty()) col->index_bytes += (int64_t)lvls[b].size();  // + a flow block's schedule
      }
      if ((col->cp_wide[b] & kLzFlow) && !lvls[b].empty()) {
        col->lvl_off[b] = (int64_t)lall.size();
        lall.insert(lall.end(), lvls[b].begin(), lvls[b].end());
      } else {
        col->cp_wide[b] &= (uint8_t)~kLzFlow;
      }
    }
    if (!lall.empty()) {
      if (!col->lvls.alloc(lall.size())) return set_error(DG_ERR_OOM, "hipMalloc lz4 level schedules");
      DG_HIP(hipMemcpy(col->lvls.p, lall.data(), lall.size(), hipMemcpyHostToDevice));
    }
    if (all.empty()) all.push_back(0);
    if (!col->cps.alloc(all.size() * 4)) return set_error(DG_ERR_OOM, "hipMalloc lz4 index");
    DG_HIP(hipMemcpy(col->cps.p, all.data(), all.size() * 4, hipMemcpyHostToDevice));
    if (!rall.empty()) {
      rall.resize(rall.size() + 16, 0);  // (k_lz4_run reads 12 bytes at a time: slack after the last table)
      if (!col->runx.alloc(rall.size())) return set_error(DG_ERR_OOM, "hipMalloc lz4 run index");
      DG_HIP(hipMemcpy(col->runx.p, rall.data(), rall.size(), hipMemcpyHostToDevice));
    }
    return col->codec == CODEC_LZ4 ? decode_tables(col) : DG_OK;
  }
  if (col->codec == CODEC_UNCOMPRESSED) {
    size_t bytes = (size_t)blocks.n * kBlockBytes;
    std::vector<uint8_t> host(bytes > 0 ? bytes : 16, 0);
    for (int32_t b = 0; b < blocks.n; ++b) {
      const uint8_t* p;
      int32_t len = blocks.get(b, &p);
      if (len < 0 || len > kBlockBytes) return set_error(DG_ERR_FORMAT, "uncompressed block %d of %d bytes", b, len);
      memcpy(host.data() + (size_t)b * kBlockBytes, p, (size_t)len);
      col->stored_bytes += len;
    }
    if (!col->raw.alloc(host.size())) return set_error(DG_ERR_OOM, "hipMalloc %zu", host.size());
    DG_HIP(hipMemcpy(col->raw.p, host.data(), host.size(), hipMemcpyHostToDevice));
    std::vector<const uint8_t*> ptrs(blocks.n > 0 ? blocks.n : 1);
    for (int32_t b = 0; b < blocks.n; ++b) ptrs[b] = col->raw.as<uint8_t>() + (size_t)b * kBlockBytes;
    if (!col->block_ptrs.alloc(ptrs.size() * sizeof(void*))) return set_error(DG_ERR_OOM, "hipMalloc ptrs");
    DG_HIP(hipMemcpy(col->block_ptrs.p, ptrs.data(), ptrs.size() * sizeof(void*), hipMemcpyHostToDevice));
    return DG_OK;
  }
  return set_error(DG_ERR_UNSUPPORTED, "compression id 0x%02x", col->codec);
}

// NONE layout: flat values directly after the header (EntireLayoutColumnar*Supplier)
int upload_flat(BlockColumn* col, const uint8_t* p, const uint8_t* end) {
  size_t bytes = (size_t)col->total * col->width;
  if ((int64_t)bytes > end - p) return set_error(DG_ERR_FORMAT, "truncated NONE column");
  if (!col->raw.alloc(bytes + 16)) return set_error(DG_ERR_OOM, "hipMalloc %zu", bytes);
  DG_HIP(hipMemcpy(col->raw.p, p, bytes, hipMemcpyHostToDevice));
  col->stored_bytes = (int64_t)bytes;
  // virtual blocks of a power-of-two row count so kernels address every layout the same way
  int l2 = 0;
  while ((2 << l2) <= kBlockBytes / col->width) l2++;
  col->log2_per = l2;
  col->size_per = 1 << l2;
  col->nblocks = (int32_t)((col->total + col->size_per - 1) / col->size_per);
  std::vector<const uint8_t*> ptrs(col->nblocks > 0 ? col->nblocks : 1);
  for (int32_t b = 0; b < col->nblocks; ++b)
    ptrs[b] = col->raw.as<uint8_t>() + (size_t)b * (size_t)col->size_per * (size_t)col->width;
  if (!col->block_ptrs.alloc(ptrs.size() * sizeof(void*))) return set_error(DG_ERR_OOM, "hipMalloc ptrs");
  DG_HIP(hipMemcpy(col->block_ptrs.p, ptrs.data(), ptrs.size() * sizeof(void*), hipMemcpyHostToDevice));
  return DG_OK;
}

// DELTA / TABLE encoding metadata (CompressionFactory.LongEncodingFormat.getReader, :153-188):
// DELTA = [u8 version 1][i64 base][i32 bitsPerValue] (DeltaLongEncodingReader.java:34-46);
// TABLE = [u8 version 1][i32 size <= 256][size x i64] with bits = getBitsForMax(size)
// (TableLongEncodingReader.java:33-52). All big-endian.
static int bits_for_max(int64_t value) {  // VSizeLongSerde.getBitsForMax (:41-59)
  static const int sizes[] = {1, 2, 4, 8, 12, 16, 20, 24, 32, 40, 48, 56, 64};
  int nbits = 0;
  int64_t max_value = 1;
  for (int sz : sizes) {
    while (nbits < sz && max_value < INT64_MAX / 2) {
      nbits++;
      max_value *= 2;
    }
    if (value <= max_value || max_value >= INT64_MAX / 2) return sz;
  }
  return 64;
}

static bool supported_bits(int b) {
  switch (b) {
    case 1: case 2: case 4: case 8: case 12: case 16: case 20: case 24: case 32: case 40: case 48: case 56: case 64:
      return true;
    default:
      return false;
  }
}

int parse_long_encoding(Column* c, uint8_t enc, Slice* s) {
  BlockColumn& col = c->data;
  if (enc == 0x00) {  // DELTA
    if (s->left() < 13) return set_error(DG_ERR_FORMAT, "%s: truncated DELTA header", c->name.c_str());
    if (s->p[0] != 0x01) return set_error(DG_ERR_FORMAT, "%s: DELTA version %d", c->name.c_str(), s->p[0]);
    col.delta_base = (int64_t)be64(s->p + 1);
    col.vbits = be32(s->p + 9);
    s->p += 13;
    if (!supported_bits(col.vbits)) return set_error(DG_ERR_FORMAT, "%s: unsupported size %d", c->name.c_str(), col.vbits);
    return DG_OK;
  }
  if (enc == 0x01) {  // TABLE
    if (s->left() < 5) return set_error(DG_ERR_FORMAT, "%s: truncated TABLE header", c->name.c_str());
    if (s->p[0] != 0x01) return set_error(DG_ERR_FORMAT, "%s: TABLE version %d", c->name.c_str(), s->p[0]);
    const int32_t n = be32(s->p + 1);
    if (n < 0 || n > 256) return set_error(DG_ERR_FORMAT, "%s: Invalid table size[%d]", c->name.c_str(), n);
    s->p += 5;
    if (s->left() < (int64_t)n * 8) return set_error(DG_ERR_FORMAT, "%s: truncated table", c->name.c_str());
    std::vector<int64_t> t(n > 0 ? n : 1, 0);
    for (int32_t i = 0; i < n; ++i) t[i] = (int64_t)be64(s->p + 8 * i);
    s->p += (size_t)n * 8;
    col.table_n = n;
    col.vbits = bits_for_max(n);
    if (!col.table.alloc(t.size() * 8)) return set_error(DG_ERR_OOM, "hipMalloc table");
    DG_HIP(hipMemcpy(col.table.p, t.data(), t.size() * 8, hipMemcpyHostToDevice));
    return DG_OK;
  }
  return set_error(DG_ERR_FORMAT, "%s: unknown long encoding %d", c->name.c_str(), enc);
}

// NONE layout of a packed column (EntireLayoutColumnarLongsSupplier over a Delta/Table reader): one
// packed stream of `total` values; addressed as virtual blocks of 8192 rows (8192 * bits / 8 bytes)
int upload_flat_packed(BlockColumn* col, const uint8_t* p, const uint8_t* end) {
  const int64_t bytes = vsize_serialized(col->vbits, col->total);
  if (bytes > end - p) return set_error(DG_ERR_FORMAT, "truncated NONE column");
  if (!col->raw.alloc((size_t)bytes + 16)) return set_error(DG_ERR_OOM, "hipMalloc %lld", (long long)bytes);
  DG_HIP(hipMemcpy(col->raw.p, p, (size_t)bytes, hipMemcpyHostToDevice));
  col->stored_bytes = bytes;
  col->log2_per = 13;
  col->size_per = 1 << 13;
  col->nblocks = (int32_t)((col->total + col->size_per - 1) / col->size_per);
  std::vector<const uint8_t*> ptrs(col->nblocks > 0 ? col->nblocks : 1);
  for (int32_t b = 0; b < col->nblocks; ++b)
    ptrs[b] = col->raw.as<uint8_t>() + (size_t)b * (size_t)col->size_per * col->vbits / 8;
  if (!col->block_ptrs.alloc(ptrs.size() * sizeof(void*))) return set_error(DG_ERR_OOM, "hipMalloc ptrs");
  DG_HIP(hipMemcpy(col->block_ptrs.p, ptrs.data(), ptrs.size() * sizeof(void*), hipMemcpyHostToDevice));
  return DG_OK;
}

int parse_numeric(Context* ctx, Column* c, Slice s, int width) {
  // [u8 version][i32 total][i32 sizePer][u8 compression (maybe flagged)][encoding?][blocks | values]
  if (s.left() < 10) return set_error(DG_ERR_FORMAT, "%s: truncated numeric column", c->name.c_str());
  uint8_t version = s.p[0];
  if (version != 0x02 && version != 0x01)
    return set_error(DG_ERR_FORMAT, "%s: Unknown version[%d]", c->name.c_str(), version);
  BlockColumn& col = c->data;
  col.total = be32(s.p + 1);
  col.size_per = be32(s.p + 5);
  int8_t cid;
  if (version == 0x01) {  // LZF_VERSION: no compression byte, LZF blocks (CompressedColumnarLongsSupplier:104-116)
    cid = (int8_t)CODEC_LZF;
    s.p += 9;
  } else {
    cid = (int8_t)s.p[9];
    s.p += 10;
  }
  if (version == 0x02 && cid < (int8_t)0xFE) {  // CompressionFactory.hasEncodingFlag
    uint8_t enc = *s.p++;
    cid = (int8_t)(cid + 126);
    if (enc != 0xFF) {
      int rc = parse_long_encoding(c, enc, &s);
      if (rc) return rc;
    }
  }
  col.codec = (uint8_t)cid;
  col.width = width;
  if (col.codec == CODEC_NONE) return col.vbits ? upload_flat_packed(&col, s.p, s.end) : upload_flat(&col, s.p, s.end);
  col.log2_per = log2i(col.size_per);
  const int64_t block_bytes = col.vbits ? vsize_serialized(col.vbits, col.size_per) : (int64_t)col.size_per * width;
  if (col.log2_per < 0 || block_bytes > kBlockBytes)
    return set_error(DG_ERR_FORMAT, "%s: bad block size %d", c->name.c_str(), col.size_per);
  GI blocks;
  if (!gi_read(s, &blocks)) return set_error(DG_ERR_FORMAT, "%s: bad block index", c->name.c_str());
  if ((int64_t)blocks.n * col.size_per < col.total) return set_error(DG_ERR_FORMAT, "%s: too few blocks", c->name.c_str());
  col.time_col = c->name == "__time";
  int rc = upload_blocks(ctx, &col, blocks);
  if (rc || !col.vbits) return rc;
  // every block must hold the packed bytes of its rows (the expansion reads exactly those)
  for (int32_t k = 0; k < col.nblocks; ++k) {
    const int64_t rows = std::min<int64_t>(col.size_per, (int64_t)col.total - (int64_t)k * col.size_per);
    if (rows <= 0) continue;
    const int64_t need = (col.vbits * rows + 7) / 8;
    const uint8_t* bp;
    // LZF blocks carry no decoded length until decoded: k_lzf_decode checks it against the expectation
    const int64_t have = col.codec == CODEC_LZ4 ? col.dec_len[k] : (col.codec == CODEC_LZF ? -1 : blocks.get(k, &bp));
    if (have >= 0 && have < need)
      return set_error(DG_ERR_FORMAT, "%s: packed block %d holds %lld of %lld bytes", c->name.c_str(), k,
                       (long long)have, (long long)need);
  }
  return DG_OK;
}

// CompressedVSizeColumnarIntsSupplier.fromByteBuffer (data/CompressedVSizeColumnarIntsSupplier.java:
// 143-168): [0x02][u8 numBytes][i32 total][i32 sizePer][u8 codec][GenericIndexed blocks], values
// little-endian numBytes wide inside a block (:254-353)
static int parse_vsize_ints(Context* ctx, BlockColumn* col, Slice* s, const char* name, const char* what) {
  if (s->left() < 11 || s->p[0] != 0x02) return set_error(DG_ERR_FORMAT, "%s: bad %s", name, what);
  col->width = s->p[1];
  col->total = be32(s->p + 2);
  col->size_per = be32(s->p + 6);
  col->codec = s->p[10];
  col->log2_per = log2i(col->size_per);
  s->p += 11;
  if (col->width < 1 || col->width > 4 || col->log2_per < 0 || col->total < 0 ||
      (int64_t)col->size_per * col->width > kBlockBytes)
    return set_error(DG_ERR_FORMAT, "%s: bad %s header", name, what);
  GI blocks;
  if (!gi_read(*s, &blocks)) return set_error(DG_ERR_FORMAT, "%s: bad %s blocks", name, what);
  if ((int64_t)blocks.n * col->size_per < col->total) return set_error(DG_ERR_FORMAT, "%s: too few %s blocks", name, what);
  return upload_blocks(ctx, col, blocks);
}

// Multi-value id parts (DictionaryEncodedColumnPartSerde.readMultiValuedColumn, :183-217), uploaded as
// two block columns: mv_off (rows + 1 value offsets, little-endian ints) and data (the value
// ids). UNCOMPRESSED_MULTI_VALUE = VSizeColumnarMultiInts [0x01][numBytes][i32 size][payload: i32
// count, count big-endian end byte offsets, big-endian numBytes values] (VSizeColumnarMultiInts.
// readFromByteBuffer / get(index)): the offsets are converted at attach, the values read in place;
// COMPRESSED + MULTI_VALUE_V3 = [0x03][CompressedColumnarIntsSupplier offsets: 0x02, i32 total,
// i32 sizePer, u8 codec, GI][CompressedVSizeColumnarIntsSupplier values: 0x02, u8 numBytes, i32,
// i32, u8 codec, GI] (V3CompressedVSizeColumnarMultiIntsSupplier.fromByteBuffer); COMPRESSED +
// MULTI_VALUE = the legacy form, both parts CompressedVSizeColumnarInts (offsets 1-4 bytes wide).
static int parse_multi_value_ids(Context* ctx, Column* c, Slice* s, int version, bool legacy) {
  BlockColumn& off = c->mv_off;
  BlockColumn& val = c->data;
  if (version == 1) {
    if (s->left() < 10 || s->p[0] != 0x01) return set_error(DG_ERR_FORMAT, "%s: bad VSize multi-ints", c->name.c_str());
    const int nb = s->p[1];
    const int32_t size = be32(s->p + 2);
    if (nb < 1 || nb > 4 || size < 4 || s->left() < 6 + (int64_t)size)
      return set_error(DG_ERR_FORMAT, "%s: truncated multi-ints", c->name.c_str());
    const uint8_t* pay = s->p + 6;
    const int32_t count = be32(pay);
    if (count < 0 || 4 + 4 * (int64_t)count > size) return set_error(DG_ERR_FORMAT, "%s: bad multi-ints count", c->name.c_str());
    std::vector<int32_t> offs((size_t)count + 1, 0);
    int64_t prev = 0;
    for (int32_t r = 0; r < count; ++r) {
      const int64_t e = be32(pay + 4 + 4 * (int64_t)r);
      if (e < prev || e % nb || 4 + 4 * (int64_t)count + e > size)
        return set_error(DG_ERR_FORMAT, "%s: bad multi-ints offsets", c->name.c_str());
      offs[(size_t)r + 1] = (int32_t)(e / nb);
      prev = e;
    }
    off.total = count + 1;
    off.width = 4;
    off.codec = CODEC_NONE;
    int rc = upload_flat(&off, reinterpret_cast<const uint8_t*>(offs.data()),
                         reinterpret_cast<const uint8_t*>(offs.data() + offs.size()));
    if (rc) return rc;
    val.width = nb;
    val.total = (int32_t)(prev / nb);
    val.codec = CODEC_NONE;
    val.big_endian = 1;
    const uint8_t* vp = pay + 4 + 4 * (int64_t)count;
    rc = upload_flat(&val, vp, s->end);
    if (rc) return rc;
    s->p += 6 + size;
    return DG_OK;
  }
  if (legacy) {
    // COMPRESSED + MULTI_VALUE (no V3 flag): CompressedVSizeColumnarMultiIntsSupplier.fromByteBuffer
    // (:77-93) = [0x02][offsets: CompressedVSizeColumnarInts, numBytes for the values count][values:
    // CompressedVSizeColumnarInts]; the offsets' width comes from their own header (1-4 bytes)
    if (s->left() < 1 || s->p[0] != 0x02) return set_error(DG_ERR_FORMAT, "%s: Unknown version[%d]", c->name.c_str(), s->left() ? s->p[0] : -1);
    s->p += 1;
    int rc = parse_vsize_ints(ctx, &off, s, c->name.c_str(), "multi-value offsets");
    if (rc) return rc;
    if (off.total < 1) return set_error(DG_ERR_FORMAT, "%s: bad multi-value offsets header", c->name.c_str());
    return parse_vsize_ints(ctx, &val, s, c->name.c_str(), "multi-value values");
  }
  if (s->left() < 1 + 10 || s->p[0] != 0x03 || s->p[1] != 0x02)
    return set_error(DG_ERR_FORMAT, "%s: bad V3 multi-value ids", c->name.c_str());
  off.total = be32(s->p + 2);
  off.size_per = be32(s->p + 6);
  off.codec = s->p[10];
  off.width = 4;
  off.log2_per = log2i(off.size_per);
  s->p += 1 + 10;
  if (off.total < 1 || off.log2_per < 0 || (int64_t)off.size_per * 4 > kBlockBytes)
    return set_error(DG_ERR_FORMAT, "%s: bad multi-value offsets header", c->name.c_str());
  GI offsets;
  if (!gi_read(*s, &offsets)) return set_error(DG_ERR_FORMAT, "%s: bad multi-value offsets", c->name.c_str());
  int rc = upload_blocks(ctx, &off, offsets);
  if (rc) return rc;
  return parse_vsize_ints(ctx, &val, s, c->name.c_str(), "multi-value values");
}

int parse_string(Context* ctx, Column* c, Slice s) {
  if (s.left() < 1) return set_error(DG_ERR_FORMAT, "%s: empty", c->name.c_str());
  int version = s.p[0];
  s.p++;
  int flags = 0;
  if (version >= 2) {
    flags = be32(s.p);
    s.p += 4;
  } else if (version == 1) {
    flags = 1;
  }
  c->multi_value = (flags & 3) != 0;
  GI dict;
  if (!gi_read(s, &dict)) return set_error(DG_ERR_FORMAT, "%s: bad dictionary", c->name.c_str());
  c->dict.resize(dict.n);
  c->dict_null.resize(dict.n);
  for (int32_t i = 0; i < dict.n; ++i) {
    const uint8_t* p;
    int32_t len = dict.get(i, &p);
    if (len < 0) return set_error(DG_ERR_FORMAT, "%s: dictionary entry %d outside its GenericIndexed", c->name.c_str(), i);
    c->dict[i].assign((const char*)p, len > 0 ? len : 0);
    c->dict_null[i] = len <= 0;  // size 0 => null (replaceWithDefault), GenericIndexed.java:369-372
  }
  c->dict_hash.resize(dict.n);
  for (int32_t i = 0; i < dict.n; ++i) c->dict_hash[i] = c->dict_null[i] ? kNullValueHash : value_hash(c->dict[i]);
  BlockColumn& col = c->data;
  if (c->multi_value) {
    // row value lists: filters run on the bitmap index, groupBy explodes the lists (dg_sort.hip)
    int rc = parse_multi_value_ids(ctx, c, &s, version, version == 2 && !(flags & 2));
    if (rc) return rc;
  } else if (version == 0 || version == 3) {
    // UNCOMPRESSED_SINGLE_VALUE / UNCOMPRESSED_WITH_FLAGS: VSizeColumnarInts.readFromByteBuffer
    // (data/VSizeColumnarInts.java:177-195): [0x00][numBytes][i32 size][big-endian values + pad].
    // Read in place: kernels load numBytes big-endian bytes per row (getInt >>> bitsToShift, :124-127).
    if (s.left() < 6 || s.p[0] != 0x00) return set_error(DG_ERR_FORMAT, "%s: bad VSize id stream", c->name.c_str());
    col.width = s.p[1];
    const int32_t nbytes = be32(s.p + 2);
    if (col.width < 1 || col.width > 4 || nbytes < 4 - col.width || s.left() < 6 + (int64_t)nbytes)
      return set_error(DG_ERR_FORMAT, "%s: bad VSize id stream header", c->name.c_str());
    col.total = (nbytes - (4 - col.width)) / col.width;
    col.codec = CODEC_NONE;
    col.big_endian = 1;
    s.p += 6;
    int rc = upload_flat(&col, s.p, s.end);
    if (rc) return rc;
    s.p += nbytes;
  } else if (version == 2) {
    if (s.left() < 11 || s.p[0] != 0x02) return set_error(DG_ERR_FORMAT, "%s: bad id stream", c->name.c_str());
    col.width = s.p[1];
    col.total = be32(s.p + 2);
    col.size_per = be32(s.p + 6);
    col.codec = s.p[10];
    s.p += 11;
    col.log2_per = log2i(col.size_per);
    if (col.width < 1 || col.width > 4 || col.log2_per < 0)
      return set_error(DG_ERR_FORMAT, "%s: bad id stream header", c->name.c_str());
    GI blocks;
    if (!gi_read(s, &blocks)) return set_error(DG_ERR_FORMAT, "%s: bad id blocks", c->name.c_str());
    int rc = upload_blocks(ctx, &col, blocks);
    if (rc) return rc;
  } else {
    return set_error(DG_ERR_FORMAT, "%s: dictionary-encoded part version %d", c->name.c_str(), version);
  }
  if (!(flags & 4)) {
    GI bms;
    if (!gi_read(s, &bms)) return set_error(DG_ERR_FORMAT, "%s: bad bitmap index", c->name.c_str());
    if (bms.n != dict.n) return set_error(DG_ERR_FORMAT, "%s: %d bitmaps for %d values", c->name.c_str(), bms.n, dict.n);
    c->has_bitmaps = true;
    c->bm_off.resize(bms.n);
    c->bm_len.resize(bms.n);
    int64_t total = 0;
    for (int32_t i = 0; i < bms.n; ++i) {
      const uint8_t* p;
      int32_t len = bms.get(i, &p);
      if (len < 0) return set_error(DG_ERR_FORMAT, "%s: bitmap %d outside its GenericIndexed", c->name.c_str(), i);
      c->bm_off[i] = total;
      c->bm_len[i] = len > 0 ? len : 0;
      total += (c->bm_len[i] + 3) & ~3;
    }
    std::vector<uint8_t> host((size_t)total + 16, 0);
    for (int32_t i = 0; i < bms.n; ++i) {
      const uint8_t* p;
      bms.get(i, &p);
      if (c->bm_len[i]) memcpy(host.data() + c->bm_off[i], p, (size_t)c->bm_len[i]);
    }
    if (!c->bm_bytes.alloc(host.size())) return set_error(DG_ERR_OOM, "hipMalloc bitmaps");
    DG_HIP(hipMemcpy(c->bm_bytes.p, host.data(), host.size(), hipMemcpyHostToDevice));
    index_bitmap_pieces(c, host);
  }
  return DG_OK;
}

// Long bitmaps are cut into pieces once, at attach, so a query expands one bitmap with many
// workgroups: a Concise bitmap into runs of kConcisePieceWords words with the row each run starts
// at (the sum of the earlier words' spans: 31 rows per literal, 31 * (blocks) per fill,
// ConciseSetUtils.java:45-75), a Roaring bitmap into its containers (portable format: cookie,
// [run bitmap], key / cardinality descriptors, [offsets], containers). A bitmap whose header does not
// parse stays whole (the per-bitmap kernel reports it).
static uint32_t le32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }
static uint32_t le16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

static bool roaring_containers(const uint8_t* p, int len, std::vector<BmPiece>* out, int64_t base_off) {
  if (len < 8) return false;
  const uint32_t cookie = le32(p);
  int pos = 4, n = 0;
  const uint8_t* runbits = nullptr;
  bool has_off = true;
  if ((cookie & 0xFFFFu) == 12347u) {
    n = (int)(cookie >> 16) + 1;
    runbits = p + pos;
    pos += (n + 7) / 8;
    has_off = n >= 4;
  } else if (cookie == 12346u) {
    n = (int)le32(p + 4);
    pos = 8;
  } else {
    return false;
  }
  if (n <= 0 || pos + 4 * n > len) return false;
  const uint8_t* desc = p + pos;
  pos += 4 * n;
  const uint8_t* offs = nullptr;
  if (has_off) {
    if (pos + 4 * n > len) return false;
    offs = p + pos;
    pos += 4 * n;
  }
  int cur = pos;
  std::vector<BmPiece> v;
  for (int c = 0; c < n; ++c) {
    const int key = (int)le16(desc + 4 * c), card = (int)le16(desc + 4 * c + 2) + 1;
    const bool run = runbits && ((runbits[c >> 3] >> (c & 7)) & 1);
    const int start = offs ? (int)le32(offs + 4 * c) : cur;
    if (start < 0 || start + 2 > len) return false;
    const int sz = run ? 2 + 4 * (int)le16(p + start) : (card <= 4096 ? 2 * card : 8192);
    if (start + sz > len) return false;
    v.push_back(BmPiece{base_off + start, (int64_t)key << 16, sz, (int32_t)((uint32_t)(card - 1) | (run ? 0x80000000u : 0u))});
    cur = start + sz;
  }
  out->insert(out->end(), v.begin(), v.end());
  return true;
}

static void index_bitmap_pieces(Column* c, const std::vector<uint8_t>& host) {
  const int n = (int)c->bm_off.size();
  std::vector<int32_t> first(n + 1, 0);
  std::vector<BmPiece> pieces;
  for (int i = 0; i < n; ++i) {
    first[i] = (int32_t)pieces.size();
    const uint8_t* p = host.data() + c->bm_off[i];
    const int len = c->bm_len[i];
    if (!c->bitmap_roaring) {
      const int nw = len / 4;
      if (nw <= 2 * kConcisePieceWords) continue;
      int64_t row = 0;
      for (int w0 = 0; w0 < nw; w0 += kConcisePieceWords) {
        const int cnt = std::min(kConcisePieceWords, nw - w0);
        pieces.push_back(BmPiece{c->bm_off[i] + 4ll * w0, row, 4 * cnt, 0});
        for (int k = w0; k < w0 + cnt; ++k) {
          const uint32_t w = (uint32_t)be32(p + 4ll * k);
          row += (w & 0x80000000u) ? 31 : 31ll * ((int64_t)(w & 0x01FFFFFFu) + 1);
        }
      }
    } else if (len > kRoaringSplitBytes) {
      roaring_containers(p, len, &pieces, c->bm_off[i]);
    }
  }
  first[n] = (int32_t)pieces.size();
  if (!pieces.empty()) {
    c->bm_piece_first.swap(first);
    c->bm_pieces.swap(pieces);
  }
}

int64_t column_device_bytes(const Column& c) {
  return (int64_t)(c.data.comp.n + c.data.raw.n + c.data.block_ptrs.n + c.bm_bytes.n + c.mv_off.comp.n +
                   c.mv_off.raw.n + c.mv_off.block_ptrs.n);
}

}  // namespace

int read_time_bounds(Segment* seg);  // dg_engine.cpp

int load_segment(Context* ctx, const char* dir, Segment** out) {
  static std::atomic<uint64_t> serial{0};
  std::unique_ptr<Segment> seg(new Segment());
  seg->ctx = ctx;
  seg->uid = ++serial;
  seg->dir = dir;
  std::string d(dir);
  {
    MappedFile vf;
    if (!vf.open(d + "/version.bin") || vf.size != 4) return set_error(DG_ERR_FORMAT, "%s: missing version.bin", dir);
    if (be32(vf.data()) != 9) return set_error(DG_ERR_FORMAT, "Expected version[9], got[%d]", be32(vf.data()));
  }
  MappedFile meta;
  if (!meta.open(d + "/meta.smoosh")) return set_error(DG_ERR_FORMAT, "%s: missing meta.smoosh", dir);
  std::string text((const char*)meta.data(), meta.size);
  size_t pos = text.find('\n');
  int nchunks = 0;
  if (sscanf(text.c_str(), "v1,%*d,%d", &nchunks) != 1 || nchunks < 0) return set_error(DG_ERR_FORMAT, "bad meta.smoosh");
  std::vector<std::unique_ptr<MappedFile>> chunks(nchunks);
  for (int i = 0; i < nchunks; ++i) {
    char name[32];
    snprintf(name, sizeof name, "/%05d.smoosh", i);
    chunks[i].reset(new MappedFile());
    if (!chunks[i]->open(d + name)) return set_error(DG_ERR_FORMAT, "%s: missing chunk %s", dir, name);
  }
  struct Entry {
    std::string name;
    Slice s;
  };
  std::vector<Entry> entries;
  Slice index_drd;
  while (pos != std::string::npos && pos + 1 < text.size()) {
    size_t nl = text.find('\n', pos + 1);
    std::string line = text.substr(pos + 1, nl == std::string::npos ? std::string::npos : nl - pos - 1);
    pos = nl;
    if (line.empty()) continue;
    size_t c3 = line.rfind(','), c2 = c3 == std::string::npos ? c3 : line.rfind(',', c3 - 1),
           c1 = c2 == std::string::npos ? c2 : line.rfind(',', c2 - 1);
    if (c1 == std::string::npos) continue;
    std::string nm = line.substr(0, c1);
    int chunk = atoi(line.c_str() + c1 + 1);
    long st = atol(line.c_str() + c2 + 1), en = atol(line.c_str() + c3 + 1);
    if (chunk < 0 || chunk >= nchunks || en < st || (size_t)en > chunks[chunk]->size)
      return set_error(DG_ERR_FORMAT, "bad smoosh entry %s", nm.c_str());
    Slice s{chunks[chunk]->data() + st, chunks[chunk]->data() + en};
    if (nm == "index.drd") index_drd = s;
    else if (nm != "metadata.drd") entries.push_back({nm, s});
  }
  if (!index_drd.p) return set_error(DG_ERR_FORMAT, "%s: missing index.drd", dir);
  {
    Slice s = index_drd;
    GI cols, dims;
    if (!gi_read(s, &cols) || !gi_read(s, &dims) || s.left() < 16) return set_error(DG_ERR_FORMAT, "bad index.drd");
    seg->istart = be64(s.p);
    seg->iend = be64(s.p + 8);
    s.p += 16;
    if (s.left() >= 4) {
      int32_t l = be32(s.p);
      if (l > 0 && l <= s.left() - 4) {
        std::string js((const char*)s.p + 4, l);
        seg->bitmap_roaring = js.find("roaring") != std::string::npos;
      }
    }
  }
  for (auto& e : entries) {
    std::unique_ptr<Column> c(new Column());
    c->name = e.name;
    if (e.s.left() < 4) return set_error(DG_ERR_FORMAT, "%s: truncated", e.name.c_str());
    int32_t jlen = be32(e.s.p);
    if (jlen < 0 || jlen > e.s.left() - 4) return set_error(DG_ERR_FORMAT, "%s: bad descriptor", e.name.c_str());
    std::string js((const char*)e.s.p + 4, jlen);
    Slice part{e.s.p + 4 + jlen, e.s.end};
    size_t parts = js.find("\"parts\"");
    std::string ptype = json_get(js, "type", parts == std::string::npos ? 0 : parts);
    std::string order = json_get(js, "byteOrder");
    int rc = DG_OK;
    bool v2 = ptype.size() > 2 && ptype.compare(ptype.size() - 2, 2, "V2") == 0;
    if (v2) {
      if (part.left() < 4) return set_error(DG_ERR_FORMAT, "%s: truncated V2", e.name.c_str());
      part.p += 4;  // int offset to the null bitmap (nulls read as 0 in default null mode)
      ptype = ptype.substr(0, ptype.size() - 2);
    }
    if (order == "BIG_ENDIAN") {
      c->type = DG_COL_UNSUPPORTED;
    } else if (ptype == "long") {
      c->type = DG_COL_LONG;
      rc = parse_numeric(ctx, c.get(), part, 8);
    } else if (ptype == "double") {
      c->type = DG_COL_DOUBLE;
      rc = parse_numeric(ctx, c.get(), part, 8);
    } else if (ptype == "float") {
      c->type = DG_COL_FLOAT;
      rc = parse_numeric(ctx, c.get(), part, 4);
    } else if (ptype == "stringDictionary") {
      c->type = DG_COL_STRING;
      size_t bsf = js.find("\"bitmapSerdeFactory\"");
      c->bitmap_roaring = bsf != std::string::npos && json_get(js, "type", bsf) == "roaring";
      rc = parse_string(ctx, c.get(), part);
    } else {
      c->type = DG_COL_UNSUPPORTED;
    }
    if (rc == DG_ERR_UNSUPPORTED) {
      c->type = DG_COL_UNSUPPORTED;  // a query touching it gets DG_ERR_UNSUPPORTED
      c->data.comp.reset();
      c->data.raw.reset();
      c->data.block_ptrs.reset();
      c->bm_bytes.reset();
    } else if (rc) {
      return rc;
    }
    seg->device_bytes += column_device_bytes(*c);
    seg->by_name[c->name] = c.get();
    seg->columns.push_back(std::move(c));
  }
  Column* t = seg->find("__time");
  if (!t || t->type != DG_COL_LONG) return set_error(DG_ERR_FORMAT, "%s: missing __time", dir);
  seg->nrows = t->data.total;
  for (auto& c : seg->columns) {
    const int64_t rows = c->multi_value ? (int64_t)c->mv_off.total - 1 : c->data.total;
    if ((c->type == DG_COL_LONG || c->type == DG_COL_FLOAT || c->type == DG_COL_DOUBLE || c->type == DG_COL_STRING) &&
        rows != seg->nrows)
      return set_error(DG_ERR_FORMAT, "%s: %lld rows, segment has %lld", c->name.c_str(), (long long)rows,
                       (long long)seg->nrows);
  }
  int rc = read_time_bounds(seg.get());
  if (rc) return rc;
  *out = seg.release();
  return DG_OK;
}

// In-memory segment from an IncrementalIndex's rows (IncrementalIndexStorageAdapter): every column a
// flat array in HBM (codec NONE); string dictionaries re-sorted into Java String order (nulls first)
// with the row ids remapped, so the engines see the sorted-dictionary contract of a persisted segment
// (IncrementalIndexStorageAdapter also answers through the sorted lookup, StringDimensionIndexer's
// SortedDimensionDictionary). No bitmap index: string filters run as row predicates on the ids, as
// the adapter's ValueMatchers do (IncrementalIndexStorageAdapter.makeCursors -> filter.makeMatcher).
int segment_from_rows(Context* ctx, int64_t nrows, const int64_t* ts, int64_t istart, int64_t iend,
                      const dg_row_column* cols, int ncols, Segment** out) {
  if (nrows < 0 || nrows > INT32_MAX - 1 || (nrows > 0 && !ts) || ncols < 0 || (ncols > 0 && !cols) || iend < istart)
    return set_error(DG_ERR_ARG, "bad row arguments");
  static std::atomic<uint64_t> serial{1ull << 62};
  std::unique_ptr<Segment> seg(new Segment());
  seg->ctx = ctx;
  seg->uid = ++serial;
  seg->dir = "<rows>";
  seg->nrows = nrows;
  seg->istart = istart;
  seg->iend = iend;
  for (int64_t r = 1; r < nrows; ++r)
    if (ts[r] < ts[r - 1]) return set_error(DG_ERR_ARG, "row timestamps must ascend (the index's time order)");
  auto add = [&](std::unique_ptr<Column> c) {
    seg->device_bytes += column_device_bytes(*c);
    seg->by_name[c->name] = c.get();
    seg->columns.push_back(std::move(c));
  };
  auto flat = [&](Column* c, const void* p, int width) {
    c->data.total = (int32_t)nrows;
    c->data.width = width;
    c->data.codec = CODEC_NONE;
    static const int64_t zero[2] = {0, 0};
    const uint8_t* b = nrows ? static_cast<const uint8_t*>(p) : reinterpret_cast<const uint8_t*>(zero);
    return upload_flat(&c->data, b, b + (size_t)nrows * width);
  };
  {
    std::unique_ptr<Column> t(new Column());
    t->name = "__time";
    t->type = DG_COL_LONG;
    int rc = flat(t.get(), ts, 8);
    if (rc) return rc;
    add(std::move(t));
  }
  for (int i = 0; i < ncols; ++i) {
    const dg_row_column& rc_ = cols[i];
    if (!rc_.name || !*rc_.name || !strcmp(rc_.name, "__time") || seg->find(rc_.name))
      return set_error(DG_ERR_ARG, "column %d: missing, reserved or repeated name", i);
    std::unique_ptr<Column> c(new Column());
    c->name = rc_.name;
    c->type = rc_.type;
    int rc = DG_OK;
    if (rc_.type == DG_COL_LONG || rc_.type == DG_COL_DOUBLE || rc_.type == DG_COL_FLOAT) {
      if (nrows && !rc_.values) return set_error(DG_ERR_ARG, "%s: null values", rc_.name);
      rc = flat(c.get(), rc_.values, rc_.type == DG_COL_FLOAT ? 4 : 8);
    } else if (rc_.type == DG_COL_STRING) {
      const int32_t card = rc_.card;
      if (card < 0 || (card > 0 && !rc_.dict) || (nrows && !rc_.ids)) return set_error(DG_ERR_ARG, "%s: bad dictionary", rc_.name);
      // DimensionDictionary ids (insertion order) -> sorted ids; "" is null (default null handling)
      std::vector<int32_t> order(card);
      for (int32_t k = 0; k < card; ++k) order[k] = k;
      auto is_null = [&](int32_t k) { return !rc_.dict[k] || !rc_.dict[k][0]; };
      std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
        const bool an = is_null(a), bn = is_null(b);
        if (an || bn) return an && !bn;
        return java_compare_str(rc_.dict[a], rc_.dict[b]) < 0;
      });
      std::vector<int32_t> remap(card);
      for (int32_t k = 0; k < card; ++k) {
        const int32_t o = order[k];
        if (k > 0) {
          const int32_t p = order[k - 1];
          const bool same = is_null(o) ? is_null(p) : (!is_null(p) && !strcmp(rc_.dict[o], rc_.dict[p]));
          if (same) return set_error(DG_ERR_ARG, "%s: dictionary value repeated", rc_.name);
        }
        remap[o] = k;
        c->dict.push_back(is_null(o) ? std::string() : std::string(rc_.dict[o]));
        c->dict_null.push_back(is_null(o) ? 1 : 0);
        c->dict_hash.push_back(is_null(o) ? kNullValueHash : value_hash(c->dict.back()));
      }
      int64_t nv = nrows;
      if (rc_.offsets) {  // multi-value rows: offsets must start at 0 and never decrease
        if (rc_.offsets[0] != 0) return set_error(DG_ERR_ARG, "%s: offsets[0] != 0", rc_.name);
        for (int64_t r = 0; r < nrows; ++r)
          if (rc_.offsets[r + 1] < rc_.offsets[r]) return set_error(DG_ERR_ARG, "%s: offsets decrease at row %lld", rc_.name, (long long)r);
        nv = rc_.offsets[nrows];
        if (nv > 0 && !rc_.ids) return set_error(DG_ERR_ARG, "%s: null ids", rc_.name);
      }
      std::vector<int32_t> ids((size_t)std::max<int64_t>(nv, 1));
      for (int64_t r = 0; r < nv; ++r) {
        const int32_t id = rc_.ids[r];
        if (id < 0 || id >= card) return set_error(DG_ERR_ARG, "%s: value %lld id %d outside [0, %d)", rc_.name, (long long)r, id, card);
        ids[r] = remap[id];
      }
      c->has_bitmaps = false;
      if (rc_.offsets) {
        c->multi_value = true;
        c->mv_off.total = (int32_t)nrows + 1;
        c->mv_off.width = 4;
        c->mv_off.codec = CODEC_NONE;
        rc = upload_flat(&c->mv_off, reinterpret_cast<const uint8_t*>(rc_.offsets),
                         reinterpret_cast<const uint8_t*>(rc_.offsets + nrows + 1));
        if (rc) return rc;
        c->data.total = (int32_t)nv;
        c->data.width = 4;
        c->data.codec = CODEC_NONE;
        static const int32_t zero[4] = {0, 0, 0, 0};
        const uint8_t* b = nv ? reinterpret_cast<const uint8_t*>(ids.data()) : reinterpret_cast<const uint8_t*>(zero);
        rc = upload_flat(&c->data, b, b + (size_t)nv * 4);
      } else {
        rc = flat(c.get(), ids.data(), 4);
      }
    } else {
      return set_error(DG_ERR_ARG, "%s: column type %d", rc_.name, rc_.type);
    }
    if (rc) return rc;
    add(std::move(c));
  }
  if (nrows) {
    seg->min_time = ts[0];
    seg->max_time = ts[nrows - 1];
  }
  *out = seg.release();
  return DG_OK;
}

}  // namespace dg
