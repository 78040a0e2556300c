/*
 * druid_oracle.c — CPU restatement of Druid's segment scan-and-aggregate path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity checker: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product path (incubator-druid_amd) never links
 * or calls it.
 *
 * It restates, scalar and in row order, the Java code of foamdino/incubator-druid that the GPU
 * engine replaces (every function cites the file:line it follows; paths are relative to the
 * reference root, processing/... = processing/src/main/java/org/apache/druid/...):
 *   - v9 segment loading: IndexIO.V9IndexLoader.load (processing/.../segment/IndexIO.java:569-673),
 *     SmooshedFileMapper (java-util/.../io/smoosh/SmooshedFileMapper.java),
 *     GenericIndexed v1 (processing/.../segment/data/GenericIndexed.java:479-572)
 *   - column decode: CompressedColumnarLongsSupplier (data/CompressedColumnarLongsSupplier.java:100-136),
 *     CompressionFactory (data/CompressionFactory.java:289-354), BlockLayoutColumnarLongsSupplier
 *     (data/BlockLayoutColumnarLongsSupplier.java:59-90), CompressedVSizeColumnarIntsSupplier
 *     (data/CompressedVSizeColumnarIntsSupplier.java:143-168,254-353), LZ4 safe decompression
 *     (data/CompressionStrategy.java:284-305 -> lz4-java 1.4.0 LZ4SafeDecompressor, LZ4 block format)
 *   - bitmaps: Concise BitIterator (extendedset/.../intset/BitIterator.java:25-282),
 *     ConciseSetUtils (extendedset/.../intset/ConciseSetUtils.java:149-281); Roaring portable
 *     format (RoaringBitmap 0.5.18, not vendored: RoaringFormatSpec)
 *   - aggregation arithmetic with Java semantics: LongSumAggregator.java:47-59,
 *     DoubleSumAggregator.java:48-61, FloatSumAggregator.java:47-59 (float accumulator),
 *     {Long,Double,Float}{Min,Max}Aggregator (Math.min/max), casts in
 *     segment/DoubleColumnSelector.java:40-55 and LongColumnSelector.java:40-54.
 * Query-level logic (filters over row sets, granularity buckets, topN result builder, merges) is
 * restated in oracle/oracle.py on top of these primitives.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* byte helpers                                                                                */
/* ------------------------------------------------------------------------------------------ */
static int32_t be32(const uint8_t* p) {
  return (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
}
static int64_t be64(const uint8_t* p) { return ((int64_t)(uint32_t)be32(p) << 32) | (uint32_t)be32(p + 4); }

typedef struct {
  uint8_t* data;
  int64_t size;
} blob;

static int read_file(const char* path, blob* out) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  out->data = (uint8_t*)malloc(n > 0 ? (size_t)n : 1);
  out->size = n;
  if (n > 0 && fread(out->data, 1, (size_t)n, f) != (size_t)n) {
    fclose(f);
    free(out->data);
    return -1;
  }
  fclose(f);
  return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* LZ4 block decompression (lz4-java safeDecompressor contract: returns bytes written, <0 error) */
/* ------------------------------------------------------------------------------------------ */
int64_t or_lz4_decompress(const uint8_t* src, int64_t n, uint8_t* dst, int64_t cap) {
  const uint8_t* ip = src;
  const uint8_t* iend = src + n;
  uint8_t* op = dst;
  uint8_t* oend = dst + cap;
  if (n == 0) return -1;
  for (;;) {
    if (ip >= iend) return -1;
    unsigned token = *ip++;
    int64_t lit = token >> 4;
    if (lit == 15) {
      unsigned b;
      do {
        if (ip >= iend) return -1;
        b = *ip++;
        lit += b;
      } while (b == 255);
    }
    if (lit > iend - ip || lit > oend - op) return -1;
    memcpy(op, ip, (size_t)lit);
    op += lit;
    ip += lit;
    if (ip == iend) break; /* last sequence carries literals only */
    if (iend - ip < 2) return -1;
    int64_t off = ip[0] | (ip[1] << 8);
    ip += 2;
    if (off == 0 || off > op - dst) return -1;
    int64_t ml = token & 15;
    if (ml == 15) {
      unsigned b;
      do {
        if (ip >= iend) return -1;
        b = *ip++;
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (ml > oend - op) return -1;
    const uint8_t* m = op - off;
    for (int64_t k = 0; k < ml; ++k) op[k] = m[k]; /* byte order matters for overlapping copies */
    op += ml;
  }
  return op - dst;
}

/* ------------------------------------------------------------------------------------------ */
/* Concise: BitIterator semantics                                                               */
/* ------------------------------------------------------------------------------------------ */
/* words are big-endian int32 in the serialized form (ImmutableConciseSet(ByteBuffer) asIntBuffer). */
int64_t or_concise_decode(const uint8_t* bytes, int64_t nbytes, int32_t* out, int64_t cap) {
  int64_t nwords = nbytes / 4;
  int64_t offset = 0, count = 0;
  for (int64_t i = 0; i < nwords; ++i) {
    int32_t w = be32(bytes + 4 * i);
    if (w < 0) { /* literal: BitIterator.literalAndZeroFillResetLiteral */
      for (int b = 0; b < 31; ++b) {
        if (w & (1 << b)) {
          if (count < cap) out[count] = (int32_t)(offset + b);
          count++;
        }
      }
      offset += 31;
    } else {
      int64_t blocks = (int64_t)(w & 0x01FFFFFF) + 1;
      int flip = ((0x3FFFFFFF & w) >> 25) - 1; /* -1: no flipped bit */
      if ((w & 0xC0000000) == 0) { /* zero fill: at most one set bit (the flipped one) */
        if (flip >= 0) {
          if (count < cap) out[count] = (int32_t)(offset + flip);
          count++;
        }
      } else { /* one fill: every bit except the flipped one (BitIterator.oneFillReset) */
        for (int64_t b = 0; b < 31 * blocks; ++b) {
          if (b == flip) continue;
          if (count < cap) out[count] = (int32_t)(offset + b);
          count++;
        }
      }
      offset += 31 * blocks;
    }
  }
  return count;
}

/* ------------------------------------------------------------------------------------------ */
/* Roaring portable format                                                                      */
/* ------------------------------------------------------------------------------------------ */
static uint16_t le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t le32(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); }

int64_t or_roaring_decode(const uint8_t* b, int64_t nbytes, int32_t* out, int64_t cap) {
  if (nbytes < 4) return nbytes == 0 ? 0 : -1;
  uint32_t cookie = le32(b);
  int64_t pos = 4;
  int32_t size;
  const uint8_t* runbits = NULL;
  int has_offsets;
  if ((cookie & 0xFFFF) == 12347) {
    size = (int32_t)(cookie >> 16) + 1;
    runbits = b + pos;
    pos += (size + 7) / 8;
    has_offsets = size >= 4;
  } else if (cookie == 12346) {
    size = (int32_t)le32(b + pos);
    pos += 4;
    has_offsets = 1;
  } else {
    return -1;
  }
  const uint8_t* desc = b + pos;
  pos += 4 * (int64_t)size;
  if (has_offsets) pos += 4 * (int64_t)size;
  int64_t count = 0;
  for (int32_t c = 0; c < size; ++c) {
    int32_t key = le16(desc + 4 * c);
    int32_t card = le16(desc + 4 * c + 2) + 1;
    int is_run = runbits && ((runbits[c / 8] >> (c % 8)) & 1);
    int64_t base = (int64_t)key << 16;
    if (is_run) {
      int32_t nruns = le16(b + pos);
      pos += 2;
      for (int32_t r = 0; r < nruns; ++r) {
        int32_t st = le16(b + pos + 4 * r), len = le16(b + pos + 4 * r + 2);
        for (int32_t v = st; v <= st + len; ++v) {
          if (count < cap) out[count] = (int32_t)(base + v);
          count++;
        }
      }
      pos += 4 * (int64_t)nruns;
    } else if (card <= 4096) {
      for (int32_t k = 0; k < card; ++k) {
        if (count < cap) out[count] = (int32_t)(base + le16(b + pos + 2 * k));
        count++;
      }
      pos += 2 * (int64_t)card;
    } else {
      for (int32_t k = 0; k < 65536; ++k) {
        if ((b[pos + k / 8] >> (k % 8)) & 1) {
          if (count < cap) out[count] = (int32_t)(base + k);
          count++;
        }
      }
      pos += 8192;
    }
    if (pos > nbytes) return -1;
  }
  return count;
}

/* ------------------------------------------------------------------------------------------ */
/* GenericIndexed v1 (GenericIndexed.java:479-572)                                             */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
  int32_t n;
  const uint8_t* header; /* n big-endian end offsets */
  const uint8_t* values;
} gindexed;

static int gi_read(const uint8_t** pp, const uint8_t* end, gindexed* g) {
  const uint8_t* p = *pp;
  if (end - p < 6 || p[0] != 0x01) return -1; /* v2 (multi-file) unsupported here */
  int32_t used = be32(p + 2);
  const uint8_t* body = p + 6;
  if (used < 4 || end - body < used) return -1;
  g->n = be32(body);
  g->header = body + 4;
  g->values = body + 4 + 4 * (int64_t)g->n;
  *pp = body + used;
  return 0;
}

/* element i: [start, end) inside values; returns length (0 means null/empty) */
static int32_t gi_get(const gindexed* g, int32_t i, const uint8_t** ptr) {
  int32_t start = i == 0 ? 4 : be32(g->header + 4 * (i - 1)) + 4;
  int32_t end = be32(g->header + 4 * i);
  *ptr = g->values + start;
  return end - start;
}

/* ------------------------------------------------------------------------------------------ */
/* minimal JSON probing of ColumnDescriptor                                                    */
/* ------------------------------------------------------------------------------------------ */
static int json_str(const char* js, int jlen, const char* key, const char* from, char* out, int cap) {
  char pat[64];
  snprintf(pat, sizeof pat, "\"%s\":", key);
  const char* s = from ? from : js;
  const char* e = js + jlen;
  size_t pl = strlen(pat);
  for (; s + pl <= e; ++s) {
    if (memcmp(s, pat, pl) == 0) {
      s += pl;
      while (s < e && *s == ' ') s++;
      if (s < e && *s == '"') {
        s++;
        int k = 0;
        while (s < e && *s != '"' && k < cap - 1) out[k++] = *s++;
        out[k] = 0;
        return 0;
      }
      int k = 0;
      while (s < e && *s != ',' && *s != '}' && k < cap - 1) out[k++] = *s++;
      out[k] = 0;
      return 0;
    }
  }
  return -1;
}

/* ------------------------------------------------------------------------------------------ */
/* segment model                                                                               */
/* ------------------------------------------------------------------------------------------ */
enum { OR_MISSING = 0, OR_LONG = 1, OR_FLOAT = 2, OR_DOUBLE = 3, OR_STRING = 4, OR_UNSUPPORTED = 5 };

typedef struct {
  char name[256];
  int kind;
  const uint8_t* part; /* after descriptor */
  const uint8_t* end;
  int little_endian;
  int bitmap_roaring;
  int multi_value;
  /* numeric */
  int32_t total, size_per;
  int compression;
  int long_enc;          /* 0xFF LONGS, 0x00 DELTA, 0x01 TABLE (CompressionFactory.LongEncodingFormat) */
  int vbits;             /* DELTA / TABLE: bits per packed value */
  int64_t delta_base;
  int32_t table_n;
  const uint8_t* table;  /* TABLE: table_n big-endian longs */
  const uint8_t* raw;    /* NONE layout */
  gindexed blocks;
  /* string */
  gindexed dict, bitmaps;
  int num_bytes;
  const uint8_t* vsize; /* uncompressed VSizeColumnarInts values (big-endian), or NULL */
  /* multi-value ids: V3 = row offsets as CompressedColumnarInts (mv_total = rows + 1 ints, blocks of
   * mv_size_per) + the values as CompressedVSizeColumnarInts in the fields above; VSizeColumnarMultiInts
   * = mv_count rows, mv_ends (big-endian end byte offsets), mv_vals (big-endian values) */
  int32_t mv_total, mv_size_per;
  int mv_compression;
  int mv_num_bytes; /* offsets' width: 4 for V3 (CompressedColumnarInts), numBytes of the legacy form */
  gindexed mv_blocks;
  int32_t mv_count;
  const uint8_t* mv_ends;
  const uint8_t* mv_vals;
} ocol;

typedef struct {
  blob* chunks;
  int nchunks;
  ocol* cols;
  int ncols;
  int64_t istart, iend;
  int64_t nrows;
  int bitmap_roaring;
  char err[512];
} oseg;

static ocol* find_col(oseg* s, const char* name) {
  for (int i = 0; i < s->ncols; ++i)
    if (strcmp(s->cols[i].name, name) == 0) return &s->cols[i];
  return NULL;
}

/* ---- VSizeLongSerde (VSizeLongSerde.java) restated: getBitsForMax (:41-59) and the per-size
 * deserializers Size1Des..Size64Des (:416-657), each reading the big-endian buffer exactly as the
 * Java get(index) does (getShort / getInt / getLong are big-endian, >> on them is arithmetic) ---- */
int or_bits_for_max(int64_t value) {
  static const int sizes[] = {1, 2, 4, 8, 12, 16, 20, 24, 32, 40, 48, 56, 64};
  if (value < 0) return -1;
  int nbits = 0;
  int64_t max_value = 1;
  for (int i = 0; i < 13; ++i) {
    while (nbits < sizes[i] && max_value < INT64_MAX / 2) {
      nbits++;
      max_value *= 2;
    }
    if (value <= max_value || max_value >= INT64_MAX / 2) return sizes[i];
  }
  return 64;
}

static int16_t j_short(const uint8_t* p) { return (int16_t)(((uint16_t)p[0] << 8) | p[1]); }
static int32_t j_int(const uint8_t* p) { return be32(p); }
static int64_t j_long(const uint8_t* p) { return be64(p); }

int64_t or_vsize_get(int bits, const uint8_t* b, int64_t index) {
  switch (bits) {
    case 1: return ((int8_t)b[index >> 3] >> (7 - (index & 7))) & 1;
    case 2: return ((int8_t)b[index >> 2] >> (6 - ((index & 3) << 1))) & 3;
    case 4: return ((int8_t)b[index >> 1] >> (((index + 1) & 1) << 2)) & 0xF;
    case 8: return b[index] & 0xFF;
    case 12: return (j_short(b + ((index * 3) >> 1)) >> (((index + 1) & 1) << 2)) & 0xFFF;
    case 16: return j_short(b + (index << 1)) & 0xFFFF;
    case 20: return (j_int(b + ((index * 5) >> 1)) >> ((((index + 1) & 1) << 2) + 8)) & 0xFFFFF;
    case 24: return (int64_t)((uint32_t)j_int(b + index * 3) >> 8);
    case 32: return (int64_t)(uint32_t)j_int(b + (index << 2));
    case 40: return (int64_t)((uint64_t)j_long(b + index * 5) >> 24);
    case 48: return (int64_t)((uint64_t)j_long(b + index * 6) >> 16);
    case 56: return (int64_t)((uint64_t)j_long(b + index * 7) >> 8);
    case 64: return j_long(b + (index << 3));
    default: return 0;
  }
}

/* one packed value -> the long the reader returns (Delta: base + v, :63-66; Table: table[v], :69-72) */
static int packed_value(const ocol* c, const uint8_t* buf, int64_t idx, int64_t* out) {
  int64_t v = or_vsize_get(c->vbits, buf, idx);
  if (c->long_enc == 0x00) {
    *out = (int64_t)((uint64_t)c->delta_base + (uint64_t)v);
    return 0;
  }
  if (v < 0 || v >= c->table_n) return -1; /* ArrayIndexOutOfBounds in the reference */
  *out = be64(c->table + 8 * v);
  return 0;
}

static int parse_numeric(ocol* c, const uint8_t* p) {
  /* CompressedColumnar{Longs,Floats,Doubles}Supplier.fromByteBuffer */
  if (p[0] != 0x02 && p[0] != 0x01) return -1;
  c->total = be32(p + 1);
  c->size_per = be32(p + 5);
  int8_t cid = (int8_t)p[9];
  const uint8_t* q = p + 10;
  if (p[0] == 0x01) { /* LZF_VERSION: no compression byte, LZF blocks, legacy LONGS encoding */
    c->compression = 0x00;
    c->long_enc = 0xFF;
    q = p + 9;
    return gi_read(&q, c->end, &c->blocks);
  }
  if (cid < (int8_t)0xFE) { /* CompressionFactory.hasEncodingFlag */
    uint8_t enc = *q++;
    cid = (int8_t)(cid + 126);
    c->long_enc = enc;
    if (enc == 0x00) { /* DeltaLongEncodingReader(ByteBuffer) :34-46 */
      if (q[0] != 0x01) return -1;
      c->delta_base = be64(q + 1);
      c->vbits = be32(q + 9);
      q += 13;
    } else if (enc == 0x01) { /* TableLongEncodingReader(ByteBuffer) :33-52 */
      if (q[0] != 0x01) return -1;
      c->table_n = be32(q + 1);
      if (c->table_n < 0 || c->table_n > 256) return -1; /* CompressionFactory.MAX_TABLE_SIZE */
      c->table = q + 5;
      c->vbits = or_bits_for_max(c->table_n);
      q += 5 + 8 * (size_t)c->table_n;
    } else if (enc != 0xFF) {
      return -1;
    }
  } else {
    c->long_enc = 0xFF;
  }
  c->compression = (uint8_t)cid;
  if (c->compression == 0xFE) {
    c->raw = q;
    return 0;
  }
  return gi_read(&q, c->end, &c->blocks);
}

static int parse_string(ocol* c, const uint8_t* p) {
  /* DictionaryEncodedColumnPartSerde deserializer (:283-345) */
  int version = p[0];
  const uint8_t* q = p + 1;
  int flags = 0;
  if (version >= 2) {
    flags = be32(q);
    q += 4;
  } else if (version == 1) {
    flags = 1;
  }
  c->multi_value = (flags & 3) != 0;
  if (gi_read(&q, c->end, &c->dict)) return -1;
  if (c->multi_value) {
    /* readMultiValuedColumn (DictionaryEncodedColumnPartSerde.java:183-217) */
    if (version == 1) {
      /* VSizeColumnarMultiInts.readFromByteBuffer: [0x01][numBytes][i32 size][payload: i32 count,
       * count big-endian end offsets (bytes into the values), the values as big-endian numBytes ints] */
      if (q[0] != 0x01) return -1;
      c->num_bytes = q[1];
      const int32_t size = be32(q + 2);
      if (c->num_bytes < 1 || c->num_bytes > 4 || size < 4) return -1;
      c->mv_count = be32(q + 6);
      if (c->mv_count < 0 || 4 + 4 * (int64_t)c->mv_count > size) return -1;
      c->mv_ends = q + 10;
      c->mv_vals = q + 10 + 4 * (int64_t)c->mv_count;
      q += 6 + size;
    } else if (version == 2 && (flags & 2)) {
      /* V3CompressedVSizeColumnarMultiIntsSupplier.fromByteBuffer: [0x03][offsets: CompressedColumnarInts
       * 0x02, i32 total, i32 sizePer, u8 codec, GI][values: CompressedVSizeColumnarInts] */
      if (q[0] != 0x03 || q[1] != 0x02) return -1;
      c->mv_total = be32(q + 2);
      c->mv_size_per = be32(q + 6);
      c->mv_compression = q[10];
      q += 11;
      c->mv_num_bytes = 4;
      if (gi_read(&q, c->end, &c->mv_blocks)) return -1;
      if (q[0] != 0x02) return -1;
      c->num_bytes = q[1];
      c->total = be32(q + 2);
      c->size_per = be32(q + 6);
      c->compression = q[10];
      q += 11;
      if (gi_read(&q, c->end, &c->blocks)) return -1;
    } else if (version == 2 && (flags & 1)) {
      /* CompressedVSizeColumnarMultiIntsSupplier.fromByteBuffer (:77-93): [0x02][offsets:
       * CompressedVSizeColumnarInts][values: CompressedVSizeColumnarInts] */
      if (q[0] != 0x02 || q[1] != 0x02) return -1;
      c->mv_num_bytes = q[2];
      c->mv_total = be32(q + 3);
      c->mv_size_per = be32(q + 7);
      c->mv_compression = q[11];
      if (c->mv_num_bytes < 1 || c->mv_num_bytes > 4) return -1;
      q += 12;
      if (gi_read(&q, c->end, &c->mv_blocks)) return -1;
      if (q[0] != 0x02) return -1;
      c->num_bytes = q[1];
      c->total = be32(q + 2);
      c->size_per = be32(q + 6);
      c->compression = q[10];
      q += 11;
      if (gi_read(&q, c->end, &c->blocks)) return -1;
    } else {
      return -2;
    }
  } else if (version == 2) { /* CompressedVSizeColumnarIntsSupplier */
    if (q[0] != 0x02) return -1;
    c->num_bytes = q[1];
    c->total = be32(q + 2);
    c->size_per = be32(q + 6);
    c->compression = q[10];
    q += 11;
    if (gi_read(&q, c->end, &c->blocks)) return -1;
  } else if (version == 0 || version == 3) {
    /* VSizeColumnarInts.readFromByteBuffer (data/VSizeColumnarInts.java:177-195):
     * [u8 ver 0][u8 numBytes][i32 size BE][size bytes: big-endian values + (4 - numBytes) pad] */
    if (q[0] != 0x00) return -1;
    c->num_bytes = q[1];
    int32_t nbytes = be32(q + 2);
    if (c->num_bytes < 1 || c->num_bytes > 4 || nbytes < 4 - c->num_bytes) return -1;
    c->total = (nbytes - (4 - c->num_bytes)) / c->num_bytes;
    c->vsize = q + 6;
    c->compression = -1;
    q += 6 + nbytes;
  } else {
    return -1;
  }
  if (!(flags & 4)) {
    if (gi_read(&q, c->end, &c->bitmaps)) return -1;
  } else {
    c->bitmaps.n = 0;
  }
  return 0;
}

void or_close(void* h) {
  oseg* s = (oseg*)h;
  if (!s) return;
  for (int i = 0; i < s->nchunks; ++i) free(s->chunks[i].data);
  free(s->chunks);
  free(s->cols);
  free(s);
}

void* or_open(const char* dir, char* err, int errlen) {
  char path[4096];
  blob b;
  oseg* s = (oseg*)calloc(1, sizeof(oseg));
#define FAIL(msg)                                 \
  do {                                            \
    snprintf(err, (size_t)errlen, "%s", msg);     \
    or_close(s);                                  \
    return NULL;                                  \
  } while (0)
  snprintf(path, sizeof path, "%s/version.bin", dir);
  if (read_file(path, &b) || b.size != 4) FAIL("missing version.bin");
  int ver = be32(b.data);
  free(b.data);
  if (ver != 9) FAIL("expected version 9");
  snprintf(path, sizeof path, "%s/meta.smoosh", dir);
  blob meta;
  if (read_file(path, &meta)) FAIL("missing meta.smoosh");
  /* first line: v1,maxChunk,numChunks */
  char* text = (char*)malloc((size_t)meta.size + 1);
  memcpy(text, meta.data, (size_t)meta.size);
  text[meta.size] = 0;
  free(meta.data);
  char* save = NULL;
  char* line = strtok_r(text, "\n", &save);
  int nchunks = 0;
  if (!line || sscanf(line, "v1,%*d,%d", &nchunks) != 1) {
    free(text);
    FAIL("bad meta.smoosh");
  }
  s->nchunks = nchunks;
  s->chunks = (blob*)calloc((size_t)nchunks, sizeof(blob));
  for (int i = 0; i < nchunks; ++i) {
    snprintf(path, sizeof path, "%s/%05d.smoosh", dir, i);
    if (read_file(path, &s->chunks[i])) {
      free(text);
      FAIL("missing smoosh chunk");
    }
  }
  int cap = 64;
  s->cols = (ocol*)calloc((size_t)cap, sizeof(ocol));
  const uint8_t* index_drd = NULL;
  const uint8_t* index_end = NULL;
  while ((line = strtok_r(NULL, "\n", &save)) != NULL) {
    char name[256];
    int chunk;
    long st, en;
    char* lastc = strrchr(line, ',');
    if (!lastc) continue;
    /* name may contain commas: parse the last three fields from the right */
    char* c3 = lastc;
    *c3 = 0;
    char* c2 = strrchr(line, ',');
    if (!c2) continue;
    *c2 = 0;
    char* c1 = strrchr(line, ',');
    if (!c1) continue;
    *c1 = 0;
    snprintf(name, sizeof name, "%s", line);
    chunk = atoi(c1 + 1);
    st = atol(c2 + 1);
    en = atol(c3 + 1);
    if (chunk < 0 || chunk >= nchunks || en > s->chunks[chunk].size) continue;
    const uint8_t* base = s->chunks[chunk].data + st;
    const uint8_t* end = s->chunks[chunk].data + en;
    if (strcmp(name, "index.drd") == 0) {
      index_drd = base;
      index_end = end;
      continue;
    }
    if (strcmp(name, "metadata.drd") == 0) continue;
    if (s->ncols == cap) {
      cap *= 2;
      s->cols = (ocol*)realloc(s->cols, sizeof(ocol) * (size_t)cap);
    }
    ocol* c = &s->cols[s->ncols++];
    memset(c, 0, sizeof *c);
    snprintf(c->name, sizeof c->name, "%s", name);
    int32_t jlen = be32(base);
    const char* js = (const char*)base + 4;
    c->part = base + 4 + jlen;
    c->end = end;
    char vt[64] = {0}, pt[64] = {0}, bo[64] = {0}, bt[64] = {0};
    json_str(js, jlen, "valueType", NULL, vt, sizeof vt);
    const char* parts = strstr(js, "\"parts\"");
    json_str(js, jlen, "type", parts, pt, sizeof pt);
    json_str(js, jlen, "byteOrder", NULL, bo, sizeof bo);
    const char* bsf = strstr(js, "\"bitmapSerdeFactory\"");
    if (bsf && bsf < js + jlen) json_str(js, jlen, "type", bsf, bt, sizeof bt);
    c->little_endian = strcmp(bo, "BIG_ENDIAN") != 0;
    c->bitmap_roaring = strcmp(bt, "roaring") == 0;
    int rc = 0;
    if (strcmp(pt, "long") == 0 || strcmp(pt, "longV2") == 0) {
      c->kind = OR_LONG;
      rc = parse_numeric(c, c->part + (strcmp(pt, "longV2") == 0 ? 4 : 0));
    } else if (strcmp(pt, "double") == 0 || strcmp(pt, "doubleV2") == 0) {
      c->kind = OR_DOUBLE;
      rc = parse_numeric(c, c->part + (strcmp(pt, "doubleV2") == 0 ? 4 : 0));
    } else if (strcmp(pt, "float") == 0 || strcmp(pt, "floatV2") == 0) {
      c->kind = OR_FLOAT;
      rc = parse_numeric(c, c->part + (strcmp(pt, "floatV2") == 0 ? 4 : 0));
    } else if (strcmp(pt, "stringDictionary") == 0) {
      c->kind = OR_STRING;
      rc = parse_string(c, c->part);
    } else {
      c->kind = OR_UNSUPPORTED;
    }
    if (rc) c->kind = OR_UNSUPPORTED;
  }
  free(text);
  if (!index_drd) FAIL("missing index.drd");
  {
    gindexed cols, dims;
    const uint8_t* q = index_drd;
    if (gi_read(&q, index_end, &cols) || gi_read(&q, index_end, &dims) || index_end - q < 16) FAIL("bad index.drd");
    s->istart = be64(q);
    s->iend = be64(q + 8);
    q += 16;
    s->bitmap_roaring = 0;
    if (index_end - q > 4) {
      int32_t l = be32(q);
      if (l > 0 && l <= index_end - q - 4 && memmem(q + 4, (size_t)l, "roaring", 7)) s->bitmap_roaring = 1;
    }
  }
  ocol* t = find_col(s, "__time");
  if (!t || t->kind != OR_LONG) FAIL("missing __time");
  s->nrows = t->total;
  return s;
#undef FAIL
}

int64_t or_num_rows(void* h) { return ((oseg*)h)->nrows; }
void or_interval(void* h, int64_t* st, int64_t* en) {
  *st = ((oseg*)h)->istart;
  *en = ((oseg*)h)->iend;
}
int or_bitmap_roaring(void* h) { return ((oseg*)h)->bitmap_roaring; }
int or_num_columns(void* h) { return ((oseg*)h)->ncols; }
const char* or_column_name(void* h, int i) { return ((oseg*)h)->cols[i].name; }
int or_column_kind(void* h, const char* name) {
  ocol* c = find_col((oseg*)h, name);
  return c ? c->kind : OR_MISSING;
}

/* compress-lzf 1.0.4 LZFDecoder.decode restated (the library is a pom dependency, not vendored):
 * a sequence of chunks "ZV" + type; type 0 = u16 BE length + raw bytes, type 1 = u16 BE compressed
 * length + u16 BE uncompressed length + liblzf data (ChunkDecoder.decodeChunk: ctrl < 32 -> ctrl + 1
 * literals, else length (ctrl >> 5) + 2 with 7 extended by the next byte, back-reference distance
 * ((ctrl & 31) << 8 | next) + 1, copied byte by byte so overlaps repeat). Returns decoded bytes or -1. */
int64_t or_lzf_decompress(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap) {
  int64_t ip = 0, op = 0;
  while (ip < n) {
    if (ip + 5 > n || in[ip] != 'Z' || in[ip + 1] != 'V') return -1;
    const int type = in[ip + 2];
    const int64_t len = ((int64_t)in[ip + 3] << 8) | in[ip + 4];
    if (type == 0) {
      ip += 5;
      if (ip + len > n || op + len > cap) return -1;
      memcpy(out + op, in + ip, (size_t)len);
      ip += len;
      op += len;
    } else if (type == 1) {
      if (ip + 7 > n) return -1;
      const int64_t ulen = ((int64_t)in[ip + 5] << 8) | in[ip + 6];
      ip += 7;
      const int64_t end = ip + len, oend = op + ulen;
      if (end > n || oend > cap) return -1;
      while (ip < end) {
        int ctrl = in[ip++];
        if (ctrl < 32) {
          int64_t run = ctrl + 1;
          if (ip + run > end || op + run > oend) return -1;
          memcpy(out + op, in + ip, (size_t)run);
          ip += run;
          op += run;
        } else {
          int64_t l = ctrl >> 5;
          if (l == 7) {
            if (ip >= end) return -1;
            l += in[ip++];
          }
          if (ip >= end) return -1;
          int64_t ref = op - ((int64_t)(ctrl & 31) << 8) - 1 - in[ip++];
          l += 2;
          if (ref < 0 || op + l > oend) return -1;
          for (int64_t k = 0; k < l; ++k) out[op + k] = out[ref + k];
          op += l;
        }
      }
      if (op != oend) return -1;
    } else {
      return -1;
    }
  }
  return op;
}

/* decode block i of a block-layout column into dst (cap bytes); returns decoded bytes */
static int64_t decode_block(ocol* c, int32_t i, uint8_t* dst, int64_t cap) {
  const uint8_t* p;
  int32_t len = gi_get(&c->blocks, i, &p);
  if (c->compression == 0x01) return or_lz4_decompress(p, len, dst, cap);
  if (c->compression == 0x00) return or_lzf_decompress(p, len, dst, cap);
  if (c->compression == 0xFF) {
    if (len > cap) return -1;
    memcpy(dst, p, (size_t)len);
    return len;
  }
  return -1;
}

/* Materialize a numeric column as raw little-endian values of its stored width. */
static int read_numeric_raw(ocol* c, uint8_t* out, int width) {
  if (c->long_enc == 0x00 || c->long_enc == 0x01) {
    /* EntireLayout (NONE): one packed stream; BlockLayout: every block restarts at index 0 */
    int64_t* o = (int64_t*)out;
    if (c->compression == 0xFE) {
      for (int64_t r = 0; r < c->total; ++r)
        if (packed_value(c, c->raw, r, &o[r])) return -1;
      return 0;
    }
    uint8_t* buf = (uint8_t*)calloc(65536 + 16, 1);
    int64_t done = 0;
    for (int32_t b = 0; b < c->blocks.n && done < c->total; ++b) {
      int64_t got = decode_block(c, b, buf, 65536 + 16);
      int64_t vals = c->size_per;
      if (vals > c->total - done) vals = c->total - done;
      if (got < 0 || got < (c->vbits * vals + 7) / 8) {
        free(buf);
        return -1;
      }
      if (got < 65536 + 16) memset(buf + got, 0, (size_t)(65536 + 16 - got));
      for (int64_t r = 0; r < vals; ++r)
        if (packed_value(c, buf, r, &o[done + r])) {
          free(buf);
          return -1;
        }
      done += vals;
    }
    free(buf);
    return done == c->total ? 0 : -1;
  }
  if (c->compression == 0xFE) {
    memcpy(out, c->raw, (size_t)c->total * (size_t)width);
    return 0;
  }
  uint8_t* buf = (uint8_t*)malloc(65536 + 16);
  int64_t done = 0;
  for (int32_t b = 0; b < c->blocks.n && done < c->total; ++b) {
    int64_t got = decode_block(c, b, buf, 65536 + 16);
    if (got < 0) {
      free(buf);
      return -1;
    }
    int64_t vals = c->size_per;
    if (vals > c->total - done) vals = c->total - done;
    if (got < vals * width) {
      free(buf);
      return -1;
    }
    memcpy(out + done * width, buf, (size_t)(vals * width));
    done += vals;
  }
  free(buf);
  return done == c->total ? 0 : -1;
}

/* Typed reads with the selector coercions of the reference (LongColumnSelector /
 * DoubleColumnSelector / FloatColumnSelector): out type is the selector's get*() type. */
static int64_t java_d2l(double d) {
  if (d != d) return 0;
  if (d >= 9223372036854775807.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}

int or_read_column(void* h, const char* name, int as_kind, void* out) {
  oseg* s = (oseg*)h;
  ocol* c = find_col(s, name);
  int64_t n = s->nrows;
  if (!c || c->kind == OR_STRING || c->kind == OR_UNSUPPORTED) {
    /* missing / non-numeric column: NilColumnValueSelector -> 0 (replaceWithDefault) */
    memset(out, 0, (size_t)n * (as_kind == OR_FLOAT ? 4 : 8));
    return c ? 1 : 0;
  }
  int width = c->kind == OR_FLOAT ? 4 : 8;
  uint8_t* raw = (uint8_t*)malloc((size_t)n * (size_t)width + 8);
  if (read_numeric_raw(c, raw, width)) {
    free(raw);
    return -1;
  }
  for (int64_t r = 0; r < n; ++r) {
    int64_t lv = 0;
    double dv = 0;
    float fv = 0;
    if (c->kind == OR_LONG) {
      memcpy(&lv, raw + 8 * r, 8);
      dv = (double)lv;
      fv = (float)lv;
    } else if (c->kind == OR_DOUBLE) {
      memcpy(&dv, raw + 8 * r, 8);
      lv = java_d2l(dv);
      fv = (float)dv;
    } else {
      memcpy(&fv, raw + 4 * r, 4);
      lv = java_d2l((double)fv);
      dv = (double)fv;
    }
    if (as_kind == OR_LONG) ((int64_t*)out)[r] = lv;
    else if (as_kind == OR_DOUBLE) ((double*)out)[r] = dv;
    else ((float*)out)[r] = fv;
  }
  free(raw);
  return 0;
}

int32_t or_dim_cardinality(void* h, const char* name) {
  ocol* c = find_col((oseg*)h, name);
  if (!c || c->kind != OR_STRING) return -1;
  return c->dict.n;
}

int32_t or_dim_value(void* h, const char* name, int32_t id, const char** ptr) {
  ocol* c = find_col((oseg*)h, name);
  if (!c || c->kind != OR_STRING || id < 0 || id >= c->dict.n) return -1;
  const uint8_t* p;
  int32_t len = gi_get(&c->dict, id, &p);
  *ptr = (const char*)p;
  return len;
}

/* CompressedVSizeColumnarInts.get (:254-353): little-endian, 3 bytes = getInt & 0xFFFFFF */
int or_dim_ids(void* h, const char* name, int32_t* out) {
  oseg* s = (oseg*)h;
  ocol* c = find_col(s, name);
  if (!c || c->kind != OR_STRING) return -1;
  if (c->multi_value) return -2; /* row value lists not restated (grouping on them unsupported) */
  if (c->vsize) { /* VSizeColumnarInts.get (:124-127): getInt(pos) >>> (32 - 8 * numBytes), big-endian */
    for (int64_t k = 0; k < c->total; ++k) {
      const uint8_t* p = c->vsize + k * c->num_bytes;
      uint32_t v = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
      out[k] = (int32_t)(v >> (32 - 8 * c->num_bytes));
    }
    return 0;
  }
  uint8_t* buf = (uint8_t*)malloc(65536 + 16);
  int64_t done = 0;
  for (int32_t b = 0; b < c->blocks.n && done < c->total; ++b) {
    memset(buf, 0, 65536 + 16);
    int64_t got = decode_block(c, b, buf, 65536 + 16);
    if (got < 0) {
      free(buf);
      return -1;
    }
    int64_t vals = c->size_per;
    if (vals > c->total - done) vals = c->total - done;
    for (int64_t k = 0; k < vals; ++k) {
      const uint8_t* p = buf + k * c->num_bytes;
      uint32_t v;
      if (c->little_endian) {
        v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
        if (c->num_bytes < 4) v &= (1u << (8 * c->num_bytes)) - 1;
      } else {
        v = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
        v >>= 32 - 8 * c->num_bytes;
      }
      out[done + k] = (int32_t)v;
    }
    done += vals;
  }
  free(buf);
  return done == c->total ? 0 : -1;
}

/* Rows [row0, row0 + n) of one column, decoding only the blocks that hold them (the CPU baseline's
 * per-chunk reads, cpu_engine.c): a plain block-layout numeric column (LONGS encoding, LZ4 / LZF /
 * UNCOMPRESSED blocks) as raw 8-byte values (`kind` OR_LONG / OR_DOUBLE, no coercion), or a
 * single-value compressed dictionary-id column as int32 ids (kind OR_STRING). -1: other layouts. */
int or_read_rows(void* h, const char* name, int kind, int64_t row0, int64_t n, void* out) {
  oseg* s = (oseg*)h;
  ocol* c = find_col(s, name);
  if (!c || n < 0 || row0 < 0 || row0 + n > s->nrows) return -1;
  const int ids = kind == OR_STRING;
  if (ids ? (c->kind != OR_STRING || c->multi_value || c->vsize || !c->little_endian) : (c->kind != kind || c->long_enc != 0xFF))
    return -1;
  if (c->compression == 0xFE || c->size_per <= 0) return -1;
  const int width = ids ? c->num_bytes : 8;
  uint8_t* buf = (uint8_t*)malloc(65536 + 16);
  int64_t r = row0;
  int rc = 0;
  while (r < row0 + n) {
    const int32_t b = (int32_t)(r / c->size_per);
    const int64_t first = (int64_t)b * c->size_per;
    int64_t last = first + c->size_per;
    if (last > row0 + n) last = row0 + n;
    memset(buf, 0, 65536 + 16);
    const int64_t got = b < c->blocks.n ? decode_block(c, b, buf, 65536 + 16) : -1;
    if (got < (last - first) * width) {
      rc = -1;
      break;
    }
    for (int64_t k = r; k < last; ++k) {
      const uint8_t* p = buf + (k - first) * width;
      if (ids) {
        uint32_t v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
        if (width < 4) v &= (1u << (8 * width)) - 1;
        ((int32_t*)out)[k - row0] = (int32_t)v;
      } else {
        memcpy((uint8_t*)out + (k - row0) * 8, p, 8);
      }
    }
    r = last;
  }
  free(buf);
  return rc;
}

/* CompressedVSizeColumnarInts values of a column (its blocks / num_bytes / little_endian), n of them */
static int read_vsize_ids(ocol* c, int64_t n, int32_t* out) {
  uint8_t* buf = (uint8_t*)malloc(65536 + 16);
  int64_t done = 0;
  for (int32_t b = 0; b < c->blocks.n && done < n; ++b) {
    memset(buf, 0, 65536 + 16);
    int64_t got = decode_block(c, b, buf, 65536 + 16);
    int64_t vals = c->size_per;
    if (vals > n - done) vals = n - done;
    if (got < vals * c->num_bytes) {
      free(buf);
      return -1;
    }
    for (int64_t k = 0; k < vals; ++k) {
      const uint8_t* p = buf + k * c->num_bytes;
      uint32_t v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
      if (c->num_bytes < 4) v &= (1u << (8 * c->num_bytes)) - 1;
      out[done + k] = (int32_t)v;
    }
    done += vals;
  }
  free(buf);
  return done == n ? 0 : -1;
}

/* Row value lists of a multi-value dimension (V3CompressedVSizeColumnarMultiIntsSupplier.get(index):
 * values offsets[index] .. offsets[index + 1]; VSizeColumnarMultiInts.get: the end byte offsets of
 * rows index - 1 and index). offsets = rows + 1 ints; values NULL: *nvalues only. */
int or_dim_multi(void* h, const char* name, int32_t* offsets, int32_t* values, int64_t* nvalues) {
  oseg* s = (oseg*)h;
  ocol* c = find_col(s, name);
  if (!c || c->kind != OR_STRING || !c->multi_value) return -1;
  const int64_t rows = s->nrows;
  if (c->mv_ends) {
    if (c->mv_count != rows) return -1;
    int64_t prev = 0;
    if (offsets) offsets[0] = 0;
    for (int64_t r = 0; r < rows; ++r) {
      const int64_t e = be32(c->mv_ends + 4 * r);
      if (e < prev || e % c->num_bytes) return -1;
      prev = e;
      if (offsets) offsets[r + 1] = (int32_t)(e / c->num_bytes);
    }
    *nvalues = prev / c->num_bytes;
    if (values)
      for (int64_t k = 0; k < *nvalues; ++k) {
        const uint8_t* p = c->mv_vals + k * c->num_bytes;
        uint32_t v = 0;
        for (int b = 0; b < c->num_bytes; ++b) v = (v << 8) | p[b];
        values[k] = (int32_t)v;
      }
    return 0;
  }
  if (c->mv_total != rows + 1) return -1;
  int32_t* off = offsets ? offsets : (int32_t*)malloc((size_t)(rows + 1) * 4);
  ocol oc = *c; /* the offsets part: little-endian ints (4 bytes for V3, numBytes for the legacy form) */
  oc.blocks = c->mv_blocks;
  oc.compression = c->mv_compression;
  oc.size_per = c->mv_size_per;
  oc.num_bytes = c->mv_num_bytes;
  int rc = read_vsize_ids(&oc, rows + 1, off);
  if (!rc) {
    for (int64_t r = 0; r < rows; ++r)
      if (off[r + 1] < off[r] || off[0] != 0) rc = -1;
  }
  if (!rc) {
    *nvalues = off[rows];
    if (*nvalues > c->total) rc = -1;
  }
  if (!offsets) free(off);
  if (rc || !values) return rc;
  return read_vsize_ids(c, *nvalues, values);
}

/* rows of dictionary id `id`'s bitmap (BitmapIndexColumnPartSupplier.getBitmap) */
int64_t or_dim_bitmap(void* h, const char* name, int32_t id, int32_t* out, int64_t cap) {
  oseg* s = (oseg*)h;
  ocol* c = find_col(s, name);
  if (!c || c->kind != OR_STRING || id < 0 || id >= c->bitmaps.n) return -1;
  const uint8_t* p;
  int32_t len = gi_get(&c->bitmaps, id, &p);
  if (c->bitmap_roaring) return or_roaring_decode(p, len, out, cap);
  return or_concise_decode(p, len, out, cap);
}

/* ------------------------------------------------------------------------------------------ */
/* Aggregation with Java semantics, rows visited in ascending order (cursor order)             */
/* ------------------------------------------------------------------------------------------ */
enum {
  AGG_COUNT = 0,
  AGG_LONG_SUM = 1,
  AGG_DOUBLE_SUM = 2,
  AGG_FLOAT_SUM = 3,
  AGG_LONG_MIN = 4,
  AGG_LONG_MAX = 5,
  AGG_DOUBLE_MIN = 6,
  AGG_DOUBLE_MAX = 7,
  AGG_FLOAT_MIN = 8,
  AGG_FLOAT_MAX = 9
};

static int is_negzero_d(double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  return u == 0x8000000000000000ull;
}
static int is_negzero_f(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u == 0x80000000u;
}
/* java.lang.Math.min/max(double, double) */
static double jmin_d(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && is_negzero_d(b)) return b;
  return a <= b ? a : b;
}
static double jmax_d(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && is_negzero_d(a)) return b;
  return a >= b ? a : b;
}
static float jmin_f(float a, float b) {
  if (a != a) return a;
  if (a == 0.0f && b == 0.0f && is_negzero_f(b)) return b;
  return a <= b ? a : b;
}
static float jmax_f(float a, float b) {
  if (a != a) return a;
  if (a == 0.0f && b == 0.0f && is_negzero_f(a)) return b;
  return a >= b ? a : b;
}

/* Initial value of an aggregator (Aggregator.reset / BufferAggregator.init). */
void or_agg_init(int kind, int32_t ngroups, void* state) {
  for (int32_t g = 0; g < ngroups; ++g) {
    switch (kind) {
      case AGG_COUNT:
      case AGG_LONG_SUM: ((int64_t*)state)[g] = 0; break;
      case AGG_LONG_MIN: ((int64_t*)state)[g] = INT64_MAX; break;
      case AGG_LONG_MAX: ((int64_t*)state)[g] = INT64_MIN; break;
      case AGG_DOUBLE_SUM: ((double*)state)[g] = 0.0; break;
      case AGG_DOUBLE_MIN: ((double*)state)[g] = INFINITY; break;
      case AGG_DOUBLE_MAX: ((double*)state)[g] = -INFINITY; break;
      case AGG_FLOAT_SUM: ((float*)state)[g] = 0.0f; break;
      case AGG_FLOAT_MIN: ((float*)state)[g] = INFINITY; break;
      case AGG_FLOAT_MAX: ((float*)state)[g] = -INFINITY; break;
    }
  }
}

/*
 * state[groups[k]] op= values[rows[k]] for k = 0..n-1 in order. values is already coerced to the
 * aggregator's input type (int64 for long aggs, double for double aggs, float for float aggs).
 */
void or_agg_apply(int kind, int64_t n, const int32_t* rows, const int32_t* groups, const void* values, void* state) {
  for (int64_t k = 0; k < n; ++k) {
    int32_t r = rows[k], g = groups[k];
    switch (kind) {
      case AGG_COUNT: ((int64_t*)state)[g] += 1; break;
      case AGG_LONG_SUM: {
        uint64_t a = (uint64_t)((int64_t*)state)[g], b = (uint64_t)((const int64_t*)values)[r];
        ((int64_t*)state)[g] = (int64_t)(a + b); /* two's complement wrap */
        break;
      }
      case AGG_LONG_MIN: {
        int64_t v = ((const int64_t*)values)[r];
        if (v < ((int64_t*)state)[g]) ((int64_t*)state)[g] = v;
        break;
      }
      case AGG_LONG_MAX: {
        int64_t v = ((const int64_t*)values)[r];
        if (v > ((int64_t*)state)[g]) ((int64_t*)state)[g] = v;
        break;
      }
      case AGG_DOUBLE_SUM: ((double*)state)[g] += ((const double*)values)[r]; break;
      case AGG_DOUBLE_MIN: ((double*)state)[g] = jmin_d(((double*)state)[g], ((const double*)values)[r]); break;
      case AGG_DOUBLE_MAX: ((double*)state)[g] = jmax_d(((double*)state)[g], ((const double*)values)[r]); break;
      case AGG_FLOAT_SUM: {
        volatile float acc = ((float*)state)[g] + ((const float*)values)[r]; /* float accumulator */
        ((float*)state)[g] = acc;
        break;
      }
      case AGG_FLOAT_MIN: ((float*)state)[g] = jmin_f(((float*)state)[g], ((const float*)values)[r]); break;
      case AGG_FLOAT_MAX: ((float*)state)[g] = jmax_f(((float*)state)[g], ((const float*)values)[r]); break;
    }
  }
}

/* AggregatorFactory.combine for two partial states (e.g. DoubleSumAggregator.combineValues,
 * FloatSumAggregator.combineValues in float, LongMaxAggregator.combineValues). */
void or_agg_combine(int kind, int32_t n, void* acc, const void* other) {
  for (int32_t i = 0; i < n; ++i) {
    switch (kind) {
      case AGG_COUNT:
      case AGG_LONG_SUM:
        ((int64_t*)acc)[i] = (int64_t)((uint64_t)((int64_t*)acc)[i] + (uint64_t)((const int64_t*)other)[i]);
        break;
      case AGG_LONG_MIN:
        if (((const int64_t*)other)[i] < ((int64_t*)acc)[i]) ((int64_t*)acc)[i] = ((const int64_t*)other)[i];
        break;
      case AGG_LONG_MAX:
        if (((const int64_t*)other)[i] > ((int64_t*)acc)[i]) ((int64_t*)acc)[i] = ((const int64_t*)other)[i];
        break;
      case AGG_DOUBLE_SUM: ((double*)acc)[i] += ((const double*)other)[i]; break;
      case AGG_DOUBLE_MIN: ((double*)acc)[i] = jmin_d(((double*)acc)[i], ((const double*)other)[i]); break;
      case AGG_DOUBLE_MAX: ((double*)acc)[i] = jmax_d(((double*)acc)[i], ((const double*)other)[i]); break;
      case AGG_FLOAT_SUM: {
        volatile float s = ((float*)acc)[i] + ((const float*)other)[i];
        ((float*)acc)[i] = s;
        break;
      }
      case AGG_FLOAT_MIN: ((float*)acc)[i] = jmin_f(((float*)acc)[i], ((const float*)other)[i]); break;
      case AGG_FLOAT_MAX: ((float*)acc)[i] = jmax_f(((float*)acc)[i], ((const float*)other)[i]); break;
    }
  }
}
