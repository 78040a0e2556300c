/*
 * segment_tools.c — native helpers for the segment writer (writer.py).
 *
 * This is the build's equivalent of the bitmap-building half of
 * StringDimensionMergerV9 (processing/.../segment/StringDimensionMergerV9.java:350-430):
 * row ids are appended in ascending order to one mutable Concise set per
 * dictionary value, exactly as WrappedConciseBitmap.add -> ConciseSet.append does
 * (extendedset/.../intset/ConciseSet.java:435-492 append, :494-539 appendLiteral,
 * :545-591 appendFill), and the words are then emitted unchanged as
 * ImmutableConciseSet.newImmutableFromMutable does (ImmutableConciseSet.java:127-133).
 *
 * Words are returned as host-order int32; writer.py byte-swaps them to the
 * big-endian on-disk order (ImmutableConciseSet.toBytes, ImmutableConciseSet.java:811-818).
 *
 * Pure C, no GPU code: segments are written once, off the query path.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ALL_ZEROS_LITERAL ((int32_t)0x80000000)
#define ALL_ONES_LITERAL ((int32_t)0xFFFFFFFF)
#define SEQUENCE_BIT ((int32_t)0x40000000)

typedef struct {
  int32_t* w;   /* caller-provided output */
  int64_t n;    /* words used */
  int32_t last; /* last set bit, -1 when empty */
} cset;

static int one_bit(uint32_t x) { return x != 0 && (x & (x - 1)) == 0; }
static int ctz32(uint32_t x) { return __builtin_ctz(x); }
static int is_literal(int32_t w) { return w < 0; }
static int is_zero_seq(int32_t w) { return (w & (int32_t)0xC0000000) == 0; }
static int is_one_seq(int32_t w) { return (w & (int32_t)0xC0000000) == SEQUENCE_BIT; }

static void append_literal(cset* s, int32_t word) {
  if (s->n == 1 && word == ALL_ZEROS_LITERAL && s->w[0] == 0x01FFFFFF) return;
  if (s->n == 0) {
    s->w[s->n++] = word;
    return;
  }
  int32_t lw = s->w[s->n - 1];
  if (word == ALL_ZEROS_LITERAL) {
    if (lw == ALL_ZEROS_LITERAL) {
      s->w[s->n - 1] = 1;
    } else if (is_zero_seq(lw)) {
      s->w[s->n - 1]++;
    } else if (one_bit((uint32_t)lw & 0x7FFFFFFFu)) {
      s->w[s->n - 1] = 1 | ((1 + ctz32((uint32_t)lw)) << 25);
    } else {
      s->w[s->n++] = word;
    }
  } else if (word == ALL_ONES_LITERAL) {
    if (lw == ALL_ONES_LITERAL) {
      s->w[s->n - 1] = SEQUENCE_BIT | 1;
    } else if (is_one_seq(lw)) {
      s->w[s->n - 1]++;
    } else if (one_bit(~(uint32_t)lw)) {
      s->w[s->n - 1] = SEQUENCE_BIT | 1 | ((1 + ctz32(~(uint32_t)lw)) << 25);
    } else {
      s->w[s->n++] = word;
    }
  } else {
    s->w[s->n++] = word;
  }
}

static void append_fill(cset* s, int32_t length, int32_t fill) {
  fill &= SEQUENCE_BIT;
  if (length == 1) {
    append_literal(s, fill == 0 ? ALL_ZEROS_LITERAL : ALL_ONES_LITERAL);
    return;
  }
  if (s->n == 0) {
    s->w[s->n++] = fill | (length - 1);
    return;
  }
  int32_t lw = s->w[s->n - 1];
  if (is_literal(lw)) {
    if (fill == 0 && lw == ALL_ZEROS_LITERAL) {
      s->w[s->n - 1] = length;
    } else if (fill == SEQUENCE_BIT && lw == ALL_ONES_LITERAL) {
      s->w[s->n - 1] = SEQUENCE_BIT | length;
    } else if (fill == 0 && one_bit((uint32_t)lw & 0x7FFFFFFFu)) {
      s->w[s->n - 1] = length | ((1 + ctz32((uint32_t)lw)) << 25);
    } else if (fill == SEQUENCE_BIT && one_bit(~(uint32_t)lw)) {
      s->w[s->n - 1] = SEQUENCE_BIT | length | ((1 + ctz32(~(uint32_t)lw)) << 25);
    } else {
      s->w[s->n++] = fill | (length - 1);
    }
  } else {
    if ((lw & (int32_t)0xC0000000) == fill) {
      s->w[s->n - 1] += length;
    } else {
      s->w[s->n++] = fill | (length - 1);
    }
  }
}

static void append_bit(cset* s, int32_t i) {
  if (s->n == 0) {
    int32_t zero_blocks = i / 31;
    if (zero_blocks == 1) {
      s->w[s->n++] = ALL_ZEROS_LITERAL;
    } else if (zero_blocks > 1) {
      s->w[s->n++] = zero_blocks - 1;
    }
    s->w[s->n++] = ALL_ZEROS_LITERAL | (1 << (i % 31));
    s->last = i;
    return;
  }
  int32_t bit = (s->last % 31) + i - s->last;
  if (bit >= 31) {
    int32_t zero_blocks = bit / 31 - 1;
    bit = bit % 31;
    if (zero_blocks > 0) append_fill(s, zero_blocks, 0);
    append_literal(s, ALL_ZEROS_LITERAL | (1 << bit));
  } else {
    s->w[s->n - 1] |= 1 << bit;
    if (s->w[s->n - 1] == ALL_ONES_LITERAL) {
      s->n--;
      append_literal(s, ALL_ONES_LITERAL);
    }
  }
  s->last = i;
}

/* Encode one ascending row list. out must hold at least n + 2 words. Returns #words. */
int64_t dgt_concise_encode(const int32_t* rows, int64_t n, int32_t* out) {
  cset s = {out, 0, -1};
  for (int64_t k = 0; k < n; ++k) append_bit(&s, rows[k]);
  return s.n;
}

/*
 * Encode the bitmap of every dictionary id of one single-value column.
 * ids[n_rows] in [0, card). Writes words for id 0, 1, ... back to back into out_words and the
 * per-id word counts into out_counts[card]. out_words must hold n_rows + 2*card words.
 * Returns total words, or -1 on bad input.
 */
int64_t dgt_concise_encode_column(const int32_t* ids, int64_t n_rows, int32_t card,
                                  int32_t* out_words, int64_t* out_counts) {
  int64_t* start = (int64_t*)calloc((size_t)card + 1, sizeof(int64_t));
  int32_t* rows = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n_rows > 0 ? n_rows : 1));
  if (!start || !rows) { free(start); free(rows); return -1; }
  for (int64_t r = 0; r < n_rows; ++r) {
    if (ids[r] < 0 || ids[r] >= card) { free(start); free(rows); return -1; }
    start[ids[r] + 1]++;
  }
  for (int32_t v = 0; v < card; ++v) start[v + 1] += start[v];
  int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(card > 0 ? card : 1));
  memcpy(fill, start, sizeof(int64_t) * (size_t)card);
  for (int64_t r = 0; r < n_rows; ++r) rows[fill[ids[r]]++] = (int32_t)r;
  int64_t total = 0;
  for (int32_t v = 0; v < card; ++v) {
    int64_t nw = dgt_concise_encode(rows + start[v], start[v + 1] - start[v], out_words + total);
    out_counts[v] = nw;
    total += nw;
  }
  free(fill);
  free(start);
  free(rows);
  return total;
}

/* ---- LZF encoder for the segment writer (compress-lzf 1.0.4 chunk format, what
 * CompressionStrategy.LZFCompressor writes through LZFEncoder.appendEncoded): the input is cut
 * into chunks of at most 65535 bytes; each chunk is "ZV" + type 1 + u16 BE compressed length +
 * u16 BE uncompressed length + liblzf data, or "ZV" + type 0 + u16 BE length + raw bytes when
 * compression does not pay. liblzf data: ctrl < 32 -> ctrl + 1 literals; otherwise a back-reference
 * of length (ctrl >> 5) + 2 (7 -> + next byte) at distance ((ctrl & 31) << 8 | next) + 1. ---- */
static int64_t lzf_chunk(const uint8_t* in, int n, uint8_t* out) {
  enum { HBITS = 14, MAX_OFF = 8192, MAX_REF = 264, MAX_LIT = 32 };
  static int32_t table[1 << HBITS];
  for (int i = 0; i < (1 << HBITS); ++i) table[i] = -1;
  int64_t op = 0;
  int lit_start = 0, ip = 0;
#define FLUSH_LITS(upto)                                 \
  while (lit_start < (upto)) {                           \
    int run = (upto) - lit_start;                        \
    if (run > MAX_LIT) run = MAX_LIT;                    \
    out[op++] = (uint8_t)(run - 1);                      \
    memcpy(out + op, in + lit_start, (size_t)run);       \
    op += run;                                           \
    lit_start += run;                                    \
  }
  while (ip + 2 < n) {
    uint32_t h = ((uint32_t)in[ip] << 16 | (uint32_t)in[ip + 1] << 8 | in[ip + 2]) * 2654435761u >> (32 - HBITS);
    int32_t ref = table[h];
    table[h] = ip;
    if (ref >= 0 && ip - ref <= MAX_OFF && in[ref] == in[ip] && in[ref + 1] == in[ip + 1] && in[ref + 2] == in[ip + 2]) {
      int len = 3;
      while (len < MAX_REF && ip + len < n && in[ref + len] == in[ip + len]) len++;
      FLUSH_LITS(ip);
      int off = ip - ref - 1, l = len - 2;
      if (l < 7) {
        out[op++] = (uint8_t)((l << 5) | (off >> 8));
      } else {
        out[op++] = (uint8_t)((7 << 5) | (off >> 8));
        out[op++] = (uint8_t)(l - 7);
      }
      out[op++] = (uint8_t)(off & 0xFF);
      ip += len;
      lit_start = ip;
    } else {
      ip++;
    }
  }
  FLUSH_LITS(n);
#undef FLUSH_LITS
  return op;
}

int64_t dgt_lzf_compress(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap) {
  int64_t op = 0;
  uint8_t* tmp = (uint8_t*)malloc(65535 * 2 + 64);
  for (int64_t pos = 0; pos < n || (n == 0 && pos == 0); ) {
    int len = (int)(n - pos > 65535 ? 65535 : n - pos);
    int64_t c = lzf_chunk(in + pos, len, tmp);
    int64_t need = c < len ? 7 + c : 5 + len;
    if (op + need > cap) {
      free(tmp);
      return -1;
    }
    out[op++] = 'Z';
    out[op++] = 'V';
    if (c < len) {
      out[op++] = 1;
      out[op++] = (uint8_t)(c >> 8);
      out[op++] = (uint8_t)c;
      out[op++] = (uint8_t)(len >> 8);
      out[op++] = (uint8_t)len;
      memcpy(out + op, tmp, (size_t)c);
      op += c;
    } else {
      out[op++] = 0;
      out[op++] = (uint8_t)(len >> 8);
      out[op++] = (uint8_t)len;
      memcpy(out + op, in + pos, (size_t)len);
      op += len;
    }
    pos += len;
    if (n == 0) break;
  }
  free(tmp);
  return op;
}
