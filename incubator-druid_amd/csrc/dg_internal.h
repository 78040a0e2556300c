// dg_internal.h — structures shared by the host engine (dg_segment.cpp, dg_engine.cpp) and the
// HIP kernels (dg_kernels.hip). Device-side descriptors are plain PODs copied into HBM per call.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/druidgpu.h"

namespace dg {

constexpr int kMaxAggs = 16;
constexpr int kBlockBytes = 65536;  // CompressedPools.BUFFER_SIZE (segment/CompressedPools.java:39)

// stored codecs (CompressionStrategy ids, data/CompressionStrategy.java:48-107)
enum Codec : int32_t { CODEC_LZF = 0x00, CODEC_LZ4 = 0x01, CODEC_UNCOMPRESSED = 0xFF, CODEC_NONE = 0xFE };

// value kinds a kernel can read from a column view
enum ViewKind : int32_t { VIEW_ABSENT = 0, VIEW_LONG = 1, VIEW_FLOAT = 2, VIEW_DOUBLE = 3, VIEW_IDS = 4 };

// accumulator slot ops (all slots are 8 bytes)
enum SlotOp : int32_t { OP_ADD_I64 = 0, OP_ADD_F64 = 1, OP_MIN_U64 = 2, OP_MAX_U64 = 3 };

// A column as the kernels see it: value(row) lives at blocks[row >> log2_per] + (row & mask) * width.
// flags: kViewBigEndian = dictionary ids stored big-endian (uncompressed VSizeColumnarInts);
// kViewFused = an aggregator's input whose tagged blocks (low pointer bit) the decoder already
// aggregated (Lz4Job.red_*): the scan takes the aggregator's identity for their rows.
struct ColView {
  const uint8_t* const* blocks;
  int32_t log2_per;
  int32_t width;
  int32_t kind;
  int32_t pad;  // flags
};
constexpr int32_t kViewBigEndian = 1;
constexpr int32_t kViewFused = 2;

// LZ4 sequence checkpoints: built once per block at attach (lz4_index_block), one entry per
// kLzSeqPerCp sequences (2 * kLzSeqPerCp for the rare block with more than kLzMaxCps * kLzSeqPerCp
// sequences) = the compressed offset where that sequence's token starts. They let the decoder
// parse every interval of a block in parallel (one interval per thread); the bytes stay LZ4.
constexpr int kLzSeqPerCp = 8;
constexpr int kLzMaxSeqPerCp = 2 * kLzSeqPerCp;  // the decoder's per-thread register budget
constexpr int kLzMaxCps = 1024;                  // one interval per decoder thread

// One LZ4 block to decode (compressed bytes are 16-byte aligned in the device image).
struct Lz4Job {
  const uint8_t* src;
  uint8_t* dst;
  const uint32_t* cp;  // checkpoints of this block
  int32_t src_len;
  int32_t expect_len;  // bytes that must come out (>= rows * width of the block)
  int32_t ncp;         // number of checkpoints; < 0: the block failed validation at attach
  int32_t dec_len;     // decoded length found at attach
  int32_t wide;        // checkpoints every 2 * kLzSeqPerCp sequences (decoded by the wide kernel)
  int32_t light;       // few sequences, short copy chains: decoded by the light kernel (k_lz4_light);
                       // > 0: sequences per light checkpoint (cp[ncp .. ncp + nfine) = the light checkpoints)
  int32_t nfine;       // light checkpoints (one per light-decoder thread)
  // 0: the block's bytes go to dst contiguously (a decode slot). > 0: the block holds 8-byte values
  // and value v goes to dst + v * vstride (a column of the groupBy payload records, written in place);
  // bytes past expect_len are then not written (they would land in the next segment's records)
  int32_t vstride;
  // run block (k_lz4_run): the block's run index (lz4_run_index) and its shape; null: another decoder
  const uint8_t* rx;
  int32_t run_n;    // intervals (one per k_lz4_run thread)
  int32_t run_far;  // bytes of the far-copy table after the intervals
  // flow block (wide & kLzFlow): its schedule (lz4_flow_schedule) and highest level
  const uint8_t* lvl;
  int32_t nlvl;
  // Decode fused with a timeseries aggregator (the block's rows share one bucket, no filter): instead
  // of writing its 8-byte values the decoder folds them with red_op (agg_input_raw(red_kind,
  // red_vkind, value)) and combines the block's result into the bucket's slot *red_dst atomically.
  // Null: the block is written out.
  uint64_t* red_dst;
  int32_t red_op;
  int32_t red_kind;
  int32_t red_vkind;
  int32_t red_code;  // kRed*: the fold in the value's own type (generic: agg_input_raw + combine_op)
  // a filtered scan's fold (round 6): only the rows whose bit is set in the segment's row bitset
  // red_bits (null: every row) fold; value v of the block is row red_row0 + v
  const uint32_t* red_bits;
  int64_t red_row0;
};
// A run of one column's LZ4 blocks of one decoder kind, decoded in one launch. Built per call in O(1)
// from the column's attach-time tables: block k = list[i] for i in [i0, i0 + n) (the column's blocks of
// that kind, ascending), its job = desc[k] (every query-independent Lz4Job field, expect_len = the bytes
// of its rows) with dst = dst_base + k * dst_step (null dst_base: a fused fold writes nothing), vstride
// and the fused fold (red_*) from the task.
struct Lz4Task {
  const Lz4Job* desc;
  const int32_t* list;
  int32_t i0, n;
  uint8_t* dst_base;
  int64_t dst_step;
  uint64_t* red_dst;
  int32_t vstride, red_op, red_kind, red_vkind, red_code;
  int32_t red_rpb;           // rows per block (the fold's row of value v of block k: k * red_rpb + v)
  const uint32_t* red_bits;  // the fold's row bitset (null: every row)
};
// A decoder launch: blocks [0, njobs) are per-block jobs, the rest belong to tasks (task_of[b - njobs] =
// the task of block b, task_first[t] = the launch block of task t's first block).
struct Lz4Launch {
  const Lz4Job* jobs;
  const Lz4Task* tasks;
  const int32_t* task_of;
  const int32_t* task_first;
  int32_t njobs;
  int32_t pad;
};
// decoder kinds of a block under the default routes (the partition run_decodes_only launches by)
enum : int32_t { kKindRun = 0, kKindGen0 = 1, kKindLight = 5, kKinds = 6 };  // kKindGen0 + wide: general

// folds of a fused decode (Lz4Job.red_code): int64 sum / max / min of a long column, double sum of a
// double column in their native types (converted to the slot encoding once per block); others generic
enum : int32_t { kRedGeneric = 0, kRedLongSum = 1, kRedDoubleSum = 2, kRedLongMax = 3, kRedLongMin = 4 };

// Light blocks (literal-heavy: random ids, high-entropy values): at most kLtMaxCps checkpoint
// intervals and copy chains of at most kLtMaxDepth hops. k_lz4_light decodes them with a small
// sequence table in LDS (many blocks per CU), resolving every output byte back to its literal.
constexpr int kLtMaxCps = 256;
#ifndef DG_LT_THREADS  // (A/B builds)
#define DG_LT_THREADS 512
#endif
constexpr int kLtThreads = DG_LT_THREADS;  // light-decoder threads (at most one light checkpoint interval each)
constexpr int kLtMaxDepth = 16;

// Run blocks: LZ4 blocks of 8-byte value runs (sequential longs, timestamps, constant columns) whose
// matches copy from at most 8 bytes back, except a few far copies. The attach-time run index cuts the
// block into intervals of >= kRunTarget output bytes at sequence boundaries and stores, per interval,
// its token offset, its output start and the 8 output bytes before it (its window); every far copy's
// bytes are listed once. k_lz4_run then decodes each interval independently in one thread: the last
// 8 output bytes ride in a register, a near copy is a shift of it, and every aligned 8-byte value is
// emitted as it completes. Index layout per block (16-byte aligned): u64 win[n], u32 tok[n] (token
// offset | far-table offset << 17), u16 out[n], zero pad to 16, the far table, zero pad to 16.
// Interval length and threads of the run decoder: one thread's serial chain is its interval, so the
// block's latency follows it; 96-byte intervals over 768 threads (round 6, same box: configs[4]a 8.03
// -> 7.46 ms, topN and the headline within noise to -3 %; 128 / 64 bytes close behind,
// profiles/r06_v51_ab_run.log) against 256 bytes over 256 threads before. (A/B builds override both.)
#ifndef DG_RUN_TARGET
#define DG_RUN_TARGET 96
#define DG_RUN_THREADS 768
#endif
constexpr int kRunThreads = DG_RUN_THREADS;  // one interval per thread (kBlockBytes / kRunTarget intervals at most)
constexpr int kRunTarget = DG_RUN_TARGET;    // output bytes per interval, at least (the last one excepted)
constexpr int kRunFarMax = 4096;   // far-copy bytes a run block may list
constexpr int kRunMaxRun = 1024;   // longest literal run / match of a run block (one thread's serial work)
constexpr int kRunLdsMax = 40960;  // staged input + far table of one run block (four workgroups per CU)
static_assert(kBlockBytes / kRunTarget <= kRunThreads, "one interval per k_lz4_run thread");
inline int run_index_bytes(int nint, int nfar) { return ((14 * nint + 15) & ~15) + ((nfar + 15) & ~15); }
inline int run_lds_bytes(int n, int nfar) { return ((n + 15) & ~15) + 16 + ((nfar + 15) & ~15) + 16; }
// Run index of one validated LZ4 block decoding to dec_len bytes, appended to *idx (16-byte aligned);
// returns false (nothing appended) when the block is not a run block.
bool lz4_run_index(const uint8_t* in, int n, int dec_len, std::vector<uint8_t>* idx, int* nint, int* nfar);
// Literal-only LZ4 block (a single sequence of literals, as LZ4 writes incompressible data): the
// offset of its literal bytes (= its decoded image), or -1.
int lz4_literal_start(const uint8_t* in, int n);
// Host decode of a validated LZ4 block into out (kBlockBytes); returns the decoded length or -1.
int lz4_decode_host(const uint8_t* in, int n, uint8_t* out);
// Decoder routes a query may take (read once per column): kRouteRun = run blocks go to k_lz4_run
// (off with DG_NO_RUN_DECODE), kRouteFlow = flow blocks go to k_lz4_decode_flow (off with
// DG_NO_FLOW_DECODE); same-box A/B and the tests of the other decoders turn them off
constexpr int kRouteRun = 1, kRouteFlow = 2;
int decode_routes();
struct BlockColumn;
// the job of LZ4 block k of a column (dst, expect and the routes given; no fused fold)
Lz4Job lz4_job(const BlockColumn& b, int32_t k, uint8_t* dst, int32_t expect, int routes);

// Flow blocks (Lz4Job.wide & kLzFlow, set at attach): general blocks of at most kLzMaxCps intervals
// that are not distance-8 class chains (at most a quarter of their bytes copied from 8 back) and whose
// copy chains are at most kFlowMaxDepth hops deep. The attach-time schedule ranks every match by its
// copy-chain level; k_lz4_decode_flow writes the literals into a byte image in LDS, then the matches
// level by level, each level's matches spread evenly over the threads.
constexpr int kLzFlow = 2;
constexpr int kFlowSideWgs = 192;  // persistent flow-decoder workgroups beside the groupBy sort (dg_engine.cpp)
constexpr int kFlowMaxDepth = 64;
constexpr int kFlowRecBytes = 48;  // schedule bytes per checkpoint interval (lz4_flow_schedule)
constexpr int kCompSlack = 64;     // bytes of zeros before and after a column's packed LZ4 blocks

// One LZF block (compress-lzf chunk stream, CompressionStrategy.LZFDecompressor) -> dst.
struct LzfJob {
  const uint8_t* src;
  uint8_t* dst;
  int32_t src_len;
  int32_t expect_len;  // bytes that must come out
};

// Expansion of one block of a DELTA / TABLE long column (CompressionFactory.LongEncodingFormat,
// CompressionFactory.java:153-188): `rows` values of `bits` bits packed MSB-first
// (VSizeLongSerde deserializers, VSizeLongSerde.java:416-657) -> little-endian int64 at dst.
struct VsJob {
  const uint8_t* src;   // packed block (decoded LZ4 slot, uncompressed block or NONE range)
  int64_t* dst;         // size_per int64 slots
  const int64_t* table; // TABLE: table values; DELTA: nullptr
  int64_t base;         // DELTA: base (DeltaLongEncodingReader.read, :63-66)
  int32_t rows;
  int32_t bits;
  int32_t table_n;
  int32_t pad;
};

// Host-side validating parse of one LZ4 block (lz4-java safe-decompressor semantics): appends the
// block's checkpoints to *cps and returns the decoded length, or -1 for a malformed block.
// *wide: bit 0 = the block keeps every other checkpoint (more than kLzMaxCps * kLzSeqPerCp sequences),
// kLzFlow = a flow block (decoded by k_lz4_decode_flow).
// *light (optional): the block qualifies for the light decoder (kLtMaxCps / kLtMaxDepth).
// *light = g > 0 when light: the block's checkpoints are followed by *nfine light checkpoints, one
// every g sequences (g the fewest sequences per checkpoint that fit the light decoder's threads).
// levels (optional): a flow block's schedule is appended (lz4_flow_schedule: per checkpoint interval
// kLzSeqPerCp u16 ranks of its matches in (level, position) order and kLzSeqPerCp u16 forwarded
// distances; then the u16 start of every level's ranks, padded to 16 bytes) and *nlvl = its highest
// level; without it no block is a flow block.
int lz4_index_block(const uint8_t* in, int n, std::vector<uint32_t>* cps, int* wide, int* light = nullptr,
                    int* nfine = nullptr, std::vector<uint8_t>* levels = nullptr, int* nlvl = nullptr);

struct AggPlan {
  int32_t n;
  int32_t kind[kMaxAggs];   // DG_AGG_*
  int32_t op[kMaxAggs];     // SlotOp
};

// One segment's share of a scan kernel.
struct ScanJob {
  int32_t nrows;
  int32_t tile_begin;       // first global tile index of this segment
  const uint32_t* bitset;   // null: every row passes the filter
  ColView time;             // VIEW_ABSENT when the time column is not needed
  int64_t t_lo, t_hi;       // rows with t in [t_lo, t_hi)
  int64_t bucket0;          // start of the first bucket (calendar: its index in `bounds`)
  int64_t period;           // 0 = ALL (single bucket); calendar: 1
  const int64_t* bounds;    // calendar granularity: ascending bucket starts (null: period grid)
  int32_t nbounds;
  int32_t desc;             // descending cursors (floatSum recurrence runs backwards)
  int32_t nbuckets;         // timeseries: buckets; topN: table keys (cardinality, x buckets when key_card)
  int32_t key_card;         // topN over granularity buckets: key = bucket * key_card + id (0: key = id)
  ColView vals[kMaxAggs];   // input column per aggregator
  const uint32_t* agg_bits[kMaxAggs];  // FilteredAggregatorFactory row matcher per aggregator (null: all rows)
  ColView key;              // topN: dimension ids (a multi-value dimension: its value stream)
  ColView key_off;          // topN over a multi-value dimension: row value offsets (VIEW_ABSENT otherwise)
  uint64_t* out;            // accumulator table of this segment
  // one-bucket timeseries (round 6): the tiles' records [tiles][1 + naggs], stored plainly and folded
  // into `out` by k_scan_combine — hundreds of tiles' atomics on one record serialised (configs[0]:
  // 1,464 on one line) — null: per-tile atomics into `out`
  uint64_t* part;
};

// groupBy by sort (dg_sort.hip) and the floatSum row-order pass. One job per segment of the call.
// A selected row becomes (key, row ref): key = [seg slot | bucket | merged id of every dimension],
// most significant field first, so ascending keys are the reference's merged row order
// (timestamp, then dimension values in Java String order, nulls first); the row ref is the row's
// index over the call's segments (row_base + row), so a stable sort keeps equal keys in
// (segment, row) order.
constexpr int kMaxGroupDims = 8;

struct GbJob {
  int32_t nrows;
  int32_t tile_begin;           // first keygen tile (kTileRows rows) of this segment
  uint32_t row_base;            // row ref of row 0
  int32_t ndims;
  const uint32_t* bitset;       // null: every row passes the filter
  ColView time;                 // VIEW_ABSENT when the time column is not needed
  int64_t t_lo, t_hi;           // rows with t in [t_lo, t_hi)
  int64_t bucket0;              // origin of the bucket index (shared by the call's segments in a merge)
  int64_t period;               // 0 = ALL; calendar: 1 (bucket index = position in `bounds`)
  const int64_t* bounds;        // calendar granularity: ascending bucket starts (null: period grid)
  int32_t nbounds;
  int32_t desc;                 // descending cursors: the floatSum pass runs each cell backwards
  int32_t seg_slot, seg_shift;  // key field of the segment (0 / 0 when the groups are merged)
  int32_t bucket_shift, bucket_bits;
  ColView dims[kMaxGroupDims];           // dictionary ids (a multi-value dimension: its value stream)
  ColView moff[kMaxGroupDims];           // multi-value dimension: row value offsets (VIEW_ABSENT otherwise)
  int32_t multi;                         // some dimension is multi-value: rows explode into groupings
  int32_t skip_empty;                    // an empty value list yields no element (topN) instead of null (groupBy)
  uint32_t inplace;                      // row-ref mode: payload columns the LZ4 decoder wrote (bit a)
  const int32_t* remap[kMaxGroupDims];  // local dictionary id -> merged id (null: identity)
  int32_t null_gid[kMaxGroupDims];      // merged id of the null value (a missing dimension's rows)
  int32_t dim_shift[kMaxGroupDims];
  int32_t dim_bits[kMaxGroupDims];
  ColView vals[kMaxAggs];
  const uint32_t* agg_bits[kMaxAggs];  // FilteredAggregatorFactory row matcher per aggregator
  // floatSum sink of the per-segment engines (timeseries / topN): slot (bucket * fs_mul + id) of this
  // segment's [keys][1 + naggs] accumulator table
  uint64_t* fs_out;
  int64_t fs_mul;
};

// Device buffers of one sort-based grouping; *_n are device words (counts known only on the device).
struct SortBufs {
  uint64_t* keys[2];      // packed (refs null): [key | row ref in the low ref_bits bits]; else keys
  uint32_t* refs[2];      // row refs when the key and the ref do not fit one word, else null
  int ref_bits;           // packed: bits of the element index (the sort key starts there); else 0
  uint64_t* payload;      // the aggregators' inputs of each element (device slot encoding): [cap][pw]
                          // by element reference
  int row_refs;           // element reference = the row's index over the call (one element per row,
                          // payload columns may be decoded in place); else the element index
  int pw;
  int cur;                // which of the ping-pong buffers holds the result
  uint32_t* tile_cnt;     // keygen tiles: selected rows, then their offsets
  uint32_t* n;            // [0] selected rows, [1] groups
  uint64_t* lb_status;    // radix look-back status per (tile, digit) of one pass: flag in the top two bits,
                          // the tile's digit count or inclusive prefix below (prefixes reach n: 64-bit)
  uint32_t* bin_total;    // [kRsMaxPasses][kMaxBins] digit totals + [kRsMaxPasses] tile counters
  uint32_t* run_cnt;      // per sort tile: run heads, then their offsets
  int64_t cap;            // element capacity (rows of the call)
  int ntiles_sort;        // sort tiles of `cap`
};

// ---------------------------------------------------------------------------------------------
// Host-side objects
// ---------------------------------------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { reset(); }
  void reset();
  bool alloc(size_t bytes);
  template <class T> T* as() const { return static_cast<T*>(p); }
};

// A block-layout column (numeric values or dictionary ids) resident in HBM.
struct BlockColumn {
  int32_t total = 0;      // rows
  int32_t size_per = 0;   // rows per block (power of two)
  int32_t log2_per = 0;
  int32_t width = 0;      // bytes per value
  int32_t codec = 0;
  int32_t nblocks = 0;
  int32_t big_endian = 0;  // VSizeColumnarInts ids (uncompressed dimension)
  // DELTA / TABLE long encodings: blocks hold `vbits`-bit packed values (0 = plain LONGS);
  // `width` stays 8, the width of the expanded view the kernels read
  int32_t vbits = 0;
  int32_t table_n = 0;
  int64_t delta_base = 0;
  DevBuf table;                        // TABLE: int64[table_n]
  int64_t stored_bytes = 0;            // on-HBM bytes of all blocks (algorithmic bytes of a full scan)
  std::vector<int64_t> comp_off;       // host copy: offset of block b inside comp
  std::vector<int32_t> comp_len;
  std::vector<int64_t> cp_off;         // LZ4: first checkpoint of block b inside cps
  std::vector<int32_t> cp_n;           // LZ4: checkpoints of block b (-1: malformed block)
  std::vector<uint8_t> cp_wide;        // LZ4: block b keeps a checkpoint every 2 * kLzSeqPerCp sequences
  std::vector<uint8_t> cp_light;       // LZ4: block b goes to the light decoder (sequences per light checkpoint)
  std::vector<int32_t> cp_fine;        // LZ4: light checkpoints of block b (after its cp_n checkpoints)
  std::vector<int32_t> dec_len;        // LZ4: decoded bytes of block b
  bool time_col = false;               // the __time column: min8 / max8 are recorded at attach
  std::vector<int64_t> min8, max8;     // __time LZ4 LONGS: smallest / largest row time of block b (host
                                       // decode at attach; the cursor's uniform-block skip needs no
                                       // assumption on the row order inside a block)
  int64_t index_bytes = 0;             // LZ4: bytes of the index a query reads (checkpoints; run index
                                       // of run blocks instead)
  std::vector<int64_t> lit_off;        // LZ4: literal-only block b's literal bytes inside comp (16-byte
                                       // aligned: its decoded image, viewed in place), -1 otherwise;
                                       // empty: no literal-only block
  std::vector<int64_t> run_off;        // LZ4: block b's run index inside runx (-1: not a run block)
  std::vector<int32_t> run_n;          // LZ4: its intervals
  std::vector<int32_t> run_far;        // LZ4: its far-copy bytes
  DevBuf runx;                         // LZ4: run indexes of the run blocks
  std::vector<int64_t> lvl_off;        // LZ4: flow block b's level schedule inside lvls (-1: none)
  std::vector<int32_t> lvl_n;          // LZ4: its highest level
  DevBuf lvls;                         // LZ4: level schedules of the flow blocks
  DevBuf comp;                         // LZ4: packed compressed blocks (16-byte aligned)
  DevBuf cps;                          // LZ4: uint32 checkpoints of every block
  DevBuf raw;                          // UNCOMPRESSED: 64 KiB slot per block; NONE: flat values
  DevBuf block_ptrs;                   // const uint8_t*[nblocks]: raw slots (UNCOMPRESSED/NONE)
  // LZ4 decode tables (attach time, default routes): every block's query-independent job (device,
  // Lz4Job[nblocks]) and, per decoder kind, the blocks of that kind ascending (host + device, at
  // kind_at[kind] in kind_dev) with the prefix sums of their stored bytes / run-index or checkpoint
  // bytes. Literal-only and empty blocks are in no list.
  DevBuf job_desc;
  DevBuf kind_dev;
  std::vector<int32_t> kind_list[kKinds];
  std::vector<int32_t> kind_pos[kKinds];    // [k] = blocks of the kind below block k (nblocks + 1): O(1) ranges
  std::vector<int64_t> kind_bytes[kKinds];  // [i] = stored bytes of list[0 .. i)
  int64_t kind_at[kKinds] = {0, 0, 0, 0, 0, 0};
};

// A piece of a long serialized bitmap: Concise = a run of whole words starting at row `row0`;
// Roaring = one container (info = cardinality - 1 | 1 << 31 for a run container).
struct BmPiece {
  int64_t off;   // byte offset of the piece's data inside the column's bm_bytes
  int64_t row0;  // first row the piece covers
  int32_t len;   // bytes
  int32_t info;  // Roaring container: (card - 1) | run << 31; Concise: 0
};
constexpr int kConcisePieceWords = 4096;  // Concise bitmaps above 2x this are cut into pieces of it
constexpr int kRoaringSplitBytes = 32768; // Roaring bitmaps above this are cut into containers

constexpr int kOrderSlots = 8;

struct Column {
  std::string name;
  int type = DG_COL_MISSING;
  BlockColumn data;
  // dictionary-encoded string column
  std::vector<std::string> dict;
  std::vector<uint8_t> dict_null;      // 1 = null / empty value
  std::vector<uint64_t> dict_hash;     // value_hash of every dictionary value (cross-segment merges)
  int bitmap_roaring = 0;
  bool has_bitmaps = false;
  bool multi_value = false;            // row r's values: data[mv_off[r] .. mv_off[r + 1])
  BlockColumn mv_off;                  // multi-value: rows + 1 value offsets (4-byte ints)
  std::vector<int64_t> bm_off;         // byte offset of each bitmap inside bm_bytes (4-byte aligned)
  std::vector<int32_t> bm_len;
  DevBuf bm_bytes;
  // long bitmaps split at attach so one bitmap's expansion spreads over many workgroups: bitmap i's
  // pieces are bm_pieces[bm_piece_first[i] .. bm_piece_first[i + 1]) (empty = not split); empty
  // vector = no bitmap of the column is split
  std::vector<int32_t> bm_piece_first;
  std::vector<BmPiece> bm_pieces;
  // dictionary orders handed in by dg_segment_set_dim_order (slot = 2 * DG_ORDER_* + inverted):
  // rank of every dictionary id under the StringComparator, comparator-equal values share a rank
  DevBuf order_rank[kOrderSlots];
  std::vector<int32_t> order_host[kOrderSlots];
  int32_t order_ties[kOrderSlots] = {};
  bool order_set[kOrderSlots] = {};
  // topN bin index (built by the first topN over the column on the device, then reused): the rows
  // grouped by dictionary-id bin (id >> kTopnIxShift), each with its id's low bits (TopnIx)
  DevBuf tix_perm, tix_lid, tix_base;
  bool tix_ready = false;
};

// Merged dictionary of one dimension over a set of segments (the union of their sorted
// dictionaries in Java String order, nulls first) + each segment's local id -> merged id table in
// HBM. GroupByMergingQueryRunnerV2 merges rows by dimension VALUE (:188-246); the engine merges by
// merged id instead, which orders exactly like the values. Built on the host once per
// (segment set, dimension) and cached in the context, like a datasource-level dictionary.
struct MergedDict {
  std::vector<uint64_t> uids;  // attach serials of the segments, in call order
  std::string dim;
  std::vector<std::string> values;
  std::vector<uint8_t> is_null;
  int32_t null_gid = -1;                        // merged id of null (-1: no null value)
  std::vector<std::unique_ptr<DevBuf>> remap;   // per segment: int32[card] (empty = identity)
};

struct Context {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::mutex mu;
  // grow-only scratch arenas reused across calls
  DevBuf scratch[6];
  DevBuf pinned_dummy;
  hipEvent_t ev[8] = {};
  // side stream: the groupBy payload columns decode on it while the main stream builds and sorts the
  // keys (the two only meet at the reduce); side_ev[0] = its inputs are staged, [1..2] = decode span
  hipStream_t side = nullptr;
  hipEvent_t side_ev[3] = {};
  // the general LZ4 decoder's own span on each stream: [0, 1] main, [2, 3] side (its roofline
  // figures, dg_metrics)
  hipEvent_t gen_ev[4] = {};
  // a small call's short decoders (run, light) on the side stream beside the general decoder:
  // [0] their jobs are staged, [1] they are done (no timing)
  hipEvent_t ovl_ev[2] = {};
  // dg_context_set_limit(DG_LIMIT_GROUP_ELEMENTS): most sort elements one groupBy call may build
  uint64_t max_elements = ~0ull;
  std::vector<std::shared_ptr<MergedDict>> dict_cache;  // most recent last
  // device blocks of groupBy results: live (size by pointer) and released for reuse
  std::map<void*, size_t> block_size;
  std::vector<std::pair<void*, size_t>> free_blocks;
};

struct Segment {
  Context* ctx = nullptr;
  uint64_t uid = 0;  // attach serial (never reused: a cache key that outlives the segment)
  std::string dir;
  int64_t nrows = 0;
  int64_t istart = 0, iend = 0;
  int64_t min_time = 0, max_time = 0;
  int bitmap_roaring = 0;
  std::vector<std::unique_ptr<Column>> columns;
  std::map<std::string, Column*> by_name;
  int64_t device_bytes = 0;
  Column* find(const std::string& n) const {
    auto it = by_name.find(n);
    return it == by_name.end() ? nullptr : it->second;
  }
};

// 64-bit hash of a dimension value (FNV-1a + avalanche); identity across segments' dictionaries
constexpr uint64_t kNullValueHash = 0x6e756c6c2d76616cull;
inline uint64_t value_hash(const std::string& v) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (unsigned char ch : v) h = (h ^ ch) * 0x100000001b3ull;
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return h == kNullValueHash ? h + 1 : h;
}

// error reporting
int set_error(int code, const char* fmt, ...);
#define DG_HIP(call)                                                                       \
  do {                                                                                     \
    hipError_t _e = (call);                                                                \
    if (_e != hipSuccess) return ::dg::set_error(DG_ERR_DEVICE, "%s: %s", #call, hipGetErrorString(_e)); \
  } while (0)

// segment loading (dg_segment.cpp)
int load_segment(Context* ctx, const char* dir, Segment** out);
int segment_from_rows(Context* ctx, int64_t nrows, const int64_t* ts, int64_t istart, int64_t iend,
                      const dg_row_column* cols, int ncols, Segment** out);
int java_compare_str(const char* a, const char* b);  // String.compareTo over UTF-8 bytes (dg_engine.cpp)

// a failed enqueue inside a void launcher (e.g. the memset of look-back status): recorded per thread,
// returned as DG_ERR_DEVICE by the call's finish_call (dg_engine.cpp)
void note_launch_error(hipError_t e);
hipError_t take_launch_error();

// kernel launchers (dg_kernels.hip)
constexpr int kLz4ProfWords = 32;  // per-block phase stamps of the decoder (diagnostic builds of the call)
// blocks of one kind: wide (2 * kLzSeqPerCp sequences per checkpoint) or not
// flow blocks (wide & kLzFlow): flow_wgs > 0 caps the grid at that many persistent workgroups
void launch_lz4_decode(const Lz4Launch& L, int nblocks, int wide, int32_t* d_err, hipStream_t s, uint64_t* d_prof = nullptr,
                       int flow_wgs = 0);
void launch_lz4_light(const Lz4Launch& L, int nblocks, int32_t* d_err, hipStream_t s, uint64_t* d_prof = nullptr);
// run blocks (rx set); stage: 0 = read the input from L1/L2 (64 KiB of LDS per block, two per CU: beside
// another stream's LDS-heavy kernels), 1 = stage it in LDS when the launch is small (latency mode),
// 2 = stage it (a launch that has the GPU to itself)
void launch_lz4_run(const Lz4Launch& L, int nblocks, int stage, int32_t* d_err, hipStream_t s);
void launch_lzf_decode(const LzfJob* d_jobs, int njobs, int32_t* d_err, hipStream_t s);
void launch_vsize_expand(const VsJob* d_jobs, int njobs, int32_t max_rows, int32_t* d_err, hipStream_t s);
// one multi-value dimension's decoded row lists, validated before use (bit 2 of the error word)
struct MvCheck {
  ColView vals;
  ColView offs;
  int64_t rows;
  int64_t nvals;  // values stored (the offsets may not pass it)
  int64_t card;   // dictionary size (every value id must be below it)
};
// measurement probes (dg_debug_probe)
void launch_probe_copy(const void* in, void* out, int64_t bytes, hipStream_t s);
void launch_probe_chain(uint32_t* word, int n, hipStream_t s);
void launch_probe_gather(const uint64_t* words, const void* rec, int64_t n, uint64_t* out, hipStream_t s);
void launch_probe_fill(uint64_t* words, void* rec, int64_t n, hipStream_t s);
// DG_PROBE_SORT: n words sorted iters times by launch_radix_sort (events around the sort only)
int probe_sort(int64_t n, int iters, double* ms, hipStream_t st);
void launch_mv_check(const MvCheck* d_jobs, int njobs, int32_t* d_err, hipStream_t s);
// VSizeLongSerde.getSerializedSize (VSizeLongSerde.java:61-65)
inline int64_t vsize_serialized(int bits, int64_t n) { return (bits * n + 7) / 8 + 4; }
// Concise words [off, off + len) whose first word starts at row row0 (null: 0), OR-ed into sets[target]
void launch_concise_or(const uint8_t* bm_base, const int64_t* d_off, const int32_t* d_len, const int32_t* d_target,
                       const int64_t* d_row0, int nbitmaps, uint32_t* const* d_sets, int64_t limit_bits, hipStream_t s);
// single Roaring containers (pieces): data at off, rows from row0, info as BmPiece; four per workgroup
void launch_roaring_pieces(const uint8_t* bm_base, const int64_t* d_off, const int64_t* d_row0, const int32_t* d_info,
                           const int32_t* d_target, int npieces, uint32_t* const* d_sets, int64_t limit_bits,
                           hipStream_t s);
void launch_roaring_or(const uint8_t* bm_base, const int64_t* d_off, const int32_t* d_len, const int32_t* d_target,
                       int nbitmaps, uint32_t* const* d_sets, int32_t* d_err, int64_t limit_bits, hipStream_t s);
void launch_filter_eval(const int32_t* d_prog, int prog_len, uint32_t* const* d_sets, uint32_t* out, int64_t nrows,
                        unsigned long long* d_count, hipStream_t s);
// Row predicate of a filter on a numeric column: the reference evaluates it per row as a post-filter
// (QueryableIndexStorageAdapter.makeCursors :244-260 -> FilteredOffset.java:40-105) through the
// column's ValueMatcher ({Long,Float,Double}ValueMatcherColumnSelectorStrategy, the filters'
// DruidLong/Float/DoublePredicate); here it becomes one more row bitset of the filter program.
enum PredKind : int32_t {
  PRED_FALSE = 0,       // matches no row (unparseable selector value, empty IN, ALWAYS_FALSE bounds)
  PRED_LONG_RANGE = 1,  // long column: [lo, hi] with strictness (makeLongPredicateFromBounds)
  PRED_LONG_SET = 2,    // long column: value in the sorted set (IN / selector)
  PRED_ORD_RANGE = 3,   // float/double column: Double.compare range on (double) value, as ordered keys
  PRED_BITS_SET = 4,    // float/double column: floatToIntBits / doubleToLongBits in the sorted set
  PRED_LONG_LEX = 5,    // long column: String.valueOf(value) vs UTF-8 bound strings (LEXICOGRAPHIC)
  PRED_ID_SET = 6,      // string column without a bitmap index: row id's bit in `set` (64-bit words)
};
struct NumPred {
  int32_t kind;
  int32_t has_lo, has_hi, lo_strict, hi_strict;
  int32_t nset;
  int64_t lo, hi;         // LONG_RANGE: bounds; ORD_RANGE: ordered keys (uint64 bit patterns)
  const int64_t* set;     // LONG_SET / BITS_SET: sorted values / canonical bit patterns
  const uint8_t* lo_str;  // LONG_LEX: bound bytes
  const uint8_t* hi_str;
  int32_t lo_len, hi_len;
};
// out: bitset words of rows [0, nrows) (bit r of word r >> 5); v: the decoded numeric column
// voff: row value offsets of a multi-value id column (VIEW_ABSENT otherwise); PRED_ID_SET over a
// multi-value column: has_lo = whether an empty row (the null value) matches
void launch_num_pred(ColView v, ColView voff, int64_t nrows, NumPred p, uint32_t* out, hipStream_t s);
// one record of accumulator slots, passed by value (a kernel argument: no staging copy)
struct SlotInit {
  uint64_t v[kMaxAggs + 1];
};
void launch_fill_u64(uint64_t* p, int64_t n_rows_of_slots, int slots_per_row, const SlotInit& init, hipStream_t s);
void launch_scan_agg(const ScanJob* d_jobs, const int32_t* d_tile_job, int ntiles, AggPlan plan, int topn, hipStream_t s);
// the tiles' records of the jobs with `part` folded into `out` (one workgroup per job, tree order)
void launch_scan_combine(const ScanJob* d_jobs, int njobs, AggPlan plan, hipStream_t s);
// topN aggregation with LDS-private dictionary-id ranges: workgroup (p, s) owns ids
// [p * range, (p + 1) * range) of segment s, scans every row of the segment and writes its range of
// the record table with plain stores (no HBM atomics). Applicable when the table needs at most
// kMaxIdRanges ranges; the caller skips the table fill.
constexpr int kPartLdsBytes = 144 * 1024;
constexpr int kMaxIdRanges = 64;
constexpr int kPartTargetGroups = 256;  // one workgroup per CU (the LDS table fills the CU)
inline int64_t topn_part_range(int naggs) { return kPartLdsBytes / (8 * (naggs + 1)); }
// row splits per (segment, id range); each split writes its own [card][1 + naggs] partial table
int topn_part_splits(int64_t max_card, int naggs, int njobs);
void launch_topn_part(const ScanJob* d_jobs, int njobs, int64_t max_card, AggPlan plan, int splits, hipStream_t s);
// topN aggregation by dictionary-id bins of 2^shift ids (radix partition of the rows, then one
// LDS table per bin); see dg_kernels.hip. bin_first[seg] = first global bin of segment seg,
// bin_seg[b] = segment of global bin b; hist/base/cursor: nbins words (hist zeroed by the caller);
// lid/vals: cap selected-row slots (vals is naggs x cap).
// topN bin index of a dimension column (Column::tix_*): bin b's rows are perm[base[b] .. base[b + 1])
// (base has bins + 1 entries), lid = each row's dictionary id & (2^shift - 1)
struct TopnIx {
  const uint32_t* perm;
  const uint16_t* lid;
  const uint32_t* base;
};
constexpr int kTopnIxShift = 8;  // ids per index bin: 256
void launch_topn_ix_build(const ScanJob* d_jobs, int seg, int64_t nrows, int shift, int nbins, uint32_t* d_cnt,
                          uint32_t* d_cursor, uint32_t* base, uint32_t* perm, uint16_t* lid, hipStream_t s);
void launch_topn_ix_reduce(const ScanJob* d_jobs, const TopnIx* d_ix, const int32_t* d_bin_first,
                           const int32_t* d_bin_seg, int nbins, int shift, AggPlan plan, hipStream_t s);
int topn_bin_shift(int naggs);
void launch_topn_bins(const ScanJob* d_jobs, const int32_t* d_tile_job, int ntiles, const int32_t* d_bin_first,
                      const int32_t* d_bin_seg, int nbins, int shift, uint32_t* d_hist, uint32_t* d_base,
                      uint32_t* d_cursor, AggPlan plan, uint16_t* d_lid, uint64_t* d_vals, int64_t cap, hipStream_t s);
// topN selection of one segment: K-th largest metric key (8-bit radix select over all touched ids,
// many workgroups per segment), candidate ids (key >= K-th) in id order, and the candidates'
// records gathered into a compact buffer for one read-back.
struct TopnSelJob {
  const uint64_t* table;  // [card][1 + naggs] accumulator records
  int64_t card;
  uint64_t* state;        // [0] = K-th key, [1] = aggregated rows, [2] = touched ids (zeroed by the host)
  int32_t* cand;          // candidate ids (capacity card)
  int32_t* ncand;
  uint64_t* gathered;     // [gather_cap][2 + naggs]: id, then the record of cand[0 .. gather_cap)
  uint64_t* keys;         // [card] metric keys (0 = untouched)
  uint32_t* hist;         // [8][256] radix histograms (zeroed by the host)
  uint64_t* rstate;       // [9][4] the radix choice after k levels: prefix, mask, keys still to take, done
                          // (k_topn_radix level k writes entry k, so each level replays one histogram)
  int32_t* blkcnt;        // [ceil(card / 1024)] candidates per workgroup
  uint16_t* order;        // [gather_cap] gather positions in builder order (filled when ncand <= 4096)
  int32_t gather_cap;
  // DimensionTopNMetricSpec: key of a touched id = its dictionary rank (smaller first), eligible when
  // lo <= id < hi and rank >= min_rank; rank == nullptr: every id has rank 0 (missing dimension)
  int32_t dim_mode;
  const int32_t* rank;
  int32_t lo, hi;
  int32_t min_rank;
  int32_t pad;
};
constexpr int kSelBlock = 1024;
constexpr int kTopnOrderCap = 4096;  // k_topn_order sorts at most this many candidates
void launch_topn_select(const TopnSelJob* d_jobs, int njobs, int64_t max_card, int naggs, int metric, int metric_op,
                        int inverted, int threshold, hipStream_t s);

constexpr int kTileRows = 2048;

// dg_sort.hip
// radix digits of up to 8 bits (9-bit digits on 4096-element tiles measured slower: 64-byte store runs);
// DG_RS_DIGIT_BITS: A/B builds
#ifndef DG_RS_DIGIT_BITS
#define DG_RS_DIGIT_BITS 8
#endif
constexpr int kMaxDigitBits = DG_RS_DIGIT_BITS;
constexpr int kMaxBins = 1 << kMaxDigitBits;
constexpr int kRsMaxPasses = 8;  // 64 key bits at >= 8 bits per digit (rows of SortBufs::bin_total)
constexpr int kSortTile = 4096;  // elements per radix / run tile (256 threads x 16)
// groupBy reduce: waves per sort tile (each reduces its own 4096 / kRedWaves elements; one carry /
// open slot per wave)
#ifndef DG_RED_WAVES
#define DG_RED_WAVES 16
#endif
constexpr int kRedWaves = DG_RED_WAVES;
constexpr int kMaxCallSegs = 1024;  // segments of one sort-based call (row-ref bases live in LDS)
inline int sort_tiles(int64_t n) { return (int)std::max<int64_t>(1, (n + kSortTile - 1) / kSortTile); }
// selected rows -> (key, element index) in (segment, row) order + their aggregator inputs in
// sb->payload; sb->n[0] = selected rows
// selected rows (groupings of rows with multi-value dimensions) per keygen tile, and their total
void launch_gb_count(const GbJob* d_jobs, const int32_t* d_tile_job, int ntiles, uint32_t* tile_cnt, uint32_t* total,
                     bool multi, hipStream_t s);
// multi-value element count: per-tile counts (0xFFFFFFFF = saturated) and their 64-bit total
void launch_gb_count_total(const GbJob* d_jobs, const int32_t* d_tile_job, int ntiles, uint32_t* tile_cnt,
                           unsigned long long* total, hipStream_t s);
// all_rows >= 0: every row of the call's jobs is an element (no filter bitset, every row's time
// inside the interval, no multi-value dimension) and all_rows is their count: no count pass before
// the keygen
void launch_gb_keygen(const GbJob* d_jobs, const int32_t* d_tile_job, int ntiles, SortBufs* sb, AggPlan plan,
                      hipStream_t s, bool multi = false, int64_t all_rows = -1);
// stable LSD radix sort of sb->keys/refs[cur] on key bits [0, key_bits)
void launch_radix_sort(SortBufs* sb, int key_bits, hipStream_t s);
// run heads of the sorted keys: sb->run_cnt = per-tile offsets, sb->n[1] = runs
void launch_run_heads(SortBufs* sb, hipStream_t s);
// head_pos[g] = first sorted element of run g (after launch_run_heads)
void launch_run_mark(SortBufs* sb, uint32_t* head_pos, hipStream_t s);
// groupBy merge of the sorted rows: one record per run, out_keys[g] and slot s of group g at
// out_slots[s * cap + g] (SoA) in the ABI slot encoding; head_pos (null unless a floatSum needs it)
// = first sorted element of run g; floatSum slots are left to launch_fsum_runs. carry_g / open_g:
// sort_tiles(cap) entries, carry_slots: sort_tiles(cap) * (1 + naggs).
void launch_gb_reduce(SortBufs* sb, AggPlan plan, uint64_t* out_keys, uint64_t* out_slots, int64_t cap,
                      uint32_t* head_pos, int64_t* carry_g, uint64_t* carry_slots, int64_t* open_g, hipStream_t s);
// floatSum aggregator `agg` as the reference computes it: a float32 sum in row order per run and
// segment (FloatSumBufferAggregator.aggregate), segments combined in order with float adds
// (FloatSumAggregator.combine). groupBy: into out_slots[(1 + agg) * cap + g]; per-segment engines
// (out_slots == null): into the job's fs_out table.
void launch_fsum_runs(const GbJob* d_jobs, int njobs, int ntiles, SortBufs* sb, AggPlan plan, int agg,
                      const uint32_t* head_pos, uint64_t* out_slots, int64_t cap, hipStream_t s, int desc = 0);
// device slot encoding -> ABI encoding (finalize) of the aggregator slots [1 + a][cap] of n_ptr[0] groups
void launch_slots_finalize(uint64_t* slots, const uint32_t* n_ptr, int64_t cap, AggPlan plan, hipStream_t s);
// SoA slots [rec][cap] -> AoS records [n][rec]
void launch_soa_to_aos(const uint64_t* soa, int64_t cap, int64_t n, int rec, uint64_t* aos, hipStream_t s);
// a result laid out for `cap` records compacted to its n groups: keys [n], slots [rec][n] (16-byte copies)
void launch_result_compact(const uint64_t* keys, const uint64_t* slots, int64_t cap, int64_t n, int rec, uint64_t* keys2,
                           uint64_t* slots2, hipStream_t s);
// groups [start, start + count): key fields -> bucket index and merged ids (int32 per dimension)
struct KeyLayout {
  int32_t ndims;
  int32_t bucket_shift, bucket_bits;
  int32_t dim_shift[kMaxGroupDims];
  int32_t dim_bits[kMaxGroupDims];
};
void launch_gb_unpack(const uint64_t* keys, int64_t start, int64_t count, KeyLayout lay, int64_t* bucket, int32_t* ids,
                      hipStream_t s);
// groups [start, start + count) packed for one device-to-host copy: times, ids, AoS values (see dg_sort.hip)
void launch_gb_fetch_pack(const uint64_t* keys, const uint64_t* slots, int64_t cap, int64_t start, int64_t count,
                          KeyLayout lay, int naggs, int64_t universal, int64_t bucket0, int64_t period,
                          const int64_t* bounds, int64_t* times, int32_t* ids, uint64_t* vals, hipStream_t s);
// cross-device merge: keys of layout lin -> layout lout (bucket index + bucket_delta, ids through maps)
struct RekeyMaps {
  const int32_t* m[kMaxGroupDims];
};
void launch_gb_rekey(const uint64_t* in, int64_t n, KeyLayout lin, KeyLayout lout, int64_t bucket_delta,
                     RekeyMaps maps, uint64_t* out, hipStream_t s);
void launch_lower_bound(const uint64_t* keys, int64_t n, const uint64_t* split, int nsplit, int64_t* pos, hipStream_t s);
// sort input of a merge (refs = record index, sb->n[0] = n)
void launch_merge_load(const uint64_t* keys, int64_t n, SortBufs* sb, hipStream_t s);
// limit push-down: key fields (bucket, dimensions) re-packed most significant first in the push-down
// order; a field's value goes through its rank table (if any) and is complemented when descending
struct LimitOrder {
  int32_t nfields;
  int32_t in_shift[kMaxGroupDims + 1];
  int32_t bits[kMaxGroupDims + 1];
  int32_t out_shift[kMaxGroupDims + 1];
  int32_t desc[kMaxGroupDims + 1];
  const int32_t* rank[kMaxGroupDims + 1];
};
void launch_limit_load(const uint64_t* keys, int64_t n, const LimitOrder& o, SortBufs* sb, hipStream_t s);
// the first m elements of the sorted order: keys[ref] and the [rec][cap] slot-major records -> [rec][ocap]
void launch_limit_gather(const SortBufs* sb, int64_t m, const uint64_t* keys, const uint64_t* slots, int64_t cap,
                         int rec, uint64_t* okeys, uint64_t* oslots, int64_t ocap, hipStream_t s);
// one record per run of the sorted merge input, partial values combined in order (device encoding,
// SoA slots [rec][cap])
void launch_merge_reduce(SortBufs* sb, const uint32_t* head_pos, const uint64_t* in_slots, AggPlan plan, int64_t cap,
                         uint64_t* out_keys, uint64_t* out_slots, hipStream_t s);

}  // namespace dg
