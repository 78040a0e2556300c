"""Druid v9 segment writer (the build's IndexMergerV9 for synthetic and fixture data).

Writes a segment directory that the reference's ``IndexIO.V9IndexLoader.load``
(processing/.../segment/IndexIO.java:569-663) would map, byte layout per column:

* smoosh container: ``version.bin`` (int 9, big-endian), ``meta.smoosh`` and
  ``00000.smoosh`` (java-util/.../io/smoosh/FileSmoosher.java, SmooshedFileMapper.java).
* ``index.drd``: GenericIndexed<String> columns, GenericIndexed<String> dimensions,
  interval (2 x int64 BE), bitmap serde JSON (IndexIO.java:584-610).
* every column: int32 BE length + ColumnDescriptor JSON, then its part
  (IndexIO.java:665-672).
* GenericIndexed v1 (processing/.../segment/data/GenericIndexed.java:52-77,479-492):
  ``[0x01][sorted][int32 numBytesUsed][int32 n][n x int32 end offsets][(int32 marker)(bytes)...]``.
* string columns: DictionaryEncodedColumnPartSerde COMPRESSED (version 2) + flags
  (serde/DictionaryEncodedColumnPartSerde.java:283-345), ids via
  CompressedVSizeColumnarIntsSerializer (data/CompressedVSizeColumnarIntsSerializer.java:47-62,
  chunk sizing data/CompressedVSizeColumnarIntsSupplier.java:82-101), one Concise or Roaring bitmap
  per dictionary value.
* long/float/double columns: BlockLayoutColumnar{Longs,Floats,Doubles}Serializer with LONGS
  encoding (data/BlockLayoutColumnarLongsSerializer.java:60-66, 8192 longs or 16384 floats per
  64 KiB block), LZ4 (id 0x01), UNCOMPRESSED blocks (0xFF) or NONE (0xFE, EntireLayout).

LZ4 blocks are produced with the system ``liblz4.so.1`` (HC level 9 by default, like
lz4-java's ``highCompressor``; "fast" for large synthetic data). Byte order inside blocks is
little-endian (IndexIO.BYTE_ORDER = nativeOrder, IndexIO.java:90).
"""
from __future__ import annotations

import ctypes
import json
import os
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _tools

BUFFER_SIZE = 65536  # CompressedPools.BUFFER_SIZE (segment/CompressedPools.java:39)

COMPRESSION_IDS = {"lzf": 0x00, "lz4": 0x01, "uncompressed": 0xFF, "none": 0xFE}

MIN_INSTANT = -(2 ** 62)  # JodaUtils.MIN_INSTANT = Long.MIN_VALUE / 2


# --------------------------------------------------------------------------------------------
# LZ4 (system liblz4; the decoder used by queries is the build's own HIP kernel)
# --------------------------------------------------------------------------------------------
_lz4 = None


def _lz4lib():
    global _lz4
    if _lz4 is None:
        lib = ctypes.CDLL("liblz4.so.1")
        lib.LZ4_compressBound.restype = ctypes.c_int
        lib.LZ4_compressBound.argtypes = [ctypes.c_int]
        lib.LZ4_compress_HC.restype = ctypes.c_int
        lib.LZ4_compress_HC.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        lib.LZ4_compress_default.restype = ctypes.c_int
        lib.LZ4_compress_default.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        _lz4 = lib
    return _lz4


def lz4_compress(data: bytes, mode: str = "hc") -> bytes:
    lib = _lz4lib()
    bound = lib.LZ4_compressBound(len(data))
    out = ctypes.create_string_buffer(bound)
    if mode == "hc":
        n = lib.LZ4_compress_HC(data, out, len(data), bound, 9)
    else:
        n = lib.LZ4_compress_default(data, out, len(data), bound)
    if n <= 0:
        raise RuntimeError("LZ4 compression failed")
    return out.raw[:n]


# --------------------------------------------------------------------------------------------
# GenericIndexed v1
# --------------------------------------------------------------------------------------------
def generic_indexed(values: Sequence[Optional[bytes]], sorted_flag: bool) -> bytes:
    """Serialize a GenericIndexed v1 (GenericIndexed.java:52-77; writer GenericIndexedWriter)."""
    n = len(values)
    ends = np.empty(n, dtype=">i4")
    parts = []
    pos = 0
    for i, v in enumerate(values):
        if v is None:
            parts.append(struct.pack(">i", -1))
            pos += 4
        else:
            parts.append(struct.pack(">i", len(v)))
            parts.append(v)
            pos += 4 + len(v)
        ends[i] = pos
    body = struct.pack(">i", n) + ends.tobytes() + b"".join(parts)
    return bytes([0x01, 0x01 if sorted_flag else 0x00]) + struct.pack(">i", len(body)) + body


def _blocks_generic_indexed(blocks: List[bytes]) -> bytes:
    return generic_indexed(blocks, sorted_flag=False)


# --------------------------------------------------------------------------------------------
# Dictionary ordering (GenericIndexed.STRING_STRATEGY: Comparators.naturalNullsFirst over
# java.lang.String.compareTo, i.e. UTF-16 code-unit order)
# --------------------------------------------------------------------------------------------
def java_string_key(s: str) -> bytes:
    return s.encode("utf-16-be", "surrogatepass")


def num_bytes_for_max(max_value: int) -> int:
    """VSizeColumnarInts.getNumBytesForMax (data/VSizeColumnarInts.java:84-99)."""
    if max_value <= 0xFF:
        return 1
    if max_value <= 0xFFFF:
        return 2
    if max_value <= 0xFFFFFF:
        return 3
    return 4


def max_ints_in_buffer_for_bytes(num_bytes: int) -> int:
    """CompressedVSizeColumnarIntsSupplier.maxIntsInBufferForBytes (:82-101)."""
    padding = 0 if num_bytes in (1, 2) else 4 - num_bytes
    max_size_per = (BUFFER_SIZE - padding) // num_bytes
    return 1 << (max_size_per.bit_length() - 1)


# --------------------------------------------------------------------------------------------
# Column part serializers
# --------------------------------------------------------------------------------------------
def _compress_blocks(raw: bytes, block_bytes: int, compression: str, lz4_mode: str) -> List[bytes]:
    blocks = []
    for off in range(0, len(raw), block_bytes):
        chunk = raw[off:off + block_bytes]
        if compression == "lz4":
            blocks.append(lz4_compress(chunk, lz4_mode))
        elif compression == "lzf":
            blocks.append(_tools.lzf_compress(chunk))
        elif compression == "uncompressed":
            blocks.append(chunk)
        else:
            raise ValueError(f"unsupported block compression {compression}")
    return blocks


VSIZE_SUPPORTED = (1, 2, 4, 8, 12, 16, 20, 24, 32, 40, 48, 56, 64)
MAX_TABLE_SIZE = 256  # CompressionFactory.MAX_TABLE_SIZE (data/CompressionFactory.java:85)
_I64_MAX = 2 ** 63 - 1


def bits_for_max(value: int) -> int:
    """VSizeLongSerde.getBitsForMax (data/VSizeLongSerde.java:41-59)."""
    if value < 0:
        raise ValueError(f"maxValue[{value}] must be positive")
    nbits, max_value = 0, 1
    for size in VSIZE_SUPPORTED:
        while nbits < size and max_value < _I64_MAX // 2:
            nbits += 1
            max_value *= 2
        if value <= max_value or max_value >= _I64_MAX // 2:
            return size
    return 64


def vsize_serialized_size(bits: int, n: int) -> int:
    """VSizeLongSerde.getSerializedSize (:61-65): packed bytes rounded up + 4 closing bytes."""
    return (bits * n + 7) // 8 + 4


def vsize_values_per_block(bits: int, block_bytes: int = BUFFER_SIZE) -> int:
    """VSizeLongSerde.getNumValuesPerBlock (:70-77)."""
    ret = 1
    while vsize_serialized_size(bits, ret) <= block_bytes:
        ret *= 2
    return ret // 2


def vsize_pack(values: np.ndarray, bits: int) -> bytes:
    """VSizeLongSerde serializers (Size1Ser, Size2Ser, Mult4Ser, Mult8Ser, :190-414): values written
    MSB-first as one big-endian bit stream, the last partial byte zero-filled, then 4 zero bytes."""
    v = np.ascontiguousarray(values, dtype=np.uint64)
    if bits % 8 == 0:
        nb = bits // 8
        body = v.astype(">u8").view(np.uint8).reshape(-1, 8)[:, 8 - nb:].tobytes()
    else:
        shifts = np.arange(bits - 1, -1, -1, dtype=np.uint64)
        bitmat = ((v[:, None] >> shifts[None, :]) & np.uint64(1)).astype(np.uint8)
        body = np.packbits(bitmat.reshape(-1)).tobytes()
    return body + bytes(4)


def choose_long_encoding(values: np.ndarray):
    """IntermediateColumnarLongsSerializer.makeDelegate (:103-124) for longEncoding=auto: TABLE when at
    most 256 distinct values (table in first-appearance order), DELTA when max - min does not overflow
    and is not Long.MAX_VALUE, LONGS otherwise. Returns (format, meta) with meta the ids/offsets."""
    v = np.asarray(values, dtype=np.int64)
    uniq, first = np.unique(v, return_index=True)
    if len(uniq) <= MAX_TABLE_SIZE:
        order = np.argsort(first, kind="stable")
        table = uniq[order]
        rank = np.empty(len(uniq), dtype=np.int64)
        rank[order] = np.arange(len(uniq))
        ids = rank[np.searchsorted(uniq, v)] if len(v) else np.zeros(0, dtype=np.int64)
        return "table", (table, ids.astype(np.uint64), bits_for_max(len(table)))
    lo, hi = int(v.min()), int(v.max())
    delta = hi - lo
    if delta <= _I64_MAX and delta != _I64_MAX:
        offsets = (v.astype(np.uint64) - np.uint64(lo & 0xFFFFFFFFFFFFFFFF))
        return "delta", (lo, offsets, bits_for_max(delta + 1))
    return "longs", None


def packed_long_column_part(values: np.ndarray, compression: str, lz4_mode: str, fmt: str, meta) -> bytes:
    """BlockLayout / EntireLayout long column with a DELTA or TABLE LongEncodingWriter:
    [0x02][i32 total][i32 sizePer][cid - 126 (encoding flag)][format id][encoding meta][blocks]
    (BlockLayoutColumnarLongsSerializer.java:37-41,60-66; DeltaLongEncodingWriter.putMeta :59-66;
    TableLongEncodingWriter.putMeta :77-86). Every block restarts the packed stream."""
    n = len(values)
    if fmt == "delta":
        base, packed, bits = meta
        enc = bytes([0x00, 0x01]) + struct.pack(">qi", base, bits)
    else:
        table, packed, bits = meta
        enc = bytes([0x01, 0x01]) + struct.pack(">i", len(table)) + np.asarray(table, dtype=">i8").tobytes()
    cid = COMPRESSION_IDS[compression]
    flagged = ((cid - 256 if cid > 127 else cid) - 126) & 0xFF  # CompressionFactory.setEncodingFlag
    if compression == "none":  # EntireLayoutColumnarLongsSerializer writes sizePer 0 (:35-39)
        return struct.pack(">Bii", 0x02, n, 0) + bytes([flagged]) + enc + vsize_pack(packed, bits)
    size_per = vsize_values_per_block(bits)
    blocks = []
    for off in range(0, n, size_per):
        chunk = vsize_pack(packed[off:off + size_per], bits)
        if compression == "lz4":
            blocks.append(lz4_compress(chunk, lz4_mode))
        elif compression == "lzf":
            blocks.append(_tools.lzf_compress(chunk))
        elif compression == "uncompressed":
            blocks.append(chunk)
        else:
            raise ValueError(f"unsupported block compression {compression}")
    return struct.pack(">Bii", 0x02, n, size_per) + bytes([flagged]) + enc + _blocks_generic_indexed(blocks)


def numeric_column_part(values: np.ndarray, kind: str, compression: str, lz4_mode: str,
                        long_encoding: str = "longs") -> bytes:
    """CompressedColumnar{Longs,Floats,Doubles}Supplier layout, LONGS encoding (legacy, no flag), or
    for longs with long_encoding="auto" the format IntermediateColumnarLongsSerializer picks."""
    if kind == "long" and long_encoding == "auto" and len(values):
        fmt, meta = choose_long_encoding(values)
        if fmt != "longs":
            return packed_long_column_part(np.asarray(values, dtype=np.int64), compression, lz4_mode, fmt, meta)
    elif long_encoding not in ("longs", "auto"):
        raise ValueError(f"unknown long encoding {long_encoding}")
    dtype = {"long": "<i8", "double": "<f8", "float": "<f4"}[kind]
    arr = np.ascontiguousarray(values, dtype=dtype)
    width = arr.dtype.itemsize
    size_per = BUFFER_SIZE // width  # 8192 longs/doubles, 16384 floats
    if compression == "lzf_v1":
        # LZF_VERSION (0x01) columns of older segments: no compression byte, LZF blocks
        # (CompressedColumnarLongsSupplier.fromByteBuffer, :102-116)
        return struct.pack(">Bii", 0x01, len(arr), size_per) + \
            _blocks_generic_indexed(_compress_blocks(arr.tobytes(), size_per * width, "lzf", lz4_mode))
    cid = COMPRESSION_IDS[compression]
    header = struct.pack(">Bii", 0x02, len(arr), size_per) + bytes([cid])
    raw = arr.tobytes()
    if compression == "none":
        # EntireLayoutColumnar{Longs,...}: values follow directly (CompressionFactory.getLongSupplier)
        return header + raw
    return header + _blocks_generic_indexed(_compress_blocks(raw, size_per * width, compression, lz4_mode))


def ids_part(ids: np.ndarray, cardinality: int, compression: str, lz4_mode: str, num_bytes: Optional[int] = None) -> bytes:
    """CompressedVSizeColumnarIntsSerializer (little-endian values, numBytes from cardinality; num_bytes
    forces a wider id, e.g. the 4-byte form CompressedVSizeColumnarIntsSupplier reads as full ints)."""
    nb = num_bytes or num_bytes_for_max(cardinality)
    size_per = max_ints_in_buffer_for_bytes(nb)
    ids32 = np.ascontiguousarray(ids, dtype="<u4")
    if nb == 4:
        raw = ids32.tobytes()
    else:
        raw = ids32.view(np.uint8).reshape(-1, 4)[:, :nb].tobytes()
    cid = COMPRESSION_IDS["uncompressed" if compression == "none" else compression]
    header = struct.pack(">BBii", 0x02, nb, len(ids32), size_per) + bytes([cid])
    comp = "uncompressed" if compression == "none" else compression
    return header + _blocks_generic_indexed(_compress_blocks(raw, size_per * nb, comp, lz4_mode))


def vsize_ids_part(ids: np.ndarray, cardinality: int, num_bytes: Optional[int] = None) -> bytes:
    """VSizeColumnarIntsSerializer (data/VSizeColumnarIntsSerializer.java:40-96): header
    [0x00][numBytes][i32 size], then each id as its low numBytes bytes big-endian, then
    4 - numBytes zero bytes so the reader's getInt never runs off the end."""
    nb = num_bytes or num_bytes_for_max(cardinality)
    be = np.ascontiguousarray(ids, dtype=">u4").view(np.uint8).reshape(-1, 4)[:, 4 - nb:].tobytes()
    payload = be + bytes(4 - nb)
    return struct.pack(">BBi", 0x00, nb, len(payload)) + payload


def concise_bitmaps(ids: np.ndarray, cardinality: int) -> List[bytes]:
    words, counts = _tools.concise_encode_column(ids, cardinality)
    out = []
    pos = 0
    be = words.astype(">i4")
    for c in counts:
        out.append(be[pos:pos + c].tobytes())
        pos += c
    return out


def roaring_serialize(rows: np.ndarray, run_optimize: bool = True) -> bytes:
    """Portable Roaring format (RoaringFormatSpec; RoaringBitmap 0.5.18 ``serialize``)."""
    rows = np.asarray(rows, dtype=np.int64)
    if len(rows) == 0:
        return struct.pack("<II", 12346, 0)
    keys = (rows >> 16).astype(np.int64)
    uk, starts = np.unique(keys, return_index=True)
    ends = np.append(starts[1:], len(rows))
    containers = []  # (key, card, kind, payload)
    for k, s, e in zip(uk, starts, ends):
        lows = (rows[s:e] & 0xFFFF).astype(np.uint16)
        card = e - s
        # run detection
        brk = np.nonzero(np.diff(lows.astype(np.int32)) != 1)[0]
        n_runs = len(brk) + 1
        run_bytes = 2 + 4 * n_runs
        arr_bytes = 2 * card if card <= 4096 else 1 << 30
        bmp_bytes = 8192
        if run_optimize and run_bytes < min(arr_bytes, bmp_bytes):
            rs = np.concatenate([[0], brk + 1])
            re_ = np.concatenate([brk, [card - 1]])
            starts_v = lows[rs].astype(np.uint16)
            lens_v = (lows[re_].astype(np.int32) - lows[rs].astype(np.int32)).astype(np.uint16)
            payload = struct.pack("<H", n_runs) + np.stack([starts_v, lens_v], axis=1).astype("<u2").tobytes()
            containers.append((int(k), card, "run", payload))
        elif card <= 4096:
            containers.append((int(k), card, "array", lows.astype("<u2").tobytes()))
        else:
            bits = np.zeros(65536, dtype=np.uint8)
            bits[lows] = 1
            containers.append((int(k), card, "bitmap", np.packbits(bits, bitorder="little").tobytes()))
    size = len(containers)
    has_run = any(c[2] == "run" for c in containers)
    out = bytearray()
    if has_run:
        out += struct.pack("<I", 12347 | ((size - 1) << 16))
        runbits = np.zeros(((size + 7) // 8) * 8, dtype=np.uint8)
        for i, c in enumerate(containers):
            if c[2] == "run":
                runbits[i] = 1
        out += np.packbits(runbits, bitorder="little").tobytes()
    else:
        out += struct.pack("<II", 12346, size)
    for k, card, _, _ in containers:
        out += struct.pack("<HH", k, card - 1)
    if (not has_run) or size >= 4:
        offset = len(out) + 4 * size
        for c in containers:
            out += struct.pack("<I", offset)
            offset += len(c[3])
    for c in containers:
        out += c[3]
    return bytes(out)


def roaring_bitmaps(ids: np.ndarray, cardinality: int) -> List[bytes]:
    order = np.argsort(ids, kind="stable")
    sorted_ids = ids[order]
    bounds = np.searchsorted(sorted_ids, np.arange(cardinality + 1))
    return [roaring_serialize(np.sort(order[bounds[v]:bounds[v + 1]])) for v in range(cardinality)]


def string_column_part(dictionary: List[Optional[str]], ids: np.ndarray, bitmap: str,
                       compression: str, lz4_mode: str, num_bytes: Optional[int] = None) -> bytes:
    card = len(dictionary)
    dict_vals = [None if (v is None or v == "") else v.encode("utf-8") for v in dictionary]
    # null / "" are both stored as a zero-length value (NullHandling.replaceWithDefault)
    dict_vals = [b"" if v is None else v for v in dict_vals]
    if compression == "uncompressed":
        # IndexSpec dimensionCompression UNCOMPRESSED: VSizeColumnarIntsSerializer, part version
        # UNCOMPRESSED_SINGLE_VALUE without flags (StringDimensionMergerV9.java:217-225,
        # DictionaryEncodedColumnPartSerde.java:191-217)
        out = bytes([0x00])
        out += generic_indexed(dict_vals, sorted_flag=True)
        out += vsize_ids_part(ids, card, num_bytes)
    else:
        out = bytes([0x02]) + struct.pack(">i", 0)  # COMPRESSED, flags = 0 (single-value, bitmaps)
        out += generic_indexed(dict_vals, sorted_flag=True)
        out += ids_part(ids, card, compression, lz4_mode, num_bytes)
    if bitmap == "concise":
        bms = concise_bitmaps(ids, card)
    else:
        bms = roaring_bitmaps(ids, card)
    out += generic_indexed(bms, sorted_flag=False)
    return out


def encode_multi_strings(rows: Sequence[Sequence[Optional[str]]]) -> Tuple[List[str], List[np.ndarray]]:
    """Multi-value rows -> (sorted dictionary, per-row sorted id arrays). MultiValueHandling
    SORTED_ARRAY (the default: values sorted, duplicates kept); an empty row is stored as [null]
    (StringDimensionIndexer / DictionaryEncodedColumnMerger), "" and null are the same value."""
    norm = [sorted(("" if v is None else str(v)) for v in r) or [""] for r in rows]
    uniq = sorted({v for r in norm for v in r}, key=java_string_key)
    index = {v: i for i, v in enumerate(uniq)}
    return uniq, [np.array(sorted(index[v] for v in r), dtype=np.int32) for r in norm]


def multi_string_column_part(dictionary: List[Optional[str]], rows: Sequence[np.ndarray], bitmap: str,
                             compression: str, lz4_mode: str, legacy: bool = False) -> bytes:
    """Multi-value dictionary-encoded column (DictionaryEncodedColumnPartSerde.java:183-217):
    compressed = version COMPRESSED + MULTI_VALUE_V3 flag, ids as V3CompressedVSizeColumnarMultiInts
    ([0x03][CompressedColumnarInts row start offsets + end][CompressedVSizeColumnarInts values],
    V3CompressedVSizeColumnarMultiIntsSerializer.java:87-120); uncompressed = version
    UNCOMPRESSED_MULTI_VALUE with VSizeColumnarMultiInts ([0x01][numBytes][i32 size][i32 count]
    [count end byte offsets][big-endian values][4 - numBytes pad], VSizeColumnarMultiInts.fromIterable).
    Value v's bitmap holds every row whose list contains v (and the null value's, rows with no value)."""
    card = len(dictionary)
    dict_vals = [b"" if (v is None or v == "") else v.encode("utf-8") for v in dictionary]
    nb = num_bytes_for_max(card)
    lens = np.array([len(r) for r in rows], dtype=np.int64)
    flat = np.concatenate([np.asarray(r, dtype=np.int32) for r in rows]) if len(rows) else np.zeros(0, np.int32)
    if legacy:  # blocks of the column's compression (NONE has no block form: UNCOMPRESSED blocks)
        bc = "uncompressed" if compression == "none" else compression
        out = bytes([0x02]) + struct.pack(">i", 0x1) + generic_indexed(dict_vals, sorted_flag=True)
        offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        total = int(offsets[-1])
        out += bytes([0x02]) + ids_part(offsets, total, bc, lz4_mode) + ids_part(flat, card, bc, lz4_mode)
    elif compression in ("uncompressed", "none"):
        out = bytes([0x01]) + generic_indexed(dict_vals, sorted_flag=True)
        ends = np.cumsum(lens * nb).astype(">i4")
        values = np.ascontiguousarray(flat, dtype=">u4").view(np.uint8).reshape(-1, 4)[:, 4 - nb:].tobytes()
        payload = struct.pack(">i", len(rows)) + ends.tobytes() + values + bytes(4 - nb)
        out += struct.pack(">BBi", 0x01, nb, len(payload)) + payload
    else:
        out = bytes([0x02]) + struct.pack(">i", 0x2) + generic_indexed(dict_vals, sorted_flag=True)
        offsets = np.concatenate([[0], np.cumsum(lens)]).astype("<i4")
        size_per = BUFFER_SIZE // 4  # CompressedColumnarIntsSupplier.MAX_INTS_IN_BUFFER
        cid = COMPRESSION_IDS[compression]
        out += bytes([0x03]) + struct.pack(">Bii", 0x02, len(offsets), size_per) + bytes([cid])
        out += _blocks_generic_indexed(_compress_blocks(offsets.tobytes(), size_per * 4, compression, lz4_mode))
        out += ids_part(flat, card, compression, lz4_mode)
    row_of = np.repeat(np.arange(len(rows), dtype=np.int64), lens)
    order = np.lexsort((row_of, flat))
    sf, sr = flat[order], row_of[order]
    bounds = np.searchsorted(sf, np.arange(card + 1))
    bms = []
    # StringDimensionMergerV9.processMergedRow / :483: rows without values join the null value's
    # bitmap when null is the dictionary's first value
    empty_rows = np.nonzero(lens == 0)[0] if card and dictionary[0] in (None, "") else np.zeros(0, np.int64)
    for v in range(card):
        rws = np.unique(sr[bounds[v]:bounds[v + 1]])
        if v == 0 and len(empty_rows):
            rws = np.union1d(rws, empty_rows)
        if bitmap == "concise":
            bms.append(_tools.concise_encode(rws).astype(">i4").tobytes())
        else:
            bms.append(roaring_serialize(rws))
    return out + generic_indexed(bms, sorted_flag=False)


def _bitmap_json(bitmap: str) -> dict:
    if bitmap == "concise":
        return {"type": "concise"}
    return {"type": "roaring", "compressRunOnSerialization": True}


def _descriptor(value_type: str, part: dict, multi: bool = False) -> bytes:
    js = json.dumps({"valueType": value_type, "hasMultipleValues": multi, "parts": [part]},
                    separators=(",", ":")).encode()
    return struct.pack(">i", len(js)) + js


# --------------------------------------------------------------------------------------------
# Dimension encoding helpers
# --------------------------------------------------------------------------------------------
def encode_strings(values: Sequence[Optional[str]]) -> Tuple[List[str], np.ndarray]:
    """Build a sorted dictionary (nulls first) and per-row ids from python strings."""
    norm = ["" if v is None else str(v) for v in values]
    uniq = sorted(set(norm), key=java_string_key)
    index = {v: i for i, v in enumerate(uniq)}
    ids = np.fromiter((index[v] for v in norm), dtype=np.int32, count=len(norm))
    return uniq, ids


def encode_int_strings(values: np.ndarray, null_mask: Optional[np.ndarray] = None) -> Tuple[List[str], np.ndarray]:
    """Fast path for integer-valued string dims: dictionary = sorted(str(v)), ids by table lookup."""
    values = np.asarray(values, dtype=np.int64)
    present = np.unique(values if null_mask is None else values[~null_mask])
    strs = [str(int(v)) for v in present]
    has_null = null_mask is not None and bool(null_mask.any())
    order = sorted(range(len(strs)), key=lambda i: java_string_key(strs[i]))
    dictionary = ([""] if has_null else []) + [strs[i] for i in order]
    rank = np.empty(len(strs), dtype=np.int32)
    rank[np.asarray(order, dtype=np.int64)] = np.arange(len(strs), dtype=np.int32) + (1 if has_null else 0)
    pos = np.searchsorted(present, values)
    pos = np.clip(pos, 0, max(len(present) - 1, 0))
    ids = rank[pos] if len(present) else np.zeros(len(values), dtype=np.int32)
    if has_null:
        ids = np.where(null_mask, 0, ids).astype(np.int32)
    return dictionary, ids.astype(np.int32)


@dataclass
class SegmentSpec:
    timestamps: np.ndarray
    dims: Dict[str, Tuple[List[str], np.ndarray]] = field(default_factory=dict)
    metrics: Dict[str, Tuple[str, np.ndarray]] = field(default_factory=dict)
    interval: Optional[Tuple[int, int]] = None


def write_segment(out_dir: str, spec: SegmentSpec, bitmap: str = "concise", compression: str = "lz4",
                  dim_compression: Optional[str] = None, lz4_mode: str = "hc", long_encoding: str = "longs",
                  id_bytes: Optional[int] = None, legacy_multi_value: bool = False, check_sorted: bool = True) -> str:
    """Write a v9 segment directory. Rows must already be in segment order (time-sorted).
    long_encoding: IndexSpec.longEncoding, "longs" (default) or "auto" (DELTA / TABLE / LONGS per column,
    __time included: IndexMergerV9 serializes it with the same long encoding).
    id_bytes: width of single-value dictionary ids (default: numBytes for the cardinality).
    legacy_multi_value: compressed multi-value dimensions in the pre-V3 CompressedVSizeColumnarMultiInts form.
    check_sorted=False: write rows out of time order (robustness tests of the engine only; IndexMergerV9
    never writes such a segment)."""
    os.makedirs(out_dir, exist_ok=True)
    n = len(spec.timestamps)
    ts = np.asarray(spec.timestamps, dtype=np.int64)
    if check_sorted and n and np.any(np.diff(ts) < 0):
        raise ValueError("segment rows must be sorted by __time")
    dim_comp = dim_compression or ("uncompressed" if compression == "none" else
                                   "lzf" if compression == "lzf_v1" else compression)
    files: Dict[str, bytes] = {}
    files["__time"] = _descriptor("LONG", {"type": "long", "byteOrder": "LITTLE_ENDIAN"}) + \
        numeric_column_part(ts, "long", compression, lz4_mode, long_encoding)
    for name, (dictionary, ids) in spec.dims.items():
        if isinstance(ids, list) and ids and isinstance(ids[0], (list, tuple, np.ndarray)):
            if len(ids) != n:
                raise ValueError(f"dimension {name} has {len(ids)} rows, expected {n}")
            part = {"type": "stringDictionary", "bitmapSerdeFactory": _bitmap_json(bitmap),
                    "byteOrder": "LITTLE_ENDIAN"}
            files[name] = _descriptor("STRING", part, multi=True) + multi_string_column_part(
                dictionary, [np.asarray(r, dtype=np.int32) for r in ids], bitmap, dim_comp, lz4_mode, legacy_multi_value)
            continue
        ids = np.asarray(ids, dtype=np.int32)
        if len(ids) != n:
            raise ValueError(f"dimension {name} has {len(ids)} rows, expected {n}")
        part = {"type": "stringDictionary", "bitmapSerdeFactory": _bitmap_json(bitmap), "byteOrder": "LITTLE_ENDIAN"}
        files[name] = _descriptor("STRING", part) + string_column_part(dictionary, ids, bitmap, dim_comp, lz4_mode,
                                                                       id_bytes)
    for name, (kind, vals) in spec.metrics.items():
        vals = np.asarray(vals)
        if len(vals) != n:
            raise ValueError(f"metric {name} has {len(vals)} rows, expected {n}")
        vt = {"long": "LONG", "double": "DOUBLE", "float": "FLOAT"}[kind]
        files[name] = _descriptor(vt, {"type": kind, "byteOrder": "LITTLE_ENDIAN"}) + \
            numeric_column_part(vals, kind, compression, lz4_mode, long_encoding)
    dims = list(spec.dims.keys())
    cols = dims + list(spec.metrics.keys())
    if spec.interval is not None:
        istart, iend = spec.interval
    else:
        istart = int(ts[0]) if n else 0
        iend = int(ts[-1]) + 1 if n else 1
    bm_json = json.dumps(_bitmap_json(bitmap), separators=(",", ":")).encode()
    files["index.drd"] = (generic_indexed([c.encode() for c in cols], sorted_flag=False)
                          + generic_indexed([d.encode() for d in dims], sorted_flag=False)
                          + struct.pack(">qq", istart, iend)
                          + struct.pack(">i", len(bm_json)) + bm_json)
    files["metadata.drd"] = json.dumps({"container": {}, "aggregators": None, "timestampSpec": None,
                                        "queryGranularity": {"type": "none"}, "rollup": False}).encode()
    _write_smoosh(out_dir, files)
    with open(os.path.join(out_dir, "version.bin"), "wb") as f:
        f.write(struct.pack(">i", 9))
    return out_dir


def _write_smoosh(out_dir: str, files: Dict[str, bytes], max_chunk: int = 2 ** 31 - 1) -> None:
    """FileSmoosher layout: numbered chunk files + meta.smoosh 'name,chunk,start,end' lines."""
    names = sorted(files.keys())
    chunks: List[List[Tuple[str, bytes]]] = [[]]
    size = 0
    for nm in names:
        b = files[nm]
        if size + len(b) > max_chunk and chunks[-1]:
            chunks.append([])
            size = 0
        chunks[-1].append((nm, b))
        size += len(b)
    lines = [f"v1,{max_chunk},{len(chunks)}"]
    for ci, chunk in enumerate(chunks):
        pos = 0
        with open(os.path.join(out_dir, f"{ci:05d}.smoosh"), "wb") as f:
            for nm, b in chunk:
                f.write(b)
                lines.append(f"{nm},{ci},{pos},{pos + len(b)}")
                pos += len(b)
    with open(os.path.join(out_dir, "meta.smoosh"), "w") as f:
        f.write("\n".join(lines) + "\n")
