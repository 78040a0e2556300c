"""Adds the long-column round-trip vectors of CompressedLongsSerdeTest to tests/golden/kats.json
("compressed_longs_serde"): processing/src/test/java/org/apache/druid/segment/data/
CompressedLongsSerdeTest.java:65-76 (values0..values8), :79-87 (addUniques: 0..255 first, the
vector at offset 256, so the auto strategy cannot pick TABLE) and :106-115 (testChunkSerde: 0..9999).
Every vector must read back exactly for each long encoding (LONGS, AUTO) and compression strategy.

    python tests/golden/make_serde_kats.py
"""
import json
import os

MAX = (1 << 63) - 1
MIN = -(1 << 63)
VECTORS = [
    [],
    [0, 1, 1, 0, 1, 1, 1, 1, 0, 0, 1, 1],
    [12, 5, 2, 9, 3, 2, 5, 1, 0, 6, 13, 10, 15],
    [1, 1, 1, 1, 1, 11, 11, 11, 11],
    [200, 200, 200, 401, 200, 301, 200, 200, 200, 404, 200, 200, 200, 200],
    [123, 632, 12, 39, 536, 0, 1023, 52, 777, 526, 214, 562, 823, 346],
    [1000000, 1000001, 1000002, 1000003, 1000004, 1000005, 1000006, 1000007, 1000008],
    [MAX, MIN, 12378, -12718243, -1236213, 12743153, 21364375452, 65487435436632, -43734526234564],
    [MAX, 0, 321, 15248425, 13523212136, 63822, 3426, 96],
]


def main():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")
    with open(path) as f:
        kats = json.load(f)
    kats["compressed_longs_serde"] = {
        "_source": "processing/src/test/java/org/apache/druid/segment/data/CompressedLongsSerdeTest.java:65-87,106-115",
        "vectors": VECTORS, "add_uniques_table_size": 256, "chunk": 10000}
    with open(path, "w") as f:
        json.dump(kats, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
