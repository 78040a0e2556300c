"""Adds the filter known-answer tests to tests/golden/kats.json ("filter_kats").

Transcribed by hand from the reference's filter tests (replaceWithDefault branch, no extraction
functions / virtual columns): each suite's input rows and, per filter, the expected list of dim0
values of the matching rows (BaseFilterTest.assertFilterMatches). Paths relative to /root/reference,
processing/src/test/java/org/apache/druid/segment/filter/. Filters use the query JSON of
incubator-druid_amd/query.py (BoundDimFilter(dimension, lower, upper, lowerStrict, upperStrict,
alphaNumeric, extractionFn, ordering) -> {"type": "bound", ...}).

    python tests/golden/make_filter_kats.py
"""
import json
import os

ALL6 = ["0", "1", "2", "3", "4", "5"]
ALL8 = ALL6 + ["6", "7"]
AF = ["a", "b", "c", "d", "e", "f"]


def sel(d, v):
    return {"type": "selector", "dimension": d, "value": v}


def inf(d, *vals):
    return {"type": "in", "dimension": d, "values": list(vals)}


def bound(d, lo, hi, ls=False, us=False, ordering="lexicographic"):
    return {"type": "bound", "dimension": d, "lower": lo, "upper": hi, "lowerStrict": ls, "upperStrict": us,
            "ordering": ordering}


def NOT(f):
    return {"type": "not", "field": f}


def AND(*fs):
    return {"type": "and", "fields": list(fs)}


# rows: dim0, dim1 (single-value; "" = null), dim2 (multi-value list; None = row without dim2)
SELECTOR_ROWS = [["0", "", ["a", "b"]], ["1", "10", []], ["2", "2", [""]], ["3", "1", ["a"]], ["4", "def", ["c"]],
                 ["5", "abc", None]]
BOUND_ROWS = SELECTOR_ROWS + [["6", "-1000", ["a"]], ["7", "-10.012", ["d"]]]
IN_ROWS = [[a] + r[1:] for a, r in zip(AF, SELECTOR_ROWS)]
AND_ROWS = [[str(i), "0", None] for i in range(6)]
NOT_ROWS = [[str(i), None, None] for i in range(6)]

SUITES = {
    "SelectorFilterTest": {
        "_source": "SelectorFilterTest.java:71-78 (rows), :103-181 (testSingleValueStringColumnWithoutNulls, "
                   "WithNulls, testMultiValueStringColumn, testMissingColumnSpecifiedInDimensionList / "
                   "NotSpecifiedInDimensionList)",
        "rows": SELECTOR_ROWS,
        "cases": [
            [sel("dim0", None), []], [sel("dim0", ""), []], [sel("dim0", "0"), ["0"]], [sel("dim0", "1"), ["1"]],
            [sel("dim1", None), ["0"]], [sel("dim1", ""), ["0"]], [sel("dim1", "10"), ["1"]], [sel("dim1", "2"), ["2"]],
            [sel("dim1", "1"), ["3"]], [sel("dim1", "def"), ["4"]], [sel("dim1", "abc"), ["5"]], [sel("dim1", "ab"), []],
            [sel("dim2", None), ["1", "2", "5"]], [sel("dim2", ""), ["1", "2", "5"]], [sel("dim2", "a"), ["0", "3"]],
            [sel("dim2", "b"), ["0"]], [sel("dim2", "c"), ["4"]], [sel("dim2", "d"), []],
            [sel("dim3", None), ALL6], [sel("dim3", ""), ALL6], [sel("dim3", "a"), []], [sel("dim3", "b"), []],
            [sel("dim3", "c"), []],
            [sel("dim4", None), ALL6], [sel("dim4", ""), ALL6], [sel("dim4", "a"), []], [sel("dim4", "b"), []],
            [sel("dim4", "c"), []],
        ],
    },
    "BoundFilterTest": {
        "_source": "BoundFilterTest.java:62-71 (rows), :90-503 (lexicographic / alphanumeric / numeric "
                   "bounds, missing column, nulls; replaceWithDefault branch)",
        "rows": BOUND_ROWS,
        "cases": (
            [[bound(d, None, "z"), ALL8] for d in ("dim0", "dim1", "dim2", "dim3")]
            + [[bound(d, "", "z"), ALL8] for d in ("dim0", "dim1", "dim2", "dim3")]
            + [[bound("dim0", "", ""), []], [bound("dim1", "", ""), ["0"]], [bound("dim2", "", ""), ["1", "2", "5"]],
               [bound("dim3", "", ""), ALL8], [bound("dim3", "", None, False, True), ALL8],
               [bound("dim3", None, "", False, True), []], [bound("dim3", "", "", True, False), []],
               [bound("dim3", "", "", False, True), []], [bound("dim3", None, "", False, False), ALL8],
               [bound("dim1", "abc", "abc", True, False), []], [bound("dim1", "abc", "abc", True, True), []],
               [bound("dim1", "abc", "abc", False, True), []], [bound("dim1", "abc", "abc"), ["5"]],
               [bound("dim1", "ab", "abd", True, True), ["5"]], [bound("dim1", "ab", None, True, True), ["4", "5"]],
               [bound("dim1", None, "abd", True, True), ["0", "1", "2", "3", "5", "6", "7"]],
               [bound("dim1", "1", "3"), ["1", "2", "3"]], [bound("dim1", "1", "3", True, True), ["1", "2"]],
               [bound("dim1", "-1", "3", True, True), ["1", "2", "3", "6", "7"]]]
            + [[bound("dim0", "", "", ordering=o), []] for o in ("alphanumeric", "numeric")]
            + [[bound("dim1", "", "", ordering=o), ["0"]] for o in ("alphanumeric", "numeric")]
            + [[bound("dim2", "", "", ordering=o), ["1", "2", "5"]] for o in ("alphanumeric", "numeric")]
            + [[bound("dim3", "", "", ordering=o), ALL8] for o in ("alphanumeric", "numeric")]
            + [[bound("dim1", "2", "2", s1, s2, ordering=o), []] for o in ("alphanumeric", "numeric")
               for s1, s2 in ((True, False), (True, True), (False, True))]
            + [[bound("dim1", "2", "2", ordering=o), ["2"]] for o in ("alphanumeric", "numeric")]
            + [[bound("dim1", "1", "3", True, True, ordering=o), ["2"]] for o in ("alphanumeric", "numeric")]
            + [[bound("dim1", "1", None, True, True, "alphanumeric"), ["1", "2", "4", "5", "6", "7"]],
               [bound("dim1", "-1", None, True, True, "alphanumeric"), ["4", "5", "6", "7"]],
               [bound("dim1", None, "2", True, True, "alphanumeric"), ["0", "3"]],
               [bound("dim1", None, "ZZZZZ", True, True, "alphanumeric"), ALL8],
               [bound("dim1", "-2000", "3", True, True, "alphanumeric"), []],
               [bound("dim1", "3", "-2000", True, True, "alphanumeric"), ["1", "6", "7"]],
               [bound("dim1", "-10.012", "-10.012", ordering="numeric"), ["7"]],
               [bound("dim1", "-11", "-10", ordering="numeric"), ["7"]],
               [bound("dim1", "1", None, True, True, "numeric"), ["1", "2"]],
               [bound("dim1", None, "2", True, True, "numeric"), ["0", "3", "4", "5", "6", "7"]],
               [bound("dim1", "-2000", "3", True, True, "numeric"), ["2", "3", "6", "7"]]]
        ),
    },
    "InFilterTest": {
        "_source": "InFilterTest.java:66-73 (rows), :95-229 (testSingleValueStringColumnWithoutNulls / "
                   "WithNulls, testMultiValueStringColumn, testMissingColumn; replaceWithDefault branch)",
        "rows": IN_ROWS,
        "cases": [
            [inf("dim0", None), []], [inf("dim0", "", ""), []], [inf("dim0", "a", "c"), ["a", "c"]],
            [inf("dim0", "e", "x"), ["e"]],
            [inf("dim1", None, ""), ["a"]], [inf("dim1", ""), ["a"]], [inf("dim1", None, "10", "abc"), ["a", "b", "f"]],
            [inf("dim1", "-1", "ab", "de"), []],
            [inf("dim2", None), ["b", "c", "f"]], [inf("dim2", None, "a"), ["a", "b", "c", "d", "f"]],
            [inf("dim2", None, "b"), ["a", "b", "c", "f"]], [inf("dim2", ""), ["b", "c", "f"]],
            [inf("dim2", "", None), ["b", "c", "f"]], [inf("dim2", "c"), ["e"]], [inf("dim2", "d"), []],
            [inf("dim3", None, None), AF], [inf("dim3", ""), AF], [inf("dim3", None, "a"), AF], [inf("dim3", "a"), []],
            [inf("dim3", "b"), []], [inf("dim3", "c"), []],
        ],
    },
    "AndFilterTest": {
        "_source": "AndFilterTest.java:59-66 (rows), :89-200 (testAnd, testNotAnd)",
        "rows": AND_ROWS,
        "cases": [
            [AND(sel("dim0", "0"), sel("dim1", "0")), ["0"]], [AND(sel("dim0", "0"), sel("dim1", "1")), []],
            [AND(sel("dim0", "1"), sel("dim1", "0")), ["1"]], [AND(sel("dim0", "1"), sel("dim1", "1")), []],
            [AND(NOT(sel("dim0", "1")), NOT(sel("dim1", "1"))), ["0", "2", "3", "4", "5"]],
            [AND(NOT(sel("dim0", "0")), NOT(sel("dim1", "0"))), []],
            [NOT(AND(sel("dim0", "0"), sel("dim1", "0"))), ["1", "2", "3", "4", "5"]],
            [NOT(AND(sel("dim0", "0"), sel("dim1", "1"))), ALL6],
            [NOT(AND(sel("dim0", "1"), sel("dim1", "0"))), ["0", "2", "3", "4", "5"]],
            [NOT(AND(sel("dim0", "1"), sel("dim1", "1"))), ALL6],
            [NOT(AND(NOT(sel("dim0", "1")), NOT(sel("dim1", "1")))), ["1"]],
            [NOT(AND(NOT(sel("dim0", "0")), NOT(sel("dim1", "0")))), ALL6],
        ],
    },
    "NotFilterTest": {
        "_source": "NotFilterTest.java:58-65 (rows), :88-107 (testNotSelector)",
        "rows": NOT_ROWS,
        "cases": [
            [NOT(sel("dim0", None)), ALL6], [NOT(sel("dim0", "")), ALL6], [NOT(sel("dim0", "0")), ["1", "2", "3", "4", "5"]],
            [NOT(sel("dim0", "1")), ["0", "2", "3", "4", "5"]],
        ],
    },
}


# numeric columns (no bitmap index: row post-filters). rows: [dim0, value of each numeric column]
LONG_ROWS = [["1", 1], ["2", 2], ["3", 3], ["4", 4], ["5", 5], ["6", 6], ["7", 100000000], ["8", 100000001],
             ["9", -25], ["10", -100000001]]
FD_ROWS = [[str(i), float(i), float(i)] for i in range(1, 7)]
ALL10 = [str(i) for i in range(1, 11)]


def _fd_cases(col):
    return [
        [sel(col, "3"), ["3"]], [sel(col, "3.0"), ["3"]],
        [bound(col, "2", "5", ordering="numeric"), ["2", "3", "4", "5"]],
        [bound(col, "2.0", "5.0", ordering="numeric"), ["2", "3", "4", "5"]],
        [bound(col, "1", "4", True, True, "numeric"), ["2", "3"]],
        [bound(col, "1.0", "4.0", True, True, "numeric"), ["2", "3"]],
        [inf(col, "2", "4", "8"), ["2", "4"]], [inf(col, "2.0", "4.0", "8.0"), ["2", "4"]],
        [inf(col, *[str(2 * i) for i in range(32)]), ["2", "4", "6"]],
        [sel(col, ""), []], [sel(col, None), []], [sel(col, "abc"), []],
        [bound(col, "a", "b", ordering="numeric"), []],
        [bound(col, " ", "4", ordering="numeric"), ["1", "2", "3", "4"]],
        [bound(col, " ", "A", ordering="numeric"), []],
    ]


def _fd_unsupported(col):
    # String.valueOf(float / double) under LEXICOGRAPHIC, regex / search over it: the engine returns
    # DG_ERR_UNSUPPORTED (the Java factory keeps its CPU engine); expected results kept for reference
    return [
        [bound(col, " ", "4", ordering="lexicographic"), ["1", "2", "3"]],
        [bound(col, " ", "4.0", ordering="lexicographic"), ["1", "2", "3", "4"]],
        [bound(col, " ", "A", ordering="lexicographic"), ["1", "2", "3", "4", "5", "6"]],
        [{"type": "regex", "dimension": col, "pattern": "4"}, ["4"]],
        [{"type": "regex", "dimension": col, "pattern": "4.0"}, ["4"]],
        [{"type": "search", "dimension": col, "query": {"type": "contains", "value": "2", "caseSensitive": True}},
         ["2"]],
    ]


NUMERIC_SUITES = {
    "LongFilteringTest": {
        "_source": "LongFilteringTest.java:88-99 (rows), :129-316 (testLongColumnFiltering, "
                   "testLongColumnFilteringWithNonNumbers)",
        "columns": {"lng": "long"},
        "rows": LONG_ROWS,
        "cases": [
            [sel("lng", "0"), []], [sel("lng", "3"), ["3"]], [sel("lng", "3.0"), ["3"]],
            [sel("lng", "3.00000000000000000000001"), []], [sel("lng", "100000001.0"), ["8"]],
            [sel("lng", "-100000001.0"), ["10"]], [sel("lng", "111119223372036854775807.674398674398"), []],
            [bound("lng", "2", "5", ordering="numeric"), ["2", "3", "4", "5"]],
            [bound("lng", "1", "4", True, True, "numeric"), ["2", "3"]],
            [bound("lng", "2.0", "5.0", ordering="numeric"), ["2", "3", "4", "5"]],
            [bound("lng", "2.0", "5.0", True, True, "numeric"), ["3", "4"]],
            [bound("lng", "1.9", "5.9", True, True, "numeric"), ["2", "3", "4", "5"]],
            [bound("lng", "2.1", "5.9", ordering="numeric"), ["3", "4", "5"]],
            [bound("lng", "111119223372036854775807.67", "5.9", ordering="numeric"), []],
            [bound("lng", "-111119223372036854775807.67", "5.9", ordering="numeric"), ["1", "2", "3", "4", "5", "9", "10"]],
            [bound("lng", "2.1", "111119223372036854775807.67", ordering="numeric"), ["3", "4", "5", "6", "7", "8"]],
            [bound("lng", "2.1", "-111119223372036854775807.67", ordering="numeric"), []],
            [bound("lng", "100000000.0", "100000001.0", True, True, "numeric"), []],
            [bound("lng", "100000000.0", "100000001.0", ordering="numeric"), ["7", "8"]],
            [inf("lng", "2", "4", "8"), ["2", "4"]],
            [inf("lng", "1.999999999999999999", "4.00000000000000000000001"), []],
            [inf("lng", "100000001.0", "99999999.999999999"), ["8"]],
            [inf("lng", "-25.0", "-99999999.999999999"), ["9"]],
            [inf("lng", *[str(2 * i) for i in range(32)]), ["2", "4", "6"]],
            [sel("lng", ""), []], [sel("lng", None), []], [sel("lng", "abc"), []],
            [bound("lng", "a", "b", ordering="numeric"), []],
            [bound("lng", " ", "4", ordering="numeric"), ["1", "2", "3", "4", "9", "10"]],
            [bound("lng", " ", "4", ordering="lexicographic"), ["1", "2", "3", "4", "7", "8", "9", "10"]],
            [bound("lng", " ", "A", ordering="numeric"), []],
            [bound("lng", " ", "A", ordering="lexicographic"), ALL10],
        ],
        "unsupported": [
            [{"type": "regex", "dimension": "lng", "pattern": "4"}, ["4"]],
            [{"type": "search", "dimension": "lng", "query": {"type": "contains", "value": "2", "caseSensitive": True}},
             ["2", "9"]],
        ],
    },
    "FloatAndDoubleFilteringTest": {
        "_source": "FloatAndDoubleFilteringTest.java:84-91 (rows), :160-290 (doTestFloatColumnFiltering, "
                   "doTestFloatColumnFilteringWithNonNumbers; float and double columns)",
        "columns": {"flt": "float", "dbl": "double"},
        "rows": FD_ROWS,
        "cases": _fd_cases("flt") + _fd_cases("dbl"),
        "unsupported": _fd_unsupported("flt") + _fd_unsupported("dbl"),
    },
}


def main():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")
    with open(path) as f:
        kats = json.load(f)
    kats["filter_kats"] = {"_source": "processing/src/test/java/org/apache/druid/segment/filter/ "
                                      "(replaceWithDefault branch; expected = dim0 values of the matching rows)",
                           "suites": SUITES, "numeric_suites": NUMERIC_SUITES}
    with open(path, "w") as f:
        json.dump(kats, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
