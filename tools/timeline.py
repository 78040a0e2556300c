"""Kernel timeline of the last bench step from a rocprofv3 kernel trace (diagnostic): every kernel of the
last `n` launches with its start relative to the first of them, its duration and its queue/stream, so
the critical path of a small query (launch gaps, stream overlap) can be read off.
    python tools/timeline.py gpurun_out/prof_trace [n]"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    qk = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    for r in rows:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f} us  q{r.get(qk, '?'):>3}  {r['Kernel_Name'][:90]}")


if __name__ == "__main__":
    main()
