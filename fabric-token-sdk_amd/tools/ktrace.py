#!/usr/bin/env python3
"""Timeline of the last `tail` dispatches in a rocprofv3 --kernel-trace CSV:
name, grid, duration and the idle gap before each (microseconds).
    python ktrace.py <kernel_trace.csv> [tail]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tail = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-tail:]
prev = None
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print("%9.1f %8.1f us  gap %7.1f  grid %9s  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, r.get("Grid_Size", "?"),
                                                      r["Kernel_Name"].split("(")[0][:48]))
    prev = e
print("span %.1f us" % ((int(rows[-1]["End_Timestamp"]) - t0) / 1e3))
