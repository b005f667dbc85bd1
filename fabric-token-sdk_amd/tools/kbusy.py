#!/usr/bin/env python3
"""GPU busy fraction over time from a rocprofv3 --kernel-trace CSV: the union
of kernel intervals per bin (default 2 ms) over the last `span_ms` of the
trace, and the overall busy fraction of that window.
    python kbusy.py <kernel_trace.csv> [span_ms] [bin_ms]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
span = float(sys.argv[2]) if len(sys.argv) > 2 else 120.0
binw = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
t_end = max(e for _, e, _ in iv)
t0 = t_end - int(span * 1e6)
iv = [(max(s, t0), e, n) for s, e, n in iv if e > t0]
# union of intervals
merged = []
for s, e, _ in iv:
    if merged and s <= merged[-1][1]:
        merged[-1][1] = max(merged[-1][1], e)
    else:
        merged.append([s, e])
nb = int(span / binw) + 1
busy = [0.0] * nb
for s, e in merged:
    while s < e:
        b = int((s - t0) / (binw * 1e6))
        be = t0 + int((b + 1) * binw * 1e6)
        seg = min(e, be) - s
        if 0 <= b < nb:
            busy[b] += seg
        s += seg
tot = sum(e - s for s, e in merged)
print("window %.1f ms, busy %.1f ms (%.1f %%)" % (span, tot / 1e6, 100 * tot / (span * 1e6)))
print(" ".join("%3d" % int(100 * b / (binw * 1e6)) for b in busy))
