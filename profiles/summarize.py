#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run (sqlite .db or kernel_trace.csv)
into the per-kernel stats table committed under profiles/.

    python profiles/summarize.py gpurun_out/prof/run_results.db > profiles/rNN_kernel_stats.txt
"""
import collections
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    con = sqlite3.connect(path)
    q = ("select s.kernel_name, d.end - d.start, s.arch_vgpr_count, s.accum_vgpr_count, s.sgpr_count, "
         "s.private_segment_size, d.grid_size_x, d.workgroup_size_x from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    return con.execute(q).fetchall()


def from_csv(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r.get("VGPR_Count"),
                     r.get("Accum_VGPR_Count", 0), r.get("SGPR_Count"), r.get("Scratch_Size", r.get("Private_Segment_Size")),
                     r.get("Grid_Size", r.get("Grid_Size_X")), r.get("Workgroup_Size", r.get("Workgroup_Size_X"))))
    return rows


def main(path):
    if os.path.isdir(path):
        c = glob.glob(os.path.join(path, "**", "*.db"), recursive=True) or \
            glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        path = c[0]
    rows = from_db(path) if path.endswith(".db") else from_csv(path)
    agg = collections.defaultdict(list)
    info = {}
    for name, ns, v, av, sg, ps, grid, wg in rows:
        short = name.split("(")[0]
        agg[short].append(ns / 1e6)
        info[short] = (v, av, sg, ps, grid, wg)
    tot = sum(sum(v) for v in agg.values())
    print("%-28s %6s %10s %10s %7s %5s %5s %5s %7s %8s" % ("kernel", "calls", "avg_ms", "total_ms", "pct", "vgpr",
                                                           "agpr", "sgpr", "scratch", "grid"))
    for n, ts in sorted(agg.items(), key=lambda x: -sum(x[1])):
        v, av, sg, ps, grid, wg = info[n]
        print("%-28s %6d %10.3f %10.3f %6.1f%% %5s %5s %5s %7s %8s" % (n[:28], len(ts), sum(ts) / len(ts), sum(ts),
                                                                     100 * sum(ts) / tot, v, av, sg, ps, grid))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
