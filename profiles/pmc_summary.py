#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc run (rocpd sqlite) per kernel: mean counter
value per dispatch.  python profiles/pmc_summary.py gpurun_out/pmcN/p_results.db"""
import collections
import sqlite3
import sys


def main(path):
    con = sqlite3.connect(path)
    rows = con.execute("select kernel_name, dispatch_id, counter_name, sum(value), max(duration) "
                       "from counters_collection group by kernel_name, dispatch_id, counter_name").fetchall()
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for k, d, c, v, dur in rows:
        agg[k.split("(")[0][:40]][c].append(v)
    names = sorted({c for k in agg for c in agg[k]})
    print("%-40s " % "kernel" + " ".join("%14s" % n.replace("SQ_", "")[:14] for n in names))
    for k in sorted(agg):
        if k.startswith("__amd"):
            continue
        print("%-40s " % k + " ".join("%14.4g" % (sum(agg[k][n]) / len(agg[k][n]) if agg[k][n] else 0) for n in names))


if __name__ == "__main__":
    main(sys.argv[1])
