#!/usr/bin/env python3
"""Summarise a same-box A/B (scripts/ab_lib.sh, scripts/pmc_ab.sh) from gpurun_out/:
    python scripts/ab_summary.py ROUNDS name1 name2 ... [--kernels k_g2_part,k_g2lines1]
One line per (round, library): value, device-only, serial ms and frac of every stage;
then SQ_INSTS_VALU per launch of the listed kernels from the PMC runs (grids > 100k)."""
import collections
import glob
import json
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
kern = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--kernels=")), "")
rounds, names = int(args[0]), args[1:]
for r in range(1, rounds + 1):
    for n in names:
        try:
            d = json.loads(open("gpurun_out/ablib_%s_%d.log" % (n, r)).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            print(n, r, "missing")
            continue
        rf = d.get("roofline") or {}
        if d.get("msm"):
            print("%-6s r%d msm %s resident %s" % (n, r, [(m["n"], m["ms"], m.get("ms_host_scalars")) for m in d["msm"]],
                                                 [(m["n"], m["ms"]) for m in d.get("msm_resident") or []]))
        if not rf.get("serial_ms"):
            continue
        print("%-6s r%d value %9.0f dev %9.0f | %s" % (
            n, r, d["value"], (d.get("device_only") or {}).get("transfers_per_s", 0),
            " ".join("%s %.3f/%.3f" % (k, rf["serial_ms"][k], rf["per_kernel_frac"][k])
                     for k in ("g1p", "g2", "miller", "fexp", "g1"))))
if kern:
    for n in names:
        dbs = glob.glob("gpurun_out/pmcab_%s/**/*.db" % n, recursive=True)
        if not dbs:
            continue
        c = sqlite3.connect(dbs[0])
        rows = c.execute("select kernel_name, grid_size, dispatch_id, sum(value) from counters_collection "
                         "where counter_name = 'SQ_INSTS_VALU' group by dispatch_id").fetchall()
        agg = collections.defaultdict(list)
        for k, g, _, v in rows:
            agg[(k.split("(")[0], g)].append(v)
        for (k, g), vs in sorted(agg.items()):
            if k in kern.split(",") and g > 30000:
                print("%-6s %s grid %d: %.4g VALU/launch (%d)" % (n, k, g, sum(vs) / len(vs), len(vs)))
