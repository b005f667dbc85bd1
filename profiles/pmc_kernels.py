#!/usr/bin/env python3
"""Per-(kernel, grid) PMC table from the rocprofv3 --pmc passes of
scripts/profile_round.sh (one counter group per pass, rocpd sqlite each):

    python profiles/pmc_kernels.py gpurun_out/prof_r02 > profiles/r02_pmc_kernels.txt

Columns are means per dispatch.  SQ_* wave-cycle counters are in quad-cycles
(MI355X_MICROARCH.md "Per-instruction cycle constants"); FETCH_SIZE is in KB
and reports half the bytes of wide reads on gfx950 (x2 applied), WRITE_SIZE in
KB.  Derived:
  valu/ns   VALU wave-instructions per ns of kernel time (chip-wide issue rate;
            the measured v_mad_u64_u32 peak is ~0.53 wave-inst/ns, madpeak)
  issue%    SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES  (lifetime share a wave issues)
  dep%      SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES    (waiting on an instruction dependency)
  mem%      SQ_WAIT_ANY / SQ_WAVE_CYCLES         (parked in s_waitcnt / barrier)
"""
import collections
import glob
import os
import sqlite3
import sys


def load(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for db in sorted(glob.glob(os.path.join(root, "pmc*", "**", "*.db"), recursive=True)):
        con = sqlite3.connect(db)
        rows = con.execute("select kernel_name, grid_size, dispatch_id, counter_name, sum(value), max(duration) "
                           "from counters_collection group by dispatch_id, counter_name").fetchall()
        for name, grid, did, cname, v, d in rows:
            key = (name.split("(")[0], int(grid))
            vals[key][cname].append(float(v))
            if cname in ("SQ_WAVES",):
                dur[key].append(float(d))
    return vals, dur


def main(root):
    vals, dur = load(root)
    mean = lambda xs: sum(xs) / len(xs) if xs else float("nan")
    cols = ["n", "us", "waves", "valu", "salu", "vmem_rd", "lds", "valu/ns", "issue%", "dep%", "mem%", "ldsconf",
            "fetch_MB", "write_MB"]
    print(("%-22s %9s " % ("kernel", "grid")) + " ".join("%9s" % c for c in cols))
    for key in sorted(vals, key=lambda k: (k[0], k[1])):
        name, grid = key
        if name.startswith("__amd") or name.startswith("void rocprim"):
            continue
        v = {c: mean(x) for c, x in vals[key].items()}
        us = mean(dur[key]) / 1e3 if dur[key] else float("nan")
        wc = v.get("SQ_WAVE_CYCLES", float("nan"))
        row = [len(dur[key]), us, v.get("SQ_WAVES", 0), v.get("SQ_INSTS_VALU", float("nan")),
               v.get("SQ_INSTS_SALU", float("nan")), v.get("SQ_INSTS_VMEM_RD", float("nan")),
               v.get("SQ_INSTS_LDS", float("nan")),
               v.get("SQ_INSTS_VALU", float("nan")) / (us * 1e3) if us == us and us > 0 else float("nan"),
               100 * v.get("SQ_ACTIVE_INST_ANY", float("nan")) / wc, 100 * v.get("SQ_WAIT_INST_ANY", float("nan")) / wc,
               100 * v.get("SQ_WAIT_ANY", float("nan")) / wc, v.get("SQ_LDS_BANK_CONFLICT", float("nan")),
               v.get("FETCH_SIZE", float("nan")) * 2 / 1024, v.get("WRITE_SIZE", float("nan")) / 1024]
        print(("%-22s %9d " % (name[:22], grid)) + " ".join("%9.4g" % x for x in row))


if __name__ == "__main__":
    main(sys.argv[1])
