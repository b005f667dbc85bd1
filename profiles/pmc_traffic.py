#!/usr/bin/env python3
"""HBM traffic per launch of the verification kernels from two rocprofv3 --pmc
passes (FETCH_SIZE and WRITE_SIZE in their own runs, FTZ_SERIAL=1 bench), per
MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE is in KB and reports half the
bytes of wide reads on gfx950 (x2 applied), WRITE_SIZE in KB.
    python profiles/pmc_traffic.py gpurun_out/pmc_fetch/p_results.db gpurun_out/pmc_write/p_results.db \\
        [gpurun_out/pmc_sq/p_results.db] > profiles/pmc_fetch.json
Keys match bench.py's roofline kernel keys."""
import collections
import json
import sqlite3
import sys


def per_grid(path, counter):
    con = sqlite3.connect(path)
    rows = con.execute("select kernel_name, grid_size, dispatch_id, sum(value) from counters_collection "
                       "where counter_name = ? group by dispatch_id", (counter,)).fetchall()
    agg = collections.defaultdict(list)
    for name, grid, _, v in rows:
        agg[(name.split("(")[0], grid)].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(fetch_db, write_db, valu_db=None):
    f, w = per_grid(fetch_db, "FETCH_SIZE"), per_grid(write_db, "WRITE_SIZE")
    vv = per_grid(valu_db, "SQ_INSTS_VALU") if valu_db else {}
    out_valu = {}
    kb = lambda k: f.get(k, 0.0) * 2 * 1024 + w.get(k, 0.0) * 1024

    def grids(name):
        return sorted(g for (n, g) in f if n == name)

    out = {}
    part, comb = grids("k_g1_part"), grids("k_g1_combine")
    if part and comb:
        out["g1"] = kb(("k_g1_part", part[-1])) + kb(("k_g1_combine", comb[-1]))
        out["g1p"] = kb(("k_g1_part", part[0])) + kb(("k_g1_combine", comb[0]))
    # "3*k" = three launches of k per pass (the final exponentiation's x-powers)
    for key, names in (("miller", ("k_miller_n", "k_miller")),
                       ("fexp", ("k_fexp_easy_a+k_fexp_binv+k_fexp_easy_b+3*k_fexp_expt+k_fexp_hard",
                                 "k_fexp_easy+3*k_fexp_expt+k_fexp_hard", "k_fexp_exact", "k_fexp")),
                       ("g2", ("k_g2_part+k_g2_sum+k_g2_binv+k_g2lines1", "k_g2_part+k_g2lines1", "k_g2lines")), ("decode", ("k_decode",))):
        for name in names:
            parts = [(int(p.split("*")[0]), p.split("*")[1]) if "*" in p else (1, p) for p in name.split("+")]
            gs = [grids(n) for _, n in parts]
            if all(gs):  # the largest grid of each kernel (the verification batch)
                out[key] = sum(m * kb((n, g[-1])) for (m, n), g in zip(parts, gs))
                if vv:
                    out_valu[key] = sum(m * vv.get((n, g[-1]), 0.0) for (m, n), g in zip(parts, gs))
                break
    h = grids("k_hash")
    if h:
        out["hash"] = kb(("k_hash", h[-1]))
    raw = {"%s[grid=%d]" % k: {"fetch_kb": round(f.get(k, 0), 1), "write_kb": round(w.get(k, 0), 1)}
           for k in sorted(f) if k[0].startswith("k_")}
    doc = {"per_launch_bytes": {k: int(v) for k, v in out.items()}, "raw_per_launch": raw,
           "method": "FETCH_SIZE*1024*2 + WRITE_SIZE*1024 per dispatch, FTZ_SERIAL=1 bench, separate passes"}
    if out_valu:
        doc["per_launch_valu"] = {k: int(v) for k, v in out_valu.items()}
        doc["valu_method"] = "SQ_INSTS_VALU (wave-instructions) per dispatch, summed like the bytes"
    json.dump(doc, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:4])
