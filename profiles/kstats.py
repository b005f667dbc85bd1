import sqlite3, glob, sys
c = sqlite3.connect(glob.glob(sys.argv[1] + '/*.db')[0])
pat = sys.argv[2] if len(sys.argv) > 2 else ''
rows = c.execute("select name, count(*), avg(duration), grid_x, workgroup_x, vgpr_count, scratch_size from kernels group by name, grid_x order by name, grid_x").fetchall()
for r in rows:
    if pat in r[0]:
        print("%-34s %4d %10.1f us grid %9d wg %4d vgpr %3d scr %d" % (r[0][:34], r[1], r[2] / 1e3, r[3], r[4], r[5], r[6]))
