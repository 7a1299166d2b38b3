#!/usr/bin/env python3
"""Per-round kernel summary from a rocprofv3 SQLite output (rocpd 'kernels' view): the last N decode
rounds, delimited by the argmax kernel that ends every round.

    python tools/prof_db_summary.py gpurun_out/prof_dir [rounds]
"""
import collections
import glob
import sqlite3
import sys


def main():
    d = sys.argv[1]
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    f = glob.glob(d + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(f)
    rows = c.execute("select name, start, end, grid_x, grid_y, workgroup_x, lds_size from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if "argmax" in r[0]]
    if len(ends) < nr + 1:
        nr = len(ends) - 1
    a, b = ends[-nr - 1] + 1, ends[-1] + 1
    sel = rows[a:b]
    wall = (sel[-1][2] - sel[0][1]) / 1e3 / nr
    busy = sum(r[2] - r[1] for r in sel) / 1e3 / nr
    print(f"# last {nr} decode rounds: wall {wall:.1f} us/round, kernel-busy {busy:.1f} us/round, "
          f"gaps {wall - busy:.1f} us/round, {len(sel) // nr} kernels/round")
    agg = collections.defaultdict(lambda: [0.0, 0, None])
    for r in sel:
        k = (r[0][:90], r[3] // max(1, r[5]), r[4])
        agg[k][0] += (r[2] - r[1]) / 1e3
        agg[k][1] += 1
    for (name, gx, gy), (t, n, _) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"  {t / nr:8.1f} us/round {n // nr:4d}/round avg {t / n:7.2f} us  grid {gx}x{gy}  {name}")


if __name__ == "__main__":
    main()
