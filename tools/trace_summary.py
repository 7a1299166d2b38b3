#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: per-kernel time over the LAST n decode rounds
(a round = the dispatches between consecutive argmax kernels), plus gaps between kernels."""
import csv, collections, sys
path = sys.argv[1]; nr = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'argmax' in r['Kernel_Name']]
a, b = idx[-nr - 1] + 1, idx[-1] + 1
sel = rows[a:b]
t0, t1 = int(sel[0]['Start_Timestamp']), int(sel[-1]['End_Timestamp'])
busy = collections.defaultdict(float); cnt = collections.Counter()
for r in sel:
    nm = r['Kernel_Name']
    key = nm.split('(')[0][:60] + (' grid=%sx%s' % (r['Grid_Size_X'], r['Grid_Size_Y']) if 'gemv' in nm else '')
    busy[key] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    cnt[key] += 1
tot = sum(busy.values()); wall = (t1 - t0) / 1e3
print(f"rounds={nr} wall={wall/nr:.1f} us/round  kernel-busy={tot/nr:.1f} us/round  gaps={(wall-tot)/nr:.1f} us/round  kernels/round={len(sel)/nr:.0f}")
for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
    print(f"{v/nr:9.1f} us/round  {cnt[k]//nr:4d}/round  avg {v/cnt[k]:7.2f} us  {k}")
