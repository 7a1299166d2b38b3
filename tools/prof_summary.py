#!/usr/bin/env python3
"""Summarise a rocprofv3 output directory (--kernel-trace --stats --output-format csv):
top kernels by total time from *_kernel_stats.csv, then the per-decode-round breakdown from the
kernel trace (a round = the dispatches between consecutive argmax/sample kernels)."""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    nr = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        rows = list(csv.DictReader(open(stats[0])))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        print(f"# kernel stats ({os.path.relpath(stats[0], d)}), total GPU time {tot / 1e6:.2f} ms")
        for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:20]:
            print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} ms {100 * float(r['TotalDurationNs']) / tot:5.1f}% "
                  f"calls={r['Calls']:>6} avg={float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:90]}")
    traces = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not traces:
        return
    rows = sorted(csv.DictReader(open(traces[0])), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "argmax" in r["Kernel_Name"] or "sample_kernel" in r["Kernel_Name"]]
    if len(idx) < nr + 1:
        return
    sel = rows[idx[-nr - 1] + 1: idx[-1] + 1]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    busy = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in sel:
        nm = r["Kernel_Name"]
        key = nm.split("(")[0][:70]
        busy[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[key] += 1
    tot = sum(busy.values())
    wall = (t1 - t0) / 1e3
    print(f"\n# last {nr} decode rounds: wall {wall / nr:.1f} us/round, kernel-busy {tot / nr:.1f} us/round, "
          f"gaps {(wall - tot) / nr:.1f} us/round, {len(sel) / nr:.0f} kernels/round")
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
        print(f"{v / nr:9.1f} us/round  {cnt[k] // nr:4d}/round  avg {v / cnt[k]:7.2f} us  {k}")
    # one layer's worth of the last round in dispatch order: duration and the gap before each kernel
    last = rows[idx[-2] + 1: idx[-1] + 1]
    n_show = int(os.environ.get("PROF_SEQ", "14"))
    if n_show > 0:
        print(f"\n# dispatch order, middle of the last round ({n_show} kernels): gap-before / duration us")
        mid = max(0, len(last) // 2 - n_show // 2)
        prev_end = int(last[mid - 1]["End_Timestamp"]) if mid > 0 else None
        for r in last[mid: mid + n_show]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
            prev_end = e
            print(f"  {gap:6.2f} {((e - s) / 1e3):8.2f}  {r['Kernel_Name'].split('(')[0][:80]}")


if __name__ == "__main__":
    main()
