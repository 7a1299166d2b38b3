#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc CSV (one row per dispatch x counter) per kernel+grid: mean counters."""
import collections, csv, glob, os, sys

for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        print(d, "no counter csv"); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        key = (r.get("Kernel_Name", "")[:60], r.get("Grid_Size", r.get("Grid_Size_X", "")))
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("==", d)
    for key, cs in agg.items():
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        wc = m.get("SQ_WAVE_CYCLES", 1) or 1
        print(f"{key[0]} grid={key[1]}")
        print("   " + "  ".join(f"{k}={v:.3g}" for k, v in sorted(m.items())))
        print(f"   wait_any/wave={m.get('SQ_WAIT_ANY',0)/wc:.2f} wait_inst/wave={m.get('SQ_WAIT_INST_ANY',0)/wc:.2f} "
              f"active/wave={m.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} valu_active/wave={m.get('SQ_ACTIVE_INST_VALU',0)/wc:.2f} "
              f"valu_insts/vmem={m.get('SQ_INSTS_VALU',0)/max(1,m.get('SQ_INSTS_VMEM_RD',1)):.1f}")
