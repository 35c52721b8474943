#!/usr/bin/env python3
"""Fill time per workgroup slot and per byte from the kernel traces of
tools/r04/gpu_h.sh (one rocprofv3 directory per layout kind).

    python tools/r04/wg_cost.py gpurun_out/r04h

Tooling only: nothing in the product imports this."""
import csv, glob, json, os, re, sys

root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*"))):
    if not os.path.isdir(d):
        continue
    traces = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not traces:
        continue
    rows = list(csv.DictReader(open(traces[0])))
    fills = [r for r in rows if re.search(r"k_fill_batch<\d+, \d+, false", r["Kernel_Name"])]
    maps = [r for r in rows if "k_batch_map" in r["Kernel_Name"] or "k_tile_map" in r["Kernel_Name"]]
    if not fills:
        continue
    dur = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in fills)
    wgs = sum(int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]) for r in fills)
    mdur = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in maps)
    print(json.dumps({"kind": os.path.basename(d), "fill_launches": len(fills), "fill_ms": round(dur / 1e6, 3),
                      "slots": wgs, "slots_per_ns": round(wgs / dur, 4), "ns_per_slot_chip": round(dur / wgs, 4),
                      "map_ms": round(mdur / 1e6, 3), "kernel": fills[0]["Kernel_Name"][:60]}))
