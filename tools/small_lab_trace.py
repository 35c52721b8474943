#!/usr/bin/env python3
"""Sum the batch kernels of each timed call of tools/small_lab.py from its
rocprofv3 kernel trace (calls are delimited by the lab's marker kernel).
    python tools/small_lab_trace.py <trace.csv> <lab.log>"""
import csv, json, sys


def main(trace, log):
    pts = [json.loads(l) for l in open(log) if l.startswith("{")]
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        if "elementwise" in n or "add" in n.lower() and "s3dg" not in n:
            cur = {"fill": 0, "map": 0, "first": None, "last": None}
            calls.append(cur)
            continue
        if cur is None or "s3dg" not in n:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        cur["fill" if "k_fill" in n else "map"] += e - s
        cur["first"] = s if cur["first"] is None else cur["first"]
        cur["last"] = e
    reps = len(calls) // len(pts)
    for i, p in enumerate(pts):
        cs = [calls[r * len(pts) + i] for r in range(reps)]
        print(json.dumps({**{k: p[k] for k in ("size", "waves", "occ", "pf", "store", "tile")},
                          "fill_ms": [round(c["fill"] / 1e6, 3) for c in cs],
                          "map_ms": [round(c["map"] / 1e6, 3) for c in cs],
                          "span_ms": [round((c["last"] - c["first"]) / 1e6, 3) for c in cs],
                          "GBps_events": p["GBps_events_median"]}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
