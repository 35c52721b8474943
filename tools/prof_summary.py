#!/usr/bin/env python3
"""Condense a tools/profile_round.sh output directory into committed evidence:

  profiles/<round>/kernel_stats_cfgN.csv   rocprofv3 --stats summary (as produced)
  profiles/<round>/kernel_trace_cfgN.csv   rocprofv3 kernel trace (as produced)
  profiles/<round>/pmc_<CTR>_cfgN.csv      PMC pass, fill-kernel rows only
  profiles/<round>/timing_cfgN.json        per-step fill time from the trace
                                           (warmup dispatches excluded) next to
                                           bench.py's HIP-event avg_launch_ms
  profiles/traffic.json                    HBM bytes per bench launch (cfg 2, 4, 6)

PMC units/corrections follow MI355X_MICROARCH.md (HBM/rocprofv3 section):
WRITE_SIZE x 1024 B; FETCH_SIZE x 1024 x 2 (gfx950 half-count).
    python tools/prof_summary.py gpurun_out/r2prof r02"""
import csv, json, os, shutil, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_line(path):
    for line in open(path):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {path}")


def main(src, rnd):
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    for c in (2, 4, 6):
        kern = "k_keystream" if c == 6 else "k_fill_"
        tr = os.path.join(src, f"trace_cfg{c}")
        if not os.path.isdir(tr):
            continue
        shutil.copy(os.path.join(tr, "run_kernel_stats.csv"), os.path.join(dst, f"kernel_stats_cfg{c}.csv"))
        shutil.copy(os.path.join(tr, "run_kernel_trace.csv"), os.path.join(dst, f"kernel_trace_cfg{c}.csv"))
        b = bench_line(os.path.join(src, f"bench_trace_cfg{c}.log"))
        steps, warm = b["steps"], b["warmup"]
        rows = [r for r in csv.DictReader(open(os.path.join(tr, "run_kernel_trace.csv")))
                if kern in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        per_step = len(rows) // (steps + warm)
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]
        steps_ms = [sum(durs[i * per_step:(i + 1) * per_step]) for i in range(steps + warm)]
        timed = steps_ms[warm:]
        name = rows[0]["Kernel_Name"].replace("void s3dg::(anonymous namespace)::", "").split("(")[0]
        out = {"kernel": name, "dispatches_per_step": per_step,
               "all_dispatch_ms_avg": round(sum(durs) / len(durs), 4),
               "timed_step_kernel_ms": [round(x, 4) for x in timed],
               "timed_step_kernel_ms_avg": round(sum(timed) / len(timed), 4),
               "bench_avg_launch_ms": b["roofline"]["avg_launch_ms"],
               "bench_achieved_GBps": b["roofline"]["achieved"],
               "trace_achieved_GBps": round(b["roofline"]["algorithmic_bytes_per_launch"]
                                            / (sum(timed) / len(timed) * 1e-3) / 1e9, 1),
               "note": "bench avg_launch_ms brackets the whole s3dg_fill_* call with HIP events "
                       "(for cfg4 also the descriptor upload and k_tile_map); warmup dispatches excluded"}
        json.dump(out, open(os.path.join(dst, f"timing_cfg{c}.json"), "w"), indent=1)
        print(json.dumps(out))
        ent = {"kernel": name, "workload": b["config"]["workload"],
               "algorithmic_bytes_per_launch": b["roofline"]["algorithmic_bytes_per_launch"]}
        for ctr, scale in (("WRITE_SIZE", 1024), ("FETCH_SIZE", 2048)):
            p = os.path.join(src, f"pmc_{ctr}_cfg{c}", "run_counter_collection.csv")
            if not os.path.exists(p):
                break
            rr = [r for r in csv.DictReader(open(p)) if kern in r["Kernel_Name"]]
            with open(os.path.join(dst, f"pmc_{ctr.lower()}_cfg{c}.csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(rr[0].keys()))
                w.writeheader()
                w.writerows(rr)
            # the PMC run is bench --steps 1 --warmup 0: one bench launch
            ent[f"{ctr.lower()}_bytes_per_launch"] = int(round(sum(float(r["Counter_Value"]) for r in rr) * scale))
        else:
            ent["traffic_bytes_per_launch"] = ent["write_size_bytes_per_launch"] + ent["fetch_size_bytes_per_launch"]
            ent["method"] = ("rocprofv3 --pmc WRITE_SIZE and --pmc FETCH_SIZE in separate passes (no tracing "
                             "domains), summed over the fill dispatches of one bench launch; WRITE_SIZE x 1024 B; "
                             "FETCH_SIZE x 1024 x 2 (gfx950 half-count correction, MI355X_MICROARCH.md)")
            ent["sources"] = [f"profiles/{rnd}/pmc_write_size_cfg{c}.csv", f"profiles/{rnd}/pmc_fetch_size_cfg{c}.csv"]
            traffic[str(c)] = ent
    json.dump(traffic, open(tpath, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
