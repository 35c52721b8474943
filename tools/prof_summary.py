#!/usr/bin/env python3
"""Condense a tools/profile_round.sh output directory into committed evidence:

  profiles/<round>/kernel_stats_cfgN.csv   rocprofv3 --stats summary (as produced)
  profiles/<round>/kernel_trace_cfgN.csv   rocprofv3 kernel trace (as produced)
  profiles/<round>/bench_trace_cfgN.log    the bench line of the traced run
  profiles/<round>/pmc_<ctr>_cfgN.csv      PMC pass, step-kernel rows only
  profiles/<round>/timing_cfgN.json        per-step kernel time from the trace
                                           (warmup steps excluded) next to the
                                           bench line's HIP-event numbers
  profiles/traffic.json                    HBM bytes per bench launch, keyed to
                                           the library source digest and commit

A step's kernels are the dispatches bench.py's step() makes: the fill
(k_fill_stream / k_fill_batch without the ablated `true` variant /
k_keystream) plus its record builders (k_tile_map_uniform, k_batch_map).
Ceilings and verification run after the timed steps and are excluded.
PMC units/corrections follow MI355X_MICROARCH.md (HBM/rocprofv3 section):
WRITE_SIZE x 1024 B; FETCH_SIZE x 1024 x 2 (gfx950 half-count).
    python tools/prof_summary.py gpurun_out/r2prof r02"""
import csv, json, os, shutil, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STEP_KERNELS = ("k_fill_stream", "k_fill_batch", "k_keystream", "k_zero_prefix", "k_tile_map_uniform", "k_batch_map")
FILL_KERNELS = ("k_fill_stream", "k_fill_batch", "k_keystream", "k_zero_prefix")


def bench_line(path):
    for line in open(path):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no bench JSON line in {path}")


def is_step(name, kinds=STEP_KERNELS):
    """A step kernel, not the store-only reference (k_fill_batch<NT, NW, true, ...>: ABL, the third
    template argument; the FLOOR instantiation carries `true` in the fourth)."""
    import re
    return any(k in name for k in kinds) and not re.search(r"k_fill_batch<\d+, \d+, true", name)


def main(src, rnd):
    import bench
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    digest = bench.source_digest()
    # keep records of other configs taken at the same library digest (several
    # profile directories per round); records of older digests are dropped
    try:
        traffic = {k: v for k, v in json.load(open(tpath)).items() if v.get("source_digest") == digest}
    except (OSError, ValueError):
        traffic = {}
    try:
        commit = subprocess.check_output(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], text=True).strip()
    except Exception:
        commit = None
    for c in sorted(bench.CONFIGS):
        tr = os.path.join(src, f"trace_cfg{c}")
        if not os.path.isdir(tr):
            continue
        shutil.copy(os.path.join(tr, "run_kernel_stats.csv"), os.path.join(dst, f"kernel_stats_cfg{c}.csv"))
        shutil.copy(os.path.join(tr, "run_kernel_trace.csv"), os.path.join(dst, f"kernel_trace_cfg{c}.csv"))
        shutil.copy(os.path.join(src, f"bench_trace_cfg{c}.log"), os.path.join(dst, f"bench_trace_cfg{c}.log"))
        b = bench_line(os.path.join(src, f"bench_trace_cfg{c}.log"))
        if b["roofline"].get("source_digest") != digest:
            print(f"cfg{c}: profiled tree digest {b['roofline'].get('source_digest')} != {digest}", file=sys.stderr)
        steps, warm = b["steps"], b["warmup"]
        rows = [r for r in csv.DictReader(open(os.path.join(tr, "run_kernel_trace.csv")))
                if is_step(r["Kernel_Name"])]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        per_step = len(rows) // (steps + warm)
        rows = rows[:per_step * (steps + warm)]
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]
        fill = [is_step(r["Kernel_Name"], FILL_KERNELS) for r in rows]
        step_ms = [sum(dur[i * per_step:(i + 1) * per_step]) for i in range(steps + warm)][warm:]
        fill_ms = [sum(d for d, f in zip(dur[i * per_step:(i + 1) * per_step], fill[i * per_step:(i + 1) * per_step])
                       if f) for i in range(steps + warm)][warm:]
        span_ms = [(int(rows[(i + 1) * per_step - 1]["End_Timestamp"]) - int(rows[i * per_step]["Start_Timestamp"]))
                   * 1e-6 for i in range(steps + warm)][warm:]
        step_bytes = b["config"]["bytes_per_step_all_ranks"] // b["n_gpus"]
        names = sorted({r["Kernel_Name"].replace("void s3dg::(anonymous namespace)::", "").replace(
            "s3dg::(anonymous namespace)::", "").split("(")[0] for r in rows})
        avg = lambda v: sum(v) / len(v)
        out = {"config": c, "workload": b["config"]["workload"], "step_kernels": names,
               "dispatches_per_step": per_step,
               "timed_step_kernel_ms": [round(x, 4) for x in step_ms],
               "timed_step_kernel_ms_avg": round(avg(step_ms), 4),
               "timed_step_fill_kernel_ms_avg": round(avg(fill_ms), 4),
               "timed_step_first_start_to_last_end_ms_avg": round(avg(span_ms), 4),
               "bench_ms_per_step": b["ms_per_step"],
               "bench_avg_launch_ms": b["roofline"]["avg_launch_ms"],
               "bench_achieved_GBps": b["roofline"]["achieved"],
               "trace_fill_GBps": round(step_bytes / (avg(fill_ms) * 1e-3) / 1e9, 1),
               "trace_step_kernels_GBps": round(step_bytes / (avg(step_ms) * 1e-3) / 1e9, 1),
               "source_digest": b["roofline"].get("source_digest"), "commit": commit,
               "note": "trace times are the kernels of bench.py's timed steps (warmup steps excluded); "
                       "bench.py's achieved brackets each s3dg_* call with HIP events on the launch stream"}
        json.dump(out, open(os.path.join(dst, f"timing_cfg{c}.json"), "w"), indent=1)
        print(json.dumps(out))
        ent = {"kernel": names, "workload": b["config"]["workload"],
               "algorithmic_bytes_per_launch": b["roofline"]["algorithmic_bytes_per_launch"],
               "source_digest": digest, "commit": commit}
        for ctr, scale in (("WRITE_SIZE", 1024), ("FETCH_SIZE", 2048)):
            p = os.path.join(src, f"pmc_{ctr}_cfg{c}", "run_counter_collection.csv")
            if not os.path.exists(p):
                break
            pb = bench_line(os.path.join(src, f"bench_pmc_{ctr}_cfg{c}.log"))
            rr = [r for r in csv.DictReader(open(p)) if is_step(r["Kernel_Name"])]
            with open(os.path.join(dst, f"pmc_{ctr.lower()}_cfg{c}.csv"), "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=list(rr[0].keys()))
                w.writeheader()
                w.writerows(rr)
            # the PMC run is bench --steps 1 --warmup 0: one step = step bytes / bytes per launch launches
            total = sum(float(r["Counter_Value"]) for r in rr) * scale
            launches = (pb["config"]["bytes_per_step_all_ranks"] // pb["n_gpus"]) / pb["roofline"][
                "algorithmic_bytes_per_launch"]
            ent[f"{ctr.lower()}_bytes_per_launch"] = int(round(total / launches))
        else:
            ent["traffic_bytes_per_launch"] = ent["write_size_bytes_per_launch"] + ent["fetch_size_bytes_per_launch"]
            ent["traffic_over_algorithmic"] = round(ent["traffic_bytes_per_launch"]
                                                    / ent["algorithmic_bytes_per_launch"], 5)
            ent["method"] = ("rocprofv3 --pmc WRITE_SIZE and --pmc FETCH_SIZE in separate passes (no tracing "
                             "domains) over bench.py --steps 1 --warmup 0, summed over the step's kernels and "
                             "divided by its launches; WRITE_SIZE x 1024 B; FETCH_SIZE x 1024 x 2 (gfx950 "
                             "half-count correction, MI355X_MICROARCH.md)")
            ent["sources"] = [f"profiles/{rnd}/pmc_write_size_cfg{c}.csv", f"profiles/{rnd}/pmc_fetch_size_cfg{c}.csv"]
            traffic[str(c)] = ent
    json.dump(traffic, open(tpath, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
