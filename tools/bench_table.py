#!/usr/bin/env python3
"""One table row per bench.py JSON line found in the given logs:
config, value GiB/s, kernel GB/s, frac, traffic ratio, launch-time
distribution (mean / p10 / p90, slow share), D2H-incl., CPU port.
    python tools/bench_table.py gpurun_out/<dir>/*.log
Tooling only."""
import json, sys

for path in sys.argv[1:]:
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        r = d.get("roofline") or {}
        dist = r.get("launch_ms_distribution") or {}
        tr = r.get("traffic")
        algo = r.get("algorithmic_bytes_per_launch") or 0
        cpu = d.get("cpu_baseline") or {}
        d2h = d.get("d2h_inclusive") or {}
        print(" | ".join(str(x) for x in [
            path.split("/")[-1], d["config"]["workload"][:70], d["value"], r.get("achieved"), r.get("frac"),
            round(tr / algo, 5) if tr and algo else None,
            f'{dist.get("mean")}/{dist.get("p10")}/{dist.get("p90")} slow {dist.get("slow_share_rate_below_p90_over_1.06")}',
            d2h.get("whole_job_GiBps") or d2h.get("value"), cpu.get("value"), d.get("verified_vs_oracle"),
            r.get("library_digest")]))
