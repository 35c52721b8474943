"""DESIGN.md §6 rows from final bench logs and the rocprof timing summaries
(tools/prof_summary.py output) of the same digest.
    python tools/design_table.py profiles/r06/final/bench profiles/r06
Tooling only."""
import glob
import json
import os
import sys


def lines(d):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "*.log"))):
        for l in open(f):
            if l.startswith("{"):
                out.append((os.path.basename(f), json.loads(l)))
    return out


def main(bench_dir, prof_dir):
    rows_dev, rows_host = [], []
    for name, d in lines(bench_dir):
        r = d["roofline"]
        cfg = d["config"]["workload"]
        c = d.get("cpu_baseline") or {}
        cpu = f'{c.get("value")} [{c["min_med_max_GiBps"][0]}–{c["min_med_max_GiBps"][2]}]' if c else "—"
        un = c.get("unpinned_min_med_max_GiBps")
        cpu += f' (unpinned {un[1]})' if un else ""
        if r.get("bound") == "pcie":
            rows_host.append(f'| {name} | {cfg} ({r.get("host_mem")}) | {d["value"]} | {round(r["avg_call_ms"] * 1e3, 1)} µs | {cpu} ({c.get("cores")}) |')
            continue
        dist = r.get("launch_ms_distribution") or {}
        tr, algo = r.get("traffic"), r.get("algorithmic_bytes_per_launch")
        d2h = d.get("d2h_inclusive") or {}
        d2hv = d2h.get("whole_job_GiBps") or d2h.get("value") or "—"
        rows_dev.append(f'| {name} | {cfg} | {d["value"]} | {r["achieved"]} | {round(100 * r["frac"], 1)} | '
                        f'{dist.get("mean")} / {dist.get("p10")} / {dist.get("p90")} ({dist.get("slow_share_rate_below_p90_over_1.06")}) | '
                        f'{round(tr / algo, 5) if tr and algo else "—"} | {d2hv} | {cpu} |')
    print("| Line | Workload | value GiB/s | Kernel GB/s (HIP events) | % of 8 TB/s | launch ms mean / p10 / p90 (slow share) | HBM traffic / algorithmic | D2H-incl. GiB/s | CPU port GiB/s [min–max] |")
    print("|---|---|---|---|---|---|---|---|---|")
    print("\n".join(rows_dev))
    print()
    print("| Line | Host-buffer workload | value GiB/s | per call | CPU port GiB/s [min–max] (threads) |")
    print("|---|---|---|---|---|")
    print("\n".join(rows_host))
    print()
    print("| Cfg | traced GB/s (fill kernels) | traced ms/step vs bench ms/step |")
    print("|---|---|---|")
    for f in sorted(glob.glob(os.path.join(prof_dir, "timing_cfg*.json")), key=lambda x: int(x.split("cfg")[-1][:-5])):
        t = json.load(open(f))
        print(f'| {t["config"]} | {t["trace_fill_GBps"]} | {t["timed_step_kernel_ms_avg"]} vs {t["bench_ms_per_step"]} |')


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
