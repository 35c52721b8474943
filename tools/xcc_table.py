"""Per-XCC table from rocprofv3 counter CSVs of tools/xcc_pmc.py (pmcx passes):
one row per (dispatch >= 1 ms, base counter), the eight XCCs' values in
millions, with the dispatch's kernel, duration and clock (GRBM_GUI_ACTIVE of
the busiest XCC / duration) when the pass has it.

    python tools/xcc_table.py gpurun_out/<dir>/*pmcx*/run_counter_collection.csv
"""
import collections
import csv
import re
import sys


def main(paths):
    for path in paths:
        rows = list(csv.DictReader(open(path)))
        d = collections.defaultdict(lambda: collections.defaultdict(dict))
        meta = {}
        for r in rows:
            m = re.match(r"X(\d)_(.*)", r["Counter_Name"])
            if not m:
                continue
            k = int(r["Dispatch_Id"])
            d[k][m.group(2)][int(m.group(1))] = float(r["Counter_Value"])
            name = r["Kernel_Name"]
            short = "k_fill_batch" if "k_fill_batch" in name else "k_keystream" if "k_keystream" in name else name[:24]
            meta[k] = (short, int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        print(f"# {path}")
        for k in sorted(d):
            short, ns = meta[k]
            if ns < 1_000_000:
                continue
            gui = d[k].get("GRBM_GUI_ACTIVE")
            clk = f" clock {max(gui.values()) / ns:.3f} GHz" if gui else ""
            print(f"dispatch {k} {short} {ns / 1e6:.3f} ms{clk}")
            for ctr, v in sorted(d[k].items()):
                vals = [v.get(x, 0.0) / 1e6 for x in range(8)]
                ev, od = sum(vals[0::2]) / 4, sum(vals[1::2]) / 4
                print(f"  {ctr:34s} " + " ".join(f"{x:8.2f}" for x in vals) +
                      f" | even {ev:8.2f} odd {od:8.2f} odd/even {od / ev if ev else 0:.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
