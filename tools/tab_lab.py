#!/usr/bin/env python3
"""Tabulate a lab log's JSON lines: rows = one key (default "setting"),
columns = another ("point"), cells = a value ("frac").
    python tools/tab_lab.py LOG [row_key col_key value_key]
Tooling only."""
import json, sys

log = sys.argv[1]
rk, ck, vk = (sys.argv[2:5] + ["setting", "point", "frac"][len(sys.argv[2:5]):])[:3]
rows = [json.loads(l) for l in open(log) if l.startswith("{") and f'"{rk}"' in l and f'"{vk}"' in l]
cols, names = [], []
for r in rows:
    if r[ck] not in cols:
        cols.append(r[ck])
    if r[rk] not in names:
        names.append(r[rk])
w = max(10, max(len(str(c)) for c in cols) + 1)
print(rk.ljust(12) + "".join(str(c).ljust(w) for c in cols))
for n in names:
    cells = []
    for c in cols:
        v = [r[vk] for r in rows if r[rk] == n and r[ck] == c]
        cells.append(str(v[0]) if v else "-")
    print(str(n).ljust(12) + "".join(x.ljust(w) for x in cells))
