#!/usr/bin/env python3
"""Diagnostic: bench.py's D2H-inclusive loop for config 2 and config 8 side by
side in one process, config 8 also with the 2D stream kernel generating
(s3dg_set_stream_tiles 0) and with the generation stream idle (copies only).
Tooling only."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from s3dlio_amd import Context, compress_ratio
    from s3dlio_amd._lib import call
    torch.cuda.set_device(0)
    ctx = Context(0, base_seed=bench.BASE_SEED)
    for rep in range(2):
        for name, c, tiles in (("cfg2", 2, -1), ("cfg8", 8, -1), ("cfg8_2d", 8, 0), ("cfg3", 3, -1)):
            ctx.set_stream_tiles(tiles)
            cfg = bench.CONFIGS[c]
            fn, fd = compress_ratio(cfg["compress"])
            d = bench.d2h_inclusive(torch, ctx, call, 0, cfg, fn, fd, 0)
            print(json.dumps({"rep": rep, "case": name, "GiBps": d["value"], "copies": d["copy_GiBps_min_med_max"],
                              "pages": d["ring_pages_per_node"]}), flush=True)
        ctx.set_stream_tiles(-1)


if __name__ == "__main__":
    main()
