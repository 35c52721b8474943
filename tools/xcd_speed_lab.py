#!/usr/bin/env python3
"""Are the keystream's slow XCDs (queues 1/3/5/7) slow at
arithmetic or at stores?  tools/xcd_speed_lab.hip: 1024 one-wave workgroups
(four per CU, as the keystream; dynamic LDS caps residency at four) run
(a) register-only Xoshiro steps, (b) contiguous 1 KiB stores, (c) the
keystream's 64-lane-region store pattern, (d) the fill's pattern (each XCD on
every 8th 4 KiB granule), each wave timing itself and
recording its XCC.  Per kernel: mean wave duration per XCC, odd/even ratio.

    python tools/xcd_speed_lab.py --build    # here
    python tools/xcd_speed_lab.py            # GPU box
Tooling only: nothing in the product imports this."""
import ctypes, json, os, statistics, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tools", "_build")
LIB = os.path.join(OUT, "libxcdspeed.so")
MiB = 1 << 20


def build():
    os.makedirs(OUT, exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-o", LIB, os.path.join(ROOT, "tools", "xcd_speed_lab.hip")])


def main():
    if "--build" in sys.argv:
        build()
        return
    import torch
    L = ctypes.CDLL(LIB)
    u32, u64, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
    L.lab_valu.argtypes = [vp, vp, u32, u32, vp]
    L.lab_store_seq.argtypes = [vp, vp, u32, u64, u32, u32, vp]
    L.lab_store_lanes.argtypes = [vp, vp, u32, u32, u32, u32, vp]
    L.lab_store_xcd.argtypes = [vp, vp, u32, u32, u32, vp]
    L.lab_store_lanes_paced.argtypes = [vp, vp, u32, u32, u32, u32, u32, vp]
    L.lab_store_window.argtypes = [vp, vp, u32, u64, u32, u32, vp]
    L.lab_store_granule.argtypes = [vp, vp, u32, u32, vp]
    L.lab_store_lanes_wait.argtypes = [vp, vp, u32, u32, u32, u32, u32, vp]
    L.lab_store_granule_work.argtypes = [vp, vp, vp, u32, u32, u32, u32, vp]
    L.lab_store_lanes_load.argtypes = [vp, vp, vp, u32, u32, u32, u32, vp]
    L.lab_store_lanes_rnd.argtypes = [vp, vp, u32, u32, u32, u32, vp]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    span = 16384               # 16 KiB lane regions (the keystream's 2048 draws)
    need = 8 * 4 * cus * 64 * span
    buf = torch.empty(need, dtype=torch.uint8, device="cuda")
    out = torch.zeros(3 * 32 * cus, dtype=torch.int64, device="cuda")
    sink = torch.zeros(32 * cus, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream()
    sh = vp(st.cuda_stream)
    kinds = {"valu": lambda: L.lab_valu(vp(out.data_ptr()), vp(sink.data_ptr()), 4 * cus, 200000, sh)}
    # LAB_WPC: waves (1-wave workgroups) per CU for the store kernels, capped by
    # dynamic LDS; the same bytes at every residency (units = 32 / wpc)
    for wpc in [int(x) for x in os.environ.get("LAB_WPC", "4").split(",")]:
        grid, units, lds = wpc * cus, 32 // wpc, (160 // wpc) * 1024
        sfx = "" if wpc == 4 else f"_{wpc}pcu"
        kinds["store_seq" + sfx] = (lambda grid=grid, units=units, lds=lds: L.lab_store_seq(
            vp(buf.data_ptr()), vp(out.data_ptr()), grid, 64 * span, units, lds, sh))
        kinds["store_lanes" + sfx] = (lambda grid=grid, units=units, lds=lds: L.lab_store_lanes(
            vp(buf.data_ptr()), vp(out.data_ptr()), grid, span, units, lds, sh))
        kinds["store_xcd" + sfx] = (lambda grid=grid, units=units, lds=lds: L.lab_store_xcd(
            vp(buf.data_ptr()), vp(out.data_ptr()), grid, units, lds, sh))
        for wn in [int(x) for x in os.environ.get("LAB_WNAP", "0").split(",")]:
            kinds["store_window" + sfx + (f"_nap{wn}" if wn else "")] = (lambda grid=grid, lds=lds, wn=wn: L.lab_store_window(
                vp(buf.data_ptr()), vp(out.data_ptr()), grid, need // 4096, wn, lds, sh))
        kinds["store_lanes_rnd" + sfx] = (lambda grid=grid, units=units, lds=lds: L.lab_store_lanes_rnd(
            vp(buf.data_ptr()), vp(out.data_ptr()), grid, span, units, lds, sh))
    # LAB_SHORT: the lane pattern as one unit per workgroup over a grid of many
    # (lane region bytes per entry), like the keystream's static grid / the
    # fill's short workgroups, four resident per CU
    short = [int(x) for x in os.environ.get("LAB_SHORT", "").split(",") if x]
    if short:
        out = torch.zeros(3 * (need // (64 * min(short))), dtype=torch.int64, device="cuda")
    for sp in short:
        g = need // (64 * sp)
        kinds[f"store_lanes_short_{sp // 1024}k"] = (lambda g=g, sp=sp: L.lab_store_lanes(
            vp(buf.data_ptr()), vp(out.data_ptr()), g, sp, 1, 40 * 1024, sh))
    # LAB_NAP: the lane pattern (4 per CU) with s_sleep(1) x nap after each 32-store burst
    for nap in [int(x) for x in os.environ.get("LAB_NAP", "").split(",") if x]:
        kinds[f"store_lanes_nap{nap}"] = (lambda nap=nap: L.lab_store_lanes_paced(
            vp(buf.data_ptr()), vp(out.data_ptr()), 4 * cus, span, 8, nap, 40 * 1024, sh))
    # LAB_WAIT: the lane pattern (4 per CU) with s_waitcnt vmcnt(N) after each burst
    for n in [int(x) for x in os.environ.get("LAB_WAIT", "").split(",") if x]:
        kinds[f"store_lanes_vmcnt{n}"] = (lambda n=n: L.lab_store_lanes_wait(
            vp(buf.data_ptr()), vp(out.data_ptr()), 4 * cus, span, 8, n, 40 * 1024, sh))
    # LAB_GRANULE: one granule per workgroup, resident workgroups per CU listed
    gran = [int(x) for x in os.environ.get("LAB_GRANULE", "").split(",") if x]
    if gran:
        out = torch.zeros(3 * (need // 4096), dtype=torch.int64, device="cuda")
    blk = torch.randint(0, 255, (4096,), dtype=torch.uint8, device="cuda")
    for wpc in [int(x) for x in os.environ.get("LAB_LLOAD", "").split(",") if x]:   # lane pattern + a read per burst
        kinds[f"store_lanes_load_{wpc}pcu"] = (lambda wpc=wpc: L.lab_store_lanes_load(
            vp(buf.data_ptr()), vp(out.data_ptr()), vp(blk.data_ptr()), wpc * cus, span, 32 // wpc, (160 // wpc) * 1024, sh))
    works = [tuple(int(y) for y in x.split("/")) for x in os.environ.get("LAB_GWORK", "").split(",") if x]
    for wpc in gran:
        kinds[f"store_granule_{wpc}pcu"] = (lambda wpc=wpc: L.lab_store_granule(
            vp(buf.data_ptr()), vp(out.data_ptr()), need // 4096, (160 // wpc) * 1024, sh))
        for work, load in works:   # LAB_GWORK "steps/load,...": VALU steps and the L2 block read before the stores
            kinds[f"store_granule_{wpc}pcu_w{work}_l{load}"] = (lambda wpc=wpc, work=work, load=load: L.lab_store_granule_work(
                vp(buf.data_ptr()), vp(out.data_ptr()), vp(blk.data_ptr()), need // 4096, work, load, (160 // wpc) * 1024, sh))
    res = {}
    for rep in range(int(os.environ.get("LAB_REPS", "5"))):
        for name, f in kinds.items():
            assert f() == 0
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            assert f() == 0
            e1.record(st)
            torch.cuda.synchronize()
            t = [r for r in out.view(-1, 3).cpu().tolist() if r[1] > 0]
            out.zero_()
            per, last = {}, {}
            t_first = min(r[0] for r in t)
            for s, e, x in t:
                per.setdefault(x, []).append((e - s) * 0.01)
                last[x] = max(last.get(x, 0), (e - t_first) * 0.01)
            res.setdefault(name, []).append((e0.elapsed_time(e1), {x: statistics.mean(v) for x, v in per.items()},
                                             {x: len(v) for x, v in per.items()}, last))
        print(f"rep {rep} done", flush=True)
    for name, v in res.items():
        xs = sorted(v[0][1])
        mean_x = {x: round(statistics.mean(r[1][x] for r in v), 2) for x in xs}
        odd = statistics.mean(mean_x[x] for x in xs if x % 2)
        even = statistics.mean(mean_x[x] for x in xs if x % 2 == 0)
        line = {"kernel": name, "event_ms": [round(r[0], 3) for r in v], "wave_us_mean_by_xcc": mean_x,
                "xcc_last_end_us": {x: round(statistics.mean(r[3][x] for r in v), 1) for x in xs},
                "waves_by_xcc": v[0][2], "odd_over_even": round(odd / even, 4)}
        if name != "valu":
            line["GBps"] = round(need / (statistics.median(r[0] for r in v) * 1e-3) / 1e9, 1)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
