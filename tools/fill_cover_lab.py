#!/usr/bin/env python3
"""Does every live k_fill_batch workgroup write its block, exactly once?
(round 4's fill_xcd_lab saw 203 / 9 791 whole 64-block
tiles of configs 2 / 3+5 without an end stamp, identical per XCD and across
reps.)

A diagnostic copy of the library (sources copied to tools/_build/src_cover;
the product tree is not touched) counts, per 4 KiB granule of the buffer,
the live workgroups that reached the end of k_fill_batch (one vector atomic
add by thread 0), and logs every workgroup that took the early exit (its
slot, tile and the 16 record words it read) plus the last slot of each
launch.  Before each fill the buffer, with 64 MiB guards on both sides, is
poisoned with 0xA5, so afterwards:
  * granules whose count is 0 / > 1 (none / several workgroups ended there),
  * blocks still all 0xA5 (never written; impossible for generated data),
  * guard bytes changed (stores outside the buffer)
are counted, and the first few of each are named (granule, object, tile).
The first fill of each configuration is the process's first launch of it.

    python tools/fill_cover_lab.py --build    # here
    python tools/fill_cover_lab.py            # GPU box
Tooling only: nothing in the product imports this."""
import ctypes, json, os, shutil, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_build")
SRC = os.path.join(OUT, "src_cover")
LIB = os.path.join(OUT, "libfillcover.so")
MiB = 1 << 20
GUARD = 64 * MiB
POISON = 0xA5
NLOG = 4096


def build():
    from s3dlio_amd.build import SOURCES, CSRC
    if os.path.isdir(SRC):
        shutil.rmtree(SRC)
    shutil.copytree(CSRC, os.path.join(SRC, "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(SRC, "include"))
    k = os.path.join(SRC, "csrc", "s3dg_kernels.hip")
    s = open(k).read()
    decl = ("__device__ unsigned int *g_cov;\n__device__ unsigned long long g_cov_n;\n"
            "__device__ unsigned long long *g_cov_exit;   // [0] count, [1] max slot, then NLOG x 18 words\n")
    anchor0 = "namespace s3dg {\n#if S3DG_KS_TRACE"
    assert s.count(anchor0) == 1
    s = s.replace(anchor0, "namespace s3dg {\n" + decl + "#if S3DG_KS_TRACE", 1)
    ex = "    if (ib < 0 || (uint64_t)ib * kBlk >= e.size) return;   // uniform for the whole workgroup\n"
    assert s.count(ex) == 1, "early exit not found"
    s = s.replace(ex, (
        "    if (t == 0 && g_cov_exit && blockIdx.x + 1 == gridDim.x) atomicMax(&g_cov_exit[1], (unsigned long long)g);\n"
        "    if (ib < 0 || (uint64_t)ib * kBlk >= e.size) {\n"
        "        if (t == 0 && g_cov_exit) {\n"
        "            const unsigned long long q = atomicAdd(&g_cov_exit[0], 1ull);\n"
        "            if (q < %d) {\n"
        "                unsigned long long *r = g_cov_exit + 2 + 18 * q;\n"
        "                r[0] = g; r[1] = tile;\n"
        "                for (int w = 0; w < 16; ++w) r[2 + w] = raw[w];\n"
        "            }\n"
        "        }\n"
        "        return;\n"
        "    }\n") % NLOG, 1)
    anchor = "\n}\n\n// Prefix parameters of one object on the device"
    assert s.count(anchor) == 1, "k_fill_batch end not found"
    s = s.replace(anchor, "\n    if (!ABL && t == 0 && g_cov) {\n"
                  "        const uint64_t gi = ((uint64_t)(bdst - dst_base) >> 12);\n"
                  "        if (gi < g_cov_n) atomicAdd(&g_cov[gi], 1u);\n"
                  "        else atomicAdd(&g_cov_exit[2 + 18 * %d], 1ull);   // out-of-range counter\n"
                  "    }" % NLOG + anchor, 1)
    s += ("\nextern \"C\" __attribute__((visibility(\"default\"))) int s3dg_diag_cover("
          "void *cnt, uint64_t n, void *exits) {\n"
          "    int r = (int)hipMemcpyToSymbol(HIP_SYMBOL(s3dg::g_cov_n), &n, sizeof(n));\n"
          "    if (r) return r;\n"
          "    r = (int)hipMemcpyToSymbol(HIP_SYMBOL(s3dg::g_cov_exit), &exits, sizeof(exits));\n"
          "    if (r) return r;\n"
          "    return (int)hipMemcpyToSymbol(HIP_SYMBOL(s3dg::g_cov), &cnt, sizeof(cnt));\n}\n")
    open(k, "w").write(s)
    srcs = [os.path.join(SRC, "csrc", os.path.basename(p)) for p in SOURCES]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-fvisibility=hidden", "-Wno-unused-function", "-mllvm", "-amdgpu-kernarg-preload-count=16",
           "-I", os.path.join(SRC, "include"), "-I", os.path.join(SRC, "csrc"), "-DS3DG_BUILD", "-o", LIB] + srcs
    subprocess.check_call(cmd)


def main():
    if "--build" in sys.argv:
        build()
        return
    import torch
    L = ctypes.CDLL(LIB, mode=os.RTLD_LOCAL)
    u64, u32 = ctypes.c_uint64, ctypes.c_uint32
    L.s3dg_diag_cover.argtypes = [ctypes.c_void_p, u64, ctypes.c_void_p]
    L.s3dg_fill_controlled_stream.argtypes = [ctypes.c_void_p] * 2 + [u64] * 4 + [u32] * 2 + [u64] * 2 + [
        ctypes.c_void_p]
    h = ctypes.c_void_p()
    assert L.s3dg_ctx_create(0, ctypes.byref(h)) == 0
    st = torch.cuda.current_stream()
    sh = ctypes.c_void_p(st.cuda_stream)
    n = int(os.environ.get("LAB_N", "10000"))
    size = 8 * MiB
    nblk = size * n // 4096
    whole = torch.empty(n * size + 2 * GUARD, dtype=torch.uint8, device="cuda")
    buf = whole[GUARD:GUARD + n * size]
    cnt = torch.zeros(nblk, dtype=torch.int32, device="cuda")
    exits = torch.zeros(2 + 18 * NLOG + 1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    print(json.dumps({"buf_granule_mod8": (buf.data_ptr() >> 12) & 7, "nblk": nblk}), flush=True)
    assert L.s3dg_diag_cover(ctypes.c_void_p(cnt.data_ptr()), u64(nblk), ctypes.c_void_p(exits.data_ptr())) == 0
    p = ctypes.c_void_p(buf.data_ptr())
    poison64 = int.from_bytes(bytes([POISON]) * 8, "little", signed=True)
    cases = {"cfg2 (d1 c1)": (1, 0, 1), "cfg3 (d4 c2)": (4, 1, 2), "cfg5 (d2 c3)": (2, 2, 3)}
    for rep in range(int(os.environ.get("LAB_REPS", "2"))):
        for name, (d, fn, fd) in cases.items():
            whole.fill_(POISON)
            cnt.zero_()
            exits.zero_()
            torch.cuda.synchronize()
            assert L.s3dg_fill_controlled_stream(h, p, u64(size), u64(size), u64(n), u64(d), u32(fn), u32(fd),
                                                 u64(0x5EED000000000001), u64(0), sh) == 0
            torch.cuda.synchronize()
            zero = torch.nonzero(cnt == 0).flatten()
            multi = torch.nonzero(cnt > 1).flatten()
            # blocks still entirely poison (never written), in 1 GiB pieces
            unwritten = []
            v = buf.view(torch.int64).view(nblk, 512)
            step = 262144
            for b0 in range(0, nblk, step):
                m = (v[b0:b0 + step] == poison64).all(dim=1)
                unwritten.append(torch.nonzero(m).flatten() + b0)
            unwritten = torch.cat(unwritten)
            guard_bad = int((whole[:GUARD] != POISON).sum().item() + (whole[GUARD + n * size:] != POISON).sum().item())
            ex = exits.cpu()
            nexit = int(ex[0])
            log = []
            for q in range(min(nexit, 8)):
                r = ex[2 + 18 * q: 2 + 18 * (q + 1)].tolist()
                words = [w & 0xFFFFFFFF for w in r[2:]]
                log.append({"slot": r[0], "tile": r[1], "dst_off": words[0] | words[1] << 32,
                            "size": words[2] | words[3] << 32, "first": words[6], "lead": words[7]})

            def name_g(t):
                t = t.cpu().tolist()
                return {"count": len(t), "first": [{"granule": x, "object": x // 2048, "tile": x // 64}
                                                  for x in t[:6]], "last": t[-1] if t else None}
            print(json.dumps({"case": name, "rep": rep, "granules_count0": name_g(zero),
                              "granules_count_gt1": name_g(multi), "blocks_unwritten": name_g(unwritten),
                              "unwritten_equals_count0": bool(torch.equal(unwritten, zero)),
                              "guard_bytes_changed": guard_bad, "early_exits": nexit, "exit_log": log,
                              "max_slot": int(ex[1]), "out_of_range_ends": int(ex[2 + 18 * NLOG])}), flush=True)


if __name__ == "__main__":
    main()
