"""Per-XCC write-path counters of the fill and the keystream in ONE process
(VERDICT r05 next #1a).  Run under rocprofv3 with the per-XCC derived
counters of tools/xcc_counters.yaml:

    rocprofv3 -E tools/xcc_counters.yaml --pmc X0_TCC_EA0_WRREQ ... -- python3 tools/xcc_pmc.py

Launches, interleaved, through the product library (s3dlio_amd): the fill
as config 2 (10 000 x 8 MiB, one k_fill_batch launch), K2 as config 6 (the
same bytes as 2 MiB Xoshiro256++ chunks, one persistent k_keystream launch)
and DG1 c1 as config 14 (one 8 GiB object per launch).  LAB_ROUNDS rounds
(default 2).  Bytes are not checked here (the product's own tests do)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MiB, GiB = 1 << 20, 1 << 30


def main():
    import torch
    from s3dlio_amd import Context, object_entropy
    from s3dlio_amd._lib import call
    dev = 0
    torch.cuda.set_device(dev)
    ctx = Context(dev, base_seed=0xBA5EB10C00000000)
    n, size = 10000, 8 * MiB
    ring = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    p = int(ring.data_ptr())
    sh = int(torch.cuda.current_stream().cuda_stream)
    sb = 0x5EED000000000001

    def fill():
        call("s3dg_fill_controlled_stream", ctx._h, p, size, size, n, 1, 0, 1, sb, 0, sh)

    def k2():
        call("s3dg_xoshiro_fill", ctx._h, p, n * size, 2 * MiB, 0, sh)

    def dg1():
        for j in range(2):
            call("s3dg_dgen_fill", ctx._h, p + j * 8 * GiB, 8 * GiB, 0, 1 << 40, 1, 0, 1,
                 object_entropy(sb, j), sh)
    for r in range(int(os.environ.get("LAB_ROUNDS", "2"))):
        for name, f in (("fill", fill), ("k2", k2), ("dg1", dg1)):
            f()
            torch.cuda.synchronize()
            print(f"round {r} {name} done", flush=True)
    print("xcc_pmc ok", flush=True)


if __name__ == "__main__":
    main()
