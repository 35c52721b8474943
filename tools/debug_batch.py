import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, s3dlio_amd as S
ctx = S.Context(0)
for waves in (1, 2, 4):
    for nobj, osz in [(2, 2**29), (7, 5 * 2**29 + 100), (1, 17 * 2**30)]:
        ctx.set_waves_per_block(waves)
        stride = (osz + 4095) // 4096 * 4096
        out = torch.empty(nobj * stride, dtype=torch.uint8, device="cuda")
        objs = [(k * stride, osz, k, 2, 2) for k in range(nobj)]
        try:
            ctx.fill_batch(out, objs); torch.cuda.synchronize(); print("ok", waves, nobj, osz)
        except Exception as e:
            print("FAIL", waves, nobj, osz, e)
        del out
