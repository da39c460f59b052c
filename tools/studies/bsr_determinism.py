import os, sys, json, torch
sys.path.insert(0, 'tools/studies'); sys.path.insert(0, '.')
import superbblas_amd as sb
from bsr_variants import op_and_vectors
dev = torch.device("cuda:0")
for dims, dtype in (((16,16,16,16), torch.complex128), ((8,8,8,8), torch.complex128), ((16,16,16,64), torch.complex64)):
    op, x, y, dimx, V, b = op_and_vectors(dims, 4, 3, 12, dtype, dev)
    px = [([0] * 8, dimx)]
    def f():
        sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx, [x],
                      0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])
    outs = []
    for k in range(4):
        y.zero_(); f(); torch.cuda.synchronize(); outs.append(y.clone())
    kern = sb.tune_get("bsr.last_kernel")
    sb.tune_set("bsr.variant", 2)
    y.zero_(); f(); torch.cuda.synchronize(); o2 = y.clone(); k2 = sb.tune_get("bsr.last_kernel")
    sb.tune_set("bsr.variant", 0)
    for k in range(1, 4):
        d = (outs[k] - outs[0]).abs()
        print(dims, "run", k, "vs 0: ndiff", int((d > 0).sum()), "maxdiff", float(d.max()), "kernel", kern, flush=True)
    d = (o2 - outs[0]).abs()
    print(dims, "variant 2 (kernel %d) vs 0: ndiff" % k2, int((d > 0).sum()), "rel", float(d.max() / outs[0].abs().max()), flush=True)
    op.destroy()
