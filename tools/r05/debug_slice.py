"""Repeat the slice backward and report run-to-run differences per output."""
import sys
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_gpu_x6t import run_slice  # noqa: E402
from test_gpu_x6 import NAMES  # noqa: E402
from d3rlpy_amd import ops  # noqa: E402

for rows, n_in in ((7936, 14), (7936, 20), (7936, 37), (1056, 37)):
    outs, ref, d = run_slice(rows, n_in, rows - 256, 2, 5)
    first = [o.clone() for o in outs]
    for rep in range(5):
        ops.call_desc("d3a_q2_bwd_x6", d)
        torch.cuda.synchronize()
        for name, a, b in zip(NAMES, first, outs):
            if not torch.equal(a, b):
                diff = (a - b).abs()
                idx = (diff > 0).nonzero()
                print(rows, n_in, rep, name, "ndiff", idx.shape[0], "max", float(diff.max()),
                      "first idx", idx[:4].tolist())
        ref_dW1 = ref["dW1"][0].cpu()
        got = outs[0].double().sum(0).cpu()
        print(rows, n_in, rep, "dW1 err vs fp64", float((got - ref_dW1).abs().max() / ref_dW1.abs().max()))
