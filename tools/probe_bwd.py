"""Timing probe: the fused forward kernel on a 256 -> 256 -> 1 problem over the
K2 critic-backward rows (what a fused backward-data kernel on transposed
weights would cost) against the current head1_bwd + input-gradient GEMM."""
import torch

from d3rlpy_amd import mlp
from d3rlpy_amd.nets import EnsembleMLP, GradSpace, ParamStore


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


dev = torch.device("cuda")
R, C = 7936, 2
for bm in (0, 64, 128):
    mlp._FUSED_BM = bm
    st = ParamStore()
    net = EnsembleMLP(st, "m", C, [256, 256, 1])
    st.allocate(dev)
    st.data.normal_(0, 0.05)
    x = torch.randn(C, R, 256, device=dev)
    acts = mlp.Acts.alloc(net, R, dev)
    us = timeit(lambda: mlp.forward(net, st, x.data_ptr(), False, 256, acts))
    print(f"fused fwd 256->256->1, {C}x{R} rows, bm={bm}: {us:.1f} us")
mlp._FUSED_BM = 0
st = ParamStore()
net = EnsembleMLP(st, "q", C, [16, 256, 256, 1])
st.allocate(dev)
st.data.normal_(0, 0.05)
x = torch.randn(R, 16, device=dev)
acts = mlp.Acts.alloc(net, R, dev)
mlp.forward(net, st, x.data_ptr(), True, 16, acts)
g = GradSpace(dev)
bs = mlp.BackwardSpace(net, R, g, dev)
dq = torch.randn(C, R, device=dev)
us = timeit(lambda: mlp.backward(bs, st, x.data_ptr(), True, 16, acts, dq.data_ptr(), 1, R, 0, R))
print(f"current critic backward (head1_bwd + GEMMs), {C}x{R} rows: {us:.1f} us")
us = timeit(lambda: mlp.backward(bs, st, x.data_ptr(), True, 16, acts, dq.data_ptr(), 1, R, 0, R,
                                 weight_grads=False))
print(f"current critic backward-data only: {us:.1f} us")
