"""Fixed cost of one kernel launch inside a replayed HIP graph on this box:
a graph of K back-to-back tiny kernels (256-element adds, and one 256-block
grid of them), replay time / K."""
import json
import torch

dev = torch.device("cuda:0")
res = {}
for name, n in (("tiny_1wg", 256), ("tiny_64wg", 256 * 64), ("tiny_1024wg", 256 * 1024)):
    x = torch.zeros(n, device=dev)
    K = 64
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(K):
            x.add_(1.0)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 200
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    res[name] = round(e0.elapsed_time(e1) * 1e3 / (reps * K), 3)
print(json.dumps({"us_per_launch_in_graph": res}))
