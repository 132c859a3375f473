"""Do independent branches of a captured HIP graph run concurrently?

Captures 40 trivial launches (d3a_soft_update_f32 on 1024 floats) as one
chain, and as 2 / 4 independent chains forked onto side streams and joined;
prints the replay time of each (median of 7 x 50 replays).
"""
import sys

import torch

sys.path.insert(0, ".")
from d3rlpy_amd import ops  # noqa: E402


def capture(n_chains, n_total, bufs):
    main = torch.cuda.current_stream()
    side = [torch.cuda.Stream() for _ in range(n_chains - 1)]
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        fork = torch.cuda.Event()
        fork.record(cap)
        per = n_total // n_chains
        joins = []
        for c in range(n_chains):
            s = cap if c == 0 else side[c - 1]
            if c > 0:
                s.wait_event(fork)
            with torch.cuda.stream(s):
                for i in range(per):
                    t, u = bufs[c]
                    ops.soft_update(t, u, 0.5)
            if c > 0:
                e = torch.cuda.Event()
                e.record(s)
                joins.append(e)
        for e in joins:
            cap.wait_event(e)
    del main
    return g


def timeit(g, reps=50):
    s = torch.cuda.current_stream()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(ts)[3]


def main():
    dev = torch.device("cuda:0")
    bufs = [(torch.zeros(1024, device=dev), torch.ones(1024, device=dev)) for _ in range(4)]
    for chains in (1, 2, 4):
        g = capture(chains, 40, bufs)
        g.replay()
        torch.cuda.synchronize()
        print(f"40 launches as {chains} chain(s): {timeit(g):.1f} us per replay", flush=True)


if __name__ == "__main__":
    main()
