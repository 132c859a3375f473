"""Per-call GEMM variant sweep over the GEMMs of one real CQL update.

Records every ops.gemm call enqueued by one eager K2 update (shapes, strides,
pointers into the live workspace), then re-issues each call with every tile
variant and prints the median time per (call, variant).  The buffers stay
alive in the implementation's workspace, so re-issuing only overwrites
scratch values.

    python tools/gemm_pipeline_sweep.py [--algo cql|td3bc]
"""
import argparse
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from d3rlpy_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="cql")
    ap.add_argument("--variants", default="0,2,3,6,7,8,9,10")
    args = ap.parse_args()
    sys.path.insert(0, "tests")
    from cql_helpers import HostBatch  # noqa: E402
    D, A, B = 11, 3, 256
    rs = np.random.RandomState(0)
    hb = HostBatch(rs.randn(B, D).astype(np.float32), rs.uniform(-1, 1, (B, A)).astype(np.float32),
                   rs.randn(B).astype(np.float32), rs.randn(B, D).astype(np.float32),
                   np.zeros(B, np.float32), np.ones(B, np.float32))
    if args.algo == "cql":
        from cql_helpers import make_impl
        impl = make_impl(D, A, [256, 256], 10)
    else:
        from td3_helpers import make_td3_impl
        impl = make_td3_impl(D, A, [256, 256])
    calls = []
    orig = ops.gemm

    def rec(*a, **k):
        calls.append((a, k))
        return orig(*a, **k)

    ops.gemm = rec
    impl.update_step(hb, use_graph=False)
    ops.gemm = orig
    torch.cuda.synchronize()
    variants = [int(v) for v in args.variants.split(",")]
    s = torch.cuda.current_stream()
    total_auto, total_best = 0.0, 0.0
    reps = 20
    for i, (a, k) in enumerate(calls):
        M, Nn, K = a[3], a[4], a[5]
        times = {}
        for v in [-1] + variants:
            kk = dict(k, variant=v)
            orig(*a, **kk)
            torch.cuda.synchronize()
            # graph-captured repetitions: kernel time without host launch cost
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(reps):
                    orig(*a, **kk)
            ts = []
            for _ in range(5):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                g.replay()
                e1.record(s)
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / reps)  # us per call
            times[v] = sorted(ts)[2]
        best = min(variants, key=lambda v: times[v])
        total_auto += times[-1]
        total_best += times[best]
        desc = (f"#{i:02d} M={M} N={Nn} K={K} b={k.get('batch', 1)} s={k.get('splits', 1)} "
                f"sA={tuple(k['sA'])} sB={tuple(k['sB'])} mask={k.get('mask') is not None} "
                f"rowsum={k.get('rowsum') is not None}")
        print(desc, f"auto={times[-1]:.1f}us best=v{best}:{times[best]:.1f}us |",
              " ".join(f"v{v}:{times[v]:.1f}" for v in variants), flush=True)
    print(f"total auto={total_auto:.1f}us best={total_best:.1f}us")


if __name__ == "__main__":
    main()
