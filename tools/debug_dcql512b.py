"""Debug: is the K5 second-step conv0 gradient error workspace state or params?"""
import copy
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from arbiter_helpers import hip_grads, max_rel, module_grads  # noqa: E402
from oracle.discrete_cql import DiscreteCQLIQNOracle, IQNTaus  # noqa: E402
from test_gpu_arbiters import _dcql_batch  # noqa: E402
from test_gpu_discrete_cql import OBS, TAU_KEYS, make_impl, oracle_state  # noqa: E402

torch.set_num_threads(16)
A, K = 4, 64
pre = "_q_funcs.0."
for B in (64, 512):
    orc = DiscreteCQLIQNOracle(OBS, A, seed=6)
    impl = make_impl(A)
    rs = np.random.RandomState(13)
    gen = torch.Generator().manual_seed(14)
    for step in range(3):
        (pb, hb), taus = _dcql_batch(rs, B, A), IQNTaus.draw(gen, B, K)
        tk = {k: getattr(taus, k).numpy() for k in TAU_KEYS}
        sd = copy.deepcopy(oracle_state(orc))
        impl.set_state_dict(sd)
        fresh = make_impl(A)
        fresh.set_state_dict(sd)
        orc.update(pb, taus)
        g32 = {pre + k: v for k, v in module_grads(orc._q_func).items()}
        impl.update_step(hb, taus=tk)
        fresh.update_step(hb, taus=tk)
        torch.cuda.synchronize()
        for name, im in (("reused", impl), ("fresh", fresh)):
            gh = hip_grads(im._refs(), im.grad)
            errs = {k.split("_encoder.")[-1]: max_rel(gh[k], g32[k]) for k in g32}
            print(f"B={B} step={step} {name}: " + " ".join(f"{k}={v:.1e}" for k, v in errs.items()))
        # second call on the same impl with the same state and data: repeatable?
        fresh.set_state_dict(sd)
        fresh.update_step(hb, taus=tk)
        torch.cuda.synchronize()
        g2 = hip_grads(fresh._refs(), fresh.grad)
        gh = hip_grads(impl._refs(), impl.grad)
        print(f"B={B} step={step} fresh-2nd-call vs reused: "
              f"{max(max_rel(g2[k], gh[k]) for k in gh):.1e}")
