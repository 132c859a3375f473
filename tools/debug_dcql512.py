"""Debug: K5 B=512 second-step conv0 gradient disagreement (HIP vs oracle)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from arbiter_helpers import hip_grads, max_rel, module_grads, to_double  # noqa: E402
from oracle.discrete_cql import DiscreteCQLIQNOracle, IQNTaus  # noqa: E402
from test_gpu_arbiters import _dcql_batch  # noqa: E402
from test_gpu_discrete_cql import OBS, TAU_KEYS, make_impl, oracle_state  # noqa: E402

torch.set_num_threads(16)
A, K, B = 4, 64, 512
orc = DiscreteCQLIQNOracle(OBS, A, seed=6)
impl = make_impl(A)
rs = np.random.RandomState(13)
gen = torch.Generator().manual_seed(14)
batches = [(_dcql_batch(rs, B, A), IQNTaus.draw(gen, B, K)) for _ in range(2)]
pre = "_q_funcs.0."
for label, order in (("step0-data", [0]), ("step1-data-fresh", [1]), ("two-steps", [0, 1])):
    orc = DiscreteCQLIQNOracle(OBS, A, seed=6)
    impl = make_impl(A)
    for j, bi in enumerate(order):
        (pb, hb), taus = batches[bi]
        impl.set_state_dict(oracle_state(orc))
        sd = oracle_state(orc)
        o64 = DiscreteCQLIQNOracle(OBS, A, seed=6)
        to_double(o64, ("_q_func", "_targ_q_func"))
        o64._scale = lambda x: x.double() / 255.0
        o64._q_func.load_state_dict({k[len(pre):]: v for k, v in sd["_q_func"].items()})
        o64._targ_q_func.load_state_dict({k[len(pre):]: v for k, v in sd["_targ_q_func"].items()})
        taus64 = IQNTaus(*(getattr(taus, f).double() for f in taus.__dataclass_fields__))
        pb64 = type(pb)(pb.observations, pb.actions, pb.rewards.double(), pb.next_observations,
                        pb.terminals.double(), pb.n_steps.double())
        orc.update(pb, taus)
        o64.update(pb64, taus64)
        tk = {k: getattr(taus, k).numpy() for k in TAU_KEYS}
        m = impl.update_step(hb, taus=tk)
        torch.cuda.synchronize()
        gh = hip_grads(impl._refs(), impl.grad)
        # rerun HIP on the same state: deterministic?
        impl.set_state_dict(sd)
        impl.update_step(hb, taus=tk)
        torch.cuda.synchronize()
        gh2 = hip_grads(impl._refs(), impl.grad)
        g32 = {pre + k: v for k, v in module_grads(orc._q_func).items()}
        g64 = {pre + k: v for k, v in module_grads(o64._q_func).items()}
        for k in g64:
            print(f"{label} j={j} {k}: hip-32 {max_rel(gh[k], g32[k]):.1e} hip-64 "
                  f"{max_rel(gh[k], g64[k]):.1e} 32-64 {max_rel(g32[k], g64[k]):.1e} "
                  f"hip-rerun {max_rel(gh2[k], gh[k]):.1e}")
        # near-zero conv0 pre-activations (fp64)
        with torch.no_grad():
            x = pb64.observations.double() / 255.0
            z = torch.nn.functional.conv2d(x, o64._q_func._encoder._convs[0].weight.detach()
                                           if False else
                                           torch.as_tensor(sd["_q_func"][pre + "_encoder._convs.0.weight"]).double(),
                                           torch.as_tensor(sd["_q_func"][pre + "_encoder._convs.0.bias"]).double(),
                                           stride=4)
            print(f"{label} j={j}: conv0 pre-acts |z|<1e-6: {int((z.abs() < 1e-6).sum())}, "
                  f"<1e-5: {int((z.abs() < 1e-5).sum())} of {z.numel()}")
