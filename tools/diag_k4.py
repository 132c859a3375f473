"""Diagnostic: HIP vs oracle critic gradients at K4 shapes for B = 256 / 512,
state flowing impl -> oracle (as the DP test) and oracle -> impl (as parity)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from cql_helpers import HostBatch, make_batch, make_impl, make_oracle, max_rel, noise_dict, oracle_state
from oracle.cql import Batch, CQLNoise
from test_gpu_cql_parity import _oracle_step

D, A, H, N = 29, 8, [256, 256], 10
for B in (256, 512):
    for direction in ("impl->orc", "orc->impl"):
        impl = make_impl(D, A, H, N)
        orc = make_oracle(D, A, H, N, seed=0)
        if direction == "impl->orc":
            for k, v in impl.get_state_dict().items():
                getattr(orc, k).load_state_dict(v)
        else:
            impl.set_state_dict(oracle_state(orc))
        rs = np.random.RandomState(5)
        gen = torch.Generator().manual_seed(6)
        arrs = make_batch(rs, B, D, A)
        nzo = CQLNoise.draw(gen, B, A, N)
        m_orc, cgrads, pgrads = _oracle_step(orc, Batch.from_numpy(*arrs), nzo, A)
        m = impl.update_step(HostBatch(*arrs), noise=noise_dict(nzo))
        torch.cuda.synchronize()
        errs = []
        for c in range(2):
            for l in range(3):
                errs.append(f"c{c}W{l}={max_rel(impl.critic_grad(impl.critic.wname(l))[c], cgrads[c][l][0]):.1e}")
        print(B, direction, " ".join(errs), "critic_loss", m["critic_loss"], m_orc["critic_loss"], flush=True)
