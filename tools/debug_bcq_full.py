"""Debug: BCQ update_step leaves the imitator gradient buffer overwritten?"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from arbiter_helpers import hip_grads, max_rel  # noqa: E402
from cql_helpers import HostBatch  # noqa: E402
from test_gpu_arbiters import _bcq, _bcq_draws  # noqa: E402
from test_gpu_bcq_parity import _batch  # noqa: E402

impl, o32, _, (D, A, N) = _bcq(seed=9)
arrs = _batch(np.random.RandomState(10), 256, D, A)
nz, _, host = _bcq_draws(256, A, N, 11)
sd0 = impl.get_state_dict()
impl.update_step(HostBatch(*arrs), noise=host)
torch.cuda.synchronize()
full = {k: hip_grads(r(), g) for k, r, g in (("imi", impl._imitator_refs, impl.imitator_grad),
                                               ("q", impl._critic_refs, impl.critic_grad),
                                               ("pi", impl._policy_refs, impl.policy_grad))}
impl.set_state_dict(sd0)
stages = {}
for k, flags, r, g in (("imi", (True, False, False, False), impl._imitator_refs, impl.imitator_grad),
                       ("q", (False, True, False, False), impl._critic_refs, impl.critic_grad),
                       ("pi", (False, False, True, True), impl._policy_refs, impl.policy_grad)):
    impl._run(HostBatch(*arrs), flags, host, True, False)
    torch.cuda.synchronize()
    stages[k] = hip_grads(r(), g)
for k in full:
    print(k, max(max_rel(full[k][n], stages[k][n]) for n in full[k]))
