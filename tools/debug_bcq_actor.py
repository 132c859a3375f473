"""Compare the HIP BCQ actor-stage intermediates with the oracle (K3 shapes)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from cql_helpers import HostBatch, max_rel  # noqa: E402
from oracle.bcq import BCQNoise, BCQOracle  # noqa: E402
from oracle.cql import Batch  # noqa: E402
from test_gpu_bcq_parity import _batch, make_bcq_impl, oracle_state  # noqa: E402

D, A, H, N, K, B = 17, 6, [256, 256], 100, 200, 256
orc = BCQOracle(D, A, n_action_samples=N, n_quantiles=K, hidden_units=H, seed=3)
impl = make_bcq_impl(D, A, H, N, K)
impl.set_state_dict(oracle_state(orc))
arrs = _batch(np.random.RandomState(0), B, D, A)
nz = BCQNoise.draw(torch.Generator().manual_seed(1), B, A, N)
tb = Batch.from_numpy(*arrs)
orc.update_imitator(tb, nz.eps_vae)
orc.update_critic(tb, nz.z_target)
impl.update_step(HostBatch(*arrs), noise={k: getattr(nz, k).numpy() for k in
                                          ("eps_vae", "z_target", "z_actor")})
torch.cuda.synchronize()
ws = impl._workspace(B)
obs = tb.observations
lat = nz.z_actor.clamp(-0.5, 0.5)
a_dec = orc._imitator.decode(obs, lat).detach()
print("a_dec", max_rel(ws.a_dec_a.cpu(), a_dec), "max|a_dec|", float(a_dec.abs().max()))
pi_in = a_dec.clone()
h = orc._policy._encoder(obs, pi_in)
raw = orc._policy._fc(h)
print("pi raw", max_rel(ws.pa_acts.out[0].cpu(), raw.detach()))
act = orc._policy(obs, a_dec).detach().requires_grad_(True)
print("action", max_rel(ws.x_qa[:, D:D + A].cpu(), act.detach()))
q = orc._q_func.q_funcs[0](obs, act)
loss = -q.mean()
loss.backward()
print("dq/da", max_rel(ws.adx[0, :, D:].cpu(), act.grad))
pre = a_dec + 0.05 * torch.tanh(raw.detach())
print("pre near +-1:", int(((pre.abs() - 1).abs() < 1e-5).sum()), "clamped:", int((pre.abs() > 1).sum()))
r2 = raw.detach().clone().requires_grad_(True)
a2 = (a_dec + 0.05 * torch.tanh(r2)).clamp(-1, 1)
a2.backward(act.grad)
print("dhead_pi", max_rel(ws.dhead_pi.cpu(), r2.grad))
d = (ws.dhead_pi.cpu() - r2.grad).abs()
i = int(d.argmax())
print("worst elem", i // A, i % A, float(ws.dhead_pi.cpu().view(-1)[i]), float(r2.grad.view(-1)[i]),
      "pre", float(pre.view(-1)[i]))

# critic parameters after the critic step: HIP vs oracle
sd = impl.get_state_dict()
ref = orc._q_func.state_dict()
for k, t in ref.items():
    d = (sd["_q_func"][k] - t).abs()
    if float(d.max()) > 1e-6:
        j = int(d.argmax())
        print("critic param", k, "max diff", float(d.max()), "at", j,
              "hip grad", float(impl.critic_grad(
                  [r[1] for r in impl._critic_refs() if r[0] == k][0])[int(k.split('.')[1])]
                  .reshape(-1)[j]))
imp = orc._imitator.state_dict()
for k, t in imp.items():
    d = (sd["_imitator"][k] - t).abs()
    if float(d.max()) > 1e-6:
        print("imitator param", k, "max diff", float(d.max()))

# dQ0/da with the HIP critic parameters loaded into the oracle modules
orc._q_func.load_state_dict(sd["_q_func"])
act2 = orc._policy(obs, a_dec).detach().requires_grad_(True)
(-orc._q_func.q_funcs[0](obs, act2).mean()).backward()
print("dq/da with HIP critic params:", max_rel(ws.adx[0, :, D:].cpu(), act2.grad))
print("dq/da oracle-params vs HIP-params (oracle math):", max_rel(act.grad, act2.grad))
