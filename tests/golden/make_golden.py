"""Generate the committed golden fixtures from the oracle (CPU restatement).

    python tests/golden/make_golden.py

Writes small .npz files: every input (initial state in the reference
checkpoint layout, minibatch, injected noise) and every output of one
update (metrics, reduced gradients, post-step state).  The reference itself
could not be run here, so these vectors come from the oracle,
which is pinned by the reference's KATs (tests/test_oracle_kats.py).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.cql import Batch, CQLNoise, CQLOracle  # noqa: E402
from oracle import gather as og  # noqa: E402
from oracle.td3bc import StandardScalerT, TD3PlusBCOracle  # noqa: E402

STATE_KEYS = ("_q_func", "_targ_q_func", "_policy", "_targ_policy", "_log_temp", "_log_alpha")


def flat_state(orc, prefix):
    out = {}
    for k in STATE_KEYS:
        for n, t in getattr(orc, k).state_dict().items():
            out[f"{prefix}{k}/{n}"] = t.detach().numpy().copy()
    return out


def cql_small():
    D, A, H, N, B = 5, 2, [32, 32], 3, 16
    orc = CQLOracle(D, A, n_critics=2, n_action_samples=N, hidden_units=H, seed=123)
    rs = np.random.RandomState(7)
    obs = rs.randn(B, D).astype(np.float32)
    act = rs.uniform(-1, 1, (B, A)).astype(np.float32)
    rew = rs.randn(B).astype(np.float32)
    nobs = rs.randn(B, D).astype(np.float32)
    term = (rs.rand(B) < 0.2).astype(np.float32)
    nst = np.ones(B, dtype=np.float32)
    nz = CQLNoise.draw(torch.Generator().manual_seed(7), B, A, N)
    data = {"cfg": np.array([D, A, H[0], len(H), N, B], dtype=np.int64),
            "obs": obs, "act": act, "rew": rew, "next_obs": nobs, "term": term, "n_steps": nst}
    data.update(flat_state(orc, "init/"))
    for k in nz.tensors():
        data[f"noise/{k}"] = getattr(nz, k).numpy()
    batch = Batch.from_numpy(obs, act, rew, nobs, term, nst)
    tl, t = orc.update_temp(batch, nz.eps_temp)
    al, a = orc.update_alpha(batch, nz)
    cl = orc.update_critic(batch, nz)
    for c, qf in enumerate(orc._q_func.q_funcs):
        for n, p in qf.named_parameters():
            data[f"grad/_q_funcs.{c}.{n}"] = p.grad.numpy().copy()
    actl = orc.update_actor(batch, nz.eps_actor)
    for n, p in orc._policy.named_parameters():
        data[f"grad/policy.{n}"] = p.grad.numpy().copy()
    orc.update_critic_target()
    orc.update_actor_target()
    data["metrics"] = np.array([tl, t, al, a, cl, actl], dtype=np.float32)
    data.update(flat_state(orc, "final/"))
    np.savez_compressed(os.path.join(HERE, "cql_small.npz"), **data)


TD3_KEYS = ("_q_func", "_targ_q_func", "_policy", "_targ_policy")


def td3bc_small():
    """Two TD3PlusBC._update steps (grad_step 0: critic + actor + targets;
    grad_step 1: critic only) with a standard scaler and n-step targets."""
    D, A, H, B = 6, 2, [32, 32], 16
    rs = np.random.RandomState(21)
    mean = rs.randn(D) * 0.5
    std = np.abs(rs.randn(D)) + 0.5
    orc = TD3PlusBCOracle(D, A, n_critics=2, hidden_units=H, scaler=StandardScalerT(mean, std),
                          seed=321)
    data = {"cfg": np.array([D, A, H[0], len(H), B], dtype=np.int64),
            "scaler_mean": mean, "scaler_std": std}
    for k in TD3_KEYS:
        for n, t in getattr(orc, k).state_dict().items():
            data[f"init/{k}/{n}"] = t.detach().numpy().copy()
    metrics = []
    for step in range(2):
        obs = (rs.randn(B, D) * 2).astype(np.float32)
        act = rs.uniform(-1, 1, (B, A)).astype(np.float32)
        rew = rs.randn(B).astype(np.float32)
        nobs = (rs.randn(B, D) * 2).astype(np.float32)
        term = (rs.rand(B) < 0.2).astype(np.float32)
        nst = rs.randint(1, 3, size=B).astype(np.float32)
        noise = torch.randn(B, A, generator=torch.Generator().manual_seed(30 + step))
        for k, v in (("obs", obs), ("act", act), ("rew", rew), ("next_obs", nobs),
                     ("term", term), ("n_steps", nst), ("noise", noise.numpy())):
            data[f"step{step}/{k}"] = v
        m = orc.update(Batch.from_numpy(obs, act, rew, nobs, term, nst), noise, grad_step=step)
        metrics.append([m["critic_loss"], m.get("actor_loss", np.nan)])
    data["metrics"] = np.array(metrics, dtype=np.float32)
    for k in TD3_KEYS:
        for n, t in getattr(orc, k).state_dict().items():
            data[f"final/{k}/{n}"] = t.detach().numpy().copy()
    np.savez_compressed(os.path.join(HERE, "td3bc_small.npz"), **data)


def gather_small():
    """Transitions of two episodes (one terminal, one not) gathered with the
    reference semantics: vector obs n_steps 1 and 3; image obs n_frames 4."""
    rs = np.random.RandomState(11)
    obs = rs.randn(12, 3).astype(np.float32)
    act = rs.randn(12, 2).astype(np.float32)
    rew = rs.randn(12).astype(np.float32)
    term = np.zeros(12, dtype=np.float32)
    ep_term = np.zeros(12, dtype=np.float32)
    term[6] = 1.0      # episode 0: rows 0..6, terminal
    ep_term[6] = 1.0
    ep_term[11] = 1.0  # episode 1: rows 7..11, timeout (not terminal)
    frames = rs.randint(0, 256, size=(12, 1, 6, 6), dtype=np.uint8)
    out = {"obs": obs, "act": act, "rew": rew, "term": term, "ep_term": ep_term,
           "frames": frames}
    trans_v, trans_i = [], []
    for (o, a, r, t), (f, _, _, _) in zip(og.to_episodes(obs, act, rew, term, ep_term),
                                          og.to_episodes(frames, act, rew, term, ep_term)):
        trans_v += og.to_transitions(o, a, r, t)
        trans_i += og.to_transitions(f, a, r, t)
    idx = np.array([0, 5, 6, 3, 7, 10, 9, 1], dtype=np.int64)
    out["idx"] = idx
    for ns in (1, 3):
        b = og.gather([trans_v[i] for i in idx], 1, ns, 0.99)
        for k, v in b.items():
            out[f"vec_n{ns}/{k}"] = v
    b = og.gather([trans_i[i] for i in idx], 4, 2, 0.99)
    for k, v in b.items():
        out[f"img_f4_n2/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "gather_small.npz"), **out)


if __name__ == "__main__":
    cql_small()
    gather_small()
    td3bc_small()
    print("golden fixtures written to", HERE)
