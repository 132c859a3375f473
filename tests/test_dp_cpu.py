"""Data-parallel exchange on CPU, world size 2 over gloo.

Two processes each run the oracle CQL update on half of a global batch with
d3rlpy_amd.dp's gradient exchange before every optimiser step; the result
must equal one oracle update on the whole batch (every CQL loss is a batch
mean, and the temp / alpha / critic / actor exchanges sit where the HIP
pipeline puts them).  Losses are averaged over the ranks like the pipeline's
metric all-reduce.  Tolerance: fp32 summation order, 2e-6 on parameters.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle.cql import Batch, CQLNoise, CQLOracle

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_rows():
    from d3rlpy_amd.dp import shard_rows
    assert [shard_rows(2048, r, 8) for r in (0, 7)] == [slice(0, 256), slice(1792, 2048)]
    with pytest.raises(ValueError):
        shard_rows(100, 0, 3)


def test_gloo_two_ranks_equal_global_batch(tmp_path):
    D, A, H, N, B, S = 6, 2, 32, 3, 32, 3
    world = 2
    orc = CQLOracle(D, A, n_critics=2, n_action_samples=N, hidden_units=[H, H], seed=1)
    torch.save({k: getattr(orc, k).state_dict() for k in ("_q_func", "_targ_q_func", "_policy",
                                                          "_targ_policy", "_log_temp",
                                                          "_log_alpha")}, tmp_path / "init.pt")
    np.savez(tmp_path / "cfg.npz", cfg=np.array([D, A, H, N, B, S]))
    rs = np.random.RandomState(2)
    gen = torch.Generator().manual_seed(3)
    steps = []
    for s in range(S):
        arrs = (rs.randn(B, D).astype(np.float32), rs.uniform(-1, 1, (B, A)).astype(np.float32),
                rs.randn(B).astype(np.float32), rs.randn(B, D).astype(np.float32),
                (rs.rand(B) < 0.1).astype(np.float32), np.ones(B, np.float32))
        nz = CQLNoise.draw(gen, B, A, N)
        steps.append((arrs, nz))
        np.savez(tmp_path / f"step{s}.npz", obs=arrs[0], act=arrs[1], rew=arrs[2],
                 next_obs=arrs[3], term=arrs[4], n_steps=arrs[5],
                 **{f"noise/{k}": v.numpy() for k, v in nz.tensors().items()})
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", CUDA_VISIBLE_DEVICES="")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dp_cpu_worker.py"), str(r),
                               str(world), str(port), str(tmp_path)], env=env)
             for r in range(world)]
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=180))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(-9)
    assert rcs == [0] * world, rcs
    ref = []
    for arrs, nz in steps:
        m = orc.update(Batch.from_numpy(*arrs), nz)
        ref.append([m[k] for k in sorted(m)])
    dm = np.load(tmp_path / "dp_metrics.npy")
    assert np.allclose(dm, np.array(ref), rtol=2e-6, atol=2e-6), (dm, ref)
    sd = torch.load(tmp_path / "dp_state.pt", weights_only=True)
    worst = 0.0
    for k, d in sd.items():
        full = getattr(orc, k).state_dict()
        for n, t in d.items():
            worst = max(worst, float((t - full[n]).abs().max()))
    assert worst <= 2e-6, worst
