"""One rank of the CPU (gloo) data-parallel check (tests/test_dp_cpu.py).

    python tests/dp_cpu_worker.py RANK WORLD PORT WORKDIR

The oracle CQL update on this rank's shard of the global batch, with every
optimiser step preceded by d3rlpy_amd.dp.DataParallel's SUM all-reduce of the
gradients scaled by 1/world — the exchange the HIP pipeline performs
(scalar temp/alpha gradients, critic, actor), here on CPU tensors.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def main():
    rank, world, port, work = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    from dp_worker import shard_noise
    from d3rlpy_amd.dp import DataParallel, shard_rows
    from oracle.cql import Batch, CQLNoise, CQLOracle
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    dp = DataParallel()
    cfg = np.load(os.path.join(work, "cfg.npz"), allow_pickle=False)
    D, A, H, N, B, S = (int(x) for x in cfg["cfg"])
    orc = CQLOracle(D, A, n_critics=2, n_action_samples=N, hidden_units=[H, H], seed=0)
    for k, sd in torch.load(os.path.join(work, "init.pt"), weights_only=True).items():
        getattr(orc, k).load_state_dict(sd)

    def wrap(opt):
        step = opt.step

        def synced_step(*a, **k):
            for grp in opt.param_groups:
                for p in grp["params"]:
                    dp.all_reduce_sum(p.grad)
                    p.grad.mul_(dp.scale)
            return step(*a, **k)
        opt.step = synced_step

    for o in (orc._critic_optim, orc._actor_optim, orc._temp_optim, orc._alpha_optim):
        wrap(o)
    sl = shard_rows(B, rank, world)
    out = []
    for step in range(S):
        g = np.load(os.path.join(work, f"step{step}.npz"), allow_pickle=False)
        arrs = [g[k][sl] for k in ("obs", "act", "rew", "next_obs", "term", "n_steps")]
        nz = shard_noise({k[6:]: g[k] for k in g.files if k.startswith("noise/")}, sl, B, N, A)
        m = orc.update(Batch.from_numpy(*arrs), CQLNoise(**{k: torch.from_numpy(v)
                                                             for k, v in nz.items()}))
        t = torch.tensor([m[k] for k in sorted(m)], dtype=torch.float64)
        dp.all_reduce_sum(t)
        out.append((t * dp.scale).numpy())
    if rank == 0:
        torch.save({k: getattr(orc, k).state_dict() for k in ("_q_func", "_policy", "_log_temp",
                                                              "_log_alpha")},
                   os.path.join(work, "dp_state.pt"))
        np.save(os.path.join(work, "dp_metrics.npy"), np.array(out))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
