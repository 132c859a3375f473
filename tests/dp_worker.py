"""One rank of the data-parallel CQL parity test (tests/test_gpu_dp.py).

    python tests/dp_worker.py RANK WORLD PORT WORKDIR

Loads the initial state, the global batches and noise written by the test,
takes its shard of every batch (rows [rank*b, (rank+1)*b)) and of every
per-row noise tensor, runs the updates with gradients averaged over the
ranks (gloo on the GPU tensors; eager launches), and writes its final state.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def shard_noise(nz, sl, B, N, A):
    out = {}
    for k, v in nz.items():
        v = np.asarray(v)
        if k in ("eps_temp", "eps_actor"):
            out[k] = v[sl]
        elif k.endswith("_rand"):
            out[k] = v.reshape(B, N, A)[sl].reshape(-1, A)
        else:
            out[k] = v[:, sl]
    return out


def main():
    rank, world, port, work = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    from cql_helpers import HostBatch, make_impl
    from d3rlpy_amd.dp import DataParallel, shard_rows
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    torch.cuda.set_device(0)
    cfg = np.load(os.path.join(work, "cfg.npz"), allow_pickle=False)
    D, A, H, L, N, B, S = (int(x) for x in cfg["cfg"])
    impl = make_impl(D, A, [H] * L, N)
    impl.set_state_dict(torch.load(os.path.join(work, "init.pt"), weights_only=True))
    impl.enable_data_parallel(DataParallel())
    sl = shard_rows(B, rank, world)
    metrics = []
    for step in range(S):
        g = np.load(os.path.join(work, f"step{step}.npz"), allow_pickle=False)
        arrs = [g[k][sl] for k in ("obs", "act", "rew", "next_obs", "term", "n_steps")]
        nz = shard_noise({k[6:]: g[k] for k in g.files if k.startswith("noise/")}, sl, B, N, A)
        m = impl.update_step(HostBatch(*arrs), noise=nz)
        metrics.append([m[k] for k in sorted(m)])
    torch.cuda.synchronize()
    # the Philox key this rank's workspace draws its own noise with
    np.save(os.path.join(work, f"seed{rank}.npy"), np.array(impl._workspace(sl.stop - sl.start).seed))
    # this rank's ReLU decisions of the critic stage (the last step's kept
    # critic activations), for the decision-aware fp64 arbiter
    from relu_arbiter import hip_critic_masks
    torch.save(hip_critic_masks(impl._workspace(sl.stop - sl.start)),
               os.path.join(work, f"masks{rank}.pt"))
    if rank == 0:
        torch.save(impl.get_state_dict(), os.path.join(work, "dp_state.pt"))
        # the gradients the last Adam steps consumed: all-reduced SUM x 1/world
        sc = impl._dp.scale
        g = {}
        for key, refs, getter in (("_q_func", impl._critic_refs(), impl.critic_grad),
                                  ("_policy", impl._policy_refs(), impl.policy_grad)):
            for k, seg, member, sl in refs:
                t = getter(seg)[member]
                g[f"{key}/{k}"] = ((t if sl is None else t[sl]) * sc).detach().cpu().clone()
        torch.save(g, os.path.join(work, "dp_grads.pt"))
        np.save(os.path.join(work, "dp_metrics.npy"), np.array(metrics))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
