#!/usr/bin/env python
"""Gradient-steps/sec of the CQL update on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): CQL on synthetic
hopper-medium-v0 shapes — obs 11, act 3, batch 256, n_critics 2,
n_action_samples 10, hidden [256, 256], reference defaults
(algos/cql.py:139-161) — over a 1M-transition synthetic D4RL-shaped dataset
resident in HBM (RandomState(0); 1000-step episodes, terminal on the last
step).  A "step" = one minibatch gather (device RandomIterator) + one full
CQL._update (temp, alpha, critic, actor, both target updates) — the inner
loop of fit() with per-step losses kept on device.

Multi-GPU: K2 does not shard: ``--gpus N`` runs N independent
learners (one per GPU, distinct seeds, "replicas"); value = steps completed
by all ranks / max-over-ranks wall time (weak scaling).  The ranks come from
torch.distributed.run (RANK / LOCAL_RANK / WORLD_SIZE in the environment) or,
when ``--gpus N > 1`` is given without them, from this script itself: the
parent starts N child processes with those variables set before anything
touches the GPU, waits for them, and relays rank 0's line (``launch_ranks``).

Prints ONE JSON line (rank 0) with roofline (dominant kernel: the critic
hidden-layer forward GEMM, fp32 MFMA) and cpu_baseline (the oracle's
op-for-op CPU restatement of the same update, timed on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


# the build round: PMC traffic files are read from profiles/r{ROUND}_*
ROUND = 6


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv, timeout: float = None) -> int:
    """Run this script as ``n`` ranks on one node (one process per GPU).

    The parent never initialises the GPU (it does not even import torch): it
    starts the children with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
    MASTER_PORT set, streams their stderr, relays rank 0's stdout, and
    returns the first non-zero exit status (the others are then stopped)."""
    import subprocess
    import threading
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv],
                                      env=env, stdout=subprocess.PIPE if r == 0 else
                                      subprocess.DEVNULL))

    def relay():
        for line in procs[0].stdout:
            sys.stdout.write(line.decode())
            sys.stdout.flush()

    t = threading.Thread(target=relay, daemon=True)
    t.start()
    rc = 0
    deadline = None if timeout is None else time.monotonic() + timeout
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is not None:
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
        if rc != 0 or (deadline is not None and time.monotonic() > deadline):
            rc = rc or 124
            for p in pending:
                p.kill()
            for p in pending:
                p.wait()
            break
        time.sleep(0.05)
    t.join(timeout=5)
    return rc


def _watchdog(seconds: float, what: str):
    """Exit this process with status 75 unless the returned event is set
    within ``seconds`` -- a rendezvous, RCCL initialisation or first graph
    capture that hangs (a rank that never joins, a wedged communicator) ends
    the job in bounded time with a non-zero status instead of at the driver's
    limit.  (os._exit: no exec, no cleanup that could block on the hung call.)"""
    import threading
    ev = threading.Event()

    def run():
        if not ev.wait(seconds):
            sys.stderr.write(f"bench: {what} did not finish within {seconds:.0f}s; exiting 75\n")
            sys.stderr.flush()
            os._exit(75)
    if seconds and seconds > 0:
        threading.Thread(target=run, daemon=True).start()
    return ev


def _dist_setup(backend: str = "nccl", timeout_s: float = 300.0):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import datetime
    tmo = datetime.timedelta(seconds=max(1.0, timeout_s))
    if backend == "gloo":  # launcher self-test: CPU only
        import torch.distributed as dist
        if ws > 1:
            dist.init_process_group("gloo", timeout=tmo)
        return ws, rank, local
    import torch
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"), timeout=tmo)
    else:
        torch.cuda.set_device(0)
    return ws, rank, local


def _barrier(ws):
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()


def _max_over_ranks(x: float, ws: int) -> float:
    if ws == 1:
        return x
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# workload per --algo: (dataset shape name, batch size, algo factory, description)
WORKLOADS = {
    "cql": ("hopper-medium-v0", 256,
            "CQL K2 (configs[1]): obs 11, act 3, batch 256, n_critics 2, n_action_samples 10, "
            "hidden [256,256], reference defaults"),
    "td3bc": ("pendulum-random", 100,
              "TD3+BC K1 (configs[0]) on 1xMI355X: obs 3, act 1, batch 100, n_critics 2, "
              "actor every 2 steps, standard scaler, hidden [256,256], reference defaults; "
              "runs on the GPU although BASELINE.json's K1 config names use_gpu=False (the "
              "reference's CPU plumbing): this build has no CPU compute path"),
    "bcq": ("halfcheetah-medium-v0", 256,
            "BCQ K3 (configs[2]): obs 17, act 6, batch 256, QR critics n_quantiles 200, "
            "n_critics 2, n_action_samples 100, hidden [256,256], reference defaults"),
    "cqldp": ("antmaze-umaze-v0", 256,
              "CQL K4 (configs[3]) data parallel: obs 29, act 8, 256 rows per GPU (global batch "
              "256 x n_gpus), n_critics 2, n_action_samples 10, hidden [256,256], reference "
              "defaults; per step three RCCL SUM all-reduces (scalar, critic, actor gradients) "
              "captured in the update graph"),
    "cqlrepro": ("hopper-medium-v0", 256,
                 "CQL reproduction (reproductions/offline/cql.py:21-37, hopper-medium-v0): obs 11, "
                 "act 3, batch 256, n_critics 2, n_action_samples 10, hidden [256,256,256], "
                 "alpha_learning_rate 0 (no update_alpha), conservative_weight 10"),
    "dcql": ("atari", 512,
             "DiscreteCQL K5 (configs[4]): 4x84x84 uint8 frame stacks (n_frames 4), IQN "
             "(64 quantiles, embed 64), batch 512, 4 actions, pixel scaler, Nature-DQN "
             "encoder, reference defaults"),
}


def _make_algo(name: str, batch: int, gpu: int = 0):
    """The workload's algorithm on GPU ``gpu`` (this rank's LOCAL_RANK)."""
    if name in ("cql", "cqldp"):
        from d3rlpy_amd.algos.cql import CQL
        return CQL(batch_size=batch, n_critics=2, n_action_samples=10, use_gpu=gpu)
    if name == "cqlrepro":
        from d3rlpy_amd.algos.cql import CQL
        from d3rlpy_amd.factories import VectorEncoderFactory
        enc = VectorEncoderFactory([256, 256, 256])
        return CQL(actor_learning_rate=1e-4, critic_learning_rate=3e-4, temp_learning_rate=1e-4,
                   actor_encoder_factory=enc, critic_encoder_factory=enc, batch_size=batch,
                   n_action_samples=10, alpha_learning_rate=0.0, conservative_weight=10.0,
                   use_gpu=gpu)
    if name == "dcql":
        from d3rlpy_amd.algos.cql import DiscreteCQL
        return DiscreteCQL(batch_size=batch, n_frames=4, q_func_factory="iqn", scaler="pixel",
                           use_gpu=gpu)
    if name == "bcq":
        from d3rlpy_amd.algos.bcq import BCQ
        from d3rlpy_amd.factories import QRQFunctionFactory
        return BCQ(batch_size=batch, q_func_factory=QRQFunctionFactory(n_quantiles=200),
                   use_gpu=gpu)
    from d3rlpy_amd.algos.td3_plus_bc import TD3PlusBC
    return TD3PlusBC(batch_size=batch, use_gpu=gpu)


def build_workload(rank: int, n_transitions: int, name: str = "cql", world: int = 1,
                   local: int = 0):
    from d3rlpy_amd.dataset import DeviceDataset
    from d3rlpy_amd.datasets import get_synthetic_d4rl
    from d3rlpy_amd.iterators import RandomIterator
    shape, batch, _ = WORKLOADS[name]
    if shape == "atari":
        from d3rlpy_amd.datasets import get_synthetic_atari
        ds = get_synthetic_atari(n_frames_total=n_transitions, action_size=4, seed=0)
    else:
        ds = get_synthetic_d4rl(shape, n=n_transitions, seed=0)
    import torch
    torch.manual_seed(rank)
    algo = _make_algo(name, batch, local)
    if algo.scaler is not None:
        algo.scaler.fit_dataset(ds)  # as fit() does before building the impl
    algo.build_with_dataset(ds)
    ddata = DeviceDataset(ds, device=f"cuda:{local}")
    assert algo.impl.device == f"cuda:{local}", (algo.impl.device, local)
    shard = (0, 1)
    seed = 1000 + rank
    if name == "cqldp" and world > 1:
        # K4: one global index stream (same seed on every rank), rank k
        # gathers rows [256k, 256k+256) of each global batch; gradients are
        # all-reduced inside the update graph (d3rlpy_amd/dp.py)
        from d3rlpy_amd.dp import DataParallel
        algo.impl.enable_data_parallel(DataParallel())
        shard, seed = (rank, world), 1000
    it = RandomIterator(ddata, n_steps_per_epoch=1 << 40, batch_size=batch,
                        n_frames=algo.n_frames, out=algo.impl.staging_batch(batch),
                        seed=seed, shard=shard)
    return algo, it


def gpu_steps(algo, it, n):
    for _ in range(n):
        batch = next(it)
        algo._update_async(batch)
        algo._grad_step += 1  # as fit() does (drives TD3+BC's delayed actor)


def measure_kernel(ws_obj, reps: int = 50, settle: int = 3):
    """Average duration of the dominant kernel via HIP events on its stream,
    over ``reps`` launches after ``settle`` untimed ones."""
    import torch
    launch, flops, desc = ws_obj.dominant_kernel()
    for _ in range(settle):
        launch()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        launch()
    e1.record(s)
    torch.cuda.synchronize()
    avg_s = e0.elapsed_time(e1) / 1e3 / reps
    return avg_s, flops, desc


def _record_all_reduces(algo):
    """For a data-parallel impl: a list that collects (numel, dtype, device)
    of every all-reduce the update pipeline issues (recorded while the first
    update runs eagerly, before the graph capture), else None."""
    dp = getattr(algo.impl, "_dp", None)
    if dp is None:
        return None
    log = {"calls": [], "armed": True}
    inner = dp.all_reduce_sum

    def rec(t):
        if log["armed"]:
            log["calls"].append((t.numel(), t.dtype, t.device))
        inner(t)
    dp.all_reduce_sum = rec
    return log


def measure_all_reduces(log, ws: int, reps: int = 200) -> dict:
    """The exchange of one data-parallel step measured on its own: the same
    all-reduces (sizes, dtypes, order) on scratch tensors of the recorded
    shapes, ``reps`` steps bracketed by HIP events on the current stream
    (RCCL runs on it), max over ranks.  Reported beside the step time as
    "allreduce": calls and bytes per step, microseconds per step."""
    import torch
    import torch.distributed as dist
    step = log["calls"]  # recorded over exactly one (eager) update
    bufs = [torch.zeros(m, dtype=dt, device=dev) for m, dt, dev in step]
    nbytes = sum(b.numel() * b.element_size() for b in bufs)
    if ws == 1 or not step:
        return {"calls_per_step": len(step), "bytes_per_step": nbytes, "us_per_step": 0.0}
    for _ in range(5):
        for b in bufs:
            dist.all_reduce(b)
    torch.cuda.synchronize()
    dist.barrier()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        for b in bufs:
            dist.all_reduce(b)
    e1.record(s)
    torch.cuda.synchronize()
    us = _max_over_ranks(e0.elapsed_time(e1) * 1e3 / reps, ws)
    return {"calls_per_step": len(step), "bytes_per_step": nbytes, "us_per_step": round(us, 2),
            "busbw_GBps": round(2 * (ws - 1) / ws * nbytes / (us * 1e-6) / 1e9, 2),
            "method": f"the step's {len(step)} RCCL SUM all-reduces replayed eagerly on "
                      f"scratch buffers of the same sizes, {reps} steps, HIP events, max over "
                      "ranks (in the update they are captured in its graph)"}


def cpu_step_fn(name: str = "cql"):
    """One step of the CPU baseline: the oracle update (torch CPU, op for op)
    + the reference's host sampler restated (per-sample np.random.randint +
    TransitionMiniBatch gather).  Returns step() -> None."""
    import torch
    from oracle.cql import Batch, CQLNoise, CQLOracle
    from oracle.gather import gather, random_indices, synthetic_dataset, to_episodes, to_transitions
    B = WORKLOADS[name][1]
    gen = torch.Generator().manual_seed(0)
    if name == "dcql":
        return _cpu_step_dcql(B, gen)
    n = 100_000
    D, A = {"cql": (11, 3), "cqlrepro": (11, 3), "cqldp": (29, 8), "td3bc": (3, 1),
            "bcq": (17, 6)}[name]
    obs, act, rew, term = synthetic_dataset(n, D, A, episode_len=1000, seed=0)
    trans = []
    for o, a, r, t in to_episodes(obs, act, rew, term):
        trans += to_transitions(o, a, r, t)
    np.random.seed(0)
    if name in ("cql", "cqldp", "cqlrepro"):
        kw = (dict(hidden_units=(256, 256, 256), alpha_learning_rate=0.0, conservative_weight=10.0)
              if name == "cqlrepro" else {})
        orc = CQLOracle(D, A, n_critics=2, n_action_samples=10, seed=0, **kw)

        def update(batch, k):
            orc.update(batch, CQLNoise.draw(gen, B, A, 10))
    elif name == "bcq":
        from oracle.bcq import BCQNoise, BCQOracle
        orc = BCQOracle(D, A, n_quantiles=200, seed=0)

        def update(batch, k):
            orc.update(batch, BCQNoise.draw(gen, B, A, 100))
    else:
        from oracle.td3bc import StandardScalerT, TD3PlusBCOracle, fit_standard_scaler
        orc = TD3PlusBCOracle(D, A, scaler=StandardScalerT(*fit_standard_scaler(obs)), seed=0)

        def update(batch, k):
            orc.update(batch, torch.randn(B, A, generator=gen), grad_step=k)
    cnt = [0]

    def step():
        idx = random_indices(len(trans), B)
        b = gather([trans[i] for i in idx])
        batch = Batch.from_numpy(b["observations"], b["actions"], b["rewards"],
                                 b["next_observations"], b["terminals"], b["n_steps"])
        update(batch, cnt[0])
        cnt[0] += 1
    return step


def cpu_baseline(seconds: float, threads: int, name: str = "cql"):
    """Bounded sample: steps/s of cpu_step_fn over ~``seconds`` after 2 warm-up
    steps with ``threads`` torch threads -> (steps/s, steps, seconds)."""
    import torch
    torch.set_num_threads(threads)
    step = cpu_step_fn(name)
    for _ in range(2):
        step()
    t0 = time.perf_counter()
    k = 0
    while True:
        step()
        k += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return k / el, k, el


def _cpu_step_dcql(B: int, gen):
    """K5 on the host: the oracle DiscreteCQL-IQN update + the reference
    sampler restated (4-frame stacks) over 20k synthetic 84x84 frames."""
    import torch
    from oracle.discrete_cql import DiscreteCQLIQNOracle, IQNTaus, PixelBatch
    from oracle.gather import gather, random_indices, to_episodes, to_transitions
    rs = np.random.RandomState(0)
    n = 20_000
    frames = rs.randint(0, 256, size=(n, 1, 84, 84), dtype=np.uint8)
    act = rs.randint(4, size=n).astype(np.int32)
    rew = rs.randint(-1, 2, size=n).astype(np.float32)
    term = np.zeros(n, dtype=np.float32)
    term[1999::2000] = 1.0
    trans = []
    for o, a, r, t in to_episodes(frames, act, rew, term):
        trans += to_transitions(o, a, r, t)
    orc = DiscreteCQLIQNOracle((4, 84, 84), 4, seed=0)
    np.random.seed(0)

    def step():
        idx = random_indices(len(trans), B)
        b = gather([trans[i] for i in idx], n_frames=4)
        pb = PixelBatch(torch.from_numpy(b["observations"]),
                        torch.from_numpy(np.asarray(b["actions"])).long().view(-1),
                        torch.from_numpy(b["rewards"]), torch.from_numpy(b["next_observations"]),
                        torch.from_numpy(b["terminals"]), torch.from_numpy(b["n_steps"]))
        orc.update(pb, IQNTaus.draw(gen, B, 64))
    return step


def host_cpu() -> dict:
    """The host CPU as this process sees it: model, logical CPUs of the
    machine, this process's CPU share (affinity) and the thread count the
    all-cores baseline uses (OMP_NUM_THREADS when set, else the share)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    share = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(share, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else share
    return {"model": model, "machine_cpus": os.cpu_count(), "process_cpus": share,
            "threads": threads}


def _selftest(args) -> None:
    """The multi-rank bracket of main() over gloo with a host stand-in for
    the step (tests/test_bench_launcher.py): rendezvous, barrier-bracketed
    timing, max over ranks, rank-0 line with the whole-job value; for
    ``cqldp`` each rank also reports its shard of the global index stream."""
    wd = _watchdog(args.init_timeout, "rendezvous")
    hang = os.environ.get("D3A_SELFTEST_HANG_RANK")
    if hang is not None and int(hang) == int(os.environ.get("RANK", "0")):
        time.sleep(3600)  # a rank that never joins the rendezvous
    ws, rank, _ = _dist_setup("gloo", args.init_timeout)
    wd.set()
    shape, batch, _ = WORKLOADS[args.algo]
    dp = args.algo == "cqldp"
    rs = np.random.RandomState(1000)
    x = np.ones((64, 64), dtype=np.float32)

    fail = os.environ.get("D3A_SELFTEST_FAIL_RANK")
    if fail is not None and int(fail) == rank:
        raise SystemExit(3)

    def step():
        g = rs.randint(1_000_000, size=batch * ws)  # one global draw per step
        mine = g[rank * batch:(rank + 1) * batch] if dp else g[:batch]
        time.sleep(0.001 * (1 + rank))  # ranks finish at different times
        return int(mine.sum()) + int((x @ x)[0, 0])

    for _ in range(args.warmup):
        step()
    _barrier(ws)
    t0 = time.perf_counter()
    chk = sum(step() for _ in range(args.steps))
    _barrier(ws)
    elapsed = _max_over_ranks(time.perf_counter() - t0, ws)
    import torch
    import torch.distributed as dist
    sums = [chk]
    if ws > 1:
        t = torch.zeros(ws, dtype=torch.int64)
        t[rank] = chk
        dist.all_reduce(t)
        sums = t.tolist()
    if rank == 0:
        value = (1 if dp else ws) * args.steps / elapsed
        print(json.dumps({"metric": "selftest", "value": round(value, 2), "n_gpus": ws,
                          "steps": args.steps, "ms_per_step": 1e3 * elapsed / args.steps,
                          "scaling": "weak", "global_batch": batch * ws,
                          "rank_checksums": sums}))
    if ws > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--transitions", type=int, default=1_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-seconds-1t", type=float, default=6.0)
    ap.add_argument("--algo", choices=sorted(WORKLOADS), default="cql",
                    help="cql = the BASELINE.json headline (K2); td3bc = K1 shapes")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--precision", choices=["fp32", "bf16", "bf16h", "sbf16x6"], default="fp32",
                    help="bf16: the critic-ensemble forward (the 15,616 + 256-row critic pass) "
                         "with one bf16 part per operand and fp32 accumulation (d3a_q2_fwd_x1), "
                         "its backward the mask-factored split-bf16 d3a_q2_bwd_x6 -- a "
                         "throughput line, never the headline; bf16h: round 3's line (every "
                         "operand of forward and backward one bf16 part, bf16 kept activations: "
                         "d3a_q2_fwd_bf16 / d3a_q2_bwd_bf16); sbf16x6: the large input-gradient "
                         "GEMMs on the bf16 matrix cores with hi/mid/lo split operands "
                         "(fp32-accurate)")
    ap.add_argument("--critic-gemm", choices=["fp32", "x6"], default=None,
                    help="GEMM arithmetic of the [n_in, 256, 256, 1] critic passes at fp32 "
                         "accuracy: fp32 = v_mfma_f32_32x32x2_f32; x6 = exact three-way split-bf16 "
                         "operands on the bf16 matrix cores (csrc/q2_x6*.hip); default: "
                         "d3rlpy_amd.ops.CRITIC_GEMM")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="host threads of the all-cores CPU baseline (default: this "
                         "process's CPU share)")
    ap.add_argument("--selftest-gloo", action="store_true",
                    help="launcher self-test without a GPU: gloo ranks, a host stand-in step")
    ap.add_argument("--init-timeout", type=float, default=300.0,
                    help="seconds allowed for the rendezvous, RCCL initialisation and the "
                         "warm-up (first graph capture); past it the rank exits with status 75")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary of the dominant kernel (tools/pmc_pass.sh); default "
                         "profiles/r01_pmc_traffic_<algo>.json")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's plain `bench.py --gpus N`: become N ranks (no GPU use here)
        return launch_ranks(args.gpus, sys.argv[1:])
    if args.selftest_gloo:
        return _selftest(args)

    import torch
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if args.precision in ("bf16", "bf16h"):
        from d3rlpy_amd import ops as _ops
        _ops.set_critic_precision(args.precision)
    if args.precision == "sbf16x6":
        from d3rlpy_amd import ops as _ops
        _ops.set_sbf16(6)
    from d3rlpy_amd import ops as _ops
    if args.critic_gemm is not None:
        _ops.set_critic_gemm(args.critic_gemm)
    wd = _watchdog(args.init_timeout, "rendezvous / RCCL init / warm-up with graph capture")
    ws, rank, local = _dist_setup("nccl", args.init_timeout)
    if ws != args.gpus:
        print(f"bench: WORLD_SIZE={ws} but --gpus {args.gpus}; reporting n_gpus={ws}",
              file=sys.stderr)
    algo, it = build_workload(rank, args.transitions, args.algo, ws, local)
    ar_log = _record_all_reduces(algo)

    gpu_steps(algo, it, 1)  # eager first update: its all-reduces are recorded
    if ar_log is not None:
        ar_log["armed"] = False
    # the dominant kernel's average launch time (HIP events on its stream),
    # over its last 500 of 1,000 back-to-back launches, taken after the first
    # (eager) warm-up step and before the others: the MI355X takes >10 ms of
    # load to reach its loaded clock (the same kernel measured 37.5 us after 5
    # warm-up steps, 34.2 after 50, 31.4 in a 300-step profile), so the
    # measurement waits for the clock, and the remaining warm-up steps then
    # run the whole step's working set through the caches right before the
    # timed region (profiles/r04_bench_window.jsonl)
    # (BENCH_MEASURE_LAST=1: the round-4 order, measurement after every warm-up
    # step, right before the timed region)
    wsp = next(iter(algo.impl._ws.values()))
    last = os.environ.get("BENCH_MEASURE_LAST", "0") == "1"
    if last:
        gpu_steps(algo, it, max(0, args.warmup - 1))
    kern_s, kflops, kdesc = measure_kernel(wsp, reps=500, settle=500)
    # the critic weight-gradient backward, measured the same way (on the last
    # forward's kept activations)
    bwd = None
    if hasattr(wsp, "backward_kernel") and wsp.backward_kernel() is not None:
        bl, bflops, bdesc = wsp.backward_kernel()
        b_s, _, _ = measure_kernel(type("K", (), {"dominant_kernel": lambda self: (bl, bflops, bdesc)})(),
                                   reps=500, settle=100)
        bwd = (b_s, bflops, bdesc)
    if not last:
        gpu_steps(algo, it, max(0, args.warmup - 1))
    torch.cuda.synchronize()
    _barrier(ws)
    wd.set()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gpu_steps(algo, it, args.steps)
    t_enq = time.perf_counter()  # host: every step enqueued (no sync inside the loop)
    torch.cuda.synchronize()
    _barrier(ws)
    t1 = time.perf_counter()
    elapsed = _max_over_ranks(t1 - t0, ws)
    # host cost of one step on its own: a burst enqueued onto an idle device
    # right after a sync (the gather launch + graph replay through ctypes /
    # torch), before the device can push back
    nb = min(20, max(1, args.steps))
    torch.cuda.synchronize()
    th0 = time.perf_counter()
    gpu_steps(algo, it, nb)
    th1 = time.perf_counter()
    torch.cuda.synchronize()
    # where the short window's time goes: device time of each step of a
    # 20-step window run like the timed one (HIP events on the stream between
    # the steps' enqueues; after the timed region, so it does not perturb it)
    import torch as _t
    st = _t.cuda.current_stream()
    _t.cuda.synchronize()
    evs = [_t.cuda.Event(enable_timing=True) for _ in range(nb + 1)]
    evs[0].record(st)
    for k in range(nb):
        gpu_steps(algo, it, 1)
        evs[k + 1].record(st)
    _t.cuda.synchronize()
    step_trace = [round(1e3 * evs[k].elapsed_time(evs[k + 1]), 1) for k in range(nb)]
    host = {"host_us_per_step": round(1e6 * (th1 - th0) / nb, 2),
            "host_loop_us_per_step": round(1e6 * (t_enq - t0) / max(1, args.steps), 2),
            "method": f"perf_counter around next(it) + _update_async with no sync: a burst of "
                      f"{nb} steps enqueued onto an idle device (host_us_per_step), and the timed "
                      "loop's enqueue time over its steps (host_loop_us_per_step: equals "
                      "ms_per_step when the device pushes back)",
            "step_trace_us": step_trace,
            "step_trace_method": f"HIP events between the enqueues of {nb} steps after a sync "
                                 "(device time per step, first step first)"}
    # sanity: the losses are finite
    names, vals = algo.impl.read_metrics_ring(None)
    # NaN in a column marks "not computed at this step" (TD3+BC's delayed
    # actor); every step computes critic_loss
    ci = names.index("critic_loss") if "critic_loss" in names else names.index("loss")
    finite = bool(np.isfinite(vals[:, ci]).all() and np.isfinite(vals[~np.isnan(vals)]).all())

    allreduce = measure_all_reduces(ar_log, ws) if ar_log is not None else None
    if rank != 0:
        if ws > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return

    # MI355X dense MFMA peaks (MI355X_MICROARCH.md): fp32-input 157.3 TF; bf16
    # 2.5 PF (the bf16 line's dominant kernel runs on the bf16 matrix cores)
    # the fp32-accurate split-bf16 critic kernels (CRITIC_GEMM "x6") run six bf16
    # MFMA products per fp32 product: their ceiling is the bf16 peak / 6
    x6 = _ops.CRITIC_GEMM == "x6" and args.precision == "fp32" and "x6" in kdesc
    # a kernel whose one operand is exact in one bf16 part (K5's uint8 pixels)
    # runs three products per fp32 product ("split-bf16 x3" in its label)
    x3 = args.precision == "fp32" and "split-bf16 x3" in kdesc
    nprod = 3 if x3 else 6
    x6 = x6 or x3
    bf16 = args.precision in ("bf16", "bf16h")
    peak_tflops = 2500.0 if bf16 else (2500.0 / nprod if x6 else 157.3)
    achieved = kflops / kern_s / 1e12
    traffic, traffic_src = None, None
    if args.traffic_json is None:
        prof = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
        # the PMC summary of THIS line's dominant kernel, this round's only:
        # r{ROUND}_pmc_traffic_<algo><suffix>.json whose bench_desc is this
        # line's kernel description (no older round's file stands in)
        suffix = f"_{args.precision}" if bf16 else "_x6" if x6 else ""
        args.traffic_json = os.path.join(prof, f"r{ROUND:02d}_pmc_traffic_{args.algo}{suffix}.json")
    if os.path.exists(args.traffic_json):
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("bench_desc") == kdesc:
                traffic = tj.get("hbm_bytes_per_launch")
                traffic_src = os.path.relpath(args.traffic_json, os.path.dirname(
                    os.path.abspath(__file__)))
        except Exception:
            traffic = None
    cpu = None
    # the CPU baseline is a rank-0, single-GPU-run measurement (not repeated per N)
    if not args.no_cpu_baseline and ws == 1:
        cpu_host = host_cpu()
        threads = args.cpu_threads or cpu_host["threads"]
        sps, k, el = cpu_baseline(args.cpu_seconds, threads, args.algo)
        sps1, k1, el1 = cpu_baseline(args.cpu_seconds_1t, 1, args.algo)
        what = {"cql": "CQL update (torch CPU, op-for-op restatement of cql_impl.py/"
                       "sac_impl.py/ddpg_impl.py)",
                "cqldp": "CQL update at antmaze shapes, batch 256 (torch CPU, op-for-op "
                         "restatement of cql_impl.py/sac_impl.py/ddpg_impl.py)",
                "cqlrepro": "CQL reproduction update (hidden [256,256,256], no update_alpha, "
                            "conservative_weight 10; torch CPU, op-for-op restatement of "
                            "cql_impl.py/sac_impl.py/ddpg_impl.py)",
                "td3bc": "TD3+BC update (torch CPU, op-for-op restatement of "
                         "td3_plus_bc_impl.py/td3_impl.py/ddpg_impl.py, standard scaler)",
                "bcq": "BCQ update (torch CPU, op-for-op restatement of bcq_impl.py/"
                       "ddpg_impl.py, QR critics)",
                "dcql": "DiscreteCQL-IQN update (torch CPU, op-for-op restatement of "
                        "dqn_impl.py/cql_impl.py/iqn_q_function.py, pixel encoder)"}[args.algo]
        cpu = {"value": round(sps, 3), "unit": "gradient-steps/s", "cores": threads,
               "kind": "port",
               "sample": f"oracle {what} + reference host sampler restated "
                         f"(np.random.randint per sample + TransitionMiniBatch gather) on a "
                         f"100k-transition synthetic dataset; bounded live sample: {k} steps "
                         f"in {el:.1f}s on {threads} threads (this process's CPU share)",
               "one_thread": {"value": round(sps1, 3), "cores": 1,
                              "sample": f"{k1} steps in {el1:.1f}s"},
               "host": cpu_host}
        # BASELINE.md's full protocol (>= 1000 steps after 50 warm-up, median
        # of 5, all cores and 1 thread), run by tools/cpu_baseline_protocol.py
        proto = next((p for p in (os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                               "profiles", f"r0{r}_cpu_baseline_{args.algo}.json")
                                  for r in (3, 2)) if os.path.exists(p)), "")
        if os.path.exists(proto):
            with open(proto) as f:
                pr = json.load(f)
            cpu["protocol"] = {"file": os.path.relpath(proto, os.path.dirname(
                os.path.abspath(__file__))), "all_cores_median": round(pr["all_cores"]["median"], 3),
                "all_cores_threads": pr["all_cores"]["threads"],
                "all_cores_note": pr["all_cores"].get("note", ""),
                "thread_sweep": [(w["threads"], round(w["steps_per_s"], 3))
                                 for w in pr.get("thread_sweep", [])],
                "one_thread_median": round(pr["one_thread"]["median"], 3),
                "steps": pr["steps"], "warmup": pr["warmup"], "runs": pr["runs"],
                "host_model": pr["host"]["model"]}
    # replicas: every rank's steps count; data parallel: one global step per
    # step of all ranks together
    dp = args.algo == "cqldp"
    value = (1 if dp else ws) * args.steps / elapsed
    shape, batch, wdesc = WORKLOADS[args.algo]
    metric = {"cql": "gradient-steps/sec (CQL, batch=256, obs=11 act=3) at 1/2/4/8 GPU",
              "cqldp": "gradient-steps/sec (CQL data-parallel, 256 rows per GPU, obs=29 act=8)",
              "cqlrepro": "gradient-steps/sec (CQL reproduction config, batch=256, obs=11 act=3, "
                          "hidden 3x256, alpha fixed)",
              "td3bc": "gradient-steps/sec (TD3+BC, batch=100, obs=3 act=1)",
              "bcq": "gradient-steps/sec (BCQ QR-200, batch=256, obs=17 act=6)",
              "dcql": "gradient-steps/sec (DiscreteCQL-IQN, batch=512, 4x84x84 pixels)"}[args.algo]
    out = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "gradient-steps/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("fp32 (critic GEMMs fp32-accurate: exact three-way split-bf16 operands, "
                  "fp32 accumulation on the bf16 matrix cores)" if x6 else "fp32")
                 if args.precision == "fp32" else
                 "bf16 (critic-ensemble forward operands one bf16 part; backward split-bf16 "
                 "mask-factored; fp32 accumulation, losses, optimiser; kernels "
                 "d3a_q2_fwd_x1 + d3a_q2_bwd_x6 -- round 3's bf16 lines are the bf16h pair)"
                 if args.precision == "bf16" else
                 "bf16 (critic-ensemble GEMM operands and kept activations; fp32 accumulation, "
                 "losses, optimiser; kernels d3a_q2_fwd_bf16 + d3a_q2_bwd_bf16, round 3's "
                 "bf16 line)"
                 if args.precision == "bf16h" else
                 "fp32 (input-gradient GEMMs: split-bf16 x6 on bf16 MFMA)",
        "data": (f"synthetic (D4RL {shape} shapes, {args.transitions} transitions, "
                 "HBM-resident)" if shape != "atari" else
                 f"synthetic Atari-shaped uint8 frames ({args.transitions} x 1x84x84, "
                 "HBM-resident, 4-frame stacks gathered on device)"),
        "config": {"workload": wdesc,
                   "global_batch": batch * ws,
                   "parallelism": (f"dp{ws} (RCCL all-reduce)" if dp and ws > 1 else
                                   "single learner" if dp else f"replicas x{ws}"),
                   "losses_finite": finite},
        "roofline": {"bound": "mfma", "achieved": round(achieved, 3), "peak": peak_tflops,
                     "unit": "TFLOP/s", "frac": round(achieved / peak_tflops, 4),
                     "traffic": traffic, "kernel": kdesc,
                     "traffic_source": traffic_src or "none: no PMC file of this round "
                                                     "names this kernel",
                     **({"bf16_mfma_frac": round(nprod * achieved / 2500.0, 4),
                         "peak_note": f"bf16 dense MFMA peak 2500 TF / {nprod} products"}
                        if x6 else {}),
                     "avg_launch_us": round(kern_s * 1e6, 3),
                     "launch_timing": "HIP events on the kernel's stream, 500 launches after 500 "
                                      "settling launches, after the first warm-up step"},
        "cpu_baseline": cpu,
    }
    if bwd is not None:
        b_s, bflops, bdesc = bwd
        # the backward's large products are the 0 / 1 ReLU mask times three
        # bf16 parts: its ceiling is the bf16 peak / 3 (fp32 MFMA: 157.3 TF)
        # (the bf16 line's backward is the same split-bf16 x3 kernel: priced alike)
        bx3 = "x3" in bdesc and args.precision in ("fp32", "bf16")
        bpeak = 2500.0 / 3 if bx3 else 157.3
        bach = bflops / b_s / 1e12
        sec = {"bound": "mfma", "achieved": round(bach, 3), "peak": round(bpeak, 1),
               "unit": "TFLOP/s", "frac": round(bach / bpeak, 4), "kernel": bdesc,
               "avg_launch_us": round(b_s * 1e6, 3),
               "launch_timing": "HIP events on the kernel's stream, 500 launches after 100 "
                                "settling launches, after the first warm-up step"}
        if bx3:
            sec["bf16_mfma_frac"] = round(3 * bach / 2500.0, 4)
        # the step's largest kernel leads: the other critic kernel beside it
        if b_s > kern_s:
            # (its PMC summary: r{ROUND}_pmc_traffic_<algo><suffix>_bwd.json,
            # tools/pmc_dominant.py --backward, matched by description)
            sec["traffic"], sec["traffic_source"] = None, None
            bj = args.traffic_json[:-5] + "_bwd.json" if args.traffic_json.endswith(".json") else None
            if bj and os.path.exists(bj):
                with open(bj) as f:
                    tj = json.load(f)
                if tj.get("bench_desc") == bdesc and tj.get("hbm_bytes_per_launch"):
                    sec["traffic"] = float(tj["hbm_bytes_per_launch"])
                    sec["traffic_source"] = os.path.relpath(bj, os.path.dirname(os.path.abspath(__file__)))
            out["roofline"], out["roofline_other"] = sec, out["roofline"]
        else:
            out["roofline_other"] = sec
    out["host"] = host
    if allreduce is not None:
        allreduce["frac_of_step"] = round(allreduce["us_per_step"] / (1e3 * out["ms_per_step"]), 4)
        out["allreduce"] = allreduce
    if cpu is not None:
        out["speedup_vs_cpu"] = round(value / cpu["value"], 1)
    print(json.dumps(out))
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
