"""BASELINE.md's CPU-baseline protocol on the GPU box's host (no GPU used).

    python tools/cpu_baseline_protocol.py --algo cql --out profiles/r02_cpu_baseline_cql.json

The step is bench.cpu_step_fn (the oracle's op-for-op CPU update + the
reference's host sampler restated).  Protocol: `--warmup` (50) untimed steps,
then `--steps` (1000) timed with time.perf_counter, median of `--runs` (5):
  * all cores: torch.set_num_threads(<this process's CPU share, capped by
    OMP_NUM_THREADS>), the runs one after another;
  * 1 thread: torch.set_num_threads(1); the runs execute concurrently as
    separate processes pinned to distinct cores of the share (a single-thread
    run is compute bound, so pinning them apart keeps them independent while
    the protocol fits one bounded call).
Writes one JSON file with both medians, every run and the host description;
bench.py reports it next to its live bounded sample.

``--threads N`` sets the all-cores leg's thread count (default: the host's
physical core count, BASELINE.md:27-28 -- on the GPU box that is more threads
than the 16-CPU share a one-GPU tenant is given, which the file records);
``--sweep 1,16,64,128`` adds a bounded sample (``--sweep-seconds`` each) at
every listed thread count.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed_run(algo: str, threads: int, steps: int, warmup: int) -> float:
    import torch
    import bench
    torch.set_num_threads(threads)
    step = bench.cpu_step_fn(algo)
    for _ in range(warmup):
        step()
    t0 = time.perf_counter()
    last = t0
    for i in range(steps):
        step()
        now = time.perf_counter()
        if now - last > 30:  # progress (a silent GPU-box command is taken for hung)
            print(f"  {threads} threads: {i + 1}/{steps} steps, {now - t0:.0f}s", flush=True)
            last = now
    return steps / (time.perf_counter() - t0)


def physical_cores() -> int:
    """Distinct (physical id, core id) pairs of /proc/cpuinfo (lscpu's
    Core(s) per socket x Socket(s)); the logical count if unreadable."""
    pairs, phys, core = set(), None, None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":", 1)[1].strip()
                elif not line.strip():
                    if phys is not None and core is not None:
                        pairs.add((phys, core))
                    phys = core = None
    except OSError:
        pass
    return len(pairs) or os.cpu_count()


def sweep(algo: str, threads, seconds: float) -> list:
    import bench
    out = []
    for n in threads:
        sps, k, el = bench.cpu_baseline(seconds, n, algo)
        out.append({"threads": n, "steps_per_s": sps, "steps": k, "seconds": el})
        print(f"sweep {n} threads: {sps:.3f} steps/s ({k} steps in {el:.1f}s)", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="cql")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--threads", type=int, default=None,
                    help="physical-cores leg thread count (default: physical cores)")
    ap.add_argument("--phys-steps", type=int, default=None,
                    help="steps per physical-cores run (default --steps; the leg can run "
                         "far slower than the best thread count on a shared host)")
    ap.add_argument("--phys-runs", type=int, default=None)
    ap.add_argument("--sweep", default="", help="comma-separated thread counts")
    ap.add_argument("--sweep-seconds", type=float, default=10.0)
    ap.add_argument("--single-on-core", type=int, default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.single_on_core is not None:
        os.sched_setaffinity(0, {args.single_on_core})
        print(json.dumps({"sps": timed_run(args.algo, 1, args.steps, args.warmup)}), flush=True)
        return
    import bench
    host = bench.host_cpu()
    host["physical_cores"] = physical_cores()
    n_phys = args.threads or host["physical_cores"]
    print(f"host {host}; physical-cores leg {n_phys} threads", flush=True)
    sw = sweep(args.algo, [int(v) for v in args.sweep.split(",") if v], args.sweep_seconds)
    # legs: the host's physical core count (BASELINE.md:27-28), the fastest
    # thread count of the sweep (when it differs), one thread
    legs = {}
    phys_steps, phys_runs = args.phys_steps or args.steps, args.phys_runs or args.runs
    runs = []
    for r in range(phys_runs):
        runs.append(timed_run(args.algo, n_phys, phys_steps, min(args.warmup, phys_steps)))
        print(f"physical-cores run {r}: {runs[-1]:.3f} steps/s", flush=True)
    legs["physical_cores"] = {"threads": n_phys, "median": statistics.median(runs), "runs": runs,
                              "steps": phys_steps, "warmup": min(args.warmup, phys_steps),
                              "note": "torch.set_num_threads(physical cores of the host)"}
    if sw:
        best = max(sw, key=lambda w: w["steps_per_s"])["threads"]
        if best != n_phys and best != 1:
            runs = []
            for r in range(args.runs):
                runs.append(timed_run(args.algo, best, args.steps, args.warmup))
                print(f"best-threads ({best}) run {r}: {runs[-1]:.3f} steps/s", flush=True)
            legs["best_threads"] = {"threads": best, "median": statistics.median(runs),
                                    "runs": runs, "steps": args.steps, "warmup": args.warmup,
                                    "note": "the fastest thread count of the sweep"}
    cores = sorted(os.sched_getaffinity(0))
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--algo", args.algo,
                               "--steps", str(args.steps), "--warmup", str(args.warmup),
                               "--single-on-core", str(cores[(2 * r) % len(cores)])],
                              stdout=subprocess.PIPE, text=True)
             for r in range(args.runs)]
    one = []
    for p in procs:
        out, _ = p.communicate()
        assert p.returncode == 0, out
        one.append(json.loads(out.strip().splitlines()[-1])["sps"])
    print(f"1-thread runs: {[round(v, 3) for v in one]}", flush=True)
    legs["one_thread"] = {"threads": 1, "median": statistics.median(one), "runs": one,
                          "steps": args.steps, "warmup": args.warmup,
                          "note": "runs concurrent, pinned to distinct cores"}
    # "all_cores": the multi-thread leg bench.py quotes -- the faster of the
    # physical-cores and best-threads legs, labelled with its thread count
    allc = max((v for k, v in legs.items() if k != "one_thread"), key=lambda v: v["median"])
    res = {"algo": args.algo, "unit": "gradient-steps/s", "steps": args.steps,
           "warmup": args.warmup, "runs": args.runs, "legs": legs,
           "all_cores": dict(allc, note=allc["note"] + " (the faster multi-thread leg)"),
           "thread_sweep": sw, "one_thread": legs["one_thread"], "host": host}
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
