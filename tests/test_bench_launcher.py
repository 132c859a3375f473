"""bench.py's multi-rank path on CPU (gloo, world size 2): the plain
``bench.py --gpus N`` form the driver uses starts N ranks itself, they
rendezvous on 127.0.0.1, time the barrier-bracketed steps, take the max over
ranks and rank 0 prints one line with ``n_gpus: N``; a failing rank fails
the job.  Also the data-parallel seed plumbing (d3rlpy_amd/dp.py)."""
import json
import os
import subprocess
import sys

import pytest

from d3rlpy_amd.dp import fold_rank

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, env=e, timeout=240)


@pytest.mark.parametrize("algo", ["cqldp", "cql"])
def test_bench_gpus2_launches_two_ranks(algo):
    r = _bench("--gpus", "2", "--selftest-gloo", "--steps", "10", "--warmup", "1",
               "--algo", algo)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 10
    assert out["global_batch"] == 512 if algo == "cqldp" else 512
    # rank 1 sleeps longer per step: the max over ranks is rank 1's time
    assert out["ms_per_step"] >= 2.0
    per_step = out["value"] * out["ms_per_step"] / 1e3
    assert per_step == pytest.approx(1 if algo == "cqldp" else 2, rel=1e-3)
    a, b = out["rank_checksums"]
    # data parallel: each rank gathers its own slice of one global stream
    assert (a != b) if algo == "cqldp" else (a == b)


def test_bench_failing_rank_fails_the_job():
    r = _bench("--gpus", "2", "--selftest-gloo", "--steps", "5", "--warmup", "1",
               env={"D3A_SELFTEST_FAIL_RANK": "1"})
    assert r.returncode != 0


def test_fold_rank_distinct_keys():
    keys = {fold_rank(12345, r) for r in range(64)}
    assert len(keys) == 64 and all(0 <= k < 2**62 for k in keys)
    assert fold_rank(12345, 0) == fold_rank(12345, 0)
    assert fold_rank(1, 3) != fold_rank(2, 3)


def test_dp_seeds_gloo():
    """Rank 0's seed reaches every rank; the policy-noise keys differ per
    rank although every rank called torch.manual_seed(0)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests",
                                                                    "dp_seed_worker.py")],
                                      env=env, stdout=subprocess.PIPE, text=True))
    outs = [json.loads(p.communicate(timeout=120)[0].strip().splitlines()[-1]) for p in procs]
    assert all(p.returncode == 0 for p in procs)
    r0, r1 = sorted(outs, key=lambda o: o["rank"])
    assert r0["own"] != r1["own"]
    assert r0["shared"] == r1["shared"] == r0["own"]
    assert r0["key"] != r1["key"]


def test_bench_hung_rank_exits_in_bounded_time():
    """A rank that never reaches the rendezvous: the others' watchdog ends the
    job with a non-zero status (75) well before any driver limit."""
    import time
    t0 = time.monotonic()
    r = _bench("--gpus", "2", "--selftest-gloo", "--steps", "5", "--warmup", "1",
               "--init-timeout", "8", env={"D3A_SELFTEST_HANG_RANK": "1"})
    el = time.monotonic() - t0
    assert r.returncode != 0
    assert el < 120, el
    assert "did not finish within" in r.stderr


def test_bench_all_reduce_accounting():
    """bench.py's data-parallel line: the all-reduces one eager update issues
    are recorded (calls, dtype, bytes) and then disarmed, so the graph capture
    and the timed replays are not counted."""
    import types
    import torch
    sys.path.insert(0, ROOT)
    import bench
    seen = []
    dp = types.SimpleNamespace(all_reduce_sum=lambda t: seen.append(t.numel()))
    algo = types.SimpleNamespace(impl=types.SimpleNamespace(_dp=dp))
    log = bench._record_all_reduces(algo)
    for n in (2, 151_000, 77_000, 8):  # scalar grads, critic, actor, metrics
        algo.impl._dp.all_reduce_sum(torch.zeros(n))
    log["armed"] = False
    algo.impl._dp.all_reduce_sum(torch.zeros(5))  # a later (captured) call
    assert seen == [2, 151_000, 77_000, 8, 5]  # every call still reaches the backend
    out = bench.measure_all_reduces(log, ws=1)
    assert out["calls_per_step"] == 4
    assert out["bytes_per_step"] == 4 * (2 + 151_000 + 77_000 + 8)
    assert bench._record_all_reduces(types.SimpleNamespace(impl=types.SimpleNamespace(_dp=None))) is None
