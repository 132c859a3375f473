"""Pin of the n-step return arithmetic (CPU).

dataset.pyx:1322-1331 accumulates ``n_step_return += reward * gamma ** i``
with C float ``gamma`` / ``reward`` and C int ``i``.  What that line computes
is fixed by the C its pinned Cython (0.29.21, requirements.txt:8) generates:
tests/golden/cython_pow_codegen.txt (made by tools/cython_pow_probe.sh on a
self-written snippet; Cython 3's cpow=True mode is the 0.29 power semantics)
records ``acc = (acc + (reward * powf(gamma, ((float)i))))`` — fp32 multiply
and add, and the C library's powf, which is NOT always the correctly rounded
power (e.g. powf(0.95f, 58) != (float)pow(0.95, 58) on glibc).

Pinned here: oracle/c/nstep_return.c (that line, compiled by gcc) == the
oracle's gather == the powf table the product hands to the HIP gather kernel,
bit for bit, including a (gamma, i) where powf differs from the rounded fp64
power.  The GPU side is tests/test_gpu_sampler.py.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import build_c
from oracle import gather as og

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def clib():
    return build_c.load()


def test_codegen_record_is_the_powf_line():
    with open(os.path.join(HERE, "golden", "cython_pow_codegen.txt")) as f:
        text = f.read()
    assert "cpow=True (0.29 semantics):  __pyx_v_acc = (__pyx_v_acc + (__pyx_v_reward * " \
           "powf(__pyx_v_gamma, ((float)__pyx_v_i))));" in text


def test_powf_is_not_the_rounded_double_power(clib):
    # the case that makes the distinction observable (glibc powf)
    p = clib.d3a_oracle_powf(0.95, 58)
    q = np.float32(np.float64(np.float32(0.95)) ** 58)
    assert np.float32(p) != q


@pytest.mark.parametrize("gamma", [0.99, 0.95, 0.9, 0.999])
def test_product_gamma_table_is_c_powf(clib, gamma):
    from d3rlpy_amd._native import gamma_powers
    got = gamma_powers(gamma, 64)
    want = [clib.d3a_oracle_powf(gamma, i) for i in range(64)]
    assert [np.float32(v).tobytes() for v in got] == [np.float32(v).tobytes() for v in want]


@pytest.mark.parametrize("gamma,n_steps", [(0.99, 1), (0.99, 3), (0.95, 60), (0.9, 8)])
def test_oracle_gather_returns_equal_c_restatement(clib, gamma, n_steps):
    rs = np.random.RandomState(n_steps)
    n = 150
    obs = rs.randn(n, 3).astype(np.float32)
    act = rs.uniform(-1, 1, (n, 2)).astype(np.float32)
    rew = (rs.randn(n, 1) * 3).astype(np.float32)
    trans = og.to_transitions(obs, act, rew, 1.0)
    batch = og.gather(trans, 1, n_steps, gamma)
    r = rew.reshape(-1)
    for i in range(len(trans)):
        used = ctypes.c_int32()
        avail = len(trans) - i
        c = clib.d3a_oracle_nstep_return(r[i:].ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                         avail, n_steps, gamma, ctypes.byref(used))
        assert np.float32(c).tobytes() == np.float32(batch["rewards"][i][0]).tobytes(), i
        assert used.value == int(batch["n_steps"][i][0])
