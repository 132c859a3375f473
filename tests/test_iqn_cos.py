"""iqn_cos (d3rlpy_amd/csrc/iqn_cos.hpp), the cosine of the IQN prior in
d3a_iqn_prior / d3a_iqn_embed_head / the recomputing head backward, checked on
the host: oracle/iqn_cos_check.cpp compiles the same header with g++ and
compares it with cos in double over the prior's arguments x = fl(fl(pi (e + 1))
tau), e < 64, tau on a grid of [0, 1) (and x up to 8192).  Bar: max error
below 1 ulp of the float result (faithful rounding; glibc's cosf reported
beside it for scale)."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_iqn_cos_faithful_on_prior_arguments(tmp_path):
    exe = tmp_path / "iqn_cos_check"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", os.path.join(ROOT, "oracle", "iqn_cos_check.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), str(1 << 16)], check=True, capture_output=True, text=True).stdout
    r = json.loads(out)
    print(r)
    assert r["args"] == 64 << 16
    assert r["max_ulp"] < 1.0 and r["max_ulp_0_8192"] < 1.0, r
