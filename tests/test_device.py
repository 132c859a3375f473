"""Device / parallel() / check_use_gpu (d3rlpy/gpu.py:14-72, context.py:4-22,
argument_utility.py:96-114) — CPU tests; the first mirrors the reference's
tests/test_gpu.py."""
import copy
from unittest.mock import patch

import pytest

from d3rlpy_amd.context import disable_parallel, get_parallel_flag, parallel
from d3rlpy_amd.factories import check_use_gpu
from d3rlpy_amd.gpu import Device


@patch("d3rlpy_amd.gpu.get_gpu_count", return_value=2)
def test_device(mock):
    device = Device()

    copy_device = copy.deepcopy(device)
    assert device.get_id() == 0
    assert copy_device.get_id() == 0

    with parallel():
        inc_device = copy.deepcopy(device)
        assert device.get_id() == 1
        assert inc_device.get_id() == 1

        # check circulation
        inc2_device = copy.deepcopy(device)
        assert device.get_id() == 0
        assert inc2_device.get_id() == 0


def test_parallel_flag_stack():
    assert not get_parallel_flag()
    with parallel():
        assert get_parallel_flag()
        with disable_parallel():
            assert not get_parallel_flag()
        assert get_parallel_flag()
    assert not get_parallel_flag()


def test_device_compare_and_params():
    assert Device(1) == Device(1) and Device(0) != Device(1)
    assert Device(3).get_params() == {"idx": 3}
    with pytest.raises(ValueError):
        Device(0) == 0  # noqa: B015


def test_check_use_gpu_follows_reference():
    assert check_use_gpu(True) == Device(0)
    assert check_use_gpu(2) == Device(2)
    d = Device(1)
    assert check_use_gpu(d) is d
    assert check_use_gpu(False) is None
    assert check_use_gpu(None) is None
    with pytest.raises(ValueError):
        check_use_gpu("cuda")


def test_cpu_selection_raises_not_implemented():
    """use_gpu=False / None is the reference's CPU path, which the HIP engine
    does not have: building an Impl with it raises (no silent GPU 0)."""
    from d3rlpy_amd.algos.cql import CQL
    algo = CQL(use_gpu=False)
    assert algo._use_gpu is None
    with pytest.raises(NotImplementedError, match="no CPU compute path"):
        algo.create_impl((11,), 3)
    assert CQL()._use_gpu == Device(0)  # the default: the GPU (documented deviation)


def test_bare_true_is_this_ranks_gpu_in_a_multi_process_launch(monkeypatch):
    """One process per GPU (torchrun / bench.launch_ranks): use_gpu=True is
    GPU LOCAL_RANK, so a rank's parameters sit beside its dataset and RCCL
    communicator; a single process (or WORLD_SIZE 1) keeps Device(0)."""
    from d3rlpy_amd.algos.cql import CQL
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert check_use_gpu(True) == Device(3)
    assert CQL()._use_gpu == Device(3)
    assert check_use_gpu(1) == Device(1)  # an explicit id still wins
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert check_use_gpu(True) == Device(0)
    monkeypatch.delenv("LOCAL_RANK")
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert check_use_gpu(True) == Device(0)
