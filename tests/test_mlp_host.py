"""Host logic of d3rlpy_amd.mlp.Acts (no GPU): the ReLU mask image the x6 Q
forward writes is used only inside the rows it wrote, [hmask_from, hmask_to)."""
import pytest
import torch

from d3rlpy_amd.mlp import Acts


def _acts(R=96, H=256):
    hs = [torch.zeros(1, R, H), torch.zeros(1, R, H)]
    a = Acts(hs, torch.zeros(1, R), R, hmask=torch.zeros(1, R, H // 32, dtype=torch.int32))
    a.hmask[0, :, 0] = 0b101  # units 0 and 2 active on every row
    a.hmask_from, a.hmask_to = 0, 64
    a.no_last_h = True
    return a


def test_relu_decisions_from_mask_bits_inside_written_rows():
    a = _acts()
    d = a.relu_decisions(0, 8, 64)
    assert d[-1].shape == (56, 256)
    assert d[-1][:, 0].all() and not d[-1][:, 1].any() and d[-1][:, 2].all()


def test_relu_decisions_refuse_rows_past_the_written_range():
    a = _acts()
    with pytest.raises(AssertionError):
        a.relu_decisions(0, 32, 96)
