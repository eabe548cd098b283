"""ops.zero_ranges (launch_list.hip cxn_zero_ranges): the arena's accumulated-gradient ranges
zeroed in one launch -- exactly the ranges, aligned or not, nothing else."""
import pytest
import torch

from cxxnet_amd import ops

pytestmark = pytest.mark.gpu


def test_zero_ranges_exact():
    torch.manual_seed(0)
    buf = torch.randn(100_003, device="cuda") + 5.0
    ref = buf.clone()
    ranges = [(0, 1), (3, 4099), (4100, 4101), (5001, 70_000), (70_003, 70_010), (99_990, 100_003)]
    assert ops.zero_ranges(buf, ranges)
    for a, b in ranges:
        ref[a:b] = 0
    assert torch.equal(buf, ref)
    assert ops.zero_ranges(buf, [])
    assert not ops.zero_ranges(buf, [(i, i + 1) for i in range(0, 40, 2)])  # > 16 ranges: caller's loop
    with pytest.raises(ValueError):
        ops.zero_ranges(buf, [(5, 200_000)])
