"""The fused metric kernel (metric_rows / metric_accum, csrc/kernels/nn_kernels.hip) against
the torch formulation of the same metrics and the native host metrics."""
import numpy as np
import pytest
import torch

from cxxnet_amd.utils.metric import DeviceMetricSet, MetricSet

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,L,B", [(1000, 1, 256), (10, 1, 37), (1, 1, 50), (12, 3, 64)])
def test_metric_kernel_matches_host(K, L, B):
    g = torch.Generator().manual_seed(K * 7 + L)
    names = {1: ["error", "logloss"], 3: ["rec@1", "rec@5"]}[L] if K >= 5 or L == 3 else ["error", "logloss"]
    if K >= 5 and L == 1:
        names = ["error", "logloss", "rec@1", "rec@5"]
    if K == 1:
        p = torch.rand(B, 1, generator=g)
        lab = (torch.rand(B, 1, generator=g) > 0.5).float()
    else:
        p = torch.softmax(torch.randn(B, K, generator=g) * 3, 1)
        lab = torch.randint(0, K, (B, L), generator=g).float()
    host = MetricSet()
    dev = DeviceMetricSet()
    for n in names:
        host.add_metric(n)
        dev.add_metric(n)
    pd = p.cuda()
    for rows in (None, B - 3):
        dev.add_eval([pd] * len(names), {"label": lab.cuda()}, rows=rows)
        b = B if rows is None else rows
        host.add_eval([p[:b].numpy()] * len(names), {"label": lab[:b].numpy()})
    hv = [float(x.split(":")[1]) for x in host.print("t").split("\t")[1:]]
    assert np.allclose(hv, dev.values(), rtol=1e-4, atol=1e-6), (hv, dev.values())


def test_rec_at_n_ties_lowest_index_first():
    """Tied scores: the kernel ranks the lowest index first (at most n labels hit), exactly as
    the torch fallback (DeviceMetricSet._one) -- the metric no longer depends on the path."""
    B, K = 64, 12
    g = torch.Generator().manual_seed(5)
    p = torch.randint(0, 3, (B, K), generator=g).float() / 4.0  # many exact ties
    lab = torch.randint(0, K, (B, 3), generator=g).float()
    for n in ("rec@1", "rec@2", "rec@5"):
        dev = DeviceMetricSet()
        dev.add_metric(n)
        dev.add_eval([p.cuda()], {"label": lab.cuda()})
        ref = DeviceMetricSet._one(n, p, lab).item() / B
        assert abs(dev.values()[0] - ref) < 1e-6, (n, dev.values()[0], ref)
