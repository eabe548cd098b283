"""DeviceMetricSet (device-side accumulation, one read-back per print) against the native
host metrics (csrc/runtime/metric.h, reference src/utils/metric.h) on the same scores."""
import numpy as np
import pytest
import torch

from cxxnet_amd.utils.metric import DeviceMetricSet, MetricSet


@pytest.mark.parametrize("K,L", [(10, 1), (1000, 1), (1, 1), (12, 3)])
def test_device_metrics_match_native(K, L):
    g = torch.Generator().manual_seed(K + L)
    names = ["error", "logloss", "rec@1", "rec@5"] if K >= 5 else ["error", "logloss"]
    if L == 3:
        names = ["rec@1", "rec@5"]
    host, dev = MetricSet(), DeviceMetricSet()
    for n in names:
        host.add_metric(n)
        dev.add_metric(n)
    for step, B in enumerate((37, 64, 5)):
        if K == 1:
            p = torch.rand(B, 1, generator=g)
            lab = (torch.rand(B, 1, generator=g) > 0.5).float()
        else:
            p = torch.softmax(torch.randn(B, K, generator=g) * 3, 1)
            lab = torch.randint(0, K, (B, L), generator=g).float()
        host.add_eval([p.numpy()] * len(names), {"label": lab.numpy()})
        rows = B - 2 if step == 2 else None  # padded tail of the last batch
        if rows is not None:
            host.clear()  # recompute the host side with the same trimming
        dev.add_eval([p] * len(names), {"label": lab}, rows=rows)
        if rows is not None:
            break
    # rebuild the host reference with identical rows
    host = MetricSet()
    for n in names:
        host.add_metric(n)
    g = torch.Generator().manual_seed(K + L)
    for step, B in enumerate((37, 64, 5)):
        if K == 1:
            p = torch.rand(B, 1, generator=g)
            lab = (torch.rand(B, 1, generator=g) > 0.5).float()
        else:
            p = torch.softmax(torch.randn(B, K, generator=g) * 3, 1)
            lab = torch.randint(0, K, (B, L), generator=g).float()
        b = B - 2 if step == 2 else B
        host.add_eval([p[:b].numpy()] * len(names), {"label": lab[:b].numpy()})
    hv = [float(x.split(":")[1]) for x in host.print("train").split("\t")[1:]]
    dv = dev.values()
    assert np.allclose(hv, dv, rtol=1e-5, atol=1e-6), (hv, dv)
    assert dev.print("train").split(":")[0] == host.print("train").split(":")[0]


def test_rmse_and_field_label():
    dev, host = DeviceMetricSet(), MetricSet()
    dev.add_metric("rmse", "aux")
    host.add_metric("rmse", "aux")
    p = torch.randn(9, 4)
    y = torch.randn(9, 4)
    dev.add_eval([p], {"aux": y})
    host.add_eval([p.numpy()], {"aux": y.numpy()})
    assert dev.print("test") == host.print("test")
    dev.clear()
    assert "nan" in dev.print("test")


def test_rec_at_n_fallback_ties():
    """rec@n fallback rule: a label's rank counts larger scores and equal scores at a lower
    index, so with all scores tied exactly the n lowest indices hit."""
    import torch
    from cxxnet_amd.utils.metric import DeviceMetricSet
    p = torch.zeros(1, 6)
    lab = torch.tensor([[0.0, 1.0, 4.0]])
    # rec@2: labels 0 and 1 rank 0 and 1 (hit), label 4 ranks 4 (miss) -> 2/3
    assert abs(DeviceMetricSet._one("rec@2", p, lab).item() - 2 / 3) < 1e-6
    # duplicate labels count once
    lab2 = torch.tensor([[0.0, 0.0, 5.0]])
    assert abs(DeviceMetricSet._one("rec@1", p, lab2).item() - 1 / 3) < 1e-6
    # larger scores outrank
    p3 = torch.tensor([[0.1, 0.9, 0.5, 0.5, 0.0, 0.2]])
    assert abs(DeviceMetricSet._one("rec@2", p3, torch.tensor([[2.0]])).item() - 1.0) < 1e-6
    assert abs(DeviceMetricSet._one("rec@2", p3, torch.tensor([[3.0]])).item() - 0.0) < 1e-6
