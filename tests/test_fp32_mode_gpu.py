"""Reference-precision (fp32) mode on the GPU as a parity oracle at production batch size.

`precision = fp32` runs the executor's fp32 formulas (the CPU path's torch code) on device
tensors.  Device weight init and the counter-hash dropout masks are the same in both modes, so
the bf16 HIP-kernel run and the fp32 run of one seed train the real AlexNet graph (max pooling,
LRN, dropout, relu fusion) from identical weights on identical data; their loss trajectories
and weights must stay within bf16 noise of each other."""
import pytest
import torch

from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.models import load_conf
from cxxnet_amd.nnet import NetTrainer
from cxxnet_amd.ops.mode import set_reference_precision

pytestmark = pytest.mark.gpu


def _train(precision, steps, batch, x, y, model="alexnet"):
    pairs = load_conf(model, [("batch_size", str(batch)), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"),
                                  ("precision", precision)])
    tr = NetTrainer()
    for k, v in pairs:
        if not k.startswith("metric"):
            tr.set_param(k, v)
    tr.init_model()
    losses = []
    lab = y.view(-1).long().cpu()
    for _ in range(steps):
        tr.update(DataBatch(x, y))
        # test-mode forward (no dropout): softmax probabilities of the last node
        p = torch.from_numpy(tr.forward_to([len(tr.net.nodes) - 1], DataBatch(x, y))[0]).reshape(batch, -1)
        losses.append(-torch.log(p.gather(1, lab.view(-1, 1)).clamp_min(1e-30)).mean().item())
    torch.cuda.synchronize()
    w = [c.layer.params[0].w.detach().float().clone() for c in tr.net.connections if c.layer.params and not c.shared]
    set_reference_precision(False)
    return losses, w


def test_alexnet_bf16_kernels_track_fp32_reference_on_gpu():
    batch, steps = 64, 6
    g = torch.Generator().manual_seed(11)
    x = torch.randn(batch, 3, 227, 227, generator=g).cuda()
    y = torch.randint(0, 1000, (batch, 1), generator=g).float().cuda()
    l16, w16 = _train("bf16", steps, batch, x, y)
    l32, w32 = _train("fp32", steps, batch, x, y)
    print("loss bf16", [round(v, 4) for v in l16])
    print("loss fp32", [round(v, 4) for v in l32])
    print("weight rel diff", [round(((a[..., :b.shape[-1]].reshape(b.shape) - b).norm() / b.norm()).item(), 5)
                              for a, b in zip(w16, w32)])
    for a, b in zip(l16, l32):
        assert abs(a - b) < 0.02 * abs(b) + 0.02, (l16, l32)
    for a, b in zip(w16, w32):
        a = a[..., :b.shape[-1]] if a.shape != b.shape else a
        rel = ((a.reshape(b.shape) - b).norm() / b.norm()).item()
        assert rel < 2e-2, rel


def test_fp32_mode_is_the_reference_path():
    """In fp32 mode the activations are fp32 on the device and no bf16 shadow weights exist."""
    pairs = load_conf("alexnet", [("batch_size", "4"), ("dev", "gpu"), ("silent", "1"), ("precision", "fp32")])
    tr = NetTrainer()
    for k, v in pairs:
        tr.set_param(k, v)
    tr.init_model()
    try:
        assert tr.net.nodes[1].data.dtype == torch.float32 and tr.net.nodes[1].data.is_cuda
        assert tr.net.arena.wb is None and not tr.net.ctx.is_gpu
    finally:
        set_reference_precision(False)


@pytest.mark.parametrize("model,shape", [("inception_v1", (3, 224, 224)), ("vgg16", (3, 224, 224)),
                                         ("bowl", (3, 40, 40)), ("mnist_conv", (1, 28, 28))])
def test_model_zoo_runs_in_fp32_mode(model, shape):
    """Every model of the zoo steps in reference precision on the GPU (concat / split / avg-pool /
    flatten reference paths on device tensors) and stays close to its bf16 run."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, *shape, generator=g).cuda()
    y = torch.randint(0, 10, (4, 1), generator=g).float().cuda()
    l16, w16 = _train("bf16", 2, 4, x, y, model)
    l32, w32 = _train("fp32", 2, 4, x, y, model)
    assert all(v == v for v in l32)
    for a, b in zip(w16, w32):
        a = a[..., :b.shape[-1]] if a.shape != b.shape else a
        assert ((a.reshape(b.shape) - b).norm() / b.norm()).item() < 5e-2
