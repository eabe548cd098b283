"""End-to-end GPU checks: the GPU executor (HIP kernels, bf16, fused relu) against the
CPU executor (fp32 torch reference) on the same weights and batch."""
import pytest
import torch

from cxxnet_amd import native
from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.models import load_conf
from cxxnet_amd.nnet import NetTrainer

pytestmark = pytest.mark.gpu


def _trainer(pairs, dev):
    tr = NetTrainer()
    for k, v in pairs + [("dev", dev), ("seed", "7")]:
        tr.set_param(k, v)
    tr.init_model()
    return tr


def _rel(a, b):
    # norm-relative error: robust to the few relu-mask flips where a pre-activation is
    # within bf16 rounding of zero (those legitimately differ between bf16 and fp32)
    a, b = a.float().cpu().reshape(-1), b.float().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("model,batch", [("alexnet", 4)])
def test_gpu_matches_cpu_one_step(model, batch):
    pairs = [(k, v) for k, v in load_conf(model) if not k.startswith("metric") and k != "dev"]
    pairs += [("batch_size", str(batch)), ("eval_train", "0"), ("silent", "1")]
    # dropout off so both devices see the same function
    pairs = [(k, ("0" if k == "threshold" else v)) for k, v in pairs]
    cpu = _trainer(pairs, "cpu")
    gpu = _trainer(pairs, "gpu")
    # round CPU weights to bf16 as the GPU computes with bf16 copies
    cpu.net.arena.w.copy_(cpu.net.arena.w.to(torch.bfloat16).float())
    for (_, sc), (_, sg) in zip(cpu.net.arena.specs, gpu.net.arena.specs):
        sg.w.zero_()
        sg.w[..., : sc.shape[-1]].copy_(sc.w)  # first conv: GPU pads input channels 3 -> 4
    gpu.net.arena.sync_shadow()
    c, h, w = cpu.net_cfg.input_shape
    g = torch.Generator().manual_seed(0)
    x = torch.randn(batch, c, h, w, generator=g).to(torch.bfloat16).float()
    y = torch.randint(0, 1000, (batch, 1), generator=g).float()
    cpu.update(DataBatch(x, y))
    gpu.update(DataBatch(x.cuda(), y.cuda()))
    torch.cuda.synchronize()
    # momentum buffer == -lr * (grad + wd w) after one step: compare it per segment
    for (li, sc), (_, sg) in zip(cpu.net.arena.specs, gpu.net.arena.specs):
        mc = cpu.net.arena.m1[sc.offset:sc.offset + sc.numel].view(sc.shape)
        mg = gpu.net.arena.m1[sg.offset:sg.offset + sg.numel].view(sg.shape)[..., : sc.shape[-1]]
        if mc.abs().max() < 1e-12:
            continue
        assert _rel(mg, mc) < 5e-2, (li, sc.tag, _rel(mg, mc))


def test_alexnet_trains_on_fixed_batch():
    pairs = [(k, v) for k, v in load_conf("alexnet") if not k.startswith("metric") and k != "dev"]
    pairs += [("batch_size", "32"), ("eval_train", "1"), ("silent", "1"), ("metric", "error"),
              ("wmat:lr", "0.01"), ("bias:lr", "0.01")]
    tr = _trainer(pairs, "gpu")
    c, h, w = tr.net_cfg.input_shape
    g = torch.Generator().manual_seed(1)
    x = torch.randn(32, c, h, w, generator=g).cuda()
    y = torch.randint(0, 10, (32, 1), generator=g).float().cuda()
    errs = []
    for r in range(30):
        tr.update(DataBatch(x, y))
        errs.append(float(tr.evaluate(None, "t").split(":")[-1]))
    assert min(errs[-5:]) < 0.5, errs
