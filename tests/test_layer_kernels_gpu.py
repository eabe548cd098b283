"""GPU kernels of batch_norm, prelu, insanity, insanity_max_pooling, bias, split, concat
(csrc/kernels/layer_kernels.hip, nn_kernels.hip) against the CPU executor's fp32 torch
formulas.  Random draws use the same counter hash on both devices, so even the
training-mode (noisy) paths compare element by element.  Inputs are bf16-representable,
so max-pool winners agree exactly."""
import pytest
import torch

from cxxnet_amd.io.data import DataBatch
from cxxnet_amd.ops import layer_ops as L

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).float()


def relerr(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def test_batch_norm_fwd_bwd():
    rows, C = 2 * 7 * 7, 24
    x = rnd(rows, C, scale=2.0, seed=1) + 0.5
    g = rnd(rows, C, seed=2)
    slope, bias = rnd(C, seed=3) + 1.0, rnd(C, seed=4)
    res = {}
    for dev in ("cpu", DEV):
        dt = torch.float32 if dev == "cpu" else torch.bfloat16
        st = L.BNState(C, dev)
        xd, yd = x.to(dev, dt).clone(), torch.empty(rows, C, device=dev, dtype=dt)
        L.bn_forward(xd, yd, slope.to(dev), bias.to(dev), 1e-10, st, True)
        gs, gb = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dx = g.to(dev, dt).clone()
        L.bn_backward(dx, xd, slope.to(dev), gs, gb, st, True)  # dx written into the x-hat node
        res[dev] = (yd, st.mean, st.inv, xd, gs, gb)
    torch.cuda.synchronize()
    for a, b in zip(res[DEV], res["cpu"]):
        assert relerr(a, b) < 2e-2


@pytest.mark.parametrize("noise", [0.0, 0.3])
def test_prelu(noise):
    rows, C = 3 * 5 * 5, 16
    x, g = rnd(rows, C, seed=5), rnd(rows, C, seed=6)
    slope = torch.rand(C, generator=torch.Generator().manual_seed(7)) * 0.5
    out = {}
    for dev in ("cpu", DEV):
        dt = torch.float32 if dev == "cpu" else torch.bfloat16
        ctr = torch.tensor([3], dtype=torch.int32, device=dev)
        xd, y = x.to(dev, dt).clone(), torch.empty(rows, C, device=dev, dtype=dt)
        L.prelu_forward(xd, y, slope.to(dev), 1234, ctr, noise)
        gs = torch.zeros(C, device=dev)
        L.prelu_backward(xd, g.to(dev, dt), xd, slope.to(dev), gs, 1234, ctr, noise, True)
        out[dev] = (y, gs, xd)
    torch.cuda.synchronize()
    for a, b in zip(out[DEV], out["cpu"]):
        assert relerr(a, b) < 2e-2


@pytest.mark.parametrize("train", [True, False])
def test_insanity(train):
    n = 4 * 6 * 6 * 8
    x, g = rnd(n, seed=8), rnd(n, seed=9)
    out = {}
    for dev in ("cpu", DEV):
        dt = torch.float32 if dev == "cpu" else torch.bfloat16
        ctr = torch.tensor([11], dtype=torch.int32, device=dev)
        xd, y2 = x.to(dev, dt).clone(), torch.empty(n, device=dev, dtype=dt)
        L.insanity_forward(xd, xd, y2, 3.0, 8.0, train, 99, ctr)
        L.insanity_backward(xd, g.to(dev, dt), xd, 3.0, 8.0, train, 99, ctr)
        out[dev] = (y2, xd)
    torch.cuda.synchronize()
    for a, b in zip(out[DEV], out["cpu"]):
        assert relerr(a, b) < 2e-2
    # the draws really are random in training (not the test-time constant divisor)
    neg = x < 0
    ratio = (x[neg] / out["cpu"][0][neg]).float()
    assert (ratio.std() > 0.5) == train


@pytest.mark.parametrize("keep", [0.6, 1.0])
def test_insanity_pooling(keep):
    N, H, W, C, K, S = 2, 9, 9, 8, 3, 2
    Ho = Wo = (H - K + S - 1) // S + 1
    x, gy = rnd(N, H, W, C, seed=10), rnd(N, Ho, Wo, C, seed=11)
    out = {}
    for dev in ("cpu", DEV):
        dt = torch.float32 if dev == "cpu" else torch.bfloat16
        ctr = torch.tensor([5], dtype=torch.int32, device=dev)
        xd = x.to(dev, dt)
        y = torch.empty(N, Ho, Wo, C, device=dev, dtype=dt)
        ys = torch.empty_like(y)
        L.ins_pool_forward(xd, y, ys, K, S, keep, 77, ctr)
        dx = torch.empty_like(xd)
        L.ins_pool_backward(xd, ys, gy.to(dev, dt), dx, K, S, keep, 77, ctr)
        out[dev] = (y, dx)
    torch.cuda.synchronize()
    assert torch.equal(out[DEV][0].float().cpu(), out["cpu"][0])  # exact: max over bf16 values
    assert relerr(out[DEV][1], out["cpu"][1]) < 2e-2


EXOTIC = """
netconfig=start
layer[0->1] = conv:c1
  kernel_size = 3
  nchannel = 16
  pad = 1
  no_bias = 1
layer[1->2] = batch_norm:bn1
layer[2->3] = prelu:pr1
  random = 0.2
layer[3->4,5] = split
layer[4->6] = conv:c2a
  kernel_size = 1
  nchannel = 8
layer[5->7] = conv:c2b
  kernel_size = 3
  nchannel = 8
  pad = 1
layer[6,7->8] = ch_concat
layer[8->9] = avg_pooling
  kernel_size = 2
  stride = 2
layer[9->10] = flatten
layer[10->11] = fullc:f1
  nhidden = 32
layer[11->11] = bias:b1
layer[11->12] = insanity
  lb = 3
  ub = 8
layer[12->13] = fullc:f2
  nhidden = 10
layer[13->13] = softmax
netconfig=end
input_shape = 8,8,8
random_type = xavier
eta = 0.1
momentum = 0.9
"""


def test_exotic_net_gpu_vs_cpu():
    """Two training steps of a net using every layer above: GPU (HIP kernels) == CPU.  (c1 has
    no bias: ahead of batch_norm its gradient is identically zero up to rounding noise.)"""
    from cxxnet_amd import native
    from cxxnet_amd.nnet import NetTrainer

    def make(dev):
        tr = NetTrainer()
        for k, v in list(native.rt().parse_config(EXOTIC)) + [("batch_size", "4"), ("dev", dev), ("seed", "2"),
                                                              ("silent", "1"), ("eval_train", "0")]:
            tr.set_param(k, v)
        tr.init_model()
        return tr

    cpu, gpu = make("cpu"), make("gpu")
    cpu.net.arena.w.copy_(cpu.net.arena.w.to(torch.bfloat16).float())
    for (_, sc), (_, sg) in zip(cpu.net.arena.specs, gpu.net.arena.specs):
        sg.w.copy_(sc.w)
    gpu.net.arena.sync_shadow()
    x = rnd(4, 8, 8, 8, seed=12)
    y = torch.randint(0, 10, (4, 1), generator=torch.Generator().manual_seed(13)).float()
    for _ in range(2):
        cpu.update(DataBatch(x, y))
        gpu.update(DataBatch(x.to(DEV), y.to(DEV)))
    torch.cuda.synchronize()
    pc, pg = cpu.net.nodes[-1].fp32_view, gpu.net.nodes[-1].fp32_view
    assert torch.isfinite(pg).all()
    assert relerr(pg, pc) < 0.05
    errs = {}
    for (li, sc), (_, sg) in zip(cpu.net.arena.specs, gpu.net.arena.specs):
        mc = cpu.net.arena.m1[sc.offset:sc.offset + sc.numel]
        mg = gpu.net.arena.m1[sg.offset:sg.offset + sg.numel]
        errs[(li, cpu.net.connections[li].layer.type_name, sc.tag)] = round(relerr(mg, mc), 4)
    assert max(errs.values()) < 0.1, errs


@pytest.mark.parametrize("nd", [1, 2, 3, 4, 5, 7])
def test_split_fanout_and_sum_kernels(nd):
    """split forward (one read, up to 4 writes per launch) and backward (fp32 sum of up
    to 4 gradients per launch) against torch."""
    from cxxnet_amd import ops
    g = torch.Generator().manual_seed(nd)
    x = torch.randn(3, 7, 5, 24, generator=g).to(torch.bfloat16).cuda()
    outs = [torch.empty_like(x) for _ in range(nd)]
    ops.fanout_copy(x, outs)
    for o in outs:
        assert torch.equal(o, x)
    grads = [torch.randn(x.shape, generator=g).to(torch.bfloat16).cuda() for _ in range(nd)]
    y = torch.empty_like(x)
    ops.sum_into(y, grads)
    ref = torch.stack([t.float() for t in grads]).sum(0)
    assert (y.float() - ref).abs().max().item() <= 0.02 * ref.abs().max().item() + 1e-6


@pytest.mark.parametrize("dist,a,b", [("normal", 0.0, 0.01), ("uniform", -0.05, 0.05), ("normal", 0.3, 2.0)])
def test_rand_fill_device_matches_host(dist, a, b):
    """Weight init on the device (rand_fill kernel) draws what the host mirror draws: the
    same integer hash, float32 Box-Muller (a few ulps apart through logf / cosf)."""
    n = 1 << 20 | 77
    gpu = L.rand_fill(torch.empty(n, device=DEV), 1234, dist, a, b).cpu()
    cpu = L.rand_fill(torch.empty(n), 1234, dist, a, b)
    assert (gpu - cpu).abs().max().item() <= 1e-5 * max(abs(a), abs(b), 1.0)
    if dist == "normal":
        assert abs(gpu.mean().item() - a) < 5e-3 * b and abs(gpu.std().item() / b - 1) < 5e-3
    else:
        assert gpu.min().item() >= a and gpu.max().item() < b


def test_model_init_on_device_matches_cpu_model():
    """A GPU model and a CPU model of one seed start from the same weights (device RNG)."""
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer

    ws = []
    for dev in ("gpu", "cpu"):
        pairs = load_conf("alexnet", [("batch_size", "2"), ("dev", dev), ("silent", "1")])
        tr = NetTrainer()
        for k, v in pairs:
            tr.set_param(k, v)
        tr.init_model()
        ws.append([c.layer.params[0].w.detach().float().cpu().clone() for c in tr.net.connections
                   if c.layer.params and not c.shared])
    for g, c in zip(*ws):
        gg, cc = g[..., :c.shape[-1]] if g.shape != c.shape else g, c
        assert (gg.reshape(cc.shape) - cc).abs().max().item() <= 1e-6 + 1e-5 * cc.abs().max().item()
