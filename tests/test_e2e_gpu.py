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
    # norm-relative error: robust to the few relu-mask / max-pool winners that legitimately
    # differ where values are within bf16 rounding of each other
    a, b = a.float().cpu().reshape(-1), b.float().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _pairs(model, batch, **over):
    pairs = [(k, v) for k, v in load_conf(model) if not k.startswith("metric") and k != "dev"]
    pairs += [("batch_size", str(batch)), ("eval_train", "0"), ("silent", "1")]
    pairs = [(k, over.get(k, v)) for k, v in pairs]
    return pairs + [(k, v) for k, v in over.items()]


def test_gpu_matches_cpu_one_step():
    batch = 8
    pairs = _pairs("alexnet", batch, threshold="0")  # dropout off: same function on both devices
    # Max-pool winners legitimately differ between bf16 and fp32 activations in ~10% of
    # windows (top-2 within bf16 rounding); avg pooling keeps the comparison about the
    # wiring and the kernels (max-pool winners are checked exactly in test_kernels_gpu).
    pairs = [(k, "avg_pooling" if v == "max_pooling" else v) for k, v in pairs]
    cpu = _trainer(pairs, "cpu")
    gpu = _trainer(pairs, "gpu")
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
        assert _rel(mg, mc) < 0.1, (li, sc.tag, _rel(mg, mc))


def _loss(tr, y):
    p = tr.net.nodes[-1].fp32_view
    return -torch.log(p[torch.arange(p.shape[0]), y.view(-1).long()] + 1e-12).mean().item()


def test_alexnet_loss_decreases_on_fixed_batch():
    pairs = _pairs("alexnet", 16, threshold="0", **{"wmat:lr": "0.001", "bias:lr": "0.002"})
    tr = _trainer(pairs, "gpu")
    c, h, w = tr.net_cfg.input_shape
    g = torch.Generator().manual_seed(1)
    x = torch.randn(16, c, h, w, generator=g).cuda()
    y = torch.randint(0, 10, (16, 1), generator=g).float().cuda()
    losses = []
    for _ in range(25):
        tr.update(DataBatch(x, y))
        losses.append(_loss(tr, y))
    assert all(l == l for l in losses), losses
    assert min(losses[-8:]) < 0.7 * losses[0], losses


def test_dropout_step_counter_changes_mask_on_gpu():
    pairs = _pairs("alexnet", 4)
    tr = _trainer(pairs, "gpu")
    c, h, w = tr.net_cfg.input_shape
    x = torch.randn(4, c, h, w).cuda()
    y = torch.zeros(4, 1).cuda()
    tr.net.set_input(x)
    tr.net.set_labels(y)
    tr.net.forward(True)
    a = tr.net.nodes[18].data.clone()
    tr.net.forward(True)
    b = tr.net.nodes[18].data.clone()
    za, zb = (a == 0), (b == 0)
    assert (za != zb).float().mean().item() > 0.1  # a fresh mask each step


@pytest.mark.parametrize("model,batch", [("alexnet", 16), ("inception_v1", 8)])
def test_cuda_graph_step_matches_eager(model, batch):
    """cuda_graph=1 (forward and backward as HIP-graph replays, eager optimizer) trains
    the same weights as the eager step: fresh batches each step (input staging), dropout
    masks that change per step (device step counter), an lr schedule that moves every
    update (expdecay: the optimizer must stay outside the graph)."""
    over = {"eval_train": "1", "metric": "error", "lr:schedule": "expdecay", "lr:gamma": "0.5", "lr:step": "2"}
    eager = _trainer(_pairs(model, batch, **over), "gpu")
    graph = _trainer(_pairs(model, batch, cuda_graph="1", **over), "gpu")
    graph.net.arena.w.copy_(eager.net.arena.w)
    graph.net.arena.sync_shadow()
    c, h, w = eager.net_cfg.input_shape
    g = torch.Generator().manual_seed(3)
    for _ in range(4):
        x = torch.randn(batch, c, h, w, generator=g).cuda()
        y = torch.randint(0, 1000, (batch, 1), generator=g).float().cuda()
        eager.update(DataBatch(x, y))
        graph.update(DataBatch(x, y))
    torch.cuda.synchronize()
    assert len(graph._graphs) == 1, "the graph path did not capture"
    assert int(graph.net.ctx.step_counter.item()) == int(eager.net.ctx.step_counter.item()) == 4
    # the whole optimizer state after 4 steps (atomic weight-grad epilogues: not bitwise)
    assert _rel(graph.net.arena.m1, eager.net.arena.m1) < 0.05
    assert _rel(graph.net.arena.w, eager.net.arena.w) < 1e-3
    assert "train-error" in graph.train_metric.print("train")


def test_profile_step_timers_and_nonfinite_check_on_gpu():
    """profile_step = 1: HIP-event fwd / bwd / opt timings; check_nonfinite = 1: the
    device flag kernel catches a NaN gradient."""
    pairs = _pairs("alexnet", 8, profile_step="1", check_nonfinite="1")
    tr = _trainer(pairs, "gpu")
    c, h, w = tr.net_cfg.input_shape
    x = torch.randn(8, c, h, w).cuda()
    y = torch.zeros(8, 1).cuda()
    for _ in range(3):
        tr.update(DataBatch(x, y))
    rep = tr.timing_report()
    assert "fwd" in rep and "img/s" in rep, rep
    x[0, 0, 0, 0] = float("nan")
    with pytest.raises(FloatingPointError):
        tr.update(DataBatch(x, y))


def test_trace_layers_ranges_run_on_gpu():
    pairs = _pairs("alexnet", 4, trace_layers="1", threshold="0")
    tr = _trainer(pairs, "gpu")
    assert tr.net.trace_layers == 1
    c, h, w = tr.net_cfg.input_shape
    tr.update(DataBatch(torch.randn(4, c, h, w).cuda(), torch.zeros(4, 1).cuda()))
    torch.cuda.synchronize()


def test_device_metrics_match_host_metrics():
    """GPU training / eval metrics accumulate on the device (DeviceMetricSet); they must
    equal the native host metrics computed from the same scores read back to the host."""
    from cxxnet_amd.utils.metric import DeviceMetricSet, MetricSet
    batch = 16
    pairs = _pairs("alexnet", batch, eval_train="1") + [("metric", "error"), ("metric", "logloss"),
                                                          ("metric", "rec@5")]
    tr = _trainer(pairs, "gpu")
    assert isinstance(tr.train_metric, DeviceMetricSet)
    c, h, w = tr.net_cfg.input_shape
    g = torch.Generator().manual_seed(3)
    x = torch.randn(batch, c, h, w, generator=g).cuda()
    y = torch.randint(0, 1000, (batch, 1), generator=g).float().cuda()
    b = DataBatch(x, y)
    scores = tr.forward_to([len(tr.net.nodes) - 1], b)[0].reshape(batch, -1)
    host = MetricSet()
    for n in ("error", "logloss", "rec@5"):
        host.add_metric(n)
    host.add_eval([scores] * 3, {"label": y.cpu().numpy()})
    tr.metric.clear()
    tr._set_batch(b)
    tr.net.forward(False)
    tr.metric.add_eval(tr._eval_scores(), tr.net.ctx.label_fields)
    hv = [float(s.split(":")[1]) for s in host.print("t").split("\t")[1:]]
    dv = tr.metric.values()
    assert all(abs(a - b_) <= 1e-4 * max(1.0, abs(a)) for a, b_ in zip(hv, dv)), (hv, dv)
    # training-time accumulation: no host copy per step, one line on print
    for _ in range(3):
        tr.update(b)
    line = tr.evaluate(None, "train")
    assert line.count("train-") == 3 and "nan" not in line


@pytest.mark.parametrize("zc", ["1", "0"])
def test_zero_copy_split_and_concat_relu_fusion_match_unfused(monkeypatch, zc):
    """GoogLeNet graph: zero-copy split (outputs alias the input, data-grads go to private
    grad buffers) and relu fused into the conv epilogue in front of ch_concat -- with zc=1 the
    zero-copy concat (branch convs write into channel slices of the concat output, strided
    GEMM epilogues / gradient reads / bias sums, relu' applied by the split sum and the pools),
    with zc=0 the relu'-masked gradient copy -- must compute what the unfused executor computes."""
    batch = 4
    pairs = _pairs("inception_v1", batch)
    monkeypatch.setenv("CXXNET_CONCAT_ZC", zc)
    fused = _trainer(pairs, "gpu")
    monkeypatch.setenv("CXXNET_FUSE", "0")
    plain = _trainer(pairs, "gpu")
    monkeypatch.delenv("CXXNET_FUSE")
    net = fused.net
    assert any(getattr(c.layer, "alias", False) for c in net.connections), "no split was aliased"
    nzc = sum(bool(getattr(c.layer, "zero_copy", False)) for c in net.connections)
    if zc == "1":
        assert nzc == 9, nzc  # every inception concat
    else:
        assert nzc == 0
        assert any(getattr(c.layer, "grad_mask_inputs", None) for c in net.connections), "no concat relu fusion"
    assert not any(getattr(c.layer, "alias", False) for c in plain.net.connections)
    # per tensor: sibling groups (NeuralNet._fuse_siblings) lay the fused arena out differently
    src = {(li, sp.tag): sp.w for li, sp in fused.net.arena.specs}
    for li, sp in plain.net.arena.specs:
        sp.w.copy_(src[(li, sp.tag)])
    plain.net.arena.sync_shadow()
    c, h, w = fused.net_cfg.input_shape
    g = torch.Generator().manual_seed(1)
    x = torch.randn(batch, c, h, w, generator=g).cuda()
    y = torch.randint(0, 1000, (batch, 1), generator=g).float().cuda()
    for _ in range(2):
        fused.update(DataBatch(x, y))
        plain.update(DataBatch(x, y))
    torch.cuda.synchronize()
    def canon(tr, buf):  # every tensor's slice of an arena buffer, in (layer, tag) order
        return torch.cat([buf[sp.offset:sp.offset + sp.numel] for _, sp in sorted(tr.net.arena.specs,
                                                                                   key=lambda t: (t[0], t[1].tag))])
    assert _rel(canon(plain, plain.net.arena.m1), canon(fused, fused.net.arena.m1)) < 1e-2
    assert _rel(canon(plain, plain.net.arena.w), canon(fused, fused.net.arena.w)) < 1e-4


def _traj(tr, batches):
    losses = []
    for x, y in batches:
        tr.update(DataBatch(x, y))
        line = tr.evaluate(None, "train")
        losses.append(float(line.split("train-logloss:")[1].split("\t")[0]))
    return losses


def _wdist(a, b, w0):
    """Per-layer weight discrepancy relative to the distance trained from the common start."""
    out = []
    for (li, sa), (_, sb), (_, s0) in zip(a.net.arena.specs, b.net.arena.specs, w0):
        wa = sa.w.detach().float().cpu()
        wb = sb.w.detach().float().cpu()[..., : wa.shape[-1]]
        d0 = s0[..., : wa.shape[-1]]
        out.append(((wa - wb).norm() / (wa - d0).norm().clamp_min(1e-12)).item())
    return out


@pytest.mark.timeout(600)
def test_alexnet_trajectory_gpu_vs_cpu_fp32():
    """The real AlexNet graph -- max pooling, LRN, dropout ON, relu fusion -- at batch 64 for 10
    SGD steps on the GPU (bf16 activations, HIP kernels) against the CPU fp32 executor started
    from the same (bf16-representable) weights with identical dropout masks (counter hash).

    Tolerances come from a measured noise floor: the same CPU fp32 run restarted with
    bf16-rounded inputs and one bf16 ulp of weight noise diverges from the reference by
    `floor`; the GPU run must stay within a small multiple of it."""
    batch, steps = 64, 10
    pairs = _pairs("alexnet", batch, eval_train="1") + [("metric", "logloss")]
    cpu = _trainer(pairs, "cpu")
    cpu2 = _trainer(pairs, "cpu")
    gpu = _trainer(pairs, "gpu")
    cpu.net.arena.w.copy_(cpu.net.arena.w.to(torch.bfloat16).float())
    g = torch.Generator().manual_seed(11)
    noise = torch.randn(cpu.net.arena.w.shape, generator=g)
    cpu2.net.arena.w.copy_(cpu.net.arena.w * (1.0 + noise * 2.0 ** -9))  # ~1 bf16 ulp
    for (_, sc), (_, sg) in zip(cpu.net.arena.specs, gpu.net.arena.specs):
        sg.w.zero_()
        sg.w[..., : sc.shape[-1]].copy_(sc.w)
    gpu.net.arena.sync_shadow()
    w0 = [(li, s.w.detach().clone()) for li, s in cpu.net.arena.specs]
    c, h, w = cpu.net_cfg.input_shape
    data = []
    for _ in range(steps):
        x = torch.randn(batch, c, h, w, generator=g).to(torch.bfloat16).float()
        y = torch.randint(0, 1000, (batch, 1), generator=g).float()
        data.append((x, y))
    l_cpu = _traj(cpu, data)
    l_cpu2 = _traj(cpu2, [(x.to(torch.bfloat16).float(), y) for x, y in data])
    l_gpu = _traj(gpu, [(x.cuda(), y.cuda()) for x, y in data])
    torch.cuda.synchronize()
    floor_loss = max(abs(a - b) / a for a, b in zip(l_cpu, l_cpu2))
    err_loss = max(abs(a - b) / a for a, b in zip(l_cpu, l_gpu))
    floor_w = _wdist(cpu, cpu2, w0)
    err_w = _wdist(cpu, gpu, w0)
    print(f"\nloss cpu {l_cpu}\nloss gpu {l_gpu}\nrel loss err {err_loss:.3g} (floor {floor_loss:.3g})\n"
          f"weight err per layer {[round(v, 4) for v in err_w]}\nfloor {[round(v, 4) for v in floor_w]}")
    assert l_gpu[-1] < l_gpu[0]  # it trains
    # measured on MI355X (round 2): loss error 4.7x the floor (0.0075 vs 0.0016); per
    # layer weight error 1.0-1.4x the floor (e.g. conv3 0.165 vs 0.140, fc7 0.264 vs 0.218)
    assert err_loss < 8 * floor_loss
    for e, f in zip(err_w, floor_w):
        assert e < 2 * f + 0.02, (err_w, floor_w)
