"""Layer-by-layer backprop comparison CPU(fp32) vs GPU(bf16)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cxxnet_amd.models import load_conf
from cxxnet_amd.nnet import NetTrainer
batch = 8
pairs = [(k, v) for k, v in load_conf("alexnet") if not k.startswith("metric") and k != "dev"]
pairs += [("batch_size", str(batch)), ("eval_train", "0"), ("silent", "1")]
pairs = [(k, ("0" if k == "threshold" else v)) for k, v in pairs]
def mk(dev):
    tr = NetTrainer()
    for k, v in pairs + [("dev", dev), ("seed", "7")]:
        tr.set_param(k, v)
    tr.init_model()
    return tr
cpu, gpu = mk("cpu"), mk("gpu")
cpu.net.arena.w.copy_(cpu.net.arena.w.to(torch.bfloat16).float())
for (_, sc), (_, sg) in zip(cpu.net.arena.specs, gpu.net.arena.specs):
    sg.w.zero_(); sg.w[..., : sc.shape[-1]].copy_(sc.w)
gpu.net.arena.sync_shadow()
c, h, w = cpu.net_cfg.input_shape
g = torch.Generator().manual_seed(0)
x = torch.randn(batch, c, h, w, generator=g).to(torch.bfloat16).float()
y = torch.randint(0, 1000, (batch, 1), generator=g).float()
for tr, xx, yy in ((cpu, x, y), (gpu, x.cuda(), y.cuda())):
    tr.net.set_input(xx); tr.net.set_labels(yy); tr.net.forward(True)
def rel(a, b):
    a = a.float().cpu().reshape(-1); b = b.float().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
print("label gpu", gpu.net.ctx.label_fields["label"].view(-1).tolist(), "cpu", cpu.net.ctx.label_fields["label"].view(-1).tolist())
for i in range(len(cpu.net.connections) - 1, 0, -1):
    cc, gc = cpu.net.connections[i], gpu.net.connections[i]
    cc.layer.backprop(True, cc.nodes_in, cc.nodes_out)
    gc.layer.backprop(True, gc.nodes_in, gc.nodes_out)
    torch.cuda.synchronize()
    for nc, ng in zip(cc.nodes_in, gc.nodes_in):
        print(f"after layer {i:2d} {type(cc.layer).__name__:>18} fused={getattr(gc.layer,'fused_into_producer',None)} mask={gc.layer.grad_mask_relu} in-node {nc.name}: rel={rel(ng.data, nc.data):.3e} maxabs={nc.data.abs().max():.3e}/{ng.data.float().abs().max():.3e}")
