"""Diagnostic: per-node forward and per-parameter gradient comparison CPU(fp32) vs GPU(bf16)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cxxnet_amd.models import load_conf
from cxxnet_amd.nnet import NetTrainer

model = sys.argv[1] if len(sys.argv) > 1 else "alexnet"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 4
pairs = [(k, v) for k, v in load_conf(model) if not k.startswith("metric") and k != "dev"]
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
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()

for i, (nc, ng) in enumerate(zip(cpu.net.nodes, gpu.net.nodes)):
    a = nc.data[..., : nc.shape[1]] if nc.shape[1] > 1 else nc.data
    b = ng.data[..., : nc.shape[1]] if nc.shape[1] > 1 else ng.data
    print(f"fwd node {i:2d} {nc.name:>6} shape={nc.shape} rel={rel(b, a):.3e}")
for tr in (cpu, gpu):
    tr.net.backprop(False)
torch.cuda.synchronize()
for (li, sc), (_, sg) in zip(cpu.net.arena.specs, gpu.net.arena.specs):
    gc = sc.g; gg = sg.g[..., : sc.shape[-1]]
    err = (gg.float().cpu() - gc).abs()
    idx = int(err.reshape(-1).argmax())
    print(f"grad layer {li:2d} {sc.tag} rel={rel(gg, gc):.3e} argmax={idx} cpu={gc.reshape(-1)[idx]:.4e} gpu={gg.reshape(-1)[idx].item():.4e} maxabs={gc.abs().max():.3e}")
# direct check of the fused relu-mask data-grad epilogue
from cxxnet_amd import ops
B, nin, nout = 4, 4096, 1000
gg = torch.Generator().manual_seed(3)
dy = torch.randn(B, nout, generator=gg).to(torch.bfloat16).float()
w = (torch.randn(nout, nin, generator=gg) * 0.02).to(torch.bfloat16).float()
old = torch.randn(B, nin, generator=gg).clamp_min(0).to(torch.bfloat16).float()
ref = (dy @ w) * (old > 0).float()
dxg = old.cuda().to(torch.bfloat16)
ops.fc_backward_data(dy.cuda().to(torch.bfloat16), w.cuda().to(torch.bfloat16), dxg, mask_relu=True)
torch.cuda.synchronize()
print("mask epilogue rel", rel(dxg, ref))
