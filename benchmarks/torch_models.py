"""Eager PyTorch-ROCm comparison for GoogLeNet (Inception-v1) and VGG-16 (BASELINE.json
configs 4 and 5), mirroring cxxnet_amd/models/confs/inception_v1.conf and vgg16.conf:
same layer shapes, ceil-mode pooling, LRN, dropout; SGD momentum 0.9; bf16 autocast,
channels_last (MIOpen convolutions, hipBLASLt GEMMs), synthetic 3x224x224 batches.

  python benchmarks/torch_models.py --model inception_v1 --batch 128
  python benchmarks/torch_models.py --model vgg16 --batch 64
Prints one JSON line with images/sec.
"""
import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


def conv(cin, cout, k, s=1, p=0):
    return nn.Sequential(nn.Conv2d(cin, cout, k, s, p), nn.ReLU(inplace=True))


class LRN(nn.Module):
    def forward(self, x):
        return F.local_response_norm(x, 5, 1e-4, 0.75, 1.0)


class Inception(nn.Module):
    def __init__(self, cin, c1, c3r, c3, c5r, c5, pp):
        super().__init__()
        self.b1 = conv(cin, c1, 1)
        self.b3 = nn.Sequential(conv(cin, c3r, 1), conv(c3r, c3, 3, 1, 1))
        self.b5 = nn.Sequential(conv(cin, c5r, 1), conv(c5r, c5, 5, 1, 2))
        self.bp = nn.Sequential(nn.MaxPool2d(3, 1, 1), conv(cin, pp, 1))

    def forward(self, x):
        return torch.cat([self.b1(x), self.b3(x), self.b5(x), self.bp(x)], 1)


def inception_v1():
    cfg = [(192, 64, 96, 128, 16, 32, 32), (256, 128, 128, 192, 32, 96, 64), "pool",
           (480, 192, 96, 208, 16, 48, 64), (512, 160, 112, 224, 24, 64, 64), (512, 128, 128, 256, 24, 64, 64),
           (512, 112, 144, 288, 32, 64, 64), (528, 256, 160, 320, 32, 128, 128), "pool",
           (832, 256, 160, 320, 32, 128, 128), (832, 384, 192, 384, 48, 128, 128)]
    layers = [conv(3, 64, 7, 2, 3), nn.MaxPool2d(3, 2, ceil_mode=True), LRN(), conv(64, 64, 1),
              conv(64, 192, 3, 1, 1), LRN(), nn.MaxPool2d(3, 2, ceil_mode=True)]
    for c in cfg:
        layers.append(nn.MaxPool2d(3, 2, ceil_mode=True) if c == "pool" else Inception(*c))
    layers += [nn.AvgPool2d(7, 1), nn.Flatten(), nn.Dropout(0.4), nn.Linear(1024, 1000)]
    return nn.Sequential(*layers)


def vgg16():
    layers, cin = [], 3
    for v in [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]:
        if v == "M":
            layers.append(nn.MaxPool2d(2, 2))
        else:
            layers.append(conv(cin, v, 3, 1, 1))
            cin = v
    layers += [nn.Flatten(), nn.Linear(25088, 4096), nn.ReLU(inplace=True), nn.Dropout(0.5),
               nn.Linear(4096, 4096), nn.ReLU(inplace=True), nn.Dropout(0.5), nn.Linear(4096, 1000)]
    return nn.Sequential(*layers)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="inception_v1", choices=["inception_v1", "vgg16"])
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    model = (inception_v1() if a.model == "inception_v1" else vgg16()).to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=2e-4)
    x = torch.randn(a.batch, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    print(json.dumps({"impl": "torch-eager", "model": a.model, "batch": a.batch,
                      "ms_per_step": round(el / a.steps * 1000, 3),
                      "images_per_sec": round(a.batch * a.steps / el, 1)}), flush=True)


if __name__ == "__main__":
    main()
