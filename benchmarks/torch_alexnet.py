"""Eager PyTorch-ROCm reference for the comparison baseline (BASELINE.md plan item 1):
the same AlexNet (example/ImageNet/ImageNet.conf: grouped conv2/4/5, LRN, ceil-mode
max-pooling, dropout 0.5) trained with torch.optim.SGD(momentum 0.9, wd 5e-4) in bf16
(weights fp32 via autocast), channels_last, MIOpen convolutions, hipBLASLt GEMMs,
synthetic 3x227x227 batches on the device.

  python benchmarks/torch_alexnet.py --batch 256 --steps 20 --warmup 5 [--compile 0]
Prints one JSON line with images/sec.
"""
import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class LRN(nn.Module):
    def __init__(self, n=5, alpha=1e-3, beta=0.75, k=1.0):
        super().__init__()
        self.n, self.alpha, self.beta, self.k = n, alpha, beta, k

    def forward(self, x):
        # cxxnet normalises alpha by n (lrn_layer-inl.hpp:53-56), as does torch's local_response_norm
        return F.local_response_norm(x, self.n, self.alpha, self.beta, self.k)


def alexnet():
    return nn.Sequential(
        nn.Conv2d(3, 96, 11, 4), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2, ceil_mode=True), LRN(),
        nn.Conv2d(96, 256, 5, 1, 2, groups=2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2, ceil_mode=True), LRN(),
        nn.Conv2d(256, 384, 3, 1, 1), nn.ReLU(inplace=True),
        nn.Conv2d(384, 384, 3, 1, 1, groups=2), nn.ReLU(inplace=True),
        nn.Conv2d(384, 256, 3, 1, 1, groups=2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2, ceil_mode=True),
        nn.Flatten(),
        nn.Linear(9216, 4096), nn.ReLU(inplace=True), nn.Dropout(0.5),
        nn.Linear(4096, 4096), nn.ReLU(inplace=True), nn.Dropout(0.5),
        nn.Linear(4096, 1000))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--compile", type=int, default=0)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    model = alexnet().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
    if a.compile:
        model = torch.compile(model)
    x = torch.randn(a.batch, 3, 227, 227, device=dev).to(memory_format=torch.channels_last)
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
    print(json.dumps({"impl": "torch-eager" + ("+compile" if a.compile else ""), "batch": a.batch,
                      "ms_per_step": round(el / a.steps * 1000, 3),
                      "images_per_sec": round(a.batch * a.steps / el, 1)}), flush=True)


if __name__ == "__main__":
    main()
