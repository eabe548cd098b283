"""Which bias gradients a model's training step still leaves to the column-sum pass (the ones no
fused epilogue -- max-pool, LRN, data-gradient, weight-gradient -- sums on the way): one line per
ctx.bias_grad call of one step, with the bytes the pass re-reads.  GPU only.

    python tools/colsum_rows.py [--model vgg16] [--batch 64]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="vgg16")
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.layers.base import LayerContext as Context
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer

    log = []
    orig = Context.bias_grad

    def logged(self, dy2d, db, mask=None):
        log.append((tuple(dy2d.shape), dy2d.stride(0), mask is not None))
        return orig(self, dy2d, db, mask)
    Context.bias_grad = logged
    pairs = load_conf(a.model, [("batch_size", str(a.batch)), ("eval_train", "0"), ("dev", "gpu"), ("silent", "1")])
    tr = NetTrainer()
    for k, v in pairs:
        if not k.startswith("metric"):
            tr.set_param(k, v)
    tr.init_model()
    c, h, w = tr.net_cfg.input_shape
    batch = DataBatch(torch.randn(a.batch, c, h, w, device="cuda"), torch.zeros(a.batch, 1, device="cuda"))
    tr.update(batch)
    torch.cuda.synchronize()
    log.clear()
    tr.update(batch)
    torch.cuda.synchronize()
    total = 0
    for (rows, cols), ld, masked in log:
        mb = rows * cols * 2 / 1e6
        total += mb
        print(f"rows {rows:8d}  channels {cols:5d}  row stride {ld:5d}  {'pooled, masked' if masked else 'full':14s}"
              f"  {mb:8.1f} MB")
    print(f"{a.model} b{a.batch}: {len(log)} column sums, {total:.1f} MB re-read per step")


if __name__ == "__main__":
    main()
