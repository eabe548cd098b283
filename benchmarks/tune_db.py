"""Build the gfx950 GEMM tile database (cxxnet_amd/ops/glds_tune_gfx950.json): run a few
training steps of each model at its benchmark batch so every GEMM signature is timed once,
then write the table.

  python benchmarks/tune_db.py [--models alexnet:256,inception_v1:64] [--out path] [--keep]

--keep extends the shipped table instead of re-timing it: only signatures it does not hold
(e.g. the conv weight-grad split-K "cws" keys) are timed.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="alexnet:256,alexnet:32,alexnet:128,inception_v1:64,vgg16:32,mnist_conv:100,"
                                        "bowl:64")
    ap.add_argument("--out", default="")
    ap.add_argument("--keep", action="store_true", help="keep the shipped entries, time only missing keys")
    ap.add_argument("--drop", default="", help="with --keep: first remove the entries of these op classes "
                                                "(comma list, e.g. cws) so that they are re-timed")
    a = ap.parse_args()
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    from cxxnet_amd.ops import gemm as G
    if not a.keep:
        G._TUNE.clear()
    for op in filter(None, a.drop.split(",")):
        for k in [k for k in G._TUNE if k.split("|")[0] == op]:
            del G._TUNE[k]
    for spec in a.models.split(","):
        name, b = spec.split(":")
        b = int(b)
        pairs = load_conf(name, [("batch_size", str(b)), ("eval_train", "0"), ("dev", "gpu"), ("silent", "1")])
        tr = NetTrainer()
        for k, v in pairs:
            if not k.startswith("metric"):
                tr.set_param(k, v)
        tr.init_model()
        c, h, w = tr.net_cfg.input_shape
        x = torch.randn(b, c, h, w, device="cuda")
        y = torch.zeros(b, 1, device="cuda")
        for _ in range(2):
            tr.update(DataBatch(x, y))
        torch.cuda.synchronize()
        print(name, b, len(G._TUNE), flush=True)
        del tr
        torch.cuda.empty_cache()
    G.save_tune_db(a.out or None)
    print("wrote", a.out or G.TUNE_DB, len(G._TUNE), "entries")


if __name__ == "__main__":
    main()
