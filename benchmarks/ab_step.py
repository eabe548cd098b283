"""Interleaved in-process A/B of whole AlexNet training steps under different kernel
configurations (per guide rule: perf deltas come from interleaved rounds in ONE process).

  python benchmarks/ab_step.py --configs "all:cf,cd,cw,fc,fw" "no_cw:cf,cd,fc,fw" --rounds 5
Each config is `name:glds-op-classes[:ov][:db=path]` ("none" = register-staged kernel everywhere;
":ov" runs the optimizer per gradient bucket on a side stream, overlapped with the rest of backward;
":db=path" lays a tile table written by benchmarks/tune_db.py over the shipped one; ":g=N" sets the
GEMM tile-order group, ops.gemm.set_tile_group).
Prints one JSON line per config: median / min ms per step over the rounds.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", required=True)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--model", default="alexnet")
    a = ap.parse_args()

    from cxxnet_amd.io.data import DataBatch, U8Images
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    from cxxnet_amd.ops import gemm as G

    dev = torch.device("cuda")
    pairs = load_conf(a.model, [("batch_size", str(a.batch)), ("eval_train", "0"), ("dev", "gpu"), ("silent", "1")])
    pairs = [(k, v) for k, v in pairs if not k.startswith("metric")]
    tr = NetTrainer()
    for k, v in pairs:
        tr.set_param(k, v)
    tr.init_model()
    c, h, w = tr.net_cfg.input_shape
    g = torch.Generator().manual_seed(0)
    pix = torch.randint(0, 256, (a.batch, h, w, c), generator=g, dtype=torch.uint8).to(dev)
    data = U8Images(pix, torch.zeros((a.batch, 4), dtype=torch.int32, device=dev),
                    torch.tensor([[1.0, 0.0]] * a.batch, device=dev),
                    torch.tensor([123.68, 116.78, 103.94][:c], device=dev), 1, 1.0)
    batch = DataBatch(data, torch.randint(0, 1000, (a.batch, 1), generator=g).float().to(dev))

    cfgs = []
    for spec in a.configs:
        name, ops, *flags = spec.split(":")
        db = {}
        grp = 0
        for f in flags:
            if f.startswith("g="):
                grp = int(f[2:])
            if f.startswith("db="):
                db = G._load_tune_db(f[3:])
                assert db, f"empty or unreadable tile table {f[3:]}"
        cfgs.append((name, [] if ops == "none" else ops.split(","), "ov" in flags, db, grp))
    shipped = dict(G._TUNE)
    net = tr.net
    ov_fn = lambda ranges: net.update(tr.epoch_counter, ranges)  # noqa: E731
    times = {n: [] for n, *_ in cfgs}
    for r in range(a.rounds):
        for name, ops, ov, db, grp in cfgs:
            G.set_glds(on=bool(ops), ops=ops)
            G.set_tile_group(grp)
            G._TUNE.clear()
            G._TUNE.update(shipped)
            G._TUNE.update(db)
            if ov:
                tr.reducer.enable_overlapped_update(ov_fn)
            else:
                tr.reducer.update_fn = None
            for _ in range(3):
                tr.update(batch, local=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                tr.update(batch, local=True)
            torch.cuda.synchronize()
            times[name].append((time.perf_counter() - t0) / a.steps * 1000.0)
    for name, *_ in cfgs:
        ts = times[name]
        print(json.dumps({"config": name, "median_ms": round(statistics.median(ts), 4), "min_ms": round(min(ts), 4),
                          "img_s_median": round(a.batch / statistics.median(ts) * 1000.0, 1)}), flush=True)


if __name__ == "__main__":
    main()
