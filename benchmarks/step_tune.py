"""Refine the tile table INSIDE the training step (greedy, one signature at a time).

The shipped table (ops/glds_tune_gfx950.json) is filled by timing each GEMM signature alone; a
kernel that wins alone can lose inside the step (L2 contents, neighbours, clocks).  Here every
signature the model looks up is re-decided by whole-step time: for each candidate tile (the
op class's tile set; for the conv weight-grad "cws" keys the (tile, split) set of
ops.gemm._wgrad_cands) the step is timed in interleaved rounds, and the best candidate replaces
the table entry only if it beats the current one by more than --margin.

    python benchmarks/step_tune.py --model alexnet --batch 256 --out table.json
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# the compiled tile sets (ops.gemm.GLDS_TILES; tests/test_tile_table_cpu.py keeps them in sync)
KK = (1, 7, 10, 15, 21, 25, 30, 31, 34, 37, 38, 39, 72, 75, 76, 77, 78, 79, 82, 114)
MM = (1, 2, 17, 23, 40, 41)
SHORT = (1, 7, 10, 15, 34, 37, 38, 75, 76, 77, 78, 79)


class LogDict(dict):
    def __init__(self, *a):
        super().__init__(*a)
        self.seen = []

    def get(self, k, d=None):
        if k not in self.seen:
            self.seen.append(k)
        return super().get(k, d)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="alexnet")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--margin", type=float, default=0.004)
    ap.add_argument("--out", required=True)
    ap.add_argument("--short", action="store_true", help="shortlist of LDS-DMA tiles (models with many signatures)")
    ap.add_argument("--ops", default="", help="only these op classes (comma list, e.g. fw)")
    ap.add_argument("--cands", default="", help="only these candidate tiles (comma list; the current entry is kept)")
    a = ap.parse_args()
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    from cxxnet_amd.ops import gemm as G
    from cxxnet_amd.ops.gemm import conv_out_size

    if os.environ.get("CXXNET_DIST_FORCE", "0") == "1":  # the data-parallel step (RCCL at world 1)
        from cxxnet_amd.parallel import init_distributed
        init_distributed()
    G._TUNE = LogDict(G._TUNE)
    pairs = load_conf(a.model, [("batch_size", str(a.batch)), ("eval_train", "0"), ("dev", "gpu"), ("silent", "1")])
    tr = NetTrainer()
    for k, v in pairs:
        if not k.startswith("metric"):
            tr.set_param(k, v)
    tr.init_model()
    c, h, w = tr.net_cfg.input_shape
    batch = DataBatch(torch.randn(a.batch, c, h, w, device="cuda"), torch.zeros(a.batch, 1, device="cuda"))
    for _ in range(3):
        tr.update(batch)
    torch.cuda.synchronize()
    keys = [k for k in G._TUNE.seen if k in G._TUNE]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def step_ms():
        for _ in range(2):
            tr.update(batch)
        s.record()
        for _ in range(a.steps):
            tr.update(batch)
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / a.steps

    log = []
    for key in keys:
        op = key.split("|")[0]
        if a.ops and op not in a.ops.split(","):
            continue
        if op in ("cf", "cd", "cr", "fc"):
            cands = list(SHORT if a.short else KK) + ([G.REG, 130, 131, 133] if op in ("cf", "cd") else [])
        elif op == "cfs":  # sibling-group forward (two destinations): the LDS-DMA tiles only
            cands = [t for t in (SHORT if a.short else KK) if t in G.SPLIT_CANDS]
        elif op in ("fw", "fws", "cwr"):
            cands = list(MM)
        elif op == "cw":  # conv weight-grad: the register split-K kernel, LDS-DMA MN tiles,
            # the direct 3x3 kernel (140; it declines other shapes and the entry then runs REG)
            cands = [G.REG] + list(MM) + [140]
        elif op == "cws":
            N, H, W, C, Co, KH, KW, st, py, px, g = (int(v) for v in key.split("|")[1:])
            Ho, Wo = conv_out_size(H, W, KH, KW, st, py, px)
            cands = list(G._wgrad_cands(KH * KW * (C // g), Co // g, g, N * Ho * Wo))
        else:
            continue
        if a.cands:
            cands = [int(t) for t in a.cands.split(",")]
        cur = G._TUNE[key]
        if cur not in cands:
            cands.append(cur)
        times = {t: [] for t in cands}
        for _ in range(a.rounds):
            for t in cands:
                G._TUNE[key] = t
                try:
                    times[t].append(step_ms())
                except Exception as ex:  # a tile the op cannot run: drop it
                    times[t] = None
                    print("skip", key, t, type(ex).__name__, flush=True)
                    G._TUNE[key] = cur
                    continue
        ok = {t: statistics.median(v) for t, v in times.items() if v}
        best = min(ok, key=ok.get)
        new = best if ok[best] < ok[cur] * (1 - a.margin) else cur
        G._TUNE[key] = new
        log.append({"key": key, "old": cur, "old_ms": round(ok[cur], 4), "new": new, "new_ms": round(ok[new], 4)})
        print(json.dumps(log[-1]), flush=True)
    with open(a.out, "w") as f:
        json.dump(dict(sorted(dict(G._TUNE).items())), f, indent=0)
    print("final step ms", round(step_ms(), 4))


if __name__ == "__main__":
    main()
