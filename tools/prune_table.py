"""Write a copy of the shipped tile table without the conv forward / data-grad entries whose
A rows (forward: Cout/groups, data-grad: C/groups) are <= --max-rows, so that tune_db.py --keep
re-times them (e.g. after adding small-row tiles).
    python tools/prune_table.py OUT.json [--max-rows 64]"""
import argparse
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--max-rows", type=int, default=64)
a = ap.parse_args()
src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cxxnet_amd", "ops",
                   "glds_tune_gfx950.json")
t = json.load(open(src))
keep = {}
for k, v in t.items():
    p = k.split("|")
    if p[0] in ("cf", "cd"):
        N, H, W, C, Cout, KH, KW, s, py, px, G = (int(x) for x in p[1:])
        rows = (Cout if p[0] == "cf" else C) // G
        if rows <= a.max_rows:
            continue
    keep[k] = v
json.dump(keep, open(a.out, "w"), indent=0)
print("kept", len(keep), "of", len(t))
