"""Per-layer GPU time from a rocprofv3 run with trace_layers = 1:

  CXXNET_TRACE_LAYERS=1 rocprofv3 --marker-trace --hip-trace --kernel-trace --output-format csv \\
      -d OUT -o run -- python3 bench.py --steps 5 --warmup 2
  python tools/layer_times.py OUT [--md layers.md]

Each kernel is attributed to the layer range (`fwd:<i>:<type>` / `bwd:<i>:<type>`) that was
open on the host thread when its launch API call ran (HIP API record and kernel dispatch
share a correlation id); kernels outside every range (optimizer, input staging) are
grouped as "other".
"""
import argparse
import bisect
import csv
import glob
import os
from collections import defaultdict


def _rows(d, suffix):
    out = []
    for p in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--md", default=None)
    ap.add_argument("--kernels", default=None, help="also write a per-layer kernel breakdown here")
    a = ap.parse_args()
    marks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], r["Thread_Id"])
             for r in _rows(a.dir, "marker_api_trace.csv")]
    marks.sort()
    starts = [m[0] for m in marks]
    launch = {}
    for r in _rows(a.dir, "hip_api_trace.csv"):
        launch[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), r["Thread_Id"])
    per = defaultdict(float)
    cnt = defaultdict(int)
    kern = defaultdict(lambda: [0.0, 0])
    for k in _rows(a.dir, "kernel_trace.csv"):
        dur = (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3  # us
        name = "other"
        li = launch.get(k["Correlation_Id"])
        if li is not None:
            t, tid = li
            j = bisect.bisect_right(starts, t) - 1
            while j >= 0 and marks[j][0] <= t:
                if marks[j][1] >= t and marks[j][3] == tid:
                    name = marks[j][2]
                    break
                j -= 1
        per[name] += dur
        cnt[name] += 1
        kk = kern[(name, k["Kernel_Name"][:90], k.get("Grid_Size_X", ""), k.get("Grid_Size_Y", ""))]
        kk[0] += dur
        kk[1] += 1
    total = sum(per.values())
    lines = [f"total kernel time {total / 1e3:.3f} ms", "", "| layer range | kernels | total us | share |",
             "|---|---|---|---|"]
    for name, us in sorted(per.items(), key=lambda kv: -kv[1]):
        lines.append(f"| `{name}` | {cnt[name]} | {us:.1f} | {100 * us / total:.1f}% |")
    text = "\n".join(lines)
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text + "\n")
    if a.kernels:
        rows = ["| layer range | kernel | grid | calls | total us | mean us |", "|---|---|---|---|---|---|"]
        order = sorted(per, key=lambda n: -per[n])
        for name in order:
            ks = sorted(((v, key) for key, v in kern.items() if key[0] == name), key=lambda t: -t[0][0])
            for (us, c), key in ks:
                rows.append(f"| `{name}` | `{key[1]}` | {key[2]}x{key[3]} | {c} | {us:.1f} | {us / c:.1f} |")
        with open(a.kernels, "w") as f:
            f.write("\n".join(rows) + "\n")


if __name__ == "__main__":
    main()
