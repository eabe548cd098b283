"""GPU idle time inside training steps from a rocprofv3 kernel trace.

    python tools/prof_gaps.py DIR [DIR...] [--marker image_u8c3_nhwc3p] [--top 12]

A step runs from one dispatch of the marker kernel (the input conversion that opens every
step) to the next.  Per directory: mean step span, mean union of kernel intervals (busy),
idle = span - busy, and the largest idle gaps (mean over steps, keyed by the kernels on both
sides of the gap).  Kernels on several queues overlap; the union counts that time once."""
import argparse
import csv
import glob
import os
from collections import defaultdict


def load(d):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r["Kernel_Name"] + " @s" + str(r.get("Stream_Id", "?"))))
    rows.sort()
    return rows


def short(name):
    """'void (anonymous namespace)::gemm_glds<...>(...) @s3' -> 'gemm_glds @s3'"""
    name, _, stream = name.rpartition(" @")
    for p in ("void ", "(anonymous namespace)::", "at::native::"):
        name = name.replace(p, "")
    for c in "<(":
        name = name.split(c)[0]
    return f"{name[:48]} @{stream}"


def analyse(rows, marker, top):
    starts = [i for i, r in enumerate(rows) if marker in r[2]]
    if len(starts) < 3:
        return None
    spans, busys = [], []
    gaps = defaultdict(float)
    nsteps = 0
    for a, b in zip(starts[1:-1], starts[2:]):  # skip the first (warm-up) step
        seg = rows[a:b]
        t0, t1 = seg[0][0], rows[b][0]
        busy, end, prev = 0, t0, None
        for s, e, n in seg:
            if s > end:
                if prev is not None:
                    gaps[(short(prev), short(n))] += (s - end) / 1000.0
            else:
                s = end
            if e > s:
                busy += e - s
                end = e
            prev = n
        spans.append((t1 - t0) / 1000.0)
        busys.append(busy / 1000.0)
        nsteps += 1
    span = sum(spans) / nsteps
    busy = sum(busys) / nsteps
    worst = sorted(((v / nsteps, k) for k, v in gaps.items()), reverse=True)[:top]
    return span, busy, nsteps, worst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--marker", default="image_u8c3_nhwc3p")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--timeline", action="store_true", help="also print one step's dispatches")
    a = ap.parse_args()
    for d in a.dirs:
        res = analyse(load(d), a.marker, a.top)
        if res is None:
            print(d, "no steps found (marker %r)" % a.marker)
            continue
        span, busy, n, worst = res
        print(f"{d}: {n} steps, span {span:.1f} us, busy {busy:.1f} us, idle {span - busy:.1f} us")
        for us, (p, q) in worst:
            print(f"  {us:7.1f} us  {p}  ->  {q}")
        if a.timeline:
            rows = load(d)
            st = [i for i, r in enumerate(rows) if a.marker in r[2]]
            if len(st) >= 3:
                t0, end = rows[st[1]][0], rows[st[1]][0]
                print("  start_us  gap_us   dur_us  kernel")
                for s_, e_, n in rows[st[1]:st[2]]:
                    print(f"  {(s_ - t0) / 1e3:8.1f} {max(0, s_ - end) / 1e3:7.1f} {(e_ - s_) / 1e3:8.1f}  {short(n)}")
                    end = max(end, e_)


if __name__ == "__main__":
    main()
