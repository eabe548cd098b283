"""One training step's kernel sequence from a rocprofv3 kernel trace: start offset, duration,
the idle gap before it (on any queue) and the stream, between two dispatches of the marker.

    python tools/step_seq.py DIR [--marker image_u8c3_nhwc3p] [--step 5] [--min-gap 0]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_gaps import load, short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="image_u8c3_nhwc3p")
    ap.add_argument("--step", type=int, default=5)
    a = ap.parse_args()
    rows = load(a.dir)
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    i0, i1 = marks[a.step], marks[a.step + 1]
    t0 = rows[i0][0]
    end = t0
    for s, e, n in rows[i0:i1]:
        gap = max(0, s - end)
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap / 1e3:8.1f}  {short(n)}")
        end = max(end, e)


if __name__ == "__main__":
    main()
