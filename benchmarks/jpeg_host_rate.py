"""Host half of JPEG decoding, per thread count: the native pool decoding to pixels (decode)
vs entropy-decoding into the GPU stage (decode_coef, io/jpeg_stage.py), on preallocated
buffers (pinned or pageable), no iterator around it.

    python benchmarks/jpeg_host_rate.py --dir /tmp/iods [--threads 1,4,16] [--pinned 0,1]"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd import native  # noqa: E402
from cxxnet_amd.io import jpeg_stage  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True, help="an io_throughput.py dataset (img/*.jpg)")
    ap.add_argument("--threads", default="1,4,16")
    ap.add_argument("--pinned", default="0,1")
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    d = os.path.join(a.dir, "img")
    recs = [open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d))[:1024]]
    rt = native.rt()
    B, h, w = 256, 227, 227
    cfg = (h, w, 3, 1, 1, 0, -1, -1, 0.0, 0.0, 1)
    cap = jpeg_stage.stage_capacity(B, h, w)
    for pin in (int(v) for v in a.pinned.split(",")):
        pin = pin and torch.cuda.is_available()

        def buf(shape, dt):
            return torch.zeros(shape, dtype=dt, pin_memory=bool(pin)).numpy()
        out = buf((B, h, w, 3), torch.uint8)
        coef, bwin, meta = buf((cap, 64), torch.int16), buf((cap,), torch.int32), buf((B, 3, 80), torch.int32)
        prm, cm = buf((B, 4), torch.int32), buf((B, 2), torch.float32)
        for nt in (int(v) for v in a.threads.split(",")):
            pool = rt.JpegDecodePool(nt)
            res = {"threads": nt, "pinned": bool(pin)}
            for mode in ("pixels", "coef"):
                ts = []
                for rep in range(a.reps):
                    items = [(i, recs[(rep * B + i) % len(recs)], rep * B + i) for i in range(B)]
                    t = time.perf_counter()
                    if mode == "pixels":
                        pool.decode(items, cfg, out, prm, cm)
                    else:
                        pool.decode_coef(items, cfg, coef, bwin, meta, prm, cm)
                    ts.append(time.perf_counter() - t)
                res[mode + "_img_s"] = round(B / statistics.median(ts[1:]))
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
