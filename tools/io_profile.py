"""Main-thread profile of the image iterator (no threadbuffer) on an io_throughput.py dataset:
where the per-batch host time goes, for the pixel path and the GPU decode stage.

    python tools/io_profile.py --dir /tmp/iods [--threads 16] [--batches 20]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cxxnet_amd.io.iterators import create_iterator  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--lst", default="train")
    a = ap.parse_args()
    for gpu in (0, 1):
        cfg = [("iter", "imgbin"), ("image_list", os.path.join(a.dir, a.lst + ".lst")),
               ("image_bin", os.path.join(a.dir, a.lst + ".bin")), ("rand_crop", "1"), ("rand_mirror", "1"),
               ("mean_value", "104,117,123"), ("decode_native", "1"), ("decode_native_threads", str(a.threads)),
               ("decode_gpu", str(gpu)), ("input_shape", "3,227,227"), ("batch_size", "256"), ("round_batch", "1"),
               ("silent", "1"), ("iter", "end")]
        it = create_iterator(cfg)
        it.init()
        it.before_first()
        for _ in range(3):
            it.next()
        pr = cProfile.Profile()
        t = time.perf_counter()
        pr.enable()
        n = 0
        while n < a.batches:
            if not it.next():
                it.before_first()
                continue
            if gpu and torch.cuda.is_available():
                it.value().data.to_u8("cuda")
            n += 1
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        pr.disable()
        print(f"decode_gpu={gpu}: {a.batches * 256 / (time.perf_counter() - t):.0f} img/s", flush=True)
        pstats.Stats(pr).sort_stats("tottime").print_stats(12)
        it.close()


if __name__ == "__main__":
    main()
