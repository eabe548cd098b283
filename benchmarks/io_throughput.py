"""IO pipeline throughput (the reference's `test_io = 1`, src/cxxnet_main.cpp:363-377) on
JPEGs generated locally with Pillow (no dataset on the box).

  python benchmarks/io_throughput.py [--n 2048] [--size 256] [--workers 4,8,16] [--modes native,process,thread]
                                     [--iters imgbin,imgbinx]

Writes N JPEG images (smooth random content, quality 90, ImageNet-like file sizes at the
given side), packs them with im2bin into 64 MB pages, then times `iter = imgbin(x)` +
`threadbuffer` with the AlexNet training augmentation (random 227 crop, random mirror,
mean_value) at batch 256 for each worker count, decoding in the native C++ pool
(decode_native), in the native pool's entropy stage + the GPU (gpu: decode_gpu, io/jpeg_stage.py),
in Pillow processes (decode_process) or in Pillow threads (decode_thread).  Prints one JSON line per setting: img/s, img/s per busy host
core, and the host cores one MI355X would need at its measured AlexNet training rate.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GPU_IMG_S = 109200.0  # AlexNet b256 on one MI355X (bench.py, round 4 baseline: profiles/r4_baseline_models_1gpu.jsonl)


def make_dataset(root, n, size, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    os.makedirs(os.path.join(root, "img"), exist_ok=True)
    yy, xx = np.mgrid[0:size, 0:size].astype(np.float32) / size
    lines = []
    nbytes = 0
    for i in range(n):
        # smooth gradients + a few blobs + mild noise: JPEG sizes like natural photos
        c = rng.uniform(0, 255, (3, 3))
        img = np.stack([c[k, 0] * xx + c[k, 1] * yy + c[k, 2] * (1 - xx) for k in range(3)], -1)
        for _ in range(4):
            cx, cy, r = rng.uniform(0, 1, 3)
            m = ((xx - cx) ** 2 + (yy - cy) ** 2) < (0.05 + 0.2 * r) ** 2
            img[m] = rng.uniform(0, 255, 3)
        img += rng.normal(0, 12, img.shape)
        p = os.path.join("img", f"{i:06d}.jpg")
        Image.fromarray(np.clip(img, 0, 255).astype(np.uint8)).save(os.path.join(root, p), quality=90)
        nbytes += os.path.getsize(os.path.join(root, p))
        lines.append(f"{i}\t{i % 1000}\t{p}\n")
    with open(os.path.join(root, "train.lst"), "w") as f:
        f.writelines(lines)
    return nbytes / n


def make_trainer(model, batch):
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    pairs = load_conf(model, [("batch_size", str(batch)), ("eval_train", "0"), ("dev", "gpu"), ("silent", "1")])
    tr = NetTrainer()
    for k, v in pairs:
        if not k.startswith("metric"):
            tr.set_param(k, v)
    tr.init_model()
    return tr


def run(root, it_type, mode, workers, batches, batch, tr=None):
    threads, procs = (workers, 0) if mode == "thread" else (1, workers)
    nat = "1" if mode in ("native", "gpu") else "0"
    from cxxnet_amd.io.iterators import create_iterator
    cfg = [("iter", it_type), ("image_list", os.path.join(root, "train.lst")),
           ("image_bin", os.path.join(root, "train.bin")), ("rand_crop", "1"), ("rand_mirror", "1"),
           ("mean_value", "104,117,123"), ("decode_thread", str(threads)), ("decode_process", str(procs)),
           ("decode_native", nat), ("decode_native_threads", str(workers)),
           ("decode_gpu", "1" if mode == "gpu" else "0"),
           ("input_shape", "3,227,227"),
           ("batch_size", str(batch)), ("round_batch", "1"), ("silent", "1"), ("iter", "threadbuffer"),
           ("iter", "end")]
    it = create_iterator(cfg)
    it.init()
    it.before_first()
    n = 0
    # one warm batch, then time
    if not it.next():
        it.before_first()
        it.next()
    t0 = time.perf_counter()
    while n < batches:
        if not it.next():
            it.before_first()
            continue
        b = it.value()
        if tr is not None:
            tr.update(b)
        elif mode == "gpu":  # decode only: finish the decode on the GPU
            b.data.to_u8("cuda")
        n += 1
    if tr is not None or mode == "gpu":
        import torch
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    it.close()
    return batches * batch / el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--workers", default="4,8,16")
    ap.add_argument("--modes", default="gpu,native,process,thread")
    ap.add_argument("--iters", default="imgbin,imgbinx")
    ap.add_argument("--batches", type=int, default=12)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--dir", default="")
    ap.add_argument("--repeat", type=int, default=1,
                    help="pack the list this many times (a multi-page .bin from few JPEGs: the page "
                         "reader's steady state)")
    ap.add_argument("--train", default="", help="also train this model (GPU) on the decoded batches")
    a = ap.parse_args()
    root = a.dir or tempfile.mkdtemp(prefix="cxxnet_io_")
    from cxxnet_amd.tools.im2bin import pack
    if os.path.exists(os.path.join(root, "train.bin")):  # reuse a dataset made by an earlier run
        imgs = os.listdir(os.path.join(root, "img"))
        avg = sum(os.path.getsize(os.path.join(root, "img", f)) for f in imgs) / max(len(imgs), 1)
    else:
        avg = make_dataset(root, a.n, a.size)
        if a.repeat > 1:
            lines = open(os.path.join(root, "train.lst")).read().splitlines()
            with open(os.path.join(root, "train.lst"), "w") as f:
                for r in range(a.repeat):
                    for i, ln in enumerate(lines):
                        _, lab, p = ln.split("\t")
                        f.write(f"{r * len(lines) + i}\t{lab}\t{p}\n")
        pack(os.path.join(root, "train.lst"), root + "/", os.path.join(root, "train.bin"))
    cores = os.cpu_count()
    tr = make_trainer(a.train, a.batch) if a.train else None
    for it_type in a.iters.split(","):
        for mode in a.modes.split(","):
            for t in [int(v) for v in a.workers.split(",")]:
                ips = run(root, it_type, mode, t, a.batches, a.batch, tr)
                per_core = ips / min(t, cores)
                print(json.dumps({"iter": it_type, "mode": mode, "workers": t, "host_cpus": cores,
                                  "train": a.train or None,
                                  "img_per_s": round(ips, 1),
                                  "img_per_s_per_busy_core": round(per_core, 1), "jpeg_side": a.size,
                                  "avg_jpeg_bytes": int(avg),
                                  "cores_for_one_mi355x_at_%d_img_s" % GPU_IMG_S: round(GPU_IMG_S / per_core, 1)}),
                      flush=True)


if __name__ == "__main__":
    main()
