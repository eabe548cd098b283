"""imgbin partition maker: split an image list into parts of at most
`partition_size` MB and write a Makefile that runs im2bin on each part.

Usage: python -m cxxnet_amd.tools.partition --img_list L --img_root R --prefix 'tr%d'
           --out DIR [--partition_size 256] [--shuffle 0] [--makefile Gen.mk]
           [--im2bin 'python -m cxxnet_amd.tools.im2bin']

Behaviour of the reference's tools/imgbin-partition-maker.py (size estimate =
file size + 4*(count+2) bytes per part, 10 KB head-room, seed 888 shuffle), in
Python 3.  The generated parts plug into `iter = imgbin` through
`image_conf_prefix = DIR/tr%d` and `image_conf_ids = 1-N`.
"""
from __future__ import annotations

import argparse
import os
import random
import sys


def make_partitions(lines, img_root, prefix, out_dir, partition_mb=256, shuffle=False, seed=888):
    """Returns [(lst_path, bin_path, [lines])]."""
    lst = list(lines)
    if shuffle:
        random.Random(seed).shuffle(lst)
    if not out_dir.endswith("/"):
        out_dir += "/"
    parts = []
    size = 0
    count = 1
    for item in lst:
        if not parts or size + 10240 > (partition_mb << 20):
            stem = out_dir + (prefix % (len(parts) + 1))
            parts.append((stem + ".lst", stem + ".bin", []))
            size = 0
            count = 1
        path = item.rstrip("\n").split("\t")[2]
        size += os.path.getsize(img_root + path) + (count + 2) * 4
        parts[-1][2].append(item if item.endswith("\n") else item + "\n")
        count += 1
    return parts


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Generate a Makefile to make partition imgbin files")
    ap.add_argument("--img_list", required=True)
    ap.add_argument("--img_root", required=True)
    ap.add_argument("--im2bin", default=f"{sys.executable} -m cxxnet_amd.tools.im2bin")
    ap.add_argument("--partition_size", default="256")
    ap.add_argument("--shuffle", default="0")
    ap.add_argument("--prefix", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--makefile", default="Gen.mk")
    a = ap.parse_args(argv)
    with open(a.img_list) as f:
        lines = f.readlines()
    parts = make_partitions(lines, a.img_root, a.prefix, a.out, int(a.partition_size), a.shuffle == "1")
    cmds = []
    for lst_path, bin_path, items in parts:
        with open(lst_path, "w") as fw:
            fw.writelines(items)
        cmds.append(f"{bin_path}: {lst_path}\n\t{a.im2bin} {lst_path} {a.img_root} {bin_path}")
    with open(a.makefile, "w") as fo:
        fo.write("all: " + " ".join(p[1] for p in parts) + "\n")
        fo.write("\n\n".join(cmds) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
