"""im2bin: pack the images named by a list file into 64 MB BinaryPages.

Usage: python -m cxxnet_amd.tools.im2bin image.lst image_root_dir output.bin

Same contract as the reference's tools/im2bin.cpp:1-80: every list line is
`index <tab> label <tab> path`; the file at image_root_dir + path is appended,
as raw encoded bytes, to the current page; a full page is flushed.  The packing
itself runs in the native runtime (``_cxxnet_rt.pack_image_bin``).
"""
from __future__ import annotations

import sys
import time

from .. import native


def pack(list_path: str, root: str, out_path: str, label_width: int = 1) -> int:
    entries = native.rt().parse_image_list(list_path, label_width)
    files = [root + e.path for e in entries]
    return native.rt().pack_image_bin(files, out_path), len(files)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 3:
        print("Usage: im2bin image.lst image_root_dir output_file", file=sys.stderr)
        return 255
    start = time.time()
    print(f"create image binary pack from {argv[0]}, this will take some time...")
    npages, nimg = pack(argv[0], argv[1], argv[2])
    print(f"finished [{nimg:8d}] images processed to {npages} pages, {int(time.time() - start)} sec elapsed")
    return 0


if __name__ == "__main__":
    sys.exit(main())
