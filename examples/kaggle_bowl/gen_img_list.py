"""Write an image list (index, label, path) for the bowl data.

Usage: python gen_img_list.py train|test sampleSubmission.csv <folder>/ out.lst

`train`: <folder>/<class>/<img> with label = column index of <class> in the
submission header.  `test`: every file in <folder>/ with label 0.  The list is
shuffled with a fixed seed.
"""
import csv
import os
import random
import sys


def main(argv):
    if len(argv) < 4:
        print(__doc__)
        return 1
    task, sub, folder, out = argv[:4]
    with open(sub) as f:
        classes = next(csv.reader(f))[1:]
    items = []
    if task == "train":
        for label, cls in enumerate(classes):
            d = os.path.join(folder, cls)
            for name in sorted(os.listdir(d)):
                items.append((label, os.path.join(d, name)))
    else:
        for name in sorted(os.listdir(folder)):
            items.append((0, os.path.join(folder, name)))
    random.Random(888).shuffle(items)
    with open(out, "w") as f:
        for i, (label, path) in enumerate(items):
            f.write(f"{i}\t{label}\t{path}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
