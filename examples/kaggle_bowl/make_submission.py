"""Join pred_raw probability rows with image names into a Kaggle submission CSV.

Usage: python make_submission.py sampleSubmission.csv test.lst test.txt out.csv
"""
import csv
import os
import sys


def main(argv):
    if len(argv) < 4:
        print(__doc__)
        return 1
    sub, lst, pred, out = argv[:4]
    with open(sub) as f:
        header = next(csv.reader(f))
    with open(lst) as f:
        names = [os.path.basename(line.rstrip("\n").split("\t")[-1]) for line in f if line.strip()]
    with open(pred) as fi, open(out, "w", newline="") as fo:
        w = csv.writer(fo, lineterminator="\n")
        w.writerow(header)
        for name, line in zip(names, fi):
            w.writerow([name] + line.split())
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
