"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db or kernel_trace.csv) into a
per-kernel table: calls, total ms, mean us, share of GPU time.

  python tools/prof_summary.py gpurun_out/prof1/run_results.db [--steps K] [--md out.md]
"""
import argparse
import collections
import csv
import glob
import os
import re
import sqlite3


def _short(name: str) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    m = re.match(r"void (\w+)<(.*)>\(", n)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.match(r"(\w[\w:]*)", n.replace("void ", ""))
    return m.group(1) if m else n[:80]


def load_db(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    rows = cur.execute(f"select s.kernel_name, d.end - d.start, d.grid_size_x, d.grid_size_y, d.grid_size_z, "
                       f"s.arch_vgpr_count, s.group_segment_size from {kd} d join {ks} s on d.kernel_id = s.id")
    return [(r[0], r[1], (r[2], r[3], r[4]), r[5], r[6]) for r in rows]


def load_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                        (r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z")),
                        r.get("VGPR_Count"), r.get("LDS_Block_Size")))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=0, help="divide totals by this many steps")
    ap.add_argument("--md", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    p = a.path
    if os.path.isdir(p):
        cands = glob.glob(os.path.join(p, "**", "*.db"), recursive=True) + \
            glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True)
        p = cands[0]
    rows = load_db(p) if p.endswith(".db") else load_csv(p)
    agg = collections.OrderedDict()
    for name, dur, grid, vgpr, lds in rows:
        key = (_short(name), grid)
        e = agg.setdefault(key, [0, 0, vgpr, lds])
        e[0] += 1
        e[1] += dur
    total = sum(v[1] for v in agg.values())
    lines = ["| kernel | grid | calls | total ms | mean us | share | vgpr | lds |", "|---|---|---|---|---|---|---|---|"]
    for (k, grid), (n, t, vgpr, lds) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        lines.append(f"| `{k[:90]}` | {grid} | {n} | {t / 1e6:.3f} | {t / n / 1e3:.1f} | {100 * t / total:.1f}% "
                     f"| {vgpr} | {lds} |")
    head = f"total GPU kernel time: {total / 1e6:.3f} ms over {len(rows)} dispatches"
    if a.steps:
        head += f" ({total / 1e6 / a.steps:.3f} ms/step over {a.steps} steps)"
    text = head + "\n\n" + "\n".join(lines) + "\n"
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
