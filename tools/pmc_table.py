"""Table of rocprofv3 --pmc results written by tools/pmc_ops.sh:
    python tools/pmc_table.py DIR op [op ...]
Per op (mean per gemm dispatch): time, achieved clock, MFMA utilisation (MFMA-busy SIMD cycles over
all 1024 SIMDs x kernel cycles), VALU and LDS instructions per MFMA, LDS bank-conflict cycles per
LDS-active cycle, share of wave cycles parked (waitcnt/barrier) and issue-stalled, and HBM bytes
read / written (FETCH_SIZE / WRITE_SIZE, KB) per dispatch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_read import read  # noqa: E402


def main():
    d = sys.argv[1]
    print("| op | us | clock GHz | MFMA util | VALU/MFMA | LDS/MFMA | LDS conflict | parked | issue-stalled | HBM read MB | HBM write MB |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for op in sys.argv[2:]:
        c, us = {}, []
        for i in range(1, 5):
            ci, ui = read(os.path.join(d, f"{op}_p{i}"))
            c.update(ci)
            if ui:
                us.append(ui)
        t = sorted(us)[len(us) // 2] if us else 0.0
        g = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0  # summed over the 8 XCDs
        clk = g / (t * 1e3) if t else 0.0
        util = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (g * 1024) if g else 0.0
        mf = max(c.get("SQ_INSTS_MFMA", 0.0), 1.0)
        wc = max(c.get("SQ_WAVE_CYCLES", 0.0), 1.0)
        lds = max(c.get("SQ_LDS_IDX_ACTIVE", 0.0), 1.0)
        print(f"| {op} | {t:.1f} | {clk:.2f} | {100 * util:.1f}% | {c.get('SQ_INSTS_VALU', 0) / mf:.2f} | "
              f"{c.get('SQ_INSTS_LDS', 0) / mf:.2f} | {c.get('SQ_LDS_BANK_CONFLICT', 0) / lds:.3f} | "
              f"{100 * c.get('SQ_WAIT_ANY', 0) / wc:.0f}% | {100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:.0f}% | "
              f"{c.get('FETCH_SIZE', 0) / 1024:.1f} | {c.get('WRITE_SIZE', 0) / 1024:.1f} |")


if __name__ == "__main__":
    main()
