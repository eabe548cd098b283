"""Audit the main loops of the inline-asm-MFMA kernels (csrc/kernels/gemm_4w.hip) in hipcc's
assembly: hipcc pads no hazard for an asm MFMA (cdna guide 5.7 item 2), so the loop must not
write an MFMA A/B operand register with a VALU instruction (the operands come from ds_read only),
must not touch the accumulators with v_accvgpr_* and must not spill.

  python benchmarks/asm_audit.py [--src cxxnet_amd/csrc/kernels/gemm_4w.hip] [--match gemm_4w]

Prints one line per kernel (loop instruction counts) and exits non-zero on a violation."""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, "cxxnet_amd", "csrc", "kernels")


def regs(tok):
    """'v[4:7]' / 'v12' -> set of ('v', n)."""
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    return set()


def kernels(asm):
    out = {}
    cur = None
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is not None:
            out[cur].append(line)
            if "s_endpgm" in line:
                cur = None
    return out


def main_loop(lines):
    """Lines of the loop that holds the most MFMAs (a label -> the last branch back to it)."""
    best = None
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", l)
        if not m:
            continue
        label = m.group(1)
        js = [j for j in range(i + 1, len(lines)) if re.search(r"s_(c?)branch\w*\s+" + re.escape(label) + r"\b", lines[j])]
        if not js:
            continue
        body = lines[i:js[-1] + 1]
        n = sum("v_mfma" in x for x in body)
        if best is None or n > best[0]:
            best = (n, body)
    return best[1] if best else []


def _dst(s):
    parts = s.split(None, 1)
    return parts[1].split(",")[0].strip() if len(parts) > 1 else ""


def audit(body):
    """For every MFMA A/B operand register, the instruction that last wrote it before the MFMA
    (scanning the loop twice, so a write late in one iteration reaches the next) must be a
    ds_read; no v_accvgpr_* and no scratch traffic in the loop."""
    insts = []
    for l in body:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
            continue
        insts.append(s)
    counts = {"mfma": 0, "ds_read": 0, "dma": 0, "valu": 0, "accvgpr": 0, "scratch": 0, "waitcnt": 0, "nop": 0}
    errs = []
    for s in insts:
        op = s.split()[0]
        if op.startswith("v_mfma"):
            counts["mfma"] += 1
        elif op.startswith("ds_read"):
            counts["ds_read"] += 1
        elif op.startswith("buffer_load") and " lds" in s:
            counts["dma"] += 1
        elif op.startswith("v_accvgpr"):
            counts["accvgpr"] += 1
            errs.append("accumulator move: " + s)
        elif op.startswith("scratch_") or op.startswith("buffer_store"):
            counts["scratch"] += 1
            errs.append("spill: " + s)
        elif op.startswith("s_waitcnt"):
            counts["waitcnt"] += 1
        elif op.startswith("s_nop"):
            counts["nop"] += 1
        if op.startswith("v_") and not op.startswith("v_mfma"):
            counts["valu"] += 1
    last = {}
    for rnd in range(2):
        for s in insts:
            op = s.split()[0]
            if op.startswith("v_mfma"):
                if rnd == 1:
                    ops = [o.strip() for o in s.split(None, 1)[1].split(",")]
                    for r in regs(ops[1]) | regs(ops[2]):
                        w = last.get(r)
                        if w is not None and not w.startswith("ds_read"):
                            errs.append(f"MFMA operand {r} last written by: {w}")
                for r in regs(s.split(None, 1)[1].split(",")[0].strip()):
                    last[r] = s
                continue
            if op.startswith("ds_read") or op.startswith("v_") or op.startswith("global_load") or \
                    (op.startswith("buffer_load") and " lds" not in s) or op.startswith("scratch_load"):
                for r in regs(_dst(s)):
                    last[r] = s
    return counts, sorted(set(errs))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(KDIR, "gemm_4w.hip"))
    ap.add_argument("--match", default="gemm_4f")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
                        "--cuda-device-only", "-S", a.src, "-I" + KDIR, "-o", out], check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        asm = open(out).read()
    bad = 0
    for name, lines in kernels(asm).items():
        if a.match not in name:
            continue
        body = main_loop(lines)
        counts, errs = audit(body)
        text = "\n".join(lines)
        print(name[:90], counts, "OK" if not errs else f"{len(errs)} VIOLATIONS")
        for e in errs[:5]:
            print("   ", e)
        bad += bool(errs)
        if "scratch_" in text:
            print("    scratch access in the kernel")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
