"""precision=fp32 on the GPU under data parallelism (2 gloo ranks on one GPU) against the
single-process step: norms of the trained distance on each side, per parameter."""
import os
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_dp_gpu as T  # noqa: E402

def main():
    EXTRA = [tuple(kv.split("=", 1)) for kv in sys.argv[1:]] or [("precision", "fp32"), ("deterministic", "1")]
    print("extra", EXTRA, flush=True)
    out = "/tmp/diag_dp_fp32_w"
    mp.spawn(T._worker, args=(2, T._free_port(), 4, out, EXTRA), nprocs=2, join=True)
    r0 = torch.load(out + ".r0", weights_only=True)
    from cxxnet_amd.io.data import DataBatch
    tr = T._make(8, EXTRA)
    w0 = tr.net.arena.w.cpu().clone()
    x, y = T._data(8)
    for _ in range(4):
        tr.update(DataBatch(x.cuda(), y.cuda()))
    torch.cuda.synchronize()
    w = tr.net.arena.w.cpu()
    for li, s in tr.net.arena.specs:
        sl = slice(s.offset, s.offset + s.numel)
        print(f"{li}:{s.tag} single |dw| {(w[sl] - w0[sl]).norm():.4g}  dp |dw| {(r0[sl] - w0[sl]).norm():.4g}"
              f"  |dp - single| {(r0[sl] - w[sl]).norm():.4g}", flush=True)


if __name__ == "__main__":
    main()
