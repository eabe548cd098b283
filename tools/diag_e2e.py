"""tests/test_e2e_gpu.py::test_cuda_graph_step_matches_eager outside pytest, with the per-parameter
m1 differences (graph vs the default eager-or-list trainer)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_e2e_gpu as T  # noqa: E402


def main():
    from cxxnet_amd.io.data import DataBatch
    model, batch = "alexnet", 16
    over = {"eval_train": "1", "metric": "error", "lr:schedule": "expdecay", "lr:gamma": "0.5", "lr:step": "2"}
    eager_over = dict(over)
    if os.environ.get("DIAG_EAGER") == "1":
        eager_over["launch_replay"] = "0"
    eager = T._trainer(T._pairs(model, batch, **eager_over), "gpu")
    graph = T._trainer(T._pairs(model, batch, cuda_graph="1", **over), "gpu")
    graph.net.arena.w.copy_(eager.net.arena.w)
    graph.net.arena.sync_shadow()
    c, h, w = eager.net_cfg.input_shape
    g = torch.Generator().manual_seed(3)
    for step in range(4):
        x = torch.randn(batch, c, h, w, generator=g).cuda()
        y = torch.randint(0, 1000, (batch, 1), generator=g).float().cuda()
        eager.update(DataBatch(x, y))
        graph.update(DataBatch(x, y))
        torch.cuda.synchronize()
        print(f"step {step}: rel m1 {T._rel(graph.net.arena.m1, eager.net.arena.m1):.3g} "
              f"eager plans {list(eager._lists)} {list(eager._graphs)} graph plans {list(graph._graphs)} "
              f"fused e {sorted(eager.net.updater.fused_offsets)} g {sorted(graph.net.updater.fused_offsets)}", flush=True)
        specs = dict(((li, s.tag), s) for li, s in eager.net.arena.specs)
        sb = specs.get((22, "bias"))
        if sb is not None:
            sl = slice(sb.offset, sb.offset + sb.numel)
            print(f"   fc8 bias |g| eager {eager.net.arena.g[sl].norm().item():.4g} graph {graph.net.arena.g[sl].norm().item():.4g}"
                  f" |w| eager {eager.net.arena.w[sl].norm().item():.4g} graph {graph.net.arena.w[sl].norm().item():.4g}", flush=True)
        for li, s in eager.net.arena.specs:
            a = graph.net.arena.m1[s.offset:s.offset + s.numel]
            b = eager.net.arena.m1[s.offset:s.offset + s.numel]
            d = (a - b).norm().item()
            if d > 0.05 * b.norm().item() + 1e-12:
                print(f"   {li}:{s.tag} |d| {d:.3g} |eager| {b.norm().item():.3g} |graph| {a.norm().item():.3g}", flush=True)


if __name__ == "__main__":
    main()
