"""Eager vs launch-list vs HIP-graph steps on one model in default mode (fused fc SGD, atomic
weight gradients, an lr schedule): per step, the norm of w / m1 on each path and the relative
differences to the eager path."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    model = sys.argv[1] if len(sys.argv) > 1 else "alexnet"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    over = {"eval_train": "1", "metric": "error", "lr:schedule": "expdecay", "lr:gamma": "0.5", "lr:step": "2"}

    def make(extra):
        tr = NetTrainer()
        pairs = [(k, v) for k, v in load_conf(model) if not k.startswith("metric") and k != "dev"]
        pairs += [("batch_size", str(batch)), ("silent", "1")] + list(over.items()) + extra + [("dev", "gpu"), ("seed", "7")]
        for k, v in pairs:
            tr.set_param(k, v)
        tr.init_model()
        return tr

    arms = {"eager": make([("launch_replay", "0"), ("cuda_graph", "0")]),
            "list": make([("launch_replay", "1"), ("cuda_graph", "0")]),
            "graph": make([("launch_replay", "0"), ("cuda_graph", "1")])}
    w0 = arms["eager"].net.arena.w
    for t in arms.values():
        t.net.arena.w.copy_(w0)
        t.net.arena.sync_shadow()
    c, h, w = arms["eager"].net_cfg.input_shape
    g = torch.Generator().manual_seed(3)
    for step in range(5):
        x = torch.randn(batch, c, h, w, generator=g).cuda()
        y = torch.randint(0, 1000, (batch, 1), generator=g).float().cuda()
        for t in arms.values():
            t.update(DataBatch(x, y))
        torch.cuda.synchronize()
        e = arms["eager"].net.arena
        line = [f"step {step}"]
        for name, t in arms.items():
            a = t.net.arena
            line.append(f"{name}: |w| {a.w.norm().item():.5g} |m1| {a.m1.norm().item():.4g} "
                        f"rel_m1 {((a.m1 - e.m1).norm() / e.m1.norm().clamp_min(1e-12)).item():.3g} "
                        f"fused {sorted(t.net.updater.fused_offsets)} plans {list(t._lists) + list(t._graphs)}")
        print(" | ".join(line), flush=True)
        for li, s in e.specs:
            for name in ("list", "graph"):
                a = arms[name].net.arena
                d = (a.m1[s.offset:s.offset + s.numel] - e.m1[s.offset:s.offset + s.numel]).norm().item()
                n = e.m1[s.offset:s.offset + s.numel].norm().item()
                if d > 0.2 * n + 1e-12:
                    print(f"   {name} {li}:{s.tag} |dm1| {d:.3g} |m1| {n:.3g}", flush=True)


if __name__ == "__main__":
    main()
