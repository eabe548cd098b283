"""Find where a launch-list replayed step departs from the eager step: two trainers (same seed,
deterministic GEMMs, fc SGD unfused), compared after every step on every node buffer, the
gradient arena and the weights."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    from test_dp_gloo import CONF
    from cxxnet_amd import native
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    from cxxnet_amd.nnet import trainer as trainer_mod
    model = sys.argv[1] if len(sys.argv) > 1 else "small"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    # argv[3]: "default" = the trainer's defaults (fc SGD fused in eager steps, atomic weight
    # gradients); otherwise deterministic GEMMs and unfused fc SGD (bitwise comparable)
    exact = not (len(sys.argv) > 3 and sys.argv[3] == "default")
    trainer_mod._FUSE_FC_SGD = not exact

    def make(rep):
        tr = NetTrainer()
        base = list(native.rt().parse_config(CONF)) if model == "small" else \
            [(k, v) for k, v in load_conf(model, []) if not k.startswith("metric")]
        for k, v in base + [("batch_size", str(batch)), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"),
                            ("seed", "5"), ("cuda_graph", "0"), ("deterministic", str(int(exact))),
                            ("launch_replay", str(rep))]:
            tr.set_param(k, v)
        tr.init_model()
        return tr

    a, b = make(0), make(1)
    shape = (3, 8, 8) if model == "small" else tuple(int(v) for v in dict(load_conf(model, [])).get("input_shape", "3,227,227").split(","))
    g = torch.Generator().manual_seed(11)
    for step in range(5):
        x = torch.randn(batch, *shape, generator=g)
        y = torch.randint(0, 5, (batch, 1), generator=g).float()
        a.update(DataBatch(x.cuda(), y.cuda()))
        b.update(DataBatch(x.cuda(), y.cuda()))
        torch.cuda.synchronize()
        diffs = []
        for i, (na, nb) in enumerate(zip(a.net.nodes, b.net.nodes)):
            if na.data is not None and not torch.equal(na.data, nb.data):
                diffs.append(f"node{i}:{(na.data.float() - nb.data.float()).abs().max().item():.3g}")
        for name in ("g", "w", "m1"):
            ta, tb = getattr(a.net.arena, name), getattr(b.net.arena, name)
            if not torch.equal(ta, tb):
                d = (ta - tb).abs()
                idx = int(d.argmax())
                owner = next((f"{li}:{s.tag}" for li, s in a.net.arena.specs if s.offset <= idx < s.offset + s.numel), "?")
                diffs.append(f"{name}:max{d.max().item():.3g}@{owner}")
        print(f"step {step} lists={list(b._lists)} diffs: {' '.join(diffs) if diffs else 'none'}", flush=True)
        if not exact:
            for name in ("w", "m1"):
                ta, tb = getattr(a.net.arena, name), getattr(b.net.arena, name)
                print(f"   {name}: rel {((ta - tb).norm() / ta.norm().clamp_min(1e-30)).item():.3g} "
                      f"finite {bool(torch.isfinite(ta).all())}/{bool(torch.isfinite(tb).all())}", flush=True)


if __name__ == "__main__":
    main()
