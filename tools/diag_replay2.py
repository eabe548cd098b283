"""(a) inception_v1 b8, exact mode: at the first step whose gradient arena differs between the
eager and the replayed trainer, every differing parameter with its layer type.
(b) alexnet b8 with a NaN in the input: does the NaN reach the nodes / gradients of the
replayed step (check_nonfinite must see it)?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make(model, batch, rep, exact=True, extra=()):
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    tr = NetTrainer()
    base = [(k, v) for k, v in load_conf(model, []) if not k.startswith("metric")]
    for k, v in base + [("batch_size", str(batch)), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"),
                        ("seed", "5"), ("cuda_graph", "0"), ("deterministic", str(int(exact))),
                        ("launch_replay", str(rep))] + list(extra):
        tr.set_param(k, v)
    tr.init_model()
    return tr


def part_a():
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.nnet import trainer as trainer_mod
    trainer_mod._FUSE_FC_SGD = False
    a, b = make("inception_v1", 8, 0), make("inception_v1", 8, 1)
    layer_of = {}
    for i, c in enumerate(a.net.connections):
        layer_of[i] = c.layer.type_name
    g = torch.Generator().manual_seed(11)
    for step in range(4):
        x = torch.randn(8, 3, 224, 224, generator=g)
        y = torch.randint(0, 5, (8, 1), generator=g).float()
        a.update(DataBatch(x.cuda(), y.cuda()))
        b.update(DataBatch(x.cuda(), y.cuda()))
        torch.cuda.synchronize()
        bad = []
        for li, s in a.net.arena.specs:
            ga = a.net.arena.g[s.offset:s.offset + s.numel]
            gb = b.net.arena.g[s.offset:s.offset + s.numel]
            if not torch.equal(ga, gb):
                bad.append(f"{li}:{layer_of.get(li, '?')}:{s.tag}:{(ga - gb).abs().max().item():.3g}"
                           f"{'' if torch.isfinite(gb).all() else ':NaN'}")
        print(f"step {step} differing grads ({len(bad)}): {' '.join(bad[:40])}", flush=True)
        if bad:
            lists = b._lists.get(8)
            if lists:
                print("  plan:", [type(i).__name__ + (f"({i.n})" if hasattr(i, "n") else "") for i in lists[0] + lists[1]][:60])
            break


def part_b():
    from cxxnet_amd.io.data import DataBatch
    for rep in (0, 1):
        tr = make("alexnet", 8, rep, exact=False, extra=[("check_nonfinite", "1")])
        x = torch.randn(8, 3, 227, 227).cuda()
        y = torch.zeros(8, 1).cuda()
        for _ in range(3):
            tr.update(DataBatch(x, y))
        x[0, 0, 0, 0] = float("nan")
        try:
            tr.update(DataBatch(x, y))
            torch.cuda.synchronize()
            raised = False
        except FloatingPointError:
            raised = True
        nan_nodes = [i for i, n in enumerate(tr.net.nodes) if n.data is not None and not torch.isfinite(n.data.float()).all()]
        print(f"replay={rep} lists={list(tr._lists)} raised={raised} g finite={bool(torch.isfinite(tr.net.arena.g).all())} "
              f"nan nodes={nan_nodes[:20]} input node0 nan={not bool(torch.isfinite(tr.net.nodes[0].data.float()).all())}",
              flush=True)


if __name__ == "__main__":
    part_b()
    part_a()
