"""CLI task driver on the CPU path: train / continue / finetune / pred / extract with a
synthetic MNIST-format dataset (gz idx files written by the test, since no dataset is
available offline).  Mirrors reference example/MNIST/MNIST.conf."""
import gzip
import os
import struct

import numpy as np
import pytest

from cxxnet_amd.cli import LearnTask


def write_idx(tmp, n=2000, seed=0):
    rng = np.random.RandomState(seed)
    labels = rng.randint(0, 10, size=n).astype(np.uint8)
    protos = rng.randint(0, 256, size=(10, 28, 28)).astype(np.float32)
    imgs = np.clip(protos[labels] * 0.7 + rng.randint(0, 80, size=(n, 28, 28)), 0, 255).astype(np.uint8)
    ip, lp = os.path.join(tmp, "img.gz"), os.path.join(tmp, "lab.gz")
    with gzip.open(ip, "wb") as f:
        f.write(struct.pack(">iiii", 2051, n, 28, 28) + imgs.tobytes())
    with gzip.open(lp, "wb") as f:
        f.write(struct.pack(">ii", 2049, n) + labels.tobytes())
    return ip, lp, labels


CONF = """
data = train
iter = mnist
    path_img = "{img}"
    path_label = "{lab}"
    shuffle = 1
iter = end
eval = test
iter = mnist
    path_img = "{img}"
    path_label = "{lab}"
iter = end
pred = {pred}
iter = mnist
    path_img = "{img}"
    path_label = "{lab}"
iter = end
netconfig=start
layer[+1:fc1] = fullc:fc1
  nhidden = 64
  init_sigma = 0.01
layer[+1:sg1] = sigmoid:se1
layer[sg1->fc2] = fullc:fc2
  nhidden = 10
  init_sigma = 0.01
layer[+0] = softmax
netconfig=end
input_shape = 1,1,784
batch_size = 100
dev = cpu
save_model = 1
max_round = 4
num_round = 4
random_type = gaussian
eta = 0.1
momentum = 0.9
wd  = 0.0
metric[label] = error
model_dir = {mdir}
silent = 1
"""


@pytest.fixture()
def conf(tmp_path):
    ip, lp, labels = write_idx(str(tmp_path))
    p = tmp_path / "mnist.conf"
    p.write_text(CONF.format(img=ip, lab=lp, pred=tmp_path / "pred.txt", mdir=tmp_path / "models"))
    return str(p), tmp_path, labels


def test_train_pred_extract_continue_finetune(conf, capfd):
    path, tmp, labels = conf
    assert LearnTask().run([path]) == 0
    err = capfd.readouterr().err.strip().splitlines()
    assert err[-1].startswith("[4]\ttrain-error:") and "\ttest-error:" in err[-1]
    final_err = float(err[-1].split(":")[-1])
    assert final_err < 0.2, err
    models = sorted(os.listdir(tmp / "models"))
    assert models == ["0000.model", "0001.model", "0002.model", "0003.model", "0004.model"]

    # pred with the final model: labels as %g lines; accuracy matches the eval error
    assert LearnTask().run([path, "task=pred", f"model_in={tmp}/models/0004.model"]) == 0
    pred = np.loadtxt(tmp / "pred.txt")
    assert pred.shape == (2000,)
    assert np.mean(pred != labels) == pytest.approx(final_err, abs=0.02)

    # extract a hidden node in text and binary form with its .meta
    assert LearnTask().run([path, "task=extract", f"model_in={tmp}/models/0004.model",
                            "extract_node_name=sg1", "output_format=txt"]) == 0
    feat = np.loadtxt(tmp / "pred.txt")
    assert feat.shape == (2000, 64)
    assert (tmp / "pred.txt.meta").read_text().strip() == "2000,1,1,64"
    assert LearnTask().run([path, "task=extract", f"model_in={tmp}/models/0004.model",
                            "extract_node_name=top[-1]", "output_format=bin"]) == 0
    raw = np.fromfile(tmp / "pred.txt", dtype=np.float32).reshape(2000, 10)
    assert np.allclose(raw.sum(1), 1.0, atol=1e-4)

    # continue: picks up 0004.model and trains up to num_round=6
    capfd.readouterr()
    assert LearnTask().run([path, "continue=1", "num_round=6", "max_round=6"]) == 0
    assert "0006.model" in os.listdir(tmp / "models")

    # finetune: new head (fc2 renamed) keeps fc1 weights from the model
    fin = LearnTask()
    ft_conf = open(path).read().replace("fullc:fc2", "fullc:fc2new")
    p2 = tmp / "ft.conf"
    p2.write_text(ft_conf.replace(str(tmp / "models"), str(tmp / "ft_models")))
    assert fin.run([str(p2), "task=finetune", f"model_in={tmp}/models/0004.model", "num_round=1",
                    "max_round=1"]) == 0
    from cxxnet_amd.nnet import NetTrainer  # noqa: F401
    src = LearnTask()
    src.set_param("dev", "cpu")
    for k, v in __import__("cxxnet_amd").native.rt().parse_config(open(path).read()):
        src.set_param(k, v)
    src.name_model_in = f"{tmp}/models/0004.model"
    src.task = "pred"
    src.load_model()
    w_old = src.trainer.get_weight("fc1", "wmat")
    # the finetuned model's first checkpoint (0000) holds the copied fc1
    data = open(tmp / "ft_models" / "0000.model", "rb").read()
    t2 = LearnTask()
    for k, v in __import__("cxxnet_amd").native.rt().parse_config(ft_conf):
        t2.set_param(k, v)
    t2.name_model_in = str(tmp / "ft_models" / "0000.model")
    t2.task = "pred"
    t2.load_model()
    # finetune copied fc1 and trained one round: it stays close to the source weights
    w_new = t2.trainer.get_weight("fc1", "wmat")
    assert np.abs(w_new - w_old).mean() < 0.2 * np.abs(w_old).mean()
    assert data[:4] == b"\x00\x00\x00\x00"


def test_checkpoint_byte_exact_roundtrip(conf):
    path, tmp, _ = conf
    assert LearnTask().run([path, "num_round=1", "max_round=1"]) == 0
    raw = open(tmp / "models" / "0001.model", "rb").read()
    t = LearnTask()
    for k, v in __import__("cxxnet_amd").native.rt().parse_config(open(path).read()):
        t.set_param(k, v)
    t.name_model_in = str(tmp / "models" / "0001.model")
    t.task = "pred"
    t.load_model()
    again = b"\x00\x00\x00\x00" + t.trainer.save_model()
    assert again == raw
    # layout: int32 net_type | NetParam(152) ...
    num_nodes, num_layers = struct.unpack_from("<ii", raw, 4)
    assert (num_nodes, num_layers) == (4, 4)


def test_optimizer_state_sidecar_roundtrip(conf):
    """save_optimizer_state = 1 writes <model>.state (momentum + counters) beside each
    byte-compatible model file; continue = 1 restores it."""
    import torch
    path, tmp, _ = conf
    t = LearnTask()
    assert t.run([path, "max_round=2", "num_round=2", "save_optimizer_state=1"]) == 0
    mdir = tmp / "models"
    assert (mdir / "0002.model").exists() and (mdir / "0002.model.state").exists()
    m1 = t.trainer.net.arena.m1.clone()
    assert m1.abs().max() > 0
    t2 = LearnTask()
    for k, v in [("save_optimizer_state", "1"), ("continue", "1"), ("model_dir", str(mdir)), ("dev", "cpu"),
                 ("silent", "1")]:
        t2.set_param(k, v)
    from cxxnet_amd import native
    for k, v in native.rt().parse_config_file(path):
        t2.set_param(k, v)
    t2.set_param("continue", "1")
    t2.set_param("save_optimizer_state", "1")
    t2.init()
    assert torch.equal(t2.trainer.net.arena.m1, m1)
    # without the key the momentum starts from zero, as in the reference
    t3 = LearnTask()
    for k, v in native.rt().parse_config_file(path):
        t3.set_param(k, v)
    t3.set_param("continue", "1")
    t3.init()
    assert t3.trainer.net.arena.m1.abs().max() == 0


def test_check_nonfinite_fails_fast(conf):
    import torch
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.nnet import NetTrainer
    from cxxnet_amd.models import load_conf
    tr = NetTrainer()
    for k, v in load_conf("mnist_mlp", [("dev", "cpu"), ("batch_size", "8"), ("silent", "1"),
                                        ("check_nonfinite", "1")]):
        tr.set_param(k, v)
    tr.init_model()
    shape = tr.net_cfg.input_shape
    tr.update(DataBatch(torch.randn(8, *shape), torch.zeros(8, 1)))  # finite: passes
    x = torch.randn(8, *shape)
    x[0, 0, 0, 0] = float("nan")
    with pytest.raises(FloatingPointError):
        tr.update(DataBatch(x, torch.zeros(8, 1)))


def test_step_timeout_watchdog_aborts():
    """A stalled job exits with code 3 within ~step_timeout instead of hanging."""
    import subprocess
    import sys
    code = ("import time\nfrom cxxnet_amd.cli import LearnTask\nt = LearnTask()\nt.set_param('step_timeout', '0.5')\n"
            "t._start_watchdog()\ntime.sleep(30)\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=60)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "step_timeout" in r.stderr
