"""Every GPU kernel of a training step's forward and backward passes must come from the library
(libcxxnet_kernels.so): the C++ launch-list executor replays only library launches, so a torch
op on that path (a .zero_(), .contiguous(), .add_() ...) runs in the recording step and silently
not in the replays.  Round 4 found three such ops by their effect (gradients never zeroed, a
stale concat-slice copy read as NaN, conv1's weight gradient never added); this test finds the
next one by its kernel name, on the real graphs, in both GEMM modes."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(model, batch, det):
    from cxxnet_amd.models import load_conf
    from cxxnet_amd.nnet import NetTrainer
    tr = NetTrainer()
    base = [(k, v) for k, v in load_conf(model, []) if not k.startswith("metric")]
    for k, v in base + [("batch_size", str(batch)), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"),
                        ("cuda_graph", "0"), ("launch_replay", "0"), ("deterministic", str(det))]:
        tr.set_param(k, v)
    tr.init_model()
    return tr


@pytest.mark.parametrize("det", [0, 1])
@pytest.mark.parametrize("model,batch", [("alexnet", 16), ("inception_v1", 8), ("vgg16", 4)])
def test_forward_backward_launch_only_library_kernels(model, batch, det):
    from torch.profiler import ProfilerActivity, profile
    from cxxnet_amd.io.data import DataBatch
    tr = _make(model, batch, det)
    c, h, w = tr.net_cfg.input_shape
    b = DataBatch(torch.randn(batch, c, h, w, device="cuda"), torch.zeros(batch, 1, device="cuda"))
    for _ in range(2):  # tile tuning and lazy buffers happen in the first steps
        tr.update(b)
    tr._set_batch(b)
    net = tr.net
    # the pass below runs unfused (no optimizer handed to the fc layers): its weight-gradient
    # signatures are timed on first use (torch ops of the tuner, never inside a recorded step)
    net.forward(True)
    net.backprop(False, first=True)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        net.forward(True)
        net.backprop(False, first=True)
        torch.cuda.synchronize()
    foreign = sorted({e.name for e in prof.events()
                      if e.device_type == torch.autograd.DeviceType.CUDA and "at::native" in e.name})
    assert not foreign, foreign


# Every layer class that declares itself replay-safe (Layer.replay_audited) appears in this net:
# a torch op added to any of them later shows up here by kernel name.
ALL_AUDITED_NET = """
netconfig=start
layer[0->1] = conv:c1
  kernel_size = 3
  nchannel = 16
  pad = 1
layer[1->2] = relu
layer[2->3,4] = split
layer[3->5] = conv:c2a
  kernel_size = 1
  nchannel = 16
layer[4->6] = conv:c2b
  kernel_size = 3
  pad = 1
  nchannel = 16
  ngroup = 2
layer[5,6->7] = ch_concat
layer[7->8] = batch_norm:bn
layer[8->9] = xelu
layer[9->10] = max_pooling
  kernel_size = 3
  stride = 2
layer[10->11] = lrn
  local_size = 5
  alpha = 0.001
  beta = 0.75
layer[11->12] = tanh
layer[12->13] = sum_pooling
  kernel_size = 2
  stride = 2
layer[13->14] = conv:c3
  kernel_size = 3
  pad = 1
  nchannel = 16
layer[14->15] = relu_max_pooling
  kernel_size = 2
  stride = 2
layer[15->16] = avg_pooling
  kernel_size = 2
  stride = 2
layer[16->17] = flatten
layer[17->18] = fullc:f1
  nhidden = 32
layer[18->19] = sigmoid
layer[19->20,21] = split
layer[20->22] = fullc:f2a
  nhidden = 16
layer[21->23] = fullc:f2b
  nhidden = 16
layer[22,23->24] = concat
layer[24->24] = bias:b
layer[24->24] = dropout
  threshold = 0.25
layer[24->25] = fullc:f3
  nhidden = 10
layer[25->25] = softmax
netconfig=end
input_shape = 8,16,16
"""


@pytest.mark.parametrize("det", [0, 1])
def test_every_audited_layer_launches_only_library_kernels(det):
    from torch.profiler import ProfilerActivity, profile
    from cxxnet_amd import native
    from cxxnet_amd.io.data import DataBatch
    from cxxnet_amd.nnet import NetTrainer
    tr = NetTrainer()
    for k, v in list(native.rt().parse_config(ALL_AUDITED_NET)) + [
            ("batch_size", "8"), ("dev", "gpu"), ("eval_train", "0"), ("silent", "1"), ("cuda_graph", "0"),
            ("launch_replay", "0"), ("deterministic", str(det))]:
        tr.set_param(k, v)
    tr.init_model()
    audited = {type(c.layer).__name__ for c in tr.net.connections if type(c.layer).replay_audited}
    from test_replay_audit_cpu import AUDITED
    assert audited == AUDITED, audited ^ AUDITED
    b = DataBatch(torch.randn(8, 8, 16, 16, device="cuda"), torch.randint(0, 10, (8, 1), device="cuda").float())
    for _ in range(2):
        tr.update(b)
    tr._set_batch(b)
    net = tr.net
    net.forward(True)
    net.backprop(False, first=True)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        net.forward(True)
        net.backprop(False, first=True)
        torch.cuda.synchronize()
    foreign = sorted({e.name for e in prof.events()
                      if e.device_type == torch.autograd.DeviceType.CUDA and "at::native" in e.name})
    assert not foreign, foreign
