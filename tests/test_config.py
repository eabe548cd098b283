"""Config language, NetConfig graph parsing and structure serialization
(reference src/utils/config.h, src/nnet/nnet_config.h)."""
import os

import pytest

from cxxnet_amd import native

REF = "/root/reference/example"


def rt():
    return native.rt()


def test_tokenizer_basic_and_comments():
    kv = rt().parse_config('a = 1\n# comment = x\nb=2 c = "hello world" # tail\nd = \'multi\nline\'\n')
    assert kv == [("a", "1"), ("b", "2"), ("c", "hello world"), ("d", "multi\nline")]


def test_tokenizer_escapes_and_equal_in_string():
    kv = rt().parse_config('path = "a\\"b=c"\nx=y')
    assert kv == [("path", 'a"b=c'), ("x", "y")]


def test_tokenizer_unterminated_string():
    with pytest.raises(RuntimeError):
        rt().parse_config('a = "abc\n')


def test_layer_types():
    gt = rt().get_layer_type
    assert gt("fullc") == 1 and gt("conv") == 10 and gt("relu_max_pooling") == 21
    assert gt("share[fc1]") == 0
    assert gt("pairtest-conv-conv") == 1024 * 10 + 10
    with pytest.raises(RuntimeError):
        gt("nonexistent")


NET = """
netconfig=start
layer[+1:fc1] = fullc:fc1
  nhidden = 100
layer[+1:sg1] = sigmoid:se1
layer[sg1->fc2] = fullc:fc2
  nhidden = 10
layer[+0] = softmax
netconfig=end
input_shape = 1,1,784
batch_size = 100
eta = 0.1
label_vec[1,3) = extra
updater = nag
"""


def test_netconfig_parse():
    c = rt().NetConfig()
    c.configure(rt().parse_config(NET))
    assert c.node_names == ["in", "fc1", "sg1", "fc2"]
    assert [(l.type, l.name, list(l.nindex_in), list(l.nindex_out)) for l in c.layers] == [
        (1, "fc1", [0], [1]), (4, "se1", [1], [2]), (1, "fc2", [2], [3]), (2, "", [3], [3])]
    assert c.input_shape == [1, 1, 784]
    assert c.layercfg[0] == [("nhidden", "100")]
    assert ("eta", "0.1") in c.defcfg
    assert c.updater_type == "nag"
    assert c.label_name_map["extra"] == 1 and c.label_range[1] == (1, 3)
    assert c.get_layer_index("fc2") == 2


def test_netconfig_roundtrip_bytes():
    c = rt().NetConfig()
    c.configure(rt().parse_config(NET))
    b = c.save_net()
    # NetParam is 152 bytes, then node names with uint64 length prefixes
    assert len(b) > 152
    c2 = rt().NetConfig()
    assert c2.load_net(b) == len(b)
    assert c2.save_net() == b
    # reconfiguring a loaded structure with the same conf is accepted
    c2.configure(rt().parse_config(NET))
    with pytest.raises(RuntimeError):
        c3 = rt().NetConfig()
        c3.load_net(b)
        c3.configure(rt().parse_config(NET.replace("fullc:fc2", "fullc:fcX")))


def test_shared_layer_and_errors():
    conf = NET.replace("layer[+0] = softmax", "layer[+1] = share[fc2]\nlayer[+0] = softmax")
    c = rt().NetConfig()
    with pytest.raises(RuntimeError):  # fc2 output 10 -> share[fc2] is structurally fine to parse
        c.configure(rt().parse_config("netconfig=start\nlayer[x->y] = relu\nnetconfig=end\n"))
    c = rt().NetConfig()
    c.configure(rt().parse_config(conf))
    assert c.layers[3].type == 0 and c.layers[3].primary_layer_index == 2


@pytest.mark.skipif(not os.path.exists(REF), reason="reference examples not mounted")
@pytest.mark.parametrize("path", ["ImageNet/ImageNet.conf", "MNIST/MNIST.conf", "MNIST/MNIST_CONV.conf",
                                  "kaggle_bowl/bowl.conf"])
def test_reference_confs_parse(path):
    kv = rt().parse_config_file(os.path.join(REF, path))
    c = rt().NetConfig()
    c.configure(kv)
    assert c.num_layers > 3 and c.init_end == 1


def test_layer_param_pod():
    p = rt().LayerParam()
    assert len(p.to_bytes()) == 328
    p.set_param("kernel_size", "5")
    p.set_param("pad", "2")
    p.set_param("random_type", "xavier")
    q = rt().LayerParam.from_bytes(p.to_bytes())
    assert (q.kernel_height, q.kernel_width, q.pad_x, q.pad_y, q.random_type) == (5, 5, 2, 2, 1)
    assert q.temp_col_max == 64 << 18 and q.init_uniform == -1.0


def test_precision_key():
    """`precision` accepts bf16 / fp32; on the CPU it changes nothing (the CPU path is fp32)."""
    import pytest as _pytest
    from cxxnet_amd.nnet import NetTrainer
    from cxxnet_amd.ops.mode import reference_precision
    tr = NetTrainer()
    tr.set_param("precision", "fp32")
    assert tr.precision == "fp32"
    with _pytest.raises(ValueError):
        tr.set_param("precision", "fp16")
    tr._apply_modes()
    assert not reference_precision()  # no GPU device: the host executor is fp32 already
