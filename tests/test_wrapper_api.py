"""Python API (DataIter / Net / train) and the CXN* C ABI (libcxxnetwrapper.so).

Mirrors the reference's integration script example/MNIST/mnist.py:57-112:
predict(iter) == predict(ndarray), extract(iter) == extract(ndarray), a manual
update loop, and get_weight -> set_weight restoring the evaluation error."""
import ctypes
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from cxxnet_amd import build, wrapper
from test_cli_cpu import write_idx

NET = """
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
random_type = gaussian
"""

PARAM = {"eta": 0.1, "momentum": 0.9, "wd": 0.0, "metric": "error", "silent": 1}


@pytest.fixture(scope="module")
def mnist(tmp_path_factory):
    d = tmp_path_factory.mktemp("mnist")
    ip, lp, labels = write_idx(str(d), n=2000)
    it_cfg = f"""
iter = mnist
  path_img = "{ip}"
  path_label = "{lp}"
  silent = 1
iter = end
input_flat = 1
batch_size = 100
"""
    return ip, lp, it_cfg


def _err(s):
    return float(s.strip().split(":")[-1])


def test_python_api_matches_reference_script(mnist):
    _, _, it_cfg = mnist
    data = wrapper.DataIter(it_cfg)
    deval = wrapper.DataIter(it_cfg)
    net = wrapper.train(NET, data, 4, PARAM, eval_data=deval)
    err0 = _err(net.evaluate(deval, "eval"))
    assert err0 < 0.5

    data.before_first()
    assert data.next()
    x, y = data.get_data(), data.get_label()
    assert x.shape == (100, 1, 1, 784) and y.shape == (100, 1)
    np.testing.assert_array_equal(net.predict(data), net.predict(x))
    np.testing.assert_allclose(net.extract(data, "sg1"), net.extract(x, "sg1"), rtol=1e-6)
    assert net.extract(x, "top[-1]").shape == (100, 1, 1, 10)

    # manual update loop on ndarrays
    for _ in range(3):
        net.update(x, y)

    # weight round trip: perturb, then restore -> same error
    w = net.get_weight("fc1", "wmat")
    b = net.get_weight("fc1", "bias")
    assert w.shape == (64, 784)
    net.set_weight(np.zeros_like(w), "fc1", "wmat")
    net.set_weight(w, "fc1", "wmat")
    net.set_weight(b, "fc1", "bias")
    np.testing.assert_array_equal(net.get_weight("fc1", "wmat"), w)


def test_python_api_save_load(mnist, tmp_path):
    _, _, it_cfg = mnist
    data = wrapper.DataIter(it_cfg)
    net = wrapper.train(NET, data, 1, PARAM)
    f = str(tmp_path / "m.model")
    net.save_model(f)
    net2 = wrapper.Net(dev="cpu", cfg=NET)
    net2.load_model(f)
    data.before_first()
    data.next()
    np.testing.assert_array_equal(net.predict(data), net2.predict(data))


def test_train_ndarray_signature(mnist):
    _, _, it_cfg = mnist
    it = wrapper.DataIter(it_cfg)
    it.next()
    x, y = it.get_data(), it.get_label()
    net = wrapper.train(NET, x, y, 2, PARAM)
    assert net.predict(x).shape == (100,)


@pytest.fixture(scope="module")
def capi_lib():
    return build.build_wrapper()


def test_capi_ctypes_in_process(mnist, capi_lib):
    """Loaded from a running interpreter: joins it rather than starting another."""
    _, _, it_cfg = mnist
    lib = ctypes.CDLL(capi_lib)
    lib.CXNIOCreateFromConfig.restype = ctypes.c_void_p
    lib.CXNNetCreate.restype = ctypes.c_void_p
    lib.CXNIOGetData.restype = ctypes.POINTER(ctypes.c_float)
    lib.CXNNetPredictIter.restype = ctypes.POINTER(ctypes.c_float)
    lib.CXNNetEvaluate.restype = ctypes.c_char_p
    for f in ("CXNIONext", "CXNIOBeforeFirst", "CXNIOGetData", "CXNNetSetParam", "CXNNetInitModel",
              "CXNNetUpdateIter", "CXNNetPredictIter", "CXNNetEvaluate", "CXNIOFree", "CXNNetFree"):
        getattr(lib, f).argtypes = None
    it = ctypes.c_void_p(lib.CXNIOCreateFromConfig(it_cfg.encode()))
    net = ctypes.c_void_p(lib.CXNNetCreate(b"cpu", NET.encode()))
    assert it.value and net.value
    for k, v in PARAM.items():
        lib.CXNNetSetParam(net, str(k).encode(), str(v).encode())
    lib.CXNNetInitModel(net)
    lib.CXNIOBeforeFirst(it)
    n = 0
    while lib.CXNIONext(it):
        lib.CXNNetUpdateIter(net, it)
        n += 1
    assert n == 20
    ev = lib.CXNNetEvaluate(net, it, b"eval").decode()
    assert "eval-error" in ev
    lib.CXNIOBeforeFirst(it)
    assert lib.CXNIONext(it)
    shape = (ctypes.c_uint * 4)()
    stride = ctypes.c_uint()
    p = lib.CXNIOGetData(it, shape, ctypes.byref(stride))
    assert list(shape) == [100, 1, 1, 784] and stride.value == 784
    assert 0.0 <= p[0] <= 1.0
    olen = ctypes.c_uint()
    pred = lib.CXNNetPredictIter(net, it, ctypes.byref(olen))
    assert olen.value == 100 and 0 <= pred[0] <= 9
    lib.CXNIOFree(it)
    lib.CXNNetFree(net)


def test_capi_embedded_from_c_program(mnist, capi_lib, tmp_path):
    """A plain C program drives training through the ABI (Python embedded)."""
    ip, lp, it_cfg = mnist
    src = tmp_path / "drive.c"
    hdr = os.path.join(os.path.dirname(build.__file__), "csrc", "capi")
    c_cfg = it_cfg.replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")
    c_net = NET.replace("\n", "\\n")
    src.write_text(textwrap.dedent(f"""
        #include <stdio.h>
        #include <string.h>
        #include "cxxnet_wrapper.h"
        int main(void) {{
          void *it = CXNIOCreateFromConfig("{c_cfg}");
          void *net = CXNNetCreate("cpu", "{c_net}");
          if (!it || !net) return 2;
          CXNNetSetParam(net, "eta", "0.1");
          CXNNetSetParam(net, "momentum", "0.9");
          CXNNetSetParam(net, "metric", "error");
          CXNNetInitModel(net);
          for (int r = 0; r < 2; ++r) {{
            CXNNetStartRound(net, r);
            CXNIOBeforeFirst(it);
            while (CXNIONext(it)) CXNNetUpdateIter(net, it);
          }}
          printf("%s\\n", CXNNetEvaluate(net, it, "eval"));
          cxx_uint shp[4], nd = 0;
          const float *w = CXNNetGetWeight(net, "fc2", "wmat", shp, &nd);
          printf("w %u %u %u %d\\n", nd, shp[0], shp[1], w != 0);
          CXNNetSaveModel(net, "{tmp_path}/c.model");
          CXNIOFree(it);
          CXNNetFree(net);
          return 0;
        }}
    """))
    exe = tmp_path / "drive"
    libdir = os.path.dirname(capi_lib)
    subprocess.run(["gcc", "-O1", str(src), "-I" + hdr, "-L" + libdir, "-lcxxnetwrapper",
                    "-Wl,-rpath," + libdir, "-o", str(exe)], check=True)
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join(p for p in sys.path if p)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert any("eval-error" in s for s in lines), r.stdout
    assert "w 2 10 64 1" in lines
    assert os.path.getsize(tmp_path / "c.model") > 0
