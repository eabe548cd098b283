"""Drive training from Python with the cxxnet API (DataIter / Net / train).

Run from this directory after placing the MNIST files in ./data/.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

from cxxnet_amd.wrapper import DataIter, Net, train  # noqa: E402

NET = """
netconfig = start
layer[+1:fc1] = fullc:fc1
  nhidden = 100
  init_sigma = 0.01
layer[+1:sg1] = sigmoid:se1
layer[sg1->fc2] = fullc:fc2
  nhidden = 10
  init_sigma = 0.01
layer[+0] = softmax
netconfig = end
input_shape = 1,1,784
batch_size = 100
random_type = gaussian
"""

ITER = """
iter = mnist
  path_img = "./data/{0}-images-idx3-ubyte.gz"
  path_label = "./data/{0}-labels-idx1-ubyte.gz"
  shuffle = {1}
iter = end
input_flat = 1
batch_size = 100
"""


def main():
    data = DataIter(ITER.format("train", 1))
    deval = DataIter(ITER.format("t10k", 0))
    param = {"eta": 0.1, "momentum": 0.9, "wd": 0.0, "metric": "error", "dev": "cpu"}
    net = train(NET, data, 1, param, eval_data=deval)

    # predictions from an iterator and from an ndarray agree
    deval.before_first()
    deval.next()
    x, y = deval.get_data(), deval.get_label()
    assert (net.predict(deval) == net.predict(x)).all()
    print("first-batch accuracy:", float((net.predict(x) == y[:, 0]).mean()))

    # hidden features, manual updates, weight round trip
    print("sg1 features:", net.extract(x, "sg1").shape)
    for _ in range(10):
        net.update(x, y)
    w = net.get_weight("fc1", "wmat")
    net.set_weight(np.zeros_like(w), "fc1", "wmat")
    net.set_weight(w, "fc1", "wmat")
    print(net.evaluate(deval, "test"))


if __name__ == "__main__":
    main()
