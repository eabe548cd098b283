"""Python API: ``DataIter``, ``Net``, ``train``, plus the bridge behind the CXN* C ABI.

Reference: wrapper/cxxnet.py:64-320 (ctypes classes over libcxxnetwrapper.so) and
wrapper/cxxnet_wrapper.cpp (WrapperIterator / WrapperNet).  Here the Python API is
the primary surface and talks to the trainer directly.  The C ABI
(csrc/capi/cxxnet_wrapper.cpp -> _native/libcxxnetwrapper.so) embeds CPython and
calls the ``_capi_*`` functions at the bottom of this module.

Arrays are numpy float32: data (batch, channel, height, width), label (batch,
label_width).  A ``Net`` trains on whatever ``dev`` names (``cpu``, ``gpu``,
``gpu:N``).  Under torchrun the same script runs data-parallel with one process
per GPU.
"""
from __future__ import annotations

import struct
import sys
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import native
from .io import create_iterator
from .io.data import DataBatch, dense

__all__ = ["DataIter", "Net", "train"]


def _parse(cfg: str) -> List[Tuple[str, str]]:
    return [(k, v) for k, v in native.rt().parse_config(cfg + "\n")]


class DataIter:
    """Iterator built from an `iter = ...` config block (WrapperIterator).  Pairs
    after `iter = end` are set on the finished chain as defaults."""

    def __init__(self, cfg: str):
        itcfg, defcfg = [], []
        it = None
        for k, v in _parse(cfg):
            if k == "iter" and v == "end":
                if it is not None:
                    raise ValueError("wrong configuration file")
                it = create_iterator(itcfg)
                continue
            (defcfg if it is not None else itcfg).append((k, v))
        if it is None:
            it = create_iterator(itcfg)
        for k, v in defcfg:
            it.set_param(k, v)
        it.init()
        self._it = it
        self.head = True
        self.tail = False

    def next(self) -> bool:
        ok = self._it.next()
        self.head = False
        self.tail = not ok
        return ok

    def before_first(self):
        self._it.before_first()
        self.head = True
        self.tail = False

    def check_valid(self):
        if self.head:
            raise RuntimeError("iterator was at head state, call next to get to valid state")
        if self.tail:
            raise RuntimeError("iterator reaches end")

    def value(self) -> DataBatch:
        self.check_valid()
        return self._it.value()

    def get_data(self) -> np.ndarray:
        return dense(self.value().data).float().cpu().numpy()

    def get_label(self) -> np.ndarray:
        return self.value().label.float().cpu().numpy()


def _as_batch(data: np.ndarray, label: Optional[np.ndarray] = None) -> DataBatch:
    data = np.ascontiguousarray(data, dtype=np.float32)
    if data.ndim != 4:
        raise ValueError("need 4 dimensional tensor (batch, channel, height, width)")
    if label is None:
        lab = torch.zeros((data.shape[0], 1), dtype=torch.float32)
    else:
        label = np.asarray(label, dtype=np.float32)
        if label.ndim == 1:
            label = label.reshape(-1, 1)
        if label.ndim != 2:
            raise ValueError("label need to be 2 dimension or one dimension ndarray")
        if label.shape[0] != data.shape[0]:
            raise ValueError("data size mismatch")
        lab = torch.from_numpy(np.ascontiguousarray(label))
    return DataBatch(torch.from_numpy(data), lab, np.arange(data.shape[0], dtype=np.uint32))


class Net:
    """A trainable network (WrapperNet).  cfg is the netconfig text plus any global
    keys; set_param adds more; init_model/load_model creates the trainer."""

    def __init__(self, dev: str = "cpu", cfg: str = ""):
        self.cfg: List[Tuple[str, str]] = []
        self.net_type = 0
        self.silent = 0
        self.round_counter = 0
        self.trainer = None
        for k, v in _parse(cfg):
            self.set_param(k, v)
        if dev:
            self.set_param("dev", dev)

    def set_param(self, name, value):
        name, value = str(name), str(value)
        if name == "net_type" and self.trainer is not None:
            self.net_type = int(value)
            return
        if name == "silent":
            self.silent = int(value)
            return
        if name == "print_step":
            return
        if self.trainer is not None:
            self.trainer.set_param(name, value)
        self.cfg.append((name, value))

    def _create(self):
        from .nnet import create_net
        tr = create_net(self.net_type)
        for k, v in self.cfg:
            tr.set_param(k, v)
        return tr

    def init_model(self):
        self.trainer = self._create()
        self.trainer.init_model()

    def save_model(self, fname: str):
        self._need()
        blob = self.trainer.save_model()
        with open(fname, "wb") as f:
            f.write(struct.pack("<i", self.net_type))
            f.write(blob)

    def load_model(self, fname: str):
        with open(fname, "rb") as f:
            data = f.read()
        self.net_type = struct.unpack_from("<i", data, 0)[0]
        self.trainer = self._create()
        self.trainer.load_model(data, 4)

    def start_round(self, round_counter: int):
        self.round_counter = int(round_counter)
        if self.trainer is not None:
            self.trainer.start_round(self.round_counter)

    def _need(self):
        if self.trainer is None:
            raise RuntimeError("call init_model or load_model first")

    def update(self, data, label=None):
        self._need()
        if isinstance(data, DataIter):
            self.trainer.update(data.value())
        elif isinstance(data, np.ndarray):
            if label is None:
                raise ValueError("Net.update: need label to use update")
            self.trainer.update(_as_batch(data, label))
        else:
            raise TypeError(f"update do not support type {type(data)}")

    def evaluate(self, data, name: str) -> str:
        self._need()
        if not isinstance(data, DataIter):
            raise TypeError(f"evaluate do not support type {type(data)}")
        return self.trainer.evaluate(data._it, name)

    def predict(self, data) -> np.ndarray:
        self._need()
        batch = data.value() if isinstance(data, DataIter) else _as_batch(data)
        return np.asarray(self.trainer.predict(batch), dtype=np.float32)

    def extract(self, data, name: str) -> np.ndarray:
        self._need()
        batch = data.value() if isinstance(data, DataIter) else _as_batch(data)
        out = np.asarray(self.trainer.extract_feature(batch, name), dtype=np.float32)
        while out.ndim < 4:
            out = out.reshape(out.shape[0], 1, 1, -1) if out.ndim == 2 else out[:, None]
        return out

    def set_weight(self, weight: np.ndarray, layer_name: str, tag: str):
        self._need()
        if tag not in ("bias", "wmat"):
            raise ValueError("tag must be bias or wmat")
        self.trainer.set_weight(np.asarray(weight, dtype=np.float32), layer_name, tag)

    def get_weight(self, layer_name: str, tag: str) -> Optional[np.ndarray]:
        self._need()
        if tag not in ("bias", "wmat"):
            raise ValueError("tag must be bias or wmat")
        return self.trainer.get_weight(layer_name, tag)


def train(cfg: str, data, *args, **kw) -> Net:
    """train(cfg, iter, num_round, param, eval_data=None) or
    train(cfg, ndarray, label, num_round, param)  (wrapper/cxxnet.py:281-312)."""
    if isinstance(data, DataIter):
        names = ["num_round", "param", "eval_data"]
    else:
        names = ["label", "num_round", "param"]
    a = dict(zip(names, args))
    a.update(kw)
    net = Net(cfg=cfg)
    param = a.get("param") or {}
    for k, v in (param.items() if isinstance(param, dict) else param):
        net.set_param(k, v)
    net.init_model()
    for r in range(int(a["num_round"])):
        net.start_round(r)
        if isinstance(data, DataIter):
            data.before_first()
            n = 0
            while data.next():
                net.update(data)
                n += 1
                if n % 100 == 0 and not net.silent:
                    print(f"[{r}] {n} batch passed")
            if a.get("eval_data") is not None:
                sys.stderr.write(net.evaluate(a["eval_data"], "eval") + "\n")
        else:
            if not net.silent:
                print(f"Training in round {r}")
            net.update(data=data, label=a["label"])
    return net


# ----------------------------------------------------------------------------- C ABI bridge
# Called from csrc/capi/cxxnet_wrapper.cpp.  Arrays come in as memoryviews over the
# caller's float buffers and go back as (bytes, shape) so the C side can own a copy.
def _arr(mv, shape) -> np.ndarray:
    return np.frombuffer(mv, dtype=np.float32).reshape(tuple(shape)).copy()


def _out(a) -> Tuple[bytes, Tuple[int, ...]]:
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    return a.tobytes(), tuple(int(s) for s in a.shape)


def _capi_io_data(it: DataIter):
    return _out(it.get_data())


def _capi_io_label(it: DataIter):
    return _out(it.get_label())


def _capi_update_batch(net: Net, mv_data, dshape, mv_label, lshape):
    net.update(_arr(mv_data, dshape), _arr(mv_label, lshape))


def _capi_predict_batch(net: Net, mv_data, dshape):
    return _out(net.predict(_arr(mv_data, dshape)))


def _capi_predict_iter(net: Net, it: DataIter):
    return _out(net.predict(it))


def _capi_extract_batch(net: Net, mv_data, dshape, node: str):
    return _out(net.extract(_arr(mv_data, dshape), node))


def _capi_extract_iter(net: Net, it: DataIter, node: str):
    return _out(net.extract(it, node))


def _capi_set_weight(net: Net, mv, size: int, layer: str, tag: str):
    net.set_weight(_arr(mv, (size,)), layer, tag)


def _capi_get_weight(net: Net, layer: str, tag: str):
    w = net.get_weight(layer, tag)
    if w is None:
        return b"", ()
    return _out(w)

