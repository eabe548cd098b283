"""The image iterators feed the trainer's device (io/image.py consumer_device): no prefetch or
GPU decode for dev = cpu, the configured GPU for dev = gpu:N, the rank's GPU by default; and a
data-parallel rank's prefetch holds only its own rows (io/data.py U8Images.on_device)."""
import types

import torch

from cxxnet_amd.io import image
from cxxnet_amd.io.data import U8Images


def test_consumer_device_follows_dev(monkeypatch):
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    assert image.consumer_device("cpu") is None
    assert image.consumer_device("gpu:1") == torch.device("cuda", 1)
    assert image.consumer_device("gpu") == torch.device("cuda", 0)
    assert image.consumer_device(None) == torch.device("cuda", 0)
    monkeypatch.setenv("LOCAL_RANK", "1")
    assert image.consumer_device(None) == torch.device("cuda", 1)


def test_consumer_device_without_gpu():
    if torch.cuda.is_available():
        return
    assert image.consumer_device("gpu:0") is None and image.consumer_device(None) is None


def test_iterator_defaults_follow_dev(monkeypatch, tmp_path):
    it = image.create_image_iterator("img")
    it.set_param("dev", "cpu")
    it.set_param("prefetch_device", "1")  # meaningless with a host consumer: forced off
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    it._dev = image.consumer_device(it.dev)
    assert it._dev is None


def _fake_prefetch(lo, n, rows_total):
    pix = torch.arange(rows_total * 2, dtype=torch.uint8).view(rows_total, 1, 2, 1)
    prm = torch.zeros(rows_total, 4, dtype=torch.int32)
    cm = torch.zeros(rows_total, 2)
    copied = [pix[lo:lo + n], prm[lo:lo + n], cm[lo:lo + n]]
    pf = types.SimpleNamespace(lo=lo, tensors=copied, take=lambda dev: copied)
    return U8Images(pix, prm, cm, pf=pf, rows=(0, rows_total)), pix


def test_sharded_prefetch_rows():
    u, pix = _fake_prefetch(4, 4, 16)  # this rank decoded and copied rows 4..7 of 16
    view = u[4:8]
    got = view.on_device("cuda:0")
    assert got is not None and torch.equal(got[0], pix[4:8])
    assert u[2:6].on_device("cuda:0") is None  # reaches rows the prefetch does not hold
    assert u.on_device("cuda:0") is None
    u2, pix2 = _fake_prefetch(0, 16, 16)
    assert torch.equal(u2[3:9].on_device("cuda:0")[0], pix2[3:9])
