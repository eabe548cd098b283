"""Image pipeline: img / imgbin / imgbinx iterators, augmenter, mean image, im2bin and
the partition maker (reference src/io/iter_*img*, tools/).  Uses PNG files so that
decoded pixels are exact."""
import os

import numpy as np
import pytest
import torch
from PIL import Image

from cxxnet_amd.io import create_iterator
from cxxnet_amd.io.data import U8Images, dense
from cxxnet_amd.io.image import load_mean_image
from cxxnet_amd.tools import im2bin, partition

N_IMG = 10


@pytest.fixture(scope="module")
def imgset(tmp_path_factory):
    d = tmp_path_factory.mktemp("imgs")
    rng = np.random.default_rng(0)
    arrays = {}
    lines = []
    for i in range(N_IMG):
        h, w = 40 + (i % 3) * 2, 44 + (i % 2) * 4
        a = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
        name = f"im{i}.png"
        Image.fromarray(a).save(d / name)
        arrays[100 + i] = a
        lines.append(f"{100 + i}\t{i % 4}\t{name}\n")
    (d / "all.lst").write_text("".join(lines))
    im2bin.main([str(d / "all.lst"), str(d) + "/", str(d / "all.bin")])
    return d, arrays


def _cfg(kind, d, **kw):
    cfg = [("iter", kind)]
    if kind == "img":
        cfg += [("image_list", str(d / "all.lst")), ("image_root", str(d) + "/")]
    else:
        cfg += [("image_list", str(d / "all.lst")), ("image_bin", str(d / "all.bin"))]
    base = {"input_shape": "3,32,32", "batch_size": "4", "silent": "1"}
    base.update({k: str(v) for k, v in kw.items()})
    cfg += list(base.items())
    cfg.append(("iter", "end"))
    return cfg


def _collect(it):
    out = []
    for b in it:
        out.append((dense(b.data).clone(), b.label.clone(), b.inst_index.copy(), b.num_batch_padd))
    return out


def _center(a, h=32, w=32):
    y, x = (a.shape[0] - h) // 2, (a.shape[1] - w) // 2
    return a[y:y + h, x:x + w]


def test_img_and_imgbin_agree_and_center_crop(imgset):
    d, arrays = imgset
    it_img = create_iterator(_cfg("img", d))
    it_img.init()
    it_bin = create_iterator(_cfg("imgbin", d))
    it_bin.init()
    a, b = _collect(it_img), _collect(it_bin)
    assert len(a) == 3 and [x[3] for x in a] == [0, 0, 2]
    for (da, la, ia, pa), (db, lb, ib, pb) in zip(a, b):
        assert torch.equal(da, db) and torch.equal(la, lb) and (ia == ib).all() and pa == pb
    # first batch pixels = center crops, CHW RGB
    for r in range(4):
        ref = torch.from_numpy(_center(arrays[int(a[0][2][r])]).copy()).permute(2, 0, 1).float()
        assert torch.equal(a[0][0][r], ref)
        assert float(a[0][1][r, 0]) == (int(a[0][2][r]) - 100) % 4


def test_round_batch_wraps(imgset):
    d, _ = imgset
    it = create_iterator(_cfg("imgbin", d, round_batch=1))
    it.init()
    batches = _collect(it)
    assert len(batches) == 3 and batches[-1][3] == 2
    assert list(batches[-1][2]) == [108, 109, 100, 101]
    # the wrapped rows were consumed: the next epoch starts after them
    it.before_first()
    assert it.next() and list(it.value().inst_index) == [102, 103, 104, 105]


def test_imgbinx_shuffle_is_permutation(imgset):
    d, _ = imgset
    seq = create_iterator(_cfg("imgbinx", d))
    seq.init()
    shuf = create_iterator(_cfg("imgbinx", d, shuffle=1))
    shuf.init()
    s = [i for b in _collect(seq) for i in b[2][: 4 - b[3]]]
    t = [i for b in _collect(shuf) for i in b[2][: 4 - b[3]]]
    assert s == list(range(100, 110))
    assert sorted(t) == s and t != s


def test_mean_value_mirror_scale(imgset):
    d, arrays = imgset
    it = create_iterator(_cfg("img", d, mean_value="10,20,30", mirror=1, scale=0.5))
    it.init()
    assert it.next()
    b = it.value()
    assert isinstance(b.data, U8Images) and b.data.mode == 1
    x = dense(b.data)
    a = _center(arrays[int(b.inst_index[0])]).astype(np.float32)[:, ::-1]
    ref = (a - np.array([10, 20, 30], np.float32)) * 0.5
    np.testing.assert_allclose(x[0].permute(1, 2, 0).numpy(), ref, rtol=0, atol=1e-5)


def test_rand_crop_mirror_deterministic(imgset):
    d, _ = imgset
    runs = []
    for _ in range(2):
        it = create_iterator(_cfg("imgbin", d, rand_crop=1, rand_mirror=1, seed_data=3))
        it.init()
        runs.append(_collect(it))
    for x, y in zip(*runs):
        assert torch.equal(x[0], y[0])


@pytest.mark.parametrize("kind", ["imgbin", "imgbinx", "img"])
def test_process_and_thread_decode_agree(imgset, kind):
    """decode_process (forkserver workers writing into shared memory) and the thread
    pool produce the same batches, random crop / mirror / contrast included, and the
    threadbuffer hands the batches over intact."""
    d, _ = imgset
    runs = {}
    for mode in ("thread", "process"):
        kw = dict(rand_crop=1, rand_mirror=1, seed_data=5, max_random_contrast=0.2, mean_value="1,2,3",
                  decode_process=(0 if mode == "thread" else 2), round_batch=1, decode_native=0)
        cfg = _cfg(kind, d, **kw)
        cfg.insert(-1, ("iter", "threadbuffer"))
        it = create_iterator(cfg)
        it.init()
        runs[mode] = _collect(it)
        raw = it.value().data
        assert raw.pix.dtype == torch.uint8 and raw.pix.shape == (4, 32, 32, 3)
        it.close()
    assert len(runs["thread"]) == len(runs["process"]) == 3
    for x, y in zip(runs["thread"], runs["process"]):
        assert torch.equal(x[0], y[0]) and torch.equal(x[1], y[1]) and (x[2] == y[2]).all()


def test_mean_image_created_and_used(imgset, tmp_path):
    d, arrays = imgset
    mpath = tmp_path / "mean.bin"
    it = create_iterator(_cfg("img", d, image_mean=str(mpath)))
    it.init()
    assert mpath.exists()
    mean = load_mean_image(str(mpath))
    ref = np.mean([_center(arrays[100 + i]).astype(np.float64) for i in range(N_IMG)], 0)
    np.testing.assert_allclose(mean.permute(1, 2, 0).numpy(), ref, rtol=1e-5, atol=1e-4)
    assert it.next()
    b = it.value()
    assert b.data.mode == 3
    x = dense(b.data)
    want = _center(arrays[int(b.inst_index[0])]).astype(np.float32) - mean.permute(1, 2, 0).numpy()
    np.testing.assert_allclose(x[0].permute(1, 2, 0).numpy(), want, atol=1e-4)


def test_affine_augment_shapes(imgset):
    d, _ = imgset
    it = create_iterator(_cfg("img", d, max_rotate_angle=15, max_shear_ratio=0.1, rand_crop=1,
                              min_random_scale=1.0, max_random_scale=1.2, fill_value=0))
    it.init()
    assert it.next()
    x = dense(it.value().data)
    assert tuple(x.shape) == (4, 3, 32, 32)
    assert float(x.max()) <= 255 and float(x.min()) >= 0


def test_partition_maker_and_conf_prefix(imgset, tmp_path):
    d, _ = imgset
    with open(d / "all.lst") as f:
        lines = f.readlines()
    # ~2.5 images per part at this tiny partition size
    parts = partition.make_partitions(lines, str(d) + "/", "part%d", str(tmp_path), partition_mb=0)
    assert len(parts) == N_IMG
    for lst, binp, items in parts:
        with open(lst, "w") as fw:
            fw.writelines(items)
        im2bin.main([lst, str(d) + "/", binp])
    cfg = [("iter", "imgbin"), ("image_conf_prefix", str(tmp_path / "part%d")),
           ("image_conf_ids", f"1-{len(parts)}"), ("input_shape", "3,32,32"), ("batch_size", "5"),
           ("silent", "1"), ("iter", "end")]
    it = create_iterator(cfg)
    it.init()
    idx = [i for b in _collect(it) for i in b[2]]
    assert idx == list(range(100, 110))
    # dist sharding of the conf ids (reference ParseImageConf)
    cfg2 = cfg[:-1] + [("dist_num_worker", "2"), ("dist_worker_rank", "1"), ("iter", "end")]
    it2 = create_iterator(cfg2)
    it2.init()
    idx2 = [i for b in _collect(it2) for i in b[2][: 5 - b[3]]]
    assert idx2 == list(range(105, 110))


def test_threadbuffer_over_images(imgset):
    d, _ = imgset
    cfg = _cfg("imgbin", d)
    cfg = cfg[:-1] + [("iter", "threadbuffer"), ("iter", "end")]
    it = create_iterator(cfg)
    it.init()
    assert len(_collect(it)) == 3
    it.close()


def test_train_on_imgbin_cpu(imgset, tmp_path):
    from cxxnet_amd.cli import LearnTask
    d, _ = imgset
    conf = tmp_path / "img.conf"
    conf.write_text(f"""
data = train
iter = imgbin
  image_list = "{d}/all.lst"
  image_bin = "{d}/all.bin"
  rand_crop = 1
  rand_mirror = 1
iter = end
netconfig = start
layer[0->1] = conv
  kernel_size = 3
  nchannel = 8
  stride = 2
layer[1->2] = relu
layer[2->3] = flatten
layer[3->4] = fullc
  nhidden = 4
layer[4->4] = softmax
netconfig = end
input_shape = 3,32,32
batch_size = 4
dev = cpu
num_round = 1
save_model = 0
eta = 0.01
silent = 1
model_dir = {tmp_path}/models
""")
    rc = LearnTask().run([str(conf)])
    assert rc == 0


# ----------------------------------------------------------------------------- native JPEG decode
@pytest.fixture(scope="module")
def jpegset(tmp_path_factory):
    """JPEGs of assorted sizes: 4:4:4, 4:2:0 and grayscale, plus one PNG (fallback path)."""
    d = tmp_path_factory.mktemp("jpgs")
    rng = np.random.default_rng(1)
    lines, raw = [], {}
    for i in range(12):
        h, w = int(rng.integers(40, 90)), int(rng.integers(40, 90))
        yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
        a = np.stack([(yy * (k + 1) * 3 + xx * (5 - k) * 2) % 256 for k in range(3)], -1)
        a = np.clip(a + rng.normal(0, 20, a.shape), 0, 255).astype(np.uint8)
        if i == 11:
            name = f"im{i}.png"
            Image.fromarray(a).save(d / name)
        elif i % 4 == 3:
            name = f"im{i}.jpg"
            Image.fromarray(a[..., 0]).save(d / name, quality=85)  # grayscale JPEG
        else:
            name = f"im{i}.jpg"
            Image.fromarray(a).save(d / name, quality=90, subsampling=(0 if i % 2 else 2))
        raw[200 + i] = (d / name).read_bytes()
        lines.append(f"{200 + i}\t{i % 5}\t{name}\n")
    (d / "all.lst").write_text("".join(lines))
    im2bin.main([str(d / "all.lst"), str(d) + "/", str(d / "all.bin")])
    return d, raw


def test_native_jpeg_crops_match_pillow_decode(jpegset):
    """The native pool's crop (crop-window-only libjpeg-turbo decode) is bit-identical to
    Pillow decoding the whole image and cropping / mirroring it at the reported position."""
    import io as _io
    from cxxnet_amd import native
    rt = native.rt()
    if not rt.JpegDecodePool.available():
        pytest.skip(rt.JpegDecodePool.error())
    d, raw = jpegset
    keys = sorted(raw)
    B = len(keys)
    items = [(i, raw[k], 1000 + 7 * i) for i, k in enumerate(keys)]
    out = np.zeros((B, 32, 32, 3), np.uint8)
    prm = np.zeros((B, 4), np.int32)
    cm = np.zeros((B, 2), np.float32)
    cfg = (32, 32, 3, 1, 1, 0, -1, -1, 0.3, 0.1, 1)
    failed = rt.JpegDecodePool(3).decode(items, cfg, out, prm, cm)
    assert failed == [B - 1]  # the PNG
    seen_mirror = set()
    for i, k in enumerate(keys[:-1]):
        full = np.asarray(Image.open(_io.BytesIO(raw[k])).convert("RGB"))
        y, x, m = (int(v) for v in prm[i, :3])
        assert 0 <= y <= full.shape[0] - 32 and 0 <= x <= full.shape[1] - 32
        ref = full[y:y + 32, x:x + 32]
        if m:
            ref = ref[:, ::-1]
        seen_mirror.add(m)
        assert np.array_equal(out[i], ref), (k, y, x, m)
        assert 0.7 <= cm[i, 0] <= 1.3 and -0.1 <= cm[i, 1] <= 0.1
    assert seen_mirror == {0, 1}
    # thread count does not change anything
    out2, prm2, cm2 = np.zeros_like(out), np.zeros_like(prm), np.zeros_like(cm)
    rt.JpegDecodePool(1).decode(items, cfg, out2, prm2, cm2)
    assert np.array_equal(out[:-1], out2[:-1]) and np.array_equal(prm[:-1], prm2[:-1])
    assert np.array_equal(cm[:-1], cm2[:-1])


@pytest.mark.parametrize("kind", ["imgbin", "img"])
def test_native_decode_iterator_matches_its_crop_params(jpegset, kind):
    """iter = imgbin / img with decode_native = 1: every row is the Pillow decode of its record
    cropped at the batch's own crop parameters (the PNG row goes through the Pillow path),
    and the batches do not depend on the native thread count."""
    import io as _io
    from cxxnet_amd import native
    if not native.rt().JpegDecodePool.available():
        pytest.skip("no libjpeg")
    d, raw = jpegset
    runs = []
    for nt in (1, 4):
        it = create_iterator(_cfg(kind, d, rand_crop=1, rand_mirror=1, seed_data=2, mean_value="1,2,3",
                                  decode_native=1, decode_native_threads=nt, round_batch=1))
        it.init()
        assert it._jpeg is not None and it._jpeg.threads == nt
        batches = []
        while it.next():
            b = it.value()
            batches.append((b.data.pix.clone(), b.data.prm.clone(), b.inst_index.copy(), b.num_batch_padd))
        runs.append(batches)
        it.close()
    assert len(runs[0]) == 3
    for (p0, q0, i0, _), (p1, q1, i1, _) in zip(*runs):
        assert torch.equal(p0, p1) and torch.equal(q0, q1) and (i0 == i1).all()
    for pix, prm, idx, padd in runs[0]:
        for r in range(4):
            full = np.asarray(Image.open(_io.BytesIO(raw[int(idx[r])])).convert("RGB"))
            y, x, m = (int(v) for v in prm[r, :3])
            ref = full[y:y + 32, x:x + 32]
            if m:
                ref = ref[:, ::-1]
            assert np.array_equal(pix[r].numpy(), ref)


def test_native_im2bin_executable_matches_python_tool(imgset, tmp_path):
    """The C++ im2bin executable (csrc/tools/im2bin.cpp, the reference tool's command line)
    writes the same pages, byte for byte, as the Python tool."""
    import subprocess
    from cxxnet_amd import build
    exe = build.build_im2bin()
    d, _ = imgset
    out = tmp_path / "native.bin"
    r = subprocess.run([exe, str(d / "all.lst"), str(d) + "/", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "images processed to 1 pages" in r.stdout
    assert out.read_bytes() == (d / "all.bin").read_bytes()
    bad = subprocess.run([exe, "only-one-arg"], capture_output=True, text=True)
    assert bad.returncode == 255 and "Usage: im2bin" in bad.stderr
