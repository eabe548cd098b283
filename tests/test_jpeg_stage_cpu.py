"""GPU JPEG decode stage, host half + numpy reference (io/jpeg_stage.py): the staged
coefficients finished by the reference arithmetic must equal libjpeg-turbo's own decode of the
same crops (the native pixel decoder, runtime/jpeg_decode.h DecodeCrop) bit for bit, over
4:2:0 / 4:2:2 / 4:4:4 / grayscale / progressive files, odd sizes, random crops and mirrors."""
import io

import numpy as np
import pytest
import torch

from cxxnet_amd import native
from cxxnet_amd.io import jpeg_stage


def _jpeg(arr, **kw):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(arr).save(b, format="JPEG", **kw)
    return b.getvalue()


def _photo(rng, h, w, gray=False):
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.stack([128 + 90 * np.sin(xx / (7 + 5 * k) + yy / (11 + 3 * k) + k) for k in range(3)], -1)
    img += rng.normal(0, 20, img.shape)
    img = np.clip(img, 0, 255).astype(np.uint8)
    return img[..., 0] if gray else img


@pytest.fixture(scope="module")
def records():
    if not native.rt().JpegDecodePool.available():
        pytest.skip("no libjpeg")
    rng = np.random.default_rng(3)
    recs = []
    for (h, w), kw, gray in [((256, 256), dict(quality=90, subsampling=2), False),
                             ((250, 301), dict(quality=75, subsampling=2), False),
                             ((241, 263), dict(quality=95, subsampling=1), False),
                             ((256, 240), dict(quality=90, subsampling=0), False),
                             ((233, 257), dict(quality=85), True),
                             ((260, 250), dict(quality=90, subsampling=2, progressive=True), False),
                             ((231, 229), dict(quality=100, subsampling=2), False),
                             ((300, 320), dict(quality=50, subsampling=1, progressive=True), False)]:
        recs.append(_jpeg(_photo(rng, h, w, gray), **kw))
    return recs


def _cfg(h, w, C=3, rand_crop=1, mirror=1, mean_mode=1):
    return (h, w, C, rand_crop, mirror, 0, -1, -1, 0.2, 0.1, mean_mode)


@pytest.mark.parametrize("hw", [(227, 227), (200, 180)])
@pytest.mark.parametrize("C", [3, 1])
def test_stage_reference_matches_libjpeg(records, hw, C):
    rt = native.rt()
    pool = rt.JpegDecodePool(4)
    h, w = hw
    cfg = _cfg(h, w, C)
    B = len(records) * 3
    items = [(r, records[r % len(records)], 1000 + 7 * r) for r in range(B)]
    ref = np.zeros((B, h, w, C), np.uint8)
    prm_ref, cm_ref = np.zeros((B, 4), np.int32), np.zeros((B, 2), np.float32)
    assert pool.decode(items, cfg, ref, prm_ref, cm_ref) == []
    coef, bwin, meta, nblk, prm, cm, failed = jpeg_stage.stage_batch(pool, items, cfg, B, h, w, C, False)
    assert failed == [] and 0 < nblk <= coef.shape[0]
    assert np.array_equal(prm.numpy(), prm_ref) and np.array_equal(cm.numpy(), cm_ref)
    assert set(prm_ref[:, 2]) == {0, 1}  # both mirror states exercised
    out = jpeg_stage.decode_reference(coef[:nblk].numpy(), bwin[:nblk].numpy(), meta.numpy(), prm.numpy(), 0, B,
                                      h, w, C)
    for r in range(B):
        assert np.array_equal(out[r], ref[r]), (r, np.abs(out[r].astype(int) - ref[r]).max())


def test_stage_windows_and_fallbacks(records):
    """Only the crop window's blocks are staged; PNG / CMYK records come back as failed rows and
    are decoded to pixels by the host path; a batch does not depend on the thread count."""
    from PIL import Image
    rt = native.rt()
    rng = np.random.default_rng(0)
    png = io.BytesIO()
    Image.fromarray(_photo(rng, 240, 240)).save(png, format="PNG")
    cmyk = io.BytesIO()
    Image.fromarray(_photo(rng, 240, 240)).convert("CMYK").save(cmyk, format="JPEG")
    big = _jpeg(_photo(rng, 640, 512), quality=90, subsampling=2)
    recs = [records[0], png.getvalue(), cmyk.getvalue(), big]
    h = w = 227
    cfg = _cfg(h, w)
    items = [(r, recs[r], 5 + r) for r in range(4)]
    runs = []
    for nt in (1, 3):
        runs.append(jpeg_stage.stage_batch(rt.JpegDecodePool(nt), items, cfg, 5, h, w, 3, False))
    coef, bwin, meta, nblk, prm, cm, failed = runs[0]
    assert sorted(failed) == [1, 2]
    m = meta.numpy()
    assert (m[[1, 2, 4], :, jpeg_stage.VALID] == 0).all() and (m[[0, 3], :, jpeg_stage.VALID] == 1).all()
    # a 640x512 photo stages no more than a 256px one: a 227 crop's window
    per_row = [int((m[r, :, jpeg_stage.BW] * m[r, :, jpeg_stage.BH]).sum()) for r in (0, 3)]
    assert per_row[1] <= 30 * 30 + 2 * 16 * 16 and nblk == sum(per_row)
    outs = [jpeg_stage.decode_reference(c[:n].numpy(), bw[:n].numpy(), mt.numpy(), p.numpy(), 0, 5, h, w, 3)
            for c, bw, mt, n, p, _, _ in runs]
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(runs[0][4], runs[1][4])
    assert not outs[0][[1, 2, 4]].any()
    seen = []

    def pillow_one(payload, seed):  # PNG and CMYK are the Pillow path's (io/augment.py)
        seen.append(seed)
        return np.full((h, w, 3), 7, np.uint8), (1, 2, 0), (1.0, 0.0)
    fb = jpeg_stage.fallback_rows(rt.JpegDecodePool(2), items, failed, cfg, (5, h, w, 3), prm, cm, False, pillow_one)
    assert sorted(seen) == [6, 7] and (fb[1] == 7).all() and (fb[2] == 7).all() and not fb[[0, 3, 4]].any()


def test_iterator_decode_gpu_matches_pixel_path(tmp_path, records):
    """iter = img with decode_gpu = 1 on the CPU: the batch is a JpegCoefImages whose reference
    decode equals the pixel path's batch (same draws, same pixels), row slices included."""
    from cxxnet_amd.io.iterators import create_iterator
    from cxxnet_amd.io.jpeg_stage import JpegCoefImages
    lst = []
    for i, r in enumerate(records):
        p = tmp_path / f"{i}.jpg"
        p.write_bytes(r)
        lst.append(f"{i}\t{i % 3}\t{p.name}\n")
    (tmp_path / "a.lst").write_text("".join(lst))
    outs = []
    for g in (0, 1):
        cfg = [("iter", "img"), ("image_list", str(tmp_path / "a.lst")), ("image_root", str(tmp_path) + "/"),
               ("rand_crop", "1"), ("rand_mirror", "1"), ("mean_value", "104,117,123"), ("input_shape", "3,227,227"),
               ("batch_size", "4"), ("round_batch", "1"), ("silent", "1"), ("decode_native", "1"),
               ("decode_native_threads", "2"), ("decode_gpu", str(g)), ("iter", "end")]
        it = create_iterator(cfg)
        it.init()
        it.before_first()
        bs = []
        while it.next():
            bs.append(it.value().data)
        it.close()
        outs.append(bs)
    assert len(outs[0]) == 2
    for a, b in zip(*outs):
        assert isinstance(b, JpegCoefImages) and tuple(b.shape) == tuple(a.shape)
        assert torch.equal(b.to_u8().pix, a.pix) and torch.equal(b.prm, a.prm)
        assert torch.equal(b.to_float(), a.to_float())
        assert torch.equal(b[1:3].to_u8().pix, a.pix[1:3])
