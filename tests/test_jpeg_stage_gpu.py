"""GPU JPEG decode stage (csrc/kernels/jpeg_kernels.hip via ops.jpeg_decode): the HIP IDCT +
upsampling + colour + crop kernels against libjpeg-turbo's own decode of the same crops (the
native pixel decoder) -- bit for bit -- and the iterator's decode_gpu batches against the
pixel path's through the image kernel into the network input."""
import numpy as np
import pytest
import torch

from cxxnet_amd import native, ops
from cxxnet_amd.io import jpeg_stage

from test_jpeg_stage_cpu import _cfg, _jpeg, _photo, records  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("hw,C", [((227, 227), 3), ((200, 180), 3), ((227, 227), 1)])
def test_gpu_stage_matches_libjpeg(records, hw, C):  # noqa: F811
    pool = native.rt().JpegDecodePool(8)
    h, w = hw
    cfg = _cfg(h, w, C)
    B = len(records) * 4
    items = [(r, records[r % len(records)], 31 + 3 * r) for r in range(B) if r != 5]  # row 5: padding
    ref = np.zeros((B, h, w, C), np.uint8)
    assert pool.decode(items, cfg, ref, np.zeros((B, 4), np.int32), np.zeros((B, 2), np.float32)) == []
    coef, bwin, meta, nblk, prm, cm, failed = jpeg_stage.stage_batch(pool, items, cfg, B, h, w, C, True)
    assert failed == []
    out = ops.jpeg_decode(coef, bwin, meta, nblk, prm, 0, B, h, w, C, torch.device("cuda"))
    got = out.cpu().numpy()
    for r in range(B):
        assert np.array_equal(got[r], ref[r]), (r, np.abs(got[r].astype(int) - ref[r]).max())
    # a row range decodes the same rows
    part = ops.jpeg_decode(coef, bwin, meta, nblk, prm, 3, 11, h, w, C, torch.device("cuda"))
    assert torch.equal(part.cpu(), out[3:11].cpu())


def test_gpu_stage_fallback_rows_and_iterator(tmp_path, records):  # noqa: F811
    """decode_gpu = 1 vs 0 through the trainer's input stage: the same bf16 NHWC input, with a
    PNG record (host fallback row) in the batch."""
    import io
    from PIL import Image
    from cxxnet_amd.io.iterators import create_iterator
    from cxxnet_amd.io.jpeg_stage import JpegCoefImages
    png = io.BytesIO()
    Image.fromarray(_photo(np.random.default_rng(1), 240, 250)).save(png, format="PNG")
    recs = list(records) + [png.getvalue()]
    lst = []
    for i, r in enumerate(recs):
        p = tmp_path / f"{i}.img"
        p.write_bytes(r)
        lst.append(f"{i}\t{i % 3}\t{p.name}\n")
    (tmp_path / "a.lst").write_text("".join(lst))
    outs = []
    for g in (0, 1):
        cfg = [("iter", "img"), ("image_list", str(tmp_path / "a.lst")), ("image_root", str(tmp_path) + "/"),
               ("rand_crop", "1"), ("rand_mirror", "1"), ("mean_value", "104,117,123"), ("input_shape", "3,227,227"),
               ("batch_size", "9"), ("round_batch", "1"), ("silent", "1"), ("decode_native", "1"),
               ("decode_gpu", str(g)), ("iter", "end")]
        it = create_iterator(cfg)
        it.init()
        it.before_first()
        assert it.next()
        d = it.value().data
        it.close()
        assert isinstance(d, JpegCoefImages) == (g == 1)
        node = torch.zeros((9, 227, 228, 3), dtype=torch.bfloat16, device="cuda")
        ops.image_to_nhwc(d, node)
        outs.append(node.float().cpu())
        if g:
            assert d.fb_rows == [8]
            assert torch.equal(d[2:9].to_u8("cuda").pix.cpu(), d.to_u8("cuda").pix.cpu()[2:9])
    assert torch.equal(outs[0], outs[1])


def test_gpu_stage_rate(records):  # noqa: F811
    """Kernel time of a 256-image AlexNet batch (informational; printed)."""
    pool = native.rt().JpegDecodePool(8)
    h = w = 227
    cfg = _cfg(h, w)
    B = 256
    items = [(r, records[r % 2], r) for r in range(B)]  # the two 4:2:0 records
    coef, bwin, meta, nblk, prm, cm, failed = jpeg_stage.stage_batch(pool, items, cfg, B, h, w, 3, True)
    dev = torch.device("cuda")
    for _ in range(3):
        ops.jpeg_decode(coef, bwin, meta, nblk, prm, 0, B, h, w, 3, dev)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        ops.jpeg_decode(coef, bwin, meta, nblk, prm, 0, B, h, w, 3, dev)
    e.record()
    e.synchronize()
    print(f"jpeg stage: {nblk} blocks, {nblk * 128 / 2 ** 20:.1f} MiB staged, "
          f"{s.elapsed_time(e) / 10 * 1e3:.0f} us per 256-image batch (incl. H2D)")
