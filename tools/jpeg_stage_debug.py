"""Split check of the GPU JPEG stage: IDCT planes vs io.jpeg_stage.idct_reference, and the colour
kernel fed the reference planes vs decode_reference (run on a GPU box)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from cxxnet_amd import native  # noqa: E402
from cxxnet_amd.io import jpeg_stage  # noqa: E402
from cxxnet_amd.ops.nn import _k, _stream  # noqa: E402
from test_jpeg_stage_cpu import _cfg, _jpeg, _photo  # noqa: E402

rng = np.random.default_rng(3)
recs = [_jpeg(_photo(rng, 256, 256), quality=90, subsampling=2), _jpeg(_photo(rng, 250, 301), quality=75)]
pool = native.rt().JpegDecodePool(4)
h = w = 227
B = 4
items = [(r, recs[r % 2], 31 + r) for r in range(B)]
coef, bwin, meta, nblk, prm, cm, failed = jpeg_stage.stage_batch(pool, items, _cfg(h, w), B, h, w, 3, True)
print("nblk", nblk, "failed", failed, "prm", prm.tolist())
q = meta.view(-1, 80)[bwin[:nblk].long(), 16:80].numpy()
ref_planes = jpeg_stage.idct_reference(coef[:nblk].numpy(), q)
dev = torch.device("cuda")
coef_d, bwin_d, meta_d = coef[:nblk].to(dev), bwin[:nblk].to(dev), meta.to(dev)
print("coef sum host", int(coef[:nblk].abs().sum()), "dev", int(coef_d.abs().sum()))
plane = torch.full((nblk, 64), 77, dtype=torch.uint8, device=dev)
rc = _k().cxn_jpeg_idct(coef_d.data_ptr(), bwin_d.data_ptr(), meta_d.data_ptr(), nblk, plane.data_ptr(), _stream())
torch.cuda.synchronize()
p = plane.cpu().numpy()
print("idct rc", rc, "equal", np.array_equal(p, ref_planes), "mismatch blocks", int((p != ref_planes).any(1).sum()))
print("gpu plane[0]", p[0][:16], "ref", ref_planes[0][:16])
out = torch.zeros((B, h, w, 3), dtype=torch.uint8, device=dev)
rp = torch.from_numpy(ref_planes).to(dev)
prm_d = prm.to(dev)
rc = _k().cxn_jpeg_color(rp.data_ptr(), meta_d.data_ptr(), prm_d.data_ptr(), B, h, w, 3, out.data_ptr(), _stream())
torch.cuda.synchronize()
ref = jpeg_stage.decode_reference(coef[:nblk].numpy(), bwin[:nblk].numpy(), meta.numpy(), prm.numpy(), 0, B, h, w, 3)
print("color rc", rc, "equal", np.array_equal(out.cpu().numpy(), ref))

# the op itself, on the same stage and on the test's larger batch
from cxxnet_amd import ops  # noqa: E402
got = ops.jpeg_decode(coef, bwin, meta, nblk, prm, 0, B, h, w, 3, dev).cpu().numpy()
print("op equal", np.array_equal(got, ref))
B2 = 32
items2 = [(r, recs[r % 2], 31 + 3 * r) for r in range(B2) if r != 5]
st = jpeg_stage.stage_batch(native.rt().JpegDecodePool(8), items2, _cfg(h, w), B2, h, w, 3, True)
coef2, bwin2, meta2, nblk2, prm2 = st[:5]
ref2 = jpeg_stage.decode_reference(coef2[:nblk2].numpy(), bwin2[:nblk2].numpy(), meta2.numpy(), prm2.numpy(), 0, B2,
                                   h, w, 3)
got2 = ops.jpeg_decode(coef2, bwin2, meta2, nblk2, prm2, 0, B2, h, w, 3, dev).cpu().numpy()
print("op B32 equal", np.array_equal(got2, ref2), "rows bad", [r for r in range(B2) if not np.array_equal(got2[r], ref2[r])])


def variant(nb, full_plane):
    cd = coef[:nblk].to(dev, non_blocking=nb)
    bd = bwin[:nblk].to(dev, non_blocking=nb)
    md = meta.to(dev, non_blocking=nb)
    pd = prm.to(dev, torch.int32, non_blocking=nb).contiguous()
    pl = (torch.full if full_plane else lambda s, v, **k: torch.empty(s, **k))((nblk, 64), 5, dtype=torch.uint8,
                                                                              device=dev)
    o = torch.empty((B, h, w, 3), dtype=torch.uint8, device=dev)
    r1 = _k().cxn_jpeg_idct(cd.data_ptr(), bd.data_ptr(), md.data_ptr(), nblk, pl.data_ptr(), _stream())
    r2 = _k().cxn_jpeg_color(pl.data_ptr(), md.data_ptr(), pd.data_ptr(), B, h, w, 3, o.data_ptr(), _stream())
    torch.cuda.synchronize()
    pp = pl.cpu().numpy()
    print("variant nb", nb, "full", full_plane, r1, r2, "plane eq", np.array_equal(pp, ref_planes),
          "plane uniq", np.unique(pp)[:5], "out eq", np.array_equal(o.cpu().numpy(), ref))


for nb in (False, True):
    for fp in (False, True):
        variant(nb, fp)
print("coef dtype", coef.dtype, coef.is_pinned(), coef[:nblk].is_contiguous(), coef.data_ptr() % 16)
