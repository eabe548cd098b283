"""The shipped gfx950 tile table names only tiles the kernels know (host-side check; the GPU
suite, tests/test_tune_table_gpu.py, checks every entry's numerics on the device)."""
import json

from cxxnet_amd.ops import gemm as G


def _table():
    with open(G.TUNE_DB) as f:
        return json.load(f)


def test_every_entry_names_a_known_tile():
    bad = []
    for key, tile in _table().items():
        op = key.split("|")[0]
        if op == "cws":  # register weight-grad: tile * 100000 + K-split slices
            ok = tile // 100000 in G.TILES and tile % 100000 >= 1
        elif op in ("cf", "cd"):  # also the direct small-map kernel's schedules (conv_direct.hip)
            ok = tile in G.GLDS_TILES or tile == G.REG or tile in G.DIRECT_TILES
        elif op in ("cw", "cfs"):
            ok = tile in G.GLDS_TILES or tile == G.REG
        else:  # cr, cwr, fc, fw, fws: LDS-DMA tiles only
            ok = tile in G.GLDS_TILES
        if not ok:
            bad.append((key, tile))
    assert not bad, bad[:10]


def test_tuning_candidates_are_known_tiles():
    assert set(G.GLDS_CANDS) <= set(G.GLDS_TILES)
    for t in (82, 114, 130, 131, 133):  # wave-quantisation (r3), one-wave-per-SIMD, halo (r4)
        assert t in G.GLDS_CANDS


def _compiled_tiles():
    """Tile ids the kernels' dispatch code accepts, read from the HIP sources."""
    import os
    import re
    kdir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(G.__file__))), "csrc", "kernels")
    src = lambda f: open(os.path.join(kdir, f)).read()
    tiles = set()
    glds = src("gemm_glds.hip")
    body = glds[glds.index("#define CXG_KK_TILES"):glds.index("#define CXG_CASE")]
    tiles |= {int(m) for m in re.findall(r"CXG_T[PC]?\((\d+),", body)}
    tiles |= {int(m) for m in re.findall(r"case (\d+): launch_4f", src("gemm_4w.hip"))}
    halo = src("conv_halo.hip")
    tiles |= {int(m) for m in re.findall(r"tile == (\d+)", halo[halo.index("int dispatch_halo"):])}
    wg = src("conv_wgrad_halo.hip")
    tiles |= {int(m) for m in re.findall(r"tile [!=]= (\d+)", wg[wg.index("int dispatch_wgrad_halo"):])}
    return tiles


def test_tile_dict_matches_compiled_kernels():
    """Every tile the Python side can name is compiled, and no compiled tile is orphaned."""
    compiled = _compiled_tiles()
    assert set(G.GLDS_TILES) == compiled, (sorted(set(G.GLDS_TILES) - compiled), sorted(compiled - set(G.GLDS_TILES)))


def test_every_compiled_tile_is_used():
    """A compiled tile is in the shipped table, a default pick, or the fc weight-grad set."""
    used = {t for k, t in _table().items() if k.split("|")[0] != "cws"}
    used |= {1, 7, 10, 15}  # _pick_glds defaults
    used |= {141, 142}  # forced patch widths of the 140 kernel (same template instances)
    used |= {82}  # 256x192 wave-quantisation tile: a step_tune candidate (AlexNet conv3 data-grad moved to the direct kernel)
    unused = sorted(_compiled_tiles() - used)
    assert not unused, unused


def test_signature_keys_are_well_formed():
    width = {"cf": 11, "cfs": 6, "cd": 11, "cw": 11, "cws": 11, "cr": 8, "cwr": 8, "fc": 5, "fw": 3, "fws": 3}
    for key in _table():
        parts = key.split("|")
        assert parts[0] in width, key
        assert len(parts) - 1 == width[parts[0]], key
        assert all(p.lstrip("-").isdigit() for p in parts[1:]), key
