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
        elif op in ("cf", "cd", "cw"):
            ok = tile in G.GLDS_TILES or tile == G.REG
        else:  # cr, cwr, fc, fw, fws: LDS-DMA tiles only
            ok = tile in G.GLDS_TILES
        if not ok:
            bad.append((key, tile))
    assert not bad, bad[:10]


def test_tuning_candidates_are_known_tiles():
    assert set(G.GLDS_CANDS) <= set(G.GLDS_TILES)
    for t in (82, 83, 110, 114, 115, 130, 131):  # wave-quantisation (r3), one-wave-per-SIMD, halo (r4)
        assert t in G.GLDS_CANDS


def test_signature_keys_are_well_formed():
    width = {"cf": 11, "cd": 11, "cw": 11, "cws": 11, "cr": 8, "cwr": 8, "fc": 5, "fw": 3, "fws": 3}
    for key in _table():
        parts = key.split("|")
        assert parts[0] in width, key
        assert len(parts) - 1 == width[parts[0]], key
        assert all(p.lstrip("-").isdigit() for p in parts[1:]), key
