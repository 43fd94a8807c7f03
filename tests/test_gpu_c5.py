"""GPU parity on BASELINE configs[4] (C5) itself, and on depth-8 trees under the persistent
bounce kernel.

C5 = 7680x4320, 1M spheres (seeded generateRandomSpheres restatement), octree depth 10,
maxSpheresPerNode 1, reflection bounce depth 4 (glsl:597-633) over the
depth-10 walk (glsl:290-481).  The tree is built on the GPU (the reference builder's output
byte for byte, tests/test_gpu_build.py) and exported whole to the host, where the oracle
walks the same arrays; a 239 M-node host build would take ~21 s.  The frame is checked on
64 rows spread over its height (four 16-row bands) and on a ragged sub-tile, with the frame's
own resolution, camera and bounce depth.  Bar: bit-exact.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

C5 = dict(width=7680, height=4320, spheres=1_000_000, depth=10, mspn=1, bounces=4)
MANIFEST = json.loads((Path(__file__).resolve().parent / "golden" / "manifest.json").read_text())


def _sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.fixture(scope="module")
def c5(ort):
    s = ort.random_spheres(C5["spheres"], 42)
    r = ort.Renderer(0)
    r.build_scene(s, C5["depth"], C5["mspn"], keep_tree=True)
    info = r.info()
    t = r.export_octree()
    # the GPU-built tree IS the reference builder's (src/octree.cpp run on the same 1M spheres:
    # tools/hash_ref_tree.py): checked before the oracle walks it, so a builder error cannot
    # hide behind an oracle walking the same wrong tree
    ref = MANIFEST["trees"]["rand1M_d10_m1"]
    assert _sha(s.center_radius, s.mat_albedo, s.fuzz_ri) == ref["spheres"]["sha256"], "C5 sphere set"
    assert (t.n_nodes, t.n_indices) == (ref["nodes"], ref["indices"])
    assert _sha(t.gpu_records(), t.object_indices) == ref["sha256"], "C5 GPU tree differs from the reference builder's"
    yield s, t, r, info
    r.close()


def _tiles():
    H = C5["height"]
    return [
        # 4 bands of 16 rows, one in each quarter of the frame (sky, horizon, sphere field)
        ("bands", (0, C5["width"], 8, 64, 16, H // 4)),
        # ragged sub-tile: odd origin and size, crossing 16x16 workgroup tiles
        ("ragged", (1237, 613, 2011, 37, 0, 0)),
    ]


def test_c5_tree_is_the_reference_tree(c5):
    """The fixture asserted the exported tree's SHA-256 against the reference builder's
    (manifest rand1M_d10_m1); here the counts and layout."""
    _, t, _, info = c5
    # the reference builder's counts for 1M spheres, depth 10, M=1
    assert info["n_nodes"] == 239_220_401 and info["n_indices"] == 172_356_841
    assert info["tree_depth"] == 10 and info["layout"] == "compact"
    assert t.n_nodes == info["n_nodes"] and t.n_indices == info["n_indices"]


@pytest.mark.parametrize("name,tile", _tiles())
def test_c5_bounce_depth_4_bit_exact(ort, oracle, c5, name, tile):
    """The C5 workload (1 spp, 4 bounces: camera-ray deep kernel, path compaction and
    coherence sort of the list, persistent refill kernel with the rejected-sphere skip for
    bounces >= 1) against the oracle on the same tree."""
    s, t, r, _ = c5
    p = ort.FrameParams.default_camera(C5["width"], C5["height"], num_samples=1, max_depth=C5["bounces"])
    tl = ort.Tile(*tile)
    got = r.render(p, tl)
    ref = oracle.render(s, t, p, tl.x0, tl.y0, tl.width, tl.rows, band_height=tl.band_height,
                        band_stride=tl.band_stride, threads=0)
    assert_same(got, ref, f"C5 {name}")
    assert float(got.max()) > 0.0  # not a blank tile


def test_c5_primary_and_counters(ort, oracle, c5):
    """Primary rays over the C5 tree, and the reference-layout work counters the bench's
    traffic model uses, against the oracle's counts of the same rows."""
    s, t, r, _ = c5
    W, H = C5["width"], C5["height"]
    tl = ort.Tile(0, W, 8, 64, 16, H // 4)
    p1 = ort.FrameParams.default_camera(W, H)
    ref1, want1 = oracle.render(s, t, p1, 0, 8, W, 64, band_height=16, band_stride=H // 4, counts=True)
    assert_same(r.render(p1, tl), ref1, "C5 primary")
    assert r.count_traffic(p1, tl) == want1
    p4 = ort.FrameParams.default_camera(W, H, max_depth=C5["bounces"])
    _, want4 = oracle.render(s, t, p4, 0, 8, W, 64, band_height=16, band_stride=H // 4, counts=True)
    got4 = r.count_traffic(p4, tl)
    assert got4 == want4
    assert got4["traversals"] > got4["pixels"]  # secondary rays were traced


@pytest.fixture(scope="module")
def scenes_d8(ort):
    s = ort.random_spheres(10_000, 3)
    return {m: (s, ort.build_octree(s, 8, m)) for m in (0, 1)}


@pytest.mark.parametrize("mspn", [0, 1])
@pytest.mark.parametrize("persistent", [2, 0])
def test_depth8_bounces_persistent(ort, oracle, renderer, scenes_d8, mspn, persistent):
    """Depth-8 trees with bounces: the persistent bounce kernel's 64-bit-mask walk
    (Masks64Plain) pushes leaf children into the level-7 byte and pops at L=7 -- a case the
    primary kernel (inline leaf children) never reaches.  Against the oracle with the
    persistent kernel on (default 2) and off."""
    s, t = scenes_d8[mspn]
    renderer.upload(s, t)
    assert renderer.info()["tree_depth"] == 8
    renderer.set_persistent(persistent)
    try:
        p = ort.FrameParams.default_camera(1280, 720, num_samples=2, max_depth=5)
        for tile in (ort.Tile(0, 1280, 3, 64, 16, 180), ort.Tile(411, 203, 250, 71)):
            got = renderer.render(p, tile)
            ref = oracle.render(s, t, p, tile.x0, tile.y0, tile.width, tile.rows, band_height=tile.band_height,
                                band_stride=tile.band_stride)
            assert_same(got, ref, f"d8 M={mspn} persistent={persistent} {tile}")
    finally:
        renderer.set_persistent(2)
