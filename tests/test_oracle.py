"""CPU tests: the oracle (oracle/rc_oracle.c) pinned against the reference's own output.

Pinning: tests/golden/md5.json holds the md5 of the P3 images the reference binary itself
writes (C/ sources built exactly as C/Makefile:4, tests/golden/make_golden.py), and
small.npz the decoded 64x64 images.  When oracle/_ref is present the oracle is also
compared image-for-image with the reference on seeded random scenes.
"""
import json
import os

import numpy as np
import pytest

from helpers import (GOLDEN, PHANTOM_LIT, SCENES, cross_nan_scene_text, golden_key, golden_table,
                     have_ref, oracle_lib, oracle_render, p3_md5, phantom_lit_scene, rc, run_ref,
                     scene_path, random_scene)

SMALL = ["simple", "reflection", "quadric", "example2", "example3", "quadric2"]


@pytest.fixture(scope="module")
def table():
    return golden_table()


@pytest.mark.parametrize("scene", SMALL)
@pytest.mark.parametrize("mode", ["parity", "fast"])
def test_oracle_small_goldens(scene, mode, table):
    """Every 64x64 and 256x256 golden (depth 0/4/6) — SURVEY.md Appendix B/B2."""
    s = rc.Scene.from_file(scene_path(scene))
    small = np.load(os.path.join(GOLDEN, "small.npz"))
    for n in (64, 256):
        for d in (0, 4, 6):
            img, _ = oracle_render(s, n, n, d, mode)
            key = golden_key(scene, n, n, d, mode)
            assert p3_md5(img) == table[key]["md5"], key
            if n == 64:
                np.testing.assert_array_equal(img, small[key])


@pytest.mark.parametrize("key", ["simple:1024x1024:d0:parity", "reflection:2048x2048:d4:parity",
                                 "reflection:2048x2048:d4:fast", "quadric:512x384:d6:parity",
                                 "quadric:333x517:d6:parity", "reflection:1x1:d6:parity",
                                 "quadric:7x3:d6:parity", "quadric:1x4096:d6:parity"])
def test_oracle_configs(key, table):
    """BASELINE configs C2/C3 plus ragged and degenerate image shapes."""
    scene, size, d, mode = key.split(":")
    w, h = map(int, size.split("x"))
    s = rc.Scene.from_file(scene_path(scene))
    img, _ = oracle_render(s, w, h, int(d[1:]), mode)
    assert p3_md5(img) == table[key]["md5"]


@pytest.mark.skipif(not os.environ.get("RC_SLOW"), reason="12 s: set RC_SLOW=1")
def test_oracle_c4(table):
    s = rc.Scene.from_file(scene_path("quadric"))
    img, st = oracle_render(s, 4096, 4096, 6, "parity")
    assert p3_md5(img) == table["quadric:4096x4096:d6:parity"]["md5"]
    assert st["dep_pixels"] == 2804464 and st["longest_segment"] == 844249


def test_oracle_stats_match_survey():
    """Work counts at C1 — these feed the roofline's flop/pixel."""
    s = rc.Scene.from_file(scene_path("simple"))
    _, st = oracle_render(s, 256, 256, 6, "parity")
    n = 256 * 256
    assert abs(st["sphere_tests"] / n - 7.631) < 1e-3
    assert abs(st["plane_tests"] / n - 2.146) < 1e-3
    assert st["dep_pixels"] == 7868
    assert st["parity_defined"] == 1


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (make ref)")
@pytest.mark.parametrize("seed", range(8))
def test_oracle_vs_reference_random_scenes(seed, tmp_path):
    rng = np.random.default_rng(seed)
    path = str(tmp_path / f"r{seed}.scene")
    random_scene(rng, path, int(rng.integers(2, 9)), int(rng.integers(1, 3)))
    s = rc.Scene.from_file(path)
    for mode in ("parity", "fast"):
        for d in (1, 6):
            img, st = oracle_render(s, 48, 40, d, mode)
            if not st["parity_defined"]:
                continue
            np.testing.assert_array_equal(img, run_ref(path, 48, 40, d, mode))


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (make ref)")
@pytest.mark.parametrize("case", ["cross-terms", "overflow-1.2e38", "overflow-1.5e38"])
def test_oracle_vs_reference_quadric_cross_terms(case, tmp_path):
    """Pins the oracle where the kernels' cross-term-free quadric form must agree with the
    reference: quadrics with non-zero d, e, f, and hit points that overflow to inf so that
    the zero cross terms turn NaN (the oracle's diagnostic counter shows that case is hit)."""
    path = tmp_path / f"{case}.scene"
    if case == "cross-terms":
        random_scene(np.random.default_rng(78), str(path), 14, 2, cross=True)
        w, h = 48, 40
    else:
        path.write_text(cross_nan_scene_text(20 if "1.2" in case else 2000, case.split("-")[1]))
        w, h = 64, 48
    s = rc.Scene.from_file(str(path))
    lib = oracle_lib()
    for mode in ("parity", "fast"):
        for d in (1, 6):
            lib.rco_cross_nan_events(1)
            img, st = oracle_render(s, w, h, d, mode)
            if case != "cross-terms" and d == 6:
                assert lib.rco_cross_nan_events(1) > 0
            if st["parity_defined"]:
                np.testing.assert_array_equal(img, run_ref(str(path), w, h, d, mode),
                                              err_msg=f"{case} {mode} d{d}")


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (make ref)")
@pytest.mark.parametrize("n_shapes", [20, 33, 64, 65, 90])
def test_oracle_vs_reference_many_shapes(n_shapes, tmp_path):
    """Scenes larger than the examples (the GPU evaluator groups 32 / 64 lanes per entry
    and stops staging shapes in LDS above 64): the oracle still equals the reference."""
    rng = np.random.default_rng(1000 + n_shapes)
    path = str(tmp_path / f"m{n_shapes}.scene")
    random_scene(rng, path, n_shapes, 2)
    s = rc.Scene.from_file(path)
    for mode in ("parity", "fast"):
        img, st = oracle_render(s, 40, 32, 6, mode)
        if st["parity_defined"]:
            np.testing.assert_array_equal(img, run_ref(path, 40, 32, 6, mode))


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (make ref)")
@pytest.mark.parametrize("kind", sorted(PHANTOM_LIT))
def test_phantom_model_lit(kind, tmp_path):
    """A lit phantom (opacity > 0) makes the image depend on the light-VLA bytes the
    reference reads as shapes_list[-1]: four lights (bytes [184, 288)) and two lights with
    L1.pos.y + L1.pos.z < 1 (bytes [40, 144)).  Oracle == the reference binary."""
    path = phantom_lit_scene(str(tmp_path / f"{kind}.scene"), kind)
    s = rc.Scene.from_file(path)
    for d in (1, 4, 6):
        img, st = oracle_render(s, 96, 96, d, "parity")
        assert st["parity_defined"] == 1 and st["phantom_shades"] > 0, (kind, d)
        np.testing.assert_array_equal(img, run_ref(path, 96, 96, d, "parity"), err_msg=f"{kind} d{d}")


def test_phantom_goldens():
    """The oracle reproduces the reference's lit-phantom images (tests/golden/phantom_md5.json,
    made by tests/golden/make_phantom_golden.py from the reference build)."""
    table = json.load(open(os.path.join(GOLDEN, "phantom_md5.json")))
    scenes = {}
    for key, want in sorted(table.items()):
        name, size, d, mode = key.split(":")
        w, h = map(int, size.split("x"))
        if name not in scenes:
            scenes[name] = rc.Scene.from_file(os.path.join(SCENES, name + ".scene"))
        img, st = oracle_render(scenes[name], w, h, int(d[1:]), mode)
        assert st["phantom_shades"] > 0, key
        assert p3_md5(img) == want["md5"], key


@pytest.mark.parametrize("scene", ["simple", "reflection", "quadric", "example2", "example3",
                                   "quadric2"])
def test_cuda_semantics_restatement(scene):
    """oracle/rc_oracle_cuda.c (CUDA/raycast.cu's semantics) shares fast
    mode's control flow (miss ends the loop) and differs only in powf-on-float arithmetic, so
    its images sit within one quantisation level of the fast-mode oracle (the reference's
    break-on-miss variant, pinned by goldens) on a handful of pixels.  Parity with the CUDA
    binary itself is unpinned: no nvcc here."""
    from helpers import oracle_render_cuda
    s = rc.Scene.from_file(scene_path(scene))
    for d in (0, 6, 50):
        fast, _ = oracle_render(s, 128, 128, d, "fast")
        cu = oracle_render_cuda(s, 128, 128, d)
        diff = np.abs(fast.astype(np.int16) - cu.astype(np.int16)).max(axis=2)
        assert diff.max() <= 1 and (diff > 0).mean() < 1e-3, (scene, d, diff.max())
        np.testing.assert_array_equal(cu, oracle_render_cuda(s, 128, 128, d))
