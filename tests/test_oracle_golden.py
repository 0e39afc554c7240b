"""Pin the oracle: the CPU restatement (oracle/oracle.c) against fixtures produced by the reference's
own sources (tests/golden/, made by tests/golden/make_golden.py from oracle/_ref/ref_render).

The oracle consumes the scene this library builds (host scene builders + flattener), so these tests
pin the whole CPU chain; the GPU tests then compare the HIP path against both.
"""
import hashlib
import os

import numpy as np
import pytest

import pyoracle
import rtc
from conftest import GOLDEN, golden_image

FULL = ["s0_400x225_10spp_d10", "s0_400x225_100spp_d50", "s1_300x168_16spp_d50", "s2_200x112_8spp_d50",
        "s3_200x112_8spp_d50", "s4_200x112_8spp_d50", "s5_200x112_16spp_d50", "s6_200x200_16spp_d50",
        "s7_200x200_8spp_d50"]


@pytest.mark.parametrize("name", FULL)
def test_oracle_matches_reference_render(manifest, name):
    e = manifest["renders"][name]
    sc = rtc.Scene.preset(e["scene"], e["width"], e["spp"], e["depth"])
    assert (sc.width, sc.height) == (e["width"], e["height"])
    img = pyoracle.render(sc)
    ref = golden_image(e)
    bad = (img != ref).any(axis=2)
    assert not bad.any(), f"{bad.sum()} pixels differ, first at {np.argwhere(bad)[0]}"
    assert hashlib.sha256(img.tobytes()).hexdigest() == e["sha256"]


def test_oracle_book1_full_width_10spp(manifest):
    """Book-1 final scene at the north-star resolution (10 spp keeps it to seconds on 8 cores)."""
    e = manifest["renders"]["s1_1200x675_10spp_d50"]
    sc = rtc.Scene.preset(1, 1200, 10, 50)
    img = pyoracle.render(sc)
    assert hashlib.sha256(img.tobytes()).hexdigest() == e["sha256"]


def test_oracle_row_subsets_are_rows_of_full_frame(manifest):
    """Interleaved row partition (the multi-GPU split) reproduces the frame's rows."""
    e = manifest["renders"]["s1_300x168_16spp_d50"]
    ref = golden_image(e)
    sc = rtc.Scene.preset(1, 300, 16, 50)
    for world in (2, 3, 8):
        for rank in range(world):
            row0, stride, n = rtc.rows_of(sc.height, rank, world)
            part = pyoracle.render(sc, row0, stride, n)
            assert np.array_equal(part, ref[row0::stride][:n])


def test_oracle_pixel_list_matches(manifest):
    e = manifest["renders"]["s0_400x225_100spp_d50"]
    ref = golden_image(e)
    sc = rtc.Scene.preset(0, 400, 100, 50)
    rng = np.random.default_rng(7)
    xs = rng.integers(0, 400, 64)
    ys = rng.integers(0, 225, 64)
    px = pyoracle.render_pixels(sc, xs, ys)
    assert np.array_equal(px, ref[ys, xs])


def test_oracle_depth_zero_is_black():
    """depth <= 0 returns black without touching the rng (src/raytracing.c:40-41)."""
    sc = rtc.Scene.preset(1, 64, 3, 0)
    sc.s.camera.max_depth = 0
    img = pyoracle.render(sc)
    assert img.max() == 0
