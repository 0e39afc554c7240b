"""The gfx950 kernel's per-pixel code (csrc/rt_device.h), compiled for the HOST with
AddressSanitizer (tests/native/kernel_host_check), against the oracle on every reference scene.

This runs without a GPU and before any GPU launch: an out-of-bounds index in the device code
aborts under ASan here instead of faulting an MI355X, and traversal-order / path-fold logic errors
show up as pixel differences.  (Device-compiler effects are covered by the -m gpu tests.)
"""
import os
import subprocess

import numpy as np
import pytest

import pyoracle
import rtc
from conftest import ROOT

EXE = os.path.join(ROOT, "tests", "native", "bin", "kernel_host_check")


@pytest.mark.parametrize("scene,width,spp,depth,variant", [
    (0, 96, 4, 50, "book1"), (1, 96, 4, 50, "book1"), (1, 64, 3, 50, "all"), (2, 96, 3, 50, "all"),
    (3, 80, 3, 50, "all"), (4, 96, 3, 50, "all"), (5, 96, 6, 50, "all"), (6, 64, 4, 50, "all"),
    (7, 80, 3, 50, "all"), (1, 33, 2, 1, "book1"), (7, 40, 2, 2, "all"),
    (1, 64, 3, 50, "pre"), (2, 96, 3, 50, "pre"), (3, 80, 3, 50, "pre"), (4, 96, 3, 50, "pre"),
    (5, 96, 6, 50, "pre"), (6, 64, 4, 50, "pre"), (7, 80, 3, 50, "pre"), (7, 40, 2, 2, "pre")])
def test_kernel_code_on_host_matches_oracle(tmp_path, scene, width, spp, depth, variant):
    """variant: book1 / all (stack trace) / pre (preorder trace_pre)"""
    out = str(tmp_path / "k.rgb")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", OMP_NUM_THREADS="8")
    r = subprocess.run([EXE, str(scene), str(width), str(spp), str(depth), out, variant], capture_output=True,
                       text=True, env=env, timeout=600, cwd=rtc.substitute_dir())
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.split()[2] == (variant if scene > 1 or variant in ("all", "pre") else "book1")
    sc = rtc.Scene.preset(scene, width, spp, depth)
    ref = pyoracle.render(sc)
    got = np.fromfile(out, np.uint8).reshape(ref.shape)
    bad = (got != ref).any(axis=2)
    assert not bad.any(), f"{bad.sum()} pixels differ; first at {np.argwhere(bad)[0]}"


CHAIN = os.path.join(ROOT, "tests", "native", "bin", "chain_sim")


@pytest.mark.parametrize("scene,width,spp,seed,kmin,kmax,margin,slack,pad,pre", [
    (1, 48, 64, 1, 2, 8, 1.5, 64, 1.0, 0),    # plain plans
    (1, 48, 64, 2, 2, 16, 1.0, 1, 1.0, 0),    # lists one record past the plan: most pixels need a continuation
    (0, 40, 40, 3, 1, 8, 1.2, 4, 1.0, 0),     # the three-spheres scene, unsplit pixels mixed in
    (1, 48, 32, 4, 4, 32, 1.0, 2, 1.0, 0),    # many short segments
    (1, 24, 200, 5, 2, 6, 1.5, 64, 1.0, 0),   # long segments
    (1, 48, 64, 6, 8, 24, 1.5, 64, 1.3, 0),   # padded plans: segments past the stream's true end
    (1, 24, 200, 7, 8, 16, 1e9, 64, 1.6, 0),  # padded long segments, lists of spp + slack (the planner's)
    (1, 48, 64, 8, 2, 16, 1.0, 1, 1.3, 0),    # padded plans with tiny lists (continuations)
    (0, 40, 40, 9, 1, 8, 1.2, 4, 2.0, 0),     # padded, unsplit pixels mixed in
    (1, 48, 64, 10, 2, 8, 1.5, 64, 1.0, 16),  # segment 0 / unsplit chains go on from the pre-pass's 16 samples
    (1, 48, 64, 11, 8, 32, 1.0, 2, 1.0, 16),  #   ... with many short segments: the pre-pass ends past segment 1's start
    (1, 48, 64, 12, 2, 16, 1.0, 1, 1.3, 8),   #   ... with padded plans and tiny lists (continuations)
    (0, 40, 40, 13, 1, 8, 1.2, 4, 2.0, 16)])  #   ... unsplit pixels mixed in
def test_chain_protocol_on_host_matches_oracle(tmp_path, scene, width, spp, seed, kmin, kmax, margin, slack, pad, pre):
    """The chain render's protocol (rt_book1.h: chain_boundary / chain_couple / chain_walk_done /
    chain_record) on the host under ASan, with random segment counts, stream-length estimates off by up
    to 2x (and padded plans, whose last segments start past the true stream end), tiny record lists and
    a random interleaving of the chains, then the fold and the continuations: every pixel must equal
    the oracle's."""
    out = str(tmp_path / "c.rgb")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([CHAIN, str(scene), str(width), str(spp), "50", out, str(seed), str(kmin), str(kmax), str(margin),
                        str(slack), str(pad), str(pre)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    sc = rtc.Scene.preset(scene, width, spp, 50)
    ref = pyoracle.render(sc)
    got = np.fromfile(out, np.uint8).reshape(ref.shape)
    bad = (got != ref).any(axis=2)
    assert not bad.any(), f"{bad.sum()} pixels differ; first at {np.argwhere(bad)[0]}; {r.stdout}"


STACK = os.path.join(ROOT, "tests", "native", "bin", "stack_check")


def test_path_record_on_host_matches_recursion():
    """The general kernel's path record (rt_general.h: PathRecord -- run-length albedo codes, the
    explicit-albedo and weight register stacks and their overflow slots, the weight-2.0f bits, the
    zero-tail shortcut) on the host under ASan at every register-stack depth RT_GEN_WREG / RT_GEN_XREG
    can select (0/0 through 8/2): random paths of 1-64 bounces with non-finite values mixed in must fold
    to the recursion's colour bit for bit (the spill indexing is pinned at every depth)."""
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([STACK, "20000"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert r.stdout.count("paths ok") == 8, r.stdout
