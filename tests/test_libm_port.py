"""The glibc-exact libm port (ray-tracing-c_amd/csrc/rt_libm.h) against the host glibc the reference
links, over the domains the hot path feeds it.

CPU: the port compiled for the host (hipcc host pass), exhaustively:
  sincosf on all 2^24 Lambertian/Sphere_rand angles phi = (2*(float)pi) * k/2^24
  powf(x, 5) on every float in [0, 2]            (Dielectric Schlick term, src/material.c:73)
  logf on all 2^24 pcg32_f32 values              (ConstantMedium, src/hittable.c:413)
  atanf on every float, acosf on every float in [-1, 1], atan2f on 2^28 random pairs and the
  sphere u,v expression on 2^26 unit normals   (Sphere_hit u,v, src/hittable.c:146-147)
GPU: the same functions compiled for gfx950, on the same domains (pow5 strided), through the
C ABI's rt_diag_libm, compared with glibc evaluated on the host.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import rtc
from conftest import ROOT

BIN = os.path.join(ROOT, "tests", "native", "bin")


@pytest.mark.parametrize("fn", ["sincos_phi", "pow5", "logf_f32", "atanf_all", "acosf_unit", "atan2f_rand",
                                "uv_sphere"])
def test_port_exhaustive_on_host(fn):
    r = subprocess.run([os.path.join(BIN, "libm_check"), fn], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and " mismatches=0 " in r.stdout, r.stdout + r.stderr


def test_port_tables_are_the_host_libm_words():
    """Provenance of the port's tables: oracle/tools/extract_libm_tables.cpp finds every table in the
    host libm.so.6 (the library the reference links) and compares it word for word with rt_libm.h."""
    exe = os.path.join(BIN, "extract_libm_tables")
    if not os.path.exists("/lib/x86_64-linux-gnu/libm.so.6"):
        pytest.skip("no x86-64 glibc libm here")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "all tables identical to the host libm" in r.stdout, r.stdout + r.stderr


def test_port_sincos_large_arguments_sample_on_host():
    """|x| >= 120 uses the 4/pi bit-table reduction (Perlin's sinf argument can get there)."""
    lo, hi = 0x42f00000, 0x42f00000 + (1 << 22)
    r = subprocess.run([os.path.join(BIN, "libm_check"), "sincos_all", hex(lo), hex(hi)], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0 and " mismatches=0 " in r.stdout, r.stdout + r.stderr


def _glibc():
    L = ctypes.CDLL(os.path.join(BIN, "libglibc_ref.so"))
    for n in ("ref_sincosf", "ref_pow5", "ref_logf", "ref_sinf", "ref_atan2f", "ref_acosf"):
        getattr(L, n).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        getattr(L, n).restype = None
    return L


def _host(fn_name, x, nout, count=None):
    """glibc over x; `count` = elements the C loop walks (pairs for ref_atan2f), default x.size."""
    out = np.empty(nout, np.float32)
    count = x.size if count is None else count
    assert count <= x.size and nout >= (2 * count if fn_name == "ref_sincosf" else count)
    getattr(_glibc(), fn_name)(x.ctypes.data, out.ctypes.data, count)
    return out


def _same_bits(a, b):
    a, b = a.view(np.uint32), b.view(np.uint32)
    nan = np.isnan(a.view(np.float32)) & np.isnan(b.view(np.float32))
    return (a == b) | nan


@pytest.mark.gpu
def test_device_sincos_phi_domain_exhaustive():
    k = np.arange(1 << 24, dtype=np.float32)
    phi = np.float32(2.0 * np.float32(np.pi)) * (k / np.float32(1 << 24))
    dev = rtc.diag_libm(0, phi)
    host = _host("ref_sincosf", phi, 2 * phi.size)
    ok = _same_bits(dev, host)
    assert ok.all(), f"{(~ok).sum()} mismatches, first phi={phi[np.argmin(ok) // 2]!r}"


@pytest.mark.gpu
def test_device_logf_f32_domain_exhaustive():
    x = (np.arange(1, 1 << 24, dtype=np.float64) / (1 << 24)).astype(np.float32)
    ok = _same_bits(rtc.diag_libm(2, x), _host("ref_logf", x, x.size))
    assert ok.all(), f"{(~ok).sum()} mismatches"


@pytest.mark.gpu
def test_device_pow5_unit_interval_strided():
    bits = np.arange(0, 0x3F800001, 13, dtype=np.uint32)  # every 13th float in [0, 1]
    x = bits.view(np.float32)
    ok = _same_bits(rtc.diag_libm(1, x), _host("ref_pow5", x, x.size))
    assert ok.all(), f"{(~ok).sum()} mismatches"


@pytest.mark.gpu
def test_device_sinf_random_and_special():
    rng = np.random.default_rng(1)
    bits = rng.integers(0, 1 << 32, 1 << 22, dtype=np.uint64).astype(np.uint32)
    x = bits.view(np.float32)
    x = x[np.isfinite(x)]
    specials = np.array([0.0, -0.0, 1e-30, 120.0, -120.0, 1e10, 3.4e38, np.pi, 2 * np.pi], np.float32)
    x = np.concatenate([x, specials]).astype(np.float32)
    ok = _same_bits(rtc.diag_libm(3, x), _host("ref_sinf", x, x.size))
    assert ok.all(), f"{(~ok).sum()} mismatches, first x={x[np.argmin(ok)]!r}"


@pytest.mark.gpu
def test_device_atan2f_acosf_sphere_uv():
    """u, v of the sphere hit record (Checker / Image textures) on the device, vs glibc."""
    rng = np.random.default_rng(3)
    v = rng.normal(size=(1 << 22, 3)).astype(np.float32)
    v /= np.sqrt((v * v).sum(axis=1, keepdims=True)).astype(np.float32)
    yx = np.stack([-v[:, 2], v[:, 0]], axis=1).astype(np.float32).ravel()
    ok = _same_bits(rtc.diag_libm(4, yx), _host("ref_atan2f", yx, yx.size // 2, count=yx.size // 2))
    assert ok.all(), f"atan2f: {(~ok).sum()} mismatches"
    a = np.concatenate([-v[:, 1], rng.uniform(-1, 1, 1 << 20).astype(np.float32),
                        np.array([-1.0, 1.0, 0.0, -0.0, 0.5, -0.5], np.float32)])
    ok = _same_bits(rtc.diag_libm(5, a), _host("ref_acosf", a, a.size))
    assert ok.all(), f"acosf: {(~ok).sum()} mismatches"


@pytest.mark.gpu
def test_device_exact_sqrt_core_all_floats():
    """Book-1 v5 sqrt_core == sqrtf on every float of its domain (0 and [2^-96, inf])."""
    assert rtc.diag_arith(0, 0, 0x7F800001) == 0


@pytest.mark.gpu
def test_device_exact_div_core_random_pairs():
    """Book-1 v5 div_core with the per-ray reciprocal == '/' on 2^32 hashed pairs of its domain."""
    assert rtc.diag_arith(1, 0, 1 << 32, seed=11) == 0


@pytest.mark.gpu
def test_device_sphere_test_v5_matches_reference_expression():
    """The guarded fast sphere test gives the reference's outcome (hit, t_max bits) on 2^30 hashed rays,
    half starting on the sphere (c ~ 0: cancelling numerators, the tiny-root argument in rt_book1.h)."""
    assert rtc.diag_arith(2, 0, 1 << 30, seed=5) == 0
