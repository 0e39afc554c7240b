"""Host side of the drop-in library (no GPU): scene construction, pcg32, TIFF bytes, C-ABI exports.

The reference has no unit tests; its CI only builds and runs `./main 1` and `./main 4`
(.github/workflows/build.yaml:20-21).  These tests check the pieces that must equal the
reference bit for bit before any pixel is traced: the scene graph each of the 8 driver scenes
builds (vs `ref_render dump`), the pcg32 stream (vs `ref_render kat`) and the TIFF writer.
"""
import ctypes
import gzip
import hashlib
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

import pyoracle
import rtc
from conftest import GOLDEN, ROOT


@pytest.mark.parametrize("scene", range(8))
def test_scene_graph_matches_reference(scene, tmp_path):
    """Same objects, materials, textures, BVH topology and camera as the reference's scene_<N>."""
    sc = rtc.Scene.preset(scene)
    mine = pyoracle.dump_flat(sc, str(tmp_path / "dump.txt"))
    with gzip.open(os.path.join(GOLDEN, f"scene{scene}.dump.gz"), "rt") as f:
        ref = f.read()
    if mine != ref:
        a, b = mine.splitlines(), ref.splitlines()
        first = next(i for i in range(min(len(a), len(b))) if a[i] != b[i]) if a[:len(b)] != b[:len(a)] else min(len(a), len(b))
        pytest.fail(f"scene {scene}: first difference at line {first}:\n mine: {a[first] if first < len(a) else None}\n"
                    f"  ref: {b[first] if first < len(b) else None}")


def _kat_lines():
    return open(os.path.join(GOLDEN, "kat.txt")).read().splitlines()


def test_pcg32_known_answers():
    L = rtc.lib()

    class PCG32(ctypes.Structure):
        _fields_ = [("state", ctypes.c_uint64), ("inc", ctypes.c_uint64)]

    L.pcg32_seed.argtypes = [ctypes.POINTER(PCG32), ctypes.c_uint64, ctypes.c_uint64]
    L.pcg32_u32.argtypes = [ctypes.POINTER(PCG32)]
    L.pcg32_u32.restype = ctypes.c_uint32
    for line in _kat_lines():
        m = re.match(r"seed (\d+) (\d+) state ([0-9a-f]+) inc ([0-9a-f]+) u32 (.*)", line)
        if not m:
            continue
        g = PCG32()
        L.pcg32_seed(ctypes.byref(g), int(m.group(1)), int(m.group(2)))
        assert (g.state, g.inc) == (int(m.group(3), 16), int(m.group(4), 16))
        got = [L.pcg32_u32(ctypes.byref(g)) for _ in range(8)]
        assert got == [int(x, 16) for x in m.group(5).split()]


def test_vec3_rand_draw_order_is_gcc_order():
    """vec3_rand fills z with the first draw (gcc right-to-left argument evaluation)."""
    L = rtc.lib()

    class PCG32(ctypes.Structure):
        _fields_ = [("state", ctypes.c_uint64), ("inc", ctypes.c_uint64)]

    class Vec3(ctypes.Structure):
        _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float)]

    L.pcg32_seed.argtypes = [ctypes.POINTER(PCG32), ctypes.c_uint64, ctypes.c_uint64]
    L.vec3_rand.argtypes = [ctypes.POINTER(PCG32)]
    L.vec3_rand.restype = Vec3
    L.vec3_rand_unit_vector.argtypes = [ctypes.POINTER(PCG32)]
    L.vec3_rand_unit_vector.restype = Vec3
    g = PCG32()
    L.pcg32_seed(ctypes.byref(g), 19, 29)
    v = L.vec3_rand(ctypes.byref(g))
    u = L.vec3_rand_unit_vector(ctypes.byref(g))
    kat = {l.split(")")[0] + ")": l.split(")")[1].split() for l in _kat_lines() if l.startswith("vec3_")}
    assert [float.fromhex(x) for x in kat["vec3_rand(seed 19 29)"]] == [v.x, v.y, v.z]
    assert [float.fromhex(x) for x in kat["vec3_rand_unit_vector(next)"]] == [u.x, u.y, u.z]


def _write_tiff(w, h, n, data):
    L = rtc.lib()
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    L.write_tiff.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    L.write_tiff.restype = ctypes.c_int
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "o.tiff")
        f = libc.fopen(p.encode(), b"wb")
        buf = np.ascontiguousarray(data, dtype=np.uint8)
        rc = L.write_tiff(f, w, h, n, buf.ctypes.data)
        libc.fclose(f)
        return rc, open(p, "rb").read()


def test_tiff_header_matches_reference():
    rc, data = _write_tiff(400, 225, 3, np.zeros(400 * 225 * 3, np.uint8))
    assert rc == 0
    assert data[:168] == open(os.path.join(GOLDEN, "tiff_header.bin"), "rb").read()
    assert len(data) == 168 + 400 * 225 * 3


def test_tiff_full_file_matches_reference(manifest):
    """Byte-identical TIFF for the reference's 400x225 1-spp depth-1 scene-0 render."""
    e = manifest["tiff_s0_400x225_1spp_d1"]
    sc = rtc.Scene.preset(0, 400, 1, 1)
    img = pyoracle.render(sc)
    rc, data = _write_tiff(400, 225, 3, img)
    assert rc == 0 and len(data) == e["size"]
    assert hashlib.sha256(data).hexdigest() == e["sha256"]


def test_tiff_grayscale_and_unsupported_channels():
    rc, data = _write_tiff(4, 2, 1, np.arange(8, dtype=np.uint8))
    assert rc == 0 and len(data) == 146 + 2 + 16 + 8 and data[-8:] == bytes(range(8))
    rc, data = _write_tiff(4, 2, 2, np.zeros(16, np.uint8))
    assert rc == 1 and len(data) == 10 + 3 * 12  # the reference bails after the first 3 entries


def _declared_functions():
    names = set()
    for fn in sorted(os.listdir(os.path.join(ROOT, "include"))):
        src = open(os.path.join(ROOT, "include", fn)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        src = re.sub(r"#[^\n]*(\\\n[^\n]*)*", "", src)  # macros (vec3_add etc. are macros)
        src = re.sub(r"typedef struct \w+ \{.*?\} \w+;", "", src, flags=re.S)
        src = re.sub(r"(struct|union|enum) \w* ?\{.*?\};", "", src, flags=re.S)
        src = re.sub(r"typedef [^;]*;", "", src)
        src = re.sub(r"static inline[^{]*\{[^}]*\}", "", src)
        for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", src):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_function():
    names = _declared_functions()
    for must in ("Camera_render", "Camera_init", "World_init", "rt_render", "rt_render_rows_async",
                 "rt_scene_upload", "rt_flatten", "write_tiff", "pcg32_seed", "BVHNode_new", "Perlin_new"):
        assert must in names
    L = rtc.lib()
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert not missing, f"declared in include/*.h but not exported: {missing}"
    assert hasattr(L, "VEC3_ZERO")


def test_product_library_does_not_link_the_oracle():
    out = subprocess.run(["ldd", rtc.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    syms = subprocess.run(["nm", "-D", "--defined-only", rtc.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in syms
    assert rtc.lib().rt_abi_version() == 1


def test_flattener_rejects_foreign_objects():
    """An object whose vtable this library did not create fails loudly instead of rendering wrong."""
    L = rtc.lib()
    sc = rtc.Scene.preset(0, 40, 1, 1)
    assert sc.features == 0 and sc.s.stack_needed >= 1
    s1 = rtc.Scene.preset(1, 40, 1, 1)
    assert s1.features & rtc.FEAT_BVH and s1.features & rtc.FEAT_DOF
    s7 = rtc.Scene.preset(7, 40, 1, 1)
    for f in (rtc.FEAT_QUAD, rtc.FEAT_XFORM, rtc.FEAT_MEDIUM, rtc.FEAT_LIGHTS, rtc.FEAT_TEX_UV, rtc.FEAT_TEX_PERLIN):
        assert s7.features & f
    assert s7.s.stack_needed <= 48
    L.rt_flatten.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.rt_flatten.restype = ctypes.c_void_p
    assert not L.rt_flatten(None, None)
    assert "NULL" in rtc.last_error()


def test_rows_partition_covers_frame_once():
    for h in (1, 2, 7, 168, 675):
        for world in (1, 2, 3, 4, 8):
            rows = []
            for r in range(world):
                row0, stride, n = rtc.rows_of(h, r, world)
                rows += [row0 + k * stride for k in range(n)]
            assert sorted(rows) == list(range(h))


def _flat_image(sc):
    """The first image texture's RGB bytes of a flattened scene (rt_flat.h: rt_image)."""
    s = sc.s
    im = ctypes.cast(s.images, ctypes.POINTER(ctypes.c_int32 * 4))[0]
    W, H = im[0], im[1]
    return np.frombuffer(ctypes.string_at(s.image_bytes, W * H * 3), np.uint8).reshape(H, W, 3)


@pytest.mark.parametrize("subsampling,mode,opts", [
    ("4:4:4", "RGB", {}), ("4:2:0", "RGB", {}), ("4:2:2", "RGB", {}), ("4:4:4", "L", {}),
    ("4:2:0", "RGB", {"optimize": True}), ("4:2:0", "RGB", {"restart_marker_rows": 1}),
    ("4:4:4", "RGB", {"restart_marker_blocks": 5})])
def test_image_new_decodes_baseline_jpeg(tmp_path, subsampling, mode, opts):
    """Image_new on a real JPEG: the reference decodes earthmap.jpg with stb_image
    (src/texture.c:38-42); host/rt_jpeg.c restates stb's baseline decoding (integer IDCT, triangle
    chroma upsampling, fixed-point YCbCr).  stb is un-vendored here, so exact parity is unpinned; an
    independent codec (Pillow's libjpeg) must agree within a few levels (different IDCT, upsampling
    and colour rounding)."""
    PIL = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(7)
    h, w = 75, 131
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.stack([xx * 255 // (w - 1), yy * 255 // (h - 1), (xx ^ yy) & 255], -1)
    img = (img + rng.integers(-20, 20, img.shape)).clip(0, 255).astype(np.uint8)
    path = tmp_path / "earthmap.jpg"
    try:
        PIL.fromarray(img).convert(mode).save(path, quality=90, subsampling=subsampling, **opts)
    except (TypeError, ValueError) as e:  # (an older Pillow without that option)
        pytest.skip(f"Pillow cannot write this variant: {e}")
    ref = np.asarray(PIL.open(path).convert("RGB")).astype(int)
    got = _flat_image(rtc.Scene.preset(3, 40, 1, 1, image_dir=str(tmp_path))).astype(int)
    assert got.shape == ref.shape
    if subsampling == "4:2:2":  # (stb's h2v1 filter weights the last chroma sample's left neighbour 3:1)
        got, ref = got[:, :-1], ref[:, :-1]
    d = np.abs(got - ref)
    assert d.max() <= 6 and d.mean() < 0.5, (d.max(), d.mean())


def test_image_new_reports_unreadable_image(tmp_path):
    """A progressive JPEG (not decoded) or a non-image file: the preset reports it (the reference and
    this library's own Image_new abort, src/texture.c:41) instead of rendering a wrong texture."""
    PIL = pytest.importorskip("PIL.Image")
    PIL.fromarray(np.zeros((16, 16, 3), np.uint8)).save(tmp_path / "earthmap.jpg", progressive=True)
    with pytest.raises(rtc.RtcError, match="progressive"):
        rtc.Scene.preset(3, 40, 1, 1, image_dir=str(tmp_path))
    (tmp_path / "earthmap.jpg").write_bytes(b"not an image")
    with pytest.raises(rtc.RtcError, match="earthmap.jpg"):
        rtc.Scene.preset(7, 40, 1, 1, image_dir=str(tmp_path))


def test_preset_substitute_picture_is_opt_in(tmp_path, monkeypatch):
    """the substitute earth picture is used only on request, and no working directory
    is changed.  Without the opt-in and without earthmap.jpg, scene 7 is reported as unreadable."""
    monkeypatch.chdir(tmp_path)
    monkeypatch.setenv("RTC_SUBSTITUTE_EARTH", "0")
    with pytest.raises(rtc.RtcError, match="earthmap.jpg"):
        rtc.Scene.preset(7, 40, 1, 1)
    sc = rtc.Scene.preset(7, 40, 1, 1, substitute_earth=True)
    assert _flat_image(sc).shape == (512, 1024, 3)
    assert os.getcwd() == str(tmp_path)


def _jpeg_fuzz_exe():
    exe = os.path.join(ROOT, "tests", "native", "bin", "jpeg_fuzz")
    src = [os.path.join(ROOT, "tests", "native", "jpeg_fuzz.c"), os.path.join(ROOT, "ray-tracing-c_amd", "host", "rt_jpeg.c")]
    if not os.path.exists(exe) or any(os.path.getmtime(s) > os.path.getmtime(exe) for s in src):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "native"), "bin/jpeg_fuzz"], check=True,
                       capture_output=True)
    return exe


def test_jpeg_decoder_survives_truncated_and_corrupted_files(tmp_path):
    """every table / header read of host/rt_jpeg.c is bounded by its segment.  The decoder,
    built with AddressSanitizer + UBSan (tests/native/jpeg_fuzz), runs over truncations at every byte of
    the headers and every 9th byte after them, and over single-byte corruptions of the headers; each
    file must decode or be rejected -- never read out of bounds (ASan exits non-zero)."""
    import jpeg_tools

    rng = np.random.default_rng(3)
    img = rng.integers(0, 255, (20, 27, 3), dtype=np.uint8)
    files = []
    for name, data in (("il", jpeg_tools.encode(img, True)), ("nil", jpeg_tools.encode(img, False)),
                       ("grey", jpeg_tools.encode(img[..., 0], False))):
        sos = data.index(b"\xff\xda")
        for n in list(range(0, sos + 16)) + list(range(sos + 16, len(data), 9)):
            files.append((f"{name}_t{n}", data[:n]))
        for n in range(2, sos + 12):
            for v in (0x00, 0xFF, data[n] ^ 0x5A, 0x01):
                files.append((f"{name}_c{n}_{v}", data[:n] + bytes([v]) + data[n + 1:]))
    # segments whose length field is shorter than the table / header they announce, at the end of the
    # file: the old walk read the announced bytes past the buffer
    il = jpeg_tools.encode(img, True)
    frame = il[:il.index(b"\xff\xc4")]  # SOI, APP0, DQT, SOF0
    for k, tail in enumerate((b"\xff\xdb\x00\x03\x00", b"\xff\xc4\x00\x03\x00", b"\xff\xdd\x00\x02",
                              b"\xff\xc0\x00\x03\x08", b"\xff\xc4\x00\x13\x00" + bytes([0] * 15) + b"\x09")):
        files.append((f"short{k}", il[:2] + tail))
    files.append(("short_sos", frame + b"\xff\xda\x00\x03\x03"))
    # a frame whose sampling factors are not whole ratios (h 3 vs 2): rejected, as stb_image does
    bad = bytearray(jpeg_tools.encode(img, True))
    sof = bad.index(b"\xff\xc0")
    bad[sof + 11], bad[sof + 14] = 0x31, 0x21
    files.append(("ratio", bytes(bad)))
    paths = []
    for name, data in files:
        p = tmp_path / f"{name}.jpg"
        p.write_bytes(data)
        paths.append(str(p))
    exe = _jpeg_fuzz_exe()
    for k in range(0, len(paths), 500):
        r = subprocess.run([exe] + paths[k:k + 500], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    r = subprocess.run([exe, paths[-1]], capture_output=True, text=True, timeout=60)
    assert r.stdout.startswith("err") and "sampling" in r.stdout, r.stdout


@pytest.mark.parametrize("grey", [False, True])
def test_image_new_decodes_non_interleaved_jpeg(tmp_path, grey):
    """a baseline JPEG whose components come in separate scans (T.81 §A.2.2; Pillow never
    writes one) decodes to exactly the pixels of the same coefficients in one interleaved scan, and
    agrees with Pillow's libjpeg within the usual IDCT / colour rounding."""
    import jpeg_tools

    rng = np.random.default_rng(11)
    h, w = 45, 70
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.stack([xx * 255 // (w - 1), yy * 255 // (h - 1), (xx ^ yy) & 255], -1)
    img = (img + rng.integers(-15, 15, img.shape)).clip(0, 255).astype(np.uint8)
    if grey:
        img = img[..., 1]
    got = {}
    for layout in (True, False):
        d = tmp_path / ("il" if layout else "nil")
        d.mkdir()
        (d / "earthmap.jpg").write_bytes(jpeg_tools.encode(img, layout))
        got[layout] = _flat_image(rtc.Scene.preset(3, 40, 1, 1, image_dir=str(d))).astype(int)
    assert np.array_equal(got[True], got[False])
    PIL = pytest.importorskip("PIL.Image")
    ref = np.asarray(PIL.open(tmp_path / "nil" / "earthmap.jpg").convert("RGB")).astype(int)
    assert ref.shape == got[False].shape
    diff = np.abs(ref - got[False])
    assert diff.max() <= 3 and diff.mean() < 0.5, (diff.max(), diff.mean())
