"""pyoracle — TEST INFRASTRUCTURE: Python handles on the oracle (liboracle.so, oracle/_ref/*).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.  The
product path (librtc_amd.so, rtc) never touches it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(ORACLE_DIR, "liboracle.so")
REF_STRICT = os.path.join(ORACLE_DIR, "_ref", "ref_render")
REF_FAST = os.path.join(ORACLE_DIR, "_ref", "ref_render_fast")
REF_DROPIN = os.path.join(ORACLE_DIR, "_ref", "ref_main_dropin")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} not built: run `make -C oracle`")
        L = ctypes.CDLL(LIB)
        L.oracle_render_rows.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.oracle_render_rows.restype = ctypes.c_int
        L.oracle_render_pixels.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_void_p]
        L.oracle_render_pixels.restype = ctypes.c_int
        L.oracle_dump_flat.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.oracle_dump_flat.restype = ctypes.c_int
        _lib = L
    return _lib


def render(scene, row0: int = 0, row_stride: int = 1, n_rows: int | None = None) -> np.ndarray:
    """CPU restatement render of `scene` (an rtc.Scene) rows row0 + k*row_stride."""
    if n_rows is None:
        n_rows = (scene.height - row0 + row_stride - 1) // row_stride
    out = np.empty((n_rows, scene.width, 3), dtype=np.uint8)
    lib().oracle_render_rows(ctypes.cast(scene.ptr, ctypes.c_void_p), row0, row_stride, n_rows, out.ctypes.data)
    return out


def render_pixels(scene, xs, ys) -> np.ndarray:
    xs = np.ascontiguousarray(xs, dtype=np.int32)
    ys = np.ascontiguousarray(ys, dtype=np.int32)
    out = np.empty((xs.size, 3), dtype=np.uint8)
    lib().oracle_render_pixels(ctypes.cast(scene.ptr, ctypes.c_void_p), xs.ctypes.data, ys.ctypes.data, xs.size,
                               out.ctypes.data)
    return out


_workdir = None


def ref_workdir() -> str:
    """A directory holding the substitute earthmap.jpg (rtc/earth.py): the reference build reads it
    from its working directory for scenes 3 and 7 (src/main.c:104, :243)."""
    global _workdir
    if _workdir is None:
        import sys
        import tempfile

        sys.path.insert(0, os.path.join(os.path.dirname(ORACLE_DIR), "ray-tracing-c_amd"))
        from rtc import earth

        _workdir = tempfile.mkdtemp(prefix="rtc_ref_")
        earth.write_substitute(_workdir)
    return _workdir


def ref_render(scene_id: int, width: int, spp: int, depth: int, out_path: str, fast: bool = False,
               threads: int | None = None, timeout: float | None = None) -> tuple[int, int]:
    """Run the reference build (oracle/_ref) and return (W, H); raw RGB goes to out_path."""
    exe = REF_FAST if fast else REF_STRICT
    env = dict(os.environ)
    if threads:
        env["OMP_NUM_THREADS"] = str(threads)
    r = subprocess.run([exe, "render", str(scene_id), str(width), str(spp), str(depth), os.path.abspath(out_path)],
                       env=env, capture_output=True, text=True, timeout=timeout, check=True, cwd=ref_workdir())
    w, h = r.stdout.split()[:2]
    return int(w), int(h)


def ref_available() -> bool:
    return os.path.exists(REF_STRICT)


def dump_flat(scene, path: str) -> str:
    """Canonical text dump of an rtc.Scene (same format as `ref_render dump`)."""
    if lib().oracle_dump_flat(ctypes.cast(scene.ptr, ctypes.c_void_p), path.encode()) != 0:
        raise RuntimeError("oracle_dump_flat failed")
    with open(path) as f:
        return f.read()
