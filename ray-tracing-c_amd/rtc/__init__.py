"""rtc — Python view of the MI355X render path (ctypes over the C ABI in include/rt_hip.h).

The product is the C library ``ray-tracing-c_amd/librtc_amd.so`` (drop-in ``Camera_render`` + the
gfx950 kernels).  This module only binds it for tests and ``bench.py``; it adds no compute of its
own and has no fallback: if the library or a GPU is missing, calls raise ``RtcError``.

Reference boundary mirrored: ``void Camera_render(const Camera*, const World*, uint8_t*)``
(reference include/raytracing.h:41, src/raytracing.c:86-135).
"""
from __future__ import annotations

import ctypes
import os
import sys
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int32, c_int64, c_void_p

import numpy as np

from . import earth

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # ray-tracing-c_amd/
# RTC_LIB: an alternative build of the same library (same-box A/B timing of two builds; tests and
# bench use the in-tree library)
LIB_PATH = os.path.abspath(os.environ.get("RTC_LIB") or os.path.join(PKG_DIR, "librtc_amd.so"))
# the diagnostic build of the same sources (-DRT_DIAG): also reads the A/B switches, timeline and
# fault-injection variables; tests select it with use_diag()
DIAG_PATH = os.path.join(PKG_DIR, "librtc_amd_diag.so")

# rt_feature_bits (include/rt_flat.h)
FEAT_BVH, FEAT_QUAD, FEAT_XFORM, FEAT_MEDIUM = 1, 2, 4, 8
FEAT_LIGHTS, FEAT_TEX_UV, FEAT_TEX_PERLIN, FEAT_EMISSIVE, FEAT_DOF = 16, 32, 64, 128, 256

# reference scene ids (src/main.c:294-329) and their names
SCENES = {
    0: "Book 1: Metal and Lambertian",
    1: "Book 1: Final scene",
    2: "Book 2: Checker",
    3: "Book 2: Earth",
    4: "Book 2: Perlin noise",
    5: "Book 2: Simple light",
    6: "Book 2: Cornell box",
    7: "Book 2: Final scene",
}


class RtcError(RuntimeError):
    pass


class RtCamera(ctypes.Structure):
    _fields_ = [
        ("width", c_int32), ("height", c_int32), ("spp", c_int32), ("max_depth", c_int32),
        ("pixel00", c_float * 3), ("dof_angle", c_float),
        ("delta_u", c_float * 3), ("light_prob", c_float),
        ("delta_v", c_float * 3), ("pad0", c_float),
        ("origin", c_float * 3), ("pad1", c_float),
        ("disc_u", c_float * 3), ("pad2", c_float),
        ("disc_v", c_float * 3), ("pad3", c_float),
        ("background", c_float * 3), ("pad4", c_float),
    ]


_COUNTS = ["n_bvh", "n_spheres", "n_quads", "n_lists", "n_list_items", "n_translates", "n_rotates",
           "n_media", "n_materials", "n_textures", "n_images", "n_perlins"]
_ARRAYS = ["bvh", "spheres", "quads", "lists", "list_items", "translates", "rotates", "media",
           "materials", "textures", "images", "perlins", "image_bytes"]


class RtFlatScene(ctypes.Structure):
    _fields_ = ([("camera", RtCamera), ("root", c_int32), ("lights", c_int32), ("features", c_int32),
                 ("stack_needed", c_int32)]
                + [(n, c_int32) for n in _COUNTS]
                + [("n_image_bytes", c_int64)]
                + [(n, c_void_p) for n in _ARRAYS])


assert ctypes.sizeof(RtCamera) == 128
assert RtFlatScene.n_image_bytes.offset == 192


_libs = {}          # loaded libraries by path
_current = LIB_PATH
_subst_dir = None


def substitute_dir() -> str:
    """A private directory holding the substitute earthmap.jpg (created once per process)."""
    global _subst_dir
    if _subst_dir is None:
        import tempfile

        _subst_dir = tempfile.mkdtemp(prefix="rtc_earth_")
        earth.write_substitute(_subst_dir)
    return _subst_dir


def _init_torch_runtime_first() -> None:
    """The PyTorch-ROCm wheel bundles its own HIP runtime (torch/lib/libamdhip64.so, no SONAME), so a
    process holding PyTorch and this library runs two HIP runtimes side by side.  PyTorch's only
    finds the GPUs when it initialises first (measured on MI355X: the other order gives "No HIP GPUs
    are available"), so when PyTorch is already imported it is initialised before this library's
    first HIP call.  Processes that import PyTorch later must initialise it before using rtc."""
    torch = sys.modules.get("torch")
    if torch is None:
        return
    try:
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:  # a CPU-only torch build: nothing to order
        pass


class use_diag:
    """Context manager: objects created inside it use the diagnostic build (librtc_amd_diag.so), which
    reads the A/B switches (RT_MODE, RT_BOOK1_LDS, RT_CHAIN_MARGIN, RT_FAULT_MIG_DROP ...) the product
    library ignores.  Both libraries can be loaded in one process (each keeps its own symbols)."""

    def __init__(self, on: bool = True):
        self.on = on

    def __enter__(self):
        global _current
        self._prev = _current
        if self.on:
            _current = DIAG_PATH
        return self

    def __exit__(self, *exc):
        global _current
        _current = self._prev
        return False


def lib() -> ctypes.CDLL:
    """Load librtc_amd.so (built by ``make -C ray-tracing-c_amd``), or the diagnostic build inside use_diag()."""
    path = _current
    if path not in _libs:
        if not os.path.exists(path):
            raise RtcError(f"{path} not built: run `make -C ray-tracing-c_amd` (or __graft_entry__.build())")
        _init_torch_runtime_first()
        L = ctypes.CDLL(path)
        P = POINTER(RtFlatScene)
        L.rt_scene_preset.argtypes = [c_int, c_int, c_int, c_int]
        L.rt_scene_preset.restype = P
        L.rt_scene_preset_in.argtypes = [c_int, c_int, c_int, c_int, c_char_p]
        L.rt_scene_preset_in.restype = P
        L.rt_flat_free.argtypes = [P]
        L.rt_flat_free.restype = None
        L.rt_device_count.restype = c_int
        L.rt_scene_upload.argtypes = [P, c_int]
        L.rt_scene_upload.restype = c_void_p
        L.rt_scene_release.argtypes = [c_void_p]
        L.rt_scene_release.restype = None
        L.rt_render_rows_async.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]
        L.rt_render_rows_async.restype = c_int
        L.rt_render.argtypes = [P, c_int, c_void_p]
        L.rt_render.restype = c_int
        L.rt_last_kernel_ms.argtypes = [c_int]
        L.rt_last_kernel_ms.restype = c_double
        if hasattr(L, "rt_render_share"):  # (older builds loaded through RTC_LIB for an A/B lack these)
            L.rt_render_share.argtypes = [P, c_int, c_int, c_int, c_void_p]
            L.rt_render_share.restype = c_int
            L.rt_render_cache_release.argtypes = []
            L.rt_render_cache_release.restype = None
            L.rt_last_share_ms.argtypes = [c_int, c_void_p]
            L.rt_last_share_ms.restype = c_int
        L.rt_diag_libm.argtypes = [c_int, c_void_p, c_void_p, c_int64, c_int]
        L.rt_diag_libm.restype = c_int
        L.rt_diag_arith.argtypes = [c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, c_void_p, c_int]
        L.rt_diag_arith.restype = c_int
        L.rt_scene_last_launch_ms.argtypes = [c_void_p]
        L.rt_scene_last_launch_ms.restype = c_double
        if hasattr(L, "rt_scene_launch_history"):  # (older builds loaded through RTC_LIB for an A/B lack it)
            L.rt_scene_launch_history.argtypes = [c_void_p, c_void_p, c_int]
            L.rt_scene_launch_history.restype = c_int
        L.rt_scene_kernel.argtypes = [c_void_p]
        L.rt_scene_kernel.restype = c_char_p
        L.rt_scene_check.argtypes = [c_void_p]
        L.rt_scene_check.restype = c_int
        L.rt_last_error.restype = c_char_p
        L.rt_abi_version.restype = c_int
        L.rt_build_id.restype = c_char_p
        L.rt_scene_chain_diag.argtypes = [c_void_p, c_void_p, c_int64]
        L.rt_scene_chain_diag.restype = c_int64
        _libs[path] = L
    return _libs[path]


def last_error(L=None) -> str:
    return ((L or lib()).rt_last_error() or b"").decode(errors="replace")


def build_id() -> str:
    """Hash of the loaded library's sources and flags (rt_hip.h: rt_build_id)."""
    return (lib().rt_build_id() or b"").decode()


class Scene:
    """An owned rt_flat_scene (host memory)."""

    def __init__(self, ptr, L=None):
        self._L = L or lib()
        if not ptr:
            raise RtcError(f"scene construction failed: {last_error(self._L)}")
        self._ptr = ptr

    @classmethod
    def preset(cls, scene_id: int, width: int = 0, spp: int = 0, max_depth: int = 0, image_dir: str | None = None,
               substitute_earth: bool | None = None) -> "Scene":
        """Reference driver scene `scene_id` (0-7) with the reference defaults (500 px, 100 spp,
        depth 50) unless overridden; aspect ratio comes from the scene (src/main.c).

        Scenes 3 and 7 read ``earthmap.jpg`` (baseline JPEG or binary PPM) from `image_dir`, else
        from the current directory, as the reference does.  The documented substitute picture
        (rtc/earth.py) is used only on request: ``substitute_earth=True``, or the
        environment variable ``RTC_SUBSTITUTE_EARTH=1`` (the test suite's and the benches' opt-in).
        No process state (working directory) is changed."""
        if substitute_earth is None:
            substitute_earth = os.environ.get("RTC_SUBSTITUTE_EARTH", "0") == "1"
        if image_dir is None and substitute_earth and int(scene_id) in (3, 7):
            image_dir = substitute_dir()
        d = image_dir.encode() if image_dir is not None else None
        L = lib()
        return cls(L.rt_scene_preset_in(int(scene_id), int(width), int(spp), int(max_depth), d), L)

    @property
    def ptr(self):
        return self._ptr

    @property
    def s(self) -> RtFlatScene:
        return self._ptr.contents

    @property
    def width(self) -> int:
        return self.s.camera.width

    @property
    def height(self) -> int:
        return self.s.camera.height

    @property
    def spp(self) -> int:
        return self.s.camera.spp

    @property
    def max_depth(self) -> int:
        return self.s.camera.max_depth

    @property
    def features(self) -> int:
        return self.s.features

    def counts(self) -> dict:
        return {n: getattr(self.s, n) for n in _COUNTS + ["stack_needed"]}

    def close(self):
        if self._ptr:
            self._L.rt_flat_free(self._ptr)
            self._ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_count() -> int:
    return lib().rt_device_count()


def render(scene: Scene, n_gpus: int = 1) -> np.ndarray:
    """Whole frame on the GPU(s) into a host (H, W, 3) uint8 array (what Camera_render does)."""
    out = np.empty((scene.height, scene.width, 3), dtype=np.uint8)
    L = lib()
    rc = L.rt_render(scene.ptr, int(n_gpus), out.ctypes.data)
    if rc != 0:
        raise RtcError(f"rt_render failed: {last_error(L)}")
    return out


def render_share(scene: Scene, share: int, n_shares: int, device: int = 0, out: np.ndarray | None = None) -> np.ndarray:
    """Rows j % n_shares == share of the frame on `device` (rt_render_share: what one process per GPU
    runs), written into those rows of `out` (a whole (H, W, 3) uint8 frame; a new zeroed one if None)."""
    if out is None:
        out = np.zeros((scene.height, scene.width, 3), dtype=np.uint8)
    if out.shape != (scene.height, scene.width, 3) or out.dtype != np.uint8 or not out.flags.c_contiguous:
        raise ValueError("out must be a C-contiguous (H, W, 3) uint8 array")
    L = lib()
    rc = L.rt_render_share(scene.ptr, int(share), int(n_shares), int(device), out.ctypes.data)
    if rc != 0:
        raise RtcError(f"rt_render_share failed: {last_error(L)}")
    return out


def release_cache() -> None:
    """Free the device scenes rt_render / rt_render_share keep between calls (rt_render_cache_release)."""
    lib().rt_render_cache_release()


def last_share_ms(share: int = 0) -> dict:
    """Host wall-clock phases of the last call's share `share` (rt_last_share_ms): setup (upload and
    allocations), run (launch to finish), d2h (rows back, completion check), total -- in ms."""
    buf = (c_double * 4)()
    if lib().rt_last_share_ms(int(share), buf) != 0:
        raise RtcError(f"rt_last_share_ms: {last_error()}")
    return dict(zip(("setup", "run", "d2h", "total"), (float(x) for x in buf)))


def last_kernel_ms(device: int = 0) -> float:
    return lib().rt_last_kernel_ms(device)


class DeviceScene:
    """Scene arrays resident in one GPU's HBM (rt_scene_upload)."""

    def __init__(self, scene: Scene, device: int = 0):
        self.scene = scene
        self.device = device
        self._L = lib()
        self._h = self._L.rt_scene_upload(scene.ptr, int(device))
        if not self._h:
            raise RtcError(f"rt_scene_upload failed: {last_error(self._L)}")

    def render_rows_async(self, row0: int, row_stride: int, n_rows: int, d_out_ptr: int, stream_ptr: int = 0):
        rc = self._L.rt_render_rows_async(self._h, int(row0), int(row_stride), int(n_rows),
                                          c_void_p(int(d_out_ptr)), c_void_p(int(stream_ptr)))
        if rc != 0:
            raise RtcError(f"rt_render_rows_async failed: {last_error(self._L)}")

    def check(self):
        """Wait for this scene's launches and raise RtcError if any work item never finished
        (rt_scene_check): the rows written are then not a valid frame."""
        if self._L.rt_scene_check(self._h) != 0:
            raise RtcError(f"rt_scene_check: {last_error(self._L)}")

    def last_launch_ms(self) -> float:
        """Duration of the last frame launch (excludes the cost pre-pass); call after it completed."""
        return float(self._L.rt_scene_last_launch_ms(self._h))

    def launch_history(self, n: int) -> list:
        """Frame-kernel milliseconds of the last min(n, 64) launches, oldest first (rt_scene_launch_history;
        call after they completed)."""
        if not hasattr(self._L, "rt_scene_launch_history"):
            return []
        buf = (c_double * max(int(n), 1))()
        m = self._L.rt_scene_launch_history(self._h, buf, int(n))
        if m < 0:
            raise RtcError(f"rt_scene_launch_history: {last_error(self._L)}")
        return [float(buf[k]) for k in range(m)]

    @property
    def kernel_name(self) -> str:
        """The kernel rt_render_rows_async launches for this scene (rocprofv3's name for it)."""
        return (self._L.rt_scene_kernel(self._h) or b"").decode()

    def chain_diag(self, max_rows: int) -> np.ndarray:
        """Item rows of the last chain launch (rt_hip.h: rt_scene_chain_diag; diagnostic build with
        RT_PX_TIME=1 at upload): (items, 16) uint32."""
        rows = np.zeros((max_rows, 16), np.uint32)
        m = self._L.rt_scene_chain_diag(self._h, rows.ctypes.data, int(max_rows))
        if m < 0:
            raise RtcError(f"rt_scene_chain_diag: {last_error(self._L)}")
        return rows[:min(m, max_rows)]

    def close(self):
        if self._h:
            self._L.rt_scene_release(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def box_identity(device: int = 0) -> dict:
    """Which machine and GPU a measurement ran on (chain-mode timings differ between
    boxes, so every probe and bench line names its box): host name, the GPU's UUID and PCI location
    as the HIP runtime reports them, and the board serial from rocm-smi when it answers."""
    import socket
    import subprocess

    ident = {"host": socket.gethostname()}
    torch = sys.modules.get("torch")
    if torch is not None:
        try:
            p = torch.cuda.get_device_properties(device)
            ident["gpu_uuid"] = str(getattr(p, "uuid", ""))
            ident["pci"] = f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:" \
                           f"{getattr(p, 'pci_device_id', 0):02x}"
        except Exception:  # no GPU visible: host only
            pass
    try:
        out = subprocess.run(["rocm-smi", "--showserial", "--json"], capture_output=True, text=True, timeout=20).stdout
        import json

        cards = json.loads(out) if out.strip().startswith("{") else {}
        serials = [v.get("Serial Number") for v in cards.values() if isinstance(v, dict) and v.get("Serial Number")]
        if serials:
            ident["smi_serial"] = serials[0] if len(serials) == 1 else serials
    except Exception:
        pass
    return ident


def rows_of(height: int, rank: int, world: int):
    """Interleaved row partition j % world == rank: (row0, stride, n_rows)."""
    n = (height - rank + world - 1) // world if rank < height else 0
    return rank, world, max(n, 0)


def assemble_frame(parts, height: int, world: int) -> np.ndarray:
    """Inverse of rows_of: parts[r] holds rank r's rows (possibly padded); returns (H, W, 3)."""
    first = np.asarray(parts[0])
    frame = np.empty((height,) + first.shape[1:], dtype=first.dtype)
    for r, p in enumerate(parts):
        row0, stride, n = rows_of(height, r, world)
        frame[row0::stride][:n] = np.asarray(p)[:n]
    return frame


def diag_arith(fn: int, start: int, count: int, seed: int = 0, device: int = 0) -> int:
    """Mismatch count of the Book-1 kernel's exact arithmetic cores vs the compiler's sqrtf / '/':
    0 sqrt over float bit patterns [start, start+count), 1 division on hashed pairs, 2 sphere-hit
    outcome on hashed rays (rt_hip.h: rt_diag_arith)."""
    out = ctypes.c_ulonglong(0)
    rc = lib().rt_diag_arith(int(fn), int(start), int(count), int(seed), ctypes.byref(out), int(device))
    if rc != 0:
        raise RtcError(f"rt_diag_arith failed: {last_error()}")
    return int(out.value)


def diag_libm(fn: int, x: np.ndarray, device: int = 0) -> np.ndarray:
    """Evaluate the device libm port on float32 inputs: 0 sincosf, 1 powf(x,5), 2 logf, 3 sinf,
    4 atan2f over interleaved (y, x) pairs, 5 acosf."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(2 * x.size if fn == 0 else x.size, dtype=np.float32)
    rc = lib().rt_diag_libm(int(fn), x.ctypes.data, out.ctypes.data, x.size, int(device))
    if rc != 0:
        raise RtcError(f"rt_diag_libm failed: {last_error()}")
    return out[: x.size // 2] if fn == 4 else out
