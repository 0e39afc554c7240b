"""How long a large device allocation takes on this box, fresh and after freeing one of the same size (the
record arena of a chain launch is up to 24 GiB).  Uses the system HIP runtime directly.
    python scripts/alloc_probe.py [GIB ...]        e.g.  2 8 24"""
import ctypes
import sys
import time

hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipFree.argtypes = [ctypes.c_void_p]
hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
hip.hipDeviceSynchronize.argtypes = []


def ms(f):
    t0 = time.perf_counter()
    rc = f()
    hip.hipDeviceSynchronize()
    return (time.perf_counter() - t0) * 1e3, rc


hip.hipSetDevice(0)
hip.hipDeviceSynchronize()
for gib in [float(x) for x in (sys.argv[1:] or ["2", "8", "24"])]:
    size = int(gib * (1 << 30))
    for rep in range(3):
        p = ctypes.c_void_p()
        t_alloc, rc = ms(lambda: hip.hipMalloc(ctypes.byref(p), size))
        if rc != 0:
            print(f"{gib} GiB: hipMalloc rc {rc}", flush=True)
            break
        t_set, _ = ms(lambda: hip.hipMemset(p, 0xff, size))
        t_free, _ = ms(lambda: hip.hipFree(p))
        print(f"{gib:5.1f} GiB rep {rep}: hipMalloc {t_alloc:8.1f} ms  memset {t_set:7.1f} ms ({size / t_set / 1e6:.0f} GB/s)  "
              f"hipFree {t_free:7.1f} ms", flush=True)
