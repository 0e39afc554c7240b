#!/usr/bin/env python3
"""Fixtures for worlds built through the reference's public C API (tests/native/api_worlds.c).

Runs oracle/_ref/api_worlds_ref -- api_worlds.c linked against the reference's own src/*.c (strict
gcc -std=c11 -O2, oracle/Makefile) -- once per world and writes tests/golden/api/world<N>.rgb.gz plus
tests/golden/api/manifest.json (name, size, sha256 of the raw RGB).  Run in the build container,
where /root/reference exists: `make -C oracle && python tests/golden/make_api_golden.py`.
"""
import gzip
import hashlib
import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref", "api_worlds_ref")
OUT = os.path.join(HERE, "api")
NAMES = ["surface_normal", "hollow_glass", "metal_fuzz_dof", "quads_xform_medium_light_dof", "depth100_mirror",
         "one_px_wide", "flat_list_120", "bvh_depth100", "bvh_1100_global_items_64spp", "bvh_1100_global_items_16spp",
         "boxes_1000_preorder_past_lds"]


def main():
    os.makedirs(OUT, exist_ok=True)
    man = {"generator": "oracle/_ref/api_worlds_ref: tests/native/api_worlds.c linked to the reference's own "
                        "src/*.c (gcc -std=c11 -O2 -fopenmp, glibc 2.35 libm)", "worlds": {}}
    with tempfile.TemporaryDirectory() as td:
        for wid, name in enumerate(NAMES):
            path = os.path.join(td, "o.rgb")
            r = subprocess.run([REF, str(wid), path], check=True, capture_output=True, text=True, cwd=td)
            w, h = (int(x) for x in r.stdout.split())
            data = open(path, "rb").read()
            assert len(data) == w * h * 3
            fname = f"world{wid}.rgb.gz"
            with gzip.GzipFile(os.path.join(OUT, fname), "wb", mtime=0) as f:
                f.write(data)
            man["worlds"][str(wid)] = {"name": name, "width": w, "height": h, "file": fname,
                                       "sha256": hashlib.sha256(data).hexdigest()}
            print(wid, name, w, h, man["worlds"][str(wid)]["sha256"][:16])
    json.dump(man, open(os.path.join(OUT, "manifest.json"), "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
