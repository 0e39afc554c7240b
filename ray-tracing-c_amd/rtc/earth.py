"""The documented substitute for the reference's earth texture.

Scenes 3 and 7 of the reference driver load ``Image_new("earthmap.jpg")`` (src/main.c:104, :243)
through stb_image, from the current directory.  The reference repository does not ship that file,
and the stb submodule is un-vendored.  Every render of those scenes here (the product library,
the reference build in oracle/_ref, the goldens) therefore reads the same synthetic picture,
written as a binary PPM file under the reference's file name: stb_image and this library both
detect the format from the file's content, not its name.

Picture: 1024 x 512 RGB8, R = 255*i/1023, G = 255*j/511, B = (i ^ j) & 255 (row j top to bottom).
Synthetic input data; no compute of the render path lives here.
"""
from __future__ import annotations

import os

import numpy as np

WIDTH, HEIGHT = 1024, 512
FILE_NAME = "earthmap.jpg"


def substitute_pixels() -> np.ndarray:
    i = np.arange(WIDTH, dtype=np.int64)[None, :]
    j = np.arange(HEIGHT, dtype=np.int64)[:, None]
    img = np.empty((HEIGHT, WIDTH, 3), dtype=np.uint8)
    img[..., 0] = (i * 255) // (WIDTH - 1)
    img[..., 1] = (j * 255) // (HEIGHT - 1)
    img[..., 2] = (i ^ j) & 255
    return img


def write_substitute(directory: str) -> str:
    """Write ``earthmap.jpg`` (binary PPM content) into `directory`; returns its path."""
    path = os.path.join(directory, FILE_NAME)
    data = b"P6\n%d %d\n255\n" % (WIDTH, HEIGHT) + substitute_pixels().tobytes()
    if not (os.path.exists(path) and os.path.getsize(path) == len(data) and open(path, "rb").read() == data):
        tmp = path + ".%d.tmp" % os.getpid()
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
    return path
