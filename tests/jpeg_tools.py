"""TEST INFRASTRUCTURE: a minimal baseline JPEG encoder (4:4:4 or grey, one quantisation table, one
Huffman table pair built from the symbols the image uses) that can write the components either in
one interleaved scan or in separate, non-interleaved scans (ITU T.81 §A.2.2) -- the layout Pillow
cannot write.  Decoders must give identical pixels for both layouts of the same coefficients."""
import math

import numpy as np

# zigzag index -> natural (row-major) index in the 8x8 block (T.81 Figure A.6)
ZIGZAG = sorted(range(64), key=lambda n: (n // 8 + n % 8, (n % 8) if (n // 8 + n % 8) % 2 == 0 else (n // 8)))
_C = np.array([[(math.sqrt(0.5) if u == 0 else 1.0) * math.cos((2 * x + 1) * u * math.pi / 16) for x in range(8)]
               for u in range(8)]) / 2.0  # orthonormal DCT-II basis


def _planes(img):
    """uint8 HxWx3 RGB (or HxW grey) -> list of float planes (JFIF YCbCr)."""
    if img.ndim == 2:
        return [img.astype(np.float64)]
    r, g, b = (img[..., k].astype(np.float64) for k in range(3))
    y = 0.299 * r + 0.587 * g + 0.114 * b
    cb = -0.168736 * r - 0.331264 * g + 0.5 * b + 128.0
    cr = 0.5 * r - 0.418688 * g - 0.081312 * b + 128.0
    return [np.clip(np.rint(p), 0, 255) for p in (y, cb, cr)]


def _blocks(plane, q):
    """Quantised coefficients in zigzag order, blocks in raster order (edges replicated)."""
    h, w = plane.shape
    H, W = -(-h // 8) * 8, -(-w // 8) * 8
    p = np.pad(plane, ((0, H - h), (0, W - w)), mode="edge") - 128.0
    out = []
    for by in range(0, H, 8):
        for bx in range(0, W, 8):
            f = _C @ p[by:by + 8, bx:bx + 8] @ _C.T
            z = np.rint(f.reshape(64) / q).astype(int)
            out.append([int(z[n]) for n in ZIGZAG])
    return out


def _cat(v):
    return 0 if v == 0 else int(abs(v)).bit_length()


def _symbols(blocks):
    """Per block: [(dc category, bits)], then AC (run/size symbol, bits) list; DC predictors per component."""
    dc_syms, ac_syms, coded = set(), set(), []
    prev = 0
    for z in blocks:
        d = z[0] - prev
        prev = z[0]
        s = _cat(d)
        dc_syms.add(s)
        items = [("dc", s, d)]
        run = 0
        last = max([k for k in range(1, 64) if z[k] != 0], default=0)
        for k in range(1, last + 1):
            if z[k] == 0:
                run += 1
                continue
            while run > 15:
                items.append(("ac", 0xF0, 0))
                ac_syms.add(0xF0)
                run -= 16
            sym = (run << 4) | _cat(z[k])
            ac_syms.add(sym)
            items.append(("ac", sym, z[k]))
            run = 0
        if last < 63:
            items.append(("ac", 0x00, 0))
            ac_syms.add(0x00)
        coded.append(items)
    return dc_syms, ac_syms, coded


def _table(symbols):
    """All symbols at one code length (8 bits: at most 255 symbols, so no all-ones code)."""
    vals = sorted(symbols)
    assert len(vals) <= 255
    bits = [0] * 16
    bits[7] = len(vals)
    return bits, vals, {v: (k, 8) for k, v in enumerate(vals)}


class _Bits:
    def __init__(self):
        self.out, self.acc, self.n = bytearray(), 0, 0

    def put(self, v, n):
        for k in range(n - 1, -1, -1):
            self.acc = (self.acc << 1) | ((v >> k) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)  # byte stuffing
                self.acc, self.n = 0, 0

    def flush(self):
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)  # pad with ones
        return bytes(self.out)


def _magnitude(v, s):
    return v if v >= 0 else v + (1 << s) - 1


def encode(img, interleaved, qstep=3):
    """Baseline JPEG bytes of `img` (uint8 HxWx3 RGB or HxW grey), 4:4:4, component ids 1..n."""
    planes = _planes(np.asarray(img))
    h, w = planes[0].shape
    nc = len(planes)
    comp_blocks = [_blocks(p, qstep) for p in planes]
    dc_all, ac_all, coded = set(), set(), []
    for blocks in comp_blocks:
        dcs, acs, items = _symbols(blocks)
        dc_all |= dcs
        ac_all |= acs
        coded.append(items)
    dcb, dcv, dcc = _table(dc_all)
    acb, acv, acc = _table(ac_all)

    def seg(marker, payload):
        return bytes([0xFF, marker]) + (len(payload) + 2).to_bytes(2, "big") + payload

    out = bytearray(b"\xff\xd8")
    out += seg(0xE0, b"JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00")
    out += seg(0xDB, bytes([0]) + bytes([qstep] * 64))
    sof = bytes([8]) + h.to_bytes(2, "big") + w.to_bytes(2, "big") + bytes([nc])
    for k in range(nc):
        sof += bytes([k + 1, 0x11, 0])
    out += seg(0xC0, sof)
    out += seg(0xC4, bytes([0x00]) + bytes(dcb) + bytes(dcv) + bytes([0x10]) + bytes(acb) + bytes(acv))

    def scan(comps):
        b = _Bits()
        nblk = len(coded[comps[0]])
        for i in range(nblk):  # 4:4:4: an MCU is one block of each component of the scan
            for k in comps:
                for kind, sym, v in coded[k][i]:
                    code, n = (dcc if kind == "dc" else acc)[sym]
                    b.put(code, n)
                    s = sym if kind == "dc" else sym & 15
                    if s:
                        b.put(_magnitude(v, s), s)
        hdr = bytes([len(comps)]) + b"".join(bytes([k + 1, 0x00]) for k in comps) + bytes([0, 63, 0])
        return seg(0xDA, hdr) + b.flush()

    if interleaved:
        out += scan(list(range(nc)))
    else:
        for k in range(nc):
            out += scan([k])
    out += b"\xff\xd9"
    return bytes(out)
