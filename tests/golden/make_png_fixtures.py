#!/usr/bin/env python3
"""PNG-input fixtures: small PNG files of every color type / bit depth the
reference CLI's reader accepts (guetzli/guetzli.cc:51-156, libpng with
PACKING | EXPAND | STRIP_16, alpha blended on black), interlaced and not,
with tRNS, several IDAT chunks and every row filter; plus bees.png (the
reference's own test image) and damaged files.  The expected RGB of each
is what the REFERENCE's ReadPNG returns (oracle/_ref/png_driver, compiled
from /root/reference by oracle/Makefile): its sha256, or "fail".

The PNG files are written by the small encoder below (zlib from the Python
standard library), so that interlacing, filters and odd bit depths are
under our control.  Writes tests/golden/png/*.png and the "png" section of
tests/golden/manifest.json.

  python tests/golden/make_png_fixtures.py        (needs oracle/_ref/png_driver)
"""
import hashlib
import json
import os
import random
import shutil
import struct
import subprocess
import sys
import tempfile
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "png")
DRIVER = os.path.join(ROOT, "oracle", "_ref", "png_driver")
CHANNELS = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}
ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2),
         (0, 1, 1, 2)]


def chunk(typ, data, bad_crc=False):
    crc = zlib.crc32(typ + data) & 0xffffffff
    if bad_crc:
        crc ^= 1
    return struct.pack(">I", len(data)) + typ + data + struct.pack(">I", crc)


def pack_row(samples, depth):
    """Samples (ints) of one row -> bytes at `depth` bits per sample."""
    if depth == 8:
        return bytes(samples)
    if depth == 16:
        return b"".join(struct.pack(">H", v) for v in samples)
    out, acc, nbits = bytearray(), 0, 0
    for v in samples:
        acc = (acc << depth) | v
        nbits += depth
        if nbits == 8:
            out.append(acc)
            acc, nbits = 0, 0
    if nbits:
        out.append(acc << (8 - nbits))
    return bytes(out)


def filter_row(raw, prev, bpp, ftype):
    out = bytearray([ftype])
    for i, x in enumerate(raw):
        a = raw[i - bpp] if i >= bpp else 0
        b = prev[i] if prev is not None else 0
        c = prev[i - bpp] if prev is not None and i >= bpp else 0
        if ftype == 0:
            p = 0
        elif ftype == 1:
            p = a
        elif ftype == 2:
            p = b
        elif ftype == 3:
            p = (a + b) // 2
        else:
            pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
            p = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
        out.append((x - p) & 0xff)
    return bytes(out)


def encode(w, h, ct, depth, pixels, interlace=False, plte=None, trns=None, rng=None,
           idat_parts=1, level=6):
    """pixels[y][x] = tuple of channel samples."""
    ch = CHANNELS[ct]
    bpp = max(1, ch * depth // 8)
    raw = bytearray()

    def scanlines(xs, ys):
        prev = None
        for y in ys:
            samples = [s for x in xs for s in pixels[y][x]]
            row = pack_row(samples, depth)
            raw.extend(filter_row(row, prev, bpp, rng.randrange(5)))
            prev = row

    if interlace:
        for x0, y0, dx, dy in ADAM7:
            xs, ys = list(range(x0, w, dx)), list(range(y0, h, dy))
            if xs and ys:
                scanlines(xs, ys)
    else:
        scanlines(list(range(w)), list(range(h)))
    z = zlib.compress(bytes(raw), level)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ct, 0, 0,
                                                                 1 if interlace else 0))
    if plte is not None:
        png += chunk(b"PLTE", bytes(v for rgb in plte for v in rgb))
    if trns is not None:
        png += chunk(b"tRNS", trns)
    step = (len(z) + idat_parts - 1) // idat_parts
    for i in range(0, len(z), step):
        png += chunk(b"IDAT", z[i:i + step])
    return png + chunk(b"IEND", b"")


def cases():
    rng = random.Random(20261016)
    out = []

    def img(w, h, ch, maxv):
        return [[tuple(rng.randint(0, maxv) for _ in range(ch)) for _ in range(w)] for _ in range(h)]

    for ct, depths in ((0, (1, 2, 4, 8, 16)), (2, (8, 16)), (3, (1, 2, 4, 8)), (4, (8, 16)),
                       (6, (8, 16))):
        for depth in depths:
            for interlace in (False, True):
                w, h = (37, 23) if not interlace else (29, 19)
                maxv = (1 << depth) - 1
                plte = trns = None
                if ct == 3:
                    n = min(256, 1 << depth)
                    plte = [(rng.randrange(256), rng.randrange(256), rng.randrange(256)) for _ in range(n)]
                    px = img(w, h, 1, n - 1)
                else:
                    px = img(w, h, CHANNELS[ct], maxv)
                name = "ct%d_d%d%s" % (ct, depth, "_i" if interlace else "")
                out.append((name, encode(w, h, ct, depth, px, interlace, plte, None, rng,
                                         idat_parts=3)))
                # tRNS: a colour key for gray / RGB (hit by some pixels), palette alphas
                if ct in (0, 2):
                    key = px[3][5]
                    trns = b"".join(struct.pack(">H", v) for v in key)
                    out.append((name + "_trns", encode(w, h, ct, depth, px, interlace, None, trns,
                                                       rng)))
                elif ct == 3:
                    trns = bytes(rng.randrange(256) for _ in range(min(len(plte), 5)))
                    out.append((name + "_trns", encode(w, h, ct, depth, px, interlace, plte, trns,
                                                       rng)))
    # stored (uncompressed) deflate blocks, one-pixel and one-row images
    out.append(("rgb_stored", encode(16, 9, 2, 8, img(16, 9, 3, 255), rng=rng, level=0)))
    out.append(("rgb_1x1", encode(1, 1, 2, 8, img(1, 1, 3, 255), rng=rng)))
    out.append(("gray_1x7_i", encode(1, 7, 0, 4, img(1, 7, 1, 15), True, rng=rng)))
    out.append(("rgba_40x1", encode(40, 1, 6, 8, img(40, 1, 4, 255), rng=rng)))
    # damaged: a bad IDAT CRC, a truncated stream
    good = encode(12, 10, 2, 8, img(12, 10, 3, 255), rng=rng)
    k = good.index(b"IDAT")
    crc_at = k + 4 + struct.unpack(">I", good[k - 4:k])[0]
    bad = good[:crc_at] + bytes([good[crc_at] ^ 0x55]) + good[crc_at + 1:]
    out.append(("bad_crc", bad))
    out.append(("truncated", good[:len(good) // 2]))
    # a header promising 30000 x 30000 RGB (2.7 GB of scanlines) over a few
    # bytes of IDAT: libpng runs out of image data; a reader must not size its
    # buffers from the header alone
    huge = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", 30000, 30000, 8, 2, 0, 0, 0))
            + chunk(b"IDAT", zlib.compress(b"\x00" * 4000)) + chunk(b"IEND", b""))
    out.append(("huge_ihdr", huge))
    return out


def main():
    if not os.path.exists(DRIVER):
        sys.exit("build oracle/_ref/png_driver first (make -C oracle)")
    os.makedirs(OUT, exist_ok=True)
    entries = {}
    files = cases()
    shutil.copy("/root/reference/tests/bees.png", os.path.join(OUT, "bees.png"))
    files_on_disk = [(n, None) for n in ["bees"]] + files
    with tempfile.TemporaryDirectory() as td:
        for name, data in files_on_disk:
            path = os.path.join(OUT, name + ".png")
            if data is not None:
                with open(path, "wb") as f:
                    f.write(data)
            rgb_path = os.path.join(td, name + ".rgb")
            r = subprocess.run([DRIVER, path, rgb_path], capture_output=True, text=True)
            e = {"file": "png/%s.png" % name}
            if r.returncode == 0:
                w, h = map(int, r.stdout.split())
                rgb = open(rgb_path, "rb").read()
                e.update(w=w, h=h, rgb_sha256=hashlib.sha256(rgb).hexdigest())
            else:
                e["fail"] = True
            entries[name] = e
    mpath = os.path.join(HERE, "manifest.json")
    m = json.load(open(mpath))
    m["png"] = entries
    json.dump(m, open(mpath, "w"), indent=1, sort_keys=True)
    print("%d PNG fixtures (%d fail)" % (len(entries), sum(1 for e in entries.values() if e.get("fail"))))


if __name__ == "__main__":
    main()
