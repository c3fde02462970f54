"""ctypes binding of the CPU oracle (oracle/gz_oracle.c) and fixture readers.

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libgz_oracle.so")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "guetzli_ref")

_lib = None


class CoeffData(ctypes.Structure):
    _fields_ = [("idx", ctypes.c_int), ("block_err", ctypes.c_float)]


COEFF_DTYPE = np.dtype([("idx", "<i4"), ("block_err", "<f4")])


def build_oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True,
                       stdout=subprocess.DEVNULL)


def lib():
    global _lib
    if _lib is None:
        build_oracle()
        L = ctypes.CDLL(ORACLE_SO)
        P = np.ctypeslib.ndpointer
        f32 = P(np.float32, flags="C")
        f64 = P(np.float64, flags="C")
        u8 = P(np.uint8, flags="C")
        i16 = P(np.int16, flags="C")
        i32 = P(np.int32, flags="C")
        sz = ctypes.c_size_t
        L.gzo_init.restype = None
        L.gzo_block_idct.argtypes = [i16, u8]
        L.gzo_coeffs_to_srgb.argtypes = [ctypes.c_int, ctypes.c_int, i16, u8]
        L.gzo_srgb_to_linear_planes.argtypes = [ctypes.c_int, ctypes.c_int, u8, f32]
        L.gzo_blur.argtypes = [sz, sz, f32, ctypes.c_float, ctypes.c_float]
        L.gzo_opsin_dynamics.argtypes = [sz, sz, f32]
        L.gzo_mask_high_intensity_change.argtypes = [sz, sz, f32, f32, f32, f32]
        L.gzo_mask.argtypes = [sz, sz, f32, f32, f32, f32]
        L.gzo_diffmap.argtypes = [sz, sz, f32, f32, f32, ctypes.c_void_p]
        L.gzo_diffmap.restype = ctypes.c_int
        L.gzo_compare.argtypes = [ctypes.c_int, ctypes.c_int, u8, i16, f32]
        L.gzo_compare.restype = ctypes.c_float
        L.gzo_block_diff_double.argtypes = [f64, f64, f64, f64, f64]
        L.gzo_sort_pairs.argtypes = [i32, f32, ctypes.c_int]
        L.gzo_block_zeroing_orders.argtypes = [ctypes.c_int, ctypes.c_int, u8, f32, i16, i16,
                                               ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_void_p]
        L.gzo_compare_block.argtypes = [ctypes.c_int, ctypes.c_int, u8, f32, ctypes.c_int, i16]
        L.gzo_compare_block.restype = ctypes.c_double
        L.gzo_srgb8_to_linear.argtypes = [ctypes.c_int]
        L.gzo_srgb8_to_linear.restype = ctypes.c_double
        L.gzo_init()
        _lib = L
    return _lib


class Stages(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("mhic0", "mhic1", "edge", "block_dc", "block_ac", "block_ac_lf", "mask",
                 "mask_dc", "combined")]


def fixture_cases():
    return sorted(d[len("stages_"):] for d in os.listdir(GOLDEN) if d.startswith("stages_"))


class Fixture:
    """Reader for one tests/golden/stages_<case>/ directory."""

    def __init__(self, case):
        self.dir = os.path.join(GOLDEN, "stages_" + case)
        meta = {}
        for line in open(os.path.join(self.dir, "meta.txt")):
            k, v = line.split()
            meta[k] = v
        self.meta = meta
        self.w, self.h = int(meta["w"]), int(meta["h"])
        self.target = float(meta["target"])
        self.bw, self.bh = (self.w + 7) // 8, (self.h + 7) // 8
        self.nb = self.bw * self.bh
        self.rw, self.rh = (self.w + 2) // 3, (self.h + 2) // 3

    def path(self, name):
        return os.path.join(self.dir, name)

    def f32(self, name):
        return np.fromfile(self.path(name), dtype=np.float32)

    def planes(self, name):
        return self.f32(name).reshape(3, self.h, self.w)

    def i16(self, name):
        return np.fromfile(self.path(name), dtype=np.int16)

    def rgb(self):
        return np.fromfile(self.path("input.rgb"), dtype=np.uint8)

    def zero_order(self, variant=None):
        """zero_order.bin, or the (lookahead, comp_mask, new_model) variant
        zero_order_la<L>_m<M>_nm<N>.bin (make_fixtures.py zero-variants)."""
        name = "zero_order.bin" if variant is None else "zero_order_la%d_m%d_nm%d.bin" % variant
        return np.fromfile(self.path(name), dtype=COEFF_DTYPE).reshape(self.nb, 192)


# (lookahead, comp_mask, new_zeroing_model) of the committed zeroing variants
ZERO_VARIANTS = [(3, 7, 1), (1, 7, 1), (2, 7, 1), (3, 1, 1), (3, 6, 1), (3, 7, 0), (2, 6, 0)]
