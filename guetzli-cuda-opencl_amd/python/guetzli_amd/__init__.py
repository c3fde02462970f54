"""Python host mirror of the reference's encode / comparator API.

Thin ctypes layer over the C ABI in include/guetzli_hip.h (libguetzli_hip.so,
built from guetzli-cuda-opencl_amd/csrc).  Names follow the reference:

  process(rgb, w, h, params)        guetzli::Process          processor.h:62-64
  Params                            guetzli::Params           processor.h:34-42
  butteraugli_score_for_quality(q)  ButteraugliScoreForQuality quality.cc:78-87
  ButteraugliComparator             guetzli::ButteraugliComparator
                                    butteraugli_comparator.h:33-81

There is no CPU fallback: every compute call goes through the HIP library and
raises GuetzliError when the library or a GPU is unavailable.
"""
import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(os.path.dirname(_HERE))
# GZ_LIB_PATH: an alternative build of the same library (A/B timing tools)
LIB_PATH = os.environ.get("GZ_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libguetzli_hip.so")

GZ_OK = 0
GZ_ERR_INVALID_ARG, GZ_ERR_DEVICE, GZ_ERR_OUT_OF_MEMORY, GZ_ERR_UNSUPPORTED, GZ_ERR_INTERNAL = 1, 2, 3, 4, 5
_STATUS = {1: "invalid argument", 2: "device error", 3: "out of memory", 4: "unsupported",
           5: "internal error"}


class GuetzliError(RuntimeError):
    def __init__(self, status, message):
        super().__init__("%s (%s)" % (message, _STATUS.get(status, status)))
        self.status = status


class _CoeffData(ctypes.Structure):
    _fields_ = [("idx", ctypes.c_int), ("block_err", ctypes.c_float)]


class _Params(ctypes.Structure):
    _fields_ = [("butteraugli_target", ctypes.c_float), ("clear_metadata", ctypes.c_int),
                ("try_420", ctypes.c_int), ("force_420", ctypes.c_int),
                ("use_silver_screen", ctypes.c_int), ("zeroing_greedy_lookahead", ctypes.c_int),
                ("new_zeroing_model", ctypes.c_int)]


class _Stats(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int), ("iterations_up", ctypes.c_int),
                ("iterations_down", ctypes.c_int), ("compares", ctypes.c_int),
                ("seconds_compare", ctypes.c_double), ("seconds_zeroing", ctypes.c_double),
                ("seconds_total", ctypes.c_double), ("seconds_setup", ctypes.c_double),
                ("seconds_write", ctypes.c_double), ("seconds_quantize", ctypes.c_double),
                ("seconds_backend", ctypes.c_double)]


_STAGE_FIELDS = ("cand_linear", "cand_xyb", "mhic0", "mhic1", "edge", "block_dc", "block_ac",
                 "block_ac_lf", "mask", "mask_dc", "combined", "distmap")


class _Stages(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in _STAGE_FIELDS]


COEFF_DTYPE = np.dtype([("idx", "<i4"), ("block_err", "<f4")])

# Every symbol include/guetzli_hip.h declares.
EXPORTED_SYMBOLS = (
    "gz_last_error", "gz_build_info", "gz_device_count", "gz_params_init",
    "gz_butteraugli_score_for_quality", "gz_free", "gz_process_rgb", "gz_process_rgb_device",
    "gz_comparator_create", "gz_comparator_destroy", "gz_comparator_compare",
    "gz_comparator_compare_stages", "gz_comparator_compare_stages_production", "gz_comparator_compare_420",
    "gz_comparator_block_max", "gz_comparator_distance_ok",
    "gz_comparator_score_output_size", "gz_comparator_start_block_comparisons",
    "gz_comparator_block_zeroing_orders", "gz_synthetic_frame", "gz_rgb_to_coeffs",
    "gz_block_error_adjustment_weights", "gz_engine_pool_trim", "gz_engine_pool_idle_bytes",
    "gz_comparator_original_coeffs", "gz_comparator_write_jpeg", "gz_write_jpeg_host",
    "gz_profile_enable", "gz_profile_reset", "gz_profile_get", "gz_profile_names",
    "gz_last_process_detail", "gz_process_rgb_strips", "gz_strip_layout",
    "gz_collectives_selftest", "gz_process_jpeg", "gz_jpeg_decode", "gz_comparator_distmap",
    "gz_comparator_compare_blocks", "gz_png_decode", "gz_comparator_compare_rgb",
    "gz_comparator_compare_blocks_rgb", "gz_rccl_unique_id", "gz_rccl_create", "gz_rccl_destroy",
    "gz_rccl_library",
)

_lib = None


# int allgather(void* ctx, const void* send, size_t bytes, void* recv)
_ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                              ctypes.c_void_p)


class _Collectives(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("rank", ctypes.c_int), ("world", ctypes.c_int),
                ("allgather", _ALLGATHER)]


def lib():
    """Load libguetzli_hip.so (raises GuetzliError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GuetzliError(2, "libguetzli_hip.so not built at %s (run __graft_entry__.build())"
                           % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, f32, u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_uint64
    L.gz_last_error.restype = ctypes.c_char_p
    L.gz_build_info.restype = ctypes.c_char_p
    L.gz_device_count.restype = i32
    L.gz_params_init.argtypes = [ctypes.POINTER(_Params)]
    L.gz_butteraugli_score_for_quality.argtypes = [ctypes.c_double]
    L.gz_butteraugli_score_for_quality.restype = ctypes.c_double
    L.gz_free.argtypes = [vp]
    L.gz_process_jpeg.argtypes = [i32, ctypes.POINTER(_Params), vp, ctypes.c_size_t,
                                  ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t),
                                  ctypes.POINTER(_Stats)]
    L.gz_png_decode.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(i32), ctypes.POINTER(i32),
                                ctypes.POINTER(vp)]
    L.gz_png_decode.restype = i32
    L.gz_jpeg_decode.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(i32), ctypes.POINTER(i32),
                                 ctypes.POINTER(i32), ctypes.POINTER(vp),
                                 ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(vp)]
    for name in ("gz_process_rgb", "gz_process_rgb_device"):
        fn = getattr(L, name)
        fn.argtypes = [i32, ctypes.POINTER(_Params), vp, i32, i32, ctypes.POINTER(vp),
                       ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(_Stats)]
        fn.restype = i32
    L.gz_comparator_create.argtypes = [i32, i32, i32, vp, f32, ctypes.POINTER(vp)]
    L.gz_comparator_create.restype = i32
    L.gz_comparator_destroy.argtypes = [vp]
    L.gz_comparator_compare.argtypes = [vp, vp, ctypes.POINTER(f32)]
    L.gz_comparator_compare.restype = i32
    L.gz_comparator_compare_stages.argtypes = [vp, vp, ctypes.POINTER(_Stages), ctypes.POINTER(f32)]
    L.gz_comparator_compare_stages.restype = i32
    L.gz_comparator_compare_stages_production.argtypes = [vp, vp, ctypes.POINTER(_Stages),
                                                          ctypes.POINTER(f32)]
    L.gz_comparator_compare_stages_production.restype = i32
    L.gz_comparator_compare_420.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.POINTER(f32)]
    L.gz_comparator_compare_420.restype = i32
    L.gz_comparator_distmap.argtypes = [vp, vp]
    L.gz_comparator_distmap.restype = i32
    L.gz_comparator_compare_blocks.argtypes = [vp, i32, vp, vp, vp]
    L.gz_comparator_compare_blocks.restype = i32
    L.gz_comparator_block_max.argtypes = [vp, vp]
    L.gz_comparator_block_max.restype = i32
    L.gz_comparator_distance_ok.argtypes = [vp, ctypes.c_double]
    L.gz_comparator_distance_ok.restype = i32
    L.gz_comparator_score_output_size.argtypes = [vp, i32]
    L.gz_comparator_score_output_size.restype = ctypes.c_double
    L.gz_comparator_start_block_comparisons.argtypes = [vp, vp]
    L.gz_comparator_start_block_comparisons.restype = i32
    L.gz_comparator_block_zeroing_orders.argtypes = [vp, vp, vp, i32, f32, i32, i32, vp]
    L.gz_comparator_block_zeroing_orders.restype = i32
    L.gz_block_error_adjustment_weights.argtypes = [i32, i32, f32, i32, i32, ctypes.c_double, i32,
                                                    i32, vp, vp]
    L.gz_block_error_adjustment_weights.restype = i32
    L.gz_engine_pool_trim.argtypes = [ctypes.c_size_t]
    L.gz_engine_pool_trim.restype = ctypes.c_size_t
    L.gz_engine_pool_idle_bytes.argtypes = []
    L.gz_engine_pool_idle_bytes.restype = ctypes.c_size_t
    L.gz_comparator_original_coeffs.argtypes = [vp, vp]
    L.gz_comparator_original_coeffs.restype = i32
    L.gz_comparator_write_jpeg.argtypes = [vp, vp, vp, ctypes.POINTER(ctypes.c_void_p),
                                           ctypes.POINTER(ctypes.c_size_t)]
    L.gz_comparator_write_jpeg.restype = i32
    L.gz_write_jpeg_host.argtypes = [i32, i32, vp, vp, ctypes.POINTER(ctypes.c_void_p),
                                     ctypes.POINTER(ctypes.c_size_t)]
    L.gz_write_jpeg_host.restype = i32
    L.gz_synthetic_frame.argtypes = [u64, i32, i32, vp]
    L.gz_synthetic_frame.restype = i32
    L.gz_rgb_to_coeffs.argtypes = [vp, i32, i32, vp]
    L.gz_rgb_to_coeffs.restype = i32
    L.gz_process_rgb_strips.argtypes = [i32, ctypes.POINTER(_Params), vp, i32, i32,
                                        ctypes.POINTER(_Collectives), ctypes.POINTER(vp),
                                        ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(_Stats)]
    L.gz_strip_layout.argtypes = [i32, i32, i32, i32] + [ctypes.POINTER(i32)] * 4
    L.gz_collectives_selftest.argtypes = [ctypes.POINTER(_Collectives)]
    L.gz_rccl_unique_id.argtypes = [ctypes.c_char_p]
    L.gz_rccl_create.argtypes = [i32, i32, i32, ctypes.c_char_p, ctypes.POINTER(vp),
                                 ctypes.POINTER(_Collectives)]
    L.gz_rccl_destroy.argtypes = [vp]
    L.gz_rccl_destroy.restype = None
    L.gz_rccl_library.argtypes = []
    L.gz_rccl_library.restype = ctypes.c_char_p
    L.gz_profile_enable.argtypes = [i32]
    L.gz_profile_get.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_long),
                                 ctypes.POINTER(ctypes.c_double)]
    L.gz_profile_get.restype = i32
    L.gz_profile_names.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    L.gz_profile_names.restype = ctypes.c_size_t
    L.gz_last_process_detail.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    L.gz_last_process_detail.restype = ctypes.c_size_t
    _lib = L
    return L


def _check(status, what):
    if status != GZ_OK:
        raise GuetzliError(status, "%s: %s" % (what, lib().gz_last_error().decode()))


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def profile_enable(on=True):
    """Per-launch HIP-event timing inside the library (gz_profile_enable)."""
    lib().gz_profile_enable(1 if on else 0)


def profile_reset():
    lib().gz_profile_reset()


def profile_read():
    """{region: (count, total_ms)} of everything recorded since the last reset."""
    L = lib()
    n = L.gz_profile_names(None, 0)
    buf = ctypes.create_string_buffer(n)
    L.gz_profile_names(buf, n)
    out = {}
    for name in filter(None, buf.value.decode().split(",")):
        c, t = ctypes.c_long(), ctypes.c_double()
        if L.gz_profile_get(name.encode(), ctypes.byref(c), ctypes.byref(t)):
            out[name] = (c.value, t.value)
    return out


def last_process_detail():
    """Host-side timers / counters of this thread's last process() call."""
    import json
    L = lib()
    n = L.gz_last_process_detail(None, 0)
    buf = ctypes.create_string_buffer(n)
    L.gz_last_process_detail(buf, n)
    return json.loads(buf.value.decode())


def _take_bytes(p, n):
    try:
        return ctypes.string_at(p.value, n.value)
    finally:
        lib().gz_free(p)


def write_jpeg_host(coeffs, quant, width, height):
    """SaveToJpegData + WriteJpeg on the host of dequantized [3][blocks][64]
    int16 coefficients with [3][64] quant tables (metadata stripped)."""
    c = np.ascontiguousarray(coeffs, dtype=np.int16).reshape(-1)
    q = np.ascontiguousarray(quant, dtype=np.int32).reshape(-1)
    p, n = ctypes.c_void_p(), ctypes.c_size_t()
    _check(lib().gz_write_jpeg_host(width, height, _ptr(c), _ptr(q), ctypes.byref(p),
                                    ctypes.byref(n)), "write_jpeg_host")
    return _take_bytes(p, n)


def device_count():
    return lib().gz_device_count()


def build_info():
    return lib().gz_build_info().decode()


def butteraugli_score_for_quality(quality):
    return lib().gz_butteraugli_score_for_quality(float(quality))


@dataclass
class Params:
    """guetzli::Params (processor.h:34-42)."""
    butteraugli_target: float = 1.0
    clear_metadata: bool = True
    try_420: bool = False
    force_420: bool = False
    use_silver_screen: bool = False
    zeroing_greedy_lookahead: int = 3
    new_zeroing_model: bool = True

    @classmethod
    def for_quality(cls, quality, **kw):
        # guetzli.cc:312-314: target = float(ButteraugliScoreForQuality(quality))
        t = float(np.float32(butteraugli_score_for_quality(quality)))
        return cls(butteraugli_target=t, **kw)

    def _c(self):
        return _Params(self.butteraugli_target, int(self.clear_metadata), int(self.try_420),
                       int(self.force_420), int(self.use_silver_screen),
                       int(self.zeroing_greedy_lookahead), int(self.new_zeroing_model))


@dataclass
class ProcessStats:
    iterations: int
    iterations_up: int
    iterations_down: int
    compares: int
    seconds_compare: float
    seconds_zeroing: float
    seconds_total: float
    seconds_setup: float = 0.0
    seconds_write: float = 0.0
    seconds_quantize: float = 0.0
    seconds_backend: float = 0.0


def _as_rgb(rgb, width, height):
    a = np.ascontiguousarray(np.frombuffer(rgb, dtype=np.uint8) if isinstance(rgb, (bytes, bytearray))
                             else np.asarray(rgb, dtype=np.uint8)).reshape(-1)
    if a.size != 3 * width * height:
        raise GuetzliError(1, "rgb has %d bytes, expected %d" % (a.size, 3 * width * height))
    return a


def process(rgb, width, height, params=None, device=0, return_stats=False):
    """guetzli::Process on an RGB8 image -> JPEG bytes (bit-identical to `guetzli --c`)."""
    L = lib()
    a = _as_rgb(rgb, width, height)
    p = (params or Params())._c()
    out = ctypes.c_void_p()
    size = ctypes.c_size_t()
    st = _Stats()
    _check(L.gz_process_rgb(device, ctypes.byref(p), _ptr(a), width, height, ctypes.byref(out),
                            ctypes.byref(size), ctypes.byref(st)), "process")
    data = ctypes.string_at(out, size.value)
    L.gz_free(out)
    if return_stats:
        return data, ProcessStats(st.iterations, st.iterations_up, st.iterations_down,
                                  st.compares, st.seconds_compare, st.seconds_zeroing,
                                  st.seconds_total, st.seconds_setup, st.seconds_write,
                                  st.seconds_quantize, st.seconds_backend)
    return data


def process_jpeg(jpeg, params=None, device=0, return_stats=False):
    """guetzli::Process on JPEG file bytes (processor.cc:1029-1066) -> JPEG
    bytes.  4:4:4 and 4:2:0 YCbCr inputs (4:2:0 forces the downsampled
    search); others raise GuetzliError(GZ_ERR_UNSUPPORTED)."""
    L = lib()
    buf = ctypes.create_string_buffer(bytes(jpeg), len(jpeg))
    p = (params or Params())._c()
    out = ctypes.c_void_p()
    size = ctypes.c_size_t()
    st = _Stats()
    _check(L.gz_process_jpeg(device, ctypes.byref(p), ctypes.cast(buf, ctypes.c_void_p), len(jpeg),
                             ctypes.byref(out), ctypes.byref(size), ctypes.byref(st)),
           "process_jpeg")
    data = ctypes.string_at(out, size.value)
    L.gz_free(out)
    if return_stats:
        return data, ProcessStats(st.iterations, st.iterations_up, st.iterations_down,
                                  st.compares, st.seconds_compare, st.seconds_zeroing,
                                  st.seconds_total, st.seconds_setup, st.seconds_write,
                                  st.seconds_quantize, st.seconds_backend)
    return data


def png_decode(png):
    """ReadPNG of the reference CLI (guetzli.cc:51-156) on the host:
    (width, height, rgb uint8 array of 3*w*h)."""
    data = bytes(png)
    w, h, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_void_p()
    _check(lib().gz_png_decode(data, len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(p)),
           "png_decode")
    n = 3 * w.value * h.value
    rgb = np.frombuffer(_take_bytes(p, ctypes.c_size_t(n)), dtype=np.uint8).copy()
    return w.value, h.value, rgb


def process_file(data, params=None, device=0, return_stats=False):
    """The reference CLI's input dispatch (guetzli.cc:284-310): a PNG file is
    decoded (png_decode) and encoded from its RGB, anything else is taken as
    a JPEG file (process_jpeg)."""
    data = bytes(data)
    if data[:8] == b"\x89PNG\r\n\x1a\n":
        w, h, rgb = png_decode(data)
        return process(rgb, w, h, params, device, return_stats)
    return process_jpeg(data, params, device, return_stats)


def jpeg_decode(jpeg):
    """ReadJpeg + DecodeJpegToRGB (host only): returns (width, height, ncomp,
    int16 quantized coefficients of all components concatenated, RGB8 array
    of shape (h, w, 3) for 4:4:4 / 4:2:0 YCbCr inputs, else None)."""
    L = lib()
    buf = ctypes.create_string_buffer(bytes(jpeg), len(jpeg))
    w, h, nc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    co, rgb = ctypes.c_void_p(), ctypes.c_void_p()
    n = ctypes.c_size_t()
    _check(L.gz_jpeg_decode(ctypes.cast(buf, ctypes.c_void_p), len(jpeg), ctypes.byref(w),
                            ctypes.byref(h), ctypes.byref(nc), ctypes.byref(co), ctypes.byref(n),
                            ctypes.byref(rgb)), "jpeg_decode")
    coeffs = np.frombuffer(ctypes.string_at(co, 2 * n.value), np.int16).copy()
    L.gz_free(co)
    img = None
    if rgb.value:
        img = np.frombuffer(ctypes.string_at(rgb, 3 * w.value * h.value), np.uint8).reshape(
            h.value, w.value, 3).copy()
        L.gz_free(rgb)
    return w.value, h.value, nc.value, coeffs, img


def process_device(rgb_dev_ptr, width, height, params=None, device=0, return_stats=False):
    """Same as process() with the RGB image already resident in HBM (device pointer)."""
    L = lib()
    p = (params or Params())._c()
    out = ctypes.c_void_p()
    size = ctypes.c_size_t()
    st = _Stats()
    _check(L.gz_process_rgb_device(device, ctypes.byref(p), ctypes.c_void_p(rgb_dev_ptr), width,
                                   height, ctypes.byref(out), ctypes.byref(size),
                                   ctypes.byref(st)), "process_device")
    data = ctypes.string_at(out, size.value)
    L.gz_free(out)
    if return_stats:
        return data, ProcessStats(st.iterations, st.iterations_up, st.iterations_down,
                                  st.compares, st.seconds_compare, st.seconds_zeroing,
                                  st.seconds_total, st.seconds_setup, st.seconds_write,
                                  st.seconds_quantize, st.seconds_backend)
    return data


class Collectives:
    """The exchange of a multi-rank encode (gz_collectives): an equal-size
    all-gather of byte blocks.  `allgather(data: bytes) -> bytes` must return
    every rank's block concatenated in rank order; or, without copies,
    `allgather_into(send_ptr, nbytes, recv_ptr)` gathers nbytes from send_ptr
    of every rank into recv_ptr (world * nbytes, rank order).  Keeps the
    ctypes callback alive for as long as the object lives."""

    def __init__(self, rank, world, allgather=None, allgather_into=None):
        self.rank, self.world = rank, world
        self._fn = allgather
        self._into = allgather_into

        def cb(_ctx, send, nbytes, recv):
            try:
                if self._into is not None:
                    self._into(send or 0, nbytes, recv or 0)
                    return 0
                data = ctypes.string_at(send, nbytes) if nbytes else b""
                out = self._fn(data)
                if len(out) != nbytes * self.world:
                    return 1
                if out:
                    ctypes.memmove(recv, out, len(out))
                return 0
            except Exception:  # an exception cannot cross the C boundary
                return 1

        self._cb = _ALLGATHER(cb)
        self._c = _Collectives(None, rank, world, self._cb)

    @classmethod
    def from_torch(cls, dist, device="cpu", group=None):
        """Bound to torch.distributed: all_gather_into_tensor of uint8 blocks on
        `device` ("cuda:N" for RCCL over xGMI with the nccl backend, "cpu" for
        gloo).  The library's buffers are wrapped, not copied: on the CPU the
        collective reads and writes them in place, on a GPU one H2D copy of
        the block and one D2H copy of the result."""
        import torch

        world, rank = dist.get_world_size(group), dist.get_rank(group)

        def wrap(ptr, n):
            return torch.frombuffer((ctypes.c_uint8 * n).from_address(ptr), dtype=torch.uint8)

        def allgather_into(send, n, recv):
            if n == 0:
                return
            src, dst = wrap(send, n), wrap(recv, n * world)
            if str(device) == "cpu":
                dist.all_gather(list(dst.view(world, n).unbind(0)), src, group=group)
            else:
                d_src = src.to(device, non_blocking=False)
                d_dst = torch.empty(world * n, dtype=torch.uint8, device=device)
                dist.all_gather_into_tensor(d_dst, d_src, group=group)
                dst.copy_(d_dst)

        return cls(rank, world, allgather_into=allgather_into)

    @classmethod
    def from_rccl(cls, device, rank, world, unique_id):
        """The library's own RCCL communicator (gz_rccl_create: staged
        all-gathers on its own HIP stream, no torch); unique_id: the 128
        bytes of rccl_unique_id() on one rank, handed to every rank.  close()
        (or the object's end) destroys the communicator."""
        obj = cls.__new__(cls)
        obj.rank, obj.world = rank, world
        obj._c = _Collectives()
        h = ctypes.c_void_p()
        uid = bytes(unique_id)
        if len(uid) != 128:
            raise GuetzliError(1, "from_rccl: the unique id has 128 bytes")
        _check(lib().gz_rccl_create(device, rank, world, uid, ctypes.byref(h), ctypes.byref(obj._c)),
               "rccl_create")
        obj._rccl = h.value
        return obj

    def close(self):
        if getattr(self, "_rccl", None):
            lib().gz_rccl_destroy(self._rccl)
            self._rccl = None

    def __del__(self):
        self.close()

    def selftest(self):
        _check(lib().gz_collectives_selftest(ctypes.byref(self._c)), "collectives_selftest")


def rccl_library():
    """Path of the librccl the library's communicators use (gz_rccl_library)."""
    return lib().gz_rccl_library().decode()


def rccl_unique_id():
    """ncclGetUniqueId (gz_rccl_unique_id): 128 bytes for Collectives.from_rccl."""
    buf = ctypes.create_string_buffer(128)
    _check(lib().gz_rccl_unique_id(buf), "rccl_unique_id")
    return buf.raw


def strip_layout(width, height, world, rank):
    """(y0, y1, e0, e1): rows rank `rank` owns and computes when one frame is
    split over `world` GPUs."""
    v = [ctypes.c_int() for _ in range(4)]
    _check(lib().gz_strip_layout(width, height, world, rank, *[ctypes.byref(x) for x in v]),
           "strip_layout")
    return tuple(x.value for x in v)


def process_strips(rgb, width, height, collectives, params=None, device=0, return_stats=False):
    """guetzli::Process of one frame split over the ranks of `collectives`
    (row strips + halo, one GPU per rank); every rank passes the whole frame
    and gets the same bytes as process()."""
    L = lib()
    a = _as_rgb(rgb, width, height)
    p = (params or Params())._c()
    out = ctypes.c_void_p()
    size = ctypes.c_size_t()
    st = _Stats()
    _check(L.gz_process_rgb_strips(device, ctypes.byref(p), _ptr(a), width, height,
                                   ctypes.byref(collectives._c), ctypes.byref(out),
                                   ctypes.byref(size), ctypes.byref(st)), "process_strips")
    data = ctypes.string_at(out, size.value)
    L.gz_free(out)
    if return_stats:
        return data, ProcessStats(st.iterations, st.iterations_up, st.iterations_down,
                                  st.compares, st.seconds_compare, st.seconds_zeroing,
                                  st.seconds_total, st.seconds_setup, st.seconds_write,
                                  st.seconds_quantize, st.seconds_backend)
    return data


def synthetic_frame(seed, width, height):
    """Deterministic synthetic sRGB frame, shape (h, w, 3) uint8."""
    out = np.zeros(3 * width * height, dtype=np.uint8)
    _check(lib().gz_synthetic_frame(seed, width, height, _ptr(out)), "synthetic_frame")
    return out.reshape(height, width, 3)


def rgb_to_coeffs(rgb, width, height):
    """q=1 DCT coefficients of an RGB image, [3][blocks][64] int16."""
    a = _as_rgb(rgb, width, height)
    nb = ((width + 7) // 8) * ((height + 7) // 8)
    out = np.zeros(3 * nb * 64, dtype=np.int16)
    _check(lib().gz_rgb_to_coeffs(_ptr(a), width, height, _ptr(out)), "rgb_to_coeffs")
    return out


def engine_pool_trim(keep_bytes=0):
    """Destroys idle pooled engines until at most keep_bytes remain."""
    return int(lib().gz_engine_pool_trim(keep_bytes))


def engine_pool_idle_bytes():
    return int(lib().gz_engine_pool_idle_bytes())


def block_error_adjustment_weights(width, height, target, direction, max_block_dist, distmap,
                                   target_mul=1.0, factor_x=1, factor_y=1, block_weight=None):
    """ComputeBlockErrorAdjustmentWeights (butteraugli_comparator.cc:169-233)
    on the host; block_weight (zeros by default) is updated and returned."""
    d = np.ascontiguousarray(distmap, dtype=np.float32).reshape(-1)
    if d.size != width * height:
        raise ValueError("distmap must hold width*height floats")
    nb = ((width + 8 * factor_x - 1) // (8 * factor_x)) * ((height + 8 * factor_y - 1) // (8 * factor_y))
    wgt = np.zeros(nb, np.float32) if block_weight is None else \
        np.ascontiguousarray(block_weight, dtype=np.float32).copy()
    _check(lib().gz_block_error_adjustment_weights(width, height, ctypes.c_float(target), direction,
                                                   max_block_dist, target_mul, factor_x, factor_y,
                                                   _ptr(d), _ptr(wgt)),
           "block_error_adjustment_weights")
    return wgt


class ButteraugliComparator:
    """guetzli::ButteraugliComparator (butteraugli_comparator.h:33-81) on the GPU."""

    def __init__(self, width, height, rgb, target_distance, device=0):
        L = lib()
        self.width, self.height = width, height
        self.blocks = ((width + 7) // 8) * ((height + 7) // 8)
        self._rgb = _as_rgb(rgb, width, height)
        h = ctypes.c_void_p()
        _check(L.gz_comparator_create(device, width, height, _ptr(self._rgb),
                                      ctypes.c_float(target_distance), ctypes.byref(h)),
               "comparator_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().gz_comparator_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _coeffs(self, coeffs):
        c = np.ascontiguousarray(coeffs, dtype=np.int16).reshape(-1)
        if c.size != 3 * self.blocks * 64:
            raise GuetzliError(1, "coefficient array has %d entries, expected %d"
                               % (c.size, 3 * self.blocks * 64))
        return c

    def compare(self, coeffs):
        """Comparator::Compare; returns distmap_aggregate()."""
        d = ctypes.c_float()
        _check(lib().gz_comparator_compare(self._h, _ptr(self._coeffs(coeffs)), ctypes.byref(d)),
               "compare")
        return d.value

    def compare_stages(self, coeffs):
        """Compare with every intermediate stage returned (parity tests)."""
        n = self.width * self.height
        rn = ((self.width + 2) // 3) * ((self.height + 2) // 3)
        sizes = {"cand_linear": 3 * n, "cand_xyb": 3 * n, "mhic0": 3 * n, "mhic1": 3 * n,
                 "edge": 3 * rn, "block_dc": 3 * rn, "block_ac": 3 * rn, "block_ac_lf": 3 * rn,
                 "mask": 3 * n, "mask_dc": 3 * n, "combined": rn, "distmap": n}
        arrs = {k: np.zeros(v, dtype=np.float32) for k, v in sizes.items()}
        st = _Stages(**{k: a.ctypes.data for k, a in arrs.items()})
        d = ctypes.c_float()
        _check(lib().gz_comparator_compare_stages(self._h, _ptr(self._coeffs(coeffs)),
                                                  ctypes.byref(st), ctypes.byref(d)),
               "compare_stages")
        arrs["distance"] = d.value
        return arrs

    def compare_420(self, y, plane_cb, plane_cr, cb=None, cr=None):
        """Compare of a 4:2:0 candidate: Y coefficients and the factor-2
        chroma pixel planes (uint16, h x w, wrapping state)."""
        n = self.width * self.height
        yy = np.ascontiguousarray(y, dtype=np.int16).reshape(-1)
        pcb = np.ascontiguousarray(plane_cb, dtype=np.uint16).reshape(-1)
        pcr = np.ascontiguousarray(plane_cr, dtype=np.uint16).reshape(-1)
        cper = ((self.width + 15) // 16) * ((self.height + 15) // 16) * 64
        if yy.size != 64 * ((self.width + 7) // 8) * ((self.height + 7) // 8) or pcb.size != n or pcr.size != n:
            raise GuetzliError(1, "compare_420: shapes")
        cbs = [None if a is None else np.ascontiguousarray(a, dtype=np.int16).reshape(-1) for a in (cb, cr)]
        if any(a is not None and a.size != cper for a in cbs):
            raise GuetzliError(1, "compare_420: chroma coefficient shapes")
        d = ctypes.c_float()
        _check(lib().gz_comparator_compare_420(self._h, _ptr(yy), None if cbs[0] is None else _ptr(cbs[0]),
                                               None if cbs[1] is None else _ptr(cbs[1]), _ptr(pcb), _ptr(pcr),
                                               ctypes.byref(d)), "compare_420")
        return d.value

    def compare_stages_production(self, coeffs):
        """Compare with the planes the search's own (fused) kernels leave in
        HBM returned: mhic0, mhic1, edge (k_block_diff's fused corner term),
        block_dc, block_ac (before the low-frequency term) and distmap."""
        n = self.width * self.height
        rn = ((self.width + 2) // 3) * ((self.height + 2) // 3)
        sizes = {"mhic0": 3 * n, "mhic1": 3 * n, "edge": 3 * rn, "block_dc": 3 * rn,
                 "block_ac": 3 * rn, "distmap": n}
        arrs = {k: np.zeros(v, dtype=np.float32) for k, v in sizes.items()}
        st = _Stages(**{k: a.ctypes.data for k, a in arrs.items()})
        d = ctypes.c_float()
        _check(lib().gz_comparator_compare_stages_production(self._h, _ptr(self._coeffs(coeffs)),
                                                             ctypes.byref(st), ctypes.byref(d)),
               "compare_stages_production")
        arrs["distance"] = d.value
        return arrs

    def distmap(self):
        """Comparator::distmap() of the last compare (h x w floats)."""
        out = np.zeros(self.width * self.height, dtype=np.float32)
        _check(lib().gz_comparator_distmap(self._h, _ptr(out)), "distmap")
        return out.reshape(self.height, self.width)

    def compare_blocks(self, blocks, candidates):
        """SwitchBlock + CompareBlock (butteraugli_comparator.cc:85-163) per
        request: block indices (n,) and candidate coefficients (n, 3, 64);
        returns CompareBlock's doubles."""
        b = np.ascontiguousarray(blocks, dtype=np.int32).reshape(-1)
        c = np.ascontiguousarray(candidates, dtype=np.int16).reshape(-1)
        if c.size != 192 * b.size:
            raise GuetzliError(1, "compare_blocks: %d candidates for %d blocks" % (c.size // 192,
                                                                                   b.size))
        err = np.zeros(b.size, dtype=np.float64)
        _check(lib().gz_comparator_compare_blocks(self._h, b.size, _ptr(b), _ptr(c), _ptr(err)),
               "compare_blocks")
        return err

    def block_max(self):
        out = np.zeros(self.blocks, dtype=np.float32)
        _check(lib().gz_comparator_block_max(self._h, _ptr(out)), "block_max")
        return out

    def distance_ok(self, target_mul):
        return bool(lib().gz_comparator_distance_ok(self._h, float(target_mul)))

    def score_output_size(self, size):
        return lib().gz_comparator_score_output_size(self._h, int(size))

    def start_block_comparisons(self):
        out = np.zeros(3 * self.blocks, dtype=np.float32)
        _check(lib().gz_comparator_start_block_comparisons(self._h, _ptr(out)),
               "start_block_comparisons")
        return out.reshape(self.blocks, 3)

    def write_jpeg(self, coeffs, quant):
        """The same JPEG as write_jpeg_host, entropy coded on the device."""
        c = self._coeffs(coeffs)
        q = np.ascontiguousarray(quant, dtype=np.int32).reshape(-1)
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        _check(lib().gz_comparator_write_jpeg(self._h, _ptr(c), _ptr(q), ctypes.byref(p),
                                              ctypes.byref(n)), "write_jpeg")
        return _take_bytes(p, n)

    def original_coeffs(self):
        """q=1 coefficients of the reference image, computed on the device."""
        out = np.zeros(3 * self.blocks * 64, dtype=np.int16)
        _check(lib().gz_comparator_original_coeffs(self._h, ctypes.c_void_p(out.ctypes.data)),
               "original_coeffs")
        return out

    def block_zeroing_orders(self, cur_coeffs, orig_coeffs, limit, comp_mask=7, lookahead=3,
                             new_zeroing_model=True):
        """Per-block greedy zeroing orders (processor.cc:376-487), blocks x 192."""
        out = np.zeros(self.blocks * 192, dtype=COEFF_DTYPE)
        _check(lib().gz_comparator_block_zeroing_orders(
            self._h, _ptr(self._coeffs(cur_coeffs)), _ptr(self._coeffs(orig_coeffs)), comp_mask,
            ctypes.c_float(limit), lookahead, 1 if new_zeroing_model else 0,
            ctypes.c_void_p(out.ctypes.data)),
            "block_zeroing_orders")
        return out.reshape(self.blocks, 192)
