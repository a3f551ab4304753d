"""Python mirror of the jmh_* C ABI (include/jmhip.h) — the MI355X JM hot path.

This module is the host-side interface tests and bench.py drive: it mirrors lencod's per-picture
use of the hot path (JM 8.6 image.c › encode_one_frame → encode_one_macroblock per MB [J]) over
ctypes.  It loads ``csrc/libjmhip.so`` (built in-tree) and fails loudly if it is missing: there is
no CPU fallback in the product path.  ``libjmhost.so`` (host plumbing: synthetic source, CAVLC
writer, deblocking) is loaded on demand for the synthetic input generator.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JMH_LIB_PATH") or os.path.join(HERE, "csrc", "libjmhip.so")   # override: A/B builds
HOST_LIB_PATH = os.path.join(HERE, "host", "build", "libjmhost.so")

JMH_OK = 0
JMH_E_INVALID_ARG, JMH_E_HIP, JMH_E_OOM, JMH_E_UNSUPPORTED_CFG, JMH_E_STATE, JMH_E_NO_DEVICE = -1, -2, -3, -4, -5, -6
JMH_P_SLICE, JMH_I_SLICE = 0, 2
JMH_ABI_VERSION = 14
JMH_FLAG_KERNEL_TIMING = 1
STATUS = {0: "ok", -1: "invalid argument", -2: "HIP runtime error", -3: "out of memory",
          -4: "unsupported configuration", -5: "invalid call order", -6: "no HIP device"}
# JM 8.6 rdopt.c QP2QUANT [J]: RDO-off lambda = QP2QUANT[max(0, qp-12)]
QP2QUANT = [1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 4, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18,
            20, 23, 25, 29, 32, 36, 40, 45, 51, 57, 64, 72, 81, 91]


def lambda_rdo_off(qp):
    return QP2QUANT[max(0, qp - 12)]


def lambda_rdo_on(qp, bit_depth=8):
    """RDOptimization 1 (host/encoder.c jm_lambda_rdo_on): (lambda_mode, LAMBDA_FACTOR(sqrt(lambda_mode)))
    with lambda_mode = 0.85 * 2^((qp + QpBdOffsetY - 12) / 3) -- the same libm pow / sqrt as the C host."""
    import math
    qpbd = 6 * (bit_depth - 8) if bit_depth > 8 else 0
    lam = 0.85 * math.pow(2.0, (qp + qpbd - 12) / 3.0)
    return lam, int(65536.0 * math.sqrt(lam) + 0.5)


class JmhConfig(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("search_range", ctypes.c_int32), ("search_mode", ctypes.c_int32),
                ("use_hadamard", ctypes.c_int32), ("restrict_search_range", ctypes.c_int32),
                ("inter_search", ctypes.c_int32 * 8), ("num_ref_frames", ctypes.c_int32),
                ("constrained_intra_pred", ctypes.c_int32), ("num_frame_slots", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("pipeline_depth", ctypes.c_int32),
                ("transform_8x8_mode", ctypes.c_int32), ("jm_version", ctypes.c_int32),
                ("quant_offset", ctypes.c_int32 * 2), ("epzs_dual_refinement", ctypes.c_int32),
                ("slice_mbs", ctypes.c_int32), ("bit_depth", ctypes.c_int32),
                ("rdo", ctypes.c_int32), ("symbol_mode", ctypes.c_int32),
                ("epzs_subpel_me", ctypes.c_int32), ("epzs_subpel_thres_scale", ctypes.c_int32),
                ("epzs_min_thres_scale", ctypes.c_int32), ("epzs_max_thres_scale", ctypes.c_int32)]


class JmhFrameParams(ctypes.Structure):
    _fields_ = [("slice_type", ctypes.c_int32), ("qp", ctypes.c_int32),
                ("lambda_mode", ctypes.c_int32), ("lambda_motion", ctypes.c_int32),
                ("chroma_qp_offset", ctypes.c_int32), ("deblock", ctypes.c_int32),
                ("lf_disable", ctypes.c_int32), ("lf_alpha_div2", ctypes.c_int32),
                ("lf_beta_div2", ctypes.c_int32), ("lambda_factor_rd", ctypes.c_int32),
                ("lambda_rd", ctypes.c_double)]


class JmhTiming(ctypes.Structure):
    _fields_ = [("interp_ms", ctypes.c_float), ("mb_ms", ctypes.c_float),
                ("total_ms", ctypes.c_float), ("mb_launches", ctypes.c_int32),
                ("pictures", ctypes.c_int32), ("interps", ctypes.c_int32),
                ("analyse_ms", ctypes.c_float), ("analyse_launches", ctypes.c_int32),
                ("final_ms", ctypes.c_float), ("final_launches", ctypes.c_int32),
                ("ticks", ctypes.c_int32), ("tick_mbs", ctypes.c_int32),
                ("pictures_done", ctypes.c_int32),
                ("flow_launches", ctypes.c_int32), ("flow_mbs", ctypes.c_int32)]


class JmhBlockSearch(ctypes.Structure):
    _fields_ = [("mb_x", ctypes.c_int32), ("mb_y", ctypes.c_int32), ("blocktype", ctypes.c_int32),
                ("block_x", ctypes.c_int32), ("block_y", ctypes.c_int32), ("pred_mv", ctypes.c_int32 * 2),
                ("centre", ctypes.c_int32 * 2), ("search_range", ctypes.c_int32), ("lambda_factor", ctypes.c_int32),
                ("search_mode", ctypes.c_int32), ("slice_p", ctypes.c_int32)]


class JmhBlockResult(ctypes.Structure):
    _fields_ = [("mv", ctypes.c_int32 * 2), ("min_mcost", ctypes.c_int32), ("fullpel_mv", ctypes.c_int32 * 2),
                ("fullpel_cost", ctypes.c_int32)]


# jmh_mb_result, field for field (include/jmhip.h)
MB_RESULT_DTYPE = np.dtype([
    ("mb_type", "<i2"), ("cbp", "<i2"), ("cbp_blk", "<i4"), ("b8mode", "i1", 4),
    ("ref_idx", "i1", 4), ("i16mode", "i1"), ("c_ipred_mode", "i1"), ("transform_8x8", "i1"), ("pad0", "i1"),
    ("ipred", "i1", 16), ("mv", "<i2", (16, 2)), ("luma", "<i2", (16, 16)),
    ("luma_dc", "<i2", 16), ("chroma_dc", "<i2", (2, 4)), ("chroma_ac", "<i2", (2, 4, 16)),
    ("min_cost", "<i4"), ("reserved", "<i4")])

_P = ctypes.c_void_p
_I = ctypes.c_int
_SIGS = {
    "jmh_create": (_I, [ctypes.POINTER(JmhConfig), _I, ctypes.POINTER(_P)]),
    "jmh_destroy": (None, [_P]),
    "jmh_strerror": (ctypes.c_char_p, [_I]),
    "jmh_abi_version": (_I, []),
    "jmh_device_count": (_I, []),
    "jmh_set_reference": (_I, [_P, _I, _I, _P, _P, _P, _I, _I]),
    "jmh_frame_submit": (_I, [_P, _P, _P, _P, _I, _I, ctypes.POINTER(JmhFrameParams)]),
    "jmh_frame_wait": (_I, [_P]),
    "jmh_frame_push": (_I, [_P, _P, _P, _P, _I, _I, ctypes.POINTER(JmhFrameParams)]),
    "jmh_frame_pop": (_I, [_P]),
    "jmh_pipeline_depth": (_I, [_P]),
    "jmh_get_mb_result": (_P, [_P, _I]),
    "jmh_read_recon": (_I, [_P, _P, _P, _P, _I, _I]),
    "jmh_read_deblocked": (_I, [_P, _P, _P, _P, _I, _I]),
    "jmh_load_frame": (_I, [_P, _I, _P, _P, _P, _I, _I]),
    "jmh_set_reference_slot": (_I, [_P, _I]),
    "jmh_encode_slot": (_I, [_P, _I, ctypes.POINTER(JmhFrameParams)]),
    "jmh_sync": (_I, [_P]),
    "jmh_wait_issued": (_I, [_P]),
    "jmh_get_timing": (_I, [_P, ctypes.POINTER(JmhTiming)]),
    "jmh_ffs_sad_table": (_I, [_P, _I, _P, _P, _P]),
    "jmh_tq4x4_batch": (_I, [_P, _I, _P, _P, _I, _I, _P, _P, _P, _P]),
    "jmh_tq8x8_batch": (_I, [_P, _I, _P, _P, _I, _I, _P, _P, _P, _P]),
    "jmh_read_qpel": (_I, [_P, _P]),
    "jmh_set_reference_u16": (_I, [_P, _I, _I, _P, _P, _P, _I, _I]),
    "jmh_frame_submit_u16": (_I, [_P, _P, _P, _P, _I, _I, ctypes.POINTER(JmhFrameParams)]),
    "jmh_frame_push_u16": (_I, [_P, _P, _P, _P, _I, _I, ctypes.POINTER(JmhFrameParams)]),
    "jmh_read_recon_u16": (_I, [_P, _P, _P, _P, _I, _I]),
    "jmh_read_deblocked_u16": (_I, [_P, _P, _P, _P, _I, _I]),
    "jmh_load_frame_u16": (_I, [_P, _I, _P, _P, _P, _I, _I]),
    "jmh_search_pictures": (_I, [_P, _P, _P, _I]),
    "jmh_block_motion_search": (_I, [_P, _I, _P, _P]),
    "jmh_search_pictures_u16": (_I, [_P, _P, _P, _I, _I]),
    "jmh_block_motion_search_u16": (_I, [_P, _I, _P, _P]),
    "jmh_ffs_sad_table_u16": (_I, [_P, _I, _P, _P, _P]),
    "jmh_tq4x4_batch_u16": (_I, [_P, _I, _P, _P, _I, _I, _I, _P, _P, _P, _P]),
    "jmh_tq8x8_batch_u16": (_I, [_P, _I, _P, _P, _I, _I, _I, _P, _P, _P, _P]),
}
EXPORTED = tuple(_SIGS)


class JmhError(RuntimeError):
    pass


_lib = None


def load(path=LIB_PATH):
    """Load libjmhip.so (raises if it was not built — the product has no fallback)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise JmhError(f"libjmhip.so not found at {path}: build it with __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.jmh_abi_version() != JMH_ABI_VERSION:
        raise JmhError(f"{path}: ABI version {lib.jmh_abi_version()} != {JMH_ABI_VERSION} (stale build?)")
    if path == LIB_PATH:
        _lib = lib
    return lib


def _check(st, what):
    if st != JMH_OK:
        raise JmhError(f"{what}: {STATUS.get(st, st)} ({st})")


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def make_config(width, height, search_range=32, search_mode=0, use_hadamard=1,
                restrict_search_range=2, inter_search=(1, 1, 1, 1, 1, 1, 1), slots=2, kernel_timing=False,
                pipeline_depth=0, transform_8x8_mode=0, jm_version=8, quant_offset=(682, 342), epzs_dual_refinement=0, slice_mbs=0,
                bit_depth=8, rdo=0, symbol_mode=None, epzs_subpel_me=0, epzs_subpel_thres_scale=0, epzs_min_thres_scale=0,
                epzs_max_thres_scale=0, constrained_intra_pred=0):
    """jm_version >= 10 selects the JM >= 10 quantisation rounding with the flat OffsetMatrix
    entries quant_offset = (I slices, P slices) at OffsetBits 11 (docs/JM_SEMANTICS.md item 45)."""
    cfg = JmhConfig()
    cfg.width, cfg.height = width, height
    cfg.search_range, cfg.search_mode = search_range, search_mode
    cfg.use_hadamard, cfg.restrict_search_range = use_hadamard, restrict_search_range
    for i, v in enumerate(inter_search):
        cfg.inter_search[i + 1] = v
    cfg.num_ref_frames, cfg.constrained_intra_pred, cfg.num_frame_slots = 1, constrained_intra_pred, slots
    cfg.flags = JMH_FLAG_KERNEL_TIMING if kernel_timing else 0
    cfg.pipeline_depth = pipeline_depth
    cfg.transform_8x8_mode = transform_8x8_mode
    cfg.jm_version = jm_version
    cfg.epzs_dual_refinement = epzs_dual_refinement
    cfg.slice_mbs = slice_mbs
    cfg.bit_depth = bit_depth
    cfg.rdo = rdo
    cfg.symbol_mode = (1 if rdo else 0) if symbol_mode is None else symbol_mode
    cfg.epzs_subpel_me, cfg.epzs_subpel_thres_scale = epzs_subpel_me, epzs_subpel_thres_scale
    cfg.epzs_min_thres_scale, cfg.epzs_max_thres_scale = epzs_min_thres_scale, epzs_max_thres_scale
    if jm_version >= 10:
        cfg.quant_offset[0], cfg.quant_offset[1] = quant_offset
    return cfg


def frame_params(slice_type, qp, chroma_qp_offset=0, deblock=None, rdo=0, bit_depth=8):
    """deblock: None (no device deblocking) or (disable_idc, alpha_div2, beta_div2); rdo: fill the
    RDOptimization 1 lambdas."""
    fp = JmhFrameParams()
    fp.slice_type, fp.qp = slice_type, qp
    fp.lambda_mode = fp.lambda_motion = lambda_rdo_off(qp)
    if rdo:
        fp.lambda_rd, fp.lambda_factor_rd = lambda_rdo_on(qp, bit_depth)
    fp.chroma_qp_offset = chroma_qp_offset
    if deblock is not None:
        fp.deblock = 1
        fp.lf_disable, fp.lf_alpha_div2, fp.lf_beta_div2 = deblock
    return fp


def split_yuv(frame, w, h):
    """I420 buffer (w*h*3/2 bytes) -> contiguous (y, u, v) uint8 planes."""
    f = np.ascontiguousarray(frame, dtype=np.uint8).reshape(-1)
    y = f[: w * h].reshape(h, w)
    u = f[w * h: w * h + w * h // 4].reshape(h // 2, w // 2)
    v = f[w * h + w * h // 4:].reshape(h // 2, w // 2)
    return np.ascontiguousarray(y), np.ascontiguousarray(u), np.ascontiguousarray(v)


class Encoder:
    """One jmh_ctx: the macroblock hot path of one video stream on one HIP device."""

    def __init__(self, width, height, device=0, **kw):
        self.lib = load()
        self.w, self.h = width, height
        self.mbw, self.mbh = width // 16, height // 16
        self.cfg = make_config(width, height, **kw)
        # High 10 contexts take 16-bit pictures through the *_u16 entry points
        self.hbd = self.cfg.bit_depth > 8
        self.sfx = "_u16" if self.hbd else ""
        self.pdt = np.uint16 if self.hbd else np.uint8
        ctx = ctypes.c_void_p()
        _check(self.lib.jmh_create(ctypes.byref(self.cfg), device, ctypes.byref(ctx)), "jmh_create")
        self.ctx = ctx

    def close(self):
        if self.ctx:
            self.lib.jmh_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _planes(self, y, u, v):
        return [np.ascontiguousarray(a, self.pdt) for a in (y, u, v)]

    def set_reference(self, y, u, v):
        y, u, v = self._planes(y, u, v)
        fn = "jmh_set_reference" + self.sfx
        _check(getattr(self.lib, fn)(self.ctx, 0, 0, _ptr(y), _ptr(u), _ptr(v), self.w, self.w // 2), fn)

    def encode(self, y, u, v, slice_type, qp, chroma_qp_offset=0, deblock=None):
        fp = frame_params(slice_type, qp, chroma_qp_offset, deblock, self.cfg.rdo, self.cfg.bit_depth)
        y, u, v = self._planes(y, u, v)
        fn = "jmh_frame_submit" + self.sfx
        _check(getattr(self.lib, fn)(self.ctx, _ptr(y), _ptr(u), _ptr(v), self.w, self.w // 2, ctypes.byref(fp)), fn)
        _check(self.lib.jmh_frame_wait(self.ctx), "jmh_frame_wait")
        return self.results(), self.recon()

    # ---- pipelined pictures (jmh_frame_push / jmh_frame_pop) ----
    def push(self, y, u, v, slice_type, qp, chroma_qp_offset=0, deblock=None):
        fp = frame_params(slice_type, qp, chroma_qp_offset, deblock, self.cfg.rdo, self.cfg.bit_depth)
        y, u, v = self._planes(y, u, v)
        fn = "jmh_frame_push" + self.sfx
        _check(getattr(self.lib, fn)(self.ctx, _ptr(y), _ptr(u), _ptr(v), self.w, self.w // 2, ctypes.byref(fp)), fn)

    def pop(self):
        """Wait for the oldest pushed picture; returns (results, recon)."""
        _check(self.lib.jmh_frame_pop(self.ctx), "jmh_frame_pop")
        return self.results(), self.recon()

    def pop_into(self, y, u, v):
        """What lencod does per picture: jmh_frame_pop, the results in place (a zero-copy view of the
        library's host array, valid until the next pop) and the deblocked picture (the recon file /
        PSNR input) into the caller's planes.  Returns the results view."""
        _check(self.lib.jmh_frame_pop(self.ctx), "jmh_frame_pop")
        fn = "jmh_read_deblocked" + self.sfx
        _check(getattr(self.lib, fn)(self.ctx, _ptr(y), _ptr(u), _ptr(v), self.w, self.w // 2), fn)
        return self.results_view()

    def results_view(self):
        n = self.mbw * self.mbh
        p = self.lib.jmh_get_mb_result(self.ctx, 0)
        if not p:
            raise JmhError("no results")
        buf = (ctypes.c_char * (n * MB_RESULT_DTYPE.itemsize)).from_address(p)
        return np.frombuffer(buf, dtype=MB_RESULT_DTYPE)

    @property
    def depth(self):
        return self.lib.jmh_pipeline_depth(self.ctx)

    def results(self):
        n = self.mbw * self.mbh
        p = self.lib.jmh_get_mb_result(self.ctx, 0)
        if not p:
            raise JmhError("no results")
        buf = (ctypes.c_char * (n * MB_RESULT_DTYPE.itemsize)).from_address(p)
        return np.frombuffer(bytes(buf), dtype=MB_RESULT_DTYPE).copy()

    def _read(self, fn):
        fn += self.sfx
        y = np.empty((self.h, self.w), self.pdt)
        u = np.empty((self.h // 2, self.w // 2), self.pdt)
        v = np.empty_like(u)
        _check(getattr(self.lib, fn)(self.ctx, _ptr(y), _ptr(u), _ptr(v), self.w, self.w // 2), fn)
        return y, u, v

    def recon(self):
        return self._read("jmh_read_recon")

    def deblocked(self):
        """DeblockFrame output of the last encode(..., deblock=...) (jmh_read_deblocked)."""
        return self._read("jmh_read_deblocked")

    # ---- device-resident path (bench) ----
    def load_frame(self, slot, y, u, v):
        y, u, v = self._planes(y, u, v)
        fn = "jmh_load_frame" + self.sfx
        _check(getattr(self.lib, fn)(self.ctx, slot, _ptr(y), _ptr(u), _ptr(v), self.w, self.w // 2), fn)

    def set_reference_slot(self, slot):
        _check(self.lib.jmh_set_reference_slot(self.ctx, slot), "jmh_set_reference_slot")

    def encode_slot(self, slot, slice_type, qp, deblock=None):
        fp = frame_params(slice_type, qp, deblock=deblock, rdo=self.cfg.rdo, bit_depth=self.cfg.bit_depth)
        _check(self.lib.jmh_encode_slot(self.ctx, slot, ctypes.byref(fp)), "jmh_encode_slot")

    def sync(self):
        """Drain: every picture in flight runs to completion (jmh_sync)."""
        _check(self.lib.jmh_sync(self.ctx), "jmh_sync")

    def wait_issued(self):
        """Wait for the launches issued so far; pictures in flight stay in flight (jmh_wait_issued)."""
        _check(self.lib.jmh_wait_issued(self.ctx), "jmh_wait_issued")

    def timing(self):
        """Event sums since the previous call (waits for the issued launches, does not drain)."""
        t = JmhTiming()
        _check(self.lib.jmh_get_timing(self.ctx, ctypes.byref(t)), "jmh_get_timing")
        return t

    # ---- unit seams ----
    def sad_table(self, mb_xy, centres):
        mb_xy = np.ascontiguousarray(mb_xy, np.int32)
        centres = np.ascontiguousarray(centres, np.int32)
        n = mb_xy.shape[0]
        side = 2 * self.cfg.search_range + 1
        out = np.empty((n, 16, side * side), np.uint16)
        _check(self.lib.jmh_ffs_sad_table(self.ctx, n, _ptr(mb_xy), _ptr(centres), _ptr(out)),
               "jmh_ffs_sad_table")
        return out

    def tq4x4(self, resid, pred, qp, intra):
        resid = np.ascontiguousarray(resid, np.int16)
        pred = np.ascontiguousarray(pred, np.uint8)
        n = resid.shape[0]
        lev = np.empty((n, 16), np.int16)
        rec = np.empty((n, 16), np.uint8)
        cc = np.empty(n, np.int32)
        nz = np.empty(n, np.int32)
        _check(self.lib.jmh_tq4x4_batch(self.ctx, n, _ptr(resid), _ptr(pred), qp, intra, _ptr(lev),
                                        _ptr(rec), _ptr(cc), _ptr(nz)), "jmh_tq4x4_batch")
        return lev, rec, cc, nz

    def tq8x8(self, resid, pred, qp, intra):
        resid = np.ascontiguousarray(resid, np.int16)
        pred = np.ascontiguousarray(pred, np.uint8)
        n = resid.shape[0]
        lev = np.empty((n, 64), np.int16)
        rec = np.empty((n, 64), np.uint8)
        cc = np.empty(n, np.int32)
        nz = np.empty(n, np.int32)
        _check(self.lib.jmh_tq8x8_batch(self.ctx, n, _ptr(resid), _ptr(pred), qp, intra, _ptr(lev),
                                        _ptr(rec), _ptr(cc), _ptr(nz)), "jmh_tq8x8_batch")
        return lev, rec, cc, nz

    def read_qpel(self):
        out = np.empty((16, self.h + 8, self.w + 8), np.uint8)
        _check(self.lib.jmh_read_qpel(self.ctx, _ptr(out)), "jmh_read_qpel")
        return out

    def search_pictures(self, cur_y, ref_y):
        cur_y, ref_y = np.ascontiguousarray(cur_y, np.uint8), np.ascontiguousarray(ref_y, np.uint8)
        _check(self.lib.jmh_search_pictures(self.ctx, _ptr(cur_y), _ptr(ref_y), self.w), "jmh_search_pictures")

    def block_motion_search(self, reqs):
        """reqs: a ctypes array of JmhBlockSearch; returns the JmhBlockResult array."""
        out = (JmhBlockResult * len(reqs))()
        _check(self.lib.jmh_block_motion_search(self.ctx, len(reqs), ctypes.cast(reqs, _P), ctypes.cast(out, _P)),
               "jmh_block_motion_search")
        return out

    # ---- High 10 seams (16-bit samples, bit_depth 8..10) ----
    def search_pictures_u16(self, cur_y, ref_y, bit_depth):
        cur_y, ref_y = np.ascontiguousarray(cur_y, np.uint16), np.ascontiguousarray(ref_y, np.uint16)
        _check(self.lib.jmh_search_pictures_u16(self.ctx, _ptr(cur_y), _ptr(ref_y), self.w, bit_depth),
               "jmh_search_pictures_u16")

    def block_motion_search_u16(self, reqs):
        out = (JmhBlockResult * len(reqs))()
        _check(self.lib.jmh_block_motion_search_u16(self.ctx, len(reqs), ctypes.cast(reqs, _P), ctypes.cast(out, _P)),
               "jmh_block_motion_search_u16")
        return out

    def sad_table_u16(self, mb_xy, centres):
        mb_xy = np.ascontiguousarray(mb_xy, np.int32)
        centres = np.ascontiguousarray(centres, np.int32)
        n = mb_xy.shape[0]
        side = 2 * self.cfg.search_range + 1
        out = np.empty((n, 16, side * side), np.uint16)
        _check(self.lib.jmh_ffs_sad_table_u16(self.ctx, n, _ptr(mb_xy), _ptr(centres), _ptr(out)), "jmh_ffs_sad_table_u16")
        return out

    def tq_u16(self, resid, pred, qp, intra, bit_depth):
        """dct_luma (resid[n][16]) or dct_luma8x8 (resid[n][64]) on 16-bit samples."""
        resid = np.ascontiguousarray(resid, np.int16)
        pred = np.ascontiguousarray(pred, np.uint16)
        n, el = resid.shape
        lev = np.empty((n, el), np.int16)
        rec = np.empty((n, el), np.uint16)
        cc = np.empty(n, np.int32)
        nz = np.empty(n, np.int32)
        fn = self.lib.jmh_tq4x4_batch_u16 if el == 16 else self.lib.jmh_tq8x8_batch_u16
        _check(fn(self.ctx, n, _ptr(resid), _ptr(pred), qp, intra, bit_depth, _ptr(lev), _ptr(rec), _ptr(cc), _ptr(nz)),
               "jmh_tq%s_batch_u16" % ("4x4" if el == 16 else "8x8"))
        return lev, rec, cc, nz


# ---- synthetic source (product host plumbing, libjmhost.so) ------------------------------
_host = None


def load_host(path=HOST_LIB_PATH):
    global _host
    if _host is None:
        if not os.path.exists(path):
            raise JmhError(f"libjmhost.so not found at {path}: build it with __graft_entry__.build()")
        _host = ctypes.CDLL(path)
        _host.jm_synth_frame.restype = None
        _host.jm_synth_frame.argtypes = [_P, _I, _I, ctypes.c_uint64, _I]
    return _host


class _JmPic(ctypes.Structure):
    _fields_ = [("w", ctypes.c_int), ("h", ctypes.c_int), ("y", _P), ("u", _P), ("v", _P),
                ("bd", ctypes.c_int), ("Y", _P), ("U", _P), ("V", _P)]


def synth_frame(disp_w, disp_h, seed, index, bit_depth=8):
    """Deterministic synthetic 4:2:0 picture (coded size = multiple of 16), as (y, u, v); bit_depth
    9 / 10: 16-bit samples (jm_synth_frame_hbd)."""
    host = load_host()
    if bit_depth > 8:
        cw, ch = (disp_w + 15) // 16 * 16, (disp_h + 15) // 16 * 16
        y = np.zeros((ch, cw), np.uint16)
        u = np.zeros((ch // 2, cw // 2), np.uint16)
        v = np.zeros_like(u)
        host.jm_synth_frame_hbd.restype = None
        host.jm_synth_frame_hbd.argtypes = [_P, _P, _P, _I, _I, _I, _I, ctypes.c_uint64, _I, _I]
        host.jm_synth_frame_hbd(_ptr(y), _ptr(u), _ptr(v), cw, ch, disp_w, disp_h, seed, index, bit_depth)
        return y, u, v
    cw, ch = (disp_w + 15) // 16 * 16, (disp_h + 15) // 16 * 16
    y = np.zeros((ch, cw), np.uint8)
    u = np.zeros((ch // 2, cw // 2), np.uint8)
    v = np.zeros_like(u)
    pic = _JmPic(cw, ch, y.ctypes.data, u.ctypes.data, v.ctypes.data, 8, None, None, None)
    host.jm_synth_frame(ctypes.byref(pic), disp_w, disp_h, seed, index)
    return y, u, v
