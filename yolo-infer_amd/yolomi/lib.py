"""ctypes binding of `include/yolomi.h` (libyolomi.so, built in-tree for gfx950 by csrc/Makefile).

There is no fallback: if the library or a GPU is missing, constructing a `Runtime` raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path
from typing import Optional

# YM_LIB: another build of the library (same-box A/B of kernel variants: tools/gpu_ab_libs.sh); default in-tree
LIB_PATH = Path(os.environ.get("YM_LIB") or Path(__file__).resolve().parent / "libyolomi.so")

YM_ERRORS = {-1: "EINVAL", -2: "EBLOB", -3: "EHIP", -4: "ENOMEM", -5: "ESTATE"}


class YMError(RuntimeError):
    pass


class ModelDesc(C.Structure):
    _fields_ = [("max_batch", C.c_int), ("max_h", C.c_int), ("max_w", C.c_int), ("scale", C.c_int), ("task", C.c_int),
                ("dtype", C.c_int), ("reserved", C.c_int * 2)]


TASK_CODES = {"detect": 1, "segment": 2}
DTYPE_CODES = {"f16": 1, "f32": 2, "i8": 3, "f8": 4, "x3": 5}


class RcclId(C.Structure):
    _fields_ = [("internal", C.c_char * 128)]


class InferArgs(C.Structure):
    _fields_ = [("conf", C.c_float), ("max_wh", C.c_float), ("iou", C.c_double), ("max_det", C.c_int),
                ("max_nms", C.c_int), ("agnostic", C.c_int), ("in_eps", C.c_float), ("has_classes", C.c_int),
                ("classes", C.c_uint32 * 4), ("use_graph", C.c_int), ("lanes", C.c_int), ("counts_after_dets", C.c_int),
                ("d_batch_max", C.c_void_p), ("reserved", C.c_int * 4)]


_lib = None


def load_library(path: os.PathLike = LIB_PATH):
    """Load libyolomi.so once. torch must be imported first so the process shares torch's HIP runtime."""
    global _lib
    if _lib is not None:
        return _lib
    import torch  # noqa: F401  (binds libamdhip64 first; our .so then resolves to the same runtime)
    if not Path(path).exists():
        raise YMError(f"{path} not found: build it with `make -C yolo-infer_amd/csrc` "
                      f"(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(str(path))
    P, I, F = C.c_void_p, C.c_int, C.POINTER(C.c_float)
    sig = {
        "ym_create": (I, [I, C.POINTER(ModelDesc), C.POINTER(P)]),
        "ym_load_weights": (I, [P, P, C.c_size_t]),
        "ym_infer": (I, [P, P, I, I, I, C.POINTER(InferArgs), P, P, P]),
        "ym_profile": (I, [P, P, I, I, I, C.POINTER(InferArgs), P, P, P, F, I]),
        "ym_calibrate": (I, [P, P, I, I, I, C.POINTER(InferArgs), P, P, C.POINTER(C.c_void_p), I, P]),
        "ym_profile_replay": (I, [P, P, I, I, I, C.POINTER(InferArgs), P, P, P, I, F, I]),
        "ym_tune": (I, [P, P, I, I, I, C.POINTER(InferArgs), P, P, P, I]),
        "ym_masks": (I, [P, P, I, I, P, I, I, I, P, P, P]),
        "ym_masks_slots": (I, [P, P, I, I, P, I, I, I, P, P, P]),
        "ym_letterbox": (I, [P, P, I, I, I, I, I, I, I, I, P, I, I, P]),
        "ym_get_op_cfg": (I, [P, I, I, I, C.POINTER(I), I]),
        "ym_set_op_cfg": (I, [P, I, I, I, C.POINTER(I), I]),
        "ym_num_ops": (I, [P]),
        "ym_op_name": (C.c_char_p, [P, I]),
        "ym_num_buffers": (I, [P]),
        "ym_buffer_info": (I, [P, I, C.POINTER(P), C.POINTER(I), C.POINTER(I), C.POINTER(I), C.POINTER(I)]),
        "ym_read_buffer": (I, [P, I, P, C.c_size_t]),
        "ym_input_max": (I, [P, P, C.c_size_t, P, P]),
        "ym_broadcast_weights": (I, [P, P, I, P]),
        "ym_broadcast_weights_local": (I, [C.POINTER(P), I, I, P]),
        "ym_rccl_get_unique_id": (I, [C.POINTER(RcclId)]),
        "ym_rccl_comm_init": (I, [I, I, C.POINTER(RcclId), I, C.POINTER(P)]),
        "ym_rccl_comm_destroy": (I, [P]),
        "ym_sync": (I, [P]),
        "ym_last_error": (C.c_char_p, []),
        "ym_destroy": (None, [P]),
        "ym_version": (I, []),
        "ym_num_conv_cfgs": (I, [I]),
        "ym_set_debug": (I, [I, I]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


EXPORTED = ("ym_create", "ym_load_weights", "ym_broadcast_weights", "ym_broadcast_weights_local", "ym_rccl_get_unique_id", "ym_rccl_comm_init",
            "ym_rccl_comm_destroy", "ym_infer", "ym_input_max", "ym_calibrate", "ym_masks", "ym_masks_slots", "ym_letterbox",
            "ym_profile", "ym_profile_replay", "ym_tune", "ym_get_op_cfg", "ym_set_op_cfg", "ym_num_ops", "ym_op_name",
            "ym_num_buffers", "ym_buffer_info", "ym_read_buffer", "ym_sync", "ym_last_error", "ym_destroy",
            "ym_version", "ym_num_conv_cfgs", "ym_set_debug")

DBG_NMS, DBG_DW_MODE, DBG_DW_TILE, DBG_CHAIN, DBG_CHAIN_LAUNCHES, DBG_STEMFUSE, DBG_ATTN_KB = 1, 2, 3, 4, 5, 6, 7
DBG_PAIRST, DBG_CONV_CFG = 8, 9  # value + 1 (0: default)  # ym_set_debug keys (include/yolomi.h)


def set_debug(key: int, value: int) -> int:
    """ym_set_debug: a process-wide kernel debug switch; returns the previous value."""
    rc = load_library().ym_set_debug(key, value)
    if rc < 0:
        _check(rc)
    return rc


def _check(rc: int):
    if rc != 0:
        msg = _lib.ym_last_error().decode(errors="replace")
        raise YMError(f"yolomi {YM_ERRORS.get(rc, rc)}: {msg}")


def rccl_unique_id() -> bytes:
    lib = load_library()
    rid = RcclId()
    _check(lib.ym_rccl_get_unique_id(C.byref(rid)))
    return C.string_at(C.addressof(rid), 128)  # all 128 bytes (a c_char array would stop at the first NUL)


def rccl_comm_init(device: int, nranks: int, uid: bytes, rank: int) -> int:
    lib = load_library()
    if len(uid) != 128:
        raise ValueError("an RCCL unique id is 128 bytes")
    rid = RcclId()
    C.memmove(C.addressof(rid), uid, 128)
    comm = C.c_void_p()
    _check(lib.ym_rccl_comm_init(device, nranks, C.byref(rid), rank, C.byref(comm)))
    return comm.value


def rccl_comm_destroy(comm: int):
    _check(load_library().ym_rccl_comm_destroy(C.c_void_p(comm)))


class Runtime:
    """One ym_ctx on one device holding one packed model."""

    def __init__(self, device_index: int, blob: Optional[bytes], scale: str = None, task: str = None,
                 dtype: str = None):
        """scale / task / dtype (optional): what the blob must be (ym_model_desc; a mismatch raises YMError).
        blob None: an empty context that receives its model through broadcast_weights."""
        self.lib = load_library()
        self.ctx = C.c_void_p()
        self.device_index = device_index
        desc = ModelDesc()
        desc.scale = ord(scale) if scale else 0
        desc.task = TASK_CODES.get(task, 0)
        desc.dtype = DTYPE_CODES.get(dtype, 0)
        _check(self.lib.ym_create(device_index, C.byref(desc), C.byref(self.ctx)))
        self.n_ops, self.op_names = 0, []
        if blob is not None:
            self.load(blob)

    def load(self, blob: bytes):
        buf = C.create_string_buffer(blob, len(blob))
        _check(self.lib.ym_load_weights(self.ctx, C.cast(buf, C.c_void_p), len(blob)))
        self.n_ops = self.lib.ym_num_ops(self.ctx)
        self.op_names = [self.lib.ym_op_name(self.ctx, i).decode() for i in range(self.n_ops)]

    def input_max(self, x_ptr: int, n: int, out_ptr: int, stream: int):
        _check(self.lib.ym_input_max(self.ctx, C.c_void_p(x_ptr), n, C.c_void_p(out_ptr), C.c_void_p(stream)))

    def broadcast_weights(self, comm: int, root: int, stream: int):
        _check(self.lib.ym_broadcast_weights(self.ctx, C.c_void_p(comm), root, C.c_void_p(stream)))
        self.n_ops = self.lib.ym_num_ops(self.ctx)
        self.op_names = [self.lib.ym_op_name(self.ctx, i).decode() for i in range(self.n_ops)]

    @staticmethod
    def broadcast_weights_local(runtimes, root: int, stream: int):
        """ym_broadcast_weights_local: runtimes[root]'s model to every other Runtime of this process (the fake
        backend of the RCCL broadcast; the receivers are empty contexts, Runtime(dev, None))."""
        arr = (C.c_void_p * len(runtimes))(*[r.ctx.value for r in runtimes])
        _check(runtimes[0].lib.ym_broadcast_weights_local(arr, len(runtimes), root, C.c_void_p(stream)))
        for r in runtimes:
            r.n_ops = r.lib.ym_num_ops(r.ctx)
            r.op_names = [r.lib.ym_op_name(r.ctx, i).decode() for i in range(r.n_ops)]

    @staticmethod
    def make_args(conf=0.25, iou=0.7, max_det=300, max_nms=30000, agnostic=False, max_wh=7680.0, in_eps=1.1920929e-07,
                  classes=None, use_graph=True, lanes=1, batch_max_ptr=0, counts_after_dets=False) -> InferArgs:
        a = InferArgs()
        a.counts_after_dets = int(bool(counts_after_dets))
        a.d_batch_max = batch_max_ptr or None
        a.conf, a.iou, a.max_det, a.max_nms = float(conf), float(iou), int(max_det), int(max_nms)
        a.agnostic, a.max_wh, a.in_eps, a.use_graph = int(bool(agnostic)), float(max_wh), float(in_eps), int(use_graph)
        a.lanes = int(lanes)
        if classes is not None:
            a.has_classes = 1
            for c in classes:
                c = int(c)
                if not 0 <= c < 128:
                    raise ValueError(f"class id {c} out of range [0, 128)")
                a.classes[c >> 5] |= 1 << (c & 31)
        return a

    def infer(self, x_ptr: int, B: int, H: int, W: int, args: InferArgs, dets_ptr: int, counts_ptr: int, stream: int):
        _check(self.lib.ym_infer(self.ctx, C.c_void_p(x_ptr), B, H, W, C.byref(args), C.c_void_p(dets_ptr),
                                 C.c_void_p(counts_ptr), C.c_void_p(stream)))

    def profile(self, x_ptr, B, H, W, args, dets_ptr, counts_ptr, stream):
        ms = (C.c_float * self.n_ops)()
        _check(self.lib.ym_profile(self.ctx, C.c_void_p(x_ptr), B, H, W, C.byref(args), C.c_void_p(dets_ptr),
                                   C.c_void_p(counts_ptr), C.c_void_p(stream), ms, self.n_ops))
        return list(ms)

    def profile_replay(self, x_ptr, B, H, W, args, dets_ptr, counts_ptr, stream, reps=20):
        ms = (C.c_float * self.n_ops)()
        _check(self.lib.ym_profile_replay(self.ctx, C.c_void_p(x_ptr), B, H, W, C.byref(args), C.c_void_p(dets_ptr),
                                          C.c_void_p(counts_ptr), C.c_void_p(stream), reps, ms, self.n_ops))
        return list(ms)

    def calibrate(self, x_ptr, B, H, W, args, dets_ptr, counts_ptr, raw_ptrs, stream):
        arr = (C.c_void_p * len(raw_ptrs))(*[p or None for p in raw_ptrs])
        _check(self.lib.ym_calibrate(self.ctx, C.c_void_p(x_ptr), B, H, W, C.byref(args), C.c_void_p(dets_ptr),
                                     C.c_void_p(counts_ptr), arr, len(raw_ptrs), C.c_void_p(stream)))

    def masks(self, dets_ptr, B, max_det, offsets_ptr, total, H, W, masks_ptr, nonempty_ptr, stream):
        _check(self.lib.ym_masks(self.ctx, C.c_void_p(dets_ptr), B, max_det, C.c_void_p(offsets_ptr), total, H, W,
                                 C.c_void_p(masks_ptr), C.c_void_p(nonempty_ptr), C.c_void_p(stream)))

    def masks_slots(self, dets_ptr, B, max_det, counts_ptr, cap, H, W, masks_ptr, flags_ptr, stream):
        _check(self.lib.ym_masks_slots(self.ctx, C.c_void_p(dets_ptr), B, max_det, C.c_void_p(counts_ptr), cap, H, W,
                                       C.c_void_p(masks_ptr), C.c_void_p(flags_ptr), C.c_void_p(stream)))

    def letterbox(self, src_ptr, h, w, row_bytes, bgr, uh, uw, top, left, dst_ptr, Hn, Wn, stream):
        _check(self.lib.ym_letterbox(self.ctx, C.c_void_p(src_ptr), h, w, row_bytes, int(bool(bgr)), uh, uw, top, left,
                                     C.c_void_p(dst_ptr), Hn, Wn, C.c_void_p(stream)))

    def tune(self, x_ptr, B, H, W, args, dets_ptr, counts_ptr, stream, reps=8):
        _check(self.lib.ym_tune(self.ctx, C.c_void_p(x_ptr), B, H, W, C.byref(args), C.c_void_p(dets_ptr),
                                C.c_void_p(counts_ptr), C.c_void_p(stream), reps))

    def get_op_cfg(self, B, H, W):
        """Per-op conv configs of shape (B, H, W), or None when the shape has no tuned/pinned table."""
        arr = (C.c_int * self.n_ops)()
        rc = self.lib.ym_get_op_cfg(self.ctx, B, H, W, arr, self.n_ops)
        if rc == 1:
            return None
        _check(rc)
        return list(arr)

    def set_op_cfg(self, B, H, W, cfg):
        arr = (C.c_int * self.n_ops)(*cfg)
        _check(self.lib.ym_set_op_cfg(self.ctx, B, H, W, arr, self.n_ops))

    def buffer_info(self, buf: int):
        p, c, h, w, e = C.c_void_p(), C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _check(self.lib.ym_buffer_info(self.ctx, buf, C.byref(p), C.byref(c), C.byref(h), C.byref(w), C.byref(e)))
        return p.value, c.value, h.value, w.value, e.value

    def read_buffer(self, buf: int, dst_ptr: int, nbytes: int):
        _check(self.lib.ym_read_buffer(self.ctx, buf, C.c_void_p(dst_ptr), nbytes))

    def sync(self):
        _check(self.lib.ym_sync(self.ctx))

    def close(self):
        if self.ctx:
            self.lib.ym_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
