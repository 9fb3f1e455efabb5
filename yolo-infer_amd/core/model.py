"""YOLO11Model / YOLO11Factory — drop-in for /root/reference/core/model.py on MI355X.

Same constructor, `predict`, `benchmark`, `get_model_info`, `.model` surface as the reference
(`core/model.py:29-295`), but `predict` runs the hand-written gfx950 path (`yolomi.engine.Engine` → libyolomi.so →
one HIP-graph replay per batch) instead of delegating to `ultralytics.YOLO.predict` (`core/model.py:133`).

Scope: tasks detect/segment, sizes n/s/m/l/x, `torch.Tensor` sources (BCHW or CHW, H,W % 32 == 0,
LoadTensor's /255 rule).  There is no CPU fallback: a CPU device or a missing libyolomi.so raises.
"""
from __future__ import annotations

import logging
import os
import time
from pathlib import Path
from typing import Any, Dict, List, Optional, Union

import numpy as np
import torch

from yolomi.engine import Engine
from yolomi.synth import synth_weights

from .results import LazyCounts, Results

logger = logging.getLogger(__name__)

COCO_NAMES = dict(enumerate((
    "person", "bicycle", "car", "motorcycle", "airplane", "bus", "train", "truck", "boat", "traffic light",
    "fire hydrant", "stop sign", "parking meter", "bench", "bird", "cat", "dog", "horse", "sheep", "cow", "elephant",
    "bear", "zebra", "giraffe", "backpack", "umbrella", "handbag", "tie", "suitcase", "frisbee", "skis", "snowboard",
    "sports ball", "kite", "baseball bat", "baseball glove", "skateboard", "surfboard", "tennis racket", "bottle",
    "wine glass", "cup", "fork", "knife", "spoon", "bowl", "banana", "apple", "sandwich", "orange", "broccoli",
    "carrot", "hot dog", "pizza", "donut", "cake", "chair", "couch", "potted plant", "bed", "dining table", "toilet",
    "tv", "laptop", "mouse", "remote", "keyboard", "cell phone", "microwave", "oven", "toaster", "sink",
    "refrigerator", "book", "clock", "vase", "scissors", "teddy bear", "hair drier", "toothbrush")))


class _ModelHandle:
    """What the reference exposes as `YOLO11Model.model` (an `ultralytics.YOLO`): callers use `.eval()`
    (speed_benchmark.py:323), `.parameters()` / `.model.parameters()` (model.py:240), `.names`."""

    def __init__(self, state_dict: Dict[str, np.ndarray], engine: Engine, names: Dict[int, str]):
        self._sd = state_dict
        self._params = {k: torch.from_numpy(np.asarray(v)) for k, v in state_dict.items()
                        if not k.endswith("num_batches_tracked")}
        for p in self._params.values():
            p.requires_grad_(True)
        self.engine = engine
        self.names = names
        self.model = self
        self.training = False

    def eval(self):
        return self

    def parameters(self):
        return iter(self._params.values())

    def state_dict(self):
        return dict(self._params)

    def state_dict_numpy(self) -> Dict[str, np.ndarray]:
        """The Ultralytics-key weights this model was packed from (what a quantizer re-packs)."""
        if not self._sd:
            raise ValueError("this model was built from a packed blob only; its weights are not on the host")
        return self._sd


def _load_state_dict(path: Path) -> Dict[str, np.ndarray]:
    """Weights file → Ultralytics-key state dict. Loaders that execute nothing from the file only."""
    suf = path.suffix.lower()
    if suf == ".safetensors":
        from safetensors.numpy import load_file
        return dict(load_file(str(path)))
    if suf == ".npz":
        with np.load(path, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    if suf == ".pt":
        try:
            obj = torch.load(path, map_location="cpu", weights_only=True)
        except Exception:  # a pickled Ultralytics model (YOLO('yolo11n.pt') checkpoints): restricted unpickler
            from yolomi.ptimport import load_ultralytics_checkpoint
            return load_ultralytics_checkpoint(str(path))
        if isinstance(obj, dict) and "state_dict" in obj:
            obj = obj["state_dict"]
        if not isinstance(obj, dict) or not all(isinstance(v, torch.Tensor) for v in obj.values()):
            raise ValueError(f"{path}: expected a state dict of tensors")
        return {k: v.float().numpy() if v.is_floating_point() else v.numpy() for k, v in obj.items()}
    raise ValueError(f"unsupported weights file {path} (use an Ultralytics .pt, a state-dict .pt, .safetensors or .npz)")


class YOLO11Model:
    SUPPORTED_TASKS = {
        "detect": "yolo11n.pt",
        "segment": "yolo11n-seg.pt",
        "classify": "yolo11n-cls.pt",
        "pose": "yolo11n-pose.pt",
        "obb": "yolo11n-obb.pt",
    }
    SUPPORTED_SIZES = ["n", "s", "m", "l", "x"]
    HIP_TASKS = ("detect", "segment")

    def __init__(self, model_path: Optional[Union[str, Path]] = None, task: str = "detect", size: str = "n",
                 device: Optional[str] = None, verbose: bool = True, dtype: str = "x3", seed: int = 0,
                 weights_blob: Optional[bytes] = None, qparams: Optional[Dict] = None,
                 state_dict: Optional[Dict[str, np.ndarray]] = None, weights_from: Optional[tuple] = None):
        """Extra keyword arguments over the reference: `dtype` — 'x3' (the default: fp32 activations, every conv GEMM
        as three fp16 MFMAs on hi/lo split operands; meets the reference fp32 path's 1e-3 px / score bar, DESIGN.md
        §3), 'f16' (opt-in throughput mode: fp16 storage + fp32 accumulate, ~0.6 px / 3e-3 off the fp32 path),
        'f32' (exact-f32 MFMA), or 'i8' / 'f8' = the PTQ plans, which need calibrated `qparams`; see
        optimization.quantization.PostTrainingQuantizer), `seed` of the synthetic weights used when no `model_path`
        is given, `weights_blob` = an already packed model (e.g. received over an RCCL broadcast from rank 0), and
        `state_dict` = weights already in memory, `weights_from` = (rccl comm, root): receive the root rank's model
        over RCCL, or a yolomi Runtime that already received it (yolomi.dist.rccl_broadcast_model)."""
        self.task = task
        self.size = size
        self.device = device or self._get_default_device()
        self.verbose = verbose
        self.model_path = model_path
        self.dtype = dtype
        self.seed = seed
        self._blob = weights_blob
        self._qparams = qparams
        self._sd = state_dict
        self._weights_from = weights_from
        self.optimization_history: List[Dict[str, Any]] = []
        # batch-sharded multi-GPU (yolomi.dist.enable_global_rule): callable x -> (1,) device max of the GLOBAL batch
        self.global_batch_max = None
        self._mask_cap = 64  # segment: mask slots per image enqueued before the sync (grows on demand)
        self._validate_inputs()
        self.model = self._load_model()
        self.original_model = None
        logger.info(f"YOLO11 model initialized: task={task}, size={size}, device={self.device}")

    def _get_default_device(self) -> str:
        return "cuda" if torch.cuda.is_available() else "cpu"

    def _validate_inputs(self):
        if self.task not in self.SUPPORTED_TASKS:
            raise ValueError(f"Unsupported task: {self.task}. Supported: {list(self.SUPPORTED_TASKS.keys())}")
        if self.size not in self.SUPPORTED_SIZES:
            raise ValueError(f"Unsupported size: {self.size}. Supported: {self.SUPPORTED_SIZES}")
        if self.task not in self.HIP_TASKS:
            raise NotImplementedError(f"task {self.task!r} has no MI355X plan (supported: {self.HIP_TASKS})")

    def _load_model(self) -> _ModelHandle:
        dev = torch.device(self.device)
        if dev.type != "cuda":
            raise RuntimeError(f"YOLO11Model runs on MI355X (gfx950) only; device {self.device!r} has no HIP path")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self._dev = dev
        try:
            if self._blob is not None or self._weights_from is not None:
                sd = self._sd or {}
            elif self._sd is not None:
                sd = self._sd
            elif self.model_path:
                sd = _load_state_dict(Path(self.model_path))
            else:  # the reference fetches yolo11{size}.pt by name; offline we synthesise weights of that graph
                sd = synth_weights(self.size, self.task, self.seed)
            nc = 80
            if sd and self._blob is None:  # the checkpoint decides the architecture, as YOLO(model_path) does
                from yolomi.arch import infer_arch
                scale, task, nc = infer_arch(sd)
                if (scale, task) != (self.size, self.task):
                    logger.warning(f"{self.model_path or 'state_dict'} holds a yolo11{scale} {task} model "
                                   f"(nc={nc}); using it instead of size={self.size!r} task={self.task!r}")
                    self.size, self.task = scale, task
            engine = Engine(self.size, self.task, sd, dev, self.dtype, blob=self._blob, qparams=self._qparams, nc=nc,
                            receive=self._weights_from)
            names = COCO_NAMES if nc == 80 else {i: f"class{i}" for i in range(nc)}
        except Exception as e:
            logger.error(f"Failed to load model: {e}")
            raise
        return _ModelHandle(sd, engine, names)

    # ------------------------------------------------------------------ hot path
    def _as_batch(self, source, imgsz: int = 640):
        """(batch tensor on the device, LoadTensor eps, image-source info or None).  Tensors follow LoadTensor; paths,
        directories, HWC uint8 BGR ndarrays and PIL images are letterboxed on the GPU (yolomi/preprocess.py)."""
        if isinstance(source, (list, tuple)) and source and all(isinstance(s, torch.Tensor) for s in source):
            source = torch.stack(list(source))
        if not isinstance(source, torch.Tensor):
            from yolomi.preprocess import expand_sources, letterbox_batch
            imgs, paths = expand_sources(source)
            stream = torch.cuda.current_stream(self._dev).cuda_stream
            im, shapes = letterbox_batch(self.model.engine.rt, imgs, self._dev, imgsz=imgsz, stream=stream)
            return im, torch.finfo(torch.float32).eps, (imgs, paths, shapes)
        im = source
        if im.dim() != 4:
            if im.dim() != 3:
                raise ValueError("torch.Tensor inputs should be BCHW i.e. shape(1, 3, 640, 640)")
            im = im.unsqueeze(0)
        if im.shape[1] != 3:
            raise ValueError(f"expected 3 input channels, got shape {tuple(im.shape)}")
        if im.shape[2] % 32 or im.shape[3] % 32:
            raise ValueError(f"torch.Tensor inputs should be BCHW divisible by stride 32, got {tuple(im.shape)}")
        if not im.is_floating_point():
            raise TypeError(f"tensor source must be floating point, got {im.dtype}")
        eps = torch.finfo(im.dtype).eps
        if im.device != self._dev:
            im = im.to(self._dev)
        im = im.float().contiguous()
        return im, eps, None

    def predict(self, source, **kwargs) -> List[Results]:
        conf = float(kwargs.get("conf", 0.25))
        iou = float(kwargs.get("iou", 0.7))
        max_det = int(kwargs.get("max_det", 300))
        classes = kwargs.get("classes", None)
        agnostic = bool(kwargs.get("agnostic_nms", False))
        t0 = time.perf_counter()
        im, eps, imsrc = self._as_batch(source, int(kwargs.get("imgsz", 640)))
        t1 = time.perf_counter()
        eng = self.model.engine
        bm = self.global_batch_max(im) if self.global_batch_max is not None and imsrc is None else None
        B = im.shape[0]
        names = self.model.names
        if self.task != "segment" and imsrc is None:
            # Asynchronous call: the NMS kernel writes this call's rows AND its B detection counts (the int32 words
            # behind the rows) into a fresh buffer, so no host sync is needed here: the Results read the counts on
            # first access (one device->host read shared by the call's B Results), and back-to-back predict() calls
            # queue their forwards with no host gap between them.
            out, cnt = eng.rows_buffer(B, max_det)
            eng.run(im, conf=conf, iou=iou, max_det=max_det, classes=classes, agnostic=agnostic, in_eps=eps,
                    batch_max=bm, dets_out=out, counts_after=True)
            lazy = LazyCounts(cnt, torch.cuda.current_stream(im.device))
            if kwargs.get("sync", False):  # per-call latency loops: return only once the forward is done
                lazy[0]
            speed = {"preprocess": (t1 - t0) * 1e3, "inference": (time.perf_counter() - t1) * 1e3,
                     "postprocess": 0.0}  # host time of the calls (the forward itself runs asynchronously)
            return [Results.from_batch(im, b, names, out, lazy, path=f"image{b}.jpg", speed=speed) for b in range(B)]
        # the NMS kernel writes this call's rows straight into a fresh tensor (the Results keep views into it)
        out = torch.empty((B, max_det, 6 + eng.nm), dtype=torch.float32, device=im.device)
        dets, counts = eng.run(im, conf=conf, iou=iou, max_det=max_det, classes=classes, agnostic=agnostic,
                               in_eps=eps, batch_max=bm, dets_out=out)
        masks = None
        if self.task == "segment":  # process_mask(upsample=True) on the GPU, in letterboxed coordinates
            # the masks of the first `cap` detections per image are enqueued behind the forward, reading the device
            # counts, so ONE device→host read returns counts and non-empty flags; a batch with more detections per
            # image than `cap` takes the exact-size two-read path (and raises `cap` for the next call)
            # Memory: the slot buffer is B x cap x H x W bytes, so it is only used within
            # YM_MASK_BUDGET_MB (256 MB by default; larger batches take the exact-size path), `cap` follows the recent
            # detection counts down as well as up (1.25x the last maximum rounded up to 16, 16..max_det: a steady
            # stream of batches keeps its slots over half full, so no compaction copy runs), and a mostly empty slot
            # buffer is compacted before the Results views are taken, so results kept by the caller retain at most
            # twice the bytes of their masks.
            H, W = im.shape[2:]
            cap = min(self._mask_cap, max_det)
            budget = int(os.environ.get("YM_MASK_BUDGET_MB", "256")) << 20
            fl = None
            if B * cap * H * W <= budget:
                mslots, flags = eng.masks_slots(out, counts[:B], cap, H, W)
                fl = flags.tolist()  # the device→host sync of a segment predict call
                n = fl[B * cap:]
            else:
                n = counts[:B].tolist()
            if fl is not None and max(n) <= cap:
                masks, keep = mslots, fl
                offs = [b * cap for b in range(B + 1)]
                if 2 * sum(n) < B * cap:  # compact the kept slots: one gather
                    rows = [b * cap + i for b in range(B) for i in range(n[b])]
                    masks = mslots.reshape(B * cap, H, W).index_select(
                        0, torch.tensor(rows, dtype=torch.long, device=mslots.device))
                    keep = [fl[r] for r in rows]
                    offs = [0]
                    for b in range(B):
                        offs.append(offs[-1] + n[b])
            else:
                masks, nonempty, offs = eng.masks(out, n, H, W)
                keep = nonempty.tolist()
            self._mask_cap = max(16, min(max_det, -(-(5 * max(max(n), 1)) // 64) * 16))  # ceil(1.25 max / 16) * 16
        else:
            n = counts[:B].tolist()  # the device→host sync of a predict call
        if imsrc is not None:  # ops.scale_boxes back to each original image
            from yolomi.preprocess import scale_boxes
            for b in range(B):
                if n[b]:
                    scale_boxes(im.shape[2:], out[b, : n[b], :4], imsrc[2][b])
        t2 = time.perf_counter()
        speed = {"preprocess": (t1 - t0) * 1e3, "inference": (t2 - t1) * 1e3, "postprocess": 0.0}
        if masks is None:
            if imsrc is None:
                return [Results.from_batch(im, b, names, out, n[b], path=f"image{b}.jpg", speed=speed)
                        for b in range(B)]
            return [Results.from_image(imsrc[0][b], imsrc[1][b], names, out[b, : n[b], :6], speed=speed)
                    for b in range(B)]
        res = []  # Segment: the predictor keeps only non-empty masks
        mb = masks.view(torch.bool).reshape(-1, H, W)  # the kernel writes 0/1 bytes: a bool view, no copy
        for b in range(B):
            kb = keep[offs[b]:offs[b] + n[b]]
            if all(kb) and imsrc is None:  # the common case: boxes, masks and input slice as views taken on access
                res.append(Results.from_batch(im, b, names, out, n[b], path=f"image{b}.jpg", speed=speed, masks=mb,
                                              moff=offs[b]))
                continue
            if all(kb):  # every kept detection has a mask pixel — views, no gathers
                bx, mk = out[b, :n[b], :6], mb[offs[b]:offs[b] + n[b]]
            else:
                sel = torch.tensor([i for i, k in enumerate(kb) if k], dtype=torch.long, device=out.device)
                bx = out[b].index_select(0, sel)[:, :6]
                mk = mb[offs[b]:offs[b] + n[b]].index_select(0, sel)
            if imsrc is None:
                res.append(Results(im[b], names, bx, path=f"image{b}.jpg", speed=speed, masks=mk))
            else:
                res.append(Results.from_image(imsrc[0][b], imsrc[1][b], names, bx, speed=speed, masks=mk))
        return res

    def __call__(self, source, **kwargs):
        return self.predict(source, **kwargs)

    # ------------------------------------------------------------------ reference surface
    def get_model_info(self) -> Dict[str, Any]:
        info = {
            "task": self.task,
            "size": self.size,
            "device": self.device,
            "model_path": self.model_path,
            "optimization_history": self.optimization_history,
        }
        params = list(self.model.model.parameters())
        total = sum(p.numel() for p in params)
        info.update({
            "total_parameters": total,
            "trainable_parameters": sum(p.numel() for p in params if p.requires_grad),
            "model_size_mb": total * 4 / (1024 * 1024),
        })
        return info

    def benchmark(self, data_source, num_runs: int = 100, warmup_runs: int = 10) -> Dict[str, float]:
        """Same protocol as the reference (core/model.py:253-291): warm-up, then wall-clock per predict()."""
        for _ in range(warmup_runs):
            _ = self.predict(data_source, verbose=False, sync=True)
        times = []
        for _ in range(num_runs):  # sync=True: each call's wall clock covers its whole forward (predict is async)
            start = time.time()
            _ = self.predict(data_source, verbose=False, sync=True)
            times.append(time.time() - start)
        avg = sum(times) / len(times)
        return {"avg_inference_time": avg, "min_inference_time": min(times), "max_inference_time": max(times),
                "fps": 1.0 / avg}

    def train(self, *a, **k):
        raise NotImplementedError("training is out of scope for the MI355X inference path (SURVEY §2)")

    val = export = train

    def __repr__(self) -> str:
        return (f"YOLO11Model(task={self.task}, size={self.size}, "
                f"device={self.device}, optimized={len(self.optimization_history) > 0})")


class YOLO11Factory:
    @staticmethod
    def create_detector(size: str = "n", **kwargs) -> YOLO11Model:
        return YOLO11Model(task="detect", size=size, **kwargs)

    @staticmethod
    def create_segmenter(size: str = "n", **kwargs) -> YOLO11Model:
        return YOLO11Model(task="segment", size=size, **kwargs)

    @staticmethod
    def create_classifier(size: str = "n", **kwargs) -> YOLO11Model:
        return YOLO11Model(task="classify", size=size, **kwargs)

    @staticmethod
    def create_pose_estimator(size: str = "n", **kwargs) -> YOLO11Model:
        return YOLO11Model(task="pose", size=size, **kwargs)

    @staticmethod
    def create_obb_detector(size: str = "n", **kwargs) -> YOLO11Model:
        return YOLO11Model(task="obb", size=size, **kwargs)
