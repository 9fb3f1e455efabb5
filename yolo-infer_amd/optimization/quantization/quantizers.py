"""PostTrainingQuantizer on MI355X — the reference's `optimization/quantization/quantizers.py:24-308` (PTQ) and
`create_quantizer` (:860-889), with the same plugin surface (`set_calibration_data`, `optimize`,
`get_optimization_info`, `evaluate`, config keys `backend` (default 'qnnpack', :42; also 'fbgemm', and 'fp8' = the
e4m3 plan of BASELINE config 4), `num_calibration_batches` (100, :41), `dtype`).

`optimize()` follows the reference's prepare → calibrate → convert (:66-77), re-designed for the GPU runtime:
  * prepare: the exact-f32 plan of the model (the float model torch.ao would observe);
  * calibrate (:146-177): up to `num_calibration_batches` forwards of the calibration batches; the torch.ao observers
    of the backend's default qconfig (:124-131) see every stored tensor and every conv output (yolomi.quant);
  * convert (:77): an int8 plan (csrc/ym_conv_i8.hip: int8 MFMA convs, int32 accumulation, requantisation).
It returns a `YOLO11Model` whose predict() runs the int8 plan.  Unlike the reference there is no silent fallback to
the float model (:79-85, :217-220): a failure raises.  Numerics: DESIGN.md §9 / oracle/quant.py.
Dynamic quantisation (a no-op on this conv-only graph) and QAT (training) are out of scope.
"""
from __future__ import annotations

import logging
import time
from typing import Any, Dict, List, Optional

import torch

from ..base import OptimizationRegistry, QuantizationOptimizer

logger = logging.getLogger(__name__)


class PostTrainingQuantizer(QuantizationOptimizer):
    def __init__(self, model: Any, config: Optional[Dict[str, Any]] = None, device: Optional[str] = None):
        super().__init__(model, config, device)
        self.num_calibration_batches = self.config.get("num_calibration_batches", 100)
        self.quantization_backend = self.config.get("backend", "qnnpack")
        self.quantization_dtype = self.config.get("dtype", torch.qint8)
        self.qparams: Optional[Dict] = None
        self.calibration_seconds = 0.0

    def optimize(self, calibration_loader: Any = None, **kwargs) -> Any:
        if calibration_loader is None and self.calibration_data is None:
            raise ValueError("Calibration data is required for post-training quantization")
        calibration_loader = calibration_loader or self.calibration_data
        if self.quantization_backend not in ("qnnpack", "fbgemm", "fp8"):
            raise ValueError(f"backend {self.quantization_backend!r}: the int8 runtime restates qnnpack and fbgemm "
                             f"(and 'fp8', the e4m3 plan)")
        logger.info("Starting post-training quantization...")
        f32 = self._prepare_model_for_quantization()
        t0 = time.perf_counter()
        self.qparams = self._calibrate_model(f32, calibration_loader)
        self.calibration_seconds = time.perf_counter() - t0
        self.optimized_model = self._convert()
        self._record_optimization_metrics()
        logger.info("Post-training quantization completed")
        return self.optimized_model

    def _source(self):
        m = self.original_model
        if not hasattr(m, "model") or not hasattr(m.model, "engine"):
            raise TypeError("PostTrainingQuantizer expects a core.model.YOLO11Model")
        return m

    def _prepare_model_for_quantization(self) -> Any:
        from core.model import YOLO11Model
        src = self._source()
        sd = src.model.state_dict_numpy()
        return YOLO11Model(task=src.task, size=src.size, device=src.device, dtype="f32", state_dict=sd)

    def _calibrate_model(self, model: Any, calibration_loader: Any = None) -> Dict:
        from yolomi.quant import calibrate
        batches: List[torch.Tensor] = []
        for i, batch in enumerate(calibration_loader):
            if i >= self.num_calibration_batches:
                break
            images = batch[0] if isinstance(batch, (list, tuple)) else batch
            if not isinstance(images, torch.Tensor):
                raise TypeError("calibration batches must be image tensors (B,3,H,W)")
            batches.append(images)
        return calibrate(model.model.engine, batches, self.quantization_backend)

    def _convert(self) -> Any:
        from core.model import YOLO11Model
        src = self._source()
        q = YOLO11Model(task=src.task, size=src.size, device=src.device,
                        dtype="f8" if self.quantization_backend == "fp8" else "i8", qparams=self.qparams,
                        state_dict=src.model.state_dict_numpy())
        q.optimization_history = list(getattr(src, "optimization_history", [])) + [
            {"type": "post_training_quantization", "backend": self.quantization_backend}]
        q.original_model = src
        return q

    def evaluate(self, test_data: Any, metrics: Optional[List[str]] = None) -> Dict[str, float]:
        """mAP50-95 of the int8 model's detections against the float model's (pseudo ground truth) on `test_data`
        image batches — the offline stand-in for the reference's `.val()` (:228-237)."""
        import numpy as np
        from yolomi.metrics import evaluate as ev
        if self.optimized_model is None:
            raise ValueError("No optimized model to evaluate. Run optimize() first.")
        preds, gts = [], []
        for x in test_data:
            preds += [r.boxes.data.cpu().numpy().astype(np.float64) for r in self.optimized_model.predict(x)]
            gts += [r.boxes.data.cpu().numpy().astype(np.float64) for r in self.original_model.predict(x)]
        m = ev(preds, gts)
        return {"mAP50-95": m["map"], "mAP50": m["map50"], "mAP75": m["map75"], "model_size_mb": self._get_model_size()}

    def _get_model_size(self) -> float:
        if self.optimized_model is None:
            return 0.0
        return len(self.optimized_model.model.engine.blob) / (1024 * 1024)

    def _record_optimization_metrics(self):
        self.optimization_metrics = {
            "optimization_type": "post_training_quantization",
            "backend": self.quantization_backend,
            "dtype": str(self.quantization_dtype),
            "num_calibration_batches": self.num_calibration_batches,
            "model_size_mb": self._get_model_size(),
            "calibration_seconds": round(self.calibration_seconds, 3),
        }

    def get_optimization_info(self) -> Dict[str, Any]:
        return {
            "optimizer_type": "PostTrainingQuantizer",
            "config": self.config,
            "metrics": self.optimization_metrics,
            "quantization_backend": self.quantization_backend,
            "quantization_dtype": str(self.quantization_dtype),
        }


OptimizationRegistry.register("ptq", PostTrainingQuantizer)


def create_quantizer(quantization_type: str, model: Any, config: Optional[Dict[str, Any]] = None,
                     **kwargs) -> QuantizationOptimizer:
    quantizer_map = {"ptq": PostTrainingQuantizer}
    if quantization_type not in quantizer_map:
        raise ValueError(f"Unsupported quantization type: {quantization_type}. Supported types: "
                         f"{list(quantizer_map)} (dynamic quantisation is a no-op on this conv-only graph and QAT is "
                         f"training: out of scope, SURVEY §2.1)")
    return quantizer_map[quantization_type](model=model, config=config, **kwargs)
