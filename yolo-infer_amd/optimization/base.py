"""Optimizer plugin interface — the reference's `optimization/base.py` (`BaseOptimizer` :18-229,
`QuantizationOptimizer` :232-261, `OptimizationRegistry` :407-439) for the one optimizer on the hot path (PTQ).
Pruning/distillation bases are abstract-only in the reference and out of scope here."""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, List, Optional

import torch


class BaseOptimizer(ABC):
    def __init__(self, model: Any, config: Optional[Dict[str, Any]] = None, device: Optional[str] = None):
        self.original_model = model
        self.optimized_model = None
        self.config = config or {}
        self.device = device or self._get_default_device()
        self.optimization_metrics: Dict[str, Any] = {}
        self.optimization_history: List[Dict[str, Any]] = []

    def _get_default_device(self) -> str:
        return "cuda" if torch.cuda.is_available() else "cpu"

    @abstractmethod
    def optimize(self, **kwargs) -> Any:
        ...

    @abstractmethod
    def evaluate(self, test_data: Any, metrics: Optional[List[str]] = None) -> Dict[str, float]:
        ...

    @abstractmethod
    def get_optimization_info(self) -> Dict[str, Any]:
        ...


class QuantizationOptimizer(BaseOptimizer):
    SUPPORTED_BACKENDS = ["fbgemm", "qnnpack", "onednn"]
    SUPPORTED_DTYPES = [torch.qint8, torch.quint8, torch.qint32]

    def __init__(self, model: Any, config: Optional[Dict[str, Any]] = None, device: Optional[str] = None):
        super().__init__(model, config, device)
        self.quantization_backend = self.config.get("backend", "qnnpack")
        self.quantization_dtype = self.config.get("dtype", torch.qint8)
        self.calibration_data = None

    def set_calibration_data(self, calibration_data: Any) -> None:
        self.calibration_data = calibration_data

    @abstractmethod
    def _prepare_model_for_quantization(self) -> Any:
        ...

    @abstractmethod
    def _calibrate_model(self, model: Any, calibration_loader: Any = None) -> Any:
        ...


class OptimizationRegistry:
    _optimizers: Dict[str, type] = {}

    @classmethod
    def register(cls, name: str, optimizer_class: type) -> None:
        cls._optimizers[name] = optimizer_class

    @classmethod
    def get(cls, name: str) -> type:
        if name not in cls._optimizers:
            raise ValueError(f"Unknown optimizer: {name}. Available: {list(cls._optimizers)}")
        return cls._optimizers[name]

    @classmethod
    def list_optimizers(cls) -> List[str]:
        return list(cls._optimizers)
