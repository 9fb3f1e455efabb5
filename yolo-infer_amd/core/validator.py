"""YOLO11Validator — the `benchmark_speed` surface of /root/reference/core/validator.py on MI355X.

`benchmark_speed` (reference `core/validator.py:158-221`) sweeps image sizes x batch sizes, times
`YOLO11Model.benchmark` (100 predicts after 10 warm-ups, `core/model.py:253-291`), adds `images_per_second`
(`validator.py:209`), summarises (`:363-386`) and writes `benchmark_results.json` + `benchmark_summary.txt`
(`:509-545`) — same schema here.  Dataset validation (`validate`/`compare_models`/`cross_validate`) is out of scope
(needs datasets and the Ultralytics val loop); `evaluate_detections` is the offline mAP used instead.
"""
from __future__ import annotations

import json
import logging
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Optional, Union

import torch

from .model import YOLO11Model

logger = logging.getLogger(__name__)


class YOLO11Validator:
    def __init__(self, model: Union[YOLO11Model, str, Path], device: Optional[str] = None,
                 output_dir: Optional[Union[str, Path]] = None):
        self.device = device or ("cuda" if torch.cuda.is_available() else "cpu")
        self.output_dir = (Path(output_dir) if output_dir
                           else Path("experiments") / f"val_{datetime.now().strftime('%Y%m%d_%H%M%S')}")
        self.output_dir.mkdir(parents=True, exist_ok=True)
        if isinstance(model, (str, Path)):
            self.model = YOLO11Model(model_path=model, device=self.device)
        elif hasattr(model, "benchmark") and hasattr(model, "get_model_info"):
            self.model = model
        else:
            raise ValueError("Model must be YOLO11Model instance or path to weights")
        self.validation_history: List[Dict[str, Any]] = []
        self.benchmark_results: Dict[str, Any] = {}
        self._setup_logging()

    def _setup_logging(self):
        fh = logging.FileHandler(self.output_dir / "validation.log")
        fh.setLevel(logging.INFO)
        fh.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s"))
        logger.addHandler(fh)

    def benchmark_speed(self, test_data, num_runs: int = 100, warmup_runs: int = 10,
                        batch_sizes: List[int] = [1, 8, 16, 32],
                        image_sizes: List[int] = [320, 640, 1280]) -> Dict[str, Any]:
        results: Dict[str, Any] = {"device": self.device, "model_info": self.model.get_model_info(),
                                   "configurations": [], "summary": {}}
        for img_size in image_sizes:
            for batch_size in batch_sizes:
                # reference quirk kept: a caller tensor is reused as-is for every (B, S) label (validator.py:193-194)
                if isinstance(test_data, torch.Tensor):
                    test_input = test_data
                else:
                    test_input = torch.randn(batch_size, 3, img_size, img_size, device=self.device)
                cfg = self.model.benchmark(data_source=test_input, num_runs=num_runs, warmup_runs=warmup_runs)
                cfg.update({"batch_size": batch_size, "image_size": img_size,
                            "images_per_second": batch_size * cfg["fps"]})
                results["configurations"].append(cfg)
        results["summary"] = self._calculate_benchmark_summary(results["configurations"])
        self._save_benchmark_results(results)
        self.benchmark_results = results
        return results

    def _calculate_benchmark_summary(self, configurations: List[Dict]) -> Dict[str, Any]:
        if not configurations:
            return {}
        fps = [c["fps"] for c in configurations]
        lat = [c["avg_inference_time"] for c in configurations]
        thr = [c.get("images_per_second", 0) for c in configurations]
        summary = {"best_fps": max(fps), "avg_fps": sum(fps) / len(fps), "best_latency": min(lat),
                   "avg_latency": sum(lat) / len(lat), "best_throughput": max(thr),
                   "total_configurations_tested": len(configurations)}
        summary["best_configuration"] = configurations[fps.index(summary["best_fps"])]
        return summary

    def _save_benchmark_results(self, results: Dict[str, Any]):
        with open(self.output_dir / "benchmark_results.json", "w") as f:
            json.dump(results, f, indent=2, default=str)
        s = results["summary"]
        with open(self.output_dir / "benchmark_summary.txt", "w") as f:
            f.write("YOLO11 Benchmark Summary\n" + "=" * 50 + "\n\n")
            f.write(f"Device: {results['device']}\n")
            f.write(f"Total configurations tested: {s['total_configurations_tested']}\n\n")
            f.write("Performance Summary:\n" + "-" * 20 + "\n")
            f.write(f"Best FPS: {s['best_fps']:.2f}\n")
            f.write(f"Average FPS: {s['avg_fps']:.2f}\n")
            f.write(f"Best Latency: {s['best_latency']:.4f} seconds\n")
            f.write(f"Average Latency: {s['avg_latency']:.4f} seconds\n")
            f.write(f"Best Throughput: {s['best_throughput']:.2f} images/second\n\n")
            b = s.get("best_configuration")
            if b:
                f.write("Best Configuration:\n" + "-" * 20 + "\n")
                f.write(f"  Batch Size: {b['batch_size']}\n")
                f.write(f"  Image Size: {b['image_size']}\n")
                f.write(f"  FPS: {b['fps']:.2f}\n")
                f.write(f"  Latency: {b['avg_inference_time']:.4f} seconds\n")

    def evaluate_detections(self, predictions, ground_truth) -> Dict[str, float]:
        """mAP50 / mAP75 / mAP50-95 of per-image (n,6) detections against (m,6) ground truth (yolomi.metrics)."""
        from yolomi.metrics import evaluate
        to_np = lambda t: t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else t  # noqa: E731
        return evaluate([to_np(p) for p in predictions], [to_np(g) for g in ground_truth])
