"""SpeedBenchmark — the timing loop of /root/reference/benchmarks/speed_benchmark.py on MI355X.

Same protocol and result keys as the reference: `_benchmark_inference` (`speed_benchmark.py:307-350`) puts the
model in eval mode, runs warm-up predicts, then times each `predict(test_input)` with wall clock and reports
avg/min/max/stdev, `fps = 1/avg` and `throughput = B/avg`; `benchmark_model_sizes` (`:61-122`) sweeps sizes x
image sizes x batch sizes; `benchmark_quantization` (`:124-209`) is the PTQ A/B (`speedup = t_original / t_quant`,
`:191`); `benchmark_throughput` (`:211-305`) is the sustained loop, with the reference's resource monitor
(`:243-244`) sampling AMD SMI instead of GPUtil (utils/helpers.py).
"""
from __future__ import annotations

import argparse
import json
import logging
import platform
import statistics
import time
from pathlib import Path
from typing import Any, Dict, List

import torch

from core.model import YOLO11Model
from optimization.quantization.quantizers import create_quantizer
from utils.helpers import ResourceMonitor

logger = logging.getLogger(__name__)


def _device_info() -> Dict[str, Any]:
    info = {"platform": platform.platform(), "python": platform.python_version(), "torch": torch.__version__,
            "hip": getattr(torch.version, "hip", None), "cuda_available": torch.cuda.is_available()}
    if torch.cuda.is_available():
        info["gpu_count"] = torch.cuda.device_count()
        info["gpu_name"] = torch.cuda.get_device_name(0)
    return info


class SpeedBenchmark:
    def __init__(self, output_dir: str = "benchmark_results", warmup_runs: int = 10, benchmark_runs: int = 100):
        self.output_dir = Path(output_dir)
        self.output_dir.mkdir(parents=True, exist_ok=True)
        self.warmup_runs = warmup_runs
        self.benchmark_runs = benchmark_runs
        self.system_info = _device_info()

    def benchmark_model_sizes(self, task: str = "detect", sizes: List[str] = ["n", "s", "m", "l", "x"],
                              image_sizes: List[int] = [320, 640, 1280],
                              batch_sizes: List[int] = [1, 4, 8, 16]) -> Dict[str, Any]:
        results = {"task": task, "system_info": self.system_info, "configurations": [], "summary": {}}
        for size in sizes:
            model = YOLO11Model(task=task, size=size)
            for img_size in image_sizes:
                for batch_size in batch_sizes:
                    test_input = torch.randn(batch_size, 3, img_size, img_size)
                    if torch.cuda.is_available():
                        test_input = test_input.cuda()
                    metrics = self._benchmark_inference(model, test_input)
                    results["configurations"].append({"model_size": size, "image_size": img_size,
                                                      "batch_size": batch_size, **metrics})
        results["summary"] = self._calculate_summary(results["configurations"])
        self._save_results(results, "model_sizes_benchmark.json")
        return results

    def benchmark_quantization(self, model_size: str = "n", task: str = "detect",
                               quantization_methods: List[str] = ["dynamic", "ptq"], image_size: int = 640,
                               batch_size: int = 1, original_dtype: str = "f32") -> Dict[str, Any]:
        """The reference's quantization A/B (`speed_benchmark.py:124-209`): time the original model, then each
        method's quantized model on the same randn input, `speedup = original avg / quantized avg`.  'ptq' calibrates
        on ten copies of the test input (`:180-183`) with the quantizer's default config (qnnpack int8); 'ptq_fp8'
        is the same flow on the fp8 e4m3 plan (BASELINE config 4).  A method that fails is recorded as
        {'error': ...} like the reference's except path (`:196-201`): 'dynamic' is one (a no-op on this conv-only
        graph).  `original_dtype` is the original model's plan: 'f32' by default — the exact-f32 plan,
        the reference's FP32 model (`:157-158`), so `speedup` is the reference's quantity; 'f16' / 'x3' time a
        faster float plan instead."""
        logger.info(f"Benchmarking quantization methods: {quantization_methods}")
        results = {"model_size": model_size, "task": task, "image_size": image_size, "batch_size": batch_size,
                   "original_dtype": original_dtype, "system_info": self.system_info, "methods": {}}
        original_model = YOLO11Model(task=task, size=model_size, dtype=original_dtype)
        test_input = torch.randn(batch_size, 3, image_size, image_size)
        if torch.cuda.is_available():
            test_input = test_input.cuda()
        original_metrics = self._benchmark_inference(original_model, test_input)
        results["methods"]["original"] = original_metrics
        for method in quantization_methods:
            logger.info(f"Benchmarking quantization method: {method}")
            try:
                if method == "ptq_fp8":
                    quantizer = create_quantizer("ptq", original_model, {"backend": "fp8"})
                else:
                    quantizer = create_quantizer(method, original_model)
                quantizer.set_calibration_data([test_input for _ in range(10)])
                quantized_model = quantizer.optimize()
                quantized_metrics = self._benchmark_inference(quantized_model, test_input)
                quantized_metrics.update({
                    "speedup": original_metrics["avg_inference_time"] / quantized_metrics["avg_inference_time"],
                    "optimization_info": quantizer.get_optimization_info()})
                results["methods"][method] = quantized_metrics
            except Exception as e:  # the reference records the failure and moves on (:196-201)
                logger.error(f"Failed to benchmark quantization method {method}: {e}")
                results["methods"][method] = {"error": str(e)}
        self._save_results(results, "quantization_benchmark.json")
        return results

    def benchmark_throughput(self, model_size: str = "n", task: str = "detect", duration_seconds: float = 60,
                             image_size: int = 640, batch_size: int = 1) -> Dict[str, Any]:
        model = YOLO11Model(task=task, size=model_size)
        test_input = torch.randn(batch_size, 3, image_size, image_size)
        if torch.cuda.is_available():
            test_input = test_input.cuda()
        monitor = ResourceMonitor(interval=1.0)  # reference :243-244
        monitor.start_monitoring()
        for _ in range(self.warmup_runs):
            model.predict(test_input, verbose=False, sync=True)
        start = time.time()
        count, times = 0, []
        while time.time() - start < duration_seconds:
            t0 = time.time()
            model.predict(test_input, verbose=False, sync=True)
            times.append(time.time() - t0)
            count += 1
        total = time.time() - start
        monitor.stop_monitoring()
        fps = count / total
        results = {"model_size": model_size, "task": task, "image_size": image_size, "batch_size": batch_size,
                   "duration_seconds": total, "total_inferences": count,
                   "avg_inference_time": statistics.mean(times), "fps": fps, "images_per_second": fps * batch_size,
                   "resource_usage": monitor.get_average_usage(), "system_info": self.system_info}
        monitor.save_history(self.output_dir / "resource_history.json")
        self._save_results(results, "throughput_benchmark.json")
        return results

    def _benchmark_inference(self, model: YOLO11Model, test_input: torch.Tensor) -> Dict[str, float]:
        model.model.eval()
        with torch.no_grad():
            for _ in range(self.warmup_runs):
                model.predict(test_input, verbose=False, sync=True)
        times = []
        with torch.no_grad():
            for _ in range(self.benchmark_runs):
                t0 = time.time()
                model.predict(test_input, verbose=False, sync=True)
                times.append(time.time() - t0)
        avg = statistics.mean(times)
        return {"avg_inference_time": avg, "min_inference_time": min(times), "max_inference_time": max(times),
                "std_inference_time": statistics.stdev(times) if len(times) > 1 else 0.0, "fps": 1.0 / avg,
                "throughput": test_input.shape[0] / avg}

    def _calculate_summary(self, configurations: List[Dict]) -> Dict[str, Any]:
        if not configurations:
            return {}
        fps = [c["fps"] for c in configurations]
        thr = [c["throughput"] for c in configurations]
        return {"best_fps": max(fps), "worst_fps": min(fps), "avg_fps": statistics.mean(fps),
                "best_throughput": max(thr), "worst_throughput": min(thr), "avg_throughput": statistics.mean(thr),
                "total_configurations": len(configurations)}

    def _save_results(self, results: Dict[str, Any], filename: str):
        with open(self.output_dir / filename, "w") as f:
            json.dump(results, f, indent=2, default=str)


def main(argv=None):
    ap = argparse.ArgumentParser(description="YOLO11 speed benchmark (MI355X)")
    ap.add_argument("--sizes", nargs="+", default=["n"])
    ap.add_argument("--image-sizes", nargs="+", type=int, default=[640])
    ap.add_argument("--batch-sizes", nargs="+", type=int, default=[1, 8])
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--runs", type=int, default=100)
    ap.add_argument("--output-dir", default="benchmark_results")
    a = ap.parse_args(argv)
    sb = SpeedBenchmark(a.output_dir, a.warmup, a.runs)
    res = sb.benchmark_model_sizes(sizes=a.sizes, image_sizes=a.image_sizes, batch_sizes=a.batch_sizes)
    print(json.dumps(res["summary"], indent=2))


if __name__ == "__main__":
    main()
