"""GPU runs of the reference's timing surfaces on the HIP model: `YOLO11Validator.benchmark_speed`
(reference core/validator.py:158-221), `SpeedBenchmark._benchmark_inference` / `benchmark_model_sizes`
(benchmarks/speed_benchmark.py:61-122, 307-350) and the quantization A/B `benchmark_quantization` (:124-209).
Small run counts: these check the protocol and result schema on the real path, not the numbers."""
import json

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_validator_benchmark_speed_on_gpu(tmp_path):
    from core.model import YOLO11Model
    from core.validator import YOLO11Validator
    m = YOLO11Model(task="detect", size="n", device="cuda:0")
    v = YOLO11Validator(m, device="cuda:0", output_dir=tmp_path)
    r = v.benchmark_speed(None, num_runs=3, warmup_runs=1, batch_sizes=[1, 8], image_sizes=[320, 640])
    assert len(r["configurations"]) == 4
    for c in r["configurations"]:
        assert c["fps"] > 0 and c["min_inference_time"] <= c["avg_inference_time"] <= c["max_inference_time"]
        assert c["images_per_second"] == pytest.approx(c["batch_size"] * c["fps"])
    assert r["summary"]["total_configurations_tested"] == 4
    assert (tmp_path / "benchmark_results.json").exists()


def test_speed_benchmark_model_sizes_on_gpu(tmp_path):
    from benchmarks.speed_benchmark import SpeedBenchmark
    sb = SpeedBenchmark(str(tmp_path), warmup_runs=1, benchmark_runs=3)
    r = sb.benchmark_model_sizes(sizes=["n"], image_sizes=[320], batch_sizes=[1, 4])
    assert [c["batch_size"] for c in r["configurations"]] == [1, 4]
    for c in r["configurations"]:
        assert c["throughput"] == pytest.approx(c["batch_size"] / c["avg_inference_time"])
    assert r["summary"]["total_configurations"] == 2
    assert json.load(open(tmp_path / "model_sizes_benchmark.json"))["task"] == "detect"


def test_speed_benchmark_quantization_ab_on_gpu(tmp_path):
    """PTQ int8 and fp8 A/B against the FP32 (exact-f32 plan) model on one randn batch, as the reference times it;
    'dynamic' records an error entry like the reference's except path."""
    from benchmarks.speed_benchmark import SpeedBenchmark
    sb = SpeedBenchmark(str(tmp_path), warmup_runs=1, benchmark_runs=3)
    r = sb.benchmark_quantization(model_size="n", quantization_methods=["dynamic", "ptq", "ptq_fp8"],
                                  image_size=320, batch_size=2)
    meth = r["methods"]
    assert r["original_dtype"] == "f32"  # the reference times the FP32 model (speed_benchmark.py:157-158)
    assert meth["original"]["fps"] > 0
    assert "error" in meth["dynamic"]
    for k, backend in (("ptq", "qnnpack"), ("ptq_fp8", "fp8")):
        assert "error" not in meth[k], meth[k]
        assert meth[k]["speedup"] == pytest.approx(meth["original"]["avg_inference_time"] /
                                                   meth[k]["avg_inference_time"])
        assert meth[k]["optimization_info"]["quantization_backend"] == backend
    assert (tmp_path / "quantization_benchmark.json").exists()
    torch.cuda.synchronize()


def test_validator_benchmark_speed_large_batches(tmp_path):
    """benchmark_speed's sweep includes B = 16 and 32 (core/validator.py:188-189): the default plan at both, 640²."""
    from core.model import YOLO11Model
    from core.validator import YOLO11Validator
    m = YOLO11Model(task="detect", size="n", device="cuda:0")
    v = YOLO11Validator(m, device="cuda:0", output_dir=tmp_path)
    r = v.benchmark_speed(None, num_runs=2, warmup_runs=1, batch_sizes=[16, 32], image_sizes=[640])
    assert [c["batch_size"] for c in r["configurations"]] == [16, 32]
    assert all(c["images_per_second"] > 0 for c in r["configurations"])


def test_throughput_benchmark_resource_monitor(tmp_path):
    """benchmark_throughput's sustained loop with the resource monitor (reference speed_benchmark.py:243-244): AMD
    SMI samples of the GPUs land in resource_usage and resource_history.json."""
    from benchmarks.speed_benchmark import SpeedBenchmark
    sb = SpeedBenchmark(str(tmp_path), warmup_runs=1, benchmark_runs=2)
    r = sb.benchmark_throughput(model_size="n", duration_seconds=2.5, image_size=320, batch_size=2)
    assert r["total_inferences"] > 0 and r["images_per_second"] > 0
    ru = r["resource_usage"]
    assert "avg_cpu_percent" in ru
    hist = json.load(open(tmp_path / "resource_history.json"))
    assert len(hist) >= 1 and "gpu_usage" in hist[0]
    if hist[0]["gpu_usage"]:  # AMD SMI reachable on this box: per-GPU load averaged like GPUtil's
        assert "avg_gpu_0_load" in ru
