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
    """PTQ int8 and fp8 A/B against the f16 model on one randn batch; 'dynamic' records an error entry like the
    reference's except path."""
    from benchmarks.speed_benchmark import SpeedBenchmark
    sb = SpeedBenchmark(str(tmp_path), warmup_runs=1, benchmark_runs=3)
    r = sb.benchmark_quantization(model_size="n", quantization_methods=["dynamic", "ptq", "ptq_fp8"],
                                  image_size=320, batch_size=2)
    meth = r["methods"]
    assert meth["original"]["fps"] > 0
    assert "error" in meth["dynamic"]
    for k, backend in (("ptq", "qnnpack"), ("ptq_fp8", "fp8")):
        assert "error" not in meth[k], meth[k]
        assert meth[k]["speedup"] == pytest.approx(meth["original"]["avg_inference_time"] /
                                                   meth[k]["avg_inference_time"])
        assert meth[k]["optimization_info"]["quantization_backend"] == backend
    assert (tmp_path / "quantization_benchmark.json").exists()
    torch.cuda.synchronize()
