"""Resource monitoring for the sustained-throughput benchmark.

Restates the reference's `ResourceMonitor` (`/root/reference/utils/helpers.py:715-834`: a daemon thread sampling
CPU / host memory with psutil and the GPUs with GPUtil every `interval` seconds, averages, a JSON history) on MI355X:
GPUtil is NVIDIA-only (`helpers.py:49,746`), so the GPU side samples AMD SMI (`amdsmi`, SURVEY §2.1 Helpers):
graphics activity (the `load` GPUtil reports), VRAM used / total (MB), hotspot temperature (°C) and socket power (W).
Sampling failures leave `gpu_usage` empty for that point, as the reference's bare `except` does.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from pathlib import Path
from typing import Any, Dict, List, Optional, Union

import psutil

logger = logging.getLogger(__name__)


class _AmdSmi:
    """Lazily initialised AMD SMI handles (None when the library or the driver is unavailable)."""

    def __init__(self):
        self.smi, self.handles = None, []
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self.smi, self.handles = amdsmi, list(amdsmi.amdsmi_get_processor_handles())
        except Exception as e:  # no driver in a CPU container, or no amdsmi
            logger.debug(f"amdsmi unavailable: {e}")

    def sample(self) -> List[Dict[str, Any]]:
        out = []
        smi = self.smi
        for i, h in enumerate(self.handles):
            d: Dict[str, Any] = {"id": i}
            try:
                d["load"] = float(smi.amdsmi_get_gpu_activity(h)["gfx_activity"])
            except Exception:
                continue
            try:
                v = smi.amdsmi_get_gpu_vram_usage(h)
                d["memory_used"], d["memory_total"] = float(v["vram_used"]), float(v["vram_total"])
            except Exception:
                pass
            try:
                d["temperature"] = float(smi.amdsmi_get_temp_metric(h, smi.AmdSmiTemperatureType.HOTSPOT,
                                                                     smi.AmdSmiTemperatureMetric.CURRENT))
            except Exception:
                pass
            try:
                p = smi.amdsmi_get_power_info(h)
                w = p.get("socket_power", p.get("current_socket_power", p.get("average_socket_power")))
                if isinstance(w, (int, float)):
                    d["power_w"] = float(w)
            except Exception:
                pass
            out.append(d)
        return out

    def close(self):
        if self.smi is not None:
            try:
                self.smi.amdsmi_shut_down()
            except Exception:
                pass


class ResourceMonitor:
    """Monitor system resource usage (`helpers.py:715`): start_monitoring / stop_monitoring / get_current_usage /
    get_average_usage / save_history, same data-point keys."""

    def __init__(self, interval: float = 1.0):
        self.interval = interval
        self.monitoring = False
        self.history: List[Dict[str, Any]] = []

    def _point(self, smi: _AmdSmi) -> Dict[str, Any]:
        memory = psutil.virtual_memory()
        return {"timestamp": time.time(), "cpu_percent": psutil.cpu_percent(interval=0.1),
                "memory_percent": memory.percent, "memory_used": memory.used, "memory_total": memory.total,
                "gpu_usage": smi.sample()}

    def start_monitoring(self):
        self.monitoring = True
        self.history = []

        def loop():
            smi = _AmdSmi()
            try:
                while self.monitoring:
                    try:
                        self.history.append(self._point(smi))
                        if len(self.history) > 1000:  # the reference keeps the last 1000 points
                            self.history.pop(0)
                        time.sleep(self.interval)
                    except Exception as e:
                        logger.error(f"Error in resource monitoring: {e}")
                        break
            finally:
                smi.close()

        self.monitor_thread = threading.Thread(target=loop, daemon=True)
        self.monitor_thread.start()
        logger.info("Resource monitoring started")

    def stop_monitoring(self):
        self.monitoring = False
        if hasattr(self, "monitor_thread"):
            self.monitor_thread.join(timeout=2)
        logger.info("Resource monitoring stopped")

    def get_current_usage(self) -> Dict[str, Any]:
        return self.history[-1] if self.history else {}

    def get_average_usage(self, last_n: Optional[int] = None) -> Dict[str, float]:
        data = self.history[-last_n:] if last_n else self.history
        if not data:
            return {}
        res = {"avg_cpu_percent": sum(d["cpu_percent"] for d in data) / len(data),
               "avg_memory_percent": sum(d["memory_percent"] for d in data) / len(data)}
        if data[0].get("gpu_usage"):
            for i, _ in enumerate(data[0]["gpu_usage"]):
                for key, name in (("load", "load"), ("power_w", "power_w"), ("memory_used", "memory_used_mb"),
                                  ("temperature", "temperature")):
                    vals = [d["gpu_usage"][i][key] for d in data if i < len(d["gpu_usage"]) and key in d["gpu_usage"][i]]
                    if vals:
                        res[f"avg_gpu_{i}_{name}"] = sum(vals) / len(vals)
        return res

    def save_history(self, file_path: Union[str, Path]):
        file_path = Path(file_path)
        file_path.parent.mkdir(parents=True, exist_ok=True)
        with open(file_path, "w") as f:
            json.dump(self.history, f, indent=2)
        logger.info(f"Resource monitoring history saved to: {file_path}")
