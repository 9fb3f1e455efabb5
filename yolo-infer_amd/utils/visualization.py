"""Result writers: `save_detection_results(results, output_path, format)` with the reference's file formats
(/root/reference/utils/visualization.py:342-437).

The reference walks the boxes one at a time (`boxes.cls[i].cpu().numpy()` ... three device->host copies per
detection); here one (n, 6) copy per Results feeds all three formats:
  * txt: `"{cls} {conf:.6f} {x1:.6f} {y1:.6f} {x2:.6f} {y2:.6f}"` per line;
  * json: `{"detections": [{"class_id", "confidence", "bbox": [x1, y1, x2, y2]}, ...]}` with indent 2;
  * csv: header `class_id,confidence,x1,y1,x2,y2`, one row per detection.
Values are the fp32 tensor values (printed through Python floats, as the reference's numpy float32 -> float).
"""
from __future__ import annotations

import csv
import json
from pathlib import Path
from typing import Any, List

import numpy as np


def _rows(results: Any) -> List[tuple]:
    boxes = getattr(results, "boxes", None)
    if boxes is None or len(boxes) == 0:
        return []
    data = boxes.data
    arr = data.detach().cpu().numpy() if hasattr(data, "detach") else np.asarray(data)
    arr = arr.astype(np.float32, copy=False)
    return [(int(r[5]), r[4], r[0], r[1], r[2], r[3]) for r in arr]


def save_detection_results(results: Any, output_path: str, format: str = "txt") -> None:
    """Save one image's detections to `output_path` as 'txt', 'json' or 'csv' (the reference's formats)."""
    Path(output_path).parent.mkdir(parents=True, exist_ok=True)
    fmt = format.lower()
    if fmt not in ("txt", "json", "csv"):
        raise ValueError(f"Unsupported format: {format}")
    rows = _rows(results)
    if fmt == "txt":
        with open(output_path, "w") as f:
            for c, conf, x1, y1, x2, y2 in rows:
                f.write(f"{c} {conf:.6f} {x1:.6f} {y1:.6f} {x2:.6f} {y2:.6f}\n")
    elif fmt == "json":
        dets = [{"class_id": c, "confidence": float(conf), "bbox": [float(x1), float(y1), float(x2), float(y2)]}
                for c, conf, x1, y1, x2, y2 in rows]
        with open(output_path, "w") as f:
            json.dump({"detections": dets}, f, indent=2)
    else:
        with open(output_path, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["class_id", "confidence", "x1", "y1", "x2", "y2"])
            for c, conf, x1, y1, x2, y2 in rows:
                w.writerow([c, float(conf), float(x1), float(y1), float(x2), float(y2)])
