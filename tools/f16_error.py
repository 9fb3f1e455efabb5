#!/usr/bin/env python3
"""Precision budget of the plans vs the CPU oracle: per plan (f32 parity / f16 throughput),
on 16 U[0,1) 640x640 images per model: matched / exempt / unmatched detections under the SURVEY §8(c) protocol,
max and 99th-percentile |Δxy| and |Δscore| of matched pairs, and the device images/s of the plan at B=8."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from core.model import YOLO11Model
    from oracle.predict import OracleModel
    from tests.golden.make_golden import make_input
    from tests.matching import MatchReport, iou_matrix, match_image
    from yolomi.synth import synth_weights
    torch.set_num_threads(16)
    out = {}
    for scale in ("n", "s"):
        om = OracleModel(scale, "detect", synth_weights(scale, "detect", 0))
        xs = [make_input("uniform", tuple(range(9000 + 8 * k, 9008 + 8 * k)), 640) for k in range(2)]
        refs = [om.predict(x) for x in xs]
        for dtype in ("f32", "f16"):
            m = YOLO11Model(size=scale, device="cuda:0", dtype=dtype, verbose=False)
            rep = MatchReport()
            dxy, ds = [], []
            for x, ref in zip(xs, refs):
                res = m.predict(x.cuda())
                for r, g in zip(ref, res):
                    rr, gg = r["boxes"].numpy(), g.boxes.data.cpu().numpy()
                    before = len(rep.pairs)
                    match_image(rr, gg, 0.25, 0.7, 1.0 if dtype == "f16" else 1e-3, 1e-2 if dtype == "f16" else 1e-3,
                                rep=rep)
                    for i, j in rep.pairs[before:]:
                        dxy.append(float(np.abs(rr[i, :4] - gg[j, :4]).max()))
                        ds.append(float(abs(rr[i, 4] - gg[j, 4])))
            eng = m.model.engine
            x8 = xs[0].cuda()
            for _ in range(5):
                eng.run(x8)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(50):
                eng.run(x8)
            torch.cuda.synchronize()
            ips = 8 * 50 / (time.perf_counter() - t)
            total = sum(len(r["boxes"]) for ref in refs for r in ref)
            d = {"oracle_dets": total, "matched": rep.matched, "exempt": rep.exempt,
                 "unmatched_ref": rep.unmatched_ref, "unmatched_build": rep.unmatched_build,
                 "max_dxy_px": round(max(dxy), 5), "p99_dxy_px": round(float(np.percentile(dxy, 99)), 5),
                 "max_dscore": round(max(ds), 6), "p99_dscore": round(float(np.percentile(ds, 99)), 6),
                 "frac_within_1e-3": round(float(np.mean([(a <= 1e-3 and b <= 1e-3) for a, b in zip(dxy, ds)])), 4),
                 "device_images_per_s_b8": round(ips, 1)}
            out[f"yolo11{scale}-{dtype}"] = d
            print(scale, dtype, d, flush=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "f16_error.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
