"""Generate the committed golden fixtures from the CPU oracle.

    python tests/golden/make_golden.py

Parity with Ultralytics itself is UNPINNED (the reference ships no fixtures/tests and Ultralytics is not installable
offline); these vectors pin the oracle + the portable synthetic weights so the GPU path and future rounds are checked
against fixed numbers.  Inputs are regenerated from seeds (splitmix64, bit-portable); outputs are stored.

Fixtures (tests/golden/*.json):
  weights_<scale>.json  : per-tensor sum / abs-sum of the synthetic state dict (seed 0) + fused conv checksums
  det_n_uniform.json    : yolo11n, 2 x U[0,1) 640x640 (seeds 1001, 1002), conf 0.25 iou 0.7: per-image (n,6) dets,
                          per-layer output checksums and sampled values (L2, L9, L16, L22, head)
  det_n_randn.json      : yolo11n, 1 x N(0,1) 640x640 (seed 2001) → LoadTensor /255 rule, conf 0.25
  det_n_320_lowconf.json: yolo11n, 1 x U[0,1) 320x320 (seed 3001), conf 0.05 (many candidates)
  det_s_uniform.json    : yolo11s, 1 x U[0,1) 640x640 (seed 4001)
  seg_s_uniform.json    : yolo11s-seg (BASELINE config 5), 4 x U[0,1) 640x640 (seeds 6001-6004), conf 0.25 iou 0.7:
                          per-image NMS rows with the 32 mask coefficients, proto checksums/samples, and per kept
                          mask its pixel count and row/column sums (the full 640x640 masks are recomputed live)
  det_n_i8_qnnpack.json : yolo11n PTQ int8 (oracle/quant.py, qnnpack qconfig): calibrated on 2 x U[0,1) 640x640
                          (seeds 5001, 5002); the qparams + int8-oracle detections of 2 other images (5101, 5102)
  det_n_i8_fbgemm_320.json: same with the fbgemm qconfig (per-channel weights, reduce_range), 320x320 (5201 / 5301)
    python tests/golden/make_golden.py i8      # regenerates only the int8 fixtures
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer_amd"))
sys.path.insert(0, ROOT)

from oracle import quant as Q  # noqa: E402
from oracle.predict import OracleModel  # noqa: E402
from yolomi.plan import fuse_conv_bn  # noqa: E402
from yolomi.synth import normal, synth_weights, uniform  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
LAYERS = (2, 9, 16, 22)


def make_input(kind: str, seeds, S: int) -> torch.Tensor:
    xs = []
    for s in seeds:
        n = 3 * S * S
        v = uniform(s, n) if kind == "uniform" else normal(s, n)
        xs.append(v.astype(np.float32).reshape(3, S, S))
    return torch.from_numpy(np.stack(xs))


def layer_stats(t: torch.Tensor):
    t = t.double()
    flat = t.reshape(-1)
    idx = np.linspace(0, flat.numel() - 1, 16).astype(np.int64)
    return {"shape": list(t.shape), "sum": float(t.sum()), "abs_sum": float(t.abs().sum()),
            "samples_idx": idx.tolist(), "samples": flat[idx].tolist()}


def det_fixture(scale, kind, seeds, S, conf=0.25, iou=0.7):
    sd = synth_weights(scale, "detect", 0)
    om = OracleModel(scale, "detect", sd)
    x = make_input(kind, seeds, S)
    im, y, ex = om.raw(x, keep=LAYERS)
    B = x.shape[0]
    no = 144
    head = torch.cat([f.view(B, no, -1) for f in ex["feats"]], 2).transpose(1, 2)
    dets = om.predict(x, conf=conf, iou=iou)
    return {
        "scale": scale, "task": "detect", "weights_seed": 0, "input": {"kind": kind, "seeds": list(seeds), "size": S},
        "conf": conf, "iou": iou, "max_det": 300,
        "layers": {f"L{i}": layer_stats(ex["saved"][i].permute(0, 2, 3, 1)) for i in LAYERS},
        "head": layer_stats(head),
        "dets": [d["boxes"].tolist() for d in dets],
    }


def seg_fixture(scale, seeds, S, conf=0.25, iou=0.7):
    from oracle import postprocess as pp
    sd = synth_weights(scale, "segment", 0)
    om = OracleModel(scale, "segment", sd)
    x = make_input("uniform", seeds, S)
    im, y, ex = om.raw(x)
    nms = pp.non_max_suppression(y, conf, iou, nc=80)
    rows = []
    for d in nms:
        d = d.clone()
        d[:, :4] = pp.clip_boxes(d[:, :4], (S, S))
        rows.append(d.tolist())
    res = om.predict(x, conf=conf, iou=iou)
    masks = []
    for r in res:
        m = r["masks"]
        masks.append([] if m is None else [[int(k.sum()), k.sum(1).nonzero().min().item(), k.sum(1).nonzero().max().item(),
                                            k.sum(0).nonzero().min().item(), k.sum(0).nonzero().max().item()]
                                           for k in m.to(torch.int64)])
    return {
        "scale": scale, "task": "segment", "weights_seed": 0, "input": {"kind": "uniform", "seeds": list(seeds), "size": S},
        "conf": conf, "iou": iou, "max_det": 300, "proto": layer_stats(ex["proto"].permute(0, 2, 3, 1)),
        "nms_rows": rows, "dets": [r["boxes"].tolist() for r in res],
        "masks": masks, "masks_note": "per kept mask: [pixels set, first row, last row, first col, last col]",
    }


def weight_fixture(scale):
    sd = synth_weights(scale, "detect", 0)
    out = {"scale": scale, "seed": 0, "tensors": {}}
    for k in sorted(sd):
        v = sd[k].astype(np.float64)
        out["tensors"][k] = [float(v.sum()), float(np.abs(v).sum())]
    fused = {}
    for k in sorted(sd):
        p = k[: -len(".conv.weight")]
        if k.endswith(".conv.weight") and p + ".bn.weight" in sd:
            w, b = fuse_conv_bn(sd[k], sd[p + ".bn.weight"], sd[p + ".bn.bias"], sd[p + ".bn.running_mean"],
                                sd[p + ".bn.running_var"])
            fused[p] = [float(w.astype(np.float64).sum()), float(b.astype(np.float64).sum())]
    out["fused"] = fused
    return out


def det_i8_fixture(scale, backend, calib_seeds, seeds, S, conf=0.25, iou=0.7):
    sd = synth_weights(scale, "detect", 0)
    net = Q.build_folded(scale, "detect", sd)
    qp = Q.calibrate(net, [make_input("uniform", calib_seeds, S)], backend)
    m = Q.Int8OracleModel(scale, "detect", sd, qp)
    x = make_input("uniform", seeds, S)
    im, y, ex = m.raw(x)
    B = x.shape[0]
    head = torch.cat([f.reshape(B, 144, -1) for f in ex["feats"]], 2).transpose(1, 2)
    dets = m.predict(x, conf=conf, iou=iou)
    return {
        "scale": scale, "task": "detect", "weights_seed": 0, "backend": backend,
        "calibration": {"kind": "uniform", "seeds": list(calib_seeds), "size": S},
        "input": {"kind": "uniform", "seeds": list(seeds), "size": S}, "conf": conf, "iou": iou, "max_det": 300,
        "qparams": Q.qparams_to_json(qp),
        "layers": {f"L{i}": layer_stats(ex["stored"][i].q.permute(0, 2, 3, 1)) for i in LAYERS},
        "head": layer_stats(head),
        "dets": [d["boxes"].tolist() for d in dets],
    }


I8_FIXTURES = {
    "det_n_i8_qnnpack": ("n", "qnnpack", (5001, 5002), (5101, 5102), 640),
    "det_n_i8_fbgemm_320": ("n", "fbgemm", (5201,), (5301,), 320),
}


# fp8 e4m3 PTQ plan (oracle/quant.py backend "fp8"): qparams from min/max observers, fp8-oracle detections
F8_FIXTURES = {
    "det_n_f8": ("n", "fp8", (5401, 5402), (5501, 5502), 640),
}


def main_f8():
    for name, (scale, backend, cs, seeds, S) in F8_FIXTURES.items():
        d = det_i8_fixture(scale, backend, cs, seeds, S)
        json.dump(d, open(os.path.join(HERE, f"{name}.json"), "w"))
        print(name, [len(x) for x in d["dets"]])


# the fp8 plan's own accumulation (oracle/quant.py accum="mfma": the restated fp8 MFMA chain of conv_i8), with
# det_n_f8's qparams, on 320x320 inputs (the emulated convs take ~9 s per 320² image on 8 threads)
F8M_FIXTURES = {
    "det_n_f8m_320": ("det_n_f8", (5501, 5502), 320),
}


def main_f8m():
    for name, (base, seeds, S) in F8M_FIXTURES.items():
        b = json.load(open(os.path.join(HERE, f"{base}.json")))
        qp = Q.qparams_from_json(b["qparams"])
        m = Q.Int8OracleModel(b["scale"], "detect", synth_weights(b["scale"], "detect", 0), qp, accum="mfma")
        x = make_input("uniform", seeds, S)
        im, y, ex = m.raw(x)
        B = x.shape[0]
        head = torch.cat([f.reshape(B, 144, -1) for f in ex["feats"]], 2).transpose(1, 2)
        dets = m.predict(x, conf=b["conf"], iou=b["iou"])
        d = {"scale": b["scale"], "task": "detect", "weights_seed": 0, "backend": "fp8", "accum": "mfma",
             "qparams_from": base, "input": {"kind": "uniform", "seeds": list(seeds), "size": S}, "conf": b["conf"],
             "iou": b["iou"], "max_det": 300, "qparams": b["qparams"],
             "layers": {f"L{i}": layer_stats(ex["stored"][i].q.permute(0, 2, 3, 1)) for i in LAYERS},
             "head": layer_stats(head), "dets": [d["boxes"].tolist() for d in dets]}
        json.dump(d, open(os.path.join(HERE, f"{name}.json"), "w"))
        print(name, [len(x) for x in d["dets"]])


def main_seg():
    d = seg_fixture("s", (6001, 6002, 6003, 6004), 640)
    json.dump(d, open(os.path.join(HERE, "seg_s_uniform.json"), "w"))
    print("seg_s_uniform", [len(x) for x in d["dets"]])


def main_i8():
    for name, (scale, backend, cs, seeds, S) in I8_FIXTURES.items():
        d = det_i8_fixture(scale, backend, cs, seeds, S)
        json.dump(d, open(os.path.join(HERE, f"{name}.json"), "w"))
        print(name, [len(x) for x in d["dets"]])


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for scale in ("n", "s"):
        json.dump(weight_fixture(scale), open(os.path.join(HERE, f"weights_{scale}.json"), "w"), indent=0)
    fx = {
        "det_n_uniform": ("n", "uniform", (1001, 1002), 640, 0.25),
        "det_n_randn": ("n", "randn", (2001,), 640, 0.25),
        "det_n_320_lowconf": ("n", "uniform", (3001,), 320, 0.05),
        "det_s_uniform": ("s", "uniform", (4001,), 640, 0.25),
    }
    for name, (scale, kind, seeds, S, conf) in fx.items():
        d = det_fixture(scale, kind, seeds, S, conf)
        json.dump(d, open(os.path.join(HERE, f"{name}.json"), "w"))
        print(name, [len(x) for x in d["dets"]])


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] in ("i8", "seg", "f8", "f8m"):
        torch.set_num_threads(min(8, os.cpu_count() or 1))
        {"i8": main_i8, "seg": main_seg, "f8": main_f8, "f8m": main_f8m}[sys.argv[1]]()
    else:
        main()
        main_seg()
        main_i8()
        main_f8()
        main_f8m()
