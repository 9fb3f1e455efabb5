"""Ultralytics .pt import (yolomi/ptimport.py) on the CPU.

No real checkpoint exists offline, so the fixture is built here: a module tree whose classes live in a fake
`ultralytics.nn.*` package (registered in sys.modules only while pickling, as in a training process), holding the
synthetic yolo11n weights in fp16 like a released checkpoint, saved with torch.save next to `train_args` etc.  The
importer must recover every tensor exactly without the package, and must refuse globals outside its allowlist."""
import io
import pickle
import sys
import types

import numpy as np
import pytest
import torch
import torch.nn as nn

from yolomi.ptimport import load_ultralytics_checkpoint
from yolomi.synth import synth_weights


def _fake_checkpoint(path, sd):
    names = ["ultralytics", "ultralytics.nn", "ultralytics.nn.tasks", "ultralytics.nn.modules",
             "ultralytics.nn.modules.conv", "ultralytics.nn.modules.block", "ultralytics.nn.modules.head"]
    mods = {n: types.ModuleType(n) for n in names}
    classes = {}

    def cls(modname, name):
        if (modname, name) not in classes:
            c = type(name, (nn.Module,), {})
            c.__module__ = modname
            setattr(mods[modname], name, c)
            classes[(modname, name)] = c
        return classes[(modname, name)]

    saved = {n: sys.modules.get(n) for n in names}
    sys.modules.update(mods)
    try:
        root = cls("ultralytics.nn.tasks", "DetectionModel")()
        for key, arr in sd.items():
            parts = key.split(".")
            m = root
            for depth, p in enumerate(parts[:-1]):
                if p not in m._modules:
                    kind = ("ultralytics.nn.modules.conv", "Conv") if depth % 2 else ("ultralytics.nn.modules.block", "C3k2")
                    if depth == 0:
                        kind = ("torch.nn.modules.container", None)
                    child = nn.Sequential() if kind[1] is None else cls(*kind)()
                    m.add_module(p, child)
                m = m._modules[p]
            t = torch.from_numpy(np.asarray(arr))
            if parts[-1] in ("running_mean", "running_var", "num_batches_tracked"):
                m.register_buffer(parts[-1], t.clone())
            else:
                m.register_parameter(parts[-1], nn.Parameter(t.clone(), requires_grad=False))
        root = root.half()
        torch.save({"model": root, "ema": None, "train_args": {"imgsz": 640, "model": "yolo11n.yaml"},
                    "date": "2024-09-29", "version": "8.3.0"}, path)
    finally:
        for n, v in saved.items():
            if v is None:
                sys.modules.pop(n, None)
            else:
                sys.modules[n] = v


def test_ultralytics_checkpoint_roundtrip(tmp_path):
    sd = synth_weights("n", "detect", 3)
    p = tmp_path / "yolo11n.pt"
    _fake_checkpoint(p, sd)
    assert "ultralytics" not in sys.modules
    with pytest.raises(Exception):
        torch.load(p, map_location="cpu", weights_only=True)  # what a plain safe load does with it
    got = load_ultralytics_checkpoint(str(p))
    assert set(got) == set(sd)
    for k, v in sd.items():
        want = np.asarray(v)
        want = want.astype(np.float16).astype(np.float32) if want.dtype.kind == "f" else want
        assert np.array_equal(got[k], want), k


def test_restricted_unpickler_refuses_foreign_globals(tmp_path):
    class Evil:
        def __reduce__(self):
            import os
            return (os.system, ("echo pwned",))
    p = tmp_path / "evil.pt"
    torch.save({"model": Evil()}, p)
    with pytest.raises(Exception, match="refusing"):
        load_ultralytics_checkpoint(str(p))
