"""Ultralytics `.pt` checkpoints → Ultralytics-key state dict, without Ultralytics.

The reference builds its model with `YOLO(model_path)` (/root/reference/core/model.py:100-116), i.e. an Ultralytics
checkpoint: a torch zip archive whose pickle holds `{"model": DetectionModel, "ema": ..., "train_args": ...}` with
the modules themselves pickled.  Ultralytics is not installed (and cannot be), and `torch.load(weights_only=True)`
refuses its classes.  This loader unpickles with a restricted Unpickler:
  * every class of `ultralytics.*` and `torch.nn.modules.*` becomes an inert stub type (no code of the class runs:
    the stub only records the pickled `__dict__`);
  * only torch's own tensor/storage reconstruction functions and a few containers are resolved to real objects;
  * any other global is refused (the load fails) — nothing named by the file is executed.
The stub tree is then walked like `nn.Module.state_dict()` (`_parameters`, `_buffers`, `_modules`), giving the keys
`model.<i>.<...>.weight` the rest of this package consumes (the same key space as `yolomi.synth`).
"""
from __future__ import annotations

import collections
import pickle
from typing import Dict

import numpy as np
import torch

_STUBS: Dict[tuple, type] = {}


class _Stub:
    """An inert stand-in for a pickled module object: accepts any construction, keeps the pickled state."""

    def __init__(self, *args, **kwargs):
        pass

    def __setstate__(self, state):
        if isinstance(state, tuple) and len(state) == 2:  # (dict state, slot state)
            state = {**(state[0] or {}), **(state[1] or {})}
        if isinstance(state, dict):
            self.__dict__.update(state)

    def __call__(self, *args, **kwargs):  # a stub reached through REDUCE: yields another inert object
        return _Stub()


def _stub(module: str, name: str) -> type:
    key = (module, name)
    if key not in _STUBS:
        _STUBS[key] = type(name, (_Stub,), {"__module_name__": module})
    return _STUBS[key]


_ALLOWED = {
    ("collections", "OrderedDict"): collections.OrderedDict,
    ("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
    ("torch._utils", "_rebuild_parameter"): torch._utils._rebuild_parameter,
    ("torch", "Size"): torch.Size,
    ("torch", "float16"): torch.float16, ("torch", "float32"): torch.float32, ("torch", "bfloat16"): torch.bfloat16,
    ("copyreg", "_reconstructor"): None,  # resolved below to a constructor that never runs the class' code
    ("builtins", "set"): set, ("builtins", "frozenset"): frozenset, ("builtins", "slice"): slice,
}
_STORAGES = {"HalfStorage", "FloatStorage", "BFloat16Storage", "DoubleStorage", "LongStorage", "IntStorage",
             "ByteStorage", "CharStorage", "ShortStorage", "BoolStorage", "UntypedStorage"}
_STUB_PREFIXES = ("ultralytics.", "torch.nn.modules.", "__main__", "models.", "utils.", "numpy", "pathlib",
                  "types", "argparse", "easydict")


def _reconstruct(cls, base, state):
    """copyreg._reconstructor restricted to stub classes: object.__new__ of the stub, nothing else."""
    if not (isinstance(cls, type) and issubclass(cls, _Stub)):
        raise pickle.UnpicklingError(f"refusing to reconstruct {cls!r}")
    return cls.__new__(cls)


class _Unpickler(pickle.Unpickler):
    def find_class(self, module, name):
        module = {"__builtin__": "builtins", "copy_reg": "copyreg"}.get(module, module)  # protocol-2 names
        if (module, name) == ("copyreg", "_reconstructor"):
            return _reconstruct
        if (module, name) in _ALLOWED:
            return _ALLOWED[(module, name)]
        if module == "torch" and name in _STORAGES:
            return getattr(torch, name)
        if module.startswith(_STUB_PREFIXES) or module in ("__main__", "numpy", "pathlib", "types"):
            return _stub(module, name)
        raise pickle.UnpicklingError(f"refusing global {module}.{name}")


class _PickleModule:
    """The `pickle_module` handed to torch.load: torch's zip reader with the restricted Unpickler."""
    Unpickler = _Unpickler
    __name__ = "yolomi_restricted_pickle"

    @staticmethod
    def load(f, **kw):
        return _Unpickler(f, **kw).load()


def _walk(mod, prefix: str, out: Dict[str, np.ndarray]):
    d = getattr(mod, "__dict__", {})
    for group in ("_parameters", "_buffers"):
        for k, v in (d.get(group) or {}).items():
            if isinstance(v, torch.Tensor):
                t = v.detach()
                out[prefix + k] = t.float().numpy() if t.is_floating_point() else t.numpy()
    for k, sub in (d.get("_modules") or {}).items():
        if sub is not None:
            _walk(sub, prefix + k + ".", out)


def load_ultralytics_checkpoint(path: str) -> Dict[str, np.ndarray]:
    """State dict (Ultralytics keys, fp32 numpy) of the EMA model of a checkpoint, or of its `model` entry."""
    ckpt = torch.load(path, map_location="cpu", pickle_module=_PickleModule, weights_only=False)
    if isinstance(ckpt, dict):
        model = ckpt.get("ema") or ckpt.get("model")
    else:
        model = ckpt
    if model is None or not isinstance(model, _Stub):
        raise ValueError(f"{path}: no pickled Ultralytics model found (keys: {list(ckpt)[:8] if isinstance(ckpt, dict) else type(ckpt)})")
    sd: Dict[str, np.ndarray] = {}
    _walk(model, "", sd)
    if not any(k.startswith("model.") for k in sd):
        raise ValueError(f"{path}: the pickled model holds no 'model.*' parameters")
    return sd
