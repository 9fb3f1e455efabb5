import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# a host crash inside libyolomi prints its native backtrace before faulthandler's Python stack (csrc/ym_runtime.cpp)
os.environ.setdefault("YM_SEGV_TRACE", "1")
for p in (os.path.join(ROOT, "yolo-infer_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libyolomi.so")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True, scope="module")
def _release_module_models(request):
    """GPU test modules cache their models (contexts, arenas, captured graphs) in module-level dicts; release them when
    the module is done, so the whole `-m gpu` suite does not keep every earlier module's contexts alive."""
    yield
    for name in ("_models", "_cache"):
        d = getattr(request.module, name, None)
        if isinstance(d, dict):
            d.clear()
    import gc
    gc.collect()
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
    except Exception:
        pass
