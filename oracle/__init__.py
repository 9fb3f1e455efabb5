"""CPU oracle for the YOLO11 inference hot path — TEST INFRASTRUCTURE ONLY.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this package, and only as
the checker / the timed CPU baseline.  The product path (`yolo-infer_amd/`) never imports it and fails loudly when
its HIP library is missing.

What it restates: the Ultralytics 8.3.x predict path that `YOLO11Model.predict` delegates to
(`/root/reference/core/model.py:118-133` → `ultralytics.YOLO.predict`): LoadTensor's /255 rule, AutoBackend's
Conv+BN fusion (eps 1e-3), the YOLO11 DetectionModel / SegmentationModel forward, Detect DFL decode, class-offset
greedy NMS (torchvision.ops.nms semantics), scale_boxes/clip and process_mask — pure PyTorch fp32 on the CPU.

PARITY UNPINNED: the reference holds no tests, golden vectors or fixtures for this path, and the arithmetic lives in
`ultralytics` (>=8.0.0, unpinned, `requirements.txt:4`) and `torchvision` (`requirements.txt:3`), neither of which
is installed or installable offline.  This oracle is therefore the build's own restatement; the
golden fixtures under `tests/golden/` are generated from it (`tests/golden/make_golden.py`), and its pieces are
cross-checked against independent compositions (F.conv2d/F.max_pool2d identities, brute-force NMS) in
`tests/test_oracle.py`.
"""
