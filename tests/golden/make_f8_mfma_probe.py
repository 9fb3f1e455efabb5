#!/usr/bin/env python3
"""Hardware vectors for the fp8 MFMA restatement (oracle/quant.py mfma_f8_step): a sample of tools/f8_mfma_probe.hip's
v_mfma_f32_32x32x16_fp8_fp8 instances (kind 0) — the e4m3 operand codes of every lane, C, and the D the MI355X
returned — 8 instances of each of the probe's 4 operand distributions.

    python tests/golden/make_f8_mfma_probe.py gpurun_out/r05h/f8probe.bin   ->  tests/golden/f8_mfma_probe.npz

Lane map of the probe (tools/f8_mfma_model.py terms): lane h*32 + r holds A[row r][k = 8h + j] and B[k = 8h + j][col r].
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tools"))
from f8_mfma_model import load  # noqa: E402


def main(path):
    n, ndist, kinds = load(path)
    KL, A, B, C, D = kinds[0]
    per = n // ndist
    idx = np.concatenate([np.arange(d * per, d * per + 8) for d in range(ndist)])
    np.savez_compressed(os.path.join(HERE, "f8_mfma_probe.npz"), A=A[idx], B=B[idx], C=C[idx], D=D[idx],
                        dist=np.repeat(np.arange(ndist), 8))


if __name__ == "__main__":
    main(sys.argv[1])
