#!/usr/bin/env python3
"""Write the block sparsity pattern (unique node pairs of the factors) of a synthetic workload for
tools/chol_bench: int64 n, int64 P, int32 lo[P], int32 hi[P].
usage: python tools/make_pairs.py CONFIG OUT.bin"""
import sys

import numpy as np

from dpgslam import synth

w = synth.generate(sys.argv[1])
F = w.factors_placeholder()
b = F[F["kind"] == 1]
lo = np.minimum(b["i"], b["j"]).astype(np.int32)
hi = np.maximum(b["i"], b["j"]).astype(np.int32)
pr = np.unique(np.stack([lo, hi], 1), axis=0)
pr = pr[pr[:, 0] != pr[:, 1]]
with open(sys.argv[2], "wb") as f:
    np.array([w.V, len(pr)], np.int64).tofile(f)
    np.ascontiguousarray(pr[:, 0]).tofile(f)
    np.ascontiguousarray(pr[:, 1]).tofile(f)
print(f"{sys.argv[1]}: n={w.V} pairs={len(pr)}")
