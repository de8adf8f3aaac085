"""The angle index is reused across batch runs on the same scan store:
the second run builds nothing, yet aligns byte for byte like the first and like a fresh context;
a change of builder (kernel form 2, the bitonic network) or of ICP variant, and a new upload,
rebuild it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(ctx):
    ctx.icp_run(compute_cov=False)
    ctx.synchronize()
    res, _ = ctx.icp_fetch(with_hessian=False)
    return res


def test_index_reused_and_rebuilt_when_needed(workload):
    from dpgslam import _abi, api
    w = workload("config2")
    p = _abi.default_icp_params()
    with api.Context(0) as ref:
        ref.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
        ref.icp_prepare(w.edges, w.est, p)
        r0 = _run(ref)
    with api.Context(0) as ctx:
        ctx.upload_scans(w.pts, w.offsets, p.downsample_icp_points_ratio)
        ctx.icp_prepare(w.edges, w.est, p)
        r1 = _run(ctx)
        built_first = ctx.kdtree_build_ms()
        r2 = _run(ctx)                       # the index of every node is current: nothing is built
        reused = ctx.kdtree_build_ms()
        assert r1.tobytes() == r0.tobytes() and r2.tobytes() == r0.tobytes()
        assert reused < built_first, (reused, built_first)
        ctx.set_icp_kernel_variant(2)        # the bitonic builder: rebuilt, same alignments
        assert _run(ctx).tobytes() == r0.tobytes()
        ctx.set_icp_kernel_variant(0)
        ctx.set_icp_variant("kdtree")        # the k-d tree overwrites the index buffers
        assert _run(ctx).tobytes() == r0.tobytes()
        ctx.set_icp_variant("angular")
        assert _run(ctx).tobytes() == r0.tobytes()
        # a new upload (the same scans in reverse node order, the edges renumbered) rebuilds it
        V = len(w.offsets) - 1
        rev = np.arange(V)[::-1]
        sizes = np.diff(w.offsets)[rev]
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(w.offsets.dtype)
        pts = np.concatenate([w.pts[w.offsets[v]:w.offsets[v + 1]] for v in rev])
        ctx.upload_scans(pts, offs, p.downsample_icp_points_ratio)
        inv = np.empty(V, dtype=np.int64)
        inv[rev] = np.arange(V)
        ctx.icp_prepare(inv[w.edges].astype(w.edges.dtype), w.est[rev], p)
        assert _run(ctx).tobytes() == r0.tobytes()
