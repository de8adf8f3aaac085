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


def test_add_node_rebuilds_stale_indexes_after_kdtree_run(workload):
    """dpg_add_node_pairs after a k-d tree batch on the same scan store: the k-d tree
    overwrote the index buffers of the older nodes, so the per-node run rebuilds every stale index,
    not only the new node's -- the alignments equal those of a store that never left the angular
    variant."""
    from dpgslam import _abi, api
    w = workload("config2")
    p = _abi.default_icp_params()
    prior = np.zeros(1, _abi.FACTOR_DTYPE)
    prior["kind"], prior["i"], prior["info"] = _abi.DPG_FACTOR_PRIOR, 0, 1.0 / np.array([0.04, 0.04, 0.0225])

    def run(detour):
        ctx = api.Context(0)
        g = api.IncGraph(ctx, mode="isam2")
        g.add_node(w.cloud(0), np.zeros(1, np.int32), w.est[0], extra=prior, icp_params=p)
        for v in (1, 2, 3):
            g.add_node(w.cloud(v), np.zeros(v + 1, np.int32), w.est[v], icp_params=p)
        if detour:
            ctx.set_icp_variant("kdtree")
            ctx.icp_prepare(np.array([[0, 1], [1, 2], [2, 3]], np.int32), w.est[:4], p)
            _run(ctx)
            ctx.set_icp_variant("angular")
        g.add_node_pairs(w.cloud(4), w.est[4], np.array([[0, 4], [1, 4], [2, 4]], np.int32), icp_params=p)
        res, _ = ctx.icp_fetch(with_hessian=False)
        X = g.poses()
        g.close()
        ctx.close()
        return res, X

    r0, X0 = run(False)
    r1, X1 = run(True)
    assert len(r0) == 4 and r1.tobytes() == r0.tobytes()
    assert np.array_equal(X0, X1)
