"""Known-answer graphs from the reference's own code."""
import math

import numpy as np


def gtsam_test_graph():
    """src/dpg_slam/dpg_slam_main.cc:224-251 (keys 1..5 -> 0..4).

    Measurements are exactly consistent (a 2 m square), so the optimum is analytic:
    x1=(0,0,0), x2=(2,0,0), x3=(4,0,pi/2), x4=(4,2,pi), x5=(2,2,-pi/2)."""
    from dpgslam import api
    prior = (0.3, 0.3, 0.1)
    model = (0.2, 0.2, 0.1)
    F = np.concatenate([
        api.prior_factor(0, (0.0, 0.0, 0.0), prior),
        api.between_factor(0, 1, (2.0, 0.0, 0.0), model),
        api.between_factor(1, 2, (2.0, 0.0, math.pi / 2), model),
        api.between_factor(2, 3, (2.0, 0.0, math.pi / 2), model),
        api.between_factor(3, 4, (2.0, 0.0, math.pi / 2), model),
        api.between_factor(4, 1, (2.0, 0.0, math.pi / 2), model),
    ])
    # the reference's sigmas are doubles (gtsam::Vector3(0.3, 0.3, 0.1)), not floats
    F["info"][0] = 1.0 / np.square(np.array(prior, np.float64))
    X0 = np.array([[0.5, 0.0, 0.2], [2.3, 0.1, -0.2], [4.1, 0.1, math.pi / 2], [4.0, 2.0, math.pi],
                   [2.1, 2.1, -math.pi / 2]])
    X_opt = np.array([[0, 0, 0], [2, 0, 0], [4, 0, math.pi / 2], [4, 2, math.pi], [2, 2, -math.pi / 2]], float)
    return X0, F, X_opt


def pose_diff(a, b):
    d = np.asarray(a, float) - np.asarray(b, float)
    d[..., 2] = np.arctan2(np.sin(d[..., 2]), np.cos(d[..., 2]))
    return d


def consistent_mesh_graph(V=3000, k=6, seed=11, noise=(0.3, 0.3, 0.2)):
    """A 2-D mesh-like pose graph with exactly consistent measurements (known optimum = the true
    poses): nodes at random positions in a square, Between factors to the k nearest neighbours plus
    the odometry chain, one prior at node 0.  Its elimination tree has large top separators (large
    Cholesky fronts: the multi-workgroup team path).  Returns (X0 perturbed, factors, X_true)."""
    from dpgslam import api
    rng = np.random.default_rng(seed)
    # nodes along a jittered serpentine path (a trajectory sweeping an area): the odometry chain
    # stays local, the k-nearest-neighbour edges close loops between neighbouring sweeps
    row = int(math.sqrt(V))
    r, c = np.divmod(np.arange(V), row)
    c = np.where(r % 2 == 0, c, row - 1 - c)
    xy = np.column_stack([c, r]).astype(float) * 1.5 + rng.normal(0, 0.3, (V, 2))
    th = rng.uniform(-math.pi, math.pi, V)
    X = np.column_stack([xy, th])

    def rel(i, j):   # Pose2 between: Xi^-1 Xj
        c, s = math.cos(X[i, 2]), math.sin(X[i, 2])
        dx, dy = X[j, 0] - X[i, 0], X[j, 1] - X[i, 1]
        d = X[j, 2] - X[i, 2]
        return (c * dx + s * dy, -s * dx + c * dy, math.atan2(math.sin(d), math.cos(d)))

    pairs = set((i, i + 1) for i in range(V - 1))
    d2 = ((xy[:, None, :] - xy[None, :, :]) ** 2).sum(-1) if V <= 4000 else None
    for i in range(V):
        for j in np.argsort(d2[i])[1:k + 1]:
            pairs.add((min(i, int(j)), max(i, int(j))))
    F = [api.prior_factor(0, tuple(X[0]), (0.1, 0.1, 0.05))]
    F[0]["info"] = 1.0 / np.square(np.array([0.1, 0.1, 0.05]))
    for i, j in sorted(pairs):
        F.append(api.between_factor(i, j, rel(i, j), (0.1, 0.1, 0.05)))
    X0 = X + rng.normal(0, 1, X.shape) * np.array(noise)
    X0[:, 2] = np.arctan2(np.sin(X0[:, 2]), np.cos(X0[:, 2]))
    return X0, np.concatenate(F), X
