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
