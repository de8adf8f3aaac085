/*
 * dpg_host.c -- host-side data path of the DPG-SLAM hot path (no GPU work here).
 *
 * R1 polar scan -> base_link cloud: MeasurementPoint ctor (src/dpg_slam/dpg_measurement.h:41-46),
 *    getPointInLaserFrame (:102-104), createNode (src/dpg_slam/dpg_slam.cc:488-513),
 *    DpgNode::getCachedPointCloudFromNode (src/dpg_slam/dpg_node.cc:8-25).
 * R2 downsamplePointCloud (dpg_slam.cc:346-360).
 * R3 runIcp initial guess (dpg_slam.cc:364-378) via math_utils::inverseTransformPoint
 *    (src/dpg_slam/math_utils.cc:21-35).
 * R9 odometry factor noise (dpg_slam.cc:53-75, 216-238).
 *
 * These run on the host in float exactly as the reference evaluates them, so the clouds the GPU
 * receives are bit-identical to what the CPU path would build.  Built with -ffp-contract=off.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../../include/dpg_slam_c.h"
#include "dpg_internal.h"

/* math_utils::AngleMod<float> (math_utils.h:13-16): float in, the subtraction runs in double. */
static float angle_mod(float a) {
    double v = (double)a;
    v -= (M_PI * 2.0) * rint(v / (M_PI * 2.0));
    return (float)v;
}

/* Eigen::Rotation2Df(theta) * (x, y): [cos -sin; sin cos] times the vector, float. */
static void rotate(float theta, float x, float y, float* ox, float* oy) {
    const float c = cosf(theta), s = sinf(theta);
    const float ms = -s;
    *ox = c * x + ms * y;
    *oy = s * x + c * y;
}

int64_t dpg_scan_to_cloud(const float* ranges, int64_t n_ranges, float angle_min, float angle_max,
                          float range_max, float laser_x, float laser_y, float laser_theta,
                          float* xy_out) {
    if (!ranges || !xy_out || n_ranges <= 0) return 0;
    /* dpg_slam.cc:497 -- (float - float) / (size - 1.0) in double, stored as float */
    const float angle_inc = (float)((double)(angle_max - angle_min) / ((double)n_ranges - 1.0));
    int64_t n = 0;
    for (int64_t i = 0; i < n_ranges; ++i) {
        const float r = ranges[i];
        if (r >= range_max) continue; /* label MAX_RANGE, skipped by the cloud cache */
        const float angle = angle_inc * (float)i + angle_min;
        const float lx = r * cosf(angle), ly = r * sinf(angle);
        float bx, by;
        rotate(laser_theta, lx, ly, &bx, &by);
        xy_out[2 * n] = laser_x + bx;
        xy_out[2 * n + 1] = laser_y + by;
        ++n;
    }
    return n;
}

int64_t dpg_downsample_cloud(const float* xy, int64_t n, int32_t ratio, float* xy_out) {
    if (!xy || !xy_out || n <= 0) return 0;
    if (ratio < 1) ratio = 1;
    int64_t k = 0;
    for (int64_t i = 0; i < n; i += ratio, ++k) {
        xy_out[2 * k] = xy[2 * i];
        xy_out[2 * k + 1] = xy[2 * i + 1];
    }
    return k;
}

void dpg_inverse_transform_point(const float a[3], const float b[3], float out[3]) {
    const float dx = a[0] - b[0], dy = a[1] - b[1];
    rotate(-b[2], dx, dy, &out[0], &out[1]);
    out[2] = angle_mod(a[2] - b[2]);
}

void dpg_transform_point(const float p[3], const float frame[3], float out[3]) {
    float rx, ry;
    rotate(frame[2], p[0], p[1], &rx, &ry);
    out[0] = frame[0] + rx;
    out[1] = frame[1] + ry;
    out[2] = angle_mod(frame[2] + p[2]);
}

void dpg_icp_guess(const float pose_src[3], const float pose_tgt[3], float g[6]) {
    float d[3];
    dpg_inverse_transform_point(pose_src, pose_tgt, d);
    const float c = cosf(d[2]), s = sinf(d[2]);
    g[0] = c;
    g[1] = -s;
    g[2] = d[0];
    g[3] = s;
    g[4] = c;
    g[5] = d[1];
}

void dpg_icp_params_default(dpg_icp_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->icp_maximum_iterations = 500;             /* parameters.h:146 */
    p->icp_use_reciprocal_correspondences = 1;   /* parameters.h:201 */
    p->icp_maximum_transformation_epsilon = 0.000000005; /* parameters.h:159 */
    p->icp_max_correspondence_distance = 0.6;    /* parameters.h:173 */
    p->ransac_iterations = 50;                   /* parameters.h:191 */
    p->downsample_icp_points_ratio = 5;          /* parameters.h:402 */
    p->laser_x_variance = 0.5f;                  /* parameters.h:374 */
    p->laser_y_variance = 0.5f;                  /* parameters.h:385 */
    p->laser_theta_variance = 0.3f;              /* parameters.h:396 */
    p->min_number_correspondences = 3;           /* pcl::Registration default */
    p->mse_threshold_absolute = 1e-12;           /* pcl DefaultConvergenceCriteria default */
}

void dpg_gn_params_default(dpg_gn_params* p) {
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->max_iterations = 100;
    p->use_error_criteria = 0;
    p->delta_tol = 1e-10;
    p->relative_error_tol = 1e-5;
    p->absolute_error_tol = 1e-5;
    p->pcg_rel_tol = 1e-12;
    p->pcg_max_iterations = 20000;
    p->pcg_check_every = 16;
    p->reuse_factorization = 1;
    p->refactor_delta = 1e-3;
}

/* R9: odometry BetweenFactor from two odom_only_estimates (dpg_slam.cc:56-75). */
int dpg_odometry_factor(const float odom_prev[3], const float odom_cur[3], int32_t i_prev, int32_t i_cur,
                        float transl_from_transl, float transl_from_rot, float rot_from_transl,
                        float rot_from_rot, dpg_factor* out) {
    float d[3];
    dpg_inverse_transform_point(odom_cur, odom_prev, d);
    const float norm = sqrtf(d[0] * d[0] + d[1] * d[1]);       /* Vector2f::norm() */
    const float transl_sd = (transl_from_transl * norm) + (transl_from_rot * fabsf(d[2]));
    const float rot_sd = (rot_from_transl * norm) + (rot_from_rot * fabsf(d[2]));
    memset(out, 0, sizeof(*out));
    out->kind = DPG_FACTOR_BETWEEN;
    out->i = i_prev;
    out->j = i_cur;
    out->z[0] = d[0];
    out->z[1] = d[1];
    out->z[2] = d[2];
    const double st = (double)transl_sd, sr = (double)rot_sd;
    if (!(st > 0.0) || !(sr > 0.0)) return DPG_ERR_NUMERIC; /* GTSAM would build a Constrained model */
    out->info[0] = 1.0 / (st * st);
    out->info[1] = 1.0 / (st * st);
    out->info[2] = 1.0 / (sr * sr);
    return DPG_OK;
}

int dpg_odometry_factors(const float* odom, int64_t n_odom, const int32_t* i_prev, const int32_t* i_cur, int64_t n,
                         float transl_from_transl, float transl_from_rot, float rot_from_transl, float rot_from_rot,
                         dpg_factor* out) {
    if (n < 0 || (n > 0 && (!odom || !i_prev || !i_cur || !out))) return DPG_ERR_ARG;
    int rc = DPG_OK;
    for (int64_t k = 0; k < n; ++k) {
        const int32_t a = i_prev[k], b = i_cur[k];
        if (a < 0 || b < 0 || a >= n_odom || b >= n_odom) return DPG_ERR_ARG;
        const int r = dpg_odometry_factor(odom + 3 * (int64_t)a, odom + 3 * (int64_t)b, a, b, transl_from_transl,
                                          transl_from_rot, rot_from_transl, rot_from_rot, out + k);
        if (r && rc == DPG_OK) rc = r;
    }
    return rc;
}

/* R9: ICP BetweenFactor (addObservationConstraint, dpg_slam.cc:331-338); the covariance is the
 * constant diagonal of calculate_ICP_COV, which GTSAM's smart Gaussian::Covariance reduces to a
 * Diagonal model with precisions 1/variance. */
void dpg_icp_factor(const dpg_icp_result* r, int32_t from_node, int32_t to_node, const dpg_icp_params* p,
                    dpg_factor* out) {
    memset(out, 0, sizeof(*out));
    out->kind = DPG_FACTOR_BETWEEN;
    out->i = from_node;
    out->j = to_node;
    out->z[0] = r->z[0];
    out->z[1] = r->z[1];
    out->z[2] = r->z[2];
    out->info[0] = 1.0 / (double)p->laser_x_variance;
    out->info[1] = 1.0 / (double)p->laser_y_variance;
    out->info[2] = 1.0 / (double)p->laser_theta_variance;
}

/* R1 over a whole scan set: ranges[V][n_beams] -> concatenated clouds + offsets[V+1]. */
int64_t dpg_scans_to_clouds(const float* ranges, int64_t n_nodes, int64_t n_beams, float angle_min,
                            float angle_max, float range_max, float laser_x, float laser_y,
                            float laser_theta, float* xy_out, int64_t* offsets_out) {
    if (!ranges || !xy_out || !offsets_out || n_nodes <= 0) return -1;
    int64_t total = 0;
    offsets_out[0] = 0;
    for (int64_t v = 0; v < n_nodes; ++v) {
        total += dpg_scan_to_cloud(ranges + v * n_beams, n_beams, angle_min, angle_max, range_max, laser_x,
                                   laser_y, laser_theta, xy_out + 2 * total);
        offsets_out[v + 1] = total;
    }
    return total;
}
