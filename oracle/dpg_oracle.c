/*
 * dpg_oracle.c -- TEST INFRASTRUCTURE ONLY (see dpg_oracle.h for the pinning status).
 *
 * Plain-C restatement of the DPG-SLAM hot path:
 *   R1  polar scan -> base_link cloud      dpg_measurement.h:41-46,102-104; dpg_slam.cc:488-513;
 *                                          dpg_node.cc:8-25; math_utils.cc:6-19
 *   R2  downsamplePointCloud               dpg_slam.cc:346-360
 *   R3  runIcp guess                       dpg_slam.cc:364-378; math_utils.cc:21-35
 *   R4  PCL determineReciprocalCorrespondences + KdTreeFLANN 1-NN (lowest-index tie rule)
 *   R5  PCL TransformationEstimationSVD/umeyama -> planar closed form, 512-lane fp64 tree
 *   R6  PCL ICP loop + DefaultConvergenceCriteria
 *   R7  calculate_ICP_COV                  cov_func_point_to_point.h:24-31,45-283,572-575
 *   R8  runIcp epilogue                    dpg_slam.cc:416-445
 *   R10 GTSAM Pose2 Prior/Between linearization, GaussNewton, CHOLESKY (block-sparse, min-degree)
 * Compiled with -ffp-contract=off: every float/double operation below is one IEEE rounding, in
 * the order written.  Nothing here is product code.
 */
#include "dpg_oracle.h"

#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ R1 - R3 (host data path) */

/* math_utils::AngleMod<float> (math_utils.h:13-16): the subtraction runs in double. */
static float angle_mod_f(float a) {
    double ad = (double)a;
    ad -= (M_PI * 2.0) * rint(ad / (M_PI * 2.0));
    return (float)ad;
}

/* Eigen::Rotation2Df(th) * v (toRotationMatrix: [c -s; s c], coefficient-wise product). */
static void rot2f(float th, float x, float y, float* ox, float* oy) {
    float c = cosf(th), s = sinf(th);
    float ns = -s;
    *ox = c * x + ns * y;
    *oy = s * x + c * y;
}

int64_t oracle_scan_to_cloud(const float* ranges, int64_t n, float angle_min, float angle_max,
                             float range_max, float lx, float ly, float lth, float* xy_out) {
    /* createNode (dpg_slam.cc:497): float diff, double division by (size - 1.0), stored float */
    float angle_inc = (float)((double)(angle_max - angle_min) / ((double)n - 1.0));
    int64_t k = 0;
    for (int64_t i = 0; i < n; ++i) {
        float angle = angle_inc * (float)i + angle_min;          /* dpg_slam.cc:506 */
        float r = ranges[i];
        if (r >= range_max) continue;                              /* MAX_RANGE, dpg_measurement.h:43 */
        float px = r * cosf(angle), py = r * sinf(angle);          /* dpg_measurement.h:102-104 */
        float rx, ry;
        rot2f(lth, px, py, &rx, &ry);                              /* math_utils.cc:10-11 */
        xy_out[2 * k] = lx + rx;                                   /* math_utils.cc:14 */
        xy_out[2 * k + 1] = ly + ry;
        ++k;
    }
    return k;
}

int64_t oracle_downsample(const float* xy, int64_t n, int32_t ratio, float* xy_out) {
    int64_t k = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (i % ratio == 0) {
            xy_out[2 * k] = xy[2 * i];
            xy_out[2 * k + 1] = xy[2 * i + 1];
            ++k;
        }
    }
    return k;
}

/* inverseTransformPoint(src = a, target frame = b) (math_utils.cc:21-35). */
void oracle_inverse_transform_point(const float a[3], const float b[3], float out[3]) {
    float tx = a[0] - b[0], ty = a[1] - b[1];
    rot2f(-b[2], tx, ty, &out[0], &out[1]);
    out[2] = angle_mod_f(a[2] - b[2]);
}

/* transformPoint(p in frame f) (math_utils.cc:6-19). */
void oracle_transform_point(const float p[3], const float f[3], float out[3]) {
    float rx, ry;
    rot2f(f[2], p[0], p[1], &rx, &ry);
    out[0] = f[0] + rx;
    out[1] = f[1] + ry;
    out[2] = angle_mod_f(f[2] + p[2]);
}

/* dpg_slam.cc:364-378: node_2 (source) expressed in node_1 (target) frame, 4x4 float guess. */
void oracle_icp_guess(const float pose_src[3], const float pose_tgt[3], float g[6]) {
    float d[3];
    oracle_inverse_transform_point(pose_src, pose_tgt, d);
    float c = cosf(d[2]), s = sinf(d[2]);
    g[0] = c; g[1] = -s; g[2] = d[0];
    g[3] = s; g[4] = c;  g[5] = d[1];
}

/* ------------------------------------------------------------------ R4 nearest neighbours */

/* FLANN L2_Simple over (x, y, z = 0): ((0 + dx*dx) + dy*dy) + 0 in float. */
static inline float sqdist(float ax, float ay, float bx, float by) {
    float dx = ax - bx, dy = ay - by;
    return dx * dx + dy * dy;
}

/* Exact 1-NN over pts[0..n), lowest index among equal distances. */
static void nn_brute(const float* pts, int64_t n, float qx, float qy, int32_t* idx, float* d) {
    float bd = INFINITY;
    int32_t bi = -1;
    for (int64_t k = 0; k < n; ++k) {
        float dd = sqdist(qx, qy, pts[2 * k], pts[2 * k + 1]);
        if (dd < bd) { bd = dd; bi = (int32_t)k; }
    }
    *idx = bi;
    *d = bd;
}

/* Uniform grid with cell >= 1.05 r: every point whose float distance is <= r^2 lies in the
 * 3x3 block of cells around the query, so the argmin over those cells (ties -> lowest index)
 * equals the brute-force argmin whenever the latter passes the r^2 test. */
typedef struct {
    float x0, y0, inv_h;
    int32_t gx, gy;
    int32_t* start;   /* gx*gy + 1 */
    int32_t* order;   /* point indices sorted by cell */
    int32_t cap_cells;
} grid_t;

static void grid_build(grid_t* g, const float* pts, int64_t n, double r) {
    float mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
    for (int64_t k = 0; k < n; ++k) {
        float x = pts[2 * k], y = pts[2 * k + 1];
        if (x < mnx) mnx = x;
        if (x > mxx) mxx = x;
        if (y < mny) mny = y;
        if (y > mxy) mxy = y;
    }
    if (n == 0) { mnx = mny = 0.f; mxx = mxy = 0.f; }
    double h = r * 1.05;
    double ex = (double)mxx - (double)mnx, ey = (double)mxy - (double)mny;
    if (ex / 64.0 > h) h = ex / 64.0;
    if (ey / 64.0 > h) h = ey / 64.0;
    g->x0 = mnx;
    g->y0 = mny;
    g->inv_h = (float)(1.0 / h);
    g->gx = (int32_t)(ex / h) + 1;
    g->gy = (int32_t)(ey / h) + 1;
    int32_t nc = g->gx * g->gy;
    if (nc + 1 > g->cap_cells) {
        free(g->start);
        g->start = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nc + 1));
        g->cap_cells = nc + 1;
    }
    memset(g->start, 0, sizeof(int32_t) * (size_t)(nc + 1));
    int32_t* cell = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
    for (int64_t k = 0; k < n; ++k) {
        int32_t cx = (int32_t)floorf((pts[2 * k] - g->x0) * g->inv_h);
        int32_t cy = (int32_t)floorf((pts[2 * k + 1] - g->y0) * g->inv_h);
        if (cx < 0) cx = 0;
        if (cx >= g->gx) cx = g->gx - 1;
        if (cy < 0) cy = 0;
        if (cy >= g->gy) cy = g->gy - 1;
        cell[k] = cy * g->gx + cx;
        g->start[cell[k] + 1]++;
    }
    for (int32_t c = 0; c < nc; ++c) g->start[c + 1] += g->start[c];
    int32_t* cur = (int32_t*)malloc(sizeof(int32_t) * (size_t)nc);
    memcpy(cur, g->start, sizeof(int32_t) * (size_t)nc);
    free(g->order);
    g->order = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n ? n : 1));
    for (int64_t k = 0; k < n; ++k) g->order[cur[cell[k]]++] = (int32_t)k;
    free(cur);
    free(cell);
}

static void grid_free(grid_t* g) {
    free(g->start);
    free(g->order);
    g->start = NULL;
    g->order = NULL;
    g->cap_cells = 0;
}

static void nn_grid(const grid_t* g, const float* pts, float qx, float qy, int32_t* idx, float* d) {
    float fx = floorf((qx - g->x0) * g->inv_h), fy = floorf((qy - g->y0) * g->inv_h);
    float bd = INFINITY;
    int32_t bi = -1;
    if (fx >= -1.f && fy >= -1.f && fx <= (float)g->gx && fy <= (float)g->gy) {
        int32_t cx = (int32_t)fx, cy = (int32_t)fy;
        for (int32_t yy = cy - 1; yy <= cy + 1; ++yy) {
            if (yy < 0 || yy >= g->gy) continue;
            int32_t c0 = cx - 1 < 0 ? 0 : cx - 1, c1 = cx + 1 >= g->gx ? g->gx - 1 : cx + 1;
            if (c0 > c1) continue;
            for (int32_t s = g->start[yy * g->gx + c0]; s < g->start[yy * g->gx + c1 + 1]; ++s) {
                int32_t k = g->order[s];
                float dd = sqdist(qx, qy, pts[2 * k], pts[2 * k + 1]);
                if (dd < bd || (dd == bd && k < bi)) { bd = dd; bi = k; }
            }
        }
    }
    *idx = bi;
    *d = bd;
}

/* ------------------------------------------------------------------ R5/R6 ICP */

/* sums (csrc/dpg_icp_tree.h): count, d, p, q, dot = px qx + py qy, cross = px qy - py qx */
enum { S_CNT = 0, S_D, S_PX, S_PY, S_QX, S_QY, S_DOT, S_CROSS, S_N };

/* The 512-lane fixed reduction (DPG_ICP_LANES = 8 waves x 64 lanes, include/dpg_slam_c.h):
 * inside each 64-lane wave acc[k] += acc[k + off] for off = 32, 16, ..., 1; then
 * ((W0 + W1) + (W2 + W3)) + ((W4 + W5) + (W6 + W7)).  GPU side: csrc/dpg_icp_tree.h. */
static void lane_tree(double acc[DPG_ICP_LANES][S_N], double out[S_N]) {
    double W[8][S_N];
    for (int w = 0; w < 8; ++w) {
        double (*a)[S_N] = acc + 64 * w;
        for (int off = 32; off >= 1; off >>= 1)
            for (int k = 0; k < off; ++k)
                for (int q = 0; q < S_N; ++q) a[k][q] = a[k][q] + a[k + off][q];
        for (int q = 0; q < S_N; ++q) W[w][q] = a[0][q];
    }
    for (int q = 0; q < S_N; ++q)
        out[q] = ((W[0][q] + W[1][q]) + (W[2][q] + W[3][q])) + ((W[4][q] + W[5][q]) + (W[6][q] + W[7][q]));
}

/* Planar rigid fit from the reduced sums; returns (c, s, tx, ty) rounded to float. */
static void rigid_from_sums(const double S[S_N], float* cf, float* sf, float* txf, float* tyf) {
    double n = S[S_CNT];
    double a = S[S_DOT] - (S[S_PX] * S[S_QX] + S[S_PY] * S[S_QY]) / n;
    double b = S[S_CROSS] - (S[S_PX] * S[S_QY] - S[S_PY] * S[S_QX]) / n;
    double h = sqrt(a * a + b * b);
    double c = 1.0, s = 0.0;
    if (h > 0.0) { c = a / h; s = b / h; }
    double mpx = S[S_PX] / n, mpy = S[S_PY] / n, mqx = S[S_QX] / n, mqy = S[S_QY] / n;
    double tx = mqx - (c * mpx - s * mpy);
    double ty = mqy - (s * mpx + c * mpy);
    *cf = (float)c;
    *sf = (float)s;
    *txf = (float)tx;
    *tyf = (float)ty;
}

int oracle_icp_align(const float* src_in, int64_t n_src, const float* tgt, int64_t n_tgt,
                     const float G[6], const dpg_icp_params* p, int nn_mode,
                     dpg_icp_result* res, int32_t* trace, int32_t trace_iters) {
    memset(res, 0, sizeof(*res));
    float* src = (float*)malloc(sizeof(float) * 2 * (size_t)(n_src ? n_src : 1));
    int32_t* fwd = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n_src ? n_src : 1));
    float* fd = (float*)malloc(sizeof(float) * (size_t)(n_src ? n_src : 1));
    double (*acc)[S_N] = (double (*)[S_N])malloc(sizeof(double) * DPG_ICP_LANES * S_N);
    grid_t tg = {0}, sg = {0};
    const double r = p->icp_max_correspondence_distance;
    const double r2 = r * r;                                   /* max_dist_sqr */
    const double eps = p->icp_maximum_transformation_epsilon;
    const double rot_thr = 1.0 - eps;                          /* rotation_threshold_ */

    /* src <- guess * src (ICP::computeTransformation, transformCloud) */
    for (int64_t i = 0; i < n_src; ++i) {
        float x = src_in[2 * i], y = src_in[2 * i + 1];
        src[2 * i] = (G[0] * x + G[1] * y) + G[2];
        src[2 * i + 1] = (G[3] * x + G[4] * y) + G[5];
    }
    float F[6];
    memcpy(F, G, sizeof(F));
    if (nn_mode == ORACLE_NN_GRID) grid_build(&tg, tgt, n_tgt, r);

    double prev_mse = DBL_MAX;
    int32_t k = 0;
    int converged = 0;
    int status = DPG_ICP_OK;
    int32_t last_cnt = 0;
    double last_mse = 0.0;
    for (;;) {
        /* R4: forward 1-NN, r^2 test, reciprocal 1-NN on the current (moved) source */
        if (nn_mode == ORACLE_NN_GRID && p->icp_use_reciprocal_correspondences)
            grid_build(&sg, src, n_src, r);
        int32_t cnt = 0;
        for (int64_t i = 0; i < n_src; ++i) {
            int32_t j;
            float d;
            if (nn_mode == ORACLE_NN_GRID) nn_grid(&tg, tgt, src[2 * i], src[2 * i + 1], &j, &d);
            else nn_brute(tgt, n_tgt, src[2 * i], src[2 * i + 1], &j, &d);
            fwd[i] = -1;
            if (j < 0 || (double)d > r2) continue;
            if (p->icp_use_reciprocal_correspondences) {
                int32_t ir;
                float dr;
                if (nn_mode == ORACLE_NN_GRID) nn_grid(&sg, src, tgt[2 * j], tgt[2 * j + 1], &ir, &dr);
                else nn_brute(src, n_src, tgt[2 * j], tgt[2 * j + 1], &ir, &dr);
                if ((double)dr > r2 || ir != (int32_t)i) continue;
            }
            fwd[i] = j;
            fd[i] = d;
            ++cnt;
        }
        if (trace && k < trace_iters) memcpy(trace + (size_t)k * (size_t)n_src, fwd, sizeof(int32_t) * (size_t)n_src);
        last_cnt = cnt;
        if (cnt < p->min_number_correspondences) {   /* "Not enough correspondences found" */
            converged = 0;
            status = DPG_ICP_TOO_FEW_CORR;
            break;
        }
        /* R5: sums over accepted pairs, 512-lane tree */
        memset(acc, 0, sizeof(double) * DPG_ICP_LANES * S_N);
        for (int64_t i = 0; i < n_src; ++i) {
            if (fwd[i] < 0) continue;
            int l = (int)(i % DPG_ICP_LANES);
            double px = src[2 * i], py = src[2 * i + 1];
            double qx = tgt[2 * fwd[i]], qy = tgt[2 * fwd[i] + 1];
            acc[l][S_CNT] = acc[l][S_CNT] + 1.0;
            acc[l][S_D] = acc[l][S_D] + (double)fd[i];
            acc[l][S_PX] = acc[l][S_PX] + px;
            acc[l][S_PY] = acc[l][S_PY] + py;
            acc[l][S_QX] = acc[l][S_QX] + qx;
            acc[l][S_QY] = acc[l][S_QY] + qy;
            acc[l][S_DOT] = acc[l][S_DOT] + (px * qx + py * qy);
            acc[l][S_CROSS] = acc[l][S_CROSS] + (px * qy - py * qx);
        }
        double S[S_N];
        lane_tree(acc, S);
        float c, s, tx, ty;
        rigid_from_sums(S, &c, &s, &tx, &ty);
        float ns = -s;
        /* transformCloud(in place) */
        for (int64_t i = 0; i < n_src; ++i) {
            float x = src[2 * i], y = src[2 * i + 1];
            src[2 * i] = (c * x + ns * y) + tx;
            src[2 * i + 1] = (s * x + c * y) + ty;
        }
        /* final_transformation_ = transformation_ * final_transformation_ */
        float N[6];
        N[0] = c * F[0] + ns * F[3];
        N[1] = c * F[1] + ns * F[4];
        N[2] = (c * F[2] + ns * F[5]) + tx;
        N[3] = s * F[0] + c * F[3];
        N[4] = s * F[1] + c * F[4];
        N[5] = (s * F[2] + c * F[5]) + ty;
        memcpy(F, N, sizeof(F));
        ++k;
        double mse = S[S_D] / S[S_CNT];                       /* calculateMSE */
        last_mse = mse;
        /* R6: DefaultConvergenceCriteria::hasConverged */
        if (k >= p->icp_maximum_iterations) { converged = 1; break; }
        float tr = ((c + c) + 1.0f) - 1.0f;
        double cos_angle = 0.5 * (double)tr;
        double tsq = (double)(tx * tx + ty * ty);
        if (cos_angle >= rot_thr && tsq <= eps) { converged = 1; break; }
        if (fabs(mse - prev_mse) < p->mse_threshold_absolute) { converged = 1; break; }
        prev_mse = mse;
    }
    memcpy(res->T, F, sizeof(F));
    res->z[0] = F[2];
    res->z[1] = F[5];
    res->z[2] = atan2f(F[3], F[0]);    /* Rotation2Df::fromRotationMatrix: std::atan2(float, float) */
    res->converged = converged;
    res->iterations = k;
    res->n_corr = last_cnt;
    res->status = status;
    res->fitness = last_mse;
    grid_free(&tg);
    grid_free(&sg);
    free(acc);
    free(fd);
    free(fwd);
    free(src);
    return 0;
}

/* ------------------------------------------------------------------ R7 covariance */

void oracle_icp_cov(const float* data, int64_t nd, const float* model, int64_t nm, const float T[6],
                    float vx, float vy, float vth, double cov[9], double hess[9]) {
    /* :572-575 -- the graph-facing output */
    memset(cov, 0, 9 * sizeof(double));
    cov[0] = (double)vx;
    cov[4] = (double)vy;
    cov[8] = (double)vth;
    if (!hess) return;
    /* :26-35 with T20 = T21 = 0, T22 = 1 (b = c = 0): yaw from the float rotation */
    double a = (double)atan2f(T[3], T[0]);   /* cov :31 yaw = atan2f(T10, T00) */
    double x = T[2], y = T[5];
    double ca = cos(a), sa = sin(a);
    double h00 = 0, h01 = 0, h02 = 0, h11 = 0, h12 = 0, h22 = 0;
    int64_t n = nd < nm ? nd : nm;
    for (int64_t s = 0; s < n; ++s) {
        double px = data[2 * s], py = data[2 * s + 1];
        double qx = model[2 * s], qy = model[2 * s + 1];
        double ux = ca * px - sa * py;                      /* R(a) p */
        double uy = sa * px + ca * py;
        double rx = (x - qx) + ux;                          /* residual t + R p - q */
        double ry = (y - qy) + uy;
        h00 += 2.0;                                         /* d2J_dx2 */
        h11 += 2.0;                                         /* d2J_dy2 */
        h02 += -2.0 * uy;                                   /* d2J_dxda */
        h12 += 2.0 * ux;                                    /* d2J_dyda */
        h22 += 2.0 * (ux * ux + uy * uy) - 2.0 * (ux * rx + uy * ry);   /* d2J_da2 */
    }
    hess[0] = h00; hess[1] = h01; hess[2] = h02;
    hess[3] = h01; hess[4] = h11; hess[5] = h12;
    hess[6] = h02; hess[7] = h12; hess[8] = h22;
}

void oracle_cov_block_literal(const float* data, int64_t nd, const float* model, int64_t nm,
                              const float T[6], double hess[9]) {
    /* The reference's generated expressions (cov :133-135, :148-160) with b = c = piz = qiz = 0
     * substituted symbol by symbol (sin(0) = 0, cos(0) = 1), evaluated without simplification. */
    double a = (double)atan2f(T[3], T[0]);   /* cov :31 yaw = atan2f(T10, T00) */
    double x = T[2], y = T[5];
    double sb = sin(0.0), cb = cos(0.0), sc = sin(0.0), cc = cos(0.0), piz = 0.0;
    double S[6] = {0, 0, 0, 0, 0, 0};
    int64_t n = nd < nm ? nd : nm;
    for (int64_t s = 0; s < n; ++s) {
        double pix = data[2 * s], piy = data[2 * s + 1], qix = model[2 * s], qiy = model[2 * s + 1];
        double sa = sin(a), ca = cos(a);
        double A1 = piz * (sa * sc + ca * cc * sb) - piy * (cc * sa - ca * sb * sc) + pix * ca * cb;
        double A2 = 2 * piz * (sa * sc + ca * cc * sb) - 2 * piy * (cc * sa - ca * sb * sc) + 2 * pix * ca * cb;
        double B1 = piy * (ca * cc + sa * sb * sc) - piz * (ca * sc - cc * sa * sb) + pix * cb * sa;
        double B2 = 2 * piy * (ca * cc + sa * sb * sc) - 2 * piz * (ca * sc - cc * sa * sb) + 2 * pix * cb * sa;
        double RY = y - qiy + B1;
        double RX = x - qix - piy * (cc * sa - ca * sb * sc) + piz * (sa * sc + ca * cc * sb) + pix * ca * cb;
        double da2 = A1 * A2 - B2 * RY + B1 * B2 - A2 * RX;
        double dxda = 2 * piz * (ca * sc - cc * sa * sb) - 2 * piy * (ca * cc + sa * sb * sc) - 2 * pix * cb * sa;
        double dyda = 2 * piz * (sa * sc + ca * cc * sb) - 2 * piy * (cc * sa - ca * sb * sc) + 2 * pix * ca * cb;
        S[0] += 2; S[1] += 2; S[2] += dxda; S[3] += dyda; S[4] += da2;
    }
    hess[0] = S[0]; hess[1] = 0; hess[2] = S[2];
    hess[3] = 0; hess[4] = S[1]; hess[5] = S[3];
    hess[6] = S[2]; hess[7] = S[3]; hess[8] = S[4];
}

int oracle_run_icp(const float* src_full, int64_t n_src, const float* tgt_full, int64_t n_tgt,
                   const float pose_src[3], const float pose_tgt[3], const dpg_icp_params* p,
                   int nn_mode, dpg_icp_result* res, double cov[9], double hess[9]) {
    int32_t ratio = p->downsample_icp_points_ratio > 0 ? p->downsample_icp_points_ratio : 1;
    float* sd = (float*)malloc(sizeof(float) * 2 * (size_t)(n_src + 1));
    float* td = (float*)malloc(sizeof(float) * 2 * (size_t)(n_tgt + 1));
    int64_t ns = oracle_downsample(src_full, n_src, ratio, sd);
    int64_t nt = oracle_downsample(tgt_full, n_tgt, ratio, td);
    float G[6];
    oracle_icp_guess(pose_src, pose_tgt, G);
    oracle_icp_align(sd, ns, td, nt, G, p, nn_mode, res, NULL, 0);
    oracle_icp_cov(src_full, n_src, tgt_full, n_tgt, res->T, p->laser_x_variance,
                   p->laser_y_variance, p->laser_theta_variance, cov, hess);
    free(sd);
    free(td);
    return 0;
}

int oracle_icp_batch(const float* pts, const int64_t* offs, int64_t n_nodes, const int32_t* edges,
                     int64_t n_edges, const float* poses, const dpg_icp_params* p, int nn_mode,
                     int n_threads, dpg_icp_result* res, double* hess) {
    (void)n_nodes;
#ifdef _OPENMP
    if (n_threads < 1) n_threads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads)
#endif
    for (int64_t e = 0; e < n_edges; ++e) {
        int32_t t = edges[2 * e], s = edges[2 * e + 1];   /* node_1 = target, node_2 = source */
        double cov[9];
        oracle_run_icp(pts + 2 * offs[s], offs[s + 1] - offs[s], pts + 2 * offs[t], offs[t + 1] - offs[t],
                       poses + 3 * s, poses + 3 * t, p, nn_mode, &res[e], cov, hess ? hess + 9 * e : NULL);
    }
    return 0;
}

/* ------------------------------------------------------------------ R10 GTSAM semantics */

/* Pose2::between (GTSAM Pose2.cpp) with H1; H2 = I. Returns h = a^-1 b as (x, y, c, s). */
static void pose_between(const double* a, const double* b, double h[4], double H1[9]) {
    double c1 = cos(a[2]), s1 = sin(a[2]), c2 = cos(b[2]), s2 = sin(b[2]);
    double c = c1 * c2 + s1 * s2, s = -s1 * c2 + c1 * s2;
    double dx = b[0] - a[0], dy = b[1] - a[1];
    h[0] = c1 * dx + s1 * dy;
    h[1] = -s1 * dx + c1 * dy;
    h[2] = c;
    h[3] = s;
    if (H1) {
        double dt1 = -s2 * dx + c2 * dy, dt2 = -c2 * dx - s2 * dy;
        H1[0] = -c; H1[1] = -s; H1[2] = dt1;
        H1[3] = s;  H1[4] = -c; H1[5] = dt2;
        H1[6] = 0;  H1[7] = 0;  H1[8] = -1;
    }
}

/* Rot2::atan2 normalization then theta(). */
static double rot_theta(double c, double s) { return atan2(s, c); }

/* error + whitening-free Jacobians of one factor (BetweenFactor::evaluateError without
 * SLOW_BUT_CORRECT_BETWEENFACTOR, PriorFactor::evaluateError; GTSAM 4.x defaults). */
void oracle_linearize(const dpg_factor* f, const double* X, double e[3], double Ai[9], double Aj[9]) {
    if (f->kind == DPG_FACTOR_PRIOR) {
        /* -Local(x, prior) = -(x^-1 prior) in the ChartAtOrigin (x, y, theta) */
        double h[4];
        pose_between(X + 3 * f->i, f->z, h, NULL);
        e[0] = -h[0];
        e[1] = -h[1];
        e[2] = -rot_theta(h[2], h[3]);
        for (int q = 0; q < 9; ++q) Ai[q] = (q % 4 == 0) ? 1.0 : 0.0;
        if (Aj) for (int q = 0; q < 9; ++q) Aj[q] = 0.0;
        return;
    }
    double h[4];
    pose_between(X + 3 * f->i, X + 3 * f->j, h, Ai);
    /* Local(z, h) = z^-1 h */
    double cz = cos(f->z[2]), sz = sin(f->z[2]);
    double n = h[2] * h[2] + h[3] * h[3];
    double ch = h[2], sh = h[3];
    if (fabs(n - 1.0) > 1e-10) { double sc = pow(n, -0.5); ch *= sc; sh *= sc; }
    double c = cz * ch + sz * sh, s = -sz * ch + cz * sh;
    double dx = h[0] - f->z[0], dy = h[1] - f->z[1];
    e[0] = cz * dx + sz * dy;
    e[1] = -sz * dx + cz * dy;
    e[2] = rot_theta(c, s);
    if (Aj) for (int q = 0; q < 9; ++q) Aj[q] = (q % 4 == 0) ? 1.0 : 0.0;
}

double oracle_graph_error(const double* X, const dpg_factor* f, int64_t nf) {
    double err = 0.0;
    for (int64_t k = 0; k < nf; ++k) {
        double e[3], Ai[9], Aj[9];
        oracle_linearize(&f[k], X, e, Ai, Aj);
        err += 0.5 * (f[k].info[0] * e[0] * e[0] + f[k].info[1] * e[1] * e[1] + f[k].info[2] * e[2] * e[2]);
    }
    return err;
}

/* ---- block-sparse symmetric system, min-degree ordering, right-looking block Cholesky ---- */

typedef struct {
    int64_t n;            /* nodes */
    double* diag;         /* [n][9] */
    double* g;            /* [n][3] */
    /* pair hash: key lo*n+hi -> block [9] storing H(lo, hi) */
    int64_t cap;
    int64_t* keys;
    double* blk;
} sys_t;

static int64_t hslot(sys_t* S, int64_t key, int create) {
    uint64_t hsh = (uint64_t)key * 0x9E3779B97F4A7C15ull;
    int64_t m = S->cap - 1;
    int64_t pos = (int64_t)(hsh >> 17) & m;
    for (;;) {
        if (S->keys[pos] == key) return pos;
        if (S->keys[pos] == -1) {
            if (!create) return -1;
            S->keys[pos] = key;
            memset(S->blk + 9 * pos, 0, 9 * sizeof(double));
            return pos;
        }
        pos = (pos + 1) & m;
    }
}

static void sys_init(sys_t* S, int64_t n, int64_t n_pairs_hint) {
    S->n = n;
    S->diag = (double*)calloc((size_t)(9 * n), sizeof(double));
    S->g = (double*)calloc((size_t)(3 * n), sizeof(double));
    int64_t cap = 16;
    while (cap < 4 * n_pairs_hint + 16) cap <<= 1;
    S->cap = cap;
    S->keys = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
    for (int64_t k = 0; k < cap; ++k) S->keys[k] = -1;
    S->blk = (double*)malloc(sizeof(double) * 9 * (size_t)cap);
}

static void sys_free(sys_t* S) {
    free(S->diag); free(S->g); free(S->keys); free(S->blk);
}

/* C += A^T diag(w) B, all 3x3 row-major */
static void atwb(const double* A, const double* w, const double* B, double* C) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double acc = 0.0;
            for (int k = 0; k < 3; ++k) acc += A[3 * k + r] * w[k] * B[3 * k + c];
            C[3 * r + c] += acc;
        }
}

static double sys_assemble(sys_t* S, const double* X, const dpg_factor* f, int64_t nf) {
    memset(S->diag, 0, sizeof(double) * 9 * (size_t)S->n);
    memset(S->g, 0, sizeof(double) * 3 * (size_t)S->n);
    for (int64_t k = 0; k < S->cap; ++k) if (S->keys[k] >= 0) memset(S->blk + 9 * k, 0, 9 * sizeof(double));
    double err = 0.0;
    for (int64_t k = 0; k < nf; ++k) {
        double e[3], Ai[9], Aj[9];
        oracle_linearize(&f[k], X, e, Ai, Aj);
        const double* w = f[k].info;
        err += 0.5 * (w[0] * e[0] * e[0] + w[1] * e[1] * e[1] + w[2] * e[2] * e[2]);
        int64_t i = f[k].i;
        atwb(Ai, w, Ai, S->diag + 9 * i);
        for (int r = 0; r < 3; ++r) {
            double acc = 0.0;
            for (int q = 0; q < 3; ++q) acc += Ai[3 * q + r] * w[q] * e[q];
            S->g[3 * i + r] += acc;
        }
        if (f[k].kind != DPG_FACTOR_BETWEEN) continue;
        int64_t j = f[k].j;
        atwb(Aj, w, Aj, S->diag + 9 * j);
        for (int r = 0; r < 3; ++r) {
            double acc = 0.0;
            for (int q = 0; q < 3; ++q) acc += Aj[3 * q + r] * w[q] * e[q];
            S->g[3 * j + r] += acc;
        }
        if (i == j) continue;
        double blk[9] = {0};
        if (i < j) atwb(Ai, w, Aj, blk);
        else atwb(Aj, w, Ai, blk);
        int64_t lo = i < j ? i : j, hi = i < j ? j : i;
        int64_t sl = hslot(S, lo * S->n + hi, 1);
        for (int q = 0; q < 9; ++q) S->blk[9 * sl + q] += blk[q];
    }
    return err;
}

/* symbolic: min-degree ordering on the node graph with bitset elimination graphs */
typedef struct {
    int64_t n;
    int64_t* perm;      /* elimination order: perm[p] = node */
    int64_t* pos;       /* pos[node] = p */
    int64_t* cptr;      /* column pointers (per elimination step) into crow */
    int64_t* crow;      /* rows (nodes) of L below the diagonal, sorted by pos */
} sym_t;

static int cmp_pos_ctx_n;
static int64_t* cmp_pos_ctx;
static int cmp_by_pos(const void* a, const void* b) {
    int64_t pa = cmp_pos_ctx[*(const int64_t*)a], pb = cmp_pos_ctx[*(const int64_t*)b];
    return (pa > pb) - (pa < pb);
}

static int sym_analyze(sym_t* Y, int64_t n, const dpg_factor* f, int64_t nf) {
    int64_t W = (n + 63) / 64;
    uint64_t* adj = (uint64_t*)calloc((size_t)(n * W), sizeof(uint64_t));
    if (!adj) return -1;
    for (int64_t k = 0; k < nf; ++k) {
        if (f[k].kind != DPG_FACTOR_BETWEEN || f[k].i == f[k].j) continue;
        int64_t i = f[k].i, j = f[k].j;
        adj[i * W + j / 64] |= 1ull << (j % 64);
        adj[j * W + i / 64] |= 1ull << (i % 64);
    }
    int64_t* deg = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    char* done = (char*)calloc((size_t)n, 1);
    for (int64_t v = 0; v < n; ++v) {
        int64_t d = 0;
        for (int64_t w = 0; w < W; ++w) d += __builtin_popcountll(adj[v * W + w]);
        deg[v] = d;
    }
    Y->n = n;
    Y->perm = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    Y->pos = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    Y->cptr = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    int64_t cap = 8 * n + 16, used = 0;
    Y->crow = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
    int64_t* nb = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
    for (int64_t p = 0; p < n; ++p) {
        int64_t v = -1, best = INT64_MAX;
        for (int64_t u = 0; u < n; ++u)
            if (!done[u] && deg[u] < best) { best = deg[u]; v = u; }
        done[v] = 1;
        Y->perm[p] = v;
        Y->pos[v] = p;
        Y->cptr[p] = used;
        int64_t m = 0;
        for (int64_t w = 0; w < W; ++w) {
            uint64_t bits = adj[v * W + w];
            while (bits) {
                int b = __builtin_ctzll(bits);
                bits &= bits - 1;
                nb[m++] = w * 64 + b;
            }
        }
        if (used + m > cap) {
            while (used + m > cap) cap *= 2;
            Y->crow = (int64_t*)realloc(Y->crow, sizeof(int64_t) * (size_t)cap);
        }
        memcpy(Y->crow + used, nb, sizeof(int64_t) * (size_t)m);
        used += m;
        /* eliminate v: neighbours become a clique */
        for (int64_t a = 0; a < m; ++a) {
            int64_t u = nb[a];
            uint64_t* au = adj + u * W;
            const uint64_t* av = adj + v * W;
            for (int64_t w = 0; w < W; ++w) au[w] |= av[w];
            au[u / 64] &= ~(1ull << (u % 64));
            au[v / 64] &= ~(1ull << (v % 64));
        }
        for (int64_t a = 0; a < m; ++a) {
            int64_t u = nb[a], d = 0;
            for (int64_t w = 0; w < W; ++w) d += __builtin_popcountll(adj[u * W + w]);
            deg[u] = d;
        }
        memset(adj + v * W, 0, sizeof(uint64_t) * (size_t)W);
    }
    Y->cptr[n] = used;
    /* sort each column's rows by elimination position */
    cmp_pos_ctx = Y->pos;
    cmp_pos_ctx_n = 1;
    for (int64_t p = 0; p < n; ++p)
        qsort(Y->crow + Y->cptr[p], (size_t)(Y->cptr[p + 1] - Y->cptr[p]), sizeof(int64_t), cmp_by_pos);
    free(nb); free(deg); free(done); free(adj);
    return 0;
}

static void sym_free(sym_t* Y) { free(Y->perm); free(Y->pos); free(Y->cptr); free(Y->crow); }

/* dense 3x3 Cholesky (lower, row-major), returns 0 on success */
static int chol3(double* A) {
    double l00 = A[0];
    if (!(l00 > 0)) return -1;
    l00 = sqrt(l00);
    double l10 = A[3] / l00, l20 = A[6] / l00;
    double d1 = A[4] - l10 * l10;
    if (!(d1 > 0)) return -1;
    double l11 = sqrt(d1);
    double l21 = (A[7] - l20 * l10) / l11;
    double d2 = A[8] - l20 * l20 - l21 * l21;
    if (!(d2 > 0)) return -1;
    double l22 = sqrt(d2);
    A[0] = l00; A[1] = 0; A[2] = 0;
    A[3] = l10; A[4] = l11; A[5] = 0;
    A[6] = l20; A[7] = l21; A[8] = l22;
    return 0;
}

/* X = B * L^-T (B: 3x3, L lower) */
static void rsolve_lt(const double* L, double* B) {
    for (int r = 0; r < 3; ++r) {
        double x0 = B[3 * r] / L[0];
        double x1 = (B[3 * r + 1] - L[3] * x0) / L[4];
        double x2 = (B[3 * r + 2] - L[6] * x0 - L[7] * x1) / L[8];
        B[3 * r] = x0; B[3 * r + 1] = x1; B[3 * r + 2] = x2;
    }
}

static int64_t col_find(const sym_t* Y, int64_t p, int64_t node) {
    int64_t lo = Y->cptr[p], hi = Y->cptr[p + 1] - 1;
    int64_t key = Y->pos[node];
    while (lo <= hi) {
        int64_t mid = (lo + hi) >> 1;
        int64_t pm = Y->pos[Y->crow[mid]];
        if (pm == key) return mid;
        if (pm < key) lo = mid + 1; else hi = mid - 1;
    }
    return -1;
}

/* Solve H x = rhs with the symbolic structure Y; H from S.  x, rhs: [n][3] */
static int chol_solve(const sym_t* Y, sys_t* S, const double* rhs, double* x) {
    int64_t n = Y->n, nnz = Y->cptr[n];
    double* Ld = (double*)malloc(sizeof(double) * 9 * (size_t)n);    /* diag per elimination step */
    double* Lo = (double*)calloc((size_t)(9 * (nnz ? nnz : 1)), sizeof(double));  /* L(row, col) */
    for (int64_t p = 0; p < n; ++p) {
        int64_t v = Y->perm[p];
        memcpy(Ld + 9 * p, S->diag + 9 * v, 9 * sizeof(double));
        for (int64_t q = Y->cptr[p]; q < Y->cptr[p + 1]; ++q) {
            int64_t u = Y->crow[q];
            int64_t lo = v < u ? v : u, hi = v < u ? u : v;
            int64_t sl = hslot(S, lo * n + hi, 0);
            if (sl < 0) continue;
            const double* B = S->blk + 9 * sl;    /* H(lo, hi) */
            double* D = Lo + 9 * q;               /* want H(u, v) */
            if (u == hi) { for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) D[3 * r + c] = B[3 * c + r]; }
            else memcpy(D, B, 9 * sizeof(double));
        }
    }
    int rc = 0;
    for (int64_t p = 0; p < n && rc == 0; ++p) {
        if (chol3(Ld + 9 * p)) { rc = -1; break; }
        const double* L = Ld + 9 * p;
        int64_t b0 = Y->cptr[p], b1 = Y->cptr[p + 1];
        for (int64_t q = b0; q < b1; ++q) rsolve_lt(L, Lo + 9 * q);
        /* Schur update of the later columns */
        for (int64_t qa = b0; qa < b1; ++qa) {
            int64_t a = Y->crow[qa];
            int64_t pa = Y->pos[a];
            const double* La = Lo + 9 * qa;
            for (int64_t qb = qa; qb < b1; ++qb) {
                int64_t b = Y->crow[qb];
                const double* Lb = Lo + 9 * qb;
                double M[9];
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c)
                        M[3 * r + c] = Lb[3 * r] * La[3 * c] + Lb[3 * r + 1] * La[3 * c + 1] + Lb[3 * r + 2] * La[3 * c + 2];
                double* T;
                if (qb == qa) T = Ld + 9 * pa;
                else {
                    int64_t s = col_find(Y, pa, b);
                    if (s < 0) { rc = -2; break; }
                    T = Lo + 9 * s;
                }
                for (int q = 0; q < 9; ++q) T[q] -= M[q];
            }
        }
    }
    if (rc == 0) {
        /* forward: L y = rhs (permuted) */
        double* y = (double*)malloc(sizeof(double) * 3 * (size_t)n);
        for (int64_t p = 0; p < n; ++p) memcpy(y + 3 * p, rhs + 3 * Y->perm[p], 3 * sizeof(double));
        for (int64_t p = 0; p < n; ++p) {
            const double* L = Ld + 9 * p;
            double* yp = y + 3 * p;
            yp[0] = yp[0] / L[0];
            yp[1] = (yp[1] - L[3] * yp[0]) / L[4];
            yp[2] = (yp[2] - L[6] * yp[0] - L[7] * yp[1]) / L[8];
            for (int64_t q = Y->cptr[p]; q < Y->cptr[p + 1]; ++q) {
                const double* B = Lo + 9 * q;
                double* yr = y + 3 * Y->pos[Y->crow[q]];
                for (int r = 0; r < 3; ++r) yr[r] -= B[3 * r] * yp[0] + B[3 * r + 1] * yp[1] + B[3 * r + 2] * yp[2];
            }
        }
        /* backward: L^T x = y */
        for (int64_t p = n - 1; p >= 0; --p) {
            double* yp = y + 3 * p;
            for (int64_t q = Y->cptr[p]; q < Y->cptr[p + 1]; ++q) {
                const double* B = Lo + 9 * q;
                const double* xr = y + 3 * Y->pos[Y->crow[q]];
                for (int c = 0; c < 3; ++c) yp[c] -= B[c] * xr[0] + B[3 + c] * xr[1] + B[6 + c] * xr[2];
            }
            const double* L = Ld + 9 * p;
            yp[2] = yp[2] / L[8];
            yp[1] = (yp[1] - L[7] * yp[2]) / L[4];
            yp[0] = (yp[0] - L[3] * yp[1] - L[6] * yp[2]) / L[0];
        }
        for (int64_t p = 0; p < n; ++p) memcpy(x + 3 * Y->perm[p], y + 3 * p, 3 * sizeof(double));
        free(y);
    }
    free(Ld);
    free(Lo);
    return rc;
}

/* Pose2 retract with the cheap ChartAtOrigin: X <- X * Pose2(dx, dy, dth). */
static void retract(double* X, const double* d) {
    double c = cos(X[2]), s = sin(X[2]);
    double cd = cos(d[2]), sd = sin(d[2]);
    double nx = X[0] + (c * d[0] - s * d[1]);
    double ny = X[1] + (s * d[0] + c * d[1]);
    double nc = c * cd - s * sd, nsn = s * cd + c * sd;
    X[0] = nx;
    X[1] = ny;
    X[2] = atan2(nsn, nc);
}

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

static int64_t count_pairs(const dpg_factor* f, int64_t nf) {
    int64_t c = 0;
    for (int64_t k = 0; k < nf; ++k) c += f[k].kind == DPG_FACTOR_BETWEEN;
    return c;
}

int oracle_gn_delta(const double* X, int64_t n, const dpg_factor* f, int64_t nf, double* delta,
                    double* error) {
    sys_t S;
    sym_t Y;
    sys_init(&S, n, count_pairs(f, nf));
    if (sym_analyze(&Y, n, f, nf)) { sys_free(&S); return -1; }
    double err = sys_assemble(&S, X, f, nf);
    double* rhs = (double*)malloc(sizeof(double) * 3 * (size_t)n);
    for (int64_t k = 0; k < 3 * n; ++k) rhs[k] = -S.g[k];
    int rc = chol_solve(&Y, &S, rhs, delta);
    if (error) *error = err;
    free(rhs);
    sym_free(&Y);
    sys_free(&S);
    return rc;
}

/* GTSAM NonlinearOptimizer::defaultOptimize + checkConvergence (use_error_criteria = 1), or the
 * batch-GN target: iterate until max|delta| < delta_tol. */
static int check_conv(const dpg_gn_params* gp, double cur, double nw) {
    if (nw <= 0.0) return 1;
    double abs_dec = cur - nw;
    double rel_dec = abs_dec / cur;
    return (gp->relative_error_tol != 0.0 && rel_dec <= gp->relative_error_tol) ||
           (abs_dec <= gp->absolute_error_tol);
}

int oracle_optimize_graph(double* X, int64_t n, const dpg_factor* f, int64_t nf,
                          const dpg_gn_params* gp, dpg_gn_stats* st) {
    double t0 = now_ms();
    sys_t S;
    sym_t Y;
    sys_init(&S, n, count_pairs(f, nf));
    if (sym_analyze(&Y, n, f, nf)) { sys_free(&S); return -1; }
    double* rhs = (double*)malloc(sizeof(double) * 3 * (size_t)n);
    double* d = (double*)malloc(sizeof(double) * 3 * (size_t)n);
    double t_iter0 = now_ms();
    double cur = sys_assemble(&S, X, f, nf);
    dpg_gn_stats local;
    memset(&local, 0, sizeof(local));
    local.initial_error = cur;
    int rc = 0;
    int it = 0;
    double dinf = 0.0;
    double nw = cur;
    if (!(cur <= 0.0) && gp->max_iterations > 0) {
        for (;;) {
            for (int64_t k = 0; k < 3 * n; ++k) rhs[k] = -S.g[k];
            if (chol_solve(&Y, &S, rhs, d)) { rc = -2; break; }
            dinf = 0.0;
            for (int64_t k = 0; k < 3 * n; ++k) if (fabs(d[k]) > dinf) dinf = fabs(d[k]);
            for (int64_t v = 0; v < n; ++v) retract(X + 3 * v, d + 3 * v);
            ++it;
            nw = sys_assemble(&S, X, f, nf);
            if (it >= gp->max_iterations) break;
            if (gp->use_error_criteria) {
                if (check_conv(gp, cur, nw) || !isfinite(cur)) break;
            } else if (dinf < gp->delta_tol) break;
            cur = nw;
        }
    }
    double t1 = now_ms();
    local.iterations = it;
    local.final_error = nw;
    local.last_delta_inf = dinf;
    local.ms_total = t1 - t0;
    local.ms_per_iteration = it ? (t1 - t_iter0) / it : 0.0;
    if (st) *st = local;
    free(rhs);
    free(d);
    sym_free(&Y);
    sys_free(&S);
    return rc;
}

/* Symbolic statistics of the block Cholesky (min-degree): out = {nnz blocks of L (off-diagonal),
 * max column count, flop estimate, elimination-tree height}. Diagnostics for solver design. */
int oracle_symbolic_stats(int64_t n, const dpg_factor* f, int64_t nf, double out[4]) {
    sym_t Y;
    if (sym_analyze(&Y, n, f, nf)) return -1;
    double flops = 0.0;
    int64_t mx = 0;
    int64_t* height = (int64_t*)calloc((size_t)n, sizeof(int64_t));
    int64_t hmax = 0;
    for (int64_t p = 0; p < n; ++p) {
        int64_t c = Y.cptr[p + 1] - Y.cptr[p];
        if (c > mx) mx = c;
        flops += 27.0 * (double)(c + 1) * (double)(c + 1);
        if (c > 0) {   /* parent = first row of the column */
            int64_t par = Y.pos[Y.crow[Y.cptr[p]]];
            if (height[p] + 1 > height[par]) height[par] = height[p] + 1;
        }
        if (height[p] > hmax) hmax = height[p];
    }
    out[0] = (double)Y.cptr[n];
    out[1] = (double)mx;
    out[2] = flops;
    out[3] = (double)hmax;
    free(height);
    sym_free(&Y);
    return 0;
}

/* The commented-out 6x6 sandwich of calculate_ICP_COV (cov_func_point_to_point.h:553-566),
 * restated literally: per index pair the full 6x6 d2J_dX2 block and the full 6x6 d2J_dZdX block
 * (rows x y z a b c, columns pix piy piz qix qiy qiz -- the reference's layouts, :271-279 and
 * :520-528), the Hessian summed over s < min(nd, nm), B_k B_k^T summed over k < min(nd, nm, 200)
 * (:307), cov_z = 0.01 I, inverse by LU with partial pivoting, cov6 = inv(H) M inv(H) * 0.01.
 * Entries at b = c = z = 0 (T20 = T21 = 0, T22 = 1, piz = qiz = 0); yaw = atan2f(T10, T00). */
static void cov6_point(double ca, double sa, double x, double y, double px, double py, double qx, double qy,
                       double H[36], double B[36]) {
    const double ux = ca * px - sa * py, uy = sa * px + ca * py;
    const double dx = x - qx, dy = y - qy;
    const double w = dx * ca + dy * sa, v = dx * sa - dy * ca;
    for (int k = 0; k < 36; ++k) { H[k] = 0.0; B[k] = 0.0; }
    /* d2J_dX2 (symmetric) */
    H[0] = 2.0; H[7] = 2.0; H[14] = 2.0;
    H[3] = H[18] = -2.0 * uy;                 /* x a */
    H[9] = H[19] = 2.0 * ux;                  /* y a */
    H[16] = H[26] = -2.0 * px;                /* z b */
    H[17] = H[32] = 2.0 * py;                 /* z c */
    H[21] = -2.0 * (ux * dx + uy * dy);       /* a a */
    H[28] = -2.0 * px * w;                    /* b b */
    H[29] = H[34] = 2.0 * py * w;             /* b c */
    H[35] = 2.0 * py * v;                     /* c c */
    /* d2J_dZdX: row = X (x y z a b c), column = Z (pix piy piz qix qiy qiz) */
    B[0] = 2.0 * ca;  B[1] = -2.0 * sa; B[3] = -2.0;
    B[6] = 2.0 * sa;  B[7] = 2.0 * ca;  B[10] = -2.0;
    B[14] = 2.0;      B[17] = -2.0;
    B[18] = -2.0 * v; B[19] = -2.0 * w; B[21] = 2.0 * uy; B[22] = -2.0 * ux;
    B[26] = 2.0 * w;  B[29] = 2.0 * px;
    B[32] = 2.0 * v;  B[35] = -2.0 * py;
}

static int inv6(const double* A, double* Ai) {
    double L[36];
    int piv[6];
    for (int k = 0; k < 36; ++k) L[k] = A[k];
    for (int i = 0; i < 6; ++i) piv[i] = i;
    for (int c = 0; c < 6; ++c) {   /* LU with partial pivoting */
        int p = c;
        for (int r = c + 1; r < 6; ++r)
            if (fabs(L[6 * r + c]) > fabs(L[6 * p + c])) p = r;
        if (!(fabs(L[6 * p + c]) > 0.0)) return -1;
        if (p != c) {
            for (int k = 0; k < 6; ++k) { double t = L[6 * p + k]; L[6 * p + k] = L[6 * c + k]; L[6 * c + k] = t; }
            int t = piv[p]; piv[p] = piv[c]; piv[c] = t;
        }
        for (int r = c + 1; r < 6; ++r) {
            L[6 * r + c] /= L[6 * c + c];
            for (int k = c + 1; k < 6; ++k) L[6 * r + k] -= L[6 * r + c] * L[6 * c + k];
        }
    }
    for (int j = 0; j < 6; ++j) {   /* column j of the inverse: solve L U x = P e_j */
        double z[6];
        for (int i = 0; i < 6; ++i) {
            double s = piv[i] == j ? 1.0 : 0.0;
            for (int k = 0; k < i; ++k) s -= L[6 * i + k] * z[k];
            z[i] = s;
        }
        for (int i = 5; i >= 0; --i) {
            double s = z[i];
            for (int k = i + 1; k < 6; ++k) s -= L[6 * i + k] * z[k];
            z[i] = s / L[6 * i + i];
        }
        for (int i = 0; i < 6; ++i) Ai[6 * i + j] = z[i];
    }
    return 0;
}

int oracle_icp_cov_sandwich(const float* data, int64_t nd, const float* model, int64_t nm, const float T6[6],
                            double cov6[36], double cov3[9]) {
    if (nd < 1 || nm < 1) return -1;
    const double a = (double)atan2f(T6[3], T6[0]);   /* cov :31 yaw = atan2f(T10, T00) */
    const double ca = cos(a), sa = sin(a), x = T6[2], y = T6[5];
    const int64_t nh = nd < nm ? nd : nm, nb = nh < 200 ? nh : 200;
    double H[36] = {0}, M[36] = {0}, Hs[36], Bk[36];
    for (int64_t s = 0; s < nh; ++s) {
        cov6_point(ca, sa, x, y, data[2 * s], data[2 * s + 1], model[2 * s], model[2 * s + 1], Hs, Bk);
        for (int k = 0; k < 36; ++k) H[k] += Hs[k];
        if (s < nb)
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j < 6; ++j) {
                    double acc = 0.0;
                    for (int k = 0; k < 6; ++k) acc += Bk[6 * i + k] * Bk[6 * j + k];
                    M[6 * i + j] += acc;
                }
    }
    double Hi[36], T1[36];
    if (inv6(H, Hi)) return -2;
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double acc = 0.0;
            for (int k = 0; k < 6; ++k) acc += Hi[6 * i + k] * M[6 * k + j];
            T1[6 * i + j] = acc;
        }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double acc = 0.0;
            for (int k = 0; k < 6; ++k) acc += T1[6 * i + k] * Hi[6 * k + j];
            cov6[6 * i + j] = 0.01 * acc;
        }
    static const int ix[3] = {0, 1, 3};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) cov3[3 * i + j] = cov6[6 * ix[i] + ix[j]];
    return 0;
}
