/*
 * dpg_icp_cov.h -- C ABI replacement for src/icp_cov/cov_func_point_to_point.h:24
 *
 *   void calculate_ICP_COV(pcl::PointCloud<pcl::PointXYZ>::Ptr data_pi,
 *                          pcl::PointCloud<pcl::PointXYZ>::Ptr model_qi,
 *                          Eigen::Matrix4f& transform, Eigen::MatrixXd& ICP_COV,
 *                          float laser_x_variance, float laser_y_variance,
 *                          float laser_theta_variance);
 *
 * The reference computes the point-to-point Hessian d2J_dX2 (cov :45-283) and d2J_dZdX
 * (:311-530), then discards both and returns the constant diag(var_x, var_y, var_theta)
 * (:572-575).  This entry point returns exactly that constant in cov_out (3x3 row-major,
 * each entry the float variance widened to double), and -- when hess_block_out is not NULL --
 * the [x, y, yaw] block (indices 0,1,3 of the commented selection at :564-566) of d2J_dX2,
 * computed on the GPU (HIP, gfx950) over index-paired points s < min(n_data, n_model)
 * (the reference reads model_qi out of bounds when it is shorter).
 *
 * data_xy / model_xy: interleaved x,y floats (z == 0, as the reference assumes at :23).
 * transform: 4x4 row-major float (T[4*r + c]); an Eigen::Matrix4f adapter must transpose.
 * ctx: NULL uses a lazily created context on HIP device 0.
 */
#ifndef DPG_ICP_COV_H
#define DPG_ICP_COV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

struct dpg_ctx;

int icp_cov_calculate(struct dpg_ctx* ctx, const float* data_xy, int64_t n_data,
                      const float* model_xy, int64_t n_model, const float transform[16],
                      float laser_x_variance, float laser_y_variance, float laser_theta_variance,
                      double cov_out[9], double hess_block_out[9]);

/* The 6x6 ICP covariance the reference computes and then discards (cov_func_point_to_point.h:
 * 553-566, commented out there; optional here, it is not what the graph uses): d2J_dX2 summed
 * over every index pair s < min(n_data, n_model) (:45-283, SURVEY Q3 for the bound), d2J_dZdX over
 * the first min(n_data, n_model, 200) pairs (:307-528), cov_z = 0.01 I (:553-554), and
 *   cov6 = inv(d2J_dX2) d2J_dZdX cov_z d2J_dZdX^T inv(d2J_dX2)      (:560)
 * in [x, y, z, yaw, pitch, roll] order (6x6 row-major), cov3 its [x, y, yaw] block (rows / columns
 * 0, 1, 3, :563-566; 3x3 row-major; either output may be NULL).  Evaluated at the transform's
 * planar angles (roll = pitch = 0, yaw = atan2f(T10, T00), z = T23 = 0): the sums on the GPU, the
 * 6x6 inverse and products on the host in fp64.  DPG_ERR_NUMERIC when d2J_dX2 is singular;
 * DPG_ERR_ARG when T is not planar (T02, T12, T20, T21, T23 != 0 or T22 != 1: the closed forms
 * hold only at z = pitch = roll = 0, where every ICP result of this library lies). */
int icp_cov_sandwich(struct dpg_ctx* ctx, const float* data_xy, int64_t n_data, const float* model_xy, int64_t n_model,
                     const float transform[16], double cov6_out[36], double cov3_out[9]);

#ifdef __cplusplus
}
#endif
#endif /* DPG_ICP_COV_H */
