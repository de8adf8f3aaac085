/*
 * dpg_slam_adapter.hpp -- header-only C++ adapter that gives the MI355X C ABI (dpg_slam_c.h,
 * dpg_icp_cov.h) the reference's own entry-point signatures, so the bodies of DpgSLAM's member
 * functions become one-line forwards (INTEGRATION.md sections 2-6 show each replacement body).
 *
 * Generic over the reference's types -- nothing here includes PCL, Eigen or GTSAM:
 *   CloudPtr   pcl::PointCloud<pcl::PointXYZ>::Ptr (->size(), ->points[i].x / .y)
 *   Matrix4f   Eigen::Matrix4f (operator()(r, c))
 *   MatrixXd   Eigen::MatrixXd (resize(r, c), operator()(r, c))
 *   Vector2f   Eigen::Vector2f (constructible from (x, y), .x(), .y())
 *   Node       dpg_slam::DpgNode (getCachedPointCloudFromNode(), getEstimatedPosition() ->
 *              std::pair<Vector2f, float>, setPosition(Vector2f, float), getPassNumber(),
 *              setInactive())
 *   PGParams   dpg_slam::PoseGraphParameters (the icp_* / laser_* / maximum_node_dist_* members,
 *              parameters.h:105-140)
 * Errors: every C call's status is checked; a failure throws dpg_adapter::Error carrying
 * dpg_last_error().
 */
#ifndef DPG_SLAM_ADAPTER_HPP
#define DPG_SLAM_ADAPTER_HPP

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <array>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "dpg_icp_cov.h"
#include "dpg_slam_c.h"

namespace dpg_adapter {

struct Error : std::runtime_error {
    explicit Error(const std::string& s) : std::runtime_error(s) {}
};

inline void check(int rc, const char* what) {
    if (rc != DPG_OK) throw Error(std::string(what) + ": " + (dpg_last_error() ? dpg_last_error() : "?"));
}

/* A GPU context, owned: one device (the constructor), or one of the multi-device forms -- every
 * adapter call below takes any of them (the batched paths shard, dpg_slam_c.h):
 *   Context::multi(n)              one process over GPUs 0 .. n-1 (the ROS node);
 *   Context::rank(dev, id, r, w)   one process per GPU, rank r of w (id from nccl_unique_id() on rank 0);
 *   Context::virtual_devices(k)    k virtual devices on one GPU (tests of the sharded paths). */
class Context {
  public:
    explicit Context(int device = 0) : c_(dpg_ctx_create(device)) { ok("dpg_ctx_create"); }
    static Context multi(int n_gpus, const int32_t* devices = nullptr) {
        return Context(dpg_ctx_create_multi(n_gpus, devices), "dpg_ctx_create_multi");
    }
    static Context rank(int device, const std::array<unsigned char, DPG_NCCL_ID_BYTES>& id, int rank, int world) {
        return Context(dpg_ctx_create_rank(device, id.data(), rank, world), "dpg_ctx_create_rank");
    }
    static Context virtual_devices(int k, int device = 0) {
        return Context(dpg_ctx_create_virtual(k, device), "dpg_ctx_create_virtual");
    }
    static std::array<unsigned char, DPG_NCCL_ID_BYTES> nccl_unique_id() {
        std::array<unsigned char, DPG_NCCL_ID_BYTES> id{};
        check(dpg_nccl_unique_id(id.data()), "dpg_nccl_unique_id");
        return id;
    }
    ~Context() { if (c_) dpg_ctx_destroy(c_); }
    Context(Context&& o) noexcept : c_(o.c_) { o.c_ = nullptr; }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    dpg_ctx* get() const { return c_; }
    int ranks() const { return dpg_ctx_num_ranks(c_); }
  private:
    Context(dpg_ctx* c, const char* what) : c_(c) { ok(what); }
    void ok(const char* what) {
        if (!c_) throw Error(std::string(what) + ": " + (dpg_last_error() ? dpg_last_error() : "?"));
    }
    dpg_ctx* c_;
};

/* The x, y of a cloud's points, interleaved (z is 0 in this 2D pipeline). */
template <class CloudPtr>
std::vector<float> xy_of(const CloudPtr& c) {
    std::vector<float> v(2 * c->size());
    for (size_t i = 0; i < c->size(); ++i) {
        v[2 * i] = c->points[i].x;
        v[2 * i + 1] = c->points[i].y;
    }
    return v;
}

template <class Node>
void pose_of(const Node& n, float out[3]) {
    const auto e = n.getEstimatedPosition();
    out[0] = e.first.x();
    out[1] = e.first.y();
    out[2] = e.second;
}

/* PoseGraphParameters -> the ICP parameter block (runIcp, dpg_slam.cc:399-412). */
template <class PGParams>
dpg_icp_params icp_params_from(const PGParams& p) {
    dpg_icp_params q;
    dpg_icp_params_default(&q);
    q.icp_maximum_iterations = p.icp_maximum_iterations_;
    q.icp_maximum_transformation_epsilon = p.icp_maximum_transformation_epsilon_;
    q.icp_max_correspondence_distance = p.icp_max_correspondence_distance_;
    q.icp_use_reciprocal_correspondences = p.icp_use_reciprocal_correspondences_ ? 1 : 0;
    q.downsample_icp_points_ratio = p.downsample_icp_points_ratio_;
    q.laser_x_variance = p.laser_x_variance_;
    q.laser_y_variance = p.laser_y_variance_;
    q.laser_theta_variance = p.laser_theta_variance_;
    return q;
}

/* calculate_ICP_COV (src/icp_cov/cov_func_point_to_point.h:24), same arguments.  ICP_COV
 * receives the constant diag(vx, vy, vth) the reference returns (:572-575); hess_block (nullable,
 * double[9]) the [x, y, yaw] block of the d2J/dX2 sum computed on the GPU. */
template <class CloudPtr, class Matrix4f, class MatrixXd>
void calculate_ICP_COV(CloudPtr data_pi, CloudPtr model_qi, Matrix4f& transform, MatrixXd& ICP_COV,
                       float laser_x_variance, float laser_y_variance, float laser_theta_variance,
                       dpg_ctx* ctx = nullptr, double* hess_block = nullptr) {
    const std::vector<float> d = xy_of(data_pi), m = xy_of(model_qi);
    float T[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) T[4 * r + c] = transform(r, c);   // the ABI takes row-major
    double cov[9];
    check(icp_cov_calculate(ctx, d.data(), (int64_t)(d.size() / 2), m.data(), (int64_t)(m.size() / 2), T,
                            laser_x_variance, laser_y_variance, laser_theta_variance, cov, hess_block),
          "icp_cov_calculate");
    ICP_COV.resize(3, 3);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) ICP_COV(r, c) = cov[3 * r + c];
}

/* DpgSLAM::runIcp (dpg_slam.h:630, dpg_slam.cc:362-446): node_2's cloud aligned to node_1's from
 * the estimated poses; icp_results = ((x, y), theta) of node_2 in node_1's frame and ICP_COV.
 * Returns hasConverged() (the reference's return value). */
template <class Node, class PGParams, class Vector2f, class MatrixXd>
bool runIcp(dpg_ctx* ctx, const PGParams& pgp, Node& node_1, Node& node_2,
            std::pair<std::pair<Vector2f, float>, MatrixXd>& icp_results) {
    const std::vector<float> src = xy_of(node_2.getCachedPointCloudFromNode());   // ICP source
    const std::vector<float> tgt = xy_of(node_1.getCachedPointCloudFromNode());   // ICP target
    float p2[3], p1[3];
    pose_of(node_2, p2);
    pose_of(node_1, p1);
    const dpg_icp_params prm = icp_params_from(pgp);
    dpg_icp_result r;
    double cov[9];
    check(dpg_run_icp(ctx, src.data(), (int64_t)(src.size() / 2), tgt.data(), (int64_t)(tgt.size() / 2), p2, p1, &prm,
                      &r, cov, nullptr),
          "dpg_run_icp");
    MatrixXd C;
    C.resize(3, 3);
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) C(a, b) = cov[3 * a + b];
    icp_results = std::make_pair(std::make_pair(Vector2f(r.z[0], r.z[1]), r.z[2]), C);
    return r.converged != 0 && r.status == DPG_ICP_OK;
}

/* The factor mirror of graph_: addObservationConstraint (dpg_slam.cc:331-338) and the prior /
 * odometry sites append here. */
inline dpg_factor prior_factor(int32_t key, double x, double y, double th, const double sigmas[3]) {
    dpg_factor f{};
    f.kind = DPG_FACTOR_PRIOR;
    f.i = key;
    f.z[0] = x; f.z[1] = y; f.z[2] = th;
    for (int q = 0; q < 3; ++q) f.info[q] = 1.0 / (sigmas[q] * sigmas[q]);
    return f;
}
inline dpg_factor between_factor(int32_t i, int32_t j, double x, double y, double th, const double info[3]) {
    dpg_factor f{};
    f.kind = DPG_FACTOR_BETWEEN;
    f.i = i;
    f.j = j;
    f.z[0] = x; f.z[1] = y; f.z[2] = th;
    for (int q = 0; q < 3; ++q) f.info[q] = info[q];
    return f;
}

/* DpgSLAM::optimizeGraph (dpg_slam.h:464, dpg_slam.cc:316-329), batch form: Gauss-Newton to
 * convergence on the accumulated factors from the nodes' estimates, written back with
 * setPosition. */
template <class NodeVec>
dpg_gn_stats optimizeGraph(dpg_ctx* ctx, NodeVec& nodes, const std::vector<dpg_factor>& factors,
                           const dpg_gn_params* params = nullptr) {
    using Vec = decltype(nodes[0].getEstimatedPosition().first);
    std::vector<double> X(3 * nodes.size());
    for (size_t k = 0; k < nodes.size(); ++k) {
        float p[3];
        pose_of(nodes[k], p);
        X[3 * k] = p[0]; X[3 * k + 1] = p[1]; X[3 * k + 2] = p[2];
    }
    dpg_gn_params gp;
    if (params) gp = *params;
    else dpg_gn_params_default(&gp);
    dpg_gn_stats st;
    check(dpg_optimize_graph(ctx, X.data(), (int64_t)nodes.size(), factors.data(), (int64_t)factors.size(), &gp, &st),
          "dpg_optimize_graph");
    for (size_t k = 0; k < nodes.size(); ++k)
        nodes[k].setPosition(Vec((float)X[3 * k], (float)X[3 * k + 1]), (float)X[3 * k + 2]);
    return st;
}

/* The incremental form of optimizeGraph (one isam_->update per node, dpg_slam.cc:255-329): the
 * device-resident graph of dpg_inc; add_node runs updatePoseGraphObsConstraints' alignments of
 * the new node as one batch and the update. */
class IncGraph {
  public:
    IncGraph(dpg_ctx* ctx, const dpg_inc_params* p = nullptr) : g_(dpg_inc_create(ctx, p)) {
        if (!g_) throw Error(std::string("dpg_inc_create: ") + (dpg_last_error() ? dpg_last_error() : "?"));
    }
    ~IncGraph() { if (g_) dpg_inc_destroy(g_); }
    IncGraph(const IncGraph&) = delete;
    IncGraph& operator=(const IncGraph&) = delete;
    dpg_inc* get() const { return g_; }
    int64_t size() const { return dpg_inc_num_nodes(g_); }
    /* the new node's cloud, the pass of every node (the new one last), its initial pose, the
       prior / odometry factor(s) that come with it */
    template <class CloudPtr, class PGParams>
    dpg_add_node_stats add_node(const CloudPtr& cloud, const std::vector<int32_t>& passes, const float init_pose[3],
                                const std::vector<dpg_factor>& extra, const PGParams& pgp, bool non_successive = true) {
        const std::vector<float> xy = xy_of(cloud);
        const dpg_icp_params ip = icp_params_from(pgp);
        dpg_reopt_params rp;
        dpg_reopt_params_default(&rp);
        rp.max_node_dist_within_pass = pgp.maximum_node_dist_within_pass_scan_comparison_;
        rp.max_node_dist_across_passes = pgp.maximum_node_dist_across_passes_scan_comparison_;
        dpg_add_node_stats st;
        check(dpg_add_node(g_, xy.data(), (int64_t)(xy.size() / 2), passes.data(), init_pose, extra.data(),
                           (int64_t)extra.size(), &ip, &rp, non_successive ? 1 : 0, &st),
              "dpg_add_node");
        return st;
    }
    /* DpgSLAM::reoptimize (dpg_slam.cc:35-120) on this graph: the sweep over the clouds already in
       the context's store (one per add_node), then the graph rebuilt from the sweep's factors --
       the reference's new ISAM2 + graph_ -- so later add_node calls build on it; the nodes receive
       the new estimates.  odom_only: odom_only_estimates_ (std::pair<Vector2f, float> per node). */
    template <class NodeVec, class OdomVec, class PGParams>
    dpg_reopt_stats reoptimize(NodeVec& nodes, const OdomVec& odom_only, const PGParams& pgp) {
        const size_t V = nodes.size();
        std::vector<float> est(3 * V), odom(3 * V);
        std::vector<int32_t> pass(V);
        for (size_t i = 0; i < V; ++i) {
            pose_of(nodes[i], &est[3 * i]);
            odom[3 * i] = odom_only[i].first.x();
            odom[3 * i + 1] = odom_only[i].first.y();
            odom[3 * i + 2] = odom_only[i].second;
            pass[i] = (int32_t)nodes[i].getPassNumber();
        }
        const dpg_icp_params ip = icp_params_from(pgp);
        dpg_reopt_params rp;
        dpg_reopt_params_default(&rp);
        rp.max_node_dist_within_pass = pgp.maximum_node_dist_within_pass_scan_comparison_;
        rp.max_node_dist_across_passes = pgp.maximum_node_dist_across_passes_scan_comparison_;
        rp.odometry_constraints = pgp.odometry_constraints_ ? 1 : 0;
        std::vector<double> X(3 * V);
        dpg_reopt_stats st;
        check(dpg_reoptimize_inc(g_, (int64_t)V, pass.data(), est.data(), odom.data(), &ip, &rp, X.data(), &st),
              "dpg_reoptimize_inc");
        write_back(nodes);
        return st;
    }
    /* graph checkpoint (dpg_inc_save / dpg_inc_load): the graph and its context's scans in one
       file; a graph loaded on ctx continues the saved run */
    void save(const char* path) const { check(dpg_inc_save(g_, path), "dpg_inc_save"); }
    static IncGraph load(dpg_ctx* ctx, const char* path) {
        dpg_inc* g = dpg_inc_load(ctx, path);
        if (!g) throw Error(std::string("dpg_inc_load: ") + (dpg_last_error() ? dpg_last_error() : "?"));
        return IncGraph(g);
    }
    IncGraph(IncGraph&& o) noexcept : g_(o.g_) { o.g_ = nullptr; }
    /* the current estimates -> the nodes (setPosition) */
    template <class NodeVec>
    void write_back(NodeVec& nodes) const {
        using Vec = decltype(nodes[0].getEstimatedPosition().first);
        std::vector<double> X(3 * nodes.size());
        check(dpg_inc_get_poses(g_, X.data(), (int64_t)nodes.size()), "dpg_inc_get_poses");
        for (size_t k = 0; k < nodes.size(); ++k)
            nodes[k].setPosition(Vec((float)X[3 * k], (float)X[3 * k + 1]), (float)X[3 * k + 2]);
    }
  private:
    explicit IncGraph(dpg_inc* g) : g_(g) {}
    dpg_inc* g_;
};

/* DpgSLAM::reoptimize (dpg_slam.cc:35-120) in one call: every node's cloud uploaded, the GPU
 * candidate search, one batched ICP of the successive + loop-closure pairs, the factors in the
 * reference's order, Gauss-Newton; the nodes receive the optimised poses.  odom_only: the
 * odom_only_estimates_ (std::pair<Vector2f, float> per node). */
template <class NodeVec, class OdomVec, class PGParams>
dpg_reopt_stats reoptimize(dpg_ctx* ctx, NodeVec& nodes, const OdomVec& odom_only, const PGParams& pgp,
                           const dpg_gn_params* gn = nullptr) {
    using Vec = decltype(nodes[0].getEstimatedPosition().first);
    const size_t V = nodes.size();
    std::vector<float> pts, est(3 * V), odom(3 * V);
    std::vector<int64_t> off(V + 1, 0);
    std::vector<int32_t> pass(V);
    for (size_t i = 0; i < V; ++i) {
        const std::vector<float> c = xy_of(nodes[i].getCachedPointCloudFromNode());   // base_link, MAX_RANGE dropped
        pts.insert(pts.end(), c.begin(), c.end());
        off[i + 1] = (int64_t)(pts.size() / 2);
        pose_of(nodes[i], &est[3 * i]);
        odom[3 * i] = odom_only[i].first.x();
        odom[3 * i + 1] = odom_only[i].first.y();
        odom[3 * i + 2] = odom_only[i].second;
        pass[i] = (int32_t)nodes[i].getPassNumber();
    }
    check(dpg_scans_upload(ctx, pts.data(), off.data(), (int64_t)V, pgp.downsample_icp_points_ratio_),
          "dpg_scans_upload");
    const dpg_icp_params ip = icp_params_from(pgp);
    dpg_reopt_params rp;
    dpg_reopt_params_default(&rp);
    rp.max_node_dist_within_pass = pgp.maximum_node_dist_within_pass_scan_comparison_;
    rp.max_node_dist_across_passes = pgp.maximum_node_dist_across_passes_scan_comparison_;
    rp.odometry_constraints = pgp.odometry_constraints_ ? 1 : 0;
    std::vector<double> X(3 * V);
    dpg_reopt_stats st;
    check(dpg_reoptimize(ctx, (int64_t)V, pass.data(), est.data(), odom.data(), &ip, gn, &rp, X.data(), &st),
          "dpg_reoptimize");
    for (size_t i = 0; i < V; ++i)
        nodes[i].setPosition(Vec((float)X[3 * i], (float)X[3 * i + 1]), (float)X[3 * i + 2]);
    return st;
}

/* The DPG node state (labels, sectors, activity) on the GPU, and executeDPG over it
 * (dpg_slam.cc:865-886).  Scans are added as createNode sees them (ranges, angle_min/max,
 * range_max, dpg_slam.cc:488-513). */
class DpgStore {
  public:
    DpgStore(dpg_ctx* ctx, const dpg_change_params* p = nullptr) : ctx_(ctx), d_(nullptr), p_() {
        if (p) p_ = *p;
        else dpg_change_params_default(&p_);
    }
    ~DpgStore() { if (d_) dpg_dpg_destroy(d_); }
    DpgStore(const DpgStore&) = delete;
    DpgStore& operator=(const DpgStore&) = delete;
    dpg_dpg* get() const { return d_; }
    void add_scan(const std::vector<float>& ranges, float angle_min, float angle_max, float range_max) {
        const int64_t off[2] = {0, (int64_t)ranges.size()};
        const float geom[3] = {angle_min, angle_max, range_max};
        if (!d_) {
            d_ = dpg_dpg_create(ctx_, 1, off, ranges.data(), geom, &p_);
            if (!d_) throw Error(std::string("dpg_dpg_create: ") + (dpg_last_error() ? dpg_last_error() : "?"));
        } else {
            check(dpg_dpg_append(d_, 1, off, ranges.data(), geom), "dpg_dpg_append");
        }
    }
    /* executeDPG after the last node was added; nodes deactivated on the GPU are mirrored with
       setInactive(); the four map lists (Vector2f-like points) are refreshed */
    template <class NodeVec, class PointVec>
    dpg_change_stats executeDPG(NodeVec& nodes, size_t current_pass_len, PointVec& active_static,
                                PointVec& active_added, PointVec& dynamic_removed, PointVec& dynamic_added) {
        return run(nodes, current_pass_len, static_cast<const NodeVec*>(nullptr), active_static, active_added,
                   dynamic_removed, dynamic_added);
    }
    /* the reference's placement: the pose chain at the poses of the current_pass_nodes_ copies
       (dpg_slam.cc:195,307,598), dpg_nodes_ (nodes) everywhere else (dpg_execute_dpg_chain) */
    template <class NodeVec, class PointVec>
    dpg_change_stats executeDPG(NodeVec& nodes, const NodeVec& current_pass_nodes, PointVec& active_static,
                                PointVec& active_added, PointVec& dynamic_removed, PointVec& dynamic_added) {
        return run(nodes, current_pass_nodes.size(), &current_pass_nodes, active_static, active_added,
                   dynamic_removed, dynamic_added);
    }
  private:
    template <class NodeVec, class PointVec>
    dpg_change_stats run(NodeVec& nodes, size_t current_pass_len, const NodeVec* pass_nodes, PointVec& active_static,
                         PointVec& active_added, PointVec& dynamic_removed, PointVec& dynamic_added) {
        using P = typename PointVec::value_type;
        const size_t V = nodes.size();
        std::vector<float> est(3 * V);
        for (size_t i = 0; i < V; ++i) pose_of(nodes[i], &est[3 * i]);
        dpg_change_stats st;
        if (pass_nodes) {
            const size_t n = std::min<size_t>(current_pass_len, (size_t)p_.current_pose_chain_len);
            std::vector<float> chain(3 * n + 3);
            for (size_t k = 0; k < n; ++k) pose_of((*pass_nodes)[current_pass_len - n + k], &chain[3 * k]);
            check(dpg_execute_dpg_chain(d_, (int64_t)V, (int64_t)current_pass_len, est.data(), chain.data(), &st),
                  "dpg_execute_dpg_chain");
        } else {
            check(dpg_execute_dpg(d_, (int64_t)V, (int64_t)current_pass_len, est.data(), &st), "dpg_execute_dpg");
        }
        std::vector<uint8_t> active(V);
        check(dpg_dpg_fetch(d_, nullptr, nullptr, active.data()), "dpg_dpg_fetch");
        for (size_t i = 0; i < V; ++i)
            if (!active[i]) nodes[i].setInactive();
        int64_t cnt[4];
        const int64_t n = dpg_active_dynamic_points(d_, (int64_t)V, est.data(), nullptr, 0, cnt);
        if (n < 0) check((int)n, "dpg_active_dynamic_points");
        std::vector<float> pts(2 * (size_t)n + 2);
        check(dpg_active_dynamic_points(d_, (int64_t)V, est.data(), pts.data(), n, cnt) < 0 ? DPG_ERR_HIP : DPG_OK,
              "dpg_active_dynamic_points");
        PointVec* lists[4] = {&active_static, &active_added, &dynamic_removed, &dynamic_added};
        size_t k = 0;
        for (int l = 0; l < 4; ++l) {
            lists[l]->clear();
            for (int64_t q = 0; q < cnt[l]; ++q, ++k) lists[l]->push_back(P(pts[2 * k], pts[2 * k + 1]));
        }
        return st;
    }
    dpg_ctx* ctx_;
    dpg_dpg* d_;
    dpg_change_params p_;
};

}  // namespace dpg_adapter

#endif /* DPG_SLAM_ADAPTER_HPP */
