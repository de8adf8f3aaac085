// adapter_check.cpp -- exercises include/dpg_slam_adapter.hpp with stand-ins for the reference's
// types (PCL cloud, Eigen matrices / vector, DpgNode, PoseGraphParameters): compiled and linked
// against lib/libdpg.so by the CPU suite (tests/test_adapter.py), run on the GPU by the gpu suite.
// Each adapter call is checked against the direct C-ABI call on the same inputs (bit for bit).
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <memory>
#include <vector>

#include "../include/dpg_slam_adapter.hpp"

namespace {

struct PointXYZ { float x, y, z; };
struct Cloud {
    std::vector<PointXYZ> points;
    size_t size() const { return points.size(); }
};
using CloudPtr = std::shared_ptr<Cloud>;
struct Vector2f {
    float v[2];
    Vector2f(float a = 0.f, float b = 0.f) : v{a, b} {}
    float x() const { return v[0]; }
    float y() const { return v[1]; }
};
struct Matrix4f {
    float m[16];
    float& operator()(int r, int c) { return m[4 * r + c]; }
};
struct MatrixXd {
    std::vector<double> m;
    int c = 0;
    void resize(int r, int cc) { m.assign((size_t)(r * cc), 0.0); c = cc; }
    double& operator()(int r, int cc) { return m[(size_t)(r * c + cc)]; }
};
struct Node {
    CloudPtr cloud;
    Vector2f loc;
    float th = 0.f;
    uint32_t pass = 0;
    bool active = true;
    CloudPtr getCachedPointCloudFromNode() const { return cloud; }
    std::pair<Vector2f, float> getEstimatedPosition() const { return {loc, th}; }
    void setPosition(const Vector2f& l, const float& t) { loc = l; th = t; }
    uint32_t getPassNumber() const { return pass; }
    void setInactive() { active = false; }
};
struct PGParams {   // parameters.h defaults
    int icp_maximum_iterations_ = 500;
    double icp_maximum_transformation_epsilon_ = 5e-9;
    double icp_max_correspondence_distance_ = 0.6;
    bool icp_use_reciprocal_correspondences_ = true;
    int downsample_icp_points_ratio_ = 5;
    float laser_x_variance_ = 0.5f, laser_y_variance_ = 0.5f, laser_theta_variance_ = 0.3f;
    float maximum_node_dist_within_pass_scan_comparison_ = 5.f, maximum_node_dist_across_passes_scan_comparison_ = 2.f;
    bool odometry_constraints_ = true;
};

// a 360-beam scan of a 10 x 6 m room from (x, y, th) (laser at the base_link origin here)
std::vector<float> room_scan(double x, double y, double th, int n) {
    std::vector<float> r((size_t)n);
    for (int b = 0; b < n; ++b) {
        const double a = th - M_PI + 2.0 * M_PI * b / (n - 1);
        const double dx = cos(a), dy = sin(a);
        double best = 30.0;
        const double walls[4][3] = {{1, 0, 10}, {1, 0, 0}, {0, 1, 6}, {0, 1, 0}};   // x = 10, x = 0, y = 6, y = 0
        for (auto& w : walls) {
            const double d = w[0] * dx + w[1] * dy;
            if (fabs(d) < 1e-12) continue;
            const double t = (w[2] - (w[0] * x + w[1] * y)) / d;
            if (t > 0 && t < best) best = t;
        }
        r[(size_t)b] = (float)best;
    }
    return r;
}

CloudPtr cloud_of(const std::vector<float>& r) {
    std::vector<float> xy(2 * r.size());
    const int64_t n = dpg_scan_to_cloud(r.data(), (int64_t)r.size(), (float)-M_PI, (float)M_PI, 30.f, 0.f, 0.f, 0.f,
                                        xy.data());
    auto c = std::make_shared<Cloud>();
    for (int64_t i = 0; i < n; ++i) c->points.push_back({xy[2 * i], xy[2 * i + 1], 0.f});
    return c;
}

int fails = 0;
#define EXPECT(cond)                                                   \
    do {                                                               \
        if (!(cond)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #cond); ++fails; } \
    } while (0)

}  // namespace

int main() {
    dpg_adapter::Context ctx(0);
    PGParams pgp;
    const double gt[4][3] = {{3.0, 3.0, 0.1}, {3.9, 3.1, 0.15}, {4.8, 3.0, 0.2}, {5.7, 2.9, 0.22}};
    std::vector<Node> nodes(4);
    std::vector<std::vector<float>> scans;
    for (int k = 0; k < 4; ++k) {
        scans.push_back(room_scan(gt[k][0], gt[k][1], gt[k][2], 360));
        nodes[(size_t)k].cloud = cloud_of(scans.back());
        nodes[(size_t)k].loc = Vector2f((float)(gt[k][0] - gt[0][0] + 0.03 * k), (float)(gt[k][1] - gt[0][1]));
        nodes[(size_t)k].th = (float)(gt[k][2] - gt[0][2]);
    }
    // runIcp (dpg_slam.h:630) against dpg_run_icp
    std::pair<std::pair<Vector2f, float>, MatrixXd> res;
    const bool conv = dpg_adapter::runIcp(ctx.get(), pgp, nodes[0], nodes[1], res);
    {
        const auto s = dpg_adapter::xy_of(nodes[1].cloud), t = dpg_adapter::xy_of(nodes[0].cloud);
        float p2[3], p1[3];
        dpg_adapter::pose_of(nodes[1], p2);
        dpg_adapter::pose_of(nodes[0], p1);
        const dpg_icp_params ip = dpg_adapter::icp_params_from(pgp);
        dpg_icp_result r;
        double cov[9];
        dpg_adapter::check(dpg_run_icp(ctx.get(), s.data(), (int64_t)s.size() / 2, t.data(), (int64_t)t.size() / 2, p2,
                                       p1, &ip, &r, cov, nullptr), "dpg_run_icp");
        EXPECT(conv == (r.converged && r.status == DPG_ICP_OK));
        EXPECT(res.first.first.x() == r.z[0] && res.first.first.y() == r.z[1] && res.first.second == r.z[2]);
        EXPECT(memcmp(res.second.m.data(), cov, sizeof(cov)) == 0);
        printf("runIcp: converged %d z = (%.4f, %.4f, %.4f), %d iterations\n", (int)conv, r.z[0], r.z[1], r.z[2],
               r.iterations);
        // calculate_ICP_COV (cov_func_point_to_point.h:24) with the final transform
        Matrix4f T{};
        T(0, 0) = r.T[0]; T(0, 1) = r.T[1]; T(0, 3) = r.T[2];
        T(1, 0) = r.T[3]; T(1, 1) = r.T[4]; T(1, 3) = r.T[5];
        T(2, 2) = 1.f; T(3, 3) = 1.f;
        MatrixXd C;
        double hb[9], hb2[9], cov2[9];
        dpg_adapter::calculate_ICP_COV(nodes[1].cloud, nodes[0].cloud, T, C, 0.5f, 0.5f, 0.3f, ctx.get(), hb);
        dpg_adapter::check(icp_cov_calculate(ctx.get(), s.data(), (int64_t)s.size() / 2, t.data(), (int64_t)t.size() / 2,
                                             T.m, 0.5f, 0.5f, 0.3f, cov2, hb2), "icp_cov_calculate");
        EXPECT(memcmp(C.m.data(), cov2, sizeof(cov2)) == 0 && memcmp(hb, hb2, sizeof(hb)) == 0);
    }
    // optimizeGraph (dpg_slam.h:464): prior + odometry chain + the ICP factor
    {
        const double sig[3] = {0.2, 0.2, 0.15}, info[3] = {2.0, 2.0, 1.0 / 0.3f};
        std::vector<dpg_factor> F{dpg_adapter::prior_factor(0, 0, 0, 0, sig)};
        for (int k = 1; k < 4; ++k)
            F.push_back(dpg_adapter::between_factor(k - 1, k, 0.9, 0.0, 0.03, info));
        F.push_back(dpg_adapter::between_factor(0, 1, res.first.first.x(), res.first.first.y(), res.first.second, info));
        std::vector<Node> a = nodes;
        const dpg_gn_stats st = dpg_adapter::optimizeGraph(ctx.get(), a, F);
        std::vector<double> X(12);
        for (int k = 0; k < 4; ++k) { X[3 * k] = nodes[k].loc.x(); X[3 * k + 1] = nodes[k].loc.y(); X[3 * k + 2] = nodes[k].th; }
        dpg_gn_params gp;
        dpg_gn_params_default(&gp);
        dpg_gn_stats st2;
        dpg_adapter::check(dpg_optimize_graph(ctx.get(), X.data(), 4, F.data(), (int64_t)F.size(), &gp, &st2),
                           "dpg_optimize_graph");
        for (int k = 0; k < 4; ++k)
            EXPECT(a[k].loc.x() == (float)X[3 * k] && a[k].loc.y() == (float)X[3 * k + 1] && a[k].th == (float)X[3 * k + 2]);
        EXPECT(st.iterations == st2.iterations);
        printf("optimizeGraph: %d iterations, error %.6g\n", st.iterations, st.final_error);
    }
    // the multi-device contexts through the same adapter calls: one
    // process over n GPUs at n = 1 (RCCL with one rank) must equal the single device byte for byte;
    // two virtual devices on this GPU run the n > 1 shard / gather / all-reduce paths
    {
        const double sig[3] = {0.2, 0.2, 0.15}, info[3] = {2.0, 2.0, 1.0 / 0.3f};
        std::vector<dpg_factor> F{dpg_adapter::prior_factor(0, 0, 0, 0, sig)};
        for (int k = 1; k < 4; ++k) F.push_back(dpg_adapter::between_factor(k - 1, k, 0.9, 0.0, 0.03, info));
        F.push_back(dpg_adapter::between_factor(0, 2, 1.8, 0.0, 0.07, info));
        std::vector<std::pair<Vector2f, float>> odom;
        for (int k = 0; k < 4; ++k) odom.emplace_back(Vector2f(0.9f * (float)k, 0.0f), 0.03f * (float)k);
        std::vector<Node> a1 = nodes, r1 = nodes;
        dpg_adapter::Context s0(0);   // its own single-device context: reoptimize uploads the scans
        const dpg_gn_stats s1 = dpg_adapter::optimizeGraph(s0.get(), a1, F);
        const dpg_reopt_stats q1 = dpg_adapter::reoptimize(s0.get(), r1, odom, pgp);
        dpg_adapter::Context m1 = dpg_adapter::Context::multi(1);
        dpg_adapter::Context v2 = dpg_adapter::Context::virtual_devices(2);
        EXPECT(m1.ranks() == 1 && v2.ranks() == 2);
        int form = 0;
        for (dpg_adapter::Context* c : {&m1, &v2}) {
            std::vector<Node> a2 = nodes, r2 = nodes;
            const dpg_gn_stats s2 = dpg_adapter::optimizeGraph(c->get(), a2, F);
            const dpg_reopt_stats q2 = dpg_adapter::reoptimize(c->get(), r2, odom, pgp);
            double worst = 0.0;
            for (int k = 0; k < 4; ++k)
                worst = std::max({worst, (double)std::fabs(a1[k].loc.x() - a2[k].loc.x()), (double)std::fabs(a1[k].th - a2[k].th),
                                  (double)std::fabs(r1[k].loc.x() - r2[k].loc.x()), (double)std::fabs(r1[k].th - r2[k].th)});
            EXPECT(s1.iterations == s2.iterations && q1.n_icp_edges == q2.n_icp_edges &&
                   q1.n_loop_closures == q2.n_loop_closures && q1.gn.iterations == q2.gn.iterations);
            EXPECT(form == 0 ? worst == 0.0 : worst < 1e-5);   // float poses: 1 ulp
            printf("%s: optimizeGraph + reoptimize through the adapter, max pose difference %.3g\n",
                   form == 0 ? "multi(1)" : "virtual(2)", worst);
            ++form;
        }
    }
    // incremental form: one add_node per node
    {
        dpg_adapter::IncGraph g(ctx.get());
        std::vector<int32_t> passes;
        const double sig[3] = {0.2, 0.2, 0.15}, info[3] = {2.0, 2.0, 1.0 / 0.3f};
        for (int k = 0; k < 4; ++k) {
            passes.push_back(0);
            float ip[3];
            dpg_adapter::pose_of(nodes[(size_t)k], ip);
            std::vector<dpg_factor> extra{k == 0 ? dpg_adapter::prior_factor(0, 0, 0, 0, sig)
                                                 : dpg_adapter::between_factor(k - 1, k, 0.9, 0.0, 0.03, info)};
            const dpg_add_node_stats st = g.add_node(nodes[(size_t)k].cloud, passes, ip, extra, pgp, true);
            EXPECT(st.update.n_nodes == k + 1);
        }
        std::vector<Node> b = nodes;
        g.write_back(b);
        EXPECT(g.size() == 4);
        printf("IncGraph: node 3 at (%.4f, %.4f, %.4f)\n", b[3].loc.x(), b[3].loc.y(), b[3].th);
        // reoptimize on the live graph (the graph is rebuilt from the sweep's factors), against the
        // direct C call on a second graph built the same way; then the graph keeps growing
        std::vector<std::pair<Vector2f, float>> odom;
        for (int k = 0; k < 4; ++k) odom.emplace_back(Vector2f(0.9f * (float)k, 0.0f), 0.03f * (float)k);
        dpg_adapter::Context ctx2(0);   // its own scan store
        dpg_adapter::IncGraph g2(ctx2.get());
        for (int k = 0; k < 4; ++k) {
            float ip[3];
            dpg_adapter::pose_of(nodes[(size_t)k], ip);
            std::vector<dpg_factor> extra{k == 0 ? dpg_adapter::prior_factor(0, 0, 0, 0, sig)
                                                 : dpg_adapter::between_factor(k - 1, k, 0.9, 0.0, 0.03, info)};
            std::vector<int32_t> ps(passes.begin(), passes.begin() + k + 1);
            g2.add_node(nodes[(size_t)k].cloud, ps, ip, extra, pgp, true);
        }
        std::vector<float> est(12), od(12);
        std::vector<int32_t> pass4(4, 0);
        for (int k = 0; k < 4; ++k) {
            dpg_adapter::pose_of(b[(size_t)k], &est[3 * (size_t)k]);
            od[3 * (size_t)k] = odom[(size_t)k].first.x();
            od[3 * (size_t)k + 1] = odom[(size_t)k].first.y();
            od[3 * (size_t)k + 2] = odom[(size_t)k].second;
        }
        const dpg_reopt_stats rs = g.reoptimize(b, odom, pgp);
        const dpg_icp_params ipar = dpg_adapter::icp_params_from(pgp);
        dpg_reopt_params rp;
        dpg_reopt_params_default(&rp);
        rp.max_node_dist_within_pass = pgp.maximum_node_dist_within_pass_scan_comparison_;
        rp.max_node_dist_across_passes = pgp.maximum_node_dist_across_passes_scan_comparison_;
        rp.odometry_constraints = pgp.odometry_constraints_ ? 1 : 0;
        std::vector<double> X2(12);
        dpg_reopt_stats rs2;
        dpg_adapter::check(dpg_reoptimize_inc(g2.get(), 4, pass4.data(), est.data(), od.data(), &ipar, &rp, X2.data(), &rs2),
                           "dpg_reoptimize_inc");
        for (int k = 0; k < 4; ++k)
            EXPECT(b[k].loc.x() == (float)X2[3 * k] && b[k].loc.y() == (float)X2[3 * k + 1] && b[k].th == (float)X2[3 * k + 2]);
        EXPECT(rs.n_factors == rs2.n_factors && rs.n_icp_edges == rs2.n_icp_edges && g.size() == 4);
        passes.push_back(0);
        float ip4[3] = {b[3].loc.x() + 0.9f, b[3].loc.y(), b[3].th};
        std::vector<dpg_factor> ex4{dpg_adapter::between_factor(3, 4, 0.9, 0.0, 0.0, info)};
        const dpg_add_node_stats st5 = g.add_node(nodes[3].cloud, passes, ip4, ex4, pgp, true);
        EXPECT(st5.update.n_nodes == 5 && g.size() == 5);
        printf("IncGraph::reoptimize: %lld factors, %lld ICP edges; then node 5 added\n", (long long)rs.n_factors,
               (long long)rs.n_icp_edges);
        // checkpoint: save, restore on a third context, both add the same node
        char path[] = "/tmp/adapter_check_graph_XXXXXX";
        const int fd = mkstemp(path);
        EXPECT(fd >= 0);
        if (fd >= 0) close(fd);
        g.save(path);
        dpg_adapter::Context ctx3(0);
        dpg_adapter::IncGraph g3 = dpg_adapter::IncGraph::load(ctx3.get(), path);
        unlink(path);
        EXPECT(g3.size() == 5);
        passes.push_back(0);
        float ip5[3] = {ip4[0] + 0.9f, ip4[1], ip4[2]};
        std::vector<dpg_factor> ex5{dpg_adapter::between_factor(4, 5, 0.9, 0.0, 0.0, info)};
        const dpg_add_node_stats sa = g.add_node(nodes[2].cloud, passes, ip5, ex5, pgp, true);
        const dpg_add_node_stats sb = g3.add_node(nodes[2].cloud, passes, ip5, ex5, pgp, true);
        std::vector<Node> c1(6), c3(6);
        g.write_back(c1);
        g3.write_back(c3);
        double worst = 0.0;
        for (int k = 0; k < 6; ++k)
            worst = std::max(worst, (double)std::max(std::fabs(c1[k].loc.x() - c3[k].loc.x()), std::fabs(c1[k].th - c3[k].th)));
        EXPECT(sa.update.n_factors == sb.update.n_factors && sa.n_icp_edges == sb.n_icp_edges && worst < 1e-5);
        printf("IncGraph::save/load: node 6 added to both, max pose difference %.3g\n", worst);
    }
    // executeDPG: the store grows scan by scan; a second pass sees the room with a wall moved
    {
        dpg_adapter::DpgStore store(ctx.get());
        std::vector<Node> nd(2);
        auto r0 = room_scan(5.0, 3.0, 0.0, 360);
        auto r1 = r0;
        for (int b = 0; b < 72; ++b) r1[(size_t)b] += 2.0f;
        store.add_scan(r0, (float)-M_PI, (float)M_PI, 30.f);
        store.add_scan(r1, (float)-M_PI, (float)M_PI, 30.f);
        std::vector<Vector2f> s0, s1, s2, s3;
        const dpg_change_stats st = store.executeDPG(nd, 1, s0, s1, s2, s3);
        int64_t cnt[4];
        const float est[6] = {0, 0, 0, 0, 0, 0};
        dpg_active_dynamic_points(store.get(), 2, est, nullptr, 0, cnt);
        EXPECT((int64_t)s0.size() == cnt[0] && (int64_t)s1.size() == cnt[1] && (int64_t)s2.size() == cnt[2] &&
               (int64_t)s3.size() == cnt[3]);
        printf("executeDPG: %lld candidates, %lld removed, lists %zu %zu %zu %zu\n", (long long)st.n_candidates,
               (long long)st.n_removed, s0.size(), s1.size(), s2.size(), s3.size());
    }
    // the reference's placement (current_pass_nodes_ copies): copies equal to the estimates give
    // the same call as the plain form
    {
        dpg_adapter::DpgStore store(ctx.get());
        std::vector<Node> nd(2);
        auto r0 = room_scan(5.0, 3.0, 0.0, 360);
        auto r1 = r0;
        for (int b = 0; b < 72; ++b) r1[(size_t)b] += 2.0f;
        store.add_scan(r0, (float)-M_PI, (float)M_PI, 30.f);
        store.add_scan(r1, (float)-M_PI, (float)M_PI, 30.f);
        const std::vector<Node> pass(nd.begin() + 1, nd.end());
        std::vector<Vector2f> s0, s1, s2, s3;
        const dpg_change_stats st = store.executeDPG(nd, pass, s0, s1, s2, s3);
        EXPECT(st.n_chain == 1 && st.n_candidates == 1);
        printf("executeDPG (current_pass_nodes_ placement): %lld candidates, %lld removed\n",
               (long long)st.n_candidates, (long long)st.n_removed);
    }
    printf(fails ? "adapter check FAILED (%d)\n" : "adapter check ok\n", fails);
    return fails ? 1 : 0;
}
