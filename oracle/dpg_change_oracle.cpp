/*
 * dpg_change_oracle.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of DPG change detection, DpgSLAM::executeDPG (src/dpg_slam/dpg_slam.cc:865-886),
 * the parity checker of the product path's dpg_execute_dpg (dpg-slam_amd/csrc/dpg_change.hip).
 * It follows the reference's data structures literally: hash-map occupancy grids keyed by cell
 * (dpg_slam.h:26-260), the sequential greedy submap (dpg_slam.cc:622-712), per-node detection
 * (:745-780), the bin score (:782-830), label commits (:714-743), sector/node deactivation
 * (:888-911, dpg_node.cc:28-96) and the map lists (:832-863).  The Q8 defects of that path are
 * fixed the same way as in the product (DESIGN.md §3 "DPG"); every fix is marked "Q8 fix".
 *
 * Parity pinning: the reference cannot be built here (ROS/PCL/GTSAM), and no reference test or
 * fixture exercises this path, so this restatement is UNPINNED against the reference; it is
 * pinned only by the hand-computed known answers in tests/test_dpg.py.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <set>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "../include/dpg_slam_c.h"

namespace {

enum CellStatus { UNKNOWN, FREE, OCCUPIED };   // dpg_slam.h:26

struct Beam {
    float angle, range;
    uint8_t label, sector;
};

struct Node {
    float pose[3];
    std::vector<Beam> beams;
    std::vector<bool> sector_active;
    int activated;
    bool active;
    float amin, amax, rmax, ainc;
};

struct Pt { int64_t node, idx; };
typedef std::pair<int, int> Key;
struct KeyHash {
    size_t operator()(const Key& k) const { return ((size_t)(uint32_t)k.first << 32) ^ (uint32_t)k.second; }
};

struct Grid {
    std::unordered_map<Key, int, KeyHash> info;                // gridInfo
    std::unordered_map<Key, std::vector<Pt>, KeyHash> pts;     // occupied_cell_info_
};

// math_utils::AngleMod<float> (math_utils.h:13-16)
float angle_mod_f(float a) {
    double ad = (double)a;
    ad -= (M_PI * 2.0) * rint(ad / (M_PI * 2.0));
    return (float)ad;
}

// Eigen::Rotation2Df(th) * v
void rot2f(float th, float x, float y, float* ox, float* oy) {
    float c = cosf(th), s = sinf(th);
    float ns = -s;
    *ox = c * x + ns * y;
    *oy = s * x + c * y;
}

}  // namespace

struct oracle_dpg {
    dpg_change_params p;
    std::vector<Node> nodes;

    // transformPoint(laser pose, node pose) (dpg_node.cc:34-36, dpg_slam.cc:971-974)
    void lidar_in_map(const Node& n, float* lx, float* ly, float* la) const { lidar_at(n.pose, lx, ly, la); }
    void lidar_at(const float* pose, float* lx, float* ly, float* la) const {
        float rx, ry;
        rot2f(pose[2], p.laser[0], p.laser[1], &rx, &ry);
        *lx = pose[0] + rx;
        *ly = pose[1] + ry;
        *la = angle_mod_f(pose[2] + p.laser[2]);
    }
    // MeasurementPoint::getPointInLaserFrame (dpg_measurement.h:102-104) then transformPoint into
    // the map with the lidar pose (dpg_slam.cc:844,979; Q8 fix: once, not twice as :985-986 does)
    void map_point(const Node& n, int64_t i, float* mx, float* my, const float* pose = nullptr) const {
        const Beam& b = n.beams[(size_t)i];
        float px = b.range * cosf(b.angle), py = b.range * sinf(b.angle);
        float lx, ly, la, rx, ry;
        lidar_at(pose ? pose : n.pose, &lx, &ly, &la);
        rot2f(la, px, py, &rx, &ry);
        *mx = lx + rx;
        *my = ly + ry;
    }
    // occupancyGrid::convertToKeyForm (dpg_slam.cc:923-929)
    Key key_of(float x, float y) const {
        return Key((int)round((double)x / p.occ_grid_resolution), (int)round((double)y / p.occ_grid_resolution));
    }
    // occupancyGrid(node) -> calculateOccupancyGrid -> convertLaserRangeToCellKey (dpg_slam.cc:913-1013);
    // pose: the node copy's pose when it differs from dpg_nodes_ (a current_pass_nodes_ entry)
    Grid node_grid(int64_t v, const float* pose = nullptr) const {
        Grid g;
        const Node& n = nodes[(size_t)v];
        if (!n.active) return g;
        if (!pose) pose = n.pose;
        float lx, ly, la;
        lidar_at(pose, &lx, &ly, &la);
        std::vector<Key> occ, fre;
        for (int64_t i = 0; i < (int64_t)n.beams.size(); ++i) {
            const Beam& b = n.beams[(size_t)i];
            if (!n.sector_active[b.sector]) continue;
            // :983-984 with include_static/include_added true; Q8 fix: NOT_YET_LABELED counts as STATIC
            float mx, my;
            map_point(n, i, &mx, &my, pose);
            Key cell = key_of(mx, my);
            if (b.label != DPG_LABEL_MAX_RANGE) {
                g.pts[cell].push_back(Pt{v, i});
                occ.push_back(cell);
            }
            // getIntermediateFreeCellsInFOV (:1059-1082)
            uint32_t num_bins = (uint32_t)round((double)b.range / p.occ_grid_resolution);
            float inc = (float)(1.0 / (double)num_bins);
            for (float t = 0.0f; (double)t < 1.0; t = t + inc) {
                float ix = (1 - t) * lx + t * mx;
                float iy = (1 - t) * ly + t * my;
                fre.push_back(key_of(ix, iy));
            }
        }
        for (const Key& k : fre) {   // setFreeCells (:1021-1029)
            int& s = g.info[k];
            if (s != OCCUPIED) s = FREE;
        }
        for (const Key& k : occ) g.info[k] = OCCUPIED;   // setOccupiedCells (:1015-1019)
        return g;
    }
    // combineOccupancyGrids (:931-956): union, OCCUPIED wins, point lists concatenated
    static void combine_into(Grid& a, const Grid& b) {
        for (const auto& kv : b.info) {
            auto it = a.info.find(kv.first);
            if (it == a.info.end()) {
                a.info.emplace(kv.first, kv.second);
            } else if (kv.second == OCCUPIED) {
                it->second = OCCUPIED;
            }
            auto bp = b.pts.find(kv.first);
            if (bp != b.pts.end()) {
                std::vector<Pt>& d = a.pts[kv.first];
                d.insert(d.end(), bp->second.begin(), bp->second.end());
            }
        }
    }
    static int status(const Grid& g, const Key& k) {
        auto it = g.info.find(k);
        return it == g.info.end() ? UNKNOWN : it->second;
    }

    int execute(int64_t V, int64_t cur_len, const float* est, const float* chain_poses, dpg_change_stats* st);
    int64_t active_dynamic(int64_t V, const float* est, float* out, int64_t cap, int64_t counts[4]);
};

int oracle_dpg::execute(int64_t V, int64_t cur_len, const float* est, const float* chain_poses, dpg_change_stats* st) {
    memset(st, 0, sizeof(*st));
    if (V > (int64_t)nodes.size() || cur_len > V || cur_len < 0) return DPG_ERR_ARG;
    for (int64_t v = 0; v < V; ++v)
        for (int d = 0; d < 3; ++d) nodes[(size_t)v].pose[d] = est[3 * v + d];
    const int64_t n_past = V - cur_len;
    int sectors_before = 0, active_before = 0;
    for (int64_t v = 0; v < V; ++v) { sectors_before += nodes[(size_t)v].activated; active_before += nodes[(size_t)v].active; }

    // computeLocalSubMap (:591-620): the last current_pose_chain_len_ nodes of the pass
    const int64_t chain_n = std::min<int64_t>(cur_len, p.current_pose_chain_len);
    std::vector<int64_t> chain;
    for (int64_t k = 0; k < chain_n; ++k) chain.push_back(V - chain_n + k);
    // poseChain = current_pass_nodes_ copies (:598): their poses place the chain grids and the
    // proximity search; without chain_poses they are the estimates (Q8 fix 8)
    auto cpose = [&](size_t k) { return chain_poses ? chain_poses + 3 * k : nodes[(size_t)chain[k]].pose; };
    std::vector<Grid> chain_grids;
    for (size_t k = 0; k < chain.size(); ++k) chain_grids.push_back(node_grid(chain[k], cpose(k)));
    st->n_chain = chain_n;

    // getSubMapCoveringCurrPoseChain (:622-701)
    std::unordered_set<Key, KeyHash> uncovered;
    for (const Grid& g : chain_grids)
        for (const auto& kv : g.info) uncovered.insert(kv.first);
    const uint64_t total = uncovered.size();
    uint64_t cur_size = uncovered.size();
    Grid submap;
    bool init = false, met = false;
    for (int64_t j = 0; j < n_past; ++j) {
        const Node& past = nodes[(size_t)j];
        if (!past.active) continue;
        bool prox = false;
        for (size_t k = 0; k < chain.size(); ++k) {
            const float* c = cpose(k);
            float dx = c[0] - past.pose[0], dy = c[1] - past.pose[1];
            if (sqrtf(dx * dx + dy * dy) <= p.distance_threshold_for_local_submap_nodes) { prox = true; break; }
        }
        if (!prox) continue;
        st->n_candidates++;   // counted past the stop too (the product reports every candidate)
        if (met) continue;
        Grid g = node_grid(j);
        // getUpdatedCoverageForCurrentPoseChain (:703-712); Q8 fix: no erase while iterating
        std::vector<Key> hit;
        for (const Key& k : uncovered)
            if (g.info.count(k)) hit.push_back(k);
        for (const Key& k : hit) uncovered.erase(k);
        if (uncovered.size() < cur_size) {
            if (!init) { submap = g; init = true; } else { combine_into(submap, g); }
            cur_size = uncovered.size();
            st->n_submap_nodes++;
        }
        double coverage = 1 - ((double)cur_size) / total;
        if (coverage >= p.current_pose_graph_coverage_threshold) met = true;   // :691-694 (break)
    }
    st->n_chain_cells = (int64_t)total;
    st->n_uncovered = (int64_t)cur_size;

    // detectAndLabelChangesForCurrentPoseChain (:714-743) / ...ForCurrentNode (:745-780)
    std::vector<Pt> added, removed_nd;
    const int32_t total_bins = p.num_bins_for_change_detection;
    for (size_t k = 0; k < chain.size(); ++k) {
        const Grid& g = chain_grids[k];
        std::vector<Pt> add_k, rem_k;
        for (const auto& kv : g.info) {
            int sub = status(submap, kv.first);
            if (kv.second == OCCUPIED && sub == FREE) {
                const std::vector<Pt>& v = g.pts.at(kv.first);
                add_k.insert(add_k.end(), v.begin(), v.end());
            } else if (kv.second == FREE && sub == OCCUPIED) {
                const std::vector<Pt>& v = submap.pts.at(kv.first);
                rem_k.insert(rem_k.end(), v.begin(), v.end());
            }
        }
        if (add_k.size() + rem_k.size() == 0) continue;
        // computeBinScoreAndCommitLabelsForNode (:782-830). Q8 fixes: the current node is the chain
        // node under test (not added_points.back()), its scan's angle range, a real ratio.
        const Node& cn = nodes[(size_t)chain[k]];
        const float amin = cn.amin, amax = cn.amax;
        const float bin_inc = (amax - amin) / (float)total_bins;
        float clx, cly, cla;
        lidar_in_map(cn, &clx, &cly, &cla);
        std::unordered_set<uint32_t> bins;
        bool commit = false;
        std::vector<Pt> changed = add_k;
        changed.insert(changed.end(), rem_k.begin(), rem_k.end());
        for (const Pt& q : changed) {
            float mx, my, rx, ry;
            map_point(nodes[(size_t)q.node], q.idx, &mx, &my);
            rot2f(-cla, mx - clx, my - cly, &rx, &ry);   // inverseTransformPoint (math_utils.cc:21-35)
            float a = atan2f(ry, rx);
            if (a > amax || a < amin) continue;
            uint16_t bin = (uint16_t)((a - amin) / bin_inc);
            bins.insert(bin);
            if ((double)bins.size() / (double)total_bins >= p.delta_change_threshold) { commit = true; break; }
        }
        if (!commit) continue;
        st->n_committed++;
        added.insert(added.end(), add_k.begin(), add_k.end());
        removed_nd.insert(removed_nd.end(), rem_k.begin(), rem_k.end());
    }
    for (const Pt& q : added) {   // setPointLabel(ADDED)
        Beam& b = nodes[(size_t)q.node].beams[(size_t)q.idx];
        if (b.label != DPG_LABEL_MAX_RANGE) b.label = DPG_LABEL_ADDED;
    }
    st->n_added = (int64_t)added.size();
    std::map<int64_t, std::set<int64_t>> by_node;
    for (const Pt& q : removed_nd) by_node[q.node].insert(q.idx);
    std::vector<Pt> removed;
    for (const auto& kv : by_node)
        for (int64_t i : kv.second) {
            Node& n = nodes[(size_t)kv.first];   // Q8 fix: the point's own node (:739 indexes by point)
            Beam& b = n.beams[(size_t)i];
            if (n.sector_active[b.sector]) { n.sector_active[b.sector] = false; n.activated--; }   // Measurement::setPointLabel
            if (b.label != DPG_LABEL_MAX_RANGE) b.label = DPG_LABEL_REMOVED;
            removed.push_back(Pt{kv.first, i});
        }
    st->n_removed = (int64_t)removed.size();

    // updateNodesAndSectorStatus (:888-911) -> DpgNode::deactivateIntersectingSectors (dpg_node.cc:28-96)
    std::vector<std::pair<float, float>> rv;
    for (const Pt& q : removed) {
        float mx, my;
        map_point(nodes[(size_t)q.node], q.idx, &mx, &my);
        rv.emplace_back(mx, my);
    }
    for (int64_t v = 0; v < n_past; ++v) {
        Node& n = nodes[(size_t)v];
        if (!n.active) continue;
        float lx, ly, la;
        lidar_in_map(n, &lx, &ly, &la);
        const float sector_size = (n.amax - n.amin) / (float)p.num_sectors;
        for (const auto& q : rv) {
            float rx, ry;
            rot2f(-la, q.first - lx, q.second - ly, &rx, &ry);
            float norm = sqrtf(rx * rx + ry * ry);
            if (norm > n.rmax) continue;
            float a = atan2f(ry, rx);
            if (a > n.amax || a < n.amin) continue;
            uint8_t s = (uint8_t)((a - n.amin) / sector_size);
            if (s >= p.num_sectors || !n.sector_active[s]) continue;   // Q8 fix: continue, not break
            float approx = (a - n.amin) / n.ainc;
            int fl = (int)floorf(approx);
            fl = std::max(0, std::min(fl, (int)n.beams.size() - 1));   // bounds guard (the reference indexes unchecked)
            float fov = n.beams[(size_t)fl].range;
            if (fl < (int)n.beams.size() - 1) fov = std::min(fov, n.beams[(size_t)fl + 1].range);
            if (fov > norm) { n.sector_active[s] = false; n.activated--; }
        }
        if (p.minimum_percent_active_sectors > ((float)n.activated) / (float)p.num_sectors) n.active = false;
    }
    int sectors_after = 0, active_after = 0;
    for (int64_t v = 0; v < V; ++v) { sectors_after += nodes[(size_t)v].activated; active_after += nodes[(size_t)v].active; }
    st->n_sectors_deactivated = sectors_before - sectors_after;
    st->n_nodes_deactivated = active_before - active_after;
    return DPG_OK;
}

// getActiveAndDynamicMapPoints (:832-863)
int64_t oracle_dpg::active_dynamic(int64_t V, const float* est, float* out, int64_t cap, int64_t counts[4]) {
    std::vector<float> lists[4];
    for (int64_t v = 0; v < V; ++v) {
        Node& n = nodes[(size_t)v];
        for (int d = 0; d < 3; ++d) n.pose[d] = est[3 * v + d];
        for (int64_t i = 0; i < (int64_t)n.beams.size(); ++i) {
            const Beam& b = n.beams[(size_t)i];
            if (b.label == DPG_LABEL_NOT_YET_LABELED || b.label == DPG_LABEL_MAX_RANGE) continue;
            float mx, my;
            map_point(n, i, &mx, &my);
            if (n.active && n.sector_active[b.sector]) {
                if (b.label == DPG_LABEL_STATIC) { lists[0].push_back(mx); lists[0].push_back(my); }
                else if (b.label == DPG_LABEL_ADDED) { lists[1].push_back(mx); lists[1].push_back(my); }
            }
            if (b.label == DPG_LABEL_ADDED) { lists[3].push_back(mx); lists[3].push_back(my); }
            else if (b.label == DPG_LABEL_REMOVED) { lists[2].push_back(mx); lists[2].push_back(my); }
        }
    }
    int64_t k = 0;
    for (int l = 0; l < 4; ++l) {
        counts[l] = (int64_t)lists[l].size() / 2;
        for (size_t q = 0; q < lists[l].size(); q += 2, ++k)
            if (k < cap) { out[2 * k] = lists[l][q]; out[2 * k + 1] = lists[l][q + 1]; }
    }
    return k;
}

extern "C" {

oracle_dpg* oracle_dpg_create(int64_t V, const int64_t* off, const float* ranges, const float* geom,
                              const dpg_change_params* p) {
    oracle_dpg* o = new oracle_dpg();
    o->p = *p;
    o->nodes.resize((size_t)V);
    for (int64_t v = 0; v < V; ++v) {
        Node& n = o->nodes[(size_t)v];
        const int64_t nb = off[v + 1] - off[v];
        n.amin = geom[3 * v]; n.amax = geom[3 * v + 1]; n.rmax = geom[3 * v + 2];
        // createNode (dpg_slam.cc:497-507)
        n.ainc = (float)((double)(n.amax - n.amin) / ((double)nb - 1.0));
        const float per_sector = ((float)nb) / (float)p->num_sectors;
        n.beams.resize((size_t)nb);
        for (int64_t i = 0; i < nb; ++i) {
            Beam& b = n.beams[(size_t)i];
            b.sector = (uint8_t)((float)i / per_sector);
            b.angle = n.ainc * (float)i + n.amin;
            b.range = ranges[off[v] + i];
            b.label = b.range >= n.rmax ? DPG_LABEL_MAX_RANGE : DPG_LABEL_NOT_YET_LABELED;
        }
        n.sector_active.assign((size_t)p->num_sectors + 1, true);
        n.sector_active[(size_t)p->num_sectors] = false;
        n.activated = p->num_sectors;
        n.active = true;
        n.pose[0] = n.pose[1] = n.pose[2] = 0.f;
    }
    return o;
}

void oracle_dpg_destroy(oracle_dpg* o) { delete o; }

int oracle_dpg_append(oracle_dpg* o, int64_t n, const int64_t* off, const float* ranges, const float* geom) {
    oracle_dpg* t = oracle_dpg_create(n, off, ranges + 0, geom, &o->p);   // same per-node construction
    for (auto& nd : t->nodes) o->nodes.push_back(nd);
    delete t;
    return DPG_OK;
}

int oracle_execute_dpg(oracle_dpg* o, int64_t V, int64_t cur_len, const float* est, dpg_change_stats* st) {
    return o->execute(V, cur_len, est, nullptr, st);
}

int oracle_execute_dpg_chain(oracle_dpg* o, int64_t V, int64_t cur_len, const float* est, const float* chain_poses,
                             dpg_change_stats* st) {
    return o->execute(V, cur_len, est, chain_poses, st);
}

void oracle_dpg_fetch(oracle_dpg* o, uint8_t* labels, uint8_t* sector_active, uint8_t* node_active) {
    int64_t b = 0;
    for (size_t v = 0; v < o->nodes.size(); ++v) {
        const Node& n = o->nodes[v];
        uint8_t m = 0;
        for (int s = 0; s < o->p.num_sectors; ++s) m |= (uint8_t)(n.sector_active[(size_t)s] ? 1u << s : 0u);
        if (sector_active) sector_active[v] = m;
        if (node_active) node_active[v] = n.active ? 1 : 0;
        for (const Beam& be : n.beams) { if (labels) labels[b] = be.label; ++b; }
    }
}

void oracle_dpg_load(oracle_dpg* o, const uint8_t* labels, const uint8_t* sector_active, const uint8_t* node_active) {
    int64_t b = 0;
    for (size_t v = 0; v < o->nodes.size(); ++v) {
        Node& n = o->nodes[v];
        if (sector_active) {
            n.activated = 0;
            for (int s = 0; s < o->p.num_sectors; ++s) {
                n.sector_active[(size_t)s] = (sector_active[v] >> s) & 1u;
                n.activated += n.sector_active[(size_t)s];
            }
        }
        if (node_active) n.active = node_active[v] != 0;
        for (Beam& be : n.beams) { if (labels) be.label = labels[b]; ++b; }
    }
}

int64_t oracle_active_dynamic_points(oracle_dpg* o, int64_t V, const float* est, float* out, int64_t cap,
                                     int64_t counts[4]) {
    return o->active_dynamic(V, est, out, cap, counts);
}

}  // extern "C"
