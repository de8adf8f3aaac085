/*
 * dpg_synth.c -- seeded synthetic workload for the benchmark configs:
 * a 2D line-segment world (rooms, doorways, boxes), a collision-free 1 m-step trajectory that
 * keeps revisiting the world (loop closures), and exactly ray-cast laser scans.
 * Deterministic for a given seed on a given libm (splitmix64 + Box-Muller in double).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#include "../../include/dpg_slam_c.h"

typedef struct { uint64_t s; } rng_t;

static uint64_t splitmix64(rng_t* r) {
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double unif(rng_t* r) { return (double)(splitmix64(r) >> 11) * (1.0 / 9007199254740992.0); }
static double gauss(rng_t* r) {
    double u1 = unif(r), u2 = unif(r);
    if (u1 < 1e-300) u1 = 1e-300;
    return sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2);
}

static int64_t push_seg(float* s, int64_t n, int64_t cap, float x0, float y0, float x1, float y1) {
    if (n >= cap) return n;
    s[4 * n] = x0; s[4 * n + 1] = y0; s[4 * n + 2] = x1; s[4 * n + 3] = y1;
    return n + 1;
}

int64_t dpg_synth_world(uint64_t seed, float W, float* s, int64_t cap) {
    rng_t r = {seed * 0x1000193ull + 17};
    int64_t n = 0;
    /* outer walls */
    n = push_seg(s, n, cap, 0, 0, W, 0);
    n = push_seg(s, n, cap, W, 0, W, W);
    n = push_seg(s, n, cap, W, W, 0, W);
    n = push_seg(s, n, cap, 0, W, 0, 0);
    /* interior walls on a room grid, each with a 2 m doorway at a random position */
    const int rooms = (int)(W / 10.0f) > 1 ? (int)(W / 10.0f) : 2;
    const float cell = W / (float)rooms;
    for (int k = 1; k < rooms; ++k) {
        const float c = cell * (float)k;
        for (int m = 0; m < rooms; ++m) {
            const float a0 = cell * (float)m, a1 = a0 + cell;
            const float door = a0 + 1.0f + (float)unif(&r) * (cell - 4.0f);
            /* vertical wall x = c, from a0 to a1 with a gap [door, door + 2] */
            n = push_seg(s, n, cap, c, a0, c, door);
            n = push_seg(s, n, cap, c, door + 2.0f, c, a1);
            const float door2 = a0 + 1.0f + (float)unif(&r) * (cell - 4.0f);
            n = push_seg(s, n, cap, a0, c, door2, c);
            n = push_seg(s, n, cap, door2 + 2.0f, c, a1, c);
        }
    }
    /* random boxes (furniture / pillars), away from the walls */
    const int boxes = rooms * rooms * 2;
    for (int b = 0; b < boxes; ++b) {
        const float cx = 1.5f + (float)unif(&r) * (W - 3.0f), cy = 1.5f + (float)unif(&r) * (W - 3.0f);
        const float hx = 0.2f + (float)unif(&r) * 0.5f, hy = 0.2f + (float)unif(&r) * 0.5f;
        n = push_seg(s, n, cap, cx - hx, cy - hy, cx + hx, cy - hy);
        n = push_seg(s, n, cap, cx + hx, cy - hy, cx + hx, cy + hy);
        n = push_seg(s, n, cap, cx + hx, cy + hy, cx - hx, cy + hy);
        n = push_seg(s, n, cap, cx - hx, cy + hy, cx - hx, cy - hy);
    }
    return n;
}

/* distance from point p to segment */
static double seg_dist(double px, double py, const float* g) {
    double ax = g[0], ay = g[1], bx = g[2], by = g[3];
    double vx = bx - ax, vy = by - ay, wx = px - ax, wy = py - ay;
    double l2 = vx * vx + vy * vy;
    double t = l2 > 0 ? (wx * vx + wy * vy) / l2 : 0.0;
    if (t < 0) t = 0;
    if (t > 1) t = 1;
    double dx = px - (ax + t * vx), dy = py - (ay + t * vy);
    return sqrt(dx * dx + dy * dy);
}

/* does segment p->q cross segment g (proper or touching)? */
static int crosses(double px, double py, double qx, double qy, const float* g) {
    double ax = g[0], ay = g[1], bx = g[2], by = g[3];
    double d1 = (bx - ax) * (py - ay) - (by - ay) * (px - ax);
    double d2 = (bx - ax) * (qy - ay) - (by - ay) * (qx - ax);
    double d3 = (qx - px) * (ay - py) - (qy - py) * (ax - px);
    double d4 = (qx - px) * (by - py) - (qy - py) * (bx - px);
    return ((d1 > 0) != (d2 > 0)) && ((d3 > 0) != (d4 > 0));
}

static int free_move(double px, double py, double qx, double qy, const float* segs, int64_t ns,
                     double W, double clearance) {
    if (qx < clearance || qy < clearance || qx > W - clearance || qy > W - clearance) return 0;
    for (int64_t k = 0; k < ns; ++k) {
        if (crosses(px, py, qx, qy, segs + 4 * k)) return 0;
        if (seg_dist(qx, qy, segs + 4 * k) < clearance) return 0;
    }
    return 1;
}

int dpg_synth_trajectory(uint64_t seed, int64_t n, const float* segs, int64_t ns, float W, float step,
                         double* gt) {
    if (n <= 0) return DPG_ERR_ARG;
    rng_t r = {seed * 0x2545F4914F6CDD1Dull + 3};
    /* start near the middle of a room */
    double x = 0.5 * (double)W / ((int)(W / 10.0f) > 1 ? (int)(W / 10.0f) : 2), y = x, th = 0.3;
    for (int tries = 0; tries < 1000 && !free_move(x, y, x, y, segs, ns, W, 0.5); ++tries) {
        x = 1.0 + unif(&r) * (W - 2.0);
        y = 1.0 + unif(&r) * (W - 2.0);
    }
    gt[0] = x; gt[1] = y; gt[2] = th;
    for (int64_t i = 1; i < n; ++i) {
        double nth = th + 0.35 * gauss(&r);
        int ok = 0;
        for (int tries = 0; tries < 200; ++tries) {
            double qx = x + step * cos(nth), qy = y + step * sin(nth);
            if (free_move(x, y, qx, qy, segs, ns, W, 0.45)) { x = qx; y = qy; th = nth; ok = 1; break; }
            nth = th + (unif(&r) * 2.0 - 1.0) * M_PI;
        }
        if (!ok) th += M_PI; /* stuck: turn around in place (still a new node, 0 m motion) */
        th = atan2(sin(th), cos(th));
        gt[3 * i] = x; gt[3 * i + 1] = y; gt[3 * i + 2] = th;
    }
    return DPG_OK;
}

typedef struct {
    const double* gt; int64_t n; const float* segs; int64_t ns; int32_t nb;
    float amin, amax, rmax, lx, ly, lth, sigma; uint64_t seed; float* out;
    int64_t v0, v1;
} scan_job;

/* segs: the segments that can be hit within range_max of (ox, oy) -- a segment farther away gives
   a hit beyond range_max, which reads range_max like no hit at all, so the scan is unchanged */
static void scan_one(const scan_job* J, int64_t v, int32_t* near) {
    rng_t r = {J->seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(v + 1))};
    const double* gt = J->gt;
    const double c = cos(gt[3 * v + 2]), s = sin(gt[3 * v + 2]);
    const double ox = gt[3 * v] + c * J->lx - s * J->ly, oy = gt[3 * v + 1] + s * J->lx + c * J->ly;
    int64_t nn = 0;
    for (int64_t k = 0; k < J->ns; ++k)
        if (seg_dist(ox, oy, J->segs + 4 * k) <= (double)J->rmax + 1e-3) near[nn++] = (int32_t)k;
    const double base = gt[3 * v + 2] + J->lth;
    const double inc = ((double)J->amax - (double)J->amin) / (double)(J->nb - 1);
    for (int32_t b = 0; b < J->nb; ++b) {
        const double a = base + (double)J->amin + inc * (double)b;
        const double dx = cos(a), dy = sin(a);
        double best = 1e30;
        for (int64_t q = 0; q < nn; ++q) {
            const float* g = J->segs + 4 * (int64_t)near[q];
            const double ex = (double)g[2] - g[0], ey = (double)g[3] - g[1];
            const double den = dx * ey - dy * ex;
            if (fabs(den) < 1e-12) continue;
            const double wx = (double)g[0] - ox, wy = (double)g[1] - oy;
            const double t = (wx * ey - wy * ex) / den;   /* along the ray */
            const double u = (wx * dy - wy * dx) / den;   /* along the segment */
            if (t > 0 && u >= 0 && u <= 1 && t < best) best = t;
        }
        const double noise = J->sigma * gauss(&r);
        double range = best + noise;
        if (best >= (double)J->rmax || range >= (double)J->rmax) range = J->rmax;
        if (range < 0.05) range = 0.05;
        J->out[(size_t)v * (size_t)J->nb + (size_t)b] = (float)range;
    }
}

static void* scan_worker(void* arg) {
    const scan_job* J = (const scan_job*)arg;
    int32_t* near = (int32_t*)malloc(sizeof(int32_t) * (size_t)(J->ns > 0 ? J->ns : 1));
    if (!near) return NULL;
    for (int64_t v = J->v0; v < J->v1; ++v) scan_one(J, v, near);
    free(near);
    return NULL;
}

int dpg_synth_scans(const double* gt, int64_t n, const float* segs, int64_t ns, int32_t nb,
                    float amin, float amax, float rmax, float lx, float ly, float lth, float sigma,
                    uint64_t seed, int32_t n_threads, float* out) {
    if (n <= 0 || nb < 2) return DPG_ERR_ARG;
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 64) n_threads = 64;
    scan_job jobs[64];
    pthread_t th[64];
    const int64_t per = (n + n_threads - 1) / n_threads;
    int started = 0;
    for (int k = 0; k < n_threads; ++k) {
        scan_job J = {gt, n, segs, ns, nb, amin, amax, rmax, lx, ly, lth, sigma, seed, out,
                      k * per, (k + 1) * per < n ? (k + 1) * per : n};
        jobs[k] = J;
        if (jobs[k].v0 >= jobs[k].v1) break;
        if (pthread_create(&th[k], NULL, scan_worker, &jobs[k]) != 0) { scan_worker(&jobs[k]); continue; }
        started = k + 1;
    }
    for (int k = 0; k < started; ++k) pthread_join(th[k], NULL);
    return DPG_OK;
}
