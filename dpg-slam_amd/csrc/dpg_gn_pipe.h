// dpg_gn_pipe.h -- the pipelined single-device Gauss-Newton loop (private).
//
// dpg_gn_run / dpg_optimize_graph on one device decide per iteration whether to stop and whether
// to reuse the last Cholesky factor (a chord step).  Taken on the host, that decision needs the
// iteration's scalars back before the next launch: the GPU idles for a host round trip every
// iteration.  Here the decision runs on the device: a one-thread control kernel at the end of
// iteration k writes the gate of iteration k + 1 (run? reuse?) plus the scalars the host reads
// later, and every launch of an iteration checks the gate first (a gated-off launch exits at
// once).  The host keeps one iteration queued ahead of the one it reads, so the queue never
// drains; an iteration enqueued after the last one is all no-ops.  The arithmetic and the
// decisions are the host loop's (dpg_api.hip gn_loop), so poses, errors and iteration counts
// are identical.
#ifndef DPG_GN_PIPE_H
#define DPG_GN_PIPE_H

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/dpg_slam_c.h"

struct dpg_gn_dev;

// the control kernel's status when the devices of a multi-device form report different max |delta|
// (after the chol status words: 1 not positive definite, 2 a bounded wait expired)
#define DPG_GN_STATUS_DIVERGED 3

// control block on the device
struct dpg_gn_ctl {
    int32_t active, reuse;          // the gate of the next iteration (gate_off in dpg_chol.hip)
    int32_t last_was_chord, have_factor, it;
    uint32_t loop;                  // the host's loop number (tags the reports of this loop)
    int32_t pad[2];
    double last_dinf, prev_dinf, cur_error, pad2;
};
// what the control kernel of an ACTIVE iteration k reports (written into host memory; a gated-off
// iteration writes nothing).  The host polls `tag` = loop << 32 | k, stored after the other fields
// and a system-scope fence: no event (and no end-of-kernel system release per iteration) is needed
struct dpg_gn_slot {
    double dinf, error, status;
    int32_t reuse, active, final_, it;
    uint64_t tag;
};

// X_v <- X_v * Pose2(d) (Pose2 retraction); returns max |d|, NaN as +inf.  Shared by the
// retraction kernel (dpg_gn.hip) and the backward solve that retracts as it goes (dpg_chol.hip).
__device__ __forceinline__ double pose_retract(double* __restrict__ Xv, double d0, double d1, double d2) {
    const double c = cos(Xv[2]), s = sin(Xv[2]);
    const double cd = cos(d2), sd = sin(d2);
    const double nx = Xv[0] + (c * d0 - s * d1);
    const double ny = Xv[1] + (s * d0 + c * d1);
    const double nc = c * cd - s * sd, ns = s * cd + c * sd;
    Xv[0] = nx;
    Xv[1] = ny;
    Xv[2] = atan2(ns, nc);
    double m = fmax(fabs(d0), fmax(fabs(d1), fabs(d2)));
    if (!(m == m)) m = __longlong_as_double(0x7ff0000000000000ll);   // NaN -> +inf (stops the loop)
    return m;
}

extern "C" {
// the fused Cholesky of this graph can run gated (dpg_chol.hip)
int dpg_chol_gated_ok(void* chol);
// X != NULL: the backward solve also retracts the poses X (by node) with the solution and keeps
// max |x| in *max_out (retract_kernel's work)
int dpg_chol_solve_gated(void* chol, const double* hb, const int32_t* gate, int prezeroed, double* X, double* max_out,
                         void* stream);
// order `stream` after the L11^-1 kernel the last gated solve ran on its side stream (before the
// control kernel rewrites the gate that kernel reads)
int dpg_chol_join_aux(void* chol, void* stream);
// the fused solve's synchronisation words (cleared before every solve)
void dpg_chol_sync_dev(void* chol, int32_t** sync, int64_t* n_words);
// set the control block for iteration 1 from the host state (g's chord bookkeeping) and the
// initial error
// the initial error comes from the device (cur_dev: the assembled chi2 word, all-reduced on the
// multi-device forms) and is reported in init->error; a loop whose initial error is not > 0 runs
// no iteration (iteration 1 reports active = 0)
// (init->tag = loop << 32 once written; the reports of iteration k carry loop << 32 | k)
int dpg_gn_pipe_init(dpg_gn_dev* g, const dpg_gn_params* gp, dpg_gn_ctl* ctl, const double* cur_dev, dpg_gn_slot* init,
                     uint32_t loop, void* stream);
// enqueue one gated iteration: solve, retract, re-linearize + assemble into g->hb_own, control
// kernel (reports into slot, a host-mapped pointer)
int dpg_gn_pipe_issue(dpg_gn_dev* g, const dpg_gn_params* gp, dpg_gn_ctl* ctl, dpg_gn_slot* slot, void* stream);
// the same in two halves for the multi-device forms (part = 1): solve from hb_own, retract and
// assemble this device's share into hb_part with its error; [the caller's all-reduce hb_part ->
// hb_own]; the control kernel, taking the error from hb_own.  part = 0 is dpg_gn_pipe_issue.
int dpg_gn_pipe_issue_solve(dpg_gn_dev* g, dpg_gn_ctl* ctl, int part, void* stream);
int dpg_gn_pipe_issue_ctl(dpg_gn_dev* g, const dpg_gn_params* gp, dpg_gn_ctl* ctl, dpg_gn_slot* slot, int part,
                          void* stream);
}

#endif
