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

#include <stdint.h>

#include "../../include/dpg_slam_c.h"

struct dpg_gn_dev;

// control block on the device
struct dpg_gn_ctl {
    int32_t active, reuse;          // the gate of the next iteration (gate_off in dpg_chol.hip)
    int32_t last_was_chord, have_factor, it, pad[3];
    double last_dinf, prev_dinf, cur_error, pad2;
};
// what the control kernel of iteration k reports (written into host memory)
struct dpg_gn_slot {
    double dinf, error, status;
    int32_t reuse, active, final_, it;
};

extern "C" {
// the fused Cholesky of this graph can run gated (dpg_chol.hip)
int dpg_chol_gated_ok(void* chol);
int dpg_chol_solve_gated(void* chol, const double* hb, const int32_t* gate, void* stream);
// set the control block for iteration 1 from the host state (g's chord bookkeeping) and the
// initial error
int dpg_gn_pipe_init(dpg_gn_dev* g, const dpg_gn_params* gp, dpg_gn_ctl* ctl, double cur_error, void* stream);
// enqueue one gated iteration: solve, retract, re-linearize + assemble into g->hb_own, control
// kernel (reports into slot, a host-mapped pointer)
int dpg_gn_pipe_issue(dpg_gn_dev* g, const dpg_gn_params* gp, dpg_gn_ctl* ctl, dpg_gn_slot* slot, void* stream);
}

#endif
