/* pocket_tts_probe.h - measurement and test hooks of libpocket_tts_hip.so.
 *
 * Not part of the drop-in boundary (include/pocket_tts.h): nothing in the reference corresponds
 * to these, and a reference-side binding never declares them. bench.py, the
 * GPU tests and tools/ use them to time single kernels of the step plan, list the plan with its
 * algorithmic costs, probe front/back overlap and test the GEMM core on off-model shapes. Same
 * conventions as pocket_tts.h (status codes, the thread-local last-error message).
 */
#ifndef POCKET_TTS_PROBE_H
#define POCKET_TTS_PROBE_H

#include "pocket_tts.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Test hook of the GEMM core (no reference counterpart): y = x w^T for x [m][k], w [n][k] (host
 * buffers, k % 32 == 0) on the engine's device, with the tile of kernel layout `layout`
 * (kernels.hip gemm_launch: the f32 tiles, and + 100 for their bf16-operand twins); splits > 1
 * writes the [splits][m][n] split-K partial slabs to y, tail_slices > 0 takes the split-tail path
 * (layouts 34 / 35). The tests run every shipped layout on shapes the model never runs. */
int ptts_test_gemm(ptts_engine* e, int layout, int m, int n, int k, int splits, int tail_slices, const float* x,
                   const float* w, float* y);
/* Measurement: replay one named kernel of the step plan `reps` times between HIP events on
 * the engine stream; returns the average duration in microseconds. */
int ptts_time_kernel(ptts_engine* e, int n_rows, const char* name, int reps, double* avg_us);
/* The step plan for n_rows: one line per op, "name<TAB>flops<TAB>bytes" (algorithmic cost of one
 * launch; 0 where not modelled). */
int ptts_plan_ops(ptts_engine* e, int n_rows, char* buf, int buflen);

/* Measurement: the step plan split at the FlowLM/flow-head -> Mimi boundary, timed as two
 * graphs alone and launched together on two streams; us8 = {front, back, both, both with the
 * front on a high-priority stream, 0, 0, 0, 0} microseconds per step. Clobbers engine state
 * (timing only). */
int ptts_probe_overlap(ptts_engine* e, int n_rows, int reps, double* us8);

#ifdef __cplusplus
}
#endif
#endif
