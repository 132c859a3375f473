/* C restatement of the reference's n-step return loop — TEST INFRASTRUCTURE.
 *
 * d3rlpy/dataset.pyx:1322-1331 (_assign_to_batch), with the C the pinned
 * Cython 0.29.21 (requirements.txt:8) generates for it: `gamma` is a C float
 * (:1298), `i` a C int, and Cython 0.29 types `float ** int` as float and
 * calls powf — the line Cython emits in its 0.29-compatible mode (cpow=True)
 * for the same statement is recorded in tests/golden/cython_pow_codegen.txt:
 *     acc = (acc + (reward * powf(gamma, ((float)i))));
 * Built with -ffp-contract=off so that line stays one fp32 multiply and one
 * fp32 add, as on the reference's x86-64 SSE build (FLT_EVAL_METHOD 0). */
#include <math.h>
#include <stdint.h>

/* rewards[0..n_avail) are the rewards of the transition chain starting at
 * the sampled transition (the walk stops at the chain's end); returns the
 * n-step return and writes the number of steps taken (i + 1). */
float d3a_oracle_nstep_return(const float* rewards, int32_t n_avail, int32_t n_steps,
                              float gamma, int32_t* n_used) {
  float n_step_return = 0.0f;
  int32_t i;
  for (i = 0; i < n_steps; ++i) {
    n_step_return = (n_step_return + (rewards[i] * powf(gamma, ((float)i))));
    if (i == n_avail - 1 || i == n_steps - 1) break;
  }
  *n_used = i + 1;
  return n_step_return;
}

float d3a_oracle_powf(float gamma, int32_t i) { return powf(gamma, (float)i); }
