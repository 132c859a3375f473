// TD loss of the DQN family with the mean Q-function, fused with its gradient.
//
// Reference (per sample b of a batch of B, one critic):
//   DQNImpl.compute_target (algos/torch/dqn_impl.py:128-137): a* = argmax_a Q_targ(s', a)
//   DoubleDQNImpl.compute_target (:162-171):                  a* = argmax_a Q(s', a)
//   target = Q_targ(s', a*)         (pick_value_by_action, q_functions/utility.py:9-15)
//   DiscreteMeanQFunction.compute_error (mean_q_function.py:25-40):
//     value = Q(s, a_b);  y = r + gamma^n * target * (1 - terminal)
//     loss  = mean_b huber(value, y)  (compute_huber_loss, utility.py:27-32, beta 1)
//   DiscreteCQLImpl.compute_loss (algos/torch/cql_impl.py:279-302):
//     + alpha * mean_b (logsumexp_a Q(s, a) - Q(s, a_b))
// and dL/dQ(s, .) for the head backward.  One workgroup; each thread owns rows
// b = tid, tid + nt, ...; the batch sums are fixed-order block reductions.
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

__device__ __forceinline__ int argmax_row(const float* q, int A) {
  int arg = 0;
  float best = q[0];
  for (int j = 1; j < A; ++j)
    if (q[j] > best) { best = q[j]; arg = j; }  // torch.argmax: first maximum
  return arg;
}

__global__ __launch_bounds__(1024) void dqn_loss_kernel(d3a_dqn_loss_desc d) {
  __shared__ float scratch[16];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int B = d.B, A = d.A;
  const float invB = 1.f / (float)B;
  float s_td = 0.f, s_cons = 0.f;
  for (int b = tid; b < B; b += nt) {
    const float* q = d.q + (int64_t)b * A;                   // Q(s_b, .)
    const float* qt = d.q_targ + (int64_t)b * A;             // Q_targ(s'_b, .)
    const int ab = d.act[b];
    const int astar = argmax_row(d.double_q ? d.q_next + (int64_t)b * A : qt, A);
    const float target = qt[astar];
    const float gam = powf(d.gamma, d.n_steps[b]);
    const float y = d.rew[b] + gam * target * (1.f - d.term[b]);
    const float value = q[ab];
    const float diff = y - value;
    const float ad = fabsf(diff);
    const bool quad = ad < 1.f;
    s_td += quad ? 0.5f * (diff * diff) : (ad - 0.5f);
    // d huber / d value = -(diff if |diff| < 1 else sign(diff)), mean over B
    const float gv = -(quad ? diff : (diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f))) * invB;
    float* g = d.dq + (int64_t)b * A;
    if (d.alpha != 0.f) {
      // torch.logsumexp: max shift (an infinite max shifts by 0)
      float mx = q[0];
      for (int j = 1; j < A; ++j) mx = fmaxf(mx, q[j]);
      if (isinf(mx)) mx = 0.f;
      float se = 0.f;
      for (int j = 0; j < A; ++j) se += expf(q[j] - mx);
      const float lse = logf(se) + mx;
      s_cons += lse - value;
      const float ga = d.alpha * invB;
      for (int j = 0; j < A; ++j) {
        const float sm = expf(q[j] - lse);
        g[j] = ga * sm - (j == ab ? ga : 0.f) + (j == ab ? gv : 0.f);
      }
    } else {
      for (int j = 0; j < A; ++j) g[j] = j == ab ? gv : 0.f;
    }
  }
  const float td = block_sum(s_td, scratch) * invB;
  const float cons = block_sum(s_cons, scratch) * invB;
  if (tid == 0) {
    d.metrics[0] = d.alpha != 0.f ? td + d.alpha * cons : td;
    d.metrics[1] = td;
    d.metrics[2] = cons;
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_dqn_loss(const d3a_dqn_loss_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->q && d->q_targ && d->act && d->rew && d->term && d->n_steps && d->dq &&
                    d->metrics,
                "d3a_dqn_loss: null operand");
  D3A_CHECK_ARG(!d->double_q || d->q_next, "d3a_dqn_loss: double_q needs q_next");
  D3A_CHECK_ARG(d->B >= 1 && d->A >= 1, "d3a_dqn_loss: bad sizes");
  hipLaunchKernelGGL(dqn_loss_kernel, dim3(1), dim3(d->B >= 512 ? 1024 : 256), 0,
                     (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_dqn_loss");
  return 0;
}
