// Elementwise / reduction stages of the TD3+BC update (K1).
//
// Reference (arithmetic restated, same op order; fp32 unless noted):
//   scaler       preprocessing/scalers.py:350-354  (x - mean) / (std + eps)
//   target       algos/torch/td3_impl.py:61-78     clamp(tanh(mu') + clamp(s*eps, -c, c), -1, 1)
//   critic loss  algos/torch/ddpg_impl.py:154-167 -> ensemble_q_function.py:75-95 ->
//                q_functions/mean_q_function.py:74-87   sum_c mean((q_c - y)^2)
//   actor loss   algos/torch/td3_plus_bc_impl.py:64-70
//                lam = alpha / mean|Q_0(s, pi(s))|;  L = -lam mean Q_0 + mean((a - pi(s))^2)
//                (bc = 0: the TD3 / DDPG loss -mean Q_0, ddpg_impl.py:244-249)
//
// The GEMM-shaped work (policy / critic layers and their backward) runs in
// gemm.hip / heads.hip; these kernels produce the layer inputs and the
// loss-side gradients between them.
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

// (x - mean) / (std + eps) with each step rounded to fp32 as torch does
__device__ __forceinline__ float standardize(float x, const float* mean, const float* std,
                                             float eps, int j) {
  if (!mean) return x;
  return __fdiv_rn(__fsub_rn(x, mean[j]), __fadd_rn(std[j], eps));
}

// x_q[b] = (scaled obs_b, act_b), x_targ[b][0:D) = scaled next_obs_b
__global__ __launch_bounds__(256) void td3_prep_kernel(d3a_td3_prep_desc d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int W = d.D + d.A;
  const int64_t n1 = (int64_t)d.B * W;
  if (i < n1) {
    const int64_t b = i / W;
    const int j = (int)(i - b * W);
    d.x_q[b * d.ldx + j] = j < d.D ? standardize(d.obs[b * d.D + j], d.mean, d.std, d.eps, j)
                                   : d.act[b * d.A + (j - d.D)];
    return;
  }
  const int64_t k = i - n1;
  if (k < (int64_t)d.B * d.D) {
    const int64_t b = k / d.D;
    const int j = (int)(k - b * d.D);
    d.x_targ[b * d.ldx + j] = standardize(d.next_obs[b * d.D + j], d.mean, d.std, d.eps, j);
  }
}

// x_targ[b][D + j] = clamp(tanh(h) + clamp(sigma * eps, -clip, clip), -1, 1)
__global__ __launch_bounds__(256) void td3_target_kernel(d3a_td3_target_desc d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)d.B * d.A) return;
  const int64_t b = i / d.A;
  const int j = (int)(i - b * d.A);
  const float a = tanhf(d.head[i]);
  const float sn = __fmul_rn(d.sigma, d.noise[i]);
  const float cn = fminf(fmaxf(sn, -d.clip), d.clip);
  const float sa = __fadd_rn(a, cn);
  d.x_targ[b * d.ldx + d.D + j] = fminf(fmaxf(sa, -1.f), 1.f);
}

// TD loss and dL/dq over the C critics (one workgroup)
__global__ __launch_bounds__(1024) void td3_critic_loss_kernel(d3a_td3_critic_loss_desc d) {
  __shared__ float scratch[16];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int B = d.B, C = d.C;
  float s = 0.f;
  for (int p = tid; p < C * B; p += nt) {
    const int c = p / B, b = p - c * B;
    float tq = d.q_targ[b];
    for (int k = 1; k < C; ++k) tq = fminf(tq, d.q_targ[k * B + b]);
    // y = rewards + gamma ** n_steps * target * (1 - terminals)
    const float gam = powf(d.gamma, d.n_steps[b]);
    const float y = __fadd_rn(d.rew[b], __fmul_rn(__fmul_rn(gam, tq), __fsub_rn(1.f, d.term[b])));
    const float diff = __fsub_rn(d.q[c * B + b], y);
    s += diff * diff;
    // mse backward: 2 (q - y) * (1 / B)
    d.dq[c * B + b] = __fmul_rn(__fmul_rn(2.f, diff), 1.f / (float)B);
  }
  const float tot = block_sum(s, scratch);
  if (tid == 0) {
    d.metrics[0] = tot / (float)B;
    if (!d.actor_step) d.metrics[1] = __int_as_float(0x7fc00000);  // NaN: not computed
  }
}

// x_actor[b] = (scaled obs_b, tanh(h_b)); pi_act = tanh(h)
__global__ __launch_bounds__(256) void td3bc_actor_input_kernel(d3a_td3bc_actor_desc d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int W = d.D + d.A;
  if (i >= (int64_t)d.B * W) return;
  const int64_t b = i / W;
  const int j = (int)(i - b * W);
  if (j < d.D) {
    d.x_actor[b * d.ldx + j] = d.x_q[b * d.ldx + j];
  } else {
    const float a = tanhf(d.head[b * d.A + (j - d.D)]);
    d.pi_act[b * d.A + (j - d.D)] = a;
    d.x_actor[b * d.ldx + j] = a;
  }
}

// lam = alpha / mean|q0| (detached); dL/dq0_b = -lam / B  (one workgroup)
__global__ __launch_bounds__(1024) void td3bc_actor_seed_kernel(d3a_td3bc_actor_desc d) {
  __shared__ double sd[16];
  __shared__ float s_lam;
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6;
  double sa = 0.0, sq = 0.0;
  for (int b = tid; b < d.B; b += nt) {
    sa += (double)fabsf(d.q0[b]);
    sq += (double)d.q0[b];
  }
  for (int o = 32; o > 0; o >>= 1) {
    sa += __shfl_xor(sa, o, 64);
    sq += __shfl_xor(sq, o, 64);
  }
  if (lane == 0) sd[wid] = sa;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int w = 0; w < (nt >> 6); ++w) t += sd[w];
    const float mabs = (float)(t / d.B);
    s_lam = d.bc ? __fdiv_rn(d.alpha, mabs) : 1.f;
  }
  __syncthreads();
  if (lane == 0) sd[wid] = sq;
  __syncthreads();
  const float lam = s_lam;
  if (tid == 0) {
    double t = 0.0;
    for (int w = 0; w < (nt >> 6); ++w) t += sd[w];
    d.scalars[0] = lam;
    d.scalars[1] = __fmul_rn(lam, -(float)(t / d.B));  // lam * -mean(q0)
  }
  const float g = __fdiv_rn(-lam, (float)d.B);
  for (int b = tid; b < d.B; b += nt) d.g[b] = g;
}

// dL/dh = (dQ0/da * 1 + d mse/da) * (1 - a^2); actor_loss metric (one workgroup)
__global__ __launch_bounds__(1024) void td3bc_actor_head_kernel(d3a_td3bc_actor_desc d) {
  __shared__ double sd[16];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int64_t n = (int64_t)d.B * d.A;
  const float gm = 1.f / (float)n;  // mean backward
  double s = 0.0;
  for (int64_t i = tid; i < n; i += nt) {
    const int64_t b = i / d.A;
    const int j = (int)(i - b * d.A);
    const float a = d.pi_act[i];
    const float g_q = d.dq_da[b * d.ld_da + d.da_off + j];
    float ga = g_q;
    if (d.bc) {
      const float diff = __fsub_rn(d.act[i], a);
      s += (double)__fmul_rn(diff, diff);
      // (actions - action) ** 2 -> d/d action = -(gm * 2 * diff)
      const float g_bc = -__fmul_rn(gm, __fmul_rn(2.f, diff));
      ga = __fadd_rn(g_q, g_bc);
    }
    d.dhead[i] = __fmul_rn(ga, __fsub_rn(1.f, __fmul_rn(a, a)));
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) sd[wid] = s;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int w = 0; w < (nt >> 6); ++w) t += sd[w];
    d.metrics[1] = d.bc ? __fadd_rn(d.scalars[1], (float)(t / (double)n)) : d.scalars[1];
  }
}

inline unsigned blocks256(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_td3_prep(const d3a_td3_prep_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->obs && d->next_obs && d->act && d->x_q && d->x_targ,
                "d3a_td3_prep: null pointer");
  D3A_CHECK_ARG(d->B >= 1 && d->D >= 1 && d->A >= 1 && d->ldx >= d->D + d->A,
                "d3a_td3_prep: bad sizes");
  D3A_CHECK_ARG(!d->mean || d->std, "d3a_td3_prep: mean without std");
  const int64_t n = (int64_t)d->B * (2 * d->D + d->A);
  hipLaunchKernelGGL(td3_prep_kernel, dim3(blocks256(n)), dim3(256), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_td3_prep");
  return 0;
}

extern "C" int d3a_td3_target(const d3a_td3_target_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->head && d->noise && d->x_targ, "d3a_td3_target: null pointer");
  D3A_CHECK_ARG(d->B >= 1 && d->A >= 1 && d->ldx >= d->D + d->A, "d3a_td3_target: bad sizes");
  hipLaunchKernelGGL(td3_target_kernel, dim3(blocks256((int64_t)d->B * d->A)), dim3(256), 0,
                     (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_td3_target");
  return 0;
}

extern "C" int d3a_td3_critic_loss(const d3a_td3_critic_loss_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->q && d->q_targ && d->rew && d->term && d->n_steps && d->dq && d->metrics,
                "d3a_td3_critic_loss: null pointer");
  D3A_CHECK_ARG(d->B >= 1 && d->C >= 1, "d3a_td3_critic_loss: bad sizes");
  hipLaunchKernelGGL(td3_critic_loss_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_td3_critic_loss");
  return 0;
}

extern "C" int d3a_td3bc_actor_input(const d3a_td3bc_actor_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->head && d->x_q && d->x_actor && d->pi_act,
                "d3a_td3bc_actor_input: null pointer");
  D3A_CHECK_ARG(d->B >= 1 && d->ldx >= d->D + d->A, "d3a_td3bc_actor_input: bad sizes");
  hipLaunchKernelGGL(td3bc_actor_input_kernel, dim3(blocks256((int64_t)d->B * (d->D + d->A))),
                     dim3(256), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_td3bc_actor_input");
  return 0;
}

extern "C" int d3a_td3bc_actor_seed(const d3a_td3bc_actor_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->q0 && d->g && d->scalars, "d3a_td3bc_actor_seed: null pointer");
  D3A_CHECK_ARG(d->B >= 1, "d3a_td3bc_actor_seed: bad sizes");
  hipLaunchKernelGGL(td3bc_actor_seed_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_td3bc_actor_seed");
  return 0;
}

extern "C" int d3a_td3bc_actor_head(const d3a_td3bc_actor_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->pi_act && d->act && d->dq_da && d->dhead && d->scalars && d->metrics,
                "d3a_td3bc_actor_head: null pointer");
  D3A_CHECK_ARG(d->B >= 1 && d->A >= 1 && d->ld_da >= d->da_off + d->A,
                "d3a_td3bc_actor_head: bad sizes");
  hipLaunchKernelGGL(td3bc_actor_head_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_td3bc_actor_head");
  return 0;
}
