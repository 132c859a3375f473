// Elementwise / reduction stages of the BCQ update (K3: continuous BCQ with
// quantile-regression critics).  The MLP layers run in mlp_fused.hip /
// gemm.hip; these kernels build their input rows and form the loss-side
// gradients between them.
//
// Reference (restated op for op, fp32):
//   ConditionalVAE.encode / decode / compute_error   models/torch/imitators.py:63-86
//   DeterministicResidualPolicy.forward               models/torch/policies.py:94-97
//   BCQImpl._sample_repeated_action / compute_target  algos/torch/bcq_impl.py:169-226
//   compute_max_with_n_actions                        models/torch/q_functions/__init__.py:8-72
//   quantile Huber loss                               models/torch/q_functions/utility.py:27-61
//   BCQImpl.compute_actor_loss                        algos/torch/bcq_impl.py:132-146
#include <algorithm>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

// a head value given as D3A_MLP_PARTS partial sums (d3a_mlp_fwd's parts path;
// part 0 holds the bias), summed in part order; np <= 1: the value itself
__device__ __forceinline__ float part_sum(const float* h, int64_t sp, int np, int64_t i) {
  if (np <= 1) return h[i];
  if (np == D3A_MLP_PARTS) {  // every load issued before the first add (same order)
    float v[D3A_MLP_PARTS];
#pragma unroll
    for (int p = 0; p < D3A_MLP_PARTS; ++p) v[p] = h[p * sp + i];
    float a = v[0];
#pragma unroll
    for (int p = 1; p < D3A_MLP_PARTS; ++p) a += v[p];
    return a;
  }
  float v = h[i];
  for (int p = 1; p < np; ++p) v += h[p * sp + i];
  return v;
}


// ---- input rows: x[r] = (obs[r / rep], f(a[r])) ----------------------------
__global__ __launch_bounds__(256) void bcq_rows_kernel(d3a_bcq_rows_desc d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int W = d.D + d.E;
  if (i >= d.rows * W) return;
  const int64_t r = i / W;
  const int j = (int)(i - r * W);
  if (j < d.D) {
    d.x[r * d.ldx + j] = d.obs[(r / d.rep) * d.D + j];
    return;
  }
  const int e = j - d.D;
  const float a = part_sum(d.a, d.s_a_part, d.a_parts, r * d.lda + e);
  float v;
  switch (d.mode) {
    case 1: v = fminf(fmaxf(a, -d.clip), d.clip); break;            // latent.clamp(-c, c)
    case 2: v = tanhf(a); break;                                      // decode: tanh(fc(h))
    case 3: {                                                         // residual policy
      const float res = __fmul_rn(d.scale, tanhf(a));
      v = fminf(fmaxf(__fadd_rn(d.base[r * d.E + e], res), -1.f), 1.f);
      break;
    }
    case 4: {                                    // residual policy on the raw decoder output
      const float res = __fmul_rn(d.scale, tanhf(a));
      v = fminf(fmaxf(__fadd_rn(tanhf(d.base[r * d.E + e]), res), -1.f), 1.f);
      break;
    }
    default: v = a;
  }
  d.x[r * d.ldx + j] = v;
  if (d.e_out) d.e_out[r * d.E + e] = v;
}

// ---- VAE encode + rsample + KL (one workgroup) ------------------------------
// head = [mu | logstd] per row; z = mu + eps * exp(clamp(logstd)); x_dec =
// (obs, z); KL(N(mu, std) || N(0, 1)) mean -> scalars[0]
__global__ __launch_bounds__(1024) void bcq_vae_sample_kernel(d3a_bcq_vae_desc d) {
  __shared__ double sd[16];
  const int t = threadIdx.x, nt = blockDim.x, lane = t & 63, wid = t >> 6;
  const int L = d.L;
  const int64_t n = (int64_t)d.B * L;
  double kl = 0.0;
  for (int64_t i = t; i < n; i += nt) {
    const int64_t b = i / L;
    const int j = (int)(i - b * L);
    const int npe = d.s_e_part ? d.head_parts : 1;
    const float mu = part_sum(d.head_e, d.s_e_part, npe, b * 2 * L + j);
    const float ls = fminf(fmaxf(part_sum(d.head_e, d.s_e_part, npe, b * 2 * L + L + j),
                                 d.min_logstd), d.max_logstd);
    const float sd_ = expf(ls);
    d.std_out[i] = sd_;
    // torch.distributions.kl: var_ratio = std^2, t1 = mu^2,
    // 0.5 * (var_ratio + t1 - 1 - log(var_ratio))
    const float vr = __fmul_rn(sd_, sd_);
    const float t1 = __fmul_rn(mu, mu);
    kl += (double)__fmul_rn(0.5f, __fsub_rn(__fsub_rn(__fadd_rn(vr, t1), 1.f), logf(vr)));
    const float z = __fadd_rn(mu, __fmul_rn(d.eps[i], sd_));
    d.x_dec[b * d.ldx + d.D + j] = z;
  }
  for (int64_t i = t; i < (int64_t)d.B * d.D; i += nt) {
    const int64_t b = i / d.D;
    const int j = (int)(i - b * d.D);
    d.x_dec[b * d.ldx + j] = d.obs[b * d.D + j];
  }
  for (int o = 32; o > 0; o >>= 1) kl += __shfl_xor(kl, o, 64);
  if (lane == 0) sd[wid] = kl;
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
    for (int w = 0; w < (nt >> 6); ++w) s += sd[w];
    d.scalars[0] = (float)(s / (double)n);
  }
}

// the same per element, one thread per (row, latent) and per obs element over
// many workgroups, the KL terms to d.kl (summed by bcq_vae_loss_kernel)
__global__ __launch_bounds__(256) void bcq_vae_sample_wide_kernel(d3a_bcq_vae_desc d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int L = d.L;
  const int64_t n = (int64_t)d.B * L;
  if (i < n) {
    const int64_t b = i / L;
    const int j = (int)(i - b * L);
    const int npe = d.s_e_part ? d.head_parts : 1;
    const float mu = part_sum(d.head_e, d.s_e_part, npe, b * 2 * L + j);
    const float ls = fminf(fmaxf(part_sum(d.head_e, d.s_e_part, npe, b * 2 * L + L + j),
                                 d.min_logstd), d.max_logstd);
    const float sd_ = expf(ls);
    d.std_out[i] = sd_;
    const float vr = __fmul_rn(sd_, sd_);
    const float t1 = __fmul_rn(mu, mu);
    d.kl[i] = __fmul_rn(0.5f, __fsub_rn(__fsub_rn(__fadd_rn(vr, t1), 1.f), logf(vr)));
    d.x_dec[b * d.ldx + d.D + j] = __fadd_rn(mu, __fmul_rn(d.eps[i], sd_));
  }
  if (i < (int64_t)d.B * d.D) {
    const int64_t b = i / d.D;
    const int j = (int)(i - b * d.D);
    d.x_dec[b * d.ldx + j] = d.obs[b * d.D + j];
  }
}

// ---- VAE decode loss: mse(tanh(head), a) + beta * KL (one workgroup) --------
__global__ __launch_bounds__(1024) void bcq_vae_loss_kernel(d3a_bcq_vae_desc d) {
  __shared__ double sd[16];
  const int t = threadIdx.x, nt = blockDim.x, lane = t & 63, wid = t >> 6;
  const int64_t n = (int64_t)d.B * d.A;
  const float gm = 1.f / (float)n;
  double s = 0.0;
  for (int64_t i = t; i < n; i += nt) {
    const float y = tanhf(part_sum(d.head_d, d.s_d_part, d.s_d_part ? d.head_parts : 1, i));
    const float diff = __fsub_rn(y, d.act[i]);
    s += (double)__fmul_rn(diff, diff);
    // mse backward: 2 (y - a) / n; tanh backward: * (1 - y^2)
    const float gy = __fmul_rn(__fmul_rn(2.f, diff), gm);
    d.dhead_d[i] = __fmul_rn(gy, __fsub_rn(1.f, __fmul_rn(y, y)));
  }
  // the KL mean from d.kl's terms (the wide sample kernel), same reduction order
  double k = 0.0;
  const int64_t nk = (int64_t)d.B * d.L;
  if (d.kl != nullptr)
    for (int64_t i = t; i < nk; i += nt) k += (double)d.kl[i];
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    k += __shfl_xor(k, o, 64);
  }
  __shared__ double sk[16];
  if (lane == 0) {
    sd[wid] = s;
    sk[wid] = k;
  }
  __syncthreads();
  if (t == 0) {
    double tot = 0.0, ktot = 0.0;
    for (int w = 0; w < (nt >> 6); ++w) {
      tot += sd[w];
      ktot += sk[w];
    }
    const float mse = (float)(tot / (double)n);
    const float klm = d.kl != nullptr ? (float)(ktot / (double)nk) : d.scalars[0];
    d.metrics[0] = __fadd_rn(mse, __fmul_rn(d.beta, klm));
  }
}

// ---- VAE encoder head gradient ---------------------------------------------
// dmu = dz + beta mu / (B L); dlogstd = (dz eps std + beta (std^2 - 1) / (B L))
// * [min_logstd <= logstd <= max_logstd]
__global__ __launch_bounds__(256) void bcq_vae_enc_grad_kernel(d3a_bcq_vae_desc d) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int L = d.L;
  const int64_t n = (int64_t)d.B * L;
  if (i >= n) return;
  const int64_t b = i / L;
  const int j = (int)(i - b * L);
  const float kscale = __fdiv_rn(d.beta, (float)n);
  const float dz = d.dx_dec[b * d.lddx + d.D + j];
  const int npe = d.s_e_part ? d.head_parts : 1;
  const float mu = part_sum(d.head_e, d.s_e_part, npe, b * 2 * L + j);
  const float lsr = part_sum(d.head_e, d.s_e_part, npe, b * 2 * L + L + j);
  const float sd_ = d.std_out[i];
  d.dhead_e[b * 2 * L + j] = __fadd_rn(dz, __fmul_rn(kscale, mu));
  const bool pass = lsr >= d.min_logstd && lsr <= d.max_logstd;
  const float g = __fadd_rn(__fmul_rn(__fmul_rn(dz, d.eps[i]), sd_),
                            __fmul_rn(kscale, __fsub_rn(__fmul_rn(sd_, sd_), 1.f)));
  d.dhead_e[b * 2 * L + L + j] = pass ? g : 0.f;
}

// ---- BCQ target: compute_max_with_n_actions over N sampled actions ---------
// q: [C][B*N][K] target-critic quantiles (row b*N + n); one workgroup of
// sixteen waves per b (the waves keep eight quantile rows each in flight)
constexpr int TG_T = 1024;
// wave 0: the argmax over n of the mix of the per-critic means sm[C][N] (the
// first n of the largest value, as a sequential strict-greater scan picks
// it; NaN never wins): each lane scans n = lane, lane + 64, .. in order, then
// the wave reduces (largest value, then smallest n)
__device__ __forceinline__ void tg_argmax(const float* sm, int C, int N, float lam, int lane, int* s_arg,
                                          int* s_cmax, int* s_cmin) {
  float best = -INFINITY;
  int arg = -1, bmax = 0, bmin = 0;
  for (int n = lane; n < N; n += 64) {
    float mx = sm[n], mn = sm[n];
    int cmx = 0, cmn = 0;
    for (int c = 1; c < C; ++c) {
      const float v = sm[c * N + n];
      if (v > mx) { mx = v; cmx = c; }
      if (v < mn) { mn = v; cmn = c; }
    }
    // mix_values = (1 - lam) * max_values + lam * min_values
    const float mix = __fadd_rn(__fmul_rn(1.f - lam, mx), __fmul_rn(lam, mn));
    if (mix > best) { best = mix; arg = n; bmax = cmx; bmin = cmn; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    const int ox = __shfl_xor(bmax, o, 64), on = __shfl_xor(bmin, o, 64);
    const bool take = oa >= 0 && (arg < 0 || ob > best || (ob == best && oa < arg));
    if (take) { best = ob; arg = oa; bmax = ox; bmin = on; }
  }
  if (lane == 0) { *s_arg = arg < 0 ? 0 : arg; *s_cmax = bmax; *s_cmin = bmin; }
}

__global__ __launch_bounds__(TG_T) void bcq_target_kernel(d3a_bcq_target_desc d) {
  extern __shared__ float sm[];  // [C][N] quantile means
  __shared__ int s_arg, s_cmax, s_cmin;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int64_t b = blockIdx.x;
  const int C = d.C, N = d.N, K = d.K;
  const int64_t BN = (int64_t)d.B * N;
  const int CN = C * N;
  if (d.means != nullptr) {
    // the target pass's epilogue formed the means (d3a_mlp_fwd_x6 row_mean)
    for (int p = t; p < CN; p += TG_T) {
      const int c = p / N, n = p - c * N;
      sm[p] = d.means[(int64_t)c * BN + b * N + n];
    }
  } else if (K <= 256) {
    // eight (c, n) rows per wave in flight (their loads issued before any
    // sum), each row summed exactly as below: lane l adds q[l], q[l + 64], ..
    // in order, then the wave butterfly -- bitwise the same means
    constexpr int PB = 8;
    for (int p0 = wid * PB; p0 < CN; p0 += (TG_T / 64) * PB) {
      float v[PB][4];
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        const int p = p0 + i < CN ? p0 + i : CN - 1;
        const int c = p / N, n = p - c * N;
        const float* q = d.q + ((int64_t)c * BN + b * N + n) * K;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = lane + 64 * u;
          v[i][u] = k < K ? q[k] : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < PB; ++i) {
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (lane + 64 * u < K) s += v[i][u];
        s = wave_sum(s);
        if (lane == 0 && p0 + i < CN) sm[p0 + i] = s / (float)K;  // values.mean(dim=3)
      }
    }
  } else {
    for (int p = wid; p < CN; p += TG_T / 64) {
      const int c = p / N, n = p - c * N;
      const float* q = d.q + ((int64_t)c * BN + b * N + n) * K;
      float s = 0.f;
      for (int k = lane; k < K; k += 64) s += q[k];
      s = wave_sum(s);
      if (lane == 0) sm[c * N + n] = s / (float)K;  // values.mean(dim=3)
    }
  }
  __syncthreads();
  if (wid == 0) tg_argmax(sm, C, N, d.lam, lane, &s_arg, &s_cmax, &s_cmin);
  __syncthreads();
  const float* qmax = d.q + ((int64_t)s_cmax * BN + b * N + s_arg) * K;
  const float* qmin = d.q + ((int64_t)s_cmin * BN + b * N + s_arg) * K;
  for (int k = t; k < K; k += TG_T)
    d.target[b * K + k] = __fadd_rn(__fmul_rn(1.f - d.lam, qmax[k]), __fmul_rn(d.lam, qmin[k]));
}

// ---- quantile Huber TD loss: one workgroup per (critic c, row b) ------------
// y_i = r + gamma^n * target_i * (1 - term); per quantile j of q:
//   l_j = sum_i |tau_j - [y_i - q_j < 0]| * huber(y_i - q_j)
// loss_cb = sum_j l_j / K; dL/dq_j = -(1/(B K)) sum_i w_ij * huber'(y_i - q_j)
// (tg_means set: the target row formed here, d3a_bcq_target's arithmetic on
// the target pass's means and quantiles, by every critic's workgroup of row b)
__global__ __launch_bounds__(256) void bcq_qr_loss_kernel(d3a_bcq_qr_desc d) {
  extern __shared__ float ys[];  // [K], then (tg_means) the means [tg_C][tg_N]
  __shared__ float scratch[16];
  __shared__ int s_arg, s_cmax, s_cmin;
  const int t = threadIdx.x;
  const int K = d.K;
  const int64_t c = blockIdx.y, b = blockIdx.x;
  // this thread's first quantile of q, loaded before the target rows (one
  // round trip fewer in front of the Huber loop)
  const float* q = d.q + (c * d.B + b) * K;
  const float qpre = q[t < K ? t : K - 1];
  const float gam = powf(d.gamma, d.n_steps[b]);
  const float nt = __fsub_rn(1.f, d.term[b]);
  if (d.tg_means != nullptr) {  // uniform
    float* sm = ys + K;
    const int TC = d.tg_C, TN = d.tg_N;
    const int64_t BN = (int64_t)d.B * TN;
    for (int p = t; p < TC * TN; p += 256) {
      const int cc = p / TN, n = p - cc * TN;
      sm[p] = d.tg_means[(int64_t)cc * BN + b * TN + n];
    }
    __syncthreads();
    if (t < 64) tg_argmax(sm, TC, TN, d.tg_lam, t, &s_arg, &s_cmax, &s_cmin);
    __syncthreads();
    const float* qmax = d.tg_q + ((int64_t)s_cmax * BN + b * TN + s_arg) * K;
    const float* qmin = d.tg_q + ((int64_t)s_cmin * BN + b * TN + s_arg) * K;
    for (int i = t; i < K; i += 256) {
      const float tg = __fadd_rn(__fmul_rn(1.f - d.tg_lam, qmax[i]), __fmul_rn(d.tg_lam, qmin[i]));
      ys[i] = __fadd_rn(d.rew[b], __fmul_rn(__fmul_rn(gam, tg), nt));
    }
  } else {
    for (int i = t; i < K; i += 256)
      ys[i] = __fadd_rn(d.rew[b], __fmul_rn(__fmul_rn(gam, d.target[b * K + i]), nt));
  }
  __syncthreads();
  const float gscale = -1.f / ((float)d.B * (float)K);
  float lsum = 0.f;
  for (int j = t; j < K; j += 256) {
    const float qj = j == t ? qpre : q[j];
    // taus = ((j + 1) / K + j / K) / 2
    const float tau = __fdiv_rn(__fadd_rn(__fdiv_rn((float)(j + 1), (float)K),
                                          __fdiv_rn((float)j, (float)K)), 2.f);
    float l = 0.f, g = 0.f;
    for (int i = 0; i < K; ++i) {
      const float diff = __fsub_rn(ys[i], qj);
      const float ad = fabsf(diff);
      const float w = fabsf(__fsub_rn(tau, diff < 0.f ? 1.f : 0.f));
      const float hub = ad < 1.f ? __fmul_rn(0.5f, __fmul_rn(diff, diff)) : __fsub_rn(ad, 0.5f);
      l += __fmul_rn(w, hub);
      const float hd = ad < 1.f ? diff : (diff < 0.f ? -1.f : 1.f);
      g = fmaf(w, hd, g);
    }
    lsum += l;
    d.dq[(c * d.B + b) * K + j] = __fmul_rn(g, gscale);
  }
  const float tot = block_sum(lsum, scratch);
  if (t == 0) d.loss_cb[c * d.B + b] = tot / (float)K;
}

// ---- actor head: -mean Q_0(s, pi(s, dec(s, z))) backward (one workgroup) ----
// a = clamp(a_dec + scale tanh(h), -1, 1);  dh = dq_da * [pass] * scale * (1 - tanh^2)
// also: critic_loss = sum_c mean_b loss_cb, actor_loss = -mean_b mean_k q0
__global__ __launch_bounds__(1024) void bcq_actor_head_kernel(d3a_bcq_actor_desc d) {
  __shared__ double sd[16];
  const int t = threadIdx.x, nt = blockDim.x, lane = t & 63, wid = t >> 6;
  const int64_t n = (int64_t)d.B * d.A;
  for (int64_t i = t; i < n; i += nt) {
    const int64_t b = i / d.A;
    const int j = (int)(i - b * d.A);
    const float th = tanhf(part_sum(d.head, d.s_head_part, d.head_parts, i));
    const float pre = __fadd_rn(d.a_dec[i], __fmul_rn(d.scale, th));
    const bool pass = pre >= -1.f && pre <= 1.f;
    const float ga = pass ? d.dq_da[b * d.ld_da + d.da_off + j] : 0.f;
    d.dhead[i] = __fmul_rn(__fmul_rn(ga, d.scale), __fsub_rn(1.f, __fmul_rn(th, th)));
  }
  // actor loss: Q_0 = mean over quantiles, then -mean over rows (16-byte
  // loads, four in flight per thread, summed in a fixed order)
  double s = 0.0;
  const int64_t nq = (int64_t)d.B * d.K;
  if ((reinterpret_cast<uintptr_t>(d.q0) & 15) == 0) {
    const float4* q4 = reinterpret_cast<const float4*>(d.q0);
    const int64_t n4 = nq / 4;
#pragma unroll 4
    for (int64_t i = t; i < n4; i += nt) {
      const float4 v = q4[i];
      s += (double)v.x;
      s += (double)v.y;
      s += (double)v.z;
      s += (double)v.w;
    }
    for (int64_t i = 4 * n4 + t; i < nq; i += nt) s += (double)d.q0[i];
  } else {
    for (int64_t i = t; i < nq; i += nt) s += (double)d.q0[i];
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) sd[wid] = s;
  __syncthreads();
  double tot = 0.0;
  if (t == 0)
    for (int w = 0; w < (nt >> 6); ++w) tot += sd[w];
  __syncthreads();
  double cl = 0.0;
  for (int64_t i = t; i < (int64_t)d.C * d.B; i += nt) cl += (double)d.loss_cb[i];
  for (int o = 32; o > 0; o >>= 1) cl += __shfl_xor(cl, o, 64);
  if (lane == 0) sd[wid] = cl;
  __syncthreads();
  if (t == 0) {
    double c2 = 0.0;
    for (int w = 0; w < (nt >> 6); ++w) c2 += sd[w];
    d.metrics[1] = (float)(c2 / (double)d.B);
    d.metrics[2] = -(float)(tot / ((double)d.B * d.K));
  }
}

inline unsigned blocks256(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_bcq_rows(const d3a_bcq_rows_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->obs && d->a && d->x, "d3a_bcq_rows: null pointer");
  D3A_CHECK_ARG(d->rep >= 1 && d->D >= 1 && d->E >= 1 && d->ldx >= d->D + d->E,
                "d3a_bcq_rows: bad sizes");
  D3A_CHECK_ARG(d->mode >= 0 && d->mode <= 4 && (d->mode < 3 || d->base),
                "d3a_bcq_rows: mode 0..4; modes 3 / 4 need base");
  if (d->rows <= 0) return 0;
  hipLaunchKernelGGL(bcq_rows_kernel, dim3(blocks256(d->rows * (d->D + d->E))), dim3(256), 0,
                     (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_bcq_rows");
  return 0;
}

extern "C" int d3a_bcq_vae_sample(const d3a_bcq_vae_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->head_e && d->eps && d->obs && d->x_dec && d->std_out && d->scalars,
                "d3a_bcq_vae_sample: null pointer");
  if (d->kl != nullptr) {
    const int64_t n = std::max((int64_t)d->B * d->L, (int64_t)d->B * d->D);
    hipLaunchKernelGGL(bcq_vae_sample_wide_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, *d);
  } else {
    hipLaunchKernelGGL(bcq_vae_sample_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, *d);
  }
  D3A_LAUNCH_CHECK("d3a_bcq_vae_sample");
  return 0;
}

extern "C" int d3a_bcq_vae_loss(const d3a_bcq_vae_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->head_d && d->act && d->dhead_d && d->metrics && d->scalars,
                "d3a_bcq_vae_loss: null pointer");
  hipLaunchKernelGGL(bcq_vae_loss_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_bcq_vae_loss");
  return 0;
}

extern "C" int d3a_bcq_vae_enc_grad(const d3a_bcq_vae_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->dx_dec && d->head_e && d->eps && d->std_out && d->dhead_e,
                "d3a_bcq_vae_enc_grad: null pointer");
  hipLaunchKernelGGL(bcq_vae_enc_grad_kernel, dim3(blocks256((int64_t)d->B * d->L)), dim3(256), 0,
                     (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_bcq_vae_enc_grad");
  return 0;
}

extern "C" int d3a_bcq_target(const d3a_bcq_target_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->q && d->target, "d3a_bcq_target: null pointer");
  D3A_CHECK_ARG(d->B >= 1 && d->N >= 1 && d->K >= 1 && d->C >= 1 && d->C * d->N <= 8192,
                "d3a_bcq_target: bad sizes");
  hipLaunchKernelGGL(bcq_target_kernel, dim3((unsigned)d->B), dim3(TG_T),
                     (size_t)d->C * d->N * sizeof(float), (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_bcq_target");
  return 0;
}

extern "C" int d3a_bcq_qr_loss(const d3a_bcq_qr_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->q && (d->target || d->tg_means) && d->rew && d->term && d->n_steps && d->dq &&
                    d->loss_cb,
                "d3a_bcq_qr_loss: null pointer");
  D3A_CHECK_ARG(d->K >= 1 && d->K <= 8192 && d->B >= 1 && d->C >= 1, "d3a_bcq_qr_loss: bad sizes");
  D3A_CHECK_ARG(d->tg_means == nullptr ||
                    (d->tg_q && d->tg_N >= 1 && d->tg_C >= 1 && d->tg_C * d->tg_N <= 8192),
                "d3a_bcq_qr_loss: the in-launch target needs tg_q and 1 <= tg_C tg_N <= 8192");
  size_t smem = ((size_t)d->K + (d->tg_means ? (size_t)d->tg_C * d->tg_N : 0)) * sizeof(float);
  // the dynamic LDS (K targets + the in-launch target's C N means) beside
  // the kernel's static arrays must fit the device's per-workgroup LDS (160
  // KB here; 64 KB on other parts): otherwise the target rows come from their
  // own launch (d3a_bcq_target into d->target) and the loss reads them
  static const size_t lds_max = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
      v = 65536;
    return (size_t)v;
  }();
  static const size_t lds_static = [] {
    hipFuncAttributes fa{};
    return hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&bcq_qr_loss_kernel)) == hipSuccess
               ? (size_t)fa.sharedSizeBytes
               : (size_t)0;
  }();
  d3a_bcq_qr_desc e = *d;
  if (d->tg_means && smem + lds_static > lds_max) {
    D3A_CHECK_ARG(d->target != nullptr,
                  "d3a_bcq_qr_loss: the in-launch target's LDS exceeds the device's; give target "
                  "(the rows are then formed by d3a_bcq_target first)");
    d3a_bcq_target_desc t{};
    t.q = d->tg_q;
    t.means = d->tg_means;
    t.target = const_cast<float*>(d->target);  // (written here, read by the loss below)
    t.B = d->B, t.N = d->tg_N, t.K = d->K, t.C = d->tg_C;
    t.lam = d->tg_lam;
    const int rc = d3a_bcq_target(&t, stream);
    if (rc != 0) return rc;
    e.tg_means = nullptr;
    smem = (size_t)d->K * sizeof(float);
  }
  D3A_CHECK_ARG(smem + lds_static <= lds_max, "d3a_bcq_qr_loss: K targets exceed the device's LDS");
  hipLaunchKernelGGL(bcq_qr_loss_kernel, dim3((unsigned)d->B, (unsigned)d->C), dim3(256), smem,
                     (hipStream_t)stream, e);
  D3A_LAUNCH_CHECK("d3a_bcq_qr_loss");
  return 0;
}

extern "C" int d3a_bcq_actor_head(const d3a_bcq_actor_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->head && d->a_dec && d->dq_da && d->dhead && d->q0 && d->loss_cb &&
                d->metrics, "d3a_bcq_actor_head: null pointer");
  hipLaunchKernelGGL(bcq_actor_head_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_bcq_actor_head");
  return 0;
}
