// Fused CQL / SAC stages of one conservative Q-learning update.
//
// Reference: d3rlpy/algos/torch/cql_impl.py (CQLImpl), sac_impl.py
// (SACImpl.update_temp / compute_actor_loss), models/torch/policies.py
// (SquashedNormalPolicy), models/torch/distributions.py
// (SquashedGaussianDistribution._log_prob_from_raw_y).
//
// The GEMM-heavy parts (policy and critic MLPs) run on gemm.hip; these
// kernels do the per-row sampling / log-prob / logsumexp / loss / gradient
// seeding work in between, so that the update never leaves the device and
// needs no host synchronisation.
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"

namespace d3a {
namespace {

constexpr float kLn2 = 0.69314718055994530942f;
// math.log(math.sqrt(2 * math.pi)) as the fp32 scalar torch uses
constexpr float kLogSqrt2Pi = 0.91893853320467274178f;

// SquashedGaussianDistribution sample + log-prob for one row:
//   std = exp(clamp(ls, lo, hi)); u = mu + eps * std; a = tanh(u)
//   logp = sum_j [Normal(mu, std).log_prob(u) - 2 (log 2 - u - softplus(-2u))]
// A head value: np partial sums at h + p * sp, summed in order (np = 1: one)
__device__ __forceinline__ float head_val(const float* h, int64_t sp, int np, int64_t j) {
  if (np == D3A_MLP_PARTS) {
    const float a = h[j], b = h[sp + j], c = h[2 * sp + j], e = h[3 * sp + j];
    return ((a + b) + c) + e;
  }
  float v = h[j];
  for (int p = 1; p < np; ++p) v += h[p * sp + j];
  return v;
}

// the head row hrow = (mu | logstd) of A + A values, given as np parts
__device__ __forceinline__ float squashed_sample(const float* hrow, int64_t sp, int np,
                                                 const float* eps, int A, float lo, float hi,
                                                 float* act, float* u_out) {
  float logp = 0.f;
  for (int j = 0; j < A; ++j) {
    const float muj = head_val(hrow, sp, np, j);
    const float l = fminf(fmaxf(head_val(hrow, sp, np, A + j), lo), hi);
    const float sd = expf(l);
    const float u = muj + eps[j] * sd;
    const float d = u - muj;
    const float var = sd * sd;
    const float lp = -(d * d) / (2.f * var) - logf(sd) - kLogSqrt2Pi;
    const float jac = 2.f * (kLn2 - u - softplus_t(-2.f * u));
    logp += lp - jac;
    if (act) act[j] = tanhf(u);
    if (u_out) u_out[j] = u;
  }
  return logp;
}

// One output row per four lanes, 64-row workgroups (the 15,872 rows of K2
// spread over ~250 CUs, four waves each).  Lane k of a row's quad takes the
// action components j = k, k + 4, .. (the Philox draw, the squashed-Gaussian
// term, tanh), so a row's serial transcendental chain is a quarter as long;
// the log-prob terms meet at lane 0 in j order (the sequential sum of
// squashed_sample, bitwise).  Rows are assembled in LDS (zero-padded to ldx)
// and leave as whole 16-byte pieces: a workgroup's rows of one destination
// matrix are contiguous, so the copy-out is fully coalesced.
constexpr int SMP_R = 64;       // rows per workgroup
constexpr int SMP_T = 4 * SMP_R;
constexpr int SMP_MAXLDX = 64;  // ldx handled by the LDS copy-out
__global__ __launch_bounds__(SMP_T) void cql_sample_kernel(d3a_cql_sample_desc d) {
  __shared__ float xs[SMP_R * (SMP_MAXLDX + 1)];
  const int64_t B = d.B, N = d.N, D = d.D;
  const int A = d.A;
  const int64_t NB = N * B;
  const int64_t DA = d.ldx;  // row stride of the Q-input matrices (>= D + A, padded)
  const int64_t R = 6 * NB + B;           // x_q rows
  const int64_t total = R + 3 * B;         // + temp, target, actor rows
  const int rl = threadIdx.x >> 2, k = threadIdx.x & 3;
  const int64_t i0 = (int64_t)blockIdx.x * SMP_R;
  const int64_t i = i0 + rl;
  constexpr int LS = SMP_MAXLDX + 1;  // LDS row stride
  float* const xl = xs + rl * LS;
  // the destination row of output row q (nullptr: no Q-input row)
  auto dest = [&](int64_t q) -> float* {
    if (q < R) return d.x_q + q * DA;
    if (q < R + B) return nullptr;
    if (q < R + 2 * B) return d.x_targ + (q - R - B) * DA;
    if (q < total) return d.x_actor + (q - R - 2 * B) * DA;
    return nullptr;
  };
  const int64_t H = 2 * A;                 // head row width
  // policy head rows (mu | logstd); with head_parts, the parts summed in order
  const int np = d.head_parts > 1 ? d.head_parts : 1;
  const int64_t sp = d.s_head_part;
  auto head_row = [&](int64_t row) { return d.head + row * H; };
  // the step's noise: drawn here from the Philox stream (gen_noise) or read
  // from the buffers the caller filled (parity mode)
  const uint64_t ctr = d.gen_noise ? (uint64_t)*d.rng_ctr : 0;
  auto noise1 = [&](const float* p) {
    return d.gen_noise ? philox_elem(d.seed, ctr, p - d.noise_base, d.n_normal, -1.f, 1.f) : *p;
  };
  // component j of a squashed-Gaussian sample (squashed_sample's loop body):
  // returns its log-prob term, writes tanh(u) and u
  auto comp = [&](const float* hrow, int j, float e, float& a, float& u) {
    const float muj = head_val(hrow, sp, np, j);
    const float l = fminf(fmaxf(head_val(hrow, sp, np, A + j), d.min_logstd), d.max_logstd);
    const float sd = expf(l);
    u = muj + e * sd;
    const float dd = u - muj;
    const float var = sd * sd;
    const float lp = -(dd * dd) / (2.f * var) - logf(sd) - kLogSqrt2Pi;
    const float jac = 2.f * (kLn2 - u - softplus_t(-2.f * u));
    a = tanhf(u);
    return lp - jac;
  };
  // the row's log-prob at lane 0 of the quad: terms t[j / 4] of lane j % 4,
  // summed in j order
  auto logp_sum = [&](const float* t) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float v = __shfl(t[j >> 2], (threadIdx.x & ~3) + (j & 3), 64);
      if (j < A) s = j == 0 ? v : s + v;
    }
    return s;
  };
  // copy D floats of an observation row into the LDS row (quad-strided)
  auto put_obs = [&](const float* o) {
    for (int64_t jj = k; jj < D; jj += 4) xl[jj] = o[jj];
  };
  float t[4] = {0.f, 0.f, 0.f, 0.f};
  // the step's critic weight images (d3a_x6_split jobs) for the critic
  // forward that follows: a thread's first piece is loaded here, ahead of its
  // row's loads, and split and stored after the row (one memory round trip
  // for both); pieces past the grid's threads (a grid smaller than the
  // images) follow in a loop
  const int64_t ps_tot = d.presplit.n_jobs > 0 ? x6::x6_split_total(d.presplit) : 0;
  const int64_t ps_p = (int64_t)blockIdx.x * SMP_T + threadIdx.x;
  x6::X6Piece ps_piece;
  if (ps_tot > 0) x6::x6_split_load(d.presplit, ps_p < ps_tot ? ps_p : ps_tot - 1, ps_piece);

  if (i >= total) {
    // past the last row: nothing (the copy-out skips it)
  } else if (i < 6 * NB) {
    const int64_t s = i / (3 * NB);        // 0 = alpha set, 1 = critic set
    const int64_t w = i % (3 * NB);
    const int64_t blk = w / NB;            // 0 pi(.|s_t), 1 pi(.|s_t+1), 2 uniform
    const int64_t r = w % NB;              // = b * N + n
    const int64_t b = r / N, n = r % N;
    put_obs(d.obs + b * D);
    if (blk < 2) {
      // policy rows: head row b (obs) or B + b (next_obs); noise [s][blk][n][b]
      const float* hrow = head_row(blk * B + b);
      const float* ep = d.eps_pi + (((s * 2 + blk) * N + n) * B + b) * A;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = k + 4 * q;
        if (j < A) {
          float a, u;
          t[q] = comp(hrow, j, noise1(ep + j), a, u);
          xl[D + j] = a;
        }
      }
      const float lp = logp_sum(t);
      if (k == 0) d.logp_is[(s * 2 + blk) * NB + r] = lp;
    } else {
      const float* up = d.u_rand + (s * NB + r) * A;
      for (int j = k; j < A; j += 4) xl[D + j] = noise1(up + j);
    }
  } else if (i < R) {
    // data rows (obs_t, a_t)
    const int64_t b = i - 6 * NB;
    put_obs(d.obs + b * D);
    for (int j = k; j < A; j += 4) xl[D + j] = d.act[b * A + j];
  } else if (i < R + B) {
    // update_temp sample: log-prob only
    const int64_t b = i - R;
    const float* hrow = head_row(b);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = k + 4 * q;
      if (j < A) {
        float a, u;
        t[q] = comp(hrow, j, noise1(d.eps_temp + b * A + j), a, u);
      }
    }
    const float lp = logp_sum(t);
    if (k == 0) d.logp_temp[b] = lp;
  } else if (i < R + 2 * B) {
    const int64_t b = i - R - B;
    const float* hrow = head_row(B + b);
    put_obs(d.next_obs + b * D);
    if (d.soft_target) {
      // SACImpl.compute_target: policy.sample_with_log_prob(next_obs)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = k + 4 * q;
        if (j < A) {
          float a, u;
          t[q] = comp(hrow, j, noise1(d.eps_targ + b * A + j), a, u);
          xl[D + j] = a;
        }
      }
      const float lp = logp_sum(t);
      if (k == 0) d.logp_targ[b] = lp;
    } else {
      // deterministic target action tanh(mu(s_t+1)) (NormalPolicy.best_action)
      for (int j = k; j < A; j += 4) xl[D + j] = tanhf(head_val(hrow, sp, np, j));
    }
  } else {
    // actor sample (rsample, with gradient later)
    const int64_t b = i - R - 2 * B;
    const float* hrow = head_row(b);
    put_obs(d.obs + b * D);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = k + 4 * q;
      if (j < A) {
        const float e = noise1(d.eps_actor + b * A + j);
        // the actor head (d3a_sac_actor_head) reads these draws again
        if (d.gen_noise) d.eps_actor_out[b * A + j] = e;
        float a, u;
        t[q] = comp(hrow, j, e, a, u);
        d.actor_u[b * A + j] = u;
        xl[D + j] = a;
      }
    }
    const float lp = logp_sum(t);
    if (k == 0) d.actor_logp[b] = lp;
  }
  // zero padding of the row (columns D + A .. ldx)
  for (int64_t jj = D + A + k; jj < DA; jj += 4) xl[jj] = 0.f;
  __syncthreads();
  // copy-out: 16-byte pieces, consecutive threads on consecutive pieces
  const int q4 = (int)(DA / 4);
  for (int e = threadIdx.x; e < SMP_R * q4; e += SMP_T) {
    const int r2 = e / q4, c4 = (e - r2 * q4) * 4;
    float* dst = dest(i0 + r2);
    if (dst == nullptr) continue;
    const float* sr = xs + r2 * LS + c4;
    *reinterpret_cast<float4*>(dst + c4) = make_float4(sr[0], sr[1], sr[2], sr[3]);
  }
  if (ps_p < ps_tot) x6::x6_split_store(ps_piece);
  for (int64_t p = ps_p + (int64_t)gridDim.x * SMP_T; p < ps_tot; p += (int64_t)gridDim.x * SMP_T)
    x6::x6_split_piece(d.presplit, p);
}

// logsumexp over the 3N importance-sampled values of (c, b) in set s.
__device__ __forceinline__ float is_value(const d3a_cql_loss_desc& d, int64_t c, int64_t s,
                                          int64_t b, int64_t j, float rand_logp) {
  const int64_t N = d.N, NB = (int64_t)d.N * d.B;
  const int64_t blk = j / N, n = j % N;
  const int64_t r = b * N + n;
  const float qv = d.q[c * d.R + s * 3 * NB + blk * NB + r];
  if (blk < 2) return qv - d.logp_is[(s * 2 + blk) * NB + r];
  return qv - rand_logp;
}

// Stage A (many waves): one wave per (sample set s, critic c, batch row b):
// lse[s][c][b] = logsumexp_j v_j over the 3N IS values (torch.logsumexp:
// amax shift, |max| == inf -> 0), and for the critic set the softmax
// weights exp(v_j - lse) = exp(v_j - max) / sum_j exp(v_j - max) into dq
// (scaled by the alpha-dependent factor in stage B).
__device__ __forceinline__ void cql_lse_wave(const d3a_cql_loss_desc& d, int64_t p, int lane) {
  const int64_t B = d.B, C = d.C, N = d.N, NB = N * B, M = 3 * N;
  if (p >= 2 * C * B) return;
  const int64_t s = p / (C * B), c = (p / B) % C, b = p % B;
  if (d.split && p == 0 && lane < 4) {
    // (split: the loss stage runs in the critic backward) the bias
    // corrections 1 - beta^t of the coming temperature / alpha Adam steps,
    // fp64 pow as cql_loss_stage computes them
    // (as the floats adam_scalar_r forms from them: lr / bc1, sqrt(bc2))
    const bool on = lane < 2 ? d.update_temp != 0 : d.update_alpha != 0;
    if (on) {
      const int64_t t = (lane < 2 ? *d.temp_step : *d.alpha_step) + 1;
      const double bc = 1.0 - pow((lane & 1) ? d.beta2 : d.beta1, (double)t);
      const double lr = lane < 2 ? d.temp_lr : d.alpha_lr;
      d.bc[lane] = (lane & 1) ? (double)(float)sqrt(bc) : (double)(float)(lr / bc);
    }
  }
  // (split, critic set) the data row's inputs, loaded with the logsumexp's
  // own loads and used after them (one memory round trip for both): lane k <
  // C the target Q of critic k, every lane the row's reward, terminal, n and Q
  const bool drow = d.split && s == 1;
  float dr_tq = 0.f, dr_rw = 0.f, dr_tm = 0.f, dr_ns = 0.f, dr_q = 0.f;
  if (drow) {
    dr_tq = d.q_targ[(lane < C ? lane : 0) * B + b];
    dr_rw = d.rew[b];
    dr_tm = d.term[b];
    dr_ns = d.n_steps[b];
    dr_q = d.q[c * d.R + 6 * NB + b];
  }
  if ((s == 0 && !d.update_alpha) || (s == 1 && !d.update_critic)) return;
  const float rand_logp = (float)log(pow(0.5, (double)d.A));
  if (M <= 64) {
    // (3N <= 64: one value a lane, loaded once -- the loops below reload it
    // for the max, the sum and the weights, three dependent round trips; the
    // same operations, so the same values)
    const float vj = lane < M ? is_value(d, c, s, b, lane, rand_logp) : -INFINITY;
    float mx = wave_max(vj);
    if (isinf(mx)) mx = 0.f;
    const float ej = lane < M ? expf(vj - mx) : 0.f;
    const float se = wave_sum(ej);
    const float l = logf(se) + mx;
    if (lane == 0) d.lse[(s * C + c) * B + b] = l;
    if (s == 1 && lane < M) {
      const int64_t blk = lane / N, n = lane % N;
      d.dq[c * d.R + 3 * NB + blk * NB + b * N + n] = __fdiv_rn(ej, se);
    }
  } else {
  float mx = -INFINITY;
  for (int64_t j = lane; j < M; j += 64) mx = fmaxf(mx, is_value(d, c, s, b, j, rand_logp));
  mx = wave_max(mx);
  if (isinf(mx)) mx = 0.f;
  float se = 0.f;
  for (int64_t j = lane; j < M; j += 64) se += expf(is_value(d, c, s, b, j, rand_logp) - mx);
  se = wave_sum(se);
  const float l = logf(se) + mx;
  if (lane == 0) d.lse[(s * C + c) * B + b] = l;
  if (s == 1) {
    // softmax weight exp(v_j - lse) formed as exp(v_j - max) / sum: the same
    // value without lse's absolute rounding (eps |lse|, shared by every j)
    // scaling all 3N weights -- that shared error survives the cancellation of
    // the sampled and data rows in the head-bias / hidden-layer gradients
    for (int64_t j = lane; j < M; j += 64) {
      const int64_t blk = j / N, n = j % N;
      d.dq[c * d.R + 3 * NB + blk * NB + b * N + n] =
          __fdiv_rn(expf(is_value(d, c, 1, b, j, rand_logp) - mx), se);
    }
  }
  }  // M > 64
  if (drow) {
    // the data row's gradient without the conservative term (subtracted by
    // the backward, which knows the new alpha) and its squared TD error --
    // cql_loss_stage's arithmetic for row 6NB + b (the min over the critics
    // in k order)
    float tq = __shfl(dr_tq, 0, 64);
    for (int64_t k = 1; k < C; ++k) {
      const float v = k < 64 ? __shfl(dr_tq, (int)k, 64) : d.q_targ[k * B + b];
      tq = fminf(tq, v);
    }
    if (lane == 0) {
      const float gam = powf(d.gamma, dr_ns);
      const float y = dr_rw + gam * tq * (1.f - dr_tm);
      const float diff = dr_q - y;
      d.dq[c * d.R + 6 * NB + b] = 2.f * diff / (float)B;
      d.td2[c * B + b] = diff * diff;
    }
  }
}

__global__ __launch_bounds__(256) void cql_lse_kernel(d3a_cql_loss_desc d) {
  cql_lse_wave(d, (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), threadIdx.x & 63);
}

// Stage B (one workgroup): temperature and alpha Adam steps, TD loss, and
// final dL/dQ (scales stage A's softmax weights by the new clipped alpha).
// Latency-bound (one CU): every input is loaded up front — the per-row values
// into registers (LOSS_MP slots per thread, the same p = tid + i * nt order
// the sums use), the scalar optimiser states by thread 0 — so the stage pays
// about one global round trip instead of one per phase.  Ensembles x batches
// beyond LOSS_MP * 1024 rows (REG = false) read the per-row values where they
// are used, in the same p = tid + i * nt order (identical sums).
constexpr int LOSS_MP = 8;

template <bool REG>
__device__ __forceinline__ void cql_loss_stage(const d3a_cql_loss_desc& d) {
  __shared__ float scratch[48];  // block_sum_k<3> over 16 waves
  __shared__ float sh[4];
  __shared__ double s_bc[4];
  const int tid = threadIdx.x, nt = blockDim.x;
  const int64_t B = d.B, C = d.C, N = d.N, NB = N * B, CB = C * B;
  const int phase = d.dp_phase;
  const bool temp_on = d.update_temp != 0, alpha_on = d.update_alpha != 0;
  const bool critic_on = d.update_critic != 0 && phase != 1;
  const bool cons_on = d.conservative != 0;

  // ---- prefetch ----
  // Adam bias corrections 1 - beta^t (fp64 pow, as torch computes them in
  // Python floats), one per wave so the four library pows run concurrently
  {
    const int w = tid >> 6;
    if ((tid & 63) == 0 && w < 4 && phase != 1 && (w < 2 ? temp_on : alpha_on)) {
      const int64_t t = (w < 2 ? *d.temp_step : *d.alpha_step) + 1;
      s_bc[w] = 1.0 - pow((w & 1) ? d.beta2 : d.beta1, (double)t);
    }
  }
  float r_lseA[LOSS_MP], r_qd[LOSS_MP], r_lseC[LOSS_MP], r_tq[LOSS_MP], r_rw[LOSS_MP],
      r_tm[LOSS_MP], r_ns[LOSS_MP];
  float ltemp = 0.f, tm_ = 0.f, tv_ = 0.f, lalpha = 0.f, am_ = 0.f, av_ = 0.f;
  int64_t tstep = 0, astep = 0;  // the optimisers' step counts (thread 0)
  if (tid == 0) {
    ltemp = *d.log_temp;
    lalpha = *d.log_alpha;
    // (read here with the other scalars: the increments below would otherwise
    // reload them behind the state stores, a dependent round trip each)
    if (temp_on) { tm_ = *d.temp_m; tv_ = *d.temp_v; tstep = *d.temp_step; }
    if (alpha_on) { am_ = *d.alpha_m; av_ = *d.alpha_v; astep = *d.alpha_step; }
  }
  float s_temp = 0.f;
  if (temp_on && phase != 2)
    for (int64_t b = tid; b < B; b += nt) s_temp += d.logp_temp[b] - (float)d.A;
  // the per-row inputs of row p = c * B + b (slot i of REG's registers)
  auto load_row = [&](int i, int64_t p) {
    r_lseA[i] = r_qd[i] = r_lseC[i] = r_tq[i] = r_rw[i] = r_tm[i] = r_ns[i] = 0.f;
    if (p >= CB) return;
    const int64_t c = p / B, b = p % B;
    if ((alpha_on && phase != 2) || critic_on) r_qd[i] = d.q[c * d.R + 6 * NB + b];
    if (alpha_on && phase != 2) r_lseA[i] = d.lse[c * B + b];
    if (critic_on) {
      float tq = d.q_targ[b];
      for (int64_t k = 1; k < C; ++k) tq = fminf(tq, d.q_targ[k * B + b]);
      r_tq[i] = tq;
      r_rw[i] = d.rew[b];
      r_tm[i] = d.term[b];
      r_ns[i] = d.n_steps[b];
      if (cons_on) r_lseC[i] = d.lse[(C + c) * B + b];
    }
  };
  // row slots per thread: LOSS_MP registers, or (REG false) one register
  // reused for every p = tid + i * nt < CB
  const int n_slot = REG ? LOSS_MP : (int)((CB + nt - 1) / nt);
  if constexpr (REG) {
#pragma unroll
    for (int i = 0; i < LOSS_MP; ++i) load_row(i, tid + (int64_t)i * nt);
  }
  auto slot = [&](int i) -> int {  // register index holding slot i's row
    if constexpr (REG) {
      return i;
    } else {
      load_row(0, tid + (int64_t)i * nt);
      return 0;
    }
  };
  __syncthreads();  // s_bc

  // the temperature's and alpha's block sums in one barrier pair (each in
  // block_sum's order)
  float tsum = 0.f, alsum = 0.f, adsum = 0.f;
  if (phase != 2 && (temp_on || alpha_on)) {
    float sl = 0.f, sd = 0.f;
    if (alpha_on) {
#pragma unroll
      for (int i = 0; i < (REG ? LOSS_MP : 1); ++i) {
        if (REG) {
          sl += r_lseA[i];
          sd += r_qd[i];
        } else {
          for (int k = 0; k < n_slot; ++k) {
            const int j = slot(k);
            sl += r_lseA[j];
            sd += r_qd[j];
          }
        }
      }
    }
    float v3[3] = {s_temp, sl, sd};
    block_sum_k<3>(v3, scratch);
    tsum = v3[0];
    alsum = v3[1];
    adsum = v3[2];
  }

  // ---- update_temp (sac_impl.py:123-146) ----
  if (temp_on) {
    if (tid == 0) {
      float g = 0.f;
      if (phase != 2) {
        const float e = expf(ltemp);
        // loss = -(exp(log_temp) * targ_temp).mean()
        d.metrics[0] = -(e * tsum) / (float)B;
        g = (-1.f / (float)B) * tsum * e;
      }
      if (phase == 1) {
        d.scalar_grads[0] = g;
      } else {
        if (phase == 2) g = d.scalar_grads[0] * d.grad_scale;
        float* pm = d.temp_m; float* pv = d.temp_v;
        const float ln = adam_scalar_r(ltemp, tm_, tv_, g, d.temp_lr, d.beta1, d.beta2,
                                       d.adam_eps, s_bc);
        *pm = tm_; *pv = tv_; *d.log_temp = ln; *d.temp_step = tstep + 1;
        ltemp = ln;
        d.metrics[1] = expf(ln);
      }
    }
  }

  // ---- update_alpha (cql_impl.py:119-141) on sample set 0 ----
  if (alpha_on) {
    if (tid == 0) {
      float g = 0.f;
      if (phase != 2) {
        const float loss = alsum / (float)CB - adsum / (float)CB;
        const float scaled = d.conservative_weight * loss;
        const float e = expf(lalpha);
        const float ca = fminf(fmaxf(e, 0.f), 1e6f);
        const float cons = ca * (scaled - d.alpha_threshold);
        const bool pass = (e >= 0.f) && (e <= 1e6f);
        g = pass ? -(scaled - d.alpha_threshold) * e : 0.f;
        d.metrics[2] = -cons;
      }
      if (phase == 1) {
        d.scalar_grads[1] = g;
      } else {
        if (phase == 2) g = d.scalar_grads[1] * d.grad_scale;
        float* pm = d.alpha_m; float* pv = d.alpha_v;
        const float ln = adam_scalar_r(lalpha, am_, av_, g, d.alpha_lr, d.beta1, d.beta2,
                                       d.adam_eps, s_bc + 2);
        *pm = am_; *pv = av_; *d.log_alpha = ln; *d.alpha_step = astep + 1;
        lalpha = ln;
        d.metrics[3] = expf(ln);
      }
    }
  }
  if (phase == 1) return;
  if (tid == 0) {
    sh[0] = fminf(fmaxf(expf(lalpha), 0.f), 1e6f);
    sh[1] = expf(ltemp);  // the temperature after update_temp
    d.scalars[0] = sh[1];
    d.scalars[1] = sh[0];
  }
  __syncthreads();
  const float ca = sh[0];
  const float temp = sh[1];

  if (!critic_on) return;
  // ---- update_critic loss and dL/dQ (ddpg_impl.py:138-165, cql_impl.py:110-117) ----
  const float gcons = cons_on ? ca * d.conservative_weight / (float)CB : 0.f;
  float s_td = 0.f, s_l = 0.f, s_d = 0.f;
#pragma unroll
  for (int k = 0; k < (REG ? LOSS_MP : 1); ++k) for (int i0 = 0; i0 < (REG ? 1 : n_slot); ++i0) {
    const int si = REG ? k : i0;
    const int64_t p = tid + (int64_t)si * nt;
    if (p >= CB) continue;
    const int i = slot(si);
    const int64_t c = p / B, b = p % B;
    float tq = r_tq[i];
    // soft backup: target - exp(log_temp) * log_prob (sac_impl.py:156-162)
    if (d.soft_target) tq = tq - temp * d.logp_targ[b];
    const float gam = powf(d.gamma, r_ns[i]);
    const float y = r_rw[i] + gam * tq * (1.f - r_tm[i]);
    const float qd = r_qd[i];
    const float diff = qd - y;
    s_td += diff * diff;
    s_d += qd;
    if (cons_on) s_l += r_lseC[i];
    d.dq[c * d.R + 6 * NB + b] = 2.f * diff / (float)B - gcons;
  }
  // critic-set IS rows keep the unscaled softmax weights of stage A; the
  // backward (d3a_head1_bwd) multiplies them by scalars[2] = gcons on read.
  if (tid == 0) d.scalars[2] = gcons;
  float v3[3] = {s_td, s_l, s_d};
  block_sum_k<3>(v3, scratch);
  const float td = v3[0] / (float)B;
  const float lsum = v3[1];
  const float dsum = v3[2];
  if (tid == 0) {
    const float loss = lsum / (float)CB - dsum / (float)CB;
    const float cons = cons_on ? ca * (d.conservative_weight * loss - d.alpha_threshold) : 0.f;
    d.metrics[4] = cons_on ? td + cons : td;
    d.metrics[6] = td;
    d.metrics[7] = cons;
  }
}

template <bool REG>
__global__ __launch_bounds__(1024) void cql_loss_kernel(d3a_cql_loss_desc d) {
  cql_loss_stage<REG>(d);
}

// Stages A and B in one launch (d.ticket set): 1,024-thread workgroups run
// stage A one wave per (s, c, b); each then counts itself done on the ticket
// (after a device-scope fence of its lse / softmax-weight writes) and the last
// one runs stage B -- the same 1,024-thread block as cql_loss_kernel, so the
// same sums in the same order -- and resets the ticket for the next launch
template <bool REG>
__global__ __launch_bounds__(1024) void cql_lse_loss_kernel(d3a_cql_loss_desc d) {
  __shared__ int s_last;
  cql_lse_wave(d, (int64_t)blockIdx.x * 16 + (threadIdx.x >> 6), threadIdx.x & 63);
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(d.ticket, 1u) == gridDim.x - 1 ? 1 : 0;
  __syncthreads();
  if (!s_last) return;
  __threadfence();  // every other workgroup's stage-A writes are visible
  if (threadIdx.x == 0) *d.ticket = 0u;
  cql_loss_stage<REG>(d);
}

__global__ __launch_bounds__(256) void sac_actor_dq_kernel(const float* q, int64_t sqc, int C,
                                                           int B, float* dq, int64_t sdq) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  int arg = 0;
  float mn = q[b];
  for (int c = 1; c < C; ++c) {
    const float v = q[c * sqc + b];
    if (v < mn) { mn = v; arg = c; }
  }
  for (int c = 0; c < C; ++c) dq[c * sdq + b] = (c == arg) ? -1.f / (float)B : 0.f;
}

// Workgroups 0..B-1: one batch row b each -- the policy-head gradient of row
// b (threads j < A), then, when dz is given, the head's input gradient
// dz[b][n] = (sum_k dhead[b][k] W_head[k][n]) * [h[b][n] > 0] for the trunk
// backward (autograd of the `_mu` / `_logstd` Linear layers, policies.py:
// 170-176; thread n, H <= 256, operands loaded before the head math).
// Workgroup B: the actor loss mean(exp(log_temp) * logp - min_c Q) into
// metrics[5] (rows summed in a fixed order).
// DQZ: dQ/da formed here from dq_dz (the first layer's action columns staged
// in 32 KB of LDS); otherwise read from dq_da and no LDS is reserved for it
template <bool DQZ>
__global__ __launch_bounds__(256) void sac_actor_head_kernel(d3a_sac_actor_head_desc d) {
  __shared__ float scratch[4];
  __shared__ float s_dh[32];
  __shared__ float s_dq[DQZ ? 4 : 1][64];  // per-wave dQ_c/da_j sums [wave][c * 16 + j]
  __shared__ float s_w0[DQZ ? 32 * 256 : 1];  // the first layer's action columns [c * A + j][k]
  const int tid = threadIdx.x;
  const int A = d.A, B = d.B, C = d.C;
  const int64_t b = blockIdx.x;
  const float et = d.scalars[0];
  // Q_c(r): the parts of d3a_sac_actor_q summed in order (dq_min), else one value
  const int np = d.dq_min ? d.n_part : 1;
  auto qv = [&](int c, int64_t r) {
    float v = d.q[c * d.sqc + r];
    for (int p = 1; p < np; ++p) v += d.q[p * d.sq_part + c * d.sqc + r];
    return v;
  };
  if (b == B) {
    float lsum = 0.f;
    for (int r = tid; r < B; r += blockDim.x) {
      float qmin = qv(0, r);
      for (int c = 1; c < C; ++c) qmin = fminf(qmin, qv(c, r));
      lsum += et * d.logp[r] - qmin;
    }
    const float tot = block_sum(lsum, scratch);
    if (tid == 0) d.metrics[5] = tot / (float)B;
    return;
  }
  const float dlogp = et / (float)B;
  const float* hrow = d.head + b * 2 * A;
  const int hp = d.head_parts > 1 ? d.head_parts : 1;
  // input-gradient operands of this thread's column
  const bool col = d.dz != nullptr && tid < d.H;
  float hv = 0.f, wk[32];
  if (col) {
    hv = d.h[b * d.ldh + tid];
    for (int k = 0; k < 2 * A; ++k) wk[k] = d.w_head[(int64_t)k * d.H + tid];
  }
  if constexpr (DQZ) {
    // dQ_c/da_j = sum_k dz0[c][b][k] w0[c][k][da_off + j].  The P = C*A weight
    // columns go to LDS (every workgroup reads the same few KB from L2), then
    // thread k's product of each pair (c, j) is summed per wave by a fixed
    // butterfly and the four wave sums are added in order.
    const int P = C * A, H0 = d.H0;
    const int n_w = P * H0;
#pragma unroll 8
    for (int e = tid; e < n_w; e += 256) {
      const int c = e / (H0 * A), r = e - c * (H0 * A), k = r / A, j = r - k * A;
      s_w0[(c * A + j) * 256 + k] = d.w0[c * d.sw0_c + (int64_t)k * d.ldw0 + d.da_off + j];
    }
    const int k = tid < H0 ? tid : H0 - 1;
    const float live = tid < H0 ? 1.f : 0.f;
    float zv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) zv[c] = d.dq_dz[(c < C ? c : C - 1) * d.sdz_c + b * d.lddqz + k];
    __syncthreads();
    const int w = tid >> 6, lane = tid & 63;
    for (int p = 0; p < P; ++p) {
      const int c = p / A, j = p - c * A;
      const float z = c == 0 ? zv[0] : c == 1 ? zv[1] : c == 2 ? zv[2] : zv[3];
      float v = live * __fmul_rn(z, s_w0[p * 256 + k]);
      for (int o = 32; o > 0; o >>= 1) v = __fadd_rn(v, __shfl_xor(v, o, 64));
      if (lane == 0) s_dq[w][c * 16 + j] = v;
    }
    __syncthreads();
  }
  if (tid < A) {
    const int j = tid;
    float da = 0.f;
    if constexpr (DQZ) {
      for (int c = 0; c < C; ++c) {
        const float* sc = &s_dq[0][c * 16 + j];
        da += ((sc[0] + sc[64]) + sc[128]) + sc[192];
      }
    } else if (d.dq_min && C <= 4 && np <= 4) {
      // backward of min over the members: the first member of least q
      // (head1_min's rule) carries dq_scale, the others nothing.  Every
      // member's dQ/da parts are loaded with the q parts (one round trip,
      // not q then the chosen member's parts), then the chosen one is summed
      float jpart[4][4], qpart[4][4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const bool on = c < C && p < np;
          jpart[c][p] = on ? d.dq_da[p * d.sda_part + c * d.sda_c + b * d.ld_da + d.da_off + j] : 0.f;
          qpart[c][p] = on ? d.q[p * d.sq_part + c * d.sqc + b] : 0.f;
        }
      auto qsum = [&](int c) {
        float v = qpart[c][0];
        for (int p = 1; p < np; ++p) v += qpart[c][p];
        return v;
      };
      int arg = 0;
      float mn = qsum(0);
#pragma unroll
      for (int c = 1; c < 4; ++c) {
        if (c >= C) break;
        const float v = qsum(c);
        if (v < mn) { mn = v; arg = c; }
      }
      float jv = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c != arg) continue;
        jv = jpart[c][0];
        for (int p = 1; p < np; ++p) jv += jpart[c][p];
      }
      da = d.dq_scale * jv;
    } else if (d.dq_min) {
      int arg = 0;
      float mn = qv(0, b);
      for (int c = 1; c < C; ++c) {
        const float v = qv(c, b);
        if (v < mn) { mn = v; arg = c; }
      }
      const float* jp = d.dq_da + arg * d.sda_c + b * d.ld_da + d.da_off + j;
      float jv = jp[0];
      for (int p = 1; p < np; ++p) jv += jp[p * d.sda_part];
      da = d.dq_scale * jv;
    } else {
      for (int c = 0; c < C; ++c) da += d.dq_da[c * d.sda_c + b * d.ld_da + d.da_off + j];
    }
    const float mu = head_val(hrow, d.s_head_part, hp, j);
    const float lsr = head_val(hrow, d.s_head_part, hp, A + j);
    const float l = fminf(fmaxf(lsr, d.min_logstd), d.max_logstd);
    const float sd = expf(l);
    const float u = d.u[b * A + j];
    const float e = d.eps[b * A + j];
    const float th = tanhf(u);
    const float dm = u - mu;
    const float var = sd * sd;
    // d logp / d u (direct): -(u-mu)/var + 2 - 4 sigmoid(-2u)
    const float dlp_du = -dm / var + 2.f - 4.f * sigmoidf_t(-2.f * u);
    const float du = da * (1.f - th * th) + dlogp * dlp_du;
    const float dmu = du + dlogp * (dm / var);
    const float dsd = du * e + dlogp * ((dm * dm) / (var * sd) - 1.f / sd);
    const bool pass = (lsr >= d.min_logstd) && (lsr <= d.max_logstd);
    const float dls = pass ? dsd * sd : 0.f;
    d.dhead[b * 2 * A + j] = dmu;
    d.dhead[b * 2 * A + A + j] = dls;
    s_dh[j] = dmu;
    s_dh[A + j] = dls;
  }
  if (d.dz == nullptr) return;
  __syncthreads();
  if (col) {
    float v = 0.f;
    for (int k = 0; k < 2 * A; ++k) v = fmaf(s_dh[k], wk[k], v);
    d.dz[b * d.lddz + tid] = hv > 0.f ? v : 0.f;
    // this row's partial of the head weight gradient dW[k][n] = dhead[k] h[n]
    if (d.dW_part) {
      float* pw = d.dW_part + b * 2 * A * d.H + tid;
      for (int k = 0; k < 2 * A; ++k) pw[(int64_t)k * d.H] = s_dh[k] * hv;
    }
  }
  if (d.db_part && tid < 2 * A) d.db_part[b * 2 * A + tid] = s_dh[tid];
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_cql_sample(const d3a_cql_sample_desc* d, void* stream) {
  D3A_CHECK_ARG(d, "d3a_cql_sample: null desc");
  D3A_CHECK_ARG(d->A >= 1 && d->A <= 16, "d3a_cql_sample: action size must be in [1,16]");
  D3A_CHECK_ARG(d->B >= 1 && d->N >= 0 && d->D >= 1, "d3a_cql_sample: bad sizes");
  D3A_CHECK_ARG(!d->soft_target || (d->eps_targ && d->logp_targ),
                "d3a_cql_sample: soft_target needs eps_targ and logp_targ");
  D3A_CHECK_ARG(d->ldx >= d->D + d->A, "d3a_cql_sample: ldx < D + A");
  D3A_CHECK_ARG(!d->gen_noise || (d->noise_base && d->rng_ctr && d->eps_actor_out),
                "d3a_cql_sample: gen_noise needs noise_base, rng_ctr and eps_actor_out");
  D3A_CHECK_ARG(d->ldx % 4 == 0 && d->ldx <= SMP_MAXLDX,
                "d3a_cql_sample: ldx must be a multiple of 4 and <= 64");
  D3A_CHECK_ARG((reinterpret_cast<uintptr_t>(d->x_q) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(d->x_targ) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(d->x_actor) & 15) == 0,
                "d3a_cql_sample: x_q / x_targ / x_actor must be 16-byte aligned");
  D3A_CHECK_ARG(x6::x6_split_ok(d->presplit),
                "d3a_cql_sample: presplit jobs need src, 16-byte aligned dst, 1 <= k <= kpad, "
                "kpad % 16 == 0");
  const int64_t total = 6LL * d->N * d->B + 4LL * d->B;
  hipLaunchKernelGGL(cql_sample_kernel, dim3((unsigned)((total + SMP_R - 1) / SMP_R)), dim3(SMP_T), 0,
                     (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_cql_sample");
  return 0;
}

extern "C" int d3a_cql_loss(const d3a_cql_loss_desc* d, void* stream) {
  D3A_CHECK_ARG(d, "d3a_cql_loss: null desc");
  D3A_CHECK_ARG(d->R == 6LL * d->N * d->B + d->B, "d3a_cql_loss: R must be 6NB+B");
  D3A_CHECK_ARG(d->lse != nullptr, "d3a_cql_loss: lse workspace required");
  D3A_CHECK_ARG(d->dp_phase >= 0 && d->dp_phase <= 2, "d3a_cql_loss: bad dp_phase");
  D3A_CHECK_ARG(d->dp_phase == 0 || d->scalar_grads != nullptr,
                "d3a_cql_loss: dp_phase needs scalar_grads");
  D3A_CHECK_ARG(!d->soft_target || d->logp_targ, "d3a_cql_loss: soft_target needs logp_targ");
  D3A_CHECK_ARG(d->conservative || !d->update_alpha,
                "d3a_cql_loss: update_alpha needs the conservative term");
  D3A_CHECK_ARG(!d->conservative || d->N >= 1, "d3a_cql_loss: the conservative term needs N >= 1");
  D3A_CHECK_ARG(!d->split || (d->conservative && d->update_critic && !d->soft_target &&
                               d->dp_phase == 0 && d->td2 && d->bc && d->stage && !d->ticket),
                "d3a_cql_loss: split needs the conservative critic update on one device, no soft "
                "target, td2, bc and stage");
  if (d->split) {
    // the logsumexp stage only (with the data rows' gradients, td2, bc); the
    // loss stage runs in d3a_q2_bwd_x6_cql
    const int64_t waves = 2LL * d->C * d->B;
    hipLaunchKernelGGL(cql_lse_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, *d);
    D3A_LAUNCH_CHECK("d3a_cql_loss");
    return 0;
  }
  // phase 2 reuses the logsumexp / softmax weights phase 1 wrote
  const bool stage_a = d->conservative && (d->update_alpha || d->update_critic) && d->dp_phase != 2;
  if (stage_a && d->ticket) {
    const int64_t waves = 2LL * d->C * d->B;
    const dim3 g((unsigned)((waves + 15) / 16));
    if ((int64_t)d->C * d->B <= (int64_t)LOSS_MP * 1024)
      hipLaunchKernelGGL(cql_lse_loss_kernel<true>, g, dim3(1024), 0, (hipStream_t)stream, *d);
    else
      hipLaunchKernelGGL(cql_lse_loss_kernel<false>, g, dim3(1024), 0, (hipStream_t)stream, *d);
    D3A_LAUNCH_CHECK("d3a_cql_loss");
    return 0;
  }
  if (stage_a) {
    const int64_t waves = 2LL * d->C * d->B;
    hipLaunchKernelGGL(cql_lse_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, *d);
  }
  if ((int64_t)d->C * d->B <= (int64_t)LOSS_MP * 1024)
    hipLaunchKernelGGL(cql_loss_kernel<true>, dim3(1), dim3(1024), 0, (hipStream_t)stream, *d);
  else
    hipLaunchKernelGGL(cql_loss_kernel<false>, dim3(1), dim3(1024), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_cql_loss");
  return 0;
}

extern "C" int d3a_sac_actor_dq(const float* q, int64_t sqc, int32_t C, int32_t B, float* dq,
                                int64_t sdq, void* stream) {
  D3A_CHECK_ARG(q && dq && C >= 1 && B >= 1, "d3a_sac_actor_dq: bad args");
  hipLaunchKernelGGL(sac_actor_dq_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, q, sqc, C, B, dq, sdq);
  D3A_LAUNCH_CHECK("d3a_sac_actor_dq");
  return 0;
}

extern "C" int d3a_sac_actor_head(const d3a_sac_actor_head_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->B >= 1 && d->A >= 1 && d->A <= 16 && d->C >= 1,
                "d3a_sac_actor_head: bad args");
  D3A_CHECK_ARG(!d->dz || (d->h && d->w_head && d->H >= 1 && d->H <= 256),
                "d3a_sac_actor_head: dz needs h, w_head and 1 <= H <= 256");
  D3A_CHECK_ARG(d->dq_dz ? (d->w0 && d->C <= 4 && d->C * d->A <= 32 && d->H0 >= 1 &&
                            d->H0 <= 256)
                         : d->dq_da != nullptr,
                "d3a_sac_actor_head: dq_dz needs w0, C <= 4, C * A <= 32, 1 <= H0 <= 256 "
                "(else dq_da)");
  D3A_CHECK_ARG(!d->dq_min || (!d->dq_dz && d->dq_da && d->q && d->n_part >= 1),
                "d3a_sac_actor_head: dq_min reads dq_da and q in n_part >= 1 parts (not dq_dz)");
  if (d->dq_dz)
    hipLaunchKernelGGL(sac_actor_head_kernel<true>, dim3((unsigned)d->B + 1), dim3(256), 0,
                       (hipStream_t)stream, *d);
  else
    hipLaunchKernelGGL(sac_actor_head_kernel<false>, dim3((unsigned)d->B + 1), dim3(256), 0,
                       (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_sac_actor_head");
  return 0;
}
