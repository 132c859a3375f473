// Stand-alone forward / backward kernels of the loss and sampling blocks of
// the update, the op set behind the PyTorch custom ops (csrc/torch_ops.cpp,
// torch.ops.d3rlpy_amd.*).  The update pipelines run fused versions of the
// same arithmetic (cql.hip, bcq.hip, iqn.hip); these entry points expose each
// block on its own so a reference-shaped torch module can call it under
// autograd.  Every reduction is in a fixed order (run-to-run bit-identical).
//
//   logsumexp          torch.logsumexp(x, dim=-1)  (CQL conservative term,
//                      cql_impl.py:208-213) and its backward g * exp(x - lse)
//   td_mse             ContinuousMeanQFunction.compute_error
//                      (mean_q_function.py:74-87): y = r + gamma * target *
//                      (1 - terminal), loss = mean((q - y)^2), per member
//   quantile_huber     compute_quantile_huber_loss (q_functions/utility.py:27-46)
//   squashed_gauss     SquashedGaussianDistribution.sample_with_log_prob
//                      (distributions.py:112-135) after SquashedNormalPolicy's
//                      logstd clamp (policies.py:196-216)
//   relu_mask          threshold_backward: dz = dy * [y > 0]
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

// ---- logsumexp over the last dimension: one wave per row ------------------
__global__ __launch_bounds__(256) void lse_fwd_kernel(const float* x, int64_t rows, int64_t n,
                                                      int64_t ldx, float* out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + r * ldx;
  float m = -INFINITY;
  for (int64_t j = lane; j < n; j += 64) m = fmaxf(m, xr[j]);
  m = wave_max(m);
  // at::logsumexp: the max is dropped when it is infinite
  const float mc = fabsf(m) == INFINITY ? 0.f : m;
  float s = 0.f;
  for (int64_t j = lane; j < n; j += 64) s += expf(__fsub_rn(xr[j], mc));
  s = wave_sum(s);
  if (lane == 0) out[r] = __fadd_rn(logf(s), mc);
}

// torch's logsumexp_backward: grad * exp(x - result)
__global__ __launch_bounds__(256) void lse_bwd_kernel(const float* x, int64_t rows, int64_t n,
                                                      int64_t ldx, const float* lse,
                                                      const float* gout, float* dx,
                                                      int64_t lddx) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * n) return;
  const int64_t r = i / n, j = i - r * n;
  dx[r * lddx + j] = __fmul_rn(gout[r], expf(__fsub_rn(x[r * ldx + j], lse[r])));
}

// ---- TD mean-squared error: one workgroup per member ----------------------
__global__ __launch_bounds__(1024) void td_mse_kernel(const float* q, const float* rew,
                                                      const float* target, const float* term,
                                                      const float* gamma, int64_t n, float* diff,
                                                      float* loss) {
  __shared__ double part[1024];
  const int64_t c = blockIdx.x;
  const float* qc = q + c * n;
  const float* tc = target + c * n;
  float* dc = diff + c * n;
  double acc = 0.0;
  for (int64_t r = threadIdx.x; r < n; r += 1024) {
    // y = rewards + gamma * target * (1 - terminals), left to right
    const float y = __fadd_rn(rew[r], __fmul_rn(__fmul_rn(gamma[r], tc[r]),
                                                 __fsub_rn(1.f, term[r])));
    const float d = __fsub_rn(qc[r], y);
    dc[r] = d;
    acc += (double)__fmul_rn(d, d);
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[c] = (float)(part[0] / (double)n);
}

// mse_loss + mean backward: dq = grad / n * 2 * diff
__global__ __launch_bounds__(256) void td_mse_bwd_kernel(const float* diff, const float* gout,
                                                         int64_t C, int64_t n, float* dq) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= C * n) return;
  const int64_t c = i / n;
  const float gm = __fdiv_rn(gout[c], (float)n);
  dq[i] = __fmul_rn(__fmul_rn(2.f, diff[i]), gm);
}

// ---- quantile Huber loss: one workgroup per batch row ----------------------
// q [B][N] (row stride ldq), y [B][M] (ldy), taus [B][N] (ldt):
//   loss[b] = (1/M) sum_j sum_i |tau_i - [y_j - q_i < 0]| * huber(y_j - q_i)
__device__ __forceinline__ float huber1(float d) {
  const float a = fabsf(d);
  return a < 1.f ? __fmul_rn(0.5f, __fmul_rn(d, d)) : __fsub_rn(a, 0.5f);
}

__global__ __launch_bounds__(256) void qhuber_fwd_kernel(const float* q, int64_t ldq,
                                                         const float* y, int64_t ldy,
                                                         const float* taus, int64_t ldt,
                                                         int64_t N, int64_t M, float* loss) {
  __shared__ double part[256];
  const int64_t b = blockIdx.x;
  const float* qb = q + b * ldq;
  const float* yb = y + b * ldy;
  const float* tb = taus + b * ldt;
  double acc = 0.0;
  for (int64_t p = threadIdx.x; p < N * M; p += 256) {
    const int64_t j = p / N, i = p - j * N;
    const float d = __fsub_rn(yb[j], qb[i]);
    const float w = fabsf(__fsub_rn(tb[i], d < 0.f ? 1.f : 0.f));
    acc += (double)__fmul_rn(w, huber1(d));
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[b] = (float)(part[0] / (double)M);
}

// d loss[b] / d q[b][i] = -(1/M) sum_j |tau_i - delta_ji| * huber'(y_j - q_i)
// (huber' = d inside the quadratic zone, sign(d) outside; delta detached)
__global__ __launch_bounds__(256) void qhuber_bwd_kernel(const float* q, int64_t ldq,
                                                         const float* y, int64_t ldy,
                                                         const float* taus, int64_t ldt,
                                                         int64_t N, int64_t M, const float* gout,
                                                         float* dq, int64_t lddq) {
  const int64_t b = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  const float qi = q[b * ldq + i], ti = taus[b * ldt + i];
  const float* yb = y + b * ldy;
  double acc = 0.0;
  for (int64_t j = 0; j < M; ++j) {
    const float d = __fsub_rn(yb[j], qi);
    const float w = fabsf(__fsub_rn(ti, d < 0.f ? 1.f : 0.f));
    const float hd = fabsf(d) < 1.f ? d : (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f));
    acc += (double)__fmul_rn(w, hd);
  }
  dq[b * lddq + i] = (float)(-acc / (double)M * (double)gout[b]);
}

// ---- squashed Gaussian sample + log-prob: one wave per row -----------------
__global__ __launch_bounds__(256) void sgauss_fwd_kernel(const float* mu, const float* logstd,
                                                         const float* eps, int64_t B, int A,
                                                         float lo, float hi, float* action,
                                                         float* logp) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  float s = 0.f;
  for (int a = lane; a < A; a += 64) {
    const int64_t k = b * A + a;
    const float ls = fminf(fmaxf(logstd[k], lo), hi);
    const float sd = expf(ls);
    const float raw = __fadd_rn(mu[k], __fmul_rn(eps[k], sd));  // rsample: loc + eps * scale
    const float d = __fsub_rn(raw, mu[k]);
    const float var = __fmul_rn(sd, sd);
    // Normal.log_prob: -((x - loc)^2) / (2 var) - log(scale) - log(sqrt(2 pi))
    const float nlp = __fsub_rn(__fsub_rn(-__fdiv_rn(__fmul_rn(d, d), __fmul_rn(2.f, var)),
                                          logf(sd)),
                                0.91893853320467274178f);
    // jacob = 2 * (log 2 - raw - softplus(-2 raw))
    const float jac = __fmul_rn(2.f, __fsub_rn(__fsub_rn(0.69314718055994530942f, raw),
                                                softplus_t(__fmul_rn(-2.f, raw))));
    s += __fsub_rn(nlp, jac);
    action[k] = tanhf(raw);
  }
  s = wave_sum(s);
  if (lane == 0) logp[b] = s;
}

__global__ __launch_bounds__(256) void sgauss_bwd_kernel(const float* mu, const float* logstd,
                                                         const float* eps, int64_t B, int A,
                                                         float lo, float hi, const float* gact,
                                                         const float* glogp, float* dmu,
                                                         float* dlogstd) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= B * A) return;
  const int64_t b = k / A;
  const float lsr = logstd[k];
  const float ls = fminf(fmaxf(lsr, lo), hi);
  const float sd = expf(ls);
  const float raw = __fadd_rn(mu[k], __fmul_rn(eps[k], sd));
  const float d = __fsub_rn(raw, mu[k]);
  const float var = __fmul_rn(sd, sd);
  const float y = tanhf(raw);
  const float gl = glogp ? glogp[b] : 0.f;
  const float ga = gact ? gact[k] : 0.f;
  // d log_prob / d raw (holding loc, scale): -d / var + 2 - 4 sigmoid(-2 raw)
  const float dlp_draw = __fadd_rn(-__fdiv_rn(d, var),
                                   __fsub_rn(2.f, __fmul_rn(4.f, sigmoidf_t(__fmul_rn(-2.f, raw)))));
  const float g_raw = __fadd_rn(__fmul_rn(ga, __fsub_rn(1.f, __fmul_rn(y, y))), __fmul_rn(gl, dlp_draw));
  // explicit loc / scale terms of Normal.log_prob
  dmu[k] = __fadd_rn(g_raw, __fmul_rn(gl, __fdiv_rn(d, var)));
  const float dnlp_dsd = __fsub_rn(__fdiv_rn(__fmul_rn(d, d), __fmul_rn(var, sd)), __fdiv_rn(1.f, sd));
  const float g_sd = __fadd_rn(__fmul_rn(g_raw, eps[k]), __fmul_rn(gl, dnlp_dsd));
  // exp backward (grad * result), clamp backward (pass inside [lo, hi])
  dlogstd[k] = (lsr >= lo && lsr <= hi) ? __fmul_rn(g_sd, sd) : 0.f;
}

__global__ __launch_bounds__(256) void relu_mask_kernel(const float* dy, const float* y, int64_t n,
                                                        float* dz) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dz[i] = y[i] > 0.f ? dy[i] : 0.f;
}

unsigned blocks(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_logsumexp_f32(const float* x, int64_t rows, int64_t n, int64_t ldx,
                                 float* out, void* stream) {
  D3A_CHECK_ARG(x && out, "d3a_logsumexp_f32: null pointer");
  D3A_CHECK_ARG(rows >= 0 && n >= 1 && ldx >= n, "d3a_logsumexp_f32: bad sizes");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(lse_fwd_kernel, dim3(blocks(rows, 4)), dim3(256), 0, (hipStream_t)stream, x,
                     rows, n, ldx, out);
  D3A_LAUNCH_CHECK("d3a_logsumexp_f32");
  return 0;
}

extern "C" int d3a_logsumexp_bwd_f32(const float* x, int64_t rows, int64_t n, int64_t ldx,
                                     const float* lse, const float* gout, float* dx,
                                     int64_t lddx, void* stream) {
  D3A_CHECK_ARG(x && lse && gout && dx, "d3a_logsumexp_bwd_f32: null pointer");
  D3A_CHECK_ARG(rows >= 0 && n >= 1 && ldx >= n && lddx >= n, "d3a_logsumexp_bwd_f32: bad sizes");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(lse_bwd_kernel, dim3(blocks(rows * n, 256)), dim3(256), 0,
                     (hipStream_t)stream, x, rows, n, ldx, lse, gout, dx, lddx);
  D3A_LAUNCH_CHECK("d3a_logsumexp_bwd_f32");
  return 0;
}

extern "C" int d3a_td_mse_f32(const float* q, const float* rew, const float* target,
                              const float* term, const float* gamma, int64_t C, int64_t n,
                              float* diff, float* loss, void* stream) {
  D3A_CHECK_ARG(q && rew && target && term && gamma && diff && loss, "d3a_td_mse_f32: null pointer");
  D3A_CHECK_ARG(C >= 1 && C < 65536 && n >= 1, "d3a_td_mse_f32: bad sizes");
  hipLaunchKernelGGL(td_mse_kernel, dim3((unsigned)C), dim3(1024), 0, (hipStream_t)stream, q, rew,
                     target, term, gamma, n, diff, loss);
  D3A_LAUNCH_CHECK("d3a_td_mse_f32");
  return 0;
}

extern "C" int d3a_td_mse_bwd_f32(const float* diff, const float* gout, int64_t C, int64_t n,
                                  float* dq, void* stream) {
  D3A_CHECK_ARG(diff && gout && dq, "d3a_td_mse_bwd_f32: null pointer");
  D3A_CHECK_ARG(C >= 1 && n >= 1, "d3a_td_mse_bwd_f32: bad sizes");
  hipLaunchKernelGGL(td_mse_bwd_kernel, dim3(blocks(C * n, 256)), dim3(256), 0,
                     (hipStream_t)stream, diff, gout, C, n, dq);
  D3A_LAUNCH_CHECK("d3a_td_mse_bwd_f32");
  return 0;
}

extern "C" int d3a_quantile_huber_f32(const float* q, int64_t ldq, const float* y, int64_t ldy,
                                      const float* taus, int64_t ldt, int64_t B, int64_t N,
                                      int64_t M, float* loss, void* stream) {
  D3A_CHECK_ARG(q && y && taus && loss, "d3a_quantile_huber_f32: null pointer");
  D3A_CHECK_ARG(B >= 0 && N >= 1 && M >= 1 && ldq >= N && ldt >= N && ldy >= M && B < (1ll << 31),
                "d3a_quantile_huber_f32: bad sizes");
  if (B == 0) return 0;
  hipLaunchKernelGGL(qhuber_fwd_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, q,
                     ldq, y, ldy, taus, ldt, N, M, loss);
  D3A_LAUNCH_CHECK("d3a_quantile_huber_f32");
  return 0;
}

extern "C" int d3a_quantile_huber_bwd_f32(const float* q, int64_t ldq, const float* y,
                                          int64_t ldy, const float* taus, int64_t ldt, int64_t B,
                                          int64_t N, int64_t M, const float* gout, float* dq,
                                          int64_t lddq, void* stream) {
  D3A_CHECK_ARG(q && y && taus && gout && dq, "d3a_quantile_huber_bwd_f32: null pointer");
  D3A_CHECK_ARG(B >= 0 && N >= 1 && M >= 1 && ldq >= N && ldt >= N && ldy >= M && lddq >= N &&
                    B < 65536,
                "d3a_quantile_huber_bwd_f32: bad sizes");
  if (B == 0) return 0;
  hipLaunchKernelGGL(qhuber_bwd_kernel, dim3(blocks(N, 256), (unsigned)B), dim3(256), 0,
                     (hipStream_t)stream, q, ldq, y, ldy, taus, ldt, N, M, gout, dq, lddq);
  D3A_LAUNCH_CHECK("d3a_quantile_huber_bwd_f32");
  return 0;
}

extern "C" int d3a_squashed_gauss_f32(const float* mu, const float* logstd, const float* eps,
                                      int64_t B, int32_t A, float min_logstd, float max_logstd,
                                      float* action, float* logp, void* stream) {
  D3A_CHECK_ARG(mu && logstd && eps && action && logp, "d3a_squashed_gauss_f32: null pointer");
  D3A_CHECK_ARG(B >= 0 && A >= 1, "d3a_squashed_gauss_f32: bad sizes");
  if (B == 0) return 0;
  hipLaunchKernelGGL(sgauss_fwd_kernel, dim3(blocks(B, 4)), dim3(256), 0, (hipStream_t)stream,
                     mu, logstd, eps, B, (int)A, min_logstd, max_logstd, action, logp);
  D3A_LAUNCH_CHECK("d3a_squashed_gauss_f32");
  return 0;
}

extern "C" int d3a_squashed_gauss_bwd_f32(const float* mu, const float* logstd, const float* eps,
                                          int64_t B, int32_t A, float min_logstd,
                                          float max_logstd, const float* grad_action,
                                          const float* grad_logp, float* dmu, float* dlogstd,
                                          void* stream) {
  D3A_CHECK_ARG(mu && logstd && eps && dmu && dlogstd, "d3a_squashed_gauss_bwd_f32: null pointer");
  D3A_CHECK_ARG(B >= 0 && A >= 1, "d3a_squashed_gauss_bwd_f32: bad sizes");
  if (B == 0) return 0;
  hipLaunchKernelGGL(sgauss_bwd_kernel, dim3(blocks(B * A, 256)), dim3(256), 0,
                     (hipStream_t)stream, mu, logstd, eps, B, (int)A, min_logstd, max_logstd,
                     grad_action, grad_logp, dmu, dlogstd);
  D3A_LAUNCH_CHECK("d3a_squashed_gauss_bwd_f32");
  return 0;
}

extern "C" int d3a_relu_mask_f32(const float* dy, const float* y, int64_t n, float* dz,
                                 void* stream) {
  D3A_CHECK_ARG(dy && y && dz, "d3a_relu_mask_f32: null pointer");
  if (n <= 0) return 0;
  hipLaunchKernelGGL(relu_mask_kernel, dim3(blocks(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     dy, y, n, dz);
  D3A_LAUNCH_CHECK("d3a_relu_mask_f32");
  return 0;
}
