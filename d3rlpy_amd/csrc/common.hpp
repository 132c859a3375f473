// Shared helpers for the d3rlpy_amd HIP library (gfx950 / CDNA4 only).
//
// Every entry point in include/d3rlpy_amd.h returns an int status: 0 on
// success, a negative code otherwise; d3a_last_error() returns the message.
// Kernels are enqueued on the caller's stream and never synchronise, so every
// entry point is legal inside hipStreamBeginCapture / torch.cuda.graph.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>

namespace d3a {

constexpr int kWave = 64;  // CDNA wavefront width

void set_error(const char* fmt, ...);

#define D3A_CHECK_ARG(cond, ...)                 \
  do {                                           \
    if (!(cond)) {                               \
      ::d3a::set_error(__VA_ARGS__);             \
      return -1;                                 \
    }                                            \
  } while (0)

#define D3A_LAUNCH_CHECK(name)                                              \
  do {                                                                      \
    hipError_t _e = hipGetLastError();                                      \
    if (_e != hipSuccess) {                                                 \
      ::d3a::set_error("%s: launch failed: %s", name, hipGetErrorString(_e)); \
      return -2;                                                            \
    }                                                                       \
  } while (0)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024).  `scratch` must
// hold blockDim.x / 64 floats.  Result is broadcast to every thread.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += scratch[i];  // fixed order: deterministic
  return s;
}

// block_sum of K values at once (one pair of barriers; each sum in the same
// order as block_sum, so bitwise equal).  `scratch` holds K * blockDim.x / 64.
template <int K>
__device__ __forceinline__ void block_sum_k(float (&v)[K], float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
  __syncthreads();
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) scratch[k * nw + wid] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += scratch[k * nw + i];
    v[k] = s;
  }
}

// Adam on a single scalar parameter (torch single-tensor path) held in
// registers; returns the new p, updates m / v (the caller stores them).
// bc = {1 - b1^t, 1 - b2^t} for the step t being taken.
__device__ __forceinline__ float adam_scalar_r(float p, float& m, float& v, float g, double lr,
                                               double b1, double b2, double eps, const double* bc) {
  float mm = fmaf((float)(1.0 - b1), __fsub_rn(g, m), m);
  float vv = __fmul_rn(v, (float)b2);
  vv = __fadd_rn(vv, __fmul_rn(__fmul_rn((float)(1.0 - b2), g), g));
  const float step_size = (float)(lr / bc[0]);
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vv), (float)sqrt(bc[1])), (float)eps);
  m = mm;
  v = vv;
  return __fadd_rn(p, __fmul_rn(-step_size, __fdiv_rn(mm, denom)));
}

// adam_scalar_r with the step's two float constants given: step_size =
// (float)(lr / bc1) and bc2_sqrt = (float)sqrt(bc2) (bitwise the same step)
__device__ __forceinline__ float adam_scalar_f(float p, float& m, float& v, float g, double b1,
                                               double b2, double eps, float step_size,
                                               float bc2_sqrt) {
  float mm = fmaf((float)(1.0 - b1), __fsub_rn(g, m), m);
  float vv = __fmul_rn(v, (float)b2);
  vv = __fadd_rn(vv, __fmul_rn(__fmul_rn((float)(1.0 - b2), g), g));
  const float denom = __fadd_rn(__fdiv_rn(__fsqrt_rn(vv), bc2_sqrt), (float)eps);
  m = mm;
  v = vv;
  return __fadd_rn(p, __fmul_rn(-step_size, __fdiv_rn(mm, denom)));
}

// torch.nn.functional.softplus(x, beta=1, threshold=20)
__device__ __forceinline__ float softplus_t(float x) {
  return x > 20.f ? x : log1pf(expf(x));
}

__device__ __forceinline__ float sigmoidf_t(float x) { return 1.f / (1.f + expf(-x)); }

// Philox-4x32-10 counter-based generator: (key, counter) -> 4 uint32.
struct Philox {
  __device__ static inline void round(uint32_t c[4], const uint32_t k[2]) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint64_t p0 = (uint64_t)M0 * c[0];
    uint64_t p1 = (uint64_t)M1 * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c[0] = hi1 ^ c[1] ^ k[0];
    c[1] = lo1;
    c[2] = hi0 ^ c[3] ^ k[1];
    c[3] = lo0;
  }
  __device__ static inline void gen(uint64_t seed, uint64_t ctr_hi, uint64_t ctr_lo,
                                    uint32_t out[4]) {
    uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t c[4] = {(uint32_t)ctr_lo, (uint32_t)(ctr_lo >> 32), (uint32_t)ctr_hi,
                     (uint32_t)(ctr_hi >> 32)};
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      round(c, k);
      k[0] += 0x9E3779B9u;
      k[1] += 0xBB67AE85u;
    }
    out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = c[3];
  }
};

// uint32 -> uniform float in (0, 1]
__device__ __forceinline__ float u01(uint32_t x) {
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// Element e of the d3a_philox_fill stream (seed, counter ctr): elements
// [0, n_normal) standard normal (Box-Muller over the 4 words of Philox call
// e / 4), the rest uniform in [lo, hi) -- bit-identical to what
// d3a_philox_fill writes at out[e], so a consumer can draw its own values.
__device__ __forceinline__ float philox_elem(uint64_t seed, uint64_t ctr, int64_t e,
                                             int64_t n_normal, float lo, float hi) {
  uint32_t r[4];
  Philox::gen(seed, ctr, (uint64_t)(e >> 2), r);
  const int q = (int)(e & 3);
  if (e < n_normal) {
    const int p = q & ~1;
    const float u1 = u01(r[p]), u2 = u01(r[p + 1]);
    const float rad = sqrtf(-2.f * logf(u1));
    return (q & 1) ? rad * sinf(6.283185307179586f * u2) : rad * cosf(6.283185307179586f * u2);
  }
  return lo + (hi - lo) * (u01(r[q]) - 0x1p-24f);
}

}  // namespace d3a
