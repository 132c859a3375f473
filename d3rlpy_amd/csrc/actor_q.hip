// d3a_sac_actor_q: the actor phase's critic pass of CQL / SAC in one launch.
//
// The actor loss (entropy - Q_min(s, a~pi)).mean() (d3rlpy/algos/torch/
// sac_impl.py:114-121) evaluates the critic ensemble [n_in, 256, 256, 1]
// (encoders.py:265-275 + mean_q_function.py:255-256) at the B rows (s, tanh u)
// and back-propagates to the action input.  Every quantity is row-local:
//   forward  z1 = W0 x + b0, h1 = relu(z1); z2 = W1 h1 + b1, h2 = relu(z2);
//            q = wh . h2 + bh
//   backward (dL/dq = 1) dz2 = wh * [h2 > 0]; dz1 = (W1^T dz2) * [h1 > 0];
//            dq/da_j = sum_k dz1[k] W0[k][da_off + j]
// dz2[u] depends on unit u of layer 2 only, and q and dq/da are linear in the
// per-unit terms, so the 256 layer-2 units are split into four parts of 64:
// a workgroup owns 16 rows, one member and one part — it recomputes the
// (narrow) first layer for all 256 units, then only its 64 rows of W1 enter
// the forward and the backward, and it writes its part of q and of dq/da.
// d3a_sac_actor_head sums the four parts in order and applies the backward of
// the min over the members.  B = 256, C = 2 gives 128 workgroups (one launch
// of 32 workgroups owning all 256 units measured 20.9 us: MFMA-bound on 32 CUs).
//
// The part's 64 rows of W1 (64 KB) are staged in LDS once, coalesced, and feed
// both products: rows (float4 along k) as the forward's A operand, columns as
// the backward's.  Four waves; MFMA v_mfma_f32_16x16x4_f32 on transposed tiles
// C^T[unit][row] (weights the A operand, activation rows the B operand), as
// mlp_small.hip.  k order inside a 16-group: lane group q = lane >> 4 supplies
// k = 16 g + 4 q + i to MFMA i on both operands (exact fp32 chains).  Head and
// dq/da partials are summed over lane groups by a fixed butterfly and over
// waves in wave order (deterministic).
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int AQ_RB = 16;     // rows per workgroup
constexpr int AQ_H = 256;     // hidden width
constexpr int AQ_P = D3A_ACTOR_Q_PARTS;
constexpr int AQ_U = AQ_H / AQ_P;  // layer-2 units per part (64)
constexpr int AQ_LDK = 260;   // row stride of 256-wide LDS rows
constexpr int AQ_LDU = 68;    // row stride of 64-wide LDS rows
constexpr int AQ_LDX = 68;    // input row stride in LDS (n_in <= 64)
constexpr int AQ_AMAX = 16;

struct AqLds {
  float w1[AQ_U * AQ_LDK];       // the part's rows of W1
  float x[AQ_RB * AQ_LDX];       // input rows, zero-padded to a multiple of 16 columns
  float h1[AQ_RB * AQ_LDK];      // layer-1 activation (the backward's mask)
  float dz[AQ_RB * AQ_LDU];      // dz2 of the part's units
  float wa[AQ_AMAX * AQ_H];      // W0's action columns, [j][k]
  float qp[4][AQ_RB];            // per-wave head partials
  float jp[4][AQ_RB][AQ_AMAX];   // per-wave dq/da partials
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(256) void sac_actor_q_kernel(d3a_sac_actor_q_desc d) {
  __shared__ __attribute__((aligned(16))) AqLds S;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 15, lq = lane >> 4;
  const int c = blockIdx.y, p = blockIdx.z;
  const int m0 = blockIdx.x * AQ_RB;
  const int K0 = d.n_in, K0p = (K0 + 15) / 16 * 16, A = d.A;
  const int U0 = p * AQ_U;
  const float* W0 = d.W0 + (int64_t)c * AQ_H * K0;
  const float* W1 = d.W1 + (int64_t)c * AQ_H * AQ_H + (int64_t)U0 * AQ_H;
  const float* b0 = d.b0 + c * AQ_H;
  const float* b1 = d.b1 + c * AQ_H + U0;
  const float* wh = d.wh + c * AQ_H + U0;

  // ---- operands, in the order they are needed: input rows, W0 (registers:
  // wave w computes layer-1 units 64 w + 16 t + lr), the part's W1 rows (LDS),
  // W0's action columns (LDS), biases and head weights
  for (int e = t; e < AQ_RB * AQ_LDX; e += 256) {
    const int m = e / AQ_LDX, k = e - m * AQ_LDX;
    const int r = m0 + m;
    S.x[e] = (k < K0 && r < d.B) ? d.x[(int64_t)r * d.ldx + k] : 0.f;
  }
  float w0r[4][16];  // tile t, group g, element i: W0[unit][min(16 g + 4 lq + i, n_in - 1)]
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = min(16 * g + 4 * lq + i, K0 - 1);
        w0r[tt][4 * g + i] = 16 * g < K0p ? W0[(64 * w + 16 * tt + lr) * K0 + k] : 0.f;
      }
  float4 w1s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int e = t + 256 * i;  // float4 index in the 64 x 256 slab
    const int u = e >> 6, k4 = e & 63;
    w1s[i] = *reinterpret_cast<const float4*>(W1 + u * AQ_H + 4 * k4);
  }
  float4 bias0[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
    bias0[tt] = *reinterpret_cast<const float4*>(b0 + 64 * w + 16 * tt + 4 * lq);
  const float4 bias1 = *reinterpret_cast<const float4*>(b1 + 16 * w + 4 * lq);
  const float4 hw = *reinterpret_cast<const float4*>(wh + 16 * w + 4 * lq);
  const float bh = p == 0 ? d.bh[c] : 0.f;
  for (int e = t; e < A * AQ_H; e += 256) {
    const int j = e / AQ_H, k = e - j * AQ_H;
    S.wa[e] = W0[k * K0 + d.da_off + j];
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int e = t + 256 * i;
    const int u = e >> 6, k4 = e & 63;
    *reinterpret_cast<float4*>(&S.w1[u * AQ_LDK + 4 * k4]) = w1s[i];
  }
  __syncthreads();

  // ---- layer 1, all 256 units (K0p <= 64: four k groups at most)
  {
    f32x4 acc[4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (16 * g < K0p) {
        const float4 a = *reinterpret_cast<const float4*>(&S.x[lr * AQ_LDX + 16 * g + 4 * lq]);
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          acc[tt] = mfma4(w0r[tt][4 * g + 0], a.x, acc[tt]);
          acc[tt] = mfma4(w0r[tt][4 * g + 1], a.y, acc[tt]);
          acc[tt] = mfma4(w0r[tt][4 * g + 2], a.z, acc[tt]);
          acc[tt] = mfma4(w0r[tt][4 * g + 3], a.w, acc[tt]);
        }
      }
    }
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const float4 bv = bias0[tt];
      const int u = 64 * w + 16 * tt + 4 * lq;
      *reinterpret_cast<float4*>(&S.h1[lr * AQ_LDK + u]) =
          make_float4(fmaxf(acc[tt][0] + bv.x, 0.f), fmaxf(acc[tt][1] + bv.y, 0.f),
                      fmaxf(acc[tt][2] + bv.z, 0.f), fmaxf(acc[tt][3] + bv.w, 0.f));
    }
  }
  __syncthreads();

  // ---- layer 2 on the part's units U0 + 16 w + (0..15), head partial, dz2
  {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* wrow = &S.w1[(16 * w + lr) * AQ_LDK];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float4 a = *reinterpret_cast<const float4*>(&S.h1[lr * AQ_LDK + 16 * g + 4 * lq]);
      const float4 wv = *reinterpret_cast<const float4*>(wrow + 16 * g + 4 * lq);
      acc = mfma4(wv.x, a.x, acc);
      acc = mfma4(wv.y, a.y, acc);
      acc = mfma4(wv.z, a.z, acc);
      acc = mfma4(wv.w, a.w, acc);
    }
    // lane: row lr, units U0 + 16 w + 4 lq + i
    const float h0 = fmaxf(acc[0] + bias1.x, 0.f), h1 = fmaxf(acc[1] + bias1.y, 0.f);
    const float h2 = fmaxf(acc[2] + bias1.z, 0.f), h3 = fmaxf(acc[3] + bias1.w, 0.f);
    float hq = 0.f;
    hq = fmaf(h0, hw.x, hq);
    hq = fmaf(h1, hw.y, hq);
    hq = fmaf(h2, hw.z, hq);
    hq = fmaf(h3, hw.w, hq);
    *reinterpret_cast<float4*>(&S.dz[lr * AQ_LDU + 16 * w + 4 * lq]) =
        make_float4(h0 > 0.f ? hw.x : 0.f, h1 > 0.f ? hw.y : 0.f, h2 > 0.f ? hw.z : 0.f,
                    h3 > 0.f ? hw.w : 0.f);
    hq += __shfl_xor(hq, 16, 64);
    hq += __shfl_xor(hq, 32, 64);
    if (lq == 0) S.qp[w][lr] = hq;
  }
  __syncthreads();

  // ---- backward over the part: dh1^T[k][row] = sum_{u in part} W1[u][k] dz2[row][u]
  // for k in wave w's tiles 64 w + 16 t + (0..15); then dz1 = dh1 * [h1 > 0] and
  // this lane's dq/da terms (row lr, k = 64 w + 16 t + 4 lq + i)
  {
    f32x4 acc[4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 a = *reinterpret_cast<const float4*>(&S.dz[lr * AQ_LDU + 16 * g + 4 * lq]);
      const float* wc = &S.w1[(16 * g + 4 * lq) * AQ_LDK + 64 * w + lr];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        acc[tt] = mfma4(wc[0 * AQ_LDK + 16 * tt], a.x, acc[tt]);
        acc[tt] = mfma4(wc[1 * AQ_LDK + 16 * tt], a.y, acc[tt]);
        acc[tt] = mfma4(wc[2 * AQ_LDK + 16 * tt], a.z, acc[tt]);
        acc[tt] = mfma4(wc[3 * AQ_LDK + 16 * tt], a.w, acc[tt]);
      }
    }
    float jpart[AQ_AMAX];
#pragma unroll
    for (int j = 0; j < AQ_AMAX; ++j) jpart[j] = 0.f;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int k = 64 * w + 16 * tt + 4 * lq;
      const float4 hv = *reinterpret_cast<const float4*>(&S.h1[lr * AQ_LDK + k]);
      const float z0 = hv.x > 0.f ? acc[tt][0] : 0.f, z1 = hv.y > 0.f ? acc[tt][1] : 0.f;
      const float z2 = hv.z > 0.f ? acc[tt][2] : 0.f, z3 = hv.w > 0.f ? acc[tt][3] : 0.f;
#pragma unroll
      for (int j = 0; j < AQ_AMAX; ++j) {
        if (j < A) {
          const float4 wv = *reinterpret_cast<const float4*>(&S.wa[j * AQ_H + k]);
          float s = jpart[j];
          s = fmaf(z0, wv.x, s);
          s = fmaf(z1, wv.y, s);
          s = fmaf(z2, wv.z, s);
          s = fmaf(z3, wv.w, s);
          jpart[j] = s;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < AQ_AMAX; ++j) {
      if (j < A) {
        float s = jpart[j];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        if (lq == 0) S.jp[w][lr][j] = s;
      }
    }
  }
  __syncthreads();

  // ---- this part's q and dq/da per row (waves summed in order)
  const int64_t pc = (int64_t)p * d.C + c;
  if (t < AQ_RB) {
    const int r = m0 + t;
    if (r < d.B)
      d.q[pc * d.B + r] = (((S.qp[0][t] + S.qp[1][t]) + S.qp[2][t]) + S.qp[3][t]) + bh;
  }
  // AQ_RB * A <= 256 entries: threads 0..255 cover every (row, action) pair
  // (waves 1..3 first, so wave 0's q stores issue alongside)
  for (int e = (t + 64) & 255; e < AQ_RB * A; e += 256) {
    const int m = e / A, j = e - m * A;
    const int r = m0 + m;
    if (r < d.B)
      d.dq_da[(pc * d.B + r) * A + j] =
          ((S.jp[0][m][j] + S.jp[1][m][j]) + S.jp[2][m][j]) + S.jp[3][m][j];
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_sac_actor_q(const d3a_sac_actor_q_desc* d, void* stream) {
  D3A_CHECK_ARG(d && d->x && d->W0 && d->b0 && d->W1 && d->b1 && d->wh && d->bh && d->q &&
                    d->dq_da,
                "d3a_sac_actor_q: null operand");
  D3A_CHECK_ARG(d->B >= 1 && d->C >= 1 && d->n_in >= 1 && d->n_in <= 64,
                "d3a_sac_actor_q: B >= 1, C >= 1, 1 <= n_in <= 64");
  D3A_CHECK_ARG(d->A >= 1 && d->A <= AQ_AMAX && d->da_off >= 0 && d->da_off + d->A <= d->n_in,
                "d3a_sac_actor_q: 1 <= A <= 16 and da_off + A <= n_in");
  D3A_CHECK_ARG(d->ldx >= d->n_in, "d3a_sac_actor_q: ldx < n_in");
  D3A_CHECK_ARG(((reinterpret_cast<uintptr_t>(d->W1) | reinterpret_cast<uintptr_t>(d->b0) |
                  reinterpret_cast<uintptr_t>(d->b1) | reinterpret_cast<uintptr_t>(d->wh)) &
                 15) == 0,
                "d3a_sac_actor_q: W1 / b0 / b1 / wh must be 16-byte aligned");
  const dim3 grid((unsigned)((d->B + AQ_RB - 1) / AQ_RB), (unsigned)d->C, (unsigned)AQ_P);
  hipLaunchKernelGGL(sac_actor_q_kernel, grid, dim3(256), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_sac_actor_q");
  return 0;
}
