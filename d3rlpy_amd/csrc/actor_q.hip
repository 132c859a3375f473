// d3a_sac_actor_q: the actor phase's critic pass of CQL / SAC in one launch.
//
// The actor loss (entropy - Q_min(s, a~pi)).mean() (d3rlpy/algos/torch/
// sac_impl.py:114-121) evaluates the critic ensemble [n_in, 256, 256, 1]
// (encoders.py:265-275 + mean_q_function.py:255-256) at the B rows (s, tanh u)
// and back-propagates to the action input.  Every quantity is row-local, so a
// workgroup owns 16 rows of one member and does the whole chain with nothing
// in HBM between the layers:
//   forward  z1 = W0 x + b0, h1 = relu(z1); z2 = W1 h1 + b1, h2 = relu(z2);
//            q = wh . h2 + bh
//   backward (dL/dq = 1) dz2 = wh * [h2 > 0]; dz1 = (W1^T dz2) * [h1 > 0];
//            dq/da_j = sum_k dz1[k] W0[k][da_off + j]
// The backward of the min over the members (which member's gradient flows,
// scaled by -1/B) is applied by d3a_sac_actor_head (dq_min mode), which reads
// every member's q and dq/da.
//
// Eight waves, wave w owning hidden units 32 w .. 32 w + 31 (two 16-unit
// tiles) on v_mfma_f32_16x16x4_f32 with the transposed product
// C^T[unit][row] (weights the A operand, activation rows the B operand from
// LDS), as mlp_small.hip; the backward's W1^T operand is read column-wise
// (16 lanes x 4 B contiguous per unit row).  k order inside a 16-group: lane
// group q = lane >> 4 supplies k = 16 g + 4 q + i to MFMA i on both operands
// (exact fp32 chains).  Head and dq/da partials are summed over lane groups by
// a fixed butterfly and over waves in wave order (deterministic).
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int AQ_RB = 16;    // rows per workgroup
constexpr int AQ_H = 256;    // hidden width
constexpr int AQ_LDK = 260;  // activation row stride in LDS
constexpr int AQ_LDX = 68;   // input row stride in LDS (n_in <= 64)
constexpr int AQ_AMAX = 16;

struct AqLds {
  float x[AQ_RB * AQ_LDX];      // input rows, zero-padded to a multiple of 16 columns
  float h1[AQ_RB * AQ_LDK];     // layer-1 activation (the backward's mask)
  float h2[AQ_RB * AQ_LDK];     // layer-2 activation, then dz2
  float wa[AQ_AMAX * AQ_H];     // W0's action columns, [j][k]
  float qp[8][AQ_RB];           // per-wave head partials
  float jp[8][AQ_RB][AQ_AMAX];  // per-wave dq/da partials
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__global__ __launch_bounds__(512) void sac_actor_q_kernel(d3a_sac_actor_q_desc d) {
  __shared__ __attribute__((aligned(16))) AqLds S;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 15, lq = lane >> 4;
  const int c = blockIdx.y;
  const int m0 = blockIdx.x * AQ_RB;
  const int K0 = d.n_in, K0p = (K0 + 15) / 16 * 16, A = d.A;
  const float* W0 = d.W0 + (int64_t)c * AQ_H * K0;
  const float* W1 = d.W1 + (int64_t)c * AQ_H * AQ_H;
  const float* b0 = d.b0 + c * AQ_H;
  const float* b1 = d.b1 + c * AQ_H;
  const float* wh = d.wh + c * AQ_H;
  const int u0 = 32 * w + lr;  // A-operand unit of tile 0 (tile 1: + 16)

  // ---- small operands first: input rows, W0 (registers), W0's action
  // columns (LDS), biases and head weights of this lane's units
  for (int e = t; e < AQ_RB * AQ_LDX; e += 512) {
    const int m = e / AQ_LDX, k = e - m * AQ_LDX;
    const int r = m0 + m;
    S.x[e] = (k < K0 && r < d.B) ? d.x[(int64_t)r * d.ldx + k] : 0.f;
  }
  float w0a[16], w0b[16];  // group g, element i: W0[unit][min(16 g + 4 lq + i, n_in - 1)]
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = min(16 * g + 4 * lq + i, K0 - 1);
      w0a[4 * g + i] = 16 * g < K0p ? W0[u0 * K0 + k] : 0.f;
      w0b[4 * g + i] = 16 * g < K0p ? W0[(u0 + 16) * K0 + k] : 0.f;
    }
  for (int e = t; e < A * AQ_H; e += 512) {
    const int j = e / AQ_H, k = e - j * AQ_H;
    S.wa[e] = W0[k * K0 + d.da_off + j];
  }
  float4 bias0[2], bias1[2], whv[2];
#pragma unroll
  for (int tl = 0; tl < 2; ++tl) {
    const int u = 32 * w + 16 * tl + 4 * lq;
    bias0[tl] = *reinterpret_cast<const float4*>(b0 + u);
    bias1[tl] = *reinterpret_cast<const float4*>(b1 + u);
    whv[tl] = *reinterpret_cast<const float4*>(wh + u);
  }
  const float bh = d.bh[c];
  __syncthreads();

  // ---- layer 1 (K0p <= 64: four k groups at most)
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    if (16 * g < K0p) {
      const float4 a = *reinterpret_cast<const float4*>(&S.x[lr * AQ_LDX + 16 * g + 4 * lq]);
      acc0 = mfma4(w0a[4 * g + 0], a.x, acc0); acc1 = mfma4(w0b[4 * g + 0], a.x, acc1);
      acc0 = mfma4(w0a[4 * g + 1], a.y, acc0); acc1 = mfma4(w0b[4 * g + 1], a.y, acc1);
      acc0 = mfma4(w0a[4 * g + 2], a.z, acc0); acc1 = mfma4(w0b[4 * g + 2], a.z, acc1);
      acc0 = mfma4(w0a[4 * g + 3], a.w, acc0); acc1 = mfma4(w0b[4 * g + 3], a.w, acc1);
    }
  }
  // layer 2's weights: rows u0, u0 + 16 (issued behind layer 1's operands)
  float4 wa[16], wb[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    wa[g] = *reinterpret_cast<const float4*>(W1 + u0 * AQ_H + 16 * g + 4 * lq);
    wb[g] = *reinterpret_cast<const float4*>(W1 + (u0 + 16) * AQ_H + 16 * g + 4 * lq);
  }
#pragma unroll
  for (int tl = 0; tl < 2; ++tl) {
    const f32x4& a = tl ? acc1 : acc0;
    const float4 bv = bias0[tl];
    const int u = 32 * w + 16 * tl + 4 * lq;
    *reinterpret_cast<float4*>(&S.h1[lr * AQ_LDK + u]) =
        make_float4(fmaxf(a[0] + bv.x, 0.f), fmaxf(a[1] + bv.y, 0.f), fmaxf(a[2] + bv.z, 0.f),
                    fmaxf(a[3] + bv.w, 0.f));
  }
  __syncthreads();

  // ---- layer 2 + head partial + dz2 (= wh * [h2 > 0], dL/dq = 1)
  acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
  acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float4 a = *reinterpret_cast<const float4*>(&S.h1[lr * AQ_LDK + 16 * g + 4 * lq]);
    acc0 = mfma4(wa[g].x, a.x, acc0); acc1 = mfma4(wb[g].x, a.x, acc1);
    acc0 = mfma4(wa[g].y, a.y, acc0); acc1 = mfma4(wb[g].y, a.y, acc1);
    acc0 = mfma4(wa[g].z, a.z, acc0); acc1 = mfma4(wb[g].z, a.z, acc1);
    acc0 = mfma4(wa[g].w, a.w, acc0); acc1 = mfma4(wb[g].w, a.w, acc1);
  }
  // the backward's W1^T operand: lane (lr, lq) of tile tl supplies
  // W1[16 g + 4 lq + i][32 w + 16 tl + lr] to MFMA i of group g
  float va[16][4], vb[16][4];
  const int k0 = 32 * w + lr;
#pragma unroll
  for (int g = 0; g < 16; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = 16 * g + 4 * lq + i;
      va[g][i] = W1[u * AQ_H + k0];
      vb[g][i] = W1[u * AQ_H + k0 + 16];
    }
  float hq = 0.f;  // this lane's part of row lr's head dot (8 units)
#pragma unroll
  for (int tl = 0; tl < 2; ++tl) {
    const f32x4& a = tl ? acc1 : acc0;
    const float4 bv = bias1[tl], hw = whv[tl];
    const int u = 32 * w + 16 * tl + 4 * lq;
    const float h0 = fmaxf(a[0] + bv.x, 0.f), h1 = fmaxf(a[1] + bv.y, 0.f);
    const float h2 = fmaxf(a[2] + bv.z, 0.f), h3 = fmaxf(a[3] + bv.w, 0.f);
    hq = fmaf(h0, hw.x, hq);
    hq = fmaf(h1, hw.y, hq);
    hq = fmaf(h2, hw.z, hq);
    hq = fmaf(h3, hw.w, hq);
    *reinterpret_cast<float4*>(&S.h2[lr * AQ_LDK + u]) =
        make_float4(h0 > 0.f ? hw.x : 0.f, h1 > 0.f ? hw.y : 0.f, h2 > 0.f ? hw.z : 0.f,
                    h3 > 0.f ? hw.w : 0.f);
  }
  hq += __shfl_xor(hq, 16, 64);
  hq += __shfl_xor(hq, 32, 64);
  if (lq == 0) S.qp[w][lr] = hq;
  __syncthreads();

  // ---- backward: dh1^T[k][row] = sum_u W1[u][k] dz2[row][u]
  acc0 = f32x4{0.f, 0.f, 0.f, 0.f};
  acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float4 a = *reinterpret_cast<const float4*>(&S.h2[lr * AQ_LDK + 16 * g + 4 * lq]);
    acc0 = mfma4(va[g][0], a.x, acc0); acc1 = mfma4(vb[g][0], a.x, acc1);
    acc0 = mfma4(va[g][1], a.y, acc0); acc1 = mfma4(vb[g][1], a.y, acc1);
    acc0 = mfma4(va[g][2], a.z, acc0); acc1 = mfma4(vb[g][2], a.z, acc1);
    acc0 = mfma4(va[g][3], a.w, acc0); acc1 = mfma4(vb[g][3], a.w, acc1);
  }
  // dz1 = dh1 * [h1 > 0]; lane: row lr, k = 32 w + 16 tl + 4 lq + i
  float jpart[AQ_AMAX];
#pragma unroll
  for (int j = 0; j < AQ_AMAX; ++j) jpart[j] = 0.f;
#pragma unroll
  for (int tl = 0; tl < 2; ++tl) {
    const f32x4& a = tl ? acc1 : acc0;
    const int k = 32 * w + 16 * tl + 4 * lq;
    const float4 hv = *reinterpret_cast<const float4*>(&S.h1[lr * AQ_LDK + k]);
    const float z0 = hv.x > 0.f ? a[0] : 0.f, z1 = hv.y > 0.f ? a[1] : 0.f;
    const float z2 = hv.z > 0.f ? a[2] : 0.f, z3 = hv.w > 0.f ? a[3] : 0.f;
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
  __syncthreads();
  // ---- per row: q (waves summed in order) and dq/da
  if (t < AQ_RB) {
    const int r = m0 + t;
    if (r < d.B) {
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) s += S.qp[v][t];
      d.q[c * d.sqc + r] = s + bh;
    }
  } else if (t >= 64 && t < 64 + AQ_RB * A) {
    const int e = t - 64, m = e / A, j = e - m * A;
    const int r = m0 + m;
    if (r < d.B) {
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) s += S.jp[v][m][j];
      d.dq_da[c * d.sda_c + (int64_t)r * d.ld_da + d.da_off + j] = s;
    }
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
  D3A_CHECK_ARG(d->ldx >= d->n_in && d->ld_da >= d->da_off + d->A,
                "d3a_sac_actor_q: row strides too small");
  D3A_CHECK_ARG(((reinterpret_cast<uintptr_t>(d->W1) | reinterpret_cast<uintptr_t>(d->b0) |
                  reinterpret_cast<uintptr_t>(d->b1) | reinterpret_cast<uintptr_t>(d->wh)) &
                 15) == 0,
                "d3a_sac_actor_q: W1 / b0 / b1 / wh must be 16-byte aligned");
  const dim3 grid((unsigned)((d->B + AQ_RB - 1) / AQ_RB), (unsigned)d->C);
  hipLaunchKernelGGL(sac_actor_q_kernel, grid, dim3(512), 0, (hipStream_t)stream, *d);
  D3A_LAUNCH_CHECK("d3a_sac_actor_q");
  return 0;
}
