// Whole-MLP forward for small row passes (hundreds of rows): 16-row
// workgroups on v_mfma_f32_16x16x4_f32.
//
// The d3a_mlp_fwd instantiation selected with block_rows = 16 for the
// latency-bound passes of the hot path -- the policy over [obs; next_obs]
// (512 rows, VectorEncoder 256-256 + mu | logstd head: encoders.py:265-275,
// policies.py:170-176), TD3+BC / BCQ policies and targets at 100-256 rows.
// Those passes do ~35 MFLOP per 256x256 layer: as per-layer launches each pays
// a dependent-kernel boundary, and the 32-row fused workgroup puts 4.2 MFLOP
// per layer on one CU.  Here a workgroup owns 16 rows (the smallest MFMA
// tile), so a 512-row pass spreads over 32 CUs and every layer's chain is
// half as long, and the whole MLP is one launch.
//
// Eight waves, wave w owning hidden units 32 w .. 32 w + 31 (two 16-unit
// tiles, two independent accumulation chains).  The MFMAs compute the
// transposed tile C^T[unit][row] = W[unit] . act[row] (W the A operand, read
// from global/L2 with every load of the layer issued up front; activation
// rows the B operand, from LDS), so a lane holds one row and four consecutive
// units: 16-byte stores to LDS and to the kept activations.  k order: group g
// of 16 k, lane group q = lane >> 4 supplying k = 16 g + 4 q + i to MFMA i
// (the same permutation on both operands: an exact fp32 chain, deterministic).
// The head (n_out <= 64 columns) reads the last layer from LDS: four threads
// per (row, column) dot, then a fixed butterfly.  A wide head (WH: 64 < n_out
// <= 256, e.g. BCQ's 200-quantile QR critics over their 256 batch rows) runs
// as one more MFMA layer instead -- wave w owning outputs 32 w .. + 31, no
// ReLU -- so those passes are one launch rather than three per-layer GEMMs.
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"

namespace d3a {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int S_RB = 16;    // rows per workgroup
constexpr int S_H = 256;    // hidden width
constexpr int S_LDK = 260;  // activation row stride in LDS
constexpr int S_JMAX = 64;

struct SmallLds {
  float x[S_RB * S_LDK];     // input rows (zero-padded to a multiple of 16)
  float h[2][S_RB * S_LDK];  // hidden activations, ping-pong
  float wh[S_JMAX * S_H];    // head weights
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// NL: hidden layers (compile time: the layer loop unrolls, so the registers
// of the prefetched weights are allocated statically)
// PROBE (timing probes only, D3A_SMALL_PROBE): bit 0 skips the 256-wide
// layers' MFMAs, bit 1 the head
template <int NL, int PROBE = 0, bool WH = false>
__global__ __launch_bounds__(512) void mlp_small_kernel(d3a_mlp_fwd_desc d) {
  __shared__ __attribute__((aligned(16))) SmallLds S;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 15, lq = lane >> 4;
  const int c = blockIdx.z;
  // (WH) the head's outputs in halves of 128 over blockIdx.y: both halves run
  // the hidden layers, half 0 keeps the activations
  const int hq = WH ? (int)blockIdx.y : 0;
  const int nb_main = (int)((d.rows + S_RB - 1) / S_RB);
  const bool aux = (int)blockIdx.x >= nb_main;
  const int m0 = aux ? ((int)blockIdx.x - nb_main) * S_RB : (int)d.r0 + (int)blockIdx.x * S_RB;
  const int rend = aux ? (int)d.aux_rows : (int)(d.r0 + d.rows);
  const int h_from = aux ? rend : (int)d.h_from;
  const int64_t wdel = aux ? d.aux_wdelta : 0;
  float* const outp = aux ? d.aux_out + c * d.aux_sout : d.out + c * d.sout;
  const int K0 = d.n_in, K0p = (K0 + 15) / 16 * 16;
  const int J = d.n_out;
  constexpr int L = NL;

  // ---- the small operands are loaded up front, in the order they are needed
  // (the vector memory counter retires in order): the input rows, the head
  // weights, the first layer's weights (narrow inputs), every bias.
  const int u0 = 32 * w + lr;  // A-operand unit of tile 0 (tile 1: + 16)
  const float* xb = aux ? d.aux_x + c * d.aux_sxb : d.x + c * d.sxb;
  const int64_t ldx = aux ? d.aux_ldx : d.ldx;
  constexpr int XS = (S_RB * S_H + 511) / 512;  // staged input elements per thread (<= 8)
  float xs[XS];
  const bool xg = d.xg_mode != 0;  // uniform: rows from the input-row builder
  if (xg) {
    // (d3a_mlp_fwd_desc.xg_*, no aux pass): quads of k, straight into LDS
    for (int e4 = t; e4 < S_RB * (K0p / 4); e4 += 512) {
      const int m = e4 / (K0p / 4), k4 = 4 * (e4 - m * (K0p / 4));
      float v[4];
      x6::input4_at(d, nullptr, 0, m0 + m, k4, rend, K0, v);
      *reinterpret_cast<float4*>(&S.x[m * S_LDK + k4]) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
#pragma unroll
  for (int i = 0; i < XS; ++i) {
    const int e = t + 512 * i;
    const int m = e / K0p, k = e - m * K0p;
    const int r = m0 + m;
    xs[i] = (!xg && e < S_RB * K0p && r < rend && k < K0) ? xb[(int64_t)r * ldx + k] : 0.f;
  }
  const float* Wh = d.W[L] + wdel + c * d.sW[L];
  constexpr int WS = (S_JMAX * S_H) / 512;  // head weights per thread (<= 32)
  float whs[WS];
#pragma unroll
  for (int i = 0; i < WS; ++i) {
    const int e = t + 512 * i;
    whs[i] = (!WH && e < J * S_H) ? Wh[e] : 0.f;
  }
  const float* W0 = d.W[0] + wdel + c * d.sW[0];
  const bool w0_regs = K0p <= 32;  // first layer's operand in registers
  float w0a[8], w0b[8];  // group g, element i: W0[unit][min(16 g + 4 lq + i, n_in - 1)]
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = min(16 * g + 4 * lq + i, K0 - 1);
      w0a[4 * g + i] = (w0_regs && 16 * g < K0p) ? W0[u0 * K0 + k] : 0.f;
      w0b[4 * g + i] = (w0_regs && 16 * g < K0p) ? W0[(u0 + 16) * K0 + k] : 0.f;
    }
  float4 bias[L][2];  // this lane's four units of each tile, every layer
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const float* b = d.b[l] + wdel + c * d.sb[l];
    bias[l][0] = *reinterpret_cast<const float4*>(b + 32 * w + 4 * lq);
    bias[l][1] = *reinterpret_cast<const float4*>(b + 32 * w + 16 + 4 * lq);
  }
  const float* bh = d.b[L] + wdel + c * d.sb[L];
  const float bh0 = WH ? 0.f : bh[((t >> 2) % J)];  // the head bias of this thread's first pair
  float4 wa[16], wb[16];
  auto load_w = [&](int l) {
    const float* W = d.W[l] + wdel + c * d.sW[l];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      wa[g] = *reinterpret_cast<const float4*>(W + u0 * S_H + 16 * g + 4 * lq);
      wb[g] = *reinterpret_cast<const float4*>(W + (u0 + 16) * S_H + 16 * g + 4 * lq);
    }
  };
  // stage the input rows and the head weights
#pragma unroll
  for (int i = 0; i < XS; ++i) {
    const int e = t + 512 * i;
    if (!xg && e < S_RB * K0p) {
      const int m = e / K0p, k = e - m * K0p;
      S.x[m * S_LDK + k] = xs[i];
    }
  }
  if constexpr (!WH) {
#pragma unroll
    for (int i = 0; i < WS; ++i) S.wh[t + 512 * i] = whs[i];
  }
  __syncthreads();

  // ---- hidden layers
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const float* src = l == 0 ? S.x : S.h[(l - 1) & 1];
    float* dst = S.h[l & 1];
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    if (l > 0 && (PROBE & 1)) {
      acc0[0] += wa[l].x + wb[l].y;
    } else if (l > 0) {
      // the layer's weights stream through this CU's L1 (256 KB per
      // workgroup: with the MFMA chain, what bounds a 16-row pass); issued
      // here rather than at kernel start, where they would queue ahead of
      // the input rows the first layer waits on (measured 15.2 vs 17.2 us on
      // the 512-row policy pass)
      load_w(l);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float4 a = *reinterpret_cast<const float4*>(&src[lr * S_LDK + 16 * g + 4 * lq]);
        acc0 = mfma4(wa[g].x, a.x, acc0); acc1 = mfma4(wb[g].x, a.x, acc1);
        acc0 = mfma4(wa[g].y, a.y, acc0); acc1 = mfma4(wb[g].y, a.y, acc1);
        acc0 = mfma4(wa[g].z, a.z, acc0); acc1 = mfma4(wb[g].z, a.z, acc1);
        acc0 = mfma4(wa[g].w, a.w, acc0); acc1 = mfma4(wb[g].w, a.w, acc1);
      }
    } else if (w0_regs) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        if (16 * g < K0p) {
          const float4 a = *reinterpret_cast<const float4*>(&src[lr * S_LDK + 16 * g + 4 * lq]);
          acc0 = mfma4(w0a[4 * g + 0], a.x, acc0); acc1 = mfma4(w0b[4 * g + 0], a.x, acc1);
          acc0 = mfma4(w0a[4 * g + 1], a.y, acc0); acc1 = mfma4(w0b[4 * g + 1], a.y, acc1);
          acc0 = mfma4(w0a[4 * g + 2], a.z, acc0); acc1 = mfma4(w0b[4 * g + 2], a.z, acc1);
          acc0 = mfma4(w0a[4 * g + 3], a.w, acc0); acc1 = mfma4(w0b[4 * g + 3], a.w, acc1);
        }
      }
    } else {
      // wide first layer (K0p > 32): W rows of n_in floats read per group (k
      // past n_in reads a clamped column times the zero padding of x: an exact 0)
      for (int g = 0; g < K0p / 16; ++g) {
        const float4 a = *reinterpret_cast<const float4*>(&src[lr * S_LDK + 16 * g + 4 * lq]);
        float va[4], vb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = min(16 * g + 4 * lq + i, K0 - 1);
          va[i] = W0[u0 * K0 + k];
          vb[i] = W0[(u0 + 16) * K0 + k];
        }
        acc0 = mfma4(va[0], a.x, acc0); acc1 = mfma4(vb[0], a.x, acc1);
        acc0 = mfma4(va[1], a.y, acc0); acc1 = mfma4(vb[1], a.y, acc1);
        acc0 = mfma4(va[2], a.z, acc0); acc1 = mfma4(vb[2], a.z, acc1);
        acc0 = mfma4(va[3], a.w, acc0); acc1 = mfma4(vb[3], a.w, acc1);
      }
    }
    // epilogue: lane holds row lr, units 32 w + 16 tile + 4 lq + i
    float* hg = (!aux && d.h[l] && hq == 0) ? d.h[l] + c * d.sh : nullptr;
    const int row = m0 + lr;
    const bool keep = hg != nullptr && row >= h_from && row < rend;
#pragma unroll
    for (int tl = 0; tl < 2; ++tl) {
      const f32x4& a = tl ? acc1 : acc0;
      const int u = 32 * w + 16 * tl + 4 * lq;
      const float4 bv = bias[l][tl];
      const float4 v = make_float4(fmaxf(a[0] + bv.x, 0.f), fmaxf(a[1] + bv.y, 0.f),
                                   fmaxf(a[2] + bv.z, 0.f), fmaxf(a[3] + bv.w, 0.f));
      *reinterpret_cast<float4*>(&dst[lr * S_LDK + u]) = v;
      if (keep) *reinterpret_cast<float4*>(hg + (int64_t)row * S_H + u) = v;
    }
    __syncthreads();
  }

  // ---- head: out[row][j] = h[row] . Wh[j] + bh[j]; four threads per pair
  const float* hl = S.h[(L - 1) & 1];
  if (PROBE & 2) return;
  if constexpr (WH) {
    // the head as one more MFMA layer: wave w (< 4 with halves) of half hq
    // owns outputs 128 hq + 32 w + 16 tile + lr (rows of Wh past n_out read row n_out - 1;
    // their outputs are not stored).  Two halves: each SIMD streams one
    // output tile's 128-MFMA chain instead of two (measured: the head was 8
    // of the pass's 22.4 us)
    const int jw = 128 * hq + 32 * w;
    if ((gridDim.y > 1 && w >= 4) || jw >= J) return;  // uniform: no outputs for this wave
    const int ja = min(jw + lr, J - 1), jb = min(jw + 16 + lr, J - 1);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      wa[g] = *reinterpret_cast<const float4*>(Wh + ja * S_H + 16 * g + 4 * lq);
      wb[g] = *reinterpret_cast<const float4*>(Wh + jb * S_H + 16 * g + 4 * lq);
    }
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float4 a = *reinterpret_cast<const float4*>(&hl[lr * S_LDK + 16 * g + 4 * lq]);
      acc0 = mfma4(wa[g].x, a.x, acc0); acc1 = mfma4(wb[g].x, a.x, acc1);
      acc0 = mfma4(wa[g].y, a.y, acc0); acc1 = mfma4(wb[g].y, a.y, acc1);
      acc0 = mfma4(wa[g].z, a.z, acc0); acc1 = mfma4(wb[g].z, a.z, acc1);
      acc0 = mfma4(wa[g].w, a.w, acc0); acc1 = mfma4(wb[g].w, a.w, acc1);
    }
    // lane: row lr, outputs 32 w + 16 tile + 4 lq + i
    const int row = m0 + lr;
    if (row < rend) {
#pragma unroll
      for (int tl = 0; tl < 2; ++tl) {
        const f32x4& a = tl ? acc1 : acc0;
        const int j0 = jw + 16 * tl + 4 * lq;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (j0 + i < J) outp[(int64_t)row * d.ldout + j0 + i] = a[i] + bh[j0 + i];
      }
    }
    return;
  }
  for (int p = t >> 2; p < S_RB * J; p += 128) {
    const int m = p / J, j = p - m * J, q = t & 3;
    float s = 0.f;
#pragma unroll 4
    for (int n = 4 * q; n < S_H; n += 16) {
      const float4 hv = *reinterpret_cast<const float4*>(&hl[m * S_LDK + n]);
      const float4 wv = *reinterpret_cast<const float4*>(&S.wh[j * S_H + n]);
      s = fmaf(hv.x, wv.x, s);
      s = fmaf(hv.y, wv.y, s);
      s = fmaf(hv.z, wv.z, s);
      s = fmaf(hv.w, wv.w, s);
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    const int r = m0 + m;
    const float bj = p == (t >> 2) ? bh0 : bh[j];
    if (q == 0 && r < rend) outp[(int64_t)r * d.ldout + j] = s + bj;
  }
}


// ---- parts variant (d3a_mlp_fwd_desc.parts): two hidden layers of 256, the
// second layer's units split into D3A_MLP_PARTS parts of 64.  A workgroup owns
// 16 rows, one member and one part: the narrow first layer for all 256 units
// (W0 in registers), its 64 units of the second layer (its W1 rows straight
// into registers), and its part of the head, out[p][row][j] = sum over its
// units of h2 Wh[j] (+ bias in part 0).  Four waves: wave w owns first-layer
// units 64 w .. 64 w + 63 (four tiles) and second-layer units U0 + 16 w ..
// U0 + 16 w + 15 (one tile, full k chain).  The head is summed over lane
// groups by a fixed butterfly and over waves in wave order.  JM: the head
// width bound, 16 (the head rows of the part's units in registers) or 32 (e.g.
// BCQ's VAE encoder, mu | logstd of 12 latents: staged in LDS instead).
constexpr int P_LDX = 68;  // input row stride in LDS (n_in <= 64)

template <int JM>
struct PartsLds {
  float x[S_RB * P_LDX];
  float h1[S_RB * S_LDK];
  float op[4][S_RB][JM];  // per-wave head partials
  float wh[JM > 16 ? JM : 1][64];  // JM 32: Wh[j][U0 .. U0 + 63]
};

template <int JM>
__global__ __launch_bounds__(256) void mlp_parts_kernel(d3a_mlp_fwd_desc d) {
  __shared__ __attribute__((aligned(16))) PartsLds<JM> S;
  {
    // workgroups past the pass's (d.presplit jobs): d3a_x6_split pieces on
    // the CUs the pass leaves idle, one piece a thread
    const int nbx = (int)((d.rows + S_RB - 1) / S_RB);
    if ((int)blockIdx.x >= nbx) {
      // (x columns nbx .. nbx + es - 1: the split jobs; the rest: the Philox job)
      const int64_t per_x = 256LL * gridDim.y * gridDim.z;
      const int64_t tot = x6::x6_split_total(d.presplit);
      const int es = (int)((tot + per_x - 1) / per_x);
      if ((int)blockIdx.x < nbx + es) {
        const int64_t nwg = (int64_t)es * gridDim.y * gridDim.z;
        const int64_t wgi = ((int64_t)(blockIdx.x - nbx) * gridDim.y + blockIdx.y) * gridDim.z + blockIdx.z;
        for (int64_t pp = wgi * 256 + threadIdx.x; pp < tot; pp += nwg * 256) x6::x6_split_piece(d.presplit, pp);
        return;
      }
      // d3a_philox_fill's body: one Philox call -> 4 outputs a thread, then
      // the last of these workgroups advances the counter
      const d3a_philox_job& ph = d.philox;
      const int64_t total = ph.n_normal + ph.n_uniform;
      const int64_t nwp = (int64_t)(gridDim.x - nbx - es) * gridDim.y * gridDim.z;
      const int64_t wgi = ((int64_t)(blockIdx.x - nbx - es) * gridDim.y + blockIdx.y) * gridDim.z + blockIdx.z;
      const int64_t step = *ph.ctr;
      const int64_t e0 = (wgi * 256 + threadIdx.x) * 4;
      if (e0 < total) {
        for (int q = 0; q < 4; ++q) {
          const int64_t e = e0 + q;
          if (e < total) ph.out[e] = philox_elem(ph.seed, (uint64_t)step, e, ph.n_normal, ph.lo, ph.hi);
        }
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        const unsigned prev = atomicAdd(ph.ticket, 1u);
        if (prev == (unsigned)(nwp - 1)) {
          *ph.ctr = step + 1;
          *ph.ticket = 0u;
        }
      }
      return;
    }
  }
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 15, lq = lane >> 4;
  const int c = blockIdx.y, p = blockIdx.z;
  const int U0 = 64 * p;
  const int m0 = (int)d.r0 + (int)blockIdx.x * S_RB;
  const int rend = (int)(d.r0 + d.rows);
  const int K0 = d.n_in, K0p = (K0 + 15) / 16 * 16, J = d.n_out;
  const float* xb = d.x + c * d.sxb;
  if (d.xg_mode != 0) {  // uniform: rows from the input-row builder (quads of k)
    // (the part-0 workgroups also write the rows out: xg_xout / xg_eout)
    const bool xo = d.xg_xout != nullptr && p == 0, eo = d.xg_eout != nullptr && p == 0;
    for (int e4 = t; e4 < S_RB * (P_LDX / 4); e4 += 256) {
      const int m = e4 / (P_LDX / 4), k4 = 4 * (e4 - m * (P_LDX / 4));
      const int r = m0 + m;
      float v[4];
      x6::input4_at(d, nullptr, 0, r, k4, rend, K0, v);
      *reinterpret_cast<float4*>(&S.x[m * P_LDX + k4]) = make_float4(v[0], v[1], v[2], v[3]);
      if (xo && r < rend && k4 < d.xg_ldxo)
        *reinterpret_cast<float4*>(d.xg_xout + (int64_t)r * d.xg_ldxo + k4) = make_float4(v[0], v[1], v[2], v[3]);
      if (eo && r < rend) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int e = k4 + j - d.xg_D;
          if (e >= 0 && e < d.xg_E) d.xg_eout[(int64_t)r * d.xg_E + e] = v[j];
        }
      }
    }
  } else {
    for (int e = t; e < S_RB * P_LDX; e += 256) {
      const int m = e / P_LDX, k = e - m * P_LDX;
      const int r = m0 + m;
      S.x[e] = (k < K0 && r < rend) ? xb[(int64_t)r * d.ldx + k] : 0.f;
    }
  }
  const float* W0 = d.W[0] + c * d.sW[0];
  float w0r[4][16];  // tile tt, group g, element i: W0[unit][min(16 g + 4 lq + i, n_in - 1)]
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = min(16 * g + 4 * lq + i, K0 - 1);
        w0r[tt][4 * g + i] = 16 * g < K0p ? W0[(64 * w + 16 * tt + lr) * K0 + k] : 0.f;
      }
  const float* W1 = d.W[1] + c * d.sW[1] + (int64_t)(U0 + 16 * w + lr) * S_H;
  float4 w1r[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) w1r[g] = *reinterpret_cast<const float4*>(W1 + 16 * g + 4 * lq);
  const float* b0 = d.b[0] + c * d.sb[0];
  float4 bias0[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
    bias0[tt] = *reinterpret_cast<const float4*>(b0 + 64 * w + 16 * tt + 4 * lq);
  const float4 bias1 =
      *reinterpret_cast<const float4*>(d.b[1] + c * d.sb[1] + U0 + 16 * w + 4 * lq);
  const float* Wh = d.W[2] + c * d.sW[2] + U0 + 16 * w + 4 * lq;
  float4 whv[16];
  if constexpr (JM <= 16) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      whv[j] = j < J ? *reinterpret_cast<const float4*>(Wh + j * S_H) : make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
    // the part's head columns, [j][64 units]: 512 float4 pieces over 256 threads
    const float* Whp = d.W[2] + c * d.sW[2] + U0;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int e = t + 256 * q, j = e >> 4, u4 = 4 * (e & 15);
      const float4 v = *reinterpret_cast<const float4*>(Whp + min(j, J - 1) * S_H + u4);
      *reinterpret_cast<float4*>(&S.wh[j][u4]) = j < J ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();

  // ---- first layer, all 256 units
  {
    f32x4 acc[4];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (16 * g < K0p) {
        const float4 a = *reinterpret_cast<const float4*>(&S.x[lr * P_LDX + 16 * g + 4 * lq]);
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          acc[tt] = mfma4(w0r[tt][4 * g + 0], a.x, acc[tt]);
          acc[tt] = mfma4(w0r[tt][4 * g + 1], a.y, acc[tt]);
          acc[tt] = mfma4(w0r[tt][4 * g + 2], a.z, acc[tt]);
          acc[tt] = mfma4(w0r[tt][4 * g + 3], a.w, acc[tt]);
        }
      }
    }
    const int row = m0 + lr;
    float* hg = (p == 0 && d.h[0]) ? d.h[0] + c * d.sh : nullptr;
    const bool keep = hg != nullptr && row >= d.h_from && row < rend;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const float4 bv = bias0[tt];
      const int u = 64 * w + 16 * tt + 4 * lq;
      const float4 v = make_float4(fmaxf(acc[tt][0] + bv.x, 0.f), fmaxf(acc[tt][1] + bv.y, 0.f),
                                   fmaxf(acc[tt][2] + bv.z, 0.f), fmaxf(acc[tt][3] + bv.w, 0.f));
      *reinterpret_cast<float4*>(&S.h1[lr * S_LDK + u]) = v;
      if (keep) *reinterpret_cast<float4*>(hg + (int64_t)row * S_H + u) = v;
    }
  }
  __syncthreads();

  // ---- the part's second-layer tile and its head terms
  {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float4 a = *reinterpret_cast<const float4*>(&S.h1[lr * S_LDK + 16 * g + 4 * lq]);
      acc = mfma4(w1r[g].x, a.x, acc);
      acc = mfma4(w1r[g].y, a.y, acc);
      acc = mfma4(w1r[g].z, a.z, acc);
      acc = mfma4(w1r[g].w, a.w, acc);
    }
    // lane: row lr, units U0 + 16 w + 4 lq + i
    const float4 v = make_float4(fmaxf(acc[0] + bias1.x, 0.f), fmaxf(acc[1] + bias1.y, 0.f),
                                 fmaxf(acc[2] + bias1.z, 0.f), fmaxf(acc[3] + bias1.w, 0.f));
    const int row = m0 + lr;
    if (d.h[1] && row >= d.h_from && row < rend)
      *reinterpret_cast<float4*>(d.h[1] + c * d.sh + (int64_t)row * S_H + U0 + 16 * w + 4 * lq) = v;
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      if (j < J) {
        const float4 wv = JM <= 16 ? whv[j < 16 ? j : 0]
                                   : *reinterpret_cast<const float4*>(&S.wh[j][16 * w + 4 * lq]);
        float s = 0.f;
        s = fmaf(v.x, wv.x, s);
        s = fmaf(v.y, wv.y, s);
        s = fmaf(v.z, wv.z, s);
        s = fmaf(v.w, wv.w, s);
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        if (lq == 0) S.op[w][lr][j] = s;
      }
    }
  }
  __syncthreads();
  for (int e = t; e < S_RB * J; e += 256) {
    const int m = e / J, j = e - m * J;
    const int r = m0 + m;
    if (r < rend) {
      float v = ((S.op[0][m][j] + S.op[1][m][j]) + S.op[2][m][j]) + S.op[3][m][j];
      if (p == 0) v += d.b[2][c * d.sb[2] + j];
      d.out[p * d.s_part + c * d.sout + (int64_t)r * d.ldout + j] = v;
    }
  }
}

}  // namespace

// d3a_mlp_fwd's parts path (the caller checked the shape); false when an
// alignment does not hold
bool mlp_parts_launch(const d3a_mlp_fwd_desc& d, hipStream_t st) {
  auto a16 = [](const void* p, int64_t stride) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && stride % 4 == 0;
  };
  if (!a16(d.W[1], d.sW[1]) || !a16(d.W[2], d.sW[2]) || !a16(d.b[0], d.sb[0]) ||
      !a16(d.b[1], d.sb[1]))
    return false;
  for (int l = 0; l < 2; ++l)
    if (d.h[l] && !a16(d.h[l], d.sh)) return false;
  const int64_t ph_total = d.philox.n_normal + d.philox.n_uniform;
  if (d.rows == 0 && d.presplit.n_jobs == 0 && ph_total <= 0) return true;
  // (presplit: enough extra workgroups for one piece a thread; philox: for
  // four outputs a thread)
  const int64_t pieces = d.presplit.n_jobs > 0 ? x6::x6_split_total(d.presplit) : 0;
  const int64_t per_x = 256LL * d.C * D3A_MLP_PARTS;
  const int64_t ex = (pieces + per_x - 1) / per_x;
  const int64_t exp = ph_total > 0 ? ((ph_total + 3) / 4 + per_x - 1) / per_x : 0;
  const dim3 grid((unsigned)((d.rows + S_RB - 1) / S_RB + ex + exp), (unsigned)d.C, (unsigned)D3A_MLP_PARTS);
  if (d.n_out <= 16)
    hipLaunchKernelGGL(mlp_parts_kernel<16>, grid, dim3(256), 0, st, d);
  else
    hipLaunchKernelGGL(mlp_parts_kernel<32>, grid, dim3(256), 0, st, d);
  return true;
}

// d3a_mlp_fwd's block_rows == 16 path; false when the shape does not fit
bool mlp_small_launch(const d3a_mlp_fwd_desc& d, hipStream_t st) {
  if (d.H != S_H || d.n_out > S_H || d.n_in > S_H || d.n_hidden < 1 || d.n_hidden > 4)
    return false;
  const bool wide = d.n_out > S_JMAX;
  if (wide && (d.n_hidden != 2 || (reinterpret_cast<uintptr_t>(d.W[d.n_hidden]) & 15) != 0 ||
               d.sW[d.n_hidden] % 4 != 0))
    return false;
  auto a16 = [](const void* p, int64_t stride) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && stride % 4 == 0;
  };
  for (int l = 1; l < d.n_hidden; ++l)
    if (!a16(d.W[l], d.sW[l])) return false;
  for (int l = 0; l < d.n_hidden; ++l)
    if (!a16(d.b[l], d.sb[l])) return false;
  for (int l = 0; l < d.n_hidden; ++l)
    if (d.h[l] && !a16(d.h[l], d.sh)) return false;
  if (d.aux_rows > 0 && d.aux_wdelta % 4) return false;
  const int64_t nb = (d.rows + S_RB - 1) / S_RB + (d.aux_rows + S_RB - 1) / S_RB;
  const dim3 grid((unsigned)nb, 1, (unsigned)d.C);
  static const int probe = [] {
    const char* e = getenv("D3A_SMALL_PROBE");
    return e ? atoi(e) : 0;
  }();
  if (wide) {
    // (the head's output halves on grid y; D3A_SMALL_WIDE_HALVES=0: one)
    static const bool halves = [] {
      const char* e = getenv("D3A_SMALL_WIDE_HALVES");
      return !(e && e[0] == '0');
    }();
    const dim3 grid((unsigned)nb, (unsigned)(halves ? (d.n_out + 127) / 128 : 1), (unsigned)d.C);
    if (probe == 1) hipLaunchKernelGGL((mlp_small_kernel<2, 1, true>), grid, dim3(512), 0, st, d);
    else if (probe == 2) hipLaunchKernelGGL((mlp_small_kernel<2, 2, true>), grid, dim3(512), 0, st, d);
    else if (probe == 3) hipLaunchKernelGGL((mlp_small_kernel<2, 3, true>), grid, dim3(512), 0, st, d);
    else hipLaunchKernelGGL((mlp_small_kernel<2, 0, true>), grid, dim3(512), 0, st, d);
    return true;
  }
  if (probe && d.n_hidden == 2) {
    if (probe == 1) hipLaunchKernelGGL((mlp_small_kernel<2, 1>), grid, dim3(512), 0, st, d);
    else if (probe == 2) hipLaunchKernelGGL((mlp_small_kernel<2, 2>), grid, dim3(512), 0, st, d);
    else hipLaunchKernelGGL((mlp_small_kernel<2, 3>), grid, dim3(512), 0, st, d);
    return true;
  }
  switch (d.n_hidden) {
    case 1: hipLaunchKernelGGL(mlp_small_kernel<1>, grid, dim3(512), 0, st, d); break;
    case 2: hipLaunchKernelGGL(mlp_small_kernel<2>, grid, dim3(512), 0, st, d); break;
    case 3: hipLaunchKernelGGL(mlp_small_kernel<3>, grid, dim3(512), 0, st, d); break;
    default: hipLaunchKernelGGL(mlp_small_kernel<4>, grid, dim3(512), 0, st, d); break;
  }
  return true;
}

}  // namespace d3a
