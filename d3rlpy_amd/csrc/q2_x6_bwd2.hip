// fp32 critic backward on the bf16 matrix cores, slice geometry: d3a_q2_bwd's
// weight gradients of [n_in <= 48 -> 256 -> 256 -> 1] with the mask-factored
// split-bf16 products of q2_x6_bwd.hip,
//
//   dh1[r][i] = g'[r] * sum_o m[r][o] (w3[o] W2[o][i]),  m = [h2 > 0]
//   R[o][i]   = sum_r m[r][o] (g'[r] h1[r][i]),           dW2 = w3[o] R[o][i]
//
// but with no kept h2 and a quarter of the row-block partials.
//
// * The forward writes the ReLU mask of h2 twice as bits: by rows (hmask,
//   8 words a row: bit o & 31 of word o >> 5) and transposed (hmaskT: word
//   [r / 32][o], bit r & 31).  Each lane expands its MFMA operand byte from
//   them through a 256-entry LDS table (byte -> eight bf16 0 / 1): no mask
//   image is staged, so no barrier couples the waves of a workgroup.
// * dW3 = g'^T h2 is not formed from h2 (the forward keeps no h2): since
//   h2 = m (W2 h1 + b2),  dW3[o] = sum_i W2[o][i] R[o][i] + b2[o] S[o] with
//   S[o] = sum_r m[r][o] g'[r] -- R is the dW2 product the kernel forms anyway
//   (the identity is exact; the roundings are fp32's, the sums of the 16-unit
//   slice in fp64), and db2 = w3[o] S[o].
// * Geometry: a workgroup owns one member, one of P row blocks (P = 8 for
//   two members: 992 rows of K2's 7,936) and a 16-unit slice of layer 1
//   (16 slices: C P 16 = 256 workgroups), the 16 slices of a (member, row
//   block) on one XCD (they read the same mask words, g' and x rows, and h1
//   rows in 64-byte halves of the same lines).  Eight waves, 16x16x32 MFMA
//   tiles, 32-row sub-blocks dealt round-robin:
//     row waves 0-3 (sub-blocks w, w + 4, ...): dh1[32 rows][16 units] over
//       all 256 o (A = mask rows, B = (w3 W2) parts from LDS), then
//       dz1 = g' dh1 [h1 > 0], db1, dW1 += dz1^T x (six products, the dz1
//       accumulator as the MFMA's A operand);
//     col waves 4-7 (the same sub-blocks): R[256 o][16 units] += m^T (g' h1)
//       (A = transposed mask bytes, B = g' h1 parts split in registers), S.
//   Each wave loads its next sub-block's operands from global memory while it
//   multiplies the current one (two register sets); the waves meet only in the
//   epilogue, where the four waves of a role are summed in fp64 in wave order.
// * Partials (summed by d3a_adam_f32 in a fixed order): dW1 / db1 / dW2 / db2 /
//   db3 one per row block [P][C][..], dW3 one per (row block, slice) [P 16][C][256].
//   P = d3a_q2_bwd_x6t_splits(rows, C) unless d.row_splits is set.
//
// Reference: the autograd backward of update_critic's loss (ddpg_impl.py:119-133
// via cql_impl.py:110-125) through VectorEncoderWithAction (encoders.py:265-275,
// 328-339) and ContinuousMeanQFunction._fc (mean_q_function.py:255-256).
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"

namespace d3a {
namespace {

using namespace x6;

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int T_H = 256;
constexpr int T_SB = 32;            // rows per sub-block
constexpr int T_IW = 16;            // layer-1 units per workgroup
constexpr int T_NQ = T_H / T_IW;    // slices
constexpr int T_NT = 512;
constexpr int T_BLD = T_H + 8;      // bf16 stride of an [i][o] row of the (w3 W2) image
constexpr int T_NDBMAX = 3;

struct TLds {
  __bf16 bw[3][T_IW * T_BLD];       // parts of (w3 W2)[o][i0 + i], [part][i][o]
  uint4 lut[256];                   // byte b -> bf16 (b >> j) & 1, j = 0..7
  f32x4 red[4][T_NQ][64];           // col waves' R: [wave][o tile][lane]
  double pr[T_H][T_IW];             // W2[o][i] R[o][i] of the slice, fp64
  double s[4][64];                  // col waves' S partials [wave][lane]
  double g3[4];                     // col waves' sum g' (slice 0)
  f32x4 w1[4][T_NDBMAX][64];        // row waves' dW1 [wave][x block][lane]
  double b1[4][64];                 // row waves' db1 [wave][lane]
  float cs[5][8];                   // (CQL) the loss stage's wave sums [sum][wave]
};

__device__ __forceinline__ f32x4 m16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// the three products of a 0 / 1 operand with the parts of b, smallest first
__device__ __forceinline__ f32x4 x3m16(bf16x8 a, const bf16x8* b, f32x4 c) {
  c = m16(a, b[2], c);
  c = m16(a, b[1], c);
  c = m16(a, b[0], c);
  return c;
}

// the six part products (x6.hpp's prod6 order)
__device__ __forceinline__ f32x4 prod6_16(const bf16x8* a, const bf16x8* b, f32x4 c) {
  c = m16(a[2], b[0], c);
  c = m16(a[1], b[1], c);
  c = m16(a[0], b[2], c);
  c = m16(a[1], b[0], c);
  c = m16(a[0], b[1], c);
  c = m16(a[0], b[0], c);
  return c;
}

// v if on, +0 otherwise, with no branch (the compiler otherwise skips the
// loads that feed v under the predicate, one waited round trip each)
__device__ __forceinline__ float keep_if(bool on, float v) {
  return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, v) & (on ? 0xFFFFFFFFu : 0u));
}

// element idx of a wave-uniform base through a 32-bit byte offset (a saddr
// load: the base stays in scalar registers, no 64-bit address per lane)
template <typename T>
__device__ __forceinline__ T ldo(const T* base, uint32_t idx) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + idx * (uint32_t)sizeof(T));
}

// operands of one sub-block, col role
struct ColOps {
  uint4 mt[T_NQ / 4]; // transposed mask words of o = 16 tt + (lane & 15), tt = 4 v + e
  uint32_t mq;        // and of o = 16 q + (lane & 15) (the slice's own tile)
  float h[8];         // h1 of rows 8 g + j at unit i0 + (lane & 15)
  float g[8];         // g' of those rows (0 past the block)
};

// operands of one sub-block, row role
template <int NDB>
struct RowOps {
  uint4 m[2][2];      // mask words 0-3 / 4-7 of rows rho(h, lane & 15)
  float h[8];
  float g[8];
};

// NDB: 16-wide blocks of x (n_in <= 16 NDB); nkw: sub-blocks per wave, a
// multiple of 4 >= ceil(sub-blocks per row block / 4).
// CQL (d3a_q2_bwd_x6_cql): the CQL loss stage (cql.hip cql_loss_stage's
// arithmetic, after the logsumexp stage of a split d3a_cql_loss) in the
// prologue of every workgroup -- the conservative scale of the rows' gradients
// from the alpha step each workgroup takes itself; workgroup 0 writes the
// metrics, scalars and the new scalar optimiser state (lc.stage)
// ST (diagnostic build, D3A_BWD_STAMPS=1; results right): s_memtime stamps of
// waves 0 and 4 of every workgroup at the phase boundaries (d3a_bwd_stamps)
__device__ unsigned long long bwd_stamps[256 * 2 * 8];
template <int NDB, bool CQL = false, bool ST = false>
__global__ __launch_bounds__(T_NT) void q2x6t_bwd_kernel(d3a_q2_bwd_desc d, int P, int rbp, int nkw,
                                                         d3a_cql_loss_desc lc) {
  __shared__ __attribute__((aligned(16))) TLds L;
  static_assert(sizeof(TLds) <= 163840, "LDS");
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  auto stamp = [&](int k) {
    if constexpr (ST) {
      if ((t == 0 || t == 256) && blockIdx.x < 256)
        bwd_stamps[(blockIdx.x * 2 + (t >> 8)) * 8 + k] = __builtin_amdgcn_s_memtime();
    }
  };
  stamp(0);
  // decode: block id b = 8 k + x (x the XCD under round-robin dispatch); the
  // 16 slices q = k & 15 of unit u = (k >> 4) 8 + x share the XCD
  const int bid = blockIdx.x;
  const int kx = bid >> 3;
  const int q = kx & (T_NQ - 1);
  const int u = (kx >> 4) * 8 + (bid & 7);
  if (u >= P * d.C) return;  // whole workgroup, before any barrier
  // (readfirstlane: the division is done on vector registers; the member's
  // base pointers must stay scalar)
  const int c = __builtin_amdgcn_readfirstlane(u / P);
  const int p = __builtin_amdgcn_readfirstlane(u - c * P);
  const int rows = (int)d.rows;
  const int rb0 = p * rbp;
  const int rb1 = min(rows, rb0 + rbp);
  const int i0 = q * T_IW;
  const int nin = d.n_in;
  const int ldx = (int)d.ldx;
  const float* h1g = d.h1 + c * d.sh;
  const float* gg = d.g + c * d.sgb;
  const float* xg = d.x + c * d.sxb;
  const float* W2g = d.W2 + c * d.sW2;
  const float* w3g = d.w3 + c * d.sw3;
  const uint32_t* m2g = reinterpret_cast<const uint32_t*>(d.m2) + c * d.sm2;
  const uint32_t* mtg = reinterpret_cast<const uint32_t*>(d.m2t) + c * d.sm2t;
  // g' scale of the first n_scaled rows; (CQL) and the term subtracted from
  // the rest, both formed after the prologue's barrier
  float gs = CQL ? 0.f : (d.gscale ? *d.gscale : 1.f);
  float gsub = 0.f;
  const int64_t pc = (int64_t)p * d.C + c;
  const bool col = w >= 4;
  const int rw = w & 3;  // wave within its role: sub-blocks rw, rw + 4, ...

  // (CQL) this thread's share of the loss stage's sums: slot p = t's values
  // loaded raw up front (clamped, masked where summed after the staging, so
  // no load waits before the staging's own loads are out): alpha's lse and
  // data Q; workgroup 0 also the critic set's lse and the squared TD errors
  const bool wg0 = blockIdx.x == 0;
  float cv[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  [[maybe_unused]] float st_lt = 0.f, st_tm = 0.f, st_tv = 0.f, st_la = 0.f, st_am = 0.f, st_av = 0.f;
  [[maybe_unused]] float r_qd = 0.f, r_la = 0.f, r_lc = 0.f, r_t2 = 0.f, r_lt = 0.f;
  const int cb_n = CQL ? lc.C * lc.B : 0;  // C B (< 2^31: checked on the host)
  auto cql_row = [&](int pp, float& qd, float& la, float& lcv, float& t2) {
    const int p2 = pp < cb_n ? pp : cb_n - 1;
    const int cc = p2 / lc.B, bb = p2 - cc * lc.B;
    // (every load unconditional -- in range -- and masked where summed: a load
    // under a branch makes the compiler wait for every load in flight)
    qd = lc.q[(int64_t)cc * lc.R + 6LL * lc.N * lc.B + bb];
    la = lc.lse[p2];
    lcv = lc.lse[cb_n + p2];
    t2 = lc.td2[p2];
  };


  // ---- prologue: the byte table and the slice's (w3 W2) parts
  if (t < 256) {
    uint4 v;
    uint32_t* vp = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      vp[k] = ((t >> (2 * k)) & 1u) * 0x3F80u | ((t >> (2 * k + 1)) & 1u) * 0x3F800000u;
    L.lut[t] = v;
  }
  {
    // o = (t >> 4) + 32 k, i = t & 15: w3[o] W2[o][i0 + i] rounded once (the
    // fp32 product q2_x6_bwd.hip forms), split into three parts
    float wv[8], w3v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int o = (t >> 4) + 32 * k;
      wv[k] = W2g[o * T_H + i0 + (t & 15)];
      w3v[k] = w3g[o];
    }
    // (CQL) the loss stage's loads after the staging's (the counter is in
    // order: the staging below waits for its own loads only)
    if constexpr (CQL) {
      cql_row(t, r_qd, r_la, r_lc, r_t2);
      r_lt = lc.logp_temp[t < lc.B ? t : lc.B - 1];  // (used by workgroup 0)
      // the scalar optimiser state (every value, updated or not: the stage
      // carries all six) as vector loads through an opaque zero index, in
      // the vector counter's order: as scalar loads the kernel-argument
      // loads' waits would wait for them
      int z0;
      asm volatile("v_mov_b32 %0, 0" : "=v"(z0));
      st_lt = lc.log_temp[z0];
      st_la = lc.log_alpha[z0];
      st_tm = lc.temp_m[z0];
      st_tv = lc.temp_v[z0];
      st_am = lc.alpha_m[z0];
      st_av = lc.alpha_v[z0];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int o = (t >> 4) + 32 * k;
      __bf16 a, b, e;
      split1(w3v[k] * wv[k], a, b, e);
      L.bw[0][(t & 15) * T_BLD + o] = a;
      L.bw[1][(t & 15) * T_BLD + o] = b;
      L.bw[2][(t & 15) * T_BLD + o] = e;
    }
  }
  stamp(1);
  // (CQL) the wave's sums published in LDS for the prologue's barrier
  auto cql_publish = [&]() {
  if constexpr (CQL) {
    // slot t's values, then (C B > 512) the rest in p order; workgroup 0's
    // temperature log-probs
    const bool ok = t < cb_n, oa = ok && lc.update_alpha, o0 = ok && wg0;
    cv[0] = keep_if(oa, r_la);
    cv[1] = keep_if(ok, r_qd);
    cv[2] = keep_if(o0, r_lc);
    cv[3] = keep_if(o0, r_t2);
    for (int pp = t + T_NT; pp < cb_n; pp += T_NT) {
      float a0, a1, a2, a3;
      cql_row(pp, a1, a0, a2, a3);
      cv[0] += keep_if(lc.update_alpha, a0);
      cv[1] += a1;
      cv[2] += keep_if(wg0, a2);
      cv[3] += keep_if(wg0, a3);
    }
    cv[4] = keep_if(wg0 && lc.update_temp && t < lc.B, r_lt - (float)lc.A);
    if (wg0 && lc.update_temp)
      for (int bb = t + T_NT; bb < lc.B; bb += T_NT) cv[4] += lc.logp_temp[bb] - (float)lc.A;
    // the wave's sums (cql_loss_stage's block_sum order: wave sums, then the
    // waves in order after the barrier)
#pragma unroll
    for (int k = 0; k < 5; ++k) cv[k] = wave_sum(cv[k]);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) L.cs[k][w] = cv[k];
    }
  }
  };
  // (CQL) after the prologue's barrier: the sums, alpha's Adam step and the
  // conservative scale, formed by every thread (workgroup 0's thread 0 also
  // the temperature's step and the stage's outputs)
  auto cql_scalars = [&]() {
    if constexpr (CQL) {
      float sum[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        float s2 = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s2 += L.cs[k][i];
        sum[k] = s2;
      }
      const float B = (float)lc.B, CB = (float)((int64_t)lc.C * lc.B);
      float lalpha = st_la, am = st_am, av = st_av;
      float alpha_loss = 0.f;
      if (lc.update_alpha) {
        const float loss = sum[0] / CB - sum[1] / CB;
        const float scaled = lc.conservative_weight * loss;
        const float e = expf(lalpha);
        const float ca0 = fminf(fmaxf(e, 0.f), 1e6f);
        alpha_loss = -(ca0 * (scaled - lc.alpha_threshold));
        const bool pass = (e >= 0.f) && (e <= 1e6f);
        const float g = pass ? -(scaled - lc.alpha_threshold) * e : 0.f;
        lalpha = adam_scalar_f(lalpha, am, av, g, lc.beta1, lc.beta2, lc.adam_eps, (float)lc.bc[2],
                               (float)lc.bc[3]);
      }
      const float ca = fminf(fmaxf(expf(lalpha), 0.f), 1e6f);
      const float gcons = ca * lc.conservative_weight / CB;
      // (every lane holds the same value: a scalar register through the loop)
      gs = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, gcons)));
      gsub = gs;
      if (wg0 && t == 0) {
        float ltemp = st_lt, tm = st_tm, tv = st_tv;
        if (lc.update_temp) {
          const float e = expf(ltemp);
          lc.metrics[0] = -(e * sum[4]) / B;
          const float g = (-1.f / B) * sum[4] * e;
          ltemp = adam_scalar_f(ltemp, tm, tv, g, lc.beta1, lc.beta2, lc.adam_eps, (float)lc.bc[0],
                                (float)lc.bc[1]);
          lc.metrics[1] = expf(ltemp);
        }
        if (lc.update_alpha) {
          lc.metrics[2] = alpha_loss;
          lc.metrics[3] = expf(lalpha);
        }
        lc.stage[0] = ltemp; lc.stage[1] = tm; lc.stage[2] = tv;
        lc.stage[3] = lalpha; lc.stage[4] = am; lc.stage[5] = av;
        const float temp = expf(ltemp);
        lc.scalars[0] = temp;
        lc.scalars[1] = ca;
        lc.scalars[2] = gcons;
        const float td = sum[3] / B;
        const float loss = sum[2] / CB - sum[1] / CB;
        const float cons = ca * (lc.conservative_weight * loss - lc.alpha_threshold);
        lc.metrics[4] = td + cons;
        lc.metrics[6] = td;
        lc.metrics[7] = cons;
      }
    }
  };
  // first row the operands of the wave's k-th sub-block are loaded from: the
  // sub-block's own (rows % 32 == 0), or the last sub-block of the rows for a
  // sub-block past the end (its rows are all invalid: g' = 0); wave-uniform,
  // so every load is a scalar base plus a loop-invariant lane offset.  Loads
  // are raw and every select / scale is applied where the value is used, so
  // no load waits early
  auto sb_row = [&](int k) { return min(rb0 + T_SB * (rw + 4 * k), rows - T_SB); };
  const int nsc = (int)min(d.n_scaled, d.rows);
  auto gprime = [&](float graw, int r) {  // g' of row r from its raw load, 0 past the block
    const float v = r < nsc ? graw * gs : (CQL ? graw - gsub : graw);
    return r < rb1 ? v : 0.f;
  };
  auto lut8 = [&](uint32_t byte) {
    return *reinterpret_cast<const bf16x8*>(&L.lut[byte]);
  };

  cql_publish();  // (before the role split: one copy of the code)
  if (col) {
    // ================= col waves: R[o][i] += m^T (g' h1), S, sum g'
    f32x4 R[T_NQ];
#pragma unroll
    for (int k = 0; k < T_NQ; ++k) R[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    double s_acc = 0.0, g_acc = 0.0;
    auto load = [&](ColOps& o, int k) {
      const int bc = sb_row(k);
      // a group's 256 words are stored lane-major: o at (o & 15) 16 + (o >> 4)
      const uint32_t* mw = mtg + (bc / T_SB) * T_H;
#pragma unroll
      for (int v = 0; v < T_NQ / 4; ++v) o.mt[v] = ldo(reinterpret_cast<const uint4*>(mw), 4 * l16 + v);
      o.mq = ldo(mw, 16 * l16 + q);
      const float* hb = h1g + bc * T_H;
      const float* gb = gg + bc;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o.h[j] = ldo(hb, (uint32_t)((8 * g + j) * T_H + i0 + l16));
        o.g[j] = ldo(gb, (uint32_t)(8 * g + j));
      }
    };
    auto compute = [&](const ColOps& o, int k) {
      const int base = rb0 + T_SB * (rw + 4 * k);
      float gv[8], gh[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        gv[j] = gprime(o.g[j], base + 8 * g + j);
        gh[j] = gv[j] * o.h[j];
      }
      bf16x8 b[3];
      split8(gh, b);
      // four tiles a group, the next group's table reads issued ahead of
      // this group's MFMAs (8 operands live, not 16)
      auto rd = [&](bf16x8* a, int v) {
        const uint4 m4 = o.mt[v];
        a[0] = lut8((m4.x >> (8 * g)) & 0xFFu);
        a[1] = lut8((m4.y >> (8 * g)) & 0xFFu);
        a[2] = lut8((m4.z >> (8 * g)) & 0xFFu);
        a[3] = lut8((m4.w >> (8 * g)) & 0xFFu);
      };
      bf16x8 aa[2][4];
      rd(aa[0], 0);
#pragma unroll
      for (int v = 0; v < T_NQ / 4; ++v) {
        if (v + 1 < T_NQ / 4) rd(aa[(v + 1) & 1], v + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < 4; ++e) R[4 * v + e] = x3m16(aa[v & 1][e], b, R[4 * v + e]);
        __builtin_amdgcn_sched_barrier(0);
      }
      // S[o] for the slice's own 16 o (tile q), rows in order; sum g' (slice 0)
      const uint32_t own = o.mq >> (8 * g);
#pragma unroll
      for (int j = 0; j < 8; ++j) s_acc += (double)keep_if((own >> j) & 1u, gv[j]);
      if (q == 0 && l16 == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j) g_acc += (double)gv[j];
      }
    };
    ColOps A, B;
    load(A, 0);
    __syncthreads();  // table and parts staged (col waves only need the table)
    stamp(2);
    cql_scalars();    // (CQL: the wave sums published by the same barrier)
    stamp(3);
    // nkw sub-blocks (a multiple of 4) in chunks of four, each chunk straight-
    // line code with no branch for the compiler to sink the prefetch loads
    // into (a sub-block past the wave's last is computed too: g' = 0 there,
    // it adds zeros), scheduling barriers keeping the loads ahead of the MFMAs;
    // the chunk's last prefetch (the next chunk's first sub-block, past the
    // end after the last chunk: loaded, never used) crosses the back edge
#pragma unroll 1
    for (int k0 = 0; k0 < nkw; k0 += 4) {
#pragma unroll
      for (int kk = 0; kk < 4; kk += 2) {
        const int k = k0 + kk;
        load(B, k + 1);
        __builtin_amdgcn_sched_barrier(0);
        compute(A, k);
        __builtin_amdgcn_sched_barrier(0);
        load(A, k + 2);
        __builtin_amdgcn_sched_barrier(0);
        compute(B, k + 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    stamp(4);
#pragma unroll
    for (int tt = 0; tt < T_NQ; ++tt) L.red[rw][tt][lane] = R[tt];
    L.s[rw][lane] = s_acc;
    // sum g' of the wave's rows: lanes 0 / 16 / 32 / 48 hold their groups'
    const double g1 = __shfl(g_acc, 16, 64), g2 = __shfl(g_acc, 32, 64), g3 = __shfl(g_acc, 48, 64);
    if (lane == 0) L.g3[rw] = ((g_acc + g1) + g2) + g3;
  } else {
    // ================= row waves: dh1, dz1, db1, dW1
    // row of M-row m in half h: 8 (m >> 2) + 4 h + (m & 3), so that the
    // accumulator's rows of lane group g are rows 8 g .. 8 g + 7
    f32x4 W1acc[NDB];
#pragma unroll
    for (int db = 0; db < NDB; ++db) W1acc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
    double b1_acc = 0.0;
    auto load = [&](RowOps<NDB>& o, int k) {
      const int bc = sb_row(k);
      const uint4* mb = reinterpret_cast<const uint4*>(m2g + bc * (T_H / 32));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t r = (uint32_t)(8 * (l16 >> 2) + 4 * h + (l16 & 3));
        o.m[h][0] = ldo(mb, 2 * r);
        o.m[h][1] = ldo(mb, 2 * r + 1);
      }
      const float* hb = h1g + bc * T_H;
      const float* gb = gg + bc;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o.h[j] = ldo(hb, (uint32_t)((8 * g + j) * T_H + i0 + l16));
        o.g[j] = ldo(gb, (uint32_t)(8 * g + j));
      }
    };
    auto compute = [&](const RowOps<NDB>& o, int k) {
      const int base = rb0 + T_SB * (rw + 4 * k);
      // x of the sub-block's rows (x[row 8 g + j][16 db + (lane & 15)], shared
      // by the 16 slices: L2-resident), the first block loaded here and used
      // after the dh1 product -- not double-buffered
      const float* xb = xg + sb_row(k) * ldx;
      auto ldx8 = [&](float* xr, int db) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          xr[j] = ldo(xb, (uint32_t)((8 * g + j) * ldx + min(16 * db + l16, nin - 1)));
      };
      float xr[8];
      ldx8(xr, 0);
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      // the B operand is re-read from LDS every sub-block (hoisted out of the
      // loop it would hold 96 registers for the whole loop)
      uint32_t boff = (uint32_t)(l16 * T_BLD + 8 * g);
      asm volatile("" : "+v"(boff));
      const __bf16* bwl = &L.bw[0][boff];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        bf16x8 b[3];
#pragma unroll
        for (int pp = 0; pp < 3; ++pp)
          b[pp] = *reinterpret_cast<const bf16x8*>(bwl + pp * (T_IW * T_BLD) + 32 * s);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint4 mv = o.m[h][s >> 2];
          const uint32_t wd = (s & 3) == 0 ? mv.x : (s & 3) == 1 ? mv.y : (s & 3) == 2 ? mv.z : mv.w;
          acc[h] = x3m16(lut8((wd >> (8 * g)) & 0xFFu), b, acc[h]);
        }
      }
      // dz1 of rows 8 g + j (j = 4 h + reg) at unit i0 + l16
      float z[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = acc[j >> 2][j & 3];
        z[j] = keep_if(o.h[j] > 0.f, gprime(o.g[j], base + 8 * g + j) * v);
        b1_acc += (double)z[j];
      }
      bf16x8 za[3];
      split8(z, za);
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        if (db > 0) ldx8(xr, db);  // the later blocks one at a time (K4's 37 inputs: three)
        float xv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[j] = 16 * db + l16 < nin ? xr[j] : 0.f;
        bf16x8 xp[3];
        split8(xv, xp);
        W1acc[db] = prod6_16(za, xp, W1acc[db]);
      }
    };
    RowOps<NDB> A, B;
    load(A, 0);
    __syncthreads();  // table and parts staged
    stamp(2);
    cql_scalars();
    stamp(3);
    // nkw sub-blocks (a multiple of 4) in chunks of four, each chunk straight-
    // line code with no branch for the compiler to sink the prefetch loads
    // into (a sub-block past the wave's last is computed too: g' = 0 there,
    // it adds zeros), scheduling barriers keeping the loads ahead of the MFMAs;
    // the chunk's last prefetch (the next chunk's first sub-block, past the
    // end after the last chunk: loaded, never used) crosses the back edge
#pragma unroll 1
    for (int k0 = 0; k0 < nkw; k0 += 4) {
#pragma unroll
      for (int kk = 0; kk < 4; kk += 2) {
        const int k = k0 + kk;
        load(B, k + 1);
        __builtin_amdgcn_sched_barrier(0);
        compute(A, k);
        __builtin_amdgcn_sched_barrier(0);
        load(A, k + 2);
        __builtin_amdgcn_sched_barrier(0);
        compute(B, k + 1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    stamp(4);
#pragma unroll
    for (int db = 0; db < NDB; ++db) L.w1[rw][db][lane] = W1acc[db];
    L.b1[rw][lane] = b1_acc;
  }
  __syncthreads();
  stamp(5);

  // ---- epilogue: the four waves of each role summed in fp64, in wave order
  float* dW2 = d.dW2 + pc * (T_H * T_H);
  {
    // R: 16 tiles x 64 lanes x 4 registers = 4096 (o, i), 8 per thread
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int it = t + T_NT * e;  // (tile, lane)
      const int tt = it >> 6, ln = it & 63;
      const f32x4 a0 = L.red[0][tt][ln], a1 = L.red[1][tt][ln], a2 = L.red[2][tt][ln],
                  a3 = L.red[3][tt][ln];
      const int i = ln & 15;
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int o = 16 * tt + 4 * (ln >> 4) + reg;
        const double r = (((double)a0[reg] + (double)a1[reg]) + (double)a2[reg]) + (double)a3[reg];
        dW2[o * T_H + i0 + i] = (float)((double)w3g[o] * r);
        L.pr[o][i] = (double)W2g[o * T_H + i0 + i] * r;
      }
    }
  }
  // dW1 / db1 partials: the slice's 16 units
  {
    for (int it = t; it < NDB * 4 * 64; it += T_NT) {
      const int db = it >> 8, reg = (it >> 6) & 3, ln = it & 63;
      const double v = (((double)L.w1[0][db][ln][reg] + (double)L.w1[1][db][ln][reg]) +
                        (double)L.w1[2][db][ln][reg]) + (double)L.w1[3][db][ln][reg];
      const int i = 4 * (ln >> 4) + reg, dc = 16 * db + (ln & 15);
      if (dc < nin) d.dW1[(pc * T_H + i0 + i) * nin + dc] = (float)v;
    }
  }
  if (t < T_IW) {
    double s = 0.0;
    for (int rw2 = 0; rw2 < 4; ++rw2)
      for (int gg2 = 0; gg2 < 4; ++gg2) s += L.b1[rw2][16 * gg2 + t];
    d.db1[pc * T_H + i0 + t] = (float)s;
  }
  __syncthreads();
  // dW3 partial of the slice (one per row block and slice), db2 / db3 partials
  if (t < T_H) {
    const int o = t;
    double s3 = 0.0;
#pragma unroll
    for (int i = 0; i < T_IW; ++i) s3 += L.pr[o][i];
    if ((o >> 4) == q) {
      // this slice's own o: S in fp64 (col waves, lane groups in order)
      const int l = o & 15;
      double S = 0.0;
      for (int rw2 = 0; rw2 < 4; ++rw2)
        for (int gg2 = 0; gg2 < 4; ++gg2) S += L.s[rw2][16 * gg2 + l];
      const float* b2g = d.b2 + c * d.sb2;
      s3 += (double)b2g[o] * S;
      d.db2[pc * T_H + o] = (float)((double)w3g[o] * S);
    }
    d.dW3[((int64_t)(p * T_NQ + q) * d.C + c) * T_H + o] = (float)s3;
    if (q == 0 && t == 0) {
      d.db3[pc] = (float)(((L.g3[0] + L.g3[1]) + L.g3[2]) + L.g3[3]);
    }
  }
  stamp(6);
}

int64_t default_splits(int64_t rows, int C) {
  // about 256 workgroups (C P 16), at least 4 sub-blocks per row block
  int64_t P = 256 / (16 * (int64_t)C);
  if (P < 1) P = 1;
  const int64_t pmax = (rows + 4 * T_SB - 1) / (4 * T_SB);
  if (P > pmax) P = pmax;
  return P < 1 ? 1 : P;
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int32_t d3a_q2_bwd_x6t_splits(int64_t rows, int32_t C) {
  if (rows < 0 || C < 1) return -1;
  return (int32_t)default_splits(rows, C);
}

namespace d3a {
int launch_q2x6t_bwd(const d3a_q2_bwd_desc& d, hipStream_t st, const d3a_cql_loss_desc* lc) {
  D3A_CHECK_ARG(d.m2 && d.m2t && d.b2, "d3a_q2_bwd_x6 (transposed mask): m2, m2t and b2 are required");
  D3A_CHECK_ARG((reinterpret_cast<uintptr_t>(d.m2) & 15) == 0 && d.sm2 % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(d.m2t) & 3) == 0,
                "d3a_q2_bwd_x6: m2 must be 16-byte aligned rows of 8 words, m2t 4-byte aligned");
  D3A_CHECK_ARG(d.sm2 >= d.rows * (T_H / 32) && d.sm2t >= (d.rows + T_SB - 1) / T_SB * T_H,
                "d3a_q2_bwd_x6: mask member strides too small");
  if (d.rows == 0) return 0;  // as d3a_q2_bwd: nothing written
  D3A_CHECK_ARG(d.rows % T_SB == 0, "d3a_q2_bwd_x6 (transposed mask): rows must be a multiple of 32");
  const int64_t P = d.row_splits > 0 ? d.row_splits : default_splits(d.rows, d.C);
  D3A_CHECK_ARG(P >= 1 && P <= 4096, "d3a_q2_bwd_x6: bad row_splits");
  const int64_t rbp = ((d.rows + P - 1) / P + T_SB - 1) / T_SB * T_SB;
  D3A_CHECK_ARG(d.rows == 0 || rbp > 0, "d3a_q2_bwd_x6: bad row blocks");
  const int64_t units = P * d.C;
  const int64_t blocks = (units + 7) / 8 * 8 * T_NQ;
  D3A_CHECK_ARG(blocks < (int64_t(1) << 31), "d3a_q2_bwd_x6: too many rows");
  // sub-blocks of the busiest wave, rounded up to the chunk of four
  const int64_t nkw = ((rbp / T_SB + 3) / 4 + 3) / 4 * 4;
  const dim3 grid((unsigned)blocks), block(T_NT);
  const int ndb = (d.n_in + 15) / 16;
  const d3a_cql_loss_desc l = lc ? *lc : d3a_cql_loss_desc{};
  const int Pi = (int)P, rbpi = (int)rbp, nkwi = (int)nkw;
  static const bool stamps = [] {
    const char* e = getenv("D3A_BWD_STAMPS");
    return e && atoi(e) != 0;
  }();
  if (stamps && ndb <= 1) {  // (diagnostic: phase stamps, d3a_bwd_stamps)
    if (lc)
      hipLaunchKernelGGL((q2x6t_bwd_kernel<1, true, true>), grid, block, 0, st, d, Pi, rbpi, nkwi, l);
    else
      hipLaunchKernelGGL((q2x6t_bwd_kernel<1, false, true>), grid, block, 0, st, d, Pi, rbpi, nkwi, l);
  } else if (lc) {
    if (ndb <= 1)
      hipLaunchKernelGGL((q2x6t_bwd_kernel<1, true>), grid, block, 0, st, d, Pi, rbpi, nkwi, l);
    else if (ndb == 2)
      hipLaunchKernelGGL((q2x6t_bwd_kernel<2, true>), grid, block, 0, st, d, Pi, rbpi, nkwi, l);
    else
      hipLaunchKernelGGL((q2x6t_bwd_kernel<3, true>), grid, block, 0, st, d, Pi, rbpi, nkwi, l);
  } else if (ndb <= 1) {
    hipLaunchKernelGGL(q2x6t_bwd_kernel<1>, grid, block, 0, st, d, Pi, rbpi, nkwi, l);
  } else if (ndb == 2) {
    hipLaunchKernelGGL(q2x6t_bwd_kernel<2>, grid, block, 0, st, d, Pi, rbpi, nkwi, l);
  } else {
    hipLaunchKernelGGL(q2x6t_bwd_kernel<3>, grid, block, 0, st, d, Pi, rbpi, nkwi, l);
  }
  D3A_LAUNCH_CHECK("d3a_q2_bwd_x6");
  return 0;
}
}  // namespace d3a

extern "C" int d3a_q2_bwd_x6_cql(const d3a_q2_bwd_desc* dp, const d3a_cql_loss_desc* lc, void* stream) {
  D3A_CHECK_ARG(dp && lc, "d3a_q2_bwd_x6_cql: null desc");
  const d3a_q2_bwd_desc& d = *dp;
  D3A_CHECK_ARG(lc->split && lc->update_critic && lc->conservative && !lc->soft_target &&
                    lc->dp_phase == 0 && lc->td2 && lc->bc && lc->stage && lc->lse && lc->metrics &&
                    lc->scalars,
                "d3a_q2_bwd_x6_cql: needs a split CQL loss desc (conservative critic update, one "
                "device, no soft target) with td2, bc, stage, lse, metrics and scalars");
  D3A_CHECK_ARG(d.g == lc->dq + 3LL * lc->N * lc->B && d.n_scaled == 3LL * lc->N * lc->B &&
                    d.C == lc->C && d.rows == 3LL * lc->N * lc->B + lc->B && d.sgb == lc->R,
                "d3a_q2_bwd_x6_cql: the backward's rows must be the loss's critic set (g = dq + 3NB, "
                "n_scaled 3NB, rows 3NB + B)");
  D3A_CHECK_ARG(d.dz2 == nullptr && d.m2t != nullptr,
                "d3a_q2_bwd_x6_cql: the slice kernel (m2t set, no dz2)");
  D3A_CHECK_ARG((int64_t)lc->C * lc->B < (int64_t(1) << 30), "d3a_q2_bwd_x6_cql: C B too large");
  return launch_q2x6t_bwd(d, (hipStream_t)stream, lc);
}

// diagnostic: copy the stamp buffer of the last D3A_BWD_STAMPS=1 launch
extern "C" int d3a_bwd_stamps(unsigned long long* dst, int n) {
  D3A_CHECK_ARG(dst && n >= 0 && n <= 256 * 2 * 8, "d3a_bwd_stamps: bad arguments");
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(bwd_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) !=
      hipSuccess) {
    set_error("d3a_bwd_stamps: copy failed");
    return -2;
  }
  return 0;
}
