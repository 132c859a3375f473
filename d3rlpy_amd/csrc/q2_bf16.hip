// bf16 throughput instantiation of the Q-ensemble forward and backward
// ("fp32 for parity, bf16 for throughput"): the same
// [n_in -> 256 -> 256 -> 1] critic passes as q2_fwd.hip / q2_bwd.hip with
// every GEMM operand rounded to bf16 and fp32 accumulation on
// v_mfma_f32_32x32x16_bf16 (16 k per instruction, 32 cycles per SIMD: 16x the
// f32-input rate).  Never the parity path: the reference computes in fp32
// (encoders.py:265-275, 328-339; mean_q_function.py:255-256); this is the
// separate `bench.py --precision bf16` line with its own tolerance test.
//
// Numerics: weights and activations are rounded to bf16 (round to nearest
// even, v_cvt_pk_bf16_f32) where they enter a product; sums, biases, ReLU,
// the head dot, every gradient and every reduction stay fp32.  Activations
// kept for the backward are stored as bf16 (half the bytes): the backward's
// ReLU masks read their sign, which bf16 rounding preserves (no positive fp32
// rounds to zero: same exponent range).
//
// Fragment maps (cdna_hip_programming.md §3): lane l (r = l & 31, h = l >> 5)
// holds A[row r][k = 8h + j] and B[k = 8h + j][col r], j < 8; the accumulator
// holds column r and rows (reg & 3) + 8 (reg >> 2) + 4h.
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
void launch_q2x1_fwd(const d3a_mlp_fwd_desc& d, hipStream_t st);  // q2_x6.hip
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int B_H = 256;
constexpr int B_RB = 128;   // forward: rows per workgroup
constexpr int B_SB = 32;
constexpr int B_NSB = B_RB / B_SB;
constexpr int B_LDH = 264;  // bf16 row stride of the LDS activation image (528 B)

__device__ __forceinline__ f32x16 mfma16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 cvt8(float4 a, float4 b) {
  bf16x8 r;
  r[0] = (__bf16)a.x; r[1] = (__bf16)a.y; r[2] = (__bf16)a.z; r[3] = (__bf16)a.w;
  r[4] = (__bf16)b.x; r[5] = (__bf16)b.y; r[6] = (__bf16)b.z; r[7] = (__bf16)b.w;
  return r;
}

template <int XL>
struct FwdLdsB {
  __bf16 h[B_RB * B_LDH];  // layer-1 activations (bf16)
  union {
    __bf16 x[B_RB * (XL + 8)];  // input rows (bf16, zero-padded to XL)
    float hp[B_NSB][8][B_SB];   // head partials [sub-block][wave][row]
  } u;
};

// Forward, same contract as d3a_mlp_fwd (mlp_fused.hip) for [n_in <= 48, 256,
// 256, 1] except that h[0] / h[1] receive bf16 rows (__bf16 [C][rows][256]).
// Workgroup = 128 rows of member blockIdx.z; wave w owns units 32 w .. + 31 of
// both hidden layers and computes the transposed tiles C^T[unit][row] (W as
// the A operand from registers, activation rows as B from LDS), so a lane
// holds one row and four runs of four consecutive units.
// PROBE (timing probes only, D3A_FWDB_PROBE): bit 0 skips the kept-activation
// stores, bit 1 loads one W1 fragment pair and replicates it, bit 2 skips the
// layer-2 MFMAs.
template <int XL, int PROBE = 0>
__global__ __launch_bounds__(512) void q2_fwd_bf16_kernel(d3a_mlp_fwd_desc d) {
  constexpr int LDX = XL + 8;
  constexpr int NS0 = XL / 16;  // layer-1 MFMA steps
  __shared__ __attribute__((aligned(16))) FwdLdsB<XL> L;
  static_assert(sizeof(FwdLdsB<XL>) <= 163840, "LDS");
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int c = blockIdx.z;
  const int nb_main = (int)((d.rows + B_RB - 1) / B_RB);
  const bool aux = (int)blockIdx.x >= nb_main;
  const int m0 = aux ? ((int)blockIdx.x - nb_main) * B_RB : (int)d.r0 + (int)blockIdx.x * B_RB;
  const int rend = aux ? (int)d.aux_rows : (int)(d.r0 + d.rows);
  const int h_from = aux ? rend : (int)d.h_from;
  const int64_t wdel = aux ? d.aux_wdelta : 0;
  float* const outp = aux ? d.aux_out + c * d.aux_sout : d.out + c * d.sout;
  const int nin = d.n_in;
  const int col = 32 * w + li;  // A-operand row (unit) of this lane
  __bf16* const h0g = (!aux && d.h[0]) ? reinterpret_cast<__bf16*>(d.h[0]) + c * d.sh : nullptr;
  __bf16* const h1g = (!aux && d.h[1]) ? reinterpret_cast<__bf16*>(d.h[1]) + c * d.sh : nullptr;

  // ---- prologue, loads in the order they are needed (the vector memory
  // counter retires in order): the input rows, W0, then W1 as raw fp32 -- W1 is
  // converted to bf16 fragments only after layer 1, so its 256 KB per workgroup
  // streams in behind the input staging and the first layer
  const float* xb = aux ? d.aux_x + c * d.aux_sxb : d.x + c * d.sxb;
  const int64_t ldx = aux ? d.aux_ldx : d.ldx;
  constexpr int X4 = XL / 4;
  constexpr int XS = (B_RB * X4 + 511) / 512;  // float4 pieces of x per thread
  float xv[XS][4];
#pragma unroll
  for (int i = 0; i < XS; ++i) {
    const int e = t + 512 * i;
    const int m = e / X4, k4 = (e - m * X4) * 4;
    const int r = m0 + m;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      xv[i][j] = (e < B_RB * X4 && r < rend && k4 + j < nin) ? xb[r * ldx + k4 + j] : 0.f;
  }
  const float* W0 = d.W[0] + wdel + c * d.sW[0];
  bf16x8 w0f[NS0];
#pragma unroll
  for (int s = 0; s < NS0; ++s) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * s + 8 * lh + j;
      w0f[s][j] = (__bf16)(k < nin ? W0[col * nin + k] : 0.f);
    }
  }
  const float* W1 = d.W[1] + wdel + c * d.sW[1];
  float4 w1raw[32];  // step s: W1[col][16 s + 8 lh + 0..7] as two float4
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const float* p = W1 + col * B_H + 16 * ((PROBE & 2) ? 0 : s) + 8 * lh;
    w1raw[2 * s] = *reinterpret_cast<const float4*>(p);
    w1raw[2 * s + 1] = *reinterpret_cast<const float4*>(p + 4);
  }
  const float b2v = (d.b[2] + wdel + c * d.sb[2])[0];
#pragma unroll
  for (int i = 0; i < XS; ++i) {
    const int e = t + 512 * i;
    if (e < B_RB * X4) {
      const int m = e / X4, k4 = (e - m * X4) * 4;
      bf16x4 b;
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = (__bf16)xv[i][j];
      *reinterpret_cast<bf16x4*>(&L.u.x[m * LDX + k4]) = b;
    }
  }
  __syncthreads();

  auto unit_of = [&](int R) { return 32 * w + 8 * R + 4 * lh; };
  float bb[16], ww[16];
  auto load_units = [&](const float* src, float* dst) {
#pragma unroll
    for (int R = 0; R < 4; ++R) {
      const float4 v = *reinterpret_cast<const float4*>(src + unit_of(R));
      dst[4 * R] = v.x; dst[4 * R + 1] = v.y; dst[4 * R + 2] = v.z; dst[4 * R + 3] = v.w;
    }
  };
  auto kept = [&](const void* base, int rb) {
    const int row = rb + li;
    return base != nullptr && row >= h_from && row < rend;
  };
  auto put4 = [&](__bf16* dst, const float* v) {  // 4 consecutive units, 8 bytes
    bf16x4 b;
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = (__bf16)v[j];
    *reinterpret_cast<bf16x4*>(dst) = b;
  };

  // ---- layer 1: four 32-row tiles
  load_units(d.b[0] + wdel + c * d.sb[0], bb);
#pragma unroll 1
  for (int tt = 0; tt < B_NSB; ++tt) {
    f32x16 a0;
#pragma unroll
    for (int r = 0; r < 16; ++r) a0[r] = 0.f;
#pragma unroll
    for (int s = 0; s < NS0; ++s)
      a0 = mfma16(w0f[s], *reinterpret_cast<const bf16x8*>(&L.u.x[(tt * B_SB + li) * LDX + 16 * s + 8 * lh]), a0);
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = fmaxf(a0[r] + bb[r], 0.f);
    __bf16* hl = &L.h[(tt * B_SB + li) * B_LDH];
#pragma unroll
    for (int R = 0; R < 4; ++R) put4(hl + unit_of(R), v + 4 * R);
  }
  load_units(d.b[1] + wdel + c * d.sb[1], bb);
  load_units(d.W[2] + wdel + c * d.sW[2], ww);
  bf16x8 w1f[16];  // step s: W1[col][16 s + 8 lh + j]
#pragma unroll
  for (int s = 0; s < 16; ++s) w1f[s] = cvt8(w1raw[2 * s], w1raw[2 * s + 1]);
  __syncthreads();  // layer-1 rows in LDS; x dead (hp aliases it)

  // h[0] leaves from LDS: wave w copies rows 16 w .. 16 w + 15 (two rows of
  // 512 B per instruction)
  if (h0g && !(PROBE & 1)) {
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
      const int rl = 16 * w + j + lh;
      const int row = m0 + rl;
      if (row >= h_from && row < rend)
        *reinterpret_cast<bf16x8*>(h0g + row * B_H + 8 * li) =
            *reinterpret_cast<const bf16x8*>(&L.h[rl * B_LDH + 8 * li]);
    }
  }

  // ---- layer 2 per 32-row tile: 16 MFMAs, then the epilogue
#pragma unroll 1
  for (int s = 0; s < B_NSB; ++s) {
    const __bf16* Bp = &L.h[(s * B_SB + li) * B_LDH + 8 * lh];
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // the tile's 16 B fragments read ahead of its MFMA chain (LDS latency paid
    // once per tile, not per MFMA)
    bf16x8 bf[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) bf[k] = *reinterpret_cast<const bf16x8*>(Bp + 16 * k);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (PROBE & 4) {
        acc[k] += (float)bf[k][0] * (float)w1f[k][1];
      } else {
        acc = mfma16(w1f[k], bf[k], acc);
      }
    }
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = fmaxf(acc[r] + bb[r], 0.f);
    const int rb = m0 + s * B_SB;
    if (kept(h1g, rb) && !(PROBE & 1)) {
#pragma unroll
      for (int R = 0; R < 4; ++R) put4(h1g + (rb + li) * B_H + unit_of(R), v + 4 * R);
    }
    float hs = v[0] * ww[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) hs = fmaf(v[r], ww[r], hs);
    const float o = __shfl_xor(hs, 32, 64);
    if (lh == 0) L.u.hp[s][w][li] = hs + o;
  }
  __syncthreads();
  if (t < B_RB) {
    const int sb = t / B_SB, rl = t % B_SB;
    float q = L.u.hp[sb][0][rl];
#pragma unroll
    for (int v = 1; v < 8; ++v) q += L.u.hp[sb][v][rl];
    const int row = m0 + t;
    if (row < rend) outp[(int64_t)row * d.ldout] = q + b2v;
  }
}

// ---------------------------------------------------------------------------
// Backward, same contract as d3a_q2_bwd (q2_bwd.hip) except that h1 / h2 are
// bf16 rows (__bf16 [C][rows][256], as d3a_q2_fwd_bf16 keeps them).  Per row:
//   g' = g (* gscale for r < n_scaled)
//   dz2 = g' w3 [h2 > 0]            dW3 = g' h2, db3 = g', db2 = dz2
//   dz1 = (dz2 W2) [h1 > 0]         dW2 = dz2^T h1, db1 = dz1, dW1 = dz1^T x
// Workgroup = 256 rows (one partial) of member c and a quarter q (64 units) of
// layer 1, walked in 32-row sub-blocks.  Per sub-block, all from LDS images
// staged one sub-block ahead (global loads two ahead):
//   waves 0, 1  dh1[32 rows][32 units] = dz2 W2[:, units]  (16 MFMAs, W2 in
//               registers), ReLU mask, dz1 to LDS (transposed), db1
//   every wave  dW2[64 w' .. 32-o block][quarter] += dz2^T h1  (2 tiles, K 32)
//   waves 2..   dW1[quarter][d block] += dz1^T x of the previous sub-block
// dz2 is formed while staging (thread = one o, 16 rows): its fp32 column sums
// (db2, dW3 of the quarter's o, db3) accumulate in fixed order.
constexpr int BB_RB = 256;   // rows per workgroup (one gradient partial)
constexpr int BB_SB = 32;
constexpr int BB_NSB = BB_RB / BB_SB;
constexpr int BB_LDR = 264;  // dz2 row image stride (bf16)
constexpr int BB_LDT = 40;   // transposed images: 32 rows + 8 (80 B rows)

template <int XB>  // XB: x columns padded to 32 (32 or 64)
struct BwdLdsB {
  __bf16 dzr[2][BB_SB * BB_LDR];   // dz2[row][o]
  __bf16 dzt[2][B_H * BB_LDT];     // dz2[o][row]
  __bf16 h1t[2][64 * BB_LDT];      // h1[row][i0 + i] as [i][row]
  __bf16 xt[3][XB * BB_LDT];       // x[row][d] as [d][row] (d >= n_in: 0)
  __bf16 z1t[2][64 * BB_LDT];      // dz1[row][i] as [i][row]
  double red[2][256];              // epilogue column sums
};

// PROBE (timing probes only, D3A_BF16_PROBE): bit 0 skips the sub-block
// loads, bit 1 the LDS staging, bit 2 the MFMA work of the loop
template <int XB, int PROBE = 0>
__global__ __launch_bounds__(512) void q2_bwd_bf16_kernel(d3a_q2_bwd_desc d) {
  constexpr int NDB = XB / 32;
  __shared__ __attribute__((aligned(16))) BwdLdsB<XB> L;
  static_assert(sizeof(BwdLdsB<XB>) <= 163840, "LDS");
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lh = lane >> 5;
  // quarters of one (row block, member) unit on one XCD (speed only)
  const int64_t P = (d.rows + BB_RB - 1) / BB_RB;
  const int64_t nunits = P * d.C;
  const int bid = blockIdx.x;
  const int kx = bid >> 3;
  const int q = kx & 3;
  const int64_t u = (int64_t)(kx >> 2) * 8 + (bid & 7);
  if (u >= nunits) return;
  const int64_t p = u / d.C;
  const int c = (int)(u - p * d.C);
  const int rows = (int)d.rows;
  const int rb0 = (int)p * BB_RB;
  const int i0 = 64 * q;
  const int nin = d.n_in;
  const __bf16* h1g = reinterpret_cast<const __bf16*>(d.h1) + c * d.sh;
  const __bf16* h2g = reinterpret_cast<const __bf16*>(d.h2) + c * d.sh;
  const float* gg = d.g + c * d.sgb;
  const float* xg = d.x + c * d.sxb;
  const float* W2g = d.W2 + c * d.sW2;
  const float gs = __builtin_bit_cast(
      float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, d.gscale ? *d.gscale : 1.f)));
  const int64_t pc = p * d.C + c;

  // x images: columns past n_in stay zero
  for (int e = t; e < 3 * XB * BB_LDT; e += 512) (&L.xt[0][0])[e] = (__bf16)0.f;

  // ---- staging (thread: dz2 column o = t & 255, rows 16 (w >> 2) .. + 15;
  // h1 unit i = t & 63, rows 4 (t >> 6) .. + 3; x element(s) t, t + 512, ..).
  // The g rows are wave-uniform (scalar loads); h2 / h1 values stay packed.
  const int so = t & 255, sr = 16 * (w >> 2);
  const int hi = t & 63, hr = 4 * w;  // (t >> 6 == w: wave-uniform rows)
  const float w3o = (d.w3 + c * d.sw3)[so];
  constexpr int XE = (BB_SB * (XB < 48 ? XB : 48) + 511) / 512;  // x elements per thread
  struct Stage {
    unsigned h2[8];  // bf16 pairs, rows sr + 2j, sr + 2j + 1
    unsigned h1[2];
    float x[XE];
  };
  const unsigned short* h2u = reinterpret_cast<const unsigned short*>(h2g);
  const unsigned short* h1u = reinterpret_cast<const unsigned short*>(h1g);
  auto clamp_row = [&](int r) { return r < rows ? r : rows - 1; };
  // row indices are wave-uniform (sr, hr from the wave index), so each load is
  // a scalar row base plus the lane's 32-bit column offset (no per-lane 64-bit
  // address arithmetic: the staging is VALU-bound)
  auto load_stage = [&](Stage& S, int sb) {
    const int base = __builtin_amdgcn_readfirstlane(rb0 + sb * BB_SB);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned short* ra = h2u + (size_t)clamp_row(base + sr + 2 * j) * B_H;
      const unsigned short* rb = h2u + (size_t)clamp_row(base + sr + 2 * j + 1) * B_H;
      S.h2[j] = (unsigned)ra[so] | ((unsigned)rb[so] << 16);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const unsigned short* ra = h1u + (size_t)clamp_row(base + hr + 2 * j) * B_H + i0;
      const unsigned short* rb = h1u + (size_t)clamp_row(base + hr + 2 * j + 1) * B_H + i0;
      S.h1[j] = (unsigned)ra[hi] | ((unsigned)rb[hi] << 16);
    }
#pragma unroll
    for (int k = 0; k < XE; ++k) {
      const int e = t + 512 * k;
      const int row = e % BB_SB, col = e / BB_SB;
      S.x[k] = (col < nin) ? xg[(int64_t)clamp_row(base + row) * d.ldx + col] : 0.f;
    }
  };
  // column sums of the quarter's o (db2, dW3), db3 (thread so == 0 of each half)
  double s_db2 = 0.0, s_dw3 = 0.0, s_db3 = 0.0;
  const bool own_o = (so >> 6) == q;
  const int n_scaled32 = d.n_scaled < (int64_t)rows ? (int)d.n_scaled : rows;
  auto write_stage = [&](const Stage& S, int sb) {
    const int b2 = sb & 1;
    const int base = rb0 + sb * BB_SB;
    // g of the wave's 16 rows (uniform: scalar loads), all issued before the
    // first LDS store -- scalar loads and LDS ops share one counter, so a
    // scalar load behind LDS stores waits for them all
    const int gr0 = __builtin_amdgcn_readfirstlane(base + sr);
    float gv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) gv[j] = gg[gr0 + j < rows ? gr0 + j : rows - 1];
    __builtin_amdgcn_sched_barrier(0);
    // row factors: 0 past the last row, gscale on the scaled rows (uniform
    // selects on scalar registers, one multiply per row)
    // per element ~6 VALU (the staging is VALU-bound: 4 cycles per wave-wide
    // VALU instruction, two waves per SIMD): the row factors g' w3[o] formed
    // once per row (row index and bounds are wave-uniform, so their tests are
    // scalar), fp32 sums over the sub-block's 16 rows, one fp64 accumulation
    // per sub-block
    float dz[16];
    float f_db2 = 0.f, f_dw3 = 0.f, f_db3 = 0.f;
    const int nsc = n_scaled32, gl = rows - gr0;  // rows gr0 + j valid for j < gl
    float gp[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float mult = j < gl ? (gr0 + j < nsc ? gs : 1.f) : 0.f;
      gp[j] = gv[j] * mult;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const unsigned pk = S.h2[j >> 1];
      const unsigned bits = (j & 1) ? (pk & 0xffff0000u) : (pk << 16);
      const float h2v = __builtin_bit_cast(float, bits);  // (rows past the end: gp = 0)
      dz[j] = (int)bits > 0 ? gp[j] * w3o : 0.f;  // h2 > 0 (bf16 sign, nonzero)
      f_db2 += dz[j];
      f_dw3 = fmaf(gp[j], h2v, f_dw3);
      f_db3 += gp[j];
    }
    if (own_o) {
      s_db2 += (double)f_db2;
      s_dw3 += (double)f_dw3;
    }
    if (so == 0) s_db3 += (double)f_db3;
    bf16x8 v0, v1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v0[j] = (__bf16)dz[j];
      v1[j] = (__bf16)dz[8 + j];
    }
    if constexpr (!(PROBE & 8)) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        L.dzr[b2][(sr + j) * BB_LDR + so] = v0[j];
        L.dzr[b2][(sr + 8 + j) * BB_LDR + so] = v1[j];
      }
    } else {
      s_db3 += (double)(float)v0[0] + (double)(float)v1[7];
    }
    if constexpr (!(PROBE & 16)) {
      *reinterpret_cast<bf16x8*>(&L.dzt[b2][so * BB_LDT + sr]) = v0;
      *reinterpret_cast<bf16x8*>(&L.dzt[b2][so * BB_LDT + sr + 8]) = v1;
    } else {
      s_db3 += (double)(float)v0[3] + (double)(float)v1[4];
    }
    unsigned hv[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      unsigned v = S.h1[j];
      if (base + hr + 2 * j >= rows) v &= 0xffff0000u;
      if (base + hr + 2 * j + 1 >= rows) v &= 0x0000ffffu;
      hv[j] = v;
    }
    *reinterpret_cast<uint2*>(&L.h1t[b2][hi * BB_LDT + hr]) = make_uint2(hv[0], hv[1]);
#pragma unroll
    for (int k = 0; k < XE; ++k) {
      const int e = t + 512 * k;
      const int row = e % BB_SB, col = e / BB_SB;
      if (col < nin)
        L.xt[sb % 3][col * BB_LDT + row] = (__bf16)(base + row < rows ? S.x[k] : 0.f);
    }
  };

  // ---- W2 fragments of the dh1 waves: B[k = o][col = unit], step k:
  // W2[16 k + 8 lh + j][i0 + 32 w + li]
  bf16x8 w2f[16];
  if (w < 2) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        w2f[k][j] = (__bf16)W2g[(16 * k + 8 * lh + j) * B_H + i0 + 32 * w + li];
  }

  f32x16 aw2[2];  // dW2 tiles (o block w, unit blocks 0 / 1)
  f32x16 aw1[NDB];  // dW1 tiles of waves 2, 3 (unit block w - 2, d blocks)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    aw2[0][r] = aw2[1][r] = 0.f;
#pragma unroll
    for (int k = 0; k < NDB; ++k) aw1[k][r] = 0.f;
  }
  float s_db1 = 0.f;  // waves 0, 1: this lane's unit, over its rows

  Stage S0, S1;
  load_stage(S0, 0);
  load_stage(S1, 1);
  __syncthreads();  // x images zeroed
  write_stage(S0, 0);
  load_stage(S0, 2);
  __syncthreads();

  auto dw1_step = [&](int sb) {  // waves 2, 3: dW1 over sub-block sb
    const int ib = w - 2;
    const __bf16* A = &L.z1t[sb & 1][(32 * ib + li) * BB_LDT + 8 * lh];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + 16 * s2);
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(
            &L.xt[sb % 3][(32 * db + li) * BB_LDT + 16 * s2 + 8 * lh]);
        aw1[db] = mfma16(a, b, aw1[db]);
      }
    }
  };

#pragma unroll 1
  for (int sb = 0; sb < BB_NSB; ++sb) {
    const int b2 = sb & 1;
    Stage& Sn = (sb & 1) ? S0 : S1;  // holds sub-block sb + 1
    Stage& Sl = (sb & 1) ? S1 : S0;  // to be loaded with sub-block sb + 3
    (void)Sl;
    // (a) dh1 -> dz1 (waves 0, 1)
    if (w < 2 && !(PROBE & 4)) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const __bf16* A = &L.dzr[b2][li * BB_LDR + 8 * lh];
#pragma unroll
      for (int k = 0; k < 16; ++k) acc = mfma16(*reinterpret_cast<const bf16x8*>(A + 16 * k), w2f[k], acc);
      // lane: unit i = 32 w + li, rows (r & 3) + 8 (r >> 2) + 4 lh
      const __bf16* hm = &L.h1t[b2][(32 * w + li) * BB_LDT];
      __bf16* zo = &L.z1t[b2][(32 * w + li) * BB_LDT];
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const int r0 = 8 * R + 4 * lh;
        const bf16x4 m = *reinterpret_cast<const bf16x4*>(hm + r0);
        bf16x4 z;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = (float)m[j] > 0.f ? acc[4 * R + j] : 0.f;
          s_db1 += v;
          z[j] = (__bf16)v;
        }
        *reinterpret_cast<bf16x4*>(zo + r0) = z;
      }
    }
    // (b) dW2[o block w][quarter] += dz2^T h1 over the sub-block's 32 rows
    if (!(PROBE & 4)) {
      const __bf16* A = &L.dzt[b2][(32 * w + li) * BB_LDT + 8 * lh];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + 16 * s2);
#pragma unroll
        for (int ib = 0; ib < 2; ++ib) {
          const bf16x8 b = *reinterpret_cast<const bf16x8*>(
              &L.h1t[b2][(32 * ib + li) * BB_LDT + 16 * s2 + 8 * lh]);
          aw2[ib] = mfma16(a, b, aw2[ib]);
        }
      }
    }
    // (c) dW1 of the previous sub-block (its dz1 met at the last barrier)
    if (w >= 2 && w < 4 && sb > 0 && !(PROBE & 4)) dw1_step(sb - 1);
    // staging: sub-block sb + 1 to LDS, sub-block sb + 3 into registers
    if (sb + 1 < BB_NSB && !(PROBE & 2)) write_stage(Sn, sb + 1);
    if (sb + 3 < BB_NSB && !(PROBE & 1)) load_stage(Sn, sb + 3);
    __syncthreads();
  }
  if (w >= 2 && w < 4) dw1_step(BB_NSB - 1);

  // ---- epilogue
  float* dW2 = d.dW2 + pc * (B_H * B_H);
#pragma unroll
  for (int ib = 0; ib < 2; ++ib)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int o = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * lh;
      dW2[o * B_H + i0 + 32 * ib + li] = aw2[ib][r];
    }
  if (w >= 2 && w < 4) {
    const int ib = w - 2;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = 32 * ib + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const int dc = 32 * db + li;
        if (dc < nin) d.dW1[(pc * B_H + i0 + i) * nin + dc] = aw1[db][r];
      }
  }
  if (w < 2) {
    const float o = __shfl_xor(s_db1, 32, 64);
    if (lh == 0) d.db1[pc * B_H + i0 + 32 * w + li] = s_db1 + o;
  }
  // column sums: the two row halves of each o (t >> 8 = 0 first)
  L.red[0][t & 255] = 0.0;
  __syncthreads();
  if (t >= 256) {
    L.red[0][so] = s_db2;
    L.red[1][so] = s_dw3;
  }
  __syncthreads();
  if (t < 256 && own_o) {
    d.db2[pc * B_H + so] = (float)(s_db2 + L.red[0][so]);
    d.dW3[pc * B_H + so] = (float)(s_dw3 + L.red[1][so]);
  }
  __syncthreads();
  if (t == 256) L.red[0][0] = s_db3;
  __syncthreads();
  if (t == 0 && q == 0) d.db3[pc] = (float)(s_db3 + L.red[0][0]);
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_q2_fwd_bf16(const d3a_mlp_fwd_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_q2_fwd_bf16: null desc");
  D3A_CHECK_ARG(dp->row_mean == nullptr, "d3a_q2_fwd_bf16: row_mean is d3a_mlp_fwd_x6 only");
  D3A_CHECK_ARG(dp->xg_mode == 0, "d3a_q2_fwd_bf16: no input-row builder (xg_mode)");
  D3A_CHECK_ARG(dp->hmask == nullptr, "d3a_q2_fwd_bf16: hmask is d3a_q2_fwd_x6 only");
  const d3a_mlp_fwd_desc& d = *dp;
  D3A_CHECK_ARG(d.x && d.out, "d3a_q2_fwd_bf16: null input / output");
  D3A_CHECK_ARG(d.n_hidden == 2 && d.H == B_H && d.n_out == 1,
                "d3a_q2_fwd_bf16: network must be [n_in, 256, 256, 1]");
  D3A_CHECK_ARG(d.n_in >= 1 && d.n_in <= 48, "d3a_q2_fwd_bf16: n_in must be 1..48");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0 && d.aux_rows >= 0 && d.h_from >= 0, "d3a_q2_fwd_bf16: bad sizes");
  for (int l = 0; l < 3; ++l) D3A_CHECK_ARG(d.W[l] && d.b[l], "d3a_q2_fwd_bf16: null layer parameters");
  auto a16 = [](const void* p, int64_t stride) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && stride % 4 == 0;
  };
  D3A_CHECK_ARG(a16(d.W[1], d.sW[1]) && a16(d.b[0], d.sb[0]) && a16(d.b[1], d.sb[1]) &&
                    a16(d.W[2], d.sW[2]),
                "d3a_q2_fwd_bf16: W1, b0, b1 and the head row must be 16-byte aligned");
  D3A_CHECK_ARG(d.aux_rows == 0 || (d.aux_x && d.aux_out && d.aux_wdelta % 4 == 0),
                "d3a_q2_fwd_bf16: bad aux pass");
  D3A_CHECK_ARG((d.h[0] == nullptr || (reinterpret_cast<uintptr_t>(d.h[0]) & 15) == 0) &&
                    (d.h[1] == nullptr || (reinterpret_cast<uintptr_t>(d.h[1]) & 15) == 0) &&
                    d.sh % 8 == 0,
                "d3a_q2_fwd_bf16: bf16 activation buffers must be 16-byte aligned");
  const int64_t rmax = (d.r0 + d.rows) > d.aux_rows ? (d.r0 + d.rows) : d.aux_rows;
  D3A_CHECK_ARG(rmax * B_H < (int64_t(1) << 31) && rmax * d.ldout < (int64_t(1) << 31) &&
                    (d.r0 + d.rows) * d.ldx < (int64_t(1) << 31) &&
                    d.aux_rows * d.aux_ldx < (int64_t(1) << 31),
                "d3a_q2_fwd_bf16: rows x row stride exceeds 2^31");
  if (d.rows == 0 && d.aux_rows == 0) return 0;
  const int64_t nb = (d.rows + B_RB - 1) / B_RB + (d.aux_rows + B_RB - 1) / B_RB;
  const dim3 grid((unsigned)nb, 1, (unsigned)d.C);
  const int xl = (d.n_in + 15) / 16 * 16;
  hipStream_t st = (hipStream_t)stream;
  static const int probe = [] {
    const char* e = getenv("D3A_FWDB_PROBE");
    return e ? atoi(e) : 0;
  }();
  // default: the split-bf16 kernel's structure with one part (q2_x6.hip);
  // D3A_FWDB_OLD=1 selects this file's round-3 kernel (A/B timing)
  static const bool old = [] {
    const char* e = getenv("D3A_FWDB_OLD");
    return e && atoi(e) != 0;
  }();
  if (!old && !probe) {
    launch_q2x1_fwd(d, st);
  } else if (probe && xl == 16) {
    switch (probe) {
      case 1: hipLaunchKernelGGL((q2_fwd_bf16_kernel<16, 1>), grid, dim3(512), 0, st, d); break;
      case 2: hipLaunchKernelGGL((q2_fwd_bf16_kernel<16, 2>), grid, dim3(512), 0, st, d); break;
      case 3: hipLaunchKernelGGL((q2_fwd_bf16_kernel<16, 3>), grid, dim3(512), 0, st, d); break;
      case 4: hipLaunchKernelGGL((q2_fwd_bf16_kernel<16, 4>), grid, dim3(512), 0, st, d); break;
      default: hipLaunchKernelGGL((q2_fwd_bf16_kernel<16, 7>), grid, dim3(512), 0, st, d); break;
    }
  } else if (xl == 16)
    hipLaunchKernelGGL(q2_fwd_bf16_kernel<16>, grid, dim3(512), 0, st, d);
  else if (xl == 32)
    hipLaunchKernelGGL(q2_fwd_bf16_kernel<32>, grid, dim3(512), 0, st, d);
  else
    hipLaunchKernelGGL(q2_fwd_bf16_kernel<48>, grid, dim3(512), 0, st, d);
  D3A_LAUNCH_CHECK("d3a_q2_fwd_bf16");
  return 0;
}

extern "C" int d3a_q2_bwd_bf16(const d3a_q2_bwd_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_q2_bwd_bf16: null desc");
  const d3a_q2_bwd_desc& d = *dp;
  D3A_CHECK_ARG(d.x && d.h1 && d.h2 && d.g && d.W2 && d.w3, "d3a_q2_bwd_bf16: null input");
  D3A_CHECK_ARG(d.m2 == nullptr, "d3a_q2_bwd_bf16: the mask image is d3a_q2_bwd_x6 only");
  D3A_CHECK_ARG(d.dW1 && d.db1 && d.dW2 && d.db2 && d.dW3 && d.db3, "d3a_q2_bwd_bf16: null output");
  D3A_CHECK_ARG(d.n_in >= 1 && d.n_in <= 48, "d3a_q2_bwd_bf16: n_in must be 1..48");
  D3A_CHECK_ARG(d.dz2 == nullptr && (d.block_rows == 0 || d.block_rows == 256),
                "d3a_q2_bwd_bf16: dz2 / block_rows are fp32-only (d3a_q2_bwd)");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0 && d.n_scaled >= 0, "d3a_q2_bwd_bf16: bad sizes");
  D3A_CHECK_ARG(d.ldh == B_H, "d3a_q2_bwd_bf16: h1 / h2 must be rows of 256 bf16");
  D3A_CHECK_ARG(d.rows * (d.ldx > B_H ? d.ldx : B_H) < (int64_t(1) << 31),
                "d3a_q2_bwd_bf16: rows x row stride exceeds 2^31");
  if (d.rows == 0) return 0;
  const int64_t units = ((d.rows + BB_RB - 1) / BB_RB) * d.C;
  const int64_t blocks = (units + 7) / 8 * 32;
  D3A_CHECK_ARG(blocks < (int64_t(1) << 31), "d3a_q2_bwd_bf16: too many rows");
  const dim3 grid((unsigned)blocks), block(512);
  static const int probe = [] {
    const char* e = getenv("D3A_BF16_PROBE");
    return e ? atoi(e) : 0;
  }();
  if (probe && d.n_in <= 32) {
    hipStream_t st = (hipStream_t)stream;
    switch (probe) {
      case 1: hipLaunchKernelGGL((q2_bwd_bf16_kernel<32, 1>), grid, block, 0, st, d); break;
      case 2: hipLaunchKernelGGL((q2_bwd_bf16_kernel<32, 2>), grid, block, 0, st, d); break;
      case 3: hipLaunchKernelGGL((q2_bwd_bf16_kernel<32, 3>), grid, block, 0, st, d); break;
      case 4: hipLaunchKernelGGL((q2_bwd_bf16_kernel<32, 4>), grid, block, 0, st, d); break;
      case 8: hipLaunchKernelGGL((q2_bwd_bf16_kernel<32, 8>), grid, block, 0, st, d); break;
      case 16: hipLaunchKernelGGL((q2_bwd_bf16_kernel<32, 16>), grid, block, 0, st, d); break;
      case 24: hipLaunchKernelGGL((q2_bwd_bf16_kernel<32, 24>), grid, block, 0, st, d); break;
      default: hipLaunchKernelGGL((q2_bwd_bf16_kernel<32, 7>), grid, block, 0, st, d); break;
    }
    D3A_LAUNCH_CHECK("d3a_q2_bwd_bf16");
    return 0;
  }
  if (d.n_in <= 32)
    hipLaunchKernelGGL(q2_bwd_bf16_kernel<32>, grid, block, 0, (hipStream_t)stream, d);
  else
    hipLaunchKernelGGL(q2_bwd_bf16_kernel<64>, grid, block, 0, (hipStream_t)stream, d);
  D3A_LAUNCH_CHECK("d3a_q2_bwd_bf16");
  return 0;
}
