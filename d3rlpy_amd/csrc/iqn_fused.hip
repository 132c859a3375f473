// The IQN head's forward in one launch: the cosine prior, the embedding
// Linear + ReLU and the head's product and Linear, per quantile row,
//
//   prior[r][e] = cos(pi (e + 1) tau[r])                      e < E
//   phi[r][u]   = relu(sum_e prior[r][e] We[u][e] + be[u])    u < F
//   q[r][a]     = sum_u (h[b(r)][u] * phi[r][u]) Wf[a][u] + bf[a]
//
// (compute_iqn_feature, iqn_q_function.py:33-47, and DiscreteIQNQFunction.
// _compute_quantiles, iqn_q_function.py:82-88).  d3a_iqn_prior + the embed
// GEMM + d3a_iqn_head_fwd wrote prior and phi ([rows][512] fp32: 268 MB for
// K5's 131,072 online rows) and read them back; here phi stays in registers
// and prior / phi are written only for the rows a backward needs (n_keep).
//
// The embedding product runs on the bf16 matrix cores with exact three-way
// split-bf16 operands (x6.hpp: fp32-accurate).  A workgroup of F / 64 waves
// walks row tiles of 32 rows; wave w owns units 64 w .. 64 w + 63 (two 32-unit
// chunks) with its We rows split once into registers, and computes the
// transposed tiles C^T[unit][row] (We the A operand, the tile's prior the B
// operand from LDS), so a lane holds one row and 16 units per chunk: the
// ReLU, the product with h (one b per tile: K % 32 == 0) and the dot with Wf
// are register work, the per-row sums meet across waves in LDS (in wave order).
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"
#include "iqn_cos.hpp"

namespace d3a {
namespace {

using namespace x6;

constexpr int IF_RB = 32;       // rows per tile
constexpr int IF_E = 64;        // embedding size (the factory default)
constexpr int IF_LDP = IF_E + 8;  // bf16 row stride of the prior image
constexpr int IF_AMAX = 8;      // actions handled here
constexpr int IF_FMAX = 512;

struct IfLds {
  __bf16 pr[2][3][IF_RB * IF_LDP];         // prior parts [buf][part][row][e]
  float qp[IF_FMAX / 64][IF_AMAX][IF_RB];  // per-wave head sums [wave][a][row]
  float be[IF_FMAX], wf[IF_AMAX][IF_FMAX];
};

// AM: the action loop's bound (4 or 8; wf rows a >= A are zero in LDS)
template <int AM>
__global__ __launch_bounds__(512) void iqn_embed_head_kernel(d3a_iqn_embed_head_desc d) {
  __shared__ __attribute__((aligned(16))) IfLds L;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int nw = blockDim.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int F = d.F, A = d.A;
  const int64_t ntiles = (d.rows + IF_RB - 1) / IF_RB;

  // ---- prologue: bias / head rows to LDS; this wave's We rows split in registers
  for (int i = t; i < F; i += blockDim.x) L.be[i] = d.be[i];
  for (int i = t; i < IF_AMAX * F; i += blockDim.x) {
    const int a = i / F;
    L.wf[a][i - a * F] = a < A ? d.Wf[i] : 0.f;
  }
  bf16x8 wa[2][IF_E / 16][3];
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    const float* wr = d.We + (int64_t)(64 * w + 32 * ch + li) * IF_E + 8 * lh;
#pragma unroll
    for (int s = 0; s < IF_E / 16; ++s) {
      const float4 x0 = *reinterpret_cast<const float4*>(wr + 16 * s);
      const float4 x1 = *reinterpret_cast<const float4*>(wr + 16 * s + 4);
      const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      split8(v, wa[ch][s]);
    }
  }
  const float pi_f = 3.14159265358979323846f;

  // the prior of a tile: 32 rows x 64 values, four per thread (row t >> 4,
  // e = 4 (t & 15) ..), as three bf16 parts; kept rows also to prior_out
  auto stage_prior = [&](int64_t tile, int buf) {
    for (int i = t; i < IF_RB * (IF_E / 4); i += blockDim.x) {
      const int m = i >> 4, e4 = 4 * (i & 15);
      const int64_t r = tile * IF_RB + m;
      float v[4];
      if (r < d.rows) {
        const float tau = d.taus[r];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          // torch: arange(1, E + 1) * pi, then * tau, cos (iqn_q_function.py:37-41)
          const float ps = __fmul_rn(pi_f, (float)(e4 + j + 1));
          v[j] = iqn_cos(__fmul_rn(ps, tau));
        }
        if (d.prior_out && r < d.n_keep)
          *reinterpret_cast<float4*>(d.prior_out + r * IF_E + e4) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = 0.f;
      }
      bf16x4 p[3];
      split4(v, p);
#pragma unroll
      for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x4*>(&L.pr[buf][q][m * IF_LDP + e4]) = p[q];
    }
  };

  int64_t tile = blockIdx.x;
  if (tile < ntiles) stage_prior(tile, 0);
  __syncthreads();  // be / wf / first prior staged
  int buf = 0;
  for (; tile < ntiles; tile += gridDim.x, buf ^= 1) {
    const int64_t r0 = tile * IF_RB;
    const int64_t row = r0 + li;
    // b of the tile (K % 32 == 0: one b per 32-row tile)
    const int g = (int)(r0 / d.group_rows);
    const int64_t b = (r0 - (int64_t)g * d.group_rows) / d.K;
    const float* hb = d.h[g] + b * F;
    const bool keep = d.phi_out != nullptr && row < d.n_keep;
    float qa[IF_AMAX];
#pragma unroll
    for (int a = 0; a < IF_AMAX; ++a) qa[a] = 0.f;
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      // the chunk's h values of this lane's units, loaded ahead of its products
      float4 hq[4];
#pragma unroll
      for (int R = 0; R < 4; ++R)
        hq[R] = *reinterpret_cast<const float4*>(hb + 64 * w + 32 * ch + 8 * R + 4 * lh);
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < IF_E / 16; ++s) {
        bf16x8 bp[3];
#pragma unroll
        for (int q = 0; q < 3; ++q)
          bp[q] = *reinterpret_cast<const bf16x8*>(&L.pr[buf][q][li * IF_LDP + 16 * s + 8 * lh]);
        acc = prod6(wa[ch][s], bp, acc);
      }
      // lane: row li, units 64 w + 32 ch + 8 R + 4 lh + i (register 4 R + i)
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        // one unit group's be / wf reads in flight at a time (scheduled ahead
        // together they hold ~40 float4 registers and spill)
        __builtin_amdgcn_sched_barrier(0);
        const int u = 64 * w + 32 * ch + 8 * R + 4 * lh;
        const float4 bv = *reinterpret_cast<const float4*>(&L.be[u]);
        const float4 hv = hq[R];
        const float bb[4] = {bv.x, bv.y, bv.z, bv.w}, hh[4] = {hv.x, hv.y, hv.z, hv.w};
        float ph[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) ph[i] = fmaxf(acc[4 * R + i] + bb[i], 0.f);
        if (keep)
          *reinterpret_cast<float4*>(d.phi_out + row * F + u) = make_float4(ph[0], ph[1], ph[2], ph[3]);
        float pr4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) pr4[i] = __fmul_rn(hh[i], ph[i]);  // prod = h * phi
#pragma unroll
        for (int a = 0; a < AM; ++a) {
          if (a >= A) break;
          const float4 wv = *reinterpret_cast<const float4*>(&L.wf[a][u]);
          qa[a] = fmaf(pr4[0], wv.x, qa[a]);
          qa[a] = fmaf(pr4[1], wv.y, qa[a]);
          qa[a] = fmaf(pr4[2], wv.z, qa[a]);
          qa[a] = fmaf(pr4[3], wv.w, qa[a]);
        }
      }
    }
    // the next tile's prior (other buffer) while the sums meet
    if (tile + gridDim.x < ntiles) stage_prior(tile + gridDim.x, buf ^ 1);
#pragma unroll
    for (int a = 0; a < IF_AMAX; ++a) {
      if (a >= A) break;
      const float o = __shfl_xor(qa[a], 32, 64);
      if (lh == 0) L.qp[w][a][li] = qa[a] + o;
    }
    __syncthreads();  // wave sums in LDS; next prior staged
    for (int i = t; i < IF_RB * A; i += blockDim.x) {
      const int m = i / A, a = i - m * A;
      const int64_t r = r0 + m;
      if (r >= d.rows) continue;
      float s = L.qp[0][a][m];
      for (int v = 1; v < nw; ++v) s += L.qp[v][a][m];
      d.q[r * A + a] = s + d.bf[a];
    }
    __syncthreads();  // qp read before the next tile's sums
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_iqn_embed_head(const d3a_iqn_embed_head_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_iqn_embed_head: null desc");
  const d3a_iqn_embed_head_desc& d = *dp;
  D3A_CHECK_ARG(d.taus && d.We && d.be && d.Wf && d.bf && d.q, "d3a_iqn_embed_head: null pointer");
  D3A_CHECK_ARG(d.E == IF_E, "d3a_iqn_embed_head: embed size must be 64");
  D3A_CHECK_ARG(d.F >= 64 && d.F <= IF_FMAX && d.F % 64 == 0, "d3a_iqn_embed_head: F must be 64..512, %64");
  D3A_CHECK_ARG(d.A >= 1 && d.A <= IF_AMAX, "d3a_iqn_embed_head: 1..8 actions");
  D3A_CHECK_ARG(d.K >= 32 && d.K % 32 == 0 && d.rows >= 0 && d.group_rows > 0 &&
                    d.group_rows % d.K == 0 && d.n_keep >= 0 && d.n_keep <= d.rows,
                "d3a_iqn_embed_head: K must be a multiple of 32 dividing group_rows");
  const int64_t G = (d.rows + d.group_rows - 1) / d.group_rows;
  D3A_CHECK_ARG(G <= D3A_IQN_MAX_GROUPS, "d3a_iqn_embed_head: too many row groups");
  for (int64_t g = 0; g < G; ++g) D3A_CHECK_ARG(d.h[g], "d3a_iqn_embed_head: null feature group");
  auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  for (int64_t g = 0; g < G; ++g) D3A_CHECK_ARG(a16(d.h[g]), "d3a_iqn_embed_head: h must be 16-byte aligned");
  D3A_CHECK_ARG(a16(d.We) && (d.prior_out == nullptr || a16(d.prior_out)) &&
                    (d.phi_out == nullptr || a16(d.phi_out)),
                "d3a_iqn_embed_head: We, prior_out and phi_out must be 16-byte aligned");
  if (d.rows == 0) return 0;
  const int64_t ntiles = (d.rows + IF_RB - 1) / IF_RB;
  // persistent workgroups, tiles strided, one per CU (measured on K5's
  // 131,072-row pass: 256 / 512 / 1,024 / 4,096 workgroups -> 628 / 622 / 612 /
  // 586 steps/s; the per-workgroup We split amortises over more tiles);
  // D3A_IQN_GRID overrides
  static const int64_t gmax = [] {
    const char* e = getenv("D3A_IQN_GRID");
    return e ? (int64_t)atoll(e) : (int64_t)256;
  }();
  const int64_t grid = ntiles < gmax ? ntiles : gmax;
  if (d.A <= 4)
    hipLaunchKernelGGL(d3a::iqn_embed_head_kernel<4>, dim3((unsigned)grid), dim3(64 * (d.F / 64)), 0,
                       (hipStream_t)stream, d);
  else
    hipLaunchKernelGGL(d3a::iqn_embed_head_kernel<8>, dim3((unsigned)grid), dim3(64 * (d.F / 64)), 0,
                       (hipStream_t)stream, d);
  D3A_LAUNCH_CHECK("d3a_iqn_embed_head");
  return 0;
}

namespace d3a {
namespace {

using namespace x6;

// ---------------------------------------------------------------------------
// The IQN head's backward over the G gradient passes in one launch: what
// d3a_iqn_head_bwd (dphi, dh, dWf / dbf) and the embed weight-gradient GEMM
// (dWe = dphi^T prior, dbe) computed through a 200 MB dphi round trip.  A
// workgroup owns NB batch rows b (thread n = feature unit n, F = 512) and
// walks their G * K rows in 32-row tiles:
//   per row (thread n, phi read from global, exactly d3a_iqn_head_bwd's ops)
//     dprod = sum_a dq[r][a] Wf[a][n];  dphi = phi > 0 ? dprod * h : 0
//     dh[b][n] += dprod * phi;  dWf[a][n] += dq[r][a] * (h * phi)
//   per tile: dphi as three bf16 parts [n][r] in LDS, the tile's prior as
//   three parts [e][r] (transposed while staged), and dWe[n][e] += dphi^T
//   prior on the bf16 matrix cores (six part products, fp32 accumulation):
//   wave w owns n = 64 w .. + 63 and all 64 e (four 32 x 32 accumulators).
// Outputs per workgroup p (partials summed in order by the Adam kernel):
// dWf_part[p][A][F], dbf_part[p][A], dWe_part[p][F][E], dbe_part[p][F]; dh
// [B][F] (times [h > 0], the encoder fc's ReLU) is whole per b.
constexpr int IB_F = 512;
constexpr int IB_RT = 32;           // rows per tile
constexpr int IB_LDR = IB_RT + 8;   // bf16 row stride of the [.][r] images

struct IbLds {
  __bf16 dT[3][IB_F * IB_LDR];      // dphi parts [n][r]
  __bf16 pT[3][IF_E * IB_LDR];      // prior parts [e][r]
  float dq[IB_RT][IF_AMAX];
};

__global__ __launch_bounds__(512) void iqn_head_bwd_fused_kernel(d3a_iqn_head_bwd_fused_desc d) {
  __shared__ __attribute__((aligned(16))) IbLds L;
  const int n = threadIdx.x, lane = n & 63;
  const int w = __builtin_amdgcn_readfirstlane(n >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int A = d.A, K = d.K;
  const int64_t BK = (int64_t)d.B * K;
  const int64_t p = blockIdx.x;
  float wv[IF_AMAX];
#pragma unroll
  for (int a = 0; a < IF_AMAX; ++a) wv[a] = a < A ? d.Wf[a * IB_F + n] : 0.f;
  float dw[IF_AMAX];
#pragma unroll
  for (int a = 0; a < IF_AMAX; ++a) dw[a] = 0.f;
  double dbe = 0.0;
  f32x16 acc[2][2];  // dWe tiles [n block][e block]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int64_t b0 = p * d.NB;
  for (int bi = 0; bi < d.NB; ++bi) {
    const int64_t b = b0 + bi;
    if (b >= d.B) break;  // workgroup-uniform
    const float hv = d.h[b * IB_F + n];
    float dh = 0.f;
    for (int g = 0; g < d.G; ++g) {
      for (int k0 = 0; k0 < K; k0 += IB_RT) {
        const int64_t rbase = g * BK + b * K + k0;
        // stage: the tile's dq rows and its prior, transposed, as bf16 parts
        for (int i = n; i < IB_RT * IF_AMAX; i += 512) {
          const int m = i / IF_AMAX, a = i - m * IF_AMAX;
          L.dq[m][a] = a < A ? d.dq[(rbase + m) * A + a] : 0.f;
        }
        {
          // thread: row m = n >> 4, e = 4 (n & 15) .. + 3
          const int m = n >> 4, e4 = 4 * (n & 15);
          const float4 pv = *reinterpret_cast<const float4*>(d.prior + (rbase + m) * IF_E + e4);
          const float v[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            __bf16 q0, q1, q2;
            split1(v[j], q0, q1, q2);
            L.pT[0][(e4 + j) * IB_LDR + m] = q0;
            L.pT[1][(e4 + j) * IB_LDR + m] = q1;
            L.pT[2][(e4 + j) * IB_LDR + m] = q2;
          }
        }
        // phi of the tile's rows for this unit, loaded before the barrier
        float ph[IB_RT];
#pragma unroll
        for (int m = 0; m < IB_RT; ++m) ph[m] = d.phi[(rbase + m) * IB_F + n];
        __syncthreads();  // dq / prior staged
        // (dphi replaces phi in ph[] once used)
#pragma unroll
        for (int m = 0; m < IB_RT; ++m) {
          float dp = 0.f;
#pragma unroll
          for (int a = 0; a < IF_AMAX; ++a) {
            if (a >= A) break;
            const float q = L.dq[m][a];
            dp = fmaf(q, wv[a], dp);
            dw[a] = fmaf(q, __fmul_rn(hv, ph[m]), dw[a]);
          }
          const float dv = ph[m] > 0.f ? __fmul_rn(dp, hv) : 0.f;
          dh = fmaf(dp, ph[m], dh);
          dbe += (double)dv;
          ph[m] = dv;
        }
#pragma unroll
        for (int m8 = 0; m8 < IB_RT; m8 += 8) {
          bf16x8 pp[3];
          split8(ph + m8, pp);
#pragma unroll
          for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x8*>(&L.dT[q][n * IB_LDR + m8]) = pp[q];
        }
        __syncthreads();  // dphi parts staged
        // dWe[n][e] += sum_r dphi[r][n] prior[r][e]: A = dT rows (n), B = pT rows (e)
#pragma unroll
        for (int s = 0; s < IB_RT / 16; ++s) {
          bf16x8 bp[2][3];
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q)
              bp[j][q] = *reinterpret_cast<const bf16x8*>(&L.pT[q][(32 * j + li) * IB_LDR + 16 * s + 8 * lh]);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            bf16x8 ap[3];
#pragma unroll
            for (int q = 0; q < 3; ++q)
              ap[q] = *reinterpret_cast<const bf16x8*>(&L.dT[q][(64 * w + 32 * i + li) * IB_LDR + 16 * s + 8 * lh]);
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = prod6(ap, bp[j], acc[i][j]);
          }
        }
        __syncthreads();  // images free for the next tile
      }
    }
    d.dh[b * IB_F + n] = hv > 0.f ? dh : 0.f;
  }
  // partials of this workgroup
#pragma unroll
  for (int a = 0; a < IF_AMAX; ++a)
    if (a < A) d.dWf_part[(p * A + a) * IB_F + n] = dw[a];
  d.dbe_part[p * IB_F + n] = (float)dbe;
  // dWe tile (i, j): lane column e = 32 j + li, rows n = 64 w + 32 i + (r & 3) + 8 (r >> 2) + 4 lh
  float* dWe = d.dWe_part + p * IB_F * IF_E;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int nn = 64 * w + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
        dWe[nn * IF_E + 32 * j + li] = acc[i][j][r];
      }
  if (n < A) {
    double s = 0.0;
    for (int bi = 0; bi < d.NB; ++bi) {
      const int64_t b = b0 + bi;
      if (b >= d.B) break;
      for (int g = 0; g < d.G; ++g)
        for (int k = 0; k < K; ++k) s += (double)d.dq[(g * BK + b * K + k) * A + n];
    }
    d.dbf_part[p * A + n] = (float)s;
  }
}

// ---------------------------------------------------------------------------
// The same backward with phi recomputed from tau (desc.taus set): the forward
// keeps nothing (d3a_iqn_embed_head n_keep = 0: no 201 MB phi / 25 MB prior
// round trip at K5's shape), and the backward rebuilds each 32-row tile's
// prior (the forward's fp32 ops: bitwise its prior) and phi = relu(We prior +
// be) on the bf16 matrix cores (split-bf16, the forward's six part products
// in the forward's order).  Units are independent in this backward, so a
// workgroup owns 256 units (wave w: 32 units u = 256 z + 32 w + (lane & 31))
// of NB batch rows b, and both products keep the unit in the lane's column:
//   phi tile  C[row][unit] = prior[row][:] . We[unit][:]   (A = the tile's
//             prior from LDS, B = the wave's We rows split once in registers)
//   per lane: rows 8 R + 4 (lane >> 5) + i (register 4 R + i) of its unit:
//             dprod, dphi, dh, dWf, dbe as registers (Wf[a][u], h[b][u] held)
//   dWe tile  C[unit][e] += dphi^T prior: A = the dphi registers themselves
//             (their rows are the k slots; the prior image is read with the
//             same row permutation), B = the prior's transposed image.
// dh, dWf, dbe meet across the two lane halves at the end; dbf sums dq in a
// fixed order.  Two LDS buffers: the next tile's prior is built while this
// one's products run (one barrier per tile).
constexpr int IR_U = 256;          // units per workgroup
constexpr int IR_LDT = IB_RT + 4;  // bf16 row stride of the transposed prior (conflict-free b64 reads)

struct IrLds {
  __bf16 pr[2][3][IB_RT * IF_LDP];  // prior parts [buf][part][row][e]  (A of the phi product)
  __bf16 pt[2][3][IF_E * IR_LDT];   // prior parts [buf][part][e][row]  (B of the dWe product)
  float dq[2][IB_RT][IF_AMAX];
  double red[256];
};

// The forward's six part products (d3a_iqn_embed_head computes C^T with We as
// A): the same terms in the same order with the operands' roles swapped.
__device__ __forceinline__ f32x16 prod6_swapped(const bf16x8* p, const bf16x8* w, f32x16 c) {
  c = mfma16(p[0], w[2], c);
  c = mfma16(p[1], w[1], c);
  c = mfma16(p[2], w[0], c);
  c = mfma16(p[0], w[1], c);
  c = mfma16(p[1], w[0], c);
  c = mfma16(p[0], w[0], c);
  return c;
}

template <int AM>  // the action loop's bound (4 or 8): dq / Wf slots a >= A are zero
__global__ __launch_bounds__(512) void iqn_head_bwd_rc_kernel(d3a_iqn_head_bwd_fused_desc d) {
  __shared__ __attribute__((aligned(16))) IrLds L;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int A = d.A, K = d.K, F = d.F;
  const int NZ = F / IR_U;
  const int z = (int)(blockIdx.x % NZ);
  const int64_t p = blockIdx.x / NZ;
  const int u = IR_U * z + 32 * w + li;
  const int64_t BK = (int64_t)d.B * K;
  const int KT = K / IB_RT, GT = d.G * KT;
  const int64_t b0 = p * d.NB;
  const int nbv = (int)(d.B - b0 < d.NB ? d.B - b0 : d.NB);
  const int nt = nbv * GT;

  // this lane's unit: We row split (B of the phi product: k = e = 16 s + 8 lh + j)
  bf16x8 wa[IF_E / 16][3];
  {
    const float* wr = d.We + (int64_t)u * IF_E + 8 * lh;
#pragma unroll
    for (int s = 0; s < IF_E / 16; ++s) {
      const float4 x0 = *reinterpret_cast<const float4*>(wr + 16 * s);
      const float4 x1 = *reinterpret_cast<const float4*>(wr + 16 * s + 4);
      const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
      split8(v, wa[s]);
    }
  }
  const float be_u = d.be[u];
  float wf[IF_AMAX], dw[IF_AMAX];
#pragma unroll
  for (int a = 0; a < IF_AMAX; ++a) {
    wf[a] = a < A ? d.Wf[a * F + u] : 0.f;
    dw[a] = 0.f;
  }
  f32x16 dacc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) dacc[j][r] = 0.f;
  double dbe = 0.0, dbf = 0.0;
  float dh = 0.f;
  const float pi_f = 3.14159265358979323846f;

  // staging: thread t builds rows m, m + 1 (m = 2 (t >> 5)) x e = e2, e2 + 1
  // (e2 = 2 (t & 31)) of the prior, and (t < 256) dq[row t >> 3][a = t & 7]
  const int sm = 2 * (t >> 5), se = 2 * (t & 31);
  const int qm = t >> 3, qa = t & 7;
  auto rbase_of = [&](int ti) -> int64_t {
    const int bi = ti / GT, rem = ti - bi * GT;
    const int g = rem / KT, kt = rem - g * KT;
    return (int64_t)g * BK + (b0 + bi) * K + (int64_t)kt * IB_RT;
  };
  float2 ptau;
  float pdq;
  auto prefetch = [&](int ti) {
    const int64_t rb = rbase_of(ti);
    ptau = *reinterpret_cast<const float2*>(d.taus + rb + sm);
    pdq = (t < IB_RT * IF_AMAX && qa < A) ? d.dq[(rb + qm) * A + qa] : 0.f;
  };
  auto stage = [&](int nb) {
    float c[2][2];  // [row][e]
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      // torch: arange(1, E + 1) * pi, then * tau, cos (iqn_q_function.py:37-41)
      const float ps = __fmul_rn(pi_f, (float)(se + j + 1));
      c[0][j] = iqn_cos(__fmul_rn(ps, ptau.x));
      c[1][j] = iqn_cos(__fmul_rn(ps, ptau.y));
    }
    __bf16 q[2][2][3];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
      for (int j = 0; j < 2; ++j) split1(c[rr][j], q[rr][j][0], q[rr][j][1], q[rr][j][2]);
    typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        bf16x2 v;
        v[0] = q[rr][0][k];
        v[1] = q[rr][1][k];
        *reinterpret_cast<bf16x2*>(&L.pr[nb][k][(sm + rr) * IF_LDP + se]) = v;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bf16x2 v;
        v[0] = q[0][j][k];
        v[1] = q[1][j][k];
        *reinterpret_cast<bf16x2*>(&L.pt[nb][k][(se + j) * IR_LDT + sm]) = v;
      }
    }
    if (t < IB_RT * IF_AMAX) {
      L.dq[nb][qm][qa] = pdq;
      dbf += (double)pdq;  // this thread's (row, a) slot over every tile, in tile order
    }
  };

  float hv = 0.f, hn = 0.f;
  if (nt > 0) {
    prefetch(0);
    stage(0);
    hv = d.h[b0 * F + u];
  }
  __syncthreads();
  for (int ti = 0; ti < nt; ++ti) {
    const int buf = ti & 1;
    const bool more = ti + 1 < nt;
    const bool bnext = (ti + 1) % GT == 0;  // last tile of this b
    if (more) {
      prefetch(ti + 1);
      if (bnext) hn = d.h[(b0 + (ti + 1) / GT) * F + u];
    }
    // phi of the tile: C[row][unit], lane column = this unit
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int s = 0; s < IF_E / 16; ++s) {
      bf16x8 ap[3];
#pragma unroll
      for (int q = 0; q < 3; ++q)
        ap[q] = *reinterpret_cast<const bf16x8*>(&L.pr[buf][q][li * IF_LDP + 16 * s + 8 * lh]);
      acc = prod6_swapped(ap, wa[s], acc);
    }
    // per row (register 4 R + i: row 8 R + 4 lh + i): d3a_iqn_head_bwd's ops;
    // dphi replaces phi in acc
    float dbt = 0.f;  // this tile's dphi sum (into dbe in fp64 once per tile)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      // one row group (R) of dq reads in flight at a time (registers)
      if ((r & 3) == 0) __builtin_amdgcn_sched_barrier(0);
      const int m = 8 * (r >> 2) + 4 * lh + (r & 3);
      const float ph = fmaxf(acc[r] + be_u, 0.f);
      if (d.phi_dbg != nullptr) d.phi_dbg[(rbase_of(ti) + m) * F + u] = ph;
      const float4 q0 = *reinterpret_cast<const float4*>(&L.dq[buf][m][0]);
      float4 q1 = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (AM > 4) q1 = *reinterpret_cast<const float4*>(&L.dq[buf][m][4]);
      const float qv[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
      const float hp = __fmul_rn(hv, ph);
      float dp = 0.f;
#pragma unroll
      for (int a = 0; a < AM; ++a) {
        if (a >= A) break;
        dp = fmaf(qv[a], wf[a], dp);
        dw[a] = fmaf(qv[a], hp, dw[a]);
      }
      const float dv = ph > 0.f ? __fmul_rn(dp, hv) : 0.f;
      dh = fmaf(dp, ph, dh);
      dbt += dv;
      acc[r] = dv;
    }
    dbe += (double)dbt;
    // dWe[u][e] += sum_rows dphi prior: k slot (lh, j) of step s = row
    // 16 s + 8 (j >> 2) + 4 lh + (j & 3) = this lane's register 8 s + j
#pragma unroll
    for (int s = 0; s < IB_RT / 16; ++s) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = acc[8 * s + j];
      bf16x8 ap[3];
      split8(v, ap);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        bf16x8 bp[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const __bf16* src = &L.pt[buf][q][(32 * jj + li) * IR_LDT + 16 * s + 4 * lh];
          const bf16x4 lo = *reinterpret_cast<const bf16x4*>(src);
          const bf16x4 hi = *reinterpret_cast<const bf16x4*>(src + 8);
          bp[q] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
        dacc[jj] = prod6(ap, bp, dacc[jj]);
      }
    }
    if (bnext) {
      // this b's dh: the two lane halves' rows meet; times [h > 0] (the fc ReLU)
      const float tot = dh + __shfl_xor(dh, 32, 64);
      if (lh == 0) d.dh[(b0 + ti / GT) * F + u] = hv > 0.f ? tot : 0.f;
      dh = 0.f;
      hv = hn;
    }
    if (more) stage(buf ^ 1);
    __syncthreads();  // next tile staged; this tile's images free
  }
  // partials of this workgroup (units of slice z)
#pragma unroll
  for (int a = 0; a < IF_AMAX; ++a) {
    if (a >= A) break;
    const float o = __shfl_xor(dw[a], 32, 64);
    if (lh == 0) d.dWf_part[(p * A + a) * F + u] = dw[a] + o;
  }
  {
    const double o = __shfl_xor(dbe, 32, 64);
    if (lh == 0) d.dbe_part[p * F + u] = (float)(dbe + o);
  }
  float* dWe = d.dWe_part + p * F * IF_E;
#pragma unroll
  for (int jj = 0; jj < 2; ++jj)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int uu = IR_U * z + 32 * w + 8 * (r >> 2) + 4 * lh + (r & 3);
      dWe[(int64_t)uu * IF_E + 32 * jj + li] = dacc[jj][r];
    }
  if (z == 0) {
    if (t < IB_RT * IF_AMAX) L.red[t] = dbf;
    __syncthreads();
    if (t < A) {
      double s = 0.0;
      for (int m = 0; m < IB_RT; ++m) s += L.red[m * IF_AMAX + t];
      d.dbf_part[p * A + t] = (float)s;
    }
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_iqn_head_bwd_fused(const d3a_iqn_head_bwd_fused_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_iqn_head_bwd_fused: null desc");
  const d3a_iqn_head_bwd_fused_desc& d = *dp;
  const bool rc = d.taus != nullptr;
  D3A_CHECK_ARG(d.h && d.dq && d.Wf && d.dh && d.dWf_part && d.dbf_part && d.dWe_part && d.dbe_part &&
                    (rc ? (d.We && d.be) : (d.phi && d.prior)),
                "d3a_iqn_head_bwd_fused: null pointer");
  D3A_CHECK_ARG(d.A >= 1 && d.A <= IF_AMAX && d.G >= 1 && d.B >= 1 && d.NB >= 1 && d.K >= 32 &&
                    d.K % 32 == 0,
                "d3a_iqn_head_bwd_fused: bad sizes (A <= 8, K a multiple of 32)");
  auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const int64_t P = (d.B + d.NB - 1) / d.NB;
  if (rc) {
    D3A_CHECK_ARG(d.E == IF_E && (d.F == 256 || d.F == 512),
                  "d3a_iqn_head_bwd_fused: recompute needs F 256 or 512, E == 64");
    D3A_CHECK_ARG(a16(d.We) && (reinterpret_cast<uintptr_t>(d.taus) & 7) == 0,
                  "d3a_iqn_head_bwd_fused: We 16-byte, taus 8-byte aligned");
    const dim3 grid((unsigned)(P * (d.F / IR_U)));
    if (d.A <= 4)
      hipLaunchKernelGGL(d3a::iqn_head_bwd_rc_kernel<4>, grid, dim3(512), 0, (hipStream_t)stream, d);
    else
      hipLaunchKernelGGL(d3a::iqn_head_bwd_rc_kernel<8>, grid, dim3(512), 0, (hipStream_t)stream, d);
    D3A_LAUNCH_CHECK("d3a_iqn_head_bwd_fused");
    return 0;
  }
  D3A_CHECK_ARG(d.F == IB_F && d.E == IF_E, "d3a_iqn_head_bwd_fused: needs F == 512, E == 64");
  D3A_CHECK_ARG(a16(d.prior), "d3a_iqn_head_bwd_fused: prior must be 16-byte aligned");
  hipLaunchKernelGGL(d3a::iqn_head_bwd_fused_kernel, dim3((unsigned)P), dim3(512), 0,
                     (hipStream_t)stream, d);
  D3A_LAUNCH_CHECK("d3a_iqn_head_bwd_fused");
  return 0;
}
