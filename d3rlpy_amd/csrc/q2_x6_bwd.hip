// fp32 critic backward on the bf16 matrix cores: d3a_q2_bwd's contract
// (every weight / bias gradient of [n_in <= 48 -> 256 -> 256 -> 1], one
// partial per 256-row block) with the two large products factored so that one
// operand of each is the ReLU mask -- exactly 0 or 1, one bf16 part:
//
//   dz2[r][o] = g'[r] w3[o] m[r][o],  m = [h2 > 0]
//   dh1[r][i] = sum_o dz2[r][o] W2[o][i] = g'[r] * sum_o m[r][o] (w3[o] W2[o][i])
//   dW2[o][i] = sum_r dz2[r][o] h1[r][i] = w3[o] * sum_r m[r][o] (g'[r] h1[r][i])
//
// so each of them is three MFMAs per 16 k (the mask times the three bf16 parts
// of the fp32 operand, every product exact, fp32 accumulation) against eight
// 64-cycle v_mfma_f32_32x32x2_f32 -- 5.3x the fp32 MFMA rate.  The rounding is
// fp32's: w3 W2 and g' h1 are rounded once each (as the reference's g' w3 is),
// the sums are fp32, and the outer factor is one more rounding.  The first
// layer's weight gradient dW1 = dz1^T x takes the six-product split of both
// operands (x6.hpp).  Reference: the autograd backward of update_critic's loss
// (ddpg_impl.py:119-133 via cql_impl.py:110-125) through
// VectorEncoderWithAction (encoders.py:265-275, 328-339) and
// ContinuousMeanQFunction._fc (mean_q_function.py:255-256).
//
// Geometry as q2_bwd.hip: a workgroup owns 256 rows of one member and a quarter
// (64 units) of layer 1, walking its rows in 32-row sub-blocks.  Eight waves:
//   waves 0-3 (ib = w & 1, kh = w >> 1 & 1): dh1[32 rows][units 32 ib ..] over
//     the o half 128 kh .. (A = mask rows [r][o] from LDS, B = w3 W2 parts in
//     registers, split once in the prologue); the two o halves meet in LDS one
//     sub-block later, where wave kh finishes the rows of its accumulator
//     registers 8 kh .. 8 kh + 7: dz1 = g' * dh1 * [h1 > 0] (g', h1 and x of
//     those rows prefetched from global memory one sub-block ahead), db1, and
//     dW1 += dz1^T x with the dz1 accumulator as the MFMA's A operand (its
//     rows are the K of that product: no LDS round trip)
//   waves 4-7: dW2[o block 64 (w - 4) ..][quarter] += m^T (g' h1) over the
//     sub-block's 32 rows (A = mask [o][r], B = g' h1 parts [i][r], both LDS)
// Every thread stages the next sub-block (mask images from h2, the g' h1
// parts) while the current one is multiplied; one barrier per sub-block.
// The head's gradients (dW3 = g'^T h2, db3 = sum g') and db2 = sum dz2 are
// accumulated in fp64 at staging, exactly as q2_bwd.hip forms them.
#include <cstdlib>
#include <type_traits>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"

namespace d3a {
namespace {

using namespace x6;

constexpr int B6_H = 256;
constexpr int B6_SB = 32;     // rows per sub-block
constexpr int B6_NSB = 8;     // sub-blocks per workgroup (one 256-row partial)
constexpr int B6_RB = B6_SB * B6_NSB;
constexpr int B6_QW = 64;     // layer-1 units per workgroup
constexpr int B6_LRO = 264;   // bf16 stride of the [r][o] mask rows (528 B)
constexpr int B6_LR = 40;     // bf16 stride of the [.][r] images (80 B)
constexpr int B6_NT = 512;

struct B6Buf {
  __bf16 mro[B6_SB * B6_LRO];      // m[r][o]
  __bf16 mor[B6_H * B6_LR];        // m[o][r]
  __bf16 hg[3][B6_QW * B6_LR];     // parts of g'[r] h1[r][i0 + i], [i][r]
};

struct B6Lds {
  B6Buf b[2];
  float ex[2][2 * 2 * 16 * 64];    // dh1 o-half partials [buf][ib][kh][reg][lane]
  // what the dX waves' finish of a sub-block reads one sub-block later (a
  // three-slot ring: the slot being finished, staged and read)
  __bf16 h1m[3][B6_QW * B6_LR];    // [h1 > 0] [i][r]
  float gp[3][B6_SB];              // g' of the rows
};

// MI (mask image; d.m2 given): the forward wrote the ReLU mask of h2 as bits
// (d3a_mlp_fwd_desc.hmask, 32 bytes a row), so the dW2 waves' staging expands
// bits: one bf16 0 / 1 [r][o] image per sub-block, 16-byte chunks XOR-swizzled by row
// (mchunk), read by rows (ds_read_b128) as the dh1 product's A operand and
// transposed (ds_read_b64_tr_b16) as the dW2 product's -- both conflict-free
// -- instead of two mask images built from h2 by VALU.  The quarter's db2 /
// dW3 sums read h2 for their 64 o only.
struct B7Buf {
  __bf16 mro[B6_SB * B6_H];        // m[r][o], chunk-swizzled rows of 512 B
  __bf16 hg[3][B6_QW * B6_LR];     // parts of g'[r] h1[r][i0 + i], [i][r]
};

struct B7Lds {
  B7Buf b[2];
  float ex[2][2 * 2 * 16 * 64];
  __bf16 h1m[3][B6_QW * B6_LR];
  float gp[3][B6_SB];
};

// element offset of 16-byte chunk c (o = 8 c .. 8 c + 7) of row r in a B7 mask image
__device__ __forceinline__ int mchunk(int r, int c) {
  return r * B6_H + 8 * (c ^ (((r & 3) << 2) | ((r >> 2) & 3)));
}

typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));

// NDB: 32-wide input blocks of dW1 (n_in <= 32 NDB).  PROBE (timing probes
// only, D3A_X6_PROBE >> 3; results are wrong): bit 0 skips the staging after
// the first sub-block, bit 1 the dX waves' finishing work, bit 2 the fp64 sums
template <int NDB, int PROBE = 0, bool MI = false>
__global__ __launch_bounds__(B6_NT) void q2x6_bwd_kernel(d3a_q2_bwd_desc d) {
  using Lds = typename std::conditional<MI, B7Lds, B6Lds>::type;
  __shared__ __attribute__((aligned(16))) Lds L;
  static_assert(sizeof(Lds) <= 163840, "LDS");
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lh = lane >> 5;
  // XCD-aware decode (as q2_bwd.hip): the four quarters of one (row block,
  // member) unit get block ids 8 apart -- one XCD under round-robin dispatch
  const int64_t P = (d.rows + B6_RB - 1) / B6_RB;
  const int64_t nunits = P * d.C;
  const int bid = blockIdx.x;
  const int kx = bid >> 3;
  const int q = kx & 3;
  const int64_t u = (int64_t)(kx >> 2) * 8 + (bid & 7);
  if (u >= nunits) return;  // whole workgroup, before any barrier
  const int64_t p = u / d.C;
  const int c = (int)(u - p * d.C);
  const int rows = (int)d.rows;
  const int rb0 = (int)(p * B6_RB);
  const int rlast = rows - 1;
  const int ldx = (int)d.ldx;
  const int nin = d.n_in;
  const float* h1g = d.h1 + c * d.sh;
  const float* h2g = d.h2 + c * d.sh;
  const float* gg = d.g + c * d.sgb;
  const float* xg = d.x + c * d.sxb;
  const float* W2g = d.W2 + c * d.sW2;
  const float* w3g = d.w3 + c * d.sw3;
  const float gs = d.gscale ? *d.gscale : 1.f;
  const int i0 = q * B6_QW;
  const bool role_dx = w < 4;
  const int ib = w & 1, kh = (w >> 1) & 1;
  const int ob0 = 64 * (w - 4);
  auto gprime = [&](int r) {  // g' of row r (r clamped to a valid row)
    float v = gg[r];
    if (r < d.n_scaled) v *= gs;
    return v;
  };

  // ---- staging.  dW2 waves (t2 = t - 256): two 4 x 4 blocks of h2 (rows
  // 4 (t2 & 7) + k, o = 4 (t2 >> 3) + e and + 128) -> the two mask images and
  // the head / bias sums; dX waves: h1 of rows 8 (t >> 6) + k at unit
  // i0 + (t & 63) -> the parts of g' h1.  (The dX waves carry the w3 W2
  // operand in registers: the heavier staging goes to the dW2 waves.)
  const int t2 = t - 256;
  const int ra = 4 * (t2 & 7), oa = 4 * (t2 >> 3);
  const int ih = t & 63, rh = 8 * (t >> 6);
  // running sums (dW2 waves) of q2_bwd.hip's definitions (db2 over unmasked
  // fp32(g' w3), dW3 over fp32(g' h2), db3 over g'): each thread's 32 rows of
  // the block in fp32, in row order (the register budget of this role has no
  // room for 16 fp64 accumulators), the eight threads of a column in fp64
  float s_db2[2][4], s_dw3[2][4];
  double s_db3 = 0.0;
#pragma unroll
  for (int bo = 0; bo < 2; ++bo)
#pragma unroll
    for (int e = 0; e < 4; ++e) s_db2[bo][e] = s_dw3[bo][e] = 0.f;
  float4 h2v[2][4];
  float ga[4];
  float h1v[8], gh[8];
  // MI: the dW2 waves copy mask chunk mc of rows mr + 8 k, and sum db2 / dW3
  // of o = i0 + (t2 & 63) over rows (t2 >> 6) + 4 k
  // the forward's mask bits: row r, word wd = o >> 5, bit o & 31
  const uint32_t* m2g = MI ? reinterpret_cast<const uint32_t*>(d.m2) + c * d.sm2 : nullptr;
  const int mwd = t2 & 7, mrr = t2 >> 3;
  const int so = t2 & 63, sr = t2 >> 6;
  uint32_t mword = 0u;
  // (the dW2 waves' h2 / g' of the sums reuse the dX waves' h1v / gh: one
  // pair of arrays for both roles keeps them in registers)
  float s_db2m = 0.f, s_dw3m = 0.f;
  auto load_sb = [&](int sb) {
    const int base = rb0 + sb * B6_SB;
    if (role_dx) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = min(base + rh + k, rlast);
        h1v[k] = h1g[r * B6_H + i0 + ih];
        gh[k] = gprime(r);
      }
    } else if constexpr (MI) {
      mword = m2g[min(base + mrr, rlast) * (B6_H / 32) + mwd];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = min(base + sr + 4 * k, rlast);
        h1v[k] = h2g[r * B6_H + i0 + so];
        gh[k] = gprime(r);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = min(base + ra + k, rlast);
#pragma unroll
        for (int bo = 0; bo < 2; ++bo)
          h2v[bo][k] = *reinterpret_cast<const float4*>(h2g + r * B6_H + oa + 128 * bo);
        ga[k] = gprime(r);
      }
    }
  };
  auto stage_sb = [&](int sb) {
    auto& B = L.b[sb & 1];
    const int base = rb0 + sb * B6_SB;
    if (role_dx) {
      const int slot = sb % 3;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        float hgv[4];
        bf16x4 mk;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool ok = base + rh + 4 * hh + k < rows && sb < B6_NSB;
          hgv[k] = ok ? gh[4 * hh + k] * h1v[4 * hh + k] : 0.f;
          mk[k] = (ok && h1v[4 * hh + k] > 0.f) ? (__bf16)1.f : (__bf16)0.f;
        }
        bf16x4 pp[3];
        split4(hgv, pp);
#pragma unroll
        for (int qq = 0; qq < 3; ++qq)
          *reinterpret_cast<bf16x4*>(&B.hg[qq][ih * B6_LR + rh + 4 * hh]) = pp[qq];
        *reinterpret_cast<bf16x4*>(&L.h1m[slot][ih * B6_LR + rh + 4 * hh]) = mk;
      }
      if (ih == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) L.gp[slot][rh + k] = gh[k];
      }
      return;
    }
    if constexpr (MI) {
      // the mask row mrr, o = 32 mwd .. + 31, expanded to bf16 0 / 1 (rows
      // past the end: zero, as the float path stages them)
      {
        const bool ok = base + mrr < rows && sb < B6_NSB;
        const uint32_t mw = ok ? mword : 0u;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          uint4 v;
          uint32_t* vp = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
          for (int j2 = 0; j2 < 4; ++j2) {
            const uint32_t lo = (mw >> (8 * cc + 2 * j2)) & 1u, hi = (mw >> (8 * cc + 2 * j2 + 1)) & 1u;
            vp[j2] = (lo * 0x3F80u) | (hi * 0x3F800000u);
          }
          *reinterpret_cast<uint4*>(&B.mro[mchunk(mrr, 4 * mwd + cc)]) = v;
        }
      }
      // the quarter's db2 / dW3 / db3 terms, in row order per thread
      const float w3o = w3g[i0 + so];
      float pg = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool ok = base + sr + 4 * k < rows && sb < B6_NSB;
        const float g = ok ? gh[k] : 0.f;
        const float hv = h1v[k];
        const bool on = ok && hv > 0.f;
        if (!(PROBE & 4)) {
          s_db2m += on ? g * w3o : 0.f;
          s_dw3m += g * (ok ? hv : 0.f);
        }
        pg += g;
      }
      if (so == 0) s_db3 += (double)pg;
      return;
    } else {
    float pg = 0.f;
    // db2 / dW3 are written for this workgroup's quarter of o only
    // (o = i0 .. i0 + 63: half bo = q >> 1, oa >> 6 = q & 1 -- wave-uniform,
    // oa >> 6 = (w - 4) >> 1): only those threads keep the sums
    const bool sums = ((oa >> 6) == (q & 1));
#pragma unroll
    for (int bo = 0; bo < 2; ++bo) {
      const bool sum_bo = sums && bo == (q >> 1);
      const float4 w4 = *reinterpret_cast<const float4*>(w3g + oa + 128 * bo);
      const float w3a[4] = {w4.x, w4.y, w4.z, w4.w};
      __bf16 m[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = base + ra + k < rows && sb < B6_NSB;
        const float g = ok ? ga[k] : 0.f;
        const float hv[4] = {h2v[bo][k].x, h2v[bo][k].y, h2v[bo][k].z, h2v[bo][k].w};
        bf16x4 mv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool on = ok && hv[e] > 0.f;
          m[k][e] = on ? (__bf16)1.f : (__bf16)0.f;
          mv[e] = m[k][e];
          if (!(PROBE & 4) && sum_bo) {
            s_db2[bo][e] += on ? g * w3a[e] : 0.f;
            s_dw3[bo][e] += g * (ok ? hv[e] : 0.f);
          }
        }
        if (bo == 0) pg += g;
        *reinterpret_cast<bf16x4*>(&B.mro[(ra + k) * B6_LRO + oa + 128 * bo]) = mv;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bf16x4 mv;
#pragma unroll
        for (int k = 0; k < 4; ++k) mv[k] = m[k][e];
        *reinterpret_cast<bf16x4*>(&B.mor[(oa + 128 * bo + e) * B6_LR + ra]) = mv;
      }
    }
    if (t2 < 8) s_db3 += (double)pg;
    }
  };

  f32x16 W1acc[NDB];  // dX waves: dW1 over the rows they finish
  double s_db1 = 0.0;
  load_sb(0);
  stage_sb(0);
  load_sb(1);
  if (role_dx) {
    // ---- B operand: (w3 W2)[o][i] for o = 128 kh + 16 s + 8 lh + j, unit
    // i0 + 32 ib + li, as three bf16 parts per k step
    bf16x8 wb[8][3];
    {
      const int ii = i0 + 32 * ib + li;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int o = 128 * kh + 16 * s + 8 * lh + j;
          v[j] = w3g[o] * W2g[o * B6_H + ii];
        }
        split8(v, wb[s]);
      }
    }
    // the rows this wave finishes of a sub-block: accumulator registers
    // 8 kh + r2, rows 16 kh + 8 (r2 >> 2) + 4 lh + (r2 & 3)
    auto frow = [&](int r2) { return 16 * kh + 8 * (r2 >> 2) + 4 * lh + (r2 & 3); };
    // x of the rows this wave finishes, prefetched from global memory; their
    // g' and [h1 > 0] come from the ring the staging wrote
    float fx[NDB][8];
    auto load_fin = [&](int sb) {
      const int base = rb0 + sb * B6_SB;
#pragma unroll
      for (int r2 = 0; r2 < 8; ++r2) {
        const int r = min(base + frow(r2), rlast);
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          const int dc = 32 * db + li;
          fx[db][r2] = dc < nin ? xg[r * ldx + dc] : 0.f;
        }
      }
    };
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) W1acc[db][r] = 0.f;
    // rows of sub-block sb this wave finishes: both o halves from LDS (o half
    // 0 first), dz1 = g' dh1 [h1 > 0], db1, dW1
    auto finish = [&](int sb) {
      const int eb = sb & 1, slot = sb % 3;
      // rows frow(0..3) and frow(4..7) are two runs of four
      const bf16x4 m0 = *reinterpret_cast<const bf16x4*>(&L.h1m[slot][(32 * ib + li) * B6_LR + frow(0)]);
      const bf16x4 m1 = *reinterpret_cast<const bf16x4*>(&L.h1m[slot][(32 * ib + li) * B6_LR + frow(4)]);
      const float4 g0 = *reinterpret_cast<const float4*>(&L.gp[slot][frow(0)]);
      const float4 g1 = *reinterpret_cast<const float4*>(&L.gp[slot][frow(4)]);
      const float gv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      float z[8];
#pragma unroll
      for (int r2 = 0; r2 < 8; ++r2) {
        const float o0 = L.ex[eb][((ib * 2 + 0) * 16 + 8 * kh + r2) * 64 + lane];
        const float o1 = L.ex[eb][((ib * 2 + 1) * 16 + 8 * kh + r2) * 64 + lane];
        const float v = __fadd_rn(o0, o1);
        const __bf16 mk = r2 < 4 ? m0[r2 & 3] : m1[r2 & 3];
        // rows past the end were staged with mask 0
        z[r2] = (float)mk != 0.f ? gv[r2] * v : 0.f;
        s_db1 += (double)z[r2];
      }
      // dW1[i][d] += sum_r dz1[r][i] x[r][d]: A = the dz1 rows (k step kh of the
      // accumulator-as-operand order), B = x of the same rows
      bf16x8 za[3];
      split8(z, za);
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        bf16x8 xb[3];
        split8(fx[db], xb);
        W1acc[db] = prod6(za, xb, W1acc[db]);
      }
    };
    load_fin(0);
    __syncthreads();  // sub-block 0 staged
#pragma unroll 1
    for (int sb = 0; sb < B6_NSB; ++sb) {
      const auto& B = L.b[sb & 1];
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        bf16x8 a;
        if constexpr (MI) {
          // mask row li, o = 128 kh + 16 s + 8 lh .. + 7: chunk 16 kh + 2 s + lh
          a = *reinterpret_cast<const bf16x8*>(&B.mro[mchunk(li, 16 * kh + 2 * s + lh)]);
        } else {
          a = *reinterpret_cast<const bf16x8*>(&B.mro[li * B6_LRO + 128 * kh + 8 * lh + 16 * s]);
        }
        acc = x3m(a, wb[s], acc);
        if (s == 1 && sb > 0 && !(PROBE & 2)) finish(sb - 1);
        if (s == 3 && sb > 0) load_fin(sb);
        if (!(PROBE & 1) && s == 5) stage_sb(sb + 1);
        if (!(PROBE & 1) && s == 7) load_sb(sb + 2 < B6_NSB ? sb + 2 : B6_NSB - 1);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) L.ex[sb & 1][((ib * 2 + kh) * 16 + r) * 64 + lane] = acc[r];
      __syncthreads();  // sub-block sb + 1 staged; sb's o-half partials in LDS
    }
    finish(B6_NSB - 1);
  } else {
    f32x16 R[4];  // R[2 ob + bi]: o block ob0 + 32 ob, unit block 32 bi
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) R[k][r] = 0.f;
    __syncthreads();  // sub-block 0 staged
#pragma unroll 1
    for (int sb = 0; sb < B6_NSB; ++sb) {
      const auto& B = L.b[sb & 1];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 a[2], hb[2][3];
#pragma unroll
        for (int ob = 0; ob < 2; ++ob) {
          if constexpr (MI) {
            // A[o = ob0 + 32 ob + (lane & 31)][r = 16 s + 8 lh + j] from the
            // [r][o] image by two transposed reads: 16-lane group G takes the
            // 4 x 16 block at rows 16 s + 8 (G >> 1) (+ 4), columns
            // ob0 + 32 ob + 16 (G & 1); lane 4 qq + p of the group addresses
            // row qq, columns 4 p .. 4 p + 3
            const int G = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
            const int cb = (ob0 + 32 * ob) / 8 + 2 * (G & 1) + (p >> 1);
            const int r0 = 16 * s + 8 * (G >> 1) + qq;
            const __bf16* m0 = &B.mro[mchunk(r0, cb) + 4 * (p & 1)];
            const __bf16* m1 = &B.mro[mchunk(r0 + 4, cb) + 4 * (p & 1)];
            const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) i16x4*)(m0));
            const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) i16x4*)(m1));
            const i16x8 v8 = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            a[ob] = __builtin_bit_cast(bf16x8, v8);
          } else {
            a[ob] = *reinterpret_cast<const bf16x8*>(&B.mor[(ob0 + 32 * ob + li) * B6_LR + 16 * s + 8 * lh]);
          }
        }
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int qq = 0; qq < 3; ++qq)
            hb[bi][qq] = *reinterpret_cast<const bf16x8*>(&B.hg[qq][(32 * bi + li) * B6_LR + 16 * s + 8 * lh]);
#pragma unroll
        for (int ob = 0; ob < 2; ++ob)
#pragma unroll
          for (int bi = 0; bi < 2; ++bi) R[2 * ob + bi] = x3m(a[ob], hb[bi], R[2 * ob + bi]);
        if (!(PROBE & 1)) {
          if (s == 0) stage_sb(sb + 1);
          else load_sb(sb + 2 < B6_NSB ? sb + 2 : B6_NSB - 1);
        }
      }
      __syncthreads();  // sub-block sb + 1 staged
    }
    // dW2[o][i] = w3[o] * R: lane column = unit 32 bi + li, rows o
    const int64_t pc = p * d.C + c;
    float* dW2 = d.dW2 + pc * (B6_H * B6_H);
#pragma unroll
    for (int ob = 0; ob < 2; ++ob)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = ob0 + 32 * ob + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const float wo = w3g[o];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) dW2[o * B6_H + i0 + 32 * bi + li] = wo * R[2 * ob + bi][r];
      }
  }

  // ---- epilogue (after the loops' last barrier every buffer is free)
  __syncthreads();
  const int64_t pc = p * d.C + c;
  float* w1s = reinterpret_cast<float*>(&L.b[0].mro[0]);             // [ib][db][16][64]
  // [ib][64]
  double* db1s;
  if constexpr (MI) db1s = reinterpret_cast<double*>(&L.b[0].hg[0][0]);
  else db1s = reinterpret_cast<double*>(&L.b[0].mor[0]);
  // [256][2][2][4] over mro + mor (MI: [4][64][2] over mro)
  double* hs = reinterpret_cast<double*>(&L.b[1].mro[0]);
  double* db3s = reinterpret_cast<double*>(&L.b[1].hg[0][0]);        // [8]
  if (role_dx && kh == 1) {
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) w1s[((ib * 2 + db) * 16 + r) * 64 + lane] = W1acc[db][r];
    db1s[ib * 64 + lane] = s_db1;
  }
  if (!role_dx) {
    if constexpr (MI) {
      hs[(sr * 64 + so) * 2 + 0] = (double)s_db2m;
      hs[(sr * 64 + so) * 2 + 1] = (double)s_dw3m;
      if (so == 0) db3s[sr] = s_db3;
    } else {
#pragma unroll
      for (int bo = 0; bo < 2; ++bo)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          hs[((t2 * 2 + bo) * 2 + 0) * 4 + e] = (double)s_db2[bo][e];
          hs[((t2 * 2 + bo) * 2 + 1) * 4 + e] = (double)s_dw3[bo][e];
        }
      if (t2 < 8) db3s[t2] = s_db3;
    }
  }
  __syncthreads();
  if (role_dx && kh == 0) {
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = __fadd_rn(W1acc[db][r], w1s[((ib * 2 + db) * 16 + r) * 64 + lane]);
        const int i = 32 * ib + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const int dc = 32 * db + li;
        if (dc < nin) d.dW1[(pc * B6_H + i0 + i) * nin + dc] = v;
      }
    }
    double s1 = s_db1 + db1s[ib * 64 + lane];
    s1 += __shfl_xor(s1, 32, 64);
    if (lh == 0) d.db1[pc * B6_H + i0 + 32 * ib + li] = (float)s1;
  }
  // db2 / dW3 of o = i0 + tt (this workgroup's quarter): the eight dW2-wave
  // threads holding o's column (rows 4 v .. 4 v + 3 of each sub-block), in order
  if (t >= 256 && t < 320) {
    const int tt = t - 256, o = i0 + tt;
    double s2 = 0.0, s3 = 0.0;
    if constexpr (MI) {
      // the four threads of o (rows sr + 4 k of each sub-block), in order
      for (int v = 0; v < 4; ++v) {
        s2 += hs[(v * 64 + tt) * 2 + 0];
        s3 += hs[(v * 64 + tt) * 2 + 1];
      }
    } else {
      const int bo = o >> 7, oo = o & 127;
      const int tb = (oo >> 2) << 3, e = oo & 3;
      for (int v = 0; v < 8; ++v) {
        s2 += hs[(((tb + v) * 2 + bo) * 2 + 0) * 4 + e];
        s3 += hs[(((tb + v) * 2 + bo) * 2 + 1) * 4 + e];
      }
    }
    d.db2[pc * B6_H + o] = (float)s2;
    d.dW3[pc * B6_H + o] = (float)s3;
  } else if (t == 320 && q == 0) {
    double sg = 0.0;
    for (int v = 0; v < (MI ? 4 : 8); ++v) sg += db3s[v];
    d.db3[pc] = (float)sg;
  }
}

}  // namespace
}  // namespace d3a

using namespace d3a;

namespace d3a {
int launch_q2x6t_bwd(const d3a_q2_bwd_desc& d, hipStream_t st,
                     const d3a_cql_loss_desc* lc = nullptr);  // q2_x6_bwd2.hip
}

extern "C" int d3a_q2_bwd_x6(const d3a_q2_bwd_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_q2_bwd_x6: null desc");
  const d3a_q2_bwd_desc& d = *dp;
  D3A_CHECK_ARG(d.dz2 == nullptr, "d3a_q2_bwd_x6: dz2 input is not supported (use d3a_q2_bwd)");
  D3A_CHECK_ARG(d.block_rows == 0 || d.block_rows == 256, "d3a_q2_bwd_x6: block_rows must be 0 / 256");
  D3A_CHECK_ARG(d.x && d.h1 && (d.h2 || d.m2t) && d.g && d.W2 && d.w3, "d3a_q2_bwd_x6: null input");
  D3A_CHECK_ARG(d.dW1 && d.db1 && d.dW2 && d.db2 && d.dW3 && d.db3, "d3a_q2_bwd_x6: null output");
  D3A_CHECK_ARG(d.n_in >= 1 && d.n_in <= 48, "d3a_q2_bwd_x6: n_in must be 1..48");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0 && d.n_scaled >= 0, "d3a_q2_bwd_x6: bad sizes");
  auto a16 = [](const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; };
  D3A_CHECK_ARG(a16(d.h1) && (d.m2t || a16(d.h2)) && d.ldh == B6_H && d.sh % 4 == 0,
                "d3a_q2_bwd_x6: h1 / h2 must be 16-byte aligned rows of 256 floats");
  D3A_CHECK_ARG(a16(d.w3) && d.sw3 % 4 == 0, "d3a_q2_bwd_x6: w3 must be 16-byte aligned");
  D3A_CHECK_ARG(d.ldx >= d.n_in, "d3a_q2_bwd_x6: ldx < n_in");
  D3A_CHECK_ARG(d.rows * (d.ldh > d.ldx ? d.ldh : d.ldx) < (int64_t(1) << 31),
                "d3a_q2_bwd_x6: rows x row stride exceeds 2^31");
  D3A_CHECK_ARG(d.m2 == nullptr || ((reinterpret_cast<uintptr_t>(d.m2) & 3) == 0 &&
                                    d.sm2 >= d.rows * (B6_H / 32)),
                "d3a_q2_bwd_x6: the mask must be rows of 8 32-bit words");
  if (d.m2t != nullptr) return launch_q2x6t_bwd(d, (hipStream_t)stream);
  if (d.rows == 0) return 0;
  const int64_t units = ((d.rows + B6_RB - 1) / B6_RB) * d.C;
  const int64_t blocks = (units + 7) / 8 * 32;
  D3A_CHECK_ARG(blocks < (int64_t(1) << 31), "d3a_q2_bwd_x6: too many rows");
  const dim3 grid((unsigned)blocks), block(B6_NT);
  static const int probe = [] {
    const char* e = getenv("D3A_X6_PROBE");
    return e ? atoi(e) >> 3 : 0;
  }();
  if (probe && d.n_in <= 32 && d.m2 == nullptr) {
    const hipStream_t st = (hipStream_t)stream;
    switch (probe & 7) {
      case 1: hipLaunchKernelGGL((q2x6_bwd_kernel<1, 1>), grid, block, 0, st, d); break;
      case 2: hipLaunchKernelGGL((q2x6_bwd_kernel<1, 2>), grid, block, 0, st, d); break;
      case 3: hipLaunchKernelGGL((q2x6_bwd_kernel<1, 3>), grid, block, 0, st, d); break;
      case 4: hipLaunchKernelGGL((q2x6_bwd_kernel<1, 4>), grid, block, 0, st, d); break;
      default: hipLaunchKernelGGL((q2x6_bwd_kernel<1, 7>), grid, block, 0, st, d); break;
    }
    D3A_LAUNCH_CHECK("d3a_q2_bwd_x6");
    return 0;
  }
  const bool mi = d.m2 != nullptr;
  if (d.n_in <= 32 && mi)
    hipLaunchKernelGGL((q2x6_bwd_kernel<1, 0, true>), grid, block, 0, (hipStream_t)stream, d);
  else if (mi)
    hipLaunchKernelGGL((q2x6_bwd_kernel<2, 0, true>), grid, block, 0, (hipStream_t)stream, d);
  else if (d.n_in <= 32)
    hipLaunchKernelGGL(q2x6_bwd_kernel<1>, grid, block, 0, (hipStream_t)stream, d);
  else
    hipLaunchKernelGGL(q2x6_bwd_kernel<2>, grid, block, 0, (hipStream_t)stream, d);
  D3A_LAUNCH_CHECK("d3a_q2_bwd_x6");
  return 0;
}
