// Split-bf16 helpers of the fp32-accurate critic kernels (q2_x6.hip,
// q2_x6_bwd.hip): the exact three-way split of an fp32 value into bf16 parts
// and the part products on v_mfma_f32_32x32x16_bf16.
#pragma once

#include <hip/hip_runtime.h>

namespace d3a {
namespace x6 {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ f32x16 mfma16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// exact three-way split of one fp32 value
__device__ __forceinline__ void split1(float x, __bf16& p0, __bf16& p1, __bf16& p2) {
  p0 = (__bf16)x;
  const float r1 = x - (float)p0;
  p1 = (__bf16)r1;
  p2 = (__bf16)(r1 - (float)p1);
}

__device__ __forceinline__ void split8(const float* x, bf16x8* p) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    __bf16 a, b, c;
    split1(x[i], a, b, c);
    p[0][i] = a;
    p[1][i] = b;
    p[2][i] = c;
  }
}

__device__ __forceinline__ void split4(const float* x, bf16x4* p) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    __bf16 a, b, c;
    split1(x[i], a, b, c);
    p[0][i] = a;
    p[1][i] = b;
    p[2][i] = c;
  }
}

// the six part products, smallest first
__device__ __forceinline__ f32x16 prod6(const bf16x8* a, const bf16x8* b, f32x16 c) {
  c = mfma16(a[2], b[0], c);
  c = mfma16(a[1], b[1], c);
  c = mfma16(a[0], b[2], c);
  c = mfma16(a[1], b[0], c);
  c = mfma16(a[0], b[1], c);
  c = mfma16(a[0], b[0], c);
  return c;
}

// the three products of a 0/1 operand a (exact in one bf16 part) with the
// parts of b, smallest first
__device__ __forceinline__ f32x16 x3m(bf16x8 a, const bf16x8* b, f32x16 c) {
  c = mfma16(a, b[2], c);
  c = mfma16(a, b[1], c);
  c = mfma16(a, b[0], c);
  return c;
}

// NP-part generalisations: NP = 3 is the exact split above (six products),
// NP = 1 a single bf16 rounding per operand (one product: the bf16 line)
template <int NP>
__device__ __forceinline__ void splitn8(const float* x, bf16x8* p) {
  if constexpr (NP == 3) {
    split8(x, p);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) p[0][i] = (__bf16)x[i];
  }
}

template <int NP>
__device__ __forceinline__ void splitn4(const float* x, bf16x4* p) {
  if constexpr (NP == 3) {
    split4(x, p);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) p[0][i] = (__bf16)x[i];
  }
}

template <int NP>
__device__ __forceinline__ f32x16 prodn(const bf16x8* a, const bf16x8* b, f32x16 c) {
  if constexpr (NP == 3) return prod6(a, b, c);
  else return mfma16(a[0], b[0], c);
}

}  // namespace x6
}  // namespace d3a

#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace x6 {

// host: the input-row builder's fields are consistent (or it is off); the
// row write-out (xg_xout / xg_eout) only on the parts path
inline bool xgen_ok(const d3a_mlp_fwd_desc& d) {
  if (d.xg_mode == 0) return true;
  const bool outs_ok =
      (d.xg_xout == nullptr && d.xg_eout == nullptr) ||
      (d.parts > 1 && (d.xg_xout == nullptr || (d.xg_ldxo >= d.n_in && d.xg_ldxo % 4 == 0 &&
                                                (reinterpret_cast<uintptr_t>(d.xg_xout) & 15) == 0)));
  return d.xg_mode >= 1 && d.xg_mode <= 5 && d.xg_obs && d.xg_a && d.xg_D >= 1 && d.xg_rep >= 1 &&
         d.xg_E >= 1 && d.xg_D + d.xg_E == d.n_in && d.aux_rows == 0 && d.xg_lda >= d.xg_E &&
         ((d.xg_mode != 3 && d.xg_mode != 4) || d.xg_base != nullptr) && d.xg_a_parts >= 0 &&
         d.xg_a_parts <= 8 && (d.xg_a_parts <= 1 || d.xg_s_apart > 0) && outs_ok;
}

// features k4 .. k4 + 3 of input row r of a forward pass, zero past nin /
// rend: x itself, or the row the descriptor's builder defines
// (d3a_mlp_fwd_desc.xg_mode; d3a_bcq_rows's arithmetic, bcq.hip).  No
// branches around the loads: every load comes from clamped (in-range)
// indices and is issued before any is used, so the row costs one memory round
// trip and the compiler's wait counts stay exact (a load under a divergent
// branch makes it wait for every load in flight, prefetches included).
// input4_issue only loads (the raw operands, to be finished later: a
// persistent kernel prefetches its next tile's rows that way).
struct XRaw4 {
  float ob[4], a[4], bs[4];
};

__device__ __forceinline__ void input4_issue(const d3a_mlp_fwd_desc& d, const float* xb, int64_t ldx, int r,
                                             int k4, int rend, int nin, XRaw4& x) {
  const int rr = r < rend ? r : rend - 1;
  int kc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) kc[j] = min(k4 + j, nin - 1);
  if (d.xg_mode == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x.ob[j] = xb[(int64_t)rr * ldx + kc[j]];
      x.a[j] = x.bs[j] = 0.f;
    }
    return;
  }
  const int D = d.xg_D;
  const float* orow = d.xg_obs + (int64_t)(rr / d.xg_rep) * D;
  const float* arow = d.xg_a + (int64_t)rr * d.xg_lda;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    x.ob[j] = orow[min(kc[j], D - 1)];
    x.a[j] = arow[max(kc[j] - D, 0)];
    x.bs[j] = 0.f;
  }
  if (d.xg_a_parts > 1) {  // uniform: a as head parts, summed in order
    for (int q = 1; q < d.xg_a_parts; ++q) {
      float t[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = arow[q * d.xg_s_apart + max(kc[j] - D, 0)];
#pragma unroll
      for (int j = 0; j < 4; ++j) x.a[j] += t[j];
    }
  }
  if (d.xg_mode == 3 || d.xg_mode == 4) {
    const float* brow = d.xg_base + (int64_t)rr * d.xg_E;
#pragma unroll
    for (int j = 0; j < 4; ++j) x.bs[j] = brow[max(kc[j] - D, 0)];
  }
}

__device__ __forceinline__ void input4_finish(const d3a_mlp_fwd_desc& d, int r, int k4, int rend, int nin,
                                              const XRaw4& x, float v[4]) {
  const bool rok = r < rend;
  if (d.xg_mode == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (rok && k4 + j < nin) ? x.ob[j] : 0.f;
    return;
  }
  const int D = d.xg_D;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float y;
    switch (d.xg_mode) {
      case 1: y = fminf(fmaxf(x.a[j], -d.xg_clip), d.xg_clip); break;
      case 2: y = tanhf(x.a[j]); break;
      case 3: y = fminf(fmaxf(__fadd_rn(x.bs[j], __fmul_rn(d.xg_scale, tanhf(x.a[j]))), -1.f), 1.f); break;
      case 4:
        y = fminf(fmaxf(__fadd_rn(tanhf(x.bs[j]), __fmul_rn(d.xg_scale, tanhf(x.a[j]))), -1.f), 1.f);
        break;
      default: y = x.a[j];  // 5: the copy
    }
    v[j] = (rok && k4 + j < nin) ? (k4 + j < D ? x.ob[j] : y) : 0.f;
  }
}

// ---- d3a_x6_split: the weights' operand images (include/d3rlpy_amd.h).
// A piece is one 8-wide k block of one row: two 16-byte loads where the row
// allows, the split8 above (the forward's own split, so a forward streaming
// the image is bitwise the forward that splits), three 16-byte stores.
__host__ __device__ inline int64_t x6_split_pieces(const d3a_x6_split_job& j) {
  return (int64_t)j.rows * (j.kpad >> 3);
}

__host__ __device__ inline int64_t x6_split_total(const d3a_x6_split_desc& d) {
  int64_t n = 0;
  for (int i = 0; i < d.n_jobs; ++i) n += x6_split_pieces(d.job[i]);
  return n;
}

// piece p of the desc's pieces (job by job), in two halves: the loads
// (branch-free: clamped indices, the padding selected to zero after the load,
// so a caller can issue them ahead of its own work without the compiler
// waiting for them early) and the split + stores
struct X6Piece {
  float v[8];
  char* dst;  // the piece's 48 bytes
};

__device__ __forceinline__ void x6_split_load(const d3a_x6_split_desc& d, int64_t p, X6Piece& o) {
  int ji = 0;
  for (; ji < d.n_jobs - 1; ++ji) {
    const int64_t n = x6_split_pieces(d.job[ji]);
    if (p < n) break;
    p -= n;
  }
  const d3a_x6_split_job& j = d.job[ji];
  const int nkb = j.kpad >> 3;
  const int64_t r = p / nkb;
  const int kb = (int)(p - r * nkb);
  const float* row = j.src + r * j.k;
  const bool vec = (j.k & 7) == 0 && (reinterpret_cast<uintptr_t>(j.src) & 15) == 0;
  if (vec) {
    // (a padding block reads the row's first block, zeroed below)
    const int kc = 8 * kb < j.k ? 8 * kb : 0;
    const float4 a = reinterpret_cast<const float4*>(row + kc)[0];
    const float4 b = reinterpret_cast<const float4*>(row + kc)[1];
    o.v[0] = a.x; o.v[1] = a.y; o.v[2] = a.z; o.v[3] = a.w;
    o.v[4] = b.x; o.v[5] = b.y; o.v[6] = b.z; o.v[7] = b.w;
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) o.v[i] = row[min(8 * kb + i, j.k - 1)];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) o.v[i] = 8 * kb + i < j.k ? o.v[i] : 0.f;
  o.dst = static_cast<char*>(j.dst) + (r * nkb + kb) * 48;
}

__device__ __forceinline__ void x6_split_store(const X6Piece& o) {
  bf16x8 pp[3];
  split8(o.v, pp);
  bf16x8* dst = reinterpret_cast<bf16x8*>(o.dst);
  dst[0] = pp[0];
  dst[1] = pp[1];
  dst[2] = pp[2];
}

__device__ __forceinline__ void x6_split_piece(const d3a_x6_split_desc& d, int64_t p) {
  X6Piece o;
  x6_split_load(d, p, o);
  x6_split_store(o);
}

inline bool x6_split_ok(const d3a_x6_split_desc& d) {
  if (d.n_jobs < 0 || d.n_jobs > D3A_X6_SPLIT_MAX_JOBS) return false;
  for (int i = 0; i < d.n_jobs; ++i) {
    const d3a_x6_split_job& j = d.job[i];
    if (!j.src || !j.dst || j.rows < 0 || j.k < 1 || j.kpad < j.k || j.kpad % 16 != 0 ||
        (reinterpret_cast<uintptr_t>(j.dst) & 15) != 0)
      return false;
  }
  return true;
}

__device__ __forceinline__ void input4_at(const d3a_mlp_fwd_desc& d, const float* xb, int64_t ldx, int r,
                                          int k4, int rend, int nin, float v[4]) {
  XRaw4 x;
  input4_issue(d, xb, ldx, r, k4, rend, nin, x);
  input4_finish(d, r, k4, rend, nin, x, v);
}

}  // namespace x6
}  // namespace d3a
