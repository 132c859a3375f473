// Batched strided fp32 GEMM on the gfx950 f32-input matrix cores.
//
// Replaces the nn.Linear forward / backward GEMMs of the reference's MLP
// trunks and heads (d3rlpy/models/torch/encoders.py:265-275,
// policies.py:57-59,170-176, q_functions/mean_q_function.py:255-256) and
// the bias gradients of those layers (fused row sums of the dY^T operand).
//
// Tiling: a workgroup of WAVES_M x WAVES_N waves computes a BM x BN tile,
// each wave WM_T x WN_T accumulators of v_mfma_f32_32x32x2_f32 (issue
// interval == dependent latency == 64 cycles, so each accumulation chain runs
// at full rate).  K is staged through double-buffered LDS tiles BK deep,
// k-major ([k][m], [k][n]) so that MFMA operand reads are 32 consecutive
// floats per half wave (conflict-free ds_read_b32).  The global->LDS loader
// reads along the operand's unit-stride dimension with 16-byte loads when
// aligned; the next K tile is loaded into registers while the current one is
// multiplied, one barrier per K tile.  Numerics: every output is an exact
// fp32 fmaf chain over k (f32-input MFMA), no reduced precision.
#include <cstdlib>
#include <type_traits>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Operand access modes: which dimension is unit-stride.
enum { MODE_GENERIC = 0, MODE_KCONTIG = 1, MODE_XCONTIG = 2 };

struct Params {
  const float* A; const float* B; float* C;
  const float* bias; const float* mask; float* rowsum;
  int64_t M, N, K, batch;
  int64_t sAb, sAm, sAk, sBb, sBk, sBn, sCb, sCm, sCn, sbias_b, sMb, sMm, sMn;
  int64_t splits, sCs, kchunk, sRb, sRs;
  float alpha;
  int relu, accumulate;
  // second batch dimension (an independent pass of the same shape, e.g. the
  // target networks): z = (t * batch + b) * splits + s, offsets t * s?b2
  int64_t batch2, sAb2, sBb2, sCb2, sbias_b2, sMb2;
  // generated A (d3a_gemm_desc.agen): the single-output head's masked input
  // gradient g'[r] * w[j] * [h[r][j] > 0], and its weight / bias gradients
  const float* hg_h; int64_t hg_shb, hg_ldh;
  const float* hg_g; int64_t hg_sgb;
  const float* hg_gscale; int64_t hg_nscaled;
  const float* hg_w; int64_t hg_swb;
  float* hg_dW; int64_t hg_sWs;
  float* hg_db; int64_t hg_sbs;
  // next layer's weight-gradient epilogue (d3a_gemm_desc.wnext)
  const float* ew_x; int64_t ew_ldx, ew_sxb, ew_nin;
  float* ew_dW; float* ew_db;
  int xcd_remap;
};

// Load a 4-vector of a tile at non-k coordinate x and reduction coordinate k.
// KCONTIG: elements k..k+3 at x; otherwise x..x+3 at k.  Out of range -> 0.
template <int MODE>
__device__ __forceinline__ float4 load4(const float* base, int64_t sx, int64_t sk, int64_t x,
                                        int64_t k, int64_t X, int64_t kend) {
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (MODE == MODE_KCONTIG) {
    if (x >= X) return r;
    const float* p = base + x * sx + k;
    if (k + 3 < kend && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
      r = *reinterpret_cast<const float4*>(p);
    } else {
      if (k + 0 < kend) r.x = p[0];
      if (k + 1 < kend) r.y = p[1];
      if (k + 2 < kend) r.z = p[2];
      if (k + 3 < kend) r.w = p[3];
    }
  } else {
    if (k >= kend) return r;
    const float* p = base + k * sk + x * sx;
    if (MODE == MODE_XCONTIG && x + 3 < X && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
      r = *reinterpret_cast<const float4*>(p);
    } else {
      if (x + 0 < X) r.x = p[0];
      if (x + 1 < X) r.y = p[sx];
      if (x + 2 < X) r.z = p[2 * sx];
      if (x + 3 < X) r.w = p[3 * sx];
    }
  }
  return r;
}

// vector v of a (X extent) x (BK) tile -> (x, k) coordinates
template <int MODE, int XT, int BK>
__device__ __forceinline__ void vcoord(int v, int& xl, int& kl) {
  if (MODE == MODE_KCONTIG) { xl = v / (BK / 4); kl = (v % (BK / 4)) * 4; }
  else { kl = v / (XT / 4); xl = (v % (XT / 4)) * 4; }
}

template <int MODE, int LD>
__device__ __forceinline__ void store4(float* lds, int xl, int kl, float4 v) {
  if (MODE == MODE_KCONTIG) {
    lds[(kl + 0) * LD + xl] = v.x;
    lds[(kl + 1) * LD + xl] = v.y;
    lds[(kl + 2) * LD + xl] = v.z;
    lds[(kl + 3) * LD + xl] = v.w;
  } else {
    *reinterpret_cast<float4*>(&lds[kl * LD + xl]) = v;
  }
}

template <int WM_T, int WN_T, int WAVES_M, int WAVES_N, int BK>
struct TileLds {
  static constexpr int BM = 32 * WM_T * WAVES_M, BN = 32 * WN_T * WAVES_N;
  float As[2][BK * (BM + 4)];
  float Bs[2][BK * (BN + 4)];
};
// + the input-row tile of the next layer's weight-gradient epilogue (EW)
template <int WM_T, int WN_T, int WAVES_M, int WAVES_N, int BK>
struct TileLdsEW : TileLds<WM_T, WN_T, WAVES_M, WAVES_N, BK> {
  float Xs[32 * WM_T * WAVES_M * 64];
};

// One BM x BN output tile (block coordinates bx, by, bz) of the GEMM p.
template <int AMODE, int BMODE, int WM_T, int WN_T, int WAVES_M, int WAVES_N, int BK,
          bool AGEN = false, bool EW = false, class LdsT = TileLds<WM_T, WN_T, WAVES_M, WAVES_N, BK>>
__device__ __forceinline__ void gemm_f32_tile(const Params& p, int64_t bx, int64_t by, int64_t bz,
                                              LdsT& L) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int BM = 32 * WM_T * WAVES_M, BN = 32 * WN_T * WAVES_N;
  constexpr int LDA = BM + 4, LDB = BN + 4;
  constexpr int AV = BM * BK / 4 / NT, BV = BN * BK / 4 / NT;  // float4 per thread
  static_assert(AV >= 1 && BV >= 1, "tile too small for the thread count");
  auto& As = L.As;
  auto& Bs = L.Bs;

  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const int64_t n0 = bx * BN;
  const int64_t m0 = by * BM;
  const int64_t bb = bz / p.splits, s = bz % p.splits;
  const int64_t b = bb % p.batch, t2 = bb / p.batch;
  const int64_t kbeg = s * p.kchunk;
  const int64_t kend = (kbeg + p.kchunk < p.K) ? kbeg + p.kchunk : p.K;
  const float* Ab = p.A + b * p.sAb + t2 * p.sAb2;
  const float* Bb = p.B + b * p.sBb + t2 * p.sBb2;

  int axl[AV], akl[AV], bxl[BV], bkl[BV];
#pragma unroll
  for (int i = 0; i < AV; ++i) vcoord<AMODE, BM, BK>(t + i * NT, axl[i], akl[i]);
#pragma unroll
  for (int i = 0; i < BV; ++i) vcoord<BMODE, BN, BK>(t + i * NT, bxl[i], bkl[i]);

  f32x16 acc[WM_T][WN_T];
#pragma unroll
  for (int i = 0; i < WM_T; ++i)
#pragma unroll
    for (int j = 0; j < WN_T; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int wm = (wid / WAVES_N) * (32 * WM_T), wn = (wid % WAVES_N) * (32 * WN_T);
  const int li = lane & 31, lk = lane >> 5;
  const bool do_rowsum = p.rowsum != nullptr && bx == 0;
  double rs = 0.0;

  float4 ra0[AV], rb0[BV];
  // Generated A (the head backward, AGEN): gload keeps the raw loads (h and,
  // per K tile, w[j..j+3] (A k-contiguous) or g[r] and its scale (A
  // m-contiguous)) in registers and lstore forms g'[r] * w[j] * [h > 0], so
  // the loads stay in flight across the MFMA work like plain operands.
  float4 rx0[AV];
  const float* hgH = AGEN ? p.hg_h + b * p.hg_shb : nullptr;
  const float* hgG = AGEN ? p.hg_g + b * p.hg_sgb : nullptr;
  const float* hgW = AGEN ? p.hg_w + b * p.hg_swb : nullptr;
  const float hg_gs = (AGEN && p.hg_gscale) ? *p.hg_gscale : 1.f;
  const bool hg_grads = AMODE == MODE_XCONTIG && AGEN && p.hg_dW != nullptr && bx == 0;
  double hg_acc[AV][4], hg_accb = 0.0;
  float hg_fix[AV][4];  // per-thread constants: g'[r] (k-contiguous A) or w[j..j+3]
#pragma unroll
  for (int i = 0; i < AV; ++i) {
#pragma unroll
    for (int q = 0; q < 4; ++q) hg_acc[i][q] = 0.0;
    if constexpr (AGEN) {
      if (AMODE == MODE_KCONTIG) {  // A(r, j): this thread's row r is fixed
        const int64_t r = m0 + axl[i];
        float g = 0.f;
        if (r < p.M) {
          g = hgG[r];
          if (r < p.hg_nscaled) g *= hg_gs;  // as d3a_head1_bwd forms g'
        }
        hg_fix[i][0] = hg_fix[i][1] = hg_fix[i][2] = hg_fix[i][3] = g;
      } else {  // A(j, r): this thread's hidden units j..j+3 are fixed
        const float4 wv = load4<MODE_XCONTIG>(hgW, 1, 0, m0 + axl[i], 0, p.M, 1);
        hg_fix[i][0] = wv.x; hg_fix[i][1] = wv.y; hg_fix[i][2] = wv.z; hg_fix[i][3] = wv.w;
      }
    }
  }
  auto gload = [&](float4* ra, float4* rx, float4* rb, int64_t k0) {
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      if constexpr (AGEN) {
        if (AMODE == MODE_KCONTIG) {
          const int64_t r = m0 + axl[i], j = k0 + akl[i];
          ra[i] = load4<MODE_KCONTIG>(hgH, p.hg_ldh, 1, r, j, p.M, kend);
          rx[i] = load4<MODE_KCONTIG>(hgW, 0, 1, 0, j, 1, kend);
        } else {
          const int64_t j = m0 + axl[i], r = k0 + akl[i];
          ra[i] = load4<MODE_XCONTIG>(hgH, 1, p.hg_ldh, j, r, p.M, kend);
          rx[i].x = r < kend ? hgG[r] : 0.f;
          rx[i].y = r < p.hg_nscaled ? hg_gs : 1.f;
        }
      } else {
        ra[i] = load4<AMODE>(Ab, p.sAm, p.sAk, m0 + axl[i], k0 + akl[i], p.M, kend);
      }
    }
#pragma unroll
    for (int i = 0; i < BV; ++i)
      rb[i] = load4<BMODE>(Bb, p.sBn, p.sBk, n0 + bxl[i], k0 + bkl[i], p.N, kend);
  };
  auto lstore = [&](const float4* ra, const float4* rx, const float4* rb, int buf) {
#pragma unroll
    for (int i = 0; i < AV; ++i) {
      if constexpr (AGEN) {
        const float4 hv = ra[i];
        float g[4], w[4];
        if (AMODE == MODE_KCONTIG) {
#pragma unroll
          for (int q = 0; q < 4; ++q) g[q] = hg_fix[i][q];
          w[0] = rx[i].x; w[1] = rx[i].y; w[2] = rx[i].z; w[3] = rx[i].w;
        } else {
          const float gr = rx[i].x * rx[i].y;  // scale 1 (exact) past n_scaled
#pragma unroll
          for (int q = 0; q < 4; ++q) { g[q] = gr; w[q] = hg_fix[i][q]; }
          if (hg_grads) {
            hg_acc[i][0] += (double)(gr * hv.x);
            hg_acc[i][1] += (double)(gr * hv.y);
            hg_acc[i][2] += (double)(gr * hv.z);
            hg_acc[i][3] += (double)(gr * hv.w);
            if (axl[i] == 0) hg_accb += (double)gr;
          }
        }
        float4 a;
        a.x = hv.x > 0.f ? g[0] * w[0] : 0.f;
        a.y = hv.y > 0.f ? g[1] * w[1] : 0.f;
        a.z = hv.z > 0.f ? g[2] * w[2] : 0.f;
        a.w = hv.w > 0.f ? g[3] * w[3] : 0.f;
        store4<AMODE, LDA>(As[buf], axl[i], akl[i], a);
      } else {
        store4<AMODE, LDA>(As[buf], axl[i], akl[i], ra[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < BV; ++i) store4<BMODE, LDB>(Bs[buf], bxl[i], bkl[i], rb[i]);
  };
  auto compute = [&](int buf) {
    const float* Ac = As[buf];
    const float* Bc = Bs[buf];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float av[WM_T], bv[WN_T];
#pragma unroll
      for (int i = 0; i < WM_T; ++i) av[i] = Ac[(kk + lk) * LDA + wm + 32 * i + li];
#pragma unroll
      for (int j = 0; j < WN_T; ++j) bv[j] = Bc[(kk + lk) * LDB + wn + 32 * j + li];
#pragma unroll
      for (int i = 0; i < WM_T; ++i)
#pragma unroll
        for (int j = 0; j < WN_T; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (do_rowsum && t < BM) {
#pragma unroll
      for (int kk = 0; kk < BK; ++kk) rs += (double)Ac[kk * LDA + t];
    }
  };

  if (kbeg < kend) {
    gload(ra0, rx0, rb0, kbeg);
    lstore(ra0, rx0, rb0, 0);
  }
  // one accumulator tile per wave: its ReLU-mask operand is loaded now and
  // stays in registers, so the epilogue does not wait a memory round trip
  constexpr bool kMaskPf = WM_T == 1 && WN_T == 1;
  float mpf[16];
  if constexpr (kMaskPf) {
    if (p.mask) {
      const float* mb = p.mask + b * p.sMb + t2 * p.sMb2;
      const int64_t n = n0 + wn + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
        mpf[r] = (m < p.M && n < p.N) ? mb[m * p.sMm + n * p.sMn] : 0.f;
      }
    }
  }
  __syncthreads();
  // the next K tile is loaded into registers while the current one is
  // multiplied, then stored to the other LDS buffer (one barrier per tile)
  int cur = 0;
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    const bool more = k0 + BK < kend;
    if (more) gload(ra0, rx0, rb0, k0 + BK);
    compute(cur);
    if (more) lstore(ra0, rx0, rb0, cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  if (do_rowsum && t < BM && m0 + t < p.M)
    p.rowsum[b * p.sRb + s * p.sRs + m0 + t] = (float)rs;

  if (hg_grads) {
    // head weight / bias gradient partials of this split: every (k, m) slot
    // of the staging tile holds one thread's running sum; slots are summed
    // over k in a fixed order (deterministic)
    static_assert(sizeof(L) >= sizeof(double) * (BK * BM + BK), "LDS reuse too small");
    double* red = reinterpret_cast<double*>(&L);
    double* redb = red + BK * BM;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < AV; ++i) {
#pragma unroll
      for (int q = 0; q < 4; ++q) red[akl[i] * BM + axl[i] + q] = hg_acc[i][q];
      if (axl[i] == 0) redb[akl[i]] = hg_accb;
    }
    __syncthreads();
    if (t < BM && m0 + t < p.M) {
      double v = 0.0;
      for (int k = 0; k < BK; ++k) v += red[k * BM + t];
      p.hg_dW[s * p.hg_sWs + b * p.M + m0 + t] = (float)v;
    }
    if (t == 0 && by == 0 && p.hg_db) {
      double v = 0.0;
      for (int k = 0; k < BK; ++k) v += redb[k];
      p.hg_db[s * p.hg_sbs + b] = (float)v;
    }
  }

  if constexpr (EW) {
    // C = dz_{l-1} (this layer's masked input gradient) is not written: the
    // tile goes to LDS and the previous layer's weight / bias gradient
    // partials of this 128-row tile are formed from it,
    //   dW[t][b][j][d] = sum_r C(r, j) x[r][d],  db[t][b][j] = sum_r C(r, j)
    // (t = by), with x (<= 64 inputs, nd 32-wide blocks) staged beside it.
    // Wave w multiplies the 32 j of block w&3 by input block (w>>2)%nd over
    // one of 4/nd row slices; the slices are summed in order (deterministic).
    static_assert(BM == 128 && BN == 128 && NT == 1024 && WM_T == 1 && WN_T == 1,
                  "EW epilogue: 128x128 tile of sixteen 32x32 waves");
    constexpr int LT = BN + 4;
    static_assert(sizeof(L.As) + sizeof(L.Bs) >= sizeof(float) * BM * LT, "T tile");
    float* T = &L.As[0][0];  // [r][LT], spans As and Bs (contiguous)
    float* X = L.Xs;         // [r][64]
    const float* maskb = p.mask ? p.mask + b * p.sMb : nullptr;
    __syncthreads();  // every wave is done with the last K tile
    {
      const int64_t n = n0 + wn + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
        const int64_t m = m0 + ml;
        float v = 0.f;
        if (m < p.M && n < p.N) {
          v = acc[0][0][r] * p.alpha;
          if (maskb && !(mpf[r] > 0.f)) v = 0.f;
        }
        T[ml * LT + wn + li] = v;
      }
      const float* xb = p.ew_x + b * p.ew_sxb;
      if (p.ew_nin <= 32) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = t + q * NT, r = e >> 5, d = e & 31;
          const int64_t m = m0 + r;
          X[r * 64 + d] = (m < p.M && d < p.ew_nin) ? xb[m * p.ew_ldx + d] : 0.f;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int e = t + q * NT, r = e >> 6, d = e & 63;
          const int64_t m = m0 + r;
          X[e] = (m < p.M && d < p.ew_nin) ? xb[m * p.ew_ldx + d] : 0.f;
        }
      }
    }
    __syncthreads();
    const int64_t C_ = p.batch;
    if (t < BN && n0 + t < p.N) {  // bias gradient partial: fp64 column sum
      double v = 0.0;
      for (int r = 0; r < BM; ++r) v += (double)T[r * LT + t];
      p.ew_db[(by * C_ + b) * p.N + n0 + t] = (float)v;
    }
    const int nd = p.ew_nin > 32 ? 2 : 1, nkq = 4 / nd;
    const int jb = wid & 3, dq = (wid >> 2) % nd, kq = (wid >> 2) / nd;
    f32x16 a2;
#pragma unroll
    for (int r = 0; r < 16; ++r) a2[r] = 0.f;
    auto ew_mma = [&](auto sl) {
      constexpr int SL = decltype(sl)::value;
#pragma unroll
      for (int kk = 0; kk < SL; kk += 2) {
        const int r = kq * SL + kk + lk;
        a2 = __builtin_amdgcn_mfma_f32_32x32x2f32(T[r * LT + jb * 32 + li],
                                                  X[r * 64 + dq * 32 + li], a2, 0, 0, 0);
      }
    };
    if (nd == 1) ew_mma(std::integral_constant<int, BM / 4>());
    else ew_mma(std::integral_constant<int, BM / 2>());
    __syncthreads();  // T is free: reuse it for the four row-quarter partials
    float* red = T;
#pragma unroll
    for (int r = 0; r < 16; ++r) red[(wid * 16 + r) * 64 + lane] = a2[r];
    __syncthreads();
    if (kq == 0) {  // waves w < 4 * nd: sum the row slices of (jb, dq) in order
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = red[(wid * 16 + r) * 64 + lane];
        for (int q = 1; q < nkq; ++q) v += red[((wid + 4 * nd * q) * 16 + r) * 64 + lane];
        const int64_t j = n0 + jb * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        const int d = dq * 32 + li;
        if (d < p.ew_nin && j < p.N) p.ew_dW[((by * C_ + b) * p.N + j) * p.ew_nin + d] = v;
      }
    }
    return;
  }

  // epilogue: C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float* Cb = p.C + b * p.sCb + t2 * p.sCb2 + s * p.sCs;
  const float* biasb = p.bias ? p.bias + b * p.sbias_b + t2 * p.sbias_b2 : nullptr;
  const float* maskb = p.mask ? p.mask + b * p.sMb + t2 * p.sMb2 : nullptr;
#pragma unroll
  for (int j = 0; j < WN_T; ++j) {
    const int64_t n = n0 + wn + 32 * j + li;
    if (n >= p.N) continue;
    const float bn = biasb ? biasb[n] : 0.f;
#pragma unroll
    for (int i = 0; i < WM_T; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (m < p.M) {
          float v = acc[i][j][r] * p.alpha;
          if (biasb) v += bn;
          if (p.relu) v = fmaxf(v, 0.f);
          if (maskb && !((kMaskPf ? mpf[r] : maskb[m * p.sMm + n * p.sMn]) > 0.f)) v = 0.f;
          float* dst = Cb + m * p.sCm + n * p.sCn;
          if (p.accumulate) *dst += v; else *dst = v;
        }
      }
    }
  }
}

// XCD-aware tile order: the dispatcher deals workgroups out to the 8 XCDs
// round-robin, so neighbouring tiles (the column tiles of one row block, the
// tiles of one split-K slice), which read the same operand rows, would each
// fetch them into a different XCD's L2.  The bijective remap below gives each
// XCD a contiguous run of logical tiles instead (cdna_hip_programming.md T1);
// a wrong guess about placement costs speed, never correctness.
__device__ __forceinline__ void xcd_tile(int64_t& bx, int64_t& by, int64_t& bz) {
  const uint32_t gx = gridDim.x, gy = gridDim.y, nwg = gx * gy * gridDim.z;
  const uint32_t orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const uint32_t xcd = orig % 8, q = nwg / 8, r = nwg % 8;
  const uint32_t id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  bx = id % gx;
  by = (id / gx) % gy;
  bz = id / (gx * gy);
}

template <int AMODE, int BMODE, int WM_T, int WN_T, int WAVES_M, int WAVES_N, int BK,
          bool AGEN = false, bool EW = false>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void gemm_f32_kernel(Params p) {
  using LdsT = typename std::conditional<EW, TileLdsEW<WM_T, WN_T, WAVES_M, WAVES_N, BK>,
                                         TileLds<WM_T, WN_T, WAVES_M, WAVES_N, BK>>::type;
  __shared__ __attribute__((aligned(16))) LdsT lds;
  int64_t bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (p.xcd_remap) xcd_tile(bx, by, bz);
  gemm_f32_tile<AMODE, BMODE, WM_T, WN_T, WAVES_M, WAVES_N, BK, AGEN, EW, LdsT>(p, bx, by, bz,
                                                                              lds);
}

// ---- register-direct split-K kernel for small problems ---------------------
// The 256-row layers of the policy / target / actor passes (M, N <= 256,
// K <= 256) give only tens of 64x64 workgroups, and the LDS pipeline above
// then waits one global-load latency per K tile.  Here each wave of a
// workgroup owns the same 32 x (32*WN) output tile over a different K slice
// and loads its MFMA operands straight into registers (no LDS, no barrier in
// the K loop): lane l covers row/col l&31 and k = k0 + 4*(l>>5) + {0..3} (one
// 16-byte load along a unit-stride k, or four coalesced loads across lanes),
// feeding four v_mfma_f32_32x32x2_f32 per 8 k.  U such groups are loaded
// before any is multiplied, so a wave has U loads per operand in flight.  The
// KW partial tiles are summed in wave order through LDS (deterministic).
template <int MODE>
__device__ __forceinline__ float4 rd_load(const float* base, int64_t sx, int64_t sk, int64_t x,
                                          int64_t X, int64_t k, int64_t kend) {
  float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
  if (x >= X) return r;
  if (MODE == MODE_KCONTIG) {
    const float* p = base + x * sx + k;
    if (k + 3 < kend && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
      r = *reinterpret_cast<const float4*>(p);
    } else {
      if (k + 0 < kend) r.x = p[0];
      if (k + 1 < kend) r.y = p[1];
      if (k + 2 < kend) r.z = p[2];
      if (k + 3 < kend) r.w = p[3];
    }
  } else {
    const float* p = base + k * sk + x * sx;
    if (k + 0 < kend) r.x = p[0];
    if (k + 1 < kend) r.y = p[sk];
    if (k + 2 < kend) r.z = p[2 * sk];
    if (k + 3 < kend) r.w = p[3 * sk];
  }
  return r;
}

// One register-direct tile: output tile (bx, by) of batch / split bz, computed
// by the KW waves w = 0 .. KW-1 (t = 64 w + lane) of the caller; red / rsum are
// the caller's LDS (KW * WN * 16 * 64 floats, KW * 32 doubles).  Every thread
// of the workgroup passes the body's one __syncthreads.
template <int AMODE, int BMODE, int KW, int WN, int U>
__device__ __forceinline__ void gemm_rd_tile(const Params& p, int64_t bx, int64_t by, int64_t bz,
                                             int t, float* red, double* rsum) {
  const int lane = t & 63, w = t >> 6;
  const int li = lane & 31, lg = lane >> 5;
  const int64_t n0 = bx * (32 * WN);
  const int64_t m0 = by * 32;
  const int64_t bb = bz / p.splits, s = bz % p.splits;
  const int64_t b = bb % p.batch, t2 = bb / p.batch;
  const int64_t sbeg = s * p.kchunk;
  const int64_t send = (sbeg + p.kchunk < p.K) ? sbeg + p.kchunk : p.K;
  // this wave's K slice (multiple of 8 so every lane group starts aligned)
  int64_t wch = (send - sbeg + KW - 1) / KW;
  wch = (wch + 7) / 8 * 8;
  const int64_t kb = sbeg + w * wch;
  const int64_t ke = (kb + wch < send) ? kb + wch : send;
  const float* Ab = p.A + b * p.sAb + t2 * p.sAb2;
  const float* Bb = p.B + b * p.sBb + t2 * p.sBb2;
  const int64_t m = m0 + li;
  const bool do_rowsum = p.rowsum != nullptr && bx == 0;

  f32x16 acc[WN];
#pragma unroll
  for (int j = 0; j < WN; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  double rs = 0.0;

  for (int64_t k0 = kb; k0 < ke; k0 += 8 * U) {
    float4 ra[U], rb[U][WN];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = k0 + 8 * u + 4 * lg;
      ra[u] = rd_load<AMODE>(Ab, p.sAm, p.sAk, m, p.M, k, ke);
#pragma unroll
      for (int j = 0; j < WN; ++j)
        rb[u][j] = rd_load<BMODE>(Bb, p.sBn, p.sBk, n0 + 32 * j + li, p.N, k, ke);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (do_rowsum) rs += (double)ra[u].x + (double)ra[u].y + (double)ra[u].z + (double)ra[u].w;
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[u].x, rb[u][j].x, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[u].y, rb[u][j].y, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[u].z, rb[u][j].z, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ra[u].w, rb[u][j].w, acc[j], 0, 0, 0);
      }
    }
  }

  if (do_rowsum) {
    rs += __shfl_xor(rs, 32, 64);
    if (lg == 0) rsum[w * 32 + li] = rs;
  }
  // The KW partial tiles are summed in wave order 0, 1, ..., KW-1 for every
  // element (deterministic); the WN * 16 accumulator slots are shared out
  // over the waves, so the reduction runs KW-wide instead of on wave 0 alone.
  constexpr int SLOTS = WN * 16;
  if (KW > 1) {
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((w * WN + j) * 16 + r) * 64 + lane] = acc[j][r];
  }
  __syncthreads();
  if (do_rowsum && w == 0 && lg == 0 && m < p.M) {
    double tot = 0.0;
    for (int v = 0; v < KW; ++v) tot += rsum[v * 32 + li];
    p.rowsum[b * p.sRb + s * p.sRs + m] = (float)tot;
  }
  float* Cb = p.C + b * p.sCb + t2 * p.sCb2 + s * p.sCs;
  const float* biasb = p.bias ? p.bias + b * p.sbias_b + t2 * p.sbias_b2 : nullptr;
  const float* maskb = p.mask ? p.mask + b * p.sMb + t2 * p.sMb2 : nullptr;
  auto emit = [&](int j, int r, float v) {
    const int64_t n = n0 + 32 * j + li;
    const int64_t mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * lg;
    if (n < p.N && mm < p.M) {
      v = v * p.alpha;
      if (biasb) v += biasb[n];
      if (p.relu) v = fmaxf(v, 0.f);
      if (maskb && !(maskb[mm * p.sMm + n * p.sMn] > 0.f)) v = 0.f;
      float* dst = Cb + mm * p.sCm + n * p.sCn;
      if (p.accumulate) *dst += v; else *dst = v;
    }
  };
  if constexpr (KW > 1) {
    for (int q = w; q < SLOTS; q += KW) {
      const int j = q / 16, r = q % 16;
      float v = red[(j * 16 + r) * 64 + lane];
      for (int u = 1; u < KW; ++u) v += red[((u * WN + j) * 16 + r) * 64 + lane];
      emit(j, r, v);
    }
  } else {
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) emit(j, r, acc[j][r]);
  }
}

template <int AMODE, int BMODE, int KW, int WN, int U>
__global__ __launch_bounds__(64 * KW) void gemm_rd_kernel(Params p) {
  // every wave's partial tile: red[w][j*16 + r][lane]
  __shared__ float red[(KW > 1 ? KW : 1) * WN * 16 * 64];
  __shared__ double rsum[KW * 32];
  gemm_rd_tile<AMODE, BMODE, KW, WN, U>(p, blockIdx.x, blockIdx.y, blockIdx.z, threadIdx.x, red,
                                        rsum);
}

// Two independent register-direct problems in one launch of 512-thread
// workgroups (the weight- and input-gradient GEMMs of one backward layer):
// workgroups [0, nb1) run problem 1 as one-wave tiles, eight per workgroup
// (wave w takes tile 8 * blockIdx.x + w), the rest run problem 2 as eight-wave
// K-split tiles.  Each tile computes exactly what its own launch computes.
template <int AM1, int BM1, int AM2, int BM2>
__global__ __launch_bounds__(512) void gemm_rd_pair_kernel(Params p1, Params p2, int64_t nb1,
                                                           int64_t n1) {
  __shared__ float red[8 * 16 * 64];
  __shared__ double rsum[8 * 32];
  const int t = threadIdx.x, w = t >> 6;
  if ((int64_t)blockIdx.x < nb1) {
    const int64_t v = (int64_t)blockIdx.x * 8 + w;
    if (v >= n1) {
      __syncthreads();  // the tile body's barrier
      return;
    }
    const int64_t gx = (p1.N + 31) / 32, gy = (p1.M + 31) / 32;
    gemm_rd_tile<AM1, BM1, 1, 1, 4>(p1, v % gx, (v / gx) % gy, v / (gx * gy), t & 63, red,
                                    rsum + w * 32);
  } else {
    const int64_t u = (int64_t)blockIdx.x - nb1;
    const int64_t gx = (p2.N + 31) / 32, gy = (p2.M + 31) / 32;
    gemm_rd_tile<AM2, BM2, 8, 1, 4>(p2, u % gx, (u / gx) % gy, u / (gx * gy), t, red, rsum);
  }
}

struct Variant {
  int wm_t, wn_t, waves_m, waves_n, bk;
};
// index = d3a_gemm_desc.variant
constexpr Variant kVariants[] = {
    {1, 1, 2, 2, 16},  // 0: 64x64   BK16
    {2, 2, 2, 2, 16},  // 1: 128x128 BK16
    {2, 1, 2, 2, 16},  // 2: 128x64  BK16
    {1, 1, 2, 2, 32},  // 3: 64x64   BK32
    {2, 2, 2, 2, 32},  // 4: 128x128 BK32
    {1, 2, 2, 2, 16},  // 5: 64x128  BK16
    {1, 1, 1, 1, 16},  // 6: 32x32   BK16, one wave
    {1, 1, 1, 1, 64},  // 7: 32x32   BK64, one wave (small, latency-bound problems)
    {1, 1, 2, 2, 64},  // 8: 64x64   BK64
    {1, 1, 1, 1, 8},   // 9: register-direct 32x32, K split over waves (gemm_rd_kernel)
    {1, 2, 1, 1, 8},   // 10: register-direct 32x64
    {1, 2, 1, 4, 32},  // 11: 32x256  BK32, 4 waves 32x64 (tall-skinny: A read once)
    {1, 2, 2, 4, 32},  // 12: 64x256  BK32, 8 waves 32x64
    {2, 2, 2, 4, 16},  // 13: 128x256 BK16, 8 waves 64x64
    {1, 1, 4, 4, 32},  // 14: 128x128 BK32, 16 waves 32x32
    {1, 2, 4, 2, 16},  // 15: 128x128 BK16, 8 waves 32x64
    {2, 1, 2, 4, 16},  // 16: 128x128 BK16, 8 waves 64x32
    {1, 1, 2, 4, 32},  // 17: 64x128  BK32, 8 waves 32x32
    {1, 1, 4, 2, 32},  // 18: 128x64  BK32, 8 waves 32x32
};
constexpr int kFirstRd = 9;
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

template <int AM, int BMd, int V, bool AGEN = false, bool EW = false>
void launch_v(const Params& p, hipStream_t st) {
  constexpr Variant v = kVariants[V];
  constexpr int BM = 32 * v.wm_t * v.waves_m, BN = 32 * v.wn_t * v.waves_n;
  dim3 grid((unsigned)((p.N + BN - 1) / BN), (unsigned)((p.M + BM - 1) / BM),
            (unsigned)(p.batch * p.batch2 * p.splits));
  hipLaunchKernelGGL((gemm_f32_kernel<AM, BMd, v.wm_t, v.wn_t, v.waves_m, v.waves_n, v.bk, AGEN, EW>), grid,
                     dim3(64 * v.waves_m * v.waves_n), 0, st, p);
}

// waves per workgroup for the register-direct kernel: ~2048 waves in flight,
// at least 32 k (one U=4 group of loads) per wave
int rd_waves(const Params& p, int wn) {
  const int64_t tiles =
      ((p.N + 32 * wn - 1) / (32 * wn)) * ((p.M + 31) / 32) * p.batch * p.batch2 * p.splits;
  int kw = 8;
  while (kw > 1 && (tiles * kw > 4096 || p.kchunk / kw < 32)) kw >>= 1;
  return kw;
}

template <int AM, int BMd, int KW, int WN>
void launch_rd_kw(const Params& p, hipStream_t st) {
  dim3 grid((unsigned)((p.N + 32 * WN - 1) / (32 * WN)), (unsigned)((p.M + 31) / 32),
            (unsigned)(p.batch * p.batch2 * p.splits));
  hipLaunchKernelGGL((gemm_rd_kernel<AM, BMd, KW, WN, 4>), grid, dim3(64 * KW), 0, st, p);
}

template <int AM, int BMd, int WN>
void launch_rd(const Params& p, hipStream_t st) {
  switch (rd_waves(p, WN)) {
    case 8: launch_rd_kw<AM, BMd, 8, WN>(p, st); break;
    case 4: launch_rd_kw<AM, BMd, 4, WN>(p, st); break;
    case 2: launch_rd_kw<AM, BMd, 2, WN>(p, st); break;
    default: launch_rd_kw<AM, BMd, 1, WN>(p, st); break;
  }
}

template <int AM, int BMd>
void launch_modes(const Params& p, int variant, hipStream_t st) {
  switch (variant) {
    case 9: launch_rd<AM, BMd, 1>(p, st); break;
    case 10: launch_rd<AM, BMd, 2>(p, st); break;
    case 1: launch_v<AM, BMd, 1>(p, st); break;
    case 2: launch_v<AM, BMd, 2>(p, st); break;
    case 3: launch_v<AM, BMd, 3>(p, st); break;
    case 4: launch_v<AM, BMd, 4>(p, st); break;
    case 5: launch_v<AM, BMd, 5>(p, st); break;
    case 6: launch_v<AM, BMd, 6>(p, st); break;
    case 7: launch_v<AM, BMd, 7>(p, st); break;
    case 8: launch_v<AM, BMd, 8>(p, st); break;
    case 11: launch_v<AM, BMd, 11>(p, st); break;
    case 12: launch_v<AM, BMd, 12>(p, st); break;
    case 13: launch_v<AM, BMd, 13>(p, st); break;
    case 14: launch_v<AM, BMd, 14>(p, st); break;
    case 15: launch_v<AM, BMd, 15>(p, st); break;
    case 16: launch_v<AM, BMd, 16>(p, st); break;
    case 17: launch_v<AM, BMd, 17>(p, st); break;
    case 18: launch_v<AM, BMd, 18>(p, st); break;
    default: launch_v<AM, BMd, 0>(p, st); break;
  }
}

// Tile choice, from per-call sweeps of every GEMM of a K2 CQL and a K1 TD3+BC
// update (tools/gemm_pipeline_sweep.py, graph-captured timings,
// profiles/r01_pipe_sweep_*.log):
//  - few output tiles (<= 256 64x64 workgroups, or a 32-wide output) with at
//    least 32 k per split: the register-direct split-K kernel (9), 1.7-2.6x
//    faster than any LDS tile on the 256-row policy / target / actor layers
//    and the narrow first-layer input gradients;
//  - large problems with both output dimensions >= 128 and >= 64 such tiles:
//    the 128x128 tile of sixteen 32x32 waves, BK 32 (14) — four waves per
//    SIMD hide the LDS and global latency the 4-wave tiles expose (K2 critic
//    backward, profiles/r02_gemm_sweep.log: dW 33.8 vs 39.2 us, dX 35.2 vs
//    40.6 us for the 64x64 tile);
//  - otherwise the 64x64 LDS tile (0);
//  - tiny K (the first layer's 11-17 inputs): one-wave 32x32 tile (6).
int choose_variant(const Params& p) {
  const int64_t blocks64 =
      ((p.M + 63) / 64) * ((p.N + 63) / 64) * p.batch * p.batch2 * p.splits;
  const int64_t blocks128 =
      ((p.M + 127) / 128) * ((p.N + 127) / 128) * p.batch * p.batch2 * p.splits;
  const int64_t kslice = (p.K + p.splits - 1) / p.splits;
  if (kslice >= 32 && (blocks64 <= 256 || p.M <= 32 || p.N <= 32)) return 9;
  if (p.M >= 128 && p.N >= 128 && blocks128 >= 64 && kslice >= 192) return 14;
  if (blocks64 >= 128) return 0;
  return 6;
}

int env_variant() {
  static int v = [] {
    const char* e = getenv("D3A_GEMM_VARIANT");
    return e ? atoi(e) : -1;
  }();
  return v;
}

}  // namespace
}  // namespace d3a

namespace d3a {
namespace {

// Validate a descriptor and fill the kernel parameters; *skip = the problem is empty.
int make_params(const d3a_gemm_desc* d, Params& p, int& variant, int& am, int& bm, bool& skip) {
  D3A_CHECK_ARG(d != nullptr, "d3a_gemm_f32: null descriptor");
  D3A_CHECK_ARG((d->A || d->agen) && d->B && (d->C || d->wnext), "d3a_gemm_f32: null operand");
  D3A_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0 && d->batch >= 0,
                "d3a_gemm_f32: negative size");
  D3A_CHECK_ARG(d->splits >= 1, "d3a_gemm_f32: splits must be >= 1");
  D3A_CHECK_ARG(d->variant >= -1 && d->variant < kNumVariants, "d3a_gemm_f32: bad variant");
  skip = d->M == 0 || d->N == 0 || d->batch == 0;
  if (skip) return 0;
  p.A = d->A; p.B = d->B; p.C = d->C; p.bias = d->bias; p.mask = d->mask;
  p.rowsum = d->rowsum;
  p.M = d->M; p.N = d->N; p.K = d->K; p.batch = d->batch;
  p.sAb = d->sAb; p.sAm = d->sAm; p.sAk = d->sAk;
  p.sBb = d->sBb; p.sBk = d->sBk; p.sBn = d->sBn;
  p.sCb = d->sCb; p.sCm = d->sCm; p.sCn = d->sCn;
  p.sbias_b = d->sbias_b; p.sMb = d->sMb; p.sMm = d->sMm; p.sMn = d->sMn;
  p.splits = d->splits; p.sCs = d->sCs; p.sRb = d->sRb; p.sRs = d->sRs;
  p.alpha = d->alpha; p.relu = d->relu; p.accumulate = d->accumulate;
  // batch2 0 (a zero-initialised descriptor) means 1
  p.batch2 = d->batch2 > 0 ? d->batch2 : 1;
  p.sAb2 = d->sAb2; p.sBb2 = d->sBb2; p.sCb2 = d->sCb2;
  p.sbias_b2 = d->sbias_b2; p.sMb2 = d->sMb2;
  p.hg_h = nullptr; p.hg_g = nullptr; p.hg_gscale = nullptr; p.hg_w = nullptr;
  p.hg_dW = nullptr; p.hg_db = nullptr;
  p.hg_shb = p.hg_ldh = p.hg_sgb = p.hg_nscaled = p.hg_swb = p.hg_sWs = p.hg_sbs = 0;
  if (d->agen) {
    const d3a_head1_bwd_desc* g = d->agen;
    D3A_CHECK_ARG(g->h && g->g && g->w && !g->q_min,
                  "d3a_gemm_f32: agen needs h, g, w (no argmin mode)");
    D3A_CHECK_ARG(p.batch2 == 1 && !d->accumulate, "d3a_gemm_f32: agen with batch2 / accumulate");
    D3A_CHECK_ARG((d->sAk == 1) != (d->sAm == 1), "d3a_gemm_f32: agen needs a contiguous A mode");
    D3A_CHECK_ARG(!g->dW || (d->sAm == 1 && g->db), "d3a_gemm_f32: agen head grads need A^T and db");
    D3A_CHECK_ARG(!g->dW || d->K >= 1, "d3a_gemm_f32: agen head grads need rows");
    p.hg_h = g->h; p.hg_shb = g->shb; p.hg_ldh = g->ldh;
    p.hg_g = g->g; p.hg_sgb = g->sgb;
    p.hg_gscale = g->gscale; p.hg_nscaled = g->n_scaled;
    p.hg_w = g->w; p.hg_swb = g->swb;
    p.hg_dW = g->dW; p.hg_sWs = g->sWs;
    p.hg_db = g->db; p.hg_sbs = g->sbs;
  }
  D3A_CHECK_ARG(p.batch2 == 1 || d->rowsum == nullptr, "d3a_gemm_f32: rowsum needs batch2 = 1");
  variant = d->variant >= 0 ? d->variant : env_variant();
  if (variant < 0) variant = choose_variant(p);
  // generated A: the LDS tiles launch_agen instantiates
  if (d->agen) variant = (d->M >= 128 && d->N >= 128) ? 14 : 0;  // as launch_agen
  p.ew_x = nullptr; p.ew_dW = nullptr; p.ew_db = nullptr;
  {
    static const int xr = [] {
      const char* e = getenv("D3A_GEMM_XCD");
      return e ? atoi(e) : 1;
    }();
    p.xcd_remap = xr;
  }
  p.ew_ldx = p.ew_sxb = p.ew_nin = 0;
  if (d->wnext) {
    const d3a_gemm_wnext* w = d->wnext;
    D3A_CHECK_ARG(w->x && w->dW && w->db && w->n_in >= 1 && w->n_in <= 64,
                  "d3a_gemm_f32: wnext needs x, dW, db and 1..64 inputs");
    D3A_CHECK_ARG(d->sAk == 1 && d->sBk != 0 && d->splits == 1 && p.batch2 == 1 &&
                      !d->rowsum && !d->accumulate && !d->bias && !d->relu,
                  "d3a_gemm_f32: wnext on a plain input-gradient GEMM (A k-contiguous)");
    D3A_CHECK_ARG(d->sBk == 1 || d->sBn == 1, "d3a_gemm_f32: wnext needs a contiguous B");
    p.ew_x = w->x; p.ew_ldx = w->ldx; p.ew_sxb = w->sxb; p.ew_nin = w->n_in;
    p.ew_dW = w->dW; p.ew_db = w->db;
    variant = 14;
  }
  const int bk = kVariants[variant].bk;
  // split K in BK multiples (every split starts on a K-tile boundary)
  int64_t kc = (d->K + d->splits - 1) / d->splits;
  kc = ((kc + bk - 1) / bk) * bk;
  p.kchunk = kc > 0 ? kc : bk;
  D3A_CHECK_ARG(d->batch * p.batch2 * d->splits < 65536,
                "d3a_gemm_f32: batch*batch2*splits too large");
  D3A_CHECK_ARG((d->M + 31) / 32 < 65536, "d3a_gemm_f32: M too large");
  am = (d->sAk == 1) ? MODE_KCONTIG : (d->sAm == 1 ? MODE_XCONTIG : MODE_GENERIC);
  bm = (d->sBk == 1) ? MODE_KCONTIG : (d->sBn == 1 ? MODE_XCONTIG : MODE_GENERIC);
  return 0;
}

// generated-A launches (d3a_gemm_desc.agen): the 16-wave 128x128 tile where
// both output dimensions reach 128, else the 64x64 tile
template <int AM, int BMd>
void launch_agen(const Params& p, hipStream_t st) {
  if (p.M >= 128 && p.N >= 128) launch_v<AM, BMd, 14, true>(p, st);
  else launch_v<AM, BMd, 0, true>(p, st);
}

void launch_params(const Params& p, int variant, int am, int bm, hipStream_t st) {
  if (p.ew_x) {  // checked: A k-contiguous, 128x128 tile
    if (p.hg_h) {
      if (bm == MODE_KCONTIG) launch_v<MODE_KCONTIG, MODE_KCONTIG, 14, true, true>(p, st);
      else launch_v<MODE_KCONTIG, MODE_XCONTIG, 14, true, true>(p, st);
    } else {
      if (bm == MODE_KCONTIG) launch_v<MODE_KCONTIG, MODE_KCONTIG, 14, false, true>(p, st);
      else launch_v<MODE_KCONTIG, MODE_XCONTIG, 14, false, true>(p, st);
    }
    return;
  }
  if (p.hg_h) {
    if (am == MODE_KCONTIG) {
      if (bm == MODE_KCONTIG) launch_agen<MODE_KCONTIG, MODE_KCONTIG>(p, st);
      else launch_agen<MODE_KCONTIG, MODE_XCONTIG>(p, st);
    } else {
      if (bm == MODE_KCONTIG) launch_agen<MODE_XCONTIG, MODE_KCONTIG>(p, st);
      else launch_agen<MODE_XCONTIG, MODE_XCONTIG>(p, st);
    }
    return;
  }
  if (am == MODE_GENERIC || bm == MODE_GENERIC) {
    // strided fallback: smallest tile, scalar loads
    if (am == MODE_GENERIC && bm == MODE_GENERIC) launch_v<MODE_GENERIC, MODE_GENERIC, 0>(p, st);
    else if (am == MODE_GENERIC) {
      if (bm == MODE_KCONTIG) launch_v<MODE_GENERIC, MODE_KCONTIG, 0>(p, st);
      else launch_v<MODE_GENERIC, MODE_XCONTIG, 0>(p, st);
    } else {
      if (am == MODE_KCONTIG) launch_v<MODE_KCONTIG, MODE_GENERIC, 0>(p, st);
      else launch_v<MODE_XCONTIG, MODE_GENERIC, 0>(p, st);
    }
  } else if (am == MODE_KCONTIG && bm == MODE_KCONTIG) {
    launch_modes<MODE_KCONTIG, MODE_KCONTIG>(p, variant, st);
  } else if (am == MODE_KCONTIG) {
    launch_modes<MODE_KCONTIG, MODE_XCONTIG>(p, variant, st);
  } else if (bm == MODE_KCONTIG) {
    launch_modes<MODE_XCONTIG, MODE_KCONTIG>(p, variant, st);
  } else {
    launch_modes<MODE_XCONTIG, MODE_XCONTIG>(p, variant, st);
  }
}

template <int AM1, int BM1, int AM2, int BM2>
void launch_pair4(const Params& p1, const Params& p2, int64_t nb1, int64_t n1, int64_t n2,
                  hipStream_t st) {
  hipLaunchKernelGGL((gemm_rd_pair_kernel<AM1, BM1, AM2, BM2>), dim3((unsigned)(nb1 + n2)),
                     dim3(512), 0, st, p1, p2, nb1, n1);
}

template <int AM1, int BM1>
void launch_pair2(const Params& p1, const Params& p2, int am2, int bm2, int64_t nb1, int64_t n1,
                  int64_t n2, hipStream_t st) {
  if (am2 == MODE_KCONTIG) {
    if (bm2 == MODE_KCONTIG) launch_pair4<AM1, BM1, MODE_KCONTIG, MODE_KCONTIG>(p1, p2, nb1, n1, n2, st);
    else launch_pair4<AM1, BM1, MODE_KCONTIG, MODE_XCONTIG>(p1, p2, nb1, n1, n2, st);
  } else {
    if (bm2 == MODE_KCONTIG) launch_pair4<AM1, BM1, MODE_XCONTIG, MODE_KCONTIG>(p1, p2, nb1, n1, n2, st);
    else launch_pair4<AM1, BM1, MODE_XCONTIG, MODE_XCONTIG>(p1, p2, nb1, n1, n2, st);
  }
}

int64_t rd_tiles(const Params& p) {
  return ((p.N + 31) / 32) * ((p.M + 31) / 32) * p.batch * p.batch2 * p.splits;
}

// p1 one-wave register-direct tiles, p2 eight-wave ones (as their own launches
// would choose), both plain (no generated A / epilogue) with contiguous modes
bool pairable(const Params& p1, int v1, int am1, int bm1, const Params& p2, int v2, int am2,
              int bm2) {
  auto plain = [](const Params& p, int v, int am, int bm) {
    return v == 9 && !p.hg_h && !p.ew_x && am != MODE_GENERIC && bm != MODE_GENERIC;
  };
  return plain(p1, v1, am1, bm1) && plain(p2, v2, am2, bm2) && rd_waves(p1, 1) == 1 &&
         rd_waves(p2, 1) == 8 && (rd_tiles(p1) + 7) / 8 + rd_tiles(p2) < (1ll << 31);
}

}  // namespace
}  // namespace d3a

extern "C" int d3a_gemm_f32_pair(const d3a_gemm_desc* d1, const d3a_gemm_desc* d2, void* stream) {
  using namespace d3a;
  Params p1, p2;
  int v1, am1, bm1, v2, am2, bm2;
  bool s1, s2;
  if (make_params(d1, p1, v1, am1, bm1, s1) != 0) return -1;
  if (make_params(d2, p2, v2, am2, bm2, s2) != 0) return -1;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const Params* q1 = &p1;
  const Params* q2 = &p2;
  int qa1 = am1, qb1 = bm1, qa2 = am2, qb2 = bm2;
  bool pair = !s1 && !s2;
  if (pair && !pairable(p1, v1, am1, bm1, p2, v2, am2, bm2)) {
    pair = pairable(p2, v2, am2, bm2, p1, v1, am1, bm1);
    if (pair) {
      q1 = &p2; q2 = &p1;
      qa1 = am2; qb1 = bm2; qa2 = am1; qb2 = bm1;
    }
  }
  if (!pair) {  // two launches, exactly as d3a_gemm_f32 twice
    if (!s1) launch_params(p1, v1, am1, bm1, st);
    if (!s2) launch_params(p2, v2, am2, bm2, st);
    D3A_LAUNCH_CHECK("d3a_gemm_f32_pair");
    return 0;
  }
  const int64_t n1 = rd_tiles(*q1), n2 = rd_tiles(*q2), nb1 = (n1 + 7) / 8;
  if (qa1 == MODE_KCONTIG) {
    if (qb1 == MODE_KCONTIG) launch_pair2<MODE_KCONTIG, MODE_KCONTIG>(*q1, *q2, qa2, qb2, nb1, n1, n2, st);
    else launch_pair2<MODE_KCONTIG, MODE_XCONTIG>(*q1, *q2, qa2, qb2, nb1, n1, n2, st);
  } else {
    if (qb1 == MODE_KCONTIG) launch_pair2<MODE_XCONTIG, MODE_KCONTIG>(*q1, *q2, qa2, qb2, nb1, n1, n2, st);
    else launch_pair2<MODE_XCONTIG, MODE_XCONTIG>(*q1, *q2, qa2, qb2, nb1, n1, n2, st);
  }
  D3A_LAUNCH_CHECK("d3a_gemm_f32_pair");
  return 0;
}

extern "C" int d3a_gemm_f32(const d3a_gemm_desc* d, void* stream) {
  using namespace d3a;
  Params p;
  int variant, am, bm;
  bool skip;
  if (make_params(d, p, variant, am, bm, skip) != 0) return -1;
  if (skip) return 0;
  launch_params(p, variant, am, bm, reinterpret_cast<hipStream_t>(stream));
  D3A_LAUNCH_CHECK("d3a_gemm_f32");
  return 0;
}
