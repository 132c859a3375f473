// Batched strided fp32 GEMM on the gfx950 f32-input matrix cores.
//
// Replaces the nn.Linear forward / backward GEMMs of the reference's MLP
// trunks and heads (d3rlpy/models/torch/encoders.py:265-275,
// policies.py:57-59,170-176, q_functions/mean_q_function.py:255-256).
//
// Tile: 64x64 output per 256-thread workgroup, 4 waves in a 2x2 grid, each
// wave one 32x32 accumulator of v_mfma_f32_32x32x2_f32 (issue interval ==
// dependent latency == 64 cycles, so one accumulation chain runs at full
// rate).  K is staged through LDS in 16-deep tiles, k-major ([k][m] and
// [k][n]) so that the MFMA operand reads are 32 consecutive floats per half
// wave (conflict-free ds_read_b32).  The global->LDS loader picks, per
// operand, the coalesced direction (the unit-stride dimension) and issues
// 16-byte loads when aligned.  The next K tile is prefetched into registers
// while the current one is multiplied.  Result numerics: each output is an
// fp32 fmaf chain over k (exact-f32 MFMA), no reduced precision.
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"

namespace d3a {
namespace {

constexpr int BM = 64, BN = 64, BK = 16;
constexpr int LDA = BM + 4, LDB = BN + 4;  // +4 floats: spread the transposing writes
constexpr int kThreads = 256;

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Operand access modes: which dimension is unit-stride.
enum { MODE_GENERIC = 0, MODE_KCONTIG = 1, MODE_XCONTIG = 2 };

struct Params {
  const float* A; const float* B; float* C;
  const float* bias; const float* mask;
  int64_t M, N, K, batch;
  int64_t sAb, sAm, sAk, sBb, sBk, sBn, sCb, sCm, sCn, sbias_b, sMb, sMm, sMn;
  int64_t splits, sCs, kchunk;
  float alpha;
  int relu, accumulate;
};

// Load a 4-vector of a tile. `x` is the non-k coordinate (m for A, n for B),
// `k` the reduction coordinate.  MODE_KCONTIG: the 4 elements are k..k+3 at x;
// MODE_XCONTIG: x..x+3 at k.  Out-of-range elements are zero.
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
  } else {  // XCONTIG or GENERIC (4 along x)
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

// Thread -> (x, k) coordinate of the 4-vector it loads inside a 64x16 tile.
template <int MODE>
__device__ __forceinline__ void tile_coord(int t, int& xl, int& kl) {
  if (MODE == MODE_KCONTIG) { xl = t >> 2; kl = (t & 3) * 4; }
  else { kl = t >> 4; xl = (t & 15) * 4; }
}

template <int MODE, int LD>
__device__ __forceinline__ void store_tile(float* lds, int xl, int kl, float4 v) {
  if (MODE == MODE_KCONTIG) {
    lds[(kl + 0) * LD + xl] = v.x;
    lds[(kl + 1) * LD + xl] = v.y;
    lds[(kl + 2) * LD + xl] = v.z;
    lds[(kl + 3) * LD + xl] = v.w;
  } else {
    *reinterpret_cast<float4*>(&lds[kl * LD + xl]) = v;
  }
}

template <int AMODE, int BMODE>
__global__ __launch_bounds__(kThreads) void gemm_f32_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) float As[BK * LDA];
  __shared__ __attribute__((aligned(16))) float Bs[BK * LDB];

  const int t = threadIdx.x;
  const int lane = t & 63, wid = t >> 6;
  const int64_t n0 = (int64_t)blockIdx.x * BN;
  const int64_t m0 = (int64_t)blockIdx.y * BM;
  const int64_t bz = blockIdx.z;
  const int64_t b = bz / p.splits, s = bz % p.splits;
  const int64_t kbeg = s * p.kchunk;
  const int64_t kend = (kbeg + p.kchunk < p.K) ? kbeg + p.kchunk : p.K;

  const float* Ab = p.A + b * p.sAb;
  const float* Bb = p.B + b * p.sBb;

  // per-thread tile coordinates
  int axl, akl, bxl, bkl;
  tile_coord<AMODE>(t, axl, akl);
  tile_coord<BMODE>(t, bxl, bkl);
  // for A: x = m, stride along x = sAm, along k = sAk
  // for B: x = n, stride along x = sBn, along k = sBk
  const int64_t a_sx = p.sAm, a_sk = p.sAk, b_sx = p.sBn, b_sk = p.sBk;

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32;
  const int li = lane & 31, lk = lane >> 5;

  float4 ra = make_float4(0.f, 0.f, 0.f, 0.f), rb = ra;
  if (kbeg < kend) {
    ra = load4<AMODE>(Ab, a_sx, a_sk, m0 + axl, kbeg + akl, p.M, kend);
    rb = load4<BMODE>(Bb, b_sx, b_sk, n0 + bxl, kbeg + bkl, p.N, kend);
  }
  for (int64_t k0 = kbeg; k0 < kend; k0 += BK) {
    store_tile<AMODE, LDA>(As, axl, akl, ra);
    store_tile<BMODE, LDB>(Bs, bxl, bkl, rb);
    __syncthreads();
    if (k0 + BK < kend) {
      ra = load4<AMODE>(Ab, a_sx, a_sk, m0 + axl, k0 + BK + akl, p.M, kend);
      rb = load4<BMODE>(Bb, b_sx, b_sk, n0 + bxl, k0 + BK + bkl, p.N, kend);
    }
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float av = As[(kk + lk) * LDA + wm + li];
      const float bv = Bs[(kk + lk) * LDB + wn + li];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    }
    __syncthreads();
  }

  // epilogue: C/D map col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float* Cb = p.C + b * p.sCb + s * p.sCs;
  const float* biasb = p.bias ? p.bias + b * p.sbias_b : nullptr;
  const float* maskb = p.mask ? p.mask + b * p.sMb : nullptr;
  const int64_t n = n0 + wn + li;
  if (n >= p.N) return;
  const float bn = biasb ? biasb[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t m = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
    if (m < p.M) {
      float v = acc[r] * p.alpha;
      if (biasb) v += bn;
      if (p.relu) v = fmaxf(v, 0.f);
      if (maskb && !(maskb[m * p.sMm + n * p.sMn] > 0.f)) v = 0.f;
      float* dst = Cb + m * p.sCm + n * p.sCn;
      if (p.accumulate) *dst += v; else *dst = v;
    }
  }
}

template <int AM, int BMd>
void launch(const Params& p, dim3 grid, hipStream_t st) {
  hipLaunchKernelGGL((gemm_f32_kernel<AM, BMd>), grid, dim3(kThreads), 0, st, p);
}

}  // namespace
}  // namespace d3a

extern "C" int d3a_gemm_f32(const d3a_gemm_desc* d, void* stream) {
  using namespace d3a;
  D3A_CHECK_ARG(d != nullptr, "d3a_gemm_f32: null descriptor");
  D3A_CHECK_ARG(d->A && d->B && d->C, "d3a_gemm_f32: null operand");
  D3A_CHECK_ARG(d->M >= 0 && d->N >= 0 && d->K >= 0 && d->batch >= 0,
                "d3a_gemm_f32: negative size");
  D3A_CHECK_ARG(d->splits >= 1, "d3a_gemm_f32: splits must be >= 1");
  if (d->M == 0 || d->N == 0 || d->batch == 0) return 0;
  Params p;
  p.A = d->A; p.B = d->B; p.C = d->C; p.bias = d->bias; p.mask = d->mask;
  p.M = d->M; p.N = d->N; p.K = d->K; p.batch = d->batch;
  p.sAb = d->sAb; p.sAm = d->sAm; p.sAk = d->sAk;
  p.sBb = d->sBb; p.sBk = d->sBk; p.sBn = d->sBn;
  p.sCb = d->sCb; p.sCm = d->sCm; p.sCn = d->sCn;
  p.sbias_b = d->sbias_b; p.sMb = d->sMb; p.sMm = d->sMm; p.sMn = d->sMn;
  p.splits = d->splits; p.sCs = d->sCs;
  // split K in BK multiples
  int64_t kc = (d->K + d->splits - 1) / d->splits;
  kc = ((kc + BK - 1) / BK) * BK;
  p.kchunk = kc > 0 ? kc : BK;
  p.alpha = d->alpha; p.relu = d->relu; p.accumulate = d->accumulate;
  D3A_CHECK_ARG(d->batch * d->splits < 65536, "d3a_gemm_f32: batch*splits too large");
  D3A_CHECK_ARG((d->M + BM - 1) / BM < 65536, "d3a_gemm_f32: M too large");

  const int am = (d->sAk == 1) ? MODE_KCONTIG : (d->sAm == 1 ? MODE_XCONTIG : MODE_GENERIC);
  const int bm = (d->sBk == 1) ? MODE_KCONTIG : (d->sBn == 1 ? MODE_XCONTIG : MODE_GENERIC);
  dim3 grid((unsigned)((d->N + BN - 1) / BN), (unsigned)((d->M + BM - 1) / BM),
            (unsigned)(d->batch * d->splits));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // GENERIC uses the XCONTIG thread mapping with strided scalar loads
  const int a = am == MODE_KCONTIG ? 1 : 2, b = bm == MODE_KCONTIG ? 1 : 2;
  if (am == MODE_GENERIC || bm == MODE_GENERIC) {
    if (am == MODE_GENERIC && bm == MODE_GENERIC) launch<MODE_GENERIC, MODE_GENERIC>(p, grid, st);
    else if (am == MODE_GENERIC) {
      if (b == 1) launch<MODE_GENERIC, MODE_KCONTIG>(p, grid, st);
      else launch<MODE_GENERIC, MODE_XCONTIG>(p, grid, st);
    } else {
      if (a == 1) launch<MODE_KCONTIG, MODE_GENERIC>(p, grid, st);
      else launch<MODE_XCONTIG, MODE_GENERIC>(p, grid, st);
    }
  } else if (a == 1 && b == 1) launch<MODE_KCONTIG, MODE_KCONTIG>(p, grid, st);
  else if (a == 1 && b == 2) launch<MODE_KCONTIG, MODE_XCONTIG>(p, grid, st);
  else if (a == 2 && b == 1) launch<MODE_XCONTIG, MODE_KCONTIG>(p, grid, st);
  else launch<MODE_XCONTIG, MODE_XCONTIG>(p, grid, st);
  D3A_LAUNCH_CHECK("d3a_gemm_f32");
  return 0;
}
