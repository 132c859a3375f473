// fp32 critic ensemble on the bf16 matrix cores: the forward of the
// [n_in <= 48 -> 256 -> 256 -> 1] Q ensemble (q2_fwd.hip's contract, d3a_mlp_fwd
// descriptor) with every GEMM evaluated as a three-way split-bf16 product.
//
// Reference: VectorEncoderWithAction [n_in -> 256 -> 256] (encoders.py:265-275,
// 328-339) + ContinuousMeanQFunction._fc [256 -> 1] (q_functions/
// mean_q_function.py:255-256), over the CQL critic pass (15,616 Q rows + 256
// target rows per member at K2) -- fp32 in the reference, fp32-accurate here.
//
// Split products.  An fp32 value x is split exactly into three bf16 parts,
//   x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1),  x = x0 + x1 + x2
// (each subtraction exact in fp32; 8 + 8 + 8 significant bits), and a product
// x * y is formed as the six part products above fp32's resolution,
//   x2 y0 + x1 y1 + x0 y2 + x1 y0 + x0 y1 + x0 y0   (dropped: x1 y2, x2 y1,
//   x2 y2, each below 2^-24 |x y|),
// on v_mfma_f32_32x32x16_bf16 with fp32 accumulation: six 32-cycle MFMAs per
// 16 k against eight 64-cycle v_mfma_f32_32x32x2_f32 -- 2.67x the fp32 MFMA
// rate on the same work.  The split GEMM is within 6e-7 (max-normalised) of
// fp64 where fp32 MFMA is within 5e-7 (profiles/r02_sbf16_accuracy.txt); the
// CQL parity suite holds at its fp32 bars on it (tests/test_gpu_x6.py).
//
// Forward structure.  A workgroup owns 128 rows of one member; eight waves,
// wave w owning hidden units 32 w .. 32 w + 31 of layer 2 over all 128 rows
// (four transposed tiles C^T[unit][row]: W1 the A operand, activation rows the
// B operand, so a lane holds one row and four runs of four consecutive units:
// 16-byte stores and a register head dot, as in q2_fwd.hip).  Layer 2's K (the
// 256 layer-1 units) is walked in eight chunks of 32.  Layer 1 produces chunk
// j + 1 (its 32 units for the 128 rows: four 32x32 tiles, one per wave of the
// half (j + 1) & 1, so each SIMD carries one producing wave per chunk) while
// layer 2 consumes chunk j; the chunk is written to a two-slot LDS ring as its
// three bf16 parts ([row][k], 80-byte rows: conflict-free 16-byte fragment
// reads), and as fp32 to h[0] for kept rows.  Each wave loads its W1 slice of
// the next chunk from global memory as fp32 one chunk ahead and splits it in
// registers.  One barrier per chunk.
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"

namespace d3a {
namespace {

using namespace x6;

constexpr int X_H = 256;    // hidden width
constexpr int X_RB = 128;   // rows per workgroup
constexpr int X_CK = 64;    // layer-2 k per chunk (= layer-1 units per chunk)
constexpr int X_NCK = X_H / X_CK;
constexpr int X_KS = X_CK / 16;  // MFMA k steps per chunk
constexpr int X_LDB = 72;   // bf16 row stride of a ring slot (144 B: conflict-free 16-B reads)

constexpr int X_NOMAX = 8;  // widest narrow head (NO = 8 instantiation)

template <int XL, int NP, int NO>
struct X6FwdLds {
  __bf16 h[2][NP][X_RB * X_LDB];    // layer-1 chunk ring: slot, part, [row][k]
  __bf16 x[NP][X_RB * (XL + 8)];    // input rows, parts, zero-padded to XL
  float hp[NO > 1 ? 1 : 8][X_RB];   // head partials [wave][row] (NO == 1)
};

// PROBE (timing probes only, D3A_X6_PROBE; results are wrong): bit 0 skips
// the layer-1 productions after the first, bit 2 the kept-activation stores,
// bit 3 the W1 reloads (chunk 0's registers reused); bit 4 (diagnostic build,
// results right) records s_memtime stamps of wave 0 at the phase boundaries
// into x6_stamps (read with d3a_x6_stamps); bit 5 the W1 split (the loaded
// words taken as the parts); bit 6 (results right) the round-4 chunk schedule
// (the production epilogue after the chunk's MFMAs, kept rows on branches);
// bit 7 (results right) the interleaved chunks without the tile-major last
// chunk (the Q head's epilogue after the MFMAs); bit 8 (results right) no
// static priority for waves 4-7
//
// NP / HT: NP = 3 the exact split (fp32-accurate, kept activations fp32);
// NP = 1, HT = __bf16 the bf16 throughput line's forward (d3a_q2_fwd_bf16's
// contract: one bf16 rounding per operand, kept activations stored as bf16)
//
// NO: the head width; 1 (the Q head: a register dot) or X_NOMAX for a narrow
// head of 2 .. 8 outputs (e.g. BCQ's VAE decoder and residual policy over the
// B*N target rows, bcq_impl.py:215-226): head rows staged in LDS, one dot per
// output, the per-wave partials over the freed chunk ring
__device__ unsigned long long x6_stamps[2048 * 10];
//
// PRE: W0 / W1 streamed as pre-split operand images (d3a_mlp_fwd_desc.wp,
// d3a_x6_split's layout, formed once per step by an earlier launch) instead
// of fp32 words split in every workgroup -- the split's vector instructions
// (W1: 128 values a lane, W0: 32) leave the MFMA gaps; bitwise the same parts
//
// NOH2 (with PRE; host: d.h[1] null, as for the slice backward, which reads
// the mask bits instead of h2): the last chunk issues no h2 stores at all
template <int XL, int PROBE = 0, int NP = 3, typename HT = float, int NO = 1, bool PRE = false,
          bool NOH2 = false>
__global__ __launch_bounds__(512) void q2x6_fwd_kernel(d3a_mlp_fwd_desc d) {
  constexpr int XLD = XL + 8;
  constexpr int NS0 = XL / 16;  // layer-1 k steps
  // the round-5 schedules (see the chunk loop): interleaved chunks (XL <= 32)
  // and, for the Q head, the tile-major last chunk carrying the epilogue
  constexpr bool CHUNKIL = (PROBE & 64) == 0 && XL <= 32;
  constexpr bool LASTIL = CHUNKIL && NO == 1 && (PROBE & 128) == 0;
  // vector instructions interleaved per MFMA (timing probes: bit 9 four, bit 10
  // sixteen)
  constexpr int VG = (PROBE & 512) ? 4 : (PROBE & 1024) ? 16 : 8;
  static_assert(!PRE || (CHUNKIL && NP == 3), "pre-split images: the interleaved schedule");
  __shared__ __attribute__((aligned(16))) X6FwdLds<XL, NP, NO> L;
  static_assert(sizeof(X6FwdLds<XL, NP, NO>) <= 163840, "LDS");
  static_assert(NO == 1 || 8 * NO * X_RB * 4 <= (int)sizeof(L.h), "head partials fit the ring");
  static_assert(NO == 1 || NO * X_H * 4 <= (int)sizeof(L.x), "head rows fit the input image");
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int c = blockIdx.z;
  const int nb_main = (int)((d.rows + X_RB - 1) / X_RB);
  const bool aux = (int)blockIdx.x >= nb_main;
  // row indices fit 32 bits (checked on the host)
  const int m0 = aux ? ((int)blockIdx.x - nb_main) * X_RB : (int)d.r0 + (int)blockIdx.x * X_RB;
  const int rend = aux ? (int)d.aux_rows : (int)(d.r0 + d.rows);
  const int h_from = aux ? rend : (int)d.h_from;
  const int64_t wdel = aux ? d.aux_wdelta : 0;
  float* const outp = aux ? d.aux_out + c * d.aux_sout : d.out + c * d.sout;
  const int nin = d.n_in;
  HT* const h0g = (!aux && d.h[0]) ? reinterpret_cast<HT*>(d.h[0]) + c * d.sh : nullptr;
  HT* const h1g = (!aux && d.h[1]) ? reinterpret_cast<HT*>(d.h[1]) + c * d.sh : nullptr;
  // the ReLU mask image of the last hidden layer (kept rows; NO == 1)
  uint32_t* const hmg = (!aux && NO == 1 && d.hmask) ? reinterpret_cast<uint32_t*>(d.hmask) + c * d.s_hmask
                                                     : nullptr;
  // and transposed (word [r >> 5][unit], bit r & 31; d.r0 % 32 == 0)
  uint32_t* const hmtg = (hmg != nullptr && d.hmaskT) ? reinterpret_cast<uint32_t*>(d.hmaskT) + c * d.s_hmaskT
                                                      : nullptr;
  // a kept run of four activations (16 bytes fp32, 8 bytes bf16)
  auto put4 = [](HT* p, const float* v) {
    if constexpr (sizeof(HT) == 4) {
      *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      bf16x4 b;
#pragma unroll
      for (int i = 0; i < 4; ++i) b[i] = (__bf16)v[i];
      *reinterpret_cast<bf16x4*>(p) = b;
    }
  };
  const float* W0 = d.W[0] + wdel + c * d.sW[0];
  const float* b0 = d.b[0] + wdel + c * d.sb[0];
  const int wg = blockIdx.x + blockIdx.z * gridDim.x;
  auto stamp = [&](int k) {
    if constexpr ((PROBE & 16) != 0) {
      if (t == 0 && wg < 2048) x6_stamps[wg * 10 + k] = __builtin_amdgcn_s_memtime();
    }
  };
  if constexpr ((PROBE & 16) != 0) {
    if (t == 0 && wg < 2048) x6_stamps[wg * 10 + 9] = __builtin_amdgcn_s_memrealtime();
  }
  stamp(0);
  // this lane's W1 row (unit 32 w + li) at k offset 8 lh
  const float* W1 = d.W[1] + wdel + c * d.sW[1] + (32 * w + li) * X_H + 8 * lh;

  // ---- operand streams.  W1: this lane's row, one 64-k chunk as fp32 loaded
  // one chunk ahead.  W0 / b0: the wave's layer-1 tile of a chunk, one
  // production ahead.
  float4 wr[X_KS][2];  // raw fp32 W1 of the chunk in flight: [k step][half]
  // (PRE) the W1 image as a four-slot ring of k steps: slot s holds step s's
  // parts of the current chunk until its last MFMA, then the next chunk's
  bf16x8 wq[X_KS][NP];
  // this lane's W1 image row (unit 32 w + li) at k block lh, and the member's
  // W0 image (rows of XL / 8 blocks of 48 bytes)
  const char* wp1l = nullptr;
  const char* wp0b = nullptr;
  if constexpr (PRE) {
    wp1l = static_cast<const char*>(aux ? d.aux_wp[1] : d.wp[1]) +
           ((int64_t)c * X_H + 32 * w + li) * (X_H * 6) + lh * 48;
    wp0b = static_cast<const char*>(aux ? d.aux_wp[0] : d.wp[0]) + (int64_t)c * X_H * (XL * 6);
  }
  auto load_w1p = [&](int j, int s) {
    const bf16x8* p = reinterpret_cast<const bf16x8*>(wp1l + (8 * j + 2 * s) * 48);
#pragma unroll
    for (int q = 0; q < NP; ++q) wq[s][q] = p[q];
  };
  auto load_w1 = [&](int j) {
#pragma unroll
    for (int s = 0; s < X_KS; ++s) {
      if constexpr (PRE) {
        load_w1p(j, s);
      } else {
        wr[s][0] = *reinterpret_cast<const float4*>(W1 + X_CK * j + 16 * s);
        wr[s][1] = *reinterpret_cast<const float4*>(W1 + X_CK * j + 16 * s + 4);
      }
    }
  };
  float w0n[NS0][8];
  bf16x8 w0p[NS0][NP];  // (PRE) the W0 image's parts
  float4 b0n[4];
  const int ut = 32 * (w >> 2);  // this wave's unit tile inside a chunk
  const int ptt = w & 3;         // and its row tile
  // (weights and bias are loaded separately, each right after its last use,
  // so that a whole chunk interval covers their latency)
  auto load_w0w = [&](int j) {
    const int u = X_CK * j + ut + li;
    if constexpr (PRE) {
      const char* rowp = wp0b + (int64_t)u * (XL * 6);
#pragma unroll
      for (int s = 0; s < NS0; ++s) {
        const bf16x8* p = reinterpret_cast<const bf16x8*>(rowp + (2 * s + lh) * 48);
#pragma unroll
        for (int q = 0; q < NP; ++q) w0p[s][q] = p[q];
      }
      return;
    }
#pragma unroll
    for (int s = 0; s < NS0; ++s)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int k = 16 * s + 8 * lh + i;
        const float v = W0[u * nin + (k < nin ? k : nin - 1)];  // branch-free
        // (the interleaved schedule zeroes the padding at the split)
        w0n[s][i] = CHUNKIL || k < nin ? v : 0.f;
      }
  };
  auto load_b0 = [&](int j) {
#pragma unroll
    for (int R = 0; R < 4; ++R) b0n[R] = *reinterpret_cast<const float4*>(b0 + X_CK * j + ut + 8 * R + 4 * lh);
  };
  // (PRE) this lane's input parts: row 32 ptt + li at k 16 s + 8 lh .. + 7 --
  // the production's B operand, the same row tile in every chunk, so it stays
  // in registers (no LDS image, no barrier before the first production)
  bf16x8 xq[NS0][NP];
  // ---- prologue: every load of the first chunk and production in flight at
  // once, then the input rows split into LDS
  if constexpr (PRE) {
    const float* xb = aux ? d.aux_x + c * d.aux_sxb : d.x + c * d.sxb;
    const int ldx = (int)(aux ? d.aux_ldx : d.ldx);
    const int r = m0 + 32 * ptt + li, rc = min(r, rend - 1);
    float4 fa[NS0][2];
#pragma unroll
    for (int s = 0; s < NS0; ++s)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        fa[s][h] = *reinterpret_cast<const float4*>(xb + (int64_t)rc * ldx + min(16 * s + 8 * lh + 4 * h, ldx - 4));
    load_w0w(0);
    load_b0(0);
    // chunk 0's first W1 k step only: the prologue's burst of loads (every
    // CU at once) is what the first production waits for, so the other three
    // steps follow the production's MFMAs (measured 0.5 % faster than all four
    // up front; all after the inputs arrived: no faster)
    load_w1p(0, 0);
#pragma unroll
    for (int s = 0; s < NS0; ++s) {
      // (through an empty asm: the whole pieces loaded, none narrowed)
      typedef float f32x4v __attribute__((ext_vector_type(4)));
      f32x4v f0 = {fa[s][0].x, fa[s][0].y, fa[s][0].z, fa[s][0].w};
      f32x4v f1 = {fa[s][1].x, fa[s][1].y, fa[s][1].z, fa[s][1].w};
      asm volatile("" : "+v"(f0), "+v"(f1));
      const float fv[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (r < rend && 16 * s + 8 * lh + i < nin) ? fv[i] : 0.f;
      splitn8<NP>(v, xq[s]);
    }
  } else if constexpr (CHUNKIL) {
    // one 16-byte piece of the 128 x 16 input rows a thread: its load issued
    // ahead of the weights' so that waiting for it does not wait for them
    // (the load counter is in order)
    constexpr int X4 = XL / 4, NPC = X_RB * X4 / 512;  // pieces a thread
    static_assert(X_RB * X4 == 512 * NPC, "whole pieces a thread");
    const float* xb = aux ? d.aux_x + c * d.aux_sxb : d.x + c * d.sxb;
    const int64_t ldx = aux ? d.aux_ldx : d.ldx;
    // (PRE: plain 16-byte rows, checked on the host -- no row-builder code,
    // whose branchy loads made the compiler wait for every load in flight,
    // the W1 stream's included, before staging x)
    const bool vec =
        PRE || (d.xg_mode == 0 && (ldx & 3) == 0 && (reinterpret_cast<uintptr_t>(xb) & 15) == 0);
    float4 f[NPC];
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc) {
      const int e = t + 512 * pc, m = e / X4, k4 = (e - m * X4) * 4, r = m0 + m;
      f[pc] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (vec) {
        const int rc = min(r, rend - 1), kc = min(k4, (int)ldx - 4);
        f[pc] = *reinterpret_cast<const float4*>(xb + (int64_t)rc * ldx + kc);
      }
    }
    load_w0w(0);
    load_b0(0);
    load_w1(0);
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc) {
      const int e = t + 512 * pc, m = e / X4, k4 = (e - m * X4) * 4, r = m0 + m;
      float v[4];
      if (vec) {
        // (the whole piece through an empty asm: the compiler otherwise
        // narrows the load to the elements the selects below may keep and
        // loads the rest under a branch that waits for every load in flight)
        typedef float f32x4v __attribute__((ext_vector_type(4)));
        f32x4v ff = {f[pc].x, f[pc].y, f[pc].z, f[pc].w};
        asm volatile("" : "+v"(ff));
        const float fv[4] = {ff.x, ff.y, ff.z, ff.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (r < rend && k4 + j < nin) ? fv[j] : 0.f;
      } else if constexpr (!PRE) {
        input4_at(d, xb, ldx, r, k4, rend, nin, v);
      }
      bf16x4 p[NP];
      splitn4<NP>(v, p);
#pragma unroll
      for (int q = 0; q < NP; ++q) *reinterpret_cast<bf16x4*>(&L.x[q][m * XLD + k4]) = p[q];
    }
  } else {
  load_w0w(0);
  load_b0(0);
  load_w1(0);
  {
    const float* xb = aux ? d.aux_x + c * d.aux_sxb : d.x + c * d.sxb;
    const int64_t ldx = aux ? d.aux_ldx : d.ldx;
    constexpr int X4 = XL / 4;
    // plain rows of 16-byte pieces: one unconditional float4 load per piece
    // (row and piece clamped, the padding selected to 0 after the load) --
    // the element path below branches per element, and each branch waits for
    // every load in flight (the W0 / W1 / b0 prefetch included)
    const bool vec = d.xg_mode == 0 && (ldx & 3) == 0 && (reinterpret_cast<uintptr_t>(xb) & 15) == 0;
    for (int e = t; e < X_RB * X4; e += 512) {
      const int m = e / X4, k4 = (e - m * X4) * 4;
      const int r = m0 + m;
      float v[4];
      if (vec) {
        const int rc = min(r, rend - 1), kc = min(k4, (int)ldx - 4);
        const float4 f = *reinterpret_cast<const float4*>(xb + (int64_t)rc * ldx + kc);
        const float fv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (r < rend && k4 + j < nin) ? fv[j] : 0.f;
      } else {
        input4_at(d, xb, ldx, r, k4, rend, nin, v);
      }
      bf16x4 p[NP];
      splitn4<NP>(v, p);
#pragma unroll
      for (int q = 0; q < NP; ++q) *reinterpret_cast<bf16x4*>(&L.x[q][m * XLD + k4]) = p[q];
    }
  }
  }  // CHUNKIL
  if constexpr (!PRE) __syncthreads();  // x parts staged
  stamp(1);

  // ---- layer 1, chunk j: every wave produces one 32 x 32 tile of it -- units
  // 64 j + ut .. + 31 of rows 32 ptt .. + 31 -- in two halves: the MFMAs
  // (issued at the start of the chunk interval, ahead of layer 2's) and the
  // epilogue (bias, ReLU, fp32 kept rows to h[0], parts to ring slot j & 1;
  // at its end, while layer 2's last MFMAs drain), so the production's
  // dependent chain never stalls the in-order wave mid-chunk
  auto produce_mma = [&](f32x16& a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) a[r] = 0.f;
#pragma unroll
    for (int s = 0; s < NS0; ++s) {
      bf16x8 wp[NP], xp[NP];
      if constexpr (PRE) {
#pragma unroll
        for (int q = 0; q < NP; ++q) wp[q] = w0p[s][q];
      } else if constexpr (CHUNKIL) {
        // (as split_w below: keeps the split of the prefetched W0 words from
        // being hoisted next to their loads)
        typedef float f32x4v __attribute__((ext_vector_type(4)));
        f32x4v r0 = {w0n[s][0], w0n[s][1], w0n[s][2], w0n[s][3]};
        f32x4v r1 = {w0n[s][4], w0n[s][5], w0n[s][6], w0n[s][7]};
        asm volatile("" : "+v"(r0), "+v"(r1));
        float v[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 16 * s + 8 * lh + i < nin ? v[i] : 0.f;
        splitn8<NP>(v, wp);
      } else {
        splitn8<NP>(w0n[s], wp);
      }
#pragma unroll
      for (int q = 0; q < NP; ++q)
        xp[q] = PRE ? xq[s][q] : *reinterpret_cast<const bf16x8*>(&L.x[q][(32 * ptt + li) * XLD + 16 * s + 8 * lh]);
      a = prodn<NP>(wp, xp, a);
    }
  };
  auto produce_epi = [&](int j, const f32x16& a) {
    float4 bv4[4];
#pragma unroll
    for (int R = 0; R < 4; ++R) bv4[R] = b0n[R];
    if (j + 1 < X_NCK) load_b0(j + 1);
    // lane: row 32 ptt + li, units 64 j + ut + 8 R + 4 lh + i (accumulator 4 R + i)
    const int row = m0 + 32 * ptt + li;
    const bool keep = h0g != nullptr && row >= h_from && row < rend;
#pragma unroll
    for (int R = 0; R < 4; ++R) {
      const int k = ut + 8 * R + 4 * lh;  // local k of the chunk
      const float4 bv = bv4[R];
      float v[4] = {fmaxf(a[4 * R + 0] + bv.x, 0.f), fmaxf(a[4 * R + 1] + bv.y, 0.f),
                    fmaxf(a[4 * R + 2] + bv.z, 0.f), fmaxf(a[4 * R + 3] + bv.w, 0.f)};
      if (keep && !(PROBE & 4)) put4(h0g + row * X_H + X_CK * j + k, v);
      bf16x4 p[NP];
      splitn4<NP>(v, p);
#pragma unroll
      for (int q = 0; q < NP; ++q)
        *reinterpret_cast<bf16x4*>(&L.h[j & 1][q][(32 * ptt + li) * X_LDB + k]) = p[q];
    }
  };
  {
    f32x16 pa;
    produce_mma(pa);
    if constexpr (PRE) {
#pragma unroll
      for (int s = 1; s < X_KS; ++s) load_w1p(0, s);
    }
    load_w0w(1);
    produce_epi(0, pa);
  }
  __syncthreads();  // chunk 0 in slot 0
  stamp(2);

  // ---- layer 2: acc[tt] = C^T[units 32 w ..][rows 32 tt ..].  The B operand
  // of each (k step, row tile) is read from LDS one tile ahead of its MFMAs.
  f32x16 acc[4];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[tt][r] = 0.f;
  float b2l = 0.f;  // (LASTIL) the head bias, loaded with the last chunk's operands
  if constexpr (CHUNKIL && (PROBE & 256) == 0) {
    // the second-dispatched half (waves 4-7, each SIMD's younger wave) at a
    // static higher issue priority: it otherwise loses every VALU
    // arbitration to its older partner (MI355X_MICROARCH.md, item 4)
    if (w >= 4) __builtin_amdgcn_s_setprio(1);
  }
  if constexpr (CHUNKIL) {
    // the chunk interval as sixteen (k step, row tile) regions of NP * NP
    // products each: region idx issues the next region's LDS reads, the
    // regions 4 s split W1 step s + 1, and regions 5, 7, 9, 11 carry the
    // next chunk's production epilogue one 8-unit run at a time -- its
    // vector work interleaved into the MFMA gaps (sched_group_barrier)
    // instead of trailing the chunk's last MFMAs, its kept-row stores
    // branch-free (masked lanes store out of the buffer's range and are
    // dropped: a branch would end the scheduling region).  (XL <= 32: with
    // XL = 48's layer-1 tiles the schedule spills)
    const __amdgpu_buffer_rsrc_t h0r =
        __builtin_amdgcn_make_buffer_rsrc(h0g, (short)0, 0x7fffffff, 0x00020000);
    const int prow = m0 + 32 * ptt + li;  // the production lane's row
    const bool pkeep = h0g != nullptr && prow >= h_from && prow < rend && !(PROBE & 4);
    auto epi_run = [&](int jn, const f32x16& a, const float4& bv, int R) {
      const int k = ut + 8 * R + 4 * lh;  // local k of the chunk
      float v[4] = {fmaxf(a[4 * R + 0] + bv.x, 0.f), fmaxf(a[4 * R + 1] + bv.y, 0.f),
                    fmaxf(a[4 * R + 2] + bv.z, 0.f), fmaxf(a[4 * R + 3] + bv.w, 0.f)};
      const uint32_t off = pkeep ? (uint32_t)((prow * X_H + X_CK * jn + k) * (int)sizeof(HT)) : 0x80000000u;
      if constexpr (sizeof(HT) == 4) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 bits = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                            __float_as_uint(v[3])};
        __builtin_amdgcn_raw_buffer_store_b128(bits, h0r, off, 0, 0);
      } else {
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        bf16x4 b;
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] = (__bf16)v[i];
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, b), h0r, off, 0, 0);
      }
      bf16x4 p[NP];
      splitn4<NP>(v, p);
#pragma unroll
      for (int q = 0; q < NP; ++q)
        *reinterpret_cast<bf16x4*>(&L.h[jn & 1][q][(32 * ptt + li) * X_LDB + k]) = p[q];
    };
    // the last chunk (LASTIL, the Q head): tile-major -- row tile tt's four k
    // steps back to back -- so tile tt's epilogue (bias, ReLU, kept h2 rows,
    // the mask bits both ways, the head dot) runs one quarter per region in
    // the MFMA gaps of tile tt + 1, every store branch-free; only tile 3's
    // epilogue trails the MFMAs
    float bb[16], ww[16];
    float vt[16];
    uint32_t bmt = 0u;  // the tile's row word of mask bits, piece 1 -> piece 2
    const __amdgpu_buffer_rsrc_t h1r =
        __builtin_amdgcn_make_buffer_rsrc(h1g, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t hmr =
        __builtin_amdgcn_make_buffer_rsrc(hmg, (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t hmtr =
        __builtin_amdgcn_make_buffer_rsrc(hmtg, (short)0, 0x7fffffff, 0x00020000);
    // (lane indices laundered through an empty asm: the compiler otherwise
    // keeps chunk 0's address arithmetic live across the kernel and spills it)
    auto opaque = [](int v) {
      asm volatile("" : "+v"(v));
      return v;
    };
    auto tile_epi = [&](int tt, int piece) {
      const int lane = opaque(t) & 63, li = lane & 31, lh = lane >> 5;
      const int row = m0 + 32 * tt + li;
      const bool in = row >= h_from && row < rend;
      if (piece == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) vt[r] = fmaxf(acc[tt][r] + bb[r], 0.f);
        const bool kp = h1g != nullptr && in && !(PROBE & 4);
#pragma unroll
        for (int R = 0; R < (NOH2 ? 0 : 4); ++R) {
          const uint32_t off =
              kp ? (uint32_t)((row * X_H + 32 * w + 8 * R + 4 * lh) * (int)sizeof(HT)) : 0x80000000u;
          if constexpr (sizeof(HT) == 4) {
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 bits = {__float_as_uint(vt[4 * R]), __float_as_uint(vt[4 * R + 1]),
                                __float_as_uint(vt[4 * R + 2]), __float_as_uint(vt[4 * R + 3])};
            __builtin_amdgcn_raw_buffer_store_b128(bits, h1r, off, 0, 0);
          } else {
            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
            bf16x4 b;
#pragma unroll
            for (int i = 0; i < 4; ++i) b[i] = (__bf16)vt[4 * R + i];
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, b), h1r, off, 0, 0);
          }
        }
      } else if (piece == 1) {
        // the lane's 16 units as bits of the wave's 32-unit word, the two
        // lane halves or-ed (both halves then store the same word)
        uint32_t bm = 0u;  // (constant bit selects, then one shift by the half)
#pragma unroll
        for (int R = 0; R < 4; ++R)
#pragma unroll
          for (int i = 0; i < 4; ++i) bm |= vt[4 * R + i] > 0.f ? 1u << (8 * R + i) : 0u;
        bm <<= 4 * lh;
        bm |= (uint32_t)__shfl_xor((int)bm, 32, 64);
        const uint32_t off = (hmg != nullptr && in) ? (uint32_t)((row * (X_H / 32) + w) * 4) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(bm, hmr, off, 0, 0);
        bmt = bm;
      } else if (piece == 2) {
        // the tile's 32 rows as one word per unit: the 32 x 32 bit matrix of
        // the lanes' row words (lane & 31 = row, bit = unit) transposed across
        // the lanes in five block-swap stages, after which lane k holds unit
        // 32 w + k's word (bit r = row r) -- the round-4 epilogue's 16 ballots
        // and lane selects cost three times the vector instructions
        const int row0 = m0 + 32 * tt;
        const bool ok = hmtg != nullptr && row0 + 31 >= h_from && row0 < rend && lane < 32;
        uint32_t a = bmt;
#pragma unroll
        for (int st = 0; st < 5; ++st) {
          const int j = 16 >> st;
          const uint32_t m = j == 16 ? 0x0000ffffu : j == 8 ? 0x00ff00ffu : j == 4 ? 0x0f0f0f0fu
                           : j == 2 ? 0x33333333u : 0x55555555u;
          const uint32_t x = (uint32_t)__shfl_xor((int)a, j, 64);
          // rows r (r & j == 0) take the partner's low-column block into their
          // high columns; rows r | j its high-column block into their low
          // (an all-ones / all-zeros lane mask selects: a ?: here compiles to
          // a branch)
          const uint32_t hs = 0u - ((uint32_t)(lane >> (4 - st)) & 1u);
          const uint32_t hv = (a & ~m) | ((x >> j) & m), lv = (a & m) | ((x << j) & ~m);
          a = (hv & hs) | (lv & ~hs);
        }
        const uint32_t off =
            ok ? (uint32_t)((((row0 >> 5) * X_H) + (lane & 15) * 16 + 2 * w + (lane >> 4)) * 4) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(a, hmtr, off, 0, 0);
      } else {
        // the head dot of the lane's 16 units in order, the halves summed
        // (both halves hold the same sum and write it to the same slot)
        float hs = vt[0] * ww[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) hs = fmaf(vt[r], ww[r], hs);
        const float o = __shfl_xor(hs, 32, 64);
        L.hp[w][32 * tt + li] = hs + o;
      }
    };
    auto last_chunk = [&](const __bf16* hb, auto& split_w) {
      {
        const float* b1 = d.b[1] + wdel + c * d.sb[1];
        const float* wh = d.W[2] + wdel + c * d.sW[2];
#pragma unroll
        for (int R = 0; R < 4; ++R) {
          const int u = 32 * w + 8 * R + 4 * lh;
          const float4 bv = *reinterpret_cast<const float4*>(b1 + u);
          const float4 hv = *reinterpret_cast<const float4*>(wh + u);
          bb[4 * R] = bv.x; bb[4 * R + 1] = bv.y; bb[4 * R + 2] = bv.z; bb[4 * R + 3] = bv.w;
          ww[4 * R] = hv.x; ww[4 * R + 1] = hv.y; ww[4 * R + 2] = hv.z; ww[4 * R + 3] = hv.w;
        }
        b2l = (d.b[2] + wdel + c * d.sb[2])[0];
      }
      asm volatile("" ::: "memory");  // (the loads stay here, a tile ahead of their use)
      constexpr int PS = X_RB * X_LDB;
      auto rd2 = [&](int s, int tt, bf16x8* bp) {
#pragma unroll
        for (int q = 0; q < NP; ++q)
          bp[q] = *reinterpret_cast<const bf16x8*>(hb + q * PS + 32 * tt * X_LDB + 16 * s);
      };
      bf16x8 wl[X_KS][NP], bcur[NP], bnx[NP];
      if constexpr (!PRE) {
#pragma unroll
        for (int s = 0; s < X_KS; ++s) split_w(s, wl[s]);
      }
      rd2(0, 0, bcur);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int idx = 0; idx < 4 * X_KS; ++idx) {
        const int tt = idx >> 2, s = idx & 3;
        if (idx + 1 < 4 * X_KS) rd2((idx + 1) & 3, (idx + 1) >> 2, bnx);
        // (each tile's epilogue one region later, so that its first read of
        // the accumulators is a whole region of MFMAs after their last write:
        // measured 0.5 % slower)
        if (tt >= 1) tile_epi(tt - 1, s);
        acc[tt] = prodn<NP>(PRE ? wq[s] : wl[s], bcur, acc[tt]);
        if (idx + 1 < 4 * X_KS) __builtin_amdgcn_sched_group_barrier(0x0100, NP, 0);  // next reads
#pragma unroll
        for (int m = 0; m < (NP == 3 ? 6 : 1); ++m) {
          __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);  // one MFMA
          __builtin_amdgcn_sched_group_barrier(0x0002, VG, 0);  // vector instructions
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NP; ++q) bcur[q] = bnx[q];
      }
#pragma unroll
      for (int piece = 0; piece < 4; ++piece) tile_epi(3, piece);
      stamp(3 + X_NCK - 1);
    };
    // W1 as a four-slot ring of k steps: slot s holds step s of the current
    // chunk until its split, then is refilled with step s of the next
#pragma unroll
    for (int j = 0; j < X_NCK; ++j) {
      const bool more = j + 1 < X_NCK && !(PROBE & 1);
      f32x16 pa;
      if (more) {
        produce_mma(pa);
        if (j + 2 < X_NCK) load_w0w(j + 2);
      }
      const bool refill = j + 1 < X_NCK && !((PROBE & 8) && j > 0);
      auto refill_w1 = [&](int s) {
        wr[s][0] = *reinterpret_cast<const float4*>(W1 + X_CK * (j + 1) + 16 * s);
        wr[s][1] = *reinterpret_cast<const float4*>(W1 + X_CK * (j + 1) + 16 * s + 4);
      };
      const __bf16* hb = &L.h[j & 1][0][li * X_LDB + 8 * lh];
      constexpr int PS = X_RB * X_LDB;  // part stride
      auto rd = [&](int idx, bf16x8* bp) {  // idx = 4 s + tt
        const int s = idx >> 2, tt = idx & 3;
#pragma unroll
        for (int q = 0; q < NP; ++q)
          bp[q] = *reinterpret_cast<const bf16x8*>(hb + q * PS + 32 * tt * X_LDB + 16 * s);
      };
      auto split_w = [&](int s, bf16x8* wa) {
        // (the raw words pass through an empty asm here: the split is pure
        // arithmetic, and the compiler otherwise hoists it above the chunk
        // barrier to right behind the refill's load, waiting for it there)
        typedef float f32x4v __attribute__((ext_vector_type(4)));
        f32x4v r0 = {wr[s][0].x, wr[s][0].y, wr[s][0].z, wr[s][0].w};
        f32x4v r1 = {wr[s][1].x, wr[s][1].y, wr[s][1].z, wr[s][1].w};
        asm volatile("" : "+v"(r0), "+v"(r1));
        const float v[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
        if constexpr ((PROBE & 32) != 0) {
#pragma unroll
          for (int q = 0; q < NP; ++q) wa[q] = __builtin_bit_cast(bf16x8, q == 0 ? wr[s][0] : wr[s][1]);
        } else {
          splitn8<NP>(v, wa);
        }
      };
      if constexpr (LASTIL) {
        if (j == X_NCK - 1) {
          last_chunk(hb, split_w);
          continue;
        }
      }
      bf16x8 wa[2][NP], bcur[NP], bnx[NP];
      if constexpr (!PRE) {
        split_w(0, wa[0]);
        if (refill) refill_w1(0);
      }
      rd(0, bcur);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int idx = 0; idx < 4 * X_KS; ++idx) {
        const int s = idx >> 2, tt = idx & 3;
        if (idx + 1 < 4 * X_KS) rd(idx + 1, bnx);
        if constexpr (PRE) {
          // slot s - 1 took its last MFMAs in the region before
          if (tt == 0 && s >= 1 && refill) load_w1p(j + 1, s - 1);
        } else if (tt == 0 && s + 1 < X_KS) {
          split_w(s + 1, wa[(s + 1) & 1]);
          if (refill) refill_w1(s + 1);
        }
        if (more && idx >= 5 && idx <= 11 && (idx & 1)) {
          const int R = (idx - 5) >> 1;
          epi_run(j + 1, pa, b0n[R], R);
        }
        acc[tt] = prodn<NP>(PRE ? wq[s] : wa[s & 1], bcur, acc[tt]);
        if (idx + 1 < 4 * X_KS) __builtin_amdgcn_sched_group_barrier(0x0100, NP, 0);  // next reads
        if constexpr (PRE) {
          if (tt == 0 && s >= 1 && refill) __builtin_amdgcn_sched_group_barrier(0x0020, NP, 0);
        } else if (tt == 0 && s + 1 < X_KS && refill) {
          __builtin_amdgcn_sched_group_barrier(0x0020, 2, 0);
        }
#pragma unroll
        for (int m = 0; m < (NP == 3 ? 6 : 1); ++m) {
          __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);  // one MFMA
          __builtin_amdgcn_sched_group_barrier(0x0002, VG, 0);  // vector instructions
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NP; ++q) bcur[q] = bnx[q];
      }
      if constexpr (PRE) {
        if (refill) load_w1p(j + 1, X_KS - 1);
      }
      if (more && j + 2 < X_NCK) load_b0(j + 2);
      __syncthreads();  // slot j & 1 free; chunk j + 1 in slot (j + 1) & 1
      stamp(3 + j);
    }
  } else {
  // (fully unrolled: a rolled loop makes the compiler drain every outstanding
  // memory operation -- the kept-row stores included -- at its back edge)
#pragma unroll
  for (int j = 0; j < X_NCK; ++j) {
    float4 wc[X_KS][2];  // this chunk's raw W1 (the next chunk's loads reuse wr)
#pragma unroll
    for (int s = 0; s < X_KS; ++s) {
      wc[s][0] = wr[s][0];
      wc[s][1] = wr[s][1];
    }
    const bool more = j + 1 < X_NCK;
    f32x16 pa;
    if (more && !(PROBE & 1)) {
      produce_mma(pa);
      if (j + 2 < X_NCK) load_w0w(j + 2);
    }
    if (more && !((PROBE & 8) && j > 0)) load_w1(j + 1);
    const __bf16* hb = &L.h[j & 1][0][li * X_LDB + 8 * lh];
    constexpr int PS = X_RB * X_LDB;  // part stride
    auto rd = [&](int idx, bf16x8* bp) {  // idx = 4 s + tt
      const int s = idx >> 2, tt = idx & 3;
#pragma unroll
      for (int q = 0; q < NP; ++q)
        bp[q] = *reinterpret_cast<const bf16x8*>(hb + q * PS + 32 * tt * X_LDB + 16 * s);
    };
    bf16x8 bcur[NP], bnx[NP];
    rd(0, bcur);
#pragma unroll
    for (int s = 0; s < X_KS; ++s) {
      bf16x8 wa[NP];
      const float v[8] = {wc[s][0].x, wc[s][0].y, wc[s][0].z, wc[s][0].w,
                          wc[s][1].x, wc[s][1].y, wc[s][1].z, wc[s][1].w};
      if constexpr ((PROBE & 32) != 0) {
        // timing probe: the loaded words as the parts, no split arithmetic
#pragma unroll
        for (int q = 0; q < NP; ++q) wa[q] = __builtin_bit_cast(bf16x8, q == 0 ? wc[s][0] : wc[s][1]);
      } else {
        splitn8<NP>(v, wa);
      }
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const int idx = 4 * s + tt;
        if (idx + 1 < 4 * X_KS) rd(idx + 1, bnx);
        // keep the next tile's reads ahead of this tile's MFMAs
        __builtin_amdgcn_sched_barrier(0);
        acc[tt] = prodn<NP>(wa, bcur, acc[tt]);
#pragma unroll
        for (int q = 0; q < NP; ++q) bcur[q] = bnx[q];
      }
    }
    if (more && !(PROBE & 1)) produce_epi(j + 1, pa);
    __syncthreads();  // slot j & 1 free; chunk j + 1 in slot (j + 1) & 1
    stamp(3 + j);
  }
  }  // PROBE & 64: the round-4 schedule

  // ---- epilogue: bias, ReLU, kept rows to h[1], the head dot of the lane's
  // 16 units in order, then the two lane halves and the eight waves in order
  if constexpr (NO > 1) {
    // head rows over the input image (free after the last production; every
    // wave passed the chunk loop's last barrier)
    float* whl = reinterpret_cast<float*>(&L.x[0][0]);  // [output][256]
    {
      const float* whg = d.W[2] + wdel + c * d.sW[2];
      for (int e = t; e < NO * X_H; e += 512) {
        const int j = e / X_H;
        whl[e] = j < d.n_out ? whg[e] : 0.f;
      }
    }
    __syncthreads();
    float bb[16];
    {
      const float* b1 = d.b[1] + wdel + c * d.sb[1];
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const float4 bv = *reinterpret_cast<const float4*>(b1 + 32 * w + 8 * R + 4 * lh);
        bb[4 * R] = bv.x; bb[4 * R + 1] = bv.y; bb[4 * R + 2] = bv.z; bb[4 * R + 3] = bv.w;
      }
    }
    float* hpn = reinterpret_cast<float*>(&L.h[0][0][0]);  // [wave][output][row]
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = fmaxf(acc[tt][r] + bb[r], 0.f);
      const int row = m0 + 32 * tt + li;
      if (!(PROBE & 4) && h1g != nullptr && row >= h_from && row < rend) {
#pragma unroll
        for (int R = 0; R < 4; ++R) put4(h1g + row * X_H + 32 * w + 8 * R + 4 * lh, v + 4 * R);
      }
#pragma unroll
      for (int j = 0; j < NO; ++j) {
        float hs = 0.f;
#pragma unroll
        for (int R = 0; R < 4; ++R) {
          const float4 wv = *reinterpret_cast<const float4*>(&whl[j * X_H + 32 * w + 8 * R + 4 * lh]);
          if (R == 0) hs = v[0] * wv.x;
          else hs = fmaf(v[4 * R], wv.x, hs);
          hs = fmaf(v[4 * R + 1], wv.y, hs);
          hs = fmaf(v[4 * R + 2], wv.z, hs);
          hs = fmaf(v[4 * R + 3], wv.w, hs);
        }
        const float o = __shfl_xor(hs, 32, 64);
        if (lh == 0) hpn[(w * NO + j) * X_RB + 32 * tt + li] = hs + o;
      }
    }
    __syncthreads();
    const float* b2 = d.b[2] + wdel + c * d.sb[2];
    for (int e = t; e < NO * X_RB; e += 512) {
      const int m = e / NO, j = e - m * NO;
      const int row = m0 + m;
      if (j >= d.n_out || row >= rend) continue;
      float q = hpn[j * X_RB + m];
#pragma unroll
      for (int v = 1; v < 8; ++v) q += hpn[(v * NO + j) * X_RB + m];
      outp[(int64_t)row * d.ldout + j] = q + b2[j];
    }
    return;
  }
  const float b2v = LASTIL ? b2l : (d.b[2] + wdel + c * d.sb[2])[0];
  if constexpr (!LASTIL) {
  float bb[16], ww[16];
  {
    const float* b1 = d.b[1] + wdel + c * d.sb[1];
    const float* wh = d.W[2] + wdel + c * d.sW[2];
#pragma unroll
    for (int R = 0; R < 4; ++R) {
      const int u = 32 * w + 8 * R + 4 * lh;
      const float4 bv = *reinterpret_cast<const float4*>(b1 + u);
      const float4 hv = *reinterpret_cast<const float4*>(wh + u);
      bb[4 * R] = bv.x; bb[4 * R + 1] = bv.y; bb[4 * R + 2] = bv.z; bb[4 * R + 3] = bv.w;
      ww[4 * R] = hv.x; ww[4 * R + 1] = hv.y; ww[4 * R + 2] = hv.z; ww[4 * R + 3] = hv.w;
    }
  }
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = fmaxf(acc[tt][r] + bb[r], 0.f);
    const int row = m0 + 32 * tt + li;
    if (!(PROBE & 4) && h1g != nullptr && row >= h_from && row < rend) {
#pragma unroll
      for (int R = 0; R < 4; ++R) put4(h1g + row * X_H + 32 * w + 8 * R + 4 * lh, v + 4 * R);
    }
    if (hmg != nullptr) {
      // the ReLU mask of the lane's 16 units as bits of the wave's 32-unit
      // word (bit = unit - 32 w), the two lane halves or-ed together
      uint32_t bm = 0u;
#pragma unroll
      for (int R = 0; R < 4; ++R)
#pragma unroll
        for (int i = 0; i < 4; ++i) bm |= (v[4 * R + i] > 0.f ? 1u : 0u) << (8 * R + 4 * lh + i);
      bm |= (uint32_t)__shfl_xor((int)bm, 32, 64);
      if (lh == 0 && row >= h_from && row < rend) hmg[(int64_t)row * (X_H / 32) + w] = bm;
    }
    if (hmtg != nullptr) {
      // the tile's 32 rows as the bits of one word per unit: register 4 R + i
      // holds unit 32 w + 8 R + i in lanes 0-31 and + 4 in lanes 32-63, so
      // one ballot is two words; lane k of the wave stores unit 32 w + k's
      const int row0 = m0 + 32 * tt;  // wave-uniform
      if (row0 + 31 >= h_from && row0 < rend) {
        int wv = 0;
#pragma unroll
        for (int R = 0; R < 4; ++R)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const unsigned long long bl = __ballot(v[4 * R + i] > 0.f);
            // (selects, not v_writelane from inline asm: the compiler does not
            // see that asm's read of the ballot's SGPRs, and the hazard between
            // the compare writing them and the lane write went unpadded)
            const int lo = (int)(uint32_t)bl, hi = (int)(uint32_t)(bl >> 32);
            wv = lane == 8 * R + i ? lo : wv;
            wv = lane == 8 * R + 4 + i ? hi : wv;
          }
        // (a group's 256 words lane-major for the backward's 16-lane tiles:
        // unit o at (o & 15) 16 + (o >> 4))
        if (lane < 32) hmtg[(int64_t)(row0 >> 5) * X_H + (lane & 15) * 16 + 2 * w + (lane >> 4)] = (uint32_t)wv;
      }
    }
    float hs = v[0] * ww[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) hs = fmaf(v[r], ww[r], hs);
    const float o = __shfl_xor(hs, 32, 64);
    if (lh == 0) L.hp[w][32 * tt + li] = hs + o;
  }
  }  // !LASTIL
  stamp(7);
  __syncthreads();
  if (t < X_RB) {
    float q = L.hp[0][t];
#pragma unroll
    for (int v = 1; v < 8; ++v) q += L.hp[v][t];
    const int row = m0 + t;
    if (row < rend) outp[(int64_t)row * d.ldout] = q + b2v;
  }
  stamp(8);
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_q2_fwd_x6(const d3a_mlp_fwd_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_q2_fwd_x6: null desc");
  D3A_CHECK_ARG(dp->row_mean == nullptr, "d3a_q2_fwd_x6: row_mean is d3a_mlp_fwd_x6 only");
  const d3a_mlp_fwd_desc& d = *dp;
  D3A_CHECK_ARG(d.n_hidden == 2 && d.H == X_H && d.n_out >= 1 && d.n_out <= X_NOMAX &&
                    d.n_in >= 1 && d.n_in <= 48,
                "d3a_q2_fwd_x6: needs [n_in <= 48, 256, 256, n_out <= 8]");
  D3A_CHECK_ARG(d.ldout >= d.n_out, "d3a_q2_fwd_x6: ldout < n_out");
  D3A_CHECK_ARG((d.x || d.xg_mode) && d.out && d.W[0] && d.W[1] && d.W[2] && d.b[0] && d.b[1] &&
                    d.b[2],
                "d3a_q2_fwd_x6: null operand");
  D3A_CHECK_ARG(xgen_ok(d), "d3a_q2_fwd_x6: bad input-row builder (xg_*)");
  D3A_CHECK_ARG(d.hmask == nullptr ||
                    (d.n_out == 1 && (reinterpret_cast<uintptr_t>(d.hmask) & 3) == 0 &&
                     d.s_hmask >= (d.r0 + d.rows) * (X_H / 32)),
                "d3a_q2_fwd_x6: hmask needs one output and rows of 8 32-bit words");
  D3A_CHECK_ARG(d.hmaskT == nullptr ||
                    (d.hmask != nullptr && d.r0 % 32 == 0 &&
                     (reinterpret_cast<uintptr_t>(d.hmaskT) & 3) == 0 &&
                     d.s_hmaskT >= (d.r0 + d.rows + 31) / 32 * X_H),
                "d3a_q2_fwd_x6: hmaskT needs hmask, r0 % 32 == 0 and [rows / 32][256] words");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0 && d.r0 >= 0 && d.h_from >= 0 && d.aux_rows >= 0,
                "d3a_q2_fwd_x6: bad sizes");
  auto a16 = [](const void* p, int64_t stride) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && stride % 4 == 0;
  };
  D3A_CHECK_ARG(a16(d.W[1], d.sW[1]) && a16(d.b[0], d.sb[0]) && a16(d.b[1], d.sb[1]) &&
                    a16(d.W[2], d.sW[2]),
                "d3a_q2_fwd_x6: W1, b0, b1 and the head row must be 16-byte aligned");
  D3A_CHECK_ARG((d.h[0] == nullptr || (reinterpret_cast<uintptr_t>(d.h[0]) & 15) == 0) &&
                    (d.h[1] == nullptr || (reinterpret_cast<uintptr_t>(d.h[1]) & 15) == 0) &&
                    d.sh % 4 == 0,
                "d3a_q2_fwd_x6: kept activations must be 16-byte aligned rows of 256");
  D3A_CHECK_ARG(d.aux_rows == 0 || (d.aux_x && d.aux_out && d.aux_wdelta % 4 == 0),
                "d3a_q2_fwd_x6: aux pass needs aux_x, aux_out and a 16-byte aligned aux_wdelta");
  D3A_CHECK_ARG((d.r0 + d.rows) * (int64_t)(d.ldout > X_H ? d.ldout : X_H) < (int64_t(1) << 31) &&
                    (d.r0 + d.rows) * d.ldx < (int64_t(1) << 31) &&
                    d.aux_rows * (int64_t)(d.aux_ldx > X_H ? d.aux_ldx : X_H) < (int64_t(1) << 31),
                "d3a_q2_fwd_x6: rows x row stride exceeds 2^31");
  D3A_CHECK_ARG((d.r0 + d.rows) * (int64_t)X_H * 4 < (int64_t(1) << 31),
                "d3a_q2_fwd_x6: kept rows exceed 2 GB (32-bit buffer offsets)");
  const bool pre = d.wp[0] != nullptr || d.wp[1] != nullptr;
  if (pre) {
    auto al = [](const void* p) { return p != nullptr && (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    D3A_CHECK_ARG(d.n_out == 1 && d.n_in <= 32 && d.xg_mode == 0 && al(d.wp[0]) && al(d.wp[1]) &&
                      (d.aux_rows == 0 || (al(d.aux_wp[0]) && al(d.aux_wp[1]))) && al(d.x) &&
                      d.ldx % 4 == 0 && d.sxb % 4 == 0 &&
                      (d.aux_rows == 0 || (al(d.aux_x) && d.aux_ldx % 4 == 0 && d.aux_sxb % 4 == 0)),
                  "d3a_q2_fwd_x6: wp needs one output, n_in <= 32, no row builder, 16-byte aligned "
                  "images for both layers (and the aux pass's) and 16-byte input rows");
  }
  if (d.rows == 0 && d.aux_rows == 0) return 0;
  const int64_t nb = (d.rows + X_RB - 1) / X_RB + (d.aux_rows + X_RB - 1) / X_RB;
  const dim3 grid((unsigned)nb, 1, (unsigned)d.C);
  const hipStream_t st = (hipStream_t)stream;
  const int xl = (d.n_in + 15) / 16 * 16;
  if (pre) {
    static const int pprobe = [] {
      const char* e = getenv("D3A_X6_PROBE");
      return e ? atoi(e) : 0;
    }();
    const bool noh2 = d.h[1] == nullptr;
    if (xl == 16 && pprobe == 16 && noh2)  // (diagnostic: phase stamps, d3a_x6_stamps)
      hipLaunchKernelGGL((q2x6_fwd_kernel<16, 16, 3, float, 1, true, true>), grid, dim3(512), 0, st, d);

    else if (xl == 16 && noh2)
      hipLaunchKernelGGL((q2x6_fwd_kernel<16, 0, 3, float, 1, true, true>), grid, dim3(512), 0, st, d);
    else if (xl == 16)
      hipLaunchKernelGGL((q2x6_fwd_kernel<16, 0, 3, float, 1, true>), grid, dim3(512), 0, st, d);
    else if (noh2)
      hipLaunchKernelGGL((q2x6_fwd_kernel<32, 0, 3, float, 1, true, true>), grid, dim3(512), 0, st, d);
    else
      hipLaunchKernelGGL((q2x6_fwd_kernel<32, 0, 3, float, 1, true>), grid, dim3(512), 0, st, d);
    D3A_LAUNCH_CHECK("d3a_q2_fwd_x6");
    return 0;
  }
  static const int probe = [] {
    const char* e = getenv("D3A_X6_PROBE");
    return e ? atoi(e) : 0;
  }();
  if (probe && xl == 16 && d.n_out == 1) {
    switch (probe & 2047) {
      case 1: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 1>), grid, dim3(512), 0, st, d); break;
      case 4: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 4>), grid, dim3(512), 0, st, d); break;
      case 5: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 5>), grid, dim3(512), 0, st, d); break;
      case 13: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 13>), grid, dim3(512), 0, st, d); break;
      case 16: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 16>), grid, dim3(512), 0, st, d); break;
      case 32: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 32>), grid, dim3(512), 0, st, d); break;
      case 64: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 64>), grid, dim3(512), 0, st, d); break;
      case 80: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 80>), grid, dim3(512), 0, st, d); break;
      case 128: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 128>), grid, dim3(512), 0, st, d); break;
      case 144: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 144>), grid, dim3(512), 0, st, d); break;
      case 256: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 256>), grid, dim3(512), 0, st, d); break;
      case 512: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 512>), grid, dim3(512), 0, st, d); break;
      case 1024: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 1024>), grid, dim3(512), 0, st, d); break;
      default: hipLaunchKernelGGL((q2x6_fwd_kernel<16, 5>), grid, dim3(512), 0, st, d); break;
    }
    D3A_LAUNCH_CHECK("d3a_q2_fwd_x6");
    return 0;
  }
  // (timing A/B: D3A_X6_LEGACY=1 runs the narrow head at XL 32 on the round-4
  // chunk schedule)
  static const bool legacy32 = [] {
    const char* e = getenv("D3A_X6_LEGACY");
    return e && atoi(e) != 0;
  }();
  if (d.n_out > 1) {
    if (xl == 16)
      hipLaunchKernelGGL((q2x6_fwd_kernel<16, 0, 3, float, X_NOMAX>), grid, dim3(512), 0, st, d);
    else if (xl == 32 && legacy32)
      hipLaunchKernelGGL((q2x6_fwd_kernel<32, 64, 3, float, X_NOMAX>), grid, dim3(512), 0, st, d);
    else if (xl == 32)
      hipLaunchKernelGGL((q2x6_fwd_kernel<32, 0, 3, float, X_NOMAX>), grid, dim3(512), 0, st, d);
    else
      hipLaunchKernelGGL((q2x6_fwd_kernel<48, 0, 3, float, X_NOMAX>), grid, dim3(512), 0, st, d);
  } else if (xl == 16)
    hipLaunchKernelGGL(q2x6_fwd_kernel<16>, grid, dim3(512), 0, st, d);
  else if (xl == 32)
    hipLaunchKernelGGL(q2x6_fwd_kernel<32>, grid, dim3(512), 0, st, d);
  else
    hipLaunchKernelGGL(q2x6_fwd_kernel<48>, grid, dim3(512), 0, st, d);
  D3A_LAUNCH_CHECK("d3a_q2_fwd_x6");
  return 0;
}

// the bf16 throughput line's forward (d3a_q2_fwd_bf16, q2_bf16.hip): this
// kernel with one bf16 part per operand and bf16 kept activations; the caller
// has checked the descriptor
namespace d3a {
void launch_q2x1_fwd(const d3a_mlp_fwd_desc& d, hipStream_t st) {
  const int64_t nb = (d.rows + X_RB - 1) / X_RB + (d.aux_rows + X_RB - 1) / X_RB;
  const dim3 grid((unsigned)nb, 1, (unsigned)d.C);
  const int xl = (d.n_in + 15) / 16 * 16;
  if (xl == 16)
    hipLaunchKernelGGL((q2x6_fwd_kernel<16, 0, 1, __bf16>), grid, dim3(512), 0, st, d);
  else if (xl == 32)
    hipLaunchKernelGGL((q2x6_fwd_kernel<32, 0, 1, __bf16>), grid, dim3(512), 0, st, d);
  else
    hipLaunchKernelGGL((q2x6_fwd_kernel<48, 0, 1, __bf16>), grid, dim3(512), 0, st, d);
}
}  // namespace d3a

// the bf16 line's forward with fp32 kept activations (the backward that reads
// them is the mask-factored split-bf16 d3a_q2_bwd_x6): one bf16 part per
// operand, fp32 accumulation
extern "C" int d3a_q2_fwd_x1(const d3a_mlp_fwd_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_q2_fwd_x1: null desc");
  D3A_CHECK_ARG(dp->row_mean == nullptr, "d3a_q2_fwd_x1: row_mean is d3a_mlp_fwd_x6 only");
  D3A_CHECK_ARG(dp->xg_mode == 0, "d3a_q2_fwd_x1: no input-row builder");
  const d3a_mlp_fwd_desc& e = *dp;  // d3a_q2_fwd_x6's contract
  // (the ReLU mask bits of the slice backward: the same epilogue as x6's)
  D3A_CHECK_ARG(e.hmask == nullptr ||
                    ((reinterpret_cast<uintptr_t>(e.hmask) & 3) == 0 &&
                     e.s_hmask >= (e.r0 + e.rows) * (X_H / 32)),
                "d3a_q2_fwd_x1: hmask needs rows of 8 32-bit words");
  D3A_CHECK_ARG(e.hmaskT == nullptr ||
                    (e.hmask != nullptr && e.r0 % 32 == 0 &&
                     (reinterpret_cast<uintptr_t>(e.hmaskT) & 3) == 0 &&
                     e.s_hmaskT >= (e.r0 + e.rows + 31) / 32 * X_H),
                "d3a_q2_fwd_x1: hmaskT needs hmask, r0 % 32 == 0 and [rows / 32][256] words");
  D3A_CHECK_ARG(e.n_hidden == 2 && e.H == X_H && e.n_out == 1 && e.n_in >= 1 && e.n_in <= 48,
                "d3a_q2_fwd_x1: needs [n_in <= 48, 256, 256, 1]");
  D3A_CHECK_ARG(e.x && e.out && e.W[0] && e.W[1] && e.W[2] && e.b[0] && e.b[1] && e.b[2],
                "d3a_q2_fwd_x1: null operand");
  D3A_CHECK_ARG(e.C >= 1 && e.rows >= 0 && e.r0 >= 0 && e.h_from >= 0 && e.aux_rows >= 0,
                "d3a_q2_fwd_x1: bad sizes");
  auto a16 = [](const void* p, int64_t stride) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && stride % 4 == 0;
  };
  D3A_CHECK_ARG(a16(e.W[1], e.sW[1]) && a16(e.b[0], e.sb[0]) && a16(e.b[1], e.sb[1]) &&
                    a16(e.W[2], e.sW[2]),
                "d3a_q2_fwd_x1: W1, b0, b1 and the head row must be 16-byte aligned");
  D3A_CHECK_ARG((e.h[0] == nullptr || (reinterpret_cast<uintptr_t>(e.h[0]) & 15) == 0) &&
                    (e.h[1] == nullptr || (reinterpret_cast<uintptr_t>(e.h[1]) & 15) == 0) &&
                    e.sh % 4 == 0,
                "d3a_q2_fwd_x1: kept activations must be 16-byte aligned rows of 256");
  D3A_CHECK_ARG(e.aux_rows == 0 || (e.aux_x && e.aux_out && e.aux_wdelta % 4 == 0),
                "d3a_q2_fwd_x1: aux pass needs aux_x, aux_out and a 16-byte aligned aux_wdelta");
  D3A_CHECK_ARG((e.r0 + e.rows) * (int64_t)(e.ldout > X_H ? e.ldout : X_H) < (int64_t(1) << 31) &&
                    (e.r0 + e.rows) * e.ldx < (int64_t(1) << 31) &&
                    e.aux_rows * (int64_t)(e.aux_ldx > X_H ? e.aux_ldx : X_H) < (int64_t(1) << 31),
                "d3a_q2_fwd_x1: rows x row stride exceeds 2^31");
  D3A_CHECK_ARG((e.r0 + e.rows) * (int64_t)X_H * 4 < (int64_t(1) << 31),
                "d3a_q2_fwd_x1: kept rows exceed 2 GB (32-bit buffer offsets)");
  if (e.rows == 0 && e.aux_rows == 0) return 0;
  const int64_t nb = (e.rows + X_RB - 1) / X_RB + (e.aux_rows + X_RB - 1) / X_RB;
  const dim3 grid((unsigned)nb, 1, (unsigned)e.C);
  const hipStream_t st = (hipStream_t)stream;
  const int xl = (e.n_in + 15) / 16 * 16;
  if (xl == 16)
    hipLaunchKernelGGL((q2x6_fwd_kernel<16, 0, 1, float>), grid, dim3(512), 0, st, e);
  else if (xl == 32)
    hipLaunchKernelGGL((q2x6_fwd_kernel<32, 0, 1, float>), grid, dim3(512), 0, st, e);
  else
    hipLaunchKernelGGL((q2x6_fwd_kernel<48, 0, 1, float>), grid, dim3(512), 0, st, e);
  D3A_LAUNCH_CHECK("d3a_q2_fwd_x1");
  return 0;
}

// ---- d3a_x6_split (include/d3rlpy_amd.h): one piece a thread
__global__ __launch_bounds__(256) void x6_split_kernel(d3a_x6_split_desc d, int64_t total) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p < total) x6::x6_split_piece(d, p);
}

extern "C" int d3a_x6_split(const d3a_x6_split_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp && x6::x6_split_ok(*dp),
                "d3a_x6_split: jobs need src, 16-byte aligned dst, 1 <= k <= kpad, kpad % 16 == 0");
  const int64_t total = x6::x6_split_total(*dp);
  if (total == 0) return 0;
  hipLaunchKernelGGL(x6_split_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, *dp, total);
  D3A_LAUNCH_CHECK("d3a_x6_split");
  return 0;
}

// diagnostic: copy the stamp buffer of the last D3A_X6_PROBE & 16 launch
extern "C" int d3a_x6_stamps(unsigned long long* dst, int n) {
  D3A_CHECK_ARG(dst && n >= 0 && n <= 2048 * 10, "d3a_x6_stamps: bad arguments");
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(x6_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost) !=
      hipSuccess) {
    set_error("d3a_x6_stamps: copy failed");
    return -2;
  }
  return 0;
}
