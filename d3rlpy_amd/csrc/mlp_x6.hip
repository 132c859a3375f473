// fp32-accurate forward of a two-hidden-layer ensemble MLP with a wide head,
// [n_in <= 64 -> 256 -> 256 -> n_out <= 256], on the bf16 matrix cores
// (exact three-way split-bf16 operands, the six part products above fp32
// resolution, fp32 accumulation: x6.hpp, q2_x6.hip).
//
// The pass it is for: BCQ's target step (bcq_impl.py:215-226 through
// compute_max_with_n_actions, q_functions/__init__.py:8-63) evaluates the
// target QR critics [obs + act -> 256 -> 256 -> 200 quantiles]
// (encoders.py:265-275, 328-339; qr_q_function.py:97-161) over B * N = 25,600
// sampled actions per member -- 12.56 GFLOP per K3 step, the largest GEMM of
// the BCQ update -- and the target residual policy [obs + act -> 256 -> 256 ->
// act] over the same rows.  d3a_mlp_fwd's contract (kept activations optional,
// no aux pass, out [C][rows][ldout]).
//
// A workgroup owns 64 rows of one member; eight waves (two per SIMD).  Every
// layer is the same product shape: wave w computes a transposed 32 x 64 block
// C^T[32 outputs][64 rows] (two v_mfma_f32_32x32x16_bf16 tiles; A = 32 weight
// rows, split from fp32 loads, B = an LDS image of the layer input's parts,
// [row][k]):
//   layer 1: units 32 w .. + 31 over K = n_in (the staged input parts), written
//     as parts to the 64 x 256 activation image;
//   layer 2: units 32 w .. + 31 over K = 256 of that image -- a stream of
//     16 k steps with no barrier, the weight rows four steps ahead;
//   head: after one barrier the layer-2 activations replace the image, and
//     wave w < ceil(n_out / 32) streams outputs 32 w .. + 31 the same way.
// Barriers: input staged, image 1 written, layer 2 read out, image 2 written
// (+ one for row_mean).  Round 5 measured the previous design (layer 1
// produced chunk by chunk inside the layer-2 loop, a barrier per chunk) at
// 71k cycles per workgroup, of which 12.5k were the interleaved production
// and 3.4k its barriers (tools/bench_wide.py ablations).
#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include "common.hpp"
#include "../../include/d3rlpy_amd.h"
#include "x6.hpp"

namespace d3a {
namespace {

using namespace x6;

constexpr int W_H = 256;    // hidden width
constexpr int W_RB = 64;    // rows per workgroup
constexpr int W_LDH = 264;  // bf16 stride of an image row (528 B)
// weight k steps in flight (8 registers a step).  It divides the 16 steps of
// a stream: the refills at a stream's end leave the next stream's steps
// 0 .. W_HD - 1 in slots 0 .. W_HD - 1.
constexpr int W_HD = 4;
static_assert(16 % W_HD == 0, "W_HD must divide 16");

template <int XL>
struct WideLds {
  __bf16 x[3][W_RB * (XL + 8)];  // input parts [row][k]
  // layer-1, then layer-2 activation parts [row][part][unit]: the parts of a
  // row adjacent, so every read of a lane's two row tiles lies within 64 KB
  // of one base (one address register + immediate offsets)
  __bf16 img[W_RB * 3 * W_LDH];
  float rs[8][W_RB];             // row_mean: per-wave output sums [wave][row]
};

// diagnostic phase stamps (STAMPS, D3A_WIDE_STAMPS=1; read with
// d3a_wide_stamps): wave 0 of each workgroup records s_memtime in its
// second tile (the steady state) at 0 the tile's start, 1 before the input
// barrier, 2 after it, 3 image 1 written, 4 layer-2 products issued, 5 image
// 2 written, 6 head products issued, 7 outputs stored; 8 = the kernel's end
// minus its start (the workgroup's whole lifetime)
constexpr int W_NST = 9;
__device__ unsigned long long wide_stamps[1024 * W_NST];
// (three hidden layers) every wave's stamps: [workgroup < 512][wave][8]
__device__ unsigned long long wide_wstamps[512 * 8 * 8];

// a weight matrix as a buffer resource: raw buffer loads are ordered by the
// compiler fences below (plain loads of read-only weights are free to sink to
// their first use, undoing the prefetch), and an offset past the matrix
// reads zero
struct WMat {
  __amdgpu_buffer_rsrc_t rs;
};
__device__ __forceinline__ WMat wmat(const void* base, int bytes) {
  return WMat{__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000)};
}
// (lane offset in voffset, the step's constant in soffset: a constant in
// voffset gets its own register per step)
__device__ __forceinline__ float4 wload(const WMat& m, int lane_off, int step_off) {
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  const f32x4v v =
      __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(m.rs, lane_off, step_off, 0));
  return make_float4(v.x, v.y, v.z, v.w);
}

// o[rt] += W[32 rows][256] x img[64 rows][256]^T for this lane's weight row
// (byte offset wo of its k = 8 lh in matrix wm): hr holds the raw fp32 of k
// steps 0 .. w_hd - 1 on entry and, on exit, steps 0 .. w_hd - 1 of the row at
// (nm, no) (the stream that follows).  Software-pipelined by hand: step s
// issues step s + 1's image reads and weight split (and the refill of the
// slot that split frees) ahead of its own twelve MFMAs; a compiler memory
// fence closes each step, and the schedule interleaves the split's vector
// instructions into the MFMA gaps (an MFMA issues 32 cycles, holding the
// vector issue for 8 of them).
// NRT: row tiles of 32 (1 for a workgroup's last odd 32-row half)
// TR: the weight matrix read transposed (the backward chain's W^T rows are W's
// columns): the lane's 8 k of a step are 8 dwords 1 KB apart (coalesced across
// the lanes of a k), lane offset wo = (8 lh * 256 + unit) * 4, step s at 16 KB s
__device__ __forceinline__ float wload1(const WMat& m, int lane_off, int step_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(m.rs, lane_off, step_off, 0));
}
template <int NRT, bool TR = false>
__device__ __forceinline__ void stream256(const WMat& wm, int wo, const WMat& nm, int no,
                                          float4 (&hr)[W_HD][2], const __bf16 (&img)[W_RB * 3 * W_LDH],
                                          int li, int lh, f32x16 (&o)[NRT]) {
  constexpr int NS = W_H / 16;
  auto split_slot = [&](int sl, bf16x8 (&wa)[3]) {
    const float v[8] = {hr[sl][0].x, hr[sl][0].y, hr[sl][0].z, hr[sl][0].w,
                        hr[sl][1].x, hr[sl][1].y, hr[sl][1].z, hr[sl][1].w};
    split8(v, wa);
  };
  auto refill = [&](int s) {  // the slot of step s, with step s + W_HD
    const int sl = s % W_HD, s2 = s + W_HD;
    const WMat& m = s2 < NS ? wm : nm;
    const int lo = s2 < NS ? wo : no;
    if constexpr (TR) {
      const int st = 16384 * (s2 < NS ? s2 : s2 - NS);
      hr[sl][0] = make_float4(wload1(m, lo, st), wload1(m, lo, st + 1024), wload1(m, lo, st + 2048),
                              wload1(m, lo, st + 3072));
      hr[sl][1] = make_float4(wload1(m, lo, st + 4096), wload1(m, lo, st + 5120),
                              wload1(m, lo, st + 6144), wload1(m, lo, st + 7168));
    } else {
      const int st = 64 * (s2 < NS ? s2 : s2 - NS);
      hr[sl][0] = wload(m, lo, st);
      hr[sl][1] = wload(m, lo, st + 16);
    }
  };
  auto read_img = [&](int s, bf16x8 (&bp)[NRT][3]) {
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        bp[rt][q] = *reinterpret_cast<const bf16x8*>(&img[((32 * rt + li) * 3 + q) * W_LDH + 16 * s + 8 * lh]);
  };
  bf16x8 wa[2][3], bp[2][NRT][3];
  split_slot(0, wa[0]);
  refill(0);
  read_img(0, bp[0]);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int cur = s & 1, nx = cur ^ 1;
    if (s + 1 < NS) {
      read_img(s + 1, bp[nx]);
      split_slot((s + 1) % W_HD, wa[nx]);
      refill(s + 1);
    }
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) o[rt] = prod6(wa[cur], bp[cur][rt], o[rt]);
    if (s + 1 < NS) {
      __builtin_amdgcn_sched_group_barrier(0x0100, 3 * NRT, 0);  // next step's image reads
      __builtin_amdgcn_sched_group_barrier(0x0020, TR ? 8 : 2, 0);  // the refill
#pragma unroll
      for (int m = 0; m < 6 * NRT; ++m) {
        __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);            // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x0002, 8 / NRT, 0);  // the split's vector instructions
      }
    }
    // a compiler memory fence: the next step's reads stay in this step
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
}

// PW: the weights as pre-split operand images (d3a_x6_split's layout: a row
// of 256 k is 32 blocks of [3 parts][8 bf16], 1536 bytes; the lane's k = 8 lh
// block at byte wo, step s at + 96 s): the ring holds each step's three parts
// and the MFMAs read them in place -- no split instructions between the
// MFMAs (with two waves a SIMD, a wave's vector instructions delay the other
// wave's products nearly one for one: tools/bench_wide3.py's wave stamps)
template <bool PW> struct WRing;
template <> struct WRing<false> { float4 r[W_HD][2]; };
template <> struct WRing<true> { bf16x8 r[W_HD][3]; };

__device__ __forceinline__ bf16x8 pload(const WMat& m, int lane_off, int step_off) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  return __builtin_bit_cast(bf16x8, __builtin_bit_cast(s16x8, __builtin_amdgcn_raw_buffer_load_b128(m.rs, lane_off, step_off, 0)));
}

template <int NRT>
__device__ __forceinline__ void stream256p(const WMat& wm, int wo, const WMat& nm, int no,
                                           WRing<true>& hq, const __bf16 (&img)[W_RB * 3 * W_LDH],
                                           int li, int lh, f32x16 (&o)[NRT]) {
  constexpr int NS = W_H / 16;
  auto refill = [&](int s) {  // the slot of step s, with step s + W_HD
    const int sl = s % W_HD, s2 = s + W_HD;
    const WMat& m = s2 < NS ? wm : nm;
    const int lo = s2 < NS ? wo : no, st = 96 * (s2 < NS ? s2 : s2 - NS);
#pragma unroll
    for (int q = 0; q < 3; ++q) hq.r[sl][q] = pload(m, lo, st + 16 * q);
  };
  auto read_img = [&](int s, bf16x8 (&bp)[NRT][3]) {
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        bp[rt][q] = *reinterpret_cast<const bf16x8*>(&img[((32 * rt + li) * 3 + q) * W_LDH + 16 * s + 8 * lh]);
  };
  bf16x8 bp[2][NRT][3];
  read_img(0, bp[0]);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int cur = s & 1, nx = cur ^ 1;
    if (s + 1 < NS) read_img(s + 1, bp[nx]);
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) o[rt] = prod6(hq.r[s % W_HD], bp[cur][rt], o[rt]);
    refill(s);  // (after the products that read the slot)
    if (s + 1 < NS) __builtin_amdgcn_sched_group_barrier(0x0100, 3 * NRT, 0);  // next step's image reads
#pragma unroll
    for (int m = 0; m < 6 * NRT; ++m) __builtin_amdgcn_sched_group_barrier(0x0008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x0020, 3, 0);  // the refill
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
}

// bias, ReLU, kept rows to hg, parts into the image: lane holds rows
// 32 rt + li, units 32 w + 8 R + 4 lh + i
template <bool KEEP, int NRT>
__device__ __forceinline__ void act_to_image(const f32x16 (&o)[NRT], const float4 (&bv)[4], float* hg, int m0,
                                             int h_from, int rend, int w, int li, int lh,
                                             __bf16 (&img)[W_RB * 3 * W_LDH]) {
#pragma unroll
  for (int R = 0; R < 4; ++R) {
    const int u = 32 * w + 8 * R + 4 * lh;
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) {
      const int rl = 32 * rt + li;
      const int row = m0 + rl;
      float v[4] = {fmaxf(o[rt][4 * R + 0] + bv[R].x, 0.f), fmaxf(o[rt][4 * R + 1] + bv[R].y, 0.f),
                    fmaxf(o[rt][4 * R + 2] + bv[R].z, 0.f), fmaxf(o[rt][4 * R + 3] + bv[R].w, 0.f)};
      if (KEEP && hg != nullptr && row >= h_from && row < rend)
        *reinterpret_cast<float4*>(hg + row * W_H + u) = make_float4(v[0], v[1], v[2], v[3]);
      bf16x4 p[3];
      split4(v, p);
#pragma unroll
      for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x4*>(&img[(rl * 3 + q) * W_LDH + u]) = p[q];
    }
  }
}

// XL: n_in rounded up to 32 (32 or 64); KEEP: some kept activations (h[0] /
// h[1] / h[2]) are written (without them no store precedes the head's).
//
// NHID: 256-wide hidden layers (2, or 3 for the CQL reproduction critic
// [obs + act, 256, 256, 256, 1], reproductions/offline/cql.py:21-37): the
// third is one more barrier-free stream over the image of the second.
// HD (one output): the Q head as a register dot -- each wave's last-layer
// activations times its 32 head weights, the lane halves and the eight waves'
// partials summed in order -- instead of a head stream on one wave while
// seven idle.
//
// Aux pass (d3a_mlp_fwd_desc.aux_rows > 0): workgroups C Gm .. C Gm + C Ga - 1
// run the same network at parameter offset aux_wdelta (the target critics)
// over aux_x, into aux_out, keeping nothing; Gm / Ga workgroups a member.
//
// Persistent: grid (G, 1, C), G <= the CU count / C, one workgroup per CU
// (the LDS image allows no second).  Member c's rows are cut into 32-row
// halves, workgroup k owning the contiguous range [k H / G, (k + 1) H / G)
// of its H halves, processed as 64-row tiles (a last odd half as a
// 32-row tile with the second row tile masked): every workgroup carries
// 2-3.5 tiles' work instead of whole 64-row blocks dealt in rounds (3.125
// rounds of 256 at K3's 800 blocks = 4 rounds).  While tile i runs its layer 2
// and head, the next tile's input rows and first weight steps are in flight
// (XRaw4 registers, the freed slots of the weight stream), so only the first
// tile pays the prologue's memory round trip.
template <int XL, bool KEEP, bool STAMPS = false, int NHID = 2, bool HD = false, bool PW = false>
__global__ __launch_bounds__(512) void mlp_x6_wide_kernel(d3a_mlp_fwd_desc d, int Gm, int Ga) {
  constexpr int XLD = XL + 8;
  constexpr int NS1 = XL / 16;  // layer-1 k steps
  constexpr int X4 = XL / 4;
  constexpr int NXQ = (W_RB * X4 + 511) / 512;  // input quads per thread
  __shared__ __attribute__((aligned(16))) WideLds<XL> L;
  static_assert(sizeof(WideLds<XL>) <= 163840, "LDS");
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lh = lane >> 5;
  // (flat grid: the main pass's C Gm workgroups, then the aux pass's C Ga)
  const int bid = (int)blockIdx.x;
  const bool aux = bid >= d.C * Gm;
  const int G = aux ? Ga : Gm;
  const int c = aux ? (bid - d.C * Gm) / Ga : bid / Gm;
  const int k = aux ? (bid - d.C * Gm) % Ga : bid % Gm;
  const int r0 = aux ? 0 : (int)d.r0, rlim = aux ? (int)d.aux_rows : (int)(d.r0 + d.rows);
  const int nh = (rlim - r0 + 31) / 32;  // 32-row halves of this member
  const int hb = (int)((int64_t)k * nh / G), he = (int)((int64_t)(k + 1) * nh / G);
  if (hb >= he) return;  // uniform: no rows for this workgroup
  const int h_from = aux ? rlim : (int)d.h_from;
  const int nin = d.n_in, nout = d.n_out;
  const int64_t wdel = aux ? d.aux_wdelta : 0;
  float* const outp = aux ? d.aux_out + c * d.aux_sout : d.out + c * d.sout;
  float* const h0g = KEEP && !aux && d.h[0] ? d.h[0] + c * d.sh : nullptr;
  float* const h1g = KEEP && !aux && d.h[1] ? d.h[1] + c * d.sh : nullptr;
  float* const h2g = KEEP && NHID == 3 && !aux && d.h[2] ? d.h[2] + c * d.sh : nullptr;
  float* const rmean = aux ? nullptr : d.row_mean;
  const int u0 = 32 * w + li;  // this lane's weight row in the hidden layers
  const float* W0r = d.W[0] + wdel + c * d.sW[0] + u0 * nin;
  // (PW: the stream matrices' images, wp[0] = W[1]'s and wp[1] = W[2]'s --
  // layer 3's, or the wide head's)
  const char* const wpi0 = PW ? static_cast<const char*>(aux ? d.aux_wp[0] : d.wp[0]) : nullptr;
  const char* const wpi1 = PW ? static_cast<const char*>(aux ? d.aux_wp[1] : d.wp[1]) : nullptr;
  const WMat W1m = PW ? wmat(wpi0 + (int64_t)c * W_H * 1536, W_H * 1536)
                      : wmat(d.W[1] + wdel + c * d.sW[1], W_H * W_H * 4);
  const WMat W2m = PW ? wmat(wpi1 + (int64_t)c * W_H * 1536, W_H * 1536)
                      : wmat(d.W[NHID == 3 ? 2 : 1] + wdel + c * d.sW[NHID == 3 ? 2 : 1], W_H * W_H * 4);
  // byte offset of this lane's W1 row piece (k = 8 lh)
  const int w1o = PW ? u0 * 1536 + lh * 48 : (u0 * W_H + 8 * lh) * 4;
  const float* b0 = d.b[0] + wdel + c * d.sb[0];
  const float* b1 = d.b[1] + wdel + c * d.sb[1];
  const float* b2 = d.b[NHID == 3 ? 2 : 1] + wdel + c * d.sb[NHID == 3 ? 2 : 1];
  const float* Wh = d.W[NHID] + wdel + c * d.sW[NHID];
  const float* bh = d.b[NHID] + wdel + c * d.sb[NHID];
  const float* xb = aux ? d.aux_x + c * d.aux_sxb : d.x + c * d.sxb;
  const int64_t ldx = aux ? d.aux_ldx : d.ldx;
  const int nkt = (nout + 31) / 32;
  const int kout = 32 * w + li;  // head: this lane's output row (rows past n_out read row 0:
  const WMat Whm = PW && NHID == 2 ? wmat(wpi1 + (int64_t)c * nout * 1536, nout * 1536)
                                   : wmat(Wh, nout * W_H * 4);
  const int who = PW && NHID == 2 ? (kout < nout ? kout : 0) * 1536 + lh * 48
                                  : ((kout < nout ? kout : 0) * W_H + 8 * lh) * 4;  // never stored)
  const int wgi = bid;
  const unsigned long long t_start = STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
  auto stamp = [&](int s, bool on) {
    if constexpr (STAMPS) {
      __builtin_amdgcn_sched_barrier(0);
      if (on && t == 0 && wgi < 1024) wide_stamps[wgi * W_NST + s] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // (three hidden layers) every wave: 0 tile start, 1 image 1 written, 2 layer
  // 2 issued, 3 past the barrier after it, 4 image 2 formed, 5 image 2
  // written, 6 layer 3 issued, 7 head written
  auto wstamp = [&](int s, bool on) {
    if constexpr (STAMPS && NHID == 3) {
      __builtin_amdgcn_sched_barrier(0);
      if (on && lane == 0 && wgi < 512) wide_wstamps[(wgi * 8 + w) * 8 + s] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // the tile starting at half h: rows [r0 + 32 h, tile_end)
  auto tile_end = [&](int h) { return min(r0 + 32 * min(h + 2, he), rlim); };
  XRaw4 xr[NXQ];
  // (the lane-dependent index arithmetic of the tile loop works from a
  // laundered thread index: hoisted out of the loop, its clamped indices and
  // lane predicates would occupy registers across the whole loop)
  auto opaque = [](int v) {
    asm volatile("" : "+v"(v));
    return v;
  };
  auto issue_x = [&](int h) {
    const int m0 = r0 + 32 * h, te = tile_end(h);
    const int tl = opaque(t);
#pragma unroll
    for (int q = 0; q < NXQ; ++q) {
      const int e = tl + 512 * q;
      const int m = min(e / X4, W_RB - 1), k4 = (e % X4) * 4;
      input4_issue(d, xb, ldx, m0 + m, k4, te, nin, xr[q]);
    }
  };
  auto stage_x = [&](int h) {
    const int m0 = r0 + 32 * h, te = tile_end(h);
    const int tl = opaque(t);
#pragma unroll
    for (int q = 0; q < NXQ; ++q) {
      const int e = tl + 512 * q;
      if (e < W_RB * X4) {
        const int m = e / X4, k4 = (e % X4) * 4;
        float v[4];
        input4_finish(d, m0 + m, k4, te, nin, xr[q], v);
        bf16x4 p[3];
        split4(v, p);
#pragma unroll
        for (int q3 = 0; q3 < 3; ++q3) *reinterpret_cast<bf16x4*>(&L.x[q3][m * XLD + k4]) = p[q3];
      }
    }
  };

  // ---- prologue: layer-2 weight steps 0 .. w_hd - 1 and the first tile's rows
  WRing<PW> ring;
#pragma unroll
  for (int s = 0; s < W_HD; ++s) {
    if constexpr (PW) {
#pragma unroll
      for (int q = 0; q < 3; ++q) ring.r[s][q] = pload(W1m, w1o, 96 * s + 16 * q);
    } else {
      ring.r[s][0] = wload(W1m, w1o, 64 * s);
      ring.r[s][1] = wload(W1m, w1o, 64 * s + 16);
    }
  }
  // one stream over the image: weights wm (this lane at byte wo), the next
  // stream's first steps from nm at no into the freed slots
  auto stream = [&](auto nrt, const WMat& wm, int wo, const WMat& nm, int no,
                    f32x16 (&oo)[decltype(nrt)::value]) {
    constexpr int NRT_ = decltype(nrt)::value;
    if constexpr (PW) stream256p<NRT_>(wm, wo, nm, no, ring, L.img, li, lh, oo);
    else stream256<NRT_>(wm, wo, nm, no, ring.r, L.img, li, lh, oo);
  };
  issue_x(hb);
  stage_x(hb);

  // one tile: 64 rows from half h (NRT = 2), or the last odd half alone
  // (NRT = 1: one row tile, half the products)
  auto tile = [&](auto nrt, int h) {
    constexpr int NRT = decltype(nrt)::value;
      const int m0 = r0 + 32 * h, rend = tile_end(h);
      const bool has_next = h + 2 < he;
      // the stamped tile: the second (the steady state), or a workgroup's only one
      const bool first = h == hb + 2 || he - hb <= 2;
      stamp(0, first);
      wstamp(0, first);
      // the layer-1 weight row (clamped k, masked at use) and bias, reloaded per
      // tile (L2 hits) so that no register holds them across the streams; a
      // wave reaching this point early waits at the barrier anyway
      const int lhl = opaque(lh);
      float w0r[NS1][8];
  #pragma unroll
      for (int s = 0; s < NS1; ++s)
  #pragma unroll
        for (int i = 0; i < 8; ++i) w0r[s][i] = W0r[min(16 * s + 8 * lhl + i, nin - 1)];
      float4 b0v[4];
  #pragma unroll
      for (int R = 0; R < 4; ++R) b0v[R] = *reinterpret_cast<const float4*>(b0 + 32 * w + 8 * R + 4 * lh);
      stamp(1, first);
      __syncthreads();  // input parts staged; the previous head done with the image
      stamp(2, first);

      // ---- layer 1: units 32 w .. over K = XL (x parts past n_in are zero, the
      // weights there masked to zero)
      f32x16 o[NRT];
  #pragma unroll
      for (int rt = 0; rt < NRT; ++rt)
  #pragma unroll
        for (int r = 0; r < 16; ++r) o[rt][r] = 0.f;
  #pragma unroll
      for (int s = 0; s < NS1; ++s) {
        float v[8];
  #pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = 16 * s + 8 * lhl + i < nin ? w0r[s][i] : 0.f;
        bf16x8 wa[3];
        split8(v, wa);
  #pragma unroll
        for (int rt = 0; rt < NRT; ++rt) {
          bf16x8 bp[3];
  #pragma unroll
          for (int q = 0; q < 3; ++q)
            bp[q] = *reinterpret_cast<const bf16x8*>(&L.x[q][(32 * rt + li) * XLD + 16 * s + 8 * lh]);
          o[rt] = prod6(wa, bp, o[rt]);
        }
      }
      float4 b1v[4];
  #pragma unroll
      for (int R = 0; R < 4; ++R) b1v[R] = *reinterpret_cast<const float4*>(b1 + 32 * w + 8 * R + 4 * lh);
      act_to_image<KEEP, NRT>(o, b0v, h0g, m0, h_from, rend, w, li, lh, L.img);
      __syncthreads();  // image 1 complete; every wave done reading the input parts
      stamp(3, first);
      wstamp(1, first);
      if (has_next) issue_x(h + 2);  // uniform

      // ---- layer 2: units 32 w .. over the image; the freed weight slots take
      // the next stream's first steps: layer 3's (NHID 3), else the head's
      // (waves with no head: the next tile's layer 2)
  #pragma unroll
      for (int rt = 0; rt < NRT; ++rt)
  #pragma unroll
        for (int r = 0; r < 16; ++r) o[rt][r] = 0.f;
      // (waves streaming a head after the last hidden layer; HD: none)
      const bool hs = !HD && w < nkt;
      if constexpr (NHID == 3) {
        stream(std::integral_constant<int, NRT>{}, W1m, w1o, W2m, w1o, o);
      } else {
        const WMat nm{hs ? Whm.rs : W1m.rs};  // uniform
        stream(std::integral_constant<int, NRT>{}, W1m, w1o, nm, hs ? who : w1o, o);
      }
      stamp(4, first);
      wstamp(2, first);
      if constexpr (NHID == 3) {
        float4 b2v[4];
  #pragma unroll
        for (int R = 0; R < 4; ++R) b2v[R] = *reinterpret_cast<const float4*>(b2 + 32 * w + 8 * R + 4 * lh);
        // (measured: forming the parts before this barrier, so that an early
        // wave splits while its SIMD's other wave multiplies, slowed that
        // wave's stream by as much -- 37.3 against 37.4 us)
        __syncthreads();  // every wave done reading image 1
        wstamp(3, first);
        act_to_image<KEEP, NRT>(o, b1v, h1g, m0, h_from, rend, w, li, lh, L.img);
        wstamp(4, first);
        __syncthreads();  // image 2 complete
        stamp(5, first);
        wstamp(5, first);
        // ---- layer 3 over image 2; the freed slots take the head's first
        // steps (no head stream: the next tile's layer 2)
  #pragma unroll
        for (int rt = 0; rt < NRT; ++rt)
  #pragma unroll
          for (int r = 0; r < 16; ++r) o[rt][r] = 0.f;
        {
          const WMat nm{hs ? Whm.rs : W1m.rs};  // uniform
          stream(std::integral_constant<int, NRT>{}, W2m, w1o, nm, hs ? who : w1o, o);
        }
        stamp(6, first);
        wstamp(6, first);
        // (the register head writes no image: no barrier; a wave that is
        // done forms its head partials while the others still multiply)
        if constexpr (!HD) __syncthreads();  // every wave done reading image 2
  #pragma unroll
        for (int R = 0; R < 4; ++R) b1v[R] = b2v[R];
      } else {
        __syncthreads();  // every wave done reading image 1
      }
      // the last hidden layer's activations: kept rows, and (no register head)
      // the image the head streams
      float* const hlg = NHID == 3 ? h2g : h1g;
      if constexpr (HD) {
        // Q head as a register dot: this lane's 16 units of each of its rows
        float hw[4][4];
  #pragma unroll
        for (int R = 0; R < 4; ++R) {
          const float4 q = *reinterpret_cast<const float4*>(Wh + 32 * w + 8 * R + 4 * lh);
          hw[R][0] = q.x, hw[R][1] = q.y, hw[R][2] = q.z, hw[R][3] = q.w;
        }
  #pragma unroll
        for (int rt = 0; rt < NRT; ++rt) {
          const int rl = 32 * rt + li;
          const int row = m0 + rl;
          float acc = 0.f;
  #pragma unroll
          for (int R = 0; R < 4; ++R) {
            const int u = 32 * w + 8 * R + 4 * lh;
            const float bb[4] = {b1v[R].x, b1v[R].y, b1v[R].z, b1v[R].w};
            float v[4];
  #pragma unroll
            for (int i = 0; i < 4; ++i) {
              v[i] = fmaxf(o[rt][4 * R + i] + bb[i], 0.f);
              acc = fmaf(v[i], hw[R][i], acc);
            }
            if (KEEP && hlg != nullptr && row >= h_from && row < rend)
              *reinterpret_cast<float4*>(hlg + row * W_H + u) = make_float4(v[0], v[1], v[2], v[3]);
          }
          const float other = __shfl_xor(acc, 32, 64);
          if (lh == 0) L.rs[w][rl] = acc + other;
        }
        if (has_next) stage_x(h + 2);  // the input region is free since image 1
        __syncthreads();  // the eight waves' head partials
        if (t < 32 * NRT) {
          float q = L.rs[0][t];
  #pragma unroll
          for (int v = 1; v < 8; ++v) q += L.rs[v][t];
          const int row = m0 + t;
          if (row < rend) {
            q += bh[0];
            outp[(int64_t)row * d.ldout] = q;
            if (rmean != nullptr) rmean[c * d.s_mean + row] = q;
          }
        }
        stamp(7, first);
        wstamp(7, first);
        return;
      } else {
      act_to_image<KEEP, NRT>(o, b1v, hlg, m0, h_from, rend, w, li, lh, L.img);
      // head bias of this lane's outputs 32 w + 8 R + 4 lh + i (clamped index)
      float bhv[4][4];
  #pragma unroll
      for (int R = 0; R < 4; ++R)
  #pragma unroll
        for (int i = 0; i < 4; ++i) bhv[R][i] = bh[min(32 * w + 8 * R + 4 * lhl + i, nout - 1)];
      if (has_next) stage_x(h + 2);  // the input region is free since image 1
      __syncthreads();  // image 2 complete
      stamp(5, first);

      // ---- head: wave w < nkt computes outputs 32 w .. + 31; its freed weight
      // slots take the next tile's first layer-2 steps
      if (w < nkt) {
  #pragma unroll
        for (int rt = 0; rt < NRT; ++rt)
  #pragma unroll
          for (int r = 0; r < 16; ++r) o[rt][r] = 0.f;
        stream(std::integral_constant<int, NRT>{}, Whm, who, W1m, w1o, o);
        stamp(6, first);
        // lane: row 32 rt + li, outputs 32 w + 8 R + 4 lh + i
        const int64_t ldo = d.ldout;
        float rsum[2] = {0.f, 0.f};  // row_mean: this lane's outputs, in output order
        const bool vec = ((reinterpret_cast<uintptr_t>(outp) & 15) == 0) && (ldo & 3) == 0;
        const int lho = opaque(lh), lio = opaque(li);
  #pragma unroll
        for (int R = 0; R < 4; ++R) {
          const int k0 = 32 * w + 8 * R + 4 * lho;
          float bv[4];
  #pragma unroll
          for (int i = 0; i < 4; ++i) bv[i] = k0 + i < nout ? bhv[R][i] : 0.f;
  #pragma unroll
          for (int rt = 0; rt < NRT; ++rt) {
            const int row = m0 + 32 * rt + lio;
            if (row >= rend) continue;
            float* op = outp + (int64_t)row * ldo + k0;
            const float v0 = o[rt][4 * R] + bv[0], v1 = o[rt][4 * R + 1] + bv[1];
            const float v2 = o[rt][4 * R + 2] + bv[2], v3 = o[rt][4 * R + 3] + bv[3];
            if (k0 + 0 < nout) rsum[rt] += v0;
            if (k0 + 1 < nout) rsum[rt] += v1;
            if (k0 + 2 < nout) rsum[rt] += v2;
            if (k0 + 3 < nout) rsum[rt] += v3;
            if (k0 + 3 < nout && vec) {
              *reinterpret_cast<float4*>(op) = make_float4(v0, v1, v2, v3);
            } else {
              if (k0 + 0 < nout) op[0] = v0;
              if (k0 + 1 < nout) op[1] = v1;
              if (k0 + 2 < nout) op[2] = v2;
              if (k0 + 3 < nout) op[3] = v3;
            }
          }
        }
        if (rmean != nullptr) {
          // the two lane halves hold interleaved runs of four outputs: the wave's
          // 32 outputs of a row as (lane half 0's 16) + (lane half 1's 16)
  #pragma unroll
          for (int rt = 0; rt < NRT; ++rt) {
            const float other = __shfl_xor(rsum[rt], 32, 64);
            if (lh == 0) L.rs[w][32 * rt + li] = rsum[rt] + other;
          }
        }
      }
      if (rmean != nullptr) {
        __syncthreads();  // uniform: row_mean is a kernel argument
        if (t < W_RB) {
          float s = L.rs[0][t];
          for (int v = 1; v < nkt; ++v) s += L.rs[v][t];
          const int row = m0 + t;
          if (row < rend) rmean[c * d.s_mean + row] = s / (float)nout;
        }
      }
      stamp(7, first);
      }  // (no register head)
  };
  int h = hb;
  for (; h + 1 < he; h += 2) tile(std::integral_constant<int, 2>{}, h);  // uniform
  if (h < he) tile(std::integral_constant<int, 1>{}, h);
  if constexpr (STAMPS) {
    if (t == 0 && wgi < 1024) wide_stamps[wgi * W_NST + 8] = __builtin_amdgcn_s_memtime() - t_start;
  }
}

// ---- the input-gradient chain of two 256 x 256 layers (round 6; the CQL
// reproduction critic's backward, d3a_mlp_bwd_chain): per 64-row tile, the
// top layer's pre-activation gradient dz_top (written by the head's backward)
// into the image, then two transposed streams,
//   dz_mid = (dz_top Wa) * [h_mid > 0],   dz_bot = (dz_mid Wb) * [h_bot > 0],
// each as the forward's stream over W^T (TR: W's columns), the mask from the
// kept activations, dz_mid through the image into the second stream and both
// written for the weight-gradient GEMMs.  The autograd backward of the
// trunk's nn.Linear + ReLU pairs (encoders.py:265-275) for its input gradients
// only; persistent over 32-row halves as mlp_x6_wide_kernel.
struct ChainLds {
  __bf16 img[W_RB * 3 * W_LDH];
};

__global__ __launch_bounds__(512) void mlp_bwd_chain_kernel(d3a_mlp_bwd_chain_desc d, int G) {
  __shared__ __attribute__((aligned(16))) ChainLds L;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int li = lane & 31, lh = lane >> 5;
  const int c = (int)blockIdx.x / G, k = (int)blockIdx.x % G;
  const int rlim = (int)d.rows;
  const int nh = (rlim + 31) / 32;
  const int hb = (int)((int64_t)k * nh / G), he = (int)((int64_t)(k + 1) * nh / G);
  if (hb >= he) return;  // uniform
  const float* dzt = d.dz_top + c * d.sdz;
  float* dzm = d.dz_mid + c * d.sdz;
  float* dzb = d.dz_bot + c * d.sdz;
  const float* hm = d.h_mid + c * d.sh;
  const float* hbt = d.h_bot + c * d.sh;
  const WMat Wa = wmat(d.Wa + c * d.sW, W_H * W_H * 4);
  const WMat Wb = wmat(d.Wb + c * d.sW, W_H * W_H * 4);
  const int u0 = 32 * w + li;
  const int wo = (8 * lh * W_H + u0) * 4;  // transposed: this lane's output unit u0, k = 8 lh
  float4 hr[W_HD][2];
#pragma unroll
  for (int s = 0; s < W_HD; ++s) {
    const int st = 16384 * s;
    hr[s][0] = make_float4(wload1(Wa, wo, st), wload1(Wa, wo, st + 1024), wload1(Wa, wo, st + 2048),
                           wload1(Wa, wo, st + 3072));
    hr[s][1] = make_float4(wload1(Wa, wo, st + 4096), wload1(Wa, wo, st + 5120),
                           wload1(Wa, wo, st + 6144), wload1(Wa, wo, st + 7168));
  }
  auto tile = [&](auto nrt, int h) {
    constexpr int NRT = decltype(nrt)::value;
    const int m0 = 32 * h;
    const int rend = min(32 * min(h + 2, he), rlim);
    // ---- dz_top rows -> image (lane: rows 32 rt + li, units 32 w + 8 R + 4 lh + i)
    float4 tv[NRT][4];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const int row = min(m0 + 32 * rt + li, rlim - 1);
        tv[rt][R] = *reinterpret_cast<const float4*>(dzt + (int64_t)row * d.ld + 32 * w + 8 * R + 4 * lh);
      }
    __syncthreads();  // the previous tile's second stream done with the image
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const int rl = 32 * rt + li, u = 32 * w + 8 * R + 4 * lh;
        const bool in = m0 + rl < rend;
        float v[4] = {in ? tv[rt][R].x : 0.f, in ? tv[rt][R].y : 0.f, in ? tv[rt][R].z : 0.f,
                      in ? tv[rt][R].w : 0.f};
        bf16x4 p[3];
        split4(v, p);
#pragma unroll
        for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x4*>(&L.img[(rl * 3 + q) * W_LDH + u]) = p[q];
      }
    __syncthreads();  // image of dz_top complete
    f32x16 o[NRT];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[rt][r] = 0.f;
    stream256<NRT, true>(Wa, wo, Wb, wo, hr, L.img, li, lh, o);
    // the mask rows of h_mid (issued under the products' drain)
    float4 hv[NRT][4];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const int row = min(m0 + 32 * rt + li, rlim - 1);
        hv[rt][R] = *reinterpret_cast<const float4*>(hm + (int64_t)row * d.ldh + 32 * w + 8 * R + 4 * lh);
      }
    __syncthreads();  // every wave done reading the dz_top image
    auto masked = [&](const f32x16& a, int R, const float4& h, float (&z)[4]) {
      z[0] = h.x > 0.f ? a[4 * R + 0] : 0.f;
      z[1] = h.y > 0.f ? a[4 * R + 1] : 0.f;
      z[2] = h.z > 0.f ? a[4 * R + 2] : 0.f;
      z[3] = h.w > 0.f ? a[4 * R + 3] : 0.f;
    };
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const int rl = 32 * rt + li, u = 32 * w + 8 * R + 4 * lh, row = m0 + rl;
        float z[4];
        masked(o[rt], R, hv[rt][R], z);
        if (row < rend)
          *reinterpret_cast<float4*>(dzm + (int64_t)row * d.ld + u) = make_float4(z[0], z[1], z[2], z[3]);
        bf16x4 p[3];
        split4(z, p);
#pragma unroll
        for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x4*>(&L.img[(rl * 3 + q) * W_LDH + u]) = p[q];
      }
    __syncthreads();  // image of dz_mid complete
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[rt][r] = 0.f;
    stream256<NRT, true>(Wb, wo, Wa, wo, hr, L.img, li, lh, o);
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const int row = min(m0 + 32 * rt + li, rlim - 1);
        hv[rt][R] = *reinterpret_cast<const float4*>(hbt + (int64_t)row * d.ldh + 32 * w + 8 * R + 4 * lh);
      }
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int R = 0; R < 4; ++R) {
        const int rl = 32 * rt + li, u = 32 * w + 8 * R + 4 * lh, row = m0 + rl;
        float z[4];
        masked(o[rt], R, hv[rt][R], z);
        if (row < rend)
          *reinterpret_cast<float4*>(dzb + (int64_t)row * d.ld + u) = make_float4(z[0], z[1], z[2], z[3]);
      }
  };
  int h = hb;
  for (; h + 1 < he; h += 2) tile(std::integral_constant<int, 2>{}, h);  // uniform
  if (h < he) tile(std::integral_constant<int, 1>{}, h);
}

}  // namespace
}  // namespace d3a

using namespace d3a;

extern "C" int d3a_mlp_fwd_x6(const d3a_mlp_fwd_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_mlp_fwd_x6: null desc");
  const d3a_mlp_fwd_desc& d = *dp;
  const int nhid = d.n_hidden;
  D3A_CHECK_ARG((nhid == 2 || nhid == 3) && d.H == W_H && d.n_out >= 1 && d.n_out <= 256 &&
                    d.n_in >= 1 && d.n_in <= 64,
                "d3a_mlp_fwd_x6: needs [n_in <= 64, 256, 256 (, 256), n_out <= 256]");
  bool ops_ok = (d.x || d.xg_mode) && d.out;
  for (int l = 0; l <= nhid; ++l) ops_ok = ops_ok && d.W[l] && d.b[l];
  D3A_CHECK_ARG(ops_ok, "d3a_mlp_fwd_x6: null operand");
  D3A_CHECK_ARG(xgen_ok(d), "d3a_mlp_fwd_x6: bad input-row builder (xg_*)");
  D3A_CHECK_ARG(d.hmask == nullptr, "d3a_mlp_fwd_x6: hmask is d3a_q2_fwd_x6 only");
  D3A_CHECK_ARG(d.parts <= 1, "d3a_mlp_fwd_x6: no parts");
  D3A_CHECK_ARG(d.aux_rows == 0 || (d.aux_rows > 0 && d.aux_x && d.aux_out && d.xg_mode == 0 &&
                                    d.row_mean == nullptr && d.aux_rows * d.aux_ldx < (int64_t(1) << 31) &&
                                    d.aux_rows * (int64_t)d.ldout < (int64_t(1) << 31)),
                "d3a_mlp_fwd_x6: aux pass needs aux_x / aux_out, no builder, no row_mean");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0 && d.r0 >= 0 && d.h_from >= 0, "d3a_mlp_fwd_x6: bad sizes");
  auto a16 = [](const void* p, int64_t stride) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && stride % 4 == 0;
  };
  // (the aux pass's parameters sit aux_wdelta floats on: a multiple of 4
  // keeps them 16-byte aligned)
  bool al = d.aux_rows == 0 || d.aux_wdelta % 4 == 0;
  for (int l = 1; l <= nhid; ++l) al = al && a16(d.W[l], d.sW[l]);
  for (int l = 0; l < nhid; ++l) al = al && a16(d.b[l], d.sb[l]);
  if (d.n_out == 1) al = al && a16(d.W[nhid], d.sW[nhid]);
  D3A_CHECK_ARG(al, "d3a_mlp_fwd_x6: hidden W / b and the head's W must be 16-byte aligned");
  bool hk = d.sh % 4 == 0;
  for (int l = 0; l < nhid; ++l) hk = hk && (d.h[l] == nullptr || (reinterpret_cast<uintptr_t>(d.h[l]) & 15) == 0);
  D3A_CHECK_ARG(hk, "d3a_mlp_fwd_x6: kept activations must be 16-byte aligned rows of 256");
  D3A_CHECK_ARG((d.r0 + d.rows) * (int64_t)(d.ldout > W_H ? d.ldout : W_H) < (int64_t(1) << 31) &&
                    (d.r0 + d.rows) * d.ldx < (int64_t(1) << 31),
                "d3a_mlp_fwd_x6: rows x row stride exceeds 2^31");
  D3A_CHECK_ARG(d.ldout >= d.n_out, "d3a_mlp_fwd_x6: ldout < n_out");
  D3A_CHECK_ARG(d.row_mean == nullptr || (d.s_mean >= d.r0 + d.rows &&
                                          d.s_mean * (int64_t)d.C < (int64_t(1) << 31)),
                "d3a_mlp_fwd_x6: row_mean member stride must cover the rows");
  if (d.rows == 0 && d.aux_rows == 0) return 0;
  // persistent: one workgroup per CU, the CUs shared between the members and
  // (aux pass) between the passes in proportion to their rows
  static const int n_cu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    return n;
  }();
  const int64_t halves = (d.rows + 31) / 32, ahalves = (d.aux_rows + 31) / 32;
  int64_t ga = 0;
  if (ahalves > 0)
    ga = std::min<int64_t>((ahalves + 1) / 2,
                           std::max<int64_t>(1, n_cu * ahalves / ((halves + ahalves) * d.C)));
  const int64_t gm = halves > 0 ? std::min<int64_t>(std::max<int64_t>(1, (n_cu - d.C * ga) / d.C),
                                                    (halves + 1) / 2)
                                : 1;
  const dim3 grid((unsigned)(d.C * (gm + ga)));
  const int Gm = (int)gm, Ga = (int)std::max<int64_t>(ga, 1);
  const hipStream_t st = (hipStream_t)stream;
  static const bool stamps = [] {
    const char* e = getenv("D3A_WIDE_STAMPS");
    return e && atoi(e) != 0;
  }();
  bool keep = false;
  for (int l = 0; l < nhid; ++l) keep = keep || d.h[l] != nullptr;
  const bool x32 = d.n_in <= 32;
  // pre-split stream images (n_in <= 32; the three-layer Q-head form or the
  // two-layer wide head: wp[0] = W[1]'s image, wp[1] = W[2]'s)
  const bool pw = d.wp[0] != nullptr;
  if (pw) {
    D3A_CHECK_ARG(x32 && d.wp[1] && ((nhid == 3 && d.n_out == 1) || (nhid == 2 && d.n_out > 1)),
                  "d3a_mlp_fwd_x6: stream images need n_in <= 32 and [.., 256, 256, 256, 1] or "
                  "[.., 256, 256, n_out > 1], wp[0] and wp[1]");
    D3A_CHECK_ARG(d.aux_rows == 0 || (d.aux_wp[0] && d.aux_wp[1]), "d3a_mlp_fwd_x6: aux pass needs aux_wp");
    bool al = true;
    for (int i = 0; i < 2; ++i)
      al = al && (reinterpret_cast<uintptr_t>(d.wp[i]) & 15) == 0 &&
           (reinterpret_cast<uintptr_t>(d.aux_wp[i]) & 15) == 0;
    D3A_CHECK_ARG(al, "d3a_mlp_fwd_x6: stream images must be 16-byte aligned");
  }
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(512), 0, st, d, Gm, Ga); };
  if (nhid == 3) {
    // the CQL reproduction critic: Q head (register dot) or a wide head
    if (d.n_out == 1) {
      if (pw && stamps && keep) go(mlp_x6_wide_kernel<32, true, true, 3, true, true>);
      else if (pw && keep) go(mlp_x6_wide_kernel<32, true, false, 3, true, true>);
      else if (pw) go(mlp_x6_wide_kernel<32, false, false, 3, true, true>);
      else if (stamps && x32 && keep) go(mlp_x6_wide_kernel<32, true, true, 3, true>);
      else if (x32 && keep) go(mlp_x6_wide_kernel<32, true, false, 3, true>);
      else if (x32) go(mlp_x6_wide_kernel<32, false, false, 3, true>);
      else if (keep) go(mlp_x6_wide_kernel<64, true, false, 3, true>);
      else go(mlp_x6_wide_kernel<64, false, false, 3, true>);
    } else {
      if (x32 && keep) go(mlp_x6_wide_kernel<32, true, false, 3>);
      else if (x32) go(mlp_x6_wide_kernel<32, false, false, 3>);
      else if (keep) go(mlp_x6_wide_kernel<64, true, false, 3>);
      else go(mlp_x6_wide_kernel<64, false, false, 3>);
    }
  } else if (pw) {
    if (keep) go(mlp_x6_wide_kernel<32, true, false, 2, false, true>);
    else go(mlp_x6_wide_kernel<32, false, false, 2, false, true>);
  } else if (stamps && x32 && !keep) {
    go(mlp_x6_wide_kernel<32, false, true>);
  } else if (x32 && keep) {
    go(mlp_x6_wide_kernel<32, true>);
  } else if (x32) {
    go(mlp_x6_wide_kernel<32, false>);
  } else if (keep) {
    go(mlp_x6_wide_kernel<64, true>);
  } else {
    go(mlp_x6_wide_kernel<64, false>);
  }
  D3A_LAUNCH_CHECK("d3a_mlp_fwd_x6");
  return 0;
}

// diagnostic (synchronous): every wave's stamps of the last three-layer
// D3A_WIDE_STAMPS=1 launch, [workgroup < 512][wave][8]
extern "C" int d3a_wide_wave_stamps(unsigned long long* dst, int n) {
  D3A_CHECK_ARG(dst && n >= 0 && n <= 512 * 64, "d3a_wide_wave_stamps: bad arguments");
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(d3a::wide_wstamps), (size_t)n * 8, 0,
                          hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("d3a_wide_wave_stamps: copy failed");
    return -1;
  }
  return 0;
}

// diagnostic (synchronous, not for graphs): the stamps of the last
// D3A_WIDE_STAMPS=1 launch, [workgroup][9]
extern "C" int d3a_wide_stamps(unsigned long long* dst, int n) {
  D3A_CHECK_ARG(dst && n >= 0 && n <= 1024 * W_NST, "d3a_wide_stamps: bad arguments");
  if (hipMemcpyFromSymbol(dst, HIP_SYMBOL(d3a::wide_stamps), (size_t)n * 8, 0,
                          hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("d3a_wide_stamps: copy failed");
    return -1;
  }
  return 0;
}

extern "C" int d3a_mlp_bwd_chain(const d3a_mlp_bwd_chain_desc* dp, void* stream) {
  D3A_CHECK_ARG(dp, "d3a_mlp_bwd_chain: null desc");
  const d3a_mlp_bwd_chain_desc& d = *dp;
  D3A_CHECK_ARG(d.dz_top && d.dz_mid && d.dz_bot && d.h_mid && d.h_bot && d.Wa && d.Wb,
                "d3a_mlp_bwd_chain: null operand");
  D3A_CHECK_ARG(d.C >= 1 && d.rows >= 0 && d.ld >= 256 && d.ldh >= 256 && d.ld % 4 == 0 &&
                    d.ldh % 4 == 0 && d.sdz % 4 == 0 && d.sh % 4 == 0 && d.sW % 4 == 0,
                "d3a_mlp_bwd_chain: bad sizes / strides (rows of >= 256, multiples of 4)");
  D3A_CHECK_ARG(d.dz_mid != d.dz_top, "d3a_mlp_bwd_chain: dz_mid must not alias dz_top");
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  D3A_CHECK_ARG(al(d.dz_top) && al(d.dz_mid) && al(d.dz_bot) && al(d.h_mid) && al(d.h_bot),
                "d3a_mlp_bwd_chain: rows must be 16-byte aligned");
  D3A_CHECK_ARG(d.rows * d.ld < (int64_t(1) << 31) && d.rows * d.ldh < (int64_t(1) << 31),
                "d3a_mlp_bwd_chain: rows x row stride exceeds 2^31");
  if (d.rows == 0) return 0;
  static const int n_cu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    return n;
  }();
  const int64_t halves = (d.rows + 31) / 32;
  const int64_t g = std::min<int64_t>(std::max(1, n_cu / d.C), (halves + 1) / 2);
  hipLaunchKernelGGL(mlp_bwd_chain_kernel, dim3((unsigned)(d.C * g)), dim3(512), 0, (hipStream_t)stream,
                     d, (int)g);
  D3A_LAUNCH_CHECK("d3a_mlp_bwd_chain");
  return 0;
}
