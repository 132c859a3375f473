// cos of the IQN cosine prior's arguments, x = fl(fl(pi (e + 1)) tau) with
// tau in [0, 1) and e < 64 (|x| < 202; compute_iqn_feature, iqn_q_function.py:
// 37-41).  ocml's cosf carries a Payne-Hanek reduction for every argument
// (~95 VALU per call, 4 calls per thread and 32-row tile in the IQN head
// kernels); here a Cody-Waite reduction by pi / 2 -- j = rint(x 2 / pi), r = x -
// j P1 - j P2 - j P3 with P1 + P2 + P3 = pi / 2, the first step exact for
// |x| <= 8192 (j P1 and x on the 2^-23 grid, |r| < 1) -- and the Cephes
// single-precision sin / cos polynomials on |r| <= pi / 4 (~20 VALU; max
// error 1 ulp of the result over the prior's arguments:
// tests/test_iqn_cos.py, oracle/iqn_cos_check.cpp).  Past |x| = 8192 the
// reduction's first step is no longer exact and the error grows with |x| (tau
// far outside [0, 1), outside the reference's sampling); NaN and inf give NaN.
// No cosf fallback branch: its Payne-Hanek code costs the callers ~40
// registers even untaken.  Shared by d3a_iqn_prior, d3a_iqn_embed_head and the recomputing
// backward so that every kernel builds the same prior bits.
#pragma once
#include <cmath>

#if defined(__HIPCC__)
#define D3A_IQN_HD __host__ __device__
#else
#define D3A_IQN_HD
#endif

D3A_IQN_HD inline float iqn_cos(float x) {
#ifdef __clang__
#pragma clang fp contract(off)  // the operations as written (hipcc contracts by default)
#endif
  const float ax = fabsf(x);
  const float j = rintf(ax * 0x1.45f306p-1f);   // 2 / pi
  // r = x - j pi / 2 as rh + rl: x - j P1 exact, + j |P2| by TwoSum with the
  // product's error, + j |P3| (pi / 2 = P1 + P2 + P3, P2 and P3 negative)
  const float r1 = fmaf(-j, 0x1.921fb6p+0f, ax);
  const float a = j * 0x1.777a5cp-25f, ae = fmaf(j, 0x1.777a5cp-25f, -a);
  const float rh = r1 + a, bb = rh - r1;
  const float rl = ((r1 - (rh - bb)) + (a - bb)) + fmaf(j, 0x1.ee59dap-50f, ae);
  const float z = rh * rh;
  // sin(rh + rl) = s(rh) + rl (1 - z / 2), cos(rh + rl) = c(rh) - rl rh
  const float hz = 0.5f * z, w = 1.0f - hz;
  const float ps = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  const float s = rh + fmaf(rh * z, ps, rl * w);
  // 1 - z / 2 compensated (w's rounding and z's), then the z^2 terms
  const float ze = fmaf(rh, rh, -z);
  const float pc = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z,
                        4.166664568298827e-2f);
  const float c = w + fmaf(z * z, pc, (((1.0f - w) - hz) - 0.5f * ze) - rl * rh);
  const int q = (int)j;
  const float v = (q & 1) ? s : c;
  return ((q + 1) & 2) ? -v : v;
}
