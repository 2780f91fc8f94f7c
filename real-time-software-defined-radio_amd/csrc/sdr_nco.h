// The NCO of fmPll (model/fmPll.py:33-37) as a function of the PLL's stored phase rows, shared
// by the PLL kernels (pll.hip: NCO rows, when an output asks for them) and the receiver's mixer
// stage (rx.hip: the mixers form cos / sin of the PLL phase where they stage their inputs, so a
// block's NCO never round-trips through HBM -- VERDICT r04 item 2).
//
//   th_k   = 2 pi (freq / Fs) (trigOffset + k + 1) + phaseEst_k        (fmPll.py:33)
//   nco[k+1] = cos(th_k scale + adj),  ncoQ[k+1] = sin(th_k scale + adj)  (:36-37)
//   nco[0] = the previous call's last value (the carried state)
//
// Per-block calls store phaseEst_k itself.  Long calls (spans) store each pseudo-block's own
// solve: the recurrence's phase is that + 2 pi x the chain's whole turns for the block + the
// loop's linear response (A^(kk+1) d)_phase to the start error d the chain accepted it with (kk:
// the step within the pseudo-block).  The response row of A^(kk+1) is a table built once per
// loop (PllResp), so every consumer forms the same double.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdr_launch.h"

namespace sdrnco {

// 2*pi split into three parts (Cody-Waite), so n*P1 and n*P2 are exact for |n| < 2^26.
constexpr double kP1 = 6.2831854820251465;       // float32(2 pi), 24 significant bits
constexpr double kP2 = -1.748455600074497e-07;    // double(2 pi - kP1)
constexpr double kP3 = -1.0687562935444062e-23;   // remainder
constexpr double kInv2Pi = 0.15915494309189535;
constexpr double kPi = 3.14159265358979323846;
constexpr double k2Pi = 6.28318530717958647692;

// r = a - 2*pi*n, n = rint(a / 2pi), |r| <= pi (up to one ulp at the boundary).
__device__ inline double reduce_2pi(double a) {
  const double n = rint(a * kInv2Pi);
  double r = fma(-n, kP1, a);
  r = fma(-n, kP2, r);
  r = fma(-n, kP3, r);
  return r;
}

// sin and cos of a reduced angle |a| <= pi (+ an ulp), for the NCO outputs (f32: 6e-8 is their
// rounding): quadrant n = rint(a 2/pi) (a two-part pi/2: exact to ~1e-32 for |n| <= 2), then
// Taylor polynomials on |y| <= pi/4 to y^13 / y^14 (truncation < 3e-14).  ~35 VALU against
// the library sincos's general-argument path.
// OPAQUE: each coefficient is made an SGPR at its use (a volatile asm): in kernels that call
// this once per call (end states) the compiler otherwise keeps all 14 in VGPRs for the whole
// kernel, which spilled the long-call fix kernel
template <bool OPAQUE = false>
__device__ __forceinline__ void sincos_red(double a, double* sv, double* cv) {
  auto K = [](double c) {
    if constexpr (OPAQUE) asm volatile("" : "+s"(c));
    return c;
  };
  constexpr double kPio2Hi = 1.5707963267948966, kPio2Lo = 6.123233995736766e-17, k2oPi = 0.6366197723675814;
  const double n = rint(a * k2oPi);
  double y = fma(-n, kPio2Hi, a);
  y = fma(-n, kPio2Lo, y);
  const double z = y * y;
  double ps = K(1.0 / 6227020800.0);                        // 1/13!
  ps = fma(ps, z, K(-1.0 / 39916800.0));
  ps = fma(ps, z, K(1.0 / 362880.0));
  ps = fma(ps, z, K(-1.0 / 5040.0));
  ps = fma(ps, z, K(1.0 / 120.0));
  ps = fma(ps, z, K(-1.0 / 6.0));
  const double sn = fma(ps * z, y, y);
  double pc = K(1.0 / 87178291200.0);                       // 1/14!
  pc = fma(pc, z, K(-1.0 / 479001600.0));
  pc = fma(pc, z, K(1.0 / 3628800.0));
  pc = fma(pc, z, K(-1.0 / 40320.0));
  pc = fma(pc, z, K(1.0 / 720.0));
  pc = fma(pc, z, K(-1.0 / 24.0));
  pc = fma(pc, z, K(0.5));
  const double cs = fma(-pc, z, 1.0);
  const int q = (int)n & 3;
  const double s0 = (q & 1) ? cs : sn, c0 = (q & 1) ? sn : cs;
  *sv = (q == 2 || q == 3) ? -s0 : s0;
  *cv = (q == 1 || q == 2) ? -c0 : c0;
}

// The PLL's view of its input (model/fmPll.py:24-27): atan2(-x sin th, x cos th) depends on x
// only through its sign -- and, for the literal general step, on the signs of the products when
// x is a zero, or on a NaN.  A span's loop inputs therefore travel as one byte per sample
// (r06): +1 / -1 for x > 0 / x < 0, 0 for +0, 2 for -0, 3 for NaN; decoded to the float with the
// same atan2 (+-1, +-0, NaN).  The parallel solve reads +1 / -1 and treats the rest as its
// general-form case, as it does the float row's zeros and NaNs.
__device__ __forceinline__ int8_t pll_code(float v) {
  return (int8_t)(v > 0.f ? 1 : v < 0.f ? -1 : v == 0.f ? (__builtin_signbit(v) ? 2 : 0) : 3);
}
__device__ __forceinline__ float pll_decode(int8_t c) {
  return c == 1 ? 1.f : c == -1 ? -1.f : c == 0 ? 0.f : c == 2 ? -0.f : __builtin_nanf("");
}

}  // namespace sdrnco

// ---- long calls: pseudo-block bookkeeping (device scratch PllJobs::work) --------------
// Per recurrence r = job * nstreams + stream: a header (the chain's position and the exact
// state at it), then one LongBlk per pseudo-block: its start guess g (warm-up), its chained
// start x (when re-solved), the end state e of its latest solve, the 2 pi shift the chain
// found for it, and its status.  States are in fmPll's 6-double order.
// u: the start (phaseEst, integrator) the current solution (theta row, e) was solved from.
// shift: the chain's whole turns for the block's phases; d: the start error (dphaseEst, dV)
// the chain accepted the block with (its stored phases + the loop's linear response to d are
// the recurrence's); margin: the solve's smallest distance of a step's fract(t_k) from a wrap,
// in turns (-1: none, the sequential kernels' solves).
struct LongBlk {
  double g[6]; double x[6]; double e[6]; double u[2]; double shift; double d[2]; double margin; int status; int solver;
};
struct LongHdr { double sp, si; int pos; int pad; double pad2; };
static_assert(sizeof(LongBlk) == 200 && sizeof(LongHdr) == 32, "long-call scratch layout");
// the first LongBlk of recurrence r in a long call's scratch
__host__ __device__ inline const LongBlk* long_blk0(const void* work, int njobs, int nstreams, int nb, int r) {
  return reinterpret_cast<const LongBlk*>(static_cast<const char*>(work) + (int64_t)njobs * nstreams * sizeof(LongHdr)) +
         (int64_t)r * nb;
}

// ---- compact phase rows (r06: the pilot loop of a span, PllJob::th32) ----------------------
// A long call's phase row in 4.5 B a step instead of 8: per line c of 32 rows (rows 32 c ..
// 32 c + 31 of the stream's row; pseudo-blocks start on a line, pb = 0 mod 32) a line {a, s}
// (f64) and per row an f32 residual r_k, with
//   stored_k = fma(s, k - 32 c, a) + r_k.
// The solve sets a line's (a, s) from the trajectory of its previous pass over the line's
// first row (its start and its slope per step), so r_k is the loop's deviation from a straight
// line over 32 steps -- <= 0.3 rad at acquisition, ~0.1 rad of detector jitter when locked (the
// pilot loop, Kp = 0.027) -- and its f32 rounding <= 2e-8 rad (tools/th32_err.py, against the
// NCO's 1e-7 check).  Inside the row's own allocation (th_stride >= n + 1 doubles): residuals at
// bytes [0, 4 n), the lines from byte th32_lines_at(n) (<= 4.5 n + 32 <= 8 n: n > 16 385 for
// every long call), the trigOffset slot th[n] (byte 8 n) unchanged.
constexpr int TH32_LINE = 32;
struct Th32Line { double a, s; };
__host__ __device__ inline int64_t th32_lines_at(int64_t n) { return (4 * n + 15) / 16 * 16; }
__device__ __forceinline__ float* th32_res(double* row) { return reinterpret_cast<float*>(row); }
__device__ __forceinline__ const float* th32_res(const double* row) { return reinterpret_cast<const float*>(row); }
__device__ __forceinline__ Th32Line* th32_lines(double* row, int64_t n) {
  return reinterpret_cast<Th32Line*>(reinterpret_cast<char*>(row) + th32_lines_at(n));
}
__device__ __forceinline__ const Th32Line* th32_lines(const double* row, int64_t n) {
  return reinterpret_cast<const Th32Line*>(reinterpret_cast<const char*>(row) + th32_lines_at(n));
}
// the residual of a stored phase against its line (the writers' one formula)
__device__ __forceinline__ float th32_residual(const Th32Line& L, int o, double stored) {
#pragma clang fp contract(off)
  return (float)(stored - fma(L.s, (double)o, L.a));
}
// stored_k of a compact row of n steps
__device__ __forceinline__ double th32_stored(const double* row, int64_t n, int64_t k) {
#pragma clang fp contract(off)
  const Th32Line L = th32_lines(row, n)[k >> 5];
  return fma(L.s, (double)(int)(k & 31), L.a) + (double)th32_res(row)[k];
}

// Where one PLL job's NCO comes from, for every stream of a receiver block.
struct NcoSrc {
  const double* theta;     // phase rows (th_stride apart); theta[n] = the call's trigOffset
  int64_t th_stride;
  const float* nco_i;      // NCO rows (out_stride apart): only [0], the carried value, is read
  const float* nco_q;      //   (nullable: no quadrature output)
  int64_t out_stride;
  double w, scale, adj;    // 2 pi freq / Fs, ncoScale, phaseAdjust
  int64_t n;               // steps of the call
  // long calls (blk != null): stream s's pseudo-blocks at blk + s * blk_stride, pb steps each;
  // resp[2 (kk + 1) + {0, 1}] = row 0 of A^(kk+1), kk < pb
  const LongBlk* blk;
  int64_t blk_stride, pb;
  int nb;                  // pseudo-blocks of the call
  const double* resp;
  const float* resp32;     // the same table in f32 (the matrix-core mixers' response: an angle <= 0.15 rad)
  int th32;                // the phase rows are compact (PllJob::th32): the matrix-core mixer's TH32 form only
};

// The recurrence's phaseEst for step kk of a long call's pseudo-block B whose solve stored
// `stored` there (the chain's turns, then the linear response to its accepted start error).
__device__ __forceinline__ double nco_phase_in(const LongBlk* B, int64_t kk, const double* resp, double stored) {
#pragma clang fp contract(off)
  const double sh = B->shift, d0 = B->d[0], d1 = B->d[1];
  double p = fma(sh, sdrnco::kP1, fma(sh, sdrnco::kP2, stored));
  if (d0 != 0.0 || d1 != 0.0) {
    const double* rr = resp + 2 * (kk + 1);
    p = p + (rr[0] * d0 + rr[1] * d1);
  }
  return p;
}

// phaseEst_j (j >= 0) of stream s.
__device__ __forceinline__ double nco_phase(const NcoSrc& N, int s, int64_t j, double stored) {
  if (N.blk == nullptr) return stored;
  int64_t b = (int64_t)((double)j / (double)N.pb);
  if (b * N.pb > j) --b;
  else if ((b + 1) * N.pb <= j) ++b;
  return nco_phase_in(N.blk + (int64_t)s * N.blk_stride + b, j - b * N.pb, N.resp, stored);
}

// ncoOut[k] / ncoOutQ[k] (k >= 1), in f64 (the caller rounds), from p = phaseEst_{k-1} and the
// call's trigOffset off; every NCO row of the library is formed here.
template <bool OPAQUE = false>
__device__ __forceinline__ void nco_value(double w, double scale, double adj, int64_t k, double p, double off,
                                          double* cv, double* sv) {
#pragma clang fp contract(off)
  const double th = w * ((off + (double)(k - 1)) + 1.0) + p;
  const double a = th * scale + adj;
  sdrnco::sincos_red<OPAQUE>(sdrnco::reduce_2pi(a), sv, cv);
}

// ---- the mixers' NCO (rx.hip): f32 cos / sin of the f64 angle ------------------------------
// The mixers only need the NCO to the f32 rounding of their product: the angle a = th scale +
// adj is formed and reduced in f64 exactly as above (|y| <= pi/4 after the quadrant), then
// y is rounded to f32 (3e-8) and cos / sin come from f32 polynomials on two samples at once
// (packed FMAs; Taylor to y^9 / y^10: truncation < 1e-9), ~1 ulp of the f32 result -- the
// error of the NCO row a mixer would otherwise read, at a third of the f64 polynomial's work.
// (The NCO rows, when an output asks for them, stay the f64 ones above.)
// Per tile: the pseudo-block records its steps fall in (a tile spans < pb steps: at most
// two), read once.
struct NcoTile {
  const double* th;        // the stream's phase row
  double off;              // the call's trigOffset
  int64_t kb, bound;       // steps j in [kb, bound): the first block, [bound, ...): the second
  double sh[2], d0[2], d1[2];
};

__device__ __forceinline__ NcoTile nco_tile(const NcoSrc& N, int s, int64_t j0) {
  NcoTile T;
  T.th = N.theta + (int64_t)s * N.th_stride;
  T.off = T.th[N.n];
  T.kb = 0;
  T.bound = INT64_MAX;
  for (int h = 0; h < 2; ++h) T.sh[h] = T.d0[h] = T.d1[h] = 0.0;
  if (N.blk != nullptr) {
    const int64_t b = max(j0, (int64_t)0) / N.pb;
    T.kb = b * N.pb;
    T.bound = T.kb + N.pb;
    const LongBlk* B = N.blk + (int64_t)s * N.blk_stride + b;
    T.sh[0] = B->shift; T.d0[0] = B->d[0]; T.d1[0] = B->d[1];
    if (b + 1 < N.nb) { T.sh[1] = B[1].shift; T.d0[1] = B[1].d[0]; T.d1[1] = B[1].d[1]; }
  }
  return T;
}

// phaseEst_j from its stored value (nco_phase_in's arithmetic)
__device__ __forceinline__ double nco_tile_p(const NcoSrc& N, const NcoTile& T, int64_t j, double stored) {
#pragma clang fp contract(off)
  const bool h = j >= T.bound;
  const double sh = h ? T.sh[1] : T.sh[0], d0 = h ? T.d0[1] : T.d0[0], d1 = h ? T.d1[1] : T.d1[0];
  double p = fma(sh, sdrnco::kP1, fma(sh, sdrnco::kP2, stored));
  if (d0 != 0.0 || d1 != 0.0) {
    const int64_t kk = j - (h ? T.bound : T.kb);
    const double* rr = N.resp + 2 * (kk + 1);
    p = p + (rr[0] * d0 + rr[1] * d1);
  }
  return p;
}

typedef float ncof2 __attribute__((ext_vector_type(2)));
// The reduced angle of output k (>= 1) from p = phaseEst_{k-1}: a = (w scale) (trigOffset + k)
// + (p scale + adj) (scale a power of two in every fmPll use: the same product as the
// reference's (th) scale, one rounding fewer), reduced by a 3-part pi/2 (exact multiples for
// |n| < 2^29: ~40 min of a 240 kS/s stream before its last bits blur, as the reference's own
// f64 angle does) to |y| <= pi/4 in f32, and its quadrant.
__device__ __forceinline__ void nco_angle_at(double ws, double scale, double adj, double offk, double p, float* y,
                                             int* q) {
#pragma clang fp contract(off)
  constexpr double k2oPi = 0.6366197723675814;
  constexpr double Q1 = 1.5707963705062866, Q2 = -4.3711390001862426e-08, Q3 = -2.6718907338610155e-24;
  const double a = fma(ws, offk, fma(p, scale, adj));       // ws = w scale, offk = trigOffset + k
  const double n = rint(a * k2oPi);
  double r = fma(-n, Q1, a);
  r = fma(-n, Q2, r);
  r = fma(-n, Q3, r);
  *y = (float)r;
  *q = (int)(int64_t)n & 3;
}
__device__ __forceinline__ void nco_angle(const NcoSrc& N, double off, int64_t k, double p, float* y, int* q) {
  nco_angle_at(N.w * N.scale, N.scale, N.adj, off + (double)(int)k, p, y, q);   // trigOffset + (k - 1) + 1
}
// cos / sin of two reduced angles (packed f32 Taylor polynomials to y^9 / y^10, then the quadrant)
__device__ __forceinline__ void nco_poly2(const float (&y)[2], const int (&q)[2], float* c, float* sn) {
  auto K = [](float v) { return ncof2{v, v}; };
  const ncof2 yf = ncof2{y[0], y[1]};
  const ncof2 z = yf * yf;
  ncof2 ps = __builtin_elementwise_fma(K(2.7557319e-06f), z, K(-1.9841270e-04f));
  ps = __builtin_elementwise_fma(ps, z, K(8.3333333e-03f));
  ps = __builtin_elementwise_fma(ps, z, K(-1.6666667e-01f));
  const ncof2 sv = __builtin_elementwise_fma(ps * z, yf, yf);
  ncof2 pc = __builtin_elementwise_fma(K(-2.7557319e-07f), z, K(2.4801587e-05f));
  pc = __builtin_elementwise_fma(pc, z, K(-1.3888889e-03f));
  pc = __builtin_elementwise_fma(pc, z, K(4.1666668e-02f));
  pc = __builtin_elementwise_fma(pc, z, K(-0.5f));
  const ncof2 cv = __builtin_elementwise_fma(pc, z, K(1.0f));
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int qq = q[u];
    const float s0 = (qq & 1) ? cv[u] : sv[u], c0 = (qq & 1) ? sv[u] : cv[u];
    sn[u] = (qq == 2 || qq == 3) ? -s0 : s0;
    c[u] = (qq == 1 || qq == 2) ? -c0 : c0;
  }
}
// cos / sin (f32) of the NCO of outputs k and k + 1 (k >= 1) from p = phaseEst_{k-1}, _k
__device__ __forceinline__ void nco_f32x2(const NcoSrc& N, double off, int64_t k, double p0, double p1, ncof2* c,
                                          ncof2* sn) {
  float y[2], cc[2], ss[2];
  int q[2];
  nco_angle(N, off, k, p0, &y[0], &q[0]);
  nco_angle(N, off, k + 1, p1, &y[1], &q[1]);
  nco_poly2(y, q, cc, ss);
  *c = ncof2{cc[0], cc[1]};
  *sn = ncof2{ss[0], ss[1]};
}

// cos / sin (f32) of the NCO of four consecutive outputs i .. i+3 (i >= 2 even: the phase pairs
// are 16-B loads), every load issued before the first use and the four angle chains
// independent.  The angle is formed as a = (w scale) (trigOffset + k) + (p scale + adj) (scale a
// power of two in every fmPll use: the same product as the reference's (th) scale, one rounding
// fewer) and reduced by a 3-part pi/2 (exact multiples for |n| < 2^29: ~40 min of a 240 kS/s
// stream before its last bits blur, as the reference's own f64 angle does).
__device__ __forceinline__ void nco_f32x4(const NcoSrc& N, const NcoTile& T, int64_t i, float (&c)[4], float (&sn)[4]) {
#pragma clang fp contract(off)
  typedef double d2n __attribute__((ext_vector_type(2)));
  double st[4];                                            // phaseEst_{i-1} .. phaseEst_{i+2}
  if (N.th32) {                                            // (compact rows, sdr_nco.h: kept RDS LPF rows)
#pragma unroll
    for (int e = 0; e < 4; ++e) st[e] = th32_stored(T.th, N.n, i - 1 + e);
  } else {
    const double* th = T.th + i - 2;
    const d2n t01 = *reinterpret_cast<const d2n*>(th), t23 = *reinterpret_cast<const d2n*>(th + 2),
              t45 = *reinterpret_cast<const d2n*>(th + 4);
    st[0] = t01.y; st[1] = t23.x; st[2] = t23.y; st[3] = t45.x;
  }
  double p[4];
  bool lin = false;
  double d0[4], d1[4];
  int64_t kk[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t j = i - 1 + e;
    const bool h = j >= T.bound;
    const double sh = h ? T.sh[1] : T.sh[0];
    d0[e] = h ? T.d0[1] : T.d0[0];
    d1[e] = h ? T.d1[1] : T.d1[0];
    kk[e] = j - (h ? T.bound : T.kb);
    lin = lin || d0[e] != 0.0 || d1[e] != 0.0;
    p[e] = fma(sh, sdrnco::kP1, fma(sh, sdrnco::kP2, st[e]));
  }
  if (lin) {
    d2n rr[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) rr[e] = *reinterpret_cast<const d2n*>(N.resp + 2 * (kk[e] + 1));
#pragma unroll
    for (int e = 0; e < 4; ++e) p[e] = p[e] + (rr[e].x * d0[e] + rr[e].y * d1[e]);
  }
  float y[4];
  int q[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) nco_angle(N, T.off, i + e, p[e], &y[e], &q[e]);
  nco_poly2({y[0], y[1]}, {q[0], q[1]}, &c[0], &sn[0]);
  nco_poly2({y[2], y[3]}, {q[2], q[3]}, &c[2], &sn[2]);
}

// The matrix-core mixers' loads of inputs i .. i+3 (i >= 1 odd), issued ahead of their use
// (software-pipelined, rx.hip): the phase pairs and, when the tile's pseudo-blocks carry a
// linear response (lin: uniform), the response rows (f32, r06).
struct Nco4Ld {
  typedef double d2n __attribute__((ext_vector_type(2)));
  typedef float f2n __attribute__((ext_vector_type(2)));
  d2n t01, t23;            // the four stored phases (TH32: t01 = the line {a, s}, t23 unused)
  float4 r;                // TH32: the four residuals
  f2n rr[4];
};
__device__ __forceinline__ bool nco_tile_lin(const NcoTile& T) {
  return T.d0[0] != 0.0 || T.d1[0] != 0.0 || T.d0[1] != 0.0 || T.d1[1] != 0.0;
}
// (i odd: the four phases phaseEst_{i-1} .. phaseEst_{i+2} are two aligned pairs, t01 and t23;
// TH32: rows i-1 .. i+2 are one 16-B run of residuals in one line -- i - 1 = 0 mod 4 -- and the
// line is 16 B)
template <bool TH32 = false>
__device__ __forceinline__ void nco4_load(const NcoSrc& N, const NcoTile& T, int64_t i, bool lin, Nco4Ld* L) {
  typedef Nco4Ld::d2n d2n;
  typedef Nco4Ld::f2n f2n;
  if constexpr (TH32) {
    // (clamped into the row: a chunk wholly past its end -- a window's tail, its inputs 0 --
    // must still form a finite angle, and past the residuals lie the lines)
    const int64_t j0 = min(i - 1, N.n - 4);
    L->r = *reinterpret_cast<const float4*>(th32_res(T.th) + j0);
    L->t01 = *reinterpret_cast<const d2n*>(th32_lines(T.th, N.n) + (j0 >> 5));
  } else {
    const double* th = T.th + i - 1;
    L->t01 = *reinterpret_cast<const d2n*>(th);
    L->t23 = *reinterpret_cast<const d2n*>(th + 2);
  }
  if (lin) {
    // the four steps' rows are consecutive from the chunk's first step's block base: a chunk
    // that crosses into the next pseudo-block reads that block's first rows from the table's
    // four repeated rows (sdr_pll_resp_table) -- one address, four immediate offsets
    const int64_t j0 = i - 1;
    const int64_t k0 = j0 - (j0 >= T.bound ? T.bound : T.kb);
    const int64_t kk = k0 > 0 ? k0 : (int64_t)0;                  // (>= 0: clamped rows)
    const f2n* rr = reinterpret_cast<const f2n*>(N.resp32) + (kk + 1);
#pragma unroll
    for (int e = 0; e < 4; ++e) L->rr[e] = rr[e];
  }
}

// The matrix-core mixers' angle, per window (rx.hip rx_stereomm_kernel / rx_cresmm_kernel):
// a_k = ws (off + k) + (phaseEst_{k-1}) scale + adj with phaseEst = stored + 2 pi shift (+ the
// linear response) is formed as
//   a_k = base_h + ws (k - kw) + stored scale (+ scale (rr . d)),
//   base_h = [ws (off + kw) mod 2 pi] + adj + 2 pi frac(scale shift_h)
// -- the large product ws (off + kw) reduced ONCE per window in double-double (its rounding
// error kept, then a 3-part 2 pi), the chain's whole turns folded in exactly (scale shift is a
// multiple of 1/2 for every fmPll scale), so each sample needs one fma for its phase and a
// 2-part pi/2 reduction of |a| < ~1e4: 8 f64 operations instead of 14, and no larger angle
// error than the reference's own f64 th (it is smaller: the reference rounds ws (off + k) at
// full magnitude).  The f32 polynomials are nco_poly2's.
struct NcoWin {
  double base[2];          // per pseudo-block half h (as NcoTile)
  float sd0[2], sd1[2];    // scale d, per half (the linear response, formed in f32: r06)
  double ws, scale;
  int64_t kw;              // the reference sample
};
__device__ __forceinline__ NcoWin nco_win(const NcoSrc& N, const NcoTile& T, int64_t kw) {
#pragma clang fp contract(off)
  NcoWin W;
  W.ws = N.w * N.scale;
  W.scale = N.scale;
  W.kw = kw;
  const double X = T.off + (double)kw;               // integer-valued: exact
  const double hi = W.ws * X, lo = fma(W.ws, X, -hi);
  const double n = rint(hi * sdrnco::kInv2Pi);
  double r = fma(-n, sdrnco::kP1, hi);
  r = fma(-n, sdrnco::kP2, r);
  r = fma(-n, sdrnco::kP3, r);
  r = (r + lo) + N.adj;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const double f = N.scale * T.sh[h];
    W.base[h] = r + (f - rint(f)) * sdrnco::k2Pi;
    W.sd0[h] = (float)(N.scale * T.d0[h]);
    W.sd1[h] = (float)(N.scale * T.d1[h]);
  }
  return W;
}
// cos / sin (f32) of outputs i .. i+3 (i odd: L from nco4_load) from the window's angle base
template <bool TH32 = false>
__device__ __forceinline__ void nco4_eval_w(const NcoTile& T, const NcoWin& W, int64_t i, const Nco4Ld& L, bool lin,
                                            float (&c)[4], float (&sn)[4]) {
#pragma clang fp contract(off)
  constexpr double k2oPi = 0.6366197723675814;
  constexpr double Q1 = 1.5707963705062866, Q2 = -4.3711390001862426e-08;   // 2-part pi/2 (|n| < 2^29)
  const double st[4] = {L.t01.x, L.t01.y, L.t23.x, L.t23.y};   // phaseEst_{i-1} .. phaseEst_{i+2} (stored)
  const int dk = (int)(i - W.kw);
  // TH32: stored_{i-1+e} = a + s (o + e) + r_e (o: row i - 1 within its line; the group never
  // crosses a line or a pseudo-block, pb = 0 mod 32), folded per group into
  //   angle = G + (ws + scale s) (dk + e) + scale r_e,  G = base_h + scale (a + s (o - dk))
  // -- 3 f64 operations a sample, as the full rows' 2 plus the residual's conversion
  const float rv[4] = {L.r.x, L.r.y, L.r.z, L.r.w};
  double G = 0.0, W2 = 0.0;
  if constexpr (TH32) {
    const bool h0 = i - 1 >= T.bound;
    const int o = (int)((i - 1) & 31);
    W2 = fma(W.scale, L.t01.y, W.ws);
    G = fma(W.scale, fma(L.t01.y, (double)(o - dk), L.t01.x), h0 ? W.base[1] : W.base[0]);
  }
  float y[4];
  int q[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t j = i - 1 + e;
    const bool h = j >= T.bound;
    // (r06: the base of output i + e in one fma, and the linear response -- an angle of at most
    // 0.3 scale rad -- in f32 (its rounding ~1e-8 rad, below the f32 cos / sin): 7 f64
    // operations a sample instead of 10)
    double a;
    if constexpr (TH32) a = fma((double)rv[e], W.scale, fma(W2, (double)(dk + e), G));
    else a = fma(st[e], W.scale, fma(W.ws, (double)(dk + e), h ? W.base[1] : W.base[0]));
    if (lin) a = a + (double)fmaf(L.rr[e].x, h ? W.sd0[1] : W.sd0[0], L.rr[e].y * (h ? W.sd1[1] : W.sd1[0]));
    const double n = rint(a * k2oPi);
    double r = fma(-n, Q1, a);
    r = fma(-n, Q2, r);
    y[e] = (float)r;
    q[e] = (int)n & 3;
  }
  nco_poly2({y[0], y[1]}, {q[0], q[1]}, &c[0], &sn[0]);
  nco_poly2({y[2], y[3]}, {q[2], q[3]}, &c[2], &sn[2]);
}

// A matrix-core mixer's chunk: inputs i0 .. i0+3 (i0 = 1 mod 4 -- so no chunk straddles the
// row's end (n = 0 mod 4) except the last, i0 = n - 3, and none its start except i0 = -3, whose
// only input in the row is x[0] with the carried NCO[0]).  Loads are clamped into the rows
// (x[n], read by the last chunk, is row padding: receiver rows are >= n + 1 long) and the
// response rows always read: branch-free, unconditional loads that the compiler counts exactly.
struct MixLd {
  float4 x;
  Nco4Ld t;
};
// (lin: whether to read the response rows -- true always for the RDS loop, whose blocks all
// carry one; the pilot loop's rarely do, and a uniform branch then costs little)
template <bool TH32 = false>
__device__ __forceinline__ void mix_load(const NcoSrc& N, const NcoTile& T, const float* xr, int64_t i0, bool lin,
                                         MixLd* L) {
  __builtin_memcpy(&L->x, xr + (i0 > 0 ? i0 : (int64_t)0), sizeof(float4));   // (4-B aligned)
  nco4_load<TH32>(N, T, i0 > 1 ? i0 : (int64_t)1, lin, &L->t);
}
// the chunk's inputs (0 outside [0, n)) and cos / sin (NCO[0]: the carried c0 / s0)
template <bool TH32 = false>
__device__ __forceinline__ void mix_eval(const NcoTile& T, const NcoWin& W, int64_t i0, int64_t n, const MixLd& L,
                                         bool lin, float c0, float s0, float (&xv)[4], float (&c)[4], float (&sn)[4]) {
  nco4_eval_w<TH32>(T, W, i0, L.t, lin, c, sn);
  // per chunk, not per sample: i0 = -3 (only x[0], with NCO[0]), i0 = n - 3 (the last three),
  // wholly outside the row, or interior
  const bool head = i0 == -3, tail = i0 == n - 3, out = (i0 < 0 && !head) || i0 >= n;
  xv[0] = (head || out) ? 0.f : L.x.x;
  xv[1] = (head || out) ? 0.f : L.x.y;
  xv[2] = (head || out) ? 0.f : L.x.z;
  xv[3] = head ? L.x.x : ((tail || out) ? 0.f : L.x.w);
  c[3] = head ? c0 : c[3];
  sn[3] = head ? s0 : sn[3];
}

// ---- the fused mixer's pairs (PllJob::pair), as the receiver's filters read them ----------
// pair[k] = 2 x[k] (cos, sin)(a_k) with a_k the NCO angle of the phase the PLL kernel stored;
// a long call's pseudo-block b is then rotated by scale (2 pi shift_b + (A^(kk+1) d_b)_phase)
// (the chain's turns and its linear response: the same correction nco_phase_in makes to the
// phase, moved past the cos / sin: x cos(a + r) = (x cos a) cos r - (x sin a) sin r).
struct MixSrc {
  const float* pair;       // pair rows: float pairs, pstride pairs apart per stream
  int64_t pstride;
  double scale;            // ncoScale
  const LongBlk* blk;      // long calls: stream s's pseudo-blocks at blk + s * blk_stride
  int64_t blk_stride, pb;
  int nb;
  const double* resp;      // the response table (row 0 of A^j, sdr_pll_resp_table)
};
struct MixTile {
  int64_t kb, bound;       // phases j in [kb, bound): the first block, [bound, ...): the second
  float rc[2], rs[2];      // cos / sin of scale 2 pi shift
  float sd0[2], sd1[2];    // scale d
  int lin[2], rot[2];
};
__device__ __forceinline__ MixTile mix_tile(const MixSrc& X, int s, int64_t j0) {
  MixTile T;
  T.kb = 0;
  T.bound = INT64_MAX;
  for (int h = 0; h < 2; ++h) {
    T.rc[h] = 1.f; T.rs[h] = 0.f; T.sd0[h] = T.sd1[h] = 0.f; T.lin[h] = T.rot[h] = 0;
  }
  if (X.blk == nullptr) return T;
  const int64_t b = max(j0, (int64_t)0) / X.pb;
  T.kb = b * X.pb;
  T.bound = T.kb + X.pb;
  for (int h = 0; h < 2 && b + h < X.nb; ++h) {
    const LongBlk* B = X.blk + (int64_t)s * X.blk_stride + b + h;
    const double turns = X.scale * B->shift;                 // the rotation, in turns
    const double f = turns - rint(turns);
    double sv, cv;
    sdrnco::sincos_red<false>(sdrnco::k2Pi * f, &sv, &cv);
    T.rc[h] = (float)cv;
    T.rs[h] = (float)sv;
    T.sd0[h] = (float)(X.scale * B->d[0]);
    T.sd1[h] = (float)(X.scale * B->d[1]);
    T.lin[h] = B->d[0] != 0.0 || B->d[1] != 0.0;
    T.rot[h] = T.lin[h] || f != 0.0;
  }
  return T;
}
// pair k (NCO index k: phase k - 1) corrected for its pseudo-block
__device__ __forceinline__ ncof2 mix_rot(const MixSrc& X, const MixTile& T, int64_t k, ncof2 pr) {
  const int64_t j = k - 1;
  if (j < 0) return pr;                                      // the carried input 0: exact
  const int h = j >= T.bound ? 1 : 0;
  if (!T.rot[h]) return pr;
  float c = T.rc[h], sn = T.rs[h];
  if (T.lin[h]) {
    const int64_t kk = j - (h ? T.bound : T.kb);
    const double* rr = X.resp + 2 * (kk + 1);
    const float dl = (float)rr[0] * T.sd0[h] + (float)rr[1] * T.sd1[h];   // |dl| <= 0.3 scale rad
    const float z = dl * dl;
    const float cd = fmaf(z, fmaf(z, fmaf(z, -1.f / 720.f, 1.f / 24.f), -0.5f), 1.f);
    const float sd = dl * fmaf(z, fmaf(z, 1.f / 120.f, -1.f / 6.f), 1.f);
    const float c2 = c * cd - sn * sd, s2 = sn * cd + c * sd;
    c = c2;
    sn = s2;
  }
  return ncof2{pr.x * c - pr.y * sn, pr.y * c + pr.x * sn};
}
