// PLL + NCO for gfx950 (stereo pilot recovery and RDS carrier recovery).
//
// Replaces model/fmPll.py:4-46 (block state: [integrator, phaseEst, feedbackI,
// feedbackQ, ncoOut[0], trigOffset]) and src/helper.cpp:13-57 (fmPLL).
// SURVEY §8a row a9.
//
// The loop is the only serial stage on the path.  It is split in two launches:
//   1. pll_loop_kernel: one lane per stream runs the recurrence in f64,
//        e_k   = atan2(-x_k fQ, x_k fI)                      (fmPll.py:24-27)
//        integ += Ki e_k ; phaseEst += Kp e_k + integ         (fmPll.py:29-31)
//        th_k  = 2 pi (freq/Fs) (trigOffset + k + 1) + phaseEst (fmPll.py:33)
//        fI, fQ = cos th_k, sin th_k                          (fmPll.py:34-35)
//      and stores th_k.  Because (fI, fQ) = (cos, sin) of the previous th, the
//      phase detector is evaluated as the exactly reduced angle -th (x > 0) or
//      pi - th (x < 0): a three-constant Cody-Waite reduction by 2 pi, identical
//      to atan2(-x sin th, x cos th) up to rounding (~1e-16 rad).  x == 0, NaN and
//      the first sample of a call (whose fI, fQ come from the caller's state)
//      take the literal sincos + atan2 form, so signed zeros behave as in Python.
//   2. nco_kernel: fully parallel ncoOut[k+1] = cos(th_k*scale + adj),
//      ncoOutQ[k+1] = sin(th_k*scale + adj) (fmPll.py:36-37).
// All phase arithmetic is f64 (SURVEY §7 hard part 5: an fp32 NCO drifts).
#include "sdr_launch.h"


namespace {

// 2*pi split into three parts (Cody-Waite), so n*P1 and n*P2 are exact for |n| < 2^26.
constexpr double kP1 = 6.2831854820251465;       // float32(2 pi), 24 significant bits
constexpr double kP2 = -1.748455600074497e-07;    // double(2 pi - kP1)
constexpr double kP3 = -1.0687562935444062e-23;   // remainder
constexpr double kInv2Pi = 0.15915494309189535;
constexpr double kPi = 3.14159265358979323846;

// r = a - 2*pi*n, n = rint(a / 2pi), |r| <= pi (up to one ulp at the boundary).
__device__ inline double reduce_2pi(double a) {
  const double n = rint(a * kInv2Pi);
  double r = fma(-n, kP1, a);
  r = fma(-n, kP2, r);
  r = fma(-n, kP3, r);
  return r;
}

// One wave per stream.  Every lane runs the same recurrence (wave-uniform values, no
// divergence); the inputs come from LDS in chunks of PCH samples, the next chunk's global
// loads are in flight (in registers) while the current chunk runs, and the phases go out
// through LDS as coalesced stores.  (A lone lane reading x[k] from global memory per step
// waits an L2 round trip every sample.)
constexpr int PCH = 512;
__global__ __launch_bounds__(64) void pll_loop_kernel(const float* in, int64_t n, int64_t in_stride,
                                                      int nstreams, PllCfg cfg, double* state,
                                                      int64_t state_stride, double* theta,
                                                      int64_t th_stride) {
#pragma clang fp contract(off)  // Python evaluates a*b + c with two roundings
  const int s = blockIdx.x;
  const int lane = threadIdx.x;
  if (s >= nstreams) return;
  __shared__ alignas(16) float xs[2][PCH];
  __shared__ double ths[PCH];
  const float* x = in + (int64_t)s * in_stride;
  double* st = state + (int64_t)s * state_stride;
  double* th = theta + (int64_t)s * th_stride;
  double integ = st[0], phase = st[1], fI = st[2], fQ = st[3];
  const double off = st[5];
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  double arg = 0.0;
  // One step of model/fmPll.py:23-41.  General form: the first sample of a call uses the
  // caller's (fI, fQ) literally, and an input of 0 or NaN takes atan2 on the products.
  auto general = [&](float xf, int64_t k, bool literal) {
    const double xv = (double)xf;
    double e;
    if (literal || !(xv > 0.0 || xv < 0.0)) {
      if (!literal) { fI = cos(arg); fQ = sin(arg); }
      e = atan2(xv * (-fQ), xv * fI);
    } else {
      e = reduce_2pi(xv > 0.0 ? -arg : kPi - arg);
      if (e <= -kPi) e += 2.0 * kPi;   // atan2 range is (-pi, pi]
    }
    integ = integ + cfg.ki * e;
    phase = phase + cfg.kp * e + integ;
    arg = w * ((off + (double)k) + 1.0) + phase;
  };
  // Fast form for x != 0: atan2(-x sin a, x cos a) = wrap(-a) or wrap(pi - a), branch-free;
  // `base` = (off + k) + 1 kept as a running exact integer in double (< 2^53).
  double base = 0.0;
  auto fast = [&](float xf) {
    const double sel = xf > 0.f ? 0.0 : kPi;                 // off the chain: x is known
    const double r = reduce_2pi(sel - arg);
    const double e = r <= -kPi ? r + 2.0 * kPi : r;
    integ = integ + cfg.ki * e;
    phase = phase + cfg.kp * e + integ;
    base = base + 1.0;
    arg = w * base + phase;
  };
  constexpr int PL = PCH / 64;
  const int64_t nch = (n + PCH - 1) / PCH;
  for (int j = 0; j < PL; ++j) {
    const int64_t k = lane + 64 * j;
    xs[0][lane + 64 * j] = k < n ? x[k] : 0.f;
  }
  __syncthreads();
  for (int64_t c = 0; c < nch; ++c) {
    const int buf = (int)(c & 1);
    float pre[PL];
#pragma unroll
    for (int j = 0; j < PL; ++j) {               // next chunk: loads in flight meanwhile
      const int64_t k = (c + 1) * PCH + lane + 64 * j;
      pre[j] = k < n ? x[k] : 0.f;
    }
    const int kn = (int)min<int64_t>(PCH, n - c * PCH);
    const float* xc = xs[buf];
    int kk = 0;
    if (c == 0) {                                // the literal first sample
      general(xc[0], 0, true);
      if (lane == 0) ths[0] = arg;
      kk = 1;
    }
    // wave vote: does the chunk hold a 0 or NaN input (the general form's other case)?
    bool odd = false;
#pragma unroll
    for (int j = 0; j < PL; ++j) {
      const int e = lane + 64 * j;
      const float v = xc[e];
      odd |= e < kn && !(v > 0.f || v < 0.f);
    }
    if (__any(odd)) {
      for (; kk < kn; ++kk) {
        general(xc[kk], c * PCH + kk, false);
        if (lane == 0) ths[kk] = arg;
      }
    } else {
      base = (off + (double)(c * PCH + kk - 1)) + 1.0;
      // groups of 4: the next group's LDS reads are in flight during this group's steps
      const int ng = (kn - kk) / 4;
      float n0 = xc[kk], n1 = xc[kk + 1], n2 = xc[kk + 2], n3 = xc[kk + 3];  // kk+3 < PCH
      for (int g = 0; g < ng; ++g, kk += 4) {
        const float c0 = n0, c1 = n1, c2 = n2, c3 = n3;
        if (g + 1 < ng) { n0 = xc[kk + 4]; n1 = xc[kk + 5]; n2 = xc[kk + 6]; n3 = xc[kk + 7]; }
        fast(c0); const double a0 = arg;
        fast(c1); const double a1 = arg;
        fast(c2); const double a2 = arg;
        fast(c3);
        if (lane == 0) { ths[kk] = a0; ths[kk + 1] = a1; ths[kk + 2] = a2; ths[kk + 3] = arg; }
      }
      for (; kk < kn; ++kk) {
        fast(xc[kk]);
        if (lane == 0) ths[kk] = arg;
      }
    }
    __syncthreads();
    for (int e = lane; e < kn; e += 64) th[c * PCH + e] = ths[e];
#pragma unroll
    for (int j = 0; j < PL; ++j) xs[buf ^ 1][lane + 64 * j] = pre[j];
    __syncthreads();
  }
  if (n > 0 && lane == 0) {
    st[0] = integ;
    st[1] = phase;
    st[2] = cos(arg);
    st[3] = sin(arg);
    st[4] = cos(arg * cfg.scale + cfg.adj);
    st[5] = off + (double)n;
  }
}

// nco[0] = carried ncoOut (state[4] before the call, passed as nco0[s]); nco[k+1] from th_k.
// ncoQ[0]: the reference leaves it uninitialised (np.empty, fmPll.py:13); here it is
// sin(th_prev*scale + adj) with th_prev rebuilt from the carried state (0 at stream start),
// the quadrature twin of ncoOut[0] (documented deviation).
__global__ void nco_kernel(const double* theta, int64_t th_stride, int64_t n, int nstreams,
                           PllCfg cfg, const double* nco0, const double* ncoq0, float* nco_i,
                           float* nco_q, int64_t out_stride) {
#pragma clang fp contract(off)
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  if (s >= nstreams || gid > n) return;
  float* oi = nco_i + (int64_t)s * out_stride;
  float* oq = nco_q ? nco_q + (int64_t)s * out_stride : nullptr;
  if (gid == 0) {
    oi[0] = (float)nco0[s];
    if (oq) oq[0] = (float)ncoq0[s];
    return;
  }
  const double a = theta[(int64_t)s * th_stride + gid - 1] * cfg.scale + cfg.adj;
  double sv, cv;
  sincos(a, &sv, &cv);
  oi[gid] = (float)cv;
  if (oq) oq[gid] = (float)sv;
}

// Before the loop: remember ncoOut[0] and build ncoOutQ[0] from the incoming state.
__global__ void nco_prologue_kernel(const double* state, int64_t state_stride, int nstreams,
                                    PllCfg cfg, double* nco0, double* ncoq0) {
#pragma clang fp contract(off)
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams) return;
  const double* st = state + (int64_t)s * state_stride;
  nco0[s] = st[4];
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  ncoq0[s] = (st[5] > 0.0) ? sin((w * st[5] + st[1]) * cfg.scale + cfg.adj) : 0.0;
}

}  // namespace

// scratch: theta (n per stream, th_stride), nco0/ncoq0 (nstreams each).
hipError_t sdr_launch_pll(const float* in, int64_t n, int64_t in_stride, int nstreams,
                          const PllCfg& cfg, double* state_dev, double* theta, int64_t th_stride,
                          double* nco0, double* ncoq0, float* nco_i, float* nco_q,
                          int64_t out_stride, hipStream_t st) {
  if (nstreams <= 0) return hipSuccess;
  const int nb = (nstreams + 63) / 64;
  hipLaunchKernelGGL(nco_prologue_kernel, dim3(nb), dim3(64), 0, st, state_dev, (int64_t)6,
                     nstreams, cfg, nco0, ncoq0);
  hipLaunchKernelGGL(pll_loop_kernel, dim3(nstreams), dim3(64), 0, st, in, n, in_stride, nstreams, cfg,
                     state_dev, (int64_t)6, theta, th_stride);
  const int64_t nout = n + 1;
  hipLaunchKernelGGL(nco_kernel, dim3((unsigned)((nout + 255) / 256), nstreams), dim3(256), 0, st,
                     theta, th_stride, n, nstreams, cfg, nco0, ncoq0, nco_i, nco_q, out_stride);
  return hipGetLastError();
}
