// PLL + NCO for gfx950 (stereo pilot recovery and RDS carrier recovery).
//
// Replaces model/fmPll.py:4-46 (block state: [integrator, phaseEst, feedbackI,
// feedbackQ, ncoOut[0], trigOffset]) and src/helper.cpp:13-57 (fmPLL).
// SURVEY §8a row a9.
//
// The loop is the only serial stage on the path.  It is split in two launches:
//   1. pll_lanes_kernel: ONE LANE PER RECURRENCE.  A launch carries a job table (the
//      stereo pilot PLL and the RDS carrier PLL of every stream); each
//      wave runs one job for up to 64 streams, lane = stream, so one wave advances 64
//      independent loops at the cost of one.  Per lane, in f64:
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
//      The lane also writes ncoOut[0] / ncoOutQ[0] (the carried values) before the loop.
//   2. nco_jobs_kernel: fully parallel ncoOut[k+1] = cos(th_k*scale + adj),
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

// Steps per group: the next group's inputs are loaded (registers) while this one runs,
// and the group's phases leave as 16-B stores.
constexpr int PG = 32;

template <bool VEC>
__global__ __launch_bounds__(64) void pll_lanes_kernel(PllJobs P) {
#pragma clang fp contract(off)  // Python evaluates a*b + c with two roundings
  // one job per wave (a lane-varying job index into the kernarg table would copy the whole
  // table to scratch); lane = stream
  const int wpj = (P.nstreams + 63) / 64;
  const int q = blockIdx.x / wpj;
  const int s = (blockIdx.x - q * wpj) * 64 + threadIdx.x;
  if (s >= P.nstreams) return;  // votes below run over the active lanes only
  const PllJob& J = P.j[q];
  struct {
    const float* in; double* th; float* nco_i; float* nco_q;
  } L{J.in + (int64_t)s * J.in_stride, J.theta + (int64_t)s * J.th_stride,
      J.nco_i + (int64_t)s * J.out_stride, J.nco_q ? J.nco_q + (int64_t)s * J.out_stride : nullptr};
  const PllCfg cfg = J.cfg;
  double* st = J.state + (int64_t)s * 6;
  const int64_t n = P.n;
  double integ = st[0], phase = st[1], fI = st[2], fQ = st[3];
  const double off = st[5];
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  // ncoOut[0] = the carried value; ncoOutQ[0]: the reference leaves it uninitialised
  // (np.empty, fmPll.py:13); here sin(th_prev*scale + adj) with th_prev rebuilt from the
  // carried state (0 at stream start), the quadrature twin of ncoOut[0].
  L.nco_i[0] = (float)st[4];
  if (L.nco_q) L.nco_q[0] = (float)((off > 0.0) ? sin((w * off + phase) * cfg.scale + cfg.adj) : 0.0);
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
  // Fast form for x != 0: atan2(-x sin a, x cos a) = wrap(-a) or wrap(pi - a), branch-free.
  // The step is issue-bound (one wave issues every instruction of the recurrence; an f64
  // op holds the SIMD ~8 cycles at wave64), so it is written for the fewest f64 ops (10: 23
  // instructions per step became 15, tools/pll_probe.hip): the loop filter's updates as
  // FMAs (one rounding where Python rounds twice: the f32 outputs cannot see the
  // difference) and a two-constant reduction (the third term is below 1e-22 rad per turn).  `base` = (off + k) + 1 is a running exact integer in double (< 2^53).
  double base = 0.0;
  auto fast = [&](float xf) {
    const double sel = xf > 0.f ? 0.0 : kPi;                 // off the chain: x is known
    const double d = sel - arg;
    // n = ceil(d/2pi - 1/2) rounds half-way cases down, so e = d - 2 pi n lies in (-pi, pi]
    // (atan2's range) without a range fix
    const double nn = ceil(fma(d, kInv2Pi, -0.5));
    const double e = fma(-nn, kP2, fma(-nn, kP1, d));
    integ = fma(cfg.ki, e, integ);
    phase = fma(cfg.kp, e, phase) + integ;
    base = base + 1.0;
    arg = fma(w, base, phase);
  };
  auto load_group = [&](float (&v)[PG], int64_t k0) {
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < PG; i += 4) {
        const float4 f = *reinterpret_cast<const float4*>(L.in + k0 + i);
        v[i] = f.x; v[i + 1] = f.y; v[i + 2] = f.z; v[i + 3] = f.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < PG; ++i) v[i] = L.in[k0 + i];
    }
  };
  const int64_t ng = n / PG;
  float cur[PG], nxt[PG];
  if (ng > 0) load_group(cur, 0);
  for (int64_t g = 0; g < ng; ++g) {
    if (g + 1 < ng) load_group(nxt, (g + 1) * PG);
    // wave vote: does any lane's group hold a 0 or NaN input (the general form's other
    // case), or is it the call's first group (literal first sample)?
    bool odd = g == 0;
#pragma unroll
    for (int i = 0; i < PG; ++i) odd |= !(cur[i] > 0.f || cur[i] < 0.f);
    if (__any(odd)) {
      // rare (first group of a call, zero or NaN inputs): a rolled loop over the inputs
      // in memory, phases stored one by one (unrolled, its atan2/sincos would spill)
      for (int i = 0; i < PG; ++i) {
        const int64_t k = g * PG + i;
        general(L.in[k], k, k == 0);
        L.th[k] = arg;
      }
    } else {
      double thv[PG];
      base = (off + (double)(g * PG - 1)) + 1.0;
#pragma unroll
      for (int i = 0; i < PG; ++i) {
        fast(cur[i]);
        thv[i] = arg;
      }
      double* tp = L.th + g * PG;
      if constexpr (VEC) {
#pragma unroll
        for (int i = 0; i < PG; i += 2) *reinterpret_cast<double2*>(tp + i) = make_double2(thv[i], thv[i + 1]);
      } else {
#pragma unroll
        for (int i = 0; i < PG; ++i) tp[i] = thv[i];
      }
    }
#pragma unroll
    for (int i = 0; i < PG; ++i) cur[i] = nxt[i];
  }
  for (int64_t k = ng * PG; k < n; ++k) {      // tail (< PG samples)
    general(L.in[k], k, k == 0);
    L.th[k] = arg;
  }
  if (n > 0) {
    st[0] = integ;
    st[1] = phase;
    st[2] = cos(arg);
    st[3] = sin(arg);
    st[4] = cos(arg * cfg.scale + cfg.adj);
    st[5] = off + (double)n;
  }
}

// nco[k+1] from th_k for every (job, stream) of the table; nco[0] is the loop kernel's.
__global__ void nco_jobs_kernel(PllJobs P) {
#pragma clang fp contract(off)
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= P.n) return;
  const int g = blockIdx.y;                 // uniform: (job, stream)
  const int q = g / P.nstreams;
  const int s = g - q * P.nstreams;
  const PllJob& J = P.j[q];
  const double a = J.theta[(int64_t)s * J.th_stride + k] * J.cfg.scale + J.cfg.adj;
  double sv, cv;
  sincos(a, &sv, &cv);
  J.nco_i[(int64_t)s * J.out_stride + k + 1] = (float)cv;
  if (J.nco_q) J.nco_q[(int64_t)s * J.out_stride + k + 1] = (float)sv;
}

}  // namespace

hipError_t sdr_launch_pll_jobs(const PllJobs& P, hipStream_t st) {
  if (P.njobs < 1 || P.njobs > SDR_PLL_MAXJ || P.nstreams <= 0 || P.n < 0) return hipErrorInvalidValue;
  // 16-B loads/stores need every lane's input row and phase row 16-B aligned
  bool vec = true;
  for (int q = 0; q < P.njobs; ++q) {
    const PllJob& J = P.j[q];
    vec = vec && ((uintptr_t)J.in % 16) == 0 && (J.in_stride % 4) == 0 && ((uintptr_t)J.theta % 16) == 0 &&
          (J.th_stride % 2) == 0;
  }
  const int lanes = P.njobs * P.nstreams;
  const dim3 grid((unsigned)(P.njobs * ((P.nstreams + 63) / 64)));
  if (vec) hipLaunchKernelGGL(pll_lanes_kernel<true>, grid, dim3(64), 0, st, P);
  else hipLaunchKernelGGL(pll_lanes_kernel<false>, grid, dim3(64), 0, st, P);
  if (P.n > 0)
    hipLaunchKernelGGL(nco_jobs_kernel, dim3((unsigned)((P.n + 255) / 256), (unsigned)lanes), dim3(256), 0, st, P);
  return hipGetLastError();
}
