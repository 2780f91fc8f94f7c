// A/B probe for the PLL fast step (not product code): times the product pll_lanes kernel
// (pll.o, sdr_launch_pll_jobs) against candidate step forms on the same inputs, and reports
// ns per sample step and the deviation of each candidate's phases from the product's.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pll_probe.hip -o tools/pll_probe \
//     -Lreal-time-software-defined-radio_amd -lsdr -Wl,-rpath,$ORIGIN/../real-time-software-defined-radio_amd
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../real-time-software-defined-radio_amd/csrc/sdr_launch.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

namespace {
constexpr double kP1 = 6.2831854820251465, kP2 = -1.748455600074497e-07, kP3 = -1.0687562935444062e-23;
constexpr double kInv2Pi = 0.15915494309189535, kPi = 3.14159265358979323846, k2Pi = 6.283185307179586;

__device__ inline double reduce_2pi(double a) {
  const double n = rint(a * kInv2Pi);
  double r = fma(-n, kP1, a);
  r = fma(-n, kP2, r);
  return fma(-n, kP3, r);
}

// V=1: reduced angle A carried step to step (A' = wrap1(A + w) + t), e by compare-select;
//      A re-anchored from the exact arg every PG steps.  Chain: sub, select, select, fma, fma, add.
// V=2: as V=1 with e by rint (one constant) instead of compare-select.
template <int V>
__global__ __launch_bounds__(64) void pll_v(const float* in, int64_t n, int64_t in_stride, int nstreams, PllCfg cfg,
                                            double* state, double* theta, int64_t th_stride) {
#pragma clang fp contract(off)
  const int s = blockIdx.x * 64 + threadIdx.x;
  if (s >= nstreams) return;
  constexpr int PG = 32;
  const float* x = in + (int64_t)s * in_stride;
  double* th = theta + (int64_t)s * th_stride;
  double* st = state + (int64_t)s * 6;
  double integ = st[0], phase = st[1], fI = st[2], fQ = st[3];
  const double off = st[5];
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  double arg = 0.0;
  {  // literal first step
    const double xv = (double)x[0];
    const double e = atan2(xv * (-fQ), xv * fI);
    integ = integ + cfg.ki * e;
    phase = phase + cfg.kp * e + integ;
    arg = w * ((off + 0.0) + 1.0) + phase;
    th[0] = arg;
  }
  double base = off + 1.0;
  const double wr = reduce_2pi(w);
  for (int64_t k0 = 1; k0 < n; k0 += PG) {
    double A = reduce_2pi(arg);           // re-anchor on the exact formula
    const int cnt = (int)min<int64_t>(PG, n - k0);
#pragma unroll 4
    for (int i = 0; i < cnt; ++i) {
      const float xf = x[k0 + i];
      const double sel = xf > 0.f ? 0.0 : kPi;
      double Aw = A + wr;
      Aw = Aw > kPi ? Aw - k2Pi : Aw;      // off the chain
      const double u = sel - A;
      double e;
      if (V == 1) {
        e = u > kPi ? u - k2Pi : (u <= -kPi ? u + k2Pi : u);
      } else {
        e = fma(-rint(u * kInv2Pi), k2Pi, u);
        e = e <= -kPi ? e + k2Pi : e;
      }
      integ = fma(cfg.ki, e, integ);
      const double t = fma(cfg.kp, e, integ);
      A = Aw + t;
      phase = phase + t;                    // off the chain: the exact accumulator for th
      base = base + 1.0;
      arg = w * base + phase;
      th[k0 + i] = arg;
    }
  }
  st[0] = integ;
  st[1] = phase;
}
}  // namespace

int main() {
  const int S = 8;
  const int64_t n = 15360;
  std::vector<float> h(S * n);
  for (int s = 0; s < S; ++s)
    for (int64_t k = 0; k < n; ++k)
      h[s * n + k] = (float)(0.1 * cos(2 * M_PI * 114e3 / 240e3 * k + 0.3 * s) + 0.01 * sin(0.001 * k * (s + 1)));
  float* din;
  double *dst, *dth, *dth2;
  float *nco_i, *nco_q;
  double* cb;
  CK(hipMalloc(&din, sizeof(float) * S * n));
  CK(hipMalloc(&dst, sizeof(double) * 6 * S));
  CK(hipMalloc(&dth, sizeof(double) * S * (n + 2)));
  CK(hipMalloc(&dth2, sizeof(double) * S * (n + 2)));
  CK(hipMalloc(&nco_i, sizeof(float) * S * (n + 1)));
  CK(hipMalloc(&nco_q, sizeof(float) * S * (n + 1)));
  const int64_t cst = n + n / 32 + 2;
  CK(hipMalloc(&cb, sizeof(double) * S * cst));
  CK(hipMemcpy(din, h.data(), sizeof(float) * S * n, hipMemcpyHostToDevice));
  const double bw = 0.001;
  PllCfg cfg{114e3, 240e3, 0.5, M_PI / 3.3 - M_PI / 1.5, bw * 2.666, bw * bw * 3.555};
  std::vector<double> st0(6 * S);
  for (int s = 0; s < S; ++s) { double v[6] = {0, 0, 1, 0, 1, 0}; for (int j = 0; j < 6; ++j) st0[6 * s + j] = v[j]; }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto reset = [&] { CK(hipMemcpy(dst, st0.data(), sizeof(double) * 6 * S, hipMemcpyHostToDevice)); };
  const int reps = 20;
  // product
  PllJobs P{};
  P.njobs = 1; P.nstreams = S; P.n = n;
  P.j[0] = PllJob{din, n, dst, dth, n + 2, nco_i, nco_q, n + 1, cfg, cb, cst};
  float ms = 0;
  for (int r = 0; r < 3; ++r) { reset(); CK(sdr_launch_pll_jobs(P, 0)); }
  CK(hipDeviceSynchronize());
  float best = 1e9;
  for (int r = 0; r < reps; ++r) {
    reset();
    CK(hipEventRecord(e0, 0));
    CK(sdr_launch_pll_jobs(P, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  printf("product  : %8.1f us  %6.1f ns/step (incl. nco kernel)\n", best * 1e3, best * 1e6 / n);
  // the product's theta rows now hold the phase estimates: rebuild th_k = w (k + 1) + phase_k
  std::vector<double> t_ref(S * (n + 2)), t_v(S * (n + 2));
  CK(hipMemcpy(t_ref.data(), dth, sizeof(double) * S * (n + 2), hipMemcpyDeviceToHost));
  for (int s = 0; s < S; ++s)
    for (int64_t k = 0; k < n; ++k)
      t_ref[s * (n + 2) + k] = 2.0 * M_PI * (cfg.freq / cfg.fs) * ((0.0 + (double)k) + 1.0) + t_ref[s * (n + 2) + k];
  auto run_v = [&](auto kern, const char* name) {
    float b = 1e9;
    for (int r = 0; r < reps + 3; ++r) {
      reset();
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, din, n, n, S, cfg, dst, dth2, n + 2);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) b = std::min(b, ms);
    }
    CK(hipMemcpy(t_v.data(), dth2, sizeof(double) * S * (n + 2), hipMemcpyDeviceToHost));
    double dmax = 0, cmax = 0;
    for (int s = 0; s < S; ++s)
      for (int64_t k = 0; k < n; ++k) {
        const double a = t_ref[s * (n + 2) + k], c = t_v[s * (n + 2) + k];
        dmax = std::max(dmax, fabs(a - c));
        cmax = std::max(cmax, fabs(cos(a * 0.5 + cfg.adj) - cos(c * 0.5 + cfg.adj)));
      }
    printf("%-9s: %8.1f us  %6.1f ns/step  max|dtheta| %.2e  max|dnco| %.2e\n", name, b * 1e3, b * 1e6 / n, dmax, cmax);
  };
  run_v(pll_v<1>, "v1 select");
  run_v(pll_v<2>, "v2 rint");
  return 0;
}
