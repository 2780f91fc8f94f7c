// Probe (not product): f64 VALU latency and issue cost for ONE wave with one active lane, the
// regime of the PLL recurrence (pll.hip).  Cycles per op (clock64) for a dependent fma chain,
// a dependent fract+fma chain, and 2 / 4 / 8 independent fma chains interleaved.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/f64_probe.hip -o tools/f64_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int N = 65536;

template <int K, bool FRACT>
__global__ void chains(double a, double b, double* out, long long* cyc) {
  if (threadIdx.x != 0) return;
  double x[K];
#pragma unroll
  for (int k = 0; k < K; ++k) x[k] = a + k;
  const long long t0 = clock64();
#pragma unroll 64
  for (int i = 0; i < N / K; ++i) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (FRACT) x[k] = fma(__builtin_amdgcn_fract(x[k]), a, b);
      else x[k] = fma(x[k], a, b);
    }
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) s += x[k];
  out[0] = s;
  cyc[0] = t1 - t0;
}

// the PLL fast step (pll.hip) with its constants in registers (no memory): cycles and
// nanoseconds per step for one lane -- the floor of the recurrence at the clock it runs at
__global__ void pll_step(double c0, double kA, double kB, double kC, double* out, long long* cyc) {
  if (threadIdx.x != 0) return;
  double phase = 0.1, V = -0.01, acc = 0.0;
  double c[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) c[i] = c0 + 0.37 * i;
  const long long t0 = clock64();
  for (int it = 0; it < N / 32; ++it) {
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const double t = fma(-0.15915494309189535, phase, c[i & 7]);
      const double f = __builtin_amdgcn_fract(t);
      const double S = phase + V;
      V = fma(kA, f, V - kB);
      phase = fma(kC, f, S);
    }
    acc += phase;
  }
  const long long t1 = clock64();
  out[0] = acc + V;
  cyc[0] = t1 - t0;
}

template <typename Kern>
void run(Kern kern, const char* name, int ops, double* d, long long* c) {
  long long best = 1LL << 62;
  for (int r = 0; r < 5; ++r) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, 0.999999, 1e-9, d, c);
    CK(hipDeviceSynchronize());
    long long h;
    CK(hipMemcpy(&h, c, sizeof h, hipMemcpyDeviceToHost));
    if (h < best) best = h;
  }
  printf("%-34s %7.2f clock64 ticks per op\n", name, (double)best / ops);
}

int main() {
  double* d;
  long long* c;
  CK(hipMalloc(&d, 8));
  CK(hipMalloc(&c, 8));
  run(chains<1, false>, "fma, 1 dependent chain", N, d, c);
  run(chains<2, false>, "fma, 2 chains", N, d, c);
  run(chains<4, false>, "fma, 4 chains", N, d, c);
  run(chains<8, false>, "fma, 8 chains", N, d, c);
  run(chains<1, true>, "fract+fma, 1 chain (per pair)", N, d, c);
  run(chains<2, true>, "fract+fma, 2 chains (per pair)", N, d, c);
  run(chains<4, true>, "fract+fma, 4 chains (per pair)", N, d, c);
  {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9f;
    long long bc = 0;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(pll_step, dim3(1), dim3(64), 0, 0, 0.3, 2e-5, 1e-5, 0.17, d, c);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      long long h;
      CK(hipMemcpy(&h, c, sizeof h, hipMemcpyDeviceToHost));
      if (ms < best) { best = ms; bc = h; }
    }
    printf("PLL fast step, constants in registers: %.2f ticks/step, %.2f ns/step incl. launch (%d steps)\n",
           (double)bc / N, best * 1e6 / N, N);
  }
  int rate = 0;
  CK(hipDeviceGetAttribute(&rate, hipDeviceAttributeClockRate, 0));
  printf("device clock attribute: %d kHz (clock64 counts shader cycles)\n", rate);
  return 0;
}
