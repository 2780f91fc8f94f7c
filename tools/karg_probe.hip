// Host cost of hipLaunchKernelGGL against the kernel-argument size (tuning aid, not product):
// 2 000 back-to-back launches of an empty kernel per size on one stream, host wall time per
// launch, then the stream drained.  hipcc --offload-arch=gfx950 -O2 tools/karg_probe.hip -o tools/karg_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

template <int N> struct Args { int v[N / 4]; };
template <int N> __global__ void k(Args<N> a, int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.v[0] == 12345) out[0] = a.v[N / 4 - 1];
}
template <int N> double probe(int* d, hipStream_t st) {
  Args<N> a{};
  for (int w = 0; w < 200; ++w) hipLaunchKernelGGL(k<N>, dim3(1), dim3(64), 0, st, a, d);
  hipStreamSynchronize(st);
  const int n = 2000;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k<N>, dim3(1), dim3(64), 0, st, a, d);
  const auto t1 = std::chrono::steady_clock::now();
  hipStreamSynchronize(st);
  const auto t2 = std::chrono::steady_clock::now();
  printf("kernarg %5d B: %.2f us per launch (host), %.2f us per launch incl. drain\n", N,
         std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
         std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
  return 0;
}
int main() {
  int* d;
  hipMalloc(&d, 64);
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  probe<16>(d, st); probe<256>(d, st); probe<512>(d, st); probe<1024>(d, st); probe<1536>(d, st); probe<2048>(d, st);
  probe<16>(d, st);
  return 0;
}
