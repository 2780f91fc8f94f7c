// Probe (not product): what one small launch costs on this GPU -- empty kernels with a small
// and a 1.2-KB kernarg, a 4-workgroup kernel with one global round trip, and back-to-back
// chains of two dependent launches; per launch, event-timed, median of 200.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/launch_probe.hip -o tools/launch_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

struct Big { float v[300]; };
__global__ void k_small(float* p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345.f) p[1] = 1.f; }
__global__ void k_big(Big b, float* p) { if (threadIdx.x == 0 && blockIdx.x == 0 && b.v[7] == 12345.f) p[1] = 1.f; }
__global__ void k_trip(const float* in, float* out) {         // one dependent global round trip
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float v = in[i];
  for (int k = 0; k < 4; ++k) v = v * 1.0001f + in[(i + 64 * k) & 4095];
  out[i] = v;
}
__global__ void k_chain(const float* in, float* out) {       // four dependent round trips
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int j = i;
  float v = 0.f;
  for (int k = 0; k < 4; ++k) { v += in[j]; j = ((int)v + i * 7 + k) & 4095; }
  out[i] = v;
}

int main() {
  float *a, *b;
  CK(hipMalloc(&a, 1 << 20));
  CK(hipMalloc(&b, 1 << 20));
  CK(hipMemset(a, 0, 1 << 20));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  Big big{};
  auto med = [&](auto launch, int per) {
    std::vector<float> t;
    for (int r = 0; r < 200; ++r) {
      CK(hipEventRecord(e0, st));
      for (int q = 0; q < per; ++q) launch();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms * 1e3f / per);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  for (int pass = 0; pass < 2; ++pass) {
    printf("pass %d\n", pass);
    printf("  empty kernel, 8-B kernarg     x1: %6.2f us   x10 back-to-back: %6.2f us/launch\n",
           med([&] { hipLaunchKernelGGL(k_small, dim3(4), dim3(128), 0, st, a); }, 1),
           med([&] { hipLaunchKernelGGL(k_small, dim3(4), dim3(128), 0, st, a); }, 10));
    printf("  empty kernel, 1.2-KB kernarg  x1: %6.2f us   x10 back-to-back: %6.2f us/launch\n",
           med([&] { hipLaunchKernelGGL(k_big, dim3(4), dim3(128), 0, st, big, a); }, 1),
           med([&] { hipLaunchKernelGGL(k_big, dim3(4), dim3(128), 0, st, big, a); }, 10));
    printf("  4 WGs, one round trip         x1: %6.2f us   x10 back-to-back: %6.2f us/launch\n",
           med([&] { hipLaunchKernelGGL(k_trip, dim3(4), dim3(128), 0, st, a, b); }, 1),
           med([&] { hipLaunchKernelGGL(k_trip, dim3(4), dim3(128), 0, st, a, b); }, 10));
    printf("  4 WGs, four dependent trips   x1: %6.2f us   x10 back-to-back: %6.2f us/launch\n",
           med([&] { hipLaunchKernelGGL(k_chain, dim3(4), dim3(128), 0, st, a, b); }, 1),
           med([&] { hipLaunchKernelGGL(k_chain, dim3(4), dim3(128), 0, st, a, b); }, 10));
  }
  // per-block transfer floor of the drop-in path (51 200 complex f32 = 409 600 B in, 4 KB out)
  const size_t nin = 409600, nout = 4096;
  std::vector<char> host(nin), hout(nout);
  void *pin, *pout;
  CK(hipHostMalloc(&pin, nin, hipHostMallocDefault));
  CK(hipHostMalloc(&pout, nout, hipHostMallocDefault));
  auto wall = [&](auto fn) {
    std::vector<double> t;
    for (int r = 0; r < 200; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      fn();
      t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  printf("host memcpy 409 KB -> pinned          : %7.2f us\n", wall([&] { memcpy(pin, host.data(), nin); }));
  printf("H2D 409 KB from pinned + sync         : %7.2f us\n", wall([&] {
    CK(hipMemcpyAsync(a, pin, nin, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st)); }));
  printf("H2D 409 KB from pageable + sync       : %7.2f us\n", wall([&] {
    CK(hipMemcpyAsync(a, host.data(), nin, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st)); }));
  printf("D2H 4 KB to pinned + sync             : %7.2f us\n", wall([&] {
    CK(hipMemcpyAsync(pout, b, nout, hipMemcpyDeviceToHost, st)); CK(hipStreamSynchronize(st)); }));
  printf("empty kernel + sync                   : %7.2f us\n", wall([&] {
    hipLaunchKernelGGL(k_small, dim3(4), dim3(128), 0, st, a); CK(hipStreamSynchronize(st)); }));
  printf("H2D + 2 kernels + D2H + one sync      : %7.2f us\n", wall([&] {
    memcpy(pin, host.data(), nin);
    CK(hipMemcpyAsync(a, pin, nin, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_trip, dim3(32), dim3(64), 0, st, a, b);
    hipLaunchKernelGGL(k_trip, dim3(4), dim3(128), 0, st, b, a);
    CK(hipMemcpyAsync(pout, a, nout, hipMemcpyDeviceToHost, st)); CK(hipStreamSynchronize(st)); }));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  auto spin = [&] {
    CK(hipEventRecord(ev, st));
    hipError_t q;
    while ((q = hipEventQuery(ev)) == hipErrorNotReady) {}
    CK(q);
  };
  printf("empty kernel + event spin             : %7.2f us\n", wall([&] {
    hipLaunchKernelGGL(k_small, dim3(4), dim3(128), 0, st, a); spin(); }));
  printf("D2H 4 KB to pinned + event spin       : %7.2f us\n", wall([&] {
    CK(hipMemcpyAsync(pout, b, nout, hipMemcpyDeviceToHost, st)); spin(); }));
  printf("H2D + 2 kernels + D2H + event spin    : %7.2f us\n", wall([&] {
    memcpy(pin, host.data(), nin);
    CK(hipMemcpyAsync(a, pin, nin, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_trip, dim3(32), dim3(64), 0, st, a, b);
    hipLaunchKernelGGL(k_trip, dim3(4), dim3(128), 0, st, b, a);
    CK(hipMemcpyAsync(pout, a, nout, hipMemcpyDeviceToHost, st)); spin(); }));
  return 0;
}
