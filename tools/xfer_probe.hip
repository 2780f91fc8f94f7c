// Probe (not product): the per-block transfer floor of the drop-in path with and without the
// DMA engines.  One 51 200-complex f32 block (409 600 B) in, 4 KB out, two small kernels in
// between, one wait; wall clock per block, median of 300:
//   a  memcpy -> pinned, SDMA H2D, k1, k2, SDMA D2H, sync      (the product's shape today)
//   b  memcpy -> pinned, copy kernel (reads pinned), k1, k2, copy kernel (writes pinned), sync
//   c  memcpy -> pinned, k1 reads pinned directly, k2 writes pinned directly, sync
//   d  as a, captured once as a hipGraph
//   e  as c, captured once as a hipGraph
// plus a dependent-load chain (ns per HBM round trip under no load).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xfer_probe.hip -o tools/xfer_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_copy(const float4* __restrict__ in, float4* __restrict__ out, int n4) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) out[i] = in[i];
}
// k1: reads the block (sum of a strided subset per thread), writes 5120 floats
__global__ void k1(const float* __restrict__ in, float* __restrict__ mid) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 5120) return;
  float s = 0.f;
  for (int k = 0; k < 20; ++k) s += in[i * 20 + k];
  mid[i] = s;
}
// k2: 1024 outputs of 5 inputs each
__global__ void k2(const float* __restrict__ mid, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 1024) return;
  float s = 0.f;
  for (int k = 0; k < 5; ++k) s += mid[i * 5 + k];
  out[i] = s;
}
__global__ void k_chase(const int* __restrict__ nxt, int steps, int* out) {
  int j = 0;
  for (int s = 0; s < steps; ++s) j = __builtin_nontemporal_load(nxt + j);
  if (threadIdx.x == 0) out[0] = j;
}

int main() {
  const size_t nin = 409600, nout = 4096;
  float *d_in, *d_mid, *d_out;
  CK(hipMalloc(&d_in, nin));
  CK(hipMalloc(&d_mid, 5120 * 4));
  CK(hipMalloc(&d_out, nout));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<char> host(nin), hres(nout);
  for (size_t i = 0; i < nin / 4; ++i) reinterpret_cast<float*>(host.data())[i] = (float)(i % 97) * 0.01f;
  float *pin, *pout;
  CK(hipHostMalloc(&pin, nin, hipHostMallocDefault));
  CK(hipHostMalloc(&pout, nout, hipHostMallocDefault));
  auto wall = [&](auto fn) {
    std::vector<double> t;
    for (int r = 0; r < 330; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      fn();
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (r >= 30) t.push_back(us);
    }
    std::sort(t.begin(), t.end());
    return std::make_pair(t[t.size() / 2], t[t.size() * 99 / 100]);
  };
  auto report = [&](const char* name, std::pair<double, double> v) {
    printf("%-62s: p50 %7.2f us  p99 %7.2f us\n", name, v.first, v.second);
  };
  const int n4 = (int)(nin / 16);
  auto chain_a = [&] {
    CK(hipMemcpyAsync(d_in, pin, nin, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k1, dim3(20), dim3(256), 0, st, d_in, d_mid);
    hipLaunchKernelGGL(k2, dim3(4), dim3(256), 0, st, d_mid, d_out);
    CK(hipMemcpyAsync(pout, d_out, nout, hipMemcpyDeviceToHost, st));
  };
  auto chain_b = [&] {
    hipLaunchKernelGGL(k_copy, dim3(100), dim3(256), 0, st, (const float4*)pin, (float4*)d_in, n4);
    hipLaunchKernelGGL(k1, dim3(20), dim3(256), 0, st, d_in, d_mid);
    hipLaunchKernelGGL(k2, dim3(4), dim3(256), 0, st, d_mid, d_out);
    hipLaunchKernelGGL(k_copy, dim3(1), dim3(256), 0, st, (const float4*)d_out, (float4*)pout, (int)(nout / 16));
  };
  auto chain_c = [&] {
    hipLaunchKernelGGL(k1, dim3(20), dim3(256), 0, st, pin, d_mid);
    hipLaunchKernelGGL(k2, dim3(4), dim3(256), 0, st, d_mid, pout);
  };
  auto check = [&](const char* name) {
    float ref[4];
    for (int i = 0; i < 4; ++i) {
      float s = 0.f;
      for (int k = 0; k < 5; ++k) {
        float t = 0.f;
        for (int q = 0; q < 20; ++q) t += reinterpret_cast<const float*>(host.data())[(i * 5 + k) * 20 + q];
        s += t;
      }
      ref[i] = s;
    }
    bool ok = true;
    for (int i = 0; i < 4; ++i) ok &= fabsf(pout[i] - ref[i]) < 1e-3f * fabsf(ref[i]) + 1e-3f;
    if (!ok) printf("  %s: WRONG output %g vs %g\n", name, pout[0], ref[0]);
    memset(pout, 0, nout);
  };
  for (int pass = 0; pass < 2; ++pass) {
    printf("pass %d\n", pass);
    report("a  memcpy, SDMA H2D, k1, k2, SDMA D2H, sync", wall([&] {
      memcpy(pin, host.data(), nin); chain_a(); CK(hipStreamSynchronize(st)); }));
    check("a");
    report("b  memcpy, copy-kernel in, k1, k2, copy-kernel out, sync", wall([&] {
      memcpy(pin, host.data(), nin); chain_b(); CK(hipStreamSynchronize(st)); }));
    check("b");
    report("c  memcpy, k1 reads pinned, k2 writes pinned, sync", wall([&] {
      memcpy(pin, host.data(), nin); chain_c(); CK(hipStreamSynchronize(st)); }));
    check("c");
    hipGraph_t g;
    hipGraphExec_t ga, gc;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    chain_a();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ga, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    chain_c();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&gc, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    report("d  memcpy, graph(a), sync", wall([&] {
      memcpy(pin, host.data(), nin); CK(hipGraphLaunch(ga, st)); CK(hipStreamSynchronize(st)); }));
    check("d");
    report("e  memcpy, graph(c), sync", wall([&] {
      memcpy(pin, host.data(), nin); CK(hipGraphLaunch(gc, st)); CK(hipStreamSynchronize(st)); }));
    check("e");
    CK(hipGraphExecDestroy(ga));
    CK(hipGraphExecDestroy(gc));
    report("k1 alone (device in), sync", wall([&] {
      hipLaunchKernelGGL(k1, dim3(20), dim3(256), 0, st, d_in, d_mid); CK(hipStreamSynchronize(st)); }));
    report("k1 alone (pinned in), sync", wall([&] {
      hipLaunchKernelGGL(k1, dim3(20), dim3(256), 0, st, pin, d_mid); CK(hipStreamSynchronize(st)); }));
  }
  // dependent HBM round trips: a random cycle over 64 MB, one lane
  const int N = 16 << 20;
  std::vector<int> nx(N), perm(N);
  for (int i = 0; i < N; ++i) perm[i] = i;
  uint64_t s = 88172645463325252ull;
  for (int i = N - 1; i > 0; --i) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; std::swap(perm[i], perm[s % (uint64_t)(i + 1)]); }
  for (int i = 0; i < N; ++i) nx[perm[i]] = perm[(i + 1) % N];
  int *d_nx, *d_r;
  CK(hipMalloc(&d_nx, sizeof(int) * N));
  CK(hipMalloc(&d_r, 4));
  CK(hipMemcpy(d_nx, nx.data(), sizeof(int) * N, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int steps : {1, 1000}) {
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0, st));
      hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, st, d_nx, steps, d_r);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
    }
    printf("dependent loads x%-5d: %8.2f us  (%.0f ns per trip)\n", steps, best * 1e3, best * 1e6 / steps);
  }
  return 0;
}
