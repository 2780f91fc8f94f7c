// Probe (not product): HBM streaming through a per-wave VGPR stage, the memory pipeline
// of fe_slot_kernel without its compute.  Each wave streams a contiguous run of 15-KiB
// tiles: wait for the stage, optionally write it to LDS (16 x ds_write_b128), reissue.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stage_probe.hip -o tools/stage_probe
#include "../real-time-software-defined-radio_amd/csrc/sdr_common.h"
#include <algorithm>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// WR: write the stage to LDS each tile; NS: stages (tiles in flight, 1 or 2)
template <bool WR, int NS, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
void stage_stream(const char* in, int64_t ntiles, float* out) {
  constexpr int NC = 15;
  __shared__ __attribute__((aligned(16))) f4v lds[16 * 64];
  const int lane = threadIdx.x;
  const int64_t G = gridDim.x;
  const int64_t t0 = blockIdx.x * ntiles / G, t1 = (blockIdx.x + 1) * ntiles / G;
  const unsigned voff = 16u * lane;
  f4v st[NS][NC];
  auto load = [&](auto S, int64_t t) {
    const char* g = in + t * 15360;
    static_for<0, NC>([&](auto C) {
      constexpr int c = C;
      gload16_nt_v<1024 * (c % 4)>(st[S][c], voff, g + 4096 * (c / 4));
    });
  };
  float acc = 0.f;
  const unsigned la = lds_addr_of(lds) + 16u * lane;
  if (t0 < t1) load(std::integral_constant<int, 0>{}, t0);
  if (NS == 2 && t0 + 1 < t1) load(std::integral_constant<int, NS - 1>{}, t0 + 1);
  for (int64_t t = t0; t < t1; t += NS) {
    static_for<0, NS>([&](auto S) {
      constexpr int sq = S;
      if (t + sq < t1) {
        if (NS == 2 && t + sq + 1 < t1) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        static_for<0, NC>([&](auto C) {
          constexpr int c = C;
          asm volatile("" : "+v"(st[sq][c]));
          if constexpr (WR) lds_write_b128_v<1024 * c>(la, st[sq][c]);
          else acc += st[sq][c].x;
        });
        if (t + sq + NS < t1) load(std::integral_constant<int, sq>{}, t + sq + NS);
      }
    });
  }
  if (WR) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); acc += reinterpret_cast<float*>(lds)[lane * 7]; }
  if (acc == 1234.5f) out[0] = acc;
}

int main() {
  const int64_t bytes = 64LL * 1024000 * 8;
  const int64_t ntiles = bytes / 15360 - 1;
  char* in; float* out;
  CK(hipMalloc(&in, bytes + 65536)); CK(hipMalloc(&out, 1024));
  CK(hipMemset(in, 1, bytes));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  struct V { const char* name; void (*f)(const char*, int64_t, float*, hipStream_t); std::vector<float> us; };
#define VV(NAME, WR, NS, WPE, W) {NAME, [](const char* i, int64_t n, float* o, hipStream_t s) { \
    hipLaunchKernelGGL((stage_stream<WR, NS, WPE>), dim3(256 * W), dim3(64), 0, s, i, n, o); }, {}}
  std::vector<V> v = {
    VV("stage1 wr   w8", true, 1, 2, 8), VV("stage1 nowr w8", false, 1, 2, 8),
    VV("stage1 wr   w4", true, 1, 1, 4), VV("stage1 nowr w4", false, 1, 1, 4),
    VV("stage2 wr   w4", true, 2, 1, 4), VV("stage2 nowr w4", false, 2, 1, 4),
    VV("stage1 wr   w6", true, 1, 1, 6), VV("stage1 nowr w2", false, 1, 1, 2),
  };
  for (auto& x : v) for (int i = 0; i < 3; ++i) x.f(in, ntiles, out, st);
  for (int i = 0; i < 300; ++i) v[0].f(in, ntiles, out, st);
  CK(hipStreamSynchronize(st));
  for (int r = 0; r < 6; ++r)
    for (auto& x : v) {
      CK(hipEventRecord(a, st));
      for (int i = 0; i < 10; ++i) x.f(in, ntiles, out, st);
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      x.us.push_back(ms * 100.f);
    }
  CK(hipGetLastError());
  for (auto& x : v) {
    std::sort(x.us.begin(), x.us.end());
    const float med = x.us[x.us.size() / 2];
    printf("%-18s median %7.2f us  %7.1f GB/s\n", x.name, med, ntiles * 15360.0 / med / 1e3);
  }
  return 0;
}
