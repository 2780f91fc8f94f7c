// Memory-pipeline probes (not part of the product): how fast can a workgroup pattern
// pull a 524 MB stream through registers / LDS on MI355X?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// each WG loads NL float4 per thread (one contiguous chunk) and exits
template <int NT, int NL, bool TO_LDS>
__global__ __launch_bounds__(NT) void wg_load(const float4* __restrict__ in, float* out) {
  __shared__ float4 lds[TO_LDS ? NT * NL : 1];
  const float4* p = in + (int64_t)blockIdx.x * NT * NL + threadIdx.x;
  float4 v[NL];
#pragma unroll
  for (int j = 0; j < NL; ++j) v[j] = p[j * NT];
  float acc = 0.f;
  if (TO_LDS) {
#pragma unroll
    for (int j = 0; j < NL; ++j) lds[j * NT + threadIdx.x] = v[j];
    __syncthreads();
    acc = lds[(threadIdx.x * 7) % (NT * NL)].x;
  } else {
#pragma unroll
    for (int j = 0; j < NL; ++j) acc += v[j].x + v[j].w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

// each wave issues NL LDS-DMA loads (1 KB each) of its chunk and waits
template <int NL>
__global__ __launch_bounds__(64) void wave_glds(const float* __restrict__ in, float* out) {
  __shared__ __attribute__((aligned(16))) float lds[NL * 256];
  const float* p = in + (int64_t)blockIdx.x * NL * 256 + 4 * threadIdx.x;
#pragma unroll
  for (int j = 0; j < NL; ++j)
    __builtin_amdgcn_global_load_lds(p + 256 * j, (__attribute__((address_space(3))) void*)(lds + 256 * j), 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const float a = lds[(threadIdx.x * 5) % (NL * 256)];
  if (a == 1234.5f) out[0] = a;
}

// persistent: each wave streams tiles of NL KB round-robin through an NB-deep LDS ring
// CONTIG: each wave takes a contiguous run of tiles (else round robin); STEP < NL*256:
// tiles overlap (halo re-read); WR: each tile also writes WR floats per lane
template <int NL, int NB, bool CONTIG = false, int STEP = NL * 256, int WR = 0, int AUX = 0, int DELAY = 0>
__global__ __launch_bounds__(64) void ring_glds(const float* __restrict__ in, int64_t ntiles, float* out) {
  __shared__ __attribute__((aligned(16))) float lds[NB * NL * 256];
  const int lane = threadIdx.x;
  const int64_t G = gridDim.x;
  const int64_t mine = CONTIG ? ((blockIdx.x + 1) * ntiles / G - blockIdx.x * ntiles / G) : (ntiles - blockIdx.x + G - 1) / G;
  const int64_t first = blockIdx.x * ntiles / G;
  auto tile = [&](int64_t u) { return CONTIG ? first + u : blockIdx.x + u * G; };
  auto issue = [&](int64_t u) {
    const float* p = in + tile(u) * STEP + 4 * lane;
    float* d = lds + (u % NB) * NL * 256;
#pragma unroll
    for (int j = 0; j < NL; ++j)
      __builtin_amdgcn_global_load_lds(p + 256 * j, (__attribute__((address_space(3))) void*)(d + 256 * j), 16, 0, AUX);
  };
  float acc = 0.f;
  float acc8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t u = 0; u < NB - 1 && u < mine; ++u) issue(u);
  for (int64_t u = 0; u < mine; ++u) {
    constexpr int S = WR == 2 ? 2 : (WR == 3 || WR == 9) ? 1 : WR == 4 ? 2 : (WR >= 6 && WR <= 8) ? 1 : 0;   // stores per tile (exact)
    if (u + NB - 1 < mine) {
      issue(u + NB - 1);
      if (u > 0 && S > 0 && WR != 5) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NL * (NB - 1) + S) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NL * (NB - 1)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    acc += lds[(u % NB) * NL * 256 + lane * 4];
    if (DELAY > 0) {                 // synthetic per-tile compute: DELAY independent-ish FMAs
      float x0 = acc, x1 = acc + 1.f, x2 = acc + 2.f, x3 = acc + 3.f;
      for (int k = 0; k < DELAY; ++k) {
        asm volatile("v_fma_f32 %0, %0, %0, %0\n\tv_fma_f32 %1, %1, %1, %1\n\tv_fma_f32 %2, %2, %2, %2\n\tv_fma_f32 %3, %3, %3, %3"
                     : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
      }
      acc += x0 + x1 + x2 + x3;
    }
    if (WR == 2) {
#pragma unroll
      for (int w = 0; w < WR; ++w) out[(tile(u) * 64 + lane) * WR + w] = acc;
    } else if (WR == 9) {          // one float2 store per lane, always to the wave's own 512 B (L2-resident)
      reinterpret_cast<float2*>(out)[blockIdx.x * 64 + lane] = make_float2(acc, acc + 1.f);
    } else if (WR == 3) {          // one float2 store per lane
      reinterpret_cast<float2*>(out)[tile(u) * 64 + lane] = make_float2(acc, acc + 1.f);
    } else if (WR == 4) {          // one nontemporal float2 store per lane
      __builtin_nontemporal_store(make_float2(acc, acc + 1.f).x, out + 2 * (tile(u) * 64 + lane));
      __builtin_nontemporal_store(acc + 1.f, out + 2 * (tile(u) * 64 + lane) + 1);
    } else if (WR >= 6 && WR <= 8) {   // float2 store with explicit cache policy bits
      float2 v = make_float2(acc, acc + 1.f);
      float2* a = reinterpret_cast<float2*>(out) + tile(u) * 64 + lane;
      if (WR == 6) asm volatile("global_store_dwordx2 %0, %1, off sc1\n\ts_nop 1" :: "v"(a), "v"(v) : "memory");
      if (WR == 7) asm volatile("global_store_dwordx2 %0, %1, off nt\n\ts_nop 1" :: "v"(a), "v"(v) : "memory");
      if (WR == 8) asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1 nt\n\ts_nop 1" :: "v"(a), "v"(v) : "memory");
    } else if (WR == 5) {          // batch: every 8th tile, 8 tiles' worth (4 KB per wave) as float4s
      acc8[u % 8] = acc;
      if (u % 8 == 7) {
        float4* o = reinterpret_cast<float4*>(out) + (tile(u) / 8) * 256 + lane;
#pragma unroll
        for (int w = 0; w < 4; ++w) o[64 * w] = make_float4(acc8[2 * w], acc8[2 * w], acc8[2 * w + 1], acc8[2 * w + 1]);
      }
    }
  }
  if (acc == 1234.5f) out[0] = acc;
}

__global__ __launch_bounds__(64) void write_only(float* out, int64_t ntiles) {
  const int lane = threadIdx.x;
  const int64_t G = gridDim.x;
  const int64_t first = blockIdx.x * ntiles / G, last = (blockIdx.x + 1) * ntiles / G;
  for (int64_t t = first; t < last; ++t) reinterpret_cast<float2*>(out)[t * 64 + lane] = make_float2(1.f, 2.f);
}

int main(int argc, char** argv) {
  const int64_t bytes = 64LL * 1024000 * 8;
  float *in, *out;
  CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes / 8));
  CK(hipMemset(in, 0, bytes));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipEventRecord(a, st));
    for (int i = 0; i < 20; ++i) launch();
    CK(hipEventRecord(b, st)); CK(hipEventSynchronize(b)); CK(hipGetLastError());
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 20;
    printf("%-60s %8.2f us %7.1f GB/s\n", name, ms * 1e3, bytes / ms / 1e6);
  };
  const int64_t n4 = bytes / 16;
#define WGL(NT, NL, L) timeit("wg_load NT=" #NT " NL=" #NL " lds=" #L, [&] { \
    hipLaunchKernelGGL((wg_load<NT, NL, L>), dim3(n4 / (NT * NL)), dim3(NT), 0, st, (const float4*)in, out); });
  WGL(64, 16, false) WGL(64, 16, true) WGL(128, 21, false) WGL(128, 21, true) WGL(256, 8, false) WGL(256, 8, true)
  WGL(256, 16, false) WGL(256, 16, true) WGL(64, 4, false) WGL(256, 4, false)
#define WGD(NL) timeit("wave_glds NL=" #NL, [&] { \
    hipLaunchKernelGGL((wave_glds<NL>), dim3(bytes / (NL * 1024)), dim3(64), 0, st, in, out); });
  WGD(4) WGD(8) WGD(16) WGD(32)
#define RING(NL, NB, W) timeit("ring_glds NL=" #NL " NB=" #NB " waves/cu=" #W, [&] { \
    hipLaunchKernelGGL((ring_glds<NL, NB>), dim3(256 * W), dim3(64), 0, st, in, bytes / (NL * 1024), out); });
  timeit("write_only 512 B per wave-tile, contiguous per wave (26 MB)", [&] {
    hipLaunchKernelGGL(write_only, dim3(256 * 7), dim3(64), 0, st, out, (bytes - 11 * 1024) / (2560 * 4)); });
  RING(16, 2, 4) RING(11, 2, 7)
#define RING2(NL, NB, W, C, STEP, WR) timeit("ring_glds NL=" #NL " NB=" #NB " w/cu=" #W " contig=" #C " step=" #STEP " wr=" #WR, [&] { \
    hipLaunchKernelGGL((ring_glds<NL, NB, C, STEP, WR>), dim3(256 * W), dim3(64), 0, st, in, (bytes - NL * 1024) / (STEP * 4), out); });
  RING2(11, 2, 7, true, 2560, 0) RING2(11, 2, 7, true, 2560, 3) RING2(11, 2, 7, false, 2560, 3)
#define RING3(NL, NB, W, C, STEP, WR, AUX) timeit("ring_glds NL=" #NL " NB=" #NB " w/cu=" #W " contig=" #C " step=" #STEP " wr=" #WR " aux=" #AUX, [&] { \
    hipLaunchKernelGGL((ring_glds<NL, NB, C, STEP, WR, AUX>), dim3(256 * W), dim3(64), 0, st, in, (bytes - NL * 1024) / (STEP * 4), out); });
  RING3(11, 2, 7, true, 2560, 0, 2) RING3(11, 2, 7, true, 2560, 3, 2)
  RING3(11, 2, 7, true, 2560, 6, 2) RING3(11, 2, 7, true, 2560, 7, 2) RING3(11, 2, 7, true, 2560, 8, 2)
  RING3(11, 2, 7, false, 2560, 6, 2) RING3(11, 2, 7, true, 2560, 6, 0)
  RING3(16, 2, 4, true, 3840, 0, 2) RING3(16, 2, 4, true, 3840, 3, 2) RING3(16, 2, 4, true, 3840, 9, 2)
  RING3(16, 2, 4, true, 3840, 5, 2) RING3(11, 2, 7, true, 2560, 9, 2) RING3(11, 2, 7, true, 2560, 5, 2)
#define RINGD(NL, NB, W, STEP, DL) timeit("ring_glds NL=" #NL " NB=" #NB " w/cu=" #W " step=" #STEP " aux=2 delay=" #DL "x4 fma", [&] { \
    hipLaunchKernelGGL((ring_glds<NL, NB, true, STEP, 0, 2, DL>), dim3(256 * W), dim3(64), 0, st, in, (bytes - NL * 1024) / (STEP * 4), out); });
  RINGD(16, 2, 4, 3840, 0) RINGD(16, 2, 4, 3840, 100) RINGD(16, 2, 4, 3840, 200) RINGD(16, 2, 4, 3840, 400) RINGD(16, 2, 4, 3840, 800)
  RINGD(16, 3, 3, 3840, 0) RINGD(16, 3, 3, 3840, 200) RINGD(16, 3, 3, 3840, 400)
  RINGD(6, 3, 8, 1280, 0) RINGD(6, 3, 8, 1280, 67) RINGD(6, 3, 8, 1280, 133) RINGD(6, 2, 8, 1280, 67) RINGD(6, 2, 8, 1280, 133)
  return 0;
}
