// Tuning harness (not part of the product): times fe_kernel tile shapes and ablations
// (MODE 1 = memory only, MODE 2 = compute only) plus a streaming-read baseline on the
// same buffer, with HIP events.  Build: hipcc --offload-arch=gfx950 -O3 tools/fe_tune.hip
#include "../real-time-software-defined-radio_amd/csrc/fe.hip"

#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void read_kernel(const float4* __restrict__ in, int64_t n4, float* out) {
  float acc = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 v = in[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

__global__ void read_chunks(const float4* __restrict__ in, int64_t n4, float* out) {
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / 64);
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int64_t per = (n4 + nw - 1) / nw;
  float acc = 0.f;
  for (int64_t i = w * per + (threadIdx.x & 63); i < (w + 1) * per && i < n4; i += 64) {
    float4 v = in[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 1234.5f) out[0] = acc;
}

__global__ void copy_kernel(const float4* __restrict__ in, int64_t n4, float4* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

template <int R, int NT, int MODE>
float time_fe(FeParams p, const TapsF32& taps, hipStream_t st, int iters) {
  constexpr int TO = NT * R;
  const int64_t M = (p.n + 9) / 10;
  p.tiles_per_stream = (int)((M + TO - 1) / TO);
  p.vec_out = 1;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((fe_kernel<101, 10, R, NT, false, MODE>), dim3(p.tiles_per_stream), dim3(NT), 0, st, p, taps);
  CK(hipEventRecord(a, st));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((fe_kernel<101, 10, R, NT, false, MODE>), dim3(p.tiles_per_stream), dim3(NT), 0, st, p, taps);
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

template <int R, int NB, int MODE>
float time_fs(FeParams p, const TapsF32& taps, hipStream_t st, int iters, int waves_per_cu) {
  constexpr int TO = 64 * R;
  const int64_t M = (p.n + 9) / 10;
  p.tiles_per_stream = (int)((M + TO - 1) / TO);
  p.vec_out = 1;
  const int64_t total = (int64_t)p.tiles_per_stream * p.nstreams;
  int grid = 256 * waves_per_cu;
  if (grid > total) grid = (int)total;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((fe_stream_kernel<101, 10, R, NB, MODE>), dim3(grid), dim3(64), 0, st, p, taps, total);
  CK(hipEventRecord(a, st));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((fe_stream_kernel<101, 10, R, NB, MODE>), dim3(grid), dim3(64), 0, st, p, taps, total);
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  CK(hipGetLastError());
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

template <int MODE>
float time_ring(FeParams p, const TapsF32& taps, hipStream_t st, int iters, int waves_per_cu) {
  const int64_t M = (p.n + 9) / 10;
  RingArgs ra;
  ra.tps = (int)((M + 191) / 192);
  ra.total = (int64_t)ra.tps * p.nstreams;
  const int64_t slots = 256LL * waves_per_cu;
  ra.per_wave = (int)((ra.total + slots - 1) / slots);
  const int grid = (int)((ra.total + ra.per_wave - 1) / ra.per_wave);
  p.tiles_per_stream = ra.tps;
  p.vec_out = 1;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((fe_ring_kernel<101, false, MODE>), dim3(grid), dim3(64), 0, st, p, taps, ra);
  CK(hipEventRecord(a, st));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((fe_ring_kernel<101, false, MODE>), dim3(grid), dim3(64), 0, st, p, taps, ra);
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  CK(hipGetLastError());
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

template <int MODE>
float time_ring_fused(FeParams p, const TapsF32& taps, const float* ataps, float* audio, hipStream_t st, int iters) {
  const int64_t M = (p.n + 9) / 10;
  RingArgs ra{};
  ra.ab = (int)((M + 959) / 960);
  ra.tps = 5 * ra.ab;
  ra.total = (int64_t)ra.ab * p.nstreams;
  ra.audio = audio; ra.audio_stride = (M + 4) / 5; ra.ataps = ataps;
  const int64_t slots = 256LL * 4;
  ra.per_wave = (int)((ra.total + slots - 1) / slots);
  const int grid = (int)((ra.total + ra.per_wave - 1) / ra.per_wave);
  p.tiles_per_stream = ra.tps;
  p.demod = nullptr;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((fe_ring_kernel<101, true, MODE>), dim3(grid), dim3(64), 0, st, p, taps, ra);
  CK(hipEventRecord(a, st));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((fe_ring_kernel<101, true, MODE>), dim3(grid), dim3(64), 0, st, p, taps, ra);
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  CK(hipGetLastError());
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

template <bool FUSED, int MODE>
float time_circ(FeParams p, const TapsF32& taps, const float* ataps, float* audio, hipStream_t st, int iters) {
  const int64_t M = (p.n + 9) / 10;
  RingArgs ra{};
  if (FUSED) { ra.ab = (int)((M + 319) / 320); ra.tps = 5 * ra.ab; ra.total = (int64_t)ra.ab * p.nstreams; }
  else { ra.tps = (int)((M + 63) / 64); ra.total = (int64_t)ra.tps * p.nstreams; }
  ra.audio = audio; ra.audio_stride = (M + 4) / 5; ra.ataps = ataps;
  const int64_t slots = 256LL * 4;
  ra.per_wave = (int)((ra.total + slots - 1) / slots);
  const int grid = (int)((ra.total + ra.per_wave - 1) / ra.per_wave);
  p.tiles_per_stream = ra.tps;
  if (FUSED) p.demod = nullptr;
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i)
    hipLaunchKernelGGL((fe_circ_kernel<101, FUSED, MODE>), dim3(grid), dim3(64), 0, st, p, taps, ra);
  CK(hipEventRecord(a, st));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL((fe_circ_kernel<101, FUSED, MODE>), dim3(grid), dim3(64), 0, st, p, taps, ra);
  CK(hipEventRecord(b, st));
  CK(hipEventSynchronize(b));
  CK(hipGetLastError());
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char** argv) {
  const int64_t n = 64LL * 1024000;  // complex samples
  const int64_t M = n / 10;
  float *iq, *out;
  CK(hipMalloc(&iq, n * 8));
  CK(hipMalloc(&out, n * 8));
  std::vector<float> h(2 * n);
  for (int64_t i = 0; i < 2 * n; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(iq, h.data(), n * 8, hipMemcpyHostToDevice));
  hipStream_t st; CK(hipStreamCreate(&st));
  TapsF32 taps{}; for (int k = 0; k < 101; ++k) taps.h[k] = 0.01f * (k % 7);
  float* tdev; CK(hipMalloc(&tdev, 1024)); CK(hipMemcpy(tdev, taps.h, 1024, hipMemcpyHostToDevice));
  FeParams p{};
  p.iq = iq; p.n = n; p.stride = n; p.hist = 0; p.nstreams = 1; p.taps_dev = tdev; p.demod = out; p.out_stride = M;
  const double bytes = n * 8.0 + M * 4.0;
  const int it = 20;
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int grid : {2048}) {
    hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, st, (const float4*)iq, n * 8 / 16, out);
    CK(hipEventRecord(a, st));
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL(read_kernel, dim3(grid), dim3(256), 0, st, (const float4*)iq, n * 8 / 16, out);
    CK(hipEventRecord(b, st)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= it;
    printf("read-only  grid %5d: %8.2f us  %7.1f GB/s\n", grid, ms * 1e3, n * 8.0 / ms / 1e6);
    CK(hipEventRecord(a, st));
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, st, (const float4*)iq, n * 8 / 32, (float4*)out);
    CK(hipEventRecord(b, st)); CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b)); ms /= it;
    printf("copy(half) grid %5d: %8.2f us  %7.1f GB/s\n", grid, ms * 1e3, n * 8.0 / ms / 1e6);
    for (int wg : {64, 256}) {
      int g2 = wg == 64 ? 1024 : 1024;
      CK(hipEventRecord(a, st));
      for (int i = 0; i < it; ++i) hipLaunchKernelGGL(read_chunks, dim3(g2), dim3(wg), 0, st, (const float4*)iq, n * 8 / 16, out);
      CK(hipEventRecord(b, st)); CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b)); ms /= it;
      printf("read-chunks %d WGs x %d thr (one contiguous region per wave): %8.2f us  %7.1f GB/s\n", g2, wg, ms * 1e3, n * 8.0 / ms / 1e6);
    }
  }
  const char* sel = argc > 1 ? argv[1] : "all";
  auto want = [&](const char* k) { return !strcmp(sel, "all") || strstr(sel, k) != nullptr; };
#define RUN(R, NT) if (want("old")) { \
    float t0 = time_fe<R, NT, 0>(p, taps, st, it), t1 = time_fe<R, NT, 1>(p, taps, st, it), t2 = time_fe<R, NT, 2>(p, taps, st, it); \
    printf("fe   R=%d NT=%3d: full %8.2f us (%7.1f GB/s)  mem-only %8.2f us  compute-only %8.2f us\n", R, NT, t0 * 1e3, bytes / t0 / 1e6, t1 * 1e3, t2 * 1e3); }
  RUN(4, 128)
#define RUNW(R, TS, tag) if (want(tag)) { \
    float t0 = time_few<R, 0, TS>(p, taps, st, it), t1 = time_few<R, 1, TS>(p, taps, st, it), t2 = time_few<R, 2, TS>(p, taps, st, it); \
    printf("wave R=%d ts=%d  : full %8.2f us (%7.1f GB/s)  mem-only %8.2f us  compute-only %8.2f us\n", R, TS, t0 * 1e3, bytes / t0 / 1e6, t1 * 1e3, t2 * 1e3); }
#define RUNS(R, NB, W, tag) if (want(tag)) { \
    float t0 = time_fs<R, NB, 0>(p, taps, st, it, W), t1 = time_fs<R, NB, 1>(p, taps, st, it, W), t2 = time_fs<R, NB, 2>(p, taps, st, it, W); \
    float t3 = time_fs<R, NB, 3>(p, taps, st, it, W); \
    printf("strm R=%d NB=%d w/cu=%d: full %8.2f us (%7.1f GB/s)  mem-only %8.2f us  compute-only %8.2f us  mem-no-epilogue %8.2f us\n", R, NB, W, t0 * 1e3, bytes / t0 / 1e6, t1 * 1e3, t2 * 1e3, t3 * 1e3); }
  RUNS(3, 2, 4, "s324") RUNS(2, 2, 7, "s227") RUNS(2, 2, 6, "s226") RUNS(3, 3, 3, "s333") RUNS(2, 3, 5, "s235") RUNS(1, 2, 12, "s1212")
#define RUNR(W, tag) if (want(tag)) { \
    float t0 = time_ring<0>(p, taps, st, it, W), t1 = time_ring<1>(p, taps, st, it, W), t2 = time_ring<2>(p, taps, st, it, W); \
    printf("ring R=3 NB=2 w/cu=%d: full %8.2f us (%7.1f GB/s)  mem-only %8.2f us  compute-only %8.2f us\n", W, t0 * 1e3, bytes / t0 / 1e6, t1 * 1e3, t2 * 1e3); }
  RUNR(4, "r4") RUNR(3, "r3") RUNR(2, "r2")
  if (want("circ")) {
    float* aud; CK(hipMalloc(&aud, (M / 5 + 64) * 4));
    float f0 = time_circ<false, 0>(p, taps, tdev, aud, st, it), f1 = time_circ<false, 1>(p, taps, tdev, aud, st, it);
    float f4 = time_circ<false, 4>(p, taps, tdev, aud, st, it);
    printf("circ FE   : full %8.2f us (%7.1f GB/s)  no-FIR %8.2f us  DMA only %8.2f us\n", f0 * 1e3, bytes / f0 / 1e6, f1 * 1e3, f4 * 1e3);
    float g0 = time_circ<true, 0>(p, taps, tdev, aud, st, it), g1 = time_circ<true, 1>(p, taps, tdev, aud, st, it);
    float g4 = time_circ<true, 4>(p, taps, tdev, aud, st, it);
    const double fb = n * 8.0 + (M / 5) * 4.0;
    printf("circ fused: full %8.2f us (%7.1f GB/s)  no-FIR %8.2f us  DMA only %8.2f us\n", g0 * 1e3, fb / g0 / 1e6, g1 * 1e3, g4 * 1e3);
  }
  if (want("fused")) {
    float* aud; CK(hipMalloc(&aud, (M / 5 + 64) * 4));
    float t0 = time_ring_fused<0>(p, taps, tdev, aud, st, it), t1 = time_ring_fused<1>(p, taps, tdev, aud, st, it);
    float t4 = time_ring_fused<4>(p, taps, tdev, aud, st, it), t5 = time_ring_fused<5>(p, taps, tdev, aud, st, it);
    const double fb = n * 8.0 + (M / 5) * 4.0;
    printf("ring fused FE+mono: full %8.2f us (%7.1f GB/s)  no-FIR %8.2f us  DMA+halo only %8.2f us  DMA(16 chunks) only %8.2f us\n",
           t0 * 1e3, fb / t0 / 1e6, t1 * 1e3, t4 * 1e3, t5 * 1e3);
    uint64_t* dbg; CK(hipMalloc(&dbg, 8 * 8 * 4096));
    p.q_ds = reinterpret_cast<float*>(dbg);
    float t6 = time_ring_fused<6>(p, taps, tdev, aud, st, 1);
    std::vector<uint64_t> hd(8 * 4096); CK(hipMemcpy(hd.data(), dbg, 8 * 8 * 4096, hipMemcpyDeviceToHost));
    double acc[6] = {0, 0, 0, 0, 0, 0}; int nw = 0;
    for (int w = 0; w < 1024; ++w) { if (!hd[8 * w + 5]) continue; ++nw; for (int k = 0; k < 6; ++k) acc[k] += (double)hd[8 * w + k]; }
    printf("instrumented %8.2f us; per wave-tile cycles: issue %.0f  wait/build %.0f  halo+FIR %.0f  epilogue %.0f  audio %.0f  (tiles/wave %.1f)\n",
           t6 * 1e3, acc[0] / acc[5], acc[1] / acc[5], acc[2] / acc[5], acc[3] / acc[5], acc[4] / acc[5], acc[5] / nw);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
