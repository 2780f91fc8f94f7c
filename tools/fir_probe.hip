// FIR-loop probe (tuning only): throughput of fe_fir_tile<101,10,R> on an LDS-resident
// tile image, with and without the atan2/DPP epilogue math, at W waves per CU.
// Isolates the per-tile FIR cost from DMA, waits and index math.
#include "../real-time-software-defined-radio_amd/csrc/fe.hip"
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int R, int EPI>
__global__ __launch_bounds__(64) void fir_probe(TapsF32 taps, int tiles, float* out) {
  constexpr int T = 101, D = 10, TO = 64 * R;
  constexpr int L = ((D * TO + T + 1) + 127) / 128 * 128;
  __shared__ __attribute__((aligned(16))) f2v buf[L + 2];
  const int lane = threadIdx.x;
  for (int e = lane; e < L + 2; e += 64) buf[e] = f2v{(float)e * 1e-3f, (float)(e & 7)};
  __syncthreads();
  f2v tp[(T + 1) / 2];
#pragma unroll
  for (int j = 0; j < (T + 1) / 2; ++j) tp[j] = f2v{taps.h[2 * j], (2 * j + 1 < T) ? taps.h[2 * j + 1] : 0.f};
#pragma unroll
  for (int j = 0; j < (T + 1) / 2; ++j) asm volatile("" : "+v"(tp[j]));
  float sum = 0.f, carry = 0.f;
  for (int t = 0; t < tiles; ++t) {
    float ai[R], aq[R];
    fe_fir_tile<T, D, R, 0>(buf, lane, tp, ai, aq);
    if (EPI) {
      float phi[R];
#pragma unroll
      for (int r = 0; r < R; ++r) phi[r] = fast_atan2f(aq[r], ai[r]);
      const float fl = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(phi[R - 1]), 0x138, 0xf, 0xf, false));
      float prev = lane == 0 ? carry : fl;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float dd = phi[r] - prev;
        if (dd > 3.14159265f) dd -= 6.2831853f; else if (dd < -3.14159265f) dd += 6.2831853f;
        sum += dd;
        prev = phi[r];
      }
      carry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[R - 1]), 63));
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) sum += ai[r] + aq[r];
    }
  }
  out[blockIdx.x * 64 + lane] = sum;
}

template <int R, int EPI>
void run(int wpc, const TapsF32& taps, float* out) {
  const int total_outputs = 6553600;                      // 65.5 M complex / 10
  const int grid = 256 * wpc;
  const int tiles = (total_outputs / (64 * R) + grid - 1) / grid;
  hipLaunchKernelGGL((fir_probe<R, EPI>), dim3(grid), dim3(64), 0, 0, taps, tiles, out);
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((fir_probe<R, EPI>), dim3(grid), dim3(64), 0, 0, taps, tiles, out);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); CK(hipGetLastError());
  float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 5;
  printf("R=%d epi=%d waves/CU=%2d tiles/wave=%4d: %8.2f us for 6.55M outputs\n", R, EPI, wpc, tiles, ms * 1e3);
}

int main() {
  TapsF32 taps{}; for (int k = 0; k < 101; ++k) taps.h[k] = 0.01f * (k % 7);
  float* out; CK(hipMalloc(&out, 256 * 16 * 64 * 4));
  for (int w : {4, 8, 12}) { run<1, 0>(w, taps, out); run<1, 1>(w, taps, out); }
  for (int w : {4, 7, 8}) { run<2, 0>(w, taps, out); run<2, 1>(w, taps, out); }
  for (int w : {4, 5}) { run<3, 0>(w, taps, out); run<3, 1>(w, taps, out); }
  return 0;
}
