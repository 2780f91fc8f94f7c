// VALU issue probe (tuning only): cycles per wave-instruction of v_pk_fma_f32 vs v_fma_f32
// at 1/2/4 waves per SIMD and different numbers of independent accumulator chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f2v __attribute__((ext_vector_type(2)));

template <int CH, bool PK>
__global__ __launch_bounds__(64) void probe(float* out, long long* cyc, int iters) {
  f2v acc[CH];
  f2v t = f2v{1.0001f + threadIdx.x * 1e-7f, 0.9999f};
  f2v x = f2v{0.5f, 0.25f + threadIdx.x * 1e-6f};
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = f2v{(float)c, (float)-c};
  long long t0 = __builtin_readcyclecounter();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 64 / CH; ++u)
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        if (PK)
          asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc[c]) : "v"(t), "v"(x));
        else
          asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc[c].x) : "v"(t.x), "v"(x.x));
      }
  }
  long long t1 = __builtin_readcyclecounter();
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c].x + acc[c].y;
  out[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH, bool PK>
void run(int wps, int cus) {
  const int grid = cus * 4 * wps, iters = 2000;
  float* out; long long* cyc;
  hipMalloc(&out, grid * 64 * 4); hipMalloc(&cyc, grid * 8);
  hipLaunchKernelGGL((probe<CH, PK>), dim3(grid), dim3(64), 0, 0, out, cyc, iters);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<CH, PK>), dim3(grid), dim3(64), 0, 0, out, cyc, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<long long> c(grid); hipMemcpy(c.data(), cyc, grid * 8, hipMemcpyDeviceToHost);
  double avg = 0; for (auto v : c) avg += v; avg /= grid;
  const double ninst = (double)iters * 64;
  printf("%s chains=%2d waves/SIMD=%d: %.2f cyc per wave-instr (s_memtime-ish counter), kernel %.3f ms, "
         "%.2f ns per instr per SIMD\n", PK ? "pk_fma" : "fma   ", CH, wps, avg / ninst, ms,
         ms * 1e6 / (ninst * wps));
  hipFree(out); hipFree(cyc);
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  for (int w : {1, 2, 4}) {
    run<2, true>(w, cus); run<4, true>(w, cus); run<8, true>(w, cus); run<16, true>(w, cus);
    run<2, false>(w, cus); run<4, false>(w, cus); run<8, false>(w, cus); run<16, false>(w, cus);
  }
  return 0;
}
