// Shared device-side definitions for the MI355X FM-SDR hot path (gfx950 only).
//
// Data layout in HBM:
//   * IQ input: interleaved [I0,Q0,I1,Q1,...] per stream, f32 (8 B / complex sample)
//     or u8 (2 B / complex sample, value (u8-128)/128 as src/iofunc.cpp:61-69 and
//     model/fmRDSblock.py:58-59).  Streams are `stream_stride` complex samples apart.
//   * Real-valued channel streams (demod, audio, stereo, RDS): f32, `stride` apart.
//   * Filter state follows scipy.signal.lfilter's `zi` convention:
//     y[n] = (b*x)[n] + zi[n] for n < taps-1; it is added to the f32 accumulator.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SDR_MAX_TAPS 256

// Taps passed by value through the kernarg segment: with compile-time tap indices
// (fully unrolled loops) the compiler reads them with s_load into SGPRs, so every
// FMA takes its tap as a scalar operand and no LDS/VGPR space is spent on taps.
struct TapsF32 {
  float h[SDR_MAX_TAPS];
};

// Wave-wide sum over 64 lanes (CDNA wave64: six xor steps).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// XCD-aware tile order: hardware deals workgroups round-robin over the 8 XCDs
// (MI355X_MICROARCH.md §Workgroup dispatch), so block b and b+8 share an L2.
// Remap so each XCD walks a contiguous run of tiles: neighbouring tiles share
// their (taps-1)-sample input halo, which then hits in the same L2.
// Speed only; correctness never depends on placement.
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t nblocks) {
  if (nblocks < 64 || (nblocks & 7)) return b;
  const int64_t per = nblocks >> 3;
  return (b & 7) * per + (b >> 3);
}
