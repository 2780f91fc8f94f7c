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

#include <type_traits>

#define SDR_MAX_TAPS 256

// Taps passed by value through the kernarg segment: with compile-time tap indices
// (fully unrolled loops) the compiler reads them with s_load into SGPRs, so every
// FMA takes its tap as a scalar operand and no LDS/VGPR space is spent on taps.
struct TapsF32 {
  float h[SDR_MAX_TAPS];
};

// Taps duplicated into (h, h) pairs: a v_pk_fma_f32 then takes the tap pair straight
// from an SGPR pair and updates the (I, Q) accumulator pair in one instruction.
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
struct TapsF2 {
  f2v h[SDR_MAX_TAPS];
};

// acc += {h, h} * x with h = the low (HI=false) or high (HI=true) half of the tap pair:
// one v_pk_fma_f32 broadcasting a half through op_sel, so tap pairs are never duplicated
// into extra registers.  (No hazards: VALU -> VALU.)
template <bool HI>
__device__ __forceinline__ void pk_fma_bcast(f2v& acc, const f2v& tap2, const f2v& x) {
  if (HI)
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(tap2), "v"(x));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]" : "+v"(acc) : "v"(tap2), "v"(x));
}

// acc += tap2 * {x, x} with x = the low (HI=false) or high (HI=true) half of x2: the
// mirror of pk_fma_bcast, broadcasting the sample instead of the tap (two filters, or two
// outputs of one filter, per sample).
template <bool HI>
__device__ __forceinline__ void pk_fma_bcast_x(f2v& acc, const f2v& tap2, const f2v& x2) {
  if (HI)
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(tap2), "v"(x2));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[1,0,1]" : "+v"(acc) : "v"(tap2), "v"(x2));
}

// ds_read_b128 issued by hand: hipcc neither splits it (into ds_read2_b64, whose 32-bank
// mapping is conflict-prone for strided lane windows) nor counts it, so every use must be
// preceded by lds_wait<N> naming the destination (N = LDS reads issued after it).
template <int OFF>
__device__ __forceinline__ f4v lds_read_b128(const void* lds_base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16-bit");
  f4v v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)lds_base;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
  return v;
}
// compile-time loop: f(std::integral_constant<int, I>{}) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int N>
__device__ __forceinline__ void lds_wait(f4v& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}

// atan2 for the discriminator: |err| <= ~2.5e-7 rad (2 ulp polynomial on [0, 1] after the
// octant reduction), ~20 VALU instead of ocml's ~40 with its inf/nan handling; exact
// zeros go to atan2f so the IEEE signed-zero results (e.g. atan2(+0, -0) = pi) hold.
__device__ __forceinline__ float fast_atan2f(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float mn = fminf(ax, ay), mx = fmaxf(ax, ay);
  if (!(mx > 0.f) || !(mx < INFINITY)) return atan2f(y, x);   // zeros, inf, nan
  const float rc = __builtin_amdgcn_rcpf(mx);
  float a = mn * rc;
  a = fmaf(fmaf(-mx, a, mn), rc, a);                  // one Newton step: ~0.5 ulp quotient
  const float s = a * a;
  float r = 0.002849547192454338f;
  r = fmaf(r, s, -0.01606736145913601f);
  r = fmaf(r, s, 0.04268963634967804f);
  r = fmaf(r, s, -0.0750415101647377f);
  r = fmaf(r, s, 0.1064087525010109f);
  r = fmaf(r, s, -0.1420363187789917f);
  r = fmaf(r, s, 0.19992618262767792f);
  r = fmaf(r, s, -0.3333307206630707f);
  r = fmaf(r, s, 1.0f);
  r *= a;
  if (ay > ax) r = 1.57079632679489662f - r;
  if (x < 0.f) r = 3.14159265358979324f - r;
  return copysignf(r, y);
}

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
