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
#define SDR_MAX_RESAMPLE_TAPS 4096   // resampler (sdr_resample*) filters: taps + zf staging fit 64 KiB of LDS
#define SDR_PSD_MAX_NFFT 4096   // PSD segment length limit: N complex f64 in 64 KiB of LDS

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
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(tap2), "v"(x));
  else
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]" : "+v"(acc) : "v"(tap2), "v"(x));
}

// acc += tap2 * {x, x} with x = the low (HI=false) or high (HI=true) half of x2: the
// mirror of pk_fma_bcast, broadcasting the sample instead of the tap (two filters, or two
// outputs of one filter, per sample).
// Not volatile: its operands come from compiler-visible loads, so the compiler orders and
// waits for them itself (a volatile asm would pin every load of the loop in place).
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
// ds_read2_b32 issued by hand: two dwords at dword offsets O0, O1 (< 256) from base.
template <int O0, int O1>
__device__ __forceinline__ f2v lds_read2_b32(const void* lds_base) {
  static_assert(O0 >= 0 && O0 < 256 && O1 >= 0 && O1 < 256, "8-bit dword offsets");
  f2v v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)lds_base;
  asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3" : "=v"(v) : "v"(a), "i"(O0), "i"(O1));
  return v;
}

// ordered (volatile) scalar FMA for hand-pipelined loops: acc += a * b
__device__ __forceinline__ void fmac_ordered(float& acc, float a, float b) {
  asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(acc) : "v"(a), "v"(b));
}
// ordered variant of pk_fma_bcast_x (for operands from hand-issued LDS reads)
template <bool HI>
__device__ __forceinline__ void pk_fma_bcast_x_ordered(f2v& acc, const f2v& tap2, const f2v& x2) {
  if (HI)
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(tap2), "v"(x2));
  else
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[1,0,1]" : "+v"(acc) : "v"(tap2), "v"(x2));
}

// ordered elementwise packed FMA: acc += a * b (both halves)
__device__ __forceinline__ void pk_fma_ordered(f2v& acc, const f2v& a, const f2v& b) {
  asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

// ds_write_b128 issued by hand (ordered with the hand-issued reads above).
__device__ __forceinline__ void lds_write_b128(void* lds_base, const f4v& v) {
  const unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds_base;
  asm volatile("ds_write_b128 %0, %1" : : "v"(a), "v"(v) : "memory");
}

// 16-B-per-lane non-temporal load into AGPRs (saddr form): the caller owns vmcnt.  AGPRs
// (the upper half of the 512-entry file at one wave per SIMD) hold in-flight staging data
// the compiler never needs for arithmetic, so it has no reason to copy a register whose
// load has not landed (a VGPR destination above 256 live registers gets "spilled" to an
// AGPR right after the load instruction, i.e. before the data arrives).
template <int OFF>
__device__ __forceinline__ void gload16_nt_a(f4v& dst, unsigned voff, const void* sbase) {
  static_assert(OFF >= 0 && OFF < 4096, "12-bit immediate");
  asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3 nt" : "=a"(dst) : "v"(voff), "s"(sbase), "i"(OFF) : "memory");
}
// the same into VGPRs (for kernels whose register budget leaves no room for an AGPR split)
template <int OFF>
__device__ __forceinline__ void gload16_nt_v(f4v& dst, unsigned voff, const void* sbase) {
  static_assert(OFF >= 0 && OFF < 4096, "12-bit immediate");
  asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3 nt" : "=v"(dst) : "v"(voff), "s"(sbase), "i"(OFF) : "memory");
}
template <int OFF>
__device__ __forceinline__ void lds_write_b128_v(unsigned lds_addr, const f4v& v) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16-bit");
  asm volatile("ds_write_b128 %0, %1 offset:%2" : : "v"(lds_addr), "v"(v), "i"(OFF) : "memory");
}
// 4-B-per-lane non-temporal load (one dword: two u8 complex samples) into a VGPR
template <int OFF>
__device__ __forceinline__ void gload4_nt_v(unsigned& dst, unsigned voff, const void* sbase) {
  static_assert(OFF >= 0 && OFF < 4096, "12-bit immediate");
  asm volatile("global_load_dword %0, %1, %2 offset:%3 nt" : "=v"(dst) : "v"(voff), "s"(sbase), "i"(OFF) : "memory");
}
// ds_write_b128 of AGPR data with an immediate offset (16-bit).
template <int OFF>
__device__ __forceinline__ void lds_write_b128_a(unsigned lds_addr, const f4v& v) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16-bit");
  asm volatile("ds_write_b128 %0, %1 offset:%2" : : "v"(lds_addr), "a"(v), "i"(OFF) : "memory");
}

// N consecutive 1-KiB chunks by 16-B-per-lane LDS-DMA in the saddr form: wave-uniform
// global base in an SGPR pair + per-lane 32-bit byte offset; the immediate offset is
// applied to BOTH the global and the LDS address (M0 = LDS byte address), so up to four
// chunks share one M0 / base setup.  Non-temporal (nt): streamed once.
// hipcc's builtin form materialises a 64-bit VGPR address and an SGPR pair per chunk.
template <int N>
__device__ __forceinline__ void glds16x(unsigned voff, const void* sbase, unsigned lds_addr) {
  static_assert(N >= 1 && N <= 4, "1..4 chunks per M0 setup (13-bit immediate)");
  // s_nop: M0 written by SALU needs one wait state before an LDS-DMA reads it
  if constexpr (N == 1)
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 offset:0 nt"
                 :: "v"(voff), "s"(sbase), "s"(lds_addr) : "memory", "m0");
  else if constexpr (N == 2)
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 offset:0 nt\n\t"
                 "global_load_lds_dwordx4 %0, %1 offset:1024 nt"
                 :: "v"(voff), "s"(sbase), "s"(lds_addr) : "memory", "m0");
  else if constexpr (N == 3)
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 offset:0 nt\n\t"
                 "global_load_lds_dwordx4 %0, %1 offset:1024 nt\n\tglobal_load_lds_dwordx4 %0, %1 offset:2048 nt"
                 :: "v"(voff), "s"(sbase), "s"(lds_addr) : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 offset:0 nt\n\t"
                 "global_load_lds_dwordx4 %0, %1 offset:1024 nt\n\tglobal_load_lds_dwordx4 %0, %1 offset:2048 nt\n\t"
                 "global_load_lds_dwordx4 %0, %1 offset:3072 nt"
                 :: "v"(voff), "s"(sbase), "s"(lds_addr) : "memory", "m0");
}
__device__ __forceinline__ unsigned lds_addr_of(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (clamped to [0, 24]; waiting for more
// than needed is always safe).  The steady-state counts are tested first.
template <int I = 24>
__device__ __forceinline__ void wait_vm_chain(int n) {
  if constexpr (I == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (n >= I) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(I) : "memory");
    else wait_vm_chain<I - 1>(n);
  }
}

// compile-time loop: f(std::integral_constant<int, I>{}) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Counted LDS wait without register operands.  Only safe where the register allocator
// cannot copy the in-flight destination before the wait; the kernels use the "+v" forms
// below (lds_wait, lds_wait2, lds_wait3), which make that impossible.
template <int N>
__device__ __forceinline__ void lds_wait_ordered() {
  asm volatile("s_waitcnt lgkmcnt(%0)" :: "n"(N));
}

template <int N>
__device__ __forceinline__ void lds_wait3(f2v& a, f4v& b, f4v& c) {
  asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "n"(N));
}
template <int N>
__device__ __forceinline__ void lds_wait2(f2v& a, f4v& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}

template <int N>
__device__ __forceinline__ void lds_wait(f4v& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}

// atan2 for the discriminator: |err| <= ~2.5e-7 rad (2 ulp polynomial on [0, 1] after the
// octant reduction), branch-free: ~30 VALU and no divergent call into ocml's atan2f.  The
// IEEE special cases are selected, not branched to: atan2(+-0, +-0), infinities (the
// quotient of two infinities is taken as 1), and NaN inputs (NaN out).
__device__ __forceinline__ float fast_atan2f(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const float mn = fminf(ax, ay), mx = fmaxf(ax, ay);
  const float mxs = fmaxf(mx, 1e-30f);                // zeros: finite quotient 0, selected below
  const float rc = __builtin_amdgcn_rcpf(mxs);
  float a = mn * rc;
  a = fmaf(fmaf(-mxs, a, mn), rc, a);                 // one Newton step: ~0.5 ulp quotient
  a = (mx == INFINITY) ? ((mn == INFINITY) ? 1.f : 0.f) : a;
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
  r = (ay > ax) ? 1.57079632679489662f - r : r;
  r = (x < 0.f) ? 3.14159265358979324f - r : r;
  asm volatile("" : "+v"(r));                          // keep the selects below branch-free
  // both zero: +0 -> 0, -0 -> pi (IEEE atan2 sign rules; copysign below gives +-)
  r = (mx == 0.f) ? (__builtin_signbitf(x) ? 3.14159265358979324f : 0.f) : r;
  r = copysignf(r, y);
  return (x != x || y != y) ? __builtin_nanf("") : r;
}

// fast_atan2f on two (y, x) pairs at once: the quotient's Newton step and the polynomial as
// packed FMAs (v_pk_fma_f32 / v_pk_mul_f32), the octant reduction and the IEEE selects per
// element -- the same arithmetic per element (every packed op rounds as its scalar twin)
__device__ __forceinline__ f2v fast_atan2f_x2(f2v y, f2v x) {
  const float ax0 = fabsf(x.x), ay0 = fabsf(y.x), ax1 = fabsf(x.y), ay1 = fabsf(y.y);
  const float mn0 = fminf(ax0, ay0), mx0 = fmaxf(ax0, ay0), mn1 = fminf(ax1, ay1), mx1 = fmaxf(ax1, ay1);
  const f2v mn = f2v{mn0, mn1};
  const f2v mxs = f2v{fmaxf(mx0, 1e-30f), fmaxf(mx1, 1e-30f)};
  const f2v rc = f2v{__builtin_amdgcn_rcpf(mxs.x), __builtin_amdgcn_rcpf(mxs.y)};
  f2v a = mn * rc;
  a = __builtin_elementwise_fma(__builtin_elementwise_fma(-mxs, a, mn), rc, a);
  a.x = (mx0 == INFINITY) ? ((mn0 == INFINITY) ? 1.f : 0.f) : a.x;
  a.y = (mx1 == INFINITY) ? ((mn1 == INFINITY) ? 1.f : 0.f) : a.y;
  const f2v s = a * a;
  auto c = [](float v) { return f2v{v, v}; };
  f2v r = c(0.002849547192454338f);
  r = __builtin_elementwise_fma(r, s, c(-0.01606736145913601f));
  r = __builtin_elementwise_fma(r, s, c(0.04268963634967804f));
  r = __builtin_elementwise_fma(r, s, c(-0.0750415101647377f));
  r = __builtin_elementwise_fma(r, s, c(0.1064087525010109f));
  r = __builtin_elementwise_fma(r, s, c(-0.1420363187789917f));
  r = __builtin_elementwise_fma(r, s, c(0.19992618262767792f));
  r = __builtin_elementwise_fma(r, s, c(-0.3333307206630707f));
  r = __builtin_elementwise_fma(r, s, c(1.0f));
  r = r * a;
  float r0 = r.x, r1 = r.y;
  r0 = (ay0 > ax0) ? 1.57079632679489662f - r0 : r0;
  r1 = (ay1 > ax1) ? 1.57079632679489662f - r1 : r1;
  r0 = (x.x < 0.f) ? 3.14159265358979324f - r0 : r0;
  r1 = (x.y < 0.f) ? 3.14159265358979324f - r1 : r1;
  asm volatile("" : "+v"(r0), "+v"(r1));
  r0 = (mx0 == 0.f) ? (__builtin_signbitf(x.x) ? 3.14159265358979324f : 0.f) : r0;
  r1 = (mx1 == 0.f) ? (__builtin_signbitf(x.y) ? 3.14159265358979324f : 0.f) : r1;
  r0 = copysignf(r0, y.x);
  r1 = copysignf(r1, y.y);
  r0 = (x.x != x.x || y.x != y.x) ? __builtin_nanf("") : r0;
  r1 = (x.y != x.y || y.y != y.y) ? __builtin_nanf("") : r1;
  return f2v{r0, r1};
}

// Deferred per-lane output queue: Q entries of 3 floats held in registers, written to HBM
// in one burst at the end of a wave's run.  Output stores interleaved with a streaming
// read lower the read rate far more than their bytes (tools/pipe_probe.hip, r02: one 768-B
// store per 15-KiB tile 80 -> 96 us, one per 5 tiles -> 86 us, the same bytes written at the
// end of each run -> 84 us), so the streaming kernels keep their outputs here until the
// run ends.  Entries are written with a wave-uniform index through a compile-time binary
// search (scalar branches, static register names: no scratch, no movrel).
template <int Q>
struct OutQ3 {
  float v[Q][3];
  template <int LO, int HI>
  __device__ __forceinline__ void put_bs(int k, float a, float b, float c) {
    if constexpr (LO == HI) {
      v[LO][0] = a; v[LO][1] = b; v[LO][2] = c;
      // a distinct marker ends each leaf: the leaves' stores cannot be merged into one
      // store at a computed index (which would move the queue to scratch memory)
      asm volatile("; oq leaf %0" :: "n"(LO));
    } else {
      constexpr int MID = (LO + HI + 1) / 2;
      if (k >= MID) put_bs<MID, HI>(k, a, b, c);
      else put_bs<LO, MID - 1>(k, a, b, c);
    }
  }
  __device__ __forceinline__ void put(int k, float a, float b, float c) {
    put_bs<0, Q - 1>(__builtin_amdgcn_readfirstlane(k), a, b, c);
  }
  // entries [0, cnt) -> p + step * j (one 12-B store per lane each); returns cnt
  __device__ __forceinline__ int flush(float* p, int64_t step, int cnt) {
    typedef float f3v __attribute__((ext_vector_type(3)));
    static_for<0, Q>([&](auto J) {
      constexpr int j = J;
      if (j < cnt) *reinterpret_cast<f3v*>(p + step * j) = f3v{v[j][0], v[j][1], v[j][2]};
    });
    return cnt;
  }
  // as flush, but element r of entry j (global index e0 + step*j + r) is stored only when
  // it lies in [lo, hi); whole entries inside the range take one 12-B store
  __device__ __forceinline__ void flush_owned(float* p, int64_t step, int cnt, int64_t e0, int64_t lo, int64_t hi) {
    typedef float f3v __attribute__((ext_vector_type(3)));
    static_for<0, Q>([&](auto J) {
      constexpr int j = J;
      if (j < cnt) {
        const int64_t e = e0 + step * j;
        float* q = p + step * j;
        if (e >= lo && e + 2 < hi) {
          *reinterpret_cast<f3v*>(q) = f3v{v[j][0], v[j][1], v[j][2]};
        } else {
          if (e >= lo && e < hi) q[0] = v[j][0];
          if (e + 1 >= lo && e + 1 < hi) q[1] = v[j][1];
          if (e + 2 >= lo && e + 2 < hi) q[2] = v[j][2];
        }
      }
    });
  }
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
