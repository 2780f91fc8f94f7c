// u8 RF front end + mono audio on the matrix cores (gfx950 v_mfma_i32_16x16x64_i8).
//
// Replaces, for u8 IQ (src/iofunc.cpp:61-69, model/fmRDSblock.py:58-59) over whole streams:
//   model/fmMonoBlock.py:86-95   lfilter(rf_coeff, 1.0, iq[0::2] / iq[1::2]) + [::10]
//   model/fmMonoBlock.py:98      fmDemodArctan (model/fmSupportLib.py:15-44), state 0
//   model/fmMonoBlock.py:101-109 lfilter(audio_coeff, ...) + [::5]
//
// Why integer MFMA: a u8 sample minus 128 is an exact int8, so the 101-tap RF FIR is an
// integer product once the taps are fixed-point.  Taps are quantised to 22-bit integers
// h_q = rint(h 2^S) (S from the largest tap) and split into three signed base-256 digits
// h_q = d0 + 256 d1 + 65536 d2; each digit's FIR is accumulated EXACTLY in int32 by the
// matrix cores, and y = (65536 acc2 + 256 acc1 + acc0) 2^-S / 128 is formed in f32 (two
// roundings; the quantisation is 2^-22 of the largest tap -- the f32 FMA chain it replaces
// rounds 101 times; the scale itself is never applied, atan2 is scale-free).  The FIR then
// costs the matrix pipe, not the VALU: on the vector path (fe_slot_kernel) 303
// v_pk_fma_f32 per 192 outputs were 56 % of the issue slots.
//
// GEMM form of one tile (256 decimated outputs m0 + 16 p + r, p, r in [0, 16)):
//   y[16p + r] = sum_j' H[r][j'] X[j'][p],  H[r][j'] = h[10 r + 104 - j'] (0 outside [0, T)),
//   X[j'][p] = x[10 m0 - 104 + 160 p + j'],  j' in [0, 256)
// so M = 16 (r), N = 16 (p), K = 256 = 4 steps of 64; per channel and digit 4 MFMAs, per
// tile 2 channels x 3 digits x 4 = 24 (K-order inside a step is the same map for A and B,
// so it cancels).  The C fragment gives lane l = (p = l & 15, g = l >> 4) the outputs
// 16 p + 4 g + i, i in [0, 4): four consecutive outputs per lane, I and Q in the same lane.
//
// Tile image: samples [10 m0 - 104, 10 m0 + 2552) (2656 = 332 chunks of 8), de-interleaved
// into two int8 planes (x - 128 = u8 ^ 0x80) in LDS; the next tile's chunks are loaded into
// registers while this tile computes.  Demod -> an LDS window of the audio block (5 tiles =
// 1280 samples = 256 audio outputs, 4 per lane) after a 150-sample history; the audio FIR
// (151 taps, f32) runs on the VALU at the block's end.  Each wave owns whole audio blocks
// (a run starting mid-stream first runs the previous tile as a warm-up: history + carry).
#include <cmath>
#include <cstdlib>

#include "sdr_launch.h"

namespace {

typedef int i4v __attribute__((ext_vector_type(4)));

constexpr float kPiF = 3.14159265358979323846f;
// Ablation builds of fe_mfma_mono_kernel (tools/build_abl.sh; never the product, which is 0):
// 1 no audio FIR, 2 no atan2, 4 no MFMAs (B reads kept), 8 no image writes, 16 no image loads
#ifndef SDR_FE_MFMA_ABL
#define SDR_FE_MFMA_ABL 0
#endif
constexpr int kAbl = SDR_FE_MFMA_ABL;
// fe_mfma_mono_kernel: 3 waves per SIMD (161 VGPRs).  r04b measured the A fragments loaded
// from L1 at every tile (123 VGPRs, 4 waves per SIMD): 77 against 67 us
#define SDR_FE_MFMA_WPE 3

constexpr float k2PiF = 6.28318530717958647692f;

struct MfmaFe {
  const unsigned char* iq;  // interleaved u8 IQ, 16-B aligned, stream bases 16-B aligned
  int64_t n, stride;        // complex samples per stream / between stream bases
  int64_t M, A;             // demod / audio samples per stream
  int bps;                  // audio blocks per stream
  int64_t total;            // audio blocks over all streams
  const float* taps;        // 101 RF taps (device)
  float qscale;             // 2^S
  const float* argev;       // the 151 audio taps reversed, zero at [-1] and [151] (TapSet::dev_rev)
  const i4v* afr;           // nullable: the A fragments built on the host (TapSet::dev_afr)
  float* audio;
  int64_t audio_stride;
};

constexpr int D = 10, T = 101, TO = 256, OFF = 104;
constexpr int IMG = D * TO + 96;          // image samples
constexpr int NCH = IMG / 8;              // 16-B raw chunks (8 complex u8 samples)
constexpr int NLD = (NCH + 63) / 64;      // chunks per lane
constexpr int TA = 151, DA = 5, AB = DA * TO, HA = 152, NW = DA * 3 + TA;   // 166
static_assert(IMG % 8 == 0 && NLD == 6, "image layout");
static_assert(D * 15 + T - 1 + (OFF - 100 - 0) < 256 && OFF - (T - 1) >= 0, "K = 256 covers the band");

// One wave per workgroup and a wave's LDS instructions execute in order, so ordering LDS
// traffic between lanes needs no s_barrier (whose fence would also drain the image
// prefetch's vmcnt): only the compiler must not move LDS accesses across this point.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ unsigned bperm(int src_lane, unsigned v) {
  return (unsigned)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

// The taps' fixed-point scale 2^S: the largest S with max|h| 2^S <= 2^23 - 2^16, i.e. the top
// signed base-256 digit within [-127, 127] -- 22.x bits of the largest tap (one to two more
// than a power-of-two bound on |h_q|; the RDS chain's pre-PLL signal, the most sensitive to the
// RF filter, moves by 2.5e-6 of its peak instead of 8e-6: tests/test_gpu_parity.py rds)
int tap_scale_exp(float hmax) { return (int)std::floor(std::log2((8388608.0 - 65536.0) / (double)hmax)); }

// one signed base-256 digit of a fixed-point tap
__device__ __forceinline__ int digit(int q, int k) {
  int d = 0;
  for (int j = 0; j <= k; ++j) {
    d = ((q & 0xff) ^ 0x80) - 0x80;
    q = (q - d) >> 8;
  }
  return d;
}

// y = 65536 acc2 + (256 acc1 + acc0), the last two digits combined in int32 (|256 acc1 + acc0|
// <= 256 * 127 * 128 * 320 + ... < 2^31) before the one conversion: two roundings, as before
__device__ __forceinline__ void combine_digits(const i4v (&acc)[2][3], float (&yi)[4], float (&yq)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    yi[i] = fmaf((float)acc[0][2][i], 65536.f, (float)(acc[0][1][i] * 256 + acc[0][0][i]));
    yq[i] = fmaf((float)acc[1][2][i], 65536.f, (float)(acc[1][1][i] * 256 + acc[1][0][i]));
  }
}
// fast_atan2f_x2 (sdr_common.h) for finite operands: the FIR sums here are integers held in
// f32, never infinite or NaN, so the IEEE special cases (|x| or |y| infinite, NaN) drop out;
// the same arithmetic otherwise, so the same results
__device__ __forceinline__ f2v atan2_x2_finite(f2v y, f2v x) {
  const float ax0 = fabsf(x.x), ay0 = fabsf(y.x), ax1 = fabsf(x.y), ay1 = fabsf(y.y);
  const float mn0 = fminf(ax0, ay0), mx0 = fmaxf(ax0, ay0), mn1 = fminf(ax1, ay1), mx1 = fmaxf(ax1, ay1);
  const f2v mn = f2v{mn0, mn1};
  const f2v mxs = f2v{fmaxf(mx0, 1e-30f), fmaxf(mx1, 1e-30f)};
  const f2v rc = f2v{__builtin_amdgcn_rcpf(mxs.x), __builtin_amdgcn_rcpf(mxs.y)};
  f2v a = mn * rc;
  a = __builtin_elementwise_fma(__builtin_elementwise_fma(-mxs, a, mn), rc, a);
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
  return f2v{copysignf(r0, y.x), copysignf(r1, y.y)};
}
// FINITE: integer sums only (the mono kernel); the demod kernel adds the caller's lfilter zi
template <bool FINITE>
__device__ __forceinline__ void atan2_4(const float (&y)[4], const float (&x)[4], float (&phi)[4]) {
  const f2v p01 = FINITE ? atan2_x2_finite(f2v{y[0], y[1]}, f2v{x[0], x[1]}) : fast_atan2f_x2(f2v{y[0], y[1]}, f2v{x[0], x[1]});
  const f2v p23 = FINITE ? atan2_x2_finite(f2v{y[2], y[3]}, f2v{x[2], x[3]}) : fast_atan2f_x2(f2v{y[2], y[3]}, f2v{x[2], x[3]});
  phi[0] = p01.x; phi[1] = p01.y; phi[2] = p23.x; phi[3] = p23.y;
}
// acc.xy += tap2.xy * x2.xy, the tap pair a 64-bit SGPR operand (a scalar load of two
// consecutive reversed taps: no SALU assembles it)
__device__ __forceinline__ void pk_fma_s(f2v& acc, f2v tap2, const f2v& x2) {
  asm("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc) : "s"(tap2), "v"(x2));
}
typedef float f2a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef const __attribute__((address_space(4))) float* cfp4;   // uniform, read-only: scalar loads
typedef const __attribute__((address_space(4))) f2a4* cfp2;

// The next tile's image loads are issued at the top of a tile and waited for at its end (r03
// measured a two-tile-deep variant with alternating staging sets: no faster, 26 more VGPRs).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SDR_FE_MFMA_WPE))) void fe_mfma_mono_kernel(MfmaFe p) {
  __shared__ __attribute__((aligned(16))) signed char img[2][IMG + 16];   // I, Q planes
  __shared__ __attribute__((aligned(16))) float dh[HA + AB + 8];

  const int lane = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * p.total / gridDim.x;
  const int64_t b1 = ((int64_t)blockIdx.x + 1) * p.total / gridDim.x;
  if (b0 >= b1) return;
  const int pl = lane & 15, gl = lane >> 4;

  // A fragments: lane (r = l & 15, g = l >> 4), byte j of K-step ks <-> j' = 64 ks + 16 g + j;
  // from the tap set's table (one 16-B load each) or built here (~700 VALU per wave)
  i4v afr[4][3];
  if (p.afr != nullptr) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int dg = 0; dg < 3; ++dg) afr[ks][dg] = p.afr[(ks * 3 + dg) * 64 + lane];
  } else
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    int w[3][4] = {};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = D * pl + OFF - (64 * ks + 16 * gl + j);
      const float h = (k >= 0 && k < T) ? p.taps[k] : 0.f;
      const int q = (int)rintf(h * p.qscale);
#pragma unroll
      for (int dg = 0; dg < 3; ++dg) w[dg][j >> 2] |= (digit(q, dg) & 0xff) << (8 * (j & 3));
    }
#pragma unroll
    for (int dg = 0; dg < 3; ++dg) afr[ks][dg] = i4v{w[dg][0], w[dg][1], w[dg][2], w[dg][3]};
  }
  // the fragments' loads retired here, in the compiler's view: otherwise its wait for them is
  // merged into the tile loop's top from the entry path and retires the image prefetch (and the
  // previous tile's stores) at every tile, before the MFMAs instead of after them
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int dg = 0; dg < 3; ++dg) asm volatile("" : : "v"(afr[ks][dg]));
  // audio taps reversed (g[j] = h[150 - j]), tap pairs as SGPR operands (scalar loads at
  // compile-time offsets, as rx.hip's fir_tile)
  const cfp4 gr = (cfp4)p.argev;

  // ---- tile images: chunk c = lane + 64 q (16 raw bytes = 8 complex u8 samples) ----
  // Interior images: hand-issued 16-B loads into a staging set, waited for by a counted
  // s_waitcnt when the image is written (compiler-placed waits serialised the loads one at a
  // time).  Only the asm loads write a staging set: a second, compiler-visible writer made the
  // compiler merge the two through register copies taken before the data landed.  Boundary
  // images (stream head / tail: zeros, 0x80, outside [0, n)) are built at write time from
  // guarded 2-B loads.
  f4v stg[NLD];
  const unsigned voff = 16u * lane;
  auto n_lo_of = [&](int64_t t) { return (int64_t)TO * D * t - OFF; };
  auto interior = [&](int64_t t) { return n_lo_of(t) >= 0 && n_lo_of(t) + IMG <= p.n; };
  auto base_of = [&](int s, int64_t t) { return p.iq + 2 * ((int64_t)s * p.stride + n_lo_of(t)); };
  // halo: the tile follows the one in LDS in the same stream -- its first HC chunks are that
  // image's last HC (moved LDS -> LDS at store time), so only the 320 new chunks (5 per lane)
  // are read: HBM reads = the stream's bytes, not 2 656 / 2 560 of them
  constexpr int HC = (IMG - D * TO) / 8;
  static_assert(D * TO / 8 == 5 * 64, "5 new chunks per lane");
  // ONE load site per staging register for both cases (the first chunk a uniform offset, the
  // last load masked by lane count): 5 full loads with the halo, 6 without
  auto load_image = [&](int s, int64_t t, bool halo) {
    const int cf = halo ? HC : 0;
    const unsigned char* base = base_of(s, t) + 16 * cf;
    if (kAbl & 16) return;
    static_for<0, NLD>([&](auto Q) {
      constexpr int q = Q;
      if (lane < NCH - cf - 64 * q) gload16_nt_v<0>(stg[q], voff, base + 1024 * q);
    });
  };
  // de-interleave (I0 Q0 I1 Q1 ...) into the int8 planes: x - 128 = u8 ^ 0x80
  auto put_chunk = [&](int c, unsigned w0, unsigned w1, unsigned w2, unsigned w3) {
    const unsigned i_lo = __builtin_amdgcn_perm(w1, w0, 0x06040200u) ^ 0x80808080u;
    const unsigned i_hi = __builtin_amdgcn_perm(w3, w2, 0x06040200u) ^ 0x80808080u;
    const unsigned q_lo = __builtin_amdgcn_perm(w1, w0, 0x07050301u) ^ 0x80808080u;
    const unsigned q_hi = __builtin_amdgcn_perm(w3, w2, 0x07050301u) ^ 0x80808080u;
    *reinterpret_cast<uint2*>(&img[0][8 * c]) = make_uint2(i_lo, i_hi);
    *reinterpret_cast<uint2*>(&img[1][8 * c]) = make_uint2(q_lo, q_hi);
  };
  // write the staged image (the audio stores wait in registers: no other VMEM is in flight)
  auto store_image = [&](bool halo) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int cf = halo ? HC : 0;
    if (halo && lane < 2 * HC) {                 // the halo to the front (both planes), before the new chunks
      const int ch = lane / HC, k = lane - ch * HC;
      const uint2 v = *reinterpret_cast<const uint2*>(&img[ch][D * TO + 8 * k]);
      *reinterpret_cast<uint2*>(&img[ch][8 * k]) = v;
    }
    lds_order();
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int c = cf + lane + 64 * q;
      if (c < NCH) {
        asm volatile("" : "+v"(stg[q]));
        if (!(kAbl & 8))
          put_chunk(c, __float_as_uint(stg[q].x), __float_as_uint(stg[q].y), __float_as_uint(stg[q].z),
                    __float_as_uint(stg[q].w));
      }
    }
  };
  auto build_guarded = [&](int s, int64_t t) {
    const int64_t n_lo = n_lo_of(t);
    const unsigned char* base = base_of(s, t);
    for (int c = lane; c < NCH; c += 64) {
      unsigned w4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t n0 = n_lo + 8 * c + 2 * e;             // samples n0, n0 + 1
        const unsigned lo = (n0 >= 0 && n0 < p.n) ? *reinterpret_cast<const unsigned short*>(base + 2 * (8 * c + 2 * e)) : 0x8080u;
        const unsigned hi = (n0 + 1 >= 0 && n0 + 1 < p.n) ? *reinterpret_cast<const unsigned short*>(base + 2 * (8 * c + 2 * e + 1)) : 0x8080u;
        w4[e] = lo | (hi << 16);
      }
      put_chunk(c, w4[0], w4[1], w4[2], w4[3]);
    }
  };

  // ---- run: audio blocks [b0, b1), warm-up tile first when starting mid-stream ----
  int s = (int)(b0 / p.bps);
  int64_t t = (b0 - (int64_t)s * p.bps) * DA;
  const int64_t tps = (int64_t)p.bps * DA;
  const bool warm = t > 0;
  if (warm) --t;
  const int64_t U = (b1 - b0) * DA + (warm ? 1 : 0);
  for (int e = lane; e < HA; e += 64) dh[e] = 0.f;          // zero history at a stream start
  if (interior(t)) {
    load_image(s, t, false);
    store_image(false);
  } else {
    build_guarded(s, t);
  }
  auto next_s = [&](int s_, int64_t t_) { return t_ + 1 == tps ? s_ + 1 : s_; };
  auto next_t = [&](int64_t t_) { return t_ + 1 == tps ? (int64_t)0 : t_ + 1; };
  int s1 = next_s(s, t);
  int64_t t1 = next_t(t);
  float carry = 0.f;
  float d4[4] = {0.f, 0.f, 0.f, 0.f};

  // deferred audio outputs: AQ blocks of 4 outputs per lane, stored when the queue is full and
  // at the run's end (the run's blocks complete in order: entry k is audio block qb + k)
  constexpr int AQ = 4;
  f4v aq[AQ];
  int nq = 0;
  int qs = (int)(b0 / p.bps);                                // entry 0: stream qs, block qj
  int qj = (int)(b0 - (int64_t)qs * p.bps);
  auto queue_flush = [&]() __attribute__((always_inline)) {
    static_for<0, AQ>([&](auto K) {
      constexpr int k = K;
      if (k < nq) {
        const int64_t j = (int64_t)TO * qj + 4 * lane;
        float* ao = p.audio + (int64_t)qs * p.audio_stride + j;
        if (j + 4 <= p.A && ((uintptr_t)ao & 15) == 0) {
          *reinterpret_cast<f4v*>(ao) = aq[k];
        } else {
          const float rv[4] = {aq[k].x, aq[k].y, aq[k].z, aq[k].w};
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (j + r < p.A) ao[r] = rv[r];
        }
        if (++qj == p.bps) { qj = 0; ++qs; }
      }
    });
    nq = 0;
  };
  auto queue_put = [&](const f4v& v) __attribute__((always_inline)) {
    static_for<0, AQ>([&](auto K) {                          // compile-time slots (no scratch)
      if ((int)K == nq) aq[K] = v;
    });
    if (++nq == AQ) queue_flush();
  };

  // the MFMAs of the tile whose image is in LDS: B fragments of both channels, one K-step at a
  // time (registers: occupancy)
  auto mfma_tile = [&](i4v (&acc)[2][3]) __attribute__((always_inline)) {
    lds_order();                                              // the image written
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int dg = 0; dg < 3; ++dg) acc[ch][dg] = i4v{0, 0, 0, 0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      i4v a[3];
#pragma unroll
      for (int dg = 0; dg < 3; ++dg) a[dg] = afr[ks][dg];
      i4v bf[2];
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) bf[ch] = *reinterpret_cast<const i4v*>(&img[ch][160 * pl + 64 * ks + 16 * gl]);
#pragma unroll
      for (int ch = 0; ch < 2; ++ch)
#pragma unroll
        for (int dg = 0; dg < 3; ++dg)
          acc[ch][dg] = (kAbl & 4) ? acc[ch][dg] + bf[ch]
                                   : __builtin_amdgcn_mfma_i32_16x16x64_i8(a[dg], bf[ch], acc[ch][dg], 0, 0, 0);
    }
  };
  // tile (s, t) from its accumulators: digits combined, demod, the audio block at its end
  auto epilogue = [&](const i4v (&acc)[2][3], int64_t u) __attribute__((always_inline)) {
    float yi[4], yq[4];
    combine_digits(acc, yi, yq);
    float phi[4];
    if (kAbl & 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) phi[i] = yq[i] * 1e-9f + yi[i] * 1e-9f;
    } else {
      atan2_4<true>(yq, yi, phi);        // atan2 is scale-free: the 2^-S / 128 is never applied
    }
    const int src = gl > 0 ? lane - 16 : (pl > 0 ? lane + 47 : 63);
    const float left = __uint_as_float(bperm(src, __float_as_uint(phi[3])));
    float prev = (lane == 0) ? carry : left;
    const int64_t mo = (int64_t)TO * t + 16 * pl + 4 * gl;     // first output of this lane
    float d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float dd = phi[i] - prev;
      if (dd > kPiF) dd -= k2PiF;
      else if (dd < -kPiF) dd += k2PiF;
      d[i] = (mo + i == 0) ? phi[i] : dd;                     // m = 0: prev_phase 0
      prev = phi[i];
    }
    carry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[3]), 63));
    const int o = 16 * pl + 4 * gl;                           // output within the tile
    const int tb = (int)(t % DA);
    if (warm && u == 0) {                                     // history of the first block
      if (o >= TO - HA) *reinterpret_cast<f4v*>(&dh[HA - TO + o]) = f4v{d[0], d[1], d[2], d[3]};
    } else {
      *reinterpret_cast<f4v*>(&dh[HA + TO * tb + o]) = f4v{d[0], d[1], d[2], d[3]};
#pragma unroll
      for (int i = 0; i < 4; ++i) d4[i] = d[i];
    }
    if (!(kAbl & 1) && !(warm && u == 0) && tb == DA - 1) {
      // audio block jb: a[j] = sum_k g[k] d[5j - k]
      lds_order();
      // window sample w, output r: tap h[150 + 5 r - w] = g[w - 5 r]; each output keeps its
      // even- and odd-sample partial sums in one packed register:
      //   acc_r.xy += (g[j], g[j+1]) * (x_w, x_{w+1}),  j = w - 5 r  (g[-1] = g[151] = 0)
      const float* aw = dh + (HA - (TA - 1)) + DA * 4 * lane;
      f2v acc[4] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}, f2v{0.f, 0.f}, f2v{0.f, 0.f}};
      static_for<0, NW / 2>([&](auto W2) {
        constexpr int w = 2 * W2;
        const f2v x2 = *reinterpret_cast<const f2v*>(aw + w);
        static_for<0, 4>([&](auto RR) {
          constexpr int j = w - DA * (int)RR;
          if constexpr (j >= -1 && j <= TA - 1) {
            const f2a4 hp = *(cfp2)(gr + j);         // (g[j], g[j+1]): float-indexed pair
            pk_fma_s(acc[RR], f2v{hp.x, hp.y}, x2);
          }
        });
      });
      // the outputs wait in registers: stores interleaved with the read stream cost far more
      // than their bytes (OutQ3); blocks leave in order, b0 + entry
      queue_put(f4v{acc[0].x + acc[0].y, acc[1].x + acc[1].y, acc[2].x + acc[2].y, acc[3].x + acc[3].y});
      lds_order();
      // this block's last 150 demod samples become the next block's history
      if (o >= TO - HA) *reinterpret_cast<f4v*>(&dh[HA - TO + o]) = f4v{d4[0], d4[1], d4[2], d4[3]};
    }
  };
  // the next image replaces this one (its B reads returned long ago); new stream: zero history
  auto advance = [&]() __attribute__((always_inline)) {
    s = s1;
    t = t1;
    if (t == 0) {
      lds_order();
      for (int e = lane; e < HA; e += 64) dh[e] = 0.f;
    }
    s1 = next_s(s, t);
    t1 = next_t(t);
  };

  // Per tile: its B reads and MFMAs go out; the next tile's image (whose loads flew during
  // the previous epilogue) is written while the MFMAs run -- a wave's LDS operations execute
  // in order, so the stores land after this tile's B reads -- then the tile after's loads go
  // out and fly during this tile's epilogue (an in-flight register never crosses the loop's
  // back edge, where the compiler may copy it: the loads are issued and retired within one
  // iteration's straight-line span of their own)
  bool staged = U > 1 && interior(t1);
  bool halo = staged && s1 == s && t1 == t + 1 && interior(t);
  if (staged) load_image(s1, t1, halo);
  i4v acc[2][3];
  for (int64_t u = 0; u < U; ++u) {
    const bool more = u + 1 < U;
    mfma_tile(acc);                                           // tile (s, t)
    if (more) {
      lds_order();
      if (staged) store_image(halo);                          // tile (s1, t1)
      else build_guarded(s1, t1);
      const int s2 = next_s(s1, t1);
      const int64_t t2 = next_t(t1);
      staged = u + 2 < U && interior(t2);
      halo = staged && s2 == s1 && t2 == t1 + 1 && interior(t1);
      if (staged) load_image(s2, t2, halo);
    }
    epilogue(acc, u);
    if (more) advance();
  }
  // nothing is in flight here (the last two tiles issue no image loads); the wait says so to
  // tools/inflight_check.py, whose scan also follows the loop exit from a tile that loaded
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  queue_flush();
}

// ---------------------------------------------------------------------------------
// The same RF FIR as the FE of the block / span receivers (C5, fm_radio_gpu): demod out,
// lfilter state in (zi, first outputs), demod phase state in (prev_phase, output 0) and out
// (last_phi, wraps: finished by the receiver's stage-A workgroups), any stream length.
//   T = 101: K = 256 (4 steps), OFF = 104;  T = 151: K = 320 (5 steps), OFF = 152
// (band: 10 x 15 + T - 1 <= K - 1 with OFF >= T - 1; OFF a multiple of 8: 16-B image loads).
// Work: contiguous runs of 256-output tiles per wave across the streams; a run starting
// mid-stream first runs the tile before as a warm-up (its last phase is the carry).
template <int T> struct DemodShape;
template <> struct DemodShape<101> { static constexpr int KS = 4, OFF = 104; };
template <> struct DemodShape<151> { static constexpr int KS = 5, OFF = 152; };

struct MfmaDemod {
  const unsigned char* iq;
  int64_t n, stride;          // complex samples per stream / between stream bases
  int64_t M;                  // demod samples per stream
  int64_t tps, total;         // tiles per stream, over all streams
  const float* taps;
  float qscale;               // 2^S
  const i4v* afr;             // nullable: the A fragments built on the host (TapSet::dev_afr)
  const double* zi_i;         // nullable: lfilter states (T - 1 per stream, zi_stride apart)
  const double* zi_q;
  int64_t zi_stride;
  const double* prev_phase;   // nullable (=> 0.0)
  float* demod;
  int64_t out_stride;
  float* last_phi;            // nullable
  int* wraps;                 // nullable
  int vec_out;                // demod rows allow 16-B stores
};

__device__ inline double unwrap_step_f64_m(double dd, int* w) {   // fe.hip unwrap_step_f64
  *w = 0;
  if (fabs(dd) < 3.14159265358979323846) return dd;
  constexpr double kPi = 3.14159265358979323846, k2Pi = 6.28318530717958647692;
  double m = fmod(dd + kPi, k2Pi);
  if (m < 0) m += k2Pi;
  double ddmod = m - kPi;
  if (ddmod == -kPi && dd > 0) ddmod = kPi;
  *w = (int)llrint((ddmod - dd) / k2Pi);
  return ddmod;
}

// The phase of ONE decimated output m (10 m >= T - 1: no lfilter zi) of stream s, exactly as
// a tile computes it: each tap digit's sum over the T samples in int32 (the matrix cores' sums
// are exact, so the order does not matter), combined and taken through the same atan2.  A run
// of tiles starting mid-stream needs the phase of the output before it (the demod's
// predecessor); this replaces a whole warm-up tile (2 560 samples read and 24 MFMAs) with T
// taps per channel over one wave.
template <int T>
__device__ __forceinline__ float output_phase(const unsigned char* iq_s, int64_t m, const float* taps, float qscale) {
  const int lane = threadIdx.x;
  int acc[2][3] = {};
  for (int k = lane; k < T; k += 64) {
    const int q = (int)rintf(taps[k] * qscale);
    const unsigned short v = *reinterpret_cast<const unsigned short*>(iq_s + 2 * (D * m - k));
    const int xi = (int)(signed char)((v & 0xff) ^ 0x80), xq = (int)(signed char)(((v >> 8) & 0xff) ^ 0x80);
#pragma unroll
    for (int dg = 0; dg < 3; ++dg) {
      const int d = digit(q, dg);
      acc[0][dg] += d * xi;
      acc[1][dg] += d * xq;
    }
  }
#pragma unroll
  for (int ch = 0; ch < 2; ++ch)
#pragma unroll
    for (int dg = 0; dg < 3; ++dg) acc[ch][dg] = wave_sum_i(acc[ch][dg]);
  const float yi = fmaf((float)acc[0][2], 65536.f, (float)(acc[0][1] * 256 + acc[0][0]));   // combine_digits
  const float yq = fmaf((float)acc[1][2], 65536.f, (float)(acc[1][1] * 256 + acc[1][0]));
  return fast_atan2f_x2(f2v{yq, yq}, f2v{yi, yi}).x;
}

template <int T>
__global__ __launch_bounds__(64) void fe_mfma_demod_kernel(MfmaDemod p) {
  constexpr int KS = DemodShape<T>::KS, OFF = DemodShape<T>::OFF, K = 64 * KS;
  constexpr int IM = 160 * 15 + K;                 // image samples (16 columns of 160, K deep)
  constexpr int NC = IM / 8, NL = (NC + 63) / 64;
  static_assert(IM % 8 == 0 && OFF % 8 == 0 && OFF >= T - 1 && D * 15 + OFF <= K - 1, "image / band layout");
  __shared__ __attribute__((aligned(16))) signed char img[2][IM + 16];

  const int lane = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * p.total / gridDim.x;
  const int64_t b1 = ((int64_t)blockIdx.x + 1) * p.total / gridDim.x;
  if (b0 >= b1) return;
  const int pl = lane & 15, gl = lane >> 4;

  i4v afr[KS][3];
  if (p.afr != nullptr) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int dg = 0; dg < 3; ++dg) afr[ks][dg] = p.afr[(ks * 3 + dg) * 64 + lane];
  } else
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    int w[3][4] = {};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = D * pl + OFF - (64 * ks + 16 * gl + j);
      const float h = (k >= 0 && k < T) ? p.taps[k] : 0.f;
      const int q = (int)rintf(h * p.qscale);
#pragma unroll
      for (int dg = 0; dg < 3; ++dg) w[dg][j >> 2] |= (digit(q, dg) & 0xff) << (8 * (j & 3));
    }
#pragma unroll
    for (int dg = 0; dg < 3; ++dg) afr[ks][dg] = i4v{w[dg][0], w[dg][1], w[dg][2], w[dg][3]};
  }
  // the fragments' loads retired here, in the compiler's view: otherwise its wait for them is
  // merged into the tile loop's top from the entry path and retires the image prefetch (and the
  // previous tile's stores) at every tile, before the MFMAs instead of after them
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int dg = 0; dg < 3; ++dg) asm volatile("" : : "v"(afr[ks][dg]));

  f4v stg[NL];
  const unsigned voff = 16u * lane;
  auto n_lo_of = [&](int64_t t) { return (int64_t)TO * D * t - OFF; };
  auto interior = [&](int64_t t) { return n_lo_of(t) >= 0 && n_lo_of(t) + IM <= p.n; };
  auto base_of = [&](int s, int64_t t) { return p.iq + 2 * ((int64_t)s * p.stride + n_lo_of(t)); };
  constexpr int HC = (IM - D * TO) / 8;          // halo chunks (as in fe_mfma_mono_kernel)
  static_assert(D * TO / 8 == 5 * 64, "5 new chunks per lane");
  auto load_image = [&](int s, int64_t t, bool halo) {   // one load site per register (above)
    const int cf = halo ? HC : 0;
    const unsigned char* base = base_of(s, t) + 16 * cf;
    static_for<0, NL>([&](auto Q) {
      constexpr int q = Q;
      if (lane < NC - cf - 64 * q) gload16_nt_v<0>(stg[q], voff, base + 1024 * q);
    });
  };
  auto put_chunk = [&](int c, unsigned w0, unsigned w1, unsigned w2, unsigned w3) {
    const unsigned i_lo = __builtin_amdgcn_perm(w1, w0, 0x06040200u) ^ 0x80808080u;
    const unsigned i_hi = __builtin_amdgcn_perm(w3, w2, 0x06040200u) ^ 0x80808080u;
    const unsigned q_lo = __builtin_amdgcn_perm(w1, w0, 0x07050301u) ^ 0x80808080u;
    const unsigned q_hi = __builtin_amdgcn_perm(w3, w2, 0x07050301u) ^ 0x80808080u;
    *reinterpret_cast<uint2*>(&img[0][8 * c]) = make_uint2(i_lo, i_hi);
    *reinterpret_cast<uint2*>(&img[1][8 * c]) = make_uint2(q_lo, q_hi);
  };
  // st1: the previous epilogue issued exactly one VMEM op (its demod store) after this
  // image's loads -- vmcnt counts loads and stores in issue order, so vmcnt(1) retires the
  // loads and leaves that store in flight; anything else (a tile at a stream's edge: zi loads,
  // last_phi, the wrap-count atomic, partial stores) waits for everything
  bool st1 = false;
  auto store_image = [&](bool halo) {
    if (__builtin_amdgcn_readfirstlane((int)st1)) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int cf = halo ? HC : 0;
    if (halo && lane < 2 * HC) {
      const int ch = lane / HC, k = lane - ch * HC;
      const uint2 v = *reinterpret_cast<const uint2*>(&img[ch][D * TO + 8 * k]);
      *reinterpret_cast<uint2*>(&img[ch][8 * k]) = v;
    }
    lds_order();
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      const int c = cf + lane + 64 * q;
      if (c < NC) {
        asm volatile("" : "+v"(stg[q]));
        put_chunk(c, __float_as_uint(stg[q].x), __float_as_uint(stg[q].y), __float_as_uint(stg[q].z),
                  __float_as_uint(stg[q].w));
      }
    }
  };
  auto build_guarded = [&](int s, int64_t t) {
    const int64_t n_lo = n_lo_of(t);
    const unsigned char* base = base_of(s, t);
    for (int c = lane; c < NC; c += 64) {
      unsigned w4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t n0 = n_lo + 8 * c + 2 * e;
        const unsigned lo = (n0 >= 0 && n0 < p.n) ? *reinterpret_cast<const unsigned short*>(base + 2 * (8 * c + 2 * e)) : 0x8080u;
        const unsigned hi = (n0 + 1 >= 0 && n0 + 1 < p.n) ? *reinterpret_cast<const unsigned short*>(base + 2 * (8 * c + 2 * e + 1)) : 0x8080u;
        w4[e] = lo | (hi << 16);
      }
      put_chunk(c, w4[0], w4[1], w4[2], w4[3]);
    }
  };

  int s = (int)(b0 / p.tps);
  int64_t t = b0 - (int64_t)s * p.tps;
  const int64_t U = b1 - b0;
  // the run's first tile continues the stream: the phase of the output before it
  float carry = t > 0 ? output_phase<T>(p.iq + 2 * (int64_t)s * p.stride, TO * t - 1, p.taps, p.qscale) : 0.f;
  if (interior(t)) {
    load_image(s, t, false);
    store_image(false);
  } else {
    build_guarded(s, t);
  }
  int s_nx = s;
  int64_t t_nx = t + 1;
  if (t_nx == p.tps) { t_nx = 0; ++s_nx; }
  int wsum = 0;
  const double zscale = (double)p.qscale * 128.0;    // real-domain zi -> the integer sum's scale

  // as fe_mfma_mono_kernel: the next image is written while this tile's MFMAs run, the loads
  // of the one after fly during this tile's epilogue
  bool staged = U > 1 && interior(t_nx);
  bool halo = staged && s_nx == s && t_nx == t + 1 && interior(t);
  if (staged) load_image(s_nx, t_nx, halo);
  for (int64_t u = 0; u < U; ++u) {
    const bool more = u + 1 < U;
    lds_order();
    i4v acc[2][3];
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int dg = 0; dg < 3; ++dg) acc[ch][dg] = i4v{0, 0, 0, 0};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      i4v bf[2];
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) bf[ch] = *reinterpret_cast<const i4v*>(&img[ch][160 * pl + 64 * ks + 16 * gl]);
#pragma unroll
      for (int ch = 0; ch < 2; ++ch)
#pragma unroll
        for (int dg = 0; dg < 3; ++dg)
          acc[ch][dg] = __builtin_amdgcn_mfma_i32_16x16x64_i8(afr[ks][dg], bf[ch], acc[ch][dg], 0, 0, 0);
    }
    if (more) {
      lds_order();
      if (staged) store_image(halo);                          // tile (s_nx, t_nx)
      else build_guarded(s_nx, t_nx);
      int s2 = s_nx;
      int64_t t2 = t_nx + 1;
      if (t2 == p.tps) { t2 = 0; ++s2; }
      staged = u + 2 < U && interior(t2);
      halo = staged && s2 == s_nx && t2 == t_nx + 1 && interior(t_nx);
      if (staged) load_image(s2, t2, halo);
    }
    const int64_t mo = (int64_t)TO * t + 16 * pl + 4 * gl;     // first output of this lane
    float yi[4], yq[4];
    combine_digits(acc, yi, yq);
    if (t == 0 && p.zi_i != nullptr) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (D * (mo + i) < T - 1) {      // lfilter zi (model/fmMonoBlock.py:86-91)
          yi[i] += (float)(p.zi_i[(int64_t)s * p.zi_stride + D * (mo + i)] * zscale);
          yq[i] += (float)(p.zi_q[(int64_t)s * p.zi_stride + D * (mo + i)] * zscale);
        }
    }
    float phi[4];
    atan2_4<false>(yq, yi, phi);         // atan2 is scale-free: the 2^-S / 128 is never applied
    const int src = gl > 0 ? lane - 16 : (pl > 0 ? lane + 47 : 63);
    const float left = __uint_as_float(bperm(src, __float_as_uint(phi[3])));
    float prev = (lane == 0) ? carry : left;
    constexpr bool keep = true;
    float d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t m = mo + i;
      int wk = 0;
      if (m == 0) {
        const double ps = p.prev_phase ? p.prev_phase[s] : 0.0;
        d[i] = (float)unwrap_step_f64_m((double)phi[i] - ps, &wk);
      } else {
        float dd = phi[i] - prev;
        if (dd > kPiF) { dd -= k2PiF; wk = -1; }
        else if (dd < -kPiF) { dd += k2PiF; wk = 1; }
        d[i] = dd;
      }
      if (keep && m < p.M) wsum += wk;
      prev = phi[i];
    }
    carry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[3]), 63));
    if (keep) {
      float* out = p.demod + (int64_t)s * p.out_stride + mo;
      if (p.vec_out && mo + 4 <= p.M) {
        *reinterpret_cast<f4v*>(out) = f4v{d[0], d[1], d[2], d[3]};
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (mo + i < p.M) out[i] = d[i];
      }
      if (p.last_phi != nullptr) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (mo + i == p.M - 1) p.last_phi[s] = phi[i];
      }
    }
    // the stream's wrap count leaves with its last tile of this run
    const bool wr = keep && (!more || s_nx != s) && p.wraps != nullptr;
    if (wr) {
      const int w = wave_sum_i(wsum);
      if (lane == 0 && w != 0) atomicAdd(p.wraps + s, w);
      wsum = 0;
    }
    st1 = keep && p.vec_out && t > 0 && (int64_t)TO * t + TO < p.M && !wr;
    if (more) {
      s = s_nx;
      t = t_nx;
      t_nx = t + 1;
      s_nx = s;
      if (t_nx == p.tps) { t_nx = 0; ++s_nx; }
    }
  }
}

template <int T>
hipError_t launch_demod_mfma_t(const FeLaunch& a, hipStream_t st) {
  float hmax = 0.f;
  for (int k = 0; k < T; ++k) hmax = std::max(hmax, std::fabs(a.taps->h[k]));
  if (!(hmax > 0.f) || !std::isfinite(hmax)) return hipErrorInvalidValue;
  const int S = tap_scale_exp(hmax);
  MfmaDemod p{};
  p.iq = static_cast<const unsigned char*>(a.iq);
  p.n = a.n;
  p.stride = a.nstreams > 1 ? a.stride : 0;
  p.M = (a.n + D - 1) / D;
  p.tps = (p.M + TO - 1) / TO;
  p.total = p.tps * a.nstreams;
  if (p.total > 0x7fffffff) return hipErrorInvalidValue;
  p.taps = a.taps_dev;
  p.qscale = std::ldexp(1.0f, S);
  p.afr = reinterpret_cast<const i4v*>(a.afr);
  p.zi_i = a.zi_i;
  p.zi_q = a.zi_q;
  p.zi_stride = a.zi_stride;
  p.prev_phase = a.prev_phase;
  p.demod = a.demod;
  p.out_stride = a.out_stride;
  p.last_phi = a.last_phi;
  p.wraps = a.wraps;
  p.vec_out = ((a.out_stride % 4) == 0 && ((uintptr_t)a.demod % 16) == 0) ? 1 : 0;
  static std::atomic<int> slot_cache[kMaxDevices];
  const int slots = per_device(slot_cache, [] {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fe_mfma_demod_kernel<T>, 64, 0) != hipSuccess || per <= 0) per = 1;
    return device_cus() * std::min(per, 12);
  });
  // the resident waves share the tiles in contiguous runs (a run's first tile takes its
  // predecessor phase from output_phase: no warm-up tile, so a run may be one tile)
  const int64_t run = std::max<int64_t>(1, (p.total + slots - 1) / slots);
  const int64_t grid = std::max<int64_t>(1, (p.total + run - 1) / run);
  hipLaunchKernelGGL(fe_mfma_demod_kernel<T>, dim3((unsigned)grid), dim3(64), 0, st, p);
  return hipGetLastError();
}

}  // namespace

// The A fragments the kernels build from the taps (fe_mfma_*_kernel prologues), on the host:
// the same f32 product h * 2^S, rintf, signed base-256 digits.
bool sdr_mfma_fragments(const float* h, int T_, std::vector<int>* out) {
  int KS, OFFT;
  if (T_ == 101) { KS = DemodShape<101>::KS; OFFT = DemodShape<101>::OFF; }
  else if (T_ == 151) { KS = DemodShape<151>::KS; OFFT = DemodShape<151>::OFF; }
  else return false;
  static_assert(DemodShape<101>::KS == 4 && DemodShape<101>::OFF == OFF, "mono and demod kernels share the T = 101 shape");
  float hmax = 0.f;
  for (int k = 0; k < T_; ++k) hmax = std::max(hmax, std::fabs(h[k]));
  if (!(hmax > 0.f) || !std::isfinite(hmax)) return false;
  const float qs = std::ldexp(1.0f, tap_scale_exp(hmax));
  out->assign((size_t)KS * 3 * 64 * 4, 0);
  for (int ks = 0; ks < KS; ++ks)
    for (int lane = 0; lane < 64; ++lane) {
      const int pl = lane & 15, gl = lane >> 4;
      for (int j = 0; j < 16; ++j) {
        const int k = D * pl + OFFT - (64 * ks + 16 * gl + j);
        const float hv = (k >= 0 && k < T_) ? h[k] : 0.f;
        int q = (int)std::rint(hv * qs);
        for (int dg = 0; dg < 3; ++dg) {
          const int d = ((q & 0xff) ^ 0x80) - 0x80;      // the kernels' digit(): q = d + 256 (q')
          q = (q - d) >> 8;
          (*out)[(((size_t)ks * 3 + dg) * 64 + lane) * 4 + (j >> 2)] |= (d & 0xff) << (8 * (j & 3));
        }
      }
    }
  return true;
}

// u8 RF front end (FIR + decimate + demod, carried state) on the matrix cores: 101 or 151
// taps at decim 10, u8 IQ with 16-B aligned stream bases, no history prefix and no
// decimated I/Q outputs; otherwise hipErrorInvalidValue (the caller runs fe_slot_kernel).
hipError_t sdr_launch_fe_mfma(const FeLaunch& a, hipStream_t st) {
  if (!a.u8 || a.D != D || a.hist != 0 || a.i_ds || a.q_ds || a.demod == nullptr) return hipErrorInvalidValue;
  if (((uintptr_t)a.iq & 15) != 0 || (a.nstreams > 1 && (a.stride % 8) != 0)) return hipErrorInvalidValue;
  if (a.n <= 0 || a.nstreams <= 0) return hipSuccess;
  if (a.T == 101) return launch_demod_mfma_t<101>(a, st);
  if (a.T == 151) return launch_demod_mfma_t<151>(a, st);
  return hipErrorInvalidValue;
}

// Fused u8 FE + mono on the matrix cores.  Supported: 101 RF taps at decim 10, 151 audio
// taps at decim 5, u8 IQ with 16-B aligned stream bases; otherwise hipErrorInvalidValue
// (the caller runs fe_slot_kernel).
hipError_t sdr_launch_fe_mono_mfma(const FeLaunch& a, const float* ataps_rev, int TA_, int DA_, float* audio,
                                   int64_t audio_stride, hipStream_t st) {
  if (!a.u8 || a.D != D || a.T != T || TA_ != TA || DA_ != DA || a.hist != 0 || a.zi_i || a.prev_phase || a.demod ||
      a.i_ds || a.last_phi || a.wraps)
    return hipErrorInvalidValue;
  if (((uintptr_t)a.iq & 15) != 0 || (a.nstreams > 1 && (a.stride % 8) != 0)) return hipErrorInvalidValue;
  if (a.n <= 0 || a.nstreams <= 0) return hipSuccess;
  float hmax = 0.f;
  for (int k = 0; k < T; ++k) hmax = std::max(hmax, std::fabs(a.taps->h[k]));
  if (!(hmax > 0.f) || !std::isfinite(hmax)) return hipErrorInvalidValue;
  const int S = tap_scale_exp(hmax);
  MfmaFe p{};
  p.iq = static_cast<const unsigned char*>(a.iq);
  p.n = a.n;
  p.stride = a.nstreams > 1 ? a.stride : 0;
  p.M = (a.n + D - 1) / D;
  p.A = (p.M + DA - 1) / DA;
  p.bps = (int)((p.M + AB - 1) / AB);
  p.total = (int64_t)p.bps * a.nstreams;
  if (p.total > 0x7fffffff) return hipErrorInvalidValue;
  p.taps = a.taps_dev;
  p.qscale = std::ldexp(1.0f, S);
  p.afr = reinterpret_cast<const i4v*>(a.afr);
  p.argev = ataps_rev;
  p.audio = audio;
  p.audio_stride = audio_stride;
  static std::atomic<int> slot_cache[kMaxDevices];
  const int slots = per_device(slot_cache, [] {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fe_mfma_mono_kernel, 64, 0) != hipSuccess || per <= 0) per = 1;
    const int cap = 4 * SDR_FE_MFMA_WPE;                 // waves per CU (r04b sweep: 12 of 8-16)
    return device_cus() * std::min(per, cap);
  });

  const int64_t grid = std::min<int64_t>(slots, p.total);
  hipLaunchKernelGGL(fe_mfma_mono_kernel, dim3((unsigned)grid), dim3(64), 0, st, p);
  return hipGetLastError();
}
