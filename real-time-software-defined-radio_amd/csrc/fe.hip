// RF front end for gfx950: interleaved IQ -> low-pass FIR -> keep every D-th
// output -> atan2 FM discriminator, fused in one pass over HBM.
//
// Replaces, per block:
//   model/fmMonoBlock.py:86-95  signal.lfilter(rf_coeff, 1.0, iq[0::2]/iq[1::2], zi) + [::10]
//   model/fmMonoBlock.py:98     fmDemodArctan(i_ds, q_ds, state_phase)  (model/fmSupportLib.py:15-44)
//   src/filter.cpp:187-219      convolveWithDecimIQ;  src/rf_module.cpp:13-34 fmDemodArctan
//   src/iofunc.cpp:61-69        u8 normalisation (u8 input variant)
//
// Algorithm per tile of TO = NT*R consecutive decimated outputs [m0, m0+TO):
//   1. The workgroup stages the input span n in [D(m0-1)-(T-1)-DELTA, D(m0+TO-1)] into
//      LDS as float2 (I,Q) with 16-B global loads (f32) or 16-B loads of 8 complex
//      u8 samples.  Only the decimated outputs are ever computed (spec p.5: no
//      9-of-10 wasted outputs as in the Python model).
//   2. Thread t owns R consecutive outputs and slides once over its D(R-1)+T input
//      window, so each LDS sample is read once per thread and feeds up to R outputs
//      (register blocking; taps are compile-time indices -> SGPR operands).
//      LDS rows are padded by one float2 every D*R samples so the per-lane stride
//      (D*R+1 float2 = odd number of 8-B slots) is bank-conflict free for ds_read_b64.
//   3. phi = atan2f(q, i); the predecessor phase of each lane comes from lane-1 by a
//      wave shuffle; lane 0 of each wave gets it from a wave-cooperative evaluation
//      of output m_w-1 (64 lanes x ceil(T/64) taps + xor-reduction), and the very
//      first output of a stream uses the carried prev_phase state in f64.
//   4. d = wrap(phi - phi_prev) reproduces np.unwrap on a 2-element list
//      (numpy _function_base_impl.py:1790-1800).  The number of
//      2*pi corrections W is reduced per stream so the host can return the
//      reference's accumulated (unwrapped) phase state: prev_out = phi_last + 2*pi*W.
#include "sdr_common.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace {

struct FeParams {
  const void* iq;            // device, interleaved IQ
  int64_t n;                 // complex samples per stream
  int64_t stride;            // complex samples between stream bases (multiple of G)
  int64_t hist;              // valid complex samples before index 0 of each stream
  int nstreams;
  int tiles_per_stream;
  const float* taps_dev;     // T taps (f32) for dynamically indexed use
  const double* zi_i;        // nullable: per stream (T-1) lfilter zi for I
  const double* zi_q;        // nullable
  int64_t zi_stride;
  const double* prev_phase;  // nullable (=> 0.0): per stream carried demod phase
  float* demod;              // per stream ceil(n/D) outputs
  int64_t out_stride;
  float* i_ds;               // nullable: decimated filtered I (for lfilter parity)
  float* q_ds;               // nullable
  float* last_phi;           // nullable: per stream atan2 phase of the last output
  int* wraps;                // nullable: per stream sum of 2*pi corrections
  int vec_out;               // 1 if out_stride % 4 == 0 and buffers 16-B aligned
};

template <bool U8> struct IqLoad;

// f32 interleaved: one 16-B load = 2 complex samples.
template <> struct IqLoad<false> {
  static constexpr int G = 2;
  using V = float4;
  __device__ static V load(const void* base, int64_t n) {  // n multiple of G
    return reinterpret_cast<const float4*>(base)[n >> 1];
  }
  __device__ static float2 get(const V& v, int j) {
    return j == 0 ? make_float2(v.x, v.y) : make_float2(v.z, v.w);
  }
  __device__ static float2 load1(const void* base, int64_t n) {
    return reinterpret_cast<const float2*>(base)[n];
  }
};

// u8 interleaved: one 16-B load = 8 complex samples, x = (u8 - 128) / 128 (exact).
template <> struct IqLoad<true> {
  static constexpr int G = 8;
  using V = uint4;
  __device__ static V load(const void* base, int64_t n) {
    return reinterpret_cast<const uint4*>(base)[n >> 3];
  }
  __device__ static float cvt(uint32_t b) { return ((float)b - 128.0f) * 0.0078125f; }
  __device__ static float2 get(const V& v, int j) {
    const uint32_t w = (j < 2) ? v.x : (j < 4) ? v.y : (j < 6) ? v.z : v.w;
    const int sh = (j & 1) * 16;
    return make_float2(cvt((w >> sh) & 0xff), cvt((w >> (sh + 8)) & 0xff));
  }
  __device__ static float2 load1(const void* base, int64_t n) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(base) + 2 * n;
    return make_float2(cvt(p[0]), cvt(p[1]));
  }
};

constexpr float kPiF = 3.14159265358979323846f;
constexpr float k2PiF = 6.28318530717958647692f;
constexpr double kPi = 3.14159265358979323846;
constexpr double k2Pi = 6.28318530717958647692;

// One step of np.unwrap([prev, cur]) in f64 (used where the carried state enters).
__device__ inline double unwrap_step_f64(double dd, int* w) {
  *w = 0;
  if (fabs(dd) < kPi) return dd;
  double m = fmod(dd + kPi, k2Pi);
  if (m < 0) m += k2Pi;
  double ddmod = m - kPi;
  if (ddmod == -kPi && dd > 0) ddmod = kPi;
  *w = (int)llrint((ddmod - dd) / k2Pi);
  return ddmod;
}

// Steps 3-5 shared by the FE kernels: zi add, atan2, predecessor phase (lane 0 gets the
// wave-reduced sums (si, sq) of output mw-1; lane l>0 shuffles from lane l-1), np.unwrap
// wrap, stores, wrap count and last phase.  Lane l of the wave owns outputs
// mw + R*l .. mw + R*l + R-1.
template <int T, int D, int R>
// If have_prev, phi_prev is the phase of output mw-1 (carried by a persistent wave from
// its previous tile) and (si, sq) are ignored.  Returns the phase of the wave's last
// output (lane 63's), broadcast to all lanes.  *one_store (if given) tells whether the
// tile issued exactly one vector-memory instruction (the full-width demod store); every
// other case (partial tile, zi/prev-phase loads, i_ds/q_ds, last_phi, wraps) ends with
// s_waitcnt vmcnt(0), so a streaming caller can count its outstanding loads exactly.
__device__ __forceinline__ float fe_epilogue(const FeParams& p, int s, int64_t M, int64_t mw, int lane,
                                             float (&ai)[R], float (&aq)[R], float si, float sq,
                                             bool have_prev = false, float phi_prev = 0.f,
                                             bool* one_store = nullptr, float* dv = nullptr,
                                             bool do_store = true) {
  const int64_t mf = mw + (int64_t)lane * R;       // first output of this lane
  const int64_t zoff = (int64_t)s * p.zi_stride;
  float phi[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t nn = D * (mf + r);
    if (p.zi_i != nullptr && nn < T - 1) {
      ai[r] += (float)p.zi_i[zoff + nn];
      aq[r] += (float)p.zi_q[zoff + nn];
    }
    phi[r] = fast_atan2f(aq[r], ai[r]);
  }
  float phi_wprev = phi_prev;
  if (mw > 0 && !have_prev) {
    const int64_t nn = D * (mw - 1);
    if (p.zi_i != nullptr && nn < T - 1) {
      si += (float)p.zi_i[zoff + nn];
      sq += (float)p.zi_q[zoff + nn];
    }
    phi_wprev = fast_atan2f(sq, si);
  }
  // lane l-1's last phase: DPP wave_shr:1 (a VALU move, no LDS round trip)
  const float from_left = __int_as_float(__builtin_amdgcn_update_dpp(
      0, __float_as_int(phi[R - 1]), 0x138 /*wave_shr:1*/, 0xf, 0xf, false));
  float prev = (lane == 0) ? phi_wprev : from_left;

  float d[R];
  int wsum = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t m = mf + r;
    int wk = 0;
    if (m == 0) {
      const double ps = p.prev_phase ? p.prev_phase[s] : 0.0;
      d[r] = (float)unwrap_step_f64((double)phi[r] - ps, &wk);
    } else {
      float dd = phi[r] - prev;
      if (dd > kPiF) { dd -= k2PiF; wk = -1; }
      else if (dd < -kPiF) { dd += k2PiF; wk = 1; }
      d[r] = dd;
    }
    if (m < M) wsum += wk;
    prev = phi[r];
  }

  if (dv != nullptr) {
#pragma unroll
    for (int r = 0; r < R; ++r) dv[r] = d[r];
  }
  // one full-width store per lane (a wave writes 64*R contiguous floats: whole cache
  // lines; per-float stores at an R*4-B lane stride cost partial-line writes)
  float* out = p.demod + (int64_t)s * p.out_stride;
  if (!do_store || p.demod == nullptr) {
  } else if (R == 4 && p.vec_out && mf + R <= M) {
    *reinterpret_cast<float4*>(out + mf) = make_float4(d[0], d[1 % R], d[2 % R], d[3 % R]);
  } else if (R == 2 && p.vec_out && mf + R <= M) {
    *reinterpret_cast<float2*>(out + mf) = make_float2(d[0], d[1 % R]);
  } else if (R == 3 && mf + R <= M) {
    typedef float f3v __attribute__((ext_vector_type(3)));
    *reinterpret_cast<f3v*>(out + mf) = f3v{d[0], d[1 % R], d[2 % R]};
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (mf + r < M) out[mf + r] = d[r];
  }
  if (p.i_ds != nullptr) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (mf + r < M) {
        p.i_ds[(int64_t)s * p.out_stride + mf + r] = ai[r];
        p.q_ds[(int64_t)s * p.out_stride + mf + r] = aq[r];
      }
  }
  if (p.last_phi != nullptr) {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (mf + r == M - 1) p.last_phi[s] = phi[r];
  }
  if (p.wraps != nullptr) {
    wsum = wave_sum_i(wsum);
    if (lane == 0 && wsum != 0) atomicAdd(p.wraps + s, wsum);
  }
  if (one_store != nullptr) {
    const int64_t mend = mw + 64 * R;   // wave-uniform
    const bool simple = mend <= M - 1 && D * (mw - 1) >= T - 1 && p.i_ds == nullptr && p.wraps == nullptr &&
                        (R == 3 || p.vec_out) && do_store && p.demod != nullptr;
    // no vector-memory instruction at all: nothing to wait for either
    const bool none = mend <= M - 1 && D * (mw - 1) >= T - 1 && p.i_ds == nullptr && p.wraps == nullptr &&
                      (!do_store || p.demod == nullptr);
    if (none) { *one_store = false; return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[R - 1]), 63)); }
    if (!simple) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *one_store = simple;
  }
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[R - 1]), 63));
}

// MODE (tuning builds only; the product uses 0): 1 = loads + LDS staging, no FIR;
// 2 = LDS staging of synthetic values + FIR, no global loads.
template <int T, int D, int R, int NT, bool U8, int MODE = 0>
__global__ __launch_bounds__(NT) void fe_kernel(FeParams p, TapsF32 taps) {
  using L8 = IqLoad<U8>;
  constexpr int G = L8::G;
  constexpr int TO = NT * R;                       // outputs per tile
  constexpr int DR = D * R;
  static_assert((DR % 2) == 0, "padded stride D*R+1 must be odd");
  static_assert((TO * D) % G == 0, "tile start must stay G-aligned");
  constexpr int SR = DR + 1;                       // padded per-lane stride (float2 slots)
  constexpr int DELTA = (G - ((D + T - 1) % G)) % G;
  constexpr int C0 = D + DELTA;                    // element of thread 0's first window sample
  constexpr int L = ((D * TO + DELTA + T) + G - 1) / G * G;
  constexpr int NSLOT = L + (L + DR - C0) / DR + 1;
  constexpr int NCHUNK = L / G;
  constexpr int NLOAD = (NCHUNK + NT - 1) / NT;
  constexpr int NI = D * (R - 1) + T;              // window length per thread

  __shared__ float2 lds[NSLOT];

  const int t = threadIdx.x;
  const int64_t blk = xcd_tile(blockIdx.x, gridDim.x);
  const int s = (int)(blk / p.tiles_per_stream);
  const int64_t tile = blk - (int64_t)s * p.tiles_per_stream;
  const int64_t m0 = tile * TO;
  const int64_t M = (p.n + D - 1) / D;             // lfilter(...)[::D] length
  const int64_t n_lo = D * (m0 - 1) - (T - 1) - DELTA;
  const char* base = reinterpret_cast<const char*>(p.iq) +
                     (int64_t)s * p.stride * (U8 ? 2 : 8);

  // ---- 1. stage the input span into padded LDS -------------------------------
  auto slot = [](int e) { return e + (e + DR - C0) / DR; };
  if (MODE == 2) {
    for (int e = t; e < L; e += NT) lds[slot(e)] = make_float2((float)e * 1e-4f, (float)t);
  } else if (n_lo >= -p.hist && n_lo + L <= p.n) {
    typename L8::V v[NLOAD];
#pragma unroll
    for (int j = 0; j < NLOAD; ++j) {
      const int q = t + j * NT;
      if (q < NCHUNK) v[j] = L8::load(base, n_lo + (int64_t)q * G);
    }
#pragma unroll
    for (int j = 0; j < NLOAD; ++j) {
      const int q = t + j * NT;
      if (q < NCHUNK) {
#pragma unroll
        for (int g = 0; g < G; ++g) lds[slot(q * G + g)] = L8::get(v[j], g);
      }
    }
  } else {
    for (int e = t; e < L; e += NT) {
      const int64_t nn = n_lo + e;
      float2 x = make_float2(0.f, 0.f);
      if (nn >= -p.hist && nn < p.n) x = L8::load1(base, nn);
      lds[slot(e)] = x;
    }
  }
  __syncthreads();

  // ---- 2. register-blocked sliding FIR over this thread's window -------------
  const float2* win = lds + (C0 + 1 + SR * t);
  float ai[R], aq[R];
#pragma unroll
  for (int r = 0; r < R; ++r) { ai[r] = 0.f; aq[r] = 0.f; }
#pragma unroll
  for (int i = 0; i < (MODE == 1 ? R : NI); ++i) {
    const float2 x = win[i + i / DR];
    if (MODE == 1) { ai[i] = x.x; aq[i] = x.y; continue; }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = D * r + T - 1 - i;             // tap index (compile time)
      if (k >= 0 && k < T) {
        const float h = taps.h[k];
        ai[r] = fmaf(h, x.x, ai[r]);
        aq[r] = fmaf(h, x.y, aq[r]);
      }
    }
  }

  // ---- 3. predecessor sums for lane 0 of each wave (output m_w - 1) -----------
  const int lane = t & 63;
  const int w = t >> 6;
  const int64_t mw = m0 + (int64_t)w * 64 * R;
  float si = 0.f, sq = 0.f;
  if (mw > 0) {
    for (int k = lane; k < T; k += 64) {
      const int e = D * w * 64 * R + (T - 1) + DELTA - k;
      const float2 x = lds[slot(e)];
      const float h = p.taps_dev[k];
      si = fmaf(h, x.x, si);
      sq = fmaf(h, x.y, sq);
    }
    si = wave_sum(si);
    sq = wave_sum(sq);
  }
  fe_epilogue<T, D, R>(p, s, M, mw, lane, ai, aq, si, sq);
}

// Register-blocked FIR of one tile image (see fe_stream_kernel): lane l produces the R
// decimated (I, Q) outputs of its window [D R l + D + DELTA, + D(R-1)+T).
// `hook(integral_constant<int, step>)` runs at the start of every step (sample pair):
// the steady ring loop uses it to spread the next tile's LDS-DMA issue over the FIR.
struct NoHook {
  template <typename I> __device__ __forceinline__ void operator()(I) const {}
};
template <int T, int D, int R, int MODE, int PF = 8, bool SAFEW = true, typename Hook = NoHook>
__device__ __forceinline__ void fe_fir_tile(const f2v* buf, int lane, const f2v (&tp)[(T + 1) / 2],
                                            float (&ai)[R], float (&aq)[R], Hook hook = Hook{}) {
  constexpr int DELTA = (2 - ((D + T - 1) % 2)) % 2;
  constexpr int NI = D * (R - 1) + T;
  const f2v* win = buf + (D * R * lane + D + DELTA);
  const float4* win4 = reinterpret_cast<const float4*>(__builtin_assume_aligned(win, 16));
  // two accumulator pairs per output (even / odd taps): 2R independent FMA chains per wave
  // (R == 1: two more, by tap index mod 4, so a lone wave is not latency-bound)
  constexpr int NA = (R == 1) ? 2 : 1;
  f2v acc[R * NA], acc2[R * NA];
#pragma unroll
  for (int r = 0; r < R * NA; ++r) { acc[r] = f2v{0.f, 0.f}; acc2[r] = f2v{0.f, 0.f}; }
  if (MODE == 1 || MODE == 3) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r * NA] = win[r];
  } else {
    // one ds_read_b128 per sample pair (the lane window starts 16-B aligned), issued by
    // hand PF pairs ahead of use with counted lgkmcnt waits: hipcc would split the 16-B
    // read into ds_read2_b64 (4-8-way bank conflicts at this lane stride) and read only
    // one pair ahead (the LDS latency then stalls the wave).
    constexpr int NP = (NI + 1) / 2;
    static_assert(PF >= 1 && PF <= 15, "lgkmcnt field");
    f4v qb[NP];
    // MODE 2 (tuning): no LDS reads, every step filters the same register values
    const f4v seed = f4v{1e-3f * lane, 2e-3f, 3e-3f, 4e-3f};
    auto rd = [&](auto I) {
      if constexpr (MODE == 2) qb[I] = seed;
      else qb[I] = lds_read_b128<16 * I>(win4);
    };
    static_for<0, (PF < NP ? PF : NP)>(rd);
    if constexpr (MODE == 2) {
    } else if constexpr (SAFEW) lds_wait<PF - 1 < NP - 1 ? PF - 1 : NP - 1>(qb[0]);
    else lds_wait_ordered<PF - 1 < NP - 1 ? PF - 1 : NP - 1>();
    static_for<0, NP>([&](auto I) {
      constexpr int ip = I;
      hook(I);
      // the wait "redefines" qb[ip] ("+v"): the register allocator may then not copy or
      // spill the in-flight value before the data has arrived (it costs one s_nop per
      // step: hipcc's gfx950 dst-forwarding hazard rule, applied conservatively to asm)
      // the read PF pairs ahead; qb[ip] itself was waited for one step earlier, so the
      // step's FMAs separate each wait from the first reader of its register
      if constexpr (ip + PF < NP) rd(std::integral_constant<int, ip + PF>{});
      const f4v q = qb[ip];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = 2 * ip + h;
        if (i >= NI) break;
        const f2v x = h ? f2v{q.z, q.w} : f2v{q.x, q.y};
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int k = D * r + T - 1 - i;
          if (k >= 0 && k < T) {
            const int a = (NA == 2) ? r * NA + ((k >> 1) & 1) : r;
            // hand-written v_pk_fma_f32 with an op_sel tap broadcast.  (The compiler's own
            // packed FMA folds the broadcast too, but then reschedules the whole loop into
            // ~370 registers with AGPR spills; as inline asm each step costs one s_nop.)
            if (k & 1) pk_fma_bcast<true>(acc2[a], tp[k >> 1], x);
            else pk_fma_bcast<false>(acc[a], tp[k >> 1], x);
          }
        }
      }
      // wait for the next step's pair: reads issued so far = min(ip + PF + 1, NP).
      // SAFEW: "+v" form (the allocator cannot copy the in-flight register; costs an s_nop
      // per step, see sdr_common.h); else an operand-free wait, valid because every reader
      // is a volatile asm and the kernel's register use leaves the allocator no reason to
      // copy (r01: T=101 at 231 VGPRs; the parity tests check each compiled kernel).
      if constexpr (ip + 1 < NP && MODE != 2) {
        constexpr int issued_r = (ip + PF + 1 < NP) ? ip + PF + 1 : NP;
        if constexpr (SAFEW) lds_wait<issued_r - (ip + 2)>(qb[ip + 1]);
        else lds_wait_ordered<issued_r - (ip + 2)>();
      }
    });
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    f2v t = acc[r * NA] + acc2[r * NA];
    if constexpr (NA == 2) t += acc[r * NA + 1] + acc2[r * NA + 1];
    ai[r] = t.x;
    aq[r] = t.y;
  }

}

// FE FIR of one R=3 tile (as fe_fir_tile) with the previous audio block's 3-output-per-
// lane audio FIR interleaved step by step (fe_ring_kernel<FUSED>, steady path): the audio
// reads (lane samples by ds_read2_b32, tap triples by broadcast ds_read_b128) are latency-
// bound on their own, the FE FIR is VALU-bound; interleaved, each covers the other.
// One static schedule: macro-step t runs FE step t and audio steps [NS*t/NP, NS*(t+1)/NP);
// reads are issued PF (FE) / APF (audio) steps ahead and every wait counts the reads
// issued after the one it needs (all compile-time; lgkmcnt <= 15 is asserted).
namespace fa {
template <int NP, int NS, int PF, int APF>
struct Sched {
  static constexpr int ab(int t) { return (NS * t) / NP; }               // first audio step of t
  static constexpr int pro() { return (PF < NP ? PF : NP) + 3 * (APF < NS ? APF : NS); }
  static constexpr int issued_at(int t) {                                 // reads issued in t
    int n = (t + PF < NP) ? 1 : 0;
    for (int k = ab(t); k < ab(t + 1); ++k) n += (k + APF < NS) ? 3 : 0;
    return n;
  }
  static constexpr int cum(int t) {                                       // after t's issue phase
    int n = pro();
    for (int u = 0; u <= t; ++u) n += issued_at(u);
    return n;
  }
  static constexpr int pos_fir(int ip) { return ip < PF ? ip : cum(ip - PF - 1); }
  static constexpr int pos_aud(int k) {
    if (k < APF) return (PF < NP ? PF : NP) + 3 * k;
    const int ki = k - APF;                                               // issued with step ki
    int t = 0;
    while (!(ki >= ab(t) && ki < ab(t + 1))) ++t;
    int n = cum(t - 1) + ((t + PF < NP) ? 1 : 0);
    for (int kk = ab(t); kk < ki; ++kk) n += (kk + APF < NS) ? 3 : 0;
    return n;
  }
  static constexpr int wait_fir(int t) { return cum(t) - (pos_fir(t) + 1); }
  static constexpr int wait_aud(int t, int k) { return cum(t) - (pos_aud(k) + 3); }
};
template <int v> struct CW { static_assert(v >= 0 && v <= 15, "lgkmcnt field"); static constexpr int value = v; };
}  // namespace fa

template <int T, int PF, int APF, typename Hook = NoHook>
__device__ __forceinline__ void fir_audio_tile(const f2v* buf, int lane, const f2v (&tp)[(T + 1) / 2],
                                               float (&ai)[3], float (&aq)[3], const float* aw,
                                               const f4v* ptab, float& o0, float& o1, float& o2,
                                               Hook hook = Hook{}) {
  constexpr int D = 10, R = 3;
  constexpr int NI = D * (R - 1) + T;
  constexpr int NP = (NI + 1) / 2;                   // FE steps (sample pairs)
  constexpr int NS = 81;                             // audio steps (161-sample window in pairs)
  using S = fa::Sched<NP, NS, PF, APF>;
  const f2v* win = buf + (D * R * lane + D);
  const float4* win4 = reinterpret_cast<const float4*>(__builtin_assume_aligned(win, 16));
  f2v acc[R], acc2[R];
#pragma unroll
  for (int r = 0; r < R; ++r) { acc[r] = f2v{0.f, 0.f}; acc2[r] = f2v{0.f, 0.f}; }
  f2v a01a = f2v{0.f, 0.f}, a01b = f2v{0.f, 0.f};
  float a2a = 0.f, a2b = 0.f;
  f4v qb[NP];
  f2v xq[NS];
  f4v ta[NS], tb[NS];
  auto rd_aud = [&](auto K) {
    constexpr int k = K;
    xq[k] = lds_read2_b32<2 * k, 2 * k + 1>(aw);
    ta[k] = lds_read_b128<32 * k>(ptab);
    tb[k] = lds_read_b128<32 * k + 16>(ptab);
  };
  static_for<0, (PF < NP ? PF : NP)>([&](auto I) { qb[I] = lds_read_b128<16 * I>(win4); });
  static_for<0, (APF < NS ? APF : NS)>(rd_aud);
  static_for<0, NP>([&](auto I) {
    constexpr int t = I;
    hook(I);
    if constexpr (t + PF < NP) qb[t + PF] = lds_read_b128<16 * (t + PF)>(win4);
    static_for<S::ab(t), S::ab(t + 1)>([&](auto K) {
      constexpr int k = K;
      if constexpr (k + APF < NS) rd_aud(std::integral_constant<int, k + APF>{});
    });
    lds_wait<fa::CW<S::wait_fir(t)>::value>(qb[t]);
    const f4v q = qb[t];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = 2 * t + h;
      if (i >= NI) break;
      const f2v x = h ? f2v{q.z, q.w} : f2v{q.x, q.y};
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int k = D * r + T - 1 - i;
        if (k >= 0 && k < T) {
          if (k & 1) pk_fma_bcast<true>(acc2[r], tp[k >> 1], x);
          else pk_fma_bcast<false>(acc[r], tp[k >> 1], x);
        }
      }
    }
    static_for<S::ab(t), S::ab(t + 1)>([&](auto K) {
      constexpr int k = K;
      lds_wait3<fa::CW<S::wait_aud(t, k)>::value>(xq[k], ta[k], tb[k]);
      pk_fma_bcast_x_ordered<false>(a01a, f2v{ta[k].x, ta[k].y}, xq[k]);
      pk_fma_bcast_x_ordered<true>(a01b, f2v{tb[k].x, tb[k].y}, xq[k]);
      fmac_ordered(a2a, ta[k].z, xq[k].x);
      fmac_ordered(a2b, tb[k].z, xq[k].y);
    });
  });
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const f2v t = acc[r] + acc2[r];
    ai[r] = t.x;
    aq[r] = t.y;
  }
  o0 = a01a.x + a01b.x;
  o1 = a01a.y + a01b.y;
  o2 = a2a + a2b;
}

// Persistent streaming f32 front end: the product kernel for f32 IQ.
//
// One wave per workgroup and WPC resident waves per CU; each wave walks a contiguous
// run of tiles (TO = 64*R decimated outputs each).  Tile images go HBM -> LDS through
// an NB-deep ring filled by 16-B LDS-DMA loads (global_load_lds_dwordx4, 1 KB per
// wave-instruction, no staging registers): tile t+1 is in flight while tile t is
// filtered (tools/mem_probe.hip: this pattern streams at 6.2-6.4 TB/s on its own).
// FIR: v_pk_fma_f32 on (I, Q) pairs; the taps stay in VGPR pairs {h[2j], h[2j+1]} for
// the whole launch and each FMA broadcasts one half through op_sel, so an output costs
// T packed FMAs and no moves.  Lane l filters samples [D R l + D + DELTA, + D(R-1)+T)
// of the tile image; the per-lane stride D*R*8 B (240 B at R=3, 400 B at R=5) puts the
// 16 lanes of each ds_read_b128 group on 16 distinct 16-B bank slots (conflict-free).
// The predecessor phase of a tile is carried from the wave's previous tile (only the
// first tile of a wave evaluates output m0-1 cooperatively).
// The ring is dynamic LDS so the compiler's occupancy target comes from
// amdgpu_waves_per_eu(2): a 256-register budget that keeps the taps (T/2 VGPR pairs)
// plus a bounded window of in-flight LDS reads, instead of hoisting every read.
template <int T, int D, int R, int NB, int MODE = 0>
__global__ __launch_bounds__(64)
void fe_stream_kernel(FeParams p, TapsF32 taps, int64_t total_tiles) {
  constexpr int TO = 64 * R;
  constexpr int G = 2;
  constexpr int DELTA = (G - ((D + T - 1) % G)) % G;
  constexpr int LRAW = D * TO + T + DELTA;
  constexpr int NG = (LRAW + 127) / 128;             // LDS-DMA wave-instructions per tile
  constexpr int L = NG * 128;
  constexpr int LB = L + 2;                          // buffer stride (f2v); +2: last pair over-read
  constexpr int NI = D * (R - 1) + T;
  constexpr int TP = (T + 1) / 2;
  static_assert(((D * R) % 2) == 0 && ((D + DELTA) % 2) == 0, "lane windows must start 16-B aligned");
  static_assert(NG * (NB - 1) <= 63, "vmcnt range");

  __shared__ __attribute__((aligned(16))) f2v lds[NB * LB];

  const int lane = threadIdx.x;
  const int64_t nw = gridDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * total_tiles / nw;
  const int64_t t1 = ((int64_t)blockIdx.x + 1) * total_tiles / nw;
  if (t0 >= t1) return;
  const int64_t M = (p.n + D - 1) / D;

  f2v tp[TP];
#pragma unroll
  for (int j = 0; j < TP; ++j) tp[j] = f2v{taps.h[2 * j], (2 * j + 1 < T) ? taps.h[2 * j + 1] : 0.f};
#pragma unroll
  for (int j = 0; j < TP; ++j) asm volatile("" : "+v"(tp[j]));   // keep taps in VGPRs

  // (stream, first output) of tile t0, advanced incrementally
  int s = (int)(t0 / p.tiles_per_stream);
  int64_t m0 = (t0 - (int64_t)s * p.tiles_per_stream) * TO;
  auto interior = [&](int ss, int64_t mm) {
    const int64_t n_lo = D * (mm - 1) - (T - 1) - DELTA;
    return MODE != 2 && n_lo >= -p.hist && n_lo + L <= p.n;
  };
  auto issue = [&](int ss, int64_t mm, int b) {
    const int64_t n_lo = D * (mm - 1) - (T - 1) - DELTA;
    const float* g = reinterpret_cast<const float*>(p.iq) + 2 * ((int64_t)ss * p.stride + n_lo) + 4 * lane;
#pragma unroll
    for (int j = 0; j < NG; ++j)
      __builtin_amdgcn_global_load_lds(g + 256 * j,
                                       (__attribute__((address_space(3))) void*)(lds + b * LB + 128 * j),
                                       16, 0, 2 /* nt: streamed once, do not keep in L2 */);
  };
  auto advance = [&](int& ss, int64_t& mm) {
    mm += TO;
    if (mm >= (int64_t)p.tiles_per_stream * TO) { mm = 0; ++ss; }
  };

  bool issued = interior(s, m0);
  if (issued) issue(s, m0, 0);
  float carry = 0.f;
  bool have = false;
  bool store_pending = false;
  int b = 0;
  for (int64_t t = t0; t < t1; ++t) {
    int s1 = s;
    int64_t m1 = m0;
    advance(s1, m1);
    const int bn = (b + 1 == NB) ? 0 : b + 1;
    const bool next = (t + 1 < t1) && interior(s1, m1);
    if (next) issue(s1, m1, bn);
    f2v* buf = lds + b * LB;
    if (issued) {
      // outstanding, oldest first: this tile's NG loads, the previous tile's demod store
      // (when the epilogue reported exactly one), the next tile's NG loads
      if (next && store_pending) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NG + 1) : "memory");
      else if (next) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NG) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      const int64_t n_lo = D * (m0 - 1) - (T - 1) - DELTA;
      const float* base = reinterpret_cast<const float*>(p.iq) + 2 * ((int64_t)s * p.stride);
      for (int e = lane; e < L; e += 64) {
        const int64_t nn = n_lo + e;
        f2v x = f2v{0.f, 0.f};
        if (MODE == 2) x = f2v{(float)e * 1e-4f, (float)lane};
        else if (nn >= -p.hist && nn < p.n) x = f2v{base[2 * nn], base[2 * nn + 1]};
        buf[e] = x;
      }
    }

    float ai[R], aq[R];
    fe_fir_tile<T, D, R, MODE>(buf, lane, tp, ai, aq);

    float si = 0.f, sq = 0.f;
    if (MODE != 3 && m0 > 0 && !have) {
      for (int k = lane; k < T; k += 64) {
        const f2v x = buf[(T - 1) + DELTA - k];
        const float h = p.taps_dev[k];
        si = fmaf(h, x.x, si);
        sq = fmaf(h, x.y, sq);
      }
      si = wave_sum(si);
      sq = wave_sum(sq);
    }
    if (MODE == 3) {   // tuning: no epilogue, raw store
      *reinterpret_cast<float2*>(p.demod + (int64_t)s * p.out_stride + m0 + R * lane) = make_float2(ai[0], aq[0]);
      store_pending = true;
    } else {
      carry = fe_epilogue<T, D, R>(p, s, M, m0, lane, ai, aq, si, sq, have, carry, &store_pending);
    }
    have = (s1 == s);          // the next tile continues this stream
    s = s1;
    m0 = m1;
    issued = next;
    b = bn;
  }
}

// ---------------------------------------------------------------------------------
// fe_ring_kernel: the product f32 front end (R = 3 outputs per lane, TO = 192 per tile).
//
// Differences from fe_stream_kernel (r01 profile: 178 SALU + 338 VALU per 128-output
// tile, 2-way LDS bank conflicts at the R=2 lane stride, 7 waves/CU spread 2-2-2-1 over
// the SIMDs, 1.087x the algorithmic HBM reads):
//  * R = 3: the lane stride (30 samples = 15 x 16 B, odd) puts every ds_read_b128 lane
//    group on 16 distinct bank quads -> conflict-free, and 20 LDS reads per output
//    instead of 28;
//  * halo reuse: consecutive tiles of a wave overlap by NCH-15 chunks; only the 15 new
//    1-KiB chunks are DMA'd and the halo is copied LDS->LDS (HBM bytes = algorithmic);
//  * LDS-DMA in the saddr form with immediate chunk offsets (glds16), exact vmcnt
//    accounting through a running issue counter, 32-bit per-tile index math;
//  * a fast epilogue for interior tiles (atan2, DPP predecessor, wrap, one 12-B store per
//    lane, wrap counts kept per lane and reduced once per stream segment); head/tail
//    tiles, zi, i_ds/q_ds and last_phi go through the general fe_epilogue;
//  * 4 resident waves per CU = one per SIMD (LDS: 2 x 16 KiB ring per wave).
// ---------------------------------------------------------------------------------
#ifndef RING_PF
#define RING_PF 12
#endif
#ifndef RING_STG             // steady loop: VGPR-staged prefetch depth (0 = LDS-DMA, 1 ahead)
#define RING_STG 0
#endif
#ifndef RING_SPREAD          // steady loop: spread the next tile's DMA issue over the FIR
#define RING_SPREAD 1
#endif
#ifndef RING_SPREAD_T0       // first FIR step that issues a group of 4 chunks
#define RING_SPREAD_T0 2
#endif
#ifndef RING_SPREAD_DT       // FIR steps between groups
#define RING_SPREAD_DT 8
#endif
struct RingArgs {
  int64_t total;       // work units: tiles (FE), or audio blocks (FUSED), over all streams
  int per_wave;        // units per wave (contiguous run)
  int tps;             // tiles per stream in the tile sequence
  int ab;              // FUSED: audio blocks per stream
  float* audio;        // FUSED: per stream ceil(M/DA) audio samples, audio_stride apart
  int64_t audio_stride;
  const float* ataps;  // FUSED: TA audio taps (device)
};

// FUSED = the continuous-stream mono receiver (sdr_fe_mono_dev): an audio block is DA
// tiles = 960 demod samples = 192 audio outputs (RA = 3 per lane).  Demod values go to
// a wave-private LDS history instead of HBM; after a block's last tile lane l computes
// audio outputs 3l..3l+2 of the block:  a[j] = sum_k g[k] d[5j - k].  A wave whose run
// starts mid-stream first runs one warm-up tile (192 >= TA-1 demod samples of history).
template <int T, bool FUSED = false, int MODE = 0>
__global__ __launch_bounds__(64)
void fe_ring_kernel(FeParams p, TapsF32 taps, RingArgs a) {
  // MODE = MB | (SV << 4): MB selects tuning ablations (0 = product), SV a DMA-issue
  // schedule for A/B runs in one process (0 = the RING_SPREAD* defaults)
  constexpr int MB = MODE & 15, SV = (MODE >> 4) & 15;
  // steady-loop ablations (tuning only): 0x100 trivial epilogue, 0x200 no audio FIR,
  // 0x400 FE FIR without LDS reads
  constexpr bool AB_NOEPI = MODE & 0x100, AB_NOAUD = MODE & 0x200, AB_NOLDS = MODE & 0x400;
  constexpr int FM = AB_NOLDS ? 2 : 0;
  // steady-loop prefetch: STG = 0 -> the next tile by LDS-DMA (one tile ahead); STG >= 2 ->
  // tiles t+1..t+STG by 16-B loads into VGPR stages, written to the free LDS slot by the
  // wave after the FIR of tile t (STG tiles in flight instead of one)
  constexpr int STG = (MODE & 0x3000) ? (((MODE >> 12) & 3) + 1) : RING_STG;

  // A/B overrides (0 = defaults): bits 16-19 FE-FIR reads in flight, 20-22 / 24-26 the
  // interleaved FE / audio read depths, 0x8000 operand-free LDS waits in the FE FIR
  constexpr int PFR = ((MODE >> 16) & 15) ? ((MODE >> 16) & 15) : RING_PF;
  constexpr int FPF = ((MODE >> 20) & 7) ? ((MODE >> 20) & 7) : 2;
  constexpr int APFX = ((MODE >> 24) & 7) ? ((MODE >> 24) & 7) : 2;
  constexpr bool SAFE = !(MODE & 0x8000);
  // A/B (tuning): 0x20000000 touches tile t+PFD's new lines (one dword per 128-B line, LDS-DMA
  // into a 256-B scratch, no VGPR destination) after the FIR of tile t, so its later DMA
  // finds them in L2 / MALL; PFD = 2, or 3 with 0x40000000
  constexpr bool PFL2 = MODE & 0x20000000;
  constexpr int PFD = (MODE & 0x40000000) ? 3 : 2;
  constexpr int SPR = SV == 0 ? RING_SPREAD : (SV == 1 ? 0 : 1);
  constexpr int ST0 = SV == 0 ? RING_SPREAD_T0 : (SV == 3 ? 4 : 2);
  constexpr int SDT = SV == 0 ? RING_SPREAD_DT : (SV == 2 ? 4 : (SV == 3 ? 14 : 8));
  constexpr int D = 10, R = 3, TO = 64 * R;
  constexpr int NEWC = D * TO / 128;                 // 15 new 1-KiB chunks per tile
  constexpr int NCH = (D * TO + T + 1 + 127) / 128;  // chunks per tile image
  constexpr int HCH = NCH - NEWC;                    // halo chunks shared with the next tile
  constexpr int L = NCH * 128;                       // image length (complex samples)
  constexpr int TP = (T + 1) / 2;
  static_assert((T & 1) == 1 && HCH >= 1 && HCH <= 2, "odd tap counts 101..235");
  static_assert(D * TO % 128 == 0, "tiles advance by whole chunks");
  // audio (FUSED): TA = 151 taps, DA = 5
  constexpr int TA = 151, DA = 5, RA = R;
  constexpr int TPB = DA;                            // tiles per audio block
  constexpr int BD = TO * TPB;                       // 960 demod samples per block
  constexpr int BO = 64 * RA;                        // 192 audio outputs per block
  constexpr int HA = 152;                            // history slots (>= TA-1)
  constexpr int NW = DA * (RA - 1) + TA;             // 161-sample audio window per lane
  static_assert(BD == DA * BO, "block bookkeeping");

  // slot stride >= 20 KiB: at most 4 resident waves per CU (one per SIMD; a 5th wave would
  // double one SIMD's load and set the pace of the whole launch)
  constexpr int LS = FUSED ? L : (L > 2560 ? L : 2560);
  __shared__ __attribute__((aligned(16))) f2v ring[2][LS];
  __shared__ __attribute__((aligned(16))) float dh[FUSED ? HA + BD + 4 : 1];
  __shared__ __attribute__((aligned(16))) f4v ptab[FUSED ? NW + 1 : 1];
  __shared__ __attribute__((aligned(16))) float pfs[PFL2 ? 64 : 1];

  const int lane = threadIdx.x;
  // FUSED: balanced tile ranges [g0, g1) over a.total tiles; FE: runs of per_wave tiles
  const int64_t g0 = FUSED ? (int64_t)blockIdx.x * a.total / gridDim.x : (int64_t)blockIdx.x * a.per_wave;
  const int64_t g1 = FUSED ? ((int64_t)blockIdx.x + 1) * a.total / gridDim.x : min<int64_t>(g0 + a.per_wave, a.total);
  if (g0 >= g1) return;
  const int64_t u0 = g0;
  const int nunits = (int)(g1 - g0);
  const int64_t M = (p.n + D - 1) / D;

  f2v tp[TP];
#pragma unroll
  for (int j = 0; j < TP; ++j) tp[j] = f2v{taps.h[2 * j], (2 * j + 1 < T) ? taps.h[2 * j + 1] : 0.f};
#pragma unroll
  for (int j = 0; j < TP; ++j) asm volatile("" : "+v"(tp[j]));

  const unsigned voff = 16u * lane;
  const float* iqf = reinterpret_cast<const float*>(p.iq);
  // tile (s, i): outputs m0 = TO*i ..; image = samples [n_lo, n_lo + L) of stream s,
  // n_lo = D*(m0-1) - (T-1) (output m0-1's window first, for the predecessor)
  auto n_lo_of = [&](int i) { return (int64_t)(D * TO) * i - D - (T - 1); };
  auto interior = [&](int64_t nl) { return MB != 2 && nl >= -p.hist && nl + L <= p.n; };
  // issue chunks [0 or HCH, NCH) of tile image nl (stream s) into ring slot b
  auto issue = [&](int s, int64_t nl, int b, bool full) {
    const char* g = reinterpret_cast<const char*>(iqf + 2 * ((int64_t)s * p.stride + nl));
    const unsigned lb = lds_addr_of(&ring[b][0]);
    auto run = [&](auto C0) {
      constexpr int c0 = decltype(C0)::value;
      static_for<0, (NCH - c0 + 3) / 4>([&](auto Q) {
        constexpr int c = c0 + 4 * Q;
        constexpr int n = (NCH - c) < 4 ? (NCH - c) : 4;
        glds16x<n>(voff, g + 1024 * c, lb + 1024 * c);
      });
    };
    if (full) run(std::integral_constant<int, 0>{});
    else run(std::integral_constant<int, HCH>{});
  };

  // tile sequence of this wave
  int s, i, U;
  bool mid = false;
  if constexpr (FUSED) {
    // a run starting mid-stream first runs the warm-up tile i0-1 (history / predecessor);
    // a run may start and end mid audio block (audio_store keeps to the outputs it owns)
    s = (int)(u0 / a.tps);
    const int i0 = (int)(u0 - (int64_t)s * a.tps);
    mid = i0 > 0;
    i = i0 - (mid ? 1 : 0);
    U = nunits + (mid ? 1 : 0);
    for (int e = lane; e < HA + BD + 4; e += 64) dh[e] = 0.f;   // finite everywhere (0 * x)
    for (int w = lane; w < NW + 1; w += 64) {               // entry NW: zero (pairs over-read)
      const int k0 = (TA - 1) - w, k1 = k0 + DA, k2 = k0 + 2 * DA;
      ptab[w] = f4v{(k0 >= 0 && k0 < TA) ? a.ataps[k0] : 0.f, (k1 >= 0 && k1 < TA) ? a.ataps[k1] : 0.f,
                    (k2 >= 0 && k2 < TA) ? a.ataps[k2] : 0.f, 0.f};
    }
  } else {
    s = (int)(u0 / a.tps);
    i = (int)(u0 - (int64_t)s * a.tps);
    U = nunits;
  }
  int64_t nl = n_lo_of(i);
  // kinds: 0 none, 1 guarded (built with plain loads at compute time), 2 DMA full, 3 DMA halo
  int kind = interior(nl) ? 2 : 1;
  int issued = 0, mark = 0;
  if (kind == 2) { issue(s, nl, 0, true); issued += NCH; mark = issued; }
  float carry = 0.f;
  bool have = false;
  int wacc = 0;
  int b = 0;
  // MB 6 (tuning): per-phase s_memtime accounting -> p.q_ds as uint64[grid][8]
  uint64_t tph[6] = {0, 0, 0, 0, 0, 0};
  uint64_t tlast = 0;
  auto stamp = [&](int k) {
    if constexpr (MB == 6) {
      uint64_t t;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
      if (k >= 0) tph[k] += t - tlast;
      tlast = t;
    }
  };
  // FUSED: demod values of tile (i) -> history; after the block's last tile, the block's
  // audio outputs (lane l: 3l..3l+2) and the history shift.  `next_same`: the following
  // tile continues this stream.
  // FUSED audio pieces: the block's outputs (lane l: 3l..3l+2) from the history, their
  // store (returns true if it drained vmcnt), and the history shift / reset
  const float* aw_lane = dh + (HA - (TA - 1) + DA * RA * lane);   // lane window in dh
  auto audio_compute = [&](float& o0, float& o1, float& o2) {
    asm volatile("" ::: "memory");
    // hand-pipelined like the FIR: per step k (samples 2k, 2k+1) one ds_read2_b32 of the
    // lane's samples + two broadcast ds_read_b128 of tap triples, APF steps ahead
    f2v acc01a = f2v{0.f, 0.f}, acc01b = f2v{0.f, 0.f};
    float a2a = 0.f, a2b = 0.f;
    constexpr int NS = (NW + 1) / 2, APF = 5;   // 3*APF <= 15 (lgkmcnt field)
    f2v xq[NS];
    f4v ta[NS], tb[NS];
    auto rd = [&](auto K) {
      constexpr int k = K;
      xq[k] = lds_read2_b32<2 * k, 2 * k + 1>(aw_lane);
      ta[k] = lds_read_b128<32 * k>(ptab);
      tb[k] = lds_read_b128<32 * k + 16>(ptab);
    };
    static_for<0, APF>(rd);
    static_for<0, NS>([&](auto K) {
      constexpr int k = K;
      if constexpr (k + APF < NS) {
        rd(std::integral_constant<int, k + APF>{});
        lds_wait3<3 * APF>(xq[k], ta[k], tb[k]);
      } else {
        lds_wait3<3 * (NS - 1 - k)>(xq[k], ta[k], tb[k]);
      }
      pk_fma_bcast_x_ordered<false>(acc01a, f2v{ta[k].x, ta[k].y}, xq[k]);
      pk_fma_bcast_x_ordered<true>(acc01b, f2v{tb[k].x, tb[k].y}, xq[k]);
      fmac_ordered(a2a, ta[k].z, xq[k].x);
      fmac_ordered(a2b, tb[k].z, xq[k].y);
    });
    o0 = acc01a.x + acc01b.x;
    o1 = acc01a.y + acc01b.y;
    o2 = a2a + a2b;
  };
  auto audio_store = [&](int64_t q, float o0, float o1, float o2) -> bool {
    // outputs of stream s this run owns: 5 j inside its tile range (each output is
    // stored by exactly one wave)
    const int64_t lo = max<int64_t>(g0 - (int64_t)s * a.tps, 0);
    const int64_t hi = min<int64_t>(g1 - (int64_t)s * a.tps, a.tps);
    const int64_t jlo = (TO * lo + DA - 1) / DA;
    const int64_t A = min<int64_t>((TO * hi + DA - 1) / DA, (M + DA - 1) / DA);
    const int64_t j = q * BO + RA * lane;
    float* ao = a.audio + (int64_t)s * a.audio_stride + j;
    if (q * BO >= jlo && q * BO + BO <= A) {
      typedef float f3v __attribute__((ext_vector_type(3)));
      *reinterpret_cast<f3v*>(ao) = f3v{o0, o1, o2};
      issued += 1;
      return false;
    }
    if (j >= jlo && j < A) ao[0] = o0;
    if (j + 1 >= jlo && j + 1 < A) ao[1] = o1;
    if (j + 2 >= jlo && j + 2 < A) ao[2] = o2;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    issued = 0;
    return true;
  };
  auto dh_shift = [&](bool next_same) {
    asm volatile("" ::: "memory");
    if (!next_same)
      for (int e = lane; e < HA; e += 64) dh[e] = 0.f;     // next block starts a new stream
    else
      for (int e = lane; e < HA; e += 64) dh[e] = dh[BD + e];
    asm volatile("" ::: "memory");
  };
  auto dh_write = [&](int i, bool warm, const float (&d)[R]) {
    const int ib = i - TPB * (i / TPB);            // tile within its audio block (warm-up: 4)
    const int rel0 = (warm ? -TO : ib * TO) + R * lane;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (rel0 + r >= -HA) dh[HA + rel0 + r] = d[r];
  };
  // FUSED (general path): demod values of tile i -> history; after the block's last tile,
  // the block's audio outputs and the history shift.  Returns true if vmcnt was drained.
  auto fused_tail = [&](int i, bool warm, const float (&d)[R], bool next_same, bool last = false) -> bool {
    dh_write(i, warm, d);
    const int ib = i - TPB * (i / TPB);
    if (warm || (ib != TPB - 1 && !last)) return false;
    float o0, o1, o2;
    audio_compute(o0, o1, o2);
    const bool drained = audio_store(i / TPB, o0, o1, o2);
    dh_shift(next_same);
    return drained;
  };
  // fast epilogue of an interior tile: phases, predecessor (DPP / carry), np.unwrap wrap
  auto fast_epi = [&](const float (&ai)[R], const float (&aq)[R], float (&d)[R]) {
    float phi[R];
#pragma unroll
    for (int r = 0; r < R; ++r) phi[r] = fast_atan2f(aq[r], ai[r]);
    const float from_left = __int_as_float(__builtin_amdgcn_update_dpp(
        0, __float_as_int(phi[R - 1]), 0x138 /*wave_shr:1*/, 0xf, 0xf, false));
    float prev = (lane == 0) ? carry : from_left;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float dd = phi[r] - prev;
      if (dd > kPiF) { dd -= k2PiF; wacc -= 1; }
      else if (dd < -kPiF) { dd += k2PiF; wacc += 1; }
      d[r] = dd;
      prev = phi[r];
    }
    carry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[R - 1]), 63));
  };
  auto wait_tile = [&](int nw) {                   // VMEM ops issued after the tile's loads
    if (nw == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (nw == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if (nw == NEWC) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NEWC) : "memory");
    else if (nw == NEWC + 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NEWC + 1) : "memory");
    else wait_vm_chain(nw);
  };
  // tile-index limits of the steady (fast) path, per stream: image interior (DMA) and
  // fast epilogue (full tile strictly before the last output)
  const int64_t j_int = (p.n + D + (T - 1) - L) / (D * TO);
  const int64_t j_fast = M >= TO + 1 ? (M - TO - 1) / TO : -1;
  // ---- staged steady run (STG >= 2): tiles i .. i+K-1 of stream s, all interior ----
  // Entry: tile i's image is in slot b (LDS-DMA in flight, counted by `mark`), or resident
  // (kind 4).  Tile i+j (j >= 1) is loaded into VGPR stage j % STG; after the FIR of tile t
  // the wave waits for stage (t+1) % STG, writes it to the other slot (plus the halo chunk
  // from this slot), and reuses the stage for tile t+1+STG.  Exit: tile i+K resident in
  // slot b (b, i, nl advanced by K); no loads outstanding.
  static_assert(STG == 0 || (STG >= 2 && STG * NEWC + 2 <= 63), "stages (vmcnt is 6-bit)");
  f4v stg[STG > 0 ? STG : 1][NEWC];
  auto staged_run = [&](int64_t K) {
    if constexpr (STG > 0) {
      const unsigned voff16 = 16u * lane;
      const char* gl = reinterpret_cast<const char*>(iqf + 2 * ((int64_t)s * p.stride + nl + D * TO)) + 1024 * HCH;
      int smark[STG];
      auto load_stage = [&](auto SQ) {       // next tile to load -> stage SQ; advances gl
        constexpr int sq = SQ;
        static_for<0, NEWC>([&](auto C) {
          constexpr int c = C;
          gload16_nt_a<1024 * (c % 4)>(stg[sq][c], voff16, gl + 4096 * (c / 4));
        });
        gl += D * TO * 8;
        issued += NEWC;
        smark[sq] = issued;
      };
      const bool resident = (kind == 4);
      const int mark0 = mark;
      static_for<1, STG + 1>([&](auto J) {
        constexpr int j = J;
        if (j <= K) load_stage(std::integral_constant<int, j % STG>{});
      });
      if (!resident) wait_tile(issued - mark0);
      float* outp = FUSED ? nullptr : p.demod + (int64_t)s * p.out_stride + (int64_t)TO * i + R * lane;
      bool pend = false;
      int64_t q_pend = 0;
      auto body = [&](auto Q, int64_t kk) {
        constexpr int sn = (Q + 1) % STG;      // stage of tile kk+1
        f2v* buf = &ring[b][0];
        f2v* nb = &ring[b ^ 1][0];
        f4v h0 = lds_read_b128<0>(buf + NEWC * 128 + 2 * lane), h1;
        if constexpr (HCH == 2) h1 = lds_read_b128<0>(buf + (NEWC + 1) * 128 + 2 * lane);
        float ai[R], aq[R];
        bool aud_drained = false;
        if constexpr (FUSED && T <= 127) {
          if (pend) {
            float o0, o1, o2;
            fir_audio_tile<T, FPF, APFX>(buf, lane, tp, ai, aq, aw_lane, ptab, o0, o1, o2);
            aud_drained = audio_store(q_pend, o0, o1, o2);
            dh_shift(true);
            pend = false;
          } else {
            fe_fir_tile<T, D, R, 0, PFR, SAFE>(buf, lane, tp, ai, aq);
          }
        } else {
          fe_fir_tile<T, D, R, 0, (T > 127 ? 8 : PFR), SAFE>(buf, lane, tp, ai, aq);
        }
        // tile kk+1 -> the other slot (its halo from this slot); refill the stage
        {
          // steady state: the later stages' loads (+ a few stores) are still outstanding
          constexpr int LO = (STG - 1) * NEWC;
          const int nw = issued - smark[sn];
          bool done = false;
          static_for<LO, LO + STG + 2>([&](auto V) {
            constexpr int v = V;
            if (!done && nw == v) { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(v) : "memory"); done = true; }
          });
          if (!done) wait_tile(nw);
        }
        const unsigned na = lds_addr_of(nb) + 16u * lane;
        static_for<0, NEWC>([&](auto C) {
          constexpr int c = C;
          asm volatile("" : "+a"(stg[sn][c]));
          lds_write_b128_a<1024 * (HCH + c)>(na, stg[sn][c]);
        });
        lds_wait<0>(h0);
        lds_write_b128(nb + 2 * lane, h0);
        if constexpr (HCH == 2) { lds_wait<0>(h1); lds_write_b128(nb + 128 + 2 * lane, h1); }
        if (kk + 1 + STG <= K) load_stage(std::integral_constant<int, sn>{});
        float d[R];
        fast_epi(ai, aq, d);
        if constexpr (!FUSED) {
          typedef float f3v __attribute__((ext_vector_type(3)));
          *reinterpret_cast<f3v*>(outp) = f3v{d[0], d[1], d[2]};
          outp += TO;
          issued += 1;
        } else if constexpr (T <= 127) {
          dh_write(i, false, d);
          if (i - TPB * (i / TPB) == TPB - 1) { pend = true; q_pend = i / TPB; }
        } else {
          fused_tail(i, false, d, true);
        }
        (void)aud_drained;
        b ^= 1;
        ++i;
        nl += D * TO;
      };
      for (int64_t k = 0; k < K; k += STG)
        static_for<0, STG>([&](auto Q) {
          if (k + Q < K) body(Q, k + Q);
        });
      if constexpr (FUSED) {
        if (pend) {
          float o0, o1, o2;
          audio_compute(o0, o1, o2);
          audio_store(q_pend, o0, o1, o2);
          dh_shift(i < a.tps);
        }
      }
      mark = issued;
    }
  };
  stamp(-1);
  for (int u = 0; u < U; ++u) {
    if constexpr (MB == 0 || MB == 6) {
      // ---- steady run: consecutive interior tiles of one stream, fixed VMEM pattern ----
      if (kind >= 2 && have && i >= 1 && p.i_ds == nullptr) {
        int64_t K = min<int64_t>(U - 1 - u, a.tps - 1 - i);
        K = min<int64_t>(K, j_int - i);
        K = min<int64_t>(K, j_fast - i + 1);
        if (STG > 0 && K > 0) {
          staged_run(K);
          u += (int)K;
          kind = 4;                          // tile u is resident in slot b (written by the run)
        } else if (K > 0) {
          const char* gn = reinterpret_cast<const char*>(iqf + 2 * ((int64_t)s * p.stride + nl + D * TO)) + 1024 * HCH;
          float* outp = FUSED ? nullptr : p.demod + (int64_t)s * p.out_stride + (int64_t)TO * i + R * lane;
          bool pend = false;                 // FUSED: a finished block's audio not yet computed
          int64_t q_pend = 0;
          for (int k = 0; k < (int)K; ++k) {
            // the next tile's new chunks go into the other slot: issued up front, or (RING_SPREAD)
            // in groups of 4 spread over the FIR steps, so the VMEM queue never stalls the wave
            const unsigned lb = lds_addr_of(&ring[b ^ 1][0]) + 1024 * HCH;
            auto issue_grp = [&](auto Q) {
              constexpr int c = 4 * Q;
              constexpr int n = (NEWC - c) < 4 ? (NEWC - c) : 4;
              glds16x<n>(voff, gn + 1024 * c, lb + 1024 * c);
            };
            auto spread = [&](auto I) {
              constexpr int t = I;
              if constexpr (SPR && t >= ST0 && (t - ST0) % SDT == 0 && (t - ST0) / SDT < (NEWC + 3) / 4)
                issue_grp(std::integral_constant<int, (t - ST0) / SDT>{});
            };
            if constexpr (!SPR) static_for<0, (NEWC + 3) / 4>(issue_grp);
            const int mark1 = issued + NEWC;
            stamp(0);
            wait_tile(issued - mark + (SPR ? 0 : NEWC));
            issued += NEWC;
            stamp(1);
            f2v* buf = &ring[b][0];
            f4v h0 = lds_read_b128<0>(buf + NEWC * 128 + 2 * lane), h1;
            if constexpr (HCH == 2) h1 = lds_read_b128<0>(buf + (NEWC + 1) * 128 + 2 * lane);
            float ai[R], aq[R];
            bool aud_drained = false;
            if constexpr (FUSED && T <= 127) {
              if (pend) {                    // previous block's audio, interleaved into this FIR
                float o0, o1, o2;
                if constexpr (AB_NOAUD || AB_NOLDS) {
                  fe_fir_tile<T, D, R, FM, PFR, SAFE>(buf, lane, tp, ai, aq, spread);
                  o0 = ai[0]; o1 = ai[1]; o2 = ai[2];
                } else {
                  fir_audio_tile<T, FPF, APFX>(buf, lane, tp, ai, aq, aw_lane, ptab, o0, o1, o2, spread);
                }
                aud_drained = audio_store(q_pend, o0, o1, o2);
                dh_shift(true);
                pend = false;
              } else {
                fe_fir_tile<T, D, R, FM, (T > 127 ? 8 : PFR), SAFE>(buf, lane, tp, ai, aq, spread);
              }
            } else {
              fe_fir_tile<T, D, R, FM, (T > 127 ? 8 : PFR), SAFE>(buf, lane, tp, ai, aq, spread);
            }
            gn += D * TO * 8;
            if constexpr (PFL2) {
              if (i + PFD <= j_int) {        // tile i+PFD's image lies inside the stream
                // gn now points at tile i+2's new chunks (15 KiB = 120 lines: lanes 0..59)
                const char* gp = gn + (PFD - 2) * (D * TO * 8);
                asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1 offset:0\n\t"
                             "global_load_lds_dword %0, %1 offset:128"
                             :: "v"(lane < 60 ? 256u * lane : 0u), "s"(gp), "s"(lds_addr_of(pfs)) : "memory", "m0");
                issued += 2;
              }
            }
            lds_wait<0>(h0);
            lds_write_b128(&ring[b ^ 1][0] + 2 * lane, h0);
            if constexpr (HCH == 2) { lds_wait<0>(h1); lds_write_b128(&ring[b ^ 1][0] + 128 + 2 * lane, h1); }
            stamp(2);
            float d[R];
            if constexpr (AB_NOEPI) {
#pragma unroll
              for (int r = 0; r < R; ++r) d[r] = ai[r] + aq[r];
            } else {
              fast_epi(ai, aq, d);
            }
            stamp(3);
            if constexpr (!FUSED) {
              typedef float f3v __attribute__((ext_vector_type(3)));
              *reinterpret_cast<f3v*>(outp) = f3v{d[0], d[1], d[2]};
              outp += TO;
              issued += 1;
            } else {
              if constexpr (T <= 127) {
                dh_write(i, false, d);
                if (i - TPB * (i / TPB) == TPB - 1) { pend = true; q_pend = i / TPB; }
                if (aud_drained) { stamp(4); mark = 0; b ^= 1; ++i; nl += D * TO; continue; }
              } else {
                if (fused_tail(i, false, d, true)) { mark = 0; b ^= 1; ++i; nl += D * TO; continue; }
              }
            }
            stamp(4);
            mark = mark1;
            b ^= 1;
            ++i;
            nl += D * TO;
          }
          if constexpr (FUSED) {
            if (pend) {                      // flush: the block ended on the steady run's last tile
              float o0, o1, o2;
              audio_compute(o0, o1, o2);
              if (audio_store(q_pend, o0, o1, o2)) mark = 0;
              dh_shift(i < a.tps);           // i: the next tile (same stream unless past the end)
            }
          }
          u += (int)K;
          kind = 3;
          // (tile u now has its halo DMA issued; have stays true, s unchanged)
        }
      }
    }
    // ---- next tile: position, kind, issue ----
    int s1 = s, i1 = i + 1;
    if (i1 == a.tps) { i1 = 0; ++s1; }
    const int64_t nl1 = (s1 == s) ? nl + D * TO : n_lo_of(0);
    int kind1 = 0, mark1 = 0;
    if (u + 1 < U) {
      if (s1 == s && MB != 2 && MB != 5 && nl1 + L <= p.n && nl1 + HCH * 128 >= -p.hist) kind1 = 3;
      else kind1 = interior(nl1) ? 2 : 1;
      if (kind1 >= 2) {
        issue(s1, nl1, b ^ 1, kind1 == 2);
        issued += (kind1 == 2) ? NCH : NEWC;
        mark1 = issued;
      }
    }
    f2v* buf = &ring[b][0];
    const int64_t m0 = (int64_t)TO * i;
    stamp(0);
    // ---- this tile's image ----
    if (kind == 4) {
      // resident: written by the staged run (the FIR's LDS waits order it)
    } else if (kind >= 2) {
      wait_tile(issued - mark);
    } else {
      const float* base = iqf + 2 * ((int64_t)s * p.stride);
      for (int e = lane; e < L; e += 64) {
        const int64_t nn = nl + e;
        f2v x = f2v{0.f, 0.f};
        if (MB == 2) x = f2v{(float)e * 1e-4f, (float)lane};
        else if (nn >= -p.hist && nn < p.n) x = f2v{base[2 * nn], base[2 * nn + 1]};
        buf[e] = x;
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      issued = 0; mark1 = 0;
    }
    stamp(1);
    // halo of the next tile: read now, written after the FIR (all reads then returned)
    f4v h0, h1;
    if (kind1 == 3) {
      h0 = lds_read_b128<0>(buf + NEWC * 128 + 2 * lane);
      if constexpr (HCH == 2) h1 = lds_read_b128<0>(buf + (NEWC + 1) * 128 + 2 * lane);
    }

    float ai[R], aq[R];
    fe_fir_tile<T, D, R, (MB == 1 || MB == 4 || MB == 5) ? 1 : 0, (T > 127 ? 8 : PFR), SAFE>(buf, lane, tp, ai, aq);

    if (kind1 == 3) {
      lds_wait<0>(h0);
      f2v* nb = &ring[b ^ 1][0];
      lds_write_b128(nb + 2 * lane, h0);
      if constexpr (HCH == 2) { lds_wait<0>(h1); lds_write_b128(nb + 128 + 2 * lane, h1); }
    }

    stamp(2);
    // ---- epilogue ----
    float d[R];
    const bool fast = i >= 1 && m0 + TO < M && p.i_ds == nullptr && have;
    if (MB == 4 || MB == 5) {          // tuning: memory pipeline only
      carry += ai[0] + aq[0];
      d[0] = d[1] = d[2] = carry;
    } else if (fast) {
      fast_epi(ai, aq, d);
      if constexpr (!FUSED) {
        typedef float f3v __attribute__((ext_vector_type(3)));
        *reinterpret_cast<f3v*>(p.demod + (int64_t)s * p.out_stride + m0 + R * lane) = f3v{d[0], d[1], d[2]};
        issued += 1;
      }
    } else {
      float si = 0.f, sq = 0.f;
      if (m0 > 0 && !have) {
        for (int k = lane; k < T; k += 64) {
          const f2v x = buf[(T - 1) - k];
          const float h = p.taps_dev[k];
          si = fmaf(h, x.x, si);
          sq = fmaf(h, x.y, sq);
        }
        si = wave_sum(si);
        sq = wave_sum(sq);
      }
      bool one = false;
      carry = fe_epilogue<T, D, R>(p, s, M, m0, lane, ai, aq, si, sq, have, carry, &one, d, !FUSED);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      issued = 0; mark1 = 0;
    }

    stamp(3);
    if constexpr (FUSED && (MB < 4 || MB == 6)) {
      const bool warm = (i + 1) % TPB == 0 && u == 0 && mid;   // warm-up tile = previous block's last
      if (fused_tail(i, warm, d, s1 == s, u + 1 == U && !(u == 0 && mid))) mark1 = 0;
    }

    stamp(4);
    // ---- advance ----
    if ((s1 != s || u + 1 == U) && p.wraps != nullptr) {
      const int w = wave_sum_i(wacc);
      if (lane == 0 && w != 0) atomicAdd(p.wraps + s, w);
      wacc = 0;
    }
    have = (s1 == s);
    s = s1; i = i1; nl = nl1;
    kind = kind1; mark = mark1;
    b ^= 1;
  }
  if constexpr (MB == 6) {
    if (lane == 0) {
      uint64_t* o = reinterpret_cast<uint64_t*>(p.q_ds) + 8 * blockIdx.x;
      for (int k = 0; k < 5; ++k) o[k] = tph[k];
      o[5] = U;
    }
  }
}

// ---------------------------------------------------------------------------------
// fe_circ_kernel: sub-tile FE with a circular per-wave chunk ring (deep prefetch).
//
// r01 measurements of fe_ring_kernel (one wave per SIMD, 2-slot ring): the per-tile
// compute (~2.2-3 us) is about the loaded memory latency of the next tile (~2.2 us), so
// a wave with ONE tile in flight exposes part of its compute.  Here a wave walks
// sub-tiles of 64 outputs (R = 1, lane l -> output m0 + l, lane stride 10 samples =
// 5 x 16 B: conflict-free ds_read_b128) through a circular ring of C = 30 one-KiB chunks
// (+ HCH mirror chunks): sub-tile g occupies chunks [5g, 5g + NCH) at ring positions
// 5g mod C .. (a sub-tile starting at position C-5 reads its last HCH chunks from the
// mirror positions C..C+HCH-1).  Consecutive sub-tiles share their halo chunks in place
// (no copies), and P = 4 sub-tiles (20 KiB) stay in flight behind the one being
// filtered, so the latency is covered by 4 sub-tiles of compute.
//   * new chunks of sub-tile g: [5g + NCH - 5, 5g + NCH) at position (5g mod C) + k
//     (k = NCH-5..NCH-1; >= C means the mirror position);
//   * a sub-tile starting at position 0 also gets its first HCH chunks DMA'd to
//     positions [0, HCH) (the previous sub-tile holds them at the mirror positions);
//   * the first sub-tile of a run, and one after a stream change, load all NCH chunks;
//     head/tail sub-tiles (outside [-hist, n)) are built with plain loads instead.
// FUSED: audio block = 5 sub-tiles = 320 demod samples = 64 audio outputs (one per
// lane); a run starting mid-stream runs 3 warm-up sub-tiles (192 >= 150 samples).
// ---------------------------------------------------------------------------------
template <int T, bool FUSED = false, int MODE = 0>
__global__ __launch_bounds__(64)
void fe_circ_kernel(FeParams p, TapsF32 taps, RingArgs a) {
  constexpr int D = 10, TO = 64;
  constexpr int NCH = (D * TO + T + 1 + 127) / 128;  // chunks per sub-tile image (6 at T=101)
  constexpr int HCH = NCH - 5;                       // halo chunks shared with the next sub-tile
  constexpr int C = 30;                              // ring positions (6 sub-tile starts)
  constexpr int P = 4;                               // sub-tiles in flight ahead
  constexpr int L = NCH * 128;
  constexpr int TP = (T + 1) / 2;
  static_assert((T & 1) == 1 && HCH >= 1 && HCH <= 2, "odd tap counts 101..235");
  static_assert(5 * P + NCH <= C, "ring must hold the computing sub-tile and P ahead");
  constexpr int TA = 151, DA = 5;
  constexpr int BD = TO * DA;                        // 320 demod samples per audio block
  constexpr int HA = 152;                            // history slots (>= TA-1)
  constexpr int NPA = (TA + 1) / 2;                  // 76 audio sample pairs per lane
  constexpr int WU = (TA - 1 + TO - 1) / TO;         // 3 warm-up sub-tiles

  constexpr int RING = C + HCH;                      // chunks incl. mirrors
  constexpr int RINGP = FUSED ? RING * 128 : (RING * 128 > 5120 ? RING * 128 : 5120);  // >= 40 KiB: 4 waves/CU
  __shared__ __attribute__((aligned(16))) f2v ring[RINGP];
  __shared__ __attribute__((aligned(16))) float dh[FUSED ? HA + BD + 8 : 1];
  __shared__ __attribute__((aligned(16))) f2v ptab[FUSED ? NPA + 1 : 1];

  const int lane = threadIdx.x;
  const int64_t u0 = (int64_t)blockIdx.x * a.per_wave;
  if (u0 >= a.total) return;
  const int nunits = (int)min<int64_t>(a.per_wave, a.total - u0);
  const int64_t M = (p.n + D - 1) / D;

  f2v tp[TP];
#pragma unroll
  for (int j = 0; j < TP; ++j) tp[j] = f2v{taps.h[2 * j], (2 * j + 1 < T) ? taps.h[2 * j + 1] : 0.f};
#pragma unroll
  for (int j = 0; j < TP; ++j) asm volatile("" : "+v"(tp[j]));

  const unsigned voff = 16u * lane;
  const float* iqf = reinterpret_cast<const float*>(p.iq);
  const unsigned ring_lds = lds_addr_of(&ring[0]);
  auto n_lo_of = [&](int i) { return (int64_t)(D * TO) * i - D - (T - 1); };

  // sub-tile sequence of this wave: (stream s, index i in stream), U sub-tiles
  int s0, i0, U;
  if constexpr (FUSED) {
    s0 = (int)(u0 / a.ab);
    const int q0 = (int)(u0 - (int64_t)s0 * a.ab);
    i0 = DA * q0 - (q0 > 0 ? WU : 0);
    U = nunits * DA + (q0 > 0 ? WU : 0);
    if (q0 == 0)
      for (int e = lane; e < HA; e += 64) dh[e] = 0.f;
    for (int e = lane; e < 8; e += 64) dh[HA + BD + e] = 0.f;
    for (int k = lane; k <= NPA; k += 64) {
      const int k0 = (TA - 1) - 2 * k, k1 = k0 - 1;
      ptab[k] = f2v{(k0 >= 0 && k < NPA) ? a.ataps[k0] : 0.f, (k1 >= 0 && k < NPA) ? a.ataps[k1] : 0.f};
    }
  } else {
    s0 = (int)(u0 / a.tps);
    i0 = (int)(u0 - (int64_t)s0 * a.tps);
    U = nunits;
  }

  // issue state (sub-tile sequence number v relative to the run; g = absolute chunk
  // base 5*v counted from the run start; ring position of sub-tile v = (5 v) mod C)
  int is = s0, ii = i0;          // stream / index of the next sub-tile to issue
  int64_t inl = n_lo_of(i0);
  int issued = 0;
  int mk[P + 1];                 // issue marks of sub-tiles v .. v+P (rotating)
  int kd[P + 1];                 // kinds: 0 none, 1 guarded, 2 DMA (image complete after wait)
#pragma unroll
  for (int k = 0; k <= P; ++k) { mk[k] = 0; kd[k] = 0; }
  bool prev_valid = false;       // previous issued sub-tile was in the same stream
  auto issue_next = [&](int v, int slot) {
    // v: sequence number of the sub-tile being issued; slot: index into mk/kd
    const int pos = (5 * v) % C;
    const bool full = !prev_valid;
    const int64_t lo = full ? inl : inl + 128 * (NCH - 5);
    const bool dma = MODE != 2 && inl >= -p.hist && inl + L <= p.n;
    (void)lo;
    if (dma) {
      const char* g = reinterpret_cast<const char*>(iqf + 2 * ((int64_t)is * p.stride + inl));
      auto chunk = [&](int k, int at) {       // chunk k of this image -> ring position `at`
        glds16x<1>(voff, g + 1024 * k, ring_lds + 1024u * at);
      };
      if (full) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) chunk(k, pos + k);
        issued += NCH;
      } else {
#pragma unroll
        for (int k = NCH - 5; k < NCH; ++k) chunk(k, pos + k);
        issued += 5;
      }
      if (pos == 0 && !full) {                // halo chunks also at [0, HCH)
#pragma unroll
        for (int k = 0; k < HCH; ++k) chunk(k, k);
        issued += HCH;
      }
      kd[slot] = 2;
    } else {
      kd[slot] = 1;
    }
    mk[slot] = issued;
    prev_valid = true;
    // advance the issue pointer
    if (++ii == a.tps) { ii = 0; ++is; inl = n_lo_of(0); prev_valid = false; }
    else inl += D * TO;
  };
  // prologue: issue sub-tiles 0 .. P-1 of the run
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (k < U) issue_next(k, k);

  int s = s0, i = i0;
  int64_t nl = n_lo_of(i0);
  float carry = 0.f;
  bool have = false;
  int wacc = 0;
  for (int v = 0; v < U; ++v) {
    // ---- issue sub-tile v + P ----
    if (v + P < U) issue_next(v + P, P);
    else { kd[P] = 0; mk[P] = issued; }
    const int pos = (5 * v) % C;
    f2v* img = ring + 128 * pos;
    const int64_t m0 = (int64_t)TO * i;
    // ---- wait / build this sub-tile's image ----
    if (kd[0] == 2) {
      const int nw = issued - mk[0];
      if (nw == 5 * P) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(5 * P) : "memory");
      else if (nw == 5 * P + 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(5 * P + 1) : "memory");
      else wait_vm_chain(nw);
    } else {
      const float* base = iqf + 2 * ((int64_t)s * p.stride);
      for (int e = lane; e < L; e += 64) {
        const int64_t nn = nl + e;
        f2v x = f2v{0.f, 0.f};
        if (MODE == 2) x = f2v{(float)e * 1e-4f, (float)lane};
        else if (nn >= -p.hist && nn < p.n) x = f2v{base[2 * nn], base[2 * nn + 1]};
        img[e] = x;
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      issued = 0;
#pragma unroll
      for (int k = 0; k <= P; ++k) mk[k] = 0;
    }

    float ai[1], aq[1];
    fe_fir_tile<T, D, 1, (MODE == 1 || MODE >= 4) ? 1 : 0>(img, lane, tp, ai, aq);

    // ---- epilogue ----
    float d[1];
    const bool fast = i >= 1 && m0 + TO < M && p.i_ds == nullptr && have;
    if (MODE >= 4) {
      carry += ai[0] + aq[0];
      d[0] = carry;
    } else if (fast) {
      const float phi = fast_atan2f(aq[0], ai[0]);
      const float from_left = __int_as_float(__builtin_amdgcn_update_dpp(
          0, __float_as_int(phi), 0x138 /*wave_shr:1*/, 0xf, 0xf, false));
      const float prev = (lane == 0) ? carry : from_left;
      float dd = phi - prev;
      if (dd > kPiF) { dd -= k2PiF; wacc -= 1; }
      else if (dd < -kPiF) { dd += k2PiF; wacc += 1; }
      d[0] = dd;
      if constexpr (!FUSED) {
        p.demod[(int64_t)s * p.out_stride + m0 + lane] = dd;
        issued += 1;
      }
      carry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi), 63));
    } else {
      float si = 0.f, sq = 0.f;
      if (m0 > 0 && !have) {
        for (int k = lane; k < T; k += 64) {
          const f2v x = img[(T - 1) - k];
          const float h = p.taps_dev[k];
          si = fmaf(h, x.x, si);
          sq = fmaf(h, x.y, sq);
        }
        si = wave_sum(si);
        sq = wave_sum(sq);
      }
      bool one = false;
      carry = fe_epilogue<T, D, 1>(p, s, M, m0, lane, ai, aq, si, sq, have, carry, &one, d, !FUSED);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      issued = 0;
#pragma unroll
      for (int k = 0; k <= P; ++k) mk[k] = 0;
    }

    // next sub-tile in compute order
    int s1 = s, i1 = i + 1;
    if (i1 == a.tps) { i1 = 0; ++s1; }

    if constexpr (FUSED && MODE < 4) {
      const int ib = i % DA;                         // sub-tile within its audio block
      const bool warm = v < U % DA;                  // leading warm-up sub-tiles of the run
      const int rel = (warm ? (ib - DA) : ib) * TO + lane;
      if (rel >= -HA) dh[HA + rel] = d[0];
      if (!warm && ib == DA - 1) {
        asm volatile("" ::: "memory");
        const int64_t q = i / DA;
        // lane window: dh[HA - (TA-1) + 5 lane + w], w = 0 .. 2*NPA-1 (pairs)
        const float* aw = dh + (HA - (TA - 1) + DA * lane);
        f2v acc0 = f2v{0.f, 0.f}, acc1 = f2v{0.f, 0.f};
        constexpr int APF = 5;                       // steps read ahead (1.5 reads per step)
        f2v xq[NPA];
        f4v tq[(NPA + 1) / 2];
        auto rd = [&](auto K) {
          constexpr int k = K;
          xq[k] = lds_read2_b32<2 * k, 2 * k + 1>(aw);
          if constexpr ((k & 1) == 0) tq[k / 2] = lds_read_b128<8 * k>(ptab);   // entries k, k+1
        };
        // reads per step: 1 (odd k) or 2 (even k); counted waits by cumulative totals
        constexpr auto nreads = [](int k) { return k + (k + 1) / 2; };   // reads issued for steps 0..k-1
        static_for<0, APF>(rd);
        static_for<0, NPA>([&](auto K) {
          constexpr int k = K;
          if constexpr (k + APF < NPA) rd(std::integral_constant<int, k + APF>{});
          constexpr int issued_r = nreads(k + APF < NPA ? k + APF + 1 : NPA);
          constexpr int needed_r = nreads(k + 1);
          constexpr int pend = issued_r - needed_r;
          lds_wait2<(pend > 15 ? 15 : pend)>(xq[k], tq[k / 2]);
          const f2v t2 = (k & 1) ? f2v{tq[k / 2].z, tq[k / 2].w} : f2v{tq[k / 2].x, tq[k / 2].y};
          if constexpr (k & 1) pk_fma_ordered(acc1, t2, xq[k]);
          else pk_fma_ordered(acc0, t2, xq[k]);
        });
        const float out = (acc0.x + acc0.y) + (acc1.x + acc1.y);
        const int64_t A = (M + DA - 1) / DA;
        const int64_t j = q * TO + lane;
        if (j < A) a.audio[(int64_t)s * a.audio_stride + j] = out;
        if (q * TO + TO <= A) issued += 1;
        else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          issued = 0;
#pragma unroll
          for (int k = 0; k <= P; ++k) mk[k] = 0;
        }
        asm volatile("" ::: "memory");
        if (s1 != s)
          for (int e = lane; e < HA; e += 64) dh[e] = 0.f;
        else
          for (int e = lane; e < HA; e += 64) dh[e] = dh[BD + e];
        asm volatile("" ::: "memory");
      }
    }

    if ((s1 != s || v + 1 == U) && p.wraps != nullptr) {
      const int w = wave_sum_i(wacc);
      if (lane == 0 && w != 0) atomicAdd(p.wraps + s, w);
      wacc = 0;
    }
    have = (s1 == s);
    nl = (s1 == s) ? nl + D * TO : n_lo_of(i1);
    s = s1; i = i1;
#pragma unroll
    for (int k = 0; k < P; ++k) { mk[k] = mk[k + 1]; kd[k] = kd[k + 1]; }
  }
}

// lfilter final state zf for the I and Q channels of an interleaved IQ block
// (scipy _signaltools.py:2153-2172), computed in f64:
//   zf[k] = sum_{j=k+1}^{T-1} b[j] * x[N-1-(j-k-1)]  +  (N+k < T-1 ? zi[N+k] : 0)
// One 256-thread block per stream (T <= 256): the T-1 newest samples and the taps are
// staged in LDS, then each output's f64 dot product runs from LDS.
template <bool U8>
__global__ __launch_bounds__(256) void iq_zf_kernel(const void* iq_all, int64_t n, int64_t stride,
                                                    const double* b, int T, const double* zi_i,
                                                    const double* zi_q, int64_t zi_stride,
                                                    double* zf_i, double* zf_q) {
  __shared__ float2 xs[SDR_MAX_TAPS];   // xs[i] = x[n-1-i]
  __shared__ double bs[SDR_MAX_TAPS];
  const int k = threadIdx.x;
  const int s = blockIdx.y;
  const void* iq = reinterpret_cast<const char*>(iq_all) + (int64_t)s * stride * (U8 ? 2 : 8);
  if (zi_i != nullptr) { zi_i += (int64_t)s * zi_stride; zi_q += (int64_t)s * zi_stride; }
  zf_i += (int64_t)s * zi_stride;
  zf_q += (int64_t)s * zi_stride;
  const int L = (int)min<int64_t>(n, T - 1);
  if (k < L) xs[k] = IqLoad<U8>::load1(iq, n - 1 - k);
  if (k < T) bs[k] = b[k];
  __syncthreads();
  if (k >= T - 1) return;
  // zf[k] = sum_{j=k+1}^{T-1} b[j] x[n-1-(j-k-1)] over the terms with a sample (j-k-1 < n)
  const int jhi = (int)min<int64_t>(T - 1, n + k);
  double si = 0.0, sq = 0.0;
#pragma unroll 4
  for (int j = k + 1; j <= jhi; ++j) {
    const float2 v = xs[j - k - 1];
    si = fma(bs[j], (double)v.x, si);
    sq = fma(bs[j], (double)v.y, sq);
  }
  if (n + k < T - 1 && zi_i != nullptr) {
    si += zi_i[n + k];
    sq += zi_q[n + k];
  }
  zf_i[k] = si;
  zf_q[k] = sq;
}

// ---------------------------------------------------------------------------------
// fe_slot_kernel: the f32 front end at two waves per SIMD (T <= 127).
//
// fe_ring_kernel holds two 16-KiB image slots per wave, hence one wave per SIMD: its VALU
// issues ~35 % of the time and a wave's per-tile work (FIR + epilogue + audio, ~2.7 us)
// is longer than the memory system needs to deliver the next tile, so that launch is
// issue/latency-bound.  Here a wave holds ONE slot: the next tile's 15 new
// 1-KiB chunks are loaded into AGPRs (16 B per lane each) while the current tile is
// filtered, and written into the slot after the FIR (the halo chunk moves from position
// 15 to 0 through a VGPR).  Half the LDS lets a second wave share each SIMD and issue
// while the first one waits.
//  * Work: contiguous, balanced tile ranges (tile granularity).
//  * FUSED (sdr_fe_mono_dev): the 5 tiles of an audio block keep their demod values in
//    VGPRs (3 per lane per tile) plus the previous block's last tile (the 150-sample
//    history).  After the block's last FIR the slot is free: history and block are
//    written into it and the audio FIR (outputs 3l..3l+2 of lane l) reads them there,
//    before the next image is written.  A run starting mid-stream first runs one warm-up
//    tile; a run ending mid-block computes that block from the tiles it has.  Audio output
//    j is stored by the wave whose tile range holds its newest input sample 5j, so every
//    output is written exactly once.
// ---------------------------------------------------------------------------------
struct SlotArgs {
  int64_t total;        // tiles over all streams
  int tps;              // tiles per stream (FUSED: 5 x audio blocks)
  float* audio;         // FUSED: ceil(M/5) outputs per stream, audio_stride apart
  int64_t audio_stride;
  const float* ataps;   // FUSED: 151 audio taps (device)
};

// audio FIR of one block (a[j] = sum_k g[k] d[5j - k]): lane l -> outputs 3l..3l+2 over
// its 161-sample window aw = dh + HA - 150 + 15 l; tap triples {g[150-w], g[155-w],
// g[160-w]} by broadcast ds_read_b128 of ptab; reads issued APF steps ahead, counted waits
__device__ __forceinline__ void audio_block3(const float* aw, const f4v* ptab, float& o0, float& o1,
                                             float& o2) {
  asm volatile("" ::: "memory");
  f2v acc01a = f2v{0.f, 0.f}, acc01b = f2v{0.f, 0.f};
  float a2a = 0.f, a2b = 0.f;
  constexpr int NS = 81, APF = 5;   // 3*APF <= 15 (lgkmcnt field)
  f2v xq[NS];
  f4v ta[NS], tb[NS];
  auto rd = [&](auto K) {
    constexpr int k = K;
    xq[k] = lds_read2_b32<2 * k, 2 * k + 1>(aw);
    ta[k] = lds_read_b128<32 * k>(ptab);
    tb[k] = lds_read_b128<32 * k + 16>(ptab);
  };
  static_for<0, APF>(rd);
  static_for<0, NS>([&](auto K) {
    constexpr int k = K;
    if constexpr (k + APF < NS) {
      rd(std::integral_constant<int, k + APF>{});
      lds_wait3<3 * APF>(xq[k], ta[k], tb[k]);
    } else {
      lds_wait3<3 * (NS - 1 - k)>(xq[k], ta[k], tb[k]);
    }
    pk_fma_bcast_x_ordered<false>(acc01a, f2v{ta[k].x, ta[k].y}, xq[k]);
    pk_fma_bcast_x_ordered<true>(acc01b, f2v{tb[k].x, tb[k].y}, xq[k]);
    fmac_ordered(a2a, ta[k].z, xq[k].x);
    fmac_ordered(a2b, tb[k].z, xq[k].y);
  });
  o0 = acc01a.x + acc01b.x;
  o1 = acc01a.y + acc01b.y;
  o2 = a2a + a2b;
}

// PF: FIR reads in flight; VST: stage in VGPRs (true) or AGPRs (false)
// MB (tuning only; 0 = product): 1 = no FIR (memory pipeline + epilogue).
// PIPE: 0 = the next image staged in registers during the FIR; 1 = no stage: the next
// image's LDS-DMA is issued after the tile and waited for at once (the SIMD's other wave
// computes meanwhile; no stage registers, and ~half the bytes in flight)
// U8: interleaved u8 IQ; the stage holds the next tile's 15 new 128-sample chunks as one
// dword per lane (2 B per complex sample), converted to (x-128)/128 f32 pairs when it is
// written into the slot (the same f32 image as the f32 input).
template <int T, bool FUSED, int PF = 4, bool VST = true, int MB = 0, int PIPE = 0, bool U8 = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2)))
void fe_slot_kernel(FeParams p, TapsF32 taps, SlotArgs a) {
  constexpr int D = 10, R = 3, TO = 64 * R;
  constexpr int NEWC = D * TO / 128;                 // 15 new 128-sample chunks per tile
  constexpr int NCH = (D * TO + T + 1 + 127) / 128;  // chunks per tile image
  constexpr int HCH = NCH - NEWC;                    // halo chunks shared with the next tile
  constexpr int L = NCH * 128;                       // image length (complex samples)
  constexpr int TP = (T + 1) / 2;
  static_assert((T & 1) == 1 && (HCH == 1 || HCH == 2), "odd tap counts 101..235");
  static_assert(!U8 || (PIPE == 0 && VST), "u8: register stage");
  constexpr int TA = 151, DA = 5, BO = 64 * R, HA = 152, NW = DA * (R - 1) + TA;
  static_assert((HA + TO * DA + 4) * 4 <= L * 8, "audio history + block fit in the slot");
  __shared__ __attribute__((aligned(16))) f2v slot[L];
  __shared__ __attribute__((aligned(16))) f4v ptab[FUSED ? NW + 1 : 1];
  float* const dh = reinterpret_cast<float*>(&slot[0]);   // FUSED audio window, aliases the slot

  const int lane = threadIdx.x;
  const int64_t g0 = (int64_t)blockIdx.x * a.total / gridDim.x;
  const int64_t g1 = ((int64_t)blockIdx.x + 1) * a.total / gridDim.x;
  if (g0 >= g1) return;
  const int64_t M = (p.n + D - 1) / D;

  // FE taps as VGPR pairs {h[2j], h[2j+1]}: held for the whole launch (FE), or re-read from
  // an LDS table before each tile's FIR (FUSED: frees the registers for the audio FIR)
  __shared__ __attribute__((aligned(16))) f2v tlds[FUSED ? TP + 1 : 1];
  f2v tp[TP];
  if constexpr (FUSED) {
    for (int j = lane; j < TP + 1; j += 64)
      tlds[j] = (j < TP) ? f2v{p.taps_dev[2 * j], (2 * j + 1 < T) ? p.taps_dev[2 * j + 1] : 0.f} : f2v{0.f, 0.f};
  } else {
#pragma unroll
    for (int j = 0; j < TP; ++j) tp[j] = f2v{taps.h[2 * j], (2 * j + 1 < T) ? taps.h[2 * j + 1] : 0.f};
#pragma unroll
    for (int j = 0; j < TP; ++j) asm volatile("" : "+v"(tp[j]));
  }
  // this lane's taps for the cooperative predecessor output (a run's first tile), loaded
  // before any stage load is in flight
  constexpr int NK = (T + 63) / 64;
  float hk[NK];
#pragma unroll
  for (int q = 0; q < NK; ++q) hk[q] = (lane + 64 * q < T) ? p.taps_dev[lane + 64 * q] : 0.f;
  if constexpr (FUSED) {
    for (int w = lane; w < NW + 1; w += 64) {               // entry NW: zero (pairs over-read)
      const int k0 = (TA - 1) - w, k1 = k0 + DA, k2 = k0 + 2 * DA;
      ptab[w] = f4v{(k0 >= 0 && k0 < TA) ? a.ataps[k0] : 0.f, (k1 >= 0 && k1 < TA) ? a.ataps[k1] : 0.f,
                    (k2 >= 0 && k2 < TA) ? a.ataps[k2] : 0.f, 0.f};
    }
  }
  const unsigned voff = 16u * lane;
  const float* iqf = reinterpret_cast<const float*>(p.iq);
  // tile (s, i): outputs TO*i ..; image = samples [n_lo, n_lo + L), n_lo = D*(m0-1) - (T-1)
  auto n_lo_of = [&](int ii) { return (int64_t)(D * TO) * ii - D - (T - 1); };
  auto interior = [&](int64_t nl) { return nl >= -p.hist && nl + L <= p.n; };
  auto cvt8 = [](unsigned b) { return fmaf((float)b, 0.0078125f, -1.0f); };   // (b-128)/128, exact

  // whole image into the slot, waited for (run start, stream change, stream head / tail):
  // LDS-DMA when interior, else guarded loads (zeros outside [-hist, n))
  auto build_sync = [&](int ss, int64_t nl) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if constexpr (U8) {
      const uint8_t* base = reinterpret_cast<const uint8_t*>(p.iq) + 2 * ((int64_t)ss * p.stride);
      for (int e = lane; e < L; e += 64) {
        const int64_t nn = nl + e;
        f2v x = f2v{0.f, 0.f};
        if (nn >= -p.hist && nn < p.n) x = f2v{cvt8(base[2 * nn]), cvt8(base[2 * nn + 1])};
        slot[e] = x;
      }
    } else if (interior(nl)) {
      const char* g = reinterpret_cast<const char*>(iqf + 2 * ((int64_t)ss * p.stride + nl));
      const unsigned lb = lds_addr_of(slot);
      static_for<0, (NCH + 3) / 4>([&](auto Q) {
        constexpr int c = 4 * Q;
        constexpr int n = (NCH - c) < 4 ? (NCH - c) : 4;
        glds16x<n>(voff, g + 1024 * c, lb + 1024 * c);
      });
    } else {
      const float* base = iqf + 2 * ((int64_t)ss * p.stride);
      for (int e = lane; e < L; e += 64) {
        const int64_t nn = nl + e;
        f2v x = f2v{0.f, 0.f};
        if (nn >= -p.hist && nn < p.n) x = f2v{base[2 * nn], base[2 * nn + 1]};
        slot[e] = x;
      }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  };
  // the next tile's new chunks [HCH, NCH) -> register stage (16 B per lane per chunk; u8:
  // 4 B per lane per chunk)
  f4v stg[U8 ? 1 : NEWC];
  unsigned stg8[U8 ? NEWC : 1];
  auto load_stage = [&](int ss, int64_t nl) {
    if constexpr (U8) {
      const char* gb = reinterpret_cast<const char*>(p.iq) + 2 * ((int64_t)ss * p.stride + nl) + 256 * HCH;
      static_for<0, NEWC>([&](auto C) {
        constexpr int c = C;
        gload4_nt_v<256 * c>(stg8[c], 4u * lane, gb);
      });
    } else {
      const char* gl = reinterpret_cast<const char*>(iqf + 2 * ((int64_t)ss * p.stride + nl)) + 1024 * HCH;
      static_for<0, NEWC>([&](auto C) {
        constexpr int c = C;
        if constexpr (VST) gload16_nt_v<1024 * (c % 4)>(stg[c], voff, gl + 4096 * (c / 4));
        else gload16_nt_a<1024 * (c % 4)>(stg[c], voff, gl + 4096 * (c / 4));
      });
    }
  };

  int s = (int)(g0 / a.tps);
  int i = (int)(g0 - (int64_t)s * a.tps);
  const bool warm0 = FUSED && i > 0;                   // FUSED: warm-up tile i-1 first
  if (warm0) --i;
  const int U = (int)(g1 - g0) + (warm0 ? 1 : 0);
  // FUSED: the audio outputs of stream s this run stores (5 j inside its tile range)
  int64_t jlo = 0, jhi = 0;
  auto own = [&]() {
    const int64_t lo = max<int64_t>(g0 - (int64_t)s * a.tps, 0);
    const int64_t hi = min<int64_t>(g1 - (int64_t)s * a.tps, a.tps);
    jlo = (TO * lo + DA - 1) / DA;
    jhi = min<int64_t>((TO * hi + DA - 1) / DA, (M + DA - 1) / DA);
  };
  if constexpr (FUSED) own();

  build_sync(s, n_lo_of(i));
  float carry = 0.f;
  bool have = false;
  int wacc = 0;
  float dblk[DA][R], hist[R];                          // FUSED: demod of the block's tiles
#pragma unroll
  for (int k = 0; k < DA; ++k)
#pragma unroll
    for (int r = 0; r < R; ++r) dblk[k][r] = 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r) hist[r] = 0.f;
  auto next_of = [&](int ss, int ii, int& s1, int& i1) {
    s1 = ss;
    i1 = ii + 1;
    if (i1 == a.tps) { i1 = 0; ++s1; }
  };
  int s1, i1;
  next_of(s, i, s1, i1);
  // u8 stage loads are dwords: a stream whose base is not 4-B aligned (odd stride, odd
  // stream) builds every image with guarded byte loads instead
  auto staged_ok = [&](int ss) { return !U8 || (((int64_t)ss * p.stride) & 1) == 0; };
  bool stg1 = U > 1 && s1 == s && interior(n_lo_of(i1)) && staged_ok(s1);   // next image via the stage
  if (PIPE == 0 && stg1) load_stage(s1, n_lo_of(i1));

  for (int u = 0; u < U; ++u) {
    const bool lastu = (u + 1 == U);
    f4v h0, h1;                                                        // halo of the next tile
    if (stg1) {
      h0 = lds_read_b128<0>(slot + NEWC * 128 + 2 * lane);
      if constexpr (HCH == 2) h1 = lds_read_b128<0>(slot + (NEWC + 1) * 128 + 2 * lane);
    }
    if constexpr (FUSED) {
      constexpr int NQ = (TP + 1) / 2;
      f4v tq[NQ];
      static_for<0, NQ>([&](auto K) { tq[K] = lds_read_b128<16 * K>(tlds); });
      static_for<0, NQ>([&](auto K) { lds_wait<0>(tq[K]); });
      static_for<0, TP>([&](auto J) {
        constexpr int j = J;
        tp[j] = (j & 1) ? f2v{tq[j / 2].z, tq[j / 2].w} : f2v{tq[j / 2].x, tq[j / 2].y};
      });
    }
    float ai[R], aq[R];
    fe_fir_tile<T, D, R, MB == 1 ? 1 : 0, PF, true>(slot, lane, tp, ai, aq);
    const int64_t m0 = (int64_t)TO * i;
    float d[R];
    bool st_fe = false;
    if (i >= 1 && m0 + TO < M && p.i_ds == nullptr && have) {
      // interior tile: phases, predecessor (DPP / carry), np.unwrap wrap
      float phi[R];
#pragma unroll
      for (int r = 0; r < R; ++r) phi[r] = fast_atan2f(aq[r], ai[r]);
      const float from_left = __int_as_float(__builtin_amdgcn_update_dpp(
          0, __float_as_int(phi[R - 1]), 0x138 /*wave_shr:1*/, 0xf, 0xf, false));
      float prev = (lane == 0) ? carry : from_left;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float dd = phi[r] - prev;
        if (dd > kPiF) { dd -= k2PiF; wacc -= 1; }
        else if (dd < -kPiF) { dd += k2PiF; wacc += 1; }
        d[r] = dd;
        prev = phi[r];
      }
      carry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[R - 1]), 63));
      st_fe = !FUSED;
    } else {
      float si = 0.f, sq = 0.f;
      if (m0 > 0 && !have) {           // output m0-1 (the predecessor): image samples [0, T)
#pragma unroll
        for (int q = 0; q < NK; ++q) {
          if (lane + 64 * q < T) {
            const f2v x = slot[(T - 1) - (lane + 64 * q)];
            si = fmaf(hk[q], x.x, si);
            sq = fmaf(hk[q], x.y, sq);
          }
        }
        si = wave_sum(si);
        sq = wave_sum(sq);
      }
      carry = fe_epilogue<T, D, R>(p, s, M, m0, lane, ai, aq, si, sq, have, carry, nullptr, d, !FUSED);
    }

    // FUSED: block bookkeeping and, after the block's last tile (or the run's), its audio
    const int sp = s;
    const int64_t jlo_t = jlo, jhi_t = jhi;
    bool aud = false;
    float o0 = 0.f, o1 = 0.f, o2 = 0.f;
    int64_t qa = 0;
    if constexpr (FUSED) {
      const int ib = i % DA;
#pragma unroll
      for (int k = 0; k < DA; ++k)
#pragma unroll
        for (int r = 0; r < R; ++r) dblk[k][r] = (ib == k) ? d[r] : dblk[k][r];
      if (!(warm0 && u == 0) && (ib == DA - 1 || lastu)) {
        // the slot is free (the FIR's and epilogue's reads have returned)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane >= 14) {
#pragma unroll
          for (int r = 0; r < R; ++r) dh[HA - 150 + 3 * (lane - 14) + r] = hist[r];
        }
#pragma unroll
        for (int k = 0; k < DA; ++k)
#pragma unroll
          for (int r = 0; r < R; ++r) dh[HA + TO * k + R * lane + r] = dblk[k][r];
        if (lane < 4) dh[HA + TO * DA + lane] = 0.f;
        audio_block3(dh + (HA - (TA - 1) + DA * R * lane), ptab, o0, o1, o2);
        aud = true;
        qa = i / DA;
      }
      if (ib == DA - 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) hist[r] = dblk[DA - 1][r];
      }
    }

    if ((s1 != s || lastu) && p.wraps != nullptr) {
      const int w = wave_sum_i(wacc);
      if (lane == 0 && w != 0) atomicAdd(p.wraps + s, w);
      wacc = 0;
    }
    // the finished tile's stores
    auto stores = [&]() {
      if (st_fe) {
        typedef float f3v __attribute__((ext_vector_type(3)));
        *reinterpret_cast<f3v*>(p.demod + (int64_t)sp * p.out_stride + m0 + R * lane) = f3v{d[0], d[1], d[2]};
      }
      if constexpr (FUSED) {
        if (aud) {
          const int64_t j0 = qa * BO, j = j0 + R * lane;
          float* ao = a.audio + (int64_t)sp * a.audio_stride + j;
          if (j0 >= jlo_t && j0 + BO <= jhi_t) {
            typedef float f3v __attribute__((ext_vector_type(3)));
            *reinterpret_cast<f3v*>(ao) = f3v{o0, o1, o2};
          } else {
            if (j >= jlo_t && j < jhi_t) ao[0] = o0;
            if (j + 1 >= jlo_t && j + 1 < jhi_t) ao[1] = o1;
            if (j + 2 >= jlo_t && j + 2 < jhi_t) ao[2] = o2;
          }
        }
      }
    };
    if (!lastu) {
      // next image into the slot, then the loads of the one after it
      if (PIPE == 1) stores();
      if (stg1 && PIPE == 1) {
        lds_wait<0>(h0);
        lds_write_b128(slot + 2 * lane, h0);
        if constexpr (HCH == 2) { lds_wait<0>(h1); lds_write_b128(slot + 128 + 2 * lane, h1); }
        const char* g = reinterpret_cast<const char*>(iqf + 2 * ((int64_t)s1 * p.stride + n_lo_of(i1))) + 1024 * HCH;
        const unsigned lb = lds_addr_of(slot) + 1024 * HCH;
        static_for<0, (NEWC + 3) / 4>([&](auto Q) {
          constexpr int c = 4 * Q;
          constexpr int n = (NEWC - c) < 4 ? (NEWC - c) : 4;
          glds16x<n>(voff, g + 1024 * c, lb + 1024 * c);
        });
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (stg1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_wait<0>(h0);
        lds_write_b128(slot + 2 * lane, h0);
        if constexpr (HCH == 2) { lds_wait<0>(h1); lds_write_b128(slot + 128 + 2 * lane, h1); }
        const unsigned na = lds_addr_of(slot) + 16u * lane;
        static_for<0, NEWC>([&](auto C) {
          constexpr int c = C;
          if constexpr (U8) {
            asm volatile("" : "+v"(stg8[c]));
            const unsigned b = stg8[c];
            const f4v v = f4v{cvt8(b & 0xff), cvt8((b >> 8) & 0xff), cvt8((b >> 16) & 0xff), cvt8(b >> 24)};
            lds_write_b128_v<1024 * (HCH + c)>(na, v);
          } else if constexpr (VST) {
            asm volatile("" : "+v"(stg[c]));
            lds_write_b128_v<1024 * (HCH + c)>(na, stg[c]);
          } else {
            asm volatile("" : "+a"(stg[c]));
            lds_write_b128_a<1024 * (HCH + c)>(na, stg[c]);
          }
        });
      } else {
        build_sync(s1, n_lo_of(i1));
      }
      have = (s1 == s);
      if (FUSED && !have) {
#pragma unroll
        for (int r = 0; r < R; ++r) hist[r] = 0.f;
      }
      s = s1;
      i = i1;
      if (FUSED && !have) own();
      next_of(s, i, s1, i1);
      stg1 = u + 2 < U && s1 == s && interior(n_lo_of(i1)) && staged_ok(s1);
      if (PIPE == 0 && stg1) load_stage(s1, n_lo_of(i1));
    }
    // (PIPE 0) queued behind the next tile's loads
    if (PIPE == 0 || lastu) stores();
  }
}

}  // namespace

// ------------------------------------------------------------------------------
// Host-side launchers (called by capi.hip).  Tile shape per tap count:
// NT=128 threads x R=4 outputs = 512 decimated outputs (5120 complex inputs) per
// workgroup: ~43 KB LDS -> 3 workgroups (12 waves) per CU.
// ------------------------------------------------------------------------------
struct FeLaunch {
  const void* iq; int64_t n; int64_t stride; int64_t hist; int nstreams;
  const float* taps_dev; const TapsF32* taps; int T; int D; int u8;
  const double* zi_i; const double* zi_q; int64_t zi_stride; const double* prev_phase;
  float* demod; int64_t out_stride; float* i_ds; float* q_ds; float* last_phi; int* wraps;
};

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      n = prop.multiProcessorCount;
    if (n <= 0) n = 256;
  }
  return n;
}

// Resident workgroups per CU for a kernel (the persistent grid must be fully resident
// for its tiles to be spread evenly; any excess would run as a second, serial round).
template <typename K>
static int resident_per_cu(K kernel, int threads) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, threads, 0) != hipSuccess || n <= 0) n = 1;
  return n;
}

// f32 front-end kernel family: "ring" (fe_ring_kernel, default) or "circ" (fe_circ_kernel),
// chosen once per process by SDR_FE_KERNEL (A/B measurement; both are parity-tested).
static bool use_circ() {
  static const bool c = [] {
    const char* e = getenv("SDR_FE_KERNEL");
    return e && strcmp(e, "circ") == 0;
  }();
  return c;
}
// fe_slot_kernel (two waves per SIMD): the default for the FE-only launch at T <= 127
// (r01 A/B: 104 vs 111 us per 65.5 M samples); the fused launch keeps fe_ring_kernel (95 vs
// 100 us), unless SDR_FE_KERNEL=slot / ring / circ picks one family for both
static bool use_slot(bool fused) {
  static const int c = [] {
    const char* e = getenv("SDR_FE_KERNEL");
    return !e ? 0 : (strcmp(e, "slot") == 0 ? 1 : 2);
  }();
  return c == 1 || (c == 0 && !fused);
}

template <int T, bool FUSED, bool U8 = false>
static hipError_t launch_slot_t(FeParams p, const TapsF32& taps, SlotArgs sa, hipStream_t st) {
  if (sa.total <= 0) return hipSuccess;
  static const int wpc = resident_per_cu(fe_slot_kernel<T, FUSED, 4, true, 0, 0, U8>, 64);
  const int64_t slots = (int64_t)cu_count() * std::max(1, std::min(wpc, 8));
  const int64_t grid = std::min<int64_t>(slots, sa.total);
  p.tiles_per_stream = sa.tps;
  hipLaunchKernelGGL((fe_slot_kernel<T, FUSED, 4, true, 0, 0, U8>), dim3((unsigned)grid), dim3(64), 0, st, p, taps, sa);
  return hipGetLastError();
}

template <int T, int D, bool U8>
static hipError_t launch_fe_t(const FeLaunch& a, hipStream_t st) {
  constexpr int NT = U8 ? 128 : 64;
  constexpr int R = U8 ? 4 : 2;
  constexpr int NB = 2;
  constexpr int TO = NT * R;
  FeParams p;
  p.iq = a.iq; p.n = a.n; p.stride = a.stride; p.hist = a.hist; p.nstreams = a.nstreams;
  const int64_t M = (a.n + D - 1) / D;
  p.tiles_per_stream = (int)((M + TO - 1) / TO);
  p.taps_dev = a.taps_dev; p.zi_i = a.zi_i; p.zi_q = a.zi_q; p.zi_stride = a.zi_stride;
  p.prev_phase = a.prev_phase; p.demod = a.demod; p.out_stride = a.out_stride;
  p.i_ds = a.i_ds; p.q_ds = a.q_ds; p.last_phi = a.last_phi; p.wraps = a.wraps;
  p.vec_out = ((a.out_stride % 4) == 0 && ((uintptr_t)a.demod % 16) == 0) ? 1 : 0;
  const int64_t tiles = (int64_t)p.tiles_per_stream * a.nstreams;
  if (tiles <= 0) return hipSuccess;
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  if constexpr (U8) {
    if (a.nstreams > 1 && a.stride % 8 != 0 && !use_slot(false)) return hipErrorInvalidValue;
    if (use_slot(false)) {   // u8 IQ: the slot kernel (2 B per sample staged, converted on write)
      SlotArgs sa{};
      sa.tps = (int)((M + 191) / 192);
      sa.total = (int64_t)sa.tps * a.nstreams;
      return launch_slot_t<T, false, true>(p, *a.taps, sa, st);
    }
    hipLaunchKernelGGL((fe_kernel<T, D, R, NT, true>), dim3((unsigned)tiles), dim3(NT), 0, st, p, *a.taps);
  } else {
    if constexpr (T <= 127) {
      if (use_slot(false)) {
        SlotArgs sa{};
        sa.tps = (int)((M + 191) / 192);
        sa.total = (int64_t)sa.tps * a.nstreams;
        return launch_slot_t<T, false>(p, *a.taps, sa, st);
      }
    }
    if (use_circ()) {
      RingArgs ra{};
      ra.tps = (int)((M + 63) / 64);
      ra.total = (int64_t)ra.tps * a.nstreams;
      static const int wpc = resident_per_cu(fe_circ_kernel<T>, 64);
      const int64_t slots = (int64_t)cu_count() * std::min(wpc, 4);
      ra.per_wave = (int)((ra.total + slots - 1) / slots);
      const int64_t grid = (ra.total + ra.per_wave - 1) / ra.per_wave;
      p.tiles_per_stream = ra.tps;
      hipLaunchKernelGGL((fe_circ_kernel<T>), dim3((unsigned)grid), dim3(64), 0, st, p, *a.taps, ra);
      return hipGetLastError();
    }
    // fe_ring_kernel: 192 outputs per tile, one resident wave per SIMD
    constexpr int TO3 = 192;
    RingArgs ra{};
    ra.tps = (int)((M + TO3 - 1) / TO3);
    ra.total = (int64_t)ra.tps * a.nstreams;
    static const int wpc = resident_per_cu(fe_ring_kernel<T>, 64);
    const int64_t slots = (int64_t)cu_count() * std::min(wpc, 4);
    ra.per_wave = (int)((ra.total + slots - 1) / slots);
    const int64_t grid = (ra.total + ra.per_wave - 1) / ra.per_wave;
    p.tiles_per_stream = ra.tps;
    hipLaunchKernelGGL((fe_ring_kernel<T>), dim3((unsigned)grid), dim3(64), 0, st, p, *a.taps, ra);
  }
  return hipGetLastError();
}

// Returns hipErrorInvalidValue for an unsupported (taps, decim) pair; the C-ABI
// reports that as SDR_EUNSUPPORTED.  Supported: the reference's RF configs
// (151 taps: model/fmMonoBlock.py:24; 101 taps: BASELINE configs) at decim 10.
hipError_t sdr_launch_fe(const FeLaunch& a, hipStream_t st) {
  if (a.D != 10) return hipErrorInvalidValue;
  switch (a.T) {
    case 101: return a.u8 ? launch_fe_t<101, 10, true>(a, st) : launch_fe_t<101, 10, false>(a, st);
    case 151: return a.u8 ? launch_fe_t<151, 10, true>(a, st) : launch_fe_t<151, 10, false>(a, st);
    default: return hipErrorInvalidValue;
  }
}

template <int T>
static hipError_t launch_fe_mono_t(const FeLaunch& a, const float* ataps, float* audio,
                                   int64_t audio_stride, hipStream_t st) {
  constexpr int D = 10, BD = 960;                  // demod samples per audio block
  FeParams p{};
  p.iq = a.iq; p.n = a.n; p.stride = a.stride; p.hist = 0; p.nstreams = a.nstreams;
  p.taps_dev = a.taps_dev;
  const int64_t M = (a.n + D - 1) / D;
  RingArgs ra{};
  ra.ab = (int)((M + BD - 1) / BD);
  ra.tps = 5 * ra.ab;
  ra.total = (int64_t)ra.ab * a.nstreams;
  if (ra.total <= 0) return hipSuccess;
  if (ra.total > 0x7fffffff / 5) return hipErrorInvalidValue;
  ra.audio = audio; ra.audio_stride = audio_stride; ra.ataps = ataps;
  if (a.u8 || use_slot(true)) {     // u8 IQ: only the slot kernel converts on the way in
    SlotArgs sa{};
    sa.tps = ra.tps;
    sa.total = (int64_t)sa.tps * a.nstreams;
    sa.audio = audio; sa.audio_stride = audio_stride; sa.ataps = ataps;
    return a.u8 ? launch_slot_t<T, true, true>(p, *a.taps, sa, st) : launch_slot_t<T, true>(p, *a.taps, sa, st);
  }
  if (use_circ()) {
    ra.ab = (int)((M + 319) / 320);
    ra.tps = 5 * ra.ab;
    ra.total = (int64_t)ra.ab * a.nstreams;
    static const int wpc = resident_per_cu(fe_circ_kernel<T, true>, 64);
    const int64_t slots = (int64_t)cu_count() * std::min(wpc, 4);
    ra.per_wave = (int)((ra.total + slots - 1) / slots);
    const int64_t grid = (ra.total + ra.per_wave - 1) / ra.per_wave;
    p.tiles_per_stream = ra.tps;
    hipLaunchKernelGGL((fe_circ_kernel<T, true>), dim3((unsigned)grid), dim3(64), 0, st, p, *a.taps, ra);
    return hipGetLastError();
  }
  static const int wpc = resident_per_cu(fe_ring_kernel<T, true>, 64);
  const int64_t slots = (int64_t)cu_count() * std::min(wpc, 4);
  ra.total = (int64_t)ra.tps * a.nstreams;           // tiles: balanced tile ranges per wave
  const int64_t grid = std::min<int64_t>(slots, ra.total);
  p.tiles_per_stream = ra.tps;
  hipLaunchKernelGGL((fe_ring_kernel<T, true>), dim3((unsigned)grid), dim3(64), 0, st, p, *a.taps, ra);
  return hipGetLastError();
}

// Fused FE + mono audio filter over whole streams (zero initial state).  Supported: f32 IQ,
// RF taps 101 at decim 10, audio taps 151 at decim 5 (model/fmMonoBlock.py:24-31, BASELINE
// configs); anything else returns hipErrorInvalidValue and the C-ABI runs the two-kernel path.
hipError_t sdr_launch_fe_mono(const FeLaunch& a, const float* ataps, int TA, int DA, float* audio,
                              int64_t audio_stride, hipStream_t st) {
  if (a.D != 10 || TA != 151 || DA != 5) return hipErrorInvalidValue;
  switch (a.T) {
    case 101: return launch_fe_mono_t<101>(a, ataps, audio, audio_stride, st);
    default: return hipErrorInvalidValue;   // 151 RF taps: 3 waves/CU by LDS -> two-kernel path
  }
}

hipError_t sdr_launch_iq_zf(const void* iq, int u8, int64_t n, int64_t stride, int nstreams,
                            const double* b_dev, int T, const double* zi_i, const double* zi_q,
                            int64_t zi_stride, double* zf_i, double* zf_q, hipStream_t st) {
  if (T <= 1 || nstreams <= 0) return hipSuccess;
  if (T > SDR_MAX_TAPS) return hipErrorInvalidValue;
  const dim3 grid(1, nstreams);
  if (u8)
    hipLaunchKernelGGL(iq_zf_kernel<true>, grid, dim3(256), 0, st, iq, n, stride, b_dev, T, zi_i, zi_q, zi_stride, zf_i, zf_q);
  else
    hipLaunchKernelGGL(iq_zf_kernel<false>, grid, dim3(256), 0, st, iq, n, stride, b_dev, T, zi_i, zi_q, zi_stride, zf_i, zf_q);
  return hipGetLastError();
}

// Standalone discriminator on separate I/Q arrays (model/fmSupportLib.py:15-44):
// one lane per sample, phi_{k-1} recomputed from (I,Q)_{k-1} (k = 0 uses the state).
__global__ __launch_bounds__(256) void demod_kernel(const float* I, const float* Q, int64_t n,
                                                   int64_t stride, const double* prev_phase,
                                                   float* out, int64_t out_stride,
                                                   float* last_phi, int* wraps) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  const float* is = I + (int64_t)s * stride;
  const float* qs = Q + (int64_t)s * stride;
  int wk = 0;
  if (k < n) {
    const float phi = atan2f(qs[k], is[k]);
    float d;
    if (k == 0) {
      const double ps = prev_phase ? prev_phase[s] : 0.0;
      d = (float)unwrap_step_f64((double)phi - ps, &wk);
    } else {
      d = phi - atan2f(qs[k - 1], is[k - 1]);
      if (d > kPiF) { d -= k2PiF; wk = -1; }
      else if (d < -kPiF) { d += k2PiF; wk = 1; }
    }
    out[(int64_t)s * out_stride + k] = d;
    if (k == n - 1 && last_phi != nullptr) last_phi[s] = phi;
  }
  if (wraps != nullptr) {
    wk = wave_sum_i(wk);
    if ((threadIdx.x & 63) == 0 && wk != 0) atomicAdd(wraps + s, wk);
  }
}

// Carried demod state after a block: the reference returns the accumulated unwrapped
// phase prev + sum(d) = phi_last + 2*pi*W (W = sum of 2*pi corrections).
__global__ void demod_state_kernel(int nstreams, int64_t m, const float* last_phi,
                                   const int* wraps, double* prev_phase) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstreams || m <= 0) return;
  prev_phase[s] = (double)last_phi[s] + k2Pi * (double)wraps[s];
}

hipError_t sdr_launch_demod(const float* I, const float* Q, int64_t n, int64_t stride, int nstreams,
                            const double* prev_phase, float* out, int64_t out_stride,
                            float* last_phi, int* wraps, hipStream_t st) {
  if (n <= 0 || nstreams <= 0) return hipSuccess;
  hipLaunchKernelGGL(demod_kernel, dim3((unsigned)((n + 255) / 256), nstreams), dim3(256), 0, st,
                     I, Q, n, stride, prev_phase, out, out_stride, last_phi, wraps);
  return hipGetLastError();
}

hipError_t sdr_launch_demod_state(int nstreams, int64_t m, const float* last_phi, const int* wraps,
                                  double* prev_phase, hipStream_t st) {
  if (nstreams <= 0) return hipSuccess;
  hipLaunchKernelGGL(demod_state_kernel, dim3((nstreams + 63) / 64), dim3(64), 0, st, nstreams, m,
                     last_phi, wraps, prev_phase);
  return hipGetLastError();
}
