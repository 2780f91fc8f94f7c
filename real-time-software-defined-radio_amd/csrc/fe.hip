// RF front end for gfx950: interleaved IQ -> low-pass FIR -> keep every D-th output ->
// atan2 FM discriminator (-> optionally the mono audio FIR), fused in one pass over HBM.
//
// Replaces, per block:
//   model/fmMonoBlock.py:86-95   signal.lfilter(rf_coeff, 1.0, iq[0::2]/iq[1::2], zi) + [::10]
//   model/fmMonoBlock.py:98      fmDemodArctan(i_ds, q_ds, state_phase)  (model/fmSupportLib.py:15-44)
//   model/fmMonoBlock.py:101-109 audio lfilter(audio_coeff, ..., zi) + [::5]   (FUSED kernels)
//   src/filter.cpp:187-219       convolveWithDecimIQ;  src/rf_module.cpp:13-34 fmDemodArctan
//   src/iofunc.cpp:61-69         u8 normalisation (u8 input: fe_slot_kernel)
//
// Per tile of TO = 64*R = 192 consecutive decimated outputs [m0, m0+TO) of one stream:
//   1. the input span n in [D(m0-1)-(T-1), D(m0+TO-1)] (the "image", 16 or 17 chunks of
//      128 complex samples) is in LDS as (I,Q) f32 pairs; only the decimated outputs are
//      ever computed (no 9-of-10 wasted outputs as in the Python model);
//   2. lane l owns outputs m0+3l .. m0+3l+2 and slides once over its 121-sample window
//      (v_pk_fma_f32 on (I,Q) pairs, taps in VGPR pairs broadcast through op_sel);
//   3. phi = atan2(q, i); the predecessor phase of lane l is lane l-1's last phase (DPP
//      wave_shr:1), lane 0 takes the wave's carried phase of output m0-1;
//   4. d = wrap(phi - phi_prev) reproduces np.unwrap on a 2-element list
//      (numpy _function_base_impl.py:1790-1800).  The number of 2*pi
//      corrections W is reduced per stream so the host can return the reference's
//      accumulated (unwrapped) phase state: prev_out = phi_last + 2*pi*W.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "sdr_launch.h"

namespace {

struct FeParams {
  const void* iq;            // device, interleaved IQ
  int64_t n;                 // complex samples per stream
  int64_t stride;            // complex samples between stream bases
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

// f32 interleaved: one complex sample = 8 B.
template <> struct IqLoad<false> {
  __device__ static float2 load1(const void* base, int64_t n) {
    return reinterpret_cast<const float2*>(base)[n];
  }
};

// u8 interleaved: x = (u8 - 128) / 128 (exact in f32).
template <> struct IqLoad<true> {
  __device__ static float cvt(uint32_t b) { return ((float)b - 128.0f) * 0.0078125f; }
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

// s_waitcnt vmcnt(n) for a wave-uniform runtime n in [0, 63] (binary search over the
// immediate; waiting for more than needed is always safe, so n is clamped down).
// a sample-index bound relative to a lane's image start, clamped into int range (images
// are < 2^16 samples): 64-bit compares per chunk would hold 64-bit registers per chunk
__device__ __forceinline__ int rel_bound(int64_t v) {
  return (int)max<int64_t>(min<int64_t>(v, 1 << 20), -(1 << 20));
}

template <int LO, int HI>
__device__ __forceinline__ void wait_vm_bs(int n) {
  if constexpr (LO == HI) {
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(LO) : "memory");
  } else {
    constexpr int MID = (LO + HI + 1) / 2;
    if (n >= MID) wait_vm_bs<MID, HI>(n);
    else wait_vm_bs<LO, MID - 1>(n);
  }
}
__device__ __forceinline__ void wait_vm(int n) {
  wait_vm_bs<0, 63>(__builtin_amdgcn_readfirstlane(n < 0 ? 0 : (n > 63 ? 63 : n)));
}

// General epilogue (head / tail / zi / i_ds tiles): zi add, atan2, predecessor phase (lane
// 0 gets the wave-reduced sums (si, sq) of output mw-1, or phi_prev when have_prev; lane
// l>0 takes lane l-1's last phase), np.unwrap wrap, stores, wrap count and last phase.
// Lane l owns outputs mw + R*l .. mw + R*l + R-1.  Returns the phase of the wave's last
// output (lane 63's).  The caller drains vmcnt afterwards.
template <int T, int D, int R>
__device__ __forceinline__ float fe_epilogue(const FeParams& p, int s, int64_t M, int64_t mw, int lane,
                                             float (&ai)[R], float (&aq)[R], float si, float sq,
                                             bool have_prev, float phi_prev, float* dv, bool do_store) {
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
#pragma unroll
  for (int r = 0; r < R; ++r) dv[r] = d[r];
  float* out = p.demod + (int64_t)s * p.out_stride;
  if (do_store && p.demod != nullptr) {
    if (R == 3 && mf + R <= M) {
      typedef float f3v __attribute__((ext_vector_type(3)));
      *reinterpret_cast<f3v*>(out + mf) = f3v{d[0], d[1 % R], d[2 % R]};
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (mf + r < M) out[mf + r] = d[r];
    }
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
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[R - 1]), 63));
}

// Register-blocked FIR of one tile image: lane l produces the R decimated (I, Q) outputs
// of its window [D R l + D, + D(R-1)+T) (odd T).  One ds_read_b128 (two complex samples)
// per step, issued by hand PF steps ahead with counted lgkmcnt waits (hipcc would split
// the 16-B read into ds_read2_b64, 4-8-way bank-conflicted at this lane stride, and read
// only one pair ahead); taps in VGPR pairs {h[2j], h[2j+1]}, broadcast by op_sel.
template <int T, int D, int R, int PF, int OFF = D>
__device__ __forceinline__ void fe_fir_tile(const f2v* buf, int lane, const f2v (&tp)[(T + 1) / 2],
                                            float (&ai)[R], float (&aq)[R]) {
  static_assert((T & 1) == 1 && (OFF & 1) == 0, "the lane window starts 16-B aligned");
  constexpr int NI = D * (R - 1) + T;
  const f2v* win = buf + (D * R * lane + OFF);
  const float4* win4 = reinterpret_cast<const float4*>(__builtin_assume_aligned(win, 16));
  f2v acc[R], acc2[R];   // even / odd taps: 2R independent FMA chains
#pragma unroll
  for (int r = 0; r < R; ++r) { acc[r] = f2v{0.f, 0.f}; acc2[r] = f2v{0.f, 0.f}; }
  constexpr int NP = (NI + 1) / 2;
  static_assert(PF >= 1 && PF <= 15, "lgkmcnt field");
  f4v qb[NP];
  static_for<0, (PF < NP ? PF : NP)>([&](auto I) { qb[I] = lds_read_b128<16 * I>(win4); });
  lds_wait<PF - 1 < NP - 1 ? PF - 1 : NP - 1>(qb[0]);
  static_for<0, NP>([&](auto I) {
    constexpr int ip = I;
    if constexpr (ip + PF < NP) qb[ip + PF] = lds_read_b128<16 * (ip + PF)>(win4);
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
          if (k & 1) pk_fma_bcast<true>(acc2[r], tp[k >> 1], x);
          else pk_fma_bcast<false>(acc[r], tp[k >> 1], x);
        }
      }
    }
    // the wait "redefines" the next step's register ("+v"), so the allocator cannot copy
    // an in-flight value before its data has arrived
    if constexpr (ip + 1 < NP) {
      constexpr int issued_r = (ip + PF + 1 < NP) ? ip + PF + 1 : NP;
      lds_wait<issued_r - (ip + 2)>(qb[ip + 1]);
    }
  });
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const f2v t = acc[r] + acc2[r];
    ai[r] = t.x;
    aq[r] = t.y;
  }
}

// FE FIR of one R=3 tile (as fe_fir_tile) with the previous audio block's 3-output-per-
// lane audio FIR interleaved step by step (fe_ring_kernel<FUSED>): the audio reads (lane
// samples by ds_read2_b32, tap triples by broadcast ds_read_b128) are latency-bound on
// their own, the FE FIR is VALU-bound; interleaved, each covers the other.  One static
// schedule: macro-step t runs FE step t and audio steps [NS*t/NP, NS*(t+1)/NP); reads are
// issued PF (FE) / APF (audio) steps ahead and every wait counts the reads issued after
// the one it needs (all compile-time; lgkmcnt <= 15 is asserted).
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

template <int T, int PF, int APF, int OFF>
__device__ __forceinline__ void fir_audio_tile(const f2v* buf, int lane, const f2v (&tp)[(T + 1) / 2],
                                               float (&ai)[3], float (&aq)[3], const float* aw,
                                               const f4v* ptab, float& o0, float& o1, float& o2) {
  constexpr int D = 10, R = 3;
  constexpr int NI = D * (R - 1) + T;
  constexpr int NP = (NI + 1) / 2;                   // FE steps (sample pairs)
  constexpr int NS = 81;                             // audio steps (161-sample window in pairs)
  using S = fa::Sched<NP, NS, PF, APF>;
  static_assert((OFF & 1) == 0, "the lane window starts 16-B aligned");
  const f2v* win = buf + (D * R * lane + OFF);
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

// ---------------------------------------------------------------------------------
// fe_ring_kernel: the product f32 front end (FE only, and FE + mono when FUSED).
//
// Persistent: one 64-lane wave per workgroup, 4 resident per CU (one per SIMD: the
// slot stride keeps a 5th wave out), each wave a balanced contiguous range of tiles.
// Memory pipeline (measured on the shape probe tools/pipe_probe.hip, r02):
//  * two LDS image slots per wave; tile t+1's 15 new 1-KiB chunks are LDS-DMA'd
//    (global_load_lds_dwordx4 nt, saddr form, four chunks per M0 setup) into the other
//    slot BEFORE the wave waits for tile t, so two tiles are in flight during every
//    wait; consecutive tiles overlap by HCH chunks, copied LDS->LDS (HBM bytes = the
//    algorithmic bytes);
//  * vmcnt is exact: a running count of the wave's VMEM instructions and a mark per tile;
//  * NO output stores during the run: the steady tiles' outputs (FE: 3 demod values per
//    lane per tile; FUSED: 3 audio values per lane per block) wait in registers (OutQ3)
//    and are written when the run ends.  Stores interleaved with the read stream cost
//    ~5x their bytes (probe: 80 us without stores, 96 us with one 768-B store per tile,
//    84 us with the same bytes written after the run).
// Head / tail tiles (zi, prev_phase, i_ds, partial tiles, stream edges) take the general
// epilogue (fe_epilogue) and store directly.
//
// FUSED (sdr_fe_mono_dev, the continuous-stream mono receiver): an audio block is 5 tiles
// = 960 demod samples = 192 audio outputs (3 per lane).  Demod values go to a
// wave-private LDS history; a block's audio FIR runs interleaved with the next tile's FE
// FIR (fir_audio_tile).  A run starting mid-stream first runs one warm-up tile (192 >=
// 150 history samples).  Output j is stored only by the wave whose tile range holds its
// newest input sample 5j, so every audio output is written exactly once.
// ---------------------------------------------------------------------------------
struct RingArgs {
  int64_t total;       // tiles over all streams
  int tps;             // tiles per stream
  float* audio;        // FUSED: per stream ceil(M/5) audio samples, audio_stride apart
  int64_t audio_stride;
  const float* ataps;  // FUSED: 151 audio taps (device)
};

template <int T, bool FUSED>
__global__ __launch_bounds__(64) void fe_ring_kernel(FeParams p, TapsF32 taps, RingArgs a) {
  constexpr int D = 10, R = 3, TO = 64 * R;
  constexpr int NEWC = D * TO / 128;                 // 15 new 1-KiB chunks per tile
  // image start n_lo = D*(m0-1) - (T-1) - DELTA, DELTA >= 0 chosen so that every chunk's
  // source address is 128-B aligned (f32: n_lo % 16 == 0): a 1-KiB LDS-DMA then covers
  // 8 whole cache lines instead of 9 partial ones
  constexpr int DELTA = (16 - (D + T - 1) % 16) % 16;
  constexpr int OFF = D + DELTA;                     // lane 0's window start in the image
  constexpr int NCH = (D * TO + T + DELTA + 127) / 128;  // chunks per tile image
  constexpr int HCH = NCH - NEWC;                    // halo chunks shared with the next tile
  constexpr int L = NCH * 128;                       // image length (complex samples)
  constexpr int TP = (T + 1) / 2;
  constexpr int PF = T > 127 ? 8 : 12;               // FE FIR LDS reads in flight
  static_assert((T & 1) == 1 && HCH >= 1 && HCH <= 2, "odd tap counts 101..235");
  static_assert(!FUSED || T <= 127, "FUSED: 16-chunk images (4 waves per CU)");
  constexpr int TA = 151, DA = 5, RA = R;            // audio: 151 taps, decim 5
  constexpr int TPB = DA;                            // tiles per audio block
  constexpr int BD = TO * TPB;                       // 960 demod samples per block
  constexpr int BO = 64 * RA;                        // 192 audio outputs per block
  constexpr int HA = 152;                            // history slots (>= TA-1)
  constexpr int NW = DA * (RA - 1) + TA;             // 161-sample audio window per lane
  // slot stride >= 20 KiB: at most 4 resident waves per CU
  constexpr int LS = FUSED ? L : (L > 2560 ? L : 2560);
  __shared__ __attribute__((aligned(16))) f2v ring[2][LS];
  __shared__ __attribute__((aligned(16))) float dh[FUSED ? HA + BD + 4 : 1];
  __shared__ __attribute__((aligned(16))) f4v ptab[FUSED ? NW + 1 : 1];

  const int lane = threadIdx.x;
  const int64_t g0 = (int64_t)blockIdx.x * a.total / gridDim.x;
  const int64_t g1 = ((int64_t)blockIdx.x + 1) * a.total / gridDim.x;
  if (g0 >= g1) return;
  const int64_t M = (p.n + D - 1) / D;

  f2v tp[TP];
#pragma unroll
  for (int j = 0; j < TP; ++j) tp[j] = f2v{taps.h[2 * j], (2 * j + 1 < T) ? taps.h[2 * j + 1] : 0.f};
#pragma unroll
  for (int j = 0; j < TP; ++j) asm volatile("" : "+v"(tp[j]));

  constexpr int NK = (T + 63) / 64;
  float hk[NK];

  const unsigned voff = 16u * lane;
  const float* iqf = reinterpret_cast<const float*>(p.iq);
  // tile i: outputs TO*i ..; image = samples [n_lo, n_lo + L), n_lo = D*(m0-1) - (T-1)
  auto n_lo_of = [&](int ii) { return (int64_t)(D * TO) * ii - D - (T - 1) - DELTA; };
  // LDS-DMA needs the image inside [-hist, n) and a 16-B aligned base (the C-ABI passes
  // 16-B aligned IQ and an even stream stride for this kernel)
  auto dma_full = [&](int64_t nl) { return nl >= -p.hist && nl + L <= p.n; };
  auto dma_halo = [&](int64_t nl) { return nl + HCH * 128 >= -p.hist && nl + L <= p.n; };
  // chunks [0 or HCH, NCH) of the image at nl (stream ss) -> ring slot sl; returns the count
  auto issue = [&](int ss, int64_t nl, int sl, bool full) -> int {
    const char* g = reinterpret_cast<const char*>(iqf + 2 * ((int64_t)ss * p.stride + nl));
    const unsigned lb = lds_addr_of(&ring[sl][0]);
    auto run = [&](auto C0) {
      constexpr int c0 = decltype(C0)::value;
      static_for<0, (NCH - c0 + 3) / 4>([&](auto Q) {
        constexpr int c = c0 + 4 * Q;
        constexpr int k = (NCH - c) < 4 ? (NCH - c) : 4;
        glds16x<k>(voff, g + 1024 * c, lb + 1024 * c);
      });
    };
    if (full) { run(std::integral_constant<int, 0>{}); return NCH; }
    run(std::integral_constant<int, HCH>{});
    return NEWC;
  };
  // guarded image build (stream edges): zeros outside [-hist, n)
  // every lane's L/64 predicated 8-B loads are issued before the first use (one memory
  // round trip; a load-use loop here serialised ~32 round trips and made the waves
  // holding a stream's head or tail the last to finish)
  auto build = [&](int ss, int64_t nl, int sl) {
    const f2v* base = reinterpret_cast<const f2v*>(iqf) + (int64_t)ss * p.stride;
    f2v* buf = &ring[sl][0];
    constexpr int NPL = L / 64;
    f2v v[NPL];
#pragma unroll
    for (int j = 0; j < NPL; ++j) {
      const int64_t nn = nl + 64 * j + lane;
      v[j] = (nn >= -p.hist && nn < p.n) ? base[nn] : f2v{0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < NPL; ++j) buf[64 * j + lane] = v[j];
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  };

  // ---- tile sequence of this wave ----
  int s = (int)(g0 / a.tps);
  int i = (int)(g0 - (int64_t)s * a.tps);
  int U = (int)(g1 - g0);
  bool mid = false;
  // a run starting mid-stream first runs the warm-up tile i-1 (history / predecessor);
  // a run may start and end mid audio block (audio_store keeps to the outputs it owns)
  if constexpr (FUSED) {
    mid = i > 0;
    if (mid) { --i; ++U; }
  }
  // image kinds: 1 guarded build, 2 DMA (whole image), 3 DMA (new chunks; halo by LDS copy)
  enum { K_NONE = 0, K_BUILD = 1, K_FULL = 2, K_HALO = 3 };
  int64_t nl = n_lo_of(i);
  int b = 0;
  int issued = 0, mark = 0;                        // VMEM instructions issued / per-tile mark
  int kind = dma_full(nl) ? K_FULL : K_BUILD;
  // r04b: the first image's DMA goes out before the prologue's own loads (this lane's taps for a
  // run's cooperative predecessor output; FUSED: the audio tap table), and one wait covers all:
  // the launch pays one memory round trip before its first tile instead of three
  if (kind == K_FULL) issue(s, nl, 0, true);
#pragma unroll
  for (int q = 0; q < NK; ++q) hk[q] = (lane + 64 * q < T) ? p.taps_dev[lane + 64 * q] : 0.f;
  if constexpr (FUSED) {
    for (int e = lane; e < HA + BD + 4; e += 64) dh[e] = 0.f;   // finite everywhere (0 * x)
    for (int w = lane; w < NW + 1; w += 64) {               // entry NW: zero (pairs over-read)
      const int k0 = (TA - 1) - w, k1 = k0 + DA, k2 = k0 + 2 * DA;
      ptab[w] = f4v{(k0 >= 0 && k0 < TA) ? a.ataps[k0] : 0.f, (k1 >= 0 && k1 < TA) ? a.ataps[k1] : 0.f,
                    (k2 >= 0 && k2 < TA) ? a.ataps[k2] : 0.f, 0.f};
    }
  }
  // the first image landed too (nothing in flight: issued = mark = 0)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int q = 0; q < NK; ++q) asm volatile("" : "+v"(hk[q]));
  float carry = 0.f;                               // phase of the previous tile's last output
  bool have = false;                               // carry valid (previous tile, same stream)
  int wacc = 0;                                    // per-lane 2*pi correction count

  // ---- deferred outputs (OutQ3): FE demod tiles / FUSED audio blocks ----
  // FUSED, r04b: 16 audio blocks (48 VGPRs of queue, 20 of them AGPRs) hold a whole run of the
  // 128-block step (13.4 blocks per wave), so no flush goes out mid-run beside the read stream
  // (12: one at block 12 of every wave at once); A/B 0.738 -> 0.747 of HBM on one box
  constexpr int QN = FUSED ? 16 : 36;             // (fixed constants)
  OutQ3<QN> oq;
  int qn = 0, qs = 0;
  int64_t q0 = 0;                                  // FE: first tile; FUSED: first audio block
  // FUSED: audio outputs [own_lo(ss), own_hi(ss)) of stream ss are this run's (5 j inside
  // its tile range): every output is stored by exactly one wave
  auto own_lo = [&](int ss) {
    const int64_t lo = max<int64_t>(g0 - (int64_t)ss * a.tps, 0);
    return (TO * lo + DA - 1) / DA;
  };
  auto own_hi = [&](int ss) {
    const int64_t hi = min<int64_t>(g1 - (int64_t)ss * a.tps, a.tps);
    return min<int64_t>((TO * hi + DA - 1) / DA, (M + DA - 1) / DA);
  };
  auto q_flush = [&]() __attribute__((always_inline)) {
    if (qn == 0) return;
    if constexpr (FUSED) {
      // masked stores: not counted in `issued` (a smaller count only makes waits longer)
      oq.flush_owned(a.audio + (int64_t)qs * a.audio_stride + q0 * BO + RA * lane, BO, qn,
                     q0 * BO + RA * lane, own_lo(qs), own_hi(qs));
    } else {
      issued += oq.flush(p.demod + (int64_t)qs * p.out_stride + q0 * TO + R * lane, TO, qn);
    }
    qn = 0;
  };
  auto q_push = [&](int64_t idx, float x0, float x1, float x2) __attribute__((always_inline)) {
    if (qn > 0 && (qs != s || q0 + qn != idx || qn == QN)) q_flush();
    if (qn == 0) { qs = s; q0 = idx; }
    oq.put(qn, x0, x1, x2);
    ++qn;
  };

  // ---- FUSED audio pieces ----
  const float* aw_lane = dh + (HA - (TA - 1) + DA * RA * lane);   // lane window in dh
  // block q's outputs go to the deferred queue (the flush keeps to the owned outputs)
  auto audio_put = [&](int64_t q, float o0, float o1, float o2) __attribute__((always_inline)) -> bool {
    q_push(q, o0, o1, o2);
    return false;
  };
  auto dh_shift = [&](bool next_same) {
    asm volatile("" ::: "memory");
    if (!next_same)
      for (int e = lane; e < HA; e += 64) dh[e] = 0.f;     // the next block starts a new stream
    else
      for (int e = lane; e < HA; e += 64) dh[e] = dh[BD + e];
    asm volatile("" ::: "memory");
  };
  auto dh_write = [&](int ii, bool warm, const float (&d)[R]) {
    const int ib = ii % TPB;                       // tile within its audio block
    const int rel0 = (warm ? -TO : ib * TO) + R * lane;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (rel0 + r >= -HA) dh[HA + rel0 + r] = d[r];
    asm volatile("" ::: "memory");
  };
  bool pend = false;                               // FUSED: a finished block's audio is due
  int64_t q_pend = 0;

  // interior tile epilogue: phases, predecessor (DPP / carry), np.unwrap wrap
  auto fast_epi = [&](const float (&ai)[R], const float (&aq)[R], float (&d)[R]) __attribute__((always_inline)) {
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
  // last tile whose image is interior (DMA) and last tile with the fast epilogue, per stream
  const int64_t jn = p.n + D + (T - 1) + DELTA - L;
  const int64_t j_int = jn >= 0 ? jn / (D * TO) : -1;
  const int64_t j_fast = M >= TO + 1 ? (M - TO - 1) / TO : -1;

  for (int u = 0; u < U; ++u) {
    // ---- steady run: consecutive interior tiles of one stream, fixed VMEM pattern ----
    // Entry: tile i's new chunks are in flight into slot b (its halo written), carry valid.
    // Per tile: the next tile's 15 chunks -> slot b^1, s_waitcnt vmcnt(15), FIR, halo,
    // fast epilogue, outputs to the deferred queue.  Exit: the same state for tile i+K.
    if (kind == K_HALO && have && p.i_ds == nullptr) {
      int64_t K = min<int64_t>(U - 1 - u, a.tps - 1 - i);
      K = min<int64_t>(K, j_int - i);
      K = min<int64_t>(K, j_fast - i + 1);
      if constexpr (!FUSED) {
        if (qn > 0 && (qs != s || q0 + qn != i)) q_flush();
        K = min<int64_t>(K, QN - qn);
      }
      if (K > 0) {
        const char* gn = reinterpret_cast<const char*>(iqf + 2 * ((int64_t)s * p.stride + nl + D * TO)) + 1024 * HCH;
        const int first_wait = issued - mark + NEWC;
        for (int k = 0; k < (int)K; ++k) {
          const unsigned lb = lds_addr_of(&ring[b ^ 1][0]) + 1024 * HCH;
          static_for<0, (NEWC + 3) / 4>([&](auto Q) {
            constexpr int c = 4 * Q;
            constexpr int nc = (NEWC - c) < 4 ? (NEWC - c) : 4;
            glds16x<nc>(voff, gn + 1024 * c, lb + 1024 * c);
          });
          gn += D * TO * 8;
          issued += NEWC;
          int mk = issued;
          // tile i: every VMEM instruction after its DMA is this tile's 15 chunks (k > 0:
          // stores issued in between only make the wait longer, never short)
          if (k == 0) wait_vm(first_wait);
          else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NEWC) : "memory");
          f2v* buf = &ring[b][0];
          f2v* nb = &ring[b ^ 1][0];
          f4v h0 = lds_read_b128<0>(buf + NEWC * 128 + 2 * lane), h1;
          if constexpr (HCH == 2) h1 = lds_read_b128<0>(buf + (NEWC + 1) * 128 + 2 * lane);
          float ai[R], aq[R];
          if constexpr (FUSED) {
            if (pend) {
              float o0, o1, o2;
              fir_audio_tile<T, 2, 2, OFF>(buf, lane, tp, ai, aq, aw_lane, ptab, o0, o1, o2);
              if (audio_put(q_pend, o0, o1, o2)) mk = issued;
              dh_shift(true);
              pend = false;
            } else {
              fe_fir_tile<T, D, R, PF, OFF>(buf, lane, tp, ai, aq);
            }
          } else {
            fe_fir_tile<T, D, R, PF, OFF>(buf, lane, tp, ai, aq);
          }
          lds_wait<0>(h0);
          lds_write_b128(nb + 2 * lane, h0);
          if constexpr (HCH == 2) { lds_wait<0>(h1); lds_write_b128(nb + 128 + 2 * lane, h1); }
          float d[R];
          fast_epi(ai, aq, d);
          if constexpr (FUSED) {
            dh_write(i, false, d);
            if (i % TPB == TPB - 1) { pend = true; q_pend = i / TPB; }
          } else {
            q_push(i, d[0], d[1], d[2]);
          }
          mark = mk;
          b ^= 1;
          ++i;
          nl += D * TO;
        }
        u += (int)K;
      }
    }
    // ---- next tile: position, kind, DMA issue (before this tile's wait) ----
    int s1 = s, i1 = i + 1;
    if (i1 == a.tps) { i1 = 0; ++s1; }
    const int64_t nl1 = (s1 == s) ? nl + D * TO : n_lo_of(0);
    int kind1 = K_NONE, mark1 = 0;
    if (u + 1 < U) {
      if (s1 == s && dma_halo(nl1)) kind1 = K_HALO;
      else kind1 = dma_full(nl1) ? K_FULL : K_BUILD;
      if (kind1 >= K_FULL) { issued += issue(s1, nl1, b ^ 1, kind1 == K_FULL); mark1 = issued; }
    }
    // ---- this tile's image ----
    f2v* buf = &ring[b][0];
    if (kind == K_BUILD) {
      build(s, nl, b);                             // drains vmcnt (the next tile's DMA too)
      issued = 0; mark1 = 0;
    } else {
      wait_vm(issued - mark);
    }
    // halo of the next tile: read now, written after the FIR
    f4v h0, h1;
    if (kind1 == K_HALO) {
      h0 = lds_read_b128<0>(buf + NEWC * 128 + 2 * lane);
      if constexpr (HCH == 2) h1 = lds_read_b128<0>(buf + (NEWC + 1) * 128 + 2 * lane);
    }
    float ai[R], aq[R];
    if constexpr (FUSED) {
      if (pend) {                                  // the previous block's audio, interleaved
        float o0, o1, o2;
        fir_audio_tile<T, 2, 2, OFF>(buf, lane, tp, ai, aq, aw_lane, ptab, o0, o1, o2);
        if (audio_put(q_pend, o0, o1, o2)) mark1 = 0;
        dh_shift(true);
        pend = false;
      } else {
        fe_fir_tile<T, D, R, PF, OFF>(buf, lane, tp, ai, aq);
      }
    } else {
      fe_fir_tile<T, D, R, PF, OFF>(buf, lane, tp, ai, aq);
    }
    if (kind1 == K_HALO) {
      f2v* nb = &ring[b ^ 1][0];
      lds_wait<0>(h0);
      lds_write_b128(nb + 2 * lane, h0);
      if constexpr (HCH == 2) { lds_wait<0>(h1); lds_write_b128(nb + 128 + 2 * lane, h1); }
    }

    // ---- epilogue ----
    const int64_t m0 = (int64_t)TO * i;
    float d[R];
    // predecessor output m0-1 of a run's first tile: image samples [0, T), register taps
    auto pred = [&](float& si, float& sq) {
      si = 0.f; sq = 0.f;
#pragma unroll
      for (int q = 0; q < NK; ++q) {
        if (lane + 64 * q < T) {
          const f2v x = buf[DELTA + (T - 1) - (lane + 64 * q)];
          si = fmaf(hk[q], x.x, si);
          sq = fmaf(hk[q], x.y, sq);
        }
      }
      si = wave_sum(si);
      sq = wave_sum(sq);
    };
    if (!have && i >= 1 && m0 + TO < M && p.i_ds == nullptr) {
      // an interior first tile (no zi, no carried phase, no store of its own): the fast path
      float si, sq;
      pred(si, sq);
      carry = fast_atan2f(sq, si);
      have = true;
    }
    if (have && i >= 1 && m0 + TO < M && p.i_ds == nullptr) {
      fast_epi(ai, aq, d);                         // interior tile; output deferred
      if constexpr (!FUSED) q_push(i, d[0], d[1], d[2]);
    } else {
      float si = 0.f, sq = 0.f;
      if (m0 > 0 && !have) pred(si, sq);           // output m0-1
      carry = fe_epilogue<T, D, R>(p, s, M, m0, lane, ai, aq, si, sq, have, carry, d, !FUSED);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      issued = 0; mark1 = 0;
    }

    // ---- FUSED: demod -> history; after a block's last tile, its audio ----
    if constexpr (FUSED) {
      const bool warm = mid && u == 0 && (i + 1) % TPB == 0;   // warm-up = previous block's last tile
      dh_write(i, warm, d);
      const bool last = (u + 1 == U) && !(mid && u == 0);
      if (!warm && (i % TPB == TPB - 1 || last)) {
        if (i % TPB == TPB - 1 && u + 1 < U && s1 == s) {
          pend = true;                             // computed during the next tile's FIR
          q_pend = i / TPB;
        } else {
          float o0, o1, o2;
          audio_block3(aw_lane, ptab, o0, o1, o2);
          if (audio_put(i / TPB, o0, o1, o2)) mark1 = 0;
          dh_shift(s1 == s);
        }
      }
    }

    // ---- advance ----
    if ((s1 != s || u + 1 == U) && p.wraps != nullptr) {
      const int w = wave_sum_i(wacc);
      if (w != 0) {
        if (lane == 0) atomicAdd(p.wraps + s, w);
        issued += 1;
      }
      wacc = 0;
    }
    have = (s1 == s);
    s = s1; i = i1; nl = nl1;
    kind = kind1; mark = mark1;
    b ^= 1;
  }
  q_flush();
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
// fe_slot_kernel: the u8-IQ front end (FE only and FUSED), two waves per SIMD.
//
// u8 IQ is 2 B per complex sample, so this launch is bound by issue, not HBM: a second
// wave per SIMD pays.  A wave holds ONE image slot: the next tile's 15 new 128-sample
// chunks are loaded into VGPRs (one dword = two complex samples per lane per chunk) while
// the current tile is filtered, converted to f32 and written into the slot after the FIR
// (the halo chunk moves from position 15 to 0 through a VGPR).
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

// U8: interleaved u8 IQ; the stage holds the next tile's 15 new 128-sample chunks as one
// dword per lane (2 B per complex sample), converted to (x-128)/128 f32 pairs when it is
// written into the slot (the same f32 image as the f32 input).  PF: FIR reads in flight.
template <int T, bool FUSED, bool U8>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2)))
void fe_slot_kernel(FeParams p, TapsF32 taps, SlotArgs a) {
  constexpr int D = 10, R = 3, TO = 64 * R;
  constexpr int NEWC = D * TO / 128;                 // 15 new 128-sample chunks per tile
  constexpr int NCH = (D * TO + T + 1 + 127) / 128;  // chunks per tile image
  constexpr int HCH = NCH - NEWC;                    // halo chunks shared with the next tile
  constexpr int L = NCH * 128;                       // image length (complex samples)
  constexpr int TP = (T + 1) / 2;
  static_assert((T & 1) == 1 && (HCH == 1 || HCH == 2), "odd tap counts 101..235");
  constexpr int PF = 4;
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
      // predicated 2-B loads (one complex u8 sample each), all in flight before the first
      // use; one per-lane base pointer with immediate offsets and 32-bit bounds (per-chunk
      // 64-bit addresses next to the tap registers spill to scratch)
      const uint16_t* bp = reinterpret_cast<const uint16_t*>(p.iq) + ((int64_t)ss * p.stride + nl + lane);
      const int lo = rel_bound(-p.hist - nl - lane), hi = rel_bound(p.n - nl - lane);
      constexpr int NPL = L / 64;
      uint32_t v[NPL];
#pragma unroll
      for (int j = 0; j < NPL; ++j) v[j] = (64 * j >= lo && 64 * j < hi) ? (uint32_t)bp[64 * j] : 0x8080u;  // 0x80 -> 0.0
#pragma unroll
      for (int j = 0; j < NPL; ++j) slot[64 * j + lane] = f2v{cvt8(v[j] & 0xff), cvt8(v[j] >> 8)};
    } else if (interior(nl)) {
      const char* g = reinterpret_cast<const char*>(iqf + 2 * ((int64_t)ss * p.stride + nl));
      const unsigned lb = lds_addr_of(slot);
      static_for<0, (NCH + 3) / 4>([&](auto Q) {
        constexpr int c = 4 * Q;
        constexpr int n = (NCH - c) < 4 ? (NCH - c) : 4;
        glds16x<n>(voff, g + 1024 * c, lb + 1024 * c);
      });
    } else {
      const f2v* bp = reinterpret_cast<const f2v*>(iqf) + ((int64_t)ss * p.stride + nl + lane);
      const int lo = rel_bound(-p.hist - nl - lane), hi = rel_bound(p.n - nl - lane);
      constexpr int NPL = L / 64;
      f2v v[NPL];
#pragma unroll
      for (int j = 0; j < NPL; ++j) v[j] = (64 * j >= lo && 64 * j < hi) ? bp[64 * j] : f2v{0.f, 0.f};
#pragma unroll
      for (int j = 0; j < NPL; ++j) slot[64 * j + lane] = v[j];
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
        gload16_nt_v<1024 * (c % 4)>(stg[c], voff, gl + 4096 * (c / 4));
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
  if (stg1) load_stage(s1, n_lo_of(i1));

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
    fe_fir_tile<T, D, R, PF>(slot, lane, tp, ai, aq);
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
      carry = fe_epilogue<T, D, R>(p, s, M, m0, lane, ai, aq, si, sq, have, carry, d, !FUSED);
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
      if (stg1) {
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
          } else {
            asm volatile("" : "+v"(stg[c]));
            lds_write_b128_v<1024 * (HCH + c)>(na, stg[c]);
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
      if (stg1) load_stage(s1, n_lo_of(i1));
    }
    // queued behind the next tile's loads
    stores();
  }
}

// ------------------------------------------------------------------------------
// Host-side launchers (called by capi.hip)
// ------------------------------------------------------------------------------
static int cu_count() { return device_cus(); }

// Resident workgroups per CU for a kernel (the persistent grid must be fully resident
// for its tiles to be spread evenly; any excess would run as a second, serial round).
template <typename K>
static int resident_per_cu(K kernel, int threads) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, threads, 0) != hipSuccess || n <= 0) n = 1;
  return n;
}

static FeParams fe_params(const FeLaunch& a) {
  FeParams p{};
  p.iq = a.iq; p.n = a.n; p.stride = a.stride; p.hist = a.hist; p.nstreams = a.nstreams;
  p.taps_dev = a.taps_dev; p.zi_i = a.zi_i; p.zi_q = a.zi_q; p.zi_stride = a.zi_stride;
  p.prev_phase = a.prev_phase; p.demod = a.demod; p.out_stride = a.out_stride;
  p.i_ds = a.i_ds; p.q_ds = a.q_ds; p.last_phi = a.last_phi; p.wraps = a.wraps;
  p.vec_out = ((a.out_stride % 4) == 0 && ((uintptr_t)a.demod % 16) == 0) ? 1 : 0;
  return p;
}

// f32 IQ: fe_ring_kernel, 4 resident waves per CU, balanced tile ranges
template <int T, bool FUSED>
static hipError_t launch_ring_t(FeParams p, const TapsF32& taps, RingArgs ra, hipStream_t st) {
  if (ra.total <= 0) return hipSuccess;
  if (ra.total > 0x7fffffff) return hipErrorInvalidValue;
  static std::atomic<int> wpc_cache[kMaxDevices];     // per device (a process may drive several)
  const int wpc = per_device(wpc_cache, [] { return resident_per_cu(fe_ring_kernel<T, FUSED>, 64); });
  const int64_t slots = (int64_t)cu_count() * std::max(1, std::min(wpc, 4));
  const int64_t grid = std::min<int64_t>(slots, ra.total);
  p.tiles_per_stream = ra.tps;
  hipLaunchKernelGGL((fe_ring_kernel<T, FUSED>), dim3((unsigned)grid), dim3(64), 0, st, p, taps, ra);
  return hipGetLastError();
}

// u8 IQ: fe_slot_kernel, 8 resident waves per CU
template <int T, bool FUSED>
static hipError_t launch_slot_t(FeParams p, const TapsF32& taps, SlotArgs sa, hipStream_t st) {
  if (sa.total <= 0) return hipSuccess;
  if (sa.total > 0x7fffffff) return hipErrorInvalidValue;
  static std::atomic<int> wpc_cache[kMaxDevices];     // per device (a process may drive several)
  const int wpc = per_device(wpc_cache, [] { return resident_per_cu(fe_slot_kernel<T, FUSED, true>, 64); });
  const int64_t slots = (int64_t)cu_count() * std::max(1, std::min(wpc, 8));
  const int64_t grid = std::min<int64_t>(slots, sa.total);
  p.tiles_per_stream = sa.tps;
  hipLaunchKernelGGL((fe_slot_kernel<T, FUSED, true>), dim3((unsigned)grid), dim3(64), 0, st, p, taps, sa);
  return hipGetLastError();
}

template <int T>
static hipError_t launch_fe_t(const FeLaunch& a, hipStream_t st) {
  constexpr int D = 10, TO = 192;
  const FeParams p = fe_params(a);
  const int64_t M = (a.n + D - 1) / D;
  const int tps = (int)((M + TO - 1) / TO);
  if (a.u8) {
    SlotArgs sa{};
    sa.tps = tps;
    sa.total = (int64_t)tps * a.nstreams;
    return launch_slot_t<T, false>(p, *a.taps, sa, st);
  }
  RingArgs ra{};
  ra.tps = tps;
  ra.total = (int64_t)tps * a.nstreams;
  return launch_ring_t<T, false>(p, *a.taps, ra, st);
}

}  // namespace

// Returns hipErrorInvalidValue for an unsupported (taps, decim) pair; the C-ABI
// reports that as SDR_EUNSUPPORTED.  Supported: the reference's RF configs
// (151 taps: model/fmMonoBlock.py:24; 101 taps: BASELINE configs) at decim 10.
hipError_t sdr_launch_fe(const FeLaunch& a, hipStream_t st) {
  if (a.D != 10) return hipErrorInvalidValue;
  // u8 IQ: the RF FIR on the int8 matrix cores where it covers the call (fe_mfma.hip)
  // (hipErrorInvalidValue: a call it does not cover, which the vector kernels take; any other
  // error is a failed launch and is returned, not retried on a different arithmetic path)
  if (a.u8) {
    const hipError_t em = sdr_launch_fe_mfma(a, st);
    if (em != hipErrorInvalidValue) return em;
  }
  switch (a.T) {
    case 101: return launch_fe_t<101>(a, st);
    case 151: return launch_fe_t<151>(a, st);
    default: return hipErrorInvalidValue;
  }
}

// Fused FE + mono audio filter over whole streams (zero initial state).  Supported: RF
// taps 101 at decim 10 (f32 or u8 IQ), audio taps 151 at decim 5 (model/fmMonoBlock.py:24-31,
// BASELINE configs); anything else returns hipErrorInvalidValue and the C-ABI runs the
// two-kernel path.
hipError_t sdr_launch_fe_mono(const FeLaunch& a, const float* ataps, const float* ataps_rev, int TA, int DA,
                              float* audio, int64_t audio_stride, hipStream_t st) {
  if (a.D != 10 || TA != 151 || DA != 5 || a.T != 101) return hipErrorInvalidValue;
  constexpr int D = 10, BD = 960;                  // demod samples per audio block
  FeParams p = fe_params(a);
  p.hist = 0;
  const int64_t M = (a.n + D - 1) / D;
  const int ab = (int)((M + BD - 1) / BD);
  const int tps = 5 * ab;
  const int64_t total = (int64_t)tps * a.nstreams;
  if (total > 0x7fffffff) return hipErrorInvalidValue;
  if (a.u8) {
    const hipError_t em = sdr_launch_fe_mono_mfma(a, ataps_rev, TA, DA, audio, audio_stride, st);
    if (em != hipErrorInvalidValue) return em;
    SlotArgs sa{};
    sa.tps = tps; sa.total = total;
    sa.audio = audio; sa.audio_stride = audio_stride; sa.ataps = ataps;
    return launch_slot_t<101, true>(p, *a.taps, sa, st);
  }
  RingArgs ra{};
  ra.tps = tps; ra.total = total;
  ra.audio = audio; ra.audio_stride = audio_stride; ra.ataps = ataps;
  return launch_ring_t<101, true>(p, *a.taps, ra, st);
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
