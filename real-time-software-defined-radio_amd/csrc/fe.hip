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

template <int T, int D, int R, int NT, bool U8>
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
  if (n_lo >= -p.hist && n_lo + L <= p.n) {
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
  for (int i = 0; i < NI; ++i) {
    const float2 x = win[i + i / DR];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = D * r + T - 1 - i;             // tap index (compile time)
      if (k >= 0 && k < T) {
        ai[r] = fmaf(taps.h[k], x.x, ai[r]);
        aq[r] = fmaf(taps.h[k], x.y, aq[r]);
      }
    }
  }

  const int64_t mf = m0 + (int64_t)t * R;          // first output of this thread
  const int64_t zoff = (int64_t)s * p.zi_stride;
  float phi[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t nn = D * (mf + r);
    if (p.zi_i != nullptr && nn < T - 1) {
      ai[r] += (float)p.zi_i[zoff + nn];
      aq[r] += (float)p.zi_q[zoff + nn];
    }
    phi[r] = atan2f(aq[r], ai[r]);
  }

  // ---- 3. predecessor phase for lane 0 of each wave --------------------------
  const int lane = t & 63;
  const int w = t >> 6;
  const int64_t mw = m0 + (int64_t)w * 64 * R;
  float phi_wprev = 0.f;
  if (mw > 0) {
    float si = 0.f, sq = 0.f;
    for (int k = lane; k < T; k += 64) {
      const int e = D * w * 64 * R + (T - 1) + DELTA - k;
      const float2 x = lds[slot(e)];
      const float h = p.taps_dev[k];
      si = fmaf(h, x.x, si);
      sq = fmaf(h, x.y, sq);
    }
    si = wave_sum(si);
    sq = wave_sum(sq);
    const int64_t nn = D * (mw - 1);
    if (p.zi_i != nullptr && nn < T - 1) {
      si += (float)p.zi_i[zoff + nn];
      sq += (float)p.zi_q[zoff + nn];
    }
    phi_wprev = atan2f(sq, si);
  }
  const float from_left = __shfl_up(phi[R - 1], 1, 64);
  float prev = (lane == 0) ? phi_wprev : from_left;

  // ---- 4. discriminator with np.unwrap semantics ------------------------------
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

  // ---- 5. stores ---------------------------------------------------------------
  if (s < p.nstreams) {
    float* out = p.demod + (int64_t)s * p.out_stride;
    if (R == 4 && p.vec_out && mf + R <= M) {
      *reinterpret_cast<float4*>(out + mf) = make_float4(d[0], d[1 % R], d[2 % R], d[3 % R]);
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
  }
}

// lfilter final state zf for the I and Q channels of an interleaved IQ block
// (scipy _signaltools.py:2153-2172), computed in f64:
//   zf[k] = sum_{j=k+1}^{T-1} b[j] * x[N-1-(j-k-1)]  +  (N+k < T-1 ? zi[N+k] : 0)
template <bool U8>
__global__ void iq_zf_kernel(const void* iq_all, int64_t n, int64_t stride, const double* b, int T,
                             const double* zi_i, const double* zi_q, int64_t zi_stride,
                             double* zf_i, double* zf_q) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= T - 1) return;
  const int s = blockIdx.y;
  const void* iq = reinterpret_cast<const char*>(iq_all) + (int64_t)s * stride * (U8 ? 2 : 8);
  if (zi_i != nullptr) { zi_i += (int64_t)s * zi_stride; zi_q += (int64_t)s * zi_stride; }
  zf_i += (int64_t)s * zi_stride;
  zf_q += (int64_t)s * zi_stride;
  double si = 0.0, sq = 0.0;
  for (int j = k + 1; j < T; ++j) {
    const int64_t idx = n - 1 - (j - k - 1);
    if (idx < 0) break;
    float2 x = IqLoad<U8>::load1(iq, idx);
    si = fma(b[j], (double)x.x, si);
    sq = fma(b[j], (double)x.y, sq);
  }
  if (n + k < T - 1 && zi_i != nullptr) {
    si += zi_i[n + k];
    sq += zi_q[n + k];
  }
  zf_i[k] = si;
  zf_q[k] = sq;
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

template <int T, int D, bool U8>
static hipError_t launch_fe_t(const FeLaunch& a, hipStream_t st) {
  constexpr int NT = 128, R = 4, TO = NT * R;
  FeParams p;
  p.iq = a.iq; p.n = a.n; p.stride = a.stride; p.hist = a.hist; p.nstreams = a.nstreams;
  const int64_t M = (a.n + D - 1) / D;
  p.tiles_per_stream = (int)((M + TO - 1) / TO);
  p.taps_dev = a.taps_dev; p.zi_i = a.zi_i; p.zi_q = a.zi_q; p.zi_stride = a.zi_stride;
  p.prev_phase = a.prev_phase; p.demod = a.demod; p.out_stride = a.out_stride;
  p.i_ds = a.i_ds; p.q_ds = a.q_ds; p.last_phi = a.last_phi; p.wraps = a.wraps;
  p.vec_out = ((a.out_stride % 4) == 0 && ((uintptr_t)a.demod % 16) == 0) ? 1 : 0;
  const int64_t blocks = (int64_t)p.tiles_per_stream * a.nstreams;
  if (blocks <= 0) return hipSuccess;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL((fe_kernel<T, D, R, NT, U8>), dim3((unsigned)blocks), dim3(NT), 0, st,
                     p, *a.taps);
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

hipError_t sdr_launch_iq_zf(const void* iq, int u8, int64_t n, int64_t stride, int nstreams,
                            const double* b_dev, int T, const double* zi_i, const double* zi_q,
                            int64_t zi_stride, double* zf_i, double* zf_q, hipStream_t st) {
  if (T <= 1 || nstreams <= 0) return hipSuccess;
  const dim3 grid((T - 1 + 255) / 256, nstreams);
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
