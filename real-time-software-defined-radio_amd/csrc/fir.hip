// Real-valued FIR family for gfx950: lfilter-compatible FIR with decimation and
// fused input pre-ops, the polyphase rational resampler, and f64 state kernels.
//
// Replaces:
//   model/fmMonoBlock.py:101-105   audio lfilter(zi) + [::5]            (D=5, PRE_NONE)
//   model/fmMonoBlock.py:117,151   stereo BPFs (D=1)
//   model/fmMonoBlock.py:155-162   mixer x2 + stereo LPF + [::5]        (PRE_MIX)
//   model/fmRDSblock.py:156-164    RDS BPF, square, BPF                 (PRE_SQUARE)
//   model/fmRDSblock.py:173-182    I/Q mixer x2 + 3 kHz LPF             (PRE_MIX)
//   model/fmRDSblock.py:184-199    zero-stuff x19, anti-image LPF, [::80]*19 (resampler)
//   model/fmRDSblock.py:202-204    RRC filter                            (D=1)
//   src/filter.cpp:96-185, 301-401 convolveFIR / convolveWithDecim* / Mixer / Mode1RDS
//
// Tiled kernel: thread t owns R consecutive outputs and slides once over its
// D(R-1)+T input window in LDS (one ds_read_b32 feeds up to R FMAs; taps are
// compile-time indices -> SGPR operands).  LDS rows are padded by one float every
// D*R samples so the per-lane stride D*R+1 is odd -> conflict-free ds_read_b32.
#include "sdr_launch.h"

enum { PRE_NONE = 0, PRE_SQUARE = 1, PRE_MIX = 2 };

struct FirParams {
  const float* x;        // input, per stream `x_stride` apart
  const float* c;        // PRE_MIX second operand (same indexing as x), else null
  float gain;            // PRE_MIX gain (reference: *2)
  int64_t n;             // input samples per stream
  int64_t x_stride;
  int64_t x_step;        // element step (generic kernel only; tiled kernel needs 1)
  int64_t hist;          // valid samples before index 0
  int nstreams;
  int tiles_per_stream;
  const double* zi;      // nullable: per stream (T-1) lfilter state
  int64_t zi_stride;
  float* y;              // per stream ceil(n/D) outputs
  int64_t y_stride;
  int vec_in;            // x (and c) 16-B aligned with stride % 4 == 0
  int vec_out;           // y 16-B aligned with stride % 4 == 0
};

template <int PRE>
__device__ __forceinline__ float pre_op(float x, float c, float g) {
  if (PRE == PRE_SQUARE) return x * x;
  if (PRE == PRE_MIX) return (x * c) * g;
  return x;
}

template <int T, int D, int R, int NT, int PRE>
__global__ __launch_bounds__(NT) void fir_kernel(FirParams p, TapsF32 taps) {
  constexpr int G = 4;
  constexpr int TO = NT * R;
  constexpr int DR = D * R;
  constexpr bool PAD = (DR % 2) == 0;
  constexpr int SR = PAD ? DR + 1 : DR;
  constexpr int DELTA = (G - ((T - 1) % G)) % G;
  constexpr int L = ((D * (TO - 1) + T + DELTA) + G - 1) / G * G;
  constexpr int NSLOT = PAD ? L + (L + DR - DELTA) / DR + 1 : L;
  constexpr int NCHUNK = L / G;
  constexpr int NLOAD = (NCHUNK + NT - 1) / NT;
  constexpr int NI = D * (R - 1) + T;
  static_assert((D * TO) % G == 0, "tile start must stay G-aligned");

  __shared__ float lds[NSLOT];

  const int t = threadIdx.x;
  const int64_t blk = xcd_tile(blockIdx.x, gridDim.x);
  const int s = (int)(blk / p.tiles_per_stream);
  const int64_t m0 = (blk - (int64_t)s * p.tiles_per_stream) * TO;
  const int64_t M = (p.n + D - 1) / D;
  const int64_t n_lo = D * m0 - (T - 1) - DELTA;
  const float* xb = p.x + (int64_t)s * p.x_stride;
  const float* cb = (PRE == PRE_MIX) ? p.c + (int64_t)s * p.x_stride : nullptr;

  auto slot = [](int e) { return PAD ? e + (e + DR - DELTA) / DR : e; };
  if (p.vec_in && n_lo >= -p.hist && n_lo + L <= p.n) {
    float4 v[NLOAD];
    float4 cv[NLOAD];
#pragma unroll
    for (int j = 0; j < NLOAD; ++j) {
      const int q = t + j * NT;
      if (q < NCHUNK) {
        v[j] = reinterpret_cast<const float4*>(xb)[(n_lo >> 2) + q];
        if (PRE == PRE_MIX) cv[j] = reinterpret_cast<const float4*>(cb)[(n_lo >> 2) + q];
      }
    }
#pragma unroll
    for (int j = 0; j < NLOAD; ++j) {
      const int q = t + j * NT;
      if (q < NCHUNK) {
        const int e = q * G;
        lds[slot(e + 0)] = pre_op<PRE>(v[j].x, cv[j].x, p.gain);
        lds[slot(e + 1)] = pre_op<PRE>(v[j].y, cv[j].y, p.gain);
        lds[slot(e + 2)] = pre_op<PRE>(v[j].z, cv[j].z, p.gain);
        lds[slot(e + 3)] = pre_op<PRE>(v[j].w, cv[j].w, p.gain);
      }
    }
  } else {
    for (int e = t; e < L; e += NT) {
      const int64_t nn = n_lo + e;
      float x = 0.f;
      if (nn >= -p.hist && nn < p.n)
        x = pre_op<PRE>(xb[nn], PRE == PRE_MIX ? cb[nn] : 0.f, p.gain);
      lds[slot(e)] = x;
    }
  }
  __syncthreads();

  const float* win = lds + (PAD ? (DELTA + 1 + SR * t) : (DELTA + DR * t));
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const float x = win[PAD ? i + i / DR : i];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k = D * r + T - 1 - i;
      if (k >= 0 && k < T) acc[r] = fmaf(taps.h[k], x, acc[r]);
    }
  }

  const int64_t mf = m0 + (int64_t)t * R;
  if (p.zi != nullptr) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t nn = D * (mf + r);
      if (nn < T - 1) acc[r] += (float)p.zi[(int64_t)s * p.zi_stride + nn];
    }
  }
  float* yb = p.y + (int64_t)s * p.y_stride;
  if (R == 4 && p.vec_out && mf + R <= M) {
    *reinterpret_cast<float4*>(yb + mf) = make_float4(acc[0], acc[1 % R], acc[2 % R], acc[3 % R]);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (mf + r < M) yb[mf + r] = acc[r];
  }
}

// Generic fallback for tap counts without a compiled tile shape (any T <= 256,
// any D): one output per thread, taps staged in LDS, input through L1/L2.
template <int PRE>
__global__ __launch_bounds__(256) void fir_generic_kernel(FirParams p, const float* taps, int T, int D) {
  __shared__ float h[SDR_MAX_TAPS];
  for (int k = threadIdx.x; k < T; k += blockDim.x) h[k] = taps[k];
  __syncthreads();
  const int64_t M = (p.n + D - 1) / D;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int s = (int)(gid / M);
  if (s >= p.nstreams) return;
  const int64_t m = gid - (int64_t)s * M;
  const float* xb = p.x + (int64_t)s * p.x_stride;
  const float* cb = (PRE == PRE_MIX) ? p.c + (int64_t)s * p.x_stride : nullptr;
  float acc = 0.f;
  for (int k = T - 1; k >= 0; --k) {
    const int64_t nn = D * m - k;
    if (nn >= -p.hist && nn < p.n)
      acc = fmaf(h[k], pre_op<PRE>(xb[nn * p.x_step], PRE == PRE_MIX ? cb[nn * p.x_step] : 0.f, p.gain), acc);
  }
  if (p.zi != nullptr && D * m < T - 1) acc += (float)p.zi[(int64_t)s * p.zi_stride + D * m];
  p.y[(int64_t)s * p.y_stride + m] = acc;
}

// Rational resampler of model/fmRDSblock.py:184-199 without materialising the
// zero-stuffed stream: u[j] = x[j/U] if j % U == 0 else 0,
//   r[m] = U * ( sum_k h[k] u[D m - k]  +  (D m < T-1 ? zi[D m] : 0) ),
// only taps with (D m - k) % U == 0 contribute (~T/U per output).
// Taps (T <= SDR_MAX_RESAMPLE_TAPS) staged in dynamic LDS.  Output m reads the zero-stuffed
// stream at j0 = D*m: the nonzero terms are k = j0 mod U, +U, ... with input index
// (j0 - k)/U walking down by one, so one division per output, none per term.
__global__ __launch_bounds__(256) void resample_kernel(const float* x, int64_t n, const float* taps,
                                                       int T, int U, int D, const double* zi,
                                                       float* y) {
  extern __shared__ float h[];
  for (int k = threadIdx.x; k < T; k += blockDim.x) h[k] = taps[k];
  __syncthreads();
  const int64_t nu = n * U;
  const int64_t M = (nu + D - 1) / D;
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  const int64_t j0 = D * m;
  const int k0 = (int)(j0 % U);
  const int khi = (int)min<int64_t>(T - 1, j0);      // terms with j0 - k >= 0
  int64_t xi = (j0 - k0) / U;
  float acc = 0.f;
  for (int k = k0; k <= khi; k += U, --xi) acc = fmaf(h[k], x[xi], acc);
  if (zi != nullptr && j0 < T - 1) acc += (float)zi[j0];
  y[m] = acc * (float)U;
}

// lfilter final state (f64) for a real stream after an optional pre-op and an
// optional zero-stuffing factor U (U = 1: plain stream):
//   zf[k] = sum_{j=k+1}^{T-1} b[j] u[NU+k-j] + (NU+k < T-1 ? zi[NU+k] : 0),  NU = n*U.
// Blocks of 256 outputs per stream (T <= SDR_MAX_RESAMPLE_TAPS): the <= T-1 newest inputs
// (pre-op applied) and the taps are staged in dynamic LDS first, so each output's f64 dot
// product runs from LDS instead of waiting a global-memory round trip per term.
__global__ __launch_bounds__(256) void zf_kernel(const float* x, const float* c, float gain, int pre,
                                                 int64_t n, int64_t x_stride, int U, const double* b,
                                                 int T, const double* zi, int64_t zi_stride, double* zf) {
  extern __shared__ double zsh[];
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  x += (int64_t)s * x_stride;
  if (c != nullptr) c += (int64_t)s * x_stride;
  if (zi != nullptr) zi += (int64_t)s * zi_stride;
  zf += (int64_t)s * zi_stride;
  const int64_t nu = n * U;
  // inputs used: x[n-L .. n-1], L = min(n, floor((T-1)/U)); us[i] = u(x[n-1-i])
  const int L = (int)min<int64_t>(n, (T - 1) / U);
  double* bs = zsh;
  double* us = zsh + T;
  for (int i = threadIdx.x; i < L; i += blockDim.x) {
    const int64_t xi = n - 1 - i;
    double v = (double)x[xi];
    if (pre == PRE_SQUARE) v = v * v;
    else if (pre == PRE_MIX) v = (double)((x[xi] * c[xi]) * gain);
    us[i] = v;
  }
  for (int i = threadIdx.x; i < T; i += blockDim.x) bs[i] = b[i];
  __syncthreads();
  if (k >= T - 1) return;
  // The terms with idx = nu + k - j >= 0 on the zero-stuffed grid (idx % U == 0): since
  // nu % U == 0 that is j = k (mod U), so j walks k+U, k+2U, ... up to min(T-1, nu+k) while
  // the input walks back from x[n-1] -- same terms, same ascending-j order, no divisions.
  const int jhi = (int)min<int64_t>(T - 1, nu + k);
  double acc = 0.0;
  int i = 0;
#pragma unroll 4
  for (int j = k + U; j <= jhi; j += U, ++i) acc = fma(bs[j], us[i], acc);
  if (zi != nullptr && nu + k < T - 1) acc += zi[nu + k];
  zf[k] = acc;
}

// ------------------------------------------------------------------------------

template <int T, int D, int PRE>
static hipError_t launch_fir_t(const FirLaunch& a, hipStream_t st) {
  constexpr int NT = 128, R = 4, TO = NT * R;
  FirParams p;
  p.x = a.x; p.c = a.c; p.gain = a.gain; p.n = a.n; p.x_stride = a.x_stride; p.x_step = 1;
  p.hist = a.hist;
  p.nstreams = a.nstreams; p.zi = a.zi; p.zi_stride = a.zi_stride; p.y = a.y; p.y_stride = a.y_stride;
  const int64_t M = (a.n + D - 1) / D;
  p.tiles_per_stream = (int)((M + TO - 1) / TO);
  p.vec_in = ((a.x_stride % 4) == 0 && ((uintptr_t)a.x % 16) == 0 &&
              (PRE != PRE_MIX || ((uintptr_t)a.c % 16) == 0)) ? 1 : 0;
  p.vec_out = ((a.y_stride % 4) == 0 && ((uintptr_t)a.y % 16) == 0) ? 1 : 0;
  const int64_t blocks = (int64_t)p.tiles_per_stream * a.nstreams;
  if (blocks <= 0) return hipSuccess;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL((fir_kernel<T, D, R, NT, PRE>), dim3((unsigned)blocks), dim3(NT), 0, st, p, *a.taps);
  return hipGetLastError();
}

template <int T, int D>
static hipError_t launch_fir_pre(const FirLaunch& a, hipStream_t st) {
  switch (a.pre) {
    case PRE_NONE: return launch_fir_t<T, D, PRE_NONE>(a, st);
    case PRE_SQUARE: return launch_fir_t<T, D, PRE_SQUARE>(a, st);
    case PRE_MIX: return launch_fir_t<T, D, PRE_MIX>(a, st);
  }
  return hipErrorInvalidValue;
}

template <int PRE>
static hipError_t launch_fir_generic(const FirLaunch& a, hipStream_t st) {
  FirParams p;
  p.x = a.x; p.c = a.c; p.gain = a.gain; p.n = a.n; p.x_stride = a.x_stride;
  p.x_step = a.x_step; p.hist = a.hist;
  p.nstreams = a.nstreams; p.zi = a.zi; p.zi_stride = a.zi_stride; p.y = a.y; p.y_stride = a.y_stride;
  p.tiles_per_stream = 0; p.vec_in = 0; p.vec_out = 0;
  const int64_t M = (a.n + a.D - 1) / a.D;
  const int64_t total = M * a.nstreams;
  if (total <= 0) return hipSuccess;
  const int64_t blocks = (total + 255) / 256;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fir_generic_kernel<PRE>, dim3((unsigned)blocks), dim3(256), 0, st, p, a.taps_dev, a.T, a.D);
  return hipGetLastError();
}

hipError_t sdr_launch_fir(const FirLaunch& a, hipStream_t st) {
  if (a.T < 1 || a.T > SDR_MAX_TAPS || a.D < 1 || a.pre < 0 || a.pre > 2) return hipErrorInvalidValue;
  if (a.x_step != 1) goto generic;
  if (a.T == 151) {
    if (a.D == 1) return launch_fir_pre<151, 1>(a, st);
    if (a.D == 5) return launch_fir_pre<151, 5>(a, st);
    if (a.D == 10) return launch_fir_pre<151, 10>(a, st);
  } else if (a.T == 101) {
    if (a.D == 1) return launch_fir_pre<101, 1>(a, st);
    if (a.D == 5) return launch_fir_pre<101, 5>(a, st);
    if (a.D == 10) return launch_fir_pre<101, 10>(a, st);
  }
generic:
  switch (a.pre) {
    case PRE_NONE: return launch_fir_generic<PRE_NONE>(a, st);
    case PRE_SQUARE: return launch_fir_generic<PRE_SQUARE>(a, st);
    default: return launch_fir_generic<PRE_MIX>(a, st);
  }
}

hipError_t sdr_launch_resample(const float* x, int64_t n, const float* taps_dev, int T, int U, int D,
                               const double* zi, float* y, hipStream_t st) {
  const int64_t M = (n * U + D - 1) / D;
  if (M <= 0) return hipSuccess;
  if (T > SDR_MAX_RESAMPLE_TAPS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(resample_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), sizeof(float) * T, st, x, n,
                     taps_dev, T, U, D, zi, y);
  return hipGetLastError();
}

hipError_t sdr_launch_zf(const float* x, const float* c, float gain, int pre, int64_t n,
                         int64_t x_stride, int nstreams, int U, const double* b_dev, int T,
                         const double* zi, int64_t zi_stride, double* zf, hipStream_t st) {
  if (T <= 1 || nstreams <= 0) return hipSuccess;
  if (T > SDR_MAX_RESAMPLE_TAPS) return hipErrorInvalidValue;
  const int64_t L = std::min<int64_t>(n, (T - 1) / U);
  hipLaunchKernelGGL(zf_kernel, dim3((T - 1 + 255) / 256, nstreams), dim3(256), sizeof(double) * (T + L), st, x, c, gain,
                     pre, n, x_stride, U, b_dev, T, zi, zi_stride, zf);
  return hipGetLastError();
}

// Stereo combiner (intended form of model/fmMonoBlock.py:166-170, as src/fm_radio.cpp:250-251):
// left = (mono + side) / 2, right = (mono - side) / 2.
__global__ void combine_kernel(const float* mono, const float* side, int64_t n, float* left,
                               float* right) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = mono[i], b = side[i];
  left[i] = (a + b) * 0.5f;
  right[i] = (a - b) * 0.5f;
}

hipError_t sdr_launch_combine(const float* mono, const float* side, int64_t n, float* left,
                              float* right, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, mono,
                     side, n, left, right);
  return hipGetLastError();
}
