// Spectral diagnostics: the Bartlett PSD estimate of
// model/fmSupportLib.py:66-140 (estimatePSD) and the direct DFT of :46-60, in f64.
//
//  * psd_seg_kernel: one 256-thread workgroup per segment.  The NFFT Hann-windowed
//    samples (window pow(sin(i*pi/N), 2), :80-82) go into LDS at bit-reversed positions
//    as complex f64, then log2(N) radix-2 butterfly stages run in LDS (twiddles from
//    sincospi of an exact binary fraction).  Bins 0..N/2-1 leave as
//    10*log10(2 * (1/(Fs*N/2)) * |X_k|^2) (:115-121), one row per segment.
//  * psd_avg_kernel: per bin, the segments' dB values summed in segment order and divided
//    by the segment count (:128-137).
//  * dft_kernel: one thread per bin m, X_m = sum_k x_k exp(i * (2*pi*(-k*m)/N)) with the
//    angle rounded as the reference's expression rounds it (:57).
// The PSD reads each sample once and the work is tiny (a diagnostic, off the hot path).
#include <hip/hip_runtime.h>
#include <cstdint>
#include "sdr_common.h"

namespace {

constexpr double kPiD = 3.14159265358979323846;
constexpr int kPsdThreads = 256;

template <typename TX>
__global__ __launch_bounds__(kPsdThreads) void psd_seg_kernel(const TX* x, int logn, double fs,
                                                               double* seg_db, int* zero_flag) {
  __shared__ double2 X[SDR_PSD_MAX_NFFT];
  const int N = 1 << logn;
  const int seg = blockIdx.x;
  const TX* xs = x + (int64_t)seg * N;
  for (int i = threadIdx.x; i < N; i += kPsdThreads) {
    const double s = sin((double)i * kPiD / (double)N);
    const double v = (double)xs[i] * (s * s);
    const int r = (int)(__builtin_bitreverse32((unsigned)i) >> (32 - logn));
    X[r] = make_double2(v, 0.0);
  }
  __syncthreads();
  for (int st = 1; st <= logn; ++st) {
    const int half = 1 << (st - 1);
    for (int j = threadIdx.x; j < N / 2; j += kPsdThreads) {
      const int k = j & (half - 1);
      const int i0 = ((j >> (st - 1)) << st) + k;
      const int i1 = i0 + half;
      double sn, cs;
      sincospi(-(double)k / (double)half, &sn, &cs);   // exp(-2 pi i k / 2half)
      const double2 a = X[i0], b = X[i1];
      const double tr = cs * b.x - sn * b.y;
      const double ti = cs * b.y + sn * b.x;
      X[i0] = make_double2(a.x + tr, a.y + ti);
      X[i1] = make_double2(a.x - tr, a.y - ti);
    }
    __syncthreads();
  }
  const double c = 1.0 / (fs * (double)N / 2.0);
  for (int k = threadIdx.x; k < N / 2; k += kPsdThreads) {
    const double m = hypot(X[k].x, X[k].y);
    const double p = 2.0 * (c * (m * m));
    if (!(p > 0.0)) atomicOr(zero_flag, 1);   // the reference's math.log10 raises here
    seg_db[(int64_t)seg * (N / 2) + k] = 10.0 * log10(p);
  }
}

__global__ void psd_avg_kernel(const double* seg_db, int64_t nseg, int half, double* out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= half) return;
  double acc = 0.0;
  for (int64_t l = 0; l < nseg; ++l) acc += seg_db[k + l * half];
  out[k] = acc / (double)nseg;
}

__global__ void dft_kernel(const double* x, int64_t n, double* X) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= n) return;
  const double w = 2.0 * kPiD;
  double re = 0.0, im = 0.0;
  for (int64_t k = 0; k < n; ++k) {
    const double ang = w * (double)((-k) * m) / (double)n;
    double sn, cs;
    sincos(ang, &sn, &cs);
    re += x[k] * cs;
    im += x[k] * sn;
  }
  X[2 * m] = re;
  X[2 * m + 1] = im;
}

}  // namespace

hipError_t sdr_launch_psd(const void* x, int f64, int64_t n, int logn, double fs, double* seg_db,
                          double* out, int* zero_flag, hipStream_t st) {
  const int N = 1 << logn;
  const int64_t nseg = n / N;
  const int half = N / 2;
  if (nseg > 0x7fffffff) return hipErrorInvalidValue;
  if (nseg > 0) {
    if (f64)
      hipLaunchKernelGGL(psd_seg_kernel<double>, dim3((unsigned)nseg), dim3(kPsdThreads), 0, st,
                         (const double*)x, logn, fs, seg_db, zero_flag);
    else
      hipLaunchKernelGGL(psd_seg_kernel<float>, dim3((unsigned)nseg), dim3(kPsdThreads), 0, st,
                         (const float*)x, logn, fs, seg_db, zero_flag);
  }
  hipLaunchKernelGGL(psd_avg_kernel, dim3((half + 255) / 256), dim3(256), 0, st, seg_db, nseg, half, out);
  return hipGetLastError();
}

hipError_t sdr_launch_dft(const double* x, int64_t n, double* X, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(dft_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n, X);
  return hipGetLastError();
}
