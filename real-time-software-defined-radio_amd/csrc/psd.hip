// Spectral diagnostics: the Bartlett PSD estimate of
// model/fmSupportLib.py:66-140 (estimatePSD) and the direct DFT of :46-60, in f64.
//
//  * psd_seg_kernel: one 256-thread workgroup per segment.  The NFFT Hann-windowed
//    samples (window pow(sin(i*pi/N), 2), :80-82) go into LDS at bit-reversed positions
//    as complex f64, then log2(N) radix-2 butterfly stages run in LDS (twiddles from
//    sincospi of an exact binary fraction).  Bins 0..N/2-1 leave as
//    10*log10(2 * (1/(Fs*N/2)) * |X_k|^2) (:115-121), one row per segment.
//  * psd_sum_kernel (twice): per bin, the segments' dB values summed (in segment order
//    within chunks of 64 segments, then over the chunks) and divided by the segment count
//    (:128-137; the reference sums in one sequential pass, so the f64 rounding of the
//    average may differ in the last bits).
//  * dft_kernel: one thread per bin m, X_m = sum_k x_k exp(i * (2*pi*(-k*m)/N)) with the
//    angle rounded as the reference's expression rounds it (:57).
// The PSD reads each sample once and the work is tiny (a diagnostic, off the hot path).
#include <hip/hip_runtime.h>
#include <cstdint>
#include "sdr_launch.h"

namespace {

constexpr double kPiD = 3.14159265358979323846;
constexpr int kPsdThreads = 256;
constexpr int kPsdChunk = 64;        // segments per first-pass partial sum
__host__ __device__ constexpr bool psd_table(int N) { return N + N / 2 <= SDR_PSD_MAX_NFFT; }

template <typename TX>
__global__ __launch_bounds__(kPsdThreads) void psd_seg_kernel(const TX* x, int logn, double fs,
                                                               double* seg_db, int* zero_flag) {
  extern __shared__ double2 X[];       // N entries (+ N/2 twiddles when N <= 2048), sized at launch
  const int N = 1 << logn;
  const int seg = blockIdx.x;
  const TX* xs = x + (int64_t)seg * N;
  for (int i = threadIdx.x; i < N; i += kPsdThreads) {
    const double s = sin((double)i * kPiD / (double)N);
    const double v = (double)xs[i] * (s * s);
    const int r = (int)(__builtin_bitreverse32((unsigned)i) >> (32 - logn));
    X[r] = make_double2(v, 0.0);
  }
  // twiddles exp(-2 pi i j / N), j < N/2, once per workgroup in the free tail of X when it
  // fits (N <= 2048); stage `half` uses entry k * N / (2 half) -- the same sincospi argument
  // -k/half exactly, so the same values as computing them per butterfly (N = 4096 does)
  const bool table = psd_table(N);
  double2* tw = X + N;
  if (table)
    for (int j = threadIdx.x; j < N / 2; j += kPsdThreads) {
      double sn, cs;
      sincospi(-2.0 * (double)j / (double)N, &sn, &cs);
      tw[j] = make_double2(cs, sn);
    }
  __syncthreads();
  for (int st = 1; st <= logn; ++st) {
    const int half = 1 << (st - 1);
    for (int j = threadIdx.x; j < N / 2; j += kPsdThreads) {
      const int k = j & (half - 1);
      const int i0 = ((j >> (st - 1)) << st) + k;
      const int i1 = i0 + half;
      double sn, cs;
      if (table) {
        const double2 w = tw[k << (logn - st)];
        cs = w.x;
        sn = w.y;
      } else {
        sincospi(-(double)k / (double)half, &sn, &cs);   // exp(-2 pi i k / 2half)
      }
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

// Per bin k: sum of rows [c*rpc, min((c+1)*rpc, nrows)) of a row-major [nrows x half]
// matrix, in row order, into out[c*half + k]; divided by `div` if `divide`.  Two passes
// (chunks of 64 segments, then the chunk sums) keep ~64 independent loads in flight per
// thread; a single serial pass over 4 687 segments waited a memory round trip per add.
__global__ void psd_sum_kernel(const double* in, int64_t nrows, int half, int rpc, int divide, double div,
                               double* out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  if (k >= half) return;
  const int64_t r0 = (int64_t)c * rpc;
  const int64_t r1 = min<int64_t>(r0 + rpc, nrows);
  double acc = 0.0;
#pragma unroll 16
  for (int64_t r = r0; r < r1; ++r) acc += in[r * half + k];
  out[(int64_t)c * half + k] = divide ? acc / div : acc;
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

int sdr_psd_chunks(int64_t nseg) { return (int)((nseg + kPsdChunk - 1) / kPsdChunk); }

// seg_db: nseg x N/2 doubles; part: sdr_psd_chunks(nseg) x N/2 doubles
hipError_t sdr_launch_psd(const void* x, int f64, int64_t n, int logn, double fs, double* seg_db,
                          double* part, double* out, int* zero_flag, hipStream_t st) {
  const int N = 1 << logn;
  const int64_t nseg = n / N;
  const int half = N / 2;
  if (nseg > 0x7fffffff) return hipErrorInvalidValue;
  const dim3 bins((half + 255) / 256);
  if (nseg == 0) {                     // the reference's 0/0: NaN in every bin
    hipLaunchKernelGGL(psd_sum_kernel, dim3(bins.x, 1), dim3(256), 0, st, seg_db, (int64_t)0, half, 1, 1, 0.0,
                       out);
    return hipGetLastError();
  }
  // LDS sized to the segment (not to the 4096 maximum), so small NFFT runs many
  // workgroups per CU
  const size_t lds = sizeof(double2) * (size_t)(N + (psd_table(N) ? N / 2 : 0));
  if (f64)
    hipLaunchKernelGGL(psd_seg_kernel<double>, dim3((unsigned)nseg), dim3(kPsdThreads), lds, st,
                       (const double*)x, logn, fs, seg_db, zero_flag);
  else
    hipLaunchKernelGGL(psd_seg_kernel<float>, dim3((unsigned)nseg), dim3(kPsdThreads), lds, st,
                       (const float*)x, logn, fs, seg_db, zero_flag);
  const int nch = sdr_psd_chunks(nseg);
  hipLaunchKernelGGL(psd_sum_kernel, dim3(bins.x, nch), dim3(256), 0, st, seg_db, nseg, half, kPsdChunk, 0, 0.0,
                     part);
  hipLaunchKernelGGL(psd_sum_kernel, dim3(bins.x, 1), dim3(256), 0, st, part, (int64_t)nch, half, nch, 1,
                     (double)nseg, out);
  return hipGetLastError();
}

hipError_t sdr_launch_dft(const double* x, int64_t n, double* X, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(dft_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n, X);
  return hipGetLastError();
}
