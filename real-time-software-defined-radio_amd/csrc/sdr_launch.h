// Internal launcher interface between the C-ABI (capi.hip) and the kernel translation
// units (fe.hip, fir.hip, pll.hip, psd.hip).  One definition of every struct that crosses a
// translation-unit boundary: each .hip file includes this header, so a field change is a
// compile error everywhere instead of a silent ODR mismatch.
#pragma once
#include <atomic>
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sdr_common.h"

// Launch geometry that depends on the device, cached per device (a process may hold contexts
// on GPUs with different CU counts, from several threads): `query` runs for the current
// device the first time, and every thread that races it there stores the same value.
constexpr int kMaxDevices = 64;
template <class Q>
inline int per_device(std::atomic<int> (&cache)[kMaxDevices], Q query) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return query();
  int v = cache[dev].load(std::memory_order_relaxed);
  if (v == 0) {
    v = query();
    cache[dev].store(v, std::memory_order_relaxed);
  }
  return v;
}
// the current device's compute units (256 if the query fails)
inline int device_cus() {
  static std::atomic<int> cache[kMaxDevices];
  return per_device(cache, [] {
    int dev = 0, n = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) n = prop.multiProcessorCount;
    return n > 0 ? n : 256;
  });
}

// RF front end (fe.hip): interleaved IQ -> FIR + decimate -> atan2 discriminator.
struct FeLaunch {
  const void* iq; int64_t n; int64_t stride; int64_t hist; int nstreams;
  const float* taps_dev; const TapsF32* taps; int T; int D; int u8;
  const double* zi_i; const double* zi_q; int64_t zi_stride; const double* prev_phase;
  float* demod; int64_t out_stride; float* i_ds; float* q_ds; float* last_phi; int* wraps;
  const int* afr;   // nullable: the taps' MFMA A fragments (TapSet::dev_afr; else built in-kernel)
};

// Real-channel FIR with decimation (fir.hip); `pre` selects a fused pre-op on the input
// (0 none, 1 x^2, 2 x*c*gain mixer).
struct FirLaunch {
  const float* x; const float* c; float gain; int pre; int64_t n; int64_t x_stride; int64_t x_step;
  int64_t hist; int nstreams; const float* taps_dev; const TapsF32* taps; int T; int D;
  const double* zi; int64_t zi_stride; float* y; int64_t y_stride;
};

// fmPll constants (pll.hip): model/fmPll.py:4-10
struct PllCfg { double freq, fs, scale, adj, kp, ki; };

hipError_t sdr_launch_fe(const FeLaunch& a, hipStream_t st);
// ataps / ataps_rev: the audio taps forward and reversed (TapSet::dev_f32 / dev_rev)
hipError_t sdr_launch_fe_mono(const FeLaunch& a, const float* ataps, const float* ataps_rev, int TA, int DA,
                              float* audio, int64_t audio_stride, hipStream_t st);
// u8 FE + mono with the RF FIR on the int8 matrix cores (fe_mfma.hip); hipErrorInvalidValue
// when the configuration is not the one it covers
// u8 FE (FIR + decimate + demod with carried state) on the int8 matrix cores (fe_mfma.hip):
// 101 / 151 taps; hipErrorInvalidValue when the configuration is not one it covers
hipError_t sdr_launch_fe_mfma(const FeLaunch& a, hipStream_t st);
// the u8 MFMA front end's A fragments of RF taps h (T = 101 or 151, decim 10), as the kernels
// would build them: ints in [ks][digit][lane][4] order; false for other T
bool sdr_mfma_fragments(const float* h, int T, std::vector<int>* out);
hipError_t sdr_launch_fe_mono_mfma(const FeLaunch& a, const float* ataps_rev, int TA, int DA, float* audio,
                                   int64_t audio_stride, hipStream_t st);
hipError_t sdr_launch_iq_zf(const void* iq, int u8, int64_t n, int64_t stride, int nstreams,
                            const double* b_dev, int T, const double* zi_i, const double* zi_q,
                            int64_t zi_stride, double* zf_i, double* zf_q, hipStream_t st);
hipError_t sdr_launch_demod(const float* I, const float* Q, int64_t n, int64_t stride, int nstreams,
                            const double* prev_phase, float* out, int64_t out_stride,
                            float* last_phi, int* wraps, hipStream_t st);
hipError_t sdr_launch_demod_state(int nstreams, int64_t m, const float* last_phi, const int* wraps,
                                  double* prev_phase, hipStream_t st);
hipError_t sdr_launch_fir(const FirLaunch& a, hipStream_t st);
hipError_t sdr_launch_resample(const float* x, int64_t n, const float* taps_dev, int T, int U, int D,
                               const double* zi, float* y, hipStream_t st);
hipError_t sdr_launch_zf(const float* x, const float* c, float gain, int pre, int64_t n,
                         int64_t x_stride, int nstreams, int U, const double* b_dev, int T,
                         const double* zi, int64_t zi_stride, double* zf, hipStream_t st);
hipError_t sdr_launch_combine(const float* mono, const float* side, int64_t n, float* left,
                              float* right, hipStream_t st);
int sdr_psd_chunks(int64_t nseg);
hipError_t sdr_launch_psd(const void* x, int f64, int64_t n, int logn, double fs, double* seg_db,
                          double* part, double* out, int* zero_flag, hipStream_t st);
hipError_t sdr_launch_dft(const double* x, int64_t n, double* X, hipStream_t st);
// PLL job table (pll.hip): one lane per (job, stream) recurrence.  Per stream: state 6
// doubles (stride 6), in[n] (in_stride), nco_i / nco_q (optional) n+1 floats (out_stride),
// and two f64 scratch rows: theta (th_stride >= n+1: the phase estimates, then the call's
// trigOffset) and cbuf (c_stride >= n + n/32: per-sample loop constants, then group flags).
#define SDR_PLL_MAXJ 4
struct PllJob {
  const float* in; int64_t in_stride; double* state; double* theta; int64_t th_stride;
  float* nco_i; float* nco_q; int64_t out_stride; PllCfg cfg; double* cbuf; int64_t c_stride;
  double off; int off_given;   // the prep kernel's trigOffset, when not read from state[5]
  const double* resp;          // long calls: the loop's response table (sdr_pll_resp_table), device
  const double* qtab;          // the solve's matrix powers (pll.hip qtab_host); set by the launcher
  const int8_t* in8;           // nullable: the input as sign codes (sdr_nco.h pll_code), in8_stride bytes
  int64_t in8_stride;          //   apart per stream; read instead of `in` (long calls, spec-only calls)
  int th32;                    // long calls: the phase rows in the compact form (sdr_nco.h "compact
                               //   phase rows"); set by the receiver for the pilot loop of a span
};
// Long calls (n > SDR_PLL_BLOCK_MAX samples): the recurrence is cut into nb pseudo-blocks of
// pb samples, solved in parallel from warm-up guesses of their start states and chained
// (pll.hip, "long calls").  Per job: the warm-up length, the loop matrix's power over a
// pseudo-block (phi: the start-state error -> end-state error map, for the pb-sample blocks
// and for the last one) and the bounds c1, c2 on the phase excursion a unit start error in
// (phaseEst, integrator) causes.  Filled by the launcher.
#define SDR_PLL_BLOCK_MAX 16385
struct PllLong {
  int64_t pb; int nb; int warm[SDR_PLL_MAXJ];
  double phi[SDR_PLL_MAXJ][4], phi_last[SDR_PLL_MAXJ][4], c1[SDR_PLL_MAXJ], c2[SDR_PLL_MAXJ];
};
struct PllJobs {
  PllJob j[SDR_PLL_MAXJ]; int njobs; int nstreams; int64_t n;
  int lpw; int qform;                  // set by the launchers
  int nco_fused;                       // per-block spec-only calls: the solve's launch writes the NCO rows
  int nco_rows;                        // 0: write only each NCO row's [0] (the carried value) and leave the
                                       //   rest to the consumer (the receiver's mixers, sdr_nco.h); 1: whole rows
  unsigned long long* stats;           // device counters (SDR_PLL_NSTATS, include/sdr.h), nullable
  void* work;                          // long calls: sdr_pll_work_bytes() of device scratch
  PllLong lg;                          // long calls: set by the launcher
};
// device scratch a long call needs (0 when n <= SDR_PLL_BLOCK_MAX)
int64_t sdr_pll_work_bytes(int njobs, int nstreams, int64_t n);
// a long call of n steps: its pseudo-block length and count (false: not a long call)
bool sdr_pll_long_geom(int64_t n, int64_t* pb, int* nb);
// the loop's response table for a long call of n steps: 2 (pb + 1) doubles, row 0 of A^j for
// j = 0 .. pb (sdr_nco.h); empty when n is not a long call
void sdr_pll_resp_table(const PllCfg& c, int64_t n, std::vector<double>* out);
// prep (per-sample constants) -> loop (one lane per recurrence) -> NCO; the three launches
// separately (the receiver puts them on different streams) or together
hipError_t sdr_launch_pll_prep(const PllJobs& jobs, hipStream_t st);
hipError_t sdr_launch_pll_loop(const PllJobs& jobs, hipStream_t st);
hipError_t sdr_launch_pll_nco(const PllJobs& jobs, hipStream_t st);
hipError_t sdr_launch_pll_jobs(const PllJobs& jobs, hipStream_t st);
