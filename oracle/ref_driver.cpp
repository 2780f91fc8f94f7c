// ORACLE — test infrastructure only.  Thin driver (this repository's code) that runs
// the REFERENCE C++ front end compiled from its own sources where they lie
// (/root/reference/src/filter.cpp, rf_module.cpp; see oracle/Makefile target `ref`).
// It mirrors src/fm_radio.cpp:62-99 (rf_thread): deinterleave, convolveWithDecimIQ
// (src/filter.cpp:187-219), fmDemodArctan (src/rf_module.cpp:13-34), and zero the
// accumulating outputs between blocks (src/fm_radio.cpp:97-98).  Used only as a
// throughput baseline: its numerics diverge from the Python model.
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "filter.h"
#include "rf_module.h"

extern "C" void ref_fe_stream(const float* iq, int64_t n_complex, int64_t block, const float* taps,
                              int T, int D, float* demod_out) {
  std::vector<float> h(taps, taps + T), zi(T - 1, 0.f), zq(T - 1, 0.f), I(block), Q(block);
  std::vector<float> yi, yq, prev(2, 0.f);
  for (int64_t b0 = 0; b0 + block <= n_complex; b0 += block) {
    for (int64_t i = 0; i < block; ++i) {
      I[i] = iq[2 * (b0 + i)];
      Q[i] = iq[2 * (b0 + i) + 1];
    }
    std::fill(yi.begin(), yi.end(), 0.f);
    std::fill(yq.begin(), yq.end(), 0.f);
    convolveWithDecimIQ(yi, I, h, zi, yq, Q, zq, D);
    float* out = demod_out + b0 / D;
    fmDemodArctan(yi, yq, prev, out);
  }
}

extern "C" void ref_fe_streams(const float* iq, int64_t n_complex, int64_t stride, int nstreams,
                               int64_t block, const float* taps, int T, int D, float* demod_out,
                               int64_t out_stride, int nthreads) {
#pragma omp parallel for num_threads(nthreads) schedule(static, 1)
  for (int s = 0; s < nstreams; ++s)
    ref_fe_stream(iq + 2 * (int64_t)s * stride, n_complex, block, taps, T, D,
                  demod_out + (int64_t)s * out_stride);
}

// Mode-1 audio resampler of the reference, src/filter.cpp:222-259 (convolveWithDecimMode1),
// run block by block as src/fm_radio.cpp:228 runs it: the output vector zeroed between
// blocks (:305) and the reference's own raw-history zi carried (T-1 floats, zero at
// start).  y_out: nblocks x floor(block*up/decim) floats.  Used to pin sdr_resample's
// 24/125 path (tests/golden/make_mode1_golden.py).
extern "C" void ref_mode1_resample_blocks(const float* x, int64_t nblocks, int64_t block,
                                          const float* taps, int T, int decim, int up, float* y_out) {
  std::vector<float> h(taps, taps + T), zi(T - 1, 0.f), xb(block), y;
  const int64_t ny = block * up / decim;
  for (int64_t b = 0; b < nblocks; ++b) {
    std::copy(x + b * block, x + (b + 1) * block, xb.begin());
    std::fill(y.begin(), y.end(), 0.f);
    convolveWithDecimMode1(y, xb, h, zi, decim, up);
    std::copy(y.begin(), y.begin() + ny, y_out + b * ny);
  }
}
