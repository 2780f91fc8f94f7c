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
#include "helper.h"
#include "rf_module.h"

#ifndef PI
#define PI 3.14159265358979323846
#endif

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

// The reference's whole per-block receiver for one stream, mode 0, as its threads run it:
// rf_thread (src/fm_radio.cpp:62-99: deinterleave, impulseResponseLPF(2.4 MHz, 100 kHz,
// rf_taps) designed per block, convolveWithDecimIQ, fmDemodArctan), mono_stero_thread
// (:153-306: mono LPF, pilot BPF + fmPLL, stereo BPF, mixer, LPF, combiner) and rds_thread
// (:321-441: extract BPF, pllCombine, mixer + LPF, the x19/80 resampler, RRC), with the
// accumulating outputs zeroed between blocks as the threads do.  iq: u8 (as read by
// src/iofunc.cpp:61-69, (x-128)/128) when u8 != 0, else f32.  Throughput baseline only
// (the C++ numerics are not the parity target).  Returns a checksum of the
// outputs so no stage can be skipped.
extern "C" double ref_rx_stream(const void* iq, int u8, int64_t n_complex, int64_t block, int rf_taps,
                                int stereo, int rds) {
  const int rf_decim = 10, audio_decim = 5, num_taps = 151;
  std::vector<float> I(block), Q(block), rf_h, zi(rf_taps - 1, 0.f), zq(rf_taps - 1, 0.f), yi, yq;
  std::vector<float> prev(2, 0.f), demod(block / rf_decim + 16);
  // mono / stereo (src/fm_radio.cpp:153-203)
  std::vector<float> mono_h, rec_h, ext_h, st_h, au_zi(num_taps - 1, 0.f), rec_zi(num_taps - 1, 0.f),
      ext_zi(num_taps - 1, 0.f), st_zi(num_taps - 1, 0.f);
  std::vector<float> audio, bpf_rec, rec_pll, bpf_ext, mixed(block / 20 + 16, 0.f), st_filt, lr;
  impulseResponseLPF(240000, 16000, num_taps, mono_h);
  impulseResponseBPF(18.5e3, 19.5e3, 240000, num_taps, rec_h);
  impulseResponseBPF(22e3, 54e3, 240000, num_taps, ext_h);
  impulseResponseLPF(240000, 16000, num_taps, st_h);
  pll_state_type pst{0.f, 0.f, 1.f, 0.f, 0.f, 1.f};
  // RDS (src/fm_radio.cpp:326-370)
  std::vector<float> ex_h, sq_h, lpf_h, anti_h, rrc_h, ex_zi(num_taps - 1, 0.f), sq_zi(num_taps - 1, 0.f),
      lpf_zi(num_taps - 1, 0.f), anti_zi(num_taps * 19 - 1, 0.f), rrc_zi(num_taps - 1, 0.f);
  std::vector<float> ex, pre_pll, post_pll, lpf_rds, res, rrc;
  impulseResponseBPF(54000, 60000, 240000, num_taps, ex_h);
  impulseResponseBPF(113500, 114500, 240000, num_taps, sq_h);
  impulseResponseLPF(240000, 3000, num_taps, lpf_h);
  impulseResponseLPF(240000 * 19, 57000 / 2, num_taps * 19, anti_h);
  impulseResponseRRC(57000, num_taps, rrc_h);
  pll_state_type prd{0.f, 0.f, 1.f, 0.f, 0.f, 1.f};
  const float phase_adj = PI / 3.3 - PI / 1.5;
  double sum = 0.0;
  for (int64_t b0 = 0; b0 + block <= n_complex; b0 += block) {
    if (u8) {
      const uint8_t* x = static_cast<const uint8_t*>(iq) + 2 * b0;
      for (int64_t i = 0; i < block; ++i) {
        I[i] = ((float)x[2 * i] - 128.f) / 128.f;
        Q[i] = ((float)x[2 * i + 1] - 128.f) / 128.f;
      }
    } else {
      const float* x = static_cast<const float*>(iq) + 2 * b0;
      for (int64_t i = 0; i < block; ++i) {
        I[i] = x[2 * i];
        Q[i] = x[2 * i + 1];
      }
    }
    impulseResponseLPF(2.4e6, 100000, rf_taps, rf_h);
    std::fill(yi.begin(), yi.end(), 0.f);
    std::fill(yq.begin(), yq.end(), 0.f);
    convolveWithDecimIQ(yi, I, rf_h, zi, yq, Q, zq, rf_decim);
    float* dp = demod.data();
    fmDemodArctan(yi, yq, prev, dp);
    const unsigned int nd = (unsigned int)(block / rf_decim);
    convolveWithDecimPointer(audio, dp, nd, mono_h, au_zi, audio_decim);
    if (stereo) {
      convolveWithDecimPointer(bpf_rec, dp, nd, rec_h, rec_zi, 1);
      fmPLL(rec_pll, bpf_rec, 19e3, 240e3, 2.0, 0.0, 0.01, pst);
      convolveWithDecimPointer(bpf_ext, dp, nd, ext_h, ext_zi, 1);
      if (mixed.size() < bpf_ext.size()) mixed.resize(bpf_ext.size());
      for (size_t i = 0; i < bpf_ext.size(); ++i) mixed[i] = bpf_ext[i] * rec_pll[i];
      convolveWithDecim(st_filt, mixed, st_h, st_zi, audio_decim);
      lr.resize(2 * audio.size());
      for (size_t i = 0; i < audio.size(); ++i) {
        lr[2 * i] = (audio[i] + st_filt[i]) / 2;
        lr[2 * i + 1] = (audio[i] - st_filt[i]) / 2;
      }
      for (float v : lr) sum += v;
      std::fill(st_filt.begin(), st_filt.end(), 0.f);
    } else {
      for (float v : audio) sum += v;
    }
    std::fill(audio.begin(), audio.end(), 0.f);
    if (rds) {
      convolveWithDecimPointer(ex, dp, nd, ex_h, ex_zi, 1);
      pllCombine(pre_pll, ex, sq_h, sq_zi, 1, post_pll, 114000, 240000, 0.5, phase_adj - PI / 1.4, 0.001, prd);
      convolveWithDecimAndMixer(lpf_rds, post_pll, ex, lpf_h, lpf_zi, 1);
      convolveWithDecimMode1RDS(res, lpf_rds, anti_h, anti_zi, 80, 19);
      convolveWithDecim(rrc, res, rrc_h, rrc_zi, 1);
      for (float v : rrc) sum += v;
      for (auto* v : {&ex, &pre_pll, &lpf_rds, &res, &rrc}) std::fill(v->begin(), v->end(), 0.f);
    }
  }
  return sum;
}

extern "C" double ref_rx_streams(const void* iq, int u8, int64_t n_complex, int64_t stride, int nstreams,
                                 int64_t block, int rf_taps, int stereo, int rds, int nthreads) {
  double sum = 0.0;
  const int64_t es = u8 ? 2 : 8;
#pragma omp parallel for num_threads(nthreads) schedule(static, 1) reduction(+ : sum)
  for (int s = 0; s < nstreams; ++s)
    sum += ref_rx_stream(static_cast<const char*>(iq) + es * (int64_t)s * stride, u8, n_complex, block, rf_taps,
                         stereo, rds);
  return sum;
}
