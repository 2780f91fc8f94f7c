// fm_radio_gpu: the live receiver -- u8 IQ on stdin, interleaved int16
// L/R at 48 kHz on stdout, every DSP stage on the GPU through libsdr's C-ABI.
//
//   rtl_sdr -f 99.9M -s 2.4M - | fm_radio_gpu | aplay -f S16_LE -c 2 -r 48000
//
// Replaces the mode-0 runtime of src/fm_radio.cpp: readStdInBlock (src/iofunc.cpp:61-69,
// blocks of 307 200 bytes, :23), rf_thread (:31-147), mono_stero_thread (:150-318) and its
// int16 writer (:286-302, value * 16384, NaN -> 0).  The DSP follows the Python model
// (model/fmMonoBlock.py:80-173 with the intended combiner) with firwin taps,
// as the parity oracle does; the reference C++'s own tap designs and its per-block state
// resets are not reproduced.
//
// Runtime: instead of four threads and a mutex/condvar queue, one host thread and the
// context's HIP stream with a two-slot pinned ring: while the GPU processes block k
// (async H2D, the receiver's launches, async D2H), the host writes block k-1's audio (and
// runs its RDS link layer) and reads block k+1.  Mode 0 runs on libsdr's block receiver
// (sdr_rx: FE, mono, stereo, RDS; every filter / demod / PLL state stays in device memory).
//
// Options: --mono (mono only, both channels = mono), --rds (also the RDS chain,
// model/fmRDSblock.py:156-204 on the GPU, and its link layer, :207-346, on the host:
// clock/data recovery, Manchester and differential decoding and the syndrome frame sync,
// printing the reference's lines to stderr -- "Syndrome A at position N", "False positive
// Syndrome A at position N", src/fm_radio.cpp:649-695), --resync (with --rds: the C++
// frame_thread's re-sync after more than 10 false positives, "~~~~~Re-Sync~~~~~",
// :697-704; the Python model has no such rule, so it is off by default), --rf-taps N
// (default 151, the reference's), --blocks N (stop after N blocks), --mode 1 (2.5 MS/s IQ,
// src/fm_radio.cpp:36; the 250 kS/s IF goes to 48 kHz through the 24/125 resampler with a
// 6 MHz, 16 kHz filter, :174-180, :228, whose up-gain the reference applies at the int16
// write, :229, :297).  Mode-1 stereo runs in its intended form: pilot and stereo band-passes
// designed at the 250 kS/s IF, fmPll at 19 kHz / Fs 250 kHz (x2), mixer x2, the stereo channel
// through the same 24/125 resampler, L/R = (m +- s)/2 -- the reference designs its mode-1
// band-passes at 6 MHz and runs its PLL at 240 kHz, :201-202, :231-252, so its own mode-1
// stereo has no working form to reproduce (parity unpinned; --mono: mono only).
// Mode-1 taps: firwin(3623, 16 kHz at 6 MHz); the reference's
// 151*24 = 3624-tap sinc design divides 0/0 at its tap 1812 (src/filter.cpp:29-33) and
// writes NaN audio, i.e. silence (:290-293).  Per block it writes floor(15360*24/125) =
// 2 949 samples, as the reference does (src/filter.cpp:264).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "../../include/sdr.h"

namespace {

constexpr int64_t kBlock = 153600;     // complex samples per block (307 200 bytes, src/fm_radio.cpp:23)
constexpr int SDR_MAX_TAPS_ABI = 256;

[[noreturn]] void die(const char* what) {
  std::fprintf(stderr, "fm_radio_gpu: %s: %s\n", what, sdr_last_error());
  std::exit(1);
}
void ck(int rc, const char* what) {
  if (rc != SDR_OK) die(what);
}
void hk(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "fm_radio_gpu: %s: %s\n", what, hipGetErrorString(e));
    std::exit(1);
  }
}

// scipy.signal.firwin(numtaps, cutoff, window='hann'[, pass_zero='bandpass']) with
// scale=True (scipy/signal/_fir_filter_design.py): windowed sum of sincs, normalised to
// unit gain at DC (low-pass) or at the band centre (band-pass).
double sinc(double x) { return x == 0.0 ? 1.0 : std::sin(M_PI * x) / (M_PI * x); }
std::vector<double> firwin(int n, double lo, double hi) {   // lo = 0: low-pass to hi
  std::vector<double> h(n);
  const double alpha = 0.5 * (n - 1);
  for (int k = 0; k < n; ++k) {
    const double m = k - alpha;
    double v = hi * sinc(hi * m);
    if (lo > 0.0) v -= lo * sinc(lo * m);
    const double w = 0.5 - 0.5 * std::cos(2.0 * M_PI * k / (n - 1));
    h[k] = v * w;
  }
  const double f = lo > 0.0 ? 0.5 * (lo + hi) : 0.0;
  double s = 0.0;
  for (int k = 0; k < n; ++k) s += h[k] * std::cos(M_PI * (k - alpha) * f);
  for (double& v : h) v /= s;
  return h;
}

// model/fmRRC.py:12-47 (impulseResponseRootRaisedCosine): roll-off 0.90 at 2375 symbols/s,
// t = (k - N/2)/Fs, the reference's three cases (t = 0, |t| = Ts/(4 beta), general).
std::vector<double> rrc(double fs, int n) {
  const double ts = 1.0 / 2375.0, beta = 0.90;
  std::vector<double> h(n);
  for (int k = 0; k < n; ++k) {
    const double t = (k - n / 2.0) / fs;
    if (t == 0.0) {
      h[k] = 1.0 + beta * (4 / M_PI - 1);
    } else if (t == -ts / (4 * beta) || t == ts / (4 * beta)) {
      const double q = M_PI / (4 * beta);
      h[k] = beta / std::sqrt(2.0) * ((1 + 2 / M_PI) * std::sin(q) + (1 - 2 / M_PI) * std::cos(q));
    } else {
      const double x = 4 * beta * t / ts;
      h[k] = (std::sin(M_PI * t * (1 - beta) / ts) + x * std::cos(M_PI * t * (1 + beta) / ts)) /
             (M_PI * t * (1 - x * x) / ts);
    }
  }
  return h;
}

struct Dev {
  sdr_ctx* c;
  void* alloc(int64_t bytes) {
    void* p = nullptr;
    ck(sdr_malloc(c, bytes, &p), "sdr_malloc");
    ck(sdr_memset(c, p, 0, bytes), "sdr_memset");
    return p;
  }
};

}  // namespace

int main(int argc, char** argv) {
  bool mono = false, print_taps = false, rds = false, resync = false;
  int rf_taps = 151, mode = 0;
  long long max_blocks = -1;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--mono")) mono = true;
    else if (!std::strcmp(argv[i], "--rds")) rds = true;
    else if (!std::strcmp(argv[i], "--resync")) resync = true;
    else if (!std::strcmp(argv[i], "--print-taps")) print_taps = true;
    else if (!std::strcmp(argv[i], "--rf-taps") && i + 1 < argc) rf_taps = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--blocks") && i + 1 < argc) max_blocks = std::atoll(argv[++i]);
    else if (!std::strcmp(argv[i], "--mode") && i + 1 < argc) mode = std::atoi(argv[++i]);
    else {
      std::fprintf(stderr, "usage: fm_radio_gpu [--mode 0|1] [--mono] [--rds [--resync]] [--rf-taps N] [--blocks N] "
                           "[--print-taps] < iq_u8 > pcm_s16le_stereo\n");
      return 2;
    }
  }
  if (mode != 0 && mode != 1) {
    std::fprintf(stderr, "fm_radio_gpu: --mode %d: modes 0 (2.4 MS/s) and 1 (2.5 MS/s)\n", mode);
    return 2;
  }
  if (mode == 1 && rds) {
    std::fprintf(stderr, "fm_radio_gpu: --rds is a mode-0 feature (src/fm_radio.cpp:321-324)\n");
    return 2;
  }
  if (rf_taps < 3 || rf_taps > SDR_MAX_TAPS_ABI) {
    std::fprintf(stderr, "fm_radio_gpu: --rf-taps %d out of range\n", rf_taps);
    return 2;
  }
  // taps (model/fmMonoBlock.py:22-45, :115, :150, :159); mode 1: RF at 2.5 MS/s and the
  // 24/125 resampler filter at 6 MHz
  const double rf_fs = mode == 1 ? 2.5e6 : 2.4e6;
  constexpr int kUp = 24, kDown = 125, kM1Taps = 151 * kUp - 1;
  const std::vector<double> rf_b = firwin(rf_taps, 0.0, 100e3 / (rf_fs / 2));
  const std::vector<double> m1_b = firwin(kM1Taps, 0.0, 16e3 / 3e6);
  const std::vector<double> au_b = firwin(151, 0.0, 16e3 / 120e3);
  const std::vector<double> pil_b = firwin(151, 18.5e3 / 120e3, 19.5e3 / 120e3);
  const std::vector<double> ext_b = firwin(151, 22e3 / 120e3, 54e3 / 120e3);
  const std::vector<double> ste_b = firwin(151, 0.0, 16e3 / 120e3);
  // RDS (model/fmRDSblock.py:88-111)
  const std::vector<double> rex_b = firwin(151, 54e3 / 120e3, 60e3 / 120e3);
  const std::vector<double> rsq_b = firwin(151, 113.5e3 / 120e3, 114.5e3 / 120e3);
  const std::vector<double> rlp_b = firwin(151, 0.0, 3e3 / 120e3);
  const std::vector<double> ran_b = firwin(151, 0.0, (57000.0 / 2) / ((240000.0 * 19) / 2));
  const std::vector<double> rrc_b = rrc(57000.0, 151);
  // mode-1 stereo, the intended form at the 250 kS/s IF (src/fm_radio.cpp:231-252 designs these
  // band-passes at 6 MHz and runs the PLL at Fs 240 kHz: DESIGN.md §8)
  const std::vector<double> pil1_b = firwin(151, 18.5e3 / 125e3, 19.5e3 / 125e3);
  const std::vector<double> ext1_b = firwin(151, 22e3 / 125e3, 54e3 / 125e3);
  if (print_taps) {                    // (no GPU) one line per filter, for the design test
    for (const auto* t : {&rf_b, &au_b, &pil_b, &ext_b, &ste_b, &m1_b, &rex_b, &rsq_b, &rlp_b, &ran_b, &rrc_b}) {
      for (size_t k = 0; k < t->size(); ++k) std::printf(k ? " %.17g" : "%.17g", (*t)[k]);
      std::printf("\n");
    }
    return 0;
  }
  sdr_ctx* c = nullptr;
  const char* dev_env = std::getenv("SDR_DEVICE");
  ck(sdr_create(dev_env ? std::atoi(dev_env) : 0, &c), "sdr_create");
  hipStream_t st = static_cast<hipStream_t>(sdr_stream(c));
  Dev d{c};
  const int64_t M = kBlock / 10, Z = rf_taps - 1;
  const int64_t A = mode == 1 ? M * kUp / kDown : M / 5;     // audio samples written per block
  const int64_t AY = mode == 1 ? (M * kUp + kDown - 1) / kDown : A;   // resampler outputs

  // device buffers of mode 1 (mode 0 runs on the receiver's own)
  auto* d_iq = static_cast<uint8_t*>(d.alloc(2 * kBlock));
  auto* rf_st = static_cast<double*>(d.alloc(8 * (2 * Z + 1)));    // zi_i | zi_q | phase
  auto* d_dm = static_cast<float*>(d.alloc(4 * M + 16));
  auto* d_au = static_cast<float*>(d.alloc(4 * AY + 16));
  auto* zi_au = static_cast<double*>(d.alloc(8 * (kM1Taps - 1)));  // mode 1
  // mode-1 stereo: pilot / stereo band-pass outputs, NCO, mixer, stereo resampler output, L, R,
  // and the carried states (band-pass zi, PLL, stereo resampler zi)
  const bool stereo1 = mode == 1 && !mono;
  float *d_pil = nullptr, *d_ext = nullptr, *d_nco = nullptr, *d_mix = nullptr, *d_side = nullptr, *d_L = nullptr,
        *d_R = nullptr;
  double *zi_pil = nullptr, *zi_ext = nullptr, *pll_st = nullptr, *zi_side = nullptr;
  const double one_tap[1] = {1.0};
  if (stereo1) {
    d_pil = static_cast<float*>(d.alloc(4 * M + 16));
    d_ext = static_cast<float*>(d.alloc(4 * M + 16));
    d_nco = static_cast<float*>(d.alloc(4 * (M + 1) + 16));
    d_mix = static_cast<float*>(d.alloc(4 * M + 16));
    d_side = static_cast<float*>(d.alloc(4 * AY + 16));
    d_L = static_cast<float*>(d.alloc(4 * AY + 16));
    d_R = static_cast<float*>(d.alloc(4 * AY + 16));
    zi_pil = static_cast<double*>(d.alloc(8 * 150));
    zi_ext = static_cast<double*>(d.alloc(8 * 150));
    zi_side = static_cast<double*>(d.alloc(8 * (kM1Taps - 1)));
    pll_st = static_cast<double*>(d.alloc(8 * 6));
    const double init[6] = {0.0, 0.0, 1.0, 0.0, 1.0, 0.0};            // model/fmMonoBlock.py:76
    hk(hipMemcpyAsync(pll_st, init, sizeof init, hipMemcpyHostToDevice, st), "H2D");
  }
  hk(hipStreamSynchronize(st), "hipStreamSynchronize");

  // two-slot pinned ring
  uint8_t* h_in[2];
  float* h_out[2];
  hipEvent_t done[2];
  for (int k = 0; k < 2; ++k) {
    hk(hipHostMalloc(reinterpret_cast<void**>(&h_in[k]), 2 * kBlock, hipHostMallocDefault), "hipHostMalloc");
    hk(hipHostMalloc(reinterpret_cast<void**>(&h_out[k]), 8 * A, hipHostMallocDefault), "hipHostMalloc");
    hk(hipEventCreateWithFlags(&done[k], hipEventDisableTiming), "hipEventCreate");
  }
  std::vector<int16_t> pcm(2 * A);
  auto emit = [&](int slot) {          // block in h_out[slot] -> int16 L/R (src/fm_radio.cpp:286-302)
    hk(hipEventSynchronize(done[slot]), "hipEventSynchronize");
    const float* L = h_out[slot];
    const float* R = h_out[slot] + A;
    for (int64_t i = 0; i < A; ++i) {
      pcm[2 * i] = std::isnan(L[i]) ? 0 : static_cast<int16_t>(L[i] * 16384.0f);
      pcm[2 * i + 1] = std::isnan(R[i]) ? 0 : static_cast<int16_t>(R[i] * 16384.0f);
    }
    if (std::fwrite(pcm.data(), sizeof(int16_t), pcm.size(), stdout) != pcm.size()) std::exit(0);
  };
  auto read_block = [&](uint8_t* dst) {
    size_t got = 0;
    while (got < (size_t)(2 * kBlock)) {
      const size_t r = std::fread(dst + got, 1, 2 * kBlock - got, stdin);
      if (r == 0) return false;        // EOF: a partial last block is dropped (as :106-109)
      got += r;
    }
    return true;
  };

  // mode 0: the block receiver (sdr_rx)
  sdr_rx* rx = nullptr;
  sdr_rds_link* link = nullptr;
  const float *o_l = nullptr, *o_r = nullptr, *o_rrc = nullptr;
  int64_t nrrc = 0;
  if (mode == 0) {
    const int flags = SDR_RX_AUDIO | (mono ? 0 : SDR_RX_STEREO) | (rds ? SDR_RX_RDS : 0);
    ck(sdr_rx_create(c, 1, kBlock, SDR_IQ_U8, flags, &rx), "sdr_rx_create");
    const std::pair<int, const std::vector<double>*> taps[] = {
        {SDR_RX_F_RF, &rf_b}, {SDR_RX_F_AUDIO, &au_b}, {SDR_RX_F_PILOT, &pil_b}, {SDR_RX_F_STEREO_BPF, &ext_b},
        {SDR_RX_F_STEREO_LPF, &ste_b}, {SDR_RX_F_RDS_EXTRACT, &rex_b}, {SDR_RX_F_RDS_SQUARE, &rsq_b},
        {SDR_RX_F_RDS_LPF, &rlp_b}, {SDR_RX_F_RDS_ANTI, &ran_b}, {SDR_RX_F_RDS_RRC, &rrc_b}};
    for (const auto& f : taps) ck(sdr_rx_set_filter(rx, f.first, f.second->data(), (int)f.second->size()), "taps");
    float* p;
    int64_t stride, n;
    ck(sdr_rx_output(rx, mono ? SDR_RX_O_AUDIO : SDR_RX_O_LEFT, &p, &stride, &n), "output");
    o_l = p;
    ck(sdr_rx_output(rx, mono ? SDR_RX_O_AUDIO : SDR_RX_O_RIGHT, &p, &stride, &n), "output");
    o_r = p;
    if (rds) {
      ck(sdr_rx_output(rx, SDR_RX_O_RDS_RRC_I, &p, &stride, &nrrc), "output");
      o_rrc = p;
      ck(sdr_rds_link_create(&link), "sdr_rds_link_create");
      if (resync) ck(sdr_rds_link_set_resync(link, 10), "sdr_rds_link_set_resync");   // :697
    }
  }
  float* h_rrc[2] = {nullptr, nullptr};
  std::vector<double> rrc_d(nrrc);
  std::vector<int64_t> ev(3 * (nrrc / 24 + 128));
  if (rds)
    for (int s2 = 0; s2 < 2; ++s2)
      hk(hipHostMalloc(reinterpret_cast<void**>(&h_rrc[s2]), 4 * nrrc, hipHostMallocDefault), "hipHostMalloc");
  // the RDS link layer of the block in slot `slot` (host, after its D2H landed): the
  // reference's stderr lines (src/fm_radio.cpp:649-704)
  auto link_block = [&](int slot) {
    for (int64_t i = 0; i < nrrc; ++i) rrc_d[i] = h_rrc[slot][i];
    int64_t ne = 0;
    ck(sdr_rds_link_block(link, rrc_d.data(), nrrc, ev.data(), (int64_t)ev.size() / 3, &ne, nullptr, 0, nullptr,
                          nullptr, 0, nullptr, nullptr, 0, nullptr), "RDS link layer");
    for (int64_t e = 0; e < ne; ++e) {
      const int64_t typ = ev[3 * e], pos = ev[3 * e + 1], ok = ev[3 * e + 2];
      if (typ == SDR_RDS_RESYNC) std::fprintf(stderr, "~~~~~Re-Sync~~~~~\n");
      else std::fprintf(stderr, "%sSyndrome %c at position %lld\n", ok ? "" : "False positive ", (char)('A' + typ),
                        (long long)pos);
    }
  };

  long long k = 0;
  int pending = -1;                    // slot whose audio is still to be written
  auto finish = [&](int slot) {
    emit(slot);
    if (link) link_block(slot);
  };
  while ((max_blocks < 0 || k < max_blocks) && read_block(h_in[k & 1])) {
    const int slot = (int)(k & 1);
    hk(hipMemcpyAsync(d_iq, h_in[slot], 2 * kBlock, hipMemcpyHostToDevice, st), "H2D");
    const float* out_l = d_au;
    const float* out_r = d_au;
    if (mode == 0) {
      ck(sdr_rx_process_dev(rx, d_iq, kBlock), "receiver");           // fmMonoBlock.py:86-173 (+ RDS)
      out_l = o_l;
      out_r = o_r;
    } else {
      ck(sdr_rf_frontend_dev(c, d_iq, SDR_IQ_U8, kBlock, kBlock, 0, 1, rf_b.data(), rf_taps, 10, rf_st,
                             rf_st + Z, Z, rf_st, rf_st + Z, rf_st + 2 * Z, d_dm, M, nullptr, nullptr),
         "front end");
      ck(sdr_resample_dev(c, d_dm, M, m1_b.data(), kM1Taps, kUp, kDown, zi_au, zi_au, d_au), "mode-1 resampler");
      if (stereo1) {
        // pilot and stereo band-passes at the IF, the pilot PLL (19 kHz at Fs 250 kHz, x2), the
        // mixer (x2, a one-tap FIR's pre-op), the stereo channel through the same 24/125
        // resampler, then L = (m + s)/2, R = (m - s)/2
        ck(sdr_fir_dev(c, d_dm, nullptr, 1.f, SDR_PRE_NONE, M, M, 0, 1, pil1_b.data(), 151, 1, zi_pil, 150, zi_pil,
                       d_pil, M), "mode-1 pilot BPF");
        ck(sdr_fir_dev(c, d_dm, nullptr, 1.f, SDR_PRE_NONE, M, M, 0, 1, ext1_b.data(), 151, 1, zi_ext, 150, zi_ext,
                       d_ext, M), "mode-1 stereo BPF");
        ck(sdr_pll_dev(c, d_pil, M, M, 1, 19e3, 250e3, 2.0, 0.0, 0.01, pll_st, d_nco, nullptr, M + 1), "mode-1 PLL");
        ck(sdr_fir_dev(c, d_ext, d_nco, 2.f, SDR_PRE_MIX, M, M, 0, 1, one_tap, 1, 1, nullptr, 0, nullptr, d_mix, M),
           "mode-1 mixer");
        ck(sdr_resample_dev(c, d_mix, M, m1_b.data(), kM1Taps, kUp, kDown, zi_side, zi_side, d_side),
           "mode-1 stereo resampler");
        ck(sdr_stereo_combine_dev(c, d_au, d_side, A, d_L, d_R), "mode-1 combiner");
        out_l = d_L;
        out_r = d_R;
      }
    }
    if (pending >= 0) {                // before reusing this slot's output buffer
      finish(pending);
      pending = -1;
    }
    hk(hipMemcpyAsync(h_out[slot], out_l, 4 * A, hipMemcpyDeviceToHost, st), "D2H");
    hk(hipMemcpyAsync(h_out[slot] + A, out_r, 4 * A, hipMemcpyDeviceToHost, st), "D2H");
    if (rds) hk(hipMemcpyAsync(h_rrc[slot], o_rrc, 4 * nrrc, hipMemcpyDeviceToHost, st), "D2H");
    hk(hipEventRecord(done[slot], st), "hipEventRecord");
    pending = slot;
    ++k;
  }
  if (pending >= 0) finish(pending);
  std::fflush(stdout);
  if (link) sdr_rds_link_destroy(link);
  if (rx) sdr_rx_destroy(rx);
  for (float* p : h_rrc)
    if (p) (void)hipHostFree(p);
  for (int s = 0; s < 2; ++s) {
    (void)hipHostFree(h_in[s]);
    (void)hipHostFree(h_out[s]);
    (void)hipEventDestroy(done[s]);
  }
  sdr_destroy(c);
  std::fprintf(stderr, "fm_radio_gpu: %lld blocks\n", k);
  return 0;
}
