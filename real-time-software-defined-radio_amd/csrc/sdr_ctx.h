// Host-side internals of a libsdr context, shared by the C-ABI translation units
// (capi.hip: the per-call entry points; rx.hip: the multi-stream block receiver).
// Not part of the public ABI (include/sdr.h).
#pragma once
#include <hip/hip_runtime.h>

#include <list>
#include <string>
#include <vector>

#include "sdr_launch.h"
#include "../../include/sdr.h"

namespace sdrint {

// scratch slots owned by a context (grown on demand, never shrunk)
enum Slot {
  S_IN, S_IN2, S_OUT, S_OUT2, S_OUT3, S_OUT4, S_STATE, S_STATE2, S_MISC, S_THETA, S_PHI, S_WRAP,
  S_PSD, S_PLLW,
  S_NSLOT
};

struct TapSet {
  std::vector<double> b;
  TapsF32 h;
  float* dev_f32 = nullptr;   // [0, cap): the taps; then, from dev_rev - 1: 0, the taps reversed, 0, 0
  float* dev_rev = nullptr;   // dev_rev[j] = h[T-1-j], dev_rev[-1] = dev_rev[T] = 0 (packed FIR tiles)
  double* dev_f64 = nullptr;
  int* dev_afr = nullptr;     // T = 101 / 151: the u8 MFMA front end's A fragments (fe_mfma.hip)
};

// a PLL loop's response table on the device (sdr_pll_resp_table), per (Kp, Ki, pseudo-block length)
struct RespTable {
  double kp = 0.0, ki = 0.0;
  int64_t pb = 0;
  double* dev = nullptr;
};

// the calling thread's last error message; returns `code`
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace sdrint

struct sdr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  void* slot[sdrint::S_NSLOT] = {};
  size_t cap[sdrint::S_NSLOT] = {};
  // uploaded tap sets (taps are designed once), least recently used first.  A list: a hit
  // is spliced to the back and an overflow evicts the front, so no pointer handed out by
  // a lookup is invalidated by the other lookups of the same entry point (<= 4 per call).
  std::list<sdrint::TapSet> taps;
  // PLL response tables of the long calls made on the context (a few loops; never evicted)
  std::list<sdrint::RespTable> resp;
  // PLL solve counters (SDR_PLL_NSTATS, device; sdr_pll_stats): every PLL launch of the
  // context and of its receivers adds to them
  unsigned long long* pll_stats = nullptr;
};

namespace sdrint {

int set_dev(sdr_ctx* c);
// context scratch slot `s` of at least `bytes` (synchronises the stream when it grows)
int scratch(sdr_ctx* c, Slot s, size_t bytes, void** out);
// device copies (f32, f64) of the tap set b[0..T) (cached per context).  max_T: SDR_MAX_TAPS
// for the FIR kernels, up to SDR_MAX_RESAMPLE_TAPS for the resampler.
int get_taps(sdr_ctx* c, const double* b, int T, const TapSet** out, int max_T = SDR_MAX_TAPS);

// the device response table of loop cfg for a long call of n steps (cached per context);
// *out = NULL when n is not a long call
int get_resp(sdr_ctx* c, const PllCfg& cfg, int64_t n, const double** out);
// the f32 copy get_resp stores after a table of pseudo-block length pb (2 (pb + 5) doubles)
inline const float* resp32_of(const double* resp, int64_t pb) {
  return resp != nullptr ? reinterpret_cast<const float*>(resp + 2 * (pb + 5)) : nullptr;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace sdrint

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return sdrint::fail(SDR_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

#define TRY(expr)                 \
  do {                            \
    int r_ = (expr);              \
    if (r_ != SDR_OK) return r_;  \
  } while (0)

#define CHECK_CTX(c) \
  if ((c) == nullptr) return sdrint::fail(SDR_EINVAL, "context is NULL")
