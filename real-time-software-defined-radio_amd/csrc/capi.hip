// C-ABI of libsdr.so: the drop-in boundary declared in include/sdr.h.
//
// Two families of entry points:
//   * host-buffer, synchronous ("drop-in"): same argument meaning as the reference
//     per-block functions (lfilter(b,1,x,zi) + [::D], fmDemodArctan, fmPll, ...);
//     inputs are copied to HBM, kernels run on the context's stream, outputs and the
//     updated filter/demod/PLL state are copied back.
//   * device-pointer, asynchronous (`*_dev`): the same kernels on caller-owned device
//     buffers, enqueued on the context's stream; used by the batched benchmark and
//     by the device-resident block pipelines (the Python package keeps all
//     intermediates and states in HBM and only fetches the outputs).
// Every entry point returns 0 or a negative SDR_E* code; sdr_last_error() gives the
// message of the calling thread's last failure.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <new>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>

#include "sdr_ctx.h"

// launchers implemented in fe.hip / fir.hip / pll.hip / psd.hip: sdr_launch.h;
// context internals shared with rx.hip: sdr_ctx.h
using namespace sdrint;

namespace {
thread_local std::string g_err;
}  // namespace

namespace sdrint {

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int set_dev(sdr_ctx* c) {
  HIP_TRY(hipSetDevice(c->device));
  return SDR_OK;
}

int scratch(sdr_ctx* c, Slot s, size_t bytes, void** out) {
  if (bytes == 0) bytes = 16;
  if (c->cap[s] < bytes) {
    if (c->slot[s]) {
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(hipFree(c->slot[s]));
      c->slot[s] = nullptr;
      c->cap[s] = 0;
    }
    size_t want = bytes + bytes / 4;
    hipError_t e = hipMalloc(&c->slot[s], want);
    if (e != hipSuccess) return fail(SDR_ENOMEM, "hipMalloc(%zu): %s", want, hipGetErrorString(e));
    c->cap[s] = want;
  }
  *out = c->slot[s];
  return SDR_OK;
}

// max_T: SDR_MAX_TAPS for the FIR kernels (taps also passed by value, TapsF32), up to
// SDR_MAX_RESAMPLE_TAPS for the resampler (device arrays only; h holds the first 256).
int get_taps(sdr_ctx* c, const double* b, int T, const TapSet** out, int max_T) {
  if (b == nullptr) return fail(SDR_EINVAL, "taps pointer is NULL");
  if (T < 1 || T > max_T) return fail(SDR_EINVAL, "taps=%d outside [1, %d]", T, max_T);
  for (auto it = c->taps.begin(); it != c->taps.end(); ++it)
    if ((int)it->b.size() == T && std::memcmp(it->b.data(), b, sizeof(double) * T) == 0) {
      c->taps.splice(c->taps.end(), c->taps, it);   // most recently used last; `it` stays valid
      *out = &*it;
      return SDR_OK;
    }
  if (c->taps.size() >= 64) {  // bounded cache: evict the least recently used set
    HIP_TRY(hipStreamSynchronize(c->stream));     // kernels in flight may still read it
    TapSet& t = c->taps.front();
    (void)hipFree(t.dev_f32);
    (void)hipFree(t.dev_f64);
    (void)hipFree(t.dev_afr);
    c->taps.pop_front();
  }
  TapSet t;
  t.b.assign(b, b + T);
  std::memset(&t.h, 0, sizeof t.h);
  std::vector<float> f(T);
  for (int k = 0; k < T; ++k) f[k] = (float)b[k];
  for (int k = 0; k < std::min(T, SDR_MAX_TAPS); ++k) t.h.h[k] = f[k];
  const int cap = std::max(T, SDR_MAX_TAPS);
  std::vector<float> fr(cap + T + 4, 0.f);          // forward | pad, 0, reversed, 0, 0
  std::copy(f.begin(), f.end(), fr.begin());
  for (int j = 0; j < T; ++j) fr[cap + 2 + j] = f[T - 1 - j];
  HIP_TRY(hipMalloc(&t.dev_f32, sizeof(float) * fr.size()));
  HIP_TRY(hipMalloc(&t.dev_f64, sizeof(double) * cap));
  t.dev_rev = t.dev_f32 + cap + 2;
  HIP_TRY(hipMemcpy(t.dev_f32, fr.data(), sizeof(float) * fr.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(t.dev_f64, b, sizeof(double) * T, hipMemcpyHostToDevice));
  std::vector<int> afr;
  if (sdr_mfma_fragments(f.data(), T, &afr)) {        // the RF taps of the u8 MFMA front end
    HIP_TRY(hipMalloc(&t.dev_afr, sizeof(int) * afr.size()));
    HIP_TRY(hipMemcpy(t.dev_afr, afr.data(), sizeof(int) * afr.size(), hipMemcpyHostToDevice));
  }
  c->taps.push_back(std::move(t));
  *out = &c->taps.back();
  return SDR_OK;
}

int get_resp(sdr_ctx* c, const PllCfg& cfg, int64_t n, const double** out) {
  *out = nullptr;
  int64_t pb;
  int nb;
  if (!sdr_pll_long_geom(n, &pb, &nb)) return SDR_OK;
  for (const RespTable& t : c->resp)
    if (t.kp == cfg.kp && t.ki == cfg.ki && t.pb == pb) {
      *out = t.dev;
      return SDR_OK;
    }
  std::vector<double> h;
  sdr_pll_resp_table(cfg, n, &h);
  RespTable t;
  t.kp = cfg.kp;
  t.ki = cfg.ki;
  t.pb = pb;
  // the f64 rows, then the same rows in f32 (NcoSrc::resp32, sdr_resp32)
  std::vector<float> hf(h.begin(), h.end());
  HIP_TRY(hipMalloc(&t.dev, sizeof(double) * h.size() + sizeof(float) * hf.size()));
  HIP_TRY(hipMemcpy(t.dev, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(t.dev + h.size(), hf.data(), sizeof(float) * hf.size(), hipMemcpyHostToDevice));
  c->resp.push_back(t);
  *out = t.dev;
  return SDR_OK;
}

}  // namespace sdrint

namespace {
// streaming copy (16 B per lane, nontemporal, 4 loads in flight per lane before their
// stores, grid-stride): the box's copy-kernel bandwidth, measured beside the path's kernels
// 
typedef float cp4 __attribute__((ext_vector_type(4)));
constexpr int CP_U = 4, RD_U = 8;
__global__ __launch_bounds__(256) void copy_probe_kernel(const cp4* __restrict__ a, cp4* __restrict__ b, int64_t n4) {
  const int64_t step = (int64_t)gridDim.x * 256 * CP_U;
  for (int64_t i0 = (int64_t)blockIdx.x * 256 * CP_U + threadIdx.x; i0 < n4; i0 += step) {
    cp4 v[CP_U];
#pragma unroll
    for (int u = 0; u < CP_U; ++u)
      if (i0 + 256 * u < n4) v[u] = __builtin_nontemporal_load(a + i0 + 256 * u);
#pragma unroll
    for (int u = 0; u < CP_U; ++u)
      if (i0 + 256 * u < n4) __builtin_nontemporal_store(v[u], b + i0 + 256 * u);
  }
}
// read-only stream (16 B per lane, nontemporal, 8 loads in flight per lane): the ceiling of a
// kernel that reads its input once and writes little (the FE: 2 or 8 B in per complex sample,
// 0.4 B out); the loads feed a sum that is stored only if it is NaN (never, on the zeroed buffer)
__global__ __launch_bounds__(256) void read_probe_kernel(const cp4* __restrict__ a, int64_t n4, cp4* sink) {
  const int64_t step = (int64_t)gridDim.x * 256 * RD_U;
  cp4 acc = cp4{0.f, 0.f, 0.f, 0.f};
  for (int64_t i0 = (int64_t)blockIdx.x * 256 * RD_U + threadIdx.x; i0 < n4; i0 += step) {
    cp4 v[RD_U];
#pragma unroll
    for (int u = 0; u < RD_U; ++u)
      v[u] = i0 + 256 * u < n4 ? __builtin_nontemporal_load(a + i0 + 256 * u) : cp4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < RD_U; ++u) acc += v[u];
  }
  if (acc.x != acc.x) sink[threadIdx.x] = acc;
}
}  // namespace

namespace {

int h2d(sdr_ctx* c, void* dst, const void* src, size_t bytes) {
  if (bytes) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  return SDR_OK;
}
int d2h(sdr_ctx* c, void* dst, const void* src, size_t bytes) {
  if (bytes) HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
  return SDR_OK;
}

}  // namespace

// ================================================================================
extern "C" {

int sdr_abi_version(void) { return SDR_ABI_VERSION; }

const char* sdr_last_error(void) { return g_err.c_str(); }

int sdr_device_count(int* n) {
  if (n == nullptr) return fail(SDR_EINVAL, "n is NULL");
  *n = 0;
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) { *n = 0; return fail(SDR_EHIP, "hipGetDeviceCount: %s", hipGetErrorString(e)); }
  return SDR_OK;
}

int sdr_device_info(int device, char* pci, int len, int* cus) {
  int n = 0;
  TRY(sdr_device_count(&n));
  if (device < 0 || device >= n) return fail(SDR_EINVAL, "device %d not in [0, %d)", device, n);
  if (pci != nullptr && len > 0) {
    const hipError_t e = hipDeviceGetPCIBusId(pci, len, device);
    if (e != hipSuccess) return fail(SDR_EHIP, "hipDeviceGetPCIBusId(%d): %s", device, hipGetErrorString(e));
  }
  if (cus != nullptr) {
    hipDeviceProp_t prop;
    const hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return fail(SDR_EHIP, "hipGetDeviceProperties(%d): %s", device, hipGetErrorString(e));
    *cus = prop.multiProcessorCount;
  }
  return SDR_OK;
}

int sdr_create(int device, sdr_ctx** out) {
  if (out == nullptr) return fail(SDR_EINVAL, "out is NULL");
  *out = nullptr;
  int n = 0;
  TRY(sdr_device_count(&n));
  if (device < 0 || device >= n) return fail(SDR_EINVAL, "device %d not in [0, %d)", device, n);
  sdr_ctx* c = new sdr_ctx;
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&c->pll_stats, sizeof(unsigned long long) * SDR_PLL_NSTATS);
  if (e == hipSuccess) e = hipMemset(c->pll_stats, 0, sizeof(unsigned long long) * SDR_PLL_NSTATS);
  if (e != hipSuccess) {
    if (c->pll_stats) (void)hipFree(c->pll_stats);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return fail(SDR_EHIP, "context creation on device %d: %s", device, hipGetErrorString(e));
  }
  *out = c;
  return SDR_OK;
}

void sdr_destroy(sdr_ctx* c) {
  if (c == nullptr) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (int s = 0; s < S_NSLOT; ++s) if (c->slot[s]) (void)hipFree(c->slot[s]);
  for (TapSet& t : c->taps) { (void)hipFree(t.dev_f32); (void)hipFree(t.dev_f64); (void)hipFree(t.dev_afr); }
  for (RespTable& t : c->resp) (void)hipFree(t.dev);
  if (c->pll_stats) (void)hipFree(c->pll_stats);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int sdr_synchronize(sdr_ctx* c) {
  CHECK_CTX(c);
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SDR_OK;
}

void* sdr_stream(sdr_ctx* c) { return c ? (void*)c->stream : nullptr; }

// ---- device memory ---------------------------------------------------------------
int sdr_malloc(sdr_ctx* c, int64_t bytes, void** out) {
  CHECK_CTX(c);
  if (out == nullptr || bytes < 0) return fail(SDR_EINVAL, "bad sdr_malloc arguments");
  TRY(set_dev(c));
  hipError_t e = hipMalloc(out, bytes ? (size_t)bytes : 16);
  if (e != hipSuccess) return fail(SDR_ENOMEM, "hipMalloc(%lld): %s", (long long)bytes, hipGetErrorString(e));
  return SDR_OK;
}

int sdr_free(sdr_ctx* c, void* p) {
  CHECK_CTX(c);
  if (p) HIP_TRY(hipFree(p));
  return SDR_OK;
}

int sdr_memcpy_h2d(sdr_ctx* c, void* dst, const void* src, int64_t bytes) {
  CHECK_CTX(c);
  TRY(h2d(c, dst, src, (size_t)bytes));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SDR_OK;
}

int sdr_memcpy_d2h(sdr_ctx* c, void* dst, const void* src, int64_t bytes) {
  CHECK_CTX(c);
  TRY(d2h(c, dst, src, (size_t)bytes));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SDR_OK;
}

int sdr_memcpy_d2d(sdr_ctx* c, void* dst, const void* src, int64_t bytes) {
  CHECK_CTX(c);
  if (bytes) HIP_TRY(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, c->stream));
  return SDR_OK;
}

int sdr_memset(sdr_ctx* c, void* dst, int value, int64_t bytes) {
  CHECK_CTX(c);
  if (bytes) HIP_TRY(hipMemsetAsync(dst, value, (size_t)bytes, c->stream));
  return SDR_OK;
}

// ---- events (timing on the context stream, where the kernels run) ------------------
int sdr_event_create(sdr_ctx* c, void** ev) {
  CHECK_CTX(c);
  if (ev == nullptr) return fail(SDR_EINVAL, "ev is NULL");
  TRY(set_dev(c));
  hipEvent_t e;
  HIP_TRY(hipEventCreate(&e));
  *ev = (void*)e;
  return SDR_OK;
}
int sdr_event_record(sdr_ctx* c, void* ev) {
  CHECK_CTX(c);
  HIP_TRY(hipEventRecord((hipEvent_t)ev, c->stream));
  return SDR_OK;
}
int sdr_event_elapsed_ms(void* ev0, void* ev1, float* ms) {
  if (ms == nullptr) return fail(SDR_EINVAL, "ms is NULL");
  HIP_TRY(hipEventSynchronize((hipEvent_t)ev1));
  HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)ev0, (hipEvent_t)ev1));
  return SDR_OK;
}
int sdr_event_destroy(void* ev) {
  if (ev) HIP_TRY(hipEventDestroy((hipEvent_t)ev));
  return SDR_OK;
}

namespace {
// best of `reps` (after two warm-ups) of the copy (read_only = 0: GB/s counting read + write)
// or read-only probe over `bytes`
int stream_probe(sdr_ctx* c, int64_t bytes, int reps, double* gbs, bool read_only, const char* name) {
  CHECK_CTX(c);
  if (gbs == nullptr || bytes < 16 || reps < 1) return fail(SDR_EINVAL, "%s: bytes %lld, reps %d", name,
                                                            (long long)bytes, reps);
  TRY(set_dev(c));
  const int64_t n4 = bytes / 16;
  void *a = nullptr, *b = nullptr;
  hipError_t e = hipMalloc(&a, (size_t)n4 * 16);
  if (e == hipSuccess) e = hipMalloc(&b, read_only ? 256 * 16 : (size_t)n4 * 16);
  if (e != hipSuccess) {
    if (a) (void)hipFree(a);
    return fail(SDR_ENOMEM, "%s: hipMalloc: %s", name, hipGetErrorString(e));
  }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, c->device) == hipSuccess) cus = prop.multiProcessorCount;
  const int U = read_only ? RD_U : CP_U;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((int64_t)cus * 8, (n4 + 256 * U - 1) / (256 * U)));
  float best = 0.f;
  e = hipMemsetAsync(a, 0, (size_t)n4 * 16, c->stream);
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  for (int r = 0; r < reps + 2 && e == hipSuccess; ++r) {
    e = hipEventRecord(e0, c->stream);
    if (read_only)
      hipLaunchKernelGGL(read_probe_kernel, dim3(grid), dim3(256), 0, c->stream, (const cp4*)a, n4, (cp4*)b);
    else
      hipLaunchKernelGGL(copy_probe_kernel, dim3(grid), dim3(256), 0, c->stream, (const cp4*)a, (cp4*)b, n4);
    if (e == hipSuccess) e = hipGetLastError();
    if (e == hipSuccess) e = hipEventRecord(e1, c->stream);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (r >= 2 && (best == 0.f || ms < best)) best = ms;    // two warm-ups
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipFree(a);
  (void)hipFree(b);
  if (e != hipSuccess) return fail(SDR_EHIP, "%s: %s", name, hipGetErrorString(e));
  *gbs = (read_only ? 1.0 : 2.0) * (double)(n4 * 16) / ((double)best * 1e-3) / 1e9;
  return SDR_OK;
}
}  // namespace

int sdr_copy_bandwidth(sdr_ctx* c, int64_t bytes, int reps, double* gbs) {
  return stream_probe(c, bytes, reps, gbs, false, "sdr_copy_bandwidth");
}

int sdr_read_bandwidth(sdr_ctx* c, int64_t bytes, int reps, double* gbs) {
  return stream_probe(c, bytes, reps, gbs, true, "sdr_read_bandwidth");
}

// ================================================================================
// Device-pointer API (asynchronous on the context stream)
// ================================================================================
int sdr_rf_frontend_dev(sdr_ctx* c, const void* iq, int iq_dtype, int64_t n, int64_t stride,
                        int64_t hist, int nstreams, const double* b, int taps, int decim,
                        const double* zi_i, const double* zi_q, int64_t zi_stride, double* zf_i,
                        double* zf_q, double* prev_phase, float* demod, int64_t out_stride,
                        float* i_ds, float* q_ds) {
  CHECK_CTX(c);
  if (n < 0 || nstreams < 0 || hist < 0) return fail(SDR_EINVAL, "negative size");
  if (iq_dtype != SDR_IQ_F32 && iq_dtype != SDR_IQ_U8) return fail(SDR_EINVAL, "iq_dtype %d", iq_dtype);
  if (decim < 1) return fail(SDR_EINVAL, "decim=%d < 1", decim);
  if ((zi_i == nullptr) != (zi_q == nullptr)) return fail(SDR_EINVAL, "zi_i/zi_q must both be set or NULL");
  if ((zf_i == nullptr) != (zf_q == nullptr)) return fail(SDR_EINVAL, "zf_i/zf_q must both be set or NULL");
  if ((i_ds == nullptr) != (q_ds == nullptr)) return fail(SDR_EINVAL, "i_ds/q_ds must both be set or NULL");
  const int64_t M = ceil_div(n, decim);
  if (n > 0 && (iq == nullptr || demod == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  if (nstreams > 1 && (out_stride < M || stride < n)) return fail(SDR_EINVAL, "stream strides too small");
  if (nstreams > 1 && (zi_i || zf_i) && zi_stride < taps - 1)
    return fail(SDR_EINVAL, "zi_stride %lld < taps-1", (long long)zi_stride);
  TRY(set_dev(c));
  const TapSet* ts;
  TRY(get_taps(c, b, taps, &ts));
  const int u8 = iq_dtype == SDR_IQ_U8;
  const int G = u8 ? 8 : 2;
  float* last_phi = nullptr;
  int* wraps = nullptr;
  if (prev_phase != nullptr) {
    TRY(scratch(c, S_PHI, sizeof(float) * (size_t)nstreams, (void**)&last_phi));
    TRY(scratch(c, S_WRAP, sizeof(int) * (size_t)nstreams, (void**)&wraps));
    HIP_TRY(hipMemsetAsync(wraps, 0, sizeof(int) * (size_t)nstreams, c->stream));
  }
  // zf first (reads zi), into scratch when it aliases zi
  double* zfi = zf_i;
  double* zfq = zf_q;
  const bool alias = zf_i && (zf_i == zi_i || zf_q == zi_q);
  const int64_t zs = nstreams > 1 ? zi_stride : (taps - 1);
  if (alias) {
    double* tmp;
    TRY(scratch(c, S_STATE2, sizeof(double) * 2 * (size_t)zs * nstreams, (void**)&tmp));
    zfi = tmp;
    zfq = tmp + zs * nstreams;
  }
  // u8: the slot kernel takes any stream stride (streams whose base is not 4-B aligned
  // build their images with guarded byte loads); f32 needs 16-B aligned stream bases
  const bool fast = (taps == 101 || taps == 151) && decim == 10 &&
                    (nstreams <= 1 || u8 || stride % G == 0) && ((uintptr_t)iq % (u8 ? 4 : 16)) == 0;
  if (fast) {
    FeLaunch a{iq, n, nstreams > 1 ? stride : ceil_div(n, G) * G, hist, nstreams,
               ts->dev_f32, &ts->h, taps, decim, u8, zi_i, zi_q, zs, prev_phase,
               demod, nstreams > 1 ? out_stride : M, i_ds, q_ds, last_phi, wraps, ts->dev_afr};
    HIP_TRY(sdr_launch_fe(a, c->stream));
  } else {
    // generic tap counts: strided FIR on I and Q, then the standalone discriminator
    if (u8) return fail(SDR_EUNSUPPORTED, "u8 IQ needs taps 101/151 and decim 10 (got %d, %d)", taps, decim);
    float *fi = i_ds, *fq = q_ds;
    const int64_t os = nstreams > 1 ? out_stride : M;
    if (fi == nullptr) {
      float* tmp;
      TRY(scratch(c, S_OUT4, sizeof(float) * 2 * (size_t)os * nstreams, (void**)&tmp));
      fi = tmp;
      fq = tmp + os * nstreams;
    }
    const float* x = (const float*)iq;
    const int64_t xs = 2 * (nstreams > 1 ? stride : n);
    FirLaunch a{x, nullptr, 1.f, 0, n, xs, 2, hist, nstreams, ts->dev_f32, &ts->h, taps, decim,
                zi_i, zs, fi, os};
    HIP_TRY(sdr_launch_fir(a, c->stream));
    a.x = x + 1; a.zi = zi_q; a.y = fq;
    HIP_TRY(sdr_launch_fir(a, c->stream));
    HIP_TRY(sdr_launch_demod(fi, fq, M, os, nstreams, prev_phase, demod, os, last_phi, wraps, c->stream));
  }
  if (zf_i != nullptr)
    HIP_TRY(sdr_launch_iq_zf(iq, u8, n, nstreams > 1 ? stride : n, nstreams, ts->dev_f64, taps,
                             zi_i, zi_q, zs, zfi, zfq, c->stream));
  if (alias) {
    HIP_TRY(hipMemcpyAsync(zf_i, zfi, sizeof(double) * zs * nstreams, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(zf_q, zfq, sizeof(double) * zs * nstreams, hipMemcpyDeviceToDevice, c->stream));
  }
  if (prev_phase != nullptr)
    HIP_TRY(sdr_launch_demod_state(nstreams, M, last_phi, wraps, prev_phase, c->stream));
  return SDR_OK;
}

int sdr_fe_mono_fused(int rf_taps, int rf_decim, int audio_taps, int audio_decim) {
  return rf_decim == 10 && rf_taps == 101 && audio_taps == 151 && audio_decim == 5;
}

int sdr_fe_mono_dev(sdr_ctx* c, const void* iq, int iq_dtype, int64_t n, int64_t stride, int nstreams,
                    const double* rf_b, int rf_taps, int rf_decim, const double* audio_b, int audio_taps,
                    int audio_decim, float* audio, int64_t audio_stride) {
  CHECK_CTX(c);
  if (n < 0 || nstreams < 0) return fail(SDR_EINVAL, "negative size");
  if (iq_dtype != SDR_IQ_F32 && iq_dtype != SDR_IQ_U8) return fail(SDR_EINVAL, "iq_dtype %d", iq_dtype);
  if (rf_decim < 1 || audio_decim < 1) return fail(SDR_EINVAL, "decim < 1");
  const int64_t M = ceil_div(n, rf_decim);
  const int64_t A = ceil_div(M, audio_decim);
  if (n > 0 && (iq == nullptr || audio == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  if (nstreams > 1 && (audio_stride < A || stride < n)) return fail(SDR_EINVAL, "stream strides too small");
  TRY(set_dev(c));
  const TapSet *rts, *ats;
  TRY(get_taps(c, audio_b, audio_taps, &ats));
  TRY(get_taps(c, rf_b, rf_taps, &rts));
  const int u8 = iq_dtype == SDR_IQ_U8;
  const int64_t xs = nstreams > 1 ? stride : ceil_div(n, 2) * 2;
  const int64_t as = nstreams > 1 ? audio_stride : A;
  const bool fused = sdr_fe_mono_fused(rf_taps, rf_decim, audio_taps, audio_decim) && xs % 2 == 0 &&
                     ((uintptr_t)iq % (u8 ? 4 : 16)) == 0 && ((uintptr_t)audio % 4) == 0;
  if (fused) {
    FeLaunch a{iq, n, xs, 0, nstreams, rts->dev_f32, &rts->h, rf_taps, rf_decim, u8, nullptr, nullptr, 0,
               nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr};
    a.afr = rts->dev_afr;
    const hipError_t e = sdr_launch_fe_mono(a, ats->dev_f32, ats->dev_rev, audio_taps, audio_decim, audio, as, c->stream);
    if (e == hipSuccess) return SDR_OK;
    if (e != hipErrorInvalidValue) HIP_TRY(e);
    // unsupported by the fused kernel: fall through to the two-kernel path
  }
  // any other configuration: front end into scratch HBM, then the audio filter
  float* dm;
  TRY(scratch(c, S_OUT3, sizeof(float) * (size_t)(M + 4) * (nstreams > 0 ? nstreams : 1), (void**)&dm));
  TRY(sdr_rf_frontend_dev(c, iq, iq_dtype, n, nstreams > 1 ? stride : n, 0, nstreams, rf_b, rf_taps,
                          rf_decim, nullptr, nullptr, 0, nullptr, nullptr, nullptr, dm, M + 4, nullptr,
                          nullptr));
  return sdr_fir_dev(c, dm, nullptr, 1.f, SDR_PRE_NONE, M, M + 4, 0, nstreams, audio_b, audio_taps,
                     audio_decim, nullptr, 0, nullptr, audio, as);
}

int sdr_fir_dev(sdr_ctx* c, const float* x, const float* mix, float gain, int pre, int64_t n,
                int64_t x_stride, int64_t hist, int nstreams, const double* b, int taps, int decim,
                const double* zi, int64_t zi_stride, double* zf, float* y, int64_t y_stride) {
  CHECK_CTX(c);
  if (n < 0 || nstreams < 0 || hist < 0) return fail(SDR_EINVAL, "negative size");
  if (decim < 1) return fail(SDR_EINVAL, "decim=%d < 1", decim);
  if (pre < SDR_PRE_NONE || pre > SDR_PRE_MIX) return fail(SDR_EINVAL, "pre=%d", pre);
  if (pre == SDR_PRE_MIX && mix == nullptr) return fail(SDR_EINVAL, "PRE_MIX needs the mix operand");
  const int64_t M = ceil_div(n, decim);
  if (n > 0 && (x == nullptr || y == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  if (nstreams > 1 && (y_stride < M || x_stride < n)) return fail(SDR_EINVAL, "stream strides too small");
  if (nstreams > 1 && (zi || zf) && zi_stride < taps - 1)
    return fail(SDR_EINVAL, "zi_stride %lld < taps-1", (long long)zi_stride);
  TRY(set_dev(c));
  const TapSet* ts;
  TRY(get_taps(c, b, taps, &ts));
  const int64_t zs = nstreams > 1 ? zi_stride : (taps - 1);
  const int64_t xs = nstreams > 1 ? x_stride : n;
  double* zfo = zf;
  const bool alias = zf && zf == zi;
  if (alias) TRY(scratch(c, S_STATE2, sizeof(double) * (size_t)zs * nstreams, (void**)&zfo));
  FirLaunch a{x, mix, gain, pre, n, xs, 1, hist, nstreams, ts->dev_f32, &ts->h, taps, decim,
              zi, zs, y, nstreams > 1 ? y_stride : M};
  HIP_TRY(sdr_launch_fir(a, c->stream));
  if (zf != nullptr)
    HIP_TRY(sdr_launch_zf(x, mix, gain, pre, n, xs, nstreams, 1, ts->dev_f64, taps, zi, zs, zfo, c->stream));
  if (alias)
    HIP_TRY(hipMemcpyAsync(zf, zfo, sizeof(double) * zs * nstreams, hipMemcpyDeviceToDevice, c->stream));
  return SDR_OK;
}

int sdr_resample_dev(sdr_ctx* c, const float* x, int64_t n, const double* b, int taps, int up,
                     int down, const double* zi, double* zf, float* y) {
  CHECK_CTX(c);
  if (n < 0 || up < 1 || down < 1) return fail(SDR_EINVAL, "bad resampler sizes");
  if (n > 0 && (x == nullptr || y == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  TRY(set_dev(c));
  const TapSet* ts;
  TRY(get_taps(c, b, taps, &ts, SDR_MAX_RESAMPLE_TAPS));
  double* zfo = zf;
  const bool alias = zf && zf == zi;
  if (alias) TRY(scratch(c, S_STATE2, sizeof(double) * (size_t)taps, (void**)&zfo));
  HIP_TRY(sdr_launch_resample(x, n, ts->dev_f32, taps, up, down, zi, y, c->stream));
  if (zf != nullptr)
    HIP_TRY(sdr_launch_zf(x, nullptr, 1.f, 0, n, n, 1, up, ts->dev_f64, taps, zi, taps - 1, zfo, c->stream));
  if (alias)
    HIP_TRY(hipMemcpyAsync(zf, zfo, sizeof(double) * (taps - 1), hipMemcpyDeviceToDevice, c->stream));
  return SDR_OK;
}

int sdr_fm_demod_dev(sdr_ctx* c, const float* I, const float* Q, int64_t n, int64_t stride,
                     int nstreams, double* prev_phase, float* out, int64_t out_stride) {
  CHECK_CTX(c);
  if (n < 0 || nstreams < 0) return fail(SDR_EINVAL, "negative size");
  if (n > 0 && (I == nullptr || Q == nullptr || out == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  TRY(set_dev(c));
  float* last_phi = nullptr;
  int* wraps = nullptr;
  if (prev_phase != nullptr) {
    TRY(scratch(c, S_PHI, sizeof(float) * (size_t)nstreams, (void**)&last_phi));
    TRY(scratch(c, S_WRAP, sizeof(int) * (size_t)nstreams, (void**)&wraps));
    HIP_TRY(hipMemsetAsync(wraps, 0, sizeof(int) * (size_t)nstreams, c->stream));
  }
  const int64_t xs = nstreams > 1 ? stride : n;
  HIP_TRY(sdr_launch_demod(I, Q, n, xs, nstreams, prev_phase, out, nstreams > 1 ? out_stride : n,
                           last_phi, wraps, c->stream));
  if (prev_phase != nullptr)
    HIP_TRY(sdr_launch_demod_state(nstreams, n, last_phi, wraps, prev_phase, c->stream));
  return SDR_OK;
}

int sdr_pll_dev(sdr_ctx* c, const float* in, int64_t n, int64_t in_stride, int nstreams,
                double freq, double fs, double nco_scale, double phase_adj, double norm_bw,
                double* state, float* nco_i, float* nco_q, int64_t out_stride) {
  CHECK_CTX(c);
  if (n < 0 || nstreams < 0) return fail(SDR_EINVAL, "negative size");
  if (state == nullptr || nco_i == nullptr || (n > 0 && in == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  if (!(fs != 0.0)) return fail(SDR_EINVAL, "Fs must be non-zero");
  TRY(set_dev(c));
  if (nstreams > 1 && (in_stride < n || out_stride < n + 1))
    return fail(SDR_EINVAL, "stream strides too small (in_stride %lld < n or out_stride %lld < n+1)",
                (long long)in_stride, (long long)out_stride);
  if (nstreams == 0) return SDR_OK;
  PllJobs P{};
  P.njobs = 1;
  P.nstreams = nstreams;
  P.n = n;
  const int64_t ths = (n + 1) / 2 * 2 + 2;          // even: 16-B aligned rows
  const int64_t cst = (n + n / 32 + 1) / 2 * 2 + 2;
  double *theta, *cbuf;
  TRY(scratch(c, S_THETA, sizeof(double) * (size_t)ths * nstreams, (void**)&theta));
  TRY(scratch(c, S_MISC, sizeof(double) * (size_t)cst * nstreams, (void**)&cbuf));
  P.j[0] = PllJob{in, nstreams > 1 ? in_stride : n, state, theta, ths, nco_i, nco_q,
                  nstreams > 1 ? out_stride : n + 1,
                  PllCfg{freq, fs, nco_scale, phase_adj, norm_bw * 2.666, norm_bw * norm_bw * 3.555}, cbuf, cst};
  P.stats = c->pll_stats;
  P.nco_rows = 1;                                   // fmPll's outputs are the NCO rows
  TRY(get_resp(c, P.j[0].cfg, n, &P.j[0].resp));
  const int64_t wb = sdr_pll_work_bytes(1, nstreams, n);    // long calls: pseudo-block records
  if (wb > 0) TRY(scratch(c, S_PLLW, (size_t)wb, &P.work));
  HIP_TRY(sdr_launch_pll_jobs(P, c->stream));
  return SDR_OK;
}

int sdr_pll_stats(sdr_ctx* c, int64_t* out, int reset) {
  CHECK_CTX(c);
  if (out == nullptr) return fail(SDR_EINVAL, "sdr_pll_stats: out is NULL");
  TRY(set_dev(c));
  unsigned long long h[SDR_PLL_NSTATS];
  HIP_TRY(hipMemcpyAsync(h, c->pll_stats, sizeof h, hipMemcpyDeviceToHost, c->stream));
  if (reset) HIP_TRY(hipMemsetAsync(c->pll_stats, 0, sizeof h, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (int i = 0; i < SDR_PLL_NSTATS; ++i) out[i] = (int64_t)h[i];
  return SDR_OK;
}

int sdr_stereo_combine_dev(sdr_ctx* c, const float* mono, const float* side, int64_t n, float* left,
                           float* right) {
  CHECK_CTX(c);
  if (n < 0) return fail(SDR_EINVAL, "negative size");
  if (n > 0 && (!mono || !side || !left || !right)) return fail(SDR_EINVAL, "NULL buffer");
  TRY(set_dev(c));
  HIP_TRY(sdr_launch_combine(mono, side, n, left, right, c->stream));
  return SDR_OK;
}

// ================================================================================
// Host-buffer drop-in API (synchronous)
// ================================================================================
int sdr_rf_frontend(sdr_ctx* c, const void* iq, int iq_dtype, int64_t n, const double* b, int taps,
                    int decim, double* zi_i, double* zi_q, double* prev_phase, float* demod,
                    float* i_ds, float* q_ds) {
  CHECK_CTX(c);
  if (n < 0) return fail(SDR_EINVAL, "negative size");
  if (iq_dtype != SDR_IQ_F32 && iq_dtype != SDR_IQ_U8) return fail(SDR_EINVAL, "iq_dtype %d", iq_dtype);
  if (taps < 1 || taps > SDR_MAX_TAPS) return fail(SDR_EINVAL, "taps=%d outside [1, %d]", taps, SDR_MAX_TAPS);
  if (decim < 1) return fail(SDR_EINVAL, "decim=%d < 1", decim);
  if ((zi_i == nullptr) != (zi_q == nullptr)) return fail(SDR_EINVAL, "zi_i/zi_q must both be set or NULL");
  if ((i_ds == nullptr) != (q_ds == nullptr)) return fail(SDR_EINVAL, "i_ds/q_ds must both be set or NULL");
  if (n > 0 && (iq == nullptr || demod == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  TRY(set_dev(c));
  const int64_t M = ceil_div(n, decim);
  const size_t in_bytes = (size_t)n * (iq_dtype == SDR_IQ_U8 ? 2 : 8);
  void* d_iq;
  float* d_out;
  double* d_st;
  TRY(scratch(c, S_IN, in_bytes, &d_iq));
  TRY(scratch(c, S_OUT, sizeof(float) * 3 * (size_t)(M + 4), (void**)&d_out));
  const int Z = taps - 1;
  TRY(scratch(c, S_STATE, sizeof(double) * (4 * (size_t)Z + 1), (void**)&d_st));
  double *dzi = d_st, *dzq = d_st + Z, *dfi = d_st + 2 * Z, *dfq = d_st + 3 * Z, *dph = d_st + 4 * Z;
  TRY(h2d(c, d_iq, iq, in_bytes));
  if (zi_i) {
    TRY(h2d(c, dzi, zi_i, sizeof(double) * Z));
    TRY(h2d(c, dzq, zi_q, sizeof(double) * Z));
  }
  const double ph0 = prev_phase ? *prev_phase : 0.0;
  TRY(h2d(c, dph, &ph0, sizeof(double)));
  float* dI = i_ds ? d_out + (M + 4) : nullptr;
  float* dQ = i_ds ? d_out + 2 * (M + 4) : nullptr;
  TRY(sdr_rf_frontend_dev(c, d_iq, iq_dtype, n, n, 0, 1, b, taps, decim, zi_i ? dzi : nullptr,
                          zi_i ? dzq : nullptr, Z, zi_i ? dfi : nullptr, zi_i ? dfq : nullptr,
                          dph, d_out, M, dI, dQ));
  TRY(d2h(c, demod, d_out, sizeof(float) * M));
  if (i_ds) {
    TRY(d2h(c, i_ds, dI, sizeof(float) * M));
    TRY(d2h(c, q_ds, dQ, sizeof(float) * M));
  }
  if (zi_i) {
    TRY(d2h(c, zi_i, dfi, sizeof(double) * Z));
    TRY(d2h(c, zi_q, dfq, sizeof(double) * Z));
  }
  double ph1 = ph0;
  TRY(d2h(c, &ph1, dph, sizeof(double)));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (prev_phase) *prev_phase = ph1;
  return SDR_OK;
}

int sdr_lfilter(sdr_ctx* c, const float* x, const float* mix, float gain, int pre, int64_t n,
                const double* b, int taps, int decim, double* zi_inout, float* y) {
  CHECK_CTX(c);
  if (n < 0) return fail(SDR_EINVAL, "negative size");
  if (taps < 1 || taps > SDR_MAX_TAPS) return fail(SDR_EINVAL, "taps=%d outside [1, %d]", taps, SDR_MAX_TAPS);
  if (decim < 1) return fail(SDR_EINVAL, "decim=%d < 1", decim);
  if (pre < SDR_PRE_NONE || pre > SDR_PRE_MIX) return fail(SDR_EINVAL, "pre=%d", pre);
  if (pre == SDR_PRE_MIX && mix == nullptr) return fail(SDR_EINVAL, "PRE_MIX needs the mix operand");
  if (n > 0 && (x == nullptr || y == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  TRY(set_dev(c));
  const int64_t M = ceil_div(n, decim);
  float *dx, *dc = nullptr, *dy;
  double* dz;
  const int Z = taps - 1;
  TRY(scratch(c, S_IN, sizeof(float) * (size_t)n, (void**)&dx));
  if (pre == SDR_PRE_MIX) TRY(scratch(c, S_IN2, sizeof(float) * (size_t)n, (void**)&dc));
  TRY(scratch(c, S_OUT, sizeof(float) * (size_t)M, (void**)&dy));
  TRY(scratch(c, S_STATE, sizeof(double) * 2 * (size_t)(Z + 1), (void**)&dz));
  TRY(h2d(c, dx, x, sizeof(float) * n));
  if (dc) TRY(h2d(c, dc, mix, sizeof(float) * n));
  if (zi_inout) TRY(h2d(c, dz, zi_inout, sizeof(double) * Z));
  TRY(sdr_fir_dev(c, dx, dc, gain, pre, n, n, 0, 1, b, taps, decim, zi_inout ? dz : nullptr, Z,
                  zi_inout ? dz + Z + 1 : nullptr, dy, M));
  TRY(d2h(c, y, dy, sizeof(float) * M));
  if (zi_inout) TRY(d2h(c, zi_inout, dz + Z + 1, sizeof(double) * Z));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SDR_OK;
}

int sdr_lfilter_decim(sdr_ctx* c, const float* x, int64_t n, const double* b, int taps, int decim,
                      double* zi_inout, float* y) {
  return sdr_lfilter(c, x, nullptr, 1.f, SDR_PRE_NONE, n, b, taps, decim, zi_inout, y);
}

int sdr_resample(sdr_ctx* c, const float* x, int64_t n, const double* b, int taps, int up, int down,
                 double* zi_inout, float* y) {
  CHECK_CTX(c);
  if (n < 0 || up < 1 || down < 1) return fail(SDR_EINVAL, "bad resampler sizes");
  if (taps < 1 || taps > SDR_MAX_RESAMPLE_TAPS)
    return fail(SDR_EINVAL, "taps=%d outside [1, %d]", taps, SDR_MAX_RESAMPLE_TAPS);
  if (n > 0 && (x == nullptr || y == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  TRY(set_dev(c));
  const int64_t M = ceil_div(n * up, down);
  float *dx, *dy;
  double* dz;
  const int Z = taps - 1;
  TRY(scratch(c, S_IN, sizeof(float) * (size_t)n, (void**)&dx));
  TRY(scratch(c, S_OUT, sizeof(float) * (size_t)M, (void**)&dy));
  TRY(scratch(c, S_STATE, sizeof(double) * 2 * (size_t)(Z + 1), (void**)&dz));
  TRY(h2d(c, dx, x, sizeof(float) * n));
  if (zi_inout) TRY(h2d(c, dz, zi_inout, sizeof(double) * Z));
  TRY(sdr_resample_dev(c, dx, n, b, taps, up, down, zi_inout ? dz : nullptr,
                       zi_inout ? dz + Z + 1 : nullptr, dy));
  TRY(d2h(c, y, dy, sizeof(float) * M));
  if (zi_inout) TRY(d2h(c, zi_inout, dz + Z + 1, sizeof(double) * Z));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SDR_OK;
}

int sdr_fm_demod(sdr_ctx* c, const float* I, const float* Q, int64_t n, double* prev_phase,
                 float* out) {
  CHECK_CTX(c);
  if (n < 0) return fail(SDR_EINVAL, "negative size");
  if (n > 0 && (I == nullptr || Q == nullptr || out == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  TRY(set_dev(c));
  float *dI, *dO;
  double* dp;
  TRY(scratch(c, S_IN, sizeof(float) * 2 * (size_t)n, (void**)&dI));
  TRY(scratch(c, S_OUT, sizeof(float) * (size_t)n, (void**)&dO));
  TRY(scratch(c, S_STATE, sizeof(double), (void**)&dp));
  TRY(h2d(c, dI, I, sizeof(float) * n));
  TRY(h2d(c, dI + n, Q, sizeof(float) * n));
  const double ph0 = prev_phase ? *prev_phase : 0.0;
  TRY(h2d(c, dp, &ph0, sizeof(double)));
  TRY(sdr_fm_demod_dev(c, dI, dI + n, n, n, 1, dp, dO, n));
  TRY(d2h(c, out, dO, sizeof(float) * n));
  double ph1 = ph0;
  TRY(d2h(c, &ph1, dp, sizeof(double)));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (prev_phase) *prev_phase = ph1;
  return SDR_OK;
}

int sdr_pll(sdr_ctx* c, const float* in, int64_t n, double freq, double fs, double nco_scale,
            double phase_adj, double norm_bw, double* state6, float* nco_i, float* nco_q) {
  CHECK_CTX(c);
  if (n < 0) return fail(SDR_EINVAL, "negative size");
  if (state6 == nullptr || nco_i == nullptr || (n > 0 && in == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  TRY(set_dev(c));
  float *dx, *dO;
  double* ds;
  TRY(scratch(c, S_IN, sizeof(float) * (size_t)(n + 1), (void**)&dx));
  TRY(scratch(c, S_OUT, sizeof(float) * 2 * (size_t)(n + 1), (void**)&dO));
  TRY(scratch(c, S_STATE, sizeof(double) * 6, (void**)&ds));
  TRY(h2d(c, dx, in, sizeof(float) * n));
  TRY(h2d(c, ds, state6, sizeof(double) * 6));
  TRY(sdr_pll_dev(c, dx, n, n, 1, freq, fs, nco_scale, phase_adj, norm_bw, ds, dO,
                  nco_q ? dO + (n + 1) : nullptr, n + 1));
  TRY(d2h(c, nco_i, dO, sizeof(float) * (n + 1)));
  if (nco_q) TRY(d2h(c, nco_q, dO + (n + 1), sizeof(float) * (n + 1)));
  TRY(d2h(c, state6, ds, sizeof(double) * 6));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SDR_OK;
}

// ---- spectral diagnostics ------------------------------------------
int sdr_psd_dev(sdr_ctx* c, const void* x, int dtype, int64_t n, int nfft, double fs, double* psd) {
  CHECK_CTX(c);
  if (n < 0) return fail(SDR_EINVAL, "negative size");
  if (dtype != SDR_REAL_F32 && dtype != SDR_REAL_F64) return fail(SDR_EINVAL, "dtype %d", dtype);
  if (nfft < 2 || nfft > SDR_PSD_MAX_NFFT || (nfft & (nfft - 1)))
    return fail(SDR_EUNSUPPORTED, "nfft=%d: a power of two in [2, %d]", nfft, SDR_PSD_MAX_NFFT);
  if (psd == nullptr || (n >= nfft && x == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  TRY(set_dev(c));
  const int64_t nseg = n / nfft;
  const int half = nfft / 2;
  const int64_t nch = sdr_psd_chunks(nseg);
  void* ws;
  TRY(scratch(c, S_PSD, sizeof(double) * (size_t)((nseg + nch) * half) + 64, &ws));
  double* seg_db = static_cast<double*>(ws);
  double* part = seg_db + nseg * half;
  int* flag = reinterpret_cast<int*>(part + nch * half);
  HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), c->stream));
  int logn = 0;
  while ((1 << logn) < nfft) ++logn;
  HIP_TRY(sdr_launch_psd(x, dtype == SDR_REAL_F64, n, logn, fs, seg_db, part, psd, flag, c->stream));
  int zero = 0;
  HIP_TRY(hipMemcpyAsync(&zero, flag, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (zero) return fail(SDR_EDOMAIN, "a bin with zero power: log10(0) (model/fmSupportLib.py:121 raises)");
  return SDR_OK;
}

int sdr_psd(sdr_ctx* c, const double* x, int64_t n, int nfft, double fs, double* psd) {
  CHECK_CTX(c);
  if (n < 0) return fail(SDR_EINVAL, "negative size");
  if (psd == nullptr || (n > 0 && x == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  if (nfft < 2 || nfft > SDR_PSD_MAX_NFFT || (nfft & (nfft - 1)))
    return fail(SDR_EUNSUPPORTED, "nfft=%d: a power of two in [2, %d]", nfft, SDR_PSD_MAX_NFFT);
  TRY(set_dev(c));
  const int64_t used = n / nfft * nfft;
  double *dx, *dp;
  TRY(scratch(c, S_IN, sizeof(double) * (size_t)used, (void**)&dx));
  TRY(scratch(c, S_OUT, sizeof(double) * (size_t)(nfft / 2), (void**)&dp));
  TRY(h2d(c, dx, x, sizeof(double) * (size_t)used));
  TRY(sdr_psd_dev(c, dx, SDR_REAL_F64, used, nfft, fs, dp));
  TRY(d2h(c, psd, dp, sizeof(double) * (size_t)(nfft / 2)));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SDR_OK;
}

int sdr_dft(sdr_ctx* c, const double* x, int64_t n, double* X) {
  CHECK_CTX(c);
  if (n < 0 || n > SDR_DFT_MAX_N) return fail(SDR_EINVAL, "n=%lld outside [0, %d]", (long long)n, SDR_DFT_MAX_N);
  if (n > 0 && (x == nullptr || X == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  if (n == 0) return SDR_OK;
  TRY(set_dev(c));
  double *dx, *dX;
  TRY(scratch(c, S_IN, sizeof(double) * (size_t)n, (void**)&dx));
  TRY(scratch(c, S_OUT, sizeof(double) * 2 * (size_t)n, (void**)&dX));
  TRY(h2d(c, dx, x, sizeof(double) * (size_t)n));
  HIP_TRY(sdr_launch_dft(dx, n, dX, c->stream));
  TRY(d2h(c, X, dX, sizeof(double) * 2 * (size_t)n));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return SDR_OK;
}

int sdr_mono_block(sdr_ctx* c, const void* iq, int iq_dtype, int64_t n, const double* rf_b,
                   int rf_taps, int rf_decim, double* zi_i, double* zi_q, double* prev_phase,
                   const double* audio_b, int audio_taps, int audio_decim, double* audio_zi,
                   float* demod_out, float* audio_out) {
  CHECK_CTX(c);
  if (n < 0) return fail(SDR_EINVAL, "negative size");
  if (iq_dtype != SDR_IQ_F32 && iq_dtype != SDR_IQ_U8) return fail(SDR_EINVAL, "iq_dtype %d", iq_dtype);
  if (rf_taps < 1 || rf_taps > SDR_MAX_TAPS || audio_taps < 1 || audio_taps > SDR_MAX_TAPS)
    return fail(SDR_EINVAL, "taps outside [1, %d]", SDR_MAX_TAPS);
  if (rf_decim < 1 || audio_decim < 1) return fail(SDR_EINVAL, "decimation < 1");
  if ((zi_i == nullptr) != (zi_q == nullptr)) return fail(SDR_EINVAL, "zi_i/zi_q must both be set or NULL");
  if (n > 0 && (iq == nullptr || audio_out == nullptr)) return fail(SDR_EINVAL, "NULL buffer");
  TRY(set_dev(c));
  const int64_t M = ceil_div(n, rf_decim);
  const int64_t A = ceil_div(M, audio_decim);
  const size_t in_bytes = (size_t)n * (iq_dtype == SDR_IQ_U8 ? 2 : 8);
  void* d_iq;
  float *d_dm, *d_au;
  double* d_st;
  TRY(scratch(c, S_IN, in_bytes, &d_iq));
  TRY(scratch(c, S_OUT, sizeof(float) * (size_t)(M + 4), (void**)&d_dm));
  TRY(scratch(c, S_OUT2, sizeof(float) * (size_t)(A + 4), (void**)&d_au));
  const int Z = rf_taps - 1, ZA = audio_taps - 1;
  TRY(scratch(c, S_STATE, sizeof(double) * (4 * (size_t)Z + 2 * (size_t)ZA + 2), (void**)&d_st));
  double *dzi = d_st, *dzq = d_st + Z, *dfi = d_st + 2 * Z, *dfq = d_st + 3 * Z;
  double *dza = d_st + 4 * Z, *dfa = dza + ZA, *dph = dfa + ZA;
  TRY(h2d(c, d_iq, iq, in_bytes));
  if (zi_i) {
    TRY(h2d(c, dzi, zi_i, sizeof(double) * Z));
    TRY(h2d(c, dzq, zi_q, sizeof(double) * Z));
  }
  if (audio_zi) TRY(h2d(c, dza, audio_zi, sizeof(double) * ZA));
  const double ph0 = prev_phase ? *prev_phase : 0.0;
  TRY(h2d(c, dph, &ph0, sizeof(double)));
  TRY(sdr_rf_frontend_dev(c, d_iq, iq_dtype, n, n, 0, 1, rf_b, rf_taps, rf_decim,
                          zi_i ? dzi : nullptr, zi_i ? dzq : nullptr, Z, zi_i ? dfi : nullptr,
                          zi_i ? dfq : nullptr, dph, d_dm, M, nullptr, nullptr));
  TRY(sdr_fir_dev(c, d_dm, nullptr, 1.f, SDR_PRE_NONE, M, M, 0, 1, audio_b, audio_taps, audio_decim,
                  audio_zi ? dza : nullptr, ZA, audio_zi ? dfa : nullptr, d_au, A));
  TRY(d2h(c, audio_out, d_au, sizeof(float) * A));
  if (demod_out) TRY(d2h(c, demod_out, d_dm, sizeof(float) * M));
  if (zi_i) {
    TRY(d2h(c, zi_i, dfi, sizeof(double) * Z));
    TRY(d2h(c, zi_q, dfq, sizeof(double) * Z));
  }
  if (audio_zi) TRY(d2h(c, audio_zi, dfa, sizeof(double) * ZA));
  double ph1 = ph0;
  TRY(d2h(c, &ph1, dph, sizeof(double)));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (prev_phase) *prev_phase = ph1;
  return SDR_OK;
}

// ---- RDS link layer (host side) --------------------------------
// model/fmRDSblock.py:207-346: clock and data recovery (every 24th RRC sample from a
// carried offset), Manchester decoding of symbol pairs, differential decoding, and the
// syndrome scan of every 26-bit window with the in-frame / false-positive rule.  Bit
// level, sequential and a few hundred bits per block: CPU code.  The one deviation: a tie
// in the block-0 screening (where the reference's start_pos is unbound) takes 0.
}  // extern "C"

struct sdr_rds_link {
  int64_t block_count = 0, int_offset = 0, printposition = 0, last_position = -1;
  int start_pos = 0, front_bit = 0, prebit = 0;
  int resync_after = 0, bad_sync = 0;     // C++ frame_thread re-sync rule (0: off, as the Python model)
  double lonely_bit = 0.0;
  std::vector<uint8_t> prev_sync_bits;
};

namespace {
// parity matrix H (26 x 10), model/fmRDSblock.py:49, one row per bit as 10-bit masks (bit i = column i)
constexpr uint8_t kRdsH[26][10] = {
    {1,0,0,0,0,0,0,0,0,0},{0,1,0,0,0,0,0,0,0,0},{0,0,1,0,0,0,0,0,0,0},{0,0,0,1,0,0,0,0,0,0},
    {0,0,0,0,1,0,0,0,0,0},{0,0,0,0,0,1,0,0,0,0},{0,0,0,0,0,0,1,0,0,0},{0,0,0,0,0,0,0,1,0,0},
    {0,0,0,0,0,0,0,0,1,0},{0,0,0,0,0,0,0,0,0,1},{1,0,1,1,0,1,1,1,0,0},{0,1,0,1,1,0,1,1,1,0},
    {0,0,1,0,1,1,0,1,1,1},{1,0,1,0,0,0,0,1,1,1},{1,1,1,0,0,1,1,1,1,1},{1,1,0,0,0,1,0,0,1,1},
    {1,1,0,1,0,1,0,1,0,1},{1,1,0,1,1,1,0,1,1,0},{0,1,1,0,1,1,1,0,1,1},{1,0,0,0,0,0,0,0,0,1},
    {1,1,1,1,0,1,1,1,0,0},{0,1,1,1,1,0,1,1,1,0},{0,0,1,1,1,1,0,1,1,1},{1,0,1,0,1,0,0,1,1,1},
    {1,1,1,0,0,0,1,1,1,1},{1,1,0,0,0,1,1,0,1,1}};
// syndromes A, B, C, D (model/fmRDSblock.py:300, :307, :314, :321)
constexpr uint8_t kRdsSyn[4][10] = {{1,1,1,1,0,1,1,0,0,0}, {1,1,1,1,0,1,0,1,0,0},
                                    {1,0,0,1,0,1,1,1,0,0}, {1,0,0,1,0,1,1,0,0,0}};
}  // namespace

extern "C" {

int sdr_rds_link_create(sdr_rds_link** out) {
  if (!out) return fail(SDR_EINVAL, "sdr_rds_link_create: out is NULL");
  *out = new (std::nothrow) sdr_rds_link();
  return *out ? SDR_OK : fail(SDR_ENOMEM, "sdr_rds_link_create: out of memory");
}

void sdr_rds_link_destroy(sdr_rds_link* l) { delete l; }

int sdr_rds_link_set_resync(sdr_rds_link* l, int after_bad_syncs) {
  if (!l || after_bad_syncs < 0) return fail(SDR_EINVAL, "sdr_rds_link_set_resync: bad arguments");
  l->resync_after = after_bad_syncs;
  return SDR_OK;
}

int sdr_rds_link_block(sdr_rds_link* l, const double* rrc_i, int64_t n, int64_t* events,
                       int64_t max_events, int64_t* n_events, double* symbols, int64_t max_symbols,
                       int64_t* n_symbols, uint8_t* bits, int64_t max_bits, int64_t* n_bits,
                       uint8_t* diff_out, int64_t max_diff, int64_t* n_diff) {
  if (!l || !rrc_i) return fail(SDR_EINVAL, "sdr_rds_link_block: NULL link or input");
  if (n < 24) return fail(SDR_EINVAL, "sdr_rds_link_block: block of %lld samples (< 24)", (long long)n);
  if (l->block_count == 0) {                                          // :208-209 first index of the max
    int64_t best = 0;
    for (int64_t k = 1; k < 24; ++k)
      if (rrc_i[k] > rrc_i[best]) best = k;
    for (int64_t k = 0; k < 24; ++k)
      if (std::isnan(rrc_i[k])) return fail(SDR_EINVAL, "sdr_rds_link_block: NaN in the first 24 samples");
    l->int_offset = best;
  }
  const int64_t io = l->int_offset;
  if (io >= n) return fail(SDR_EINVAL, "sdr_rds_link_block: symbol offset %lld beyond the block", (long long)io);
  std::vector<double> s;                                              // :216
  for (int64_t k = io; k < n; k += 24) s.push_back(rrc_i[k]);
  const int64_t ns = (int64_t)s.size();
  {                                                                   // :219 value search
    int64_t j = -1;
    for (int64_t k = 0; k < 24 && j < 0; ++k)
      if (rrc_i[n - 24 + k] == s.back()) j = k;
    if (j < 0) return fail(SDR_EINVAL, "sdr_rds_link_block: last symbol not in the last 24 samples");
    l->int_offset = 24 - j;
  }
  if (l->block_count == 0) {                                          // :233-249
    int64_t c0 = 0, c1 = 0;
    for (int64_t m = 0; m < ns / 4; ++m) {
      if ((s[2 * m] > 0 && s[2 * m + 1] > 0) || (s[2 * m] < 0 && s[2 * m + 1] < 0)) ++c0;
      else if ((s[2 * m + 1] > 0 && s[2 * m + 2] > 0) || (s[2 * m + 1] < 0 && s[2 * m + 2] < 0)) ++c1;
    }
    l->start_pos = c0 > c1 ? 1 : 0;
  }
  const int sp = l->start_pos;
  std::vector<uint8_t> b((size_t)std::max<int64_t>(ns / 2 - sp, 0), 0);   // :251
  if (sp == 1 && l->block_count != 0) {                               // :255-259
    if (l->lonely_bit > s[0]) l->front_bit = 1;
    else if (l->lonely_bit < s[0]) l->front_bit = 0;
  }
  for (int64_t k = 0; k < (int64_t)b.size(); ++k) {                   // :261-269
    if (sp + 2 * k + 1 > ns - 1) break;
    if (s[2 * k + sp] > s[2 * k + 1 + sp]) b[k] = 1;
    else if (s[2 * k + sp] < s[2 * k + 1 + sp]) b[k] = 0;
  }
  if (sp == 1) {                                                      // :271-276
    b.insert(b.begin(), (uint8_t)l->front_bit);
    l->lonely_bit = s.back();
  }
  if (b.empty()) return fail(SDR_EINVAL, "sdr_rds_link_block: no bits in the block");
  int64_t off = 0;
  if (l->block_count == 0) {                                          // :280-284
    l->prebit = b[0];
    off = 1;
  }
  std::vector<uint8_t> d(l->block_count != 0 ? l->prev_sync_bits : std::vector<uint8_t>());   // :295-296
  for (int64_t t = 0; t + off < (int64_t)b.size(); ++t) {             // :286-289
    d.push_back((uint8_t)(l->prebit ^ b[t + off]));
    l->prebit = b[t + off];
  }
  l->prebit = b.back();                                               // :291
  if (d.size() < 26) return fail(SDR_EINVAL, "sdr_rds_link_block: %zu bits to scan (< 26)", d.size());
  int64_t ne = 0;
  int64_t position = 0;
  for (;;) {                                                          // :299-341
    uint8_t syn[10] = {0};
    for (int i = 0; i < 10; ++i)
      for (int j = 0; j < 26; ++j) syn[i] ^= (uint8_t)(d[position + j] & kRdsH[j][i]);
    for (int typ = 0; typ < 4; ++typ) {
      if (std::memcmp(syn, kRdsSyn[typ], 10) != 0) continue;
      const int64_t pp = l->printposition;
      const bool ok = l->last_position == -1 || pp - l->last_position == 26;
      if (ok) l->last_position = pp;
      if (events && ne < max_events) {
        events[3 * ne] = typ;
        events[3 * ne + 1] = pp;
        events[3 * ne + 2] = ok ? 1 : 0;
      }
      ++ne;
      l->bad_sync = ok ? 0 : l->bad_sync + 1;
      break;
    }
    if (l->resync_after > 0 && l->bad_sync > l->resync_after) {   // src/fm_radio.cpp:697-704
      if (events && ne < max_events) {
        events[3 * ne] = SDR_RDS_RESYNC;
        events[3 * ne + 1] = l->printposition;
        events[3 * ne + 2] = 0;
      }
      ++ne;
      l->bad_sync = 0;
      l->last_position = -1;
    }
    ++position;
    if (position + 26 > (int64_t)d.size() - 1) break;
    ++l->printposition;
  }
  l->prev_sync_bits.assign(d.begin() + (position - 1), d.end());      // :343
  ++l->block_count;
  if (n_events) *n_events = ne;
  if (n_symbols) *n_symbols = ns;
  if (n_bits) *n_bits = (int64_t)b.size();
  if (n_diff) *n_diff = (int64_t)d.size();
  if (events && ne > max_events) return fail(SDR_EINVAL, "sdr_rds_link_block: %lld events > max %lld", (long long)ne, (long long)max_events);
  if (symbols) {
    if (ns > max_symbols) return fail(SDR_EINVAL, "sdr_rds_link_block: symbols buffer too small");
    std::copy(s.begin(), s.end(), symbols);
  }
  if (bits) {
    if ((int64_t)b.size() > max_bits) return fail(SDR_EINVAL, "sdr_rds_link_block: bits buffer too small");
    std::copy(b.begin(), b.end(), bits);
  }
  if (diff_out) {
    if ((int64_t)d.size() > max_diff) return fail(SDR_EINVAL, "sdr_rds_link_block: diff buffer too small");
    std::copy(d.begin(), d.end(), diff_out);
  }
  return SDR_OK;
}

}  // extern "C"
