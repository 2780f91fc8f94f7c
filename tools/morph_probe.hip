// Tuning aid (not product): morph the pipeline probe (tools/pipe_probe.hip, pipe_w<0>:
// 2 LDS slots per wave, LDS-DMA of the next tile before the wait, FIR-shaped compute, no
// stores) into the product fe_ring_kernel<101,false> one feature at a time, all in one
// process, to find where the product loses time.  V bits:
//   1 the product FIR (fe_fir_tile<101,10,3,12>, taps from the kernarg TapsF32)
//   2 the product fast epilogue (atan2, DPP predecessor, carry, wrap count)
//   4 deferred outputs (OutQ3<36> push per tile, burst at the end of the run)
//   8 static __shared__ ring[2][2560] instead of dynamic LDS
//  16 the product's per-tile bookkeeping (int64 tile position, kind checks)
#include <functional>
#include <vector>

#include "../real-time-software-defined-radio_amd/csrc/fe.hip"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace {
constexpr int MNEWC = 15;
constexpr int MTP = 51;

template <int C>
__device__ __forceinline__ void probe_fir(const f2v* buf, int lane, const f2v (&tp)[MTP], float (&ai)[3], float (&aq)[3]) {
  f2v acc[3] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}, f2v{0.f, 0.f}};
  f2v acc2[3] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}, f2v{0.f, 0.f}};
  constexpr int PF = 12;
  const f2v* win = buf + 30 * lane + 10;
  f4v qb[C];
  static_for<0, PF>([&](auto I) { qb[I] = lds_read_b128<16 * I>(win); });
  lds_wait<PF - 1>(qb[0]);
  static_for<0, C>([&](auto I) {
    constexpr int ip = I;
    if constexpr (ip + PF < C) qb[ip + PF] = lds_read_b128<16 * (ip + PF)>(win);
    const f4v q = qb[ip];
    pk_fma_bcast<false>(acc[0], tp[(ip * 2) % MTP], f2v{q.x, q.y});
    pk_fma_bcast<true>(acc2[0], tp[(ip * 2 + 1) % MTP], f2v{q.z, q.w});
    pk_fma_bcast<false>(acc[1], tp[(ip * 2 + 7) % MTP], f2v{q.x, q.y});
    pk_fma_bcast<true>(acc2[1], tp[(ip * 2 + 9) % MTP], f2v{q.z, q.w});
    pk_fma_bcast<false>(acc[2], tp[(ip * 2 + 13) % MTP], f2v{q.x, q.y});
    if constexpr (ip + 1 < C) {
      constexpr int issued = (ip + PF + 1 < C) ? ip + PF + 1 : C;
      lds_wait<issued - (ip + 2)>(qb[ip + 1]);
    }
  });
  for (int r = 0; r < 3; ++r) { const f2v t = acc[r] + acc2[r]; ai[r] = t.x; aq[r] = t.y; }
}

template <int V>
__global__ __launch_bounds__(64) void morph(const float* __restrict__ in, int64_t ntiles, float* out, TapsF32 taps,
                                            int64_t n) {
  extern __shared__ __attribute__((aligned(16))) f2v dring[];
  __shared__ __attribute__((aligned(16))) f2v sring[(V & 8) ? 2 : 1][(V & 8) ? 2560 : 1];
  f2v* ring = (V & 8) ? &sring[0][0] : dring;
  constexpr int LS = (V & 8) ? 2560 : 2048;
  const int lane = threadIdx.x;
  const int64_t g0 = (int64_t)blockIdx.x * ntiles / gridDim.x, g1 = ((int64_t)blockIdx.x + 1) * ntiles / gridDim.x;
  const int n_ = (int)(g1 - g0);
  if (n_ <= 0) return;
  f2v tp[MTP];
#pragma unroll
  for (int j = 0; j < MTP; ++j)
    tp[j] = (V & 1) ? f2v{taps.h[2 * j], (2 * j + 1 < 101) ? taps.h[2 * j + 1] : 0.f} : f2v{1e-3f * j, 2e-3f * j};
#pragma unroll
  for (int j = 0; j < MTP; ++j) asm volatile("" : "+v"(tp[j]));
  const unsigned voff = 16u * lane;
  auto gnew = [&](int64_t t) { return reinterpret_cast<const char*>(in + t * 3840); };
  int issued = 0, mk[2] = {0, 0};
  auto issue_new = [&](int64_t t, int slot) {
    const char* g = gnew(t);
    const unsigned lb = lds_addr_of(ring + slot * LS) + 1024;
    static_for<0, 4>([&](auto Q) {
      constexpr int c = 4 * Q;
      constexpr int k = (MNEWC - c) < 4 ? (MNEWC - c) : 4;
      glds16x<k>(voff, g + 1024 * c, lb + 1024 * c);
    });
    issued += MNEWC;
  };
  glds16x<1>(voff, gnew(g0) - 1024, lds_addr_of(ring));
  issued += 1;
  issue_new(g0, 0);
  mk[0] = issued;
  OutQ3<36> oq;
  int qn = 0;
  float carry = 0.f;
  int wacc = 0;
  float sink = 0.f;
  int s = 0, i = (int)g0;
  int64_t nl = (int64_t)1920 * g0 - 110;
  const int64_t M = n / 10;
  for (int u = 0; u < n_; ++u) {
    const int slot = u & 1;
    if constexpr (V & 16) {
      // the product's per-tile position / kind bookkeeping (results feed a sink)
      int s1 = s, i1 = i + 1;
      if (i1 == 0x7fffffff) { i1 = 0; ++s1; }
      const int64_t nl1 = (s1 == s) ? nl + 1920 : -110;
      const bool halo = nl1 + 128 >= 0 && nl1 + 2048 <= n;
      const bool fast = i >= 1 && (int64_t)192 * i + 192 < M;
      sink += (halo ? 1.f : 0.f) + (fast ? 1.f : 0.f);
      s = s1; i = i1; nl = nl1;
    }
    if (u + 1 < n_) { issue_new(g0 + u + 1, slot ^ 1); if (slot) mk[0] = issued; else mk[1] = issued; }
    wait_vm(issued - (slot ? mk[1] : mk[0]));
    const f2v* buf = ring + slot * LS;
    f4v h = lds_read_b128<0>(buf + MNEWC * 128 + 2 * lane);
    float ai[3], aq[3];
    if constexpr (V & 1) {
      fe_fir_tile<101, 10, 3, 12>(buf, lane, tp, ai, aq);
    } else {
      probe_fir<61>(buf, lane, tp, ai, aq);
    }
    lds_wait<0>(h);
    if (u + 1 < n_) lds_write_b128(ring + (slot ^ 1) * LS + 2 * lane, h);
    float d[3];
    if constexpr (V & 2) {
      float phi[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) phi[r] = fast_atan2f(aq[r], ai[r]);
      const float from_left = __int_as_float(__builtin_amdgcn_update_dpp(
          0, __float_as_int(phi[2]), 0x138 /*wave_shr:1*/, 0xf, 0xf, false));
      float prev = (lane == 0) ? carry : from_left;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        float dd = phi[r] - prev;
        if (dd > kPiF) { dd -= k2PiF; wacc -= 1; }
        else if (dd < -kPiF) { dd += k2PiF; wacc += 1; }
        d[r] = dd;
        prev = phi[r];
      }
      carry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[2]), 63));
    } else {
      for (int r = 0; r < 3; ++r) d[r] = fast_atan2f(aq[r], ai[r] + 1e-3f * lane);
    }
    if constexpr (V & 4) {
      if (qn == 36) { issued += oq.flush(out + (g0 + u - 36) * 192 + 3 * lane, 192, 36); qn = 0; }
      oq.put(qn, d[0], d[1], d[2]);
      ++qn;
    } else {
      sink += d[0] + d[1] + d[2];
    }
  }
  if constexpr (V & 4) oq.flush(out + (g0 + n_ - qn) * 192 + 3 * lane, 192, qn);
  if (sink == 1234.5f || wacc == 12345) out[0] = sink + carry;
}
}  // namespace

int main() {
  const int64_t n = 64LL * 1024000;
  const int64_t bytes = n * 8;
  const int64_t ntiles = (bytes - 1024) / (MNEWC * 1024) - 1;
  std::vector<float> h(bytes / 4 + 65536 / 4);
  uint32_t x = 12345u; float ph = 0.f;
  for (size_t k = 0; k + 1 < h.size(); k += 2) {
    x = x * 1664525u + 1013904223u; ph += 1.5f * ((x >> 8) * (1.f / 16777216.f) - 0.5f);
    h[k] = 0.5f * cosf(ph); h[k + 1] = 0.5f * sinf(ph);
  }
  float *in, *out;
  CK(hipMalloc(&in, bytes + 65536)); CK(hipMalloc(&out, (ntiles + 8) * 192 * 4 + 65536));
  CK(hipMemcpy(in, h.data(), bytes + 65536, hipMemcpyHostToDevice));
  in += 256;
  TapsF32 taps{}; for (int k = 0; k < 101; ++k) taps.h[k] = 0.01f * sinf(0.1f * k);
  hipStream_t st; CK(hipStreamCreate(&st)); hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  struct Var { const char* nm; std::function<void()> go; };
  std::vector<Var> vs;
#define MV(V) vs.push_back({"morph V=" #V, [=] { \
    hipLaunchKernelGGL((morph<V>), dim3(1024), dim3(64), (V & 8) ? 0 : 40896, st, in, ntiles - 1, out, taps, n); }});
  MV(0) MV(1) MV(2) MV(4) MV(8) MV(16) MV(3) MV(7) MV(15) MV(31)
  for (auto& v : vs) v.go();
  CK(hipStreamSynchronize(st)); CK(hipGetLastError());
  const bool quick = getenv("AB_QUICK") != nullptr;   // counter runs: few launches
  for (int i = 0; i < (quick ? 0 : 3000); ++i) vs[0].go();
  for (int pass = quick ? 1 : 0; pass < 2; ++pass)
    for (auto& v : vs) {
      for (int i = 0; i < (quick ? 5 : 200); ++i) v.go();
      CK(hipEventRecord(a, st));
      for (int i = 0; i < (quick ? 5 : 50); ++i) v.go();
      CK(hipEventRecord(b, st)); CK(hipEventSynchronize(b)); CK(hipGetLastError());
      float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 50;
      printf("pass %d  %-20s %8.2f us\n", pass, v.nm, ms * 1e3);
      fflush(stdout);
    }
  return 0;
}
