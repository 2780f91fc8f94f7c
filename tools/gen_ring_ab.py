#!/usr/bin/env python3
"""Tuning aid (not product): generate tools/_ring_ab.hip, an ablation copy of the product
fe_ring_kernel timed beside the product launchers of this tree and those of round 1 (built
from git into tools/_fe_r01.hip with renamed entry points).

KN bits: 1 trivial fast epilogue, 2 no deferred-output queue (outputs dropped), 4 no halo
copy, 8 fixed steady vmcnt wait, 16 taps from constants, 32 FUSED: no audio FIR,
64 FUSED: no history writes, 128 FUSED: no warm-up tile (wrong audio at run starts; timing), 256 FUSED: no run-end
audio block (timing).

build:  python3 tools/gen_ring_ab.py && cd tools && \
        hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-inline-asm _ring_ab.hip _fe_r01.hip -o ring_ab
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R01_COMMIT = "bf204f6"
src = open(os.path.join(ROOT, "real-time-software-defined-radio_amd", "csrc", "fe.hip")).read()
a = src.index("template <int T, bool FUSED>\n__global__ __launch_bounds__(64) void fe_ring_kernel")
b = src.index("// lfilter final state zf", a)
k = src[a:b]
k = k.replace("template <int T, bool FUSED>\n__global__ __launch_bounds__(64) void fe_ring_kernel(",
              "template <int T, bool FUSED, int KN>\n__global__ __launch_bounds__(64) void ring_ab(")
reps = [
    ("      float prev = (lane == 0) ? carry : from_left;\n",
     "      float prev = (lane == 0) ? carry : from_left;\n"
     "      if constexpr (KN & 1) { for (int r = 0; r < R; ++r) d[r] = ai[r] + aq[r]; } else {\n"),
    ("      carry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[R - 1]), 63));\n",
     "      }\n      carry = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(phi[R - 1]), 63));\n"),
    ("      if constexpr (!FUSED) q_push(i, d[0], d[1], d[2]);",
     "      if constexpr (!FUSED && !(KN & 2)) q_push(i, d[0], d[1], d[2]);\n"
     "      if constexpr (KN & 2) { if (d[0] == 1234.5f) p.demod[0] = d[1]; }"),
    ("    if (kind1 == K_HALO) {\n      h0 =", "    if (!(KN & 4) && kind1 == K_HALO) {\n      h0 ="),
    ("    if (kind1 == K_HALO) {\n      f2v* nb", "    if (!(KN & 4) && kind1 == K_HALO) {\n      f2v* nb"),
    ("        fir_audio_tile<T, 2, 2, OFF>(buf, lane, tp, ai, aq, aw_lane, ptab, o0, o1, o2);",
     "        if constexpr (KN & 32) { fe_fir_tile<T, D, R, PF, OFF>(buf, lane, tp, ai, aq); o0 = o1 = o2 = ai[0]; }\n"
     "        else fir_audio_tile<T, 2, 2, OFF>(buf, lane, tp, ai, aq, aw_lane, ptab, o0, o1, o2);"),
    ("      q_push(q, o0, o1, o2);\n      return false;",
     "      if constexpr (!(KN & 2)) q_push(q, o0, o1, o2);\n      return false;"),
    ("      dh_write(i, warm, d);", "      if constexpr (!(KN & 64)) dh_write(i, warm, d);"),
    ("    mid = i > 0;\n", "    mid = (KN & 128) ? false : i > 0;\n"),
    ("          audio_block3(aw_lane, ptab, o0, o1, o2);",
     "          if constexpr (KN & 256) { o0 = o1 = o2 = aw_lane[0]; } else audio_block3(aw_lane, ptab, o0, o1, o2);"),
    ("      wait_vm(issued - mark);",
     "      if constexpr (KN & 8) { if (issued - mark == 15) asm volatile(\"s_waitcnt vmcnt(15)\" ::: \"memory\");"
     " else asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\"); }\n      else wait_vm(issued - mark);"),
    ("  for (int j = 0; j < TP; ++j) tp[j] = f2v{taps.h[2 * j], (2 * j + 1 < T) ? taps.h[2 * j + 1] : 0.f};",
     "  for (int j = 0; j < TP; ++j) tp[j] = (KN & 16) ? f2v{1e-3f * j, 2e-3f * j} : "
     "f2v{taps.h[2 * j], (2 * j + 1 < T) ? taps.h[2 * j + 1] : 0.f};"),
]
for x, y in reps:
    if x in k:
        k = k.replace(x, y, 1)
    else:
        print("gen_ring_ab: knob site not found (skipped):", x.strip()[:70])

main = r'''
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
hipError_t r01_launch_fe(const FeLaunch& a, hipStream_t st);
hipError_t r01_launch_fe_mono(const FeLaunch& a, const float* ataps, int TA, int DA, float* audio,
                              int64_t audio_stride, hipStream_t st);
int main() {
  const int64_t n = 64LL * 1024000;
  std::vector<float> h(2 * n);
  uint32_t x = 12345u; float ph = 0.f;
  for (int64_t k = 0; k < n; ++k) {
    x = x * 1664525u + 1013904223u; ph += 1.5f * ((x >> 8) * (1.f / 16777216.f) - 0.5f);
    h[2 * k] = 0.5f * cosf(ph) + 0.01f * ((x & 255) - 127.5f) / 128.f; h[2 * k + 1] = 0.5f * sinf(ph);
  }
  float *iq, *dm, *au;
  CK(hipMalloc(&iq, 8 * n + 65536)); CK(hipMalloc(&dm, 4 * (n / 10) + 65536)); CK(hipMalloc(&au, 4 * (n / 50) + 65536));
  CK(hipMemcpy(iq, h.data(), 8 * n, hipMemcpyHostToDevice));
  TapsF32 taps{}; for (int k = 0; k < 101; ++k) taps.h[k] = 0.01f * sinf(0.1f * k);
  TapsF32 at{}; for (int k = 0; k < 151; ++k) at.h[k] = 0.006f * cosf(0.05f * k);
  float *tdev, *adev;
  CK(hipMalloc(&tdev, 4 * 256)); CK(hipMemcpy(tdev, taps.h, 4 * 256, hipMemcpyHostToDevice));
  CK(hipMalloc(&adev, 4 * 256)); CK(hipMemcpy(adev, at.h, 4 * 256, hipMemcpyHostToDevice));
  FeParams p{}; p.iq = iq; p.n = n; p.stride = n; p.nstreams = 1; p.taps_dev = tdev; p.demod = dm; p.out_stride = n / 10;
  RingArgs ra{}; ra.tps = (int)((n / 10 + 191) / 192); ra.total = ra.tps; p.tiles_per_stream = ra.tps;
  RingArgs rf = ra; rf.tps = 5 * (int)((n / 10 + 959) / 960); rf.total = rf.tps; rf.audio = au;
  rf.audio_stride = n / 50; rf.ataps = adev;
  FeParams pf = p; pf.tiles_per_stream = rf.tps;
  FeLaunch la{iq, n, n, 0, 1, tdev, &taps, 101, 10, 0, nullptr, nullptr, 0, nullptr, dm, n / 10, nullptr, nullptr,
              nullptr, nullptr};
  hipStream_t st; CK(hipStreamCreate(&st)); hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  struct V { const char* nm; std::function<void()> go; };
  std::vector<V> vs;
#define FE(NM, K) vs.push_back({NM, [=] { hipLaunchKernelGGL((ring_ab<101, false, K>), dim3(1024), dim3(64), 0, st, p, taps, ra); }});
#define FU(NM, K) vs.push_back({NM, [=] { hipLaunchKernelGGL((ring_ab<101, true, K>), dim3(1024), dim3(64), 0, st, pf, taps, rf); }});
  vs.push_back({"FE product (this tree)", [=] { CK(sdr_launch_fe(la, st)); }});
  vs.push_back({"FE r01 (slot)", [=] { CK(r01_launch_fe(la, st)); }});
  FE("FE KN=0", 0) FE("FE KN=2 no queue", 2) FE("FE KN=8 fixed wait", 8) FE("FE KN=10", 10) FE("FE KN=15", 15)
  vs.push_back({"FUSED product (this tree)", [=] { CK(sdr_launch_fe_mono(la, adev, 151, 5, au, n / 50, st)); }});
  vs.push_back({"FUSED r01 (ring)", [=] { CK(r01_launch_fe_mono(la, adev, 151, 5, au, n / 50, st)); }});
  FU("FUSED KN=0", 0) FU("FUSED KN=2 no queue", 2) FU("FUSED KN=8 fixed wait", 8) FU("FUSED KN=32 no audio", 32)
  FU("FUSED KN=64 no dh", 64) FU("FUSED KN=96", 96) FU("FUSED KN=1 trivial epi", 1) FU("FUSED KN=111", 111)
  FU("FUSED KN=128 no warm-up", 128) FU("FUSED KN=224 no warm/audio/dh", 224) FU("FUSED KN=239", 239)
  FU("FUSED KN=256 no run-end audio", 256) FU("FUSED KN=384 no warm-up/run-end", 384)
  const bool quick = getenv("AB_QUICK") != nullptr;   // counter runs: few launches
  for (auto& v : vs) v.go();
  CK(hipStreamSynchronize(st));
  for (int i = 0; i < (quick ? 0 : 3000); ++i) vs[0].go();
  for (int pass = quick ? 1 : 0; pass < 2; ++pass)
    for (auto& v : vs) {
      for (int i = 0; i < (quick ? 5 : 200); ++i) v.go();
      CK(hipEventRecord(a, st));
      for (int i = 0; i < (quick ? 5 : 50); ++i) v.go();
      CK(hipEventRecord(b, st)); CK(hipEventSynchronize(b)); CK(hipGetLastError());
      float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 50;
      printf("pass %d %-36s %8.2f us  %7.1f GB/s (8 B/sample in)\n", pass, v.nm, ms * 1e3, 8.0 * n / ms / 1e6);
      fflush(stdout);
    }
  return 0;
}
'''
out = ('#include <functional>\n#include "../real-time-software-defined-radio_amd/csrc/fe.hip"\n\nnamespace {\n'
       + k + '}  // namespace\n' + main)
open(os.path.join(ROOT, "tools", "_ring_ab.hip"), "w").write(out)

# round-1 kernels with renamed entry points (A/B baseline)
r01 = subprocess.run(["git", "-C", ROOT, "show", R01_COMMIT + ":real-time-software-defined-radio_amd/csrc/fe.hip"],
                     capture_output=True, text=True, check=True).stdout
for x, y in [("sdr_launch_fe_mono", "r01_launch_fe_mono"), ("sdr_launch_fe(", "r01_launch_fe("),
             ("sdr_launch_iq_zf", "r01_iq_zf"), ("sdr_launch_demod_state", "r01_demod_state"),
             ("sdr_launch_demod(", "r01_demod("), ("demod_state_kernel", "r01_demod_state_kernel"),
             ("demod_kernel", "r01_demod_kernel"), ("struct FeLaunch {", "struct FeLaunchR01 {"),
             ("const FeLaunch&", "const FeLaunchR01&")]:
    r01 = r01.replace(x, y)
r01 = r01.replace('#include "sdr_common.h"', '#include "../real-time-software-defined-radio_amd/csrc/sdr_launch.h"')
r01 += ("\nhipError_t r01_launch_fe(const FeLaunch& a, hipStream_t st) {\n"
        "  return r01_launch_fe(reinterpret_cast<const FeLaunchR01&>(a), st);\n}\n"
        "hipError_t r01_launch_fe_mono(const FeLaunch& a, const float* t, int TA, int DA, float* au, int64_t as,\n"
        "                              hipStream_t st) {\n"
        "  return r01_launch_fe_mono(reinterpret_cast<const FeLaunchR01&>(a), t, TA, DA, au, as, st);\n}\n")
open(os.path.join(ROOT, "tools", "_fe_r01.hip"), "w").write(r01)
