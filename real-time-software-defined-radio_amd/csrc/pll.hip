// PLL + NCO for gfx950 (stereo pilot recovery and RDS carrier recovery).
//
// Replaces model/fmPll.py:4-46 (block state: [integrator, phaseEst, feedbackI,
// feedbackQ, ncoOut[0], trigOffset]) and src/helper.cpp:13-57 (fmPLL).
// SURVEY §8a row a9.
//
// The loop is the only serial stage on the path, and one wave issues every instruction of
// it (an f64 op holds the SIMD ~8 cycles at wave64), so the step is issue-bound: what is
// not a function of the loop state is taken out of the loop.  Three launches per call:
//   1. pll_prep_kernel (parallel over samples): c_k = sel_k - w*(trigOffset + k), where
//      sel_k = 0 for x_k > 0 and pi for x_k < 0, and per 32-sample group a flag for a 0 or
//      NaN input (the general form's case).  For x != 0, atan2(-x sin th, x cos th) of the
//      previous step's angle th_{k-1} = w (trigOffset + k) + phaseEst_{k-1} is
//      wrap(sel_k - th_{k-1}) = wrap(c_k - phaseEst_{k-1}), reduced by a two-constant
//      Cody-Waite step.
//   2. pll_lanes_kernel: ONE LANE PER RECURRENCE.  A launch carries a job table (the
//      stereo pilot PLL and the RDS carrier PLL of every stream); each
//      wave runs one job for up to 64 streams, lane = stream.  Per step, in f64:
//        e_k   = wrap(c_k - phaseEst)                        (fmPll.py:24-27)
//        integ += Ki e_k ; phaseEst += Kp e_k + integ         (fmPll.py:29-31)
//      (6 f64 ops, 3 of them dependent: the wrap is 2 pi (fract(c'_k - phaseEst/2pi) - 1/2)
//      with c'_k = c_k/2pi + 1/2 from the prep kernel, and the loop filter is rewritten on
//      fract's output) and the lane stores phaseEst_k.  The first sample of a call (whose fI, fQ
//      come from the caller's state) and groups holding a 0 or NaN input take the literal
//      sincos + atan2 form, so signed zeros behave as in Python.  The lane also writes
//      ncoOut[0] / ncoOutQ[0] (the carried values) before the loop.
//   3. nco_jobs_kernel (parallel): th_k = 2 pi (freq/Fs) (trigOffset + k + 1) + phaseEst_k
//      (fmPll.py:33, Python's rounding), ncoOut[k+1] = cos(th_k*scale + adj),
//      ncoOutQ[k+1] = sin(th_k*scale + adj) (fmPll.py:36-37).
// All phase arithmetic is f64 (SURVEY §7 hard part 5: an fp32 NCO drifts).
//
// Before the loop kernel, pll_spec_kernel solves each recurrence of up to SDR_PLL_BLOCK_MAX
// samples in parallel (one workgroup per recurrence) and the loop kernel skips what it
// completed.  Longer calls (a device-resident span of many of the reference's blocks) are cut
// into pseudo-blocks, one workgroup each, whose start states are guessed by a warm-up and then
// chained exactly ("long calls", below).  How every recurrence was solved is counted in the
// context's device counters (sdr_pll_stats, include/sdr.h).
#include <stdlib.h>

#include <cmath>
#include <mutex>

#include "sdr_launch.h"
#include "sdr_nco.h"
#include "../../include/sdr.h"

using namespace sdrnco;

namespace {

// device counters (nullable): vector atomics on a plain global array
__device__ __forceinline__ void stat_add(unsigned long long* s, int k, unsigned long long v) {
  if (s != nullptr) atomicAdd(s + k, v);
}
__device__ __forceinline__ void stat_max(unsigned long long* s, int k, double v) {
  if (s != nullptr && v >= 0.0) atomicMax(s + k, (unsigned long long)__double_as_longlong(v));
}
// wave-aggregated: every lane of the wave calls it (uniform control flow); one atomic per wave
// for the lanes with `on` (thousands of lanes adding to one counter serialise at the L2)
__device__ __forceinline__ void stat_add_wave(unsigned long long* s, int k, bool on) {
  const uint64_t m = __ballot(on);
  if (s != nullptr && m != 0 && (threadIdx.x & 63) == __builtin_ctzll(m)) atomicAdd(s + k, (unsigned long long)__popcll(m));
}
__device__ __forceinline__ void stat_max_wave(unsigned long long* s, int k, bool on, double v) {
  double x = on ? v : -1.0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o, 64));
  if ((threadIdx.x & 63) == 0) stat_max(s, k, x);
}

// A call's end state from its last angle arg (fmPll.py:39-44): feedbackI/Q = cos/sin(arg) and
// ncoOut[-1] = cos(arg scale + adj), through the NCO kernels' reduction -- so the next call's
// ncoOut[0] is this call's last NCO value bit for bit, and a growing angle never takes the
// library's large-argument path.
__device__ __forceinline__ void end_trig(double arg, double scale, double adj, double* st) {
  double sv, cv;
  sincos_red<true>(reduce_2pi(arg), &sv, &cv);
  st[2] = cv;
  st[3] = sv;
  sincos_red<true>(reduce_2pi(arg * scale + adj), &sv, &cv);
  st[4] = cv;
}

// The loop's per-sample constant (pll_prep_kernel's, plain form): c_k = (sel_k - w (off + k)) / 2pi
// + 1/2, offk = off + k exactly; NaN for a 0 / NaN input.  Long calls compute it where it is
// used instead of storing a row of it.
// (r04: one rounding, fma(-offk, w / 2pi, 1/2 + sel_k / 2pi), where r03 rounded three times
// -- the same value to an ulp of |c_k|, the order of the reference's own rounding of its angle
// w (off + k + 1); every kernel forms c_k this way, so all agree bit for bit)
__device__ __forceinline__ double pll_c(float x, double w, double offk) {
  const double cv = fma(-offk, w * kInv2Pi, x > 0.f ? 0.5 : 1.0);
  return (x > 0.f || x < 0.f) ? cv : __builtin_nan("");
}

// The low byte of floor(t) (|t| < 2^51): t - fract(t) is floor(t) exactly, and adding 1.5 2^52
// puts that integer in the low word -- two f64 adds instead of a floor and a conversion that
// saturates beyond 2^31.  The solve records and compares the integers m_k by this byte (a
// guess and its check never disagree by a multiple of 256 turns).
__device__ __forceinline__ int8_t floor_byte(double t, double f) {
  const double u = (t - f) + 6755399441055744.0;
  return (int8_t)(__double2loint(u) & 0xff);
}

// Steps per group: the next group's inputs are loaded (registers) while this one runs,
// and the group's phases leave as 16-B stores.
constexpr int PG = 32;
// Recurrences per wave (P.lpw, chosen by the launcher): one per workgroup (pll_chunk_kernel,
// a recurrence wave + a loader wave) up to 128 recurrences -- 64 streams x 2 PLLs; C5 blocks:
// 8 streams 379 us, 64 streams 454 us -- and beyond that several per wave
// (pll_lanes_kernel: a wave's f64 step slows with its active lanes, 30 ns for one stream,
// 54 ns for 64).
constexpr int kMaxPllWaves = 128;

template <bool VEC>
__global__ __launch_bounds__(64) void pll_lanes_kernel(PllJobs P) {
#pragma clang fp contract(off)  // Python evaluates a*b + c with two roundings
  // one job per wave (a lane-varying job index into the kernarg table would copy the whole
  // table to scratch); lane = stream
  const int lpw = P.lpw;
  const int wpj = (P.nstreams + lpw - 1) / lpw;
  const int q = blockIdx.x / wpj;
  const int s = (blockIdx.x - q * wpj) * lpw + threadIdx.x;
  if ((int)threadIdx.x >= lpw || s >= P.nstreams) return;  // votes below run over the active lanes only
  const PllJob& J = P.j[q];
  struct {
    const float* in; double* th; const double* c; float* nco_i; float* nco_q;
  } L{J.in + (int64_t)s * J.in_stride, J.theta + (int64_t)s * J.th_stride, J.cbuf + (int64_t)s * J.c_stride,
      J.nco_i + (int64_t)s * J.out_stride, J.nco_q ? J.nco_q + (int64_t)s * J.out_stride : nullptr};
  if (P.n > 0 && L.c[0] == __builtin_inf()) return;      // solved by pll_spec_kernel
  const PllCfg cfg = J.cfg;
  double* st = J.state + (int64_t)s * 6;
  const int64_t n = P.n;
  double integ = st[0], phase = st[1], fI = st[2], fQ = st[3];
  const double off = st[5];
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  // ncoOut[0] = the carried value; ncoOutQ[0]: the reference leaves it uninitialised
  // (np.empty, fmPll.py:13); here sin(th_prev*scale + adj) with th_prev rebuilt from the
  // carried state (0 at stream start), the quadrature twin of ncoOut[0].
  L.nco_i[0] = (float)st[4];
  if (L.nco_q) L.nco_q[0] = (float)((off > 0.0) ? sin((w * off + phase) * cfg.scale + cfg.adj) : 0.0);
  double arg = 0.0;
  // One step of model/fmPll.py:23-41.  General form: the first sample of a call uses the
  // caller's (fI, fQ) literally, and an input of 0 or NaN takes atan2 on the products.
  auto general = [&](float xf, int64_t k, bool literal) {
    const double xv = (double)xf;
    double e;
    if (literal || !(xv > 0.0 || xv < 0.0)) {
      if (!literal) { fI = cos(arg); fQ = sin(arg); }
      e = atan2(xv * (-fQ), xv * fI);
    } else {
      e = reduce_2pi(xv > 0.0 ? -arg : kPi - arg);
      if (e <= -kPi) e += 2.0 * kPi;   // atan2 range is (-pi, pi]
    }
    integ = integ + cfg.ki * e;
    phase = phase + cfg.kp * e + integ;
    arg = w * ((off + (double)k) + 1.0) + phase;
  };
  // Fast step (x != 0): e = wrap(c_k - phaseEst) (atan2's (-pi, pi] differs only at e = -pi
  // exactly); the loop filter's updates as FMAs (fewer roundings than Python's: the f32
  // outputs cannot see the difference).  tools/pll_probe.hip, DESIGN.md §4.
  // c = (sel - w (off + k)) / 2pi + 1/2: t = d/2pi + 1/2 and e = 2pi (fract(t) - 1/2) = d -
  // 2pi round(d/2pi), in [-pi, pi); t's rounding (ulp of the accumulated angle) is the same
  // order as the rounding of the reference's own th = w (off + k + 1) + phaseEst.  With
  // f = fract(t): integ' = integ + Ki e and phaseEst' = phaseEst + integ + (Kp + Ki) e, so
  // phaseEst' = fma(2pi (Kp+Ki), f, S) with S = phaseEst + integ - pi (Kp+Ki) formed off the
  // chain: three dependent ops per step (t, fract, phaseEst'), six f64 ops in all.  V tracks
  // integ - pi (Kp+Ki).
  const double kA = k2Pi * cfg.ki, kB = kPi * cfg.ki;
  const double kC = k2Pi * (cfg.kp + cfg.ki), kD = kPi * (cfg.kp + cfg.ki);
  double V = 0.0;
  auto fast = [&](double c) {
    const double t = fma(-kInv2Pi, phase, c);
    const double f = __builtin_amdgcn_fract(t);
    const double S = phase + V;
    V = fma(kA, f, V - kB);
    phase = fma(kC, f, S);
  };
  const double* cr = L.c;
  auto load_group = [&](double (&v)[PG], int64_t k0) {
    if constexpr (VEC) {
#pragma unroll
      for (int i = 0; i < PG; i += 2) {
        const double2 f = *reinterpret_cast<const double2*>(cr + k0 + i);
        v[i] = f.x;
        v[i + 1] = f.y;
      }
    } else {
#pragma unroll
      for (int i = 0; i < PG; ++i) v[i] = cr[k0 + i];
    }
  };
  const int64_t ng = n / PG;
  double cur[PG], nxt[PG];
  double flag = 0.0, flag_n = 0.0;                 // group flags: 1.0 = a 0 / NaN input
  if (ng > 0) { load_group(cur, 0); flag = cr[n]; }
  for (int64_t g = 0; g < ng; ++g) {
    if (g + 1 < ng) { load_group(nxt, (g + 1) * PG); flag_n = cr[n + g + 1]; }
    // wave vote: the call's first group (literal first sample), or a 0 / NaN input
    if (__any(g == 0 || flag != 0.0)) {
      // rare: a rolled loop over the inputs in memory (unrolled, its atan2/sincos would spill)
      for (int i = 0; i < PG; ++i) {
        const int64_t k = g * PG + i;
        general(L.in[k], k, k == 0);
        L.th[k] = phase;
      }
    } else {
      double ph[PG];
      V = integ - kD;
#pragma unroll
      for (int i = 0; i < PG; ++i) {
        fast(cur[i]);
        ph[i] = phase;
      }
      integ = V + kD;
      arg = w * ((off + (double)(g * PG + PG - 1)) + 1.0) + phase;   // for a later general step
      double* tp = L.th + g * PG;
      if constexpr (VEC) {
#pragma unroll
        for (int i = 0; i < PG; i += 2) *reinterpret_cast<double2*>(tp + i) = make_double2(ph[i], ph[i + 1]);
      } else {
#pragma unroll
        for (int i = 0; i < PG; ++i) tp[i] = ph[i];
      }
    }
#pragma unroll
    for (int i = 0; i < PG; ++i) cur[i] = nxt[i];
    flag = flag_n;
  }
  for (int64_t k = ng * PG; k < n; ++k) {      // tail (< PG samples)
    general(L.in[k], k, k == 0);
    L.th[k] = phase;
  }
  L.th[n] = off;                                // the NCO kernel's trigOffset (st[5] changes below)
  if (n > 0) {
    st[0] = integ;
    st[1] = phase;
    end_trig(arg, cfg.scale, cfg.adj, st);
    st[5] = off + (double)n;
    stat_add(P.stats, SDR_PLL_ST_RECURRENCES, 1);
    stat_add(P.stats, SDR_PLL_ST_SEQUENTIAL, 1);
  }
}

// One recurrence per workgroup (P.lpw == 1): wave 0's lane 0 runs it, wave 1 feeds it.  A
// lone recurrence issues its 6 f64 ops in ~26 cycles per step (11 ns, tools/f64_probe.hip);
// fed by its own per-step 16-B loads it ran at ~30 ns -- vmcnt counts at most 63
// operations, so with a load and a store every two steps no more than ~2 groups of
// constants could be in flight against a ~1 us load latency -- and with its constants and
// phases staged through LDS by the same wave, at 67 cycles per step (a single wave's wide LDS
// stores run at half rate).  Here wave 1 brings the constants into an LDS ring by 64-lane
// LDS-DMA (128 steps = 1 KiB per instruction, NPF chunks ahead; it alone issues loads, so its
// vmcnt waits are exact), the waves meet at one raw s_barrier per chunk (no fence: the DMA
// stays in flight), and lane 0 reads each group's 32 constants in one LDS burst and stores
// its phases straight to HBM (stores only: it never waits on vmcnt).  Constants of 0 / NaN
// inputs are NaN (pll_prep_kernel): a fast group that meets one ends in a NaN phase and is
// redone in the general form from its checkpoint.
constexpr int CH = 128;     // steps per chunk (64 lanes x 16 B)
constexpr int NPF = 4;      // chunks of constants in flight

typedef double d2v __attribute__((ext_vector_type(2)));
// a group's 32 constants, read from LDS by hand in one burst and waited for once (left to
// itself the compiler read them 4 at a time, each batch waiting out the LDS latency)
template <int J = 0>
__device__ __forceinline__ void lds_group_rd(f4v (&c)[PG / 2], const double* src) {
  if constexpr (J < PG / 2) {
    c[J] = lds_read_b128<16 * J>(src);
    lds_group_rd<J + 1>(c, src);
  }
}
// ONE wait naming all 16 registers: per-register waits let the compiler sink them into the
// steps, and the next group's reads (ordered after the waits) then went out at the end of
// the group instead of its start
__device__ __forceinline__ void lds_group_wait(f4v (&c)[PG / 2]) {
  static_assert(PG / 2 == 16, "16 registers");
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]),
                 "+v"(c[8]), "+v"(c[9]), "+v"(c[10]), "+v"(c[11]), "+v"(c[12]), "+v"(c[13]), "+v"(c[14]),
                 "+v"(c[15]));
}
__device__ __forceinline__ double dbl(const f4v& v, int h) {
  const d2v d = __builtin_bit_cast(d2v, v);
  return h ? d.y : d.x;
}

__global__ __launch_bounds__(128) void pll_chunk_kernel(PllJobs P) {
#pragma clang fp contract(off)  // Python evaluates a*b + c with two roundings
  __shared__ __attribute__((aligned(16))) double cring[NPF][CH];
  const int q = blockIdx.x / P.nstreams;   // one stream per workgroup
  const int s = blockIdx.x - q * P.nstreams;
  const bool loader = threadIdx.x >= 64;
  const int lane = threadIdx.x & 63;
  const PllJob& J = P.j[q];
  const int64_t n = P.n;
  const int64_t nch = n / CH;
  const double* cr = J.cbuf + (int64_t)s * J.c_stride;
  if (n > 0 && cr[0] == __builtin_inf()) return;        // solved by pll_spec_kernel
  if (loader) {
    // ---- wave 1: constants -> LDS ring, one barrier per chunk ----
    const unsigned voff = 16u * lane;
    int64_t next = 0;                                    // next chunk to fetch
    for (; next < nch && next < NPF; ++next) glds16x<1>(voff, cr + next * CH, lds_addr_of(&cring[next % NPF][0]));
    for (int64_t ch = 0; ch < nch; ++ch) {
      wait_vm_chain<NPF>((int)(next - ch - 1));          // chunk ch has landed
      __builtin_amdgcn_s_barrier();                      // ready; and lane 0 is done with ch-1
      if (ch >= 1 && next < nch) {                       // ch-1's slot -> chunk ch-1+NPF
        glds16x<1>(voff, cr + next * CH, lds_addr_of(&cring[next % NPF][0]));
        ++next;
      }
    }
    return;
  }
  // ---- wave 0: the recurrence on lane 0 (the other lanes only take the barriers) ----
  const bool rec = lane == 0;
  const float* in = J.in + (int64_t)s * J.in_stride;
  double* th = J.theta + (int64_t)s * J.th_stride;
  float* nco_i = J.nco_i + (int64_t)s * J.out_stride;
  float* nco_q = J.nco_q ? J.nco_q + (int64_t)s * J.out_stride : nullptr;
  const PllCfg cfg = J.cfg;
  double* st = J.state + (int64_t)s * 6;
  double integ = st[0], phase = st[1], fI = st[2], fQ = st[3];
  const double off = st[5];
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  if (rec) {
    nco_i[0] = (float)st[4];
    if (nco_q) nco_q[0] = (float)((off > 0.0) ? sin((w * off + phase) * cfg.scale + cfg.adj) : 0.0);
  }
  double arg = 0.0;
  auto general = [&](float xf, int64_t k, bool literal) {   // as pll_lanes_kernel
    const double xv = (double)xf;
    double e;
    if (literal || !(xv > 0.0 || xv < 0.0)) {
      if (!literal) { fI = cos(arg); fQ = sin(arg); }
      e = atan2(xv * (-fQ), xv * fI);
    } else {
      e = reduce_2pi(xv > 0.0 ? -arg : kPi - arg);
      if (e <= -kPi) e += 2.0 * kPi;
    }
    integ = integ + cfg.ki * e;
    phase = phase + cfg.kp * e + integ;
    arg = w * ((off + (double)k) + 1.0) + phase;
  };
  // Q-form (5 f64 ops per step, P.qform): the integrator's constant drift -pi Ki per step is
  // absorbed into the constants.  Within a group (step i = k mod 32), W_i = V_i + i kB and
  // Q_i = phase_i + kB i(i-1)/2 obey W' = W + kA f, Q' = Q + W + kC f, and with the prep
  // kernel's c'_i = c_i + kB i(i-1)/(4 pi), t = c'_i - Q_i/2pi is the same t.  Q is what
  // the theta row holds (for every step of the call, general ones included); the NCO kernel
  // takes kB (i+1) i / 2 back off.
  const double kA = k2Pi * cfg.ki, kB = kPi * cfg.ki;
  const double kC = k2Pi * (cfg.kp + cfg.ki), kD = kPi * (cfg.kp + cfg.ki);
  double W = 0.0;
  auto fastq = [&](double c) {
    const double t = fma(-kInv2Pi, phase, c);
    const double f = __builtin_amdgcn_fract(t);
    const double S = phase + W;
    W = fma(kA, f, W);
    phase = fma(kC, f, S);
  };
  auto qof = [&](double ph, int64_t k) {                 // the stored Q of step k's result
    const double i = (double)(k % PG);
    return ph + kB * ((i + 1.0) * i * 0.5);
  };
  for (int64_t ch = 0; ch < nch; ++ch) {
    __builtin_amdgcn_s_barrier();                        // chunk ch is in LDS
    asm volatile("" ::: "memory");
    if (rec) {
      const double* cc = &cring[ch % NPF][0];
      // two register buffers: group g+1's constants are read while group g runs
      f4v ca[PG / 2], cb[PG / 2];
      auto group = [&](f4v (&cv)[PG / 2], f4v (&nx)[PG / 2], int g) {
        lds_group_wait(cv);                              // read a group ago
        if (g + 1 < CH / PG) lds_group_rd(nx, cc + (g + 1) * PG);
        // the steps depend on phase: pinning it here keeps the next group's reads (volatile,
        // so after the wait) ahead of this group's steps instead of sunk behind them
        asm volatile("" : "+v"(phase), "+v"(integ));
        const int64_t k0 = ch * CH + g * PG;
        bool redo = k0 == 0;                             // the call's literal first sample
        if (!redo) {
          const double ph0 = phase, in0 = integ, ar0 = arg;
          double pv[PG];
          W = integ - kD;                                // V_0 = W_0
#pragma unroll
          for (int i = 0; i < PG; ++i) {
            fastq(dbl(cv[i / 2], i & 1));
            pv[i] = phase;                               // Q_{i+1}
          }
          if (phase != phase) {                          // a 0 / NaN input in the group
            phase = ph0; integ = in0; arg = ar0;
            redo = true;
          } else {
            phase -= kB * (double)(PG * (PG - 1) / 2);   // Q_32 -> phase_32
            integ = (W - kB * (double)PG) + kD;          // W_32 -> V_32 -> integ
            arg = w * ((off + (double)(k0 + PG - 1)) + 1.0) + phase;
            double* tp = th + k0;
#pragma unroll
            for (int i = 0; i < PG; i += 2) *reinterpret_cast<double2*>(tp + i) = make_double2(pv[i], pv[i + 1]);
          }
        }
        if (redo) {
          for (int i = 0; i < PG; ++i) {
            general(in[k0 + i], k0 + i, k0 + i == 0);
            th[k0 + i] = qof(phase, k0 + i);
          }
        }
      };
      static_assert(CH / PG == 4, "two buffers, four groups per chunk");
      lds_group_rd(ca, cc);
      group(ca, cb, 0);
      group(cb, ca, 1);
      group(ca, cb, 2);
      group(cb, ca, 3);
    }
    asm volatile("" ::: "memory");
  }
  if (rec) {
    for (int64_t k = nch * CH; k < n; ++k) {      // tail (< CH samples)
      general(in[k], k, k == 0);
      th[k] = qof(phase, k);
    }
    th[n] = off;                                  // the NCO kernel's trigOffset
    if (n > 0) {
      st[0] = integ;
      st[1] = phase;
      end_trig(arg, cfg.scale, cfg.adj, st);
      st[5] = off + (double)n;
      stat_add(P.stats, SDR_PLL_ST_RECURRENCES, 1);
      stat_add(P.stats, SDR_PLL_ST_SEQUENTIAL, 1);
    }
  }
}

// ---------------------------------------------------------------------------------
// pll_spec_kernel: the recurrence of a block solved in parallel, then checked (one
// workgroup of SPEC_T threads per recurrence; launched before the loop kernel, which skips
// every recurrence this kernel completed).
//
// With the wrap's integer part m_k = floor(t_k) known, the fast step is LINEAR in the
// state x = (phaseEst, V): f = (c_k - m_k) - phase/2pi, so
//   x' = A x + u_k,  A = [[1 - kC/2pi, 1], [-kA/2pi, 1]],  u_k = (kC d_k, kA d_k - kB), d_k = c_k - m_k
// and A is a contraction (|eig| = sqrt(1 - Kp) = 0.987 per step at the reference's bandwidth).
//   1. Guess: thread j runs the true (nonlinear) step over the SPEC_W samples before its
//      chunk, from the state after sample 0 (the loop pulls the guess onto the
//      trajectory), then over its chunk,
//      keeping each step's m_k (LDS, a byte relative to floor(c_k)).
//   2. Solve: each chunk's response to its d_k from zero state, then the chunk-start states by
//      a Hillis-Steele scan of y_{j+1} = A^L y_j + z_j across the threads (y_0 exact).
//   3. Check: every thread reruns the true step from its y_j, stores the phases, and compares
//      each step's m_k with the one the solve used.  No mismatch anywhere => every chunk ran
//      from its exact start state (induction over chunks), i.e. the sequential recurrence,
//      up to rounding (the scan's association; the f32 outputs cannot see it).  Otherwise
//      the rerun's m_k are the next guess (each round fixes at least the first wrong chunk).
// A locked loop keeps fract(t) >= 0.2 away from the wrap (tools/pll_spec_probe.py), so the
// guess holds after a few hundred samples; the sequential kernel remains the path for what
// does not converge in SPEC_IT rounds (acquisition transients, noise), for 0 / NaN inputs
// (the general form) and for blocks beyond SPEC_NMAX samples.  Sample 0 of a call is the
// literal general step (fI, fQ from the caller's state), as in the loop kernels.  A completed
// recurrence is marked by c[0] = +inf (c[0] is the literal sample's slot: the loop kernels
// never read it, and the prep kernel rewrites it every call).
// warm-up samples before each chunk (a fixed constant; r03-r05 A/B builds measured it).  r04: 32 -- the guess runs
// the true step from the measured phase, and in the per-block solve of one recurrence (C4, a
// 256-thread workgroup: one wave per SIMD, no other wave to hide the f64 latency behind) the
// 128-step warm-up was 40 % of the kernel (spec_prof: 22 k of 52 k cycles).  r03, per-block solves at 64
// streams x 2 PLLs (profiles/r03/iter/specw_*): 256 -> 86 us, 128 -> 73 us, 64 -> 66 us per
// block, every recurrence in round 0 at each, the offset sweep (tests/test_offsets.py) too;
// 128 keeps a margin for inputs noisier than the synthetic ones
constexpr int SPEC_W = 32;
// ... in a long call's pseudo-block: its start is a converged guess or the chained state and
// its drift is measured, so the guess needs little settling (r03 A/B on the S8 K256 span: 0,
// 16, 32 and 64 steps all solve every pseudo-block in round 0; 16 is the fastest)
constexpr int SPEC_W_LONG = 16;
constexpr int SPEC_IT = 3;           // solve / check rounds before the sequential kernel takes over
constexpr int SPEC_NMAX = SDR_PLL_BLOCK_MAX; // samples per call (the sign codes of steps 1.. in LDS: 16 KiB)
static_assert(SPEC_NMAX == 16384 + 1, "LDS sizing");
constexpr int SPEC_N256 = 10240;             // longest call the 256-thread solve takes (512 above; fixed, r04 A/B)
constexpr int SPEC_LDS = 32 * 516;           // padded transposed bytes: 512 chunks of <= 32 steps (or 256 of <= 40)
constexpr int SB = 8;                        // steps per batch of LDS reads in the step loops
// The solve's matrix-power table (qtab_host): per chunk length L = SB, 2 SB, .., QT_NL SB
// (SPEC_T = 256 takes up to SPEC_N256 steps: L <= 40), QT_N 2x2 matrices of Q = A^L --
// Q^e for e = 0 .. 64, then Q^(64 w) for w = 0 .. 7 (the waves of a 512-thread solve)
constexpr int QT_N = 65 + 8, QT_NL = 5;
// compact phase rows: lines per pseudo-block (pb <= LONG_PB = SPEC_NMAX - 1 - 2048, below)
constexpr int TH32_LINES = (SPEC_NMAX - 1 - 2048) / TH32_LINE;

// ---- long calls: pseudo-block bookkeeping (device scratch P.work; LongBlk / LongHdr in
// sdr_nco.h, which the receiver's mixers read too) ---------------------------------------
enum { LB_NEED_G = 0, LB_DONE_G = 1, LB_NEED_X = 2, LB_DONE_X = 3, LB_ACCEPTED = 4 };
constexpr int SOLVER_SEQ = 3;        // solver codes: 0..2 = parallel solve round, 3 = sequential
__device__ __forceinline__ LongHdr* long_hdr(const PllJobs& P, int r) { return static_cast<LongHdr*>(P.work) + r; }
__device__ __forceinline__ LongBlk* long_blk(const PllJobs& P, int r, int b) {
  return reinterpret_cast<LongBlk*>(static_cast<char*>(P.work) + (int64_t)P.njobs * P.nstreams * sizeof(LongHdr)) +
         (int64_t)r * P.lg.nb + b;
}
__device__ __forceinline__ int64_t long_len(const PllJobs& P, int b) {
  return b < P.lg.nb - 1 ? P.lg.pb : P.n - (int64_t)(P.lg.nb - 1) * P.lg.pb;
}

__device__ __forceinline__ double wave_prefix_sum(double v, int lane) {   // inclusive
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// DPP moves for the wave scans (r06: instead of ds_bpermute shuffles, ~100+ cycles each in a
// dependent chain): lanes whose source lies outside the pattern, or in rows ROWS leaves out,
// keep `old`.  CTRL: row_shr:n = 0x110 + n (within rows of 16), row_bcast:15 = 0x142 (lane 15
// of rows 0 / 2 into rows 1 / 3 with ROWS = 0xa), row_bcast:31 = 0x143 (lane 31 into rows 2, 3
// with ROWS = 0xc), wave_shr:1 = 0x138.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ float dpp_f32(float old, float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, ROWS, 0xf, false));
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ double dpp_f64(double old, double v) {
  const long long o = __double_as_longlong(old), x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)x, CTRL, ROWS, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(x >> 32), CTRL, ROWS, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// a wave-uniform f64 held in SGPRs (readfirstlane of both halves): the compiler computes
// uniform f64 values on the VALU and would otherwise keep them in VGPRs
__device__ __forceinline__ double sgpr_d(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// 2x2 matrices (row-major a, b, c, d) for the loop's linear form
struct Mat2 { double a, b, c, d; };
__device__ __forceinline__ Mat2 mmul(const Mat2& x, const Mat2& y) {
  return {x.a * y.a + x.b * y.c, x.a * y.b + x.b * y.d, x.c * y.a + x.d * y.c, x.c * y.b + x.d * y.d};
}
__device__ __forceinline__ Mat2 mpow2(Mat2 x, int e) {
  Mat2 r{1.0, 0.0, 0.0, 1.0};
  for (; e > 0; e >>= 1, x = mmul(x, x))
    if (e & 1) r = mmul(r, x);
  return r;
}

// SPEC_T threads (chunks) per recurrence: 256 (one wave per SIMD) up to 10 240 samples, 512
// beyond (the warm-up is the same length either way; 512 halves the chunks, and a second
// wave per SIMD then pays: c5 blocks 56 -> ~50 us, c4 blocks slower).
// LONG: one workgroup per pseudo-block of a long call, from its start guess (status
// LB_NEED_G) or its chained start (LB_NEED_X); the end state goes to the block's record and
// the call's own state, trigOffset slot and NCO[0] are left to the long-call kernels.
// The body is a device function of the workgroup: pll_spec_kernel runs it once per workgroup
// (bid = blockIdx.x); pll_long_fix_kernel re-solves single pseudo-blocks with it.  first (long
// calls): the call's first solve -- the pseudo-block records are not initialised yet (the
// bookkeeping is done here, for this block, instead of by a kernel of its own).
template <int SPEC_T, bool LONG, bool first = false>
__device__ __forceinline__ bool spec_body(const PllJobs& P, const int bid, const int tid) {
#pragma clang fp contract(off)
  // Per step k = 1 .. n-1, at slot i * CSTR + j (step i of chunk j, see the staging below):
  // the sign code of x_k (+1: x > 0, -1: x < 0, 0: 0 / NaN; r04b: the sign itself, as the correlation uses it) -- the constant c_k is a function
  // of it and k alone (pll_c), recomputed where it is used, which keeps the workgroup's LDS
  // at ~68 KB (two per CU) instead of a 128 KiB f64 image -- and the low byte of m_k
  // (jb = floor(phaseEst_1 / 2pi)).  tb: per wave, SB steps x 64 chunks of phases on their
  // way to coalesced theta stores (stride TBS = 4 mod 32 doubles: both its write and its
  // transposed read are conflict-free); the chunk scans' scratch (yb) shares its space.
  // CSTR = 4 mod 256 bytes: the staging's byte writes (consecutive lanes on consecutive rows)
  // fall in consecutive banks -- SPEC_T + 1 put every 4 lanes in one bank; the padding column
  // SPEC_T stays
  constexpr int CSTR = SPEC_T + 4, NW = SPEC_T / 64, TBS = 68;
  static_assert(CSTR * (SPEC_T == 512 ? 32 : 40) <= SPEC_LDS, "rows fit");
  static_assert(NW * SB * TBS >= 2 * SPEC_T, "yb fits in tb");
  __shared__ int8_t code[SPEC_LDS];
  // the integers m_k chunk-major (a thread's own steps contiguous): MSTR an odd number of dwords,
  // so the 64 lanes' per-step byte accesses fall in 64 different banks (step-major put four
  // lanes in every dword)
  constexpr int MSTR = SPEC_T == 512 ? 36 : 44;
  static_assert(MSTR >= (SPEC_T == 512 ? 32 : 40) && (MSTR / 4) % 2 == 1 && MSTR % 4 == 0, "m_k rows");
  __shared__ int8_t mrel[SPEC_T * MSTR];
  __shared__ double tb[NW * SB * TBS];
  __shared__ d2v wsum[NW];
  __shared__ double x1s[2];
  __shared__ float mg[NW + 1];                   // the waves' smallest wrap margins (+ the literal step's)
  __shared__ double wsh;                         // w for the end state (no register across the solve)
  __shared__ double kds;                         // kD for the cold paths after the staging (registers)
  d2v* yb = reinterpret_cast<d2v*>(tb);
  const int lane = tid & 63, wv = tid >> 6;
  int q, s, status = 0;
  int64_t n, base = 0;
  int pre = 0;                                   // LONG, guessed start: pre-roll steps (below)
  LongBlk* LB = nullptr;
  bool from_call = false;                        // LONG: the start is the call's own state
  if constexpr (LONG) {
    const int nb = P.lg.nb;
    const int r = bid / nb;
    const int b = bid - r * nb;
    q = r / P.nstreams;
    s = r - q * P.nstreams;
    LB = long_blk(P, r, b);
    if constexpr (first) {
      // every pseudo-block unsolved, no shift; the first starts from the call's state (exact),
      // the others from the guess their pre-roll finds (below).  Block 0 also leaves the
      // call's NCO[0] and trigOffset slot as the per-call kernels do.
      status = LB_NEED_G;
      from_call = b == 0;
      if (tid == 0) {
        const PllJob& Jq = P.j[q];
        const double* sc = Jq.state + (int64_t)s * 6;
        LB->shift = 0.0;
        LB->d[0] = LB->d[1] = 0.0;
        LB->margin = -1.0;
        LB->status = LB_NEED_G;
        LB->solver = -1;
        for (int i = 0; i < 6; ++i) LB->g[i] = b == 0 ? sc[i] : __builtin_nan("");
        if (b == 0) {
          const double w0 = 2.0 * kPi * (Jq.cfg.freq / Jq.cfg.fs);
          LongHdr* H = long_hdr(P, r);
          H->sp = sc[1];
          H->si = sc[0];
          H->pos = 0;
          Jq.nco_i[(int64_t)s * Jq.out_stride] = (float)sc[4];
          if (Jq.nco_q)
            Jq.nco_q[(int64_t)s * Jq.out_stride] =
                (float)((sc[5] > 0.0) ? sin((w0 * sc[5] + sc[1]) * Jq.cfg.scale + Jq.cfg.adj) : 0.0);
          Jq.theta[(int64_t)s * Jq.th_stride + P.n] = sc[5];     // the NCO kernel's trigOffset
        }
      }
    } else {
      status = LB->status;
      if (status != LB_NEED_G && status != LB_NEED_X) return true;
    }
    base = (int64_t)b * P.lg.pb;
    n = long_len(P, b);
    // a pseudo-block after the first, not yet reached by the chain: its start is unknown, so
    // the solve runs `pre` steps of the previous pseudo-block's range first, from the phase
    // the input measures there (mod 2 pi) and the span's start integrator.  The loop contracts
    // the seed's error by sqrt(1 - Kp) a step, so the state at the block's start converges to
    // the recurrence's up to whole turns (the chain finds them) -- the sequential warm-up of a
    // start guess, solved in parallel with the block.  Its phases are not stored.
    if (status == LB_NEED_G && b > 0) pre = P.lg.warm[q];
    n += pre;
    base -= pre;
  } else {
    q = bid / P.nstreams;
    s = bid - q * P.nstreams;
    n = P.n;
  }
  const PllJob& J = P.j[q];
  const float* in = J.in + (int64_t)s * J.in_stride + base;
  const int8_t* in8 = J.in8 != nullptr ? J.in8 + (int64_t)s * J.in8_stride + base : nullptr;
  double* th = J.theta + (int64_t)s * J.th_stride + base;
  double* cr = J.cbuf + (int64_t)s * J.c_stride + base;
  const PllCfg cfg = J.cfg;
  // compact phase rows (sdr_nco.h, LONG with J.th32): the pseudo-block's lines (a, s), set each
  // round by the thread whose steps hold a line's first row, read by every thread's stores
  const bool t32 = LONG && J.th32 != 0;
  Th32Line* tl = nullptr;
  if constexpr (LONG) {
    __shared__ Th32Line tl_[TH32_LINES];
    tl = tl_;
  }
  double* rowp = J.theta + (int64_t)s * J.th_stride;   // the stream's row (compact: residuals, then lines)
  const int64_t rb = base + pre;                        // the pseudo-block's first row
  // the row's lines, formed once here and held in SGPRs (readfirstlane: otherwise the compiler
  // reloads the call's length from the kernel arguments where the solve first needs it -- a
  // scalar load and an lgkmcnt(0) wait after the guess barrier)
  Th32Line* lrow = nullptr;
  if (t32) {
    const uintptr_t a = (uintptr_t)th32_lines(rowp, P.n);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    lrow = reinterpret_cast<Th32Line*>(((uintptr_t)hi << 32) | lo);
  }
#ifdef SDR_PLL_SPEC_PROF    // phase timers (diagnostic builds only, tools/build_dbg.sh)
#ifndef SDR_PLL_SPEC_PROF_TID
#define SDR_PLL_SPEC_PROF_TID 0   // the thread whose timers print (-D...=448: wave 7, a storing wave)
#endif
  long long tp[16];
  int ntp = 0;
  tp[ntp++] = clock64();
#define SPEC_TP() do { if (ntp < 16) tp[ntp++] = clock64(); } while (0)
#else
#define SPEC_TP() do {} while (0)
#endif
  const double* st_call = J.state + (int64_t)s * 6;
  double* st = LONG ? (from_call ? J.state + (int64_t)s * 6 : status == LB_NEED_G ? LB->g : LB->x)
                    : J.state + (int64_t)s * 6;
  double* st_out = LONG ? LB->e : st;
  const double off = sgpr_d(pre ? st_call[5] + (double)base : st[5]);   // trigOffset of local step 0
  const double w = sgpr_d(2.0 * kPi * (cfg.freq / cfg.fs));
  const double kA = sgpr_d(k2Pi * cfg.ki), kB = sgpr_d(kPi * cfg.ki);
  const double kC = sgpr_d(k2Pi * (cfg.kp + cfg.ki)), kD = sgpr_d(kPi * (cfg.kp + cfg.ki));
  // what the theta row holds for step k: the phase itself (every launch of the solve -- per-block,
  // long call, fix kernel -- runs with qform = 0, sdr_launch_pll_loop; the Q-form rows are the
  // sequential chunk kernel's alone)
  auto thval = [&](double ph, int64_t) { return ph; };
  // c_k from the sign code: pll_c's arithmetic exactly (code 0, a 0 / NaN input, is caught by
  // the guess: the solve is abandoned to the general form, so its value here does not matter)
  const double w2pi = sgpr_d(w * kInv2Pi);
  if (tid == 0) { wsh = w; kds = kD; }
  auto cval = [&](int cd, int k) { return fma(-(off + (double)k), w2pi, cd > 0 ? 0.5 : 1.0); };
  // ... from offk = off + k itself: the step loops carry offk as an f64 counter (+1.0 a step, exact
  // for the integer-valued trigOffset) instead of converting k every step (cval's value exactly)
  auto cvk = [&](int cd, double offk) { return fma(-offk, w2pi, cd > 0 ? 0.5 : 1.0); };
  // sample 0: the literal general step (thread 0), as the loop kernels' general() (a
  // pre-roll's seed is set from the measured phase instead, below)
  if (tid == 0 && pre == 0) {
    const double xv = (double)(in8 != nullptr ? pll_decode(in8[0]) : in[0]);
    const double e = atan2(xv * (-st[3]), xv * st[2]);
    mg[NW] = (float)((kPi - fabs(e)) * kInv2Pi);  // the literal step's distance from the wrap
    const double integ = st[0] + cfg.ki * e;
    const double phase = st[1] + cfg.kp * e + integ;
    x1s[0] = phase;
    x1s[1] = integ - kD;
  }
  const int N = (int)n - 1;                      // steps 1 .. n-1
  // chunk length: a multiple of SB (the step loops run in batches of SB, their LDS reads issued
  // ahead of the dependent steps; a step past a chunk's end is computed and discarded)
  const int L = (N + SPEC_T * SB - 1) / (SPEC_T * SB) * SB;
  const int TE = (N + L - 1) / L;                // chunks in use; chunks 0 .. TE-2 are full
  const int k0 = 1 + tid * L;
  const int len = tid < TE ? min(L, (int)n - k0) : 0;   // steps of this thread's chunk
  // the solve's matrix powers (Q = A^L: Q^e, e <= 64, and Q^(64 w)) into LDS; their loads go
  // out with the staging's, so the solve never waits on memory (r06: a per-thread global load
  // at the solve waited ~10 k cycles behind the other workgroups' staging traffic)
  __shared__ d2v qt2[2 * QT_N];
  d2v qv{0.0, 0.0};
  if (tid < 2 * QT_N) qv = reinterpret_cast<const d2v*>(J.qtab)[(int64_t)(L / SB - 1) * 2 * QT_N + tid];
  // stage the sign codes, transposed -- step i of chunk j at i * CSTR + j -- so that the
  // threads' per-step reads of their own chunks are consecutive bytes; the global loads go
  // out SG at a time before the first is used.  (Slots of steps past N hold whatever was
  // there: only discarded steps read them, and every slot is in the array.)
  {
    // r04b: no per-element branch (the guards' branches were ~13 SALU a step): every thread
    // loads and writes all SG of its elements, a load past N clamped into the array.  Such an
    // element's slot (kk mod L, kk / L) is a step past its chunk's end or of an unused chunk
    // (only discarded steps read them) -- or, when kk / L passes the row's end (L = 24: up to
    // 682 > CSTR), the next row's real slot: its column is clamped to the padding column
    // (chunk SPEC_T, never in use)
    constexpr int SG = SPEC_T == 512 ? 32 : 40;
    static_assert(SG * SPEC_T >= (SPEC_T == 512 ? SPEC_NMAX : SPEC_N256) - 1, "one pass of SG loads covers a call");
    // (a span's sign-code row: a quarter of the bytes, r06; its codes other than +-1 -- zeros,
    // NaN -- are the solve's general-form case, 0, as the float row's)
    float xv[SG];
    // (r06: a full-length pseudo-block's sign codes as each thread's own chunk -- 32 codes, two
    // 16-B loads instead of 32 byte loads; chunk j's steps 1 + 32 j .. 32 + 32 j start on a 16-B
    // boundary after the 2 049-step pre-roll -- written into its column)
    // (first: only a long call's first solve has pre-rolls; the repair kernel's registers are full)
    const bool fast8 = first && SPEC_T == 512 && in8 != nullptr && L == 32 && N == SPEC_T * 32 &&
                       ((uintptr_t)(in8 + 1) % 16) == 0;
    if (fast8) {
      const int4* src = reinterpret_cast<const int4*>(in8 + 1 + 32 * tid);
      const int4 q0 = src[0], q1 = src[1];
      const int w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
      for (int e = 0; e < 32; ++e) {
        const int c = (int)(int8_t)(w[e >> 2] >> (8 * (e & 3)));
        code[e * CSTR + tid] = (int8_t)((c == 1 || c == -1) ? c : 0);
      }
    } else if (in8 != nullptr) {
      int8_t cv[SG];
#pragma unroll
      for (int u = 0; u < SG; ++u) cv[u] = in8[min(tid + u * SPEC_T, N - 1) + 1];
#pragma unroll
      for (int u = 0; u < SG; ++u) xv[u] = (cv[u] == 1 || cv[u] == -1) ? (float)cv[u] : 0.f;
    } else {
#pragma unroll
      for (int u = 0; u < SG; ++u) xv[u] = in[min(tid + u * SPEC_T, N - 1) + 1];
    }
    auto cod = [](float x) { return (int8_t)(x > 0.f ? 1 : (x < 0.f ? -1 : 0)); };
    if (fast8) {
      // (staged above)
    } else if (SPEC_T % L == 0) {
      // element kk = tid + u SPEC_T: i = tid mod L for every u, j = tid / L + u SPEC_T / L
      const int i = tid % L, j0 = tid / L, js = SPEC_T / L;
#pragma unroll
      for (int u = 0; u < SG; ++u) {
        const int j = j0 + u * js;
        code[i * CSTR + min(j, SPEC_T)] = cod(xv[u]);
      }
    } else {
      // kk / L by a multiply-high (L <= 64, kk < 2^16: exact with m = floor(2^32 / L) + 1)
      const unsigned mL = 0xffffffffu / (unsigned)L + 1u;
#pragma unroll
      for (int u = 0; u < SG; ++u) {
        const int kk = tid + u * SPEC_T;
        const int j = (int)__umulhi((unsigned)kk, mL), i = kk - j * L;
        code[i * CSTR + min(j, SPEC_T)] = cod(xv[u]);
      }
    }
  }
  if (tid < 2 * QT_N) qt2[tid] = qv;
  __syncthreads();
  SPEC_TP();
  // r04b: a wave whose chunks are all full runs the step loops without a per-step "inside the
  // chunk" predicate (its selects and compares were a fifth of the check loop's VALU); the wave
  // holding the last, partial chunk (and the unused ones) keeps them.  wfast: also every chunk
  // after a long call's pre-roll, so every step's wrap margin counts and every phase is stored.
  const bool wfull = __all(len == L);
  const bool wfast = wfull && __all(k0 >= pre);
  const bool wpre = wfull && __all(k0 + L <= pre);      // (r06: the pre-roll wave of a full-length pseudo-block)
  // 0. where the locked phase estimate goes within the block, measured from the input: a
  // locked loop keeps its angle th_{k-1} = w (off + k) + phaseEst_{k-1} on the input tone's
  // phase, so z_j = sum over chunk j of x_k exp(-i w (off + k)) ~ (A/2) exp(i phaseEst) (+ an
  // image term at twice the carrier, averaged down by summing 5 chunks).  The chunk phases,
  // unwrapped by a scan of their differences (a chunk drifts by ~0.02 rad at a 30 Hz carrier
  // offset), give D_j = phaseEst(chunk j) - phaseEst(chunk 0), bias-free.  (A 2 Hz pilot offset
  // is a 12 Hz RDS carrier offset, 4.8 rad per 15 360-sample block: from the block's first
  // state alone, the RDS loop's 256-step warm-ups (contraction ~0.7) cannot catch it up.
  // Extrapolating by integ does worse: integ swings with the loop's own oscillation.)
  {
    // sign(x_k) exp(-i w (off + k)) = exp(-i 2 pi fract(1/2 - c_k)): a hard-limited
    // correlation, as the loop's detector.  The nominal NCO's phasor exp(i w (off + k)) is
    // rotated by exp(i w) from the chunk's first step in f32 (L <= 64 steps: a drift of ~1e-6,
    // far below what a guess needs -- the check, not the guess, makes the solve exact)
    // r04b: packed f32 -- the phasor (cr, ci) and the sums in register pairs: per step one
    // v_pk_fma_f32 accumulates sg (cr, ci) (zi = -its second half) and a v_pk_mul + v_pk_fma
    // rotate the phasor: (cr, ci) <- (cr dc - ci ds, ci dc + cr ds) (the swapped operand by
    // op_sel); the sign code IS sg.  (A guess: the check, not this, makes the solve exact.)
    f2v z = f2v{0.f, 0.f};
    {
      const double a0 = __builtin_amdgcn_fract(w2pi * (off + (double)k0));
      float ci, cr, ds, dc;
      __sincosf((float)(k2Pi * a0), &ci, &cr);
      __sincosf((float)w, &ds, &dc);
      f2v c = f2v{cr, ci};
      f2v dcv = f2v{dc, dc}, dsv = f2v{-ds, ds};
      auto corr = [&](auto FC) __attribute__((always_inline)) {
        constexpr bool F = decltype(FC)::value;
        f2v rs = dsv;
        for (int i0 = 0; i0 < L; i0 += SB) {
          int cd[SB];
#pragma unroll
          for (int u = 0; u < SB; ++u) cd[u] = code[(i0 + u) * CSTR + tid];
#pragma unroll
          for (int u = 0; u < SB; ++u) {
            // x > 0: +exp(-i a); x < 0: -exp(-i a) (the pi of sel); 0 / NaN / past the chunk: 0
            const float sg = (F || i0 + u < len) ? (float)cd[u] : 0.f;
            const f2v sgv = f2v{sg, sg};
            asm("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(z) : "v"(sgv), "v"(c));
            const f2v t = c * dcv;
            asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1]" : "=v"(c) : "v"(c), "v"(rs), "v"(t));
          }
        }
      };
      if (wfull) corr(std::true_type{});
      else corr(std::false_type{});
    }
    SPEC_TP();
    yb[tid] = d2v{(double)z.x, -(double)z.y};
    __syncthreads();
    // the 5-chunk sums around this chunk and around the one before it: each thread forms both
    // angles, so their difference needs no second exchange (r06: 3 barriers instead of 5), and
    // the unwrapped differences are summed in f32 (a guess: the check, not this, is exact)
    double sr = 0.0, si = 0.0, qr = 0.0, qi = 0.0;
    for (int o = -3; o <= 2; ++o) {
      const int j = tid + o;
      if (j >= 0 && j < TE) {
        const d2v v = yb[j];
        if (o >= -2) { sr += v.x; si += v.y; }
        if (o <= 1) { qr += v.x; qi += v.y; }
      }
    }
    const float ang = atan2f((float)si, (float)sr), angp = atan2f((float)qi, (float)qr);
    if (pre > 0 && tid == 0) {                   // the pre-roll's seed: measured phase, span's integrator
      x1s[0] = (double)ang;
      x1s[1] = st_call[0] - kds;
    }
    float d = 0.f;
    if (tid >= 1 && tid < TE) {
      d = ang - angp;
      d -= 6.28318548f * rintf(d * 0.159154937f);
    }
    // inclusive prefix sum of the differences: within each wave by DPP moves (within rows of
    // 16, then rows 1 / 3 from lane 15 of rows 0 / 2, then rows 2, 3 from lane 31), then the
    // waves' totals
    d += dpp_f32<0x111>(0.f, d);
    d += dpp_f32<0x112>(0.f, d);
    d += dpp_f32<0x114>(0.f, d);
    d += dpp_f32<0x118>(0.f, d);
    d += dpp_f32<0x142, 0xa>(0.f, d);
    d += dpp_f32<0x143, 0xc>(0.f, d);
    if (lane == 63) wsum[wv].x = (double)d;
    __syncthreads();
    double D = (double)d;
    for (int i = 0; i < wv; ++i) D += wsum[i].x;
    yb[tid].x = D;                               // D_j
    __syncthreads();
  }
  SPEC_TP();
  const double p1 = x1s[0], v1 = x1s[1];
  // 1. guess.  With every m_k fixed at the floor the pass itself takes, a pass over a chunk IS
  // the loop's linear form x' = A x + u_k, so the chunk's response from zero state -- what the
  // scan needs -- is its end state less A^L times its start: z_j = x_end - Q x_start (the
  // solve needs no pass of its own; the check below validates whatever this rounds to)
  bool bad = false;
  double xs_p = 0.0, xs_v = 0.0, xe_p = 0.0, xe_v = 0.0;
  {
    // the true step from a seed on the measured drift: phaseEst ~ p1 + D at the warm-up's
    // start, the integrator the block's first; the SW warm-up steps of the loop then pull the
    // guess onto the trajectory (r05: the seed no longer estimates integ from the drift -- that
    // needed a warm-up of >= 64 steps, longer than SW since r04)
    constexpr int SW = LONG ? SPEC_W_LONG : SPEC_W;
    const int kw = max(1, k0 - SW);
    const int jw = (kw - 1) / L;
    double p = p1 + yb[jw].x, V = v1;
    const int W = tid < TE ? k0 - kw : 0;        // warm-up steps (over the chunks before this one)
    if (wfull && SW <= 2 * L) {
      // every warm-up is the last SW steps before the chunk: the last SW - L of chunk j-2 when
      // SW > L (the per-block C4 solve: L = 24, SW = 32), then the last min(SW, L) of chunk j-1.
      // Threads with a shorter warm-up (j = 0: none; j = 1 when SW > L: L steps) run the same
      // passes over chunk 0 and take their seed back before the part that is theirs.
      const double p0 = p, v0 = V;
      double kd = off + (double)(k0 - SW);
      auto pass = [&](int jc, int ib, int ns) __attribute__((always_inline)) {
#pragma unroll 1
        for (int i0 = 0; i0 < ns; i0 += SB) {
          int cd[SB];
#pragma unroll
          for (int u = 0; u < SB; ++u) cd[u] = code[(ib + i0 + u) * CSTR + jc];
#pragma unroll
          for (int u = 0; u < SB; ++u) {
            const double t = fma(-kInv2Pi, p, cvk(cd[u], kd));
            kd += 1.0;
            const double f = __builtin_amdgcn_fract(t);
            const double S = p + V;
            V = fma(kA, f, V - kB);
            p = fma(kC, f, S);
          }
        }
      };
      if (SW > L) {
        pass(max(tid - 2, 0), 2 * L - SW, SW - L);
        if (W < SW) { p = p0; V = v0; }
      }
      const int s2 = SW > L ? L : SW;
      pass(max(tid - 1, 0), L - s2, s2);
      if (W == 0) { p = p0; V = v0; }
    } else {
      int jc = jw, ic = (kw - 1) - jw * L;       // (chunk, step) of step kw
      for (int i0 = 0; i0 < W; i0 += SB) {
        int cd[SB];
#pragma unroll
        for (int u = 0; u < SB; ++u) {           // (past the warm-up: slots of this chunk, unused)
          cd[u] = code[ic * CSTR + jc];
          if (++ic == L) { ic = 0; ++jc; }
        }
#pragma unroll
        for (int u = 0; u < SB; ++u) {
          const double t = fma(-kInv2Pi, p, cval(cd[u], kw + i0 + u));
          const double f = __builtin_amdgcn_fract(t);
          const double S = p + V;
          const double nV = fma(kA, f, V - kB), np = fma(kC, f, S);
          const bool act = i0 + u < W;
          V = act ? nV : V;
          p = act ? np : p;
        }
      }
    }
    SPEC_TP();
    __syncthreads();                             // yb (D_j) read before tb reuses its space
    xs_p = p;                                    // the guess's chunk start (after the warm-up)
    xs_v = V;
    auto guess = [&](auto FC) __attribute__((always_inline)) {
      constexpr bool F = decltype(FC)::value;
      double kd = off + (double)k0;
      for (int i0 = 0; i0 < L; i0 += SB) {
        int cd[SB];
#pragma unroll
        for (int u = 0; u < SB; ++u) cd[u] = code[(i0 + u) * CSTR + tid];
#pragma unroll
        for (int u = 0; u < SB; ++u) {
          const int i = i0 + u;
          const double t = fma(-kInv2Pi, p, cvk(cd[u], kd));
          kd += 1.0;
          const bool act = F || i < len;
          bad |= act && cd[u] == 0;                // a 0 / NaN input: the general form's case
          const double f = __builtin_amdgcn_fract(t);
          if (act) mrel[tid * MSTR + i] = floor_byte(t, f);
          const double S = p + V;
          const double nV = fma(kA, f, V - kB), np = fma(kC, f, S);
          if constexpr (F) {
            V = nV;
            p = np;
          } else {
            V = act ? nV : V;
            p = act ? np : p;
          }
        }
      }
    };
    if (wfull) guess(std::true_type{});
    else guess(std::false_type{});
    SPEC_TP();
    xe_p = p;                                    // ... and its end
    xe_v = V;
  }
  if (__syncthreads_or(bad)) return false;       // a 0 / NaN input (the general form's case)
  SPEC_TP();
  // Q = A^L's powers from the job's table (qtab_host, built once per loop on the host, staged in
  // LDS with the sign codes): Q^(2^i) for the scan's offsets, Q^(lane+1) and Q^tid = Q^(64 w)
  // Q^lane for the chunk starts -- r06: instead of thread 0 forming them (A^L step by step, then
  // the squarings, behind a barrier) and every thread multiplying up to 9 of them (phase timers:
  // ~10 k of a pseudo-block's ~66 k cycles)
  const Mat2* QT = reinterpret_cast<const Mat2*>(qt2);
  auto qp = [&](int i) { return QT[1 << i]; };   // Q^(2^i), i <= 6
  double* tw = tb + wv * SB * TBS;               // this wave's transpose tile
  for (int round = 0; round < SPEC_IT; ++round) {
    // compact rows: the line whose first row (row kk = 0 mod 32 of the pseudo-block, step
    // kk + pre) is among the rows from this thread's start state (row k0 - 1) to its last step
    // but one -- at most one, L <= 32; the ranges tile the solve -- from this thread's last
    // pass over its chunk: its start and its slope.  (The pseudo-block's last row, when it
    // starts a line, is left to the end of the solve.)  Written before the scan's barrier, read
    // by the stores after it
    if (t32 && tid < TE) {
      const int kk = ((max(k0 - 1, pre) - pre) + TH32_LINE - 1) & ~(TH32_LINE - 1);
      if (kk + pre < k0 + len - 1) {
        const double sl = (xe_p - xs_p) / (double)len;
        const Th32Line ln{fma(sl, (double)(kk + pre - (k0 - 1)), xs_p), sl};
        tl[kk / TH32_LINE] = ln;
        lrow[(rb + kk) / TH32_LINE] = ln;
      }
    }
    SPEC_TP();                                   // (the phase timers: the compact rows' lines)
    // 2. solve: the chunk's response from zero state to the current integers, from the last
    // pass over it (the guess in round 0, the previous check after): z_j = x_end - Q x_start
    double zp, zv;
    {
      const Mat2 Q = qp(0);
      zp = xe_p - (Q.a * xs_p + Q.b * xs_v);
      zv = xe_v - (Q.c * xs_p + Q.d * xs_v);
    }
    // chunk starts y_j = Q^j x_1 + Y_{j-1}, Y_j = sum_{i<=j} Q^(j-i) z_i (Q = A^L): an inclusive
    // scan of the z_i within each wave by shuffles (offset o combines with Q^o), then across the
    // waves through their totals (Y at a wave's end = its total + Q^64 Y at the previous end).
    // Y_{j-1} of a wave's lane 0 is that carry itself (r06: no second exchange of the totals)
    const Mat2 Ql = QT[lane + 1], Qj = mmul(QT[65 + wv], QT[lane]);   // Q^(lane+1), Q^tid
    double yp = tid < TE ? zp : 0.0, yv = tid < TE ? zv : 0.0;
    double cp = 0.0, cv = 0.0;                   // Y at the end of the previous wave
    SPEC_TP();                                   // (the phase timers: z and the Q powers)
    {
      // (r06: DPP moves -- offsets 1, 2, 4, 8 within rows of 16, a lane past its row's start
      // adding Q^o x the lane o before it; then rows 1 / 3 take Q^((lane & 15) + 1) x lane 15 of
      // rows 0 / 2, and rows 2, 3 Q^((lane & 31) + 1) x lane 31: the same sums as the shuffled
      // Hillis-Steele scan, associated differently, which the check's exactness does not see)
      auto step = [&](const Mat2& Qo, double up, double uv) {
        yp = yp + (Qo.a * up + Qo.b * uv);
        yv = yv + (Qo.c * up + Qo.d * uv);
      };
      step(qp(0), dpp_f64<0x111>(0.0, yp), dpp_f64<0x111>(0.0, yv));
      step(qp(1), dpp_f64<0x112>(0.0, yp), dpp_f64<0x112>(0.0, yv));
      step(qp(2), dpp_f64<0x114>(0.0, yp), dpp_f64<0x114>(0.0, yv));
      step(qp(3), dpp_f64<0x118>(0.0, yp), dpp_f64<0x118>(0.0, yv));
      step(QT[(lane & 15) + 1], dpp_f64<0x142, 0xa>(0.0, yp), dpp_f64<0x142, 0xa>(0.0, yv));
      step(QT[(lane & 31) + 1], dpp_f64<0x143, 0xc>(0.0, yp), dpp_f64<0x143, 0xc>(0.0, yv));
      if (lane == 63) wsum[wv] = d2v{yp, yv};
      SPEC_TP();                                 // (the phase timers: the scan's shuffles / its barrier)
      __syncthreads();
      SPEC_TP();
      // the carry, Y at the previous wave's end = sum over the waves before of Q^(64 (wv-1-i))
      // x their totals (QT[65 + w] = Q^(64 w)): independent products, not a chain of wv
      // dependent steps (r06: the last wave waited out seven)
#pragma unroll
      for (int i = 0; i < NW - 1; ++i) {
        if (i < wv) {
          const Mat2 M = QT[65 + wv - 1 - i];
          const d2v t = wsum[i];
          cp = cp + (M.a * t.x + M.b * t.y);
          cv = cv + (M.c * t.x + M.d * t.y);
        }
      }
      yp = yp + (Ql.a * cp + Ql.b * cv);
      yv = yv + (Ql.c * cp + Ql.d * cv);
      SPEC_TP();
    }
    // Y_{j-1}: the previous lane's (lane 0: the carry); the check's barrier orders these wsum
    // reads before the next round's writes
    double vp = dpp_f64<0x138>(cp, yp), vv = dpp_f64<0x138>(cv, yv);   // (wave_shr:1; lane 0 keeps the carry)
    vp = vp + (Qj.a * p1 + Qj.b * v1);           // + Q^j x_1
    vv = vv + (Qj.c * p1 + Qj.d * v1);
    SPEC_TP();
    // 3. check: the true step from y_j.  The phases go out as the theta row on every round (a
    // later round or the sequential kernel overwrites a failed one): each batch of SB steps
    // of the wave's 64 chunks turns through tw so that a store covers 8 chunks x SB steps
    // (64-B runs) instead of 64 scattered doubles
    bool miss = false;
    double p = vp, V = vv;
    xs_p = vp;                                   // this pass's start and (below) end: the next
    xs_v = vv;                                   // round's responses to the integers it records
    // smallest / largest fract(t) of the block's own steps, as f32 bit patterns (non-negative:
    // integer min / max order them; the margin is min(lo, 1 - hi))
    unsigned mlo = 0x3f800000u, mhi = 0u;
    // PO (a wave of pre-roll chunks only, F too): no phases to store, no wrap margins of its own
    // AF (compact rows, a32 wave of full chunks after a pre-roll of 1 mod 32 steps: each chunk
    // is exactly its own line): the residuals against the chunk's own start, a flat line {vp, 0}
    // -- one subtraction a step from a value the check holds anyway, no line lookup per store.
    // (Such chunks follow the loop's acquisition, which the first pseudo-block of a stream
    // holds: a locked loop moves ~0.1 rad in 32 steps, f32 rounding ~6e-9 rad; a loop drifting
    // 1 rad in 32 steps still rounds to 6e-8.)
    auto check = [&](auto FC, auto POC, auto AC) __attribute__((always_inline)) {
      constexpr bool F = decltype(FC)::value, PO = decltype(POC)::value, AF = decltype(AC)::value;
      if constexpr (AF)   // (its line: the pseudo-block's line tid - (pre >> 5), pre = 1 mod 32 and L = 32)
        lrow[(rb >> 5) + tid - (pre >> 5)] = Th32Line{xs_p, 0.0};
      double kd = off + (double)k0;
      for (int i0 = 0; i0 < L; i0 += SB) {
        int cd[SB / 2];                          // (half a batch of codes at a time: registers)
        int8_t mm[SB / 2];
#pragma unroll
        for (int u = 0; u < SB; ++u) {
          if (u % (SB / 2) == 0) {
#pragma unroll
            for (int v = 0; v < SB / 2; ++v) {
              cd[v] = code[(i0 + u + v) * CSTR + tid];
              mm[v] = mrel[tid * MSTR + i0 + u + v];
            }
          }
          const int i = i0 + u;
          const double t = fma(-kInv2Pi, p, cvk(cd[u % (SB / 2)], kd));
          kd += 1.0;
          const bool act = F || i < len;
          const double f = __builtin_amdgcn_fract(t);
          const int8_t r = floor_byte(t, f);
          miss |= act && r != mm[u % (SB / 2)];
          const double S = p + V;
          const double nV = fma(kA, f, V - kB), np = fma(kC, f, S);
          const unsigned fb = __float_as_uint((float)f);
          if constexpr (PO) {
            V = nV;
            p = np;
          } else if constexpr (F) {
            V = nV;
            p = np;
            mlo = min(mlo, fb);
            mhi = max(mhi, fb);
          } else {
            V = act ? nV : V;
            p = act ? np : p;
            const bool own = act && k0 + i >= pre;
            mlo = min(mlo, own ? fb : 0x3f800000u);
            mhi = max(mhi, own ? fb : 0u);
          }
          if (act) mrel[tid * MSTR + i] = r;
          if constexpr (AF) tw[u * TBS + lane] = p - xs_p;
          else if constexpr (!PO) tw[u * TBS + lane] = thval(p, k0 + i);
        }
        if constexpr (PO) continue;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int u = lane & (SB - 1), cw = lane / SB;   // this lane stores step i0 + u of chunk 8 r + cw
#pragma unroll
        for (int r8 = 0; r8 < 64 / SB; ++r8) {
          const int ch = r8 * SB + cw;                   // chunk within the wave
          const int k = 1 + (wv * 64 + ch) * L + i0 + u;
          const double v = tw[u * TBS + ch];
          const bool keep = F || (k >= pre && k < (int)n);
          if constexpr (AF) {
            th32_res(rowp)[rb + (k - pre)] = (float)v;   // (F: every step kept)
          } else if (t32) {                              // (uniform) its residual against its line
            const int kk = k - pre;
            const Th32Line ln = tl[min(max(kk, 0) / TH32_LINE, TH32_LINES - 1)];
            const float rv = th32_residual(ln, kk & (TH32_LINE - 1), v);
            if (keep) th32_res(rowp)[rb + kk] = rv;
          } else if (keep) {
            th[k] = v;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    };
    if constexpr (LONG) {
      // (three forms, so the solve stays within its registers: a long call's full waves are
      // AF when their pseudo-block allows it -- every middle pseudo-block of a span -- and take
      // the general form otherwise: its first and last pseudo-blocks, repairs, calls without
      // compact rows)
      if (wfast && t32 && L == TH32_LINE && (pre & (TH32_LINE - 1)) == 1)
        check(std::true_type{}, std::false_type{}, std::true_type{});
      else if (wpre) check(std::true_type{}, std::true_type{}, std::false_type{});
      else check(std::false_type{}, std::false_type{}, std::false_type{});
    } else {
      if (wfast) check(std::true_type{}, std::false_type{}, std::false_type{});
      else if (wpre) check(std::true_type{}, std::true_type{}, std::false_type{});
      else check(std::false_type{}, std::false_type{}, std::false_type{});
    }
    SPEC_TP();
    float mth = fminf(__uint_as_float(mlo), 1.f - __uint_as_float(mhi));
    xe_p = p;
    xe_v = V;
    if constexpr (LONG) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mth = fminf(mth, __shfl_xor(mth, o, 64));
      if (lane == 0) mg[wv] = mth;
    }
    const int nmiss = __syncthreads_count(miss);
    SPEC_TP();
#ifdef SDR_PLL_SPEC_PROF
    if (tid == SDR_PLL_SPEC_PROF_TID && nmiss == 0 && (bid == 0 || (bid % 479) == 3))
      printf("spec_prof blk %d L %d: stage %lld corrloop %lld corrscan %lld warm %lld guessloop %lld guesssync %lld "
             "lines %lld zq %lld wshfl %lld wbar %lld xscan %lld ystart %lld checkloop %lld checksync %lld (%d marks)\n",
             bid, L, tp[1] - tp[0], tp[2] - tp[1], tp[3] - tp[2], tp[4] - tp[3], tp[5] - tp[4], tp[6] - tp[5],
             tp[7] - tp[6], tp[8] - tp[7], tp[9] - tp[8], tp[10] - tp[9], tp[11] - tp[10], tp[12] - tp[11],
             tp[13] - tp[12], tp[14] - tp[13], ntp);
#endif
    if (nmiss == 0) {
      if constexpr (LONG) {
        // a pre-roll's state at the block start (after step pre - 1): the thread whose chunk
        // holds that step reruns its check steps up to it -- the same arithmetic, so the same
        // state (a per-step test for it in the check loop cost the registers that spilled)
        if (pre > 0) {
          const int ic = (pre - 1) - k0;
          if (ic >= 0 && ic < len) {
            double p = xs_p, V = xs_v;
            for (int i = 0; i <= ic; ++i) {
              const double t = fma(-kInv2Pi, p, cval(code[i * CSTR + tid], k0 + i));
              const double f = __builtin_amdgcn_fract(t);
              const double S = p + V;
              V = fma(kA, f, V - kB);
              p = fma(kC, f, S);
            }
            x1s[0] = p;
            x1s[1] = V;
          }
          __syncthreads();
        }
      }
      // done: the caller-visible results exactly as the loop kernels leave them
      if (tid == 0) {
        if (pre == 0) {
          if (t32) th32_res(rowp)[rb] = th32_residual(tl[0], 0, p1);
          else th[0] = thval(p1, 0);
        }
        if constexpr (!LONG) {
          J.nco_i[(int64_t)s * J.out_stride] = (float)st[4];
          if (J.nco_q)
            J.nco_q[(int64_t)s * J.out_stride] =
                (float)((off > 0.0) ? sin((wsh * off + st[1]) * cfg.scale + cfg.adj) : 0.0);
        }
      }
      __syncthreads();                           // st[1], st[4] read before the last chunk writes st
      if (tid == TE - 1) {
        if (t32 && ((n - 1 - pre) & (TH32_LINE - 1)) == 0) {   // the last row starts a line: the line is its own
          const int64_t kl = rb + (n - 1 - pre);
          lrow[kl / TH32_LINE] = Th32Line{p, 0.0};
          th32_res(rowp)[kl] = 0.f;
        }
        const double arg = wsh * ((off + (double)(n - 1)) + 1.0) + p;
        if constexpr (!LONG) th[n] = off;
        st_out[0] = V + kds;
        st_out[1] = p;
        end_trig(arg, cfg.scale, cfg.adj, st_out);
        st_out[5] = off + (double)n;
      }
      if (tid == 0) {
        if constexpr (LONG) {                    // counted when the chain accepts the block
          if (pre > 0) {                         // the pre-roll's state at the block start: its guess
            const double gpv = x1s[0], gvv = x1s[1];
            const double ofs = off + (double)(pre - 1);          // the previous step's trigOffset
            const double arg = wsh * (ofs + 1.0) + gpv;
            LB->g[0] = gvv + kds;
            LB->g[1] = gpv;
            double sv, cv;
            sincos_red<true>(reduce_2pi(arg), &sv, &cv);
            LB->g[2] = cv;
            LB->g[3] = sv;
            LB->g[4] = 0.0;
            LB->g[5] = off + (double)pre;
            LB->u[0] = gvv + kds;
            LB->u[1] = gpv;
          } else {
            LB->u[0] = st[0];
            LB->u[1] = st[1];
          }
          float m = pre == 0 ? mg[NW] : 1.f;
          for (int i = 0; i < NW; ++i) m = fminf(m, mg[i]);
          LB->margin = m;
          LB->d[0] = LB->d[1] = 0.0;             // its phases are its own solve's
          LB->status = status + 1;               // LB_NEED_G -> LB_DONE_G, LB_NEED_X -> LB_DONE_X
          LB->solver = round;
        } else {
          cr[0] = __builtin_inf();               // the loop kernel skips this recurrence
          stat_add(P.stats, SDR_PLL_ST_RECURRENCES, 1);
          stat_add(P.stats, SDR_PLL_ST_SPEC_R0 + round, 1);
        }
      }
      return true;
    }
  }
  return false;
}

__device__ void seq_run(const PllCfg& cfg, const float* in, const int8_t* in8, double* th, int64_t n, const double* st,
                        double* so, float* r32 = nullptr, Th32Line* lines = nullptr);

// A per-block call's recurrence the solve does not complete (a 0 / NaN input, a loop not yet
// locked) runs sequentially in the same workgroup (one thread, seq_run's general form) --
// no prep / loop kernels behind the solve, so a per-block PLL call is this launch and the NCO's.
__device__ void spec_fallback(const PllJobs& P, const int bid) {
#pragma clang fp contract(off)
  const int q = bid / P.nstreams, s = bid - q * P.nstreams;
  const PllJob& J = P.j[q];
  const PllCfg cfg = J.cfg;
  double* st = J.state + (int64_t)s * 6;
  double* th = J.theta + (int64_t)s * J.th_stride;
  const double off = st[5];
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  J.nco_i[(int64_t)s * J.out_stride] = (float)st[4];
  if (J.nco_q)
    J.nco_q[(int64_t)s * J.out_stride] = (float)((off > 0.0) ? sin((w * off + st[1]) * cfg.scale + cfg.adj) : 0.0);
  double so[6];
  seq_run(cfg, J.in + (int64_t)s * J.in_stride, J.in8 != nullptr ? J.in8 + (int64_t)s * J.in8_stride : nullptr, th, P.n,
          st, so);
  th[P.n] = off;                                   // the NCO kernel's trigOffset
  for (int i = 0; i < 6; ++i) st[i] = so[i];
  stat_add(P.stats, SDR_PLL_ST_RECURRENCES, 1);
  stat_add(P.stats, SDR_PLL_ST_SEQUENTIAL, 1);
}

// nco[k+1] from phaseEst_k for step k of recurrence g = (job, stream): th_k by the reference's
// formula (fmPll.py:33, sdr_nco.h nco_value), the Q-form row converted back when the loop
// kernels left one.
__device__ __forceinline__ void nco_out(const PllJobs& P, const PllJob& J, int s, double off, int64_t k, double p) {
#pragma clang fp contract(off)
  const double w = 2.0 * kPi * (J.cfg.freq / J.cfg.fs);
  if (P.qform) {                                        // Q_{i+1} -> phase_{i+1}
    const double i = (double)(k % PG);
    p = p - (kPi * J.cfg.ki) * ((i + 1.0) * i * 0.5);
  }
  // the reference's angle grows with the stream (~1e7 rad after a minute): nco_value reduces it
  // by the 3-part Cody-Waite step (exact multiples of 2 pi for |n| < 2^26)
  double sv, cv;
  nco_value<true>(w, J.cfg.scale, J.cfg.adj, k + 1, p, off, &cv, &sv);
  J.nco_i[(int64_t)s * J.out_stride + k + 1] = (float)cv;
  if (J.nco_q) J.nco_q[(int64_t)s * J.out_stride + k + 1] = (float)sv;
}
__device__ __forceinline__ void nco_step(const PllJobs& P, int g, int64_t k) {
  const int q = g / P.nstreams;
  const int s = g - q * P.nstreams;
  const PllJob& J = P.j[q];
  const double* ph = J.theta + (int64_t)s * J.th_stride;
  nco_out(P, J, s, ph[P.n], k, ph[k]);
}
// a recurrence's whole NCO row by one workgroup of NT threads: NB outputs per thread at a time,
// their phases loaded first and their sincos chains independent (one wave per SIMD: the
// chains' latency, not their issue, is what a single pass would wait on)
template <int NT>
__device__ __forceinline__ void nco_row(const PllJobs& P, int g, int tid) {
  constexpr int NB = 4;
  const int q = g / P.nstreams;
  const int s = g - q * P.nstreams;
  const PllJob& J = P.j[q];
  const double* ph = J.theta + (int64_t)s * J.th_stride;
  const double off = ph[P.n];
  for (int64_t k0 = tid; k0 < P.n; k0 += NB * NT) {
    double pv[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) pv[b] = k0 + b * NT < P.n ? ph[k0 + b * NT] : 0.0;
#pragma unroll
    for (int b = 0; b < NB; ++b)
      if (k0 + b * NT < P.n) nco_out(P, J, s, off, k0 + b * NT, pv[b]);
  }
}

template <int SPEC_T, bool LONG>
__global__ __launch_bounds__(SPEC_T) __attribute__((amdgpu_waves_per_eu(SPEC_T == 512 ? 4 : 2))) void pll_spec_kernel(PllJobs P) {
  // (LONG: a long call's first solve of every block, which also initialises its record)
  const bool done = spec_body<SPEC_T, LONG, LONG>(P, (int)blockIdx.x, (int)threadIdx.x);
  if constexpr (!LONG) {
    if (P.lpw == 0) {
      // a per-block call (spec-only): the sequential fallback when the solve could not complete
      // the recurrence, then its NCO row here -- the theta row is this workgroup's own (visible
      // after the barrier), and the NCO needs no launch of its own
      if (!done && threadIdx.x == 0) spec_fallback(P, (int)blockIdx.x);
      if (P.nco_fused) {
        __syncthreads();
        nco_row<SPEC_T>(P, (int)blockIdx.x, (int)threadIdx.x);
      }
    }
  }
}

// ================================================================================
// Long calls (n > SDR_PLL_BLOCK_MAX): a device-resident span of many blocks is one recurrence
// of n steps, cut into nb pseudo-blocks of pb <= LONG_PB (14 336) steps so that every pseudo-block
// (with its pre-roll) is one pll_spec_kernel workgroup and the whole span fills the GPU.  A
// pseudo-block's start state is the previous one's end state, unknown until that one is
// solved, so two launches:
//   1. pll_spec_kernel<512, LONG> (first = 1): every pseudo-block solved (and its record
//      initialised).  One after the first is solved together with a PRE-ROLL: the `warm`
//      steps before it, from the phase the input measures there and the span's start
//      integrator; the loop contracts errors by sqrt(1 - Kp) per step, and its dynamics are
//      invariant under phaseEst -> phaseEst + 2 pi, so the pre-roll's state at the block's
//      start -- its GUESS -- has converged to the true state up to a whole number of turns
//      (the parallel form of a sequential warm-up over the same steps).
//   2. pll_long_fix_kernel (one workgroup per recurrence): the CHAIN -- from the exact state
//      at the chain's position, the 2 pi shift n between the exact start and each block's
//      solved start is taken out, and the remaining start error (dp, dV) bounds the phase
//      deviation of the block's solution by err = c1 |dp| + c2 |dV| (c1, c2: the largest phase
//      excursion the loop's linear form makes from a unit start error):
//        err <= 1e-9 rad: accepted -- its phases + 2 pi n are the recurrence's (to a deviation
//                         below the reference's own rounding of its ~1e6 rad angle), and its
//                         end state + 2 pi n is the next block's exact start;
//        err <= 0.3 rad and every step's wrap margin above err: accepted with the loop's
//                         linear response to the start error (no integer m_k can move; the
//                         NCO kernel adds the response);
//        else:            the chain stops there.
//      A stop is repaired in the same kernel: the block at the chain's position is re-solved
//      from its exact start by the whole workgroup (spec_body; the sequential step if the
//      solve cannot complete it -- a 0 / NaN input), and the chain continues; the blocks after
//      it keep their solutions and are judged again against the new exact prefix.  After
//      LONG_FIXES repairs the rest runs sequentially from the chain's position (never on a
//      locked signal: counted).  On a locked signal the kernel makes one chain pass and exits:
//      no launches for repair rounds that have nothing to do.
//   The NCO kernel adds 2 pi n (and any linear response) to an accepted block's phases.
constexpr double LONG_ACCEPT = 1e-9;   // rad: accepted deviation bound
constexpr double LONG_LINEAR = 0.3;    // rad: deviation bound under which the integers m_k are kept
constexpr double LONG_MARGIN_TOL = 1e-6;   // turns: wrap margin kept clear of rounding
constexpr int LONG_FIXES = 24;         // repairs (re-solves at the chain's position) before the tail

// The reference's recurrence run sequentially from state st over n steps (the general form:
// literal first step from the state's (fI, fQ); 0 / NaN inputs by atan2 on the products; the
// rest by the constants pll_c).  Inputs from `in`, or decoded from the sign codes in8 when
// given.  Phases into th[0..n), the end state into so -- or, compact rows (lines != null, th
// the first row of a line), residuals into r32[0..n) against lines[k / 32], each line set at
// its first row from the phase there and the integrator (the loop's mean step).
__device__ void seq_run(const PllCfg& cfg, const float* in, const int8_t* in8, double* th, int64_t n, const double* st,
                        double* so, float* r32, Th32Line* lines) {
#pragma clang fp contract(off)
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  double integ = st[0], phase = st[1];
  const double off = st[5];
  // inputs 16 at a time, one group ahead (a load per step would wait out the memory latency)
  constexpr int G = 16;
  float xa[G], xn[G];
  Th32Line ln{0.0, 0.0};
  auto ld = [&](float (&v)[G], int64_t k0) {
#pragma unroll
    for (int i = 0; i < G; ++i) v[i] = k0 + i < n ? (in8 != nullptr ? pll_decode(in8[k0 + i]) : in[k0 + i]) : 0.f;
  };
  ld(xa, 0);
  for (int64_t k0 = 0; k0 < n; k0 += G) {
    ld(xn, k0 + G);
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int64_t k = k0 + i;
      if (k >= n) break;
      const float xf = xa[i];
      const double xv = (double)xf;
      double e;
      if (k == 0 || !(xv > 0.0 || xv < 0.0)) {
        double fI = st[2], fQ = st[3];
        if (k > 0) {
          const double arg = w * ((off + (double)(k - 1)) + 1.0) + phase;
          sincos_red<true>(reduce_2pi(arg), &fQ, &fI);
        }
        e = atan2(xv * (-fQ), xv * fI);
      } else {
        const double t = fma(-kInv2Pi, phase, pll_c(xf, w, off + (double)k));
        e = k2Pi * (__builtin_amdgcn_fract(t) - 0.5);
      }
      integ = integ + cfg.ki * e;
      phase = phase + cfg.kp * e + integ;
      if (lines != nullptr) {
        if ((k & (TH32_LINE - 1)) == 0) {
          ln = Th32Line{phase, integ};
          lines[k / TH32_LINE] = ln;
        }
        r32[k] = th32_residual(ln, (int)(k & (TH32_LINE - 1)), phase);
      } else {
        th[k] = phase;
      }
    }
#pragma unroll
    for (int i = 0; i < G; ++i) xa[i] = xn[i];
  }
  const double arg = w * ((off + (double)(n - 1)) + 1.0) + phase;
  so[0] = integ;
  so[1] = phase;
  end_trig(arg, cfg.scale, cfg.adj, so);
  so[5] = off + (double)n;
}

// The chain pass (CHAIN_T threads, one per pseudo-block of a CHAIN_T-block window; the
// windows in order).  With A_j the start block j's current solution was solved from, E_j its
// end and S_j the chained start, the residual R_j = S_j - A_j splits into n_j whole turns and
// rho_j = R_j - 2 pi n_j, and
//     R_{j+1} = (E_j - A_{j+1}) + 2 pi n_j + Phi_j rho_j.
// The turns are a prefix sum of the local integers rint((E_j - A_{j+1})_phase / 2 pi), and with
// C_j = E_j - A_{j+1} less its turns, rho_{j+1} = C_j + Phi rho_j (Phi = A^pb, the loop matrix
// over a pseudo-block): an exact scan below (Phi is ~1e-8 over a long call's pseudo-block but
// ~0.1 over a split per-block call's on the RDS loop).  Then per block the bound
// err = c1 |rho_p| + c2 |rho_v| decides, as described above.  The accepted
// prefix moves the chain's position; the first block after it that is not accepted gets its
// exact start (LB_NEED_X) for a re-solve.  Returns the new position (every thread).
constexpr int CHAIN_T = 512;
__device__ int chain_pass(const PllJobs& P, const int r) {
#pragma clang fp contract(off)
  constexpr int NWV = CHAIN_T / 64;
  __shared__ double sA[2][CHAIN_T + 1];    // A_j (phase, integrator), and the next window's first
  __shared__ double sC[2][CHAIN_T];        // C_j
  __shared__ double sE[3][CHAIN_T];        // E_j + 2 pi n_j (phase), E_j (integrator), and n_j
  __shared__ double sR[2][CHAIN_T];        // rho_j
  __shared__ double wtot[NWV];
  __shared__ int wfa[NWV];
  __shared__ int spos;
  __shared__ Mat2 fpw[10];                 // Phi^(2^i): Phi = A^pb, the loop over one pseudo-block
  __shared__ double wY[2][NWV];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nb = P.lg.nb;
  LongHdr* H = long_hdr(P, r);
  __syncthreads();                          // (the previous pass / re-solve: records written)
  const int pos0 = H->pos;
  if (pos0 >= nb) return pos0;
  const int q = r / P.nstreams, s = r - q * P.nstreams;
  const PllJob& J = P.j[q];
  const PllCfg cfg = J.cfg;
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  const double c1 = P.lg.c1[q], c2 = P.lg.c2[q];
  double* st = J.state + (int64_t)s * 6;
  const double off0 = st[5];
  const int64_t pb = P.lg.pb;
  if (tid == 0) {
    const double* pp = P.lg.phi[q];
    Mat2 x{pp[0], pp[1], pp[2], pp[3]};
    for (int i = 0; i < 10; ++i, x = mmul(x, x)) fpw[i] = x;
  }
  __syncthreads();
  double Cp = H->sp, Ci = H->si;     // the carried (exact) start of the window's first block
  int pos = pos0;
  double Xp = Cp, Xi = Ci;           // the exact state at `pos`
  for (int w0 = pos0; w0 < nb; w0 += CHAIN_T) {
    const int j = w0 + tid;
    const bool valid = j < nb;
    int sj = -1, solver = 0;
    double ap = 0.0, ai = 0.0, ep = 0.0, ei = 0.0, margin = -1.0;
    if (valid) {
      const LongBlk* B = long_blk(P, r, j);
      sj = B->status;
      const bool fromg = sj == LB_DONE_G;
      ap = fromg ? B->g[1] : B->x[1];
      ai = fromg ? B->g[0] : B->x[0];
      ep = B->e[1];
      ei = B->e[0];
      solver = B->solver;
      margin = B->margin;
    }
    const bool solved = valid && (sj == LB_DONE_G || sj == LB_DONE_X);
    sA[0][tid] = ap;
    sA[1][tid] = ai;
    if (tid == CHAIN_T - 1) {                       // the next window's first block
      double np = 0.0, ni = 0.0;
      if (j + 1 < nb) {
        const LongBlk* B = long_blk(P, r, j + 1);
        const bool fromg = B->status == LB_DONE_G;
        np = fromg ? B->g[1] : B->x[1];
        ni = fromg ? B->g[0] : B->x[0];
      }
      sA[0][CHAIN_T] = np;
      sA[1][CHAIN_T] = ni;
    }
    __syncthreads();
    const double anp = sA[0][tid + 1], ani = sA[1][tid + 1];
    const double a0p = sA[0][0], a0i = sA[1][0];
    // C_j = E_j - A_{j+1} less its turns (this block's outgoing step)
    const double cd = ep - anp;
    const double dn = rint(cd * kInv2Pi);
    const double cp = fma(-dn, kP2, fma(-dn, kP1, cd));
    const double cv = ei - ani;
    sC[0][tid] = cp;
    sC[1][tid] = cv;
    // the first block's residual from the carried start
    const double d0 = Cp - a0p;
    const double n0 = rint(d0 * kInv2Pi);
    const double r0p = fma(-n0, kP2, fma(-n0, kP1, d0)), r0v = Ci - a0i;
    // whole turns: n_0 from the carry, then the prefix sum of the outgoing integers
    double pre_dn = wave_prefix_sum(dn, lane);
    if (lane == 63) wtot[wv] = pre_dn;
    __syncthreads();
    for (int i = 0; i < wv; ++i) pre_dn += wtot[i];
    const double nj = n0 + (pre_dn - dn);
    // rho_l = C_{l-1} + Phi rho_{l-1} (rho_0: the carried residual), exactly: with the inclusive
    // scan Y_l = sum_{i<=l} Phi^(l-i) C_i, rho_l = Y_{l-1} + Phi^l rho_0.  (Phi = A^pb is tiny
    // for the long calls' 14 336-step pseudo-blocks -- there rho_l = C_{l-1} + Phi C_{l-2}
    // already -- but not for a split per-block call's ~1 500-step ones on the RDS loop,
    // where Phi ~ 0.1: its powers must be carried.)
    double rp, rv;
    {
      double yp = cp, yv = cv;
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int o = 1 << i;
        const double up = __shfl_up(yp, o, 64), uv = __shfl_up(yv, o, 64);
        if (lane >= o) {
          const Mat2 F = fpw[i];
          yp = yp + (F.a * up + F.b * uv);
          yv = yv + (F.c * up + F.d * uv);
        }
      }
      if (lane == 63) { wY[0][wv] = yp; wY[1][wv] = yv; }
      __syncthreads();
      double cwp = 0.0, cwv = 0.0;                   // Y at the end of the previous wave
      for (int i = 0; i < wv; ++i) {
        const Mat2 F = fpw[6];                       // Phi^64
        const double np = wY[0][i] + (F.a * cwp + F.b * cwv), nv = wY[1][i] + (F.c * cwp + F.d * cwv);
        cwp = np; cwv = nv;
      }
      {
        Mat2 Fl{1.0, 0.0, 0.0, 1.0};                 // Phi^(lane + 1)
        for (int i = 0, e = lane + 1; e > 0; ++i, e >>= 1)
          if (e & 1) Fl = mmul(Fl, fpw[i]);
        yp = yp + (Fl.a * cwp + Fl.b * cwv);
        yv = yv + (Fl.c * cwp + Fl.d * cwv);
      }
      // Y_{tid-1}: the previous lane's (lane 0: the previous wave's last, through LDS)
      double vp = __shfl_up(yp, 1, 64), vv = __shfl_up(yv, 1, 64);
      __syncthreads();                               // wY read before it is rewritten
      if (lane == 63) { wY[0][wv] = yp; wY[1][wv] = yv; }
      __syncthreads();
      if (lane == 0) {
        vp = wv > 0 ? wY[0][wv - 1] : 0.0;
        vv = wv > 0 ? wY[1][wv - 1] : 0.0;
      }
      Mat2 Ft{1.0, 0.0, 0.0, 1.0};                   // Phi^tid
      for (int i = 0, e = tid; e > 0; ++i, e >>= 1)
        if (e & 1) Ft = mmul(Ft, fpw[i]);
      rp = vp + (Ft.a * r0p + Ft.b * r0v);
      rv = vv + (Ft.c * r0p + Ft.d * r0v);
      if (tid == 0) { rp = r0p; rv = r0v; }
    }
    const double err = c1 * fabs(rp) + c2 * fabs(rv);
    // accepted: the solve started within LONG_ACCEPT of the chained start, or within the linear
    // bound with every step's wrap further from the boundary than the largest phase deviation
    // err (then no integer m_k moves: the block's phases + its linear response to the start
    // error rho are the recurrence's, up to rounding -- nco_long_kernel adds the response)
    const bool lina = err <= LONG_LINEAR && k2Pi * (margin - LONG_MARGIN_TOL) > err;
    const bool acc = solved && (err <= LONG_ACCEPT || lina);   // (a NaN fails both)
    {                                                // the first block not accepted (CHAIN_T: none)
      const uint64_t na = __ballot(!acc);           // (invalid blocks are not accepted)
      if (lane == 0) wfa[wv] = na ? wv * 64 + __builtin_ctzll(na) : CHAIN_T;
    }
    const double ejp = fma(nj, kP1, fma(nj, kP2, ep));  // E_j + 2 pi n_j
    sE[0][tid] = ejp;
    sE[1][tid] = ei;
    sE[2][tid] = nj;
    sR[0][tid] = rp;
    sR[1][tid] = rv;
    __syncthreads();
    int nacc = CHAIN_T;
    for (int i = 0; i < NWV; ++i) nacc = min(nacc, wfa[i]);
    if (valid && tid < nacc) {
      LongBlk* B = long_blk(P, r, j);
      B->status = LB_ACCEPTED;
      B->shift = nj;
      B->d[0] = err <= LONG_ACCEPT ? 0.0 : rp;      // the linear response the NCO kernel adds
      B->d[1] = err <= LONG_ACCEPT ? 0.0 : rv;
    } else if (valid && tid == nacc) {              // the chain's next block: its exact start
      // S_j = A_j + 2 pi n_j + rho_j when it was solved; else the previous block's end + its
      // turns + Phi rho (block `pos0`: the carry)
      double sp, si;
      if (solved) {
        sp = fma(nj, kP1, fma(nj, kP2, ap)) + rp;
        si = ai + rv;
      } else if (tid == 0) {
        sp = Cp;
        si = Ci;
      } else {
        const double* pp = P.lg.phi[q];
        sp = sE[0][tid - 1] + (pp[0] * sR[0][tid - 1] + pp[1] * sR[1][tid - 1]);
        si = sE[1][tid - 1] + (pp[2] * sR[0][tid - 1] + pp[3] * sR[1][tid - 1]);
      }
      LongBlk* B = long_blk(P, r, j);
      B->u[0] = ai;
      B->u[1] = ap;
      B->solver = -1;
      if (j == 0) {                                 // the call's own first step: its state as given
        for (int i = 0; i < 6; ++i) B->x[i] = st[i];
      } else {
        const double offp = off0 + (double)((int64_t)(j - 1) * pb);
        const double arg = w * ((offp + (double)(pb - 1)) + 1.0) + sp;
        B->x[0] = si;
        B->x[1] = sp;
        sincos_red<true>(reduce_2pi(arg), &B->x[3], &B->x[2]);
        B->x[4] = 0.0;
        B->x[5] = off0 + (double)((int64_t)j * pb);
      }
      B->shift = 0.0;
      B->d[0] = B->d[1] = 0.0;
      B->status = LB_NEED_X;
    }
    {                                                   // the counters, one atomic per wave each
      const bool a = valid && tid < nacc, ex = err <= LONG_ACCEPT;
      stat_add_wave(P.stats, SDR_PLL_ST_RECURRENCES, a);
      stat_add_wave(P.stats, SDR_PLL_ST_SEQUENTIAL, a && solver == SOLVER_SEQ);
      for (int r0 = 0; r0 < SPEC_IT; ++r0) stat_add_wave(P.stats, SDR_PLL_ST_SPEC_R0 + r0, a && solver == r0);
      stat_add_wave(P.stats, SDR_PLL_ST_LONG_GUESSED, a && sj == LB_DONE_G && ex);
      stat_add_wave(P.stats, SDR_PLL_ST_LONG_CHAINED, a && !(sj == LB_DONE_G && ex));
      stat_add_wave(P.stats, SDR_PLL_ST_LONG_LINEAR, a && !ex);
      stat_max_wave(P.stats, SDR_PLL_ST_LONG_MAXGAP, a && ex, err);
      stat_add_wave(P.stats, SDR_PLL_ST_LONG_STOPS, valid && tid == nacc);
    }
    // the state after the accepted prefix: E + 2 pi n + Phi rho of its last block
    if (nacc > 0) {
      const int l = nacc - 1;
      const double* phl = (w0 + l == nb - 1) ? P.lg.phi_last[q] : P.lg.phi[q];
      Xp = sE[0][l] + (phl[0] * sR[0][l] + phl[1] * sR[1][l]);
      Xi = sE[1][l] + (phl[2] * sR[0][l] + phl[3] * sR[1][l]);
      pos = min(w0 + nacc, nb);
    }
    if (nacc < CHAIN_T || w0 + CHAIN_T >= nb) break;   // stopped, or the last window
    Cp = Xp;                                            // carry: the exact state at the next window
    Ci = Xi;
    __syncthreads();                                    // the window's LDS read before the next writes it
  }
  if (tid == 0) {
    H->pos = pos;
    H->sp = Xp;
    H->si = Xi;
    if (pos == nb) {                                                   // the call's state
      const double offl = off0 + (double)((int64_t)(nb - 1) * pb);
      const double arg = w * ((offl + (double)(long_len(P, nb - 1) - 1)) + 1.0) + Xp;
      st[0] = Xi;
      st[1] = Xp;
      end_trig(arg, cfg.scale, cfg.adj, st);
      st[5] = off0 + (double)P.n;
    }
    spos = pos;
  }
  __syncthreads();
  return spos;
}

// Sequential from the chain's exact position to the end (after LONG_FIXES repairs), by one thread.
__device__ void long_tail(const PllJobs& P, const int r, const int pos) {
#pragma clang fp contract(off)
  const int nb = P.lg.nb;
  LongHdr* H = long_hdr(P, r);
  const int q = r / P.nstreams, s = r - q * P.nstreams;
  const PllJob& J = P.j[q];
  const PllCfg cfg = J.cfg;
  double* st = J.state + (int64_t)s * 6;
  for (int b = pos + (int)threadIdx.x; b < nb; b += blockDim.x) {
    long_blk(P, r, b)->shift = 0.0;
    long_blk(P, r, b)->d[0] = long_blk(P, r, b)->d[1] = 0.0;
  }
  if (threadIdx.x != 0) return;
  const int64_t pb = P.lg.pb;
  const int64_t base = (int64_t)pos * pb;
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  const double off0 = st[5];
  double s0[6];
  if (pos == 0) {
    for (int i = 0; i < 6; ++i) s0[i] = st[i];
  } else {
    const double offp = off0 + (double)(base - pb);
    const double arg = w * ((offp + (double)(pb - 1)) + 1.0) + H->sp;
    s0[0] = H->si; s0[1] = H->sp; s0[4] = 0.0; s0[5] = off0 + (double)base;
    sincos_red<true>(reduce_2pi(arg), &s0[3], &s0[2]);
  }
  double so[6];
  double* rowp = J.theta + (int64_t)s * J.th_stride;
  seq_run(cfg, J.in + (int64_t)s * J.in_stride + base,
          J.in8 != nullptr ? J.in8 + (int64_t)s * J.in8_stride + base : nullptr, rowp + base, P.n - base, s0, so,
          J.th32 ? th32_res(rowp) + base : nullptr, J.th32 ? th32_lines(rowp, P.n) + base / TH32_LINE : nullptr);
  for (int i = 0; i < 5; ++i) st[i] = so[i];
  st[5] = off0 + (double)P.n;
  H->pos = nb;
  stat_add(P.stats, SDR_PLL_ST_RECURRENCES, (unsigned long long)(nb - pos));
  stat_add(P.stats, SDR_PLL_ST_SEQUENTIAL, (unsigned long long)(nb - pos));
  stat_add(P.stats, SDR_PLL_ST_LONG_TAIL, (unsigned long long)(nb - pos));
}

// 2. The chain with its repairs: one workgroup per recurrence (CHAIN_T == the solve's 512
// threads, so spec_body runs in it).  Locked signal: one chain pass, done.
static_assert(CHAIN_T == 512, "pll_long_fix_kernel runs spec_body<512, true>");
__global__ __launch_bounds__(CHAIN_T) void pll_long_fix_kernel(PllJobs P) {
  const int r = blockIdx.x;
  const int nb = P.lg.nb;
  int pos = chain_pass(P, r);
  for (int fix = 0; pos < nb; ++fix) {
    if (fix == LONG_FIXES) {
      long_tail(P, r, pos);
      return;
    }
    // the block at the chain's position has its exact start (LB_NEED_X): solve it in parallel.
    // (The thread index goes in opaque: otherwise the compiler hoists the solve's per-thread
    // LDS addresses out of this loop for its whole length, and spills.)
    int tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
    spec_body<512, true>(P, r * nb + pos, tid);
    __syncthreads();
    LongBlk* B = long_blk(P, r, pos);
    if (threadIdx.x == 0 && B->status == LB_NEED_X) {   // not completed (0 / NaN input): the sequential step
      const int q = r / P.nstreams, s = r - q * P.nstreams;
      const PllJob& J = P.j[q];
      const int64_t base = (int64_t)pos * P.lg.pb;
      double* rowp = J.theta + (int64_t)s * J.th_stride;
      seq_run(J.cfg, J.in + (int64_t)s * J.in_stride + base,
              J.in8 != nullptr ? J.in8 + (int64_t)s * J.in8_stride + base : nullptr, rowp + base, long_len(P, pos),
              B->x, B->e, J.th32 ? th32_res(rowp) + base : nullptr,
              J.th32 ? th32_lines(rowp, P.n) + base / TH32_LINE : nullptr);
      B->u[0] = B->x[0];
      B->u[1] = B->x[1];
      B->d[0] = B->d[1] = 0.0;
      B->margin = -1.0;                              // (general steps: no linear acceptance)
      B->status = LB_DONE_X;
      B->solver = SOLVER_SEQ;
    }
    pos = chain_pass(P, r);
  }
}

// Per-sample constants of the loop (parallel): c_k = (sel_k - w (off + k)) / 2pi + 1/2 and one flag per
// PG-sample group holding a 0 or NaN input; c row layout: c[0..n) | flags[0..n/PG).
__global__ __launch_bounds__(256) void pll_prep_kernel(PllJobs P) {
#pragma clang fp contract(off)
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int g = blockIdx.y;                 // uniform: (job, stream)
  const int q = g / P.nstreams;
  const int s = g - q * P.nstreams;
  const PllJob& J = P.j[q];
  const double off = J.off_given ? J.off : J.state[(int64_t)s * 6 + 5];
  const double w = 2.0 * kPi * (J.cfg.freq / J.cfg.fs);
  double* c = J.cbuf + (int64_t)s * J.c_stride;
  bool odd = false;
  if (k < P.n) {
    const float x = J.in[(int64_t)s * J.in_stride + k];
    odd = !(x > 0.f || x < 0.f);
    // pll_c (the previous step's w (off + k)); a 0 / NaN input gets a NaN constant: a fast
    // group over it ends in a NaN phase, which pll_chunk_kernel takes as its signal to redo
    // the group in the general form
    double cv = fma(-(off + (double)k), w * kInv2Pi, x > 0.f ? 0.5 : 1.0);
    if (P.qform) {                                      // pll_chunk_kernel's Q-form
      const double i = (double)(k % PG);
      cv = cv + (kPi * J.cfg.ki) * kInv2Pi * (i * (i - 1.0) * 0.5);
    }
    c[k] = odd ? __builtin_nan("") : cv;
  }
  // groups of PG = 32 lanes: the low and high half of each wave
  const uint64_t m = __ballot(odd);
  const int lane = threadIdx.x & 63;
  const int64_t grp = k / PG;
  if ((lane == 0 || lane == 32) && grp < P.n / PG)
    c[P.n + grp] = ((lane == 0 ? (m & 0xffffffffull) : (m >> 32)) != 0) ? 1.0 : 0.0;
}

// nco[k+1] from phaseEst_k for every (job, stream) of the table (th_k by the reference's
// formula, fmPll.py:33); nco[0] is the loop kernel's.
__global__ void nco_jobs_kernel(PllJobs P) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < P.n) nco_step(P, (int)blockIdx.y, k);
}


// The NCO of a long call: phaseEst_k = the stored phase + 2 pi (the chain's turns for its
// pseudo-block) + (A^(kk+1) d)_phase, the loop's linear response to the start error d the
// chain accepted the pseudo-block with (kk: the step within it; zero for most blocks), from
// the response table (sdr_nco.h nco_phase_in: the receiver's mixers form the same double).
// Workgroup: 256 x NCO_NR consecutive steps of ONE pseudo-block (grid.x = pseudo-blocks x
// tiles per block), thread t the steps t + 256 i (coalesced).  Runs only when an NCO row is an
// output (P.nco_rows); the receiver's mixers otherwise take the phases directly.
constexpr int NCO_NR = 8;              // outputs per thread of nco_long_kernel
__host__ __device__ inline int nco_tiles_per_block(int64_t pb) { return (int)((pb + 256 * NCO_NR - 1) / (256 * NCO_NR)); }
__global__ __launch_bounds__(256) void nco_long_kernel(PllJobs P) {
#pragma clang fp contract(off)
  const int g = blockIdx.y;                 // uniform: (job, stream) = the recurrence
  const int q = g / P.nstreams;
  const int s = g - q * P.nstreams;
  const PllJob& J = P.j[q];
  const PllCfg cfg = J.cfg;
  const int64_t pb = P.lg.pb;
  const int tpb = nco_tiles_per_block(pb);
  const int b = (int)blockIdx.x / tpb;
  const int64_t kb = (int64_t)b * pb;                          // the pseudo-block's first step
  const int64_t kk0 = (int64_t)((int)blockIdx.x - b * tpb) * (256 * NCO_NR);
  const int64_t len = min(pb, P.n - kb);
  if (kk0 >= len) return;                                      // uniform
  const LongBlk* B = long_blk(P, g, b);
  const double* ph = J.theta + (int64_t)s * J.th_stride;
  const double off = ph[P.n];
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  // every phase of the thread is loaded before the first is used (one memory round trip)
  const int64_t k0 = kb + kk0 + threadIdx.x;
  const int64_t kend = kb + len;
  double phv[NCO_NR];
#pragma unroll
  for (int i = 0; i < NCO_NR; ++i) {
    const int64_t k = k0 + (int64_t)i * 256;
    phv[i] = k < kend ? (J.th32 ? th32_stored(ph, P.n, k) : ph[k]) : 0.0;
  }
  float* oi = J.nco_i + (int64_t)s * J.out_stride + 1;
  float* oq = J.nco_q ? J.nco_q + (int64_t)s * J.out_stride + 1 : nullptr;
#pragma unroll
  for (int i = 0; i < NCO_NR; ++i) {
    const int64_t k = k0 + (int64_t)i * 256;
    if (k >= kend) break;
    const double p = nco_phase_in(B, k - kb, J.resp, phv[i]);
    double sv, cv;
    nco_value<true>(w, cfg.scale, cfg.adj, k + 1, p, off, &cv, &sv);
    oi[k] = (float)cv;
    if (oq) oq[k] = (float)sv;
  }
}

}  // namespace

namespace {
// the job table's strides and whether every row allows 16-B loads / stores
// recurrences per wave as the loop launcher picks them, and whether pll_chunk_kernel (and so
// the Q-form, which the prep and NCO kernels must agree on) runs
int pll_lpw(const PllJobs& P) {
  int lpw = 1;
  while (lpw < 64 && P.njobs * ((P.nstreams + lpw - 1) / lpw) > kMaxPllWaves) lpw *= 2;
  return lpw;
}
// a per-block call (n >= 2) is solved by pll_spec_kernel alone (its own sequential fallback):
// no prep or loop kernel, plain (not Q-form) phase rows, and its NCO rows (when asked for,
// P.nco_rows) written by the solve's own launch.  The sequential kernels run 1-sample calls.
bool spec_only(const PllJobs& P) { return P.n >= 2; }
hipError_t pll_check(const PllJobs& P, bool* vec) {
  if (P.njobs < 1 || P.njobs > SDR_PLL_MAXJ || P.nstreams <= 0 || P.n < 0) return hipErrorInvalidValue;
  *vec = true;
  for (int q = 0; q < P.njobs; ++q) {
    const PllJob& J = P.j[q];
    if (J.th_stride < P.n + 1 || J.c_stride < P.n + P.n / PG) return hipErrorInvalidValue;
    *vec = *vec && ((uintptr_t)J.cbuf % 16) == 0 && (J.c_stride % 2) == 0 && ((uintptr_t)J.theta % 16) == 0 &&
           (J.th_stride % 2) == 0;
  }
  return hipSuccess;
}
}  // namespace

namespace {
// ---- long calls: host-side setup ---------------------------------------------------
// (r04 measured splitting per-block calls into pseudo-blocks too -- slower: every
// pseudo-block pays its pre-roll; removed in r05)
bool long_n(int64_t n) { return n > SPEC_NMAX; }
bool pll_long(const PllJobs& P) { return long_n(P.n); }

// pseudo-blocks of <= LONG_PB steps: with a pre-roll of <= LONG_PRE_MAX steps one solve is at
// most SPEC_NMAX - 1 steps (its LDS image)
constexpr int LONG_PRE_MAX = 2048;
constexpr int LONG_PB = SPEC_NMAX - 1 - LONG_PRE_MAX;
// r06: pseudo-blocks of exactly LONG_PB steps (the last one shorter) whenever that leaves the
// last at least 2 steps -- so that with the LONG_PRE_MAX + 1-step pre-roll (warm_len) a middle
// pseudo-block's solve is SPEC_NMAX steps: 512 full chunks of 32, every wave on the full-chunk
// loops, and the pre-roll exactly the first wave's chunks (r05 balanced the lengths, 14 299 at
// a C5 span: the last wave ran its partial chunk's predicated loops and the workgroup's
// barriers waited for it -- the phase timers' guess and check barriers)
static_assert(TH32_LINES * TH32_LINE >= LONG_PB, "compact rows: a pseudo-block's lines fit the solve's table");
void long_geom(int64_t n, int64_t* pb, int* nb) {
  const int64_t k = (n + LONG_PB - 1) / LONG_PB;
  *nb = (int)k;
  *pb = n - (k - 1) * LONG_PB >= 2 ? LONG_PB : (n + k - 1) / k;
}

// the loop's linear form on the start error (dphaseEst, dV): A = [[1 - kC/2pi, 1], [-kA/2pi, 1]]
struct M2 { double a, b, c, d; };
M2 mul(const M2& x, const M2& y) {
  return {x.a * y.a + x.b * y.c, x.a * y.b + x.b * y.d, x.c * y.a + x.d * y.c, x.c * y.b + x.d * y.d};
}
M2 loop_matrix(const PllCfg& c) {
  const double kA = 2.0 * M_PI * c.ki, kC = 2.0 * M_PI * (c.kp + c.ki);
  return {1.0 - kC / (2.0 * M_PI), 1.0, -kA / (2.0 * M_PI), 1.0};
}
M2 mpow(M2 x, int64_t e) {
  M2 r{1.0, 0.0, 0.0, 1.0};
  for (; e > 0; e >>= 1, x = mul(x, x))
    if (e & 1) r = mul(r, x);
  return r;
}
// c1, c2: the largest |phase deviation| over the steps after a unit start error in phaseEst
// (c1) or in the integrator (c2), iterated until the loop has damped it (cached per loop)
struct Bounds { double kp, ki, c1, c2; };
void loop_bounds(const PllCfg& c, double* c1, double* c2) {
  static std::mutex mu;
  static Bounds cache[16];
  static int ncache = 0;
  std::lock_guard<std::mutex> g(mu);
  for (int i = 0; i < ncache; ++i)
    if (cache[i].kp == c.kp && cache[i].ki == c.ki) { *c1 = cache[i].c1; *c2 = cache[i].c2; return; }
  const M2 A = loop_matrix(c);
  double p1 = 1.0, v1 = 0.0, p2 = 0.0, v2 = 1.0, m1 = 1.0, m2 = 0.0;
  for (int k = 0; k < 400000; ++k) {
    const double np1 = A.a * p1 + A.b * v1, nv1 = A.c * p1 + A.d * v1;
    const double np2 = A.a * p2 + A.b * v2, nv2 = A.c * p2 + A.d * v2;
    p1 = np1; v1 = nv1; p2 = np2; v2 = nv2;
    m1 = std::max(m1, std::fabs(p1));
    m2 = std::max(m2, std::fabs(p2));
    if (k > 64 && std::fabs(p1) + std::fabs(v1) < 1e-6 * m1 && std::fabs(p2) + std::fabs(v2) < 1e-6 * m2) break;
  }
  if (ncache < 16) cache[ncache++] = Bounds{c.kp, c.ki, m1, m2};
  *c1 = m1;
  *c2 = m2;
}

// pre-roll length: the error contracts by sqrt(1 - Kp) per step; enough steps to bring the
// seed's error (the measured phase: ~0.1 rad) within LONG_ACCEPT (the stereo loop: ~1 500),
// unless that exceeds LONG_PRE_MAX = 2 048 (the RDS loop would need ~15 000) -- then 1 024
// steps, enough for the linear bound; such blocks are fixed up from the chained start.
// Full-length pseudo-blocks (long_geom) take LONG_PRE_MAX + 1 = 2 049 for both loops.
int warm_len(const PllCfg& c, double c1, int64_t pb) {
  // full-length pseudo-blocks: the pre-roll fills the solve (SPEC_NMAX steps), longer than
  // either loop needs (below) -- chunk-aligned: the first wave's 64 x 32 steps exactly
  if (pb == LONG_PB) return SPEC_NMAX - LONG_PB;
  constexpr int cap = LONG_PRE_MAX;
  const double rate = -0.5 * std::log1p(-std::min(std::max(c.kp, 1e-12), 0.999));
  const double want = std::log(std::max(c1, 1.0) * 0.1 / LONG_ACCEPT) / rate;   // from a 0.1 rad seed
  int64_t wl = (int64_t)std::ceil(want / 256.0) * 256;
  if (wl > cap) wl = 1024;            // cannot reach the acceptance bound: enough for the linear one
  wl = std::min<int64_t>(wl, pb / 2);
  return (int)std::max<int64_t>(wl, 64);
}

hipError_t long_setup(PllJobs& L) {
  if (L.work == nullptr) return hipErrorInvalidValue;
  long_geom(L.n, &L.lg.pb, &L.lg.nb);
  const int64_t last = L.n - (int64_t)(L.lg.nb - 1) * L.lg.pb;
  if (last < 2) return hipErrorInvalidValue;
  for (int q = 0; q < L.njobs; ++q) {
    const PllCfg& c = L.j[q].cfg;
    loop_bounds(c, &L.lg.c1[q], &L.lg.c2[q]);
    const M2 A = loop_matrix(c);
    const M2 F = mpow(A, L.lg.pb), G = mpow(A, last);
    const double f[4] = {F.a, F.b, F.c, F.d}, g[4] = {G.a, G.b, G.c, G.d};
    for (int i = 0; i < 4; ++i) { L.lg.phi[q][i] = f[i]; L.lg.phi_last[q][i] = g[i]; }
    L.lg.warm[q] = warm_len(c, L.lg.c1[q], L.lg.pb);
  }
  return hipSuccess;
}
// compact phase rows (PllJob::th32): long calls whose pseudo-blocks start on a line only
hipError_t th32_check(const PllJobs& L) {
  for (int q = 0; q < L.njobs; ++q)
    if (L.j[q].th32 && (!pll_long(L) || L.lg.pb % TH32_LINE != 0)) return hipErrorInvalidValue;
  return hipSuccess;
}
}  // namespace

bool sdr_pll_long_geom(int64_t n, int64_t* pb, int* nb) {
  if (!long_n(n)) return false;
  long_geom(n, pb, nb);
  return true;
}

void sdr_pll_resp_table(const PllCfg& c, int64_t n, std::vector<double>* out) {
  out->clear();
  int64_t pb;
  int nb;
  if (!sdr_pll_long_geom(n, &pb, &nb)) return;
  const M2 A = loop_matrix(c);
  out->resize(2 * (size_t)(pb + 1 + 4));
  double r0 = 1.0, r1 = 0.0;                        // row 0 of A^j, j = 0, 1, ...
  for (int64_t j = 0; j <= pb; ++j) {
    (*out)[2 * j] = r0;
    (*out)[2 * j + 1] = r1;
    const double n0 = r0 * A.a + r1 * A.c, n1 = r0 * A.b + r1 * A.d;
    r0 = n0;
    r1 = n1;
  }
  // rows pb + 1 .. pb + 4 repeat rows 1 .. 4: a consumer reading four consecutive steps' rows
  // from one pseudo-block's base (sdr_nco.h nco4_load) reads the next block's first rows there
  for (int64_t t = 1; t <= 4; ++t) {
    (*out)[2 * (pb + t)] = (*out)[2 * t];
    (*out)[2 * (pb + t) + 1] = (*out)[2 * t + 1];
  }
}

int64_t sdr_pll_work_bytes(int njobs, int nstreams, int64_t n) {
  if (!long_n(n)) return 0;
  int64_t pb;
  int nb;
  long_geom(n, &pb, &nb);
  const int64_t R = (int64_t)njobs * nstreams;
  return R * (int64_t)sizeof(LongHdr) + R * nb * (int64_t)sizeof(LongBlk);
}

// The solve's matrix powers for loop c (QT_NL x QT_N matrices, row-major 2x2 doubles), formed
// with the arithmetic the device used to (r05: thread 0 computed them in every workgroup):
// Q = A^L as P <- A P, L times; Q^(2^i) by squaring; Q^e as the product of the Q^(2^i) of e's
// bits, lowest first -- separate roundings (no contraction).
namespace {
struct HM2 { double a, b, c, d; };
HM2 hmul(const HM2& x, const HM2& y) {
#pragma clang fp contract(off)
  return {x.a * y.a + x.b * y.c, x.a * y.b + x.b * y.d, x.c * y.a + x.d * y.c, x.c * y.b + x.d * y.d};
}
void qtab_host(const PllCfg& cfg, std::vector<double>* out) {
#pragma clang fp contract(off)
  const double kA = k2Pi * cfg.ki, kC = k2Pi * (cfg.kp + cfg.ki);
  const double a00 = 1.0 - kC * kInv2Pi, a10 = -kA * kInv2Pi;
  out->assign((size_t)QT_NL * QT_N * 4, 0.0);
  for (int li = 0; li < QT_NL; ++li) {
    const int L = (li + 1) * SB;
    double P00 = 1.0, P01 = 0.0, P10 = 0.0, P11 = 1.0;
    for (int i = 0; i < L; ++i) {
      const double n00 = a00 * P00 + P10, n01 = a00 * P01 + P11;
      const double n10 = a10 * P00 + P10, n11 = a10 * P01 + P11;
      P00 = n00; P01 = n01; P10 = n10; P11 = n11;
    }
    HM2 q[10];
    HM2 x{P00, P01, P10, P11};
    for (int i = 0; i < 10; ++i, x = hmul(x, x)) q[i] = x;
    auto pw = [&](int e) {                          // Q^e from the Q^(2^i) of e's bits, lowest first
      HM2 r{1.0, 0.0, 0.0, 1.0};
      for (int i = 0; e > 0; ++i, e >>= 1)
        if (e & 1) r = hmul(r, q[i]);
      return r;
    };
    HM2* t = reinterpret_cast<HM2*>(out->data()) + (size_t)li * QT_N;
    for (int e = 0; e <= 64; ++e) t[e] = pw(e);
    for (int w = 0; w < 8; ++w) t[65 + w] = pw(64 * w);
  }
}
// device copies, per (device, kp, ki), for the life of the process (QT_NL x QT_N x 32 B = 12 KB each)
struct QTab { int dev; double kp, ki; double* d; };
hipError_t qtab_get(const PllCfg& cfg, const double** out) {
  static std::mutex mu;
  static std::vector<QTab> cache;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(mu);
  for (const QTab& t : cache)
    if (t.dev == dev && t.kp == cfg.kp && t.ki == cfg.ki) { *out = t.d; return hipSuccess; }
  std::vector<double> h;
  qtab_host(cfg, &h);
  QTab t{dev, cfg.kp, cfg.ki, nullptr};
  e = hipMalloc(&t.d, sizeof(double) * h.size());
  if (e == hipSuccess) e = hipMemcpy(t.d, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice);
  if (e != hipSuccess) return e;
  cache.push_back(t);
  *out = t.d;
  return hipSuccess;
}
hipError_t qtab_fill(PllJobs& L) {
  for (int q = 0; q < L.njobs; ++q) {
    const hipError_t e = qtab_get(L.j[q].cfg, &L.j[q].qtab);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
}  // namespace

hipError_t sdr_launch_pll_prep(const PllJobs& P, hipStream_t st) {
  bool vec;
  const hipError_t e = pll_check(P, &vec);
  if (e != hipSuccess) return e;
  if (pll_long(P) || spec_only(P)) return hipSuccess;   // the solve computes its constants where it uses them (pll_c)
  for (int q = 0; q < P.njobs; ++q)
    if (P.j[q].in8 != nullptr) return hipErrorInvalidValue;
  PllJobs L = P;
  L.qform = !pll_long(P) && vec && pll_lpw(P) == 1;
  if (P.n > 0)
    hipLaunchKernelGGL(pll_prep_kernel, dim3((unsigned)((P.n + 255) / 256), (unsigned)(P.njobs * P.nstreams)),
                       dim3(256), 0, st, L);
  return hipGetLastError();
}

hipError_t sdr_launch_pll_loop(const PllJobs& P, hipStream_t st) {
  bool vec;
  hipError_t e = pll_check(P, &vec);
  if (e != hipSuccess) return e;
  PllJobs L = P;
  if (pll_long(P)) {
    // long call: every pseudo-block solved (from warm-up guesses), then the chain with its repairs
    L.qform = 0;
    e = long_setup(L);
    if (e == hipSuccess) e = th32_check(L);
    if (e == hipSuccess) e = qtab_fill(L);
    if (e != hipSuccess) return e;
    const int R = L.njobs * L.nstreams;
    hipLaunchKernelGGL((pll_spec_kernel<512, true>), dim3((unsigned)(R * L.lg.nb)), dim3(512), 0, st, L);
    hipLaunchKernelGGL(pll_long_fix_kernel, dim3((unsigned)R), dim3(CHAIN_T), 0, st, L);
    return hipGetLastError();
  }
  if (th32_check(P) != hipSuccess) return hipErrorInvalidValue;    // (compact rows: long calls only)
  if (spec_only(P)) {
    // one launch: every recurrence solved in parallel, or sequentially in its own workgroup
    // when the solve cannot complete it (lpw = 0 tells the kernel so)
    L.lpw = 0;
    L.qform = 0;
    L.nco_fused = P.nco_rows ? 1 : 0;
    e = qtab_fill(L);
    if (e != hipSuccess) return e;
    const dim3 g((unsigned)(L.njobs * L.nstreams));
    if (L.n > SPEC_N256) hipLaunchKernelGGL((pll_spec_kernel<512, false>), g, dim3(512), 0, st, L);
    else hipLaunchKernelGGL((pll_spec_kernel<256, false>), g, dim3(256), 0, st, L);
    return hipGetLastError();
  }
  for (int q = 0; q < P.njobs; ++q)                  // (the sequential kernels read float rows only)
    if (P.j[q].in8 != nullptr) return hipErrorInvalidValue;
  L.lpw = pll_lpw(P);
  L.qform = vec && L.lpw == 1;
  const dim3 grid((unsigned)(L.njobs * ((L.nstreams + L.lpw - 1) / L.lpw)));
  if (vec && L.lpw == 1) hipLaunchKernelGGL(pll_chunk_kernel, grid, dim3(128), 0, st, L);
  else if (vec) hipLaunchKernelGGL(pll_lanes_kernel<true>, grid, dim3(64), 0, st, L);
  else hipLaunchKernelGGL(pll_lanes_kernel<false>, grid, dim3(64), 0, st, L);
  return hipGetLastError();
}

hipError_t sdr_launch_pll_nco(const PllJobs& P, hipStream_t st) {
  bool vec;
  hipError_t e = pll_check(P, &vec);
  if (e != hipSuccess) return e;
  PllJobs L = P;
  L.qform = !pll_long(P) && !spec_only(P) && vec && pll_lpw(P) == 1;
  if (pll_long(P)) {
    e = long_setup(L);
    if (e != hipSuccess) return e;
  }
  if (th32_check(L) != hipSuccess) return hipErrorInvalidValue;
  if (pll_long(P)) {
    if (!P.nco_rows) return hipSuccess;                // the consumer forms the NCO (sdr_nco.h)
    for (int q = 0; q < P.njobs; ++q)
      if (P.j[q].resp == nullptr) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nco_long_kernel, dim3((unsigned)(L.lg.nb * nco_tiles_per_block(L.lg.pb)), (unsigned)(P.njobs * P.nstreams)),
                       dim3(256), 0, st, L);
  } else if (P.n > 0 && !spec_only(P)) {              // (spec-only: the solve's launch wrote the rows)
    hipLaunchKernelGGL(nco_jobs_kernel, dim3((unsigned)((P.n + 255) / 256), (unsigned)(P.njobs * P.nstreams)),
                       dim3(256), 0, st, L);
  }
  return hipGetLastError();
}

hipError_t sdr_launch_pll_jobs(const PllJobs& P, hipStream_t st) {
  hipError_t e = sdr_launch_pll_prep(P, st);
  if (e == hipSuccess) e = sdr_launch_pll_loop(P, st);
  if (e == hipSuccess) e = sdr_launch_pll_nco(P, st);
  return e;
}
