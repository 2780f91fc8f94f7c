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
#include <stdlib.h>

#include "sdr_launch.h"

namespace {

// 2*pi split into three parts (Cody-Waite), so n*P1 and n*P2 are exact for |n| < 2^26.
constexpr double kP1 = 6.2831854820251465;       // float32(2 pi), 24 significant bits
constexpr double kP2 = -1.748455600074497e-07;    // double(2 pi - kP1)
constexpr double kP3 = -1.0687562935444062e-23;   // remainder
constexpr double kInv2Pi = 0.15915494309189535;
constexpr double kPi = 3.14159265358979323846;
constexpr double k2Pi = 6.28318530717958647692;

// r = a - 2*pi*n, n = rint(a / 2pi), |r| <= pi (up to one ulp at the boundary).
__device__ inline double reduce_2pi(double a) {
  const double n = rint(a * kInv2Pi);
  double r = fma(-n, kP1, a);
  r = fma(-n, kP2, r);
  r = fma(-n, kP3, r);
  return r;
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
    st[2] = cos(arg);
    st[3] = sin(arg);
    st[4] = cos(arg * cfg.scale + cfg.adj);
    st[5] = off + (double)n;
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
      st[2] = cos(arg);
      st[3] = sin(arg);
      st[4] = cos(arg * cfg.scale + cfg.adj);
      st[5] = off + (double)n;
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
constexpr int SPEC_W = 256;          // warm-up samples before each chunk
constexpr int SPEC_IT = 3;           // solve / check rounds before the sequential kernel takes over
constexpr int SPEC_NMAX = 16384 + 1; // samples per call (the constants of steps 1.. in LDS: 128 KiB)

// SPEC_T threads (chunks) per recurrence: 256 (one wave per SIMD) up to 10 240 samples, 512
// beyond (the warm-up is the same length either way; 512 halves the chunks, and a second
// wave per SIMD then pays: c5 blocks 56 -> ~50 us, c4 blocks slower)
template <int SPEC_T>
__global__ __launch_bounds__(SPEC_T) void pll_spec_kernel(PllJobs P) {
#pragma clang fp contract(off)
  __shared__ double cl[SPEC_NMAX - 1];         // c_k of steps 1 .. n-1 (plain form)
  __shared__ int8_t mrel[SPEC_NMAX - 1];       // m_k - floor(c_k) + jb, jb = floor(phaseEst_1 / 2pi)
  __shared__ d2v yb[SPEC_T];
  __shared__ double x1s[2];
  const int q = blockIdx.x / P.nstreams;
  const int s = blockIdx.x - q * P.nstreams;
  const int tid = threadIdx.x;
  const PllJob& J = P.j[q];
  const int64_t n = P.n;
  const float* in = J.in + (int64_t)s * J.in_stride;
  double* th = J.theta + (int64_t)s * J.th_stride;
  double* cr = J.cbuf + (int64_t)s * J.c_stride;
  const PllCfg cfg = J.cfg;
  double* st = J.state + (int64_t)s * 6;
  const double off = st[5];
  const double w = 2.0 * kPi * (cfg.freq / cfg.fs);
  const double kA = k2Pi * cfg.ki, kB = kPi * cfg.ki;
  const double kC = k2Pi * (cfg.kp + cfg.ki), kD = kPi * (cfg.kp + cfg.ki);
  // the prep kernel's constants are in the Q-form when the chunk kernel is the loop kernel
  auto cplain = [&](int64_t k) {
    double c = cr[k];
    if (P.qform) {
      const double i = (double)(k % PG);
      c = c - (kPi * cfg.ki) * kInv2Pi * (i * (i - 1.0) * 0.5);
    }
    return c;
  };
  auto thval = [&](double ph, int64_t k) {       // what the theta row holds for step k
    if (!P.qform) return ph;
    const double i = (double)(k % PG);
    return ph + kB * ((i + 1.0) * i * 0.5);
  };
  // sample 0: the literal general step (thread 0), as the loop kernels' general()
  if (tid == 0) {
    const double xv = (double)in[0];
    const double e = atan2(xv * (-st[3]), xv * st[2]);
    const double integ = st[0] + cfg.ki * e;
    const double phase = st[1] + cfg.kp * e + integ;
    x1s[0] = phase;
    x1s[1] = integ - kD;
  }
  __syncthreads();
  const double p1 = x1s[0], v1 = x1s[1];
  const int64_t N = n - 1;                       // steps 1 .. n-1
  // every step reads its constant several times: stage them (plain form) in LDS
  for (int64_t k = tid; k < N; k += SPEC_T) cl[k] = cplain(k + 1);
  __syncthreads();
  // the integer part relative to floor(c_k) is floor(-phaseEst/2pi + frac(c_k)): near -jb
  // within a block, so it fits a byte once jb is taken off (a drifting phase estimate moves jb)
  const double jb = floor(kInv2Pi * p1);
  auto rel_of = [&](double t, double c) { return floor(t) - floor(c) + jb; };
  const int L = (int)((N + SPEC_T - 1) / SPEC_T);
  const int TE = (int)((N + L - 1) / L);         // chunks in use; chunks 0 .. TE-2 are full
  const int64_t k0 = 1 + (int64_t)tid * L;
  const int64_t k1 = tid < TE ? min<int64_t>(k0 + L, n) : k0;
  // 1. guess
  bool bad = false;
  {
    // from the block's first state: a locked estimate moves little within a block (a 3 Hz
    // pilot offset: 1.2 rad over 15 360 samples), and 256 steps of the loop shrink that
    // ~30-fold.  (Extrapolating by integ does worse: integ swings with the loop's own
    // oscillation, and a 64-step mean of it mispredicts a block's drift by up to 4 rad.)
    const int64_t kw = max<int64_t>(1, k0 - SPEC_W);
    double p = p1, V = v1;
#pragma unroll 8
    for (int64_t k = kw; k < k0 && tid < TE; ++k) {
      const double t = fma(-kInv2Pi, p, cl[k - 1]);
      const double f = __builtin_amdgcn_fract(t);
      const double S = p + V;
      V = fma(kA, f, V - kB);
      p = fma(kC, f, S);
    }
    for (int64_t k = k0; k < k1; ++k) {
      const double c = cl[k - 1];
      const double t = fma(-kInv2Pi, p, c);
      const double r = rel_of(t, c);
      bad |= !(r >= -127.0 && r <= 127.0);       // also a NaN constant (a 0 / NaN input)
      mrel[k - 1] = (int8_t)(bad ? 0.0 : r);
      const double f = __builtin_amdgcn_fract(t);
      const double S = p + V;
      V = fma(kA, f, V - kB);
      p = fma(kC, f, S);
    }
  }
  if (__syncthreads_or(bad)) return;             // a 0 / NaN input (the general form's case)
  // A^L and its squarings (every thread the same operations)
  const double a00 = 1.0 - kC * kInv2Pi, a10 = -kA * kInv2Pi;
  double P00 = 1.0, P01 = 0.0, P10 = 0.0, P11 = 1.0;
  for (int i = 0; i < L; ++i) {                  // P = A P
    const double n00 = a00 * P00 + P10, n01 = a00 * P01 + P11;
    const double n10 = a10 * P00 + P10, n11 = a10 * P01 + P11;
    P00 = n00; P01 = n01; P10 = n10; P11 = n11;
  }
  for (int round = 0; round < SPEC_IT; ++round) {
    // 2. solve: the chunk's response from zero state
    double zp = 0.0, zv = 0.0;
#pragma unroll 4
    for (int64_t k = k0; k < k1; ++k) {
      const double c = cl[k - 1];
      const double d = c - (floor(c) + ((double)mrel[k - 1] - jb));
      const double np = a00 * zp + zv + kC * d;
      const double nv = a10 * zp + zv + (kA * d - kB);
      zp = np; zv = nv;
    }
    __syncthreads();                             // mrel reads done before the checks below
    // v_0 = x_1, v_j = z_{j-1}; y_j = sum_{i<=j} (A^L)^(j-i) v_i
    double vp = 0.0, vv = 0.0;
    if (tid + 1 < SPEC_T) yb[tid + 1] = d2v{zp, zv};
    if (tid == 0) yb[0] = d2v{p1, v1};
    __syncthreads();
    if (tid < TE) { vp = yb[tid].x; vv = yb[tid].y; }
    double Q00 = P00, Q01 = P01, Q10 = P10, Q11 = P11;
    for (int o = 1; o < SPEC_T; o <<= 1) {
      __syncthreads();
      yb[tid] = d2v{vp, vv};
      __syncthreads();
      if (tid >= o && tid < TE) {
        const d2v u = yb[tid - o];
        vp = vp + (Q00 * u.x + Q01 * u.y);
        vv = vv + (Q10 * u.x + Q11 * u.y);
      }
      const double n00 = Q00 * Q00 + Q01 * Q10, n01 = Q00 * Q01 + Q01 * Q11;
      const double n10 = Q10 * Q00 + Q11 * Q10, n11 = Q10 * Q01 + Q11 * Q11;
      Q00 = n00; Q01 = n01; Q10 = n10; Q11 = n11;
    }
    // 3. check: the true step from y_j
    bool miss = false;
    double p = vp, V = vv;
    for (int64_t k = k0; k < k1; ++k) {
      const double c = cl[k - 1];
      const double t = fma(-kInv2Pi, p, c);
      const double r = rel_of(t, c);
      miss |= r != (double)mrel[k - 1];          // (out of a byte's range: a miss, and so on)
      mrel[k - 1] = (int8_t)(r >= -127.0 && r <= 127.0 ? r : 0.0);
      const double f = __builtin_amdgcn_fract(t);
      const double S = p + V;
      V = fma(kA, f, V - kB);
      p = fma(kC, f, S);
      th[k] = thval(p, k);
    }
    const int nmiss = __syncthreads_count(miss);
    if (P.spec_dbg && tid == 0) printf("pll_spec q%d s%d n%ld T%d L%d TE%d round %d: %d chunks missed\n", q, s, (long)n, SPEC_T, L, TE, round, nmiss);
    if (nmiss == 0) {
      // done: the caller-visible results exactly as the loop kernels leave them
      if (tid == 0) {
        th[0] = thval(p1, 0);
        J.nco_i[(int64_t)s * J.out_stride] = (float)st[4];
        if (J.nco_q)
          J.nco_q[(int64_t)s * J.out_stride] =
              (float)((off > 0.0) ? sin((w * off + st[1]) * cfg.scale + cfg.adj) : 0.0);
      }
      __syncthreads();                           // st[1], st[4] read before the last chunk writes st
      if (tid == TE - 1) {
        const double arg = w * ((off + (double)(n - 1)) + 1.0) + p;
        th[n] = off;
        st[0] = V + kD;
        st[1] = p;
        st[2] = cos(arg);
        st[3] = sin(arg);
        st[4] = cos(arg * cfg.scale + cfg.adj);
        st[5] = off + (double)n;
      }
      if (tid == 0) cr[0] = __builtin_inf();      // the loop kernel skips this recurrence
      return;
    }
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
    const double cc = (x > 0.f ? 0.0 : kPi) - w * (off + (double)k);   // the previous step's w (off + k)
    // a 0 / NaN input gets a NaN constant: a fast group over it ends in a NaN phase, which
    // pll_chunk_kernel takes as its signal to redo the group in the general form
    double cv = fma(cc, kInv2Pi, 0.5);
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
#pragma clang fp contract(off)
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= P.n) return;
  const int g = blockIdx.y;                 // uniform: (job, stream)
  const int q = g / P.nstreams;
  const int s = g - q * P.nstreams;
  const PllJob& J = P.j[q];
  const double* ph = J.theta + (int64_t)s * J.th_stride;
  const double off = ph[P.n];
  const double w = 2.0 * kPi * (J.cfg.freq / J.cfg.fs);
  double p = ph[k];
  if (P.qform) {                                        // Q_{i+1} -> phase_{i+1}
    const double i = (double)(k % PG);
    p = p - (kPi * J.cfg.ki) * ((i + 1.0) * i * 0.5);
  }
  const double th = w * ((off + (double)k) + 1.0) + p;
  const double a = th * J.cfg.scale + J.cfg.adj;
  double sv, cv;
  sincos(a, &sv, &cv);
  J.nco_i[(int64_t)s * J.out_stride + k + 1] = (float)cv;
  if (J.nco_q) J.nco_q[(int64_t)s * J.out_stride + k + 1] = (float)sv;
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
// the parallel solve runs ahead of the loop kernel unless SDR_PLL_SPEC=0 (A/B runs)
bool pll_spec_enabled() {
  static const bool on = [] { const char* e = getenv("SDR_PLL_SPEC"); return !(e && e[0] == '0'); }();
  return on;
}
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

hipError_t sdr_launch_pll_prep(const PllJobs& P, hipStream_t st) {
  bool vec;
  const hipError_t e = pll_check(P, &vec);
  if (e != hipSuccess) return e;
  PllJobs L = P;
  L.qform = vec && pll_lpw(P) == 1;
  if (P.n > 0)
    hipLaunchKernelGGL(pll_prep_kernel, dim3((unsigned)((P.n + 255) / 256), (unsigned)(P.njobs * P.nstreams)),
                       dim3(256), 0, st, L);
  return hipGetLastError();
}

hipError_t sdr_launch_pll_loop(const PllJobs& P, hipStream_t st) {
  bool vec;
  const hipError_t e = pll_check(P, &vec);
  if (e != hipSuccess) return e;
  PllJobs L = P;
  L.lpw = pll_lpw(P);
  L.qform = vec && L.lpw == 1;
  const dim3 grid((unsigned)(L.njobs * ((L.nstreams + L.lpw - 1) / L.lpw)));
  if (pll_spec_enabled() && L.n >= 2 && L.n <= SPEC_NMAX) {
    PllJobs S = L;
    S.spec_dbg = getenv("SDR_PLL_SPEC_DEBUG") != nullptr;   // per-round prints (A/B runs)
    const dim3 g((unsigned)(L.njobs * L.nstreams));
    if (L.n > 10240) hipLaunchKernelGGL(pll_spec_kernel<512>, g, dim3(512), 0, st, S);
    else hipLaunchKernelGGL(pll_spec_kernel<256>, g, dim3(256), 0, st, S);
  }
  if (vec && L.lpw == 1) hipLaunchKernelGGL(pll_chunk_kernel, grid, dim3(128), 0, st, L);
  else if (vec) hipLaunchKernelGGL(pll_lanes_kernel<true>, grid, dim3(64), 0, st, L);
  else hipLaunchKernelGGL(pll_lanes_kernel<false>, grid, dim3(64), 0, st, L);
  return hipGetLastError();
}

hipError_t sdr_launch_pll_nco(const PllJobs& P, hipStream_t st) {
  bool vec;
  const hipError_t e = pll_check(P, &vec);
  if (e != hipSuccess) return e;
  PllJobs L = P;
  L.qform = vec && pll_lpw(P) == 1;
  if (P.n > 0)
    hipLaunchKernelGGL(nco_jobs_kernel, dim3((unsigned)((P.n + 255) / 256), (unsigned)(P.njobs * P.nstreams)),
                       dim3(256), 0, st, L);
  return hipGetLastError();
}

hipError_t sdr_launch_pll_jobs(const PllJobs& P, hipStream_t st) {
  hipError_t e = sdr_launch_pll_prep(P, st);
  if (e == hipSuccess) e = sdr_launch_pll_loop(P, st);
  if (e == hipSuccess) e = sdr_launch_pll_nco(P, st);
  return e;
}
