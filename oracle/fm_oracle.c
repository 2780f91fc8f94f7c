/* ORACLE — test infrastructure only (never linked into the product).
 *
 * Plain-C float64 restatement of the reference Python model's front end and mono
 * path, used (a) by tests as a fast checker at sizes the numpy oracle is slow for and
 * (b) as bench.py's CPU baseline (cpu_baseline.kind = "port"), OpenMP over independent
 * streams, one stream per thread.  Pinned through tests/test_oracle.py against the
 * numpy oracle (oracle/fm_oracle.py) and the golden vectors of tests/golden/.
 *
 *   orc_fir_decim     lfilter(b, 1.0, x, zi)[::D] (scipy _signaltools.py:2153-2172),
 *                     as model/fmMonoBlock.py:86-95,101-105; computes only kept outputs.
 *   orc_demod         fmDemodArctan, model/fmSupportLib.py:15-44 (np.unwrap step).
 *   orc_fe_mono       one stream: RF LPF + [::10] (I and Q) -> demod -> audio LPF + [::5].
 *   orc_fe_mono_streams  the same over nstreams streams, OpenMP-parallel.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* y[m] = sum_k b[k] x[D m - k] (+ zi[D m] if D m < T-1), x[<0] = 0; x read with `step`.
 * If zi != NULL it is replaced by the lfilter final state (zf). */
void orc_fir_decim(const float* x, int64_t step, int64_t n, const double* b, int T, int D,
                   double* zi, double* y) {
  const int64_t M = (n + D - 1) / D;
  for (int64_t m = 0; m < M; ++m) {
    const int64_t c = (int64_t)D * m;
    const int kmax = (int)(c < T - 1 ? c : T - 1);
    double acc = 0.0;
#pragma omp simd reduction(+ : acc)
    for (int k = 0; k <= kmax; ++k) acc += b[k] * (double)x[(c - k) * step];
    if (zi && c < T - 1) acc += zi[c];
    y[m] = acc;
  }
  if (zi) {
    double* zf = (double*)malloc(sizeof(double) * (T > 1 ? T - 1 : 1));
    for (int k = 0; k < T - 1; ++k) {
      double acc = 0.0;
      for (int j = k + 1; j < T; ++j) {
        const int64_t idx = n + k - j;
        if (idx < 0) break;
        if (idx < n) acc += b[j] * (double)x[idx * step];
      }
      if (n + k < T - 1) acc += zi[n + k];
      zf[k] = acc;
    }
    memcpy(zi, zf, sizeof(double) * (T - 1));
    free(zf);
  }
}

/* Same on an f64 input stream (the demod -> audio stage). */
void orc_fir_decim_f64(const double* x, int64_t n, const double* b, int T, int D, double* zi,
                       double* y) {
  const int64_t M = (n + D - 1) / D;
  for (int64_t m = 0; m < M; ++m) {
    const int64_t c = (int64_t)D * m;
    const int kmax = (int)(c < T - 1 ? c : T - 1);
    double acc = 0.0;
#pragma omp simd reduction(+ : acc)
    for (int k = 0; k <= kmax; ++k) acc += b[k] * x[c - k];
    if (zi && c < T - 1) acc += zi[c];
    y[m] = acc;
  }
  if (zi) {
    double* zf = (double*)malloc(sizeof(double) * (T > 1 ? T - 1 : 1));
    for (int k = 0; k < T - 1; ++k) {
      double acc = 0.0;
      for (int j = k + 1; j < T; ++j) {
        const int64_t idx = n + k - j;
        if (idx < 0) break;
        if (idx < n) acc += b[j] * x[idx];
      }
      if (n + k < T - 1) acc += zi[n + k];
      zf[k] = acc;
    }
    memcpy(zi, zf, sizeof(double) * (T - 1));
    free(zf);
  }
}

/* fmDemodArctan with np.unwrap([prev, cur]) semantics; *prev is the accumulated phase. */
void orc_demod(const double* I, const double* Q, int64_t n, double* prev, double* out) {
  double p = prev ? *prev : 0.0;
  for (int64_t k = 0; k < n; ++k) {
    const double cur = atan2(Q[k], I[k]);
    const double dd = cur - p;
    double corr = 0.0;
    if (!(fabs(dd) < M_PI)) {
      double m = fmod(dd + M_PI, 2.0 * M_PI);
      if (m < 0) m += 2.0 * M_PI;
      double ddmod = m - M_PI;
      if (ddmod == -M_PI && dd > 0) ddmod = M_PI;
      corr = ddmod - dd;
    }
    const double cu = cur + corr;
    out[k] = cu - p;
    p = cu;
  }
  if (prev) *prev = p;
}

/* One stream, zero initial state: FE (rf taps T, decim 10) + audio (TA taps, decim 5).
 * demod_out (ceil(n/10)) may be NULL; audio_out: ceil(ceil(n/10)/5). */
void orc_fe_mono(const float* iq, int64_t n, const double* rf_b, int T, const double* au_b, int TA,
                 double* demod_out, double* audio_out) {
  const int64_t M = (n + 9) / 10;
  double* yi = (double*)malloc(sizeof(double) * (M + 1));
  double* yq = (double*)malloc(sizeof(double) * (M + 1));
  double* dm = demod_out ? demod_out : (double*)malloc(sizeof(double) * (M + 1));
  orc_fir_decim(iq, 2, n, rf_b, T, 10, NULL, yi);
  orc_fir_decim(iq + 1, 2, n, rf_b, T, 10, NULL, yq);
  double ph = 0.0;
  orc_demod(yi, yq, M, &ph, dm);
  orc_fir_decim_f64(dm, M, au_b, TA, 5, NULL, audio_out);
  if (!demod_out) free(dm);
  free(yi);
  free(yq);
}

/* nstreams independent streams `stride` complex samples apart, one per OpenMP thread. */
void orc_fe_mono_streams(const float* iq, int64_t n, int64_t stride, int nstreams, const double* rf_b,
                         int T, const double* au_b, int TA, double* audio_out, int64_t audio_stride,
                         int nthreads) {
#pragma omp parallel for num_threads(nthreads) schedule(static, 1)
  for (int s = 0; s < nstreams; ++s)
    orc_fe_mono(iq + 2 * (int64_t)s * stride, n, rf_b, T, au_b, TA, NULL, audio_out + (int64_t)s * audio_stride);
}

/* fmPll (model/fmPll.py:4-46), restated operation for operation as oracle/fm_oracle.py::fm_pll
 * (Python's float arithmetic and the same libm atan2 / cos / sin: no contraction, so the
 * results are bit-identical -- tests/test_oracle.py::test_c_oracle_pll).  state: the 6-list
 * [integrator, phaseEst, feedbackI, feedbackQ, ncoOut[0], trigOffset], updated in place.
 * nco / ncoq: n + 1 values (ncoq may be NULL); ncoq[0] as fm_pll defines it. */
__attribute__((optimize("fp-contract=off")))
void orc_pll(const double* x, int64_t n, double freq, double fs, double scale, double adj, double bw,
             double* state, double* nco, double* ncoq) {
  /* called through pointers: the compiler would otherwise merge cos(a) and sin(a) into one
   * sincos() call, whose results differ from the separate calls Python makes in the last bit */
  double (*volatile vcos)(double) = cos;
  double (*volatile vsin)(double) = sin;
  double (*volatile vatan2)(double, double) = atan2;
  const double Kp = bw * 2.666;
  const double Ki = bw * bw * 3.555;
  double integ = state[0], phase = state[1], fI = state[2], fQ = state[3];
  const double off = state[5];
  const double w = 2 * M_PI * (freq / fs);
  nco[0] = state[4];
  if (ncoq) ncoq[0] = off > 0 ? vsin((w * off + phase) * scale + adj) : 0.0;
  for (int64_t k = 0; k < n; ++k) {
    const double e = vatan2(x[k] * (-fQ), x[k] * (+fI));
    integ = integ + Ki * e;
    phase = phase + Kp * e + integ;
    const double arg = w * (off + (double)k + 1) + phase;
    fI = vcos(arg);
    fQ = vsin(arg);
    nco[k + 1] = vcos(arg * scale + adj);
    if (ncoq) ncoq[k + 1] = vsin(arg * scale + adj);
  }
  state[0] = integ;
  state[1] = phase;
  state[2] = fI;
  state[3] = fQ;
  state[4] = nco[n];
  state[5] = off + (double)n;
}
