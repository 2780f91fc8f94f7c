// Multi-stream block receiver (sdr_rx_*): the per-block loops of model/fmMonoBlock.py:80-173
// (mono + stereo) and model/fmRDSblock.py:127-204 (RDS up to the RRC output) for S
// independent streams at once, every state and intermediate resident in HBM.  This is
// SURVEY §8a C5 (8 streams, mono + stereo + RDS, B = 153 600, src/fm_radio.cpp:783-792 runs
// the same stages as four threads per stream) and the per-block drop-in path of C3/C4.
//
// One block of all S streams is a fixed chain of launches on the context stream:
//   FE        RF FIR + decimate + atan2 demod (fe.hip; zf and demod state included)
//   stage A   every filter that reads demod: mono LPF (decim 5), pilot BPF, stereo BPF,
//             RDS extract BPF -- one launch, one job table (rx_stage_kernel)
//   stage B   RDS square + BPF (model/fmRDSblock.py:161-164)
//   PLL       stereo pilot PLL and RDS carrier PLL of every stream: one lane per
//             recurrence (pll.hip), then the NCO outputs
//   stage C   stereo mixer + LPF + decimate with the L/R combiner fused into its store;
//             RDS I and Q mixers + 3 kHz LPF
//   stage D   RDS rational resamplers (x19 zero-stuff, anti-image LPF, [::80] x19), I and Q
//   stage E   RDS RRC filters, I and Q
// Every stage launch also carries its filters' lfilter final states: extra workgroups after
// the output tiles compute zf (f64) from the block's last inputs.  zi and
// zf live in two state banks that swap every block, so no zf write races a zi read.
// Launches per block: 1 FE (+ its zf / phase kernels) + up to 5 stages + 2 PLL = 10 at
// full C5, whatever S is.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <type_traits>
#include <vector>

#include "sdr_ctx.h"
#include "sdr_nco.h"

using namespace sdrint;

namespace {

constexpr int RX_MAXJ = 6;          // jobs per stage launch
constexpr int RX_NT = 256;          // threads per workgroup
constexpr int RX_R = 4;             // outputs per thread of the generic tiles (any T, resampler)
constexpr int RX_TO = RX_NT * RX_R;  // outputs per generic tile
constexpr int RX_LDS = 6144;        // floats of LDS per workgroup (largest: 151 taps, decim 5: 5 796)

enum { JK_FIR = 0, JK_RESAMPLE = 1 };
// PRE_NCO: the mixer of PRE_MIX whose second operand, the PLL's NCO, is formed from the PLL's
// phase rows where the input is staged (sdr_nco.h) instead of read from an NCO row
enum { PRE_NONE = SDR_PRE_NONE, PRE_SQUARE = SDR_PRE_SQUARE, PRE_MIX = SDR_PRE_MIX, PRE_NCO = 3 };

// One filter of a stage, applied to `nstreams` streams.
struct StageJob {
  const float* x;        // input rows, x_stride apart
  const float* c;        // PRE_MIX second operand (same indexing as x)
  const float* taps;     // f32 taps (device)
  const float* rtaps;    // the same reversed, zero at [-1] and [T] (TapSet::dev_rev: fir_tile's pairs)
  const double* taps64;  // f64 taps (device, for zf)
  const double* zi;      // lfilter state in (T-1 per stream, zi_stride apart), nullable
  double* zf;            // lfilter state out (same layout), nullable
  float* y;              // outputs, y_stride apart
  const float* mono;     // combiner: mono audio rows (y_stride apart), or null
  float* left;
  float* right;
  float* yh;             // host mirrors (pinned, rows yh_stride apart) of y / left / right, nullable:
  float* lh;             //   sdr_rx_run's outputs are stored straight into pinned host memory
  float* rh;             //   by the producing tile instead of coming back by a copy
  int64_t n, x_stride, zi_stride, y_stride, yh_stride;
  int64_t b0;            // first workgroup of this job's tiles
  float gain;
  int pre, D, U, kind, T, tiles;
  int small;             // D = 1 FIR: 4 outputs per lane (a launch with few tiles: more workgroups)
  int sym;               // the f32 taps are symmetric (linear phase: every firwin design)
  int fold;              // > 1: the leader of `fold` consecutive symmetric jobs on the same input,
                         //   computed together by fold_tile (the others get no tile workgroups)
  int nco_sin;           // PRE_NCO: the quadrature NCO (sin) instead of cos
  int mma;               // the tiles run on the matrix cores (rx_mma_kernel); this launch keeps its zf
  int wgs;               // rx_mma_kernel: the job's workgroups (each runs every wgs-th tile)
  NcoSrc nco;            // PRE_NCO: where the NCO comes from
  int8_t* y8;            // nullable: the outputs' sign codes too (sdr_nco.h pll_code: a PLL's input),
  int64_t y8_stride;     //   y8_stride bytes apart; y may then be null (matrix-core jobs only)
};

// The front end's carried state, finished by the first stage launch after the FE kernel:
// the I/Q lfilter final states (f64, from the block's last T-1 IQ samples) and the demod
// phase prev = phi_last + 2 pi W (W = the block's wrap count, which is reset for the next
// block).  One workgroup per stream.
struct FeState {
  const void* iq;
  int64_t n, stride;          // complex samples per block / between streams
  const double* b;            // f64 taps
  const double* zi_i;
  const double* zi_q;
  double* zf_i;
  double* zf_q;
  int64_t zs;                 // state stride
  const float* last_phi;
  int* wraps;
  double* phase;
  int T, u8, on;
};

struct StageJobs {
  StageJob j[RX_MAXJ];
  int njobs, nstreams;
  int64_t tile_blocks;        // tile workgroups (after the final-state ones, rx_stage_kernel)
  int zfj[RX_MAXJ], nzf;      // nzf * nstreams workgroups compute final states (grid front)
  FeState fe;                 // then (fe.on ? nstreams : 0) workgroups finish the FE state
};

__device__ __forceinline__ float pre_op(int pre, float x, float c, float g) {
  return pre == PRE_SQUARE ? x * x : (pre == PRE_MIX || pre == PRE_NCO) ? (x * c) * g : x;
}

// ncoOut[k] and ncoOutQ[k] of stream s as the mixers take them (f32, sdr_nco.h nco_f32x2):
// [0] is the carried value the PLL kernel stored, [k >= 1] is formed from phaseEst_{k-1}.
// (Single samples: the tiles' cold paths and the final-state workgroups; the tiles' staging
// takes two at a time with the pseudo-block records read once per tile.)
__device__ __forceinline__ void nco_at(const NcoSrc& N, int s, int64_t k, float* c, float* sn) {
  if (k == 0) {
    *c = N.nco_i[(int64_t)s * N.out_stride];
    *sn = N.nco_q ? N.nco_q[(int64_t)s * N.out_stride] : 0.f;
    return;
  }
  const NcoTile T = nco_tile(N, s, k - 1);
  const double p = nco_tile_p(N, T, k - 1, N.th32 ? th32_stored(T.th, N.n, k - 1) : T.th[k - 1]);   // (compact rows: the
                                                                                                     // stereo mixer's final states)
  ncof2 c2, s2;
  nco_f32x2(N, T.off, k, p, p, &c2, &s2);
  *c = c2.x;
  *sn = s2.x;
}
__device__ __forceinline__ float nco_one(const StageJob& J, int s, int64_t k) {
  float c, sn;
  nco_at(J.nco, s, k, &c, &sn);
  return J.nco_sin ? sn : c;
}

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f2a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef const __attribute__((address_space(4))) float* ctaps_t;   // uniform, read-only: scalar loads
typedef const __attribute__((address_space(4))) f2a4* ctaps2_t;

// acc.xy += h.xy * x.xy in one v_pk_fma_f32, the tap pair as a 64-bit SGPR operand (a scalar
// load of two consecutive reversed taps): the compiler neither moves taps into vector
// registers nor assembles packed operands with a v_mov per FMA
__device__ __forceinline__ void pk_fma_s(f2& acc, f2 h, f2 x) {
  asm("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc) : "s"(h), "v"(x));
}

// acc.xy += h.{lo or hi} * x.xy: the tap broadcast from a 64-bit SGPR pair by op_sel
template <bool HI>
__device__ __forceinline__ void pk_fma_sb(f2& acc, f2 h, f2 x) {
  if (HI) asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "s"(h), "v"(x));
  else asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]" : "+v"(acc) : "s"(h), "v"(x));
}

// The lfilter FIR tile for compile-time (T, D): lane t owns R consecutive outputs and slides
// once over its D(R-1)+T-sample window in LDS two samples at a time (ds_read_b64), each
// output's two partial sums -- even and odd window samples -- in one packed register:
//   acc_r.xy += (g[j], g[j+1]) * (x_i, x_{i+1}),  j = i - D r,  g = the taps reversed
// (g[j] = h[T-1-j], zero at j = -1 and j = T: TapSet::dev_rev), i.e. acc_r.x += h[D r+T-1-i] x_i
// and acc_r.y += h[D r+T-2-i] x_{i+1}; y_r = acc_r.x + acc_r.y.  16 outputs per lane at D = 1
// (16 packed FMAs per ds_read_b64: VALU-bound), 4 at D = 5.  The tile image has two pad
// floats after every lane's D*R samples (even lane stride SR = 2 mod 4 dwords: 8-B aligned,
// conflict-free ds_read_b64), and starts DELTA samples early so that its global loads are
// 16-B aligned.
template <int T, int D, int R_ = (D == 1 ? 16 : 4)>
struct FirShape {
  static constexpr int G = 4, NT = RX_NT, R = R_, TO = NT * R, DR = D * R;
  static constexpr int SR = DR + 2;                          // lane stride in LDS (floats)
  static constexpr int DELTA = (G - ((T - 1) % G)) % G;
  static constexpr int L = D * (TO - 1) + T + DELTA;         // image samples
  static constexpr int LG = (L + G - 1) / G * G;
  static constexpr int NI = D * (R - 1) + T;                 // per-lane window
  static constexpr int NSLOT = LG + 2 * (LG / DR) + 2;
  static_assert((D * TO) % G == 0, "tile start must stay G-aligned");
  static_assert(NSLOT <= RX_LDS, "tile image fits the stage LDS");
  static_assert(SR % 4 == 2 && DELTA % 2 == 0 && NI % 2 == 0, "8-B aligned, conflict-free sample pairs");
  __device__ static constexpr int slot(int u) { return u < DELTA ? u : u + 2 * ((u - DELTA) / DR); }
};

template <int T, int D, int R_ = (D == 1 ? 16 : 4), bool NCO = false>
__device__ __forceinline__ void fir_tile(const StageJob& J, int s, int64_t tile, float* lds) {
  using S = FirShape<T, D, R_>;
  constexpr int R = S::R, DR = S::DR, DELTA = S::DELTA;
  const int t = threadIdx.x;
  const int64_t m0 = tile * S::TO;
  const int64_t M = (J.n + D - 1) / D;
  const int64_t n_lo = D * m0 - (T - 1) - DELTA;           // image sample 0
  const int64_t mf = m0 + (int64_t)t * R;
  const float* xb = J.x + (int64_t)s * J.x_stride;
  const float* cb = J.c ? J.c + (int64_t)s * J.x_stride : nullptr;
  const int pre = J.pre;
  const float g = J.gain;
  // the zi terms and the combiner inputs are loaded up front, not after the FIR: at the
  // reference's block sizes a stage is a handful of workgroups whose time is the number of
  // dependent memory round trips
  float zr[R], mr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t nn = D * (mf + r);
    zr[r] = (J.zi != nullptr && nn < T - 1) ? (float)J.zi[(int64_t)s * J.zi_stride + nn] : 0.f;
    mr[r] = (J.mono != nullptr && mf + r < M) ? J.mono[(int64_t)s * J.y_stride + mf + r] : 0.f;
  }
  if (n_lo >= 0 && n_lo + S::LG <= J.n) {            // interior: 16-B loads (rows are aligned)
    NcoTile nt{};
    if (NCO && pre == PRE_NCO) nt = nco_tile(J.nco, s, n_lo - 1);   // the pseudo-block records, once
    // every load of the thread's chunks is issued before the first is used (one memory
    // round trip per tile, not one per chunk)
    constexpr int NCH = S::LG / S::G, NQ = (NCH + S::NT - 1) / S::NT;
    float4 v[NQ], cv[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int q = t + j * S::NT;
      if (q < NCH) {
        v[j] = reinterpret_cast<const float4*>(xb + n_lo)[q];
        cv[j] = pre == PRE_MIX ? reinterpret_cast<const float4*>(cb + n_lo)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int q = t + j * S::NT;
      if (q < NCH) {
        const int u = q * S::G;
        if (NCO && pre == PRE_NCO) {                 // the NCO of these 4 inputs, from the PLL phases
          const int64_t nn = n_lo + u;
          if (nn >= 2) {                             // (nn is a multiple of 4: 16-B phase pairs)
            float c4[4], s4[4];
            nco_f32x4(J.nco, nt, nn, c4, s4);
            cv[j] = J.nco_sin ? make_float4(s4[0], s4[1], s4[2], s4[3]) : make_float4(c4[0], c4[1], c4[2], c4[3]);
          } else {
            cv[j] = make_float4(nco_one(J, s, nn), nco_one(J, s, nn + 1), nco_one(J, s, nn + 2), nco_one(J, s, nn + 3));
          }
        }
        lds[S::slot(u + 0)] = pre_op(pre, v[j].x, cv[j].x, g);
        lds[S::slot(u + 1)] = pre_op(pre, v[j].y, cv[j].y, g);
        lds[S::slot(u + 2)] = pre_op(pre, v[j].z, cv[j].z, g);
        lds[S::slot(u + 3)] = pre_op(pre, v[j].w, cv[j].w, g);
      }
    }
  } else {
    for (int u = t; u < S::LG; u += S::NT) {
      const int64_t nn = n_lo + u;
      float x = 0.f;
      if (nn >= 0 && nn < J.n)
        x = pre_op(pre, xb[nn], pre == PRE_MIX ? cb[nn] : (NCO && pre == PRE_NCO) ? nco_one(J, s, nn) : 0.f, g);
      lds[S::slot(u)] = x;
    }
  }
  __syncthreads();
  const ctaps_t gr = (ctaps_t)J.rtaps;
  const float* win = lds + DELTA + S::SR * t;
  f2 pacc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) pacc[r] = f2{0.f, 0.f};
  static_for<0, S::NI / 2>([&](auto I) {
    constexpr int i = 2 * I;
    const f2 x = *reinterpret_cast<const f2*>(win + i + 2 * (i / DR));
    static_for<0, R>([&](auto RR) {
      constexpr int r = RR;
      constexpr int j = i - D * r;
      if constexpr (j >= -1 && j <= T - 1) {
        const f2a4 hp = *(ctaps2_t)(gr + j);         // (g[j], g[j+1]): float-indexed pair
        pk_fma_s(pacc[r], f2{hp.x, hp.y}, x);
      }
    });
  });
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = (pacc[r].x + pacc[r].y) + zr[r];
  float* yb = J.y + (int64_t)s * J.y_stride;
  if (mf + R <= M) {
#pragma unroll
    for (int r = 0; r < R; r += 4)
      *reinterpret_cast<float4*>(yb + mf + r) = make_float4(acc[r], acc[r + 1], acc[r + 2], acc[r + 3]);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (mf + r < M) yb[mf + r] = acc[r];
  }
  if (J.yh != nullptr) {                             // host rows are packed: scalar stores
    float* hb = J.yh + (int64_t)s * J.yh_stride;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (mf + r < M) hb[mf + r] = acc[r];
  }
  if (J.mono != nullptr) {                           // stereo combiner (fmMonoBlock.py:166-170)
    float* lb = J.left + (int64_t)s * J.y_stride;
    float* rb = J.right + (int64_t)s * J.y_stride;
    float* lhb = J.lh ? J.lh + (int64_t)s * J.yh_stride : nullptr;
    float* rhb = J.rh ? J.rh + (int64_t)s * J.yh_stride : nullptr;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (mf + r < M) {
        const float lv = (mr[r] + acc[r]) * 0.5f, rv = (mr[r] - acc[r]) * 0.5f;
        lb[mf + r] = lv;
        rb[mf + r] = rv;
        if (lhb) lhb[mf + r] = lv;
        if (rhb) rhb[mf + r] = rv;
      }
    }
  }
}

// ---- D = 1 FIR tiles on a pair image (stages A, B, E) ---------------------------------------
// A tile's TO = 2 H outputs are two halves, [m0, m0 + H) and [m0 + H, m0 + 2 H): lane t owns
// outputs m0 + R2 t + o and m0 + H + R2 t + o (o < R2) as the two halves of ONE packed register
// acc[o].  The LDS image is of sample PAIRS, P[v] = (x[a + v], x[a + H + v]) with a = m0 - (T-1)
// - DELTA, so at every tap k each packed register's operand is one aligned pair:
//   acc[o] += h[k] * P[R2 t + DELTA + o - k + T - 1]             (one v_pk_fma_f32, h broadcast)
// and from tap k to k + 1 the operand of o is the one o - 1 had: a lane's R2 operands live in
// registers and slide, one new pair per tap (ds_read_b64, conflict-free: the lane stride is
// R2 + 1 pairs, a pad pair after every R2) for R2 packed FMAs.  The taps come from LDS too
// (broadcast ds_read_b64 of two taps, one tap pair ahead) and the new pairs two taps ahead:
// LDS reads retire in order, so no wait in the loop drains the pipe for a scalar load (r05d:
// an s_load per tap step with an lgkmcnt(0) after it, 34 % of stage A's wave time parked, and
// ds_read2_b32 odd pairs with 2-way bank conflicts -- both gone here).
// FOLD: F symmetric filters on the same input at once (stage A: the pilot, stereo and RDS
// extract band-passes of the demod, model/fmMonoBlock.py:117,151, model/fmRDSblock.py:156) on
// the folded sums of linear-phase taps (h[k] = h[T-1-k], every firwin design):
//   y_f[n] = sum_{k<C} h_f[k] (x[n-k] + x[n-T+1+k]) + h_f[C] x[n-C],   C = (T-1)/2
// -- the right operands P[... + o + k] slide the other way; one v_pk_add_f32 per output pair
// and tap, shared by the F filters (F = 3: 75 adds + 228 multiply-adds per output, not 453).
template <int T, int R2>
struct PairShape {
  static constexpr int G = 4, NT = RX_NT, H = NT * R2, TO = 2 * H;
  static constexpr int DELTA = (G - ((T - 1) % G)) % G;             // x[a] is 16-B aligned
  static constexpr int LV = (H + T - 1 + DELTA + G - 1) / G * G;    // pairs staged
  __device__ static constexpr int slot(int v) { return v < DELTA ? v : v + (v - DELTA) / R2; }
  static constexpr int NSLOT = LV + (LV - DELTA) / R2 + 1;
  static constexpr int TAPS = (2 * NSLOT + 3) / 4 * 4;              // float offset of the tap table
  static_assert(DELTA % 2 == 0, "pad pairs split a 4-pair chunk only in halves");
};

// acc.xy += h.{lo or hi} * x.xy, the tap broadcast by op_sel from a VGPR pair
template <bool HI>
__device__ __forceinline__ void pk_fma_vb(f2& acc, f2 h, f2 x) {
  if (HI) asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(h), "v"(x));
  else asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]" : "+v"(acc) : "v"(h), "v"(x));
}

template <int T, int R2, int F, bool FOLD>
__device__ __forceinline__ void pair_tile(const StageJob* Jf, int s, int64_t tile, float* lds) {
  using S = PairShape<T, R2>;
  constexpr int H = S::H, DELTA = S::DELTA, C = (T - 1) / 2;
  constexpr int NK = FOLD ? C + 1 : T;                 // tap steps
  constexpr int TP = (NK + 1) / 2 * 2;                 // tap table row (even: 8-B pairs)
  static_assert(S::TAPS + F * TP <= RX_LDS, "pair image + taps fit the stage LDS");
  static_assert(FOLD || F == 1, "the unfolded tile runs one filter");
  static_assert(H >= T - 1, "zi terms only in the low half");
  const StageJob& J = Jf[0];
  const int t = threadIdx.x;
  const int64_t m0 = tile * S::TO;
  const int64_t M = J.n;
  const int64_t a = m0 - (T - 1) - DELTA;              // sample of P[0].x
  const float* xb = J.x + (int64_t)s * J.x_stride;
  const float* cb = J.c ? J.c + (int64_t)s * J.x_stride : nullptr;
  const int pre = J.pre;
  const float g = J.gain;
  f2* P = reinterpret_cast<f2*>(lds);
  if (a >= 0 && a + H + S::LV <= J.n) {                // interior: 16-B loads of both halves
    constexpr int NCH = S::LV / S::G, NQ = (NCH + S::NT - 1) / S::NT;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 lo[NQ], hi[NQ], clo[NQ], chi[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int q = t + j * S::NT;
      lo[j] = hi[j] = clo[j] = chi[j] = z4;
      if (q < NCH) {
        lo[j] = reinterpret_cast<const float4*>(xb + a)[q];
        hi[j] = reinterpret_cast<const float4*>(xb + a + H)[q];
        if (pre == PRE_MIX) {
          clo[j] = reinterpret_cast<const float4*>(cb + a)[q];
          chi[j] = reinterpret_cast<const float4*>(cb + a + H)[q];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int q = t + j * S::NT;
      if (q < NCH) {
        const int v = q * S::G;
        P[S::slot(v + 0)] = f2{pre_op(pre, lo[j].x, clo[j].x, g), pre_op(pre, hi[j].x, chi[j].x, g)};
        P[S::slot(v + 1)] = f2{pre_op(pre, lo[j].y, clo[j].y, g), pre_op(pre, hi[j].y, chi[j].y, g)};
        P[S::slot(v + 2)] = f2{pre_op(pre, lo[j].z, clo[j].z, g), pre_op(pre, hi[j].z, chi[j].z, g)};
        P[S::slot(v + 3)] = f2{pre_op(pre, lo[j].w, clo[j].w, g), pre_op(pre, hi[j].w, chi[j].w, g)};
      }
    }
  } else {
    for (int v = t; v < S::LV; v += S::NT) {
      const int64_t n0 = a + v, n1 = a + H + v;
      f2 p{0.f, 0.f};
      if (n0 >= 0 && n0 < J.n) p.x = pre_op(pre, xb[n0], pre == PRE_MIX ? cb[n0] : 0.f, g);
      if (n1 >= 0 && n1 < J.n) p.y = pre_op(pre, xb[n1], pre == PRE_MIX ? cb[n1] : 0.f, g);
      P[S::slot(v)] = p;
    }
  }
  float* tl = lds + S::TAPS;                           // filter f's forward taps at tl + f TP
  for (int i = t; i < F * TP; i += S::NT) {
    const int f = i / TP, k = i - f * TP;
    tl[i] = k < NK ? Jf[f].taps[k] : 0.f;
  }
  __syncthreads();
  const f2* win = P + DELTA + (R2 + 1) * t;
  auto ld = [&](int i) -> f2 { return win[i + i / R2]; };      // window pair i (compile-time i)
  const f2* tq = reinterpret_cast<const f2*>(tl);
  f2 acc[F][R2];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (int o = 0; o < R2; ++o) acc[f][o] = f2{0.f, 0.f};
  f2 lw[R2], rw[R2];                                   // operands of tap k: lw[o] = pair o - k + T - 1, rw[o] = pair o + k
  static_for<0, R2>([&](auto O) {
    constexpr int o = O;
    lw[o] = ld(o + T - 1);
    if constexpr (FOLD) rw[o] = ld(o);
  });
  constexpr int PD = 2;                                // new pairs read PD taps ahead
  f2 ln[PD], rn[PD], tc[F], tn[F];
#pragma unroll
  for (int f = 0; f < F; ++f) tc[f] = tq[f * (TP / 2)];
  static_for<1, PD>([&](auto JJ) {
    constexpr int j = JJ;
    if constexpr (j < NK) ln[j % PD] = ld(T - 1 - j);
    if constexpr (FOLD && j < C) rn[j % PD] = ld(R2 - 1 + j);
  });
  static_for<0, NK>([&](auto KK) {
    constexpr int k = KK;
    if constexpr (k + PD < NK) ln[k % PD] = ld(T - 1 - (k + PD));
    if constexpr (FOLD && k + PD < C) rn[k % PD] = ld(R2 - 1 + k + PD);
    if constexpr (k % 2 == 0 && k + 2 < NK) {
#pragma unroll
      for (int f = 0; f < F; ++f) tn[f] = tq[f * (TP / 2) + k / 2 + 1];
    }
    static_for<0, R2>([&](auto O) {
      constexpr int o = O;
      if constexpr (FOLD) {
        f2 sum = lw[o];
        if constexpr (k < C) sum = sum + rw[o];        // v_pk_add_f32
#pragma unroll
        for (int f = 0; f < F; ++f) pk_fma_vb<k % 2 == 1>(acc[f][o], tc[f], sum);
      } else {
        pk_fma_vb<k % 2 == 1>(acc[0][o], tc[0], lw[o]);
      }
    });
    if constexpr (k + 1 < NK) {
#pragma unroll
      for (int o = R2 - 1; o > 0; --o) lw[o] = lw[o - 1];
      lw[0] = ln[(k + 1) % PD];
      if constexpr (FOLD && k + 1 < C) {
#pragma unroll
        for (int o = 0; o < R2 - 1; ++o) rw[o] = rw[o + 1];
        rw[R2 - 1] = rn[(k + 1) % PD];
      }
      if constexpr (k % 2 == 1) {
#pragma unroll
        for (int f = 0; f < F; ++f) tc[f] = tn[f];
      }
    }
    // one tap step's reads stay with its arithmetic (hoisted, they outgrow the registers)
    __builtin_amdgcn_sched_barrier(0);
  });
  const int64_t nlo = m0 + (int64_t)R2 * t, nhi = nlo + H;
#pragma unroll
  for (int f = 0; f < F; ++f) {
    const StageJob& Jj = Jf[f];
    float ol[R2], oh[R2];
#pragma unroll
    for (int o = 0; o < R2; ++o) {
      const int64_t nn = nlo + o;                      // lfilter zi: the block's first T - 1 outputs
      const float z = (Jj.zi != nullptr && nn < T - 1) ? (float)Jj.zi[(int64_t)s * Jj.zi_stride + nn] : 0.f;
      ol[o] = acc[f][o].x + z;
      oh[o] = acc[f][o].y;
    }
    float* yb = Jj.y + (int64_t)s * Jj.y_stride;
    auto put = [&](float* row, int64_t n0, const float* v) {
      if (n0 + R2 <= M) {
        if constexpr (R2 % 4 == 0) {
#pragma unroll
          for (int o = 0; o < R2; o += 4) *reinterpret_cast<float4*>(row + n0 + o) = make_float4(v[o], v[o + 1], v[o + 2], v[o + 3]);
        } else {
#pragma unroll
          for (int o = 0; o < R2; o += 2) *reinterpret_cast<float2*>(row + n0 + o) = make_float2(v[o], v[o + 1]);
        }
      } else {
#pragma unroll
        for (int o = 0; o < R2; ++o)
          if (n0 + o < M) row[n0 + o] = v[o];
      }
    };
    put(yb, nlo, ol);
    put(yb, nhi, oh);
    if (Jj.yh != nullptr) {                            // host rows are packed: scalar stores
      float* hb = Jj.yh + (int64_t)s * Jj.yh_stride;
#pragma unroll
      for (int o = 0; o < R2; ++o) {
        if (nlo + o < M) hb[nlo + o] = ol[o];
        if (nhi + o < M) hb[nhi + o] = oh[o];
      }
    }
  }
}

// ---- D = 1 FIRs on the matrix cores (stages A, B, E at span sizes) ------------------------
// y[n] = sum_k h[k] x[n-k] for 256 consecutive outputs n = n0 + 16 c + b (c, b < 16) is the
// product Y = A X of the 16 x 32 KS Toeplitz tap matrix A[b][j] = h[b + KOFF - j] (zero
// outside 0 <= b + KOFF - j < T) and the Hankel window matrix X[j][c] = x[n0 + 16 c + j - KOFF]:
// KS v_mfma_f32_16x16x32_f16 steps, lane l holding A[l & 15][8 (l >> 4) + 0..7] (the taps: in
// registers for the whole launch), X[32 s + 8 (l >> 4) + 0..7][l & 15] (8 consecutive samples:
// one ds_read_b128 of the staged window, conflict-free) and outputs n0 + 16 (l & 15) + 4 (l >> 4)
// + 0..3 (one float4 store).  f32 accuracy from f16 operands: every x and h is split as
// v = hi + lo / 2048 (hi = f16(v), lo = f16((v - hi) 2048): 22 significant bits) and
//   y = sum(h_hi x_hi) + (sum(h_hi x_lo) + sum(h_lo x_hi)) / 2048
// with f32 accumulation -- three MFMAs per step, the h_lo x_lo term (2^-22) dropped
// (tests/test_mma_fir.py: the split form's error against f64 lfilter is the f32 direct form's).
// F filters on the same input share the staged window and the X fragments (stage A's pilot,
// stereo and RDS extract band-passes: F = 3).
// Every wave works alone -- no workgroup barrier after the tap fragments are built: a wave
// stages its own MM_WT-output window (MM_WT + 16 + 32 (KS - 1) samples, hi and lo) into its own
// LDS slice, runs its MFMAs, stores, and moves to its next window, whose samples it loaded
// into registers while the MFMAs ran.  Persistent: each wave owns every nw-th window of its job.
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef _Float16 h4v __attribute__((ext_vector_type(4)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int MM_NB = 4;                          // 256-output column blocks per wave window
constexpr int MM_WT = MM_NB * 256;                // outputs per wave window
constexpr float MM_LO = 2048.f;                   // the lo parts' scale
constexpr int MM_MIN_WIN = 32;                    // a row of fewer windows stays on the VALU tiles

template <int T>
struct MmaShape {
  static constexpr int KS = (16 + T - 1 + 31) / 32;                  // K steps of 32
  static constexpr int KOFF = (T - 1 + 7) / 8 * 8;                   // window start: 16-B aligned
  static constexpr int LU = MM_WT + 16 + 32 * (KS - 1);              // staged samples per window
  static constexpr int NCH = LU / 4, NQ = (NCH + 63) / 64;           // 16-B chunks, per lane
  static_assert(KOFF >= T - 1 && KOFF <= 32 * KS - 16, "every tap inside the K steps");
  static_assert(LU % 8 == 0, "16-B fragments");
};
constexpr int MM_LU_MAX = MmaShape<151>::LU;
constexpr int MM_TAPS_MAX = 3 * 151;
template <int FMAX> constexpr int mm_waves_per_cu() { return FMAX == 1 ? 12 : 8; }   // the VGPR limit

struct MmHL { _Float16 hi, lo; };
__device__ __forceinline__ MmHL mm_split(float v) {
  const _Float16 h = (_Float16)v;
  return MmHL{h, (_Float16)((v - (float)h) * MM_LO)};
}
// four samples at once: v_cvt_pk_f16_f32 pairs, the residuals as packed f32 ops
__device__ __forceinline__ void mm_split4(float4 x, h4v* hi, h4v* lo) {
  const f2 a{x.x, x.y}, c{x.z, x.w};
  const h2v ha = __builtin_convertvector(a, h2v), hc = __builtin_convertvector(c, h2v);
  const f2 ra = (a - __builtin_convertvector(ha, f2)) * MM_LO, rc = (c - __builtin_convertvector(hc, f2)) * MM_LO;
  const h2v la = __builtin_convertvector(ra, h2v), lc = __builtin_convertvector(rc, h2v);
  *hi = h4v{ha.x, ha.y, hc.x, hc.y};
  *lo = h4v{la.x, la.y, lc.x, lc.y};
}

// A buffer descriptor over bytes [p, p + bytes) from wave-uniform values (readfirstlane: the
// compiler cannot prove a wave-id-derived address uniform and would wrap every access in a
// waterfall loop).  Raw buffer accesses outside it read 0 / are dropped by the hardware.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mm_rsrc(const void* p, int64_t bytes) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int nb = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uintptr_t)hi << 32) | lo), 0, nb, 0x00020000);
}
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

// wave w of job group Jf: windows gw, gw + nw, ... of the job's (stream, window) list.  Every
// global access is a raw buffer access (the range check zero-fills samples outside the row and
// drops stores past its end: no edge paths) and unconditional, so the compiler's vmcnt waits
// count exactly; the loads of window i + 2 go out after window i's stores, and window i + 1's
// staging waits for its own loads only -- never for a store.
template <int T, int F>
__device__ __forceinline__ void mma_run(const StageJob* Jf, int S, int64_t gw, int64_t nw, _Float16* img,
                                        const float* tap_s) {
  using Sh = MmaShape<T>;
  constexpr int KS = Sh::KS, KOFF = Sh::KOFF, LU = Sh::LU, NCH = Sh::NCH, NQ = Sh::NQ;
  static_assert(F * T <= MM_TAPS_MAX && LU <= MM_LU_MAX, "the window fits the kernel's LDS");
  static_assert(NQ >= 2 && 1024 * (NQ - 2) < 4096, "chunk offsets: immediates up to NQ - 2");
  const StageJob& J = Jf[0];
  const int l = threadIdx.x & 63;
  const int b = l & 15, g = l >> 4;
  const int64_t wins = (J.n + MM_WT - 1) / MM_WT;   // per stream
  const int64_t total = wins * S;
  const int pre = J.pre;
  _Float16* xh = img;
  _Float16* xl = img + LU;
  // the tap fragments: lane l holds A[b = l & 15][j = 32 st + 8 (l >> 4) + e] = h[b + KOFF - j]
  h8v ah[F][KS], al[F][KS];
#pragma unroll
  for (int f = 0; f < F; ++f)
#pragma unroll
    for (int st = 0; st < KS; ++st)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = b + KOFF - (32 * st + 8 * g + e);
        const MmHL p = mm_split((k >= 0 && k < T) ? tap_s[f * T + k] : 0.f);
        ah[f][st][e] = p.hi;
        al[f][st][e] = p.lo;
      }
  // window i's samples: 16-B chunks l + 64 j of x[m0 - KOFF ...], at byte offset
  // 4 (m0 - KOFF) + 16 l + 1 024 j of the stream's row (negative: before the row, read as 0)
  constexpr int PFD = 2;                             // windows in flight
  u4v v[PFD][NQ];
  auto load = [&](int64_t i, u4v* vv) {
    const int s = (int)(i / wins);
    const int64_t m0 = (i - s * wins) * MM_WT;
    const __amdgpu_buffer_rsrc_t r = mm_rsrc(J.x + (int64_t)s * J.x_stride, J.n * 4);
    const int o = (int)(4 * (m0 - KOFF)) + 16 * l;
#pragma unroll
    for (int j = 0; j < NQ - 1; ++j) vv[j] = __builtin_amdgcn_raw_buffer_load_b128(r, o + 1024 * j, 0, 0);
    vv[NQ - 1] = __builtin_amdgcn_raw_buffer_load_b128(r, o + 1024 * (NQ - 1), 0, 0);
  };
#pragma unroll
  for (int d = 0; d < PFD; ++d) load(gw + d * nw, v[d]);   // (past the job's end: loads of 0 bytes' worth, unused)
  for (int64_t i = gw; i < total; i += nw) {
    const int s = (int)(i / wins);
    const int64_t m0 = (i - s * wins) * MM_WT;
    // stage: the wave's own LDS slice (its previous window's fragment reads retired in order)
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int q = l + j * 64;
      if (q < NCH) {
        float4 x = __builtin_bit_cast(float4, v[0][j]);
        if (pre == PRE_SQUARE) x = make_float4(x.x * x.x, x.y * x.y, x.z * x.z, x.w * x.w);
        h4v hv, lv;
        mm_split4(x, &hv, &lv);
        *reinterpret_cast<h4v*>(xh + 4 * q) = hv;
        *reinterpret_cast<h4v*>(xl + 4 * q) = lv;
      }
    }
#pragma unroll
    for (int d = 0; d + 1 < PFD; ++d)
#pragma unroll
      for (int j = 0; j < NQ; ++j) v[d][j] = v[d + 1][j];
    // the column blocks' K steps as one unrolled sequence, the X fragments of step q + 1 read
    // while step q's MFMAs run
    constexpr int NSTEP = MM_NB * KS;
    auto frag = [&](int q, h8v* bh, h8v* bl) {
      const int u = 256 * (q / KS) + 16 * b + 8 * g + 32 * (q % KS);
      *bh = *reinterpret_cast<const h8v*>(xh + u);
      *bl = *reinterpret_cast<const h8v*>(xl + u);
    };
    h8v fh[2], fl[2];
    f4v acc_h[F], acc_c[F];
    const bool head = m0 < T - 1;                    // the block's first T - 1 outputs: + lfilter zi
    __amdgpu_buffer_rsrc_t ry[F], r8[F];
#pragma unroll
    for (int f = 0; f < F; ++f) {
      // (a null row: an empty range -- its stores are dropped)
      ry[f] = mm_rsrc(Jf[f].y + (Jf[f].y ? (int64_t)s * Jf[f].y_stride + m0 : 0), Jf[f].y ? (J.n - m0) * 4 : 0);
      r8[f] = mm_rsrc(Jf[f].y8 + (Jf[f].y8 ? (int64_t)s * Jf[f].y8_stride + m0 : 0), Jf[f].y8 ? J.n - m0 : 0);
    }
    frag(0, &fh[0], &fl[0]);
    static_for<0, NSTEP>([&](auto Q) {
      constexpr int q = Q, st = q % KS, c = q / KS;
      if constexpr (q + 1 < NSTEP) frag(q + 1, &fh[(q + 1) % 2], &fl[(q + 1) % 2]);
      if constexpr (st == 0) {
#pragma unroll
        for (int f = 0; f < F; ++f) acc_h[f] = acc_c[f] = f4v{0.f, 0.f, 0.f, 0.f};
      }
      const h8v bh = fh[q % 2], bl = fl[q % 2];
#pragma unroll
      for (int f = 0; f < F; ++f) {
        acc_h[f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[f][st], bh, acc_h[f], 0, 0, 0);
        acc_c[f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[f][st], bl, acc_c[f], 0, 0, 0);
        acc_c[f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[f][st], bh, acc_c[f], 0, 0, 0);
      }
      if constexpr (st == KS - 1) {
        const int ol = 256 * c + 16 * b + 4 * g;     // this lane's 4 outputs: m0 + ol ...
#pragma unroll
        for (int f = 0; f < F; ++f) {
          const StageJob& Jj = Jf[f];
          float4 o = make_float4(fmaf(acc_c[f][0], 1.f / MM_LO, acc_h[f][0]), fmaf(acc_c[f][1], 1.f / MM_LO, acc_h[f][1]),
                                 fmaf(acc_c[f][2], 1.f / MM_LO, acc_h[f][2]), fmaf(acc_c[f][3], 1.f / MM_LO, acc_h[f][3]));
          if (head && Jj.zi != nullptr) {            // uniform: the stream's first window only
            const double* zi = Jj.zi + (int64_t)s * Jj.zi_stride;
            const int64_t n0 = m0 + ol;
            if (n0 + 0 < T - 1) o.x += (float)zi[n0 + 0];
            if (n0 + 1 < T - 1) o.y += (float)zi[n0 + 1];
            if (n0 + 2 < T - 1) o.z += (float)zi[n0 + 2];
            if (n0 + 3 < T - 1) o.w += (float)zi[n0 + 3];
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, o), ry[f], 4 * ol, 0, 0);
          if (Jj.y8 != nullptr) {                    // uniform: the four outputs' sign codes, one dword
            using sdrnco::pll_code;
            const uint32_t cw = (uint32_t)(uint8_t)pll_code(o.x) | (uint32_t)(uint8_t)pll_code(o.y) << 8 |
                                (uint32_t)(uint8_t)pll_code(o.z) << 16 | (uint32_t)(uint8_t)pll_code(o.w) << 24;
            __builtin_amdgcn_raw_buffer_store_b32(cw, r8[f], ol, 0, 0);
          }
          if (Jj.yh != nullptr) {                    // host rows (per-call runs): plain stores
            float* hb = Jj.yh + (int64_t)s * Jj.yh_stride;
            const int64_t n0 = m0 + ol;
            const float ov[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n0 + r < J.n) hb[n0 + r] = ov[r];
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    const int64_t nf = i + PFD * nw;                 // after this window's stores: see above
    if (nf < total) load(nf, v[PFD - 1]);
  }
}

// Any T (<= SDR_MAX_TAPS) and D: taps in LDS, inputs through the caches; outputs
// m0 + t + NT*r.  Also the combiner when asked.
__device__ __forceinline__ void fir_tile_any(const StageJob& J, int s, int64_t tile, float* lds) {
  const int t = threadIdx.x;
  for (int k = t; k < J.T; k += RX_NT) lds[k] = J.taps[k];
  __syncthreads();
  const int64_t M = (J.n + J.D - 1) / J.D;
  const float* xb = J.x + (int64_t)s * J.x_stride;
  const float* cb = J.c ? J.c + (int64_t)s * J.x_stride : nullptr;
  for (int r = 0; r < RX_R; ++r) {
    const int64_t m = tile * RX_TO + t + RX_NT * r;
    if (m >= M) break;
    const int64_t j0 = (int64_t)J.D * m;
    float acc = 0.f;
    const int khi = (int)min<int64_t>(J.T - 1, j0);
    for (int k = khi; k >= 0; --k)
      acc = fmaf(lds[k], pre_op(J.pre, xb[j0 - k], J.pre == PRE_MIX ? cb[j0 - k] : 0.f, J.gain), acc);
    if (J.zi != nullptr && j0 < J.T - 1) acc += (float)J.zi[(int64_t)s * J.zi_stride + j0];
    J.y[(int64_t)s * J.y_stride + m] = acc;
    if (J.yh) J.yh[(int64_t)s * J.yh_stride + m] = acc;
    if (J.mono != nullptr) {
      const float a = J.mono[(int64_t)s * J.y_stride + m];
      const float lv = (a + acc) * 0.5f, rv = (a - acc) * 0.5f;
      J.left[(int64_t)s * J.y_stride + m] = lv;
      J.right[(int64_t)s * J.y_stride + m] = rv;
      if (J.lh) J.lh[(int64_t)s * J.yh_stride + m] = lv;
      if (J.rh) J.rh[(int64_t)s * J.yh_stride + m] = rv;
    }
  }
}

// Rational resampler (model/fmRDSblock.py:184-199): lfilter on the x U zero-stuffed stream,
// [::D], times U, without materialising the zero-stuffed stream (only the taps with
// (D m - k) % U == 0 contribute; the input index walks down by one per term).
__device__ __forceinline__ void resample_tile(const StageJob& J, int s, int64_t tile, float* lds) {
  const int t = threadIdx.x;
  const int U = J.U, D = J.D;
  const int64_t M = (J.n * U + D - 1) / D;
  const float* xb = J.x + (int64_t)s * J.x_stride;
  // the tile's input window (outputs [m0, m0 + RX_TO) read x[(D m - k) / U] for k < T) and the
  // taps, staged in LDS: each output is ~T/U multiply-adds, so the tile is bound by how fast its
  // inputs arrive, not by arithmetic
  const int64_t m0 = tile * RX_TO;
  const int64_t xlo = max<int64_t>(0, (D * m0 - (J.T - 1)) / U - 1);
  const int64_t xhi = min<int64_t>(J.n, (D * (m0 + RX_TO - 1)) / U + 1);
  const int nx = (int)max<int64_t>(0, xhi - xlo);
  float* tap = lds;
  float* xs = lds + SDR_MAX_TAPS;
  if (J.T <= SDR_MAX_TAPS && nx <= RX_LDS - SDR_MAX_TAPS) {
    for (int k = t; k < J.T; k += RX_NT) tap[k] = J.taps[k];
    for (int i = t; i < nx; i += RX_NT) xs[i] = xb[xlo + i];
    __syncthreads();
    for (int r = 0; r < RX_R; ++r) {
      const int64_t m = m0 + t + RX_NT * r;
      if (m >= M) break;
      const int64_t j0 = (int64_t)D * m;
      const int k0 = (int)(j0 % U);
      const int khi = (int)min<int64_t>(J.T - 1, j0);
      int xi = (int)((j0 - k0) / U - xlo);
      float acc = 0.f;
      for (int k = k0; k <= khi; k += U, --xi) acc = fmaf(tap[k], xs[xi], acc);
      if (J.zi != nullptr && j0 < J.T - 1) acc += (float)J.zi[(int64_t)s * J.zi_stride + j0];
      J.y[(int64_t)s * J.y_stride + m] = acc * (float)U;
      if (J.yh) J.yh[(int64_t)s * J.yh_stride + m] = acc * (float)U;
    }
    return;
  }
  for (int k = t; k < J.T; k += RX_NT) lds[k] = J.taps[k];     // (taps beyond the LDS window: through the caches)
  __syncthreads();
  for (int r = 0; r < RX_R; ++r) {
    const int64_t m = m0 + t + RX_NT * r;
    if (m >= M) break;
    const int64_t j0 = (int64_t)D * m;
    const int k0 = (int)(j0 % U);
    const int khi = (int)min<int64_t>(J.T - 1, j0);
    int64_t xi = (j0 - k0) / U;
    float acc = 0.f;
    for (int k = k0; k <= khi; k += U, --xi) acc = fmaf(k < RX_LDS ? lds[k] : J.taps[k], xb[xi], acc);
    if (J.zi != nullptr && j0 < J.T - 1) acc += (float)J.zi[(int64_t)s * J.zi_stride + j0];
    J.y[(int64_t)s * J.y_stride + m] = acc * (float)U;
    if (J.yh) J.yh[(int64_t)s * J.yh_stride + m] = acc * (float)U;
  }
}

// lfilter final state of one (job, stream), f64, on the (zero-stuffed when U > 1) input:
//   zf[k] = sum_{j=k+1}^{T-1} b[j] u[NU+k-j] + (NU+k < T-1 ? zi[NU+k] : 0),  NU = n*U
// (the zf_kernel of fir.hip as extra workgroups of the producing stage).
template <bool NCO>
__device__ __forceinline__ void zf_block(const StageJobs& P, int64_t zb, float* lds) {
  const int q = P.zfj[zb / P.nstreams];
  const int s = (int)(zb % P.nstreams);
  const StageJob& J = P.j[q];
  const int U = J.kind == JK_RESAMPLE ? J.U : 1;
  const int T = J.T;
  const float* x = J.x + (int64_t)s * J.x_stride;
  const float* c = J.c ? J.c + (int64_t)s * J.x_stride : nullptr;
  const double* zi = J.zi ? J.zi + (int64_t)s * J.zi_stride : nullptr;
  double* zf = J.zf + (int64_t)s * J.zi_stride;
  const int64_t n = J.n, nu = n * U;
  const int L = (int)min<int64_t>(n, (T - 1) / U);
  double* bs = reinterpret_cast<double*>(lds);
  double* us = bs + T;
  for (int i = threadIdx.x; i < L; i += RX_NT) {
    const int64_t xi = n - 1 - i;
    double v = (double)x[xi];
    if (J.pre == PRE_SQUARE) v = v * v;
    else if (J.pre == PRE_MIX) v = (double)((x[xi] * c[xi]) * J.gain);
    else if (NCO && J.pre == PRE_NCO) v = (double)((x[xi] * nco_one(J, s, xi)) * J.gain);
    us[i] = v;
  }
  for (int i = threadIdx.x; i < T; i += RX_NT) bs[i] = J.taps64[i];
  __syncthreads();
  for (int k = threadIdx.x; k < T - 1; k += RX_NT) {
    const int jhi = (int)min<int64_t>(T - 1, nu + k);
    // four independent partial sums: a single accumulator is a chain of up to T-1
    // dependent f64 FMAs, each behind an LDS read (~7 us per launch at T = 151)
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int j = k + U, i = 0;
    for (; j + 3 * U <= jhi; j += 4 * U, i += 4) {
      a0 = fma(bs[j], us[i], a0);
      a1 = fma(bs[j + U], us[i + 1], a1);
      a2 = fma(bs[j + 2 * U], us[i + 2], a2);
      a3 = fma(bs[j + 3 * U], us[i + 3], a3);
    }
    for (; j <= jhi; j += U, ++i) a0 = fma(bs[j], us[i], a0);
    double acc = (a0 + a1) + (a2 + a3);
    if (zi != nullptr && nu + k < T - 1) acc += zi[nu + k];
    zf[k] = acc;
  }
}

// I/Q final states of one stream (the iq_zf_kernel of fe.hip as workgroups of stage A):
//   zf[k] = sum_{j=k+1}^{T-1} b[j] x[n-1-(j-k-1)] + (n+k < T-1 ? zi[n+k] : 0)
// and the demod phase state.
__device__ __forceinline__ void fe_state_block(const FeState& F, int s, float* lds) {
  float2* xs = reinterpret_cast<float2*>(lds);                  // xs[i] = x[n-1-i]
  double* bs = reinterpret_cast<double*>(lds + 2 * SDR_MAX_TAPS);
  const int t = threadIdx.x;
  const int64_t base = (int64_t)s * F.stride;
  const int L = (int)min<int64_t>(F.n, F.T - 1);
  for (int i = t; i < L; i += RX_NT) {
    const int64_t k = base + F.n - 1 - i;
    if (F.u8) {
      const uint8_t* q = static_cast<const uint8_t*>(F.iq) + 2 * k;
      xs[i] = make_float2(((float)q[0] - 128.f) / 128.f, ((float)q[1] - 128.f) / 128.f);
    } else {
      xs[i] = static_cast<const float2*>(F.iq)[k];
    }
  }
  for (int i = t; i < F.T; i += RX_NT) bs[i] = F.b[i];
  __syncthreads();
  const double* zii = F.zi_i + (int64_t)s * F.zs;
  const double* ziq = F.zi_q + (int64_t)s * F.zs;
  for (int k = t; k < F.T - 1; k += RX_NT) {
    const int jhi = (int)min<int64_t>(F.T - 1, F.n + k);
    double si0 = 0.0, sq0 = 0.0, si1 = 0.0, sq1 = 0.0;   // two partial sums per channel
    int j = k + 1;
    for (; j + 1 <= jhi; j += 2) {
      const float2 v0 = xs[j - k - 1], v1 = xs[j - k];
      si0 = fma(bs[j], (double)v0.x, si0);
      sq0 = fma(bs[j], (double)v0.y, sq0);
      si1 = fma(bs[j + 1], (double)v1.x, si1);
      sq1 = fma(bs[j + 1], (double)v1.y, sq1);
    }
    if (j <= jhi) {
      const float2 v = xs[j - k - 1];
      si0 = fma(bs[j], (double)v.x, si0);
      sq0 = fma(bs[j], (double)v.y, sq0);
    }
    double si = si0 + si1, sq = sq0 + sq1;
    if (F.n + k < F.T - 1) {
      si += zii[F.n + k];
      sq += ziq[F.n + k];
    }
    F.zf_i[(int64_t)s * F.zs + k] = si;
    F.zf_q[(int64_t)s * F.zs + k] = sq;
  }
  if (t == 0 && F.n > 0) {                     // model/fmSupportLib.py:40-44: accumulated phase
    F.phase[s] = (double)F.last_phi[s] + 6.28318530717958647692 * (double)F.wraps[s];
    F.wraps[s] = 0;
  }
}

// One stage launch.  T > 0: every FIR job of the launch has T taps (compile-time tiles for
// D = 1 and 5); T == 0: any tap count.  Workgroups map to (job, stream, tile) in job order,
// then to the zf work.  NCO: the launch has PRE_NCO jobs (stage C's mixers; T > 0 only) --
// a separate instantiation, so the other stages keep their registers.
template <int T, bool NCO = false, bool FOLD = false>
__global__ __launch_bounds__(RX_NT) void rx_stage_kernel(StageJobs P) {
  static_assert(!NCO || T > 0, "PRE_NCO jobs run on the compile-time tiles");
  static_assert(!FOLD || (T == 151 && !NCO), "fold groups: 151 taps, no NCO jobs");
  __shared__ __attribute__((aligned(16))) float lds[RX_LDS];
  // the final-state workgroups first: each is a short serial f64 pass, dispatched ahead of the
  // tiles it would otherwise trail at the end of the launch
  const int64_t nzb = (int64_t)P.nzf * P.nstreams, nfront = nzb + (P.fe.on ? P.nstreams : 0);
  if ((int64_t)blockIdx.x < nfront) {
    const int64_t zb = blockIdx.x;
    if (zb < nzb) zf_block<NCO>(P, zb, lds);
    else fe_state_block(P.fe, (int)(zb - nzb), lds);
    return;
  }
  const int64_t b = blockIdx.x - nfront;
  int q = 0;
  for (int i = 1; i < P.njobs; ++i)
    if (b >= P.j[i].b0) q = i;
  const StageJob& J = P.j[q];
  const int64_t bl = b - J.b0;
  const int s = (int)(bl / J.tiles);
  const int64_t tile = bl - (int64_t)s * J.tiles;
  if (J.kind == JK_RESAMPLE) {
    resample_tile(J, s, tile, lds);
    return;
  }
  if constexpr (FOLD) {
    if (J.fold == 3) { pair_tile<151, 8, 3, true>(&J, s, tile, lds); return; }
    if (J.fold == 2) { pair_tile<151, 8, 2, true>(&J, s, tile, lds); return; }
  }
  if constexpr (T > 0) {
    if (J.D == 1) {
      if (NCO && J.pre == PRE_NCO) {                 // the mixers forming their NCO
        if (J.small) fir_tile<T, 1, 4, NCO>(J, s, tile, lds);
        else fir_tile<T, 1, 16, NCO>(J, s, tile, lds);
      } else if (J.small) {
        pair_tile<T, 2, 1, false>(&J, s, tile, lds);
      } else {
        pair_tile<T, 8, 1, false>(&J, s, tile, lds);
      }
      return;
    }
    if (J.D == 5) { fir_tile<T, 5, 4, NCO>(J, s, tile, lds); return; }
  }
  fir_tile_any(J, s, tile, lds);
}

// The matrix-core FIR launch of one tap class and group width: job q (a group of F = fold
// filters on one input) owns workgroups [b0, b0 + wgs), i.e. waves 4 b0 ... 4 (b0 + wgs) - 1,
// each running every (4 wgs)-th window of the job's streams x windows (mma_run).
template <int T, int FMAX>
__global__ __launch_bounds__(RX_NT) __attribute__((amdgpu_waves_per_eu(mm_waves_per_cu<FMAX>() / 4)))
void rx_mma_kernel(StageJobs P) {
  __shared__ __attribute__((aligned(16))) _Float16 img[4][2 * MmaShape<T>::LU];
  __shared__ float tap_s[FMAX * T];
  // the final-state workgroups first (the jobs' zf, and the FE state when the launch carries
  // it): they run beside the persistent waves instead of in a launch of their own
  const int64_t nzb = (int64_t)P.nzf * P.nstreams, nfront = nzb + (P.fe.on ? P.nstreams : 0);
  if ((int64_t)blockIdx.x < nfront) {
    float* lf = reinterpret_cast<float*>(&img[0][0]);
    if ((int64_t)blockIdx.x < nzb) zf_block<false>(P, blockIdx.x, lf);
    else fe_state_block(P.fe, (int)(blockIdx.x - nzb), lf);
    return;
  }
  const int64_t b = blockIdx.x - nfront;
  int q = 0;
  for (int i = 1; i < P.njobs; ++i)
    if (b >= P.j[i].b0) q = i;
  const StageJob& J = P.j[q];
  const int F = J.fold;
  for (int i = threadIdx.x; i < F * T; i += RX_NT) tap_s[i] = P.j[q + i / T].taps[i % T];
  __syncthreads();
  // the wave id, provably uniform (readfirstlane): everything derived from it -- stream, window,
  // row addresses, pseudo-block records -- stays in scalar registers
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t gw = (b - J.b0) * 4 + w, nw = (int64_t)J.wgs * 4;
  if constexpr (FMAX == 1) {
    mma_run<T, 1>(&J, P.nstreams, gw, nw, img[w], tap_s);
  } else {
    if (F == 3) mma_run<T, 3>(&J, P.nstreams, gw, nw, img[w], tap_s);
    else mma_run<T, 2>(&J, P.nstreams, gw, nw, img[w], tap_s);
  }
}

// ---- decimate-by-5 LPFs on the matrix cores (spans): stage C's stereo mixer + LPF + L/R
// combiner (MIX) and stage A's mono audio LPF ------------------------------------------------
// y[m] = sum_k h[k] u[5 m - k] with u = x (mono, model/fmMonoBlock.py:101-109) or u[i] = (x[i]
// nco[i]) g (stereo, :155-162, the NCO formed from the pilot PLL's phases, sdr_nco.h): the 16
// outputs m = m0 + 16 c + b of column c of a 256-output window are Y = A X with A[b][j] =
// h[5 b + 151 - j] (zero outside the taps) and X[j][c] = u[5 m0 + 80 c + j - 151], j < 256 --
// the Hankel form of the composite kernel (columns 80 inputs apart; odd window starts: each
// chunk's four phases are two aligned pairs), one channel; A's 8 K steps built once per
// workgroup into LDS.  MIX's epilogue is the combiner (:166-170): L = (mono + y) / 2,
// R = (mono - y) / 2; every global access of the loop is unconditional (buffer loads / stores
// with the range check at the row ends), so the compiler's vmcnt waits count exactly and the
// next window's prefetched chunks are never waited for early.
constexpr int SM_KS = 8, SM_KOFF = 151, SM_D = 5;
constexpr int SM_LU = 80 * 15 + 32 * SM_KS;         // 1 456 inputs staged per window
constexpr int SM_NG = SM_LU / 4, SM_NQ = (SM_NG + 63) / 64;
template <bool MIX> constexpr int sm_wpe() { return MIX ? 2 : 4; }   // waves per SIMD (registers; LDS: 4 x 39.7 KB)
static_assert(SM_D * 15 + SM_KOFF < 32 * SM_KS && SM_KOFF >= 150 && SM_KOFF % 2 == 1, "LPF window");

// TH32 (MIX): the pilot loop's phase rows are compact (sdr_nco.h, PllJob::th32)
template <bool MIX, bool TH32 = false>
__global__ __launch_bounds__(RX_NT) __attribute__((amdgpu_waves_per_eu(sm_wpe<MIX>()))) void rx_decmm_kernel(StageJobs P,
                                                                                                             int wgs) {
  const StageJob& J = P.j[0];                        // (in the kernel arguments: no private copy)
  const int S = P.nstreams;
  __shared__ __attribute__((aligned(16))) _Float16 img[4][2 * SM_LU];   // per wave: hi, lo
  __shared__ __attribute__((aligned(16))) h8v afr[2][SM_KS][64];         // A fragments: hi, lo
  const int nfront = P.nzf * S + (P.fe.on ? S : 0);
  if ((int)blockIdx.x < nfront) {                    // final states first (as rx_mma_kernel)
    float* lf = reinterpret_cast<float*>(&img[0][0]);
    if ((int)blockIdx.x < P.nzf * S) zf_block<MIX>(P, blockIdx.x, lf);
    else fe_state_block(P.fe, (int)blockIdx.x - P.nzf * S, lf);
    return;
  }
  const int bx = (int)blockIdx.x - nfront;
  constexpr int T = 151;
  for (int idx = threadIdx.x; idx < SM_KS * 64; idx += RX_NT) {
    const int st = idx >> 6, ln = idx & 63, bb = ln & 15, gg = ln >> 4;
    h8v hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = SM_D * bb + SM_KOFF - (32 * st + 8 * gg + e);
      const MmHL p = mm_split((k >= 0 && k < T) ? J.taps[k] : 0.f);
      hi[e] = p.hi;
      lo[e] = p.lo;
    }
    afr[0][st][ln] = hi;
    afr[1][st][ln] = lo;
  }
  __syncthreads();
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // uniform: see rx_mma_kernel
  const int l = threadIdx.x & 63, b = l & 15, g = l >> 4;
  const int64_t gw = (int64_t)bx * 4 + w, nw = (int64_t)wgs * 4;
  _Float16* xh = img[w];
  _Float16* xl = xh + SM_LU;
  const int64_t n = J.n, M = (J.n + SM_D - 1) / SM_D;
  const int64_t wins = (M + 255) / 256;              // per stream
  const int64_t total = wins * S;
  const float gain = J.gain;
  // A window's geometry (and, MIX, pseudo-block records); every window (row ends included:
  // mix_eval) takes the same branch-free path.  The chunks' loads run PD chunks ahead of their
  // arithmetic through the window seams: the last PD chunks of a window issue the next
  // window's first ones (its records were read a window earlier).
  static_assert((SM_D * 256 - SM_KOFF) % 4 == 1 && SM_KOFF % 4 == 3, "chunks start at 1 mod 4 (mix_load)");
  struct Win { int s; int64_t m0, a; const float* x; NcoTile nt; bool lin; };
  auto winfo = [&](int64_t i, Win* v) {
    v->s = (int)(i / wins);
    const int64_t W = i - (int64_t)v->s * wins;
    v->m0 = 256 * W;
    v->a = SM_D * v->m0 - SM_KOFF;                   // input of element 0
    v->x = J.x + (int64_t)v->s * J.x_stride;
    if constexpr (MIX) {
      v->nt = nco_tile(J.nco, v->s, max<int64_t>(v->a, 1) - 1);
      v->lin = nco_tile_lin(v->nt);
    }
  };
  constexpr int PD = 2;
  static_assert(SM_NQ % PD == 0, "ring slots line up across windows");
  MixLd gb[PD];
  auto ldg = [&](const Win& v, int j, MixLd* gg) {
    const int64_t i0 = v.a + 4 * min(l + 64 * j, SM_NG - 1);
    if constexpr (MIX) mix_load<TH32>(J.nco, v.nt, v.x, i0, v.lin, gg);
    else __builtin_memcpy(&gg->x, v.x + (i0 > 0 ? i0 : (int64_t)0), sizeof(float4));
  };
  Win cur{}, nxt{};
  if (gw < total) {
    winfo(gw, &cur);
    static_for<0, PD>([&](auto D) { ldg(cur, D, &gb[D]); });
  }
  for (int64_t i = gw; i < total; i += nw) {
    const bool more = i + nw < total;
    if (more) winfo(i + nw, &nxt);
    const int s = cur.s;
    const int64_t m0 = cur.m0, a = cur.a;
    const int64_t n0 = m0 + 16 * b + 4 * g;          // this lane's 4 outputs
    // (MIX) the combiner's mono inputs, loaded before this window's prefetches: waiting for
    // them later never waits for those
    f4v mv = f4v{0.f, 0.f, 0.f, 0.f};
    if constexpr (MIX) {
      const __amdgpu_buffer_rsrc_t rm = mm_rsrc(J.mono + (int64_t)s * J.y_stride + m0, (M - m0) * 4);
      mv = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rm, (int)(4 * (n0 - m0)), 0, 0));
    }
    {
      NcoWin nwin{};
      float c0 = 0.f;
      if constexpr (MIX) {
        nwin = nco_win(J.nco, cur.nt, a);
        c0 = J.nco.nco_i[(int64_t)s * J.nco.out_stride];   // the carried NCO[0]
      }
      static_for<0, SM_NQ>([&](auto JJ) {
        constexpr int j = JJ;
        const int q = min(l + 64 * j, SM_NG - 1);
        const MixLd gc = gb[j % PD];
        if constexpr (j + PD < SM_NQ) ldg(cur, j + PD, &gb[j % PD]);
        else ldg(more ? nxt : cur, j + PD - SM_NQ, &gb[j % PD]);
        const int64_t i0 = a + 4 * q;
        float u[4];
        if constexpr (MIX) {
          float xv[4], c[4], sn[4];
          mix_eval<TH32>(cur.nt, nwin, i0, n, gc, cur.lin, c0, 0.f, xv, c, sn);
#pragma unroll
          for (int e = 0; e < 4; ++e) u[e] = pre_op(PRE_NCO, xv[e], c[e], gain);
        } else {                                     // (the edges as mix_eval)
          const bool head = i0 == -3, tail = i0 == n - 3, out = (i0 < 0 && !head) || i0 >= n;
          u[0] = (head || out) ? 0.f : gc.x.x;
          u[1] = (head || out) ? 0.f : gc.x.y;
          u[2] = (head || out) ? 0.f : gc.x.z;
          u[3] = head ? gc.x.x : ((tail || out) ? 0.f : gc.x.w);
        }
        h4v hv, lv;
        mm_split4(make_float4(u[0], u[1], u[2], u[3]), &hv, &lv);
        *reinterpret_cast<h4v*>(xh + 4 * q) = hv;
        *reinterpret_cast<h4v*>(xl + 4 * q) = lv;
        __builtin_amdgcn_sched_barrier(0);
      });
    }
    f4v acc_h = f4v{0.f, 0.f, 0.f, 0.f}, acc_c = acc_h;
    struct Fr { h8v xh, xl, ah, al; };
    Fr fr[2];
    auto frag = [&](int st, Fr* d) {
      const int uu = 80 * b + 32 * st + 8 * g;
      d->xh = *reinterpret_cast<const h8v*>(xh + uu);
      d->xl = *reinterpret_cast<const h8v*>(xl + uu);
      d->ah = afr[0][st][l];
      d->al = afr[1][st][l];
    };
    frag(0, &fr[0]);
    static_for<0, SM_KS>([&](auto ST) {
      constexpr int st = ST;
      if constexpr (st + 1 < SM_KS) frag(st + 1, &fr[(st + 1) % 2]);
      const Fr& f = fr[st % 2];
      acc_h = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.ah, f.xh, acc_h, 0, 0, 0);
      acc_c = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.ah, f.xl, acc_c, 0, 0, 0);
      acc_c = __builtin_amdgcn_mfma_f32_16x16x32_f16(f.al, f.xh, acc_c, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    // outputs n0 .. n0 + 3: the LPF (and, MIX, the combiner's L and R)
    f4v y;
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = fmaf(acc_c[r], 1.f / MM_LO, acc_h[r]);
    if (m0 == 0 && J.zi != nullptr) {                // lfilter zi: the stream's first outputs
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t nn = SM_D * (n0 + r);
        if (nn < T - 1) y[r] += (float)J.zi[(int64_t)s * J.zi_stride + nn];
      }
    }
    const int ob = (int)(4 * (n0 - m0));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, y),
                                           mm_rsrc(J.y + (int64_t)s * J.y_stride + m0, (M - m0) * 4), ob, 0, 0);
    f4v lv, rv;
    if constexpr (MIX) {
      lv = (mv + y) * 0.5f;
      rv = (mv - y) * 0.5f;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, lv),
                                             mm_rsrc(J.left + (int64_t)s * J.y_stride + m0, (M - m0) * 4), ob, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, rv),
                                             mm_rsrc(J.right + (int64_t)s * J.y_stride + m0, (M - m0) * 4), ob, 0, 0);
    }
    if (J.yh != nullptr || (MIX && (J.lh != nullptr || J.rh != nullptr))) {   // host rows (per-call runs)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n0 + r < M) {
          if (J.yh) J.yh[(int64_t)s * J.yh_stride + n0 + r] = y[r];
          if constexpr (MIX) {
            if (J.lh) J.lh[(int64_t)s * J.yh_stride + n0 + r] = lv[r];
            if (J.rh) J.rh[(int64_t)s * J.yh_stride + n0 + r] = rv[r];
          }
        }
    }
    cur = nxt;
  }
}

// outputs per tile of a job in a launch of tap class `key` (as rx_stage_kernel<key> picks the tile)
int64_t tile_outputs(const StageJob& j, int key) {
  static_assert(PairShape<151, 2>::TO == FirShape<151, 1, 4>::TO && PairShape<151, 8>::TO == FirShape<151, 1>::TO &&
                PairShape<101, 2>::TO == FirShape<101, 1, 4>::TO && PairShape<101, 8>::TO == FirShape<101, 1>::TO,
                "pair tiles and the mixers' fir tiles cover the same outputs");
  if (j.kind == JK_FIR && key == 151 && j.D == 1 && j.small) return FirShape<151, 1, 4>::TO;
  if (j.kind == JK_FIR && key == 101 && j.D == 1 && j.small) return FirShape<101, 1, 4>::TO;
  if (j.kind == JK_FIR && key == 151 && j.D == 1) return FirShape<151, 1>::TO;
  if (j.kind == JK_FIR && key == 151 && j.D == 5) return FirShape<151, 5>::TO;
  if (j.kind == JK_FIR && key == 101 && j.D == 1) return FirShape<101, 1>::TO;
  if (j.kind == JK_FIR && key == 101 && j.D == 5) return FirShape<101, 5>::TO;
  return RX_TO;
}

// Launch the jobs of one stage, one launch per tap-count class.
hipError_t launch_stage(std::vector<StageJob> jobs, int S, hipStream_t st, const FeState* fe = nullptr) {
  auto cls = [](const StageJob& j) { return (j.kind == JK_FIR && (j.T == 101 || j.T == 151)) ? j.T : 0; };
  // matrix-core FIR launches first: D = 1 filters of 101 / 151 taps on 16-B aligned rows of at
  // least MM_MIN_WIN windows per stream (spans; per-block calls keep the VALU tiles' finer
  // grain) -- decided per job from its length alone, so a stream's outputs do not depend on how
  // many streams share the launch.  Their final states stay with the VALU launch below (tiles = 0).
  auto al16 = [](const void* p, int64_t stride) { return p != nullptr && ((uintptr_t)p % 16) == 0 && stride % 4 == 0; };
  auto mmable = [&](const StageJob& j, int key) {
    return j.kind == JK_FIR && j.D == 1 && j.T == key && (j.pre == PRE_NONE || j.pre == PRE_SQUARE) &&
           al16(j.x, j.x_stride) && (al16(j.y, j.y_stride) || (j.y == nullptr && j.y8 != nullptr)) &&
           j.n >= (int64_t)MM_MIN_WIN * MM_WT &&
           j.n % 4 == 0 && j.n < (int64_t)1 << 28;      // (buffer ranges: 32-bit byte offsets)
  };
  for (StageJob& j : jobs) j.mma = 0;
  bool fe_done = fe == nullptr || !fe->on;
  // the decimate-by-5 LPFs: stage C's stereo mixer + LPF + combiner, stage A's mono LPF
  // (rx_decmm_kernel; zf and the FE state ride on the launch)
  for (StageJob& j : jobs) {
    const bool mix = j.pre == PRE_NCO && !j.nco_sin && j.mono != nullptr && j.left != nullptr && j.right != nullptr &&
                     j.nco.theta != nullptr && al16(j.mono, j.y_stride) && al16(j.left, j.y_stride) &&
                     al16(j.right, j.y_stride);
    const bool mono = j.pre == PRE_NONE && j.mono == nullptr;
    if (!(j.kind == JK_FIR && j.D == SM_D && j.T == 151 && (mix || mono) && al16(j.y, j.y_stride) &&
          j.x != nullptr && j.n >= (int64_t)MM_MIN_WIN * MM_WT && j.n < (int64_t)1 << 28 && j.n % 4 == 0))
      continue;                                      // (n = 0 mod 4: the chunks' edges, mix_load)
    const int64_t wins = (j.n / SM_D + 256) / 256 * S;
    const int wgs = (int)std::min<int64_t>((mix ? sm_wpe<true>() : sm_wpe<false>()) * 256, (wins + 3) / 4);
    StageJobs Q{};
    Q.j[0] = j;
    Q.njobs = 1;
    Q.nstreams = S;
    if (j.zf != nullptr && j.T > 1) Q.zfj[Q.nzf++] = 0;
    if (!fe_done) {
      Q.fe = *fe;
      fe_done = true;
    }
    const unsigned grid = (unsigned)(wgs + Q.nzf * S + (Q.fe.on ? S : 0));
    if (mix && j.nco.th32) hipLaunchKernelGGL((rx_decmm_kernel<true, true>), dim3(grid), dim3(RX_NT), 0, st, Q, wgs);
    else if (mix) hipLaunchKernelGGL(rx_decmm_kernel<true>, dim3(grid), dim3(RX_NT), 0, st, Q, wgs);
    else hipLaunchKernelGGL(rx_decmm_kernel<false>, dim3(grid), dim3(RX_NT), 0, st, Q, wgs);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    j.mma = 1;
    j.zf = nullptr;                                  // (written by that launch)
  }
  for (int key : {151, 101})
    for (int wide : {1, 0}) {                        // groups of 2-3 filters / single filters
      StageJobs Q{};
      Q.nstreams = S;
      std::vector<size_t> members;
      for (size_t ji = 0; ji < jobs.size(); ++ji) {
        if (!mmable(jobs[ji], key) || jobs[ji].mma) continue;
        int g = 1;                                   // jobs on the same input: one group (<= 3)
        while (jobs[ji].pre == PRE_NONE && g < 3 && ji + g < jobs.size() && mmable(jobs[ji + g], key) &&
               jobs[ji + g].pre == PRE_NONE && jobs[ji + g].x == jobs[ji].x && jobs[ji + g].x_stride == jobs[ji].x_stride &&
               jobs[ji + g].n == jobs[ji].n)
          ++g;
        if ((g > 1) != (wide == 1) || Q.njobs + g > RX_MAXJ) {
          ji += g - 1;
          continue;
        }
        for (int m = 0; m < g; ++m) {
          StageJob j = jobs[ji + m];
          j.fold = m == 0 ? g : 0;
          j.wgs = 0;
          if (j.zf != nullptr && j.T > 1) Q.zfj[Q.nzf++] = Q.njobs;
          Q.j[Q.njobs++] = j;
          members.push_back(ji + m);
        }
        ji += g - 1;
      }
      if (Q.njobs == 0) continue;
      // persistent waves: mm_waves_per_cu per CU over the launch, shared by the groups in
      // proportion to their windows (every group at least one workgroup)
      const int64_t waves = 256 * (wide ? mm_waves_per_cu<3>() : mm_waves_per_cu<1>());
      int64_t wins = 0;
      for (int i = 0; i < Q.njobs; ++i)
        if (Q.j[i].fold > 0) wins += (Q.j[i].n + MM_WT - 1) / MM_WT * S;
      const int64_t per = std::max<int64_t>(1, (wins + waves - 1) / waves);     // windows per wave
      int64_t blocks = 0;
      for (int i = 0; i < Q.njobs; ++i) {
        StageJob& j = Q.j[i];
        j.b0 = blocks;
        if (j.fold > 0) {
          const int64_t jw = (j.n + MM_WT - 1) / MM_WT * S;
          j.wgs = (int)std::max<int64_t>(1, (jw + 4 * per - 1) / (4 * per));
          blocks += j.wgs;
        }
      }
      Q.tile_blocks = blocks;
      if (!fe_done) {                                // the FE state rides on the first launch
        Q.fe = *fe;
        fe_done = true;
      }
      const int64_t grid = blocks + (int64_t)Q.nzf * S + (Q.fe.on ? S : 0);
      if (key == 151 && wide) hipLaunchKernelGGL((rx_mma_kernel<151, 3>), dim3((unsigned)grid), dim3(RX_NT), 0, st, Q);
      else if (key == 151) hipLaunchKernelGGL((rx_mma_kernel<151, 1>), dim3((unsigned)grid), dim3(RX_NT), 0, st, Q);
      else if (wide) hipLaunchKernelGGL((rx_mma_kernel<101, 3>), dim3((unsigned)grid), dim3(RX_NT), 0, st, Q);
      else hipLaunchKernelGGL((rx_mma_kernel<101, 1>), dim3((unsigned)grid), dim3(RX_NT), 0, st, Q);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      for (size_t m : members) {
        jobs[m].mma = 1;
        jobs[m].zf = nullptr;                        // (written by that launch)
      }
    }
  for (const StageJob& j : jobs)                     // sign-code outputs: the matrix-core tiles only
    if (!j.mma && (j.y8 != nullptr || j.y == nullptr)) return hipErrorInvalidValue;
  for (int key : {151, 101, 0}) {
    StageJobs P{};
    P.nstreams = S;
    int64_t blocks = 0;
    // a launch whose tiles would give fewer than ~2.5 workgroups per CU (C5 per-block at 64
    // streams: RDS x^2 + BPF, mixers + LPFs, RRC; not the 4-filter stage A) runs its D = 1 jobs
    // in 1 024-output tiles (4 per lane): latency-bound launches get 4x the waves
    int64_t big = 0;
    for (const StageJob& j : jobs)
      if (cls(j) == key && !j.mma) {
        const int64_t nout = j.kind == JK_RESAMPLE ? (j.n * j.U + j.D - 1) / j.D : (j.n + j.D - 1) / j.D;
        big += (nout + 1023) / 1024 * S;
      }
    const bool small = key > 0 && big < 10 * 256;
    // symmetric 151-tap D = 1 jobs on one input, consecutive in the list: folded together (fold_tile)
    auto foldable = [&](const StageJob& a) {
      return key == 151 && !small && !a.mma && a.kind == JK_FIR && a.D == 1 && a.pre == PRE_NONE && a.T == 151 && a.sym;
    };
    int follow = 0;                                  // jobs left in the current fold group
    for (size_t ji = 0; ji < jobs.size(); ++ji) {
      const StageJob& j0 = jobs[ji];
      if (cls(j0) != key) continue;
      if (P.njobs == RX_MAXJ) return hipErrorInvalidValue;
      StageJob j = j0;
      const int64_t nout = j.kind == JK_RESAMPLE ? (j.n * j.U + j.D - 1) / j.D : (j.n + j.D - 1) / j.D;
      j.small = (small && j.kind == JK_FIR && j.D == 1) ? 1 : 0;
      j.fold = 0;
      if (follow == 0 && foldable(j)) {
        int g = 1;
        while (g < 3 && ji + g < jobs.size() && foldable(jobs[ji + g]) && jobs[ji + g].x == j.x &&
               jobs[ji + g].x_stride == j.x_stride && jobs[ji + g].n == j.n && P.njobs + g < RX_MAXJ)
          ++g;
        if (g > 1) { j.fold = g; follow = g; }
      }
      const bool follower = follow > 0 && j.fold == 0;
      if (follow > 0) --follow;
      const int64_t to = tile_outputs(j, key);
      j.tiles = (follower || j.mma) ? 0 : (int)std::max<int64_t>((nout + to - 1) / to, 0);
      j.b0 = blocks;
      blocks += (int64_t)j.tiles * S;
      if (j.zf != nullptr && j.T > 1) P.zfj[P.nzf++] = P.njobs;
      P.j[P.njobs++] = j;
    }
    if (P.njobs == 0 && (fe_done || key != 0)) continue;
    if (!fe_done) {                       // the FE state rides on the first launch
      P.fe = *fe;
      fe_done = true;
    }
    P.tile_blocks = blocks;
    const int64_t grid = blocks + (int64_t)P.nzf * S + (P.fe.on ? S : 0);
    if (grid <= 0) continue;
    if (grid > 0x7fffffff) return hipErrorInvalidValue;
    bool nco = false;
    for (int i = 0; i < P.njobs; ++i) nco = nco || P.j[i].pre == PRE_NCO;
    if (nco && key == 0) return hipErrorInvalidValue;     // (the receiver never asks: stage_nco_ok)
    bool fold = false;
    for (int i = 0; i < P.njobs; ++i) fold = fold || P.j[i].fold > 1;
    if (fold && (nco || key != 151)) return hipErrorInvalidValue;
    if (fold) hipLaunchKernelGGL((rx_stage_kernel<151, false, true>), dim3((unsigned)grid), dim3(RX_NT), 0, st, P);
    else if (key == 151 && nco) hipLaunchKernelGGL((rx_stage_kernel<151, true>), dim3((unsigned)grid), dim3(RX_NT), 0, st, P);
    else if (key == 151) hipLaunchKernelGGL(rx_stage_kernel<151>, dim3((unsigned)grid), dim3(RX_NT), 0, st, P);
    else if (key == 101 && nco) hipLaunchKernelGGL((rx_stage_kernel<101, true>), dim3((unsigned)grid), dim3(RX_NT), 0, st, P);
    else if (key == 101) hipLaunchKernelGGL(rx_stage_kernel<101>, dim3((unsigned)grid), dim3(RX_NT), 0, st, P);
    else hipLaunchKernelGGL(rx_stage_kernel<0>, dim3((unsigned)grid), dim3(RX_NT), 0, st, P);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// ---- RDS: I/Q mixers + 3 kHz LPF + x19 zero-stuff + anti-image LPF + [::80] x19 as ONE
// composite polyphase filter (model/fmRDSblock.py:172-199) ------------
// With mixed_{I,Q}[i] = 2 x[i] nco_{I,Q}[i], lpf = h * mixed (151 taps at 240 kS/s) and
// u[19 i] = lpf[i] (zero elsewhere), the resampler's output is
//   r[m] = 19 sum_j g[j] u[80 m - j] = 19 sum_{s} g[rho + 19 s] lpf[i0 - s],
//   i0 = floor(80 m / 19), rho = 80 m mod 19 (only j = rho + 19 s hits a stuffed sample)
//        = sum_{t=0}^{157} C_rho[t] x[i0 - t] nco[i0 - t],   C_rho[t] = 38 sum_s g[rho + 19 s] h[t - s]
// -- 158 multiply-adds per output and channel where the two-stage form spends 151 per INPUT
// (4.2 inputs per output) plus the resampler: 4x fewer.  Block starts carry the lfilter
// states exactly: the LPF's zi enters lpf[i < 150] and the anti-image zi enters a[q < 150]
// (the head corrections below), and one workgroup per stream writes both filters' final
// states (the LPF's from the last 150 mixed inputs, the anti-image's from the last 8 lpf
// values, as lfilter would).  The lpf rows themselves are only computed when asked for.
//
// Tile: 64 groups x 19 phases = 1 216 outputs m = m0 + 19 L + c (m0 = 1 216 tile): output
// (c, L) reads the 158 inputs before i0 = I0 + 80 L + base_c (I0 = 80 m0 / 19, base_c =
// floor(80 c / 19)), so group L's 19 outputs share a window of 234 inputs starting at
// I0 + 80 L - 158.  The tile's window (5 274 inputs, I and Q mixed) is staged in LDS once;
// lane L of wave w computes phases [5w, 5w + 5) of group L: per pair of window samples one
// 16-B LDS read, and per phase one tap pair (a 64-bit SGPR operand, compile-time offset) and
// two v_pk_fma_f32 (I and Q together, the tap broadcast by op_sel).  The phase's taps are
// uniform across the wave because 80 * 19 = 4 * 19 * 20: outputs 19 apart share rho.
constexpr int CR_U = 19, CR_D = 80, CR_T = 151;
constexpr int CR_CT = CR_T + (CR_T - 1) / CR_U;          // 158 composite taps per phase
constexpr int CR_G = 64, CR_NW = 4, CR_NT = 64 * CR_NW;
constexpr int CR_TO = CR_U * CR_G;                       // outputs per tile
constexpr int CR_IN = CR_D * CR_G;                       // inputs per tile
__host__ __device__ constexpr int cr_base(int c) { return (CR_D * c) / CR_U; }
constexpr int CR_SH = 2;                                 // the window starts 160 inputs early (16-B aligned)
constexpr int CR_LW = cr_base(CR_U - 1) + CR_CT + 1 + CR_SH;   // 236 window pairs per group (pairs 0-2 unused)
constexpr int CR_NP = CR_IN - CR_D + CR_LW;              // 5 276 window pairs per tile
// LDS float offset of window pair p: 4 pad floats after every group's 80 pairs (group stride
// 164 floats = 41 x 16 B, odd: conflict-free 16-B reads across the lanes)
__host__ __device__ constexpr int cr_addr(int p) { return 2 * p + 4 * (p / CR_D); }
constexpr int CR_LDS = cr_addr(CR_NP + 1) + 4;
__host__ __device__ constexpr int cr_c0(int w) { return 5 * w; }
__host__ __device__ constexpr int cr_c1(int w) { return 5 * w + 5 < CR_U ? 5 * w + 5 : CR_U; }
// window pair u of group L is input I0 - 160 + 80 L + u; phase c reads u in [base_c + 3, base_c + 160]
__host__ __device__ constexpr int cr_ulo(int w) { return (cr_base(cr_c0(w)) + 1 + CR_SH) & ~1; }
__host__ __device__ constexpr int cr_uhi(int w) { return cr_base(cr_c1(w) - 1) + CR_CT + CR_SH; }      // inclusive
__host__ __device__ constexpr int cr_npair(int w) { return (cr_uhi(w) - cr_ulo(w)) / 2 + 1; }
// the taps of wave w start at float cr_toff(w): [pair u2][phase c - c0][(tap at u2, at u2 + 1)]
__host__ __device__ constexpr int cr_toff(int w) {
  int o = 0;
  for (int i = 0; i < w; ++i) o += cr_npair(i) * (cr_c1(i) - cr_c0(i)) * 2;
  return o;
}
constexpr int CR_NTAPS = cr_toff(CR_NW);
static_assert(cr_c1(CR_NW - 1) == CR_U && cr_uhi(CR_NW - 1) < CR_LW, "phases and window");
static_assert((80 * CR_U) % CR_U == 0 && CR_D % 2 == 0, "16-B pair reads stay inside a group's block");

struct CresJob {
  const float* x;            // RDS extract rows (x_stride apart), M samples
  int64_t n, x_stride;
  NcoSrc nco;                // the RDS PLL's NCO: from its phases (theta != null) or rows
  const float* ctaps;        // composite taps (device, CR_NTAPS floats)
  const double* h64;         // LPF taps (f64, 151)
  const double* g64;         // anti-image taps (f64, 151)
  const double* zi_l[2];     // LPF I / Q lfilter state in (150 per stream, zs apart)
  const double* zi_a[2];     // anti-image I / Q state in
  double* zf_l[2];           // ... out
  double* zf_a[2];
  int64_t zs;
  float* y[2];               // resample I / Q rows (y_stride apart), R = ceil(19 M / 80) outputs
  float* yh[2];              // pinned host mirrors (yh_stride apart), nullable
  int64_t y_stride, yh_stride, R;
  int tiles, nstreams;
};

typedef const __attribute__((address_space(4))) f2a4* ctaps2c_t;

template <int W>
__device__ __forceinline__ void cres_fir(const float* win, const float* taps, f2 (&acc)[5]) {
  constexpr int c0 = cr_c0(W), nc = cr_c1(W) - c0, ulo = cr_ulo(W);
  const ctaps2c_t tw = (ctaps2c_t)(taps + cr_toff(W));
  static_for<0, cr_npair(W)>([&](auto I) {
    constexpr int u2 = ulo + 2 * I;
    const float4 v = *reinterpret_cast<const float4*>(win + 2 * u2 + 4 * (u2 / CR_D));
    static_for<0, nc>([&](auto C) {
      constexpr int c = c0 + C;
      constexpr bool v0 = u2 >= cr_base(c) + 1 + CR_SH && u2 <= cr_base(c) + CR_CT + CR_SH;
      constexpr bool v1 = u2 + 1 >= cr_base(c) + 1 + CR_SH && u2 + 1 <= cr_base(c) + CR_CT + CR_SH;
      if constexpr (v0 || v1) {
        const f2a4 hp = tw[I * nc + C];
        if constexpr (v0) pk_fma_sb<false>(acc[C], f2{hp.x, hp.y}, f2{v.x, v.y});
        if constexpr (v1) pk_fma_sb<true>(acc[C], f2{hp.x, hp.y}, f2{v.z, v.w});
      }
    });
  });
}

// final states of one stream: the LPF's (I, Q) from the last 150 mixed inputs and the
// anti-image filter's from the last 8 lpf values (f32, as the lpf rows hold them), each as
// rx.hip's zf_block computes it (on the x19 stream for the anti-image)
__device__ void cres_zf_block(const CresJob& J, int s, float* lds) {
  constexpr int T = CR_T, L8 = (CR_T - 1) / CR_U + 1;      // 8 lpf values
  constexpr int NM = T - 1 + L8;                             // 158 mixed inputs
  double* mx = reinterpret_cast<double*>(lds);               // mx[ch][i] = mixed_ch[n-1-i]
  double* hs = mx + 2 * NM;
  double* gs = hs + T;
  double* lp = gs + T;                                       // lp[ch][i] = lpf_ch[n-1-i]
  const int t = threadIdx.x;
  const int64_t n = J.n;
  const float* x = J.x + (int64_t)s * J.x_stride;
  for (int i = t; i < NM; i += CR_NT) {
    const int64_t xi = n - 1 - i;
    double vi = 0.0, vq = 0.0;
    if (xi >= 0) {
      float c, sn;
      if (J.nco.theta) nco_at(J.nco, s, xi, &c, &sn);
      else { c = J.nco.nco_i[(int64_t)s * J.nco.out_stride + xi]; sn = J.nco.nco_q[(int64_t)s * J.nco.out_stride + xi]; }
      vi = (double)((x[xi] * c) * 2.0f);                     // the mixer (fmRDSblock.py:173-176)
      vq = (double)((x[xi] * sn) * 2.0f);
    }
    mx[i] = vi;
    mx[NM + i] = vq;
  }
  for (int i = t; i < T; i += CR_NT) { hs[i] = J.h64[i]; gs[i] = J.g64[i]; }
  __syncthreads();
  // the LPF's final states, and the last 8 lpf values
  for (int w = t; w < 2 * (T - 1) + 2 * L8; w += CR_NT) {
    const int ch = w < 2 * (T - 1) ? w / (T - 1) : (w - 2 * (T - 1)) / L8;
    const double* m = mx + ch * NM;
    const double* zi = J.zi_l[ch] + (int64_t)s * J.zs;
    if (w < 2 * (T - 1)) {
      const int k = w - ch * (T - 1);
      const int jhi = (int)min<int64_t>(T - 1, n + k);
      double a0 = 0.0, a1 = 0.0;
      int j = k + 1;
      for (; j + 1 <= jhi; j += 2) {
        a0 = fma(hs[j], m[j - k - 1], a0);
        a1 = fma(hs[j + 1], m[j - k], a1);
      }
      if (j <= jhi) a0 = fma(hs[j], m[j - k - 1], a0);
      double acc = a0 + a1;
      if (n + k < T - 1) acc += zi[n + k];
      J.zf_l[ch][(int64_t)s * J.zs + k] = acc;
    } else {
      const int i = w - 2 * (T - 1) - ch * L8;                // lpf[n-1-i]
      const int64_t li = n - 1 - i;
      double acc = 0.0;
      if (li >= 0) {
        for (int k = 0; k < T && i + k < NM && li - k >= 0; ++k) acc = fma(hs[k], m[i + k], acc);
        if (li < T - 1) acc += zi[li];
      }
      lp[ch * L8 + i] = (double)(float)acc;
    }
  }
  __syncthreads();
  // the anti-image filter's final states: zf[k] = sum_{m >= 1, k + 19 m <= 150} g[k + 19 m] lpf[n - m]
  const int64_t nu = n * CR_U;
  for (int w = t; w < 2 * (T - 1); w += CR_NT) {
    const int ch = w / (T - 1), k = w - ch * (T - 1);
    double acc = 0.0;
    for (int m = 1; k + CR_U * m <= T - 1 && m <= n; ++m) acc = fma(gs[k + CR_U * m], lp[ch * L8 + m - 1], acc);
    if (nu + k < T - 1) acc += J.zi_a[ch][(int64_t)s * J.zs + nu + k];
    J.zf_a[ch][(int64_t)s * J.zs + k] = acc;
  }
}

__global__ __launch_bounds__(CR_NT) void rx_cres_kernel(CresJob J) {
  __shared__ __attribute__((aligned(16))) float lds[CR_LDS];
  const int b = blockIdx.x;
  const int t = threadIdx.x;
  if (b >= J.tiles * J.nstreams) {
    cres_zf_block(J, b - J.tiles * J.nstreams, lds);
    return;
  }
  const int s = b / J.tiles;
  const int64_t tile = b - (int64_t)s * J.tiles;
  const int64_t I0 = tile * CR_IN, ws = I0 - (CR_CT + CR_SH);   // window pair p <-> input ws + p
  const float* x = J.x + (int64_t)s * J.x_stride;
  const int64_t n = J.n;
  // stage the window: 4 inputs per chunk (16-B loads), mixed I and Q (the gain 2 is in the taps)
  constexpr int NCHK = (CR_NP + 3) / 4, NR = (NCHK + CR_NT - 1) / CR_NT;
  NcoTile nt{};
  if (J.nco.theta != nullptr) nt = nco_tile(J.nco, s, ws - 1);   // the pseudo-block records, once
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int j = t + r * CR_NT;
    if (j < NCHK) {
      const int64_t i = ws + 4 * j;
      float xv[4], c[4], sn[4];
      if (i >= 2 && i + 3 < n && J.nco.theta != nullptr) {
        const float4 x4 = *reinterpret_cast<const float4*>(x + i);
        xv[0] = x4.x; xv[1] = x4.y; xv[2] = x4.z; xv[3] = x4.w;
        nco_f32x4(J.nco, nt, i, c, sn);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {                           // block ends (and the carried NCO[0])
          const int64_t ie = i + e;
          xv[e] = c[e] = sn[e] = 0.f;
          if (ie < 0 || ie >= n) continue;
          xv[e] = x[ie];
          if (J.nco.theta) nco_at(J.nco, s, ie, &c[e], &sn[e]);
          else { c[e] = J.nco.nco_i[(int64_t)s * J.nco.out_stride + ie]; sn[e] = J.nco.nco_q[(int64_t)s * J.nco.out_stride + ie]; }
        }
      }
      float* dst = lds + cr_addr(4 * j);
      *reinterpret_cast<float4*>(dst) = make_float4(xv[0] * c[0], xv[0] * sn[0], xv[1] * c[1], xv[1] * sn[1]);
      *reinterpret_cast<float4*>(dst + 4) = make_float4(xv[2] * c[2], xv[2] * sn[2], xv[3] * c[3], xv[3] * sn[3]);
    }
  }
  __syncthreads();
  const int w = t >> 6, L = t & 63;
  const float* win = lds + (2 * CR_D + 4) * L;
  f2 acc[5];
#pragma unroll
  for (int c = 0; c < 5; ++c) acc[c] = f2{0.f, 0.f};
  if (w == 0) cres_fir<0>(win, J.ctaps, acc);
  else if (w == 1) cres_fir<1>(win, J.ctaps, acc);
  else if (w == 2) cres_fir<2>(win, J.ctaps, acc);
  else cres_fir<3>(win, J.ctaps, acc);
  const int c0 = cr_c0(w), nc = cr_c1(w) - c0;
  const int64_t m0 = tile * CR_TO + (int64_t)CR_U * L;
#pragma unroll
  for (int C = 0; C < 5; ++C) {
    if (C >= nc) break;
    const int c = c0 + C;
    const int64_t m = m0 + c;
    if (m >= J.R) continue;
    float yi = acc[C].x, yq = acc[C].y;
    const int64_t i0 = (CR_D * m) / CR_U;
    if (i0 < CR_CT - 1 || CR_D * m < CR_T - 1) {
      // block head: the LPF's zi (in lpf[i < 150]) and the anti-image zi (in a[q < 150])
      const int rho = (int)(CR_D * m - (int64_t)CR_U * i0);
      double ci = 0.0, cq = 0.0;
      for (int ss = 0; rho + CR_U * ss <= CR_T - 1; ++ss) {
        const int64_t li = i0 - ss;
        if (li >= 0 && li < CR_T - 1) {
          ci = fma(J.g64[rho + CR_U * ss], J.zi_l[0][(int64_t)s * J.zs + li], ci);
          cq = fma(J.g64[rho + CR_U * ss], J.zi_l[1][(int64_t)s * J.zs + li], cq);
        }
      }
      if (CR_D * m < CR_T - 1) {
        ci += J.zi_a[0][(int64_t)s * J.zs + CR_D * m];
        cq += J.zi_a[1][(int64_t)s * J.zs + CR_D * m];
      }
      yi += (float)(CR_U * ci);
      yq += (float)(CR_U * cq);
    }
    J.y[0][(int64_t)s * J.y_stride + m] = yi;
    J.y[1][(int64_t)s * J.y_stride + m] = yq;
    if (J.yh[0]) J.yh[0][(int64_t)s * J.yh_stride + m] = yi;
    if (J.yh[1]) J.yh[1][(int64_t)s * J.yh_stride + m] = yq;
  }
}

// ---- the composite RDS filter on the matrix cores (spans) --------------------------------
// Per window of 16 groups L (304 outputs m = m0 + 19 L + c): Y_ch[c][L] = sum_j A[c][j]
// X_ch[j][L], A[c][j] = the composite tap of phase c at window pair j + 1 (tap(c, j + 1) of
// cres_taps: 19 rows in two 16-row tiles), X_ch[j][L] = mixed_ch[I0 + 80 L - 159 + j], j < 256
// (8 K steps) -- the Hankel form of mma_run with columns 80 inputs apart (fragment reads at
// 160 L + 64 s + 16 g bytes: conflict-free); the I and Q channels share A.  A's fragments
// (the 13 K steps that hold taps) are built once per workgroup into LDS and read per step.
// The mixed inputs are formed where they are staged, from the RDS PLL's phases (sdr_nco.h),
// four inputs i .. i+3 per lane and chunk with i odd (the window starts at an odd input) so
// that their four phases are two aligned 16-B loads; every chunk's loads go out three chunks
// ahead of its arithmetic.  Waves work alone and persist; one wave's staging (VALU: the NCO)
// runs beside another's MFMAs.  Workgroups [0, S) write the streams' final states.
constexpr int CM_RT = 2, CM_KS = 8, CM_KOFF = CR_CT + CR_SH - 1;   // 159: odd window starts
constexpr int CM_LU = CR_D * 15 + 32 * CM_KS;       // 1 456 inputs staged per window
constexpr int CM_NG = CM_LU / 4, CM_NQ = (CM_NG + 63) / 64;
constexpr int CM_WO = 16 * CR_U;                   // 304 outputs per window
constexpr int CM_WI = 16 * CR_D;                   // 1 280 inputs per window
constexpr int CM_AROWS = 16 * CM_RT, CM_ACOLS = 32 * CM_KS;
constexpr int CM_WGS = 2 * 256;                    // persistent workgroups (2 per CU: LDS)
static_assert(CM_KOFF % 2 == 1 && CM_WI % 4 == 0, "odd window starts: chunk phases are aligned pairs");
static_assert(cr_base(CR_U - 1) + CR_CT + CR_SH - 1 < CM_ACOLS && CR_U <= CM_AROWS, "every composite tap inside A");
// the K steps holding row tile rt's taps: phase c's at j in [base_c + SH, base_c + CT + SH - 1]
__host__ __device__ constexpr int cm_st0(int rt) { return (cr_base(16 * rt) + CR_SH) / 32; }
__host__ __device__ constexpr int cm_st1(int rt) {
  return (cr_base(rt == 0 ? 15 : CR_U - 1) + CR_CT + CR_SH - 1) / 32 + 1;
}
__host__ __device__ constexpr int cm_fi(int rt, int st) { return (rt == 0 ? 0 : cm_st1(0) - cm_st0(0)) + st - cm_st0(rt); }
constexpr int CM_NF = cm_st1(0) - cm_st0(0) + cm_st1(1) - cm_st0(1);
static_assert(cm_st1(1) <= CM_KS && CM_NF == 13, "row tiles' K steps");

template <bool TH32 = false>   // TH32: the RDS loop's phase rows are compact (sdr_nco.h, PllJob::th32)
__global__ __launch_bounds__(RX_NT) __attribute__((amdgpu_waves_per_eu(2))) void rx_cresmm_kernel(CresJob J,
                                                                                               const float* amat, int wgs) {
  __shared__ __attribute__((aligned(16))) _Float16 img[4][4 * CM_LU];   // per wave: I hi, I lo, Q hi, Q lo
  __shared__ __attribute__((aligned(16))) h8v afr[2][CM_NF][64];         // A fragments: hi, lo
  const int S = J.nstreams;
  if ((int)blockIdx.x < S) {
    cres_zf_block(J, blockIdx.x, reinterpret_cast<float*>(&img[0][0]));
    return;
  }
  for (int idx = threadIdx.x; idx < CM_NF * 64; idx += RX_NT) {
    const int fi = idx >> 6, ln = idx & 63;
    const int rt = fi < cm_st1(0) - cm_st0(0) ? 0 : 1;
    const int st = fi - (rt ? cm_st1(0) - cm_st0(0) : 0) + cm_st0(rt);
    const float* ar = amat + (16 * rt + (ln & 15)) * CM_ACOLS + 32 * st + 8 * (ln >> 4);
    h8v hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const MmHL p = mm_split(ar[e]);
      hi[e] = p.hi;
      lo[e] = p.lo;
    }
    afr[0][fi][ln] = hi;
    afr[1][fi][ln] = lo;
  }
  __syncthreads();
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // uniform: see rx_mma_kernel
  const int l = threadIdx.x & 63, b = l & 15, g = l >> 4;
  const int64_t gw = ((int64_t)blockIdx.x - S) * 4 + w, nw = (int64_t)wgs * 4;
  _Float16* Ih = img[w];
  _Float16* Il = Ih + CM_LU;
  _Float16* Qh = Il + CM_LU;
  _Float16* Ql = Qh + CM_LU;
  const int64_t n = J.n, R = J.R;
  const int64_t wins = (R + CM_WO - 1) / CM_WO;     // per stream
  const int64_t total = wins * S;
  // A window's geometry and pseudo-block records (the RDS loop's blocks carry a linear
  // response: its pre-roll stops short of LONG_ACCEPT, pll.hip warm_len); one branch-free path
  // for every window, the chunks' loads PD chunks ahead through the seams (rx_decmm_kernel)
  static_assert((CM_WI - CM_KOFF) % 4 == 1 && CM_KOFF % 4 == 3, "chunks start at 1 mod 4 (mix_load)");
  struct Win { int s; int64_t W, m0, a; const float* x; NcoTile nt; };
  auto winfo = [&](int64_t i, Win* v) {
    v->s = (int)(i / wins);
    v->W = i - (int64_t)v->s * wins;
    v->m0 = CM_WO * v->W;
    v->a = CM_WI * v->W - CM_KOFF;                   // input of element 0
    v->x = J.x + (int64_t)v->s * J.x_stride;
    v->nt = nco_tile(J.nco, v->s, max<int64_t>(v->a, 1) - 1);
  };
  constexpr int PD = 2;
  static_assert(CM_NQ % PD == 0, "ring slots line up across windows");
  MixLd gb[PD];
  auto ldg = [&](const Win& v, int j, MixLd* gg) {
    mix_load<TH32>(J.nco, v.nt, v.x, v.a + 4 * min(l + 64 * j, CM_NG - 1), true, gg);
  };
  Win cur{}, nxt{};
  if (gw < total) {
    winfo(gw, &cur);
    static_for<0, PD>([&](auto D) { ldg(cur, D, &gb[D]); });
  }
  for (int64_t i = gw; i < total; i += nw) {
    const bool more = i + nw < total;
    if (more) winfo(i + nw, &nxt);
    const int s = cur.s;
    const int64_t W = cur.W, m0 = cur.m0, a = cur.a;
    {
      const NcoWin nwin = nco_win(J.nco, cur.nt, a);
      const bool lin = nco_tile_lin(cur.nt);
      const float c0 = J.nco.nco_i[(int64_t)s * J.nco.out_stride], s0 = J.nco.nco_q[(int64_t)s * J.nco.out_stride];
      static_for<0, CM_NQ>([&](auto JJ) {
        constexpr int j = JJ;
        const int q = min(l + 64 * j, CM_NG - 1);
        const MixLd gc = gb[j % PD];
        if constexpr (j + PD < CM_NQ) ldg(cur, j + PD, &gb[j % PD]);
        else ldg(more ? nxt : cur, j + PD - CM_NQ, &gb[j % PD]);
        float xv[4], c[4], sn[4];
        mix_eval<TH32>(cur.nt, nwin, a + 4 * q, n, gc, lin, c0, s0, xv, c, sn);
        h4v hv, lv;
        mm_split4(make_float4(xv[0] * c[0], xv[1] * c[1], xv[2] * c[2], xv[3] * c[3]), &hv, &lv);
        *reinterpret_cast<h4v*>(Ih + 4 * q) = hv;
        *reinterpret_cast<h4v*>(Il + 4 * q) = lv;
        mm_split4(make_float4(xv[0] * sn[0], xv[1] * sn[1], xv[2] * sn[2], xv[3] * sn[3]), &hv, &lv);
        *reinterpret_cast<h4v*>(Qh + 4 * q) = hv;
        *reinterpret_cast<h4v*>(Ql + 4 * q) = lv;
        __builtin_amdgcn_sched_barrier(0);
      });
    }
    // the K steps, fragments of step st + 1 read while step st's MFMAs run
    f4v aIh[CM_RT], aIc[CM_RT], aQh[CM_RT], aQc[CM_RT];
#pragma unroll
    for (int rt = 0; rt < CM_RT; ++rt) aIh[rt] = aIc[rt] = aQh[rt] = aQc[rt] = f4v{0.f, 0.f, 0.f, 0.f};
    struct Fr { h8v x[4], a[CM_RT][2]; };
    Fr fr[2];
    auto frag = [&](auto ST, Fr* d) {
      constexpr int st = ST;
      const int u = CR_D * b + 32 * st + 8 * g;
      d->x[0] = *reinterpret_cast<const h8v*>(Ih + u);
      d->x[1] = *reinterpret_cast<const h8v*>(Il + u);
      d->x[2] = *reinterpret_cast<const h8v*>(Qh + u);
      d->x[3] = *reinterpret_cast<const h8v*>(Ql + u);
      static_for<0, CM_RT>([&](auto RT) {
        constexpr int rt = RT;
        if constexpr (st >= cm_st0(rt) && st < cm_st1(rt)) {
          d->a[rt][0] = afr[0][cm_fi(rt, st)][l];
          d->a[rt][1] = afr[1][cm_fi(rt, st)][l];
        }
      });
    };
    frag(std::integral_constant<int, 0>{}, &fr[0]);
    static_for<0, CM_KS>([&](auto ST) {
      constexpr int st = ST;
      if constexpr (st + 1 < CM_KS) frag(std::integral_constant<int, st + 1>{}, &fr[(st + 1) % 2]);
      const Fr& f = fr[st % 2];
      static_for<0, CM_RT>([&](auto RT) {
        constexpr int rt = RT;
        if constexpr (st >= cm_st0(rt) && st < cm_st1(rt)) {
          const h8v ah = f.a[rt][0], al = f.a[rt][1];
          aIh[rt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, f.x[0], aIh[rt], 0, 0, 0);
          aIc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, f.x[1], aIc[rt], 0, 0, 0);
          aIc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, f.x[0], aIc[rt], 0, 0, 0);
          aQh[rt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, f.x[2], aQh[rt], 0, 0, 0);
          aQc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, f.x[3], aQc[rt], 0, 0, 0);
          aQc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, f.x[2], aQc[rt], 0, 0, 0);
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
    // outputs: lane (b, g) holds phases c = 16 rt + 4 g + r of group L = b
    const bool head = W == 0;                        // the stream's first window: the zi terms
#pragma unroll
    for (int rt = 0; rt < CM_RT; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * rt + 4 * g + r;
        const int64_t m = m0 + CR_U * b + c;
        if (c >= CR_U || m >= R) continue;
        float yi = fmaf(aIc[rt][r], 1.f / MM_LO, aIh[rt][r]), yq = fmaf(aQc[rt][r], 1.f / MM_LO, aQh[rt][r]);
        const int64_t i0 = (CR_D * m) / CR_U;
        if (head && (i0 < CR_CT - 1 || CR_D * m < CR_T - 1)) {
          // block head: the LPF's zi (in lpf[i < 150]) and the anti-image zi (in a[q < 150])
          const int rho = (int)(CR_D * m - (int64_t)CR_U * i0);
          double ci = 0.0, cq = 0.0;
          for (int ss = 0; rho + CR_U * ss <= CR_T - 1; ++ss) {
            const int64_t li = i0 - ss;
            if (li >= 0 && li < CR_T - 1) {
              ci = fma(J.g64[rho + CR_U * ss], J.zi_l[0][(int64_t)s * J.zs + li], ci);
              cq = fma(J.g64[rho + CR_U * ss], J.zi_l[1][(int64_t)s * J.zs + li], cq);
            }
          }
          if (CR_D * m < CR_T - 1) {
            ci += J.zi_a[0][(int64_t)s * J.zs + CR_D * m];
            cq += J.zi_a[1][(int64_t)s * J.zs + CR_D * m];
          }
          yi += (float)(CR_U * ci);
          yq += (float)(CR_U * cq);
        }
        J.y[0][(int64_t)s * J.y_stride + m] = yi;
        J.y[1][(int64_t)s * J.y_stride + m] = yq;
        if (J.yh[0]) J.yh[0][(int64_t)s * J.yh_stride + m] = yi;
        if (J.yh[1]) J.yh[1][(int64_t)s * J.yh_stride + m] = yq;
      }
    cur = nxt;
  }
}

// the composite taps (host, f64 then f32) in the kernel's order; empty unless both filters
// have CR_T taps
void cres_taps(const std::vector<double>& h, const std::vector<double>& g, std::vector<float>* out) {
  out->clear();
  if ((int)h.size() != CR_T || (int)g.size() != CR_T) return;
  std::vector<double> C((size_t)CR_U * CR_CT, 0.0);            // C[rho][t]
  for (int rho = 0; rho < CR_U; ++rho)
    for (int ss = 0; rho + CR_U * ss < CR_T; ++ss)
      for (int k = 0; k < CR_T; ++k) C[(size_t)rho * CR_CT + ss + k] += g[rho + CR_U * ss] * h[k];
  out->assign(CR_NTAPS, 0.f);
  auto tap = [&](int c, int u) -> float {
    const int tt = cr_base(c) + CR_CT + CR_SH - u;
    if (tt < 0 || tt >= CR_CT) return 0.f;
    const int rho = CR_D * c - CR_U * cr_base(c);
    return (float)(2.0 * CR_U * C[(size_t)rho * CR_CT + tt]);
  };
  for (int w = 0; w < CR_NW; ++w) {
    const int c0 = cr_c0(w), nc = cr_c1(w) - c0;
    for (int I = 0; I < cr_npair(w); ++I) {
      const int u2 = cr_ulo(w) + 2 * I;
      for (int C2 = 0; C2 < nc; ++C2) {
        const int o = cr_toff(w) + (I * nc + C2) * 2;
        (*out)[o] = tap(c0 + C2, u2);
        (*out)[o + 1] = tap(c0 + C2, u2 + 1);
      }
    }
  }
  // then the dense A of rx_cresmm_kernel: A[c][j] = tap(c, j + 1), rows 19 .. 31 zero
  out->resize(CR_NTAPS + CM_AROWS * CM_ACOLS, 0.f);
  for (int c = 0; c < CR_U; ++c)
    for (int j = 0; j < CM_ACOLS; ++j) (*out)[CR_NTAPS + c * CM_ACOLS + j] = tap(c, j + 1);
}

// state-bank slots (f64 lfilter states, T-1 per stream each)
enum Zs {
  Z_FE_I, Z_FE_Q, Z_AUDIO, Z_PILOT, Z_BAND, Z_EXTRACT, Z_SQUARE, Z_SLPF, Z_RLPF_I, Z_RLPF_Q,
  Z_ANTI_I, Z_ANTI_Q, Z_RRC_I, Z_RRC_Q, Z_N
};

int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

}  // namespace

struct sdr_rx {
  sdr_ctx* c = nullptr;
  int S = 0;
  int64_t B = 0;
  int u8 = 0, flags = 0;
  int rf_decim = 10, audio_decim = 5, rds_up = 19, rds_down = 80;
  std::vector<double> taps[SDR_RX_NFILTERS];
  PllCfg pll[2] = {};
  bool ready = false;
  int64_t M = 0, A = 0, R = 0;
  float* out[SDR_RX_NOUTPUTS] = {};    // the rows of the latest block (one of outs[])
  float* outs[3][SDR_RX_NOUTPUTS] = {}; // row sets: nq when pipelined, else one
  int64_t out_n[SDR_RX_NOUTPUTS] = {}, out_stride[SDR_RX_NOUTPUTS] = {};
  void* mem = nullptr;                 // one allocation for outputs, states and phases
  double* bank[2] = {};
  int64_t zoff[Z_N] = {}, zlen[Z_N] = {};
  int64_t bank_len = 0;
  double* phase = nullptr;             // demod prev_phase per stream
  int* wraps = nullptr;                // FE kernel scratch: per-block wrap count, last phase
  float* last_phi = nullptr;
  double* pll_state[2] = {};           // 6 per stream (stereo, RDS)
  double* theta = nullptr;             // PLL phases: 2 x S rows of ths per row set
  int64_t ths = 0;
  double* pllc = nullptr;              // PLL per-sample constants: 2 x S rows of cst per row set
  int64_t cst = 0;
  int8_t* pcode = nullptr;             // spans: the PLLs' inputs as sign codes (sdr_nco.h pll_code): 2 x S rows
  int64_t pcs = 0;                     //   of pcs bytes per row set
  char* pllw = nullptr;                // long blocks (M > SDR_PLL_BLOCK_MAX): the PLL's pseudo-block
  int64_t pllw_bytes = 0;              //   records, one region per row set
  void* pin_in = nullptr;              // pinned host staging (sdr_rx_run)
  size_t pin_in_cap = 0;
  float* pin_out = nullptr;
  size_t pin_out_cap = 0;
  float* mirror[SDR_RX_NOUTPUTS] = {};  // sdr_rx_run: pinned host rows (out_n apart) the producing
                                        // stage stores each requested output into, or null
  int parity = 0;
  int64_t blocks = 0;
  // sdr_rx_set_pipeline: block k's front half (FE, stage A) runs on `front` while block
  // k-1's back half (B, PLLs, C, D, E) runs on the context stream; row set k % nq
  int pipe = 0;
  hipStream_t last_fs = nullptr;        // the stream block k-1's front half ran on
  int64_t host_done = -1;               // the latest block the host has waited for (deliver)
  int nq = 2;                           // row sets when pipelined (3 with sdr_rx_set_depth >= 2)
  hipStream_t front = nullptr;          // FE, stages A and B
  hipStream_t mid = nullptr;            // the PLLs (prep, lanes, NCO)
  hipEvent_t ev_front[3] = {}, ev_mid[3] = {}, ev_back[3] = {}, ev_done[4] = {};
  // sdr_rx_submit: depth blocks in flight before a submit waits (sdr_rx_set_depth); pinned
  // slots (input and outputs) per block, depth + 1 of them; the blocks in flight, oldest first
  int depth = 1;
  size_t in_slot = 0, out_slot = 0;
  int64_t subs = 0;
  struct Pending {
    int slot = 0, nout = 0;
    hipEvent_t ev = nullptr;           // the block's completion (ev_done[slot], or its row set's ev_back)
    int64_t blk = 0;                   // its index (sdr_rx::blocks numbering)
    int which[SDR_RX_MAXOUT] = {};
    float* out[SDR_RX_MAXOUT] = {};
    int64_t os[SDR_RX_MAXOUT] = {};
    size_t region[SDR_RX_NOUTPUTS] = {};
  } pq[4];                             // depth + 1 at most (the new block before k-depth leaves)
  int pq_head = 0, pq_n = 0;
  bool timing = false;                 // events between the stages of each block
  hipEvent_t ev[SDR_RX_NSTAGES + 1] = {};
  // outputs process_dev materialises (sdr_rx_set_keep; bit o = SDR_RX_O_o): the NCO rows and
  // the RDS LPF rows are intermediates the chain does not need (the mixers form the NCO from
  // the PLL phases, the RDS LPF runs inside the composite resampler)
  uint64_t keep = ~0ull;
  uint64_t keep_now = ~0ull;           // this call's (sdr_rx_submit: what it was asked for)
  bool made[SDR_RX_NOUTPUTS] = {};     // what the latest block materialised
  float* ctaps = nullptr;              // the composite RDS taps (rx_cres_kernel), device; null: two-stage path
};

namespace {

PllCfg pll_cfg(double freq, double fs, double scale, double adj, double bw) {
  return PllCfg{freq, fs, scale, adj, bw * 2.666, bw * bw * 3.555};   // model/fmPll.py:7-10
}

bool need_out(const sdr_rx* r, int o) {
  const bool au = r->flags & (SDR_RX_AUDIO | SDR_RX_STEREO), st = r->flags & SDR_RX_STEREO,
             rd = r->flags & SDR_RX_RDS;
  switch (o) {
    case SDR_RX_O_DEMOD: return true;
    case SDR_RX_O_AUDIO: return au;
    case SDR_RX_O_BPF_RECOVERY: case SDR_RX_O_STEREO_NCO: case SDR_RX_O_BPF_EXTRACTION:
    case SDR_RX_O_STEREO: case SDR_RX_O_LEFT: case SDR_RX_O_RIGHT: return st;
    default: return rd;
  }
}

int filter_of_zs(int z) {
  switch (z) {
    case Z_FE_I: case Z_FE_Q: return SDR_RX_F_RF;
    case Z_AUDIO: return SDR_RX_F_AUDIO;
    case Z_PILOT: return SDR_RX_F_PILOT;
    case Z_BAND: return SDR_RX_F_STEREO_BPF;
    case Z_EXTRACT: return SDR_RX_F_RDS_EXTRACT;
    case Z_SQUARE: return SDR_RX_F_RDS_SQUARE;
    case Z_SLPF: return SDR_RX_F_STEREO_LPF;
    case Z_RLPF_I: case Z_RLPF_Q: return SDR_RX_F_RDS_LPF;
    case Z_ANTI_I: case Z_ANTI_Q: return SDR_RX_F_RDS_ANTI;
    default: return SDR_RX_F_RDS_RRC;
  }
}

bool filter_used(const sdr_rx* r, int f) {
  const bool au = r->flags & (SDR_RX_AUDIO | SDR_RX_STEREO), st = r->flags & SDR_RX_STEREO,
             rd = r->flags & SDR_RX_RDS;
  switch (f) {
    case SDR_RX_F_RF: return true;
    case SDR_RX_F_AUDIO: return au;
    case SDR_RX_F_PILOT: case SDR_RX_F_STEREO_BPF: case SDR_RX_F_STEREO_LPF: return st;
    default: return rd;
  }
}

const char* kFilterName[SDR_RX_NFILTERS] = {"rf", "audio", "pilot", "stereo_bpf", "stereo_lpf",
                                            "rds_extract", "rds_square", "rds_lpf", "rds_anti", "rds_rrc"};

// Allocate and zero everything once the configuration is known (first block).
int rx_finalize(sdr_rx* r) {
  for (int f = 0; f < SDR_RX_NFILTERS; ++f)
    if (filter_used(r, f) && r->taps[f].empty())
      return fail(SDR_EINVAL, "sdr_rx: the %s filter taps are not set", kFilterName[f]);
  const int64_t M = ceil_div(r->B, r->rf_decim);
  r->M = M;
  r->A = ceil_div(M, r->audio_decim);
  r->R = ceil_div(M * r->rds_up, r->rds_down);
  const int64_t ms = round_up(M + 1, 64), as = round_up(r->A, 64), rs = round_up(r->R, 64);
  const int64_t S = r->S;
  int64_t floats = 0;
  for (int o = 0; o < SDR_RX_NOUTPUTS; ++o) {
    if (!need_out(r, o)) continue;
    int64_t n, st;
    switch (o) {
      case SDR_RX_O_AUDIO: case SDR_RX_O_STEREO: case SDR_RX_O_LEFT: case SDR_RX_O_RIGHT:
        n = r->A; st = as; break;
      case SDR_RX_O_STEREO_NCO: case SDR_RX_O_RDS_NCO_I: case SDR_RX_O_RDS_NCO_Q:
        n = M + 1; st = ms; break;
      case SDR_RX_O_RDS_RES_I: case SDR_RX_O_RDS_RES_Q: case SDR_RX_O_RDS_RRC_I: case SDR_RX_O_RDS_RRC_Q:
        n = r->R; st = rs; break;
      default: n = M; st = ms; break;
    }
    r->out_n[o] = n;
    r->out_stride[o] = st;
  }
  for (int q = 0; q < (r->pipe ? r->nq : 1); ++q)
    for (int o = 0; o < SDR_RX_NOUTPUTS; ++o) {
      if (!need_out(r, o)) continue;
      r->outs[q][o] = reinterpret_cast<float*>((intptr_t)floats);   // offset for now
      floats += r->out_stride[o] * S + 64;
    }
  int64_t zl = 0;
  for (int z = 0; z < Z_N; ++z) {
    const int f = filter_of_zs(z);
    if (!filter_used(r, f)) continue;
    r->zoff[z] = zl;
    r->zlen[z] = std::max<int64_t>((int64_t)r->taps[f].size() - 1, 1);
    zl += round_up(r->zlen[z] * S, 2);
  }
  r->bank_len = zl;
  r->ths = round_up(M, 2) + 2;
  r->cst = round_up(M + M / 32, 2) + 2;
  const int64_t S2 = round_up(S, 2);                 // keeps the phase rows 16-B aligned
  const int nsets = r->pipe ? r->nq : 1;
  const int64_t doubles = 2 * zl + 3 * S2 + 2 * 6 * S2 + nsets * (2 * S * r->ths + 2 * S * r->cst);
  r->pllw_bytes = round_up(sdr_pll_work_bytes(2, r->S, M), 256);
  r->pcs = round_up(M + 16, 256);
  const size_t code_bytes = (r->flags & (SDR_RX_STEREO | SDR_RX_RDS)) ? (size_t)(nsets * 2 * S * r->pcs) : 0;
  const size_t bytes = (size_t)floats * 4 + 64 + (size_t)doubles * 8 + 256 + (size_t)(nsets * r->pllw_bytes) + code_bytes;
  TRY(set_dev(r->c));
  hipError_t e = hipMalloc(&r->mem, bytes);
  if (e != hipSuccess) return fail(SDR_ENOMEM, "sdr_rx: hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  char* base = static_cast<char*>(r->mem);
  for (int q = 0; q < (r->pipe ? r->nq : 1); ++q)
    for (int o = 0; o < SDR_RX_NOUTPUTS; ++o)
      if (need_out(r, o)) r->outs[q][o] = reinterpret_cast<float*>(base) + (intptr_t)r->outs[q][o];
  std::memcpy(r->out, r->outs[0], sizeof r->out);
  double* d = reinterpret_cast<double*>(base + round_up(floats * 4, 64));
  r->bank[0] = d;
  r->bank[1] = d + zl;
  r->phase = d + 2 * zl;
  r->wraps = reinterpret_cast<int*>(r->phase + S2);
  r->last_phi = reinterpret_cast<float*>(r->phase + 2 * S2);
  r->pll_state[0] = r->phase + 3 * S2;
  r->pll_state[1] = r->pll_state[0] + 6 * S2;
  r->theta = r->pll_state[1] + 6 * S2;
  r->pllc = r->theta + nsets * 2 * S * r->ths;
  r->pllw = reinterpret_cast<char*>(round_up((int64_t)(uintptr_t)(r->pllc + nsets * 2 * S * r->cst), 256));
  r->pcode = code_bytes ? reinterpret_cast<int8_t*>(r->pllw + nsets * r->pllw_bytes) : nullptr;
  if ((r->flags & SDR_RX_RDS) && r->rds_up == CR_U && r->rds_down == CR_D) {
    std::vector<float> ct;
    cres_taps(r->taps[SDR_RX_F_RDS_LPF], r->taps[SDR_RX_F_RDS_ANTI], &ct);
    if (!ct.empty()) {
      HIP_TRY(hipMalloc(&r->ctaps, sizeof(float) * ct.size()));
      HIP_TRY(hipMemcpy(r->ctaps, ct.data(), sizeof(float) * ct.size(), hipMemcpyHostToDevice));
    }
  }
  r->ready = true;
  return sdr_rx_reset(r);
}

}  // namespace

extern "C" {

int sdr_rx_create(sdr_ctx* c, int nstreams, int64_t block, int iq_dtype, int flags, sdr_rx** out) {
  CHECK_CTX(c);
  if (out == nullptr) return fail(SDR_EINVAL, "sdr_rx_create: out is NULL");
  *out = nullptr;
  if (nstreams < 1 || block < 1) return fail(SDR_EINVAL, "sdr_rx_create: nstreams %d, block %lld", nstreams, (long long)block);
  if (iq_dtype != SDR_IQ_F32 && iq_dtype != SDR_IQ_U8) return fail(SDR_EINVAL, "sdr_rx_create: iq_dtype %d", iq_dtype);
  if (flags & ~(SDR_RX_AUDIO | SDR_RX_STEREO | SDR_RX_RDS)) return fail(SDR_EINVAL, "sdr_rx_create: flags 0x%x", flags);
  sdr_rx* r = new (std::nothrow) sdr_rx();
  if (!r) return fail(SDR_ENOMEM, "sdr_rx_create: out of memory");
  r->c = c;
  r->S = nstreams;
  r->B = block;
  r->u8 = iq_dtype == SDR_IQ_U8;
  r->flags = flags;
  // model/fmMonoBlock.py:119 (19 kHz, x2, BW 0.01); model/fmRDSblock.py:167 (114 kHz, x0.5)
  r->pll[0] = pll_cfg(19e3, 240e3, 2.0, 0.0, 0.01);
  r->pll[1] = pll_cfg(114e3, 240e3, 0.5, M_PI / 3.3 - M_PI / 1.5, 0.001);
  *out = r;
  return SDR_OK;
}

void sdr_rx_destroy(sdr_rx* r) {
  if (r == nullptr) return;
  if (r->c) {
    (void)hipSetDevice(r->c->device);
    if (r->front) (void)hipStreamSynchronize(r->front);
    if (r->mid) (void)hipStreamSynchronize(r->mid);
    (void)hipStreamSynchronize(r->c->stream);
  }
  if (r->mem) (void)hipFree(r->mem);
  if (r->ctaps) (void)hipFree(r->ctaps);
  if (r->pin_in) (void)hipHostFree(r->pin_in);
  if (r->pin_out) (void)hipHostFree(r->pin_out);
  for (hipEvent_t e : r->ev)
    if (e) (void)hipEventDestroy(e);
  for (int q = 0; q < 3; ++q)
    for (hipEvent_t e : {r->ev_front[q], r->ev_mid[q], r->ev_back[q]})
      if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : r->ev_done)
    if (e) (void)hipEventDestroy(e);
  if (r->front) (void)hipStreamDestroy(r->front);
  if (r->mid) (void)hipStreamDestroy(r->mid);
  delete r;
}

int sdr_rx_set_filter(sdr_rx* r, int which, const double* b, int taps) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (r->ready) return fail(SDR_EINVAL, "sdr_rx_set_filter: the receiver has processed a block");
  if (which < 0 || which >= SDR_RX_NFILTERS) return fail(SDR_EINVAL, "sdr_rx_set_filter: filter %d", which);
  if (b == nullptr || taps < 1 || taps > SDR_MAX_TAPS)
    return fail(SDR_EINVAL, "sdr_rx_set_filter: taps=%d outside [1, %d]", taps, SDR_MAX_TAPS);
  r->taps[which].assign(b, b + taps);
  return SDR_OK;
}

int sdr_rx_set_decim(sdr_rx* r, int rf_decim, int audio_decim, int rds_up, int rds_down) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (r->ready) return fail(SDR_EINVAL, "sdr_rx_set_decim: the receiver has processed a block");
  if (rf_decim < 1 || audio_decim < 1 || rds_up < 1 || rds_down < 1) return fail(SDR_EINVAL, "sdr_rx_set_decim: factor < 1");
  r->rf_decim = rf_decim;
  r->audio_decim = audio_decim;
  r->rds_up = rds_up;
  r->rds_down = rds_down;
  return SDR_OK;
}

int sdr_rx_set_pll(sdr_rx* r, int which, double freq, double fs, double nco_scale, double phase_adj,
                   double norm_bw) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (which != 0 && which != 1) return fail(SDR_EINVAL, "sdr_rx_set_pll: which=%d (0 stereo, 1 RDS)", which);
  if (!(fs != 0.0)) return fail(SDR_EINVAL, "sdr_rx_set_pll: Fs must be non-zero");
  r->pll[which] = pll_cfg(freq, fs, nco_scale, phase_adj, norm_bw);
  return SDR_OK;
}

int sdr_rx_reset(sdr_rx* r) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (!r->ready) return SDR_OK;   // nothing allocated yet: the first block starts from zero
  TRY(set_dev(r->c));
  hipStream_t st = r->c->stream;
  if (r->front) HIP_TRY(hipStreamSynchronize(r->front));
  if (r->mid) HIP_TRY(hipStreamSynchronize(r->mid));
  r->pq_n = 0;                                   // submitted blocks' outputs are dropped
  // state banks, phases and wrap counters (contiguous)
  HIP_TRY(hipMemsetAsync(r->bank[0], 0, sizeof(double) * (size_t)(2 * r->bank_len + 2 * round_up(r->S, 2)), st));
  std::vector<double> ps(6 * (size_t)r->S);
  for (int s = 0; s < r->S; ++s) {               // model/fmMonoBlock.py:76, model/fmRDSblock.py:96
    const double init[6] = {0.0, 0.0, 1.0, 0.0, 1.0, 0.0};
    std::memcpy(&ps[6 * (size_t)s], init, sizeof init);
  }
  HIP_TRY(hipMemcpyAsync(r->pll_state[0], ps.data(), sizeof(double) * ps.size(), hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(r->pll_state[1], ps.data(), sizeof(double) * ps.size(), hipMemcpyHostToDevice, st));
  HIP_TRY(hipStreamSynchronize(st));
  r->parity = 0;
  r->blocks = 0;
  r->last_fs = nullptr;
  r->host_done = -1;
  std::memcpy(r->out, r->outs[0], sizeof r->out);
  return SDR_OK;
}

int sdr_rx_set_pipeline(sdr_rx* r, int on) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (r->ready) return fail(SDR_EINVAL, "sdr_rx_set_pipeline: the receiver has processed a block");
  if (on && !r->front) {
    TRY(set_dev(r->c));
    // (default priorities: an A/B of a high-priority PLL stream, a high-priority front stream and
    // low-priority front + PLL streams on one box measured C5 339-349 k against 352-355 k MS/s
    // for equal priorities, profiles/r06/e/prio_ab.txt)
    HIP_TRY(hipStreamCreateWithFlags(&r->front, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&r->mid, hipStreamNonBlocking));
    for (int q = 0; q < 3; ++q) {
      HIP_TRY(hipEventCreateWithFlags(&r->ev_front[q], hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&r->ev_mid[q], hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&r->ev_back[q], hipEventDisableTiming));
    }
  }
  r->pipe = on != 0;
  return SDR_OK;
}

int sdr_rx_process_dev(sdr_rx* r, const void* iq, int64_t iq_stride) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (iq == nullptr) return fail(SDR_EINVAL, "sdr_rx_process_dev: iq is NULL");
  if (r->S > 1 && iq_stride < r->B) return fail(SDR_EINVAL, "sdr_rx_process_dev: iq_stride %lld < block", (long long)iq_stride);
  if (!r->ready) TRY(rx_finalize(r));
  sdr_ctx* c = r->c;
  TRY(set_dev(c));
  hipStream_t st = c->stream;             // the back half (everything when not pipelined)
  const int S = r->S;
  const int64_t M = r->M;
  double* zi = r->bank[r->parity];
  double* zf = r->bank[r->parity ^ 1];
  const int q = r->pipe ? (int)(r->blocks % r->nq) : 0;
  // FE: RF FIR + decimate + demod (fe.hip).  The tiled kernels take the reference's RF
  // configurations; their carried state (I/Q zf, demod phase) is finished by workgroups of
  // the stage-A launch.  Other configurations run sdr_rf_frontend_dev's generic path (on the
  // context stream, so a pipelined receiver's front half runs there for such blocks).
  const int Trf = (int)r->taps[SDR_RX_F_RF].size();
  const int64_t xs = S > 1 ? iq_stride : r->B;
  const int G = r->u8 ? 8 : 2;
  const bool fast = (Trf == 101 || Trf == 151) && r->rf_decim == 10 && (S <= 1 || r->u8 || xs % G == 0) &&
                    ((uintptr_t)iq % (r->u8 ? 4 : 16)) == 0;
  hipStream_t fs = (r->pipe && fast) ? r->front : st;
  if (r->pipe) {
    // states of block k-1 (r04b: not when its front half ran on this same stream, in order)
    if (r->blocks >= 1 && r->last_fs != fs) HIP_TRY(hipStreamWaitEvent(fs, r->ev_front[(q + r->nq - 1) % r->nq], 0));
    r->last_fs = fs;
    // set q read by k-nq (not when the host has already waited for that block: submissions)
    if (r->blocks >= r->nq && r->blocks - r->nq > r->host_done) HIP_TRY(hipStreamWaitEvent(fs, r->ev_back[q], 0));
  }
  auto mark = [&](int k, hipStream_t s) { return r->timing ? hipEventRecord(r->ev[k], s) : hipSuccess; };
  HIP_TRY(mark(0, fs));
  auto zin = [&](int z) { return zi + r->zoff[z]; };
  auto out_of = [&](const float* y) {
    for (int o = 0; o < SDR_RX_NOUTPUTS; ++o)
      if (r->outs[q][o] == y && need_out(r, o)) return o;
    return -1;
  };
  auto mirror_of = [&](const float* y) { const int o = out_of(y); return o < 0 ? nullptr : r->mirror[o]; };
  auto host_n = [&](const float* y) { const int o = out_of(y); return o < 0 ? (int64_t)0 : r->out_n[o]; };
  auto zout = [&](int z) { return zf + r->zoff[z]; };
  // device taps (cached per context; the pointers stay valid for this call)
  const TapSet* ts[SDR_RX_NFILTERS] = {};
  for (int f = 0; f < SDR_RX_NFILTERS; ++f)
    if (filter_used(r, f)) TRY(get_taps(c, r->taps[f].data(), (int)r->taps[f].size(), &ts[f]));
  float** o = r->outs[q];
  const int64_t ms = r->out_stride[SDR_RX_O_DEMOD];
  FeState fst{};
  if (fast) {
    const int64_t fstride = S > 1 ? xs : ceil_div(r->B, G) * G;
    FeLaunch a{iq, r->B, fstride, 0, S, ts[SDR_RX_F_RF]->dev_f32, &ts[SDR_RX_F_RF]->h, Trf, r->rf_decim, r->u8,
               zin(Z_FE_I), zin(Z_FE_Q), r->zlen[Z_FE_I], r->phase, o[SDR_RX_O_DEMOD], ms, nullptr, nullptr,
               r->last_phi, r->wraps, ts[SDR_RX_F_RF]->dev_afr};
    HIP_TRY(sdr_launch_fe(a, fs));
    fst = FeState{iq, r->B, xs, ts[SDR_RX_F_RF]->dev_f64, zin(Z_FE_I), zin(Z_FE_Q), zout(Z_FE_I), zout(Z_FE_Q),
                  r->zlen[Z_FE_I], r->last_phi, r->wraps, r->phase, Trf, r->u8, 1};
  } else {
    TRY(sdr_rf_frontend_dev(c, iq, r->u8 ? SDR_IQ_U8 : SDR_IQ_F32, r->B, xs, 0, S, r->taps[SDR_RX_F_RF].data(),
                            Trf, r->rf_decim, zin(Z_FE_I), zin(Z_FE_Q), r->zlen[Z_FE_I], zout(Z_FE_I), zout(Z_FE_Q),
                            r->phase, o[SDR_RX_O_DEMOD], ms, nullptr, nullptr));
  }
  HIP_TRY(mark(1 + SDR_RX_ST_FE, fs));
  auto fir = [&](int f, int z, const float* x, int64_t n, int64_t xs, float* y, int64_t ys, int D, int pre = PRE_NONE,
                 const float* cmix = nullptr) {
    StageJob j{};
    j.x = x; j.c = cmix; j.taps = ts[f]->dev_f32; j.rtaps = ts[f]->dev_rev; j.taps64 = ts[f]->dev_f64;
    j.zi = zin(z); j.zf = zout(z); j.zi_stride = r->zlen[z];
    j.y = y; j.y_stride = ys; j.n = n; j.x_stride = xs;
    j.gain = 2.0f;                      // the reference's mixer gain (fmMonoBlock.py:156, fmRDSblock.py:173)
    j.pre = pre; j.D = D; j.U = 1; j.kind = JK_FIR; j.T = (int)r->taps[f].size();
    j.sym = 1;                          // linear phase (f32 taps mirror-equal): fold_tile may take it
    for (int k = 0; k < j.T / 2 && j.T <= SDR_MAX_TAPS; ++k)
      if (ts[f]->h.h[k] != ts[f]->h.h[j.T - 1 - k]) j.sym = 0;
    j.yh = mirror_of(y);
    j.yh_stride = host_n(y);
    return j;
  };
  const bool au = r->flags & (SDR_RX_AUDIO | SDR_RX_STEREO), stx = r->flags & SDR_RX_STEREO,
             rd = r->flags & SDR_RX_RDS;
  const int64_t as = au ? r->out_stride[SDR_RX_O_AUDIO] : 0;
  // What this block materialises beyond what the chain needs (sdr_rx_set_keep / the outputs a
  // submit asks for)
  auto kept = [&](int o) { return (r->keep_now >> o) & 1ull; };
  // Spans (the matrix-core rows): the PLLs take their inputs as sign codes (sdr_nco.h pll_code,
  // r06) -- all the recurrence reads of them -- stored by the pilot BPF's and the RDS x^2 + BPF's
  // tiles beside (or, when those rows are not kept, instead of) their f32 rows
  auto mm_taps = [&](int f) { const size_t t = r->taps[f].size(); return t == 101 || t == 151; };
  const bool codes = (stx || rd) && r->pcode != nullptr && M >= (int64_t)MM_MIN_WIN * MM_WT && M % 4 == 0 &&
                     M < ((int64_t)1 << 28) && (!stx || mm_taps(SDR_RX_F_PILOT)) && (!rd || mm_taps(SDR_RX_F_RDS_SQUARE));
  int8_t* c8 = codes ? r->pcode + (int64_t)q * 2 * S * r->pcs : nullptr;   // [PLL k][stream] rows, pcs bytes apart
  auto coded = [&](StageJob j, int k, int o) {
    if (codes) {
      j.y8 = c8 + (int64_t)k * S * r->pcs;
      j.y8_stride = r->pcs;
      if (!kept(o)) j.y = nullptr;
    }
    return j;
  };
  // stage A: every filter of the demodulated signal (model/fmMonoBlock.py:101-105, :117,
  // :151; model/fmRDSblock.py:156)
  std::vector<StageJob> A;
  if (au) A.push_back(fir(SDR_RX_F_AUDIO, Z_AUDIO, o[SDR_RX_O_DEMOD], M, ms, o[SDR_RX_O_AUDIO], as, r->audio_decim));
  if (stx) {
    A.push_back(coded(fir(SDR_RX_F_PILOT, Z_PILOT, o[SDR_RX_O_DEMOD], M, ms, o[SDR_RX_O_BPF_RECOVERY], ms, 1), 0,
                      SDR_RX_O_BPF_RECOVERY));
    A.push_back(fir(SDR_RX_F_STEREO_BPF, Z_BAND, o[SDR_RX_O_DEMOD], M, ms, o[SDR_RX_O_BPF_EXTRACTION], ms, 1));
  }
  if (rd) A.push_back(fir(SDR_RX_F_RDS_EXTRACT, Z_EXTRACT, o[SDR_RX_O_DEMOD], M, ms, o[SDR_RX_O_RDS_EXTRACT], ms, 1));
  HIP_TRY(launch_stage(A, S, fs, &fst));
  HIP_TRY(mark(1 + SDR_RX_ST_A, fs));
  // stage B: RDS squaring non-linearity + BPF (model/fmRDSblock.py:161-164)
  if (rd) HIP_TRY(launch_stage({coded(fir(SDR_RX_F_RDS_SQUARE, Z_SQUARE, o[SDR_RX_O_RDS_EXTRACT], M, ms,
                                          o[SDR_RX_O_RDS_PRE_PLL], ms, 1, PRE_SQUARE), 1, SDR_RX_O_RDS_PRE_PLL)}, S, fs));
  HIP_TRY(mark(1 + SDR_RX_ST_B, fs));
  // PLLs (model/fmMonoBlock.py:119, model/fmRDSblock.py:167): one lane per recurrence.
  // Pipelined, the three launches go to three streams: the per-sample constants with the
  // front half (trigOffset = M x blocks since reset, known here), the recurrence alone on
  // its own stream -- block k's starts as soon as block k-1's is done, beside block k-1's
  // NCO and stages C-E and block k+1's front half -- and the NCO with the back half.  Phase
  // and constant rows alternate with the row set; set q is free once block k-2's back half
  // (which waited for its recurrence) is done.
  const bool plls = stx || rd;
  // Beyond the chain: the NCO rows, and the RDS LPF rows.  Without them the stage-C mixers
  // form the NCO from the PLL phase rows where they stage their inputs (PRE_NCO, sdr_nco.h) and
  // the RDS LPF + resampler is the composite filter (rx_cres_kernel), which runs either way.
  const bool cres = rd && r->ctaps != nullptr;
  const int tsl = stx ? (int)r->taps[SDR_RX_F_STEREO_LPF].size() : 151;
  const bool tiles_ok = (tsl == 101 || tsl == 151) && (r->audio_decim == 1 || r->audio_decim == 5);   // PRE_NCO tiles
  const bool nco_rows = (stx && kept(SDR_RX_O_STEREO_NCO)) || (rd && (kept(SDR_RX_O_RDS_NCO_I) || kept(SDR_RX_O_RDS_NCO_Q))) ||
                        M < 2 || (rd && !cres) || !tiles_ok;
  const bool lpf_rows = rd && (!cres || kept(SDR_RX_O_RDS_LPF_I) || kept(SDR_RX_O_RDS_LPF_Q));
  // The recurrences get a stream of their own (block k's beside block k-1's NCO and stages
  // C-E) whenever the receiver is pipelined.  Round 4 kept a few per-block recurrences (c4:
  // one, ~26 us) on the back stream, where each cross-stream hop then cost more than the
  // overlap returned (c4 790-840 -> 950 MS/s); with two blocks in flight and the trimmed
  // event calls (r04b) the hop pays: c4 1 022 -> 1 090 MS/s (medians of 8 interleaved runs,
  // profiles/r04/iter/r04b/pllstream/).
  const bool mid = r->pipe;
  hipStream_t ps = mid ? r->mid : st;
  PllJobs P{};
  NcoSrc nsrc[2] = {};                 // per PLL (0 stereo, 1 RDS): where stage C takes its NCO from
  if (plls) {
    P.nstreams = S;
    P.n = M;
    P.stats = c->pll_stats;
    P.nco_rows = nco_rows ? 1 : 0;
    P.work = r->pllw_bytes ? r->pllw + (int64_t)q * r->pllw_bytes : nullptr;
    double* th = r->theta + (int64_t)q * 2 * S * r->ths;
    double* pc = r->pllc + (int64_t)q * 2 * S * r->cst;
    const double off = (double)M * (double)r->blocks;
    int64_t pb = 0;
    int nb = 0;
    const bool lng = sdr_pll_long_geom(M, &pb, &nb);
    // the loops' phase rows in the compact form (sdr_nco.h, r06): half the bytes of the solve's
    // stores and of the mixers' loads.  Every reader decodes them -- the matrix-core mixers
    // (TH32 forms), the VALU tiles and final states (nco_f32x4, nco_at), the NCO kernel -- so
    // the form depends only on the call's geometry (pseudo-blocks on a line), never on what a
    // block keeps
#ifdef SDR_NO_TH32   // diagnostic builds only (tools/build_dbg.sh): the full rows, for an A/B of the outputs
    const bool th32 = false, th32r = false;
#else
    const bool th32 = lng && pb % TH32_LINE == 0 && stx, th32r = lng && pb % TH32_LINE == 0 && rd;
#endif
    auto add = [&](int k, const float* in, double* thk, float* ni, float* nq, double* pck) -> int {
      const double* resp = nullptr;
      TRY(get_resp(c, r->pll[k], M, &resp));
      const int jq = P.njobs;
      P.j[P.njobs++] = PllJob{in, ms, r->pll_state[k], thk, r->ths, ni, nq, ms, r->pll[k], pck, r->cst, off, 1, resp};
      if (codes) {
        P.j[jq].in8 = c8 + (int64_t)k * S * r->pcs;
        P.j[jq].in8_stride = r->pcs;
      }
      NcoSrc& N = nsrc[k];
      N.theta = M >= 2 ? thk : nullptr;   // (M < 2: the sequential kernels' Q-form rows; mix from the NCO rows)
      if ((k == 0 && th32) || (k == 1 && th32r)) P.j[jq].th32 = N.th32 = 1;
      N.th_stride = r->ths;
      N.nco_i = ni;
      N.nco_q = nq;
      N.out_stride = ms;
      N.w = 2.0 * M_PI * (r->pll[k].freq / r->pll[k].fs);
      N.scale = r->pll[k].scale;
      N.adj = r->pll[k].adj;
      N.n = M;
      if (lng) {
        N.blk = long_blk0(P.work, 0, S, nb, jq * S);        // njobs fixed up below
        N.blk_stride = nb;
        N.nb = nb;
        N.pb = pb;
        N.resp = resp;
        N.resp32 = resp32_of(resp, pb);
      }
      return SDR_OK;
    };
    if (stx) TRY(add(0, o[SDR_RX_O_BPF_RECOVERY], th, o[SDR_RX_O_STEREO_NCO], nullptr, pc));
    if (rd) TRY(add(1, o[SDR_RX_O_RDS_PRE_PLL], th + (int64_t)S * r->ths, o[SDR_RX_O_RDS_NCO_I], o[SDR_RX_O_RDS_NCO_Q],
                    pc + (int64_t)S * r->cst));
    if (lng)                                                // the records follow P.njobs x S headers
      for (NcoSrc& N : nsrc)
        if (N.blk) N.blk = reinterpret_cast<const LongBlk*>(reinterpret_cast<const char*>(N.blk) +
                                                              (int64_t)P.njobs * S * sizeof(LongHdr));
    HIP_TRY(sdr_launch_pll_prep(P, fs));
  }
  if (r->pipe) {
    HIP_TRY(hipEventRecord(r->ev_front[q], fs));
    if (plls && mid) {
      HIP_TRY(hipStreamWaitEvent(ps, r->ev_front[q], 0));
      if (r->blocks >= r->nq && r->blocks - r->nq > r->host_done) HIP_TRY(hipStreamWaitEvent(ps, r->ev_back[q], 0));
    } else {
      HIP_TRY(hipStreamWaitEvent(st, r->ev_front[q], 0));
    }
  }
  if (plls) HIP_TRY(sdr_launch_pll_loop(P, ps));
  HIP_TRY(mark(1 + SDR_RX_ST_PLL, ps));
  if (mid && plls) {
    HIP_TRY(hipEventRecord(r->ev_mid[q], ps));
    HIP_TRY(hipStreamWaitEvent(st, r->ev_mid[q], 0));
  }
  if (plls) HIP_TRY(sdr_launch_pll_nco(P, st));
  // stage C: the stereo mixer + LPF (its store also forms L and R); the RDS I/Q mixer + LPF
  // rows only when they are kept (or without the composite filter)
  auto mixer = [&](StageJob j, int k, int sin_) {
    if (nsrc[k].theta != nullptr && (j.T == 101 || j.T == 151) && (j.D == 1 || j.D == 5)) {
      j.pre = PRE_NCO;
      j.nco = nsrc[k];
      j.nco_sin = sin_;
      j.c = nullptr;
    }
    return j;
  };
  std::vector<StageJob> C;
  if (stx) {
    StageJob j = fir(SDR_RX_F_STEREO_LPF, Z_SLPF, o[SDR_RX_O_BPF_EXTRACTION], M, ms, o[SDR_RX_O_STEREO], as,
                     r->audio_decim, PRE_MIX, o[SDR_RX_O_STEREO_NCO]);          // fmMonoBlock.py:155-162
    j.mono = o[SDR_RX_O_AUDIO];                                                 // :166-170 (intended)
    j.left = o[SDR_RX_O_LEFT];
    j.right = o[SDR_RX_O_RIGHT];
    j.lh = r->mirror[SDR_RX_O_LEFT];
    j.rh = r->mirror[SDR_RX_O_RIGHT];
    j.yh_stride = r->out_n[SDR_RX_O_STEREO];                                    // == out_n of L and R
    C.push_back(mixer(j, 0, 0));
  }
  if (lpf_rows) {                                                              // fmRDSblock.py:173-182
    for (int k = 0; k < 2; ++k) {
      StageJob j = fir(SDR_RX_F_RDS_LPF, k ? Z_RLPF_Q : Z_RLPF_I, o[SDR_RX_O_RDS_EXTRACT], M, ms,
                       o[k ? SDR_RX_O_RDS_LPF_Q : SDR_RX_O_RDS_LPF_I], ms, 1, PRE_MIX,
                       o[k ? SDR_RX_O_RDS_NCO_Q : SDR_RX_O_RDS_NCO_I]);
      if (cres) j.zf = nullptr;                 // the composite kernel writes the LPF's final states
      C.push_back(mixer(j, 1, k));
    }
  }
  HIP_TRY(launch_stage(C, S, st));
  HIP_TRY(mark(1 + SDR_RX_ST_C, st));
  if (rd) {
    const int64_t rs = r->out_stride[SDR_RX_O_RDS_RES_I];
    if (cres) {
      // stage D: the RDS mixers + LPF + x19 / 80 resampler as one composite filter, and the
      // LPF's and anti-image filter's final states
      CresJob J{};
      J.x = o[SDR_RX_O_RDS_EXTRACT];
      J.n = M;
      J.x_stride = ms;
      J.nco = nsrc[1];
      J.ctaps = r->ctaps;
      J.h64 = ts[SDR_RX_F_RDS_LPF]->dev_f64;
      J.g64 = ts[SDR_RX_F_RDS_ANTI]->dev_f64;
      J.zi_l[0] = zin(Z_RLPF_I); J.zi_l[1] = zin(Z_RLPF_Q);
      J.zi_a[0] = zin(Z_ANTI_I); J.zi_a[1] = zin(Z_ANTI_Q);
      J.zf_l[0] = zout(Z_RLPF_I); J.zf_l[1] = zout(Z_RLPF_Q);
      J.zf_a[0] = zout(Z_ANTI_I); J.zf_a[1] = zout(Z_ANTI_Q);
      J.zs = r->zlen[Z_RLPF_I];
      J.y[0] = o[SDR_RX_O_RDS_RES_I]; J.y[1] = o[SDR_RX_O_RDS_RES_Q];
      J.yh[0] = r->mirror[SDR_RX_O_RDS_RES_I]; J.yh[1] = r->mirror[SDR_RX_O_RDS_RES_Q];
      J.y_stride = rs;
      J.yh_stride = r->out_n[SDR_RX_O_RDS_RES_I];
      J.R = r->R;
      J.tiles = (int)ceil_div(r->R, CR_TO);
      J.nstreams = S;
      const int64_t grid = (int64_t)J.tiles * S + S;
      if (grid > 0x7fffffff || r->zlen[Z_ANTI_I] != J.zs) return fail(SDR_EINVAL, "sdr_rx: composite RDS geometry");
      // spans: the matrix-core form (per job length, as launch_stage decides: a stream's outputs
      // do not depend on how many streams share the launch)
      if (M >= (int64_t)MM_MIN_WIN * MM_WT && M % 4 == 0 && J.nco.theta != nullptr) {
        const int64_t wins = ceil_div(r->R, CM_WO) * S;
        const int wgs = (int)std::min<int64_t>(CM_WGS, ceil_div(wins, 4));
        if (J.nco.th32)
          hipLaunchKernelGGL(rx_cresmm_kernel<true>, dim3((unsigned)(S + wgs)), dim3(RX_NT), 0, st, J, r->ctaps + CR_NTAPS, wgs);
        else
          hipLaunchKernelGGL(rx_cresmm_kernel<false>, dim3((unsigned)(S + wgs)), dim3(RX_NT), 0, st, J, r->ctaps + CR_NTAPS, wgs);
      } else {
        hipLaunchKernelGGL(rx_cres_kernel, dim3((unsigned)grid), dim3(CR_NT), 0, st, J);
      }
      HIP_TRY(hipGetLastError());
    } else {
      // stage D: rational resamplers (fmRDSblock.py:184-199)
      std::vector<StageJob> Dj;
      for (int k = 0; k < 2; ++k) {
        StageJob j = fir(SDR_RX_F_RDS_ANTI, k ? Z_ANTI_Q : Z_ANTI_I, o[k ? SDR_RX_O_RDS_LPF_Q : SDR_RX_O_RDS_LPF_I], M, ms,
                         o[k ? SDR_RX_O_RDS_RES_Q : SDR_RX_O_RDS_RES_I], rs, r->rds_down);
        j.kind = JK_RESAMPLE;
        j.U = r->rds_up;
        Dj.push_back(j);
      }
      HIP_TRY(launch_stage(Dj, S, st));
    }
    HIP_TRY(mark(1 + SDR_RX_ST_D, st));
    // stage E: RRC (fmRDSblock.py:202-204)
    HIP_TRY(launch_stage({fir(SDR_RX_F_RDS_RRC, Z_RRC_I, o[SDR_RX_O_RDS_RES_I], r->R, rs, o[SDR_RX_O_RDS_RRC_I], rs, 1),
                          fir(SDR_RX_F_RDS_RRC, Z_RRC_Q, o[SDR_RX_O_RDS_RES_Q], r->R, rs, o[SDR_RX_O_RDS_RRC_Q], rs, 1)},
                         S, st));
  } else {
    HIP_TRY(mark(1 + SDR_RX_ST_D, st));
  }
  for (int oo = 0; oo < SDR_RX_NOUTPUTS; ++oo) {
    const bool nco_o = oo == SDR_RX_O_STEREO_NCO || oo == SDR_RX_O_RDS_NCO_I || oo == SDR_RX_O_RDS_NCO_Q;
    const bool lpf_o = oo == SDR_RX_O_RDS_LPF_I || oo == SDR_RX_O_RDS_LPF_Q;
    const bool pin_o = oo == SDR_RX_O_BPF_RECOVERY || oo == SDR_RX_O_RDS_PRE_PLL;      // (codes: when kept)
    r->made[oo] = need_out(r, oo) && (!nco_o || nco_rows) && (!lpf_o || lpf_rows) && (!pin_o || !codes || kept(oo));
  }
  HIP_TRY(mark(1 + SDR_RX_ST_E, st));
  if (r->pipe) HIP_TRY(hipEventRecord(r->ev_back[q], st));
  std::memcpy(r->out, r->outs[q], sizeof r->out);
  r->parity ^= 1;
  ++r->blocks;
  return SDR_OK;
}

namespace {
// grow a pinned host buffer (synchronising first: work in flight may use it).  Coherent
// (uncached by the GPU): the device reads the IQ the host wrote for this block, and the
// host reads what the stage kernels stored, with no copy engine in between.
int grow_pinned(sdr_rx* r, void** p, size_t* cap, size_t bytes) {
  if (*cap >= bytes) return SDR_OK;
  if (*p) {
    HIP_TRY(hipStreamSynchronize(r->c->stream));
    HIP_TRY(hipHostFree(*p));
    *p = nullptr;
    *cap = 0;
  }
  hipError_t e = hipHostMalloc(p, bytes, hipHostMallocCoherent);
  if (e != hipSuccess) return fail(SDR_ENOMEM, "sdr_rx: hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
  *cap = bytes;
  return SDR_OK;
}
// outputs a stage kernel stores (and can store a host copy of); the demod (FE kernel) and
// the NCOs (PLL) come back by copy
bool stage_output(int o) {
  return o != SDR_RX_O_DEMOD && o != SDR_RX_O_STEREO_NCO && o != SDR_RX_O_RDS_NCO_I && o != SDR_RX_O_RDS_NCO_Q;
}

// Deliver the block in flight: wait for it, copy its rows out of pinned memory.
// the oldest block in flight: wait for it, copy its outputs out of its pinned slot
int deliver(sdr_rx* r) {
  if (r->pq_n == 0) return SDR_OK;
  const sdr_rx::Pending& P = r->pq[r->pq_head];
  r->pq_head = (r->pq_head + 1) % 4;
  --r->pq_n;
  HIP_TRY(hipEventSynchronize(P.ev));
  r->host_done = std::max(r->host_done, P.blk);
  const float* base = r->pin_out + (size_t)P.slot * r->out_slot / sizeof(float);
  for (int i = 0; i < P.nout; ++i) {
    const int64_t n = r->out_n[P.which[i]];
    const float* src = base + P.region[P.which[i]];
    for (int s = 0; s < r->S; ++s) std::memcpy(P.out[i] + s * P.os[i], src + s * n, sizeof(float) * (size_t)n);
  }
  return SDR_OK;
}

}  // namespace

int sdr_rx_process(sdr_rx* r, const void* iq_host, int64_t iq_stride) {
  return sdr_rx_run(r, iq_host, iq_stride, 0, nullptr, nullptr, nullptr);
}

// One block from host memory, without waiting for it.  The per-block cost at the
// reference's block sizes is the number of engine hand-offs, not bytes
// (tools/xfer_probe.hip: an SDMA upload, two kernels, an SDMA download and a wait take
// 35 us; the same kernels reading and writing pinned host memory directly, 25 us), so: the
// IQ is copied into a pinned slot and the FE kernel reads it from there over PCIe; each
// requested output is stored into the slot's pinned output region by the stage kernel that
// produces it (the demod and NCO rows, which no stage kernel stores, come back by copy).
// depth + 1 slots (sdr_rx_set_depth, default 1): while block k runs, the host delivers block
// k-depth's outputs (into the buffers given with it) and returns; sdr_rx_flush delivers the rest.
int sdr_rx_submit(sdr_rx* r, const void* iq_host, int64_t iq_stride, int nout, const int* which, float* const* out,
                  const int64_t* out_stride) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (iq_host == nullptr) return fail(SDR_EINVAL, "sdr_rx_submit: iq is NULL");
  if (r->S > 1 && iq_stride < r->B) return fail(SDR_EINVAL, "sdr_rx_submit: iq_stride %lld < block", (long long)iq_stride);
  if (nout < 0 || nout > SDR_RX_MAXOUT || (nout > 0 && (which == nullptr || out == nullptr)))
    return fail(SDR_EINVAL, "sdr_rx_submit: %d outputs (at most %d)", nout, SDR_RX_MAXOUT);
  if (!r->ready) TRY(rx_finalize(r));
  for (int i = 0; i < nout; ++i) {
    if (which[i] < 0 || which[i] >= SDR_RX_NOUTPUTS || !need_out(r, which[i]))
      return fail(SDR_EINVAL, "sdr_rx_submit: output %d is not produced by flags 0x%x", which[i], r->flags);
    if (out[i] == nullptr) return fail(SDR_EINVAL, "sdr_rx_submit: output buffer %d is NULL", i);
    if (r->S > 1 && out_stride && out_stride[i] < r->out_n[which[i]])
      return fail(SDR_EINVAL, "sdr_rx_submit: out_stride[%d] too small", i);
  }
  TRY(set_dev(r->c));
  hipStream_t st = r->c->stream;
  const int64_t es = r->u8 ? 2 : 8;                      // bytes per complex sample
  const int64_t xs = r->S > 1 ? iq_stride : r->B;
  const size_t bytes = (size_t)(xs * (r->S - 1) + r->B) * es;
  // pinned output regions, one per distinct requested output (rows out_n apart)
  sdr_rx::Pending P;
  bool want[SDR_RX_NOUTPUTS] = {};
  size_t obytes = 0;
  for (int i = 0; i < nout; ++i) {
    const int o = which[i];
    P.which[i] = o;
    P.out[i] = out[i];
    P.os[i] = (r->S > 1 && out_stride) ? out_stride[i] : r->out_n[o];
    if (want[o]) continue;
    want[o] = true;
    P.region[o] = obytes / sizeof(float);
    obytes += sizeof(float) * (size_t)(r->out_n[o] * r->S);
  }
  const size_t in_slot = (bytes + 255) / 256 * 256, out_slot = (std::max<size_t>(obytes, 16) + 255) / 256 * 256;
  const int nslot = r->depth + 1;
  if (in_slot > r->in_slot || out_slot > r->out_slot) {   // grow (the blocks in flight are delivered first)
    while (r->pq_n > 0) TRY(deliver(r));
    r->in_slot = std::max(r->in_slot, in_slot);
    r->out_slot = std::max(r->out_slot, out_slot);
    TRY(grow_pinned(r, &r->pin_in, &r->pin_in_cap, nslot * r->in_slot));
    TRY(grow_pinned(r, reinterpret_cast<void**>(&r->pin_out), &r->pin_out_cap, nslot * r->out_slot));
    for (int q = 0; q < nslot; ++q)
      if (!r->ev_done[q]) HIP_TRY(hipEventCreateWithFlags(&r->ev_done[q], hipEventDisableTiming));
  }
  const int slot = (int)(r->subs % nslot);
  // slot `slot` was last used by block k-depth-1, delivered (waited for) by the previous call
  char* pin = static_cast<char*>(r->pin_in) + (size_t)slot * r->in_slot;
  float* pout = r->pin_out + (size_t)slot * r->out_slot / sizeof(float);
  std::memcpy(pin, iq_host, bytes);
  for (int o = 0; o < SDR_RX_NOUTPUTS; ++o) r->mirror[o] = want[o] && stage_output(o) ? pout + P.region[o] : nullptr;
  uint64_t wmask = 0;                                     // materialise what this call returns
  for (int o = 0; o < SDR_RX_NOUTPUTS; ++o)
    if (want[o]) wmask |= 1ull << o;
  r->keep_now = wmask;
  const int rc = sdr_rx_process_dev(r, pin, xs);
  r->keep_now = r->keep;
  for (float*& m : r->mirror) m = nullptr;
  TRY(rc);
  bool copied = false;
  for (int o = 0; o < SDR_RX_NOUTPUTS; ++o) {
    if (!want[o] || stage_output(o)) continue;
    copied = true;
    const int64_t n = r->out_n[o];
    HIP_TRY(hipMemcpy2DAsync(pout + P.region[o], sizeof(float) * (size_t)n, r->out[o],
                             sizeof(float) * (size_t)r->out_stride[o], sizeof(float) * (size_t)n, (size_t)r->S,
                             hipMemcpyDeviceToHost, st));
  }
  const int qb = (int)((r->blocks - 1) % r->nq);
  if (r->pipe && !copied && r->depth < r->nq) {
    // nothing after the back half: its row-set event marks the block's completion (one event
    // call fewer per block).  Not at depth 3 (nq 3): block k+3 re-records the set's event
    // before block k is delivered, and the host would wait for the newest block each time --
    // the pipeline drained at every call (c4 1 163 -> 472 MS/s)
    P.ev = r->ev_back[qb];
  } else {
    // the row set is free for block k+nq once these copies have read it too (the event the
    // front half of block k+nq waits for is recorded again, after them)
    if (r->pipe) HIP_TRY(hipEventRecord(r->ev_back[qb], st));
    HIP_TRY(hipEventRecord(r->ev_done[slot], st));
    P.ev = r->ev_done[slot];
  }
  ++r->subs;
  P.slot = slot;
  P.nout = nout;
  P.blk = r->blocks - 1;
  r->pq[(r->pq_head + r->pq_n) % 4] = P;
  ++r->pq_n;
  while (r->pq_n > r->depth) TRY(deliver(r));            // block k-depth
  return SDR_OK;
}

int sdr_rx_flush(sdr_rx* r) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (r->pq_n == 0) return SDR_OK;
  TRY(set_dev(r->c));
  while (r->pq_n > 0) TRY(deliver(r));
  return SDR_OK;
}

int sdr_rx_set_depth(sdr_rx* r, int depth) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (r->ready) return fail(SDR_EINVAL, "sdr_rx_set_depth: the receiver has processed a block");
  if (depth < 1 || depth > 3) return fail(SDR_EINVAL, "sdr_rx_set_depth: depth %d outside [1, 3]", depth);
  r->depth = depth;
  r->nq = depth >= 2 ? 3 : 2;
  return SDR_OK;
}

// One block from host memory, waited for: the per-block drop-in call of fmMonoBlock.py's loop.
int sdr_rx_run(sdr_rx* r, const void* iq_host, int64_t iq_stride, int nout, const int* which, float* const* out,
               const int64_t* out_stride) {
  if (r != nullptr) TRY(sdr_rx_flush(r));                // an earlier submit's block first
  TRY(sdr_rx_submit(r, iq_host, iq_stride, nout, which, out, out_stride));
  return sdr_rx_flush(r);
}

int sdr_rx_output(sdr_rx* r, int which, float** dev, int64_t* stride, int64_t* n) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (which < 0 || which >= SDR_RX_NOUTPUTS) return fail(SDR_EINVAL, "sdr_rx_output: output %d", which);
  if (!r->ready) TRY(rx_finalize(r));
  if (!need_out(r, which)) return fail(SDR_EINVAL, "sdr_rx_output: output %d is not produced by flags 0x%x", which, r->flags);
  if (dev) *dev = r->out[which];
  if (stride) *stride = r->out_stride[which];
  if (n) *n = r->out_n[which];
  return SDR_OK;
}

int sdr_rx_set_keep(sdr_rx* r, uint64_t mask) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  r->keep = r->keep_now = mask;
  return SDR_OK;
}

int sdr_rx_fetch(sdr_rx* r, int which, float* host, int64_t host_stride) {
  float* d;
  int64_t ds, n;
  TRY(sdr_rx_output(r, which, &d, &ds, &n));
  if (!r->made[which])
    return fail(SDR_EINVAL, "sdr_rx_fetch: output %d was not materialised by the latest block (sdr_rx_set_keep)", which);
  if (host == nullptr) return fail(SDR_EINVAL, "sdr_rx_fetch: host is NULL");
  if (r->S > 1 && host_stride < n) return fail(SDR_EINVAL, "sdr_rx_fetch: host_stride %lld < %lld", (long long)host_stride, (long long)n);
  TRY(set_dev(r->c));
  HIP_TRY(hipMemcpy2DAsync(host, sizeof(float) * (size_t)(r->S > 1 ? host_stride : n), d, sizeof(float) * (size_t)ds,
                           sizeof(float) * (size_t)n, (size_t)r->S, hipMemcpyDeviceToHost, r->c->stream));
  HIP_TRY(hipStreamSynchronize(r->c->stream));
  return SDR_OK;
}

int sdr_rx_set_timing(sdr_rx* r, int on) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  TRY(set_dev(r->c));
  if (on && !r->ev[0])
    for (hipEvent_t& e : r->ev) HIP_TRY(hipEventCreate(&e));
  r->timing = on != 0;
  return SDR_OK;
}

int sdr_rx_stage_ms(sdr_rx* r, float* ms) {
  if (r == nullptr || ms == nullptr) return fail(SDR_EINVAL, "sdr_rx_stage_ms: NULL argument");
  if (!r->timing || r->blocks == 0) return fail(SDR_EINVAL, "sdr_rx_stage_ms: no timed block (sdr_rx_set_timing)");
  HIP_TRY(hipEventSynchronize(r->ev[SDR_RX_NSTAGES]));
  for (int k = 0; k < SDR_RX_NSTAGES; ++k) HIP_TRY(hipEventElapsedTime(&ms[k], r->ev[k], r->ev[k + 1]));
  return SDR_OK;
}

int sdr_rx_pll_stats(sdr_rx* r, int64_t* out, int reset) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  TRY(set_dev(r->c));
  if (r->front) HIP_TRY(hipStreamSynchronize(r->front));
  if (r->mid) HIP_TRY(hipStreamSynchronize(r->mid));
  HIP_TRY(hipStreamSynchronize(r->c->stream));
  return sdr_pll_stats(r->c, out, reset);
}

int sdr_rx_state(sdr_rx* r, double* phase, double* pll_stereo, double* pll_rds) {
  if (r == nullptr) return fail(SDR_EINVAL, "sdr_rx is NULL");
  if (!r->ready) TRY(rx_finalize(r));
  TRY(set_dev(r->c));
  hipStream_t st = r->c->stream;
  const size_t S = (size_t)r->S;
  if (phase) HIP_TRY(hipMemcpyAsync(phase, r->phase, sizeof(double) * S, hipMemcpyDeviceToHost, st));
  if (pll_stereo) HIP_TRY(hipMemcpyAsync(pll_stereo, r->pll_state[0], sizeof(double) * 6 * S, hipMemcpyDeviceToHost, st));
  if (pll_rds) HIP_TRY(hipMemcpyAsync(pll_rds, r->pll_state[1], sizeof(double) * 6 * S, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return SDR_OK;
}

}  // extern "C"
