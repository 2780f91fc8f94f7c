/* libsdr.so — C-ABI of the MI355X-native FM-SDR hot path (gfx950 HIP kernels).
 *
 * This is the drop-in boundary for the reference's per-block signal-processing
 * functions.  Plain pointers and sizes only; no torch/numpy types.
 * Each entry point names the reference interface it replaces (file:line under the
 * reference repository m1nty/Real-Time-Software-Defined-Radio).
 *
 * Conventions
 *   - Return value: SDR_OK (0) or a negative SDR_E* code; sdr_last_error() returns
 *     the calling thread's last error message (the Python layer raises ValueError
 *     for SDR_EINVAL, NotImplementedError for SDR_EUNSUPPORTED, RuntimeError else;
 *     mirroring scipy.signal.lfilter's ValueError/NotImplementedError,
 *     scipy/signal/_signaltools.py:2143-2151).
 *   - Filter state `zi` uses scipy.signal.lfilter's convention (length taps-1,
 *     f64): y[n] = (b*x)[n] + zi[n] for n < taps-1, and the returned zf is the tail
 *     of the full convolution.  Host `*_inout` state arrays are overwritten with the
 *     new state, so reference and libsdr calls can be mixed block by block.
 *   - Decimated outputs are y[D*m] for m = 0 .. ceil(n/D)-1 (lfilter(...)[::D]).
 *   - Demod phase state is the reference's accumulated unwrapped phase
 *     (model/fmSupportLib.py:40-44), returned as phi_last + 2*pi*(number of wraps).
 *   - A context (sdr_ctx) owns one HIP stream and scratch memory on one device; it is
 *     not thread-safe: one context per host thread per GPU.
 *   - Host-buffer functions are synchronous.  `*_dev` functions take device
 *     pointers and are asynchronous on the context's stream (sdr_stream()).
 *   - Numerics: samples are processed in f32 (inputs f32 or u8); filter-state (zf)
 *     and PLL phase arithmetic are f64.
 */
#ifndef SDR_H_
#define SDR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDR_ABI_VERSION 1

enum {
  SDR_OK = 0,
  SDR_EINVAL = -1,      /* bad argument (shape, NULL, range) */
  SDR_EHIP = -2,        /* HIP runtime error */
  SDR_ENOMEM = -3,      /* device allocation failed */
  SDR_EUNSUPPORTED = -4, /* valid but not implemented configuration */
  SDR_EDOMAIN = -5       /* math domain error the reference raises (log10 of 0) */
};

enum { SDR_IQ_F32 = 0, SDR_IQ_U8 = 1 };                  /* interleaved IQ sample types */
enum { SDR_PRE_NONE = 0, SDR_PRE_SQUARE = 1, SDR_PRE_MIX = 2 }; /* FIR input pre-ops */
enum { SDR_REAL_F32 = 0, SDR_REAL_F64 = 1 };              /* real sample types (PSD) */
#define SDR_DFT_MAX_N (1 << 16)
#define SDR_MAX_RESAMPLE_TAPS 4096                           /* sdr_resample* filter length */

typedef struct sdr_ctx sdr_ctx;

/* ---- library / context ------------------------------------------------------- */
int sdr_abi_version(void);
const char* sdr_last_error(void);
int sdr_device_count(int* n);
/* Which physical GPU `device` is (bench.py's multi-rank line proves its rank -> device map
 * with it): its PCI bus id ("dddd:bb:dd.f", NUL-terminated into pci[len]) and compute units. */
int sdr_device_info(int device, char* pci, int len, int* cus);
int sdr_create(int device, sdr_ctx** out);
void sdr_destroy(sdr_ctx* ctx);
int sdr_synchronize(sdr_ctx* ctx);
void* sdr_stream(sdr_ctx* ctx); /* the hipStream_t all kernels of this context use */

/* ---- device memory and timing (replace the static float[5][307200] ring and the
 *      std::queue<void*> hand-off of src/fm_radio.cpp:22,51,86-145) ---------------- */
int sdr_malloc(sdr_ctx* ctx, int64_t bytes, void** out);
int sdr_free(sdr_ctx* ctx, void* p);
int sdr_memcpy_h2d(sdr_ctx* ctx, void* dst, const void* src, int64_t bytes);
int sdr_memcpy_d2h(sdr_ctx* ctx, void* dst, const void* src, int64_t bytes);
int sdr_memcpy_d2d(sdr_ctx* ctx, void* dst, const void* src, int64_t bytes); /* async */
int sdr_memset(sdr_ctx* ctx, void* dst, int value, int64_t bytes);          /* async */
int sdr_event_create(sdr_ctx* ctx, void** ev);
int sdr_event_record(sdr_ctx* ctx, void* ev);
int sdr_event_elapsed_ms(void* ev0, void* ev1, float* ms);
int sdr_event_destroy(void* ev);
/* The box's copy-kernel bandwidth (the roofline fraction beside a measured copy):
 * a 16-B-per-lane streaming copy of `bytes` on the context stream, best of `reps` after two
 * warm-ups; *gbs counts read + write.  Synchronous; allocates 2 x bytes for the call. */
int sdr_copy_bandwidth(sdr_ctx* ctx, int64_t bytes, int reps, double* gbs);
/* The read-only stream: `bytes` read once (16 B per lane, nontemporal, 8 loads in flight per
 * lane), best of `reps` after two warm-ups, GB/s.  The ceiling for kernels that read their
 * input once and write little (the front ends). */
int sdr_read_bandwidth(sdr_ctx* ctx, int64_t bytes, int reps, double* gbs);

/* ================================================================================
 * Host-buffer drop-in entry points (synchronous)
 * ================================================================================ */

/* RF front end: lfilter(rf_coeff, 1.0, iq[0::2], zi_i)[::decim], same for Q, then
 * fmDemodArctan(i_ds, q_ds, prev_phase).
 * Replaces model/fmMonoBlock.py:86-98 (model/fmSupportLib.py:15-44) and
 * src/fm_radio.cpp:66-84 -> src/filter.cpp:187-219 (convolveWithDecimIQ) +
 * src/rf_module.cpp:13-34 (fmDemodArctan).  iq: n complex samples interleaved,
 * f32 or u8 ((u8-128)/128, src/iofunc.cpp:61-69).  zi_i/zi_q (taps-1, in/out) may
 * both be NULL (zero initial state, no state out); prev_phase may be NULL (0.0).
 * demod: ceil(n/decim) floats; i_ds/q_ds (optional, both or neither): the decimated
 * filter outputs.  Fast tiled kernel for taps 101/151 at decim 10; other f32 shapes
 * use the generic kernels; u8 needs the fast shape (else SDR_EUNSUPPORTED). */
int sdr_rf_frontend(sdr_ctx* ctx, const void* iq, int iq_dtype, int64_t n, const double* b,
                    int taps, int decim, double* zi_i, double* zi_q, double* prev_phase,
                    float* demod, float* i_ds, float* q_ds);

/* lfilter(b, 1.0, x, zi)[::decim] on a real f32 stream.
 * Replaces model/fmMonoBlock.py:101-105 (audio), :117/:151 (stereo BPFs, decim 1),
 * model/fmRDSblock.py:156/:164/:180/:202 and src/filter.cpp:96-185
 * (convolveFIR, convolveWithDecim, convolveWithDecimPointer). */
int sdr_lfilter_decim(sdr_ctx* ctx, const float* x, int64_t n, const double* b, int taps,
                      int decim, double* zi_inout, float* y);

/* lfilter with a fused input pre-op: PRE_SQUARE filters x*x
 * (model/fmRDSblock.py:161-164, src/filter.cpp:342-370), PRE_MIX filters
 * (x*mix)*gain (model/fmMonoBlock.py:155-160, model/fmRDSblock.py:173-182,
 * src/filter.cpp:373-401 convolveWithDecimAndMixer). */
int sdr_lfilter(sdr_ctx* ctx, const float* x, const float* mix, float gain, int pre, int64_t n,
                const double* b, int taps, int decim, double* zi_inout, float* y);

/* Rational resampler: lfilter(b, 1.0, zero-stuff(x, up), zi)[::down] * up, without
 * materialising the zero-stuffed stream; zi lives on the upsampled stream.
 * Replaces model/fmRDSblock.py:184-199 and src/filter.cpp:301-339
 * (convolveWithDecimMode1RDS), and the mode-1 audio resampler src/filter.cpp:222-298
 * (convolveWithDecimMode1[Pointer], 24/125 at 6 MHz, src/fm_radio.cpp:174-180, :228) whose
 * output is y/up (the reference applies the up gain at the int16 conversion, :297).
 * taps <= SDR_MAX_RESAMPLE_TAPS.  y: ceil(n*up/down) floats. */
int sdr_resample(sdr_ctx* ctx, const float* x, int64_t n, const double* b, int taps, int up,
                 int down, double* zi_inout, float* y);

/* fmDemodArctan(I, Q, prev_phase): model/fmSupportLib.py:15-44
 * (C++: src/rf_module.cpp:13-34, which is a non-arctan approximation; this follows
 * the Python model).  prev_phase in/out (NULL = 0.0, no state out). */
int sdr_fm_demod(sdr_ctx* ctx, const float* I, const float* Q, int64_t n, double* prev_phase,
                 float* out);

/* fmPll(pllIn, freq, Fs, state, ncoScale, phaseAdjust, normBandwidth):
 * model/fmPll.py:4-46 (C++ src/helper.cpp:13-57 fmPLL, src/helper.h:17-19 state).
 * state6 = [integrator, phaseEst, feedbackI, feedbackQ, ncoOut[0], trigOffset], in/out.
 * nco_i/nco_q: n+1 floats (index 0 = carried value); nco_q may be NULL. */
int sdr_pll(sdr_ctx* ctx, const float* in, int64_t n, double freq, double fs, double nco_scale,
            double phase_adj, double norm_bw, double* state6, float* nco_i, float* nco_q);

/* How the context's PLL calls were solved (device counters, accumulated since the context was
 * created or last reset; sdr_pll*, and the receivers built on the context).  A recurrence is
 * one (stream, PLL) of a call, or one pseudo-block of a long call (n > SDR_PLL_BLOCK_MAX =
 * 16 385 samples, which is cut into pseudo-blocks solved in parallel and chained).
 *   RECURRENCES   recurrences solved
 *   SPEC_R0..R2   ... by the parallel solve (guess + scan + check) in its 1st / 2nd / 3rd round
 *   SEQUENTIAL    ... by the sequential kernel (the fallback: acquisition, 0 / NaN input)
 *   LONG_GUESSED  long calls: pseudo-blocks kept as solved from their pre-roll start guess
 *                 (start within the acceptance bound of the chained state after a 2 pi shift)
 *   LONG_CHAINED  long calls: pseudo-blocks completed from the start the chain computed (the
 *                 linear response to the start error added, or solved again from it)
 *   LONG_MAXGAP   largest bound on the phase deviation between a pseudo-block's solved start
 *                 and the chained state among those kept as solved (radians, the bits of an f64)
 *   LONG_STOPS    long calls: pseudo-blocks whose start guess was beyond the linear bound (the
 *                 chain stopped there that round and re-solved it from the exact start)
 *   LONG_TAIL     long calls: pseudo-blocks left after the rounds, solved sequentially from the
 *                 chain's exact position (also counted in SEQUENTIAL)
 *   LONG_LINEAR   long calls: pseudo-blocks completed by the linear response to their start
 *                 error (every step's wrap further than the deviation bound: also in CHAINED)
 * out: SDR_PLL_NSTATS int64 (LONG_MAXGAP: reinterpret as double).  Synchronises the context
 * stream; reset != 0 zeroes the counters after reading. */
enum {
  SDR_PLL_ST_RECURRENCES, SDR_PLL_ST_SPEC_R0, SDR_PLL_ST_SPEC_R1, SDR_PLL_ST_SPEC_R2, SDR_PLL_ST_SEQUENTIAL,
  SDR_PLL_ST_LONG_GUESSED, SDR_PLL_ST_LONG_CHAINED, SDR_PLL_ST_LONG_MAXGAP, SDR_PLL_ST_LONG_STOPS,
  SDR_PLL_ST_LONG_TAIL, SDR_PLL_ST_LONG_LINEAR, SDR_PLL_NSTATS
};
int sdr_pll_stats(sdr_ctx* ctx, int64_t* out, int reset);

/* Fused mono block: RF front end + audio lfilter + [::audio_decim], intermediate demod
 * kept in HBM.  Replaces the body of model/fmMonoBlock.py:80-109 (one loop
 * iteration) and src/fm_radio.cpp:66-84 + :258.  demod_out optional. */
int sdr_mono_block(sdr_ctx* ctx, const void* iq, int iq_dtype, int64_t n, const double* rf_b,
                   int rf_taps, int rf_decim, double* zi_i, double* zi_q, double* prev_phase,
                   const double* audio_b, int audio_taps, int audio_decim, double* audio_zi,
                   float* demod_out, float* audio_out);

/* ================================================================================
 * Device-pointer entry points (asynchronous on the context stream)
 * Batched over `nstreams` independent streams laid out `stride` elements apart.
 * `hist` = number of valid samples in memory before each stream's index 0 (0: zero
 * pre-history as lfilter).  zf may alias zi (handled through scratch).
 * ================================================================================ */
int sdr_rf_frontend_dev(sdr_ctx* ctx, const void* iq, int iq_dtype, int64_t n, int64_t stride,
                        int64_t hist, int nstreams, const double* b, int taps, int decim,
                        const double* zi_i, const double* zi_q, int64_t zi_stride, double* zf_i,
                        double* zf_q, double* prev_phase, float* demod, int64_t out_stride,
                        float* i_ds, float* q_ds);

/* Fused continuous-stream mono receiver: per stream,
 *   audio = lfilter(audio_b, 1, fmDemodArctan(lfilter(rf_b, 1, I)[::rf_decim],
 *                                             lfilter(rf_b, 1, Q)[::rf_decim]))[::audio_decim]
 * with zero initial filter/demod state -- model/fmMonoBasic.py:70-111 (whole-signal mono
 * path; per block: model/fmMonoBlock.py:86-105, src/fm_radio.cpp:66-84).  The demodulated
 * stream stays on chip (f32 IQ, rf_taps 101/151 at decim 10, audio 151 taps at decim 5);
 * other configurations run the front end into scratch HBM, then the audio filter.
 * audio: nstreams x audio_stride floats, ceil(ceil(n/rf_decim)/audio_decim) per stream. */
/* 1 if sdr_fe_mono_dev runs the single fused kernel for this configuration (16-B aligned f32
 * / 4-B aligned u8 IQ rows, even stride), 0 if it runs the front end + audio FIR pair. */
int sdr_fe_mono_fused(int rf_taps, int rf_decim, int audio_taps, int audio_decim);
int sdr_fe_mono_dev(sdr_ctx* ctx, const void* iq, int iq_dtype, int64_t n, int64_t stride, int nstreams,
                    const double* rf_b, int rf_taps, int rf_decim, const double* audio_b, int audio_taps,
                    int audio_decim, float* audio, int64_t audio_stride);

int sdr_fir_dev(sdr_ctx* ctx, const float* x, const float* mix, float gain, int pre, int64_t n,
                int64_t x_stride, int64_t hist, int nstreams, const double* b, int taps, int decim,
                const double* zi, int64_t zi_stride, double* zf, float* y, int64_t y_stride);

int sdr_resample_dev(sdr_ctx* ctx, const float* x, int64_t n, const double* b, int taps, int up,
                     int down, const double* zi, double* zf, float* y);

int sdr_fm_demod_dev(sdr_ctx* ctx, const float* I, const float* Q, int64_t n, int64_t stride,
                     int nstreams, double* prev_phase, float* out, int64_t out_stride);

int sdr_pll_dev(sdr_ctx* ctx, const float* in, int64_t n, int64_t in_stride, int nstreams,
                double freq, double fs, double nco_scale, double phase_adj, double norm_bw,
                double* state, float* nco_i, float* nco_q, int64_t out_stride);

/* Stereo combiner, intended form of model/fmMonoBlock.py:166-170 (as in
 * src/fm_radio.cpp:250-251): left = (mono+side)/2, right = (mono-side)/2. */
int sdr_stereo_combine_dev(sdr_ctx* ctx, const float* mono, const float* side, int64_t n,
                           float* left, float* right);

/* ---- multi-stream block receiver ----------------------------------
 * The per-block loops of model/fmMonoBlock.py:80-173 (mono, stereo; intended L/R combiner)
 * and model/fmRDSblock.py:127-204 (RDS up to the RRC output) for `nstreams` independent
 * streams at once, every filter state, demod phase and PLL state carried in HBM from block
 * to block (C++: the rf / mono_stereo / rds threads of src/fm_radio.cpp:31-441, 783-792).
 * One block of all streams is a fixed chain of ~10 launches on the context stream,
 * whatever nstreams is: the FE, one launch per stage for all filters of that stage (with
 * their lfilter final states), and one lane per PLL recurrence.
 *   flags: SDR_RX_AUDIO (mono audio), SDR_RX_STEREO (implies AUDIO), SDR_RX_RDS.
 *   Filters (taps f64, designed by the caller, <= SDR_MAX_TAPS, set before the first block):
 *   SDR_RX_F_RF (+ rf_decim), F_AUDIO (+ audio_decim), F_PILOT, F_STEREO_BPF, F_STEREO_LPF
 *   (decim audio_decim), F_RDS_EXTRACT, F_RDS_SQUARE, F_RDS_LPF, F_RDS_ANTI (on the
 *   x rds_up zero-stuffed stream, then [::rds_down] x rds_up), F_RDS_RRC.
 *   PLLs default to the reference's: stereo 19 kHz x2 BW 0.01 (fmMonoBlock.py:119), RDS
 *   114 kHz x0.5 phase pi/3.3-pi/1.5 BW 0.001 (fmRDSblock.py:167), both at Fs 240 kHz.
 * Outputs live in receiver-owned device memory, `stride` floats apart per stream, and are
 * overwritten by the next block: M = ceil(block/rf_decim) demod-rate samples (NCOs: M+1,
 * index 0 = the carried value), A = ceil(M/audio_decim) audio-rate, R = ceil(M*up/down)
 * RDS-rate.  Inputs: nstreams rows of `block` interleaved complex samples, iq_stride
 * complex samples apart (f32 or u8). */
typedef struct sdr_rx sdr_rx;
enum { SDR_RX_AUDIO = 1, SDR_RX_STEREO = 2, SDR_RX_RDS = 4 };
enum {
  SDR_RX_F_RF, SDR_RX_F_AUDIO, SDR_RX_F_PILOT, SDR_RX_F_STEREO_BPF, SDR_RX_F_STEREO_LPF,
  SDR_RX_F_RDS_EXTRACT, SDR_RX_F_RDS_SQUARE, SDR_RX_F_RDS_LPF, SDR_RX_F_RDS_ANTI, SDR_RX_F_RDS_RRC,
  SDR_RX_NFILTERS
};
enum {
  SDR_RX_O_DEMOD, SDR_RX_O_AUDIO,                                   /* fm_demod, audio_block */
  SDR_RX_O_BPF_RECOVERY, SDR_RX_O_STEREO_NCO, SDR_RX_O_BPF_EXTRACTION, SDR_RX_O_STEREO,
  SDR_RX_O_LEFT, SDR_RX_O_RIGHT,                                    /* fmMonoBlock.py:115-170 */
  SDR_RX_O_RDS_EXTRACT, SDR_RX_O_RDS_PRE_PLL, SDR_RX_O_RDS_NCO_I, SDR_RX_O_RDS_NCO_Q,
  SDR_RX_O_RDS_LPF_I, SDR_RX_O_RDS_LPF_Q, SDR_RX_O_RDS_RES_I, SDR_RX_O_RDS_RES_Q,
  SDR_RX_O_RDS_RRC_I, SDR_RX_O_RDS_RRC_Q,                           /* fmRDSblock.py:156-204 */
  SDR_RX_NOUTPUTS
};
int sdr_rx_create(sdr_ctx* ctx, int nstreams, int64_t block, int iq_dtype, int flags, sdr_rx** out);
void sdr_rx_destroy(sdr_rx* rx);
int sdr_rx_set_filter(sdr_rx* rx, int which, const double* b, int taps);
int sdr_rx_set_decim(sdr_rx* rx, int rf_decim, int audio_decim, int rds_up, int rds_down);
int sdr_rx_set_pll(sdr_rx* rx, int which /* 0 stereo, 1 RDS */, double freq, double fs,
                   double nco_scale, double phase_adj, double norm_bw);
int sdr_rx_reset(sdr_rx* rx);                       /* all states back to the stream start */
int sdr_rx_process_dev(sdr_rx* rx, const void* iq, int64_t iq_stride);   /* async, device IQ */
int sdr_rx_process(sdr_rx* rx, const void* iq, int64_t iq_stride);       /* sync, host IQ */
/* sync, host IQ in and the `nout` requested outputs (which[i]: SDR_RX_O_*) out into
 * out[i] (nstreams rows, out_stride[i] floats apart; NULL out_stride = packed), through
 * pinned staging with one wait: the per-block drop-in call of fmMonoBlock.py's loop */
int sdr_rx_run(sdr_rx* rx, const void* iq, int64_t iq_stride, int nout, const int* which,
               float* const* out, const int64_t* out_stride);
/* The same without waiting for the block: the IQ is copied into one of two pinned slots and
 * the chain is launched; then the PREVIOUSLY submitted block is waited for and its outputs
 * written into the buffers given with it, and the call returns (so the host prepares block
 * k+1 while block k runs: the reference's rf / audio thread overlap, src/fm_radio.cpp:783-792).
 * The `out` buffers must stay valid until the next sdr_rx_submit / sdr_rx_flush / sdr_rx_run
 * returns.  sdr_rx_flush delivers the last submitted block.  nout <= SDR_RX_MAXOUT. */
enum { SDR_RX_MAXOUT = 32 };
int sdr_rx_submit(sdr_rx* rx, const void* iq, int64_t iq_stride, int nout, const int* which,
                  float* const* out, const int64_t* out_stride);
int sdr_rx_flush(sdr_rx* rx);
/* Submission depth (set before the first block; 1..3, default 1): sdr_rx_submit of block k
 * delivers block k-depth (not k-1), so `depth` blocks stay in flight while the host prepares
 * the next one -- the reference's RF thread running ahead of its audio thread through its
 * queue (src/fm_radio.cpp:783-792).  sdr_rx_flush delivers every block still in flight,
 * oldest first.  With depth >= 2 a pipelined receiver keeps three output row sets (block k's
 * rows stay valid until block k+3 is processed). */
int sdr_rx_set_depth(sdr_rx* rx, int depth);
/* Pipelined receiver (set before the first block): block k's front half (FE and the
 * filters of the demod) runs on a second stream, its PLLs on a third once block k-1's PLLs
 * are done, and its stereo / RDS stages on the context stream -- so block k's PLLs start
 * while block k-1's stages C-E and block k+1's front half run; the output rows alternate
 * between two sets
 * (sdr_rx_output gives the latest block's; block k's stay valid until block k+2 is
 * processed).  sdr_rx_process_dev then does NOT order the front half after earlier work on
 * the context stream: its IQ must be ready when it is called (device-resident data, or an
 * upload that has been waited for).  The back half and everything after it on the context
 * stream see block k complete, as without pipelining. */
int sdr_rx_set_pipeline(sdr_rx* rx, int on);
int sdr_rx_output(sdr_rx* rx, int which, float** dev, int64_t* stride, int64_t* n);
int sdr_rx_fetch(sdr_rx* rx, int which, float* host, int64_t host_stride); /* sync, all streams */
/* Outputs sdr_rx_process_dev materialises (bit 1 << SDR_RX_O_*; default: every output of the
 * flags).  The NCO rows (SDR_RX_O_STEREO_NCO, _RDS_NCO_I/_Q) and the RDS LPF rows (_RDS_LPF_I/_Q)
 * are intermediates the chain itself does not need: without them the mixers form the NCO
 * from the PLL phases where they stage their inputs and the RDS LPF runs inside the composite
 * LPF + x19/80 resampler, so neither round-trips through HBM.  On spans (rows of >= 32 768
 * demod samples, the matrix-core tiles) the PLLs' f32 input rows (SDR_RX_O_BPF_RECOVERY,
 * _RDS_PRE_PLL) are such intermediates too: the loops read their inputs as one sign-code
 * byte per sample, which the producing tiles always store (the other outputs, which later
 * stages read, are always written; every output's values are the same either way).
 * sdr_rx_run / sdr_rx_submit materialise what they are asked for.  sdr_rx_fetch of an output
 * the latest block did not materialise is SDR_EINVAL (sdr_rx_output still gives its row). */
int sdr_rx_set_keep(sdr_rx* rx, uint64_t mask);
/* per-stage timing of the last block (HIP events between the receiver's launches, on the
 * context stream): FE, stage A (filters of demod), B (RDS square), PLL, C (mixers + LPFs),
 * D (resamplers), E (RRC); ms: SDR_RX_NSTAGES floats.  Timing adds event records between
 * launches; keep it off in measured loops. */
enum { SDR_RX_ST_FE, SDR_RX_ST_A, SDR_RX_ST_B, SDR_RX_ST_PLL, SDR_RX_ST_C, SDR_RX_ST_D, SDR_RX_ST_E,
       SDR_RX_NSTAGES };
int sdr_rx_set_timing(sdr_rx* rx, int on);
int sdr_rx_stage_ms(sdr_rx* rx, float* ms);
/* carried states (host copies; any may be NULL): demod prev_phase [nstreams], PLL states
 * [nstreams][6] in fmPll's order (model/fmPll.py:39-44) */
int sdr_rx_state(sdr_rx* rx, double* phase, double* pll_stereo, double* pll_rds);
/* sdr_pll_stats of the receiver's context, after waiting for every block in flight */
int sdr_rx_pll_stats(sdr_rx* rx, int64_t* out, int reset);

/* ---- spectral diagnostics -----------------------------------------
 * Bartlett PSD, model/fmSupportLib.py:66-140 (estimatePSD; the C++ src/fourier.cpp:36-110
 * advances sample and list positions by the same nfft/2 and is not the parity target):
 * floor(n/nfft) non-overlapping segments, Hann window pow(sin(i*pi/nfft), 2), FFT in f64,
 * 10*log10(2/(fs*nfft/2) * |X_k|^2) for k < nfft/2, averaged over segments in dB.
 * psd: nfft/2 doubles (NaN when n < nfft, as the reference's 0/0).  nfft: a power of two in
 * [2, SDR_PSD_MAX_NFFT = 4096].  SDR_EDOMAIN if a bin has zero power (the reference's
 * math.log10 raises).  The frequency axis np.arange(0, fs/2, fs/nfft) is the caller's.
 * sdr_psd: host f64 samples.  sdr_psd_dev: device samples (SDR_REAL_F32 / _F64), device psd. */
int sdr_psd(sdr_ctx* ctx, const double* x, int64_t n, int nfft, double fs, double* psd);
int sdr_psd_dev(sdr_ctx* ctx, const void* x, int dtype, int64_t n, int nfft, double fs, double* psd);

/* Direct DFT, model/fmSupportLib.py:46-60: X_m = sum_k x_k exp(i*2*pi*(-k*m)/n), f64, the
 * angle rounded as the reference's expression rounds it.  X: 2n doubles (re, im
 * interleaved = numpy complex128).  n <= SDR_DFT_MAX_N. */
int sdr_dft(sdr_ctx* ctx, const double* x, int64_t n, double* X);

/* ---- RDS link layer (host code) -----------------------------------
 * model/fmRDSblock.py:207-346 (src/fm_radio.cpp:444-729 frame_thread): per block of the
 * in-phase RRC output (57 kS/s, 24 samples per symbol), clock and data recovery from a
 * carried symbol offset, Manchester decoding of symbol pairs (with the carried lone
 * symbol), differential decoding, and the syndrome scan of every 26-bit window.
 * events: 3 int64 per syndrome match {type 0..3 = A..D, position, accepted}, where
 * accepted = 1 for the reference's "Syndrome X at position N" prints and 0 for its
 * "False positive" prints; positions count across blocks as the reference's printposition.
 * symbols / bits / diff (optional, NULL to skip): the sampled symbols, the Manchester bits
 * and the bits the scan saw (carried bits first), each count written to n_*.
 * The state (offset, start position, lone symbol, previous bit, carried bits, positions)
 * lives in the sdr_rds_link object; one object per stream.  No GPU is used. */
typedef struct sdr_rds_link sdr_rds_link;
enum { SDR_RDS_RESYNC = 4 };   /* event type of a re-sync (only with sdr_rds_link_set_resync) */
int sdr_rds_link_create(sdr_rds_link** out);
void sdr_rds_link_destroy(sdr_rds_link* link);
/* The C++ frame_thread's re-sync rule (src/fm_radio.cpp:697-704): after more than
 * `after_bad_syncs` false-positive syndromes since the last accepted one, forget the frame
 * position (the next syndrome is accepted) and emit an SDR_RDS_RESYNC event.  0 (default):
 * off, as the Python model (model/fmRDSblock.py:299-341), which has no such rule; the C++
 * uses 10. */
int sdr_rds_link_set_resync(sdr_rds_link* link, int after_bad_syncs);
int sdr_rds_link_block(sdr_rds_link* link, const double* rrc_i, int64_t n, int64_t* events,
                       int64_t max_events, int64_t* n_events, double* symbols, int64_t max_symbols,
                       int64_t* n_symbols, uint8_t* bits, int64_t max_bits, int64_t* n_bits,
                       uint8_t* diff, int64_t max_diff, int64_t* n_diff);

#ifdef __cplusplus
}
#endif
#endif /* SDR_H_ */
