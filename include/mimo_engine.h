/* mimo_engine.h -- C ABI of the MI355X Monte-Carlo BER engine (libmimo_engine.so).
 *
 * This is the drop-in boundary for the reference's hot path
 * (MarcinWachowiak/m-mimo-ofdm-with-nonlinear-pa-sim).  The reference is pure Python
 * with no FFI; the entry points below are what its object API binds to through ctypes
 * (see INTEGRATION.md), one group per reference seam:
 *
 *   coarse seam  mp_model.Link                    mp_model.py:32-329
 *     mimo_engine_create        <- Link.__init__                       mp_model.py:32-87
 *     mimo_engine_set_point     <- Link.update_distortion / set_snr    mp_model.py:230-251
 *     mimo_engine_run           <- Link.simulate (trial loop)          mp_model.py:89-228
 *     mimo_engine_run_points    <- the drivers' grid loops over (IBO, Eb/N0), one launch
 *                                  for many points   main_mp_miso_cnc_constant_ber_req_ebn0_vs_ibo.py:100-215
 *   fine seams (float64 stage kernels, caller-owned host arrays)
 *     mimo_qam_map              <- modulation.modulate                 modulation.py:13-25
 *     mimo_qam_slice            <- demodulate / symbol_detection       modulation.py:63-88,138-146
 *     mimo_qam_llr              <- soft_decoding                       modulation.py:29-59
 *     mimo_ofdm_tx / _rx        <- _tx_ofdm_symbol / _rx_ofdm_symbol   modulation.py:248-293
 *     mimo_fft                  <- utilities.to_freq/time_domain       utilities.py:311-339
 *     mimo_pa                   <- SoftLimiter/Rapp/ThirdOrderNonLin.process  distortion.py
 *     mimo_calc_alpha           <- Modem.calc_alpha                    modulation.py:178-189
 *     mimo_mrt_precode          <- AntennaArray.set_precoding_matrix   antenna_array.py:162-185
 *     mimo_combine              <- Miso*Fd.propagate                   channel.py:74-89,277-292
 *     mimo_awgn                 <- Awgn.process                        noise.py:45-83
 *     mimo_count_bit_errors     <- utilities.count_mismatched_bits     utilities.py:94-104
 *     mimo_cnc_receive          <- CncReceiver.receive                 corrector.py:52-112
 *     mimo_cnc_receive_ex       <- CncReceiver.receive(return_bits=False) corrector.py:80-84
 *
 * Conventions: complex arrays are interleaved (re, im) doubles; sizes are element
 * counts; functions return 0 on success and a negative MIMO_E* code on error, with a
 * message from mimo_last_error() (thread-local).  No HIP call happens before the first
 * compute call, so a Python parent may create engines and fork workers (the
 * reference's drivers fork after building Link, main_mp_miso_cnc_ber_vs_ebn0.py:124-132).
 */
#ifndef MIMO_ENGINE_H
#define MIMO_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIMO_ABI_VERSION 8

enum { MIMO_OK = 0, MIMO_EINVAL = -1, MIMO_EHIP = -2, MIMO_ENOKERNEL = -3, MIMO_ENOMEM = -4 };
enum { MIMO_PA_NONE = 0, MIMO_PA_SOFTLIM = 1, MIMO_PA_RAPP = 2, MIMO_PA_TOI = 3 };
enum { MIMO_CH_RAYLEIGH = 1, MIMO_CH_LOS = 2, MIMO_CH_TWOPATH = 3, MIMO_CH_TABLE = 4 };
enum { MIMO_RX_CNC = 1, MIMO_RX_MCNC = 2 };
enum { MIMO_PREC_F64 = 0, MIMO_PREC_F32 = 1 };

typedef struct mimo_engine mimo_engine;

/* System description: everything Link deep-copies at construction.  Arrays are copied. */
typedef struct mimo_config {
  int32_t n_ant;            /* antennas (AntennaArray.n_elements)                   */
  int32_t n_sub_carr;       /* data sub-carriers S (multiple of 4, S <= n_fft - 2)  */
  int32_t n_fft;            /* FFT size F: power of two, 128 ... 8192               */
  int32_t constel_size;     /* square QAM order M (4 ... 4096)                      */
  int32_t cp_len;           /* cyclic prefix (BER-neutral: memoryless PA, circular channel) */
  int32_t channel_kind;     /* MIMO_CH_* (TABLE: a fixed matrix, see chan_table)     */
  int32_t receiver_kind;    /* MIMO_RX_*                                            */
  int32_t device;           /* HIP device ordinal, -1 = current                      */
  double rx_pos[3];         /* nominal RX position [m]                               */
  double rx_loc_var;        /* LoS / two-path RX jitter span [m] (mp_model.py:192-199) */
  int32_t reroll_chan;      /* 1: per-trial channel reroll (Link.simulate reroll_chan) */
  int32_t precision;        /* MIMO_PREC_F64 (0, default: the reference's complex128 /
                               float64, modulation.py:270) or MIMO_PREC_F32 (fast variant) */
  const double* tx_pos;     /* [n_ant][3] antenna positions [m]                      */
  const double* carrier_freqs; /* [n_fft] carrier frequencies [Hz] in FFT-bin order  */
  const double* chan_table; /* MIMO_CH_TABLE only: [n_ant][n_fft] complex channel matrix
                               (Miso*Fd.channel_mat_fd), the same for every trial -- what
                               Link.simulate(reroll_chan=False) uses (mp_model.py:190-206) */
  int32_t chan_replay_period; /* 0 (default): an independent Rayleigh channel per trial.
                               > 0 (diagnostic, Rayleigh only): trial i draws the channel of
                               trial i mod period, emulating the reference's workers that all
                               replay one seeded channel sequence (channel.py:209-212);
                               bits and noise stay per trial.  Used to size the published
                               curves' channel variance (tests/test_gpu_link.py).  (ABI 5) */
  uint64_t csi_seed;        /* MIMO_CH_TABLE with CSI error: Philox key of the one erroneous
                               estimate every trial and every run shares -- Link.__init__ draws it
                               once from its noise generator, default_rng(0) (mp_model.py:74,87,272), so the
                               workers of a point see the same estimate whatever their seeds.
                               0: the run's seed (ABI 5 behaviour).  (ABI 6) */
} mimo_config;

/* Grid-point parameters: what Link keeps in its PA / receiver / noise objects. */
typedef struct mimo_point {
  double ibo_db;            /* IBO used by the per-antenna Bussgang AGC (mp_model.py:315-317) */
  double snr_db;            /* Link.set_snr value                                    */
  double avg_symbol_power;  /* Es = mean |C|^2 (modulation.py:218)                    */
  int32_t pa_kind;          /* array PA model                                        */
  int32_t cnc_pa_kind;      /* CNC receiver's PA copy                                */
  double sat_pow;           /* array PA saturation power (softlim / rapp)            */
  double p_hardness;        /* Rapp p                                                */
  double toi_coeff;         /* array PA cubic coefficient (toi)                      */
  double cnc_sat_pow;       /* CNC PA saturation power                                */
  double cnc_toi_coeff;     /* CNC PA cubic coefficient                               */
  double cnc_alpha;         /* CNC alpha (corrector.py:106-110)                      */
  double csi_eps;           /* CSI error epsilon; < 0 = perfect CSI.  With CSI error: n_ant <= 512,
                               and the run fails with MIMO_EINVAL (before any launch) if the
                               instance's static LDS plus the n_ant-real power table exceed the
                               CU's LDS (round 6)                                    */
  double array_alpha;       /* 0: each antenna's Bussgang gain from its precoding power
                               (Link, mp_model.py:315-317).  > 0: that gain for every antenna --
                               the TOI drivers' measured alpha_estimate
                               (main_miso_cnc_ber_vs_ebn0_toi.py:95-121,247-249).  Not with the
                               float32 F = 8192 instance (MIMO_EINVAL).  (ABI 8) */
} mimo_point;

int32_t mimo_abi_version(void);
const char* mimo_last_error(void);
int32_t mimo_device_count(void);

/* Coarse seam ------------------------------------------------------------------- */
mimo_engine* mimo_engine_create(const mimo_config* cfg);
int32_t mimo_engine_set_point(mimo_engine* e, const mimo_point* pt);
/* Runs trials [first_trial, first_trial + n_trials) of the point, keyed by `seed`.
 * iters: sorted, unique receiver iterations to record (0 = standard RX), each in [0, 31].
 * Counter layout (mp_model.py:127-131,217-222): [clean if incl_clean] + one per iter.
 * err_out / bits_out: n_idx totals (ADDED to, like the reference's shared counters).
 * per_trial: optional [n_trials][n_idx] bit-error counts, NULL to skip. */
int32_t mimo_engine_run(mimo_engine* e, uint64_t seed, uint64_t first_trial, uint64_t n_trials,
                        const int32_t* iters, int32_t n_iters, int32_t incl_clean,
                        uint64_t* err_out, uint64_t* bits_out, uint32_t* per_trial);
/* Many grid points of the same system in one go (BASELINE config 4 sweeps): point i runs
 * trials [first_trial[i], first_trial[i] + n_trials[i]) keyed by seeds[i] with the
 * parameters points[i].  Every point's trials are a contiguous block range of one kernel
 * launch (launches hold up to 2^20 trials), so a grid of small points fills the GPU.
 * All points share iters / incl_clean and must agree on CSI error on / off.
 * err_out / bits_out: [n_points][n_idx] totals (ADDED to).  per_trial: optional
 * [sum n_trials][n_idx] counts in point order, NULL to skip.  mimo_engine_run(...) is
 * this call with the engine's current point. */
int32_t mimo_engine_run_points(mimo_engine* e, int32_t n_points, const mimo_point* points, const uint64_t* seeds,
                               const uint64_t* first_trial, const uint64_t* n_trials, const int32_t* iters,
                               int32_t n_iters, int32_t incl_clean, uint64_t* err_out, uint64_t* bits_out,
                               uint32_t* per_trial);
/* Device time of the trial kernels of the last run, in ms (HIP events on the engine stream). */
double mimo_engine_last_kernel_ms(const mimo_engine* e);
/* Which kernel instance the current config selects: "F=2048 T=128 slots=8 aligned ..." */
const char* mimo_engine_describe(const mimo_engine* e);
void mimo_engine_destroy(mimo_engine* e);

/* Fine seams (float64) ------------------------------------------------------------ */
int32_t mimo_qam_map(int32_t constel_size, const int32_t* labels, int64_t n, double* out_iq);
int32_t mimo_qam_slice(int32_t constel_size, const double* in_iq, int64_t n, int32_t* labels_out);
int32_t mimo_qam_llr(int32_t constel_size, const double* in_iq, int64_t n, const double* noise_var, double* llr_out);
int32_t mimo_fft(int32_t n_fft, int64_t batch, int32_t inverse, const double* in_iq, double* out_iq);
int32_t mimo_ofdm_tx(int32_t n_fft, int32_t n_sub_carr, int32_t cp_len, int64_t batch, const double* sym_iq,
                     double* td_iq);
int32_t mimo_ofdm_rx(int32_t n_fft, int32_t n_sub_carr, int32_t cp_len, int64_t batch, const double* td_iq,
                     double* sym_iq);
int32_t mimo_pa(int32_t kind, double sat_pow, double p_hardness, double toi_coeff, const double* in_iq, int64_t n,
                double* out_iq);
/* Bussgang gain alpha(IBO) for n IBO values [dB], by the trial kernel's segment table
 * (alpha_fit.h: the float64 kernels' alpha for antennas outside the per-point fit).  (ABI 6) */
int32_t mimo_calc_alpha(const double* ibo_db, int64_t n, double* out);
int32_t mimo_mrt_precode(int32_t n_ant, int32_t n_cols, const double* h_iq, double* p_iq);
int32_t mimo_combine(int32_t n_ant, int64_t n, const double* h_iq, const double* y_iq, double* out_iq);
int32_t mimo_awgn(uint64_t seed, uint64_t counter, int64_t n, double noise_std, const double* in_iq, double* out_iq);
int32_t mimo_count_bit_errors(const int64_t* a, const int64_t* b, int64_t n, int64_t* out);
int32_t mimo_cnc_receive(int32_t constel_size, int32_t n_fft, int32_t n_sub_carr, int32_t pa_kind, double sat_pow,
                         double p_hardness, double toi_coeff, double alpha, const int32_t* iters, int32_t n_iters,
                         const double* in_sc_iq, int32_t* labels_out);
/* ABI 7: the same loop with optional outputs -- labels_out [n_iters][S] and/or
 * corrected_iq_out [n_iters][S] (re, im), the slicer input rx - d of each listed iteration,
 * which CncReceiver.receive(return_bits=False) returns (corrector.py:80-84).  Either may be
 * null. */
int32_t mimo_cnc_receive_ex(int32_t constel_size, int32_t n_fft, int32_t n_sub_carr, int32_t pa_kind, double sat_pow,
                            double p_hardness, double toi_coeff, double alpha, const int32_t* iters, int32_t n_iters,
                            const double* in_sc_iq, int32_t* labels_out, double* corrected_iq_out);

#ifdef __cplusplus
}
#endif
#endif /* MIMO_ENGINE_H */
