/*
 * uhsdr.h -- C ABI of the MI355X-native UHSDR RX DSP hot path (libuhsdr_amd.so).
 *
 * Drop-in boundary for the reference firmware's per-block receive chain
 * (SURVEY.md §8(b)):
 *
 *   reference                                             this ABI
 *   ---------------------------------------------------   --------------------------------
 *   AudioDriver_SetProcessingChain(dmod_mode, reset)      uhsdr_rx_plan_build()  (host setup,
 *     drivers/audio/audio_driver.c:1093-1251                restates the chain selection,
 *   AudioFilter_SetRxHilbertAndDecimationFIR()              filter tables, biquad designers
 *     drivers/audio/audio_filter.c:1134-1223                and AGC parameter math)
 *   AudioAgc_SetupAgcWdsp(rate, remove_dc)
 *     drivers/audio/audio_agc.c:126-339
 *   AudioDriver_Init() + SetProcessingChain()             uhsdr_rx_create() / uhsdr_rx_reset()
 *     audio_driver.c:677-704                                (zeroes all per-channel state)
 *   AudioDriver_I2SCallback(audio, iq, dst, 32)           uhsdr_rx_process()  -- C channels x
 *     audio_driver.c:2962-3049 ->                           N frames per call, N % 32 == 0,
 *   AudioDriver_RxProcessor(iq, audio, 32, mute)            one call == N/32 consecutive ISR
 *     audio_driver.c:2603-2942                              invocations on every channel
 *
 * Buffers follow the firmware's DMA formats, channel-major:
 *   iq    : IqSample_t    {int32 l (I), int32 r (Q)}  [C][N]  (audio_driver.h:44-52)
 *   audio : float         adb.a_buffer[1]             [C][N]  (audio_driver.h:147-157)
 *   dst   : AudioSample_t {int32 l, int32 r}           [C][N]  codec frames (audio_driver.c:2911-2923)
 * Device pointers are HIP device allocations.  Status codes follow CMSIS arm_status
 * (CMSIS/Include/arm_math.h:375-382): 0 success, -1 argument error, -2 length error.
 *
 * Threading: a handle is not re-entrant (like the ISR, audio_driver.c:1804-1806); calls on
 * one handle are ordered on the handle's HIP stream.  Different handles are independent.
 */
#ifndef UHSDR_H
#define UHSDR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UHSDR_ABI_VERSION 5

typedef enum
{
    UHSDR_OK = 0,                 /* ARM_MATH_SUCCESS */
    UHSDR_ARGUMENT_ERROR = -1,    /* ARM_MATH_ARGUMENT_ERROR */
    UHSDR_LENGTH_ERROR = -2,      /* ARM_MATH_LENGTH_ERROR: N % 32 != 0, bad sizes */
    UHSDR_UNSUPPORTED = -10,      /* mode / filter path not implemented on the device yet */
    UHSDR_DEVICE_ERROR = -11,     /* HIP runtime error */
    UHSDR_TIMEOUT = -12           /* a bounded device-side poll gave up (the pipelined device hand-off,
                                     uhsdr_rx_set_pipelined 2): outputs and handle state are invalid
                                     until uhsdr_rx_reset */
} uhsdr_status;

/* sam_sideband_t, drivers/audio/audio_driver.h:181-190 (STEREO: USE_TWO_CHANNEL_AUDIO, OVI40) */
enum { UHSDR_SAM_SIDEBAND_BOTH = 0, UHSDR_SAM_SIDEBAND_LSB = 1, UHSDR_SAM_SIDEBAND_USB = 2,
       UHSDR_SAM_SIDEBAND_STEREO = 3 };

/* DemodModes_t, hardware/uhsdr_board.h:72-85 (SSBSTEREO / IQ: USE_TWO_CHANNEL_AUDIO, OVI40) */
enum { UHSDR_DEMOD_USB = 0, UHSDR_DEMOD_LSB = 1, UHSDR_DEMOD_CW = 2, UHSDR_DEMOD_AM = 3,
       UHSDR_DEMOD_SAM = 4, UHSDR_DEMOD_FM = 5, UHSDR_DEMOD_DIGI = 6, UHSDR_DEMOD_SSBSTEREO = 7,
       UHSDR_DEMOD_IQ = 8 };

/* FREQ_IQ_CONV_*, drivers/audio/audio_driver.h:520-526 */
enum { UHSDR_IQ_CONV_OFF = 0, UHSDR_IQ_CONV_P6KHZ = 1, UHSDR_IQ_CONV_M6KHZ = 2,
       UHSDR_IQ_CONV_P12KHZ = 3, UHSDR_IQ_CONV_M12KHZ = 4 };

/* ts.dsp.active bits honoured by the chain (drivers/audio/audio_driver.h:195-200) */
#define UHSDR_DSP_NOTCH_ENABLE  0x04      /* LMS auto notch (AudioDriver_NotchFilter) */
#define UHSDR_DSP_MNOTCH_ENABLE 0x10
#define UHSDR_DSP_MPEAK_ENABLE  0x20

#define UHSDR_IQ_BLOCK_SIZE 32        /* IQ_BLOCK_SIZE, hardware/uhsdr_board_config.h:217 */
#define UHSDR_FILTER_PATH_NUM 87      /* AUDIO_FILTER_PATH_NUM, audio_filter.h:139 */
#define UHSDR_MAX_FIR_TAPS 200        /* IQ_RX_NUM_TAPS_MAX (199 rounded) */
#define UHSDR_MAX_DEC_TAPS 96         /* 89-tap AM tables reused as decimator */
#define UHSDR_MAX_LATTICE 10          /* IIR_RXAUDIO_NUM_STAGES_MAX */
#define UHSDR_MAX_INTERP 16
#define UHSDR_AGC_RING 192            /* AGC_WDSP_RB_SIZE, audio_agc.c:19 */

/*
 * User-facing receiver configuration: the subset of TransceiverState `ts` /
 * AudioDriverState `ads` / agc_wdsp_conf that the RX chain reads.  Defaults
 * (uhsdr_rx_config_default) are the firmware's, drivers/ui/ui_configuration.c:70-230.
 */
typedef struct uhsdr_rx_config
{
    int32_t dmod_mode;            /* ts.dmod_mode */
    int32_t filter_path;          /* ts.filter_path_mem[mode][0]: index into FilterPathInfo */
    int32_t iq_freq_mode;         /* ts.iq_freq_mode */
    int32_t iq_auto_correction;   /* ts.iq_auto_correction */
    float   iq_gain_i;            /* ts.rx_adj_gain_var.i */
    float   iq_gain_q;            /* ts.rx_adj_gain_var.q */
    float   iq_phase_balance;     /* ads.iq_phase_balance_rx */
    int32_t dsp_active;           /* ts.dsp.active (MNOTCH / MPEAK bits) */
    int32_t notch_frequency;      /* ts.dsp.notch_frequency */
    int32_t peak_frequency;       /* ts.dsp.peak_frequency */
    int32_t bass_gain;            /* ts.dsp.bass_gain */
    int32_t treble_gain;          /* ts.dsp.treble_gain */
    int32_t cw_lsb;               /* ts.cw_lsb */
    int32_t digi_lsb;             /* ts.digi_lsb */
    int32_t agc_mode;             /* agc_wdsp_conf.mode */
    int32_t agc_slope;            /* agc_wdsp_conf.slope */
    int32_t agc_thresh;           /* agc_wdsp_conf.thresh */
    int32_t agc_hang_enable;      /* agc_wdsp_conf.hang_enable */
    int32_t agc_hang_time;        /* agc_wdsp_conf.hang_time (500) */
    int32_t agc_hang_thresh;      /* agc_wdsp_conf.hang_thresh (45) */
    int32_t agc_tau_decay[6];     /* agc_wdsp_conf.tau_decay[] */
    int32_t agc_tau_hang_decay;   /* agc_wdsp_conf.tau_hang_decay */
    int32_t sam_sideband;         /* ads.sam_sideband: 0 both, 1 LSB, 2 USB (audio_driver.h:181-190) */
    int32_t sam_pll_fmax;         /* ads.pll_fmax_int (2500) */
    int32_t sam_zeta;             /* ads.zeta_int, zeta x 100 (65) */
    int32_t sam_omega_n;          /* ads.omegaN_int (250) */
    int32_t fade_leveler;         /* ads.fade_leveler (1) */
    int32_t fm_sql_threshold;     /* ts.fm_sql_threshold (FM_SQUELCH_DEFAULT 12, audio_driver.h:449) */
    int32_t fm_deviation_5k;      /* FLAGS2_FM_MODE_DEVIATION_5KHZ (RadioManagement_FmDevIs5khz) */
    int32_t cw_sidetone_freq;     /* ts.cw_sidetone_freq (750): the CW decoder's Goertzel frequency */
    int32_t cw_decoder_blocksize; /* cw_decoder_config.blocksize (88, 8..128, cw_decoder.h:12-13) */
    int32_t cw_decoder_thresh;    /* cw_decoder_config.thresh (32000, cw_decoder.h:15-17) */
    int32_t cw_decoder_noisecancel; /* cw_decoder_config.noisecancel_enable (1) */
    /* ABI 2 */
    int32_t notch_mu;             /* ts.dsp.notch_mu (DSP_NOTCH_MU_DEFAULT 10, 0..40): LMS auto notch
                                     convergence; the notch runs with UHSDR_DSP_NOTCH_ENABLE in dsp_active */
    int32_t fm_tone_det;          /* ts.fm_subaudible_tone_det_select: 0 off, else index into
                                     fm_subaudible_tone_table (FM subaudible tone detector) */
    int32_t beep_frequency;       /* ts.beep_frequency (DEFAULT_BEEP_FREQUENCY 1000 Hz) */
    int32_t beep_loudness;        /* ts.beep_loudness (DEFAULT_BEEP_LOUDNESS 10) */
    int32_t stereo_enable;        /* ts.stereo_enable: two-channel audio in DEMOD_SSBSTEREO, DEMOD_IQ and
                                     SAM with UHSDR_SAM_SIDEBAND_STEREO (audio_driver.c:2618) */
    /* ABI 3 */
    int32_t board;                /* UHSDR_BOARD_OVI40 (default: USE_TWO_CHANNEL_AUDIO, the oracle's build)
                                     or UHSDR_BOARD_MCHF (single-channel audio, UI_BRD_MCHF) */
    int32_t spkr_gain;            /* ts.rx_gain[RX_AUDIO_SPKR].value (mcHF: a software gain above
                                     CODEC_SPEAKER_MAX_VOLUME 16, audio_driver.c:2880-2885) */
    int32_t reserved[9];
} uhsdr_rx_config;

/* the UI board the firmware is built for (hardware/uhsdr_board_config.h:16-24): its output stage
   (audio_driver.c:2856-2897).  OVI40 (USE_TWO_CHANNEL_AUDIO): a_buffer[1] x10 in place, a_buffer[0]
   its copy (or the second channel), key beep on both.  mcHF (no USE_TWO_CHANNEL_AUDIO): a_buffer[0]
   = 10 x a_buffer[1] (line out), a_buffer[1] the speaker channel with the software gain
   (spkr_gain / 2.5 - 5.35, ui_driver.c:3083-3092) above volume 16, key beep on a_buffer[1] only; no
   two-channel modes (DEMOD_SSBSTEREO / DEMOD_IQ unsupported, no SAM_SIDEBAND_STEREO). */
enum { UHSDR_BOARD_OVI40 = 0, UHSDR_BOARD_MCHF = 1 };

/* AudioAgc_SetupAgcWdsp() results (audio_agc.c:126-339) */
typedef struct uhsdr_agc_plan
{
    int32_t mode;                 /* 5 == fixed gain (AGC off) */
    int32_t hang_enable;
    int32_t remove_dc;
    int32_t ring_buffsize;        /* 192 */
    int32_t attack_buffsize;      /* ceilf(rate * n_tau * tau_attack): 49 at 12 ksps */
    int32_t out_index0;           /* -1 */
    int32_t in_index0;            /* (attack_buffsize + out_index0) % ring_buffsize */
    int32_t hang_counter_init;    /* (int)(hangtime * sample_rate) */
    float   sample_rate;
    float   fixed_gain, attack_mult, decay_mult, fast_decay_mult, fast_backmult;
    float   onemfast_backmult, hang_backmult, onemhang_backmult, hang_decay_mult;
    float   pop_ratio, hang_level, min_volts, inv_max_input, out_target, slope_constant;
    float   hangtime, hang_thresh, var_gain, max_gain, inv_out_target;
} uhsdr_agc_plan;

/*
 * Resolved processing chain (what SetProcessingChain leaves in the driver's instances).
 * Built on the host; uploaded once per handle; read-only for the kernels.
 */
typedef struct uhsdr_rx_plan
{
    int32_t dmod_mode, filter_path, lsb;
    int32_t decimation_rate;      /* ads.decimation_rate */
    int32_t decimated_freq;       /* ads.decimated_freq */
    int32_t use_decimated_iq;     /* audio_driver.c:2718-2720 */
    int32_t iq_auto_correction;
    float   iq_gain_i, iq_gain_q, iq_phase_balance;
    int32_t freq_shift_hz;        /* AudioDriver_GetTranslateFreq(), audio_driver.c:445-464 */
    int32_t shift_kind;           /* 0 none, 1 Fs/4 exchange, 2 recursive oscillator */
    int32_t shift_up;             /* dir == FREQ_SHIFT_UP (freq_shift.c:324) */
    float   osc_cos, osc_sin;     /* FreqShift_Approx_Prepare, freq_shift.c:40-52 */
    int32_t hilbert_taps;         /* 0 => Hilbert skipped (AM/SAM) */
    float   hilbert_i[UHSDR_MAX_FIR_TAPS];
    float   hilbert_q[UHSDR_MAX_FIR_TAPS];
    int32_t dec_taps;
    float   dec[UHSDR_MAX_DEC_TAPS];
    int32_t pre_stages;
    float   pre_k[UHSDR_MAX_LATTICE];
    float   pre_v[UHSDR_MAX_LATTICE + 1];
    int32_t interp_L, interp_phase;  /* INTERPOLATE_RX: L, phaseLength (quirk: numTaps/L) */
    float   interp[UHSDR_MAX_INTERP];
    int32_t aa_stages;
    float   aa_k[UHSDR_MAX_LATTICE];
    float   aa_v[UHSDR_MAX_LATTICE + 1];
    float   biquad1[20];          /* IIR_biquad_1: 4 stages {b0,b1,b2,a1,a2} */
    float   biquad2[5];           /* IIR_biquad_2: 1 stage */
    float   post_agc_scale;       /* audio_driver.c:2513-2524 */
    float   line_out_scale;       /* LINE_OUT_SCALING_FACTOR, audio_driver.h:396 (mcHF: 1, see below) */
    uhsdr_agc_plan agc;
    /* AM / SAM (AudioDriver_DemodSAM, audio_driver.c:1990-2166) */
    float   dec_q[UHSDR_MAX_DEC_TAPS];  /* DECIMATE_RX_Q taps: the path's Q table for AM/SAM (audio_filter.c:1167-1176) */
    int32_t sam_sideband, fade_leveler;
    /* AudioDriver_SetSamPllParameters, audio_driver.c:709-745 */
    float   sam_omega_min, sam_omega_max, sam_g1, sam_g2;
    float   fade_mtauR, fade_onem_mtauR, fade_mtauI, fade_onem_mtauI;
    /* FM (AudioDriver_DemodFM, audio_driver.c:1544-1737) */
    float   fm_scale;             /* FM_RX_SCALING_2K5 10000 or _5K 5000 (audio_driver.c:1494-1495) */
    int32_t fm_sql_threshold;
    int32_t sq_stages;            /* IIR_Squelch_HPF = IIR_15k_hpf (audio_driver.c:481-484) */
    float   sq_k[UHSDR_MAX_LATTICE];
    float   sq_v[UHSDR_MAX_LATTICE + 1];
    /* CW decoder front end (CwDecode_RxProcessor, cw_decoder.c:383-397, 182-316): Goertzel per
       block on a_buffer[0] after biquad_1, in CW / AM / SAM at 12 ksps (audio_driver.c:2550-2557) */
    int32_t cw_enabled, cw_blocksize, cw_noisecancel;
    float   cw_thresh;
    float   cw_r, cw_cos, cw_sin;     /* AudioFilter_CalcGoertzel (audio_filter.c:1281-1288) */
    /* ABI 2 */
    /* LMS auto notch: AudioDriver_NotchFilter (audio_driver.c:1746-1763) -> arm_lms_norm_f32 on
       a_buffer[0] at the decimated rate, before the pre-filter (:2443-2456); set up at :1166-1186 */
    int32_t notch_enabled;        /* DSP_NOTCH_ENABLE, not in CW, not in SAM at 24 ksps */
    int32_t notch_taps;           /* ts.dsp.notch_numtaps (DSP_NOTCH_NUMTAPS_DEFAULT 64) */
    int32_t notch_delay_len;      /* ts.dsp.notch_delaybuf_len (DSP_NOTCH_DELAYBUF_DEFAULT 128) */
    float   notch_mu;             /* log10f(((notch_mu + 1.0) / 1500.0) + 1.0) */
    /* FM subaudible tone detector (audio_driver.c:1665-1734), Goertzels of
       AudioManagement_CalcSubaudibleDetFreq (audio_management.c:313-326): FM_HIGH, FM_LOW, FM_CTR */
    int32_t tone_det_enabled;
    float   tone_r[3], tone_cos[3], tone_sin[3];
    /* key beep: softdds step and loudness (AudioManagement_KeyBeepPrepare, audio_management.c:354-363) */
    uint32_t beep_step;
    float   beep_scale;
    /* OVI40 two-channel audio (use_stereo, audio_driver.c:2618): 0 mono, 1 SSB stereo
       (a_buffer[0] = I + Q, [1] = I - Q), 2 IQ (a_buffer[0] = I, [1] = Q), 3 SAM stereo */
    int32_t stereo;
    int16_t dds_table[1024];      /* softdds DDS_TABLE (softdds/dds_table.c) */
    /* ABI 3: output stage of the board (uhsdr_rx_config.board).  line_out_scale above is
       LINE_OUT_SCALING_FACTOR on OVI40 (a_buffer[1] x10 in place) and 1 on mcHF, where a_buffer[0]
       = line_out0_scale (LINE_OUT_SCALING_FACTOR) x biquad_2's output and a_buffer[1] = spkr_scale
       (the speaker's software gain, 1 at volume <= 16) x the same */
    int32_t single_channel;       /* 1: mcHF output stage */
    float   line_out0_scale;
    float   spkr_scale;
    int32_t reserved[29];
} uhsdr_rx_plan;

typedef struct uhsdr_rx_s* uhsdr_rx_handle;

/* ---- host setup layer ---- */
void         uhsdr_rx_config_default(uhsdr_rx_config* cfg);
uhsdr_status uhsdr_rx_plan_build(const uhsdr_rx_config* cfg, uhsdr_rx_plan* plan);
/* 1 if the device chain implements this plan, 0 otherwise */
int          uhsdr_rx_plan_supported(const uhsdr_rx_plan* plan);
/* 1 if uhsdr_rx_set_precision accepts UHSDR_PRECISION_FMA for this plan: the Hilbert-first
 * families whose FMA output was measured within 1e-5 normwise of the reference
 * (tools/fma_sweep.py, tests/test_gpu_fma.py), 0 otherwise */
int          uhsdr_rx_plan_fma_ok(const uhsdr_rx_plan* plan);

/* ---- batched device chain ---- */
/* stream: hipStream_t to order all work of this handle on (NULL = default stream). */
uhsdr_status uhsdr_rx_create(const uhsdr_rx_config* cfg, int32_t num_channels, int32_t frames_per_call,
                             void* stream, uhsdr_rx_handle* out);
uhsdr_status uhsdr_rx_reset(uhsdr_rx_handle h);
/* iq, audio, dst: device pointers ([C][N][2] int32, [C][N] f32, [C][N][2] int32).
   audio or dst may be NULL (not written).  Asynchronous on the handle's stream. */
uhsdr_status uhsdr_rx_process(uhsdr_rx_handle h, const int32_t* iq, float* audio, int32_t* dst);
/* OVI40 two-channel modes (plan.stereo != 0): audio = adb.a_buffer[1] (channel 0, codec left),
   audio0 = adb.a_buffer[0] (channel 1, codec right), dst = both channels {l, r}; either may be
   NULL.  Without stereo on OVI40, audio0 is not written (a_buffer[0] is a copy of a_buffer[1]);
   on mcHF (uhsdr_rx_config.board) audio0 gets a_buffer[0], the line-out channel. */
uhsdr_status uhsdr_rx_process_stereo(uhsdr_rx_handle h, const int32_t* iq, float* audio, float* audio0, int32_t* dst);
/* Same with host buffers: copies in, processes, copies out, synchronises. */
uhsdr_status uhsdr_rx_process_host(uhsdr_rx_handle h, const int32_t* iq, float* audio, int32_t* dst);
uhsdr_status uhsdr_rx_get_plan(uhsdr_rx_handle h, uhsdr_rx_plan* plan);
uhsdr_status uhsdr_rx_set_stream(uhsdr_rx_handle h, void* stream);
uhsdr_status uhsdr_rx_destroy(uhsdr_rx_handle h);

/* Wait until every call enqueued on the handle has finished (both streams when pipelined). */
uhsdr_status uhsdr_rx_synchronize(uhsdr_rx_handle h);

/* Pipelined mode (off by default).  On: rx_back runs on a private side stream and the
   decimated hand-off rotates over three buffers, so rx_front runs up to two calls ahead of rx_back —
   the streaming throughput of back-to-back ISR calls is max(front, back) instead of the sum.
   Results are identical; only their completion point moves: the audio / dst / CW outputs of
   a call are complete after uhsdr_rx_synchronize(), or for work enqueued on the handle's
   stream after uhsdr_rx_join() (which orders the handle stream after every rx_back issued
   so far).  The caller must not overwrite an output buffer still being written: reuse across
   calls is safe (rx_back launches are ordered on the side stream).  Replaces nothing in the
   reference (the firmware runs one ISR at a time); uhsdr_rx_process_host joins itself.
   enable = 1: each rx_back waits for its rx_front through a cross-stream event.
   enable = 2 (device hand-off): rx_front stores the decimated hand-off write-through and each of
   its waves, once its stores have completed, bumps an arrival counter of its 64-channel group;
   rx_back -- the wave-pipeline back end without a demodulator or notch (SSB / CW / DIGI), while
   its grid is at most half the CUs -- polls its group's counter on the device and reads the
   hand-off with L1-bypassing sc1 loads: no cross-stream wait and no extra kernel per call, so the
   side stream's back ends run back to back.  When the next call's front has already arrived, a
   back-end launch also runs its first pipeline roles ahead into that call instead of draining
   (bit-identical; the next launch then starts without a pipeline fill).  Other calls keep the
   event.
   enable = 3 (persistent back end): the device hand-off, and one rx_back launch runs call after
   call -- wave-pipeline back ends without the CW decoder and with calls of 256+ frames; others as
   enable = 2.  Each uhsdr_rx_process writes the call's descriptor (its hand-off buffer, outputs and
   key beep) into host-mapped memory and grants the call to the running launch, which takes it with
   its state in registers; a launch that finds no grant when it needs the next call ends (the host
   then starts a new one with the next call).  uhsdr_rx_join, uhsdr_rx_synchronize, uhsdr_rx_reset
   and every mode or schedule change end the running launch after the calls granted so far, so a
   device-wide synchronisation (or join) completes without further calls.  The host waits in
   uhsdr_rx_process before refilling a hand-off buffer the back end has not read yet (8 calls
   back).  Same failure contract as enable = 2 (a give-up inside a launch poisons the call it
   waited for, and may poison the end of the call before it).  A running launch waits for fronts
   enqueued after it, so the handle's side stream (made at the first uhsdr_rx_set_pipelined) must not
   share a hardware queue with the handle's stream: HIP spreads streams over GPU_MAX_HW_QUEUES queues
   (4 by default), so make the handle before other streams of the process (a shared queue shows as a
   give-up, UHSDR_TIMEOUT, never as silent output).  Any other enable value returns
   UHSDR_ARGUMENT_ERROR.
   Failure contract of the device hand-off.  The poll is bounded (uhsdr_rx_set_handoff_bound,
   default 2^24 polls: seconds).  If rx_back gives up -- the handle's stream held the call's
   rx_front back that long behind other work, or a profiler serialised the two streams' dispatches
   -- then (1) that launch is poisoned: every frame of the call's audio is NaN (its codec frames
   carry what the reference's float -> int32 conversion makes of NaN, 0), so it cannot pass for
   output; (2) the handle's host-mapped failure word is set, and from
   then on uhsdr_rx_process, uhsdr_rx_join and uhsdr_rx_synchronize return UHSDR_TIMEOUT (join
   reports it once the give-up has happened, synchronize always after the calls before it); (3)
   uhsdr_rx_handoff_timeouts returns 1; (4) uhsdr_rx_reset clears the word and the poisoned state.
   Under a profiler that serialises dispatches (rocprofv3 --pmc) use enable = 1. */
uhsdr_status uhsdr_rx_set_pipelined(uhsdr_rx_handle h, int32_t enable);
/* Poll bound of the device hand-off (polls of >= 128 shader cycles each); for tests of the
   failure contract.  0 is UHSDR_ARGUMENT_ERROR.  A running persistent launch keeps the bound it
   started with. */
uhsdr_status uhsdr_rx_set_handoff_bound(uhsdr_rx_handle h, uint32_t polls);
/* Test hook of the persistent back end (enable = 3): out[0..7] = its grant word, the launch epoch,
   its exit and decision words, group 0's consumed word, whether a launch may take the next grant, the last call granted,
   and the launches started.  UHSDR_UNSUPPORTED before the mode was first entered. */
uhsdr_status uhsdr_rx_debug_persist(uhsdr_rx_handle h, uint32_t* out);
/* 1 if a device hand-off poll gave up since the last uhsdr_rx_reset, else 0; -1 on error.
   Synchronises. */
int32_t      uhsdr_rx_handoff_timeouts(uhsdr_rx_handle h);

/* Arithmetic of the FIR dot products in rx_front (Hilbert pair, decimators, AM/FM I/Q filters).
   EXACT (default): a rounded multiply then a rounded add per tap, in tap order -- the binary32
   sequence of CMSIS arm_fir_f32 / arm_fir_decimate_f32 as the reference builds them, so every
   output is bit-identical to the reference chain.  FMA: one fused multiply-add per tap
   (v_pk_fma_f32), half the VALU issue; outputs within north_star's 1e-5 normwise relative
   tolerance of the reference (max|diff| / max|ref| per channel), not bit-identical.  The
   recursive stages (lattices, AGC, biquads, demodulators) always run the reference sequence.
   FMA is accepted only on the Hilbert-first families (wide SSB / CW / DIGI at 12 and 24 ksps,
   FM), where it stays within 1e-5; the decimate-first families (narrow SSB / CW, AM, SAM)
   amplify the FIR rounding difference past 1e-5 (1.3e-5 .. 1.8e-5 measured), so there the call
   returns UHSDR_UNSUPPORTED and the handle stays EXACT.
   Takes effect from the next uhsdr_rx_process. */
enum { UHSDR_PRECISION_EXACT = 0, UHSDR_PRECISION_FMA = 1 };
uhsdr_status uhsdr_rx_set_precision(uhsdr_rx_handle h, int32_t precision);
int32_t      uhsdr_rx_get_precision(uhsdr_rx_handle h);   /* -1 for a null handle */
uhsdr_status uhsdr_rx_join(uhsdr_rx_handle h);

/* Kernel schedule of a call (a launch-shape choice: outputs are bit-identical under every one).
 *   AUTO        (default) SPLIT_FUSED from 131072 channels on, else SPLIT_PIPE; CHAIN only
 *               when requested
 *   SPLIT_PIPE  rx_front, then rx_back: one wave per back-end stage, a pipeline over 32-frame
 *               calls (short per-call critical path: small batches)
 *   SPLIT_FUSED rx_front, then rx_back_fused: every back-end stage in one wave per 64 channels
 *   CHAIN       rx_chain: one kernel, each wave runs the front passes of its 64 channels and then
 *               their back end, the decimated hand-off kept in LDS (large batches).  SSB / CW /
 *               DIGI mono paths (no notch, no stereo, not AM / SAM / FM) with one front pass per
 *               call; elsewhere UHSDR_UNSUPPORTED.
 * Stereo, AM / SAM / FM and the LMS notch have their own back-end kernels and ignore SPLIT_*.
 * Returns UHSDR_UNSUPPORTED (handle unchanged) for a schedule the handle's path cannot run.
 * Takes effect from the next uhsdr_rx_process; get returns the resolved schedule. */
enum { UHSDR_SCHEDULE_AUTO = 0, UHSDR_SCHEDULE_SPLIT_PIPE = 1, UHSDR_SCHEDULE_SPLIT_FUSED = 2,
       UHSDR_SCHEDULE_CHAIN = 3 };
uhsdr_status uhsdr_rx_set_schedule(uhsdr_rx_handle h, int32_t schedule);
int32_t      uhsdr_rx_get_schedule(uhsdr_rx_handle h);    /* -1 for a null handle */
/* FIR outputs per lane of the front passes: 8 (default: more waves per batch) or 16 (fewer LDS
   window reads per MAC); UHSDR_UNSUPPORTED when the call size does not admit it.  Bit-identical. */
uhsdr_status uhsdr_rx_set_front_block(uhsdr_rx_handle h, int32_t outputs_per_lane);

/* ---- status side outputs: the RX chain's signals to the control plane ----
 * ADC clip indicators (audio_driver.c:2660-2676): per channel, the sticky flags ads.adc_clip /
 * ads.adc_half_clip / ads.adc_quarter_clip, set when |I| >> 16 of any frame exceeds
 * ADC_CLIP_WARN_THRESHOLD (4096, audio_driver.h:81) / its half / its quarter -- the S-meter's
 * red indicator and the auto RF-gain trigger / release.  The firmware's UI reads and clears
 * them; here the kernels OR the bits of every frame they process into clip[c] (device memory,
 * [C] uint32, the caller zeroes it and clears it after reading).  NULL (default) = not computed.
 * The magnitude is taken as unsigned, so a full-scale negative sample (INT32_MIN, where the
 * reference's abs() is undefined) counts as a clip. */
#define UHSDR_ADC_CLIP          1
#define UHSDR_ADC_HALF_CLIP     2
#define UHSDR_ADC_QUARTER_CLIP  4
uhsdr_status uhsdr_rx_set_clip_output(uhsdr_rx_handle h, uint32_t* clip);
/* Twin-peaks I/Q fault detector (AudioDriver_RxHandleTwinpeaks, audio_driver.c:2173-2248), run
 * per 32-frame call with automatic I/Q correction: 1000 calls of settling, then 50 calls of the
 * Moseley & Slump phase estimate asin(teta1 / teta3), smoothed; more than 22.5 degrees requests a
 * codec restart, the fourth consecutive one declares the fault uncorrectable.  Per channel state
 * ts.twinpeaks_tested (hardware/uhsdr_board.h:647-651), WAIT after create / reset
 * (src/uhsdr_main.c:339). */
enum { UHSDR_TWINPEAKS_SAMPLING = 0, UHSDR_TWINPEAKS_DONE = 1, UHSDR_TWINPEAKS_WAIT = 2,
       UHSDR_TWINPEAKS_UNCORRECTABLE = 3, UHSDR_TWINPEAKS_CODEC_RESTART = 4 };
/* copies the C states (int32) to `state` (device memory), ordered on the handle's stream */
uhsdr_status uhsdr_rx_twinpeaks_state(uhsdr_rx_handle h, int32_t* state);
/* the UI's acknowledgement after it restarted the codec (ui_driver.c:7422-7426): every channel in
 * CODEC_RESTART goes back to WAIT; ordered on the handle's stream */
uhsdr_status uhsdr_rx_twinpeaks_rearm(uhsdr_rx_handle h);

/* ---- device memory for plain-C hosts (no HIP headers needed) ---- */
void*        uhsdr_device_alloc(uint64_t bytes);             /* NULL on failure */
void         uhsdr_device_free(void* p);
uhsdr_status uhsdr_copy_to_device(void* dst, const void* src, uint64_t bytes);
uhsdr_status uhsdr_copy_to_host(void* dst, const void* src, uint64_t bytes);

/* ================================ transmit ================================
 * TxProcessor_Run (drivers/audio/tx_processor.c:891-1078) for SSB (USB / LSB) voice:
 *   codec audio frames -> mic gain -> TX band-pass lattice -> bass/treble biquads ->
 *   ALC compressor with its 288-sample look-ahead delay -> 201-tap Hilbert pair ->
 *   FreqShift -> I/Q gain + phase -> int32 IQ frames for the DAC.
 * AM voice (TxProcessor_AM, :715-800, dispatch :1000-1008): the same voice chain with
 *   AM_ALC_GAIN_CORRECTION, the Hilbert pair, both sidebands plus carrier
 *   (I - Q + 2 * AM_CARRIER_LEVEL, Q - I - 2 * AM_CARRIER_LEVEL), FreqShift.
 * FM voice: the voice chain, pre-emphasis and the softdds modulator (:534-588).
 * USB I/Q source (TX_AUDIO_DIGIQ, :950-961): the input frames are the I/Q itself, straight to the
 *   final gain / phase stage (not in CW or TUNE, where the voice path runs as usual).
 * One uhsdr_tx_process call == N/32 TX-mode AudioDriver_I2SCallback invocations per channel.
 */
#define UHSDR_TX_HILBERT_TAPS 201    /* iq_tx_wide, drivers/audio/filters/iq_tx_filter.h:22 */
#define UHSDR_TX_DELAY 320           /* AUDIO_DELAY_BUFSIZE, audio_driver.h:516 */

/* TX_AUDIO_*, hardware/uhsdr_board.h:128-132 (DIG: USB audio in place of the codec's, no bass /
   treble; DIGIQ: USB I/Q).  Modes: UHSDR_DEMOD_USB / LSB (SSB voice), UHSDR_DEMOD_AM and
   UHSDR_DEMOD_FM (both need iq_freq_mode != OFF like the reference, tx_processor.c:1000-1011) */
enum { UHSDR_TX_AUDIO_MIC = 0, UHSDR_TX_AUDIO_LINEIN_L = 1, UHSDR_TX_AUDIO_LINEIN_R = 2, UHSDR_TX_AUDIO_DIG = 3,
       UHSDR_TX_AUDIO_DIGIQ = 4 };

typedef struct uhsdr_tx_config
{
    int32_t dmod_mode;            /* ts.dmod_mode: UHSDR_DEMOD_USB, _LSB, _AM or _FM */
    int32_t iq_freq_mode;         /* ts.iq_freq_mode */
    int32_t audio_source;         /* ts.tx_audio_source: MIC, LINEIN_L, LINEIN_R, DIG, DIGIQ */
    int32_t mic_gain_mult;        /* ts.tx_mic_gain_mult (codec.c:313-321) */
    int32_t mic_boost;            /* ts.tx_mic_boost */
    int32_t comp_level;           /* ts.tx_comp_level: -1 off, 0..12 presets, 13 = stored values */
    int32_t alc_decay;            /* ts.alc_decay (EEPROM, used by comp_level 13) */
    int32_t alc_postfilt_gain;    /* ts.alc_tx_postfilt_gain (EEPROM, used by comp_level 13) */
    int32_t tx_filter;            /* ts.tx_filter: 0/1 soprano, 2 tenor, 3 bass */
    int32_t bass_gain;            /* ts.dsp.tx_bass_gain */
    int32_t treble_gain;          /* ts.dsp.tx_treble_gain */
    int32_t filter_disable;       /* FLAGS1_SSB_TX_FILTER_DISABLE (SSB) / FLAGS1_AM_TX_FILTER_DISABLE (AM) */
    float   power_factor;         /* ts.tx_power_factor */
    float   gain_i, gain_q;       /* ts.tx_adj_gain_var[trans].i / .q */
    float   phase_balance;        /* ads.iq_phase_balance_tx[trans] */
    int32_t fm_deviation_5k;      /* FLAGS2_FM_MODE_DEVIATION_5KHZ: FM transmit deviation 5 kHz (else 2.5) */
    int32_t fm_subaudible_tone;   /* ts.fm_subaudible_tone_gen_select: index into fm_subaudible_tone_table, 0 = off */
    int32_t fm_tone_burst_mode;   /* ts.fm_tone_burst_mode: 0 off, 1 1750 Hz, 2 2135 Hz (fm_tone_burst_freq,
                                     audio_management.c:328), sent while uhsdr_tx_set_tone_burst is on */
    int32_t reserved[13];
} uhsdr_tx_config;

typedef struct uhsdr_tx_plan
{
    int32_t dmod_mode, lsb, audio_source;
    float   in_gain;              /* gain_calc of TxProcessor_AudioBufferFill (tx_processor.c:354-381) */
    int32_t apply_in_gain;        /* gain_calc != 1.0 */
    int32_t run_lattice, run_biquad;
    int32_t lat_stages;
    float   lat_k[UHSDR_MAX_LATTICE];
    float   lat_v[UHSDR_MAX_LATTICE + 1];
    float   biquad[15];           /* IIR_TX_biquad: treble shelf 1700 Hz, bass shelf 300 Hz, passthrough */
    int32_t comp_on;              /* ts.tx_comp_level > -1 */
    float   postfilt_gain;        /* alc_tx_postfilt_gain_var / 2.0 + 0.5 */
    float   alc_decay;            /* ads.alc_decay (audio_management.c:15-19) */
    float   alc_gain_scaling;     /* SSB_ALC_GAIN_CORRECTION */
    float   hilbert_i[UHSDR_TX_HILBERT_TAPS + 7];   /* already swapped for LSB (tx_processor.c:477-478) */
    float   hilbert_q[UHSDR_TX_HILBERT_TAPS + 7];
    int32_t freq_shift_hz, shift_kind, shift_up;
    float   osc_cos, osc_sin;
    float   final_i_gain, final_q_gain;   /* tx_power_factor * tx_adj_gain_var * SSB_GAIN_COMP * 2^16 */
    float   phase_balance;
    /* FM transmit (TxProcessor_FM, tx_processor.c:534-588): pre-emphasis, optional sub-audible
       tone from a softdds NCO, 16-bit accumulator NCO over the softdds sine table */
    int32_t fm;
    float   fm_mod_mult;          /* 2 with 5 kHz deviation, else 1 */
    uint32_t fm_word;             /* (65536 * |translate_freq|) / 48000 */
    int32_t fm_swap;              /* translate_freq < 0: I and Q buffers exchanged */
    int32_t fm_sub_on;
    uint32_t fm_sub_step;         /* softdds_stepForSampleRate(tone, 48000) (softdds.c:26-32) */
    float   fm_sub_scale;         /* FM_SUBAUDIBLE_TONE_AMPLITUDE_SCALING * fm_mod_mult */
    int16_t dds_table[1024];      /* DDS_TABLE, softdds/dds_table.c */
    /* softdds tones: TUNE (AudioManagement_SetSidetoneForDemodMode, audio_management.c:377-404:
       SSB_TUNE_FREQ 750 Hz, two-tone + 1950 Hz) and the FM tone burst (LoadToneBurstMode :339-349) */
    uint32_t tune_step[2];
    uint32_t tone_burst_step;
    float   tone_burst_scale;     /* FM_TONE_BURST_AMPLITUDE_SCALING * fm_mod_mult */
    int32_t am;                   /* TxProcessor_AM: both sidebands + carrier after the Hilbert pair */
    int32_t digiq;                /* TX_AUDIO_DIGIQ: the input frames are I/Q for the final stage */
    float   digiq_i_gain, digiq_q_gain;   /* final gains with iq_gain_comp 1.0 (tx_processor.c:924) */
    int32_t reserved[24];
} uhsdr_tx_plan;

typedef struct uhsdr_tx_s* uhsdr_tx_handle;

void         uhsdr_tx_config_default(uhsdr_tx_config* cfg);
uhsdr_status uhsdr_tx_plan_build(const uhsdr_tx_config* cfg, uhsdr_tx_plan* plan);
/* audio: device AudioSample_t [C][N][2] int32 in; iq: device IqSample_t [C][N][2] int32 out;
   a0: optional device f32 [C][N], the compressed audio (adb.a_buffer[0]) */
uhsdr_status uhsdr_tx_create(const uhsdr_tx_config* cfg, int32_t num_channels, int32_t frames_per_call,
                             void* stream, uhsdr_tx_handle* out);
uhsdr_status uhsdr_tx_reset(uhsdr_tx_handle h);
uhsdr_status uhsdr_tx_process(uhsdr_tx_handle h, const int32_t* audio, int32_t* iq, float* a0);
uhsdr_status uhsdr_tx_get_plan(uhsdr_tx_handle h, uhsdr_tx_plan* plan);
uhsdr_status uhsdr_tx_destroy(uhsdr_tx_handle h);
/* pipelined mode (no reference counterpart; off by default): tx_iq -- the Hilbert pair, FreqShift
 * and DAC frames -- runs on a private side stream and the compressed-audio hand-off rotates over
 * two buffers, so tx_voice of call k+1 (one lane per channel, latency-bound) overlaps tx_iq of
 * call k.  Outputs are bit-identical; iq of a call is complete once uhsdr_tx_join has ordered the
 * handle's stream after the side stream (then synchronize that stream as usual). */
uhsdr_status uhsdr_tx_set_pipelined(uhsdr_tx_handle h, int32_t enable);
int32_t      uhsdr_tx_get_pipelined(uhsdr_tx_handle h);
uhsdr_status uhsdr_tx_join(uhsdr_tx_handle h);
/* Arithmetic of the 201-tap Hilbert pair in tx_iq (no reference counterpart; EXACT by default).
   EXACT: a rounded multiply then a rounded add per tap, in tap order -- arm_fir_f32's binary32
   sequence, bit-identical DAC frames.  FMA: one fused multiply-add per tap (v_pk_fma_f32), half
   the pair's VALU issue; the DAC frames stay within north_star's 1e-5 normwise relative tolerance
   (max|diff| / max|ref| per channel) of the reference.  The voice chain (lattice, biquads, ALC)
   and FM always run the reference sequence: the pair's output feeds no recursion, so its rounding
   difference is not amplified (every SSB / AM mode and frequency translation measured, tests/
   test_gpu_tx_precision.py).  Takes effect from the next uhsdr_tx_process. */
uhsdr_status uhsdr_tx_set_precision(uhsdr_tx_handle h, int32_t precision);
int32_t      uhsdr_tx_get_precision(uhsdr_tx_handle h);   /* -1 for a null handle */
/* TxProcessor_PrepareRun (tx_processor.c:63-66): clear the ALC look-ahead delay line only,
   the first time back to TX; all other TX state carries on */
uhsdr_status uhsdr_tx_prepare_run(uhsdr_tx_handle h);
/* TUNE (ts.tune with ts.tune_tone_mode): from the next uhsdr_tx_process on, the transmitter's audio
   is the softdds tone instead of the codec input (TxProcessor_AudioBufferFill, tx_processor.c:344-347;
   softdds_runIQ into one buffer keeps the quadrature sample), the TX filters and the post-filter
   gain are skipped (:444-447, :179), the ALC runs.  Entering and leaving TUNE reconfigures the
   tone generator with its phase reset (AudioManagement_SetSidetoneForDemodMode, as
   RadioManagement_SwitchTxRx does, radio_management.c:1035).  Common to all channels. */
enum { UHSDR_TUNE_OFF = 0, UHSDR_TUNE_SINGLE = 1, UHSDR_TUNE_TWO = 2 };
uhsdr_status uhsdr_tx_set_tune(uhsdr_tx_handle h, int32_t tune);
/* FM tone burst ("whistle-up", ads.fm_conf.tone_burst_active, tx_processor.c:555-564): while on,
   the fm_tone_burst_mode tone replaces the sub-audible tone in the FM modulator.  No effect for
   SSB or with fm_tone_burst_mode 0. */
uhsdr_status uhsdr_tx_set_tone_burst(uhsdr_tx_handle h, int32_t active);
int32_t      uhsdr_sizeof_tx_config(void);
int32_t      uhsdr_sizeof_tx_plan(void);

/* ---- the firmware's ISR entry for one transceiver ----
 * AudioDriver_I2SCallback(audio, iq, audioDst, blockSize) (audio_driver.c:2962-3049) with the
 * firmware's own DMA half-buffers in host memory: AudioSample_t / IqSample_t = {int32 l, r}.
 * One receiver (uhsdr_rx_* with 1 channel) and optionally one transmitter (uhsdr_tx_*), both
 * with frames_per_call = block_size (32 on the firmware).
 *   RX (txrx_mode 0): iq in, codec frames out in `audio`.  The first call after TX, and while
 *       the input-mute counter runs, the firmware silences iq in place, still runs the chain
 *       and mutes the output (AudioDriver_IqFillSilence, RxProcessor external_mute :2845-2853).
 *   TX (txrx_mode 1): mic / line frames in `audio`, DAC I/Q out in `iq`, the codec sidetone in
 *       `audioDst` (zero for the voice modes, tx_processor.c:154-163, radio_management.c:450).
 *       The first call after RX runs TxProcessor_PrepareRun and, like a counted input mute,
 *       silences `audio` and skips the chain (external_mute: "do nothing", :946-949), so the I/Q
 *       out is zero and the TX state does not advance.
 * A call is synchronous: outputs are in the host buffers on return. */
/* ---- batched arm_fir_f32 (CMSIS FilteringFunctions/arm_fir_f32.c:482-560) ----
 * C channels, one shared tap set (CMSIS order, time-reversed), each channel's T-1 carried samples
 * on the device; one call == arm_fir_f32(S_c, src_c, dst_c, B) on every channel.  C5's long
 * narrow filter and the north_star's FIR-as-GEMM:
 *   UHSDR_FIR_EXACT  bit-identical to arm_fir_f32 (VALU, the reference's operation order)
 *   UHSDR_FIR_MFMA   the FIR as a GEMM on v_mfma_f32_16x16x4_f32 (fused multiply-adds in tap
 *                    order: within 1e-5 relative of the reference, not bit-identical)
 * block_size B: a multiple of 256.  src / dst: device f32 [C][B]. */
enum { UHSDR_FIR_EXACT = 0, UHSDR_FIR_MFMA = 1 };
typedef struct uhsdr_fir_s* uhsdr_fir_handle;

uhsdr_status uhsdr_fir_create(const float* coeffs, int32_t num_taps, int32_t num_channels, int32_t block_size,
                              int32_t mode, void* stream, uhsdr_fir_handle* out);
uhsdr_status uhsdr_fir_reset(uhsdr_fir_handle h);
uhsdr_status uhsdr_fir_process(uhsdr_fir_handle h, const float* src, float* dst);
uhsdr_status uhsdr_fir_synchronize(uhsdr_fir_handle h);
uhsdr_status uhsdr_fir_destroy(uhsdr_fir_handle h);
/* waves per workgroup of the FIR kernel (results do not depend on it): EXACT 1, 2 or 4 (default
 * 2); MFMA 1 .. 16 (default: as many as one workgroup's LDS holds, up to 16).
 * UHSDR_ARGUMENT_ERROR for another value, UHSDR_LENGTH_ERROR when that many windows do not fit
 * one workgroup's LDS (the setting is then unchanged). */
uhsdr_status uhsdr_fir_set_waves(uhsdr_fir_handle h, int32_t waves);
int32_t uhsdr_fir_get_waves(uhsdr_fir_handle h);

typedef struct uhsdr_i2s_s* uhsdr_i2s_handle;

uhsdr_status uhsdr_i2s_create(const uhsdr_rx_config* rx, const uhsdr_tx_config* tx /* NULL: receive only */,
                              int32_t block_size, void* stream, uhsdr_i2s_handle* out);
uhsdr_status uhsdr_i2s_set_txrx_mode(uhsdr_i2s_handle h, int32_t txrx_mode);   /* ts.txrx_mode: 0 RX, 1 TX */
uhsdr_status uhsdr_i2s_set_input_mute(uhsdr_i2s_handle h, int32_t calls);      /* ts.audio_processor_input_mute_counter */
uhsdr_status uhsdr_i2s_callback(uhsdr_i2s_handle h, int32_t* audio, int32_t* iq, int32_t* audioDst, int16_t blockSize);
uhsdr_status uhsdr_i2s_destroy(uhsdr_i2s_handle h);

/* ---- spectrum display ----
 * Replaces the no-zoom producer AudioDriver_SpectrumNoZoomProcessSamples (audio_driver.c:
 * 1811-1851: I/Q-corrected samples into an interleaved [Q, I] ring) and the consumer
 * UiSpectrum_RedrawSpectrum states 0-3 (drivers/ui/lcd/ui_spectrum.c:1350-1446): Hann window,
 * arm_cfft_f32 (CMSIS TransformFunctions/arm_cfft_f32.c:574-632), arm_cmplx_mag_f32 and the IIR
 * average clamped at 1.  Batched semantics: every fft_len consecutive input samples of a channel
 * (counted from reset) form one display frame; the firmware's main loop snapshots the ring at
 * arbitrary times, the batch takes it exactly when fft_len new samples have arrived.
 * The I/Q correction runs on the handle's own copy of the auto-correction state (it depends only
 * on the input), so a spectrum handle beside an RX handle sees what the firmware's ring sees.
 * magnify > 0 replaces the producer with the zoom one (AudioDriver_SpectrumZoomProcessSamples,
 * audio_driver.c:1860-1909): corrected I/Q, translated by iq_freq_mode (FreqShift), low-passed
 * and decimated by 2^magnify, so a display frame spans fft_len * 2^magnify input frames.
 */
#define UHSDR_SPECTRUM_MAX_LEN 1024
#define UHSDR_SPECTRUM_MAX_BITREV 1800   /* ARMBITREVINDEXTABLE1024_TABLE_LENGTH, arm_common_tables.h:96 */

typedef struct uhsdr_spectrum_config
{
    int32_t fft_len;              /* 256 (320x240), 512 (480x320 / 800x480: ui_spectrum.c:966-984) or 1024 */
    int32_t spectrum_filter;      /* ts.spectrum_filter 1..20, default 4 (ui_spectrum.h:143-145) */
    int32_t iq_auto_correction;   /* ts.iq_auto_correction, as uhsdr_rx_config */
    float   iq_gain_i, iq_gain_q; /* ts.rx_adj_gain_var.i / .q */
    float   iq_phase_balance;     /* ads.iq_phase_balance_rx */
    int32_t magnify;              /* sd.magnify 0..5: zoom 2^magnify (0: no zoom, ui_spectrum.c) */
    int32_t iq_freq_mode;         /* ts.iq_freq_mode: the translation the zoom producer sees */
    int32_t reserved[8];
} uhsdr_spectrum_config;

typedef struct uhsdr_spectrum_plan
{
    int32_t fft_len;
    int32_t window_formula;       /* 0: x *= window[i] (von_Hann_512/1024 tables, USE_PREDEFINED_WINDOW_DATA);
                                     1: x = 0.5 * ((window[i]) * x) with window = 1 - arm_cos_f32(2 pi i / (2L - 1))
                                        (ui_spectrum.c:403-406; no 2048-float table exists) */
    int32_t iq_auto_correction;
    float   iq_gain_i, iq_gain_q, iq_phase_balance;
    float   filt_factor;          /* 1 / (float)spectrum_filter (ui_spectrum.c:1434) */
    int32_t bitrev_len;           /* S->bitRevLength */
    float   window[2 * UHSDR_SPECTRUM_MAX_LEN];    /* per float of the interleaved [Q, I] frame */
    float   twiddle[2 * UHSDR_SPECTRUM_MAX_LEN];   /* twiddleCoef_<L> (arm_common_tables.c) */
    uint16_t bitrev[UHSDR_SPECTRUM_MAX_BITREV];    /* armBitRevIndexTable<L>: byte-offset swap pairs */
    uint16_t perm[UHSDR_SPECTRUM_MAX_LEN];         /* bin k of the output = butterfly result perm[k] */
    uint16_t iperm[UHSDR_SPECTRUM_MAX_LEN];        /* butterfly result p lands in bin iperm[p] */
    float   tw_lane[8][64][2];    /* the first-stage twiddles each of 64 lanes uses, laid out per lane
                                     (same values as twiddle[]; device read coalescing only) */
    /* zoom producer (AudioDriver_SpectrumZoomProcessSamples, audio_driver.c:1860-1909), magnify > 0:
       after I/Q correction and FreqShift, I and Q each through IIR_biquad_Zoom_FFT_I/_Q (4 stages,
       mag_coeffs[magnify]) and DECIMATE_ZOOM_FFT_I/_Q (FirZoomFFTDecimate[magnify]) */
    int32_t magnify;
    int32_t zoom_decimation;      /* 2^magnify */
    int32_t zoom_taps;
    int32_t freq_shift_hz, shift_kind, shift_up;   /* as uhsdr_rx_plan */
    float   osc_cos, osc_sin;
    float   zoom_biquad[20];
    float   zoom_fir[8];
    int32_t reserved[16];
} uhsdr_spectrum_plan;

typedef struct uhsdr_spectrum_s* uhsdr_spectrum_handle;

void         uhsdr_spectrum_config_default(uhsdr_spectrum_config* cfg);
uhsdr_status uhsdr_spectrum_plan_build(const uhsdr_spectrum_config* cfg, uhsdr_spectrum_plan* plan);
/* frames_per_call N: a multiple of 32 and either a multiple of fft_len (N/L display frames per
   call) or a divisor of it (one frame every L/N calls); otherwise UHSDR_LENGTH_ERROR. */
uhsdr_status uhsdr_spectrum_create(const uhsdr_spectrum_config* cfg, int32_t num_channels, int32_t frames_per_call,
                                   void* stream, uhsdr_spectrum_handle* out);
uhsdr_status uhsdr_spectrum_reset(uhsdr_spectrum_handle h);
/* iq: device IqSample_t [C][N][2] int32 (the RX input).  mag / avg: optional device f32
   [C][F][L], F = max(1, N/L): per completed frame sd.FFT_MagData and sd.FFT_AVGData (natural
   FFT bin order, as arm_cfft_f32 leaves them).  *frames (optional) = frames completed by this
   call (0 .. F); nothing is written to mag / avg when it is 0. */
uhsdr_status uhsdr_spectrum_process(uhsdr_spectrum_handle h, const int32_t* iq, float* mag, float* avg,
                                    int32_t* frames);
uhsdr_status uhsdr_spectrum_get_plan(uhsdr_spectrum_handle h, uhsdr_spectrum_plan* plan);
uhsdr_status uhsdr_spectrum_destroy(uhsdr_spectrum_handle h);
int32_t      uhsdr_sizeof_spectrum_config(void);
int32_t      uhsdr_sizeof_spectrum_plan(void);

/* CW decoder front end outputs of the following uhsdr_rx_process calls (device pointers, either
   may be NULL): signal = ads.CW_signal after every 32-frame call, uint8 [C][N/32];
   energy = the Goertzel energy of every CW block completed, f32 [C][uhsdr_rx_cw_blocks_max(h)],
   the first uhsdr_rx_cw_blocks_last(h) of them valid after a call. */
uhsdr_status uhsdr_rx_set_cw_outputs(uhsdr_rx_handle h, uint8_t* signal, float* energy);
int32_t      uhsdr_rx_cw_blocks_max(uhsdr_rx_handle h);
int32_t      uhsdr_rx_cw_blocks_last(uhsdr_rx_handle h);

/* Key beep (AudioManagement_KeyBeep, audio_management.c:368-375 -> the softdds tone added to the
   output at audio_driver.c:2891-2898): the beep's DDS accumulator restarts at 0 and the tone
   (config beep_frequency / beep_loudness) is added to every channel's output for the next
   `calls` 32-frame calls (the firmware's ts.beep_timing countdown, here counted in ISR calls);
   0 stops a running beep.  Like the firmware's single key beep, it is common to all channels. */
uhsdr_status uhsdr_rx_key_beep(uhsdr_rx_handle h, int32_t calls);

/* ---- diagnostics ---- */
const char*  uhsdr_version(void);
/* UHSDR_ABI_VERSION the library was built with: a binding compares it with the header it mirrors
   (a stale library would otherwise ignore config words it does not know) */
int32_t      uhsdr_abi_version(void);
/* sizeof(uhsdr_rx_config), sizeof(uhsdr_rx_plan): lets FFI bindings check their layouts */
int32_t      uhsdr_sizeof_config(void);
int32_t      uhsdr_sizeof_plan(void);
const char*  uhsdr_last_error(void);
/* number of kernel slots uhsdr_rx_kernel_times reports: rx_front, rx_back (any back-end kernel),
   rx_chain; a call enqueues rx_front + rx_back, or rx_chain alone */
int32_t      uhsdr_rx_kernel_count(uhsdr_rx_handle h);
/* Per-kernel device timing: while enabled (enable = k > 0), every k-th uhsdr_rx_process call
   (the 1st, (k+1)-th, ...) brackets each kernel with hipEvents on the stream it runs on; k = 1
   times every call.  Sampling keeps the event records' own host and device cost (~30 us per
   bracketed call) out of a throughput measurement.  uhsdr_rx_kernel_times() synchronises and
   returns, per kernel, the summed milliseconds and launch count of the timed calls since the
   last enable. */
uhsdr_status uhsdr_rx_enable_timing(uhsdr_rx_handle h, int32_t enable);
int32_t      uhsdr_rx_kernel_times(uhsdr_rx_handle h, float* total_ms, int32_t* launches, int32_t max_kernels);
const char*  uhsdr_rx_kernel_name(int32_t index);

#ifdef __cplusplus
}
#endif
#endif /* UHSDR_H */
