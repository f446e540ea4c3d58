/*
 * ORACLE TEST INFRASTRUCTURE -- command-line driver for the reference RX chain.
 *
 * Runs ONE channel through the reference firmware's own entry points, exactly as the
 * radio does at boot and per DMA interrupt:
 *     AudioDriver_Init();                       audio_driver.c:677-704
 *     AudioDriver_SetProcessingChain(mode,0);   audio_driver.c:1093-1251
 *     AudioDriver_I2SCallback(dst, iq, 0, 32)   audio_driver.c:2962-3049, once per 32 frames
 * One process = one channel, because the driver keeps its DSP state in globals and
 * function-local statics (e.g. FreqShift's NCO, audio_agc.c:578 `wold`).
 *
 * usage: uhsdr_ref key=value ...
 *   in=<file>      int32 I/Q frames {l,r} (IqSample_t, audio_driver.h:44-52)
 *   n=<frames>     number of frames (multiple of 32)
 *   out_a=<file>   f32 adb.a_buffer[1] after each call (audio_driver.h:147-157)
 *   out_dst=<file> int32 codec frames {l,r} (AudioSample_t)
 *   mode= path= iqmode= agc_mode= agc_thresh= agc_slope= agc_hang= bass= treble=
 *   iq_auto= gain_i= gain_q= phase= dsp= notch= peak= sam_sb= pll_fmax= zeta= omegan=
 *   fade= sql= fm5k= block=
 *   notch_mu=      ts.dsp.notch_mu (LMS auto notch, on with dsp=4 / DSP_NOTCH_ENABLE)
 *   tonedet=       ts.fm_subaudible_tone_det_select (FM subaudible tone detector)
 *   beep=b0:K      key beep on calls b0 .. b0+K-1 (AudioManagement_KeyBeep at call b0)
 *   beepfreq= beeploud=   ts.beep_frequency / ts.beep_loudness
 *   stereo=1       ts.stereo_enable (two-channel modes: mode=7 SSB stereo, mode=8 IQ, SAM sam_sb=3)
 *   out_a0=<file>  f32 adb.a_buffer[0] after each call (the second channel in stereo)
 *   board=         0 OVI40 (this build's default), 1 mcHF: must match the build (the mcHF variant,
 *                  make mchf, compiles the sources without USE_TWO_CHANNEL_AUDIO)
 *   spkr=          ts.rx_gain[RX_AUDIO_SPKR].value (AUDIO_GAIN_DEFAULT 16); its active_value as the
 *                  UI's volume update sets it (ui_driver.c:3083-3092)
 *   out_clip=<file> uint8 per call: ads.adc_clip | adc_half_clip << 1 | adc_quarter_clip << 2,
 *                  read and cleared after every call (the UI's role)
 *   out_tp=<file>  uint8 per call: ts.twinpeaks_tested after the call (AudioDriver_RxHandleTwinpeaks)
 *   uiperiod=P     the UI loop's codec restart handling (ui_driver.c:7422-7426: CODEC_RESTART ->
 *                  WAIT) runs after every P-th call (default 1)
 *   tx=1           transmit: in= holds codec audio frames {l,r}, out_dst= gets the IQ frames
 *                  TxProcessor_Run writes (tx_processor.c:891-1078), out_a= a_buffer[0]
 *   micmult= boost= comp= txfilter= txbass= txtreble= txpwr= txgi= txgq= txphase=
 *   txsrc=         ts.tx_audio_source (0 mic, 1/2 line in L/R, 3 USB audio, 4 USB I/Q): for 3 / 4
 *                  the USB buffer (UsbdAudio_FillTxBuffer) delivers the in= block of the call
 *   flags1=        ts.flags1 (FLAGS1_AM_TX_FILTER_DISABLE 0x08, FLAGS1_SSB_TX_FILTER_DISABLE 0x40)
 *   tune=t0:K:M    TUNE on calls t0 .. t0+K-1, M = 1 single tone, 2 two-tone (ts.tune, ts.tune_tone_mode,
 *                  AudioManagement_SetSidetoneForDemodMode on entry and exit, as RadioManagement does)
 *   burst=t0:K     FM tone burst on calls t0 .. t0+K-1 (ads.fm_conf.tone_burst_active)
 *   burstmode=     ts.fm_tone_burst_mode (0 off, 1 1750 Hz, 2 2135 Hz)
 *   dump=setup     print the configured chain (coefficients as raw bits) as JSON
 *   dump=paths     print FilterPathInfo[] (audio_filter.c:147-922) as JSON
 */
/* reference headers first (see ref_harness.c on `bool`) */
#include "uhsdr_board.h"
#include "audio_driver.h"
#include "audio_filter.h"
#include "audio_agc.h"
#include "ui_spectrum.h"
#include "filters.h"
#include "cw_decoder.h"
#include "dds_table.h"
#include "audio_management.h"
#include "codec.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

extern __IO TransceiverState ts;
extern const AudioSample_t* oracle_usb_tx_block;
extern SpectrumDisplay sd;
extern AudioDriverState ads;
extern AudioDriverBuffer adb;
const arm_biquad_casd_df1_inst_f32* oracle_ref_biquad1(void);
const arm_biquad_casd_df1_inst_f32* oracle_ref_biquad2(void);
const arm_iir_lattice_instance_f32* oracle_ref_prefilter(void);
const arm_iir_lattice_instance_f32* oracle_ref_antialias(void);
const arm_fir_interpolate_instance_f32* oracle_ref_interpolate(void);
const arm_iir_lattice_instance_f32* oracle_ref_squelch(void);
float oracle_ref_notch_mu(void);
const arm_iir_lattice_instance_f32* oracle_ref_tx_lattice(void);
const arm_biquad_casd_df1_inst_f32* oracle_ref_tx_biquad(void);
extern arm_fir_instance_f32 Fir_Tx_Hilbert_I, Fir_Tx_Hilbert_Q;
void oracle_ref_agc_dump(void);
unsigned long oracle_harness_layout(void);
unsigned long oracle_driver_layout(void);
int ref_spec_ring_len(int L);
void ref_spec_setup(int L, int magnify);
void ref_spec_snapshot(float* out);
void ref_spec_frame(int L, int spectrum_filter, const float* ring, float* mag, float* avg);
void ref_spec_dump(void);
extern float oracle_cw_energy_log[4096];
extern int oracle_cw_energy_count;
const Goertzel* oracle_ref_cw_goertzel(void);
const float* oracle_ref_subaudible_table(int* n);
extern const int16_t DDS_TABLE[];

static void print_fvec(const char* name, const float* p, int n, int last);

/* dump=txextra: softdds sine table (softdds/dds_table.c) and the FM sub-audible tone table */
static void dump_txextra(void)
{
    int n = 0;
    const float* t = oracle_ref_subaudible_table(&n);
    printf("{\"dds_table\": [");
    for (int i = 0; i < DDS_TBL_SIZE; ++i) printf("%s%d", i ? "," : "", DDS_TABLE[i]);
    printf("], ");
    print_fvec("subaudible", t, n, 1);
    printf("}\n");
}
extern arm_fir_instance_f32 Fir_Rx_Hilbert_I, Fir_Rx_Hilbert_Q;
extern arm_fir_decimate_instance_f32 DECIMATE_RX_I, DECIMATE_RX_Q;

static const char* arg(int argc, char** argv, const char* key, const char* dflt)
{
    size_t k = strlen(key);
    for (int i = 1; i < argc; i++)
        if (strncmp(argv[i], key, k) == 0 && argv[i][k] == '=') return argv[i] + k + 1;
    return dflt;
}
static long iarg(int argc, char** argv, const char* key, long dflt)
{
    const char* v = arg(argc, argv, key, NULL);
    return v ? strtol(v, NULL, 0) : dflt;
}
static float farg(int argc, char** argv, const char* key, float dflt)
{
    const char* v = arg(argc, argv, key, NULL);
    return v ? strtof(v, NULL) : dflt;
}

static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static void print_fvec(const char* name, const float* p, int n, int last)
{
    printf("  \"%s\": [", name);
    for (int i = 0; i < n; i++) printf("%s%u", i ? "," : "", p ? bits(p[i]) : 0u);
    printf("]%s\n", last ? "" : ",");
}

static void dump_paths(void)
{
    printf("[\n");
    for (int i = 0; i < AUDIO_FILTER_PATH_NUM; i++)
    {
        const FilterPathDescriptor* f = &FilterPathInfo[i];
        printf("{\"index\":%d,\"id\":%u,\"name\":\"%s\",\"mode\":%u,\"select\":%u,\"fir_taps\":%u,"
               "\"sample_rate_dec\":%u,\"offset\":%u,\n", i, f->id, f->name ? f->name : "", f->mode,
               f->filter_select_id, f->FIR_numTaps, f->sample_rate_dec, f->offset);
        print_fvec("fir_i", f->FIR_I_coeff_file, f->FIR_I_coeff_file ? f->FIR_numTaps : 0, 0);
        print_fvec("fir_q", f->FIR_Q_coeff_file, f->FIR_Q_coeff_file ? f->FIR_numTaps : 0, 0);
        print_fvec("dec", f->dec ? f->dec->pCoeffs : NULL, f->dec ? f->dec->numTaps : 0, 0);
        print_fvec("pre_k", f->pre_instance ? f->pre_instance->pkCoeffs : NULL, f->pre_instance ? f->pre_instance->numStages : 0, 0);
        print_fvec("pre_v", f->pre_instance ? f->pre_instance->pvCoeffs : NULL, f->pre_instance ? f->pre_instance->numStages + 1 : 0, 0);
        print_fvec("interp", f->interpolate ? f->interpolate->pCoeffs : NULL, f->interpolate ? f->interpolate->phaseLength : 0, 0);
        print_fvec("aa_k", f->iir_instance ? f->iir_instance->pkCoeffs : NULL, f->iir_instance ? f->iir_instance->numStages : 0, 0);
        print_fvec("aa_v", f->iir_instance ? f->iir_instance->pvCoeffs : NULL, f->iir_instance ? f->iir_instance->numStages + 1 : 0, 1);
        printf("}%s\n", i + 1 < AUDIO_FILTER_PATH_NUM ? "," : "");
    }
    printf("]\n");
}

static void dump_setup(void)
{
    const arm_biquad_casd_df1_inst_f32* b1 = oracle_ref_biquad1();
    const arm_biquad_casd_df1_inst_f32* b2 = oracle_ref_biquad2();
    const arm_iir_lattice_instance_f32* pre = oracle_ref_prefilter();
    const arm_iir_lattice_instance_f32* aa = oracle_ref_antialias();
    const arm_fir_interpolate_instance_f32* ip = oracle_ref_interpolate();
    printf("{\n");
    printf("  \"filter_path\": %u, \"decimation_rate\": %u, \"decimated_freq\": %u,\n",
           ts.filter_path, ads.decimation_rate, (unsigned)ads.decimated_freq);
    printf("  \"hilbert_taps\": %u, \"decim_taps\": %u, \"pre_stages\": %u, \"aa_stages\": %u,"
           " \"interp_L\": %u, \"interp_phase\": %u,\n", Fir_Rx_Hilbert_I.numTaps, DECIMATE_RX_I.numTaps,
           pre->numStages, aa->numStages, ip->L, ip->phaseLength);
    print_fvec("biquad1", b1->pCoeffs, 5 * b1->numStages, 0);
    print_fvec("biquad2", b2->pCoeffs, 5 * b2->numStages, 0);
    print_fvec("interp", ip->pCoeffs, ip->phaseLength * ip->L, 0);
    print_fvec("hilbert_i", Fir_Rx_Hilbert_I.pCoeffs, Fir_Rx_Hilbert_I.numTaps, 0);
    print_fvec("hilbert_q", Fir_Rx_Hilbert_Q.pCoeffs, Fir_Rx_Hilbert_Q.numTaps, 0);
    print_fvec("decim", DECIMATE_RX_I.pCoeffs, DECIMATE_RX_I.numTaps, 0);
    print_fvec("decim_q", DECIMATE_RX_Q.pCoeffs, DECIMATE_RX_Q.numTaps, 0);
    {
        const float sam[8] = { adb.sam.omega_min, adb.sam.omega_max, adb.sam.g1, adb.sam.g2,
                               adb.sam.mtauR, adb.sam.onem_mtauR, adb.sam.mtauI, adb.sam.onem_mtauI };
        print_fvec("sam", sam, 8, 0);
    }
    print_fvec("pre_k", pre->pkCoeffs, pre->numStages, 0);
    print_fvec("pre_v", pre->pvCoeffs, pre->numStages ? pre->numStages + 1 : 0, 0);
    print_fvec("aa_k", aa->pkCoeffs, aa->numStages, 0);
    print_fvec("aa_v", aa->pvCoeffs, aa->numStages ? aa->numStages + 1 : 0, 0);
    const arm_iir_lattice_instance_f32* sq = oracle_ref_squelch();   /* FM squelch HPF, audio_driver.c:481-484 */
    print_fvec("squelch_k", sq->pkCoeffs, sq->numStages, 0);
    print_fvec("squelch_v", sq->pvCoeffs, sq->numStages + 1, 0);
    /* transmit chain (TxProcessor_Set, tx_processor.c:72-120; AudioManagement_CalcTxCompLevel) */
    const arm_iir_lattice_instance_f32* txl = oracle_ref_tx_lattice();
    const arm_biquad_casd_df1_inst_f32* txb = oracle_ref_tx_biquad();
    print_fvec("tx_k", txl->pkCoeffs, txl->numStages, 0);
    print_fvec("tx_v", txl->pvCoeffs, txl->numStages + 1, 0);
    print_fvec("tx_biquad", txb->pCoeffs, 5 * txb->numStages, 0);
    print_fvec("tx_hilbert_i", Fir_Tx_Hilbert_I.pCoeffs, Fir_Tx_Hilbert_I.numTaps, 0);
    print_fvec("tx_hilbert_q", Fir_Tx_Hilbert_Q.pCoeffs, Fir_Tx_Hilbert_Q.numTaps, 0);
    {
        const float alc[2] = { ads.alc_decay, (float)ts.alc_tx_postfilt_gain_var };
        print_fvec("tx_alc", alc, 2, 0);
    }
    {   /* LMS auto notch mu (audio_driver.c:1170), key beep (AudioManagement_KeyBeepPrepare,
           audio_management.c:354-363), FM subaudible tone detector Goertzels (audio_management.c:313-326) */
        const float nm[1] = { oracle_ref_notch_mu() };
        print_fvec("notch_mu", nm, 1, 0);
        printf("  \"beep_step\": %u,\n", (unsigned)ads.beep.step);
        const float bl[1] = { ads.beep_loudness_factor };
        print_fvec("beep_scale", bl, 1, 0);
        const float tg[9] = { ads.fm_conf.goertzel[FM_HIGH].r, ads.fm_conf.goertzel[FM_HIGH].cos, ads.fm_conf.goertzel[FM_HIGH].sin,
                              ads.fm_conf.goertzel[FM_LOW].r, ads.fm_conf.goertzel[FM_LOW].cos, ads.fm_conf.goertzel[FM_LOW].sin,
                              ads.fm_conf.goertzel[FM_CTR].r, ads.fm_conf.goertzel[FM_CTR].cos, ads.fm_conf.goertzel[FM_CTR].sin };
        print_fvec("tone_goertzel", tg, 9, 0);
        printf("  \"tone_det_freq\": %u,\n", bits(ads.fm_conf.subaudible_tone_det_freq));
    }
    {   /* CW decoder Goertzel (CwDecode_Filter_Set via SetProcessingChain, audio_driver.c:1158) */
        const Goertzel* g = oracle_ref_cw_goertzel();
        const float cw[3] = { g->r, g->cos, g->sin };
        print_fvec("cw_goertzel", cw, 3, 1);
    }
    printf("}\n");
}

int main(int argc, char** argv)
{
    const unsigned long mine = (unsigned long)sizeof(TransceiverState) * 100000ul +
                               (unsigned long)((char*)&ts.dsp.active - (char*)&ts);
    if (mine != oracle_driver_layout() || mine != oracle_harness_layout())
    {
        fprintf(stderr, "TransceiverState layout mismatch between TUs (%lu %lu %lu)\n", mine,
                oracle_driver_layout(), oracle_harness_layout());
        return 3;
    }
    const char* dump = arg(argc, argv, "dump", "");
    if (strcmp(dump, "paths") == 0) { dump_paths(); return 0; }
    if (strcmp(dump, "spectrum") == 0) { ref_spec_dump(); return 0; }
    if (strcmp(dump, "txextra") == 0) { dump_txextra(); return 0; }
    if (strcmp(dump, "cmsis") == 0) { extern int ref_cmsis_dump(const char*); return ref_cmsis_dump(arg(argc, argv, "out", ".")); }

    const int mode = (int)iarg(argc, argv, "mode", DEMOD_USB);
    const int path = (int)iarg(argc, argv, "path", 0);
    const int block = (int)iarg(argc, argv, "block", IQ_BLOCK_SIZE);

    /* settings the firmware loads from its config store before AudioDriver_Init
       (drivers/ui/ui_configuration.c:70-230 defaults unless overridden) */
    ts.txrx_mode = TRX_MODE_RX;                    /* src/uhsdr_main.c:181-182 */
    ts.samp_rate = IQ_SAMPLE_RATE;
    ts.dmod_mode = mode;
    ts.rx_iq_source = RX_IQ_CODEC;
    ts.tx_audio_source = iarg(argc, argv, "txsrc", TX_AUDIO_MIC);
    ts.flags1 = iarg(argc, argv, "flags1", 0);
    ts.iq_freq_mode = iarg(argc, argv, "iqmode", FREQ_IQ_CONV_M12KHZ);
    ts.iq_auto_correction = iarg(argc, argv, "iq_auto", 0);
    ts.rx_adj_gain_var.i = farg(argc, argv, "gain_i", 1.0f);
    ts.rx_adj_gain_var.q = farg(argc, argv, "gain_q", 1.0f);
    ads.iq_phase_balance_rx = farg(argc, argv, "phase", 0.0f);
    ts.dsp.active = iarg(argc, argv, "dsp", 0);
    ts.dsp.notch_frequency = iarg(argc, argv, "notch", 800);
    ts.dsp.peak_frequency = iarg(argc, argv, "peak", 750);
    ts.dsp.bass_gain = iarg(argc, argv, "bass", 2);
    ts.dsp.treble_gain = iarg(argc, argv, "treble", 0);
#ifdef USE_TWO_CHANNEL_AUDIO
    ts.stereo_enable = iarg(argc, argv, "stereo", 0);
    if (iarg(argc, argv, "board", 0) != 0) { fprintf(stderr, "board=1 needs the mcHF build (make mchf)\n"); return 2; }
#else
    if (iarg(argc, argv, "board", 1) != 1) { fprintf(stderr, "this is the mcHF build: board=1\n"); return 2; }
#endif
    /* speaker volume and its software gain (UiDriver_TaskHandler_HighPrioTasks, ui_driver.c:3083-3092) */
    ts.rx_gain[RX_AUDIO_SPKR].value = iarg(argc, argv, "spkr", AUDIO_GAIN_DEFAULT);
    ts.rx_gain[RX_AUDIO_SPKR].active_value = 1;
    if (ts.rx_gain[RX_AUDIO_SPKR].value > CODEC_SPEAKER_MAX_VOLUME)
        ts.rx_gain[RX_AUDIO_SPKR].active_value = (((float32_t)ts.rx_gain[RX_AUDIO_SPKR].value) / 2.5) - 5.35;
    /* LMS auto notch (audio_driver.c:1166-1186; defaults audio_driver.h:486-495) */
    ts.dsp.notch_numtaps = DSP_NOTCH_NUMTAPS_DEFAULT;
    ts.dsp.notch_delaybuf_len = DSP_NOTCH_DELAYBUF_DEFAULT;
    ts.dsp.notch_mu = iarg(argc, argv, "notch_mu", DSP_NOTCH_MU_DEFAULT);
    ts.fm_subaudible_tone_det_select = iarg(argc, argv, "tonedet", 0);
    ts.beep_frequency = iarg(argc, argv, "beepfreq", DEFAULT_BEEP_FREQUENCY);
    ts.beep_loudness = iarg(argc, argv, "beeploud", DEFAULT_BEEP_LOUDNESS);
    ts.cw_sidetone_freq = iarg(argc, argv, "sidetone", CW_SIDETONE_FREQ_DEFAULT);   /* CW decoder Goertzel */
    ts.cw_keyer_speed = 20;                        /* CW_KEYER_SPEED_DEFAULT (ui_configuration.h:59) */
    ts.cw_keyer_weight = CW_KEYER_WEIGHT_DEFAULT;
    cw_decoder_config.blocksize = iarg(argc, argv, "cwblock", CW_DECODER_BLOCKSIZE_DEFAULT);
    cw_decoder_config.thresh = iarg(argc, argv, "cwthresh", CW_DECODER_THRESH_DEFAULT);
    cw_decoder_config.noisecancel_enable = iarg(argc, argv, "cwnc", 1);
    ts.cw_keyer_mode = CW_KEYER_MODE_STRAIGHT;
    ts.fm_sql_threshold = iarg(argc, argv, "sql", FM_SQUELCH_DEFAULT);
    if (iarg(argc, argv, "fm5k", 0)) ts.flags2 |= FLAGS2_FM_MODE_DEVIATION_5KHZ;
    ads.sam_sideband = iarg(argc, argv, "sam_sb", SAM_SIDEBAND_BOTH);
    ads.pll_fmax_int = iarg(argc, argv, "pll_fmax", 2500);
    ads.zeta_int = iarg(argc, argv, "zeta", 65);
    ads.omegaN_int = iarg(argc, argv, "omegan", 250);
    ads.fade_leveler = iarg(argc, argv, "fade", 1);
    agc_wdsp_conf.mode = iarg(argc, argv, "agc_mode", 2);
    agc_wdsp_conf.hang_enable = iarg(argc, argv, "agc_hang", 0);
    agc_wdsp_conf.thresh = iarg(argc, argv, "agc_thresh", 20);
    agc_wdsp_conf.slope = iarg(argc, argv, "agc_slope", 70);
    agc_wdsp_conf.tau_decay[0] = 4000;
    agc_wdsp_conf.tau_decay[1] = 2000;
    agc_wdsp_conf.tau_decay[2] = 500;
    agc_wdsp_conf.tau_decay[3] = 250;
    agc_wdsp_conf.tau_decay[4] = 50;
    agc_wdsp_conf.tau_hang_decay = 500;
    sd.fft_iq_len = 0;          /* spectrum tap off unless spec=L (ref_spectrum.c) */
    const int spec = (int)iarg(argc, argv, "spec", 0);
    const int spec_filter = (int)iarg(argc, argv, "specfilt", 4);   /* SPECTRUM_FILTER_DEFAULT */
    const int magnify = (int)iarg(argc, argv, "mag", 0);            /* sd.magnify: zoom 2^mag */
    const long zd = 1L << magnify;                                  /* ring samples per input frame: 1/zd */
    /* transmit settings (hardware/uhsdr_board.h:301-460, defaults ui_configuration.c) */
    const int tx = (int)iarg(argc, argv, "tx", 0);
    ts.tx_mic_gain_mult = iarg(argc, argv, "micmult", 15);
    ts.tx_mic_boost = iarg(argc, argv, "boost", 0);
    ts.tx_comp_level = iarg(argc, argv, "comp", TX_AUDIO_COMPRESSION_DEFAULT);
    ts.alc_decay = ALC_DECAY_DEFAULT;
    ts.alc_tx_postfilt_gain = ALC_POSTFILT_GAIN_DEFAULT;
    ts.tx_filter = iarg(argc, argv, "txfilter", 0);
    ts.fm_subaudible_tone_gen_select = iarg(argc, argv, "subtone", 0);   /* FM_SUBAUDIBLE_TONE_OFF */
    ts.fm_tone_burst_mode = iarg(argc, argv, "burstmode", 0);           /* FM_TONE_BURST_OFF */
    ts.dsp.tx_bass_gain = iarg(argc, argv, "txbass", 4);
    ts.dsp.tx_treble_gain = iarg(argc, argv, "txtreble", 4);
    ts.tx_power_factor = farg(argc, argv, "txpwr", 0.5f);
    ts.tx_adj_gain_var[IQ_TRANS_ON].i = ts.tx_adj_gain_var[IQ_TRANS_OFF].i = farg(argc, argv, "txgi", 1.0f);
    ts.tx_adj_gain_var[IQ_TRANS_ON].q = ts.tx_adj_gain_var[IQ_TRANS_OFF].q = farg(argc, argv, "txgq", 1.0f);
    ads.iq_phase_balance_tx[IQ_TRANS_ON] = ads.iq_phase_balance_tx[IQ_TRANS_OFF] = farg(argc, argv, "txphase", 0.0f);

    ts.filter_path_mem[AudioFilter_GetFilterModeFromDemodMode(mode)][0] = path;

    AudioDriver_Init();
    AudioDriver_SetProcessingChain(mode, false);

    if (strcmp(dump, "setup") == 0) { dump_setup(); return 0; }
    if (strcmp(dump, "agc") == 0) { oracle_ref_agc_dump(); return 0; }

    const long n = iarg(argc, argv, "n", 0);
    const char* in = arg(argc, argv, "in", NULL);
    const char* out_a = arg(argc, argv, "out_a", NULL);
    const char* out_dst = arg(argc, argv, "out_dst", NULL);
    if (!in || n <= 0 || (n % block) != 0) { fprintf(stderr, "need in= and n= (multiple of %d)\n", block); return 2; }

    IqSample_t* iq = malloc(sizeof(IqSample_t) * n);
    AudioSample_t* dst = calloc(n, sizeof(AudioSample_t));
    float* a1 = calloc(n, sizeof(float));
    FILE* f = fopen(in, "rb");
    if (!f || fread(iq, sizeof(IqSample_t), n, f) != (size_t)n) { fprintf(stderr, "read %s failed\n", in); return 2; }
    fclose(f);

    IqSample_t blk[IQ_BLOCK_SIZE];
    long beep0 = -1, beepn = 0;
    {
        const char* b = arg(argc, argv, "beep", NULL);
        if (b && sscanf(b, "%ld:%ld", &beep0, &beepn) != 2) { fprintf(stderr, "beep=b0:K\n"); return 2; }
        if (b) ts.flags2 |= FLAGS2_KEY_BEEP_ENABLE;
    }
    const char* out_a0 = arg(argc, argv, "out_a0", NULL);
    const char* out_clip = arg(argc, argv, "out_clip", NULL);
    const char* out_tp = arg(argc, argv, "out_tp", NULL);
    const long uiperiod = iarg(argc, argv, "uiperiod", 1);
    uint8_t* tps = out_tp ? calloc(n / block, 1) : NULL;
    ts.twinpeaks_tested = TWINPEAKS_WAIT;                  /* src/uhsdr_main.c:339 */
    float* a0s = out_a0 ? calloc(n, sizeof(float)) : NULL;
    uint8_t* clips = out_clip ? calloc(n / block, 1) : NULL;
    const char* out_cw = arg(argc, argv, "out_cw", NULL);        /* Goertzel energy per CW block */
    const char* out_cws = arg(argc, argv, "out_cws", NULL);      /* ads.CW_signal after each call */
    uint8_t* cw_signal = out_cws ? calloc(n / block, 1) : NULL;
    float* stream = NULL;
    int ring = 0;
    if (spec)
    {
        if ((spec != 256 && spec != 512 && spec != 1024) || n % (spec * zd) || magnify < 0 || magnify > 5)
        { fprintf(stderr, "spec=256|512|1024 with spec*2^mag dividing n, mag 0..5\n"); return 2; }
        ring = ref_spec_ring_len(spec);
        ref_spec_setup(spec, magnify);
        stream = calloc(2 * n, sizeof(float));
    }
    if (tx)
    {
        /* TX: the codec's audio frames in, IQ frames out (AudioDriver_I2SCallback TX branch,
           audio_driver.c:3010-3036 -> TxProcessor_Run); the sidetone goes to a scratch buffer */
        ts.txrx_mode = TRX_MODE_TX;
        AudioSample_t ablk[IQ_BLOCK_SIZE], side[IQ_BLOCK_SIZE];
        IqSample_t oblk[IQ_BLOCK_SIZE];
        long tune0 = -1, tunen = 0, tunem = 1, burst0 = -1, burstn = 0;
        {
            const char* t = arg(argc, argv, "tune", NULL);
            if (t && sscanf(t, "%ld:%ld:%ld", &tune0, &tunen, &tunem) != 3) { fprintf(stderr, "tune=t0:K:M\n"); return 2; }
            const char* b = arg(argc, argv, "burst", NULL);
            if (b && sscanf(b, "%ld:%ld", &burst0, &burstn) != 2) { fprintf(stderr, "burst=t0:K\n"); return 2; }
        }
        for (long off = 0; off < n; off += block)
        {
            const long call = off / block;
            if (call == tune0 || (tune0 >= 0 && call == tune0 + tunen))
            {
                ts.tune = call == tune0;
                ts.tune_tone_mode = tunem == 2 ? TUNE_TONE_TWO : TUNE_TONE_SINGLE;
                AudioManagement_SetSidetoneForDemodMode(ts.dmod_mode, ts.tune);
            }
            ads.fm_conf.tone_burst_active = burst0 >= 0 && call >= burst0 && call < burst0 + burstn;
            memcpy(ablk, iq + off, sizeof(AudioSample_t) * block);
            oracle_usb_tx_block = ablk;                     /* the USB sources see the same block */
            AudioDriver_I2SCallback(ablk, oblk, side, block);
            memcpy(dst + off, oblk, sizeof(IqSample_t) * block);
            memcpy(a1 + off, adb.a_buffer[0], sizeof(float) * block);
        }
    }
    else
    for (long off = 0; off < n; off += block)
    {
        memcpy(blk, iq + off, sizeof(IqSample_t) * block);   /* the ISR's DMA half-buffer */
        const long call = off / block;
        if (beep0 >= 0)
        {
            /* AudioManagement_KeyBeep (audio_management.c:368-375) at call b0, then the UI's
               countdown of ts.beep_timing (ui_driver.c:7214-7216) held to K calls */
            if (call == beep0) AudioManagement_KeyBeep();
            ts.beep_timing = (call >= beep0 && call < beep0 + beepn) ? 1 : 0;
        }
        AudioDriver_I2SCallback(dst + off, blk, NULL, block);
        memcpy(a1 + off, adb.a_buffer[1], sizeof(float) * block);
        if (a0s) memcpy(a0s + off, adb.a_buffer[0], sizeof(float) * block);
        if (clips)
        {
            clips[call] = (uint8_t)((ads.adc_clip ? 1 : 0) | (ads.adc_half_clip ? 2 : 0) | (ads.adc_quarter_clip ? 4 : 0));
            ads.adc_clip = ads.adc_half_clip = ads.adc_quarter_clip = 0;
        }
        if (tps) tps[call] = ts.twinpeaks_tested;
        if ((call + 1) % uiperiod == 0 && ts.twinpeaks_tested == TWINPEAKS_CODEC_RESTART)
            ts.twinpeaks_tested = TWINPEAKS_WAIT;          /* ui_driver.c:7422-7426, after Codec_RestartI2S */
        if (cw_signal) cw_signal[off / block] = ads.CW_signal;
        if (spec && (off + block) % (ring / 2 * zd) == 0)  /* the ring holds ring/2 new samples */
            ref_spec_snapshot(stream + 2 * ((off + block) / zd - ring / 2));
    }
    if (spec)
    {
        const char* out_mag = arg(argc, argv, "out_mag", NULL);
        const char* out_avg = arg(argc, argv, "out_avg", NULL);
        float* mag = calloc(n, sizeof(float));
        float* avgs = calloc(n, sizeof(float));
        float avg[1024] = { 0 };                /* sd.FFT_AVGData starts zeroed (global) */
        for (long fr = 0; fr < n / zd / spec; ++fr)
        {
            ref_spec_frame(spec, spec_filter, stream + 2 * fr * spec, mag + fr * spec, avg);
            memcpy(avgs + fr * spec, avg, sizeof(float) * spec);
        }
        if (out_mag) { f = fopen(out_mag, "wb"); fwrite(mag, sizeof(float), n, f); fclose(f); }
        if (out_avg) { f = fopen(out_avg, "wb"); fwrite(avgs, sizeof(float), n, f); fclose(f); }
        free(mag); free(avgs); free(stream);
    }
    if (out_a) { f = fopen(out_a, "wb"); fwrite(a1, sizeof(float), n, f); fclose(f); }
    if (out_cw)
    {
        const int cnt = oracle_cw_energy_count < 4096 ? oracle_cw_energy_count : 4096;
        f = fopen(out_cw, "wb"); fwrite(oracle_cw_energy_log, sizeof(float), cnt, f); fclose(f);
    }
    if (out_cws) { f = fopen(out_cws, "wb"); fwrite(cw_signal, 1, n / block, f); fclose(f); free(cw_signal); }
    if (out_dst) { f = fopen(out_dst, "wb"); fwrite(dst, sizeof(AudioSample_t), n, f); fclose(f); }
    if (a0s) { f = fopen(out_a0, "wb"); fwrite(a0s, sizeof(float), n, f); fclose(f); free(a0s); }
    if (clips) { f = fopen(out_clip, "wb"); fwrite(clips, 1, n / block, f); fclose(f); free(clips); }
    if (tps) { f = fopen(out_tp, "wb"); fwrite(tps, 1, n / block, f); fclose(f); free(tps); }
    free(iq); free(dst); free(a1);
    return 0;
}
