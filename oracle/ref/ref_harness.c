/*
 * ORACLE TEST INFRASTRUCTURE -- the environment the reference audio driver expects.
 *
 * On the radio, the audio driver (drivers/audio/*.c, compiled unmodified from
 * /root/reference) is surrounded by the control plane (UI, menus, USB, CAT, FreeDV,
 * CW/RTTY/PSK modems, codec DMA).  Those subsystems are out of scope (SURVEY.md §2
 * rows 11-22) and are not compiled.  This file provides, for the host build only:
 *   - the global state objects those subsystems own (ts, sd, mmb, ...), zero-initialised
 *     and then configured by oracle/ref/ref_main.c exactly as the firmware's config
 *     loader would;
 *   - the control-plane callbacks the driver invokes, as no-ops.  Each is a hook whose
 *     feature is disabled in every oracle configuration (NR, FreeDV, modems, CW decoder,
 *     USB audio, LEDs), so none of them can influence the DSP samples;
 *   - three one-line radio_management.c / ui_driver.c predicates, restated verbatim in
 *     behaviour (citations inline), because their TUs drag in the whole UI/HAL.
 * No DSP arithmetic lives here: every sample the oracle produces is computed by the
 * reference's own audio_driver.c / audio_agc.c / freq_shift.c / CMSIS-DSP code.
 */
/* Reference headers first and no <stdbool.h>: the firmware's own `bool` is
   `typedef int bool` (hardware/uhsdr_types.h:38-39) and TransceiverState must have the same
   layout here as in audio_driver.c (checked at start-up by ref_main.c). */
#include "uhsdr_board.h"
#include "audio_driver.h"
#include "ui_spectrum.h"
#include "freedv_uhsdr.h"
#include "profiling.h"
#include "radio_management.h"
#include "rb.h"
#include <stdint.h>

__IO TransceiverState ts;
SpectrumDisplay sd;
MultiModeBuffer_t mmb;
EventProfile_t eventProfile;
freedv_conf_t freedv_conf;
RingBuffer_data_t fdv_audio_rb;
RingBuffer_data_t fdv_demod_rb;
RingBuffer_data_t fdv_iq_rb;

/* drivers/ui/ui_driver.c:405-433 */
bool is_dsp_nb_active(void) { return false; /* is_dsp_nb() && nb_setting > 0; NB is off in all oracle configs */ }
bool is_dsp_nr(void) { return (ts.dsp.active & DSP_NR_ENABLE) != 0; }
bool is_dsp_mnotch(void) { return (ts.dsp.active & DSP_MNOTCH_ENABLE) != 0; }
bool is_dsp_mpeak(void) { return (ts.dsp.active & DSP_MPEAK_ENABLE) != 0; }

/* drivers/ui/radio_management.c:1643-1663 */
bool RadioManagement_UsesBothSidebands(uint16_t dmod_mode)
{
    bool retval = (dmod_mode == DEMOD_AM)
               || (dmod_mode == DEMOD_SAM && (ads.sam_sideband == SAM_SIDEBAND_BOTH))
               || (dmod_mode == DEMOD_FM);
#ifdef USE_TWO_CHANNEL_AUDIO
    retval = retval || (dmod_mode == DEMOD_SSBSTEREO) || (dmod_mode == DEMOD_IQ)
               || (dmod_mode == DEMOD_SAM && ads.sam_sideband == SAM_SIDEBAND_STEREO);
#endif
    return retval;
}

/* drivers/ui/radio_management.c:1665-1692 */
bool RadioManagement_LSBActive(uint16_t dmod_mode)
{
    switch (dmod_mode)
    {
    case DEMOD_SAM:  return ads.sam_sideband == SAM_SIDEBAND_LSB;
    case DEMOD_LSB:  return true;
    case DEMOD_CW:   return ts.cw_lsb;
    case DEMOD_DIGI: return ts.digi_lsb;
    default:         return false;
    }
}

/* drivers/ui/radio_management.c:1962-1965 */
bool RadioManagement_FmDevIs5khz(void) { return (ts.flags2 & FLAGS2_FM_MODE_DEVIATION_5KHZ) != 0; }

unsigned long oracle_harness_layout(void) { return (unsigned long)sizeof(TransceiverState) * 100000ul + (unsigned long)((char*)&ts.dsp.active - (char*)&ts); }

/* drivers/ui/radio_management.c:587-605 (no FreeDV/PSK/RTTY in oracle configs) */
bool RadioManagement_IsTxAtZeroIF(uint8_t dmod_mode, uint8_t digital_mode)
{
    (void)digital_mode;
    return dmod_mode == DEMOD_CW;
}
/* drivers/ui/radio_management.c:450-453 (no RTTY/PSK/tune in oracle configs) */
bool RadioManagement_UsesTxSidetone(void) { return ts.dmod_mode == DEMOD_CW; }

/* ---- control-plane hooks (features disabled in every oracle configuration) ---- */
void Board_GreenLed(ledstate_t s) { (void)s; }


int32_t FreeDV_Iq_Get_FrameLen(void) { return 0; }
void NR_Init(void) {}
bool NR_in_buffer_add(void* c) { (void)c; return false; }
bool NR_out_buffer_peek(void** c) { (void)c; return false; }
bool NR_out_buffer_remove(void** c) { (void)c; return false; }
bool NR_out_has_data(void) { return false; }
void Psk_Modem_Init(uint32_t output_sample_rate) { (void)output_sample_rate; }
void Psk_Demodulator_ProcessSample(float32_t sample) { (void)sample; }
int16_t Psk_Modulator_GenSample(void) { return 0; }
void UhsdrHwI2s_Codec_ClearTxDmaBuffer(void) {}
void UiDriver_Callback_AudioISR(void) {}
/* the USB audio the TX chain reads for ts.tx_audio_source DIG / DIGIQ (tx_processor.c:929-938):
   the harness points this at the call's input block (ref_main.c, txsrc=) */
const AudioSample_t* oracle_usb_tx_block;
void UsbdAudio_FillTxBuffer(AudioSample_t* buffer, uint32_t len)
{
    for (uint32_t i = 0; i < len; i++) buffer[i] = oracle_usb_tx_block ? oracle_usb_tx_block[i] : (AudioSample_t){ 0, 0 };
}
void UsbdAudio_PutSample(int16_t sample) { (void)sample; }

/* hardware / CAT / UI / digital-mode hooks of the CW keyer and decoder (cw_gen.c, cw_decoder.c):
   no key lines pressed, no CAT, no text output, empty digital-mode TX buffer */
#include "uhsdr_digi_buffer.h"
bool Board_DitLinePressed(void) { return false; }
bool Board_PttDahLinePressed(void) { return false; }
void Board_RedLed(ledstate_t state) { (void)state; }
bool CatDriver_CWKeyPressed(void) { return false; }
bool CatDriver_CatPttActive(void) { return false; }
uint8_t DigiModes_TxBufferHasDataFor(digi_buff_consumer_t consumer) { (void)consumer; return 0; }
bool DigiModes_TxBufferRemove(uint8_t* c_ptr, digi_buff_consumer_t consumer) { (void)c_ptr; (void)consumer; return false; }
int32_t DigiModes_TxBufferPutChar(uint8_t c, digi_buff_consumer_t source) { (void)c; (void)source; return 0; }
void DigiModes_TxBufferPutSign(const char* s, digi_buff_consumer_t source) { (void)s; (void)source; }
void RadioManagement_Request_TxOn(void) {}
void RadioManagement_Request_TxOff(void) {}
void UiDriver_TextMsgPutChar(char ch) { (void)ch; }
