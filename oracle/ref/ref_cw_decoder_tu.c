/*
 * ORACLE TEST INFRASTRUCTURE -- compiles the reference's CW decoder (drivers/audio/cw/
 * cw_decoder.c) for the x86 host, included from where it lies (nothing copied).
 *
 * The RX chain calls CwDecode_RxProcessor (audio_driver.c:2555) on a_buffer[0] at 12 ksps in
 * CW / AM / SAM.  The Goertzel energy of each block (cw_decoder.c:199-204) is a local of
 * CW_Decode_exe; to observe it, the call to AudioFilter_GoertzelEnergy is routed through a
 * recorder that calls the reference function (audio_filter.c:1296-1305) and keeps its result.
 */
#include "uhsdr_board_config.h"
#include "audio_filter.h"

float32_t oracle_cw_goertzel_energy(Goertzel* goertzel);
#define AudioFilter_GoertzelEnergy oracle_cw_goertzel_energy
#include "cw_decoder.c"
#undef AudioFilter_GoertzelEnergy

float oracle_cw_energy_log[4096];
int oracle_cw_energy_count;

float32_t oracle_cw_goertzel_energy(Goertzel* goertzel)
{
    const float32_t e = AudioFilter_GoertzelEnergy(goertzel);
    if (oracle_cw_energy_count < 4096) oracle_cw_energy_log[oracle_cw_energy_count] = e;
    oracle_cw_energy_count++;
    return e;
}

const Goertzel* oracle_ref_cw_goertzel(void) { return &cw_goertzel; }
