/*
 * Internal declarations shared by the host setup layer and the device runtime.
 */
#ifndef UHSDR_INTERNAL_H
#define UHSDR_INTERNAL_H

#include <stdint.h>
#include "../../include/uhsdr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One FilterPathDescriptor (drivers/audio/audio_filter.h:108-136), tables as raw bits. */
typedef struct
{
    uint8_t id;                 /* FilterInfo index (bandwidth) */
    uint16_t mode;              /* FILTER_MASK_* of applicable filter modes */
    uint8_t sample_rate_dec;    /* RX_DECIMATION_RATE_{12,24,48}KHZ == 4, 2, 1 */
    uint16_t fir_taps;
    const uint32_t* fir_i;
    const uint32_t* fir_q;
    uint16_t dec_taps;
    const uint32_t* dec;
    uint16_t pre_stages;
    const uint32_t* pre_k;
    const uint32_t* pre_v;
    uint16_t interp_taps;       /* the descriptor's `phaseLength` field, really numTaps */
    const uint32_t* interp;
    uint16_t aa_stages;
    const uint32_t* aa_k;
    const uint32_t* aa_v;
} uhsdr_filter_path_desc;

extern const uhsdr_filter_path_desc uhsdr_filter_paths[UHSDR_FILTER_PATH_NUM];

typedef struct
{
    uint16_t stages;
    const uint32_t* k;
    const uint32_t* v;
} uhsdr_lattice_desc;

extern const uhsdr_lattice_desc uhsdr_tx_lattices[4];
extern const int16_t uhsdr_dds_table[1024];
extern const uint32_t* const uhsdr_fm_subaudible;
extern const int uhsdr_fm_subaudible_count;
extern const uint32_t* const uhsdr_tx_hilbert_i;
extern const uint32_t* const uhsdr_tx_hilbert_q;
extern const int uhsdr_tx_hilbert_taps;

/* spectrum display tables (tools/gen_filter_tables.py from tests/golden/spectrum_tables.json) */
typedef struct
{
    int fft_len, window_formula;
    const uint32_t* twiddle;      /* 2L floats */
    const uint32_t* window;       /* 2L floats */
    const uint16_t* bitrev;
    int bitrev_len;
} uhsdr_spectrum_desc;
extern const uhsdr_spectrum_desc uhsdr_spectrum_tables[3];
typedef struct
{
    int decimation, taps;
    const uint32_t* biquad;       /* 4 stages x {b0, b1, b2, a1, a2} */
    const uint32_t* fir;          /* taps */
} uhsdr_zoom_desc;
extern const uhsdr_zoom_desc uhsdr_zoom_tables[5];

int uhsdr_rx_mode_supported(const uhsdr_rx_plan* p);

/* thread-local last error text for uhsdr_last_error() */
void uhsdr_set_error(const char* fmt, ...);

#ifdef __cplusplus
}
#endif
#endif
