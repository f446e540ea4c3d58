// The firmware's ISR entry, AudioDriver_I2SCallback (drivers/audio/audio_driver.c:2962-3049),
// for one transceiver over the batched device chains (include/uhsdr.h, uhsdr_i2s_*): the RX /
// TX switch, the first-call-after-switch silencing, the input-mute counter and the TX
// PrepareRun, around one uhsdr_rx_process / uhsdr_tx_process of a single channel.  Host code
// only; the DSP runs in the rx / tx kernels.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "uhsdr_internal.h"

struct uhsdr_i2s_s
{
    uhsdr_rx_handle rx;
    uhsdr_tx_handle tx;
    int B;
    hipStream_t stream;
    int32_t* d_iq;           // [B][2]
    int32_t* d_audio;        // [B][2]  RX codec frames / TX mic-line frames
    int txrx_mode;           // ts.txrx_mode
    int mute_counter;        // ts.audio_processor_input_mute_counter
    bool to_rx, to_tx;       // the callback's statics (audio_driver.c:2964-2965)
};

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { uhsdr_set_error("%s: %s", #x, hipGetErrorString(e_)); return UHSDR_DEVICE_ERROR; } } while (0)

extern "C" uhsdr_status uhsdr_i2s_destroy(uhsdr_i2s_handle h)
{
    if (!h) return UHSDR_ARGUMENT_ERROR;
    if (h->rx) uhsdr_rx_destroy(h->rx);
    if (h->tx) uhsdr_tx_destroy(h->tx);
    if (h->d_iq) (void)hipFree(h->d_iq);
    if (h->d_audio) (void)hipFree(h->d_audio);
    free(h);
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_i2s_create(const uhsdr_rx_config* rx, const uhsdr_tx_config* tx, int32_t block_size,
                                         void* stream, uhsdr_i2s_handle* out)
{
    if (!rx || !out || block_size <= 0) { uhsdr_set_error("bad argument"); return UHSDR_ARGUMENT_ERROR; }
    *out = nullptr;
    uhsdr_i2s_s* h = (uhsdr_i2s_s*)calloc(1, sizeof(uhsdr_i2s_s));
    if (!h) return UHSDR_DEVICE_ERROR;
    h->B = block_size;
    h->stream = (hipStream_t)stream;
    uhsdr_status st = uhsdr_rx_create(rx, 1, block_size, stream, &h->rx);
    if (st == UHSDR_OK && tx) st = uhsdr_tx_create(tx, 1, block_size, stream, &h->tx);
    if (st == UHSDR_OK && (hipMalloc((void**)&h->d_iq, sizeof(int32_t) * 2 * block_size) != hipSuccess ||
                           hipMalloc((void**)&h->d_audio, sizeof(int32_t) * 2 * block_size) != hipSuccess))
    {
        uhsdr_set_error("hipMalloc failed");
        st = UHSDR_DEVICE_ERROR;
    }
    if (st != UHSDR_OK)
    {
        uhsdr_i2s_destroy(h);
        return st;
    }
    *out = h;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_i2s_set_txrx_mode(uhsdr_i2s_handle h, int32_t txrx_mode)
{
    if (!h || txrx_mode < 0 || txrx_mode > 1 || (txrx_mode == 1 && !h->tx)) return UHSDR_ARGUMENT_ERROR;
    h->txrx_mode = txrx_mode;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_i2s_set_input_mute(uhsdr_i2s_handle h, int32_t calls)
{
    if (!h || calls < 0) return UHSDR_ARGUMENT_ERROR;
    h->mute_counter = calls;
    return UHSDR_OK;
}

extern "C" uhsdr_status uhsdr_i2s_callback(uhsdr_i2s_handle h, int32_t* audio, int32_t* iq, int32_t* audioDst,
                                           int16_t blockSize)
{
    if (!h || !audio || !iq) { uhsdr_set_error("null argument"); return UHSDR_ARGUMENT_ERROR; }
    if (blockSize != h->B) { uhsdr_set_error("blockSize %d, handle made for %d", blockSize, h->B); return UHSDR_LENGTH_ERROR; }
    const size_t bytes = sizeof(int32_t) * 2 * (size_t)blockSize;
    bool muted = false;
    if (h->txrx_mode == 0)
    {
        if (h->to_rx || h->mute_counter > 0)              // audio_driver.c:2975-2988
        {
            muted = true;
            memset(iq, 0, bytes);                         // AudioDriver_IqFillSilence, in the DMA buffer
            if (h->mute_counter > 0) h->mute_counter--;
            h->to_rx = false;
        }
        HIPCHK(hipMemcpyAsync(h->d_iq, iq, bytes, hipMemcpyHostToDevice, h->stream));
        uhsdr_status st = uhsdr_rx_process(h->rx, h->d_iq, nullptr, h->d_audio);
        if (st != UHSDR_OK) return st;
        HIPCHK(hipMemcpyAsync(audio, h->d_audio, bytes, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        if (muted) memset(audio, 0, bytes);               // external_mute (:2845-2853, 2904-2908)
        h->to_tx = true;
    }
    else
    {
        if (h->to_tx)
        {
            uhsdr_status st = uhsdr_tx_prepare_run(h->tx);   // TxProcessor_PrepareRun (:3012-3015)
            if (st != UHSDR_OK) return st;
        }
        if (h->to_tx || h->mute_counter > 0)              // :3016-3025
        {
            muted = true;
            memset(audio, 0, bytes);                      // AudioDriver_AudioFillSilence
            h->to_tx = false;
            if (h->mute_counter > 0) h->mute_counter--;
        }
        if (muted)
            memset(iq, 0, bytes);                         // chain skipped, zero I/Q (tx_processor.c:946-949, 1018-1022)
        else
        {
            HIPCHK(hipMemcpyAsync(h->d_audio, audio, bytes, hipMemcpyHostToDevice, h->stream));
            uhsdr_status st = uhsdr_tx_process(h->tx, h->d_audio, h->d_iq, nullptr);
            if (st != UHSDR_OK) return st;
            HIPCHK(hipMemcpyAsync(iq, h->d_iq, bytes, hipMemcpyDeviceToHost, h->stream));
            HIPCHK(hipStreamSynchronize(h->stream));
        }
        if (audioDst) memset(audioDst, 0, bytes);         // sidetone: voice modes use none (:1026)
        h->to_rx = true;
    }
    return UHSDR_OK;
}
