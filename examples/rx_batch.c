/*
 * rx_batch -- plain C host for libuhsdr_amd.so (no HIP headers, gcc only).
 *
 * What a firmware-side integration looks like: configure the receiver exactly as
 * AudioDriver_SetProcessingChain would (uhsdr_rx_config, drivers/ui/ui_configuration.c
 * defaults), then feed IqSample_t frames of C channels in calls of `frames` frames -- each
 * call standing for frames/32 AudioDriver_I2SCallback invocations per channel
 * (drivers/audio/audio_driver.c:2962-3049) -- and collect adb.a_buffer[1] audio.
 *
 *   rx_batch <iq.bin> <audio.bin> <channels> <total_frames> <frames_per_call> [filter_path [dmod_mode]]
 *     iq.bin     int32 [channels][total_frames][2]   ({l = I, r = Q} per frame)
 *     audio.bin  f32   [channels][total_frames]      (written)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "uhsdr.h"

static int fail(const char* what, uhsdr_status st)
{
    fprintf(stderr, "%s failed (%d): %s\n", what, (int)st, uhsdr_last_error());
    return 1;
}

int main(int argc, char** argv)
{
    if (argc < 6)
    {
        fprintf(stderr, "usage: %s iq.bin audio.bin channels total_frames frames_per_call [filter_path [dmod_mode]]\n"
                        "library: %s\n", argv[0], uhsdr_version());
        return 2;
    }
    const int C = atoi(argv[3]), total = atoi(argv[4]), N = atoi(argv[5]);
    uhsdr_rx_config cfg;
    uhsdr_rx_config_default(&cfg);
    if (argc > 6) cfg.filter_path = atoi(argv[6]);
    if (argc > 7) cfg.dmod_mode = atoi(argv[7]);
    if (C <= 0 || N <= 0 || total % N) { fprintf(stderr, "total_frames must be a multiple of frames_per_call\n"); return 2; }

    int32_t* iq = malloc(sizeof(int32_t) * 2 * (size_t)C * total);
    float* audio = malloc(sizeof(float) * (size_t)C * total);
    int32_t* blk = malloc(sizeof(int32_t) * 2 * (size_t)C * N);
    float* ablk = malloc(sizeof(float) * (size_t)C * N);
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(iq, sizeof(int32_t) * 2, (size_t)C * total, f) != (size_t)C * total) { fprintf(stderr, "read %s\n", argv[1]); return 2; }
    fclose(f);

    uhsdr_rx_handle h;
    uhsdr_status st = uhsdr_rx_create(&cfg, C, N, NULL, &h);
    if (st != UHSDR_OK) return fail("uhsdr_rx_create", st);
    void* d_iq = uhsdr_device_alloc(sizeof(int32_t) * 2 * (uint64_t)C * N);
    void* d_audio = uhsdr_device_alloc(sizeof(float) * (uint64_t)C * N);
    if (!d_iq || !d_audio) return fail("uhsdr_device_alloc", UHSDR_DEVICE_ERROR);

    for (int off = 0; off < total; off += N)
    {
        for (int c = 0; c < C; ++c)          /* this call's frames of every channel, [C][N][2] */
            memcpy(blk + (size_t)c * N * 2, iq + ((size_t)c * total + off) * 2, sizeof(int32_t) * 2 * N);
        if ((st = uhsdr_copy_to_device(d_iq, blk, sizeof(int32_t) * 2 * (uint64_t)C * N)) != UHSDR_OK) return fail("copy in", st);
        if ((st = uhsdr_rx_process(h, d_iq, d_audio, NULL)) != UHSDR_OK) return fail("uhsdr_rx_process", st);
        if ((st = uhsdr_rx_synchronize(h)) != UHSDR_OK) return fail("uhsdr_rx_synchronize", st);
        if ((st = uhsdr_copy_to_host(ablk, d_audio, sizeof(float) * (uint64_t)C * N)) != UHSDR_OK) return fail("copy out", st);
        for (int c = 0; c < C; ++c)
            memcpy(audio + (size_t)c * total + off, ablk + (size_t)c * N, sizeof(float) * N);
    }
    f = fopen(argv[2], "wb");
    if (!f || fwrite(audio, sizeof(float), (size_t)C * total, f) != (size_t)C * total) { fprintf(stderr, "write %s\n", argv[2]); return 2; }
    fclose(f);
    uhsdr_device_free(d_iq);
    uhsdr_device_free(d_audio);
    uhsdr_rx_destroy(h);
    free(iq); free(audio); free(blk); free(ablk);
    return 0;
}
