/*
 * ORACLE TEST INFRASTRUCTURE -- forced include (-include) of every TU of the mcHF output-stage
 * variant of the reference build (make -C oracle/ref mchf -> oracle/_ref/mchf/uhsdr_ref).
 *
 * The mcHF board configuration itself does not compile on x86 (its
 * uhsdr_board.h path needs the F4 HAL and mcp23008.h).  Its only effect on the RX chain is the
 * UI board's audio output: no USE_TWO_CHANNEL_AUDIO (UHSDR_UI_ovi40_config.h:45 defines it for
 * OVI40 only) and UI_BRD_MCHF (the speaker software gain, audio_driver.c:2880-2885, and
 * CODEC_SPEAKER_MAX_VOLUME 16, codec.h:26-27).  So the OVI40 build's board configuration is read
 * first -- its include guard then keeps it from being re-read -- and those two macros are
 * switched to the mcHF setting before any reference source sees them.  The reference sources
 * are compiled unmodified from /root/reference.
 */
#include "uhsdr_board_config.h"
#undef USE_TWO_CHANNEL_AUDIO
#undef UI_BRD_OVI40
#define UI_BRD_MCHF
