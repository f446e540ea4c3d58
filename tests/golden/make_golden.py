#!/usr/bin/env python3
"""Generate the golden RX-chain fixtures from the reference firmware itself.

Runs ``oracle/_ref/uhsdr_ref`` -- the reference's own audio_driver.c / audio_agc.c /
freq_shift.c / CMSIS-DSP compiled for x86 by ``oracle/ref/Makefile`` -- once per channel
(one process per channel: the firmware keeps DSP state in globals/statics) and stores

    tests/golden/rx_<name>.npz
        iq      int32 [C, N, 2]   IqSample_t frames fed to AudioDriver_I2SCallback
        a1      f32   [C, N]      adb.a_buffer[1] after every 32-frame call
        dst     int32 [C, N, 2]   AudioSample_t frames the driver wrote for the codec
        setup   json             configured chain, coefficient bits (dump=setup)
        agc     json             AudioAgc_SetupAgcWdsp parameter block bits (dump=agc)
        args    json             the uhsdr_ref key=value configuration

plus tests/golden/filter_paths.json (FilterPathInfo[], audio_filter.c:147-922, as raw
float bits), the TX / spectrum / CW fixtures (tx_*, spec_*, cw_*.npz) and
tests/golden/cmsis_vectors.npz (CMSIS-DSP f32 call sequences, dump=cmsis, oracle/ref/ref_cmsis.c),
and the status fixtures (st_*.npz: per-call ADC clip flags and twin-peaks state over >130k
frames; the input is regenerated from uhsdr_amd.synth and checked by its crc32).  Only runs where /root/reference exists (build container); the fixtures
are committed and the GPU box never needs the reference.

    python tests/golden/make_golden.py [--only NAME]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from uhsdr_amd import synth  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "uhsdr_ref")
# the mcHF output-stage variant (single-channel audio; make -C oracle/ref mchf), for board=1
REF_MCHF = os.path.join(ROOT, "oracle", "_ref", "mchf", "uhsdr_ref")


def ref_bin(args: dict) -> str:
    return REF_MCHF if int(args.get("board", 0)) == 1 else REF
NCH = 4
NFRAMES = 2048

# name -> (uhsdr_ref args, signal kwargs)
CONFIGS = {
    "p48_usb": ({"mode": 0, "path": 48}, {}),
    "p48_lsb": ({"mode": 1, "path": 48}, {"lsb": True}),
    "p48_c1": ({"mode": 0, "path": 48}, {"kind": "c1"}),
    "p35_usb": ({"mode": 0, "path": 35}, {}),
    "p55_usb": ({"mode": 0, "path": 55}, {}),
    "p61_usb": ({"mode": 0, "path": 61}, {}),
    "p44_usb": ({"mode": 0, "path": 44}, {}),
    "p4_cw": ({"mode": 2, "path": 4}, {}),
    "p48_iqauto": ({"mode": 0, "path": 48, "iq_auto": 1}, {}),
    "p48_iqman": ({"mode": 0, "path": 48, "gain_i": 1.03125, "gain_q": 0.96875, "phase": -0.0125}, {}),
    "p48_iqman2": ({"mode": 0, "path": 48, "gain_i": 0.98, "gain_q": 1.01, "phase": 0.02}, {}),
    "p48_eq": ({"mode": 0, "path": 48, "dsp": 0x30, "bass": -6, "treble": 4, "notch": 1200, "peak": 900}, {}),
    "p48_agcoff": ({"mode": 0, "path": 48, "agc_mode": 5}, {}),
    "p48_agcfast": ({"mode": 0, "path": 48, "agc_mode": 4, "agc_thresh": 40, "agc_slope": 30}, {}),
    "p48_agchang": ({"mode": 0, "path": 48, "agc_mode": 1, "agc_hang": 1}, {}),
    "p48_agcfrank": ({"mode": 0, "path": 48, "agc_mode": 0}, {}),
    "p48_p12k": ({"mode": 0, "path": 48, "iqmode": 3}, {"center": -12000.0}),
    "p48_m6k": ({"mode": 0, "path": 48, "iqmode": 2}, {"carrier": 6000.0}),
    "p48_p6k": ({"mode": 0, "path": 48, "iqmode": 1}, {"center": -6000.0}),
    "p48_off": ({"mode": 0, "path": 48, "iqmode": 0}, {"center": 0.0}),
    # AM / SAM (C3): AM carrier at +12 kHz +- 200 Hz, 50 % modulation with a 1 kHz tone
    "p70_am": ({"mode": 3, "path": 70}, {"am": True}),
    "p70_sam": ({"mode": 4, "path": 70}, {"am": True}),
    "p70_sam_nofade": ({"mode": 4, "path": 70, "fade": 0}, {"am": True}),
    "p70_sam_dx": ({"mode": 4, "path": 70, "zeta": 20, "omegan": 70, "pll_fmax": 1000}, {"am": True}),
    "p75_sam": ({"mode": 4, "path": 75}, {"am": True}),
    "p83_am": ({"mode": 3, "path": 83}, {"am": True}),
    "p86_sam": ({"mode": 4, "path": 86}, {"am": True}),
    "p70_sam_agcoff": ({"mode": 4, "path": 70, "agc_mode": 5}, {"am": True}),
    "p70_sam_usb": ({"mode": 4, "path": 70, "sam_sb": 2}, {"am": True}),
    "p70_sam_lsb": ({"mode": 4, "path": 70, "sam_sb": 1}, {"am": True}),
    # FM (C4): 1 kHz tone at 2.5 kHz deviation; 8192 frames = 256 calls, so the squelch
    # (evaluated every 200 calls, audio_driver.c:1605) decides once inside the fixture
    "p1_fm": ({"mode": 5, "path": 1}, {"fm": True, "frames": 8192}),
    "p1_fm_sql0": ({"mode": 5, "path": 1, "sql": 0}, {"fm": True, "frames": 8192}),
    "p2_fm5k": ({"mode": 5, "path": 2, "sql": 2, "fm5k": 1}, {"fm": True, "frames": 8192, "deviation": 5000.0}),
    "p3_fm_noise": ({"mode": 5, "path": 3, "sql": 18}, {"fm": True, "frames": 8192, "amplitude": 40.0}),
    # LMS auto notch (DSP_NOTCH_ENABLE = 4; AudioDriver_NotchFilter, audio_driver.c:1746-1763,
    # called at :2443-2456 except in CW and in SAM at 24 ksps)
    "p48_notch": ({"mode": 0, "path": 48, "dsp": 4}, {}),
    "p48_notch_mu25_lsb": ({"mode": 1, "path": 48, "dsp": 4 | 0x30, "notch_mu": 25}, {"lsb": True}),
    "p35_notch": ({"mode": 0, "path": 35, "dsp": 4, "notch_mu": 3}, {}),
    "p55_notch": ({"mode": 0, "path": 55, "dsp": 4, "notch_mu": 40}, {}),
    "p70_am_notch": ({"mode": 3, "path": 70, "dsp": 4}, {"am": True}),
    "p70_sam_notch": ({"mode": 4, "path": 70, "dsp": 4, "notch_mu": 20}, {"am": True}),
    "p83_am_notch": ({"mode": 3, "path": 83, "dsp": 4}, {"am": True}),
    "p83_sam_notch": ({"mode": 4, "path": 83, "dsp": 4}, {"am": True}),
    "p4_cw_notch": ({"mode": 2, "path": 4, "dsp": 4}, {}),
    # key beep (audio_driver.c:2891-2898, softdds): AudioManagement_KeyBeep at call b0, tone for
    # K calls (beep=b0:K; b0 on an 8-call boundary so 256-frame device calls can replay it)
    "p48_beep": ({"mode": 0, "path": 48, "beep": "8:20"}, {}),
    "p48_beep_loud": ({"mode": 0, "path": 48, "beep": "0:64", "beepfreq": 740, "beeploud": 20}, {}),
    "p70_sam_beep": ({"mode": 4, "path": 70, "beep": "16:33", "beepfreq": 1750}, {"am": True}),
    "p1_fm_beep": ({"mode": 5, "path": 1, "sql": 0, "beep": "40:100"}, {"fm": True, "frames": 8192}),
    # FM subaudible tone detector (audio_driver.c:1665-1734): Goertzel window of 400 calls,
    # debounce 2, so 1280 calls (40960 frames) see three detector decisions
    "p1_fm_tone": ({"mode": 5, "path": 1, "tonedet": 10}, {"fm": True, "frames": 40960, "subtone": 91.5, "nch": 2}),
    "p1_fm_tone_absent": ({"mode": 5, "path": 1, "tonedet": 10, "sql": 0}, {"fm": True, "frames": 40960, "nch": 2}),
    # OVI40 two-channel audio (USE_TWO_CHANNEL_AUDIO, use_stereo at audio_driver.c:2618): SSB stereo
    # (a_buffer[0] = I + Q, [1] = I - Q), IQ (I, Q), SAM stereo (LSB, USB); a0 stored too
    "p48_ssbstereo": ({"mode": 7, "path": 48, "stereo": 1}, {}),
    "p35_ssbstereo": ({"mode": 7, "path": 35, "stereo": 1}, {}),
    "p55_ssbstereo": ({"mode": 7, "path": 55, "stereo": 1, "agc_mode": 4}, {}),
    "p48_iq_stereo": ({"mode": 8, "path": 48, "stereo": 1, "dsp": 0x30}, {}),
    "p35_iq_stereo": ({"mode": 8, "path": 35, "stereo": 1, "agc_mode": 5}, {}),
    "p48_iq_mono": ({"mode": 8, "path": 48}, {}),
    "p48_ssbstereo_mono": ({"mode": 7, "path": 48}, {}),
    "p70_sam_stereo": ({"mode": 4, "path": 70, "sam_sb": 3, "stereo": 1}, {"am": True}),
    "p83_sam_stereo": ({"mode": 4, "path": 83, "sam_sb": 3, "stereo": 1, "fade": 0}, {"am": True}),
    # mcHF (board=1: the reference built without USE_TWO_CHANNEL_AUDIO, with UI_BRD_MCHF): a_buffer[0]
    # = 10 x a_buffer[1] (line out), the speaker's software gain above volume 16, the key beep on
    # a_buffer[1] only (audio_driver.c:2870-2897); a0 stored too
    "p48_usb_mchf": ({"mode": 0, "path": 48, "board": 1}, {}),
    "p48_beep_mchf_spkr24": ({"mode": 0, "path": 48, "board": 1, "spkr": 24, "beep": "8:20"}, {}),
    "p35_lsb_mchf_spkr30": ({"mode": 1, "path": 35, "board": 1, "spkr": 30}, {"lsb": True}),
    "p70_sam_mchf_beep": ({"mode": 4, "path": 70, "board": 1, "spkr": 17, "beep": "16:33"}, {"am": True}),
    "p1_fm_mchf_beep": ({"mode": 5, "path": 1, "board": 1, "sql": 0, "spkr": 20, "beep": "40:100"},
                        {"fm": True, "frames": 8192}),
    "p1_fm_mchf_squelched": ({"mode": 5, "path": 1, "board": 1, "spkr": 28, "beep": "8:20"}, {"fm": True, "frames": 4096}),
    "p70_sam_stereo_mono": ({"mode": 4, "path": 70, "sam_sb": 3}, {"am": True}),
    "p48_ssbstereo_notch_beep": ({"mode": 7, "path": 48, "stereo": 1, "dsp": 4, "beep": "16:20"}, {}),
    "p70_sam_stereo_notch": ({"mode": 4, "path": 70, "sam_sb": 3, "stereo": 1, "dsp": 4}, {"am": True}),
    "p2_fm_tone_sql3": ({"mode": 5, "path": 2, "tonedet": 10, "fm5k": 1, "sql": 3},
                        {"fm": True, "frames": 40960, "subtone": 91.5, "deviation": 5000.0, "nch": 2}),
}

# SSB transmit (C4, TxProcessor_Run): microphone two-tone in, IQ frames out (tests/golden/tx_*.npz)
TX_CONFIGS = {
    "usb": {"mode": 0, "path": 48},
    "lsb": {"mode": 1, "path": 48},
    "usb_bass": {"mode": 0, "path": 48, "txfilter": 3, "txbass": -4, "txtreble": 2},
    "usb_tenor": {"mode": 0, "path": 48, "txfilter": 2, "comp": 5},
    "usb_comp_off": {"mode": 0, "path": 48, "comp": -1},
    "usb_comp_hi": {"mode": 0, "path": 48, "comp": 11, "micmult": 40, "boost": 1},
    "usb_iqadj": {"mode": 0, "path": 48, "txgi": 0.97, "txgq": 1.02, "txphase": -0.015, "txpwr": 0.8},
    "usb_m6k": {"mode": 0, "path": 48, "iqmode": 2},
    "usb_off": {"mode": 0, "path": 48, "iqmode": 0, "txphase": 0.01},
    # FM transmit (TxProcessor_FM, tx_processor.c:534-588): pre-emphasis + 16-bit softdds NCO
    "fm": {"mode": 5, "path": 1, "iqmode": 4},
    "fm_p12k_5k": {"mode": 5, "path": 1, "iqmode": 3, "fm5k": 1},
    "fm_subtone": {"mode": 5, "path": 1, "iqmode": 4, "subtone": 10},
    "fm_m6k_subtone": {"mode": 5, "path": 1, "iqmode": 2, "subtone": 33, "fm5k": 1, "comp": 3},
    "fm_p6k_iqadj": {"mode": 5, "path": 1, "iqmode": 1, "txgi": 0.97, "txgq": 1.02, "txphase": 0.02},
    # TUNE tones (softdds_runIQ into the voice chain) and the FM tone burst; events on call indices
    # that are multiples of 8 so 256-frame device calls can switch them between launches
    "usb_tune": {"mode": 0, "path": 48, "tune": "8:40:1"},
    "lsb_tune2": {"mode": 1, "path": 48, "comp": 5, "tune": "16:32:2"},
    "usb_tune_comp_off": {"mode": 0, "path": 48, "comp": -1, "tune": "0:64:1"},
    "fm_tune2": {"mode": 5, "path": 1, "iqmode": 4, "tune": "8:24:2"},
    "fm_burst": {"mode": 5, "path": 1, "iqmode": 4, "subtone": 10, "burstmode": 1, "burst": "16:24"},
    "fm_burst2_5k": {"mode": 5, "path": 1, "iqmode": 3, "fm5k": 1, "burstmode": 2, "burst": "8:16"},
    # AM transmit (TxProcessor_AM, tx_processor.c:715-800): the SSB voice chain with
    # AM_ALC_GAIN_CORRECTION, Hilbert pair, both sidebands + carrier, FreqShift
    "am": {"mode": 3, "path": 70},
    "am_p6k_comp": {"mode": 3, "path": 70, "iqmode": 1, "comp": 8, "txphase": 0.01},
    "am_filter_off": {"mode": 3, "path": 70, "flags1": 0x08, "txfilter": 2},
    "am_tune": {"mode": 3, "path": 70, "iqmode": 3, "tune": "8:24:1"},
    # FLAGS1_SSB_TX_FILTER_DISABLE (tx_processor.c:991): no TX band-pass lattice
    "usb_filter_off": {"mode": 0, "path": 48, "flags1": 0x40},
    # USB audio source (TX_AUDIO_DIG: gain 1, no bass / treble, tx_processor.c:374-377,445)
    "lsb_dig": {"mode": 1, "path": 48, "txsrc": 3},
    # USB I/Q source (TX_AUDIO_DIGIQ, :950-961): the frames are the I/Q; TUNE runs the voice path
    "usb_digiq": {"mode": 0, "path": 48, "txsrc": 4, "txgi": 0.98, "txphase": -0.01},
    "am_digiq_m6k": {"mode": 3, "path": 70, "txsrc": 4, "iqmode": 2, "txpwr": 0.9},
    # USB I/Q source in AM / FM with the frequency translation OFF: the passthrough branch comes
    # first (:950), so the I/Q is transmitted; under TUNE the AM / FM branch does nothing (:996-1016)
    "am_digiq_off_tune": {"mode": 3, "path": 70, "txsrc": 4, "iqmode": 0, "tune": "8:24:1"},
    "fm_digiq_off_tune": {"mode": 5, "path": 1, "txsrc": 4, "iqmode": 0, "tune": "16:32:2"},
}
# TX_AUDIO_DIGIQ fixtures take 16-bit I/Q (the USB audio class delivers int16 samples; the final
# stage scales by 2^16 with no headroom for the codec's left-aligned frames)
TX_DIGIQ_INPUT = ("usb_digiq", "am_digiq_m6k", "am_digiq_off_tune", "fm_digiq_off_tune")


def make_tx(name: str):
    args = dict(TX_CONFIGS[name], tx=1)
    audio = synth.tx_audio(np.arange(NCH), 0, NFRAMES)
    if name in TX_DIGIQ_INPUT:
        audio = synth.ssb_iq(np.arange(NCH), 0, NFRAMES) >> 16
    a0 = np.empty((NCH, NFRAMES), np.float32)
    iq = np.empty((NCH, NFRAMES, 2), np.int32)
    for c in range(NCH):
        a0[c], iq[c] = run_ref(args, audio[c])
    np.savez_compressed(os.path.join(HERE, f"tx_{name}.npz"), audio=audio, a0=a0, iq=iq,
                        setup=json.dumps(ref_json(args, "setup")), args=json.dumps(args))
    print(f"tx_{name:12s} peak|iq|={int(np.abs(iq).max()):11d}  peak|a0|={float(np.abs(a0).max()):9.1f}")


def tx_tables():
    """TX lattice band-pass per voice profile (TxProcessor_Set, tx_processor.c:88-107) and the
    201-tap TX Hilbert pair, as raw bits from the compiled reference."""
    out = {"lattice": {}}
    for f in (1, 2, 3):
        d = ref_json({"mode": 0, "path": 48, "tx": 1, "txfilter": f}, "setup")
        out["lattice"][str(f)] = {"k": d["tx_k"], "v": d["tx_v"]}
        out["hilbert_i"], out["hilbert_q"] = d["tx_hilbert_i"], d["tx_hilbert_q"]
    d = ref_json({"mode": 5, "path": 1, "tx": 1}, "setup")      # IIR_TX_2k7_FM (tx_processor.c:104-107)
    out["lattice"]["fm"] = {"k": d["tx_k"], "v": d["tx_v"]}
    x = ref_json({"mode": 0, "path": 48}, "txextra")              # softdds DDS_TABLE, sub-audible tones
    out["dds_table"], out["subaudible"] = x["dds_table"], x["subaudible"]
    with open(os.path.join(HERE, "tx_tables.json"), "w") as fo:
        json.dump(out, fo, separators=(",", ":"))


# spectrum display (a19): name -> (uhsdr_ref args incl. spec=L, signal kwargs).  The firmware's
# producer (audio_driver.c:1838-1851) fills the ring while the RX chain runs in `mode`/`path`.
SPEC_CONFIGS = {
    "p70_sam_1024": ({"mode": 4, "path": 70, "spec": 1024}, {"am": True}),          # C3
    "p48_usb_512": ({"mode": 0, "path": 48, "spec": 512}, {}),                      # 480x320 display
    "p48_usb_256": ({"mode": 0, "path": 48, "spec": 256, "specfilt": 1}, {}),       # 320x240 display
    "p48_iqauto_256": ({"mode": 0, "path": 48, "spec": 256, "iq_auto": 1}, {}),
    "p48_iqman_1024": ({"mode": 0, "path": 48, "spec": 1024, "gain_i": 1.03125, "gain_q": 0.96875,
                        "phase": -0.0125, "specfilt": 20}, {}),
    "p48_iqman2_512": ({"mode": 0, "path": 48, "spec": 512, "gain_i": 0.98, "gain_q": 1.01, "phase": 0.02,
                        "specfilt": 7}, {}),
    # zoom FFT producer (audio_driver.c:1860-1909): sd.magnify = mag, the ring gets the
    # translated I/Q low-passed (4-stage biquad) and decimated by 2^mag; signal center 0 Hz after
    # the translation (the default -12 kHz conversion puts the SSB tones at +12.7/13.9 kHz)
    "p48_zoom2_256": ({"mode": 0, "path": 48, "spec": 256, "mag": 1}, {}),
    "p48_zoom8_512_iqauto": ({"mode": 0, "path": 48, "spec": 512, "mag": 3, "iq_auto": 1}, {"frames": 16384}),
    "p48_zoom32_256_m6k": ({"mode": 0, "path": 48, "spec": 256, "mag": 5, "iqmode": 2, "specfilt": 2},
                           {"frames": 16384, "carrier": 6000.0}),
    "p48_zoom4_1024_off": ({"mode": 0, "path": 48, "spec": 1024, "mag": 2, "iqmode": 0,
                            "gain_i": 1.03125, "gain_q": 0.96875, "phase": -0.0125}, {"frames": 16384, "carrier": 0.0}),
    "p48_zoom16_256_p12k": ({"mode": 0, "path": 48, "spec": 256, "mag": 4, "iqmode": 3}, {"frames": 8192, "carrier": -12000.0}),
}
SPEC_FRAMES = 4096

# CW decoder front end (a20): name -> (uhsdr_ref args, signal kwargs).  Keyed CW at the sidetone
# pitch; thresholds low enough that the signal state toggles.
CW_CONFIGS = {
    "p4_cw": ({"mode": 2, "path": 4, "cwthresh": 1000}, {"cw": True}),
    "p4_cw_nonc": ({"mode": 2, "path": 4, "cwthresh": 1500, "cwnc": 0}, {"cw": True}),
    "p10_cw_b60": ({"mode": 2, "path": 10, "cwthresh": 1000, "cwblock": 60, "sidetone": 700}, {"cw": True, "tone": 700.0}),
    "p4_cw_b90": ({"mode": 2, "path": 4, "cwthresh": 800, "cwblock": 90}, {"cw": True}),
    "p70_sam_cw": ({"mode": 4, "path": 70, "cwthresh": 20000}, {"am": True}),
    "p4_cw_default": ({"mode": 2, "path": 4}, {"cw": True}),
}
CW_FRAMES = 8192


# Status side outputs (ADC clip flags, twin-peaks detector): name -> (uhsdr_ref args, frames).
# Input synth.status_iq (regenerated by the tests; its crc32 is stored), 5 channels with I/Q phase
# errors 0 / 12 / 30 / 60 / 89 degrees, auto I/Q on; the UI acknowledges codec restarts every
# `uiperiod` calls.  Long enough for four restart cycles (1001 + 50 calls each) -> UNCORRECTABLE.
STATUS_CONFIGS = {
    "p48_usb_tp": ({"mode": 0, "path": 48, "iq_auto": 1, "uiperiod": 8}, 4400 * 32),
    "p35_lsb_tp": ({"mode": 1, "path": 35, "iq_auto": 1, "uiperiod": 4}, 1152 * 32),
    "p70_am_tp": ({"mode": 3, "path": 70, "iq_auto": 1, "uiperiod": 16}, 2176 * 32),
}
STATUS_NCH = 5


def make_status(name: str):
    import zlib
    args, nfr = STATUS_CONFIGS[name]
    iq = synth.status_iq(np.arange(STATUS_NCH), 0, nfr)
    calls = nfr // 32
    tp = np.empty((STATUS_NCH, calls), np.uint8)
    clip = np.empty((STATUS_NCH, calls), np.uint8)
    a1 = np.empty((STATUS_NCH, nfr), np.float32)
    for c in range(STATUS_NCH):
        with tempfile.TemporaryDirectory() as td:
            fin, fa, ft, fc = (os.path.join(td, x) for x in ("in.bin", "a.bin", "t.bin", "c.bin"))
            iq[c].astype(np.int32).tofile(fin)
            cmd = [REF, f"in={fin}", f"n={nfr}", f"out_a={fa}", f"out_tp={ft}", f"out_clip={fc}"]
            subprocess.run(cmd + [f"{k}={v}" for k, v in args.items()], check=True)
            a1[c] = np.fromfile(fa, dtype=np.float32)
            tp[c] = np.fromfile(ft, dtype=np.uint8)
            clip[c] = np.fromfile(fc, dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, f"st_{name}.npz"), tp=tp, clip=clip, a1_head=a1[:, :2048],
                        a1_tail=a1[:, -2048:], frames=nfr, iq_crc32=zlib.crc32(np.ascontiguousarray(iq).tobytes()),
                        args=json.dumps(args))
    final = [int(x) for x in tp[:, -1]]
    print(f"st_{name:12s} calls={calls} final twinpeaks={final} clip calls={[(clip[c] != 0).sum() for c in range(STATUS_NCH)]}")


def make_cw(name: str):
    args, sig = CW_CONFIGS[name]
    sig = dict(sig)
    if sig.pop("am", False):
        iq = synth.am_iq(np.arange(NCH), 0, CW_FRAMES)
    else:
        sig.pop("cw")
        iq = synth.cw_iq(np.arange(NCH), 0, CW_FRAMES, **sig)
    calls = CW_FRAMES // 32
    a1 = np.empty((NCH, CW_FRAMES), np.float32)
    sg = np.empty((NCH, calls), np.uint8)
    en = []
    for c in range(NCH):
        with tempfile.TemporaryDirectory() as td:
            fin, fa, fcw, fs = (os.path.join(td, x) for x in ("in.bin", "a.bin", "cw.bin", "s.bin"))
            iq[c].astype(np.int32).tofile(fin)
            cmd = [REF, f"in={fin}", f"n={CW_FRAMES}", f"out_a={fa}", f"out_cw={fcw}", f"out_cws={fs}"]
            subprocess.run(cmd + [f"{k}={v}" for k, v in args.items()], check=True)
            a1[c] = np.fromfile(fa, dtype=np.float32)
            sg[c] = np.fromfile(fs, dtype=np.uint8)
            en.append(np.fromfile(fcw, dtype=np.float32))
    en = np.stack(en)
    np.savez_compressed(os.path.join(HERE, f"cw_{name}.npz"), iq=iq, signal=sg, energy=en,
                        setup=json.dumps(ref_json(args, "setup")), args=json.dumps(args))
    print(f"cw_{name:14s} blocks={en.shape[1]:4d} on-fraction={float(sg.mean()):.3f} peak energy={float(en.max()):.1f}")


def make_spec(name: str):
    args, sig = SPEC_CONFIGS[name]
    sig = dict(sig)
    nfr = sig.pop("frames", SPEC_FRAMES)
    if sig.pop("am", False):
        iq = synth.am_iq(np.arange(NCH), 0, nfr)
    else:
        iq = synth.ssb_iq(np.arange(NCH), 0, nfr, **sig)
    L = args["spec"]
    zd = 1 << args.get("mag", 0)
    mag = np.empty((NCH, nfr // zd // L, L), np.float32)
    avg = np.empty_like(mag)
    for c in range(NCH):
        with tempfile.TemporaryDirectory() as td:
            fin, fm, fa = (os.path.join(td, x) for x in ("in.bin", "m.bin", "a.bin"))
            iq[c].astype(np.int32).tofile(fin)
            cmd = [REF, f"in={fin}", f"n={nfr}", f"out_mag={fm}", f"out_avg={fa}"]
            subprocess.run(cmd + [f"{k}={v}" for k, v in args.items()], check=True)
            F = mag.shape[1]                        # the harness writes n floats: frames first
            mag[c] = np.fromfile(fm, dtype=np.float32)[:F * L].reshape(-1, L)
            avg[c] = np.fromfile(fa, dtype=np.float32)[:F * L].reshape(-1, L)
    np.savez_compressed(os.path.join(HERE, f"spec_{name}.npz"), iq=iq, mag=mag, avg=avg, args=json.dumps(args))
    print(f"spec_{name:14s} peak mag={float(mag.max()):10.2f}  min avg={float(avg.min()):6.2f}")


def spectrum_tables():
    """CMSIS twiddle / bit-reversal tables of arm_cfft_sR_f32_len256/512/1024
    (arm_const_structs.c:63-73, arm_common_tables.c) and the Hann windows of
    ui_spectrum.c:359-406, as raw bits from the compiled reference."""
    d = ref_json({"mode": 0, "path": 48}, "spectrum")
    with open(os.path.join(HERE, "spectrum_tables.json"), "w") as fo:
        json.dump(d, fo, separators=(",", ":"))


def run_ref(args: dict, iq: np.ndarray, want_a0: bool = False):
    n = iq.shape[0]
    with tempfile.TemporaryDirectory() as td:
        fin, fa, fd, fa0 = (os.path.join(td, x) for x in ("in.bin", "a.bin", "d.bin", "a0.bin"))
        iq.astype(np.int32).tofile(fin)
        cmd = [ref_bin(args), f"in={fin}", f"n={n}", f"out_a={fa}", f"out_dst={fd}"]
        if want_a0:
            cmd.append(f"out_a0={fa0}")
        cmd += [f"{k}={v}" for k, v in args.items()]
        subprocess.run(cmd, check=True)
        a1 = np.fromfile(fa, dtype=np.float32)
        dst = np.fromfile(fd, dtype=np.int32).reshape(n, 2)
        if want_a0:
            return a1, dst, np.fromfile(fa0, dtype=np.float32)
    return a1, dst


def ref_json(args: dict, what: str):
    cmd = [ref_bin(args), f"dump={what}"] + [f"{k}={v}" for k, v in args.items()]
    return json.loads(subprocess.run(cmd, check=True, capture_output=True, text=True).stdout)


def make(name: str):
    args, sig = CONFIGS[name]
    sig = dict(sig)
    center = sig.pop("center", None)
    nframes = sig.pop("frames", NFRAMES)
    nch = sig.pop("nch", NCH)
    if sig.pop("fm", False):
        iq = synth.fm_iq(np.arange(nch), 0, nframes, **sig)
    elif sig.pop("am", False):
        iq = synth.am_iq(np.arange(NCH), 0, NFRAMES)
    else:
        carrier = sig.pop("carrier", 12000.0)
        iq = synth.ssb_iq(np.arange(NCH), 0, NFRAMES, carrier=center if center is not None else carrier, **sig)
    C = iq.shape[0]
    a1 = np.empty((C, iq.shape[1]), np.float32)
    dst = np.empty((C, iq.shape[1], 2), np.int32)
    extra = {}
    stereo = True          # a_buffer[0] too: the second channel in stereo, a copy of [1] otherwise
    if stereo:
        extra["a0"] = np.empty((C, iq.shape[1]), np.float32)
    for c in range(C):
        if stereo:
            a1[c], dst[c], extra["a0"][c] = run_ref(args, iq[c], want_a0=True)
        else:
            a1[c], dst[c] = run_ref(args, iq[c])
    np.savez_compressed(os.path.join(HERE, f"rx_{name}.npz"), iq=iq, a1=a1, dst=dst, **extra,
                        setup=json.dumps(ref_json(args, "setup")), agc=json.dumps(ref_json(args, "agc")),
                        args=json.dumps(args))
    peak = float(np.abs(a1).max())
    print(f"{name:14s} peak|a1|={peak:9.1f}  rms={float(np.sqrt((a1.astype(np.float64)**2).mean())):9.1f}")


def make_cmsis():
    """CMSIS-DSP f32 golden vectors (uhsdr_ref dump=cmsis, oracle/ref/ref_cmsis.c): per case its
    parameters and every array, stored as tests/golden/cmsis_vectors.npz with keys
    '<case>.<field>' and a JSON manifest under 'manifest'."""
    with tempfile.TemporaryDirectory() as td:
        out = subprocess.run([REF, "dump=cmsis", f"out={td}"], check=True, capture_output=True, text=True).stdout
        man = json.loads(out)
        arrs = {}
        for case, d in man.items():
            for field, n in d["fields"].items():
                x = np.fromfile(os.path.join(td, f"{case}.{field}.f32"), dtype=np.float32)
                assert x.size == n, (case, field)
                arrs[f"{case}.{field}"] = x
    np.savez_compressed(os.path.join(HERE, "cmsis_vectors.npz"), manifest=json.dumps(man), **arrs)
    print(f"cmsis_vectors: {len(man)} cases")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    if not os.path.exists(REF):
        sys.exit(f"{REF} missing: run `make -C oracle/ref` (needs /root/reference)")
    if not os.path.exists(REF_MCHF):
        sys.exit(f"{REF_MCHF} missing: run `make -C oracle/ref mchf`")
    if a.only == "cmsis":
        make_cmsis()
        return
    if a.only in STATUS_CONFIGS:
        make_status(a.only)
        return
    make_cmsis()
    paths = subprocess.run([REF, "dump=paths"], check=True, capture_output=True, text=True).stdout
    with open(os.path.join(HERE, "filter_paths.json"), "w") as f:
        json.dump(json.loads(paths), f, separators=(",", ":"))
    tx_tables()
    spectrum_tables()
    for name in STATUS_CONFIGS:
        if a.only and name != a.only:
            continue
        make_status(name)
    for name in CW_CONFIGS:
        if a.only and name != a.only:
            continue
        make_cw(name)
    for name in SPEC_CONFIGS:
        if a.only and name != a.only:
            continue
        make_spec(name)
    for name in CONFIGS:
        if a.only and name != a.only:
            continue
        make(name)
    for name in TX_CONFIGS:
        if a.only and f"tx_{name}" != a.only:
            continue
        make_tx(name)


if __name__ == "__main__":
    main()
