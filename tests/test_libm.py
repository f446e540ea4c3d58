"""uhsdr_amd/csrc/uhsdr_libm.h (the device's sincosf / atan2f) reproduces the host glibc bit for
bit -- the SAM PLL and FM discriminator of the reference call glibc (audio_driver.c:2039,
2128, 1581).  tools/libm_check.c is compiled here and run on a strided subset (every 251st
float of [-2pi, 2pi]) and on 2e6 atan2f operand pairs; the exhaustive run (every float of
[-2pi, 2pi], 2e8 atan2f pairs) is recorded in tests/golden/libm_pin.txt."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path):
    exe = str(tmp_path / "libm_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, os.path.join(ROOT, "tools", "libm_check.c"), "-lm"],
                   check=True)
    return exe


def test_sincosf_matches_glibc(tmp_path):
    r = subprocess.run([_build(tmp_path), "sincos", "251"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert " 0 of " in r.stdout


def test_atan2f_matches_glibc(tmp_path):
    r = subprocess.run([_build(tmp_path), "atan2", "2000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert " 0 of " in r.stdout


def test_atan2f_x_one_matches_glibc(tmp_path):
    """atan2f(y, 1) -- fdlibm's atanf(y) case, which the branch-free ul_atan2f folds into its main
    path: every 4099th binary32 y here, every y in the exhaustive run (libm_pin.txt)."""
    r = subprocess.run([_build(tmp_path), "atan2x1", "4099"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert " 0 of " in r.stdout


def test_atanf_nonnegative_matches_glibc(tmp_path):
    """ul_atanf_pos, atan2f's reduction of |y / x|: every 1021st float of [0, inf] here, every one in
    the exhaustive run (libm_pin.txt)."""
    r = subprocess.run([_build(tmp_path), "atanpos", "1021"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert " 0 of " in r.stdout


def test_asinf_matches_glibc(tmp_path):
    """The twin-peaks detector's asinf (audio_driver.c:2211); exhaustive run in libm_pin.txt."""
    r = subprocess.run([_build(tmp_path), "asin", "127"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout
    assert " 0 of " in r.stdout
