"""The CPU oracle (oracle/uhsdr_oracle.c) is pinned bit-for-bit to the reference firmware.

Fixtures: tests/golden/rx_*.npz, produced by the reference's own audio_driver.c + CMSIS-DSP
compiled for x86 (oracle/ref/, tests/golden/make_golden.py).
"""
import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact, drive, golden_file, golden_files, load


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: p.split("rx_")[-1][:-4])
def test_oracle_matches_reference(path):
    g = load(path)
    plan = U.build_plan(U.config_from_ref_args(g["args"]))
    o = oracle.OracleRx(plan, g["iq"].shape[0])
    a1, a0, dst = drive(g, 256, o.process2, o.key_beep)
    assert_bitexact(a1, g["a1"], g["name"])
    if "a0" in g:
        assert_bitexact(a0, g["a0"], g["name"] + " a_buffer[0]")
    np.testing.assert_array_equal(dst, g["dst"])


@pytest.mark.parametrize("chunk", [32, 64, 416, 2048])
def test_oracle_call_granularity(chunk):
    """Splitting the stream into calls of any multiple of 32 frames gives the same samples
    (state is carried exactly as across ISR invocations)."""
    g = load(golden_file("p48_usb"))
    plan = U.build_plan(U.config_from_ref_args(g["args"]))
    o = oracle.OracleRx(plan, g["iq"].shape[0])
    outs = []
    n = g["iq"].shape[1]
    for off in range(0, n, chunk):
        outs.append(o.process(g["iq"][:, off:off + chunk])[0])
    assert_bitexact(np.concatenate(outs, axis=1), g["a1"], f"chunk={chunk}")


def test_oracle_threads_equal_single():
    g = load(golden_file("p48_usb"))
    plan = U.build_plan(U.config_from_ref_args(g["args"]))
    a = oracle.OracleRx(plan, 4).process(g["iq"], threads=1)[0]
    b = oracle.OracleRx(plan, 4).process(g["iq"], threads=4)[0]
    assert_bitexact(a, b, "threads")
