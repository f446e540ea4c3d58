"""C-ABI boundary checks that need no GPU: the library loads, exports every entry point that
include/uhsdr.h declares, its struct layouts match, and argument errors follow arm_status."""
import ctypes as C
import os
import re

import uhsdr_amd as U
from uhsdr_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "uhsdr.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(uhsdr_[a-z0-9_]+)\s*\(", src)))


def test_header_and_bindings_agree():
    decl = declared_functions()
    assert decl, "no functions parsed from include/uhsdr.h"
    assert set(decl) == set(_abi.SIGNATURES), set(decl) ^ set(_abi.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = U.load()
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_struct_sizes():
    lib = U.load()
    assert lib.uhsdr_sizeof_config() == C.sizeof(U.RxConfig)
    assert lib.uhsdr_sizeof_plan() == C.sizeof(U.RxPlan)


def test_create_rejects_bad_lengths_without_touching_the_device():
    lib = U.load()
    cfg = U.default_config()
    h = C.c_void_p()
    assert lib.uhsdr_rx_create(C.byref(cfg), 16, 100, None, C.byref(h)) == -2   # N % 32 != 0
    assert lib.uhsdr_rx_create(C.byref(cfg), 0, 64, None, C.byref(h)) == -1
    assert lib.uhsdr_rx_create(None, 16, 64, None, C.byref(h)) == -1
    bad = U.default_config(filter_path=200)
    assert lib.uhsdr_rx_create(C.byref(bad), 16, 64, None, C.byref(h)) == -1
    assert b"filter_path" in lib.uhsdr_last_error()
    assert lib.uhsdr_rx_process(None, None, None, None) == -1


def test_unsupported_modes_are_reported():
    lib = U.load()
    # FM without the I/Q translation: the reference demodulator bails out (audio_driver.c:1548)
    plan = U.build_plan(U.default_config(dmod_mode=U.DEMOD_FM, filter_path=1, iq_freq_mode=0))
    assert lib.uhsdr_rx_plan_supported(C.byref(plan)) == 0
    plan = U.build_plan(U.default_config(dmod_mode=U.DEMOD_FM, filter_path=1))
    assert lib.uhsdr_rx_plan_supported(C.byref(plan)) == 1
    plan = U.build_plan(U.default_config())
    assert lib.uhsdr_rx_plan_supported(C.byref(plan)) == 1


def test_plain_c_host_links_against_the_abi():
    """examples/rx_batch.c (gcc, no HIP headers) links against libuhsdr_amd.so; run without
    arguments it only prints usage (no device call)."""
    import subprocess
    exe = os.path.join(ROOT, "examples", "build", "rx_batch")
    assert os.path.exists(exe), "run `make` first"
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 2 and "uhsdr_amd" in r.stderr
