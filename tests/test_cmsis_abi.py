"""CMSIS-signature shims (include/uhsdr_cmsis.h, libuhsdr_cmsis.so), checks that need no GPU:
the header, the ctypes binding and the library's exports agree; the instance structs have the
CMSIS layout (checked against gcc on the header); the init functions follow CMSIS's argument
rules (arm_fir_decimate_init_f32.c, arm_fir_interpolate_init_f32.c) and zero the state."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from uhsdr_amd import cmsis

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "uhsdr_cmsis.h")


def declared():
    src = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    return sorted(set(re.findall(r"\b((?:arm|uhsdr)_[a-z0-9_]+)\s*\(", src)))


def test_header_and_bindings_agree():
    assert set(declared()) == set(cmsis.SIGNATURES), set(declared()) ^ set(cmsis.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = cmsis.load()
    for name in declared():
        assert hasattr(lib, name), name


@pytest.mark.parametrize("name", ["arm_fir_instance_f32", "arm_fir_decimate_instance_f32",
                                  "arm_fir_interpolate_instance_f32", "arm_iir_lattice_instance_f32",
                                  "arm_biquad_casd_df1_inst_f32", "arm_cfft_instance_f32",
                                  "arm_lms_norm_instance_f32"])
def test_instance_layout_matches_header(name, tmp_path):
    st = getattr(cmsis, name)
    src = tmp_path / "sz.c"
    fields = [f for f, _ in st._fields_]
    body = " ".join(f'printf("%zu ", (size_t)offsetof({name}, {f}));' for f in fields)
    src.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "uhsdr_cmsis.h"\n'
                   f'int main(void) {{ printf("%zu ", sizeof({name})); {body} return 0; }}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got == [C.sizeof(st)] + [getattr(st, f).offset for f in fields]


def test_init_functions_follow_cmsis_rules():
    lib = cmsis.load()
    c = np.ones(8, np.float32)
    state = np.full(8 + 12 - 1, 7.0, np.float32)
    S = cmsis.arm_fir_decimate_instance_f32()
    assert lib.arm_fir_decimate_init_f32(C.byref(S), 8, 4, cmsis._fp(c), cmsis._fp(state), 10) == -2
    assert lib.arm_fir_decimate_init_f32(C.byref(S), 8, 4, cmsis._fp(c), cmsis._fp(state), 12) == 0
    assert (S.M, S.numTaps) == (4, 8) and not state.any()
    I = cmsis.arm_fir_interpolate_instance_f32()
    st2 = np.full(16, 3.0, np.float32)
    assert lib.arm_fir_interpolate_init_f32(C.byref(I), 3, 8, cmsis._fp(c), cmsis._fp(st2), 4) == -2
    assert lib.arm_fir_interpolate_init_f32(C.byref(I), 4, 8, cmsis._fp(c), cmsis._fp(st2), 4) == 0
    assert I.phaseLength == 2 and not st2[:5].any()


def test_cfft_vectors_cover_every_cmsis_length():
    """tests/golden/cmsis_vectors.npz holds arm_cfft_f32 sequences of the reference build for every
    length arm_cfft_f32.c:594-611 dispatches, with the instance tables; each output is the DFT
    of its input (float64 check of the fixture itself, tolerance of binary32 rounding)."""
    import json
    import os
    import numpy as np
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cmsis_vectors.npz"))
    man = json.loads(str(d["manifest"]))
    lens = set()
    for case, m in man.items():
        if not case.startswith(("cfft_", "icfft_")):
            continue
        p = m["params"]
        L = p["fftLen"]
        lens.add(L)
        assert d[f"{case}.twiddle"].size == 2 * L and d[f"{case}.bitrev"].size == p["bitRevLength"]
        if not p["bitReverseFlag"]:
            continue
        x = d[f"{case}.src"].astype(np.float64).view(np.complex128)
        y = d[f"{case}.dst"].astype(np.float64).view(np.complex128)
        ref = np.fft.ifft(x) if p["ifftFlag"] else np.fft.fft(x)
        assert np.abs(y - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max()), case
    assert lens == {16, 32, 64, 128, 256, 512, 1024, 2048, 4096}


def test_lms_vectors_follow_the_nlms_recursion():
    """The arm_lms_norm_f32 fixtures of the reference build (tests/golden/cmsis_vectors.npz,
    lms_*) against a binary32 restatement of arm_lms_norm_f32.c:205-300 (every operation
    rounded to float32, in the reference's order): bit-exact outputs, errors, coefficients,
    carried window, energy and x0."""
    import json
    f32 = np.float32
    d = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cmsis_vectors.npz"))
    man = json.loads(str(d["manifest"]))
    cases = [c for c in man if c.startswith("lms_")]
    assert len(cases) >= 4
    for case in cases:
        p = man[case]["params"]
        T, B, K, mu = p["numTaps"], p["blockSize"], p["calls"], f32(p["mu"])
        w = d[f"{case}.coeffs0"].copy()
        src, ref = d[f"{case}.src"], d[f"{case}.ref"]
        win = np.zeros(T - 1, np.float32)
        energy, x0 = f32(0), f32(0)
        out, err = [], []
        for k in range(K):
            x = np.concatenate([win, src[k * B:(k + 1) * B]])
            for n in range(B):
                xin = x[n + T - 1]
                energy = f32(energy - f32(x0 * x0))
                energy = f32(energy + f32(xin * xin))
                acc = f32(0)
                for t in range(T):
                    acc = f32(acc + f32(x[n + t] * w[t]))
                e = f32(ref[k * B + n] - acc)
                step = f32(f32(e * mu) / f32(energy + f32(0.000000119209289)))
                w = (w + (step * x[n:n + T]).astype(np.float32)).astype(np.float32)
                x0 = x[n]
                out.append(acc)
                err.append(e)
            win = x[B:]
        for name, got in (("out", np.array(out, np.float32)), ("err", np.array(err, np.float32)), ("coeffs", w),
                          ("state", win), ("energy_x0", np.array([energy, x0], np.float32))):
            want = d[f"{case}.{name}"]
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (case, name)
