"""Batched arm_fir_f32 on the device (uhsdr_fir_*, C5's long filter and the FIR-as-GEMM):

  * EXACT: bit-identical to the reference's own CMSIS arm_fir_f32 (tests/golden/cmsis_vectors.npz
    fir_513x256, the same sequence fed to every channel of ragged batches) and to the CPU
    oracle (pinned to those vectors, tests/test_fir_oracle.py) on distinct channels;
  * MFMA: within north_star's 1e-5 relative of the same references, normwise per channel
    (measured ~1e-7: every multiply-add fused, tap order kept)."""
import json
import os

import numpy as np
import pytest

import oracle
import uhsdr_amd as U

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_Z = np.load(os.path.join(GOLD, "cmsis_vectors.npz"))
MAN = json.loads(str(_Z["manifest"]))
TOL = 1e-5


def run(fir, x, B):
    import torch
    C, n = x.shape
    out = np.empty_like(x)
    d_y = torch.empty((C, B), dtype=torch.float32, device="cuda")
    for k in range(n // B):
        fir.process(torch.from_numpy(np.ascontiguousarray(x[:, k * B:(k + 1) * B])).cuda(), d_y)
        torch.cuda.synchronize()
        out[:, k * B:(k + 1) * B] = d_y.cpu().numpy()
    return out


def normwise(got, ref):
    return float(np.max(np.abs(got.astype(np.float64) - ref), axis=-1).max() /
                 max(float(np.abs(ref).max()), 1e-30))


@pytest.mark.parametrize("mode", [U.fir.EXACT, U.fir.MFMA], ids=["exact", "mfma"])
@pytest.mark.parametrize("channels", [1, 37, 130])
def test_fir_matches_reference_cmsis(cuda, mode, channels):
    case = "fir_513x256"
    p = MAN[case]["params"]
    B = p["blockSize"]
    src = _Z[f"{case}.src"]
    ref = _Z[f"{case}.dst"]
    fir = U.FirBatch(_Z[f"{case}.coeffs"], channels, B, mode)
    got = run(fir, np.tile(src, (channels, 1)), B)
    fir.close()
    if mode == U.fir.EXACT:
        for c in range(channels):
            np.testing.assert_array_equal(got[c].view(np.uint32), ref.view(np.uint32))
    else:
        assert normwise(got, np.tile(ref, (channels, 1))) < TOL


@pytest.mark.parametrize("mode", [U.fir.EXACT, U.fir.MFMA], ids=["exact", "mfma"])
@pytest.mark.parametrize("T,B", [(513, 256), (513, 512), (89, 256), (7, 768)])
def test_fir_matches_oracle_distinct_channels(cuda, mode, T, B):
    rng = np.random.default_rng(T * 1000 + B)
    C = 70
    taps = np.load(os.path.join(GOLD, "fir513_kaiser.npy")) if T == 513 else rng.uniform(-0.3, 0.3, T).astype(np.float32)
    x = rng.normal(0, 1000, (C, 3 * B)).astype(np.float32)
    fir = U.FirBatch(taps, C, B, mode)
    got = run(fir, x, B)
    fir.close()
    o = oracle.OracleFir(taps, C)
    ref = np.concatenate([o.process(x[:, k * B:(k + 1) * B]) for k in range(3)], axis=1)
    if mode == U.fir.EXACT:
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    else:
        assert normwise(got, ref) < TOL


WAVE_CASES = [(m, w) for m in (U.fir.EXACT, U.fir.MFMA) for w in (1, 2, 4)] + [(U.fir.MFMA, w) for w in (7, 8, 16)]


def mfma_default_waves(T):
    """513 taps (K = 528 = 16 x 33): fir_mfma_rb, the taps' B fragments in registers, 8 waves per
    workgroup at most; every other tap count: fir_mfma, 16 windows"""
    return 8 if (T + 15 + 15) // 16 == 33 else 16


@pytest.mark.parametrize("mode,waves", WAVE_CASES, ids=[f"{'mfma' if m else 'exact'}-{w}" for m, w in WAVE_CASES])
@pytest.mark.parametrize("T,B", [(513, 256), (89, 512)])
def test_fir_waves_per_workgroup(cuda, mode, waves, T, B):
    """uhsdr_fir_set_waves changes the launch shape only: every count gives the oracle's output
    (EXACT bit-exact), across a call boundary and over 300 channels (several groups per
    workgroup at 4 waves, ragged last group)."""
    rng = np.random.default_rng(7 * T + waves)
    C = 300
    taps = np.load(os.path.join(GOLD, "fir513_kaiser.npy")) if T == 513 else rng.uniform(-0.3, 0.3, T).astype(np.float32)
    x = rng.normal(0, 1000, (C, 2 * B)).astype(np.float32)
    fir = U.FirBatch(taps, C, B, mode)
    assert fir.waves == (mfma_default_waves(T) if mode == U.fir.MFMA else 2)
    if mode == U.fir.MFMA and waves > mfma_default_waves(T):
        with pytest.raises(RuntimeError):
            fir.set_waves(waves)
        fir.close()
        return
    fir.set_waves(waves)
    assert fir.waves == waves
    got = run(fir, x, B)
    fir.close()
    o = oracle.OracleFir(taps, C)
    ref = np.concatenate([o.process(x[:, k * B:(k + 1) * B]) for k in range(2)], axis=1)
    if mode == U.fir.EXACT:
        np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    else:
        assert normwise(got, ref) < TOL


def test_fir_set_waves_rejects(cuda):
    fir = U.FirBatch(np.ones(9, np.float32), 4, 256)
    for bad in (0, 3, 8, -1):
        with pytest.raises(RuntimeError):
            fir.set_waves(bad)
        assert fir.waves == 2
    fir.close()
    fir = U.FirBatch(np.ones(9, np.float32), 4, 256, U.fir.MFMA)
    for bad in (0, 17, -1):
        with pytest.raises(RuntimeError):
            fir.set_waves(bad)
        assert fir.waves == 16
    fir.close()
    fir = U.FirBatch(np.ones(513, np.float32), 4, 256, U.fir.MFMA)
    for bad in (0, 9, 16, -1):
        with pytest.raises(RuntimeError):
            fir.set_waves(bad)
        assert fir.waves == 8
    fir.close()


def test_fir_rejects_bad_block(cuda):
    with pytest.raises(RuntimeError):
        U.FirBatch(np.ones(9, np.float32), 4, 100)
