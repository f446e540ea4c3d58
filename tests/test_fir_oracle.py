"""The CPU checker of the batched FIR (oracle/uhsdr_oracle.c uo_fir_batch) pinned bit-for-bit
against the reference's own CMSIS arm_fir_f32 call sequences (tests/golden/cmsis_vectors.npz,
oracle/ref/ref_cmsis.c), including the 513-tap C5 case, outputs and carried state."""
import json
import os

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cmsis_vectors.npz")
_Z = np.load(GOLD)
MAN = json.loads(str(_Z["manifest"]))


@pytest.mark.parametrize("case", [c for c in MAN if c.startswith("fir_")])
def test_oracle_fir_matches_reference_cmsis(case):
    p = MAN[case]["params"]
    B, K = p["blockSize"], p["calls"]
    f = oracle.OracleFir(_Z[f"{case}.coeffs"], 1)
    src = _Z[f"{case}.src"]
    got = np.concatenate([f.process(src[None, k * B:(k + 1) * B])[0] for k in range(K)])
    np.testing.assert_array_equal(got.view(np.uint32), _Z[f"{case}.dst"].view(np.uint32))
    np.testing.assert_array_equal(f.hist[0].view(np.uint32), _Z[f"{case}.state"].view(np.uint32))
