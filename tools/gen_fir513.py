#!/usr/bin/env python3
"""C5's synthetic 513-tap narrow filter (the reference's FIRs stop at 201
taps, so the long CW/RTTY filter is designed once here and committed): a Kaiser-window low-pass
at the decimated 12 ksps rate, 600 Hz cutoff, beta 8, float32, CMSIS tap order (symmetric, so
time reversal is the identity).  Writes tests/golden/fir513_kaiser.npy."""
import os

import numpy as np
from scipy.signal import firwin

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
taps = firwin(513, 600.0, window=("kaiser", 8.0), fs=12000.0).astype(np.float32)
np.save(os.path.join(ROOT, "tests", "golden", "fir513_kaiser.npy"), taps)
print(f"513 taps, sum {float(taps.sum()):.6f}, peak {float(taps.max()):.6f}")
