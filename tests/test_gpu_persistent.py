"""Persistent back end (uhsdr_rx_set_pipelined 3): one rx_back launch runs call after call, taking
each call the host grants through host-mapped control words, and closes when no grant is there (or at
join / synchronize).  Results must be the same bits as the serial chain (the CPU oracle) whatever the
launch boundaries turn out to be: back-to-back runs, a join after every call, host pauses that let the
launch close by itself, fronts held back so the back end waits inside a launch, mode switches, and
a give-up that must fail loudly.
"""
import time

import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact
from test_gpu_pipelined import CALLS, run_pipelined
from uhsdr_amd import synth

pytestmark = pytest.mark.gpu

# N / 32 >= 8 runs on the persistent back end (SSB / CW / DIGI without the CW decoder); the others
# keep the device hand-off's one launch per call and must be unaffected by the mode
CASES = [
    ("p48_usb", dict(filter_path=48, dmod_mode=U.DEMOD_USB), synth.ssb_iq, 300, 256),
    ("p48_usb_n16", dict(filter_path=48, dmod_mode=U.DEMOD_USB), synth.ssb_iq, 130, 512),
    ("p48_mchf", dict(filter_path=48, board=U.BOARD_MCHF, spkr_gain=24), synth.ssb_iq, 97, 256),
    ("p48_agc_hang_eq", dict(agc_mode=1, agc_hang_enable=1, bass_gain=-8, treble_gain=6), synth.ssb_iq, 200, 256),
    ("p35_lsb_n4", dict(filter_path=35, dmod_mode=U.DEMOD_LSB), synth.ssb_iq, 130, 128),
    ("p4_cw", dict(filter_path=4, dmod_mode=U.DEMOD_CW), synth.cw_iq, 65, 256),
    ("p70_am_event", dict(filter_path=70, dmod_mode=U.DEMOD_AM), synth.am_iq, 129, 256),
]


@pytest.mark.parametrize("name,kw,gen,C,N", CASES, ids=[c[0] for c in CASES])
def test_persistent_matches_oracle(cuda, name, kw, gen, C, N):
    cfg = U.default_config(**kw)
    iq = gen(np.arange(C), 0, CALLS * N)
    tmo = []
    a1, dst = run_pipelined(cfg, iq, N, mode=3, timeouts=tmo)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"persistent {name}")
    np.testing.assert_array_equal(dst, ref_dst)
    assert tmo == [0]


def test_persistent_join_each(cuda):
    """join() after every call closes the launch at that call: one launch per call, still exact."""
    cfg = U.default_config()
    C, N = 200, 256
    iq = synth.ssb_iq(np.arange(C), 0, 10 * N)
    tmo = []
    a1, dst = run_pipelined(cfg, iq, N, mode=3, join_each=True, timeouts=tmo)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, "persistent, join each call")
    np.testing.assert_array_equal(dst, ref_dst)
    assert tmo == [0]


def test_persistent_mode_switches(cuda):
    """The persistent back end, the device and event hand-offs and the serial mode alternating
    between calls (each switch into or out of mode 3 synchronises)."""
    cfg = U.default_config()
    C, N = 96, 256
    iq = synth.ssb_iq(np.arange(C), 0, 17 * N)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    tmo = []
    a1, dst = run_pipelined(cfg, iq, N, mode=3, modes={3: 2, 5: 3, 9: 0, 10: 3, 13: 1, 14: 3}, timeouts=tmo)
    assert_bitexact(a1, ref_a1, "persistent, modes switched")
    np.testing.assert_array_equal(dst, ref_dst)
    assert tmo == [0]


def _c2_run(cuda, calls, pool, before=None, sync=None):
    """`calls` C2-shape calls in mode 3 over `pool` device-generated blocks; before(k) runs ahead of
    call k's process() (host pauses, front delays), sync(k) after it; sampled channels checked."""
    import torch
    cfg = U.default_config()
    C, N = 4096, 256
    chain = U.RxChain(cfg, channels=C, frames=N, stream=torch.cuda.current_stream().cuda_stream)
    chain.set_pipelined(3)
    xs = [synth.ssb_iq_torch(0, C, k * N, N, cuda) for k in range(pool)]
    pick = np.arange(5, C, 97)
    full = torch.empty((calls, C, N), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for k in range(calls):
        if before is not None:
            before(k)
        chain.process(xs[k % pool], full[k], None)
        if sync is not None:
            sync(k)
    chain.synchronize()
    assert chain.handoff_timeouts() == 0
    chain.close()
    audio = full[:, torch.from_numpy(pick).cuda(), :]
    iq = np.concatenate([xs[k % pool].cpu().numpy()[pick] for k in range(calls)], axis=1)
    ref, _ = oracle.OracleRx(U.build_plan(cfg), len(pick)).process(np.ascontiguousarray(iq), threads=8)
    return audio.permute(1, 0, 2).reshape(len(pick), calls * N).cpu().numpy(), ref


def test_persistent_long_run(cuda):
    """120 calls back to back at the C2 shape: one launch takes them all (every hand-off buffer and
    descriptor slot reused many times, the host waiting on PC_CONSUMED)."""
    got, ref = _c2_run(cuda, 120, 6)
    assert_bitexact(got, ref, "persistent, 120 calls")


def test_persistent_host_pauses(cuda):
    """The host pauses (~3 ms) before some calls: the launch finds no grant, closes itself, and the
    next call starts a new one; and a torch.cuda.synchronize() without join mid-stream (the launch
    must end on its own, not wait for a call that never comes)."""
    import torch

    def before(k):
        if k % 4 == 3 or k in (9, 10):
            time.sleep(0.003)

    def sync(k):
        if k == 13:
            torch.cuda.synchronize()

    got, ref = _c2_run(cuda, 22, 5, before=before, sync=sync)
    assert_bitexact(got, ref, "persistent, host pauses")


def test_persistent_fronts_delayed(cuda):
    """Fronts held back on the handle's stream (~75-100 us spin kernels) on every third call and on
    two in a row: the running launch waits for an arrival inside itself, bit-exact."""
    import torch

    def before(k):
        if k % 3 == 2 or k in (10, 11):
            torch.cuda._sleep(150_000)

    got, ref = _c2_run(cuda, 19, 7, before=before)
    assert_bitexact(got, ref, "persistent, fronts delayed")


def test_persistent_give_up_fails_loudly(cuda):
    """The failure contract in mode 3: a 64-poll bound and call 3's front held back ~25 ms while the
    launch that ran calls 0-2 is still taking grants, so it gives up inside the launch.  Call 3's
    audio is NaN, calls 0-1 exact, synchronize / process / join raise UHSDR_TIMEOUT,
    handoff_timeouts() == 1; after reset() the handle runs bit-exact again."""
    import torch
    cfg = U.default_config()
    C, N = 256, 256
    iq = synth.ssb_iq(np.arange(C), 0, 6 * N)
    xs = [torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda() for k in range(6)]
    chain = U.RxChain(cfg, channels=C, frames=N, stream=torch.cuda.current_stream().cuda_stream)
    chain.set_pipelined(3)
    chain.set_handoff_bound(64)
    audio = torch.zeros((6, C, N), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for k in range(3):
        chain.process(xs[k], audio[k], None)
    torch.cuda._sleep(50_000_000)                    # ~25 ms ahead of call 3's rx_front
    chain.process(xs[3], audio[3], None)
    with pytest.raises(U.UhsdrError) as e:
        chain.synchronize()
    assert e.value.status == U.UHSDR_TIMEOUT
    assert chain.handoff_timeouts() == 1
    with pytest.raises(U.UhsdrError) as e:
        chain.process(xs[4], audio[4], None)
    assert e.value.status == U.UHSDR_TIMEOUT
    with pytest.raises(U.UhsdrError) as e:
        chain.join()
    assert e.value.status == U.UHSDR_TIMEOUT
    got = audio.cpu().numpy()
    assert np.isnan(got[3]).all(), "the give-up's output must be poisoned"
    ref, _ = oracle.OracleRx(U.build_plan(cfg), C).process(np.ascontiguousarray(iq[:, :3 * N]), threads=8)
    assert_bitexact(got[:2].transpose(1, 0, 2).reshape(C, 2 * N), ref[:, :2 * N], "calls before the give-up")
    chain.reset()
    chain.set_handoff_bound(1 << 24)
    assert chain.handoff_timeouts() == 0
    for k in range(3):
        chain.process(xs[k], audio[k], None)
    chain.synchronize()
    assert chain.handoff_timeouts() == 0
    assert_bitexact(audio[:3].cpu().numpy().transpose(1, 0, 2).reshape(C, 3 * N), ref, "after reset")
    with pytest.raises(U.UhsdrError):
        chain.set_pipelined(4)                       # modes are 0 .. 3
    chain.close()

