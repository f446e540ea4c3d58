"""Pipelined mode (uhsdr_rx_set_pipelined): call k+1's rx_front overlaps call k's rx_back on a
side stream, with the decimated hand-off double-buffered.  The results must be the same bits as
the serial chain: back-to-back calls with no synchronisation between them, checked against the
CPU oracle (SSB, AM / SAM with their second hand-off buffer, FM, CW with the decoder outputs),
plus join() ordering on the handle's stream, toggling the mode mid-stream, and the host entry.
"""
import numpy as np
import pytest

import oracle
import uhsdr_amd as U
from golden_util import assert_bitexact
from uhsdr_amd import synth

pytestmark = pytest.mark.gpu


def run_pipelined(cfg, iq, N, toggle_at=None, join_each=False, switch=None, mode=1, modes=None, timeouts=None):
    import torch
    C, n, _ = iq.shape
    calls = n // N
    chain = U.RxChain(cfg, channels=C, frames=N)
    chain.set_pipelined(mode)
    xs = [torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda() for k in range(calls)]
    audio = torch.empty((calls, C, N), dtype=torch.float32, device="cuda")
    dst = torch.empty((calls, C, N, 2), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for k in range(calls):
        if toggle_at is not None and k == toggle_at:
            chain.set_pipelined(False)
        if toggle_at is not None and k == toggle_at + 1:
            chain.set_pipelined(True)
        if switch is not None and k in switch:
            chain.set_schedule(switch[k])     # change kernel schedule between calls, still pipelined
        if modes is not None and k in modes:
            chain.set_pipelined(modes[k])     # hand-off kind (0 serial, 1 event, 2 device) between calls
        chain.process(xs[k], audio[k], dst[k])
        if join_each:
            chain.join()
    chain.synchronize()
    if timeouts is not None:
        timeouts.append(chain.handoff_timeouts())
    a = audio.permute(1, 0, 2).reshape(C, n).cpu().numpy()
    d = dst.permute(1, 0, 2, 3).reshape(C, n, 2).cpu().numpy()
    chain.close()
    return a, d


CASES = [
    ("p48_usb", dict(filter_path=48, dmod_mode=U.DEMOD_USB), synth.ssb_iq, 300, 256),
    ("p35_lsb", dict(filter_path=35, dmod_mode=U.DEMOD_LSB), synth.ssb_iq, 130, 128),
    ("p70_am", dict(filter_path=70, dmod_mode=U.DEMOD_AM), synth.am_iq, 200, 256),
    ("p70_sam", dict(filter_path=70, dmod_mode=U.DEMOD_SAM), synth.am_iq, 129, 256),
    ("p1_fm_event", dict(filter_path=1, dmod_mode=U.DEMOD_FM, fm_sql_threshold=12), synth.fm_iq, 100, 256),
    ("p4_cw", dict(filter_path=4, dmod_mode=U.DEMOD_CW), synth.cw_iq, 65, 64),
]


# The hand-off buffers are reused per group of PIPE_GROUP = 4 calls (PIPE_BUFS = 8): group g waits
# for the last rx_back of group g-2.  15 calls = groups 0..3, the last one partial, so every buffer
# is reused and the cross-group wait runs.
CALLS = 15


@pytest.mark.parametrize("name,kw,gen,C,N", CASES, ids=[c[0] for c in CASES])
def test_pipelined_matches_oracle(cuda, back, name, kw, gen, C, N):
    cfg = U.default_config(**kw)
    iq = gen(np.arange(C), 0, CALLS * N)
    a1, dst = run_pipelined(cfg, iq, N)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"pipelined {name}")
    np.testing.assert_array_equal(dst, ref_dst)


def test_pipelined_toggle_and_join(cuda):
    cfg = U.default_config()
    C, N = 96, 128
    iq = synth.ssb_iq(np.arange(C), 0, 17 * N)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    a1, dst = run_pipelined(cfg, iq, N, toggle_at=3)
    assert_bitexact(a1, ref_a1, "pipelined, off for call 3")
    a1, dst = run_pipelined(cfg, iq, N, toggle_at=10)
    assert_bitexact(a1, ref_a1, "pipelined, off for call 10 (inside group 2)")
    a1, dst = run_pipelined(cfg, iq, N, join_each=True)
    assert_bitexact(a1, ref_a1, "pipelined, join after every call")
    np.testing.assert_array_equal(dst, ref_dst)


@pytest.mark.parametrize("mode", [1, 2], ids=["event", "device"])
@pytest.mark.parametrize("first,second", [(1, 2), (2, 1)], ids=["pipe_then_fused", "fused_then_pipe"])
def test_pipelined_schedule_switch_mid_group(cuda, first, second, mode):
    """Pipelined across 17 calls while the schedule switches to CHAIN inside group 1 and back
    inside group 2: the hand-off buffers and their events must stay ordered; with the
    device hand-off too (CHAIN again for two calls inside group 2)."""
    cfg = U.default_config()
    C, N = 96, 128
    iq = synth.ssb_iq(np.arange(C), 0, 17 * N)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    sw = {0: first, 5: 3, 9: second, 14: first}
    if mode == 2:
        sw.update({11: 3, 13: second})
    a1, dst = run_pipelined(cfg, iq, N, switch=sw, mode=mode)
    assert_bitexact(a1, ref_a1, f"pipelined, schedule {first} -> chain -> {second} -> {first}")
    np.testing.assert_array_equal(dst, ref_dst)


def test_pipelined_join_orders_handle_stream(cuda):
    """After join(), work the caller enqueues on the handle's stream sees the outputs."""
    import torch
    cfg = U.default_config()
    C, N = 4096, 256
    iq = synth.ssb_iq(np.arange(C), 0, N)
    s = torch.cuda.Stream()
    chain = U.RxChain(cfg, channels=C, frames=N, stream=s.cuda_stream)
    chain.set_pipelined(True)
    x = torch.from_numpy(iq).cuda()
    audio = torch.zeros((C, N), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        chain.process(x, audio, None)
        chain.join()
        copy = audio.clone()                 # enqueued on s after the join
    torch.cuda.synchronize()
    ref, _ = oracle.OracleRx(U.build_plan(cfg), 64).process(iq[:64], threads=8)
    assert_bitexact(copy[:64].cpu().numpy(), ref, "copy after join")
    chain.close()


def test_pipelined_host_entry(cuda):
    cfg = U.default_config(filter_path=70, dmod_mode=U.DEMOD_AM)
    C, N = 33, 256
    iq = synth.am_iq(np.arange(C), 0, 2 * N)
    chain = U.RxChain(cfg, channels=C, frames=N)
    chain.set_pipelined(True)
    outs = [chain.process_host(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])) for k in range(2)]
    chain.close()
    ref_a1, _ = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(np.concatenate([o[0] for o in outs], axis=1), ref_a1, "pipelined host entry")


# mcHF in the pipelined mode: the board's
# output stage runs inline in every back end -- in the wave pipeline on its tail waves, one step
# behind the output role -- with no finishing pass or scratch row since round 6.  No
# synchronisation between calls; a key beep starts in the last call of group 0 and runs into group 1.
MCHF_PIPE_CASES = [
    ("p48_usb", dict(filter_path=48, spkr_gain=24), synth.ssb_iq, 130, 256, 15),
    ("p70_sam", dict(filter_path=70, dmod_mode=U.DEMOD_SAM, spkr_gain=30), synth.am_iq, 97, 256, 17),
    # 16 x 32-frame calls per launch: the squelch's first decision (every 200 calls) falls in call 12
    ("p1_fm_sql0", dict(filter_path=1, dmod_mode=U.DEMOD_FM, fm_sql_threshold=0, spkr_gain=20), synth.fm_iq, 65, 512, 16),
]


@pytest.mark.parametrize("name,kw,gen,C,N,calls", MCHF_PIPE_CASES, ids=[c[0] for c in MCHF_PIPE_CASES])
def test_pipelined_mchf_matches_oracle(cuda, name, kw, gen, C, N, calls):
    import torch
    cfg = U.default_config(board=U.BOARD_MCHF, **kw)
    iq = gen(np.arange(C), 0, calls * N)
    o = oracle.OracleRx(U.build_plan(cfg), C)
    chain = U.RxChain(cfg, channels=C, frames=N)
    chain.set_pipelined(True)
    xs = [torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda() for k in range(calls)]
    a1 = torch.empty((calls, C, N), dtype=torch.float32, device="cuda")
    a0 = torch.empty((calls, C, N), dtype=torch.float32, device="cuda")
    dst = torch.empty((calls, C, N, 2), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    beep_at, beep_calls = 3, N // 32 + 5
    ref = [[], [], []]
    for k in range(calls):
        if k == beep_at:
            chain.key_beep(beep_calls)
            o.key_beep(beep_calls)
        chain.process_stereo(xs[k], a1[k], a0[k], dst[k])
        for lst, r in zip(ref, o.process2(np.ascontiguousarray(iq[:, k * N:(k + 1) * N]))):
            lst.append(r)
    chain.synchronize()
    got = [t.permute(1, 0, *range(2, t.dim())).reshape((C, calls * N) + tuple(t.shape[3:])).cpu().numpy()
           for t in (a1, a0, dst)]
    chain.close()
    ref = [np.concatenate(x, axis=1) for x in ref]
    assert_bitexact(got[0], ref[0], f"pipelined mcHF {name} a_buffer[1]")
    assert_bitexact(got[1], ref[1], f"pipelined mcHF {name} a_buffer[0]")
    np.testing.assert_array_equal(got[2], ref[2])
    assert np.abs(ref[0]).max() > 0


# The device hand-off (uhsdr_rx_set_pipelined 2): rx_front's waves store adec write-through and bump
# their 64-channel group's arrival counter, and rx_back polls it on the device and then reads adec
# with sc1 loads, instead of waiting on a cross-stream event per call (and runs ahead into the next
# call when it has arrived: BackSched).  Used for the
# wave-pipeline back end without a demodulator or notch (SSB / CW / DIGI) up to half the CUs' worth
# of back-end workgroups; every other case keeps the event, so the AM, FM and large-batch cases check
# that fallback.  No poll may give up (uhsdr_rx_handoff_timeouts).
HANDOFF_CASES = [
    ("p48_usb", dict(filter_path=48, dmod_mode=U.DEMOD_USB), synth.ssb_iq, 300, 256),
    ("p48_usb_n16", dict(filter_path=48, dmod_mode=U.DEMOD_USB), synth.ssb_iq, 130, 512),
    ("p35_lsb", dict(filter_path=35, dmod_mode=U.DEMOD_LSB), synth.ssb_iq, 130, 128),
    ("p4_cw", dict(filter_path=4, dmod_mode=U.DEMOD_CW), synth.cw_iq, 65, 64),
    ("p48_mchf", dict(filter_path=48, board=U.BOARD_MCHF, spkr_gain=24), synth.ssb_iq, 97, 256),
    ("p48_agc_hang_eq", dict(agc_mode=1, agc_hang_enable=1, bass_gain=-8, treble_gain=6), synth.ssb_iq, 200, 128),
    ("p70_am_event", dict(filter_path=70, dmod_mode=U.DEMOD_AM), synth.am_iq, 129, 256),
    ("p1_fm_event", dict(filter_path=1, dmod_mode=U.DEMOD_FM, fm_sql_threshold=12), synth.fm_iq, 100, 256),
    ("p2_fm_tone_event", dict(filter_path=2, dmod_mode=U.DEMOD_FM, fm_sql_threshold=0, fm_tone_det=10),
     synth.fm_iq, 70, 512),
]


@pytest.mark.parametrize("name,kw,gen,C,N", HANDOFF_CASES, ids=[c[0] for c in HANDOFF_CASES])
def test_device_handoff_matches_oracle(cuda, name, kw, gen, C, N):
    cfg = U.default_config(**kw)
    iq = gen(np.arange(C), 0, CALLS * N)
    tmo = []
    a1, dst = run_pipelined(cfg, iq, N, mode=2, timeouts=tmo)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    assert_bitexact(a1, ref_a1, f"device hand-off {name}")
    np.testing.assert_array_equal(dst, ref_dst)
    assert tmo == [0]


def test_device_handoff_mode_switches(cuda):
    """Event and device hand-offs and the serial mode alternating between calls, inside groups."""
    cfg = U.default_config()
    C, N = 96, 128
    iq = synth.ssb_iq(np.arange(C), 0, 17 * N)
    ref_a1, ref_dst = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    tmo = []
    a1, dst = run_pipelined(cfg, iq, N, mode=2, modes={3: 1, 5: 2, 9: 0, 10: 2, 14: 1, 15: 2}, timeouts=tmo)
    assert_bitexact(a1, ref_a1, "device hand-off, modes switched")
    np.testing.assert_array_equal(dst, ref_dst)
    assert tmo == [0]


@pytest.mark.parametrize("C", [4096, 20000], ids=["c2", "above_grid_limit"])
def test_device_handoff_large_unsynchronised(cuda, C):
    """The C2 shape (64 back-end workgroups: the device hand-off) and a batch past half the CUs'
    worth of back-end workgroups (the event fallback), 12 calls back to back; sampled channels
    against the oracle."""
    import torch
    cfg = U.default_config()
    N, calls = 256, 12
    chain = U.RxChain(cfg, channels=C, frames=N)
    chain.set_pipelined(2)
    xs = [synth.ssb_iq_torch(0, C, k * N, N, cuda) for k in range(calls)]
    audio = torch.empty((calls, C, N), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for k in range(calls):
        chain.process(xs[k], audio[k], None)
    chain.synchronize()
    assert chain.handoff_timeouts() == 0
    chain.close()
    pick = np.arange(0, C, 61)
    iq = np.concatenate([x.cpu().numpy()[pick] for x in xs], axis=1)
    ref, _ = oracle.OracleRx(U.build_plan(cfg), len(pick)).process(np.ascontiguousarray(iq), threads=8)
    got = audio.permute(1, 0, 2).reshape(C, calls * N).cpu().numpy()[pick]
    assert_bitexact(got, ref, f"device hand-off C={C}")


def test_device_handoff_long_run(cuda):
    """120 calls back to back at the C2 shape with the device hand-off (every hand-off buffer reused
    40 times, 30 group transitions): sampled channels against the oracle, no poll giving up.  The
    inputs cycle through 6 device-generated blocks, so consecutive calls see different data."""
    import torch
    cfg = U.default_config()
    C, N, calls, pool = 4096, 256, 120, 6
    chain = U.RxChain(cfg, channels=C, frames=N)
    chain.set_pipelined(2)
    xs = [synth.ssb_iq_torch(0, C, k * N, N, cuda) for k in range(pool)]
    pick = np.arange(5, C, 97)
    full = torch.empty((calls, C, N), dtype=torch.float32, device="cuda")   # 0.5 GB: no join needed
    torch.cuda.synchronize()
    for k in range(calls):
        chain.process(xs[k % pool], full[k], None)     # no synchronisation: fronts run ahead
    chain.synchronize()
    audio = full[:, torch.from_numpy(pick).cuda(), :]
    assert chain.handoff_timeouts() == 0
    chain.close()
    iq = np.concatenate([xs[k % pool].cpu().numpy()[pick] for k in range(calls)], axis=1)
    ref, _ = oracle.OracleRx(U.build_plan(cfg), len(pick)).process(np.ascontiguousarray(iq), threads=8)
    got = audio.permute(1, 0, 2).reshape(len(pick), calls * N).cpu().numpy()
    assert_bitexact(got, ref, "device hand-off, 120 calls")


def test_device_handoff_front_delayed(cuda):
    """every call's rx_front is held back on the handle's stream (a spin kernel of
    ~100 us ahead of it, torch.cuda._sleep), so each rx_back -- already running on the side stream
    -- really polls the sequence word while its front runs, and then reads adec written from another
    XCD through sc1 loads.  Bit-exact against the oracle, no poll giving up."""
    import torch
    cfg = U.default_config()
    C, N, calls = 4096, 256, 10
    chain = U.RxChain(cfg, channels=C, frames=N, stream=torch.cuda.current_stream().cuda_stream)
    chain.set_pipelined(2)
    xs = [synth.ssb_iq_torch(0, C, k * N, N, cuda) for k in range(calls)]
    audio = torch.empty((calls, C, N), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for k in range(calls):
        torch.cuda._sleep(200_000)                   # on the handle's stream, ahead of rx_front
        chain.process(xs[k], audio[k], None)
    chain.synchronize()
    assert chain.handoff_timeouts() == 0
    chain.close()
    pick = np.arange(3, C, 67)
    iq = np.concatenate([x.cpu().numpy()[pick] for x in xs], axis=1)
    ref, _ = oracle.OracleRx(U.build_plan(cfg), len(pick)).process(np.ascontiguousarray(iq), threads=8)
    got = audio.permute(1, 0, 2).reshape(C, calls * N).cpu().numpy()[pick]
    assert_bitexact(got, ref, "device hand-off, fronts delayed")


def test_device_handoff_give_up_fails_loudly(cuda):
    """the failure contract of the device hand-off.  The poll bound is cut to 64
    polls and call 3's rx_front is held back ~25 ms on the handle's stream, so its rx_back gives up.
    Then: the call's audio is NaN (poisoned), synchronize() and every later process() raise
    UHSDR_TIMEOUT, handoff_timeouts() == 1; after reset() the handle runs bit-exact again."""
    import torch
    cfg = U.default_config()
    C, N = 256, 256
    iq = synth.ssb_iq(np.arange(C), 0, 6 * N)
    xs = [torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda() for k in range(6)]
    chain = U.RxChain(cfg, channels=C, frames=N, stream=torch.cuda.current_stream().cuda_stream)
    chain.set_pipelined(2)
    audio = torch.zeros((6, C, N), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for k in range(3):
        chain.process(xs[k], audio[k], None)
    chain.synchronize()
    assert chain.handoff_timeouts() == 0
    chain.set_handoff_bound(64)
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
    assert_bitexact(got[:3].transpose(1, 0, 2).reshape(C, 3 * N), ref, "calls before the give-up")
    # reset clears the failure word and the poisoned state; the default bound again
    chain.reset()
    chain.set_handoff_bound(1 << 24)
    assert chain.handoff_timeouts() == 0
    for k in range(3):
        chain.process(xs[k], audio[k], None)
    chain.synchronize()
    assert chain.handoff_timeouts() == 0
    assert_bitexact(audio[:3].cpu().numpy().transpose(1, 0, 2).reshape(C, 3 * N), ref, "after reset")
    with pytest.raises(U.UhsdrError):
        chain.set_pipelined(4)                       # modes are 0 .. 3 (3: persistent)
    chain.close()


@pytest.mark.parametrize("N", [128, 256], ids=["n4", "n8"])
def test_device_handoff_skew_transitions(cuda, N):
    """BackSched (the skewed wave pipeline): a launch runs ahead into the next
    call only when that call's front has already published; fronts delayed on every third call (and
    two in a row) make launches alternate between running ahead, draining, filling and starting
    skewed, in every combination, with N / 32 == BACK_SKEW (n4: the pre role has none of its own call
    left in a skewed launch) and 8.  Bit-exact against the oracle, no poll giving up."""
    import torch
    cfg = U.default_config()
    C, calls = 640, 19
    chain = U.RxChain(cfg, channels=C, frames=N, stream=torch.cuda.current_stream().cuda_stream)
    chain.set_pipelined(2)
    iq = synth.ssb_iq(np.arange(C), 0, calls * N)
    xs = [torch.from_numpy(np.ascontiguousarray(iq[:, k * N:(k + 1) * N])).cuda() for k in range(calls)]
    audio = torch.empty((calls, C, N), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for k in range(calls):
        if k % 3 == 2 or k in (10, 11):
            torch.cuda._sleep(150_000)
        chain.process(xs[k], audio[k], None)
    chain.synchronize()
    assert chain.handoff_timeouts() == 0
    chain.close()
    ref, _ = oracle.OracleRx(U.build_plan(cfg), C).process(iq, threads=8)
    got = audio.permute(1, 0, 2).reshape(C, calls * N).cpu().numpy()
    assert_bitexact(got, ref, f"skew transitions N={N}")
