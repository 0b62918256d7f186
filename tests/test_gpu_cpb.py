"""The batched code-predictor frame as ONE persistent launch (persist_cpb.hip) against the launch-per-op graph it
replaces (engine.cpp decoder_stack_mm + head GEMMs + k_select_embed_norm, ~570 launches per frame at 64 slots).

Every projection of the persistent frame is the per-op MFMA tile with the same K quarters, split-K slices and LDS sum
order, every residual + RMSNorm is k_resid_norm's arithmetic, the attention is k_attn_small's source (attn_small.h) and
the selection is k_select_embed_norm's: codes, and everything downstream of them, are compared BIT-EXACT.  A stale or
torn in-launch hand-off (flags + sc1 payloads, MI355X_MICROARCH.md hand-off table row 1) shows up as a mismatch.
Slot counts cover one token tile (4, 17, 32) and two (33, 64), partial tiles included; the talker step embedding the
frame hands to the next talker step is covered through generate() and continuous batching.
"""
import os
import sys

import numpy as np
import pytest

from q3t_testutil import REPO, prompt, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))

pytestmark = pytest.mark.gpu


def _engine(tts, tok, cpb, **kw):
    import q3t
    old = os.environ.get("Q3T_PERSIST_CPB")
    os.environ["Q3T_PERSIST_CPB"] = "1" if cpb else "0"
    try:
        return q3t.Engine(tts, tok, device=0, **kw)
    finally:
        if old is None:
            del os.environ["Q3T_PERSIST_CPB"]
        else:
            os.environ["Q3T_PERSIST_CPB"] = old


@pytest.fixture(scope="module")
def engines():
    tts, tok = synth_dir("full")
    ep = _engine(tts, None, True, max_slots=64, max_ctx=96)
    eg = _engine(tts, None, False, max_slots=64, max_ctx=96)
    assert ep.persist_kernels() & 16, "the batched persistent code-predictor frame is not in use on this device"
    assert not eg.persist_kernels() & 16
    yield ep, eg
    ep.close()
    eg.close()


@pytest.mark.parametrize("S", [4, 17, 32, 33, 64])
@pytest.mark.parametrize("temperature", [0.0, 0.9])
def test_cpb_frame_bit_exact(engines, S, temperature):
    ep, eg = engines
    H = ep.cfg["hidden"]
    rng = np.random.default_rng(100 + S)
    for frame in range(3):
        hid = (rng.standard_normal((S, H)) * 1.5).astype(np.float32)
        cb0 = rng.integers(0, 2048, S).astype(np.int32)
        cp = ep.codepred_frame(hid, cb0, temperature=temperature, top_k=50, seed=5, frame=frame)
        cg = eg.codepred_frame(hid, cb0, temperature=temperature, top_k=50, seed=5, frame=frame)
        bad = [s for s in range(S) if not np.array_equal(cp[s], cg[s])]
        assert not bad, (frame, bad[:8], cp[bad[0]], cg[bad[0]])
    assert ep.persist_status() == 0


@pytest.mark.parametrize("n_utt", [5, 40])
def test_cpb_generate_bit_exact(engines, n_utt):
    """whole generate() runs: the frame's selections, its talker step embedding (x / xn of the next talker step) and
    the talker steps that consume it"""
    ep, eg = engines
    H = ep.cfg["hidden"]
    base = prompt("full")
    prompts = [base[:4] + [(t + 7 * i) % 900 + 20 for t in base[4:]] for i in range(n_utt)]
    spk = [np.zeros(H, np.float32)] * n_utt
    for kw in (dict(temperature=0.0), dict(temperature=0.9, top_k=50, seed=7)):
        a = ep.generate(prompts, speakers=spk, max_len=24, force_frames=24, **kw)
        b = eg.generate(prompts, speakers=spk, max_len=24, force_frames=24, **kw)
        bad = [i for i in range(n_utt) if not np.array_equal(a[i], b[i])]
        assert not bad, (kw, bad[:8])
    assert ep.persist_status() == 0


def test_cpb_queue_bit_exact(engines):
    """continuous batching: frames of 8..S_eff slots with parked (admitting / finished) slots beside running ones"""
    ep, eg = engines
    H = ep.cfg["hidden"]
    base = prompt("full")
    n = 24
    prompts = [base[:4] + [(t + 11 * i) % 900 + 20 for t in base[4:]][: 2 + i % 9] for i in range(n)]
    kw = dict(temperature=0.9, top_k=50, seed=3, max_len=20)
    a = ep.generate_queue(prompts, max_active=12, **kw)
    b = eg.generate_queue(prompts, max_active=12, **kw)
    bad = [i for i in range(n) if not np.array_equal(a[i], b[i])]
    assert not bad, bad[:8]
    assert ep.persist_status() == 0


def test_cpb_stage_time(engines):
    """the 64-slot frame replays (time_stage) on the persistent launch without a fault, faster than the per-op graph"""
    ep, eg = engines
    tp = ep.time_stage(1, 64, 0, 5)
    tg = eg.time_stage(1, 64, 0, 5)
    assert ep.persist_status() == 0
    print(f"64-slot CP frame: persistent {tp:.3f} ms, per-op {tg:.3f} ms")


def test_cpb_slot_invariance(engines):
    """a slot's codes do not depend on how many slots the frame runs: the first 8 slots of a 64-slot frame equal an
    8-slot frame on the same inputs (one token tile vs two; the MFMA columns, split-K slices and norms are per token)"""
    ep, _ = engines
    H = ep.cfg["hidden"]
    rng = np.random.default_rng(77)
    hid = (rng.standard_normal((64, H)) * 1.5).astype(np.float32)
    cb0 = rng.integers(0, 2048, 64).astype(np.int32)
    for temperature in (0.0, 0.9):
        c64 = ep.codepred_frame(hid, cb0, temperature=temperature, top_k=50, seed=9, frame=3)
        c8 = ep.codepred_frame(hid[:8], cb0[:8], temperature=temperature, top_k=50, seed=9, frame=3)
        c33 = ep.codepred_frame(hid[:33], cb0[:33], temperature=temperature, top_k=50, seed=9, frame=3)
        assert np.array_equal(c64[:8], c8), temperature
        assert np.array_equal(c64[:33], c33), temperature
    assert ep.persist_status() == 0
