"""The batched talker step as ONE persistent launch (persist_tkb.hip) against the launch-per-op graph it replaces
(engine.cpp decoder_stack_mm + codec-head GEMM + select_tokens: 7 launches per layer, ~200 per step at >= 16 slots).

Every projection of the persistent step is the per-op MFMA tile with the same K quarters, split-K slices and LDS sum
order, every residual + RMSNorm is k_resid_norm's arithmetic, the attention is k_attn_seq's source (attn_seq.h) and the
CB0 selection is select_tokens': hidden states, logits and codes are compared BIT-EXACT.  A stale or torn in-launch
hand-off (flags + sc1 payloads, granules; MI355X_MICROARCH.md hand-off table) shows up as a mismatch.  Slot counts cover
one token tile (16, 17, 32) and two (33, 64), positions cross the attention's 64-position chunks (whole and last).
"""
import os
import sys

import numpy as np
import pytest

from q3t_testutil import REPO, prompt, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))

pytestmark = pytest.mark.gpu


def _engine(tts, tok, tkb, **kw):
    import q3t
    old = os.environ.get("Q3T_PERSIST_TKB")
    os.environ["Q3T_PERSIST_TKB"] = "1" if tkb else "0"
    try:
        return q3t.Engine(tts, tok, device=0, **kw)
    finally:
        if old is None:
            del os.environ["Q3T_PERSIST_TKB"]
        else:
            os.environ["Q3T_PERSIST_TKB"] = old


@pytest.fixture(scope="module")
def engines():
    tts, tok = synth_dir("full")
    ep = _engine(tts, None, True, max_slots=64, max_ctx=160)
    eg = _engine(tts, None, False, max_slots=64, max_ctx=160)
    assert ep.persist_kernels() & 32, "the batched persistent talker step is not in use on this device"
    assert not eg.persist_kernels() & 32
    yield ep, eg
    ep.close()
    eg.close()


@pytest.mark.parametrize("S", [16, 17, 32, 33, 64])
def test_tkb_step_bit_exact(engines, S):
    """talker_forward steps with per-slot positions: hidden state (the final norm's side output) and codec-head logits"""
    ep, eg = engines
    H = ep.cfg["hidden"]
    rng = np.random.default_rng(200 + S)
    off = np.arange(S) % 7
    for step in list(range(0, 70, 3)) + [126, 127, 128, 140]:
        pos = (step + off).astype(np.int32)
        x = (rng.standard_normal((S, H)) * 0.5).astype(np.float32)
        hp, lp = ep.talker_forward(x, pos)
        hg, lg = eg.talker_forward(x, pos)
        bad = [s for s in range(S) if not (np.array_equal(hp[s], hg[s]) and np.array_equal(lp[s], lg[s]))]
        assert not bad, (step, bad[:8], float(np.abs(hp[bad[0]] - hg[bad[0]]).max()), float(np.abs(lp[bad[0]] - lg[bad[0]]).max()))
    assert ep.persist_status() == 0


@pytest.mark.parametrize("n_utt", [16, 40, 64])
def test_tkb_generate_bit_exact(engines, n_utt):
    """whole generate() runs: CB0 selections inside the step, the hidden state the code-predictor frame reads, the K/V
    rows later steps read"""
    ep, eg = engines
    H = ep.cfg["hidden"]
    base = prompt("full")
    prompts = [base[:4] + [(t + 5 * i) % 900 + 20 for t in base[4:]] for i in range(n_utt)]
    spk = [np.zeros(H, np.float32)] * n_utt
    for kw in (dict(temperature=0.0), dict(temperature=0.9, top_k=50, seed=11)):
        a = ep.generate(prompts, speakers=spk, max_len=40, force_frames=12, **kw)
        b = eg.generate(prompts, speakers=spk, max_len=40, force_frames=12, **kw)
        bad = [i for i in range(n_utt) if not np.array_equal(a[i], b[i])]
        assert not bad, (kw, bad[:8])
    assert ep.persist_status() == 0


def test_tkb_queue_bit_exact(engines):
    """continuous batching at 20 active slots: parked (admitting / finished) slots beside running ones"""
    ep, eg = engines
    base = prompt("full")
    n = 30
    prompts = [base[:4] + [(t + 13 * i) % 900 + 20 for t in base[4:]][: 2 + i % 9] for i in range(n)]
    kw = dict(temperature=0.9, top_k=50, seed=4, max_len=24)
    a = ep.generate_queue(prompts, max_active=20, **kw)
    b = eg.generate_queue(prompts, max_active=20, **kw)
    bad = [i for i in range(n) if not np.array_equal(a[i], b[i])]
    assert not bad, bad[:8]
    assert ep.persist_status() == 0


def test_tkb_stage_time(engines):
    """the 64-slot step replays (time_stage) on the persistent launch without a fault"""
    ep, eg = engines
    tp = ep.time_stage(0, 64, 140, 5)
    tg = eg.time_stage(0, 64, 140, 5)
    assert ep.persist_status() == 0
    print(f"64-slot talker step at position 140: persistent {tp:.3f} ms, per-op {tg:.3f} ms")


def test_tkb_slot_invariance(engines):
    """a slot's hidden state and logits do not depend on how many slots the step runs: the first 16 (and 33) slots of
    a 64-slot step equal a 16-slot (33-slot) step on the same inputs and positions"""
    ep, _ = engines
    H = ep.cfg["hidden"]
    rng = np.random.default_rng(78)
    pos = (np.arange(64) % 9 + 40).astype(np.int32)
    x = (rng.standard_normal((64, H)) * 0.5).astype(np.float32)
    h64, l64 = ep.talker_forward(x, pos)
    for n in (16, 33):
        hn, ln = ep.talker_forward(x[:n], pos[:n])   # the same K/V rows rewritten with the same values
        assert np.array_equal(h64[:n], hn) and np.array_equal(l64[:n], ln), n
    assert ep.persist_status() == 0
