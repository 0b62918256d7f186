"""The causal prefill (Engine::prefill, q3t_talker_prefill; reference TTSTransformer::forward_prefill,
src/tts_transformer.cpp:1233-1374, 1829-1920): every prompt row of every utterance in ONE pass of the talker stack.

The prefill runs the projections with the kernels and K split of an S-slot decode step (family_slots = S) and its
attention reproduces the decode kernel's reduction tree over the first 64-position chunk, so for S <= 8 every
prefill row (final-norm hidden state, last-row logits) and every K/V row it writes equal the S-slot decode step
replayed position by position, BIT-EXACT.  From 16 slots the decode step switches to k_attn_seq (a different
summation order, checked against the oracle rather than bit for bit), so there the prefill is compared within the
oracle tolerance of tests/test_gpu_parity.py.  The oracle check pins the prefill rows to the CPU restatement.
"""
import os
import sys

import numpy as np
import pytest

from oracle_py import Oracle
from q3t_testutil import REPO, rel_err, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))

pytestmark = pytest.mark.gpu
TOL = {"tiny": 3e-3, "full": 5e-3}   # tests/test_gpu_parity.py


@pytest.fixture(scope="module", params=["tiny", "full"])
def eng(request):
    import q3t
    tts, tok = synth_dir(request.param)
    e = q3t.Engine(tts, None, device=0, max_slots=16, max_ctx=64)
    yield request.param, e, tts, tok
    e.close()


def _rows(e, n_utt, plen, seed):
    H = e.cfg["hidden"]
    return (np.random.default_rng(seed).standard_normal((n_utt, plen, H)) * 0.5).astype(np.float32)


def _replay(e, x):
    """the decode step replayed row by row with n_utt slots: hidden [n][plen][H], last-row logits [n][V]"""
    n, plen, _ = x.shape
    hid = np.zeros_like(x)
    lg = None
    for t in range(plen):
        h, lg = e.talker_forward(x[:, t], [t] * n)
        hid[:, t] = h
    return hid, lg


@pytest.mark.parametrize("n_utt", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("plen", [8, 10])
def test_prefill_equals_step_replay_bit_exact(eng, n_utt, plen):
    cfg, e, _, _ = eng
    x = _rows(e, n_utt, plen, 100 + n_utt * 16 + plen)
    hp, lp = e.talker_prefill(x)
    nxt = _rows(e, n_utt, 1, 7)[:, 0]
    # the K/V rows the prefill wrote: the next decode step at position plen reads them
    hn_p, ln_p = e.talker_forward(nxt, [plen] * n_utt)
    hr, lr = _replay(e, x)
    hn_r, ln_r = e.talker_forward(nxt, [plen] * n_utt)
    assert np.array_equal(hp, hr), (n_utt, plen, float(np.abs(hp - hr).max()))
    assert np.array_equal(lp, lr), (n_utt, plen, float(np.abs(lp - lr).max()))
    assert np.array_equal(hn_p, hn_r) and np.array_equal(ln_p, ln_r)


def test_prefill_family_is_per_row(eng):
    """an utterance's prefill rows depend on the kernel family only, not on the utterances run alongside"""
    cfg, e, _, _ = eng
    x = _rows(e, 6, 9, 5)
    full, lg_full = e.talker_prefill(x, family_slots=6)
    for u in (0, 3, 5):
        one, lg_one = e.talker_prefill(x[u:u + 1], family_slots=6)
        assert np.array_equal(one[0], full[u]) and np.array_equal(lg_one[0], lg_full[u])


def test_prefill_16_slots_within_tolerance(eng):
    cfg, e, _, _ = eng
    x = _rows(e, 16, 9, 9)
    hp, lp = e.talker_prefill(x)
    hr, lr = _replay(e, x)
    assert rel_err(hp, hr) < TOL[cfg]
    assert rel_err(lp, lr) < TOL[cfg]


def test_prefill_matches_oracle(eng):
    cfg, e, tts, tok = eng
    x = _rows(e, 1, 10, 21)
    hp, lp = e.talker_prefill(x)
    orc = Oracle(tts, tok)
    try:
        kv = orc.kv_new(64, 0)
        for t in range(10):
            ho, lo = orc.talker_step(kv, x[0, t], t)
            assert rel_err(hp[0, t], ho) < TOL[cfg], t
        assert rel_err(lp[0], lo) < TOL[cfg]
        orc.kv_free(kv)
    finally:
        orc.close()


def test_prefill_edge_cases(eng):
    import q3t
    cfg, e, _, _ = eng
    one, lg = e.talker_prefill(_rows(e, 1, 1, 3))
    h, l1 = e.talker_forward(_rows(e, 1, 1, 3)[:, 0], [0])
    assert np.array_equal(one[:, 0], h) and np.array_equal(lg, l1)
    with pytest.raises(q3t.Q3TError):
        e.talker_prefill(_rows(e, 1, 11, 3))   # more rows than the prefill holds
    with pytest.raises(q3t.Q3TError):
        e.talker_prefill(_rows(e, 17, 8, 3))   # more utterances than slots
