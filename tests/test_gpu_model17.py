"""GPU parity of the 1.7B model layout: a code predictor narrower than the talker (its own hidden / FFN width and head
counts) fed through code_pred.mtp_proj, which projects every code-predictor input -- the talker hidden state of
pass 0 and the talker-space table rows of passes 1..15 -- into the code predictor's space.

Reference: src/tts_transformer.cpp:370-389 (the code_predictor.* config keys, falling back to the talker's values),
:600-616 / :709-712 (code_pred.* tensor shapes; mtp_proj.{weight,bias}), :1554-1560 (projection in the prefill graph),
:1709-1714 (projection in the step graph); src/trt_code_predictor.cpp:399-416 / :453-471 (its GPU upload).  No fixture
in the reference covers the 1.7B path: parity is against the oracle's restatement (parity unpinned).

Configs (tools/q3t_synth.c): tiny17 = talker 512 wide (8 q / 2 kv heads of 64), code predictor 256 wide (4 q / 2 kv
heads); full17 = the real 1.7B shapes (talker 2048 / FFN 6144, code predictor 1024 / 3072).  These models run every
projection on the vector GEMV kernels with a 1-slot K split (the batched matrix-core stack is built for the 0.6B
widths); the persistent kernels do not cover them.  Tolerances: those of test_gpu_parity.py.
"""
import os
import sys

import numpy as np
import pytest

from oracle_py import Oracle
from q3t_testutil import REPO, check_decisions, check_token, prompt, rel_err, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tiny17():
    import q3t
    tts, tok = synth_dir("tiny17")
    eng = q3t.Engine(tts, tok, device=0, max_slots=4, max_ctx=96)
    orc = Oracle(tts, tok)
    yield eng, orc
    eng.close()
    orc.close()


def test_config_reports_code_predictor_geometry(tiny17):
    eng, orc = tiny17
    c = eng.cfg
    assert (c["hidden"], c["cp_hidden"], c["cp_intermediate"], c["cp_heads"], c["cp_kv_heads"], c["has_mtp"]) == \
        (orc.cfg["hidden"], orc.cfg["cp_hidden"], orc.cfg["cp_inter"], orc.cfg["cp_heads"], orc.cfg["cp_kv"], 1)
    assert c["cp_hidden"] != c["hidden"]
    assert eng.persist_status() == -1   # launch-per-op graphs (a 256-wide code predictor: no persistent frame)


def test_talker_step_matches_oracle(tiny17):
    eng, orc = tiny17
    H = eng.cfg["hidden"]
    rng = np.random.default_rng(3)
    kv = orc.kv_new(96, 0)
    for pos in range(12):
        e = (rng.standard_normal(H) * 0.5).astype(np.float32)
        hg, lg = eng.talker_forward(e[None], [pos])
        ho, lo = orc.talker_step(kv, e, pos)
        assert rel_err(hg[0], ho) < 3e-3, pos
        assert rel_err(lg[0], lo) < 3e-3, pos
    orc.kv_free(kv)


@pytest.mark.parametrize("temperature", [0.0, 0.9])
def test_codepred_frame_matches_oracle(tiny17, temperature):
    """15 passes through mtp_proj: logits teacher-forced on the GPU's own codes, every code the oracle's decision"""
    eng, orc = tiny17
    H = eng.cfg["hidden"]
    rng = np.random.default_rng(7)
    hid = (rng.standard_normal((3, H)) * 1.5).astype(np.float32)
    cb0 = np.array([11, 700, 2047], np.int32)
    codes, lg = eng.codepred_frame(hid, cb0, temperature=temperature, top_k=50, seed=4, frame=2, want_logits=True)
    off = 0
    for s in range(3):
        ol = orc.cp_frame_forced(hid[s], int(cb0[s]), codes[s])
        assert np.abs(lg[s] - ol).max() < 5e-2, s
        if temperature <= 0:
            off += sum(check_token(ol[i], int(codes[s, i]), 0.0, 0, 0.0) for i in range(15))
    assert off <= 2


@pytest.mark.parametrize("slots,temperature", [(1, 0.0), (1, 0.9), (4, 0.9)])
def test_generate_matches_oracle(tiny17, slots, temperature):
    eng, orc = tiny17
    H = eng.cfg["hidden"]
    base = prompt("tiny17")
    prompts = [base[:4] + [(t + 37 * i) % 900 + 20 for t in base[4:]] for i in range(slots)]
    spk = [np.zeros(H, np.float32)] * slots
    outs = eng.generate(prompts, speakers=spk, max_len=24, temperature=temperature, top_k=50, seed=31, force_frames=24)
    for i, out in enumerate(outs):
        assert out.shape == (24, 16)
        n_off, n_dec, worst = check_decisions(orc, prompts[i], spk[i], out, max_len=24, force_frames=24,
                                              temperature=temperature, top_k=50, seed=31, utt=i, max_off_frac=0.05)
        print(f"tiny17 slots={slots} T={temperature} utt {i}: {n_dec - n_off}/{n_dec} exact, worst {worst:.3g}")


def test_full17_shapes_generate_and_vocoder():
    """the real 1.7B geometry (talker 2048 / 6144, code predictor 1024 / 3072 behind mtp_proj) end to end: codes
    teacher-forced against the oracle, then the FULL vocoder on them"""
    import q3t
    tts, tok = synth_dir("full17")
    eng = q3t.Engine(tts, tok, device=0, max_slots=1, max_ctx=64)
    orc = Oracle(tts, tok)
    try:
        c = eng.cfg
        assert (c["hidden"], c["intermediate"], c["cp_hidden"], c["cp_intermediate"], c["has_mtp"]) == (2048, 6144, 1024, 3072, 1)
        # the talker step at the real widths (K 2,048 / 6,144 GEMVs: NL 16 / 24 weight loads in flight, whole-round
        # grids) against the oracle, position by position (2e-3: ~2.5x the observed 7.8e-4)
        H = c["hidden"]
        rng = np.random.default_rng(5)
        kv = orc.kv_new(64, 0)
        worst = 0.0
        for pos in range(6):
            e = (rng.standard_normal(H) * 0.5).astype(np.float32)
            hg, lg = eng.talker_forward(e[None], [pos])
            ho, lo = orc.talker_step(kv, e, pos)
            worst = max(worst, rel_err(hg[0], ho), rel_err(lg[0], lo))
            assert rel_err(hg[0], ho) < 2e-3 and rel_err(lg[0], lo) < 2e-3, (pos, rel_err(hg[0], ho), rel_err(lg[0], lo))
        orc.kv_free(kv)
        print(f"full17 talker step vs oracle: worst rel err {worst:.3g}")
        toks = prompt("full17")
        spk = np.zeros(c["hidden"], np.float32)
        out = eng.generate([toks], speakers=[spk], max_len=12, temperature=0.0, force_frames=12)[0]
        assert out.shape == (12, 16)
        n_off, n_dec, worst = check_decisions(orc, toks, spk, out, max_len=12, force_frames=12, temperature=0.0,
                                              max_off_frac=0.05)
        print(f"full17 B=1 12 frames: {n_dec - n_off}/{n_dec} exact, worst {worst:.3g}")
        pcm = eng.vocoder(out)
        ref = orc.vocoder(out)
        assert pcm.shape == ref.shape
        assert np.abs(pcm - ref).max() < 1e-2
    finally:
        eng.close()
        orc.close()


def test_full17_persistent_code_predictor_bit_exact():
    """1.7B at one slot: the code-predictor frame runs as the persistent launch (its code predictor has the 0.6B
    shapes) on projected table rows and a projected pass-0 input; it must equal the launch-per-op frame bit for bit
    (the per-op code predictor with its attention as its own launch, the arithmetic the persistent frame reproduces)"""
    import q3t
    tts, tok = synth_dir("full17")
    env = {"Q3T_PERSIST": "0", "Q3T_CP_FUSED_ATTN": "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ref = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=64)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    eng = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=64)
    try:
        assert eng.persist_status() == 0 and ref.persist_status() == -1
        assert eng.persist_kernels() & 4, eng.persist_kernels()   # the role-specialised frame (persist_cp.hip)
        H = eng.cfg["hidden"]
        rng = np.random.default_rng(9)
        for frame in range(6):
            hid = (rng.standard_normal(H) * 1.5).astype(np.float32)
            cb0 = int(rng.integers(0, 2048))
            for T in (0.0, 0.9):
                a = eng.codepred_frame(hid[None], [cb0], temperature=T, top_k=50, seed=3, frame=frame)
                b = ref.codepred_frame(hid[None], [cb0], temperature=T, top_k=50, seed=3, frame=frame)
                assert np.array_equal(a, b), (frame, T, a, b)
        toks = prompt("full17")
        kw = dict(speakers=[np.zeros(H, np.float32)], max_len=16, temperature=0.9, top_k=50, seed=5, force_frames=16)
        want = ref.generate([toks], **kw)[0]
        assert np.array_equal(eng.generate([toks], **kw)[0], want)
        assert eng.persist_status() == 0
        # a 1-slot replica (weights copied device to device after its layout) builds its projected table from the
        # copied weights, not from the empty arena: same codes as its source
        rep = eng.replica(0, 1, 64)
        try:
            assert rep.persist_status() == 0
            assert np.array_equal(rep.generate([toks], **kw)[0], want)
        finally:
            rep.close()
    finally:
        eng.close()
        ref.close()
