"""GPU tests of the C++ mirror of the reference runtime classes (qwen3-tts-jetson_amd/cpp/qwen3_tts_hip.h).

tests/cpp/test_host_api.cpp drives qwen3_tts::TTSTransformer / AudioTokenizerDecoder / TRTVocoderDecoder the way
src/qwen3_tts.cpp:437-463,518 drives the reference classes, self-checks the host contract (errors, callback frames
== output, stop on false, prefill == step replay, sample counts) and writes its numeric outputs; this file checks
those against the CPU oracle (talker step, code predictor, generate: teacher-forced decisions) and against the
ctypes path over the same C ABI (vocoders: identical kernels, so identical samples).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle_py import Oracle
from q3t_testutil import REPO, check_decisions, check_token, prompt, rel_err, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))

pytestmark = pytest.mark.gpu
BIN = os.path.join(REPO, "tests", "cpp", "_build", "test_host_api")
TOL = {"tiny": 3e-3, "full": 5e-3}


@pytest.fixture(scope="module", params=["tiny", "full"])
def run(request, tmp_path_factory):
    cfg = request.param
    assert os.path.exists(BIN), "tests/cpp/_build/test_host_api missing: run __graft_entry__.build()"
    tts, tok = synth_dir(cfg)
    d = tmp_path_factory.mktemp(f"cpp_{cfg}")
    toks = prompt(cfg)
    np.asarray(toks, np.int32).tofile(d / "prompt.bin")
    r = subprocess.run([BIN, tts, tok, str(d)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout, (r.returncode, r.stdout, r.stderr[-3000:])
    orc = Oracle(tts, tok)
    yield cfg, tts, tok, d, toks, orc
    orc.close()


def _f32(d, n):
    return np.fromfile(d / n, np.float32)


def _i32(d, n):
    return np.fromfile(d / n, np.int32)


def test_cpp_forward_step_matches_oracle(run):
    cfg, tts, tok, d, toks, orc = run
    embd = _f32(d, "step_embd.bin").reshape(4, -1)
    H = embd.shape[1]
    logits = _f32(d, "step_logits.bin").reshape(4, -1)
    hidden = _f32(d, "step_hidden.bin").reshape(4, H)
    kv = orc.kv_new(64, 0)
    for p in range(4):
        ho, lo = orc.talker_step(kv, embd[p], p)
        assert rel_err(hidden[p], ho) < TOL[cfg], p
        assert rel_err(logits[p], lo) < TOL[cfg], p
    orc.kv_free(kv)


def test_cpp_predict_codes_matches_oracle(run):
    cfg, tts, tok, d, toks, orc = run
    hid = _f32(d, "cp_hidden.bin")
    codes = _i32(d, "cp_codes.bin")
    assert codes.shape == (15,)
    ol = orc.cp_frame_forced(hid, 77, codes)
    off = sum(check_token(ol[i], int(codes[i]), 0.0, 0, 0.0) for i in range(15))
    assert off <= 1, off


def test_cpp_generate_matches_oracle_and_ctypes_path(run):
    cfg, tts, tok, d, toks, orc = run
    import q3t
    codes = _i32(d, "gen_codes.bin").reshape(-1, 16)
    H = _f32(d, "cp_hidden.bin").shape[0]
    spk = np.zeros(H, np.float32)
    check_decisions(orc, toks, spk, codes, max_len=10, temperature=0.0)
    eng = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=10 + 10 + 8)
    try:
        ref = eng.generate([toks], speakers=[spk], max_len=10, temperature=0.0)[0]
    finally:
        eng.close()
    assert np.array_equal(ref, codes)


def test_cpp_generate_batch_sampling_matches_oracle(run):
    cfg, tts, tok, d, toks, orc = run
    lens = _i32(d, "batch_lens.bin")
    flat = _i32(d, "batch_codes.bin")
    pflat = _i32(d, "batch_prompts.bin")
    H = _f32(d, "cp_hidden.bin").shape[0]
    spk = np.zeros(H, np.float32)
    off = pos = 0
    for u, n in enumerate(lens):
        pl = int(pflat[pos])
        p = [int(x) for x in pflat[pos + 1:pos + 1 + pl]]
        pos += 1 + pl
        c = flat[off * 16:(off + n) * 16].reshape(n, 16)
        off += n
        check_decisions(orc, p, spk, c, max_len=10, temperature=0.9, top_k=50, seed=99, utt=u, max_off_frac=0.06)


def test_cpp_vocoders_match_ctypes_path(run):
    cfg, tts, tok, d, toks, orc = run
    import q3t
    codes = _i32(d, "voc_codes.bin").reshape(-1, 16)
    eng = q3t.Engine(None, tok, device=0)
    try:
        full = eng.vocoder(codes, q3t.VOCODER_FULL)
        c40 = eng.vocoder(codes, q3t.VOCODER_CHUNK40)
        c16 = eng.vocoder_chunked(codes, 16)
        # a vocoder-only context rejects the talker entry points
        import ctypes as C
        ms = C.c_double(0)
        assert q3t.lib().q3t_time_stage(eng.h, 0, 1, 0, 1, C.byref(ms)) != 0
        assert b"vocoder-only" in q3t.lib().q3t_last_error()
    finally:
        eng.close()
    np.testing.assert_allclose(_f32(d, "voc_full.bin"), full, rtol=0, atol=1e-6)
    np.testing.assert_allclose(_f32(d, "voc_chunk40.bin"), c40, rtol=0, atol=1e-6)
    np.testing.assert_allclose(_f32(d, "voc_chunk16.bin"), c16, rtol=0, atol=1e-6)
    assert c16.shape[0] == codes.shape[0] * 1920
    # chunked semantics: chunks are independent (no left context), so the first 16-frame chunk equals the chunked
    # decode of frames 0..15 alone
    eng = q3t.Engine(None, tok, device=0)
    try:
        first = eng.vocoder_chunked(codes[:16], 16)
    finally:
        eng.close()
    np.testing.assert_allclose(c16[:16 * 1920], first, rtol=0, atol=1e-6)
