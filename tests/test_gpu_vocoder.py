"""GPU parity of the vocoder (tokenizer decoder) against the CPU oracle: FULL (GGML decoder semantics,
audio_tokenizer_decoder.cpp:622-802) and CHUNK40 (TRT streaming semantics, trt_vocoder.cpp:98-170).

PCM tolerance: both sides round every conv/matmul input to f16 and differ only in f32 summation order
(MFMA vs AVX2); measured max |dPCM| is printed and bounded by PCM_TOL below (PCM is in [-1, 1])."""
import os
import sys

import numpy as np
import pytest

from oracle_py import Oracle
from q3t_testutil import REPO, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
pytestmark = pytest.mark.gpu
PCM_TOL = {"tiny": 6e-3, "full": 6e-3}   # measured max |dPCM| 3.7e-3 / 3.6e-3 (3.8e-3 at 512 frames), rms <= 7e-4


@pytest.fixture(scope="module", params=["tiny", "full"])
def pair(request):
    import q3t
    cfg = request.param
    tts, tok = synth_dir(cfg)
    eng = q3t.Engine(tts, tok, device=0, max_slots=1, max_ctx=64)
    orc = Oracle(tts, tok)
    yield cfg, eng, orc
    eng.close()
    orc.close()


def _codes(F, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 2048, size=(F, 16), dtype=np.int32)


@pytest.mark.parametrize("F", [1, 7, 40])
def test_vocoder_full_matches_oracle(pair, F):
    cfg, eng, orc = pair
    codes = _codes(F, F)
    g = eng.vocoder(codes, 0)
    o = orc.vocoder(codes, 0)
    assert g.shape == o.shape == (eng.vocoder_num_samples(F, 0),)
    err = float(np.abs(g - o).max())
    rms = float(np.sqrt(np.mean((g - o) ** 2)))
    print(f"{cfg} F={F} full: max|d|={err:.3e} rms={rms:.3e} pcm_std={o.std():.3f}")
    assert err < PCM_TOL[cfg] and rms < 2e-3


def test_vocoder_chunk40_matches_oracle(pair):
    cfg, eng, orc = pair
    F = 47   # one full chunk + a ragged 7-frame chunk
    codes = _codes(F, 3)
    g = eng.vocoder(codes, 1)
    o = orc.vocoder(codes, 1)
    assert g.shape == o.shape == (F * 1920,)
    err = float(np.abs(g - o).max())
    print(f"{cfg} chunk40: max|d|={err:.3e}")
    assert err < PCM_TOL[cfg]


def test_vocoder_lengths(pair):
    cfg, eng, orc = pair
    for F in (1, 2, 40, 513):
        assert eng.vocoder_num_samples(F, 0) == orc.vocoder_len(F, 0)
        assert eng.vocoder_num_samples(F, 1) == F * 1920
    assert eng.vocoder(np.zeros((0, 16), np.int32), 0).shape == (0,)


def test_vocoder_batch_matches_single(pair):
    """q3t_vocoder_decode_batch: utterances of different lengths through shared launches (padded to the batch's
    longest, causal end to end) equal their single decodes BIT-EXACT (the row GEMVs' kernel family and K split are
    pinned to one batch size, vocoder.cpp row_gemv, so a row's summation order does not depend on the row count), and
    the oracle within PCM_TOL; a batch_frames cap forces several batches"""
    cfg, eng, orc = pair
    lens = [33, 7, 40, 1, 64, 12]
    codes = [_codes(F, 100 + F) for F in lens]
    for cap in (4096, 80):   # one batch / several batches of <= 80 frames
        eng.vocoder_set_batch_frames(cap)
        outs = eng.vocoder_batch(codes, 0)
        worst = 0.0
        for c, g in zip(codes, outs):
            s = eng.vocoder(c, 0)
            assert g.shape == s.shape
            worst = max(worst, float(np.abs(g - s).max()))
        print(f"{cfg} batch(cap {cap}) vs single: max|d|={worst:.3e}")
        assert worst == 0.0, worst
    eng.vocoder_set_batch_frames(4096)
    for i in (0, 3):
        o = orc.vocoder(codes[i], 0)
        assert float(np.abs(outs[i] - o).max()) < PCM_TOL[cfg]


def test_vocoder_batch_chunk40(pair):
    """CHUNK40 through the batch entry: every 40-frame chunk of every utterance is one sequence of the batch"""
    cfg, eng, orc = pair
    lens = [47, 40, 5]
    codes = [_codes(F, 200 + F) for F in lens]
    outs = eng.vocoder_batch(codes, 1, 40)
    for c, g in zip(codes, outs):
        assert g.shape == (c.shape[0] * 1920,)
        s = eng.vocoder_chunked(c, 40)
        assert float(np.abs(g - s).max()) < 2e-3
    o = orc.vocoder(codes[0], 1)
    assert float(np.abs(outs[0] - o).max()) < PCM_TOL[cfg]


@pytest.mark.parametrize("F,nutt", [(40, 1), (200, 1), (33, 3)])
def test_fused_residual_unit_bit_exact(F, nutt):
    """the 96-channel residual units as one launch each (vocoder_resunit.hip) against their two-conv form
    (Q3T_VOC_FUSE=0): bit-identical PCM, single decodes and an utterance batch"""
    import q3t
    tts, tok = synth_dir("full")
    old = os.environ.get("Q3T_VOC_FUSE")
    os.environ["Q3T_VOC_FUSE"] = "0"
    try:
        ref = q3t.Engine(None, tok, device=0)
    finally:
        if old is None:
            del os.environ["Q3T_VOC_FUSE"]
        else:
            os.environ["Q3T_VOC_FUSE"] = old
    fused = q3t.Engine(None, tok, device=0)
    try:
        cl = [_codes(F + 7 * u, 100 + u) for u in range(nutt)]
        if nutt == 1:
            a, b = [fused.vocoder(cl[0], 0)], [ref.vocoder(cl[0], 0)]
        else:
            a, b = fused.vocoder_batch(cl, 0), ref.vocoder_batch(cl, 0)
        for x, y in zip(a, b):
            assert x.shape == y.shape
            assert np.array_equal(x, y), float(np.abs(x - y).max())
    finally:
        fused.close()
        ref.close()


@pytest.mark.parametrize("lens", [(512,), (280, 300, 271)])
def test_pipelined_conv_bit_exact(lens):
    """the wide blocks' dilated 7-tap convs on k_conv_pd (LDS-DMA double-buffered K chunks; 256- and 512-row tiles)
    against k_conv_mt (Q3T_CONV_PD=0, read at every launch): bit-identical PCM.  512 frames put the 768-, 384- and
    192-channel blocks' convs on the pipelined kernel (the 768-channel block needs >= 512 frames), the 3-utterance
    batch the 384- and 192-channel blocks with grid z"""
    import q3t
    tts, tok = synth_dir("full")
    eng = q3t.Engine(None, tok, device=0)
    old = os.environ.get("Q3T_CONV_PD")
    try:
        cl = [_codes(F, 300 + F) for F in lens]
        run = (lambda: [eng.vocoder(cl[0], 0)]) if len(cl) == 1 else (lambda: eng.vocoder_batch(cl, 0))
        os.environ["Q3T_CONV_PD"] = "0"
        ref = run()
        for mode in ("1", "2"):   # 256- and 512-row tiles
            os.environ["Q3T_CONV_PD"] = mode
            got = run()
            for x, y in zip(got, ref):
                assert x.shape == y.shape
                assert np.array_equal(x, y), (mode, float(np.abs(x - y).max()))
    finally:
        if old is None:
            os.environ.pop("Q3T_CONV_PD", None)
        else:
            os.environ["Q3T_CONV_PD"] = old
        eng.close()
