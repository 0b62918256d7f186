"""normalize_codebooks (src/audio_tokenizer_decoder.cpp:40-73).

A tokenizer GGUF that still carries per-codebook `tok_dec.vq_{first.0,rest.N}.usage` tensors (an unconverted
checkpoint; the converter divides and drops them, scripts/convert_tokenizer_to_gguf.py:347-359) must be decoded with
every codebook row multiplied by 1 / max(usage[row], 1e-5) and re-rounded to f16.

CPU: the oracle's normalisation equals a numpy restatement of the reference loop, read straight from the file.
GPU: libq3t.so decodes the usage file exactly like the oracle, and differently from the same file without usage.
"""
import os
import sys

import numpy as np
import pytest

from gguf_py import GGUF
from oracle_py import Oracle
from q3t_testutil import REPO, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))


def _normalize_ref(cb, usage):
    """audio_tokenizer_decoder.cpp:52-62 restated: u = max(usage[r], 1e-5); row *= 1/u in f32, stored as f16"""
    u = np.maximum(usage.astype(np.float32), np.float32(1e-5))
    inv = (np.float32(1.0) / u).astype(np.float32)
    return (cb.astype(np.float32) * inv[:, None]).astype(np.float16).astype(np.float32)


def test_oracle_normalises_codebooks_like_the_reference():
    tts, tok = synth_dir("tiny", variant="usage")
    g = GGUF(tok)
    assert "tok_dec.vq_first.0.usage" in g.tensors
    orc = Oracle(tts, tok)
    try:
        for i in (0, 1, 15):
            pre = "tok_dec.vq_first.0." if i == 0 else f"tok_dec.vq_rest.{i - 1}."
            want = _normalize_ref(g.tensor(pre + "codebook"), g.tensor(pre + "usage"))
            got = orc.codebook(i)
            np.testing.assert_array_equal(got, want)
            assert not np.array_equal(got, g.tensor(pre + "codebook").astype(np.float32))
    finally:
        orc.close()


def test_plain_file_is_left_unchanged():
    tts, tok = synth_dir("tiny")
    g = GGUF(tok)
    assert not any(n.endswith(".usage") for n in g.tensors)
    orc = Oracle(tts, tok)
    try:
        np.testing.assert_array_equal(orc.codebook(3), g.tensor("tok_dec.vq_rest.2.codebook").astype(np.float32))
    finally:
        orc.close()


@pytest.mark.gpu
def test_gpu_vocoder_applies_usage():
    import q3t
    tts, tok = synth_dir("tiny", variant="usage")
    _, tok_plain = synth_dir("tiny")
    eng = q3t.Engine(None, tok, device=0, max_slots=1, max_ctx=64)
    plain = q3t.Engine(None, tok_plain, device=0, max_slots=1, max_ctx=64)
    orc = Oracle(tts, tok)
    try:
        codes = np.random.default_rng(4).integers(0, 2048, size=(9, 16), dtype=np.int32)
        g = eng.vocoder(codes, q3t.VOCODER_FULL)
        o = orc.vocoder(codes, 0)
        assert g.shape == o.shape
        assert float(np.abs(g - o).max()) < 1e-2
        assert float(np.abs(g - plain.vocoder(codes, q3t.VOCODER_FULL)).max()) > 1e-3   # the division took effect
    finally:
        eng.close()
        plain.close()
        orc.close()
