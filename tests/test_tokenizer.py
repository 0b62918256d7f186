"""Text tokenizer (src/text_tokenizer.cpp): the product tokenizer (csrc/tokenizer.cpp through the C ABI)
against the reference's own known-answer vector and against the Python restatement oracle/text_tokenizer_ref.py.

Pinning: the reference's known-answer test (tests/test_tokenizer.cpp:11-14) expects
[151644, 77091, 198, 9707, 13, 151645, 198, 151644, 77091, 198] for encode_for_tts("Hello.") with the real Qwen vocab.
That vocab is not in this container, so the synthetic TTS GGUF (tools/q3t_synth.c build_vocab) places the tokens that
vector needs at their Qwen ids (byte symbols 0..255 in Qwen's order, "Hello" = 9707, "assistant" = 77091, the
converter's "[PAD<id>]" rows from 151643 on); everything else is "parity pinned to the restatement" only.
No GPU: the tokenizer is host code."""
import os
import random
import zlib
import sys

import pytest

from q3t_testutil import REPO, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
from text_tokenizer_ref import RefTokenizer, read_gguf_kv  # noqa: E402

KNOWN_ANSWER = [151644, 77091, 198, 9707, 13, 151645, 198, 151644, 77091, 198]


def _pair(cfg):
    import q3t
    tts, _ = synth_dir(cfg)
    return q3t.Tokenizer(tts), RefTokenizer(read_gguf_kv(tts))


@pytest.fixture(scope="module")
def tiny():
    t, r = _pair("tiny")
    yield t, r
    t.close()


@pytest.fixture(scope="module")
def full():
    t, r = _pair("full")
    yield t, r
    t.close()


def test_known_answer_hello(full):
    tok, ref = full
    assert tok.vocab_size == 151936
    assert (tok.bos, tok.eos, tok.pad) == (151644, 151645, 151643)   # text_tokenizer.h:13-18 defaults
    assert tok.encode("Hello.") == [9707, 13]                          # test_tokenizer.cpp:81-83
    assert tok.encode_for_tts("Hello.") == KNOWN_ANSWER               # test_tokenizer.cpp:14
    assert ref.encode_for_tts("Hello.") == KNOWN_ANSWER
    assert tok.decode(tok.encode("Hello.")) == b"Hello."               # test_tokenizer.cpp:133-139
    assert tok.decode([151644]) == b"[PAD151644]"                      # special ids are converter pads


WORDS = ["Hello", "hello", "world", "the", "voice", "model", "quick", "brown", "fox", "assistant", "jumps", "GPU",
         "speech", "test", "2026", "ing", "héllo", "wörld", "日本語", "naïve", "🙂", "...", "!!", "a", "tion"]
SEPS = [" ", "  ", ", ", ". ", "\n", "\t", "", "-", " \n "]


def _random_texts(n, seed):
    rng = random.Random(seed)
    out = ["", " ", "  ", "\n", "Hello", " Hello", "Hello  world", "hello\n\nworld", "\x00\x01\x7f", "é", "ĠĊ"]
    for _ in range(n):
        k = rng.randint(1, 12)
        out.append("".join(rng.choice(WORDS) + rng.choice(SEPS) for _ in range(k)))
    out.append("".join(chr(rng.randint(32, 0x2FFF)) for _ in range(200)))
    return out


@pytest.mark.parametrize("cfg", ["tiny", "full"])
def test_encode_matches_restatement(cfg, request):
    tok, ref = request.getfixturevalue(cfg)
    for text in _random_texts(150, seed=zlib.crc32(cfg.encode())):
        assert tok.encode(text) == ref.encode(text), repr(text)
        assert tok.encode_for_tts(text) == ref.encode_for_tts(text), repr(text)


@pytest.mark.parametrize("cfg", ["tiny", "full"])
def test_decode_round_trip(cfg, request):
    """byte symbols are a bijection, so decode(encode(x)) == x whenever every piece is in the vocab or falls back to
    single-byte symbols of ASCII (the reference's fallback re-encodes multi-byte symbols' bytes: not a round trip)"""
    tok, ref = request.getfixturevalue(cfg)
    for text in ["Hello world", "the quick brown fox jumps over the lazy dog", "a\nb\tc", "x  y", "12345!!"]:
        ids = tok.encode(text)
        assert tok.decode(ids) == ref.decode(ids) == text.encode()
    for text in _random_texts(50, seed=7):
        ids = tok.encode(text)
        assert tok.decode(ids) == ref.decode(ids)


def _write_vocab_gguf(path, tokens, merges, extra_u32=()):
    """a tensor-less GGUF v3 holding only tokenizer keys"""
    import struct

    def s(x):
        b = x.encode("utf-8", errors="surrogateescape")
        return struct.pack("<Q", len(b)) + b

    kv = [(s("tokenizer.ggml.tokens"), struct.pack("<IIQ", 9, 8, len(tokens)) + b"".join(s(t) for t in tokens)),
          (s("tokenizer.ggml.merges"), struct.pack("<IIQ", 9, 8, len(merges)) + b"".join(s(m) for m in merges))]
    kv += [(s(k), struct.pack("<II", 4, v)) for k, v in extra_u32]
    with open(path, "wb") as f:
        f.write(b"GGUF" + struct.pack("<IQQ", 3, 0, len(kv)) + b"".join(k + v for k, v in kv))


def test_unknown_piece_fallback_and_rank_quirks(tmp_path):
    """text_tokenizer.cpp quirks on a hand-made vocab:
    - a merged piece missing from the vocab falls back to the ids of BYTE_TO_UNICODE[b] for each UTF-8 BYTE of the
      piece's symbol string (:278-285): "é" = symbols "Ã" (C3 83) "©" (C2 A9) merged into the unknown "Ã©" gives
      the symbol ids of bytes C3, 83, C2, A9;
    - a duplicated merge takes the rank of its LAST occurrence (:123), a duplicated token its last id (:106);
    - ids from tokenizer.ggml.{bos,eos,padding}_token_id override the defaults (:130-143); "Ġassistant" is the
      fallback of "assistant" (:151-155)."""
    import q3t
    from text_tokenizer_ref import BYTE_TO_UNICODE
    syms = [BYTE_TO_UNICODE[b] for b in range(256)]
    tokens = syms + ["ab", "bc", "ab", "Ġassistant", "Ċ"]
    merges = ["Ã ©", "b c", "a b", "b c"]   # "b c" ranks 3 (last), so "a b" (2) wins on "abc"
    path = str(tmp_path / "v.gguf")
    _write_vocab_gguf(path, tokens, merges, [("tokenizer.ggml.bos_token_id", 7), ("tokenizer.ggml.eos_token_id", 8)])
    tok, ref = q3t.Tokenizer(path), RefTokenizer(read_gguf_kv(path))
    try:
        got = tok.encode("é")
        assert got == ref.encode("é") == [tokens.index(BYTE_TO_UNICODE[b]) for b in "Ã©".encode()]
        assert tok.encode("abc") == ref.encode("abc") == [258, syms.index("c")]   # "ab" -> its last id 258
        assert (tok.bos, tok.eos, tok.pad) == (7, 8, 151643)
        assert tok.encode_for_tts("") == ref.encode_for_tts("") == [7, 259, 260, 8, 260, 7, 259, 260]
    finally:
        tok.close()


def test_missing_vocab_is_an_error(tmp_path):
    import q3t
    _, tokf = synth_dir("tiny")   # the vocoder GGUF carries no tokenizer.ggml.tokens
    with pytest.raises(q3t.Q3TError, match="tokenizer.ggml.tokens"):
        q3t.Tokenizer(tokf)
