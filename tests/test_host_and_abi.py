"""CPU tests (no GPU): the C ABI library and its header, the host-side rules of the decode path as restated by the
oracle (known answers derived from the reference's own code), and the synthetic model files.

Reference rules pinned here (paths relative to the reference repo):
  CB0 logit processing   src/tts_transformer.cpp:2416-2499  (vocab mask, repetition penalty, EOS ramp, top-k ties)
  prefill structure      src/tts_transformer.cpp:1093-1231  (prefill_len 10 with speaker, trailing_len n-8, n>=4)
  CHUNK40 vocoder length src/trt_vocoder.h:50, src/trt_vocoder.cpp:150-164 (1920 samples per frame)
"""
import ctypes as C
import hashlib
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from q3t_testutil import REPO, build_synth, prompt, synth_dir

PKG = os.path.join(REPO, "qwen3-tts-jetson_amd")
HEADER = os.path.join(REPO, "include", "q3t_backend.h")
EOS = 2150


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w \*]*?\b(q3t_\w+|gpu_\w+)\s*\(", txt, flags=re.M)
    return sorted(set(names))


# ------------------------------------------------------------------------------------------------ C ABI
def test_header_declares_the_replaced_reference_interfaces():
    names = header_functions()
    # the four extern "C" wrappers of src/trt_cuda_kernels.cu:10,60,78,183 keep their exact names
    for n in ("gpu_fp32_to_fp16", "gpu_argmax_f32", "gpu_embedding_lookup_by_gpu_id", "gpu_sample_topk_f32"):
        assert n in names
    for n in ("q3t_ctx_create", "q3t_generate", "q3t_vocoder_decode", "q3t_talker_forward", "q3t_codepred_frame"):
        assert n in names


def test_library_exports_every_header_symbol():
    sys.path.insert(0, PKG)
    import q3t
    lib = C.CDLL(q3t.LIB_PATH)
    names = header_functions()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"libq3t.so lacks {missing}"
    assert sorted(q3t.EXPORTS) == names, "q3t.EXPORTS out of sync with include/q3t_backend.h"
    # and the exported C symbols are unmangled (extern "C"): nm must show them verbatim
    out = subprocess.run(["nm", "-D", "--defined-only", q3t.LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    assert set(names) <= syms


def test_ctx_create_without_gpu_fails_loudly():
    """No CPU fallback: creating a context needs the HIP device; on a GPU-less host the call returns Q3T_ERR with a
    message (it must not crash and must not silently compute on the CPU)."""
    import hip_py
    if hip_py.device_count() > 0:
        pytest.skip("a GPU is visible")
    sys.path.insert(0, PKG)
    import q3t
    tts, _ = synth_dir("tiny")
    with pytest.raises(q3t.Q3TError) as ei:
        q3t.Engine(tts, None, max_slots=1, max_ctx=64)
    assert str(ei.value)


CPP_LIB = os.path.join(PKG, "cpp", "libqwen3_tts_hip.so")
CPP_TEST = os.path.join(REPO, "tests", "cpp", "_build", "test_host_api")


def test_cpp_mirror_exports_the_reference_runtime_classes():
    """qwen3_tts_hip.h keeps the reference's C++ surface (SURVEY §8(b) layer 2): qwen3_tts::TTSTransformer
    (src/tts_transformer.h:164-245), AudioTokenizerDecoder (src/audio_tokenizer_decoder.h:158-180) and
    TRTVocoderDecoder (src/trt_vocoder.h:18-42), same method names, built over libq3t.so (build() makes it)."""
    assert os.path.exists(CPP_LIB), "libqwen3_tts_hip.so missing: run __graft_entry__.build()"
    out = subprocess.run(["nm", "-D", "-C", "--defined-only", CPP_LIB], capture_output=True, text=True,
                         check=True).stdout
    for m in ("TTSTransformer::load_model(", "TTSTransformer::unload_model(", "TTSTransformer::init_kv_cache(",
              "TTSTransformer::clear_kv_cache(", "TTSTransformer::forward_text(", "TTSTransformer::forward_prefill(",
              "TTSTransformer::forward_step(", "TTSTransformer::get_hidden_states(",
              "TTSTransformer::predict_codes_autoregressive(", "TTSTransformer::generate(",
              "AudioTokenizerDecoder::load_model(", "AudioTokenizerDecoder::decode(",
              "TRTVocoderDecoder::load_engine(", "TRTVocoderDecoder::decode(", "TRTVocoderDecoder::unload("):
        assert "qwen3_tts::" + m in out, m
    # the mirror calls only the C ABI: every libq3t symbol it needs is one the header declares
    und = subprocess.run(["nm", "-D", "--undefined-only", CPP_LIB], capture_output=True, text=True, check=True).stdout
    used = {ln.split()[-1] for ln in und.splitlines() if ln.split() and ln.split()[-1].startswith(("q3t_", "gpu_"))}
    assert used and used <= set(header_functions()), used - set(header_functions())


def test_cpp_mirror_error_paths_without_gpu():
    """The C++ driver's first block (errors before/without load, bool + get_error(), nothing thrown) runs on a
    GPU-less host; load_model then fails loudly instead of falling back to the CPU."""
    import hip_py
    if hip_py.device_count() > 0:
        pytest.skip("a GPU is visible")
    assert os.path.exists(CPP_TEST), "tests/cpp/_build/test_host_api missing: run __graft_entry__.build()"
    import tempfile
    tts, tok = synth_dir("tiny")
    with tempfile.TemporaryDirectory() as d:
        np.asarray(prompt("tiny"), np.int32).tofile(os.path.join(d, "prompt.bin"))
        r = subprocess.run([CPP_TEST, tts, tok, d], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1, (r.returncode, r.stdout, r.stderr)
    assert "FAIL" not in r.stderr, r.stderr
    assert "load_model:" in r.stderr and "device" in r.stderr, r.stderr


def test_default_params_match_reference_tts_params():
    sys.path.insert(0, PKG)
    import q3t
    p = q3t.default_params()
    # tts_params defaults (src/qwen3_tts.h:18-43) and generate()'s language id (src/qwen3_tts.cpp:459-463)
    assert p.max_len == 4096 and p.top_k == 50 and p.language_id == 2050 and p.force_frames == 0
    assert abs(p.temperature - 0.9) < 1e-7 and abs(p.repetition_penalty - 1.05) < 1e-7


# ------------------------------------------------------------------------------------------------ CB0 rules
@pytest.fixture(scope="module")
def orc_tiny():
    from oracle_py import Oracle
    tts, tok = synth_dir("tiny")
    o = Oracle(tts, tok)
    yield o
    o.close()


def _flat(V, val=0.0):
    return np.full(V, val, np.float32)


def test_cb0_masks_codec_control_range_except_eos(orc_tiny):
    V = orc_tiny.cfg["codec_vocab"]
    lg = _flat(V)
    lg[2500] = 50.0    # inside [V-1024, V): masked
    lg[17] = 1.0
    tok, _ = orc_tiny.cb0_select(lg, np.zeros(V, np.uint8), frame=0, n_tokens=16, rep=1.0)
    assert tok == 17
    lg[EOS] = 60.0     # EOS is the one control id that survives the mask
    tok, _ = orc_tiny.cb0_select(lg, np.zeros(V, np.uint8), frame=0, n_tokens=16, rep=1.0)
    assert tok == EOS


def test_cb0_repetition_penalty_divides_positive_multiplies_negative(orc_tiny):
    V = orc_tiny.cfg["codec_vocab"]
    seen = np.zeros(V, np.uint8)
    lg = _flat(V, -5.0)
    lg[10], lg[11] = 10.0, 9.6
    seen[10] = 1
    tok, out = orc_tiny.cb0_select(lg, seen, frame=0, n_tokens=16, rep=1.05)
    assert tok == 11                       # 10 / 1.05 = 9.52 < 9.6
    assert abs(out[10] - 10.0 / 1.05) < 1e-5
    seen[20] = 1
    lg2 = lg.copy()
    lg2[20] = -2.0
    _, out2 = orc_tiny.cb0_select(lg2, seen, frame=0, n_tokens=16, rep=1.05)
    assert abs(out2[20] - (-2.0 * 1.05)) < 1e-5


def test_cb0_eos_ramp(orc_tiny):
    V = orc_tiny.cfg["codec_vocab"]
    n_tokens = 16
    expected = max(20, 4 * n_tokens)       # src/tts_transformer.cpp:2439
    lg = _flat(V)
    lg[5] = 3.0
    lg[EOS] = -4.0
    z = np.zeros(V, np.uint8)
    tok, out = orc_tiny.cb0_select(lg, z, frame=expected - 1, n_tokens=n_tokens, rep=1.0)
    assert tok == 5 and abs(out[EOS] + 4.0) < 1e-6          # ramp not started
    f = expected + expected // 2                            # ramp = 0.5
    tok, out = orc_tiny.cb0_select(lg, z, frame=f, n_tokens=n_tokens, rep=1.0)
    ramp = min(1.0, (f - expected) / expected)
    assert abs(out[EOS] - (-4.0 + ramp * ((3.0 + 5.0) - (-4.0)))) < 1e-5
    tok, out = orc_tiny.cb0_select(lg, z, frame=2 * expected, n_tokens=n_tokens, rep=1.0)
    assert tok == EOS and abs(out[EOS] - 8.0) < 1e-5        # ramp 1: max + 5
    # bench force_frames masks EOS entirely
    tok, _ = orc_tiny.cb0_select(lg, z, frame=2 * expected, n_tokens=n_tokens, rep=1.0, eos_mask=1)
    assert tok == 5


def test_topk_ties_survive_and_eos_is_kept(orc_tiny):
    """top-k threshold with `< thr -> -inf`: every logit equal to the k-th largest survives
    (src/tts_transformer.cpp:2456-2464); the EOS logit is restored after top-k (:2466-2470)."""
    V = orc_tiny.cfg["codec_vocab"]
    lg = _flat(V, -30.0)
    lg[100:110] = 5.0                       # 10-way tie at the top, top_k = 3
    z = np.zeros(V, np.uint8)
    picks = set()
    for u in np.linspace(0.01, 0.99, 25):
        tok, _ = orc_tiny.cb0_select(lg, z, frame=0, n_tokens=16, rep=1.0, temperature=1.0, top_k=3, u=float(u))
        picks.add(tok)
    assert picks <= set(range(100, 110)) and len(picks) > 3
    lg[EOS] = 4.0                           # below the top-3 but restored
    got_eos = any(orc_tiny.cb0_select(lg, z, frame=0, n_tokens=16, rep=1.0, temperature=1.0, top_k=3, u=float(u))[0] == EOS
                  for u in np.linspace(0.9, 0.999, 20))
    assert got_eos


# ------------------------------------------------------------------------------------------------ prefill / vocoder
def test_prefill_structure(orc_tiny):
    toks = prompt("tiny")
    H = orc_tiny.cfg["hidden"]
    pre, tr, pad = orc_tiny.prefill_embd(toks, spk=np.zeros(H, np.float32))
    assert pre.shape[0] == 10 and tr.shape[0] == len(toks) - 8 and pad.shape == (H,)
    pre2, _, _ = orc_tiny.prefill_embd(toks, spk=None)
    assert pre2.shape[0] == 9
    with pytest.raises(RuntimeError):
        orc_tiny.prefill_embd(toks[:3])


def test_chunk40_vocoder_is_1920_samples_per_frame(orc_tiny):
    for F in (1, 39, 40, 41, 97):
        assert orc_tiny.vocoder_len(F, 1) == F * 1920
    # FULL: each convT stage maps L -> (L + 1) * s - K with K trimmed on both sides (audio_tokenizer_decoder.cpp:590-613)
    assert orc_tiny.vocoder_len(10, 0) > 0


# ------------------------------------------------------------------------------------------------ synthetic model files
def test_synth_gguf_is_deterministic_and_0p6b_shaped(tmp_path):
    exe = build_synth()
    from gguf_py import GGUF
    for d in ("a", "b"):
        (tmp_path / d).mkdir()
        subprocess.run([exe, "tiny", str(tmp_path / d), str(0x51E3775)], check=True)
    h = [hashlib.sha256(open(tmp_path / d / "qwen3-tts-0.6b-f16.gguf", "rb").read()).hexdigest() for d in ("a", "b")]
    assert h[0] == h[1]
    tts, _ = synth_dir("full")
    g = GGUF(tts)
    # shapes of SURVEY 8(a) a1, ggml ne order [in, out]
    assert g.tensors["talker.blk.0.attn_q.weight"][0] == [1024, 2048]
    assert g.tensors["talker.blk.27.ffn_down.weight"][0] == [3072, 1024]
    assert g.tensors["code_pred.lm_head.14.weight"][0] == [1024, 2048]
    assert int(g.kv["qwen3-tts.block_count"]) == 28
