"""Quantised / F32 weight files: every dtype the reference converters can emit loads and decodes.

The converters' --outtype policy (convert_tts_to_gguf.py:250-335, convert_tokenizer_to_gguf.py:265-296) is mirrored
by tools/q3t_synth.c; the ggml block decoders the loaders restate (dequantize_row_q8_0 / q4_0 / q4_K of ggml-quants.c,
the ggml submodule the reference pins but does not vendor) are pinned here by an independent numpy decode of the raw
blocks.  Product loader and oracle both dequantise at open and round to F16 (gguf.h header), so GPU-vs-oracle parity
on a quantised file is as tight as on the F16 file.  The reference's ggml CPU matmul on Q8_0/Q4_K weights quantises
the activations too (vec_dot_type): that numeric path is not restated (parity unpinned against it)."""
import os
import struct
import sys

import numpy as np
import pytest

from oracle_py import Oracle
from q3t_testutil import REPO, check_decisions, prompt, rel_err, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))

VARIANTS = ["q8_0", "q4_k", "q4_0", "f32"]
GGML = {"F32": 0, "F16": 1, "Q4_0": 2, "Q8_0": 8, "Q4_K": 12}


def read_tensors(path):
    """{name: (ne, type, raw bytes view)} of a GGUF v3 file"""
    with open(path, "rb") as f:
        buf = f.read()
    p = 4

    def u(fmt):
        nonlocal p
        v = struct.unpack_from(fmt, buf, p)
        p += struct.calcsize(fmt)
        return v[0]

    def s():
        nonlocal p
        n = u("<Q")
        v = buf[p:p + n]
        p += n
        return v.decode("utf-8", errors="surrogateescape")

    def skip(t):
        if t == 8:
            s()
        elif t == 9:
            et, n = u("<I"), u("<Q")
            for _ in range(n):
                skip(et)
        else:
            u({0: "<B", 1: "<b", 2: "<H", 3: "<h", 4: "<I", 5: "<i", 6: "<f", 7: "<?", 10: "<Q", 11: "<q", 12: "<d"}[t])

    u("<I")
    nt, nkv = u("<Q"), u("<Q")
    for _ in range(nkv):
        s()
        skip(u("<I"))
    infos = []
    for _ in range(nt):
        name = s()
        nd = u("<I")
        ne = [u("<Q") for _ in range(nd)]
        infos.append((name, ne, u("<I"), u("<Q")))
    base = (p + 31) // 32 * 32
    return {n: (ne, t, memoryview(buf)[base + off:]) for n, ne, t, off in infos}


def dequant(t, raw, n):
    """numpy restatement of ggml's block decoders (float32 arithmetic in ggml's order)"""
    if t == GGML["F32"]:
        return np.frombuffer(raw, np.float32, n).copy()
    if t == GGML["F16"]:
        return np.frombuffer(raw, np.float16, n).astype(np.float32)
    if t == GGML["Q8_0"]:
        b = np.frombuffer(raw, np.uint8, n // 32 * 34).reshape(-1, 34)
        d = b[:, :2].copy().view(np.float16).astype(np.float32)
        return (d * b[:, 2:].view(np.int8).astype(np.float32)).ravel()
    if t == GGML["Q4_0"]:
        b = np.frombuffer(raw, np.uint8, n // 32 * 18).reshape(-1, 18)
        d = b[:, :2].copy().view(np.float16).astype(np.float32)
        q = b[:, 2:]
        lo = ((q & 15).astype(np.int32) - 8).astype(np.float32) * d
        hi = ((q >> 4).astype(np.int32) - 8).astype(np.float32) * d
        return np.concatenate([lo, hi], axis=1).ravel()
    if t == GGML["Q4_K"]:
        b = np.frombuffer(raw, np.uint8, n // 256 * 144).reshape(-1, 144)
        d = b[:, 0:2].copy().view(np.float16).astype(np.float32)[:, 0]
        dmin = b[:, 2:4].copy().view(np.float16).astype(np.float32)[:, 0]
        sc, qs = b[:, 4:16].astype(np.int32), b[:, 16:]
        out = np.zeros((b.shape[0], 256), np.float32)
        for j in range(8):
            if j < 4:
                s_, m_ = sc[:, j] & 63, sc[:, j + 4] & 63
            else:
                s_ = (sc[:, j + 4] & 15) | ((sc[:, j - 4] >> 6) << 4)
                m_ = (sc[:, j + 4] >> 4) | ((sc[:, j] >> 6) << 4)
            q = qs[:, (j // 2) * 32:(j // 2) * 32 + 32]
            q = (q & 15) if j % 2 == 0 else (q >> 4)
            d1 = (d * s_.astype(np.float32))[:, None]
            m1 = (dmin * m_.astype(np.float32))[:, None]
            out[:, j * 32:(j + 1) * 32] = d1 * q.astype(np.float32) - m1
        return out.ravel()
    raise ValueError(t)


@pytest.fixture(scope="module", params=VARIANTS)
def variant(request):
    tts, tok = synth_dir("tiny", variant=request.param)
    o = Oracle(tts, tok)
    yield request.param, tts, tok, o
    o.close()


def test_dtype_policy_and_dequant(variant):
    v, tts, tok, o = variant
    tt, tk = read_tensors(tts), read_tensors(tok)
    want = {"q8_0": GGML["Q8_0"], "q4_k": GGML["Q4_K"], "q4_0": GGML["Q4_0"], "f32": GGML["F32"]}[v]
    checks = [("talker.blk.0.attn_q.weight", tt, want), ("code_pred.blk.0.ffn_down.weight", tt, want),
              ("talker.codec_embd.weight", tt, GGML["F32"] if v == "f32" else GGML["F16"]),   # _embd kept
              ("talker.codec_head.weight", tt, GGML["F32"] if v == "f32" else GGML["F16"]),
              ("talker.blk.0.attn_norm.weight", tt, GGML["F32"])]                              # 1-D: F32
    tok_mat = next(n for n, (ne, t, _) in tk.items() if len(ne) == 2 and ne[0] % 32 == 0 and "codebook" not in n)
    checks.append((tok_mat, tk, {"q8_0": GGML["Q8_0"], "f32": GGML["F32"]}.get(v, GGML["F16"])))
    for name, tab, t_want in checks:
        ne, t, raw = tab[name]
        n = int(np.prod(ne))
        assert t == t_want, (name, t, t_want)
        ref = dequant(t, raw, n)
        if len(ne) >= 2:
            ref = ref.astype(np.float16).astype(np.float32)   # matrices are held as F16 after loading
        got, src = o.tensor(name, n)
        assert src == t
        assert np.array_equal(got, ref), name
    if v != "f32":   # quantisation error of the synthetic weights stays at the format's resolution
        ne, t, raw = tt["talker.blk.0.attn_q.weight"]
        f16 = read_tensors(synth_dir("tiny")[0])["talker.blk.0.attn_q.weight"]
        x = dequant(f16[1], f16[2], int(np.prod(ne)))
        err = np.abs(dequant(t, raw, x.size) - x).max() / np.abs(x).max()
        assert err < {"q8_0": 0.01, "q4_k": 0.1, "q4_0": 0.15}[v], err


@pytest.mark.gpu
def test_gpu_generate_and_vocoder_on_quantised_file(variant):
    import q3t
    v, tts, tok, o = variant
    eng = q3t.Engine(tts, tok, device=0, max_slots=1, max_ctx=64)
    try:
        toks = prompt("tiny")
        spk = np.zeros(eng.cfg["hidden"], np.float32)
        codes = eng.generate([toks], speakers=[spk], max_len=12, temperature=0.0, force_frames=12)[0]
        assert codes.shape == (12, 16)
        check_decisions(o, toks, spk, codes, max_len=12, force_frames=12, temperature=0.0)
        pcm = eng.vocoder(codes)
        ref = o.vocoder(codes)
        assert pcm.shape == ref.shape
        assert rel_err(pcm, ref) < 1e-2, rel_err(pcm, ref)
    finally:
        eng.close()
