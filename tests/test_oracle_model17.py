"""CPU: the oracle's 1.7B restatement (code predictor geometry + code_pred.mtp_proj; src/tts_transformer.cpp:370-389,
:600-616, :1554-1560, :1709-1714) on the tiny17 synthetic model, checked against an independent numpy restatement of
one code-predictor pass at position 0 (where attention over the single cached row returns that row's f16 V, so the
pass is a plain chain of projections).  Parity unpinned: the reference holds no 1.7B fixture."""
import numpy as np
import pytest

from gguf_py import GGUF
from oracle_py import Oracle
from q3t_testutil import prompt, synth_dir


@pytest.fixture(scope="module")
def m17():
    tts, tok = synth_dir("tiny17")
    o = Oracle(tts, tok)
    yield GGUF(tts), o
    o.close()


def test_config_and_tensor_shapes(m17):
    g, o = m17
    c = o.cfg
    assert (c["hidden"], c["cp_hidden"], c["cp_inter"], c["cp_heads"], c["cp_kv"], c["has_mtp"]) == (512, 256, 512, 4, 2, 1)
    assert g.tensor("code_pred.mtp_proj.weight").shape == (256, 512)      # [cp hidden][talker hidden]
    assert g.tensor("code_pred.lm_head.0.weight").shape == (2048, 256)    # lm_head in code-predictor space
    assert g.tensor("code_pred.codec_embd.0.weight").shape == (2048, 512)  # embeddings stay in talker space


def _f16(x):
    return np.asarray(x, np.float32).astype(np.float16).astype(np.float32)


def _rms(x, w, eps):
    return (x / np.sqrt(np.mean(x.astype(np.float64) ** 2) + eps).astype(np.float32)) * w


def _mm(g, name, x):   # ggml mul_mat: f16 weights, f16-rounded input, f32 accumulation
    return g.tensor(name).astype(np.float32) @ _f16(x)


def test_cp_pass0_matches_numpy_restatement(m17):
    g, o = m17
    c = o.cfg
    rng = np.random.default_rng(2)
    xin = (rng.standard_normal(c["hidden"]) * 1.5).astype(np.float32)
    # numpy: mtp_proj + bias, then the code-predictor layers at position 0 (attention = the row's f16 V per head)
    x = _mm(g, "code_pred.mtp_proj.weight", xin) + g.tensor("code_pred.mtp_proj.bias")
    D, nh, nkv = c["cp_head_dim"], c["cp_heads"], c["cp_kv"]
    for il in range(c["cp_layers"]):
        t = lambda n: f"code_pred.blk.{il}.{n}"
        xn = _rms(x, g.tensor(t("attn_norm.weight")), c["eps"])
        v = _f16(_mm(g, t("attn_v.weight"), xn)).reshape(nkv, D)
        att = np.concatenate([v[h // (nh // nkv)] for h in range(nh)])
        x = x + _mm(g, t("attn_output.weight"), att)
        xn = _rms(x, g.tensor(t("ffn_norm.weight")), c["eps"])
        a, b = _mm(g, t("ffn_gate.weight"), xn), _mm(g, t("ffn_up.weight"), xn)
        x = x + _mm(g, t("ffn_down.weight"), (a / (1.0 + np.exp(-a))) * b)
    ref = _rms(x, g.tensor("code_pred.output_norm.weight"), c["eps"])
    kv = o.kv_new(16, 1)
    hid, _ = o.cp_pass(kv, xin, 0, -1)
    o.kv_free(kv)
    assert hid.shape == ref.shape == (c["cp_hidden"],)
    assert np.abs(hid - ref).max() / np.abs(ref).max() < 2e-3


def test_generate_runs(m17):
    _, o = m17
    codes = o.generate(prompt("tiny17"), max_len=6, force_frames=6)
    assert codes.shape == (6, 16)
    assert codes[:, 1:].max() < o.cfg["cp_vocab"]
