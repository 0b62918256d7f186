#!/usr/bin/env python3
"""Generate golden vectors from the REFERENCE's own PyTorch harness (run in the build container only).

The reference's Python caller of the code-predictor path is the ONNX/TRT export harness
`scripts/export_code_predictor.py` (class CodePredLayersExport, :45-231): a fixed 16-slot-KV one-token
Qwen3 decoder step (RMSNorm, q/k head-norm, NEOX RoPE, GQA, SwiGLU, output RMSNorm).  It is imported here
from /root/reference (never copied) and driven exactly like the TRT loop in src/trt_code_predictor.cpp:484-600:
  pass 0: talker hidden at position 0, no lm_head
  pass 1: codec_embd[cb0] at position 1 -> lm_head[0] -> argmax
  pass s: code_pred.codec_embd[s-2][code_{s-1}] at position s -> lm_head[s-1] -> argmax   (s = 2..15)
The same class with the talker's layers and output norm pins the talker decode step at positions < 16
(the talker block is the same Qwen3 block, src/tts_transformer.cpp:1410-1512).

Weights come from tools/q3t_synth (portable counter-based hash, exact in f16), so the fixtures only hold
inputs and outputs; the GPU box regenerates identical weights from the seed.

usage: python tests/golden/make_golden.py            (writes tests/golden/*.npz)
"""
import importlib.util
import os
import subprocess
import sys

import numpy as np

sys.dont_write_bytecode = True          # never write into /root/reference
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
from gguf_py import GGUF  # noqa: E402

REF_SCRIPT = "/root/reference/scripts/export_code_predictor.py"
SEED = 0x51E3775


def load_ref_class():
    spec = importlib.util.spec_from_file_location("ref_export_code_predictor", REF_SCRIPT)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.CodePredLayersExport


def synth(cfg, out_dir):
    from q3t_testutil import build_synth
    exe = build_synth()
    os.makedirs(out_dir, exist_ok=True)
    subprocess.run([exe, cfg, out_dir, str(SEED)], check=True)
    return os.path.join(out_dir, "qwen3-tts-0.6b-f16.gguf")


def state_dict(g, prefix, n_layers, norm_name):
    import torch
    sd = {}
    m = {"attn_norm": "input_layernorm", "ffn_norm": "post_attention_layernorm", "attn_q": "self_attn.q_proj",
         "attn_k": "self_attn.k_proj", "attn_v": "self_attn.v_proj", "attn_output": "self_attn.o_proj",
         "attn_q_norm": "self_attn.q_norm", "attn_k_norm": "self_attn.k_norm", "ffn_gate": "mlp.gate_proj",
         "ffn_up": "mlp.up_proj", "ffn_down": "mlp.down_proj"}
    for i in range(n_layers):
        for gk, hk in m.items():
            sd[f"layers.{i}.{hk}.weight"] = torch.from_numpy(np.array(g.tensor(f"{prefix}.blk.{i}.{gk}.weight"), np.float32))
    sd["norm.weight"] = torch.from_numpy(np.array(g.tensor(norm_name), np.float32))
    return sd


def run(cfg, out_dir):
    import torch
    Ref = load_ref_class()
    path = synth(cfg, out_dir)
    g = GGUF(path)
    kv = g.kv
    H = kv["qwen3-tts.embedding_length"]
    nH = kv["qwen3-tts.attention.head_count"]
    nKV = kv["qwen3-tts.attention.head_count_kv"]
    D = kv["qwen3-tts.attention.key_length"]
    I = kv["qwen3-tts.feed_forward_length"]
    L = kv["qwen3-tts.block_count"]
    Lcp = kv["qwen3-tts.code_predictor.layer_count"]
    eps = kv["qwen3-tts.attention.layer_norm_rms_epsilon"]
    theta = kv["qwen3-tts.rope.freq_base"]
    rng = np.random.default_rng(7)

    def make(nl, prefix, norm):
        conf = {"num_hidden_layers": nl, "hidden_size": H, "num_attention_heads": nH, "num_key_value_heads": nKV,
                "head_dim": D, "intermediate_size": I, "rms_norm_eps": eps, "rope_theta": theta}
        mdl = Ref(conf, "", state_dict(g, prefix, nl, norm))
        mdl.float().eval()
        return mdl

    def step(mdl, x, pos, past):
        args = [torch.from_numpy(x.reshape(1, 1, H)), torch.tensor([pos], dtype=torch.int64)]
        # the harness signature has exactly 5 (past_key, past_value) pairs; unused layers get zero caches
        for il in range(5):
            k, v = past[il] if il < len(past) else (torch.zeros(1, nKV, 16, D), torch.zeros(1, nKV, 16, D))
            args += [k, v]
        with torch.no_grad():
            out = mdl(*args)
        new = [(out[1 + 2 * i], out[2 + 2 * i]) for i in range(len(past))]
        return out[0].reshape(H).numpy().astype(np.float32), new

    files = {}
    # ---- code predictor: 16 passes with greedy codes
    assert Lcp <= 5, "harness has 5 layer slots"
    cp = make(Lcp, "code_pred", "code_pred.output_norm.weight")
    past = [(torch.zeros(1, nKV, 16, D), torch.zeros(1, nKV, 16, D)) for _ in range(Lcp)]
    hidden = rng.standard_normal(H).astype(np.float32)
    cb0 = 137
    codec_embd = np.array(g.tensor("talker.codec_embd.weight"), np.float32)
    xs, outs, logits, logits_h, codes = [], [], [], [], []
    x = hidden
    for p in range(16):
        if p == 1:
            x = codec_embd[cb0]
        elif p >= 2:
            x = np.array(g.tensor(f"code_pred.codec_embd.{p - 2}.weight")[codes[-1]], np.float32)
        xs.append(x.copy())
        o, past = step(cp, x, p, past)
        outs.append(o)
        if p >= 1:
            W = np.array(g.tensor(f"code_pred.lm_head.{p - 1}.weight"), np.float32)
            lg = W @ o
            logits.append(lg)
            # TRT path: fp32->fp16 of the hidden before the FP16 GemmEx (trt_code_predictor.cpp:343-362)
            logits_h.append(W @ o.astype(np.float16).astype(np.float32))
            codes.append(int(np.argmax(lg)))
    files[f"cp_{cfg}.npz"] = dict(hidden=hidden, cb0=np.int32(cb0), inputs=np.stack(xs), outputs=np.stack(outs),
                                  logits=np.stack(logits), logits_f16in=np.stack(logits_h),
                                  codes=np.array(codes, np.int32),
                                  k_cache_l0=past[0][0].numpy(), v_cache_l0=past[0][1].numpy())
    # ---- talker step at positions 0..15 (harness capacity), arbitrary input embeddings
    # the harness has 5 layer slots: pin the first min(L,5) talker layers + output norm
    Lt = min(L, 5)
    tk = make(Lt, "talker", "talker.output_norm.weight")
    past = [(torch.zeros(1, nKV, 16, D), torch.zeros(1, nKV, 16, D)) for _ in range(Lt)]
    xin = (rng.standard_normal((16, H)) * 0.5).astype(np.float32)
    outs, lgs = [], []
    Wh = np.array(g.tensor("talker.codec_head.weight"), np.float32)
    for p in range(16):
        o, past = step(tk, xin[p], p, past)
        outs.append(o)
        lgs.append(Wh @ o)
    files[f"talker{Lt}_{cfg}.npz"] = dict(inputs=xin, outputs=np.stack(outs), logits=np.stack(lgs),
                                         n_layers=np.int32(Lt))
    for name, d in files.items():
        np.savez_compressed(os.path.join(HERE, name), **d)
        print("wrote", name, {k: v.shape for k, v in d.items()})


if __name__ == "__main__":
    cfgs = sys.argv[1:] or ["tiny", "full"]
    for c in cfgs:
        run(c, f"/tmp/q3t_golden_{c}")
