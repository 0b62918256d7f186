"""Shared test helpers: synthetic GGUF generation (tools/q3t_synth.c) and prompts."""
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SYNTH_SRC = os.path.join(REPO, "tools", "q3t_synth.c")
SYNTH_EXE = os.path.join(REPO, "tools", "_build", "q3t_synth")
SEED = 0x51E3775

# 8 fixed content ids wrapped in the TTS chat template (src/text_tokenizer.cpp:293-330)
PROMPT_FULL = [151644, 77091, 198, 9707, 11, 1879, 13, 1096, 374, 264, 1273, 151645, 198, 151644, 77091, 198]
PROMPT_TINY = [1003, 50, 10, 900, 901, 902, 903, 904, 905, 906, 907, 20, 10, 1003, 50, 10]


def build_synth():
    if not os.path.exists(SYNTH_EXE) or os.path.getmtime(SYNTH_EXE) < os.path.getmtime(SYNTH_SRC):
        os.makedirs(os.path.dirname(SYNTH_EXE), exist_ok=True)
        subprocess.run(["gcc", "-O2", "-fopenmp", "-o", SYNTH_EXE, SYNTH_SRC, "-lm"], check=True)
    return SYNTH_EXE


def synth_dir(cfg, seed=SEED):
    """Writes (once) the synthetic GGUF pair for cfg in a temp dir; returns (tts_path, tok_path)."""
    root = os.environ.get("Q3T_SYNTH_CACHE", "/tmp")
    d = os.path.join(root, f"q3t_synth_{cfg}_{seed:x}")
    tts = os.path.join(d, "qwen3-tts-0.6b-f16.gguf")
    tok = os.path.join(d, "qwen3-tts-tokenizer-f16.gguf")
    stamp = os.path.join(d, ".done")
    if not os.path.exists(stamp) or os.path.getmtime(stamp) < os.path.getmtime(SYNTH_SRC):
        os.makedirs(d, exist_ok=True)
        subprocess.run([build_synth(), cfg, d, str(seed)], check=True)
        open(stamp, "w").close()
    return tts, tok


def prompt(cfg):
    return list(PROMPT_FULL if cfg == "full" else PROMPT_TINY)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))
