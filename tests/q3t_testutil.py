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


def synth_dir(cfg, seed=SEED, variant=""):
    """Writes (once) the synthetic GGUF pair for cfg in a temp dir; returns (tts_path, tok_path).
    variant "usage": the tokenizer file keeps per-codebook usage tensors (see tools/q3t_synth.c)."""
    root = os.environ.get("Q3T_SYNTH_CACHE", "/tmp")
    d = os.path.join(root, f"q3t_synth_{cfg}_{seed:x}" + (f"_{variant}" if variant else ""))
    tts = os.path.join(d, "qwen3-tts-0.6b-f16.gguf")
    tok = os.path.join(d, "qwen3-tts-tokenizer-f16.gguf")
    stamp = os.path.join(d, ".done")
    if not os.path.exists(stamp) or os.path.getmtime(stamp) < os.path.getmtime(SYNTH_SRC):
        os.makedirs(d, exist_ok=True)
        subprocess.run([build_synth(), cfg, d, str(seed)] + ([variant] if variant else []), check=True)
        open(stamp, "w").close()
    return tts, tok


def prompt(cfg):
    return list(PROMPT_FULL if cfg.startswith("full") else PROMPT_TINY)


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def _sample_interval(logits, temperature, top_k, keep_id):
    """CDF interval bookkeeping of the shared sampler (oracle q3o_sample): returns (exps, total)."""
    l = np.asarray(logits, np.float64) / temperature
    keep = l[keep_id] if keep_id >= 0 else None
    if 0 < top_k < len(l):
        thr = np.sort(l)[-top_k]
        l = np.where(l < thr, -np.inf, l)
    if keep_id >= 0:
        l[keep_id] = keep
    e = np.exp(l - l.max())
    return e, e.sum()


def check_token(lg, tok, temperature, top_k, u, keep_id=-1, tol_logit=5e-2, tol_cdf=5e-2):
    """one decision: 0 if tok is exactly what the oracle logits select, 1 if within tolerance (else AssertionError)."""
    if temperature <= 0:
        gap = float(lg.max() - lg[tok])
        assert gap <= tol_logit, gap
        return int(gap > 0)
    e, tot = _sample_interval(lg, temperature, top_k, keep_id)
    cum = np.cumsum(e)
    lo = cum[tok - 1] if tok > 0 else 0.0
    target = u * tot
    if lo <= target <= cum[tok]:
        return 0
    err = max(lo - target, target - cum[tok]) / tot
    assert err <= tol_cdf, err
    return 1


def check_decisions(orc, toks, spk, codes, *, max_len, force_frames=0, temperature=0.0, top_k=50, seed=0, utt=0,
                    rep=1.05, tol_logit=2.5e-2, tol_cdf=2.5e-2, max_off_frac=0.03, eos_id=2150, from_frame=0):
    """Teacher-forced parity of a GPU-generated code sequence against the oracle (per-decision tolerance 2.5e-2: ~2x
    the worst observed in the GPU suite, 0.011 on the 16-slot batched family; it was 5e-2 through round 4).

    The oracle replays the GPU's codes (q3o_generate_forced) and records every decision's logits.  Greedy: each
    GPU token must be the oracle argmax or within tol_logit of it (near-tie); sampling: u*total must fall in the
    token's CDF interval up to tol_cdf.  At most max_off_frac of the decisions may take the tolerance branch.
    If the GPU stopped before max_len, the oracle must also pick EOS (within tolerance) at that frame.
    from_frame > 0: only the decisions of frames >= from_frame are checked (the oracle replays the earlier frames'
    codes through the talker alone)."""
    from oracle_py import uniform
    codes = np.asarray(codes, np.int32).reshape(-1, 16)
    F = codes.shape[0]
    stopped = F < max_len
    forced = np.concatenate([codes, np.zeros((1, 16), np.int32)]) if stopped else codes
    cb0, cp = orc.generate_forced(toks, forced, spk=spk, rep=rep, force_frames=force_frames, from_frame=from_frame)
    n_dec = n_off = 0
    worst = 0.0
    offs = []
    for f in range(from_frame, forced.shape[0]):
        last = stopped and f == F
        for c in range(1 if last else 16):
            lg = cb0[f - from_frame] if c == 0 else cp[f - from_frame, c - 1]
            tok = eos_id if last else int(codes[f, c])
            n_dec += 1
            if temperature <= 0:
                gap = float(lg.max() - lg[tok])
                if gap > 0:
                    n_off += 1
                    worst = max(worst, gap)
                    offs.append((f, c, round(gap, 6)))
            else:
                keep = eos_id if (c == 0 and not (force_frames and f < force_frames)) else -1
                e, tot = _sample_interval(lg, temperature, top_k, keep)
                u = uniform(seed, utt, f, c)
                target = u * tot
                cum = np.cumsum(e)
                lo = cum[tok - 1] if tok > 0 else 0.0
                hi = cum[tok]
                if not (lo <= target <= hi):
                    n_off += 1
                    err = max(lo - target, target - hi) / tot
                    worst = max(worst, err)
                    offs.append((f, c, round(err, 6)))
    tol = tol_logit if temperature <= 0 else tol_cdf
    ok = worst <= tol and n_off <= max(1, int(max_off_frac * n_dec))
    if not ok:   # printed at once (the assertion report only comes at the end of the session)
        print(f"check_decisions FAILED: {n_off}/{n_dec} off (allowed {max(1, int(max_off_frac * n_dec))}), worst {worst:.4g} "
              f"(tol {tol}); off decisions (frame, codebook, gap): {offs[:40]}", flush=True)
    assert worst <= tol, (worst, offs[:20])
    assert n_off <= max(1, int(max_off_frac * n_dec)), (n_off, n_dec, worst, offs)
    return n_off, n_dec, worst


def check_pooled(results, max_off_frac):
    """the near-tie allowance over several check_decisions results (each run with max_off_frac=1.0: its gap / CDF
    tolerance still asserted per decision) pooled: a fraction of 128 decisions of one utterance is a noisy sample."""
    n_off = sum(r[0] for r in results)
    n_dec = sum(r[1] for r in results)
    allowed = max(1, int(max_off_frac * n_dec))
    if n_off > allowed:
        print(f"check_pooled FAILED: {n_off}/{n_dec} off (allowed {allowed})", flush=True)
    assert n_off <= allowed, (n_off, n_dec, allowed)

