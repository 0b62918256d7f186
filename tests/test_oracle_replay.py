"""The oracle's partial teacher-forced replay (q3o_generate_forced_from), used by the long-form parity tests to check
the decisions of late frames without re-running the code predictor for every earlier frame: its traces must equal the
full replay's for the traced frames (CPU only)."""
import numpy as np

from oracle_py import Oracle
from q3t_testutil import prompt, synth_dir


def test_partial_replay_equals_full_replay():
    tts, tok = synth_dir("tiny")
    orc = Oracle(tts, tok)
    try:
        toks = prompt("tiny")
        spk = (np.random.default_rng(8).standard_normal(orc.cfg["hidden"]) * 0.02).astype(np.float32)
        codes = orc.generate(toks, spk=spk, max_len=14, temperature=0.9, top_k=50, seed=3, force_frames=14)
        assert codes.shape == (14, 16)
        cb_full, cp_full = orc.generate_forced(toks, codes, spk=spk, force_frames=14)
        cb_part, cp_part = orc.generate_forced(toks, codes, spk=spk, force_frames=14, from_frame=9)
        assert cb_part.shape[0] == cp_part.shape[0] == 5
        np.testing.assert_array_equal(cb_part, cb_full[9:])
        np.testing.assert_array_equal(cp_part, cp_full[9:])
    finally:
        orc.close()
