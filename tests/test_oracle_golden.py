"""Pins the CPU oracle (oracle/q3t_oracle.c) against golden vectors produced by the reference's own PyTorch
export harness (scripts/export_code_predictor.py:45-231, see tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

from oracle_py import Oracle
from q3t_testutil import rel_err, synth_dir

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CFGS = ["tiny", pytest.param("full", marks=pytest.mark.slow)]


@pytest.mark.parametrize("cfg", CFGS)
def test_cp_passes_fp32_match_reference_harness(cfg):
    g = np.load(os.path.join(GOLD, f"cp_{cfg}.npz"))
    tts, _ = synth_dir(cfg)
    o = Oracle(tts, None, ggml_rounding=False)
    kv = o.kv_new(16, 1)
    for p in range(16):
        hid, lg = o.cp_pass(kv, g["inputs"][p], p, head=p - 1 if p >= 1 else -1)
        assert rel_err(hid, g["outputs"][p]) < 2e-5, p
        if p >= 1:
            assert rel_err(lg, g["logits"][p - 1]) < 2e-5, p
    o.kv_free(kv)
    # greedy 15-code sequence (argmax of lm_head on the fp32 hidden) is reproduced exactly
    codes = o.cp_frame(g["hidden"], int(g["cb0"]), temperature=0.0)
    np.testing.assert_array_equal(codes, g["codes"])


@pytest.mark.parametrize("cfg", CFGS)
def test_talker_layers_fp32_match_reference_harness(cfg):
    g = np.load(os.path.join(GOLD, f"talker5_{cfg}.npz"))
    tts, _ = synth_dir(cfg)
    o = Oracle(tts, None, ggml_rounding=False)
    kv = o.kv_new(16, 0)
    nl = int(g["n_layers"])
    for p in range(16):
        hid, lg = o.talker_step(kv, g["inputs"][p], p, n_layers=nl)
        assert rel_err(hid, g["outputs"][p]) < 2e-5, p
        assert rel_err(lg, g["logits"][p]) < 2e-5, p
    o.kv_free(kv)


@pytest.mark.parametrize("cfg", CFGS)
def test_ggml_rounding_mode_stays_close_to_fp32_reference(cfg):
    """The GGML-CPU semantics (f16 matmul inputs, F16 KV) differ from fp32 only by f16 rounding noise."""
    g = np.load(os.path.join(GOLD, f"cp_{cfg}.npz"))
    tts, _ = synth_dir(cfg)
    o = Oracle(tts, None, ggml_rounding=True)
    kv = o.kv_new(16, 1)
    for p in range(16):
        hid, lg = o.cp_pass(kv, g["inputs"][p], p, head=p - 1 if p >= 1 else -1)
        assert rel_err(hid, g["outputs"][p]) < 5e-3, p
    o.kv_free(kv)
