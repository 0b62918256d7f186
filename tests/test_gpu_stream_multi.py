"""GPU: the streaming frame callback (a15) and the multi-GPU weight path (§8(e)) through the C ABI.

Streaming follows TTSTransformer::generate's on_frames contract (src/tts_transformer.cpp:2517-2523, 2563-2570):
  - every `interval` frames the callback receives exactly the newest `interval` frames of the utterance;
  - after the loop, one final flush delivers the remainder (< interval frames);
  - returning false ends the utterance after the frames delivered so far (no flush follows).
The concatenated chunks must equal the codes generate() returns, and equal a run without the callback (the callback
changes nothing on the device).

Weights: q3t_ctx_create_replica lays out the weight blobs from the GGUF headers only and fills them device to device,
which is the receive side of the RCCL broadcast of q3t_ctx_create_shared; a replica must decode bit-identically.
The single-rank shared context exercises RCCL init, the blob-size agreement all-reduce and the broadcast call.
"""
import os
import sys

import numpy as np
import pytest

from q3t_testutil import REPO, prompt, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import q3t
    tts, tok = synth_dir("tiny")
    e = q3t.Engine(tts, tok, device=0, max_slots=3, max_ctx=256)
    yield e
    e.close()


def _prompts(n):
    base = prompt("tiny")
    return [base[:4] + [(t + 7 * i) % 1000 + 10 for t in base[4:]] for i in range(n)]


def test_stream_chunks_equal_generate(eng):
    prompts = _prompts(3)
    H = eng.cfg["hidden"]
    spk = [np.zeros(H, np.float32)] * 3
    kw = dict(max_len=100, temperature=0.9, top_k=50, seed=11, force_frames=100)
    ref = eng.generate(prompts, speakers=spk, **kw)
    got = {u: [] for u in range(3)}
    sizes = {u: [] for u in range(3)}

    def cb(u, codes):
        got[u].append(codes)
        sizes[u].append(len(codes))
        return True

    out = eng.generate_stream(prompts, cb, interval=40, speakers=spk, **kw)
    for u in range(3):
        assert sizes[u] == [40, 40, 20], sizes[u]
        np.testing.assert_array_equal(np.concatenate(got[u]), out[u])
        np.testing.assert_array_equal(out[u], ref[u])


def test_stream_stop_and_eos(eng):
    prompts = _prompts(2)
    H = eng.cfg["hidden"]
    spk = [np.zeros(H, np.float32)] * 2
    calls = {0: 0, 1: 0}

    def cb(u, codes):
        calls[u] += 1
        return u != 0   # utterance 0 stops after its first chunk

    kw = dict(max_len=130, temperature=0.0, top_k=50, seed=3, force_frames=130)
    out = eng.generate_stream(prompts, cb, interval=40, speakers=spk, **kw)
    assert calls[0] == 1 and len(out[0]) == 40
    assert calls[1] == 4 and len(out[1]) == 130   # 3 full chunks + the flush of 10
    ref = eng.generate(prompts, speakers=spk, **kw)
    np.testing.assert_array_equal(out[0], ref[0][:40])
    np.testing.assert_array_equal(out[1], ref[1])
    # EOS allowed (no force): chunk sizes sum to the produced frames; partial chunks only in the flush
    got = []
    out = eng.generate_stream(prompts[:1], lambda u, c: got.append(len(c)) or True, interval=8, speakers=spk[:1],
                              max_len=64, temperature=0.9, top_k=50, seed=5)
    assert sum(got) == len(out[0])
    assert all(n == 8 for n in got[:-1]) and 0 < got[-1] <= 8


def test_replica_decodes_identically(eng):
    rep = eng.replica(device=0, max_slots=1, max_ctx=128)
    try:
        p = _prompts(1)
        kw = dict(max_len=24, temperature=0.9, top_k=50, seed=7, force_frames=24)
        a = eng.generate(p, **kw)[0]
        b = rep.generate(p, **kw)[0]
        np.testing.assert_array_equal(a, b)
        codes = a[:12]
        np.testing.assert_array_equal(eng.vocoder(codes), rep.vocoder(codes))
    finally:
        rep.close()


def test_full_replica_persistent_frame_matches_source():
    """a 1-slot replica of the full model runs the persistent code-predictor frame with the layer-0 QKV table; the table
    is derived from the weights, so it must be built after the device-to-device copy (not from the empty arena at
    layout time): codes identical to the source context's at T = 0.9"""
    import q3t
    tts, _ = synth_dir("full")
    src = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=64)
    rep = src.replica(0, 1, 64)
    try:
        assert src.persist_status() == 0 and rep.persist_status() == 0
        H = src.cfg["hidden"]
        kw = dict(speakers=[np.zeros(H, np.float32)], max_len=12, temperature=0.9, top_k=50, seed=11, force_frames=12)
        toks = prompt("full")
        np.testing.assert_array_equal(rep.generate([toks], **kw)[0], src.generate([toks], **kw)[0])
    finally:
        rep.close()
        src.close()


def test_shared_single_rank_rccl():
    import q3t
    tts, tok = synth_dir("tiny")
    uid = q3t.comm_unique_id()
    assert len(uid) == q3t.COMM_ID_BYTES
    e = q3t.Engine.shared(tts, tok, 0, 1, 128, 0, 1, uid)
    try:
        v = e.allreduce_max([1.5, -2.0, 3.0])
        np.testing.assert_array_equal(v, [1.5, -2.0, 3.0])
        ref = q3t.Engine(tts, tok, device=0, max_slots=1, max_ctx=128)
        p = _prompts(1)
        kw = dict(max_len=16, temperature=0.0, top_k=50, force_frames=16)
        np.testing.assert_array_equal(e.generate(p, **kw)[0], ref.generate(p, **kw)[0])
        ref.close()
    finally:
        e.close()


def test_concurrent_batched_contexts_and_persistent_exclusion():
    """contexts on one device driven from several host threads: batched runs (shared device lock) overlap and decode
    exactly as they do alone; a single-slot run (persistent kernels, exclusive lock) in the middle of them is held
    back until they drain and decodes exactly as alone (no hand-off timeout, no fallback)"""
    import threading
    import q3t
    tts, tok = synth_dir("full")
    a = q3t.Engine(tts, None, device=0, max_slots=8, max_ctx=64)
    b = a.replica(0, 8, 64)
    c = a.replica(0, 1, 64)
    assert c.persist_status() == 0   # the full model's single-slot context runs the persistent kernels
    try:
        H = a.cfg["hidden"]
        kw = dict(max_len=12, temperature=0.9, top_k=50, seed=5, force_frames=12)
        base = prompt("full")
        pa = [base[:4] + [(t + 7 * i) % 1000 + 10 for t in base[4:]] for i in range(8)]
        pb = pa[::-1]
        spk8 = [np.zeros(H, np.float32)] * 8
        ref_a = a.generate(pa, speakers=spk8, **kw)
        ref_b = b.generate(pb, speakers=spk8, **kw)
        ref_c = c.generate(pa[:1], speakers=spk8[:1], **kw)
        out = {}

        def run(name, e, p, n):
            for _ in range(3):
                out[name] = e.generate(p, speakers=spk8[:n], **kw)
        th = [threading.Thread(target=run, args=("a", a, pa, 8)), threading.Thread(target=run, args=("b", b, pb, 8)),
              threading.Thread(target=run, args=("c", c, pa[:1], 1))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for x, y in zip(out["a"], ref_a):
            assert np.array_equal(x, y)
        for x, y in zip(out["b"], ref_b):
            assert np.array_equal(x, y)
        assert np.array_equal(out["c"][0], ref_c[0])
        assert c.persist_status() == 0   # never fell back
    finally:
        c.close()
        b.close()
        a.close()
