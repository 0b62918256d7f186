"""GPU: contexts sharing one device from several host threads (ADVICE r02 capi.cpp / engine.cpp).

Every entry point that puts work on a device holds the per-device lock of devlock.h: single-slot decode runs (the only
ones that launch the 256-workgroup persistent kernels) exclusively, everything else shared.  So

  - a vocoder or speaker-encoder call on another context never runs beside a persistent grid: the single-slot run
    stays on its persistent kernels (no hand-off timeout, persist_status() 0) and both produce what they produce alone;
  - creating (growing) a context while another context decodes on the same device changes neither: buffers are
    zeroed on the new context's own stream (no device-wide synchronisation inside an allocation any more);
  - a hand-off fault inside a single-slot continuous-batching queue falls back to the bit-identical launch-per-op
    graphs and re-runs the queue, like generate() does.
"""
import os
import sys
import threading

import numpy as np
import pytest

from q3t_testutil import REPO, prompt, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
pytestmark = pytest.mark.gpu


def _env_engine(env, *a, **kw):
    import q3t
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return q3t.Engine(*a, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _prompts(n):
    base = prompt("full")
    return [base[:4] + [(t + 7 * i) % 1000 + 10 for t in base[4:]] for i in range(n)]


def test_single_slot_beside_vocoder_thread():
    import q3t
    tts, tok = synth_dir("full")
    a = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=96)
    v = q3t.Engine(None, tok, device=0, max_slots=1, max_ctx=64)
    try:
        assert a.persist_status() == 0
        H = a.cfg["hidden"]
        kw = dict(speakers=[np.zeros(H, np.float32)], max_len=48, temperature=0.9, top_k=50, seed=13, force_frames=48)
        p = _prompts(1)
        want = a.generate(p, **kw)[0]
        rng = np.random.default_rng(3)
        batch = [rng.integers(0, 2048, size=(n, 16), dtype=np.int32) for n in (40, 64, 17)]
        want_pcm = v.vocoder_batch(batch, q3t.VOCODER_FULL)
        got, pcm = [], []
        stop = threading.Event()

        def voc_loop():
            while not stop.is_set():
                pcm.append(v.vocoder_batch(batch, q3t.VOCODER_FULL))

        t = threading.Thread(target=voc_loop)
        t.start()
        try:
            for _ in range(4):
                got.append(a.generate(p, **kw)[0])
        finally:
            stop.set()
            t.join()
        assert a.persist_status() == 0, "a persistent grid ran beside vocoder work and timed out"
        for g in got:
            assert np.array_equal(g, want)
        assert len(pcm) >= 1
        for out in pcm:
            for x, y in zip(out, want_pcm):
                assert np.array_equal(x, y)
    finally:
        v.close()
        a.close()


def test_context_growth_beside_decoding():
    """Qwen3TTS::ensure_slots (cpp/qwen3_tts_pipeline.cpp) grows capacity by creating a larger replica context; here
    replicas are created while another context decodes a batch on the same device, then decode themselves"""
    import q3t
    tts, tok = synth_dir("full")
    a = q3t.Engine(tts, None, device=0, max_slots=8, max_ctx=64)
    try:
        H = a.cfg["hidden"]
        spk8 = [np.zeros(H, np.float32)] * 8
        kw = dict(max_len=24, temperature=0.9, top_k=50, seed=21, force_frames=24)
        pa = _prompts(8)
        ref_a = a.generate(pa, speakers=spk8, **kw)
        out_a = []
        stop = threading.Event()

        def decode_loop():
            while not stop.is_set():
                out_a.append(a.generate(pa, speakers=spk8, **kw))

        t = threading.Thread(target=decode_loop)
        t.start()
        reps = []
        try:
            for slots in (4, 12, 16):
                reps.append(a.replica(0, slots, 64))
            got = [r.generate(pa[:4], speakers=spk8[:4], **kw) for r in reps]
        finally:
            stop.set()
            t.join()
            for r in reps:
                r.close()
        assert len(out_a) >= 1
        for o in out_a:
            for x, y in zip(o, ref_a):
                assert np.array_equal(x, y)
        for g in got:   # the 4-slot replica runs the 4-slot kernels; 12 / 16 slots the same arithmetic per token
            for x, y in zip(g, got[0]):
                assert np.array_equal(x, y)
        # the 4-utterance batch of every replica equals the 4-slot batch on a fresh context of the same shape
        fresh = q3t.Engine(tts, None, device=0, max_slots=4, max_ctx=64)
        try:
            for x, y in zip(fresh.generate(pa[:4], speakers=spk8[:4], **kw), got[0]):
                assert np.array_equal(x, y)
        finally:
            fresh.close()
    finally:
        a.close()


def test_queue_single_slot_fault_recovers():
    """ADVICE r02 engine.cpp:1527: a hand-off fault in a 1-slot queue (injected on the 21st persistent launch) is
    recovered like generate(): per-op graphs, queue re-run, the codes of a launch-per-op context"""
    tts, tok = synth_dir("full")
    env_ref = {"Q3T_PERSIST": "0", "Q3T_CP_FUSED_ATTN": "0"}
    ref = _env_engine(env_ref, tts, None, device=0, max_slots=1, max_ctx=72)
    flt = _env_engine({"Q3T_PERSIST_FAULT_AT": "21"}, tts, None, device=0, max_slots=1, max_ctx=72)
    try:
        assert flt.persist_status() == 0
        H = flt.cfg["hidden"]
        p = _prompts(3)
        kw = dict(speakers=[np.zeros(H, np.float32)] * 3, max_len=30, temperature=0.9, top_k=50, seed=17)
        want = ref.generate_queue(p, **kw)
        got = flt.generate_queue(p, **kw)
        assert flt.persist_status() == 2, "the injected fault did not trigger the fallback"
        for x, y in zip(got, want):
            assert np.array_equal(x, y)
        for x, y in zip(flt.generate_queue(p, **kw), want):   # and keeps working
            assert np.array_equal(x, y)
    finally:
        flt.close()
        ref.close()


def _hbm_used():
    """device 0's used HBM in bytes (hipMemGetInfo through the HIP runtime libq3t.so links)"""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    free, total = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
    return total.value - free.value


def test_hbm_per_context_and_replica():
    """per-context HBM: the bench's single-slot context (weights, KV, state, the code predictor's 520 MB per-token QKV
    table) and a replica of it on the same device, which copies the weights but shares the table (one copy per device
    and weight file, engine.cpp CpTables); the table is freed with the last context that uses it"""
    import q3t
    tts, tok = synth_dir("full")
    u0 = _hbm_used()
    a = q3t.Engine(tts, tok, device=0, max_slots=1, max_ctx=544)
    u1 = _hbm_used()
    r = a.replica(0, 1, 544)
    u2 = _hbm_used()
    try:
        assert a.persist_kernels() & 4 and r.persist_kernels() & 4
        ctx_mb, rep_mb = (u1 - u0) / 2**20, (u2 - u1) / 2**20
        print(f"HBM per context: {ctx_mb:.0f} MiB (first, table included), replica {rep_mb:.0f} MiB (table shared)")
        assert rep_mb < ctx_mb - 400, (ctx_mb, rep_mb)
        H = a.cfg["hidden"]
        hid = (np.random.default_rng(3).standard_normal((1, H)) * 1.5).astype(np.float32)
        ca = a.codepred_frame(hid, [77], temperature=0.9, top_k=50, seed=5, frame=3)
        cr = r.codepred_frame(hid, [77], temperature=0.9, top_k=50, seed=5, frame=3)
        assert np.array_equal(ca, cr)
    finally:
        r.close()
        a.close()
    u3 = _hbm_used()
    print(f"after both closed: {(u3 - u0) / 2**20:.0f} MiB above the start")
    assert u3 - u0 < 64 * 2**20
