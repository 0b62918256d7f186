"""The persistent single-slot talker step (persist.hip) against the launch-per-phase graph it replaces.

Both paths compute every phase with the same lane-to-element mapping and summation order (persist.hip header), so
for a split chunk of 64 positions (n_ctx <= 2048) hidden states, logits and every selected code are compared
BIT-EXACT: any stale or torn in-launch hand-off shows up as a mismatch.  Positions run past 64 so the split
flash-decode combine (last-arriving split) is exercised, and generate() is compared at temperature 0 and 0.9.
Long contexts use a wider chunk (different summation order): compared against the oracle tolerance instead.
"""
import os
import sys

import numpy as np
import pytest

from q3t_testutil import REPO, prompt, rel_err, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))

pytestmark = pytest.mark.gpu


def _engine(tts, tok, persist, roles=True, **kw):
    """persist=False: the launch-per-op graphs, with the code predictor's attention as its own k_attn launch
    (Q3T_CP_FUSED_ATTN=0), whose arithmetic the persistent frame reproduces bit for bit; roles=False: the all-role
    persistent kernels (k_persist<0,CH>, k_persist<1,16>), the production fallback where the role kernels are not
    resident"""
    import q3t
    env = {"Q3T_PERSIST": "1" if persist else "0", "Q3T_CP_FUSED_ATTN": "1" if persist else "0",
           "Q3T_TK_ROLES": "1" if roles else "0", "Q3T_CP_ROLES": "1" if roles else "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return q3t.Engine(tts, tok, device=0, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def engines():
    tts, tok = synth_dir("full")
    ep = _engine(tts, tok, True, max_slots=1, max_ctx=320)
    eg = _engine(tts, tok, False, max_slots=1, max_ctx=320)
    assert ep.persist_status() == 0, "persistent talker step not in use on this device"
    assert ep.persist_kernels() == 1 | 4, ep.persist_kernels()   # k_tk_roles + k_cp_roles
    assert eg.persist_status() == -1
    yield ep, eg
    ep.close()
    eg.close()


def test_talker_step_bit_exact(engines):
    ep, eg = engines
    H = ep.cfg["hidden"]
    rng = np.random.default_rng(11)
    bad = []
    for pos in range(0, 200):
        e = (rng.standard_normal(H) * 0.5).astype(np.float32)
        hp, lp = ep.talker_forward(e[None], [pos])
        hg, lg = eg.talker_forward(e[None], [pos])
        if not (np.array_equal(hp, hg) and np.array_equal(lp, lg)):
            bad.append((pos, float(np.abs(hp - hg).max()), float(np.abs(lp - lg).max())))
    assert not bad, (len(bad), bad[:8])
    assert ep.persist_status() == 0


def test_talker_step_bit_exact_role_kernel_long_context():
    """the role-specialised step (persist_tk.hip) at max_ctx 2048: up to 32 attention chunks, so the O workgroups'
    combine runs several poll sweeps (8 chunks each) -- positions on both sides of every sweep boundary, bit-exact
    against the launch-per-op graph (unwritten cache positions are zero in both contexts)"""
    tts, tok = synth_dir("full")
    ep = _engine(tts, None, True, max_slots=1, max_ctx=2048)
    eg = _engine(tts, None, False, max_slots=1, max_ctx=2048)
    try:
        assert ep.persist_kernels() & 1, ep.persist_kernels()   # k_tk_roles
        H = ep.cfg["hidden"]
        rng = np.random.default_rng(23)
        bad = []
        for pos in (0, 1, 63, 64, 65, 300, 511, 512, 513, 575, 1023, 1024, 1500, 1535, 1536, 2000, 2046, 2047):
            e = (rng.standard_normal(H) * 0.5).astype(np.float32)
            hp, lp = ep.talker_forward(e[None], [pos])
            hg, lg = eg.talker_forward(e[None], [pos])
            if not (np.array_equal(hp, hg) and np.array_equal(lp, lg)):
                bad.append((pos, float(np.abs(hp - hg).max()), float(np.abs(lp - lg).max())))
        assert not bad, (len(bad), bad[:8])
        assert ep.persist_status() == 0
    finally:
        ep.close()
        eg.close()


@pytest.mark.parametrize("temperature", [0.0, 0.9])
def test_cp_frame_bit_exact(engines, temperature):
    """the 16-pass code-predictor frame as one persistent launch vs 16 x (5 layers + head + selection) launches"""
    ep, eg = engines
    H = ep.cfg["hidden"]
    rng = np.random.default_rng(21)
    for frame in range(12):
        hid = (rng.standard_normal(H) * 1.5).astype(np.float32)
        cb0 = int(rng.integers(0, 2048))
        cp = ep.codepred_frame(hid[None], [cb0], temperature=temperature, top_k=50, seed=3, frame=frame)
        cg = eg.codepred_frame(hid[None], [cb0], temperature=temperature, top_k=50, seed=3, frame=frame)
        assert np.array_equal(cp, cg), (frame, cp, cg)
    assert ep.persist_status() == 0


def test_all_role_kernels_bit_exact():
    """the all-role persistent kernels (Q3T_TK_ROLES=0, Q3T_CP_ROLES=0: k_persist<0,64>, k_persist<1,16>) against the
    launch-per-op graph: talker step positions across the split combine, code-predictor frames greedy and sampled"""
    tts, tok = synth_dir("full")
    ea = _engine(tts, tok, True, roles=False, max_slots=1, max_ctx=320)
    eg = _engine(tts, tok, False, max_slots=1, max_ctx=320)   # fresh caches on both sides
    try:
        assert ea.persist_status() == 0 and ea.persist_kernels() == 2 | 8, ea.persist_kernels()
        H = ea.cfg["hidden"]
        rng = np.random.default_rng(31)
        for pos in range(0, 140):
            e = (rng.standard_normal(H) * 0.5).astype(np.float32)
            ha, la = ea.talker_forward(e[None], [pos])
            hg, lg = eg.talker_forward(e[None], [pos])
            assert np.array_equal(ha, hg) and np.array_equal(la, lg), pos
        for frame, temperature in ((0, 0.0), (1, 0.9), (2, 0.9)):
            hid = (rng.standard_normal(H) * 1.5).astype(np.float32)
            cb0 = int(rng.integers(0, 2048))
            ca = ea.codepred_frame(hid[None], [cb0], temperature=temperature, top_k=50, seed=3, frame=frame)
            cg = eg.codepred_frame(hid[None], [cb0], temperature=temperature, top_k=50, seed=3, frame=frame)
            assert np.array_equal(ca, cg), (frame, ca, cg)
        assert ea.persist_status() == 0
    finally:
        ea.close()
        eg.close()


@pytest.mark.parametrize("temperature", [0.0, 0.9])
def test_generate_bit_exact(engines, temperature):
    ep, eg = engines
    toks = prompt("full")
    H = ep.cfg["hidden"]
    spk = np.zeros(H, np.float32)
    kw = dict(speakers=[spk], max_len=96, temperature=temperature, top_k=50, seed=5, force_frames=96)
    cp = ep.generate([toks], **kw)[0]
    cg = eg.generate([toks], **kw)[0]
    assert cp.shape == cg.shape == (96, 16)
    assert np.array_equal(cp, cg), int(np.argmax(np.any(cp != cg, axis=1)))
    assert ep.persist_status() == 0


def test_repeated_replays_stay_consistent(engines):
    """the same step replayed many times (stale granules of the previous replay carry identical payloads, so only the
    tags can tell them apart) must keep producing the same result; the bench replays it this way"""
    ep, _ = engines
    H = ep.cfg["hidden"]
    e = (np.random.default_rng(5).standard_normal(H) * 0.5).astype(np.float32)
    ref = ep.talker_forward(e[None], [150])
    for _ in range(20):
        ep.time_stage(0, 1, 150, 5)
        h, lg = ep.talker_forward(e[None], [150])
        assert np.array_equal(h, ref[0]) and np.array_equal(lg, ref[1])
    assert ep.persist_status() == 0


def test_long_context_chunk(engines):
    """n_ctx 4114 (configs[4]'s 4096-frame streaming): split chunk 192, against the launch-per-phase path"""
    tts, tok = synth_dir("full")
    ep = _engine(tts, tok, True, max_slots=1, max_ctx=4114)
    eg = _engine(tts, tok, False, max_slots=1, max_ctx=4114)
    try:
        assert ep.persist_status() == 0
        H = ep.cfg["hidden"]
        rng = np.random.default_rng(2)
        # fill positions 0..599 identically, then compare steps across split counts 1..4 of the 192 chunk
        for pos in range(0, 600):
            e = (rng.standard_normal(H) * 0.5).astype(np.float32)
            hp, lp = ep.talker_forward(e[None], [pos])
            hg, lg = eg.talker_forward(e[None], [pos])
            if pos % 50 == 0 or pos in (191, 192, 193, 383, 384, 599):
                assert rel_err(hp[0], hg[0]) < 1e-2, pos
                assert rel_err(lp[0], lg[0]) < 1e-2, pos
        assert ep.persist_status() == 0
    finally:
        ep.close()
        eg.close()


def test_injected_fault_falls_back_bit_exact():
    """A hand-off fault (injected: the 40th persistent launch flags it, mid-stream) must never reach the caller: no
    chunk is delivered from a faulted launch, the context drops to the bit-identical launch-per-op graphs and re-runs,
    every frame is delivered exactly once, and later calls keep working (VERDICT r01 weak #8 / ADVICE persist.hip)."""
    import q3t
    tts, tok = synth_dir("full")
    ref = _engine(tts, None, False, max_slots=1, max_ctx=160)
    old = os.environ.get("Q3T_PERSIST_FAULT_AT")
    os.environ["Q3T_PERSIST_FAULT_AT"] = "40"
    try:
        flt = _engine(tts, None, True, max_slots=1, max_ctx=160)
    finally:
        if old is None:
            del os.environ["Q3T_PERSIST_FAULT_AT"]
        else:
            os.environ["Q3T_PERSIST_FAULT_AT"] = old
    try:
        assert flt.persist_status() == 0
        toks = prompt("full")
        spk = np.zeros(flt.cfg["hidden"], np.float32)
        kw = dict(speakers=[spk], max_len=60, temperature=0.9, top_k=50, seed=8, force_frames=60)
        want = ref.generate([toks], **kw)[0]
        got_chunks = []
        codes = flt.generate_stream([toks], lambda u, c: got_chunks.append(c) or True, interval=10, **kw)[0]
        assert flt.persist_status() == 2, "the injected fault did not trigger the fallback"
        assert np.array_equal(codes, want)
        streamed = np.concatenate(got_chunks)
        assert streamed.shape == want.shape and np.array_equal(streamed, want)
        # the context keeps working on the per-op graphs
        assert np.array_equal(flt.generate([toks], **kw)[0], want)
        h1, l1 = flt.talker_forward(np.ones((1, flt.cfg["hidden"]), np.float32), [5])
        h2, l2 = ref.talker_forward(np.ones((1, ref.cfg["hidden"]), np.float32), [5])
        assert np.isfinite(h1).all() and np.isfinite(l1).all()
    finally:
        flt.close()
        ref.close()


def test_two_contexts_on_one_device_serialise():
    """two persistent contexts on the same device, driven from two host threads at once: the per-device lock keeps
    their persistent grids from overlapping, so both stay fault-free and produce identical codes"""
    import threading
    import q3t
    tts, tok = synth_dir("full")
    a = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=96)
    b = q3t.Engine(tts, None, device=0, max_slots=1, max_ctx=96)
    try:
        assert a.persist_status() == 0 and b.persist_status() == 0
        toks = prompt("full")
        spk = np.zeros(a.cfg["hidden"], np.float32)
        kw = dict(speakers=[spk], max_len=48, temperature=0.9, top_k=50, seed=3, force_frames=48)
        res = {}

        def run(name, eng):
            res[name] = [eng.generate([toks], **kw)[0] for _ in range(3)]

        ts = [threading.Thread(target=run, args=(n, e)) for n, e in (("a", a), ("b", b))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert a.persist_status() == 0 and b.persist_status() == 0
        for x in res["a"] + res["b"]:
            assert np.array_equal(x, res["a"][0])
    finally:
        a.close()
        b.close()
