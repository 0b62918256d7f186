"""configs[4] long-form streaming without the speaker encoder: 4096 frames at context 4114
(tts_transformer.cpp:2383-2388) with a seeded N(0, 0.02) speaker row, generate_stream at interval 40 with every chunk
decoded by the CHUNK40 vocoder inside the callback (qwen3_tts.cpp:437-463, trt_vocoder.cpp:98-170).

Checks: the streamed chunks are exactly the returned codes; the callback's concatenated PCM equals one
vocoder_chunked(all codes, 40) call; the decisions of the first and the last 40-frame chunk are teacher-forced against
the CPU oracle (the last one through the oracle's partial replay: q3o_generate_forced_from)."""
import os
import sys
import time

import numpy as np
import pytest

from oracle_py import Oracle
from q3t_testutil import REPO, check_decisions, prompt, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
pytestmark = pytest.mark.gpu


def test_configs4_4096_frames_chunk40_stream():
    import q3t
    tts, tok = synth_dir("full")
    NF, IV, SEED = 4096, 40, 4242
    eng = q3t.Engine(tts, tok, device=0, max_slots=1, max_ctx=NF + 32)
    orc = Oracle(tts, tok)
    try:
        assert eng.persist_status() == 0
        toks = prompt("full")
        spk = (np.random.default_rng(5).standard_normal(eng.cfg["hidden"]) * 0.02).astype(np.float32)
        chunks, pcm = [], []

        def on_frames(utt, c):
            chunks.append(c)
            pcm.append(eng.vocoder(c, q3t.VOCODER_CHUNK40))
            return True

        t0 = time.time()
        codes = eng.generate_stream([toks], on_frames, interval=IV, speakers=[spk], max_len=NF, temperature=0.9,
                                    top_k=50, seed=SEED, force_frames=NF)[0]
        t_gpu = time.time() - t0
        print(f"4096 frames streamed + CHUNK40 in {t_gpu:.1f} s", flush=True)
        assert codes.shape == (NF, 16)
        assert len(chunks) == NF // IV + (NF % IV > 0)
        assert np.array_equal(np.concatenate(chunks), codes)
        whole = eng.vocoder_chunked(codes, IV)
        assert whole.shape == (NF * 1920,)
        assert np.array_equal(np.concatenate(pcm), whole)
        assert np.isfinite(whole).all() and np.abs(whole).max() <= 1.0
        t0 = time.time()
        first = check_decisions(orc, toks, spk, codes[:IV], max_len=IV, force_frames=NF, temperature=0.9, top_k=50,
                                seed=SEED)
        print(f"first chunk checked ({time.time() - t0:.1f} s); replaying {NF - IV} frames in the oracle", flush=True)
        last = check_decisions(orc, toks, spk, codes, max_len=NF, force_frames=NF, temperature=0.9, top_k=50,
                               seed=SEED, from_frame=NF - IV)
        print(f"4096 frames streamed + CHUNK40 in {t_gpu:.1f} s (GPU); oracle checks {time.time() - t0:.1f} s; "
              f"first chunk {first[1] - first[0]}/{first[1]} exact, last chunk {last[1] - last[0]}/{last[1]} exact")
        assert eng.persist_status() == 0
    finally:
        orc.close()
        eng.close()
