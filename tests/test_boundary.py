"""Drop-in boundary check: the reference's own src/qwen3_tts.cpp and src/main.cpp, read in place and
never copied, compile against qwen3_tts_hip.h and link with libqwen3_tts_hip.so + libq3t.so (tests/boundary/Makefile).
What had to change: nothing in the reference sources; its five component headers (text_tokenizer.h,
tts_transformer.h, audio_tokenizer_encoder.h, audio_tokenizer_decoder.h, trt_vocoder.h) resolve to one-line shims that
include qwen3_tts_hip.h, and gguf_loader.h (ggml) is a stand-in whose "context" is the GGUF path.

CPU: the build itself (needs /root/reference, so it runs in the build container only).
GPU: the resulting reference CLI (_build/qwen3-tts-cli-ref, built here and shipped with the tree) synthesises on the
MI355X runtime and writes the same PCM as this repository's own qwen3-tts-cli, with the whole-utterance vocoder and
with the chunked one (a vocoder_decoder_40.trt file in the model dir, qwen3_tts.cpp:168-198)."""
import os
import subprocess

import numpy as np
import pytest

from q3t_testutil import REPO, synth_dir

BOUNDARY = os.path.join(REPO, "tests", "boundary")
REF_CLI = os.path.join(BOUNDARY, "_build", "qwen3-tts-cli-ref")
OUR_CLI = os.path.join(REPO, "qwen3-tts-jetson_amd", "cpp", "qwen3-tts-cli")
REF_SRC = "/root/reference/src"


@pytest.mark.skipif(not os.path.isdir(REF_SRC), reason="reference sources absent (GPU box)")
def test_reference_pipeline_compiles_against_drop_in():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "qwen3-tts-jetson_amd", "cpp")], check=True)
    r = subprocess.run(["make", "-B", "-C", BOUNDARY, f"REF={REF_SRC}"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert os.path.exists(REF_CLI)
    # -h exits before any model or GPU work (main.cpp:179-181)
    h = subprocess.run([REF_CLI, "-h"], capture_output=True, text=True, timeout=60)
    assert h.returncode == 0 and "Server mode:" in h.stderr


def _model_dir(tmp_path, chunked):
    tts, tok = synth_dir("full")
    d = tmp_path / ("chunk" if chunked else "full")
    d.mkdir()
    os.symlink(tts, d / "qwen3-tts-0.6b-f16.gguf")
    os.symlink(tok, d / "qwen3-tts-tokenizer-f16.gguf")
    if chunked:
        (d / "vocoder_decoder_40.trt").write_bytes(b"not a TensorRT plan")
    return str(d)


@pytest.mark.gpu
@pytest.mark.parametrize("chunked", [False, True])
def test_reference_cli_on_mi355x_runtime(tmp_path, chunked):
    if not os.path.exists(REF_CLI):
        pytest.skip("tests/boundary/_build/qwen3-tts-cli-ref not built (make -C tests/boundary)")
    d = _model_dir(tmp_path, chunked)
    outs = []
    for cli, name in ((REF_CLI, "ref.wav"), (OUR_CLI, "ours.wav")):
        out = str(tmp_path / name)
        r = subprocess.run([cli, "-m", d, "-t", "Hello. This is a test.", "-o", out, "--max-tokens", "48",
                            "--temperature", "0.9"], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, (cli, r.stderr[-3000:])
        if cli == REF_CLI:
            assert ("TRT vocoder ready: 40 fixed frames" in r.stderr) == chunked, r.stderr[-2000:]
            assert "Throughput:" in r.stderr
        with open(out, "rb") as f:
            outs.append(f.read())
    assert len(outs[0]) > 44 and outs[0] == outs[1]
    pcm = np.frombuffer(outs[0][44:], np.int16)
    assert np.abs(pcm).max() > 0
