"""The public surface of SURVEY §8(f)#2: Qwen3TTS + qwen3-tts-cli (src/qwen3_tts.{h,cpp}, src/main.cpp).

CPU: the host-only driver tests/cpp/test_pipeline_cpu.cpp (WAV reader/writer, resampling, TextTokenizer mirror,
error convention) and the CLI's argument handling (main.cpp:165-235).
GPU: the CLI end to end on the synthetic 0.6B model dir -- single shot (PCM identical to the ctypes path: tokenizer ->
generate with a ZERO speaker row (qwen3_tts.cpp:241-245) -> FULL vocoder -> PCM16 truncation), the chunked vocoder
selected by a vocoder_decoder_40.trt file in the model dir (qwen3_tts.cpp:168-198) and streamed from the frame
callback, voice cloning with the <ref>.embd cache (main.cpp:37-91, 246-255), and --serve (sequential and --batch)."""
import os
import subprocess
import sys
import wave

import numpy as np
import pytest

from q3t_testutil import REPO, synth_dir

sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
CPP = os.path.join(REPO, "qwen3-tts-jetson_amd", "cpp")
CLI = os.path.join(CPP, "qwen3-tts-cli")
DRIVER = os.path.join(REPO, "tests", "cpp", "_build", "test_pipeline_cpu")


def _build():
    if not (os.path.exists(CLI) and os.path.exists(DRIVER)):
        subprocess.run(["make", "-s", "-C", CPP], check=True)


def test_pipeline_host_driver(tmp_path):
    _build()
    tts, _ = synth_dir("full")
    r = subprocess.run([DRIVER, tts, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "all checks passed" in r.stdout


@pytest.mark.parametrize("args,rc,msg", [
    ([], 1, "Error: model directory is required"),
    (["-m", "/nonexistent"], 1, "Error: text is required (or use --serve)"),
    (["-m"], 1, "Error: missing model directory"),
    (["--bogus"], 1, "Error: unknown argument: --bogus"),
    (["-h"], 0, "Usage:"),
    (["-m", "/nonexistent", "-t", "hi"], 1, "Error: Failed to load text tokenizer"),
    (["--top-k", "x"], 1, "Error: invalid numeric argument"),
])
def test_cli_arguments(args, rc, msg):
    _build()
    r = subprocess.run([CLI] + args, capture_output=True, text=True, timeout=120)
    assert r.returncode == rc, r.stderr
    assert msg in r.stderr


# ---------------------------------------------------------------------------------------------------- GPU
def _model_dir(tmp_path, chunked=False):
    tts, tok = synth_dir("full")
    d = tmp_path / ("models_chunk" if chunked else "models")
    d.mkdir()
    os.symlink(tts, d / "qwen3-tts-0.6b-f16.gguf")
    os.symlink(tok, d / "qwen3-tts-tokenizer-f16.gguf")
    if chunked:
        (d / "vocoder_decoder_40.trt").write_bytes(b"")   # presence selects the 40-frame chunked vocoder
    return str(d)


def _run(args, **kw):
    r = subprocess.run([CLI] + args, capture_output=True, text=True, timeout=600, **kw)
    assert r.returncode == 0, r.stderr[-3000:]
    return r


def _read_wav(path):
    with wave.open(path, "rb") as w:
        assert w.getnchannels() == 1 and w.getsampwidth() == 2 and w.getframerate() == 24000
        return np.frombuffer(w.readframes(w.getnframes()), np.int16)


def _pcm16(x):
    return (np.clip(x, -1, 1) * np.float32(32767.0)).astype(np.float32).astype(np.int16)


@pytest.fixture(scope="module")
def engine():
    import q3t
    tts, tok = synth_dir("full")
    e = q3t.Engine(tts, tok, device=0, max_slots=1, max_ctx=128)
    t = q3t.Tokenizer(tts)
    yield e, t
    e.close()
    t.close()


FR = 24   # frames per test utterance (--max-tokens)


@pytest.mark.gpu
def test_cli_single_shot_matches_engine(tmp_path, engine):
    _build()
    eng, tok = engine
    d = _model_dir(tmp_path)
    out = str(tmp_path / "hello.wav")
    r = _run(["-m", d, "-t", "Hello. This is a test.", "-o", out, "--max-tokens", str(FR), "--temperature", "0.9",
              "--seed", "5"])
    for line in ("Text tokenizer loaded: vocab_size=151936", "Throughput:", "RTF=", "Audio duration:",
                 "Output saved to: " + out):
        assert line in r.stderr, line
    got = _read_wav(out)
    ids = tok.encode_for_tts("Hello. This is a test.")
    codes = eng.generate([ids], speakers=[np.zeros(1024, np.float32)], max_len=FR, temperature=0.9, seed=5)[0]
    want = _pcm16(eng.vocoder(codes))
    assert got.shape == want.shape and len(got) == eng.vocoder_num_samples(codes.shape[0])
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_cli_chunked_vocoder_and_voice_clone(tmp_path, engine):
    _build()
    eng, tok = engine
    d = _model_dir(tmp_path, chunked=True)
    # reference audio: 2 s stereo PCM16 at 16 kHz (resampled to 24 kHz, qwen3_tts.cpp:260-266)
    t = np.arange(32000) / 16000.0
    sig = 0.3 * np.sin(2 * np.pi * 180 * t) * (0.6 + 0.4 * np.sin(2 * np.pi * 3 * t))
    ref = str(tmp_path / "ref.wav")
    with wave.open(ref, "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(np.repeat((sig * 32767).astype(np.int16), 2).tobytes())
    out = str(tmp_path / "clone.wav")
    r = _run(["-m", d, "-t", "Hello.", "-r", ref, "-o", out, "--max-tokens", str(FR), "--temperature", "0"])
    assert "Chunked vocoder ready: 40 fixed frames" in r.stderr
    assert "Saved speaker embedding to: " + ref + ".embd (1024 floats)" in r.stderr
    emb = np.fromfile(ref + ".embd", np.float32)
    assert emb.shape == (1024,) and np.isfinite(emb).all()
    # the embedding the CLI cached is the engine's encoder on the same (resampled PCM16) samples
    x16 = (sig * 32767).astype(np.int16) / 32768.0
    ratio = 16000 / 24000
    n = int(len(x16) / ratio)
    src = np.arange(n) * ratio
    i0 = src.astype(np.int64)
    x24 = np.where(i0 + 1 >= len(x16), x16[-1], (1 - (src - i0)) * x16[i0] + (src - i0) * x16[np.minimum(i0 + 1, len(x16) - 1)])
    e2 = eng.encode_speaker(x24.astype(np.float32))
    assert np.abs(emb - e2).max() <= 1e-3 * np.abs(e2).max()
    codes = eng.generate([tok.encode_for_tts("Hello.")], speakers=[emb], max_len=FR, temperature=0.0)[0]
    want = _pcm16(eng.vocoder_chunked(codes, 40))
    assert np.array_equal(_read_wav(out), want)
    # second run: the cache is read back instead of re-encoding (main.cpp:68-73)
    r2 = _run(["-m", d, "-t", "Hello.", "-r", ref, "-o", out, "--max-tokens", "4", "--temperature", "0"])
    assert "Loaded cached speaker embedding: " + ref + ".embd (1024 floats)" in r2.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 3])
def test_cli_serve(tmp_path, batch):
    _build()
    d = _model_dir(tmp_path)
    reqs = [("Hello.", str(tmp_path / "a.wav")), ("This is a test.", str(tmp_path / "b.wav")),
            ("hello world", str(tmp_path / "c.wav"))]
    stdin = "".join(f"{t}\t{o}\n" for t, o in reqs) + "\nquit\n"
    r = subprocess.run([CLI, "-m", d, "--serve", "--batch", str(batch), "--max-tokens", str(FR), "--temperature", "0"],
                       input=stdin, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().split("\n")
    assert len(lines) == 3, r.stdout
    for (t, o), line in zip(reqs, lines):
        f = line.split("\t")
        assert f[0] == "OK" and f[3] == o, line
        pcm = _read_wav(o)
        assert abs(float(f[1]) - len(pcm) / 24000) < 0.01
    assert "Server shutting down." in r.stderr
