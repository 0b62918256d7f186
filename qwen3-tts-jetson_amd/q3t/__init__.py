"""Python host mirror of the MI355X Qwen3-TTS decode path (ctypes over include/q3t_backend.h / libq3t.so).

The compute runs in libq3t.so (hand-written gfx950 HIP kernels).  There is NO CPU fallback: importing this
module fails loudly if the in-tree extension is missing, and every call raises Q3TError with
q3t_last_error() when the C ABI reports failure (the reference's bool + get_error() convention).
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# Q3T_DEV_LIB=1 loads the development build (make -C csrc DEV=1: debug hooks for tools/dev), Q3T_DEV_LIB=<name> an
# experiment build (make -C csrc VARIANT=<name>: libq3t_<name>.so); never the default
_dev = os.environ.get("Q3T_DEV_LIB", "")
LIB_PATH = os.path.join(_HERE, "libq3t.so" if not _dev else "libq3t_dev.so" if _dev == "1" else f"libq3t_{_dev}.so")

VOCODER_FULL = 0
VOCODER_CHUNK40 = 1


class Q3TError(RuntimeError):
    pass


if not os.path.exists(LIB_PATH):
    raise ImportError(f"libq3t.so not built at {LIB_PATH}: run `python -c 'import __graft_entry__ as g; g.build()'` "
                      "(make -C qwen3-tts-jetson_amd/csrc)")

_lib = C.CDLL(LIB_PATH)


class Config(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "hidden", "n_layers", "n_heads", "n_kv_heads", "head_dim", "intermediate", "codec_vocab", "n_codebooks",
        "text_vocab", "text_dim", "cp_layers", "cp_vocab", "codec_eos", "has_vocoder", "sample_rate", "max_slots",
        "max_ctx", "cp_hidden", "cp_intermediate", "cp_heads", "cp_kv_heads", "has_mtp")]


class GenParams(C.Structure):
    _fields_ = [("max_len", C.c_int32), ("language_id", C.c_int32), ("repetition_penalty", C.c_float),
                ("temperature", C.c_float), ("top_k", C.c_int32), ("seed", C.c_uint64), ("force_frames", C.c_int32)]


_P, _I, _F = C.c_void_p, C.c_int, C.c_float
_fp = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_lib.q3t_last_error.restype = C.c_char_p
_lib.q3t_default_params.argtypes = [C.POINTER(GenParams)]
_lib.q3t_ctx_create.argtypes = [C.c_char_p, C.c_char_p, _I, _I, _I, C.POINTER(_P)]
_lib.q3t_ctx_destroy.argtypes = [_P]
_lib.q3t_get_config.argtypes = [_P, C.POINTER(Config)]
_lib.q3t_generate.argtypes = [_P, _I, C.POINTER(C.POINTER(C.c_int32)), _ip, C.POINTER(C.POINTER(C.c_float)),
                              C.POINTER(GenParams), _ip, _ip]
_lib.q3t_generate_queue.argtypes = [_P, _I, C.POINTER(C.POINTER(C.c_int32)), _ip, C.POINTER(C.POINTER(C.c_float)),
                                    C.POINTER(GenParams), _ip, _ip, C.c_int32]
FRAME_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.c_int32, C.c_int32)
_lib.q3t_generate_stream.argtypes = [_P, _I, C.POINTER(C.POINTER(C.c_int32)), _ip, C.POINTER(C.POINTER(C.c_float)),
                                     C.POINTER(GenParams), _ip, _ip, FRAME_CB, C.c_void_p, C.c_int32]
COMM_ID_BYTES = 128
_lib.q3t_comm_unique_id.argtypes = [C.c_char_p]
_lib.q3t_ctx_create_shared.argtypes = [C.c_char_p, C.c_char_p, _I, _I, _I, _I, _I, C.c_char_p, C.POINTER(_P)]
_lib.q3t_ctx_create_replica.argtypes = [_P, _I, _I, _I, C.POINTER(_P)]
_lib.q3t_plan_weight_layout.argtypes = [C.c_char_p, _P, _I, C.POINTER(_I), C.POINTER(C.c_uint64)]
_lib.q3t_comm_allreduce_max.argtypes = [_P, np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS"), _I]
_lib.q3t_set_mfma_min_batch.argtypes = [_I]
_lib.q3t_synchronize.argtypes = [_P]
_lib.q3t_last_timing.argtypes = [_P, C.POINTER(C.c_double), C.POINTER(C.c_double)]
_lib.q3t_time_stage.argtypes = [_P, _I, _I, _I, _I, C.POINTER(C.c_double)]
_lib.q3t_persist_status.argtypes = [_P]
_lib.q3t_persist_kernels.argtypes = [_P]
if hasattr(_lib, "q3t_debug_read"):   # development builds only (make -C csrc DEV=1)
    _lib.q3t_debug_read.argtypes = [_P, _I, _P, C.c_size_t]
_lib.q3t_vocoder_num_samples.restype = C.c_int64
_lib.q3t_vocoder_num_samples.argtypes = [_P, C.c_int32, _I]
_lib.q3t_vocoder_flops.restype = C.c_double
_lib.q3t_vocoder_flops.argtypes = [_P, C.c_int32]
_lib.q3t_vocoder_decode.argtypes = [_P, _ip, C.c_int32, _I, _fp, C.POINTER(C.c_int64)]
_lib.q3t_vocoder_decode_chunked.argtypes = [_P, _ip, C.c_int32, C.c_int32, C.c_int32, _fp, C.POINTER(C.c_int64)]
_lib.q3t_vocoder_decode_batch.argtypes = [_P, C.c_int32, C.POINTER(C.c_void_p), _ip, _I, C.c_int32,
                                          C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]
_lib.q3t_vocoder_set_batch_frames.argtypes = [_P, C.c_int32]
_lib.q3t_speaker_dim.argtypes = [_P]
_lib.q3t_ctx_create_speaker.argtypes = [C.c_char_p, _I, C.POINTER(_P)]
_lib.q3t_speaker_encode.argtypes = [_P, _fp, C.c_int32, _fp]
_lib.q3t_speaker_mel.argtypes = [_P, _fp, C.c_int32, _P, C.c_int32, C.POINTER(C.c_int32)]
_lib.q3t_tokenizer_load.argtypes = [C.c_char_p, C.POINTER(_P)]
_lib.q3t_tokenizer_free.argtypes = [_P]
_lib.q3t_tokenizer_info.argtypes = [_P] + [C.POINTER(C.c_int32)] * 4
_lib.q3t_tokenizer_encode.argtypes = [_P, C.c_char_p, C.c_int64, _I, _P, C.c_int32, C.POINTER(C.c_int32)]
_lib.q3t_tokenizer_decode.argtypes = [_P, _P, C.c_int32, _P, C.c_int64, C.POINTER(C.c_int64)]
_lib.q3t_talker_forward.argtypes = [_P, _I, _fp, _ip, _P, _P]
_lib.q3t_talker_prefill.argtypes = [_P, _I, _I, _fp, _I, _P, _P]
_lib.q3t_codepred_frame.argtypes = [_P, _I, _fp, _ip, _F, C.c_int32, C.c_uint64, C.c_int32, _ip, _P]
_lib.q3t_cb0_select.argtypes = [_P, _I, _fp, np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS"), _ip, _ip,
                                C.POINTER(GenParams), _ip]
_lib.q3t_project_text.argtypes = [_P, _I, _ip, _fp]
_lib.q3t_prefill_embd.argtypes = [_P, _ip, _I, _P, _I, _fp, C.POINTER(C.c_int32), _fp, C.POINTER(C.c_int32), _fp]

# names the C ABI must export (checked by tests without a GPU)
EXPORTS = ["q3t_last_error", "q3t_default_params", "q3t_ctx_create", "q3t_ctx_destroy", "q3t_get_config",
           "q3t_generate", "q3t_generate_stream", "q3t_generate_queue", "q3t_comm_unique_id", "q3t_ctx_create_shared",
           "q3t_plan_weight_layout", "q3t_ctx_create_replica", "q3t_comm_allreduce_max", "q3t_set_mfma_min_batch", "q3t_synchronize", "q3t_last_timing", "q3t_time_stage", "q3t_persist_status", "q3t_persist_kernels", "q3t_vocoder_num_samples", "q3t_vocoder_flops", "q3t_vocoder_decode",
           "q3t_vocoder_decode_chunked", "q3t_vocoder_decode_batch", "q3t_vocoder_set_batch_frames", "q3t_speaker_dim", "q3t_ctx_create_speaker", "q3t_speaker_encode", "q3t_speaker_mel",
           "q3t_tokenizer_load", "q3t_tokenizer_free", "q3t_tokenizer_info", "q3t_tokenizer_encode",
           "q3t_tokenizer_decode", "q3t_talker_forward", "q3t_talker_prefill",
           "q3t_codepred_frame", "q3t_cb0_select", "q3t_project_text", "q3t_prefill_embd", "gpu_fp32_to_fp16",
           "gpu_argmax_f32", "gpu_embedding_lookup_by_gpu_id", "gpu_sample_topk_f32"]


def lib():
    return _lib


def _check(rc):
    if rc != 0:
        raise Q3TError(_lib.q3t_last_error().decode(errors="replace"))


def default_params(**kw):
    p = GenParams()
    _lib.q3t_default_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _addr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def set_mfma_min_batch(b):
    """Process-wide: batches of >= b slots use the matrix-core GEMM (0 = never).  Affects contexts created later."""
    _check(_lib.q3t_set_mfma_min_batch(int(b)))


def comm_unique_id():
    """RCCL unique id (rank 0), Q3T_COMM_ID_BYTES bytes to hand to every rank of q3t_ctx_create_shared."""
    buf = C.create_string_buffer(COMM_ID_BYTES)
    _check(_lib.q3t_comm_unique_id(buf))
    return buf.raw


def plan_weight_layout(tts_gguf):
    """Host-only weight layout of a model file (no device): (byte offset of every allocation of the talker blob in
    order, bytes used) -- what each rank of a shared start-up computes from the GGUF headers before the broadcast."""
    n = C.c_int(0)
    used = C.c_uint64(0)
    _check(_lib.q3t_plan_weight_layout(str(tts_gguf).encode(), None, 0, C.byref(n), C.byref(used)))
    off = np.zeros(max(n.value, 1), np.uint64)
    _check(_lib.q3t_plan_weight_layout(str(tts_gguf).encode(), _addr(off), n.value, C.byref(n), C.byref(used)))
    return off[:n.value], int(used.value)


class Tokenizer:
    """TextTokenizer (src/text_tokenizer.h): byte-level BPE + the TTS template, read from the TTS GGUF.  Host only."""

    def __init__(self, gguf_path):
        h = _P()
        _check(_lib.q3t_tokenizer_load(gguf_path.encode(), C.byref(h)))
        self.h = h
        v, b, e, p = (C.c_int32() for _ in range(4))
        _check(_lib.q3t_tokenizer_info(self.h, C.byref(v), C.byref(b), C.byref(e), C.byref(p)))
        self.vocab_size, self.bos, self.eos, self.pad = v.value, b.value, e.value, p.value

    def close(self):
        if getattr(self, "h", None):
            _lib.q3t_tokenizer_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode(self, text, for_tts=False):
        raw = text.encode("utf-8", errors="surrogateescape") if isinstance(text, str) else bytes(text)
        n = C.c_int32(0)
        _check(_lib.q3t_tokenizer_encode(self.h, raw, len(raw), int(bool(for_tts)), None, 0, C.byref(n)))
        out = np.zeros(max(n.value, 1), np.int32)
        _check(_lib.q3t_tokenizer_encode(self.h, raw, len(raw), int(bool(for_tts)), _addr(out), n.value, C.byref(n)))
        return out[:n.value].tolist()

    def encode_for_tts(self, text):
        return self.encode(text, for_tts=True)

    def decode(self, ids):
        """bytes of the decoded text"""
        a = np.ascontiguousarray(ids, np.int32)
        nb = C.c_int64(0)
        _check(_lib.q3t_tokenizer_decode(self.h, _addr(a), len(a), None, 0, C.byref(nb)))
        buf = C.create_string_buffer(max(nb.value, 1))
        _check(_lib.q3t_tokenizer_decode(self.h, _addr(a), len(a), buf, nb.value, C.byref(nb)))
        return buf.raw[:nb.value]


class Engine:
    """One device context (TTSTransformer + code predictor + vocoder resident in HBM)."""

    def __init__(self, tts_gguf=None, tokenizer_gguf=None, device=0, max_slots=1, max_ctx=4096 + 32, *, _handle=None):
        if _handle is None:
            h = _P()
            _check(_lib.q3t_ctx_create(tts_gguf.encode() if tts_gguf else None,
                                       tokenizer_gguf.encode() if tokenizer_gguf else None,
                                       int(device), int(max_slots), int(max_ctx), C.byref(h)))
            _handle = h
        self.h = _handle
        c = Config()
        _check(_lib.q3t_get_config(self.h, C.byref(c)))
        self.cfg = {n: getattr(c, n) for n, _ in Config._fields_}

    @classmethod
    def shared(cls, tts_gguf, tokenizer_gguf, device, max_slots, max_ctx, rank, world, uid):
        """One rank of a multi-GPU job: rank 0 reads the weights, RCCL broadcasts them to the others."""
        assert len(uid) == COMM_ID_BYTES
        h = _P()
        _check(_lib.q3t_ctx_create_shared(tts_gguf.encode(), tokenizer_gguf.encode() if tokenizer_gguf else None,
                                          int(device), int(max_slots), int(max_ctx), int(rank), int(world), uid,
                                          C.byref(h)))
        return cls(_handle=h)

    @classmethod
    def speaker_only(cls, tts_gguf, device=0):
        """a context with only the speaker encoder loaded (AudioTokenizerEncoder::load_model)"""
        h = _P()
        _check(_lib.q3t_ctx_create_speaker(tts_gguf.encode(), int(device), C.byref(h)))
        return cls(_handle=h)

    def replica(self, device=0, max_slots=1, max_ctx=4096 + 32):
        """A second context whose weights are copied device-to-device from this one (no file reads)."""
        h = _P()
        _check(_lib.q3t_ctx_create_replica(self.h, int(device), int(max_slots), int(max_ctx), C.byref(h)))
        return Engine(_handle=h)

    def allreduce_max(self, values):
        v = np.ascontiguousarray(values, np.float64).copy()
        _check(_lib.q3t_comm_allreduce_max(self.h, v, len(v)))
        return v

    def close(self):
        if getattr(self, "h", None):
            _lib.q3t_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- hot path
    def generate(self, prompts, speakers=None, **params):
        """prompts: list of token-id lists.  Returns list of [n_frames][16] int32 arrays."""
        p = default_params(**params)
        n = len(prompts)
        toks = [np.ascontiguousarray(t, np.int32) for t in prompts]
        tarr = (C.POINTER(C.c_int32) * n)(*[t.ctypes.data_as(C.POINTER(C.c_int32)) for t in toks])
        ntok = np.array([len(t) for t in toks], np.int32)
        sarr = None
        keep = []
        if speakers is not None:
            sp = [np.ascontiguousarray(s, np.float32) for s in speakers]
            keep = sp
            sarr = (C.POINTER(C.c_float) * n)(*[s.ctypes.data_as(C.POINTER(C.c_float)) for s in sp])
        codes = np.zeros((n, p.max_len, 16), np.int32)
        nf = np.zeros(n, np.int32)
        _check(_lib.q3t_generate(self.h, n, tarr, ntok, sarr, C.byref(p), codes, nf))
        del keep
        return [codes[i, :nf[i]].copy() for i in range(n)]

    def generate_queue(self, prompts, speakers=None, max_active=0, **params):
        """continuous batching (q3t_generate_queue): any number of prompts through the context's slots, a finished
        utterance's slot refilled with the next prompt.  Returns list of [n_frames][16] int32 arrays."""
        p = default_params(**params)
        n = len(prompts)
        toks = [np.ascontiguousarray(t, np.int32) for t in prompts]
        tarr = (C.POINTER(C.c_int32) * n)(*[t.ctypes.data_as(C.POINTER(C.c_int32)) for t in toks])
        ntok = np.array([len(t) for t in toks], np.int32)
        sarr = None
        keep = []
        if speakers is not None:
            sp = [np.ascontiguousarray(s, np.float32) for s in speakers]
            keep = sp
            sarr = (C.POINTER(C.c_float) * n)(*[s.ctypes.data_as(C.POINTER(C.c_float)) for s in sp])
        codes = np.zeros((n, p.max_len, 16), np.int32)
        nf = np.zeros(n, np.int32)
        _check(_lib.q3t_generate_queue(self.h, n, tarr, ntok, sarr, C.byref(p), codes, nf, int(max_active)))
        del keep
        return [codes[i, :nf[i]].copy() for i in range(n)]

    def generate_stream(self, prompts, on_frames, interval=40, speakers=None, **params):
        """generate() with the reference's frame callback: on_frames(utt, codes [n][16]) -> bool, every `interval`
        frames plus a final flush; returning False stops that utterance.  Returns the codes like generate()."""
        p = default_params(**params)
        n = len(prompts)
        toks = [np.ascontiguousarray(t, np.int32) for t in prompts]
        tarr = (C.POINTER(C.c_int32) * n)(*[t.ctypes.data_as(C.POINTER(C.c_int32)) for t in toks])
        ntok = np.array([len(t) for t in toks], np.int32)
        sarr = None
        sp = []
        if speakers is not None:
            sp = [np.ascontiguousarray(s, np.float32) for s in speakers]
            sarr = (C.POINTER(C.c_float) * n)(*[s.ctypes.data_as(C.POINTER(C.c_float)) for s in sp])
        codes = np.zeros((n, p.max_len, 16), np.int32)
        nf = np.zeros(n, np.int32)
        errors = []

        def _cb(_user, utt, ptr, nfr, ncb):
            try:
                arr = np.ctypeslib.as_array(ptr, shape=(nfr * ncb,)).reshape(nfr, ncb).copy()
                return 1 if on_frames(int(utt), arr) is not False else 0
            except Exception as e:  # never let an exception unwind through the C frames
                errors.append(e)
                return 0

        cb = FRAME_CB(_cb)
        _check(_lib.q3t_generate_stream(self.h, n, tarr, ntok, sarr, C.byref(p), codes, nf, cb, None, int(interval)))
        del sp
        if errors:
            raise errors[0]
        return [codes[i, :nf[i]].copy() for i in range(n)]

    def synchronize(self):
        _check(_lib.q3t_synchronize(self.h))

    def last_timing(self):
        a, b = C.c_double(0), C.c_double(0)
        _check(_lib.q3t_last_timing(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def time_stage(self, stage, n_slots, pos, iters):
        ms = C.c_double(0)
        _check(_lib.q3t_time_stage(self.h, int(stage), int(n_slots), int(pos), int(iters), C.byref(ms)))
        return ms.value

    def persist_status(self):
        """-1: single-slot path runs launch-per-phase; 0: persistent launches in use; 1: one flagged a hand-off
        fault; 2: persistent launches disabled after a fault (bit-identical launch-per-op graphs in use)."""
        return _lib.q3t_persist_status(self.h)

    def persist_kernels(self):
        """bit mask of the single-slot persistent kernels in use: 1 talker roles (persist_tk.hip), 2 talker all-role
        (persist.hip), 4 code-predictor roles (persist_cp.hip), 8 code-predictor all-role (persist.hip)"""
        return _lib.q3t_persist_kernels(self.h)

    def debug_read(self, which, nbytes):
        """development builds only: raw bytes of a device state buffer (0 K, 1 V cache, 2 QKV, 3 attention, 5 timeline)"""
        buf = np.zeros(nbytes, np.uint8)
        _check(_lib.q3t_debug_read(self.h, int(which), _addr(buf), int(nbytes)))
        return buf

    # ---- vocoder
    def vocoder_num_samples(self, n_frames, mode=VOCODER_FULL):
        return _lib.q3t_vocoder_num_samples(self.h, int(n_frames), int(mode))

    def vocoder_flops(self, n_frames):
        """algorithmic FLOPs of one FULL decode of n_frames"""
        return _lib.q3t_vocoder_flops(self.h, int(n_frames))

    def vocoder(self, codes, mode=VOCODER_FULL):
        codes = np.ascontiguousarray(codes, np.int32).reshape(-1, 16)
        n = self.vocoder_num_samples(codes.shape[0], mode)
        if n < 0:
            raise Q3TError("vocoder not loaded")
        pcm = np.zeros(max(n, 1), np.float32)
        ns = C.c_int64(0)
        _check(_lib.q3t_vocoder_decode(self.h, codes, codes.shape[0], int(mode), pcm, C.byref(ns)))
        return pcm[:ns.value]

    def vocoder_chunked(self, codes, chunk_frames):
        """TRTVocoderDecoder::decode with the engine's fixed_frames (src/trt_vocoder.cpp:98-170)."""
        codes = np.ascontiguousarray(codes, np.int32).reshape(-1, 16)
        pcm = np.zeros(max(codes.shape[0] * 1920, 1), np.float32)
        ns = C.c_int64(0)
        _check(_lib.q3t_vocoder_decode_chunked(self.h, codes, codes.shape[0], 16, int(chunk_frames), pcm, C.byref(ns)))
        return pcm[:ns.value]

    def vocoder_batch(self, codes_list, mode=VOCODER_FULL, chunk_frames=40):
        """several utterances through shared launches (q3t_vocoder_decode_batch): returns one PCM array per
        utterance, each equal to vocoder(codes) (FULL) or vocoder_chunked(codes, chunk_frames) (CHUNK40)"""
        cs = [np.ascontiguousarray(c, np.int32).reshape(-1, 16) for c in codes_list]
        n = len(cs)
        nf = np.array([c.shape[0] for c in cs], np.int32)
        pcms = [np.zeros(max(self.vocoder_num_samples(int(f), mode), 1), np.float32) for f in nf]
        cp = (C.c_void_p * max(n, 1))(*[c.ctypes.data for c in cs])
        pp = (C.c_void_p * max(n, 1))(*[p.ctypes.data for p in pcms])
        ns = (C.c_int64 * max(n, 1))()
        _check(_lib.q3t_vocoder_decode_batch(self.h, n, cp, nf, int(mode), int(chunk_frames), pp, ns))
        return [pcms[i][:ns[i]] for i in range(n)]

    def vocoder_set_batch_frames(self, frames):
        _check(_lib.q3t_vocoder_set_batch_frames(self.h, int(frames)))

    # ---- speaker encoder
    def speaker_dim(self):
        """embedding length of the model's speaker encoder (0: the GGUF has none)"""
        return _lib.q3t_speaker_dim(self.h)

    def encode_speaker(self, samples):
        """AudioTokenizerEncoder::encode (src/audio_tokenizer_encoder.h:107-108): 24 kHz samples in [-1, 1] ->
        speaker embedding [speaker_dim]"""
        x = np.ascontiguousarray(samples, np.float32).ravel()
        emb = np.zeros(max(self.speaker_dim(), 1), np.float32)
        _check(_lib.q3t_speaker_encode(self.h, x, len(x), emb))
        return emb

    def speaker_mel(self, samples):
        """the speaker encoder's log-mel front end, [n_frames][128] (time-major)"""
        x = np.ascontiguousarray(samples, np.float32).ravel()
        nf = C.c_int32(0)
        _check(_lib.q3t_speaker_mel(self.h, x, len(x), None, 0, C.byref(nf)))
        mel = np.zeros((max(nf.value, 1), 128), np.float32)
        _check(_lib.q3t_speaker_mel(self.h, x, len(x), _addr(mel), nf.value, C.byref(nf)))
        return mel[:nf.value]

    # ---- stages
    def talker_forward(self, embd, pos):
        embd = np.ascontiguousarray(embd, np.float32).reshape(-1, self.cfg["hidden"])
        n = embd.shape[0]
        pos = np.ascontiguousarray(np.broadcast_to(np.asarray(pos, np.int32), (n,)))
        hid = np.zeros((n, self.cfg["hidden"]), np.float32)
        lg = np.zeros((n, self.cfg["codec_vocab"]), np.float32)
        _check(_lib.q3t_talker_forward(self.h, n, embd, pos, _addr(hid), _addr(lg)))
        return hid, lg

    def talker_prefill(self, embd, family_slots=0):
        """causal prefill from position 0: embd [n_utt][n_rows][H] -> (hidden [n_utt][n_rows][H], last-row logits
        [n_utt][V]); K/V rows [0, n_rows) of slots 0..n_utt-1 (TTSTransformer::forward_prefill)"""
        H = self.cfg["hidden"]
        embd = np.ascontiguousarray(embd, np.float32)
        if embd.ndim == 2:
            embd = embd[None]
        n_utt, n_rows = embd.shape[0], embd.shape[1]
        hid = np.zeros((n_utt, n_rows, H), np.float32)
        lg = np.zeros((n_utt, self.cfg["codec_vocab"]), np.float32)
        _check(_lib.q3t_talker_prefill(self.h, n_utt, n_rows, embd.reshape(-1), int(family_slots), _addr(hid), _addr(lg)))
        return hid, lg

    def codepred_frame(self, hidden, cb0, temperature=0.0, top_k=50, seed=0, frame=0, want_logits=False):
        hidden = np.ascontiguousarray(hidden, np.float32).reshape(-1, self.cfg["hidden"])
        n = hidden.shape[0]
        cb0 = np.ascontiguousarray(np.broadcast_to(np.asarray(cb0, np.int32), (n,)))
        codes = np.zeros((n, 15), np.int32)
        lg = np.zeros((n, 15, self.cfg["cp_vocab"]), np.float32) if want_logits else None
        _check(_lib.q3t_codepred_frame(self.h, n, hidden, cb0, float(temperature), int(top_k), int(seed), int(frame),
                                       codes, _addr(lg)))
        return (codes, lg) if want_logits else codes

    def cb0_select(self, logits, seen, frame, n_tokens, **params):
        p = default_params(**params)
        logits = np.ascontiguousarray(logits, np.float32).reshape(-1, self.cfg["codec_vocab"])
        n = logits.shape[0]
        seen = np.ascontiguousarray(seen, np.uint8).reshape(n, -1)
        frame = np.ascontiguousarray(np.broadcast_to(np.asarray(frame, np.int32), (n,)))
        nt = np.ascontiguousarray(np.broadcast_to(np.asarray(n_tokens, np.int32), (n,)))
        out = np.zeros(n, np.int32)
        _check(_lib.q3t_cb0_select(self.h, n, logits, seen, frame, nt, C.byref(p), out))
        return out

    def project_text(self, toks):
        toks = np.ascontiguousarray(toks, np.int32)
        out = np.zeros((len(toks), self.cfg["hidden"]), np.float32)
        _check(_lib.q3t_project_text(self.h, len(toks), toks, out))
        return out

    def prefill_embd(self, toks, speaker=None, language_id=2050):
        toks = np.ascontiguousarray(toks, np.int32)
        H = self.cfg["hidden"]
        pre = np.zeros((10, H), np.float32)
        tr = np.zeros((max(1, len(toks) - 8), H), np.float32)
        pad = np.zeros(H, np.float32)
        pl, tl = C.c_int32(0), C.c_int32(0)
        sp = None if speaker is None else np.ascontiguousarray(speaker, np.float32)
        _check(_lib.q3t_prefill_embd(self.h, toks, len(toks), _addr(sp), int(language_id), pre, C.byref(pl), tr,
                                     C.byref(tl), pad))
        return pre[:pl.value], tr[:tl.value], pad
