"""ctypes binding of the CPU oracle (oracle/_build/libq3t_oracle.so).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "_build", "libq3t_oracle.so")

_CFG_FIELDS = [
    "hidden", "n_layers", "n_heads", "n_kv", "head_dim", "inter", "codec_vocab", "n_codebooks", "text_vocab",
    "text_dim", "cp_layers", "cp_vocab", "eps", "rope_theta", "codec_pad", "codec_bos", "codec_eos", "tts_bos",
    "tts_eos", "tts_pad", "think", "nothink", "think_bos", "think_eos", "has_vocoder", "cb_dim", "cb_size",
    "voc_hidden", "voc_latent", "voc_heads", "voc_layers", "voc_ffn", "dec_dim", "up_k",
]


class OracleConfig(C.Structure):
    _fields_ = [(n, C.c_float if n in ("eps", "rope_theta") else C.c_int) for n in _CFG_FIELDS] + [
        ("conv_t_k", C.c_int * 4), ("rates", C.c_int * 4)] + [
        (n, C.c_int) for n in ("cp_hidden", "cp_inter", "cp_heads", "cp_kv", "cp_head_dim", "has_mtp")]


def build_oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build_oracle()
        L = C.CDLL(ORACLE_SO)
        P, I, F, U64 = C.c_void_p, C.c_int, C.c_float, C.c_uint64
        fp = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        ip = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        L.q3o_error.restype = C.c_char_p
        L.q3o_load.restype = P
        L.q3o_load.argtypes = [C.c_char_p, C.c_char_p, I]
        L.q3o_free.argtypes = [P]
        L.q3o_get_config.argtypes = [P, C.POINTER(OracleConfig)]
        L.q3o_set_threads.argtypes = [I]
        L.q3o_kv_new.restype = P
        L.q3o_kv_new.argtypes = [P, I, I]
        L.q3o_kv_free.argtypes = [P]
        L.q3o_talker_step.argtypes = [P, P, fp, I, fp, fp]
        L.q3o_talker_step_n.argtypes = [P, P, fp, I, I, fp, fp]
        L.q3o_project_text.argtypes = [P, ip, I, fp]
        L.q3o_prefill_embd.argtypes = [P, ip, I, P, I, fp, C.POINTER(I), fp, C.POINTER(I), fp]
        L.q3o_cp_pass.argtypes = [P, P, fp, I, I, P, P]
        L.q3o_cp_frame.argtypes = [P, fp, I, F, I, P, ip, P]
        L.q3o_cp_frame_forced.argtypes = [P, fp, I, ip, fp]
        L.q3o_sample.argtypes = [fp, I, F, I, F, I]
        L.q3o_cb0_select.argtypes = [P, fp, np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS"), I, I, F, F, I, F, I]
        L.q3o_uniform.restype = F
        L.q3o_uniform.argtypes = [U64, U64, U64, U64]
        L.q3o_generate.argtypes = [P, ip, I, P, I, I, F, F, I, U64, U64, I, ip, C.POINTER(I), P, P]
        L.q3o_generate_forced.argtypes = [P, ip, I, P, I, F, I, ip, I, P, P]
        L.q3o_generate_forced_from.argtypes = [P, ip, I, P, I, F, I, ip, I, I, P, P]
        L.q3o_vocoder_decode.argtypes = [P, ip, I, I, P, C.POINTER(C.c_int64)]
        L.q3o_codebook.argtypes = [P, I, fp]
        L.q3o_mel.argtypes = [P, fp, I, P, C.POINTER(I)]
        L.q3o_speaker_encode.argtypes = [P, fp, I, fp]
        L.q3o_speaker_dim.argtypes = [P]
        L.q3o_tensor.argtypes = [P, C.c_char_p, fp, C.c_int64, C.POINTER(I)]
        L.q3o_vocoder_len.restype = C.c_int64
        L.q3o_vocoder_len.argtypes = [P, I, I]
        L.q3o_f32_to_f16.restype = C.c_uint16
        L.q3o_f32_to_f16.argtypes = [F]
        L.q3o_rope_cache.argtypes = [F, I, F, fp]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Oracle:
    def __init__(self, tts_gguf, tok_gguf=None, ggml_rounding=True, threads=None):
        L = lib()
        if threads:
            L.q3o_set_threads(int(threads))
        self.h = L.q3o_load(tts_gguf.encode(), tok_gguf.encode() if tok_gguf else None, 1 if ggml_rounding else 0)
        if not self.h:
            raise RuntimeError("oracle load failed: " + L.q3o_error().decode())
        c = OracleConfig()
        L.q3o_get_config(self.h, C.byref(c))
        self.cfg = {n: getattr(c, n) for n in _CFG_FIELDS}
        self.cfg["conv_t_k"] = list(c.conv_t_k)
        self.cfg["rates"] = list(c.rates)
        for n in ("cp_hidden", "cp_inter", "cp_heads", "cp_kv", "cp_head_dim", "has_mtp"):
            self.cfg[n] = getattr(c, n)

    def close(self):
        if self.h:
            lib().q3o_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- talker
    def kv_new(self, n_ctx, which=0):
        return lib().q3o_kv_new(self.h, n_ctx, which)

    def kv_free(self, kv):
        lib().q3o_kv_free(kv)

    def talker_step(self, kv, embd, pos, n_layers=0):
        H, V = self.cfg["hidden"], self.cfg["codec_vocab"]
        hid = np.zeros(H, np.float32)
        lg = np.zeros(V, np.float32)
        if not lib().q3o_talker_step_n(self.h, kv, np.ascontiguousarray(embd, np.float32), pos, n_layers, hid, lg):
            raise RuntimeError(lib().q3o_error().decode())
        return hid, lg

    def project_text(self, toks):
        toks = np.ascontiguousarray(toks, np.int32)
        out = np.zeros((len(toks), self.cfg["hidden"]), np.float32)
        if not lib().q3o_project_text(self.h, toks, len(toks), out):
            raise RuntimeError(lib().q3o_error().decode())
        return out

    def prefill_embd(self, toks, spk=None, language_id=2050):
        toks = np.ascontiguousarray(toks, np.int32)
        H = self.cfg["hidden"]
        pre = np.zeros((10, H), np.float32)
        tr = np.zeros((max(1, len(toks) - 8), H), np.float32)
        pad = np.zeros(H, np.float32)
        pl, tl = C.c_int(0), C.c_int(0)
        spk_a = None if spk is None else np.ascontiguousarray(spk, np.float32)
        if not lib().q3o_prefill_embd(self.h, toks, len(toks), _ptr(spk_a), language_id, pre, C.byref(pl), tr,
                                      C.byref(tl), pad):
            raise RuntimeError(lib().q3o_error().decode())
        return pre[:pl.value], tr[:tl.value], pad

    # ---- code predictor
    def cp_frame(self, hidden, cb0, temperature=0.0, top_k=50, u15=None, want_logits=False):
        codes = np.zeros(15, np.int32)
        lg = np.zeros((15, self.cfg["cp_vocab"]), np.float32) if want_logits else None
        u = None if u15 is None else np.ascontiguousarray(u15, np.float32)
        lib().q3o_cp_frame(self.h, np.ascontiguousarray(hidden, np.float32), int(cb0), float(temperature),
                           int(top_k), _ptr(u), codes, _ptr(lg))
        return (codes, lg) if want_logits else codes

    def cp_frame_forced(self, hidden, cb0, codes15):
        lg = np.zeros((15, self.cfg["cp_vocab"]), np.float32)
        lib().q3o_cp_frame_forced(self.h, np.ascontiguousarray(hidden, np.float32), int(cb0),
                                  np.ascontiguousarray(codes15, np.int32), lg)
        return lg

    def cp_pass(self, kv, x, pos, head=-1):
        H = self.cfg["cp_hidden"] or self.cfg["hidden"]   # x: talker space; the hidden output: code-predictor space
        hid = np.zeros(H, np.float32)
        lg = np.zeros(self.cfg["cp_vocab"], np.float32)
        lib().q3o_cp_pass(self.h, kv, np.ascontiguousarray(x, np.float32), pos, head, _ptr(hid), _ptr(lg))
        return hid, lg

    def cb0_select(self, logits, seen, frame, n_tokens, rep=1.05, temperature=0.0, top_k=50, u=0.0, eos_mask=0):
        lg = np.array(logits, np.float32, copy=True)
        tok = lib().q3o_cb0_select(self.h, lg, np.ascontiguousarray(seen, np.uint8), frame, n_tokens, rep,
                                   temperature, top_k, u, eos_mask)
        return tok, lg

    def generate(self, toks, spk=None, max_len=32, language_id=2050, rep=1.05, temperature=0.0, top_k=50,
                 seed=1234, utt=0, force_frames=0, trace=False):
        toks = np.ascontiguousarray(toks, np.int32)
        codes = np.zeros((max_len, self.cfg["n_codebooks"]), np.int32)
        nf = C.c_int(0)
        spk_a = None if spk is None else np.ascontiguousarray(spk, np.float32)
        lt = np.zeros((max_len, self.cfg["codec_vocab"]), np.float32) if trace else None
        ht = np.zeros((max_len, self.cfg["hidden"]), np.float32) if trace else None
        if not lib().q3o_generate(self.h, toks, len(toks), _ptr(spk_a), max_len, language_id, rep, temperature,
                                  top_k, seed, utt, force_frames, codes, C.byref(nf), _ptr(lt), _ptr(ht)):
            raise RuntimeError(lib().q3o_error().decode())
        n = nf.value
        if trace:
            return codes[:n], lt[:n], ht[:n]
        return codes[:n]

    def generate_forced(self, toks, forced, spk=None, language_id=2050, rep=1.05, force_frames=0, from_frame=0):
        """teacher-forced replay: returns (processed CB0 logits [F'][Vc], CP logits [F'][15][Vcp]) for the frames
        from_frame..F-1 (earlier frames only advance the talker with their forced codes)."""
        toks = np.ascontiguousarray(toks, np.int32)
        forced = np.ascontiguousarray(forced, np.int32).reshape(-1, 16)
        F = forced.shape[0]
        nt = max(F - from_frame, 0)
        cb0 = np.zeros((max(nt, 1), self.cfg["codec_vocab"]), np.float32)
        cp = np.zeros((max(nt, 1), 15, self.cfg["cp_vocab"]), np.float32)
        spk_a = None if spk is None else np.ascontiguousarray(spk, np.float32)
        if not lib().q3o_generate_forced_from(self.h, toks, len(toks), _ptr(spk_a), language_id, rep, force_frames,
                                              forced, F, int(from_frame), _ptr(cb0), _ptr(cp)):
            raise RuntimeError(lib().q3o_error().decode())
        return cb0[:nt], cp[:nt]

    # ---- vocoder
    def codebook(self, i):
        out = np.zeros((self.cfg["cb_size"], self.cfg["cb_dim"]), np.float32)
        if not lib().q3o_codebook(self.h, int(i), out):
            raise RuntimeError(lib().q3o_error().decode())
        return out

    def vocoder_len(self, n_frames, mode=0):
        return lib().q3o_vocoder_len(self.h, n_frames, mode)

    def vocoder(self, codes, mode=0):
        codes = np.ascontiguousarray(codes, np.int32)
        F = codes.shape[0]
        n = self.vocoder_len(F, mode)
        pcm = np.zeros(max(n, 1), np.float32)
        ns = C.c_int64(0)
        if not lib().q3o_vocoder_decode(self.h, codes, F, mode, _ptr(pcm), C.byref(ns)):
            raise RuntimeError(lib().q3o_error().decode())
        return pcm[:ns.value]


    def tensor(self, name, n):
        """(values as loaded [n] f32, on-disk GGML type)"""
        out = np.zeros(n, np.float32)
        st = C.c_int(0)
        if not lib().q3o_tensor(self.h, name.encode(), out, int(n), C.byref(st)):
            raise RuntimeError(lib().q3o_error().decode())
        return out, st.value

    # ---- speaker encoder
    def speaker_dim(self):
        return lib().q3o_speaker_dim(self.h)

    def mel(self, samples):
        """[n_frames][128] (transposed from the oracle's [128][F] to the engine's time-major layout)"""
        x = np.ascontiguousarray(samples, np.float32)
        nf = C.c_int(0)
        if not lib().q3o_mel(self.h, x, len(x), None, C.byref(nf)):
            raise RuntimeError(lib().q3o_error().decode())
        mel = np.zeros((128, max(nf.value, 1)), np.float32)
        if not lib().q3o_mel(self.h, x, len(x), _ptr(mel), C.byref(nf)):
            raise RuntimeError(lib().q3o_error().decode())
        return np.ascontiguousarray(mel[:, :nf.value].T)

    def encode_speaker(self, samples):
        x = np.ascontiguousarray(samples, np.float32)
        emb = np.zeros(max(self.speaker_dim(), 1), np.float32)
        if not lib().q3o_speaker_encode(self.h, x, len(x), emb):
            raise RuntimeError(lib().q3o_error().decode())
        return emb


def uniform(seed, utt, frame, cb):
    return lib().q3o_uniform(seed, utt, frame, cb)
