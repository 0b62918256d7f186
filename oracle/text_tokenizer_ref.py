"""CPU restatement of the reference text tokenizer (src/text_tokenizer.cpp) -- TEST INFRASTRUCTURE.

Only tests/ may import this file; it is the checker of the product tokenizer (qwen3-tts-jetson_amd/csrc/tokenizer.cpp),
never part of it.  Pure Python: small inputs only.

Reference behaviour restated (every quirk kept, each one cited):
  - vocab: tokenizer.ggml.tokens, later duplicates win in the string->id map (:99-108);
  - merges: "first second" split at the first space, later duplicates overwrite the rank (:111-127);
  - special ids: tokenizer.ggml.{bos,eos,padding}_token_id when present, else 151644 / 151645 / 151643 (:129-143,
    text_tokenizer.h:13-18); "assistant" (else "Ġassistant") and "Ċ" (else "\\n") looked up by content, -1 when
    absent (:145-161);
  - encode: bytes -> GPT-2 unicode symbols, words split before every "Ġ" only (no regex pre-tokenisation, :244-268),
    BPE = repeatedly merge every non-overlapping occurrence of the lowest-rank adjacent pair (:167-232), unknown BPE
    pieces fall back to the vocab ids of BYTE_TO_UNICODE of each UTF-8 BYTE of the piece's unicode string (:278-285);
  - encode_for_tts: bos, assistant, newline, text, eos, newline, bos, assistant, newline (:293-330);
  - decode: GPT-2 symbols back to bytes, unknown symbols kept as-is (:62-78, :332-349).
"""
import struct


def _bytes_to_unicode_table():
    bs = list(range(33, 127)) + list(range(161, 173)) + list(range(174, 256))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {b: chr(c) for b, c in zip(bs, cs)}


BYTE_TO_UNICODE = _bytes_to_unicode_table()          # text_tokenizer.cpp:12-29
UNICODE_TO_BYTE = {v: k for k, v in BYTE_TO_UNICODE.items()}


def read_gguf_kv(path):
    """the KV section of a GGUF v2/v3 file (strings, scalars, arrays); tensors are not read"""
    scal = {0: "<B", 1: "<b", 2: "<H", 3: "<h", 4: "<I", 5: "<i", 6: "<f", 7: "<?", 10: "<Q", 11: "<q", 12: "<d"}
    with open(path, "rb") as f:
        assert f.read(4) == b"GGUF"
        ver, = struct.unpack("<I", f.read(4))
        assert ver in (2, 3)
        _nt, nkv = struct.unpack("<QQ", f.read(16))

        def rstr():
            n, = struct.unpack("<Q", f.read(8))
            return f.read(n).decode("utf-8", errors="surrogateescape")

        def rval(t):
            if t == 8:
                return rstr()
            if t == 9:
                et, n = struct.unpack("<IQ", f.read(12))
                return [rval(et) for _ in range(n)]
            fmt = scal[t]
            return struct.unpack(fmt, f.read(struct.calcsize(fmt)))[0]

        kv = {}
        for _ in range(nkv):
            k = rstr()
            t, = struct.unpack("<I", f.read(4))
            kv[k] = rval(t)
    return kv


def _utf8_len(b):   # text_tokenizer.cpp:46-52, on the first byte of a UTF-8 sequence
    if b & 0x80 == 0:
        return 1
    if b & 0xE0 == 0xC0:
        return 2
    if b & 0xF0 == 0xE0:
        return 3
    if b & 0xF8 == 0xF0:
        return 4
    return 1


def _chars(s_bytes):
    """split a UTF-8 byte string into per-character byte strings by the reference's utf8_len"""
    out, i = [], 0
    while i < len(s_bytes):
        n = _utf8_len(s_bytes[i])
        out.append(s_bytes[i:i + n])
        i += n
    return out


class RefTokenizer:
    def __init__(self, kv):
        tokens = kv["tokenizer.ggml.tokens"]
        self.id_to_token = [t.encode("utf-8", errors="surrogateescape") for t in tokens]
        self.vocab = {}
        for i, t in enumerate(self.id_to_token):
            self.vocab[t] = i
        self.ranks = {}
        for i, m in enumerate(kv.get("tokenizer.ggml.merges", [])):
            mb = m.encode("utf-8", errors="surrogateescape")
            sp = mb.find(b" ")
            if sp >= 0:
                self.ranks[(mb[:sp], mb[sp + 1:])] = i
        self.bos = int(kv.get("tokenizer.ggml.bos_token_id", 151644))
        self.eos = int(kv.get("tokenizer.ggml.eos_token_id", 151645))
        self.pad = int(kv.get("tokenizer.ggml.padding_token_id", 151643))
        a = self.vocab.get("assistant".encode(), self.vocab.get("Ġassistant".encode(), -1))
        self.assistant = a
        self.newline = self.vocab.get("Ċ".encode(), self.vocab.get(b"\n", -1))

    def bpe(self, word):
        w = _chars(word)
        if len(w) <= 1:
            return w
        while True:
            best, best_rank = None, None
            for i in range(len(w) - 1):
                r = self.ranks.get((w[i], w[i + 1]))
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = (w[i], w[i + 1]), r
            if best is None:
                break
            nw, j = [], 0
            while j < len(w):
                if j + 1 < len(w) and w[j] == best[0] and w[j + 1] == best[1]:
                    nw.append(best[0] + best[1])
                    j += 2
                else:
                    nw.append(w[j])
                    j += 1
            w = nw
            if len(w) == 1:
                break
        return w

    def encode(self, text):
        u = "".join(BYTE_TO_UNICODE[b] for b in text.encode("utf-8")).encode("utf-8")
        words, cur = [], b""
        sp = "Ġ".encode()
        for ch in _chars(u):
            if ch == sp:
                if cur:
                    words.append(cur)
                cur = ch
            else:
                cur += ch
        if cur:
            words.append(cur)
        out = []
        for w in words:
            for tok in self.bpe(w):
                if tok in self.vocab:
                    out.append(self.vocab[tok])
                else:
                    for b in tok:   # each BYTE of the piece's UTF-8 string (the reference's fallback quirk)
                        i = self.vocab.get(BYTE_TO_UNICODE[b].encode())
                        if i is not None:
                            out.append(i)
        return out

    def encode_for_tts(self, text):
        return ([self.bos, self.assistant, self.newline] + self.encode(text) +
                [self.eos, self.newline, self.bos, self.assistant, self.newline])

    def decode_token(self, i):
        if i < 0 or i >= len(self.id_to_token):
            return b""
        out = b""
        for ch in _chars(self.id_to_token[i]):
            c = ch.decode("utf-8", errors="surrogateescape")
            out += bytes([UNICODE_TO_BYTE[c]]) if c in UNICODE_TO_BYTE else ch
        return out

    def decode(self, ids):
        return b"".join(self.decode_token(i) for i in ids)
