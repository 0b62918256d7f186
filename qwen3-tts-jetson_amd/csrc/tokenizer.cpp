// tokenizer.cpp — see tokenizer.h.
#include "tokenizer.h"

#include <climits>

#include "q3t_common.h"

namespace q3t {

namespace {
// GPT-2 bytes_to_unicode: printable latin-1 bytes keep their code point, the other 68 map to U+0100.. in byte order
struct ByteSyms {
    std::string sym[256];
    std::unordered_map<std::string, uint8_t> back;
    ByteSyms() {
        int n = 0;
        for (int b = 0; b < 256; ++b) {
            const bool keep = (b >= 33 && b <= 126) || (b >= 161 && b <= 172) || b >= 174;
            const int cp = keep ? b : 256 + n++;
            std::string s;
            if (cp < 0x80) s.push_back((char)cp);
            else { s.push_back((char)(0xC0 | (cp >> 6))); s.push_back((char)(0x80 | (cp & 0x3F))); }
            sym[b] = s;
            back[s] = (uint8_t)b;
        }
    }
};
const ByteSyms &syms() {
    static const ByteSyms s;
    return s;
}
// length of the UTF-8 sequence a lead byte starts; stray continuation bytes count as 1 (text_tokenizer.cpp:46-52)
inline size_t u8len(unsigned char c) {
    if ((c & 0x80) == 0) return 1;
    if ((c & 0xE0) == 0xC0) return 2;
    if ((c & 0xF0) == 0xE0) return 3;
    if ((c & 0xF8) == 0xF0) return 4;
    return 1;
}
std::string pair_key(const std::string &a, const std::string &b) {
    std::string k;
    k.reserve(a.size() + b.size() + 1);
    k.append(a).push_back('\0');
    k.append(b);
    return k;
}
}  // namespace

bool TextTokenizer::load(const std::string &gguf_path) {
    Gguf g;
    if (!g.open(gguf_path)) { set_error(g.error()); return false; }
    return load(g);
}

bool TextTokenizer::load(const Gguf &g) {
    const GgufValue *toks = g.get("tokenizer.ggml.tokens");
    if (!toks) { set_error("tokenizer.ggml.tokens not found in GGUF"); return false; }
    if (toks->sarr.empty()) { set_error("Empty vocabulary"); return false; }
    id_to_token_ = toks->sarr;
    vocab_.clear();
    vocab_.reserve(id_to_token_.size() * 2);
    for (size_t i = 0; i < id_to_token_.size(); ++i) vocab_[id_to_token_[i]] = (int32_t)i;   // later duplicates win
    ranks_.clear();
    if (const GgufValue *m = g.get("tokenizer.ggml.merges")) {
        ranks_.reserve(m->sarr.size() * 2);
        for (size_t i = 0; i < m->sarr.size(); ++i) {
            const std::string &s = m->sarr[i];
            const size_t sp = s.find(' ');
            if (sp != std::string::npos) ranks_[pair_key(s.substr(0, sp), s.substr(sp + 1))] = (int32_t)i;
        }
    }
    bos_ = (int32_t)g.get_int({"tokenizer.ggml.bos_token_id"}, 151644);
    eos_ = (int32_t)g.get_int({"tokenizer.ggml.eos_token_id"}, 151645);
    pad_ = (int32_t)g.get_int({"tokenizer.ggml.padding_token_id"}, 151643);
    auto find = [&](const std::string &t) { auto it = vocab_.find(t); return it == vocab_.end() ? -1 : it->second; };
    assistant_ = find("assistant");
    if (assistant_ < 0) assistant_ = find("\xC4\xA0" "assistant");   // "Ġassistant"
    newline_ = find("\xC4\x8A");                                     // "Ċ"
    if (newline_ < 0) newline_ = find("\n");
    std::lock_guard<std::mutex> lk(cache_mu_);
    cache_.clear();
    return true;
}

int32_t TextTokenizer::rank(const std::string &a, const std::string &b) const {
    auto it = ranks_.find(pair_key(a, b));
    return it == ranks_.end() ? INT32_MAX : it->second;
}

void TextTokenizer::bpe(const std::string &token, std::vector<std::string> &w) const {
    w.clear();
    for (size_t i = 0; i < token.size();) {
        const size_t n = u8len((unsigned char)token[i]);
        w.push_back(token.substr(i, n));
        i += n;
    }
    if (w.size() < 2) return;
    // lowest-rank adjacent pair (first occurrence on equal rank), then merge every non-overlapping occurrence left to
    // right (text_tokenizer.cpp:167-232); ranks of the current pairs are kept in a vector and refreshed locally
    std::vector<int32_t> r(w.size() - 1);
    for (size_t i = 0; i + 1 < w.size(); ++i) r[i] = rank(w[i], w[i + 1]);
    while (w.size() > 1) {
        int32_t best = INT32_MAX;
        size_t at = 0;
        for (size_t i = 0; i < r.size(); ++i)
            if (r[i] < best) { best = r[i]; at = i; }
        if (best == INT32_MAX) break;
        const std::string a = w[at], b = w[at + 1];
        std::vector<std::string> nw;
        nw.reserve(w.size());
        for (size_t j = 0; j < w.size();) {
            if (j + 1 < w.size() && w[j] == a && w[j + 1] == b) { nw.push_back(a + b); j += 2; }
            else nw.push_back(w[j++]);
        }
        w.swap(nw);
        r.assign(w.size() > 0 ? w.size() - 1 : 0, 0);
        for (size_t i = 0; i + 1 < w.size(); ++i) r[i] = rank(w[i], w[i + 1]);
    }
}

std::vector<int32_t> TextTokenizer::encode(const std::string &text) const {
    std::vector<int32_t> out;
    if (id_to_token_.empty()) return out;
    const ByteSyms &S = syms();
    const std::string &space = S.sym[(unsigned char)' '];
    // words: a new word starts at every space symbol and keeps it (text_tokenizer.cpp:244-268)
    std::vector<std::string> words;
    std::string cur;
    for (unsigned char c : text) {
        if (S.sym[c] == space) {
            if (!cur.empty()) words.push_back(cur);
            cur = space;
        } else {
            cur += S.sym[c];
        }
    }
    if (!cur.empty()) words.push_back(cur);
    std::vector<std::string> pieces;
    for (const std::string &word : words) {
        {
            std::lock_guard<std::mutex> lk(cache_mu_);
            auto it = cache_.find(word);
            if (it != cache_.end()) { out.insert(out.end(), it->second.begin(), it->second.end()); continue; }
        }
        std::vector<int32_t> ids;
        bpe(word, pieces);
        for (const std::string &p : pieces) {
            auto it = vocab_.find(p);
            if (it != vocab_.end()) { ids.push_back(it->second); continue; }
            for (unsigned char c : p) {   // unknown piece: byte symbols of its UTF-8 bytes (:278-285)
                auto bt = vocab_.find(S.sym[c]);
                if (bt != vocab_.end()) ids.push_back(bt->second);
            }
        }
        out.insert(out.end(), ids.begin(), ids.end());
        std::lock_guard<std::mutex> lk(cache_mu_);
        if (cache_.size() < (1u << 16)) cache_.emplace(word, std::move(ids));
    }
    return out;
}

std::vector<int32_t> TextTokenizer::encode_for_tts(const std::string &text) const {
    if (id_to_token_.empty()) return {};
    std::vector<int32_t> t{bos_, assistant_, newline_};
    const std::vector<int32_t> body = encode(text);
    t.insert(t.end(), body.begin(), body.end());
    t.insert(t.end(), {eos_, newline_, bos_, assistant_, newline_});
    return t;
}

std::string TextTokenizer::decode_token(int32_t id) const {
    if (id < 0 || id >= (int32_t)id_to_token_.size()) return "";
    const std::string &t = id_to_token_[id];
    const ByteSyms &S = syms();
    std::string out;
    for (size_t i = 0; i < t.size();) {
        const size_t n = u8len((unsigned char)t[i]);
        const std::string ch = t.substr(i, n);
        auto it = S.back.find(ch);
        if (it != S.back.end()) out.push_back((char)it->second);
        else out += ch;   // not a byte symbol: kept as-is (:71-74)
        i += n;
    }
    return out;
}

std::string TextTokenizer::decode(const std::vector<int32_t> &ids) const {
    std::string s;
    for (int32_t id : ids) s += decode_token(id);
    return s;
}

}  // namespace q3t
