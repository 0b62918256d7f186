// tokenizer.h — byte-level BPE text tokenizer with the TTS chat template.
//
// Same observable behaviour as qwen3_tts::TextTokenizer (src/text_tokenizer.{h,cpp}), including its simplifications:
// words split only before spaces (no regex pre-tokeniser, :244-268), unknown BPE pieces fall back to the byte symbols
// of the piece's UTF-8 bytes (:278-285), special ids from the GGUF or the defaults of text_tokenizer.h:13-18.
// Host code: tokenisation is microseconds per utterance and never on the decode path.  Faster than the reference's
// std::map lookups and O(n^2) rescans: pair ranks in one hash map keyed by "first\x01second", and a per-word cache.
#pragma once
#include <cstdint>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "gguf.h"

namespace q3t {

class TextTokenizer {
public:
    // tokenizer.ggml.tokens / merges / *_token_id of a GGUF (the TTS model file); false + set_error when absent
    bool load(const Gguf &g);
    bool load(const std::string &gguf_path);
    std::vector<int32_t> encode(const std::string &text) const;
    // <|im_start|>assistant\n{text}<|im_end|>\n<|im_start|>assistant\n (text_tokenizer.cpp:293-330)
    std::vector<int32_t> encode_for_tts(const std::string &text) const;
    std::string decode(const std::vector<int32_t> &ids) const;
    std::string decode_token(int32_t id) const;

    int32_t vocab_size() const { return (int32_t)id_to_token_.size(); }
    int32_t bos() const { return bos_; }
    int32_t eos() const { return eos_; }
    int32_t pad() const { return pad_; }
    int32_t assistant() const { return assistant_; }
    int32_t newline() const { return newline_; }

private:
    void bpe(const std::string &word, std::vector<std::string> &out) const;
    int32_t rank(const std::string &a, const std::string &b) const;

    std::unordered_map<std::string, int32_t> vocab_;
    std::vector<std::string> id_to_token_;
    std::unordered_map<std::string, int32_t> ranks_;
    int32_t bos_ = 151644, eos_ = 151645, pad_ = 151643, assistant_ = -1, newline_ = -1;
    mutable std::mutex cache_mu_;
    mutable std::unordered_map<std::string, std::vector<int32_t>> cache_;   // word -> ids
};

}  // namespace q3t
