// gguf_loader.h — stand-in for the reference's ggml-based src/gguf_loader.h (the one header the drop-in does not
// provide: this library has no ggml).  src/qwen3_tts.cpp:136-150 only opens the TTS GGUF to hand the tokenizer its
// context; the MI355X TextTokenizer::load_from_gguf reads the vocabulary from the path itself, so the stand-in loader
// carries the path as its "context".
#pragma once
#include <cstdio>
#include <string>

namespace qwen3_tts {

class GGUFLoader {
public:
    bool open(const std::string &path) {
        FILE *f = std::fopen(path.c_str(), "rb");
        if (!f) { error_ = "Failed to open file: " + path; return false; }
        std::fclose(f);
        path_ = path;
        return true;
    }
    const std::string &get_ctx() const { return path_; }
    const std::string &get_error() const { return error_; }

private:
    std::string path_, error_;
};

}  // namespace qwen3_tts
