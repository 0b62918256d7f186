// gguf.h — GGUF v2/v3 reader (mmap) for the Qwen3-TTS model files.
// Replaces the reference's ggml-based GGUFLoader (src/gguf_loader.h:15-80) without depending on ggml.
#pragma once
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace q3t {

enum GgmlType { GGML_TYPE_F32 = 0, GGML_TYPE_F16 = 1 };

struct GgufTensor {
    std::string name;
    int n_dims = 0;
    int64_t ne[4] = {1, 1, 1, 1};
    int type = 0;
    uint64_t offset = 0;
    const void *data = nullptr;
    size_t nbytes() const;
    int64_t nelements() const { return ne[0] * ne[1] * ne[2] * ne[3]; }
};

struct GgufValue {
    int type = -1;
    uint64_t u = 0;
    double f = 0.0;
    std::string s;
    std::vector<int64_t> arr;
    std::vector<std::string> sarr;   // string arrays (tokenizer.ggml.tokens / merges)
};

class Gguf {
public:
    ~Gguf();
    bool open(const std::string &path);
    void close();
    const GgufTensor *find(const std::string &name) const;
    // first present key wins, like the lambdas of tts_transformer.cpp:289-307
    int64_t get_int(std::initializer_list<const char *> keys, int64_t def) const;
    float get_f32(std::initializer_list<const char *> keys, float def) const;
    const GgufValue *get(const std::string &key) const;
    const std::vector<GgufTensor> &tensors() const { return tensors_; }
    const std::string &error() const { return err_; }

private:
    std::string err_;
    uint8_t *map_ = nullptr;
    size_t size_ = 0;
    std::vector<GgufTensor> tensors_;
    std::unordered_map<std::string, size_t> index_;
    std::unordered_map<std::string, GgufValue> kv_;
};

}  // namespace q3t
