// gguf.h — GGUF v2/v3 reader (mmap) for the Qwen3-TTS model files.
// Replaces the reference's ggml-based GGUFLoader (src/gguf_loader.h:15-80) without depending on ggml.
//
// Weight dtypes: every file the reference converters can write loads (convert_tts_to_gguf.py:276-335,
// convert_tokenizer_to_gguf.py:265-296): F16; F32 (1-D tensors stay F32, 2-D+ are rounded to F16); Q8_0, Q4_0 and
// Q4_K matrices are dequantised at open (ggml's dequantize_row_q8_0 / q4_0 / q4_K, ggml-quants.c of the ggml
// submodule the reference pins; restated here, the submodule is not vendored) and then rounded to F16.  Loaders
// therefore see the F16 file layout; GgufTensor::src_type keeps the on-disk type.  One resident F16 copy is the
// MI355X layout choice: every decode kernel streams F16 rows (at batch 1 the step is hand-off bound, not byte
// bound), so in-kernel dequantisation would add a second code path for no measured gain.
#pragma once
#include <cstdint>
#include <string>
#include <unordered_map>
#include <vector>

namespace q3t {

enum GgmlType { GGML_TYPE_F32 = 0, GGML_TYPE_F16 = 1, GGML_TYPE_Q4_0 = 2, GGML_TYPE_Q8_0 = 8, GGML_TYPE_Q4_K = 12 };

struct GgufTensor {
    std::string name;
    int n_dims = 0;
    int64_t ne[4] = {1, 1, 1, 1};
    int type = 0;       // as loaded: F16 / F32 (see above)
    int src_type = 0;   // as stored in the file
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
    std::vector<std::vector<uint16_t>> owned_;   // dequantised / rounded F16 copies
};

// bytes of n elements of a GGML type (0: unsupported); block-quantised types need n % block == 0
size_t ggml_type_bytes(int type, int64_t n);
// one row of a supported on-disk type -> f32 (dequantize_row_* of ggml-quants.c)
bool ggml_to_f32(int type, const void *src, float *dst, int64_t n);

}  // namespace q3t
