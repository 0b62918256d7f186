// vocoder.h — MI355X-native Qwen3-TTS tokenizer decoder ("vocoder"), replacing TRTVocoderDecoder
// (src/trt_vocoder.cpp) and the GGML AudioTokenizerDecoder (src/audio_tokenizer_decoder.cpp).
#pragma once
#include <string>
#include <vector>

#include "gguf.h"
#include "kernels.h"

namespace q3t {

class Vocoder {
public:
    ~Vocoder();
    bool load(const std::string &tok_gguf, hipStream_t s);
    // mode 0 = FULL (GGML decoder semantics), 1 = CHUNK40 (TRT streaming semantics)
    int64_t n_samples(int n_frames, int mode) const;
    bool decode(const int32_t *codes_host, int n_frames, int mode, float *pcm_host, int64_t *n_out);
    bool decode_device(const int32_t *codes_dev, int n_frames, float *pcm_dev, int64_t *n_out, hipStream_t s);
    bool loaded() const { return loaded_; }

private:
    bool loaded_ = false;
    hipStream_t stream_ = nullptr;
    std::vector<void *> allocs_;
};

}  // namespace q3t
