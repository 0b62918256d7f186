// qwen3_tts_pipeline.h — the reference's pipeline surface (src/qwen3_tts.h:17-156): tts_params, tts_result, Qwen3TTS,
// load_audio_file, save_audio_file, over the component classes of qwen3_tts_hip.h.  Same names, fields, defaults and
// error convention; the deliberate differences are listed in qwen3_tts_hip.h.  Library: libqwen3_tts_pipeline.so.
#ifndef QWEN3_TTS_PIPELINE_H
#define QWEN3_TTS_PIPELINE_H

#include "qwen3_tts_hip.h"

namespace qwen3_tts {

// ====================================================================================== pipeline (src/qwen3_tts.h)
struct tts_params {
    int32_t max_audio_tokens = 4096;
    float temperature = 0.9f;
    float top_p = 1.0f;       // accepted, unused (as in the reference: no top-p stage exists in its sampler)
    int32_t top_k = 50;
    int32_t n_threads = 4;    // accepted, unused (host threads do no numeric work here)
    bool print_progress = false;
    bool print_timing = true;
    float repetition_penalty = 1.05f;
};

struct tts_result {
    std::vector<float> audio;
    int32_t sample_rate = 24000;
    bool success = false;
    std::string error_msg;
    int64_t t_load_ms = 0;
    int64_t t_tokenize_ms = 0;
    int64_t t_encode_ms = 0;
    int64_t t_generate_ms = 0;
    int64_t t_decode_ms = 0;
    int64_t t_total_ms = 0;
    uint64_t mem_rss_start_bytes = 0;
    uint64_t mem_rss_end_bytes = 0;
    uint64_t mem_rss_peak_bytes = 0;
    uint64_t mem_phys_start_bytes = 0;
    uint64_t mem_phys_end_bytes = 0;
    uint64_t mem_phys_peak_bytes = 0;
};

class Qwen3TTS {
public:
    Qwen3TTS();
    ~Qwen3TTS();
    Qwen3TTS(const Qwen3TTS &) = delete;
    Qwen3TTS &operator=(const Qwen3TTS &) = delete;

    // model_dir holds qwen3-tts-0.6b-f16.gguf and qwen3-tts-tokenizer-f16.gguf (qwen3_tts.cpp:117-118)
    bool load_models(const std::string &model_dir);
    tts_result synthesize(const std::string &text, const tts_params &params = tts_params());
    tts_result synthesize_with_voice(const std::string &text, const std::string &reference_audio,
                                     const tts_params &params = tts_params());
    tts_result synthesize_with_voice(const std::string &text, const float *ref_samples, int32_t n_ref_samples,
                                     const tts_params &params = tts_params());
    bool encode_speaker(const std::string &reference_audio, std::vector<float> &embedding);
    tts_result synthesize_with_embedding(const std::string &text, const std::vector<float> &speaker_embedding,
                                         const tts_params &params = tts_params());
    const std::string &get_error() const { return error_msg_; }
    bool is_loaded() const { return models_loaded_; }

    // ---- MI355X extensions
    bool set_device(int device);           // before load_models
    void set_seed(uint64_t seed) { seed_ = seed; }
    // 0: whole-utterance vocoder after generation; n > 0: n-frame chunks streamed from the frame callback
    void set_vocoder_chunk(int32_t frames) { vocoder_chunk_ = frames; }
    int32_t vocoder_chunk() const { return vocoder_chunk_; }
    // n utterances decoded together on one GPU (lock-step slots); speaker_embeddings empty or one per text (an empty
    // vector = no speaker row); results[i] as synthesize_with_embedding's
    std::vector<tts_result> synthesize_batch(const std::vector<std::string> &texts,
                                             const std::vector<std::vector<float>> &speaker_embeddings,
                                             const tts_params &params = tts_params());

private:
    tts_result synthesize_internal(const std::string &text, const float *speaker_embedding, const tts_params &params,
                                   tts_result &result);
    bool ensure_slots(int32_t slots, int32_t max_len);

    TextTokenizer tokenizer_;
    q3t_ctx *ctx_ = nullptr;
    int device_ = 0;
    uint64_t seed_ = 0;
    int32_t slots_ = 0, n_ctx_ = 0, hidden_ = 1024;
    int32_t vocoder_chunk_ = 0;
    bool models_loaded_ = false;
    std::string error_msg_;
    std::string tts_model_path_;
    std::string decoder_model_path_;
};

// WAV: RIFF PCM16 / PCM32 / IEEE float32, channels averaged to mono (qwen3_tts.cpp:567-706)
bool load_audio_file(const std::string &path, std::vector<float> &samples, int &sample_rate);
// WAV PCM16 mono, samples clamped to [-1, 1] and scaled by 32767 (qwen3_tts.cpp:708-759)
bool save_audio_file(const std::string &path, const std::vector<float> &samples, int sample_rate);
// linear resampling used for reference audio (qwen3_tts.cpp:83-101)
void resample_linear(const float *input, int input_len, int input_rate, std::vector<float> &output, int output_rate);

}  // namespace qwen3_tts

#endif
