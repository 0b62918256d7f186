// qwen3_tts_hip.h — the reference's model-runtime C++ surface (SURVEY §8(b) layer 2) over the C ABI of libq3t.so.
//
// Same namespace, class names, method names, argument meaning and error convention (bool + get_error()) as
//   qwen3_tts::TTSTransformer        src/tts_transformer.h:164-245
//   qwen3_tts::AudioTokenizerDecoder src/audio_tokenizer_decoder.h:156-180
//   qwen3_tts::TRTVocoderDecoder     src/trt_vocoder.h:18-42
//   qwen3_tts::TextTokenizer         src/text_tokenizer.h:21-86
//   qwen3_tts::AudioTokenizerEncoder src/audio_tokenizer_encoder.h:95-125
// so a caller switches by including this header instead of those and linking libqwen3_tts_hip.so + libq3t.so
// (tests/boundary: the reference's own src/qwen3_tts.cpp + src/main.cpp compile and link against it unchanged).
// The pipeline above them (Qwen3TTS, src/qwen3_tts.h) is qwen3_tts_pipeline.h / libqwen3_tts_pipeline.so.  Every
// method forwards to q3t_* calls; all weights, KV caches and scratch stay resident in HBM inside a q3t_ctx.  No
// exceptions cross this surface.
//
// Differences a caller can see (each one deliberate):
//  - generate() draws its samples from a counter-based generator keyed by set_seed() (default 0) instead of
//    std::mt19937 seeded from std::random_device (src/tts_transformer.cpp:2371): runs are reproducible.
//  - on_frames is called with the same frames as the reference's callback, one chunk later in wall time (the GPU
//    keeps decoding while the host reads a chunk); returning false stops generation after the frames delivered.
//  - The KV cache is sized once for prefill + max_len + 8 positions (grown on demand by re-laying out the context
//    from the resident weights, never from the file), not re-allocated per generate() call.
//  - TRTVocoderDecoder::load_engine takes the tokenizer GGUF (there is no TensorRT engine on MI355X); given a path
//    that is not a GGUF (the reference's <model_dir>/vocoder_decoder_<n>.trt) it loads qwen3-tts-tokenizer-f16.gguf
//    from the same directory.  fixed_frames keeps its meaning: the independent chunk length of decode().
//  - TextTokenizer::load_from_gguf takes the GGUF path (the reference takes a ggml gguf_context *: this library has no
//    ggml); encode / encode_for_tts / decode are token-for-token the reference's (tests/test_tokenizer.py).
//  - Qwen3TTS keeps talker, code predictor, vocoder and speaker encoder in ONE device context (one weight upload, one
//    stream); the speaker encoder is loaded with it instead of lazily.  QWEN3_TTS_LOW_MEM is accepted and ignored
//    (everything stays resident in 288 GB of HBM).  The vocoder follows the reference's load order: a chunked decode
//    with the fixed_frames of the first vocoder_decoder_{40,30}.trt / vocoder_decoder_fixed.trt present in the model
//    directory (qwen3_tts.cpp:168-198), streamed from the frame callback every 40 frames; otherwise the whole-utterance
//    decode after generation (:492-529).
//  - Extensions (MI355X-native, no reference counterpart): set_device(), set_seed(), generate_batch(),
//    Qwen3TTS::synthesize_batch() / set_vocoder_chunk() / set_device() / set_seed().
#ifndef QWEN3_TTS_HIP_H
#define QWEN3_TTS_HIP_H

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

struct q3t_ctx;
struct q3t_tokenizer;

namespace qwen3_tts {

// src/tts_transformer.h:21-69 (field names and defaults); filled from the GGUF by load_model
struct tts_transformer_config {
    int32_t text_vocab_size = 151936;
    int32_t text_embd_dim = 2048;
    int32_t hidden_size = 1024;
    int32_t n_layers = 28;
    int32_t n_attention_heads = 16;
    int32_t n_key_value_heads = 8;
    int32_t intermediate_size = 3072;
    int32_t head_dim = 128;
    float rms_norm_eps = 1e-6f;
    float rope_theta = 1000000.0f;
    int32_t codec_vocab_size = 3072;
    int32_t n_codebooks = 16;
    int32_t code_pred_layers = 5;
    int32_t code_pred_vocab_size = 2048;
    int32_t codec_pad_id = 2148;
    int32_t codec_bos_id = 2149;
    int32_t codec_eos_id = 2150;
    int32_t english_language_id = 2050;
};

// src/audio_tokenizer_decoder.h:14-28
struct audio_decoder_config {
    int32_t sample_rate = 24000;
    int32_t n_codebooks = 16;
    int32_t codebook_size = 2048;
    int32_t codebook_dim = 256;
    int32_t latent_dim = 1024;
    int32_t hidden_dim = 512;
    int32_t n_pre_tfm_layers = 8;
    int32_t n_heads = 16;
    int32_t ffn_dim = 1024;
    int32_t decoder_dim = 1536;
    int32_t upsample_rates[4] = {8, 5, 4, 3};
};

class TTSTransformer {
public:
    TTSTransformer();
    ~TTSTransformer();
    TTSTransformer(const TTSTransformer &) = delete;
    TTSTransformer &operator=(const TTSTransformer &) = delete;

    bool load_model(const std::string &model_path);
    void unload_model();

    // the talker KV cache holds n_ctx positions (prefill + frames); grown if needed, kept otherwise
    bool init_kv_cache(int32_t n_ctx);
    // positions are addressed explicitly by n_past; nothing to clear in HBM
    void clear_kv_cache();
    // the code predictor's 16-position cache per slot is fixed in HBM: n_ctx must be <= 16
    bool init_code_pred_kv_cache(int32_t n_ctx);
    void clear_code_pred_kv_cache();

    // project_text_tokens + speaker row added to every row + forward_prefill (src/tts_transformer.cpp:1922-1950)
    bool forward_text(const int32_t *text_tokens, int32_t n_tokens, const float *speaker_embd, int32_t n_past,
                      std::vector<float> &output);
    // causal forward of n_tokens rows at positions n_past.. (output: hidden rows [n][H]; logits_out: last row's
    // codec logits) (src/tts_transformer.cpp:1829-1920)
    bool forward_prefill(const float *prefill_embd, int32_t n_tokens, int32_t n_past, std::vector<float> &output,
                         std::vector<float> *logits_out = nullptr);
    // one talker step at n_past: output = codec logits [V], hidden_out = final hidden [H] (:1952-2028)
    bool forward_step(const float *step_embd, int32_t n_past, std::vector<float> &output,
                      std::vector<float> *hidden_out = nullptr);
    bool get_hidden_states(std::vector<float> &hidden) const;

    // 15 codes for codebooks 1..15 (src/tts_transformer.cpp:2153-2340; GPU form trt_code_predictor.cpp:484-600)
    bool predict_codes_autoregressive(const float *hidden, int32_t codebook_0_token, std::vector<int32_t> &output,
                                      float temperature = 0.9f, int32_t top_k = 50);

    using frame_callback_t = std::function<bool(const int32_t *, int32_t, int32_t)>;

    // src/tts_transformer.h:233-241; output [n_frames][16] row-major
    bool generate(const int32_t *text_tokens, int32_t n_tokens, const float *speaker_embd, int32_t max_len,
                  std::vector<int32_t> &output, int32_t language_id = 2050, float repetition_penalty = 1.05f,
                  float temperature = 0.9f, int32_t top_k = 50, frame_callback_t on_frames = nullptr,
                  int32_t callback_interval = 40);

    const tts_transformer_config &get_config() const { return config_; }
    const std::string &get_error() const { return error_msg_; }

    // ---- MI355X extensions
    bool set_device(int device);   // before load_model
    void set_seed(uint64_t seed) { seed_ = seed; }
    // n_utt utterances decoded in lock-step on one GPU (SURVEY §8(b) "must add: batched entry points");
    // outputs[u] = [n_frames_u][16]
    bool generate_batch(const std::vector<std::vector<int32_t>> &text_tokens,
                        const std::vector<const float *> &speaker_embds, int32_t max_len,
                        std::vector<std::vector<int32_t>> &outputs, int32_t language_id = 2050,
                        float repetition_penalty = 1.05f, float temperature = 0.9f, int32_t top_k = 50);
    q3t_ctx *handle() const { return ctx_; }

private:
    bool ensure(int32_t slots, int32_t n_ctx);
    bool fail();

    q3t_ctx *ctx_ = nullptr;
    int device_ = 0;
    int32_t slots_ = 0, n_ctx_ = 0;
    uint64_t seed_ = 0;
    int32_t cp_calls_ = 0;   // RNG frame counter of predict_codes_autoregressive
    tts_transformer_config config_;
    std::vector<float> last_hidden_;
    std::string error_msg_;
};

class AudioTokenizerDecoder {
public:
    AudioTokenizerDecoder();
    ~AudioTokenizerDecoder();
    AudioTokenizerDecoder(const AudioTokenizerDecoder &) = delete;
    AudioTokenizerDecoder &operator=(const AudioTokenizerDecoder &) = delete;

    bool load_model(const std::string &model_path);
    void unload_model();
    // whole-utterance decode, codes [n_frames][16] -> samples in [-1, 1] at 24 kHz (:375-879)
    bool decode(const int32_t *codes, int32_t n_frames, std::vector<float> &samples);

    const audio_decoder_config &get_config() const { return config_; }
    const std::string &get_error() const { return error_msg_; }
    bool set_device(int device);

private:
    q3t_ctx *ctx_ = nullptr;
    int device_ = 0;
    audio_decoder_config config_;
    std::string error_msg_;
};

class TRTVocoderDecoder {
public:
    TRTVocoderDecoder();
    ~TRTVocoderDecoder();
    TRTVocoderDecoder(const TRTVocoderDecoder &) = delete;
    TRTVocoderDecoder &operator=(const TRTVocoderDecoder &) = delete;

    // engine_path: the tokenizer GGUF; fixed_frames: chunk length of decode()
    bool load_engine(const std::string &engine_path, int32_t fixed_frames);
    // independent fixed_frames-long chunks, n_frames * 1920 samples (src/trt_vocoder.cpp:98-170)
    bool decode(const int32_t *codes, int32_t n_frames, int32_t n_codebooks, std::vector<float> &samples);

    bool is_loaded() const { return ctx_ != nullptr; }
    const std::string &get_error() const { return error_msg_; }
    int32_t get_fixed_frames() const { return fixed_frames_; }
    void unload();
    bool set_device(int device);

private:
    q3t_ctx *ctx_ = nullptr;
    int device_ = 0;
    int32_t fixed_frames_ = 0;
    std::string error_msg_;
};

// ============================================================================ text tokenizer (src/text_tokenizer.h)
struct tokenizer_config {
    int32_t vocab_size = 151936;
    int32_t pad_token_id = 151643;
    int32_t eos_token_id = 151645;   // <|im_end|>
    int32_t bos_token_id = 151644;   // <|im_start|>
};

class TextTokenizer {
public:
    TextTokenizer();
    ~TextTokenizer();
    TextTokenizer(const TextTokenizer &) = delete;
    TextTokenizer &operator=(const TextTokenizer &) = delete;

    bool load_from_gguf(const std::string &gguf_path);
    std::vector<int32_t> encode(const std::string &text) const;
    // <|im_start|>assistant\n{text}<|im_end|>\n<|im_start|>assistant\n
    std::vector<int32_t> encode_for_tts(const std::string &text) const;
    std::string decode(const std::vector<int32_t> &tokens) const;
    std::string decode_token(int32_t token_id) const;
    const tokenizer_config &get_config() const { return config_; }
    const std::string &get_error() const { return error_msg_; }
    bool is_loaded() const { return tok_ != nullptr; }
    int32_t bos_token_id() const { return config_.bos_token_id; }
    int32_t eos_token_id() const { return config_.eos_token_id; }
    int32_t pad_token_id() const { return config_.pad_token_id; }

private:
    ::q3t_tokenizer *tok_ = nullptr;
    tokenizer_config config_;
    std::string error_msg_;
};

// ================================================================ speaker encoder (src/audio_tokenizer_encoder.h)
struct speaker_encoder_config {
    int32_t sample_rate = 24000;
    int32_t n_mels = 128;
    int32_t n_fft = 1024;
    int32_t hop_length = 256;
    int32_t win_length = 1024;
    int32_t embedding_dim = 1024;
    int32_t hidden_dim = 512;
    int32_t n_res2net_blocks = 3;
    int32_t res2net_scale = 8;
    float f_min = 0.0f;
    float f_max = 12000.0f;
};

class AudioTokenizerEncoder {
public:
    AudioTokenizerEncoder();
    ~AudioTokenizerEncoder();
    AudioTokenizerEncoder(const AudioTokenizerEncoder &) = delete;
    AudioTokenizerEncoder &operator=(const AudioTokenizerEncoder &) = delete;

    // the TTS GGUF; only its spk_enc.* tensors are read
    bool load_model(const std::string &model_path);
    // samples in [-1, 1] at 24 kHz -> embedding [embedding_dim]
    bool encode(const float *samples, int32_t n_samples, std::vector<float> &embedding);
    const speaker_encoder_config &get_config() const { return config_; }
    const std::string &get_error() const { return error_msg_; }
    bool set_device(int device);

private:
    q3t_ctx *ctx_ = nullptr;
    int device_ = 0;
    speaker_encoder_config config_;
    std::string error_msg_;
};

}  // namespace qwen3_tts

#endif
