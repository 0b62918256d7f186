// qwen3_tts_hip.cpp — TTSTransformer / AudioTokenizerDecoder / TRTVocoderDecoder over libq3t.so's C ABI.
// See qwen3_tts_hip.h for the reference interfaces mirrored and the deliberate differences.
#include "qwen3_tts_hip.h"

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "q3t_backend.h"

namespace qwen3_tts {

namespace {

// reference generate(): n_ctx = prefill_len + max_len + 8 (src/tts_transformer.cpp:2383), prefill_len = 10 with a
// speaker row (9 without, :1093-1231)
constexpr int32_t kPrefillLen = 10;
constexpr int32_t kDefaultMaxLen = 4096;   // tts_params::max_audio_tokens (src/qwen3_tts.h:20)

std::string last_error() {
    const char *e = q3t_last_error();
    return e && *e ? std::string(e) : std::string("unknown error");
}

int frame_trampoline(void *user, int32_t /*utterance*/, const int32_t *codes, int32_t n_frames, int32_t n_codebooks) {
    auto *f = static_cast<TTSTransformer::frame_callback_t *>(user);
    try {
        return (*f)(codes, n_frames, n_codebooks) ? 1 : 0;
    } catch (...) {
        return 0;   // an exception in the caller's callback stops the utterance; nothing unwinds through the C ABI
    }
}

q3t_gen_params gen_params(int32_t max_len, int32_t language_id, float repetition_penalty, float temperature,
                          int32_t top_k, uint64_t seed) {
    q3t_gen_params p;
    q3t_default_params(&p);
    p.max_len = max_len;
    p.language_id = language_id;
    p.repetition_penalty = repetition_penalty;
    p.temperature = temperature;
    p.top_k = top_k;
    p.seed = seed;
    p.force_frames = 0;
    return p;
}

}  // namespace

// ============================================================================================ TTSTransformer

TTSTransformer::TTSTransformer() = default;
TTSTransformer::~TTSTransformer() { unload_model(); }

bool TTSTransformer::fail() {
    error_msg_ = last_error();
    return false;
}

bool TTSTransformer::set_device(int device) {
    if (ctx_) { error_msg_ = "set_device must precede load_model"; return false; }
    device_ = device;
    return true;
}

bool TTSTransformer::load_model(const std::string &model_path) {
    unload_model();
    const int32_t n_ctx = kPrefillLen + kDefaultMaxLen + 8;
    if (q3t_ctx_create(model_path.c_str(), nullptr, device_, 1, n_ctx, &ctx_) != Q3T_OK) {
        ctx_ = nullptr;
        return fail();
    }
    slots_ = 1;
    n_ctx_ = n_ctx;
    q3t_config c;
    if (q3t_get_config(ctx_, &c) != Q3T_OK) return fail();
    config_ = tts_transformer_config();
    config_.text_vocab_size = c.text_vocab;
    config_.text_embd_dim = c.text_dim;
    config_.hidden_size = c.hidden;
    config_.n_layers = c.n_layers;
    config_.n_attention_heads = c.n_heads;
    config_.n_key_value_heads = c.n_kv_heads;
    config_.intermediate_size = c.intermediate;
    config_.head_dim = c.head_dim;
    config_.codec_vocab_size = c.codec_vocab;
    config_.n_codebooks = c.n_codebooks;
    config_.code_pred_layers = c.cp_layers;
    config_.code_pred_vocab_size = c.cp_vocab;
    config_.codec_eos_id = c.codec_eos;
    cp_calls_ = 0;
    error_msg_.clear();
    return true;
}

void TTSTransformer::unload_model() {
    if (ctx_) q3t_ctx_destroy(ctx_);
    ctx_ = nullptr;
    slots_ = n_ctx_ = 0;
    last_hidden_.clear();
}

// grow the context (slots / positions) by re-laying it out from the resident weights: device-to-device copy of
// the weight blobs, no file reads (q3t_ctx_create_replica)
bool TTSTransformer::ensure(int32_t slots, int32_t n_ctx) {
    if (!ctx_) { error_msg_ = "Model not loaded"; return false; }
    if (slots <= slots_ && n_ctx <= n_ctx_) return true;
    q3t_ctx *grown = nullptr;
    const int32_t s = std::max(slots, slots_), n = std::max(n_ctx, n_ctx_);
    if (q3t_ctx_create_replica(ctx_, device_, s, n, &grown) != Q3T_OK) return fail();
    q3t_ctx_destroy(ctx_);
    ctx_ = grown;
    slots_ = s;
    n_ctx_ = n;
    return true;
}

bool TTSTransformer::init_kv_cache(int32_t n_ctx) {
    if (n_ctx <= 0) { error_msg_ = "n_ctx must be > 0"; return false; }
    return ensure(1, n_ctx);
}

void TTSTransformer::clear_kv_cache() {}

bool TTSTransformer::init_code_pred_kv_cache(int32_t n_ctx) {
    if (n_ctx <= 0 || n_ctx > 16) { error_msg_ = "code predictor n_ctx must be in [1, 16]"; return false; }
    return ctx_ ? true : (error_msg_ = "Model not loaded", false);
}

void TTSTransformer::clear_code_pred_kv_cache() {}

bool TTSTransformer::forward_text(const int32_t *text_tokens, int32_t n_tokens, const float *speaker_embd,
                                  int32_t n_past, std::vector<float> &output) {
    if (!text_tokens) { error_msg_ = "text_tokens is null"; return false; }
    if (n_tokens <= 0) { error_msg_ = "n_tokens must be > 0"; return false; }
    if (!ctx_) { error_msg_ = "Model not loaded"; return false; }
    const int32_t H = config_.hidden_size;
    std::vector<float> projected((size_t)n_tokens * H);
    if (q3t_project_text(ctx_, n_tokens, text_tokens, projected.data()) != Q3T_OK) return fail();
    if (speaker_embd)
        for (int32_t t = 0; t < n_tokens; ++t)
            for (int32_t h = 0; h < H; ++h) projected[(size_t)t * H + h] += speaker_embd[h];
    return forward_prefill(projected.data(), n_tokens, n_past, output, nullptr);
}

bool TTSTransformer::forward_prefill(const float *prefill_embd, int32_t n_tokens, int32_t n_past,
                                     std::vector<float> &output, std::vector<float> *logits_out) {
    if (!ctx_) { error_msg_ = "Model not loaded"; return false; }
    if (!prefill_embd || n_tokens <= 0 || n_past < 0) { error_msg_ = "invalid prefill arguments"; return false; }
    if (!ensure(1, n_past + n_tokens)) return false;
    const int32_t H = config_.hidden_size;
    output.resize((size_t)n_tokens * H);
    if (logits_out) logits_out->resize(config_.codec_vocab_size);
    if (n_past == 0 && n_tokens <= 10) {
        // the causal prefill pass (every row equals the single-slot decode step replayed at its position)
        std::vector<float> lg(config_.codec_vocab_size);
        if (q3t_talker_prefill(ctx_, 1, n_tokens, prefill_embd, 1, output.data(), lg.data()) != Q3T_OK) return fail();
        if (logits_out) *logits_out = lg;
        last_hidden_.assign(output.end() - H, output.end());
        return true;
    }
    // longer or continued prompts: row i attends to positions <= n_past + i, the decode step replayed row by row
    for (int32_t i = 0; i < n_tokens; ++i) {
        const int32_t pos = n_past + i;
        float *lg = (logits_out && i == n_tokens - 1) ? logits_out->data() : nullptr;
        if (q3t_talker_forward(ctx_, 1, prefill_embd + (size_t)i * H, &pos, output.data() + (size_t)i * H, lg) != Q3T_OK)
            return fail();
    }
    last_hidden_.assign(output.end() - H, output.end());
    return true;
}

bool TTSTransformer::forward_step(const float *step_embd, int32_t n_past, std::vector<float> &output,
                                  std::vector<float> *hidden_out) {
    if (!ctx_) { error_msg_ = "Model not loaded"; return false; }
    if (!step_embd) { error_msg_ = "step_embd is null"; return false; }
    if (n_past < 0) { error_msg_ = "n_past must be >= 0"; return false; }
    if (!ensure(1, n_past + 1)) return false;
    const int32_t H = config_.hidden_size;
    output.resize(config_.codec_vocab_size);
    last_hidden_.resize(H);
    if (q3t_talker_forward(ctx_, 1, step_embd, &n_past, last_hidden_.data(), output.data()) != Q3T_OK) return fail();
    if (hidden_out) *hidden_out = last_hidden_;
    return true;
}

bool TTSTransformer::get_hidden_states(std::vector<float> &hidden) const {
    if (last_hidden_.empty()) return false;
    hidden = last_hidden_;
    return true;
}

bool TTSTransformer::predict_codes_autoregressive(const float *hidden, int32_t codebook_0_token,
                                                  std::vector<int32_t> &output, float temperature, int32_t top_k) {
    if (!ctx_) { error_msg_ = "Model not loaded"; return false; }
    if (!hidden) { error_msg_ = "hidden is null"; return false; }
    output.resize(15);
    if (q3t_codepred_frame(ctx_, 1, hidden, &codebook_0_token, temperature, top_k, seed_, cp_calls_++, output.data(),
                           nullptr) != Q3T_OK)
        return fail();
    return true;
}

bool TTSTransformer::generate(const int32_t *text_tokens, int32_t n_tokens, const float *speaker_embd, int32_t max_len,
                              std::vector<int32_t> &output, int32_t language_id, float repetition_penalty,
                              float temperature, int32_t top_k, frame_callback_t on_frames,
                              int32_t callback_interval) {
    output.clear();
    if (!ctx_) { error_msg_ = "Model not loaded"; return false; }
    if (!text_tokens || n_tokens <= 0) { error_msg_ = "text_tokens is null or empty"; return false; }
    if (max_len <= 0) return true;
    if (!ensure(1, kPrefillLen + max_len + 8)) return false;
    const q3t_gen_params p = gen_params(max_len, language_id, repetition_penalty, temperature, top_k, seed_);
    std::vector<int32_t> codes((size_t)max_len * 16);
    int32_t n_frames = 0;
    const float *spk[1] = {speaker_embd};
    const int32_t *toks[1] = {text_tokens};
    int rc;
    if (on_frames) {
        if (callback_interval <= 0) { error_msg_ = "callback_interval must be > 0"; return false; }
        rc = q3t_generate_stream(ctx_, 1, toks, &n_tokens, speaker_embd ? spk : nullptr, &p, codes.data(), &n_frames,
                                 frame_trampoline, &on_frames, callback_interval);
    } else {
        rc = q3t_generate(ctx_, 1, toks, &n_tokens, speaker_embd ? spk : nullptr, &p, codes.data(), &n_frames);
    }
    if (rc != Q3T_OK) return fail();
    output.assign(codes.begin(), codes.begin() + (size_t)n_frames * 16);
    return true;
}

bool TTSTransformer::generate_batch(const std::vector<std::vector<int32_t>> &text_tokens,
                                    const std::vector<const float *> &speaker_embds, int32_t max_len,
                                    std::vector<std::vector<int32_t>> &outputs, int32_t language_id,
                                    float repetition_penalty, float temperature, int32_t top_k) {
    const int32_t n = (int32_t)text_tokens.size();
    outputs.assign(n, {});
    if (!ctx_) { error_msg_ = "Model not loaded"; return false; }
    if (n == 0 || max_len <= 0) return true;
    if (!speaker_embds.empty() && (int32_t)speaker_embds.size() != n) {
        error_msg_ = "speaker_embds must be empty or hold one entry per utterance";
        return false;
    }
    if (!ensure(n, kPrefillLen + max_len + 8)) return false;
    std::vector<const int32_t *> toks(n);
    std::vector<int32_t> n_toks(n), n_frames(n);
    for (int32_t u = 0; u < n; ++u) {
        if (text_tokens[u].empty()) { error_msg_ = "empty token list"; return false; }
        toks[u] = text_tokens[u].data();
        n_toks[u] = (int32_t)text_tokens[u].size();
    }
    const q3t_gen_params p = gen_params(max_len, language_id, repetition_penalty, temperature, top_k, seed_);
    std::vector<int32_t> codes((size_t)n * max_len * 16);
    if (q3t_generate(ctx_, n, toks.data(), n_toks.data(), speaker_embds.empty() ? nullptr : speaker_embds.data(), &p,
                     codes.data(), n_frames.data()) != Q3T_OK)
        return fail();
    for (int32_t u = 0; u < n; ++u) {
        const int32_t *c = codes.data() + (size_t)u * max_len * 16;
        outputs[u].assign(c, c + (size_t)n_frames[u] * 16);
    }
    return true;
}

// ===================================================================================== AudioTokenizerDecoder

AudioTokenizerDecoder::AudioTokenizerDecoder() = default;
AudioTokenizerDecoder::~AudioTokenizerDecoder() { unload_model(); }

bool AudioTokenizerDecoder::set_device(int device) {
    if (ctx_) { error_msg_ = "set_device must precede load_model"; return false; }
    device_ = device;
    return true;
}

bool AudioTokenizerDecoder::load_model(const std::string &model_path) {
    unload_model();
    if (q3t_ctx_create(nullptr, model_path.c_str(), device_, 1, 32, &ctx_) != Q3T_OK) {
        ctx_ = nullptr;
        error_msg_ = last_error();
        return false;
    }
    error_msg_.clear();
    return true;
}

void AudioTokenizerDecoder::unload_model() {
    if (ctx_) q3t_ctx_destroy(ctx_);
    ctx_ = nullptr;
}

bool AudioTokenizerDecoder::decode(const int32_t *codes, int32_t n_frames, std::vector<float> &samples) {
    if (!ctx_) { error_msg_ = "Model not loaded"; return false; }
    if (!codes || n_frames <= 0) { error_msg_ = "no codes to decode"; return false; }
    const int64_t n = q3t_vocoder_num_samples(ctx_, n_frames, Q3T_VOCODER_FULL);
    if (n < 0) { error_msg_ = last_error(); return false; }
    samples.resize((size_t)n);
    int64_t got = 0;
    if (q3t_vocoder_decode(ctx_, codes, n_frames, Q3T_VOCODER_FULL, samples.data(), &got) != Q3T_OK) {
        error_msg_ = last_error();
        return false;
    }
    samples.resize((size_t)got);
    return true;
}

// ========================================================================================= TRTVocoderDecoder

TRTVocoderDecoder::TRTVocoderDecoder() = default;
TRTVocoderDecoder::~TRTVocoderDecoder() { unload(); }

bool TRTVocoderDecoder::set_device(int device) {
    if (ctx_) { error_msg_ = "set_device must precede load_engine"; return false; }
    device_ = device;
    return true;
}

bool TRTVocoderDecoder::load_engine(const std::string &engine_path, int32_t fixed_frames) {
    unload();
    if (fixed_frames <= 0) { error_msg_ = "fixed_frames must be > 0"; return false; }
    // the reference passes a TensorRT plan (<model_dir>/vocoder_decoder_<n>.trt, qwen3_tts.cpp:171-188): there is no
    // TensorRT on MI355X, so a path that is not a GGUF resolves to the tokenizer GGUF next to it
    std::string gguf = engine_path;
    char magic[4] = {0};
    FILE *f = std::fopen(engine_path.c_str(), "rb");
    const bool is_gguf = f && std::fread(magic, 1, 4, f) == 4 && std::memcmp(magic, "GGUF", 4) == 0;
    if (f) std::fclose(f);
    if (!is_gguf) {
        const size_t slash = engine_path.find_last_of('/');
        gguf = (slash == std::string::npos ? std::string(".") : engine_path.substr(0, slash)) +
               "/qwen3-tts-tokenizer-f16.gguf";
    }
    if (q3t_ctx_create(nullptr, gguf.c_str(), device_, 1, 32, &ctx_) != Q3T_OK) {
        ctx_ = nullptr;
        error_msg_ = last_error();
        return false;
    }
    fixed_frames_ = fixed_frames;
    error_msg_.clear();
    return true;
}

void TRTVocoderDecoder::unload() {
    if (ctx_) q3t_ctx_destroy(ctx_);
    ctx_ = nullptr;
    fixed_frames_ = 0;
}

bool TRTVocoderDecoder::decode(const int32_t *codes, int32_t n_frames, int32_t n_codebooks,
                               std::vector<float> &samples) {
    if (!ctx_) { error_msg_ = "Engine not loaded"; return false; }
    if (!codes || n_frames <= 0) { error_msg_ = "no codes to decode"; return false; }
    samples.resize((size_t)n_frames * 1920);
    int64_t got = 0;
    if (q3t_vocoder_decode_chunked(ctx_, codes, n_frames, n_codebooks, fixed_frames_, samples.data(), &got) != Q3T_OK) {
        error_msg_ = last_error();
        return false;
    }
    samples.resize((size_t)got);
    return true;
}

// ================================================================================================ TextTokenizer

TextTokenizer::TextTokenizer() = default;
TextTokenizer::~TextTokenizer() {
    if (tok_) q3t_tokenizer_free(tok_);
}

bool TextTokenizer::load_from_gguf(const std::string &gguf_path) {
    if (tok_) { q3t_tokenizer_free(tok_); tok_ = nullptr; }
    if (q3t_tokenizer_load(gguf_path.c_str(), &tok_) != Q3T_OK) {
        tok_ = nullptr;
        error_msg_ = last_error();
        return false;
    }
    q3t_tokenizer_info(tok_, &config_.vocab_size, &config_.bos_token_id, &config_.eos_token_id, &config_.pad_token_id);
    return true;
}

std::vector<int32_t> TextTokenizer::encode(const std::string &text) const {
    std::vector<int32_t> ids;
    int32_t n = 0;
    if (!tok_ || q3t_tokenizer_encode(tok_, text.data(), (int64_t)text.size(), 0, nullptr, 0, &n) != Q3T_OK) return ids;
    ids.resize(n);
    if (n > 0 && q3t_tokenizer_encode(tok_, text.data(), (int64_t)text.size(), 0, ids.data(), n, &n) != Q3T_OK) ids.clear();
    return ids;
}

std::vector<int32_t> TextTokenizer::encode_for_tts(const std::string &text) const {
    std::vector<int32_t> ids;
    int32_t n = 0;
    if (!tok_ || q3t_tokenizer_encode(tok_, text.data(), (int64_t)text.size(), 1, nullptr, 0, &n) != Q3T_OK) return ids;
    ids.resize(n);
    if (q3t_tokenizer_encode(tok_, text.data(), (int64_t)text.size(), 1, ids.data(), n, &n) != Q3T_OK) ids.clear();
    return ids;
}

std::string TextTokenizer::decode(const std::vector<int32_t> &tokens) const {
    if (!tok_) return "";
    int64_t nb = 0;
    if (q3t_tokenizer_decode(tok_, tokens.data(), (int32_t)tokens.size(), nullptr, 0, &nb) != Q3T_OK) return "";
    std::string s((size_t)nb, '\0');
    if (nb > 0 && q3t_tokenizer_decode(tok_, tokens.data(), (int32_t)tokens.size(), &s[0], nb, &nb) != Q3T_OK) return "";
    return s;
}

std::string TextTokenizer::decode_token(int32_t token_id) const { return decode(std::vector<int32_t>{token_id}); }

// ======================================================================================= AudioTokenizerEncoder

AudioTokenizerEncoder::AudioTokenizerEncoder() = default;
AudioTokenizerEncoder::~AudioTokenizerEncoder() {
    if (ctx_) q3t_ctx_destroy(ctx_);
}

bool AudioTokenizerEncoder::set_device(int device) {
    if (ctx_) { error_msg_ = "set_device must precede load_model"; return false; }
    device_ = device;
    return true;
}

bool AudioTokenizerEncoder::load_model(const std::string &model_path) {
    if (ctx_) { q3t_ctx_destroy(ctx_); ctx_ = nullptr; }
    if (q3t_ctx_create_speaker(model_path.c_str(), device_, &ctx_) != Q3T_OK) {
        ctx_ = nullptr;
        error_msg_ = last_error();
        return false;
    }
    config_.embedding_dim = q3t_speaker_dim(ctx_);
    return true;
}

bool AudioTokenizerEncoder::encode(const float *samples, int32_t n_samples, std::vector<float> &embedding) {
    if (!ctx_) { error_msg_ = "Model not loaded"; return false; }
    embedding.resize(config_.embedding_dim);
    if (q3t_speaker_encode(ctx_, samples, n_samples, embedding.data()) != Q3T_OK) {
        error_msg_ = last_error();
        return false;
    }
    return true;
}

}  // namespace qwen3_tts
