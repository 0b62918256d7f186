// qwen3_tts_pipeline.cpp — TextTokenizer, AudioTokenizerEncoder, Qwen3TTS and the WAV helpers of qwen3_tts_hip.h.
//
// Qwen3TTS drives ONE q3t context (talker + code predictor + vocoder + speaker encoder resident in HBM) the way
// src/qwen3_tts.cpp drives its four components: tokenize -> generate (optionally streaming chunked vocoder decodes
// from the frame callback) -> whole-utterance vocoder, with the same timing / RTF / memory report on stderr.
#include <sys/resource.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "q3t_backend.h"
#include "qwen3_tts_pipeline.h"

namespace qwen3_tts {

namespace {

int64_t now_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

std::string q3t_error() {
    const char *e = q3t_last_error();
    return e && *e ? std::string(e) : std::string("unknown error");
}

// process memory as the reference samples it on Linux: getrusage max RSS for both figures (qwen3_tts.cpp:29-57)
bool rss_bytes(uint64_t &rss) {
    struct rusage u = {};
    if (getrusage(RUSAGE_SELF, &u) != 0) return false;
    rss = (uint64_t)u.ru_maxrss * 1024ULL;
    return true;
}

std::string format_bytes(uint64_t bytes) {   // qwen3_tts.cpp:59-70
    static const char *units[] = {"B", "KB", "MB", "GB", "TB"};
    double v = (double)bytes;
    int u = 0;
    while (v >= 1024.0 && u < 4) { v /= 1024.0; ++u; }
    char b[64];
    snprintf(b, sizeof b, "%.2f %s", v, units[u]);
    return b;
}

void log_memory(const char *label) {
    uint64_t r = 0;
    if (!rss_bytes(r)) { fprintf(stderr, "  [mem] %-24s unavailable\n", label); return; }
    fprintf(stderr, "  [mem] %-24s rss=%s  phys=%s\n", label, format_bytes(r).c_str(), format_bytes(r).c_str());
}

struct MemSampler {
    tts_result &r;
    bool print;
    void operator()(const char *stage) const {
        uint64_t m = 0;
        if (!rss_bytes(m)) return;
        if (r.mem_rss_start_bytes == 0) { r.mem_rss_start_bytes = m; r.mem_phys_start_bytes = m; }
        r.mem_rss_end_bytes = m;
        r.mem_phys_end_bytes = m;
        r.mem_rss_peak_bytes = std::max(r.mem_rss_peak_bytes, m);
        r.mem_phys_peak_bytes = std::max(r.mem_phys_peak_bytes, m);
        if (print) fprintf(stderr, "  [mem] %-24s rss=%s  phys=%s\n", stage, format_bytes(m).c_str(), format_bytes(m).c_str());
    }
};

// Timing / RTF / memory report, format of qwen3_tts.cpp:536-561
void print_report(const tts_result &r) {
    const double audio_sec = r.sample_rate > 0 ? (double)r.audio.size() / (double)r.sample_rate : 0.0;
    const double wall_sec = (double)r.t_total_ms / 1000.0;
    const double rtf = audio_sec > 0.0 ? wall_sec / audio_sec : 0.0;
    const double xrt = wall_sec > 0.0 ? audio_sec / wall_sec : 0.0;
    fprintf(stderr, "\nTiming:\n");
    fprintf(stderr, "  Tokenization:    %lld ms\n", (long long)r.t_tokenize_ms);
    fprintf(stderr, "  Speaker encode:  %lld ms\n", (long long)r.t_encode_ms);
    fprintf(stderr, "  Code generation: %lld ms\n", (long long)r.t_generate_ms);
    fprintf(stderr, "  Vocoder decode:  %lld ms\n", (long long)r.t_decode_ms);
    fprintf(stderr, "  Total:           %lld ms\n", (long long)r.t_total_ms);
    fprintf(stderr, "  Audio duration:  %.2f s\n", audio_sec);
    fprintf(stderr, "  Throughput:      %.2fx realtime (RTF=%.3f)\n", xrt, rtf);
    fprintf(stderr, "\nMemory:\n");
    fprintf(stderr, "  RSS start/end:   %s -> %s\n", format_bytes(r.mem_rss_start_bytes).c_str(),
            format_bytes(r.mem_rss_end_bytes).c_str());
    fprintf(stderr, "  RSS peak:        %s\n", format_bytes(r.mem_rss_peak_bytes).c_str());
    fprintf(stderr, "  Phys start/end:  %s -> %s\n", format_bytes(r.mem_phys_start_bytes).c_str(),
            format_bytes(r.mem_phys_end_bytes).c_str());
    fprintf(stderr, "  Phys peak:       %s\n", format_bytes(r.mem_phys_peak_bytes).c_str());
}

bool file_exists(const std::string &p) {
    FILE *f = fopen(p.c_str(), "rb");
    if (!f) return false;
    fclose(f);
    return true;
}

constexpr int32_t kPrefillLen = 10;   // prefill rows with a speaker row (tts_transformer.cpp:1093-1231)
constexpr int32_t kSampleRate = 24000;

struct StreamState {
    q3t_ctx *ctx = nullptr;
    int32_t chunk = 0;
    std::vector<float> *audio = nullptr;
    int64_t decode_ms = 0;
    bool error = false;
    std::string error_msg;
};

// generate_stream callback: decode each delivered chunk with the chunked vocoder (qwen3_tts.cpp:437-453)
int stream_cb(void *user, int32_t /*utt*/, const int32_t *codes, int32_t n_frames, int32_t n_cb) {
    auto *s = static_cast<StreamState *>(user);
    const int64_t t0 = now_ms();
    std::vector<float> pcm((size_t)n_frames * 1920);
    int64_t got = 0;
    if (q3t_vocoder_decode_chunked(s->ctx, codes, n_frames, n_cb, s->chunk, pcm.data(), &got) != Q3T_OK) {
        s->error = true;
        s->error_msg = q3t_error();
        return 0;
    }
    s->audio->insert(s->audio->end(), pcm.begin(), pcm.begin() + got);
    s->decode_ms += now_ms() - t0;
    return 1;
}

}  // namespace

// ===================================================================================================== Qwen3TTS

Qwen3TTS::Qwen3TTS() = default;
Qwen3TTS::~Qwen3TTS() {
    if (ctx_) q3t_ctx_destroy(ctx_);
}

bool Qwen3TTS::set_device(int device) {
    if (ctx_) { error_msg_ = "set_device must precede load_models"; return false; }
    device_ = device;
    return true;
}

bool Qwen3TTS::load_models(const std::string &model_dir) {
    const int64_t t_start = now_ms();
    log_memory("load/start");
    if (ctx_) { q3t_ctx_destroy(ctx_); ctx_ = nullptr; }
    models_loaded_ = false;
    tts_model_path_ = model_dir + "/qwen3-tts-0.6b-f16.gguf";
    decoder_model_path_ = model_dir + "/qwen3-tts-tokenizer-f16.gguf";
    const char *low = std::getenv("QWEN3_TTS_LOW_MEM");
    if (low && low[0] != '\0' && low[0] != '0')
        fprintf(stderr, "  Low-memory mode requested: ignored (all models stay resident in HBM)\n");
    fprintf(stderr, "Loading TTS model from %s...\n", tts_model_path_.c_str());
    const int64_t t_tok = now_ms();
    if (!tokenizer_.load_from_gguf(tts_model_path_)) {
        error_msg_ = "Failed to load text tokenizer: " + tokenizer_.get_error();
        return false;
    }
    fprintf(stderr, "  Text tokenizer loaded: vocab_size=%d (%lld ms)\n", tokenizer_.get_config().vocab_size,
            (long long)(now_ms() - t_tok));
    log_memory("load/after-tokenizer");
    // vocoder choice in the reference's order (qwen3_tts.cpp:168-218): a chunked "TRT" engine file if present
    if (vocoder_chunk_ == 0) {
        if (file_exists(model_dir + "/vocoder_decoder_40.trt")) vocoder_chunk_ = 40;
        else if (file_exists(model_dir + "/vocoder_decoder_30.trt")) vocoder_chunk_ = 30;
        else if (file_exists(model_dir + "/vocoder_decoder_fixed.trt")) vocoder_chunk_ = 20;
    }
    const int64_t t_model = now_ms();
    slots_ = 1;
    n_ctx_ = kPrefillLen + 4096 + 8;
    if (q3t_ctx_create(tts_model_path_.c_str(), decoder_model_path_.c_str(), device_, slots_, n_ctx_, &ctx_) != Q3T_OK) {
        ctx_ = nullptr;
        error_msg_ = "Failed to load TTS transformer: " + q3t_error();
        return false;
    }
    q3t_config c;
    q3t_get_config(ctx_, &c);
    hidden_ = c.hidden;
    fprintf(stderr, "  TTS transformer loaded: hidden_size=%d, n_layers=%d (%lld ms)\n", c.hidden, c.n_layers,
            (long long)(now_ms() - t_model));
    if (vocoder_chunk_ > 0)
        fprintf(stderr, "  Chunked vocoder ready: %d fixed frames (%.1f s max per chunk)\n", vocoder_chunk_,
                vocoder_chunk_ / 12.5f);
    else
        fprintf(stderr, "  Vocoder loaded: sample_rate=%d, n_codebooks=%d\n", c.sample_rate, c.n_codebooks);
    if (q3t_speaker_dim(ctx_) > 0) fprintf(stderr, "  Speaker encoder: resident (dim %d)\n", q3t_speaker_dim(ctx_));
    models_loaded_ = true;
    fprintf(stderr, "All models loaded in %lld ms\n", (long long)(now_ms() - t_start));
    log_memory("load/end");
    return true;
}

bool Qwen3TTS::ensure_slots(int32_t slots, int32_t max_len) {
    const int32_t n_ctx = kPrefillLen + max_len + 8;
    if (slots <= slots_ && n_ctx <= n_ctx_) return true;
    q3t_ctx *grown = nullptr;
    const int32_t s = std::max(slots, slots_), n = std::max(n_ctx, n_ctx_);
    if (q3t_ctx_create_replica(ctx_, device_, s, n, &grown) != Q3T_OK) { error_msg_ = q3t_error(); return false; }
    q3t_ctx_destroy(ctx_);
    ctx_ = grown;
    slots_ = s;
    n_ctx_ = n;
    return true;
}

tts_result Qwen3TTS::synthesize(const std::string &text, const tts_params &params) {
    tts_result result;
    if (!models_loaded_) { result.error_msg = "Models not loaded"; return result; }
    // a zero speaker row, not an absent one (qwen3_tts.cpp:241-245)
    std::vector<float> zero(hidden_, 0.0f);
    return synthesize_internal(text, zero.data(), params, result);
}

tts_result Qwen3TTS::synthesize_with_voice(const std::string &text, const std::string &reference_audio,
                                           const tts_params &params) {
    tts_result result;
    std::vector<float> ref;
    int sr = 0;
    if (!load_audio_file(reference_audio, ref, sr)) {
        result.error_msg = "Failed to load reference audio: " + reference_audio;
        return result;
    }
    if (sr != kSampleRate) {
        fprintf(stderr, "Resampling audio from %d Hz to %d Hz...\n", sr, kSampleRate);
        std::vector<float> rs;
        resample_linear(ref.data(), (int)ref.size(), sr, rs, kSampleRate);
        ref.swap(rs);
    }
    return synthesize_with_voice(text, ref.data(), (int32_t)ref.size(), params);
}

tts_result Qwen3TTS::synthesize_with_voice(const std::string &text, const float *ref_samples, int32_t n_ref_samples,
                                           const tts_params &params) {
    tts_result result;
    if (!models_loaded_) { result.error_msg = "Models not loaded"; return result; }
    const int32_t dim = q3t_speaker_dim(ctx_);
    if (dim <= 0) { result.error_msg = "Failed to load speaker encoder: No speaker encoder tensors found in model"; return result; }
    const int64_t t0 = now_ms();
    std::vector<float> emb(dim);
    if (q3t_speaker_encode(ctx_, ref_samples, n_ref_samples, emb.data()) != Q3T_OK) {
        result.error_msg = "Failed to extract speaker embedding: " + q3t_error();
        return result;
    }
    result.t_encode_ms = now_ms() - t0;
    if (params.print_progress) fprintf(stderr, "Speaker embedding extracted: %zu floats\n", emb.size());
    return synthesize_internal(text, emb.data(), params, result);
}

bool Qwen3TTS::encode_speaker(const std::string &reference_audio, std::vector<float> &embedding) {
    if (!models_loaded_) { error_msg_ = "Models not loaded"; return false; }
    std::vector<float> ref;
    int sr = 0;
    if (!load_audio_file(reference_audio, ref, sr)) {
        error_msg_ = "Failed to load reference audio: " + reference_audio;
        return false;
    }
    if (sr != kSampleRate) {
        std::vector<float> rs;
        resample_linear(ref.data(), (int)ref.size(), sr, rs, kSampleRate);
        ref.swap(rs);
    }
    const int32_t dim = q3t_speaker_dim(ctx_);
    if (dim <= 0) { error_msg_ = "Failed to load speaker encoder: No speaker encoder tensors found in model"; return false; }
    embedding.resize(dim);
    if (q3t_speaker_encode(ctx_, ref.data(), (int32_t)ref.size(), embedding.data()) != Q3T_OK) {
        error_msg_ = "Failed to extract speaker embedding: " + q3t_error();
        return false;
    }
    return true;
}

tts_result Qwen3TTS::synthesize_with_embedding(const std::string &text, const std::vector<float> &speaker_embedding,
                                               const tts_params &params) {
    tts_result result;
    if (!models_loaded_) { result.error_msg = "Models not loaded"; return result; }
    return synthesize_internal(text, speaker_embedding.data(), params, result);
}

tts_result Qwen3TTS::synthesize_internal(const std::string &text, const float *speaker_embedding,
                                         const tts_params &params, tts_result &result) {
    const int64_t t_total = now_ms();
    MemSampler mem{result, params.print_timing};
    mem("synth/start");
    const int64_t t_tok = now_ms();
    std::vector<int32_t> tokens = tokenizer_.encode_for_tts(text);
    result.t_tokenize_ms = now_ms() - t_tok;
    mem("synth/after-tokenize");
    if (tokens.empty()) { result.error_msg = "Failed to tokenize text"; return result; }
    if (params.print_progress) {
        fprintf(stderr, "Text tokenized: %zu tokens\n", tokens.size());
        fprintf(stderr, "  Tokens: ");
        for (size_t i = 0; i < std::min(tokens.size(), (size_t)10); ++i) fprintf(stderr, "%d ", tokens[i]);
        if (tokens.size() > 10) fprintf(stderr, "...");
        fprintf(stderr, "\n");
    }
    const int64_t t_gen = now_ms();
    const int32_t max_len = std::max(params.max_audio_tokens, 0);
    if (!ensure_slots(1, std::max(max_len, 1))) { result.error_msg = "Failed to generate speech codes: " + error_msg_; return result; }
    q3t_gen_params p;
    q3t_default_params(&p);
    p.max_len = max_len;
    p.language_id = 2050;
    p.repetition_penalty = params.repetition_penalty;
    p.temperature = params.temperature;
    p.top_k = params.top_k;
    p.seed = seed_;
    std::vector<int32_t> codes((size_t)std::max(max_len, 1) * 16);
    int32_t n_frames = 0, n_tok = (int32_t)tokens.size();
    const int32_t *tok_ptr[1] = {tokens.data()};
    const float *spk[1] = {speaker_embedding};
    StreamState st;
    st.ctx = ctx_;
    st.chunk = vocoder_chunk_;
    st.audio = &result.audio;
    int rc;
    if (max_len == 0) rc = Q3T_OK;
    else if (vocoder_chunk_ > 0)
        rc = q3t_generate_stream(ctx_, 1, tok_ptr, &n_tok, speaker_embedding ? spk : nullptr, &p, codes.data(),
                                 &n_frames, stream_cb, &st, 40);
    else
        rc = q3t_generate(ctx_, 1, tok_ptr, &n_tok, speaker_embedding ? spk : nullptr, &p, codes.data(), &n_frames);
    if (rc != Q3T_OK) { result.error_msg = "Failed to generate speech codes: " + q3t_error(); return result; }
    if (st.error) { result.error_msg = "TRT vocoder decode failed: " + st.error_msg; return result; }
    result.t_generate_ms = now_ms() - t_gen;
    mem("synth/after-generate");
    if (params.print_progress) fprintf(stderr, "Speech codes generated: %d frames x %d codebooks\n", n_frames, 16);
    if (n_frames == 0) { result.error_msg = "No speech codes generated"; return result; }
    const int64_t t_dec = now_ms();
    if (vocoder_chunk_ <= 0) {
        const int64_t n = q3t_vocoder_num_samples(ctx_, n_frames, Q3T_VOCODER_FULL);
        result.audio.resize((size_t)std::max<int64_t>(n, 0));
        int64_t got = 0;
        if (n < 0 || q3t_vocoder_decode(ctx_, codes.data(), n_frames, Q3T_VOCODER_FULL, result.audio.data(), &got) != Q3T_OK) {
            result.error_msg = "Failed to decode speech codes: " + q3t_error();
            return result;
        }
        result.audio.resize((size_t)got);
    }
    result.sample_rate = kSampleRate;
    result.t_decode_ms = st.decode_ms + (now_ms() - t_dec);
    mem("synth/after-decode");
    result.success = true;
    result.t_total_ms = now_ms() - t_total;
    mem("synth/end");
    if (params.print_timing) print_report(result);
    return result;
}

std::vector<tts_result> Qwen3TTS::synthesize_batch(const std::vector<std::string> &texts,
                                                   const std::vector<std::vector<float>> &speaker_embeddings,
                                                   const tts_params &params) {
    const int32_t n = (int32_t)texts.size();
    std::vector<tts_result> out(n);
    auto fail_all = [&](const std::string &m) {
        for (auto &r : out) r.error_msg = m;
        return out;
    };
    if (!models_loaded_) return fail_all("Models not loaded");
    if (n == 0) return out;
    if (!speaker_embeddings.empty() && (int32_t)speaker_embeddings.size() != n)
        return fail_all("speaker_embeddings must be empty or hold one entry per text");
    const int64_t t0 = now_ms();
    std::vector<std::vector<int32_t>> toks(n);
    std::vector<const int32_t *> tp(n);
    std::vector<int32_t> nt(n), nf(n);
    const std::vector<float> zero(hidden_, 0.0f);
    std::vector<const float *> spk(n);
    for (int32_t i = 0; i < n; ++i) {
        const int64_t t = now_ms();
        toks[i] = tokenizer_.encode_for_tts(texts[i]);
        out[i].t_tokenize_ms = now_ms() - t;
        if (toks[i].empty()) return fail_all("Failed to tokenize text");
        tp[i] = toks[i].data();
        nt[i] = (int32_t)toks[i].size();
        spk[i] = speaker_embeddings.empty() || speaker_embeddings[i].empty() ? zero.data() : speaker_embeddings[i].data();
    }
    const int32_t max_len = std::max(params.max_audio_tokens, 1);
    if (!ensure_slots(n, max_len)) return fail_all("Failed to generate speech codes: " + error_msg_);
    q3t_gen_params p;
    q3t_default_params(&p);
    p.max_len = max_len;
    p.repetition_penalty = params.repetition_penalty;
    p.temperature = params.temperature;
    p.top_k = params.top_k;
    p.seed = seed_;
    std::vector<int32_t> codes((size_t)n * max_len * 16);
    const int64_t tg = now_ms();
    if (q3t_generate(ctx_, n, tp.data(), nt.data(), spk.data(), &p, codes.data(), nf.data()) != Q3T_OK)
        return fail_all("Failed to generate speech codes: " + q3t_error());
    const int64_t gen_ms = now_ms() - tg;
    for (int32_t i = 0; i < n; ++i) {
        tts_result &r = out[i];
        r.t_generate_ms = gen_ms;
        if (nf[i] == 0) { r.error_msg = "No speech codes generated"; continue; }
        const int32_t *c = codes.data() + (size_t)i * max_len * 16;
        const int64_t td = now_ms();
        int64_t got = 0;
        int rc;
        if (vocoder_chunk_ > 0) {
            r.audio.resize((size_t)nf[i] * 1920);
            rc = q3t_vocoder_decode_chunked(ctx_, c, nf[i], 16, vocoder_chunk_, r.audio.data(), &got);
        } else {
            r.audio.resize((size_t)std::max<int64_t>(q3t_vocoder_num_samples(ctx_, nf[i], Q3T_VOCODER_FULL), 0));
            rc = q3t_vocoder_decode(ctx_, c, nf[i], Q3T_VOCODER_FULL, r.audio.data(), &got);
        }
        if (rc != Q3T_OK) { r.error_msg = "Failed to decode speech codes: " + q3t_error(); r.audio.clear(); continue; }
        r.audio.resize((size_t)got);
        r.t_decode_ms = now_ms() - td;
        r.sample_rate = kSampleRate;
        r.success = true;
    }
    const int64_t total = now_ms() - t0;
    for (auto &r : out) r.t_total_ms = total;
    return out;
}

// ======================================================================================================= audio

void resample_linear(const float *input, int input_len, int input_rate, std::vector<float> &output, int output_rate) {
    const double ratio = (double)input_rate / output_rate;
    const int out_len = (int)((double)input_len / ratio);
    output.resize(std::max(out_len, 0));
    for (int i = 0; i < out_len; ++i) {
        const double src = i * ratio;
        const int i0 = (int)src, i1 = i0 + 1;
        const double frac = src - i0;
        output[i] = i1 >= input_len ? input[input_len - 1] : (float)((1.0 - frac) * input[i0] + frac * input[i1]);
    }
}

bool load_audio_file(const std::string &path, std::vector<float> &samples, int &sample_rate) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) { fprintf(stderr, "ERROR: Cannot open WAV file: %s\n", path.c_str()); return false; }
    auto done = [&](bool ok) { fclose(f); return ok; };
    char tag[4];
    uint32_t u32 = 0;
    if (fread(tag, 1, 4, f) != 4 || memcmp(tag, "RIFF", 4) != 0) { fprintf(stderr, "ERROR: Not a RIFF file\n"); return done(false); }
    if (fread(&u32, 4, 1, f) != 1) return done(false);
    if (fread(tag, 1, 4, f) != 4 || memcmp(tag, "WAVE", 4) != 0) { fprintf(stderr, "ERROR: Not a WAVE file\n"); return done(false); }
    uint16_t fmt = 0, ch = 0, bits = 0;
    uint32_t sr = 0;
    for (;;) {
        uint32_t size = 0;
        if (fread(tag, 1, 4, f) != 4 || fread(&size, 4, 1, f) != 1) break;
        if (memcmp(tag, "fmt ", 4) == 0) {
            if (fread(&fmt, 2, 1, f) != 1 || fread(&ch, 2, 1, f) != 1 || fread(&sr, 4, 1, f) != 1) break;
            fseek(f, 6, SEEK_CUR);   // byte rate + block align
            if (fread(&bits, 2, 1, f) != 1) break;
            if (size > 16) fseek(f, size - 16, SEEK_CUR);
        } else if (memcmp(tag, "data", 4) == 0) {
            sample_rate = (int)sr;
            if (ch == 0) return done(false);
            const int width = (fmt == 1 && bits == 16) ? 2 : ((fmt == 1 && bits == 32) || fmt == 3) ? 4 : 0;
            if (width == 0) {
                if (fmt == 1) fprintf(stderr, "ERROR: Unsupported bits per sample: %d\n", bits);
                else fprintf(stderr, "ERROR: Unsupported audio format: %d\n", fmt);
                return done(false);
            }
            const size_t n = size / ((size_t)width * ch);
            std::vector<uint8_t> raw(n * ch * width);
            if (fread(raw.data(), (size_t)width, n * ch, f) != n * ch) return done(false);
            samples.resize(n);
            for (size_t i = 0; i < n; ++i) {
                float sum = 0.0f;
                for (int c = 0; c < ch; ++c) {
                    const uint8_t *p = raw.data() + (i * ch + c) * width;
                    if (width == 2) { int16_t v; memcpy(&v, p, 2); sum += v / 32768.0f; }
                    else if (fmt == 1) { int32_t v; memcpy(&v, p, 4); sum += v / 2147483648.0f; }
                    else { float v; memcpy(&v, p, 4); sum += v; }
                }
                samples[i] = sum / ch;
            }
            return done(true);
        } else {
            fseek(f, size, SEEK_CUR);
        }
    }
    fprintf(stderr, "ERROR: No data chunk found\n");
    return done(false);
}

bool save_audio_file(const std::string &path, const std::vector<float> &samples, int sample_rate) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) { fprintf(stderr, "ERROR: Cannot create WAV file: %s\n", path.c_str()); return false; }
    const uint16_t ch = 1, bits = 16, block = ch * bits / 8, fmt = 1;
    const uint32_t sr = (uint32_t)sample_rate, byte_rate = sr * block, data = (uint32_t)(samples.size() * block);
    const uint32_t riff = 36 + data, fmt_size = 16;
    std::vector<uint8_t> h;
    auto put = [&](const void *p, size_t n) { h.insert(h.end(), (const uint8_t *)p, (const uint8_t *)p + n); };
    put("RIFF", 4); put(&riff, 4); put("WAVE", 4);
    put("fmt ", 4); put(&fmt_size, 4); put(&fmt, 2); put(&ch, 2); put(&sr, 4); put(&byte_rate, 4); put(&block, 2);
    put(&bits, 2);
    put("data", 4); put(&data, 4);
    std::vector<int16_t> pcm(samples.size());
    for (size_t i = 0; i < samples.size(); ++i) {
        const float s = std::min(1.0f, std::max(-1.0f, samples[i]));
        pcm[i] = (int16_t)(s * 32767.0f);   // truncation toward zero, as the reference's cast
    }
    const bool ok = fwrite(h.data(), 1, h.size(), f) == h.size() &&
                    (pcm.empty() || fwrite(pcm.data(), 2, pcm.size(), f) == pcm.size());
    fclose(f);
    return ok;
}

}  // namespace qwen3_tts
