// capi.cpp — extern "C" boundary (include/q3t_backend.h).  No exception crosses it.
#include "../../include/q3t_backend.h"

#include <algorithm>
#include <exception>

#include "comm.h"
#include "devlock.h"
#include "engine.h"
#include "speaker.h"
#include "tokenizer.h"
#include "vocoder.h"

struct q3t_tokenizer {
    q3t::TextTokenizer tok;
};

struct q3t_ctx {
    q3t::Engine engine;
    q3t::Comm *comm = nullptr;   // set by q3t_ctx_create_shared
    ~q3t_ctx() { q3t::comm_destroy(comm); }
};

namespace {
q3t::GenParams to_gp(const q3t_gen_params *p) {
    q3t::GenParams g;
    if (!p) return g;
    g.max_len = p->max_len;
    g.language_id = p->language_id;
    g.rep_penalty = p->repetition_penalty;
    g.temperature = p->temperature;
    g.top_k = p->top_k;
    g.seed = p->seed;
    g.force_frames = p->force_frames;
    return g;
}
#define GUARD_BEGIN try {
#define GUARD_END                                                   \
    }                                                               \
    catch (const std::exception &e) {                               \
        q3t::set_error(std::string("exception: ") + e.what());      \
        return Q3T_ERR;                                             \
    }                                                               \
    catch (...) {                                                   \
        q3t::set_error("unknown exception");                        \
        return Q3T_ERR;                                             \
    }
#define CHECK_CTX(c) if (!(c)) { q3t::set_error("null context"); return Q3T_ERR; }
}  // namespace
#define CHECK_TALKER(c)                                                                                   \
    do {                                                                                                   \
        if (!(c)->engine.has_talker()) {                                                                   \
            q3t::set_error("vocoder-only context (created without a TTS GGUF)");                            \
            return Q3T_ERR;                                                                                \
        }                                                                                                  \
    } while (0)

extern "C" {

const char *q3t_last_error(void) { return q3t::last_error().c_str(); }

void q3t_default_params(q3t_gen_params *p) {
    if (!p) return;
    p->max_len = 4096;
    p->language_id = 2050;
    p->repetition_penalty = 1.05f;
    p->temperature = 0.9f;
    p->top_k = 50;
    p->seed = 0;
    p->force_frames = 0;
}

int q3t_ctx_create(const char *tts_gguf, const char *tokenizer_gguf, int device, int max_slots, int max_ctx, q3t_ctx **out) {
    GUARD_BEGIN
    if (!out || (!tts_gguf && !tokenizer_gguf)) { q3t::set_error("null argument"); return Q3T_ERR; }
    *out = nullptr;
    q3t_ctx *c = new q3t_ctx();
    if (!c->engine.load(tts_gguf ? tts_gguf : "", tokenizer_gguf ? tokenizer_gguf : "", device, max_slots, max_ctx)) {
        delete c;
        return Q3T_ERR;
    }
    *out = c;
    return Q3T_OK;
    GUARD_END
}

int q3t_comm_unique_id(uint8_t *id) {
    GUARD_BEGIN
    if (!id) { q3t::set_error("null argument"); return Q3T_ERR; }
    return q3t::comm_unique_id(id) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_ctx_create_shared(const char *tts_gguf, const char *tokenizer_gguf, int device, int max_slots, int max_ctx,
                          int rank, int world, const uint8_t *id, q3t_ctx **out) {
    GUARD_BEGIN
    if (!out || !tts_gguf || !id) { q3t::set_error("null argument"); return Q3T_ERR; }
    *out = nullptr;
    q3t_ctx *c = new q3t_ctx();
    if (!q3t::comm_init(&c->comm, world, rank, id, device) ||
        !c->engine.load(tts_gguf, tokenizer_gguf ? tokenizer_gguf : "", device, max_slots, max_ctx, rank != 0) ||
        !q3t::comm_bcast_arenas(c->comm, c->engine.weight_arenas(), c->engine.stream()) ||
        (rank != 0 && !c->engine.finish_weights())) {
        delete c;
        return Q3T_ERR;
    }
    *out = c;
    return Q3T_OK;
    GUARD_END
}

int q3t_plan_weight_layout(const char *tts_gguf, uint64_t *offsets, int max_n, int *n_alloc, uint64_t *used) {
    GUARD_BEGIN
    if (!tts_gguf || !n_alloc || !used) { q3t::set_error("null argument"); return Q3T_ERR; }
    std::vector<size_t> off;
    size_t u = 0;
    {
        q3t::Engine e;
        if (!e.plan_layout(tts_gguf, off, u)) return Q3T_ERR;
    }
    *n_alloc = (int)off.size();
    *used = u;
    if (offsets)
        for (int i = 0; i < std::min<int>(max_n, (int)off.size()); ++i) offsets[i] = off[i];
    return Q3T_OK;
    GUARD_END
}

int q3t_ctx_create_replica(q3t_ctx *src, int device, int max_slots, int max_ctx, q3t_ctx **out) {
    GUARD_BEGIN
    if (!out || !src) { q3t::set_error("null argument"); return Q3T_ERR; }
    *out = nullptr;
    q3t_ctx *c = new q3t_ctx();
    if (!c->engine.load(src->engine.tts_path(), src->engine.tok_path(), device, max_slots, max_ctx, true) ||
        !c->engine.copy_weights_from(src->engine)) {
        delete c;
        return Q3T_ERR;
    }
    *out = c;
    return Q3T_OK;
    GUARD_END
}

int q3t_comm_allreduce_max(q3t_ctx *ctx, double *values, int n) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    if (n > 0 && !values) { q3t::set_error("null argument"); return Q3T_ERR; }
    if (!ctx->comm) return Q3T_OK;   // a single-process context: nothing to reduce
    return q3t::comm_allreduce_max(ctx->comm, values, n, ctx->engine.stream()) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

void q3t_ctx_destroy(q3t_ctx *ctx) { delete ctx; }

int q3t_set_mfma_min_batch(int min_batch) {
    q3t::gemm_mfma_set_min_batch(min_batch);
    return Q3T_OK;
}

int q3t_get_config(const q3t_ctx *ctx, q3t_config *o) {
    CHECK_CTX(ctx);
    if (!o) { q3t::set_error("null argument"); return Q3T_ERR; }
    const q3t::Config &c = ctx->engine.cfg();
    o->hidden = c.hidden; o->n_layers = c.n_layers; o->n_heads = c.n_heads; o->n_kv_heads = c.n_kv;
    o->head_dim = c.head_dim; o->intermediate = c.inter; o->codec_vocab = c.codec_vocab; o->n_codebooks = c.n_codebooks;
    o->text_vocab = c.text_vocab; o->text_dim = c.text_dim; o->cp_layers = c.cp_layers; o->cp_vocab = c.cp_vocab;
    o->codec_eos = c.codec_eos;
    q3t::Vocoder *v = const_cast<q3t::Engine &>(ctx->engine).vocoder();
    o->has_vocoder = v && v->loaded() ? 1 : 0;
    o->sample_rate = 24000;
    o->max_slots = ctx->engine.max_slots();
    o->max_ctx = ctx->engine.max_ctx();
    o->cp_hidden = c.cp_hidden; o->cp_intermediate = c.cp_inter; o->cp_heads = c.cp_heads; o->cp_kv_heads = c.cp_kv;
    o->has_mtp = c.has_mtp ? 1 : 0;
    return Q3T_OK;
}

int q3t_generate(q3t_ctx *ctx, int n_utt, const int32_t *const *tokens, const int32_t *n_tokens, const float *const *speaker,
                 const q3t_gen_params *p, int32_t *codes, int32_t *n_frames) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    if (n_utt < 0 || (n_utt > 0 && (!tokens || !n_tokens || !codes || !n_frames))) { q3t::set_error("null argument"); return Q3T_ERR; }
    return ctx->engine.generate(n_utt, tokens, n_tokens, speaker, to_gp(p), codes, n_frames) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_generate_stream(q3t_ctx *ctx, int n_utt, const int32_t *const *tokens, const int32_t *n_tokens,
                        const float *const *speaker, const q3t_gen_params *p, int32_t *codes, int32_t *n_frames,
                        q3t_frame_cb on_frames, void *user, int32_t interval) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    if (n_utt < 0 || (n_utt > 0 && (!tokens || !n_tokens || !codes || !n_frames))) { q3t::set_error("null argument"); return Q3T_ERR; }
    return ctx->engine.generate(n_utt, tokens, n_tokens, speaker, to_gp(p), codes, n_frames, on_frames, user, interval)
               ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_generate_queue(q3t_ctx *ctx, int n_utt, const int32_t *const *tokens, const int32_t *n_tokens,
                       const float *const *speaker, const q3t_gen_params *p, int32_t *codes, int32_t *n_frames,
                       int32_t max_active) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    if (n_utt < 0 || (n_utt > 0 && (!tokens || !n_tokens || !codes || !n_frames))) { q3t::set_error("null argument"); return Q3T_ERR; }
    return ctx->engine.generate_queue(n_utt, tokens, n_tokens, speaker, to_gp(p), codes, n_frames, max_active) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_synchronize(q3t_ctx *ctx) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    if (hipSetDevice(ctx->engine.device()) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        q3t::set_error("q3t_synchronize: device synchronize failed");
        return Q3T_ERR;
    }
    return Q3T_OK;
    GUARD_END
}

int q3t_last_timing(const q3t_ctx *ctx, double *prefill_ms, double *frames_ms) {
    CHECK_CTX(ctx);
    if (prefill_ms) *prefill_ms = ctx->engine.last_prefill_ms;
    if (frames_ms) *frames_ms = ctx->engine.last_frames_ms;
    return Q3T_OK;
}

int q3t_time_stage(q3t_ctx *ctx, int stage, int n, int pos, int iters, double *ms) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    if (!ms) { q3t::set_error("null argument"); return Q3T_ERR; }
    return ctx->engine.time_stage(stage, n, pos, iters, ms) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

#ifdef Q3T_DEV
// development builds only (make DEV=1): raw device state for the timeline tools under tools/dev
int q3t_debug_read(q3t_ctx *ctx, int which, void *dst, size_t bytes) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    return ctx->engine.debug_read(which, dst, bytes) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}
#endif

int q3t_persist_status(q3t_ctx *ctx) {
    if (!ctx || !ctx->engine.has_talker()) return -1;
    if (ctx->engine.persist_fell_back()) return 2;
    if (!ctx->engine.persist_enabled()) return -1;
    return ctx->engine.persist_error() ? 1 : 0;
}

int q3t_persist_kernels(q3t_ctx *ctx) {
    if (!ctx || !ctx->engine.has_talker()) return 0;
    return ctx->engine.persist_kernels();
}

int64_t q3t_vocoder_num_samples(const q3t_ctx *ctx, int32_t n_frames, int mode) {
    if (!ctx) return -1;
    q3t::Vocoder *v = const_cast<q3t::Engine &>(ctx->engine).vocoder();
    if (!v || !v->loaded()) return -1;
    return v->n_samples(n_frames, mode);
}

double q3t_vocoder_flops(const q3t_ctx *ctx, int32_t n_frames) {
    if (!ctx) return -1.0;
    q3t::Vocoder *v = const_cast<q3t::Engine &>(ctx->engine).vocoder();
    if (!v || !v->loaded()) return -1.0;
    return v->decode_flops(n_frames);
}

int q3t_vocoder_decode(q3t_ctx *ctx, const int32_t *codes, int32_t n_frames, int mode, float *pcm, int64_t *n_samples) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    q3t::Vocoder *v = ctx->engine.vocoder();
    if (!v || !v->loaded()) { q3t::set_error("vocoder not loaded (no tokenizer GGUF given)"); return Q3T_ERR; }
    if (mode != Q3T_VOCODER_FULL && mode != Q3T_VOCODER_CHUNK40) { q3t::set_error("bad vocoder mode"); return Q3T_ERR; }
    if (n_frames > 0 && (!codes || !pcm)) { q3t::set_error("null argument"); return Q3T_ERR; }
    q3t::DeviceLock lk(false, ctx->engine.device());   // never beside a persistent grid (devlock.h)
    return v->decode(codes, n_frames, mode, pcm, n_samples) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_vocoder_decode_chunked(q3t_ctx *ctx, const int32_t *codes, int32_t n_frames, int32_t n_codebooks,
                               int32_t chunk_frames, float *pcm, int64_t *n_samples) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    q3t::Vocoder *v = ctx->engine.vocoder();
    if (!v || !v->loaded()) { q3t::set_error("vocoder not loaded (no tokenizer GGUF given)"); return Q3T_ERR; }
    if (n_codebooks != 16) { q3t::set_error("n_codebooks must be 16"); return Q3T_ERR; }
    if (chunk_frames <= 0) { q3t::set_error("chunk_frames must be > 0"); return Q3T_ERR; }
    if (n_frames > 0 && (!codes || !pcm)) { q3t::set_error("null argument"); return Q3T_ERR; }
    q3t::DeviceLock lk(false, ctx->engine.device());   // never beside a persistent grid (devlock.h)
    return v->decode(codes, n_frames, Q3T_VOCODER_CHUNK40, pcm, n_samples, chunk_frames) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_vocoder_decode_batch(q3t_ctx *ctx, int32_t n_utt, const int32_t *const *codes, const int32_t *n_frames,
                             int mode, int32_t chunk_frames, float *const *pcm, int64_t *n_samples) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    q3t::Vocoder *v = ctx->engine.vocoder();
    if (!v || !v->loaded()) { q3t::set_error("vocoder not loaded (no tokenizer GGUF given)"); return Q3T_ERR; }
    if (mode != Q3T_VOCODER_FULL && mode != Q3T_VOCODER_CHUNK40) { q3t::set_error("bad vocoder mode"); return Q3T_ERR; }
    if (n_utt < 0 || (n_utt > 0 && (!codes || !n_frames || !pcm || !n_samples))) { q3t::set_error("null argument"); return Q3T_ERR; }
    for (int u = 0; u < n_utt; ++u)
        if (n_frames[u] > 0 && (!codes[u] || !pcm[u])) { q3t::set_error("null argument"); return Q3T_ERR; }
    if (mode == Q3T_VOCODER_CHUNK40 && chunk_frames <= 0) { q3t::set_error("chunk_frames must be > 0"); return Q3T_ERR; }
    std::vector<int> nf(n_frames, n_frames + n_utt);
    q3t::DeviceLock lk(false, ctx->engine.device());   // never beside a persistent grid (devlock.h)
    return v->decode_batch(n_utt, codes, nf.data(), mode, pcm, n_samples, chunk_frames) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_vocoder_set_batch_frames(q3t_ctx *ctx, int32_t frames) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    q3t::Vocoder *v = ctx->engine.vocoder();
    if (!v || !v->loaded()) { q3t::set_error("vocoder not loaded (no tokenizer GGUF given)"); return Q3T_ERR; }
    v->set_batch_frames(frames);
    return Q3T_OK;
    GUARD_END
}

int q3t_ctx_create_speaker(const char *tts_gguf, int device, q3t_ctx **out) {
    GUARD_BEGIN
    if (!out || !tts_gguf) { q3t::set_error("null argument"); return Q3T_ERR; }
    *out = nullptr;
    q3t_ctx *c = new q3t_ctx();
    if (!c->engine.load_speaker_only(tts_gguf, device)) {
        delete c;
        return Q3T_ERR;
    }
    *out = c;
    return Q3T_OK;
    GUARD_END
}

int q3t_speaker_dim(const q3t_ctx *ctx) {
    if (!ctx) return 0;
    q3t::SpeakerEncoder *s = const_cast<q3t::Engine &>(ctx->engine).speaker();
    return s && s->loaded() ? s->dim() : 0;
}

int q3t_speaker_encode(q3t_ctx *ctx, const float *samples, int32_t n_samples, float *embedding) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    q3t::SpeakerEncoder *s = ctx->engine.speaker();
    if (!s || !s->loaded()) { q3t::set_error("Model not loaded (no speaker encoder tensors in the TTS GGUF)"); return Q3T_ERR; }
    if (!samples || !embedding || n_samples <= 0) { q3t::set_error("null argument"); return Q3T_ERR; }
    q3t::DeviceLock lk(false, ctx->engine.device());   // never beside a persistent grid (devlock.h)
    return s->encode(samples, n_samples, embedding) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_speaker_mel(q3t_ctx *ctx, const float *samples, int32_t n_samples, float *mel, int32_t cap_frames,
                    int32_t *n_frames) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    q3t::SpeakerEncoder *s = ctx->engine.speaker();
    if (!s || !s->loaded()) { q3t::set_error("Model not loaded (no speaker encoder tensors in the TTS GGUF)"); return Q3T_ERR; }
    if (!samples || !n_frames || n_samples <= 0) { q3t::set_error("null argument"); return Q3T_ERR; }
    std::vector<float> m;
    int F = 0;
    q3t::DeviceLock lk(false, ctx->engine.device());
    if (!s->mel(samples, n_samples, m, &F)) return Q3T_ERR;
    *n_frames = F;
    if (mel) {
        if (cap_frames < F) { q3t::set_error("mel buffer too small"); return Q3T_ERR; }
        std::copy(m.begin(), m.end(), mel);
    }
    return Q3T_OK;
    GUARD_END
}

int q3t_tokenizer_load(const char *gguf_path, q3t_tokenizer **out) {
    GUARD_BEGIN
    if (!gguf_path || !out) { q3t::set_error("null argument"); return Q3T_ERR; }
    *out = nullptr;
    q3t_tokenizer *t = new q3t_tokenizer();
    if (!t->tok.load(std::string(gguf_path))) { delete t; return Q3T_ERR; }
    *out = t;
    return Q3T_OK;
    GUARD_END
}

void q3t_tokenizer_free(q3t_tokenizer *tok) { delete tok; }

int q3t_tokenizer_info(const q3t_tokenizer *tok, int32_t *vocab_size, int32_t *bos_id, int32_t *eos_id, int32_t *pad_id) {
    if (!tok) { q3t::set_error("null tokenizer"); return Q3T_ERR; }
    if (vocab_size) *vocab_size = tok->tok.vocab_size();
    if (bos_id) *bos_id = tok->tok.bos();
    if (eos_id) *eos_id = tok->tok.eos();
    if (pad_id) *pad_id = tok->tok.pad();
    return Q3T_OK;
}

int q3t_tokenizer_encode(const q3t_tokenizer *tok, const char *text, int64_t n_bytes, int for_tts, int32_t *tokens,
                         int32_t cap, int32_t *n_tokens) {
    GUARD_BEGIN
    if (!tok || !text || !n_tokens) { q3t::set_error("null argument"); return Q3T_ERR; }
    const std::string t = n_bytes < 0 ? std::string(text) : std::string(text, (size_t)n_bytes);
    const std::vector<int32_t> ids = for_tts ? tok->tok.encode_for_tts(t) : tok->tok.encode(t);
    *n_tokens = (int32_t)ids.size();
    if (tokens) {
        if (cap < (int32_t)ids.size()) { q3t::set_error("token buffer too small"); return Q3T_ERR; }
        std::copy(ids.begin(), ids.end(), tokens);
    }
    return Q3T_OK;
    GUARD_END
}

int q3t_tokenizer_decode(const q3t_tokenizer *tok, const int32_t *tokens, int32_t n, char *text, int64_t cap,
                         int64_t *n_bytes) {
    GUARD_BEGIN
    if (!tok || !n_bytes || (n > 0 && !tokens)) { q3t::set_error("null argument"); return Q3T_ERR; }
    const std::string s = tok->tok.decode(std::vector<int32_t>(tokens, tokens + std::max(n, 0)));
    *n_bytes = (int64_t)s.size();
    if (text) {
        if (cap < (int64_t)s.size()) { q3t::set_error("text buffer too small"); return Q3T_ERR; }
        std::copy(s.begin(), s.end(), text);
    }
    return Q3T_OK;
    GUARD_END
}

int q3t_talker_forward(q3t_ctx *ctx, int n, const float *embd, const int32_t *pos, float *hidden, float *logits) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    if (!embd || !pos) { q3t::set_error("null argument"); return Q3T_ERR; }
    return ctx->engine.talker_forward(n, embd, pos, hidden, logits) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_talker_prefill(q3t_ctx *ctx, int n_utt, int n_rows, const float *embd, int family_slots, float *hidden,
                       float *logits) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    if (!embd) { q3t::set_error("null argument"); return Q3T_ERR; }
    return ctx->engine.talker_prefill(n_utt, n_rows, embd, family_slots, hidden, logits) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_codepred_frame(q3t_ctx *ctx, int n, const float *hidden, const int32_t *cb0, float temperature, int32_t top_k,
                       uint64_t seed, int32_t frame, int32_t *codes15, float *logits) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    if (!hidden || !cb0 || !codes15) { q3t::set_error("null argument"); return Q3T_ERR; }
    return ctx->engine.codepred_frame(n, hidden, cb0, temperature, top_k, seed, frame, codes15, logits) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_cb0_select(q3t_ctx *ctx, int n, const float *logits, const uint8_t *seen, const int32_t *frame,
                   const int32_t *n_tokens, const q3t_gen_params *p, int32_t *tokens) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    if (!logits || !seen || !frame || !n_tokens || !tokens) { q3t::set_error("null argument"); return Q3T_ERR; }
    return ctx->engine.cb0_select_host(n, logits, seen, frame, n_tokens, to_gp(p), tokens) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_project_text(q3t_ctx *ctx, int n, const int32_t *tokens, float *out) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    if (n > 0 && (!tokens || !out)) { q3t::set_error("null argument"); return Q3T_ERR; }
    return ctx->engine.project_text(n, tokens, out) ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

int q3t_prefill_embd(q3t_ctx *ctx, const int32_t *tokens, int n, const float *speaker, int language_id, float *prefill,
                     int32_t *prefill_len, float *trailing, int32_t *trailing_len, float *tts_pad) {
    GUARD_BEGIN
    CHECK_CTX(ctx);
    CHECK_TALKER(ctx);
    if (!tokens || !prefill || !prefill_len || !trailing || !trailing_len || !tts_pad) { q3t::set_error("null argument"); return Q3T_ERR; }
    return ctx->engine.prefill_embd(tokens, n, speaker, language_id, prefill, prefill_len, trailing, trailing_len, tts_pad)
               ? Q3T_OK : Q3T_ERR;
    GUARD_END
}

void gpu_fp32_to_fp16(const float *in, void *out, int n, void *stream) {
    q3t::launch_f32_to_f16(in, static_cast<uint16_t *>(out), n, static_cast<hipStream_t>(stream));
}
void gpu_argmax_f32(const float *in, int32_t *out, int n, void *stream) {
    q3t::launch_argmax_f32(in, out, n, static_cast<hipStream_t>(stream));
}
void gpu_embedding_lookup_by_gpu_id(const int32_t *token_id_ptr, const float *table, float *output, int embd_dim, void *stream) {
    q3t::launch_embed_lookup(token_id_ptr, table, output, embd_dim, static_cast<hipStream_t>(stream));
}
void gpu_sample_topk_f32(const float *logits, const float *rand_val, int32_t *out, float temperature, int32_t top_k,
                         int32_t vocab_size, void *stream) {
    if (vocab_size > 4096) { q3t::set_error("gpu_sample_topk_f32: vocab_size > 4096"); return; }
    q3t::launch_sample_topk_f32(logits, rand_val, out, temperature, top_k, vocab_size, static_cast<hipStream_t>(stream));
}

}  // extern "C"
