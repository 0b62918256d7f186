// engine.cpp — see engine.h.
#include "engine.h"
#include "persist.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/stat.h>
#include <algorithm>
#include <condition_variable>
#include <mutex>

#include "devlock.h"
#include <chrono>
#include <condition_variable>
#include "speaker.h"
#include "vocoder.h"

namespace q3t {

Engine::Engine() = default;

namespace {
WPLock g_device_rw[64];
thread_local int t_device_depth[64];
}  // namespace

// devlock.h: exclusive for single-slot (persistent-kernel) runs, shared for everything else
DeviceLock::DeviceLock(bool exclusive, int device) : dev_(device & 63) {
    if (t_device_depth[dev_]++ > 0) return;
    mode_ = exclusive ? 2 : 1;
    if (exclusive) g_device_rw[dev_].lock();
    else g_device_rw[dev_].lock_shared();
}
DeviceLock::~DeviceLock() {
    --t_device_depth[dev_];
    if (mode_ == 2) g_device_rw[dev_].unlock();
    else if (mode_ == 1) g_device_rw[dev_].unlock_shared();
}

namespace {
bool env_flag(const char *name, bool dflt) {
    const char *e = std::getenv(name);
    return e ? std::atoi(e) != 0 : dflt;
}
}  // namespace

Options Options::from_env() {
    Options o;
    o.persist = env_flag("Q3T_PERSIST", true);
    o.persist_cp = env_flag("Q3T_PERSIST_CP", true);
    o.cp_fused_attn = env_flag("Q3T_CP_FUSED_ATTN", true);
    o.cp_qkv_table = env_flag("Q3T_CP_QKV_TABLE", true);
    o.cp_roles = env_flag("Q3T_CP_ROLES", true);
    o.mm_cp_table = env_flag("Q3T_MM_CP_TABLE", true);
    o.fold_advance = env_flag("Q3T_FOLD_ADVANCE", true);
    o.tk_roles = env_flag("Q3T_TK_ROLES", true);
    o.cpb = env_flag("Q3T_PERSIST_CPB", true);
    o.tkb = env_flag("Q3T_PERSIST_TKB", true);
    o.fused_select = env_flag("Q3T_FUSED_SELECT", true);
    o.defer_cp_select = env_flag("Q3T_CP_DEFER_SELECT", true);
    o.attn_split = env_flag("Q3T_ATTN_SPLIT", false);
    if (const char *e = std::getenv("Q3T_PERSIST_FAULT_AT")) o.persist_fault_at = (unsigned)std::max(0, std::atoi(e));
#ifdef Q3T_DEV
    if (const char *e = std::getenv("Q3T_POLL_EVERY")) o.poll_every = std::max(1, std::atoi(e));
#endif
    return o;
}

Engine::~Engine() {
    if (device_ >= 0) hipSetDevice(device_);
    for (auto &kv : g_talker_) hipGraphExecDestroy(kv.second);
    for (auto &kv : g_frame_) hipGraphExecDestroy(kv.second);
    for (auto &kv : g_prefill_) hipGraphExecDestroy(kv.second);
    for (auto &kv : g_cp_) hipGraphExecDestroy(kv.second);
    voc_.reset();
    for (void *p : allocs_) hipFree(p);
    if (qout_) hipFree(qout_);
    if (pin_) hipHostFree(pin_);
    for (PinnedChunk &c : chunk_pool_) { hipHostFree(c.codes); hipEventDestroy(c.ev); }
    if (stream_) hipStreamDestroy(stream_);
    if (astream_) hipStreamDestroy(astream_);
}

template <class T>
T *Engine::dalloc(size_t n) {
    void *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
    allocs_.push_back(p);
    // zeroed on the context's own stream, and drained before any other stream (the admission stream, or a
    // synchronous null-stream copy into the buffer right after this call) can touch it: without the ordering a first
    // launch could read what a previous context freed in the same process left in this memory (DESIGN §2e').  Only
    // this context's stream is waited for, never the device.
    if (hipMemsetAsync(p, 0, std::max<size_t>(n, 1) * sizeof(T), stream_) != hipSuccess ||
        hipStreamSynchronize(stream_) != hipSuccess) {
        set_error("dalloc: zeroing failed");
        return nullptr;
    }
    return static_cast<T *>(p);
}


// the pinned / device scratch of generate() and generate_queue(), kept across calls: a per-call hipFree or
// hipHostFree would synchronise the whole device (every other context on it included)
bool Engine::ensure_pinned(size_t bytes) {
    if (bytes <= pin_cap_) return true;
    if (pin_) hipHostFree(pin_);
    pin_ = nullptr;
    pin_cap_ = 0;
    if (hipHostMalloc(&pin_, bytes, hipHostMallocDefault) != hipSuccess) { pin_ = nullptr; set_error("hipHostMalloc failed"); return false; }
    pin_cap_ = bytes;
    return true;
}
bool Engine::ensure_qout(size_t bytes) {
    if (bytes <= qout_cap_) return true;
    if (qout_) hipFree(qout_);
    qout_ = nullptr;
    qout_cap_ = 0;
    if (hipMalloc(&qout_, bytes) != hipSuccess) { qout_ = nullptr; set_error("device allocation failed"); return false; }
    qout_cap_ = bytes;
    return true;
}

namespace {
bool check_shape(const GgufTensor *t, const char *name, int64_t cols, int64_t rows, int type) {
    if (!t) { set_error(std::string("missing tensor ") + name); return false; }
    const bool lead_ok = t->ne[0] == cols || (t->n_dims == 3 && t->ne[0] == 1 && t->ne[1] == cols);
    if (t->type != type || !lead_ok || t->nelements() != cols * rows) {
        set_error(std::string("tensor ") + name + ": unexpected shape/type");
        return false;
    }
    return true;
}
}  // namespace

// parse_config key aliases / defaults: src/tts_transformer.cpp:288-442 (GGUF header keys only: every rank, and the
// host-only layout plan, compute the same config)
bool Engine::parse_config(const Gguf &g) {
    c_.text_vocab = (int)g.get_int({"qwen3-tts.text.vocab_size", "qwen3-tts.text_vocab_size"}, 151936);
    c_.text_dim = (int)g.get_int({"qwen3-tts.text.embedding_dim", "qwen3-tts.text_hidden_size"}, 2048);
    c_.hidden = (int)g.get_int({"qwen3-tts.talker.embedding_length", "qwen3-tts.embedding_length"}, 1024);
    c_.n_layers = (int)g.get_int({"qwen3-tts.talker.block_count", "qwen3-tts.block_count"}, 28);
    c_.n_heads = (int)g.get_int({"qwen3-tts.talker.attention.head_count", "qwen3-tts.attention.head_count"}, 16);
    c_.n_kv = (int)g.get_int({"qwen3-tts.talker.attention.head_count_kv", "qwen3-tts.attention.head_count_kv"}, 8);
    c_.inter = (int)g.get_int({"qwen3-tts.talker.feed_forward_length", "qwen3-tts.feed_forward_length"}, 3072);
    c_.head_dim = (int)g.get_int({"qwen3-tts.talker.attention.key_length", "qwen3-tts.attention.key_length"}, 128);
    c_.eps = g.get_f32({"qwen3-tts.talker.attention.layer_norm_rms_epsilon", "qwen3-tts.attention.layer_norm_rms_epsilon"}, 1e-6f);
    c_.rope_theta = g.get_f32({"qwen3-tts.talker.rope.freq_base", "qwen3-tts.rope.freq_base"}, 1000000.0f);
    c_.codec_vocab = (int)g.get_int({"qwen3-tts.talker.codec_vocab_size", "qwen3-tts.vocab_size"}, 3072);
    c_.n_codebooks = (int)g.get_int({"qwen3-tts.talker.num_codebooks", "qwen3-tts.num_code_groups"}, 16);
    c_.cp_layers = (int)g.get_int({"qwen3-tts.code_pred.layer_count", "qwen3-tts.code_predictor.layer_count"}, 5);
    c_.cp_vocab = (int)g.get_int({"qwen3-tts.code_pred.vocab_size", "qwen3-tts.code_predictor.vocab_size"}, 2048);
    c_.codec_pad = (int)g.get_int({"qwen3-tts.codec.pad_id"}, 2148);
    c_.codec_bos = (int)g.get_int({"qwen3-tts.codec.bos_id"}, 2149);
    c_.codec_eos = (int)g.get_int({"qwen3-tts.codec.eos_id", "qwen3-tts.codec.eos_token_id"}, 2150);
    c_.tts_bos = (int)g.get_int({"qwen3-tts.tts_bos_token_id", "qwen3-tts.tts.bos_token_id", "qwen3-tts.tts.bos_id"}, 151672);
    c_.tts_eos = (int)g.get_int({"qwen3-tts.tts_eos_token_id", "qwen3-tts.tts.eos_token_id", "qwen3-tts.tts.eos_id"}, 151673);
    c_.tts_pad = (int)g.get_int({"qwen3-tts.tts_pad_token_id", "qwen3-tts.tts.pad_token_id", "qwen3-tts.tts.pad_id"}, 151671);
    c_.think = (int)g.get_int({"qwen3-tts.codec.think_id", "qwen3-tts.codec_think_id"}, 2154);
    c_.nothink = (int)g.get_int({"qwen3-tts.codec.nothink_id", "qwen3-tts.codec_nothink_id"}, 2155);
    c_.think_bos = (int)g.get_int({"qwen3-tts.codec.think_bos_id", "qwen3-tts.codec_think_bos_id"}, 2156);
    c_.think_eos = (int)g.get_int({"qwen3-tts.codec.think_eos_id", "qwen3-tts.codec_think_eos_id"}, 2157);
    // code predictor architecture (falls back to the talker's values: 0.6B), tts_transformer.cpp:370-389
    c_.cp_hidden = (int)g.get_int({"qwen3-tts.code_predictor.embedding_length"}, c_.hidden);
    c_.cp_inter = (int)g.get_int({"qwen3-tts.code_predictor.feed_forward_length"}, c_.inter);
    c_.cp_heads = (int)g.get_int({"qwen3-tts.code_predictor.attention.head_count"}, c_.n_heads);
    c_.cp_kv = (int)g.get_int({"qwen3-tts.code_predictor.attention.head_count_kv"}, c_.n_kv);
    const int cp_head_dim = (int)g.get_int({"qwen3-tts.code_predictor.attention.key_length"}, c_.head_dim);
    c_.has_mtp = g.find("code_pred.mtp_proj.weight") != nullptr;
    if (c_.cp_hidden != c_.hidden && !c_.has_mtp) {
        set_error("code predictor hidden != talker hidden without code_pred.mtp_proj");
        return false;
    }
    if (cp_head_dim != c_.head_dim) { set_error("code predictor head_dim must equal the talker's (shared RoPE table)"); return false; }
    cpc_ = c_;
    cpc_.hidden = c_.cp_hidden; cpc_.inter = c_.cp_inter; cpc_.n_heads = c_.cp_heads; cpc_.n_kv = c_.cp_kv;
    // the batched matrix-core stack (hoisted norms, k_resid_norm) is built for widths <= 1024 and the 0.6B layout;
    // other models (1.7B) run every projection on the vector kernels with a 1-slot K split at any batch size
    mm_ok_ = !c_.has_mtp && c_.hidden <= 1024 && c_.cp_hidden <= 1024;
    fam1_ = mm_ok_ ? 0 : 1;
    if (c_.n_codebooks != 16) { set_error("n_codebooks must be 16"); return false; }
    // the fused code-predictor attention prologue is specialised to the 0.6B head layout (16 q / 8 kv heads x 128)
    cp_fused_attn_ = cp_fused_attn_ && c_.cp_heads == 16 && c_.cp_kv == 8 && c_.head_dim == 128 && c_.cp_hidden == 1024;
    return true;
}

bool Engine::load(const std::string &tts_gguf, const std::string &tok_gguf, int device, int max_slots, int max_ctx,
                  bool recv_weights) {
    DeviceLock lk(false, device);   // allocation zeroing / weight upload run kernels and copies on this device
    device_ = device;
    tts_path_ = tts_gguf;
    tok_path_ = tok_gguf;
    wa_.recv = recv_weights;
    opt_ = Options::from_env();
    cp_fused_attn_ = opt_.cp_fused_attn;
    defer_cp_select_ = opt_.defer_cp_select;
    fused_select_ = opt_.fused_select;
    persist_ = opt_.persist;
    poll_every_ = opt_.poll_every;
    max_slots_ = std::max(1, max_slots);
    max_ctx_ = std::max(32, max_ctx);
    if (max_ctx_ > ATTN_CHUNK * ATTN_MAX_SPLITS) { set_error("max_ctx exceeds " + std::to_string(ATTN_CHUNK * ATTN_MAX_SPLITS)); return false; }
    Q3T_HIP(hipSetDevice(device));
    Q3T_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    if (tts_gguf.empty()) {
        // vocoder-only context (AudioTokenizerDecoder / TRTVocoderDecoder load without a talker model)
        if (tok_gguf.empty()) { set_error("no model file given"); return false; }
        talker_ = false;
        voc_.reset(new Vocoder());
        if (!voc_->load(tok_gguf, stream_, recv_weights)) return false;
        Q3T_HIP(hipStreamSynchronize(stream_));
        return true;
    }
    Gguf g;
    if (!g.open(tts_gguf)) { set_error(g.error()); return false; }
    if (!parse_config(g)) return false;
    if (!upload_weights(g)) return false;
    if (!alloc_state()) return false;
#ifdef Q3T_DEV
    if (const char *e = std::getenv("Q3T_TALKER_LAYERS")) {   // truncated talker stack (development builds only)
        const int n = std::atoi(e);
        if (n > 0 && n < c_.n_layers) { c_.n_layers = n; L_.resize(n); }
    }
#endif
    if (!setup_persist()) return false;
    if (!setup_cpb()) return false;
    if (!setup_tkb()) return false;
    if (!tok_gguf.empty()) {
        voc_.reset(new Vocoder());
        if (!voc_->load(tok_gguf, stream_, recv_weights)) return false;
    }
    Q3T_HIP(hipStreamSynchronize(stream_));
    return true;
}

bool Engine::load_speaker_only(const std::string &tts_gguf, int device) {
    DeviceLock lk(false, device);
    device_ = device;
    tts_path_ = tts_gguf;
    talker_ = false;
    Q3T_HIP(hipSetDevice(device));
    Q3T_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    Gguf g;
    if (!g.open(tts_gguf)) { set_error(g.error()); return false; }
    size_t total = 0;
    for (const GgufTensor &t : g.tensors())
        if (t.name.rfind("spk_enc.", 0) == 0) total += (t.nbytes() + 255) & ~(size_t)255;
    if (total == 0) { set_error("No speaker encoder tensors found in model"); return false; }
    if (!wa_.reserve(total + ((size_t)1 << 20))) return false;
    spk_.reset(new SpeakerEncoder());
    if (!spk_->load(g, wa_, stream_)) return false;
    Q3T_HIP(hipStreamSynchronize(stream_));
    return true;
}

std::vector<WeightArena *> Engine::weight_arenas() {
    std::vector<WeightArena *> v{&wa_};
    if (voc_ && voc_->loaded()) v.push_back(&voc_->weights());
    return v;
}

bool Engine::upload_weights(const Gguf &g) { return layout_weights(g) && upload_weights_rest(); }

// every weight tensor into the arena, in a fixed order that depends on the GGUF shapes alone
bool Engine::layout_weights(const Gguf &g) {
    const int H = c_.hidden, D = c_.head_dim;
    // every weight goes into the arena (one blob: the unit of the RCCL broadcast); receiving ranks touch only the
    // GGUF headers, never the tensor bytes
    size_t total = 0;
    for (const GgufTensor &t : g.tensors()) total += (t.nbytes() + 255) & ~(size_t)255;
    if (!wa_.reserve(total + ((size_t)1 << 20))) return false;
    const bool recv = wa_.recv;
    auto up16 = [&](const char *name, int64_t cols, int64_t rows) -> uint16_t * {
        const GgufTensor *t = g.find(name);
        if (!check_shape(t, name, cols, rows, GGML_TYPE_F16)) return nullptr;
        uint16_t *d = wa_.alloc<uint16_t>((size_t)cols * rows);
        if (!d || !wa_.put(d, t->data, t->nbytes())) return nullptr;
        return d;
    };
    auto up32 = [&](const char *name, int64_t n) -> float * {
        const GgufTensor *t = g.find(name);
        if (!t || t->type != GGML_TYPE_F32 || t->nelements() != n) { set_error(std::string("bad f32 tensor ") + name); return nullptr; }
        float *d = wa_.alloc<float>((size_t)n);
        if (!d || !wa_.put(d, t->data, t->nbytes())) return nullptr;
        return d;
    };
    auto rows16 = [&](const std::string &name, int64_t cols, int64_t rows, std::vector<uint16_t> &dst, size_t at) -> bool {
        const GgufTensor *t = g.find(name);
        if (!check_shape(t, name.c_str(), cols, rows, GGML_TYPE_F16)) return false;
        if (!recv) std::memcpy(dst.data() + at, t->data, t->nbytes());
        return true;
    };
    auto layer = [&](const char *pfx, int i, DevLayer &l, const Config &lc) -> bool {
        const int H = lc.hidden, Dq = lc.n_heads * D, Dkv = lc.n_kv * D, I = lc.inter;
        if (I % 16 != 0 || H % 8 != 0) { set_error("unsupported hidden/intermediate size"); return false; }
        char b[160];
        auto nm = [&](const char *s) { snprintf(b, sizeof b, "%s.blk.%d.%s", pfx, i, s); return std::string(b); };
        // fused [Wq; Wk; Wv] rows
        const size_t n_qkv = (size_t)(Dq + 2 * Dkv) * H;
        std::vector<uint16_t> qkv(recv ? 0 : n_qkv);
        if (!rows16(nm("attn_q.weight"), H, Dq, qkv, 0) || !rows16(nm("attn_k.weight"), H, Dkv, qkv, (size_t)Dq * H) ||
            !rows16(nm("attn_v.weight"), H, Dkv, qkv, (size_t)(Dq + Dkv) * H))
            return false;
        if (!(l.qkv = wa_.alloc<uint16_t>(n_qkv)) || !wa_.put(l.qkv, qkv.data(), n_qkv * 2)) return false;
        // gate/up interleaved in 16-row blocks (k_gemv ACT_SWIGLU layout)
        const size_t n_gu = (size_t)2 * I * H;
        std::vector<uint16_t> gate(recv ? 0 : (size_t)I * H), up(recv ? 0 : (size_t)I * H), gu(recv ? 0 : n_gu);
        if (!rows16(nm("ffn_gate.weight"), H, I, gate, 0) || !rows16(nm("ffn_up.weight"), H, I, up, 0)) return false;
        if (!recv)
            for (int blk = 0; blk < I / 16; ++blk) {
                std::memcpy(gu.data() + (size_t)(blk * 32) * H, gate.data() + (size_t)(blk * 16) * H, (size_t)16 * H * 2);
                std::memcpy(gu.data() + (size_t)(blk * 32 + 16) * H, up.data() + (size_t)(blk * 16) * H, (size_t)16 * H * 2);
            }
        if (!(l.gu = wa_.alloc<uint16_t>(n_gu)) || !wa_.put(l.gu, gu.data(), n_gu * 2)) return false;
        if (!(l.o = up16(nm("attn_output.weight").c_str(), Dq, H))) return false;
        if (!(l.down = up16(nm("ffn_down.weight").c_str(), I, H))) return false;
        if (!(l.attn_norm = up32(nm("attn_norm.weight").c_str(), H))) return false;
        if (!(l.ffn_norm = up32(nm("ffn_norm.weight").c_str(), H))) return false;
        if (!(l.qn = up32(nm("attn_q_norm.weight").c_str(), D))) return false;
        if (!(l.kn = up32(nm("attn_k_norm.weight").c_str(), D))) return false;
        return true;
    };
    L_.resize(c_.n_layers);
    CP_.resize(c_.cp_layers);
    for (int i = 0; i < c_.n_layers; ++i) if (!layer("talker", i, L_[i], c_)) return false;
    for (int i = 0; i < c_.cp_layers; ++i) if (!layer("code_pred", i, CP_[i], cpc_)) return false;
    if (c_.has_mtp) {   // code_pred.mtp_proj (1.7B): tts_transformer.cpp:611-616, 709-712
        if (!(mtp_ = up16("code_pred.mtp_proj.weight", H, c_.cp_hidden))) return false;
        if (g.find("code_pred.mtp_proj.bias") && !(mtp_b_ = up32("code_pred.mtp_proj.bias", c_.cp_hidden))) return false;
    }
    if (!(text_embd_ = up16("talker.text_embd.weight", c_.text_dim, c_.text_vocab))) return false;
    if (!(fc1_ = up16("talker.text_proj.fc1.weight", c_.text_dim, c_.text_dim))) return false;
    if (!(fc2_ = up16("talker.text_proj.fc2.weight", c_.text_dim, H))) return false;
    if (!(fc1_b_ = up32("talker.text_proj.fc1.bias", c_.text_dim))) return false;
    if (!(fc2_b_ = up32("talker.text_proj.fc2.bias", H))) return false;
    if (!(codec_embd_ = up16("talker.codec_embd.weight", H, c_.codec_vocab))) return false;
    if (!(codec_head_ = up16("talker.codec_head.weight", H, c_.codec_vocab))) return false;
    if (!(out_norm_ = up32("talker.output_norm.weight", H))) return false;
    if (!(cp_out_norm_ = up32("code_pred.output_norm.weight", c_.cp_hidden))) return false;
    cp_embd_.resize(15);
    cp_head_.resize(15);
    for (int i = 0; i < 15; ++i) {
        char b[96];
        snprintf(b, sizeof b, "code_pred.codec_embd.%d.weight", i);
        if (!(cp_embd_[i] = up16(b, H, c_.cp_vocab))) return false;
        snprintf(b, sizeof b, "code_pred.lm_head.%d.weight", i);
        if (!(cp_head_[i] = up16(b, c_.cp_hidden, c_.cp_vocab))) return false;
    }
    // speaker encoder (ECAPA-TDNN, audio_tokenizer_encoder.cpp): optional, the GGUF's spk_enc.* tensors
    if (g.find("spk_enc.conv0.weight")) {
        spk_.reset(new SpeakerEncoder());
        if (!spk_->load(g, wa_, stream_)) return false;
    }
    return true;
}

// the weight arena of a model file laid out on the host only (WeightArena::plan): the offsets of every allocation in
// order and the bytes used -- what every rank of a shared start-up computes from the GGUF headers before the RCCL
// broadcast (comm_bcast_arenas checks the sizes; tests/test_dist_cpu.py compares whole layouts across gloo ranks)
bool Engine::plan_layout(const std::string &tts_gguf, std::vector<size_t> &offsets, size_t &used) {
    Gguf g;
    if (!g.open(tts_gguf)) { set_error(g.error()); return false; }
    if (!parse_config(g)) return false;
    wa_.plan = wa_.recv = true;
    wa_.trace = &offsets;
    const bool ok = layout_weights(g);
    wa_.trace = nullptr;
    used = wa_.used;
    return ok;
}

bool Engine::upload_weights_rest() {
    const int D = c_.head_dim;
    // the 16 tables of the step embedding: codec_embd (code 0) + code_pred.codec_embd[0..14] (codes 1..15)
    std::vector<uint16_t *> tabs16(16);
    tabs16[0] = codec_embd_;
    for (int i = 0; i < 15; ++i) tabs16[1 + i] = cp_embd_[i];
    tabs16_dev_ = dalloc<uint16_t *>(16);
    Q3T_HIP(hipMemcpyAsync(tabs16_dev_, tabs16.data(), 16 * sizeof(uint16_t *), hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    // RoPE cos/sin table with ggml_rope_cache_init's f32 recurrence (theta *= theta_scale), NEOX pairs
    rope_len_ = std::max(max_ctx_, 16);
    std::vector<float> rope((size_t)rope_len_ * D);
    const float theta_scale = powf(c_.rope_theta, -2.0f / (float)D);
    for (int p = 0; p < rope_len_; ++p) {
        float theta = (float)p;
        for (int i0 = 0; i0 < D; i0 += 2) {
            rope[(size_t)p * D + i0] = cosf(theta);
            rope[(size_t)p * D + i0 + 1] = sinf(theta);
            theta *= theta_scale;
        }
    }
    rope_ = dalloc<float>(rope.size());
    Q3T_HIP(hipMemcpyAsync(rope_, rope.data(), rope.size() * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    return true;
}

bool Engine::alloc_state() {
    const int S = max_slots_, H = c_.hidden, D = c_.head_dim;
    const int QKV = std::max(c_.n_heads + 2 * c_.n_kv, c_.cp_heads + 2 * c_.cp_kv) * D;   // talker / code predictor
    const int max_splits = (max_ctx_ + ATTN_CHUNK - 1) / ATTN_CHUNK;
    max_trailing_ = 512;
    x_ = dalloc<float>((size_t)S * H);
    qkv_ = dalloc<float>((size_t)S * QKV);
    logits_ = dalloc<float>((size_t)S * c_.codec_vocab);
    hidden_ = dalloc<float>((size_t)S * H);
    cpx_ = dalloc<float>((size_t)S * c_.cp_hidden);
    cp_in1_ = dalloc<float>((size_t)S * H);
    cp_logits_ = dalloc<float>((size_t)S * c_.cp_vocab);
    // (the code-predictor stack runs attn_decode on these too: sized for the wider of the two head layouts)
    part_ = dalloc<float>((size_t)S * std::max(c_.n_heads, c_.cp_heads) * max_splits * (D + 2));
    ticket_ = dalloc<unsigned>((size_t)S * std::max(c_.n_kv, c_.cp_kv));
    sel_ticket_ = dalloc<unsigned>((size_t)S);
    attn_ = dalloc<uint16_t>((size_t)S * std::max(c_.n_heads, c_.cp_heads) * D);
    hmlp_ = dalloc<uint16_t>((size_t)S * std::max(c_.inter, c_.cp_inter));
    xn_ = dalloc<uint16_t>((size_t)S * H);
    parts_ = dalloc<float>((size_t)4 * S * H);
    const size_t kv_layer = (size_t)S * c_.n_kv * max_ctx_ * D;
    kc_ = dalloc<uint16_t>(kv_layer * c_.n_layers);
    vc_ = dalloc<uint16_t>(kv_layer * c_.n_layers);
    const size_t cpkv_layer = (size_t)S * c_.cp_kv * 16 * D;
    cpkc_ = dalloc<uint16_t>(cpkv_layer * c_.cp_layers);
    cpvc_ = dalloc<uint16_t>(cpkv_layer * c_.cp_layers);
    pos_ = dalloc<int>(S);
    frame_ = dalloc<int>(S);
    done_ = dalloc<int>(S);
    token_ = dalloc<int>(S);
    tokens_ = dalloc<int>((size_t)S * 16);
    n_tokens_ = dalloc<int>(S);
    force_ = dalloc<int>(S);
    trailing_len_ = dalloc<int>(S);
    cp_pos_ = dalloc<int>((size_t)16 * S);
    seen_ = dalloc<uint8_t>((size_t)S * c_.codec_vocab);
    utt_ = dalloc<uint64_t>(S);
    seed_dev_ = dalloc<uint64_t>(1);
    slot_iota_ = dalloc<int>(S);
    trailing_ = dalloc<float>((size_t)S * max_trailing_ * H);
    tts_pad_ = dalloc<float>((size_t)S * H);
    prefill_ = dalloc<float>((size_t)S * 10 * H);
    codes_max_len_ = max_ctx_;
    codes_ = dalloc<int32_t>((size_t)S * codes_max_len_ * 16);
    proj_cap_ = S * (max_trailing_ + 16);
    proj_idx_ = dalloc<int>(proj_cap_);
    proj_h_ = dalloc<uint16_t>((size_t)proj_cap_ * c_.text_dim);
    proj_out_ = dalloc<float>((size_t)proj_cap_ * H);
    recipe_cap_ = S * (max_trailing_ + 16);
    recipe_ = dalloc<RowRecipe>(recipe_cap_);
    if (!x_ || !kc_ || !vc_ || !recipe_ || !proj_out_) { set_error("device allocation failed"); return false; }
    std::vector<int> cpp((size_t)16 * S);
    for (int p = 0; p < 16; ++p) for (int s = 0; s < S; ++s) cpp[(size_t)p * S + s] = p;
    Q3T_HIP(hipMemcpyAsync(cp_pos_, cpp.data(), cpp.size() * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    std::vector<uint64_t> utt(S);
    for (int s = 0; s < S; ++s) utt[s] = (uint64_t)s;
    Q3T_HIP(hipMemcpyAsync(utt_, utt.data(), S * 8, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    std::vector<int> iota(S);
    for (int s = 0; s < S; ++s) iota[s] = s;
    Q3T_HIP(hipMemcpyAsync(slot_iota_, iota.data(), S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    return true;
}

// the persistent single-slot talker step (persist.hip): layer pointer table + zeroed hand-off state; off when the
// shapes or the device do not match what the kernel is built for (the launch-per-phase graph is used then)
bool Engine::setup_persist() {
    int n_cu = 0;
    Q3T_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device_));
    const bool use = persist_ && fused_select_;
    persist_ = use && persist_supported(c_.hidden, c_.n_heads, c_.n_kv, c_.head_dim, c_.inter, c_.codec_vocab, max_ctx_, n_cu);
    // the code-predictor frame needs the 0.6B code-predictor shapes only: the 1.7B one (a 2,048-wide talker) runs it
    // too, on projected table rows (build_cp_proj_table) with a projected pass-0 input
    const bool cp_ok = use && opt_.persist_cp && c_.cp_vocab == 2048 && c_.codec_vocab == 3072 && CP_.size() >= 1 &&
                       CP_.size() <= 32 && cp_head_.size() == 15 && c_.cp_hidden == 1024 && c_.cp_inter == 3072 &&
                       c_.cp_heads == 16 && c_.cp_kv == 8 && c_.head_dim == 128 && n_cu >= 256;
    // every instantiation must fit one workgroup per CU on this device (occupancy query with its LDS request)
    persist_ = persist_ && persist_resident(device_, max_ctx_, cp_ok);
    persist_cp_ = cp_ok && persist_resident_cp(device_);
    cp_roles_ = persist_cp_ && opt_.cp_roles && c_.cp_layers == 5 && persist_cp_roles_resident(device_);
    tk_roles_ = persist_ && opt_.tk_roles && persist_chunk(max_ctx_) == 64 && persist_tk_roles_supported(max_ctx_) &&
                persist_tk_roles_resident(device_, max_ctx_);
    if (!persist_ && !persist_cp_) return wa_.recv || build_persist_tables();   // (the batched path's table)
    pstate_ = dalloc<uint8_t>(persist_state_bytes());
    if (!pstate_) { set_error("device allocation failed"); return false; }
    if (persist_) {
        std::vector<PLayerW> pl(L_.size());
        for (size_t i = 0; i < L_.size(); ++i)
            pl[i] = PLayerW{L_[i].qkv, L_[i].o, L_[i].gu, L_[i].down, L_[i].attn_norm, L_[i].ffn_norm, L_[i].qn, L_[i].kn};
        pl_dev_ = dalloc<PLayerW>(pl.size());
        if (!pl_dev_) { set_error("device allocation failed"); return false; }
        Q3T_HIP(hipMemcpyAsync(pl_dev_, pl.data(), pl.size() * sizeof(PLayerW), hipMemcpyHostToDevice, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
    }
    // the code-predictor frame (persist_cp_frame): its 5 layers and 15 lm_heads
    if (persist_cp_) {
        std::vector<PLayerW> cpl(CP_.size());
        for (size_t i = 0; i < CP_.size(); ++i)
            cpl[i] = PLayerW{CP_[i].qkv, CP_[i].o, CP_[i].gu, CP_[i].down, CP_[i].attn_norm, CP_[i].ffn_norm, CP_[i].qn, CP_[i].kn};
        pl_cp_dev_ = dalloc<PLayerW>(cpl.size());
        heads_dev_ = dalloc<const uint16_t *>(16);
        if (!pl_cp_dev_ || !heads_dev_) { set_error("device allocation failed"); return false; }
        Q3T_HIP(hipMemcpyAsync(pl_cp_dev_, cpl.data(), cpl.size() * sizeof(PLayerW), hipMemcpyHostToDevice, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
        std::vector<const uint16_t *> hp(cp_head_.begin(), cp_head_.end());
        Q3T_HIP(hipMemcpyAsync(heads_dev_, hp.data(), hp.size() * sizeof(void *), hipMemcpyHostToDevice, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
        // the per-token tables are computed from the weights: a receiving context (replica, non-root rank) builds
        // them once its arena has been filled (finish_weights, after copy_weights_from / the RCCL broadcast)
        if (!wa_.recv && !build_persist_tables()) return false;
    }
    // (pstate_ was zeroed on the context stream by dalloc)
#ifdef Q3T_DEV
    if (std::getenv("Q3T_PERSIST_PROF")) pprof_ = dalloc<uint64_t>((size_t)PROF_WG * PROF_PH * 4);
#endif
    return true;
}

// the batched code-predictor frame (persist_cpb.hip): the 0.6B code-predictor shapes on the matrix-core family, with
// layer 0 of passes 1..15 from the per-token QKV table (as decoder_stack_mm reads it), on a device that holds its 256
// workgroups at one per CU
bool Engine::setup_cpb() {
    int n_cu = 0;
    Q3T_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device_));
    cpb_ = opt_.cpb && mm_ok_ && max_slots_ > 1 && opt_.mm_cp_table && opt_.cp_qkv_table && !c_.has_mtp &&
           c_.cp_vocab == 2048 && c_.codec_vocab == 3072 && CP_.size() == 5 && cp_head_.size() == 15 && cp_embd_.size() >= 14 &&
           c_.cp_hidden == 1024 && c_.hidden == 1024 && c_.cp_inter == 3072 && c_.cp_heads == 16 && c_.cp_kv == 8 &&
           c_.head_dim == 128 && n_cu >= 256 && cpb_resident(device_);
    if (!cpb_) return true;
    cpb_state_ = dalloc<uint8_t>(cpb_state_bytes());
    if (!cpb_state_) { set_error("device allocation failed"); return false; }
#ifdef Q3T_DEV
    if (std::getenv("Q3T_PERSIST_PROF") && !pprof_) pprof_ = dalloc<uint64_t>((size_t)PROF_WG * PROF_PH * 4);
#endif
    if (!pl_cp_dev_) {
        std::vector<PLayerW> cpl(CP_.size());
        for (size_t i = 0; i < CP_.size(); ++i)
            cpl[i] = PLayerW{CP_[i].qkv, CP_[i].o, CP_[i].gu, CP_[i].down, CP_[i].attn_norm, CP_[i].ffn_norm, CP_[i].qn, CP_[i].kn};
        pl_cp_dev_ = dalloc<PLayerW>(cpl.size());
        if (!pl_cp_dev_) { set_error("device allocation failed"); return false; }
        Q3T_HIP(hipMemcpyAsync(pl_cp_dev_, cpl.data(), cpl.size() * sizeof(PLayerW), hipMemcpyHostToDevice, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
    }
    if (!heads_dev_) {
        heads_dev_ = dalloc<const uint16_t *>(16);
        if (!heads_dev_) { set_error("device allocation failed"); return false; }
        std::vector<const uint16_t *> hp(cp_head_.begin(), cp_head_.end());
        Q3T_HIP(hipMemcpyAsync(heads_dev_, hp.data(), hp.size() * sizeof(void *), hipMemcpyHostToDevice, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
    }
    return true;
}
// the batched talker step (persist_tkb.hip): the 0.6B talker shapes on the matrix-core family, on a device that holds its
// 256 workgroups at one per CU
bool Engine::setup_tkb() {
    int n_cu = 0;
    Q3T_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device_));
    tkb_ = opt_.tkb && mm_ok_ && max_slots_ > 1 && !c_.has_mtp && c_.n_layers == 28 && c_.hidden == 1024 &&
           c_.n_heads == 16 && c_.n_kv == 8 && c_.head_dim == 128 && c_.inter == 3072 && c_.codec_vocab == 3072 &&
           n_cu >= 256 && tkb_resident(device_);
    if (!tkb_) return true;
    tkb_state_ = dalloc<uint8_t>(tkb_state_bytes());
    if (!tkb_state_) { set_error("device allocation failed"); return false; }
#ifdef Q3T_DEV
    if (std::getenv("Q3T_PERSIST_PROF") && !pprof_) pprof_ = dalloc<uint64_t>((size_t)PROF_WG * PROF_PH * 4);
#endif
    if (!pl_dev_) {
        std::vector<PLayerW> pl(L_.size());
        for (size_t i = 0; i < L_.size(); ++i)
            pl[i] = PLayerW{L_[i].qkv, L_[i].o, L_[i].gu, L_[i].down, L_[i].attn_norm, L_[i].ffn_norm, L_[i].qn, L_[i].kn};
        pl_dev_ = dalloc<PLayerW>(pl.size());
        if (!pl_dev_) { set_error("device allocation failed"); return false; }
        Q3T_HIP(hipMemcpyAsync(pl_dev_, pl.data(), pl.size() * sizeof(PLayerW), hipMemcpyHostToDevice, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
    }
    return true;
}
// the slot counts the step serves: the per-op family it reproduces (decoder_stack_mm with k_attn_seq: >= 16 policy
// slots, no forced split attention; split-K 4 for every S_main of these shapes)
bool Engine::use_tkb(int S) const {
    const int S_main = policy_slots_ > 0 ? policy_slots_ : S;
    return tkb_ && use_mm(S) && S <= 64 && S_main >= 16 && S_main <= 64 && !opt_.attn_split;
}
// the slot counts the frame serves: the matrix-core family (decoder_stack_mm) with the split-K of <= 64 slots
bool Engine::use_cpb(int S) const {
    const int S_main = policy_slots_ > 0 ? policy_slots_ : S;
    return cpb_ && cp_qkvtab_ && use_mm(S) && S <= 64 && S_main <= 64;
}

// The code predictor's per-token tables (the layer-0 QKV rows, 520 MB of f32; 1.7B: the projected pass inputs, 130 MB)
// are functions of the weights alone.  One copy per device serves every context that loaded the same weight file
// (path, size and modification time: replicas and test contexts of one model), built by the first of them on its own
// stream and freed with the last one's destruction -- no per-context copy, and no free outside context destruction:
// hipFree synchronises the whole device, and a free while other contexts' threads capture graphs invalidated those
// captures (round 4).
struct CpTables {
    int device = -1;
    std::string key;
    float *qkv = nullptr, *proj = nullptr;
    size_t bytes = 0;
    bool built = false;
    std::mutex build;   // held by the building context; later users wait for the finished tables
    // drop whatever a failed build allocated, so the next context with the same key starts from scratch (no leaked HBM,
    // no bytes counted twice)
    void reset() {
        int prev = -1;
        hipGetDevice(&prev);
        if (device >= 0) hipSetDevice(device);
        if (qkv) hipFree(qkv);
        if (proj) hipFree(proj);
        qkv = proj = nullptr;
        bytes = 0;
        if (prev >= 0) hipSetDevice(prev);   // the caller's current device is restored
    }
    ~CpTables() { reset(); }
};
namespace {
std::mutex g_cp_tables_m;
std::vector<std::weak_ptr<CpTables>> g_cp_tables;
std::shared_ptr<CpTables> cp_tables_for(int device, const std::string &key) {
    std::lock_guard<std::mutex> g(g_cp_tables_m);
    for (auto it = g_cp_tables.begin(); it != g_cp_tables.end();) {
        if (auto t = it->lock()) {
            if (t->device == device && t->key == key) return t;
            ++it;
        } else {
            it = g_cp_tables.erase(it);
        }
    }
    auto t = std::make_shared<CpTables>();
    t->device = device;
    t->key = key;
    g_cp_tables.push_back(t);
    return t;
}
}  // namespace

size_t cp_tables_live_bytes(int device) {   // development / test accounting
    std::lock_guard<std::mutex> g(g_cp_tables_m);
    size_t b = 0;
    for (auto &w : g_cp_tables)
        if (auto t = w.lock())
            if (t->device == device) b += t->bytes;
    return b;
}

// Built whenever a path reads them: the persistent frame (persist_cp_), or the batched code predictor
// (Q3T_MM_CP_TABLE, 0.6B shapes), so the batched arithmetic depends on the shapes and options, not on whether this
// device runs persistent kernels.
bool Engine::build_persist_tables() {
    if (tables_built_) return true;
    const bool qkv_shapes = opt_.cp_qkv_table && c_.codec_vocab == 3072 && c_.cp_vocab == 2048 && (int)cp_embd_.size() >= 14 &&
                            cpc_.hidden == 1024 && (int)CP_.size() >= 1;
    const bool want_proj = persist_cp_ && c_.has_mtp;
    const bool want_qkv = qkv_shapes && (persist_cp_ || (opt_.mm_cp_table && mm_ok_ && max_slots_ > 1));
    if (!want_proj && !want_qkv) { tables_built_ = true; return true; }
    struct stat st{};
    if (stat(tts_path_.c_str(), &st) != 0) { set_error("stat failed: " + tts_path_); return false; }
    const std::string key = tts_path_ + "|" + std::to_string((long long)st.st_size) + "|" + std::to_string((long long)st.st_mtime) +
                            (want_proj ? "|proj" : "") + (want_qkv ? "|qkv" : "");
    cp_tables_ = cp_tables_for(device_, key);
    std::lock_guard<std::mutex> g(cp_tables_->build);
    if (!cp_tables_->built) {
        // any failure below leaves the entry empty (not half-built) for the next context of this key
        struct Undo {
            CpTables *t;
            bool armed = true;
            ~Undo() { if (armed) t->reset(); }
        } undo{cp_tables_.get()};
        table_iota_ = dalloc<int>(c_.codec_vocab);
        if (!table_iota_) { set_error("device allocation failed (table token iota)"); return false; }
        std::vector<int> ih(c_.codec_vocab);
        for (int i = 0; i < c_.codec_vocab; ++i) ih[i] = i;
        Q3T_HIP(hipMemcpyAsync(table_iota_, ih.data(), ih.size() * 4, hipMemcpyHostToDevice, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
        const int QKV = (cpc_.n_heads + 2 * cpc_.n_kv) * cpc_.head_dim;
        const size_t rows = persist_qkv_table_rows();
        if (want_qkv) {
            if (hipMalloc(&cp_tables_->qkv, rows * QKV * sizeof(float)) != hipSuccess) {
                cp_tables_->qkv = nullptr;
                set_error("device allocation failed (code-predictor QKV table)");
                return false;
            }
            cp_tables_->bytes += rows * QKV * sizeof(float);
        }
        if (want_proj) {
            if (hipMalloc(&cp_tables_->proj, rows * c_.cp_hidden * sizeof(float)) != hipSuccess) {
                cp_tables_->proj = nullptr;
                set_error("device allocation failed (code-predictor projected table)");
                return false;
            }
            cp_tables_->bytes += rows * c_.cp_hidden * sizeof(float);
        }
        cp_qkvtab_ = cp_tables_->qkv;
        cp_projtab_ = cp_tables_->proj;
        if (want_proj && !build_cp_proj_table()) return false;
        if (want_qkv && !build_cp_qkv_table()) return false;
        cp_tables_->built = true;
        undo.armed = false;
    }
    cp_qkvtab_ = cp_tables_->qkv;
    cp_projtab_ = cp_tables_->proj;
    tables_built_ = true;
    return true;
}

bool Engine::finish_weights() {
    DeviceLock lk(false, device_);
    Q3T_HIP(hipSetDevice(device_));
    Q3T_HIP(hipStreamSynchronize(stream_));   // the arena fill (copy or broadcast) ran on this stream
    return build_persist_tables();
}

// Layer 0 of code-predictor passes 1..15 starts from a table row (codec_embd / code_pred.codec_embd[p-2]), so its
// raw QKV row is a function of the token alone: computed here once for every token of the 15 tables with the per-op
// pass-input GEMV (PRO_RMS_G1, the K split of a 1-slot step: family_b = 1), whose arithmetic the persistent frame's
// phase A reproduces bit for bit.  The persistent frame then reads the row instead of running layer 0's norm + QKV
// phase and its all-to-all edge (persist.hip).  520 MB of f32.
bool Engine::build_cp_qkv_table() {
    const int H = cpc_.hidden, QKV = (cpc_.n_heads + 2 * cpc_.n_kv) * cpc_.head_dim;
    const int *iota = table_iota_;
    size_t row0 = 0;
    for (int t = 0; t < 15; ++t) {
        const int V = t == 0 ? c_.codec_vocab : c_.cp_vocab;
        GemvParams g;
        g.W = CP_[0].qkv; g.N = QKV; g.K = H; g.B = V;
        g.pro = PRO_RMS_G1; g.nw = CP_[0].attn_norm; g.eps = c_.eps;
        g.gs.tok = iota; g.gs.tok_ld = 1; g.gs.tok_col0 = 0;
        g.gs.tab0 = t == 0 ? codec_embd_ : cp_embd_[t - 1];
        if (cp_projtab_) {   // 1.7B: layer 0 normalises the projected row (the per-op path's PRO_RMS on cpx_)
            g.pro = PRO_RMS; g.x = cp_projtab_ + row0 * H; g.ldx = H;
        }
        g.out_f32 = cp_qkvtab_ + row0 * QKV; g.ldo = QKV;
        g.family_b = 1;
        if (!gemv(g, stream_)) return false;
        row0 += V;
    }
    Q3T_HIP(hipStreamSynchronize(stream_));
    return true;
}

// 1.7B: every code-predictor pass input is mtp_proj . f16(row) + b of a talker-space row; for passes 1..15 the row is a
// table row, so the projected input is a function of the token: computed once here for the 15 tables with the per-op
// path's own launches (k_gather_sum + the mtp_proj GEMV with a 1-slot K split), the persistent frame then reads it
// (130 MB of f32).
bool Engine::build_cp_proj_table() {
    const int H = c_.hidden, CH = c_.cp_hidden;
    const int *iota = table_iota_;
    // scratch rows: the QKV table's first codec_vocab x H floats when it exists (written after this build), else kept
    float *rowbuf = cp_qkvtab_ ? cp_qkvtab_ : dalloc<float>((size_t)c_.codec_vocab * H);
    if (!cp_projtab_ || !rowbuf) { set_error("device allocation failed (code-predictor projected table)"); return false; }
    size_t row0 = 0;
    for (int t = 0; t < 15; ++t) {
        const int V = t == 0 ? c_.codec_vocab : c_.cp_vocab;
        GatherSum gs;
        gs.tok = iota; gs.tok_ld = 1; gs.tok_col0 = 0;
        gs.tab0 = t == 0 ? codec_embd_ : cp_embd_[t - 1];
        if (!gather_sum(gs, 1, V, H, rowbuf, H, stream_)) return false;
        GemvParams g;
        g.W = mtp_; g.N = CH; g.K = H; g.B = V;
        g.pro = PRO_F32; g.x = rowbuf; g.ldx = H;
        g.bias = mtp_b_;
        g.out_f32 = cp_projtab_ + row0 * CH; g.ldo = CH; g.family_b = 1;
        if (!gemv(g, stream_)) return false;
        row0 += V;
    }
    Q3T_HIP(hipStreamSynchronize(stream_));
    return true;
}

bool Engine::persist_recover() {
    Q3T_HIP(hipStreamSynchronize(stream_));
    fprintf(stderr, "[q3t] persistent kernel flagged an in-launch hand-off fault on device %d: "
                    "falling back to the launch-per-op graphs for this context\n", device_);
    if (pstate_) Q3T_HIP(hipMemsetAsync(pstate_, 0, persist_state_bytes(), stream_));   // ordered before the re-run on stream_
    if (cpb_state_ && !cpb_clear(cpb_state_, stream_)) return false;
    if (tkb_state_ && !tkb_clear(tkb_state_, stream_)) return false;
    Q3T_HIP(hipStreamSynchronize(stream_));
    for (auto &kv : g_talker_) hipGraphExecDestroy(kv.second);
    for (auto &kv : g_frame_) hipGraphExecDestroy(kv.second);
    for (auto &kv : g_cp_) hipGraphExecDestroy(kv.second);
    g_talker_.clear(); g_frame_.clear(); g_cp_.clear();
    persist_ = persist_cp_ = cp_roles_ = tk_roles_ = cpb_ = tkb_ = false;
    // the tables (serving only the persistent frame) stay allocated until the context is destroyed: a hipFree here
    // would synchronise the device and invalidate graph captures other contexts' threads have in progress
    // the per-op code predictor with its attention as its own launch reproduces the persistent frame bit for bit
    // (as does the per-op talker step for n_ctx <= 2048), so a re-run regenerates the frames already delivered exactly
    cp_fused_attn_ = false;
    persist_fallback_ = true;
    return true;
}

#ifdef Q3T_DEV
bool Engine::debug_read(int which, void *dst, size_t bytes) {
    if (which == 5 && pprof_) {   // persistent-step timeline (dev)
        Q3T_HIP(hipStreamSynchronize(stream_));
        Q3T_HIP(hipMemcpy(dst, pprof_, std::min<size_t>(bytes, (size_t)PROF_WG * PROF_PH * 4 * 8), hipMemcpyDeviceToHost));
        return true;
    }
    if (which == 4 && !pstate_) {   // launch-per-phase attention partial buffer (dev dumps)
        Q3T_HIP(hipStreamSynchronize(stream_));
        Q3T_HIP(hipMemcpy(dst, part_, std::min<size_t>(bytes, (size_t)max_slots_ * c_.n_heads * ((max_ctx_ + ATTN_CHUNK - 1) / ATTN_CHUNK) * (c_.head_dim + 2) * 4), hipMemcpyDeviceToHost));
        return true;
    }
    if (which == 4 && pstate_) {   // persistent-step partial buffer (dev dumps)
        PersistParams pp;
        persist_carve(pstate_, pp);
        Q3T_HIP(hipStreamSynchronize(stream_));
        Q3T_HIP(hipMemcpy(dst, pp.part, std::min<size_t>(bytes, 8 * 32 * 2 * 130 * 4), hipMemcpyDeviceToHost));
        return true;
    }
    const void *src = which == 0 ? (const void *)kc_ : which == 1 ? (const void *)vc_ : which == 2 ? (const void *)qkv_ : (const void *)attn_;
    const size_t kvb = (size_t)max_slots_ * c_.n_kv * max_ctx_ * c_.head_dim * c_.n_layers * 2;
    const size_t cap = which <= 1 ? kvb : which == 2 ? (size_t)max_slots_ * (c_.n_heads + 2 * c_.n_kv) * c_.head_dim * 4
                                                     : (size_t)max_slots_ * c_.n_heads * c_.head_dim * 2;
    if (which < 0 || which > 3 || bytes > cap) { set_error("debug_read: bad buffer or size"); return false; }
    Q3T_HIP(hipStreamSynchronize(stream_));
    Q3T_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return true;
}
#endif

// test hook (Q3T_PERSIST_FAULT_AT=n): the graph replay that contains the n-th persistent launch of this context runs
// with the abort word already set, exactly as if one of its hand-off waits had given up.  Host-side on purpose: a
// device-side launch counter in k_persist's prologue cost 32 us per talker step in code generation alone.
bool Engine::persist_fault_hook(int S, int n_launches) {
    if (!opt_.persist_fault_at || S != 1 || !persist_enabled() || !pstate_) return true;
    const unsigned before = persist_launches_;
    persist_launches_ += (unsigned)n_launches;
    if (before < opt_.persist_fault_at && opt_.persist_fault_at <= persist_launches_) {
        PersistParams p;
        persist_carve(pstate_, p);
        Q3T_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(p.err), 1, 1, stream_));
    }
    return true;
}

bool Engine::persist_error() {
    if (cpb_ && cpb_state_) {
        bool e = false;
        if (!cpb_error(cpb_state_, stream_, &e) || e) return true;
    }
    if (tkb_ && tkb_state_) {
        bool e = false;
        if (!tkb_error(tkb_state_, stream_, &e) || e) return true;
    }
    if (!(persist_ || persist_cp_) || !pstate_) return false;
    PersistParams p;
    persist_carve(pstate_, p);
    // on the context's own (non-blocking) stream: a null-stream copy would order against, and break, graph captures
    // in progress on other threads' streams
    unsigned e = 0;
    if (hipMemcpyAsync(&e, p.err, 4, hipMemcpyDeviceToHost, stream_) != hipSuccess || hipStreamSynchronize(stream_) != hipSuccess)
        return true;
    return e != 0;
}

struct StackInput {
    int pro = PRO_RMS;
    bool prenormed = false;              // batched: x / xn already hold layer 0's input (select_embed_norm)
    const float *x = nullptr;
    GatherSum gs;
    SelectSpec sel;                      // PRO_SEL_G1: selection of the gathered token
    const float *sel_logits = nullptr;
};

// ------------------------------------------------------------------------------------------ batched decoder stack
// matrix-core path (S >= gemm_mfma_min_batch()): 7 launches per layer so that every projection fills the chip:
//   [QKV GEMM on xn] [attention] [O GEMM, split-K slabs] [resid + RMSNorm(ffn) -> xn] [gate/up GEMM + SwiGLU]
//   [down GEMM, split-K slabs] [resid + RMSNorm(next attn_norm | final norm) -> xn]
// The norms are hoisted out of the GEMM prologues (each projection workgroup used to recompute the norm of its
// tokens: ~12 us of chained double math per launch at 64 slots) and the N = 1024 projections split K four ways
// (32 row tiles x 2 token tiles would leave 192 of 256 CUs idle).  final_norm null: no normalisation after the last
// layer (code-predictor pass 0 has no head).
static int splitk_for(int N, int S, int K) {
    const int tiles = (N / 32) * ((S + 31) / 32), nch = K / 256;
    // K chunks per slice must be one of the GEMM kernel's instantiations (gemm_mfma_supported)
    auto ok = [&](int ks) { const int nk = nch % ks == 0 ? nch / ks : 0; return nk == 1 || nk == 2 || nk == 3 || nk == 4 || nk == 8 || nk == 12; };
    for (int ks : {1, 2, 3, 4})
        if (ok(ks) && tiles * ks >= 256) return ks;
    for (int ks : {4, 3, 2})
        if (ok(ks)) return ks;
    return 1;
}
// the causal prefill's attention in place of the decode launch: layer `il`'s cache and the stack's activations
static bool prefill_layer_attn(const PrefillAttnParams &pf, const Config &c, const DevLayer &l, const float *qkv,
                               const float *rope, uint16_t *kc, uint16_t *vc, int n_ctx, uint16_t *attn, hipStream_t s) {
    PrefillAttnParams q = pf;
    q.qkv = qkv; q.qn = l.qn; q.kn = l.kn; q.eps = c.eps; q.rope = rope; q.kc = kc; q.vc = vc;
    q.n_ctx = n_ctx; q.nH = c.n_heads; q.nKV = c.n_kv; q.D = c.head_dim; q.out = attn;
    return prefill_attn(q, s);
}

// weight prefetch of the batched talker stack: 0 off (default), 1 the norms before QKV and gate/up, 2 also the gate/up
// GEMM for the down projection (its 64-token tiles leave a quarter of the CUs free).  Off since round 5: level 2 saved
// 0.3 % of the 64-slot step (1.5960 -> 1.5912 ms, two A/B pairs) for 755 MB more fabric reads per step (FETCH 3,111 ->
// 3,866 MB: every prefetched line is read twice, once into the Infinity Cache and once by the GEMM)
static const int g_mm_prefetch = [] { const char *e = std::getenv("Q3T_MM_PREFETCH"); return e ? std::atoi(e) : 0; }();
// gate/up on 64-token tiles: 192 workgroups of one per CU instead of 384 (two on half the CUs, which set the tail);
// the other projections keep 32-token tiles.  64-slot talker step 1.574 -> 1.549 ms (two A/B pairs,
// tools/dev/exp_gutt.sh); the tile never changes a row's arithmetic.  Q3T_MM_GU_TT=1 restores 32-token tiles.
static const int g_mm_gu_tt = [] { const char *e = std::getenv("Q3T_MM_GU_TT"); return e ? std::atoi(e) : 2; }();
static bool decoder_stack_mm(const Config &c, bool attn_split, const std::vector<DevLayer> &layers, int S, float *x, uint16_t *xn,
                             float *parts, float *qkv, uint16_t *attn, uint16_t *hmlp, uint16_t *kc, uint16_t *vc,
                             size_t kv_layer, int n_ctx, int max_splits, const int *pos, const float *rope, float *part,
                             unsigned *ticket, hipStream_t s, const StackInput *in0, const float *final_norm,
                             float *final_side, int S_main = 0, bool cp_attn = false, const PrefillAttnParams *pf = nullptr,
                             const AttnParams *l0tab = nullptr) {
    // S_main: the batch whose kernel choices this stack reproduces (a continuous-batching admission runs ONE slot
    // with the S_main-slot kernels, so its per-token arithmetic is the batch's)
    if (S_main <= 0) S_main = S;
    const bool force = S < gemm_mfma_min_batch();
    const int H = c.hidden, D = c.head_dim, QKV = (c.n_heads + 2 * c.n_kv) * D;
    ResidNorm rn;
    rn.S = S; rn.H = H; rn.eps = c.eps; rn.x = x; rn.xn = xn;
    if (in0 && in0->prenormed) {
        // the previous launch (token selection) gathered and normalised layer 0's input
    } else if (in0 && (in0->pro == PRO_RMS_G1 || in0->pro == PRO_RMS_G16)) {
        if (!gather_sum(in0->gs, in0->pro == PRO_RMS_G16 ? 16 : 1, S, H, x, H, s)) return false;
    } else if (in0 && in0->x) {
        rn.xin = in0->x;   // copied into the residual stream by the norm
    }
    rn.nw = layers[0].attn_norm;
    if (!(in0 && in0->prenormed) && !resid_norm(rn, s)) return false;
    rn.xin = nullptr;
    // the code predictor's <= 16 positions run on k_attn_small, which can read layer 0's raw QKV rows from the per-token
    // table (l0tab: passes 1..15) instead of a QKV GEMM over xn
    const bool small = cp_attn && n_ctx <= 16 && D == 128 && c.n_heads == 2 * c.n_kv;
#ifdef Q3T_NO_SMALL_ATTN
    const bool use_tab = false;
#else
    const bool use_tab = small && l0tab && l0tab->qkv_tab && !pf;
#endif
    for (size_t il = 0; il < layers.size(); ++il) {
        const DevLayer &l = layers[il];
        GemvParams g;
        g.W = l.qkv; g.N = QKV; g.K = H; g.B = S;
        g.pro = PRO_F16; g.x = xn; g.ldx = H;
        g.out_f32 = qkv; g.ldo = QKV; g.force_mm = force;
        if (!(il == 0 && use_tab) && !gemv(g, s)) return false;
        AttnParams a;
        a.qkv = qkv; a.qn = l.qn; a.kn = l.kn; a.eps = c.eps; a.rope = rope; a.pos = pos;
        a.kc = kc + il * kv_layer; a.vc = vc + il * kv_layer;
        a.n_ctx = n_ctx; a.S = S; a.nH = c.n_heads; a.nKV = c.n_kv; a.D = D;
        a.max_splits = max_splits;   // chunk 128 measured no faster at 64 slots (1.79 vs 1.77 ms per step)
        a.seqk = S_main >= 16 && !attn_split;   // enough (slot, kv head) pairs to fill the chip
        // the code predictor's <= 16 positions: one wave per (slot, kv head) (the 0.6B head layout)
        a.small = small;
        if (il == 0 && use_tab) {
            a.qkv_tab = l0tab->qkv_tab; a.tab_tok = l0tab->tab_tok; a.tab_ld = l0tab->tab_ld; a.tab_col = l0tab->tab_col;
            a.tab_row0 = l0tab->tab_row0;
        }
#ifdef Q3T_NO_SMALL_ATTN
        a.small = 0;   // experiment builds: the code predictor on k_attn_seq / k_attn as before
#endif
        a.part = part; a.ticket = ticket; a.out = attn;
        if (pf ? !prefill_layer_attn(*pf, c, l, qkv, rope, a.kc, a.vc, n_ctx, attn, s) : !attn_decode(a, s)) return false;
        // code-predictor pass 0 (no head): its last layer's K/V rows, appended above, are all that is ever read
        if (il + 1 == layers.size() && !final_norm) break;
        GemvParams o;
        o.W = l.o; o.N = H; o.K = c.n_heads * D; o.B = S;
        o.pro = PRO_F16; o.x = attn; o.ldx = c.n_heads * D;
        o.parts = parts; o.ksplit = splitk_for(H, S_main, o.K); o.force_mm = force;
        if (!gemv(o, s)) return false;
        rn.parts = parts; rn.ksplit = o.ksplit; rn.nw = l.ffn_norm; rn.side = nullptr;
        // the talker's weights stream from HBM each step: the norm before a projection touches that projection's lines
        // (the code predictor's 157 MB stay in the Infinity Cache across its 16 passes anyway)
        const bool pf_w = !cp_attn && g_mm_prefetch > 0;
        rn.prefetch = pf_w ? l.gu : nullptr; rn.prefetch_bytes = (size_t)2 * c.inter * H * 2;
        if (!resid_norm(rn, s)) return false;
        GemvParams gu;
        gu.W = l.gu; gu.N = 2 * c.inter; gu.K = H; gu.B = S;
        gu.pro = PRO_F16; gu.x = xn; gu.ldx = H;
        gu.act = ACT_SWIGLU; gu.out_f16 = hmlp; gu.ldo = c.inter; gu.force_mm = force; gu.mm_tt = g_mm_gu_tt;
        if (pf_w && g_mm_prefetch > 1) { gu.prefetch = l.down; gu.prefetch_bytes = (size_t)c.inter * H * 2; }
        if (!gemv(gu, s)) return false;
        GemvParams dn;
        dn.W = l.down; dn.N = H; dn.K = c.inter; dn.B = S;
        dn.pro = PRO_F16; dn.x = hmlp; dn.ldx = c.inter;
        dn.parts = parts; dn.ksplit = splitk_for(H, S_main, dn.K); dn.force_mm = force;
        dn.xcd_slices = true;   // each XCD fetches 1 / ksplit of hmlp (FETCH 1.42x -> 1.06x of the algorithmic bytes)
        if (!gemv(dn, s)) return false;
        const bool last = il + 1 == layers.size();
        if (last && !final_norm) break;   // code-predictor pass 0: only its K/V caches are read afterwards
        rn.parts = parts; rn.ksplit = dn.ksplit;
        rn.nw = last ? (final_norm ? final_norm : l.ffn_norm) : layers[il + 1].attn_norm;
        rn.side = last ? final_side : nullptr;
        rn.prefetch = pf_w && !last ? layers[il + 1].qkv : nullptr; rn.prefetch_bytes = (size_t)QKV * H * 2;
        if (!resid_norm(rn, s)) return false;
        rn.prefetch = nullptr;
    }
    return true;
}

// ------------------------------------------------------------------------------------------ one decoder stack
// 5 launches per layer: [RMSNorm+QKV GEMV] [head-norm+RoPE+KV-append+attention] [O GEMV + residual]
// [RMSNorm+gate/up GEMV+SwiGLU] [down GEMV + residual]   (tts_transformer.cpp:1410-1494)
// `in0` (optional) replaces layer 0's activation source: a gather prologue or another f32 buffer, with the raw
// rows written to x (the residual stream) by the QKV kernel itself.

static bool decoder_stack(const Config &c, const std::vector<DevLayer> &layers, int S, float *x, float *qkv,
                          uint16_t *attn, uint16_t *hmlp, uint16_t *kc, uint16_t *vc, size_t kv_layer, int n_ctx,
                          int max_splits, const int *pos, const float *rope, float *part, unsigned *ticket,
                          hipStream_t s, const StackInput *in0 = nullptr, bool fused_cp_attn = false,
                          const PrefillAttnParams *pf = nullptr, int family_b = 0) {
    // pf: the causal prefill (S = its rows, run with the vector kernels of a family_b-slot step)
    const int H = c.hidden, D = c.head_dim, QKV = (c.n_heads + 2 * c.n_kv) * D;
    // batched (matrix-core) path: gathers become their own launch and the code predictor's attention runs unfused
    const bool mm = (family_b > 0 ? family_b : S) >= gemm_mfma_min_batch();
    if (mm) fused_cp_attn = false;
    for (size_t il = 0; il < layers.size(); ++il) {
        const DevLayer &l = layers[il];
        GemvParams g;
        g.W = l.qkv; g.N = QKV; g.K = H; g.B = S;
        g.pro = PRO_RMS; g.x = x; g.ldx = H; g.nw = l.attn_norm; g.eps = c.eps;
        if (il == 0 && in0) {
            // the gather as its own launch: batched path (no gather prologue in the GEMM), or rows wider than the
            // GEMV's gather prologue (K > 1024: the 1.7B talker) -- the same summation order either way
            if ((mm || H > 1024) && (in0->pro == PRO_RMS_G1 || in0->pro == PRO_RMS_G16)) {
                if (!gather_sum(in0->gs, in0->pro == PRO_RMS_G16 ? 16 : 1, S, H, x, H, s)) return false;
            } else {
                g.pro = in0->pro; g.x = in0->x; g.gs = in0->gs; g.raw_out = x;
                g.sel = in0->sel; g.sel_logits = in0->sel_logits;
            }
        }
        g.out_f32 = qkv; g.ldo = QKV; g.family_b = family_b;
        if (!gemv(g, s)) return false;
        GemvParams o;
        o.W = l.o; o.N = H; o.K = c.n_heads * D; o.B = S; o.family_b = family_b;
        if (pf) {
            if (!prefill_layer_attn(*pf, c, l, qkv, rope, kc + il * kv_layer, vc + il * kv_layer, n_ctx, attn, s)) return false;
            o.pro = PRO_F16; o.x = attn; o.ldx = c.n_heads * D;
        } else if (fused_cp_attn) {
            // code predictor: attention recomputed inside the O-projection prologue (<= 16 positions)
            o.pro = PRO_CPATT;
            o.att.qkv = qkv; o.att.ld = QKV; o.att.qn = l.qn; o.att.kn = l.kn; o.att.eps = c.eps;
            o.att.rope = rope; o.att.pos = pos; o.att.kc = kc + il * kv_layer; o.att.vc = vc + il * kv_layer;
        } else {
            AttnParams a;
            a.qkv = qkv; a.qn = l.qn; a.kn = l.kn; a.eps = c.eps; a.rope = rope; a.pos = pos;
            a.kc = kc + il * kv_layer; a.vc = vc + il * kv_layer;
            a.n_ctx = n_ctx; a.S = S; a.nH = c.n_heads; a.nKV = c.n_kv; a.D = D;
            a.max_splits = max_splits; a.part = part; a.ticket = ticket; a.out = attn;
#ifdef Q3T_DEV
            if (il == 0 && std::getenv("Q3T_PERSIST_DBG")) a.dbg = part;
#endif
            if (!attn_decode(a, s)) return false;
            o.pro = PRO_F16; o.x = attn; o.ldx = c.n_heads * D;
        }
        o.resid = x; o.ldr = H; o.out_f32 = x; o.ldo = H;
        if (!gemv(o, s)) return false;
        GemvParams gu;
        gu.W = l.gu; gu.N = 2 * c.inter; gu.K = H; gu.B = S;
        gu.pro = PRO_RMS; gu.x = x; gu.ldx = H; gu.nw = l.ffn_norm; gu.eps = c.eps;
        gu.act = ACT_SWIGLU; gu.out_f16 = hmlp; gu.ldo = c.inter; gu.family_b = family_b;
        if (!gemv(gu, s)) return false;
        GemvParams dn;
        dn.W = l.down; dn.N = H; dn.K = c.inter; dn.B = S; dn.family_b = family_b;
        dn.pro = PRO_F16; dn.x = hmlp; dn.ldx = c.inter;
        dn.resid = x; dn.ldr = H; dn.out_f32 = x; dn.ldo = H;
        if (!gemv(dn, s)) return false;
    }
    return true;
}

bool Engine::enqueue_talker_step(int S, hipStream_t s) { return enqueue_talker(S, s, false, false); }

SelectSpec Engine::select_spec(int mode, const GenParams &gp, int frame_offset, int step) const {
    SelectSpec sp;
    sp.mode = mode;
    sp.V = mode == SEL_CB0 ? c_.codec_vocab : c_.cp_vocab;
    sp.ticket = sel_ticket_;
    sp.tokens = tokens_; sp.codes = codes_; sp.max_len = codes_max_len_; sp.ncb = 16;
    sp.frame = frame_; sp.frame_offset = frame_offset; sp.done = done_;
    sp.temperature = gp.temperature; sp.top_k = gp.top_k; sp.seed = gp.seed; sp.seed_dev = seed_dev_; sp.utt = utt_;
    sp.step = step;
    sp.seen = seen_; sp.n_tokens = n_tokens_; sp.force_frames = force_; sp.eos = c_.codec_eos; sp.rep = gp.rep_penalty;
    return sp;
}

// gather_input: the step embedding (tts_transformer.cpp:2529-2553) is assembled by layer 0's QKV prologue from the
// frame's 16 codes (PRO_RMS_G16) instead of being read from x_
// select_next: the codec head's last workgroup also selects CB0 of the NEXT frame (frame_ + 1) in the same launch
bool Engine::enqueue_talker(int S, hipStream_t s, bool gather_input, bool select_next, bool prenormed, bool *fold_advance) {
    const int H = c_.hidden;
    const size_t kv_layer = (size_t)max_slots_ * c_.n_kv * max_ctx_ * c_.head_dim;
    const int max_splits = (max_ctx_ + ATTN_CHUNK - 1) / ATTN_CHUNK;
    if (S == 1 && persist_) {
        PersistParams p;
        persist_carve(pstate_, p);
        p.L = pl_dev_; p.n_layers = c_.n_layers; p.eps = c_.eps;
        p.gather = gather_input ? 1 : 0;
        p.x_in = x_;
        p.gs.tok = tokens_; p.gs.tok_ld = 16; p.gs.tabs = tabs16_dev_;
        p.gs.tr = trailing_; p.gs.tr_len = trailing_len_; p.gs.frame = frame_;
        p.gs.tr_ld = max_trailing_ * H; p.gs.pad = tts_pad_;
        p.rope = rope_; p.pos = pos_; p.kc = kc_; p.vc = vc_; p.kv_layer = kv_layer; p.n_ctx = max_ctx_;
        p.head = codec_head_; p.out_norm = out_norm_; p.hidden = hidden_; p.logits = logits_;
        if (select_next) p.sel = select_spec(SEL_CB0, gp_, 1, 0);
        p.prof = pprof_;
        if (tk_roles_) {
            if (fold_advance && opt_.fold_advance) {
                p.adv_pos = pos_; p.adv_frame = frame_; p.adv_done = done_;
                *fold_advance = true;
            }
            return persist_tk_roles(p, s);
        }
        return persist_talker_step(p, s);
    }
    StackInput in0;
    if (gather_input) {
        in0.pro = PRO_RMS_G16;
        in0.gs.tok = tokens_; in0.gs.tok_ld = 16; in0.gs.tabs = tabs16_dev_;
        in0.gs.tr = trailing_; in0.gs.tr_len = trailing_len_; in0.gs.frame = frame_;
        in0.gs.tr_ld = max_trailing_ * H; in0.gs.pad = tts_pad_;
        in0.prenormed = prenormed;
    }
    const bool mm = use_mm(S);   // batched: one selection workgroup per slot after the head
    if (use_tkb(S)) {   // batched: the whole step as one persistent launch (persist_tkb.hip)
        if (gather_input && !prenormed && !gather_sum(in0.gs, 16, S, H, x_, H, s)) return false;
        TkbParams p;
        p.L = pl_dev_; p.n_layers = c_.n_layers; p.head = codec_head_; p.out_norm = out_norm_;
        p.x_in = x_; p.hidden = hidden_; p.logits = logits_;
        p.rope = rope_; p.pos = pos_; p.kc = kc_; p.vc = vc_; p.kv_layer = kv_layer; p.n_ctx = max_ctx_;
        if (select_next) { p.select = 1; p.sel = select_spec(SEL_CB0, gp_, 1, 0); }
        p.S = S; p.eps = c_.eps;
        p.state = tkb_state_;
        p.prof = pprof_;
        return persist_talker_batched(p, s);
    }
    if (mm) {
        if (!decoder_stack_mm(c_, opt_.attn_split, L_, S, x_, xn_, parts_, qkv_, attn_, hmlp_, kc_, vc_, kv_layer, max_ctx_, max_splits, pos_,
                              rope_, part_, ticket_, s, gather_input ? &in0 : nullptr, out_norm_, hidden_, policy_slots_))
            return false;
    } else if (!decoder_stack(c_, L_, S, x_, qkv_, attn_, hmlp_, kc_, vc_, kv_layer, max_ctx_, max_splits, pos_, rope_, part_,
                              ticket_, s, gather_input ? &in0 : nullptr, false, nullptr, fam1_)) {
        return false;
    }
    // final RMSNorm (hidden_states, side output) + codec_head -> logits  (:1496-1505); batched: the stack's last
    // resid_norm already normalised x into xn (and wrote hidden_)
    GemvParams h;
    h.W = codec_head_; h.N = c_.codec_vocab; h.K = H; h.B = S;
    h.pro = PRO_RMS; h.x = x_; h.ldx = H; h.nw = out_norm_; h.eps = c_.eps; h.side_out = hidden_; h.family_b = fam1_;
    if (mm) { h.pro = PRO_F16; h.x = xn_; h.nw = nullptr; h.side_out = nullptr; }
    h.out_f32 = logits_; h.ldo = c_.codec_vocab;
    if (select_next && !mm) h.sel = select_spec(SEL_CB0, gp_, 1, 0);
    if (!gemv(h, s)) return false;
    if (select_next && mm) return select_tokens(select_spec(SEL_CB0, gp_, 1, 0), logits_, S, s);
    return true;
}

// 16 passes of the 5-layer code predictor, token chosen on device each pass (trt_code_predictor.cpp:484-600).
// Pass inputs are assembled by layer 0's QKV prologue: pass 0 the talker hidden state, pass 1 codec_embd[code 0],
// pass p >= 2 code_pred.codec_embd[p-2][code p-1]; the raw row lands in cpx_ (the pass's residual stream).
// logits_host (tests only, never captured): every head's logits copied out after its GEMV.
bool Engine::cp_project(int S, const float *x_talker, int ldx, hipStream_t s) {
    GemvParams g;   // ggml_mul_mat(mtp_proj, cur) + ggml_add(bias): f16-rounded input, f32 accumulation
    g.W = mtp_; g.N = c_.cp_hidden; g.K = c_.hidden; g.B = S;
    g.pro = PRO_F32; g.x = x_talker; g.ldx = ldx;
    g.bias = mtp_b_;
    g.out_f32 = cpx_; g.ldo = c_.cp_hidden; g.family_b = fam1_;
    return gemv(g, s);
}

bool Engine::enqueue_cp_frame(int S, hipStream_t s, float *logits_host, bool talker_next) {
    const int H = cpc_.hidden;   // code-predictor width (the talker's for 0.6B)
    const size_t kv_layer = (size_t)max_slots_ * cpc_.n_kv * 16 * cpc_.head_dim;
    std::vector<float> lg;
    // vector path with fused selection: heads 0..13 only produce logits; the next pass's QKV launch selects the token
    // in every workgroup while its weights stream (PRO_SEL_G1), so the head's 256 -> 1 arrival chain and the serial
    // selection leave the critical path.  Head 14 (its token feeds the next talker step) keeps the fused selection.
    if (S == 1 && persist_cp_ && !logits_host) {   // the whole frame as one persistent launch
        PersistParams p;
        persist_carve(pstate_, p);
        p.L = pl_cp_dev_; p.n_layers = c_.cp_layers; p.eps = c_.eps;
        p.x_in = hidden_;
        if (c_.has_mtp) {   // 1.7B: pass 0's projected input by the per-op GEMV, passes 1..15 from the projected table
            if (!cp_project(1, hidden_, c_.hidden, s)) return false;
            p.x_in = cpx_;
            p.xtab = cp_projtab_;
        }
        p.gs.tok = tokens_; p.gs.tok_ld = 16; p.gs.tabs = tabs16_dev_;
        p.rope = rope_; p.kc = cpkc_; p.vc = cpvc_; p.kv_layer = kv_layer; p.n_ctx = 16;
        p.heads = heads_dev_; p.out_norm = cp_out_norm_; p.logits = cp_logits_;
        p.qkvtab = cp_qkvtab_;
        p.sel = select_spec(SEL_CP, gp_, 0, 0);
        p.prof = pprof_;
        if (cp_roles_ && p.qkvtab) return persist_cp_roles(p, s);   // (1.7B: layer 0's residual rows from xtab)
        return persist_cp_frame(p, s);
    }
    if (use_cpb(S) && !logits_host) {   // batched: the whole frame as one persistent launch (persist_cpb.hip)
        CpbParams p;
        p.L = pl_cp_dev_; p.heads = heads_dev_; p.tabs = tabs16_dev_; p.out_norm = cp_out_norm_; p.qkvtab = cp_qkvtab_;
        p.x_in = hidden_; p.rope = rope_; p.pos = cp_pos_; p.pos_ld = max_slots_; p.kc = cpkc_; p.vc = cpvc_;
        p.kv_layer = kv_layer; p.logits = cp_logits_; p.sel = select_spec(SEL_CP, gp_, 0, 0); p.S = S; p.eps = c_.eps;
        if (talker_next) {
            p.talker_next = 1;
            p.tx = x_; p.txn = xn_; p.tnw = L_[0].attn_norm;
            p.tr = trailing_; p.tr_len = trailing_len_; p.frame = frame_; p.tr_ld = max_trailing_ * H; p.pad = tts_pad_;
        }
        p.state = cpb_state_;
        p.prof = pprof_;
        return persist_cp_batched(p, s);
    }
    const bool fsel_all = fused_select_ && !use_mm(S);
    // deferred selection gathers the next pass's table row inside its QKV launch: not with a projected input (1.7B)
    const bool defer = fsel_all && defer_cp_select_ && !c_.has_mtp;
    bool next_prenormed = false;   // batched: this pass's input was prepared by the previous selection launch
    for (int p = 0; p < 16; ++p) {
        StackInput in0;
        in0.prenormed = next_prenormed;
        next_prenormed = false;
        if (c_.has_mtp) {
            // 1.7B: the pass input (talker hidden / table row, talker space) projected into cpx_ by code_pred.mtp_proj
            // (tts_transformer.cpp:1554-1560, :1709-1714); layer 0 then normalises cpx_ like any later layer
            const float *src = hidden_;
            if (p > 0) {
                GatherSum gs;
                gs.tok = tokens_; gs.tok_ld = 16; gs.tok_col0 = p - 1;
                gs.tab0 = p == 1 ? codec_embd_ : cp_embd_[p - 2];
                if (!gather_sum(gs, 1, S, c_.hidden, cp_in1_, c_.hidden, s)) return false;
                src = cp_in1_;
            }
            if (!cp_project(S, src, c_.hidden, s)) return false;
            in0.pro = PRO_RMS; in0.x = cpx_;
        } else if (p == 0) {
            in0.pro = PRO_RMS; in0.x = hidden_;
        } else {
            in0.pro = PRO_RMS_G1;
            in0.gs.tok = tokens_; in0.gs.tok_ld = 16; in0.gs.tok_col0 = p - 1;
            in0.gs.tab0 = p == 1 ? codec_embd_ : cp_embd_[p - 2];
            if (defer && p >= 2) {
                in0.pro = PRO_SEL_G1;
                in0.sel = select_spec(SEL_CP, gp_, 0, p - 2);
                in0.sel_logits = cp_logits_;
            }
        }
        const bool mm = use_mm(S);
        if (mm) {
            // passes 1..15: layer 0's raw QKV rows from the per-token table (the 0.6B layout; the table's rows are the
            // 1-slot GEMV's, within the batched family's f32 tolerance of its MFMA GEMM)
            AttnParams l0;
            if (p >= 1 && cp_qkvtab_ && !c_.has_mtp) {
                l0.qkv_tab = cp_qkvtab_; l0.tab_tok = tokens_; l0.tab_ld = 16; l0.tab_col = p - 1;
                l0.tab_row0 = p == 1 ? 0 : (size_t)c_.codec_vocab + (size_t)(p - 2) * c_.cp_vocab;
            }
            if (!decoder_stack_mm(cpc_, opt_.attn_split, CP_, S, cpx_, xn_, parts_, qkv_, attn_, hmlp_, cpkc_, cpvc_, kv_layer, 16, 1,
                                  cp_pos_ + (size_t)p * max_slots_, rope_, part_, ticket_, s, &in0,
                                  p == 0 ? nullptr : cp_out_norm_, nullptr, policy_slots_, true, nullptr,
                                  opt_.mm_cp_table ? &l0 : nullptr))
                return false;
        } else if (!decoder_stack(cpc_, CP_, S, cpx_, qkv_, attn_, hmlp_, cpkc_, cpvc_, kv_layer, 16, 1,
                                  cp_pos_ + (size_t)p * max_slots_, rope_, part_, ticket_, s, c_.has_mtp ? nullptr : &in0,
                                  cp_fused_attn_, nullptr, fam1_)) {
            return false;
        }
        if (p == 0) continue;
        const int step = p - 1;
        GemvParams h;
        h.W = cp_head_[step]; h.N = c_.cp_vocab; h.K = H; h.B = S;
        h.pro = PRO_RMS; h.x = cpx_; h.ldx = H; h.nw = cp_out_norm_; h.eps = c_.eps; h.family_b = fam1_;
        if (mm) { h.pro = PRO_F16; h.x = xn_; h.nw = nullptr; }
        h.out_f32 = cp_logits_; h.ldo = c_.cp_vocab;
        const bool fsel = fsel_all && (!defer || step == 14);
        if (fsel) h.sel = select_spec(SEL_CP, gp_, 0, step);
        if (!gemv(h, s)) return false;
        if (logits_host) {
            lg.resize((size_t)S * c_.cp_vocab);
            Q3T_HIP(hipMemcpyAsync(lg.data(), cp_logits_, lg.size() * 4, hipMemcpyDeviceToHost, s));
            Q3T_HIP(hipStreamSynchronize(s));
            for (int b = 0; b < S; ++b)
                std::memcpy(logits_host + ((size_t)b * 15 + step) * c_.cp_vocab, lg.data() + (size_t)b * c_.cp_vocab, c_.cp_vocab * 4);
        }
#ifdef Q3T_NO_SELFUSE
        if (false) {
#else
        if (mm && (step < 14 || talker_next)) {
#endif
            // batched: the selecting workgroup of each slot also gathers and normalises the next stage's input (the
            // next pass's table row, or the talker step embedding after the last pass)
            EmbedNorm en;
            en.gs.tok = tokens_; en.gs.tok_ld = 16;
            if (step < 14) {
                en.nt = 1; en.gs.tok_col0 = step + 1; en.gs.tab0 = cp_embd_[step];
                en.x = cpx_; en.nw = CP_[0].attn_norm;
            } else {
                en.nt = 16; en.gs.tabs = tabs16_dev_; en.gs.tr = trailing_; en.gs.tr_len = trailing_len_;
                en.gs.frame = frame_; en.gs.tr_ld = max_trailing_ * H; en.gs.pad = tts_pad_;
                en.x = x_; en.nw = L_[0].attn_norm;
            }
            en.xn = xn_; en.eps = c_.eps; en.H = c_.hidden;   // (mm: no projection, code predictor width == talker's)
            if (!select_embed_norm(select_spec(SEL_CP, gp_, 0, step), cp_logits_, en, S, s)) return false;
            next_prenormed = true;
            continue;
        }
        if (!fsel && !(defer && step < 14) && !select_tokens(select_spec(SEL_CP, gp_, 0, step), cp_logits_, S, s)) return false;
    }
    return true;
}

// one frame = [CB0 select] -> 16 code-predictor passes -> talker step -> pos/frame advance.  With fused selection
// the CB0 of frame f+1 is chosen inside frame f's talker head launch (frame 0's by generate() after the prefill).
bool Engine::enqueue_frame(int S, hipStream_t s) {
    if (!fused_select_ && !select_tokens(select_spec(SEL_CB0, gp_, 0, 0), logits_, S, s)) return false;
    // batched: the last code-predictor selection also assembles and normalises the talker step's input
#ifdef Q3T_NO_SELFUSE
    const bool mm = false;
#else
    const bool mm = use_mm(S);
#endif
    if (!enqueue_cp_frame(S, s, nullptr, mm)) return false;
    bool folded = false;   // the single-slot role kernel advances pos / frame itself
    if (!enqueue_talker(S, s, true, fused_select_, mm, &folded)) return false;
    return folded || advance(pos_, frame_, done_, S, s);
}

bool Engine::graph_for(std::map<int, hipGraphExec_t> &cache, int S, bool (Engine::*fn)(int, hipStream_t)) {
    return graph_for_key(cache, S, S, fn);
}

bool Engine::graph_for_key(std::map<int, hipGraphExec_t> &cache, int key, int S, bool (Engine::*fn)(int, hipStream_t)) {
    if (cache.count(key)) return true;
    hipGraph_t graph = nullptr;
    Q3T_HIP(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
    const bool ok = (this->*fn)(S, stream_);
    hipError_t e = hipStreamEndCapture(stream_, &graph);
    if (!ok) { if (graph) hipGraphDestroy(graph); return false; }
    if (e != hipSuccess) { set_error(std::string("graph capture: ") + hipGetErrorString(e)); return false; }
    hipGraphExec_t exec = nullptr;
    e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    hipGraphDestroy(graph);
    if (e != hipSuccess) { set_error(std::string("graph instantiate: ") + hipGetErrorString(e)); return false; }
    cache[key] = exec;
    return true;
}

bool Engine::set_slot_state(int S, const std::vector<int> &pos, const std::vector<int> &frame) {
    Q3T_HIP(hipMemcpyAsync(pos_, pos.data(), S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(frame_, frame.data(), S * 4, hipMemcpyHostToDevice, stream_));
    return true;
}

// ------------------------------------------------------------------------------------------ causal prefill
// build_prefill_forward_graph (src/tts_transformer.cpp:1233-1374): the plen prompt rows of n_utt utterances in ONE
// pass of the talker stack -- every projection over all n_utt * plen rows (one weight stream for the whole prompt
// instead of plen), causal attention per utterance (prefill_attn) writing the K/V rows [0, plen) of slot pf_slot_[u]
// directly.  The projections run the kernels of an S_main-slot decode step with its K split (family_b / S_main),
// and the attention reproduces the decode kernel's reduction tree over its first positions, so every row equals the
// S_main-slot step replayed at its position bit for bit (tests/cpp/test_host_api.cpp, tests/test_gpu_prefill.py).
// Outputs: pf_hid_ / pf_logits_ rows u * plen + plen - 1 (final-norm hidden state and codec logits of the last row).
bool Engine::ensure_prefill() {
    if (pf_x_) return true;
    const size_t R = (size_t)max_slots_ * 10, H = c_.hidden, D = c_.head_dim;
    const size_t QKV = (size_t)(c_.n_heads + 2 * c_.n_kv) * D;
    pf_x_ = dalloc<float>(R * H);
    pf_xn_ = dalloc<uint16_t>(R * H);
    pf_parts_ = dalloc<float>(4 * R * H);
    pf_qkv_ = dalloc<float>(R * QKV);
    pf_attn_ = dalloc<uint16_t>(R * c_.n_heads * D);
    pf_hmlp_ = dalloc<uint16_t>(R * c_.inter);
    pf_hid_ = dalloc<float>(R * H);
    pf_logits_ = dalloc<float>(R * c_.codec_vocab);
    pf_slot_ = dalloc<int>(max_slots_);
    if (!pf_x_ || !pf_xn_ || !pf_parts_ || !pf_qkv_ || !pf_attn_ || !pf_hmlp_ || !pf_hid_ || !pf_logits_ || !pf_slot_) {
        set_error("device allocation failed");
        return false;
    }
    return true;
}

// the captured body: key = (S_main * 1024 + n_utt) * 16 + plen
bool Engine::enqueue_prefill_rows(int key, hipStream_t s) {
    const int plen = key % 16, n_utt = key / 16 % 1024, S_main = key / (16 * 1024);
    const int rows = n_utt * plen, H = c_.hidden, V = c_.codec_vocab;
    const size_t kv_layer = (size_t)max_slots_ * c_.n_kv * max_ctx_ * c_.head_dim;
    const int max_splits = (max_ctx_ + ATTN_CHUNK - 1) / ATTN_CHUNK;
    PrefillAttnParams pf;
    pf.slot = pf_slot_; pf.n_utt = n_utt; pf.plen = plen;
    GemvParams h;   // final RMSNorm (hidden side output) + codec head over every row, as the S_main-slot step
    h.W = codec_head_; h.N = V; h.K = H; h.B = rows; h.out_f32 = pf_logits_; h.ldo = V;
    if (use_mm(S_main)) {
        if (!decoder_stack_mm(c_, opt_.attn_split, L_, rows, pf_x_, pf_xn_, pf_parts_, pf_qkv_, pf_attn_, pf_hmlp_, kc_, vc_,
                              kv_layer, max_ctx_, max_splits, pos_, rope_, part_, ticket_, s, nullptr, out_norm_, pf_hid_,
                              S_main, false, &pf))
            return false;
        h.pro = PRO_F16; h.x = pf_xn_; h.ldx = H; h.force_mm = true;
        return gemv(h, s);
    }
    if (!decoder_stack(c_, L_, rows, pf_x_, pf_qkv_, pf_attn_, pf_hmlp_, kc_, vc_, kv_layer, max_ctx_, max_splits, pos_, rope_,
                       part_, ticket_, s, nullptr, false, &pf, S_main))
        return false;
    h.pro = PRO_RMS; h.x = pf_x_; h.ldx = H; h.nw = out_norm_; h.eps = c_.eps; h.side_out = pf_hid_; h.family_b = S_main;
    return gemv(h, s);
}

// src: [n_utt][10][H] prompt rows (rows [0, plen) of each used); pf_slot_[0, n_utt) must hold the target slots
bool Engine::prefill(int n_utt, int plen, const float *src, int S_main, hipStream_t s) {
    const int H = c_.hidden;
    if (n_utt <= 0 || n_utt > max_slots_ || plen < 1 || plen > 10 || S_main < 1 || S_main > 4096) {
        set_error("prefill: bad shape");
        return false;
    }
    if (!ensure_prefill()) return false;
    if (!mm_ok_) S_main = 1;   // every step of this model runs the 1-slot vector kernels (fam1_)
    Q3T_HIP(hipMemcpy2DAsync(pf_x_, (size_t)plen * H * 4, src, (size_t)10 * H * 4, (size_t)plen * H * 4, n_utt,
                             hipMemcpyDeviceToDevice, s));
    const int key = (S_main * 1024 + n_utt) * 16 + plen;
    if (!g_prefill_.count(key)) {
        hipGraph_t graph = nullptr;
        Q3T_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        const bool ok = enqueue_prefill_rows(key, s);
        hipError_t e = hipStreamEndCapture(s, &graph);
        if (!ok) { if (graph) hipGraphDestroy(graph); return false; }
        if (e != hipSuccess) { set_error(std::string("graph capture: ") + hipGetErrorString(e)); return false; }
        hipGraphExec_t exec = nullptr;
        e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
        hipGraphDestroy(graph);
        if (e != hipSuccess) { set_error(std::string("graph instantiate: ") + hipGetErrorString(e)); return false; }
        g_prefill_[key] = exec;
    }
    Q3T_HIP(hipGraphLaunch(g_prefill_[key], s));
    return true;
}

// ------------------------------------------------------------------------------------------ prefill pieces
bool Engine::enqueue_text_projection(int n_rows, hipStream_t s) {
    return enqueue_text_projection(n_rows, s, proj_idx_, proj_h_, proj_out_);
}

bool Engine::enqueue_text_projection(int n_rows, hipStream_t s, const int *idx, uint16_t *hbuf, float *out) {
    // text_embd row gather -> fc1 + b -> SiLU -> fc2 + b   (tts_transformer.cpp:1050-1055)
    GemvParams a;
    a.W = fc1_; a.N = c_.text_dim; a.K = c_.text_dim; a.B = n_rows;
    a.pro = PRO_F16; a.x = text_embd_; a.ldx = c_.text_dim; a.x_idx = idx;
    a.bias = fc1_b_; a.act = ACT_SILU; a.out_f16 = hbuf; a.ldo = c_.text_dim;
    if (!gemv(a, s)) return false;
    GemvParams b;
    b.W = fc2_; b.N = c_.hidden; b.K = c_.text_dim; b.B = n_rows;
    b.pro = PRO_F16; b.x = hbuf; b.ldx = c_.text_dim;
    b.bias = fc2_b_; b.out_f32 = out; b.ldo = c_.hidden;
    return gemv(b, s);
}

bool Engine::project_text(int n, const int32_t *toks, float *out) {
    if (n <= 0) return true;
    if (n > proj_cap_) { set_error("too many text rows"); return false; }
    DeviceLock lk(false, device_);
    for (int i = 0; i < n; ++i)
        if (toks[i] < 0 || toks[i] >= c_.text_vocab) { set_error("text token out of range"); return false; }
    Q3T_HIP(hipMemcpyAsync(proj_idx_, toks, n * 4, hipMemcpyHostToDevice, stream_));
    if (!enqueue_text_projection(n, stream_)) return false;
    Q3T_HIP(hipMemcpyAsync(out, proj_out_, (size_t)n * c_.hidden * 4, hipMemcpyDeviceToHost, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    return true;
}

namespace {
struct SlotPlan { int rb, n, plen, tcount; };
}

// Prefill assembly for slots 0..n_utt-1 on device (build_prefill_graph, tts_transformer.cpp:1093-1231).
// Projection rows of slot s start at rb: [tts_bos, tts_eos, tts_pad, tok0, tok1, tok2, tok3, tok4 .. tok(n-6)]
static bool plan_rows(const Config &c, int n_utt, const int32_t *const *tokens, const int *n_tokens, int max_trailing,
                      std::vector<int> &idx, std::vector<SlotPlan> &plan) {
    idx.clear();
    plan.clear();
    for (int s = 0; s < n_utt; ++s) {
        const int n = n_tokens[s];
        if (n < 4) { set_error("Need at least 4 text tokens for generation"); return false; }
        const int tcount = std::max(0, n - 9);
        if (tcount + 1 > max_trailing) { set_error("prompt too long for the trailing-text buffer"); return false; }
        SlotPlan p{(int)idx.size(), n, 0, tcount};
        idx.push_back(c.tts_bos); idx.push_back(c.tts_eos); idx.push_back(c.tts_pad);
        for (int i = 0; i < 4; ++i) idx.push_back(tokens[s][i]);
        for (int i = 0; i < tcount; ++i) idx.push_back(tokens[s][4 + i]);
        plan.push_back(p);
    }
    for (int v : idx)
        if (v < 0 || v >= c.text_vocab) { set_error("text token out of range"); return false; }
    return true;
}

bool Engine::prefill_embd(const int32_t *toks, int n, const float *spk, int language_id, float *prefill, int *prefill_len,
                          float *trailing, int *trailing_len, float *tts_pad) {
    // host entry for the parity tests: run the same device assembly as generate() on slot 0
    DeviceLock lk(false, device_);
    const int32_t *tk[1] = {toks};
    std::vector<int> idx;
    std::vector<SlotPlan> plan;
    if (!plan_rows(c_, 1, tk, &n, max_trailing_, idx, plan)) return false;
    GenParams gp = gp_;
    gp.language_id = language_id;
    (void)gp;
    const int H = c_.hidden;
    Q3T_HIP(hipMemcpyAsync(proj_idx_, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, stream_));
    if (!enqueue_text_projection((int)idx.size(), stream_)) return false;
    float *spk_dev = nullptr;
    if (spk) {
        spk_dev = cp_in1_;   // scratch
        Q3T_HIP(hipMemcpyAsync(spk_dev, spk, H * 4, hipMemcpyHostToDevice, stream_));
    }
    // recipe (same as generate)
    std::vector<RowRecipe> rec;
    const SlotPlan &p = plan[0];
    const float *P = proj_out_ + (size_t)p.rb * H;
    auto prow = [&](int i) { return RowTerm{P + (size_t)i * H, 0}; };
    auto crow = [&](int id) { return RowTerm{codec_embd_ + (size_t)id * H, 1}; };
    std::vector<RowTerm> cin;
    if (language_id < 0) { cin = {crow(c_.nothink), crow(c_.think_bos), crow(c_.think_eos)}; }
    else { cin = {crow(c_.think), crow(c_.think_bos), crow(language_id), crow(c_.think_eos)}; }
    if (language_id >= c_.codec_vocab) { set_error("language id out of range"); return false; }
    if (spk) cin.push_back(RowTerm{spk_dev, 0});
    cin.push_back(crow(c_.codec_pad));
    cin.push_back(crow(c_.codec_bos));
    const int ol = (int)cin.size() - 1, plen = 3 + ol + 1;
    float *out = prefill_;
    for (int r = 0; r < 3; ++r) rec.push_back(RowRecipe{out + (size_t)r * H, {prow(3 + r), {nullptr, 0}, {nullptr, 0}}});
    for (int t = 0; t < ol; ++t) rec.push_back(RowRecipe{out + (size_t)(3 + t) * H, {t == ol - 1 ? prow(0) : prow(2), cin[t], {nullptr, 0}}});
    rec.push_back(RowRecipe{out + (size_t)(plen - 1) * H, {prow(6), cin.back(), {nullptr, 0}}});
    for (int i = 0; i < p.tcount; ++i) rec.push_back(RowRecipe{trailing_ + (size_t)i * H, {prow(7 + i), {nullptr, 0}, {nullptr, 0}}});
    rec.push_back(RowRecipe{trailing_ + (size_t)p.tcount * H, {prow(1), {nullptr, 0}, {nullptr, 0}}});
    rec.push_back(RowRecipe{tts_pad_, {prow(2), {nullptr, 0}, {nullptr, 0}}});
    Q3T_HIP(hipMemcpyAsync(recipe_, rec.data(), rec.size() * sizeof(RowRecipe), hipMemcpyHostToDevice, stream_));
    if (!rows_recipe(recipe_, (int)rec.size(), H, stream_)) return false;
    Q3T_HIP(hipMemcpyAsync(prefill, prefill_, (size_t)plen * H * 4, hipMemcpyDeviceToHost, stream_));
    Q3T_HIP(hipMemcpyAsync(trailing, trailing_, (size_t)(p.tcount + 1) * H * 4, hipMemcpyDeviceToHost, stream_));
    Q3T_HIP(hipMemcpyAsync(tts_pad, tts_pad_, (size_t)H * 4, hipMemcpyDeviceToHost, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    *prefill_len = plen;
    *trailing_len = p.tcount + 1;
    return true;
}

// ------------------------------------------------------------------------------------------ hot path
bool Engine::set_seed(uint64_t seed, hipStream_t s) {
    seed_host_ = seed;   // a member: the (pageable) source outlives the copy
    Q3T_HIP(hipMemcpyAsync(seed_dev_, &seed_host_, 8, hipMemcpyHostToDevice, s));
    return true;
}

bool Engine::copy_weights_from(Engine &src) {
    DeviceLock lk(false, device_);
    std::vector<WeightArena *> a = weight_arenas(), b = src.weight_arenas();
    if (a.size() != b.size()) { set_error("copy_weights_from: contexts differ in vocoder presence"); return false; }
    for (size_t i = 0; i < a.size(); ++i) {
        if (a[i]->used != b[i]->used) { set_error("copy_weights_from: weight blobs differ in size"); return false; }
        if (a[i]->used) Q3T_HIP(hipMemcpyPeerAsync(a[i]->base, device_, b[i]->base, src.device_, a[i]->used, stream_));
    }
    Q3T_HIP(hipStreamSynchronize(stream_));
    return build_persist_tables();   // the tables derived from the weights, now that they are in place
}

bool Engine::generate(int n_utt, const int32_t *const *tokens, const int *n_tokens, const float *const *speaker,
                      const GenParams &gp, int32_t *codes, int *n_frames, FrameCb on_frames, void *user, int interval) {
    if (n_utt <= 0) return true;
    if (n_utt > max_slots_) { set_error("n_utt exceeds max_slots"); return false; }
    // only single-slot runs launch the persistent kernels: batched contexts on one device run concurrently
    DeviceLock lk(persist_exclusive(n_utt), device_);
    StreamState st;
    st.delivered.assign(n_utt, 0);
    st.stop_at.assign(n_utt, -1);
    bool fault = false;
    if (generate_once(n_utt, tokens, n_tokens, speaker, gp, codes, n_frames, on_frames, user, interval, st, &fault))
        return true;
    if (!fault) return false;
    // a persistent launch gave up on a hand-off: nothing it produced was delivered (every chunk is checked before it
    // is handed out); re-run on the launch-per-op graphs, which are bit-identical, skipping the delivered chunks
    if (!persist_recover()) return false;
    return generate_once(n_utt, tokens, n_tokens, speaker, gp, codes, n_frames, on_frames, user, interval, st, &fault);
}

bool Engine::generate_once(int n_utt, const int32_t *const *tokens, const int *n_tokens, const float *const *speaker,
                           const GenParams &gp, int32_t *codes, int *n_frames, FrameCb on_frames, void *user,
                           int interval, StreamState &st, bool *fault) {
    *fault = false;
    const int S = n_utt, H = c_.hidden, NCB = 16;
    for (int s = 0; s < S; ++s) n_frames[s] = 0;
    if (gp.max_len <= 0) return true;
    if (gp.language_id >= c_.codec_vocab) { set_error("language id out of range"); return false; }
    std::vector<int> idx;
    std::vector<SlotPlan> plan;
    if (!plan_rows(c_, S, tokens, n_tokens, max_trailing_, idx, plan)) return false;
    const bool has_spk = speaker && speaker[0];
    for (int s = 0; s < S; ++s)
        if ((speaker && speaker[s]) != has_spk) { set_error("speaker embedding must be given for all or none of the utterances"); return false; }
    const int n_pre = gp.language_id < 0 ? 3 : 4;
    const int plen = 3 + (n_pre + (has_spk ? 1 : 0) + 2 - 1) + 1;
    if (plen + gp.max_len + 8 > max_ctx_) { set_error("max_len exceeds the context reserved at ctx creation"); return false; }
    if (!(gp.temperature == gp_.temperature && gp.top_k == gp_.top_k && gp.rep_penalty == gp_.rep_penalty)) {
        for (auto &kv : g_frame_) hipGraphExecDestroy(kv.second);
        g_frame_.clear();
    }
    gp_ = gp;
    if (!set_seed(gp.seed, stream_)) return false;
    if (!ensure_prefill()) return false;
    hipEvent_t e0, e1, e2;
    hipEventCreate(&e0); hipEventCreate(&e1); hipEventCreate(&e2);
    Q3T_HIP(hipEventRecord(e0, stream_));
    // ---- text projection for every slot, one batched pass
    Q3T_HIP(hipMemcpyAsync(proj_idx_, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, stream_));
    if (!enqueue_text_projection((int)idx.size(), stream_)) return false;
    // ---- prefill / trailing / pad rows
    float *spk_dev = cp_in1_;   // scratch [S][H]
    if (has_spk)
        for (int s = 0; s < S; ++s) Q3T_HIP(hipMemcpyAsync(spk_dev + (size_t)s * H, speaker[s], H * 4, hipMemcpyHostToDevice, stream_));
    std::vector<RowRecipe> rec;
    std::vector<int> tl(S), ntok(S), force(S, gp.force_frames), pos0(S, 0), frame0(S, 0), done0(S, -1);
    for (int s = 0; s < S; ++s) {
        const SlotPlan &p = plan[s];
        const float *P = proj_out_ + (size_t)p.rb * H;
        auto prow = [&](int i) { return RowTerm{P + (size_t)i * H, 0}; };
        auto crow = [&](int id) { return RowTerm{codec_embd_ + (size_t)id * H, 1}; };
        std::vector<RowTerm> cin;
        if (gp.language_id < 0) cin = {crow(c_.nothink), crow(c_.think_bos), crow(c_.think_eos)};
        else cin = {crow(c_.think), crow(c_.think_bos), crow(gp.language_id), crow(c_.think_eos)};
        if (has_spk) cin.push_back(RowTerm{spk_dev + (size_t)s * H, 0});
        cin.push_back(crow(c_.codec_pad));
        cin.push_back(crow(c_.codec_bos));
        const int ol = (int)cin.size() - 1;
        float *out = prefill_ + (size_t)s * 10 * H;
        for (int r = 0; r < 3; ++r) rec.push_back(RowRecipe{out + (size_t)r * H, {prow(3 + r), {nullptr, 0}, {nullptr, 0}}});
        for (int t = 0; t < ol; ++t) rec.push_back(RowRecipe{out + (size_t)(3 + t) * H, {t == ol - 1 ? prow(0) : prow(2), cin[t], {nullptr, 0}}});
        rec.push_back(RowRecipe{out + (size_t)(plen - 1) * H, {prow(6), cin.back(), {nullptr, 0}}});
        float *tr = trailing_ + (size_t)s * max_trailing_ * H;
        for (int i = 0; i < p.tcount; ++i) rec.push_back(RowRecipe{tr + (size_t)i * H, {prow(7 + i), {nullptr, 0}, {nullptr, 0}}});
        rec.push_back(RowRecipe{tr + (size_t)p.tcount * H, {prow(1), {nullptr, 0}, {nullptr, 0}}});
        rec.push_back(RowRecipe{tts_pad_ + (size_t)s * H, {prow(2), {nullptr, 0}, {nullptr, 0}}});
        tl[s] = p.tcount + 1;
        ntok[s] = p.n;
    }
    if ((int)rec.size() > recipe_cap_) { set_error("recipe overflow"); return false; }
    Q3T_HIP(hipMemcpyAsync(recipe_, rec.data(), rec.size() * sizeof(RowRecipe), hipMemcpyHostToDevice, stream_));
    if (!rows_recipe(recipe_, (int)rec.size(), H, stream_)) return false;
    Q3T_HIP(hipMemcpyAsync(trailing_len_, tl.data(), S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(n_tokens_, ntok.data(), S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(force_, force.data(), S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(done_, done0.data(), S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemsetAsync(seen_, 0, (size_t)S * c_.codec_vocab, stream_));
    Q3T_HIP(hipMemsetAsync(codes_, 0, (size_t)S * codes_max_len_ * NCB * 4, stream_));
    // ---- prefill: one causal pass over the plen rows of every slot; the last row's hidden state / logits per slot
    Q3T_HIP(hipMemcpyAsync(pf_slot_, slot_iota_, S * 4, hipMemcpyDeviceToDevice, stream_));
    if (!prefill(S, plen, prefill_, policy_slots_ > 0 ? policy_slots_ : S, stream_)) return false;
    Q3T_HIP(hipMemcpy2DAsync(hidden_, H * 4, pf_hid_ + (size_t)(plen - 1) * H, (size_t)plen * H * 4, H * 4, S,
                             hipMemcpyDeviceToDevice, stream_));
    Q3T_HIP(hipMemcpy2DAsync(logits_, (size_t)c_.codec_vocab * 4, pf_logits_ + (size_t)(plen - 1) * c_.codec_vocab,
                             (size_t)plen * c_.codec_vocab * 4, (size_t)c_.codec_vocab * 4, S, hipMemcpyDeviceToDevice, stream_));
    std::vector<int> posv(S);
    for (int s = 0; s < S; ++s) posv[s] = plen;
    if (!set_slot_state(S, posv, frame0)) return false;
    if (fused_select_ && !select_tokens(select_spec(SEL_CB0, gp_, 0, 0), logits_, S, stream_)) return false;
#ifdef Q3T_DEV
    const bool dbg = std::getenv("Q3T_DEBUG") != nullptr;
#else
    constexpr bool dbg = false;
#endif
    if (dbg) { fprintf(stderr, "[q3t] prefill enqueued (plen %d)\n", plen); fflush(stderr); }
    Q3T_HIP(hipEventRecord(e1, stream_));
    // ---- frame loop: one graph per frame; done flags polled every 16 frames
    if (!graph_for(g_frame_, S, &Engine::enqueue_frame)) return false;
    if (!ensure_pinned((size_t)S * 4)) return false;
    int *done_h = static_cast<int *>(pin_);
    // streaming (frame callback): chunk [start, start+interval) of every slot copied to pinned memory behind the
    // frame that completes it; delivered one chunk late so the GPU keeps running the queued frames meanwhile.  The
    // pinned chunks are the context's (chunk_pool_), reused across calls.
    const bool stream_cb = on_frames && interval > 0;
    struct Chunk { int start; int32_t *codes; int *done; hipEvent_t ev; };
    const size_t chunk_bytes = ((size_t)S * std::max(interval, 1) * NCB + S) * 4;
    size_t next_chunk = 0;   // chunk_pool_[0, next_chunk) are in use by this call
    std::vector<Chunk> pend;
    std::vector<Chunk> pool;
    auto take_chunk = [&](Chunk &c) -> bool {
        if (next_chunk == chunk_pool_.size()) chunk_pool_.push_back(PinnedChunk{});
        PinnedChunk &pc = chunk_pool_[next_chunk++];
        if (pc.cap < chunk_bytes) {
            if (pc.codes) hipHostFree(pc.codes);
            pc.codes = nullptr;
            pc.cap = 0;
            Q3T_HIP(hipHostMalloc(&pc.codes, chunk_bytes, hipHostMallocDefault));
            pc.cap = chunk_bytes;
        }
        if (!pc.ev) Q3T_HIP(hipEventCreateWithFlags(&pc.ev, hipEventDisableTiming));
        c.codes = pc.codes;
        c.done = pc.codes + (size_t)S * interval * NCB;
        c.ev = pc.ev;
        return true;
    };
    std::vector<int> &delivered = st.delivered, &stop_at = st.stop_at;
    int n_live = S;   // a fallback re-run regenerates utterances stopped earlier too (their frames are returned)
    auto release = [&]() {
        pend.clear();
        pool.clear();
        hipEventDestroy(e0); hipEventDestroy(e1); hipEventDestroy(e2);
    };
    // a chunk is handed to the caller only once the persistent kernels behind it are known to be fault-free
    auto deliver = [&](Chunk &c) -> bool {
        Q3T_HIP(hipEventSynchronize(c.ev));
        if (persist_error()) { *fault = true; return false; }
        for (int s = 0; s < S; ++s) {
            if (stop_at[s] >= 0) continue;
            const int nf = c.done[s] >= 0 ? c.done[s] : gp.max_len;
            if (nf < c.start + interval) continue;   // partial chunks go to the final flush, as in the reference
            if (c.start + interval <= delivered[s]) continue;   // delivered before a fallback re-run
            delivered[s] = c.start + interval;
            if (!on_frames(user, s, c.codes + (size_t)s * interval * NCB, interval, NCB)) {
                stop_at[s] = c.start + interval;
                const int d = stop_at[s];
                Q3T_HIP(hipMemcpyAsync(done_ + s, &d, 4, hipMemcpyHostToDevice, stream_));
                Q3T_HIP(hipStreamSynchronize(stream_));   // &d is a stack value
                --n_live;
            }
        }
        return true;
    };
    bool all_done = false;
    for (int f = 0; f < gp.max_len && !all_done && n_live > 0; ++f) {
        if (!persist_fault_hook(S, (persist_ ? 1 : 0) + (persist_cp_ ? 1 : 0))) return false;
        Q3T_HIP(hipGraphLaunch(g_frame_[S], stream_));
        if (dbg) { fprintf(stderr, "[q3t] frame %d launched\n", f); fflush(stderr); }
        if (stream_cb && (f + 1) % interval == 0) {
            Chunk c;
            if (!pool.empty()) { c = pool.back(); pool.pop_back(); }
            else if (!take_chunk(c)) { release(); return false; }
            c.start = f + 1 - interval;
            for (int s = 0; s < S; ++s)
                Q3T_HIP(hipMemcpyAsync(c.codes + (size_t)s * interval * NCB, codes_ + ((size_t)s * codes_max_len_ + c.start) * NCB,
                                       (size_t)interval * NCB * 4, hipMemcpyDeviceToHost, stream_));
            Q3T_HIP(hipMemcpyAsync(c.done, done_, S * 4, hipMemcpyDeviceToHost, stream_));
            Q3T_HIP(hipEventRecord(c.ev, stream_));
            pend.push_back(c);
            if (pend.size() > 1) {
                Chunk front = pend.front();
                pend.erase(pend.begin());
                pool.push_back(front);
                if (!deliver(front)) {
                    Q3T_HIP(hipStreamSynchronize(stream_));
                    release();
                    return false;
                }
            }
        }
        if ((f + 1) % poll_every_ == 0 && f + 1 < gp.max_len) {
            Q3T_HIP(hipMemcpyAsync(done_h, done_, S * 4, hipMemcpyDeviceToHost, stream_));
            Q3T_HIP(hipStreamSynchronize(stream_));
            all_done = true;
            for (int s = 0; s < S; ++s) all_done = all_done && done_h[s] >= 0;
        }
    }
    Q3T_HIP(hipEventRecord(e2, stream_));
    if (dbg) { fprintf(stderr, "[q3t] frame loop enqueued\n"); fflush(stderr); }
    Q3T_HIP(hipMemcpyAsync(done_h, done_, S * 4, hipMemcpyDeviceToHost, stream_));
    // one 1-D copy per slot into the caller's [n_utt][max_len][16] buffer (a pitched 2-D copy into pageable host memory
    // was observed to overrun the destination under rocprofv3 on ROCm 7.2)
    for (int s = 0; s < S; ++s)
        Q3T_HIP(hipMemcpyAsync(codes + (size_t)s * gp.max_len * NCB, codes_ + (size_t)s * codes_max_len_ * NCB,
                               (size_t)gp.max_len * NCB * 4, hipMemcpyDeviceToHost, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    if (dbg) { fprintf(stderr, "[q3t] frame loop done\n"); fflush(stderr); }
    if (persist_error()) {
        set_error("persistent kernel: an in-launch hand-off timed out");
        *fault = true;
        release();
        return false;
    }
    for (int s = 0; s < S; ++s) n_frames[s] = done_h[s] >= 0 ? std::min(done_h[s], gp.max_len) : gp.max_len;
    if (stream_cb) {
        std::vector<Chunk> last;
        last.swap(pend);
        for (Chunk &c : last) pool.push_back(c);
        for (Chunk &c : last)
            if (!deliver(c)) { release(); return false; }
        for (int s = 0; s < S; ++s) {
            if (stop_at[s] >= 0) { n_frames[s] = std::min(n_frames[s], stop_at[s]); continue; }
            if (n_frames[s] > delivered[s])   // final flush (tts_transformer.cpp:2563-2570)
                on_frames(user, s, codes + ((size_t)s * gp.max_len + delivered[s]) * NCB, n_frames[s] - delivered[s], NCB);
        }
    }
    float ms1 = 0, ms2 = 0;
    hipEventElapsedTime(&ms1, e0, e1);
    hipEventElapsedTime(&ms2, e1, e2);
    last_prefill_ms = ms1;
    last_frames_ms = ms2;
    release();
    return true;
}

// ------------------------------------------------------------------------------------------ continuous batching
// Admissions run on their own stream with private scratch, overlapping the frame loop of the other slots (at many
// slots the decode step leaves most of the chip idle).  The slots freed since the last admission are admitted
// together: their prompts are projected in one pass and run through ONE causal prefill (Engine::prefill), which
// writes the K/V rows [0, plen) of the target slots directly.  A target slot is parked in the frame loop meanwhile
// (done >= 0: no selection, no advance, its position >= plen): the frame graph still runs it, but writes only its own
// x / hidden / logits rows and the KV row at its parked position, none of which the admission writes.  The slot joins
// the frame loop (activate_slot, main stream, between two frames) once its admission batch has finished.  The prefill
// runs the running batch's kernels (S_main = q_slots_), whose per-row arithmetic does not depend on the other rows: a
// slot's prefill is what generate()'s prefill computes for it, whichever slots were admitted alongside.
bool Engine::alloc_admission() {
    if (astream_) return true;
    const int S = max_slots_, H = c_.hidden;
    if (!ensure_prefill()) return false;
    aprefill_ = dalloc<float>((size_t)S * 10 * H);
    ahidden_ = dalloc<float>((size_t)S * H);
    alogits_ = dalloc<float>((size_t)S * c_.codec_vocab);
    aproj_cap_ = S * (max_trailing_ + 16);
    aproj_idx_ = dalloc<int>(aproj_cap_);
    aproj_h_ = dalloc<uint16_t>((size_t)aproj_cap_ * c_.text_dim);
    aproj_out_ = dalloc<float>((size_t)aproj_cap_ * H);
    arecipe_ = dalloc<RowRecipe>(aproj_cap_);
    if (!aprefill_ || !ahidden_ || !alogits_ || !aproj_idx_ || !aproj_h_ || !aproj_out_ || !arecipe_) {
        set_error("device allocation failed");
        return false;
    }
    // every buffer was zeroed on stream_ and drained by dalloc before the admission stream exists
    Q3T_HIP(hipStreamCreateWithFlags(&astream_, hipStreamNonBlocking));
    return true;
}

// admission batch on stream `as`: utterances utt[j] into slots tgt[j] (text projection, prefill / trailing / pad
// rows, the causal prefill into the target slots, hidden / logits rows per target slot).  tgt_h: pinned
// copy of tgt (alive until the batch has run); trailing_len[j]: the slot's trailing-text length
bool Engine::admit_batch(const std::vector<int> &tgt, const std::vector<int> &utt, const int32_t *const *tokens,
                         const int *n_tokens, const float *const *speaker, const GenParams &gp, int plen, hipStream_t as,
                         int *tgt_h, std::vector<int> &trailing_len) {
    const int H = c_.hidden, a = (int)tgt.size();
    std::vector<const int32_t *> tk(a);
    std::vector<int> nt(a);
    for (int j = 0; j < a; ++j) { tk[j] = tokens[utt[j]]; nt[j] = n_tokens[utt[j]]; }
    std::vector<int> idx;
    std::vector<SlotPlan> plan;
    if (!plan_rows(c_, a, tk.data(), nt.data(), max_trailing_, idx, plan)) return false;
    if ((int)idx.size() > aproj_cap_) { set_error("too many text rows"); return false; }
    Q3T_HIP(hipMemcpyAsync(aproj_idx_, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, as));
    if (!enqueue_text_projection((int)idx.size(), as, aproj_idx_, aproj_h_, aproj_out_)) return false;
    std::vector<RowRecipe> rec;
    auto crow = [&](int id) { return RowTerm{codec_embd_ + (size_t)id * H, 1}; };
    for (int j = 0; j < a; ++j) {
        const int k = tgt[j];
        const float *spk = speaker ? speaker[utt[j]] : nullptr;
        float *spk_dev = cp_in1_ + (size_t)k * H;
        if (spk) Q3T_HIP(hipMemcpyAsync(spk_dev, spk, H * 4, hipMemcpyHostToDevice, as));
        const SlotPlan &p = plan[j];
        const float *P = aproj_out_ + (size_t)p.rb * H;
        auto prow = [&](int i) { return RowTerm{P + (size_t)i * H, 0}; };
        std::vector<RowTerm> cin;
        if (gp.language_id < 0) cin = {crow(c_.nothink), crow(c_.think_bos), crow(c_.think_eos)};
        else cin = {crow(c_.think), crow(c_.think_bos), crow(gp.language_id), crow(c_.think_eos)};
        if (spk) cin.push_back(RowTerm{spk_dev, 0});
        cin.push_back(crow(c_.codec_pad));
        cin.push_back(crow(c_.codec_bos));
        const int ol = (int)cin.size() - 1;
        if (3 + ol + 1 != plen) { set_error("admit_batch: prefill length mismatch"); return false; }
        float *out = aprefill_ + (size_t)j * 10 * H;
        for (int r = 0; r < 3; ++r) rec.push_back(RowRecipe{out + (size_t)r * H, {prow(3 + r), {nullptr, 0}, {nullptr, 0}}});
        for (int t = 0; t < ol; ++t) rec.push_back(RowRecipe{out + (size_t)(3 + t) * H, {t == ol - 1 ? prow(0) : prow(2), cin[t], {nullptr, 0}}});
        rec.push_back(RowRecipe{out + (size_t)(plen - 1) * H, {prow(6), cin.back(), {nullptr, 0}}});
        float *tr = trailing_ + (size_t)k * max_trailing_ * H;
        for (int i = 0; i < p.tcount; ++i) rec.push_back(RowRecipe{tr + (size_t)i * H, {prow(7 + i), {nullptr, 0}, {nullptr, 0}}});
        rec.push_back(RowRecipe{tr + (size_t)p.tcount * H, {prow(1), {nullptr, 0}, {nullptr, 0}}});
        rec.push_back(RowRecipe{tts_pad_ + (size_t)k * H, {prow(2), {nullptr, 0}, {nullptr, 0}}});
        trailing_len[j] = p.tcount + 1;
    }
    if ((int)rec.size() > aproj_cap_) { set_error("recipe overflow"); return false; }
    Q3T_HIP(hipMemcpyAsync(arecipe_, rec.data(), rec.size() * sizeof(RowRecipe), hipMemcpyHostToDevice, as));
    if (!rows_recipe(arecipe_, (int)rec.size(), H, as)) return false;
    // the causal prefill of the batch with the running batch's kernels (S_main = q_slots_), K/V straight into the
    // target slots' rows [0, plen)
    for (int j = 0; j < a; ++j) tgt_h[j] = tgt[j];
    Q3T_HIP(hipMemcpyAsync(pf_slot_, tgt_h, a * 4, hipMemcpyHostToDevice, as));
    if (!prefill(a, plen, aprefill_, q_slots_, as)) return false;
    const int V = c_.codec_vocab;
    for (int j = 0; j < a; ++j) {
        const size_t r = (size_t)j * plen + plen - 1;
        Q3T_HIP(hipMemcpyAsync(ahidden_ + (size_t)tgt[j] * H, pf_hid_ + r * H, H * 4, hipMemcpyDeviceToDevice, as));
        Q3T_HIP(hipMemcpyAsync(alogits_ + (size_t)tgt[j] * V, pf_logits_ + r * V, (size_t)V * 4, hipMemcpyDeviceToDevice, as));
    }
    return true;
}

// slot k joins the frame loop (main stream, between two frames, after its admission batch): per-slot state, the
// last prefill step's hidden state, and the CB0 of its first frame selected from the last prefill logits.
// state_h: pinned [8]
bool Engine::activate_slot(int k, uint64_t utt, int trailing_len, int n_tok, const GenParams &gp, int plen, int *state_h) {
    const int H = c_.hidden, NCB = 16;
    state_h[0] = trailing_len; state_h[1] = n_tok; state_h[2] = gp.force_frames; state_h[3] = -1;
    state_h[4] = plen; state_h[5] = 0;
    std::memcpy(state_h + 6, &utt, 8);
    Q3T_HIP(hipMemcpyAsync(trailing_len_ + k, state_h + 0, 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(n_tokens_ + k, state_h + 1, 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(force_ + k, state_h + 2, 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(utt_ + k, state_h + 6, 8, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemsetAsync(seen_ + (size_t)k * c_.codec_vocab, 0, c_.codec_vocab, stream_));
    Q3T_HIP(hipMemsetAsync(codes_ + (size_t)k * codes_max_len_ * NCB, 0, (size_t)codes_max_len_ * NCB * 4, stream_));
    Q3T_HIP(hipMemcpyAsync(hidden_ + (size_t)k * H, ahidden_ + (size_t)k * H, H * 4, hipMemcpyDeviceToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(pos_ + k, state_h + 4, 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(frame_ + k, state_h + 5, 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(done_ + k, state_h + 3, 4, hipMemcpyHostToDevice, stream_));
    SelectSpec sp = select_spec(SEL_CB0, gp_, 0, 0);   // the slot's rows of every per-slot array
    sp.tokens += (size_t)k * 16; sp.codes += (size_t)k * codes_max_len_ * NCB; sp.frame += k; sp.done += k; sp.utt += k;
    sp.seen += (size_t)k * c_.codec_vocab; sp.n_tokens += k; sp.force_frames += k;
    if (sp.ticket) sp.ticket += k;
    return select_tokens(sp, alogits_ + (size_t)k * c_.codec_vocab, 1, stream_);
}

bool Engine::generate_queue_once(int n_utt, const int32_t *const *tokens, const int *n_tokens, const float *const *speaker,
                                 const GenParams &gp, int32_t *codes, int *n_frames, int max_active, bool *faulted) {
    *faulted = false;
    if (n_utt <= 0) return true;
    const int S = std::min(max_slots_, n_utt), NCB = 16;
    if (max_active <= 0 || max_active > S) max_active = S;
    for (int u = 0; u < n_utt; ++u) n_frames[u] = 0;
    if (gp.max_len <= 0) return true;
    if (gp.language_id >= c_.codec_vocab) { set_error("language id out of range"); return false; }
    const bool has_spk = speaker && speaker[0];
    for (int u = 0; u < n_utt; ++u)
        if ((speaker && speaker[u]) != has_spk) { set_error("speaker embedding must be given for all or none of the utterances"); return false; }
    {   // validate every prompt before anything runs
        std::vector<int> idx;
        std::vector<SlotPlan> plan;
        if (!plan_rows(c_, n_utt, tokens, n_tokens, max_trailing_, idx, plan)) return false;
    }
    const int n_pre = gp.language_id < 0 ? 3 : 4;
    const int plen = 3 + (n_pre + (has_spk ? 1 : 0) + 2 - 1) + 1;
    if (plen + gp.max_len + 8 > max_ctx_) { set_error("max_len exceeds the context reserved at ctx creation"); return false; }
    if (gp.max_len > codes_max_len_) { set_error("max_len exceeds the code buffer"); return false; }
    if (!alloc_admission()) return false;
    q_slots_ = S;
    // the single-slot context runs persistent kernels, which need the whole device: admissions go on the main stream
    hipStream_t as = (S == 1 && persist_enabled()) ? stream_ : astream_;
    if (!(gp.temperature == gp_.temperature && gp.top_k == gp_.top_k && gp.rep_penalty == gp_.rep_penalty)) {
        for (auto &kv : g_frame_) hipGraphExecDestroy(kv.second);
        g_frame_.clear();
    }
    gp_ = gp;
    if (!set_seed(gp.seed, stream_)) return false;
    // the finished utterances' codes, copied to the caller once at the end (device scratch kept by the context)
    if (!ensure_qout((size_t)n_utt * gp.max_len * NCB * 4)) return false;
    int32_t *out_dev = static_cast<int32_t *>(qout_);
    // [S][8] activation staging, [S] done flags, [S] admission targets, one constant 0 (parking): pinned, kept
    if (!ensure_pinned(((size_t)S * 10 + 1) * 4)) return false;
    int *pin = static_cast<int *>(pin_);
    int *done_h = pin + (size_t)S * 8, *tgt_h = pin + (size_t)S * 9, *park = pin + (size_t)S * 10;
    *park = 0;
    hipEvent_t aev = nullptr, pev = nullptr;
    auto cleanup = [&]() {
        hipStreamSynchronize(as);
        hipStreamSynchronize(stream_);
        if (aev) hipEventDestroy(aev);
        if (pev) hipEventDestroy(pev);
        policy_slots_ = 0;
        std::vector<uint64_t> ident(max_slots_);   // generate() keys sampling by slot index again
        for (int k = 0; k < max_slots_; ++k) ident[k] = (uint64_t)k;
        hipMemcpyAsync(utt_, ident.data(), max_slots_ * 8, hipMemcpyHostToDevice, stream_);
        hipStreamSynchronize(stream_);
    };
    Q3T_HIP(hipEventCreateWithFlags(&aev, hipEventDisableTiming));
    Q3T_HIP(hipEventCreateWithFlags(&pev, hipEventDisableTiming));
    // every slot starts parked: done = 0 (no selection, no advance), position plen (above the rows a prefill writes),
    // valid code ids for the gathers it still runs through, no trailing text
    {
        std::vector<int> pl(S, plen);
        Q3T_HIP(hipMemsetAsync(done_, 0, S * 4, stream_));
        Q3T_HIP(hipMemcpyAsync(pos_, pl.data(), S * 4, hipMemcpyHostToDevice, stream_));
        Q3T_HIP(hipMemsetAsync(frame_, 0, S * 4, stream_));
        Q3T_HIP(hipMemsetAsync(tokens_, 0, (size_t)S * 16 * 4, stream_));
        Q3T_HIP(hipMemsetAsync(trailing_len_, 0, S * 4, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
    }
    enum { FREE, PENDING, ACTIVE };
    std::vector<int> state(S, FREE), slot_utt(S, -1), started(S, 0), tl(S, 0);
    std::vector<int> batch_tgt, batch_tl;   // the admission batch in flight (at most one)
    int next = 0, f = 0, n_fin = 0, n_busy = 0;
    auto admit = [&]() -> bool {   // every free slot, up to max_active busy, one batch
        std::vector<int> tgt, utt;
        for (int k = 0; k < S && next + (int)tgt.size() < n_utt && n_busy + (int)tgt.size() < max_active; ++k)
            if (state[k] == FREE) { tgt.push_back(k); utt.push_back(next + (int)tgt.size() - 1); }
        if (tgt.empty()) return true;
        batch_tl.assign(tgt.size(), 0);
        if (!admit_batch(tgt, utt, tokens, n_tokens, has_spk ? speaker : nullptr, gp, plen, as, tgt_h, batch_tl)) return false;
        Q3T_HIP(hipEventRecord(aev, as));
        for (size_t j = 0; j < tgt.size(); ++j) {
            state[tgt[j]] = PENDING;
            slot_utt[tgt[j]] = utt[j];
            tl[tgt[j]] = batch_tl[j];
        }
        next += (int)tgt.size();
        n_busy += (int)tgt.size();
        batch_tgt = tgt;
        return true;
    };
    auto activate = [&]() -> bool {   // the batch in flight has finished: its slots join the frame loop
        if (as != stream_) Q3T_HIP(hipStreamWaitEvent(stream_, aev, 0));
        for (int k : batch_tgt) {
            const int u = slot_utt[k];
            if (!activate_slot(k, (uint64_t)u, tl[k], n_tokens[u], gp, plen, pin + (size_t)k * 8)) return false;
            state[k] = ACTIVE;
            started[k] = f;
        }
        batch_tgt.clear();
        return true;
    };
    if (!admit() || !activate()) { cleanup(); return false; }
    // frame graph over slots [0, S_eff): S_eff = the highest busy slot + 1, rounded up to 8, never below the smallest
    // batch that keeps the S-slot kernel family (matrix cores from 4 slots, k_attn_seq from 16), whose per-token
    // arithmetic the graph reproduces (policy_slots_ = S): a draining queue stops paying for parked slots
    const int fam = !mm_ok_ ? 1 : S >= 16 ? 16 : S >= gemm_mfma_min_batch() ? gemm_mfma_min_batch() : S;
    policy_slots_ = S;
    auto frame_graph = [&](hipGraphExec_t *g) -> bool {
        int hi = 0;
        for (int k = 0; k < S; ++k) if (state[k] != FREE) hi = k + 1;
        int se = fam < S ? std::max(fam, std::min(S, (hi + 7) / 8 * 8)) : S;
        if (!graph_for_key(g_frame_, se + 65536 * S, se, &Engine::enqueue_frame)) return false;
        *g = g_frame_[se + 65536 * S];
        return true;
    };
    bool polled = false;   // one frame in flight: frame f is launched before frame f-1's done flags are read
    while (n_fin < n_utt) {
        int n_active = 0;
        for (int k = 0; k < S; ++k) n_active += state[k] == ACTIVE;
        if (n_active == 0) {   // only an admission in flight: wait for it instead of running empty frames
            if (batch_tgt.empty() && !admit()) { cleanup(); return false; }
            Q3T_HIP(hipEventSynchronize(aev));
            if (!activate()) { cleanup(); return false; }
            polled = false;
            continue;
        }
        hipGraphExec_t fg = nullptr;
        if (!frame_graph(&fg)) { cleanup(); return false; }
        if (!persist_fault_hook(S, (persist_ ? 1 : 0) + (persist_cp_ ? 1 : 0))) { cleanup(); return false; }
        Q3T_HIP(hipGraphLaunch(fg, stream_));
        ++f;
        if (polled) {
            Q3T_HIP(hipEventSynchronize(pev));
            for (int k = 0; k < S; ++k) {   // done_h: after frame f-1
                if (state[k] != ACTIVE) continue;
                const int ran = f - 1 - started[k];
                const int d = done_h[k];
                if (d < 0 && ran < gp.max_len) continue;
                const int u = slot_utt[k];
                n_frames[u] = d >= 0 ? std::min(d, gp.max_len) : gp.max_len;
                Q3T_HIP(hipMemcpyAsync(out_dev + (size_t)u * gp.max_len * NCB, codes_ + (size_t)k * codes_max_len_ * NCB,
                                       (size_t)gp.max_len * NCB * 4, hipMemcpyDeviceToDevice, stream_));
                if (d < 0)   // stopped at max_len: park the slot (no selection, no advance)
                    Q3T_HIP(hipMemcpyAsync(done_ + k, park, 4, hipMemcpyHostToDevice, stream_));
                state[k] = FREE;
                slot_utt[k] = -1;
                --n_busy;
                ++n_fin;
            }
        }
        if (!batch_tgt.empty() && (as == stream_ || hipEventQuery(aev) == hipSuccess) && !activate()) { cleanup(); return false; }
        if (batch_tgt.empty() && next < n_utt && !admit()) { cleanup(); return false; }
        if (as == stream_ && !batch_tgt.empty() && !activate()) { cleanup(); return false; }
        Q3T_HIP(hipMemcpyAsync(done_h, done_, S * 4, hipMemcpyDeviceToHost, stream_));
        Q3T_HIP(hipEventRecord(pev, stream_));
        polled = true;
        if (f > (n_utt + 1) * (gp.max_len + plen + 2)) { cleanup(); set_error("generate_queue: no progress"); return false; }
    }
    for (int u = 0; u < n_utt; ++u)
        Q3T_HIP(hipMemcpyAsync(codes + (size_t)u * gp.max_len * NCB, out_dev + (size_t)u * gp.max_len * NCB,
                               (size_t)gp.max_len * NCB * 4, hipMemcpyDeviceToHost, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    const bool fault = persist_error();
    cleanup();
    if (fault) { set_error("persistent kernel: an in-launch hand-off timed out"); *faulted = true; return false; }
    return true;
}

bool Engine::generate_queue(int n_utt, const int32_t *const *tokens, const int *n_tokens, const float *const *speaker,
                            const GenParams &gp, int32_t *codes, int *n_frames, int max_active) {
    const int S = std::min(max_slots_, std::max(n_utt, 1));
    DeviceLock lk(persist_exclusive(S), device_);
    bool fault = false;
    if (generate_queue_once(n_utt, tokens, n_tokens, speaker, gp, codes, n_frames, max_active, &fault)) return true;
    if (!fault) return false;
    // a single-slot persistent launch gave up on a hand-off: continue on the launch-per-op graphs, which are
    // bit-identical, and re-run the queue (sampling is keyed by utterance, so the re-run gives the same codes)
    if (!persist_recover()) return false;
    return generate_queue_once(n_utt, tokens, n_tokens, speaker, gp, codes, n_frames, max_active, &fault);
}

bool Engine::time_stage(int stage, int S, int pos, int iters, double *ms) {
    if (S <= 0 || S > max_slots_ || pos < 0 || pos >= max_ctx_ || iters <= 0) { set_error("time_stage: bad arguments"); return false; }
    DeviceLock lk(persist_exclusive(S), device_);
    std::vector<int> pv(S, pos), fr(S, 0), dn(S, -1);
    Q3T_HIP(hipMemcpyAsync(pos_, pv.data(), S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(frame_, fr.data(), S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(done_, dn.data(), S * 4, hipMemcpyHostToDevice, stream_));
    hipGraphExec_t g = nullptr;
    if (stage == 0) { if (!graph_for(g_talker_, S, &Engine::enqueue_talker_step)) return false; g = g_talker_[S]; }
    else { if (!graph_for(g_cp_, S, &Engine::enqueue_cp_only)) return false; g = g_cp_[S]; }
    Q3T_HIP(hipGraphLaunch(g, stream_));   // warm
    // one event pair around EACH replay, on the stream the kernels run on: the mean is the replay's own duration (for
    // the persistent stages, the one kernel's), without the host-side gap between two graph launches
    std::vector<hipEvent_t> ev(2 * (size_t)iters, nullptr);
    for (hipEvent_t &e : ev) Q3T_HIP(hipEventCreate(&e));
    for (int i = 0; i < iters; ++i) {
        Q3T_HIP(hipEventRecord(ev[2 * i], stream_));
        Q3T_HIP(hipGraphLaunch(g, stream_));
        Q3T_HIP(hipEventRecord(ev[2 * i + 1], stream_));
    }
    Q3T_HIP(hipEventSynchronize(ev.back()));
    double sum = 0.0;
    for (int i = 0; i < iters; ++i) {
        float t = 0;
        hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]);
        sum += t;
    }
    for (hipEvent_t e : ev) hipEventDestroy(e);
    *ms = sum / iters;
    if (persist_error()) {   // time the launch-per-op fallback instead of a faulted persistent launch
        if (!persist_recover()) return false;
        return time_stage(stage, S, pos, iters, ms);
    }
    return true;
}

// ------------------------------------------------------------------------------------------ test entry points
bool Engine::talker_prefill(int n_utt, int n_rows, const float *embd, int family_slots, float *hidden, float *logits) {
    if (n_utt <= 0 || n_utt > max_slots_) { set_error("bad utterance count"); return false; }
    if (n_rows <= 0 || n_rows > 10 || n_rows > max_ctx_) { set_error("prefill rows must be in [1, 10]"); return false; }
    if (family_slots < 0 || family_slots > 4096) { set_error("bad family slot count"); return false; }
    const int H = c_.hidden, V = c_.codec_vocab;
    DeviceLock lk(false, device_);
    if (!ensure_prefill()) return false;
    Q3T_HIP(hipMemcpy2DAsync(prefill_, (size_t)10 * H * 4, embd, (size_t)n_rows * H * 4, (size_t)n_rows * H * 4, n_utt,
                             hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(pf_slot_, slot_iota_, n_utt * 4, hipMemcpyDeviceToDevice, stream_));
    if (!prefill(n_utt, n_rows, prefill_, family_slots > 0 ? family_slots : n_utt, stream_)) return false;
    if (hidden) Q3T_HIP(hipMemcpyAsync(hidden, pf_hid_, (size_t)n_utt * n_rows * H * 4, hipMemcpyDeviceToHost, stream_));
    if (logits)
        Q3T_HIP(hipMemcpy2DAsync(logits, (size_t)V * 4, pf_logits_ + (size_t)(n_rows - 1) * V, (size_t)n_rows * V * 4,
                                 (size_t)V * 4, n_utt, hipMemcpyDeviceToHost, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    return true;
}

bool Engine::talker_forward(int S, const float *embd, const int *pos, float *hidden, float *logits) {
    if (S <= 0 || S > max_slots_) { set_error("bad slot count"); return false; }
    for (int s = 0; s < S; ++s) if (pos[s] < 0 || pos[s] >= max_ctx_) { set_error("Context length exceeded"); return false; }
    const int H = c_.hidden;
    DeviceLock lk(persist_exclusive(S), device_);
    for (int attempt = 0; attempt < 2; ++attempt) {
        Q3T_HIP(hipMemcpyAsync(x_, embd, (size_t)S * H * 4, hipMemcpyHostToDevice, stream_));
        Q3T_HIP(hipMemcpyAsync(pos_, pos, S * 4, hipMemcpyHostToDevice, stream_));
        if (!graph_for(g_talker_, S, &Engine::enqueue_talker_step)) return false;
        Q3T_HIP(hipGraphLaunch(g_talker_[S], stream_));
        if (hidden) Q3T_HIP(hipMemcpyAsync(hidden, hidden_, (size_t)S * H * 4, hipMemcpyDeviceToHost, stream_));
        if (logits) Q3T_HIP(hipMemcpyAsync(logits, logits_, (size_t)S * c_.codec_vocab * 4, hipMemcpyDeviceToHost, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
        if (!persist_error()) return true;
        if (!persist_recover()) return false;   // re-run this position on the launch-per-op graph
    }
    set_error("talker step: persistent fallback failed");
    return false;
}

bool Engine::codepred_frame(int S, const float *hidden, const int *cb0, float temperature, int top_k, uint64_t seed,
                            int frame, int32_t *codes15, float *logits_all) {
    if (S <= 0 || S > max_slots_) { set_error("bad slot count"); return false; }
    const int H = c_.hidden;
    for (int s = 0; s < S; ++s) if (cb0[s] < 0 || cb0[s] >= c_.codec_vocab) { set_error("cb0 out of range"); return false; }
    DeviceLock lk(persist_exclusive(S), device_);
    GenParams gp = gp_;
    gp.temperature = temperature; gp.top_k = top_k; gp.seed = seed;
    gp_ = gp;
    if (!set_seed(seed, stream_)) return false;
    for (auto &kv : g_frame_) hipGraphExecDestroy(kv.second);
    g_frame_.clear();
    Q3T_HIP(hipMemcpyAsync(hidden_, hidden, (size_t)S * H * 4, hipMemcpyHostToDevice, stream_));
    std::vector<int> tk0((size_t)S * 16, 0);
    for (int s = 0; s < S; ++s) tk0[(size_t)s * 16] = cb0[s];
    Q3T_HIP(hipMemcpyAsync(tokens_, tk0.data(), tk0.size() * 4, hipMemcpyHostToDevice, stream_));
    std::vector<int> fr(S, frame), dn(S, -1);
    Q3T_HIP(hipMemcpyAsync(frame_, fr.data(), S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(done_, dn.data(), S * 4, hipMemcpyHostToDevice, stream_));
    if (!enqueue_cp_frame(S, stream_, logits_all)) return false;
    std::vector<int> tk((size_t)S * 16);
    Q3T_HIP(hipMemcpyAsync(tk.data(), tokens_, tk.size() * 4, hipMemcpyDeviceToHost, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    if (persist_error()) {   // re-run the frame on the per-op launches
        if (!persist_recover()) return false;
        Q3T_HIP(hipMemcpyAsync(tokens_, tk0.data(), tk0.size() * 4, hipMemcpyHostToDevice, stream_));
        if (!enqueue_cp_frame(S, stream_, logits_all)) return false;
        Q3T_HIP(hipMemcpyAsync(tk.data(), tokens_, tk.size() * 4, hipMemcpyDeviceToHost, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
    }
    for (int s = 0; s < S; ++s) for (int i = 0; i < 15; ++i) codes15[s * 15 + i] = tk[(size_t)s * 16 + 1 + i];
    return true;
}

bool Engine::cb0_select_host(int S, const float *logits, const uint8_t *seen, const int *frame, const int *n_tokens,
                             const GenParams &gp, int *tok) {
    if (S <= 0 || S > max_slots_) { set_error("bad slot count"); return false; }
    const int V = c_.codec_vocab;
    DeviceLock lk(false, device_);
    Q3T_HIP(hipMemcpyAsync(logits_, logits, (size_t)S * V * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(seen_, seen, (size_t)S * V, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(frame_, frame, S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(n_tokens_, n_tokens, S * 4, hipMemcpyHostToDevice, stream_));
    std::vector<int> force(S, gp.force_frames), dn(S, -1);
    Q3T_HIP(hipMemcpyAsync(force_, force.data(), S * 4, hipMemcpyHostToDevice, stream_));
    Q3T_HIP(hipMemcpyAsync(done_, dn.data(), S * 4, hipMemcpyHostToDevice, stream_));
    SelectSpec sp = select_spec(SEL_CB0, gp, 0, 0);
    sp.seed_dev = nullptr;
    if (!select_tokens(sp, logits_, S, stream_)) return false;
    std::vector<int> tk((size_t)S * 16);
    Q3T_HIP(hipMemcpyAsync(tk.data(), tokens_, tk.size() * 4, hipMemcpyDeviceToHost, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    for (int s = 0; s < S; ++s) tok[s] = tk[(size_t)s * 16];
    return true;
}

}  // namespace q3t
