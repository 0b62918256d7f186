// vocoder.cpp — Qwen3-TTS tokenizer decoder on MI355X (see vocoder.h).  Restates, stage by stage,
// AudioTokenizerDecoder::build_graph (src/audio_tokenizer_decoder.cpp:622-802) with time-major activations.
#include "vocoder.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "vocoder_kernels.h"

namespace q3t {

Vocoder::~Vocoder() {
    for (void *p : allocs_) hipFree(p);
    for (void *p : scratch_) hipFree(p);
}

template <class T>
T *Vocoder::dalloc(size_t n) {
    void *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
    allocs_.push_back(p);
    return static_cast<T *>(p);
}

namespace {
const uint16_t *f16p(const GgufTensor *t) { return static_cast<const uint16_t *>(t->data); }
}  // namespace

bool Vocoder::load(const std::string &path, hipStream_t s, bool recv_weights) {
    stream_ = s;
    Gguf g;
    if (!g.open(path)) { set_error(g.error()); return false; }
    wa_.recv = recv_weights;
    const bool recv = recv_weights;   // shapes only: the tensor bytes are never read on receiving ranks
    size_t total = 0;
    for (const GgufTensor &t : g.tensors()) total += (t.nbytes() + 255) & ~(size_t)255;
    if (!wa_.reserve(total + ((size_t)1 << 20))) return false;
    auto T = [&](const std::string &n) -> const GgufTensor * {
        const GgufTensor *t = g.find(n);
        if (!t) set_error("missing vocoder tensor " + n);
        return t;
    };
    auto up16 = [&](const void *src, size_t n) -> uint16_t * {
        uint16_t *d = wa_.alloc<uint16_t>(n);
        if (d && !wa_.put(d, src, n * 2)) return nullptr;
        return d;
    };
    auto up32n = [&](const float *src, size_t n) -> float * {
        float *d = wa_.alloc<float>(n);
        if (d && !wa_.put(d, src, n * 4)) return nullptr;
        return d;
    };
    auto vec = [&](const std::string &n, int64_t expect) -> float * {
        const GgufTensor *t = T(n);
        if (!t) return nullptr;
        if (t->type != GGML_TYPE_F32 || (expect > 0 && t->nelements() != expect)) { set_error("bad f32 tensor " + n); return nullptr; }
        return up32n((const float *)t->data, (size_t)t->nelements());
    };
    // conv weight ne [K, C_in, C_out] (PyTorch [oc][ic][k]) -> per-tap [K][C_out][C_in]
    auto conv_w = [&](const std::string &n, Conv &c) -> bool {
        const GgufTensor *t = T(n);
        if (!t || t->type != GGML_TYPE_F16 || t->n_dims != 3) { set_error("bad conv " + n); return false; }
        c.k = (int)t->ne[0]; c.ic = (int)t->ne[1]; c.oc = (int)t->ne[2];
        const size_t nw = (size_t)c.k * c.oc * c.ic;
        std::vector<uint16_t> w(recv ? 0 : nw);
        const uint16_t *src = f16p(t);
        if (!recv)
            for (int oc = 0; oc < c.oc; ++oc)
                for (int ic = 0; ic < c.ic; ++ic)
                    for (int k = 0; k < c.k; ++k) w[((size_t)k * c.oc + oc) * c.ic + ic] = src[((size_t)oc * c.ic + ic) * c.k + k];
        c.w = up16(w.data(), nw);
        return c.w != nullptr;
    };
    // conv-transpose weight ne [K, C_out, C_in] (PyTorch [ic][oc][k]) -> per-tap [K][C_out][C_in]
    auto convT_w = [&](const std::string &n, Conv &c) -> bool {
        const GgufTensor *t = T(n);
        if (!t || t->type != GGML_TYPE_F16 || t->n_dims != 3) { set_error("bad conv_t " + n); return false; }
        c.k = (int)t->ne[0]; c.oc = (int)t->ne[1]; c.ic = (int)t->ne[2];
        const size_t nw = (size_t)c.k * c.oc * c.ic;
        std::vector<uint16_t> w(recv ? 0 : nw);
        const uint16_t *src = f16p(t);
        if (!recv)
            for (int ic = 0; ic < c.ic; ++ic)
                for (int oc = 0; oc < c.oc; ++oc)
                    for (int k = 0; k < c.k; ++k) w[((size_t)k * c.oc + oc) * c.ic + ic] = src[((size_t)ic * c.oc + oc) * c.k + k];
        c.w = up16(w.data(), nw);
        return c.w != nullptr;
    };
    auto mat = [&](const std::string &n, int &rows, int &cols) -> uint16_t * {
        const GgufTensor *t = T(n);
        if (!t || t->type != GGML_TYPE_F16) { set_error("bad matrix " + n); return nullptr; }
        cols = (int)(t->ne[0] == 1 && t->n_dims == 3 ? t->ne[1] : t->ne[0]);
        rows = (int)(t->nelements() / cols);
        return up16(t->data, (size_t)t->nelements());
    };
    // SnakeBeta: x + exp(-beta) * sin^2(exp(alpha) * x) (apply_snake, :375-402); exps precomputed once
    auto snake = [&](const std::string &pa, const std::string &pb, Snake &sn) -> bool {
        const GgufTensor *a = T(pa), *b = T(pb);
        if (!a || !b || a->type != GGML_TYPE_F32 || b->nelements() != a->nelements()) { set_error("bad snake " + pa); return false; }
        const size_t n = (size_t)a->nelements();
        std::vector<float> ea(recv ? 0 : n), ib(recv ? 0 : n);
        if (!recv)
            for (size_t i = 0; i < n; ++i) {
                ea[i] = expf(((const float *)a->data)[i]);
                ib[i] = expf(-((const float *)b->data)[i]);
            }
        sn.a = up32n(ea.data(), n);
        sn.ib = up32n(ib.data(), n);
        sn.n = (int)a->nelements();
        return sn.a && sn.ib;
    };

    // codebooks, divided by their usage counts when the file still carries them (normalize_codebooks,
    // src/audio_tokenizer_decoder.cpp:40-73: row r *= 1 / max(usage[r], 1e-5), re-rounded to f16).  The converter
    // already divides and drops *.usage (scripts/convert_tokenizer_to_gguf.py:347-359), so this is normally a no-op.
    auto codebook = [&](const std::string &name, const std::string &usage_name, uint16_t *&dst) -> bool {
        const GgufTensor *t = T(name);
        if (!t || t->type != GGML_TYPE_F16 || t->ne[0] != cb_dim_ || t->ne[1] != cb_size_) { set_error("bad codebook " + name); return false; }
        const GgufTensor *u = g.find(usage_name);
        if (!u) { dst = up16(t->data, (size_t)t->nelements()); return dst != nullptr; }
        if (u->type != GGML_TYPE_F32 || u->nelements() != cb_size_) { set_error("bad codebook usage " + usage_name); return false; }
        std::vector<uint16_t> w(recv ? 0 : (size_t)t->nelements());
        if (!recv) {
            const uint16_t *src = f16p(t);
            const float *us = static_cast<const float *>(u->data);
            for (int r = 0; r < cb_size_; ++r) {
                const float inv = 1.0f / std::max(us[r], 1e-5f);
                for (int d = 0; d < cb_dim_; ++d) {
                    const size_t i = (size_t)r * cb_dim_ + d;
                    _Float16 h;
                    std::memcpy(&h, src + i, 2);
                    const _Float16 o = (_Float16)((float)h * inv);   // round to nearest even
                    std::memcpy(&w[i], &o, 2);
                }
            }
        }
        dst = up16(w.data(), (size_t)t->nelements());
        ++n_usage_;
        return dst != nullptr;
    };
    const GgufTensor *cb = T("tok_dec.vq_first.0.codebook");
    if (!cb) return false;
    cb_dim_ = (int)cb->ne[0];
    cb_size_ = (int)cb->ne[1];
    if (!codebook("tok_dec.vq_first.0.codebook", "tok_dec.vq_first.0.usage", cb_first_)) return false;
    for (int i = 0; i < 15; ++i) {
        const std::string pre = "tok_dec.vq_rest." + std::to_string(i) + ".";
        if (!codebook(pre + "codebook", pre + "usage", cb_rest_[i])) return false;
    }
    int r, c;
    if (!(vq_first_out_ = mat("tok_dec.vq_first.output_proj.weight", r, c))) return false;
    hidden_ = r;
    if (c != cb_dim_) { set_error("vq output_proj shape"); return false; }
    if (!(vq_rest_out_ = mat("tok_dec.vq_rest.output_proj.weight", r, c))) return false;
    if (!conv_w("tok_dec.pre_conv.weight", pre_conv_)) return false;
    if (!(pre_conv_.b = vec("tok_dec.pre_conv.bias", pre_conv_.oc))) return false;
    latent_ = pre_conv_.oc;
    if (!(in_proj_ = mat("tok_dec.pre_tfm.input_proj.weight", r, c))) return false;
    if (!(in_proj_b_ = vec("tok_dec.pre_tfm.input_proj.bias", hidden_))) return false;
    n_heads_ = (int)g.get_int({"qwen3-tts-tokenizer.decoder.num_heads"}, 16);   // reference default 16
    head_dim_ = latent_ / n_heads_;
    for (int i = 0;; ++i) {
        const std::string p = "tok_dec.pre_tfm.blk." + std::to_string(i) + ".";
        if (!g.find(p + "attn_q.weight")) break;
        Layer L;
        std::vector<uint16_t> qkv;
        size_t n_qkv = 0;
        for (const char *nm : {"attn_q.weight", "attn_k.weight", "attn_v.weight"}) {
            const GgufTensor *t = T(p + nm);
            if (!t || t->ne[0] != hidden_ || t->ne[1] != latent_) { set_error("bad pre_tfm qkv"); return false; }
            if (!recv) qkv.insert(qkv.end(), f16p(t), f16p(t) + t->nelements());
            n_qkv += (size_t)t->nelements();
        }
        L.qkv = up16(qkv.data(), n_qkv);
        const GgufTensor *gt = T(p + "ffn_gate.weight"), *ut = T(p + "ffn_up.weight");
        if (!gt || !ut) return false;
        ffn_ = (int)gt->ne[1];
        if (ffn_ % 16) { set_error("pre_tfm ffn % 16"); return false; }
        const size_t n_gu = (size_t)2 * ffn_ * hidden_;
        std::vector<uint16_t> gu(recv ? 0 : n_gu);
        if (!recv)
            for (int blk = 0; blk < ffn_ / 16; ++blk) {
                std::memcpy(gu.data() + (size_t)(blk * 32) * hidden_, f16p(gt) + (size_t)(blk * 16) * hidden_, (size_t)16 * hidden_ * 2);
                std::memcpy(gu.data() + (size_t)(blk * 32 + 16) * hidden_, f16p(ut) + (size_t)(blk * 16) * hidden_, (size_t)16 * hidden_ * 2);
            }
        L.gu = up16(gu.data(), n_gu);
        if (!(L.o = mat(p + "attn_output.weight", r, c))) return false;
        if (!(L.down = mat(p + "ffn_down.weight", r, c))) return false;
        if (!(L.attn_norm = vec(p + "attn_norm.weight", hidden_)) || !(L.ffn_norm = vec(p + "ffn_norm.weight", hidden_)) ||
            !(L.attn_scale = vec(p + "attn_scale", hidden_)) || !(L.ffn_scale = vec(p + "ffn_scale", hidden_)))
            return false;
        layers_.push_back(L);
    }
    if (!(pre_norm_ = vec("tok_dec.pre_tfm.norm.weight", hidden_))) return false;
    if (!(out_proj_ = mat("tok_dec.pre_tfm.output_proj.weight", r, c))) return false;
    if (!(out_proj_b_ = vec("tok_dec.pre_tfm.output_proj.bias", latent_))) return false;
    for (int u = 0; u < 2; ++u) {
        const std::string p = "tok_dec.upsample." + std::to_string(u) + ".";
        Up &U = up_[u];
        if (!convT_w(p + "conv.weight", U.ct)) return false;
        if (!(U.ct.b = vec(p + "conv.bias", U.ct.oc))) return false;
        const GgufTensor *dw = T(p + "dwconv.weight");
        if (!dw || dw->ne[1] != 1) { set_error("bad dwconv"); return false; }
        U.dw_k = (int)dw->ne[0];
        U.dw = up16(dw->data, (size_t)dw->nelements());
        if (!(U.dw_b = vec(p + "dwconv.bias", U.ct.oc)) || !(U.norm_w = vec(p + "norm.weight", U.ct.oc)) ||
            !(U.norm_b = vec(p + "norm.bias", U.ct.oc)) || !(U.gamma = vec(p + "gamma", U.ct.oc)))
            return false;
        if (!(U.pw1 = mat(p + "pwconv1.weight", U.pw_dim, c))) return false;
        if (!(U.pw1_b = vec(p + "pwconv1.bias", U.pw_dim))) return false;
        if (!(U.pw2 = mat(p + "pwconv2.weight", r, c))) return false;
        if (!(U.pw2_b = vec(p + "pwconv2.bias", U.ct.oc))) return false;
    }
    if (!conv_w("tok_dec.dec.0.conv.weight", dec0_)) return false;
    if (!(dec0_.b = vec("tok_dec.dec.0.conv.bias", dec0_.oc))) return false;
    const int rates[4] = {8, 5, 4, 3};   // audio_tokenizer_decoder.cpp:766
    for (int d = 0; d < 4; ++d) {
        const std::string p = "tok_dec.dec." + std::to_string(d + 1) + ".";
        Dec &D = dec_[d];
        D.rate = rates[d];
        if (!snake(p + "snake.alpha", p + "snake.beta", D.snake)) return false;
        if (!convT_w(p + "conv_t.weight", D.ct)) return false;
        if (!(D.ct.b = vec(p + "conv_t.bias", D.ct.oc))) return false;
        if (D.ct.k > 2 * D.rate || D.ct.k < D.rate) { set_error("unsupported conv_t kernel size"); return false; }
        for (int ri = 0; ri < 3; ++ri) {
            const std::string q = p + "res." + std::to_string(ri + 2) + ".";
            Res &R = D.res[ri];
            R.dil = ri == 0 ? 1 : ri == 1 ? 3 : 9;   // :324-328
            if (!snake(q + "act1.alpha", q + "act1.beta", R.a1) || !snake(q + "act2.alpha", q + "act2.beta", R.a2)) return false;
            if (!conv_w(q + "conv1.weight", R.c1) || !conv_w(q + "conv2.weight", R.c2)) return false;
            if (!(R.c1.b = vec(q + "conv1.bias", R.c1.oc)) || !(R.c2.b = vec(q + "conv2.bias", R.c2.oc))) return false;
        }
    }
    if (!snake("tok_dec.dec.5.snake.alpha", "tok_dec.dec.5.snake.beta", dec5_)) return false;
    if (!conv_w("tok_dec.dec.6.conv.weight", dec6_)) return false;
    if (!(dec6_.b = vec("tok_dec.dec.6.conv.bias", dec6_.oc))) return false;
    if (head_dim_ != 64) { set_error("vocoder head_dim must be 64"); return false; }
    loaded_ = true;
    return true;
}

int64_t Vocoder::full_len(int F) const {
    if (F <= 0) return 0;
    int64_t T = F;
    for (int u = 0; u < 2; ++u) T = (T - 1) * 2 + up_[u].ct.k;
    for (int d = 0; d < 4; ++d) { const int s = dec_[d].rate, K = dec_[d].ct.k; T = (T - 1) * s + K - 2 * (K - s); }
    return T;
}
double Vocoder::decode_flops(int F) const {
    if (F <= 0 || !loaded_) return 0.0;
    const double f = F, VH = hidden_, LAT = latent_;
    auto conv = [](double T_out, const Conv &c) { return 2.0 * T_out * c.ic * c.oc * c.k; };
    double fl = 16.0 * 2.0 * f * cb_dim_ * VH;                 // RVQ output projections
    fl += conv(f, pre_conv_) + 2.0 * f * LAT * VH;             // pre-conv, input_proj
    for (size_t l = 0; l < layers_.size(); ++l)
        fl += 2.0 * f * VH * 3 * LAT + 2.0 * 2.0 * (f * (f + 1) / 2) * LAT + 2.0 * f * LAT * VH +
              2.0 * f * VH * 2 * ffn_ + 2.0 * f * ffn_ * VH;
    fl += 2.0 * f * VH * LAT;                                  // output_proj
    double T = f;
    for (int u = 0; u < 2; ++u) {
        const double T1 = (T - 1) * 2 + up_[u].ct.k;
        fl += conv(T, up_[u].ct) + 2.0 * T1 * LAT * up_[u].dw_k + 2.0 * 2.0 * T1 * LAT * up_[u].pw_dim;
        T = T1;
    }
    fl += conv(T, dec0_);
    for (int d = 0; d < 4; ++d) {
        const Dec &D = dec_[d];
        const double T2 = (T - 1) * D.rate + D.ct.k - 2 * (D.ct.k - D.rate);
        fl += conv(T, D.ct);   // every input row meets every tap once (before trimming)
        for (int r = 0; r < 3; ++r) fl += conv(T2, D.res[r].c1) + conv(T2, D.res[r].c2);
        T = T2;
    }
    return fl + conv(T, dec6_);
}

int64_t Vocoder::n_samples(int n_frames, int mode) const {
    if (n_frames <= 0) return 0;
    return mode == 0 ? full_len(n_frames) : (int64_t)n_frames * 1920;
}

// scratch for nb utterances of F frames: sized by the totals (largest activation x nb, frames x nb), so a batch of
// short utterances reuses the scratch of one long one
bool Vocoder::ensure(int F, int nb) {
    size_t big = 0;   // largest [T][C] activation of one utterance over the stages
    int64_t T = F;
    big = std::max(big, (size_t)F * std::max(latent_, 3 * latent_));
    for (int u = 0; u < 2; ++u) { T = (T - 1) * 2 + up_[u].ct.k; big = std::max(big, (size_t)T * up_[u].pw_dim / 2 + (size_t)T * latent_); }
    big = std::max(big, (size_t)T * dec0_.oc);
    for (int d = 0; d < 4; ++d) {
        const int s = dec_[d].rate, K = dec_[d].ct.k;
        T = (T - 1) * s + K - 2 * (K - s);
        big = std::max(big, (size_t)T * dec_[d].ct.oc);
    }
    big *= (size_t)nb;
    const size_t frames = (size_t)F * nb;
    const size_t pcm = (size_t)nb * std::max<int64_t>(full_len(F), (int64_t)F * 1920);
    if (big <= cap_big_ && frames <= cap_ftot_ && pcm <= cap_pcm_ && F <= cap_frames_) return true;
    big = std::max(big, cap_big_);
    const size_t fr = std::max(frames, cap_ftot_), pc = std::max(pcm, cap_pcm_);
    F = std::max(F, cap_frames_);
    for (void *p : scratch_) hipFree(p);
    scratch_.clear();
    cap_big_ = cap_ftot_ = cap_pcm_ = 0;
    cap_frames_ = 0;
    auto alloc = [&](size_t bytes) -> void * {
        void *p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        scratch_.push_back(p);
        return p;
    };
    for (int i = 0; i < 3; ++i) if (!(buf_[i] = (float *)alloc(big * 4))) { set_error("vocoder scratch alloc"); return false; }
    if (!(xh_ = (uint16_t *)alloc(big * 2)) || !(xh2_ = (uint16_t *)alloc(big * 2))) { set_error("vocoder scratch alloc"); return false; }
    codes_ = (int32_t *)alloc(fr * 16 * 4);
    cols_ = (int *)alloc(fr * 16 * 4);
    pcm_ = (float *)alloc(pc * 4);
    // RoPE cos/sin table (theta 1e4, head_dim 64) with the ggml_rope_cache_init recurrence
    std::vector<float> rope((size_t)F * head_dim_);
    const float theta_scale = powf(10000.0f, -2.0f / (float)head_dim_);
    for (int p = 0; p < F; ++p) {
        float theta = (float)p;
        for (int i0 = 0; i0 < head_dim_; i0 += 2) {
            rope[(size_t)p * head_dim_ + i0] = cosf(theta);
            rope[(size_t)p * head_dim_ + i0 + 1] = sinf(theta);
            theta *= theta_scale;
        }
    }
    rope_ = (float *)alloc(rope.size() * 4);
    if (!codes_ || !cols_ || !pcm_ || !rope_) { set_error("vocoder scratch alloc"); return false; }
    Q3T_HIP(hipMemcpy(rope_, rope.data(), rope.size() * 4, hipMemcpyHostToDevice));
    cap_big_ = big; cap_ftot_ = fr; cap_pcm_ = pc;
    cap_frames_ = F;
    return true;
}

// causal conv (ggml_pad_ext left + ggml_conv_1d, stride 1) as one implicit-GEMM launch
bool Vocoder::run_conv(const Conv &c, const float *x, int T, int pad, int dil, const Snake *sn, float *y,
                       const float *resid, int act, hipStream_t s) {
    ConvParams p;
    p.x = x; p.T_in = T; p.C_in = c.ic;
    if (c.ic % 8 == 0) {   // SnakeBeta + f16 rounding once per element, not once per output tile and tap window
        if (!snake_f16(x, sn ? sn->a : nullptr, sn ? sn->ib : nullptr, xh_, (int64_t)T * nb_, c.ic, s)) return false;
        p.xh = xh_;
    } else if (sn) {
        p.snake_a = sn->a; p.snake_ib = sn->ib;
    }
    p.n_taps = c.k;
    for (int j = 0; j < c.k; ++j) p.taps[j] = ConvTap{c.w + (size_t)j * c.oc * c.ic, j * dil - pad};
    p.dmin = -pad; p.dmax = (c.k - 1) * dil - pad;
    p.y = y; p.C_out = c.oc; p.M = T + pad - dil * (c.k - 1); p.so = 1; p.ob = 0;
    p.bias = c.b; p.resid = resid; p.act = act;
    p.nb = nb_; p.xbs = T; p.ybs = p.M;
    return conv(p, s);
}

// ggml_conv_transpose_1d (stride st, no padding) followed by trimming `trim` samples on both sides, + bias,
// decomposed into st output phases: output t = st*m + phi gathers taps k = k0 + j*st with input row m + dj.
bool Vocoder::run_convT(const Conv &c, const float *x, int T, int st, int trim, const Snake *sn, float *y, int T_out,
                        hipStream_t s) {
    const bool pre = c.ic % 8 == 0;   // one snake/f16 pass shared by the st output phases
    if (pre && !snake_f16(x, sn ? sn->a : nullptr, sn ? sn->ib : nullptr, xh_, (int64_t)T * nb_, c.ic, s)) return false;
    for (int phi = 0; phi < st; ++phi) {
        ConvParams p;
        p.x = x; p.T_in = T; p.C_in = c.ic;
        if (pre) p.xh = xh_;
        else if (sn) { p.snake_a = sn->a; p.snake_ib = sn->ib; }
        const int k0 = (phi + trim) % st;
        int n = 0, dmin = 1 << 30, dmax = -(1 << 30);
        for (int k = k0; k < c.k; k += st) {
            const int dj = (phi + trim - k) / st;   // exact: (phi + trim - k) divisible by st
            p.taps[n++] = ConvTap{c.w + (size_t)k * c.oc * c.ic, dj};
            dmin = std::min(dmin, dj);
            dmax = std::max(dmax, dj);
        }
        if (n == 0) continue;
        p.n_taps = n; p.dmin = dmin; p.dmax = dmax;
        p.y = y; p.C_out = c.oc; p.M = (T_out - phi + st - 1) / st; p.so = st; p.ob = phi;
        p.bias = c.b;
        p.nb = nb_; p.xbs = T; p.ybs = T_out;
        if (!conv(p, s)) return false;
    }
    return true;
}

bool Vocoder::conv16(const Conv &c, const uint16_t *xh, int T, int pad, int dil, float *y, const float *resid,
                     uint16_t *y16, const Snake *next, hipStream_t s) {
    ConvParams p;
    p.xh = xh; p.T_in = T; p.C_in = c.ic;
    p.n_taps = c.k;
    for (int j = 0; j < c.k; ++j) p.taps[j] = ConvTap{c.w + (size_t)j * c.oc * c.ic, j * dil - pad};
    p.dmin = -pad; p.dmax = (c.k - 1) * dil - pad;
    p.y = y; p.C_out = c.oc; p.M = T + pad - dil * (c.k - 1); p.so = 1; p.ob = 0;
    p.bias = c.b; p.resid = resid;
    p.y16 = y16;
    if (next) { p.y16_a = next->a; p.y16_ib = next->ib; }
    p.nb = nb_; p.xbs = T; p.ybs = p.M;
    return conv(p, s);
}

bool Vocoder::convT16(const Conv &c, const uint16_t *xh, int T, int st, int trim, float *y, int T_out, uint16_t *y16,
                      const Snake *next, hipStream_t s) {
    if (c.ic % 32 == 0 && (c.oc % 96 == 0 || c.oc % 64 == 0) && c.k <= st * CONV_MAX_TAPS) {
        // every output phase in one launch (grid z)
        ConvParams p;
        p.xh = xh; p.T_in = T; p.C_in = c.ic;
        p.ct_w = c.w; p.ct_k = c.k; p.ct_st = st; p.ct_trim = trim; p.T_out = T_out;
        p.y = y; p.C_out = c.oc; p.bias = c.b; p.y16 = y16;
        if (next) { p.y16_a = next->a; p.y16_ib = next->ib; }
        p.nb = nb_; p.xbs = T; p.ybs = T_out;
        return conv(p, s);
    }
    for (int phi = 0; phi < st; ++phi) {
        ConvParams p;
        p.xh = xh; p.T_in = T; p.C_in = c.ic;
        const int k0 = (phi + trim) % st;
        int n = 0, dmin = 1 << 30, dmax = -(1 << 30);
        for (int k = k0; k < c.k; k += st) {
            const int dj = (phi + trim - k) / st;
            p.taps[n++] = ConvTap{c.w + (size_t)k * c.oc * c.ic, dj};
            dmin = std::min(dmin, dj);
            dmax = std::max(dmax, dj);
        }
        if (n == 0) continue;
        p.n_taps = n; p.dmin = dmin; p.dmax = dmax;
        p.y = y; p.C_out = c.oc; p.M = (T_out - phi + st - 1) / st; p.so = st; p.ob = phi;
        p.bias = c.b;
        p.y16 = y16;
        if (next) { p.y16_a = next->a; p.y16_ib = next->ib; }
        p.nb = nb_; p.xbs = T; p.ybs = T_out;
        if (!conv(p, s)) return false;
    }
    return true;
}

bool Vocoder::decode_device(const int32_t *codes_dev, int F, float *pcm_dev, int64_t *n_out, hipStream_t s, int nb) {
    if (nb < 1 || F > cap_frames_ || (size_t)F * nb > cap_ftot_) { set_error("vocoder: decode larger than ensure()"); return false; }
    nb_ = nb;
    const bool ok = decode_rows(codes_dev, F, pcm_dev, n_out, s);
    nb_ = 1;
    return ok;
}

// the row GEMVs of a decode: kernel family and K split pinned to one batch size, so a row's arithmetic does not depend
// on how many frame rows the launch covers (an utterance decoded alone, or padded into a batch, gives the same bits)
static GemvParams row_gemv() {
    GemvParams g;
    g.family_b = 64;
    return g;
}

// one decode of nb_ utterances of F frames: row-wise stages (RVQ, projections, norms, 1-tap convs) run over all
// nb_*F rows, sequence stages (causal convs, transposed convs, attention) carry the utterance as grid z
bool Vocoder::decode_rows(const int32_t *codes_dev, int F, float *pcm_dev, int64_t *n_out, hipStream_t s) {
    const int VH = hidden_, LAT = latent_;
    const int FR = F * nb_;   // frame rows of the batch
    float *A = buf_[0], *B = buf_[1], *C = buf_[2];
    // 1) RVQ: latent = W_first . cb_first[c0] + sum_k W_rest . cb_rest_k[c_{k+1}]   (:650-703)
    if (!codes_cols(codes_dev, cols_, FR, 16, s)) return false;
    GemvParams g = row_gemv();
    g.N = VH; g.K = cb_dim_; g.B = FR; g.pro = PRO_F16; g.ldx = cb_dim_; g.ldo = VH;
    for (int k = 0; k < 15; ++k) {
        g.W = vq_rest_out_; g.x = cb_rest_[k]; g.x_idx = cols_ + (size_t)(k + 1) * FR;
        g.resid = k == 0 ? nullptr : B; g.ldr = VH; g.out_f32 = B;
        if (!gemv(g, s)) return false;
    }
    g.W = vq_first_out_; g.x = cb_first_; g.x_idx = cols_; g.resid = nullptr; g.aux = B; g.lda = VH; g.out_f32 = A;
    if (!gemv(g, s)) return false;
    // 2) causal pre-conv k3 (left pad 2) -> [F][LAT]   (:705-718)
    if (!run_conv(pre_conv_, A, F, 2, 1, nullptr, C, nullptr, 0, s)) return false;
    // 3) input_proj + bias -> x [F][VH]
    GemvParams ip = row_gemv();
    ip.W = in_proj_; ip.N = VH; ip.K = LAT; ip.B = FR; ip.pro = PRO_F32; ip.x = C; ip.ldx = LAT;
    ip.bias = in_proj_b_; ip.out_f32 = A; ip.ldo = VH;
    if (!gemv(ip, s)) return false;
    float *x = A;
    float *qkv = B;                                        // [F][3*LAT]
    uint16_t *att = reinterpret_cast<uint16_t *>(C);       // [F][LAT] f16
    uint16_t *hm = reinterpret_cast<uint16_t *>(C) + (size_t)FR * LAT;   // [F][ffn] f16
    // large-M projections (M = frames or upsampled steps) run as 1-tap convs on the implicit-GEMM conv kernel over
    // pre-normalised f16 rows (norm_f16 reproduces the GEMM prologue's norm); the decode-shaped GEMM path stays for
    // the shapes the conv tiles do not cover
    const bool qkv_conv = VH % 32 == 0 && VH <= 1024 && VH % 4 == 0 && (3 * LAT) % 96 == 0;
    for (const Layer &L : layers_) {
        if (qkv_conv) {
            if (!norm_f16(x, L.attn_norm, nullptr, 1e-5f, 0, xh_, FR, VH, s)) return false;
            ConvParams q;
            q.xh = xh_; q.T_in = FR; q.C_in = VH; q.n_taps = 1; q.taps[0] = ConvTap{L.qkv, 0};
            q.y = qkv; q.C_out = 3 * LAT; q.M = FR;
            if (!conv(q, s)) return false;
        } else {
            GemvParams q = row_gemv();
            q.W = L.qkv; q.N = 3 * LAT; q.K = VH; q.B = FR; q.pro = PRO_RMS; q.x = x; q.ldx = VH; q.nw = L.attn_norm;
            q.eps = 1e-5f; q.out_f32 = qkv; q.ldo = 3 * LAT;
            if (!gemv(q, s)) return false;
        }
        if (!attn_prefill(qkv, rope_, att, F, n_heads_, head_dim_, s, nb_)) return false;
        GemvParams o = row_gemv();
        o.W = L.o; o.N = VH; o.K = LAT; o.B = FR; o.pro = PRO_F16; o.x = att; o.ldx = LAT;
        o.scale = L.attn_scale; o.resid = x; o.ldr = VH; o.out_f32 = x; o.ldo = VH;
        if (!gemv(o, s)) return false;
        GemvParams gu = row_gemv();
        gu.W = L.gu; gu.N = 2 * ffn_; gu.K = VH; gu.B = FR; gu.pro = PRO_RMS; gu.x = x; gu.ldx = VH; gu.nw = L.ffn_norm;
        gu.eps = 1e-5f; gu.act = ACT_SWIGLU; gu.out_f16 = hm; gu.ldo = ffn_;
        if (!gemv(gu, s)) return false;
        GemvParams dn = row_gemv();
        dn.W = L.down; dn.N = VH; dn.K = ffn_; dn.B = FR; dn.pro = PRO_F16; dn.x = hm; dn.ldx = ffn_;
        dn.scale = L.ffn_scale; dn.resid = x; dn.ldr = VH; dn.out_f32 = x; dn.ldo = VH;
        if (!gemv(dn, s)) return false;
    }
    // final RMSNorm + output_proj + bias -> [F][LAT]   (:740-744)
    GemvParams op = row_gemv();
    op.W = out_proj_; op.N = LAT; op.K = VH; op.B = FR; op.pro = PRO_RMS; op.x = x; op.ldx = VH; op.nw = pre_norm_;
    op.eps = 1e-5f; op.bias = out_proj_b_; op.out_f32 = B; op.ldo = LAT;
    if (!gemv(op, s)) return false;
    float *cur = B;
    float *f0 = A, *f1 = C;
    int64_t T = F;
    // 4) ConvNeXt upsample blocks (:490-549)
    for (int u = 0; u < 2; ++u) {
        const Up &U = up_[u];
        const int64_t T1 = (T - 1) * 2 + U.ct.k;
        float *h = f0;                                   // conv-transpose output = residual [T1][LAT]
        if (!run_convT(U.ct, cur, (int)T, 2, 0, nullptr, h, (int)T1, s)) return false;
        float *dwo = f1;                                 // [T1][LAT]
        if (!dwconv(h, U.dw, U.dw_b, dwo, (int)T1, LAT, U.dw_k, s, nb_)) return false;
        uint16_t *pw = reinterpret_cast<uint16_t *>(cur);  // [T1][pw_dim] f16, cur is dead now (ensure() sizes it)
        const bool pw_conv = LAT % 32 == 0 && LAT <= 1024 && U.pw_dim % 64 == 0 && U.pw_dim % 32 == 0 && LAT % 64 == 0;
        if (pw_conv) {
            // LayerNorm -> f16 rows, pw1 + bias + GELU -> f16, pw2 + bias, x gamma, + residual (in place)
            if (!norm_f16(dwo, U.norm_w, U.norm_b, 1e-6f, 1, xh_, (int)T1 * nb_, LAT, s)) return false;
            ConvParams c1;
            c1.xh = xh_; c1.T_in = (int)T1 * nb_; c1.C_in = LAT; c1.n_taps = 1; c1.taps[0] = ConvTap{U.pw1, 0};
            c1.C_out = U.pw_dim; c1.M = (int)T1 * nb_; c1.bias = U.pw1_b; c1.act = 4; c1.y16 = pw;
            if (!conv(c1, s)) return false;
            ConvParams c2;
            c2.xh = pw; c2.T_in = (int)T1 * nb_; c2.C_in = U.pw_dim; c2.n_taps = 1; c2.taps[0] = ConvTap{U.pw2, 0};
            c2.C_out = LAT; c2.M = (int)T1 * nb_; c2.bias = U.pw2_b; c2.scale = U.gamma; c2.resid = h; c2.y = h;
            if (!conv(c2, s)) return false;
        } else {
            GemvParams p1 = row_gemv();
            p1.W = U.pw1; p1.N = U.pw_dim; p1.K = LAT; p1.B = (int)T1 * nb_; p1.pro = PRO_LN; p1.x = dwo; p1.ldx = LAT;
            p1.nw = U.norm_w; p1.nb = U.norm_b; p1.eps = 1e-6f; p1.bias = U.pw1_b; p1.act = ACT_GELU;
            p1.out_f16 = pw; p1.ldo = U.pw_dim;
            if (!gemv(p1, s)) return false;
            GemvParams p2 = row_gemv();
            p2.W = U.pw2; p2.N = LAT; p2.K = U.pw_dim; p2.B = (int)T1 * nb_; p2.pro = PRO_F16; p2.x = pw; p2.ldx = U.pw_dim;
            p2.bias = U.pw2_b; p2.scale = U.gamma; p2.resid = h; p2.ldr = LAT; p2.out_f32 = h; p2.ldo = LAT;
            if (!gemv(p2, s)) return false;
        }
        float *nxt = h;
        f0 = cur; cur = nxt; T = T1;
    }
    // 5) dec0 conv k7 (left pad 6) -> [T][dec_dim]   (:759-763).  From here on every conv input is the f16
    // SnakeBeta of its predecessor's output, written by that conv's epilogue (snake + rounding once per element,
    // the f32 tensor itself only where a residual needs it): ha / hb ping-pong
    uint16_t *ha = xh_, *hb = xh2_;
    if (!snake_f16(cur, nullptr, nullptr, ha, T * nb_, dec0_.ic, s)) return false;
    if (!conv16(dec0_, ha, (int)T, 6, 1, nullptr, nullptr, hb, &dec_[0].snake, s)) return false;   // snake(dec0) only
    std::swap(ha, hb);
    // 6) decoder blocks: SnakeBeta -> conv-transpose (trim K-s both sides) + bias -> 3 residual units (:551-620)
    for (int d = 0; d < 4; ++d) {
        const Dec &D = dec_[d];
        const int st = D.rate, K = D.ct.k;
        const int64_t T2 = (T - 1) * st + K - 2 * (K - st);
        // x = convT(snake(x)): f32 residual stream + f16 snake1 of residual unit 0
        if (!convT16(D.ct, ha, (int)T, st, K - st, f0, (int)T2, hb, &D.res[0].a1, s)) return false;
        std::swap(ha, hb);
        std::swap(cur, f0);
        T = T2;
        for (int ri = 0; ri < 3; ++ri) {
            const Res &R = D.res[ri];
            const Snake *next = ri < 2 ? &D.res[ri + 1].a1 : d < 3 ? &dec_[d + 1].snake : &dec5_;
            // the last unit of the last block feeds only the output conv's f16 input: no f32 residual stream out
            float *xout = d == 3 && ri == 2 ? nullptr : cur;
            if (fuse_res_ && R.c1.ic == 96 && R.c1.oc == 96 && R.c1.k == 7 && R.c2.ic == 96 && R.c2.oc == 96 && R.c2.k == 1 &&
                R.dil <= 9 && R.c1.b && R.c2.b) {
                // the whole unit in one launch (vocoder_resunit.hip): h stays on chip, bit-identical to the two convs
                ResUnitParams u;
                u.xh = ha; u.x = cur; u.y = xout; u.y16 = hb; u.T = (int)T; u.dil = R.dil;
                u.w1 = R.c1.w; u.b1 = R.c1.b; u.a2 = R.a2.a; u.ib2 = R.a2.ib;
                u.w2 = R.c2.w; u.b2 = R.c2.b; u.an = next->a; u.ibn = next->ib;
                u.nb = nb_; u.bs = T;
                if (!resunit96(u, s)) return false;
                std::swap(ha, hb);
                continue;
            }
            // h1 = conv1(snake1(x)) with causal pad 6*dil -> only snake2(h1) in f16; x += conv2(snake2(h1)) (f32, in
            // place) plus the next conv's f16 input
            if (!conv16(R.c1, ha, (int)T, 6 * R.dil, R.dil, nullptr, nullptr, hb, &R.a2, s)) return false;
            if (!conv16(R.c2, hb, (int)T, 0, 1, xout, cur, ha, next, s)) return false;
        }
    }
    // 7) SnakeBeta -> conv k7 (pad 6) -> tanh   (:775-790): ha holds f16(snake(dec5)) of the stream
    if (dec6_.oc == 1 && dec6_.ic % 8 == 0 && dec6_.ic <= 104 && dec6_.k <= 8) {
        if (!conv_out1(ha, dec6_.w, dec6_.b, pcm_dev, (int)T, dec6_.ic, dec6_.k, s, nb_)) return false;
        *n_out = T;
        return true;
    }
    ConvParams p6;
    p6.xh = ha; p6.T_in = (int)T; p6.C_in = dec6_.ic;
    p6.n_taps = dec6_.k;
    for (int j = 0; j < dec6_.k; ++j) p6.taps[j] = ConvTap{dec6_.w + (size_t)j * dec6_.oc * dec6_.ic, j - 6};
    p6.dmin = -6; p6.dmax = dec6_.k - 1 - 6;
    p6.y = pcm_dev; p6.C_out = dec6_.oc; p6.M = (int)T + 6 - (dec6_.k - 1); p6.bias = dec6_.b; p6.act = 1;
    p6.nb = nb_; p6.xbs = T; p6.ybs = p6.M;
    if (!conv(p6, s)) return false;
    *n_out = T;
    return true;
}

bool Vocoder::decode(const int32_t *codes, int F, int mode, float *pcm, int64_t *n_out, int chunk_frames) {
    *n_out = n_samples(F, mode);
    if (F <= 0) return true;
    if (mode == 0) {
        if (!ensure(F)) return false;
        Q3T_HIP(hipMemcpyAsync(codes_, codes, (size_t)F * 16 * 4, hipMemcpyHostToDevice, stream_));
        int64_t n = 0;
        if (!decode_device(codes_, F, pcm_, &n, stream_)) return false;
        Q3T_HIP(hipMemcpyAsync(pcm, pcm_, (size_t)n * 4, hipMemcpyDeviceToHost, stream_));
        Q3T_HIP(hipStreamSynchronize(stream_));
        *n_out = n;
        return true;
    }
    // CHUNK40: every chunk of the utterance in shared launches
    return decode_batch(1, &codes, &F, mode, &pcm, n_out, chunk_frames);
}

bool Vocoder::decode_batch(int n_utt, const int32_t *const *codes, const int *n_frames, int mode, float *const *pcm,
                           int64_t *n_out, int chunk_frames) {
    // a sequence = one utterance (FULL) or one chunk_frames-long chunk of one (CHUNK40, trt_vocoder.cpp:98-170:
    // independent fixed-length chunks, zero-padded codes, chunk_frames*1920 samples kept)
    struct Seq { int u, off, nf; };
    std::vector<Seq> seqs;
    if (mode != 0 && chunk_frames <= 0) { set_error("vocoder: chunk_frames must be > 0"); return false; }
    for (int u = 0; u < n_utt; ++u) {
        const int nf = std::max(n_frames[u], 0);
        n_out[u] = n_samples(nf, mode);
        if (mode == 0) {
            if (nf > 0) seqs.push_back({u, 0, nf});
        } else {
            for (int off = 0; off < nf; off += chunk_frames) seqs.push_back({u, off, std::min(chunk_frames, nf - off)});
        }
    }
    // FULL: longest first, so each batch pads its utterances to a similar length (the decoder is causal end to end:
    // frames appended after an utterance change none of its samples)
    if (mode == 0) std::stable_sort(seqs.begin(), seqs.end(), [](const Seq &a, const Seq &b) { return a.nf > b.nf; });
    std::vector<int32_t> hc;
    for (size_t i = 0; i < seqs.size();) {
        const int F = mode == 0 ? seqs[i].nf : chunk_frames;
        const int nb = (int)std::min<size_t>(seqs.size() - i, (size_t)std::max(1, batch_frames_ / F));
        if (!ensure(F, nb)) return false;
        hc.assign((size_t)nb * F * 16, 0);
        for (int j = 0; j < nb; ++j) {
            const Seq &q = seqs[i + j];
            std::memcpy(hc.data() + (size_t)j * F * 16, codes[q.u] + (size_t)q.off * 16, (size_t)q.nf * 16 * 4);
        }
        Q3T_HIP(hipMemcpyAsync(codes_, hc.data(), hc.size() * 4, hipMemcpyHostToDevice, stream_));
        int64_t per = 0;   // samples per sequence of this batch
        if (!decode_device(codes_, F, pcm_, &per, stream_, nb)) return false;
        for (int j = 0; j < nb; ++j) {
            const Seq &q = seqs[i + j];
            const float *src = pcm_ + (size_t)j * per;
            if (mode == 0) {
                Q3T_HIP(hipMemcpyAsync(pcm[q.u], src, (size_t)n_out[q.u] * 4, hipMemcpyDeviceToHost, stream_));
            } else {
                const int64_t want = (int64_t)q.nf * 1920, have = std::min(want, per);
                Q3T_HIP(hipMemcpyAsync(pcm[q.u] + (size_t)q.off * 1920, src, (size_t)have * 4, hipMemcpyDeviceToHost, stream_));
                for (int64_t k = have; k < want; ++k) pcm[q.u][(size_t)q.off * 1920 + k] = 0.0f;
            }
        }
        Q3T_HIP(hipStreamSynchronize(stream_));
        i += nb;
    }
    return true;
}

}  // namespace q3t
