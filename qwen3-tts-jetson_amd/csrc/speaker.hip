// speaker.hip — speaker encoder (ECAPA-TDNN) kernels and host driver; see speaker.h.
// Reference: src/audio_tokenizer_encoder.cpp (mel :281-364, graph :438-694, encode :696-750).
#include "speaker.h"

#include <cmath>
#include <cstring>

namespace q3t {

namespace {
constexpr int NFFT = 1024, HOP = 256, WIN = 1024, NMEL = 128, NBIN = NFFT / 2 + 1, SPK_SR = 24000;
constexpr int HID = 512, BR = 64, MFA = 1536;

// STFT frames: reflect-padded samples ((n_fft - hop) / 2 each side, :285-305) times the centred Hann window
__global__ void k_frames(const float *x, int n, const float *win, float *fr, int F) {
    const int f = blockIdx.x, pad = (NFFT - HOP) / 2;
    for (int i = threadIdx.x; i < NFFT; i += 256) {
        const int j = f * HOP + i;
        int src = j < pad ? pad - j : j >= pad + n ? 2 * n - (j - pad) - 2 : j - pad;
        src = min(max(src, 0), n - 1);
        fr[(size_t)f * NFFT + i] = x[src] * win[i];
    }
}

// C[M][N] = A[M][K] . B[K][N], f32, row-major; 64 x 64 tiles, 256 threads x (4 x 4) outputs, K chunks of 16 in LDS
__global__ void __launch_bounds__(256) k_gemm_f32(const float *A, const float *B, float *C, int M, int N, int K) {
    __shared__ float As[16][64 + 4], Bs[16][64 + 4];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += 16) {
        for (int e = threadIdx.x; e < 16 * 64; e += 256) {
            const int r = e / 16, kk = e % 16;   // A tile row r, column kk
            As[kk][r] = (m0 + r < M && k0 + kk < K) ? A[(size_t)(m0 + r) * K + k0 + kk] : 0.0f;
            const int kb = e / 64, c = e % 64;
            Bs[kb][c] = (k0 + kb < K && n0 + c < N) ? B[(size_t)(k0 + kb) * N + n0 + c] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
            float a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) { a[i] = As[kk][ty * 4 + i]; b[i] = Bs[kk][tx * 4 + i]; }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int m = m0 + ty * 4 + i, c = n0 + tx * 4 + j;
            if (m < M && c < N) C[(size_t)m * N + c] = acc[i][j];
        }
}

// magnitude sqrt(re^2 + im^2 + 1e-9) (:346-348) from interleaved (re, im) columns
__global__ void k_mag(const float *spec, float *mag, int F) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)F * NBIN) return;
    const float re = spec[2 * i], im = spec[2 * i + 1];
    mag[i] = sqrtf(re * re + im * im + 1e-9f);
}
__global__ void k_log_clamp(float *x, size_t n) {   // log(max(x, 1e-5)) (:358-359)
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) x[i] = logf(fmaxf(x[i], 1e-5f));
}

// f16 conv input: out[i][c] = f16(x[r(i)][c] (+ x2[r(i)][c])), r = reflect index over pad rows each side
// (apply_reflect_pad_1d, :366-408)
__global__ void k_pad_f16(const float *x, int ldx, const float *x2, int ldx2, int T, int C, int pad, uint16_t *out) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    const int Tp = T + 2 * pad;
    if (idx >= (size_t)Tp * C) return;
    const int i = (int)(idx / C), c = (int)(idx % C);
    const int t = i < pad ? pad - i : i >= pad + T ? T - 2 - (i - pad - T) : i - pad;
    float v = x[(size_t)t * ldx + c];
    if (x2) v += x2[(size_t)t * ldx2 + c];
    out[idx] = f2h(v);
}

// per-column mean over time, one thread per column, sequential f32 sum (ggml_pool_1d AVG)
__global__ void k_colmean(const float *x, int ld, int T, int C, float *out) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    float s = 0.0f;
    for (int t = 0; t < T; ++t) s += x[(size_t)t * ld + c];
    out[c] = s / (float)T;
}
// per-column mean and clamped std over time (ASP global statistics, :613-622)
__global__ void k_colstats(const float *x, int ld, int T, int C, float *mu, float *sd) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    float s = 0.0f, q = 0.0f;
    for (int t = 0; t < T; ++t) { const float v = x[(size_t)t * ld + c]; s += v; q += v * v; }
    const float m = s / (float)T;
    const float var = fminf(fmaxf(q / (float)T - m * m, 1e-12f), 1e10f);
    mu[c] = m;
    sd[c] = sqrtf(var);
}

// out[o] = act(b[o] + W[o][:] . f16(x)), W [O][I] f16 (a 1x1 conv on one time step); one wave per output.
// act: 0 none, 2 ReLU, 4 sigmoid
__global__ void k_matvec(const uint16_t *W, const float *b, const float *x, int O, int I, int act, float *out) {
    const int o = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (o >= O) return;
    float s = 0.0f;
    for (int i = lane; i < I; i += 64) s += h2f(W[(size_t)o * I + i]) * f16r(x[i]);
    s = wave_sum(s);
    if (lane == 0) {
        float v = s + (b ? b[o] : 0.0f);
        if (act == 2) v = fmaxf(v, 0.0f);
        if (act == 4) v = 1.0f / (1.0f + expf(-v));
        out[o] = v;
    }
}

// SE scale + residual: y[t][c] = y[t][c] * se[c] + res[t][c] (:581-586); y written to out (row stride ldo)
__global__ void k_se_apply(const float *y, const float *se, const float *res, int ldr, float *out, int ldo, int T, int C) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)T * C) return;
    const int t = (int)(idx / C), c = (int)(idx % C);
    out[(size_t)t * ldo + c] = y[idx] * se[c] + res[(size_t)t * ldr + c];
}

// ASP attention input [T][4608] f16: [hs | mean | std] (:628-634)
__global__ void k_att_in(const float *hs, const float *mu, const float *sd, int T, uint16_t *out) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (size_t)T * 3 * MFA) return;
    const int t = (int)(idx / (3 * MFA)), c = (int)(idx % (3 * MFA));
    const float v = c < MFA ? hs[(size_t)t * MFA + c] : c < 2 * MFA ? mu[c - MFA] : sd[c - 2 * MFA];
    out[idx] = f2h(v);
}

// softmax over time of the attention logits a[T][C], then attention-weighted mean / std of hs (:652-673), one thread
// per channel in the reference's sequential order; pooled = [mean | std]
__global__ void k_asp_pool(const float *a, const float *hs, int T, float *pooled) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= MFA) return;
    float mx = -INFINITY;
    for (int t = 0; t < T; ++t) mx = fmaxf(mx, a[(size_t)t * MFA + c]);
    double sum = 0.0;
    for (int t = 0; t < T; ++t) sum += (double)expf(a[(size_t)t * MFA + c] - mx);
    const float inv = (float)(1.0 / sum);
    float wm = 0.0f;
    for (int t = 0; t < T; ++t) wm += (expf(a[(size_t)t * MFA + c] - mx) * inv) * hs[(size_t)t * MFA + c];
    wm = (wm / (float)T) * (float)T;
    float wv = 0.0f;
    for (int t = 0; t < T; ++t) {
        const float d = hs[(size_t)t * MFA + c] - wm;
        wv += (expf(a[(size_t)t * MFA + c] - mx) * inv) * (d * d);
    }
    wv = fminf(fmaxf((wv / (float)T) * (float)T, 1e-12f), 1e10f);
    pooled[c] = wm;
    pooled[MFA + c] = sqrtf(wv);
}

unsigned nblk(size_t n) { return (unsigned)((n + 255) / 256); }
}  // namespace

SpeakerEncoder::~SpeakerEncoder() {
    for (void *p : allocs_) hipFree(p);
    for (void *p : scratch_) hipFree(p);
    if (samples_) hipFree(samples_);
}

template <class T>
T *SpeakerEncoder::dalloc(size_t n) {
    void *p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
    allocs_.push_back(p);
    return static_cast<T *>(p);
}

bool SpeakerEncoder::load(const Gguf &g, WeightArena &wa, hipStream_t s) {
    stream_ = s;
    const bool recv = wa.recv;
    sample_rate_ = (int)g.get_int({"qwen3-tts.speaker_encoder.sample_rate"}, 24000);
    // conv weight ne [K, IC, OC] (PyTorch [oc][ic][k]) -> per-tap [K][OC][IC] (the conv kernels' layout)
    auto conv = [&](const std::string &nm, Conv &c, int ic, int oc, int k) -> bool {
        const GgufTensor *w = g.find("spk_enc." + nm + ".weight"), *b = g.find("spk_enc." + nm + ".bias");
        if (!w || !b || w->type != GGML_TYPE_F16 || b->type != GGML_TYPE_F32 || w->ne[0] != k || w->ne[1] != ic ||
            w->ne[2] != oc || b->nelements() != oc) {
            set_error("speaker encoder: missing or malformed tensor spk_enc." + nm);
            return false;
        }
        c.k = k; c.ic = ic; c.oc = oc;
        const size_t nw = (size_t)k * oc * ic;
        std::vector<uint16_t> t(recv ? 0 : nw);
        if (!recv) {
            const uint16_t *src = static_cast<const uint16_t *>(w->data);
            for (int o = 0; o < oc; ++o)
                for (int i = 0; i < ic; ++i)
                    for (int j = 0; j < k; ++j) t[((size_t)j * oc + o) * ic + i] = src[((size_t)o * ic + i) * k + j];
        }
        if (!(c.w = wa.alloc<uint16_t>(nw)) || !wa.put(c.w, t.data(), nw * 2)) return false;
        if (!(c.b = wa.alloc<float>(oc)) || !wa.put(c.b, b->data, (size_t)oc * 4)) return false;
        return true;
    };
    const GgufTensor *fc = g.find("spk_enc.fc.weight");
    if (!fc) { set_error("No speaker encoder tensors found in model"); return false; }
    dim_ = (int)fc->ne[2];
    if (!conv("conv0", conv0_, NMEL, HID, 5)) return false;
    for (int i = 0; i < 3; ++i) {
        const std::string p = "blk." + std::to_string(i + 1) + ".";
        if (!conv(p + "tdnn1", blk_[i].tdnn1, HID, HID, 1) || !conv(p + "tdnn2", blk_[i].tdnn2, HID, HID, 1) ||
            !conv(p + "se.conv1", blk_[i].se1, HID, 128, 1) || !conv(p + "se.conv2", blk_[i].se2, 128, HID, 1))
            return false;
        for (int r = 0; r < 7; ++r)
            if (!conv(p + "res2net." + std::to_string(r), blk_[i].res[r], BR, BR, 3)) return false;
    }
    if (!conv("mfa", mfa_, MFA, MFA, 1) || !conv("asp.tdnn", asp_tdnn_, 3 * MFA, 128, 1) ||
        !conv("asp.conv", asp_conv_, 128, MFA, 1) || !conv("fc", fc_, 2 * MFA, dim_, 1))
        return false;
    if (wa.plan) return true;   // host-only layout: the arena part is all a plan records
    // front-end constants with the reference's own expressions (computed per rank, outside the weight blob)
    std::vector<float> basis((size_t)NFFT * 2 * NBIN), win(NFFT, 0.0f), fbT((size_t)NBIN * NMEL, 0.0f);
    for (int k = 0; k < NBIN; ++k)
        for (int t = 0; t < NFFT; ++t) {
            const float angle = -2.0f * M_PI * k * t / NFFT;   // compute_dft, :101
            basis[(size_t)t * 2 * NBIN + 2 * k] = cosf(angle);
            basis[(size_t)t * 2 * NBIN + 2 * k + 1] = sinf(angle);
        }
    const int off = (NFFT - WIN) / 2;   // compute_centered_window, :109-118
    for (int i = 0; i < WIN; ++i) win[off + i] = 0.5f * (1.0f - cosf(2.0f * M_PI * i / WIN));
    {   // compute_mel_filterbank_slaney (:16-94), stored transposed [bin][mel] for the GEMM
        const float f_sp = 200.0f / 3.0f, min_log_hz = 1000.0f, min_log_mel = (min_log_hz - 0.0f) / f_sp;
        const float logstep = logf(6.4f) / 27.0f;
        auto hz2mel = [&](float hz) { return hz < min_log_hz ? (hz - 0.0f) / f_sp : min_log_mel + logf(hz / min_log_hz) / logstep; };
        auto mel2hz = [&](float m) { return m < min_log_mel ? 0.0f + f_sp * m : min_log_hz * expf(logstep * (m - min_log_mel)); };
        const float mel_min = hz2mel(0.0f), mel_max = hz2mel(12000.0f);
        std::vector<float> hz(NMEL + 2);
        for (int i = 0; i < NMEL + 2; ++i) hz[i] = mel2hz(mel_min + (mel_max - mel_min) * i / (NMEL + 1));
        for (int m = 0; m < NMEL; ++m) {
            const float fl = hz[m], fc = hz[m + 1], fr = hz[m + 2], enorm = 2.0f / (fr - fl);
            for (int k = 0; k < NBIN; ++k) {
                const float freq = (float)k * SPK_SR / NFFT;
                float v = 0.0f;
                if (freq >= fl && freq <= fc) { if (fc > fl) v = enorm * (freq - fl) / (fc - fl); }
                else if (freq > fc && freq <= fr) { if (fr > fc) v = enorm * (fr - freq) / (fr - fc); }
                fbT[(size_t)k * NMEL + m] = v;
            }
        }
    }
    if (!(basis_ = dalloc<float>(basis.size())) || !(win_ = dalloc<float>(NFFT)) || !(fb_ = dalloc<float>(fbT.size()))) {
        set_error("speaker encoder: device allocation failed");
        return false;
    }
    Q3T_HIP(hipMemcpy(basis_, basis.data(), basis.size() * 4, hipMemcpyHostToDevice));
    Q3T_HIP(hipMemcpy(win_, win.data(), NFFT * 4, hipMemcpyHostToDevice));
    Q3T_HIP(hipMemcpy(fb_, fbT.data(), fbT.size() * 4, hipMemcpyHostToDevice));
    loaded_ = true;
    return true;
}

bool SpeakerEncoder::ensure(int T) {
    if (T <= cap_T_) return true;
    for (void *p : scratch_) hipFree(p);
    scratch_.clear();
    auto alloc = [&](size_t bytes) -> void * {
        void *p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        scratch_.push_back(p);
        return p;
    };
    const size_t Tz = (size_t)T + 32;
    frames_ = (float *)alloc(Tz * NFFT * 4);
    spec_ = (float *)alloc(Tz * 2 * NBIN * 4);
    mag_ = (float *)alloc(Tz * NBIN * 4);
    mel_ = (float *)alloc(Tz * NMEL * 4);
    x0_ = (float *)alloc(Tz * HID * 4);
    h_ = (float *)alloc(Tz * HID * 4);
    cat_ = (float *)alloc(Tz * HID * 4);
    y_ = (float *)alloc(Tz * HID * 4);
    blocks_ = (float *)alloc(Tz * MFA * 4);
    mfa_out_ = (float *)alloc(Tz * MFA * 4);
    att_ = (float *)alloc(Tz * 128 * 4);
    att2_ = (float *)alloc(Tz * MFA * 4);
    vec_ = (float *)alloc((size_t)8 * 4096 * 4);
    xh_ = (uint16_t *)alloc(Tz * 3 * MFA * 2 + (size_t)64 * HID * 2);
    if (!frames_ || !spec_ || !mag_ || !mel_ || !x0_ || !h_ || !cat_ || !y_ || !blocks_ || !mfa_out_ || !att_ || !att2_ ||
        !vec_ || !xh_) {
        set_error("speaker encoder: scratch allocation failed");
        return false;
    }
    cap_T_ = T;
    return true;
}

bool SpeakerEncoder::upload(const float *samples, int n) {
    if (n > cap_n_) {
        if (samples_) hipFree(samples_);
        samples_ = nullptr;
        cap_n_ = 0;
        Q3T_HIP(hipMalloc((void **)&samples_, (size_t)n * 4));
        cap_n_ = n;
    }
    Q3T_HIP(hipMemcpyAsync(samples_, samples, (size_t)n * 4, hipMemcpyHostToDevice, stream_));
    return true;
}

bool SpeakerEncoder::conv(const Conv &c, const float *x, int ldx, const float *x2, int ldx2, int T, int pad, int dil,
                          float *y, int ldy, int act) {
    const int Tp = T + 2 * pad;
    hipLaunchKernelGGL(k_pad_f16, dim3(nblk((size_t)Tp * c.ic)), dim3(256), 0, stream_, x, ldx, x2, ldx2, T, c.ic, pad, xh_);
    Q3T_HIP(hipGetLastError());
    ConvParams p;
    p.xh = xh_; p.T_in = Tp; p.C_in = c.ic;
    p.n_taps = c.k;
    for (int j = 0; j < c.k; ++j) p.taps[j] = ConvTap{c.w + (size_t)j * c.oc * c.ic, j * dil};
    p.dmin = 0; p.dmax = (c.k - 1) * dil;
    p.y = y; p.ldy = ldy; p.C_out = c.oc; p.M = T; p.bias = c.b; p.act = act;
    return q3t::conv(p, stream_);
}

bool SpeakerEncoder::run_mel(const float *x, int n, int F) {
    hipLaunchKernelGGL(k_frames, dim3(F), dim3(256), 0, stream_, x, n, win_, frames_, F);
    Q3T_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_gemm_f32, dim3((2 * NBIN + 63) / 64, (F + 63) / 64), dim3(256), 0, stream_, frames_, basis_, spec_,
                       F, 2 * NBIN, NFFT);
    Q3T_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_mag, dim3(nblk((size_t)F * NBIN)), dim3(256), 0, stream_, spec_, mag_, F);
    Q3T_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_gemm_f32, dim3((NMEL + 63) / 64, (F + 63) / 64), dim3(256), 0, stream_, mag_, fb_, mel_, F, NMEL, NBIN);
    Q3T_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_log_clamp, dim3(nblk((size_t)F * NMEL)), dim3(256), 0, stream_, mel_, (size_t)F * NMEL);
    Q3T_HIP(hipGetLastError());
    return true;
}

static int n_frames_of(int n) {
    const int pad = (NFFT - HOP) / 2, plen = n + 2 * pad;
    return n < 2 ? 0 : (plen - NFFT) / HOP + 1;
}

bool SpeakerEncoder::mel(const float *samples, int n, std::vector<float> &out, int *n_frames) {
    const int F = n_frames_of(n);
    if (!loaded_) { set_error("speaker encoder not loaded"); return false; }
    if (F <= 0) { set_error("Audio too short for mel spectrogram"); return false; }
    if (!ensure(F) || !upload(samples, n)) return false;
    const bool ok = run_mel(samples_, n, F);
    out.resize((size_t)F * NMEL);
    if (ok) Q3T_HIP(hipMemcpyAsync(out.data(), mel_, out.size() * 4, hipMemcpyDeviceToHost, stream_));
    Q3T_HIP(hipStreamSynchronize(stream_));
    *n_frames = F;
    return ok;
}

bool SpeakerEncoder::encode(const float *samples, int n, float *emb) {
    if (!loaded_) { set_error("Model not loaded"); return false; }
    const int T = n_frames_of(n);
    if (T <= 0) { set_error("Audio too short for mel spectrogram"); return false; }
    if (T < 5) { set_error("Audio too short for the speaker encoder"); return false; }   // reflect pads need T > pad
    if (!ensure(T) || !upload(samples, n)) return false;
    bool ok = run_mel(samples_, n, T);
    // conv0 k5 (reflect 2) + ReLU -> x0 [T][512]   (:463-478)
    ok = ok && conv(conv0_, mel_, NMEL, nullptr, 0, T, 2, 1, x0_, HID, 2);
    const int dils[3] = {2, 3, 4};
    for (int b = 0; b < 3 && ok; ++b) {
        const Blk &B = blk_[b];
        const float *res = b == 0 ? x0_ : blocks_ + (size_t)(b - 1) * HID;   // block input (residual)
        const int ldres = b == 0 ? HID : MFA;
        ok = ok && conv(B.tdnn1, res, ldres, nullptr, 0, T, 0, 1, h_, HID, 2);                       // tdnn1 + ReLU
        // Res2Net: branch 0 identity; branch j = conv_j(h_j (+ out_{j-1})) + ReLU, k3 dilation d, reflect d (:508-547)
        for (int j = 1; j < 8 && ok; ++j) {
            const float *prev = j >= 2 ? cat_ + (size_t)(j - 1) * BR : nullptr;
            ok = ok && conv(B.res[j - 1], h_ + (size_t)j * BR, HID, prev, HID, T, dils[b], dils[b], cat_ + (size_t)j * BR, HID, 2);
        }
        // branch 0 copied into the concatenation: cat[:, 0:64] = h[:, 0:64]
        if (ok && hipMemcpy2DAsync(cat_, HID * 4, h_, HID * 4, BR * 4, T, hipMemcpyDeviceToDevice, stream_) != hipSuccess) {
            set_error("speaker encoder: copy failed");
            ok = false;
        }
        ok = ok && conv(B.tdnn2, cat_, HID, nullptr, 0, T, 0, 1, y_, HID, 2);                        // tdnn2 + ReLU
        if (!ok) break;
        // SE: mean over time -> conv1 + ReLU -> conv2 + sigmoid -> y * se + residual  (:569-586)
        hipLaunchKernelGGL(k_colmean, dim3(nblk(HID)), dim3(256), 0, stream_, y_, HID, T, HID, vec_);
        hipLaunchKernelGGL(k_matvec, dim3((128 + 3) / 4), dim3(256), 0, stream_, B.se1.w, B.se1.b, vec_, 128, HID, 2, vec_ + 1024);
        hipLaunchKernelGGL(k_matvec, dim3((HID + 3) / 4), dim3(256), 0, stream_, B.se2.w, B.se2.b, vec_ + 1024, HID, 128, 4, vec_ + 2048);
        hipLaunchKernelGGL(k_se_apply, dim3(nblk((size_t)T * HID)), dim3(256), 0, stream_, y_, vec_ + 2048, res, ldres,
                           blocks_ + (size_t)b * HID, MFA, T, HID);
        Q3T_HIP(hipGetLastError());
    }
    // MFA: the three block outputs side by side [T][1536] -> 1x1 conv + ReLU  (:599-606)
    ok = ok && conv(mfa_, blocks_, MFA, nullptr, 0, T, 0, 1, mfa_out_, MFA, 2);
    if (ok) {
        // ASP (:611-673): global mean / std, [hs | mean | std] -> tdnn + ReLU + tanh -> conv -> softmax over time ->
        // attention-weighted mean / std
        hipLaunchKernelGGL(k_colstats, dim3(nblk(MFA)), dim3(256), 0, stream_, mfa_out_, MFA, T, MFA, vec_, vec_ + MFA);
        hipLaunchKernelGGL(k_att_in, dim3(nblk((size_t)T * 3 * MFA)), dim3(256), 0, stream_, mfa_out_, vec_, vec_ + MFA, T, xh_);
        Q3T_HIP(hipGetLastError());
        ConvParams p;
        p.xh = xh_; p.T_in = T; p.C_in = 3 * MFA; p.n_taps = 1; p.taps[0] = ConvTap{asp_tdnn_.w, 0};
        p.y = att_; p.C_out = 128; p.M = T; p.bias = asp_tdnn_.b; p.act = 3;
        ok = q3t::conv(p, stream_);
        ok = ok && conv(asp_conv_, att_, 128, nullptr, 0, T, 0, 1, att2_, MFA, 0);
    }
    if (ok) {
        hipLaunchKernelGGL(k_asp_pool, dim3(nblk(MFA)), dim3(256), 0, stream_, att2_, mfa_out_, T, vec_ + 4096);
        // FC 3072 -> dim  (:679-681)
        hipLaunchKernelGGL(k_matvec, dim3((dim_ + 3) / 4), dim3(256), 0, stream_, fc_.w, fc_.b, vec_ + 4096, dim_, 2 * MFA, 0, vec_);
        Q3T_HIP(hipGetLastError());
        Q3T_HIP(hipMemcpyAsync(emb, vec_, (size_t)dim_ * 4, hipMemcpyDeviceToHost, stream_));
    }
    Q3T_HIP(hipStreamSynchronize(stream_));
    return ok;
}

}  // namespace q3t
