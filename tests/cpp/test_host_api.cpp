// test_host_api.cpp — drives the C++ mirror of the reference runtime surface (qwen3_tts_hip.h: TTSTransformer,
// AudioTokenizerDecoder, TRTVocoderDecoder) the way src/qwen3_tts.cpp:437-463,518 drives the reference classes.
// Self-checks the host-side semantics (error convention, callback contract, sizes) and writes the numeric outputs
// to <outdir> for tests/test_gpu_cpp_api.py, which checks them against the CPU oracle and the ctypes path.
//
// usage: test_host_api <tts.gguf> <tokenizer.gguf> <outdir>   (<outdir>/prompt.bin: int32 chat-template ids)
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "qwen3_tts_hip.h"

using namespace qwen3_tts;

static int g_fail = 0;
#define CHECK(cond, ...)                                                   \
    do {                                                                   \
        if (!(cond)) {                                                     \
            std::fprintf(stderr, "FAIL %s:%d: %s: ", __FILE__, __LINE__, #cond); \
            std::fprintf(stderr, __VA_ARGS__);                             \
            std::fprintf(stderr, "\n");                                    \
            ++g_fail;                                                      \
        }                                                                  \
    } while (0)

template <typename T>
static bool write_bin(const std::string &path, const std::vector<T> &v) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const size_t n = v.empty() ? 0 : std::fwrite(v.data(), sizeof(T), v.size(), f);
    std::fclose(f);
    return n == v.size();
}

static std::vector<int32_t> read_i32(const std::string &path) {
    std::vector<int32_t> v;
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) return v;
    int32_t x;
    while (std::fread(&x, 4, 1, f) == 1) v.push_back(x);
    std::fclose(f);
    return v;
}

// deterministic inputs (splitmix64 -> [-0.5, 0.5))
static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static float frand() {
    uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)((z >> 40) * (1.0 / 16777216.0)) - 0.5f;
}

int main(int argc, char **argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s <tts.gguf> <tokenizer.gguf> <outdir>\n", argv[0]);
        return 2;
    }
    const std::string tts = argv[1], tok = argv[2], out = argv[3];
    const std::vector<int32_t> prompt = read_i32(out + "/prompt.bin");
    if (prompt.size() < 4) {
        std::fprintf(stderr, "missing or short %s/prompt.bin\n", out.c_str());
        return 2;
    }

    // ---- error convention: bool + get_error(), nothing thrown
    {
        TTSTransformer t;
        std::vector<int32_t> codes;
        CHECK(!t.generate(prompt.data(), (int32_t)prompt.size(), nullptr, 4, codes), "generate before load");
        CHECK(t.get_error() == "Model not loaded", "error text '%s'", t.get_error().c_str());
        CHECK(!t.load_model(out + "/does_not_exist.gguf"), "load of a missing file");
        CHECK(!t.get_error().empty(), "empty error after failed load");
        AudioTokenizerDecoder d;
        std::vector<float> pcm;
        CHECK(!d.decode(prompt.data(), 1, pcm), "decode before load");
        TRTVocoderDecoder v;
        CHECK(!v.is_loaded(), "fresh TRTVocoderDecoder reports loaded");
        CHECK(!v.load_engine(tok, 0), "fixed_frames 0 accepted");
    }

    TTSTransformer t;
    if (!t.load_model(tts)) {
        std::fprintf(stderr, "load_model: %s\n", t.get_error().c_str());
        return 1;
    }
    const tts_transformer_config &cfg = t.get_config();
    const int H = cfg.hidden_size, V = cfg.codec_vocab_size;
    CHECK(H > 0 && V > 0 && cfg.n_codebooks == 16, "config H=%d V=%d ncb=%d", H, V, cfg.n_codebooks);
    CHECK(t.init_kv_cache(64), "%s", t.get_error().c_str());
    CHECK(t.init_code_pred_kv_cache(16), "%s", t.get_error().c_str());
    CHECK(!t.init_code_pred_kv_cache(17), "CP cache beyond 16 positions accepted");

    // ---- forward_step at positions 0..3 (the oracle replays the same embeddings)
    {
        const int NS = 4;
        std::vector<float> embd((size_t)NS * H), logits((size_t)NS * V), hidden((size_t)NS * H), lg, hd, gh;
        for (float &x : embd) x = frand();
        for (int p = 0; p < NS; ++p) {
            CHECK(t.forward_step(embd.data() + (size_t)p * H, p, lg, &hd), "%s", t.get_error().c_str());
            CHECK((int)lg.size() == V && (int)hd.size() == H, "step output sizes");
            CHECK(t.get_hidden_states(gh) && gh == hd, "get_hidden_states != hidden_out");
            std::memcpy(logits.data() + (size_t)p * V, lg.data(), (size_t)V * 4);
            std::memcpy(hidden.data() + (size_t)p * H, hd.data(), (size_t)H * 4);
        }
        write_bin(out + "/step_embd.bin", embd);
        write_bin(out + "/step_logits.bin", logits);
        write_bin(out + "/step_hidden.bin", hidden);
        // forward_prefill over the same rows must reproduce the step results (causal, row by row)
        std::vector<float> rows, last_logits;
        CHECK(t.forward_prefill(embd.data(), NS, 0, rows, &last_logits), "%s", t.get_error().c_str());
        float dh = 0.0f, dl = 0.0f;
        for (size_t i = 0; i < rows.size(); ++i) dh = std::fmax(dh, std::fabs(rows[i] - hidden[i]));
        for (int i = 0; i < V; ++i) dl = std::fmax(dl, std::fabs(last_logits[i] - logits[(size_t)(NS - 1) * V + i]));
        CHECK(dh == 0.0f && dl == 0.0f, "prefill vs step: hidden %g logits %g", dh, dl);
    }

    // ---- code predictor, greedy
    {
        std::vector<float> hid(H);
        for (float &x : hid) x = 2.0f * frand();
        std::vector<int32_t> codes;
        CHECK(t.predict_codes_autoregressive(hid.data(), 77, codes, 0.0f, 50), "%s", t.get_error().c_str());
        CHECK(codes.size() == 15, "15 codes");
        for (int32_t c : codes) CHECK(c >= 0 && c < cfg.code_pred_vocab_size, "code %d out of range", c);
        write_bin(out + "/cp_hidden.bin", hid);
        write_bin(out + "/cp_codes.bin", codes);
    }

    // ---- generate: plain, streaming (interval 3), stopped by the callback
    const int32_t max_len = 10;
    std::vector<float> spk(H, 0.0f);
    std::vector<int32_t> plain;
    CHECK(t.generate(prompt.data(), (int32_t)prompt.size(), spk.data(), max_len, plain, 2050, 1.05f, 0.0f, 50),
          "%s", t.get_error().c_str());
    CHECK(!plain.empty() && plain.size() % 16 == 0 && plain.size() <= (size_t)max_len * 16, "plain size %zu",
          plain.size());
    write_bin(out + "/gen_codes.bin", plain);
    {
        std::vector<int32_t> streamed, got;
        std::vector<int32_t> sizes;
        auto cb = [&](const int32_t *codes, int32_t n, int32_t ncb) {
            CHECK(ncb == 16, "n_codebooks %d", ncb);
            sizes.push_back(n);
            got.insert(got.end(), codes, codes + (size_t)n * ncb);
            return true;
        };
        CHECK(t.generate(prompt.data(), (int32_t)prompt.size(), spk.data(), max_len, streamed, 2050, 1.05f, 0.0f, 50,
                         cb, 3),
              "%s", t.get_error().c_str());
        CHECK(streamed == plain, "streamed output != plain output (greedy)");
        CHECK(got == streamed, "callback frames (%zu) != output (%zu)", got.size(), streamed.size());
        for (size_t i = 0; i + 1 < sizes.size(); ++i) CHECK(sizes[i] == 3, "chunk %zu has %d frames", i, sizes[i]);
        // returning false stops generation after the frames delivered so far
        std::vector<int32_t> stopped;
        int calls = 0;
        auto stop = [&](const int32_t *, int32_t, int32_t) { return ++calls < 1; };
        CHECK(t.generate(prompt.data(), (int32_t)prompt.size(), spk.data(), max_len, stopped, 2050, 1.05f, 0.0f, 50,
                         stop, 3),
              "%s", t.get_error().c_str());
        CHECK(calls == 1, "callback called %d times after returning false", calls);
        CHECK(stopped.size() <= 3 * 16 || plain.size() <= 3 * 16, "stopped run produced %zu values",
              stopped.size());
        CHECK(std::equal(stopped.begin(), stopped.end(), plain.begin()), "stopped prefix differs");
    }

    // ---- batched extension: 3 utterances in lock-step (seeded sampling)
    {
        std::vector<std::vector<int32_t>> prompts(3, prompt), outs;
        for (int u = 1; u < 3; ++u)
            for (size_t i = 4; i < prompts[u].size(); ++i) prompts[u][i] = (prompts[u][i] + 13 * u) % 900 + 20;
        std::vector<const float *> spks(3, spk.data());
        t.set_seed(99);
        CHECK(t.generate_batch(prompts, spks, max_len, outs, 2050, 1.05f, 0.9f, 50), "%s", t.get_error().c_str());
        CHECK(outs.size() == 3, "batch outputs");
        std::vector<int32_t> lens, flat;
        for (auto &o : outs) {
            lens.push_back((int32_t)(o.size() / 16));
            flat.insert(flat.end(), o.begin(), o.end());
        }
        std::vector<int32_t> pflat;
        for (auto &p : prompts) {
            pflat.push_back((int32_t)p.size());
            pflat.insert(pflat.end(), p.begin(), p.end());
        }
        write_bin(out + "/batch_lens.bin", lens);
        write_bin(out + "/batch_codes.bin", flat);
        write_bin(out + "/batch_prompts.bin", pflat);
    }

    // ---- vocoders on fixed codes (40+7 frames: one full and one partial chunk)
    {
        const int F = 47;
        std::vector<int32_t> codes((size_t)F * 16);
        for (size_t i = 0; i < codes.size(); ++i) codes[i] = (int32_t)((i * 2654435761u) % 2048);
        write_bin(out + "/voc_codes.bin", codes);
        AudioTokenizerDecoder d;
        std::vector<float> full;
        CHECK(d.load_model(tok), "%s", d.get_error().c_str());
        CHECK(d.get_config().sample_rate == 24000, "sample rate");
        CHECK(d.decode(codes.data(), F, full), "%s", d.get_error().c_str());
        CHECK(!full.empty(), "empty FULL decode");
        write_bin(out + "/voc_full.bin", full);
        for (int fixed : {40, 16}) {
            TRTVocoderDecoder v;
            std::vector<float> pcm;
            CHECK(v.load_engine(tok, fixed) && v.is_loaded() && v.get_fixed_frames() == fixed, "%s",
                  v.get_error().c_str());
            CHECK(v.decode(codes.data(), F, 16, pcm), "%s", v.get_error().c_str());
            CHECK(pcm.size() == (size_t)F * 1920, "chunked samples %zu", pcm.size());
            CHECK(!v.decode(codes.data(), F, 8, pcm), "n_codebooks 8 accepted");
            write_bin(out + "/voc_chunk" + std::to_string(fixed) + ".bin", pcm);
            v.unload();
            CHECK(!v.is_loaded(), "unload");
        }
    }

    t.unload_model();
    std::vector<int32_t> none;
    CHECK(!t.generate(prompt.data(), (int32_t)prompt.size(), nullptr, 4, none), "generate after unload");
    std::printf("test_host_api: %s (%d failures)\n", g_fail ? "FAIL" : "PASS", g_fail);
    return g_fail ? 1 : 0;
}
