// test_pipeline_cpu.cpp — host-only checks of the pipeline surface of qwen3_tts_hip.h (no GPU call is made):
//   WAV reader/writer semantics of src/qwen3_tts.cpp:567-759 (PCM16 / PCM32 / float32, channel averaging, skipped
//   chunks, fmt chunks longer than 16 bytes, clamp + x32767 truncation on write), resample_linear (:83-101), the
//   TextTokenizer mirror against the reference's known-answer vector (tests/test_tokenizer.cpp:14), and the error
//   convention of an unloaded Qwen3TTS.
//
// usage: test_pipeline_cpu <tts.gguf with the full synthetic vocab> <scratch dir>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "qwen3_tts_pipeline.h"

using namespace qwen3_tts;

static int g_fail = 0;
#define CHECK(cond, ...)                                                          \
    do {                                                                          \
        if (!(cond)) {                                                            \
            std::fprintf(stderr, "FAIL %s:%d: %s: ", __FILE__, __LINE__, #cond);  \
            std::fprintf(stderr, __VA_ARGS__);                                    \
            std::fprintf(stderr, "\n");                                           \
            ++g_fail;                                                             \
        }                                                                         \
    } while (0)

// a WAV file with a custom fmt chunk size and an extra chunk before "data"
static void write_wav(const std::string &path, uint16_t fmt, uint16_t ch, uint32_t sr, uint16_t bits,
                      const std::vector<uint8_t> &data, bool extra_chunk, uint32_t fmt_size = 16) {
    FILE *f = std::fopen(path.c_str(), "wb");
    auto u16 = [&](uint16_t v) { std::fwrite(&v, 2, 1, f); };
    auto u32 = [&](uint32_t v) { std::fwrite(&v, 4, 1, f); };
    std::fwrite("RIFF", 1, 4, f);
    u32(0);   // size unused by the reader
    std::fwrite("WAVE", 1, 4, f);
    std::fwrite("fmt ", 1, 4, f);
    u32(fmt_size);
    u16(fmt); u16(ch); u32(sr); u32(sr * ch * bits / 8); u16((uint16_t)(ch * bits / 8)); u16(bits);
    for (uint32_t i = 16; i < fmt_size; ++i) std::fputc(0, f);
    if (extra_chunk) {
        std::fwrite("LIST", 1, 4, f);
        u32(6);
        std::fwrite("abcdef", 1, 6, f);
    }
    std::fwrite("data", 1, 4, f);
    u32((uint32_t)data.size());
    std::fwrite(data.data(), 1, data.size(), f);
    std::fclose(f);
}

template <class T>
static std::vector<uint8_t> bytes_of(const std::vector<T> &v) {
    std::vector<uint8_t> b(v.size() * sizeof(T));
    std::memcpy(b.data(), v.data(), b.size());
    return b;
}

int main(int argc, char **argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: %s <tts.gguf> <dir>\n", argv[0]); return 2; }
    const std::string gguf = argv[1], dir = argv[2];

    // ---- WAV reading
    {
        const std::vector<int16_t> st = {1000, -3000, 32767, -32768, 0, 2};   // 3 stereo frames
        write_wav(dir + "/s16.wav", 1, 2, 16000, 16, bytes_of(st), true, 18);
        std::vector<float> x;
        int sr = 0;
        CHECK(load_audio_file(dir + "/s16.wav", x, sr), "pcm16 stereo");
        CHECK(sr == 16000 && x.size() == 3, "sr %d n %zu", sr, x.size());
        for (size_t i = 0; i < x.size() && i < 3; ++i) {
            const float want = (st[2 * i] / 32768.0f + st[2 * i + 1] / 32768.0f) / 2;
            CHECK(x[i] == want, "pcm16 frame %zu: %g vs %g", i, x[i], want);
        }
        const std::vector<int32_t> p32 = {1 << 30, -(1 << 30), 123456789};
        write_wav(dir + "/s32.wav", 1, 1, 24000, 32, bytes_of(p32), false);
        CHECK(load_audio_file(dir + "/s32.wav", x, sr) && x.size() == 3 && sr == 24000, "pcm32");
        CHECK(x.size() == 3 && x[0] == 0.5f && x[1] == -0.5f && x[2] == 123456789 / 2147483648.0f, "pcm32 values");
        const std::vector<float> fl = {0.25f, 0.75f, -1.5f, 0.5f};
        write_wav(dir + "/f32.wav", 3, 2, 48000, 32, bytes_of(fl), true);
        CHECK(load_audio_file(dir + "/f32.wav", x, sr) && x.size() == 2 && sr == 48000, "float32");
        CHECK(x.size() == 2 && x[0] == 0.5f && x[1] == -0.5f, "float32 values");
        write_wav(dir + "/u8.wav", 1, 1, 24000, 8, {1, 2, 3}, false);
        CHECK(!load_audio_file(dir + "/u8.wav", x, sr), "8-bit PCM must be rejected");
        write_wav(dir + "/alaw.wav", 6, 1, 24000, 8, {1, 2, 3}, false);
        CHECK(!load_audio_file(dir + "/alaw.wav", x, sr), "format 6 must be rejected");
        CHECK(!load_audio_file(dir + "/missing.wav", x, sr), "missing file");
    }
    // ---- WAV writing: header, clamp, truncation toward zero
    {
        const std::vector<float> s = {0.0f, 0.5f, -0.5f, 1.5f, -2.0f, 0.99999f, -0.00001f};
        CHECK(save_audio_file(dir + "/out.wav", s, 24000), "save");
        FILE *f = std::fopen((dir + "/out.wav").c_str(), "rb");
        std::vector<uint8_t> b(44 + s.size() * 2);
        CHECK(f && std::fread(b.data(), 1, b.size(), f) == b.size(), "read back");
        if (f) std::fclose(f);
        uint32_t riff, data, sr, br;
        uint16_t fmt, ch, ba, bits;
        std::memcpy(&riff, &b[4], 4); std::memcpy(&fmt, &b[20], 2); std::memcpy(&ch, &b[22], 2);
        std::memcpy(&sr, &b[24], 4); std::memcpy(&br, &b[28], 4); std::memcpy(&ba, &b[32], 2);
        std::memcpy(&bits, &b[34], 2); std::memcpy(&data, &b[40], 4);
        CHECK(!std::memcmp(&b[0], "RIFF", 4) && !std::memcmp(&b[8], "WAVEfmt ", 8) && !std::memcmp(&b[36], "data", 4),
              "tags");
        CHECK(riff == 36 + s.size() * 2 && data == s.size() * 2 && fmt == 1 && ch == 1 && sr == 24000 &&
                  br == 48000 && ba == 2 && bits == 16,
              "header fields");
        const int16_t want[] = {0, 16383, -16383, 32767, -32767, 32766, 0};
        for (size_t i = 0; i < s.size(); ++i) {
            int16_t v;
            std::memcpy(&v, &b[44 + 2 * i], 2);
            CHECK(v == want[i], "sample %zu: %d vs %d", i, v, want[i]);
        }
        std::vector<float> back;
        int sr2 = 0;
        CHECK(load_audio_file(dir + "/out.wav", back, sr2) && back.size() == s.size(), "round trip");
        CHECK(back.size() > 1 && back[1] == 16383 / 32768.0f, "round trip value");
    }
    // ---- resample_linear
    {
        std::vector<float> in(1000), out;
        for (int i = 0; i < 1000; ++i) in[i] = std::sin(0.01f * i);
        resample_linear(in.data(), 1000, 16000, out, 24000);
        CHECK(out.size() == 1500, "len %zu", out.size());
        for (int i = 0; i < (int)out.size(); ++i) {
            const double src = i * (16000.0 / 24000.0);
            const int i0 = (int)src;
            const float want = i0 + 1 >= 1000 ? in[999] : (float)((1.0 - (src - i0)) * in[i0] + (src - i0) * in[i0 + 1]);
            if (out[i] != want) { CHECK(false, "resample %d", i); break; }
        }
        resample_linear(in.data(), 1000, 48000, out, 24000);
        CHECK(out.size() == 500 && out[10] == in[20], "downsample");
    }
    // ---- TextTokenizer mirror (tests/test_tokenizer.cpp flow)
    {
        TextTokenizer tok;
        CHECK(!tok.is_loaded(), "initially unloaded");
        CHECK(tok.encode("x").empty(), "unloaded encode");
        CHECK(tok.load_from_gguf(gguf), "load: %s", tok.get_error().c_str());
        CHECK(tok.get_config().vocab_size == 151936, "vocab %d", tok.get_config().vocab_size);
        CHECK(tok.bos_token_id() == 151644 && tok.eos_token_id() == 151645 && tok.pad_token_id() == 151643, "ids");
        const std::vector<int32_t> want = {151644, 77091, 198, 9707, 13, 151645, 198, 151644, 77091, 198};
        CHECK(tok.encode_for_tts("Hello.") == want, "known answer");
        CHECK(tok.encode("Hello.") == (std::vector<int32_t>{9707, 13}), "encode");
        CHECK(tok.decode(tok.encode("Hello.")) == "Hello.", "decode");
        CHECK(tok.decode_token(198) == "\n", "decode_token newline");
        TextTokenizer bad;
        CHECK(!bad.load_from_gguf(dir + "/missing.gguf") && !bad.get_error().empty(), "missing gguf");
    }
    // ---- pipeline error convention without models
    {
        Qwen3TTS tts;
        CHECK(!tts.is_loaded(), "unloaded");
        tts_result r = tts.synthesize("hi");
        CHECK(!r.success && r.error_msg == "Models not loaded", "%s", r.error_msg.c_str());
        std::vector<float> e;
        CHECK(!tts.encode_speaker(dir + "/s16.wav", e) && tts.get_error() == "Models not loaded", "encode unloaded");
        CHECK(!tts.load_models(dir + "/no_such_dir"), "load from a missing dir fails");
        CHECK(!tts.get_error().empty(), "load error text");
    }
    if (g_fail) { std::fprintf(stderr, "%d check(s) failed\n", g_fail); return 1; }
    std::printf("test_pipeline_cpu: all checks passed\n");
    return 0;
}
