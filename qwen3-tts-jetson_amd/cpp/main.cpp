// qwen3-tts-cli — command line front end of the MI355X pipeline (qwen3_tts_hip.h: Qwen3TTS).
//
// Same flags, defaults, messages, exit codes, .embd cache and --serve protocol as the reference's src/main.cpp:
//   single shot   -m <dir> -t <text> [-o out.wav] [-r ref.wav] [-e speaker.embd] [sampling flags]
//   --serve       stdin lines "text<TAB>output.wav" -> stdout "OK<TAB>duration_s<TAB>time_ms<TAB>output.wav" or
//                 "ERR<TAB>message"; "quit" / "exit" ends (main.cpp:109-163)
//   -r without -e caches the embedding in <ref>.embd (raw float32, main.cpp:37-91, 246-255)
// MI355X extensions (no reference counterpart):
//   --device <n>         GPU ordinal
//   --seed <n>           sampling seed (the counter-based sampler is reproducible per seed)
//   --vocoder-chunk <n>  0 = whole-utterance vocoder; n > 0 = n-frame chunks streamed during generation
//   --batch <n>          --serve decodes up to n queued requests together on the GPU (lock-step slots): requests
//                        already waiting on stdin when one is read are batched; replies keep request order
#include <poll.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "qwen3_tts_pipeline.h"

namespace {

void print_usage(const char *program) {
    fprintf(stderr, "Usage: %s [options] -m <model_dir> -t <text>\n", program);
    fprintf(stderr, "\n");
    fprintf(stderr, "Options:\n");
    fprintf(stderr, "  -m, --model <dir>      Model directory (required)\n");
    fprintf(stderr, "  -t, --text <text>      Text to synthesize (required unless --serve)\n");
    fprintf(stderr, "  -o, --output <file>    Output WAV file (default: output.wav)\n");
    fprintf(stderr, "  -r, --reference <file> Reference audio for voice cloning\n");
    fprintf(stderr, "  -e, --embedding <file> Cached speaker embedding (.bin)\n");
    fprintf(stderr, "  --temperature <val>    Sampling temperature (default: 0.9, 0=greedy)\n");
    fprintf(stderr, "  --top-k <n>            Top-k sampling (default: 50, 0=disabled)\n");
    fprintf(stderr, "  --top-p <val>          Top-p sampling (default: 1.0)\n");
    fprintf(stderr, "  --max-tokens <n>       Maximum audio tokens (default: 4096)\n");
    fprintf(stderr, "  --repetition-penalty <val> Repetition penalty (default: 1.05)\n");
    fprintf(stderr, "  -j, --threads <n>      Number of threads (default: 4)\n");
    fprintf(stderr, "  --serve                Server mode: read requests from stdin\n");
    fprintf(stderr, "  --device <n>           GPU ordinal (default: 0)\n");
    fprintf(stderr, "  --seed <n>             Sampling seed (default: 0)\n");
    fprintf(stderr, "  --vocoder-chunk <n>    Vocoder chunk frames, 0 = whole utterance (default: model dir)\n");
    fprintf(stderr, "  --batch <n>            Server mode: decode up to n queued requests together (default: 1)\n");
    fprintf(stderr, "  -h, --help             Show this help\n");
    fprintf(stderr, "\n");
    fprintf(stderr, "Example:\n");
    fprintf(stderr, "  %s -m ./models -t \"Hello, world!\" -o hello.wav\n", program);
    fprintf(stderr, "  %s -m ./models -t \"Hello!\" -r reference.wav -o cloned.wav\n", program);
    fprintf(stderr, "\n");
    fprintf(stderr, "Server mode:\n");
    fprintf(stderr, "  %s -m ./models -e speaker.bin --serve\n", program);
    fprintf(stderr, "  Then send lines: text<TAB>output.wav\n");
    fprintf(stderr, "  Responds with:   OK<TAB>duration_s<TAB>time_ms<TAB>output.wav\n");
    fprintf(stderr, "  Send 'quit' to exit.\n");
}

std::vector<float> load_embedding(const std::string &path) {   // raw float32 (main.cpp:37-50)
    std::vector<float> e;
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return e;
    fseek(f, 0, SEEK_END);
    const long size = ftell(f);
    fseek(f, 0, SEEK_SET);
    e.resize(size > 0 ? (size_t)size / sizeof(float) : 0);
    const size_t got = e.empty() ? 0 : fread(e.data(), sizeof(float), e.size(), f);
    fclose(f);
    if (got != e.size()) e.clear();
    return e;
}

bool save_embedding(const std::string &path, const std::vector<float> &e) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = e.empty() || fwrite(e.data(), sizeof(float), e.size(), f) == e.size();
    fclose(f);
    return ok;
}

bool resolve_embedding(qwen3_tts::Qwen3TTS &tts, const std::string &embedding_file, const std::string &reference_audio,
                       std::vector<float> &embd) {   // main.cpp:62-91
    if (embedding_file.empty()) return false;
    embd = load_embedding(embedding_file);
    if (!embd.empty()) {
        fprintf(stderr, "Loaded cached speaker embedding: %s (%zu floats)\n", embedding_file.c_str(), embd.size());
        return true;
    }
    if (reference_audio.empty()) {
        fprintf(stderr, "Error: embedding file not found and no --reference provided\n");
        return false;
    }
    fprintf(stderr, "Encoding speaker embedding from: %s\n", reference_audio.c_str());
    if (!tts.encode_speaker(reference_audio, embd)) {
        fprintf(stderr, "Error: %s\n", tts.get_error().c_str());
        return false;
    }
    if (save_embedding(embedding_file, embd))
        fprintf(stderr, "Saved speaker embedding to: %s (%zu floats)\n", embedding_file.c_str(), embd.size());
    return true;
}

qwen3_tts::tts_result synthesize_one(qwen3_tts::Qwen3TTS &tts, const std::string &text,
                                     const std::vector<float> &speaker_embd, const std::string &reference_audio,
                                     const qwen3_tts::tts_params &params) {
    if (!speaker_embd.empty()) return tts.synthesize_with_embedding(text, speaker_embd, params);
    if (!reference_audio.empty()) return tts.synthesize_with_voice(text, reference_audio, params);
    return tts.synthesize(text, params);
}

struct Request {
    std::string text, output;
};

// one request line; false on EOF / quit
bool read_request(Request &r, bool &quit) {
    static char line[8192];
    for (;;) {
        if (!fgets(line, sizeof line, stdin)) return false;
        size_t len = strlen(line);
        while (len > 0 && (line[len - 1] == '\n' || line[len - 1] == '\r')) line[--len] = '\0';
        if (len == 0) continue;
        if (strcmp(line, "quit") == 0 || strcmp(line, "exit") == 0) { quit = true; return false; }
        const char *tab = strchr(line, '\t');
        r.text = tab ? std::string(line, tab - line) : std::string(line);
        r.output = tab ? std::string(tab + 1) : std::string("output.wav");
        return true;
    }
}

bool stdin_ready() {
    // data already buffered by stdio, or readable on the descriptor right now
    if (stdin->_IO_read_ptr < stdin->_IO_read_end) return true;
    struct pollfd p = {STDIN_FILENO, POLLIN, 0};
    return poll(&p, 1, 0) > 0 && (p.revents & POLLIN);
}

void reply(const qwen3_tts::tts_result &result, const Request &q) {
    if (!result.success) {
        fprintf(stdout, "ERR\t%s\n", result.error_msg.c_str());
        fflush(stdout);
        return;
    }
    if (!qwen3_tts::save_audio_file(q.output, result.audio, result.sample_rate)) {
        fprintf(stdout, "ERR\tfailed to save %s\n", q.output.c_str());
        fflush(stdout);
        return;
    }
    const float duration = (float)result.audio.size() / result.sample_rate;
    fprintf(stdout, "OK\t%.2f\t%lld\t%s\n", duration, (long long)result.t_total_ms, q.output.c_str());
    fflush(stdout);
    fprintf(stderr, "  Done: %.2fs audio in %lldms (RTF=%.1f)\n", duration, (long long)result.t_total_ms,
            (float)result.t_total_ms / 1000.0f / duration);
}

int run_server(qwen3_tts::Qwen3TTS &tts, const std::vector<float> &speaker_embd, const std::string &reference_audio,
               const qwen3_tts::tts_params &params, int batch) {   // main.cpp:109-163
    fprintf(stderr, "\nServer ready. Send: text<TAB>output.wav  (or 'quit' to exit)\n");
    fflush(stderr);
    bool quit = false;
    for (;;) {
        std::vector<Request> reqs(1);
        if (!read_request(reqs[0], quit)) break;
        while ((int)reqs.size() < batch && !quit && stdin_ready()) {
            Request r;
            if (!read_request(r, quit)) break;
            reqs.push_back(r);
        }
        for (const Request &q : reqs) fprintf(stderr, "Synthesizing: \"%s\" -> %s\n", q.text.c_str(), q.output.c_str());
        if (reqs.size() == 1 || (speaker_embd.empty() && !reference_audio.empty())) {
            for (const Request &q : reqs) reply(synthesize_one(tts, q.text, speaker_embd, reference_audio, params), q);
        } else {
            std::vector<std::string> texts;
            for (const Request &q : reqs) texts.push_back(q.text);
            std::vector<std::vector<float>> spk;
            if (!speaker_embd.empty()) spk.assign(reqs.size(), speaker_embd);
            const std::vector<qwen3_tts::tts_result> res = tts.synthesize_batch(texts, spk, params);
            for (size_t i = 0; i < reqs.size(); ++i) reply(res[i], reqs[i]);
        }
        if (quit) break;
    }
    fprintf(stderr, "Server shutting down.\n");
    return 0;
}

}  // namespace

int main(int argc, char **argv) {
    std::string model_dir, text, output_file = "output.wav", reference_audio, embedding_file;
    bool serve_mode = false;
    int device = 0, batch = 1, vocoder_chunk = -1;
    unsigned long long seed = 0;
    qwen3_tts::tts_params params;
    auto need = [&](int &i, const char *what) -> const char * {
        if (++i >= argc) {
            fprintf(stderr, "Error: missing %s\n", what);
            return nullptr;
        }
        return argv[i];
    };
    try {
        for (int i = 1; i < argc; i++) {
            const std::string arg = argv[i];
            const char *v = nullptr;
            if (arg == "-h" || arg == "--help") { print_usage(argv[0]); return 0; }
            else if (arg == "-m" || arg == "--model") { if (!(v = need(i, "model directory"))) return 1; model_dir = v; }
            else if (arg == "-t" || arg == "--text") { if (!(v = need(i, "text"))) return 1; text = v; }
            else if (arg == "-o" || arg == "--output") { if (!(v = need(i, "output file"))) return 1; output_file = v; }
            else if (arg == "-r" || arg == "--reference") { if (!(v = need(i, "reference audio"))) return 1; reference_audio = v; }
            else if (arg == "-e" || arg == "--embedding") { if (!(v = need(i, "embedding file"))) return 1; embedding_file = v; }
            else if (arg == "--temperature") { if (!(v = need(i, "temperature value"))) return 1; params.temperature = std::stof(v); }
            else if (arg == "--top-k") { if (!(v = need(i, "top-k value"))) return 1; params.top_k = std::stoi(v); }
            else if (arg == "--top-p") { if (!(v = need(i, "top-p value"))) return 1; params.top_p = std::stof(v); }
            else if (arg == "--max-tokens") { if (!(v = need(i, "max-tokens value"))) return 1; params.max_audio_tokens = std::stoi(v); }
            else if (arg == "--repetition-penalty") { if (!(v = need(i, "repetition-penalty value"))) return 1; params.repetition_penalty = std::stof(v); }
            else if (arg == "-j" || arg == "--threads") { if (!(v = need(i, "threads value"))) return 1; params.n_threads = std::stoi(v); }
            else if (arg == "--serve") serve_mode = true;
            else if (arg == "--device") { if (!(v = need(i, "device"))) return 1; device = std::stoi(v); }
            else if (arg == "--seed") { if (!(v = need(i, "seed"))) return 1; seed = std::stoull(v); }
            else if (arg == "--vocoder-chunk") { if (!(v = need(i, "vocoder-chunk value"))) return 1; vocoder_chunk = std::stoi(v); }
            else if (arg == "--batch") { if (!(v = need(i, "batch value"))) return 1; batch = std::max(1, std::stoi(v)); }
            else {
                fprintf(stderr, "Error: unknown argument: %s\n", arg.c_str());
                print_usage(argv[0]);
                return 1;
            }
        }
    } catch (const std::exception &e) {   // std::stoi / stof on a malformed number
        fprintf(stderr, "Error: invalid numeric argument (%s)\n", e.what());
        return 1;
    }
    if (model_dir.empty()) {
        fprintf(stderr, "Error: model directory is required\n");
        print_usage(argv[0]);
        return 1;
    }
    if (!serve_mode && text.empty()) {
        fprintf(stderr, "Error: text is required (or use --serve)\n");
        print_usage(argv[0]);
        return 1;
    }
    qwen3_tts::Qwen3TTS tts;
    tts.set_device(device);
    tts.set_seed(seed);
    if (vocoder_chunk >= 0) tts.set_vocoder_chunk(vocoder_chunk);
    fprintf(stderr, "Loading models from: %s\n", model_dir.c_str());
    if (!tts.load_models(model_dir)) {
        fprintf(stderr, "Error: %s\n", tts.get_error().c_str());
        return 1;
    }
    if (vocoder_chunk == 0) tts.set_vocoder_chunk(0);   // explicit 0 overrides engine files found in the model dir
    std::vector<float> speaker_embd;
    if (embedding_file.empty() && !reference_audio.empty()) embedding_file = reference_audio + ".embd";
    if (!embedding_file.empty() && !resolve_embedding(tts, embedding_file, reference_audio, speaker_embd)) return 1;
    if (serve_mode) return run_server(tts, speaker_embd, reference_audio, params, batch);
    fprintf(stderr, "Synthesizing: \"%s\"\n", text.c_str());
    if (!reference_audio.empty() && speaker_embd.empty()) fprintf(stderr, "Reference audio: %s\n", reference_audio.c_str());
    const qwen3_tts::tts_result result = synthesize_one(tts, text, speaker_embd, reference_audio, params);
    if (!result.success) {
        fprintf(stderr, "\nError: %s\n", result.error_msg.c_str());
        return 1;
    }
    fprintf(stderr, "\n");
    if (!qwen3_tts::save_audio_file(output_file, result.audio, result.sample_rate)) {
        fprintf(stderr, "Error: failed to save output file: %s\n", output_file.c_str());
        return 1;
    }
    fprintf(stderr, "Output saved to: %s\n", output_file.c_str());
    fprintf(stderr, "Audio duration: %.2f seconds\n", (float)result.audio.size() / result.sample_rate);
    if (params.print_timing) {
        fprintf(stderr, "\nTiming:\n");
        fprintf(stderr, "  Load:      %6lld ms\n", (long long)result.t_load_ms);
        fprintf(stderr, "  Tokenize:  %6lld ms\n", (long long)result.t_tokenize_ms);
        fprintf(stderr, "  Encode:    %6lld ms\n", (long long)result.t_encode_ms);
        fprintf(stderr, "  Generate:  %6lld ms\n", (long long)result.t_generate_ms);
        fprintf(stderr, "  Decode:    %6lld ms\n", (long long)result.t_decode_ms);
        fprintf(stderr, "  Total:     %6lld ms\n", (long long)result.t_total_ms);
    }
    return 0;
}
