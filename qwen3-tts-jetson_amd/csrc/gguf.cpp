// gguf.cpp — GGUF v2/v3 reader.  Layout: magic "GGUF", u32 version, u64 n_tensors, u64 n_kv, kv pairs,
// tensor infos (name, n_dims, ne[], type, offset), padding to general.alignment (default 32), data.
#include "gguf.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>

namespace q3t {

size_t GgufTensor::nbytes() const {
    return (size_t)nelements() * (type == GGML_TYPE_F16 ? 2 : type == GGML_TYPE_F32 ? 4 : 0);
}

Gguf::~Gguf() { close(); }

void Gguf::close() {
    if (map_) munmap(map_, size_);
    map_ = nullptr;
    size_ = 0;
    tensors_.clear();
    index_.clear();
    kv_.clear();
}

namespace {
struct Reader {
    const uint8_t *p, *end;
    bool ok = true;
    template <class T> T get() {
        T v{};
        if ((size_t)(end - p) < sizeof(T)) { ok = false; return v; }
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    std::string str() {
        const uint64_t n = get<uint64_t>();
        if (!ok || (uint64_t)(end - p) < n) { ok = false; return {}; }
        std::string s(reinterpret_cast<const char *>(p), n);
        p += n;
        return s;
    }
};
const size_t kScalarSize[13] = {1, 1, 2, 2, 4, 4, 4, 1, 0, 0, 8, 8, 8};

bool read_value(Reader &r, uint32_t type, GgufValue &v, int depth = 0) {
    v.type = (int)type;
    if (type == 8) { v.s = r.str(); return r.ok; }
    if (type == 9) {
        const uint32_t et = r.get<uint32_t>();
        const uint64_t n = r.get<uint64_t>();
        if (!r.ok || depth > 2) return false;
        for (uint64_t i = 0; i < n; ++i) {
            GgufValue e;
            if (!read_value(r, et, e, depth + 1)) return false;
            if (et == 8) v.sarr.push_back(std::move(e.s));
            else v.arr.push_back((int64_t)e.u);
        }
        return true;
    }
    if (type > 12 || kScalarSize[type] == 0) return false;
    uint8_t b[8] = {0};
    if ((size_t)(r.end - r.p) < kScalarSize[type]) return false;
    std::memcpy(b, r.p, kScalarSize[type]);
    r.p += kScalarSize[type];
    switch (type) {
        case 0: v.u = b[0]; v.f = b[0]; break;
        case 1: v.u = (uint64_t)(int64_t)(int8_t)b[0]; v.f = (int8_t)b[0]; break;
        case 2: { uint16_t x; std::memcpy(&x, b, 2); v.u = x; v.f = x; } break;
        case 3: { int16_t x; std::memcpy(&x, b, 2); v.u = (uint64_t)(int64_t)x; v.f = x; } break;
        case 4: { uint32_t x; std::memcpy(&x, b, 4); v.u = x; v.f = x; } break;
        case 5: { int32_t x; std::memcpy(&x, b, 4); v.u = (uint64_t)(int64_t)x; v.f = x; } break;
        case 6: { float x; std::memcpy(&x, b, 4); v.u = (uint64_t)(int64_t)x; v.f = x; } break;
        case 7: v.u = b[0]; v.f = b[0]; break;
        case 10: { uint64_t x; std::memcpy(&x, b, 8); v.u = x; v.f = (double)x; } break;
        case 11: { int64_t x; std::memcpy(&x, b, 8); v.u = (uint64_t)x; v.f = (double)x; } break;
        case 12: { double x; std::memcpy(&x, b, 8); v.u = (uint64_t)(int64_t)x; v.f = x; } break;
    }
    return true;
}
}  // namespace

bool Gguf::open(const std::string &path) {
    close();
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) { err_ = "Failed to open GGUF file: " + path; return false; }
    struct stat st;
    if (fstat(fd, &st) != 0) { ::close(fd); err_ = "stat failed: " + path; return false; }
    size_ = (size_t)st.st_size;
    void *m = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) { err_ = "mmap failed: " + path; size_ = 0; return false; }
    map_ = static_cast<uint8_t *>(m);
    Reader r{map_, map_ + size_};
    if (size_ < 24 || std::memcmp(map_, "GGUF", 4) != 0) { err_ = "not a GGUF file: " + path; close(); return false; }
    r.p += 4;
    const uint32_t version = r.get<uint32_t>();
    if (version < 2 || version > 3) { err_ = "unsupported GGUF version " + std::to_string(version); close(); return false; }
    const uint64_t nt = r.get<uint64_t>(), nkv = r.get<uint64_t>();
    for (uint64_t i = 0; i < nkv && r.ok; ++i) {
        std::string key = r.str();
        const uint32_t type = r.get<uint32_t>();
        GgufValue v;
        if (!read_value(r, type, v)) { err_ = "bad GGUF kv: " + key; close(); return false; }
        kv_[key] = std::move(v);
    }
    uint64_t alignment = 32;
    auto it = kv_.find("general.alignment");
    if (it != kv_.end() && it->second.u) alignment = it->second.u;
    tensors_.resize(nt);
    for (uint64_t i = 0; i < nt && r.ok; ++i) {
        GgufTensor &t = tensors_[i];
        t.name = r.str();
        t.n_dims = (int)r.get<uint32_t>();
        if (t.n_dims < 1 || t.n_dims > 4) { err_ = "bad tensor dims: " + t.name; close(); return false; }
        for (int d = 0; d < t.n_dims; ++d) t.ne[d] = (int64_t)r.get<uint64_t>();
        t.type = (int)r.get<uint32_t>();
        t.offset = r.get<uint64_t>();
    }
    if (!r.ok) { err_ = "truncated GGUF header"; close(); return false; }
    const uint64_t pos = (uint64_t)(r.p - map_);
    const uint64_t data_off = (pos + alignment - 1) / alignment * alignment;
    for (size_t i = 0; i < tensors_.size(); ++i) {
        GgufTensor &t = tensors_[i];
        if (t.type != GGML_TYPE_F16 && t.type != GGML_TYPE_F32) continue;   // quantised types: not supported
        if (data_off + t.offset + t.nbytes() > size_) { err_ = "tensor data out of range: " + t.name; close(); return false; }
        t.data = map_ + data_off + t.offset;
        index_[t.name] = i;
    }
    return true;
}

const GgufTensor *Gguf::find(const std::string &name) const {
    auto it = index_.find(name);
    return it == index_.end() ? nullptr : &tensors_[it->second];
}

const GgufValue *Gguf::get(const std::string &key) const {
    auto it = kv_.find(key);
    return it == kv_.end() ? nullptr : &it->second;
}

int64_t Gguf::get_int(std::initializer_list<const char *> keys, int64_t def) const {
    for (const char *k : keys) {
        auto it = kv_.find(k);
        if (it != kv_.end()) return (int64_t)it->second.u;
    }
    return def;
}
float Gguf::get_f32(std::initializer_list<const char *> keys, float def) const {
    for (const char *k : keys) {
        auto it = kv_.find(k);
        if (it != kv_.end()) return (float)it->second.f;
    }
    return def;
}

}  // namespace q3t
