// gguf.cpp — GGUF v2/v3 reader.  Layout: magic "GGUF", u32 version, u64 n_tensors, u64 n_kv, kv pairs,
// tensor infos (name, n_dims, ne[], type, offset), padding to general.alignment (default 32), data.
#include "gguf.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>

namespace q3t {

size_t GgufTensor::nbytes() const { return ggml_type_bytes(type, nelements()); }

namespace {
float h2f_host(uint16_t h) {
    const uint32_t sign = (uint32_t)(h >> 15) << 31, exp = (h >> 10) & 0x1f, mant = h & 0x3ff;
    uint32_t u;
    if (exp == 0) {
        if (mant == 0) u = sign;
        else {   // subnormal
            int e = -1;
            uint32_t m = mant;
            do { ++e; m <<= 1; } while (!(m & 0x400));
            u = sign | (uint32_t)(127 - 15 - e) << 23 | (m & 0x3ff) << 13;
        }
    } else if (exp == 31) {
        u = sign | 0x7f800000u | mant << 13;
    } else {
        u = sign | (exp + 112) << 23 | mant << 13;
    }
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
uint16_t f2h_host(float x) {   // round to nearest even
    uint32_t u;
    std::memcpy(&u, &x, 4);
    const uint32_t sign = (u >> 16) & 0x8000u, mant = u & 0x7fffffu;
    const int32_t e8 = (int32_t)((u >> 23) & 0xff), exp = e8 - 127 + 15;
    if (e8 == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0));
    if (exp >= 31) return (uint16_t)(sign | 0x7c00u);
    if (exp <= 0) {
        if (exp < -10) return (uint16_t)sign;
        const uint32_t m = mant | 0x800000u;
        const int shift = 14 - exp;
        uint32_t r = m >> shift;
        const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (r & 1))) ++r;
        return (uint16_t)(sign | r);
    }
    uint32_t h = sign | ((uint32_t)exp << 10) | (mant >> 13);
    const uint32_t rem = mant & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1))) ++h;
    return (uint16_t)h;
}
// ggml_get_scale_min_k4: 6-bit scale / min j of a Q4_K super-block's 12 packed bytes
inline void scale_min_k4(int j, const uint8_t *q, uint8_t &d, uint8_t &m) {
    if (j < 4) { d = q[j] & 63; m = q[j + 4] & 63; }
    else { d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4); m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4); }
}
}  // namespace

size_t ggml_type_bytes(int type, int64_t n) {
    switch (type) {
        case GGML_TYPE_F32: return (size_t)n * 4;
        case GGML_TYPE_F16: return (size_t)n * 2;
        case GGML_TYPE_Q8_0: return n % 32 ? 0 : (size_t)(n / 32) * 34;     // {f16 d; int8 q[32]}
        case GGML_TYPE_Q4_0: return n % 32 ? 0 : (size_t)(n / 32) * 18;     // {f16 d; uint8 q[16]}
        case GGML_TYPE_Q4_K: return n % 256 ? 0 : (size_t)(n / 256) * 144;  // {f16 d, dmin; u8 scales[12]; u8 q[128]}
        default: return 0;
    }
}

bool ggml_to_f32(int type, const void *src, float *y, int64_t n) {
    const uint8_t *b = static_cast<const uint8_t *>(src);
    auto rd16 = [](const uint8_t *p) { uint16_t h; std::memcpy(&h, p, 2); return h2f_host(h); };
    switch (type) {
        case GGML_TYPE_F32: std::memcpy(y, src, (size_t)n * 4); return true;
        case GGML_TYPE_F16:
            for (int64_t i = 0; i < n; ++i) y[i] = rd16(b + 2 * i);
            return true;
        case GGML_TYPE_Q8_0:   // dequantize_row_q8_0: y = d * q
            if (n % 32) return false;
            for (int64_t blk = 0; blk < n / 32; ++blk, b += 34) {
                const float d = rd16(b);
                for (int j = 0; j < 32; ++j) y[blk * 32 + j] = d * (float)(int8_t)b[2 + j];
            }
            return true;
        case GGML_TYPE_Q4_0:   // dequantize_row_q4_0: low nibbles -> 0..15, high -> 16..31, offset 8
            if (n % 32) return false;
            for (int64_t blk = 0; blk < n / 32; ++blk, b += 18) {
                const float d = rd16(b);
                for (int j = 0; j < 16; ++j) {
                    y[blk * 32 + j] = (float)((b[2 + j] & 0x0F) - 8) * d;
                    y[blk * 32 + j + 16] = (float)((b[2 + j] >> 4) - 8) * d;
                }
            }
            return true;
        case GGML_TYPE_Q4_K:   // dequantize_row_q4_K: 8 sub-blocks of 32, y = d*sc*q - dmin*m
            if (n % 256) return false;
            for (int64_t blk = 0; blk < n / 256; ++blk, b += 144) {
                const float d = rd16(b), dmin = rd16(b + 2);
                const uint8_t *sc = b + 4, *q = b + 16;
                float *o = y + blk * 256;
                for (int j = 0, is = 0; j < 256; j += 64, is += 2, q += 32) {
                    uint8_t s0, m0, s1, m1;
                    scale_min_k4(is, sc, s0, m0);
                    scale_min_k4(is + 1, sc, s1, m1);
                    const float d1 = d * s0, mm1 = dmin * m0, d2 = d * s1, mm2 = dmin * m1;
                    for (int l = 0; l < 32; ++l) *o++ = d1 * (q[l] & 0xF) - mm1;
                    for (int l = 0; l < 32; ++l) *o++ = d2 * (q[l] >> 4) - mm2;
                }
            }
            return true;
        default: return false;
    }
}

Gguf::~Gguf() { close(); }

void Gguf::close() {
    if (map_) munmap(map_, size_);
    map_ = nullptr;
    size_ = 0;
    tensors_.clear();
    index_.clear();
    kv_.clear();
    owned_.clear();
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
        t.src_type = t.type;
        const size_t nb = ggml_type_bytes(t.type, t.nelements());
        if (nb == 0) continue;   // an unsupported type: the tensor is reported missing by find()
        if (data_off + t.offset + nb > size_) { err_ = "tensor data out of range: " + t.name; close(); return false; }
        t.data = map_ + data_off + t.offset;
        if (t.type != GGML_TYPE_F16 && !(t.type == GGML_TYPE_F32 && t.n_dims == 1)) {
            // quantised, or a 2-D+ F32 weight: one resident F16 copy (header comment)
            const int64_t n = t.nelements(), row = t.ne[0];
            std::vector<uint16_t> h((size_t)n);
            std::vector<float> f((size_t)row);
            const size_t row_bytes = ggml_type_bytes(t.type, row);
            if (row_bytes == 0) continue;
            const uint8_t *src = static_cast<const uint8_t *>(t.data);
            for (int64_t r = 0; r < n / row; ++r) {
                if (!ggml_to_f32(t.type, src + (size_t)r * row_bytes, f.data(), row)) { err_ = "dequantisation failed: " + t.name; close(); return false; }
                for (int64_t c = 0; c < row; ++c) h[(size_t)r * row + c] = f2h_host(f[c]);
            }
            owned_.push_back(std::move(h));
            t.data = owned_.back().data();
            t.type = GGML_TYPE_F16;
        }
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
