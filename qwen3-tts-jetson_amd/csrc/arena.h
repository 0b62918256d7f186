// arena.h — every weight tensor of a loader lives in ONE contiguous HBM blob.
//
// rank 0 reads the GGUF and broadcasts the packed weight blob over RCCL/xGMI; the other ranks only
// parse the GGUF headers (shapes), lay out the same blob and receive its bytes.  The allocation sequence depends
// on tensor shapes alone, so every rank computes identical offsets.  Nothing in the blob may hold a device
// pointer (pointer tables live outside it: their values differ per rank).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <string>
#include <vector>

#include "q3t_common.h"

namespace q3t {

struct WeightArena {
    bool recv = false;      // true: shapes only, the bytes arrive later (broadcast / device copy)
    bool plan = false;      // true: host-only layout (no device memory; implies recv): the offsets every rank computes
    std::vector<size_t> *trace = nullptr;   // plan: the offset of every allocation, in order
    char *base = nullptr;
    size_t cap = 0, used = 0;

    WeightArena() = default;
    WeightArena(const WeightArena &) = delete;
    WeightArena &operator=(const WeightArena &) = delete;
    ~WeightArena() {
        if (base && !plan) hipFree(base);
    }
    bool reserve(size_t bytes) {
        cap = (bytes + 255) & ~(size_t)255;
        if (plan) {   // an address that is never dereferenced: only offsets from it are recorded
            base = reinterpret_cast<char *>((size_t)1 << 44);
            return true;
        }
        if (hipMalloc(&base, cap) != hipSuccess) {
            base = nullptr;
            set_error("weight arena: hipMalloc of " + std::to_string(cap) + " B failed");
            return false;
        }
        return true;
    }
    template <class T>
    T *alloc(size_t n) {
        const size_t bytes = (std::max<size_t>(n, 1) * sizeof(T) + 255) & ~(size_t)255;
        if (!base || used + bytes > cap) {
            set_error("weight arena overflow (" + std::to_string(used + bytes) + " > " + std::to_string(cap) + " B)");
            return nullptr;
        }
        T *p = reinterpret_cast<T *>(base + used);
        if (trace) trace->push_back(used);
        used += bytes;
        return p;
    }
    // host -> arena copy; a no-op on receiving ranks (their bytes come from the broadcast)
    bool put(void *dst, const void *src, size_t bytes) {
        if (recv || plan || bytes == 0) return true;
        if (hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice) != hipSuccess) {
            set_error("weight arena: upload failed");
            return false;
        }
        return true;
    }
};

}  // namespace q3t
