#include "vocoder.h"
namespace q3t {
Vocoder::~Vocoder() { for (void *p : allocs_) hipFree(p); }
bool Vocoder::load(const std::string &, hipStream_t s) { stream_ = s; loaded_ = false; return true; }
int64_t Vocoder::n_samples(int, int) const { return 0; }
bool Vocoder::decode(const int32_t *, int, int, float *, int64_t *) { set_error("vocoder not implemented yet"); return false; }
bool Vocoder::decode_device(const int32_t *, int, float *, int64_t *, hipStream_t) { set_error("vocoder not implemented yet"); return false; }
}
