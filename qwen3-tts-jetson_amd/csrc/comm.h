// comm.h — the multi-GPU exchange of the decode path: one process per GPU, RCCL over xGMI.
// Utterances shard across ranks with no data-path collective; the one exchange step is the broadcast of the packed
// weight blobs from rank 0 at start-up, plus small all-reduces of metrics.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "arena.h"

namespace q3t {

constexpr int COMM_ID_BYTES = 128;   // NCCL_UNIQUE_ID_BYTES

struct Comm;
bool comm_unique_id(uint8_t *id);
bool comm_init(Comm **out, int world, int rank, const uint8_t *id, int device);
void comm_destroy(Comm *c);
int comm_rank(const Comm *c);
int comm_world(const Comm *c);
// rank 0's arenas -> every rank (sizes checked first: every rank must have laid out identical blobs)
bool comm_bcast_arenas(Comm *c, const std::vector<WeightArena *> &arenas, hipStream_t s);
// element-wise max over ranks of n host doubles (metrics; also a barrier)
bool comm_allreduce_max(Comm *c, double *v, int n, hipStream_t s);

}  // namespace q3t
