// devlock.h — per-device reader/writer lock shared by every entry point that puts work on a GPU.
//
// Persistent grids (persist.hip: one 256-thread workgroup per CU, granule hand-offs) must never share the device with
// other work: a 256-workgroup grid launched next to another context's kernels could be left partly non-resident, and
// every hand-off would then time out into the launch-per-op fallback.  Single-slot decode runs (the only ones that
// launch persistent kernels) hold the lock exclusively; everything else (batched decode, the vocoder, the speaker
// encoder, context creation) holds it shared, so those run concurrently with each other but never beside a
// persistent grid.  Every holder keeps it until its GPU work has drained (the entry points all return synchronised).
// Re-entrant per thread: a retry, or a frame callback calling back into the library on the same thread, keeps the
// hold it has (a callback must not start a single-slot generation on another context of the same device).
// Frame callbacks (q3t_generate_stream, q3t_generate_queue) run while their generate holds the lock.  Waiting writers
// are preferred over new readers for at most 20 ms (engine.cpp WPLock): a callback that waits for another thread's
// shared-hold work on the same device (a vocoder worker) is therefore delayed, never deadlocked, by a single-slot
// generate queued meanwhile.
#pragma once
#include <mutex>
#include <shared_mutex>

namespace q3t {

class DeviceLock {
public:
    DeviceLock(bool exclusive, int device);
    ~DeviceLock();
    DeviceLock(const DeviceLock &) = delete;
    DeviceLock &operator=(const DeviceLock &) = delete;

private:
    int dev_, mode_ = 0;
};

}  // namespace q3t
