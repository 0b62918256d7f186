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
// are preferred over new readers for at most 20 ms per bypassing reader (WPLock below): a callback that waits for
// another thread's shared-hold work on the same device (a vocoder worker) is therefore delayed, never deadlocked, by a
// single-slot generate queued meanwhile.
#pragma once
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <shared_mutex>

namespace q3t {

// The lock behind DeviceLock (header-only so tests/cpp/test_devlock.cpp drives it on the CPU): writer-preferring.
// Once an exclusive holder waits, a new shared hold waits up to kReaderYield from its arrival, so a single-slot
// generate is not starved by overlapping shared holds (vocoder + batched contexts in a serving loop; glibc's
// std::shared_mutex prefers readers).  The preference is bounded: a frame callback runs under its generate's shared
// hold and may wait for another thread that needs a shared hold on the same device (a vocoder worker behind a bounded
// queue); with an unbounded preference a single-slot generate queued meanwhile would leave that worker, and the
// callback, waiting forever.  A reader that has waited kReaderYield is admitted beside the waiting writer, and each
// such admission re-arms the preference with a doubled gap (20, 40, 80 ... ms, reset when a writer gets in): while a
// writer waits, readers bypass it one at a time and ever more rarely, so overlapping holds of any finite length drain
// and the writer's wait is bounded (about twice the hold length), while a reader another holder depends on still gets
// in.
class WPLock {
public:
    using clock = std::chrono::steady_clock;
    static constexpr std::chrono::milliseconds kReaderYield{20};
    void lock() {
        std::unique_lock<std::mutex> g(m_);
        ++waiting_w_;
        cv_.wait(g, [&] { return !writer_ && readers_ == 0; });
        --waiting_w_;
        writer_ = true;
        gap_ = kReaderYield;
    }
    void unlock() {
        { std::lock_guard<std::mutex> g(m_); writer_ = false; }
        cv_.notify_all();
    }
    void lock_shared() {
        std::unique_lock<std::mutex> g(m_);
        const clock::time_point arrival = clock::now();
        for (;;) {
            if (!writer_ && waiting_w_ == 0) break;
            const clock::time_point due = std::max(arrival + kReaderYield, last_yield_ + gap_);
            if (!writer_ && clock::now() >= due) {   // waited its yield: admitted beside the queued writer, re-arm
                last_yield_ = clock::now();
                gap_ = std::min<clock::duration>(2 * gap_, std::chrono::seconds(1));
                break;
            }
            if (writer_) cv_.wait(g);
            else cv_.wait_until(g, due);
        }
        ++readers_;
    }
    void unlock_shared() {
        bool wake;
        { std::lock_guard<std::mutex> g(m_); wake = --readers_ == 0; }
        if (wake) cv_.notify_all();
    }

private:
    std::mutex m_;
    std::condition_variable cv_;
    int readers_ = 0, waiting_w_ = 0;
    bool writer_ = false;
    clock::time_point last_yield_{};
    clock::duration gap_ = kReaderYield;
};

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
