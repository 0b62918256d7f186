// CPU test of the device lock's writer preference (qwen3-tts-jetson_amd/csrc/devlock.h WPLock; tests/test_devlock.py):
//   starve: 8 threads keep overlapping shared holds of 30 ms (each re-requests at once); a writer queued 100 ms in
//           must get the lock within 500 ms (with every yielded reader admitted it waited until the readers stopped)
//   yield:  a shared hold requested while a writer waits behind an existing shared hold is admitted after ~20 ms
//           (the callback / vocoder-worker case: the writer cannot get in until that hold's owner finishes, and the
//           owner waits for the new reader), i.e. no deadlock
// Prints one line per case; exit status 0 when both hold.
#include "devlock.h"

#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

using namespace std::chrono;
using q3t::WPLock;

static int starve() {
    WPLock L;
    std::atomic<bool> stop{false};
    std::vector<std::thread> rd;
    for (int i = 0; i < 8; ++i)
        rd.emplace_back([&, i] {
            std::this_thread::sleep_for(milliseconds(4 * i));
            while (!stop.load()) {
                L.lock_shared();
                std::this_thread::sleep_for(milliseconds(30));
                L.unlock_shared();
            }
        });
    std::this_thread::sleep_for(milliseconds(100));
    std::atomic<double> waited{-1.0};
    std::thread wr([&] {
        const auto t0 = steady_clock::now();
        L.lock();
        waited = duration<double, std::milli>(steady_clock::now() - t0).count();
        L.unlock();
    });
    // the readers stop after the writer got in, or after 3 s (a starved writer then gets in and the case fails)
    for (int i = 0; i < 300 && waited.load() < 0.0; ++i) std::this_thread::sleep_for(milliseconds(10));
    std::this_thread::sleep_for(milliseconds(50));
    stop = true;
    wr.join();
    for (auto &t : rd) t.join();
    std::printf("starve: writer waited %.1f ms beside 8 overlapping 30 ms readers (bound 500)\n", waited.load());
    return waited.load() < 500.0 ? 0 : 1;
}

static int yield_case() {
    WPLock L;
    std::atomic<bool> worker_done{false};
    L.lock_shared();   // the callback's generate
    std::thread writer([&] { L.lock(); L.unlock(); });
    std::this_thread::sleep_for(milliseconds(20));   // the writer is queued now
    const auto t0 = steady_clock::now();
    std::thread worker([&] { L.lock_shared(); L.unlock_shared(); worker_done = true; });   // the vocoder worker
    while (!worker_done.load() && steady_clock::now() - t0 < seconds(2)) std::this_thread::sleep_for(milliseconds(1));
    const double waited = duration<double, std::milli>(steady_clock::now() - t0).count();
    L.unlock_shared();
    worker.join();
    writer.join();
    std::printf("yield: a reader behind a queued writer got in after %.1f ms (expected ~20, bound 200)\n", waited);
    return worker_done.load() && waited < 200.0 ? 0 : 1;
}

int main() { return starve() | yield_case(); }
