// gol-mi355x: progress watchdog (GOL_WATCHDOG=<seconds>).
//
// The reference has no failure detection: a rank that dies after MPI_Init leaves the others
// blocked in MPI_Wait forever (gol-main.c:110-111; survey Q11).  Here a watchdog thread watches two
// kinds of progress:
//   * host progress — the engine kicks the watchdog whenever it issues or completes a step of work
//     (a superstep enqueued, a blocking host exchange returned, an init phase done);
//   * GPU progress — a probe callback, run on the watchdog thread every tick, retires the engine's
//     completed progress markers (HIP events recorded at superstep ends, no extra records on the
//     sub-tile path) and reports whether GPU work is still outstanding.  The same probe polls the
//     data plane's asynchronous error state (ncclCommGetAsyncError), so an RCCL failure is noticed
//     even while the host thread is blocked in hipStreamSynchronize.
// The watchdog fires when the probe reports an error, or when nothing has progressed for the
// timeout while the watchdog is armed (the engine is running, initialising or synchronising) or GPU
// work is outstanding.  The fire callback aborts every rank through the transport (ncclCommAbort /
// MPI_Abort / socket teardown) instead of hanging.  Because the probe runs off the host thread, the
// engine never has to fence the GPU to feed the watchdog: the sub-tile schedule stays on with it.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>

namespace gol {

class Watchdog {
   public:
    struct Probe {
        std::string error;                 // non-empty: fire now
        unsigned long long completed = 0;  // GPU progress markers retired so far (monotonic)
        bool pending = false;              // GPU work is outstanding
    };
    using Fire = std::function<void(const std::string& what)>;
    using ProbeFn = std::function<Probe()>;
    Watchdog(double timeout_s, Fire fire, ProbeFn probe = nullptr);
    ~Watchdog();
    Watchdog(const Watchdog&) = delete;
    Watchdog& operator=(const Watchdog&) = delete;

    // Progress was made; `phase` (a string literal) names what the rank does next.
    void kick(const char* phase);
    // Nested arming: the watchdog is armed while any Armed scope (run, init, synchronize) is open.
    void arm(bool on) {
        if (on) {
            kick("armed");
            armed_.fetch_add(1);
        } else {
            armed_.fetch_sub(1);
        }
    }
    double timeout() const { return timeout_s_; }
    unsigned long long kicks() const { return kicks_.load(); }
    // Start polling the probe (after the engine's members it reads are constructed).
    void enable_probe() { probe_on_.store(true); }

   private:
    void loop();
    using Clock = std::chrono::steady_clock;
    double timeout_s_;
    Fire fire_;
    ProbeFn probe_;
    std::atomic<bool> probe_on_{false};
    std::atomic<long long> last_ns_;
    std::atomic<const char*> phase_;
    std::atomic<unsigned long long> kicks_{0};
    std::atomic<int> armed_{0};
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
    std::thread th_;
};

}  // namespace gol
