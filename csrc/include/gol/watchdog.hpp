// gol-mi355x: progress watchdog (GOL_WATCHDOG=<seconds>).
//
// The reference has no failure detection: a rank that dies after MPI_Init leaves the others
// blocked in MPI_Wait forever (gol-main.c:110-111; survey Q11).  The engine kicks a Watchdog every
// time a superstep is known to have COMPLETED (host transports: after the blocking exchange; HIP:
// when the bounded-lookahead fence observes the GPU event, which also polls the transport's
// asynchronous error state, e.g. ncclCommGetAsyncError).  If no kick arrives within the timeout the
// watchdog thread reports the stuck phase and calls the fire callback, which aborts every rank
// through the transport (ncclCommAbort / MPI_Abort / socket teardown) instead of hanging.
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
    using Fire = std::function<void(const std::string& what)>;
    Watchdog(double timeout_s, Fire fire);
    ~Watchdog();
    Watchdog(const Watchdog&) = delete;
    Watchdog& operator=(const Watchdog&) = delete;

    // Progress was made; `phase` (a string literal) names what the rank does next.
    void kick(const char* phase);
    // Only an armed watchdog fires (the engine arms it while it runs generations).
    void arm(bool on) {
        if (on) kick("armed");
        armed_.store(on);
    }
    double timeout() const { return timeout_s_; }
    unsigned long long kicks() const { return kicks_.load(); }

   private:
    void loop();
    using Clock = std::chrono::steady_clock;
    double timeout_s_;
    Fire fire_;
    std::atomic<long long> last_ns_;
    std::atomic<const char*> phase_;
    std::atomic<unsigned long long> kicks_{0};
    std::atomic<bool> armed_{false};
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
    std::thread th_;
};

}  // namespace gol
