// gol-mi355x: progress watchdog (see watchdog.hpp).
#include "gol/watchdog.hpp"

#include "gol/common.hpp"

namespace gol {

namespace {
long long now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}
}  // namespace

Watchdog::Watchdog(double timeout_s, Fire fire, ProbeFn probe)
    : timeout_s_(timeout_s), fire_(std::move(fire)), probe_(std::move(probe)), last_ns_(now_ns()), phase_("start") {
    if (!(timeout_s_ > 0)) throw Error("watchdog timeout must be positive");
    th_ = std::thread([this] { loop(); });
}

Watchdog::~Watchdog() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
}

void Watchdog::kick(const char* phase) {
    last_ns_.store(now_ns(), std::memory_order_relaxed);
    phase_.store(phase, std::memory_order_relaxed);
    kicks_.fetch_add(1, std::memory_order_relaxed);
}

void Watchdog::loop() {
    const long long limit = (long long)(timeout_s_ * 1e9);
    // poll at a quarter of the timeout (bounded to [1 ms, 250 ms])
    long long tick_ns = limit / 4;
    if (tick_ns < 1000000) tick_ns = 1000000;
    if (tick_ns > 250000000) tick_ns = 250000000;
    unsigned long long seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
        cv_.wait_for(lk, std::chrono::nanoseconds(tick_ns));
        if (stop_) break;
        Probe pr;
        if (probe_ && probe_on_.load()) {
            lk.unlock();
            pr = probe_();
            lk.lock();
            if (stop_) break;
            if (pr.completed != seen) {  // a GPU marker completed since the last tick
                seen = pr.completed;
                last_ns_.store(now_ns(), std::memory_order_relaxed);
            }
        }
        std::string what;
        if (!pr.error.empty()) {
            what = pr.error;
        } else if (armed_.load() > 0 || pr.pending) {
            const long long idle = now_ns() - last_ns_.load(std::memory_order_relaxed);
            if (idle > limit) {
                const char* ph = phase_.load(std::memory_order_relaxed);
                what = strprintf("no progress for %.1f s (limit %.1f s) in phase '%s'%s", idle * 1e-9, timeout_s_,
                                 ph ? ph : "?", pr.pending ? ", GPU work outstanding" : "");
            }
        }
        if (!what.empty()) {
            lk.unlock();
            fire_(what);  // normally does not return (aborts the job)
            lk.lock();
            last_ns_.store(now_ns(), std::memory_order_relaxed);
        }
    }
}

}  // namespace gol
