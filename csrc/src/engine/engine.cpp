// gol-mi355x: engine base (superstep loop, halo plan, compat mode, fault injection) + CPU backend.
#include "gol/engine.hpp"

#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>

#include "gol/cpu.hpp"
#include "gol/trace.hpp"

namespace gol {

// ---------------------------------------------------------------------------------------------
// Base
// ---------------------------------------------------------------------------------------------

Engine::Engine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t)
    : g_(g), cfg_(c), t_(std::move(t)) {
    if (!t_) throw Error("engine needs a transport");
    xchg_self_ = cfg_.self_exchange && !cfg_.compat;
    if (t_->size() != g_.dec.P || t_->rank() != g_.rank)
        throw Error(strprintf("transport (rank %d of %d) does not match the geometry (rank %d of %d)", t_->rank(),
                              t_->size(), g_.rank, g_.dec.P));
    // auto depth: 32 generations per superstep (the tile-kernel autotune tries passes of up to 32
    // on one rank); with neighbours (or self-exchange, which stands in for them on one GPU), 128 for
    // 1-D strips of >= 2048 rows and 56 for 2-D tiles of >= 2048 rows (the column halo is one word:
    // <= 63): an exchange costs an RCCL kernel plus ~15 us of cross-stream event latency however
    // small it is (kernel traces of the 4096 x 32768 strip of config 3 strong-scaled over 8 GPUs:
    // 11-13 us RCCL + 14 us event wait per superstep, profiles/), while the ghost rows a deeper
    // superstep recomputes cost < 1.5% at 2048 rows.
    // The HIP backend runs a superstep as kernel passes of K (auto 8) generations (deep halos).
    // (from the average strip height, identical on every rank: all ranks must cut the same
    // supersteps, and uneven strips differ by a row)
    const i64 strip_rows = g_.dec.H / std::max(1, g_.dec.Py);
    const bool nbrs = g_.dec.P > 1 || xchg_self_;
    const bool tall_strips = nbrs && !two_d() && strip_rows >= 2048;
    const bool tall_tiles = nbrs && two_d() && strip_rows >= 2048;
    // ... and 128 when the two-sub-tile mode can run (HIP, GOL_SUBTILES auto or 2, 1-D tiles of >=
    // 24576 rows, aligned width, no measurement / compat mode; any transport: device transports
    // run the halves' exchange stream ordered, host transports stage it): its halves wait for each
    // other once per superstep (a kernel trace
    // showed ~47 us of one queue and ~12 us of both idle at every boundary), so longer supersteps
    // pay that less often: 32768^2, 2048 generations, 10.01-10.05 us/gen at 64, 9.94-9.98 at 96,
    // 9.70-9.79 at 128 (profiles/subtile_superstep_boundaries.txt).  Rank-invariant inputs only.
    const bool sub_tall = cfg_.backend == "hip" && (cfg_.subtiles == 2 || cfg_.subtiles < 0) && !two_d() && strip_rows >= kSubtileMinRows &&
                          g_.dec.W % 64 == 0 && !cfg_.force_split && !cfg_.profile && !cfg_.compat &&
                          cfg_.kernel != "lds" && cfg_.kernel != "tile" && cfg_.kernel != "pipe";
    // (1-D strips with neighbours: 128 measured 1-3% faster than 64 through RCCL self-exchange,
    // 4096 x 32768 2.44 -> 2.36, 8192 x 65536 5.93 -> 5.85 us/gen; profiles/per_rank_tiles_self_exchange.txt)
    const int want = cfg_.halo_depth > 0 ? cfg_.halo_depth : (sub_tall || tall_strips ? 128 : (tall_tiles ? 56 : 32));
    int R = clamp_halo_depth(g_.dec, want);
    if (two_d()) R = std::min(R, 63);  // the column halo is one 64-cell word
    if (cfg_.compat) {
        if (two_d()) throw Error("GOL_COMPAT=reference supports 1-D row strips only");
        R = 1;
    }
    L_ = Layout(g_.h, g_.w, R);
    stats_.depth = R;
    std::string f = env_str("GOL_FAULT", "");
    if (!f.empty()) {
        int fr = -1;
        long long fg = -1;
        char mode[16] = {0};
        const int n = sscanf(f.c_str(), "%d:%lld:%15s", &fr, &fg, mode);
        if (n >= 2 && fr == g_.rank) {
            fault_gen_ = fg;
            if (n == 3) fault_mode_ = mode;
            if (fault_mode_ != "abort" && fault_mode_ != "hang" && fault_mode_ != "exit")
                throw Error("GOL_FAULT mode must be abort, hang or exit (got '" + fault_mode_ + "')");
        }
    }
    if (cfg_.watchdog_s > 0) {
        // (the probe is a virtual call on the watchdog thread: it is enabled at the end of init(),
        // once the backend is fully constructed, and backends stop the watchdog first on destruction)
        wd_ = std::make_unique<Watchdog>(
            cfg_.watchdog_s, [this](const std::string& what) { fatal("watchdog: " + what, 4); },
            [this] { return probe(); });
    }
}

void Engine::fatal(const std::string& what, int code) {
    fprintf(stderr, "[gol] rank %d, generation %llu: %s; aborting the job\n", g_.rank, (unsigned long long)gen_,
            what.c_str());
    fflush(stderr);
    // The transport's abort (ncclCommAbort, MPI_Abort, socket teardown) must not be able to hang
    // the exit: a last-resort timer ends the process regardless.
    std::thread([code] {
        std::this_thread::sleep_for(std::chrono::seconds(15));
        fprintf(stderr, "[gol] transport abort did not return within 15 s; exiting\n");
        fflush(stderr);
        _exit(code);
    }).detach();
    t_->abort(code);
    _exit(code);  // not reached: Transport::abort does not return
}

void Engine::progress(const char* next_phase) {
    if (!wd_) return;
    note_progress();
    wd_->kick(next_phase);
}

std::unique_ptr<Engine> Engine::create(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t) {
    if (c.backend == "cpu") return make_cpu_engine(g, c, std::move(t));
    if (c.backend == "hip") return make_hip_engine(g, c, std::move(t));
    throw Error("unknown backend '" + c.backend + "' (expected cpu or hip)");
}

std::string Engine::describe() const {
    const std::string wg = cfg_.backend == "hip" ? strprintf(", tile workgroup %d waves", cfg_.tile_waves) : "";
    return strprintf("%s backend, %s, rank %d tile %lldx%lld at (%lld,%lld), halo depth %d, transport %s%s%s",
                     backend_name().c_str(), g_.dec.describe().c_str(), g_.rank, (long long)g_.h, (long long)g_.w,
                     (long long)g_.row0, (long long)g_.col0, L_.R, t_->name().c_str(), wg.c_str(),
                     cfg_.compat ? ", compat=reference" : "");
}

std::vector<Engine::HaloItem> Engine::halo_items(int k) const {
    std::vector<HaloItem> items;
    const i64 h = L_.h, nw = L_.nw, P = L_.pitch;
    auto add = [&](Dir d, Rect s, Rect r, bool contig) {
        const int sp = g_.nbr[d], rp = g_.nbr[opposite(d)];
        if (sp == g_.rank && rp == g_.rank && !xchg_self_) return;  // self direction: wrap by addressing
        items.push_back({d, sp, rp, s, r, contig});
    };
    if (!two_d()) {
        if (!self_y()) {
            add(DIR_N, {0, k, -1, P}, {h, k, -1, P}, true);
            add(DIR_S, {h - k, k, -1, P}, {-k, k, -1, P}, true);
        }
    } else {
        if (!self_y()) {
            add(DIR_N, {0, k, 0, nw}, {h, k, 0, nw}, false);
            add(DIR_S, {h - k, k, 0, nw}, {-k, k, 0, nw}, false);
        }
        add(DIR_W, {0, h, 0, 1}, {0, h, nw, 1}, false);
        add(DIR_E, {0, h, nw - 1, 1}, {0, h, -1, 1}, false);
        if (!self_y()) {
            add(DIR_NW, {0, k, 0, 1}, {h, k, nw, 1}, false);
            add(DIR_NE, {0, k, nw - 1, 1}, {h, k, -1, 1}, false);
            add(DIR_SW, {h - k, k, 0, 1}, {-k, k, nw, 1}, false);
            add(DIR_SE, {h - k, k, nw - 1, 1}, {-k, k, -1, 1}, false);
        }
    }
    return items;
}

void Engine::init(const PatternSpec& p) {
    trace::Range range("gol.init");
    Armed armed(wd_.get());
    gen_ = 0;
    stats_ = EngineStats{};
    stats_.depth = L_.R;
    stats_.kernel = backend_name() == "cpu" ? "cpu" : cfg_.kernel;
    stats_.schedule = halo_items(L_.R).empty() ? "local" : "full";
    stats_.kernel_depth = L_.R;
    do_init(p);
    if (cfg_.compat) setup_compat();
    if (wd_) wd_->enable_probe();
}

void Engine::setup_compat() {
    // Reference halo semantics (survey Q1-Q3): the rows a rank sends are its GENERATION-0 first/last
    // rows (gol-with-cuda.cu:35-47, never refreshed), posted as Irecv(prev), Irecv(next),
    // Isend(first -> prev), Isend(last -> next) with one tag (gol-main.c:97-107).  Per-pair FIFO
    // matching of that exact order gives, for P >= 3, above = prev.last / below = next.first, and
    // for P <= 2 (prev == next) the swapped above = prev.first / below = next.last.  The ghost
    // rows are therefore constant and are installed once, in both buffers.
    const int prev = g_.nbr[DIR_N], next = g_.nbr[DIR_S];
    std::vector<u64> first = read_row(0), last = read_row(L_.h - 1);
    std::vector<u64> above(first.size()), below(first.size());
    if (t_->size() == 1) {
        above = first;  // FIFO of the two self-sends: first row arrives first
        below = last;
    } else {
        std::vector<Message> sends = {{prev, first.data(), first.size() * 8}, {next, last.data(), last.size() * 8}};
        std::vector<Message> recvs = {{prev, above.data(), above.size() * 8}, {next, below.data(), below.size() * 8}};
        t_->exchange_host(sends, recvs);
    }
    do_set_compat_halos(above, below);
}

void Engine::maybe_inject_fault() {
    if (fault_gen_ >= 0 && (i64)gen_ >= fault_gen_) {
        fprintf(stderr, "[gol] GOL_FAULT: injected %s on rank %d at generation %llu\n", fault_mode_.c_str(), g_.rank,
                (unsigned long long)gen_);
        fflush(stderr);
        if (fault_mode_ == "hang") {
            fault_gen_ = -1;
            for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));  // only a watchdog ends this
        }
        if (fault_mode_ == "exit") _exit(3);  // crash without telling the peers
        t_->abort(3);
    }
}

void Engine::run(u64 generations) {
    trace::Range range("gol.eager");  // (the HIP engine's run() opens "gol.run" before its graph replays)
    Armed armed(wd_.get());
    while (generations > 0) {
        maybe_inject_fault();
        int k = cfg_.compat ? 1 : supported_depth((int)std::min<u64>((u64)superstep_depth(), generations));
        {
            trace::Range r("gol.superstep");
            do_superstep(k);
        }
        gen_ += (u64)k;
        generations -= (u64)k;
        stats_.generations += (u64)k;
        stats_.supersteps += 1;
        progress("superstep");
    }
    maybe_inject_fault();
}

std::vector<double> Engine::time_runs(u64 gens, int reps) {
    std::vector<double> v;
    for (int r = 0; r < reps; ++r) {
        device_barrier();
        const auto t0 = std::chrono::steady_clock::now();
        run(gens);
        device_sync();
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        v.push_back(t_->allreduce_max(dt) * 1e6 / (double)std::max<u64>(1, gens));
    }
    return v;
}

u64 Engine::population() { return t_->allreduce_sum(local_reduce().first); }
u64 Engine::fingerprint() { return t_->allreduce_sum(local_reduce().second); }

// ---------------------------------------------------------------------------------------------
// CPU backend
// ---------------------------------------------------------------------------------------------

namespace {

class CpuEngine : public Engine {
   public:
    CpuEngine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t) : Engine(g, c, std::move(t)) {
        a_.assign((size_t)L_.words(), 0);
        b_.assign((size_t)L_.words(), 0);
        cur_ = a_.data();
        oth_ = b_.data();
    }
    std::string backend_name() const override { return "cpu"; }
    void synchronize() override {}

    std::vector<u64> tile_words() override {
        std::vector<u64> d((size_t)(L_.h * L_.nw));
        cpu::extract_words(cur_, L_, d.data());
        return d;
    }
    void set_tile_words(const std::vector<u64>& dense) override {
        if ((i64)dense.size() != L_.h * L_.nw) throw Error("set_tile_words: wrong size");
        cpu::insert_words(cur_, L_, dense.data());
        refresh_local(cur_);
    }
    std::pair<u64, u64> local_reduce() override {
        return {cpu::population(cur_, L_),
                cpu::fingerprint(cur_, L_, g_.row0, g_.word0(), g_.global_words())};
    }

   protected:
    void do_init(const PatternSpec& p) override {
        cpu::init_tile(cur_, L_, g_, p);
        std::fill(oth_, oth_ + L_.words(), 0);
        refresh_local(cur_);
    }

    void refresh_local(u64* buf) {
        if (self_x()) cpu::fill_ghost_cols_wrap(buf, L_, 0, L_.h);
        if (self_y() && !cfg_.compat) cpu::fill_ghost_rows_wrap(buf, L_);
    }

    void exchange(int k) {
        std::vector<HaloItem> items = halo_items(k);
        if (items.empty()) return;
        std::vector<Message> sends, recvs;
        stage_s_.resize(items.size());
        stage_r_.resize(items.size());
        for (size_t i = 0; i < items.size(); ++i) {
            const HaloItem& it = items[i];
            if (it.contiguous) {
                sends.push_back({it.send_peer, cur_ + L_.index(it.send.r0, it.send.c0), (size_t)it.send.count() * 8});
                recvs.push_back({it.recv_peer, cur_ + L_.index(it.recv.r0, it.recv.c0), (size_t)it.recv.count() * 8});
            } else {
                stage_s_[i].resize((size_t)it.send.count());
                stage_r_[i].resize((size_t)it.recv.count());
                for (i64 r = 0; r < it.send.rows; ++r)
                    memcpy(&stage_s_[i][(size_t)(r * it.send.words)], cur_ + L_.index(it.send.r0 + r, it.send.c0),
                           (size_t)it.send.words * 8);
                sends.push_back({it.send_peer, stage_s_[i].data(), stage_s_[i].size() * 8});
                recvs.push_back({it.recv_peer, stage_r_[i].data(), stage_r_[i].size() * 8});
            }
            stats_.halo_bytes += (u64)it.send.count() * 8;
        }
        t_->exchange_host(sends, recvs);
        for (size_t i = 0; i < items.size(); ++i) {
            const HaloItem& it = items[i];
            if (it.contiguous) continue;
            for (i64 r = 0; r < it.recv.rows; ++r)
                memcpy(cur_ + L_.index(it.recv.r0 + r, it.recv.c0), &stage_r_[i][(size_t)(r * it.recv.words)],
                       (size_t)it.recv.words * 8);
        }
        stats_.exchanges += 1;
    }

    void do_superstep(int k) override {
        if (!cfg_.compat) {
            exchange(k);
            if (self_y()) cpu::fill_ghost_rows_wrap(cur_, L_);
        }
        u64* res = cpu::superstep(cur_, oth_, L_, k);
        if (res != cur_) std::swap(cur_, oth_);
        if (self_x()) cpu::fill_ghost_cols_wrap(cur_, L_, 0, L_.h);
    }

    void do_set_compat_halos(const std::vector<u64>& above, const std::vector<u64>& below) override {
        for (u64* buf : {a_.data(), b_.data()}) {
            memcpy(buf + L_.index(-1, -1), above.data(), (size_t)L_.pitch * 8);
            memcpy(buf + L_.index(L_.h, -1), below.data(), (size_t)L_.pitch * 8);
            if (self_x()) {
                cpu::fill_ghost_cols_wrap(buf, L_, -1, 0);
                cpu::fill_ghost_cols_wrap(buf, L_, L_.h, L_.h + 1);
            }
        }
    }

    std::vector<u64> read_row(i64 r) override {
        return std::vector<u64>(cur_ + L_.index(r, -1), cur_ + L_.index(r, -1) + L_.pitch);
    }

   private:
    std::vector<u64> a_, b_;
    u64* cur_;
    u64* oth_;
    std::vector<std::vector<u64>> stage_s_, stage_r_;
};

}  // namespace

std::unique_ptr<Engine> make_cpu_engine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t) {
    return std::make_unique<CpuEngine>(g, c, std::move(t));
}

}  // namespace gol
