// gol-mi355x: the generation engine (superstep scheduler) — CPU and HIP backends.
//
// Reference loop (gol-main.c:93-116, gol-with-cuda.cu:264-284): for every generation, 2 Irecv +
// 2 Isend of one byte row, wait for the receives, launch gol_kernel, cudaDeviceSynchronize, swap.
//
// Engine loop: generations are grouped into supersteps of k <= R generations.  Per superstep:
//   1. halo refresh — exchange k-deep halos with the neighbours (canonical order, one transport call:
//      1-D: 2 contiguous full-pitch row blocks sent straight from / received straight into the board;
//      2-D: 8 packed regions incl. corners).  Self-neighbour directions need nothing: the kernel
//      wraps rows / columns by addressing.
//   2. compute — k generations in one pass of the temporal kernel.  With overlap, the interior
//      (rows that only need local data) runs on the compute stream while the exchange runs on the
//      comm stream; the boundary bands follow once the halo has landed.
//   3. swap (parity flip).
// On the HIP backend supersteps are captured into hipGraphs (pairs, so parity is preserved) and
// replayed; there is no host synchronisation inside run().
#pragma once

#include <algorithm>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "gol/geometry.hpp"
#include "gol/pattern.hpp"
#include "gol/plan.hpp"
#include "gol/transport.hpp"
#include "gol/watchdog.hpp"

namespace gol {

// Tile rows from which GOL_SUBTILES=auto uses two sub-tiles (measured: 32768^2 +3-5% per generation,
// 65536^2 equal, 16384^2 -3%; docs/PERFORMANCE.md).
constexpr i64 kSubtileMinRows = 24576;

struct EngineConfig {
    std::string backend = "cpu";      // cpu | hip
    int halo_depth = 0;               // R: generations per halo exchange (0 = auto: 8 on one rank,
                                      // 32 for 1-D multi-rank; clamped to the geometry)
    int kernel_depth = 0;             // K: generations per kernel pass (0 = auto; HIP)
    bool overlap = true;              // interior/boundary split with comm-stream exchange
    bool graph = true;                // hipGraph capture of superstep pairs
    bool compat = false;              // reference halo quirks (Q1/Q2), 1-D only, k = 1
    int device = -1;                  // HIP device (-1: current)
    i64 rows_per_wave = 0;            // plan segment height override (0 = auto)
    int waves_target = 0;             // plan wave-count target (0 = auto)
    int plan_xcds = 8;                // XCD-aware plan order (workgroup b runs on XCD b % n; 1 = off)
    std::string kernel = "auto";      // auto (timed at init) | temporal (register pipeline) |
                                      // tile (LDS-resident) | lds (1 gen, reference-class LDS tile)
    int tile_waves = 8;               // tile kernel: waves per workgroup (4, 8, 16)
    bool tune_tile_waves = true;      // GOL_KERNEL=auto may also try 8 waves (false: GOL_TILE_WAVES set)
    std::string transport = "auto";   // auto | device | host  (host = stage halos through host memory)
    bool profile = false;             // per-phase event timing
    int graph_supersteps = 0;         // supersteps per captured graph (0 = auto, even)
    int subtiles = -1;                // HIP, 1-D: two sub-tiles per rank on two streams (GOL_SUBTILES:
                                      // 2 on, 0 off, -1 auto = on for tiles of >= kSubtileMinRows rows)
    u64 run_hint = 0;                 // generations of the runs to come (CLI: iterations); the HIP
                                      // engine captures one graph covering them (<= 256 supersteps)
    int graph_rccl = -1;              // one-tile supersteps whose exchange is an RCCL group, captured in
                                      // hipGraphs (GOL_GRAPH_RCCL: 1 on, 0 off, -1 = a candidate of the
                                      // init-time schedule timing, "full+graph")
    int subtile_overlap = -1;         // sub-tiles with neighbours: half 0 starts its first pass (all but
                                      // its band next to the rank's north halo) while the exchange is in
                                      // flight (GOL_SUBTILE_OVERLAP: 1 on, 0 off, -1 = a candidate of the
                                      // init-time schedule timing, "subtiles+ov")
    int sub_occ = 2;                  // sub-tile plans: waves per SIMD each half is sized for (GOL_SUB_OCC;
                                      // 0 = the single-tile tuned occupancy)
    bool self_exchange = false;       // GOL_SELF_EXCHANGE: directions whose neighbour is this rank go
                                      // through the transport (peer == rank) instead of wrapping by
                                      // addressing: runs every halo path of the multi-GPU engine on
                                      // one rank (e.g. a 1-rank RCCL communicator)
    double watchdog_s = 0;            // abort the job after this long without progress (0 = off)
    bool force_split = false;         // run the interior/boundary edge schedule even without neighbours
    std::string sched = "auto";       // auto (timed at init) | split (overlap, with neighbours) | full
};

struct EngineStats {
    u64 generations = 0;
    u64 supersteps = 0;
    u64 exchanges = 0;
    u64 halo_bytes = 0;       // bytes sent by this rank
    u64 graph_launches = 0;
    int depth = 0;            // R (generations per halo exchange)
    int kernel_depth = 0;     // K (generations per kernel pass)
    int tile_waves = 0;       // HIP: workgroup size of the LDS tile kernel (waves)
    i64 plan_waves = 0;       // waves of the full-tile plan
    double lane_efficiency = 0;  // output words / (64 * input rows * waves) for the full plan
    // HIP: us per generation of the chosen schedule, timed at the end of init the way a hinted run
    // executes (same supersteps, graphs or eager launches, after a device barrier, from an idle GPU);
    // 0 when not measured
    double predicted_us_per_gen = 0;
    int predicted_gens = 0;     // generations of the timed supersteps behind it
    double t_exchange_ms = 0;  // profile only
    double t_compute_ms = 0;   // profile only
    std::string kernel;        // stencil kernel in use (HIP: temporal | tile | lds; CPU: cpu)
    std::string schedule;      // superstep schedule: local (no neighbours) | split | full
    std::string tuning;        // init-time measurements behind the auto choices (HIP)
    bool registered = false;   // HIP + RCCL: the boards are registered with the communicator (zero-copy halos)
};

class Engine {
   public:
    static std::unique_ptr<Engine> create(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t);
    virtual ~Engine() = default;

    void init(const PatternSpec& p);
    virtual void run(u64 generations);
    virtual void synchronize() = 0;
    // True when none of the engine's own GPU work is outstanding (non-blocking query; CPU: always).
    virtual bool gpu_idle() { return true; }

    // Local tile as dense masked words (h * nw), and the reverse (halos are refreshed).
    virtual std::vector<u64> tile_words() = 0;
    virtual void set_tile_words(const std::vector<u64>& dense) = 0;
    // (population, fingerprint) of the local tile.
    virtual std::pair<u64, u64> local_reduce() = 0;
    // Global values (collective over the transport).
    u64 population();
    u64 fingerprint();
    // Collective: align the ranks right before a timed region.  Host barrier; with a device
    // transport also a 1-element all-reduce on the compute stream, waited for, so every rank leaves
    // when the collective has completed on the GPUs, not when a host barrier happened to release it.
    virtual void device_barrier() { t_->barrier(); }
    // The end of a timed region: every GPU stream of this rank drained (HIP: device-wide when the device
    // is not shared with other ranks of the process, as torch.cuda.synchronize() in bench.py).
    virtual void device_sync() { synchronize(); }
    // Collective: `reps` timed runs of `gens` generations on the live board (it advances), each bracketed
    // as bench.py brackets its timed run (device_barrier, the run, device_sync); us per generation, max
    // over the ranks.  Used by the HIP engine's init-time prediction and by tools/predict_gap.py.
    std::vector<double> time_runs(u64 gens, int reps);
    // Collective, untimed: per-phase GPU costs of a k-generation superstep of the schedule in use, in
    // us: "exchange_us" (the halo exchange alone, when there is one) and "superstep_us" (a whole
    // superstep, exchange included), each the best of a few rounds.  Runs on scratch state: the
    // board and the generation count are unchanged.  Empty on backends without a GPU clock.
    virtual std::map<std::string, double> phase_probe(int k) {
        (void)k;
        return {};
    }

    const Geometry& geometry() const { return g_; }
    const Layout& layout() const { return L_; }
    const EngineConfig& config() const { return cfg_; }
    Transport& transport() { return *t_; }
    std::shared_ptr<Transport> transport_ptr() { return t_; }
    const EngineStats& stats() const { return stats_; }
    u64 generation() const { return gen_; }
    std::string describe() const;
    virtual std::string backend_name() const = 0;

    // One halo region in tile coordinates (rows [r0, r0+rows), words [c0, c0+words); c0 may be -1).
    struct Rect {
        i64 r0, rows, c0, words;
        i64 count() const { return rows * words; }
    };
    struct HaloItem {
        Dir d;
        int send_peer, recv_peer;
        Rect send, recv;
        bool contiguous;  // full-pitch rows: can be sent straight from the board
    };
    // Canonical-order halo messages of a k-deep superstep (self directions omitted).
    std::vector<HaloItem> halo_items(int k) const;
    // Halo layout: 2-D blocks (column halos, 8 directions) or 1-D row strips.
    bool two_d() const { return g_.dec.Px > 1 || (xchg_self_ && g_.dec.want_2d); }
    // Directions whose neighbour is this rank wrap by addressing (no messages), unless the
    // self-exchange mode routes them through the transport (x only has halos in the 2-D layout).
    bool self_x() const {
        return g_.nbr[DIR_W] == g_.rank && g_.nbr[DIR_E] == g_.rank && !(xchg_self_ && two_d());
    }
    bool self_y() const { return g_.nbr[DIR_N] == g_.rank && g_.nbr[DIR_S] == g_.rank && !xchg_self_; }
    bool xwrap_by_plan() const { return self_x() && L_.aligned(); }
    // Rows of the smallest tile of the job (identical on every rank).
    i64 min_tile_rows() const {
        i64 m = g_.dec.H;
        for (int i = 0; i < g_.dec.Py; ++i) m = std::min(m, g_.dec.row_starts[i + 1] - g_.dec.row_starts[i]);
        return m;
    }

   protected:
    Engine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t);
    virtual void do_init(const PatternSpec& p) = 0;
    virtual void do_superstep(int k) = 0;
    // Compat mode: install constant depth-1 ghost rows (both buffers); rows are full-pitch.
    virtual void do_set_compat_halos(const std::vector<u64>& above, const std::vector<u64>& below) = 0;
    virtual std::vector<u64> read_row(i64 r) = 0;  // full-pitch row r of the current buffer
    // Largest superstep depth <= want that the backend can run (HIP: instantiated kernel depths).
    virtual int supported_depth(int want) const { return want; }
    // Generations per full superstep (<= the halo depth R; HIP: a multiple of the tuned pass depth
    // when the rank has no neighbours, so no superstep ends with a short, slow pass).
    virtual int superstep_depth() const { return L_.R; }
    void setup_compat();
    void maybe_inject_fault();
    // Watchdog mode: a superstep (or graph replay) has been issued: record its progress marker
    // (backend hook) and kick the watchdog.  No-op without a watchdog.
    void progress(const char* next_phase);
    virtual void note_progress() {}
    // Watchdog probe, run on the watchdog thread (watchdog.hpp): GPU progress markers retired so far,
    // outstanding GPU work, and the data plane's asynchronous error state.
    virtual Watchdog::Probe probe() {
        Watchdog::Probe p;
        p.error = t_->async_error();
        return p;
    }
    [[noreturn]] void fatal(const std::string& what, int code);
    struct Armed {  // arms the watchdog (if any) for the lifetime of a run() / init() / synchronize() call
        explicit Armed(Watchdog* w) : w_(w) {
            if (w_) w_->arm(true);
        }
        ~Armed() {
            if (w_) w_->arm(false);
        }
        Watchdog* w_;
    };

    Geometry g_;
    EngineConfig cfg_;
    std::shared_ptr<Transport> t_;
    Layout L_;
    EngineStats stats_;
    u64 gen_ = 0;
    i64 fault_gen_ = -1;
    std::string fault_mode_ = "abort";  // GOL_FAULT=rank:gen[:abort|hang|exit]
    std::unique_ptr<Watchdog> wd_;
    bool xchg_self_ = false;  // cfg_.self_exchange (not in compat mode)
};

std::unique_ptr<Engine> make_cpu_engine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t);
std::unique_ptr<Engine> make_hip_engine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t);

// HIP runtime helpers used by the CLI / bindings (no-ops without a GPU).
int hip_device_count(int* err = nullptr);
void hip_set_device(int dev);
int hip_try_set_device(int dev);  // hipError_t of hipSetDevice (0 = success)

}  // namespace gol
