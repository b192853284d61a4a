// gol-mi355x: the HIP engine class (private to csrc/src/engine).
//
// One class, its member functions defined by topic:
//   engine_hip.hip           construction, the run loop, board I/O, one-tile supersteps
//   engine_hip_plan.hip      work plans, pass cuts, interior/boundary regions
//   engine_hip_tune.hip      kernel autotune, schedule choice, pass-cost measurement
//   engine_hip_subtiles.hip  two sub-tiles per rank on two streams
//   engine_hip_graph.hip     hipGraph capture and replay of one-tile supersteps
//   engine_hip_halo.hip      halo exchange (device transport or host staging)
//   engine_hip_resident.hip  whole runs as one resident launch (step_resident)
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <thread>

#include "gol/bits.hpp"
#include "gol/trace.hpp"
#include "gol/engine.hpp"
#include "gol/hip_kernels.hpp"

#define HIP_CHECK(x)                                                                                    \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess)                                                                           \
            throw ::gol::Error(::gol::strprintf("%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, \
                                                __LINE__));                                             \
    } while (0)

namespace gol {
namespace hipeng {

struct DevPlan {
    LaneDesc* d = nullptr;
    i64 waves = 0;
    i64 rows = 0;  // rows per chunk
    u32 tflags = 0;  // tile kernel: variant bits (LDS levels per pass, in place, folded)
    bool fold = false;  // tile kernel: folded 32-lane tiles (plan.hpp build_plan(..., fold))
    PlanStats st;
};

struct DevCopies {
    hipk::CopyDesc* pack = nullptr;
    hipk::CopyDesc* unpack = nullptr;
    int npack = 0, nunpack = 0;
    i64 max_pack = 0, max_unpack = 0;
};

class HipEngine : public Engine {
   public:
    HipEngine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t);

    // Host -> device copy ordered on the compute stream; returns when the data is in HBM.
    void upload(void* dst, const void* src, size_t n) {
        HIP_CHECK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s_comp_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));
    }

    // Every buffer-writing operation on the compute stream ends with this: the next superstep's
    // waits (ready / interior / boundary) all see completed work.
    void mark_ready() {
        // Nothing waits on these when the compute stream is the only stream (no exchange, no
        // split schedule): skip them — an event record between two kernels costs ~15 us on the
        // GPU (a release fence), measured between eager supersteps on one MI355X.
        if (!events_needed_) return;
        events_synced_ = false;
        HIP_CHECK(hipEventRecord(ev_ready_, s_comp_));
    }
    // The exchange (and, for one-pass split supersteps, the bands) done on the comm stream.
    void record_halo() {
        events_synced_ = false;
        HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
    }
    // A split superstep of one pass left its bands on the comm stream unjoined: the compute stream waits
    // for them before it touches the board again (skipped once both streams were synchronised).
    void join_halo() {
        if (!halo_pending_) return;
        halo_pending_ = false;
        wait_pending(s_comp_, ev_halo_);
    }

    ~HipEngine() override;

    std::string backend_name() const override { return "hip"; }

    void synchronize() override {
        // (blocking: with a watchdog, its thread polls the GPU progress markers and the transport's
        // asynchronous error state meanwhile, and aborts the job if either stalls or fails)
        Armed armed(wd_.get());
        HIP_CHECK(hipStreamSynchronize(s_comm_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));
        events_synced_ = true;
        halo_pending_ = false;
    }

    bool gpu_idle() override {
        for (hipStream_t s : {s_comp_, s_comm_}) {
            const hipError_t e = hipStreamQuery(s);
            if (e == hipErrorNotReady) return false;
            HIP_CHECK(e);
        }
        return true;
    }

    std::vector<u64> tile_words() override;

    void set_tile_words(const std::vector<u64>& dense) override;

    std::pair<u64, u64> local_reduce() override {
        sync_canonical();
        check_res_status();
        HIP_CHECK(hipMemsetAsync(d_red_, 0, 2 * sizeof(u64), s_comp_));
        hipk::launch_reduce_board(buf_[cur_], L_, g_.row0, g_.word0(), g_.global_words(), d_red_, s_comp_);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(h_red_, d_red_, 2 * sizeof(u64), hipMemcpyDeviceToHost, s_comp_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));
        return {h_red_[0], h_red_[1]};
    }

    bool graph_shape(int& k, int& m);

    // Replay shapes {m supersteps of k, then one superstep of rem < k generations}, largest first:
    // the run-length hint as ONE graph (its whole superstep count, at most 256, plus its remainder:
    // the driver's 20-generation bench is a single replay), then M, 4 and 1 supersteps, then the
    // hint's remainder alone.  Every graph boundary costs ~8.5 us of GPU idle (8192^2 x 1000 through
    // the CLI: 5 boundaries, 3% of the run).
    struct Shape {
        int m, rem;
    };
    std::vector<Shape> graph_ladder(int k, int M) const;

    // Buffer parity of the captured (one-tile) mode.
    int par() const { return cur_; }
    void set_par(int p) { cur_ = p; }

    void prewarm_graph();

    void run_graphed(u64& generations);

    void replay(hipGraphExec_t exec, int k, int m, int rem);
    // Buffer-parity flip of a shape (one flip per kernel pass).
    int graph_flip(int k, int m, int rem) {
        size_t n = pass_depths(k).size() * (size_t)m;
        if (rem) n += pass_depths(rem).size();
        return (int)(n & 1);
    }

    void run(u64 generations) override;

    void device_barrier() override;
    std::map<std::string, double> phase_probe(int k) override;

    // ----- two sub-tiles per rank (1-D) -----
    // The tile's rows are split into two halves, each with THREE buffers of R ghost rows, each
    // running a superstep's passes on its own stream with a plan sized for the whole GPU.  The two
    // kernels of a pass overlap: while one drains, the other's waves fill the freed SIMD slots (two
    // half-board kernels on two streams: 9.8 vs 11.0 us/gen at 32768^2, docs/PERFORMANCE.md).
    //   * A superstep's first pass reads the other half's edge rows (and the torus wrap) in place
    //     (STEP_SEAM): no seam copy, no event between the copy and the first kernel.
    //   * So that the other half can read them at any time during the superstep, a superstep never
    //     writes the buffer it started from: its passes alternate between the other two buffers.
    //   * Each stream waits only for the other half's end of the previous superstep (and, with
    //     neighbours, the compute stream runs the rank's canonical RCCL messages first and the
    //     second stream waits for them).
    // Whether a rank runs one tile or two sub-tiles is decided by measurement at init
    // (choose_schedule).
    // Requested (GOL_SUBTILES=2) or auto-wanted: inputs identical on every rank (the mode is a
    // candidate of the collective schedule timing): mode, layout, average strip height, halo depth,
    // transport kind.
    bool dual_wanted() const {
        const bool want = cfg_.subtiles == 2 ||
                          (cfg_.subtiles < 0 && g_.dec.H / std::max(1, g_.dec.Py) >= kSubtileMinRows && L_.R >= 64);
        return want && !two_d() && !cfg_.compat && !cfg_.profile && !cfg_.force_split && L_.aligned() &&
               cfg_.kernel != "lds" && cfg_.kernel != "tile" && cfg_.kernel != "pipe";
    }
    // Rank-local conditions (agreed over the ranks by the caller): a tile tall enough for two
    // halves, and memory for one more board pair.  (The halves always run the temporal kernel, at
    // its own pass depth, whatever the one-tile kernel autotune picked.)
    bool dual_local_ok() const {
        if (L_.h < 8 * (i64)L_.R) return false;
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) return false;
        return 3 * alloc_bytes_ + ((size_t)1 << 30) < fr;  // 3 buffers of half a tile per half
    }

    void setup_dual();
    void teardown_dual();
    // Plans and copy lists of a k-generation sub-tile superstep (built before any capture).
    void prepare_dual(int k) {
        const std::vector<int>& ps = pass_depths(k);
        for (size_t j = 0; j < ps.size(); ++j)
            for (int s = 0; s < 2; ++s) sub_plan(s, ps[j], ext_after(ps, j));
        if (sub_overlap_ && !self_y())
            for (int part : {1, 2}) sub_plan(0, ps[0], ext_after(ps, 0), part);
    }

    // part: 0 the whole pass; a first pass split around the exchange (sub_overlap_): 1 all output
    // rows but the band next to the rank's halo (half 0: north, half 1: south), 2 that band
    const DevPlan& sub_plan(int s, int k, i64 e, int part = 0);

    u32 sub_flags() const { return step_flags() & ~hipk::STEP_WRAP_Y; }  // sub-tiles always have ghost rows

    // rows [r0, r0 + n) of sub-tile s in its buffer `par` (0..2; full pitch, contiguous)
    u64* sub_rows(int s, int par, i64 r0) { return sub_buf_[s][par] + sub_L_[s].index(r0, -1); }
    size_t rows_bytes(int s, i64 n) const { return (size_t)(n * sub_L_[s].pitch) * 8; }

    void dual_copy(u64* dst, const u64* src, size_t bytes) {
        HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s_comp_));
    }

    // Both halves done -> the canonical buffer (before anything reads it).
    void sync_canonical() {
        join_halo();
        if (!canon_stale_) return;
        HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_sub_b_, 0));  // the second half's last superstep
        for (int s = 0; s < 2; ++s)
            dual_copy(buf_[cur_] + L_.index(sub_r0_[s], -1), sub_rows(s, sub_cur_, 0), rows_bytes(s, sub_L_[s].h));
        canon_stale_ = false;
    }

    // Make `s` wait for `ev` unless it has completed already.  A cross-queue wait costs the waiting
    // queue ~20 us even on a completed event (kernel trace of the driver's 20-generation bench: the
    // second half's first kernel started 23 us after the first half's), and at the start of a run()
    // that follows a synchronisation every event has completed.  (Never inside a graph capture: the
    // sub-tile supersteps are not captured.)
    void wait_pending(hipStream_t s, hipEvent_t ev) {
        // ev_sub_a_ / ev_sub_b_ are recorded only where events_synced_ is cleared: after synchronize()
        // and before the next record they are complete, so the query (a runtime call before the
        // superstep's first launch) is skipped
        if (events_synced_) return;
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) HIP_CHECK(q);
        HIP_CHECK(hipStreamWaitEvent(s, ev, 0));
    }

    void dual_superstep(int k);
    void dual_messages(int p, int k, std::vector<Message>& sends, std::vector<Message>& recvs);
    void exchange_rows(const std::vector<Message>& sends, const std::vector<Message>& recvs, hipStream_t s);

    void launch_half(int s, int p, int k, hipStream_t st, int only = -1, int part = 0);

    const DevPlan& full_plan_stats() {
        const int R = superstep_depth();
        return plan(0, pass_depths(R)[0], ext_after(pass_depths(R), 0));
    }

    // A one-tile rank without neighbours (nothing to exchange) cuts its supersteps at the largest
    // multiple of the tuned pass depth within R, so none ends with a short pass (8192^2: tile passes
    // of 24 in 32-generation supersteps ran 24 + 8, and an 8-generation tile pass is 27% slower per
    // generation).  With neighbours every rank keeps R: the exchanges must match.
    int superstep_depth() const override {
        if (res_) return std::max(L_.R, res_run_depth());
        if (dual_ || !tuned_ || cfg_.compat || kdepth_ <= 0 || kdepth_ >= L_.R || !halo_items(L_.R).empty())
            return L_.R;
        return (L_.R / kdepth_) * kdepth_;
    }

   protected:
    void do_init(const PatternSpec& p) override;

    // Superstep depths prepared at init: the full superstep, and the hinted run's remainder.
    std::vector<int> init_depths() const {
        if (cfg_.compat) return {1};
        const int R = superstep_depth();
        std::vector<int> ks = {R};
        for (u64 n : {cfg_.run_hint}) {
            const int r = (int)(n % (u64)R);
            if (r > 0 && std::find(ks.begin(), ks.end(), r) == ks.end()) ks.push_back(r);
        }
        return ks;
    }

    void do_superstep(int k) override {
        if (dual_)
            dual_superstep(k);
        else
            tile_superstep(k);
    }

    void tile_superstep(int k);

    const std::vector<int>& pass_depths(int k);
    // Generations still to run after pass j of a superstep (the "extension" of pass j's output:
    // that many ghost rows when y has neighbours, plus the ghost words when x has neighbours).
    i64 ext_after(const std::vector<int>& ps, size_t j) const {
        i64 e = 0;
        for (size_t i = j + 1; i < ps.size(); ++i) e += ps[i];
        return e;
    }
    static int supported_kernel_depth(int want) {
        while (want > 1 && !hipk::step_depth_supported(want)) --want;
        return std::max(1, want);
    }

    void first_pass(int kx, int kp, i64 e, bool split);
    // The compute stream is being captured into a graph.
    bool capturing() const {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIP_CHECK(hipStreamIsCapturing(s_comp_, &cs));
        return cs == hipStreamCaptureStatusActive;
    }

    void spin_up();

    void measure_pass_costs();

    // Pick the superstep schedule by measurement.  Candidates (every rank builds the same list from
    // rank-invariant inputs, and agrees on the sub-tile mode's rank-local conditions by a reduction,
    // because the timing is collective):
    //   local / full  one tile; with neighbours the exchange runs on the compute stream, then one
    //                 full-region kernel pass (plus the later passes)
    //   split         one tile; the exchange on the comm stream overlaps the interior kernel, then the
    //                 boundary bands (needs an interior on every rank)
    //   subtiles      two half-tiles on two streams (1-D; dual_superstep)
    // Each candidate runs whole R-generation supersteps on scratch state (one tile: every pass reads
    // the board and writes the scratch buffer, the exchange writes the ghost rows a real superstep
    // writes; sub-tiles: their own buffers, loaded from the board at the next run), timed in three
    // interleaved rounds, best round per candidate, max over ranks.  The smallest time per
    // generation wins.
    static constexpr int kSchedReps = 4;
    void choose_schedule();
    // Close calls are settled on the real run() path: the runners-up of the timing within kConfirmMargin of
    // the pick are set up in full and predicted (predict_run) like the pick, and the fastest prediction is
    // kept (confirm_schedule; GOL_SCHED_CONFIRM=0 turns it off).  The timing runs one
    // superstep per sample on scratch state; the 2-D tile's split and full+graph timed within 1-2% of each
    // other and picked full+graph in half the inits, whose runs then measured 9.1-9.35 against split's 8.5
    // us/gen (docs/PERFORMANCE.md section 17).
    static constexpr double kConfirmMargin = 0.05;
    static constexpr int kMaxConfirm = 2;        // runners-up predicted at most (the weak rank has three close schedules)
    std::vector<std::string> sched_runners_up_;  // set by choose_schedule when the call is close
    std::string confirm_note_;     // the two predictions, appended to stats.tuning
    void apply_schedule(const std::string& pick);
    void finish_init();  // labels, plans, graphs, spin-up and the prediction of the current schedule
    void confirm_schedule();

    // (eager: the one-tile candidates without their graph replay; used to capture those graphs)
    void time_schedule(const std::string& c, int k, int reps, bool eager = false);
    double sample_schedule(const std::string& c, int k, int reps);
    void predict_run();
    // The end of a timed sample: bench.py's device-wide synchronisation when this process's engines do not
    // share the device (one rank, or RCCL: one rank per GPU), else the engine's own streams (thread ranks
    // on one GPU: a device-wide wait could wait for a peer's exchange this thread has yet to issue).
    void device_sync() override { end_sync(); }
    void end_sync() {
        if (t_->size() > 1 && t_->name().rfind("rccl", 0) != 0) return synchronize();
        Armed armed(wd_.get());
        HIP_CHECK(hipDeviceSynchronize());
        events_synced_ = true;
        halo_pending_ = false;
    }

    void do_set_compat_halos(const std::vector<u64>& above, const std::vector<u64>& below) override;

    std::vector<u64> read_row(i64 r) override {
        sync_canonical();
        synchronize();
        check_res_status();
        std::vector<u64> row((size_t)L_.pitch);
        HIP_CHECK(hipMemcpyAsync(row.data(), buf_[cur_] + L_.index(r, -1), (size_t)L_.pitch * 8, hipMemcpyDeviceToHost,
                                 s_comp_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));
        return row;
    }

    int supported_depth(int want) const override {
        // Depends on the CONFIGURED kernel only: every rank must cut the same supersteps (the halo
        // exchange sizes follow k), even when GOL_KERNEL=auto resolves differently per rank.
        if (cfg_.kernel == "lds") return 1;
        if (cfg_.kernel == "tile" || multipass_) return std::max(1, want);  // any depth: passes
        return supported_kernel_depth(want);
    }

   private:
    // ----- plans -----
    u32 step_flags() const {
        u32 f = 0;
        if (self_y() && !cfg_.compat) f |= hipk::STEP_WRAP_Y;
        if (xwrap_by_plan()) f |= hipk::STEP_WRAP_X;
        return f;
    }
    // Tile-kernel variant bits of a plan (tile_plan_flags).  Generations per LDS pass (GOL_TILE_LEVELS
    // 1, 2 or 4): auto 4 for a double-buffered tile of <= 8 waves, else 2 (kbench, 8 waves: 4 levels
    // 0.4-2% faster double-buffered, 1-2% slower in place; 16 waves: 3-7% slower;
    // profiles/tile_levels_ab.txt, profiles/tile_inplace_ab.txt).
    u32 tile_bits(bool inplace) const {
        const int lv = tile_lv_ > 0 ? tile_lv_ : (!inplace && cfg_.tile_waves <= 8 ? 4 : 2);
        return (lv == 2 ? hipk::STEP_TILE_L2 : 0u) | (lv == 4 ? hipk::STEP_TILE_L4 : 0u) |
               (inplace ? hipk::STEP_TILE_INPLACE : 0u);
    }
    // Most rows a tile may hold at depth k (the in-place variant's capacity unless GOL_TILE_INPLACE=0).
    i64 tile_rows_cap(int k) const {
        return hipk::tile_max_rows(k, cfg_.tile_waves, step_flags() | tile_bits(tile_inplace_ != 0));
    }

    // The tuned kernel of plan kind `kind` is the LDS tile kernel (every depth of that kind runs it).
    bool tile_kernel(int kind) const { return kern_[kind] == "tile"; }
    // step_pipe geometry: nw waves per workgroup (one loader + nw - 1 stages of l generations), wg
    // workgroups per CU in its plans; depth (nw - 1) l.
    struct PipeGeo {
        int nw = 0, l = 0, wg = 0;
    };
    // The step_pipe geometry of a pass of depth k: after measure_pass_costs, the measured cheapest one
    // where step_pipe beat step_temporal at that depth (pipe_geo_); before, the tuned geometry at its own
    // depth only.  nullptr: no step_pipe pass of that depth.
    const PipeGeo* pipe_geo(int k) const {
        if (!pipe_geo_.empty()) {
            auto it = pipe_geo_.find(k);
            return it == pipe_geo_.end() ? nullptr : &it->second;
        }
        return pipe_k_ > 0 && k == pipe_k_ ? &pipe_cur_ : nullptr;
    }
    // The kernel of a pass of plan kind `kind` at depth k: the LDS tile kernel when tuned so; step_pipe when
    // that kind's tuned kernel is step_pipe (the interior of a split first pass too, when the full tile's
    // is) and a geometry of depth k exists; else step_temporal where it is instantiated, else the tile
    // kernel (any depth: the bands of a first pass at a step_pipe depth).
    enum PassKernel { PK_TEMPORAL, PK_TILE, PK_PIPE };
    PassKernel pass_kernel(int kind, int k) const {
        if (kern_[kind] == "tile") return PK_TILE;
        // (an interior explicitly tuned to step_temporal keeps it: tune_split_kinds times it as such)
        if ((kern_[kind] == "pipe" || (kind == 1 && kern_[0] == "pipe" && kern_[1] != "temporal")) && pipe_geo(k))
            return PK_PIPE;
        return hipk::step_depth_supported(k) ? PK_TEMPORAL : PK_TILE;
    }
    bool tile_pass(int kind, int k) const { return pass_kernel(kind, k) == PK_TILE; }
    bool pipe_pass(int kind, int k) const { return pass_kernel(kind, k) == PK_PIPE; }
    void set_pipe(int nw, int l, int wg) {
        pipe_cur_ = {nw, l, wg};
        pipe_k_ = (nw - 1) * l;
    }

    // Rounds of one-tile-per-CU the LDS tile kernel needs for a plan (cheap estimate, no plan).
    // Plans are explicit (one descriptor row per tile), so huge boards are left to step_temporal.
    static constexpr i64 kMaxTileRounds = 16;
    i64 tile_rounds(int kind, int k, i64 e) const {
        const i64 rmax = std::max<i64>(1, tile_rows_cap(k));
        i64 tiles = 0;
        for (const Region& r : regions(kind, k, e))
            tiles += ceil_div(r.r1 - r.r0, rmax) * ceil_div(r.c1 - r.c0, (i64)kSegWords);
        return ceil_div(tiles, (i64)cus_);
    }

    // Whether supersteps use the interior (kind 1) / boundary (kind 2) split.
    bool split_used() const {
        return !cfg_.compat && cfg_.overlap && can_overlap() && (!halo_items(L_.R).empty() || cfg_.force_split);
    }

    void autotune_kernel();
    void tune_split_kinds(int k);

    bool can_overlap() const {
        // an interior must exist on EVERY rank (the schedule timing is collective, so the decision
        // uses the smallest strip, not this rank's), and the LDS kernel reads ghost words for every
        // row (2-D needs them)
        if (min_tile_rows() <= 2 * (i64)L_.R) return false;
        if (kernel_ == "lds" && two_d()) return false;
        return true;
    }

    std::vector<Region> regions(int kind, int k, i64 rem = 0) const;

    const DevPlan& plan(int kind, int k, i64 e = 0);

    void launch(int kind, int k, i64 e, const u64* src, u64* dst, hipStream_t s, u32 xflags = 0);

    // Ghost words for widths that are not a multiple of 64 when the tile is its own E/W neighbour.
    void post(u64* buf, hipStream_t s, i64 rem = 0) {
        const i64 e = self_y() ? 0 : rem;
        if (self_x() && !L_.aligned()) hipk::launch_fill_ghost_cols(buf, L_, -e, L_.h + e, s);
    }

    // ----- halo exchange -----
    // A graph capture never gets an exchange on any stream but its origin, the compute stream: an RCCL group
    // on a stream forked into a capture crashed librccl at capture time (round 5's split+graph superstep;
    // tools/rccl_capture_probe.cpp, docs/PERFORMANCE.md §17).  Throws instead, before any RCCL call, so a
    // capture attempt falls back to eager supersteps (graph_for) and a timing candidate is dropped.
    void guard_exchange_stream(hipStream_t s) const {
        if (s == s_comp_) return;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIP_CHECK(hipStreamIsCapturing(s, &cs));
        if (cs != hipStreamCaptureStatusNone || capturing())
            throw Error("exchange on a stream other than the capture's origin stream refused (an RCCL group on a "
                        "stream forked into a graph capture crashes librccl)");
    }
    const std::vector<HaloItem>& items_for(int k) {
        auto it = items_.find(k);
        if (it != items_.end()) return it->second;
        return items_.emplace(k, halo_items(k)).first->second;
    }

    void prepare(int k);

    const DevCopies& copies(int k, int parity);

    void build_messages(int k, const std::vector<HaloItem>& items, int parity, std::vector<Message>& sends,
                        std::vector<Message>& recvs);

    void exchange_device(int k, const std::vector<HaloItem>& items, int parity, hipStream_t s);

    void exchange_staged(int k, const std::vector<HaloItem>& items, int parity, hipStream_t s);

    void account(const std::vector<HaloItem>& items) {
        stats_.exchanges += 1;
        for (const HaloItem& it : items) stats_.halo_bytes += (u64)it.send.count() * 8;
    }

    void record_profile(bool with_exchange);

    // ----- graphs -----
    // The captured kernels bake in the buffer pointers, so a replay must start at the parity it was
    // captured at (an odd-pass remainder superstep flips it between run() calls).
    i64 graph_key(int k, int m, int rem) const { return (((i64)k * 1000 + m) * 1000 + rem) * 2 + par(); }
    hipGraphExec_t graph_for(int k, int m, int rem);

    // ----- resident kernel (step_resident, resident_kernel.hip) -----
    // Ranks without neighbours whose board fits in the registers of one workgroup per CU (small
    // boards, BASELINE config 2) may run a whole run() superstep as ONE launch: tiles exchange K-deep
    // halos with their neighbour tiles through HBM every K generations, inside the kernel.  A
    // candidate of the kernel autotune (timed against the best streaming / LDS-tile kernel), or forced
    // with GOL_KERNEL=resident.
    struct ResPlan {
        LaneDesc* d = nullptr;
        u32* nbr_off = nullptr;
        u32* nbr = nullptr;
        u32* counters = nullptr;  // per tile: supersteps completed (kernel-maintained)
        i64 tiles = 0;            // 0: the board does not fit resident at this depth
        int nw = 16, B = 0, kin = 0;
        i64 rows = 0;
    };
    bool resident_eligible() const {
        return halo_items(L_.R).empty() && !two_d() && self_y() && xwrap_by_plan() && !cfg_.compat && !cfg_.profile &&
               !cfg_.force_split && L_.h >= 64;
    }
    const ResPlan& res_plan(int kin);
    // One launch of G generations, src -> dst (the kernel also writes src on its way; odd superstep
    // count, so the result is in dst).
    void res_launch(int G, u64* src, u64* dst, hipStream_t s);
    // Generations per run() superstep of the resident kernel: the hinted run length (one launch per run).
    int res_run_depth() const {
        return cfg_.run_hint > 0 ? (int)std::min<u64>(std::max<u64>(cfg_.run_hint, 64), 4096) : 1024;
    }
    void check_res_status();
    // time resident launches of G generations from a scratch copy of the board; ms per generation
    float time_resident(int kin, int G);

    // ----- watchdog support: progress markers -----
    // With a watchdog, every superstep (or graph replay) publishes a marker: HIP events recorded at
    // its end on the streams it used.  The watchdog thread retires completed markers (probe), so GPU
    // progress is observed without the host ever waiting on the GPU; the host waits only when all
    // kMarkers markers are in flight (bounded lookahead).  The sub-tile path publishes its
    // end-of-superstep events (ev_sub_a_/ev_sub_b_, recorded anyway) as the marker: no extra event
    // records on the hot path.
    static constexpr int kMarkers = 64;
    struct Marker {
        hipEvent_t ev[2] = {nullptr, nullptr};
        int n = 0;  // events recorded for this marker
    };
    Marker& marker_slot();  // the next free slot (waits for the oldest marker when all are in flight)
    void publish_marker() {
        std::lock_guard<std::mutex> lk(mk_mu_);
        ++mk_count_;
    }
    // retire the completed markers at the head of the ring (mk_mu_ held); false on a HIP error
    bool retire_markers_locked(std::string* err);
    void note_progress() override;
    Watchdog::Probe probe() override;

    int dev_ = 0, cus_ = 256;
    std::string kernel_;  // resolved kernel: temporal | tile | lds (auto resolves at init)
    std::string kern_[3];  // per plan kind (full / interior / boundary), resolved by autotune
    int kdepth_ = 8;       // kernel pass depth K (<= halo depth R)
    int tdepth_ = 8;       // temporal-kernel pass depth (the sub-tile mode's, whatever kernel one tile uses)
    // temporal-kernel plans: waves per SIMD the one-round plan is sized for (0: the kernel's full
    // occupancy).  Small tiles pay (K+1)/S of vertical halo with S rows per wave, so fewer, taller
    // waves can win there; the autotuner tries 2 per SIMD against the full occupancy (3 at K=8).
    int occ_ = 0;
    // tile kernel: one LDS buffer updated in place (1), double-buffered (0), or per plan (-1, auto)
    // One timed step of the init measurements is done: progress for the watchdog (a big board's
    // autotune can take longer than its timeout in total), and with GOL_INIT_LOG=1 a line on stderr.
    const bool init_log_ = env_int("GOL_INIT_LOG", 0) != 0;
    const std::chrono::steady_clock::time_point init_t0_ = std::chrono::steady_clock::now();
    void init_step(const char* phase, const char* what, int k, float us_per_gen) {
        if (wd_) wd_->kick(phase);
        if (init_log_)
            fprintf(stderr, "[gol] rank %d init %.2f s: %s %s@%d %.3f us/gen\n", g_.rank,
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - init_t0_).count(), phase, what, k,
                    us_per_gen);
    }
    // Streaming-kernel segment height beyond which a plan takes several rounds (plan.hpp
    // round_balanced_rows): GOL_ROUND_ROWS_PER_LEVEL (default 45) x the pass depth; 0 = one round always
    i64 round_rows_per_level_ = env_int("GOL_ROUND_ROWS_PER_LEVEL", 45);
    i64 round_rows(int k) const { return round_rows_per_level_ > 0 ? round_rows_per_level_ * k : 0; }

    int tile_inplace_ = (int)env_int("GOL_TILE_INPLACE", -1);
    int tile_fold_ = (int)env_int("GOL_TILE_FOLD", -1);
    PipeGeo pipe_cur_;  // the tuned step_pipe geometry (set_pipe); depth pipe_k_
    int pipe_k_ = 0;
    std::map<int, PipeGeo> pipe_geo_;  // measure_pass_costs: depth -> step_pipe geometry, where it wins
    bool pipe_used_ = false;                                    // some pass ran step_pipe (fault check)
    int tile_lv_ = (int)env_int("GOL_TILE_LEVELS", 0);  // tile kernel: generations per LDS pass (1, 2, 4; 0 auto)
    bool multipass_ = false;
    std::map<int, std::vector<int>> passes_;
    bool split_ = false;   // superstep schedule: interior/boundary split with overlapped exchange
    bool halo_pending_ = false;  // split: the last superstep's bands on the comm stream are not joined (join_halo)
    std::map<std::string, double> sched_us_;  // choose_schedule: us per generation per candidate
    // measure_pass_costs: us per pass by depth, [0] one tile (kind-0 passes), [1] the two sub-tiles
    std::map<int, double> pass_us_[2];
    const std::map<int, double>& pass_costs() const { return pass_us_[dual_ ? 1 : 0]; }
    bool tuned_ = false;
    std::map<std::string, float> tune_ms_;
    Marker mk_[kMarkers];
    int mk_head_ = 0, mk_count_ = 0;  // published, unretired markers: mk_[mk_head_ ..] (under mk_mu_)
    unsigned long long mk_done_ = 0;  // markers retired so far
    std::mutex mk_mu_;
    bool mk_published_ = false;  // this superstep's marker is already published (sub-tile path)
    u64* buf_[2] = {nullptr, nullptr};
    size_t alloc_bytes_ = 0;
    int cur_ = 0;
    hipStream_t s_comp_ = nullptr, s_comm_ = nullptr;
    hipEvent_t ev_ready_ = nullptr, ev_halo_ = nullptr;
    hipEvent_t ev_t0_ = nullptr, ev_t1_ = nullptr, ev_t2_ = nullptr, ev_t3_ = nullptr;
    u64* d_red_ = nullptr;
    u64* h_red_ = nullptr;
    bool device_transport_ = false;
    // Flags of the engine's stream-ordering events.  (Without the system-scope fence an event record
    // between two kernels costs 0.5 instead of 1.7 us, tools/rccl_gap_probe.hip, but the engine ran
    // slower with such events: driver command 11.49-12.89 vs 11.11-11.57 us/gen, and the self-exchange
    // cut lost its overlapped schedule, 13.5-13.8 vs 12.1-12.2; profiles/event_fence_ab.txt.)
    static constexpr unsigned event_flags() { return hipEventDisableTiming; }
    bool graph_ok_ = true;
    const bool split_capture_test_ = env_int("GOL_GRAPH_SPLIT", 0) != 0;
    const bool split_int_first_ = env_int("GOL_SPLIT_INT_FIRST", 1) != 0;  // split: interior issued before the exchange
    const bool first_pass_mark_ = env_int("GOL_FIRST_PASS_MARK", 0) != 0;  // (A/B: the ready event after every first pass)
    const bool split_bands_comm_ = env_int("GOL_SPLIT_BANDS_COMM", 1) != 0;  // split bands beside the interior (first_pass)
    const bool split_value_wait_ = env_int("GOL_SPLIT_VALUE_WAIT", 1) != 0;  // the compute stream waits for the bands by value
    u32* d_seq_ = nullptr;  // its flag (device memory) and the last value written
    u32 seq_ = 0;
    bool graph_rccl_on_ = false;  // one-tile supersteps with an RCCL exchange are captured (choose_schedule)
    // timing graphs of the graphed schedule candidates ("local", "full+graph"), by name
    struct SchedGraph {
        hipGraphExec_t exec = nullptr;
        int reps = 0;
    };
    std::map<std::string, SchedGraph> sched_graphs_;
    std::set<std::string> sched_graph_failed_;  // candidates whose capture failed (dropped)
    void destroy_sched_graphs() {
        if (sched_graphs_.empty()) return;
        hipStreamSynchronize(s_comp_);
        for (auto& kv : sched_graphs_)
            if (kv.second.exec) hipGraphExecDestroy(kv.second.exec);
        sched_graphs_.clear();
    }
    std::string sched_pick_;     // the schedule candidate choose_schedule picked (phase_probe times it)
    bool events_needed_ = true;  // another stream waits on ev_ready_
    std::vector<void*> deferred_free_;
    std::map<i64, DevPlan> plans_;
    // GOL_SUBTILES=2 state
    bool dual_ = false;
    // Exchange overlap of the sub-tile superstep (timed candidates): 0 none ("subtiles"); 1 half 0's
    // first pass, but for its band next to the north halo, runs while the exchange is in flight
    // ("subtiles+ov")
    int sub_overlap_ = 0;
    Layout sub_L_[2];
    i64 sub_r0_[2] = {0, 0};
    u64* sub_buf_[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};
    int sub_cur_ = 0;  // buffer (0..2) holding both halves' current generation
    bool sub_current_ = false;  // the halves hold the current board
    bool canon_stale_ = false;  // buf_[cur_] lags the halves (sync_canonical before reading it)
    std::map<int, DevPlan> sub_plans_;
    hipEvent_t ev_sub_a_ = nullptr, ev_sub_b_ = nullptr;  // half 0 / half 1 done with its last superstep
    bool events_synced_ = false;  // both streams synchronised since ev_sub_a_ / ev_sub_b_ were last recorded
                                                           // (ev_sub_own_, or a progress marker's pair)
    hipEvent_t ev_sub_own_[2] = {nullptr, nullptr};
    hipEvent_t ev_sub_x_ = nullptr;                        // the rank's exchange (into both halves) done
    std::map<int, DevCopies> copies_;
    std::map<int, std::vector<HaloItem>> items_;
    std::map<i64, hipGraphExec_t> graphs_;
    std::vector<u64*> dstage_s_, dstage_r_, hstage_s_, hstage_r_;
    bool res_ = false;  // supersteps run the resident kernel
    int res_kin_ = 0;   // its generations per in-kernel halo exchange
    std::map<int, ResPlan> res_plans_;
    u32* res_status_ = nullptr;
    u64* res_scratch_[2] = {nullptr, nullptr};  // timing / probe boards (the kernel rewrites its source)
    std::vector<u64*> xhs_, xhr_;  // sub-tile host staging (exchange_rows), xh_bytes_ each
    void* reg_[2] = {nullptr, nullptr};  // RCCL user-buffer registrations of buf_[0], buf_[1]
    bool stats_registered_ = false;
    size_t xh_bytes_ = 0;
};

}  // namespace hipeng
}  // namespace gol
