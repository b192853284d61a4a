// gol-mi355x: HIP backend of the engine.
//
// Board memory: two bit-packed tiles in HBM (hipMalloc, never managed memory — the reference
// migrates managed pages host<->device every generation, gol-with-cuda.cu:35-51 + gol-main.c:97-100).
// Streams: s_comp (kernels) and s_comm (halo exchange).  A superstep of R generations = one halo
// exchange + R/K kernel passes (the earlier passes also compute the ghost rows/words the later
// ones read).  With neighbours, the first pass runs one of two schedules (chosen by measurement):
//   split:  s_comm:  wait(ev_ready) -> pack (2-D) -> RCCL group send/recv (or host staging) -> unpack -> ev_halo
//           s_comp:  interior kernel -> wait(ev_halo) -> boundary kernel -> later passes -> ev_ready
//   full:   s_comp:  exchange -> full-region kernel -> later passes
// With graphs on, G/(m*R) captures of m supersteps (even pass count => parity preserved) are replayed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <chrono>
#include <cstring>
#include <map>
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

int hip_device_count(int* err) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (err) *err = (int)e;
    return e == hipSuccess ? n : 0;
}

void hip_set_device(int dev) { HIP_CHECK(hipSetDevice(dev)); }
int hip_try_set_device(int dev) { return (int)hipSetDevice(dev); }

namespace {

struct DevPlan {
    LaneDesc* d = nullptr;
    i64 waves = 0;
    i64 rows = 0;  // rows per chunk
    u32 tflags = 0;  // tile kernel: variant bits (LDS levels per pass, in place)
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
    HipEngine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t) : Engine(g, c, std::move(t)) {
        if (cfg_.device >= 0) HIP_CHECK(hipSetDevice(cfg_.device));
        HIP_CHECK(hipGetDevice(&dev_));
        hipDeviceProp_t prop;
        HIP_CHECK(hipGetDeviceProperties(&prop, dev_));
        cus_ = prop.multiProcessorCount;
        int R = L_.R;
        kernel_ = cfg_.kernel;
        hipk::ensure_trash();  // before any launch or graph capture
        // Kernel pass depth K (generations per HBM pass) vs halo depth R (generations per
        // exchange).  In 1-D (and on a single rank) a superstep of R generations runs as several
        // passes of <= K, the earlier ones also producing the ghost rows the later ones read, so
        // one exchange serves R generations (communication-avoiding deep halos).
        multipass_ = !cfg_.compat && kernel_ != "lds";
        // auto K: 8, the measured optimum of the register pipeline (3 waves/SIMD at 163 VGPRs);
        // GOL_KERNEL=auto may raise it for the LDS tile kernel (autotune_kernel)
        int K = cfg_.kernel_depth > 0 ? cfg_.kernel_depth : 8;
        K = std::min(K, R);
        if (kernel_ == "lds") {
            R = K = 1;
        } else if (kernel_ == "tile") {
            K = std::min(K, 32);  // any depth; LDS rows bound it (tile_max_rows)
        } else if (kernel_ == "temporal" || kernel_ == "auto") {
            // auto: the depth must suit both candidates (instantiated temporal depths)
            K = supported_kernel_depth(std::min(K, hipk::max_step_depth()));
        } else {
            throw Error("GOL_KERNEL must be auto, temporal, tile or lds (got '" + kernel_ + "')");
        }
        if (!multipass_) R = std::min(R, K);
        kdepth_ = K;
        tdepth_ = supported_kernel_depth(std::min(K, hipk::max_step_depth()));
        if (R != L_.R) L_ = Layout(L_.h, L_.w, R);
        stats_.depth = R;
        // slack rows: the temporal kernel prefetches 3 (shallow passes: 6) rows past a segment's last input row
        const size_t bytes = (size_t)(L_.words() + hipk::kSlackRows * L_.pitch) * 8;
        for (int i = 0; i < 2; ++i) HIP_CHECK(hipMalloc(&buf_[i], bytes));
        alloc_bytes_ = bytes;
        device_transport_ = t_->device_buffers() && cfg_.transport != "host";
        if (cfg_.transport == "device" && !t_->device_buffers())
            throw Error("GOL_TRANSPORT=device needs a device transport (RCCL)");
        for (auto& kk : kern_) kk = kernel_;
        // The two streams must sit on different hardware queues, or their kernels serialise.  HIP
        // multiplexes streams onto GPU_MAX_HW_QUEUES (4) queues, and once an RCCL communicator exists
        // (it creates streams of its own) two plain streams created afterwards were measured to land
        // on ONE queue (tools/queue_probe.cpp, profiles/queue_probe.txt: 1.68 vs 0.86 ms for two
        // concurrent kernels), which serialised the sub-tile halves and the split schedule's
        // exchange.  Streams of different priority get different queues in every case measured, so
        // the comm / second-half stream is created with the greatest priority.
        int prio_least = 0, prio_greatest = 0;
        HIP_CHECK(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
        HIP_CHECK(hipStreamCreateWithPriority(&s_comp_, hipStreamNonBlocking, 0));
        HIP_CHECK(hipStreamCreateWithPriority(&s_comm_, hipStreamNonBlocking,
                                              env_int("GOL_COMM_PRIORITY", 1) ? prio_greatest : 0));
        events_needed_ = cfg_.force_split || !halo_items(L_.R).empty();
        // All device memory work is ordered on the engine's own streams.  (They are non-blocking:
        // null-stream calls such as hipMemset, or a pageable hipMemcpy whose DMA may still be in
        // flight when it returns, would NOT be ordered before their kernels.)
        for (int i = 0; i < 2; ++i) HIP_CHECK(hipMemsetAsync(buf_[i], 0, bytes, s_comp_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));
        // Stream-ordering events (never read by the host).  GOL_EVENT_SCOPE=device asks for a
        // device-scope release instead of the default system-scope fence (measurement knob).
        const unsigned evf = hipEventDisableTiming |
                             (env_str("GOL_EVENT_SCOPE", "system") == "device" ? hipEventReleaseToDevice : 0u);
        HIP_CHECK(hipEventCreateWithFlags(&ev_ready_, evf));
        HIP_CHECK(hipEventCreateWithFlags(&ev_halo_, evf));
        if (cfg_.profile) {
            for (auto* e : {&ev_t0_, &ev_t1_, &ev_t2_, &ev_t3_}) HIP_CHECK(hipEventCreate(e));
        }
        HIP_CHECK(hipMalloc(&d_red_, 2 * sizeof(u64)));
        HIP_CHECK(hipHostMalloc(&h_red_, 2 * sizeof(u64), hipHostMallocDefault));
    }

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
        HIP_CHECK(hipEventRecord(ev_ready_, s_comp_));
    }

    ~HipEngine() override {
        hipStreamSynchronize(s_comp_);
        hipStreamSynchronize(s_comm_);
        destroy_dual_graphs();
        for (auto& kv : sub_plans_) hipFree(kv.second.d);
        for (auto& sb : sub_buf_)
            for (u64* b : sb)
                if (b) hipFree(b);
        if (ev_sub_a_) hipEventDestroy(ev_sub_a_);
        if (ev_sub_b_) hipEventDestroy(ev_sub_b_);
        if (ev_sub_x_) hipEventDestroy(ev_sub_x_);
        for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
        for (auto& kv : plans_) hipFree(kv.second.d);
        for (auto& kv : copies_) {
            hipFree(kv.second.pack);
            hipFree(kv.second.unpack);
        }
        for (auto& v : {&dstage_s_, &dstage_r_})
            for (u64* p : *v) hipFree(p);
        for (auto& v : {&hstage_s_, &hstage_r_})
            for (u64* p : *v) hipHostFree(p);
        for (int i = 0; i < 2; ++i) hipFree(buf_[i]);
        for (void* p : deferred_free_) hipFree(p);
        hipFree(d_red_);
        hipHostFree(h_red_);
        hipEventDestroy(ev_ready_);
        hipEventDestroy(ev_halo_);
        for (auto e : fence_ev_)
            if (e) hipEventDestroy(e);
        for (auto e : {ev_sync_comm_, ev_sync_comp_})
            if (e) hipEventDestroy(e);
        if (cfg_.profile)
            for (auto e : {ev_t0_, ev_t1_, ev_t2_, ev_t3_}) hipEventDestroy(e);
        hipStreamDestroy(s_comp_);
        hipStreamDestroy(s_comm_);
    }

    std::string backend_name() const override { return "hip"; }

    void synchronize() override {
        if (wd_) {  // poll instead of blocking, so asynchronous transport errors surface
            HIP_CHECK(hipEventRecord(ev_sync_comm_ ? ev_sync_comm_ : make_sync_events(), s_comm_));
            HIP_CHECK(hipEventRecord(ev_sync_comp_, s_comp_));
            wait_watched(ev_sync_comm_);
            wait_watched(ev_sync_comp_);
        }
        HIP_CHECK(hipStreamSynchronize(s_comm_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));
    }
    hipEvent_t make_sync_events() {
        HIP_CHECK(hipEventCreateWithFlags(&ev_sync_comm_, hipEventDisableTiming));
        HIP_CHECK(hipEventCreateWithFlags(&ev_sync_comp_, hipEventDisableTiming));
        return ev_sync_comm_;
    }

    std::vector<u64> tile_words() override {
        sync_canonical();
        synchronize();
        std::vector<u64> d((size_t)(L_.h * L_.nw));
        // stream-ordered (never the legacy null stream: in thread mode another rank's engine may be
        // capturing a graph, and a null-stream copy would have to depend on the capturing stream)
        HIP_CHECK(hipMemcpy2DAsync(d.data(), (size_t)L_.nw * 8, buf_[cur_] + L_.index(0, 0), (size_t)L_.pitch * 8,
                                   (size_t)L_.nw * 8, (size_t)L_.h, hipMemcpyDeviceToHost, s_comp_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));
        // device storage is split-format (bits.hpp); the API is natural-order words
        for (i64 r = 0; r < L_.h; ++r)
            for (i64 c = 0; c < L_.nw; ++c) {
                u64& x = d[(size_t)(r * L_.nw + c)];
                x = merge_word(x) & L_.mask(c);
            }
        return d;
    }

    void set_tile_words(const std::vector<u64>& dense) override {
        sub_current_ = false;  // the canonical board is rewritten: sub-tiles reload at the next run()
        canon_stale_ = false;
        if ((i64)dense.size() != L_.h * L_.nw) throw Error("set_tile_words: wrong size");
        synchronize();
        std::vector<u64> m = dense;
        for (i64 r = 0; r < L_.h; ++r)
            for (i64 c = 0; c < L_.nw; ++c) {
                u64& x = m[(size_t)(r * L_.nw + c)];
                x = split_word(x & L_.mask(c));
            }
        HIP_CHECK(hipMemcpy2DAsync(buf_[cur_] + L_.index(0, 0), (size_t)L_.pitch * 8, m.data(), (size_t)L_.nw * 8,
                                   (size_t)L_.nw * 8, (size_t)L_.h, hipMemcpyHostToDevice, s_comp_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));  // m is pageable and goes out of scope
        post(buf_[cur_], s_comp_);
        mark_ready();
        synchronize();
    }

    std::pair<u64, u64> local_reduce() override {
        sync_canonical();
        HIP_CHECK(hipMemsetAsync(d_red_, 0, 2 * sizeof(u64), s_comp_));
        hipk::launch_reduce_board(buf_[cur_], L_, g_.row0, g_.word0(), g_.global_words(), d_red_, s_comp_);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(h_red_, d_red_, 2 * sizeof(u64), hipMemcpyDeviceToHost, s_comp_));
        HIP_CHECK(hipStreamSynchronize(s_comp_));
        return {h_red_[0], h_red_[1]};
    }

    // Graph shape of run(): m supersteps of k generations per replay; false when run() stays eager.
    bool graph_shape(int& k, int& m) {
        if (!cfg_.graph || cfg_.profile) return false;
        // Sub-tile supersteps are not captured as a whole: captured with their fork/join across two
        // streams they replayed slower than eager launches on MI355X / ROCm 7.2 (32768^2: 14.2 vs
        // 12.8 us/gen over 20 generations, 13.0 vs 10.4 over 256; profiles/short_run_probe.txt).
        // A single-stream graph per half and superstep is available (GOL_SUBTILE_GRAPHS=1), also slower.
        if (dual_) return false;
        k = cfg_.compat ? 1 : superstep_depth();
        m = cfg_.graph_supersteps;
        if (m <= 0) m = k >= 8 ? 16 : 32;
        m += m & 1;  // even: the graph returns to the same buffer parity
        bool local = cfg_.compat || halo_items(k).empty();
        if (!local && !device_transport_) return false;  // host-staged exchange cannot be captured
        // RCCL inside captured graphs is opt-in: with R-deep supersteps (hundreds of us each) the
        // eager launch cost is negligible, and an eager exchange keeps RCCL's own error handling.
        if (!local && !cfg_.graph_rccl) return false;
        return true;
    }

    // Replay shapes {m supersteps of k, then one superstep of rem < k generations}, largest first:
    // the run-length hint as ONE graph (its whole superstep count, at most 256, plus its remainder:
    // the driver's 20-generation bench is a single replay), then M, 4 and 1 supersteps, then the
    // hint's remainder alone.  Every graph boundary costs ~8.5 us of GPU idle (8192^2 x 1000 through
    // the CLI: 5 boundaries, 3% of the run).
    struct Shape {
        int m, rem;
    };
    std::vector<Shape> graph_ladder(int k, int M) const {
        std::vector<Shape> v;
        const u64 hm = std::min<u64>(cfg_.run_hint / (u64)std::max(1, k), 256);
        const int hr = cfg_.compat || cfg_.run_hint / (u64)std::max(1, k) > 256 ? 0 : (int)(cfg_.run_hint % (u64)k);
        if (hm > 0 && hm + (hr > 0) > 1) v.push_back({(int)hm, hr});
        for (int m : {M, 4, 1})
            if (m <= M && !(m == (int)hm && hr == 0)) v.push_back({m, 0});
        if (hr > 0) v.push_back({0, hr});
        std::sort(v.begin(), v.end(), [&](const Shape& a, const Shape& b) {
            return (u64)a.m * k + a.rem > (u64)b.m * k + b.rem;
        });
        return v;
    }

    // Buffer parity of the captured (one-tile) mode.
    int par() const { return cur_; }
    void set_par(int p) { cur_ = p; }

    // Capture and instantiate the replay graphs at init, so no timed run() ever pays for
    // stream capture or graph instantiation (a 16-superstep capture costs milliseconds: more than
    // a whole 8192^2 x 1000 run).
    void prewarm_graph() {
        int k = 0, M = 0;
        if (!graph_shape(k, M)) return;
        for (const Shape& sh : graph_ladder(k, M)) {
            // both parities: a remainder graph of odd pass count leaves the other one current
            for (int p = 0; p < 2; ++p) {
                const int p0 = par();
                set_par(p);
                // upload now: the first launch of an exec otherwise pays for it (in a timed region)
                if (hipGraphExec_t ex = graph_for(k, sh.m, sh.rem)) HIP_CHECK(hipGraphUpload(ex, s_comp_));
                set_par(p0);
            }
        }
        mark_ready();
        synchronize();
    }

    // Replays, largest shape first (eager launches of a superstep cost ~15 us of GPU idle each;
    // graph replays none), every shape captured at init; what no shape covers runs eagerly.
    void run_graphed(u64& generations) {
        int k = 0, M = 0;
        if (!graph_shape(k, M)) return;
        for (const Shape& sh : graph_ladder(k, M)) {
            const u64 per = (u64)sh.m * (u64)k + (u64)sh.rem;
            while (generations >= per && graph_ok_) {
                hipGraphExec_t exec = graph_for(k, sh.m, sh.rem);
                if (!exec) return;
                replay(exec, k, sh.m, sh.rem);
                generations -= per;
            }
        }
    }

    void replay(hipGraphExec_t exec, int k, int m, int rem) {
        const u64 per = (u64)m * (u64)k + (u64)rem;
        maybe_inject_fault();
        {
            trace::Range r("gol.graph_launch");
            HIP_CHECK(hipGraphLaunch(exec, s_comp_));
        }
        set_par(par() ^ graph_flip(k, m, rem));
        // Events recorded during capture are not re-recorded by replays: re-mark them after
        // the graph so later eager supersteps (and the comm stream) wait for its work.
        mark_ready();
        gen_ += per;
        stats_.generations += per;
        stats_.supersteps += (u64)m + (rem > 0);
        stats_.graph_launches += 1;
        progress("graph");
    }
    // Buffer-parity flip of a shape (one flip per kernel pass).
    int graph_flip(int k, int m, int rem) {
        size_t n = pass_depths(k).size() * (size_t)m;
        if (rem) n += pass_depths(rem).size();
        return (int)(n & 1);
    }

    void run(u64 generations) override {
        Armed armed(wd_.get());
        if (dual_ && !sub_current_) {
            // canonical board -> sub-tiles (interior rows), unless the sub-tiles already hold the
            // board (consecutive run() calls keep it in the halves; readers sync it back lazily)
            for (int s = 0; s < 2; ++s)
                dual_copy(sub_rows(s, sub_cur_, 0), buf_[cur_] + L_.index(sub_r0_[s], -1), rows_bytes(s, sub_L_[s].h));
            // both halves' first superstep waits for the copy (each waits on the other's "done" event)
            HIP_CHECK(hipEventRecord(ev_sub_a_, s_comp_));
            HIP_CHECK(hipEventRecord(ev_sub_b_, s_comp_));
            sub_current_ = true;
        }
        run_graphed(generations);
        Engine::run(generations);
        if (dual_) canon_stale_ = true;  // copied back by the next reader (sync_canonical)
    }

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
        return want && !two_d() && !cfg_.compat && !cfg_.profile && !cfg_.force_split && !wd_ && L_.aligned() &&
               (halo_items(L_.R).empty() || device_transport_) && cfg_.kernel != "lds" && cfg_.kernel != "tile";
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

    void setup_dual() {
        if (sub_buf_[0][0]) return;
        const i64 h0 = L_.h / 2;
        sub_r0_[0] = 0;
        sub_r0_[1] = h0;
        for (int s = 0; s < 2; ++s) {
            const i64 hs = s == 0 ? h0 : L_.h - h0;
            sub_L_[s] = Layout(hs, L_.w, L_.R);
            const size_t bytes = (size_t)(sub_L_[s].words() + hipk::kSlackRows * sub_L_[s].pitch) * 8;
            for (int i = 0; i < 3; ++i) {
                HIP_CHECK(hipMalloc(&sub_buf_[s][i], bytes));
                HIP_CHECK(hipMemsetAsync(sub_buf_[s][i], 0, bytes, s_comp_));
            }
        }
        if (!ev_sub_a_) {
            HIP_CHECK(hipEventCreateWithFlags(&ev_sub_a_, hipEventDisableTiming));
            HIP_CHECK(hipEventCreateWithFlags(&ev_sub_b_, hipEventDisableTiming));
            HIP_CHECK(hipEventCreateWithFlags(&ev_sub_x_, hipEventDisableTiming));
        }
        HIP_CHECK(hipStreamSynchronize(s_comp_));
    }
    // Free the sub-tile buffers, plans and copy lists (the measurement chose one tile).
    void teardown_dual() {
        synchronize();
        destroy_dual_graphs();
        for (auto& kv : sub_plans_) hipFree(kv.second.d);
        sub_plans_.clear();
        for (auto& sb : sub_buf_)
            for (u64*& b : sb) {
                if (b) hipFree(b);
                b = nullptr;
            }
        dual_ = false;
        sub_current_ = canon_stale_ = false;
    }
    // Plans and copy lists of a k-generation sub-tile superstep (built before any capture).
    void prepare_dual(int k) {
        const std::vector<int>& ps = pass_depths(k);
        for (size_t j = 0; j < ps.size(); ++j)
            for (int s = 0; s < 2; ++s) sub_plan(s, ps[j], ext_after(ps, j));
    }
    void destroy_dual_graphs() {
        for (auto& kv : dual_graphs_) hipGraphExecDestroy(kv.second);
        dual_graphs_.clear();
    }

    const DevPlan& sub_plan(int s, int k, i64 e) {
        const int key = (s * 100000 + (int)e * 100 + k);
        auto it = sub_plans_.find(key);
        if (it != sub_plans_.end()) return it->second;
        const Layout& L = sub_L_[s];
        std::vector<Region> rg = {{-e, L.h + e, 0, L.nw}};
        i64 bpc = hipk::step_blocks_per_cu(k, sub_flags());
        // waves/SIMD each half's plan is sized for: two concurrent halves fill the SIMDs between
        // them, so 2-wave plans (taller segments, less halo) measured best (kbench: 9.85 vs 10.11
        // us/gen at 32768^2); GOL_SUB_OCC overrides (0 = the single-tile tuned occupancy)
        // (at the temporal pass depth; shallower passes are memory bound and want every resident
        // wave: profiles/kb_depth_sweep.txt)
        if (k >= tdepth_) {
            if (cfg_.sub_occ > 0)
                bpc = std::min<i64>(bpc, cfg_.sub_occ);
            else if (occ_ > 0)
                bpc = std::min<i64>(bpc, occ_);
        }
        const i64 rows = balanced_rows_per_chunk(rg, L.nw, L.h, k, bpc * kWavesPerBlock * cus_, 2 * (i64)k, true);
        DevPlan p;
        std::vector<LaneDesc> lanes = build_plan(rg, L.nw, L.h, rows, k, true, &p.st, kWavesPerBlock, cfg_.plan_xcds);
        const std::string bad = validate_plan(lanes, L.nw, L.h, L.R, k, false);
        if (!bad.empty()) throw Error(strprintf("refusing to launch an unsafe sub-tile plan: %s", bad.c_str()));
        p.waves = (i64)lanes.size() / kWaveLanes;
        p.rows = rows;
        HIP_CHECK(hipMalloc(&p.d, lanes.size() * sizeof(LaneDesc)));
        upload(p.d, lanes.data(), lanes.size() * sizeof(LaneDesc));
        return sub_plans_.emplace(key, p).first->second;
    }

    u32 sub_flags() const { return step_flags() & ~hipk::STEP_WRAP_Y; }  // sub-tiles always have ghost rows

    // rows [r0, r0 + n) of sub-tile s in its buffer `par` (0..2; full pitch, contiguous)
    u64* sub_rows(int s, int par, i64 r0) { return sub_buf_[s][par] + sub_L_[s].index(r0, -1); }
    size_t rows_bytes(int s, i64 n) const { return (size_t)(n * sub_L_[s].pitch) * 8; }

    void dual_copy(u64* dst, const u64* src, size_t bytes) {
        HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s_comp_));
    }

    // Both halves done -> the canonical buffer (before anything reads it).
    void sync_canonical() {
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
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) HIP_CHECK(q);
        HIP_CHECK(hipStreamWaitEvent(s, ev, 0));
    }

    // One sub-tile superstep: sub-tile 0 on the compute stream, 1 on the second stream.
    void dual_superstep(int k) {
        prepare_dual(k);
        const int p = sub_cur_;
        const int a = (p + 1) % 3, b = (p + 2) % 3;  // the passes alternate a, b, a, ... (never p)
        const i64 h1 = sub_L_[1].h;
        wait_pending(s_comp_, ev_sub_b_);  // half 1's previous superstep is done
        if (!self_y()) {
            // the one-tile engine's canonical messages (Engine::halo_items, 1-D): N then S
            std::vector<Message> sends, recvs;
            sends.push_back({g_.nbr[DIR_N], sub_rows(0, p, 0), rows_bytes(0, k)});
            recvs.push_back({g_.nbr[DIR_S], sub_rows(1, p, h1), rows_bytes(1, k)});
            sends.push_back({g_.nbr[DIR_S], sub_rows(1, p, h1 - k), rows_bytes(1, k)});
            recvs.push_back({g_.nbr[DIR_N], sub_rows(0, p, -k), rows_bytes(0, k)});
            t_->exchange(sends, recvs, (void*)s_comp_);
            stats_.exchanges += 1;
            stats_.halo_bytes += (u64)(rows_bytes(0, k) + rows_bytes(1, k));
            HIP_CHECK(hipEventRecord(ev_sub_x_, s_comp_));  // also implies half 0's previous superstep
            HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_sub_x_, 0));
        } else {
            wait_pending(s_comm_, ev_sub_a_);  // half 0's previous superstep is done
        }
        // Each half's passes: eager launches on its stream, alternating between the halves (pass j
        // of half 0, pass j of half 1, ...: issued half by half, the second stream's first kernel
        // started ~20 us after the first's, three host launches later, and the superstep ended on one
        // half's lone tail; kernel traces of the driver's 20-generation bench), or
        // (GOL_SUBTILE_GRAPHS=1) one replay per half of a graph captured at init per half, start
        // buffer and depth.  The cross-half order stays in the events around them.
        hipGraphExec_t gx[2] = {dual_graph(0, p, k), dual_graph(1, p, k)};
        if (gx[0] && gx[1]) {
            for (int s = 0; s < 2; ++s) HIP_CHECK(hipGraphLaunch(gx[s], s ? s_comm_ : s_comp_));
            stats_.graph_launches += 2;
        } else {
            const int np = (int)pass_depths(k).size();
            for (int j = 0; j < np; ++j)
                for (int s = 0; s < 2; ++s) launch_half(s, p, k, s ? s_comm_ : s_comp_, j);
        }
        HIP_CHECK(hipEventRecord(ev_sub_a_, s_comp_));
        HIP_CHECK(hipEventRecord(ev_sub_b_, s_comm_));
        HIP_CHECK(hipGetLastError());
        sub_cur_ = (pass_depths(k).size() % 2) ? a : b;
    }

    // The kernel passes of half s in a superstep of k generations that starts from buffer p (only
    // pass `only` when >= 0).
    void launch_half(int s, int p, int k, hipStream_t st, int only = -1) {
        const std::vector<int>& ps = pass_depths(k);
        const int a = (p + 1) % 3, b = (p + 2) % 3;  // the passes alternate a, b, a, ... (never p)
        const Layout& Ls = sub_L_[s];
        const int o = 1 - s;  // the other half
        hipk::StepParams sp{Ls.pitch, (i32)Ls.h, (i32)Ls.nw, Ls.R, sub_flags()};
        hipk::StepParams sp0 = sp;
        sp0.flags |= hipk::STEP_SEAM;
        // rows above half 0 / below half 1: the rank's ghost rows (exchanged) or, on a torus without
        // neighbours, the other half's far edge; between the halves: the other half's edge
        const bool wrap = self_y();
        const i64 h0 = sub_L_[0].h, h1 = sub_L_[1].h;
        sp0.above = s == 0 ? (wrap ? sub_rows(o, p, sub_L_[o].h) : sub_rows(s, p, 0)) : sub_rows(o, p, h0);
        sp0.below = s == 1 ? (wrap ? sub_rows(o, p, 0) : sub_rows(s, p, h1)) : sub_rows(o, p, 0);
        int q = p;
        for (size_t j = 0; j < ps.size(); ++j) {
            const int dsti = (j % 2 == 0) ? a : b;
            if (only < 0 || (int)j == only) {
                const DevPlan& pl = sub_plan(s, ps[j], ext_after(ps, j));
                hipk::launch_step(ps[j], sub_buf_[s][q], sub_buf_[s][dsti], pl.d, pl.waves, j == 0 ? sp0 : sp, st);
            }
            q = dsti;
        }
    }

    // Graph of launch_half(s, p, k): captured at init only (capture_dual_graphs), nullptr otherwise.
    // Opt-in (GOL_SUBTILE_GRAPHS=1): replayed per half and superstep, these measured slower than the
    // eager launches on MI355X / ROCm 7.2 (32768^2, same box, alternating: 20 generations 13.06-13.23
    // vs 12.75-12.96 us/gen, 2000 generations 10.35 vs 10.24; profiles/subtile_graphs_ab.txt), as did
    // one graph of both halves with fork/join events (see graph_shape).
    bool dual_graphs_on() const { return cfg_.graph && !cfg_.profile && graph_ok_ && env_int("GOL_SUBTILE_GRAPHS", 0) != 0; }
    hipGraphExec_t dual_graph(int s, int p, int k) {
        if (!dual_graphs_on()) return nullptr;
        auto it = dual_graphs_.find((s * 3 + p) * 1000 + k);
        return it == dual_graphs_.end() ? nullptr : it->second;
    }
    void capture_dual_graphs(int k) {
        if (!dual_graphs_on()) return;
        for (int s = 0; s < 2; ++s)
            for (int p = 0; p < 3; ++p) {
                const int key = (s * 3 + p) * 1000 + k;
                if (dual_graphs_.count(key)) continue;
                hipStream_t st = s ? s_comm_ : s_comp_;
                hipGraph_t graph = nullptr;
                hipGraphExec_t exec = nullptr;
                try {
                    HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
                    launch_half(s, p, k, st);
                    HIP_CHECK(hipStreamEndCapture(st, &graph));
                    HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
                    HIP_CHECK(hipGraphDestroy(graph));
                    HIP_CHECK(hipGraphUpload(exec, st));
                } catch (const Error& e) {
                    hipGraph_t g2 = nullptr;
                    hipStreamEndCapture(st, &g2);
                    if (g2) hipGraphDestroy(g2);
                    hipGetLastError();
                    graph_ok_ = false;
                    fprintf(stderr, "[gol] sub-tile graph capture disabled: %s\n", e.what());
                    return;
                }
                dual_graphs_[key] = exec;
            }
    }

    const DevPlan& full_plan_stats() {
        const int R = superstep_depth();
        return plan(0, pass_depths(R)[0], ext_after(pass_depths(R), 0));
    }

    // A one-tile rank without neighbours (nothing to exchange) cuts its supersteps at the largest
    // multiple of the tuned pass depth within R, so none ends with a short pass (8192^2: tile passes
    // of 24 in 32-generation supersteps ran 24 + 8, and an 8-generation tile pass is 27% slower per
    // generation).  With neighbours every rank keeps R: the exchanges must match.
    int superstep_depth() const override {
        if (dual_ || !tuned_ || cfg_.compat || kdepth_ <= 0 || kdepth_ >= L_.R || !halo_items(L_.R).empty())
            return L_.R;
        return (L_.R / kdepth_) * kdepth_;
    }

   protected:
    void do_init(const PatternSpec& p) override {
        sub_current_ = false;
        canon_stale_ = false;
        synchronize();
        for (int i = 0; i < 2; ++i) HIP_CHECK(hipMemsetAsync(buf_[i], 0, alloc_bytes_, s_comp_));
        hipk::InitParams ip{g_.row0, g_.word0(), g_.global_words(), p.seed,
                            p.fill == Fill::Ones ? 1 : (p.fill == Fill::Random ? 2 : 0)};
        cur_ = 0;
        if (p.fill != Fill::Zero) hipk::launch_init_fill(buf_[cur_], L_, ip, s_comp_);
        std::vector<i64> cells;
        for (const auto& rc : p.cells) {
            i64 r = rc.first - g_.row0, c = rc.second - g_.col0;
            if (r < 0 || r >= L_.h || c < 0 || c >= L_.w) continue;
            cells.push_back(r);
            cells.push_back(c);
        }
        i64* dcells = nullptr;
        if (!cells.empty()) {
            HIP_CHECK(hipMalloc(&dcells, cells.size() * sizeof(i64)));
            HIP_CHECK(hipMemcpyAsync(dcells, cells.data(), cells.size() * sizeof(i64), hipMemcpyHostToDevice, s_comp_));
            hipk::launch_set_cells(buf_[cur_], L_, dcells, (i64)cells.size() / 2, s_comp_);
        }
        post(buf_[cur_], s_comp_);
        HIP_CHECK(hipGetLastError());
        mark_ready();
        synchronize();
        if (dcells) deferred_free_.push_back(dcells);  // hipFree may synchronise the whole device
        if (!tuned_) {
            if (cfg_.kernel == "auto") autotune_kernel();
            choose_schedule();  // collective when ranks have neighbours
            measure_pass_costs();
            tuned_ = true;
            passes_.clear();  // the pass cuts may depend on the tuned kernel (pass_depths)
            // The comm stream waits on the compute stream's ready event only in the split
            // schedule (and the forced-split measurement mode).  The full schedule
            // exchanges on the compute stream itself: recording the event there every superstep
            // only idles the GPU (~15 us per record, a release fence).  GOL_READY_EVENTS=always
            // restores the record (measurement knob).
            events_needed_ = cfg_.force_split || (split_ && !halo_items(L_.R).empty()) ||
                             env_str("GOL_READY_EVENTS", "") == "always";
        }
        stats_.kernel = split_ ? kern_[1] + "+boundary:" + kern_[2] : kern_[0];
        stats_.schedule = split_ ? "split" : (halo_items(L_.R).empty() ? "local" : "full");
        if (dual_) stats_.schedule += "+subtiles2";
        stats_.kernel_depth = kdepth_;
        stats_.tile_waves = cfg_.tile_waves;
        std::string tn;
        for (const auto& kv : tune_ms_) tn += strprintf("%s%s=%.3fus/gen", tn.empty() ? "" : " ", kv.first.c_str(), kv.second * 1e3);
        for (const auto& kv : sched_us_)
            tn += strprintf("%ssched:%s=%.3fus/gen", tn.empty() ? "" : " ", kv.first.c_str(), kv.second);
        for (const auto& kv : pass_us_) tn += strprintf("%spass%d=%.1fus", tn.empty() ? "" : " ", kv.first, kv.second);
        stats_.tuning = tn;
        // Build the plans of the supersteps the runs will use now (the full superstep and the
        // remainder of the hinted run length), so neither graph capture nor a hinted timed loop
        // builds or uploads a plan.  Other remainders are built on first use.
        for (int k : init_depths()) {
            if (dual_) {
                prepare_dual(k);
                capture_dual_graphs(k);
            } else {
                prepare(k);
            }
        }
        prewarm_graph();
        if (dual_) {
            // One scratch superstep of each prepared depth (the halves are reloaded from the board at
            // the next run): the first launch of a kernel variant loads its code object, ~20 us that
            // a short timed run would otherwise pay (the seam-reading first-pass kernels run in no
            // tuning step).  Identical on every rank: the exchanges match.
            for (int k : init_depths()) dual_superstep(k);
            sub_current_ = false;
            synchronize();
            stats_.exchanges = 0;
            stats_.halo_bytes = 0;
            stats_.graph_launches = 0;
        }
        spin_up();  // init ends with the GPU at its steady clock (plan building and captures idle it)
        const DevPlan& fp = full_plan_stats();
        stats_.plan_waves = fp.waves;
        stats_.lane_efficiency =
            fp.st.lane_rows ? (double)fp.st.out_words / (double)fp.st.lane_rows : 0.0;
    }

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

    void tile_superstep(int k) {
        const std::vector<int>& ps = pass_depths(k);
        first_pass(k, ps[0], ext_after(ps, 0), split_);
        cur_ ^= 1;
        for (size_t j = 1; j < ps.size(); ++j) {
            // later passes need no halo: the ghost rows computed by the earlier passes carry the
            // neighbours' cells forward (communication-avoiding deep halos)
            const i64 e = ext_after(ps, j);
            launch(0, ps[j], e, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
            post(buf_[cur_ ^ 1], s_comp_, e);
            cur_ ^= 1;
        }
        if (ps.size() > 1) mark_ready();  // the next exchange reads what the last pass wrote
    }

    // Kernel passes of a superstep of k generations.  Once the pass costs are measured
    // (measure_pass_costs), the cheapest cut over the instantiated depths <= K; before that (and with
    // an explicit GOL_KERNEL_DEPTH) the fewest passes of at most K with depths as equal as possible
    // (20 = 7 + 7 + 6, not 8 + 8 + 4).  A pass streams the board through HBM once whatever its
    // depth, so shallow passes cost nearly as much as deep ones (32768^2: ~70-80 us for any depth
    // <= 6, ~90 us at 8; profiles/kb_depth_sweep.txt).
    const std::vector<int>& pass_depths(int k) {
        const int key = k + (dual_ ? (1 << 20) : 0);
        auto it = passes_.find(key);
        if (it != passes_.end()) return it->second;
        // every kind may be temporal, unless only the (any-depth) tile kernel runs; sub-tiles always
        // run the temporal kernel at its own depth
        const bool any_depth = !dual_ && (cfg_.kernel == "tile" || (tuned_ && !split_ && tile_kernel(0)));
        auto ok = [&](int d) { return any_depth || hipk::step_depth_supported(d); };
        const int K = std::max(1, dual_ ? tdepth_ : kdepth_);
        std::vector<int> ps;
        if (tuned_ && !pass_us_.empty() && !any_depth) {
            // cheapest cut by the measured per-depth pass times (dynamic programming over k)
            std::vector<double> best((size_t)k + 1, 1e300);
            std::vector<int> pick((size_t)k + 1, 0);
            best[0] = 0;
            for (int x = 1; x <= k; ++x)
                for (const auto& dc : pass_us_)
                    if (dc.first <= x && best[(size_t)(x - dc.first)] + dc.second < best[(size_t)x]) {
                        best[(size_t)x] = best[(size_t)(x - dc.first)] + dc.second;
                        pick[(size_t)x] = dc.first;
                    }
            for (int x = k; x > 0; x -= pick[(size_t)x]) ps.push_back(pick[(size_t)x]);
            std::sort(ps.begin(), ps.end(), std::greater<int>());
            return passes_.emplace(key, ps).first->second;
        }
        const int n = (k + K - 1) / K;
        bool balanced = true;
        for (int j = 0; j < n; ++j) {
            const int d = k / n + (j < k % n ? 1 : 0);
            if (!ok(d)) balanced = false;
            ps.push_back(d);
        }
        if (!balanced) {  // greedy over the instantiated depths
            ps.clear();
            for (int left = k; left > 0;) {
                int d = std::min(left, K);
                if (!any_depth) d = supported_kernel_depth(d);
                ps.push_back(d);
                left -= d;
            }
        }
        return passes_.emplace(key, ps).first->second;
    }
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

    // Exchange the kx-deep halo and run the first kernel pass (depth kp, output rows extended by e
    // beyond the tile): buf[cur] -> buf[cur^1]; the caller flips the parity.  `split`: interior +
    // boundary bands with the exchange overlapped (else exchange, then one full-region kernel).
    void first_pass(int kx, int kp, i64 e, bool split) {
        prepare(kx);
        u64* src = buf_[cur_];
        u64* dst = buf_[cur_ ^ 1];
        const std::vector<HaloItem>& items = items_for(kx);
        const bool prof = cfg_.profile;
        if (cfg_.compat || (items.empty() && !cfg_.force_split)) {
            if (prof) HIP_CHECK(hipEventRecord(ev_t2_, s_comp_));
            launch(0, kp, e, src, dst, s_comp_);
            post(dst, s_comp_, e);
            if (prof) {
                HIP_CHECK(hipEventRecord(ev_t3_, s_comp_));
                HIP_CHECK(hipEventSynchronize(ev_t3_));
                float ms = 0;
                HIP_CHECK(hipEventElapsedTime(&ms, ev_t2_, ev_t3_));
                stats_.t_compute_ms += ms;
            }
        } else if (split) {
            if (items.empty()) {
                // GOL_FORCE_SPLIT on a rank without neighbours: the multi-GPU stream structure
                // with an empty exchange (measures the split schedule's own cost on one GPU)
                HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_ready_, 0));
                HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
                launch(1, kp, 0, src, dst, s_comp_);
            } else if (device_transport_) {
                HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_ready_, 0));
                if (prof) HIP_CHECK(hipEventRecord(ev_t0_, s_comm_));
                exchange_device(kx, items, cur_, s_comm_);
                if (prof) HIP_CHECK(hipEventRecord(ev_t1_, s_comm_));
                HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
                if (prof) HIP_CHECK(hipEventRecord(ev_t2_, s_comp_));
                launch(1, kp, 0, src, dst, s_comp_);
            } else {
                if (prof) HIP_CHECK(hipEventRecord(ev_t2_, s_comp_));
                launch(1, kp, 0, src, dst, s_comp_);  // interior first: runs while the host exchanges
                HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_ready_, 0));
                if (prof) HIP_CHECK(hipEventRecord(ev_t0_, s_comm_));
                exchange_staged(kx, items, cur_, s_comm_);
                if (prof) HIP_CHECK(hipEventRecord(ev_t1_, s_comm_));
                HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
            }
            HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_halo_, 0));
            launch(2, kp, e, src, dst, s_comp_);
            post(dst, s_comp_, e);
            if (prof) record_profile(true);
        } else {
            if (prof) HIP_CHECK(hipEventRecord(ev_t0_, s_comp_));
            if (device_transport_)
                exchange_device(kx, items, cur_, s_comp_);
            else
                exchange_staged(kx, items, cur_, s_comp_);
            if (prof) {
                HIP_CHECK(hipEventRecord(ev_t1_, s_comp_));
                HIP_CHECK(hipEventRecord(ev_t2_, s_comp_));
            }
            launch(0, kp, e, src, dst, s_comp_);
            post(dst, s_comp_, e);
            if (prof) record_profile(true);
        }
        mark_ready();
    }

    // Bring the GPU to its steady clock before anything is timed.  From idle, sclk ramps up over
    // the first ~20-30 ms of load (measured on MI355X: 32768^2 passes shrink from ~97 to ~87 us
    // while rocm-smi shows sclk rising to 2.4 GHz), which would bias the kernel autotune towards
    // whichever candidate runs last and make the first generations of a run slower than the rest.
    // The full-board kernel runs on the scratch buffer (the board is untouched) for GOL_SPINUP_MS
    // (default 100 ms for boards of >= 2^24 cells, 20 ms below; 0 = off).
    void spin_up() {
        const bool big = (double)L_.h * (double)L_.w >= (double)(1 << 24);
        const double budget_ms = (double)env_int("GOL_SPINUP_MS", big ? 100 : 20);
        if (budget_ms <= 0 || cfg_.compat || kernel_ == "lds") return;
        const std::string saved = kern_[0];
        if (cfg_.kernel != "tile") kern_[0] = "temporal";  // the register kernel runs on any board
        const int k = tile_kernel(0) ? kdepth_ : supported_kernel_depth(std::min(kdepth_, hipk::max_step_depth()));
        const auto t0 = std::chrono::steady_clock::now();
        for (int it = 0; it < 100000; ++it) {
            for (int j = 0; j < 4; ++j) launch(0, k, 0, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
            HIP_CHECK(hipStreamSynchronize(s_comp_));
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (ms >= budget_ms) break;
        }
        kern_[0] = saved;
    }

    // Per-depth pass times of the chosen mode (temporal kernel: one tile, or the two halves on two
    // streams without joins between passes, as inside a superstep), for the pass cuts of supersteps
    // (pass_depths).  Measured rather than modelled: the cost is an HBM streaming floor plus the
    // VALU work of the depth, and code generation differs per depth (32768^2 one tile: depth 7 is
    // slower per pass than depth 8; profiles/kb_depth_sweep.txt).  Rank-local: the cut only changes
    // kernel passes, never the exchanges.
    void measure_pass_costs() {
        pass_us_.clear();
        if (cfg_.compat || cfg_.kernel_depth > 0 || kernel_ == "lds" || (!dual_ && tile_kernel(0))) return;
        const int K = dual_ ? tdepth_ : kdepth_;
        std::vector<int> ds;
        for (int d = 1; d <= K; ++d)
            if (hipk::step_depth_supported(d)) ds.push_back(d);
        if (ds.size() < 2) return;
        for (int d : ds) {  // every plan first: plan building idles the GPU and drops its clock
            if (dual_) {
                sub_plan(0, d, 0);
                sub_plan(1, d, 0);
            } else {
                plan(0, d, 0);
            }
        }
        hipEvent_t e0, e1;
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
        spin_up();
        const int reps = 4;
        std::map<int, double> best;
        for (int round = 0; round < 3; ++round)
            for (int d : ds) {
                HIP_CHECK(hipEventRecord(e0, s_comp_));
                if (dual_) {
                    HIP_CHECK(hipStreamWaitEvent(s_comm_, e0, 0));
                    for (int i = 0; i < reps; ++i)
                        for (int sub = 0; sub < 2; ++sub) {
                            const DevPlan& pl = sub_plan(sub, d, 0);
                            const Layout& Ls = sub_L_[sub];
                            hipk::StepParams sp{Ls.pitch, (i32)Ls.h, (i32)Ls.nw, Ls.R, sub_flags()};
                            hipk::launch_step(d, sub_buf_[sub][sub_cur_], sub_buf_[sub][(sub_cur_ + 1) % 3], pl.d,
                                              pl.waves, sp, sub ? s_comm_ : s_comp_);
                        }
                    HIP_CHECK(hipEventRecord(ev_sub_b_, s_comm_));
                    HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_sub_b_, 0));
                } else {
                    for (int i = 0; i < reps; ++i) launch(0, d, 0, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
                }
                HIP_CHECK(hipEventRecord(e1, s_comp_));
                HIP_CHECK(hipEventSynchronize(e1));
                float ms = 0;
                HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1e3 / reps;
                best[d] = round == 0 ? us : std::min(best[d], us);
            }
        HIP_CHECK(hipEventDestroy(e0));
        HIP_CHECK(hipEventDestroy(e1));
        HIP_CHECK(hipGetLastError());
        pass_us_ = best;
        passes_.clear();
    }

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
    void choose_schedule() {
        const bool nbrs = !halo_items(L_.R).empty();  // identical on every rank (uniform grid)
        std::vector<std::string> cands;
        if (cfg_.force_split || (cfg_.sched == "split" && split_used())) {
            cands = {"split"};
        } else {
            cands.push_back(nbrs ? "full" : "local");
            if (cfg_.sched == "auto" && split_used()) cands.push_back("split");
        }
        bool dual_ok = cfg_.subtiles != 0 && cands[0] != "split" && dual_wanted();
        if (dual_ok) {
            double ok = dual_local_ok() ? 1.0 : 0.0;
            if (t_->size() > 1) ok = t_->allreduce_min(ok);
            dual_ok = ok > 0;
        }
        if (dual_ok) {
            if (cfg_.subtiles == 2)
                cands = {"subtiles"};
            else
                cands.push_back("subtiles");
        }
        std::string pick = cands[0];
        if (cands.size() > 1) {
            const int k = L_.R;
            std::vector<double> best(cands.size(), 1e30);
            spin_up();
            for (int round = 0; round < 3; ++round)
                for (size_t c = 0; c < cands.size(); ++c) {
                    if (round == 0) time_schedule(cands[c], k, 1);  // warm-up: connections, plans
                    synchronize();
                    t_->barrier();
                    const auto t0 = std::chrono::steady_clock::now();
                    time_schedule(cands[c], k, kSchedReps);
                    synchronize();
                    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    best[c] = std::min(best[c], t_->allreduce_max(dt) * 1e6 / (kSchedReps * k));
                }
            size_t bi = 0;
            for (size_t c = 0; c < cands.size(); ++c) {
                sched_us_[cands[c]] = best[c];
                if (best[c] < best[bi]) bi = c;
            }
            pick = cands[bi];
            stats_.exchanges = 0;  // the timing exchanges are not part of the run
            stats_.halo_bytes = 0;
        }
        split_ = pick == "split";
        dual_ = pick == "subtiles";
        if (dual_) {
            setup_dual();
            sub_current_ = false;  // the halves hold timing scratch: load the board at the next run
        } else if (sub_buf_[0][0]) {
            teardown_dual();
        }
        passes_.clear();
    }

    // `reps` supersteps of k generations of schedule `c` on scratch state (see choose_schedule).
    void time_schedule(const std::string& c, int k, int reps) {
        if (c == "subtiles") {
            setup_dual();
            dual_ = true;
            for (int i = 0; i < reps; ++i) dual_superstep(k);
            dual_ = false;
            return;
        }
        split_ = c == "split";
        const std::vector<int>& ps = pass_depths(k);
        for (int i = 0; i < reps; ++i) {
            first_pass(k, ps[0], ext_after(ps, 0), split_);
            for (size_t j = 1; j < ps.size(); ++j) {
                const i64 e = ext_after(ps, j);
                launch(0, ps[j], e, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
                post(buf_[cur_ ^ 1], s_comp_, e);
            }
            // the next exchange waits for the whole superstep, as in tile_superstep (without this
            // record the timed split schedule overlapped each exchange with the previous superstep's
            // later passes, which a real run cannot: 2.78 timed vs 3.26 us/gen run, 4096 x 32768)
            if (ps.size() > 1) mark_ready();
        }
        split_ = false;
    }

    void do_set_compat_halos(const std::vector<u64>& above, const std::vector<u64>& below) override {
        synchronize();
        for (int i = 0; i < 2; ++i) {
            upload(buf_[i] + L_.index(-1, -1), above.data(), (size_t)L_.pitch * 8);
            upload(buf_[i] + L_.index(L_.h, -1), below.data(), (size_t)L_.pitch * 8);
            if (self_x() && !L_.aligned()) {
                hipk::launch_fill_ghost_cols(buf_[i], L_, -1, 0, s_comp_);
                hipk::launch_fill_ghost_cols(buf_[i], L_, L_.h, L_.h + 1, s_comp_);
            }
        }
        mark_ready();
        synchronize();
    }

    std::vector<u64> read_row(i64 r) override {
        sync_canonical();
        synchronize();
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

    bool tile_kernel(int kind) const { return kern_[kind] == "tile"; }

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

    // GOL_KERNEL=auto: for every plan kind a run uses (full tile; interior + boundary bands when
    // split), time one superstep of each candidate kernel (into the scratch buffer, so the board is
    // untouched) and keep the faster one.  The register pipeline wins on big regions; the
    // LDS-resident tile kernel on small ones — its vertical halo is shared by a whole workgroup and
    // its dependency chains are short, which is what the k-row boundary bands need.
    void autotune_kernel() {
        hipEvent_t e0, e1;
        HIP_CHECK(hipEventCreate(&e0));
        HIP_CHECK(hipEventCreate(&e1));
        // time one pass of kernel `kern` at depth k on plan `kind`; returns ms per generation
        // build_only: construct (and upload) the plan only.  Every plan of a tuning round is built
        // before the GPU is spun up and the kernels are timed: building a tile plan for a large
        // board is ~0.1 s of host work, long enough for the clock to drop again.
        auto time_pass = [&](int kind, const char* kern, int k, bool build_only = false) -> float {
            kern_[kind] = kern;
            if (kern_[kind] == "tile" && (tile_rows_cap(k) < 1 || tile_rounds(kind, k, 0) > kMaxTileRounds))
                return 1e30f;  // LDS tiles only pay off for small regions (docs/PERFORMANCE.md)
            if (kern_[kind] == "temporal" && !hipk::step_depth_supported(k)) return 1e30f;
            if (build_only) {
                plan(kind, k, 0);
                return 0.f;
            }
            const bool tile = kern_[kind] == "tile";
            hipStream_t s = s_comp_;
            launch(kind, k, 0, buf_[cur_], buf_[cur_ ^ 1], s);  // warm-up (and plan build)
            HIP_CHECK(hipEventRecord(e0, s));
            for (int i = 0; i < 3; ++i) launch(kind, k, 0, buf_[cur_], buf_[cur_ ^ 1], s);
            HIP_CHECK(hipEventRecord(e1, s));
            HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0;
            HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            const float per_gen = ms / 3 / (float)k;
            const std::string key = tile ? strprintf("%d:%s@%dx%dw", kind, kern, k, cfg_.tile_waves)
                                         : (occ_ ? strprintf("%d:%s@%d/%dw", kind, kern, k, occ_)
                                                 : strprintf("%d:%s@%d", kind, kern, k));
            auto it = tune_ms_.find(key);
            tune_ms_[key] = it == tune_ms_.end() ? per_gen : std::min(it->second, per_gen);  // best round
            return per_gen;
        };
        // full-tile kernel and pass depth: the register pipeline at the auto depth, the LDS tile
        // kernel at that depth and (deeper passes amortise its staging) twice that depth
        // The tile workgroup size (the threadsPerBlock hint, or GOL_TILE_WAVES) is a candidate
        // dimension too unless GOL_TILE_WAVES fixed it: the measured default, 8 waves, is also tried.
        struct Cand {
            const char* kern;
            int k, nw;
            int occ = 0;  // temporal: waves per SIMD of the plan (0 = full occupancy)
        };
        const int k0 = cfg_.compat ? 1 : kdepth_;
        const int nw0 = cfg_.tile_waves;
        std::vector<int> nws = {nw0};
        if (cfg_.tune_tile_waves && nw0 != 8) nws.push_back(8);
        std::vector<Cand> cands = {{"temporal", k0, nw0}};
        // fewer, taller temporal waves (2 per SIMD instead of 3) for small tiles: less vertical halo
        if (!cfg_.compat && cfg_.rows_per_wave <= 0 && cfg_.waves_target <= 0 &&
            hipk::step_blocks_per_cu(k0, step_flags()) > 2)
            cands.push_back({"temporal", k0, nw0, 2});
        // Deeper tile passes: 2 k0 always; 3 k0 and 4 k0 (any depth) when the full-tile plan is the
        // only kind a superstep runs (no split), so the passes need not suit the register kernel.
        // 8192^2 on one GPU: tile@16 1.51-1.52, tile@24 1.475, tile@32 1.496 us/gen.
        std::vector<int> kts = {k0};
        if (!cfg_.compat && cfg_.kernel_depth == 0) {
            const int kmax = std::min(L_.R, 32);
            const int k2 = supported_kernel_depth(std::min(2 * k0, kmax));
            if (k2 > k0) kts.push_back(k2);
            if (!split_used())
                for (int m = 3; m <= 4 && m * k0 <= kmax; ++m) kts.push_back(m * k0);
        }
        for (int nw : nws)
            for (int k : kts) cands.push_back({"tile", k, nw});
        for (const auto& c : cands) {
            occ_ = c.occ;
            time_pass(0, c.kern, c.k, true);
        }
        spin_up();
        // Three interleaved rounds, best of each candidate: some candidates are within 1-2% of each
        // other (32768^2: the 3- and 2-waves/SIMD plans), and one 3-pass sample picks on noise.
        std::vector<float> tbest(cands.size(), 1e30f);
        for (int round = 0; round < 3; ++round)
            for (size_t i = 0; i < cands.size(); ++i) {
                cfg_.tile_waves = cands[i].nw;
                occ_ = cands[i].occ;
                tbest[i] = std::min(tbest[i], time_pass(0, cands[i].kern, cands[i].k));
            }
        float best = 1e30f;
        Cand pick = cands[0];
        for (size_t i = 0; i < cands.size(); ++i)
            if (tbest[i] < best) {
                best = tbest[i];
                pick = cands[i];
            }
        kern_[0] = pick.kern;
        kdepth_ = pick.k;
        cfg_.tile_waves = pick.nw;
        occ_ = pick.occ;
        passes_.clear();
        // interior / boundary plans of split supersteps, at the chosen pass depth
        if (split_used()) {
            for (int kind : {1, 2})
                for (const char* c : {"temporal", "tile"}) time_pass(kind, c, kdepth_, true);
            spin_up();
            for (int kind : {1, 2}) {
                float bk = 1e30f;
                const char* pk = "temporal";
                for (const char* c : {"temporal", "tile"}) {
                    const float t = time_pass(kind, c, kdepth_);
                    if (t < bk) {
                        bk = t;
                        pk = c;
                    }
                }
                kern_[kind] = pk;
            }
        }
        HIP_CHECK(hipEventDestroy(e0));
        HIP_CHECK(hipEventDestroy(e1));
        kernel_ = kern_[0];
    }

    bool can_overlap() const {
        // an interior must exist on EVERY rank (the schedule timing is collective, so the decision
        // uses the smallest strip, not this rank's), and the LDS kernel reads ghost words for every
        // row (2-D needs them)
        if (min_tile_rows() <= 2 * (i64)L_.R) return false;
        if (kernel_ == "lds" && two_d()) return false;
        return true;
    }

    // Output regions of a pass of depth k whose output rows extend e rows beyond the tile (into
    // the ghost rows, 1-D multi-pass supersteps): kind 0 full, 1 interior, 2 boundary bands.
    std::vector<Region> regions(int kind, int k, i64 rem = 0) const {
        const i64 h = L_.h, nw = L_.nw;
        const bool two_d = this->two_d();
        // multi-pass: earlier passes also produce the ghost rows (y neighbours) and the ghost
        // words, columns -1 and nw (x neighbours), that later passes read
        const i64 e = self_y() ? 0 : rem;
        const i64 xe = (!self_x() && rem > 0) ? 1 : 0;
        if (kind == 0 || h <= 2 * (i64)k)
            return kind == 1 ? std::vector<Region>{} : std::vector<Region>{{-e, h + e, -xe, nw + xe}};
        if (kind == 1) {
            if (two_d) return nw > 2 ? std::vector<Region>{{k, h - k, 1, nw - 1}} : std::vector<Region>{};
            return {{k, h - k, 0, nw}};
        }
        std::vector<Region> r = {{-e, k, -xe, nw + xe}, {h - k, h + e, -xe, nw + xe}};
        if (two_d) {
            if (nw > 2) {
                r.push_back({k, h - k, -xe, 1});
                r.push_back({k, h - k, nw - 1, nw + xe});
            } else {
                r.push_back({k, h - k, -xe, nw + xe});
            }
        }
        return r;
    }

    const DevPlan& plan(int kind, int k, i64 e = 0) {
        // plans depend on e only through regions(): rows beyond the tile when y has neighbours,
        // ghost words when x has neighbours (so one plan serves every e of a local rank)
        const i64 ek = self_y() ? (self_x() ? 0 : (e > 0 ? 1 : 0)) : e;
        // tile plans also depend on the workgroup size (the LDS rows a tile may hold)
        const i64 key = ((((i64)occ_ * 2 + (tile_kernel(kind) ? 1 : 0)) * 32 + (tile_kernel(kind) ? cfg_.tile_waves : 0)) * 4 +
                         kind) * 100000 + (i64)ek * 100 + k;
        auto it = plans_.find(key);
        if (it != plans_.end()) return it->second;
        std::vector<Region> rg = regions(kind, k, e);
        DevPlan p;
        i64 rows = cfg_.rows_per_wave;
        if (tile_kernel(kind)) {
            // step_tile: one workgroup per plan wave, one tile per CU per round; rows are capped by
            // the 160 KiB of LDS (2k halo rows + the tile, double-buffered or in place), extra rounds
            // beyond that.  The double-buffered tile is used when one round of tiles fits it (cheaper:
            // no halo copies, one barrier per LDS pass; 8192^2: 1.45 vs 1.65 us/gen), the in-place one
            // (twice the rows) when the double buffer would need more rounds (4096 x 32768: 2.36 vs
            // 2.70, 16384^2: 4.58 vs 4.69; profiles/tile_inplace_ab.txt).  GOL_TILE_INPLACE=0/1 forces.
            const i64 rdb = hipk::tile_max_rows(k, cfg_.tile_waves, step_flags() | tile_bits(false));
            const i64 rip = hipk::tile_max_rows(k, cfg_.tile_waves, step_flags() | tile_bits(true));
            const i64 r1 = balanced_rows_per_chunk(rg, L_.nw, L_.h, k, cus_, 1, xwrap_by_plan());
            bool ip = tile_inplace_ > 0 || (tile_inplace_ < 0 && r1 > rdb && rip > rdb);
            if (tile_inplace_ < 0 && rows > 0) ip = rows > rdb;
            const i64 rmax = ip ? rip : rdb;
            p.tflags = tile_bits(ip);
            if (rmax < 1) throw Error(strprintf("GOL_KERNEL=tile: depth %d leaves no LDS rows", k));
            if (rows > rmax) rows = rmax;
            if (tile_rounds(kind, k, e) > kMaxTileRounds)
                throw Error(strprintf("GOL_KERNEL=tile: this tile needs %lld rounds of LDS tiles; use the temporal "
                                      "kernel for boards this large",
                                      (long long)tile_rounds(kind, k, e)));
            if (rows <= 0) {
                const i64 rounds = ceil_div(r1, rmax);
                rows = rounds <= 1 ? r1
                                   : std::min(rmax, balanced_rows_per_chunk(rg, L_.nw, L_.h, k, rounds * cus_, 1,
                                                                            xwrap_by_plan()));
            }
        } else {
            if (rows <= 0 && cfg_.waves_target > 0)
                rows = choose_rows_per_chunk(rg, k, cfg_.waves_target, 4 * (i64)k);
            if (rows <= 0) {
                // one full round of resident waves (occupancy of this kernel instantiation)
                i64 bpc = hipk::step_blocks_per_cu(k, step_flags());
                // 256-thread blocks per CU = waves per SIMD; the tuned cap applies to the tuned depth
                // only (shallower passes are memory bound and want every resident wave)
                if (occ_ > 0 && k == kdepth_) bpc = std::min<i64>(bpc, occ_);
                const i64 resident = bpc * kWavesPerBlock * cus_;
                rows = balanced_rows_per_chunk(rg, L_.nw, L_.h, k, resident, 2 * (i64)k, xwrap_by_plan());
            }
        }
        std::vector<LaneDesc> lanes = build_plan(rg, L_.nw, L_.h, rows, k, xwrap_by_plan(), &p.st,
                                                 tile_kernel(kind) ? 1 : kWavesPerBlock, cfg_.plan_xcds);
        const std::string bad = validate_plan(lanes, L_.nw, L_.h, L_.R, k, (step_flags() & hipk::STEP_WRAP_Y) != 0);
        if (!bad.empty()) throw Error(strprintf("refusing to launch an unsafe plan (kind %d, k %d, e %lld): %s", kind, k,
                                                (long long)e, bad.c_str()));
        p.waves = (i64)lanes.size() / kWaveLanes;
        p.rows = rows;
        HIP_CHECK(hipMalloc(&p.d, lanes.size() * sizeof(LaneDesc)));
        upload(p.d, lanes.data(), lanes.size() * sizeof(LaneDesc));
        return plans_.emplace(key, p).first->second;
    }

    void launch(int kind, int k, i64 e, const u64* src, u64* dst, hipStream_t s) {
        if (kernel_ == "lds") {
            // full-row bands only (the LDS variant is never split by columns: can_overlap)
            for (const Region& r : regions(kind, 1))
                if (r.c0 == 0) hipk::launch_step_lds(src, dst, L_, r.r0, r.r1, step_flags(), s);
        } else {
            const DevPlan& p = plan(kind, k, e);
            if (p.st.out_words == 0) return;
            hipk::StepParams sp{L_.pitch, (i32)L_.h, (i32)L_.nw, L_.R, step_flags() | p.tflags};
            if (tile_kernel(kind))
                hipk::launch_step_tile(cfg_.tile_waves, k, src, dst, p.d, p.waves, p.rows, sp, s);
            else
                hipk::launch_step(k, src, dst, p.d, p.waves, sp, s);
        }
        HIP_CHECK(hipGetLastError());
    }

    // Ghost words for widths that are not a multiple of 64 when the tile is its own E/W neighbour.
    void post(u64* buf, hipStream_t s, i64 rem = 0) {
        const i64 e = self_y() ? 0 : rem;
        if (self_x() && !L_.aligned()) hipk::launch_fill_ghost_cols(buf, L_, -e, L_.h + e, s);
    }

    // ----- halo exchange -----
    const std::vector<HaloItem>& items_for(int k) {
        auto it = items_.find(k);
        if (it != items_.end()) return it->second;
        return items_.emplace(k, halo_items(k)).first->second;
    }

    void prepare(int k) {
        const std::vector<int>& ps = pass_depths(k);
        plan(0, ps[0], ext_after(ps, 0));
        if (can_overlap()) {
            plan(1, ps[0]);
            plan(2, ps[0], ext_after(ps, 0));
        }
        for (size_t j = 1; j < ps.size(); ++j) plan(0, ps[j], ext_after(ps, j));
        const std::vector<HaloItem>& items = items_for(k);
        if (items.empty()) return;
        // staging buffers sized for the deepest halo (k = R)
        const std::vector<HaloItem>& deep = items_for(L_.R);
        if (dstage_s_.empty()) {
            for (const HaloItem& itm : deep) {
                u64 *ds, *dr, *hs = nullptr, *hr = nullptr;
                HIP_CHECK(hipMalloc(&ds, (size_t)itm.send.count() * 8));
                HIP_CHECK(hipMalloc(&dr, (size_t)itm.recv.count() * 8));
                if (!device_transport_) {
                    HIP_CHECK(hipHostMalloc(&hs, (size_t)itm.send.count() * 8, hipHostMallocDefault));
                    HIP_CHECK(hipHostMalloc(&hr, (size_t)itm.recv.count() * 8, hipHostMallocDefault));
                }
                dstage_s_.push_back(ds);
                dstage_r_.push_back(dr);
                hstage_s_.push_back(hs);
                hstage_r_.push_back(hr);
            }
        }
        for (int parity = 0; parity < 2; ++parity) copies(k, parity);
    }

    const DevCopies& copies(int k, int parity) {
        const int key = k * 2 + parity;
        auto it = copies_.find(key);
        if (it != copies_.end()) return it->second;
        const std::vector<HaloItem>& items = items_for(k);
        std::vector<hipk::CopyDesc> pk, up;
        DevCopies dc;
        u64* b = buf_[parity];
        for (size_t i = 0; i < items.size(); ++i) {
            const HaloItem& itm = items[i];
            if (itm.contiguous) continue;
            pk.push_back({b + L_.index(itm.send.r0, itm.send.c0), dstage_s_[i], L_.pitch, itm.send.words,
                          (i32)itm.send.rows, (i32)itm.send.words});
            up.push_back({dstage_r_[i], b + L_.index(itm.recv.r0, itm.recv.c0), itm.recv.words, L_.pitch,
                          (i32)itm.recv.rows, (i32)itm.recv.words});
            dc.max_pack = std::max(dc.max_pack, itm.send.count());
            dc.max_unpack = std::max(dc.max_unpack, itm.recv.count());
        }
        dc.npack = (int)pk.size();
        dc.nunpack = (int)up.size();
        if (!pk.empty()) {
            HIP_CHECK(hipMalloc(&dc.pack, pk.size() * sizeof(hipk::CopyDesc)));
            upload(dc.pack, pk.data(), pk.size() * sizeof(hipk::CopyDesc));
            HIP_CHECK(hipMalloc(&dc.unpack, up.size() * sizeof(hipk::CopyDesc)));
            upload(dc.unpack, up.data(), up.size() * sizeof(hipk::CopyDesc));
        }
        return copies_.emplace(key, dc).first->second;
    }

    void build_messages(int k, const std::vector<HaloItem>& items, int parity, std::vector<Message>& sends,
                        std::vector<Message>& recvs) {
        (void)k;
        u64* b = buf_[parity];
        for (size_t i = 0; i < items.size(); ++i) {
            const HaloItem& itm = items[i];
            u64* sp = itm.contiguous ? b + L_.index(itm.send.r0, itm.send.c0) : dstage_s_[i];
            u64* rp = itm.contiguous ? b + L_.index(itm.recv.r0, itm.recv.c0) : dstage_r_[i];
            sends.push_back({itm.send_peer, sp, (size_t)itm.send.count() * 8});
            recvs.push_back({itm.recv_peer, rp, (size_t)itm.recv.count() * 8});
        }
    }

    void exchange_device(int k, const std::vector<HaloItem>& items, int parity, hipStream_t s) {
        trace::Range r("gol.exchange_device");
        const DevCopies& dc = copies(k, parity);
        if (dc.npack) hipk::launch_copy_regions(dc.pack, dc.npack, dc.max_pack, s);
        std::vector<Message> sends, recvs;
        build_messages(k, items, parity, sends, recvs);
        t_->exchange(sends, recvs, (void*)s);
        if (dc.nunpack) hipk::launch_copy_regions(dc.unpack, dc.nunpack, dc.max_unpack, s);
        HIP_CHECK(hipGetLastError());
        account(items);
    }

    void exchange_staged(int k, const std::vector<HaloItem>& items, int parity, hipStream_t s) {
        trace::Range r("gol.exchange_staged");
        const DevCopies& dc = copies(k, parity);
        if (dc.npack) hipk::launch_copy_regions(dc.pack, dc.npack, dc.max_pack, s);
        std::vector<Message> dsends, drecvs;
        build_messages(k, items, parity, dsends, drecvs);
        std::vector<Message> hsends, hrecvs;
        for (size_t i = 0; i < items.size(); ++i) {
            HIP_CHECK(hipMemcpyAsync(hstage_s_[i], dsends[i].buf, dsends[i].bytes, hipMemcpyDeviceToHost, s));
            hsends.push_back({dsends[i].peer, hstage_s_[i], dsends[i].bytes});
            hrecvs.push_back({drecvs[i].peer, hstage_r_[i], drecvs[i].bytes});
        }
        HIP_CHECK(hipStreamSynchronize(s));
        t_->exchange_host(hsends, hrecvs);
        for (size_t i = 0; i < items.size(); ++i)
            HIP_CHECK(hipMemcpyAsync(drecvs[i].buf, hstage_r_[i], drecvs[i].bytes, hipMemcpyHostToDevice, s));
        if (dc.nunpack) hipk::launch_copy_regions(dc.unpack, dc.nunpack, dc.max_unpack, s);
        HIP_CHECK(hipGetLastError());
        account(items);
    }

    void account(const std::vector<HaloItem>& items) {
        stats_.exchanges += 1;
        for (const HaloItem& it : items) stats_.halo_bytes += (u64)it.send.count() * 8;
    }

    void record_profile(bool with_exchange) {
        HIP_CHECK(hipEventRecord(ev_t3_, s_comp_));
        HIP_CHECK(hipEventSynchronize(ev_t3_));
        float ms = 0;
        if (with_exchange) {
            HIP_CHECK(hipEventElapsedTime(&ms, ev_t0_, ev_t1_));
            stats_.t_exchange_ms += ms;
        }
        HIP_CHECK(hipEventElapsedTime(&ms, ev_t2_, ev_t3_));
        stats_.t_compute_ms += ms;
    }

    // ----- graphs -----
    // The captured kernels bake in the buffer pointers, so a replay must start at the parity it was
    // captured at (an odd-pass remainder superstep flips it between run() calls).
    i64 graph_key(int k, int m, int rem) const { return (((i64)k * 1000 + m) * 1000 + rem) * 2 + par(); }
    hipGraphExec_t graph_for(int k, int m, int rem) {
        const i64 key = graph_key(k, m, rem);
        auto it = graphs_.find(key);
        if (it != graphs_.end()) return it->second;
        for (int kk : {k, rem}) {
            if (kk <= 0) continue;
            if (dual_)
                prepare_dual(kk);
            else
                prepare(kk);
        }
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
        const int p0 = par();
        try {
            HIP_CHECK(hipStreamBeginCapture(s_comp_, hipStreamCaptureModeRelaxed));
            mark_ready();  // fork points for the comm stream, recorded inside the capture
            for (int i = 0; i < m; ++i) do_superstep(k);
            if (rem) do_superstep(rem);
            HIP_CHECK(hipStreamEndCapture(s_comp_, &graph));
            HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
            HIP_CHECK(hipGraphDestroy(graph));
        } catch (const Error& e) {
            hipGraph_t g2 = nullptr;
            hipStreamEndCapture(s_comp_, &g2);
            if (g2) hipGraphDestroy(g2);
            hipGetLastError();
            set_par(p0);
            graph_ok_ = false;
            fprintf(stderr, "[gol] hipGraph capture disabled: %s\n", e.what());
            mark_ready();
            return nullptr;
        }
        set_par(p0);  // capture does not execute: the replay flips the parity (graph_flip)
        graphs_[key] = exec;
        return exec;
    }

    // ----- watchdog support -----
    // Wait for `ev` without blocking in the driver, so a stuck or failed exchange is noticed: the
    // transport's asynchronous error state is polled while waiting.
    void wait_watched(hipEvent_t ev) {
        for (;;) {
            const hipError_t e = hipEventQuery(ev);
            if (e == hipSuccess) return;
            if (e != hipErrorNotReady) HIP_CHECK(e);
            const std::string ae = t_->async_error();
            if (!ae.empty()) fatal(ae, 5);
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
    // Bounded lookahead: the host runs at most kFenceDepth units (supersteps or graph launches)
    // ahead of the GPU, so watchdog kicks track completed GPU work.
    static constexpr int kFenceDepth = 4;
    void fence() override {
        if (!fence_ev_[0])
            for (auto& e : fence_ev_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_CHECK(hipEventRecord(fence_ev_[fence_i_], s_comp_));
        fence_used_[fence_i_] = true;
        fence_i_ = (fence_i_ + 1) % kFenceDepth;
        if (fence_used_[fence_i_]) wait_watched(fence_ev_[fence_i_]);
    }

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
    int tile_inplace_ = (int)env_int("GOL_TILE_INPLACE", -1);
    int tile_lv_ = (int)env_int("GOL_TILE_LEVELS", 0);  // tile kernel: generations per LDS pass (1, 2, 4; 0 auto)
    bool multipass_ = false;
    std::map<int, std::vector<int>> passes_;
    bool split_ = false;   // superstep schedule: interior/boundary split with overlapped exchange
    std::map<std::string, double> sched_us_;  // choose_schedule: us per generation per candidate
    std::map<int, double> pass_us_;           // measure_pass_costs: us per pass by depth (chosen mode)
    bool tuned_ = false;
    std::map<std::string, float> tune_ms_;
    hipEvent_t fence_ev_[kFenceDepth] = {};
    hipEvent_t ev_sync_comm_ = nullptr, ev_sync_comp_ = nullptr;
    bool fence_used_[kFenceDepth] = {};
    int fence_i_ = 0;
    u64* buf_[2] = {nullptr, nullptr};
    size_t alloc_bytes_ = 0;
    int cur_ = 0;
    hipStream_t s_comp_ = nullptr, s_comm_ = nullptr;
    hipEvent_t ev_ready_ = nullptr, ev_halo_ = nullptr;
    hipEvent_t ev_t0_ = nullptr, ev_t1_ = nullptr, ev_t2_ = nullptr, ev_t3_ = nullptr;
    u64* d_red_ = nullptr;
    u64* h_red_ = nullptr;
    bool device_transport_ = false;
    bool graph_ok_ = true;
    bool events_needed_ = true;  // another stream waits on ev_ready_
    std::vector<void*> deferred_free_;
    std::map<i64, DevPlan> plans_;
    // GOL_SUBTILES=2 state
    bool dual_ = false;
    Layout sub_L_[2];
    i64 sub_r0_[2] = {0, 0};
    u64* sub_buf_[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};
    int sub_cur_ = 0;  // buffer (0..2) holding both halves' current generation
    bool sub_current_ = false;  // the halves hold the current board
    bool canon_stale_ = false;  // buf_[cur_] lags the halves (sync_canonical before reading it)
    std::map<int, DevPlan> sub_plans_;
    std::map<int, hipGraphExec_t> dual_graphs_;  // (half, start buffer, depth) -> launch_half graph
    hipEvent_t ev_sub_a_ = nullptr, ev_sub_b_ = nullptr;  // half 0 / half 1 done with its last superstep
    hipEvent_t ev_sub_x_ = nullptr;                        // the rank's exchange (into both halves) done
    std::map<int, DevCopies> copies_;
    std::map<int, std::vector<HaloItem>> items_;
    std::map<i64, hipGraphExec_t> graphs_;
    std::vector<u64*> dstage_s_, dstage_r_, hstage_s_, hstage_r_;
};

}  // namespace

std::unique_ptr<Engine> make_hip_engine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t) {
    int err = 0;
    if (hip_device_count(&err) <= 0) throw Error("no HIP device available");
    return std::make_unique<HipEngine>(g, c, std::move(t));
}

}  // namespace gol
