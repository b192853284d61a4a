// gol-mi355x: HIP backend of the engine.
//
// Board memory: two bit-packed tiles in HBM (hipMalloc, never managed memory — the reference
// migrates managed pages host<->device every generation, gol-with-cuda.cu:35-51 + gol-main.c:97-100).
// Streams: s_comp (kernels) and s_comm (halo exchange).  A superstep of R generations = one halo
// exchange + R/K kernel passes (the earlier passes also compute the ghost rows/words the later
// ones read).  With neighbours, the first pass runs one of two schedules (chosen by measurement):
//   split:  s_comm:  wait(ev_ready) -> pack (2-D) -> RCCL group send/recv (or host staging) -> unpack -> ev_halo
//           s_comp:  interior kernel -> wait(ev_halo) -> boundary kernel -> later passes -> ev_ready
//           (a one-pass superstep runs its boundary kernel on s_comm after the exchange instead,
//           concurrently with the interior, and joins the streams at the next superstep)
//   full:   s_comp:  exchange -> full-region kernel -> later passes
// With graphs on, G/(m*R) captures of m supersteps (even pass count => parity preserved) are replayed.
//
// The class is declared in hip_engine.hpp (member functions by topic in engine_hip_*.hip).
#include "hip_engine.hpp"

namespace gol {

int hip_device_count(int* err) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (err) *err = (int)e;
    return e == hipSuccess ? n : 0;
}

void hip_set_device(int dev) { HIP_CHECK(hipSetDevice(dev)); }
int hip_try_set_device(int dev) { return (int)hipSetDevice(dev); }

namespace hipeng {

HipEngine::HipEngine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t)
    : Engine(g, c, std::move(t)) {
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
    } else if (kernel_ == "temporal" || kernel_ == "auto" || kernel_ == "resident") {
        // auto: the depth must suit both candidates (instantiated temporal depths)
        K = supported_kernel_depth(std::min(K, hipk::max_step_depth()));
    } else if (kernel_ == "pipe") {
        // GOL_PIPE=nw,L,wg: the step_pipe geometry (default 9,3,2: K = 24)
        const std::string g = env_str("GOL_PIPE", "9,3,2");
        int nw = 0, l = 0, wg = 0;
        if (sscanf(g.c_str(), "%d,%d,%d", &nw, &l, &wg) != 3 || !hipk::pipe_supported(nw, l) || wg < 1 || wg > 8)
            throw Error("GOL_PIPE must be nw,L,wg with nw in {5,7,9,11,13,16}, L in 1..4 (got '" + g + "')");
        set_pipe(nw, l, wg);
        if (pipe_k_ > R)
            throw Error(strprintf("GOL_KERNEL=pipe: its pass depth %d exceeds the halo depth %d (GOL_HALO_DEPTH)", pipe_k_, R));
        K = pipe_k_;
    } else {
        throw Error("GOL_KERNEL must be auto, temporal, tile, pipe, lds or resident (got '" + kernel_ + "')");
    }
    if (!multipass_) R = std::min(R, K);
    kdepth_ = K;
    tdepth_ = supported_kernel_depth(std::min(kernel_ == "pipe" ? 8 : K, hipk::max_step_depth()));
    if (R != L_.R) L_ = Layout(L_.h, L_.w, R);
    stats_.depth = R;
    // slack rows: the temporal kernel prefetches 3 (shallow passes: 6) rows past a segment's last input row
    const size_t bytes = (size_t)(L_.words() + hipk::kSlackRows * L_.pitch) * 8;
    for (int i = 0; i < 2; ++i) HIP_CHECK(hipMalloc(&buf_[i], bytes));
    alloc_bytes_ = bytes;
    device_transport_ = t_->device_buffers() && cfg_.transport != "host";
    // Register both boards (their ghost and edge rows are what the one-tile exchanges send and receive)
    // with the device transport: RCCL's user-buffer registration (ncclCommRegister) lets peer
    // transfers read and write them directly instead of staging through its FIFOs.  Sub-tile halves
    // and 2-D staging buffers stay unregistered.  Default: on for a one-rank communicator (the
    // self-exchange proxy, where it was measured: 13.21 vs 13.29 us/gen, exchange 14.96 vs 15.2 us,
    // profiles/round4_batch_c.txt — the sub-tile schedule that wins there sends from the unregistered
    // halves), off with peers until a multi-GPU run has measured it; GOL_RCCL_REGISTER=0/1 forces.
    const int reg_default = t_->size() == 1 ? 1 : 0;
    if (device_transport_ && env_int("GOL_RCCL_REGISTER", reg_default) != 0 && !halo_items(L_.R).empty()) {
        for (int i = 0; i < 2; ++i) reg_[i] = t_->register_buffer(buf_[i], bytes);
        stats_registered_ = reg_[0] != nullptr && reg_[1] != nullptr;
    }
    if (cfg_.transport == "device" && !t_->device_buffers())
        throw Error("GOL_TRANSPORT=device needs a device transport (RCCL)");
    for (auto& kk : kern_) kk = kernel_ == "resident" ? "auto" : kernel_;
    if (kernel_ == "resident") kernel_ = "auto";
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
                                          prio_greatest));
    events_needed_ = cfg_.force_split || !halo_items(L_.R).empty();
    // All device memory work is ordered on the engine's own streams.  (They are non-blocking:
    // null-stream calls such as hipMemset, or a pageable hipMemcpy whose DMA may still be in
    // flight when it returns, would NOT be ordered before their kernels.)
    for (int i = 0; i < 2; ++i) HIP_CHECK(hipMemsetAsync(buf_[i], 0, bytes, s_comp_));
    HIP_CHECK(hipStreamSynchronize(s_comp_));
    // Stream-ordering events (never read by the host for data; event_flags: no system-scope fence)
    HIP_CHECK(hipEventCreateWithFlags(&ev_ready_, event_flags()));
    HIP_CHECK(hipEventCreateWithFlags(&ev_halo_, event_flags()));
    if (cfg_.profile) {
        for (auto* e : {&ev_t0_, &ev_t1_, &ev_t2_, &ev_t3_}) HIP_CHECK(hipEventCreate(e));
    }
    HIP_CHECK(hipMalloc(&d_red_, 2 * sizeof(u64)));
    HIP_CHECK(hipHostMalloc(&h_red_, 2 * sizeof(u64), hipHostMallocDefault));
    if (wd_)
        for (auto& m : mk_)
            for (auto& e : m.ev) HIP_CHECK(hipEventCreateWithFlags(&e, event_flags()));
}

HipEngine::Marker& HipEngine::marker_slot() {
    for (;;) {
        {
            std::lock_guard<std::mutex> lk(mk_mu_);
            std::string err;
            if (!retire_markers_locked(&err)) throw Error("progress marker: " + err);
            if (mk_count_ < kMarkers) return mk_[(mk_head_ + mk_count_) % kMarkers];
        }
        // every marker in flight: the host is kMarkers supersteps ahead of the GPU
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

bool HipEngine::retire_markers_locked(std::string* err) {
    while (mk_count_ > 0) {
        const Marker& m = mk_[mk_head_];
        for (int i = 0; i < m.n; ++i) {
            const hipError_t q = hipEventQuery(m.ev[i]);
            if (q == hipErrorNotReady) return true;
            if (q != hipSuccess) {
                *err = strprintf("hipEventQuery: %s", hipGetErrorString(q));
                return false;
            }
        }
        mk_head_ = (mk_head_ + 1) % kMarkers;
        --mk_count_;
        ++mk_done_;
    }
    return true;
}

void HipEngine::note_progress() {
    if (mk_published_) {  // the sub-tile superstep published its own end-of-superstep events
        mk_published_ = false;
        return;
    }
    Marker& m = marker_slot();
    HIP_CHECK(hipEventRecord(m.ev[0], s_comp_));
    m.n = 1;
    if (halo_pending_) {  // a one-pass split superstep left its exchange and bands on the comm stream
        HIP_CHECK(hipEventRecord(m.ev[1], s_comm_));
        m.n = 2;
    }
    publish_marker();
}

Watchdog::Probe HipEngine::probe() {
    Watchdog::Probe p;
    p.error = t_->async_error();
    std::lock_guard<std::mutex> lk(mk_mu_);
    std::string err;
    if (!retire_markers_locked(&err) && p.error.empty()) p.error = err;
    p.completed = mk_done_;
    p.pending = mk_count_ > 0;
    return p;
}

HipEngine::~HipEngine() {
    wd_.reset();  // its thread calls probe(), which reads the members destroyed below
    hipStreamSynchronize(s_comp_);
    hipStreamSynchronize(s_comm_);
    for (auto& kv : sub_plans_) hipFree(kv.second.d);
    for (auto& sb : sub_buf_)
        for (u64* b : sb)
            if (b) hipFree(b);
    for (auto e : ev_sub_own_)
        if (e) hipEventDestroy(e);
    if (ev_sub_x_) hipEventDestroy(ev_sub_x_);
    for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
    for (auto& kv : plans_) hipFree(kv.second.d);
    for (auto& kv : copies_) {
        hipFree(kv.second.pack);
        hipFree(kv.second.unpack);
    }
    for (auto& v : {&dstage_s_, &dstage_r_})
        for (u64* p : *v) hipFree(p);
    for (auto& v : {&hstage_s_, &hstage_r_, &xhs_, &xhr_})
        for (u64* p : *v) hipHostFree(p);
    for (void* h : reg_)
        if (h) t_->deregister_buffer(h);
    for (int i = 0; i < 2; ++i) hipFree(buf_[i]);
    for (auto& kv : res_plans_)
        for (void* q : {(void*)kv.second.d, (void*)kv.second.nbr_off, (void*)kv.second.nbr, (void*)kv.second.counters})
            if (q) hipFree(q);
    for (void* q : {(void*)res_status_, (void*)res_scratch_[0], (void*)res_scratch_[1]})
        if (q) hipFree(q);
    for (void* p : deferred_free_) hipFree(p);
    hipFree(d_red_);
    hipHostFree(h_red_);
    hipEventDestroy(ev_ready_);
    hipEventDestroy(ev_halo_);
    if (d_seq_) hipFree(d_seq_);
    for (auto& m : mk_)
        for (auto e : m.ev)
            if (e) hipEventDestroy(e);
    if (cfg_.profile)
        for (auto e : {ev_t0_, ev_t1_, ev_t2_, ev_t3_}) hipEventDestroy(e);
    hipStreamDestroy(s_comp_);
    hipStreamDestroy(s_comm_);
}

std::vector<u64> HipEngine::tile_words() {
    sync_canonical();
    synchronize();
    check_res_status();
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

void HipEngine::set_tile_words(const std::vector<u64>& dense) {
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

void HipEngine::run(u64 generations) {
    trace::Range range("gol.run");
    Armed armed(wd_.get());
    if (dual_ && !sub_current_) {
        // canonical board -> sub-tiles (interior rows), unless the sub-tiles already hold the
        // board (consecutive run() calls keep it in the halves; readers sync it back lazily)
        for (int s = 0; s < 2; ++s)
            dual_copy(sub_rows(s, sub_cur_, 0), buf_[cur_] + L_.index(sub_r0_[s], -1), rows_bytes(s, sub_L_[s].h));
        // both halves' first superstep waits for the copy (each waits on the other's "done" event)
        events_synced_ = false;
        HIP_CHECK(hipEventRecord(ev_sub_a_, s_comp_));
        HIP_CHECK(hipEventRecord(ev_sub_b_, s_comp_));
        sub_current_ = true;
    }
    run_graphed(generations);
    Engine::run(generations);
    if (dual_) canon_stale_ = true;  // copied back by the next reader (sync_canonical)
}

void HipEngine::do_init(const PatternSpec& p) {
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
        auto kick = [this](const char* phase) {
            if (wd_) wd_->kick(phase);
        };
        kick("init: kernel autotune");
        if (cfg_.kernel == "auto" || cfg_.kernel == "resident") autotune_kernel();
        // The one-tile pass costs first: the schedule candidates are timed on the pass cuts the runs
        // will use (config 3's strip: one step_pipe pass of 20 instead of 7 + 7 + 6 changed the winner)
        kick("init: pass costs");
        measure_pass_costs();
        // the split first pass's kernels again, at the depth the hinted superstep's cut starts with
        if (split_used() && !pass_costs().empty()) {
            const int kh = cfg_.run_hint > 0 && cfg_.run_hint < (u64)L_.R ? supported_depth((int)cfg_.run_hint) : L_.R;
            const int d0 = pass_depths(kh)[0];
            if (d0 != kdepth_) tune_split_kinds(d0);
        }
        kick("init: schedule timing");
        pass_us_[1].clear();  // (the halves' pass costs are measured when a sub-tile schedule is applied)
        choose_schedule();  // collective when ranks have neighbours
        kick("init: plans and graphs");
        tuned_ = true;
        finish_init();
        if (!sched_runners_up_.empty()) confirm_schedule();
        return;
    }
    finish_init();
}

void HipEngine::finish_init() {
    stats_.kernel = split_ ? kern_[1] + "+boundary:" + kern_[2] : (dual_ ? std::string("temporal") : kern_[0]);
    if (!split_ && !dual_ && kern_[0] == "pipe")
        stats_.kernel = strprintf("pipe@%d(%dx%d,%d/CU)", pipe_k_, pipe_cur_.nw - 1, pipe_cur_.l, pipe_cur_.wg);
    if (res_) {
        const ResPlan& rp = res_plan(res_kin_);
        stats_.kernel = strprintf("resident@%d(%lld tiles x %d waves x %d rows)", res_kin_, (long long)rp.tiles, rp.nw, rp.B);
    }
    stats_.schedule = split_ ? "split" : (halo_items(L_.R).empty() ? "local" : "full");
    if (dual_) stats_.schedule += sub_overlap_ ? "+subtiles2ov" : "+subtiles2";
    stats_.kernel_depth = dual_ ? tdepth_ : kdepth_;
    stats_.tile_waves = cfg_.tile_waves;
    std::string tn;
    for (const auto& kv : tune_ms_) tn += strprintf("%s%s=%.3fus/gen", tn.empty() ? "" : " ", kv.first.c_str(), kv.second * 1e3);
    for (const auto& kv : sched_us_)
        tn += strprintf("%ssched:%s=%.3fus/gen", tn.empty() ? "" : " ", kv.first.c_str(), kv.second);
    for (const auto& kv : pass_costs()) tn += strprintf("%spass%d=%.1fus", tn.empty() ? "" : " ", kv.first, kv.second);
    // the kernel passes of the supersteps the runs use (the full superstep, the hinted run's remainder)
    if (!dual_ && !res_ && kernel_ != "lds")
        for (int k : init_depths()) {
            std::string c;
            const std::vector<int>& ps = pass_depths(k);
            for (size_t j = 0; j < ps.size(); ++j) {
                const int kind = j == 0 && split_ ? 1 : 0;
                const PipeGeo* g = pipe_geo(ps[j]);
                const PassKernel pk = pass_kernel(kind, ps[j]);
                c += (j ? "+" : "") + (pk == PK_PIPE   ? strprintf("pipe@%d(%dx%d,%d/CU)", ps[j], g->nw - 1, g->l, g->wg)
                                       : pk == PK_TILE ? strprintf("tile@%d", ps[j])
                                                       : strprintf("temporal@%d", ps[j]));
            }
            tn += strprintf("%scut%d=%s", tn.empty() ? "" : " ", k, c.c_str());
        }
    if (!split_ && !dual_ && !res_ && tile_kernel(0) && kernel_ != "lds") {  // the tile variant the full superstep runs
        const DevPlan& p0 = plan(0, kdepth_, 0);
        tn += strprintf("%stile_plan=%s,%lldrows,%lldtiles", tn.empty() ? "" : " ",
                        p0.fold ? ((p0.tflags & hipk::STEP_TILE_INPLACE) ? "fold-inplace" : "fold")
                                : ((p0.tflags & hipk::STEP_TILE_INPLACE) ? "inplace" : "double"),
                        (long long)p0.rows, (long long)p0.waves);
    }
    stats_.tuning = tn + confirm_note_;
    stats_.registered = stats_registered_;
    // Build the plans of the supersteps the runs will use now (the full superstep and the
    // remainder of the hinted run length), so neither graph capture nor a hinted timed loop
    // builds or uploads a plan.  Other remainders are built on first use.
    for (int k : init_depths()) {
        if (dual_)
            prepare_dual(k);
        else
            prepare(k);
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
    predict_run();
    if (res_) {
        stats_.plan_waves = res_plan(res_kin_).tiles;  // workgroups of the resident launch
        stats_.lane_efficiency = 0;
    } else {
        const DevPlan& fp = full_plan_stats();
        stats_.plan_waves = fp.waves;
        stats_.lane_efficiency = fp.st.lane_rows ? (double)fp.st.out_words / (double)fp.st.lane_rows : 0.0;
    }
}

void HipEngine::tile_superstep(int k) {
    if (res_) {  // the whole superstep is one resident launch (no neighbours: nothing to exchange)
        res_launch(k, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
        cur_ ^= 1;
        return;
    }
    const std::vector<int>& ps = pass_depths(k);
    first_pass(k, ps[0], ext_after(ps, 0), split_);
    cur_ ^= 1;
    for (size_t j = 1; j < ps.size(); ++j) {
        // later passes need no halo: the ghost rows computed by the earlier passes carry the
        // neighbours' cells forward (communication-avoiding deep halos)
        join_halo();
        const i64 e = ext_after(ps, j);
        launch(0, ps[j], e, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
        post(buf_[cur_ ^ 1], s_comp_, e);
        cur_ ^= 1;
    }
    if (ps.size() > 1) mark_ready();  // the next exchange reads what the last pass wrote
}

// Exchange the kx-deep halo and run the first kernel pass (depth kp, output rows extended by e
// beyond the tile): buf[cur] -> buf[cur^1]; the caller flips the parity.  `split`: interior +
// boundary bands with the exchange overlapped (else exchange, then one full-region kernel).
void HipEngine::first_pass(int kx, int kp, i64 e, bool split) {
    prepare(kx);
    join_halo();
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
        bool bands_multi = false;  // the bands ran on the comm stream (a superstep with later passes)
        if (items.empty()) {
            // GOL_FORCE_SPLIT on a rank without neighbours: the multi-GPU stream structure
            // with an empty exchange (measures the split schedule's own cost on one GPU)
            HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_ready_, 0));
            HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
            launch(1, kp, 0, src, dst, s_comp_);
        } else if (device_transport_) {
            // The exchange on the comm stream (it waits only for the previous superstep), the interior
            // on the compute stream meanwhile.  A superstep of ONE pass (e == 0) also runs its bands on
            // the comm stream, right after the exchange and concurrently with the interior, and leaves
            // the two streams unjoined: the next superstep, or whatever reads the board, joins them
            // (join_halo).  A wait on an event still pending costs the waiting queue ~17 us after the
            // event, more than the ~14 us exchange it would hide (kernel traces of config 3's strip,
            // profiles/strip_split_round5.txt); with later passes the bands follow the interior on the
            // compute stream, whose wait then finds the exchange done.
            // (Not when the ghost columns of an unaligned self-wrapped width are refilled after the pass:
            // post() reads the first and last words of EVERY row, so it must follow both the interior and
            // the bands on one stream.)
            const bool bands_comm = e == 0 && !prof && !(self_x() && !L_.aligned());
            // With later passes too, the bands run on the comm stream right after the exchange, beside the
            // interior's tail, and the compute stream waits for them before the next pass.  The bands read the
            // old board and the fresh ghost rows and write rows the interior does not, so they need only the
            // exchange; on the compute stream they waited for the interior as well and added their whole pass
            // to the critical path.  Weak rank 11.75-12.17 against 12.32-12.54 us/gen, config 4's 2-D tile
            // 7.72-7.80 against 7.88-7.99 (profiles/split_order_round6.txt, b30); GOL_SPLIT_BANDS_COMM=0
            // restores the bands on the compute stream.
            bands_multi = split_bands_comm_ && e > 0 && !prof && !(self_x() && !L_.aligned());
            // The interior is issued first, before the exchange's host-side RCCL group launch: the interior
            // then starts ~17 us after run() instead of ~46, and the exchange still runs beside it (its kernel
            // stretches, 37.8 -> 43.6 us, the interior does not).  Config 4's 2-D tile 7.94 against 8.55-8.70
            // us/gen, the weak rank's split 12.43-12.87 against 12.90-13.02 (profiles/split_order_round6.txt);
            // the strip's step_pipe interior: 3.46-3.57 against 3.63-3.91 (profiles/strip_split_round5.txt).
            // GOL_SPLIT_INT_FIRST=0 restores the exchange-first order.  (Raising the bands' wave priority
            // instead, s_setprio, slowed the interior more than it sped the bands: 3.90-6.35, round 5.)
            guard_exchange_stream(s_comm_);  // (before any event query or launch of a capture attempt)
            const bool int_first = split_int_first_;
            if (int_first) launch(1, kp, 0, src, dst, s_comp_);
            wait_pending(s_comm_, ev_ready_);
            if (prof) HIP_CHECK(hipEventRecord(ev_t0_, s_comm_));
            exchange_device(kx, items, cur_, s_comm_);
            if (prof) HIP_CHECK(hipEventRecord(ev_t1_, s_comm_));
            if (!bands_comm && !bands_multi) record_halo();
            if (prof) HIP_CHECK(hipEventRecord(ev_t2_, s_comp_));
            if (!int_first) launch(1, kp, 0, src, dst, s_comp_);
            if (bands_comm) {
                launch(2, kp, e, src, dst, s_comm_);
                post(dst, s_comm_, e);
                record_halo();
                halo_pending_ = true;
                mark_ready();
                return;
            }
            if (bands_multi) {
                launch(2, kp, e, src, dst, s_comm_);
                if (split_value_wait_) {
                    // The compute stream waits for the bands with a stream memory op on a value written after
                    // them, not with the event: the runtime polls it from a one-workgroup kernel queued right
                    // behind the interior, and the next pass follows that kernel with no gap, where the event
                    // wait cost the compute queue ~10-20 us.  Config 4's 2-D tile 7.41-7.48 against 7.70-8.02
                    // us/gen, the weak rank's split 11.68-11.96 against 11.97-12.19 (profiles/split_order_round6.txt,
                    // b33).  The write is always enqueued before the wait (no deadlock on a shared hardware queue),
                    // and the next write only after the wait has passed (the next exchange waits for the superstep's
                    // end), so waiting for equality is exact and immune to wrap-around.  GOL_SPLIT_VALUE_WAIT=0: the event.
                    if (!d_seq_) {
                        HIP_CHECK(hipMalloc(&d_seq_, sizeof(u32)));
                        HIP_CHECK(hipMemsetAsync(d_seq_, 0, sizeof(u32), s_comm_));
                    }
                    ++seq_;
                    HIP_CHECK(hipStreamWriteValue32(s_comm_, d_seq_, seq_, 0));
                }
                record_halo();
            }
        } else {
            if (prof) HIP_CHECK(hipEventRecord(ev_t2_, s_comp_));
            launch(1, kp, 0, src, dst, s_comp_);  // interior first: runs while the host exchanges
            HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_ready_, 0));
            if (prof) HIP_CHECK(hipEventRecord(ev_t0_, s_comm_));
            exchange_staged(kx, items, cur_, s_comm_);
            if (prof) HIP_CHECK(hipEventRecord(ev_t1_, s_comm_));
            HIP_CHECK(hipEventRecord(ev_halo_, s_comm_));
        }
        if (bands_multi && split_value_wait_)
            HIP_CHECK(hipStreamWaitValue32(s_comp_, d_seq_, seq_, hipStreamWaitValueEq, 0xFFFFFFFFu));
        else
            HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_halo_, 0));
        if (!bands_multi) launch(2, kp, e, src, dst, s_comp_);
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
    // The ready event marks the end of the superstep, for the next exchange: with later passes to come the
    // caller records it after the last one (tile_superstep, time_schedule), and a record here would only put
    // a release barrier between this pass and the next (a ~5.7 us gap on the compute queue: config 4's 2-D
    // tile trace, profiles/split_order_round6.txt).  GOL_FIRST_PASS_MARK=1 restores it (A/B knob).
    if (pass_depths(kx).size() == 1 || first_pass_mark_) mark_ready();
}

void HipEngine::do_set_compat_halos(const std::vector<u64>& above, const std::vector<u64>& below) {
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

void HipEngine::launch(int kind, int k, i64 e, const u64* src, u64* dst, hipStream_t s, u32 xflags) {
    if (kernel_ == "lds") {
        // full-row bands only (the LDS variant is never split by columns: can_overlap)
        for (const Region& r : regions(kind, 1))
            if (r.c0 == 0) hipk::launch_step_lds(src, dst, L_, r.r0, r.r1, step_flags(), s);
    } else {
        const DevPlan& p = plan(kind, k, e);
        if (p.st.out_words == 0) return;
        hipk::StepParams sp{L_.pitch, (i32)L_.h, (i32)L_.nw, L_.R, step_flags() | p.tflags | xflags};
        const PassKernel pk = pass_kernel(kind, k);
        if (pk == PK_TILE) {
            hipk::launch_step_tile(cfg_.tile_waves, k, src, dst, p.d, p.waves, p.rows, sp, s);
        } else if (pk == PK_PIPE) {
            const PipeGeo* g = pipe_geo(k);
            hipk::launch_step_pipe(g->nw, g->l, src, dst, p.d, p.waves, sp, s);
            pipe_used_ = true;
        } else
            hipk::launch_step(k, src, dst, p.d, p.waves, sp, s);
    }
    HIP_CHECK(hipGetLastError());
}

}  // namespace hipeng

std::unique_ptr<Engine> make_hip_engine(const Geometry& g, const EngineConfig& c, std::shared_ptr<Transport> t) {
    int err = 0;
    if (hip_device_count(&err) <= 0) throw Error("no HIP device available");
    return std::make_unique<hipeng::HipEngine>(g, c, std::move(t));
}

}  // namespace gol
