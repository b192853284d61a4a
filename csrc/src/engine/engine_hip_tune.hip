// gol-mi355x: HipEngine — measurement at init: kernel autotune, superstep schedule choice, per-depth pass costs.
#include "hip_engine.hpp"

namespace gol {
namespace hipeng {

// Bring the GPU to its steady clock before anything is timed.  From idle, sclk ramps up over
// the first ~20-30 ms of load (measured on MI355X: 32768^2 passes shrink from ~97 to ~87 us
// while rocm-smi shows sclk rising to 2.4 GHz), which would bias the kernel autotune towards
// whichever candidate runs last and make the first generations of a run slower than the rest.
// The full-board kernel runs on the scratch buffer (the board is untouched) for GOL_SPINUP_MS
// (default 100 ms for boards of >= 2^24 cells, 20 ms below; 0 = off).
void HipEngine::spin_up() {
    const bool big = (double)L_.h * (double)L_.w >= (double)(1 << 24);
    const double budget_ms = (double)env_int("GOL_SPINUP_MS", big ? 100 : 20);
    if (budget_ms <= 0 || cfg_.compat || kernel_ == "lds") return;
    const std::string saved = kern_[0];
    int k = 0;
    if (!dual_ && kern_[0] == "pipe" && pipe_k_ > 0) {
        k = pipe_k_;  // the kernel the runs use
    } else {
        if (cfg_.kernel != "tile") kern_[0] = "temporal";  // the register kernel runs on any board
        // (sub-tiles: their own pass depth; a deep full-tile depth, e.g. a pipe candidate's 36, would
        // spin the GPU up on a 1-wave-per-SIMD kernel of a different power draw)
        k = tile_kernel(0) ? kdepth_ : supported_kernel_depth(std::min(dual_ ? tdepth_ : kdepth_, hipk::max_step_depth()));
    }
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
void HipEngine::measure_pass_costs() {
    std::map<int, double>& costs = pass_us_[dual_ ? 1 : 0];
    costs.clear();
    if (!dual_) pipe_geo_.clear();
    if (cfg_.compat || cfg_.kernel_depth > 0 || kernel_ == "lds" || res_ || (!dual_ && tile_kernel(0))) return;
    // every instantiated depth up to the pass depth, and the deeper ones a superstep could use: a
    // 20-generation superstep cut 12 + 8 measured cheaper than 8 + 8 + 4 (the K=12 pass runs 2 waves
    // per SIMD at ~10.6 us/gen as two halves, vs 10.3 at K=8; profiles/pingpong_loop_ab.txt)
    const int K = dual_ ? tdepth_ : kdepth_;
    const int kmax = std::min(superstep_depth(), hipk::max_step_depth());
    struct Cand {
        int d;
        PipeGeo g;  // g.nw > 0: a step_pipe pass of this geometry
    };
    std::vector<Cand> cs;
    for (int d = 1; d <= std::max(K, kmax); ++d)
        if (hipk::step_depth_supported(d)) cs.push_back({d, {}});
    // A one tile whose tuned kernel is step_pipe: its passes may be step_pipe at any depth one of these
    // geometries reaches (and the superstep allows), so a superstep is cut into the cheapest mix, e.g.
    // the driver's 20-generation run on config 3's 4096 x 32768 strip as ONE step_pipe pass of 20
    // (10 stages x 2) instead of three step_temporal passes of 7 + 7 + 6.
    // (Round 6: also one generation per stage, and two workgroups per CU -- twice the waves per SIMD to hide
    // the stage chain's latency, with rings of nw <= 9 waves, whose LDS fits twice in a CU's 160 KiB.)
    if (!dual_ && kern_[0] == "pipe" && pipe_k_ > 0) {
        std::vector<PipeGeo> gs = {pipe_cur_};
        for (int l : {1, 2, 3})
            for (int nw : {5, 7, 9, 11, 13, 16})
                if (!(l == 3 && (nw == 11 || nw == 16))) gs.push_back({nw, l, 1});
        for (int l : {1, 2, 3})
            for (int nw : {5, 7, 9})
                if (2 * hipk::pipe_lds_bytes(nw) <= 160 * 1024) gs.push_back({nw, l, 2});
        for (const PipeGeo& g : gs) {
            const int d = (g.nw - 1) * g.l;
            if (d > superstep_depth() || !hipk::pipe_supported(g.nw, g.l)) continue;
            bool dup = false;
            for (const Cand& c : cs) dup = dup || (c.g.nw == g.nw && c.g.l == g.l && c.g.wg == g.wg);
            if (!dup) cs.push_back({d, g});
        }
    }
    if (cs.size() < 2) return;
    // pipe_geo_ lists exactly the depths that run step_pipe (the -1 entry marks it as authoritative)
    auto select = [&](const Cand& c) {
        pipe_geo_.clear();
        pipe_geo_[-1] = PipeGeo{};
        if (c.g.nw > 0) pipe_geo_[c.d] = c.g;
    };
    for (const Cand& c : cs) {  // every plan first: plan building idles the GPU and drops its clock
        if (dual_) {
            sub_plan(0, c.d, 0);
            sub_plan(1, c.d, 0);
        } else {
            select(c);
            plan(0, c.d, 0);
        }
    }
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    if (!dual_) pipe_geo_.clear();  // (the spin-up runs the tuned kernel at its own depth, not a candidate's)
    spin_up();
    const int reps = 4;
    std::vector<double> best(cs.size(), 1e30);
    std::vector<char> dropped(cs.size(), 0);
    for (int round = 0; round < 3; ++round)
        for (size_t i = 0; i < cs.size(); ++i) {
            if (dropped[i]) continue;
            const int d = cs[i].d;
            HIP_CHECK(hipEventRecord(e0, s_comp_));
            if (dual_) {
                HIP_CHECK(hipStreamWaitEvent(s_comm_, e0, 0));
                for (int r = 0; r < reps; ++r)
                    for (int sub = 0; sub < 2; ++sub) {
                        const DevPlan& pl = sub_plan(sub, d, 0);
                        const Layout& Ls = sub_L_[sub];
                        hipk::StepParams sp{Ls.pitch, (i32)Ls.h, (i32)Ls.nw, Ls.R, sub_flags()};
                        hipk::launch_step(d, sub_buf_[sub][sub_cur_], sub_buf_[sub][(sub_cur_ + 1) % 3], pl.d,
                                          pl.waves, sp, sub ? s_comm_ : s_comp_);
                    }
                events_synced_ = false;
                HIP_CHECK(hipEventRecord(ev_sub_b_, s_comm_));
                HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_sub_b_, 0));
            } else {
                select(cs[i]);
                for (int r = 0; r < reps; ++r) launch(0, d, 0, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
            }
            HIP_CHECK(hipEventRecord(e1, s_comp_));
            HIP_CHECK(hipEventSynchronize(e1));
            float ms = 0;
            HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
            best[i] = std::min(best[i], ms * 1e3 / reps);
            // A step_pipe geometry whose ring wait timed out is dropped, as the kernel autotune drops one: the
            // candidates write only the scratch buffer, so the board is still valid (pipe_fault clears the flag)
            if (cs[i].g.nw > 0 && hipk::pipe_fault()) {
                fprintf(stderr, "[gol] step_pipe %dx%d: a ring wait timed out while measuring pass costs; candidate dropped\n",
                        cs[i].g.nw - 1, cs[i].g.l);
                dropped[i] = 1;
                best[i] = 1e30;
            }
            const std::string what =
                cs[i].g.nw ? strprintf("pipe pass %dx%d,%d/CU", cs[i].g.nw - 1, cs[i].g.l, cs[i].g.wg) : std::string("pass");
            init_step("init: pass costs", what.c_str(), d, (float)(best[i] / d));
        }
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
    HIP_CHECK(hipGetLastError());
    std::map<int, PipeGeo> geo = {{-1, PipeGeo{}}};
    for (size_t i = 0; i < cs.size(); ++i) {
        if (dropped[i]) continue;
        auto it = costs.find(cs[i].d);
        if (it != costs.end() && it->second <= best[i]) continue;
        costs[cs[i].d] = best[i];
        if (cs[i].g.nw > 0)
            geo[cs[i].d] = cs[i].g;
        else
            geo.erase(cs[i].d);
    }
    if (!dual_) {
        pipe_geo_.clear();
        if (kern_[0] == "pipe") pipe_geo_ = geo;  // (otherwise no step_pipe passes: the tuned default)
    }
    passes_.clear();
}

void HipEngine::choose_schedule() {
    const bool nbrs = !halo_items(L_.R).empty();  // identical on every rank (uniform grid)
    std::vector<std::string> cands;
    if (cfg_.force_split || (cfg_.sched == "split" && split_used())) {
        cands = {"split"};
    } else {
        cands.push_back(nbrs ? "full" : "local");
        if (cfg_.sched == "auto" && split_used()) cands.push_back("split");
        // the one-tile superstep with its RCCL group captured in a graph (one replay per run)
        if (nbrs && device_transport_ && t_->graph_capturable() && cfg_.graph && !cfg_.profile && !cfg_.compat &&
            cfg_.graph_rccl < 0)
            cands.push_back("full+graph");
    }
    graph_rccl_on_ = cfg_.graph_rccl == 1;
    bool dual_ok = cfg_.subtiles != 0 && cands[0] != "split" && dual_wanted();
    if (dual_ok) {
        double ok = dual_local_ok() ? 1.0 : 0.0;
        if (t_->size() > 1) ok = t_->allreduce_min(ok);
        dual_ok = ok > 0;
    }
    if (dual_ok) {
        // the overlapped variant needs the exchange (neighbours, or the self-exchange)
        std::vector<std::string> dc;
        if (cfg_.subtile_overlap <= 0 || self_y()) dc.push_back("subtiles");
        if (cfg_.subtile_overlap != 0 && !self_y()) dc.push_back("subtiles+ov");
        if (cfg_.subtiles == 2) cands.clear();
        cands.insert(cands.end(), dc.begin(), dc.end());
    }
    std::string pick = cands[0];
    if (cands.size() > 1) {
        // Supersteps of the length the runs will use: kSchedReps back-to-back R-generation supersteps,
        // or, when the hinted run is shorter than R (the driver's 20-generation bench is a single
        // 20-generation superstep), that one superstep started from an idle GPU, as the run will
        // be: its launch latency, exchange and drain weigh more there, and the candidates are
        // within a few % of each other, so it gets more rounds.
        const bool short_run = cfg_.run_hint > 0 && cfg_.run_hint < (u64)L_.R;
        const int k = short_run ? supported_depth((int)cfg_.run_hint) : L_.R;
        const int reps = short_run ? 1 : kSchedReps;
        const int rounds = short_run ? 15 : 3;
        std::vector<double> best(cands.size(), 1e30);
        // (a short run is ONE superstep, a single sample of its latency: the candidates are ranked by
        // their median round there, not their best one, which favoured a candidate of wide spread --
        // full+graph timed 12.6 against subtiles+ov's 12.3-12.5 us/gen at best, won one init in five,
        // and that run measured 13.4 against 12.0-12.4 us/gen, driver's cut through the self-exchange)
        std::vector<std::vector<double>> samples(cands.size());
        spin_up();
        for (int round = 0; round < rounds; ++round)
            for (size_t c = 0; c < cands.size(); ++c) {
                if (round == 0) time_schedule(cands[c], k, reps);  // warm-up: connections, plans, graphs
                const double us = sample_schedule(cands[c], k, reps);
                samples[c].push_back(us);
                best[c] = std::min(best[c], us);
                if (short_run) {
                    std::vector<double> v = samples[c];
                    std::sort(v.begin(), v.end());
                    best[c] = v[(v.size() - 1) / 2];
                }
                init_step("init: schedule timing", cands[c].c_str(), k, (float)best[c]);
            }
        size_t bi = 0;
        for (size_t c = 0; c < cands.size(); ++c) {
            // a candidate whose timing graph could not be captured on some rank is dropped
            if (t_->allreduce_max(sched_graph_failed_.count(cands[c]) ? 1.0 : 0.0) > 0) best[c] = 1e30;
            sched_us_[cands[c]] = best[c];
            if (best[c] < best[bi]) bi = c;
        }
        pick = cands[bi];
        // The split schedule must win by 3% over full: its timing (4 supersteps) favoured it by ~1% on
        // 1-D strips whose runs then went 2-4% slower than full (8192 x 65536 through RCCL: split
        // timed 6.41 vs 6.48, ran 6.01 vs 5.85 us/gen); the 2-D tiles where it wins do so by 3-5%.
        if (pick == "split" && sched_us_.count("full") && sched_us_["split"] > 0.97 * sched_us_["full"]) {
            size_t b2 = cands.size();
            for (size_t c = 0; c < cands.size(); ++c)
                if (cands[c] != "split" && (b2 == cands.size() || best[c] < best[b2])) b2 = c;
            pick = cands[b2];
        }
        // the runners-up (at most kMaxConfirm, fastest first) that timed within kConfirmMargin of the pick
        // (identical on every rank: the timings are maxima over the ranks)
        // (GOL_SCHED_CONFIRM=2, a test knob: confirm whatever the margin)
        const int confirm = env_int("GOL_SCHED_CONFIRM", 1);
        std::vector<size_t> order;
        for (size_t c = 0; c < cands.size(); ++c)
            if (cands[c] != pick && best[c] < 1e29) order.push_back(c);
        std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return best[a] < best[b]; });
        for (size_t c : order)
            if (cfg_.run_hint > 0 && confirm != 0 && (int)sched_runners_up_.size() < kMaxConfirm &&
                (confirm == 2 || best[c] <= (1.0 + kConfirmMargin) * sched_us_[pick]))
                sched_runners_up_.push_back(cands[c]);
        stats_.exchanges = 0;  // the timing exchanges and replays are not part of the run
        stats_.halo_bytes = 0;
        stats_.graph_launches = 0;
    }
    destroy_sched_graphs();  // (they captured the communicator: destroy them before the comm can go)
    apply_schedule(pick);
}

// Make `pick` the schedule of the runs (choose_schedule, confirm_schedule).  The board is canonical
// (buf_[cur_]) whenever this runs: at the end of the timing, or after predict_run.
void HipEngine::apply_schedule(const std::string& pick) {
    synchronize();
    // the run graphs were captured for the previous schedule (their keys do not name it)
    for (auto& kv : graphs_) HIP_CHECK(hipGraphExecDestroy(kv.second));
    graphs_.clear();
    sched_pick_ = pick;
    split_ = pick == "split";
    dual_ = pick.rfind("subtiles", 0) == 0;
    sub_overlap_ = pick == "subtiles+ov" ? 1 : 0;
    graph_rccl_on_ = cfg_.graph_rccl == 1 || pick == "full+graph";
    if (dual_) {
        setup_dual();
        sub_current_ = false;  // the halves hold timing scratch: load the board at the next run
        if (pass_us_[1].empty()) measure_pass_costs();  // the two halves' (the candidates ran the default cuts)
    } else if (sub_buf_[0][0]) {
        teardown_dual();
    }
    passes_.clear();  // the pass cuts depend on the schedule (pass_costs) and the tuned kernels
    // The comm stream waits on the compute stream's ready event only in the split schedule (and the
    // forced-split measurement mode).  The full schedule exchanges on the compute stream itself:
    // recording the event there every superstep only idles the GPU (~15 us per record, a release fence).
    events_needed_ = cfg_.force_split || (split_ && !halo_items(L_.R).empty());
}

// The close call of choose_schedule settled on the real run() path: each runner-up set up in full and
// predicted like the pick was (finish_init -> predict_run: the hinted run on a snapshot of the board,
// bracketed as bench.py brackets it, max over the ranks); the fastest prediction is kept.  Collective:
// the predictions are identical on every rank, so is the decision.
void HipEngine::confirm_schedule() {
    const std::vector<std::string> runners = sched_runners_up_;
    sched_runners_up_.clear();
    std::string best = sched_pick_;
    double pbest = stats_.predicted_us_per_gen;
    if (pbest <= 0 || runners.empty()) return;  // (no prediction: no hinted run, or fault injection)
    std::string note = strprintf(" confirm:%s=%.3fus/gen", best.c_str(), pbest);
    std::string current = best;
    for (const std::string& c : runners) {
        if (wd_) wd_->kick("init: schedule confirm");
        apply_schedule(c);
        finish_init();
        current = c;
        const double p = stats_.predicted_us_per_gen;
        note += strprintf(",%s=%.3fus/gen", c.c_str(), p);
        if (p > 0 && p < pbest) {
            best = c;
            pbest = p;
        }
    }
    init_step("init: schedule confirm", best.c_str(), 0, (float)pbest);
    confirm_note_ = note;
    if (best != current) {
        apply_schedule(best);
        finish_init();  // (appends confirm_note_ to stats.tuning)
    } else {
        stats_.tuning += confirm_note_;
    }
}

// One timed sample of `reps` supersteps of k generations of schedule `c`, bracketed as bench.py
// brackets its timed run: the engine's streams synchronised, the ranks aligned by device_barrier (host
// barrier, then the transport's device barrier completed on the GPU), the supersteps, then a device-wide
// synchronisation (bench.py: torch.cuda.synchronize()).  us per generation, the max over the ranks.
double HipEngine::sample_schedule(const std::string& c, int k, int reps) {
    device_barrier();
    const auto t0 = std::chrono::steady_clock::now();
    time_schedule(c, k, reps);
    if (wd_) note_progress();  // (a run publishes a progress marker per superstep or replay: an event record)
    end_sync();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return t_->allreduce_max(dt) * 1e6 / ((double)reps * k);
}

// The chosen schedule timed at the end of init the way the hinted runs execute it: the real run() path
// (graph replay or eager supersteps, pass cuts, kernels, progress markers) on a snapshot of the board,
// each sample bracketed as bench.py brackets its timed run (sample_run), the median of a few samples,
// reported as stats.predicted_us_per_gen next to what a run then measures.  The board, its parity and
// the generation count are restored afterwards.  Without memory for the snapshot (agreed over the
// ranks) the samples run the schedule on scratch state instead (sample_schedule).  Collective.  Long
// samples (big boards) are cut short.  Skipped with fault injection (the samples would advance the
// generation count it watches).
void HipEngine::predict_run() {
    if (cfg_.run_hint == 0 || cfg_.compat || sched_pick_.empty()) return;
    // (fault injection is set on the faulting rank only: agreed, since everything below is collective)
    if (t_->allreduce_max(fault_gen_ >= 0 ? 1.0 : 0.0) > 0) return;
    const int k = supported_depth((int)std::min<u64>(cfg_.run_hint, (u64)superstep_depth()));
    const int reps = (int)std::min<u64>(kSchedReps, std::max<u64>(1, cfg_.run_hint / (u64)k));
    u64 gens = (u64)k * (u64)reps;  // (snapshot path: the hinted run itself, when it takes <= ~50 ms)
    const EngineStats saved = stats_;
    std::vector<double> v;
    int rounds = reps == 1 ? 9 : 5;
    sync_canonical();
    synchronize();
    size_t fr = 0, tot = 0;
    // (GOL_PREDICT_SNAPSHOT=0, a test knob: behave as if no memory were free for the snapshot, as on BASELINE
    // config 5's 2^20-row tile, so the scratch-state branch below runs on a small board)
    double snap_ok = env_int("GOL_PREDICT_SNAPSHOT", 1) != 0 && hipMemGetInfo(&fr, &tot) == hipSuccess &&
                             fr > alloc_bytes_ + ((size_t)1 << 30)
                         ? 1.0
                         : 0.0;
    if (t_->size() > 1) snap_ok = t_->allreduce_min(snap_ok);
    u64* snap = nullptr;
    if (snap_ok > 0 && hipMalloc(&snap, alloc_bytes_) != hipSuccess) {
        hipGetLastError();
        snap = nullptr;
    }
    if (t_->size() > 1) snap_ok = t_->allreduce_min(snap ? 1.0 : 0.0);
    if (snap_ok <= 0) {
        if (snap) hipFree(snap);
        snap = nullptr;
    }
    auto over = [&](std::chrono::steady_clock::time_point t0) {  // (agreed: every rank stops together)
        return t_->allreduce_max(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count()) > 1.0;
    };
    if (snap) {
        const int cur0 = cur_;
        const u64 gen0 = gen_;
        HIP_CHECK(hipMemcpyAsync(snap, buf_[cur0], alloc_bytes_, hipMemcpyDeviceToDevice, s_comp_));
        synchronize();
        // warm-up (loads the sub-tile halves, as a warmup run does before a timed one), then the samples
        // run the whole hinted run when it is short enough: a 1000-generation run of 8192^2 is one graph
        // replay, which samples of 4 supersteps would charge four graph launches per 128 generations
        const double w = time_runs(gens, 1)[0];
        const u64 fit = (u64)(0.05e6 / std::max(1e-3, w));
        gens = std::max<u64>(gens, std::min<u64>(cfg_.run_hint, fit));
        if (gens > (u64)k * reps) {
            rounds = 5;
            run(gens);
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < rounds; ++r) {
            v.push_back(time_runs(gens, 1)[0]);
            if (over(t0)) break;
        }
        synchronize();
        cur_ = cur0;
        HIP_CHECK(hipMemcpyAsync(buf_[cur0], snap, alloc_bytes_, hipMemcpyDeviceToDevice, s_comp_));
        synchronize();
        HIP_CHECK(hipFree(snap));
        gen_ = gen0;
        sub_current_ = false;  // the halves hold a later generation: reload them from the board at the next run
        canon_stale_ = false;
    } else if (res_) {
        for (int r = 0; r < rounds; ++r) v.push_back((double)time_resident(res_kin_, k) * 1e3);
    } else {
        time_schedule(sched_pick_, k, reps);  // warm-up (and the candidate's timing graph)
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < rounds; ++r) {
            v.push_back(sample_schedule(sched_pick_, k, reps));
            if (over(t0)) break;
        }
        synchronize();
        destroy_sched_graphs();
        if (dual_) sub_current_ = false;  // the halves hold timing scratch: load the board at the next run
    }
    std::sort(v.begin(), v.end());
    stats_ = saved;  // the samples' exchanges and replays are not part of any run
    stats_.predicted_us_per_gen = v[(v.size() - 1) / 2];
    stats_.predicted_gens = (int)gens;
    init_step("init: prediction", sched_pick_.c_str(), k, (float)stats_.predicted_us_per_gen);
}

// `reps` supersteps of k generations of schedule `c` on scratch state (see choose_schedule).
void HipEngine::time_schedule(const std::string& c, int k, int reps, bool eager) {
    if (c.rfind("subtiles", 0) == 0) {
        setup_dual();
        const bool d0 = dual_;
        const int o0 = sub_overlap_;
        dual_ = true;
        sub_overlap_ = c == "subtiles+ov" ? 1 : 0;
        for (int i = 0; i < reps; ++i) dual_superstep(k);
        dual_ = d0;
        sub_overlap_ = o0;
        return;
    }
    // One-tile supersteps as the runs replay them (graphs: "local" always, the "full+graph"
    // candidate): `reps` supersteps captured once per candidate (round 0's warm-up call,
    // after one eager superstep that loads every kernel variant), one replay per call.
    const bool graphed = !eager && (c == "full+graph" ||
                                    (c == "local" && cfg_.graph && !cfg_.profile && !cfg_.compat && graph_ok_));
    if (graphed) {
        const std::string base = c == "local" ? "local" : "full";
        SchedGraph& sg = sched_graphs_[c];
        if (sg.exec && sg.reps != reps) {
            HIP_CHECK(hipStreamSynchronize(s_comp_));
            HIP_CHECK(hipGraphExecDestroy(sg.exec));
            sg.exec = nullptr;
        }
        if (!sg.exec && !sched_graph_failed_.count(c)) {
            prepare(k);
            time_schedule(base, k, 1, true);
            synchronize();  // (also joins the streams: no event query inside the capture)
            hipGraph_t graph = nullptr;
            try {
                HIP_CHECK(hipStreamBeginCapture(s_comp_, hipStreamCaptureModeRelaxed));
                time_schedule(base, k, reps, true);
                HIP_CHECK(hipStreamEndCapture(s_comp_, &graph));
                HIP_CHECK(hipGraphInstantiate(&sg.exec, graph, nullptr, nullptr, 0));
                HIP_CHECK(hipGraphDestroy(graph));
                HIP_CHECK(hipGraphUpload(sg.exec, s_comp_));
            } catch (const Error& e) {
                hipGraph_t g2 = nullptr;
                hipStreamEndCapture(s_comp_, &g2);
                if (g2) hipGraphDestroy(g2);
                hipGetLastError();
                sg.exec = nullptr;
                sched_graph_failed_.insert(c);  // the candidate is dropped (agreed over the ranks)
                fprintf(stderr, "[gol] rank %d: schedule graph capture failed: %s\n", g_.rank, e.what());
            }
            sg.reps = reps;
        }
        if (sg.exec)
            HIP_CHECK(hipGraphLaunch(sg.exec, s_comp_));
        else
            time_schedule(base, k, reps, true);  // the same exchanges as the peers' replays
        return;
    }
    const bool split0 = split_;
    split_ = c == "split";
    const std::vector<int>& ps = pass_depths(k);
    for (int i = 0; i < reps; ++i) {
        first_pass(k, ps[0], ext_after(ps, 0), split_);
        for (size_t j = 1; j < ps.size(); ++j) {
            const i64 e = ext_after(ps, j);
            join_halo();
            launch(0, ps[j], e, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
            post(buf_[cur_ ^ 1], s_comp_, e);
        }
        // the next exchange waits for the whole superstep, as in tile_superstep (without this
        // record the timed split schedule overlapped each exchange with the previous superstep's
        // later passes, which a real run cannot: 2.78 timed vs 3.26 us/gen run, 4096 x 32768)
        if (ps.size() > 1) mark_ready();
    }
    split_ = split0;
}

// The kernels of a split superstep's first pass at depth k: the interior (kind 1) and the bands next to
// the halos (kind 2), each timed among step_temporal (where instantiated), the LDS tile kernel and, when
// the full tile runs step_pipe, step_pipe (the bands' passes at the depths of step_pipe passes are
// latency-bound: 10 stages x 2 generations stream a 60-row segment, where the tile kernel runs 20
// generations of barriers, 38 us for a 20-row band of config 3's strip; profiles/strip_split_round5.txt).
void HipEngine::tune_split_kinds(int k) {
    if (cfg_.kernel != "auto" && cfg_.kernel != "resident") return;
    std::vector<const char*> cands = {"temporal", "tile"};
    if (kern_[0] == "pipe") cands.push_back("pipe");
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    auto usable = [&](int kind, const char* c) {
        kern_[kind] = c;
        if (kern_[kind] == "tile") return tile_rows_cap(k) >= 1 && tile_rounds(kind, k, 0) <= kMaxTileRounds;
        if (kern_[kind] == "temporal") return hipk::step_depth_supported(k);
        return pipe_geo(k) != nullptr;
    };
    for (int kind : {1, 2})  // every plan first (plan building idles the GPU)
        for (const char* c : cands)
            if (usable(kind, c)) plan(kind, k, 0);
    spin_up();
    for (int kind : {1, 2}) {
        float bk = 1e30f, bpipe = 1e30f;
        const char* pk = "temporal";
        for (int round = 0; round < 2; ++round)
            for (const char* c : cands) {
                if (!usable(kind, c)) continue;
                launch(kind, k, 0, buf_[cur_], buf_[cur_ ^ 1], s_comp_);  // warm-up
                HIP_CHECK(hipEventRecord(e0, s_comp_));
                for (int i = 0; i < 3; ++i) launch(kind, k, 0, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
                HIP_CHECK(hipEventRecord(e1, s_comp_));
                HIP_CHECK(hipEventSynchronize(e1));
                float ms = 0;
                HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
                float per_gen = ms / 3 / (float)k;
                if (kern_[kind] == "pipe" && hipk::pipe_fault()) per_gen = 1e30f;  // a ring wait timed out
                init_step("init: split kernels", c, k, per_gen * 1e3f);
                const std::string key = strprintf("%d:%s@%d", kind, c, k);
                auto it = tune_ms_.find(key);
                tune_ms_[key] = it == tune_ms_.end() ? per_gen : std::min(it->second, per_gen);
                if (kern_[kind] == "pipe") bpipe = std::min(bpipe, per_gen);
                if (per_gen < bk) {
                    bk = per_gen;
                    pk = c;
                }
            }
        // The interior runs beside the exchange: a step_pipe interior (59 VGPRs per wave, 92 KiB of LDS per
        // workgroup) leaves every CU room for RCCL's kernel and the bands, the tile kernel does not, so
        // step_pipe is kept within 5% of the fastest alone (config 3's strip: interior tile@20 2.35 vs
        // pipe@20 2.37 us/gen alone, the split superstep 4.28 vs 3.52-3.58 us/gen with them;
        // profiles/strip_split_round5.txt)
        if (kind == 1 && bpipe <= 1.05f * bk) pk = "pipe";
        kern_[kind] = pk;
    }
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
    pipe_used_ = false;  // (the candidates ran on scratch; faults were checked above)
    passes_.clear();
}

// GOL_KERNEL=auto: for every plan kind a run uses (full tile; interior + boundary bands when
// split), time one superstep of each candidate kernel (into the scratch buffer, so the board is
// untouched) and keep the faster one.  The register pipeline wins on big regions; the
// LDS-resident tile kernel on small ones — its vertical halo is shared by a whole workgroup and
// its dependency chains are short, which is what the k-row boundary bands need.
void HipEngine::autotune_kernel() {
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
        const bool pipe = kern_[kind] == "pipe";
        hipStream_t s = s_comp_;
        launch(kind, k, 0, buf_[cur_], buf_[cur_ ^ 1], s);  // warm-up (and plan build)
        HIP_CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < 3; ++i) launch(kind, k, 0, buf_[cur_], buf_[cur_ ^ 1], s);
        HIP_CHECK(hipEventRecord(e1, s));
        HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        float per_gen = ms / 3 / (float)k;
        init_step("init: kernel autotune", kern, k, per_gen * 1e3f);
        if (pipe && hipk::pipe_fault()) {  // a ring wait timed out: never pick this geometry
            fprintf(stderr, "[gol] step_pipe %dx%d: a ring wait timed out in the kernel autotune; candidate dropped\n",
                    pipe_cur_.nw - 1, pipe_cur_.l);
            per_gen = 1e30f;
        }
        const std::string key = tile   ? strprintf("%d:%s@%dx%dw", kind, kern, k, cfg_.tile_waves)
                                : pipe ? strprintf("%d:pipe@%d(%dx%d,%d/CU)", kind, k, pipe_cur_.nw - 1, pipe_cur_.l, pipe_cur_.wg)
                                : occ_ ? strprintf("%d:%s@%d/%dw", kind, kern, k, occ_)
                                       : strprintf("%d:%s@%d", kind, kern, k);
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
        int pnw = 0, pl = 0, pwg = 0;  // pipe: waves per workgroup, generations per stage, workgroups per CU
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
    // The level-pipelined workgroup kernel (step_pipe) when the full-tile plan is the only kind a
    // superstep runs: 8 or 12 stages (balanced over the 4 SIMDs, with the loader), 2 or 3 generations
    // each.  kbench, one MI355X (docs/PERFORMANCE.md §13): 32768^2 8x3 at 2/CU 10.16-10.21 vs
    // temporal 10.56 us/gen; 4096 x 32768 12x3 2.15 vs 2.35; 16384^2 8x3 3.45 vs 3.61; 8192^2
    // loses to the folded tile kernel (1.50 vs 1.38).
    // (With neighbours it is the kernel of the "full" schedule's first pass and of the later passes;
    // when the schedule timing then picks "split", the interior / boundary kernels are tuned below
    // and the later passes run step_temporal at the measured depths.)
    if (!cfg_.compat && cfg_.kernel_depth == 0 && env_int("GOL_PIPE_TUNE", 1) != 0) {
        // ({16, 2, 1}: 15 waves x 2 levels, one workgroup per CU, the fastest geometry on config 3's
        // per-rank strip, 4096 x 32768: 2.10 vs 2.17 us/gen for {9, 3, 2}; profiles/strip_pipe_sweep.txt)
        const int geo[][3] = {{9, 3, 2}, {13, 2, 1}, {13, 3, 1}, {9, 2, 2}, {16, 2, 1}};
        for (const auto& g : geo) {
            const int k = (g[0] - 1) * g[1];
            if (k <= L_.R && hipk::pipe_supported(g[0], g[1])) cands.push_back({"pipe", k, nw0, 0, g[0], g[1], g[2]});
        }
    }
    for (const auto& c : cands) {
        occ_ = c.occ;
        if (c.pnw) set_pipe(c.pnw, c.pl, c.pwg);
        time_pass(0, c.kern, c.k, true);
    }
    spin_up();
    // Three interleaved rounds, best of each candidate: some candidates are within 1-2% of each
    // other (32768^2: the 3- and 2-waves/SIMD plans), and one 3-pass sample picks on noise.
    // Candidates more than 1.5x slower than the best one after the first round are not timed again
    // (they cannot win on noise; on a 2^20-row tile the losing step_pipe geometries took ~24 s of the
    // ~37 s init).
    std::vector<float> tbest(cands.size(), 1e30f);
    for (int round = 0; round < 3; ++round)
        for (size_t i = 0; i < cands.size(); ++i) {
            if (round > 0 && tbest[i] > 1.5f * *std::min_element(tbest.begin(), tbest.end())) continue;
            cfg_.tile_waves = cands[i].nw;
            occ_ = cands[i].occ;
            if (cands[i].pnw) set_pipe(cands[i].pnw, cands[i].pl, cands[i].pwg);
            tbest[i] = std::min(tbest[i], time_pass(0, cands[i].kern, cands[i].k));
        }
    // Near-ties (within 2% of the best) get four more interleaved rounds: on config 3's strip the
    // 15x2 and 8x3 step_pipe geometries time within 1-3% of each other, and one 3-round sample
    // picked the slower one in one init of two (2.17 vs 2.10 us/gen in the run;
    // profiles/strip_pipe_sweep.txt).
    {
        const float b0 = *std::min_element(tbest.begin(), tbest.end());
        std::vector<size_t> close;
        for (size_t i = 0; i < cands.size(); ++i)
            if (tbest[i] <= 1.02f * b0) close.push_back(i);
        if (close.size() > 1)
            for (int round = 0; round < 4; ++round)
                for (size_t i : close) {
                    cfg_.tile_waves = cands[i].nw;
                    occ_ = cands[i].occ;
                    if (cands[i].pnw) set_pipe(cands[i].pnw, cands[i].pl, cands[i].pwg);
                    tbest[i] = std::min(tbest[i], time_pass(0, cands[i].kern, cands[i].k));
                }
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
    if (pick.pnw) {
        set_pipe(pick.pnw, pick.pl, pick.pwg);
        tdepth_ = supported_kernel_depth(std::min(8, hipk::max_step_depth()));  // the remainders' depth
    } else {
        pipe_k_ = 0;
    }
    passes_.clear();
    // interior / boundary plans of split supersteps, at the chosen pass depth (tuned again at the
    // first-pass depth of the hinted superstep once the pass costs fix the cut: tune_split_kinds)
    if (split_used()) tune_split_kinds(kdepth_);
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
    kernel_ = kern_[0];
    pipe_used_ = false;  // (the candidates ran on scratch; faults were checked above)
    // The resident kernel (small boards without neighbours): one launch per run, halos exchanged
    // between tiles inside the kernel every kin generations.  Timed on launches of the hinted run's
    // length (at most 256 generations) against the best pass kernel above.
    if (resident_eligible() && !split_used()) {
        const int G = std::min(res_run_depth(), 256);
        float rbest = 1e30f;
        int rk = 0;
        for (int kin : {8, 12, 16, 24}) {
            if (cfg_.kernel_depth > 0 && kin != cfg_.kernel_depth) continue;
            const float t = time_resident(kin, G);
            if (t < 1e29f) tune_ms_[strprintf("0:resident@%d", kin)] = t;
            if (t < rbest) {
                rbest = t;
                rk = kin;
            }
        }
        if (rk && (cfg_.kernel == "resident" || rbest < best)) {
            res_ = true;
            res_kin_ = rk;
            passes_.clear();
        } else if (cfg_.kernel == "resident") {
            throw Error("GOL_KERNEL=resident: this board does not fit the resident kernel");
        }
    } else if (cfg_.kernel == "resident") {
        throw Error("GOL_KERNEL=resident needs a rank without neighbours, a 1-D tile of width % 64 == 0 and >= 64 rows");
    }
}

void HipEngine::device_barrier() {
    synchronize();
    t_->barrier();
    if (device_transport_) {
        t_->device_barrier((void*)s_comp_);
        Armed armed(wd_.get());
        HIP_CHECK(hipStreamSynchronize(s_comp_));
    }
}

// Per-phase costs for the scaling model (docs/PERFORMANCE.md): the exchange of a k-deep halo alone,
// and whole k-generation supersteps of the chosen schedule, timed with events on scratch state
// (time_schedule) after the board has been synchronised back to the canonical buffer.  Collective:
// every rank runs the same exchanges; rounds start from a host barrier.
std::map<std::string, double> HipEngine::phase_probe(int k) {
    Armed armed(wd_.get());
    std::map<std::string, double> out;
    k = supported_depth(std::max(1, std::min(k, superstep_depth())));
    if (res_) {  // one resident launch per superstep, timed on scratch boards
        out["superstep_us"] = (double)time_resident(res_kin_, k) * 1e3 * k;
        out["superstep_gens"] = k;
        return out;
    }
    sync_canonical();
    synchronize();
    const EngineStats saved = stats_;
    const bool was_dual = dual_, was_split = split_;
    const int was_ov = sub_overlap_;
    hipEvent_t e0, e1;
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    auto elapsed_us = [&] {
        HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        return (double)ms * 1e3;
    };
    const bool xchg = dual_ ? !self_y() : !items_for(k).empty();
    if (xchg) {
        if (!dual_) prepare(k);
        double best = 1e30;
        for (int round = 0; round < 4; ++round) {
            t_->barrier();
            HIP_CHECK(hipEventRecord(e0, s_comp_));
            if (dual_) {
                std::vector<Message> sends, recvs;
                dual_messages(sub_cur_, k, sends, recvs);
                exchange_rows(sends, recvs, s_comp_);
            } else if (device_transport_) {
                exchange_device(k, items_for(k), cur_, s_comp_);
            } else {
                exchange_staged(k, items_for(k), cur_, s_comp_);
            }
            HIP_CHECK(hipEventRecord(e1, s_comp_));
            const double us = elapsed_us();
            if (round > 0) best = std::min(best, us);  // round 0 warms the connections up
        }
        out["exchange_us"] = best;
    }
    // the schedule the runs use, as choose_schedule timed it (graph variants included)
    std::string sched = sched_pick_;
    if (sched.empty())
        sched = dual_ ? (sub_overlap_ ? "subtiles+ov" : "subtiles")
                      : (split_ ? "split" : (halo_items(L_.R).empty() ? "local" : "full"));
    const int reps = 2;
    double best = 1e30;
    for (int round = 0; round < 3; ++round) {
        t_->barrier();
        HIP_CHECK(hipEventRecord(e0, s_comp_));
        if (was_dual) HIP_CHECK(hipStreamWaitEvent(s_comm_, e0, 0));
        time_schedule(sched, k, reps);
        if (was_dual) HIP_CHECK(hipStreamWaitEvent(s_comp_, ev_sub_b_, 0));
        HIP_CHECK(hipEventRecord(e1, s_comp_));
        best = std::min(best, elapsed_us() / reps);
    }
    out["superstep_us"] = best;
    out["superstep_gens"] = k;
    synchronize();
    destroy_sched_graphs();
    HIP_CHECK(hipEventDestroy(e0));
    HIP_CHECK(hipEventDestroy(e1));
    dual_ = was_dual;
    sub_overlap_ = was_ov;
    split_ = was_split;
    if (dual_) {
        sub_current_ = false;  // the halves hold probe scratch: reload the board at the next run
        canon_stale_ = false;
    }
    stats_ = saved;  // the probe's exchanges and supersteps are not part of any run
    return out;
}

}  // namespace hipeng
}  // namespace gol
