// gol-mi355x: HipEngine — two sub-tiles per rank (1-D), each half on its own stream.
#include "hip_engine.hpp"

namespace gol {
namespace hipeng {

void HipEngine::setup_dual() {
    if (sub_buf_[0][0]) return;
    // equal halves (52/48 and 48/52 splits measured no better: docs/PERFORMANCE.md §6)
    const i64 frac = 500;
    const i64 h0 = std::max<i64>(8 * (i64)L_.R, std::min<i64>(L_.h - 8 * (i64)L_.R, L_.h * frac / 1000));
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
    if (!ev_sub_own_[0]) {
        for (auto& e : ev_sub_own_) HIP_CHECK(hipEventCreateWithFlags(&e, event_flags()));
        HIP_CHECK(hipEventCreateWithFlags(&ev_sub_x_, event_flags()));
        ev_sub_a_ = ev_sub_own_[0];
        ev_sub_b_ = ev_sub_own_[1];
    }
    HIP_CHECK(hipStreamSynchronize(s_comp_));
}

// Free the sub-tile buffers, plans and copy lists (the measurement chose one tile).
void HipEngine::teardown_dual() {
    synchronize();
    for (auto& kv : sub_plans_) hipFree(kv.second.d);
    sub_plans_.clear();
    for (auto& sb : sub_buf_)
        for (u64*& b : sb) {
            if (b) hipFree(b);
            b = nullptr;
        }
    dual_ = false;
    sub_overlap_ = 0;
    sub_current_ = canon_stale_ = false;
}

const DevPlan& HipEngine::sub_plan(int s, int k, i64 e, int part) {
    const int key = part * 1000000 + s * 100000 + (int)e * 100 + k;
    auto it = sub_plans_.find(key);
    if (it != sub_plans_.end()) return it->second;
    const Layout& L = sub_L_[s];
    // output rows -e .. h+e; part 1 stops k rows short of the rank's halo (half 0: starts k rows
    // below its top, half 1: ends k rows above its bottom), so its inputs never reach the ghost rows
    // the exchange writes; part 2 is that band
    std::vector<Region> rg = {{-e, L.h + e, 0, L.nw}};
    if (part == 1) (s == 0 ? rg[0].r0 : rg[0].r1) = s == 0 ? k : L.h - k;
    if (part == 2) (s == 0 ? rg[0].r1 : rg[0].r0) = s == 0 ? k : L.h - k;
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
        // the two halves' kernels must fit on the SIMDs together: a depth whose kernel holds only 2
        // waves per SIMD (K=12) gets 1-wave plans, or the second half waits for the first one's
        // waves to retire (20-generation runs cut 12 + 8 took 14.5-14.8 instead of 11.8 us/gen in a
        // quarter of the runs, profiles/pingpong_loop_ab.txt)
        if (hipk::step_blocks_per_cu(k, sub_flags()) <= 2) bpc = 1;
    }
    // A band (part 2) is a few rows tall and runs while little else does: its time is the serial
    // level pipeline of one wave, ~(S + K) x K row-levels for S rows per wave, so it is cut into
    // 4-row segments (K = 12, 28-row band: ~38 us as one segment per column, ~14 us in 4-row ones;
    // 23 us measured in the driver-cut trace, profiles/kernel_trace_selfx_round4.txt; the band on the
    // LDS tile kernel instead, one workgroup per 62-word column, measured no faster end to end:
    // profiles/selfx_band_and_order_ab.txt).
    // One round per half even on big tiles: the two halves' kernels already fill each other's tails
    // (131072^2: multi-round halves 141.9-142.4 vs 140.2-141.0 us/gen, profiles/bigboard_rounds.txt).
    const i64 rows = part == 2 ? 4
                               : balanced_rows_per_chunk(rg, L.nw, L.h, k, bpc * kWavesPerBlock * cus_, 2 * (i64)k, true);
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

// One sub-tile superstep: sub-tile 0 on the compute stream, 1 on the second stream.
void HipEngine::dual_superstep(int k) {
    prepare_dual(k);
    const int p = sub_cur_;
    const int a = (p + 1) % 3, b = (p + 2) % 3;  // the passes alternate a, b, a, ... (never p)
    wait_pending(s_comp_, ev_sub_b_);  // half 1's previous superstep is done
    // With neighbours, half 0's first pass can start before the exchange: all its output rows but
    // the k next to the north halo read only rows the halves already hold (its own, and half 1's
    // edge across the seam); that band runs after the exchange.  The exchange then goes on the
    // second stream, the one of greatest priority, so the RCCL kernel is dispatched ahead of the
    // half-tile kernel when both become ready (a kernel that has filled the CUs first would hold
    // it back).  Chosen by measurement (schedule "subtiles+ov"): it costs a second, small kernel
    // per superstep.  (Both halves' interiors first, with the exchange between half 0's interior
    // and its band, measured slower everywhere: 13.2-13.7 vs 12.7-12.8 us/gen at 20 generations
    // through the RCCL self-exchange, the exchange and its ~10 us tail then sit on half 0's critical
    // path; docs/PERFORMANCE.md section 6.  Round 5: the exchange first on the compute stream with half
    // 1's interior beside it, 12.36-12.52 against 12.30-12.64, and the exchange replayed from a captured
    // graph, no faster either; both removed, profiles/strip_split_round5.txt.)
    const bool ov = sub_overlap_ == 1 && !self_y();
    if (!self_y()) {
        hipStream_t xs = s_comp_;
        if (ov) {
            launch_half(0, p, k, s_comp_, 0, 1);
            wait_pending(s_comm_, ev_sub_a_);  // the exchange sends half 0's edge and writes its halo
            xs = s_comm_;
        }
        std::vector<Message> sends, recvs;
        dual_messages(p, k, sends, recvs);
        exchange_rows(sends, recvs, xs);
        stats_.exchanges += 1;
        stats_.halo_bytes += (u64)(rows_bytes(0, k) + rows_bytes(1, k));
        // (full: also implies half 0's previous superstep, which ran on the same stream)
        HIP_CHECK(hipEventRecord(ev_sub_x_, xs));
        HIP_CHECK(hipStreamWaitEvent(ov ? s_comp_ : s_comm_, ev_sub_x_, 0));
        if (ov) launch_half(0, p, k, s_comp_, 0, 2);
    } else {
        wait_pending(s_comm_, ev_sub_a_);  // half 0's previous superstep is done
    }
    // Each half's passes: eager launches on its stream, alternating between the halves (pass j of
    // half 0, pass j of half 1, ...: issued half by half, the second stream's first kernel started
    // ~20 us after the first's, three host launches later, and the superstep ended on one half's
    // lone tail; kernel traces of the driver's 20-generation bench).  The cross-half order stays in
    // the events around them.  (Per-half graphs of these passes, replayed per superstep, measured
    // slower than the eager launches on MI355X / ROCm 7.2: 20 generations 13.06-13.23 vs 12.75-12.96
    // us/gen, 2000 generations 10.35 vs 10.24; profiles/subtile_graphs_ab.txt.)
    const int np = (int)pass_depths(k).size();
    for (int j = 0; j < np; ++j)
        for (int s = 0; s < 2; ++s) {  // half 0's pass first (half 1 first measured no better: docs/PERFORMANCE.md §6)
            if (ov && s == 0 && j == 0) continue;
            if (j == 0 && s == 0) trace::mark("gol.launch0");  // (GOL_ROCTX: host side of the launch latency)
            launch_half(s, p, k, s ? s_comm_ : s_comp_, j);
            if (j == 0 && s == 0) trace::mark("gol.launch0_done");
        }
    if (wd_) {
        // with a watchdog the end-of-superstep events are the superstep's progress marker (a fresh
        // pair from the marker ring; ev_sub_a_ / ev_sub_b_ always name the latest pair)
        Marker& m = marker_slot();
        ev_sub_a_ = m.ev[0];
        ev_sub_b_ = m.ev[1];
        m.n = 2;
    }
    events_synced_ = false;
    HIP_CHECK(hipEventRecord(ev_sub_a_, s_comp_));
    HIP_CHECK(hipEventRecord(ev_sub_b_, s_comm_));
    if (wd_) {
        publish_marker();
        mk_published_ = true;
    }
    HIP_CHECK(hipGetLastError());
    sub_cur_ = (pass_depths(k).size() % 2) ? a : b;
}

// The one-tile engine's canonical messages (Engine::halo_items, 1-D): N then S, from / into the
// halves' buffer p.
void HipEngine::dual_messages(int p, int k, std::vector<Message>& sends, std::vector<Message>& recvs) {
    const i64 h1 = sub_L_[1].h;
    sends.push_back({g_.nbr[DIR_N], sub_rows(0, p, 0), rows_bytes(0, k)});
    recvs.push_back({g_.nbr[DIR_S], sub_rows(1, p, h1), rows_bytes(1, k)});
    sends.push_back({g_.nbr[DIR_S], sub_rows(1, p, h1 - k), rows_bytes(1, k)});
    recvs.push_back({g_.nbr[DIR_N], sub_rows(0, p, -k), rows_bytes(0, k)});
}

// Device transports (RCCL) are stream ordered on `s`.  Host transports are staged through pinned
// host memory and block: the rows to send are complete once `s` has drained (the caller orders both
// halves' previous superstep before `s`), the receives land on `s`.
void HipEngine::exchange_rows(const std::vector<Message>& sends, const std::vector<Message>& recvs, hipStream_t s) {
    if (device_transport_) {
        t_->exchange(sends, recvs, (void*)s);
        return;
    }
    trace::Range r("gol.exchange_staged");
    size_t need = 0;
    for (const auto* v : {&sends, &recvs})
        for (const Message& m : *v) need = std::max(need, m.bytes);
    if (xhs_.size() < sends.size() || xhr_.size() < recvs.size() || need > xh_bytes_) {
        HIP_CHECK(hipStreamSynchronize(s));
        for (auto* v : {&xhs_, &xhr_}) {
            for (u64* q : *v) HIP_CHECK(hipHostFree(q));
            v->clear();
        }
        xh_bytes_ = std::max(need, (size_t)rows_bytes(0, L_.R));
        for (size_t i = 0; i < sends.size(); ++i) {
            u64* q = nullptr;
            HIP_CHECK(hipHostMalloc(&q, xh_bytes_, hipHostMallocDefault));
            xhs_.push_back(q);
        }
        for (size_t i = 0; i < recvs.size(); ++i) {
            u64* q = nullptr;
            HIP_CHECK(hipHostMalloc(&q, xh_bytes_, hipHostMallocDefault));
            xhr_.push_back(q);
        }
    }
    std::vector<Message> hs, hr;
    for (size_t i = 0; i < sends.size(); ++i) {
        HIP_CHECK(hipMemcpyAsync(xhs_[i], sends[i].buf, sends[i].bytes, hipMemcpyDeviceToHost, s));
        hs.push_back({sends[i].peer, xhs_[i], sends[i].bytes});
    }
    for (size_t i = 0; i < recvs.size(); ++i) hr.push_back({recvs[i].peer, xhr_[i], recvs[i].bytes});
    HIP_CHECK(hipStreamSynchronize(s));
    t_->exchange_host(hs, hr);
    for (size_t i = 0; i < recvs.size(); ++i)
        HIP_CHECK(hipMemcpyAsync(recvs[i].buf, xhr_[i], recvs[i].bytes, hipMemcpyHostToDevice, s));
}

// The kernel passes of half s in a superstep of k generations that starts from buffer p (only
// pass `only` when >= 0; `part` selects a sub_plan part for the first pass).
void HipEngine::launch_half(int s, int p, int k, hipStream_t st, int only, int part) {
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
            const DevPlan& pl = sub_plan(s, ps[j], ext_after(ps, j), j == 0 ? part : 0);
            hipk::launch_step(ps[j], sub_buf_[s][q], sub_buf_[s][dsti], pl.d, pl.waves, j == 0 ? sp0 : sp, st);
        }
        q = dsti;
    }
}

}  // namespace hipeng
}  // namespace gol
