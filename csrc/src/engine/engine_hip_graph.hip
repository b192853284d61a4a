// gol-mi355x: HipEngine — hipGraph capture and replay of one-tile supersteps.
#include "hip_engine.hpp"

namespace gol {
namespace hipeng {

// Graph shape of run(): m supersteps of k generations per replay; false when run() stays eager.
bool HipEngine::graph_shape(int& k, int& m) {
    if (!cfg_.graph || cfg_.profile) return false;
    // Sub-tile supersteps are not captured as a whole: captured with their fork/join across two
    // streams they replayed slower than eager launches on MI355X / ROCm 7.2 (32768^2: 14.2 vs
    // 12.8 us/gen over 20 generations, 13.0 vs 10.4 over 256; profiles/short_run_probe.txt).
    // (A single-stream graph per half and superstep measured slower too: engine_hip_subtiles.hip.)
    if (dual_) return false;
    k = cfg_.compat ? 1 : superstep_depth();
    m = cfg_.graph_supersteps;
    if (m <= 0) m = k >= 8 ? 16 : 32;
    m += m & 1;  // even: the graph returns to the same buffer parity
    bool local = cfg_.compat || halo_items(k).empty();
    if (!local && !device_transport_) return false;  // host-staged exchange cannot be captured
    // RCCL inside captured graphs: a candidate of the schedule timing ("full+graph", choose_schedule)
    // or forced with GOL_GRAPH_RCCL=1; eager otherwise (an eager exchange keeps RCCL's own error
    // handling, and with R-deep supersteps the eager launch cost is small).
    if (!local && !graph_rccl_on_) return false;
    // Split supersteps with an exchange stay eager: captured (the RCCL group on the capture's origin
    // stream, the interior on a forked one) the exchange kernel started ~140 us into the replay,
    // 5.5 ms per 20-generation strip run against 4.1-4.9 eager (profiles/strip_split_round5.txt).
    // (GOL_GRAPH_SPLIT=1, a test knob, attempts that capture anyway: guard_exchange_stream refuses the
    // exchange on the comm stream, the capture fails and the supersteps run eagerly)
    if (!local && split_ && !split_capture_test_) return false;
    return true;
}

std::vector<HipEngine::Shape> HipEngine::graph_ladder(int k, int M) const {
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

// Capture and instantiate the replay graphs at init, so no timed run() ever pays for
// stream capture or graph instantiation (a 16-superstep capture costs milliseconds: more than
// a whole 8192^2 x 1000 run).
void HipEngine::prewarm_graph() {
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
// graph replays none), every ladder shape captured at init.  The remainder no shape covers runs
// eagerly.  (A graph of that one short remainder, captured on first use, did not change the 8192^2
// warmup anomaly, docs/PERFORMANCE.md §6, and was removed.)
void HipEngine::run_graphed(u64& generations) {
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

void HipEngine::replay(hipGraphExec_t exec, int k, int m, int rem) {
    const u64 per = (u64)m * (u64)k + (u64)rem;
    maybe_inject_fault();
    join_halo();
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

hipGraphExec_t HipEngine::graph_for(int k, int m, int rem) {
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
    join_halo();  // (never inside the capture)
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

}  // namespace hipeng
}  // namespace gol
