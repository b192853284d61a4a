// gol-mi355x: HipEngine — supersteps as ONE dependency-driven launch (step_flow, flow_kernel.hip).
//
// A one-tile superstep of k generations normally runs k / K kernel passes, each a launch that starts
// only when the previous pass's last wave has drained (docs/PERFORMANCE.md §6).  In flow mode the
// whole superstep is one launch of a persistent grid: the passes' plan waves become work items in one
// ticket order, and each item waits only for the items of the previous pass it reads from or
// overwrites (plan.hpp build_flow_plan).  With neighbours the exchange runs first on the compute
// stream (the "full" schedule: the first pass reads the ghost rows it wrote), or ("flow+ov") on the
// comm stream while the launch's interior items run.  Opt-in (GOL_SCHEDULE=flow|flow+ov forces it,
// GOL_FLOW=1 makes it a candidate of the schedule timing, engine_hip_tune.hip): it measured slower
// than the pass schedules on every configuration (docs/PERFORMANCE.md §15).
// Reference: the generation loop gol-main.c:93-116, one launch + device sync per generation in
// gol-with-cuda.cu:264-284.
#include <algorithm>
#include <map>
#include <mutex>

#include "hip_engine.hpp"

namespace gol {
namespace hipeng {

namespace {
std::mutex g_dev_mu;
std::map<int, std::vector<const HipEngine*>> g_dev_engines;
}  // namespace

std::pair<int, int> HipEngine::engines_on_device(int dev, const HipEngine* e, int op) {
    std::lock_guard<std::mutex> lk(g_dev_mu);
    std::vector<const HipEngine*>& v = g_dev_engines[dev];
    auto it = std::find(v.begin(), v.end(), e);
    if (op > 0 && it == v.end()) v.push_back(e);
    if (op < 0 && it != v.end()) v.erase(it);
    it = std::find(v.begin(), v.end(), e);
    return {it == v.end() ? -1 : (int)(it - v.begin()), (int)v.size()};
}

// The CU-restricted compute stream of flow+ov (hip_engine.hpp kOvReservedCus): CUs [0, cus - reserved)
// split evenly over the engines of this device, so the top kOvReservedCus stay free for the exchange's
// kernels on the (unrestricted) comm stream.
bool HipEngine::ov_stream() {
    if (s_ov_) return true;
    const std::pair<int, int> sn = engines_on_device(dev_, this, 0);
    const int usable = cus_ - kOvReservedCus;
    if (sn.first < 0 || usable < sn.second) return false;
    const int lo = (int)((i64)sn.first * usable / sn.second), hi = (int)((i64)(sn.first + 1) * usable / sn.second);
    std::vector<u32> mask((size_t)(cus_ + 31) / 32, 0u);
    for (int c = lo; c < hi; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
    hipStream_t s = nullptr;
    if (hipExtStreamCreateWithCUMask(&s, (u32)mask.size(), mask.data()) != hipSuccess || !s) {
        (void)hipGetLastError();
        return false;
    }
    s_ov_ = s;
    ov_cus_ = hi - lo;
    return true;
}

bool HipEngine::flow_eligible() {
    // one tile; every pass is a step_temporal pass (no LDS-tile / pipe / LDS kernels, no split bands);
    // ghost words of a non-aligned self-wrapping width are refreshed by a kernel after every pass,
    // which a single launch cannot do
    if (cfg_.compat || cfg_.profile || cfg_.force_split || kernel_ == "lds" || res_) return false;
    if (cfg_.kernel == "pipe" || cfg_.kernel == "resident") return false;
    return !(self_x() && !L_.aligned());
}

// Passes of a flow superstep: as few as the items' deepest depth allows, as equal as possible
// (20 = 7 + 7 + 6).  GOL_FLOW_KMAX lowers the deepest depth (measurement knob).
std::vector<int> HipEngine::flow_cut(int k) {
    auto cut = [&](int deepest) {
        const int kmax = std::max(1, std::min<int>(deepest, (int)env_int("GOL_FLOW_KMAX", deepest)));
        const int n = (k + kmax - 1) / kmax;
        std::vector<int> ps;
        for (int j = 0; j < n; ++j) ps.push_back(k / n + (j < k % n ? 1 : 0));
        return ps;
    };
    // tile items: passes of the tuned tile depth (any depth runs), when their variant has a flow twin;
    // waves: the flow kernel's deepest
    if (flow_tiles()) {
        std::vector<int> ps = cut(std::max(1, kdepth_));
        if (flow_tile_cut_ok(ps)) return ps;
    }
    return cut(hipk::flow_max_depth());
}

bool HipEngine::flow_tile_cut_ok(const std::vector<int>& ps) {
    if (!flow_tiles() || ps.empty()) return false;
    const int kmax = *std::max_element(ps.begin(), ps.end());
    return hipk::flow_tile_supported(cfg_.tile_waves, step_flags() | plan(0, kmax, ext_after(ps, 0)).tflags);
}

const HipEngine::FlowDev& HipEngine::flow_plan(int k) {
    const bool ov = flow_ov_active(k);
    const int key = k * 2 + (ov ? 1 : 0);
    auto it = flow_plans_.find(key);
    if (it != flow_plans_.end()) return it->second;
    if (ov && !ov_stream()) throw Error("flow plan: no CU-restricted stream for the exchange-overlapped launch");
    const i64 cus = flow_cus(ov);
    if (!flow_ctl_) {
        HIP_CHECK(hipMalloc(&flow_ctl_, sizeof(hipk::FlowCtl)));
        HIP_CHECK(hipMemsetAsync(flow_ctl_, 0, sizeof(hipk::FlowCtl), s_comp_));
    }
    const std::vector<int> ps = flow_cut(k);
    const bool wrapy = (step_flags() & hipk::STEP_WRAP_Y) != 0;
    FlowDev fd;
    std::vector<FlowPass> fps;
    const int kmax = *std::max_element(ps.begin(), ps.end());
    if (flow_tile_cut_ok(ps)) {
        // LDS tile items: every pass uses the tile variant and chunk height of the deepest pass's plan
        // (a shallower pass needs less LDS), capped at the flow variant's capacity (its ticket slot)
        const DevPlan& p0 = plan(0, kmax, ext_after(ps, 0));
        fd.tile = true;
        fd.kmax = kmax;
        fd.tflags = p0.tflags;
        const u32 f = step_flags() | p0.tflags;
        fd.rows = std::min<i64>(p0.rows, hipk::flow_tile_max_rows(kmax, cfg_.tile_waves, f));
        if (p0.fold && fd.rows < hipk::kFoldMinRows) throw Error("flow plan: folded tiles do not fit with the ticket slot");
        fd.blocks = (i64)hipk::flow_tile_blocks_per_cu(cfg_.tile_waves, fd.rows, kmax, f) * cus;
        for (size_t j = 0; j < ps.size(); ++j)
            fps.push_back({ps[j], regions(0, ps[j], ext_after(ps, j)), fd.rows, p0.fold});
    } else {
        fd.blocks = (i64)hipk::flow_blocks_per_cu(step_flags()) * cus;
        const i64 resident = fd.blocks * kWavesPerBlock;
        // items per pass: one round of the persistent grid (GOL_FLOW_ROUNDS in percent scales it; big
        // tiles take several rounds of ~45K-row segments, as the pass kernels' plans)
        const double scale = (double)env_int("GOL_FLOW_ROUNDS", 100) / 100.0;
        for (size_t j = 0; j < ps.size(); ++j) {
            const std::vector<Region> rg = regions(0, ps[j], ext_after(ps, j));
            const i64 target = std::max<i64>(1, (i64)(scale * (double)resident));
            const i64 rows = round_balanced_rows(rg, L_.nw, L_.h, ps[j], target, 2 * (i64)ps[j], xwrap_by_plan(),
                                                 round_rows(ps[j]));
            fps.push_back({ps[j], rg, rows});
        }
    }
    FlowPlan fp;
    const std::string err = build_flow_plan(fps, L_.nw, L_.h, xwrap_by_plan(), wrapy, fp, ov);
    if (!err.empty()) throw Error("flow plan: " + err);
    for (size_t j = 0; j < ps.size(); ++j) {
        const std::vector<LaneDesc> part(fp.lanes.begin() + (size_t)fp.pass_begin[j] * kWaveLanes,
                                         fp.lanes.begin() + (size_t)fp.pass_begin[j + 1] * kWaveLanes);
        const std::string bad = validate_plan(part, L_.nw, L_.h, L_.R, ps[j], wrapy);
        if (!bad.empty())
            throw Error(strprintf("refusing to launch an unsafe flow plan (k %d, pass %zu): %s", k, j, bad.c_str()));
    }
    fd.cut = ps;
    fd.n_items = (u32)fp.items.size();
    fd.st = fp.st;
    fd.max_deps = fp.max_deps;
    HIP_CHECK(hipMalloc(&fd.lanes, std::max<size_t>(1, fp.lanes.size()) * sizeof(LaneDesc)));
    HIP_CHECK(hipMalloc(&fd.items, std::max<size_t>(1, fp.items.size()) * sizeof(FlowItem)));
    HIP_CHECK(hipMalloc(&fd.deps, std::max<size_t>(1, fp.deps.size()) * sizeof(u32)));
    HIP_CHECK(hipMalloc(&fd.flags, std::max<size_t>(1, fp.items.size()) * sizeof(u32)));
    if (!fp.lanes.empty()) upload(fd.lanes, fp.lanes.data(), fp.lanes.size() * sizeof(LaneDesc));
    if (!fp.items.empty()) upload(fd.items, fp.items.data(), fp.items.size() * sizeof(FlowItem));
    if (!fp.deps.empty()) upload(fd.deps, fp.deps.data(), fp.deps.size() * sizeof(u32));
    // flags start below every epoch a launch will wait for
    HIP_CHECK(hipMemsetAsync(fd.flags, 0, std::max<size_t>(1, fp.items.size()) * sizeof(u32), s_comp_));
    HIP_CHECK(hipStreamSynchronize(s_comp_));
    return flow_plans_.emplace(key, fd).first->second;
}

void HipEngine::flow_launch(int k, const u64* src, u64* dst, hipStream_t s) {
    const FlowDev& fd = flow_plan(k);
    if (fd.n_items == 0) return;
    hipk::FlowArgs a{};
    a.a = const_cast<u64*>(src);  // (pass 0 reads it; an odd pass count never writes it, an even one does)
    a.b = dst;
    a.lanes = fd.lanes;
    a.items = fd.items;
    a.deps = fd.deps;
    a.flags = fd.flags;
    a.ctl = flow_ctl_;
    a.n_items = fd.n_items;
    a.epoch = next_flow_epoch();
    // one ticket sequence per XCD, or one for all while another engine shares the device (its grid may
    // hold a whole XCD: flow_kernel.hip, deadlock freedom)
    if (flow_nseq_ <= 0) {
        int x = 1;
        if (hipDeviceGetAttribute(&x, hipDeviceAttributeNumberOfXccs, dev_) != hipSuccess || x < 1) x = 1;
        flow_nseq_ = std::min(x, hipk::kFlowSeqs);
    }
    a.nseq = engines_on_device(dev_, this, 0).second > 1 ? 1u : (u32)flow_nseq_;
    hipk::StepParams sp{L_.pitch, (i32)L_.h, (i32)L_.nw, L_.R, step_flags() | fd.tflags};
    if (fd.tile)
        hipk::launch_step_flow_tile(cfg_.tile_waves, a, fd.blocks, fd.rows, fd.kmax, sp, s);
    else
        hipk::launch_step_flow(a, fd.blocks, sp, s);
    HIP_CHECK(hipGetLastError());
    flow_epoch_ = a.epoch;
    flow_used_ = true;
}

// One flow superstep: (with neighbours) the exchange of the k-deep halo, then the single launch; the
// result lands in buf[cur ^ (passes & 1)].
//   "flow":    the exchange on the compute stream, then the launch (its first pass reads the ghost rows).
//   "flow+ov": the exchange on the comm stream (after the previous superstep's launch, ev_ready_),
//              followed by a device flag (hipStreamWriteValue32 of the launch's epoch); the launch goes
//              to the compute stream
//              at once, with no cross-queue event wait.  Its plan (build_flow_plan mark_exch) runs the
//              items from the middle of the tile outwards and makes the first pass's items that read
//              ghost cells wait for the flag, so the interior hides the exchange and only the bands next
//              to the halos wait for it.  Pass 1 overwrites the edge rows the exchange sends; its items
//              there depend on those flag-waiting items, so they start only after the exchange is done.
void HipEngine::flow_superstep(int k) {
    const std::vector<int>& ps = pass_depths(k);
    const std::vector<HaloItem>& items = items_for(k);
    if (flow_ov_active(k)) {
        if (s_comp_ != s_ov_) throw Error("flow+ov superstep outside the CU-restricted compute stream");
        flow_plan(k);  // (allocates the control block the flag lives in)
        prepare(k);
        HIP_CHECK(hipStreamWaitEvent(s_comm_, ev_ready_, 0));
        exchange_device(k, items, cur_, s_comm_);
        HIP_CHECK(hipStreamWriteValue32(s_comm_, &flow_ctl_->exch, next_flow_epoch(), 0));
        flow_launch(k, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
        if (ps.size() & 1) cur_ ^= 1;
        HIP_CHECK(hipEventRecord(ev_ready_, s_comp_));  // the next exchange reads this launch's edge rows
        return;
    }
    if (!items.empty()) {
        prepare(k);
        if (device_transport_)
            exchange_device(k, items, cur_, s_comp_);
        else
            exchange_staged(k, items, cur_, s_comp_);
    }
    flow_launch(k, buf_[cur_], buf_[cur_ ^ 1], s_comp_);
    if (ps.size() & 1) cur_ ^= 1;
    mark_ready();
}

}  // namespace hipeng
}  // namespace gol
