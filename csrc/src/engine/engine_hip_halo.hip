// gol-mi355x: HipEngine — halo exchange: copy lists, device transport (RCCL) and host staging.
#include "hip_engine.hpp"

namespace gol {
namespace hipeng {

void HipEngine::prepare(int k) {
    if (res_) {
        res_plan(res_kin_);
        return;
    }
    const std::vector<int>& ps = pass_depths(k);
    plan(0, ps[0], ext_after(ps, 0));
    if (split_used()) {  // (only split supersteps run the interior / band plans)
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

const DevCopies& HipEngine::copies(int k, int parity) {
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

void HipEngine::build_messages(int k, const std::vector<HaloItem>& items, int parity, std::vector<Message>& sends,
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

void HipEngine::exchange_device(int k, const std::vector<HaloItem>& items, int parity, hipStream_t s) {
    trace::Range r("gol.exchange_device");
    guard_exchange_stream(s);
    const DevCopies& dc = copies(k, parity);
    if (dc.npack) hipk::launch_copy_regions(dc.pack, dc.npack, dc.max_pack, s);
    std::vector<Message> sends, recvs;
    build_messages(k, items, parity, sends, recvs);
    t_->exchange(sends, recvs, (void*)s);
    if (dc.nunpack) hipk::launch_copy_regions(dc.unpack, dc.nunpack, dc.max_unpack, s);
    HIP_CHECK(hipGetLastError());
    account(items);
}

void HipEngine::exchange_staged(int k, const std::vector<HaloItem>& items, int parity, hipStream_t s) {
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

void HipEngine::record_profile(bool with_exchange) {
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

}  // namespace hipeng
}  // namespace gol
