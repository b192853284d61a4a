// gol-mi355x: RCCL data plane over xGMI.
//
// Replaces the reference's per-generation MPI_Irecv/Isend/Wait of managed-memory byte rows
// (gol-main.c:97-111) with one ncclGroupStart/End per superstep of ncclSend/ncclRecv on device
// pointers, enqueued on the engine's comm stream (stream ordered, graph capturable).  Messages are
// k rows deep, so one group serves k generations.  The control plane (unique-id broadcast,
// barriers, timing reductions) is delegated to a host transport (TCP / MPI / threads /
// torch.distributed callback).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

#include "gol/transport.hpp"

namespace gol {

namespace {

void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw Error(strprintf("%s failed: %s", what, ncclGetErrorString(r)));
}

class RcclTransport : public Transport {
   public:
    RcclTransport(std::shared_ptr<Transport> control, const ncclUniqueId& id) : ctl_(std::move(control)) {
        nccl_check(ncclCommInitRank(&comm_, ctl_->size(), id, ctl_->rank()), "ncclCommInitRank");
    }
    ~RcclTransport() override {
        if (comm_) ncclCommDestroy(comm_);
        if (dbuf_) (void)hipFree(dbuf_);
    }
    int rank() const override { return ctl_->rank(); }
    int size() const override { return ctl_->size(); }
    std::string name() const override { return "rccl+" + ctl_->name(); }
    void send_bytes(int peer, const void* buf, size_t n) override { ctl_->send_bytes(peer, buf, n); }
    void recv_bytes(int peer, void* buf, size_t n) override { ctl_->recv_bytes(peer, buf, n); }
    bool device_buffers() const override { return true; }
    bool graph_capturable() const override { return true; }

    void exchange(const std::vector<Message>& sends, const std::vector<Message>& recvs, void* stream) override {
        // Canonical order: sends[i] and recvs[i] belong to the same direction; RCCL matches
        // per peer in issue order, which is identical on both sides of every pair.
        hipStream_t s = (hipStream_t)stream;
        nccl_check(ncclGroupStart(), "ncclGroupStart");
        for (size_t i = 0; i < sends.size(); ++i) {
            const Message& a = sends[i];
            nccl_check(ncclSend(a.buf, a.bytes / 8, ncclUint64, a.peer, comm_, s), "ncclSend");
            if (i < recvs.size()) {
                const Message& b = recvs[i];
                nccl_check(ncclRecv(b.buf, b.bytes / 8, ncclUint64, b.peer, comm_, s), "ncclRecv");
            }
        }
        for (size_t i = sends.size(); i < recvs.size(); ++i) {
            const Message& b = recvs[i];
            nccl_check(ncclRecv(b.buf, b.bytes / 8, ncclUint64, b.peer, comm_, s), "ncclRecv");
        }
        nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    }
    void exchange_host(const std::vector<Message>& sends, const std::vector<Message>& recvs) override {
        ctl_->exchange_host(sends, recvs);
    }
    void barrier() override { ctl_->barrier(); }
    void broadcast(void* buf, size_t n, int root) override { ctl_->broadcast(buf, n, root); }
    double allreduce_max(double v) override { return ctl_->allreduce_max(v); }
    double allreduce_min(double v) override { return ctl_->allreduce_min(v); }
    u64 allreduce_sum(u64 v) override { return ctl_->allreduce_sum(v); }
    void gatherv(const void* send, size_t n, std::vector<std::vector<u8>>* out, int root) override {
        ctl_->gatherv(send, n, out, root);
    }
    void* register_buffer(void* buf, size_t bytes) override {
        void* h = nullptr;
        if (!comm_ || ncclCommRegister(comm_, buf, bytes, &h) != ncclSuccess) return nullptr;
        return h;
    }
    void deregister_buffer(void* handle) override {
        if (comm_ && handle) (void)ncclCommDeregister(comm_, handle);
    }
    int data_plane_ranks() override {
        int n = -1;
        if (comm_ && ncclCommCount(comm_, &n) != ncclSuccess) return -1;
        return n;
    }
    void device_barrier(void* stream) override {
        if (!dbuf_) {
            const hipError_t e = hipMalloc(&dbuf_, sizeof(float) * 2);  // on the current (engine's) device
            if (e != hipSuccess) throw Error(strprintf("device_barrier: hipMalloc: %s", hipGetErrorString(e)));
        }
        nccl_check(ncclAllReduce(dbuf_, dbuf_, 1, ncclFloat32, ncclSum, comm_, (hipStream_t)stream), "ncclAllReduce");
    }
    std::string async_error() override {
        if (!comm_) return "";
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) return "ncclCommGetAsyncError failed";
        if (st == ncclSuccess || st == ncclInProgress) return "";
        return std::string("RCCL asynchronous error: ") + ncclGetErrorString(st);
    }
    [[noreturn]] void abort(int code) override {
        if (comm_) ncclCommAbort(comm_);
        comm_ = nullptr;
        ctl_->abort(code);
        _Exit(code);
    }

   private:
    std::shared_ptr<Transport> ctl_;
    ncclComm_t comm_ = nullptr;
    void* dbuf_ = nullptr;  // device_barrier's all-reduce operand
};

}  // namespace

bool rccl_available() { return true; }

std::string rccl_unique_id() {
    ncclUniqueId id;
    nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return std::string(id.internal, sizeof(id.internal));
}

std::shared_ptr<Transport> make_rccl_transport_with_id(std::shared_ptr<Transport> control, const std::string& uid) {
    if (uid.size() != sizeof(ncclUniqueId)) throw Error("bad ncclUniqueId size");
    ncclUniqueId id;
    memcpy(id.internal, uid.data(), sizeof(id.internal));
    return std::make_shared<RcclTransport>(std::move(control), id);
}

std::shared_ptr<Transport> make_rccl_transport(std::shared_ptr<Transport> control) {
    std::string uid(sizeof(ncclUniqueId), '\0');
    if (control->rank() == 0) uid = rccl_unique_id();
    control->broadcast(&uid[0], uid.size(), 0);
    return make_rccl_transport_with_id(std::move(control), uid);
}

}  // namespace gol
