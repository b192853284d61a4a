// gol-mi355x: in-process emulation of the RCCL data plane (GOL_TRANSPORT=p2p, thread mode).
//
// RCCL needs one rank per GPU, so a one-GPU machine cannot run the device-transport code paths
// (device halos, stream-ordered exchange on the comm stream, 2-D pack/unpack around it, the split
// schedule and its collective autotuning).  This transport gives ranks that are threads of one
// process the same semantics on a shared GPU:
//   * an exchange is a rendezvous: for every receive the receiver posts an offer (its device
//     buffer + an event recorded on ITS stream, i.e. "my earlier work on this buffer is done");
//   * the sender takes the offers addressed to it in per-peer FIFO order (RCCL's matching rule),
//     makes its stream wait for the receiver's event, copies device-to-device into the receiver's
//     buffer and records a completion event on its stream;
//   * the receiver's stream waits for that completion before anything it enqueues later.
// Everything is stream ordered and nothing synchronises the host with the GPU, like ncclSend/Recv.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <map>
#include <mutex>

#include "gol/transport.hpp"

namespace gol {

namespace {

#define P2P_CHECK(x)                                                                                 \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) throw Error(strprintf("%s failed: %s", #x, hipGetErrorString(e_))); \
    } while (0)

struct Offer {
    void* dst = nullptr;
    size_t bytes = 0;
    hipEvent_t ready = nullptr;  // receiver's stream reached the exchange
    hipEvent_t done = nullptr;   // sender's copy into dst finished
    bool copied = false;
    ~Offer() {
        if (ready) (void)hipEventDestroy(ready);
        if (done) (void)hipEventDestroy(done);
    }
};

class OfferBoard {
   public:
    explicit OfferBoard(int n) : n_(n), q_((size_t)n * n) {}
    void post(int sender, int receiver, std::shared_ptr<Offer> o) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_[(size_t)sender * n_ + receiver].push_back(std::move(o));
        }
        cv_.notify_all();
    }
    std::shared_ptr<Offer> take(int sender, int receiver) {
        std::unique_lock<std::mutex> lk(mu_);
        auto& q = q_[(size_t)sender * n_ + receiver];
        cv_.wait(lk, [&] { return !q.empty() || aborted_; });
        if (aborted_) throw Error("p2p emulation aborted");
        auto o = std::move(q.front());
        q.pop_front();
        return o;
    }
    void mark_copied(Offer& o) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            o.copied = true;
        }
        cv_.notify_all();
    }
    void wait_copied(Offer& o) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return o.copied || aborted_; });
        if (aborted_) throw Error("p2p emulation aborted");
    }
    void abort() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            aborted_ = true;
        }
        cv_.notify_all();
    }

   private:
    int n_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<std::deque<std::shared_ptr<Offer>>> q_;  // [sender][receiver]
    bool aborted_ = false;
};

std::mutex g_reg_mu;
std::map<const void*, std::weak_ptr<OfferBoard>> g_reg;

std::shared_ptr<OfferBoard> board_for(const void* key, int n) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_reg.find(key);
    if (it != g_reg.end())
        if (auto b = it->second.lock()) return b;
    auto b = std::make_shared<OfferBoard>(n);
    g_reg[key] = b;
    return b;
}

class P2pEmulationTransport : public Transport {
   public:
    P2pEmulationTransport(std::shared_ptr<Transport> control, const void* key)
        : ctl_(std::move(control)), board_(board_for(key, ctl_->size())) {}
    int rank() const override { return ctl_->rank(); }
    int size() const override { return ctl_->size(); }
    std::string name() const override { return "p2p-emulation+" + ctl_->name(); }
    void send_bytes(int peer, const void* buf, size_t n) override { ctl_->send_bytes(peer, buf, n); }
    void recv_bytes(int peer, void* buf, size_t n) override { ctl_->recv_bytes(peer, buf, n); }
    bool device_buffers() const override { return true; }

    void exchange(const std::vector<Message>& sends, const std::vector<Message>& recvs, void* stream) override {
        hipStream_t s = (hipStream_t)stream;
        const int me = rank();
        std::vector<std::shared_ptr<Offer>> mine;
        for (const Message& r : recvs) {  // post every receive first: no circular waits
            auto o = std::make_shared<Offer>();
            o->dst = r.buf;
            o->bytes = r.bytes;
            P2P_CHECK(hipEventCreateWithFlags(&o->ready, hipEventDisableTiming));
            P2P_CHECK(hipEventCreateWithFlags(&o->done, hipEventDisableTiming));
            P2P_CHECK(hipEventRecord(o->ready, s));
            board_->post(r.peer, me, o);
            mine.push_back(std::move(o));
        }
        for (const Message& m : sends) {
            auto o = board_->take(me, m.peer);
            if (o->bytes != m.bytes)
                throw Error(strprintf("p2p message size mismatch %d->%d: %zu vs %zu bytes", me, m.peer, m.bytes,
                                      o->bytes));
            P2P_CHECK(hipStreamWaitEvent(s, o->ready, 0));
            if (m.bytes) P2P_CHECK(hipMemcpyAsync(o->dst, m.buf, m.bytes, hipMemcpyDeviceToDevice, s));
            P2P_CHECK(hipEventRecord(o->done, s));
            board_->mark_copied(*o);
        }
        for (auto& o : mine) {
            board_->wait_copied(*o);
            P2P_CHECK(hipStreamWaitEvent(s, o->done, 0));
            retired_.push_back(std::move(o));
        }
        while (retired_.size() > 4096) retired_.pop_front();  // events freed long after completion
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
    [[noreturn]] void abort(int code) override {
        board_->abort();
        ctl_->abort(code);
        std::_Exit(code);
    }

   private:
    std::shared_ptr<Transport> ctl_;
    std::shared_ptr<OfferBoard> board_;
    std::deque<std::shared_ptr<Offer>> retired_;
};

}  // namespace

std::shared_ptr<Transport> make_p2p_emulation_transport(std::shared_ptr<Transport> control) {
    auto* tt = dynamic_cast<ThreadTransport*>(control.get());
    if (!tt) throw Error("GOL_TRANSPORT=p2p (RCCL emulation) needs thread-mode ranks (GOL_NRANKS)");
    return std::make_shared<P2pEmulationTransport>(std::move(control), tt->group_key());
}

}  // namespace gol
