// gol-mi355x: transport defaults, SelfTransport and ThreadTransport (see transport.hpp).
#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>

#include <unistd.h>

#include "gol/transport.hpp"

namespace gol {

// ---------------------------------------------------------------------------------------------
// Defaults
// ---------------------------------------------------------------------------------------------

void Transport::exchange(const std::vector<Message>& sends, const std::vector<Message>& recvs, void*) {
    // Host transports with buffered sends: post every send, then drain the receives.
    for (const Message& m : sends) send_bytes(m.peer, m.buf, m.bytes);
    for (const Message& m : recvs) recv_bytes(m.peer, m.buf, m.bytes);
}

void Transport::barrier() {
    u8 tok = 0;
    if (size() == 1) return;
    if (rank() == 0) {
        for (int r = 1; r < size(); ++r) recv_bytes(r, &tok, 1);
        for (int r = 1; r < size(); ++r) send_bytes(r, &tok, 1);
    } else {
        send_bytes(0, &tok, 1);
        recv_bytes(0, &tok, 1);
    }
}

void Transport::broadcast(void* buf, size_t n, int root) {
    if (size() == 1) return;
    if (rank() == root) {
        for (int r = 0; r < size(); ++r)
            if (r != root) send_bytes(r, buf, n);
    } else {
        recv_bytes(root, buf, n);
    }
}

template <typename T, typename Op>
static T allreduce_linear(Transport& t, T v, Op op) {
    if (t.size() == 1) return v;
    if (t.rank() == 0) {
        for (int r = 1; r < t.size(); ++r) {
            T x;
            t.recv_bytes(r, &x, sizeof(T));
            v = op(v, x);
        }
    } else {
        t.send_bytes(0, &v, sizeof(T));
    }
    t.broadcast(&v, sizeof(T), 0);
    return v;
}

double Transport::allreduce_max(double v) {
    return allreduce_linear(*this, v, [](double a, double b) { return std::max(a, b); });
}
double Transport::allreduce_min(double v) {
    return allreduce_linear(*this, v, [](double a, double b) { return std::min(a, b); });
}
u64 Transport::allreduce_sum(u64 v) {
    return allreduce_linear(*this, v, [](u64 a, u64 b) { return a + b; });
}

void Transport::gatherv(const void* send, size_t n, std::vector<std::vector<u8>>* out, int root) {
    if (rank() == root) {
        out->assign((size_t)size(), {});
        for (int r = 0; r < size(); ++r) {
            if (r == root) {
                (*out)[r].assign((const u8*)send, (const u8*)send + n);
                continue;
            }
            u64 len = 0;
            recv_bytes(r, &len, sizeof(len));
            (*out)[r].resize(len);
            if (len) recv_bytes(r, (*out)[r].data(), len);
        }
    } else {
        u64 len = n;
        send_bytes(root, &len, sizeof(len));
        if (n) send_bytes(root, send, n);
    }
}

void Transport::abort(int code) {
    fflush(stdout);
    fflush(stderr);
    _exit(code);
}

// ---------------------------------------------------------------------------------------------
// SelfTransport
// ---------------------------------------------------------------------------------------------

// Loopback: messages to rank 0 (itself) queue in FIFO order (the engine's self-exchange mode sends
// every halo to itself before receiving it).
void SelfTransport::send_bytes(int peer, const void* buf, size_t n) {
    if (peer != 0) throw Error(strprintf("SelfTransport: no rank %d", peer));
    box_.emplace_back((const u8*)buf, (const u8*)buf + n);
}
void SelfTransport::recv_bytes(int peer, void* buf, size_t n) {
    if (peer != 0) throw Error(strprintf("SelfTransport: no rank %d", peer));
    if (box_.empty()) throw Error("SelfTransport: receive without a matching send (would block forever)");
    if (box_.front().size() != n)
        throw Error(strprintf("SelfTransport: message size mismatch (%zu vs %zu bytes)", box_.front().size(), n));
    if (n) memcpy(buf, box_.front().data(), n);
    box_.pop_front();
}

// ---------------------------------------------------------------------------------------------
// ThreadTransport: mailboxes[dst][src] of byte messages; sends never block.
// ---------------------------------------------------------------------------------------------

class ThreadGroup {
   public:
    explicit ThreadGroup(int n) : n_(n), boxes_((size_t)n * n) {}
    int size() const { return n_; }
    void push(int src, int dst, const void* buf, size_t len) {
        std::vector<u8> m((const u8*)buf, (const u8*)buf + len);
        {
            std::lock_guard<std::mutex> lk(mu_);
            boxes_[(size_t)dst * n_ + src].push_back(std::move(m));
        }
        cv_.notify_all();
    }
    void pop(int src, int dst, void* buf, size_t len) {
        std::unique_lock<std::mutex> lk(mu_);
        auto& q = boxes_[(size_t)dst * n_ + src];
        cv_.wait(lk, [&] { return !q.empty() || aborted_; });
        if (aborted_ && q.empty()) throw Error(strprintf("thread group aborted (exit code %d)", code_));
        std::vector<u8> m = std::move(q.front());
        q.pop_front();
        lk.unlock();
        if (m.size() != len)
            throw Error(strprintf("message size mismatch %d->%d: got %zu bytes, expected %zu", src, dst,
                                  m.size(), len));
        if (len) memcpy(buf, m.data(), len);
    }
    void abort(int code) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!aborted_) code_ = code;
            aborted_ = true;
        }
        cv_.notify_all();
    }
    int abort_code() {
        std::lock_guard<std::mutex> lk(mu_);
        return aborted_ ? code_ : 0;
    }

   private:
    int n_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<std::deque<std::vector<u8>>> boxes_;
    bool aborted_ = false;
    int code_ = 0;  // exit code of the first rank that aborted the group
};

int thread_group_abort_code(ThreadGroup& g) { return g.abort_code(); }

std::shared_ptr<ThreadGroup> make_thread_group(int nranks) {
    if (nranks < 1) throw Error("thread group needs >= 1 rank");
    return std::make_shared<ThreadGroup>(nranks);
}

ThreadTransport::ThreadTransport(std::shared_ptr<ThreadGroup> g, int rank) : g_(std::move(g)), rank_(rank) {}
int ThreadTransport::size() const { return g_->size(); }
void ThreadTransport::send_bytes(int peer, const void* buf, size_t n) { g_->push(rank_, peer, buf, n); }
void ThreadTransport::recv_bytes(int peer, void* buf, size_t n) { g_->pop(peer, rank_, buf, n); }
void ThreadTransport::abort(int code) {
    g_->abort(code);
    Transport::abort(code);
}

}  // namespace gol
