// gol-mi355x: TCP transport with a torchrun-style rendezvous (MASTER_ADDR / MASTER_PORT).
//
// Lets the native `gol` binary run multi-process without MPI: `torchrun --nproc-per-node P gol ...`
// or any launcher that exports RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT.  It is the control
// plane under RCCL (unique-id broadcast, barriers, timing reductions) and the data plane of the
// CPU backend.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <deque>
#include <thread>

#include "gol/transport.hpp"

namespace gol {

namespace {

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void write_all(int fd, const void* buf, size_t n) {
    const char* p = (const char*)buf;
    while (n) {
        ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            throw Error(strprintf("tcp send failed: %s", strerror(errno)));
        }
        p += k;
        n -= (size_t)k;
    }
}

void read_all(int fd, void* buf, size_t n) {
    char* p = (char*)buf;
    while (n) {
        ssize_t k = ::recv(fd, p, n, 0);
        if (k == 0) throw Error("tcp peer closed the connection");
        if (k < 0) {
            if (errno == EINTR) continue;
            throw Error(strprintf("tcp recv failed: %s", strerror(errno)));
        }
        p += k;
        n -= (size_t)k;
    }
}

void tune(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

int listen_on(int port, int* bound_port) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) throw Error("socket() failed");
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    a.sin_port = htons((uint16_t)port);
    if (bind(fd, (sockaddr*)&a, sizeof(a)) < 0)
        throw Error(strprintf("bind(port %d) failed: %s", port, strerror(errno)));
    if (listen(fd, 256) < 0) throw Error("listen() failed");
    socklen_t len = sizeof(a);
    getsockname(fd, (sockaddr*)&a, &len);
    if (bound_port) *bound_port = ntohs(a.sin_port);
    return fd;
}

int accept_one(int lfd, double deadline, sockaddr_in* peer) {
    for (;;) {
        pollfd p{lfd, POLLIN, 0};
        int ms = (int)std::max(0.0, (deadline - now_s()) * 1000.0);
        int rc = poll(&p, 1, ms);
        if (rc < 0 && errno == EINTR) continue;
        if (rc <= 0) throw Error("tcp rendezvous timed out waiting for peers");
        socklen_t len = sizeof(sockaddr_in);
        int fd = accept(lfd, (sockaddr*)peer, &len);
        if (fd >= 0) {
            tune(fd);
            return fd;
        }
    }
}

int connect_to(u32 ip_be, int port, double deadline) {
    for (;;) {
        int fd = socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = ip_be;
        a.sin_port = htons((uint16_t)port);
        if (connect(fd, (sockaddr*)&a, sizeof(a)) == 0) {
            tune(fd);
            return fd;
        }
        close(fd);
        if (now_s() > deadline) throw Error(strprintf("tcp connect to port %d timed out", port));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
}

u32 resolve(const std::string& host) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res)
        throw Error("cannot resolve MASTER_ADDR " + host);
    u32 ip = ((sockaddr_in*)res->ai_addr)->sin_addr.s_addr;
    freeaddrinfo(res);
    return ip;
}

struct PeerEntry {
    u32 ip;
    i32 port;
};

class TcpTransport : public Transport {
   public:
    TcpTransport(int rank, int size, const std::string& addr, int port, double timeout) : rank_(rank), size_(size) {
        fds_.assign((size_t)size, -1);
        if (size == 1) return;
        double deadline = now_s() + timeout;
        std::vector<PeerEntry> table((size_t)size);
        int my_port = 0;
        int lfd = -1;
        if (rank == 0) {
            lfd = listen_on(port, &my_port);
            table[0] = {resolve(addr), port};
            for (int i = 1; i < size; ++i) {
                sockaddr_in peer{};
                int fd = accept_one(lfd, deadline, &peer);
                i32 hello[2];
                read_all(fd, hello, sizeof(hello));
                if (hello[0] <= 0 || hello[0] >= size || fds_[hello[0]] >= 0) throw Error("bad tcp rendezvous hello");
                fds_[hello[0]] = fd;
                table[hello[0]] = {peer.sin_addr.s_addr, hello[1]};
            }
            for (int i = 1; i < size; ++i) write_all(fds_[i], table.data(), table.size() * sizeof(PeerEntry));
        } else {
            lfd = listen_on(0, &my_port);
            int fd0 = connect_to(resolve(addr), port, deadline);
            i32 hello[2] = {rank, my_port};
            write_all(fd0, hello, sizeof(hello));
            read_all(fd0, table.data(), table.size() * sizeof(PeerEntry));
            fds_[0] = fd0;
            for (int j = 1; j < rank; ++j) {
                int fd = connect_to(table[j].ip, table[j].port, deadline);
                i32 me = rank;
                write_all(fd, &me, sizeof(me));
                fds_[j] = fd;
            }
            for (int j = rank + 1; j < size; ++j) {
                sockaddr_in peer{};
                int fd = accept_one(lfd, deadline, &peer);
                i32 who = -1;
                read_all(fd, &who, sizeof(who));
                if (who <= rank || who >= size || fds_[who] >= 0) throw Error("bad tcp mesh hello");
                fds_[who] = fd;
            }
        }
        if (lfd >= 0) close(lfd);
    }
    ~TcpTransport() override {
        for (int fd : fds_)
            if (fd >= 0) close(fd);
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    std::string name() const override { return "tcp"; }
    void send_bytes(int peer, const void* buf, size_t n) override { write_all(fds_.at(peer), buf, n); }
    void recv_bytes(int peer, void* buf, size_t n) override { read_all(fds_.at(peer), buf, n); }

    void exchange(const std::vector<Message>& sends, const std::vector<Message>& recvs, void*) override {
        // Progress every send and receive concurrently (per-peer FIFO), so large halos never
        // deadlock on full socket buffers.
        struct Op {
            const Message* m;
            size_t done;
        };
        std::vector<std::deque<Op>> sq((size_t)size_), rq((size_t)size_);
        for (const Message& m : sends) sq[m.peer].push_back({&m, 0});
        for (const Message& m : recvs) rq[m.peer].push_back({&m, 0});
        for (;;) {
            // zero-length messages complete immediately
            for (int p = 0; p < size_; ++p) {
                while (!sq[p].empty() && sq[p].front().m->bytes == 0) sq[p].pop_front();
                while (!rq[p].empty() && rq[p].front().m->bytes == 0) rq[p].pop_front();
            }
            std::vector<pollfd> pf;
            for (int p = 0; p < size_; ++p) {
                short ev = 0;
                if (!sq[p].empty()) ev |= POLLOUT;
                if (!rq[p].empty()) ev |= POLLIN;
                if (ev) pf.push_back({fds_[p], ev, 0});
            }
            if (pf.empty()) return;
            int rc = poll(pf.data(), pf.size(), 60000);
            if (rc < 0 && errno == EINTR) continue;
            if (rc <= 0) throw Error("tcp halo exchange timed out");
            for (const pollfd& q : pf) {
                int p = -1;
                for (int i = 0; i < size_; ++i)
                    if (fds_[i] == q.fd) p = i;
                if ((q.revents & POLLOUT) && !sq[p].empty()) {
                    Op& op = sq[p].front();
                    ssize_t k = ::send(q.fd, (const char*)op.m->buf + op.done, op.m->bytes - op.done,
                                       MSG_DONTWAIT | MSG_NOSIGNAL);
                    if (k > 0) op.done += (size_t)k;
                    if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
                        throw Error(strprintf("tcp send failed: %s", strerror(errno)));
                    if (op.done == op.m->bytes) sq[p].pop_front();
                }
                if ((q.revents & (POLLIN | POLLHUP | POLLERR)) && !rq[p].empty()) {
                    Op& op = rq[p].front();
                    ssize_t k = ::recv(q.fd, (char*)op.m->buf + op.done, op.m->bytes - op.done, MSG_DONTWAIT);
                    if (k == 0) throw Error("tcp peer closed the connection");
                    if (k > 0) op.done += (size_t)k;
                    if (k < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
                        throw Error(strprintf("tcp recv failed: %s", strerror(errno)));
                    if (op.done == op.m->bytes) rq[p].pop_front();
                }
            }
        }
    }

   private:
    int rank_, size_;
    std::vector<int> fds_;
};

}  // namespace

std::shared_ptr<Transport> make_tcp_transport(int rank, int size, const std::string& addr, int port,
                                              double timeout_s) {
    return std::make_shared<TcpTransport>(rank, size, addr, port, timeout_s);
}

}  // namespace gol
