// gol-mi355x: communication layer.
//
// The reference talks MPI directly from its generation loop: MPI_Irecv x2 + MPI_Isend x2 of one byte
// row per generation, MPI_Wait on the receives only, MPI_Barrier + MPI_Wtime for timing
// (gol-main.c:58-62, 89-111, 118-122).  Here communication is an interface with two planes:
//
//  * control plane — small host-side messages: barrier, broadcast, max/sum reductions and a gather
//    used for timing, fingerprints and the 2-D dump.  Built on blocking, per-pair-FIFO host p2p.
//  * data plane    — the halo exchange.  One call per superstep carries every halo message
//    (2 in 1-D, 8 in 2-D) in *canonical order*: for each direction d, send(edge_d -> nbr[d]) then
//    recv(halo_opp(d) <- nbr[opp(d)]).  Matching is purely by per-peer order (RCCL has no tags), so
//    this order is what makes P <= 2 rings (prev == next) correct — the reference's Q2 bug.
//    Device transports (RCCL over xGMI) take device pointers and are stream ordered; host transports
//    complete before returning.
//
// Implementations: SelfTransport (P=1), ThreadTransport (P ranks as threads of one process),
// RcclTransport (RCCL over xGMI, control plane delegated), MpiTransport (optional, mpirun launch),
// TcpTransport (env-rendezvous, torchrun-style MASTER_ADDR/PORT), and a Python-callback transport
// (torch.distributed / gloo) in the bindings.
#pragma once

#include <deque>
#include <memory>
#include <string>
#include <vector>

#include "gol/common.hpp"

namespace gol {

struct Message {
    int peer;
    void* buf;
    size_t bytes;
};

class Transport {
   public:
    virtual ~Transport() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    virtual std::string name() const = 0;

    // Control plane primitives: blocking host p2p, FIFO per (sender, receiver) pair.
    virtual void send_bytes(int peer, const void* buf, size_t n) = 0;
    virtual void recv_bytes(int peer, void* buf, size_t n) = 0;

    // Data plane.  device_buffers(): messages hold device pointers and `stream` (a hipStream_t)
    // orders the exchange; otherwise host pointers and the call is synchronous.
    virtual bool device_buffers() const { return false; }
    virtual void exchange(const std::vector<Message>& sends, const std::vector<Message>& recvs, void* stream);
    // Host-memory exchange with the same ordering rules (device transports forward it to their
    // control plane).
    virtual void exchange_host(const std::vector<Message>& sends, const std::vector<Message>& recvs) {
        exchange(sends, recvs, nullptr);
    }

    // Collectives (defaults: linear algorithms over send_bytes/recv_bytes through rank 0).
    virtual void barrier();
    virtual void broadcast(void* buf, size_t n, int root);
    virtual double allreduce_max(double v);
    virtual double allreduce_min(double v);
    virtual u64 allreduce_sum(u64 v);
    // Variable-size gather to `root`; `out` (root only) receives size() byte vectors.
    virtual void gatherv(const void* send, size_t n, std::vector<std::vector<u8>>* out, int root);
    // Fatal error on this rank: make every rank exit instead of hanging (reference Q11).
    [[noreturn]] virtual void abort(int code);
    // Asynchronous failure of the data plane (e.g. ncclCommGetAsyncError); empty when healthy.
    virtual std::string async_error() { return ""; }
    // Ranks of the device data plane's communicator as the library reports them (RCCL:
    // ncclCommCount); -1 for host transports.
    virtual int data_plane_ranks() { return -1; }
    // Device transports: enqueue a collective on `stream` (a hipStream_t) that completes on every
    // rank's GPU only once every rank has reached it (RCCL: a 1-element all-reduce).  Used to align
    // the ranks' timed regions on the GPUs themselves; host transports need nothing beyond barrier().
    virtual void device_barrier(void* stream) { (void)stream; }
    // Whether exchange() may be captured into a hipGraph (RCCL: its kernels become graph nodes; the
    // thread-rank emulation rendezvous across streams of several threads and cannot be captured).
    virtual bool graph_capturable() const { return false; }
    // Device transports: register a device buffer the exchanges send from / receive into (RCCL:
    // ncclCommRegister, user-buffer registration for zero-copy peer transfers).  Returns a handle for
    // deregister_buffer, or nullptr when the transport does not register (or registration failed:
    // the exchanges then use the unregistered path).
    virtual void* register_buffer(void* buf, size_t bytes) {
        (void)buf;
        (void)bytes;
        return nullptr;
    }
    virtual void deregister_buffer(void* handle) { (void)handle; }
};

// P = 1.
class SelfTransport : public Transport {
   public:
    int rank() const override { return 0; }
    int size() const override { return 1; }
    std::string name() const override { return "self"; }
    void send_bytes(int peer, const void* buf, size_t n) override;
    void recv_bytes(int peer, void* buf, size_t n) override;

   private:
    std::deque<std::vector<u8>> box_;  // loopback FIFO
};

// P ranks as threads of one process; host-memory mailboxes.
class ThreadGroup;
class ThreadTransport : public Transport {
   public:
    ThreadTransport(std::shared_ptr<ThreadGroup> g, int rank);
    int rank() const override { return rank_; }
    int size() const override;
    std::string name() const override { return "threads"; }
    void send_bytes(int peer, const void* buf, size_t n) override;
    void recv_bytes(int peer, void* buf, size_t n) override;
    [[noreturn]] void abort(int code) override;
    const void* group_key() const { return g_.get(); }  // identifies the ranks of one group

   private:
    std::shared_ptr<ThreadGroup> g_;
    int rank_;
};
std::shared_ptr<ThreadGroup> make_thread_group(int nranks);
// Exit code of the rank that aborted the group (0 while none has): the other ranks, woken by the
// abort, exit with the same code, so the process status does not depend on which thread exits first.
int thread_group_abort_code(ThreadGroup& g);

// RCCL-semantics data plane for thread-mode ranks sharing one GPU (device buffers, stream-ordered
// rendezvous copies, per-peer FIFO matching): exercises the device-transport engine paths without
// a second GPU.  `control` must be a ThreadTransport.
std::shared_ptr<Transport> make_p2p_emulation_transport(std::shared_ptr<Transport> control);

// Torchrun-style rendezvous over TCP: rank 0 listens on MASTER_ADDR:MASTER_PORT, every rank
// connects to every other rank (full mesh of sockets, P <= a few dozen).
std::shared_ptr<Transport> make_tcp_transport(int rank, int size, const std::string& addr, int port,
                                              double timeout_s = 120.0);

// RCCL data plane over an existing control plane.  `device` must already be current.
std::shared_ptr<Transport> make_rccl_transport(std::shared_ptr<Transport> control);
// Same, with an externally supplied ncclUniqueId (e.g. broadcast by torch.distributed).
std::shared_ptr<Transport> make_rccl_transport_with_id(std::shared_ptr<Transport> control,
                                                      const std::string& unique_id);
std::string rccl_unique_id();  // 128 raw bytes
bool rccl_available();

// MPI (only when built with GOL_WITH_MPI); nullptr otherwise.
std::shared_ptr<Transport> make_mpi_transport(int* argc, char*** argv);
bool mpi_launched();  // environment looks like an mpirun/mpiexec launch

}  // namespace gol
