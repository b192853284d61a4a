// gol-mi355x: MPI transport (optional; compiled with MPI headers when GOL_WITH_MPI is defined).
//
// Keeps the reference's launch contract `mpirun -n P ./gol ...` (gol-main.c:58-62) working.  Used as
// the control plane under RCCL and as a host data plane.  Unlike the reference (gol-main.c:89-111),
// every request is completed (MPI_Waitall on sends and receives) and fatal errors call MPI_Abort.
//
// The MPI library is loaded with dlopen only when the process was actually started by mpirun, so
// the `gol` binary has no link-time MPI dependency (and no foreign library directory in its rpath
// that could shadow the system C++ runtime the ROCm libraries need).
#include <cstdlib>
#include <cstring>

#include "gol/transport.hpp"

#ifdef GOL_WITH_MPI
#include <dlfcn.h>
#include <mpi.h>
#ifndef GOL_MPI_LIB_PATH
#define GOL_MPI_LIB_PATH "libmpi.so.12"
#endif
#endif

namespace gol {

bool mpi_launched() {
    static const char* vars[] = {"PMI_RANK", "PMI_SIZE", "OMPI_COMM_WORLD_RANK", "MPI_LOCALRANKID", "PMIX_RANK"};
    for (const char* v : vars)
        if (getenv(v)) return true;
    return false;
}

#ifdef GOL_WITH_MPI

namespace {

struct MpiApi {
#define MPI_FN_SLOT(name) decltype(&::name) name = nullptr;
    MPI_FN_SLOT(MPI_Init)
    MPI_FN_SLOT(MPI_Initialized)
    MPI_FN_SLOT(MPI_Finalized)
    MPI_FN_SLOT(MPI_Finalize)
    MPI_FN_SLOT(MPI_Comm_rank)
    MPI_FN_SLOT(MPI_Comm_size)
    MPI_FN_SLOT(MPI_Send)
    MPI_FN_SLOT(MPI_Recv)
    MPI_FN_SLOT(MPI_Isend)
    MPI_FN_SLOT(MPI_Irecv)
    MPI_FN_SLOT(MPI_Waitall)
    MPI_FN_SLOT(MPI_Barrier)
    MPI_FN_SLOT(MPI_Bcast)
    MPI_FN_SLOT(MPI_Allreduce)
    MPI_FN_SLOT(MPI_Abort)
#undef MPI_FN_SLOT
};

const MpiApi& mpi() {
    static MpiApi api;
    static bool loaded = false;
    if (loaded) return api;
    const char* path = getenv("GOL_MPI_LIB");
    void* h = dlopen(path && *path ? path : GOL_MPI_LIB_PATH, RTLD_NOW | RTLD_GLOBAL);
    if (!h) throw Error(std::string("cannot load the MPI library: ") + dlerror());
#define MPI_SYM_SLOT(name)                                                     \
    api.name = reinterpret_cast<decltype(api.name)>(dlsym(h, #name));        \
    if (!api.name) throw Error("MPI library lacks " #name);
    MPI_SYM_SLOT(MPI_Init)
    MPI_SYM_SLOT(MPI_Initialized)
    MPI_SYM_SLOT(MPI_Finalized)
    MPI_SYM_SLOT(MPI_Finalize)
    MPI_SYM_SLOT(MPI_Comm_rank)
    MPI_SYM_SLOT(MPI_Comm_size)
    MPI_SYM_SLOT(MPI_Send)
    MPI_SYM_SLOT(MPI_Recv)
    MPI_SYM_SLOT(MPI_Isend)
    MPI_SYM_SLOT(MPI_Irecv)
    MPI_SYM_SLOT(MPI_Waitall)
    MPI_SYM_SLOT(MPI_Barrier)
    MPI_SYM_SLOT(MPI_Bcast)
    MPI_SYM_SLOT(MPI_Allreduce)
    MPI_SYM_SLOT(MPI_Abort)
#undef MPI_SYM_SLOT
    loaded = true;
    return api;
}

class MpiTransport : public Transport {
   public:
    MpiTransport(int* argc, char*** argv) {
        int inited = 0;
        mpi().MPI_Initialized(&inited);
        if (!inited) {
            mpi().MPI_Init(argc, argv);
            owner_ = true;
        }
        mpi().MPI_Comm_rank(MPI_COMM_WORLD, &rank_);
        mpi().MPI_Comm_size(MPI_COMM_WORLD, &size_);
    }
    ~MpiTransport() override {
        int fin = 0;
        mpi().MPI_Finalized(&fin);
        if (owner_ && !fin) mpi().MPI_Finalize();
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    std::string name() const override { return "mpi"; }
    void send_bytes(int peer, const void* buf, size_t n) override {
        mpi().MPI_Send(buf, (int)n, MPI_BYTE, peer, 7, MPI_COMM_WORLD);
    }
    void recv_bytes(int peer, void* buf, size_t n) override {
        mpi().MPI_Recv(buf, (int)n, MPI_BYTE, peer, 7, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    }
    void exchange(const std::vector<Message>& sends, const std::vector<Message>& recvs, void*) override {
        std::vector<MPI_Request> req(sends.size() + recvs.size());
        size_t j = 0;
        // one tag: matching is by per-pair order, exactly like RCCL (canonical order)
        for (const Message& m : recvs)
            mpi().MPI_Irecv(m.buf, (int)m.bytes, MPI_BYTE, m.peer, 11, MPI_COMM_WORLD, &req[j++]);
        for (const Message& m : sends)
            mpi().MPI_Isend(m.buf, (int)m.bytes, MPI_BYTE, m.peer, 11, MPI_COMM_WORLD, &req[j++]);
        mpi().MPI_Waitall((int)req.size(), req.data(), MPI_STATUSES_IGNORE);
    }
    void barrier() override { mpi().MPI_Barrier(MPI_COMM_WORLD); }
    void broadcast(void* buf, size_t n, int root) override { mpi().MPI_Bcast(buf, (int)n, MPI_BYTE, root, MPI_COMM_WORLD); }
    double allreduce_max(double v) override {
        double r;
        mpi().MPI_Allreduce(&v, &r, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
        return r;
    }
    double allreduce_min(double v) override {
        double r;
        mpi().MPI_Allreduce(&v, &r, 1, MPI_DOUBLE, MPI_MIN, MPI_COMM_WORLD);
        return r;
    }
    u64 allreduce_sum(u64 v) override {
        unsigned long long a = v, r = 0;
        mpi().MPI_Allreduce(&a, &r, 1, MPI_UNSIGNED_LONG_LONG, MPI_SUM, MPI_COMM_WORLD);
        return r;
    }
    [[noreturn]] void abort(int code) override {
        fflush(stdout);
        fflush(stderr);
        mpi().MPI_Abort(MPI_COMM_WORLD, code);
        _Exit(code);
    }

   private:
    int rank_ = 0, size_ = 1;
    bool owner_ = false;
};

}  // namespace

std::shared_ptr<Transport> make_mpi_transport(int* argc, char*** argv) {
    return std::make_shared<MpiTransport>(argc, argv);
}

#else

std::shared_ptr<Transport> make_mpi_transport(int*, char***) { return nullptr; }

#endif

}  // namespace gol
