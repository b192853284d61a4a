// Probe: does a 1-rank RCCL communicator accept grouped ncclSend/ncclRecv with peer == rank, also
// inside a captured hipGraph?  (Engine self-exchange mode, GOL_SELF_EXCHANGE=1, depends on it.)
//   hipcc -O2 --offload-arch=gfx950 tools/rccl_self_probe.cpp -lrccl -o build/rccl_self_probe
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        auto r_ = (x);                                                                 \
        if (r_ != 0) {                                                                 \
            fprintf(stderr, "%s failed: %d at line %d\n", #x, (int)r_, __LINE__);      \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int mode = argc > 1 ? atoi(argv[1]) : 0;  // 0: eager + graph, 1: eager only
    int ver = 0;
    ncclGetVersion(&ver);
    printf("rccl version %d\n", ver);
    ncclUniqueId id;
    CK(ncclGetUniqueId(&id));
    printf("unique id ok\n");
    ncclComm_t comm;
    CK(ncclCommInitRank(&comm, 1, id, 0));
    int n = 0;
    CK(ncclCommCount(comm, &n));
    printf("comm count %d\n", n);
    const size_t words = 64 * 512;  // 64 rows of a 32768-wide bit-packed board
    std::vector<unsigned long long> h(2 * words);
    for (size_t i = 0; i < words; ++i) h[i] = 0x9E3779B97F4A7C15ull * (i + 1), h[words + i] = ~h[i];
    unsigned long long *a, *b;
    CK(hipMalloc(&a, 2 * words * 8));
    CK(hipMalloc(&b, 2 * words * 8));
    CK(hipMemcpy(a, h.data(), 2 * words * 8, hipMemcpyHostToDevice));
    CK(hipMemset(b, 0, 2 * words * 8));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    auto exch = [&]() {
        CK(ncclGroupStart());
        CK(ncclSend(a, words, ncclUint64, 0, comm, s));
        CK(ncclRecv(b + words, words, ncclUint64, 0, comm, s));
        CK(ncclSend(a + words, words, ncclUint64, 0, comm, s));
        CK(ncclRecv(b, words, ncclUint64, 0, comm, s));
        CK(ncclGroupEnd());
    };
    printf("first exchange enqueue\n");
    exch();
    printf("enqueued, syncing\n");
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> g(2 * words);
    CK(hipMemcpy(g.data(), b, 2 * words * 8, hipMemcpyDeviceToHost));
    // FIFO per peer: first send (a[0:words]) -> first recv (b[words:]); second -> b[0:words]
    size_t bad = 0;
    for (size_t i = 0; i < words; ++i) bad += (g[words + i] != h[i]) + (g[i] != h[words + i]);
    printf("eager self exchange: %s (%zu bad words)\n", bad ? "MISMATCH" : "ok", bad);
    // timing
    for (int i = 0; i < 10; ++i) exch();
    CK(hipStreamSynchronize(s));
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 100; ++i) exch();
    CK(hipStreamSynchronize(s));
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 100;
    printf("eager self exchange: %.2f us per group (2 x %zu KiB)\n", us, words * 8 / 1024);
    if (mode == 1) {
        printf("destroying comm (no graph captured)\n");
        auto td = std::chrono::steady_clock::now();
        CK(ncclCommDestroy(comm));
        printf("destroyed in %.3f s\nPROBE_DONE\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - td).count());
        return 0;
    }
    // graph capture
    CK(hipMemset(b, 0, 2 * words * 8));
    hipGraph_t graph;
    hipGraphExec_t exec;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
    for (int i = 0; i < 4; ++i) exch();
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    CK(hipGraphLaunch(exec, s));
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(g.data(), b, 2 * words * 8, hipMemcpyDeviceToHost));
    bad = 0;
    for (size_t i = 0; i < words; ++i) bad += (g[words + i] != h[i]) + (g[i] != h[words + i]);
    printf("graph self exchange: %s (%zu bad words)\n", bad ? "MISMATCH" : "ok", bad);
    t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 25; ++i) CK(hipGraphLaunch(exec, s));
    CK(hipStreamSynchronize(s));
    us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 100;
    printf("graph self exchange: %.2f us per group\n", us);
    ncclResult_t st;
    CK(ncclCommGetAsyncError(comm, &st));
    printf("async error state: %s\n", ncclGetErrorString(st));
    CK(hipGraphExecDestroy(exec));
    CK(hipGraphDestroy(graph));
    CK(hipStreamSynchronize(s));
    printf("graph destroyed; finalizing comm\n");
    auto td = std::chrono::steady_clock::now();
    CK(ncclCommFinalize(comm));
    printf("finalized in %.3f s\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - td).count());
    CK(ncclCommDestroy(comm));
    printf("destroyed in %.3f s\nPROBE_DONE\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - td).count());
    return 0;
}
