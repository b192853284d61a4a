// rccl_capture_probe: an RCCL send/recv group captured into a hipGraph on a stream FORKED from the
// capture's origin stream (round 5: the engine's split+graph superstep crashed in librccl at capture,
// docs/PERFORMANCE.md §16).  A 1-rank communicator; the group sends a buffer to rank 0 itself.
//
//   mode fork      origin s0: BeginCapture, record e0; s1 waits e0 (forked into the capture);
//                  s1: ncclGroupStart / ncclSend + ncclRecv / ncclGroupEnd, record e1; s0 waits e1 (join),
//                  a kernel on s0, EndCapture, instantiate, launch x3, check the received bytes.
//   mode origin    the same group on s0 itself (what the engine's full+graph captures), the kernel on s1.
//   mode eager     no capture: the group on s1 (sanity check of the communicator).
//   mode unjoined  as fork, but s1 is never joined back to s0 before EndCapture (which must fail), then
//                  the communicator is used eagerly and destroyed.
//   mode query     as fork, with a hipEventQuery of the event recorded inside the capture before the
//                  fork (what the engine's wait_pending() does before a cross-stream wait).
//   suffix "+reg"  both buffers registered with the communicator (ncclCommRegister), as the engine
//                  registers its boards for a one-rank communicator.
// Every step prints a line (stderr, unbuffered) before it runs; SIGSEGV / SIGABRT print the host
// backtrace (backtrace_symbols_fd) and exit with 128 + signal.
//
//   hipcc --offload-arch=gfx950 -O2 -g -rdynamic -o build/rccl_capture_probe tools/rccl_capture_probe.cpp -lrccl
//   build/rccl_capture_probe fork+reg
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "FAIL %s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(3);                                                                         \
        }                                                                                    \
    } while (0)
#define NK(x)                                                                                \
    do {                                                                                     \
        ncclResult_t r_ = (x);                                                               \
        if (r_ != ncclSuccess) {                                                             \
            fprintf(stderr, "FAIL %s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_)); \
            exit(4);                                                                         \
        }                                                                                    \
    } while (0)

static void on_signal(int sig) {
    static const char msg[] = "\n*** signal caught; host backtrace:\n";
    (void)!write(2, msg, sizeof(msg) - 1);
    void* frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    _exit(128 + sig);
}

static void step(const char* what) { fprintf(stderr, "step: %s\n", what); }

__global__ void touch(unsigned* p) {
    if (threadIdx.x == 0) p[0] += 1;
}

int main(int argc, char** argv) {
    signal(SIGSEGV, on_signal);
    signal(SIGABRT, on_signal);
    signal(SIGBUS, on_signal);
    setvbuf(stderr, nullptr, _IONBF, 0);
    const std::string arg = argc > 1 ? argv[1] : "fork";
    const bool reg = arg.find("+reg") != std::string::npos;
    const std::string mode = arg.substr(0, arg.find('+'));
    const size_t words = 10240;  // 80 KiB, one strip halo
    printf("rccl_capture_probe mode=%s registered=%d NCCL %d\n", mode.c_str(), (int)reg, NCCL_VERSION_CODE);
    fflush(stdout);
    CK(hipSetDevice(0));
    ncclUniqueId id;
    NK(ncclGetUniqueId(&id));
    ncclComm_t comm;
    step("ncclCommInitRank (1 rank)");
    NK(ncclCommInitRank(&comm, 1, id, 0));
    hipStream_t s0, s1;
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&s0, hipStreamNonBlocking, 0));
    CK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, hi));  // as the engine's comm stream
    unsigned long long *sb, *rb;
    unsigned* ctr;
    CK(hipMalloc(&sb, words * 8));
    CK(hipMalloc(&rb, words * 8));
    CK(hipMalloc(&ctr, 64));
    CK(hipMemset(ctr, 0, 64));
    std::vector<unsigned long long> h(words);
    for (size_t i = 0; i < words; ++i) h[i] = 0x9E3779B97F4A7C15ull * (i + 1);
    CK(hipMemcpy(sb, h.data(), words * 8, hipMemcpyHostToDevice));
    CK(hipMemset(rb, 0, words * 8));
    void *hs = nullptr, *hr = nullptr;
    if (reg) {
        step("ncclCommRegister x2");
        NK(ncclCommRegister(comm, sb, words * 8, &hs));
        NK(ncclCommRegister(comm, rb, words * 8, &hr));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    auto group = [&](hipStream_t s) {
        step("ncclGroupStart");
        NK(ncclGroupStart());
        step("ncclSend");
        NK(ncclSend(sb, words, ncclUint64, 0, comm, s));
        step("ncclRecv");
        NK(ncclRecv(rb, words, ncclUint64, 0, comm, s));
        step("ncclGroupEnd");
        NK(ncclGroupEnd());
    };
    if (mode == "eager") {
        group(s1);
        CK(hipStreamSynchronize(s1));
    } else {
        hipGraph_t g = nullptr;
        hipGraphExec_t ex = nullptr;
        step("hipStreamBeginCapture(s0)");
        CK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
        CK(hipEventRecord(e0, s0));
        if (mode == "query") {
            step("hipEventQuery(e0) inside the capture");
            const hipError_t q = hipEventQuery(e0);
            fprintf(stderr, "hipEventQuery -> %s\n", hipGetErrorString(q));
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            (void)hipStreamIsCapturing(s0, &cs);
            fprintf(stderr, "capture status after the query: %d\n", (int)cs);
        }
        if (mode == "unjoined") {
            CK(hipStreamWaitEvent(s1, e0, 0));
            group(s1);
            step("hipStreamEndCapture (s1 unjoined)");
            hipGraph_t g2 = nullptr;
            const hipError_t ec = hipStreamEndCapture(s0, &g2);
            fprintf(stderr, "hipStreamEndCapture -> %s, graph %p\n", hipGetErrorString(ec), (void*)g2);
            if (g2) (void)hipGraphDestroy(g2);
            (void)hipGetLastError();
            step("eager group on s1 after the failed capture");
            group(s1);
            CK(hipStreamSynchronize(s1));
            CK(hipStreamSynchronize(s0));
        } else if (mode == "fork" || mode == "query") {
            step("s1 waits e0 (fork)");
            CK(hipStreamWaitEvent(s1, e0, 0));
            hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s0, ctr);
            group(s1);
            CK(hipEventRecord(e1, s1));
            step("s0 waits e1 (join)");
            CK(hipStreamWaitEvent(s0, e1, 0));
        } else {
            CK(hipStreamWaitEvent(s1, e0, 0));
            hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s1, ctr);
            group(s0);
            CK(hipEventRecord(e1, s1));
            CK(hipStreamWaitEvent(s0, e1, 0));
        }
        if (mode != "unjoined") {
            step("hipStreamEndCapture");
            CK(hipStreamEndCapture(s0, &g));
            size_t nn = 0;
            CK(hipGraphGetNodes(g, nullptr, &nn));
            fprintf(stderr, "captured graph: %zu nodes\n", nn);
            step("hipGraphInstantiate");
            CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
            for (int r = 0; r < 3; ++r) {
                step("hipGraphLaunch");
                CK(hipGraphLaunch(ex, s0));
            }
            step("hipStreamSynchronize");
            CK(hipStreamSynchronize(s0));
            CK(hipGraphExecDestroy(ex));
            CK(hipGraphDestroy(g));
        }
    }
    std::vector<unsigned long long> got(words);
    CK(hipMemcpy(got.data(), rb, words * 8, hipMemcpyDeviceToHost));
    const bool ok = memcmp(got.data(), h.data(), words * 8) == 0;
    printf("mode=%s registered=%d: received %s\n", mode.c_str(), (int)reg, ok ? "OK" : "WRONG");
    if (reg) {
        NK(ncclCommDeregister(comm, hs));
        NK(ncclCommDeregister(comm, hr));
    }
    NK(ncclCommDestroy(comm));
    return ok ? 0 : 5;
}
