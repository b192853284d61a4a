// Probe: do two HIP streams still run kernels concurrently once an RCCL communicator exists in the
// process?  (Kernel traces of the sub-tile mode with a 1-rank RCCL communicator showed both
// streams' kernels serialised on one hardware queue.)  Two 1-workgroup spin kernels of ~2 ms are
// launched on two streams; concurrent -> ~2 ms, serialised -> ~4 ms.
//   hipcc -O2 --offload-arch=gfx950 tools/queue_probe.cpp -lrccl -o build/queue_probe
//   build/queue_probe <mode>   0: no RCCL   1: RCCL, then streams   2: streams, then RCCL
//                              3: RCCL, then streams with different priorities
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
    do {                                                                          \
        auto r_ = (x);                                                            \
        if (r_ != 0) {                                                            \
            fprintf(stderr, "%s failed: %d at line %d\n", #x, (int)r_, __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

__global__ void spin(long long cycles, int* out) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    int* d;
    CK(hipMalloc(&d, 1024));
    ncclComm_t comm = nullptr;
    hipStream_t s[2];
    auto make_streams = [&]() {
        if (mode == 3) {
            int lo = 0, hi = 0;
            CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
            printf("priority range %d..%d\n", lo, hi);
            CK(hipStreamCreateWithPriority(&s[0], hipStreamNonBlocking, lo));
            CK(hipStreamCreateWithPriority(&s[1], hipStreamNonBlocking, hi));
        } else {
            for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        }
    };
    auto make_comm = [&]() {
        ncclUniqueId id;
        CK(ncclGetUniqueId(&id));
        CK(ncclCommInitRank(&comm, 1, id, 0));
    };
    if (mode == 2) {
        make_streams();
        make_comm();
    } else {
        if (mode == 1 || mode == 3) make_comm();
        make_streams();
    }
    // calibrate: ~2 ms at the current clock
    const long long cyc = 200000000LL / 100;  // ~2e6 cycles (clock64 runs at the shader clock / a fixed rate)
    for (int w = 0; w < 2; ++w) {
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[0], cyc, d);
        CK(hipStreamSynchronize(s[0]));
    }
    auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[0], cyc, d);
    CK(hipStreamSynchronize(s[0]));
    const double one = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[0], cyc, d);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[1], cyc, d);
    CK(hipStreamSynchronize(s[0]));
    CK(hipStreamSynchronize(s[1]));
    const double two = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("mode %d: one kernel %.3f ms, two kernels on two streams %.3f ms -> %s\n", mode, one, two,
           two < 1.5 * one ? "CONCURRENT" : "SERIALISED");
    if (comm) CK(ncclCommDestroy(comm));
    return 0;
}
