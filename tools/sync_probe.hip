// Cross-queue synchronisation latency on one MI355X: how long after kernel A (stream 1) ends does
// kernel B (stream 2) start when B waits for A through
//   event      hipEventRecord(s1) + hipStreamWaitEvent(s2)
//   value      hipStreamWriteValue32(s1) + hipStreamWaitValue32(s2, >=)   (signal memory)
// and, on one stream, how long an event record between two kernels delays the second.  Kernels
// stamp wall_clock64() (100 MHz) at their start and end (thread 0 of block 0: start; the last block
// to finish: end), so no profiler is involved.  Each wait is bounded: B is enqueued only after the
// write (value mode) is enqueued, so every wait has its signal in flight.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            return 1;                                                              \
        }                                                                          \
    } while (0)

// busy kernel: every block spins ~us microseconds; stamps[0] = start (block 0), stamps[1] = end
// (last block to finish, via an atomic counter)
__global__ void busy(unsigned long long* stamps, unsigned* done, unsigned nblocks, unsigned long long ticks) {
    if (threadIdx.x == 0 && blockIdx.x == 0) stamps[0] = wall_clock64();
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const unsigned n = atomicAdd(done, 1u) + 1;
        if (n == nblocks) stamps[1] = wall_clock64();
    }
}

int main() {
    int dev = 0;
    CK(hipSetDevice(dev));
    int can_wait = 0;
    CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, dev));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, 0));
    CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, hi));
    const int nk = 64;
    unsigned long long* st = nullptr;
    unsigned* done = nullptr;
    CK(hipMalloc(&st, nk * 2 * sizeof(unsigned long long)));
    CK(hipMalloc(&done, nk * sizeof(unsigned)));
    unsigned* sig = nullptr;
    if (can_wait) CK(hipExtMallocWithFlags((void**)&sig, 8, hipMallocSignalMemory));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const unsigned nblocks = 256;
    const unsigned long long ticks = 3000;  // 30 us at 100 MHz
    printf("hipStreamWaitValue32 supported: %d\n", can_wait);
    for (int mode = 0; mode < 4; ++mode) {
        if (mode == 2 && !can_wait) continue;
        // 0: same stream, nothing between; 1: same stream, event record between; 2: two streams, value;
        // 3: two streams, event
        CK(hipMemset(done, 0, nk * sizeof(unsigned)));
        if (sig) CK(hipMemset(sig, 0, 8));
        CK(hipDeviceSynchronize());
        for (int i = 0; i < nk; i += 2) {
            hipLaunchKernelGGL(busy, dim3(nblocks), dim3(256), 0, s1, st + 2 * i, done + i, nblocks, ticks);
            hipStream_t sb = s1;
            if (mode == 1) CK(hipEventRecord(ev, s1));
            if (mode == 2) {
                CK(hipStreamWriteValue32(s1, sig, (uint32_t)(i / 2 + 1), 0));
                CK(hipStreamWaitValue32(s2, sig, (uint32_t)(i / 2 + 1), hipStreamWaitValueGte, 0xffffffffu));
                sb = s2;
            }
            if (mode == 3) {
                CK(hipEventRecord(ev, s1));
                CK(hipStreamWaitEvent(s2, ev, 0));
                sb = s2;
            }
            hipLaunchKernelGGL(busy, dim3(nblocks), dim3(256), 0, sb, st + 2 * (i + 1), done + i + 1, nblocks, ticks);
            // keep the pairs apart: the next A starts after this B on both streams
            CK(hipStreamSynchronize(s2));
            CK(hipStreamSynchronize(s1));
        }
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> h(nk * 2);
        CK(hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        std::vector<double> gaps;
        for (int i = 2; i < nk; i += 2) gaps.push_back((double)(h[2 * (i + 1)] - h[2 * i + 1]) * 0.01);  // us
        std::sort(gaps.begin(), gaps.end());
        static const char* names[] = {"same stream, back to back", "same stream, event record between",
                                      "two streams, write/wait value", "two streams, event record/wait"};
        printf("%-36s gap A end -> B start: min %6.2f  median %6.2f  max %6.2f us\n", names[mode], gaps.front(),
               gaps[gaps.size() / 2], gaps.back());
    }
    return 0;
}
