// rccl_gap_probe: how long after RCCL's send/recv kernel does the next kernel on the same stream start?
// (Driver-cut trace with the RCCL self-exchange: the half-tile pass queued right behind the exchange
// started ~10 us after the RCCL kernel ended, profiles/kernel_trace_selfx_round4.txt.)  A 1-rank
// communicator; on one stream: stamp kernel A, [the exchange: ncclGroupStart / ncclSend + ncclRecv to
// self / ncclGroupEnd], [optional hipEventRecord], stamp kernel B.  The stamp kernels record
// s_memrealtime at their start; B.start - A.start is reported (median of 41), for:
//   0: A, B                     (baseline: one kernel boundary)
//   1: A, exchange, B
//   2: A, exchange, event record, B
//   3: A, exchange of 0 bytes (group with no ops), B
//   4: A, a hipMemcpyAsync D2D of the same bytes, B   (a copy instead of RCCL)
//   5: A, exchange, event (hipEventDisableSystemFence), B
//   6: A, exchange, event (hipEventReleaseToDevice), B
//   7: A, event (default), B                   (the event alone)
//   8: A, event (hipEventDisableSystemFence), B
//   9: A, exchange, hipStreamWriteValue32, B
//  10: A, hipStreamWriteValue32, B
//  11: A, hipStreamWaitValue32 on a value already written, B
//   build/rccl_gap_probe [bytes=81920]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)
#define NK(x)                                                                                   \
    do {                                                                                        \
        ncclResult_t r_ = (x);                                                                  \
        if (r_ != ncclSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_));   \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__global__ void stamp(unsigned long long* out, int slot) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[slot] = __builtin_amdgcn_s_memrealtime();
}

int main(int argc, char** argv) {
    const size_t bytes = argc > 1 ? (size_t)atoll(argv[1]) : 81920;
    CK(hipSetDevice(0));
    ncclUniqueId id;
    NK(ncclGetUniqueId(&id));
    ncclComm_t comm;
    NK(ncclCommInitRank(&comm, 1, id, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    char *sb, *rb;
    CK(hipMalloc(&sb, bytes));
    CK(hipMalloc(&rb, bytes));
    unsigned long long* st;
    CK(hipMalloc(&st, 64));
    hipEvent_t ev, ev_nf, ev_dev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev_nf, hipEventDisableTiming | hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&ev_dev, hipEventDisableTiming | hipEventReleaseToDevice));
    const char* names[] = {"A, B", "A, exchange, B", "A, exchange, event, B", "A, empty group, B", "A, D2D copy, B",
                           "A, exchange, event nofence, B", "A, exchange, event device, B", "A, event, B",
                           "A, event nofence, B", "A, exchange, write value, B", "A, write value, B",
                           "A, wait value (satisfied), B"};
    printf("rccl_gap_probe: %zu bytes each way, NCCL %d\n", bytes, NCCL_VERSION_CODE);
        unsigned* flag = nullptr;
    CK(hipMalloc(&flag, 256));
    CK(hipMemset(flag, 0, 256));
    for (int mode = 0; mode < 12; ++mode) {
        std::vector<double> d;
        for (int t = 0; t < 45; ++t) {
            hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, s, st, 0);
            if (mode == 1 || mode == 2 || mode == 5 || mode == 6 || mode == 9) {
                NK(ncclGroupStart());
                NK(ncclSend(sb, bytes, ncclChar, 0, comm, s));
                NK(ncclRecv(rb, bytes, ncclChar, 0, comm, s));
                NK(ncclGroupEnd());
                if (mode == 2) CK(hipEventRecord(ev, s));
                if (mode == 5) CK(hipEventRecord(ev_nf, s));
                if (mode == 6) CK(hipEventRecord(ev_dev, s));
                if (mode == 9) CK(hipStreamWriteValue32(s, flag, (unsigned)t + 1u, 0));
            } else if (mode == 10) {
                CK(hipStreamWriteValue32(s, flag, (unsigned)t + 1u, 0));
            } else if (mode == 11) {
                CK(hipStreamWaitValue32(s, flag, 0u, hipStreamWaitValueGte, 0xFFFFFFFFu));
            } else if (mode == 7 || mode == 8) {
                CK(hipEventRecord(mode == 7 ? ev : ev_nf, s));
            } else if (mode == 3) {
                NK(ncclGroupStart());
                NK(ncclGroupEnd());
            } else if (mode == 4) {
                CK(hipMemcpyAsync(rb, sb, bytes, hipMemcpyDeviceToDevice, s));
            }
            hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, s, st, 1);
            CK(hipStreamSynchronize(s));
            unsigned long long h[2];
            CK(hipMemcpy(h, st, 16, hipMemcpyDeviceToHost));
            if (t >= 4) d.push_back((double)(h[1] - h[0]) * 1e-2);  // 100 MHz ticks -> us
        }
        std::sort(d.begin(), d.end());
        printf("%-32s B.start - A.start: min %7.2f med %7.2f p90 %7.2f us\n", names[mode], d[0], d[d.size() / 2],
               d[d.size() * 9 / 10]);
    }
    NK(ncclCommDestroy(comm));
    return 0;
}
