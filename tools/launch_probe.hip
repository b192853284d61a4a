// launch_probe: what the FIRST hipLaunchKernel after a host synchronisation costs on the host, and what
// moves it.  (The driver's timed run spends ~10 us inside its first launch call, 2.9 -> 13.0 us after
// run() is entered: profiles/launch_latency_round3.txt.)  Each case: a burst of `burst` kernels, a
// synchronisation, an optional action, then two timed launch calls (host wall of the call itself) and
// the time until the first kernel has run (hipStreamSynchronize after it).  Median of 41 trials.
//   build/launch_probe [burst=64]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

__global__ void tiny(unsigned* p, unsigned v) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && v == 0xFFFFFFFFu) p[0] = v;
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

int main(int argc, char** argv) {
    const int burst = argc > 1 ? atoi(argv[1]) : 64;
    unsigned* d = nullptr;
    CK(hipMalloc(&d, 256));
    hipStream_t s = nullptr, sp = nullptr;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&sp, hipStreamNonBlocking, hi));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    auto launch = [&](hipStream_t st) { hipLaunchKernelGGL(tiny, dim3(768), dim3(256), 0, st, d, 1u); };
    struct Case {
        const char* name;
        std::function<void(hipStream_t)> before;  // after the synchronisation, outside the timed call
        bool prio;
        bool device_sync;
    };
    std::vector<Case> cases = {
        {"stream sync, launch at once", [](hipStream_t) {}, false, false},
        {"device sync, launch at once", [](hipStream_t) {}, false, true},
        {"stream sync, hipStreamQuery first", [](hipStream_t st) { (void)hipStreamQuery(st); }, false, false},
        {"stream sync, event record+sync first", [&](hipStream_t st) { CK(hipEventRecord(ev, st)); CK(hipEventSynchronize(ev)); }, false, false},
        {"stream sync, 200 us idle first", [](hipStream_t) { std::this_thread::sleep_for(std::chrono::microseconds(200)); }, false, false},
        {"stream sync, 2 ms idle first", [](hipStream_t) { std::this_thread::sleep_for(std::chrono::milliseconds(2)); }, false, false},
        {"priority stream, stream sync", [](hipStream_t) {}, true, false},
        {"stream sync, hipGetLastError first", [](hipStream_t) { (void)hipGetLastError(); }, false, false},
    };
    for (int w = 0; w < 200; ++w) launch(s);
    CK(hipDeviceSynchronize());
    printf("launch_probe: burst %d, tiny kernel 768 x 256\n", burst);
    for (const Case& c : cases) {
        hipStream_t st = c.prio ? sp : s;
        std::vector<double> call1, call2, done;
        for (int t = 0; t < 41; ++t) {
            for (int i = 0; i < burst; ++i) launch(st);
            if (c.device_sync)
                CK(hipDeviceSynchronize());
            else
                CK(hipStreamSynchronize(st));
            c.before(st);
            const auto t0 = clk::now();
            launch(st);
            const auto t1 = clk::now();
            launch(st);
            const auto t2 = clk::now();
            CK(hipStreamSynchronize(st));
            const auto t3 = clk::now();
            call1.push_back(us(t0, t1));
            call2.push_back(us(t1, t2));
            done.push_back(us(t0, t3));
        }
        auto med = [](std::vector<double> v) {
            std::sort(v.begin(), v.end());
            return v[v.size() / 2];
        };
        printf("%-40s first call %6.2f us, second %6.2f us, both kernels done %6.2f us\n", c.name, med(call1), med(call2),
               med(done));
    }
    return 0;
}
