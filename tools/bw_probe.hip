// HBM streaming roofline probe (one MI355X): hipMemcpy D2D and a plain copy kernel over a 128 MiB
// board-sized buffer (read + write 256 MiB per pass), the floor of a shallow step_temporal pass.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                      \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

__global__ void copy16(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void copy8(const uint2* __restrict__ a, uint2* __restrict__ b, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// The temporal kernel's access pattern without its compute: each wave streams a column segment of 64
// words (uint2 per lane) down `rows` rows of `pitch` words, copying to the same place in `b`.
__global__ void colwalk(const uint2* __restrict__ a, uint2* __restrict__ b, long pitch, int nseg, int rows, int H) {
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int seg = wave % nseg, band = wave / nseg;
    const long r0 = (long)band * rows;
    if (r0 >= H) return;
    const long c = (long)seg * 62 + lane;
    if (c >= pitch) return;
    const uint2* p = a + r0 * pitch + c;
    uint2* q = b + r0 * pitch + c;
    const int n = (int)(r0 + rows <= H ? rows : H - r0);
    for (int i = 0; i < n; ++i) q[(long)i * pitch] = p[(long)i * pitch];
}
// The same, but like step_temporal's plan: lanes 0 and 63 are halo lanes that load and do not
// store (62-word output segments, 1 + 62 s .. 62 s + 62), and every row's store waits for the
// load two rows ahead (the 3-row window).
__global__ void colwalk62(const uint2* __restrict__ a, uint2* __restrict__ b, long pitch, int nseg, int rows, int H) {
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int seg = wave % nseg, band = wave / nseg;
    const long r0 = (long)band * rows;
    if (r0 >= H) return;
    const long c = (long)seg * 62 + lane;
    if (c >= pitch) return;
    const uint2* p = a + r0 * pitch + c;
    uint2* q = b + r0 * pitch + c;
    const int n = (int)(r0 + rows <= H ? rows : H - r0);
    const bool out = lane != 0 && lane != 63;
    uint2 w0 = p[0], w1 = p[pitch];
    for (int i = 0; i < n; ++i) {
        const uint2 w2 = p[(long)(i + 2) * pitch];
        const uint2 v = make_uint2(w0.x ^ w1.x ^ w2.x, w0.y ^ w1.y ^ w2.y);
        if (out) q[(long)i * pitch] = v;
        w0 = w1;
        w1 = w2;
    }
}

int main() {
    const size_t bytes = (size_t)128 << 20;
    void *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int variant = 0; variant < 5; ++variant) {
        float best = 1e30f;
        for (int rep = 0; rep < 20; ++rep) {
            CK(hipEventRecord(e0, 0));
            if (variant == 0) CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0));
            if (variant == 1) hipLaunchKernelGGL(copy16, dim3(256 * 8), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16);
            if (variant == 2) hipLaunchKernelGGL(copy16, dim3(256 * 32), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16);
            if (variant == 3) hipLaunchKernelGGL(copy8, dim3(256 * 8), dim3(256), 0, 0, (const uint2*)a, (uint2*)b, bytes / 8);
            if (variant == 4) hipLaunchKernelGGL(copy8, dim3(256 * 32), dim3(256), 0, 0, (const uint2*)a, (uint2*)b, bytes / 8);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        static const char* names[] = {"hipMemcpy D2D", "copy16 2048 WGs", "copy16 8192 WGs", "copy8 2048 WGs",
                                      "copy8 8192 WGs"};
        printf("%-18s 128 MiB: %7.1f us  %.2f TB/s (read+write)\n", names[variant], best * 1e3,
               2.0 * bytes / (best * 1e-3) / 1e12);
    }
    // column walks over a 32768 x 32768 bit board (pitch 514 words as the engine pads it, or 512)
    for (long pitch : {514L, 512L, 520L}) {
        for (int rows : {45, 90, 360, 32768}) {
            const int H = 32768, nseg = (int)((pitch - 2 + 61) / 62);
            const int waves = nseg * ((H + rows - 1) / rows);
            float best = 1e30f;
            for (int rep = 0; rep < 10; ++rep) {
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(colwalk, dim3((waves + 3) / 4), dim3(256), 0, 0, (const uint2*)a, (uint2*)b, pitch, nseg,
                                   rows, (int)((bytes / 8) / pitch));
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            printf("colwalk pitch %ld rows/wave %5d waves %6d: %7.1f us\n", pitch, rows, waves, best * 1e3);
        }
    }
    for (int rows : {34, 45, 90}) {
        const long pitch = 514;
        // rows the 128 MiB buffer holds, minus the two rows the window reads ahead
        const int H = (int)((bytes / 8) / pitch) - 2, nseg = (int)((pitch - 2 + 61) / 62);
        const int waves = nseg * ((H + rows - 1) / rows);
        float best = 1e30f;
        for (int rep = 0; rep < 10; ++rep) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(colwalk62, dim3((waves + 3) / 4), dim3(256), 0, 0, (const uint2*)a, (uint2*)b, pitch, nseg,
                               rows, H);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        printf("colwalk62 (halo lanes do not store, 3-row window) rows/wave %d waves %d: %7.1f us\n", rows, waves, best * 1e3);
    }
    return 0;
}
