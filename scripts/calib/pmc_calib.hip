// Calibration of the L2 memory-side request counters on gfx950 against known byte counts
// (MI355X_MICROARCH.md, HBM: "other access widths are uncalibrated: calibrate on a known byte count
// in your own access pattern").  Each kernel touches a 1 GiB buffer (4x the Infinity Cache) once in
// one of the access patterns the engine's kernels use; scripts/pmc_traffic.py compares FETCH_SIZE,
// the size-resolved read requests (TCC_EA0_RDREQ_32B/64B/128B) and WRITE_SIZE with these counts.
//
//   k_rd16   16 B per lane, coalesced          1 GiB read
//   k_rd8     8 B per lane, coalesced          1 GiB read
//   k_rd4     4 B per lane, coalesced          1 GiB read
//   k_gat16  16 B per lane at random 16-B slots (the vote's member records)   2^24 gathers
//   k_gat4    4 B per lane at random 4-B slots (the pairing's key lookups)    2^24 gathers
//   k_wr16   16 B per lane, coalesced          1 GiB written
//   k_wr4     4 B per lane, coalesced          1 GiB written
//
// Each read kernel folds what it read into one word per thread (2 MiB of output), so the reads
// cannot be dropped.  Build: hipcc --offload-arch=gfx950 -O3 -o build/calib/pmc_calib pmc_calib.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

constexpr int T = 256, B = 2048;   // 2^19 threads

template <typename V>
__device__ __forceinline__ uint32_t fold(const V& v);
template <>
__device__ __forceinline__ uint32_t fold(const uint4& v) { return v.x ^ v.y ^ v.z ^ v.w; }
template <>
__device__ __forceinline__ uint32_t fold(const uint2& v) { return v.x ^ v.y; }
template <>
__device__ __forceinline__ uint32_t fold(const uint32_t& v) { return v; }

template <typename V>
__global__ __launch_bounds__(T) void k_rd(const V* __restrict__ a, int64_t n, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    const int64_t stride = (int64_t)gridDim.x * T;
    for (int64_t i = (int64_t)blockIdx.x * T + threadIdx.x; i < n; i += stride) acc ^= fold(a[i]);
    out[(int64_t)blockIdx.x * T + threadIdx.x] = acc;
}

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

template <typename V>
__global__ __launch_bounds__(T) void k_gat(const V* __restrict__ a, int64_t n, int64_t g, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    const int64_t stride = (int64_t)gridDim.x * T;
    for (int64_t i = (int64_t)blockIdx.x * T + threadIdx.x; i < g; i += stride) acc ^= fold(a[mix((uint64_t)i) % (uint64_t)n]);
    out[(int64_t)blockIdx.x * T + threadIdx.x] = acc;
}

template <typename V>
__global__ __launch_bounds__(T) void k_wr(V* __restrict__ a, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * T;
    for (int64_t i = (int64_t)blockIdx.x * T + threadIdx.x; i < n; i += stride) {
        V v;
        uint32_t* w = reinterpret_cast<uint32_t*>(&v);
        for (int k = 0; k < (int)(sizeof(V) / 4); ++k) w[k] = (uint32_t)i + k;
        a[i] = v;
    }
}

int main() {
    const int64_t bytes = 1LL << 30, gathers = 1LL << 24;
    void* buf;
    uint32_t* out;
    CHK(hipMalloc(&buf, bytes));
    CHK(hipMalloc((void**)&out, sizeof(uint32_t) * T * B));
    CHK(hipMemset(buf, 1, bytes));
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto timed = [&](const char* name, double known, auto launch) {
        CHK(hipEventRecord(e0, 0));
        launch();
        CHK(hipEventRecord(e1, 0));
        CHK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"kernel\": \"%s\", \"known_bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}\n", name, known, ms,
                    known / (ms * 1e6));
    };
    for (int rep = 0; rep < 2; ++rep) {   // (the second round is the one to read: warm code, same counts)
        timed("k_rd16", (double)bytes, [&] {
            hipLaunchKernelGGL(k_rd<uint4>, dim3(B), dim3(T), 0, 0, (const uint4*)buf, bytes / 16, out);
        });
        timed("k_rd8", (double)bytes, [&] {
            hipLaunchKernelGGL(k_rd<uint2>, dim3(B), dim3(T), 0, 0, (const uint2*)buf, bytes / 8, out);
        });
        timed("k_rd4", (double)bytes, [&] {
            hipLaunchKernelGGL(k_rd<uint32_t>, dim3(B), dim3(T), 0, 0, (const uint32_t*)buf, bytes / 4, out);
        });
        timed("k_gat16", (double)gathers * 16, [&] {
            hipLaunchKernelGGL(k_gat<uint4>, dim3(B), dim3(T), 0, 0, (const uint4*)buf, bytes / 16, gathers, out);
        });
        timed("k_gat4", (double)gathers * 4, [&] {
            hipLaunchKernelGGL(k_gat<uint32_t>, dim3(B), dim3(T), 0, 0, (const uint32_t*)buf, bytes / 4, gathers, out);
        });
        timed("k_wr16", (double)bytes, [&] { hipLaunchKernelGGL(k_wr<uint4>, dim3(B), dim3(T), 0, 0, (uint4*)buf, bytes / 16); });
        timed("k_wr4", (double)bytes, [&] { hipLaunchKernelGGL(k_wr<uint32_t>, dim3(B), dim3(T), 0, 0, (uint32_t*)buf, bytes / 4); });
    }
    CHK(hipGetLastError());
    CHK(hipDeviceSynchronize());
    CHK(hipFree(buf));
    CHK(hipFree(out));
    return 0;
}
