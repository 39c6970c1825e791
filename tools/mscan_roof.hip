// tools/mscan_roof.hip — the attainable duration of ONE launch that moves
// mscan_kernel's bytes on C3 (1M candidates: 4-B scan-order slot id, 1-B
// alive, 2 x 4-B Min/MaxCount, 2 fields x (1-B kind + 8-B value), one 4-B
// write per candidate: 35 MB), measured with the same start/stop event pair
// the library binds to its dispatch (hipExtLaunchKernelGGL).  Variants:
//   direct   columns indexed by position (no slot indirection), loads only
//   gather   slot = order[i], then the columns at slot (mscan's chain)
//   grid     one round of 512-candidate workgroups (mscan's shape) vs a
//            grid-stride loop over 2 x CUs workgroups (persistent shape)
// and two states before the launch: "cold" (10 ms of host sleep after a
// 512 MB write that evicts L2 and the Infinity Cache, as after the pass's host
// replay) and "warm" (right after an identical launch).  Also a 2 GB stream
// for the chip's sustained rate.  Output: one line per (variant, state):
// median microseconds over 20 launches and the implied GB/s of 35 MB.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Cols {
    const uint32_t* order;
    const uint8_t* alive;
    const int32_t* minc;
    const int32_t* maxc;
    const uint8_t* k0;
    const uint8_t* k1;
    const int64_t* v0;
    const int64_t* v1;
    uint32_t* out;
    uint32_t n;
};

constexpr int kBlock = 256;

template <bool GATHER>
__device__ __forceinline__ uint32_t touch(const Cols& c, uint32_t i) {
    const uint32_t s = GATHER ? c.order[i] : i;
    const uint32_t a = c.alive[s];
    const int32_t mn = c.minc[s], mx = c.maxc[s];
    const uint32_t ka = c.k0[s], kb = c.k1[s];
    const int64_t va = c.v0[s], vb = c.v1[s];
    // a predicate shaped like a pool signature's (alive, count range, two terms)
    const bool m = a && mn >= 10 && mx <= 10 && ka == 1 && kb == 1 && va == 3 && vb == 5;
    return m ? s : ~0u;
}

// one round: 2 candidates per lane, both loaded before either is used
template <bool GATHER>
__global__ __launch_bounds__(kBlock) void round_kernel(Cols c) {
    const uint32_t i0 = blockIdx.x * 2 * kBlock + threadIdx.x, i1 = i0 + kBlock;
    const uint32_t a = i0 < c.n ? touch<GATHER>(c, i0) : ~0u;
    const uint32_t b = i1 < c.n ? touch<GATHER>(c, i1) : ~0u;
    if (i0 < c.n) c.out[i0] = a;
    if (i1 < c.n) c.out[i1] = b;
}

template <bool GATHER>
__global__ __launch_bounds__(kBlock) void stride_kernel(Cols c) {
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < c.n; i += gridDim.x * kBlock) c.out[i] = touch<GATHER>(c, i);
}

__global__ void stream_kernel(const uint4* __restrict__ in, size_t n, uint4* __restrict__ out) {
    uint4 acc{0, 0, 0, 0};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = in[i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if (acc.x == 0x9e3779b9u) out[0] = acc;
}

__global__ void fill_kernel(uint4* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = uint4{(uint32_t)i, 0, 0, 0};
}

int main() {
    const uint32_t n = 1u << 20;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    std::vector<uint32_t> order(n);
    for (uint32_t i = 0; i < n; i++) order[i] = i;
    Cols c{};
    c.n = n;
    void* p;
    CK(hipMalloc(&p, n * 4)); c.order = (const uint32_t*)p;
    CK(hipMemcpy(p, order.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&p, n)); CK(hipMemset(p, 1, n)); c.alive = (const uint8_t*)p;
    CK(hipMalloc(&p, n * 4)); CK(hipMemset(p, 0, n * 4)); c.minc = (const int32_t*)p;
    CK(hipMalloc(&p, n * 4)); CK(hipMemset(p, 0, n * 4)); c.maxc = (const int32_t*)p;
    CK(hipMalloc(&p, n)); CK(hipMemset(p, 1, n)); c.k0 = (const uint8_t*)p;
    CK(hipMalloc(&p, n)); CK(hipMemset(p, 1, n)); c.k1 = (const uint8_t*)p;
    CK(hipMalloc(&p, n * 8)); CK(hipMemset(p, 0, n * 8)); c.v0 = (const int64_t*)p;
    CK(hipMalloc(&p, n * 8)); CK(hipMemset(p, 0, n * 8)); c.v1 = (const int64_t*)p;
    CK(hipMalloc(&p, n * 4)); c.out = (uint32_t*)p;
    const double bytes = (double)n * (4 + 1 + 8 + 2 * 9 + 4);
    const size_t evict_n = (512ull << 20) / 16, stream_n = (2048ull << 20) / 16;
    uint4 *evict, *big, *sink;
    CK(hipMalloc(&evict, evict_n * 16));
    CK(hipMalloc(&big, stream_n * 16));
    CK(hipMalloc(&sink, 16));
    hipLaunchKernelGGL(fill_kernel, dim3(cus * 8), dim3(256), 0, 0, big, stream_n);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());

    auto run = [&](int variant) -> hipError_t {
        const dim3 b(kBlock);
        switch (variant) {
            case 0: hipExtLaunchKernelGGL(round_kernel<false>, dim3((n + 2 * kBlock - 1) / (2 * kBlock)), b, 0, s, e0, e1, 0, c); break;
            case 1: hipExtLaunchKernelGGL(round_kernel<true>, dim3((n + 2 * kBlock - 1) / (2 * kBlock)), b, 0, s, e0, e1, 0, c); break;
            case 2: hipExtLaunchKernelGGL(stride_kernel<false>, dim3(cus * 2), b, 0, s, e0, e1, 0, c); break;
            case 3: hipExtLaunchKernelGGL(stride_kernel<true>, dim3(cus * 2), b, 0, s, e0, e1, 0, c); break;
            case 4: hipExtLaunchKernelGGL(stride_kernel<true>, dim3(cus * 8), b, 0, s, e0, e1, 0, c); break;
        }
        return hipGetLastError();
    };
    const char* names[] = {"round direct", "round gather", "stride2xCU direct", "stride2xCU gather", "stride8xCU gather"};
    for (int v = 0; v < 5; v++) {
        for (int cold = 1; cold >= 0; cold--) {
            std::vector<float> t;
            for (int r = 0; r < 21; r++) {
                if (cold) {
                    hipLaunchKernelGGL(fill_kernel, dim3(cus * 8), dim3(256), 0, s, evict, evict_n);
                    CK(hipStreamSynchronize(s));
                    std::this_thread::sleep_for(std::chrono::milliseconds(10));
                } else {
                    CK(run(v));
                }
                CK(run(v));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            const double us = 1e3 * t[t.size() / 2];
            std::printf("%-20s %-4s median %7.2f us  min %7.2f us  -> %6.0f GB/s of 35.65 MB (frac %.3f)\n", names[v],
                        cold ? "cold" : "warm", us, 1e3 * t[0], bytes / us / 1e3, bytes / us / 1e3 / 8000.0);
        }
    }
    // sustained: 2 GB streamed
    std::vector<float> t;
    for (int r = 0; r < 6; r++) {
        hipExtLaunchKernelGGL(stream_kernel, dim3(cus * 8), dim3(256), 0, s, e0, e1, 0, (const uint4*)big, stream_n, sink);
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    std::printf("stream 2 GiB          median %7.2f us -> %6.0f GB/s\n", 1e3 * t[t.size() / 2],
                (double)stream_n * 16 / (1e3 * t[t.size() / 2]) / 1e3);
    // a launch that does nothing: the event pair's floor
    t.clear();
    for (int r = 0; r < 21; r++) {
        Cols z = c;
        z.n = 0;
        hipExtLaunchKernelGGL(round_kernel<false>, dim3(2048), dim3(kBlock), 0, s, e0, e1, 0, z);
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    std::printf("empty 2048-WG launch  median %7.2f us\n", 1e3 * t[t.size() / 2]);
    return 0;
}
