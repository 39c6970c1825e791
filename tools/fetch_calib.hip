// tools/fetch_calib.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on
// gfx950 for the access widths search_kernel uses (MI355X_MICROARCH.md: the
// counters are exact only for 16-B/lane streams; other widths must be
// calibrated on a known byte count).  Each kernel touches a known number of
// bytes of a 1 GiB buffer (4x the 256 MiB Infinity Cache, so nothing is served
// on-die); tools/pmc_traffic.py divides the counter by that count.
//
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib      (and --pmc WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <typename T>
__global__ void read_stream(const T* __restrict__ in, size_t n, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = in[i];
        const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
        for (size_t k = 0; k < (sizeof(T) + 3) / 4; k++) acc ^= w[k];
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;  // keeps the loads alive; never true on zeroed memory
}

__global__ void read_u8(const uint8_t* __restrict__ in, size_t n, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= in[i];
    if (acc == 0x9eu) sink[0] = acc;  // zeroed memory: never true
}

// gather every 8th u32 (one pool of 8 interleaved pools): touches every line
__global__ void read_stride8(const uint32_t* __restrict__ in, size_t n, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i * 8 < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= in[i * 8];
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

template <typename T>
__global__ void write_stream(T* __restrict__ out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = T{};
}

struct alignas(16) V16 { uint32_t a, b, c, d; };

int main() {
    const size_t bytes = 1ull << 30;
    uint8_t* buf;
    uint32_t* sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(buf, 0, bytes));
    const dim3 grid(4096), block(256);
    // launch order is the calibration table's row order (tools/pmc_traffic.py)
    read_stream<V16><<<grid, block>>>((const V16*)buf, bytes / 16, sink);
    read_stream<uint64_t><<<grid, block>>>((const uint64_t*)buf, bytes / 8, sink);
    read_stream<uint32_t><<<grid, block>>>((const uint32_t*)buf, bytes / 4, sink);
    read_u8<<<grid, block>>>(buf, bytes, sink);
    read_stride8<<<grid, block>>>((const uint32_t*)buf, bytes / 4, sink);
    write_stream<V16><<<grid, block>>>((V16*)buf, bytes / 16);
    write_stream<uint64_t><<<grid, block>>>((uint64_t*)buf, bytes / 8);
    write_stream<uint32_t><<<grid, block>>>((uint32_t*)buf, bytes / 4);
    write_stream<uint8_t><<<grid, block>>>(buf, bytes);
    CK(hipDeviceSynchronize());
    std::printf("fetch_calib: ok (%zu bytes per kernel)\n", bytes);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
