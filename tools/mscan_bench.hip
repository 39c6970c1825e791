// tools/mscan_bench.hip — the library's mscan_kernel in isolation on C3's
// shape (1M candidates in scan order, 8 term-only pool signatures over two
// keyword fields, Min = Max = 10), timed with the dispatch's start/stop event
// pair "cold" (after an evicting 512 MB write and 10 ms of host sleep, as
// after the pass's host replay) and "warm" (right after an identical launch),
// next to tools/mscan_roof.hip's loads-only floor.  Compiles the kernels'
// translation unit itself (mm_kernels.hip) so kernel variants can be A/B'd
// without the rest of the pass.
#include "../nakama_amd/csrc/mm_kernels.hip"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void evict_kernel(uint4* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = uint4{(uint32_t)i, 0, 0, 0};
}

int main() {
    using namespace nkm;
    const uint32_t n = 1u << 20;
    std::vector<uint32_t> order(n);
    std::vector<uint8_t> alive(n, 1), kind(n, KIND_KEYWORD);
    std::vector<int32_t> cnt(n, 10);
    std::vector<int64_t> mode(n), region(n);
    uint64_t x = 0x5EED0003;
    for (uint32_t i = 0; i < n; i++) {
        order[i] = i;
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        mode[i] = 1 + ((x >> 33) & 1);
        region[i] = 3 + ((x >> 40) & 3);
    }
    auto up = [](const void* h, size_t bytes) {
        void* d = nullptr;
        (void)hipMalloc(&d, bytes);
        (void)hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
        return d;
    };
    DStore st{};
    st.alive = (const uint8_t*)up(alive.data(), n);
    st.minc = (const int32_t*)up(cnt.data(), 4 * (size_t)n);
    st.maxc = (const int32_t*)up(cnt.data(), 4 * (size_t)n);
    st.party = nullptr;
    st.order = (const uint32_t*)up(order.data(), 4 * (size_t)n);
    const int64_t* fv[2] = {(const int64_t*)up(mode.data(), 8 * (size_t)n), (const int64_t*)up(region.data(), 8 * (size_t)n)};
    const uint8_t* fk[2] = {(const uint8_t*)up(kind.data(), n), (const uint8_t*)up(kind.data(), n)};
    st.fval = (const int64_t* const*)up(fv, sizeof fv);
    st.fkind = (const uint8_t* const*)up(fk, sizeof fk);
    DMScan ms{};
    ms.src_off = 0;
    ms.src_len = n;
    ms.n_sigs = 8;
    ms.chunk = (uint32_t)mscan_chunk_len(8);
    ms.n_chunks = (n + ms.chunk - 1) / ms.chunk;
    ms.n_fields = 2;
    ms.n_clauses = 0;
    ms.field[0] = 0;
    ms.field[1] = 1;
    std::vector<DMSig> sigs(8);
    for (int q = 0; q < 8; q++) {
        DMSig& g = sigs[q];
        std::memset(&g, 0, sizeof g);
        g.req[0] = 1 + (q & 1);
        g.req[1] = 3 + (q >> 1);
        g.tmin = 10;
        g.tmax = 10;
        g.term_only = 1;
        g.req_mask = 3;
        g.qkind = QK_BOOL;
    }
    const DMSig* d_sigs = (const DMSig*)up(sigs.data(), sigs.size() * sizeof(DMSig));
    DClause dummy{};
    const DClause* d_mcl = (const DClause*)up(&dummy, sizeof dummy);
    uint32_t* d_cells;
    DGroupResult* d_res;
    CK(hipMalloc(&d_cells, (size_t)ms.n_sigs * ms.n_chunks * ms.chunk * 4));
    CK(hipMalloc(&d_res, (size_t)ms.n_sigs * ms.n_chunks * sizeof(DGroupResult)));
    const size_t evict_n = (512ull << 20) / 16;
    uint4* evict;
    CK(hipMalloc(&evict, evict_n * 16));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipDeviceSynchronize());
    const double bytes = (double)n * (5 + 8 + 18) + (double)n * 4;  // PassStats.k_bytes[2]: every candidate live, one hit each
    for (int cold = 1; cold >= 0; cold--) {
        std::vector<float> t;
        for (int r = 0; r < 21; r++) {
            if (cold) {
                hipLaunchKernelGGL(evict_kernel, dim3(2048), dim3(256), 0, s, evict, evict_n);
                CK(hipStreamSynchronize(s));
                std::this_thread::sleep_for(std::chrono::milliseconds(10));
            } else {
                CK(launch_mscan(st, ms, d_sigs, d_mcl, d_cells, d_res, false, s, e0, e1));
            }
            CK(launch_mscan(st, ms, d_sigs, d_mcl, d_cells, d_res, false, s, e0, e1));
            CK(hipEventSynchronize(e1));
            float ms_;
            CK(hipEventElapsedTime(&ms_, e0, e1));
            if (r) t.push_back(ms_);
        }
        std::sort(t.begin(), t.end());
        const double us = 1e3 * t[t.size() / 2];
        std::printf("mscan_kernel (chunk %u) %-4s median %7.2f us  min %7.2f us -> %6.0f GB/s of %.2f MB (frac %.3f)\n",
                    ms.chunk, cold ? "cold" : "warm", us, 1e3 * t[0], bytes / us / 1e3, bytes / 1e6,
                    bytes / us / 1e3 / 8000.0);
    }
    // the hits: every candidate matches exactly one signature
    std::vector<DGroupResult> res((size_t)ms.n_sigs * ms.n_chunks);
    CK(hipMemcpy(res.data(), d_res, res.size() * sizeof(DGroupResult), hipMemcpyDeviceToHost));
    uint64_t hits = 0;
    for (auto& r : res) hits += r.count;
    std::printf("hits %llu of %u candidates\n", (unsigned long long)hits, n);
    return hits == n ? 0 : 2;
}
