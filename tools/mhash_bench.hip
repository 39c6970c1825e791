// tools/mhash_bench.hip — the library's hashed mscan (mscan_hash_kernel +
// mscan_base_kernel + mscan_place_kernel) in isolation, on C4's shape (4M
// candidates, 64 term-only pool signatures over two keyword fields) and C3's
// (1M, 8), every chunk shape (gathered J = 2/4, contiguous J = 4/8), timed by
// the hash kernel's start/stop event pair cold (after an evicting 512 MB
// write) and warm; then the same with phases switched off (NKM_MH_DEBUG:
// 1 = no table probe, 2 = no ranking/scatter, 4 = no LDS signature load) to
// find where the time goes.  Checks every list against a host partition.
#define NKM_MH_DEBUG 1
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
// evicts by reading (clean lines): no write-backs left for the timed kernel
__global__ void evict_read_kernel(const uint4* p, size_t n, uint32_t* sink) {
    uint32_t x = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) x ^= p[i].x;
    if (x == 0x12345678u) sink[0] = x;
}

static int run_shape(uint32_t n, int nmode, int nregion, uint4* evict, size_t evict_n) {
    using namespace nkm;
    const uint32_t nq = (uint32_t)(nmode * nregion);
    std::vector<uint32_t> order(n);
    std::vector<uint8_t> alive(n, 1), kind(n, KIND_KEYWORD);
    std::vector<int32_t> cnt(n, 2);
    std::vector<int64_t> mode(n), region(n);
    uint64_t x = 0x5EED0004;
    for (uint32_t i = 0; i < n; i++) {
        order[i] = i;
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        mode[i] = 100 + (int64_t)((x >> 33) % nmode);
        region[i] = 200 + (int64_t)((x >> 45) % nregion);
        if ((x >> 20) % 97 == 0) alive[i] = 0;
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
    st.order = (const uint32_t*)up(order.data(), 4 * (size_t)n);
    const int64_t* fv[2] = {(const int64_t*)up(mode.data(), 8 * (size_t)n), (const int64_t*)up(region.data(), 8 * (size_t)n)};
    const uint8_t* fk[2] = {(const uint8_t*)up(kind.data(), n), (const uint8_t*)up(kind.data(), n)};
    st.fval = (const int64_t* const*)up(fv, sizeof fv);
    st.fkind = (const uint8_t* const*)up(fk, sizeof fk);
    // signatures, output offsets, table: the host side of mm_process.cpp
    std::vector<DMSig> sigs(nq);
    std::vector<uint64_t> listlen(nq, 0);
    for (uint32_t i = 0; i < n; i++)
        if (alive[i]) listlen[(mode[i] - 100) * nregion + (region[i] - 200)]++;
    std::vector<uint64_t> dst(nq);
    uint64_t off = 0;
    for (uint32_t q = 0; q < nq; q++) {
        DMSig& g = sigs[q];
        std::memset(&g, 0, sizeof g);
        g.req[0] = 100 + q / nregion;
        g.req[1] = 200 + q % nregion;
        g.tmin = 2;
        g.tmax = 2;
        g.term_only = 1;
        g.req_mask = 3;
        g.qkind = QK_BOOL;
        dst[q] = off;
        off += listlen[q] + 7;
    }
    // the cuckoo table, as mm_process.cpp plan_mscan_hash builds it
    auto hash = [](uint32_t seed, const DMSig& m) { return msig_fin(msig_mix(msig_mix(seed, (uint32_t)m.req[0]), (uint32_t)m.req[1])); };
    uint32_t cap = 4, s0 = 0, s1 = 0;
    std::vector<uint32_t> slot;
    for (bool placed = false; !placed; cap <<= 1) {
        if (cap < 2 * nq) continue;
        for (uint32_t attempt = 0; attempt < 32 && !placed; attempt++) {
            s0 = 0x2545F491u * (2 * attempt + 1);
            s1 = 0x9E3779B9u * (2 * attempt + 2);
            slot.assign(cap, kMHashEmpty);
            bool ok = true;
            for (uint32_t q = 0; q < nq && ok; q++) {
                uint32_t cur = q, pos = hash(s0, sigs[q]) & (cap - 1);
                for (uint32_t kick = 0;; kick++) {
                    if (slot[pos] == kMHashEmpty) { slot[pos] = cur; break; }
                    if (kick == 4 * cap) { ok = false; break; }
                    std::swap(cur, slot[pos]);
                    const uint32_t p0 = hash(s0, sigs[cur]) & (cap - 1), p1 = hash(s1, sigs[cur]) & (cap - 1);
                    pos = pos == p0 ? p1 : p0;
                }
            }
            placed = ok;
        }
        if (placed) break;
    }
    std::vector<DMHashEntry> htab(cap, DMHashEntry{});
    for (uint32_t p = 0; p < cap; p++) {
        htab[p].q = slot[p];
        if (slot[p] == kMHashEmpty) continue;
        htab[p].key[0] = (uint32_t)sigs[slot[p]].req[0];
        htab[p].key[1] = (uint32_t)sigs[slot[p]].req[1];
        htab[p].tmin = sigs[slot[p]].tmin;
        htab[p].tmax = sigs[slot[p]].tmax;
    }
    // the key grid (mm_process.cpp plan_key_grid): modes x regions cells
    const uint32_t cells = (uint32_t)(nmode * nregion);
    const size_t gbytes = ((size_t)cells * 2 + 15) & ~(size_t)15;
    std::vector<char> grid(gbytes + (((size_t)nq * 8 + 15) & ~(size_t)15), 0);
    for (uint32_t k = 0; k < cells; k++) reinterpret_cast<uint16_t*>(grid.data())[k] = 0xFFFFu;
    for (uint32_t q = 0; q < nq; q++) {
        const uint32_t idx = (uint32_t)(sigs[q].req[0] - 100) * nregion + (uint32_t)(sigs[q].req[1] - 200);
        reinterpret_cast<uint16_t*>(grid.data())[idx] = (uint16_t)q;
        reinterpret_cast<int32_t*>(grid.data() + gbytes)[2 * q] = sigs[q].tmin;
        reinterpret_cast<int32_t*>(grid.data() + gbytes)[2 * q + 1] = sigs[q].tmax;
    }
    std::vector<char> blob(mscan_hash_blob_bytes(nq, cap, cells));
    std::memcpy(blob.data(), sigs.data(), nq * sizeof(DMSig));
    std::memcpy(blob.data() + nq * sizeof(DMSig), dst.data(), nq * 8);
    std::memcpy(blob.data() + mscan_hash_table_off(nq), htab.data(), cap * sizeof(DMHashEntry));
    std::memcpy(blob.data() + mscan_hash_table_off(nq) + cap * sizeof(DMHashEntry), grid.data(), grid.size());
    std::printf("cuckoo table: %u entries for %u signatures\n", cap, nq);
    const void* d_blob = up(blob.data(), blob.size());
    uint32_t* d_out;
    CK(hipMalloc(&d_out, (off + n) * 4 + 64));  // dbg 1 places by another partition
    DGroupResult* d_res;
    CK(hipMalloc(&d_res, nq * sizeof(DGroupResult)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    // algorithmic bytes: per candidate its slot id (gathered only), alive flag,
    // counts and two (kind, value) columns; per hit its 4-B slot id
    auto bytes_of = [&](bool contig) { return (double)n * (contig ? 1 + 8 + 18 : 5 + 8 + 18) + (double)n * 4; };
    // grid: the key-grid lookup (else the cuckoo table); loop 2: counts only
    struct Shape { int contig, j, grid, loop; };
    const Shape shapes[] = {{0, 4, 0, 0}, {0, 4, 1, 0}, {1, 4, 0, 0}, {1, 4, 1, 0}, {1, 8, 0, 0}, {1, 8, 1, 0},
                            {1, 2, 1, 0}, {1, 4, 1, 2}, {1, 8, 1, 2}, {1, 2, 1, 2}, {1, 4, 0, 2}};
    for (const Shape& sh : shapes) {
        for (uint32_t dbg : {0u, 1u, 2u}) {
            if (sh.loop && dbg) continue;
            DMScan ms{};
            ms.src_off = 0;
            ms.src_len = n;
            ms.n_sigs = nq;
            ms.n_fields = 2;
            ms.field[0] = 0;
            ms.field[1] = 1;
            ms.hmask = cap - 1;
            ms.hseed[0] = s0;
            ms.hseed[1] = s1;
            if (sh.grid) {
                ms.dsize = cells;
                ms.dlo[0] = 100;
                ms.dlo[1] = 200;
                ms.drng[0] = (uint32_t)nmode;
                ms.drng[1] = (uint32_t)nregion;
            }
            ms.contig = (uint32_t)sh.contig;
            ms.chunk = (uint32_t)(sh.j * 256);
            ms.n_chunks = (n + ms.chunk - 1) / ms.chunk;
            ms.pad = dbg;
            uint32_t* d_work;
            const uint64_t ww = mscan_hash_work_words(ms) + (uint64_t)ms.n_chunks * 256 + 16;  // dbg 2: a word per thread
            CK(hipMalloc(&d_work, ww * 4));
            for (int cold = 2; cold >= 0; cold--) {  // 2: evicted by writes, 1: by reads, 0: warm
                std::vector<float> t, tall;
                for (int r = 0; r < 11; r++) {
                    if (cold == 2) hipLaunchKernelGGL(evict_kernel, dim3(2048), dim3(256), 0, s, evict, evict_n);
                    if (cold == 1)
                        hipLaunchKernelGGL(evict_read_kernel, dim3(2048), dim3(256), 0, s, evict, evict_n,
                                           reinterpret_cast<uint32_t*>(d_res));
                    if (cold) {
                        CK(hipStreamSynchronize(s));
                        std::this_thread::sleep_for(std::chrono::milliseconds(5));
                    }
                    const int ph = kMHashEval | kMHashPlace | (sh.loop == 2 ? kMHashCount : 0);
                    CK(launch_mscan_hash(st, ms, d_blob, d_work, d_res, d_out, s, e0, e1, ph, 0, UINT32_MAX));
                    CK(hipEventRecord(e2, s));
                    CK(hipEventSynchronize(e2));
                    float a, b;
                    CK(hipEventElapsedTime(&a, e0, e1));
                    CK(hipEventElapsedTime(&b, e0, e2));
                    if (r) { t.push_back(a); tall.push_back(b); }
                }
                std::sort(t.begin(), t.end());
                std::sort(tall.begin(), tall.end());
                const double us = 1e3 * t[t.size() / 2];
                std::printf("n %u sigs %3u %s J%d %s %s dbg %u %-4s hash kernel %7.2f us (frac %.3f)  all %7.2f us\n", n, nq,
                            sh.contig ? "contig" : "gather", sh.j, sh.grid ? "grid  " : "cuckoo", sh.loop == 2 ? "count" : "lists",
                            dbg, cold == 2 ? "cldW" : cold ? "cldR" : "warm", us,
                            (sh.loop == 2 ? bytes_of(sh.contig) - (double)n * 4 : bytes_of(sh.contig)) / us / 1e3 / 8000.0, 1e3 * tall[tall.size() / 2]);
            }
            if (dbg == 0) {  // every list equals the host partition in scan order (counts only: the counts)
                std::vector<uint32_t> got(off);
                CK(hipMemcpy(got.data(), d_out, off * 4, hipMemcpyDeviceToHost));
                std::vector<DGroupResult> res(nq);
                CK(hipMemcpy(res.data(), d_res, nq * sizeof(DGroupResult), hipMemcpyDeviceToHost));
                std::vector<uint64_t> at(dst);
                bool ok = true;
                for (uint32_t i = 0; i < n && ok && sh.loop != 2; i++) {
                    if (!alive[i]) continue;
                    const uint32_t q = (uint32_t)((mode[i] - 100) * nregion + (region[i] - 200));
                    ok = got[at[q]++] == i;
                }
                for (uint32_t q = 0; q < nq && ok; q++) ok = res[q].count == listlen[q];
                std::printf("  lists %s\n", ok ? "ok" : "WRONG");
                if (!ok) return 2;
            }
            CK(hipFree(d_work));
        }
    }
    return 0;
}

int main() {
    const size_t evict_n = (512ull << 20) / 16;
    uint4* evict;
    CK(hipMalloc(&evict, evict_n * 16));
    if (int r = run_shape(4u << 20, 8, 8, evict, evict_n)) return r;
    return run_shape(1u << 20, 2, 4, evict, evict_n);
}
