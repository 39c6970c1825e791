// tools/rsrc_bench.hip — the library's range-batch sort (rsrc_tile_kernel +
// rsrc_merge_kernel launches + rsrc_bounds_kernel, launch_rsrc) in isolation
// on C2's shape: 4 pools
// of 25,000 candidates whose numeric values repeat (integer skills ~ N(1500,
// 300)), 54k bound queries.  Times every launch by its event pair (warm, back
// to back, as in the pass: the store was just uploaded) and checks the sorted
// positions and the bounds against a host sort.  argv[1]: pools (default 4),
// argv[2]: candidates per pool (25000), argv[3]: bound queries (54000).
#include "../nakama_amd/csrc/mm_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
    using namespace nkm;
    const uint32_t np = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 4;
    const uint32_t per = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 25000;
    const uint32_t nq = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 54000;
    const uint32_t n = np * per;
    std::mt19937_64 rng(7);
    std::normal_distribution<double> skill(1500.0, 300.0);
    std::vector<uint32_t> post(n);
    std::vector<uint8_t> alive(n, 1), kind(n, KIND_NUMERIC);
    std::vector<int64_t> val(n);
    for (uint32_t i = 0; i < n; i++) {
        post[i] = i;
        val[i] = (int64_t)std::lround(skill(rng)) << 20;
        if (rng() % 50 == 0) alive[i] = 0;
    }
    auto up = [](const void* h, size_t bytes) {
        void* d = nullptr;
        (void)hipMalloc(&d, bytes);
        (void)hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
        return d;
    };
    DStore st{};
    st.alive = (const uint8_t*)up(alive.data(), n);
    st.postings = (const uint32_t*)up(post.data(), 4 * (size_t)n);
    const int64_t* fv[1] = {(const int64_t*)up(val.data(), 8 * (size_t)n)};
    const uint8_t* fk[1] = {(const uint8_t*)up(kind.data(), n)};
    st.fval = (const int64_t* const*)up(fv, sizeof fv);
    st.fkind = (const uint8_t* const*)up(fk, sizeof fk);
    std::vector<DRangePool> pools(np);
    std::vector<DRangeTile> tiles;
    std::vector<uint32_t> blk;
    uint32_t n_elems = 0, max_pad = 0;
    for (uint32_t p = 0; p < np; p++) {
        DRangePool& d = pools[p];
        d = DRangePool{};
        d.src_off = p * per;
        d.src_len = per;
        d.out_off = n_elems;
        d.pad_len = (per + 255) & ~255u;
        d.field = 0;
        n_elems += d.pad_len;
        max_pad = std::max(max_pad, d.pad_len);
        for (uint32_t s0 = 0; s0 < d.pad_len; s0 += kRsrcTile)
            tiles.push_back(DRangeTile{p, s0, std::min(kRsrcTile, d.pad_len - s0), 0});
        for (uint32_t b = 0; b < d.pad_len / 256; b++) blk.push_back(p);
    }
    std::vector<DRangeBound> q(nq);
    for (uint32_t t = 0; t < nq; t++) {
        q[t].pool = (uint32_t)(rng() % np);
        q[t].key = (int64_t)std::lround(skill(rng) + ((t & 1) ? 200 : -200)) << 20;
        q[t].upper = t & 1;
    }
    DRangePool* d_pools = (DRangePool*)up(pools.data(), pools.size() * sizeof(DRangePool));
    DRangeTile* d_tiles = (DRangeTile*)up(tiles.data(), tiles.size() * sizeof(DRangeTile));
    uint32_t* d_blk = (uint32_t*)up(blk.data(), blk.size() * 4);
    DRangeBound* d_q = (DRangeBound*)up(q.data(), q.size() * sizeof(DRangeBound));
    int64_t* dk[2];
    uint32_t* dp[2];
    for (int b = 0; b < 2; b++) {
        CK(hipMalloc(&dk[b], 8 * (size_t)n_elems));
        CK(hipMalloc(&dp[b], 4 * (size_t)n_elems));
    }
    uint32_t* d_bounds;
    CK(hipMalloc(&d_bounds, 4 * (size_t)nq));

    hipStream_t s;
    CK(hipStreamCreate(&s));
    constexpr int kMax = 20;
    hipEvent_t ev[2 + 2 * kMax];
    for (auto& evx : ev) CK(hipEventCreate(&evx));
    std::vector<double> t_tile, t_rank[kMax], t_all, t_bound;
    int which = 0, nm = 0;
    for (int rep = 0; rep < 25; rep++) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a, s));
        CK(launch_rsrc(st, d_pools, max_pad, d_tiles, (uint32_t)tiles.size(), d_blk, n_elems, dk, dp, d_q, nq, d_bounds,
                       &which, s, ev[0], ev[1], ev + 2, kMax, &nm));
        CK(hipEventRecord(b, s));
        CK(hipStreamSynchronize(s));
        float ms;
        if (rep < 5) continue;
        CK(hipEventElapsedTime(&ms, ev[0], ev[1]));
        t_tile.push_back(ms * 1e3);
        for (int m = 0; m < nm; m++) {
            CK(hipEventElapsedTime(&ms, ev[2 + 2 * m], ev[3 + 2 * m]));
            t_rank[m].push_back(ms * 1e3);
        }
        CK(hipEventElapsedTime(&ms, a, b));
        t_all.push_back(ms * 1e3);
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? 0.0 : v[v.size() / 2]; };
    std::printf("rsrc: %u pools x %u, %u elements, %zu tiles, %d merge launches, %u bounds\n", np, per, n_elems,
                tiles.size(), nm, nq);
    std::printf("  tile %.2f us", med(t_tile));
    for (int m = 0; m < nm; m++) std::printf(" | merge%d %.2f us", m, med(t_rank[m]));
    std::printf(" | all (events around the launches, bounds included) %.2f us\n", med(t_all));
    // check
    std::vector<uint32_t> got(n_elems), gb(nq);
    CK(hipMemcpy(got.data(), dp[which], 4 * (size_t)n_elems, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gb.data(), d_bounds, 4 * (size_t)nq, hipMemcpyDeviceToHost));
    int bad = 0;
    std::vector<std::vector<int64_t>> sorted_keys(np);
    for (uint32_t p = 0; p < np; p++) {
        const DRangePool& d = pools[p];
        std::vector<std::pair<int64_t, uint32_t>> e;
        for (uint32_t i = 0; i < d.pad_len; i++) {
            if (i < d.src_len && alive[d.src_off + i]) e.push_back({val[d.src_off + i], i});
            else e.push_back({INT64_MAX, kRsrcInvalid | i});
        }
        std::sort(e.begin(), e.end());
        for (uint32_t i = 0; i < d.pad_len; i++) {
            const uint32_t gv = got[d.out_off + i];
            if (gv != e[i].second && !(gv & kRsrcInvalid && e[i].second & kRsrcInvalid)) {
                if (bad++ < 5) std::printf("  pool %u element %u: got %x want %x\n", p, i, gv, e[i].second);
            }
            sorted_keys[p].push_back(e[i].first);
        }
    }
    for (uint32_t t = 0; t < nq; t++) {
        const auto& k = sorted_keys[q[t].pool];
        const uint32_t want = (uint32_t)((q[t].upper ? std::upper_bound(k.begin(), k.end(), q[t].key)
                                                     : std::lower_bound(k.begin(), k.end(), q[t].key)) - k.begin());
        if (gb[t] != want && bad++ < 10) std::printf("  bound %u: got %u want %u\n", t, gb[t], want);
    }
    std::printf("  check: %s\n", bad ? "FAILED" : "ok");
    return bad ? 1 : 0;
}
