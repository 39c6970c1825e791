// tools/replay_bench.cpp — times the host greedy replay (replay_core.h) alone,
// on a C3-shaped pool: one pool's tickets interleaved with 7 others in slot
// order (as the store holds them), party sizes {1:60%,2:20%,3:10%,4:5%,5:5%},
// one session per presence, Min=Max=10, CountMultiple=5, a complete
// constant-score hit list = the pool's tickets in created order.  Prints the
// time per replay of the pool and a checksum of the groups so that variants
// of the replay can be compared for speed and identical output.
//
//   make -C tools replay_bench && tools/replay_bench [tickets] [reps] [threads]   (RB_POOLS=n pools, RB_DENSE=1)
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <thread>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include "../nakama_amd/csrc/replay_core.h"

using namespace nkm;

struct NoDevice : ReplayCore {
    using ReplayCore::ReplayCore;
    void fetch_more(BGroup&) override { std::abort(); }
    bool pair_slow(const BGroup&, uint32_t, uint32_t) override { std::abort(); }
};

// RB_PROF=1: a SIGPROF sampler of the instruction pointer (no profiler in the
// image); addresses go to llvm-symbolizer.
static uint64_t g_samples[1 << 16];
static volatile size_t g_ns = 0;
static void on_prof(int, siginfo_t*, void* ctx) {
    if (g_ns < (1u << 16)) g_samples[g_ns++] = (uint64_t)((ucontext_t*)ctx)->uc_mcontext.gregs[REG_RIP];
}

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const uint32_t N = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1000000;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const int nthreads = argc > 3 ? std::atoi(argv[3]) : 0;  // >0: replay every pool, one thread per pool
    const bool dense = std::getenv("RB_DENSE") && *std::getenv("RB_DENSE");   // DenseReplay instead of replay_pool
    const int npools = std::getenv("RB_POOLS") ? std::atoi(std::getenv("RB_POOLS")) : 8;
    uint64_t rng = 0x5EED0003ull;
    std::vector<HotRec> hot(N);
    std::vector<uint32_t> party(N), pres_sess;
    std::vector<int32_t> intervals(N, 0), count(N), minc(N, 10), maxc(N, 10);
    std::vector<uint8_t> live(N, 1);
    std::vector<int64_t> created(N);
    std::vector<uint32_t> pool(N);
    uint32_t next_party = 0, next_sess = 0;
    for (uint32_t i = 0; i < N; i++) {
        const double u = (splitmix(rng) >> 11) * 0x1.0p-53;
        const int ps = u < 0.60 ? 1 : u < 0.80 ? 2 : u < 0.90 ? 3 : u < 0.95 ? 4 : 5;
        pool[i] = (uint32_t)(splitmix(rng) % npools);
        party[i] = ps > 1 ? next_party++ : kNoParty;
        HotRec& h = hot[i];
        h.party = party[i];
        h.pres_off = (uint32_t)pres_sess.size();
        for (int p = 0; p < ps; p++) pres_sess.push_back(next_sess++);
        h.sess0 = pres_sess[h.pres_off];
        h.count = count[i] = ps;
        h.minc = 10;
        h.maxc = 10;
        h.cm = 5;
        h.smask = 0;
        for (int p = 0; p < ps; p++) h.smask |= 1u << (pres_sess[h.pres_off + p] & 31);
        created[i] = 1700000000000000000ll + 1024ll * i;
    }
    // pool 0's hit list and rows
    std::vector<DHit> hits;
    std::vector<uint32_t> brow, bis;
    for (uint32_t i = 0; i < N; i++)
        if (pool[i] == 0) {
            hits.push_back(DHit{i, (uint32_t)hits.size(), 0});
            bis.push_back((uint32_t)brow.size());
            brow.push_back(i);
        }
    ReplayView v{hot.data(), pres_sess.data(), party.data(), intervals.data(), live.data(), count.data(), created.data()};
    if (nthreads > 0) {
        // every pool at once, `nthreads` threads taking pools from a counter
        std::vector<std::vector<DHit>> ph(npools);
        std::vector<std::vector<uint32_t>> pbrow(npools), pbis(npools);
        for (uint32_t i = 0; i < N; i++) {
            const uint32_t p = pool[i];
            ph[p].push_back(DHit{i, (uint32_t)ph[p].size(), 0});
            pbis[p].push_back((uint32_t)pbrow[p].size());
            pbrow[p].push_back(i);
        }
        for (int r = 0; r < reps; r++) {
            std::atomic<int> next{0};
            std::vector<double> task(npools);
            const auto t0 = std::chrono::steady_clock::now();
            std::vector<std::thread> th;
            for (int t = 0; t < nthreads; t++)
                th.emplace_back([&] {
                    std::vector<uint8_t> ps(N, 0), pr(N, 0);
                    std::vector<uint32_t> pos_of(N, kNoSlot);
                    DenseReplay dr;
                    PoolOut po;
                    for (int p; (p = next.fetch_add(1)) < npools;) {
                        const auto a = std::chrono::steady_clock::now();
                        BGroup g;
                        g.hits = ph[p].data();
                        g.n = (uint32_t)ph[p].size();
                        NoDevice rp(v, ps, false, 2);
                        po.recs.clear();
                        po.ents.clear();
                        if (dense) dr.run(v, 2, g, pbis[p], pbrow[p].data(), pos_of, po);
                        else replay_pool(rp, pbis[p], pbrow[p].data(), [&](uint32_t) -> BGroup& { return g; }, ps,
                                         pr.data(), minc.data(), maxc.data(), po);
                        task[p] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
                    }
                });
            for (auto& t : th) t.join();
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            double mx = 0, sm = 0;
            for (double x : task) mx = std::max(mx, x), sm += x;
            std::printf("%d pools on %d threads: wall %.3f ms | task max %.3f mean %.3f ms\n", npools, nthreads, ms, mx,
                        sm / npools);
        }
        return 0;
    }
    std::vector<uint8_t> psel(N, 0), proc(N, 0);
    PoolOut o;  // reused across reps, as the library keeps its pool outputs
    std::vector<uint32_t> pos_of(N, kNoSlot);
    DenseReplay dr;
    const bool prof = std::getenv("RB_PROF") != nullptr;
    if (prof) {
        struct sigaction sa {};
        sa.sa_sigaction = on_prof;
        sa.sa_flags = SA_SIGINFO | SA_RESTART;
        sigaction(SIGPROF, &sa, nullptr);
        itimerval it{{0, 200}, {0, 200}};
        setitimer(ITIMER_PROF, &it, nullptr);
    }
    double best = 1e30, total = 0;
    uint64_t sum = 0;
    size_t groups = 0, rows = 0, hits_seen = 0;
    for (int r = 0; r < reps; r++) {
        BGroup g;
        g.hits = hits.data();
        g.n = (uint32_t)hits.size();
        g.complete = true;
        NoDevice rp(v, psel, false, 2);
        o.recs.clear();
        o.ents.clear();
        const auto t0 = std::chrono::steady_clock::now();
        if (dense) dr.run(v, 2, g, bis, brow.data(), pos_of, o);
        else replay_pool(rp, bis, brow.data(), [&](uint32_t) -> BGroup& { return g; }, psel, proc.data(), minc.data(),
                         maxc.data(), o);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        best = std::min(best, ms);
        total += ms;
        sum = 1469598103934665603ull;
        for (auto& e : o.ents) sum = (sum ^ (e.first * 131ull + (uint64_t)e.second)) * 1099511628211ull;
        for (auto& rc : o.recs) sum = (sum ^ (rc.bi * 7ull + rc.matched)) * 1099511628211ull;
        groups = o.recs.back().gcum;
        rows = o.recs.size() - 1;
        hits_seen = dense ? dr.hits_seen / (r + 1) : rp.hits_seen;
    }
    if (prof) {
        itimerval off{};
        setitimer(ITIMER_PROF, &off, nullptr);
        std::map<uint64_t, size_t> h;
        for (size_t i = 0; i < g_ns; i++) h[g_samples[i]]++;
        FILE* f = std::fopen("/tmp/rb_prof.txt", "w");
        for (auto& kv : h) std::fprintf(f, "%zu 0x%llx\n", kv.second, (unsigned long long)kv.first);
        std::fclose(f);
    }
    std::printf("pool of %zu tickets: %zu rows, %zu groups, %zu hits walked | best %.3f ms, mean %.3f ms "
                "(%.1f ns/row) | checksum %016llx\n",
                hits.size(), rows, groups, hits_seen, best, total / reps, best * 1e6 / rows, (unsigned long long)sum);
    return 0;
}
