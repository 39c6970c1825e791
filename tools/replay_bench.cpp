// tools/replay_bench.cpp — times the host greedy replay (replay_core.h) alone
// and checks that its variants agree, on synthetic pools shaped like the
// bench configs: NPOOLS pools interleaved in slot order (as the store holds
// them), one session per presence, one complete constant-score hit list per
// pool = the pool's tickets in created order.
//
//   RB_MODE=c3     party sizes {1:60%,2:20%,3:10%,4:5%,5:5%}, Min=Max=10, CM=5 (default)
//   RB_MODE=solo2  solo tickets, Min=Max=2 (1v1)
//   RB_MODE=mixed  parties, Min 4..10 / Max 10, CM 1 or 2, Intervals 0..2
//                  (exercises the last-interval rule and the CountMultiple trim)
//
//   tools/replay_bench [tickets] [reps] [threads]
//     threads = 0: pool 0 only, single thread: generic replay_pool vs the
//                  dense walk (checksums must match; exit status 1 if not)
//     threads > 0: every pool, dense: gathers in chunks, then one walk per
//                  pool, on `threads` threads
//   RB_POOLS=n (default 8), RB_PROF=1 (SIGPROF sampler -> /tmp/rb_prof.txt; 2:
//   the identity walk only), RB_SHUFFLE=1 (c5: the buckets' tickets at random
//   slots, as a store filled in arrival order holds them),
//   RB_FAST=0 (threads > 0: exact walk only; sessions here are exclusive, so
//   the fast walks apply by default)
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <signal.h>
#include <string>
#include <sys/time.h>
#include <thread>
#include <ucontext.h>
#include <linux/perf_event.h>
#include <sys/ioctl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "../nakama_amd/csrc/replay_core.h"
#include "perf_group.h"

using namespace nkm;

struct NoDevice : ReplayCore {
    using ReplayCore::ReplayCore;
    void fetch_more(BGroup&) override { std::abort(); }
    bool pair_slow(const BGroup&, uint32_t, uint32_t) override { std::abort(); }
};

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

// RB_PERF=1: hardware counters around the identity walk (perf_group.h)

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static uint64_t checksum(const PoolOut& o) {
    uint64_t sum = 1469598103934665603ull;
    for (auto& e : o.ents) sum = (sum ^ (e.first * 131ull + (uint64_t)e.second)) * 1099511628211ull;
    for (auto& rc : o.recs)
        sum = (sum ^ (rc.bi * 7ull + rc.matched * 3ull + rc.expired + rc.len * 11ull + rc.off * 13ull + rc.gcum * 17ull +
                      rc.xcum * 19ull)) * 1099511628211ull;
    return sum;
}

// RB_MODE=c5: C5's packed RevPrecision batch — solo tickets in buckets of 8
// consecutive slots, Min 2 / Max 4, each row's list = its bucket's members
// with skill >= own - 100 ordered by (score desc, position), reverse bits and
// 8-bit pair words as rpack_kernel writes them; every bucket replayed by
// replay_pool through a per-row view (as Core::process_default's packed path).
static int bench_c5(uint32_t N, int reps) {
    constexpr int S = 8;
    uint64_t rng = 0x5EED0005ull;
    std::vector<HotRec> hot(N);
    std::vector<uint32_t> party(N, kNoParty), pres_sess(N);
    std::vector<int32_t> intervals(N, 0), count(N, 1), minc(N, 2), maxc(N, 4);
    std::vector<uint8_t> live(N, 1);
    std::vector<int64_t> created(N);
    std::vector<int> skill(N);
    for (uint32_t i = 0; i < N; i++) {
        const double u1 = ((splitmix(rng) >> 11) + 1) * 0x1.0p-53, u2 = (splitmix(rng) >> 11) * 0x1.0p-53;
        skill[i] = (int)std::lround(1500.0 + 300.0 * std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2));
        pres_sess[i] = i;
        HotRec& h = hot[i];
        h = HotRec{kNoParty, i, i, 1, 2, 4, 1, 1u << (i & 31)};
        created[i] = 1700000000000000000ll + 1024ll * i;
    }
    // packed lists (C5's query "+bucket:b skill:>=s-100^2": the bucket is
    // required, the skill clause only scores): every member of the row's
    // bucket is a hit, those with skill >= own - 100 first (higher score),
    // then the rest, each part in bucket order; every reverse check and pair
    // check holds (every query accepts its whole bucket)
    std::vector<uint32_t> slots((size_t)N * S), brow(N);
    std::vector<uint8_t> cnt(N), revb(N), pm((size_t)N * S);
    for (uint32_t i = 0; i < N; i++) {
        brow[i] = i;
        const uint32_t b0 = i / S * S;
        uint32_t n = 0;
        for (int part = 0; part < 2; part++)
            for (uint32_t j = b0; j < b0 + S && j < N; j++)
                if ((skill[j] >= skill[i] - 100) == (part == 0)) slots[(size_t)i * S + n++] = j;
        cnt[i] = (uint8_t)n;
        revb[i] = (uint8_t)((1u << n) - 1);
        for (uint32_t a = 0; a < n; a++) pm[(size_t)i * S + a] = (uint8_t)((1u << n) - 1);
    }
    if (std::getenv("RB_SHUFFLE")) {
        // the buckets' tickets at random slots (as a store filled in arrival
        // order holds them); rows stay in bucket order
        std::vector<uint32_t> pi(N);
        for (uint32_t i = 0; i < N; i++) pi[i] = i;
        for (uint32_t i = N - 1; i > 0; i--) std::swap(pi[i], pi[splitmix(rng) % (i + 1)]);
        auto perm = [&](auto& a) {
            auto b = a;
            for (uint32_t i = 0; i < N; i++) b[pi[i]] = a[i];
            a.swap(b);
        };
        perm(hot); perm(party); perm(intervals); perm(count); perm(minc); perm(maxc); perm(live); perm(created);
        for (uint32_t i = 0; i < N; i++) brow[i] = pi[i];
        for (auto& x : slots) x = pi[x];
    }
    ReplayView v{hot.data(), pres_sess.data(), party.data(), intervals.data(), live.data(), count.data(), created.data(),
                 true};
    std::vector<uint8_t> psel(N, 0), proc(N, 0);
    double best = 1e30;
    uint64_t sum = 0;
    size_t groups = 0;
    const bool prof = std::getenv("RB_PROF") != nullptr;
    if (prof) {
        struct sigaction sa {};
        sa.sa_sigaction = on_prof;
        sa.sa_flags = SA_SIGINFO | SA_RESTART;
        sigaction(SIGPROF, &sa, nullptr);
        itimerval it{{0, 200}, {0, 200}};
        setitimer(ITIMER_PROF, &it, nullptr);
    }
    const bool fast = !std::getenv("RB_FAST") || std::atoi(std::getenv("RB_FAST")) != 0;
    for (int r = 0; r < reps; r++) {
        NoDevice rp(v, psel, true, 2);
        rp.fast = fast;
        BGroup g;
        auto view = [&](uint32_t bi) -> BGroup& {
            g.set_slots(slots.data() + (size_t)bi * S);
            g.rev_packed = true;
            g.rev_bits = revb[bi];
            g.pm = pm.data() + (size_t)bi * S;
            g.pm_w = 1;
            g.n = cnt[bi];
            g.pm_n = cnt[bi];
            g.complete = true;
            g.head = 0;
            return g;
        };
        PoolOut o;
        std::vector<uint32_t> bis;
        groups = 0;
        const double t0 = now_ms();
        for (uint32_t b0 = 0; b0 < N; b0 += S) {
            bis.clear();
            for (uint32_t j = b0; j < b0 + S && j < N; j++) bis.push_back(j);
            o.recs.clear();
            o.ents.clear();
            replay_pool(rp, bis, brow.data(), view, psel, proc.data(), minc.data(), maxc.data(), o);
            if (r == 0) sum ^= checksum(o);  // rep 0 checks; the later reps time the replay alone
            groups += o.recs.back().gcum;
        }
        if (r > 0 || reps == 1) best = std::min(best, now_ms() - t0);
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
    std::printf("[c5] %u rows in buckets of %d: %zu groups | replay %.3f ms single thread (%.1f ns/row) | checksum %016llx\n",
                N, S, groups, best, best * 1e6 / N, (unsigned long long)sum);
    return 0;
}

int main(int argc, char** argv) {
    const uint32_t N = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1000000;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const int nthreads = argc > 3 ? std::atoi(argv[3]) : 0;
    const int npools = std::getenv("RB_POOLS") ? std::atoi(std::getenv("RB_POOLS")) : 8;
    const std::string mode = std::getenv("RB_MODE") ? std::getenv("RB_MODE") : "c3";
    if (mode == "c5") return bench_c5(N, reps);
    const int maxI = 2;
    uint64_t rng = 0x5EED0003ull;
    std::vector<HotRec> hot(N);
    std::vector<uint32_t> party(N), pres_sess;
    std::vector<int32_t> intervals(N, 0), count(N), minc(N), maxc(N);
    std::vector<uint8_t> live(N, 1);
    std::vector<int64_t> created(N);
    std::vector<uint32_t> pool(N);
    uint32_t next_party = 0, next_sess = 0;
    for (uint32_t i = 0; i < N; i++) {
        const double u = (splitmix(rng) >> 11) * 0x1.0p-53;
        int ps = u < 0.60 ? 1 : u < 0.80 ? 2 : u < 0.90 ? 3 : u < 0.95 ? 4 : 5;
        int mn = 10, mx = 10, cm = 5;
        if (mode == "solo2") ps = 1, mn = mx = 2, cm = 1;
        if (mode == "mixed") {
            mn = 4 + (int)(splitmix(rng) % 7);
            mx = 10;
            cm = splitmix(rng) % 3 == 0 ? 2 : 1;
            intervals[i] = (int)(splitmix(rng) % 3);
        }
        pool[i] = (uint32_t)(splitmix(rng) % npools);
        party[i] = ps > 1 ? next_party++ : kNoParty;
        HotRec& h = hot[i];
        h.party = party[i];
        h.pres_off = (uint32_t)pres_sess.size();
        for (int p = 0; p < ps; p++) pres_sess.push_back(next_sess++);
        h.sess0 = pres_sess[h.pres_off];
        h.count = count[i] = ps;
        h.minc = minc[i] = mn;
        h.maxc = maxc[i] = mx;
        h.cm = cm;
        h.smask = 0;
        for (int p = 0; p < ps; p++) h.smask |= 1u << (pres_sess[h.pres_off + p] & 31);
        created[i] = 1700000000000000000ll + 1024ll * i;
    }
    std::vector<std::vector<DHit>> ph(npools);
    std::vector<std::vector<uint32_t>> pbis(npools);
    std::vector<uint32_t> brow(N);  // batch row i = slot i
    for (uint32_t i = 0; i < N; i++) {
        brow[i] = i;
        ph[pool[i]].push_back(DHit{i, (uint32_t)ph[pool[i]].size(), 0});
        pbis[pool[i]].push_back(i);
    }
    ReplayView v{hot.data(), pres_sess.data(), party.data(), intervals.data(), live.data(), count.data(), created.data(),
                 true};  // one session per presence: sessions are exclusive
    const bool fast = !std::getenv("RB_FAST") || std::atoi(std::getenv("RB_FAST")) != 0;
    std::vector<uint32_t> pos_of(N, kNoSlot);

    if (nthreads == 0) {
        // pool 0: the generic and dense walks, each exact (row()/step()) and
        // fast (exclusive sessions): all four must give the same output
        std::vector<uint8_t> psel(N, 0), proc(N, 0);
        PoolOut out[5];
        const char* name[5] = {"generic", "generic-fast", "dense", "dense-fast", "identity-walk-only"};
        double best[5] = {1e30, 1e30, 1e30, 1e30, 1e30};
        DensePool P;
        DenseRun run;
        BGroup g;
        g.set_hits(ph[0].data());
        g.n = (uint32_t)ph[0].size();
        const bool prof = std::getenv("RB_PROF") != nullptr;
        const bool prof_walk = prof && std::atoi(std::getenv("RB_PROF")) == 2;  // the identity walk only
        if (prof) {
            struct sigaction sa {};
            sa.sa_sigaction = on_prof;
            sa.sa_flags = SA_SIGINFO | SA_RESTART;
            sigaction(SIGPROF, &sa, nullptr);
            if (!prof_walk) {
                itimerval it{{0, 200}, {0, 200}};
                setitimer(ITIMER_PROF, &it, nullptr);
            }
        }
        for (int r = 0; r < reps; r++) {
            for (int k = 0; k < 2; k++) {
                out[k].recs.clear();
                out[k].ents.clear();
                g.head = 0;
                NoDevice rp(v, psel, false, maxI);
                rp.fast = k == 1;
                const double t0 = now_ms();
                replay_pool(rp, pbis[0], brow.data(), [&](uint32_t) -> BGroup& { return g; }, psel, proc.data(),
                            minc.data(), maxc.data(), out[k]);
                best[k] = std::min(best[k], now_ms() - t0);
            }
            for (int k = 2; k < 4; k++) {
                const double t0 = now_ms();
                P.reset(g, pbis[0].data(), (uint32_t)pbis[0].size(), brow.data());
                P.gather(v, 0, P.n, pos_of.data());
                run.fast = k == 3;
                run.reset(P.n);
                run.walk(P, v, maxI, pos_of.data(), 0, P.nrows);
                run.finish(out[k]);
                P.clear_pos(0, P.n, pos_of.data());
                best[k] = std::min(best[k], now_ms() - t0);
            }
            {  // the product's identity pools: the walk alone (gathered untimed)
                P.reset(g, pbis[0].data(), (uint32_t)pbis[0].size(), brow.data());
                P.identity = true;
                P.gather(v, 0, P.n, pos_of.data());
                run.fast = true;
                run.reset(P.n);
                if (prof_walk) {
                    itimerval it{{0, 100}, {0, 100}};
                    setitimer(ITIMER_PROF, &it, nullptr);
                }
                static PerfGroup pg;
                const bool perf = std::getenv("RB_PERF") != nullptr && pg.ok();
                if (perf) pg.start();
                const double t0 = now_ms();
#ifdef NKM_WALK_STATS
                std::memset(g_walk_stats, 0, sizeof g_walk_stats);
#endif
                run.walk(P, v, maxI, pos_of.data(), 0, P.nrows);
                best[4] = std::min(best[4], now_ms() - t0);
#ifdef NKM_WALK_STATS
                if (r == 0) {
                    const double rows = (double)run.recs.size();
                    std::printf("[stats] per processed row: head steps %.2f, first-fit steps %.2f, hits placed %.2f, "
                                "member checks %.2f, skip loops %.2f, hits seen %.2f, entries %.2f\n",
                                g_walk_stats[0] / rows, g_walk_stats[1] / rows, g_walk_stats[2] / rows,
                                g_walk_stats[3] / rows, g_walk_stats[4] / rows, run.hits_seen / rows,
                                run.ents.size() / rows);
                }
#endif
                if (perf) {
                    pg.stop();
                    if (r + 1 == reps) {
                        const double steps = (double)run.recs.size();
                        std::printf("[perf] identity walk, %d reps: per processed row %.0f cycles, %.0f instructions "
                                    "(IPC %.2f), %.2f branch misses, %.2f L1D read misses; hits examined %.2f per row\n",
                                    reps, pg.v[0] / steps / reps, pg.v[1] / steps / reps, (double)pg.v[1] / (double)pg.v[0],
                                    pg.v[2] / steps / reps, pg.v[3] / steps / reps, run.hits_seen / steps);
                    }
                } else if (std::getenv("RB_PERF") && r == 0) {
                    std::printf("[perf] no PMU here\n");
                }
                if (prof_walk) {
                    itimerval off{};
                    setitimer(ITIMER_PROF, &off, nullptr);
                }
                run.finish(out[4]);
            }
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
        bool same = true;
        const uint64_t c0 = checksum(out[0]);
        for (int k = 1; k < 5; k++) same &= checksum(out[k]) == c0;
        std::printf("[%s] pool of %u tickets: %zu rows, %u groups |", mode.c_str(), g.n, out[0].recs.size() - 1,
                    out[0].recs.back().gcum);
        for (int k = 0; k < 5; k++) std::printf(" %s %.3f ms", name[k], best[k]);
        std::printf(" | checksum %016llx %s\n", (unsigned long long)c0, same ? "MATCH" : "MISMATCH");
        return same ? 0 : 1;
    }

    // every pool, dense: gathers in chunks, then one walk per pool, on `nthreads` threads
    std::vector<DensePool> P(npools);
    std::vector<DenseRun> runs(npools);
    std::vector<PoolOut> outs(npools);
    std::vector<BGroup> gs(npools);
    for (int p = 0; p < npools; p++) {
        gs[p].set_hits(ph[p].data());
        gs[p].n = (uint32_t)ph[p].size();
    }
    auto par = [&](size_t n, const std::function<void(size_t)>& f) {
        std::atomic<size_t> next{0};
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; t++)
            th.emplace_back([&] {
                for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
            });
        for (auto& t : th) t.join();
    };
    constexpr uint32_t kChunk = 16384;
    // RB_IDENT=1: identity pools (the product's C3 / C4 walks: row j is list
    // position j); RB_SELFGATHER=1: each walk gathers its own pool first (in its
    // timed task) instead of the chunked gather across the threads
    const bool ident = std::getenv("RB_IDENT") && std::atoi(std::getenv("RB_IDENT")) != 0;
    const bool selfg = std::getenv("RB_SELFGATHER") && std::atoi(std::getenv("RB_SELFGATHER")) != 0;
    for (int r = 0; r < reps; r++) {
        const double t0 = now_ms();
        std::vector<std::pair<int, uint32_t>> chunks;
        bool all_ident = ident;
        for (int p = 0; p < npools; p++) {
            P[p].reset(gs[p], pbis[p].data(), (uint32_t)pbis[p].size(), brow.data());
            all_ident = all_ident && P[p].nrows == P[p].n && P[p].rows_are_list(0, P[p].n);
            for (uint32_t c = 0; c * kChunk < P[p].n && !selfg; c++) chunks.push_back({p, c});
        }
        for (int p = 0; p < npools; p++) P[p].identity = all_ident;
        if (r == 0 && ident && !all_ident) std::printf("RB_IDENT: the pools' rows are not their lists\n");
        par(chunks.size(), [&](size_t t) {
            DensePool& q = P[chunks[t].first];
            const uint32_t lo = chunks[t].second * kChunk;
            q.gather(v, lo, std::min(q.n, lo + kChunk), pos_of.data());
        });
        const double t1 = now_ms();
        std::vector<double> task(npools);
        par(npools, [&](size_t p) {
            const double a = now_ms();
            if (selfg) P[p].gather(v, 0, P[p].n, pos_of.data());
            runs[p].reset(P[p].n);
            runs[p].fast = fast;
            runs[p].walk(P[p], v, maxI, pos_of.data(), 0, P[p].nrows);
            runs[p].finish(outs[p]);
            task[p] = now_ms() - a;
        });
        const double t2 = now_ms();
        par(npools, [&](size_t p) { P[p].clear_pos(0, P[p].n, pos_of.data()); });
        uint64_t sum = 0;
        for (auto& o : outs) sum ^= checksum(o);
        double mx = 0, mean = 0;
        for (double x : task) mx = std::max(mx, x), mean += x / npools;
        std::printf("[%s] %d pools on %d threads: wall %.3f ms (gather %.3f, walks %.3f: task max %.3f mean %.3f) | "
                    "xor-checksum %016llx\n",
                    mode.c_str(), npools, nthreads, now_ms() - t0, t1 - t0, t2 - t1, mx, mean, (unsigned long long)sum);
    }
    return 0;
}
