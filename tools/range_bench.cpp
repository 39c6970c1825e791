// tools/range_bench.cpp — checks the range walk (range_walk.h: min tree over a
// pool's value-sorted candidates, tier lists from build_tiers) against the
// list replay (replay_core.h: replay_pool over each row's full hit list in the
// reference's order), and times the walk.  One pool of N tickets in created
// order (slot = hit rank = row), each searching a C2-shaped skill window:
//   +term  +skill:>=s-200  +skill:<=s+200  skill:>=s-50^2  skill:<=s+50^2
// (mixed mode adds a MUST_NOT range and a ^0.5 range, parties of 1-3, shared
// sessions, Min/Max/CountMultiple shapes and Intervals, and tickets without a
// number in the field).  The hit lists apply the device search's filters (the
// searching ticket's party, MinCount >= Min, MaxCount <= Max).
//
//   tools/range_bench [tickets] [mode: solo|mixed|mixedx] [seed] [noref|ref] [exact: no fast body]
// prints the records' checksum for both and the walk time; exit status 1 when
// they differ.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../nakama_amd/csrc/range_walk.h"
#include "../nakama_amd/csrc/replay_core.h"
#include "perf_group.h"

using namespace nkm;

struct NoDevice : ReplayCore {
    using ReplayCore::ReplayCore;
    void fetch_more(BGroup&) override { std::abort(); }
    bool pair_slow(const BGroup&, uint32_t, uint32_t) override { std::abort(); }
};

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static double uni(uint64_t& s) { return (double)(splitmix(s) >> 11) * (1.0 / 9007199254740992.0); }

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const uint32_t N = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 5000;
    // mixed: shared sessions too (the exact row body); mixedx: exclusive
    // sessions (the fast body, bailing to the exact one at the CountMultiple trim)
    const bool mixed = argc > 2 && (std::string(argv[2]) == "mixed" || std::string(argv[2]) == "mixedx");
    const bool share = argc > 2 && std::string(argv[2]) == "mixed";
    uint64_t seed = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 1;
    const int maxI = 3;
    // ---- tickets ----
    std::vector<HotRec> hot(N);
    std::vector<uint32_t> pres_sess, party(N, kNoParty);
    std::vector<int32_t> intervals(N, 0), count(N), minc(N), maxc(N);
    std::vector<uint8_t> live(N, 1), numeric(N, 1);
    std::vector<int64_t> created(N), val(N, 0);
    std::vector<int> skill(N);
    bool shared = false;
    for (uint32_t i = 0; i < N; i++) {
        const double u1 = std::max(uni(seed), 1e-12), u2 = uni(seed);
        skill[i] = (int)std::lround(1500.0 + 300.0 * std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2));
        val[i] = sortable_i64((double)skill[i]);
        created[i] = 1000 + (int64_t)i;
        int c = 1, mn = 2, mx = 2, cm = 1;
        if (mixed) {
            const double u = uni(seed);
            c = u < 0.7 ? 1 : u < 0.9 ? 2 : 3;
            const int shape = (int)(splitmix(seed) % 3);
            if (shape == 1) { mn = 2; mx = 4; }
            if (shape == 2) { mn = 4; mx = 6; cm = 2; }
            intervals[i] = (int)(splitmix(seed) % 3);
            numeric[i] = uni(seed) < 0.95;
            if (c > 1) party[i] = i;
        }
        HotRec& h = hot[i];
        h.party = party[i];
        h.pres_off = (uint32_t)pres_sess.size();
        h.count = c;
        h.minc = mn;
        h.maxc = mx;
        h.cm = cm;
        h.smask = 0;
        for (int p = 0; p < c; p++) {
            uint32_t s = i * 4 + (uint32_t)p;
            if (share && i > 0 && uni(seed) < 0.03) {  // an earlier ticket's session
                const uint32_t j = (uint32_t)(splitmix(seed) % i);
                s = pres_sess[hot[j].pres_off];
                shared = true;
            }
            pres_sess.push_back(s);
            h.smask |= 1u << (s & 31);
        }
        h.sess0 = pres_sess[h.pres_off];
        count[i] = c;
        minc[i] = mn;
        maxc[i] = mx;
    }
    ReplayView v{hot.data(), pres_sess.data(), party.data(), intervals.data(), live.data(), count.data(), created.data(),
                 !shared};
    // ---- queries (clause order as the compiler emits it) ----
    auto clauses_of = [&](uint32_t i, std::vector<DClause>& cl) {
        const double s = skill[i];
        cl.clear();
        cl.push_back(DClause{0, 0, 1.0, 7, 0, OP_TERM, OCC_MUST});
        cl.push_back(DClause{sortable_i64(s - 200), INT64_MAX, 1.0, 0, 1, OP_RANGE, OCC_MUST});
        cl.push_back(DClause{INT64_MIN, sortable_i64(s + 200), 1.0, 0, 1, OP_RANGE, OCC_MUST});
        cl.push_back(DClause{sortable_i64(s - 50), INT64_MAX, 2.0, 0, 1, OP_RANGE, OCC_SHOULD});
        cl.push_back(DClause{INT64_MIN, sortable_i64(s + 50), 2.0, 0, 1, OP_RANGE, OCC_SHOULD});
        if (mixed && (i % 3) == 0) {
            cl.push_back(DClause{sortable_i64(s + 150), sortable_i64(s + 170), 1.0, 0, 1, OP_RANGE, OCC_MUSTNOT});
            cl.push_back(DClause{sortable_i64(s - 120), sortable_i64(s - 20), 0.5, 0, 1, OP_RANGE, OCC_SHOULD});
        }
    };
    auto score = [&](const std::vector<DClause>& cl, uint32_t j, int64_t* key) {  // eval_parsed on the host
        double ms = 0, ss = 0;
        bool any = false, fail = false;
        for (const DClause& c : cl) {
            const bool h = c.op == OP_TERM ? true : (numeric[j] && val[j] >= c.lo && val[j] <= c.hi);
            if (c.occur == OCC_MUST) { if (h) ms += c.score; else fail = true; }
            else if (c.occur == OCC_SHOULD) { if (h) { ss += c.score; any = true; } }
            else if (h) fail = true;
        }
        if (fail) return false;
        *key = sortable_i64(((any ? ms + ss : ms) + 1.0) + 1.0);
        return true;
    };
    // ---- the list replay ----
    std::vector<uint32_t> bis(N), brow(N);
    for (uint32_t i = 0; i < N; i++) bis[i] = brow[i] = i;
    std::vector<uint8_t> sel(N, 0), proc(N, 0);
    NoDevice rp(v, sel, false, maxI);
    BGroup g;
    std::vector<DHit> hits;
    std::vector<DClause> cl;
    auto group_of = [&](uint32_t bi) -> BGroup& {
        const uint32_t T = brow[bi];
        clauses_of(T, cl);
        hits.clear();
        for (uint32_t j = 0; j < N; j++) {
            if (party[T] != kNoParty && party[j] == party[T]) continue;
            if (minc[j] < minc[T] || maxc[j] > maxc[T]) continue;
            int64_t k;
            if (score(cl, j, &k)) hits.push_back(DHit{j, j, k});
        }
        std::stable_sort(hits.begin(), hits.end(), [](const DHit& a, const DHit& b) { return a.key > b.key; });
        g.reset();
        g.set_hits(hits.data());
        g.n = (uint32_t)hits.size();
        g.complete = true;
        return g;
    };
    PoolOut ref;
    const bool no_ref = argc > 4 && std::string(argv[4]) == "noref";  // timing only
    const double r0 = now_ms();
    if (!no_ref) replay_pool(rp, bis, brow.data(), group_of, sel, proc.data(), minc.data(), maxc.data(), ref);
    const double r1 = now_ms();
    // ---- the range walk ----
    std::vector<uint32_t> leaves;
    for (uint32_t j = 0; j < N; j++)
        if (numeric[j]) leaves.push_back(j);
    std::sort(leaves.begin(), leaves.end(), [&](uint32_t a, uint32_t b) { return val[a] != val[b] ? val[a] < val[b] : a < b; });
    const uint32_t nv = (uint32_t)leaves.size();
    std::vector<int64_t> skeys(nv);
    std::vector<uint32_t> lslot(nv), lrank(nv), leaf_of(N, kNoSlot), leaf_of_slot(N, kNoSlot);
    for (uint32_t k = 0; k < nv; k++) {
        skeys[k] = val[leaves[k]];
        lslot[k] = lrank[k] = leaves[k];
        leaf_of[leaves[k]] = k;
        leaf_of_slot[leaves[k]] = k;
    }
    const double w0 = now_ms();
    RangeSrc src;
    src.n = nv;
    src.slot = lslot.data();
    src.rank = lrank.data();
    src.leaf_of = leaf_of.data();
    std::vector<HotRec> lhot(nv);
    std::vector<int32_t> livl(nv);
    for (uint32_t k = 0; k < nv; k++) {
        lhot[k] = hot[lslot[k]];
        livl[k] = intervals[lslot[k]];
    }
    src.lhot = lhot.data();
    src.livl = livl.data();
    src.tree.build(lrank.data(), nv);
    std::vector<RRange> tiers;
    std::vector<uint32_t> t0(N), t1(N);
    for (uint32_t i = 0; i < N; i++) {  // bounds as rsrc_bounds_kernel finds them
        clauses_of(i, cl);
        uint32_t lo[32], hi[32];
        int nr = 0;
        for (const DClause& c : cl)
            if (c.op == OP_RANGE) {
                lo[nr] = (uint32_t)(std::lower_bound(skeys.begin(), skeys.end(), c.lo) - skeys.begin());
                hi[nr] = (uint32_t)(std::upper_bound(skeys.begin(), skeys.end(), c.hi) - skeys.begin());
                nr++;
            }
        t0[i] = (uint32_t)tiers.size();
        build_tiers(cl.data(), (int)cl.size(), lo, hi, nv, tiers);
        t1[i] = (uint32_t)tiers.size();
    }
    const double w1 = now_ms();
    std::vector<uint8_t> psel(N, 0), proc2(N, 0);
    RangeRun run{};
    run.v = v;
    run.max_intervals = maxI;
    run.psel = psel.data();
    run.proc = proc2.data();
    run.leaf_of_slot = leaf_of_slot.data();
    run.fast = !(argc > 5 && std::string(argv[5]) == "exact");
    PoolOut out;
    run.walk(src, bis.data(), N, brow.data(),
             [&](uint32_t bi, const RRange*& base, uint32_t& a, uint32_t& b) {
                 base = tiers.data();
                 a = t0[brow[bi]];
                 b = t1[brow[bi]];
             },
             out);
    const double w2 = now_ms();
    // RB_PERF=1: the walk again (fresh tree), RB_REPS times, under the PMU
    if (std::getenv("RB_PERF")) {
        const int reps = std::getenv("RB_REPS") ? std::atoi(std::getenv("RB_REPS")) : 5;
        PerfGroup pg;
        double best = 1e30;
        uint64_t rows = 0, hits = 0;
        for (int r = 0; r < reps; r++) {
            src.tree.build(lrank.data(), nv);
            PoolOut o2;
            run.hits_seen = 0;
            const double a0 = now_ms();
            pg.start();
            run.walk(src, bis.data(), N, brow.data(),
                     [&](uint32_t bi, const RRange*& base, uint32_t& a, uint32_t& b) {
                         base = tiers.data();
                         a = t0[brow[bi]];
                         b = t1[brow[bi]];
                     },
                     o2);
            pg.stop();
            best = std::min(best, now_ms() - a0);
            rows += o2.recs.size() - 1;  // processed rows (the last record is the sentinel)
            hits += run.hits_seen;
        }
        if (pg.ok() && rows)
            std::printf("[perf] range walk, %d reps: per processed row %.0f cycles, %.0f instructions (IPC %.2f), %.2f "
                        "branch misses, %.2f L1D read misses; hits examined %.2f; best walk %.3f ms\n",
                        reps, (double)pg.v[0] / rows, (double)pg.v[1] / rows, (double)pg.v[1] / pg.v[0],
                        (double)pg.v[2] / rows, (double)pg.v[3] / rows, (double)hits / rows, best);
        else
            std::printf("[perf] no PMU here; best walk %.3f ms over %d reps\n", best, reps);
    }
    // ---- compare ----
    auto digest = [](const PoolOut& o) {
        uint64_t h = 1469598103934665603ull;
        auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
        for (const PoolRec& r : o.recs) {
            mix(r.bi); mix(r.matched); mix(r.expired); mix(r.len); mix(r.gcum); mix(r.xcum);
        }
        for (auto& e : o.ents) { mix(e.first); mix((uint64_t)e.second); }
        return h;
    };
    const uint64_t a = digest(ref), b = digest(out);
    size_t groups = 0;
    for (const PoolRec& r : out.recs) groups += r.matched;
    std::printf("range_bench: %u tickets (%s%s), %zu groups | list replay %016llx %.1f ms | range walk %016llx "
                "(tiers %.2f ms, walk %.2f ms = %.0f ns/row, %llu hits) | %s\n",
                N, mixed ? "mixed" : "solo", shared ? ", shared sessions" : "", groups, (unsigned long long)a, r1 - r0,
                (unsigned long long)b, w1 - w0, w2 - w1, (w2 - w1) * 1e6 / N, (unsigned long long)run.hits_seen,
                no_ref ? "timing only" : a == b ? "MATCH" : "DIFFER");
    return a == b || no_ref ? 0 : 1;
}
