// tools/synth.cpp — seeded synthetic ticket sets for the five BASELINE configs
// (SURVEY.md 8(d)).  Bench/test tooling: produces mm_ticket arrays that are
// handed unchanged to mm_insert of either the HIP library or the CPU oracle,
// so both see byte-identical inputs.
//
//   CreatedAt = T0 + 1024*i (float64-exact, distinct), ticket id = UUID text
//   from splitmix64(seed, i), one unique session per presence, Intervals = 0.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <string>
#include <string_view>
#include <deque>
#include <unordered_set>
#include <vector>

#include "../include/nakama_mm.h"

namespace {

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Rng {
    uint64_t s;
    uint64_t next() { s = splitmix64(s); return s; }
    double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    double normal(double mu, double sd) {
        double u1 = uni(), u2 = uni();
        if (u1 < 1e-300) u1 = 1e-300;
        return mu + sd * std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    }
};

std::string uuid_of(uint64_t seed, uint64_t i) {
    uint64_t a = splitmix64(seed * 0x100000001B3ull + i), b = splitmix64(a ^ 0xD6E8FEB86659FD93ull);
    char buf[40];
    std::snprintf(buf, sizeof buf, "%08x-%04x-4%03x-%04x-%012llx", (unsigned)(a >> 32), (unsigned)((a >> 16) & 0xffff),
                  (unsigned)(a & 0xfff), (unsigned)(0x8000 | ((b >> 48) & 0x3fff)),
                  (unsigned long long)(b & 0xffffffffffffull));
    return buf;
}

struct Synth {
    std::vector<mm_ticket> t;
    std::vector<mm_presence> pres;
    std::vector<mm_str_prop> sp;
    std::vector<mm_num_prop> np;
    std::deque<std::string> strs;  // owned strings (deque: stable addresses)
    const char* keep(const std::string& s) {
        strs.push_back(s);
        return strs.back().c_str();
    }
};

const char* kModes[8] = {"ranked", "casual", "arena", "coop", "draft", "blitz", "custom", "event"};
const char* kRegions[8] = {"eu", "na", "sa", "ap", "me", "af", "oc", "cn"};

}  // namespace

extern "C" {

// Pool (mode x region partition) of ticket i for the pool-partitioned configs
// (2: its 4 region pools, 3: 2x4 = 8 pools, 4: 8x8 = 64 pools); -1 for the
// others.  Uses the same draws as synth_make, so it agrees with the generated
// properties.
int synth_pool_of(int config, uint64_t seed, uint64_t i) {
    Rng r{splitmix64(seed ^ (i * 0x9E3779B97F4A7C15ull))};
    if (config == 2) return (int)(r.next() & 3);
    if (config == 3) {
        (void)r.uni();
        const int mode = (int)(r.next() & 1), region = (int)(r.next() & 3);
        return mode * 4 + region;
    }
    if (config == 4) {
        const int mode = (int)(r.next() & 7), region = (int)(r.next() & 7);
        return mode * 8 + region;
    }
    return -1;
}

void* synth_make_impl(int config, uint64_t seed, int64_t first, int64_t n, int64_t t0, uint64_t pool_mask, int shard,
                      int pool_groups = 0);

// The pool group of ticket i in a scaled set (synth_make_scaled).
int synth_group_of(uint64_t seed, uint64_t i, int pool_groups) {
    return pool_groups > 0 ? (int)(splitmix64(seed ^ 0xA5A5A5A5ull ^ (i * 0xD1B54A32D192ED03ull)) % (uint64_t)pool_groups) : 0;
}

// The N-GPU weak-scaling set of configs 1-4 as ONE ticket set: every region
// value carries "-g<h>" with h = synth_group_of(i) in [0, pool_groups), so C3's
// 8 pools become 8 * pool_groups pools of the same size, spread over the whole
// index range (any rank's ingest slice holds tickets of every pool; the
// cluster front routes them).
void* synth_make_scaled(int config, uint64_t seed, int64_t first, int64_t n, int64_t t0, int pool_groups) {
    return synth_make_impl(config, seed, first, n, t0, ~0ull, -1, pool_groups);
}

// config: 1..5 as BASELINE.json configs[0..4], 6 = mixed, 7 = regexp/wildcard/fuzzy.  Generates tickets [first, first+n).
void* synth_make(int config, uint64_t seed, int64_t first, int64_t n, int64_t t0) {
    return synth_make_impl(config, seed, first, n, t0, ~0ull, -1);
}

// Same, with every region value suffixed "-g<shard>" (configs 1-4): shard s is
// a disjoint copy of the config's pool set (8 pools of C3 become 8 new ones),
// so N shards are the weak-scaling workload of an N-GPU pool-sharded run in
// which every GPU owns exactly one config instance.
void* synth_make_shard(int config, uint64_t seed, int64_t first, int64_t n, int64_t t0, int shard) {
    return synth_make_impl(config, seed, first, n, t0, ~0ull, shard);
}

// Same, keeping only tickets whose pool bit is set in pool_mask (pool-sharded
// multi-GPU runs: each rank generates exactly its pools' tickets).
void* synth_make_pools(int config, uint64_t seed, int64_t first, int64_t n, int64_t t0, uint64_t pool_mask) {
    return synth_make_impl(config, seed, first, n, t0, pool_mask, -1);
}

void* synth_make_impl(int config, uint64_t seed, int64_t first, int64_t n_all, int64_t t0, uint64_t pool_mask, int shard,
                      int pool_groups) {
    char sfx[16] = "";
    if (shard >= 0) std::snprintf(sfx, sizeof sfx, "-g%d", shard);
    std::vector<const char*> shard_regions(8);  // region values of this shard
    for (int k = 0; k < 8; k++) shard_regions[k] = kRegions[k];
    auto* S = new Synth();
    // scaled sets: region values per pool group
    std::vector<std::vector<const char*>> grp_regions(std::max(pool_groups, 0), std::vector<const char*>(8));
    for (int g = 0; g < pool_groups; g++)
        for (int k = 0; k < 8; k++) grp_regions[g][k] = S->keep(std::string(kRegions[k]) + "-g" + std::to_string(g));
    std::vector<uint64_t> idx;
    idx.reserve((size_t)n_all);
    for (int64_t k = 0; k < n_all; k++) {
        const uint64_t i = (uint64_t)(first + k);
        const int p = pool_mask == ~0ull ? -1 : synth_pool_of(config, seed, i);
        if (p < 0 || ((pool_mask >> p) & 1)) idx.push_back(i);
    }
    const int64_t n = (int64_t)idx.size();
    if (shard >= 0)
        for (int k = 0; k < 8; k++) shard_regions[k] = S->keep(std::string(kRegions[k]) + sfx);
    S->t.resize((size_t)n);
    S->pres.reserve((size_t)n * 5);
    S->sp.reserve((size_t)n * 3);
    S->np.reserve((size_t)n * 2);
    struct Tmp { size_t p0, np, s0, ns, n0, nn; };
    std::vector<Tmp> tmp((size_t)n);
    for (int64_t k = 0; k < n; k++) {
        const uint64_t i = idx[(size_t)k];
        Rng r{splitmix64(seed ^ (i * 0x9E3779B97F4A7C15ull))};
        mm_ticket& t = S->t[(size_t)k];
        std::memset(&t, 0, sizeof t);
        const std::string id = uuid_of(seed, i);
        t.ticket = S->keep(id);
        t.created_at = t0 + 1024 * (int64_t)i;
        t.node = "node1";
        t.count_multiple = 1;
        int party = 1;
        std::string query;
        Tmp& tm = tmp[(size_t)k];
        tm.s0 = S->sp.size();
        tm.n0 = S->np.size();
        const std::vector<const char*>& shard_regions_i =
            pool_groups > 0 ? grp_regions[synth_group_of(seed, i, pool_groups)] : shard_regions;
        switch (config) {
        case 1: {
            const char* mode = kModes[r.next() & 1];
            const char* region = shard_regions_i[r.next() & 3];
            S->sp.push_back({"mode", mode});
            S->sp.push_back({"region", region});
            query = std::string("+properties.mode:ranked +properties.region:") +
                    (pool_groups > 0 ? std::string(shard_regions_i[0]) : std::string("eu") + sfx);
            t.min_count = t.max_count = 2;
            break;
        }
        case 2: {
            const char* region = shard_regions_i[r.next() & 3];
            const int s = (int)std::lround(r.normal(1500.0, 300.0));
            S->sp.push_back({"region", region});
            S->np.push_back({"skill", (double)s});
            char q[256];
            std::snprintf(q, sizeof q,
                          "+properties.region:%s +properties.skill:>=%d +properties.skill:<=%d "
                          "properties.skill:>=%d^2 properties.skill:<=%d^2",
                          region, s - 200, s + 200, s - 50, s + 50);
            query = q;
            t.min_count = t.max_count = 2;
            break;
        }
        case 3: {
            const double u = r.uni();
            party = u < 0.60 ? 1 : u < 0.80 ? 2 : u < 0.90 ? 3 : u < 0.95 ? 4 : 5;
            const char* mode = kModes[r.next() & 1];
            const char* region = shard_regions_i[r.next() & 3];
            S->sp.push_back({"mode", mode});
            S->sp.push_back({"region", region});
            query = std::string("+properties.mode:") + mode + " +properties.region:" + region;
            t.min_count = t.max_count = 10;
            t.count_multiple = 5;
            break;
        }
        case 4: {
            const char* mode = kModes[r.next() & 7];
            const char* region = shard_regions_i[r.next() & 7];
            S->sp.push_back({"mode", mode});
            S->sp.push_back({"region", region});
            query = std::string("+properties.mode:") + mode + " +properties.region:" + region;
            t.min_count = t.max_count = 2;
            break;
        }
        case 5:
        case 11: {  // 11: C5 with buckets of 64 -> 63 filtered hits per row, where
                    // processCustom hands over no candidate (matchmaker_process.go:588)
            const int s = (int)std::lround(r.normal(1500.0, 300.0));
            char b[32];
            std::snprintf(b, sizeof b, "b%lld", (long long)(i / (config == 11 ? 64 : 8)));
            S->sp.push_back({"bucket", S->keep(b)});
            S->np.push_back({"skill", (double)s});
            char q[160];
            std::snprintf(q, sizeof q, "+properties.bucket:%s properties.skill:>=%d^2", b, s - 100);
            query = q;
            t.min_count = 2;
            t.max_count = 4;
            break;
        }
        case 13: {  // C5 variant, buckets of 12 (packed RevPrecision lists of stride 16):
                    // parties of 1-3, Min < Max, CountMultiple 2 on a third of the tickets
            const double u = r.uni();
            party = u < 0.6 ? 1 : u < 0.9 ? 2 : 3;
            const int s = (int)std::lround(r.normal(1500.0, 300.0));
            char b[32];
            std::snprintf(b, sizeof b, "c%lld", (long long)(i / 12));
            S->sp.push_back({"bucket", S->keep(b)});
            S->np.push_back({"skill", (double)s});
            char q[200];
            std::snprintf(q, sizeof q, "+properties.bucket:%s properties.skill:>=%d^2 properties.skill:<=%d^3", b, s - 150,
                          s + 100);
            query = q;
            const int shape = (int)(r.next() % 3);
            t.min_count = 2;
            t.max_count = shape == 0 ? 6 : 4;
            if (shape == 0) t.count_multiple = 2;
            break;
        }
        case 15:
        case 16: {  // C2 variant for the range batches (mm_range.cpp): parties of 1-3,
                    // Min<Max and CountMultiple shapes, MUST_NOT and fractional-boost
                    // ranges, tickets whose skill is a keyword (never a range hit);
                    // 16: every ticket in one region (a single pool)
            const double u = r.uni();
            party = u < 0.7 ? 1 : u < 0.9 ? 2 : 3;
            const char* region = shard_regions_i[config == 16 ? 0 : (r.next() & 3)];
            const int s = (int)std::lround(r.normal(1500.0, 300.0));
            S->sp.push_back({"region", region});
            if (r.uni() < 0.95) S->np.push_back({"skill", (double)s});
            else S->sp.push_back({"skill", "unrated"});
            char q[320];
            if (r.next() % 3 == 0)
                std::snprintf(q, sizeof q,
                              "+properties.region:%s +properties.skill:>=%d +properties.skill:<=%d "
                              "properties.skill:>=%d^2 properties.skill:<=%d^2 -properties.skill:>%d "
                              "properties.skill:<%d^0.5",
                              region, s - 250, s + 250, s - 60, s + 60, s + 200, s - 100);
            else
                std::snprintf(q, sizeof q,
                              "+properties.region:%s +properties.skill:>=%d +properties.skill:<=%d "
                              "properties.skill:>=%d^2 properties.skill:<=%d^2",
                              region, s - 200, s + 200, s - 50, s + 50);
            query = q;
            const int shape = (int)(r.next() % 3);
            if (shape == 0) { t.min_count = 2; t.max_count = 2; }
            else if (shape == 1) { t.min_count = 2; t.max_count = 4; }
            else { t.min_count = 4; t.max_count = 6; t.count_multiple = 2; }
            break;
        }
        case 17:
        case 18: {  // MaxCount % CountMultiple != 0 (Add / Insert accept it; the
                    // pipeline does not): combos formed at l == MaxCount = 5 are
                    // trimmed for CountMultiple 2 / 3 and often rejected by a
                    // member's own CountMultiple (matchmaker_process.go:234-296).
                    // 17: C3's 8 mode x region pools, one search per pool (the
                    // dense walk); 18: config 15's range searches (the range walk)
            const double u = r.uni();
            party = u < 0.6 ? 1 : u < 0.85 ? 2 : 3;
            t.count_multiple = (int)(r.next() % 3) + 1;
            t.min_count = 3;
            t.max_count = 5;
            if (config == 17) {
                const char* mode = kModes[r.next() & 1];
                const char* region = shard_regions_i[r.next() & 3];
                S->sp.push_back({"mode", mode});
                S->sp.push_back({"region", region});
                query = std::string("+properties.mode:") + mode + " +properties.region:" + region;
            } else {
                const char* region = shard_regions_i[r.next() & 3];
                const int s = (int)std::lround(r.normal(1500.0, 300.0));
                S->sp.push_back({"region", region});
                S->np.push_back({"skill", (double)s});
                char q[256];
                std::snprintf(q, sizeof q,
                              "+properties.region:%s +properties.skill:>=%d +properties.skill:<=%d "
                              "properties.skill:>=%d^2 properties.skill:<=%d^2",
                              region, s - 300, s + 300, s - 80, s + 80);
                query = q;
            }
            break;
        }
        case 14: {  // C5 variant, buckets of 24 (stride 32), a required skill range, 3-player groups
            const int s = (int)std::lround(r.normal(1500.0, 300.0));
            char b[32];
            std::snprintf(b, sizeof b, "d%lld", (long long)(i / 24));
            S->sp.push_back({"bucket", S->keep(b)});
            S->np.push_back({"skill", (double)s});
            char q[200];
            std::snprintf(q, sizeof q, "+properties.bucket:%s +properties.skill:>=%d properties.skill:>=%d^2", b, s - 400,
                          s - 100);
            query = q;
            t.min_count = t.max_count = 3;
            break;
        }
        case 7: {  // multi-term clauses: regexp / wildcard / fuzzy (blocked-list pattern of
                   // TestMatchmakerPropertyRegexSubmatch, server/matchmaker_test.go:162-286)
            static const char* kMaps[8] = {"map1", "map2", "map3", "map4", "map5", "map6", "some_map", "other_map"};
            party = r.uni() < 0.8 ? 1 : 2;
            const char* mode = kModes[r.next() & 1];
            const char* map = kMaps[r.next() & 7];
            char id[24], tag[24], blocked[64];
            std::snprintf(id, sizeof id, "u%llu", (unsigned long long)(i % 200));
            std::snprintf(tag, sizeof tag, "p%d", (int)(r.next() % 40));
            std::snprintf(blocked, sizeof blocked, "u%d u%d", (int)(r.next() % 200), (int)(r.next() % 200));
            S->sp.push_back({"mode", mode});
            S->sp.push_back({"map", map});
            S->sp.push_back({"id", S->keep(id)});
            S->sp.push_back({"tag", S->keep(tag)});
            S->sp.push_back({"blocked", S->keep(blocked)});
            char q[200];
            switch ((int)(r.next() % 8)) {
            case 0: std::snprintf(q, sizeof q, "+properties.mode:%s -properties.blocked:/.*%s([\\^0-9].*)?/", mode, id); break;
            case 1: std::snprintf(q, sizeof q, "+properties.mode:%s +properties.map:/(map[1-3]|some_map)/", mode); break;
            case 2: std::snprintf(q, sizeof q, "+properties.mode:%s properties.map:ma*1^2", mode); break;
            case 3: std::snprintf(q, sizeof q, "+properties.mode:%s properties.map:mapp2~1", mode); break;
            case 4: std::snprintf(q, sizeof q, "+properties.map:map~2 -properties.tag:/p[0-9]/"); break;
            case 5: std::snprintf(q, sizeof q, "+properties.mode:%s +properties.tag:p?", mode); break;
            case 6: std::snprintf(q, sizeof q, "+properties.mode:%s -properties.map:/(/", mode); break;
            default:
                std::snprintf(q, sizeof q, "+properties.mode:%s properties.map:/\\w+_map/^4 properties.tag:p1*", mode);
            }
            query = q;
            const int shape = (int)(r.next() % 2);
            t.min_count = 2;
            t.max_count = shape == 0 ? 2 : 4;
            break;
        }
        case 9: {  // C2's skill windows without the region must: every search crosses the
                   // region pools (the row-sharded mode's workload, include/nakama_cluster.h)
            const char* region = shard_regions_i[r.next() & 3];
            const int s = (int)std::lround(r.normal(1500.0, 300.0));
            S->sp.push_back({"region", region});
            S->np.push_back({"skill", (double)s});
            char q[256];
            std::snprintf(q, sizeof q,
                          "+properties.skill:>=%d +properties.skill:<=%d properties.skill:>=%d^2 "
                          "properties.skill:<=%d^2 properties.region:%s",
                          s - 200, s + 200, s - 50, s + 50, region);
            query = q;
            t.min_count = t.max_count = 2;
            break;
        }
        case 10: {  // wide queries: 1-6 distinct fields per query (keyword and numeric), every occur,
                    // so the kernels' preloaded-column paths (<= 2 / <= 4 fields) and their
                    // per-clause fallbacks all run
            static const char* kf[3] = {"k0", "k1", "k2"};
            static const char* nf[3] = {"n0", "n1", "n2"};
            static const char* kv[3] = {"a", "b", "c"};
            for (int f = 0; f < 3; f++)
                if (r.next() % 8) S->sp.push_back({kf[f], kv[r.next() % 3]});
            for (int f = 0; f < 3; f++)
                if (r.next() % 8) S->np.push_back({nf[f], (double)(r.next() % 20)});
            const int nfield = 1 + (int)(r.next() % 6);
            std::string q;
            bool any_pos = false;
            for (int c = 0; c < nfield; c++) {
                const int f = c % 3;
                const int occ = (int)(r.next() % 4);  // 0,1: must, 2: should (^2), 3: mustNot
                const char* pre = occ <= 1 ? "+" : occ == 3 ? "-" : "";
                char cl[96];
                if (c < 3) std::snprintf(cl, sizeof cl, "%sproperties.%s:%s", pre, kf[f], kv[r.next() % 3]);
                else std::snprintf(cl, sizeof cl, "%sproperties.%s:>=%d", pre, nf[f], (int)(r.next() % 12));
                if (occ == 2) std::strcat(cl, "^2");
                any_pos |= occ != 3;
                q += (q.empty() ? "" : " ") + std::string(cl);
            }
            if (!any_pos) q += " properties.n0:<=15";
            query = q;
            t.min_count = 2;
            t.max_count = (r.next() % 2) ? 2 : 3;
            break;
        }
        case 8: {  // datetime-typed string properties (blugeProcessProperty, match_common.go:161-170,221-236)
                   // and RFC3339 date-range clauses (query_string_parser.go:234-250)
            party = r.uni() < 0.85 ? 1 : 2;
            const char* mode = kModes[r.next() & 1];
            const int day = (int)(r.next() % 60), hh = (int)(r.next() % 24), mi = (int)(r.next() % 60),
                      ss = (int)(r.next() % 60);
            const int mon = 1 + day / 28, dd = 1 + day % 28;
            char since[64];
            switch ((int)(r.next() % 6)) {  // the five layouts bluge tries, and a string none parses
            case 0: std::snprintf(since, sizeof since, "2024-%02d-%02dT%02d:%02d:%02dZ", mon, dd, hh, mi, ss); break;
            case 1:
                std::snprintf(since, sizeof since, "2024-%02d-%02dT%02d:%02d:%02d.%09d+02:00", mon, dd, hh, mi, ss,
                              (int)(r.next() % 1000000000));
                break;
            case 2: std::snprintf(since, sizeof since, "2024-%02d-%02dT%02d:%02d:%02d", mon, dd, hh, mi, ss); break;
            case 3: std::snprintf(since, sizeof since, "2024-%02d-%02d %02d:%02d:%02d", mon, dd, hh, mi, ss); break;
            case 4: std::snprintf(since, sizeof since, "2024-%02d-%02d", mon, dd); break;
            default: std::snprintf(since, sizeof since, "2024-%02d-%02dX%02d", mon, dd, hh); break;  // keyword
            }
            S->sp.push_back({"mode", mode});
            S->sp.push_back({"since", S->keep(since)});
            const int d0 = (int)(r.next() % 50), d1 = d0 + 3 + (int)(r.next() % 20);
            char lo[40], hi[40];
            std::snprintf(lo, sizeof lo, "2024-%02d-%02dT00:00:00Z", 1 + d0 / 28, 1 + d0 % 28);
            std::snprintf(hi, sizeof hi, "2024-%02d-%02dT12:00:00+01:00", 1 + (d1 % 56) / 28, 1 + d1 % 28);
            char q[256];
            switch ((int)(r.next() % 4)) {
            case 0: std::snprintf(q, sizeof q, "+properties.mode:%s +properties.since:>=\"%s\"", mode, lo); break;
            case 1:
                std::snprintf(q, sizeof q, "+properties.mode:%s properties.since:>\"%s\"^2 properties.since:<=\"%s\"",
                              mode, lo, hi);
                break;
            case 2: std::snprintf(q, sizeof q, "+properties.mode:%s -properties.since:<\"%s\"", mode, lo); break;
            default: std::snprintf(q, sizeof q, "+properties.since:>=\"%s\" +properties.since:<=\"%s\"", lo, hi);
            }
            query = q;
            t.min_count = 2;
            t.max_count = (r.next() % 2) ? 2 : 3;
            break;
        }
        default: {  // 6: small mixed workload for parity (parties, ranges, boosts, Min<Max)
            const double u = r.uni();
            party = u < 0.7 ? 1 : u < 0.9 ? 2 : 3;
            const char* mode = kModes[r.next() & 1];
            const int s = (int)(r.next() % 50);
            S->sp.push_back({"mode", mode});
            S->np.push_back({"skill", (double)s});
            char q[200];
            const int v = (int)(r.next() % 4);
            if (v == 0) std::snprintf(q, sizeof q, "+properties.mode:%s", mode);
            else if (v == 1) std::snprintf(q, sizeof q, "+properties.mode:%s properties.skill:>=%d^2", mode, s);
            else if (v == 2) std::snprintf(q, sizeof q, "properties.skill:<=%d properties.mode:%s^3", s + 10, mode);
            else std::snprintf(q, sizeof q, "+properties.skill:>=%d -properties.mode:nope", s - 20);
            // 12: the same workload with every query pinned to its own mode
            // (pools by mode: the multi-GPU fronts' Min<Max / CountMultiple case)
            query = config == 12 ? std::string("+properties.mode:") + mode + " " + q : std::string(q);
            const int shape = (int)(r.next() % 3);
            if (shape == 0) { t.min_count = 2; t.max_count = 2; }
            else if (shape == 1) { t.min_count = 2; t.max_count = 4; }
            else { t.min_count = 4; t.max_count = 6; t.count_multiple = 2; }
            break;
        }
        }
        t.query = S->keep(query);
        tm.p0 = S->pres.size();
        for (int p = 0; p < party; p++) {
            char u[48], s[48];
            std::snprintf(u, sizeof u, "u%llu-%d", (unsigned long long)i, p);
            std::snprintf(s, sizeof s, "s%llu-%d", (unsigned long long)i, p);
            const char* us = S->keep(u);
            S->pres.push_back({us, S->keep(s), us, "node1"});
        }
        tm.np = (size_t)party;
        if (party > 1) {
            char pid[48];
            std::snprintf(pid, sizeof pid, "party-%llu", (unsigned long long)i);
            t.party_id = S->keep(pid);
            t.session_id = "";
        } else {
            t.party_id = "";
            t.session_id = S->pres.back().session_id;
        }
        tm.ns = S->sp.size() - tm.s0;
        tm.nn = S->np.size() - tm.n0;
    }
    for (int64_t k = 0; k < n; k++) {  // vectors are final now: wire the pointers
        mm_ticket& t = S->t[(size_t)k];
        const Tmp& tm = tmp[(size_t)k];
        t.presences = S->pres.data() + tm.p0;
        t.n_presences = (int32_t)tm.np;
        t.str_props = S->sp.data() + tm.s0;
        t.n_str_props = (int32_t)tm.ns;
        t.num_props = S->np.data() + tm.n0;
        t.n_num_props = (int32_t)tm.nn;
    }
    return S;
}

const mm_ticket* synth_tickets(void* h) { return static_cast<Synth*>(h)->t.data(); }
int64_t synth_count(void* h) { return (int64_t)static_cast<Synth*>(h)->t.size(); }
int64_t synth_presences(void* h) { return (int64_t)static_cast<Synth*>(h)->pres.size(); }
void synth_free(void* h) { delete static_cast<Synth*>(h); }

// The bench's MatchmakerOverride (a RuntimeMatchmakerOverrideFunction,
// server/runtime.go:212, stands in for user code): keeps every candidate group
// none of whose tickets an earlier kept group holds, in candidate order.
// Tickets are told apart by their ids' text.  Writes the kept groups'
// offsets (n_kept + 1) and entries into the caller's arrays (sized like the
// candidates'); returns the number of kept groups.
//
// Each distinct entry pointer is mapped once to a ticket number (its text
// hashed into a table of ids), then "taken" is a flag per ticket number: a
// library whose entries share one pointer per ticket (the product) hashes
// each id's text once, and the candidates of one row — a handful of tickets
// over and over — hit a small direct-mapped pointer cache; a library whose
// entries are copies (the oracle) hashes every entry's text, as before.
int32_t synth_override_first_disjoint(const int32_t* offs, const mm_entry_ref* ents, int32_t n_groups,
                                      int32_t* out_offs, mm_entry_ref* out_ents) {
    auto hash = [](const char* p, size_t n) {
        uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
        size_t i = 0;
        for (; i + 8 <= n; i += 8) {
            uint64_t w;
            std::memcpy(&w, p + i, 8);
            h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
            h ^= h >> 31;
        }
        if (i < n) {
            uint64_t w = 0;
            std::memcpy(&w, p + i, n - i);
            h = (h ^ w) * 0x94D049BB133111EBull;
        }
        return h ^ (h >> 29);
    };
    // ticket numbers by text
    struct TKey {
        const char* p;
        uint32_t n, tag, id;
    };
    std::vector<TKey> ttab(1u << 16, TKey{nullptr, 0, 0, 0});
    uint32_t n_ids = 0;
    auto text_id = [&](const char* p) -> uint32_t {
        const size_t n = std::strlen(p);
        const uint64_t h = hash(p, n);
        for (;;) {
            const size_t mask = ttab.size() - 1;
            for (size_t i = h & mask;; i = (i + 1) & mask) {
                TKey& k = ttab[i];
                if (!k.p) {
                    if (2 * (n_ids + 1) > ttab.size()) break;  // grow first
                    k = TKey{p, (uint32_t)n, (uint32_t)(h >> 32), n_ids};
                    return n_ids++;
                }
                if (k.tag == (uint32_t)(h >> 32) && k.n == n && (k.p == p || !std::memcmp(k.p, p, n))) return k.id;
            }
            std::vector<TKey> old(ttab.size() * 2, TKey{nullptr, 0, 0, 0});
            old.swap(ttab);
            const size_t m2 = ttab.size() - 1;
            for (const TKey& o : old) {
                if (!o.p) continue;
                size_t i = hash(o.p, o.n) & m2;
                while (ttab[i].p) i = (i + 1) & m2;
                ttab[i] = o;
            }
        }
    };
    // ticket numbers by pointer, behind a direct-mapped cache
    struct PKey {
        const char* p;
        uint32_t id;
    };
    std::vector<PKey> ptab(1u << 16, PKey{nullptr, 0});
    size_t pused = 0;
    auto pmix = [](const char* p) { return ((uint64_t)(uintptr_t)p * 0x9E3779B97F4A7C15ull) >> 20; };
    auto ptr_id = [&](const char* p) -> uint32_t {
        size_t mask = ptab.size() - 1;
        size_t i = pmix(p) & mask;
        for (; ptab[i].p; i = (i + 1) & mask)
            if (ptab[i].p == p) return ptab[i].id;
        const uint32_t id = text_id(p);
        ptab[i] = PKey{p, id};
        if (2 * ++pused > ptab.size()) {
            std::vector<PKey> old(ptab.size() * 2, PKey{nullptr, 0});
            old.swap(ptab);
            mask = ptab.size() - 1;
            for (const PKey& o : old) {
                if (!o.p) continue;
                size_t k = pmix(o.p) & mask;
                while (ptab[k].p) k = (k + 1) & mask;
                ptab[k] = o;
            }
        }
        return id;
    };
    PKey cache[256];
    for (PKey& c : cache) c = PKey{nullptr, 0};
    auto id_of = [&](const char* p) -> uint32_t {
        PKey& c = cache[((uintptr_t)p >> 4) & 255];
        if (c.p == p) return c.id;
        c = PKey{p, ptr_id(p)};
        return c.id;
    };
    std::vector<uint8_t> taken;
    auto is_taken = [&](uint32_t id) { return id < taken.size() && taken[id]; };
    int32_t kept = 0, e = 0;
    out_offs[0] = 0;
    for (int32_t g = 0; g < n_groups; g++) {
        bool free = true;
        for (int32_t k = offs[g]; k < offs[g + 1] && free; k++) free = !is_taken(id_of(ents[k].ticket));
        if (!free) continue;
        for (int32_t k = offs[g]; k < offs[g + 1]; k++) {
            const uint32_t id = id_of(ents[k].ticket);
            if (id >= taken.size()) taken.resize(std::max<size_t>(2 * taken.size(), id + 1), 0);
            taken[id] = 1;
            out_ents[e++] = ents[k];
        }
        out_offs[++kept] = e;
    }
    return kept;
}

// ---- digests of pass results (tests/golden/full_*.json, tools/make_full_golden.py) ----
// SHA-256 (FIPS 180-4) over a canonical text of a group list or a post-pass
// state, streamed so that 100M-entry candidate lists need no buffer:
//   groups: per group, per entry "<ticket>:<presence index>," then "\n";
//   state:  per remaining ticket in ascending id order "<ticket>:<intervals>\n".
// Python's hashlib over the same bytes gives the same digest
// (tools/make_full_golden.py merges pool lists in Python that way).
struct Sha256 {
    uint32_t h[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                     0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
    uint8_t buf[64];
    size_t nbuf = 0;
    uint64_t total = 0;
    static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
    void block(const uint8_t* p) {
        static const uint32_t K[64] = {
            0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
            0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
            0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
            0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
            0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
            0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
            0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
            0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
        uint32_t w[64];
        for (int i = 0; i < 16; i++)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; i++) {
            const uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
            const uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int i = 0; i < 64; i++) {
            const uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
            const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
    void update(const void* data, size_t n) {
        const uint8_t* p = static_cast<const uint8_t*>(data);
        total += n;
        while (n) {
            const size_t k = std::min(n, 64 - nbuf);
            std::memcpy(buf + nbuf, p, k);
            nbuf += k; p += k; n -= k;
            if (nbuf == 64) { block(buf); nbuf = 0; }
        }
    }
    void final(uint8_t out[32]) {
        const uint64_t bits = total * 8;
        const uint8_t one = 0x80, zero = 0;
        update(&one, 1);
        while (nbuf != 56) update(&zero, 1);
        uint8_t len[8];
        for (int i = 0; i < 8; i++) len[i] = (uint8_t)(bits >> (56 - 8 * i));
        update(len, 8);
        for (int i = 0; i < 8; i++)
            for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
    }
};

// The bench's delivery callback (mm_deliver_fn, include/nakama_mm.h) standing
// in for the reference's per-group delivery to a no-op router
// (matchmaker.go:374-440: per group the users list and envelope are built
// from every entry, then one SendToPresenceIDs per entry): it reads every
// entry's ticket id and presence index, counts the delivered groups, tickets
// (presence index 0) and presences, and its own time.  ctx: SynthDelivered.
struct SynthDelivered {
    int64_t passes, groups, tickets, presences, id_bytes, ns;
};
void synth_deliver_noop(void* ctx, const mm_matched* m, int64_t) {
    const auto t0 = std::chrono::steady_clock::now();
    SynthDelivered* d = static_cast<SynthDelivered*>(ctx);
    int64_t tickets = 0, bytes = 0;
    for (int32_t g = 0; g < m->n_groups; g++)
        for (int32_t e = m->group_offsets[g]; e < m->group_offsets[g + 1]; e++) {
            const mm_entry_ref& r = m->entries[e];
            tickets += r.presence_index == 0;
            bytes += r.ticket ? (int64_t)std::strlen(r.ticket) : 0;
        }
    d->passes++;
    d->groups += m->n_groups;
    d->tickets += tickets;
    d->presences += m->n_entries;
    d->id_bytes += bytes;
    d->ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

void* synth_sha_new() { return new Sha256(); }
void synth_sha_bytes(void* s, const uint8_t* p, int64_t n) { static_cast<Sha256*>(s)->update(p, (size_t)n); }
// Appends groups [0, n_groups) of a CSR group list; returns the entry count.
int64_t synth_sha_groups(void* s, const int32_t* offs, const mm_entry_ref* ents, int32_t n_groups) {
    Sha256& h = *static_cast<Sha256*>(s);
    char num[16];
    for (int32_t g = 0; g < n_groups; g++) {
        for (int32_t k = offs[g]; k < offs[g + 1]; k++) {
            h.update(ents[k].ticket, std::strlen(ents[k].ticket));
            const int m = std::snprintf(num, sizeof num, ":%d,", ents[k].presence_index);
            h.update(num, (size_t)m);
        }
        h.update("\n", 1);
    }
    return n_groups ? offs[n_groups] - offs[0] : 0;
}
// Appends a post-pass state: the extract list's (ticket, intervals) in
// ascending ticket order.
void synth_sha_extract(void* s, const mm_ticket* ts, int32_t n) {
    Sha256& h = *static_cast<Sha256*>(s);
    std::vector<int32_t> ord((size_t)n);
    for (int32_t i = 0; i < n; i++) ord[(size_t)i] = i;
    std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return std::strcmp(ts[a].ticket, ts[b].ticket) < 0; });
    char num[24];
    for (int32_t i : ord) {
        h.update(ts[i].ticket, std::strlen(ts[i].ticket));
        const int m = std::snprintf(num, sizeof num, ":%d\n", ts[i].intervals);
        h.update(num, (size_t)m);
    }
}
void synth_sha_final(void* s, uint8_t* out32) {
    static_cast<Sha256*>(s)->final(out32);
    delete static_cast<Sha256*>(s);
}

}  // extern "C"
