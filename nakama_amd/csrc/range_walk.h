// nakama_amd/csrc/range_walk.h — processDefault's greedy walk over a
// numeric-range source (the C2 skill-window searches).
//
// A range-source search (Sig::rs_field) is "+term:<pool> and numeric range
// clauses on one field f" (MUST / SHOULD / MUST_NOT, with boosts): every
// candidate of its pool that holds a number in f scores by which clauses
// contain that number, so the hit list in the reference's order (score desc,
// created_at asc, doc order; matchmaker_process.go:86-90 over
// bluge/search/searcher/search_numeric_range.go:26-83) is: tier by tier (one
// score each, highest first), the tier's candidates in source order.  With the
// pool's candidates sorted by f on the device (rsrc_* kernels), a tier is a
// few leaf intervals of that order.  The walk keeps, per pool, a min tree over
// the leaves holding each candidate's source position (its hit rank), or
// kInf once it is selected: a row's next hit is the smallest rank over the
// current tier's intervals — O(log n) per hit, whatever the depth at which the
// reference's walk finds it (a list-based replay skips every earlier-selected
// hit, so late rows walked thousands of entries and lists ran out).  Hits the
// row has read are masked (kInf) until the row ends, so the row sees exactly
// the reference's sequence; the loop body is ReplayCore::row's.
//
// Pure host code over plain arrays (no store, no HIP): timed and checked on
// its own by tools/range_bench.cpp.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "gocompat.h"
#include "mm_device.h"
#include "qcompile.h"
#include "replay_core.h"

namespace nkm {

#define NKM_INLINE inline __attribute__((always_inline))

// Lane masks of a 16-entry block: kLaneBelow.m[l] has lanes j < l all ones,
// kLaneFrom.m[h] lanes j >= h (OR-ed into a block, they read as kInf).
struct alignas(64) LaneMasks {
    uint32_t m[17][16];
};
constexpr LaneMasks make_lane_masks(bool below) {
    LaneMasks t{};
    for (int i = 0; i <= 16; i++)
        for (int j = 0; j < 16; j++) t.m[i][j] = (below ? j < i : j >= i) ? 0xFFFFFFFFu : 0u;
    return t;
}
inline constexpr LaneMasks kLaneBelow = make_lane_masks(true), kLaneFrom = make_lane_masks(false);

// Min over leaf intervals with point updates: fan-out 16 levels (a query
// touches at most two partial blocks per level; 25k leaves are 4 levels).
// (gcc's -Wpsabi note on the 64-B vector returns: they are always inlined)
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wpsabi"
struct MinTree16 {
    static constexpr uint32_t kInf = 0xFFFFFFFFu;
    // level k's storage (16 spare entries: lp[k] is its first 64-B boundary,
    // so a 16-entry block is exactly one cache line, not two)
    std::vector<std::vector<uint32_t>> lv;
    // lp[0]: leaves; lp[k][i] = min of lp[k-1][16i, 16i + 16) (range_min / set
    // read them per level: one load instead of the vector-of-vectors' two)
    uint32_t* lp[8] = {};
    uint32_t nlev = 0;
    void build(const uint32_t* v, uint32_t n) {
        size_t L = 1;
        for (uint32_t m = n; m > 16; m = (m + 15) / 16) L++;
        lv.resize(L);
        uint32_t m = n;
        for (size_t k = 0; k < L; k++, m = (m + 15) / 16) {
            const size_t len = ((size_t)m + 15) & ~(size_t)15;
            lv[k].resize(len + 16);
            lp[k] = reinterpret_cast<uint32_t*>((reinterpret_cast<uintptr_t>(lv[k].data()) + 63) & ~(uintptr_t)63);
            std::fill(lp[k], lp[k] + len, kInf);
        }
        std::memcpy(lp[0], v, (size_t)n * 4);
        m = n;
        for (size_t k = 1; k < L; k++) {
            m = (m + 15) / 16;
            const uint32_t* c = lp[k - 1];
            for (uint32_t i = 0; i < m; i++) lp[k][i] = min16(c + 16 * (size_t)i);  // padding is kInf
        }
        nlev = (uint32_t)L;
    }
    // 16-lane vector mins (4 x 128 bits, or 2 x 256 bits in the walk's AVX2
    // instantiation, RangeRun::walk)
    static NKM_INLINE uint32_t min16(const uint32_t* p) { return reduce(load16(p)); }
    // min over leaves [a, b)
    NKM_INLINE uint32_t range_min(uint32_t a, uint32_t b) const {
        V16 acc = V16{} - 1u;
        range_min_acc(a, b, acc);
        return reduce(acc);
    }
    // Lane-wise min over leaves [a, b) into acc, without a horizontal reduce
    // per block: per level, the blocks holding a and b - 1 with the lanes
    // outside [a, b) OR-ed to all ones (= kInf, so they never win); the
    // blocks strictly between are the next level's elements.
    // (GNU vector extensions: clang and gcc; unsigned lane compares -> pminud)
    using V16 = uint32_t __attribute__((vector_size(64)));
    using V8 = uint32_t __attribute__((vector_size(32)));
    using V4 = uint32_t __attribute__((vector_size(16)));
    static NKM_INLINE V16 load16(const uint32_t* p) {
        V16 x;
        std::memcpy(&x, p, 64);
        return x;
    }
    static NKM_INLINE uint32_t reduce(const V16& x) {
        V8 h0, h1;
        std::memcpy(&h0, &x, 32);
        std::memcpy(&h1, reinterpret_cast<const char*>(&x) + 32, 32);
        h0 = h1 < h0 ? h1 : h0;
        V4 q0, q1;
        std::memcpy(&q0, &h0, 16);
        std::memcpy(&q1, reinterpret_cast<const char*>(&h0) + 16, 16);
        q0 = q1 < q0 ? q1 : q0;
        const uint32_t a = q0[0] < q0[1] ? q0[0] : q0[1], b = q0[2] < q0[3] ? q0[2] : q0[3];
        return a < b ? a : b;
    }
    NKM_INLINE void range_min_acc(uint32_t a, uint32_t b, V16& acc) const {
        for (size_t k = 0; a < b; k++) {
            const uint32_t* v = lp[k];
            const uint32_t ab = a >> 4, bb = (b - 1) >> 4;
            if (ab == bb) {
                const V16 x = load16(v + 16 * (size_t)ab) | load16(kBelow[a & 15]) | load16(kFrom[((b - 1) & 15) + 1]);
                acc = x < acc ? x : acc;
                return;
            }
            const V16 x = load16(v + 16 * (size_t)ab) | load16(kBelow[a & 15]);
            const V16 y = load16(v + 16 * (size_t)bb) | load16(kFrom[((b - 1) & 15) + 1]);
            const V16 m = x < y ? x : y;
            acc = m < acc ? m : acc;
            a = ab + 1;
            b = bb;
        }
    }
    static constexpr const uint32_t (*kBelow)[16] = kLaneBelow.m;
    static constexpr const uint32_t (*kFrom)[16] = kLaneFrom.m;
    NKM_INLINE void set(uint32_t i, uint32_t x) {
        lp[0][i] = x;
        for (uint32_t k = 1; k < nlev; k++) {
            const uint32_t blk = i >> 4;
            const uint32_t nm = min16(lp[k - 1] + ((size_t)blk << 4));
            if (lp[k][blk] == nm) return;  // the parents are unchanged
            lp[k][blk] = nm;
            i = blk;
        }
    }
};

// One leaf interval of a tier; `tend` is the index (in the signature's range
// list) one past the tier's last interval.
struct RRange {
    uint32_t a, b, tend;
};

// The tiers of a range-source signature over its pool's sorted leaves
// [0, n_valid): clause c (in clause order, range clauses only) contains the
// leaves [lo[c], hi[c]).  Each elementary interval between the clauses'
// boundaries is scored exactly as search_kernel's eval_parsed sums it for
// every candidate inside (same clause order, same double additions), so the
// tier keys equal the device's score keys bit for bit.  Appends the tiers,
// highest key first, each a list of disjoint intervals in leaf order.
inline void build_tiers(const DClause* cl, int n, const uint32_t* lo, const uint32_t* hi, uint32_t n_valid,
                        std::vector<RRange>& out) {
    uint32_t xs[2 + 2 * 64];
    int nx = 0;
    xs[nx++] = 0;
    xs[nx++] = n_valid;
    int nr = 0;
    for (int i = 0; i < n; i++)
        if (cl[i].op == OP_RANGE) {
            xs[nx++] = std::min(lo[nr], n_valid);
            xs[nx++] = std::min(hi[nr], n_valid);
            nr++;
        }
    std::sort(xs, xs + nx);
    nx = (int)(std::unique(xs, xs + nx) - xs);
    struct E { int64_t key; uint32_t a, b; };
    E es[2 + 2 * 64];
    int ne = 0;
    for (int k = 0; k + 1 < nx; k++) {
        const uint32_t a = xs[k], b = xs[k + 1];
        double ms = 0.0, ss = 0.0;
        bool has_must = false, any_should = false, fail = false;
        int r = 0;
        for (int i = 0; i < n; i++) {
            bool h = true;  // the pool's MUST term: every candidate holds it
            if (cl[i].op == OP_RANGE) {
                h = std::min(lo[r], n_valid) <= a && b <= std::min(hi[r], n_valid);
                r++;
            }
            if (cl[i].occur == OCC_MUST) {
                has_must = true;
                if (h) ms += cl[i].score;
                else fail = true;
            } else if (cl[i].occur == OCC_SHOULD) {
                if (h) { ss += cl[i].score; any_should = true; }
            } else if (h) {
                fail = true;
            }
        }
        if (fail || !has_must) continue;
        const double sp = any_should ? ms + ss : ms;
        es[ne++] = E{sortable_i64((sp + 1.0) + 1.0), a, b};
    }
    std::stable_sort(es, es + ne, [](const E& x, const E& y) { return x.key > y.key; });
    for (int k = 0; k < ne;) {
        int j = k;
        while (j < ne && es[j].key == es[k].key) j++;
        // [k, j): one tier, intervals ascending (stable sort), adjacent ones merged
        const size_t t0 = out.size();
        for (int q = k; q < j; q++) {
            if (out.size() > t0 && out.back().b == es[q].a) out.back().b = es[q].b;
            else out.push_back(RRange{es[q].a, es[q].b, 0});
        }
        for (size_t q = t0; q < out.size(); q++) out[q].tend = (uint32_t)out.size();
        k = j;
    }
}

// One pool's candidates in value order (the device sort's valid prefix).
// The fields the walk reads of a hit are copied per leaf (a pool's hits are
// value-neighbours: its leaves are its working set, not the whole store).
struct RangeSrc {
    uint32_t n = 0;               // leaves
    const uint32_t* slot = nullptr;  // per leaf: ticket slot
    const uint32_t* rank = nullptr;  // per leaf: source position (hit rank)
    const uint32_t* leaf_of = nullptr;  // per rank: its leaf
    const HotRec* lhot = nullptr;    // per leaf: the ticket's HotRec
    const int32_t* livl = nullptr;   // per leaf: the ticket's Intervals
    MinTree16 tree;
};

// The walk of one pool's rows (RangeRun::walk); records as replay_pool's.
struct RangeRun {
    ReplayView v;
    int max_intervals;
    uint8_t* psel;  // per slot: selected in this batch (starts and ends all zero)
    uint8_t* proc;  // per slot: processed earlier in this batch (pending Intervals)
    uint32_t* leaf_of_slot;  // per slot: its leaf in this pool, or kNoSlot (rows' own leaves)
    std::vector<std::vector<CE>> combos;
    std::vector<uint32_t> cmask, open, masked;
    std::vector<std::pair<uint32_t, int>> grp;
    uint64_t hits_seen = 0;
    bool fast = true;  // fast_row() for the rows it covers (NKM_FAST=0: row() only)
    FastCombos fcb;
    uint32_t mleaf[kFastComb][kFastMem];  // fast_row: the members' leaves (fcb.mem's slots)

    // iterator over one row's hits: tier by tier, smallest rank first;
    // every hit read is masked until the row ends
    RangeSrc* S = nullptr;
    const RRange* rg = nullptr;
    uint32_t cur = 0, end = 0;
    NKM_INLINE void mask(uint32_t leaf) {
        S->tree.set(leaf, MinTree16::kInf);
        masked.push_back(leaf);
    }
    NKM_INLINE bool next(uint32_t& leaf) {
        while (cur < end) {
            const uint32_t te = rg[cur].tend;
            MinTree16::V16 acc = MinTree16::V16{} - 1u;
            for (uint32_t k = cur; k < te; k++) S->tree.range_min_acc(rg[k].a, rg[k].b, acc);
            const uint32_t m = MinTree16::reduce(acc);
            if (m != MinTree16::kInf) {
                leaf = S->leaf_of[m];
                return true;
            }
            cur = te;
        }
        return false;
    }

    bool share_session(const HotRec& a, const HotRec& b) const {
        if (a.count == 1 && b.count == 1) return a.sess0 == b.sess0;
        for (uint32_t p = a.pres_off; p < a.pres_off + (uint32_t)a.count; p++)
            for (uint32_t q = b.pres_off; q < b.pres_off + (uint32_t)b.count; q++)
                if (v.pres_sess[p] == v.pres_sess[q]) return true;
        return false;
    }
    bool has_session(const HotRec& h, uint32_t sess) const {
        if (h.count == 1) return h.sess0 == sess;
        for (uint32_t q = h.pres_off; q < h.pres_off + (uint32_t)h.count; q++)
            if (v.pres_sess[q] == sess) return true;
        return false;
    }

    // processDefault's loop body (ReplayCore::row) for row T, whose search's
    // tiers are rg[r0, r1).  Candidates the device search would not return —
    // the searching ticket's party (:80-85) and the count-range musts
    // (MinCount >= T's Min, MaxCount <= T's Max) — are not hits: they are
    // skipped without counting.  Returns MATCHED / NOMATCH; group_out = grp.
    // row() when no two live tickets share a session (ReplayCore::fast_row
    // without the reverse checks): a combo is its member slots and entry
    // count.  BAIL when the row reaches the CountMultiple trim or outgrows the
    // fixed combos: nothing is selected yet, the caller restores the masks and
    // takes row().
    NKM_INLINE ReplayCore::Status fast_row(uint32_t T, uint32_t self_leaf, const RRange* r, uint32_t r0, uint32_t r1) {
        const HotRec& ht = v.hot[T];
        const bool last = v.intervals[T] + 1 >= max_intervals || ht.minc == ht.maxc;
        const int tcount = ht.count, tmax = ht.maxc, tmin = ht.minc, tcm = ht.cm;
        const int room = tmax - tcount;
        const uint32_t tparty = ht.party;
        auto is_hit = [&](const HotRec& hh) {
            return !(tparty != kNoParty && hh.party == tparty) && hh.minc >= tmin && hh.maxc <= tmax;
        };
        rg = r;
        cur = r0;
        end = r1;
        masked.clear();
        if (self_leaf != kNoSlot) mask(self_leaf);
        int ncomb = 0;
        uint32_t leaf;
        while (next(leaf)) {
            const uint32_t H = S->slot[leaf];
            mask(leaf);
            const HotRec& hh = S->lhot[leaf];
            if (!is_hit(hh)) continue;
            hits_seen++;
            if (tmax < hh.maxc && S->livl[leaf] + proc[H] <= max_intervals) continue;  // :150-153
            const int hc = hh.count;
            int f = 0;  // first fit (:167-226)
            while (f < ncomb && fcb.size[f] + hc > room) f++;
            if (f == ncomb) {
                if (f == kFastComb) return ReplayCore::BAIL;
                fcb.size[f] = 0;
                fcb.nmem[f] = 0;
                ncomb++;
            } else if (fcb.nmem[f] == (uint32_t)kFastMem) {
                return ReplayCore::BAIL;
            }
            fcb.size[f] += hc;
            mleaf[f][fcb.nmem[f]] = leaf;
            fcb.mem[f][fcb.nmem[f]++] = H;
            const int l = fcb.size[f] + tcount;
            bool form = l == tmax;  // :233
            if (!form && last && l >= tmin && l <= tmax) {
                bool more = false;
                uint32_t pl;
                while (!more && next(pl)) {
                    if (is_hit(S->lhot[pl])) more = true;
                    else mask(pl);
                }
                form = !more;
            }
            if (!form) continue;
            if (!multiple_of(l, tcm)) return ReplayCore::BAIL;
            bool failed = false;  // :287-296 (the members' HotRecs: this pool's leaf copies)
            for (uint32_t k = 0; k < fcb.nmem[f] && !failed; k++) {
                if (!v.live[fcb.mem[f][k]]) continue;
                const HotRec& hs = S->lhot[mleaf[f][k]];
                failed = hs.minc > l || hs.maxc < l || !multiple_of(l, hs.cm);
            }
            if (failed) continue;
            grp.clear();
            for (uint32_t k = 0; k < fcb.nmem[f]; k++) {
                const uint32_t m = fcb.mem[f][k];
                for (int e = 0, c = S->lhot[mleaf[f][k]].count; e < c; e++) grp.push_back({m, e});
            }
            for (int e = 0; e < tcount; e++) grp.push_back({T, e});
            return ReplayCore::MATCHED;
        }
        return ReplayCore::NOMATCH;
    }

    NKM_INLINE ReplayCore::Status row(uint32_t T, uint32_t self_leaf, const RRange* r, uint32_t r0, uint32_t r1) {
        const HotRec& ht = v.hot[T];
        const bool last = v.intervals[T] + 1 >= max_intervals || ht.minc == ht.maxc;
        const int tcount = ht.count, tmax = ht.maxc, tmin = ht.minc, tcm = ht.cm;
        const uint32_t tparty = ht.party;
        auto is_hit = [&](const HotRec& hh) {
            return !(tparty != kNoParty && hh.party == tparty) && hh.minc >= tmin && hh.maxc <= tmax;
        };
        rg = r;
        cur = r0;
        end = r1;
        masked.clear();
        if (self_leaf != kNoSlot) mask(self_leaf);  // self (:112-126)
        size_t ncomb = 0;
        open.clear();
        uint32_t leaf;
        while (next(leaf)) {
            const uint32_t H = S->slot[leaf];
            mask(leaf);
            const HotRec& hh = S->lhot[leaf];
            if (!is_hit(hh)) continue;
            hits_seen++;
            if (tmax < hh.maxc && S->livl[leaf] + proc[H] <= max_intervals) continue;          // :150-153
            if (!v.sessions_exclusive && (ht.smask & hh.smask) && share_session(ht, hh)) continue;  // :155-165
            bool sconf = false;  // sticky across combos of this hit (:156, :174-176, :206)
            int found = -1;
            const int hcount = hh.count;
            const uint32_t hp = hh.pres_off;
            size_t w = 0, q = 0;  // first fit over the open combos, dropping full ones on the way
            for (; q < open.size(); q++) {
                const uint32_t ci = open[q];
                auto& combo = combos[ci];
                if ((int)combo.size() + tcount >= tmax) continue;  // full for good
                open[w++] = ci;
                if ((int)combo.size() + hcount + tcount <= tmax) {
                    if (!v.sessions_exclusive && (cmask[ci] & hh.smask) != 0)
                        for (const CE& e : combo)
                            if (has_session(hh, e.sess)) { sconf = true; break; }
                    if (sconf) continue;
                    for (int k = 0; k < hcount; k++)
                        combo.push_back(CE{H, (uint32_t)k, leaf, hcount == 1 ? hh.sess0 : v.pres_sess[hp + k]});
                    cmask[ci] |= hh.smask;
                    found = (int)ci;
                    q++;
                    break;
                }
            }
            for (; q < open.size(); q++) open[w++] = open[q];
            open.resize(w);
            if (found < 0) {
                if (ncomb == combos.size()) {
                    combos.emplace_back();
                    cmask.push_back(0);
                }
                std::vector<CE>& nc = combos[ncomb];
                nc.clear();
                for (int k = 0; k < hcount; k++) nc.push_back(CE{H, (uint32_t)k, leaf, hcount == 1 ? hh.sess0 : v.pres_sess[hp + k]});
                cmask[ncomb] = hh.smask;
                found = (int)ncomb++;
                if (hcount + tcount < tmax) open.push_back((uint32_t)found);
            }
            std::vector<CE>& fc = combos[found];
            int l = (int)fc.size() + tcount;
            bool form = l == tmax;
            if (!form && last && l >= tmin && l <= tmax) {
                // another hit after this one? (:130, :233) — peek, skipping non-hits
                bool more = false;
                uint32_t pl;
                while (!more && next(pl)) {
                    if (is_hit(S->lhot[pl])) more = true;
                    else mask(pl);
                }
                form = !more;
            }
            if (!form) continue;
            const int rem = l % tcm;
            if (rem != 0) {                                                              // :234-280
                std::vector<uint32_t> elig;
                for (const CE& e : fc) {
                    if (!v.live[e.slot] || v.count[e.slot] > rem) continue;
                    if (std::find(elig.begin(), elig.end(), e.slot) == elig.end()) elig.push_back(e.slot);
                }
                std::vector<IG> groups;
                group_indexes(elig, 0, rem, v.count, v.created, groups);
                if (groups.empty()) continue;
                std::stable_sort(groups.begin(), groups.end(), [](const IG& a, const IG& b) { return a.avg < b.avg; });
                for (uint32_t gs : groups[0].idx) {
                    for (int k = 0; k < (int)fc.size(); k++) {
                        if (fc[k].slot == gs) {
                            fc[k] = fc.back();
                            fc.pop_back();
                            k--;
                        }
                    }
                }
                l = (int)fc.size() + tcount;
                close_trimmed(open, (uint32_t)found);
                if (!multiple_of(l, tcm)) continue;
            }
            bool failed = false;                                                         // :287-296
            for (const CE& e : fc) {
                const uint32_t s = e.slot;
                const HotRec& hs = v.hot[s];
                if (!v.live[s]) continue;
                if (hs.minc > l || hs.maxc < l || !multiple_of(l, hs.cm)) { failed = true; break; }
            }
            if (failed) continue;
            grp.clear();
            for (const CE& e : fc) grp.push_back({e.slot, (int)e.pi});
            for (int k = 0; k < tcount; k++) grp.push_back({T, k});
            return ReplayCore::MATCHED;
        }
        return ReplayCore::NOMATCH;
    }

    // The hits the row masked go back into the tree, except the selected.
    NKM_INLINE void unmask() {
        for (uint32_t leaf : masked)
            if (!psel[S->slot[leaf]]) S->tree.set(leaf, S->rank[leaf]);
        masked.clear();
    }

    // Walks a pool's rows (batch rows `bis`, ascending; slot brow[bi]);
    // sig_range(bi, base, r0, r1) gives the row's tier list base[r0, r1)
    // (one `base` for every row).  The rows' tier ranges and own leaves are
    // looked up first, in one pass whose independent misses overlap.
    // Appends records + a sentinel to `o`; psel / proc / the tree's masks are
    // restored on return except for the selections (the tree keeps them).
    template <class SigRange>
    void walk(RangeSrc& src, const uint32_t* bis, uint32_t nrows, const uint32_t* brow, SigRange sig_range, PoolOut& o) {
        if (__builtin_cpu_supports("avx2")) walk_avx2(src, bis, nrows, brow, sig_range, o);
        else walk_impl(src, bis, nrows, brow, sig_range, o);
    }
    template <class SigRange>
    __attribute__((target("avx2"))) void walk_avx2(RangeSrc& src, const uint32_t* bis, uint32_t nrows,
                                                   const uint32_t* brow, SigRange sig_range, PoolOut& o) {
        walk_impl(src, bis, nrows, brow, sig_range, o);
    }
    template <class SigRange>
    NKM_INLINE void walk_impl(RangeSrc& src, const uint32_t* bis, uint32_t nrows, const uint32_t* brow,
                              SigRange sig_range, PoolOut& o) {
        S = &src;
        uint32_t gcum = 0, xcum = 0;
        static thread_local std::vector<uint32_t> pre;  // per row: r0, r1, own leaf
        pre.resize((size_t)3 * nrows);
        const RRange* base = nullptr;
        for (uint32_t j = 0; j < nrows; j++) {
            const uint32_t bi = bis[j];
            sig_range(bi, base, pre[3 * (size_t)j], pre[3 * (size_t)j + 1]);
            pre[3 * (size_t)j + 2] = leaf_of_slot[brow[bi]];
        }
        for (uint32_t j = 0; j < nrows; j++) {
            const uint32_t bi = bis[j];
            const uint32_t T = brow[bi];
            if (j + 6 < nrows) {  // the next rows' records (their hits are unknown until searched;
                                  // about half the rows are skipped as selected, so 6 rows are ~3 walked)
                const uint32_t T2 = brow[bis[j + 6]];
                __builtin_prefetch(&v.hot[T2]);
                __builtin_prefetch(&psel[T2]);
                __builtin_prefetch(&v.intervals[T2]);
            }
            if (psel[T]) continue;
            const uint32_t r0 = pre[3 * (size_t)j], r1 = pre[3 * (size_t)j + 1], self = pre[3 * (size_t)j + 2];
            auto status = fast && v.sessions_exclusive ? fast_row(T, self, base, r0, r1) : ReplayCore::BAIL;
            if (status == ReplayCore::BAIL) {
                unmask();  // nothing selected yet: every mask goes back
                status = row(T, self, base, r0, r1);
            }
            const HotRec& ht = v.hot[T];
            PoolRec rec{bi, 0, (uint8_t)(v.intervals[T] + 1 >= max_intervals || ht.minc == ht.maxc),
                        (uint32_t)o.ents.size(), 0, gcum, xcum};
            xcum += rec.expired;
            if (status == ReplayCore::MATCHED) {
                rec.matched = 1;
                rec.len = (uint32_t)grp.size();
                gcum++;
                for (auto& e : grp) {
                    psel[e.first] = 1;
                    o.ents.push_back(e);
                }
            }
            unmask();
            proc[T] = 1;
            o.recs.push_back(rec);
        }
        for (auto& e : o.ents) psel[e.first] = 0;
        for (size_t k = 0; k < o.recs.size(); k++) proc[brow[o.recs[k].bi]] = 0;
        o.recs.push_back(PoolRec{UINT32_MAX, 0, 0, (uint32_t)o.ents.size(), 0, gcum, xcum});  // sentinel
    }
};
#pragma GCC diagnostic pop

}  // namespace nkm
