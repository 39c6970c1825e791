// nakama_amd/csrc/replay_core.h — the exact greedy replay of processDefault's
// loop body (server/matchmaker_process.go:105-330) over a hit list that the
// device searches produced.  Pure host code over plain per-slot arrays (no HIP
// calls): paging a truncated list and single RevPrecision pair checks are
// hooks the device-backed subclass (mm_process.cpp) implements.  Kept free of
// the store so the replay can be timed and tested on its own
// (tools/replay_bench.cpp).
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <stdexcept>
#include <cstring>
#include <utility>
#include <vector>

#include "mm_device.h"

namespace nkm {

// Per-slot fields the replay reads, packed (one 32-B record per ticket).
struct HotRec {
    uint32_t party;     // kNoParty for ""
    uint32_t sess0;     // session of presence 0
    uint32_t pres_off;  // first presence in pres_sess
    int32_t count, minc, maxc, cm;
    uint32_t smask;     // OR of 1 << (session id & 31) over the presences: disjoint masks share no session
};
static_assert(sizeof(HotRec) == 32, "HotRec is half a cache line");

// l % cm == 0 by a table of the multiples below 64 when l < 64 and cm <= 64
// (the group-forming checks run it once per row and once per member: an
// integer division each otherwise)
struct MultipleTable {
    uint64_t m[65] = {};
    constexpr MultipleTable() {
        for (int c = 1; c <= 64; c++)
            for (int l = 0; l < 64; l += c) m[c] |= 1ull << l;
    }
};
inline constexpr MultipleTable kMultiples{};
inline bool multiple_of(int l, int cm) {
    return (unsigned)l < 64u && (unsigned)(cm - 1) < 64u ? ((kMultiples.m[cm] >> l) & 1u) != 0 : l % cm == 0;
}

struct CE {  // combo entry: (ticket slot, presence index, list position of its hit, session)
    uint32_t slot;
    uint32_t pi;
    uint32_t lpos;
    uint32_t sess;
};

// groupIndexes (server/matchmaker.go:132-167), int64 wrapping arithmetic.
struct IG { std::vector<uint32_t> idx; int64_t avg; };
inline void group_indexes(const std::vector<uint32_t>& in, size_t from, int required, const int32_t* cnt,
                          const int64_t* created, std::vector<IG>& out) {
    if (from >= in.size() || required <= 0) return;
    const uint32_t cur = in[from];
    if (cnt[cur] > required) { group_indexes(in, from + 1, required, cnt, created, out); return; }
    if (cnt[cur] == required) {
        out.push_back(IG{{cur}, created[cur]});
    } else {
        std::vector<IG> fill;
        group_indexes(in, from + 1, required - cnt[cur], cnt, created, fill);
        for (auto& f : fill) {
            const int64_t n = (int64_t)f.idx.size();
            f.avg = (int64_t)((uint64_t)f.avg * (uint64_t)n + (uint64_t)created[cur]) / (n + 1);
            f.idx.push_back(cur);
            out.push_back(std::move(f));
        }
    }
    group_indexes(in, from + 1, required, cnt, created, out);
}

// After the CountMultiple trim the combo is out of the first-fit scan for the
// rest of the row, whatever follows.  Go trims `foundCombo`, a slice header
// over the backing array of entryCombos[foundComboIdx]
// (matchmaker_process.go:213-214, 262-271): the stored slice keeps its
// pre-trim length (tail slots nil'd), so a trimmed combo that is then rejected
// (:276-279, :294-296) still counts as full at :170 — it formed at
// l == MaxCount — and never takes another hit.  (A trim in the last-interval
// branch happens at the row's last hit, after which nothing is scanned.)
inline void close_trimmed(std::vector<uint32_t>& open, uint32_t combo) {
    auto it = std::find(open.begin(), open.end(), combo);
    if (it != open.end()) open.erase(it);
}

// The smallest mask >= x with at most c bits set (c >= 1).  Every value
// skipped lies in (x, x + lowbit(x)) for an x with more than c bits, i.e. it
// holds x's bits plus lower ones: combineIndexes (matchmaker_process.go:
// 586-590) `continue`s on all of them, so walking the masks this way visits
// exactly the subsets its ascending loop emits, in the same order, without
// the 2^n iterations.
inline uint64_t next_mask_le(uint64_t x, int c) {
    while (__builtin_popcountll(x) > c) x += x & (~x + 1);
    return x;
}

// A batch search and its (possibly extended) hit list.
struct BGroup {
    uint32_t sig = 0;
    uint16_t n_fields = 0;        // field columns the signature reads (roofline bytes)
    uint32_t nrows = 0;
    uint32_t row_slot = kNoSlot;  // RevPrecision: the single searching row
    bool retry = false;           // holds the row a truncated list stopped: its search returns every tier
    DGroup d{};
    // The hit list: `hits` (16-B DHit, slot + source position + score key) or,
    // for mscan lists (never cut, so no cursor needs their keys), 4-B slot
    // ids only.  slot(i) reads either: sp/ss = the first slot and the stride
    // in u32 words (4 over a DHit array, 1 over a slot list).
    const DHit* hits = nullptr;
    const uint32_t* sp = nullptr;
    uint32_t ss = 4;
    // a slot list's last entry (its pagination cursor: score key and source
    // position) is kept by the batch beside the lists (Core::h_last_): its
    // index there, or UINT32_MAX (an mscan list: complete, never paged)
    uint32_t last_i = UINT32_MAX;
    uint32_t slot(uint32_t i) const { return sp[(size_t)i * ss]; }
    void set_hits(const DHit* h) {
        hits = h;
        sp = h ? &h->slot : nullptr;
        ss = 4;
    }
    void set_slots(const uint32_t* s) {
        hits = nullptr;
        sp = s;
        ss = 1;
    }
    // RevPrecision reverse-check flags: one byte per entry (`rev`), or, for a
    // packed row (rpack_kernel: <= 64 entries), bits in entry order (rev_bits)
    const uint8_t* rev = nullptr;
    uint64_t rev_bits = 0;
    bool rev_packed = false;
    bool rev_at(uint32_t i) const { return rev_packed ? ((rev_bits >> i) & 1u) != 0 : rev[i] != 0; }
    // pair-matrix words per entry (rev rows with combos): pm_w bytes each
    // (4: search / rsmall lists; 1 or 2: packed rows of 8 or 16 entries)
    const void* pm = nullptr;
    uint32_t pm_n = 0;             // entries covered by pm
    uint8_t pm_w = 4;
    uint32_t pm_at(uint32_t a) const {
        return pm_w == 4 ? static_cast<const uint32_t*>(pm)[a]
                         : pm_w == 2 ? static_cast<const uint16_t*>(pm)[a] : static_cast<const uint8_t*>(pm)[a];
    }
    bool has_src_term = false;     // source = posting list of (src_field, src_term)
    uint16_t src_field = 0;
    uint32_t src_term = 0;
    uint32_t n = 0;
    bool complete = true;
    // an mscan list proven equal to the search's own batch rows (Core::
    // list_proven): its host buffer (sp) is not filled — the dense walk takes
    // row j's slot as position j; any other reader fills it first
    // (Core::fill_row_lists)
    bool rows_list = false;
    uint32_t head = 0;
    std::vector<DHit> ext;
    std::vector<uint8_t> ext_rev;
    // back to a default-constructed search, keeping the vectors' capacity
    // (a reused batch array is refilled in place by the host workers)
    void reset() {
        sig = 0;
        n_fields = 0;
        nrows = 0;
        row_slot = kNoSlot;
        retry = false;
        d = DGroup{};
        hits = nullptr;
        sp = nullptr;
        ss = 4;
        last_i = UINT32_MAX;
        rev = nullptr;
        rev_bits = 0;
        rev_packed = false;
        pm = nullptr;
        pm_n = 0;
        pm_w = 4;
        has_src_term = false;
        src_field = 0;
        src_term = 0;
        n = 0;
        complete = true;
        rows_list = false;
        head = 0;
        ext.clear();
        ext_rev.clear();
        last_i = UINT32_MAX;
    }
};

// Read-only per-slot views of the store that the replay consults.
struct ReplayView {
    const HotRec* hot;
    const uint32_t* pres_sess;  // per presence: session dictionary id
    const uint32_t* party;      // per slot: party dictionary id (kNoParty for "")
    const int32_t* intervals;
    const uint8_t* live;        // in m.indexes
    const int32_t* count;
    const int64_t* created;
    // no two live tickets share a session (sessionTickets holds one ticket
    // per session): every session check of the loop body is false
    bool sessions_exclusive = false;
};

// Combos of the fast walks: member tickets (slots, or list positions in the
// dense walk) and entry counts only — what the loop body needs when no
// session check can fire.  A row that outgrows them takes the exact path.
constexpr int kFastComb = 32, kFastMem = 32;
struct FastCombos {
    int32_t size[kFastComb];            // entries
    uint32_t nmem[kFastComb];
    uint32_t mem[kFastComb][kFastMem];  // members, in the order they joined
    // RevPrecision (lists of <= 32 entries, all covered by the pair words):
    // the members' list positions, and the AND of the live members' pair words
    // (bit b: every live member's query matches entry b's document)
    uint64_t pos[kFastComb];
    uint64_t rcol[kFastComb];
};

struct ReplayCore {
    ReplayView v;
    std::vector<uint8_t>& sel;
    // RevPrecision reverse checks; cleared for the rest of the pass once the
    // RevThreshold timer fires (matchmaker_process.go:40-46,139,178)
    bool rev;
    const int max_intervals;
    std::vector<std::vector<CE>> combos;  // pool: the first ncomb are this row's entryCombos
    std::vector<uint32_t> cmask;          // per combo: OR of its entries' session masks (a superset)
    size_t ncomb = 0;
    // this row's combos that can still take an entry (size + T's count < MaxCount),
    // in index order.  A combo changes only when a hit joins it, which needs
    // room, so one that is full stays full: dropping it from the first-fit scan
    // is exact, and a row whose hits can never share a combo (T's party fills
    // MaxCount) scans nothing instead of every earlier hit's combo.
    std::vector<uint32_t> open;
    uint64_t hits_seen = 0;  // profiling: hit-list entries the rows walked
    // (row, candidate) pairs decided: the source lengths of the rows that
    // searched (PassStats::pairs_decided)
    uint64_t pairs = 0;
    // pool-parallel replay: rows this worker processed earlier in the batch,
    // whose Intervals increments are applied after the batch (1 = one pending)
    const uint8_t* proc = nullptr;
    static constexpr uint32_t kPrefetch = 8;
    static constexpr uint32_t kPairP = 32;  // pair matrices cover the first 32 entries of a list
    // fast_row() for rows it covers (NKM_FAST=0: row() only)
    bool fast = true;
    FastCombos fcb;

    ReplayCore(const ReplayView& view, std::vector<uint8_t>& s, bool r, int mi)
        : v(view), sel(s), rev(r), max_intervals(mi) {}
    virtual ~ReplayCore() = default;

    // Next page of a truncated list (device search with a cursor).
    virtual void fetch_more(BGroup& g) = 0;
    // validateMatch for a pair outside the list's pair matrix.
    virtual bool pair_slow(const BGroup& g, uint32_t from_pos, uint32_t to_pos) = 0;

    bool share_session(const HotRec& a, const HotRec& b) const {
        if (a.count == 1 && b.count == 1) return a.sess0 == b.sess0;
        for (uint32_t p = a.pres_off; p < a.pres_off + (uint32_t)a.count; p++)
            for (uint32_t q = b.pres_off; q < b.pres_off + (uint32_t)b.count; q++)
                if (v.pres_sess[p] == v.pres_sess[q]) return true;
        return false;
    }
    bool share_session(uint32_t a, uint32_t b) const { return share_session(v.hot[a], v.hot[b]); }
    bool has_session(const HotRec& h, uint32_t sess) const {
        if (h.count == 1) return h.sess0 == sess;
        for (uint32_t q = h.pres_off; q < h.pres_off + (uint32_t)h.count; q++)
            if (v.pres_sess[q] == sess) return true;
        return false;
    }
    // the party mustNot of the search (matchmaker_process.go:80-85)
    bool same_party(uint32_t T, uint32_t H) const {
        return v.party[T] != kNoParty && v.hot[H].party == v.party[T];
    }

    // validateMatch(from's query, to) for two entries of the same list.
    bool pair_ok(const BGroup& g, uint32_t from_pos, uint32_t to_pos) {
        if (g.pm && from_pos < g.pm_n && to_pos < g.pm_n) return (g.pm_at(from_pos) >> to_pos) & 1u;
        return pair_slow(g, from_pos, to_pos);
    }

    enum Status { MATCHED, NOMATCH, EXHAUSTED, BAIL };

    // processDefault's loop body for T: fast_row() when it applies (and does
    // not bail), else row().
    Status decide(uint32_t T, BGroup& g, bool can_fetch, std::vector<std::pair<uint32_t, int>>& group_out) {
        Status s = BAIL;
        if (fast && v.sessions_exclusive && g.complete && (!rev || (g.pm && g.pm_n >= g.n && g.n <= kPairP)))
            s = fast_row(T, g, group_out);
        if (s == BAIL) s = row(T, g, can_fetch, group_out);
        if (s != EXHAUSTED) pairs += g.d.src_len;  // the row searched: its source's candidates decided
        return s;
    }

    // row() when no two live tickets share a session, over a complete list:
    // every session check is false, so a combo is its member slots and entry
    // count.  With RevPrecision the list's pair words cover every entry, and
    // a combo also keeps its members' positions and the AND of its live
    // members' pair words, so validateMatch both ways against every member
    // (matchmaker_process.go:178-203) is two mask tests.  Returns BAIL, having
    // changed nothing but the list head, when the row reaches the
    // CountMultiple trim (:234-280) or outgrows the fixed combos.
    Status fast_row(uint32_t T, BGroup& g, std::vector<std::pair<uint32_t, int>>& group_out) {
        // members the loop reads are copied into locals (`sel` is a byte
        // array: a char load may alias any member, see DenseRun::fast_step)
        const HotRec* const hot = v.hot;
        const HotRec& ht = hot[T];
        const bool last = v.intervals[T] + 1 >= max_intervals || ht.minc == ht.maxc;
        const int tcount = ht.count, tmax = ht.maxc, tmin = ht.minc, tcm = ht.cm;
        const int room = tmax - tcount;  // entries a combo may hold
        const uint32_t tparty = ht.party;
        const uint8_t* const S = sel.data();
        const uint8_t* const pr = proc;
        const int32_t* const ivl = v.intervals;
        const uint8_t* const lv = v.live;
        const bool rv = rev;
        const int maxI = max_intervals;
        const uint32_t n = g.n;
        uint32_t h0 = g.head;
        while (h0 < n && S[g.slot(h0)]) h0++;
        g.head = h0;
        int ncomb = 0;
        uint64_t seen = 0;
        Status st = NOMATCH;
        int ff = -1;
        int lf = 0;
        for (uint32_t i = h0; i < n; i++) {
            if (i + kPrefetch < n) {
                const uint32_t P = g.slot(i + kPrefetch);
                __builtin_prefetch(&S[P]);
                __builtin_prefetch(&hot[P]);
            }
            const uint32_t H = g.slot(i);
            seen++;
            if (H == T || S[H]) continue;
            const HotRec& hh = hot[H];
            if (tparty != kNoParty && hh.party == tparty) continue;                          // :80-85
            if (rv && !g.rev_at(i)) continue;                                               // :139-148
            if (tmax < hh.maxc && ivl[H] + (pr ? pr[H] : 0) <= maxI) continue;              // :150-153
            const int hc = hh.count;
            int f = 0;  // first fit (:167-226)
            if (rv) {
                const uint64_t mine = g.pm_at(i), bit = 1ull << i;
                while (f < ncomb && (fcb.size[f] + hc > room || (mine & fcb.pos[f]) != fcb.pos[f] || !(fcb.rcol[f] & bit)))
                    f++;
            } else {
                while (f < ncomb && fcb.size[f] + hc > room) f++;
            }
            if (f == ncomb) {
                if (f == kFastComb) { st = BAIL; break; }
                fcb.size[f] = 0;
                fcb.nmem[f] = 0;
                fcb.pos[f] = 0;
                fcb.rcol[f] = ~0ull;
                ncomb++;
            } else if (fcb.nmem[f] == (uint32_t)kFastMem) {
                st = BAIL;
                break;
            }
            fcb.size[f] += hc;
            fcb.mem[f][fcb.nmem[f]++] = H;
            if (rv) {
                fcb.pos[f] |= 1ull << i;
                if (lv[H]) fcb.rcol[f] &= g.pm_at(i);
            }
            const int l = fcb.size[f] + tcount;
            bool form = l == tmax;  // :233
            if (!form && last && l >= tmin && l <= tmax) {
                bool more = false;
                for (uint32_t q = i + 1; q < n && !more; q++) {
                    const uint32_t s2 = g.slot(q);
                    more = s2 != T && !S[s2] && !same_party(T, s2);
                }
                form = !more;
            }
            if (!form) continue;
            if (!multiple_of(l, tcm)) { st = BAIL; break; }
            bool failed = false;  // :287-296
            for (uint32_t k = 0; k < fcb.nmem[f] && !failed; k++) {
                const uint32_t s2 = fcb.mem[f][k];
                if (!lv[s2]) continue;
                const HotRec& hs = hot[s2];
                failed = hs.minc > l || hs.maxc < l || !multiple_of(l, hs.cm);
            }
            if (failed) continue;
            st = MATCHED;
            ff = f;
            lf = l;
            break;
        }
        hits_seen += seen;
        (void)lf;
        if (st != MATCHED) return st;
        group_out.clear();
        for (uint32_t k = 0; k < fcb.nmem[ff]; k++) {
            const uint32_t m = fcb.mem[ff][k];
            for (int e = 0; e < hot[m].count; e++) group_out.push_back({m, e});
        }
        for (int e = 0; e < tcount; e++) group_out.push_back({T, e});
        return MATCHED;
    }

    // Is there an unselected, non-self hit after position i?  (the
    // hitCounter >= lastHitCounter test, matchmaker_process.go:130,233)
    int more_hits_after(BGroup& g, uint32_t i, uint32_t T, bool can_fetch) {
        for (uint32_t j = i + 1;; j++) {
            if (j >= g.n) {
                if (g.complete) return 0;
                if (!can_fetch) return -1;
                fetch_more(g);
                if (j >= g.n) {
                    if (g.complete) return 0;
                    j--;  // nothing new yet: look at position j again
                    continue;
                }
            }
            const uint32_t s = g.slot(j);
            if (s != T && !sel[s] && !same_party(T, s)) return 1;
        }
    }

    // processDefault's loop body for one active ticket T.
    Status row(uint32_t T, BGroup& g, bool can_fetch, std::vector<std::pair<uint32_t, int>>& group_out) {
        const HotRec& ht = v.hot[T];
        const bool last = v.intervals[T] + 1 >= max_intervals || ht.minc == ht.maxc;
        const int tcount = ht.count, tmax = ht.maxc, tmin = ht.minc, tcm = ht.cm;
        const uint32_t tparty = ht.party;
        ncomb = 0;
        open.clear();
        while (g.head < g.n && sel[g.slot(g.head)]) g.head++;
        for (uint32_t i = g.head;; i++) {
            if (i >= g.n) {
                if (g.complete) break;
                if (!can_fetch) return EXHAUSTED;
                fetch_more(g);
                if (i >= g.n) { if (g.complete) break; i--; continue; }
            }
            if (i + kPrefetch < g.n) {  // the walk's next slots
                const uint32_t P = g.slot(i + kPrefetch);
                __builtin_prefetch(&sel[P]);
                __builtin_prefetch(&v.hot[P]);
            }
            const uint32_t H = g.slot(i);
            hits_seen++;
            if (H == T || sel[H]) continue;
            const HotRec& hh = v.hot[H];
            if (tparty != kNoParty && hh.party == tparty) continue;                       // :80-85
            if (rev && !g.rev_at(i)) continue;                                         // :139-148
            if (tmax < hh.maxc && v.intervals[H] + (proc ? proc[H] : 0) <= max_intervals) continue;  // :150-153
            if (!v.sessions_exclusive && (ht.smask & hh.smask) && share_session(ht, hh)) continue;  // :155-165
            bool sconf = false;  // sticky across combos of this hit (:156, :174-176, :206)
            int found = -1;
            const int hcount = hh.count;
            const uint32_t hp = hh.pres_off;
            size_t w = 0, r = 0;  // first fit over the open combos, dropping full ones on the way
            for (; r < open.size(); r++) {
                const uint32_t ci = open[r];
                auto& combo = combos[ci];
                if ((int)combo.size() + tcount >= tmax) continue;  // full for good
                open[w++] = ci;
                if ((int)combo.size() + hcount + tcount <= tmax) {
                    bool mconf = false;
                    const bool may_share = !v.sessions_exclusive && (cmask[ci] & hh.smask) != 0;
                    if (may_share || rev) for (const CE& e : combo) {
                        if (may_share && has_session(hh, e.sess)) { sconf = true; break; }
                        if (rev) {
                            if (!pair_ok(g, i, e.lpos)) { mconf = true; break; }
                            if (v.live[e.slot] && !pair_ok(g, e.lpos, i)) { mconf = true; break; }
                        }
                    }
                    if (sconf || mconf) continue;
                    for (int k = 0; k < hcount; k++)
                        combo.push_back(CE{H, (uint32_t)k, i, hcount == 1 ? hh.sess0 : v.pres_sess[hp + k]});
                    cmask[ci] |= hh.smask;
                    found = (int)ci;
                    r++;
                    break;
                }
            }
            for (; r < open.size(); r++) open[w++] = open[r];
            open.resize(w);
            if (found < 0) {
                if (ncomb == combos.size()) {
                    combos.emplace_back();
                    cmask.push_back(0);
                }
                std::vector<CE>& nc = combos[ncomb];
                nc.clear();
                for (int k = 0; k < hcount; k++) nc.push_back(CE{H, (uint32_t)k, i, hcount == 1 ? hh.sess0 : v.pres_sess[hp + k]});
                cmask[ncomb] = hh.smask;
                found = (int)ncomb++;
                if (hcount + tcount < tmax) open.push_back((uint32_t)found);
            }
            std::vector<CE>& fc = combos[found];
            int l = (int)fc.size() + tcount;
            bool form = l == tmax;
            if (!form && last && l >= tmin && l <= tmax) {
                int more = more_hits_after(g, i, T, can_fetch);
                if (more < 0) return EXHAUSTED;
                form = more == 0;
            }
            if (!form) continue;
            const int rem = l % tcm;
            if (rem != 0) {                                                                // :234-280
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
            bool failed = false;                                                           // :287-296
            int32_t last_cm = 0;  // l % cm for the previous entry's cm (entries mostly share one)
            bool last_ok = true;
            for (const CE& e : fc) {
                const uint32_t s = e.slot;
                const HotRec& hs = v.hot[s];
                if (!v.live[s]) continue;
                if (hs.minc > l || hs.maxc < l) { failed = true; break; }
                if (hs.cm != last_cm) { last_cm = hs.cm; last_ok = multiple_of(l, hs.cm); }
                if (!last_ok) { failed = true; break; }
            }
            if (failed) continue;
            group_out.clear();
            for (const CE& e : fc) group_out.push_back({e.slot, (int)e.pi});
            for (int k = 0; k < tcount; k++) group_out.push_back({T, k});
            return MATCHED;
        }
        return NOMATCH;
    }
};

// One pool's share of a parallel replay: a record per processed row, in row
// order, and the matched groups' entries.
struct PoolRec {
    uint32_t bi;  // batch row (UINT32_MAX: the list's end sentinel)
    uint8_t matched, expired;
    uint32_t off, len;  // into PoolOut::ents (off: entries before this row)
    uint32_t gcum, xcum;  // matched / expired rows before this one
};
// Over-aligned: the workers of a parallel replay fill different pools'
// outputs at once, and vector headers sharing a cache line would bounce
// between their cores on every push_back.
struct alignas(128) PoolOut {
    std::vector<PoolRec> recs;
    std::vector<std::pair<uint32_t, int>> ents;
};

// Replays one pool's rows (batch rows `bis`, ascending; slot brow[bi]):
// group_of(bi) gives the row's search.  `psel` and `proc` start all zero and
// are restored to zero on return (the caller's thread keeps them across
// tasks).  Appends the records + a sentinel to `o`.  A row whose truncated
// list runs out (EXHAUSTED: its search must re-run after the batch) stops the
// pool there: returns its batch row, else UINT32_MAX.
template <class GroupOf>
uint32_t replay_pool(ReplayCore& rp, const uint32_t* bis, size_t nbis, const uint32_t* brow, GroupOf group_of,
                     std::vector<uint8_t>& psel, uint8_t* proc, const int32_t* minc, const int32_t* maxc, PoolOut& o) {
    static thread_local std::vector<std::pair<uint32_t, int>> grp;  // (C5: 10^5 pools of 8 rows per pass)
    uint32_t gcum = 0, xcum = 0, stop = UINT32_MAX;
    rp.proc = proc;
    for (size_t j = 0; j < nbis; j++) {
        const uint32_t bi = bis[j];
        const uint32_t T = brow[bi];
        if (psel[T]) continue;
        auto status = rp.decide(T, group_of(bi), false, grp);
        if (status == ReplayCore::EXHAUSTED) {
            stop = bi;
            break;
        }
        proc[T] = 1;
        PoolRec rec{bi, 0, (uint8_t)(rp.v.intervals[T] + 1 >= rp.max_intervals || minc[T] == maxc[T]),
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
        o.recs.push_back(rec);
    }
    for (auto& e : o.ents) psel[e.first] = 0;
    for (const PoolRec& r : o.recs) proc[brow[r.bi]] = 0;
    o.recs.push_back(PoolRec{UINT32_MAX, 0, 0, (uint32_t)o.ents.size(), 0, gcum, xcum});  // sentinel
    return stop;
}
template <class GroupOf>
uint32_t replay_pool(ReplayCore& rp, const std::vector<uint32_t>& bis, const uint32_t* brow, GroupOf group_of,
                     std::vector<uint8_t>& psel, uint8_t* proc, const int32_t* minc, const int32_t* maxc, PoolOut& o) {
    return replay_pool(rp, bis.data(), bis.size(), brow, group_of, psel, proc, minc, maxc, o);
}

// ---- dense pool replay (a pool with one complete search, no RevPrecision) ----
//
// The same loop body as ReplayCore::row, but every per-ticket field the walk
// reads is first gathered into arrays indexed by list position (in parallel
// chunks), so the walk streams contiguous memory instead of chasing slots
// through the store.  Output is identical to replay_pool over the same list
// (tools/replay_bench.cpp checks it; tests/test_gpu_parity.py checks the
// parallel paths against the serial one).
//
// (A pool's walk is not cut into speculative segments.  A walk is "empty"
// at row j — nothing before j unselected, nothing after it selected — only
// where the position prefix holds a multiple of the gcd of the allowed group
// sizes (10 on C3), so a segment must start at such a row to ever meet the
// exact walk; cut there, every C3 segment joined within a few rows, but the
// segment walks compete with the gathers for the process's 16 CPUs and the
// pass got slower: DESIGN.md §9, profiles/r03t_spec_ab.txt.)

// The per-position fields every walk reads (24 B: 2.7 records per cache line,
// none straddling two when aligned in threes).  The exact walk's session
// fields (HotRec's sess0 / pres_off / smask) are read from the store through
// the position's slot: only step() needs them, and not gathering them saves
// the gather 12 of its 40 written bytes per position.
#ifdef NKM_WALK_STATS
inline uint64_t g_walk_stats[8];
#define NKM_WS(k) (g_walk_stats[k]++)
#else
#define NKM_WS(k) ((void)0)
#endif
struct DenseRec {
    int32_t count, minc, maxc, cm;
    uint32_t party;
    // Intervals (< 2^31) | the ticket's live_ flag << 31 (live_ is constant
    // during a pass: mutators queue), read with the record
    uint32_t ivl_live;
    uint32_t intervals() const { return ivl_live & 0x7fffffffu; }
    bool live() const { return (ivl_live >> 31) != 0; }
};

// One pool's per-position copies (filled by gather, in parallel chunks).
struct DensePool {
    const uint32_t* sp = nullptr;  // the list's slots (BGroup::slot)
    uint32_t ss = 4;
    uint32_t n = 0;
    uint32_t src_len = 0;  // the pool's search source (pairs decided per row that searches)
    const uint32_t* bis = nullptr;  // the pool's batch rows, ascending
    uint32_t nrows = 0;
    const uint32_t* brow = nullptr;  // batch row -> slot
    std::vector<DenseRec> rec;
    std::vector<uint32_t> slot;
    bool rows_list = false;  // BGroup::rows_list: position k's slot is brow[bis[k]], sp unfilled
    // identity: the pool's rows are its list, in list order (row j's ticket is
    // position j — every pool member searches, batch order = scan order, as in
    // a pool of fresh tickets): no slot -> position map is needed
    bool identity = false;
    // pipelined gather (identity pools): pieces [0, *front) of `pieces` are
    // gathered; null: the whole list is gathered before the walk
    const std::atomic<uint32_t>* front = nullptr;
    uint32_t pieces = 1;
    // set when another task of the pipelined job failed: a walk waiting for a
    // gather piece that will never come throws instead of spinning
    const std::atomic<bool>* abort = nullptr;

    void reset(const BGroup& g, const uint32_t* rows, uint32_t n_rows, const uint32_t* batch_slots) {
        sp = g.sp;
        ss = g.ss;
        n = g.n;
        src_len = g.d.src_len;
        rows_list = g.rows_list;
        bis = rows;
        nrows = n_rows;
        brow = batch_slots;
        identity = false;
        front = nullptr;
        abort = nullptr;
        pieces = 1;
        if (rec.size() < n) rec.resize(n);
        if (slot.size() < n) slot.resize(n);
    }
    uint32_t piece_lo(uint32_t t) const { return t >= pieces ? n : (uint32_t)((uint64_t)n * t / pieces); }
    // the gathered bound once position i (< n) is gathered (spins meanwhile)
    uint32_t wait_pos(uint32_t i) const {
        for (;;) {
            const uint32_t f = front->load(std::memory_order_acquire);
            const uint32_t a = piece_lo(f);
            if (i < a) return a;
            if (abort && abort->load(std::memory_order_relaxed)) throw std::runtime_error("parallel replay: a task failed");
            __builtin_ia32_pause();
        }
    }
    // does row j's ticket sit at list position j for every row? (positions [lo, hi))
    bool rows_are_list(uint32_t lo, uint32_t hi) const {
        if (rows_list) return true;
        for (uint32_t k = lo; k < hi; k++)
            if (sp[(size_t)k * ss] != brow[bis[k]]) return false;
        return true;
    }
    // positions [lo, hi): records, slots, and (unless identity) pos_of[slot] = position
    void gather(const ReplayView& v, uint32_t lo, uint32_t hi, uint32_t* pos_of) {
        const bool map = !identity;
        for (uint32_t k = lo; k < hi; k++) {
            const uint32_t s = rows_list ? brow[bis[k]] : sp[(size_t)k * ss];
            if (k + 16 < hi) {
                const uint32_t p = rows_list ? brow[bis[k + 16]] : sp[(size_t)(k + 16) * ss];
                __builtin_prefetch(&v.hot[p]);
                __builtin_prefetch(&v.intervals[p]);
                __builtin_prefetch(&v.live[p]);
                if (map) __builtin_prefetch(&pos_of[p], 1);
            }
            const HotRec& h = v.hot[s];
            rec[k] = DenseRec{h.count, h.minc, h.maxc, h.cm, h.party,
                              (uint32_t)v.intervals[s] | (v.live[s] ? 0x80000000u : 0u)};
            slot[k] = s;
            if (map) pos_of[s] = k;
        }
    }
    void clear_pos(uint32_t lo, uint32_t hi, uint32_t* pos_of) const {
        if (identity) return;
        for (uint32_t k = lo; k < hi; k++) pos_of[slot[k]] = kNoSlot;
    }
};

// The state and output of one walk over a range of a pool's rows.
struct DenseRun {
    std::vector<uint8_t> sel, proc;  // by position
    uint32_t head = 0;               // positions before head are all selected
    // output: one record per processed row, and the matched groups' entries
    std::vector<PoolRec> recs;
    std::vector<std::pair<uint32_t, int>> ents;
    uint64_t hits_seen = 0;
    uint32_t g_run = 0, x_run = 0;  // matched / expired records so far (PoolRec::gcum / xcum)
    // scratch
    std::vector<std::vector<CE>> combos;
    std::vector<uint32_t> cmask;
    std::vector<uint32_t> open;  // combos with room (ReplayCore::open)
    std::vector<std::pair<uint32_t, int>> grp;
    FastCombos fcb;
    bool fast = true;  // fast_step() for the rows it covers (NKM_FAST=0: step() only)
    uint32_t avail = 0;  // positions known gathered (pipelined gather, DensePool::front)

    // position i (< P.n) gathered before its copies are read
    __attribute__((always_inline)) void need(const DensePool& P, uint32_t i) {
        if (i >= avail) avail = P.wait_pos(i);
    }
    // row j's ticket T and its position kT.  An identity pool's row j is
    // position j (checked position by position, or proven, before any walk:
    // replay_parallel): T is the gathered copy's slot, read in sequence
    // instead of through the batch rows (a cache miss per row when the pools
    // interleave: C4's 64).  Else the gather's slot -> position map.
    __attribute__((always_inline)) void row_at(const DensePool& P, const uint32_t* pos_of, uint32_t j, uint32_t& T, uint32_t& kT) {
        if (P.identity) {
            need(P, j);
            T = P.slot[j];
            kT = j;
        } else {
            T = P.brow[P.bis[j]];
            kT = pos_of[T];
        }
    }

    void reset(uint32_t n) {
        sel.assign(n, 0);
        proc.assign(n, 0);
        head = 0;
        recs.clear();
        ents.clear();
        hits_seen = 0;
        g_run = x_run = 0;
    }

    // processDefault's loop body for row index j (ReplayCore::row over the
    // dense copies).  Returns false when the row's ticket is already selected.
    bool step(const DensePool& P, const ReplayView& v, int max_intervals, const uint32_t* pos_of, uint32_t j) {
        const uint32_t n = P.n;
        const uint32_t bi = P.bis[j];
        uint32_t T, kT;
        row_at(P, pos_of, j, T, kT);
        if (kT != kNoSlot && sel[kT]) return false;
        DenseRec rt;
        const HotRec& rc = v.hot[T];  // the session fields
        const uint32_t* tpres = v.pres_sess;
        if (kT != kNoSlot) {
            rt = P.rec[kT];
        } else {
            rt = DenseRec{rc.count, rc.minc, rc.maxc, rc.cm, rc.party,
                          (uint32_t)v.intervals[T] | (v.live[T] ? 0x80000000u : 0u)};
        }
        const bool last = (int)rt.intervals() + 1 >= max_intervals || rt.minc == rt.maxc;
        const int tcount = rt.count, tmax = rt.maxc, tmin = rt.minc, tcm = rt.cm;
        const uint32_t tparty = rt.party;
        auto t_has = [&](uint32_t sess) {
            if (tcount == 1) return rc.sess0 == sess;
            for (int q = 0; q < tcount; q++)
                if (tpres[rc.pres_off + q] == sess) return true;
            return false;
        };
        auto h_has = [&](const DenseRec& h, const HotRec& c, uint32_t sess) {
            if (h.count == 1) return c.sess0 == sess;
            for (int q = 0; q < h.count; q++)
                if (v.pres_sess[c.pres_off + q] == sess) return true;
            return false;
        };
        size_t ncomb = 0;
        open.clear();  // combos with room (see ReplayCore::open)
        while (head < n && sel[head]) head++;
        bool matched = false;
        for (uint32_t i = head; i < n; i++) {
            hits_seen++;
            if (i == kT || sel[i]) continue;
            need(P, i);
            const DenseRec& hh = P.rec[i];
            const HotRec& hc0 = v.hot[P.slot[i]];  // session fields only
            if (tparty != kNoParty && hh.party == tparty) continue;                      // :80-85
            if (tmax < hh.maxc && (int)hh.intervals() + proc[i] <= max_intervals) continue;  // :150-153
            if (!v.sessions_exclusive && (rc.smask & hc0.smask)) {                       // :155-165
                bool shared = false;
                if (hh.count == 1) shared = t_has(hc0.sess0);
                else
                    for (int q = 0; q < hh.count && !shared; q++) shared = t_has(v.pres_sess[hc0.pres_off + q]);
                if (shared) continue;
            }
            bool sconf = false;  // sticky across combos of this hit (:156, :174-176, :206)
            int found = -1;
            const int hcount = hh.count;
            size_t w = 0, r = 0;
            for (; r < open.size(); r++) {
                const uint32_t ci = open[r];
                auto& combo = combos[ci];
                if ((int)combo.size() + tcount >= tmax) continue;  // full for good
                open[w++] = ci;
                if ((int)combo.size() + hcount + tcount <= tmax) {
                    if (!v.sessions_exclusive && (cmask[ci] & hc0.smask))
                        for (const CE& e : combo)
                            if (h_has(hh, hc0, e.sess)) { sconf = true; break; }
                    if (sconf) continue;
                    for (int k = 0; k < hcount; k++)
                        combo.push_back(CE{P.slot[i], (uint32_t)k, i, hcount == 1 ? hc0.sess0 : v.pres_sess[hc0.pres_off + k]});
                    cmask[ci] |= hc0.smask;
                    found = (int)ci;
                    r++;
                    break;
                }
            }
            for (; r < open.size(); r++) open[w++] = open[r];
            open.resize(w);
            if (found < 0) {
                if (ncomb == combos.size()) {
                    combos.emplace_back();
                    cmask.push_back(0);
                }
                std::vector<CE>& nc = combos[ncomb];
                nc.clear();
                for (int k = 0; k < hcount; k++)
                    nc.push_back(CE{P.slot[i], (uint32_t)k, i, hcount == 1 ? hc0.sess0 : v.pres_sess[hc0.pres_off + k]});
                cmask[ncomb] = hc0.smask;
                found = (int)ncomb++;
                if (hcount + tcount < tmax) open.push_back((uint32_t)found);
            }
            std::vector<CE>& fc = combos[found];
            int l = (int)fc.size() + tcount;
            bool form = l == tmax;
            if (!form && last && l >= tmin && l <= tmax) {
                bool more = false;  // an unselected, non-self, non-party hit after i (:130, :233)
                for (uint32_t q = i + 1; q < n && !more; q++) {
                    if (q == kT || sel[q]) continue;
                    need(P, q);
                    more = !(tparty != kNoParty && P.rec[q].party == tparty);
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
            int32_t last_cm = 0;
            bool last_ok = true;
            for (const CE& e : fc) {
                const DenseRec& hs = P.rec[e.lpos];
                if (!hs.live()) continue;
                if (hs.minc > l || hs.maxc < l) { failed = true; break; }
                if (hs.cm != last_cm) { last_cm = hs.cm; last_ok = multiple_of(l, hs.cm); }
                if (!last_ok) { failed = true; break; }
            }
            if (failed) continue;
            grp.clear();
            for (const CE& e : fc) {
                grp.push_back({e.slot, (int)e.pi});
                sel[e.lpos] = 1;
            }
            for (int k = 0; k < tcount; k++) grp.push_back({T, k});
            if (kT != kNoSlot) sel[kT] = 1;
            matched = true;
            break;
        }
        if (kT != kNoSlot) proc[kT] = 1;
        recs.push_back(PoolRec{bi, (uint8_t)matched, (uint8_t)last, (uint32_t)ents.size(),
                               matched ? (uint32_t)grp.size() : 0u, g_run, x_run});
        g_run += matched;
        x_run += last;
        if (matched) ents.insert(ents.end(), grp.begin(), grp.end());
        return true;
    }

    // step() when no two live tickets share a session: combos are member
    // positions + entry counts.  Returns 0 (row already selected), 1 (done),
    // or 2 when the row reaches the CountMultiple trim or outgrows the fixed
    // combos — nothing changed but the head; step() then decides the row.
    int fast_step(const DensePool& P, const ReplayView& v, int max_intervals, const uint32_t* pos_of, uint32_t j) {
        // Members used in the loops are read into locals first: `sel` is a
        // byte array, and a char-typed load may alias any member, so member
        // counters (hits_seen, head, avail) would otherwise be stored and
        // reloaded around every one (the box's PMU: 1,043 instructions per
        // processed C3 row, 5.8 branch misses; tools/replay_bench RB_PERF=1)
        const uint32_t n = P.n;
        const uint32_t bi = P.bis[j];
        uint32_t T, kT;
        row_at(P, pos_of, j, T, kT);
        const uint8_t* const S = sel.data();
        if (kT != kNoSlot && S[kT]) return 0;
        const DenseRec* const R = P.rec.data();
        int32_t tcount, tmin, tmax, tcm;
        uint32_t tparty, tivl;
        if (kT != kNoSlot) {
            const DenseRec& r = R[kT];
            tcount = r.count; tmin = r.minc; tmax = r.maxc; tcm = r.cm; tparty = r.party; tivl = r.intervals();
        } else {
            const HotRec& h = v.hot[T];
            tcount = h.count; tmin = h.minc; tmax = h.maxc; tcm = h.cm; tparty = h.party;
            tivl = (uint32_t)v.intervals[T];
        }
        const bool last = (int)tivl + 1 >= max_intervals || tmin == tmax;
        const int room = tmax - tcount;
        const uint8_t* const pr = proc.data();
        uint32_t av = avail;
        auto ready = [&](uint32_t i) {
            if (i >= av) av = P.wait_pos(i);
        };
        uint32_t h0 = head;
        // the selected run after the head (the last group's members, ~6 on
        // C3) skipped 8 bytes a time: the first unselected byte of a word is
        // its lowest zero (selection bytes are 0 / 1), so the scan ends
        // without a data-dependent branch per byte
        while (h0 + 8 <= n) {
            uint64_t w;
            std::memcpy(&w, S + h0, 8);
            const uint64_t z = ~w & 0x0101010101010101ull;  // bit 8k: byte k is 0
            NKM_WS(0);
            if (z) {
                h0 += (uint32_t)(__builtin_ctzll(z) >> 3);
                break;
            }
            h0 += 8;
        }
        while (h0 < n && S[h0]) { h0++; NKM_WS(0); }
        head = h0;
        int32_t* const csize = fcb.size;
        uint32_t* const cnmem = fcb.nmem;
        int ncomb = 0, fi = -1;
        uint64_t seen = 0;
        bool bail = false;
        for (uint32_t i = h0; i < n; i++) {
            seen++;
            if (i == kT || S[i]) continue;
            ready(i);
            const DenseRec& hh = R[i];
            if (tparty != kNoParty && hh.party == tparty) continue;                    // :80-85
            if (tmax < hh.maxc && (int)hh.intervals() + pr[i] <= max_intervals) continue;  // :150-153
            const int hc = hh.count;
            int f = 0;  // first fit (:167-226)
            while (f < ncomb && csize[f] + hc > room) { f++; NKM_WS(1); }
            NKM_WS(2);
            if (f == ncomb) {
                if (f == kFastComb) { bail = true; break; }
                csize[f] = 0;
                cnmem[f] = 0;
                ncomb++;
            } else if (cnmem[f] == (uint32_t)kFastMem) {
                bail = true;
                break;
            }
            const int sz = csize[f] + hc;
            csize[f] = sz;
            fcb.mem[f][cnmem[f]++] = i;
            const int l = sz + tcount;
            bool form = l == tmax;  // :233
            if (!form && last && l >= tmin && l <= tmax) {
                bool more = false;
                for (uint32_t q = i + 1; q < n && !more; q++) {
                    if (q == kT || S[q]) continue;
                    ready(q);
                    more = !(tparty != kNoParty && R[q].party == tparty);
                }
                form = !more;
            }
            if (!form) continue;
            if (!multiple_of(l, tcm)) { bail = true; break; }  // the CountMultiple trim: step()
            bool failed = false;                                 // :287-296
            const uint32_t* mem = fcb.mem[f];
            for (uint32_t k = 0, nm = cnmem[f]; k < nm && !failed; k++) {
                NKM_WS(3);
                const DenseRec& hs = R[mem[k]];
                if (!hs.live()) continue;
                failed = hs.minc > l || hs.maxc < l || !multiple_of(l, hs.cm);
            }
            if (failed) continue;
            fi = f;
            break;
        }
        hits_seen += seen;
        avail = av;
        if (bail) return 2;
        const uint32_t off = (uint32_t)ents.size();
        if (fi >= 0) {
            const uint32_t* mem = fcb.mem[fi];
            const uint32_t nm = cnmem[fi];
            // entries first, the selection bytes after (a byte store between
            // push_backs would make the vector's end pointer reload each time)
            for (uint32_t k = 0; k < nm; k++) {
                const uint32_t m = mem[k];
                const uint32_t s = P.slot[m];
                for (int e = 0, c = R[m].count; e < c; e++) ents.push_back({s, e});
            }
            for (int e = 0; e < tcount; e++) ents.push_back({T, e});
            uint8_t* const W = sel.data();
            for (uint32_t k = 0; k < nm; k++) W[mem[k]] = 1;
            if (kT != kNoSlot) W[kT] = 1;
        }
        if (kT != kNoSlot) proc[kT] = 1;
        recs.push_back(PoolRec{bi, (uint8_t)(fi >= 0), (uint8_t)last, off, (uint32_t)ents.size() - off, g_run, x_run});
        g_run += fi >= 0;
        x_run += last;
        return 1;
    }

    // An identity pool's row j is list position j: the rows an earlier row's
    // group selected (C3: ~5 of every 6) are skipped by scanning `sel` (eight
    // at a time) up to `end`, without a step call each.  Returns the first
    // row at or after j that is unselected, or `end`.
    uint32_t skip_selected(const DensePool& P, uint32_t j, uint32_t end) const {
        if (!P.identity) return j;
        const uint8_t* s = sel.data();
        while (j < end && s[j]) {
            NKM_WS(4);
            uint64_t w;
            while (j + 8 <= end && (std::memcpy(&w, s + j, 8), w == 0x0101010101010101ull)) j += 8;
            while (j < end && s[j]) j++;
        }
        return j;
    }

    void walk(const DensePool& P, const ReplayView& v, int max_intervals, const uint32_t* pos_of, uint32_t j0,
              uint32_t j1) {
        avail = P.front ? 0 : P.n;
        const bool f = fast && v.sessions_exclusive;
        for (uint32_t j = skip_selected(P, j0, j1); j < j1; j = skip_selected(P, j + 1, j1))
            if (!f || fast_step(P, v, max_intervals, pos_of, j) == 2) step(P, v, max_intervals, pos_of, j);
    }

    // walk() over all rows that records, for every merge chunk boundary
    // bnd[c] (batch rows, ascending; c < nbnd), the number of records of the
    // pool's rows before it — cut[c] — and publishes the count of boundaries
    // passed (release) for the pipelined merge, which then reads its chunk's
    // records [cut[c-1], cut[c]) with no search.  The caller reserved recs and
    // ents so that neither reallocates under the readers.
    void walk_cuts(const DensePool& P, const ReplayView& v, int max_intervals, const uint32_t* pos_of,
                   const uint32_t* bnd, uint32_t nbnd, uint32_t* cut, std::atomic<uint32_t>* ncut) {
        avail = P.front ? 0 : P.n;
        const bool f = fast && v.sessions_exclusive;
        uint32_t nc = 0, next = nbnd ? bnd[0] : UINT32_MAX;
        auto pass = [&](uint32_t j) {  // the rows before j are done
            const uint32_t b = j < P.nrows ? P.bis[j] : UINT32_MAX;
            if (b < next) return;
            const uint32_t r = (uint32_t)recs.size();
            do cut[nc++] = r;
            while (nc < nbnd && b >= bnd[nc]);
            next = nc < nbnd ? bnd[nc] : UINT32_MAX;
            ncut->store(nc, std::memory_order_release);
        };
        for (uint32_t j = skip_selected(P, 0, P.nrows); j < P.nrows; j = skip_selected(P, j + 1, P.nrows)) {
            pass(j);
            if (!f || fast_step(P, v, max_intervals, pos_of, j) == 2) step(P, v, max_intervals, pos_of, j);
        }
        if (nc < nbnd) pass(P.nrows);
    }

    // Hands the records to a PoolOut (running offsets/counts, sentinel).
    void finish(PoolOut& o) {
        uint32_t g = 0, x = 0, off = 0;
        for (PoolRec& r : recs) {
            r.off = off;
            r.gcum = g;
            r.xcum = x;
            off += r.len;
            g += r.matched;
            x += r.expired;
        }
        recs.push_back(PoolRec{UINT32_MAX, 0, 0, off, 0, g, x});
        o.recs.swap(recs);
        o.ents.swap(ents);
    }
};

}  // namespace nkm
