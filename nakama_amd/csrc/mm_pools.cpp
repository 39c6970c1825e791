// nakama_amd/csrc/mm_pools.cpp — the pool-parallel replay (plan_pools,
// replay_parallel and the merges back into the pinned row order) and the
// packed RevPrecision batches (assembly, rpack_kernel's launch, per-row
// views).  Part of Core's pass (mm_process.cpp).
#include <sched.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <stdexcept>
#include <thread>
#include <unordered_set>
#include <cstdlib>
#include <cstring>
#include <map>
#include "gocompat.h"
#include "mm_core.h"
#include "mm_pass.h"

namespace nkm {

// Pool-parallel replay.  When every search of the batch draws its hits from a
// posting list of the same field with a distinct term, every searching ticket
// carries its own search's term, and every list is complete, then each
// search's rows only ever select tickets of its own posting list: the greedy
// pass decomposes exactly into independent per-pool passes (processDefault's
// sequential order is preserved within each pool, and no ticket is shared
// across pools).  The pools run on host threads; results are merged back into
// the pinned row order.  Returns false (nothing done) when the conditions fail.
// The part of the pool-parallel replay that needs no hit list — the pool
// keys and the rows bucketed per pool — run while the batch's searches are
// on the device.  Returns false when the batch does not partition into pools.
bool Core::plan_parallel(const std::vector<BGroup>& bg, const UVec<uint32_t>& brow,
                         const UVec<uint32_t>& brow_group, ParPlan& P, PassStats& stats) {
    return plan_pools(
        bg.size(), [&](size_t i) { return bg[i].sig; }, [&](size_t bi) { return brow_group[bi]; },
        [&](size_t i) { return bg[i].row_slot; }, brow, P, stats);
}

// plan_fused: the rows are bucketed per search already (assemble_parallel,
// which also checked that every row carries its own search's terms); the
// searches are the pools when their keys — their MUST terms on the fields
// every search requires a term on — are pairwise distinct.  Only the
// searches are read here (C3: 8), not the rows.  Otherwise plan_parallel.
bool Core::plan_fused(const std::vector<BGroup>& bg, const UVec<uint32_t>& brow, const UVec<uint32_t>& brow_group,
                      ParPlan& P, PassStats& stats) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const size_t G = bg.size();
    P.ok = false;
    P.runs = false;
    std::vector<uint16_t> keyf;
    for (auto& mt : sigs_[bg[0].sig].must_terms)
        if (std::find(keyf.begin(), keyf.end(), mt.first) == keyf.end()) keyf.push_back(mt.first);
    for (size_t i = 1; i < G && !keyf.empty(); i++) {
        const auto& mts = sigs_[bg[i].sig].must_terms;
        keyf.erase(std::remove_if(keyf.begin(), keyf.end(),
                                  [&](uint16_t f) {
                                      return std::none_of(mts.begin(), mts.end(), [&](const std::pair<uint16_t, uint32_t>& m) {
                                          return m.first == f;
                                      });
                                  }),
                   keyf.end());
    }
    bool ok = !keyf.empty();
    for (uint16_t f : keyf) ok = ok && fkind_[f].size() == nslots();
    std::vector<std::vector<uint32_t>> key(G, std::vector<uint32_t>(keyf.size(), UINT32_MAX));
    for (size_t i = 0; i < G && ok; i++)
        for (auto& mt : sigs_[bg[i].sig].must_terms)
            for (size_t k = 0; k < keyf.size(); k++)
                if (mt.first == keyf[k]) {
                    if (key[i][k] != UINT32_MAX && key[i][k] != mt.second) ok = false;  // two terms on one field
                    key[i][k] = mt.second;
                }
    if (ok) {
        std::vector<uint32_t> ord(G);
        for (uint32_t i = 0; i < G; i++) ord[i] = i;
        std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
        for (size_t i = 1; i < G && ok; i++) ok = key[ord[i]] != key[ord[i - 1]];
    }
    if (!ok) return plan_parallel(bg, brow, brow_group, P, stats);
    P.ng = G;
    grow_to(P.search_pool, G);
    for (uint32_t i = 0; i < G; i++) P.search_pool[i] = i;
    P.self_rows.assign(G, 1);
    if (keyf.size() == 1) {
        grow_to(P.pool_key1, G);
        for (size_t i = 0; i < G; i++) P.pool_key1[i] = key[i][0];
    } else {
        P.pool_key1.clear();
    }
    P.ok = true;
    stats.par_bucket_ms += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    if (batch_profile_) std::fprintf(stderr, "[nkm]   plan_fused: %zu pools (the assembly's buckets)\n", G);
    return true;
}

// plan_parallel over `nsearch` searches: sig_of(i) is search i's signature,
// group_of(bi) batch row bi's search (a packed RevPrecision batch: the row
// itself), row_of(i) the slot of a one-row search (RevPrecision) or kNoSlot.
// Every step is a parallel sweep over the searches or the rows; the pools are
// numbered in first-appearance order (C5: 125k pools per 1M rows).  A one-row
// search whose ticket carries its own search's terms (self_match_) takes its
// pool key from its own column, not from the signature's term list.
template <class SigOf, class GroupOf, class RowOf>
bool Core::plan_pools(size_t nsearch, SigOf sig_of, GroupOf group_of, RowOf row_of, const UVec<uint32_t>& brow,
                      ParPlan& P, PassStats& stats) {
    P.ok = false;
    P.runs = false;
    if (nsearch < 2) return false;
    using clk = std::chrono::steady_clock;
    auto msd = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto tp0 = clk::now();
    WorkPool& wp = workers();
    const bool par = nsearch >= par_min(65536) && par_mode_;
    const unsigned nsch = par ? wp.size() * 2 : 1;
    auto sweep = [&](size_t n, unsigned nch, auto&& fn) {  // fn(chunk, lo, hi) over [0, n) in nch chunks
        if (nch > 1)
            wp.run(nch, [&](size_t c) { fn(c, n * c / nch, n * (c + 1) / nch); });
        else
            fn(0, 0, n);
    };
    // pool key fields: fields every search requires a keyword term on (the
    // candidates are the first search's; each chunk of searches checks them)
    std::vector<uint16_t> cand;
    for (auto& mt : sigs_[sig_of(0)].must_terms)
        if (std::find(cand.begin(), cand.end(), mt.first) == cand.end()) cand.push_back(mt.first);
    std::vector<std::vector<uint8_t>> has(nsch, std::vector<uint8_t>(cand.size(), 1));
    // fields below 63: the signatures' must-field masks (no term lists read)
    uint64_t cmask = 0;
    bool narrow = true;
    for (uint16_t f : cand) {
        if (f >= 63) narrow = false;
        else cmask |= 1ull << f;
    }
    std::vector<uint64_t> hmask(nsch, ~0ull);
    sweep(nsearch, nsch, [&](size_t ch, size_t lo, size_t hi) {
        if (narrow) {
            uint64_t m = cmask;
            for (size_t i = lo; i < hi && m; i++) m &= sig_fmask_[sig_of(i)];
            hmask[ch] = m;
            return;
        }
        for (size_t i = lo; i < hi; i++) {
            const auto& mts = sigs_[sig_of(i)].must_terms;
            for (size_t k = 0; k < cand.size(); k++) {
                if (!has[ch][k]) continue;
                bool h = false;
                for (auto& m2 : mts) h |= m2.first == cand[k];
                if (!h) has[ch][k] = 0;
            }
        }
    });
    if (narrow)
        for (unsigned ch = 0; ch < nsch; ch++)
            for (size_t k = 0; k < cand.size(); k++) has[ch][k] = (hmask[ch] >> cand[k]) & 1;
    std::vector<uint16_t> keyf;
    for (size_t k = 0; k < cand.size(); k++) {
        bool all = true;
        for (unsigned ch = 0; ch < nsch; ch++) all = all && has[ch][k];
        if (all) keyf.push_back(cand[k]);
    }
    if (keyf.empty()) return false;
    for (uint16_t f : keyf)
        if (fkind_[f].size() != nslots()) return false;
    // pool key of each search; a search requiring two different terms on one
    // field matches nothing (the batch then takes the serial replay).  One key
    // field (C5's buckets: ~10^5 pools): keys extracted on the workers and
    // pools numbered in parallel through dictionary-id tables; more fields
    // (mode x region: few pools): an ordered map.
    std::vector<uint32_t>& search_pool = P.search_pool;
    grow_to(search_pool, nsearch);
    std::vector<uint32_t>& pool_key1 = P.pool_key1;  // one key field: pool -> its term
    std::vector<std::vector<uint32_t>> pool_keys;    // several: pool -> its terms
    auto key_of = [&](size_t i, uint32_t* key) {
        for (size_t k = 0; k < keyf.size(); k++) key[k] = UINT32_MAX;
        for (size_t k = 0; k < keyf.size(); k++)
            for (auto& mt : sigs_[sig_of(i)].must_terms)
                if (mt.first == keyf[k]) {
                    if (key[k] != UINT32_MAX && key[k] != mt.second) return false;
                    key[k] = mt.second;
                }
        return true;
    };
    size_t ng = 0;
    if (keyf.size() == 1) {
        std::vector<uint32_t>& k1 = search_pool;  // the key term first, renumbered in place below
        std::vector<uint8_t> bad(nsch, 0);
        const size_t nd = dict_.size();
        // first[t]: the lowest search index with term t (atomic min over the
        // chunks); the heads (first[t] == i) are numbered in index order.
        // Every entry is UINT32_MAX between calls: the heads reset their own
        // on the way out, so a pass costs O(searches), not O(dictionary) (the
        // dictionary only grows: C5's bench adds 125k bucket terms a step)
        std::atomic<uint32_t>* first = pool_first_table(nd);
        std::vector<uint32_t>& tpool = pool_remap_;  // term -> pool (written by its head only)
        grow_to(tpool, nd);
        std::vector<size_t> heads(nsch + 1, 0);
        const uint16_t f0 = keyf[0];
        sweep(nsearch, nsch, [&](size_t ch, size_t lo, size_t hi) {
            uint32_t kk[4];
            for (size_t i = lo; i < hi; i++) {
                const uint32_t r = row_of(i);
                if (r != kNoSlot && self_match_[r] && indexed_[r] && sig_[r] == sig_of(i) &&
                    fkind_[f0][r] == KIND_KEYWORD)
                    kk[0] = (uint32_t)fval_[f0][r];  // the row carries its search's term on f0
                else if (!key_of(i, kk))
                    kk[0] = UINT32_MAX;
                if (kk[0] == UINT32_MAX || kk[0] >= nd) { bad[ch] = 1; return; }
                k1[i] = kk[0];
                uint32_t cur = first[kk[0]].load(std::memory_order_relaxed);
                while ((uint32_t)i < cur && !first[kk[0]].compare_exchange_weak(cur, (uint32_t)i, std::memory_order_relaxed)) {
                }
            }
        });
        if (std::any_of(bad.begin(), bad.end(), [](uint8_t b) { return b != 0; })) {
            sweep(pool_first_cap_, nsch, [&](size_t, size_t lo, size_t hi) {  // back to all-empty
                for (size_t t = lo; t < hi; t++) first[t].store(UINT32_MAX, std::memory_order_relaxed);
            });
            return false;
        }
        sweep(nsearch, nsch, [&](size_t ch, size_t lo, size_t hi) {
            size_t h = 0;
            for (size_t i = lo; i < hi; i++) h += first[k1[i]].load(std::memory_order_relaxed) == (uint32_t)i;
            heads[ch + 1] = h;
        });
        for (unsigned ch = 0; ch < nsch; ch++) heads[ch + 1] += heads[ch];
        ng = heads[nsch];
        grow_to(pool_key1, ng);
        sweep(nsearch, nsch, [&](size_t ch, size_t lo, size_t hi) {
            size_t p = heads[ch];
            for (size_t i = lo; i < hi; i++)
                if (first[k1[i]].load(std::memory_order_relaxed) == (uint32_t)i) {
                    tpool[k1[i]] = (uint32_t)p;
                    pool_key1[p++] = k1[i];
                }
        });
        sweep(nsearch, nsch, [&](size_t, size_t lo, size_t hi) {
            for (size_t i = lo; i < hi; i++) {
                const uint32_t t = k1[i];
                k1[i] = tpool[t];
                if (first[t].load(std::memory_order_relaxed) == (uint32_t)i)  // the head clears its term's entry
                    first[t].store(UINT32_MAX, std::memory_order_relaxed);
            }
        });
    } else {
        pool_key1.clear();
        std::map<std::vector<uint32_t>, uint32_t> pool_of;
        std::vector<uint32_t> key(keyf.size());
        for (size_t i = 0; i < nsearch; i++) {
            if (!key_of(i, key.data())) return false;
            auto it = pool_of.emplace(key, (uint32_t)pool_of.size());
            if (it.second) pool_keys.push_back(key);
            search_pool[i] = it.first->second;
        }
        ng = pool_keys.size();
    }
    if (ng < 2) return false;
    P.ng = ng;
    auto pool_key = [&](size_t p, size_t f) { return keyf.size() == 1 ? pool_key1[p] : pool_keys[p][f]; };
    // every searching ticket must itself belong to its search's pool: a row
    // not known to carry its own search's terms (self_match_) must hold the
    // pool's key values, and its pool is then not known to hold all its rows
    const size_t nb = brow.size();
    const unsigned nchunk = nb >= par_min(65536) ? wp.size() : 1;
    auto row_check = [&](size_t bi, uint32_t p) -> int {  // 0 self, 1 foreign, 2 not in its pool
        const uint32_t r = brow[bi];
        const uint32_t gi = group_of(bi);
        if (self_match_[r] && indexed_[r] && sig_[r] == sig_of(gi)) return 0;
        for (size_t f = 0; f < keyf.size(); f++)
            if (fkind_[keyf[f]][r] != KIND_KEYWORD || (uint32_t)fval_[keyf[f]][r] != pool_key(p, f)) return 2;
        return 1;
    };
    // Contiguous pools (C5: a bucket's tickets arrive together): when the row
    // pool ids never decrease and step by at most one (pools are numbered in
    // first appearance), every pool's rows are one run of the batch and the
    // batch is its own CSR — no counting sort.
    {
        const auto tq0 = clk::now();
        std::vector<uint8_t> ok(nchunk, 1), bad(nchunk, 0);
        std::vector<uint32_t> pfirst(nchunk, 0), plast(nchunk, 0);
        grow_to(P.self_rows, ng);
        sweep(ng, ng >= 65536 ? nchunk : 1, [&](size_t, size_t lo, size_t hi) {
            std::memset(P.self_rows.data() + lo, 1, hi - lo);
        });
        sweep(nb, nchunk, [&](size_t c, size_t lo, size_t hi) {
            if (lo >= hi) return;
            uint32_t prev = search_pool[group_of(lo)];
            pfirst[c] = prev;
            for (size_t bi = lo; bi < hi; bi++) {
                const uint32_t p = search_pool[group_of(bi)];
                if (p != prev && p != prev + 1) { ok[c] = 0; return; }
                prev = p;
                const int k = row_check(bi, p);
                if (k == 2) { bad[c] = 1; return; }
                if (k == 1) P.self_rows[p] = 0;  // benign: every writer stores 0
            }
            plast[c] = prev;
        });
        bool mono = nb > 0;
        for (unsigned c = 0; c < nchunk && mono; c++) {
            if (bad[c]) return false;
            mono = ok[c] != 0;
        }
        bool seen = false;
        uint32_t last = 0;
        for (unsigned c = 0; c < nchunk && mono; c++) {
            if (nb * c / nchunk >= nb * (c + 1) / nchunk) continue;  // an empty chunk
            if (seen) mono = pfirst[c] == last || pfirst[c] == last + 1;
            seen = true;
            last = plast[c];
        }
        mono = mono && search_pool[group_of(0)] == 0 && search_pool[group_of(nb - 1)] + 1 == ng;
        if (mono) {
            grow_to(P.pool_off, ng + 1);
            grow_to(P.pool_rows, nb);
            sweep(nb, nchunk, [&](size_t, size_t lo, size_t hi) {
                for (size_t bi = lo; bi < hi; bi++) {
                    P.pool_rows[bi] = (uint32_t)bi;
                    const uint32_t p = search_pool[group_of(bi)];
                    if (bi == 0 || search_pool[group_of(bi - 1)] != p) P.pool_off[p] = (uint32_t)bi;
                }
            });
            P.pool_off[ng] = (uint32_t)nb;
            stats.par_bucket_ms += msd(tp0, clk::now());
            if (batch_profile_)
                std::fprintf(stderr, "[nkm]   plan_pools: %zu pools (contiguous runs) | keys %.2f runs %.2f ms\n", ng,
                             msd(tp0, tq0), msd(tq0, clk::now()));
            P.ok = true;
            P.runs = true;
            return true;
        }
    }
    // otherwise the rows are bucketed per pool in batch order (CSR: per-chunk
    // counts, then every chunk scatters at its offsets; counters stay
    // thread-private)
    UVec<uint32_t>& cnt = pool_cnt_;  // [chunk][pool]: each chunk writes its row in full
    grow_to(cnt, (size_t)nchunk * ng);
    std::vector<uint8_t> cbad(nchunk, 0);
    // per (chunk, pool): a row that is not known to carry its own search's
    // terms (self_match_) — the pool is then not known to hold all its rows
    UVec<uint8_t>& cforeign = pool_foreign_;
    grow_to(cforeign, (size_t)nchunk * ng);
    const auto tp1 = clk::now();
    sweep(nb, nchunk, [&](size_t c, size_t lo, size_t hi) {
        // thread-private counters (few pools: the chunks' rows of cnt share
        // cache lines), copied out at the end
        static thread_local std::vector<uint32_t> k;
        static thread_local std::vector<uint8_t> fo;
        k.assign(ng, 0);
        fo.assign(ng, 0);
        for (size_t bi = lo; bi < hi; bi++) {
            const uint32_t p = search_pool[group_of(bi)];
            k[p]++;
            const int rc = row_check(bi, p);
            if (rc == 2) {
                cbad[c] = 1;
                return;
            }
            if (rc == 1) fo[p] = 1;
        }
        std::memcpy(cnt.data() + c * ng, k.data(), ng * sizeof(uint32_t));
        std::memcpy(cforeign.data() + c * ng, fo.data(), ng);
    });
    const auto tp2 = clk::now();
    for (unsigned c = 0; c < nchunk; c++)
        if (cbad[c]) return false;
    // per pool: rows and self flag (ranges of pools on the workers), the
    // pool offsets (one scan), then each (chunk, pool)'s first position
    grow_to(P.self_rows, ng);
    grow_to(P.pool_off, ng + 1);
    const unsigned npch = ng >= 65536 && nchunk > 1 ? nchunk : 1;
    sweep(ng, npch, [&](size_t, size_t lo, size_t hi) {
        for (size_t p = lo; p < hi; p++) {
            uint32_t t = 0;
            uint8_t f = 0;
            for (unsigned c = 0; c < nchunk; c++) {
                t += cnt[c * ng + p];
                f |= cforeign[c * ng + p];
            }
            P.pool_off[p + 1] = t;
            P.self_rows[p] = f ? 0 : 1;
        }
    });
    P.pool_off[0] = 0;
    for (size_t p = 0; p < ng; p++) P.pool_off[p + 1] += P.pool_off[p];
    sweep(ng, npch, [&](size_t, size_t lo, size_t hi) {
        for (size_t p = lo; p < hi; p++) {
            uint32_t run = P.pool_off[p];
            for (unsigned c = 0; c < nchunk; c++) {
                const uint32_t v = cnt[c * ng + p];
                cnt[c * ng + p] = run;
                run += v;
            }
        }
    });
    grow_to(P.pool_rows, nb);
    const auto tp3 = clk::now();
    sweep(nb, nchunk, [&](size_t c, size_t lo, size_t hi) {
        static thread_local std::vector<uint32_t> at;
        at.assign(cnt.begin() + c * ng, cnt.begin() + (c + 1) * ng);
        for (size_t bi = lo; bi < hi; bi++) P.pool_rows[at[search_pool[group_of(bi)]]++] = (uint32_t)bi;
    });
    const auto tp4 = clk::now();
    stats.par_bucket_ms += msd(tp0, tp4);
    if (batch_profile_)
        std::fprintf(stderr, "[nkm]   plan_pools: %zu pools | keys %.2f count %.2f offsets %.2f scatter %.2f ms\n", ng,
                     msd(tp0, tp1), msd(tp1, tp2), msd(tp2, tp3), msd(tp3, tp4));
    P.ok = true;
    return true;
}

// Pool-parallel replay over the bucketed rows (plan_parallel); false when a
// pool's list came back truncated (the serial replay then decides the batch).
// Pools are walked on the host workers (largest first, small ones bundled
// into tasks); every processed row leaves a record at its batch position, and
// one pass over the batch in row order assembles the groups, the expired list
// and the Intervals increments — processDefault's sequential order, because
// no pool ever selects another pool's ticket.
// A proven list's sp points at its reserved words in the library's pinned
// host list buffer (Core::h_out_, run_batch's cg_off), which the download
// would have filled: the batch rows are written there instead.
void Core::fill_row_lists(std::vector<BGroup>& bg, const UVec<uint32_t>& brow, const UVec<uint32_t>& brow_group) {
    if (!row_lists_pending_) return;
    row_lists_pending_ = false;
    std::vector<uint32_t> at(bg.size(), 0);
    for (size_t bi = 0; bi < brow.size(); bi++) {
        const uint32_t gi = brow_group[bi];
        BGroup& g = bg[gi];
        if (!g.rows_list) continue;
        if (at[gi] >= g.n || g.ss != 1) throw std::logic_error("fill_row_lists: a proven list is shorter than its rows");
        const_cast<uint32_t*>(g.sp)[at[gi]++] = brow[bi];
    }
    for (size_t gi = 0; gi < bg.size(); gi++) {
        if (bg[gi].rows_list && at[gi] != bg[gi].n) throw std::logic_error("fill_row_lists: a proven list is longer than its rows");
        bg[gi].rows_list = false;
    }
}

void Core::check_row_lists(const std::vector<BGroup>& bg, const UVec<uint32_t>& brow, const UVec<uint32_t>& brow_group) {
    if (!row_lists_pending_) return;
    std::vector<uint32_t> at(bg.size(), 0);
    for (size_t bi = 0; bi < brow.size(); bi++) {
        const uint32_t gi = brow_group[bi];
        const BGroup& g = bg[gi];
        if (!g.rows_list) continue;
        if (at[gi] >= g.n || g.slot(at[gi]) != brow[bi])
            throw std::logic_error("NKM_LISTPROOF=2: a proven mscan list differs from its search's rows");
        at[gi]++;
    }
    for (size_t gi = 0; gi < bg.size(); gi++)
        if (bg[gi].rows_list && at[gi] != bg[gi].n)
            throw std::logic_error("NKM_LISTPROOF=2: a proven mscan list is longer than its search's rows");
}

bool Core::replay_parallel(const ParPlan& P, std::vector<BGroup>& bg, const UVec<uint32_t>& brow,
                           const UVec<uint32_t>& brow_group, std::vector<uint8_t>& sel,
                           GroupList& out_groups,
                           UVec<uint32_t>& expired, UVec<uint32_t>& newly, PassStats& stats, bool rev,
                           uint32_t* min_stop, const std::function<BGroup&(uint32_t)>* view) {
    *min_stop = UINT32_MAX;
    if (!P.ok) return false;
    // Truncated lists are allowed: a pool whose row runs past the end of its
    // list stops there (the row's search re-runs in the next batch), the other
    // pools carry on; every row a pool processed is decided (pools never share
    // a ticket), and the pass puts the groups back in row order at its end.
    // view: a packed batch (rpack_kernel) — row bi's search is view(bi), a
    // thread-local BGroup over the row's packed list (complete by construction)
    bool all_complete = true;
    if (!view)
        for (const BGroup& g : bg) all_complete = all_complete && g.complete;
    if (!all_complete && !partial_mode_) return false;
    if (P.runs && runs_mode_ && P.ng > 64 && !(dense_mode_ && !rev && !view))
        return replay_runs(P, bg, brow, brow_group, sel, out_groups, expired, newly, stats, rev, min_stop, view);
    using clk = std::chrono::steady_clock;
    auto msd = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto tp1 = clk::now();
    const size_t nsearch = bg.size(), ng = P.ng, nb = brow.size();
    const std::vector<uint32_t>& search_pool = P.search_pool;
    WorkPool& wp = workers();
    const int maxI = cfg_.max_intervals;
    // each pool's searches (CSR) and each search's index among them: only
    // the dense walk reads them (one search per pool, no RevPrecision)
    const bool want_dense = dense_mode_ && !rev && !view;
    std::vector<uint32_t> soff(want_dense ? ng + 1 : 0, 0), sidx(want_dense ? nsearch : 0);
    if (want_dense) {
        for (size_t i = 0; i < nsearch; i++) soff[search_pool[i] + 1]++;
        for (size_t p = 0; p < ng; p++) soff[p + 1] += soff[p];
        std::vector<uint32_t> at(soff.begin(), soff.end() - 1);
        for (size_t i = 0; i < nsearch; i++) {
            const uint32_t p = search_pool[i];
            sidx[at[p]++] = (uint32_t)i;
        }
    }
    auto prows = [&](size_t p) { return P.pool_off[p + 1] - P.pool_off[p]; };
    // tasks: pools by size (largest first), the small ones bundled; many
    // pools (C5's 10^5 buckets) are bundled in pool order unsorted — every
    // task holds many, so the largest-first order buys no balance
    std::vector<uint32_t> order_g(ng);
    for (size_t i = 0; i < ng; i++) order_g[i] = (uint32_t)i;
    if (ng <= 4096)
        std::sort(order_g.begin(), order_g.end(), [&](uint32_t a, uint32_t b) { return prows(a) > prows(b); });
    const size_t per_task = std::max<size_t>(1, nb / ((size_t)wp.size() * 8));
    std::vector<uint32_t> task_off{0};
    for (size_t k = 0, acc = 0; k < ng; k++) {
        acc += prows(order_g[k]);
        if (acc >= per_task || k + 1 == ng) {
            task_off.push_back((uint32_t)(k + 1));
            acc = 0;
        }
    }
    const size_t ntask = task_off.size() - 1;
    // Few pools (C3's 8, C4's 64): each pool keeps its records in its own
    // array and the merge interleaves them (their rows interleave finely in
    // batch order, so per-row stores from several walks would share cache
    // lines).  Many pools (C5's buckets: each a short run of the batch):
    // records go straight to their batch rows.
    const bool few = ng <= 64;
    if (task_ents_.size() < ntask) task_ents_.resize(ntask);
    if (few && pool_outs_.size() < ng) pool_outs_.resize(ng);
    if (!few && row_recs_.size() < nb) grow_to(row_recs_, nb);
    RowRec* rr = few ? nullptr : row_recs_.data();
    if (!few)
        wp.run(wp.size(), [&](size_t c) {  // rows no pool processes (selected before they were reached) stay zero
            std::memset((void*)(rr + nb * c / wp.size()), 0, (nb * (c + 1) / wp.size() - nb * c / wp.size()) * sizeof(RowRec));
        });
    // Pools with one search (no RevPrecision) walk dense per-position copies
    // of their list (DensePool/DenseRun), gathered first in chunks across the
    // workers; the others take the generic walk over the store.
    if (dense_pools_.size() < ng) dense_pools_.resize(ng);
    if (pos_of_.size() < nslots()) pos_of_.resize(nslots(), kNoSlot);
    const ReplayView rv = replay_view();
    // The gathers run in tasks that each take the same fraction of EVERY
    // dense pool's list: the pools interleave in scan order, so task t's
    // pieces all read one slot region and the store lines it touches (2
    // HotRecs, 16 Intervals / pos_of words per line) are shared by the pools'
    // pieces while they sit in the core's cache — per-pool tasks read each
    // line once per pool (C4: 64 pools, every read a miss).
    constexpr uint32_t kGatherTask = 16384;  // list positions per task, over all pools
    std::vector<uint8_t> dense(ng, 0);
    std::vector<uint32_t> dense_ids;
    uint64_t dense_total = 0;
    for (size_t gi = 0; gi < ng && want_dense; gi++) {
        if (soff[gi + 1] - soff[gi] != 1) continue;  // the dense walk has no reverse checks
        if (!bg[sidx[soff[gi]]].complete) continue;                        // nor pages
        dense[gi] = 1;
        DensePool& D = dense_pools_[gi];
        D.reset(bg[sidx[soff[gi]]], P.pool_rows.data() + P.pool_off[gi], (uint32_t)prows(gi), brow.data());
        dense_ids.push_back((uint32_t)gi);
        dense_total += D.n;
    }
    const size_t ntask_g = (size_t)((dense_total + kGatherTask - 1) / kGatherTask);
    auto piece = [&](const DensePool& D, size_t t, uint32_t& lo, uint32_t& hi) {
        lo = (uint32_t)((uint64_t)D.n * t / ntask_g);
        hi = (uint32_t)((uint64_t)D.n * (t + 1) / ntask_g);
    };
    // Pipelined merge: with few pools, all dense, the merge runs in the same
    // job as the walks — tasks [0, ntask) walk, the next nch tasks merge one
    // chunk of batch rows each as soon as every walk has passed the chunk's
    // end (tasks are claimed in index order, so every walk is running before
    // any merge waits).  C3's 8 walks would otherwise leave 8 of 16 workers
    // idle while the merge waits for the slowest walk.
    const size_t nch0 = nb >= par_min(65536) ? (size_t)wp.size() * 2 : 1;
    const bool pipe = few && pipe_mode_ && !dense_ids.empty() && dense_ids.size() == ng && nch0 > 1;
    // the pipelined merge's chunks: the last one waits for the slowest walk,
    // so its size is the merge's tail
    const size_t nch = pipe ? (size_t)wp.size() * (size_t)kMergeMult : nch0;
    // Identity pools: when every pool's rows are its list in list order
    // (C3 / C4: every member of a pool of fresh tickets searches, and batch
    // order is scan order) row j's ticket is list position j — no slot ->
    // position map is built or read (a walk's map lookup is a cache miss per
    // row when the pools interleave in the store: C4's 64).  Pipelined
    // gather on top, when a worker is left beyond the walks: the gathers run
    // in the walks' job, tasks after the walks gather piece t of every pool
    // and publish each pool's gathered prefix, and a walk reads a position
    // once it is covered (DenseRun::need); otherwise the copies are gathered
    // before the walks.
    const auto tg0 = clk::now();
    bool ident = false;
    if (few && gpipe_mode_ && !dense_ids.empty() && dense_ids.size() == ng) {
        bool all = true;
        for (uint32_t gi : dense_ids) all = all && dense_pools_[gi].nrows == dense_pools_[gi].n;
        // Compared position by position (a parallel pass over the rows,
        // ~0.1 ms at C3's 1M; nothing to compare for a proven list,
        // BGroup::rows_list): identity is decided before any walk or merge
        // changes the pass state, so a wrong guess can never be caught
        // half-way — the walks then read row j's slot from position j.
        if (all) {
            std::vector<uint8_t> ok(ntask_g, 1);
            wp.run(ntask_g, [&](size_t t) {
                for (uint32_t gi : dense_ids) {
                    const DensePool& D = dense_pools_[gi];
                    uint32_t lo, hi;
                    piece(D, t, lo, hi);
                    if (!D.rows_are_list(lo, hi)) { ok[t] = 0; return; }
                }
            });
            ident = std::all_of(ok.begin(), ok.end(), [](uint8_t x) { return x != 0; });
        }
    }
    // proven lists (BGroup::rows_list) not downloaded: only the identity walk
    // goes without them
    const auto tg_ident = clk::now();
    if (!ident && !view) fill_row_lists(bg, brow, brow_group);
    const bool gpipe = ident && pipe && wp.size() > ntask;
    // (Identity pools with more walks than workers, C4's 64 on 16, gather
    // in a separate phase before the walks: gathering each pool inside its
    // walk's task measured even, profiles/r04ab_tgather.txt, and was removed.)
    if (ident)
        for (uint32_t gi : dense_ids) dense_pools_[gi].identity = true;
    std::unique_ptr<std::atomic<uint32_t>[]> gfront(gpipe ? new std::atomic<uint32_t>[ng] : nullptr);
    // a task of the pipelined job threw: the tasks waiting on others (merge
    // chunks on the walks' cuts, walks on the gather front) return instead of
    // spinning, and WorkPool::run rethrows the error once every task is done
    std::atomic<bool> job_failed{false};
    std::unique_ptr<std::atomic<uint8_t>[]> gdone(gpipe ? new std::atomic<uint8_t>[ng * ntask_g] : nullptr);
    if (gpipe) {
        for (size_t gi = 0; gi < ng; gi++) gfront[gi].store(0);
        for (size_t k = 0; k < ng * ntask_g; k++) gdone[k].store(0);
        for (uint32_t gi : dense_ids) {
            DensePool& D = dense_pools_[gi];
            D.pieces = (uint32_t)ntask_g;
            D.front = &gfront[gi];
            D.abort = &job_failed;
        }
    }
    // piece t of every pool, then each pool's published prefix advanced over
    // the pieces done (whichever worker completes the next piece moves it on)
    auto gather_piece = [&](size_t t) {
        for (uint32_t gi : dense_ids) {
            DensePool& D = dense_pools_[gi];
            uint32_t lo, hi;
            piece(D, t, lo, hi);
            D.gather(rv, lo, hi, pos_of_.data());
            gdone[gi * ntask_g + t].store(1);
            uint32_t f = gfront[gi].load();
            while (f < ntask_g && gdone[gi * ntask_g + f].load())
                if (gfront[gi].compare_exchange_weak(f, f + 1)) f++;
        }
    };
    // each pool's entry bound (every ticket of its list and rows joins at
    // most one group): the walk reserves it so readers never see a move
    const auto tg_setup = clk::now();
    std::vector<uint64_t> esum(pipe && !gpipe ? ntask_g * ng : 0, 0);
    if (!gpipe)
        wp.run(ntask_g, [&](size_t t) {
            for (uint32_t gi : dense_ids) {
                DensePool& D = dense_pools_[gi];
                uint32_t lo, hi;
                piece(D, t, lo, hi);
                D.gather(rv, lo, hi, pos_of_.data());
                if (!pipe) continue;
                uint64_t e = 0;
                for (uint32_t k = lo; k < hi; k++) e += (uint64_t)D.rec[k].count;
                const uint32_t r0 = (uint32_t)((uint64_t)D.nrows * t / ntask_g), r1 = (uint32_t)((uint64_t)D.nrows * (t + 1) / ntask_g);
                for (uint32_t j = r0; j < r1; j++) e += (uint64_t)rv.hot[brow[D.bis[j]]].count;
                esum[t * ng + gi] = e;
            }
        });
    const auto tg_gather = clk::now();
    struct alignas(128) Prog {
        std::atomic<uint32_t> ncut{0};  // merge chunk boundaries the walk has passed
        const PoolRec* recs = nullptr;
        const std::pair<uint32_t, int>* ents = nullptr;
        uint32_t* cut = nullptr;  // per boundary: the walk's records before it
    };
    std::unique_ptr<Prog[]> prog(pipe ? new Prog[ng] : nullptr);
    // the merge chunks' ends (batch rows), and per pool its record counts there
    std::vector<uint32_t> chunk_end(pipe ? nch : 0);
    for (size_t c = 0; c < chunk_end.size(); c++) chunk_end[c] = (uint32_t)(nb * (c + 1) / nch);
    if (pipe) {
        grow_to(pool_cuts_, ng * nch);
        for (size_t gi = 0; gi < ng; gi++) prog[gi].cut = pool_cuts_.data() + gi * nch;
    }
    std::vector<uint64_t> ebound(pipe ? ng : 0, 0);
    uint64_t ebound_all = 0;
    for (size_t t = 0; pipe && !gpipe && t < ntask_g; t++)
        for (size_t gi = 0; gi < ng; gi++) ebound[gi] += esum[t * ng + gi];
    if (gpipe)  // identity pools: the rows are list members, whose entries are at most max_pres_ each
        for (uint32_t gi : dense_ids) ebound[gi] = (uint64_t)dense_pools_[gi].n * (uint64_t)std::max(1, max_pres_);
    for (uint64_t e : ebound) ebound_all += e;
    const size_t g0 = out_groups.size(), e0 = out_groups.ents.size(), x0 = expired.size(), n0 = newly.size();
    if (pipe) {  // bounds now (no zero-fill: default-initialising vectors), the totals after the job
        grow_to(out_groups.off, g0 + 1 + nb);
        grow_to(out_groups.ents, e0 + ebound_all);
        grow_to(expired, x0 + nb);
        grow_to(newly, n0 + ebound_all);
    }
    // the result entries too, when every earlier group of the pass is filled
    // and the output arena is (or can be) this pass's
    const bool fill = pipe && filled_groups_ == g0 && (arena_claimed_ || !out_in_use_.exchange(true));
    if (fill) {
        arena_claimed_ = true;
        if (out_offs_.size() < g0 + 1 + nb) grow_to(out_offs_, g0 + 1 + nb);
        if (out_ents_.size() < e0 + ebound_all) grow_to(out_ents_, e0 + ebound_all);
        if (out_created_.size() < g0 + nb) grow_to(out_created_, g0 + nb);
        out_offs_[0] = 0;
    }
    // one chunk of the pipelined merge (merge_pools' chunk body, offsets
    // from the pools' running counts instead of a global prefix)
    std::vector<double> mch_wait(pipe ? nch : 0, 0.0), mch_ms(pipe ? nch : 0, 0.0);  // NKM_PROFILE=2 split
    auto merge_chunk = [&](size_t c) {
        const auto tm0 = clk::now();
        const uint32_t lo = (uint32_t)(nb * c / nch), hi = (uint32_t)(nb * (c + 1) / nch);
        size_t gk = g0, ek = e0, xk = x0;
        static thread_local std::vector<uint64_t> span;  // per pool: records [a, b) of the chunk
        span.assign(ng, 0);
        for (size_t gi = 0; gi < ng; gi++) {
            // waiting for the walks: sched_yield (sleeping instead measured
            // slower, profiles/r05/r05l_mwait_ab.txt)
            while (prog[gi].ncut.load(std::memory_order_acquire) <= c) {
                if (job_failed.load(std::memory_order_relaxed)) return;
                std::this_thread::yield();
            }
            // the chunk's records [a, b) from the walk's cuts (no search: a
            // binary search per pool per chunk was a miss chain each, 64
            // pools x 128 chunks on C4); the running counts after record a - 1
            const uint32_t a = c ? prog[gi].cut[c - 1] : 0u, b = prog[gi].cut[c];
            if (a) {
                const PoolRec& l = prog[gi].recs[a - 1];
                gk += l.gcum + l.matched;
                ek += l.off + l.len;
                xk += l.xcum + l.expired;
            }
            span[gi] = ((uint64_t)b << 32) | a;
        }
        const auto tm1 = clk::now();
        static thread_local std::vector<uint64_t> at_row;  // (pool << 32 | record) + 1; 0: no record
        at_row.assign(hi - lo, 0);
        // the pools' arrays and every output's base pointer in locals: the
        // loop's byte stores (decided, selected) may alias any memory, so
        // pointers read through members or the Prog array would be reloaded
        // after each one
        static thread_local std::vector<const PoolRec*> precs;
        static thread_local std::vector<const std::pair<uint32_t, int>*> pents;
        precs.resize(ng);
        pents.resize(ng);
        uint64_t* const AR = at_row.data();
        for (size_t gi = 0; gi < ng; gi++) {
            const PoolRec* R = prog[gi].recs;
            precs[gi] = R;
            pents[gi] = prog[gi].ents;
            for (uint32_t k = (uint32_t)span[gi]; k < (uint32_t)(span[gi] >> 32); k++)
                AR[R[k].bi - lo] = (((uint64_t)gi << 32) | k) + 1;
        }
        const PoolRec* const* const PR = precs.data();
        const std::pair<uint32_t, int>* const* const PE = pents.data();
        const uint32_t* const B = brow.data();
        int32_t* const IV = intervals_.data();
        uint8_t* const DEC = dec_.data();
        uint8_t* const SEL = sel.data();
        uint32_t* const XP = expired.data();
        GroupList::Entry* const OGE = out_groups.ents.data();
        uint32_t* const OGO = out_groups.off.data();
        uint32_t* const NW = newly.data() + n0 - e0;  // entry k's slot at NW[k]
        mm_entry_ref* const OE = fill ? out_ents_.data() : nullptr;
        int64_t* const OC = fill ? out_created_.data() : nullptr;
        int32_t* const OO = fill ? out_offs_.data() : nullptr;
        const char* const* const TK = tk_ptr_.data();
        const int64_t* const CR = created_.data();
        // rows interleave the pools' record and entry arrays (C4: 64 pools,
        // 128 streams — past what the hardware prefetchers track): each row's
        // record is prefetched 16 rows ahead, its entries 8 ahead
        const uint32_t nrow = hi - lo;
        for (uint32_t i = 0; i < nrow; i++) {
            if (i + 16 < nrow && AR[i + 16]) {
                const uint64_t w = AR[i + 16] - 1;
                __builtin_prefetch(PR[w >> 32] + (uint32_t)w);
            }
            if (i + 8 < nrow && AR[i + 8]) {
                const uint64_t w = AR[i + 8] - 1;
                __builtin_prefetch(PE[w >> 32] + PR[w >> 32][(uint32_t)w].off);
            }
            if (!AR[i]) continue;
            const uint64_t v = AR[i] - 1;
            const PoolRec r = PR[v >> 32][(uint32_t)v];
            const std::pair<uint32_t, int>* const ents = PE[v >> 32] + r.off;
            const uint32_t T = B[r.bi];
            IV[T]++;     // the row's pending Intervals increment
            DEC[T] = 1;  // decided: a later batch of the pass skips it
            if (r.expired) XP[xk++] = T;
            if (!r.matched) continue;
            for (uint32_t k = 0; k < r.len; k++) {
                const std::pair<uint32_t, int> e = ents[k];
                OGE[ek + k] = GroupList::Entry(e.first, e.second);
                NW[ek + k] = e.first;
                SEL[e.first] = 1;
                if (fill) OE[ek + k] = mm_entry_ref{TK[e.first], e.second, 0};
            }
            if (fill) OC[gk] = CR[T];  // the group's searching ticket (its last entry)
            ek += r.len;
            OGO[++gk] = (uint32_t)ek;
            if (fill) OO[gk] = (int32_t)ek;
        }
        mch_wait[c] = msd(tm0, tm1);
        mch_ms[c] = msd(tm0, clk::now());
    };
    std::vector<double> task_ms(ntask, 0.0), walk_prep_ms(ntask, 0.0), walk_ms(ntask, 0.0);  // NKM_PROFILE=2 split
    std::vector<double> walk_end_ms(ntask, 0.0);  // since the job's start
    std::vector<int> walk_cpu(2 * ntask, -1);       // NKM_PROFILE=2: the CPU a walk started / ended on
    clk::time_point tjob0 = clk::now();
    std::vector<uint64_t> task_hits(ntask, 0), task_pairs(ntask, 0);
    std::vector<uint32_t> pool_stop(ng, UINT32_MAX);  // per pool: the batch row its list ran out at
    auto to_rows = [&](const PoolOut& o, uint32_t task, std::vector<std::pair<uint32_t, int>>& ents) {
        const uint32_t base = (uint32_t)ents.size();
        ents.insert(ents.end(), o.ents.begin(), o.ents.end());
        for (size_t k = 0; k + 1 < o.recs.size(); k++) {  // the last record is the sentinel
            const PoolRec& r = o.recs[k];
            rr[r.bi] = RowRec{base + r.off, r.len, task, r.matched, r.expired, 1, 0};
        }
    };
    auto worker = [&](size_t t) {
        const auto tw0 = clk::now();
        auto& ents = task_ents_[t];
        ents.clear();
        static thread_local PoolOut o;
        static thread_local DenseRun run;
        // The worker thread's masks are all zero between pools.  Starting
        // from zero is exact: this batch's rows and hit lists hold no ticket
        // an earlier batch selected (assembly skips them; the device alive
        // mask dropped them before this batch's searches).  Intervals stay
        // unwritten during the walk (slots of all pools share its cache
        // lines): a row's increment is pending in tl_proc until the merge.
        static thread_local TlFlags tl;
        tl.ready(sel.size(), g_scratch_epoch.load(std::memory_order_relaxed));
        std::vector<uint8_t>& tl_sel = tl.sel;
        std::vector<uint8_t>& tl_proc = tl.proc;
        PassStats ls;
        const std::unique_ptr<ReplayCore> rpp = make_replay(tl_sel, rev, maxI, ls);
        ReplayCore& rp = *rpp;
        uint64_t hits = 0, pairs = 0;  // task_hits / task_pairs[t] at the end: neighbouring tasks' counters share a line
        for (uint32_t k = task_off[t]; k < task_off[t + 1]; k++) {
            const uint32_t gi = order_g[k];
            PoolOut& po = few ? pool_outs_[gi] : o;
            po.recs.clear();
            po.ents.clear();
            if (dense[gi] && pipe) {
                const DensePool& D = dense_pools_[gi];
                const auto tr0 = clk::now();
                run.reset(D.n);
                run.fast = fast_mode_;
                run.recs.reserve((size_t)D.nrows + 1);
                run.ents.reserve(ebound[gi]);
                prog[gi].recs = run.recs.data();
                prog[gi].ents = run.ents.data();
                const auto tr1 = clk::now();
                if (batch_profile_) walk_cpu[2 * t] = sched_getcpu();
                run.walk_cuts(D, rv, maxI, pos_of_.data(), chunk_end.data(), (uint32_t)nch, prog[gi].cut,
                              &prog[gi].ncut);
                const auto tr2 = clk::now();
                walk_prep_ms[t] += msd(tr0, tr1);
                walk_ms[t] += msd(tr1, tr2);
                walk_end_ms[t] = msd(tjob0, tr2);
                if (batch_profile_) walk_cpu[2 * t + 1] = sched_getcpu();
                if (run.ents.data() != prog[gi].ents || run.recs.data() != prog[gi].recs)
                    std::abort();  // the bound above was wrong: readers hold the old buffers
                hits += run.hits_seen;
                pairs += (uint64_t)run.recs.size() * D.src_len;
                // the sentinel (its capacity was reserved), then the buffers to
                // the pool's PoolOut (a header swap: the readers' pointers stay)
                run.recs.push_back(PoolRec{UINT32_MAX, 0, 0, (uint32_t)run.ents.size(), 0, run.g_run, run.x_run});
                po.recs.swap(run.recs);
                po.ents.swap(run.ents);
                continue;
            }
            if (dense[gi]) {
                run.reset(dense_pools_[gi].n);
                run.fast = fast_mode_;
                run.walk(dense_pools_[gi], rv, maxI, pos_of_.data(), 0, dense_pools_[gi].nrows);
                hits += run.hits_seen;
                pairs += (uint64_t)run.recs.size() * dense_pools_[gi].src_len;
                if (few) {
                    run.finish(po);
                    continue;
                }
                // the walk's records straight to the rows (entries offsets are run.ents')
                const uint32_t base = (uint32_t)ents.size();
                if (ents.empty()) ents.swap(run.ents);
                else ents.insert(ents.end(), run.ents.begin(), run.ents.end());
                for (const PoolRec& r : run.recs)
                    rr[r.bi] = RowRec{base + r.off, r.len, (uint32_t)t, r.matched, r.expired, 1, 0};
                continue;
            } else {
                const uint32_t* prow = P.pool_rows.data() + P.pool_off[gi];
                const size_t npr = P.pool_off[gi + 1] - P.pool_off[gi];
                rp.hits_seen = 0;
                rp.pairs = 0;
                const uint32_t stop =
                    view ? replay_pool(rp, prow, npr, brow.data(), *view, tl_sel, tl_proc.data(), minc_.data(),
                                       maxc_.data(), po)
                         : replay_pool(rp, prow, npr, brow.data(),
                                       [&](uint32_t bi) -> BGroup& { return bg[brow_group[bi]]; }, tl_sel,
                                       tl_proc.data(), minc_.data(), maxc_.data(), po);
                if (stop != UINT32_MAX) pool_stop[gi] = stop;
                hits += rp.hits_seen;
                pairs += rp.pairs;
            }
            if (!few) to_rows(o, (uint32_t)t, ents);
        }
        task_hits[t] = hits;
        task_pairs[t] = pairs;
        task_ms[t] = msd(tw0, clk::now());
    };
    const auto tg1 = clk::now();
    tjob0 = tg1;
    stats.par_gather_ms += msd(tg0, tg1);
    if (pipe) {
        const size_t ngt = gpipe ? ntask_g : 0;
        wp.run(ntask + ngt + nch, [&](size_t t) {
            try {
                if (t < ntask) worker(t);
                else if (t < ntask + ngt) gather_piece(t - ntask);
                else merge_chunk(t - ntask - ngt);
            } catch (...) {
                job_failed.store(true);
                throw;
            }
        });
        size_t G = 0, E = 0, X = 0;  // totals: the pools' sentinels
        for (size_t gi = 0; gi < ng; gi++) {
            const PoolRec& sr = pool_outs_[gi].recs.back();
            G += sr.gcum;
            E += sr.off;
            X += sr.xcum;
        }
        out_groups.off.resize(g0 + 1 + G);
        out_groups.ents.resize(e0 + E);
        expired.resize(x0 + X);
        newly.resize(n0 + E);
        if (fill) filled_groups_ = g0 + G;
    } else {
        wp.run(ntask, worker);
    }
    const auto tg2 = clk::now();
    stats.par_job_ms += msd(tg1, tg2);
    if (!gpipe) wp.run(ntask_g, [&](size_t t) {
        for (uint32_t gi : dense_ids) {
            const DensePool& D = dense_pools_[gi];
            uint32_t lo, hi;
            piece(D, t, lo, hi);
            D.clear_pos(lo, hi, pos_of_.data());
        }
    });
    const auto tp2 = clk::now();
    stats.par_clear_ms += msd(tg2, tp2);
    for (uint32_t v : pool_stop) *min_stop = std::min(*min_stop, v);
    if (pipe) {
    } else if (few) {
        merge_pools(ng, nch, brow, sel, out_groups, expired, newly);
    } else {
        merge_rows(nb, nch, brow, sel, out_groups, expired, newly);
    }
    const auto tp3 = clk::now();
    stats.par_work_ms += msd(tp1, tp2);
    stats.par_merge_ms += msd(tp2, tp3);
    for (size_t k = 0; k < ntask; k++) {
        stats.par_task_max_ms = std::max(stats.par_task_max_ms, task_ms[k]);
        stats.par_hits += task_hits[k];
        if (!row_shard() || shard_rank_ == 0) stats.pairs_decided += (int64_t)task_pairs[k];
    }
    if (batch_profile_ && pipe) {
        double sp = 0, sw = 0, st = 0, mw = 0, we = 0;
        for (size_t k = 0; k < ntask; k++) {
            sp += walk_prep_ms[k];
            sw += walk_ms[k];
            st += task_ms[k];
            mw = std::max(mw, walk_ms[k]);
            we = std::max(we, walk_end_ms[k]);
        }
        double cw = 0, cm = 0;
        for (size_t c = 0; c < nch; c++) {
            cw += mch_wait[c];
            cm += mch_ms[c];
        }
        std::fprintf(stderr, "[nkm]   pool walks: %zu tasks, %zu pools on %u workers | sum: tasks %.2f, walks %.2f (max %.2f), "
                     "gather+reset+reserve %.2f ms | gather %s | last walk ends %.2f, job %.2f ms (%zu merge chunks: "
                     "sum %.2f, of it waiting %.2f ms) | before the job: identity check %.2f, lists + setup %.2f, "
                     "gather %.2f, bounds %.2f ms\n",
                     ntask, ng, wp.size(), st, sw, mw, sp, gpipe ? "beside" : "before", we, msd(tg1, tg2), nch, cm, cw,
                     msd(tg0, tg_ident), msd(tg_ident, tg_setup), msd(tg_setup, tg_gather), msd(tg_gather, tg1));
        if (ntask <= 16) {  // each walk: pool, ms, rows, ends at (ms into the job), CPU at start/end
            std::string w;
            char buf[96];
            for (size_t k = 0; k < ntask; k++) {
                const uint32_t gi = order_g[task_off[k]];
                std::snprintf(buf, sizeof buf, " [p%u %.2f ms %u rows end %.2f cpu %d/%d]", gi, walk_ms[k],
                              dense_pools_[gi].nrows, walk_end_ms[k], walk_cpu[2 * k], walk_cpu[2 * k + 1]);
                w += buf;
            }
            std::fprintf(stderr, "[nkm]   walks:%s\n", w.c_str());
        }
    }
    stats.par_rows += nb;
    return true;
}

// Pools in contiguous runs of the batch (ParPlan::runs — C5's buckets: a
// bucket's tickets arrive together), none dense: a task takes consecutive
// pools, i.e. one range of batch rows, so the tasks' outputs in task order
// are the row order and no per-row record or merge_rows pass is needed.
// Pools share no ticket (replay_parallel's premise), so every ticket a task
// reads or writes — its rows, their hits — is its own: the workers update
// the pass state directly (Intervals, decided, selected) instead of through
// thread-local masks and a merge, and each row's Intervals increment is
// visible to the pool's later rows exactly as the sequential pass sees it.
// The outputs are then placed at their offsets in one parallel copy (plus
// the result arena's entries when this pass owns it, as the pipelined merge).
bool Core::replay_runs(const ParPlan& P, std::vector<BGroup>& bg, const UVec<uint32_t>& brow,
                       const UVec<uint32_t>& brow_group, std::vector<uint8_t>& sel, GroupList& out_groups,
                       UVec<uint32_t>& expired, UVec<uint32_t>& newly, PassStats& stats, bool rev,
                       uint32_t* min_stop, const std::function<BGroup&(uint32_t)>* view) {
    using clk = std::chrono::steady_clock;
    auto msd = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto tp1 = clk::now();
    WorkPool& wp = workers();
    const size_t ng = P.ng, nb = brow.size();
    const int maxI = cfg_.max_intervals;
    if (!view) fill_row_lists(bg, brow, brow_group);
    const size_t per_task = std::max<size_t>(1, nb / ((size_t)wp.size() * 8));
    std::vector<uint32_t> task_off{0};  // pools [task_off[t], task_off[t+1])
    for (size_t p = 0, acc = 0; p < ng; p++) {
        acc += P.pool_off[p + 1] - P.pool_off[p];
        if (acc >= per_task || p + 1 == ng) {
            task_off.push_back((uint32_t)(p + 1));
            acc = 0;
        }
    }
    const size_t ntask = task_off.size() - 1;
    if (run_outs_.size() < ntask) run_outs_.resize(ntask);
    std::vector<uint32_t> task_stop(ntask, UINT32_MAX);
    int32_t* iv = intervals_.data();
    uint8_t* dec = dec_.data();
    auto worker = [&](size_t t) {
        const auto tw0 = clk::now();
        RunOut& o = run_outs_[t];
        o.gend.clear();
        o.gT.clear();
        o.ents.clear();
        o.expired.clear();
        PassStats ls;
        const std::unique_ptr<ReplayCore> rpp = make_replay(sel, rev, maxI, ls);
        ReplayCore& rp = *rpp;
        rp.proc = nullptr;  // increments are written as the rows go
        static thread_local std::vector<std::pair<uint32_t, int>> grp;
        for (uint32_t p = task_off[t]; p < task_off[t + 1]; p++) {
            for (uint32_t bi = P.pool_off[p]; bi < P.pool_off[p + 1]; bi++) {
                const uint32_t T = brow[bi];
                if (sel[T]) continue;
                BGroup& g = view ? (*view)(bi) : bg[brow_group[bi]];
                const auto status = rp.decide(T, g, false, grp);
                if (status == ReplayCore::EXHAUSTED) {  // the pool stops here; its search re-runs next batch
                    task_stop[t] = std::min(task_stop[t], bi);
                    break;
                }
                if (iv[T] + 1 >= maxI || minc_[T] == maxc_[T]) o.expired.push_back(T);
                iv[T]++;
                dec[T] = 1;
                if (status != ReplayCore::MATCHED) continue;
                for (const auto& e : grp) {
                    sel[e.first] = 1;
                    o.ents.push_back(e);
                }
                o.gend.push_back((uint32_t)o.ents.size());
                o.gT.push_back(T);
            }
        }
        o.hits = rp.hits_seen;
        o.pairs = rp.pairs;
        o.ms = msd(tw0, clk::now());
    };
    wp.run(ntask, worker);
    const auto tp2 = clk::now();
    // offsets: the tasks in order
    struct Cnt { size_t g = 0, e = 0, x = 0; };
    std::vector<Cnt> at(ntask + 1);
    for (size_t t = 0; t < ntask; t++) {
        const RunOut& o = run_outs_[t];
        at[t + 1] = {at[t].g + o.gend.size(), at[t].e + o.ents.size(), at[t].x + o.expired.size()};
    }
    const size_t g0 = out_groups.size(), e0 = out_groups.ents.size(), x0 = expired.size(), n0 = newly.size();
    const size_t G = at[ntask].g, E = at[ntask].e, X = at[ntask].x;
    grow_to(out_groups.off, g0 + 1 + G);
    grow_to(out_groups.ents, e0 + E);
    grow_to(expired, x0 + X);
    grow_to(newly, n0 + E);
    const bool fill = filled_groups_ == g0 && (arena_claimed_ || !out_in_use_.exchange(true));
    if (fill) {
        arena_claimed_ = true;
        if (out_offs_.size() < g0 + 1 + G) grow_to(out_offs_, g0 + 1 + G);
        if (out_ents_.size() < e0 + E) grow_to(out_ents_, e0 + E);
        if (out_created_.size() < g0 + G) grow_to(out_created_, g0 + G);
        out_offs_[0] = 0;
    }
    wp.run(ntask, [&](size_t t) {
        const RunOut& o = run_outs_[t];
        const size_t gk = g0 + at[t].g, ek = e0 + at[t].e;
        for (size_t k = 0; k < o.gend.size(); k++) {
            out_groups.off[gk + 1 + k] = (uint32_t)(ek + o.gend[k]);
            if (fill) {
                out_offs_[gk + 1 + k] = (int32_t)(ek + o.gend[k]);
                out_created_[gk + k] = created_[o.gT[k]];
            }
        }
        for (size_t k = 0; k < o.ents.size(); k++) {
            const auto& e = o.ents[k];
            out_groups.ents[ek + k] = e;
            newly[n0 + (ek - e0) + k] = e.first;
            if (fill) out_ents_[ek + k] = mm_entry_ref{tk_ptr_[e.first], e.second, 0};
        }
        std::copy(o.expired.begin(), o.expired.end(), expired.begin() + (ptrdiff_t)(x0 + at[t].x));
    });
    out_groups.off.resize(g0 + 1 + G);
    out_groups.ents.resize(e0 + E);
    expired.resize(x0 + X);
    newly.resize(n0 + E);
    if (fill) filled_groups_ = g0 + G;
    const auto tp3 = clk::now();
    *min_stop = UINT32_MAX;
    for (uint32_t s : task_stop) *min_stop = std::min(*min_stop, s);
    stats.par_job_ms += msd(tp1, tp2);
    stats.par_work_ms += msd(tp1, tp2);
    stats.par_merge_ms += msd(tp2, tp3);
    for (size_t t = 0; t < ntask; t++) {
        const RunOut& o = run_outs_[t];
        stats.par_task_max_ms = std::max(stats.par_task_max_ms, o.ms);
        stats.par_hits += o.hits;
        if (!row_shard() || shard_rank_ == 0) stats.pairs_decided += (int64_t)o.pairs;
    }
    if (batch_profile_) {
        double sum = 0;
        for (size_t t = 0; t < ntask; t++) sum += run_outs_[t].ms;
        std::fprintf(stderr, "[nkm]   pool runs: %zu tasks, %zu pools on %u workers | tasks sum %.2f ms (mean %.3f) | "
                     "job %.2f copy %.2f ms\n", ntask, ng, wp.size(), sum, sum / (double)ntask, msd(tp1, tp2),
                     msd(tp2, tp3));
    }
    stats.par_rows += nb;
    return true;
}

// Merge of per-row records (many pools) back into the pinned row order.
void Core::merge_rows(size_t nb, size_t nch, const UVec<uint32_t>& brow, std::vector<uint8_t>& sel,
                      GroupList& out_groups, UVec<uint32_t>& expired, UVec<uint32_t>& newly) {
    WorkPool& wp = workers();
    const RowRec* rr = row_recs_.data();
    struct Cnt { size_t g = 0, e = 0, x = 0; };
    // Back into the pinned row order: per chunk of the batch, its groups /
    // entries / expired counts, then every chunk fills its share at its
    // offsets and applies its rows' pending Intervals increments.
    std::vector<Cnt> at(nch + 1);
    wp.run(nch, [&](size_t c) {
        Cnt k;
        for (size_t bi = nb * c / nch; bi < nb * (c + 1) / nch; bi++) {
            const RowRec& r = rr[bi];
            if (!r.processed) continue;
            k.x += r.expired;
            if (r.matched) k.g++, k.e += r.len;
        }
        at[c + 1] = k;
    });
    for (size_t c = 0; c < nch; c++) at[c + 1] = {at[c].g + at[c + 1].g, at[c].e + at[c + 1].e, at[c].x + at[c + 1].x};
    const size_t g0 = out_groups.size(), e0 = out_groups.ents.size(), x0 = expired.size(), n0 = newly.size();
    grow_to(out_groups.off, g0 + 1 + at[nch].g);
    grow_to(out_groups.ents, e0 + at[nch].e);
    grow_to(expired, x0 + at[nch].x);
    grow_to(newly, n0 + at[nch].e);
    wp.run(nch, [&](size_t c) {
        size_t gk = g0 + at[c].g, ek = e0 + at[c].e, xk = x0 + at[c].x;
        for (size_t bi = nb * c / nch; bi < nb * (c + 1) / nch; bi++) {
            const RowRec& r = rr[bi];
            if (!r.processed) continue;
            const uint32_t T = brow[bi];
            intervals_[T]++;  // the row's pending Intervals increment
            dec_[T] = 1;      // decided: a later batch of the pass skips it
            if (r.expired) expired[xk++] = T;
            if (!r.matched) continue;
            const auto* src = task_ents_[r.task].data() + r.ent;
            for (uint32_t k = 0; k < r.len; k++) {
                out_groups.ents[ek + k] = src[k];
                newly[n0 + (ek - e0) + k] = src[k].first;
                sel[src[k].first] = 1;
            }
            ek += r.len;
            out_groups.off[++gk] = (uint32_t)ek;
        }
    });
}

// Merge of few pools' record arrays back into the pinned row order.  The
// batch's row range is cut into chunks; each pool's records (ascending in
// batch row, with running group / entry / expiry counts) are located in every
// chunk by binary search, so each chunk knows its output offsets up front and
// merges its share of the pools' records independently (through a
// chunk-local row map).  Applies the rows' pending Intervals increments on
// the way.
void Core::merge_pools(size_t ng, size_t nch, const UVec<uint32_t>& brow, std::vector<uint8_t>& sel,
                       GroupList& out_groups, UVec<uint32_t>& expired, UVec<uint32_t>& newly) {
    using Rec = PoolRec;
    auto& outs = pool_outs_;
    WorkPool& wp = workers();
    const size_t nb = brow.size();
    std::vector<uint32_t> cut((nch + 1) * ng);  // [c][pool]: first record with bi >= chunk start
    for (size_t c = 0; c <= nch; c++) {
        const uint32_t lo = (uint32_t)(nb * c / nch);
        for (size_t gi = 0; gi < ng; gi++) {
            const auto& r = outs[gi].recs;  // sentinel at the end (bi = UINT32_MAX)
            cut[c * ng + gi] = c == nch ? (uint32_t)(r.size() - 1)
                                        : (uint32_t)(std::lower_bound(r.begin(), r.end(), lo,
                                                                      [](const Rec& x, uint32_t v) { return x.bi < v; }) -
                                                     r.begin());
        }
    }
    struct Cnt { size_t g = 0, e = 0, x = 0; };
    std::vector<Cnt> at(nch + 1);
    for (size_t c = 0; c < nch; c++) {
        Cnt k;
        for (size_t gi = 0; gi < ng; gi++) {
            const Rec& a0 = outs[gi].recs[cut[c * ng + gi]];
            const Rec& a1 = outs[gi].recs[cut[(c + 1) * ng + gi]];
            k.g += a1.gcum - a0.gcum;
            k.e += a1.off - a0.off;
            k.x += a1.xcum - a0.xcum;
        }
        at[c + 1] = {at[c].g + k.g, at[c].e + k.e, at[c].x + k.x};
    }
    const size_t g0 = out_groups.size(), e0 = out_groups.ents.size(), x0 = expired.size(), n0 = newly.size();
    grow_to(out_groups.off, g0 + 1 + at[nch].g);
    grow_to(out_groups.ents, e0 + at[nch].e);
    grow_to(expired, x0 + at[nch].x);
    grow_to(newly, n0 + at[nch].e);
    wp.run(nch, [&](size_t c) {
        // the chunk's records placed by batch row (a chunk-local map written by
        // this worker alone), then swept in row order: linear in the chunk for
        // any number of pools
        const uint32_t lo = (uint32_t)(nb * c / nch), hi = (uint32_t)(nb * (c + 1) / nch);
        static thread_local std::vector<uint64_t> at_row;  // (pool << 32 | record) + 1; 0: no record
        at_row.assign(hi - lo, 0);
        for (size_t gi = 0; gi < ng; gi++) {
            const auto& recs = outs[gi].recs;
            for (uint32_t k = cut[c * ng + gi]; k < cut[(c + 1) * ng + gi]; k++)
                at_row[recs[k].bi - lo] = (((uint64_t)gi << 32) | k) + 1;
        }
        size_t gk = g0 + at[c].g, ek = e0 + at[c].e, xk = x0 + at[c].x;
        for (uint32_t i = 0; i < hi - lo; i++) {
            if (!at_row[i]) continue;
            const uint64_t v = at_row[i] - 1;
            const PoolOut& o = outs[v >> 32];
            const Rec& r = o.recs[(uint32_t)v];
            const uint32_t T = brow[r.bi];
            intervals_[T]++;  // the row's pending Intervals increment
            dec_[T] = 1;      // decided: a later batch of the pass skips it
            if (r.expired) expired[xk++] = T;
            if (!r.matched) continue;
            for (uint32_t k = 0; k < r.len; k++) {
                const auto& e = o.ents[r.off + k];
                out_groups.ents[ek + k] = e;
                newly[n0 + (ek - e0) + k] = e.first;
                sel[e.first] = 1;
            }
            ek += r.len;
            out_groups.off[++gk] = (uint32_t)ek;
        }
    });
}

// Row bi of a packed batch as the replay's search view (its fixed-stride
// list, reverse bits and pair words in the pinned output buffer).  The list
// comes as source positions: `src` is the row's source (its posting or order
// list on the host mirror), `slots` the thread's buffer its slot ids go to.
static inline void fill_packed(BGroup& g, const uint8_t* base, const PackLayout& L, uint32_t bi, uint32_t T,
                               uint32_t sig, const uint32_t* src, uint32_t* slots) {
    const uint32_t n = base[L.cnt + bi];
    const uint32_t P = L.S < 32 ? (uint32_t)L.S : 32u;
    const uint8_t* pos = base + L.pos + (size_t)bi * L.S;
    for (uint32_t k = 0; k < n; k++) slots[k] = src[pos[k]];
    g.sig = sig;
    g.row_slot = T;
    g.d.rev_slot = T;
    g.nrows = 1;
    g.set_slots(slots);
    g.last_i = UINT32_MAX;
    g.rev = nullptr;
    g.rev_packed = true;
    const uint8_t* rv = base + L.rev;
    g.rev_bits = L.rev_w == 1 ? rv[bi]
               : L.rev_w == 2 ? reinterpret_cast<const uint16_t*>(rv)[bi]
               : L.rev_w == 4 ? reinterpret_cast<const uint32_t*>(rv)[bi]
                              : reinterpret_cast<const uint64_t*>(rv)[bi];
    g.pm = base + L.pm + (size_t)bi * P * L.pm_w;
    g.pm_w = (uint8_t)L.pm_w;
    g.pm_n = std::min(n, P);
    g.n = n;
    g.complete = true;
    g.head = 0;
}

// Packed RevPrecision batch assembly: the pass rows [pos, end) not yet
// selected or decided, each its ticket's slot and source (source_of's choice:
// the posting list of its most selective required term), straight into the
// pinned upload buffer.  False (nothing changed) when some row's source holds
// more than 64 entries: the per-search path then takes the batch.
bool Core::assemble_packed(const std::vector<uint32_t>& rows, size_t pos, size_t cap, UVec<uint32_t>& brow,
                           PackBatch& pb) {
    const size_t nr = std::min({rows.size() - pos, kMaxBatchRows, cap});
    WorkPool& wp = workers();
    const bool par = par_mode_ && nr >= par_min(65536);
    const size_t nch = par ? (size_t)wp.size() * 4 : 1;
    grow_to(pk_tmp_, nr);
    std::vector<size_t> at(nch + 1, 0);
    std::vector<uint32_t> maxlen(nch, 0);
    std::vector<uint8_t> bad(nch, 0);
    std::vector<uint64_t> scanned(nch, 0);
    std::vector<double> live_w(nch, 0.0);
    auto pass1 = [&](size_t c) {
        size_t k = 0;
        uint32_t mx = 0;
        uint64_t sc = 0;
        double lw = 0.0;
        for (size_t i = nr * c / nch; i < nr * (c + 1) / nch; i++) {
            const uint32_t r = rows[pos + i];
            DSmallRow& o = pk_tmp_[i];
            if (sel_[r] | dec_[r]) {
                o.slot = kNoSlot;
                continue;
            }
            // the signature's 16-B summary (ids follow first appearance, so
            // the rows read it nearly in sequence), the Sig itself only for
            // a search with several MUST terms
            const uint32_t sgi = sig_[r];
            const SigLite& sl = sig_lite_[sgi];
            DGroup d;
            if (sl.key1 != UINT64_MAX) source_of_key1(sl.key1, d);
            else source_of(sigs_[sgi], d);
            if (d.src_len > 64) {
                bad[c] = 1;
                return;
            }
            o = DSmallRow{r, d.src_off, d.src_len | (d.src_kind == 0 ? kSrcOrder : 0u)};
            k++;
            mx = std::max(mx, d.src_len);
            sc += d.src_len;
            // per live candidate (search_bytes' rev form): Min/MaxCount, the
            // query's field columns, the hit's query descriptor and clauses
            lw += (double)d.src_len * (double)(8 + 9 * sl.n_fields + 8 + 32 * sl.n_clauses);
        }
        at[c + 1] = k;
        maxlen[c] = mx;
        scanned[c] = sc;
        live_w[c] = lw;
    };
    using aclk = std::chrono::steady_clock;
    const auto ta0 = aclk::now();
    if (nch > 1) wp.run(nch, pass1);
    else pass1(0);
    const auto ta1 = aclk::now();
    for (uint8_t b : bad)
        if (b) return false;
    for (size_t c = 0; c < nch; c++) at[c + 1] += at[c];
    const size_t n = at[nch];
    h_srows_.reserve(std::max<size_t>(n, 1));
    grow_to(brow, n);
    auto pass2 = [&](size_t c) {
        size_t o = at[c];
        for (size_t i = nr * c / nch; i < nr * (c + 1) / nch; i++) {
            const DSmallRow& d = pk_tmp_[i];
            if (d.slot == kNoSlot) continue;
            h_srows_.p[o] = d;
            brow[o] = d.slot;
            o++;
        }
    };
    if (nch > 1) wp.run(nch, pass2);
    else pass2(0);
    const auto ta2 = aclk::now();
    pb = PackBatch{};
    pb.n = n;
    pb.end = pos + nr;
    uint32_t mx = 0;
    for (size_t c = 0; c < nch; c++) {
        mx = std::max(mx, maxlen[c]);
        pb.scanned += scanned[c];
        pb.live_w += live_w[c];
    }
    while ((uint32_t)pb.S < mx) pb.S *= 2;
    // distinct candidates per wave (its 64 / S rows' source ranges merged):
    // what the wave's loads bring in, each once (the roofline's bytes; C5's
    // square waves: the 8 rows ARE their shared source, 8 candidates)
    const uint32_t rpw = 64u / (uint32_t)pb.S;
    const size_t nw = (n + rpw - 1) / rpw;
    const size_t wch = par && nw >= 4096 ? (size_t)wp.size() * 4 : 1;
    std::vector<uint64_t> uniq(wch, 0);
    auto pass3 = [&](size_t c) {
        uint64_t u = 0;
        std::pair<uint64_t, uint64_t> rg[64];
        for (size_t w = nw * c / wch; w < nw * (c + 1) / wch; w++) {
            const size_t r0 = w * rpw, r1 = std::min(n, r0 + rpw);
            int k = 0;
            for (size_t r = r0; r < r1; r++) {
                const DSmallRow& d = h_srows_.p[r];
                const uint64_t base = (d.src_len & kSrcOrder) ? (1ull << 40) : 0;  // order[] vs postings[]
                const uint64_t a = base + d.src_off;
                rg[k++] = {a, a + (d.src_len & ~kSrcOrder)};
            }
            // insertion sort: a wave's rows are mostly one bucket's, their
            // ranges equal or ascending already (std::sort measured ~100 ns a
            // wave, 125k waves per C5 pass)
            for (int q = 1; q < k; q++) {
                const std::pair<uint64_t, uint64_t> x = rg[q];
                int p = q - 1;
                while (p >= 0 && x < rg[p]) { rg[p + 1] = rg[p]; p--; }
                rg[p + 1] = x;
            }
            uint64_t hi = 0;
            for (int q = 0; q < k; q++) {
                const uint64_t lo = std::max(rg[q].first, hi);
                if (rg[q].second > lo) u += rg[q].second - lo;
                hi = std::max(hi, rg[q].second);
            }
        }
        uniq[c] = u;
    };
    if (wch > 1) wp.run(wch, pass3);
    else pass3(0);
    for (uint64_t u : uniq) pb.unique += u;
    if (batch_profile_) {
        auto ms = [](aclk::time_point a, aclk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "[nkm]   assemble_packed: %zu rows | sources %.2f compact %.2f wave bytes %.2f ms\n", n,
                     ms(ta0, ta1), ms(ta1, ta2), ms(ta2, aclk::now()));
    }
    return true;
}

// One packed batch on the device: rows up, rpack_kernel, the whole output
// down in one copy (the host `overlap` work runs meanwhile).
PackLayout Core::run_packed(const PackBatch& pb, PassStats& stats, const std::function<void()>& overlap) {
    flush_apply();  // the previous batch's selections, before this batch's searches
    PackLayout L = pack_layout(pb.n, pb.S);
    const DStore st = dstore();
    {  // the columns the square wave prefetches: every field a clause names, when at most 2
        uint32_t k = 0;
        bool ok = true;
        for (size_t f = 0; f < field_used_.size() && ok; f++) {
            if (!field_used_[f]) continue;
            if (k == 2 || f >= d_fval_.size() || !d_fval_[f] || !d_fkind_[f]) { ok = false; break; }
            L.pf[k] = (uint16_t)f;
            L.pf_val[k] = d_fval_[f]->p;
            L.pf_kind[k] = d_fkind_[f]->p;
            k++;
        }
        L.npf = ok ? k : 0;
    }
    d_srows_.reserve(std::max<size_t>(pb.n, 1), false);
    d_pack_.reserve(L.total, false);
    h_pack_.reserve(L.total);
    if (pb.n) {
        NKM_HIP(hipMemcpyAsync(d_srows_.p, h_srows_.p, pb.n * sizeof(DSmallRow), hipMemcpyHostToDevice, stream_));
        NKM_HIP(launch_rpack(st, d_srows_.p, (uint32_t)pb.n, d_pack_.p, L, stream_, ev_[7], ev_[8]));
        NKM_HIP(hipMemcpyAsync(h_pack_.p, d_pack_.p, L.total, hipMemcpyDeviceToHost, stream_));
    }
    if (overlap) overlap();
    NKM_HIP(hipStreamSynchronize(stream_));
    stats.batches++;
    if (!pb.n) return L;
    float ms = 0.f;
    NKM_HIP(hipEventElapsedTime(&ms, ev_[7], ev_[8]));
    stats.k_ms[3] += ms;
    stats.k_launches[3]++;
    stats.rpack = true;
    uint64_t live = 0, ents = 0;
    const uint32_t* lw = reinterpret_cast<const uint32_t*>(h_pack_.p + L.live);
    for (uint32_t b = 0; b < L.blocks; b++) {
        live += lw[2 * b];
        ents += lw[2 * b + 1];
    }
    // algorithmic bytes: per row its descriptor and its query / count range;
    // per distinct candidate of a wave (pb.unique: the wave's loads bring each
    // in once, the S x S evaluations re-read them from L1 / LDS) its slot id,
    // alive flag and columns, query descriptor and clauses (the rows' average
    // per-candidate bytes, weighted by source length); per entry its source position (1 B);
    // per row its pair words, reverse bits and count (4-B slot ids per entry
    // until round 5).  (Rounds 1-3 charged
    // every (row, candidate) pair's loads: C5 894 MB per launch vs 170 MB of
    // PMC traffic, profiles/r04q_c5_traffic.json.)
    (void)live;
    const double per_live = pb.scanned ? pb.live_w / (double)pb.scanned : 0.0;
    const int P = pb.S < 32 ? pb.S : 32;
    stats.k_bytes[3] += (int64_t)pb.n * (int64_t)(sizeof(DSmallRow) + 16) +
                        (int64_t)((double)pb.unique * (5.0 + per_live)) + (int64_t)ents +
                        (int64_t)pb.n * (int64_t)(P * L.pm_w + L.rev_w + 1);
    stats.pair_evals += (int64_t)pb.scanned;
    return L;
}

// The dictionary id -> first search table plan_pools numbers pools with: all
// entries UINT32_MAX between calls (every user resets what it set).
std::atomic<uint32_t>* Core::pool_first_table(size_t nd) {
    if (pool_first_cap_ < nd) {
        pool_first_.reset(new std::atomic<uint32_t>[nd + nd / 4]);
        pool_first_cap_ = nd + nd / 4;
        std::atomic<uint32_t>* f = pool_first_.get();
        WorkPool& wp = workers();
        const size_t nch = pool_first_cap_ >= 65536 ? wp.size() : 1;
        auto clear = [&](size_t c) {
            for (size_t t = pool_first_cap_ * c / nch; t < pool_first_cap_ * (c + 1) / nch; t++)
                f[t].store(UINT32_MAX, std::memory_order_relaxed);
        };
        if (nch > 1) wp.run(nch, clear);
        else clear(0);
    }
    return pool_first_.get();
}

// plan_pools' one-key-field contiguous case in three sweeps (C5: a bucket's
// tickets arrive together, so every pool is one run of the packed batch):
//   A  each row's pool term (its own column when it carries its search's
//      terms, else its signature's required term), the row check, and an
//      atomic min of first[term] at every run start;
//   B  per chunk: run starts, and those that are their term's first (heads);
//   C  when every run start is a head (no term comes back after its run),
//      each chunk numbers the runs starting in it (pool = run index, the
//      first-appearance order plan_pools uses) and fills the CSR, the pool
//      terms and the self flags, and clears first[] for its heads.
// 1: planned; 0: not this shape (nothing changed; plan_pools decides);
// -1: plan_pools would fail too (a search without the key, two terms on it,
// a row outside its pool).  first[] is all-empty again on every return.
int Core::plan_packed_runs(size_t n, const UVec<uint32_t>& brow, ParPlan& P, PassStats& stats) {
    using clk = std::chrono::steady_clock;
    const auto tp0 = clk::now();
    WorkPool& wp = workers();
    if (n < 2 || !par_mode_ || n < par_min(65536) || n >= (1u << 31)) return 0;
    const auto& mts0 = sigs_[sig_[brow[0]]].must_terms;
    if (mts0.empty()) return 0;
    const uint16_t f0 = mts0[0].first;
    for (auto& mt : mts0)
        if (mt.first != f0) return 0;  // several key candidates: plan_pools
    if (f0 >= 63 || fkind_[f0].size() != nslots()) return 0;
    const size_t nd = dict_.size();
    if (nd >= (1u << 31)) return 0;
    constexpr uint32_t kForeign = 1u << 31, kTerm = kForeign - 1;
    std::atomic<uint32_t>* first = pool_first_table(nd);
    std::vector<uint32_t>& k1 = run_terms_;  // per row: term | kForeign
    grow_to(k1, n);
    grow_to(P.search_pool, n);
    const unsigned nch = wp.size() * 2;
    std::vector<uint8_t> bad(nch, 0);
    const uint64_t fbit = 1ull << f0;
    // the row's pool term and foreign flag (UINT32_MAX: plan_pools fails)
    auto term_of = [&](size_t i) -> uint32_t {
        const uint32_t r = brow[i];
        const uint32_t s = sig_[r];
        if (!(sig_fmask_[s] & fbit)) return UINT32_MAX;
        const bool self = self_match_[r] && indexed_[r];
        const bool kw = fkind_[f0][r] == KIND_KEYWORD;
        if (self && kw) return (uint32_t)fval_[f0][r];
        uint32_t t = UINT32_MAX;
        for (auto& mt : sigs_[s].must_terms)
            if (mt.first == f0) {
                if (t != UINT32_MAX && t != mt.second) return UINT32_MAX;
                t = mt.second;
            }
        if (t >= nd) return UINT32_MAX;
        if (self) return t;
        if (!kw || (uint32_t)fval_[f0][r] != t) return UINT32_MAX;  // not in its search's pool
        return t | kForeign;
    };
    {  // a prefix where a term comes back after its run (C2's interleaved
       // region pools): not this shape, decided before any sweep
        std::unordered_set<uint32_t> seen;
        uint32_t prev = UINT32_MAX;
        for (size_t i = 0; i < std::min<size_t>(n, 2048); i++) {
            const uint32_t k = term_of(i);
            if (k == UINT32_MAX) break;  // the sweeps report it
            const uint32_t t = k & kTerm;
            if (t != prev && !seen.insert(t).second) return 0;
            prev = t;
        }
    }
    auto reset_first = [&] {
        wp.run(nch, [&](size_t c) {
            for (size_t t = pool_first_cap_ * c / nch; t < pool_first_cap_ * (c + 1) / nch; t++)
                first[t].store(UINT32_MAX, std::memory_order_relaxed);
        });
    };
    wp.run(nch, [&](size_t c) {  // A
        const size_t lo = n * c / nch, hi = n * (c + 1) / nch;
        if (lo >= hi) return;
        uint32_t prev = lo ? term_of(lo - 1) : UINT32_MAX;
        if (prev != UINT32_MAX) prev &= kTerm;
        for (size_t i = lo; i < hi; i++) {
            const uint32_t k = term_of(i);
            if (k == UINT32_MAX || (k & kTerm) >= nd) { bad[c] = 1; return; }
            k1[i] = k;
            const uint32_t t = k & kTerm;
            if (t != prev) {
                uint32_t cur = first[t].load(std::memory_order_relaxed);
                while ((uint32_t)i < cur && !first[t].compare_exchange_weak(cur, (uint32_t)i, std::memory_order_relaxed)) {
                }
            }
            prev = t;
        }
    });
    if (std::any_of(bad.begin(), bad.end(), [](uint8_t b) { return b != 0; })) {
        reset_first();
        return -1;
    }
    std::vector<size_t> heads(nch + 1, 0), starts(nch + 1, 0);
    auto run_start = [&](size_t i) { return i == 0 || ((k1[i] ^ k1[i - 1]) & kTerm) != 0; };
    wp.run(nch, [&](size_t c) {  // B
        size_t h = 0, st = 0;
        for (size_t i = n * c / nch; i < n * (c + 1) / nch; i++)
            if (run_start(i)) {
                st++;
                h += first[k1[i] & kTerm].load(std::memory_order_relaxed) == (uint32_t)i;
            }
        heads[c + 1] = h;
        starts[c + 1] = st;
    });
    for (unsigned c = 0; c < nch; c++) {
        heads[c + 1] += heads[c];
        starts[c + 1] += starts[c];
    }
    const size_t ng = heads[nch];
    if (ng != starts[nch]) {  // a term returns after its run: plan_pools' counting sort
        wp.run(nch, [&](size_t c) {
            for (size_t i = n * c / nch; i < n * (c + 1) / nch; i++)
                if (run_start(i)) first[k1[i] & kTerm].store(UINT32_MAX, std::memory_order_relaxed);
        });
        return 0;
    }
    grow_to(P.pool_key1, ng);
    grow_to(P.self_rows, ng);
    grow_to(P.pool_off, ng + 1);
    grow_to(P.pool_rows, n);
    wp.run(nch, [&](size_t c) {  // C: the runs starting in [lo, hi), each to its end
        size_t p = heads[c];
        for (size_t i = n * c / nch; i < n * (c + 1) / nch; i++) {
            if (!run_start(i)) continue;
            const uint32_t t = k1[i] & kTerm;
            first[t].store(UINT32_MAX, std::memory_order_relaxed);
            P.pool_key1[p] = t;
            P.pool_off[p] = (uint32_t)i;
            uint32_t fo = 0;
            size_t j = i;
            for (; j < n && (k1[j] & kTerm) == t; j++) {
                fo |= k1[j];
                P.pool_rows[j] = (uint32_t)j;
            }
            P.self_rows[p] = (fo & kForeign) ? 0 : 1;
            for (size_t q = i; q < j; q++) P.search_pool[q] = (uint32_t)p;
            p++;
        }
    });
    P.pool_off[ng] = (uint32_t)n;
    stats.par_bucket_ms += std::chrono::duration<double, std::milli>(clk::now() - tp0).count();
    if (batch_profile_)
        std::fprintf(stderr, "[nkm]   plan_pools: %zu pools (contiguous runs, 3 sweeps) %.2f ms\n", ng,
                     std::chrono::duration<double, std::milli>(clk::now() - tp0).count());
    if (ng < 2) return -1;
    P.ng = ng;
    P.ok = true;
    P.runs = true;
    return 1;
}

// plan_pools over a packed batch: search i is batch row i (its ticket's
// signature), and every search is one row.
bool Core::plan_packed(size_t n, const UVec<uint32_t>& brow, ParPlan& P, PassStats& stats) {
    P.ok = false;
    P.runs = false;
    if (runs_mode_ && pruns_mode_) {
        const int k = plan_packed_runs(n, brow, P, stats);
        if (k != 0) return k > 0;
    }
    return plan_pools(
        n, [&](size_t i) { return sig_[brow[i]]; }, [](size_t bi) { return (uint32_t)bi; },
        [&](size_t i) { return brow[i]; }, brow, P, stats);
}

// The replay's search view of a packed batch's row bi (a thread-local
// BGroup refilled per row from the output buffer).
std::function<BGroup&(uint32_t)> Core::packed_view(const PackLayout& L, const UVec<uint32_t>& brow) {
    const uint8_t* base = h_pack_.p;
    return [this, base, L, &brow](uint32_t bi) -> BGroup& {
        static thread_local BGroup g;
        static thread_local uint32_t slots[64];
        const uint32_t T = brow[bi];
        const DSmallRow& d = h_srows_.p[bi];
        const uint32_t* src = ((d.src_len & kSrcOrder) ? order_.data() : postings_.data()) + d.src_off;
        fill_packed(g, base, L, bi, T, sig_[T], src, slots);
        g.d.src_len = d.src_len & ~kSrcOrder;  // the row's source (pairs decided)
        return g;
    };
}


}  // namespace nkm
