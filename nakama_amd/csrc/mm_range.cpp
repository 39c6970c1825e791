// nakama_amd/csrc/mm_range.cpp — range batches (range_walk.h): a pass whose
// remaining rows are all range-source searches (Sig::rs_field: a pool term and
// numeric ranges on one field, e.g. C2's skill windows with ^boost) is decided
// in ONE batch.  The device sorts every pool's candidates by their value and
// finds each signature's range bounds in that order (rsrc_tile / rsrc_merge /
// rsrc_bounds kernels); the host walks each pool's rows on its own worker
// with a min tree over the sorted candidates, so a row's next hit costs
// O(log n) instead of a walk over its hit list past every earlier selection
// (matchmaker_process.go:86-130 over bluge's numeric range searcher,
// bluge/search/searcher/search_numeric_range.go:26-83).  Pools are independent
// exactly as in the pool-parallel replay (plan_pools): rows of one pool only
// select tickets of that pool.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "mm_core.h"
#include "mm_pass.h"
#include "range_walk.h"

namespace nkm {

void Core::reset_pass_scratch() {
    for (size_t k = 0; k < rs_mark_cap_; k++) rs_mark_[k].store(0, std::memory_order_relaxed);
    for (size_t k = 0; k < pool_first_cap_; k++) pool_first_[k].store(UINT32_MAX, std::memory_order_relaxed);
    std::fill(rs_leaf_.begin(), rs_leaf_.end(), kNoSlot);
    std::fill(pos_of_.begin(), pos_of_.end(), kNoSlot);
    g_scratch_epoch.fetch_add(1, std::memory_order_relaxed);
}

bool Core::range_batch(const std::vector<uint32_t>& rows, size_t pos, GroupList& out_groups,
                       UVec<uint32_t>& expired, UVec<uint32_t>& newly, PassStats& stats) {
    using clk = std::chrono::steady_clock;
    auto msd = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto t0 = clk::now();
    std::vector<uint8_t>& sel = sel_;
    std::vector<uint8_t>& dec = dec_;
    size_t p0 = pos;
    while (p0 < rows.size() && (sel[rows[p0]] | dec[rows[p0]])) p0++;
    if (p0 >= rows.size() || sigs_[sig_[rows[p0]]].rs_field == Sig::kNoRange) return false;  // the common refusal: O(1)
    WorkPool& wp = workers();
    auto sweep = [&](size_t nch, auto&& fn) {
        if (nch > 1) wp.run(nch, fn);
        else fn(0);
    };
    // ---- the batch: every undecided row, each a range-source search of a pool
    // on the first row's key field, carrying its own pool's term ----
    const uint16_t kf = sigs_[sig_[rows[p0]]].must_terms[0].first;
    const size_t nr = rows.size() - p0;
    const size_t nch = par_mode_ && nr >= par_min(16384) ? wp.size() : 1;
    std::vector<size_t> at(nch + 1, 0);
    std::vector<uint8_t> bad(nch, 0);
    sweep(nch, [&](size_t c) {
        size_t k = 0;
        for (size_t i = p0 + nr * c / nch; i < p0 + nr * (c + 1) / nch; i++) {
            const uint32_t r = rows[i];
            if (sel[r] | dec[r]) continue;
            const Sig& s = sigs_[sig_[r]];
            if (s.rs_field == Sig::kNoRange || s.must_terms[0].first != kf || !self_match_[r] || !indexed_[r]) {
                bad[c] = 1;
                return;
            }
            k++;
        }
        at[c + 1] = k;
    });
    for (uint8_t b : bad)
        if (b) return false;
    for (size_t c = 0; c < nch; c++) at[c + 1] += at[c];
    UVec<uint32_t>& brow = brow_;
    const size_t nb = at[nch];
    grow_to(brow, nb);
    sweep(nch, [&](size_t c) {
        size_t o = at[c];
        for (size_t i = p0 + nr * c / nch; i < p0 + nr * (c + 1) / nch; i++)
            if (!(sel[rows[i]] | dec[rows[i]])) brow[o++] = rows[i];
    });
    // ---- pools: plan_pools with every row its own search (several pools), or
    // one pool when every row requires the same term ----
    const auto tp_rows = clk::now();
    ParPlan& P = par_plan_;
    if (!plan_packed(nb, brow, P, stats)) {
        const uint32_t t0term = sigs_[sig_[brow[0]]].must_terms[0].second;
        std::vector<uint8_t> other(nch, 0);
        sweep(nch, [&](size_t c) {
            for (size_t bi = nb * c / nch; bi < nb * (c + 1) / nch && !other[c]; bi++)
                other[c] = sigs_[sig_[brow[bi]]].must_terms[0].second != t0term;
        });
        for (uint8_t o : other)
            if (o) return false;
        P.ng = 1;
        grow_to(P.search_pool, nb);
        grow_to(P.pool_rows, nb);
        sweep(nch, [&](size_t c) {
            for (size_t bi = nb * c / nch; bi < nb * (c + 1) / nch; bi++) {
                P.search_pool[bi] = 0;
                P.pool_rows[bi] = (uint32_t)bi;
            }
        });
        P.pool_off.assign({0u, (uint32_t)nb});
        P.pool_key1.assign(1, t0term);
        P.ok = true;
    }
    const size_t ng = P.ng;
    if (P.pool_key1.size() < ng) return false;  // several key fields: not a range batch's pools
    // each pool's range field (its first row's), the same for all its rows
    if (rs_pools_.size() < ng) rs_pools_.resize(ng);
    for (size_t p = 0; p < ng; p++) {
        RangePoolHost& H = rs_pools_[p];
        H.term = P.pool_key1[p];
        H.field = sigs_[sig_[brow[P.pool_rows[P.pool_off[p]]]]].rs_field;
    }
    // From here on the batch is taken: nothing below declines but the
    // per-signature field check after the claims (every row's range field
    // must be its pool's; a row's pool is its signature's MUST term's).
    const auto tp_pools = clk::now();
    // ---- device, first: pools (posting ranges), tiles, block -> pool, and
    // the sort, which runs while the host claims the batch's signatures
    // below; the bound queries follow once those are known ----
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    uint64_t n_elems = 0, src_total = 0;
    uint32_t max_pad = 0, n_tiles = 0;
    for (size_t p = 0; p < ng; p++) {
        RangePoolHost& H = rs_pools_[p];
        DRangePool& d = H.d;
        d = DRangePool{};
        if (PostingRange* it = postings_map_.find(((uint64_t)kf << 32) | H.term)) {
            PostingRange& pr = *it;
            while (pr.head < pr.len && !live_[postings_[pr.off + pr.head]]) pr.head++;  // the dead prefix
            d.src_off = pr.off + pr.head;
            d.src_len = pr.len - pr.head;
        }
        d.out_off = (uint32_t)n_elems;
        d.pad_len = (uint32_t)al(d.src_len);
        d.field = H.field;
        n_elems += d.pad_len;
        src_total += d.src_len;
        max_pad = std::max(max_pad, d.pad_len);
        n_tiles += (d.pad_len + kRsrcTile - 1) / kRsrcTile;
    }
    if (n_elems >= (1ull << 31)) throw std::runtime_error("range batch: more than 2^31 candidates");
    const size_t o_tiles = al(ng * sizeof(DRangePool)), o_blk = o_tiles + al((size_t)n_tiles * sizeof(DRangeTile)),
                 blob = o_blk + al((size_t)(n_elems / 256) * 4);
    h_rblob_.reserve(blob);
    d_rblob_.reserve(blob, false);
    DRangePool* hp = reinterpret_cast<DRangePool*>(h_rblob_.p);
    DRangeTile* ht = reinterpret_cast<DRangeTile*>(h_rblob_.p + o_tiles);
    uint32_t* hb = reinterpret_cast<uint32_t*>(h_rblob_.p + o_blk);
    for (size_t p = 0, t = 0; p < ng; p++) {
        const DRangePool& d = rs_pools_[p].d;
        hp[p] = d;
        for (uint32_t s0 = 0; s0 < d.pad_len; s0 += kRsrcTile)
            ht[t++] = DRangeTile{(uint32_t)p, s0, std::min(kRsrcTile, d.pad_len - s0), 0};
        for (uint32_t b = 0; b < d.pad_len / 256; b++) hb[d.out_off / 256 + b] = (uint32_t)p;
    }
    flush_apply();  // earlier batches' selections, before the candidates are read
    for (auto& a : d_rkey_) a.reserve(std::max<uint64_t>(n_elems, 1), false);
    for (auto& a : d_rpos_) a.reserve(std::max<uint64_t>(n_elems, 1), false);
    h_rpos_.reserve(std::max<uint64_t>(n_elems, 1));
    if (!rs_ev_[0])
        for (auto& e : rs_ev_) NKM_HIP(hipEventCreate(&e));
    NKM_HIP(hipMemcpyAsync(d_rblob_.p, h_rblob_.p, blob, hipMemcpyHostToDevice, stream_));
    int which = 0, n_merge = 0;
    int64_t* dk[2] = {d_rkey_[0].p, d_rkey_[1].p};
    uint32_t* dp[2] = {d_rpos_[0].p, d_rpos_[1].p};
    const uint8_t* db = d_rblob_.p;
    const DRangePool* d_pools = reinterpret_cast<const DRangePool*>(db);
    NKM_HIP(launch_rsrc(dstore(), d_pools, max_pad, reinterpret_cast<const DRangeTile*>(db + o_tiles), n_tiles,
                        reinterpret_cast<const uint32_t*>(db + o_blk), (uint32_t)n_elems, dk, dp, nullptr, 0, nullptr,
                        &which, stream_, rs_ev_[0], rs_ev_[1], rs_ev_ + 2, kRsrcMaxMerge, &n_merge));
    if (n_elems) NKM_HIP(hipMemcpyAsync(h_rpos_.p, d_rpos_[which].p, n_elems * 4, hipMemcpyDeviceToHost, stream_));
    const auto tp_sort = clk::now();
    // ---- the batch's signatures (each claimed once, by an atomic flag) ----
    const size_t nsig = sigs_.size();
    if (rs_mark_cap_ < nsig) {
        rs_mark_cap_ = nsig + nsig / 4;
        rs_mark_.reset(new std::atomic<uint8_t>[rs_mark_cap_]);
        for (size_t k = 0; k < rs_mark_cap_; k++) rs_mark_[k].store(0, std::memory_order_relaxed);
    }
    std::vector<std::vector<uint32_t>> claimed(nch);
    sweep(nch, [&](size_t c) {
        std::vector<uint32_t> mine;  // thread-private (the chunks' vector headers share cache lines)
        for (size_t bi = nb * c / nch; bi < nb * (c + 1) / nch; bi++) {
            const uint32_t sg = sig_[brow[bi]];
            if (!rs_mark_[sg].load(std::memory_order_relaxed) && !rs_mark_[sg].exchange(1, std::memory_order_relaxed))
                mine.push_back(sg);
        }
        claimed[c] = std::move(mine);
    });
    std::vector<uint32_t> lsig;
    for (auto& v : claimed) lsig.insert(lsig.end(), v.begin(), v.end());
    if (rs_sig_loc_.size() < nsig) grow_to(rs_sig_loc_, nsig);
    // per batch signature: its pool and its first bound query
    const size_t ns = lsig.size();
    std::vector<uint32_t> ls_pool(ns), ls_q(ns + 1, 0);
    const size_t sch = ns >= 4096 ? nch : 1;
    std::vector<uint8_t> field_bad(sch, 0);
    sweep(sch, [&](size_t c) {
        bool fb = false;
        for (size_t k = ns * c / sch; k < ns * (c + 1) / sch; k++) {
            const uint32_t sg = lsig[k];
            rs_sig_loc_[sg] = (uint32_t)k;
            const Sig& s = sigs_[sg];
            ls_pool[k] = ng == 1 ? 0u : pool_remap_[s.must_terms[0].second];
            ls_q[k + 1] = 2 * (uint32_t)s.rs_nrange;
            fb |= s.rs_field != rs_pools_[ls_pool[k]].field;
        }
        field_bad[c] = fb;
    });
    if (std::any_of(field_bad.begin(), field_bad.end(), [](uint8_t b) { return b != 0; })) {
        // declined: the claims are released; the sort issued above wrote only
        // the range buffers, and is waited for here
        for (size_t k = 0; k < ns; k++) rs_mark_[lsig[k]].store(0, std::memory_order_relaxed);
        NKM_HIP(hipStreamSynchronize(stream_));
        return false;
    }
    for (size_t k = 0; k < ns; k++) ls_q[k + 1] += ls_q[k];
    const uint32_t nq = ls_q[ns];
    const auto tp_sigs = clk::now();
    // ---- device, then: the bound queries over the sorted keys ----
    const size_t qbytes = std::max<size_t>((size_t)nq * sizeof(DRangeBound), sizeof(DRangeBound));
    h_rq_.reserve(qbytes);
    d_rq_.reserve(qbytes, false);
    d_rbound_.reserve(std::max<uint32_t>(nq, 1), false);
    h_rbound_.reserve(std::max<uint32_t>(nq, 1));
    DRangeBound* hq = reinterpret_cast<DRangeBound*>(h_rq_.p);
    const size_t qch = ns >= 4096 ? nch : 1;
    sweep(qch, [&](size_t c) {
        for (size_t k = ns * c / qch; k < ns * (c + 1) / qch; k++) {
            const Sig& s = sigs_[lsig[k]];
            uint32_t q = ls_q[k];
            for (uint32_t i = 0; i < s.n_clauses; i++) {
                const DClause& cl = clauses_[s.clause_off + i];
                if (cl.op != OP_RANGE) continue;
                hq[q++] = DRangeBound{cl.lo, ls_pool[k], 0};
                hq[q++] = DRangeBound{cl.hi, ls_pool[k], 1};
            }
        }
    });
    const auto t1 = clk::now();
    if (nq && n_elems && n_tiles) {
        NKM_HIP(hipMemcpyAsync(d_rq_.p, h_rq_.p, (size_t)nq * sizeof(DRangeBound), hipMemcpyHostToDevice, stream_));
        NKM_HIP(launch_rsrc_bounds(d_pools, dk[which], reinterpret_cast<const DRangeBound*>(d_rq_.p), nq, d_rbound_.p,
                                   stream_));
        NKM_HIP(hipMemcpyAsync(h_rbound_.p, d_rbound_.p, (size_t)nq * 4, hipMemcpyDeviceToHost, stream_));
    } else if (nq) {
        std::memset(h_rbound_.p, 0, (size_t)nq * 4);  // no candidates: every bound is 0 (build_tiers clamps to 0 anyway)
    }
    NKM_HIP(hipStreamSynchronize(stream_));
    const auto t2 = clk::now();
    stats.batches++;
    stats.parallel_batches++;
    if (n_tiles) {
        float ms = 0.f;
        NKM_HIP(hipEventElapsedTime(&ms, rs_ev_[0], rs_ev_[1]));
        stats.k_ms[5] += ms;
        stats.k_launches[5]++;
    }
    for (int m = 0; m < n_merge; m++) {
        float ms = 0.f;
        NKM_HIP(hipEventElapsedTime(&ms, rs_ev_[2 + 2 * m], rs_ev_[3 + 2 * m]));
        stats.k_ms[4] += ms;
        stats.k_launches[4]++;
    }
    // ---- host: each pool's sorted candidates, min tree, then its rows' walk ----
    if (rs_leaf_.size() < nslots()) rs_leaf_.resize(nslots(), kNoSlot);
    const ReplayView rv = replay_view();
    const int maxI = cfg_.max_intervals;
    auto prows = [&](size_t p) { return P.pool_off[p + 1] - P.pool_off[p]; };
    std::vector<uint32_t> order_p(ng);
    for (size_t p = 0; p < ng; p++) order_p[p] = (uint32_t)p;
    if (ng <= 4096) std::sort(order_p.begin(), order_p.end(), [&](uint32_t a, uint32_t b) { return prows(a) > prows(b); });
    const size_t per_task = std::max<size_t>(1, nb / ((size_t)wp.size() * 8));
    std::vector<uint32_t> task_off{0};
    for (size_t k = 0, acc = 0; k < ng; k++) {
        acc += prows(order_p[k]);
        if (acc >= per_task || k + 1 == ng) {
            task_off.push_back((uint32_t)(k + 1));
            acc = 0;
        }
    }
    const size_t ntask = task_off.size() - 1;
    const bool few = ng <= 64;
    if (few && pool_outs_.size() < ng) pool_outs_.resize(ng);
    if (!few && row_recs_.size() < nb) grow_to(row_recs_, nb);
    if (task_ents_.size() < ntask) task_ents_.resize(ntask);
    RowRec* rr = few ? nullptr : row_recs_.data();
    if (!few) std::memset((void*)rr, 0, nb * sizeof(RowRec));
    std::vector<uint64_t> task_hits(ntask, 0), task_pairs(ntask, 0);
    std::vector<double> pool_build_ms(ng, 0.0), pool_walk_ms(ng, 0.0);  // NKM_PROFILE=2
    // each pool's valid candidates: a prefix of its sorted elements
    std::vector<uint32_t> valid(ng, 0);
    for (size_t p = 0; p < ng; p++) {
        const DRangePool& d = rs_pools_[p].d;
        const uint32_t* pv = h_rpos_.p + d.out_off;
        uint32_t lo = 0, hi = d.pad_len;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (pv[mid] & kRsrcInvalid) hi = mid;
            else lo = mid + 1;
        }
        valid[p] = lo;
    }
    // every signature's tiers (on all the workers, before the walks): at most
    // 2 x ranges + 1 intervals each, at its own offset of one flat array
    const uint32_t* hbound = h_rbound_.p;
    std::vector<uint32_t> ls_t0(ns), ls_t1(ns);
    for (size_t k = 0; k < ns; k++) ls_t0[k] = ls_q[k] + (uint32_t)k;
    grow_to(rs_tiers_, (size_t)nq + ns);
    const size_t tch = ns >= 512 ? (size_t)wp.size() * 2 : 1;
    // every pool's leaves (slot, rank, HotRec and Intervals copies, the
    // slot -> leaf maps), in pieces, by the pool's walker before its walk (the
    // walk then finds them in this core's cache; gathering them across the
    // workers measured slower on C2 — its walks then read other cores' lines:
    // slowest walk 1.7 -> 2.0-2.7 ms, profiles/r05/r05j)
    constexpr uint32_t kLeafPiece = 4096;
    std::vector<uint64_t> piece_at{0};  // pools' pieces, prefix
    for (size_t p = 0; p < ng; p++) {
        RangePoolHost& H = rs_pools_[p];
        const uint32_t nv = valid[p];
        grow_to(H.slot, nv);
        grow_to(H.rank, nv);
        grow_to(H.leaf_of, H.d.src_len);
        grow_to(H.lhot, nv);
        grow_to(H.livl, nv);
        piece_at.push_back(piece_at.back() + (nv + kLeafPiece - 1) / kLeafPiece);
    }
    const size_t npiece = piece_at.back();
    std::vector<uint8_t> leaf_bad(npiece, 0);
    auto leaf_piece = [&](size_t t) {
        const size_t p = (size_t)(std::upper_bound(piece_at.begin(), piece_at.end(), (uint64_t)t) - piece_at.begin()) - 1;
        RangePoolHost& H = rs_pools_[p];
        const DRangePool& d = H.d;
        const uint32_t* pv = h_rpos_.p + d.out_off;
        const uint32_t j0 = (uint32_t)(t - piece_at[p]) * kLeafPiece, j1 = std::min(valid[p], j0 + kLeafPiece);
        for (uint32_t j = j0; j < j1; j++) {
            const uint32_t rk = pv[j];
            if (rk >= d.src_len) { leaf_bad[t] = 1; return; }
            if (j + 8 < j1 && pv[j + 8] < d.src_len) {
                const uint32_t s8 = postings_[d.src_off + pv[j + 8]];
                __builtin_prefetch(&hot_[s8]);
                __builtin_prefetch(&intervals_[s8]);
            }
            const uint32_t s = postings_[d.src_off + rk];
            H.rank[j] = rk;
            H.slot[j] = s;
            H.leaf_of[rk] = j;
            rs_leaf_[s] = j;
            H.lhot[j] = hot_[s];
            H.livl[j] = intervals_[s];
        }
    };
    auto tier_chunk = [&](size_t c) {
        static thread_local std::vector<RRange> tmp;
        for (size_t k = ns * c / tch; k < ns * (c + 1) / tch; k++) {
            const Sig& s = sigs_[lsig[k]];
            uint32_t blo[32], bhi[32];
            const uint32_t nrg = (ls_q[k + 1] - ls_q[k]) / 2;
            for (uint32_t q = 0; q < nrg; q++) {
                blo[q] = hbound[ls_q[k] + 2 * q];
                bhi[q] = hbound[ls_q[k] + 2 * q + 1];
            }
            tmp.clear();
            build_tiers(clauses_.data() + s.clause_off, s.n_clauses, blo, bhi, valid[ls_pool[k]], tmp);
            RRange* o = rs_tiers_.data() + ls_t0[k];
            for (size_t q = 0; q < tmp.size(); q++) o[q] = RRange{tmp[q].a, tmp[q].b, tmp[q].tend + ls_t0[k]};
            ls_t1[k] = ls_t0[k] + (uint32_t)tmp.size();
        }
    };
    // The tiers and the pools' leaf builds are independent: with a thread to
    // spare beyond the walk tasks, one job runs both — the walk tasks first
    // (claimed in index order, so the tier chunks are claimed by the other
    // threads and always finish), each building its pools' leaves while the
    // tiers are built and waiting for all of them before its first walk.
    const bool tier_overlap = tch > 1 && ntask < wp.size();
    std::atomic<size_t> tiers_done{0};
    std::atomic<bool> tiers_failed{false};
    if (!tier_overlap) sweep(tch, tier_chunk);
    const auto t2b = clk::now();
    auto worker = [&](size_t t) {
        static thread_local TlFlags tl;
        tl.ready(sel.size(), g_scratch_epoch.load(std::memory_order_relaxed));
        std::vector<uint8_t>& tl_sel = tl.sel;
        std::vector<uint8_t>& tl_proc = tl.proc;
        static thread_local RangeRun run{};
        run.v = rv;
        run.max_intervals = maxI;
        run.psel = tl_sel.data();
        run.proc = tl_proc.data();
        run.leaf_of_slot = rs_leaf_.data();
        run.fast = fast_mode_;
        run.hits_seen = 0;
        static thread_local PoolOut o;
        auto& ents = task_ents_[t];
        ents.clear();
        uint64_t pairs = 0;
        for (uint32_t k = task_off[t]; k < task_off[t + 1]; k++) {
            const uint32_t p = order_p[k];
            RangePoolHost& H = rs_pools_[p];
            const DRangePool& d = H.d;
            const auto tb0 = clk::now();
            const uint32_t nv = valid[p];
            bool bad = false;
            for (uint64_t q = piece_at[p]; q < piece_at[p + 1]; q++) {
                leaf_piece(q);
                bad |= leaf_bad[q] != 0;
            }
            if (bad) {
                // a device position out of range: this pool is not walked (its
                // copies are partly unfilled); the leaf map entries its pieces
                // did set are cleared, and the error is raised after the job
                const uint32_t* pv = h_rpos_.p + d.out_off;
                for (uint64_t q = piece_at[p]; q < piece_at[p + 1]; q++) {
                    const uint32_t j0 = (uint32_t)(q - piece_at[p]) * kLeafPiece, j1 = std::min(nv, j0 + kLeafPiece);
                    for (uint32_t j = j0; j < j1 && pv[j] < d.src_len; j++) rs_leaf_[postings_[d.src_off + pv[j]]] = kNoSlot;
                }
                continue;
            }
            H.src.n = nv;
            H.src.slot = H.slot.data();
            H.src.rank = H.rank.data();
            H.src.leaf_of = H.leaf_of.data();
            H.src.lhot = H.lhot.data();
            H.src.livl = H.livl.data();
            H.src.tree.build(H.rank.data(), nv);
            const auto tb1 = clk::now();
            if (tier_overlap) {
                while (tiers_done.load(std::memory_order_acquire) < tch) __builtin_ia32_pause();
                if (tiers_failed.load(std::memory_order_acquire)) return;  // the tier chunk's exception ends the pass
            }
            const auto tw = clk::now();
            PoolOut& po = few ? pool_outs_[p] : o;
            po.recs.clear();
            po.ents.clear();
            run.walk(H.src, P.pool_rows.data() + P.pool_off[p], (uint32_t)prows(p), brow.data(),
                     [&](uint32_t bi, const RRange*& base, uint32_t& r0, uint32_t& r1) {
                         const uint32_t ls = rs_sig_loc_[sig_[brow[bi]]];
                         base = rs_tiers_.data();
                         r0 = ls_t0[ls];
                         r1 = ls_t1[ls];
                     },
                     po);
            pool_walk_ms[p] = msd(tw, clk::now());
            pairs += (uint64_t)(po.recs.size() - 1) * d.src_len;  // rows that searched (the last record is the sentinel)
            pool_build_ms[p] = msd(tb0, tb1);
            for (uint32_t j = 0; j < nv; j++) rs_leaf_[H.slot[j]] = kNoSlot;
            if (!few) {
                const uint32_t base = (uint32_t)ents.size();
                ents.insert(ents.end(), o.ents.begin(), o.ents.end());
                for (size_t q = 0; q + 1 < o.recs.size(); q++) {  // the last record is the sentinel
                    const PoolRec& r = o.recs[q];
                    rr[r.bi] = RowRec{base + r.off, r.len, (uint32_t)t, r.matched, r.expired, 1, 0};
                }
            }
        }
        task_hits[t] = run.hits_seen;
        task_pairs[t] = pairs;
    };
    if (tier_overlap) {
        wp.run(ntask + tch, [&](size_t i) {
            if (i < ntask) {
                worker(i);
                return;
            }
            // counted done even when it throws (the walks wait on the count)
            struct Count {
                std::atomic<size_t>& n;
                ~Count() { n.fetch_add(1, std::memory_order_release); }
            } count{tiers_done};
            try {
                tier_chunk(i - ntask);
            } catch (...) {
                tiers_failed.store(true, std::memory_order_release);
                throw;
            }
        });
    } else {
        wp.run(ntask, worker);
    }
    for (uint8_t b : leaf_bad)
        if (b) throw DeviceError{hipErrorUnknown, "range source: a sorted position out of range", __LINE__};
    const auto t3 = clk::now();
    for (size_t k = 0; k < ns; k++) rs_mark_[lsig[k]].store(0, std::memory_order_relaxed);
    const size_t mch = nb >= par_min(65536) ? (size_t)wp.size() * 2 : 1;
    if (few) merge_pools(ng, mch, brow, sel, out_groups, expired, newly);
    else merge_rows(nb, mch, brow, sel, out_groups, expired, newly);
    const auto t4 = clk::now();
    // algorithmic bytes: the tile kernel reads every source entry's slot id and
    // alive flag (5 B), the valid candidates' kind and value (9 B), and writes
    // each element's key and position (12 B); a merge reads and writes them
    uint64_t nvalid = 0;
    for (uint32_t v : valid) nvalid += v;
    stats.k_bytes[5] += (int64_t)(src_total * 5 + nvalid * 9 + n_elems * 12);
    stats.k_bytes[4] += (int64_t)(n_merge * n_elems * 24);
    stats.pair_evals += (int64_t)src_total;
    for (uint64_t q : task_pairs) stats.pairs_decided += (int64_t)q;
    for (uint64_t h : task_hits) stats.par_hits += h;
    stats.par_rows += nb;
    stats.assemble_ms += msd(t0, t1);
    stats.search_ms += msd(t1, t2);
    stats.replay_ms += msd(t2, t4);
    stats.par_gather_ms += msd(t2, t2b);
    stats.par_work_ms += msd(t2, t3);
    stats.par_merge_ms += msd(t3, t4);
    if (batch_profile_) {
        const size_t pm = (size_t)(std::max_element(pool_walk_ms.begin(), pool_walk_ms.end()) - pool_walk_ms.begin());
        std::fprintf(stderr,
                     "[nkm]   batch %d (range): rows %zu pools %zu signatures %zu candidates %llu (valid %llu), %d merges "
                     "| plan %.2f (rows %.2f pools %.2f sort issue %.2f signatures %.2f queries %.2f) device %.2f "
                     "tiers %.2f walks %.2f merge %.2f ms | slowest pool: %u rows, build %.2f walk %.2f ms\n",
                     stats.batches, nb, ng, ns, (unsigned long long)src_total, (unsigned long long)nvalid, n_merge,
                     msd(t0, t1), msd(t0, tp_rows), msd(tp_rows, tp_pools), msd(tp_pools, tp_sort),
                     msd(tp_sort, tp_sigs), msd(tp_sigs, t1),
                     msd(t1, t2), msd(t2, t2b), msd(t2b, t3), msd(t3, t4), (unsigned)prows(pm),
                     pool_build_ms[pm], pool_walk_ms[pm]);
    }
    return true;
}

}  // namespace nkm
