// nakama_amd/csrc/mm_process.cpp — the interval pass.
//
// Process() (server/matchmaker.go:282-372) with processDefault
// (server/matchmaker_process.go:27-334) restated as:
//   1. batch the active tickets in the pinned (CreatedAt, Ticket) order;
//   2. one device search per compiled signature present in the batch
//      (mm_kernels.hip), returning hit lists already sorted the way bluge's
//      TopN collector sorts them (-score, created_at, doc order);
//   3. an exact host replay of the greedy grouping over those lists.
// Tickets selected earlier in the batch are skipped in the lists (the
// reference deletes them from the index before the next search, and deleting
// never reorders the remaining hits).  When a list runs out before the row is
// decided, the batch ends there and the next batch re-runs the search with the
// device alive mask up to date; the first row of a batch may page further
// through its list with a cursor, so every batch makes progress.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <stdexcept>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <map>

#include "gocompat.h"
#include "mm_core.h"
#include "mm_pass.h"

namespace nkm {

hipError_t launch_pairmat(const DStore& st, const DGroup* d_groups, const DGroupResult* d_res, int n_groups,
                          const DHit* d_out, uint32_t* d_pm, hipStream_t stream);

struct Replay : ReplayCore {
    Core& c;
    PassStats& stats;
    DStore st;
    hipStream_t stream;
    // processCustom: every batch row searches (pairs decided counted per batch);
    // processDefault counts the rows that searched as they are decided
    bool all_rows_search = false;

    static ReplayView view(const Core& core) {
        return ReplayView{core.hot_.data(), core.pres_sess_.data(), core.party_.data(), core.intervals_.data(),
                          core.live_.data(), core.count_.data(), core.created_.data(), core.sess_slots_.more.empty()};
    }
    Replay(Core& core, std::vector<uint8_t>& s, bool r, int mi, PassStats& ps, DStore ds, hipStream_t sm)
        : ReplayCore(view(core), s, r, mi), c(core), stats(ps), st(ds), stream(sm), lg(core.lg_),
          lg_group(core.lg_group_) {
        fast = core.fast_mode_;
    }

    // Fetches the next page of a group's list (cursor = its last entry).
    void fetch_more(BGroup& g) override {
        stats.refetches++;
        // A slot list (run_batch's packed lists) becomes a DHit list: its
        // entries' slots, and as the last entry the cursor the batch kept
        // (Core::h_last_) — the only entry whose key and position are read.
        if (!g.hits && g.sp && g.n) {
            if (g.last_i == UINT32_MAX)  // an mscan list: complete by construction
                throw DeviceError{hipErrorUnknown, "page of a slot list without a cursor", __LINE__};
            g.ext.resize(g.n);
            for (uint32_t k = 0; k < g.n; k++) g.ext[k] = DHit{g.sp[k], 0u, 0};
            g.ext[g.n - 1] = c.h_last_.p[g.last_i];
            if (g.rev) g.ext_rev.assign(g.rev, g.rev + g.n);
            g.set_hits(g.ext.data());
        } else if (g.ext.empty() && g.n) {
            g.ext.assign(g.hits, g.hits + g.n);
            if (g.rev) g.ext_rev.assign(g.rev, g.rev + g.n);
        }
        DGroup d = g.d;
        d.out_off = 0;
        d.has_cursor = g.n ? 1 : 0;
        if (g.n) {
            d.cur_key = g.hits[g.n - 1].key;
            d.cur_idx = g.hits[g.n - 1].idx;
        }
        // constant-score pages double, but never past the rest of the source
        d.k = d.var_score ? (uint32_t)var_k_capacity()
                          : std::min<uint32_t>(std::max<uint32_t>(4096, 2 * d.k), std::max<uint32_t>(d.src_len, 1));
        c.h_groups_.reserve(1);
        c.h_groups_.p[0] = d;
        c.d_groups_.reserve(1, false);
        c.d_out_.reserve(d.k, false);
        c.d_rev_.reserve(d.k, false);
        c.d_res_.reserve(1, false);
        NKM_HIP(hipMemcpyAsync(c.d_groups_.p, c.h_groups_.p, sizeof(DGroup), hipMemcpyHostToDevice, stream));
        NKM_HIP(launch_search(st, c.d_groups_.p, 1, c.d_out_.p, rev ? c.d_rev_.p : nullptr, c.d_res_.p, stream,
                              c.ev_[0], c.ev_[1], d.var_score ? 2 : 1));
        c.h_res_.reserve(1);
        NKM_HIP(hipMemcpyAsync(c.h_res_.p, c.d_res_.p, sizeof(DGroupResult), hipMemcpyDeviceToHost, stream));
        // up to kPage1 entries come back in the same round trip (pinned); a
        // larger page copies the rest once its count is known
        constexpr uint32_t kPage1 = 4096;
        const uint32_t first = std::min(d.k, kPage1);
        c.h_page_.reserve(d.k);
        NKM_HIP(hipMemcpyAsync(c.h_page_.p, c.d_out_.p, (size_t)first * sizeof(DHit), hipMemcpyDeviceToHost, stream));
        if (rev) {
            c.h_page_rev_.reserve(d.k);
            NKM_HIP(hipMemcpyAsync(c.h_page_rev_.p, c.d_rev_.p, first, hipMemcpyDeviceToHost, stream));
        }
        NKM_HIP(hipStreamSynchronize(stream));
        if (c.h_res_.p[0].count > first) {
            const uint32_t rest = c.h_res_.p[0].count - first;
            NKM_HIP(hipMemcpyAsync(c.h_page_.p + first, c.d_out_.p + first, (size_t)rest * sizeof(DHit),
                                   hipMemcpyDeviceToHost, stream));
            if (rev)
                NKM_HIP(hipMemcpyAsync(c.h_page_rev_.p + first, c.d_rev_.p + first, rest, hipMemcpyDeviceToHost, stream));
            NKM_HIP(hipStreamSynchronize(stream));
        }
        float ms = 0.f;
        NKM_HIP(hipEventElapsedTime(&ms, c.ev_[0], c.ev_[1]));
        stats.k_ms[0] += ms;
        const DGroupResult r = c.h_res_.p[0];
        stats.pair_evals += r.scanned;
        stats.k_bytes[0] += search_bytes(c.sigs_[g.sig].n_fields, d, r);
        stats.k_launches[0]++;
        g.ext.insert(g.ext.end(), c.h_page_.p, c.h_page_.p + r.count);
        if (rev) g.ext_rev.insert(g.ext_rev.end(), c.h_page_rev_.p, c.h_page_rev_.p + r.count);
        g.set_hits(g.ext.data());
        g.rev = rev ? g.ext_rev.data() : nullptr;
        g.n = (uint32_t)g.ext.size();
        g.complete = r.complete != 0;
        g.d.k = d.k;
    }

    // Runs one batch of searches, each on one of three kernels:
    //  * mscan_kernel: the batch's large constant-score searches, when they
    //    together cover at least half of the scan order and read <= 4 fields:
    //    one pass over the scan order evaluates all of them (DMScan);
    //  * scan_kernel: other large constant-score searches, split into chunks
    //    of their posting list (one workgroup per chunk);
    //  * search_kernel: everything else, one workgroup per search (top-K for
    //    variable scores, RevPrecision, cursors).
    // stitch_kernel places the chunk outputs of the first two back in source
    // order on the device — the hit order when every hit scores the same.
    // d_groups_ holds [whole searches, chunks]; d_res_ holds [whole searches,
    // chunks, mscan (signature x chunk) cells]; d_out_ holds every search's
    // output region.
    std::vector<DGroup>& lg;                // whole searches, then chunks (Core::lg_: capacity kept)
    std::vector<uint32_t>& lg_group;        // owning BGroup of each entry of lg
    std::vector<DChunkMap> lmap;            // per chunk, then per mscan cell
    std::vector<uint32_t> cg_list;          // chunked / mscan BGroups, in order
    std::vector<uint64_t> cg_off;           // their output offsets in d_out_
    std::vector<uint32_t> cg_first, cg_end; // their result cells (indexes into d_res_ after the whole searches)
    std::vector<uint32_t> m_list;           // BGroups on mscan_kernel
    std::vector<DClause> mcl;               // their clauses, field = index into DMScan::field
    std::vector<DMSig> msig;
    std::vector<uint32_t> small_rows;       // rsmall_kernel's searches (indexes into lg)

    // The mscan descriptor of one search; a term-only signature gets its
    // required values per scanned field and its hit key, summed exactly as
    // the device sums clause scores (clause order, from 0.0; then +1 +1 for
    // the min/max count musts).
    DMSig make_msig(const DGroup& d, uint32_t clause_off) const {
        DMSig m{};
        m.tmin = d.tmin;
        m.tmax = d.tmax;
        m.clause_off = clause_off;
        m.n_clauses = d.n_clauses;
        m.qkind = d.qkind;
        bool term_only = d.qkind == QK_BOOL && d.n_clauses > 0;
        double ms = 0.0;
        for (uint32_t k = 0; k < d.n_clauses && term_only; k++) {
            const DClause& cl = mcl[clause_off + k];
            if (cl.op != OP_TERM || cl.occur != OCC_MUST) { term_only = false; break; }
            const int64_t want = (int64_t)cl.term;
            if ((m.req_mask >> cl.field) & 1u) {
                if (m.req[cl.field] != want) m.qkind = QK_MATCHNONE;  // two different terms on one field
            } else {
                m.req_mask |= (uint8_t)(1u << cl.field);
                m.req[cl.field] = want;
            }
            ms += cl.score;
        }
        if (!term_only) {
            m.qkind = d.qkind;
            m.req_mask = 0;
            for (auto& r : m.req) r = 0;
            return m;
        }
        m.term_only = m.qkind == QK_MATCHNONE ? 0 : 1;
        m.key = sortable_i64((ms + 1.0) + 1.0);
        return m;
    }

    // Picks the searches for mscan_kernel (see above); fills m_list / mcl / ms.
    bool plan_mscan(const std::vector<BGroup>& bg, uint32_t chunk, DMScan& ms) {
        m_list.clear();
        mcl.clear();
        const int km = c.kernel_mode_;
        if (rev || km == Core::KM_SEARCH || km == Core::KM_SCAN || c.order_head_ >= c.order_.size() ||
            c.shard_world_ > (int)kMaxShardBlocks)
            return false;
        const bool any_size = km == Core::KM_MSCAN;
        const uint64_t order_len = c.order_.size() - c.order_head_;
        uint64_t covered = 0;
        std::vector<uint16_t> fields;
        for (uint32_t i = 0; i < bg.size(); i++) {
            const DGroup& d = bg[i].d;
            if (d.var_score || d.has_cursor || d.tparty != kNoParty) continue;
            if (!any_size && (d.src_len <= chunk || d.k <= chunk / 4)) continue;
            const Sig& sg = c.sigs_[bg[i].sig];
            for (uint32_t k = 0; k < sg.n_clauses; k++) {
                const DClause& cl = c.clauses_[sg.clause_off + k];
                if (cl.op != OP_FALSE && std::find(fields.begin(), fields.end(), cl.field) == fields.end())
                    fields.push_back(cl.field);
            }
            m_list.push_back(i);
            covered += d.src_len;
        }
        size_t nclauses = 0;
        for (uint32_t i : m_list) nclauses += c.sigs_[bg[i].sig].n_clauses;
        if (m_list.empty() || m_list.size() > (size_t)kMHashSigs || fields.size() > (size_t)mscan_max_fields() ||
            (!any_size && 2 * covered < order_len)) {
            m_list.clear();
            return false;
        }
        ms = DMScan{};
        ms.src_off = c.order_head_;
        ms.src_len = (uint32_t)order_len;
        ms.n_sigs = (uint32_t)m_list.size();
        ms.n_fields = (uint32_t)fields.size();
        ms.n_clauses = (uint32_t)nclauses;
        for (size_t f = 0; f < fields.size(); f++) ms.field[f] = fields[f];
        msig.clear();
        for (uint32_t i : m_list) {
            const Sig& sg = c.sigs_[bg[i].sig];
            const uint32_t off = (uint32_t)mcl.size();
            for (uint32_t k = 0; k < sg.n_clauses; k++) {
                DClause cl = c.clauses_[sg.clause_off + k];
                cl.field = cl.op == OP_FALSE ? 0
                                             : (uint16_t)(std::find(fields.begin(), fields.end(), cl.field) - fields.begin());
                mcl.push_back(cl);
            }
            msig.push_back(make_msig(bg[i].d, off));
        }
        // The hashed lookup, when every signature is term-only on the same
        // fields with distinct values: past mscan_kernel's 16 signatures, when
        // the scan is contiguous (its vector loads: C3 1M 15.1-15.9 us against
        // mscan_kernel's 16.1-18.9 us on the same box, profiles/r03km_*), or
        // on request (NKM_MHASH=1; 2: never)
        // Row-sharded: the hashed scan only — each rank scans one block of
        // the chunks, and the blocks' per-chunk outputs are all-gathered
        // before every rank places the lists (run_batch).
        const bool hashable = plan_mscan_hash(ms);
        const bool contig_ok = c.order_identity_ && c.mcontig_mode_;
        if (ms.n_sigs > (uint32_t)mscan_max_sigs() || nclauses > (size_t)mscan_max_clauses() || c.mhash_mode_ == 1 ||
            (c.mhash_mode_ == 0 && hashable && contig_ok) || c.row_shard()) {
            if (!hashable) {
                m_list.clear();
                mcl.clear();
                msig.clear();
                return false;
            }
        } else {
            ms.hmask = 0;
            ms.dsize = 0;
            htab.clear();
            dgrid.clear();
        }
        ms.contig = ms.hmask && c.order_identity_ && c.mcontig_mode_ ? 1u : 0u;
        ms.chunk = (uint32_t)(ms.hmask ? mscan_hash_chunk_len(ms.contig != 0) : mscan_chunk_len(ms.n_sigs));
        if (ms.contig) {  // chunks: slot ranges aligned to the chunk length
            const uint64_t g0 = ms.src_off & ~(uint64_t)(ms.chunk - 1);
            ms.n_chunks = (uint32_t)(((uint64_t)ms.src_off + ms.src_len - g0 + ms.chunk - 1) / ms.chunk);
        } else {
            ms.n_chunks = (ms.src_len + ms.chunk - 1) / ms.chunk;
        }
        if (c.row_shard()) {  // rank r scans chunks [cb[r], cb[r + 1])
            const uint32_t W = (uint32_t)c.shard_world_;
            ms.n_blk = W;
            for (uint32_t r = 0; r <= W; r++) ms.cb[r] = (uint32_t)((uint64_t)ms.n_chunks * r / W);
        }
        return true;
    }

    // The hashed lookup's cuckoo table (ms.hmask, ms.hseed, htab) when the
    // signatures allow it: term-only, the same required fields, keyword ids
    // (32 bits), pairwise distinct values.  Seeds are tried in a fixed order
    // (deterministic tables), the capacity doubles if none places every key.
    std::vector<DMHashEntry> htab;
    bool plan_mscan_hash(DMScan& ms) {
        ms.hmask = 0;
        ms.dsize = 0;
        htab.clear();
        dgrid.clear();
        if (c.mhash_mode_ == 2 || ms.n_fields == 0) return false;
        const uint8_t all = (uint8_t)((1u << ms.n_fields) - 1);
        for (const DMSig& m : msig) {
            if (!m.term_only || m.req_mask != all) return false;
            for (uint32_t f = 0; f < ms.n_fields; f++)
                if (m.req[f] < 0 || m.req[f] > (int64_t)UINT32_MAX) return false;
        }
        auto hash = [&](uint32_t seed, const DMSig& m) {
            uint32_t h = seed;
            for (uint32_t f = 0; f < ms.n_fields; f++) h = msig_mix(h, (uint32_t)m.req[f]);
            return msig_fin(h);
        };
        for (uint32_t cap = 4; cap <= kMHashCap; cap <<= 1) {
            if (cap < 2 * ms.n_sigs) continue;
            for (uint32_t attempt = 0; attempt < 32; attempt++) {
                const uint32_t s0 = 0x2545F491u * (2 * attempt + 1), s1 = 0x9E3779B9u * (2 * attempt + 2);
                std::vector<uint32_t> slot(cap, kMHashEmpty);
                bool ok = true;
                for (uint32_t q = 0; q < ms.n_sigs && ok; q++) {
                    uint32_t cur = q, pos = hash(s0, msig[q]) & (cap - 1);
                    for (uint32_t kick = 0;; kick++) {
                        if (slot[pos] == kMHashEmpty) { slot[pos] = cur; break; }
                        if (kick == 4 * cap) { ok = false; break; }
                        std::swap(cur, slot[pos]);  // evict; the evicted key goes to its other position
                        const uint32_t p0 = hash(s0, msig[cur]) & (cap - 1), p1 = hash(s1, msig[cur]) & (cap - 1);
                        pos = pos == p0 ? p1 : p0;
                    }
                }
                if (!ok) continue;
                // distinct values: two signatures with equal keys would share both positions
                for (uint32_t q = 0; q < ms.n_sigs; q++)
                    for (uint32_t r = q + 1; r < ms.n_sigs; r++) {
                        bool eq = true;
                        for (uint32_t f = 0; f < ms.n_fields; f++) eq = eq && msig[q].req[f] == msig[r].req[f];
                        if (eq) return false;
                    }
                htab.assign(cap, DMHashEntry{});
                for (uint32_t p = 0; p < cap; p++) {
                    DMHashEntry& e = htab[p];
                    e.q = slot[p];
                    if (slot[p] == kMHashEmpty) continue;
                    const DMSig& m = msig[slot[p]];
                    for (uint32_t f = 0; f < ms.n_fields; f++) e.key[f] = (uint32_t)m.req[f];
                    e.tmin = m.tmin;
                    e.tmax = m.tmax;
                }
                ms.hmask = cap - 1;
                ms.hseed[0] = s0;
                ms.hseed[1] = s1;
                plan_key_grid(ms);
                return true;
            }
        }
        return false;
    }

    // The direct lookup (DMScan::dsize) beside the cuckoo table: when the
    // signatures' values span at most kMHashGrid cells over all fields (pool
    // values are dictionary ids, interned close together), a grid cell per
    // value combination holds its signature (u16, 0xFFFF none), followed by
    // the signatures' count ranges; the kernel reads one 2-B cell per
    // candidate instead of two 32-B cuckoo entries.
    std::vector<uint8_t> dgrid;
    void plan_key_grid(DMScan& ms) {
        ms.dsize = 0;
        dgrid.clear();
        if (!c.mhash_grid_mode_) return;
        uint64_t cells = 1;
        for (uint32_t f = 0; f < ms.n_fields; f++) {
            int64_t lo = INT64_MAX, hi = INT64_MIN;
            for (const DMSig& m : msig) {
                lo = std::min(lo, m.req[f]);
                hi = std::max(hi, m.req[f]);
            }
            ms.dlo[f] = (uint32_t)lo;
            ms.drng[f] = (uint32_t)(hi - lo + 1);
            cells *= (uint64_t)(hi - lo + 1);
            if (cells > kMHashGrid) return;
        }
        const size_t gbytes = ((size_t)cells * 2 + 15) & ~(size_t)15;
        dgrid.assign(gbytes + (((size_t)ms.n_sigs * 8 + 15) & ~(size_t)15), 0);
        uint16_t* g = reinterpret_cast<uint16_t*>(dgrid.data());
        for (uint64_t k = 0; k < cells; k++) g[k] = 0xFFFFu;
        int32_t* lim = reinterpret_cast<int32_t*>(dgrid.data() + gbytes);
        for (uint32_t q = 0; q < ms.n_sigs; q++) {
            uint64_t idx = 0;
            for (uint32_t f = 0; f < ms.n_fields; f++) idx = idx * ms.drng[f] + (uint64_t)(msig[q].req[f] - ms.dlo[f]);
            g[idx] = (uint16_t)q;
            lim[2 * q] = msig[q].tmin;
            lim[2 * q + 1] = msig[q].tmax;
        }
        ms.dsize = (uint32_t)cells;
    }

    // The hashed scan of a row-sharded batch: this rank's block of chunks,
    // the blocks' chunk outputs (scratch) and count columns all-gathered in
    // place — over RCCL between the devices, or through the host exchange —
    // then every rank places every list (mscan_base + mscan_place), so the
    // lists and result cells are identical on every rank.  Gathered: 4 B per
    // scanned candidate + 4 B per (signature + 1, chunk).
    void mscan_hash_sharded(const DMScan& ms, uint32_t* work, DGroupResult* cres) {
        const int W = c.shard_world_, r = c.shard_rank_;
        NKM_HIP(launch_mscan_hash(st, ms, c.d_msig_.p, work, cres, reinterpret_cast<uint32_t*>(c.d_out_.p), stream,
                                  c.ev_[4], c.ev_[5], kMHashEval, ms.cb[r], ms.cb[r + 1]));
        const uint64_t cw = mscan_hash_counts_word(ms), w1 = ms.n_sigs + 1;
        std::vector<int64_t> o_sc(W + 1), o_cn(W + 1);
        for (int q = 0; q <= W; q++) {
            o_sc[q] = (int64_t)((uint64_t)ms.cb[q] * ms.chunk * 4);
            o_cn[q] = (int64_t)((cw + w1 * ms.cb[q]) * 4);
        }
        if (c.nccl_comm_) {
            c.shard_gather_device(work, o_sc);
            c.shard_gather_device(work, o_cn);
        } else {
            const uint64_t words = cw + w1 * ms.n_chunks;
            c.h_mx_.reserve(words);
            char* h = reinterpret_cast<char*>(c.h_mx_.p);
            char* d = reinterpret_cast<char*>(work);
            for (const auto* o : {&o_sc, &o_cn})
                if ((*o)[r + 1] > (*o)[r])
                    NKM_HIP(hipMemcpyAsync(h + (*o)[r], d + (*o)[r], (size_t)((*o)[r + 1] - (*o)[r]),
                                           hipMemcpyDeviceToHost, stream));
            NKM_HIP(hipStreamSynchronize(stream));
            c.shard_gather_host(h, o_sc);
            c.shard_gather_host(h, o_cn);
            for (const auto* o : {&o_sc, &o_cn})
                for (int q = 0; q < W; q++)
                    if (q != r && (*o)[q + 1] > (*o)[q])
                        NKM_HIP(hipMemcpyAsync(d + (*o)[q], h + (*o)[q], (size_t)((*o)[q + 1] - (*o)[q]),
                                               hipMemcpyHostToDevice, stream));
        }
        NKM_HIP(launch_mscan_hash(st, ms, c.d_msig_.p, work, cres, reinterpret_cast<uint32_t*>(c.d_out_.p), stream,
                                  nullptr, nullptr, kMHashPlace));
    }

    // overlap: host work run while the batch's kernels and copies are in
    // flight (the pool bucketing of the rows, which needs no hit list).
    // rows_self: every batch row carries its own search's terms and is
    // indexed (assemble_parallel's fused plan) — a hashed-scan list may then
    // be proven equal to its search's rows (Core::list_proof_mode_).
    void run_batch(std::vector<BGroup>& bg, bool need_pm, const std::function<void()>& overlap = nullptr,
                   bool rows_self = false) {
        using rclk = std::chrono::steady_clock;
        auto rms = [](rclk::time_point a, rclk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        const auto r0 = rclk::now();
        c.flush_apply();  // the previous batch's selections, before this batch's searches
        const uint32_t kChunk = (uint32_t)scan_chunk_len();
        lg.clear();
        lg_group.clear();
        lmap.clear();
        cg_list.clear();
        cg_off.clear();
        cg_first.clear();
        cg_end.clear();
        DMScan ms{};
        const bool use_m = plan_mscan(bg, kChunk, ms);
        std::vector<uint8_t> on_m(bg.size(), 0);
        for (uint32_t i : m_list) {
            on_m[i] = 1;
            // an mscan list is never cut: its hit positions are scan-order
            // positions, which a cursor page over the search's own source
            // (fetch_more) could not continue from
            bg[i].d.k = std::max(bg[i].d.k, bg[i].d.src_len);
        }
        uint64_t off = 0;
        std::vector<uint32_t> chunked;
        std::vector<uint32_t> full_var;
        // output entries the batch reserves: full-list promotions (below) may
        // only use what batch assembly left of kOutCap
        uint64_t budget = 0;
        for (const BGroup& g : bg) budget += g.d.k;
        // A large RevPrecision batch (every search whole: no chunks, full
        // lists or promotions) builds its descriptors on the workers.
        const bool par_lg = rev && c.par_mode_ && m_list.empty() && bg.size() >= c.par_min(65536);
        // Top-tier lists (search_kernel path 2) for the variable-score
        // searches whose scores sum exactly: an exact list prefix of any
        // length, so the rows of a large batch reach their partners without
        // running off a 512-entry top-K list and restarting the batch (C2:
        // 11 batches).  The searches share what the batch budget leaves (half
        // of kOutCap), up to kTierMax entries each; the row a list stopped is
        // re-searched with every tier (retry).
        const auto tier_ok = [&](const BGroup& g) {
            return c.tier_mode_ && !rev && g.d.var_score && !g.d.has_cursor && !g.retry && g.d.ub_key != INT64_MAX &&
                   c.sigs_[g.sig].exact_scores && g.d.src_len > 0;
        };
        uint64_t tier_share = 0;
        if (!par_lg && c.tier_mode_ && !rev) {
            uint64_t n_tier = 0, other = 0;
            for (const BGroup& g : bg) {
                if (tier_ok(g)) n_tier++;
                else other += g.d.k;
            }
            if (n_tier && other < kOutCap / 2) tier_share = std::min<uint64_t>(kTierMax, (kOutCap * 7 / 8 - other) / n_tier);
        }
        if (par_lg) {
            WorkPool& wp = c.workers();
            const size_t nb = bg.size(), nch = (size_t)wp.size() * 4;
            grow_to(lg, nb);
            grow_to(lg_group, nb);
            std::vector<uint64_t> at(nch + 1, 0);
            const uint32_t small_max = (uint32_t)small_src_max();
            wp.run(nch, [&](size_t ch) {
                uint64_t k = 0;
                for (size_t i = nb * ch / nch; i < nb * (ch + 1) / nch; i++) {
                    const DGroup& d = bg[i].d;
                    DGroup& w = lg[i];
                    w = d;
                    w.path = 0;
                    if (d.rev_slot != kNoSlot && !d.has_cursor && d.src_len > 0 && d.src_len <= small_max) {
                        w.path = 1;
                        w.k = d.src_len;
                    }
                    k += w.k;
                    lg_group[i] = (uint32_t)i;
                }
                at[ch + 1] = k;
            });
            for (size_t ch = 0; ch < nch; ch++) at[ch + 1] += at[ch];
            wp.run(nch, [&](size_t ch) {
                uint64_t o = at[ch];
                for (size_t i = nb * ch / nch; i < nb * (ch + 1) / nch; i++) {
                    lg[i].out_off = o;
                    o += lg[i].k;
                }
            });
            off = at[nch];
        }
        for (uint32_t i = 0; i < bg.size() && !par_lg; i++) {
            if (on_m[i]) continue;
            const DGroup& d = bg[i].d;
            const bool big = d.src_len > kChunk && d.k > kChunk / 4;
            if (!d.var_score && !rev && !d.has_cursor && d.src_len > 0 && !c.row_shard() &&
                (c.kernel_mode_ == Core::KM_SCAN || (c.kernel_mode_ != Core::KM_SEARCH && big))) {
                chunked.push_back(i);
                continue;
            }
            DGroup w = d;
            w.path = 0;
            // a RevPrecision row over a short source: rsmall_kernel, whole list
            if (d.rev_slot != kNoSlot && rev && !d.has_cursor && d.src_len > 0 &&
                d.src_len <= (uint32_t)small_src_max()) {
                w.path = 1;
                w.k = d.src_len;
            }
            // A variable-score search whose rows need more than the LDS top-K
            // (k was capped at kVarK) over a small source runs as a full list:
            // the constant-score path emits every hit with its own score key
            // in source order, and the host sorts it stably by key (source
            // order breaks ties, as the top-K does), so the list is complete.
            if (w.path == 0 && d.var_score && !rev && !d.has_cursor && d.k >= (uint32_t)var_k_capacity() && d.src_len > d.k &&
                d.src_len <= kFullVarMax && c.full_var_mode_ && budget + (d.src_len - d.k) <= kOutCap) {
                budget += d.src_len - d.k;
                w.var_score = 0;
                w.k = d.src_len;
                full_var.push_back((uint32_t)lg.size());
                stats.full_lists++;
            }
            // A constant-score search over a source the batch can afford in
            // full (a quarter of kOutCap for all promotions) returns its whole
            // list: rows that walk far (a row that matches nothing walks all
            // of it) then never page it one synchronous launch at a time.
            if (w.path == 0 && !d.var_score && !rev && !d.has_cursor && d.k < d.src_len &&
                budget + (d.src_len - d.k) <= kOutCap / 4) {
                budget += d.src_len - d.k;
                w.k = d.src_len;
            }
            if (w.path == 0 && w.var_score && tier_share > d.k && tier_ok(bg[i])) {
                w.path = 2;  // var_score stays set: both search_kernel instantiations take part
                w.k = (uint32_t)std::min<uint64_t>(tier_share, d.src_len);
                budget += w.k - std::min<uint64_t>(w.k, d.k);
                stats.tier_lists++;
            }
            w.out_off = off;
            off += w.k;
            lg.push_back(w);
            lg_group.push_back(i);
        }
        const int nwhole = (int)lg.size();
        uint64_t scratch = 0;
        for (uint32_t i : chunked) {
            const DGroup& d = bg[i].d;
            cg_list.push_back(i);
            cg_first.push_back((uint32_t)(lg.size() - nwhole));
            cg_off.push_back(off);
            for (uint32_t s0 = 0; s0 < d.src_len; s0 += kChunk) {
                DGroup dc = d;
                dc.src_off = d.src_off + s0;
                dc.src_len = std::min(kChunk, d.src_len - s0);
                dc.k = dc.src_len;
                dc.out_off = scratch;
                scratch += dc.src_len;
                lmap.push_back(DChunkMap{cg_first.back(), s0, d.k, 0u, off, dc.out_off});
                lg.push_back(dc);
                lg_group.push_back(i);
            }
            cg_end.push_back((uint32_t)(lg.size() - nwhole));
            off += d.k;
        }
        const int nchunks = (int)lg.size() - nwhole;
        // The lists of whole and chunked searches come back to the host as
        // 4-B slot ids plus each list's last DHit (its cursor) — unless the
        // host needs every key (full-list searches are sorted by key here) or
        // the lists are exchanged between ranks as DHits (row-sharded).
        // NKM_SLOTLISTS=2 packs RevPrecision batches too (A/B).
        const uint64_t scan_end = off;
        const bool slots_only = c.slot_lists_mode_ && full_var.empty() && !c.row_shard() &&
                                (!rev || c.slot_lists_rev_) && scan_end > 0;
        // mscan: signatures (DMSig, clause_off indexing mcl), result cells
        // after the chunks — one per (signature, chunk) for stitch_kernel, or
        // one per signature from the hashed scan's own placement
        const uint32_t mchunk = ms.chunk;
        const uint64_t mscratch = scratch;
        const bool hashed = use_m && ms.hmask != 0;
        const size_t n_stitch = cg_list.size();  // searches stitch_kernel places
        // The mscan lists are 4-B slot ids packed back to back from slot word
        // 4 * off (cg_off holds each list's first slot word): one contiguous
        // region the first D2H round can copy whole (below).
        std::vector<uint64_t> mdst;
        const uint64_t mw0 = 4 * off;
        uint64_t mw = mw0;
        for (uint32_t q = 0; q < m_list.size(); q++) {
            const uint32_t i = m_list[q];
            const DGroup& d = bg[i].d;
            cg_list.push_back(i);
            cg_off.push_back(mw);
            if (hashed) {
                cg_first.push_back((uint32_t)nchunks + q);
                cg_end.push_back((uint32_t)nchunks + q + 1);
                mdst.push_back(mw);
                mw += d.k;
                continue;
            }
            const uint32_t first = (uint32_t)nchunks + q * ms.n_chunks;
            cg_first.push_back(first);
            cg_end.push_back(first + ms.n_chunks);
            // u32 cells and output: `so` and dst_off in slot words
            for (uint32_t ch = 0; ch < ms.n_chunks; ch++)
                lmap.push_back(DChunkMap{first, ch * mchunk, d.k, 1u, mw,
                                         4 * mscratch + ((uint64_t)q * ms.n_chunks + ch) * mchunk});
            mw += d.k;
        }
        off += (mw - mw0 + 3) / 4;
        // copied in the first round when the capacity is at most 2 slot ids
        // per scanned candidate (C3 / C4: every candidate in at most one list)
        // unless proven (Core::list_proof_mode_): a list whose count is its
        // search's batch rows is those rows, not downloaded (mode 2: it is,
        // and the claim checked against it)
        const bool proof = hashed && rows_self && c.list_proof_mode_ != 0 && c.monotone_ && !c.row_shard() && !rev;
        const bool skip_lists = proof && c.list_proof_mode_ == 1;
        // counts only (Core::mhash_count_mode_): every list is expected proven
        const bool count_only = skip_lists && ms.contig && c.mhash_count_mode_ && c.mhash_spec_pause_ == 0;
        if (c.mhash_spec_pause_) c.mhash_spec_pause_--;
        const int mh_phases = kMHashEval | kMHashPlace | (count_only ? kMHashCount : 0);
        const bool m_precopy = use_m && !c.row_shard() && mw - mw0 <= 2 * (uint64_t)ms.src_len && !skip_lists;
        const uint32_t ncells = !use_m ? 0 : hashed ? ms.n_sigs : ms.n_sigs * ms.n_chunks;
        if (hashed) scratch += (mscan_hash_work_words(ms) + 3) / 4;
        else if (use_m) scratch += ((uint64_t)ncells * mchunk + 3) / 4;  // 4-B slots in 16-B DHit units
        const int ng = (int)lg.size();
        const uint32_t nres = (uint32_t)(nwhole + nchunks) + ncells, nmap = (uint32_t)lmap.size();
        c.h_groups_.reserve(ng);
        if (ng >= 65536 && c.par_mode_) {  // 80 B per search: large batches copy on the workers
            const size_t nch = c.workers().size();
            c.workers().run(nch, [&](size_t ch) {
                const size_t lo = (size_t)ng * ch / nch, hi = (size_t)ng * (ch + 1) / nch;
                std::memcpy(c.h_groups_.p + lo, lg.data() + lo, (hi - lo) * sizeof(DGroup));
            });
        } else {
            std::memcpy(c.h_groups_.p, lg.data(), ng * sizeof(DGroup));
        }
        c.d_groups_.reserve(ng, false);
        c.d_res_.reserve(std::max<uint32_t>(nres, 1), false);
        c.d_out_.reserve(std::max<uint64_t>(off, 1), false);
        if (rev) c.d_rev_.reserve(std::max<uint64_t>(off, 1), false);
        if (nmap || hashed) c.d_scan_.reserve(std::max<uint64_t>(scratch, 1), false);
        if (nmap) {
            c.h_map_.reserve(nmap);
            std::memcpy(c.h_map_.p, lmap.data(), nmap * sizeof(DChunkMap));
            c.d_map_.reserve(nmap, false);
            NKM_HIP(hipMemcpyAsync(c.d_map_.p, c.h_map_.p, nmap * sizeof(DChunkMap), hipMemcpyHostToDevice, stream));
        }
        if (use_m) {
            // the signatures; hashed: then the output word offsets and the table
            const size_t blob = hashed ? mscan_hash_blob_bytes(ms.n_sigs, ms.hmask + 1, ms.dsize) : msig.size() * sizeof(DMSig);
            const size_t nblob = (blob + sizeof(DMSig) - 1) / sizeof(DMSig);
            c.h_msig_.reserve(nblob);
            char* hb = reinterpret_cast<char*>(c.h_msig_.p);
            std::memcpy(hb, msig.data(), msig.size() * sizeof(DMSig));
            if (hashed) {
                std::memcpy(hb + msig.size() * sizeof(DMSig), mdst.data(), mdst.size() * sizeof(uint64_t));
                std::memcpy(hb + mscan_hash_table_off(ms.n_sigs), htab.data(), htab.size() * sizeof(DMHashEntry));
                if (ms.dsize)
                    std::memcpy(hb + mscan_hash_table_off(ms.n_sigs) + htab.size() * sizeof(DMHashEntry), dgrid.data(),
                                dgrid.size());
            }
            c.d_msig_.reserve(nblob, false);
            NKM_HIP(hipMemcpyAsync(c.d_msig_.p, c.h_msig_.p, blob, hipMemcpyHostToDevice, stream));
            c.h_mcl_.reserve(std::max<size_t>(mcl.size(), 1));
            std::memcpy(c.h_mcl_.p, mcl.data(), mcl.size() * sizeof(DClause));
            c.d_mcl_.reserve(std::max<size_t>(mcl.size(), 1), false);
            NKM_HIP(hipMemcpyAsync(c.d_mcl_.p, c.h_mcl_.p, mcl.size() * sizeof(DClause), hipMemcpyHostToDevice, stream));
        }
        NKM_HIP(hipMemcpyAsync(c.d_groups_.p, c.h_groups_.p, ng * sizeof(DGroup), hipMemcpyHostToDevice, stream));
        // row-sharded: this rank evaluates the block [b0, b1) of the whole
        // searches, cut at the world's quantiles of their source lengths
        int b0 = 0, b1 = nwhole;
        std::vector<int> blk;
        if (c.row_shard()) {
            const int W = c.shard_world_;
            uint64_t tot = 0;
            for (int i = 0; i < nwhole; i++) tot += lg[i].src_len + 64;
            blk.assign(W + 1, nwhole);
            blk[0] = 0;
            uint64_t run = 0;
            int q = 1;
            for (int i = 0; i < nwhole && q < W; i++) {
                run += lg[i].src_len + 64;
                while (q < W && run * W >= tot * (uint64_t)q) blk[q++] = i + 1;
            }
            b0 = blk[c.shard_rank_];
            b1 = blk[c.shard_rank_ + 1];
        }
        // per eval kernel, the start/stop events of its dispatch (per-kernel roofline in bench.py)
        // (read from lg: the pinned copy may be write-combined)
        int kinds = 0;
        // rsmall_kernel's rows of this rank's block
        std::vector<uint32_t>& small = small_rows;
        small.clear();
        if (b1 - b0 >= 65536 && c.par_mode_) {
            WorkPool& wp = c.workers();
            const size_t nblk = (size_t)(b1 - b0), nch = (size_t)wp.size() * 4;
            std::vector<int> ck(nch, 0);
            std::vector<size_t> at(nch + 1, 0);
            wp.run(nch, [&](size_t ch) {
                int k = 0;
                size_t m = 0;
                for (size_t i = b0 + nblk * ch / nch; i < b0 + nblk * (ch + 1) / nch; i++) {
                    k |= lg[i].path == 2 ? 3 : lg[i].var_score ? 2 : 1;
                    m += lg[i].path == 1;
                }
                ck[ch] = k;
                at[ch + 1] = m;
            });
            for (size_t ch = 0; ch < nch; ch++) {
                kinds |= ck[ch];
                at[ch + 1] += at[ch];
            }
            small.resize(at[nch]);
            wp.run(nch, [&](size_t ch) {
                size_t o = at[ch];
                for (size_t i = b0 + nblk * ch / nch; i < b0 + nblk * (ch + 1) / nch; i++)
                    if (lg[i].path == 1) small[o++] = (uint32_t)i;
            });
        } else {
            for (int i = b0; i < b1; i++) kinds |= lg[i].path == 2 ? 3 : lg[i].var_score ? 2 : 1;
            for (int i = b0; i < b1; i++)
                if (lg[i].path == 1) small.push_back((uint32_t)i);
        }
        if (small.size() == (size_t)(b1 - b0)) kinds = 0;  // no search_kernel work
        NKM_HIP(launch_search(st, c.d_groups_.p + b0, b1 - b0, c.d_out_.p, rev ? c.d_rev_.p : nullptr, c.d_res_.p + b0,
                              stream, c.ev_[0], c.ev_[1], kinds));
        if (need_pm) c.d_pm_.reserve(std::max<uint64_t>(off, 1), false);  // one word per list entry
        if (!small.empty()) {
            c.h_small_.reserve(small.size());
            std::memcpy(c.h_small_.p, small.data(), small.size() * sizeof(uint32_t));
            c.d_small_.reserve(small.size(), false);
            NKM_HIP(hipMemcpyAsync(c.d_small_.p, c.h_small_.p, small.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                   stream));
            NKM_HIP(launch_rsmall(st, c.d_groups_.p, c.d_small_.p, (uint32_t)small.size(), c.d_out_.p,
                                  rev ? c.d_rev_.p : nullptr, need_pm ? c.d_pm_.p : nullptr, c.d_res_.p, stream,
                                  c.ev_[7], c.ev_[8]));
        }
        NKM_HIP(launch_scan(st, c.d_groups_.p + nwhole, nchunks, c.d_scan_.p, c.d_res_.p + nwhole, stream, c.ev_[2],
                            c.ev_[3]));
        stats.mhash |= hashed;
        if (hashed && c.row_shard())
            mscan_hash_sharded(ms, reinterpret_cast<uint32_t*>(c.d_scan_.p + mscratch), c.d_res_.p + nwhole + nchunks);
        else if (hashed)
            NKM_HIP(launch_mscan_hash(st, ms, c.d_msig_.p, reinterpret_cast<uint32_t*>(c.d_scan_.p + mscratch),
                                      c.d_res_.p + nwhole + nchunks, reinterpret_cast<uint32_t*>(c.d_out_.p), stream,
                                      c.ev_[4], c.ev_[5], mh_phases));
        else if (use_m)
            NKM_HIP(launch_mscan(st, ms, c.d_msig_.p, c.d_mcl_.p, reinterpret_cast<uint32_t*>(c.d_scan_.p + mscratch),
                                 c.d_res_.p + nwhole + nchunks,
                                 std::any_of(msig.begin(), msig.end(), [](const DMSig& m) { return !m.term_only; }),
                                 stream, c.ev_[4], c.ev_[5]));
        // a marker between the eval kernels and stitch_kernel: without it the
        // runtime may complete mscan_kernel's dispatch together with the next
        // one, and its stop event then reads the stitch's end
        NKM_HIP(hipEventRecord(c.ev_[6], stream));
        if (nmap) {
            const size_t ns = hashed ? n_stitch : cg_list.size();
            c.h_cranges_.reserve(2 * ns);
            for (size_t k = 0; k < ns; k++) {
                c.h_cranges_.p[2 * k] = cg_first[k];
                c.h_cranges_.p[2 * k + 1] = cg_end[k];
            }
            c.d_cranges_.reserve(2 * ns, false);
            c.d_coffs_.reserve(nmap, false);
            NKM_HIP(hipMemcpyAsync(c.d_cranges_.p, c.h_cranges_.p, 2 * ns * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
            NKM_HIP(launch_stitch(c.d_map_.p, (int)nmap, c.d_res_.p + nwhole, c.d_cranges_.p, (int)ns, c.d_coffs_.p,
                                  c.d_scan_.p, c.d_out_.p, stream));
        }
        if (need_pm && kinds)
            NKM_HIP(launch_pairmat(st, c.d_groups_.p + b0, c.d_res_.p + b0, b1 - b0, c.d_out_.p, c.d_pm_.p, stream));
        if (slots_only) {
            c.d_slots_.reserve(scan_end, false);
            c.h_slots_.reserve(scan_end);
            c.d_last_.reserve(std::max(nwhole, 1), false);
            c.h_last_.reserve((size_t)nwhole + cg_list.size() + 1);
            NKM_HIP(launch_pack_slots(c.d_out_.p, scan_end, c.d_slots_.p, c.d_groups_.p, c.d_res_.p, nwhole, c.d_last_.p,
                                      stream));
        }
        c.h_res_.reserve(std::max<uint32_t>(nres, 1));
        c.h_out_.reserve(std::max<uint64_t>(off, 1));
        if (rev) c.h_rev_.reserve(std::max<uint64_t>(off, 1));
        if (need_pm) c.h_pm_.reserve(std::max<uint64_t>(off, 1));
        const uint64_t whole_off = nwhole ? lg[nwhole - 1].out_off + lg[nwhole - 1].k : 0;
        // the blocks' byte ranges in each exchanged buffer: result records,
        // hit lists, RevPrecision flags, pair matrices
        std::vector<int64_t> o_res, o_out, o_rev, o_pm;
        if (c.row_shard()) {
            for (int q = 0; q <= c.shard_world_; q++) {
                const int b = blk[q];
                const uint64_t oo = b < nwhole ? lg[b].out_off : whole_off;
                o_res.push_back((int64_t)b * (int64_t)sizeof(DGroupResult));
                o_out.push_back((int64_t)(oo * sizeof(DHit)));
                o_rev.push_back((int64_t)oo);
                o_pm.push_back((int64_t)(oo * sizeof(uint32_t)));
            }
        }
        const bool host_x = c.row_shard() && !c.nccl_comm_;
        if (c.row_shard() && c.nccl_comm_) {  // every block to every rank, in place, over xGMI
            c.shard_gather_device(c.d_res_.p, o_res);
            c.shard_gather_device(c.d_out_.p, o_out);
            if (rev) c.shard_gather_device(c.d_rev_.p, o_rev);
            if (need_pm) c.shard_gather_device(c.d_pm_.p, o_pm);
        }
        if (host_x) {  // this rank's block to the host; the others' arrive through the host all-gather
            auto d2h = [&](void* h, const void* d, const std::vector<int64_t>& o) {
                const int64_t n = o[c.shard_rank_ + 1] - o[c.shard_rank_];
                if (n > 0)
                    NKM_HIP(hipMemcpyAsync((char*)h + o[c.shard_rank_], (const char*)d + o[c.shard_rank_], (size_t)n,
                                           hipMemcpyDeviceToHost, stream));
            };
            d2h(c.h_res_.p, c.d_res_.p, o_res);
            d2h(c.h_out_.p, c.d_out_.p, o_out);
            if (use_m)  // the hashed scan's result cells: every rank placed every list
                NKM_HIP(hipMemcpyAsync(c.h_res_.p + nwhole + nchunks, c.d_res_.p + nwhole + nchunks,
                                       (size_t)ncells * sizeof(DGroupResult), hipMemcpyDeviceToHost, stream));
            if (rev) d2h(c.h_rev_.p, c.d_rev_.p, o_rev);
            if (need_pm) d2h(c.h_pm_.p, c.d_pm_.p, o_pm);
        } else {
            NKM_HIP(hipMemcpyAsync(c.h_res_.p, c.d_res_.p, nres * sizeof(DGroupResult), hipMemcpyDeviceToHost, stream));
            if (whole_off && slots_only) {
                NKM_HIP(hipMemcpyAsync(c.h_slots_.p, c.d_slots_.p, whole_off * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                       stream));
                NKM_HIP(hipMemcpyAsync(c.h_last_.p, c.d_last_.p, (size_t)nwhole * sizeof(DHit), hipMemcpyDeviceToHost,
                                       stream));
            } else if (whole_off) {
                NKM_HIP(hipMemcpyAsync(c.h_out_.p, c.d_out_.p, whole_off * sizeof(DHit), hipMemcpyDeviceToHost, stream));
            }
            if (m_precopy && mw > mw0)
                NKM_HIP(hipMemcpyAsync(reinterpret_cast<uint32_t*>(c.h_out_.p) + mw0,
                                       reinterpret_cast<const uint32_t*>(c.d_out_.p) + mw0, (mw - mw0) * sizeof(uint32_t),
                                       hipMemcpyDeviceToHost, stream));
            if (rev) NKM_HIP(hipMemcpyAsync(c.h_rev_.p, c.d_rev_.p, off, hipMemcpyDeviceToHost, stream));
            if (need_pm && whole_off)
                NKM_HIP(hipMemcpyAsync(c.h_pm_.p, c.d_pm_.p, whole_off * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        }
        const auto r1 = rclk::now();
        if (overlap) overlap();
        const auto r2 = rclk::now();
        NKM_HIP(hipStreamSynchronize(stream));
        const auto r3 = rclk::now();
        stats.rb_prep_ms += rms(r0, r1);
        stats.rb_overlap_ms += rms(r1, r2);
        stats.rb_wait_ms += rms(r2, r3);
        if (host_x) {
            c.shard_gather_host(c.h_res_.p, o_res);
            c.shard_gather_host(c.h_out_.p, o_out);
            if (rev) c.shard_gather_host(c.h_rev_.p, o_rev);
            if (need_pm) c.shard_gather_host(c.h_pm_.p, o_pm);
        }
        const bool ran[4] = {kinds != 0, nchunks > 0, use_m, !small.empty()};
        static const int ev0[4] = {0, 2, 4, 7};
        for (int kk = 0; kk < 4; kk++) {
            if (!ran[kk]) continue;
            float ms_k = 0.f;
            NKM_HIP(hipEventElapsedTime(&ms_k, c.ev_[ev0[kk]], c.ev_[ev0[kk] + 1]));
            stats.k_ms[kk] += ms_k;
            stats.k_launches[kk]++;
        }
        stats.batches++;
        if (all_rows_search && (!c.row_shard() || c.shard_rank_ == 0))  // processCustom: every row searches
            for (const BGroup& g : bg) stats.pairs_decided += (int64_t)g.nrows * (int64_t)g.d.src_len;
        {
            // per-search accounting (on the workers for large batches)
            const size_t ns = (size_t)(nwhole + nchunks);
            const size_t nch = ns >= 65536 && c.par_mode_ ? c.workers().size() : 1;
            std::vector<std::array<int64_t, 5>> acc(nch, std::array<int64_t, 5>{0, 0, 0, 0, 0});
            auto count = [&](size_t ch) {
                std::array<int64_t, 5> a{0, 0, 0, 0, 0};  // thread-private: the chunks' sums share cache lines
                for (size_t t = ns * ch / nch; t < ns * (ch + 1) / nch; t++) {
                    if ((int)t < b0 || ((int)t >= b1 && (int)t < nwhole)) continue;  // another rank's block
                    a[4] += c.h_res_.p[t].scanned;
                    const int kk = (int)t >= nwhole ? 1 : lg[t].path == 1 ? 3 : 0;
                    a[kk] += search_bytes(bg[lg_group[t]].n_fields, lg[t], c.h_res_.p[t]);
                }
                acc[ch] = a;
            };
            if (nch > 1) c.workers().run(nch, count);
            else count(0);
            for (auto& a : acc) {
                for (int kk = 0; kk < 4; kk++) stats.k_bytes[kk] += a[kk];
                stats.pair_evals += a[4];
            }
        }
        if (use_m) {
            // columns read once per candidate for all signatures; hits written per signature
            // bytes each candidate's signature lookup loads: the alive flag,
            // Min/MaxCount and per field a kind and a value (the contiguous
            // hashed scan reads no slot id: 1 + 8 + 9 NF B; otherwise + 4);
            // then 4 B per hit.  pair_evals: (row, candidate) decisions — one
            // per scanned candidate and signature for mscan_kernel, one per
            // scanned candidate for the hashed lookup (a candidate is tested
            // against the one signature its values select).
            const int64_t per_scan = ms.contig ? 1 : 5;
            const int64_t per_live = 8 + 9 * (int64_t)ms.n_fields;
            const DGroupResult* mr = c.h_res_.p + nwhole + nchunks;
            // row-sharded: this rank scanned its block of the chunks
            const double share = hashed && ms.n_blk > 1
                                     ? (double)(ms.cb[c.shard_rank_ + 1] - ms.cb[c.shard_rank_]) / (double)ms.n_chunks
                                     : 1.0;
            int64_t kb = 0, pe = 0;
            const int64_t per_hit = count_only ? 0 : 4;  // counts only: no list written
            for (uint32_t t = 0; t < ncells; t++) {
                kb += (int64_t)mr[t].scanned * per_scan + (int64_t)mr[t].live * per_live + (int64_t)mr[t].count * per_hit;
                pe += (int64_t)mr[t].scanned * (hashed ? 1 : ms.n_sigs);
            }
            stats.k_bytes[2] += (int64_t)((double)kb * share) +
                                (int64_t)(ms.n_sigs * sizeof(DMSig) + mcl.size() * sizeof(DClause));
            stats.pair_evals += (int64_t)((double)pe * share);
        }
        for (uint32_t i : full_var) {
            DHit* h = c.h_out_.p + lg[i].out_off;
            std::stable_sort(h, h + c.h_res_.p[i].count, [](const DHit& a, const DHit& b) { return a.key > b.key; });
        }
        auto wire = [&](size_t lo, size_t hi) {
            for (size_t i = lo; i < hi; i++) {
                BGroup& g = bg[lg_group[i]];
                const DGroupResult& r = c.h_res_.p[i];
                g.head = 0;
                g.rows_list = false;
                if (slots_only) {
                    g.set_slots(c.h_slots_.p + lg[i].out_off);
                    g.last_i = (uint32_t)i;
                } else {
                    g.set_hits(c.h_out_.p + lg[i].out_off);
                }
                g.rev = rev ? c.h_rev_.p + lg[i].out_off : nullptr;
                g.pm = need_pm ? c.h_pm_.p + lg[i].out_off : nullptr;
                g.pm_n = need_pm ? std::min<uint32_t>(r.count, kPairP) : 0;
                g.n = r.count;
                g.complete = r.complete != 0;
            }
        };
        if (nwhole >= 65536 && c.par_mode_) {
            const size_t nch = c.workers().size();
            c.workers().run(nch, [&](size_t ch) { wire((size_t)nwhole * ch / nch, (size_t)nwhole * (ch + 1) / nch); });
        } else {
            wire(0, (size_t)nwhole);
        }
        const auto r4 = rclk::now();
        stats.rb_post_ms += rms(r3, r4);
        // chunked / mscan searches: exact hit counts are known now; copy just
        // those (an mscan list: 4-B slot ids, copied in the first round when
        // m_precopy)
        const size_t n_scan_cg = cg_list.size() - (use_m ? m_list.size() : 0);
        bool m_copied = false;
        c.row_lists_pending_ = false;
        if (count_only) {
            // a list the counts do not prove was never written: the full scan
            // for this batch, and the speculation pauses
            bool all_proven = true;
            for (size_t k = n_scan_cg; k < cg_list.size() && all_proven; k++) {
                uint64_t n = 0;
                for (uint32_t t = cg_first[k]; t < cg_end[k]; t++) n += c.h_res_.p[nwhole + t].count;
                all_proven = n == bg[cg_list[k]].nrows;
            }
            if (!all_proven) {
                NKM_HIP(launch_mscan_hash(st, ms, c.d_msig_.p, reinterpret_cast<uint32_t*>(c.d_scan_.p + mscratch),
                                          c.d_res_.p + nwhole + nchunks, reinterpret_cast<uint32_t*>(c.d_out_.p), stream,
                                          nullptr, nullptr, mh_phases & ~kMHashCount));
                stats.mhash_respec++;
                c.mhash_spec_pause_ = Core::kSpecPause;
            }
        }
        for (size_t k = 0; k < cg_list.size(); k++) {
            BGroup& g = bg[cg_list[k]];
            const bool slots = k >= n_scan_cg;
            uint64_t n = 0;
            for (uint32_t t = cg_first[k]; t < cg_end[k]; t++) n += c.h_res_.p[nwhole + t].count;
            bool complete = true;
            if (n > g.d.k) { n = g.d.k; complete = false; }
            if (slots && !complete)  // mscan lists are sized to their whole source (plan above)
                throw DeviceError{hipErrorUnknown, "mscan list cut", __LINE__};
            const bool packed = !slots && slots_only;  // a chunked list: slot ids + its last DHit
            uint32_t* const h32 = reinterpret_cast<uint32_t*>(c.h_out_.p);
            g.rows_list = false;
            if (slots) {  // an mscan list: cg_off is its first slot word
                const bool proven = proof && n == g.nrows;
                if (n && !m_precopy && !(proven && skip_lists)) {
                    NKM_HIP(hipMemcpyAsync(h32 + cg_off[k], reinterpret_cast<const uint32_t*>(c.d_out_.p) + cg_off[k],
                                           n * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
                    m_copied = true;
                }
                g.rows_list = proven;
                c.row_lists_pending_ = c.row_lists_pending_ || proven;
                stats.mscan_lists++;
                stats.lists_proven += proven;
            } else if (n && packed) {
                NKM_HIP(hipMemcpyAsync(c.h_slots_.p + cg_off[k], c.d_slots_.p + cg_off[k], n * sizeof(uint32_t),
                                       hipMemcpyDeviceToHost, stream));
                NKM_HIP(hipMemcpyAsync(c.h_last_.p + nwhole + k, c.d_out_.p + cg_off[k] + n - 1, sizeof(DHit),
                                       hipMemcpyDeviceToHost, stream));
            } else if (n) {
                NKM_HIP(hipMemcpyAsync(c.h_out_.p + cg_off[k], c.d_out_.p + cg_off[k], n * sizeof(DHit),
                                       hipMemcpyDeviceToHost, stream));
            }
            g.head = 0;
            g.last_i = packed ? (uint32_t)(nwhole + k) : UINT32_MAX;
            if (slots) g.set_slots(h32 + cg_off[k]);
            else if (packed) g.set_slots(c.h_slots_.p + cg_off[k]);
            else g.set_hits(c.h_out_.p + cg_off[k]);
            g.rev = nullptr;
            g.pm = nullptr;
            g.pm_n = 0;
            g.n = (uint32_t)n;
            g.complete = complete;
        }
        if (n_scan_cg || m_copied) NKM_HIP(hipStreamSynchronize(stream));
        stats.rb_lists_ms += rms(r4, rclk::now());
    }

    bool pair_slow(const BGroup& g, uint32_t from_pos, uint32_t to_pos) override {
        // slow path: evaluate the single pair on the device (pool workers of a
        // RevPrecision parallel replay share the stream and the buffers)
        std::lock_guard<std::mutex> lk(c.pair_mu_);
        uint32_t pr[2] = {g.slot(from_pos), g.slot(to_pos)};
        c.d_slots_tmp_.reserve(2, false);
        c.d_pair_out_.reserve(1, false);
        NKM_HIP(hipMemcpyAsync(c.d_slots_tmp_.p, pr, sizeof pr, hipMemcpyHostToDevice, stream));
        NKM_HIP(launch_pairs(st, c.d_slots_tmp_.p, 1, c.d_pair_out_.p, stream));
        uint8_t ok = 0;
        NKM_HIP(hipMemcpyAsync(&ok, c.d_pair_out_.p, 1, hipMemcpyDeviceToHost, stream));
        NKM_HIP(hipStreamSynchronize(stream));
        return ok != 0;
    }
};

ReplayView Core::replay_view() const { return Replay::view(*this); }

std::unique_ptr<ReplayCore> Core::make_replay(std::vector<uint8_t>& sel, bool rev, int max_intervals, PassStats& stats) {
    return std::unique_ptr<ReplayCore>(new Replay(*this, sel, rev, max_intervals, stats, dstore(), stream_));
}

// choose_source without advancing the posting lists' dead-prefix heads (safe
// on the host workers): the same list, possibly starting at dead entries.
// source_of for a signature with one MUST term (its posting key: field << 32
// | term): that term's posting list (C5's bucket)
void Core::source_of_key1(uint64_t key1, DGroup& g) const {
    const PostingRange* it = postings_map_.find(key1);
    g.src_kind = 1;
    g.src_off = it ? it->off + it->head : 0;
    g.src_len = it ? it->len - it->head : 0;
}

void Core::source_of(const Sig& s, DGroup& g, SrcChoice* ch) const {
    if (s.must_key1 != UINT64_MAX) {  // one MUST term: its posting list
        source_of_key1(s.must_key1, g);
        if (ch) {
            ch->has_term = true;
            ch->field = (uint16_t)(s.must_key1 >> 32);
            ch->term = (uint32_t)s.must_key1;
        }
        return;
    }
    g.src_kind = 0;
    g.src_off = order_head_;
    g.src_len = (uint32_t)order_.size() - order_head_;
    bool have = false;
    if (ch) ch->has_term = false;
    for (auto& mt : s.must_terms) {
        const PostingRange* it = postings_map_.find(((uint64_t)mt.first << 32) | mt.second);
        uint32_t off = 0, len = 0;
        if (it) {
            off = it->off + it->head;
            len = it->len - it->head;
        }
        if (!have || len < g.src_len) {
            if (ch) { ch->has_term = true; ch->field = mt.first; ch->term = mt.second; }
            g.src_kind = 1;
            g.src_off = off;
            g.src_len = len;
            have = true;
        }
    }
}

void Core::choose_source(const Sig& s, DGroup& g, SrcChoice* ch) {
    g.src_kind = 0;
    g.src_off = order_head_;
    g.src_len = (uint32_t)order_.size() - order_head_;
    bool have = false;
    if (ch) ch->has_term = false;
    for (auto& mt : s.must_terms) {
        PostingRange* it = postings_map_.find(((uint64_t)mt.first << 32) | mt.second);
        uint32_t off = 0, len = 0;
        if (it) {
            PostingRange& r = *it;
            while (r.head < r.len && !live_[postings_[r.off + r.head]]) r.head++;  // skip the dead prefix
            off = r.off + r.head;
            len = r.len - r.head;
        }
        if (!have || len < g.src_len) {
            if (ch) { ch->has_term = true; ch->field = mt.first; ch->term = mt.second; }
            g.src_kind = 1;
            g.src_off = off;
            g.src_len = len;
            have = true;
        }
    }
}

int Core::process_default(GroupList& out_groups,
                          UVec<uint32_t>& expired, PassStats& stats) {
    const auto tp0 = std::chrono::steady_clock::now();
    const uint32_t N = (uint32_t)nslots();
    filled_groups_ = 0;
    std::vector<uint8_t>& sel = sel_;
    std::vector<uint8_t>& dec = dec_;  // rows decided ahead of `pos` by a partial parallel replay
    if (par_mode_ && N >= par_min(1u << 20) && sel.size() == N && dec.size() == N) {
        WorkPool& wp = workers();  // 2 x 1 MB at C3: cleared on the workers
        const size_t nch = wp.size();
        wp.run(nch, [&](size_t c) {
            const size_t lo = (size_t)N * c / nch, hi = (size_t)N * (c + 1) / nch;
            std::memset(sel.data() + lo, 0, hi - lo);
            std::memset(dec.data() + lo, 0, hi - lo);
        });
    } else {
        sel.assign(N, 0);
        dec.assign(N, 0);
    }
    bool out_of_order = false;         // groups appended out of row order (sorted at the end)
    std::vector<uint32_t>& rowpos = list_tmp_;  // slot -> pinned position (set when out_of_order)
    bool rev = cfg_.rev_precision != 0;
    RevTimer timer(rev && active_flag_ && cfg_.rev_threshold > 0,
                   (double)cfg_.interval_sec * (double)cfg_.rev_threshold);
    const int maxI = cfg_.max_intervals;
    std::vector<uint32_t>& rows = rows_;
    precount_.valid = false;
    if (active_exact_ && big_list(active_list_)) {  // every entry is a row: one parallel copy
        rows.resize(active_list_.size());
        WorkPool& wp = workers();
        const size_t n = active_list_.size(), nch = wp.size(), nsig = sigs_.size();
        // with few signatures (assemble_parallel's own limit), the copy also
        // counts them per chunk: the first batch's count sweep (C3: 1M rows)
        const bool pre = par_mode_ && !cfg_.rev_precision && nsig <= 65536;
        PreCount& pc = precount_;
        if (pre) {
            pc.first.resize(nch);
            pc.cnt.resize(nch);
            pc.n.assign(nch, 0);
            pc.self.assign(nch, 1);
        }
        wp.run(nch, [&](size_t c) {
            const size_t lo = n * c / nch, hi = n * (c + 1) / nch;
            if (!pre) {
                std::memcpy(rows.data() + lo, active_list_.data() + lo, (hi - lo) * sizeof(uint32_t));
                return;
            }
            std::vector<uint32_t> first, cnt(nsig, 0);  // thread-private until the end (shared lines)
            const uint32_t* const A = active_list_.data();
            uint32_t* const W = rows.data();
            const uint32_t* const SG = sig_.data();
            const uint8_t* const SM = self_match_.data();
            const uint8_t* const IX = indexed_.data();
            uint8_t self = 1;
            for (size_t i = lo; i < hi; i++) {
                const uint32_t r = A[i];
                W[i] = r;
                const uint32_t sg = SG[r];
                if (!cnt[sg]++) first.push_back(sg);
                self &= (uint8_t)(SM[r] & IX[r]);
            }
            pc.first[c] = std::move(first);
            pc.cnt[c] = std::move(cnt);
            pc.n[c] = hi - lo;
            pc.self[c] = self;
        });
        if (pre) {
            pc.valid = true;
            pc.n_rows = n;
        }
    } else {
        filter_slots(big_list(active_list_) ? &workers() : nullptr, active_list_, rows,
                     [&](uint32_t s) { return live_[s] && is_active_[s]; });
    }
    stats.prologue_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0).count();

    if (!active_flag_) {  // paused: intervals still advance (matchmaker_process.go:53-63)
        for (uint32_t r : rows) {
            intervals_[r]++;
            if (intervals_[r] >= maxI || minc_[r] == maxc_[r]) expired.push_back(r);
        }
        return MM_OK;
    }

    const DStore st = dstore();
    Replay rp(*this, sel, rev, maxI, stats, st, stream_);
    std::vector<int32_t> sig_group(sigs_.size(), -1);
    std::vector<BGroup>& bg = bg_;  // kept across passes: no page faults on the hot path
    bg.clear();
    UVec<uint32_t>& brow = brow_;
    UVec<uint32_t>& brow_group = brow_group_;
    UVec<uint32_t>& newly = newly_;
    std::vector<std::pair<uint32_t, int>> grp;
    const uint32_t kvar = (uint32_t)var_k_capacity();
    size_t pos = 0;
    uint32_t retry_slot = kNoSlot;
    size_t win = SIZE_MAX;  // rows per batch (kWinMin)
    // floor of a variable-score search's capacity: doubles (up to the top-K
    // capacity) each time a batch ends on a list that ran out
    uint32_t vfloor = kVarKMin;
    while (order_head_ < order_.size() && !live_[order_[order_head_]]) order_head_++;

    while (true) {
        while (pos < rows.size() && (sel[rows[pos]] | dec[rows[pos]])) pos++;
        if (pos >= rows.size()) break;
        // the RevThreshold timer fired: the remaining rows search as without
        // RevPrecision (row-sharded: decided at batch starts, OR-ed over the ranks)
        if (rev && (row_shard() ? shard_any(timer.check()) : timer.check())) rev = rp.rev = false;
        // ---- range batch (mm_range.cpp): every remaining row decided at once ----
        if (!rev && range_mode_ && kernel_mode_ == KM_AUTO && retry_slot == kNoSlot && !row_shard() && par_mode_) {
            newly.clear();
            if (range_batch(rows, pos, out_groups, expired, newly, stats)) {
                defer_apply(newly);
                continue;
            }
        }
        // ---- packed RevPrecision batch (rpack_kernel) ----
        if (rev && pack_mode_ && kernel_mode_ == KM_AUTO && retry_slot == kNoSlot && !row_shard()) {
            using pclk = std::chrono::steady_clock;
            auto pms = [](pclk::time_point a, pclk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            const auto ta0 = pclk::now();
            PackBatch pb;
            if (assemble_packed(rows, pos, win, brow, pb)) {
                const auto tb0 = pclk::now();
                stats.assemble_ms += pms(ta0, tb0);
                ParPlan& plan = par_plan_;
                plan.ok = false;
                const bool timer_live = timer.armed && !timer.fired;
                const PackLayout L = run_packed(pb, stats, [&] {  // pools bucketed while the rows search
                    if (par_mode_ && !timer_live) plan_packed(pb.n, brow, plan, stats);
                });
                const auto tb1 = pclk::now();
                stats.search_ms += pms(tb0, tb1);
                const std::function<BGroup&(uint32_t)> view = packed_view(L, brow);
                newly.clear();
                uint32_t stop_bi = UINT32_MAX;
                if (par_mode_ && replay_parallel(plan, bg, brow, brow_group, sel, out_groups, expired, newly, stats, rev,
                                                 &stop_bi, &view)) {
                    stats.parallel_batches++;
                    if (stop_bi != UINT32_MAX) throw std::runtime_error("packed batch: a complete list ran out");
                } else {
                    for (size_t bi = 0; bi < pb.n; bi++) {
                        const uint32_t T = brow[bi];
                        if (sel[T]) continue;
                        BGroup& g = view((uint32_t)bi);
                        if (rp.rev && timer.check()) rp.rev = false;  // later rows skip the reverse checks
                        const auto status = rp.decide(T, g, false, grp);
                        if (status == Replay::EXHAUSTED) throw std::runtime_error("packed batch: a complete list ran out");
                        intervals_[T]++;
                        if (intervals_[T] >= maxI || minc_[T] == maxc_[T]) expired.push_back(T);
                        if (status == Replay::MATCHED) {
                            for (auto& e : grp) {
                                if (!sel[e.first]) {
                                    sel[e.first] = 1;
                                    newly.push_back(e.first);
                                }
                            }
                            out_groups.push(grp);
                        }
                    }
                }
                const auto tb2 = pclk::now();
                stats.replay_ms += pms(tb1, tb2);
                defer_apply(newly);
                if (batch_profile_)
                    std::fprintf(stderr, "[nkm]   batch %d (packed, S %d%s): rows %zu | assemble %.2f search %.2f replay %.2f ms\n",
                                 stats.batches, pb.S, plan.ok ? ", parallel" : "", pb.n, pms(ta0, tb0), pms(tb0, tb1),
                                 pms(tb1, tb2));
                pos = pb.end;
                if (win != SIZE_MAX) win = win > SIZE_MAX / 2 ? SIZE_MAX : 2 * win;
                continue;
            }
        }
        // ---- assemble the batch ----
        const auto ta0 = std::chrono::steady_clock::now();
        for (auto& g : bg)
            if (!rev) sig_group[g.sig] = -1;
        // RevPrecision batches refill the array in place on the workers
        // (assemble_parallel_rev clears it whenever it declines)
        if (!(rev && par_mode_)) bg.clear();
        brow.clear();
        brow_group.clear();
        size_t q = pos;
        auto new_group = [&](uint32_t sig, uint32_t r) {
            BGroup g;
            g.sig = sig;
            const Sig& s = sigs_[g.sig];
            g.n_fields = s.n_fields;
            g.d.clause_off = s.clause_off;
            g.d.n_clauses = s.n_clauses;
            g.d.qkind = s.qkind;
            g.d.var_score = s.var_score ? 1 : 0;
            g.d.tmin = s.tmin;
            g.d.tmax = s.tmax;
            g.d.tparty = s.tparty;
            g.d.rev_slot = rev ? r : kNoSlot;
            g.d.ub_key = s.ub_key;
            g.d.has_cursor = 0;
            SrcChoice ch;
            choose_source(s, g.d, &ch);
            g.has_src_term = ch.has_term;
            g.src_field = ch.field;
            g.src_term = ch.term;
            g.d.k = 0;
            g.row_slot = rev ? r : kNoSlot;
            return g;
        };
        // a search's hit capacity after `nrows` rows, the last with MaxCount m
        auto cap_k = [&](const BGroup& g, uint64_t nrows, int m) {
            const uint64_t want = nrows * (uint64_t)std::max(2, m) * 2 + 32;
            const uint32_t k = g.d.var_score ? (uint32_t)std::min<uint64_t>(std::min<uint32_t>(kvar, std::max<uint32_t>(g.d.src_len, 1)),
                                                                         std::max<uint64_t>(want, vfloor))
                                             : (uint32_t)std::min<uint64_t>(std::max<uint32_t>(g.d.src_len, 1), want + 224);
            return std::max<uint32_t>(k, 1);
        };
        // Parallel assembly (same batch as the serial loop below): chunks of
        // the rows count their signatures, groups are numbered in first-
        // appearance order, and each search's capacity is the serial loop's
        // final value.  The batch is the remaining rows up to the window
        // (the first `win` undecided rows: a per-chunk count finds the cut);
        // taken only when even an upper bound of the serial loop's running
        // capacity total stays within kOutCap (so it would not have cut the
        // batch earlier).
        size_t q_par = rows.size();  // the batch's end in rows (the serial loop's q)
        bool fused_plan = false;     // assemble_parallel bucketed the rows per search (plan_fused)
        auto assemble_parallel = [&]() -> bool {
            size_t nr = rows.size() - pos;
            const size_t nsig = sigs_.size();
            if (rev || !par_mode_ || nr < par_min(65536) || nsig > 65536) return false;
            // the row a list stopped is the batch's first undecided row (the
            // rows before it were decided): its search returns every tier
            if (retry_slot != kNoSlot && (sel[rows[pos]] | dec[rows[pos]] || rows[pos] != retry_slot)) return false;
            WorkPool& wp = workers();
            const unsigned nch = wp.size();
            q_par = rows.size();
            if (nr > win || nr > kMaxBatchRows) {  // the window's cut: the row after its win-th undecided row
                const size_t cap = std::min<size_t>(win, kMaxBatchRows);
                std::vector<size_t> und(nch, 0);
                wp.run(nch, [&](size_t c) {
                    size_t k = 0;
                    for (size_t i = pos + nr * c / nch; i < pos + nr * (c + 1) / nch; i++) k += !(sel[rows[i]] | dec[rows[i]]);
                    und[c] = k;
                });
                size_t seen = 0;
                for (unsigned c = 0; c < nch && q_par == rows.size(); c++) {
                    if (seen + und[c] < cap) { seen += und[c]; continue; }
                    for (size_t i = pos + nr * c / nch; i < pos + nr * (c + 1) / nch; i++)
                        if (!(sel[rows[i]] | dec[rows[i]]) && ++seen == cap) { q_par = i + 1; break; }
                }
                nr = q_par - pos;
                if (nr < par_min(65536)) return false;
            }
            struct Chunk {
                std::vector<uint32_t> first, cnt;
                size_t n = 0;
                bool self = true;  // every row carries its own search's terms (self_match_) and is indexed
            };
            std::vector<Chunk> ch(nch);
            const auto ts0 = std::chrono::steady_clock::now();
            std::vector<double> cnt_task_us(nch, 0.0), cnt_start_us(nch, 0.0);  // NKM_PROFILE=2
            // the prologue counted these rows in this split already (the
            // pass's first batch, nothing selected or decided: every row counts)
            PreCount& pc = precount_;
            const bool pre = pc.valid && pos == 0 && nr == rows.size() && pc.n_rows == nr && pc.n.size() == nch &&
                             retry_slot == kNoSlot;
            pc.valid = false;
            if (pre) {
                for (unsigned c = 0; c < nch; c++) {
                    ch[c].first = std::move(pc.first[c]);
                    ch[c].cnt = std::move(pc.cnt[c]);
                    ch[c].n = pc.n[c];
                    ch[c].self = pc.self[c] != 0;
                }
            } else
            wp.run(nch, [&](size_t c) {
                const auto tc0 = std::chrono::steady_clock::now();
                // thread-private until the end (adjacent Chunks share cache
                // lines: a per-row k.n++ made this sweep 3-4x slower)
                // (a row's MaxCount is its signature's: signatures key on the
                // searching ticket's Min / MaxCount, Core::sig_eq — so it is
                // read per search below, not per row)
                std::vector<uint32_t> first, cnt(nsig, 0);
                size_t n = 0;
                bool self = true;
                for (size_t i = pos + nr * c / nch; i < pos + nr * (c + 1) / nch; i++) {
                    const uint32_t r = rows[i];
                    if (sel[r] | dec[r]) continue;
                    const uint32_t sg = sig_[r];
                    if (!cnt[sg]++) first.push_back(sg);
                    self = self && self_match_[r] && indexed_[r];
                    n++;
                }
                Chunk& k = ch[c];
                k.first = std::move(first);
                k.cnt = std::move(cnt);
                k.n = n;
                k.self = self;
                const auto tc1 = std::chrono::steady_clock::now();
                cnt_start_us[c] = std::chrono::duration<double, std::micro>(tc0 - ts0).count();
                cnt_task_us[c] = std::chrono::duration<double, std::micro>(tc1 - tc0).count();
            });
            const auto tce = std::chrono::steady_clock::now();
            stats.asm_count_ms += std::chrono::duration<double, std::milli>(tce - ts0).count();
            if (batch_profile_)
                std::fprintf(stderr, "[nkm]   assemble count sweep: tasks max %.0f us, last start %.0f us\n",
                             *std::max_element(cnt_task_us.begin(), cnt_task_us.end()),
                             *std::max_element(cnt_start_us.begin(), cnt_start_us.end()));
            uint64_t bound = 0;
            for (unsigned c = 0; c < nch; c++)
                for (uint32_t sg : ch[c].first)
                    if (sig_group[sg] < 0) {
                        sig_group[sg] = (int32_t)bg.size();
                        bg.push_back(new_group(sg, kNoSlot));
                    }
            for (BGroup& g : bg) {
                uint64_t nrows = 0;
                for (unsigned c = 0; c < nch; c++) nrows += ch[c].cnt[g.sig];
                const int32_t lastm = std::max(2, sigs_[g.sig].tmax), maxm = lastm;
                g.nrows = (uint32_t)nrows;
                g.d.k = cap_k(g, nrows, lastm);
                if (retry_slot != kNoSlot && g.sig == sig_[retry_slot]) {  // the serial loop's retry capacity
                    g.retry = true;
                    if (nrows == 1) g.d.k = g.d.var_score ? kvar : std::max<uint32_t>(g.d.src_len, 1);
                }
                bound += std::max<uint64_t>(cap_k(g, nrows, maxm), g.d.k);
            }
            if (bound > kOutCap) {  // the serial loop may cut this batch: let it
                for (auto& g : bg) sig_group[g.sig] = -1;
                bg.clear();
                return false;
            }
            std::vector<size_t> at(nch + 1, 0);
            for (unsigned c = 0; c < nch; c++) at[c + 1] = at[c] + ch[c].n;
            grow_to(brow, at[nch]);
            grow_to(brow_group, at[nch]);
            // The rows bucketed per search in the same sweep (plan_fused: the
            // pool-parallel replay's plan when every search is its own pool):
            // pool_rows holds each search's batch rows, ascending.
            const size_t G = bg.size();
            fused_plan = G >= 2 && G <= 4096 && par_mode_ &&
                         std::all_of(ch.begin(), ch.end(), [](const Chunk& k) { return k.self; });
            std::vector<uint32_t> gat;  // [chunk][search]: the chunk's next position in pool_rows
            if (fused_plan) {
                ParPlan& P = par_plan_;
                grow_to(P.pool_off, G + 1);
                P.pool_off[0] = 0;
                for (size_t g = 0; g < G; g++) P.pool_off[g + 1] = P.pool_off[g] + bg[g].nrows;
                gat.resize(nch * G);
                for (size_t g = 0; g < G; g++) {
                    uint32_t run = P.pool_off[g];
                    for (unsigned c = 0; c < nch; c++) {
                        gat[c * G + g] = run;
                        run += ch[c].cnt[bg[g].sig];
                    }
                }
                grow_to(P.pool_rows, at[nch]);
            }
            const auto ts1 = std::chrono::steady_clock::now();
            std::vector<double> sc_task_us(nch, 0.0), sc_start_us(nch, 0.0);  // NKM_PROFILE=2
            wp.run(nch, [&](size_t c) {
                const auto tc0 = std::chrono::steady_clock::now();
                size_t o = at[c];
                // the chunk's positions, thread-private (the chunks' rows of gat share cache lines)
                static thread_local std::vector<uint32_t> gl;
                uint32_t* ga = nullptr;
                if (fused_plan) {
                    gl.assign(gat.begin() + c * G, gat.begin() + (c + 1) * G);
                    ga = gl.data();
                }
                uint32_t* prow = par_plan_.pool_rows.data();
                for (size_t i = pos + nr * c / nch; i < pos + nr * (c + 1) / nch; i++) {
                    const uint32_t r = rows[i];
                    if (sel[r] | dec[r]) continue;
                    const uint32_t gi = (uint32_t)sig_group[sig_[r]];
                    brow[o] = r;
                    brow_group[o] = gi;
                    if (ga) prow[ga[gi]++] = (uint32_t)o;
                    o++;
                }
                sc_start_us[c] = std::chrono::duration<double, std::micro>(tc0 - ts1).count();
                sc_task_us[c] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - tc0).count();
            });
            stats.asm_scatter_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts1).count();
            if (batch_profile_)
                std::fprintf(stderr, "[nkm]   assemble scatter: tasks max %.0f us, last start %.0f us; serial between sweeps %.0f us\n",
                             *std::max_element(sc_task_us.begin(), sc_task_us.end()),
                             *std::max_element(sc_start_us.begin(), sc_start_us.end()),
                             std::chrono::duration<double, std::micro>(ts1 - tce).count());
            return true;
        };
        // RevPrecision: one search per row; large batches build them on the
        // workers (sources from a non-mutating lookup of the posting ranges)
        auto assemble_parallel_rev = [&]() -> bool {
            const size_t nr = rows.size() - pos;
            if (!rev || retry_slot != kNoSlot || !par_mode_ || nr < par_min(65536) || nr > kMaxBatchRows || nr > win) {
                bg.clear();
                return false;
            }
            WorkPool& wp = workers();
            const unsigned nch = wp.size() * 4;
            // count, then every chunk builds its rows' searches in place
            std::vector<size_t> at(nch + 1, 0);
            wp.run(nch, [&](size_t c) {
                size_t k = 0;
                for (size_t i = pos + nr * c / nch; i < pos + nr * (c + 1) / nch; i++) k += !(sel[rows[i]] | dec[rows[i]]);
                at[c + 1] = k;
            });
            for (unsigned c = 0; c < nch; c++) at[c + 1] += at[c];
            const size_t n = at[nch];
            std::vector<uint64_t> ck(nch, 0);
            bg.resize(n);  // constructs only past the array's previous size
            grow_to(brow, n);
            grow_to(brow_group, n);
            wp.run(nch, [&](size_t c) {
                size_t o = at[c];
                uint64_t kc = 0;  // thread-private (ck's words share cache lines)
                for (size_t i = pos + nr * c / nch; i < pos + nr * (c + 1) / nch; i++) {
                    const uint32_t r = rows[i];
                    if (sel[r] | dec[r]) continue;
                    BGroup& g = bg[o];
                    g.reset();
                    g.sig = sig_[r];
                    const Sig& sg = sigs_[g.sig];
                    g.n_fields = sg.n_fields;
                    g.d.clause_off = sg.clause_off;
                    g.d.n_clauses = sg.n_clauses;
                    g.d.qkind = sg.qkind;
                    g.d.var_score = sg.var_score ? 1 : 0;
                    g.d.tmin = sg.tmin;
                    g.d.tmax = sg.tmax;
                    g.d.tparty = sg.tparty;
                    g.d.rev_slot = r;
                    g.d.ub_key = sg.ub_key;
                    SrcChoice ch;
                    source_of(sg, g.d, &ch);
                    g.has_src_term = ch.has_term;
                    g.src_field = ch.field;
                    g.src_term = ch.term;
                    g.row_slot = r;
                    g.nrows = 1;
                    g.d.k = cap_k(g, 1, maxc_[r]);
                    kc += g.d.k;
                    brow[o] = r;
                    brow_group[o] = (uint32_t)o;
                    o++;
                }
                ck[c] = kc;
            });
            uint64_t tot = 0;
            for (unsigned c = 0; c < nch; c++) tot += ck[c];
            if (tot > kOutCap) {  // the serial loop cuts the batch
                bg.clear();
                brow.clear();
                brow_group.clear();
                return false;
            }
            return true;
        };
        bool par_asm = false;
        if (assemble_parallel_rev()) {
            q = rows.size();
        } else if (!(par_asm = assemble_parallel())) {
            q_par = rows.size();
            uint64_t total_k = 0;
            for (; q < rows.size() && brow.size() < kMaxBatchRows && brow.size() < win; q++) {
                const uint32_t r = rows[q];
                if (sel[r] | dec[r]) continue;
                int32_t gi = rev ? -1 : sig_group[sig_[r]];
                if (gi < 0) {
                    gi = (int32_t)bg.size();
                    bg.push_back(new_group(sig_[r], r));
                    if (!rev) sig_group[sig_[r]] = gi;
                }
                BGroup& g = bg[gi];
                g.nrows++;
                uint32_t k = cap_k(g, g.nrows, maxc_[r]);
                if (r == retry_slot) {
                    k = g.d.var_score ? kvar : std::max<uint32_t>(g.d.src_len, 1);
                    g.retry = true;
                }
                total_k += (uint64_t)k - g.d.k;
                g.d.k = k;
                brow.push_back(r);
                brow_group.push_back((uint32_t)gi);
                if (total_k > kOutCap && brow.size() > 1) { q++; break; }
            }
        } else {
            q = q_par;
        }
        // ---- device search ----
        bool need_pm = false;
        if (rev) {
            for (size_t i = 0; i < bg.size() && !need_pm; i++) {
                const uint32_t r = bg[i].row_slot;
                need_pm = maxc_[r] - count_[r] >= 2;
            }
        }
        auto tb0 = std::chrono::steady_clock::now();
        stats.assemble_ms += std::chrono::duration<double, std::milli>(tb0 - ta0).count();
        ParPlan& plan = par_plan_;
        plan.ok = false;
        // a RevThreshold timer that may still fire is read per row: serial replay
        const bool timer_live = rev && timer.armed && !timer.fired;
        rp.run_batch(
            bg, need_pm,
            [&] {  // pools bucketed while the searches run
                if (par_mode_ && !timer_live)
                    (par_asm && fused_plan) ? plan_fused(bg, brow, brow_group, plan, stats)
                                            : plan_parallel(bg, brow, brow_group, plan, stats);
            },
            par_asm && fused_plan);
        if (list_proof_mode_ == 2) check_row_lists(bg, brow, brow_group);
        auto tb1 = std::chrono::steady_clock::now();
        stats.search_ms += std::chrono::duration<double, std::milli>(tb1 - tb0).count();
        // ---- replay ----
        newly.clear();
        size_t done = 0;
        bool exhausted = false;
        uint32_t stop_bi = UINT32_MAX;
        if (par_mode_ && replay_parallel(plan, bg, brow, brow_group, sel, out_groups, expired, newly, stats, rev,
                                         &stop_bi)) {
            row_lists_pending_ = false;  // consumed by the walk (or filled by replay_parallel)
            stats.parallel_batches++;
            const auto tr = std::chrono::steady_clock::now();
            stats.replay_ms += std::chrono::duration<double, std::milli>(tr - tb1).count();
            defer_apply(newly);
            stats.apply_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr).count();
            if (batch_profile_)
                std::fprintf(stderr,
                             "[nkm]   batch %d (parallel%s): rows %zu searches %zu%s | assemble %.2f search %.2f replay %.2f ms\n",
                             stats.batches, par_asm ? ", parallel assembly" : "", brow.size(), bg.size(),
                             stop_bi != UINT32_MAX ? " (a list ran out)" : "",
                             std::chrono::duration<double, std::milli>(tb0 - ta0).count(),
                             std::chrono::duration<double, std::milli>(tb1 - tb0).count(),
                             std::chrono::duration<double, std::milli>(tr - tb1).count());
            if (stop_bi == UINT32_MAX) {
                pos = q;
                retry_slot = kNoSlot;
                if (win != SIZE_MAX) win = win > SIZE_MAX / 2 ? SIZE_MAX : 2 * win;
            } else {
                // pools past their stop are decided (dec); the row whose list ran
                // out re-searches first, the window sized like the serial path's
                if (!out_of_order) {  // the pinned positions, for the final reorder
                    grow_to(rowpos, N);
                    for (uint32_t k = 0; k < rows.size(); k++) rowpos[rows[k]] = k;
                }
                out_of_order = true;
                retry_slot = brow[stop_bi];
                // the rest of the pass skips decided and selected rows for good
                size_t w = pos;
                for (size_t k = pos; k < rows.size(); k++)
                    if (!(sel[rows[k]] | dec[rows[k]])) rows[w++] = rows[k];
                rows.resize(w);
                win = std::max(kWinMin, 2 * (size_t)stop_bi);
                vfloor = std::min<uint32_t>(kvar, 2 * vfloor);
            }
            continue;
        }
        fill_row_lists(bg, brow, brow_group);  // the serial replay reads every list
        for (size_t bi = 0; bi < brow.size(); bi++) {
            const uint32_t T = brow[bi];
            if (sel[T]) { done = bi + 1; continue; }
            // a row past the end of its truncated list pages it with a cursor (the
            // batch's first row, and with page_mode_ any row of a constant-score
            // search, whose page holds >= 4096 hits; variable-score rows instead
            // end the batch and the searches re-run, since their 512-entry pages
            // would be fetched one synchronous launch at a time).  A page may
            // hold tickets selected earlier in this batch, which the walk skips,
            // so the list stays exact.
            BGroup& bgr = bg[brow_group[bi]];
            if (rp.rev && !row_shard() && timer.check()) rp.rev = false;  // later rows skip the reverse checks
            auto status = rp.decide(T, bgr, bi == 0 || (page_mode_ && !bgr.d.var_score), grp);
            if (status == Replay::EXHAUSTED) {
                exhausted = true;
                retry_slot = T;
                break;
            }
            intervals_[T]++;
            if (intervals_[T] >= maxI || minc_[T] == maxc_[T]) expired.push_back(T);
            if (status == Replay::MATCHED) {
                for (auto& e : grp) {
                    if (!sel[e.first]) {
                        sel[e.first] = 1;
                        newly.push_back(e.first);
                    }
                }
                out_groups.push(grp);
            }
            done = bi + 1;
        }
        const auto tb2 = std::chrono::steady_clock::now();
        stats.replay_ms += std::chrono::duration<double, std::milli>(tb2 - tb1).count();
        defer_apply(newly);
        if (batch_profile_)
            std::fprintf(stderr, "[nkm]   batch %d: rows %zu searches %zu decided %zu%s | assemble %.2f search %.2f replay %.2f ms\n",
                         stats.batches, brow.size(), bg.size(), done, exhausted ? " (list ran out)" : "",
                         std::chrono::duration<double, std::milli>(tb0 - ta0).count(),
                         std::chrono::duration<double, std::milli>(tb1 - tb0).count(),
                         std::chrono::duration<double, std::milli>(tb2 - tb1).count());
        // advance past the rows this batch decided
        if (exhausted) {
            while (pos < rows.size() && rows[pos] != retry_slot) pos++;
            win = std::max(kWinMin, 2 * done);
            vfloor = std::min<uint32_t>(kvar, 2 * vfloor);
        } else {
            pos = q;
            retry_slot = kNoSlot;
            if (win != SIZE_MAX) win = win > SIZE_MAX / 2 ? SIZE_MAX : 2 * win;
        }
    }
    // rows that searched x their sources (the parallel replays add theirs);
    // row-sharded: the replicated replay decides every row on every rank
    if (!row_shard() || shard_rank_ == 0) stats.pairs_decided += (int64_t)rp.pairs;
    if (out_of_order) {
        filled_groups_ = 0;  // the early-filled result entries are in the old order
        // back into the pinned row order: a group's searching ticket (its last
        // entry) is the row that formed it
        const size_t ng = out_groups.size();
        std::vector<uint32_t> ord(ng);
        for (uint32_t g = 0; g < ng; g++) ord[g] = g;
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
            return rowpos[out_groups.end(a)[-1].first] < rowpos[out_groups.end(b)[-1].first];
        });
        GroupList sorted;
        sorted.reserve_more(ng, out_groups.ents.size());
        for (uint32_t g : ord) sorted.push(out_groups.begin(g), out_groups.end(g));
        std::swap(out_groups.off, sorted.off);
        std::swap(out_groups.ents, sorted.ents);
    }
    return MM_OK;
}

// processCustom (matchmaker_process.go:336-612), up to the override call.
int Core::process_custom(GroupList& cands, UVec<uint32_t>& expired,
                         PassStats& stats) {
    const bool rev_cfg = cfg_.rev_precision != 0;
    const int maxI = cfg_.max_intervals;
    RevTimer timer(rev_cfg && active_flag_ && cfg_.rev_threshold > 0,
                   (double)cfg_.interval_sec * (double)cfg_.rev_threshold);  // :340-346
    std::vector<uint32_t> rows;
    for (uint32_t s : active_list_)
        if (live_[s] && is_active_[s]) rows.push_back(s);
    for (uint32_t r : rows) intervals_[r]++;  // :347-350
    for (uint32_t r : rows)
        if (intervals_[r] >= maxI || minc_[r] == maxc_[r]) expired.push_back(r);
    if (!active_flag_) return MM_OK;
    bool rev = rev_cfg;
    const DStore st = dstore();
    std::vector<uint8_t> sel(nslots(), 0);  // processCustom never selects
    Replay rp(*this, sel, rev, maxI, stats, st, stream_);
    rp.all_rows_search = true;
    // packed batches (assemble_packed) skip selected / decided rows: none here
    sel_.assign(nslots(), 0);
    dec_.assign(nslots(), 0);
    while (order_head_ < order_.size() && !live_[order_[order_head_]]) order_head_++;
    const uint32_t kvar = (uint32_t)var_k_capacity();
    // every row is independent: one search per row, in chunks
    for (size_t base = 0; base < rows.size(); base += kMaxBatchRows / 4) {
        const size_t end = std::min(rows.size(), base + kMaxBatchRows / 4);
        if (rev && (row_shard() ? shard_any(timer.check()) : timer.check())) rev = rp.rev = false;
        std::vector<BGroup>& bg = bg_;  // kept across passes (refilled in place: no allocation per row)
        const size_t nchunk = end - base;
        // RevPrecision rows whose sources hold <= 64 entries (C5's buckets)
        // search as one packed batch (rpack_kernel, as processDefault's
        // packed batches): a row's hits, reverse bits and pair words come
        // back in its fixed-stride section, read through packed_view.
        bool packed = false;
        std::function<BGroup&(uint32_t)> view;
        const auto tc0 = std::chrono::steady_clock::now();
        if (rev && pack_mode_ && kernel_mode_ == KM_AUTO && !row_shard()) {
            PackBatch pb;
            if (assemble_packed(rows, base, nchunk, brow_, pb) && pb.n == nchunk) {
                const auto tp1 = std::chrono::steady_clock::now();
                stats.assemble_ms += std::chrono::duration<double, std::milli>(tp1 - tc0).count();
                const PackLayout L = run_packed(pb, stats, nullptr);
                view = packed_view(L, brow_);
                stats.pairs_decided += (int64_t)pb.scanned;  // every row one search over its own source
                stats.search_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp1).count();
                packed = true;
            }
        }
        // row i's search: its packed section, or the per-row search below
        auto G = [&](size_t i) -> BGroup& { return packed ? view((uint32_t)i) : bg[i]; };
        if (!packed) bg.resize(nchunk);
        // the rows' searches (built on the workers for large chunks: the
        // sources from the non-mutating posting lookup)
        auto build = [&](size_t lo, size_t hi) {
            for (size_t i = lo; i < hi; i++) {
                const uint32_t r = rows[base + i];
                BGroup& g = bg[i];
                g.reset();
                g.sig = sig_[r];
                const Sig& s = sigs_[g.sig];
                g.n_fields = s.n_fields;
                g.d.clause_off = s.clause_off;
                g.d.n_clauses = s.n_clauses;
                g.d.qkind = s.qkind;
                g.d.var_score = s.var_score ? 1 : 0;
                g.d.tmin = s.tmin;
                g.d.tmax = s.tmax;
                g.d.tparty = s.tparty;
                g.d.rev_slot = rev ? r : kNoSlot;
                g.d.ub_key = s.ub_key;
                source_of(s, g.d);
                g.d.k = g.d.var_score ? std::min<uint32_t>(kvar, std::max<uint32_t>(g.d.src_len, 1))
                                       : std::min<uint32_t>(std::max<uint32_t>(g.d.src_len, 1), 128);
                g.row_slot = r;
                g.nrows = 1;  // one row per search (processCustom)
            }
        };
        const bool par = par_mode_ && nchunk >= par_min(4096);
        if (!packed) {
            if (par) {
                WorkPool& wp = workers();
                const size_t nch = (size_t)wp.size() * 4;
                wp.run(nch, [&](size_t c) { build(bg.size() * c / nch, bg.size() * (c + 1) / nch); });
            } else {
                build(0, bg.size());
            }
            const auto tc1 = std::chrono::steady_clock::now();
            rp.run_batch(bg, rev);
            stats.assemble_ms += std::chrono::duration<double, std::milli>(tc1 - tc0).count();
            stats.search_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc1).count();
        }
        const auto tc2 = std::chrono::steady_clock::now();
        // Every row is independent (processCustom selects nothing): chunks of
        // rows run on the workers into their own candidate lists, appended in
        // row order — unless a RevThreshold timer that may still fire is read
        // per row.  Device round trips (pages past a truncated list, pair
        // checks past the pair matrix) take turns on the stream.
        std::mutex dev_mu;
        struct Scratch {
            std::vector<uint32_t> hits, hpos, combo, sess_seen, pq, pr;
            std::vector<uint64_t> pm;
            std::vector<uint8_t> po;
            std::vector<std::pair<uint32_t, int>> me;
        };
        // The row's filtered hits (:425-468) and, with RevPrecision, their
        // pairwise validateMatch masks; false: the row yields no candidates.
        auto filter_row = [&](size_t i, Scratch& sc, bool row_rev, int& cmin, int& cmax) -> bool {
            BGroup& g = G(i);
            const uint32_t T = g.row_slot;
            // all hits (paging through the list), filtered as :425-468
            std::vector<uint32_t>& hits = sc.hits;
            std::vector<uint32_t>& hpos = sc.hpos;
            hits.clear();
            hpos.clear();
            uint32_t j = 0;
            bool too_many = false;
            for (;; j++) {
                if (j >= g.n) {
                    if (g.complete) break;
                    {
                        std::lock_guard<std::mutex> lk(dev_mu);
                        rp.fetch_more(g);
                    }
                    if (j >= g.n) break;
                }
                const uint32_t H = g.slot(j);
                if (H == T || rp.same_party(T, H)) continue;
                // a ticket an earlier processCustom pass retired is still in
                // the search index, but not in indexesCopy: "missing index" (:432-437)
                if (!live_[H]) continue;
                if (row_rev && !g.rev_at(j)) continue;
                if (maxc_[T] < maxc_[H] && intervals_[H] <= maxI) continue;
                if (rp.share_session(T, H)) continue;
                hits.push_back(H);
                hpos.push_back(j);
                if (hits.size() >= 63) { too_many = true; break; }
            }
            // combineIndexes: Go's `1 << length` is 0 / negative for length >= 63 -> no subsets
            if (too_many) return false;
            const size_t L = hits.size();
            cmin = minc_[T] - count_[T];
            cmax = maxc_[T] - count_[T];
            if (L == 0 || cmax <= 0) return false;  // every subset holds >= 1 ticket > max: none emitted
            // pairwise reverse checks among the hits (validateMatch both ways, incl. self)
            std::vector<uint64_t>& pm = sc.pm;
            pm.clear();
            bool covered = g.pm != nullptr;
            for (size_t a = 0; a < L && covered; a++) covered = hpos[a] < g.pm_n;
            if (row_rev && covered) {  // from the batch's pair matrices
                pm.assign(L, 0);
                for (size_t a = 0; a < L; a++)
                    for (size_t b = 0; b < L; b++)
                        if ((g.pm_at(hpos[a]) >> hpos[b]) & 1u) pm[a] |= 1ull << b;
            } else if (row_rev) {
                std::vector<uint32_t>& pr = sc.pr;
                pr.clear();
                for (size_t a = 0; a < L; a++)
                    for (size_t b = 0; b < L; b++) { pr.push_back(hits[a]); pr.push_back(hits[b]); }
                sc.po.assign(L * L, 0);
                {
                    std::lock_guard<std::mutex> lk(dev_mu);
                    d_slots_tmp_.reserve(pr.size(), false);
                    d_pair_out_.reserve(L * L, false);
                    NKM_HIP(hipMemcpyAsync(d_slots_tmp_.p, pr.data(), pr.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                           stream_));
                    NKM_HIP(launch_pairs(st, d_slots_tmp_.p, (uint32_t)(L * L), d_pair_out_.p, stream_));
                    NKM_HIP(hipMemcpyAsync(sc.po.data(), d_pair_out_.p, L * L, hipMemcpyDeviceToHost, stream_));
                    NKM_HIP(hipStreamSynchronize(stream_));
                }
                pm.assign(L, 0);
                for (size_t a = 0; a < L; a++)
                    for (size_t b = 0; b < L; b++)
                        if (sc.po[a * L + b]) pm[a] |= 1ull << b;
            }
            return true;
        };
        auto do_row = [&](size_t i, GroupList& out, Scratch& sc, bool row_rev) {
            int cmin, cmax;
            if (!filter_row(i, sc, row_rev, cmin, cmax)) return;
            const uint32_t T = G(i).row_slot;
            const std::vector<uint32_t>& hits = sc.hits;
            const std::vector<uint64_t>& pm = sc.pm;
            const size_t L = hits.size();
            const uint64_t limit = 1ull << L;
            std::vector<uint32_t>& combo = sc.combo;
            // combineIndexes' ascending bitmask loop (:586-610), visiting only
            // the masks its `count > max` test lets through (next_mask_le)
            for (uint64_t bits = next_mask_le(1, cmax); bits < limit; bits = next_mask_le(bits + 1, cmax)) {
                combo.clear();
                int entry_count = 0;
                bool over = false;
                for (size_t el = 0; el < L; el++) {
                    if ((bits >> el) & 1) {
                        entry_count += count_[hits[el]];
                        if (entry_count > cmax) { over = true; break; }
                        combo.push_back((uint32_t)el);
                    }
                }
                if (over || entry_count < cmin) continue;
                const int hit_count = entry_count + count_[T];
                if (hit_count > maxc_[T] || hit_count < minc_[T]) continue;
                if (hit_count % cm_[T] != 0) continue;
                bool reject = false;
                for (uint32_t el : combo) {
                    const uint32_t h = hits[el];
                    if (hit_count > maxc_[h] || hit_count < minc_[h] || hit_count % cm_[h] != 0 ||
                        (hit_count < maxc_[h] && intervals_[h] <= maxI)) { reject = true; break; }
                }
                if (reject) continue;
                // session conflicts across the combo; mutual checks between its hits
                bool conflict = false;
                std::vector<uint32_t>& sess_seen = sc.sess_seen;
                std::vector<uint32_t>& pq = sc.pq;  // hits whose query is already in parsedQueries
                sess_seen.clear();
                pq.clear();
                for (uint32_t el : combo) {
                    const uint32_t h = hits[el];
                    for (uint32_t p = pres_off_[h]; p < pres_off_[h + 1] && !conflict; p++) {
                        bool dup_in_ticket = false;
                        for (uint32_t p2 = pres_off_[h]; p2 < p; p2++) dup_in_ticket |= pres_sess_[p2] == pres_sess_[p];
                        if (dup_in_ticket) continue;  // SessionIDs is a set
                        const uint32_t sid = pres_sess_[p];
                        if (std::find(sess_seen.begin(), sess_seen.end(), sid) != sess_seen.end()) { conflict = true; break; }
                        sess_seen.push_back(sid);
                        if (row_rev) {
                            for (uint32_t o : pq) {
                                if (!((pm[el] >> o) & 1ull) || !((pm[o] >> el) & 1ull)) { conflict = true; break; }
                            }
                            if (conflict) break;
                            if (std::find(pq.begin(), pq.end(), el) == pq.end()) pq.push_back(el);
                        }
                    }
                    if (conflict) break;
                }
                if (conflict) continue;
                std::vector<std::pair<uint32_t, int>>& me = sc.me;
                me.clear();
                for (uint32_t el : combo)
                    for (int k = 0; k < count_[hits[el]]; k++) me.push_back({hits[el], k});
                for (int k = 0; k < count_[T]; k++) me.push_back({T, k});
                out.push(me);
            }
        };
        const bool timer_live = rev && !row_shard() && timer.armed && !timer.fired;
        if (dev_enum_mode_ && !timer_live && Replay::view(*this).sessions_exclusive) {
            // Device enumeration (enum_kernel): the rows' filtered hits are
            // gathered on the workers and every row's masks are cut into work
            // items; a count pass, the host's scan of the counts, and a write
            // pass straight into the candidate list (row order, masks
            // ascending, as the host loop below appends them).
            struct EnumChunk {
                std::vector<DEnumRow> rows;
                std::vector<DEnumHit> hits;
                std::vector<DEnumItem> items;
            };
            WorkPool& wp = workers();
            const size_t nch = par ? (size_t)wp.size() * 4 : 1;
            std::vector<EnumChunk> ec(nch);
            std::vector<uint8_t> huge(nch, 0);
            auto gather = [&](size_t c) {
                Scratch sc;
                EnumChunk& E = ec[c];
                for (size_t i = nchunk * c / nch; i < nchunk * (c + 1) / nch; i++) {
                    int cmin, cmax;
                    if (!filter_row(i, sc, rev, cmin, cmax)) continue;
                    const uint32_t T = G(i).row_slot;
                    const int L = (int)sc.hits.size();
                    const uint64_t V = masks_le(L, std::min(cmax, L));  // ranks 1 .. V-1 (rank 0: the empty mask)
                    if ((V - 1) / kEnumSpan >= (1ull << 26)) {
                        huge[c] = 1;
                        return;
                    }
                    const uint32_t r = (uint32_t)E.rows.size();
                    E.rows.push_back(DEnumRow{(uint32_t)E.hits.size(), T, L, (int32_t)count_[T], cmin, cmax,
                                              (int32_t)minc_[T], (int32_t)maxc_[T], (int32_t)cm_[T], 0});
                    for (int el = 0; el < L; el++) {
                        const uint32_t h = sc.hits[el];
                        DEnumHit d{};
                        d.pm = rev ? sc.pm[el] : ~0ull;
                        d.slot = h;
                        d.count = (int32_t)count_[h];
                        d.minc = (int32_t)minc_[h];
                        d.maxc = (int32_t)maxc_[h];
                        d.cm = (int32_t)cm_[h];
                        d.wait = intervals_[h] <= maxI;
                        bool multi = false;  // two distinct sessions (SessionIDs is a set)
                        for (uint32_t p = pres_off_[h] + 1; p < pres_off_[h + 1] && !multi; p++)
                            multi = pres_sess_[p] != pres_sess_[pres_off_[h]];
                        d.self_ok = !rev || !multi || ((sc.pm[el] >> el) & 1ull);
                        E.hits.push_back(d);
                    }
                    for (uint64_t r0 = 1; r0 < V; r0 += kEnumSpan)
                        E.items.push_back(DEnumItem{r0, r, (uint32_t)std::min<uint64_t>(kEnumSpan, V - r0)});
                }
            };
            using eclk = std::chrono::steady_clock;
            auto ems = [](eclk::time_point a, eclk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            const auto te0 = eclk::now();
            if (nch > 1) wp.run(nch, gather);
            else gather(0);
            const auto te1 = eclk::now();
            for (uint8_t x : huge)
                if (x) throw std::length_error("processCustom: a row's subsets exceed the enumeration limit");
            std::vector<size_t> rb(nch + 1, 0), hb(nch + 1, 0), ib(nch + 1, 0);
            for (size_t c = 0; c < nch; c++) {
                rb[c + 1] = rb[c] + ec[c].rows.size();
                hb[c + 1] = hb[c] + ec[c].hits.size();
                ib[c + 1] = ib[c] + ec[c].items.size();
            }
            const size_t nrow = rb[nch], nhit = hb[nch], nitem = ib[nch];
            if (nhit >= UINT32_MAX || nitem >= UINT32_MAX)
                throw std::length_error("processCustom: too many enumeration items");
            if (nitem) {
                h_erows_.reserve(nrow);
                h_ehits_.reserve(nhit);
                h_eitems_.reserve(nitem);
                auto pack = [&](size_t c) {
                    const EnumChunk& E = ec[c];
                    for (size_t k = 0; k < E.rows.size(); k++) {
                        DEnumRow r = E.rows[k];
                        r.hit_off += (uint32_t)hb[c];
                        h_erows_.p[rb[c] + k] = r;
                    }
                    if (!E.hits.empty()) std::memcpy(h_ehits_.p + hb[c], E.hits.data(), E.hits.size() * sizeof(DEnumHit));
                    for (size_t k = 0; k < E.items.size(); k++) {
                        DEnumItem it = E.items[k];
                        it.row += (uint32_t)rb[c];
                        h_eitems_.p[ib[c] + k] = it;
                    }
                };
                if (nch > 1) wp.run(nch, pack);
                else pack(0);
                d_erows_.reserve(nrow, false);
                d_ehits_.reserve(nhit, false);
                d_eitems_.reserve(nitem, false);
                d_ecnt_.reserve(2 * nitem, false);
                h_ecnt_.reserve(2 * nitem);
                NKM_HIP(hipMemcpyAsync(d_erows_.p, h_erows_.p, nrow * sizeof(DEnumRow), hipMemcpyHostToDevice, stream_));
                NKM_HIP(hipMemcpyAsync(d_ehits_.p, h_ehits_.p, nhit * sizeof(DEnumHit), hipMemcpyHostToDevice, stream_));
                NKM_HIP(hipMemcpyAsync(d_eitems_.p, h_eitems_.p, nitem * sizeof(DEnumItem), hipMemcpyHostToDevice, stream_));
                NKM_HIP(launch_enum(d_erows_.p, d_ehits_.p, d_eitems_.p, (uint32_t)nitem, d_ecnt_.p, nullptr, 0, nullptr,
                                    nullptr, stream_));
                NKM_HIP(hipMemcpyAsync(h_ecnt_.p, d_ecnt_.p, 2 * nitem * sizeof(uint32_t), hipMemcpyDeviceToHost, stream_));
                NKM_HIP(hipStreamSynchronize(stream_));
                const auto te2 = eclk::now();
                h_ebase_.reserve(2 * nitem);  // exclusive scan: every item's first group and entry
                uint64_t G = 0, E = 0;
                const size_t sch = nch > 1 && nitem >= 65536 ? (size_t)wp.size() : 1;  // chunk sums, then bases
                std::vector<uint64_t> cg(sch + 1, 0), ce(sch + 1, 0);
                auto scan_sum = [&](size_t c) {
                    uint64_t g = 0, e = 0;
                    for (size_t k = nitem * c / sch; k < nitem * (c + 1) / sch; k++) {
                        g += h_ecnt_.p[2 * k];
                        e += h_ecnt_.p[2 * k + 1];
                    }
                    cg[c + 1] = g;
                    ce[c + 1] = e;
                };
                auto scan_put = [&](size_t c) {
                    uint64_t g = cg[c], e = ce[c];
                    for (size_t k = nitem * c / sch; k < nitem * (c + 1) / sch; k++) {
                        h_ebase_.p[2 * k] = g;
                        h_ebase_.p[2 * k + 1] = e;
                        g += h_ecnt_.p[2 * k];
                        e += h_ecnt_.p[2 * k + 1];
                    }
                };
                if (sch > 1) wp.run(sch, scan_sum);
                else scan_sum(0);
                for (size_t c = 0; c < sch; c++) {
                    cg[c + 1] += cg[c];
                    ce[c + 1] += ce[c];
                }
                if (sch > 1) wp.run(sch, scan_put);
                else scan_put(0);
                G = cg[sch];
                E = ce[sch];
                const size_t g0 = cands.size(), e0 = cands.ents.size();
                // mm_matched holds int32 entry counts and group offsets
                if (e0 + E > (size_t)INT32_MAX || g0 + G > (size_t)INT32_MAX)
                    throw std::length_error("processCustom: more than 2^31 - 1 candidate entries");
                // The whole candidate list from the device straight into the
                // result arena (custom_direct_): the entries come down in
                // pinned chunks while the workers turn the previous chunk into
                // result entries, instead of one pageable copy into the
                // candidate list and a second pass (fill_matched) over it.
                const bool direct = G && g0 == 0 && e0 == 0 && par && custom_direct_mode_ && !row_shard() &&
                                    !out_in_use_.exchange(true);
                if (direct) {
                    struct Release {  // the arena goes back unless the result is handed out
                        std::atomic<bool>& f;
                        bool keep = false;
                        ~Release() { if (!keep) f.store(false); }
                    } rel{out_in_use_};
                    d_ebase_.reserve(2 * nitem, false);
                    d_eents_.reserve(2 * E, false);
                    d_eoff_.reserve(G, false);
                    NKM_HIP(hipMemcpyAsync(d_ebase_.p, h_ebase_.p, 2 * nitem * sizeof(uint64_t), hipMemcpyHostToDevice,
                                           stream_));
                    const bool slots = max_pres_ <= 1;  // every presence index 0: slot ids + group sizes
                    NKM_HIP(launch_enum(d_erows_.p, d_ehits_.p, d_eitems_.p, (uint32_t)nitem, nullptr, d_ebase_.p, 0u,
                                        d_eents_.p, d_eoff_.p, stream_, slots));
                    fill_custom_direct(G, E, slots);
                    rel.keep = true;
                } else if (G) {
                    static_assert(sizeof(GroupList::Entry) == 8, "(slot, presence index) word pairs");
                    d_ebase_.reserve(2 * nitem, false);
                    d_eents_.reserve(2 * E, false);
                    d_eoff_.reserve(G, false);
                    NKM_HIP(hipMemcpyAsync(d_ebase_.p, h_ebase_.p, 2 * nitem * sizeof(uint64_t), hipMemcpyHostToDevice,
                                           stream_));
                    NKM_HIP(launch_enum(d_erows_.p, d_ehits_.p, d_eitems_.p, (uint32_t)nitem, nullptr, d_ebase_.p,
                                        (uint32_t)e0, d_eents_.p, d_eoff_.p, stream_));
                    grow_to(cands.ents, e0 + E);
                    grow_to(cands.off, g0 + 1 + G);
                    NKM_HIP(hipMemcpyAsync(cands.ents.data() + e0, d_eents_.p, E * sizeof(GroupList::Entry),
                                           hipMemcpyDeviceToHost, stream_));
                    NKM_HIP(hipMemcpyAsync(cands.off.data() + g0 + 1, d_eoff_.p, G * sizeof(uint32_t),
                                           hipMemcpyDeviceToHost, stream_));
                    NKM_HIP(hipStreamSynchronize(stream_));
                }
                if (batch_profile_)
                    std::fprintf(stderr,
                                 "[nkm]   custom enum: rows %zu hits %zu items %zu | gather %.2f, pack+count %.2f, "
                                 "scan+write+copy %.2f ms | %llu candidates, %llu entries\n",
                                 nrow, nhit, nitem, ems(te0, te1), ems(te1, te2), ems(te2, eclk::now()),
                                 (unsigned long long)G, (unsigned long long)E);
            }
        } else if (par && !timer_live) {
            WorkPool& wp = workers();
            const size_t nch = (size_t)wp.size() * 4;
            std::vector<GroupList> outs(nch);
            wp.run(nch, [&](size_t c) {
                Scratch sc;
                for (size_t i = nchunk * c / nch; i < nchunk * (c + 1) / nch; i++) do_row(i, outs[c], sc, rev);
            });
            size_t ng = 0, ne = 0;
            for (auto& o : outs) ng += o.size(), ne += o.ents.size();
            cands.reserve_more(ng, ne);
            for (auto& o : outs) {
                const uint32_t e0 = (uint32_t)cands.ents.size();
                cands.ents.insert(cands.ents.end(), o.ents.begin(), o.ents.end());
                for (size_t g = 1; g < o.off.size(); g++) cands.off.push_back(e0 + o.off[g]);
            }
        } else {
            Scratch sc;
            for (size_t i = 0; i < nchunk; i++) {
                if (rev && !row_shard() && timer.check()) rev = rp.rev = false;  // :353-358
                do_row(i, cands, sc, rev);
            }
        }
        stats.replay_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc2).count();
    }
    return MM_OK;
}

int Core::process(mm_matched* out) {
    std::memset(out, 0, sizeof(*out));
    const auto t0 = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> pl(process_mu_);
    std::unique_lock<std::mutex> lk(mu_);
    if (custom_open_) return MM_ERR_STATE;
    if (arena_claimed_) {  // an earlier pass that claimed the arena failed before handing it out
        arena_claimed_ = false;
        out_in_use_.store(false);
    }
    bool any_active = false;
    for (uint32_t s : active_list_)
        if (live_[s] && is_active_[s]) { any_active = true; break; }
    GroupList& groups = pass_groups_;  // kept across passes: no page faults on the hot path
    groups.clear();
    if (!any_active) {  // matchmaker.go:294-298
        fill_matched(groups, out, false);
        return MM_OK;
    }
    sync_device();
    if (!active_sorted_) {
        std::sort(active_list_.begin(), active_list_.end(), [&](uint32_t a, uint32_t b) {
            if (created_[a] != created_[b]) return created_[a] < created_[b];
            return tk(a) < tk(b);
        });
        active_sorted_ = true;
    }
    UVec<uint32_t>& expired = expired_;
    expired.clear();
    PassStats stats;
    // the snapshot is taken: mutators queue until the pass ends (matchmaker.go:309)
    pass_running_ = true;
    lk.unlock();
    auto hook = [&] {
        if (pass_hook_) pass_hook_(pass_hook_ctx_);
    };
    // A pass that fails (a device error) closes without a result: the handle
    // lock is taken back, the queued mutations are applied, mutators stop
    // queueing, the pass's selections are forgotten (no ticket left the
    // index) and the device alive mask is re-uploaded whole at the next
    // pass; only the decided rows' Intervals increments stay.  Then the
    // error goes to the caller (mm_capi maps it).
    struct Unwind {
        Core& c;
        std::unique_lock<std::mutex>& lk;
        bool armed = true;
        ~Unwind() {
            if (!armed) return;
            if (!lk.owns_lock()) lk.lock();
            try {
                c.apply_pending();
            } catch (...) {
            }
            c.pass_running_ = false;
            c.custom_open_ = false;
            if (c.custom_filled_) c.out_in_use_.store(false);  // the candidates' arena was never handed out
            c.custom_filled_ = false;
            c.reset_pass_scratch();  // a walk may have thrown with its flags set
            c.sel_.assign(c.sel_.size(), 0);
            c.apply_defer_.clear();
            c.dev_slots_ = 0;  // sync_device: every slot's alive flag again
        }
    } unwind{*this, lk};
    if (cfg_.override_enabled) {
        const auto t1 = std::chrono::steady_clock::now();
        process_custom(groups, expired, stats);
        hook();
        const auto t2 = std::chrono::steady_clock::now();
        lk.lock();
        out->n_expired = (int32_t)expired.size();
        if (groups.empty() && !custom_filled_) {
            apply_pending();
            GroupList none;
            finish_pass(expired, none, true);
            pass_running_ = false;
            fill_matched(none, out, false);
        } else {
            // the pass stays open (mutators keep queueing) until
            // mm_process_commit hands back the override's choice
            custom_open_ = true;
            custom_expired_ = expired;
            if (custom_filled_) {  // the candidates are in the arena already (fill_custom_direct)
                out->group_created = out_created_.data();
                out->n_groups = (int32_t)custom_filled_g_;
                out->n_entries = (int32_t)custom_filled_e_;
                out->group_offsets = out_offs_.data();
                out->entries = out_ents_.data();
                out->is_candidates = 1;
                out->reserved2 = 1;  // the handle's arena
                custom_filled_ = false;
            } else {
                fill_matched(groups, out, true);
            }
        }
        if (std::getenv("NKM_PROFILE")) {
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            std::fprintf(stderr,
                         "[nkm] custom: sync %.2f ms | pass %.2f ms (build %.2f, search %.2f ms [kernel %.2f ms], "
                         "combos %.2f ms, %d refetches) | candidates %d (%d entries) | fill %.2f ms\n",
                         ms(t0, t1), ms(t1, t2), stats.assemble_ms, stats.search_ms, stats.eval_ms(), stats.replay_ms,
                         stats.refetches, out->n_groups, out->n_entries, ms(t2, std::chrono::steady_clock::now()));
        }
    } else {
        const auto t1 = std::chrono::steady_clock::now();
        process_default(groups, expired, stats);
        hook();
        const auto t2 = std::chrono::steady_clock::now();
        lk.lock();  // matchmaker.go:320
        out->n_expired = (int32_t)expired.size();
        const bool mutated = !pending_.empty();
        apply_pending();
        const bool fused = finish_fill_fast(expired, groups, out, mutated);
        if (!fused) finish_pass(expired, groups, true);
        pass_running_ = false;
        const auto t3 = std::chrono::steady_clock::now();
        if (!fused) fill_matched(groups, out, false);
        const auto t4 = std::chrono::steady_clock::now();
        if (std::getenv("NKM_PROFILE")) {
            auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            std::fprintf(stderr,
                         "[nkm] sync %.2f ms | pass %.2f ms (assemble %.2f, search %.2f ms [kernel %.2f ms], replay %.2f "
                         "ms, apply %.2f ms, %d batches (%d parallel), %d refetches, %d launches, %d tier lists) | finish %.2f ms | "
                         "fill %.2f ms | groups %zu | slots %zu live %u active %zu sigs %zu dict %zu | par bucket %.2f work %.2f "
                         "merge %.2f ms (task max %.2f ms, rows %llu, hits %llu) | batch: prep %.2f overlap %.2f wait %.2f "
                         "post %.2f lists %.2f (%d of %d proven, %d re-run) | replay: gather %.2f job %.2f clear %.2f | prologue %.2f asm: count %.2f scatter %.2f\n",
                         ms(t0, t1), ms(t1, t2), stats.assemble_ms, stats.search_ms, stats.eval_ms(), stats.replay_ms,
                         stats.apply_ms, stats.batches,
                         stats.parallel_batches, stats.refetches, stats.launches(), stats.tier_lists, ms(t2, t3), ms(t3, t4),
                         groups.size(), nslots(), n_live_, active_list_.size(), sigs_.size(),
                         dict_.size(), stats.par_bucket_ms, stats.par_work_ms, stats.par_merge_ms,
                         stats.par_task_max_ms, (unsigned long long)stats.par_rows, (unsigned long long)stats.par_hits,
                         stats.rb_prep_ms, stats.rb_overlap_ms, stats.rb_wait_ms, stats.rb_post_ms, stats.rb_lists_ms, stats.lists_proven,
                         stats.mscan_lists, stats.mhash_respec, stats.par_gather_ms, stats.par_job_ms, stats.par_clear_ms, stats.prologue_ms, stats.asm_count_ms,
                         stats.asm_scatter_ms);
        }
    }
    unwind.armed = false;
    const int dk = stats.dominant();  // bench.py's roofline kernel
    out->eval_kernel = dk == 2 && stats.mhash ? 4 : dk == 3 && stats.rpack ? 5 : dk == 4 ? 6 : dk == 5 ? 7 : dk;
    out->eval_ms = stats.k_ms[dk];
    out->pair_evals = stats.pair_evals;
    out->pairs_decided = stats.pairs_decided;
    out->eval_bytes = stats.k_bytes[dk];
    out->eval_launches = stats.k_launches[dk];
    out->n_batches = stats.batches;
    out->full_lists = stats.full_lists;
    out->pass_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return MM_OK;
}

int Core::process_commit(const int32_t* offs, const mm_entry_ref* ents, int32_t n_groups, mm_matched* out) {
    std::memset(out, 0, sizeof(*out));
    const auto t0 = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> pl(process_mu_);
    std::lock_guard<std::mutex> lk(mu_);
    if (!custom_open_) return MM_ERR_STATE;
    // the mutations queued while the pass was open come first: a chosen
    // group that lost a ticket is then dropped by the re-check (:326-341)
    apply_pending();
    // the chosen groups' entries back to slots (a ticket no longer known
    // becomes kNoSlot: its group fails the re-check), on the workers
    for (int g = 0; g < n_groups; g++)
        if (offs[g + 1] < offs[g]) return MM_ERR_ARG;
    GroupList groups;
    const int32_t o0 = n_groups > 0 ? offs[0] : 0;
    const size_t ne = n_groups > 0 ? (size_t)(offs[n_groups] - o0) : 0;
    groups.off.resize((size_t)n_groups + 1);
    for (int g = 0; g <= n_groups; g++) groups.off[g] = (uint32_t)(n_groups > 0 ? offs[g] - o0 : 0);
    groups.ents.resize(ne);
    auto look = [&](size_t lo, size_t hi) {
        for (size_t k = lo; k < hi; k++) {
            const mm_entry_ref& e = ents[o0 + k];
            const int64_t s = slot_of_ticket(e.ticket ? e.ticket : "");
            groups.ents[k] = {s < 0 ? kNoSlot : (uint32_t)s, e.presence_index};
        }
    };
    if (par_mode_ && ne >= par_min(65536)) {
        WorkPool& wp = workers();
        const size_t nch = (size_t)wp.size() * 4;
        wp.run(nch, [&](size_t c) { look(ne * c / nch, ne * (c + 1) / nch); });
    } else {
        look(0, ne);
    }
    // processCustom never deletes from the index during the pass; matched
    // tickets leave it here (their zombie documents would be filtered as
    // "missing index" by later passes, matchmaker_process.go:432-437).
    const auto t1 = std::chrono::steady_clock::now();
    UVec<uint32_t> exp = custom_expired_;
    finish_pass(exp, groups, false);
    custom_open_ = false;
    pass_running_ = false;
    custom_expired_.clear();
    const auto t2 = std::chrono::steady_clock::now();
    fill_matched(groups, out, false);
    if (std::getenv("NKM_PROFILE")) {
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "[nkm] commit: %d groups | lookup %.2f ms | finish %.2f ms | fill %.2f ms\n", n_groups,
                     ms(t0, t1), ms(t1, t2), ms(t2, std::chrono::steady_clock::now()));
    }
    return MM_OK;
}

}  // namespace nkm

extern "C" int32_t mm_debug_group_indexes(const int32_t* counts, const int64_t* created_at, int32_t n,
                                          int32_t required, int32_t* group_offsets, int32_t* group_members,
                                          int64_t* avg_created_at, int32_t cap) {
    std::vector<int32_t> cnt(counts, counts + n);
    std::vector<int64_t> cr(created_at, created_at + n);
    std::vector<uint32_t> in(n);
    for (int32_t i = 0; i < n; i++) in[i] = (uint32_t)i;
    std::vector<nkm::IG> out;
    nkm::group_indexes(in, 0, required, cnt.data(), cr.data(), out);
    int32_t g = 0, k = 0;
    group_offsets[0] = 0;
    for (auto& gr : out) {
        if (g >= cap) break;
        for (uint32_t m : gr.idx)
            if (k < 8 * cap) group_members[k++] = (int32_t)m;
        avg_created_at[g] = gr.avg;
        group_offsets[++g] = k;
    }
    return g;
}

extern "C" int mm_debug_term_match(int32_t kind, const char* pattern, int32_t fuzziness, const char* term,
                                   double* boost) try {
    nkm::TermMatcher m;
    *boost = 0.0;
    if (kind == 2) {
        if (fuzziness < 0 || fuzziness > 2) return -1;
        m.kind = nkm::TermMatcher::K_FUZZY;
        m.pattern = pattern;
        m.fuzziness = fuzziness;
    } else {
        m.kind = nkm::TermMatcher::K_REGEXP;
        m.pattern = kind == 3 ? nkm::wildcard_to_regexp(pattern) : std::string(pattern);
        nkm::MtStatus st = m.re.compile(m.pattern);
        if (st != nkm::MT_OK) return st == nkm::MT_UNSUPPORTED ? -2 : -1;
    }
    return m.accept(term, boost) ? 1 : 0;
} catch (...) {
    return -1;
}

extern "C" int mm_debug_compile(const char* query) {
    try {
        nkm::CompiledQuery cq;
        int rc = nkm::compile_query(query ? query : "", &cq);
        return rc == nkm::CQ_OK ? MM_OK : rc == nkm::CQ_UNSUPPORTED ? MM_ERR_UNSUPPORTED : MM_ERR_QUERY_INVALID;
    } catch (...) {
        return MM_ERR_INDEX;
    }
}

namespace nkm {

int32_t Core::debug_hits(const std::string& ticket, const char** tk, double* sc, int32_t cap) {
    std::lock_guard<std::mutex> pl(process_mu_);  // the pass owns the stream and the device buffers
    std::lock_guard<std::mutex> lk(mu_);
    int64_t T = slot_of_ticket(ticket);
    if (T < 0) return -1;
    sync_device();
    const DStore st = dstore();
    PassStats stats;
    std::vector<uint8_t> sel(nslots(), 0);
    Replay rp(*this, sel, cfg_.rev_precision != 0, cfg_.max_intervals, stats, st, stream_);
    BGroup g;
    g.sig = sig_[T];
    const Sig& s = sigs_[sig_[T]];
    g.n_fields = s.n_fields;
    g.d.clause_off = s.clause_off;
    g.d.n_clauses = s.n_clauses;
    g.d.qkind = s.qkind;
    g.d.var_score = s.var_score ? 1 : 0;
    g.d.tmin = s.tmin;
    g.d.tmax = s.tmax;
    g.d.tparty = s.tparty;
    g.d.rev_slot = kNoSlot;
    g.d.ub_key = s.ub_key;
    while (order_head_ < order_.size() && !live_[order_[order_head_]]) order_head_++;
    choose_source(s, g.d);
    g.d.k = 1;
    g.n = 0;
    g.complete = false;
    while (!g.complete) rp.fetch_more(g);
    debug_strings_.clear();
    int32_t n = 0;
    auto skip = [&](uint32_t i) { return g.slot(i) == (uint32_t)T || rp.same_party((uint32_t)T, g.slot(i)); };
    for (uint32_t i = 0; i < g.n; i++) {
        if (skip(i)) continue;
        debug_strings_.emplace_back(this->tk(g.slot(i)));
    }
    for (uint32_t i = 0; i < g.n; i++) {
        if (skip(i)) continue;
        if (n < cap) {
            if (tk) tk[n] = debug_strings_[n].c_str();
            int64_t key = g.hits[i].key;
            if (key < 0) key ^= INT64_MAX;
            double d;
            std::memcpy(&d, &key, 8);
            if (sc) sc[n] = d;
        }
        n++;
    }
    return n;
}

}  // namespace nkm
