// nakama_amd/csrc/mm_kernels.hip — CDNA4 (gfx950) kernels of the interval pass.
//
// search_kernel: one 256-thread workgroup (4 wave64) per search.  The search
// streams its candidate source (a posting list of its most selective required
// term, or the created-at scan order) in tiles of 256 candidates, one
// candidate per lane: coalesced 4-B slot ids, then gathers of the SoA columns
// the compiled query references (alive, Min/MaxCount, party, field columns).
// Each lane evaluates the predicate/score bytecode (wave-uniform clause loop,
// scalar loads) — the bluge search of matchmaker_process.go:65-103 restated as
// a flat predicate.  Survivors are:
//   * constant-score searches: compacted in source order with wave ballots +
//     an LDS scan across the 4 waves (source order == the reference's
//     (-score, created_at, doc) sort when every hit scores the same);
//   * variable-score searches: merged into an LDS top-K list ordered by
//     (score desc, source position asc) with a rank merge, with early exit once
//     the K-th score reaches the query's score upper bound.
// With RevPrecision the lane also evaluates the hit's own query against the
// searching ticket's document (validateMatch, matchmaker.go:1042-1068).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdlib>

#include "mm_device.h"
#include "qcompile.h"

namespace nkm {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr int kVarK = 512;  // LDS capacity of a variable-score top-K list (search_kernel<kVarK>)

__device__ __forceinline__ int64_t dsortable(double f) {
    int64_t i = __double_as_longlong(f);
    return i < 0 ? (i ^ 0x7fffffffffffffffLL) : i;
}

// OP_TERMSET: is keyword id `val` in the matcher's accepted set?  Binary search
// of the set's ascending ids; *sc = the clause's score for that term.
__device__ __forceinline__ bool termset_hit(const DStore& st, uint32_t set, int64_t val, double* sc) {
    const uint32_t off = st.tset_desc[2 * set];
    uint32_t lo = 0, hi = st.tset_desc[2 * set + 1];
    const uint32_t v = (uint32_t)val;
    const uint32_t* __restrict__ ids = st.tset_ids + off;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ids[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    if (lo < st.tset_desc[2 * set + 1] && ids[lo] == v) { *sc = st.tset_sc[off + lo]; return true; }
    return false;
}

// Parsed-query evaluation on document `s` (bluge BooleanSearcher semantics,
// search_boolean.go:174-244).  *sp receives the parsed query's score.
__device__ __forceinline__ bool eval_parsed(const DStore& st, uint8_t qkind, const DClause* __restrict__ cl, int n,
                                            uint32_t s, double* sp) {
    if (qkind == QK_MATCHALL) { *sp = 1.0; return true; }
    if (qkind == QK_MATCHNONE) return false;
    double ms = 0.0, ss = 0.0;
    bool has_must = false, has_should = false, any_should = false, fail = false;
    for (int i = 0; i < n; i++) {
        const DClause c = cl[i];
        bool h = false;
        double sc = c.score;
        if (c.op != OP_FALSE) {
            // global, not flat, loads (a column pointer read from memory is generic)
            const uint8_t kind = ((const __attribute__((address_space(1))) uint8_t*)st.fkind[c.field])[s];
            const int64_t val = ((const __attribute__((address_space(1))) int64_t*)st.fval[c.field])[s];
            if (c.op == OP_TERM) h = kind == KIND_KEYWORD && val == (int64_t)c.term;
            else if (c.op == OP_RANGE) h = kind == KIND_NUMERIC && val >= c.lo && val <= c.hi;
            else if (c.op == OP_TERMSET) h = kind == KIND_KEYWORD && termset_hit(st, c.term, val, &sc);
            else h = (kind == KIND_KEYWORD && val == (int64_t)c.term) || (kind == KIND_NUMERIC && val == c.lo);
        }
        if (c.occur == OCC_MUST) { has_must = true; if (h) ms += sc; else fail = true; }
        else if (c.occur == OCC_SHOULD) { has_should = true; if (h) { ss += sc; any_should = true; } }
        else if (h) fail = true;
    }
    if (fail) return false;
    if (!has_must && !has_should) { *sp = 1.0; return true; }  // only mustNots: MatchAll(1)
    if (!has_must) { *sp = ss; return any_should; }
    *sp = any_should ? ms + ss : ms;
    return true;
}

// eval_parsed with its loads in two batched rounds: a query of at most
// kEvalBatch clauses has every clause loaded at once, then every clause's
// column value and kind at slot s at once (the column pointers of the first
// kFieldLds fields from the workgroup's LDS table, load_field_table), instead
// of a clause -> pointer -> column chain per clause in turn.  The hit and
// score logic, and the order of the double additions, are eval_parsed's, so
// the score bits are identical.  Longer queries: eval_parsed.
constexpr int kEvalBatch = 4;
constexpr uint32_t kFieldLds = 64;
struct FieldTable {
    const int64_t* val[kFieldLds];
    const uint8_t* kind[kFieldLds];
};
// threads [0, kFieldLds) copy the table; the caller syncs before use.  A
// kernel uses eval_batched only when the table holds every field
// (field_table_ok: a uniform test), eval_parsed otherwise.
__device__ __forceinline__ void load_field_table(const DStore& st, FieldTable& ft) {
    if (threadIdx.x < kFieldLds && threadIdx.x < st.n_fields) {
        ft.val[threadIdx.x] = st.fval[threadIdx.x];
        ft.kind[threadIdx.x] = st.fkind[threadIdx.x];
    }
}
__device__ __forceinline__ bool field_table_ok(const DStore& st) { return st.n_fields <= kFieldLds; }
template <int NB = kEvalBatch>
__device__ __forceinline__ bool eval_batched(const DStore& st, const FieldTable& ft, uint8_t qkind,
                                             const DClause* __restrict__ cl, int n, uint32_t s, double* sp) {
    // every load first and unconditional — clause indexes clamped into the
    // list (the table's first clause for an empty one), field ids into the
    // table (OP_FALSE names no column) — so the clauses come in one round and
    // their columns in the next; the uncommon query shapes are decided after
    const int nn = n < 1 ? 1 : (n > NB ? NB : n);
    const DClause* __restrict__ cb = n >= 1 ? cl : st.clauses;
    DClause c[NB];
#pragma unroll
    for (int i = 0; i < NB; i++) c[i] = cb[i < nn ? i : nn - 1];
    uint8_t kind[NB];
    int64_t val[NB];
    // global (not flat) loads: a flat load also counts against lgkmcnt, so
    // every LDS wait would wait for it
    typedef const __attribute__((address_space(1))) uint8_t gu8;
    typedef const __attribute__((address_space(1))) int64_t gi64;
#pragma unroll
    for (int i = 0; i < NB; i++) {
        const uint32_t f = c[i].op == OP_FALSE ? 0u : min((uint32_t)c[i].field, st.n_fields - 1);
        kind[i] = ((gu8*)ft.kind[f])[s];
        val[i] = ((gi64*)ft.val[f])[s];
    }
    if (qkind == QK_MATCHALL) { *sp = 1.0; return true; }
    if (qkind == QK_MATCHNONE) return false;
    if (n > NB) return eval_parsed(st, qkind, cl, n, s, sp);
    if (n <= 0) { *sp = 1.0; return true; }  // eval_parsed: no must, no should -> MatchAll(1)
    double ms = 0.0, ss = 0.0;
    bool has_must = false, has_should = false, any_should = false, fail = false;
#pragma unroll
    for (int i = 0; i < NB; i++) {
        if (i >= n) break;
        bool h = false;
        double sc = c[i].score;
        if (c[i].op != OP_FALSE) {
            if (c[i].op == OP_TERM) h = kind[i] == KIND_KEYWORD && val[i] == (int64_t)c[i].term;
            else if (c[i].op == OP_RANGE) h = kind[i] == KIND_NUMERIC && val[i] >= c[i].lo && val[i] <= c[i].hi;
            else if (c[i].op == OP_TERMSET) h = kind[i] == KIND_KEYWORD && termset_hit(st, c[i].term, val[i], &sc);
            else h = (kind[i] == KIND_KEYWORD && val[i] == (int64_t)c[i].term) || (kind[i] == KIND_NUMERIC && val[i] == c[i].lo);
        }
        if (c[i].occur == OCC_MUST) { has_must = true; if (h) ms += sc; else fail = true; }
        else if (c[i].occur == OCC_SHOULD) { has_should = true; if (h) { ss += sc; any_should = true; } }
        else if (h) fail = true;
    }
    if (fail) return false;
    if (!has_must && !has_should) { *sp = 1.0; return true; }
    if (!has_must) { *sp = ss; return any_should; }
    *sp = any_should ? ms + ss : ms;
    return true;
}

// eval_batched<NB> on document s whose values of up to two fields (pf: the
// launch's prefetch fields, npf of them) are already in registers (pk / pv):
// a clause naming one of them reads the register, any other clause loads
// its column as eval_batched does.  Same hit and score logic, same order of
// the double additions.
template <int NB>
__device__ __forceinline__ bool eval_batched_pf(const DStore& st, const FieldTable& ft, uint8_t qkind,
                                                const DClause* __restrict__ cl, int n, uint32_t s, double* sp,
                                                uint32_t npf, const uint16_t* pf, const uint8_t* pk, const int64_t* pv) {
    const int nn = n < 1 ? 1 : (n > NB ? NB : n);
    const DClause* __restrict__ cb = n >= 1 ? cl : st.clauses;
    DClause c[NB];
#pragma unroll
    for (int i = 0; i < NB; i++) c[i] = cb[i < nn ? i : nn - 1];
    uint8_t kind[NB];
    int64_t val[NB];
    typedef const __attribute__((address_space(1))) uint8_t gu8;
    typedef const __attribute__((address_space(1))) int64_t gi64;
#pragma unroll
    for (int i = 0; i < NB; i++) {
        const uint32_t f = c[i].op == OP_FALSE ? 0u : min((uint32_t)c[i].field, st.n_fields - 1);
        if (npf > 0 && f == pf[0]) {
            kind[i] = pk[0];
            val[i] = pv[0];
        } else if (npf > 1 && f == pf[1]) {
            kind[i] = pk[1];
            val[i] = pv[1];
        } else {
            kind[i] = ((gu8*)ft.kind[f])[s];
            val[i] = ((gi64*)ft.val[f])[s];
        }
    }
    if (qkind == QK_MATCHALL) { *sp = 1.0; return true; }
    if (qkind == QK_MATCHNONE) return false;
    if (n > NB) return eval_parsed(st, qkind, cl, n, s, sp);
    if (n <= 0) { *sp = 1.0; return true; }
    double ms = 0.0, ss = 0.0;
    bool has_must = false, has_should = false, any_should = false, fail = false;
    bool tset = false;
#pragma unroll
    for (int i = 0; i < NB; i++) tset |= (i < n) & (c[i].op == OP_TERMSET);
    if (__ballot(tset) == 0) {
        // no regexp / wildcard / fuzzy clause in the wave: every clause's hit
        // and contribution by selects, no branch per clause (a skipped
        // addition is an addition of +0.0: the sums' bits are the loop's)
#pragma unroll
        for (int i = 0; i < NB; i++) {
            const bool act = i < n;
            const bool kw = kind[i] == KIND_KEYWORD, nu = kind[i] == KIND_NUMERIC;
            const bool eqt = val[i] == (int64_t)c[i].term;
            const uint8_t op = c[i].op;
            const bool h = act & (((op == OP_TERM) & kw & eqt) |
                                  ((op == OP_RANGE) & nu & (val[i] >= c[i].lo) & (val[i] <= c[i].hi)) |
                                  ((op == OP_NUMLIT) & ((kw & eqt) | (nu & (val[i] == c[i].lo)))));
            const bool must = act & (c[i].occur == OCC_MUST), should = act & (c[i].occur == OCC_SHOULD);
            const bool mnot = act & (c[i].occur == OCC_MUSTNOT);
            has_must |= must;
            has_should |= should;
            ms += (must & h) ? c[i].score : 0.0;
            ss += (should & h) ? c[i].score : 0.0;
            any_should |= should & h;
            fail |= (must & !h) | (mnot & h);
        }
    } else {
#pragma unroll
        for (int i = 0; i < NB; i++) {
            if (i >= n) break;
            bool h = false;
            double sc = c[i].score;
            if (c[i].op != OP_FALSE) {
                if (c[i].op == OP_TERM) h = kind[i] == KIND_KEYWORD && val[i] == (int64_t)c[i].term;
                else if (c[i].op == OP_RANGE) h = kind[i] == KIND_NUMERIC && val[i] >= c[i].lo && val[i] <= c[i].hi;
                else if (c[i].op == OP_TERMSET) h = kind[i] == KIND_KEYWORD && termset_hit(st, c[i].term, val[i], &sc);
                else h = (kind[i] == KIND_KEYWORD && val[i] == (int64_t)c[i].term) || (kind[i] == KIND_NUMERIC && val[i] == c[i].lo);
            }
            if (c[i].occur == OCC_MUST) { has_must = true; if (h) ms += sc; else fail = true; }
            else if (c[i].occur == OCC_SHOULD) { has_should = true; if (h) { ss += sc; any_should = true; } }
            else if (h) fail = true;
        }
    }
    if (fail) return false;
    if (!has_must && !has_should) { *sp = 1.0; return true; }
    if (!has_must) { *sp = ss; return any_should; }
    *sp = any_should ? ms + ss : ms;
    return true;
}

struct Cand {
    uint32_t slot;
    uint32_t idx;
    int64_t key;
    uint8_t rev;
    bool m;
    bool live;
};

__device__ __forceinline__ Cand eval_candidate(const DStore& st, const DGroup& g, const uint32_t* __restrict__ src,
                                               uint32_t idx) {
    Cand c{0, idx, 0, 1, false, false};
    if (g.src_len == 0) return c;
    // unconditional loads (a clamped position past the end, masked below):
    // the slot id, then alive / Min / Max / party in one round trip
    const bool valid = idx < g.src_len;
    const uint32_t s = src[g.src_off + (valid ? idx : g.src_len - 1)];
    const uint8_t al = st.alive[s];
    const int32_t mn = st.minc[s], mx = st.maxc[s];
    const uint32_t pt = g.tparty != kNoParty ? st.party[s] : 0u;
    if (!valid) return c;
    c.slot = s;
    bool m = al != 0;
    c.live = m;
    m = m && mn >= g.tmin && mx <= g.tmax && (g.tparty == kNoParty || pt != g.tparty);
    double sp = 0.0;
    if (m) m = eval_parsed(st, g.qkind, st.clauses + g.clause_off, g.n_clauses, s, &sp);
    if (m) {
        // top-level BooleanQuery{must: parsed, min_count range, max_count range}
        c.key = dsortable((sp + 1.0) + 1.0);
        if (g.has_cursor) m = c.key < g.cur_key || (c.key == g.cur_key && idx > g.cur_idx);
    }
    if (m && g.rev_slot != kNoSlot) {
        const DQuery q = st.squery[s];
        double d;
        c.rev = eval_parsed(st, q.kind, st.clauses + q.clause_off, q.n_clauses, g.rev_slot, &d) ? 1 : 0;
    }
    c.m = m;
    return c;
}

// VK = 0: the instantiation for constant-score searches (no top-K list in
// LDS); VK = kVarK: variable-score searches.  Both are launched over the same
// group array and each returns at once on the other kind's groups, so the
// constant-score searches keep a small LDS footprint (full occupancy).
template <int VK>
__global__ __launch_bounds__(kBlock) void search_kernel(DStore st, const DGroup* __restrict__ groups,
                                                        DHit* __restrict__ out, uint8_t* __restrict__ out_rev,
                                                        DGroupResult* __restrict__ res) {
    constexpr int LV = VK > 0 ? VK : 1;
    __shared__ uint32_t wave_cnt[kWaves];
    __shared__ int64_t wave_max[kWaves];
    // variable-score list (double-buffered) + tile staging
    __shared__ int64_t lkey[2][LV];
    __shared__ uint32_t lidx[2][LV];
    __shared__ uint32_t lslot[2][LV];
    __shared__ uint8_t lrev[2][LV];
    __shared__ int64_t tkey[kBlock];
    __shared__ int64_t tsk[kBlock];  // the tile's keys in rank order (descending)
    __shared__ uint32_t tidx[kBlock];
    __shared__ uint32_t tslot[kBlock];
    __shared__ uint8_t trev[kBlock];

    DGroup g = groups[blockIdx.x];
    // path 2: a top-tier list.  The constant-score instantiation (launched
    // first) compacts the hits scoring exactly ub_key in source order; the
    // variable-score one then appends, when that tier ended before the
    // capacity, the top-K of the hits scoring below it (see below).
    const bool tier = g.path == 2;
    if (tier ? false : ((g.var_score != 0) != (VK > 0) || g.path != 0)) return;  // another instantiation's / kernel's search
    const uint32_t* src = g.src_kind == 0 ? st.order : st.postings;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const uint32_t K = g.k;
    __shared__ uint32_t s_live;
    uint32_t my_live = 0;
    if (tid == 0) s_live = 0;
    __syncthreads();

    if (VK == 0) {
        // ---- ordered compaction -------------------------------------------------
        uint32_t count = 0;
        uint32_t base = 0;
        bool stopped = false;
        for (; base < g.src_len; base += kBlock) {
            Cand c = eval_candidate(st, g, src, base + tid);
            my_live += c.live;
            // A variable-score search's list is sorted by (score desc, source
            // position asc): its hits scoring the top score ub_key come first,
            // in source order, so compacting only those gives an exact prefix
            // of the sorted list of any length (the LDS top-K stops at kVarK).
            // The host takes this path only when every clause score sums
            // exactly in any order (ub_key is then the top tier's exact key).
            if (tier) c.m = c.m && c.key == g.ub_key;
            const uint64_t mask = __ballot(c.m);
            if (lane == 0) wave_cnt[wave] = (uint32_t)__popcll(mask);
            __syncthreads();
            uint32_t off = 0, tot = 0;
            for (int w = 0; w < kWaves; w++) {
                const uint32_t v = wave_cnt[w];
                off += (w < wave) ? v : 0;
                tot += v;
            }
            if (c.m) {
                const uint32_t pos = count + off + (uint32_t)__popcll(mask & lt_mask);
                if (pos < K) {
                    out[g.out_off + pos] = DHit{c.slot, c.idx, c.key};
                    if (out_rev) out_rev[g.out_off + pos] = c.rev;
                }
            }
            count += tot;
            __syncthreads();
            if (count > K) { stopped = true; base += kBlock; break; }
        }
        atomicAdd(&s_live, my_live);
        __syncthreads();
        if (tid == 0) {
            // a top-tier list is never complete: lower-scoring hits may follow
            res[blockIdx.x] = DGroupResult{count < K ? count : K, stopped || tier ? 0u : 1u,
                                           base < g.src_len ? base : g.src_len, count, s_live, 0u};
        }
        return;
    }

    // ---- variable-score top-K ------------------------------------------------------
    // A top-tier list's tail: the hits scoring below ub_key (a cursor at
    // (ub_key, past every position)), at most the capacity left, written
    // after the tier; nothing when the tier filled the list (it is cut there).
    DGroupResult r0{0, 0, 0, 0, 0, 0};
    uint32_t K_avail = K;
    if (tier) {
        r0 = res[blockIdx.x];
        if (r0.count >= K) return;
        K_avail = K - r0.count;
        g.has_cursor = 1;
        g.cur_key = g.ub_key;
        g.cur_idx = 0xFFFFFFFFu;
        g.out_off += r0.count;
    }
    const uint32_t KK = K_avail < (uint32_t)VK ? K_avail : (uint32_t)VK;
    uint32_t n = 0, total = 0;
    int cur = 0;
    bool early = false;
    uint32_t base = 0;
    for (; base < g.src_len; base += kBlock) {
        Cand c = eval_candidate(st, g, src, base + tid);
        my_live += c.live;
        const uint64_t pre = __ballot(c.m);
        if (n == KK && c.m) c.m = c.key > lkey[cur][KK - 1];
        const uint64_t mask = __ballot(c.m);
        if (lane == 0) { wave_cnt[wave] = (uint32_t)__popcll(mask); wave_max[wave] = (int64_t)__popcll(pre); }
        __syncthreads();
        uint32_t off = 0, cnt = 0;
        for (int w = 0; w < kWaves; w++) {
            const uint32_t v = wave_cnt[w];
            off += (w < wave) ? v : 0;
            cnt += v;
            total += (uint32_t)wave_max[w];
        }
        if (cnt == 0) { __syncthreads(); continue; }
        if (c.m) {
            const uint32_t p = off + (uint32_t)__popcll(mask & lt_mask);
            tkey[p] = c.key; tidx[p] = c.idx; tslot[p] = c.slot; trev[p] = c.rev;
        }
        __syncthreads();
        const int nxt = cur ^ 1;
        if ((uint32_t)tid < cnt) {
            const int64_t k = tkey[tid];
            // rank among the old list: entries with key >= k (list is sorted desc)
            uint32_t lo = 0, hi = n;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (lkey[cur][mid] >= k) lo = mid + 1; else hi = mid;
            }
            // rank within the tile (ties: earlier source position first)
            uint32_t rt = 0;
            for (uint32_t t = 0; t < cnt; t++) {
                const int64_t kt = tkey[t];
                rt += (kt > k) || (kt == k && t < (uint32_t)tid);
            }
            tsk[rt] = k;
            const uint32_t r = lo + rt;
            if (r < KK) { lkey[nxt][r] = k; lidx[nxt][r] = tidx[tid]; lslot[nxt][r] = tslot[tid]; lrev[nxt][r] = trev[tid]; }
        }
        __syncthreads();
        for (uint32_t i = tid; i < n; i += kBlock) {
            const int64_t k = lkey[cur][i];
            // tile keys strictly above k: binary search of the rank-ordered tile
            uint32_t lo = 0, hi = cnt;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (tsk[mid] > k) lo = mid + 1; else hi = mid;
            }
            const uint32_t r = i + lo;
            if (r < KK) { lkey[nxt][r] = k; lidx[nxt][r] = lidx[cur][i]; lslot[nxt][r] = lslot[cur][i]; lrev[nxt][r] = lrev[cur][i]; }
        }
        n = (n + cnt < KK) ? n + cnt : KK;
        cur = nxt;
        __syncthreads();
        if (n == KK && lkey[cur][KK - 1] >= g.ub_key) { early = true; base += kBlock; break; }
    }
    for (uint32_t i = tid; i < n; i += kBlock) {
        out[g.out_off + i] = DHit{lslot[cur][i], lidx[cur][i], lkey[cur][i]};
        if (out_rev) out_rev[g.out_off + i] = lrev[cur][i];
    }
    atomicAdd(&s_live, my_live);
    __syncthreads();
    if (tid == 0) {
        const bool complete = !early && total <= KK;
        const uint32_t scanned = base < g.src_len ? base : g.src_len;
        res[blockIdx.x] = DGroupResult{r0.count + n, complete ? 1u : 0u, scanned > r0.scanned ? scanned : r0.scanned,
                                       r0.matched + total, r0.live + s_live, 0u};
    }
}

// ---- constant-score scan (chunked) -----------------------------------------------
// One 256-thread workgroup per chunk of kScanJ*256 source positions of a
// constant-score search (every hit scores the same, so the hit order is the
// source order).  Lane-major layout: position j*256+tid is the lane's j-th
// candidate, so every column load is one coalesced (slot ids) or gathered
// access per j, and all kScanJ loads of a column are in flight together —
// one memory round trip per column instead of one per 256-candidate tile.
// Survivors are compacted in source order (ballots + one LDS exchange) into
// the chunk's scratch region; stitch_kernel places the chunks.
constexpr int kScanJ = 8;
constexpr int kScanChunk = kScanJ * kBlock;

__global__ __launch_bounds__(kBlock) void scan_kernel(DStore st, const DGroup* __restrict__ chunks,
                                                      DHit* __restrict__ out, DGroupResult* __restrict__ res) {
    __shared__ uint32_t wcnt[kScanJ][kWaves];
    __shared__ uint32_t wlive[kWaves];
    const DGroup g = chunks[blockIdx.x];
    const uint32_t* __restrict__ src = (g.src_kind == 0 ? st.order : st.postings) + g.src_off;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t s[kScanJ];
    bool m[kScanJ];
#pragma unroll
    for (int j = 0; j < kScanJ; j++) {
        const uint32_t i = (uint32_t)(j * kBlock + tid);
        s[j] = i < g.src_len ? src[i] : kNoSlot;
    }
#pragma unroll
    for (int j = 0; j < kScanJ; j++) m[j] = s[j] != kNoSlot && st.alive[s[j]] != 0;
    uint32_t live = 0;
#pragma unroll
    for (int j = 0; j < kScanJ; j++) live += m[j];
#pragma unroll
    for (int j = 0; j < kScanJ; j++)
        if (m[j]) m[j] = st.minc[s[j]] >= g.tmin && st.maxc[s[j]] <= g.tmax;
    if (g.tparty != kNoParty) {
#pragma unroll
        for (int j = 0; j < kScanJ; j++)
            if (m[j]) m[j] = st.party[s[j]] != g.tparty;
    }
    // parsed query (eval_parsed, one clause at a time over the lane's candidates)
    double ms[kScanJ], ss[kScanJ];
    bool anys[kScanJ];
#pragma unroll
    for (int j = 0; j < kScanJ; j++) { ms[j] = 0.0; ss[j] = 0.0; anys[j] = false; }
    bool has_must = false, has_should = false;
    if (g.qkind == QK_MATCHNONE) {
#pragma unroll
        for (int j = 0; j < kScanJ; j++) m[j] = false;
    } else if (g.qkind != QK_MATCHALL) {
        const DClause* __restrict__ cl = st.clauses + g.clause_off;
        for (int c = 0; c < g.n_clauses; c++) {
            const DClause k = cl[c];
            has_must |= k.occur == OCC_MUST;
            has_should |= k.occur == OCC_SHOULD;
            const int64_t* __restrict__ fv = st.fval[k.field];
            const uint8_t* __restrict__ fk = st.fkind[k.field];
#pragma unroll
            for (int j = 0; j < kScanJ; j++) {
                if (!m[j]) continue;
                bool h = false;
                double sc = k.score;
                if (k.op != OP_FALSE) {
                    const uint8_t kind = fk[s[j]];
                    const int64_t val = fv[s[j]];
                    if (k.op == OP_TERM) h = kind == KIND_KEYWORD && val == (int64_t)k.term;
                    else if (k.op == OP_RANGE) h = kind == KIND_NUMERIC && val >= k.lo && val <= k.hi;
                    else if (k.op == OP_TERMSET) h = kind == KIND_KEYWORD && termset_hit(st, k.term, val, &sc);
                    else h = (kind == KIND_KEYWORD && val == (int64_t)k.term) || (kind == KIND_NUMERIC && val == k.lo);
                }
                if (k.occur == OCC_MUST) { if (h) ms[j] += sc; else m[j] = false; }
                else if (k.occur == OCC_SHOULD) { if (h) { ss[j] += sc; anys[j] = true; } }
                else if (h) m[j] = false;
            }
        }
    }
    int64_t key[kScanJ];
#pragma unroll
    for (int j = 0; j < kScanJ; j++) {
        double sp = 1.0;  // MatchAll, or only mustNots: MatchAll(1)
        if (g.qkind != QK_MATCHALL && (has_must || has_should)) {
            if (!has_must) { sp = ss[j]; m[j] = m[j] && anys[j]; }
            else sp = anys[j] ? ms[j] + ss[j] : ms[j];
        }
        key[j] = dsortable((sp + 1.0) + 1.0);  // top-level {parsed, min_count, max_count} conjunction
    }
    // ordered compaction: position j*256+tid precedes (j, tid+1) and (j+1, *)
    uint64_t mask[kScanJ];
#pragma unroll
    for (int j = 0; j < kScanJ; j++) {
        mask[j] = __ballot(m[j]);
        if (lane == 0) wcnt[j][wave] = (uint32_t)__popcll(mask[j]);
    }
    uint32_t wl = live;
    for (int o = 32; o > 0; o >>= 1) wl += __shfl_xor(wl, o);
    if (lane == 0) wlive[wave] = wl;
    __syncthreads();
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < kScanJ; j++) {
        uint32_t before = 0, tot = 0;
        for (int w = 0; w < kWaves; w++) {
            const uint32_t v = wcnt[j][w];
            before += (w < wave) ? v : 0;
            tot += v;
        }
        if (m[j]) {
            const uint32_t pos = run + before + (uint32_t)__popcll(mask[j] & lt_mask);
            out[g.out_off + pos] = DHit{s[j], (uint32_t)(j * kBlock + tid), key[j]};
        }
        run += tot;
    }
    if (tid == 0) {
        uint32_t lv = 0;
        for (int w = 0; w < kWaves; w++) lv += wlive[w];
        res[blockIdx.x] = DGroupResult{run, 1u, g.src_len, run, lv, 0u};
    }
}

// ---- multi-signature scan over the scan order ---------------------------------------
// When a batch's constant-score searches together cover most of the store
// (C3: 8 pool signatures, each a quarter of the store through its region
// posting list), gathering every signature's candidates through posting
// lists re-reads the same column lines once per signature.  mscan_kernel
// instead streams the scan order (created-at order: near-contiguous slots)
// once, loads each candidate's columns once into registers, and evaluates
// every signature of the batch on them — a (signatures x candidates) tile per
// workgroup, the signatures read wave-uniformly through the scalar cache.
// Each signature's survivors are compacted in scan order (= its hit order
// when all its hits score the same) into the (signature, chunk) scratch cell;
// stitch_kernel places the cells.  (A single-pass variant that ranked its
// chunks by a look-back over the earlier chunks' published counts ran 46 us
// against this kernel's + stitch's on C3 1M: every chunk of the one-round
// grid waited on the slowest earlier one; DESIGN.md.)
// MJ candidates per lane (a chunk = MJ * 256 candidates per workgroup; the
// 64-bit match word holds 64 / MJ signatures).
constexpr int kMaxMSig = 16;
constexpr int kMaxMField = 4;
constexpr int kMaxMClause = 64;           // clauses of all the batch's mscan signatures
__host__ __device__ constexpr uint64_t sig_stride(int mj) {  // bit q * mj of every signature q
    return mj == 8 ? 0x0101010101010101ull : mj == 4 ? 0x1111111111111111ull : 0x5555555555555555ull;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// NF: fields the signatures read, 0-4 (registers per candidate scale with it);
// GEN: some signature is not term-only (the clause loop is compiled in).
template <int NF, bool GEN, int kMJ>
__global__ __launch_bounds__(kBlock) void mscan_kernel(DStore st, DMScan ms, const DMSig* __restrict__ sigs,
                                                       const DClause* __restrict__ mcl, uint32_t* __restrict__ out,
                                                       DGroupResult* __restrict__ res) {
    static_assert(kMJ == 2 || kMJ == 4 || kMJ == 8, "2, 4 or 8 candidates per lane");
    constexpr int kMChunk = kMJ * kBlock;
    constexpr int kNSig = 64 / kMJ < kMaxMSig ? 64 / kMJ : kMaxMSig;  // signatures the 64-bit match word holds
    constexpr uint64_t kSigStride = sig_stride(kMJ);
    __shared__ uint32_t wcnt[kNSig][kMJ][kWaves];   // hits per (signature, j, wave); then exclusive prefixes
    __shared__ uint64_t wmask[kNSig][kMJ][kWaves];  // their ballots
    __shared__ uint32_t qtot[kMaxMSig];
    __shared__ uint32_t wlive[kWaves];
    const uint32_t c = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t nq = ms.n_sigs;
    const uint32_t base = c * (uint32_t)kMChunk;
    const uint32_t len = ms.src_len - base < (uint32_t)kMChunk ? ms.src_len - base : (uint32_t)kMChunk;
    const uint32_t* __restrict__ src = st.order + ms.src_off + base;
    // hits are 4-B slot ids: an mscan search is constant-score and never cut,
    // so its list needs neither score keys nor source positions.
    // Every load below is unconditional — the chunk's tail lanes read a
    // clamped position / slot and are masked afterwards — so the compiler
    // issues each round's loads back to back before one wait: the slot ids,
    // then all columns of all kMJ candidates (one HBM round trip each) instead
    // of a branch and a wait around every load.  The field columns' base
    // pointers are scalar loads issued ahead of the slot ids.
    constexpr int NFA = NF > 0 ? NF : 1;  // array extent (NF = 0: signature sets that read no field)
    // The column base pointers come from a pointer table: marked global so
    // the loads are global_load (a flat load also counts in lgkmcnt, so every
    // later LDS / scalar wait would wait for the columns too).
    typedef const __attribute__((address_space(1))) uint8_t gu8;
    typedef const __attribute__((address_space(1))) int64_t gi64;
    gu8* fkp[NFA];
    gi64* fvp[NFA];
#pragma unroll
    for (int f = 0; f < NF; f++) {
        fkp[f] = (gu8*)st.fkind[ms.field[f]];
        fvp[f] = (gi64*)st.fval[ms.field[f]];
    }
    uint32_t s[kMJ], sl[kMJ];
#pragma unroll
    for (int j = 0; j < kMJ; j++) {
        const uint32_t i = (uint32_t)(j * kBlock + tid);
        sl[j] = src[i < len ? i : len - 1];
        s[j] = i < len ? sl[j] : kNoSlot;
    }
    // The signatures' filter fields into LDS, one thread per signature, while
    // the column loads are in flight: the signature loop then reads LDS
    // instead of a scalar load per field and a vector load per byte field
    // (term_only, req_mask) with a full memory wait in every iteration.
    __shared__ int64_t sq_req[kMaxMSig][NFA];
    __shared__ int32_t sq_tmin[kMaxMSig], sq_tmax[kMaxMSig];
    __shared__ uint32_t sq_flags[kMaxMSig];  // term_only | req_mask << 8
    if ((uint32_t)tid < nq) {
        const DMSig g = sigs[tid];
#pragma unroll
        for (int f = 0; f < NF; f++) sq_req[tid][f] = g.req[f];
        sq_tmin[tid] = g.tmin;
        sq_tmax[tid] = g.tmax;
        sq_flags[tid] = (uint32_t)g.term_only | ((uint32_t)g.req_mask << 8);
    }
    uint8_t al[kMJ];
    int32_t mn[kMJ], mx[kMJ];
    uint8_t kk[NFA][kMJ];
    int64_t vv[NFA][kMJ];
#pragma unroll
    for (int j = 0; j < kMJ; j++) {
        al[j] = st.alive[sl[j]];
        mn[j] = st.minc[sl[j]];
        mx[j] = st.maxc[sl[j]];
#pragma unroll
        for (int f = 0; f < NF; f++) {
            kk[f][j] = fkp[f][sl[j]];
            vv[f][j] = fvp[f][sl[j]];
        }
    }
    bool a[kMJ];
#pragma unroll
    for (int j = 0; j < kMJ; j++) {
        const bool v = s[j] != kNoSlot;
        a[j] = v && al[j] != 0;
#pragma unroll
        for (int f = 0; f < NF; f++)
            if (!v) kk[f][j] = (uint8_t)KIND_ABSENT;
    }
    uint32_t live = 0;
#pragma unroll
    for (int j = 0; j < kMJ; j++) live += a[j];
    for (int o = 32; o > 0; o >>= 1) live += __shfl_xor(live, o);
    if (lane == 0) wlive[wave] = live;
    // a candidate's keyword value per field, or a value no term id takes
    int64_t kw[NFA][kMJ];
#pragma unroll
    for (int f = 0; f < NF; f++)
#pragma unroll
        for (int j = 0; j < kMJ; j++) kw[f][j] = kk[f][j] == KIND_KEYWORD ? vv[f][j] : INT64_MIN;
    __syncthreads();  // the signature fields are in LDS
    // phase 1: every signature on the lane's candidates -> bit q * kMJ + j
    uint64_t bits = 0;
    if constexpr (!GEN) {
        // pool signatures only: equality on the required keyword fields.
        // Unrolled over the signature capacity, so every signature's LDS
        // fields are read up front and the bit positions are constants.
#pragma unroll
        for (int q = 0; q < kNSig; q++) {
            if ((uint32_t)q >= nq) continue;
            const uint32_t flags = sq_flags[q];
            const int32_t tmin = sq_tmin[q], tmax = sq_tmax[q];
            bool m[kMJ];
#pragma unroll
            for (int j = 0; j < kMJ; j++) m[j] = a[j] & (mn[j] >= tmin) & (mx[j] <= tmax);
#pragma unroll
            for (int f = 0; f < NF; f++) {
                const int64_t want = sq_req[q][f];
                const bool need = (flags >> (8 + f)) & 1u;
#pragma unroll
                for (int j = 0; j < kMJ; j++) m[j] = m[j] & (!need | (kw[f][j] == want));
            }
#pragma unroll
            for (int j = 0; j < kMJ; j++) bits |= (uint64_t)m[j] << (q * kMJ + j);
        }
    }
    for (uint32_t q = 0; GEN && q < nq; q++) {
        const uint32_t flags = sq_flags[q];
        const int32_t tmin = sq_tmin[q], tmax = sq_tmax[q];
        bool m[kMJ];
#pragma unroll
        for (int j = 0; j < kMJ; j++) m[j] = a[j] && mn[j] >= tmin && mx[j] <= tmax;
        if (!GEN || (flags & 0xffu)) {
            // a pool signature: equality on the required keyword fields
#pragma unroll
            for (int f = 0; f < NF; f++) {
                if (!((flags >> (8 + f)) & 1u)) continue;
                const int64_t want = sq_req[q][f];
#pragma unroll
                for (int j = 0; j < kMJ; j++) m[j] = m[j] && kw[f][j] == want;
            }
        } else if constexpr (GEN) {
            const DMSig& g = sigs[q];
            double msc[kMJ], ssc[kMJ];
            bool anys[kMJ];
#pragma unroll
            for (int j = 0; j < kMJ; j++) {
                msc[j] = 0.0;
                ssc[j] = 0.0;
                anys[j] = false;
            }
            bool has_must = false, has_should = false;
            if (g.qkind == QK_MATCHNONE) {
#pragma unroll
                for (int j = 0; j < kMJ; j++) m[j] = false;
            } else if (g.qkind != QK_MATCHALL) {
                for (int ci = 0; ci < g.n_clauses; ci++) {
                    const DClause k = mcl[g.clause_off + ci];  // field = index into ms.field
                    has_must |= k.occur == OCC_MUST;
                    has_should |= k.occur == OCC_SHOULD;
#pragma unroll
                    for (int j = 0; j < kMJ; j++) {
                        uint8_t kind = KIND_ABSENT;
                        int64_t val = 0;
#pragma unroll
                        for (int f = 0; f < NF; f++)
                            if (k.field == f) { kind = kk[f][j]; val = vv[f][j]; }
                        bool h = false;
                        double sc = k.score;
                        if (k.op == OP_TERM) h = kind == KIND_KEYWORD && val == (int64_t)k.term;
                        else if (k.op == OP_RANGE) h = kind == KIND_NUMERIC && val >= k.lo && val <= k.hi;
                        else if (k.op == OP_TERMSET) h = kind == KIND_KEYWORD && termset_hit(st, k.term, val, &sc);
                        else if (k.op != OP_FALSE)
                            h = (kind == KIND_KEYWORD && val == (int64_t)k.term) || (kind == KIND_NUMERIC && val == k.lo);
                        if (k.occur == OCC_MUST) { if (h) msc[j] += sc; else m[j] = false; }
                        else if (k.occur == OCC_SHOULD) { if (h) { ssc[j] += sc; anys[j] = true; } }
                        else if (h) m[j] = false;
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < kMJ; j++)  // a query of SHOULD clauses only: one of them must hit
                if (g.qkind != QK_MATCHALL && !has_must && has_should) m[j] = m[j] && anys[j];
            (void)msc;
            (void)ssc;
        }
#pragma unroll
        for (int j = 0; j < kMJ; j++) bits |= (uint64_t)m[j] << (q * kMJ + j);
    }
    // per (signature, j, wave): the ballot and its count
#pragma unroll
    for (int q = 0; q < kNSig; q++) {
        if ((uint32_t)q >= nq) continue;
#pragma unroll
        for (int j = 0; j < kMJ; j++) {
            const uint64_t mask = __ballot((int)((bits >> (q * kMJ + j)) & 1ull));
            if (lane == 0) {
                wmask[q][j][wave] = mask;
                wcnt[q][j][wave] = (uint32_t)__popcll(mask);
            }
        }
    }
    __syncthreads();
    // exclusive prefix of every signature's counts in (j, wave) order — the
    // candidate order j * 256 + tid — one thread per signature
    if ((uint32_t)tid < nq) {
        uint32_t run = 0;
        for (int j = 0; j < kMJ; j++)
            for (int w = 0; w < kWaves; w++) {
                const uint32_t v = wcnt[tid][j][w];
                wcnt[tid][j][w] = run;
                run += v;
            }
        qtot[tid] = run;
    }
    __syncthreads();
    // phase 2: ordered compaction into the (signature, chunk) cells.  A
    // candidate matching one signature (every candidate of a pool batch)
    // stores once; a wave holding a candidate that matches several
    // signatures takes the per-signature loop.
    const uint64_t cell0 = (uint64_t)c * kMChunk, cstride = (uint64_t)ms.n_chunks * kMChunk;
    bool multi = false;
#pragma unroll
    for (int j = 0; j < kMJ; j++) multi |= __popcll((bits >> j) & kSigStride) > 1;
    if (!__any(multi)) {
#pragma unroll
        for (int j = 0; j < kMJ; j++) {
            const uint64_t t = (bits >> j) & kSigStride;
            if (!t) continue;
            const uint32_t q = (uint32_t)__builtin_ctzll(t) / kMJ;
            const uint32_t pos = wcnt[q][j][wave] + lanes_below(wmask[q][j][wave]);
            out[q * cstride + cell0 + pos] = s[j];
        }
    } else {
        for (uint32_t q = 0; q < nq; q++) {
#pragma unroll
            for (int j = 0; j < kMJ; j++) {
                if (!((bits >> (q * kMJ + j)) & 1ull)) continue;
                const uint32_t pos = wcnt[q][j][wave] + lanes_below(wmask[q][j][wave]);
                out[q * cstride + cell0 + pos] = s[j];
            }
        }
    }
    if ((uint32_t)tid < nq) {
        uint32_t lv = 0;
        for (int w = 0; w < kWaves; w++) lv += wlive[w];
        // the chunk's columns are read once for all signatures: its
        // scanned/live counts are accounted to signature 0 only
        const uint32_t n = qtot[tid];
        res[(uint64_t)tid * ms.n_chunks + c] = DGroupResult{n, 1u, tid == 0 ? len : 0u, n, tid == 0 ? lv : 0u, 0u};
    }
}

// ---- hashed multi-signature scan ----------------------------------------------------
// mscan_kernel holds one match bit per (signature, candidate) and a ballot per
// signature: its cost grows with the signature count, and past 16 signatures
// (C4: 64 mode x region pools on one GPU) the batch fell back to scan_kernel
// over region posting lists shared by 8 modes (7.5x the column bytes).  When
// the signatures are term-only pool signatures requiring the same fields with
// distinct values, a candidate matches at most one: its required values find
// that signature through the LDS hash table, so the per-candidate work is one
// probe whatever the signature count.  The scan order is then stably
// partitioned by signature in three launches:
//   mscan_hash_kernel   per chunk: lookup, rank within (signature, chunk), the
//                       chunk's hits signature-major into scratch, counts row;
//   mscan_base_kernel   per signature: exclusive prefix over the chunks;
//   mscan_place_kernel  per chunk: its hits to their signature's list.
// Counts/bases are row-major [chunk][signature + 1] (column n_sigs: live
// candidates, for the accounting).  Every list is in scan order — the hit
// order of a constant-score search — exactly as mscan_kernel + stitch emit it.
// kMJ consecutive candidates of one lane, from a column at slot `gs`
// (aligned to kMJ elements): 16-B loads where they fit, one smaller load else.
template <int N, typename T>
__device__ __forceinline__ void load_run(T (&dst)[N], const T* p) {
    constexpr int B = N * (int)sizeof(T);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    typedef const __attribute__((address_space(1))) u32x4 g16;
    typedef const __attribute__((address_space(1))) u32x2 g8;
    typedef const __attribute__((address_space(1))) uint32_t g4;
    typedef const __attribute__((address_space(1))) uint16_t g2;
    if constexpr (B >= 16) {
#pragma unroll
        for (int k = 0; k < B / 16; k++) {
            const u32x4 v = ((g16*)p)[k];
            __builtin_memcpy(reinterpret_cast<char*>(dst) + 16 * k, &v, 16);
        }
    } else if constexpr (B == 8) {
        const u32x2 v = *(g8*)p;
        __builtin_memcpy(dst, &v, 8);
    } else if constexpr (B == 4) {
        const uint32_t v = *(g4*)p;
        __builtin_memcpy(dst, &v, 4);
    } else {
        static_assert(B == 2, "run of 2-64 bytes");
        const uint16_t v = *(g2*)p;
        __builtin_memcpy(dst, &v, 2);
    }
}

// CONTIG (ms.contig): the scan order is the slot order (tickets added in
// created-at order: order[p] == p), so a chunk is a slot range aligned to the
// chunk length and every lane loads its kMJ consecutive candidates' columns
// with 4-16-B vector loads (one instruction per column per lane instead of
// kMJ gathers, and no slot ids read); the signatures found are handed through
// LDS to the strided layout (candidate j * 256 + tid) the ranking uses.
// LDS is sized at launch: the lookup (cuckoo table or key grid, tab_bytes),
// the (j, wave, signature) counts, the chunk's signature offsets, its staged
// hits, and CONTIG's hand-over — 12 KB for C4's 64 signatures, so occupancy
// stays high.
template <int kMJ, bool CONTIG>
struct MHashLds {
    uint32_t tab_bytes, nq;
    __host__ __device__ constexpr uint32_t table_off() const { return 0; }
    __host__ __device__ constexpr uint32_t cnt_off() const { return (tab_bytes + 15u) & ~15u; }
    __host__ __device__ constexpr uint32_t loff_off() const { return cnt_off() + ((nq * kMJ * kWaves * 2u + 15u) & ~15u); }
    __host__ __device__ constexpr uint32_t stage_off() const { return loff_off() + ((nq * 4u + 15u) & ~15u); }
    __host__ __device__ constexpr uint32_t qs_off() const { return stage_off() + kMJ * kBlock * 4u; }
    __host__ __device__ constexpr uint32_t bytes() const { return qs_off() + (CONTIG ? kMJ * kBlock * 2u : 0u); }
};
// the lookup's LDS bytes: the key grid (u16 per cell) + the signatures' count
// ranges, or the cuckoo table
__host__ __device__ inline uint32_t mhash_tab_bytes(const DMScan& ms) {
    return ms.dsize ? ((ms.dsize * 2u + 15u) & ~15u) + ((ms.n_sigs * 8u + 15u) & ~15u) : (ms.hmask + 1) * 32u;
}

// COUNT: only the per-(signature, chunk) counts are written, no ranking into
// scratch — the proven-list pass (Core::mhash_count_mode_), whose lists are
// never placed.
//
// The lookup.  A candidate's required keyword values select at most one
// signature.  When the signatures' values span small ranges per field (every
// pool value a dictionary id: C3 / C4's modes and regions), the key grid
// (ms.dsize cells of u16, indexed by the values' offsets from the ranges'
// lows) gives it with one 2-B LDS read — exact, no key compare.  Otherwise
// two-choice cuckoo hashing: two 32-B entries, whose random 16-B LDS reads
// are bank-conflicted (rocprofv3 on C4's 64-signature table:
// SQ_LDS_BANK_CONFLICT ~7 cycles per LDS instruction, the kernel LDS-bound
// at ~36 us warm or cold, profiles/r05c_*).
template <int NF, int kMJ, bool CONTIG, bool COUNT>
__global__ __launch_bounds__(kBlock) void mscan_hash_kernel(DStore st, DMScan ms, const DMHashEntry* __restrict__ htab,
                                                            uint32_t* __restrict__ scratch,
                                                            uint32_t* __restrict__ counts, uint32_t c0) {
    static_assert(NF >= 1 && NF <= 4, "1-4 required fields");
    static_assert(!CONTIG || kMJ == 2 || kMJ == 4 || kMJ == 8, "runs of 2, 4 or 8 candidates");
    constexpr int kMChunk = kMJ * kBlock;
    constexpr uint32_t kNone = kMHashEmpty;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ uint32_t wsum[kWaves], wlive[kWaves];
    const uint32_t nq = ms.n_sigs, hmask = ms.hmask;
    const bool grid = ms.dsize != 0;
    const MHashLds<kMJ, CONTIG> L{mhash_tab_bytes(ms), nq};
    DMHashEntry* tab = reinterpret_cast<DMHashEntry*>(lds + L.table_off());
    uint16_t* dgrid = reinterpret_cast<uint16_t*>(lds + L.table_off());
    int32_t* dlim = reinterpret_cast<int32_t*>(lds + L.table_off() + ((ms.dsize * 2u + 15u) & ~15u));
    uint16_t* cnt = reinterpret_cast<uint16_t*>(lds + L.cnt_off());  // [j][wave][q]: count, then its rank base
    uint32_t* loff = reinterpret_cast<uint32_t*>(lds + L.loff_off());
    uint32_t* stage = reinterpret_cast<uint32_t*>(lds + L.stage_off());  // the chunk's hits, signature-major
    uint16_t* qs = reinterpret_cast<uint16_t*>(lds + L.qs_off());
    const uint32_t c = blockIdx.x + c0;  // c0: a row-sharded rank's first chunk
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef NKM_MH_DEBUG  // tools/mhash_bench.hip: phases switched off one by one (ms.pad bits)
    const uint32_t dbg = ms.pad;
#else
    constexpr uint32_t dbg = 0;
#endif
    typedef const __attribute__((address_space(1))) uint8_t gu8;
    typedef const __attribute__((address_space(1))) int64_t gi64;
    gu8* fkp[NF];
    gi64* fvp[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) {
        fkp[f] = (gu8*)st.fkind[ms.field[f]];
        fvp[f] = (gi64*)st.fval[ms.field[f]];
    }
    // CONTIG: the chunk's slots [cs0, cs0 + kMChunk), the scan's [vlo, vhi)
    const uint32_t cs0 = (ms.src_off & ~(uint32_t)(kMChunk - 1)) + c * (uint32_t)kMChunk;
    const uint32_t vlo = ms.src_off, vhi = ms.src_off + ms.src_len;
    uint32_t s[kMJ], sl[kMJ];
    if constexpr (!CONTIG) {
        // unconditional loads, tail lanes clamped (as in mscan_kernel)
        const uint32_t base = c * (uint32_t)kMChunk;
        const uint32_t len = ms.src_len - base < (uint32_t)kMChunk ? ms.src_len - base : (uint32_t)kMChunk;
        const uint32_t* __restrict__ src = st.order + ms.src_off + base;
#pragma unroll
        for (int j = 0; j < kMJ; j++) {
            const uint32_t i = (uint32_t)(j * kBlock + tid);
            sl[j] = src[i < len ? i : len - 1];
            s[j] = i < len ? sl[j] : kNoSlot;
        }
    }
    // the lookup and zeroed counts into LDS while the column loads are in flight
    if (!(dbg & 4)) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* __restrict__ g4 = reinterpret_cast<const u32x4*>(htab);  // the grid follows the cuckoo table
        u32x4* t4 = reinterpret_cast<u32x4*>(tab);
        const uint32_t g0 = grid ? 2 * (hmask + 1) : 0u, nv = L.tab_bytes / 16u;
        for (uint32_t t = (uint32_t)tid; t < nv; t += kBlock) t4[t] = g4[g0 + t];
        uint32_t* c4 = reinterpret_cast<uint32_t*>(cnt);
        for (uint32_t t = (uint32_t)tid; t < (nq * kMJ * kWaves + 1) / 2; t += kBlock) c4[t] = 0u;
    }
    uint8_t al[kMJ];
    int32_t mn[kMJ], mx[kMJ];
    uint8_t kk[NF][kMJ];
    int64_t vv[NF][kMJ];
    bool a[kMJ];
    if constexpr (CONTIG) {
        // wave w takes the chunk's candidates [w * 64 kMJ, (w + 1) * 64 kMJ) in
        // pairs: lane l's candidates j = 2p, 2p + 1 are wb + 128 p + 2 l + {0, 1},
        // so each column load instruction of the wave reads one contiguous
        // span (an int64 pair per lane: 1 KB; an int32 pair: 512 B) — the
        // fully coalesced shape, where a lane-contiguous run of kMJ values
        // spread every instruction over kMJ / 2 times the cache lines
        const uint32_t wb = cs0 + (uint32_t)wave * 64u * kMJ;
        if (wb >= vlo && wb + 64u * kMJ <= vhi) {
#pragma unroll
            for (int p = 0; p < kMJ / 2; p++) {
                const uint32_t x = wb + 128u * p + 2u * (uint32_t)lane;
                uint8_t a2[2], k2[NF][2];
                int32_t n2[2], m2[2];
                int64_t v2[NF][2];
                load_run(a2, st.alive + x);
                load_run(n2, st.minc + x);
                load_run(m2, st.maxc + x);
#pragma unroll
                for (int f = 0; f < NF; f++) {
                    load_run(k2[f], (const uint8_t*)(fkp[f] + x));
                    load_run(v2[f], (const int64_t*)(fvp[f] + x));
                }
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    al[2 * p + e] = a2[e];
                    mn[2 * p + e] = n2[e];
                    mx[2 * p + e] = m2[e];
#pragma unroll
                    for (int f = 0; f < NF; f++) {
                        kk[f][2 * p + e] = k2[f][e];
                        vv[f][2 * p + e] = v2[f][e];
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < kMJ; j++) a[j] = al[j] != 0;
        } else {  // the scan's first / last chunk: per candidate, in range only
#pragma unroll
            for (int j = 0; j < kMJ; j++) {
                const uint32_t x = wb + 128u * (uint32_t)(j / 2) + 2u * (uint32_t)lane + (uint32_t)(j & 1);
                a[j] = x >= vlo && x < vhi;
                al[j] = 0;
                mn[j] = mx[j] = 0;
#pragma unroll
                for (int f = 0; f < NF; f++) {
                    kk[f][j] = (uint8_t)KIND_ABSENT;
                    vv[f][j] = 0;
                }
                if (!a[j]) continue;
                al[j] = st.alive[x];
                mn[j] = st.minc[x];
                mx[j] = st.maxc[x];
#pragma unroll
                for (int f = 0; f < NF; f++) {
                    kk[f][j] = fkp[f][x];
                    vv[f][j] = fvp[f][x];
                }
                a[j] = al[j] != 0;
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < kMJ; j++) {
            al[j] = st.alive[sl[j]];
            mn[j] = st.minc[sl[j]];
            mx[j] = st.maxc[sl[j]];
#pragma unroll
            for (int f = 0; f < NF; f++) {
                kk[f][j] = fkp[f][sl[j]];
                vv[f][j] = fvp[f][sl[j]];
            }
        }
#pragma unroll
        for (int j = 0; j < kMJ; j++) a[j] = s[j] != kNoSlot && al[j] != 0;
    }
    uint32_t live = 0;
#pragma unroll
    for (int j = 0; j < kMJ; j++) {
        live += a[j];
#pragma unroll
        for (int f = 0; f < NF; f++) a[j] = a[j] && kk[f][j] == KIND_KEYWORD;  // every field is required
    }
    for (int o = 32; o > 0; o >>= 1) live += __shfl_xor(live, o);
    if (lane == 0) wlive[wave] = live;
    __syncthreads();  // lookup and zeroed counts are in LDS
    // each candidate's signature (at most one), then the signature's
    // count-range musts.  A keyword value is a dictionary id (< 2^32), so the
    // 32-bit keys compare exactly.
    uint32_t q[kMJ];
    if (grid) {
#pragma unroll
        for (int j = 0; j < kMJ; j++) {
            uint32_t idx = 0;
            bool in = a[j];
#pragma unroll
            for (int f = 0; f < NF; f++) {
                const uint32_t d = (uint32_t)vv[f][j] - ms.dlo[f];
                in = in && d < ms.drng[f];
                idx = idx * ms.drng[f] + d;
            }
            const uint32_t qq = in ? (uint32_t)dgrid[idx] : 0xFFFFu;
            const bool hit = qq != 0xFFFFu;
            const int32_t tmin = hit ? dlim[2 * qq] : 0, tmax = hit ? dlim[2 * qq + 1] : 0;
            q[j] = hit && mn[j] >= tmin && mx[j] <= tmax ? qq : kNone;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kMJ; j++) {
            uint32_t h1 = ms.hseed[0], h2 = ms.hseed[1];
#pragma unroll
            for (int f = 0; f < NF; f++) {
                h1 = msig_mix(h1, (uint32_t)vv[f][j]);
                h2 = msig_mix(h2, (uint32_t)vv[f][j]);
            }
            const DMHashEntry& e1 = tab[msig_fin(h1) & hmask];
            const DMHashEntry& e2 = tab[msig_fin(h2) & hmask];
            bool m1 = e1.q != kNone, m2 = e2.q != kNone;
#pragma unroll
            for (int f = 0; f < NF; f++) {
                m1 = m1 && e1.key[f] == (uint32_t)vv[f][j];
                m2 = m2 && e2.key[f] == (uint32_t)vv[f][j];
            }
            const uint32_t qq = m1 ? e1.q : e2.q;
            const int32_t tmin = m1 ? e1.tmin : e2.tmin, tmax = m1 ? e1.tmax : e2.tmax;
            q[j] = a[j] && (m1 || m2) && mn[j] >= tmin && mx[j] <= tmax ? qq : kNone;
        }
    }
#pragma unroll
    for (int j = 0; j < kMJ; j++)
        if (dbg & 1) q[j] = a[j] ? (uint32_t)(vv[0][j] ^ vv[NF - 1][j]) & (nq - 1) : kNone;  // no lookup
    if constexpr (COUNT) {
        // counts only: the order of the hits does not matter, so no exchange
        // and no ranking — one LDS increment per hit (the zeroed counts'
        // first nq words)
        uint32_t* cq = reinterpret_cast<uint32_t*>(cnt);
#pragma unroll
        for (int j = 0; j < kMJ; j++)
            if (q[j] != kNone) atomicAdd(&cq[q[j]], 1u);
        __syncthreads();
        if ((uint32_t)tid < nq) counts[mhash_cidx(ms, (uint32_t)tid, c)] = cq[tid];
        if (tid == 0) {
            uint32_t lv = 0;
            for (int w = 0; w < kWaves; w++) lv += wlive[w];
            counts[mhash_cidx(ms, nq, c)] = lv;
        }
        return;
    }
    if constexpr (CONTIG) {
        // (wave, pair, lane, e) -> the strided layout j * 256 + tid (candidate
        // order), through LDS
#pragma unroll
        for (int j = 0; j < kMJ; j++)
            qs[(uint32_t)wave * 64u * kMJ + 128u * (uint32_t)(j / 2) + 2u * (uint32_t)lane + (uint32_t)(j & 1)] =
                (uint16_t)q[j];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kMJ; j++) {
            const uint32_t i = (uint32_t)(j * kBlock + tid);
            q[j] = qs[i];
            s[j] = cs0 + i;
        }
    }
    if (dbg & 2) {  // no ranking, prefix or scatter: a checksum of the signatures found
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < kMJ; j++) x += q[j];
        counts[(uint64_t)c * kBlock + tid] = x;
        return;
    }
    // rank within (signature, j, wave): the lanes holding the same signature
    // are found with one ballot per signature-index bit
    const uint32_t nbits = nq > 1 ? 32u - (uint32_t)__clz(nq - 1) : 0u;
    uint32_t rk[kMJ];
#pragma unroll
    for (int j = 0; j < kMJ; j++) {
        const bool m = q[j] != kNone;
        uint64_t peer = __ballot((int)m);
        for (uint32_t b = 0; b < nbits; b++) {
            const bool bit = (q[j] >> b) & 1u;
            const uint64_t bb = __ballot((int)(m && bit));
            peer &= bit ? bb : ~bb;
        }
        rk[j] = lanes_below(peer);
        if (m && rk[j] == 0) cnt[(j * kWaves + wave) * nq + q[j]] = (uint16_t)__popcll(peer);
    }
    __syncthreads();
    // per signature: rank bases in candidate order (j, wave) — thread q reads
    // column q of the [j][wave][q] counts (consecutive threads, consecutive
    // halfwords); the chunk's signature-major offsets by a block scan of the totals
    uint32_t tot = 0;
    if ((uint32_t)tid < nq) {
        uint32_t run = 0;
#pragma unroll
        for (int k = 0; k < kMJ * kWaves; k++) {
            uint16_t* cq = cnt + (uint32_t)k * nq + (uint32_t)tid;
            const uint32_t v = *cq;
            *cq = (uint16_t)run;
            run += v;
        }
        tot = run;
        counts[mhash_cidx(ms, (uint32_t)tid, c)] = tot;  // column-major: mscan_base_kernel reads columns
    }
    if (tid == 0) {
        uint32_t lv = 0;
        for (int w = 0; w < kWaves; w++) lv += wlive[w];
        counts[mhash_cidx(ms, nq, c)] = lv;
    }
    uint32_t incl = tot;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o);
        if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t ex = incl - tot, total = 0;
    for (int w = 0; w < kWaves; w++) {
        if (w < wave) ex += wsum[w];
        total += wsum[w];
    }
    if ((uint32_t)tid < nq) loff[tid] = ex;
    __syncthreads();
    // ranked into LDS, then out in 16-B stores: with many signatures a
    // wave's hits fall in as many signature segments, and direct 4-B stores
    // would cost one partial-line write each
#pragma unroll
    for (int j = 0; j < kMJ; j++)
        if (q[j] != kNone) stage[loff[q[j]] + cnt[(j * kWaves + wave) * nq + q[j]] + rk[j]] = s[j];
    __syncthreads();
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4* __restrict__ cs4 = reinterpret_cast<u32x4*>(scratch + (uint64_t)c * kMChunk);
    const u32x4* st4 = reinterpret_cast<const u32x4*>(stage);
    for (uint32_t v = (uint32_t)tid; 4 * v < total; v += kBlock) cs4[v] = st4[v];
}

// Per column of the counts (a signature, or n_sigs: live candidates), stored
// column-major [column][chunk]: the exclusive prefix over the chunks into
// bases[column][chunk] (entry n_chunks: the total) and the signature's result
// record.  Each thread loads its run of up to 16 counts in one round trip.
__global__ __launch_bounds__(kBlock) void mscan_base_kernel(DMScan ms, const uint32_t* __restrict__ counts,
                                                            uint32_t* __restrict__ bases,
                                                            DGroupResult* __restrict__ res) {
    __shared__ uint32_t wsum[kWaves];
    const uint32_t q = blockIdx.x, n = ms.n_chunks;
    // one block (the common case): the column is contiguous
    const uint32_t* __restrict__ col = counts + (uint64_t)q * n;
    const bool blocked = ms.n_blk > 1;
    uint32_t* __restrict__ bcol = bases + (uint64_t)q * (n + 1);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t per = (n + kBlock - 1) / kBlock;
    const uint32_t lo = min(n, per * (uint32_t)tid), hi = min(n, per * (uint32_t)(tid + 1));
    constexpr int kUnroll = 16;  // C4 4M: 4,096 chunks -> 16 per thread
    const bool unrolled = per <= (uint32_t)kUnroll;
    uint32_t v[kUnroll];
    uint32_t sum = 0;
    if (unrolled) {
#pragma unroll
        for (int k = 0; k < kUnroll; k++)
            v[k] = lo + k < hi ? (blocked ? counts[mhash_cidx(ms, q, lo + k)] : col[lo + k]) : 0u;
#pragma unroll
        for (int k = 0; k < kUnroll; k++) sum += v[k];
    } else {
        for (uint32_t i = lo; i < hi; i++) sum += blocked ? counts[mhash_cidx(ms, q, i)] : col[i];
    }
    uint32_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o);
        if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - sum, total = 0;
    for (int w = 0; w < kWaves; w++) {
        if (w < wave) run += wsum[w];
        total += wsum[w];
    }
    if (unrolled) {
#pragma unroll
        for (int k = 0; k < kUnroll; k++) {
            if (lo + k < hi) bcol[lo + k] = run;
            run += v[k];
        }
    } else {
        for (uint32_t i = lo; i < hi; i++) {
            const uint32_t x = blocked ? counts[mhash_cidx(ms, q, i)] : col[i];
            bcol[i] = run;
            run += x;
        }
    }
    if (tid != 0) return;
    bcol[n] = total;
    if (q == ms.n_sigs) {  // the chunk's columns are accounted to signature 0 (as mscan_kernel does)
        res[0].live = total;
        return;
    }
    res[q].count = total;
    res[q].complete = 1u;
    res[q].matched = total;
    res[q].scanned = q == 0 ? ms.src_len : 0u;
    res[q].pad = 0u;
    if (q != 0) res[q].live = 0u;
}

// Per chunk: its hits (signature-major in scratch) to out32[dst[q] + base + r].
// Every thread loads its up-to-8 hits (e = k * 256 + tid) in one round trip,
// finds each one's signature by a binary search of the chunk's signature
// offsets in LDS, and stores it (a signature's run stays contiguous).
__global__ __launch_bounds__(kBlock) void mscan_place_kernel(DMScan ms, const uint32_t* __restrict__ bases,
                                                             const uint32_t* __restrict__ scratch,
                                                             const uint64_t* __restrict__ dst,
                                                             uint32_t* __restrict__ out32) {
    __shared__ uint32_t loff[kMHashSigs];
    __shared__ uint64_t lpos[kMHashSigs];
    __shared__ uint32_t wsum[kWaves];
    const uint32_t c = blockIdx.x, nq = ms.n_sigs, n1 = ms.n_chunks + 1;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t n = 0, b = 0;
    if ((uint32_t)tid < nq) {
        const uint32_t* __restrict__ bq = bases + (uint64_t)tid * n1 + c;
        b = bq[0];
        n = bq[1] - b;
    }
    // the chunk's hits, loaded before their count is known (clamped to the chunk)
    constexpr int kMaxPer = 8;
    const uint32_t per = ms.chunk / kBlock;
    const uint32_t* __restrict__ cs = scratch + (uint64_t)c * ms.chunk;
    uint32_t v[kMaxPer];
#pragma unroll
    for (int k = 0; k < kMaxPer; k++) v[k] = (uint32_t)k < per ? cs[k * kBlock + tid] : 0u;
    uint32_t incl = n;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o);
        if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t ex = incl - n, total = 0;
    for (int w = 0; w < kWaves; w++) {
        if (w < wave) ex += wsum[w];
        total += wsum[w];
    }
    if ((uint32_t)tid < nq) {
        loff[tid] = ex;
        lpos[tid] = dst[tid] + b;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kMaxPer; k++) {
        const uint32_t e = (uint32_t)(k * kBlock + tid);
        if ((uint32_t)k >= per || e >= total) continue;
        // the last signature whose offset is <= e (empty ones share it and lose)
        uint32_t lo = 0, hi = nq;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (loff[mid] <= e) lo = mid;
            else hi = mid;
        }
        out32[lpos[lo] + (e - loff[lo])] = v[k];
    }
}

// Places every chunk's compacted hits at its search's output, at the chunk's
// rank from cell_scan_kernel; entries past the search's capacity are dropped
// (the host marks it incomplete).
// Exclusive prefix of the chunk counts of each chunked / mscan search (one
// workgroup per search, cell range [ranges[2b], ranges[2b+1])): the rank of
// every chunk's first hit in its search, for stitch_kernel.
__global__ __launch_bounds__(kBlock) void cell_scan_kernel(const uint32_t* __restrict__ ranges,
                                                           const DGroupResult* __restrict__ cres,
                                                           uint32_t* __restrict__ offs) {
    __shared__ uint32_t wsum[kWaves];
    const uint32_t b = ranges[2 * blockIdx.x], n = ranges[2 * blockIdx.x + 1] - b;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t per = (n + kBlock - 1) / kBlock;  // each thread: a contiguous run of cells
    const uint32_t lo = b + min(n, per * (uint32_t)tid), hi = b + min(n, per * (uint32_t)(tid + 1));
    uint32_t sum = 0;
    constexpr int kUnroll = 8;  // C3: 2048 cells per search -> 8 per thread, loaded in one round trip
    const bool unrolled = per <= (uint32_t)kUnroll;
    uint32_t v[kUnroll];
    if (unrolled) {
#pragma unroll
        for (int k = 0; k < kUnroll; k++) v[k] = lo + k < hi ? cres[lo + k].count : 0u;
#pragma unroll
        for (int k = 0; k < kUnroll; k++) sum += v[k];
    } else {
        for (uint32_t i = lo; i < hi; i++) sum += cres[i].count;
    }
    uint32_t incl = sum;  // inclusive scan of the threads' sums: within waves, then across them
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o);
        if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (int w = 0; w < wave; w++) run += wsum[w];
    if (unrolled) {
#pragma unroll
        for (int k = 0; k < kUnroll; k++) {
            if (lo + k < hi) offs[lo + k] = run;
            run += v[k];
        }
        return;
    }
    for (uint32_t i = lo; i < hi; i++) {
        offs[i] = run;
        run += cres[i].count;
    }
}

__global__ __launch_bounds__(kBlock) void stitch_kernel(const DChunkMap* __restrict__ map,
                                                        const DGroupResult* __restrict__ cres,
                                                        const uint32_t* __restrict__ offs,
                                                        const DHit* __restrict__ scratch, DHit* __restrict__ out,
                                                        uint32_t n_cells) {
    // one wave per cell (C3: 16k cells of ~64 slot ids — a workgroup each
    // spent more on dispatch than on the copy)
    const uint32_t c = blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (c >= n_cells) return;  // wave-uniform
    const DChunkMap mp = map[c];
    const int tid = threadIdx.x & 63;
    const uint32_t prefix = offs[c];
    const uint32_t n = cres[c].count;
    const uint64_t so = mp.so;
    if (mp.u32) {  // an mscan cell: 4-B slot ids, `so` and dst_off in slot words
        const uint32_t* __restrict__ s32 = reinterpret_cast<const uint32_t*>(scratch);
        uint32_t* __restrict__ o32 = reinterpret_cast<uint32_t*>(out);
        const uint32_t lim = mp.cap > prefix ? mp.cap - prefix : 0u;
        const uint32_t m = n < lim ? n : lim;
        for (uint32_t e = tid; e < m; e += 64) o32[mp.dst_off + prefix + e] = s32[so + e];
        return;
    }
    for (uint32_t e = tid; e < n; e += 64) {
        const uint32_t pos = prefix + e;
        if (pos >= mp.cap) break;
        DHit h = scratch[so + e];
        h.idx += mp.start;
        out[mp.dst_off + pos] = h;
    }
}

// Hit lists for the host as 4-B slot ids: the replay walks slots only, so the
// D2H of a batch's lists moves a quarter of the 16-B DHit bytes (C2's
// top-512 lists: 55 MB -> 14 MB per batch).  Entries [0, n) of the DHit
// output (unwritten capacity included: contiguous, one copy), and each whole
// search's last written entry (its pagination cursor: key and source position).
__global__ __launch_bounds__(kBlock) void pack_slots_kernel(const DHit* __restrict__ out, uint64_t n,
                                                            uint32_t* __restrict__ slots) {
    for (uint64_t e = blockIdx.x * (uint64_t)kBlock + threadIdx.x; e < n; e += (uint64_t)gridDim.x * kBlock)
        slots[e] = out[e].slot;
}

__global__ __launch_bounds__(kBlock) void last_hits_kernel(const DGroup* __restrict__ groups,
                                                           const DGroupResult* __restrict__ res, int n,
                                                           const DHit* __restrict__ out, DHit* __restrict__ last) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = res[i].count;
    last[i] = c ? out[groups[i].out_off + c - 1] : DHit{kNoSlot, 0u, 0};
}

// processCustom's candidate enumeration (combineIndexes, matchmaker_process.go:
// 578-612, and the checks :470-546 applied to each subset), one thread per work
// item (a run of kEnumSpan masks of one row, mm_device.h).  COUNT: the item's
// candidate and entry counts -> cnt[2 item], cnt[2 item + 1].  Otherwise the
// item's candidates at the bases the host scanned from those counts: entries
// as (slot, presence index) word pairs — the hits in ascending bit order, each
// with all its presences, then T's — and every group's end offset (+ e0).
// Sessions are exclusive on this path (no two live tickets share one), so the
// pairwise session test (:509-519) never rejects; the mutual validateMatch
// test is a mask test: every member's pm covers the other members.
// SLOTS (every ticket holds one presence, so every presence index is 0):
// entries as slot ids alone and each group's size as one byte (<= 63 entries)
// in place of its end offset — half the entry bytes and a quarter of the
// offsets' for the host copy.
template <bool COUNT, bool SLOTS = false>
__global__ __launch_bounds__(kBlock) void enum_kernel(const DEnumRow* __restrict__ rows,
                                                      const DEnumHit* __restrict__ hits,
                                                      const DEnumItem* __restrict__ items, uint32_t n_items,
                                                      uint32_t* __restrict__ cnt, const uint64_t* __restrict__ base,
                                                      uint32_t e0, uint32_t* __restrict__ ents,
                                                      uint32_t* __restrict__ off) {
    const uint32_t it = blockIdx.x * kBlock + threadIdx.x;
    if (it >= n_items) return;
    const DEnumItem item = items[it];
    const DEnumRow row = rows[item.row];
    const DEnumHit* __restrict__ h = hits + row.hit_off;
    const int c = row.cmax < row.L ? row.cmax : row.L;
    uint64_t m = unrank_mask(item.rank, row.L, c);
    uint32_t ng = 0, ne = 0;
    uint64_t gk = 0, ek = 0;
    if (!COUNT) {
        gk = base[2 * (size_t)it];
        ek = base[2 * (size_t)it + 1];
    }
    for (uint32_t s = 0; s < item.n; s++) {
        if (s) {  // the next mask with at most c bits
            m++;
            while (__popcll(m) > c) m += m & (~m + 1);
        }
        int entries = 0;  // :593-600
        bool over = false;
        for (uint64_t b = m; b; b &= b - 1) {
            entries += h[__builtin_ctzll(b)].count;
            if (entries > row.cmax) { over = true; break; }
        }
        if (over || entries < row.cmin) continue;
        const int hc = entries + row.tcount;  // :470-486
        if (hc > row.tmax || hc < row.tmin || hc % row.tcm != 0) continue;
        bool ok = true;
        for (uint64_t b = m; b && ok; b &= b - 1) {  // :487-498, :520-546
            const int el = __builtin_ctzll(b);
            const DEnumHit& e = h[el];
            ok = !(hc > e.maxc || hc < e.minc || hc % e.cm != 0 || (hc < e.maxc && e.wait)) && e.self_ok &&
                 ((e.pm | (1ull << el)) & m) == m;
        }
        if (!ok) continue;
        if (COUNT) {
            ng++;
            ne += (uint32_t)hc;
            continue;
        }
        if (SLOTS) {
            for (uint64_t b = m; b; b &= b - 1, ek++) ents[ek] = h[__builtin_ctzll(b)].slot;
            ents[ek++] = row.T;
            reinterpret_cast<uint8_t*>(off)[gk++] = (uint8_t)hc;
            continue;
        }
        for (uint64_t b = m; b; b &= b - 1) {
            const DEnumHit& e = h[__builtin_ctzll(b)];
            for (int k = 0; k < e.count; k++, ek++) {
                ents[2 * ek] = e.slot;
                ents[2 * ek + 1] = (uint32_t)k;
            }
        }
        for (int k = 0; k < row.tcount; k++, ek++) {
            ents[2 * ek] = row.T;
            ents[2 * ek + 1] = (uint32_t)k;
        }
        off[gk++] = e0 + (uint32_t)ek;
    }
    if (COUNT) {
        cnt[2 * (size_t)it] = ng;
        cnt[2 * (size_t)it + 1] = ne;
    }
}

// Sets the device alive flag of the listed slots (0: selected / removed; 1:
// restored, for the members of a group the post-pass re-check dropped).
__global__ void clear_alive_kernel(uint8_t* __restrict__ alive, const uint32_t* __restrict__ slots, uint32_t n,
                                   uint8_t value) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) alive[slots[i]] = value;
}

// validateMatch for explicit (from, to) pairs: does `to`'s document match
// `from`'s parsed query?  (matchmaker.go:1042-1068)
__global__ void pair_kernel(DStore st, const uint32_t* __restrict__ pairs, uint32_t n, uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t from = pairs[2 * i], to = pairs[2 * i + 1];
    const DQuery q = st.squery[from];
    double d;
    out[i] = (st.alive[to] && eval_parsed(st, q.kind, st.clauses + q.clause_off, q.n_clauses, to, &d)) ? 1 : 0;
}

// Pair matrices for RevPrecision combos (matchmaker_process.go:178-203): for
// the first 32 entries a, b of each search's list, bit b of pm[out_off + a]
// is "entry b's document matches entry a's parsed query" (one word per list
// entry, beside the entry).  rsmall_kernel writes its searches' own.
__global__ void pairmat_kernel(DStore st, const DGroup* __restrict__ groups, const DGroupResult* __restrict__ res,
                               int n_groups, const DHit* __restrict__ out, uint32_t* __restrict__ pm) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int g = t >> 5, a = t & 31;
    if (g >= n_groups || groups[g].path != 0) return;
    const uint32_t n = res[g].count < 32u ? res[g].count : 32u;
    if ((uint32_t)a >= n) return;
    uint32_t mask = 0;
    const uint64_t base = groups[g].out_off;
    const uint32_t from = out[base + a].slot;
    const DQuery q = st.squery[from];
    for (uint32_t b = 0; b < n; b++) {
        double d;
        if (eval_parsed(st, q.kind, st.clauses + q.clause_off, q.n_clauses, out[base + b].slot, &d)) mask |= 1u << b;
    }
    pm[base + a] = mask;
}

// ---- RevPrecision rows over short sources ---------------------------------------
// With RevPrecision every row is its own search (the reverse check depends on
// the row), and with bucketed queries (C5: buckets of 8) a row's source is a
// few entries: search_kernel would spend a 256-lane workgroup per row.  Here
// one wave takes one row (4 rows per workgroup): lane j evaluates source entry
// j (the predicate, its score key, and the reverse check Q_H(T)), the wave
// ranks its matches by (score key desc, source position asc) with shuffles —
// the hit order of search_kernel's top-K — and writes the whole list, its
// reverse flags and (pm != null) the pair matrix of its first 32 entries.
constexpr int kSmallSrc = 64;

__global__ __launch_bounds__(kBlock) void rsmall_kernel(DStore st, const DGroup* __restrict__ groups,
                                                        const uint32_t* __restrict__ rows, uint32_t n_rows,
                                                        DHit* __restrict__ out, uint8_t* __restrict__ out_rev,
                                                        uint32_t* __restrict__ pm, DGroupResult* __restrict__ res) {
    const int lane = threadIdx.x & 63;
    const uint32_t r = blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (r >= n_rows) return;  // wave-uniform
    const uint32_t gi = rows[r];
    const DGroup g = groups[gi];
    const uint32_t* src = (g.src_kind == 0 ? st.order : st.postings) + g.src_off;
    const uint32_t j = (uint32_t)lane;
    bool m = false, live = false;
    uint32_t s = kNoSlot;
    int64_t key = 0;
    uint8_t rv = 1;
    if (j < g.src_len) {
        s = src[j];
        live = st.alive[s] != 0;
        m = live && st.minc[s] >= g.tmin && st.maxc[s] <= g.tmax && (g.tparty == kNoParty || st.party[s] != g.tparty);
        double sp = 0.0;
        if (m) m = eval_parsed(st, g.qkind, st.clauses + g.clause_off, g.n_clauses, s, &sp);
        if (m) {
            key = dsortable((sp + 1.0) + 1.0);
            const DQuery q = st.squery[s];
            double d;
            rv = eval_parsed(st, q.kind, st.clauses + q.clause_off, q.n_clauses, g.rev_slot, &d) ? 1 : 0;
        }
    }
    const uint64_t mask = __ballot(m);
    // rank among the matches: higher keys first, then earlier source positions
    uint32_t rank = 0;
    for (uint64_t rest = mask; rest; rest &= rest - 1) {
        const int i = __builtin_ctzll(rest);
        const int64_t ki = __shfl(key, i);
        rank += (ki > key) || (ki == key && (uint32_t)i < j);
    }
    if (m) {
        out[g.out_off + rank] = DHit{s, j, key};
        if (out_rev) out_rev[g.out_off + rank] = rv;
    }
    const uint32_t cnt = (uint32_t)__popcll(mask);
    if (pm) {
        // entry `rank` (a < 32): bit b = entry b's document matches this entry's query
        uint32_t pmask = 0;
        const DQuery q = m ? st.squery[s] : DQuery{};
        for (uint64_t rest = mask; rest; rest &= rest - 1) {
            const int i = __builtin_ctzll(rest);
            const uint32_t si = (uint32_t)__shfl((int)s, i);
            const int64_t ki = __shfl(key, i);
            uint32_t ri = 0;  // entry i's rank
            for (uint64_t rr = mask; rr; rr &= rr - 1) {
                const int t = __builtin_ctzll(rr);
                const int64_t kt = __shfl(key, t);
                ri += (kt > ki) || (kt == ki && t < i);
            }
            if (m && rank < 32 && ri < 32) {
                double d;
                if (eval_parsed(st, q.kind, st.clauses + q.clause_off, q.n_clauses, si, &d)) pmask |= 1u << ri;
            }
        }
        if (m && rank < 32) pm[g.out_off + rank] = pmask;
    }
    const uint32_t nlive = (uint32_t)__popcll(__ballot(live));
    if (lane == 0) res[gi] = DGroupResult{cnt, 1u, g.src_len, cnt, nlive, 0u};
}

// ---- packed RevPrecision rows (rpack_kernel) -------------------------------------
// A RevPrecision batch whose every search is one row over a source of at most
// S entries (C5: buckets of 8 -> S = 8) packs 64 / S rows into each wave
// (rsmall_kernel's one row per wave left 56 of 64 lanes idle on C5): lane j
// of a row's S-lane segment evaluates source entry j — the predicate with the
// row's own query and count range, its score key, and the reverse check
// Q_H(T).  The segment's ballot bits rank the matches by (score key desc,
// source position asc), search_kernel's top-K order, in S wave-uniform shuffle
// steps; a second S steps give every entry its pair-matrix row (bit b: entry
// b's document matches this entry's query) and the row its reverse bits in
// entry order.  Outputs are fixed-stride per row (pack_layout: no offsets, no
// per-row result record, no 80-B descriptor — the row is its 12-B DSmallRow).
template <int S> struct PackT;
template <> struct PackT<8> { using pm = uint8_t; using rv = uint8_t; };
template <> struct PackT<16> { using pm = uint16_t; using rv = uint16_t; };
template <> struct PackT<32> { using pm = uint32_t; using rv = uint32_t; };
template <> struct PackT<64> { using pm = uint32_t; using rv = uint64_t; };

// Lane `base + i` of this lane's 8-lane segment (i a constant after
// unrolling): ds_swizzle in bitmask mode — lane = (lane & 0x18) | i within
// each 32-lane half — with no address operand (__shfl is a ds_bpermute).
__device__ __forceinline__ int seg8_bcast(int v, int i) {
    switch (i & 7) {
        case 0: return __builtin_amdgcn_ds_swizzle(v, 0x18 | (0 << 5));
        case 1: return __builtin_amdgcn_ds_swizzle(v, 0x18 | (1 << 5));
        case 2: return __builtin_amdgcn_ds_swizzle(v, 0x18 | (2 << 5));
        case 3: return __builtin_amdgcn_ds_swizzle(v, 0x18 | (3 << 5));
        case 4: return __builtin_amdgcn_ds_swizzle(v, 0x18 | (4 << 5));
        case 5: return __builtin_amdgcn_ds_swizzle(v, 0x18 | (5 << 5));
        case 6: return __builtin_amdgcn_ds_swizzle(v, 0x18 | (6 << 5));
        default: return __builtin_amdgcn_ds_swizzle(v, 0x18 | (7 << 5));
    }
}
__device__ __forceinline__ int64_t seg8_bcast64(int64_t v, int i) {
    const int lo = seg8_bcast((int)(uint32_t)v, i), hi = seg8_bcast((int)(uint32_t)((uint64_t)v >> 32), i);
    return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// OR of a 64-bit value over the lane's 8-lane segment (ds_swizzle xor 1, 2, 4)
__device__ __forceinline__ uint64_t seg8_or64(uint64_t v) {
    auto x = [](uint64_t w, int which) -> uint64_t {
        const int lo = (int)(uint32_t)w, hi = (int)(uint32_t)(w >> 32);
        int l2, h2;
        if (which == 1) { l2 = __builtin_amdgcn_ds_swizzle(lo, 0x1F | (1 << 10)); h2 = __builtin_amdgcn_ds_swizzle(hi, 0x1F | (1 << 10)); }
        else if (which == 2) { l2 = __builtin_amdgcn_ds_swizzle(lo, 0x1F | (2 << 10)); h2 = __builtin_amdgcn_ds_swizzle(hi, 0x1F | (2 << 10)); }
        else { l2 = __builtin_amdgcn_ds_swizzle(lo, 0x1F | (4 << 10)); h2 = __builtin_amdgcn_ds_swizzle(hi, 0x1F | (4 << 10)); }
        return ((uint64_t)(uint32_t)h2 << 32) | (uint32_t)l2;
    };
    v |= x(v, 1);
    v |= x(v, 2);
    v |= x(v, 4);
    return v;
}
// bit i of b (8 bits) -> byte i of the result, 0x00 or 0xFF
__device__ __forceinline__ uint64_t byte_mask8(uint32_t b) {
    uint64_t x = b & 0xFFu;
    x = (x | (x << 28)) & 0x0000000F0000000Full;
    x = (x | (x << 14)) & 0x0003000300030003ull;
    x = (x | (x << 7)) & 0x0101010101010101ull;
    return x * 0xFFull;
}
// OR of the 8 bytes of x
__device__ __forceinline__ uint32_t or_bytes(uint64_t x) {
    x |= x >> 32;
    x |= x >> 16;
    x |= x >> 8;
    return (uint32_t)(x & 0xFFu);
}

template <int S>
__global__ __launch_bounds__(kBlock, 8) void rpack_kernel(DStore st, const DSmallRow* __restrict__ rows, uint32_t n_rows,
                                                       uint8_t* __restrict__ obuf, PackLayout L) {
    using PmT = typename PackT<S>::pm;
    using RvT = typename PackT<S>::rv;
    constexpr int R = 64 / S;           // rows per wave
    constexpr int P = S < 32 ? S : 32;  // pair-matrix entries per row
    __shared__ uint32_t wlive[kWaves], wmatch[kWaves];
    __shared__ FieldTable ft;
    const bool batched = field_table_ok(st);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int seg = lane / S, j = lane % S, base = seg * S;
    const uint32_t r = (blockIdx.x * kWaves + wave) * R + seg;
    const bool have = r < n_rows;
    // Unconditional loads (a lane past the last row reads the last row's
    // record, then is masked), in dependent rounds: the row record; then its
    // source entry, its own query and count range together
    const DSmallRow d = rows[have ? r : n_rows - 1];
    const uint32_t len = d.src_len & ~kSrcOrder;
    const uint32_t* srcb = (d.src_len & kSrcOrder) ? st.order : st.postings;
    const uint32_t s_src = len ? srcb[d.src_off + ((uint32_t)j < len ? (uint32_t)j : len - 1)] : kNoSlot;
    const DQuery rq = st.squery[d.slot];
    const int32_t rmin = st.minc[d.slot], rmax = st.maxc[d.slot];
    // A square wave's entry j is row j's ticket: its alive flag, counts and
    // prefetch-field values load now, from the row records, in the round of
    // the row's query and source (checked against the source below)
    uint32_t row_j = 0;
    uint8_t al_j = 0, pk[2] = {0, 0};
    int32_t smin_j = 0, smax_j = 0;
    int64_t pv[2] = {0, 0};
    if constexpr (S == 8) {
        typedef const __attribute__((address_space(1))) uint8_t gu8;
        typedef const __attribute__((address_space(1))) int64_t gi64;
        row_j = (uint32_t)__shfl((int)d.slot, j * S);  // the slot of the row whose segment is j
        al_j = st.alive[row_j];
        smin_j = st.minc[row_j];
        smax_j = st.maxc[row_j];
        if (L.npf > 0) {
            pk[0] = ((gu8*)L.pf_kind[0])[row_j];
            pv[0] = ((gi64*)L.pf_val[0])[row_j];
        }
        if (L.npf > 1) {
            pk[1] = ((gu8*)L.pf_kind[1])[row_j];
            pv[1] = ((gi64*)L.pf_val[1])[row_j];
        }
    }
    // the column table in this round too (its copy into LDS waits for its
    // loads: issued first, it cost the kernel a round of its own)
    load_field_table(st, ft);
    __syncthreads();  // ft
    bool m = false, live = false, rv = false;
    uint32_t s = kNoSlot;
    int64_t key = 0;
    // A square wave (S = 8: C5's buckets): its 8 rows search one common
    // source of 8 entries that ARE the rows, in order.  Every check of the
    // wave — forward Q_row(doc), reverse Q_entry(doc_row), pair matrix
    // Q_entry(doc_other) — is then an entry of the 8 x 8 matrix
    // E[a][b] = Q_{member a}(doc of member b), and lane (a, b) computes exactly
    // E[a][b] as its forward evaluation: one ballot hands the matrix to every
    // lane, instead of up to 1 + 1 + 8 evaluations (and their dependent
    // clause and column gathers) per lane.
    bool square = false;
    if constexpr (S == 8) {
        const uint32_t off0 = __shfl(d.src_off, 0), len0 = __shfl(d.src_len, 0);
        const uint32_t s_sq = have && (uint32_t)j < len ? s_src : kNoSlot;
        square = __ballot(have && d.src_off == off0 && d.src_len == len0 && len == (uint32_t)S && s_sq == row_j) == ~0ull;
    }
    uint64_t Ebits = 0;
    if (square) {  // wave-uniform: entry j is row j (its loads above), then the row query's clauses
        s = s_src;
        const uint8_t al = al_j;
        const int32_t smin = smin_j, smax = smax_j;
        live = al != 0;
        double sp = 0.0;
        // every row of the wave with at most 2 clauses (C5's bucket term and
        // skill range): the 2-clause batch (half the registers: 8 waves per
        // SIMD instead of 5), its columns from the prefetched values
        const bool two = __ballot(rq.n_clauses > 2) == 0;
        const bool e = batched && two ? eval_batched_pf<2>(st, ft, rq.kind, st.clauses + rq.clause_off, rq.n_clauses, s,
                                                           &sp, L.npf, L.pf, pk, pv)
                                      : eval_parsed(st, rq.kind, st.clauses + rq.clause_off, rq.n_clauses, s, &sp);
        Ebits = __ballot(e);  // bit a * 8 + b: member a's query matches member b's document
        m = live && e && smin >= rmin && smax <= rmax;
        if (m) key = dsortable((sp + 1.0) + 1.0);
        rv = m && ((Ebits >> (j * S + seg)) & 1);
    } else if (have && (uint32_t)j < len) {
        s = s_src;
        const uint8_t al = st.alive[s];
        const int32_t smin = st.minc[s], smax = st.maxc[s];
        const DQuery h = st.squery[s];
        live = al != 0;
        if (live) {
            m = smin >= rmin && smax <= rmax;
            if (m) {
                double sp = 0.0;
                m = eval_parsed(st, rq.kind, st.clauses + rq.clause_off, rq.n_clauses, s, &sp);
                key = dsortable((sp + 1.0) + 1.0);
            }
            if (m) {
                double dd;
                rv = eval_parsed(st, h.kind, st.clauses + h.clause_off, h.n_clauses, d.slot, &dd);
            }
        }
    }
    const uint64_t ball = __ballot(m);
    const uint64_t mine = S == 64 ? ball : (ball >> base) & ((1ull << (S & 63)) - 1);
    uint32_t rank = 0;
    // the keys' low words all zero (C5's scores are small sums of boosts):
    // the int64 order is the high words' signed order, one 32-bit exchange
    // per entry instead of two (wave-uniform)
    // and, beyond that, the high words non-negative with their 3 low bits
    // zero: key and entry index fold into one 32-bit word whose unsigned
    // order is the ranking order (larger key first, then smaller index;
    // unmatched lanes 0), so the rank is a count of larger words
    const uint32_t khw = (uint32_t)((uint64_t)key >> 32);
    const bool k32c = S == 8 && __ballot(m && (((uint32_t)key != 0u) | ((khw & 0x80000007u) != 0u))) == 0;
    const bool k32 = S == 8 && !k32c && __ballot(m && (uint32_t)key != 0u) == 0;
    if (k32c) {
        const uint32_t cw = m ? ((khw | 0x80000000u) | (uint32_t)(7 - j)) : 0u;
#pragma unroll
        for (int i = 0; i < S; i++) rank += (uint32_t)((uint32_t)seg8_bcast((int)cw, i) > cw);
    } else if (k32) {
        const int32_t kh = (int32_t)((uint64_t)key >> 32);
#pragma unroll
        for (int i = 0; i < S; i++) {
            const int32_t ki = seg8_bcast(kh, i);
            rank += (uint32_t)((mine >> i) & 1) & (uint32_t)((ki > kh) | ((ki == kh) & (i < j)));
        }
    } else {
#pragma unroll
        for (int i = 0; i < S; i++) {
            const int64_t ki = S == 8 ? seg8_bcast64(key, i) : __shfl(key, base + i);
            rank += (uint32_t)(((mine >> i) & 1) && (ki > key || (ki == key && i < j)));
        }
    }
    PmT pmask = 0;
    RvT rbits = 0;
    if (S == 8 && square) {
        // byte i of `ranked`: entry i's rank as a bit (0 when it did not
        // match), from one OR over the segment; then, with E's bytes as
        // masks, the reverse bits (entry i's reverse check E[i][seg]) and this
        // entry's pair-matrix row (its query against entry i's document,
        // E[j][i]) are ORs of the selected bytes — no per-entry loop
        const uint64_t ranked = seg8_or64((uint64_t)(m ? (1u << rank) : 0u) << (8 * j));
        rbits = (RvT)or_bytes(ranked & (((Ebits >> seg) & 0x0101010101010101ull) * 0xFFull));
        if (m) pmask = (PmT)or_bytes(ranked & byte_mask8((uint32_t)(Ebits >> (8 * j))));
    } else if (square) {
#pragma unroll
        for (int i = 0; i < S; i++) {
            const uint32_t ri = (uint32_t)__shfl((int)rank, base + i);
            if (!((mine >> i) & 1)) continue;
            // entry i's reverse bit: rv of lane i = its match (mine bit i) and
            // E[i][seg] — from the ballot, no exchange
            if ((Ebits >> (i * S + seg)) & 1) rbits |= (RvT)((RvT)1 << ri);
            // entry j's query against entry i's document: E[j][i]
            if (m && rank < (uint32_t)P && ri < (uint32_t)P && ((Ebits >> (j * S + i)) & 1)) pmask |= (PmT)((PmT)1 << ri);
        }
    } else {
        const DQuery q = m ? st.squery[s] : DQuery{0u, 0, 0, 0};
        for (int i = 0; i < S; i++) {
            const uint32_t si = (uint32_t)__shfl((int)s, base + i);
            const uint32_t ri = (uint32_t)__shfl((int)rank, base + i);
            const int rvi = __shfl((int)rv, base + i);
            if (!((mine >> i) & 1)) continue;  // segment-uniform: the shuffles above ran on every lane
            if (rvi) rbits |= (RvT)((RvT)1 << ri);
            if (m && rank < (uint32_t)P && ri < (uint32_t)P) {
                double dd;
                if (eval_parsed(st, q.kind, st.clauses + q.clause_off, q.n_clauses, si, &dd)) pmask |= (PmT)((PmT)1 << ri);
            }
        }
    }
    uint8_t* __restrict__ o_pos = obuf + L.pos;
    PmT* __restrict__ o_pm = reinterpret_cast<PmT*>(obuf + L.pm);
    RvT* __restrict__ o_rev = reinterpret_cast<RvT*>(obuf + L.rev);
    if (m) o_pos[(uint64_t)r * S + rank] = (uint8_t)j;  // the entry's source position
    if (m && rank < (uint32_t)P) o_pm[(uint64_t)r * P + rank] = pmask;
    if (have && j == 0) {
        o_rev[r] = rbits;
        obuf[L.cnt + r] = (uint8_t)__popcll(mine);
    }
    const uint32_t wl = (uint32_t)__popcll(__ballot(live)), wm = (uint32_t)__popcll(ball);
    if (lane == 0) {
        wlive[wave] = wl;
        wmatch[wave] = wm;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0, u = 0;
        for (int w = 0; w < kWaves; w++) {
            t += wlive[w];
            u += wmatch[w];
        }
        uint32_t* o = reinterpret_cast<uint32_t*>(obuf + L.live) + 2 * (uint64_t)blockIdx.x;
        o[0] = t;
        o[1] = u;
    }
}

hipError_t launch_rpack(const DStore& st, const DSmallRow* d_rows, uint32_t n_rows, uint8_t* d_obuf, const PackLayout& L,
                        hipStream_t stream, hipEvent_t ev0, hipEvent_t ev1) {
    if (n_rows == 0) return hipSuccess;
    if (L.blocks != (n_rows + kPackRowsPerBlock(L.S) - 1) / kPackRowsPerBlock(L.S)) return hipErrorInvalidValue;
    const dim3 grid(L.blocks), block(kBlock);
    switch (L.S) {
        case 8: hipExtLaunchKernelGGL(rpack_kernel<8>, grid, block, 0, stream, ev0, ev1, 0, st, d_rows, n_rows, d_obuf, L); break;
        case 16: hipExtLaunchKernelGGL(rpack_kernel<16>, grid, block, 0, stream, ev0, ev1, 0, st, d_rows, n_rows, d_obuf, L); break;
        case 32: hipExtLaunchKernelGGL(rpack_kernel<32>, grid, block, 0, stream, ev0, ev1, 0, st, d_rows, n_rows, d_obuf, L); break;
        case 64: hipExtLaunchKernelGGL(rpack_kernel<64>, grid, block, 0, stream, ev0, ev1, 0, st, d_rows, n_rows, d_obuf, L); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_rsmall(const DStore& st, const DGroup* d_groups, const uint32_t* d_rows, uint32_t n_rows, DHit* d_out,
                         uint8_t* d_rev, uint32_t* d_pm, DGroupResult* d_res, hipStream_t stream, hipEvent_t ev0,
                         hipEvent_t ev1) {
    if (n_rows == 0) return hipSuccess;
    hipExtLaunchKernelGGL(rsmall_kernel, dim3((n_rows + kWaves - 1) / kWaves), dim3(kBlock), 0, stream, ev0, ev1, 0, st,
                          d_groups, d_rows, n_rows, d_out, d_rev, d_pm, d_res);
    return hipGetLastError();
}
int small_src_max() { return kSmallSrc; }

hipError_t launch_pairmat(const DStore& st, const DGroup* d_groups, const DGroupResult* d_res, int n_groups,
                          const DHit* d_out, uint32_t* d_pm, hipStream_t stream) {
    if (n_groups <= 0) return hipSuccess;
    const int threads = n_groups * 32;
    hipLaunchKernelGGL(pairmat_kernel, dim3((threads + 255) / 256), dim3(256), 0, stream, st, d_groups, d_res, n_groups,
                       d_out, d_pm);
    return hipGetLastError();
}

// The eval kernels' launches carry an optional start/stop event pair: the
// events take the dispatch's own timestamps (what rocprofv3 reports as the
// kernel's duration), not the host-side enqueue around it.
hipError_t launch_search(const DStore& st, const DGroup* d_groups, int n_groups, DHit* d_out, uint8_t* d_rev,
                         DGroupResult* d_res, hipStream_t stream, hipEvent_t ev0, hipEvent_t ev1, int kinds) {
    if (n_groups <= 0 || !(kinds & 3)) return hipSuccess;
    // bit 0: some search is constant-score, bit 1: some is variable-score; the
    // event pair spans both dispatches
    if (kinds & 1)
        hipExtLaunchKernelGGL(search_kernel<0>, dim3(n_groups), dim3(kBlock), 0, stream, ev0, (kinds & 2) ? nullptr : ev1,
                              0, st, d_groups, d_out, d_rev, d_res);
    if (kinds & 2)
        hipExtLaunchKernelGGL(search_kernel<kVarK>, dim3(n_groups), dim3(kBlock), 0, stream, (kinds & 1) ? nullptr : ev0,
                              ev1, 0, st, d_groups, d_out, d_rev, d_res);
    return hipGetLastError();
}

hipError_t launch_clear_alive(uint8_t* d_alive, const uint32_t* d_slots, uint32_t n, hipStream_t stream,
                              uint8_t value) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(clear_alive_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_alive, d_slots, n, value);
    return hipGetLastError();
}

hipError_t launch_enum(const DEnumRow* d_rows, const DEnumHit* d_hits, const DEnumItem* d_items, uint32_t n_items,
                       uint32_t* d_cnt, const uint64_t* d_base, uint32_t e0, uint32_t* d_ents, uint32_t* d_off,
                       hipStream_t stream, bool slots) {
    if (n_items == 0) return hipSuccess;
    const dim3 grid((n_items + kBlock - 1) / kBlock);
    if (d_base == nullptr)
        hipLaunchKernelGGL(enum_kernel<true>, grid, dim3(kBlock), 0, stream, d_rows, d_hits, d_items, n_items, d_cnt,
                           nullptr, 0u, nullptr, nullptr);
    else if (slots)
        hipLaunchKernelGGL((enum_kernel<false, true>), grid, dim3(kBlock), 0, stream, d_rows, d_hits, d_items, n_items,
                           nullptr, d_base, e0, d_ents, d_off);
    else
        hipLaunchKernelGGL(enum_kernel<false>, grid, dim3(kBlock), 0, stream, d_rows, d_hits, d_items, n_items, nullptr,
                           d_base, e0, d_ents, d_off);
    return hipGetLastError();
}

hipError_t launch_pairs(const DStore& st, const uint32_t* d_pairs, uint32_t n, uint8_t* d_out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(pair_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, st, d_pairs, n, d_out);
    return hipGetLastError();
}

hipError_t launch_scan(const DStore& st, const DGroup* d_chunks, int n_chunks, DHit* d_scratch, DGroupResult* d_cres,
                       hipStream_t stream, hipEvent_t ev0, hipEvent_t ev1) {
    if (n_chunks <= 0) return hipSuccess;
    hipExtLaunchKernelGGL(scan_kernel, dim3(n_chunks), dim3(kBlock), 0, stream, ev0, ev1, 0, st, d_chunks, d_scratch,
                          d_cres);
    return hipGetLastError();
}

hipError_t launch_pack_slots(const DHit* d_out, uint64_t n, uint32_t* d_slots, const DGroup* d_groups,
                             const DGroupResult* d_res, int n_whole, DHit* d_last, hipStream_t stream) {
    if (n) {
        const uint64_t blocks = (n + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(pack_slots_kernel, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(kBlock), 0, stream,
                           d_out, n, d_slots);
    }
    if (n_whole > 0)
        hipLaunchKernelGGL(last_hits_kernel, dim3((n_whole + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, d_groups,
                           d_res, n_whole, d_out, d_last);
    return hipGetLastError();
}

hipError_t launch_stitch(const DChunkMap* d_map, int n_chunks, const DGroupResult* d_cres, const uint32_t* d_ranges,
                         int n_searches, uint32_t* d_offs, const DHit* d_scratch, DHit* d_out, hipStream_t stream) {
    if (n_chunks <= 0) return hipSuccess;
    hipLaunchKernelGGL(cell_scan_kernel, dim3(n_searches), dim3(kBlock), 0, stream, d_ranges, d_cres, d_offs);
    hipLaunchKernelGGL(stitch_kernel, dim3((n_chunks + kWaves - 1) / kWaves), dim3(kBlock), 0, stream, d_map, d_cres, d_offs,
                       d_scratch, d_out, (uint32_t)n_chunks);
    return hipGetLastError();
}

hipError_t launch_mscan(const DStore& st, const DMScan& ms, const DMSig* d_sigs, const DClause* d_mcl, uint32_t* d_out,
                        DGroupResult* d_cres, bool gen, hipStream_t stream, hipEvent_t ev0, hipEvent_t ev1) {
    if (ms.n_chunks == 0 || ms.n_sigs == 0) return hipSuccess;
    if (ms.n_sigs > (uint32_t)kMaxMSig || ms.n_fields > (uint32_t)kMaxMField || ms.n_clauses > (uint32_t)kMaxMClause)
        return hipErrorInvalidValue;
    const dim3 grid(ms.n_chunks), block(kBlock);
    const int sel = (int)ms.n_fields * 2 + (gen ? 1 : 0);
    const uint32_t mj = ms.chunk / kBlock;
    if (ms.chunk % kBlock || (mj != 2 && mj != 4 && mj != 8) || (mj == 8 && ms.n_sigs > 8)) return hipErrorInvalidValue;
#define NKM_MSCAN_J(NF, G, J)                                                                                 \
    hipExtLaunchKernelGGL(mscan_kernel<NF, G, J>, grid, block, 0, stream, ev0, ev1, 0, st, ms, d_sigs, d_mcl, d_out, \
                          d_cres)
#define NKM_MSCAN(NF, G)                 \
    do {                                 \
        if (mj == 8)                     \
            NKM_MSCAN_J(NF, G, 8);       \
        else if (mj == 4)                \
            NKM_MSCAN_J(NF, G, 4);       \
        else                             \
            NKM_MSCAN_J(NF, G, 2);       \
    } while (0)
    switch (sel) {
        case 0: NKM_MSCAN(0, false); break;
        case 1: NKM_MSCAN(0, true); break;
        case 2: NKM_MSCAN(1, false); break;
        case 3: NKM_MSCAN(1, true); break;
        case 4: NKM_MSCAN(2, false); break;
        case 5: NKM_MSCAN(2, true); break;
        case 6: NKM_MSCAN(3, false); break;
        case 7: NKM_MSCAN(3, true); break;
        case 8: NKM_MSCAN(4, false); break;
        default: NKM_MSCAN(4, true); break;
    }
#undef NKM_MSCAN
#undef NKM_MSCAN_J
    return hipGetLastError();
}

// The hashed scan's three launches (see mscan_hash_kernel).  d_blob: the
// DMSig array, then n_sigs u64 output word offsets, then the hmask + 1 cuckoo
// entries (DMHashEntry, 32-B aligned), then (ms.dsize > 0) the key grid —
// dsize u16 cells (q, 0xFFFF none), padded to 16 B — and the signatures'
// count ranges (tmin, tmax int32 pairs); d_work (16-B aligned): chunks x
// chunk scratch words, then (n_sigs + 1) x chunks counts, then (n_sigs + 1) x
// (chunks + 1) bases (column-major).  phases kMHashCount (contiguous chunks):
// the scan writes counts only and the placement is the bases alone.
size_t mscan_hash_table_off(uint32_t n_sigs) {
    return ((size_t)n_sigs * (sizeof(DMSig) + sizeof(uint64_t)) + 31) & ~(size_t)31;
}
size_t mscan_hash_blob_bytes(uint32_t n_sigs, uint32_t cap, uint32_t dsize) {
    return mscan_hash_table_off(n_sigs) + (size_t)cap * sizeof(DMHashEntry) +
           (dsize ? (((size_t)dsize * 2 + 15) & ~(size_t)15) + (((size_t)n_sigs * 8 + 15) & ~(size_t)15) : 0);
}
uint64_t mscan_hash_counts_word(const DMScan& ms) { return (uint64_t)ms.n_chunks * ms.chunk; }
hipError_t launch_mscan_hash(const DStore& st, const DMScan& ms, const void* d_blob, uint32_t* d_work,
                             DGroupResult* d_cres, uint32_t* d_out32, hipStream_t stream, hipEvent_t ev0, hipEvent_t ev1,
                             int phases, uint32_t c_lo, uint32_t c_hi) {
    if (ms.n_chunks == 0 || ms.n_sigs == 0) return hipSuccess;
    c_hi = c_hi < ms.n_chunks ? c_hi : ms.n_chunks;
    if (c_lo > c_hi || ms.n_blk > kMaxShardBlocks) return hipErrorInvalidValue;
    if (ms.n_blk > 1) {  // the blocks tile [0, n_chunks) in order
        if (ms.cb[0] != 0 || ms.cb[ms.n_blk] != ms.n_chunks) return hipErrorInvalidValue;
        for (uint32_t r = 0; r < ms.n_blk; r++)
            if (ms.cb[r] > ms.cb[r + 1]) return hipErrorInvalidValue;
    }
    const uint32_t mj = ms.chunk / kBlock;
    const uint64_t covered = ms.contig ? (uint64_t)(ms.src_off & ~(ms.chunk - 1)) + (uint64_t)ms.n_chunks * ms.chunk
                                       : (uint64_t)ms.n_chunks * ms.chunk;
    uint64_t cells = 1;
    for (uint32_t f = 0; f < ms.n_fields && f < 4; f++) cells *= ms.dsize ? (uint64_t)ms.drng[f] : 1u;
    if (ms.n_sigs > kMHashSigs || ms.hmask + 1 > kMHashCap || ((ms.hmask + 1) & ms.hmask) || ms.hmask + 1 < 2 * ms.n_sigs ||
        ms.n_fields < 1 || ms.n_fields > 4 || ms.chunk % kBlock || (ms.chunk & (ms.chunk - 1)) ||
        (ms.contig ? mj != 2 && mj != 4 && mj != 8 : mj != 2 && mj != 4) ||
        covered < (ms.contig ? (uint64_t)ms.src_off + ms.src_len : (uint64_t)ms.src_len) ||
        ms.dsize > kMHashGrid || (ms.dsize && cells != ms.dsize))
        return hipErrorInvalidValue;
    const uint64_t* dst = reinterpret_cast<const uint64_t*>(static_cast<const DMSig*>(d_blob) + ms.n_sigs);
    const DMHashEntry* htab =
        reinterpret_cast<const DMHashEntry*>(static_cast<const char*>(d_blob) + mscan_hash_table_off(ms.n_sigs));
    const uint64_t w1 = ms.n_sigs + 1;
    uint32_t* scratch = d_work;  // first: 16-B aligned for the chunks' vector stores
    uint32_t* counts = scratch + (uint64_t)ms.n_chunks * ms.chunk;
    uint32_t* bases = counts + (uint64_t)ms.n_chunks * w1;
    const dim3 grid(ms.n_chunks), egrid(c_hi - c_lo), block(kBlock);
    const bool count_only = ms.contig && (phases & kMHashCount);
    const uint32_t tb = mhash_tab_bytes(ms);
#define NKM_MHASH_K(NF, J, C, CNT)                                                                                  \
    hipExtLaunchKernelGGL(mscan_hash_kernel<NF, J, C, CNT>, egrid, block, (MHashLds<J, C>{tb, ms.n_sigs}.bytes()), \
                          stream, ev0, ev1, 0, st, ms, htab, scratch, counts, c_lo)
#define NKM_MHASH(NF)                                                         \
    do {                                                                      \
        if (ms.contig && mj == 8 && count_only) NKM_MHASH_K(NF, 8, true, true); \
        else if (ms.contig && mj == 8) NKM_MHASH_K(NF, 8, true, false);       \
        else if (ms.contig && mj == 2 && count_only) NKM_MHASH_K(NF, 2, true, true); \
        else if (ms.contig && mj == 2) NKM_MHASH_K(NF, 2, true, false);       \
        else if (ms.contig && count_only) NKM_MHASH_K(NF, 4, true, true);     \
        else if (ms.contig) NKM_MHASH_K(NF, 4, true, false);                  \
        else if (mj == 4) NKM_MHASH_K(NF, 4, false, false);                   \
        else NKM_MHASH_K(NF, 2, false, false);                                \
    } while (0)
    if ((phases & kMHashEval) && c_hi > c_lo) {
        switch (ms.n_fields) {
            case 1: NKM_MHASH(1); break;
            case 2: NKM_MHASH(2); break;
            case 3: NKM_MHASH(3); break;
            default: NKM_MHASH(4); break;
        }
    }
#undef NKM_MHASH
#undef NKM_MHASH_K
#ifdef NKM_MH_DEBUG
    if (ms.pad & 2) return hipGetLastError();  // no counts to place
#endif
    if (!(phases & kMHashPlace)) return hipGetLastError();
    hipLaunchKernelGGL(mscan_base_kernel, dim3(ms.n_sigs + 1), block, 0, stream, ms, counts, bases, d_cres);
    if (!count_only)  // counts only: the lists are never placed (proven, Core::list_proof_mode_)
        hipLaunchKernelGGL(mscan_place_kernel, grid, block, 0, stream, ms, bases, scratch, dst, d_out32);
    return hipGetLastError();
}
uint64_t mscan_hash_work_words(const DMScan& ms) {
    const uint64_t w1 = ms.n_sigs + 1;
    return (uint64_t)ms.n_chunks * w1 + (uint64_t)(ms.n_chunks + 1) * w1 + (uint64_t)ms.n_chunks * ms.chunk;
}
// candidates per lane: 4, gathered or contiguous (C4: 4 and 8 per lane
// measured the same, profiles/r05/r05ar_contig_j_kernel_ab.txt; the 2 / 8
// instantiations stay for tools/mhash_bench)
int mscan_hash_chunk_len(bool) { return 4 * kBlock; }

// Candidates per lane: 2 (C3 1M measured 21.7 us at 2, 24.6 at 4, 35.2 at 8
// candidates per lane — more, shorter waves hide more latency; the 4 / 8
// instantiations stay for tools/mscan_bench).
int mscan_chunk_len(uint32_t) { return 2 * kBlock; }
int mscan_max_sigs() { return kMaxMSig; }
int mscan_max_fields() { return kMaxMField; }
int mscan_max_clauses() { return kMaxMClause; }

// ---- range sources (range_walk.h) -----------------------------------------
// A range batch's pools sorted by (value, source position): rsrc_tile_kernel
// sorts tiles of kRsrcTile elements in LDS, rsrc_merge_kernel merges runs of R
// into runs of 2R (R = kRsrcTile, 2 kRsrcTile, ...), rsrc_bounds_kernel finds
// the clauses' bounds in the sorted keys.  Elements are (key, position) pairs,
// distinct within a pool (positions are), so a merge places an element at its
// index in its run plus its rank in the partner run — a binary search, no
// ties to break.

// Non-short-circuit: with || / && the compiler sinks the position's load into
// a branch taken on equal keys, and a search step on C2's repeated skill values
// becomes two dependent reads (load key, compare, load position) instead of one
// round (tools/rsrc_bench).
__device__ __forceinline__ bool rsrc_less(int64_t ka, uint32_t va, int64_t kb, uint32_t vb) {
    return (ka < kb) | ((ka == kb) & (va < vb));
}

// One tile per workgroup of kRsrcTile lanes, one element each (loaded
// coalesced: the posting entry, then alive / kind / value of that slot), then
// merged in LDS from runs of 1 up to the tile: each lane's binary search in
// the partner run is log2(run) dependent LDS reads, one element per lane.
constexpr int kRsrcBlock = (int)kRsrcTile;
__global__ __launch_bounds__(kRsrcBlock) void rsrc_tile_kernel(DStore st, const DRangePool* __restrict__ pools,
                                                               const DRangeTile* __restrict__ tiles,
                                                               int64_t* __restrict__ okey, uint32_t* __restrict__ opos) {
    __shared__ int64_t sk[2][kRsrcTile];
    __shared__ uint32_t sv[2][kRsrcTile];
    const DRangeTile t = tiles[blockIdx.x];
    const DRangePool P = pools[t.pool];
    const int64_t* __restrict__ fv = st.fval[P.field];
    const uint8_t* __restrict__ fk = st.fkind[P.field];
    const uint32_t e = threadIdx.x;
    const uint32_t i = t.start + e;  // position in the pool's source
    int64_t k = INT64_MAX;
    uint32_t v = kRsrcInvalid | i;
    if (e < t.len && i < P.src_len) {
        const uint32_t s = st.postings[P.src_off + i];
        if (st.alive[s] && fk[s] == KIND_NUMERIC) {
            k = fv[s];
            v = i;
        }
    }
    sk[0][e] = k;
    sv[0][e] = v;
    __syncthreads();
    int b = 0;
    for (uint32_t r = 1; r < t.len; r <<= 1, b ^= 1) {
        if (e < t.len) {
            k = sk[b][e];  // the element now at this position
            v = sv[b][e];
            const uint32_t run = e / r, ps = (run ^ 1u) * r;
            uint32_t o = e;
            if (ps < t.len) {
                uint32_t lo = ps, hi = min(ps + r, t.len);
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (rsrc_less(sk[b][mid], sv[b][mid], k, v)) lo = mid + 1;
                    else hi = mid;
                }
                o = (run & ~1u) * r + (e - run * r) + (lo - ps);
            }
            sk[b ^ 1][o] = k;
            sv[b ^ 1][o] = v;
        }
        __syncthreads();
    }
    if (e < t.len) {
        const uint64_t base = (uint64_t)P.out_off + t.start;
        okey[base + e] = sk[b][e];
        opos[base + e] = sv[b][e];
    }
}

// Runs of R -> runs of 2R over every pool at once (one thread per element;
// blk_pool: the pool of each 256-element block, pools being 256-aligned).
__global__ __launch_bounds__(kBlock) void rsrc_merge_kernel(const DRangePool* __restrict__ pools,
                                                            const uint32_t* __restrict__ blk_pool,
                                                            const int64_t* __restrict__ ik, const uint32_t* __restrict__ ip,
                                                            int64_t* __restrict__ ok, uint32_t* __restrict__ op, uint32_t R) {
    const DRangePool P = pools[blk_pool[blockIdx.x]];
    const uint32_t g = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t e = g - P.out_off;
    const int64_t k = ik[g];
    const uint32_t v = ip[g];
    const uint32_t run = e / R, ps = (run ^ 1u) * R;
    uint32_t o = e;
    if (ps < P.pad_len) {
        const int64_t* __restrict__ bk = ik + P.out_off;
        const uint32_t* __restrict__ bp = ip + P.out_off;
        uint32_t lo = ps, hi = min(ps + R, P.pad_len);
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (rsrc_less(bk[mid], bp[mid], k, v)) lo = mid + 1;
            else hi = mid;
        }
        o = (run & ~1u) * R + (e - run * R) + (lo - ps);
    }
    ok[(uint64_t)P.out_off + o] = k;
    op[(uint64_t)P.out_off + o] = v;
}

__global__ __launch_bounds__(kBlock) void rsrc_bounds_kernel(const DRangePool* __restrict__ pools,
                                                             const int64_t* __restrict__ key,
                                                             const DRangeBound* __restrict__ q, uint32_t nq,
                                                             uint32_t* __restrict__ out) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= nq) return;
    const DRangeBound b = q[t];
    const DRangePool P = pools[b.pool];
    const int64_t* __restrict__ k = key + P.out_off;
    uint32_t lo = 0, hi = P.pad_len;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (b.upper ? k[mid] <= b.key : k[mid] < b.key) lo = mid + 1;
        else hi = mid;
    }
    out[t] = lo;
}

// The whole sort + bounds.  Buffers: keys / positions 2 x n_elems each (ping-
// pong); the sorted ones end in *which (0 or 1).  Event pairs: ev_tile around
// the tile launch, ev_merge[2m], ev_merge[2m + 1] around merge launch m (at
// most max_merge of them).  Returns the number of merge launches in *n_merge.
hipError_t launch_rsrc(const DStore& st, const DRangePool* d_pools, uint32_t max_pad, const DRangeTile* d_tiles,
                       uint32_t n_tiles, const uint32_t* d_blk_pool, uint32_t n_elems, int64_t* d_key[2],
                       uint32_t* d_pos[2], const DRangeBound* d_q, uint32_t nq, uint32_t* d_bounds, int* which,
                       hipStream_t stream, hipEvent_t ev_tile0, hipEvent_t ev_tile1, const hipEvent_t* ev_merge,
                       int max_merge, int* n_merge) {
    *which = 0;
    *n_merge = 0;
    if (n_elems == 0 || n_tiles == 0) return hipSuccess;
    if (n_elems % kBlock) return hipErrorInvalidValue;
    hipExtLaunchKernelGGL(rsrc_tile_kernel, dim3(n_tiles), dim3(kRsrcBlock), 0, stream, ev_tile0, ev_tile1, 0, st,
                          d_pools, d_tiles, d_key[0], d_pos[0]);
    int b = 0, m = 0;
    for (uint32_t R = kRsrcTile; R < max_pad; R <<= 1, b ^= 1, m++) {
        if (m >= max_merge) return hipErrorInvalidValue;
        hipExtLaunchKernelGGL(rsrc_merge_kernel, dim3(n_elems / kBlock), dim3(kBlock), 0, stream, ev_merge[2 * m],
                              ev_merge[2 * m + 1], 0, d_pools, d_blk_pool, d_key[b], d_pos[b], d_key[b ^ 1], d_pos[b ^ 1],
                              R);
    }
    if (nq)
        hipLaunchKernelGGL(rsrc_bounds_kernel, dim3((nq + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, d_pools,
                           d_key[b], d_q, nq, d_bounds);
    *which = b;
    *n_merge = m;
    return hipGetLastError();
}

// The bound queries alone, over keys a launch_rsrc (nq = 0) already sorted on
// this stream (mm_range.cpp issues the sort before the batch's signatures
// are known and the queries once they are).
hipError_t launch_rsrc_bounds(const DRangePool* d_pools, const int64_t* d_key, const DRangeBound* d_q, uint32_t nq,
                              uint32_t* d_bounds, hipStream_t stream) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(rsrc_bounds_kernel, dim3((nq + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, d_pools, d_key, d_q,
                       nq, d_bounds);
    return hipGetLastError();
}

int var_k_capacity() { return kVarK; }
int scan_chunk_len() { return kScanChunk; }

}  // namespace nkm
