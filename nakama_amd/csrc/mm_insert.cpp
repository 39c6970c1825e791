// nakama_amd/csrc/mm_insert.cpp — Insert of a large batch on the host workers.
//
// Insert (server/matchmaker.go:567-682) parses every ticket's query, maps its
// document (MapMatchmakerIndex, :1026-1040; blugeProcessProperty,
// match_common.go:148-212) and files it under m.indexes, m.activeIndexes,
// sessionTickets and partyTickets.  Core::add_locked does that one ticket at a
// time (~0.8 us per ticket: a 1M-ticket Insert took 0.8 s, C5's unique
// queries 2.2 s).  Here a batch is done as data-parallel sweeps on the
// store's WorkPool, with the few inherently serial steps (new signatures, the
// sessionTickets sets) in between:
//   1. ticket ids hashed and checked: a batch that re-inserts a known id, or
//      names one id twice, takes the per-ticket path (replacement order);
//   2. distinct query texts (parallel dedup by hash) compiled in parallel,
//      distinct (query, MinCount, MaxCount) triples resolved to signatures —
//      described and looked up on the workers, committed serially in
//      first-appearance order;
//   3. session, party, node and keyword-property strings interned in bulk
//      (parallel lookup, parallel dedup of the misses, ids in first-appearance
//      order, one arena block, concurrent index insertion);
//   4. every per-slot column resized once and written by the workers.
// The store state equals the per-ticket path's except for the numbering of
// dictionary entries first seen in the batch (ids are compared for equality
// only: a value's id never changes a search, a hit order or a group).
#include <algorithm>
#include <stdexcept>
#include <atomic>
#include <chrono>
#include <cstring>
#include <unordered_map>

#include "gocompat.h"
#include "mm_core.h"

namespace nkm {

namespace {

using clk = std::chrono::steady_clock;
double ms_since(clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); }
std::string_view SV(const char* p) { return p ? std::string_view(p) : std::string_view(); }

// Ordered compaction: the k in [0, n) with keep(k), ascending.
template <class Keep>
std::vector<uint32_t> select(WorkPool& wp, size_t n, Keep keep) {
    const size_t nch = std::max<size_t>(1, std::min<size_t>((size_t)wp.size() * 4, (n + 4095) / 4096));
    std::vector<size_t> at(nch + 1, 0);
    wp.run(nch, [&](size_t c) {
        size_t m = 0;
        for (size_t k = n * c / nch; k < n * (c + 1) / nch; k++) m += keep(k) ? 1 : 0;
        at[c + 1] = m;
    });
    for (size_t c = 0; c < nch; c++) at[c + 1] += at[c];
    std::vector<uint32_t> out(at[nch]);
    wp.run(nch, [&](size_t c) {
        size_t o = at[c];
        for (size_t k = n * c / nch; k < n * (c + 1) / nch; k++)
            if (keep(k)) out[o++] = (uint32_t)k;
    });
    return out;
}

// rep[k] = the first k' <= k whose key equals k's (hash h[k'] == h[k] and
// eq(k', k)).  The keys are partitioned by their hash's top byte (a stable
// scatter: each part keeps ascending k), and each part is resolved by one
// task with its own open-addressing table.
template <class Eq>
void dedup(WorkPool& wp, size_t n, const uint64_t* h, Eq eq, std::vector<uint32_t>& rep) {
    rep.resize(n);
    if (n == 0) return;
    constexpr size_t P = 256;
    const size_t nch = std::max<size_t>(1, std::min<size_t>((size_t)wp.size() * 4, (n + 4095) / 4096));
    std::vector<uint32_t> cnt(nch * P, 0);
    wp.run(nch, [&](size_t c) {
        uint32_t* ct = cnt.data() + c * P;
        for (size_t k = n * c / nch; k < n * (c + 1) / nch; k++) ct[h[k] >> 56]++;
    });
    std::vector<uint64_t> start(P + 1, 0), pos(nch * P);
    uint64_t run = 0;
    for (size_t p = 0; p < P; p++) {
        start[p] = run;
        for (size_t c = 0; c < nch; c++) {
            pos[c * P + p] = run;
            run += cnt[c * P + p];
        }
    }
    start[P] = run;
    std::vector<uint32_t> idx(n);
    wp.run(nch, [&](size_t c) {
        uint64_t* ps = pos.data() + c * P;
        for (size_t k = n * c / nch; k < n * (c + 1) / nch; k++) idx[ps[h[k] >> 56]++] = (uint32_t)k;
    });
    wp.run(P, [&](size_t p) {
        const size_t a = start[p], b = start[p + 1];
        if (a == b) return;
        size_t cap = 16;
        while (cap < 2 * (b - a)) cap <<= 1;
        std::vector<uint32_t> tab(cap, UINT32_MAX);
        const size_t mask = cap - 1;
        for (size_t i = a; i < b; i++) {
            const uint32_t k = idx[i];
            size_t j = (size_t)h[k] & mask;
            for (;; j = (j + 1) & mask) {
                const uint32_t f = tab[j];
                if (f == UINT32_MAX) {
                    tab[j] = k;
                    rep[k] = k;
                    break;
                }
                if (h[f] == h[k] && eq(f, k)) {
                    rep[k] = f;
                    break;
                }
            }
        }
    });
}

// Interns n strings (s[k], hash h[k]; skip[k]: leave ids[k] alone) into d:
// existing ones are found on the workers; the missing ones are deduplicated,
// numbered in first-appearance order, copied into one arena block and added
// to the index concurrently.
void bulk_intern(WorkPool& wp, Dict& d, size_t n, const std::string_view* s, const uint64_t* h, uint32_t* ids,
                 const uint8_t* skip = nullptr) {
    const size_t nch = std::max<size_t>(1, std::min<size_t>((size_t)wp.size() * 4, (n + 4095) / 4096));
    wp.run(nch, [&](size_t c) {
        for (size_t k = n * c / nch; k < n * (c + 1) / nch; k++) {
            if (skip && skip[k]) continue;
            const int64_t f = d.idx.find(h[k], [&](uint32_t id) { return d.str(id) == s[k]; });
            ids[k] = f >= 0 ? (uint32_t)f : UINT32_MAX;
        }
    });
    const std::vector<uint32_t> miss = select(wp, n, [&](size_t k) { return !(skip && skip[k]) && ids[k] == UINT32_MAX; });
    const size_t m = miss.size();
    if (!m) return;
    const size_t nchm = std::max<size_t>(1, std::min<size_t>((size_t)wp.size() * 4, (m + 4095) / 4096));
    std::vector<uint64_t> mh(m);
    wp.run(nchm, [&](size_t c) {
        for (size_t i = m * c / nchm; i < m * (c + 1) / nchm; i++) mh[i] = h[miss[i]];
    });
    std::vector<uint32_t> rep;
    dedup(wp, m, mh.data(), [&](uint32_t a, uint32_t b) { return s[miss[a]] == s[miss[b]]; }, rep);
    const std::vector<uint32_t> first = select(wp, m, [&](size_t i) { return rep[i] == i; });
    const uint32_t base = (uint32_t)d.size();
    std::vector<uint32_t> nid(m, 0);  // at each first: its new id
    std::vector<uint64_t> boff(first.size() + 1, 0);
    {
        // new ids and arena offsets (a prefix sum of the sizes) in chunks
        const size_t nfirst = first.size();
        const size_t ncf = std::max<size_t>(1, std::min<size_t>((size_t)wp.size() * 4, (nfirst + 4095) / 4096));
        std::vector<uint64_t> part(ncf + 1, 0);
        wp.run(ncf, [&](size_t c) {
            uint64_t b = 0;
            for (size_t j = nfirst * c / ncf; j < nfirst * (c + 1) / ncf; j++) {
                nid[first[j]] = base + (uint32_t)j;
                b += s[miss[first[j]]].size() + 1;
                boff[j + 1] = b;  // chunk-local, rebased below
            }
            part[c + 1] = b;
        });
        for (size_t c = 0; c < ncf; c++) part[c + 1] += part[c];
        wp.run(ncf, [&](size_t c) {
            for (size_t j = nfirst * c / ncf; j < nfirst * (c + 1) / ncf; j++) boff[j + 1] += part[c];
        });
    }
    char* blk = d.arena.block(boff[first.size()]);
    d.ptr.resize(base + first.size());
    d.len.resize(base + first.size());
    d.idx.reserve(base + first.size());
    const size_t nf = first.size(), nchf = std::max<size_t>(1, std::min<size_t>((size_t)wp.size() * 4, (nf + 1023) / 1024));
    wp.run(nchf, [&](size_t c) {
        for (size_t j = nf * c / nchf; j < nf * (c + 1) / nchf; j++) {
            const std::string_view v = s[miss[first[j]]];
            char* p = blk + boff[j];
            if (!v.empty()) std::memcpy(p, v.data(), v.size());
            p[v.size()] = 0;
            d.ptr[base + j] = p;
            d.len[base + j] = (uint32_t)v.size();
            d.idx.put_new_concurrent(h[miss[first[j]]], base + (uint32_t)j);
        }
    });
    d.idx.n += nf;
    wp.run(nchm, [&](size_t c) {
        for (size_t i = m * c / nchm; i < m * (c + 1) / nchm; i++) ids[miss[i]] = nid[rep[i]];
    });
}

inline uint64_t mix3(uint64_t a, uint64_t b, uint64_t c) {
    uint64_t x = (a + 0x9E3779B97F4A7C15ull) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ b ^ (x >> 31)) * 0x94D049BB133111EBull;
    x = (x ^ c ^ (x >> 29)) * 0xBF58476D1CE4E5B9ull;
    return x ^ (x >> 32);
}

inline size_t rec_str(std::string_view v) { return 4 + v.size() + 1; }
inline char* put_u32(char* p, uint32_t v) {
    std::memcpy(p, &v, 4);
    return p + 4;
}
inline char* put_str(char* p, std::string_view v) {
    p = put_u32(p, (uint32_t)v.size());
    if (!v.empty()) std::memcpy(p, v.data(), v.size());
    p[v.size()] = 0;
    return p + v.size() + 1;
}

}  // namespace

// The new signatures of a bulk Insert, committed on the workers (the serial
// sig_commit per triple was 160-350 ms of a C5 1M Insert: up to a million
// new signatures, one push_back chain each): the new triples are
// deduplicated among themselves (distinct query strings can compile to one
// signature), numbered in first-appearance order — the ids the serial loop
// assigns — and their clauses, descriptors, field flags and index entries
// written in parallel.  tfound[j] >= 0: triple j's existing signature.
template <class Get>
void Core::commit_new_sigs(WorkPool& wp, size_t nt, const std::vector<int64_t>& tfound,
                           const std::vector<uint64_t>& thash, std::vector<Sig>& tsig, std::vector<uint32_t>& tsg,
                           Get get) {
    std::vector<uint32_t> nw;  // the new triples, in order
    for (size_t j = 0; j < nt; j++) {
        if (tfound[j] >= 0) tsg[j] = (uint32_t)tfound[j];
        else nw.push_back((uint32_t)j);
    }
    const size_t nn = nw.size();
    if (nn == 0) return;
    std::vector<uint64_t> nh(nn);
    for (size_t k = 0; k < nn; k++) nh[k] = thash[nw[k]];
    std::vector<uint32_t> rep;
    dedup(wp, nn, nh.data(), [&](uint32_t a, uint32_t b) {
        const DClause *da, *db;
        size_t na, nb;
        uint8_t ka, kb;
        int32_t mna, mxa, mnb, mxb;
        get(nw[a], da, na, ka, mna, mxa);
        get(nw[b], db, nb, kb, mnb, mxb);
        return ka == kb && mna == mnb && mxa == mxb && na == nb && (na == 0 || std::memcmp(da, db, na * sizeof(DClause)) == 0);
    }, rep);
    // ids and clause offsets of the distinct new signatures, in order
    std::vector<uint32_t> nid(nn), coff(nn, 0);
    const uint32_t id0 = (uint32_t)sigs_.size();
    const uint64_t c0 = clauses_.size();
    uint32_t nd = 0;
    uint64_t ncl = 0;
    for (size_t k = 0; k < nn; k++) {
        if (rep[k] != k) continue;
        const DClause* dc;
        size_t ndc;
        uint8_t kind;
        int32_t mn, mx;
        get(nw[k], dc, ndc, kind, mn, mx);
        nid[k] = id0 + nd++;
        coff[k] = (uint32_t)(c0 + ncl);
        ncl += ndc;
    }
    if (c0 + ncl > UINT32_MAX) throw std::length_error("clause table past 2^32 entries");
    sigs_.resize((size_t)id0 + nd);
    sig_fmask_.resize((size_t)id0 + nd);
    sig_lite_.resize((size_t)id0 + nd);
    clauses_.resize(c0 + ncl);
    sig_idx_.reserve(sig_idx_.n + nd);
    const size_t nf = field_used_.size();
    const size_t nch = std::max<size_t>(1, std::min<size_t>((size_t)wp.size() * 4, (nn + 4095) / 4096));
    std::vector<std::vector<uint8_t>> used(nch), posting(nch);
    wp.run(nch, [&](size_t c) {
        std::vector<uint8_t>& u = used[c];
        std::vector<uint8_t>& pst = posting[c];
        u.assign(nf, 0);
        pst.assign(nf, 0);
        for (size_t k = nn * c / nch; k < nn * (c + 1) / nch; k++) {
            const uint32_t j = nw[k];
            if (rep[k] != k) continue;
            const DClause* dc;
            size_t ndc;
            uint8_t kind;
            int32_t mn, mx;
            get(j, dc, ndc, kind, mn, mx);
            Sig& g = tsig[j];
            g.clause_off = coff[k];
            for (size_t x = 0; x < ndc; x++) {
                if (dc[x].op != OP_FALSE) u[dc[x].field] = 1;
                clauses_[coff[k] + x] = dc[x];
            }
            for (auto& mt : g.must_terms) pst[mt.first] = 1;
            const uint32_t id = nid[k];
            sig_fmask_[id] = g.must_fmask;
            sig_lite_[id] = lite_of(g);
            sigs_[id] = std::move(g);
            sig_idx_.put_new_concurrent(thash[j], id);
        }
    });
    sig_idx_.n += nd;
    for (size_t c = 0; c < nch; c++)
        for (size_t f = 0; f < nf; f++) {
            if (used[c][f]) field_used_[f] = 1;
            if (posting[c][f] && !field_posting_[f]) {
                field_posting_[f] = 1;
                index_dirty_ = true;
            }
        }
    for (size_t k = 0; k < nn; k++) tsg[nw[k]] = nid[rep[k]];
}

bool Core::insert_bulk(const mm_ticket* ts, int32_t n_in, double* ph) {
    const size_t n = (size_t)n_in;
    if (field_used_.size() > F_PARTY && (field_used_[F_TICKET] || field_used_[F_PARTY])) return false;  // id-valued fields
    WorkPool& wp = workers();
    const size_t nch = std::max<size_t>(1, std::min<size_t>((size_t)wp.size() * 4, (n + 4095) / 4096));
    auto par = [&](const std::function<void(size_t, size_t)>& fn) {  // fn(lo, hi) over the batch in chunks
        wp.run(nch, [&](size_t c) { fn(n * c / nch, n * (c + 1) / nch); });
    };
    auto t0 = clk::now();
    // ---- 1. ticket ids: a known id or a repeated one -> the per-ticket path
    std::vector<uint64_t> th(n);
    std::atomic<bool> clash{false};
    par([&](size_t lo, size_t hi) {
        bool c = false;
        for (size_t k = lo; k < hi; k++) {
            const std::string_view id = SV(ts[k].ticket);
            th[k] = str_hash(id);
            if (!c && slot_of_.n)  // live, or a dead record the per-ticket path's put() would overwrite
                c = slot_of_.find(th[k], [&](uint32_t v) { return tk(v) == id; }) >= 0;
        }
        if (c) clash = true;
    });
    if (clash) return false;
    {
        std::vector<uint32_t> rep;
        dedup(wp, n, th.data(), [&](uint32_t a, uint32_t b) { return SV(ts[a].ticket) == SV(ts[b].ticket); }, rep);
        std::atomic<bool> dup{false};
        par([&](size_t lo, size_t hi) {
            for (size_t k = lo; k < hi; k++)
                if (rep[k] != k) { dup = true; return; }
        });
        if (dup) return false;
    }
    ph[0] = ms_since(t0);
    t0 = clk::now();
    // ---- 2. queries -> signatures
    std::vector<uint64_t> qh(n);
    par([&](size_t lo, size_t hi) {
        for (size_t k = lo; k < hi; k++) qh[k] = str_hash(SV(ts[k].query));
    });
    auto tlap = t0;
    auto lap = [&](int k) {  // ph[5..10]: the signature phase's parts (NKM_PROFILE)
        const auto now = clk::now();
        ph[k] += std::chrono::duration<double, std::milli>(now - tlap).count();
        tlap = now;
    };
    std::vector<uint32_t> qrep;
    dedup(wp, n, qh.data(), [&](uint32_t a, uint32_t b) {  // a shared query string compares by pointer
        return ts[a].query == ts[b].query || SV(ts[a].query) == SV(ts[b].query);
    }, qrep);
    const std::vector<uint32_t> qfirst = select(wp, n, [&](size_t k) { return qrep[k] == k; });
    const size_t nq = qfirst.size();
    std::vector<uint32_t> qpos(n, 0);  // at each first: its distinct-query index
    for (size_t j = 0; j < nq; j++) qpos[qfirst[j]] = (uint32_t)j;
    lap(5);  // query hashes, dedup
    std::vector<CompiledQuery> cq(nq);
    std::vector<int> cst(nq);
    wp.run(std::max<size_t>(1, std::min<size_t>(nq, (size_t)wp.size() * 8)), [&](size_t c) {
        const size_t nc = std::max<size_t>(1, std::min<size_t>(nq, (size_t)wp.size() * 8));
        for (size_t j = nq * c / nc; j < nq * (c + 1) / nc; j++)
            cst[j] = compile_query(SV(ts[qfirst[j]].query), &cq[j]);
    });
    lap(6);  // compiles
    // tickets whose query does not compile are skipped (the reference logs and continues)
    std::vector<uint32_t> qof(n);
    par([&](size_t lo, size_t hi) {
        for (size_t k = lo; k < hi; k++) qof[k] = qpos[qrep[k]];
    });
    std::vector<uint32_t> keep = select(wp, n, [&](size_t k) { return cst[qof[k]] == CQ_OK; });
    const size_t m = keep.size();  // the batch's tickets, in order
    // distinct (query, MinCount, MaxCount) of the kept tickets
    std::vector<uint64_t> trh(m);
    wp.run(nch, [&](size_t c) {
        for (size_t i = m * c / nch; i < m * (c + 1) / nch; i++) {
            const mm_ticket& t = ts[keep[i]];
            trh[i] = mix3(qof[keep[i]], (uint32_t)t.min_count, (uint32_t)t.max_count);
        }
    });
    std::vector<uint32_t> trep;
    dedup(wp, m, trh.data(), [&](uint32_t a, uint32_t b) {
        const mm_ticket &x = ts[keep[a]], &y = ts[keep[b]];
        return qof[keep[a]] == qof[keep[b]] && x.min_count == y.min_count && x.max_count == y.max_count;
    }, trep);
    const std::vector<uint32_t> tfirst = select(wp, m, [&](size_t i) { return trep[i] == i; });
    const size_t nt = tfirst.size();
    lap(7);  // (query, Min, Max) triples
    // the distinct queries' field names and terms: names are few (serial
    // field_of for the new ones), terms are interned in bulk
    std::vector<uint8_t> used_q(nq, 0);
    for (uint32_t i : tfirst) used_q[qof[keep[i]]] = 1;
    std::vector<uint64_t> cl_off(nq + 1, 0);
    for (size_t j = 0; j < nq; j++) cl_off[j + 1] = cl_off[j] + (used_q[j] ? cq[j].clauses.size() : 0);
    const size_t ncl = cl_off[nq];
    std::vector<std::string_view> cl_field(ncl), cl_term(ncl);
    std::vector<uint64_t> cl_fh(ncl), cl_thash(ncl);
    std::vector<uint8_t> cl_noterm(ncl, 1);
    std::vector<uint32_t> cl_fid(ncl, UINT32_MAX), cl_tid(ncl, 0);
    std::vector<uint8_t> serial_q(nq, 0);  // a regexp / wildcard / fuzzy clause: the signature is made by sig_of
    wp.run(std::max<size_t>(1, std::min<size_t>(nq, (size_t)wp.size() * 4)), [&](size_t c) {
        const size_t nc = std::max<size_t>(1, std::min<size_t>(nq, (size_t)wp.size() * 4));
        for (size_t j = nq * c / nc; j < nq * (c + 1) / nc; j++) {
            if (!used_q[j]) continue;
            for (size_t x = 0; x < cq[j].clauses.size(); x++) {
                const HostClause& hc = cq[j].clauses[x];
                const size_t o = cl_off[j] + x;
                if (hc.op == OP_TERMSET) serial_q[j] = 1;
                if (hc.op == OP_FALSE) continue;
                cl_field[o] = hc.field;
                cl_fh[o] = str_hash(cl_field[o]);
                const int64_t f = field_dict_.idx.find(cl_fh[o], [&](uint32_t id) { return field_dict_.str(id) == cl_field[o]; });
                if (f >= 0) cl_fid[o] = (uint32_t)f;
                if (hc.op == OP_TERM || hc.op == OP_NUMLIT) {
                    cl_term[o] = hc.term;
                    cl_thash[o] = str_hash(cl_term[o]);
                    cl_noterm[o] = 0;
                }
            }
        }
    });
    for (size_t o = 0; o < ncl; o++)
        if (cl_fid[o] == UINT32_MAX && !cl_field[o].empty()) cl_fid[o] = field_of(std::string(cl_field[o]));
    for (size_t o = 0; o < ncl; o++)  // OP_FALSE clauses keep field 0 (sig_of's convention)
        if (cl_fid[o] == UINT32_MAX) cl_fid[o] = 0;
    bulk_intern(wp, dict_, ncl, cl_term.data(), cl_thash.data(), cl_tid.data(), cl_noterm.data());
    // each distinct query's compiled clauses (they do not depend on the
    // counts) and their hash, on the workers
    std::vector<DClause> qdc(ncl);
    std::vector<uint64_t> qch(nq, 0);
    wp.run(std::max<size_t>(1, std::min<size_t>(nq, (size_t)wp.size() * 4)), [&](size_t c) {
        const size_t nc = std::max<size_t>(1, std::min<size_t>(nq, (size_t)wp.size() * 4));
        for (size_t q = nq * c / nc; q < nq * (c + 1) / nc; q++) {
            if (!used_q[q] || serial_q[q]) continue;
            for (size_t x = 0; x < cq[q].clauses.size(); x++) {
                const HostClause& hc = cq[q].clauses[x];
                const size_t o = cl_off[q] + x;
                DClause d{};
                d.op = hc.op;
                d.occur = hc.occur;
                d.lo = hc.lo;
                d.hi = hc.hi;
                d.score = hc.score;
                d.field = hc.op == OP_FALSE ? 0 : (uint16_t)cl_fid[o];
                d.term = (hc.op == OP_TERM || hc.op == OP_NUMLIT) ? cl_tid[o] : 0;
                qdc[o] = d;
            }
            qch[q] = sig_clause_hash(qdc.data() + cl_off[q], cq[q].clauses.size());
        }
    });
    lap(8);  // fields, terms, clause words
    // every distinct triple: looked up on the workers (described when new),
    // committed in first-appearance order
    std::vector<uint64_t> thash(nt, 0);
    std::vector<Sig> tsig(nt);
    std::vector<int64_t> tfound(nt, -1);
    auto triple = [&](size_t j, uint32_t& q, const mm_ticket*& t) {
        t = &ts[keep[tfirst[j]]];
        q = qof[keep[tfirst[j]]];
    };
    wp.run(std::max<size_t>(1, std::min<size_t>(nt, (size_t)wp.size() * 4)), [&](size_t c) {
        const size_t nc = std::max<size_t>(1, std::min<size_t>(nt, (size_t)wp.size() * 4));
        std::vector<DClause> dcv;
        for (size_t j = nt * c / nc; j < nt * (c + 1) / nc; j++) {
            uint32_t q;
            const mm_ticket* t;
            triple(j, q, t);
            if (serial_q[q]) continue;
            const DClause* dc = qdc.data() + cl_off[q];
            const size_t ndc = cq[q].clauses.size();
            thash[j] = sig_hash(qch[q], cq[q].kind, t->min_count, t->max_count, kNoParty);
            tfound[j] = sig_idx_.find(thash[j], [&](uint32_t id) {
                return sig_eq(id, cq[q].kind, t->min_count, t->max_count, kNoParty, dc, ndc);
            });
            if (tfound[j] < 0) {
                dcv.assign(dc, dc + ndc);
                sig_describe(tsig[j], dcv, cq[q], t->min_count, t->max_count, kNoParty);
            }
        }
    });
    lap(9);  // lookups, descriptors
    std::vector<uint32_t> tsg(nt);
    bool any_serial = false;
    for (size_t j = 0; j < nt && !any_serial; j++) any_serial = serial_q[qof[keep[tfirst[j]]]] != 0;
    if (any_serial) {
        // a regexp / wildcard / fuzzy query (sig_of interns its matchers): one
        // triple at a time, in first-appearance order
        for (size_t j = 0; j < nt; j++) {
            uint32_t q;
            const mm_ticket* t;
            triple(j, q, t);
            if (serial_q[q]) {
                tsg[j] = sig_of(cq[q], t->min_count, t->max_count, kNoParty);
            } else if (tfound[j] >= 0) {
                tsg[j] = (uint32_t)tfound[j];
            } else {
                const DClause* dc = qdc.data() + cl_off[q];
                const size_t ndc = cq[q].clauses.size();
                const int64_t f = sig_idx_.find(thash[j], [&](uint32_t id) {  // an earlier triple may have made it
                    return sig_eq(id, cq[q].kind, t->min_count, t->max_count, kNoParty, dc, ndc);
                });
                tsg[j] = f >= 0 ? (uint32_t)f : sig_commit(std::move(tsig[j]), dc, ndc, thash[j], false);
            }
        }
    } else {
        commit_new_sigs(wp, nt, tfound, thash, tsig, tsg, [&](size_t j, const DClause*& dc, size_t& ndc, uint8_t& kind,
                                                              int32_t& mn, int32_t& mx) {
            uint32_t q;
            const mm_ticket* t;
            triple(j, q, t);
            dc = qdc.data() + cl_off[q];
            ndc = cq[q].clauses.size();
            kind = cq[q].kind;
            mn = t->min_count;
            mx = t->max_count;
        });
    }
    lap(10);  // commits
    // A query of this batch may be the first to read the ticket / party_id
    // field (sig_commit switched it on): those columns are filled per ticket
    // (add_locked), so the batch takes the per-ticket path.  Nothing of the
    // store is written yet — the signatures and interned terms made above are
    // what that path looks up; the fields they switched on get their columns
    // over the existing slots first (sig_commit deferred that to step 3).
    if (field_used_.size() > F_PARTY && (field_used_[F_TICKET] || field_used_[F_PARTY])) {
        materialize_fields();
        return false;
    }
    std::vector<uint32_t> tpos(m, 0);
    for (size_t j = 0; j < nt; j++) tpos[tfirst[j]] = (uint32_t)j;
    ph[1] = ms_since(t0);
    t0 = clk::now();
    // ---- 3. strings: sessions, parties, nodes, property keys and keyword values
    std::vector<uint64_t> poff(m + 1, 0), spoff(m + 1, 0), npoff(m + 1, 0);
    for (size_t i = 0; i < m; i++) {
        const mm_ticket& t = ts[keep[i]];
        poff[i + 1] = poff[i] + (uint64_t)std::max(t.n_presences, 0);
        spoff[i + 1] = spoff[i] + (uint64_t)std::max(t.n_str_props, 0);
        npoff[i + 1] = npoff[i] + (uint64_t)std::max(t.n_num_props, 0);
    }
    const size_t np = poff[m], nsp = spoff[m], nnp = npoff[m];
    std::vector<std::string_view> sv(np), pv(m), nv(m), kv(nsp + nnp), vv(nsp);
    std::vector<uint64_t> sh(np), ph_(m), nh(m), vh(nsp);
    std::vector<uint8_t> nopart(m), vskip(nsp, 0);
    std::vector<int64_t> vdt(nsp, 0);  // a datetime value's UnixNano
    wp.run(nch, [&](size_t c) {
        for (size_t i = m * c / nch; i < m * (c + 1) / nch; i++) {
            const mm_ticket& t = ts[keep[i]];
            for (int x = 0; x < t.n_presences; x++) {
                sv[poff[i] + x] = SV(t.presences[x].session_id);
                sh[poff[i] + x] = str_hash(sv[poff[i] + x]);
            }
            pv[i] = SV(t.party_id);
            nopart[i] = pv[i].empty();
            ph_[i] = str_hash(pv[i]);
            nv[i] = SV(t.node);  // Insert keeps the ticket's node (add_locked, from_insert)
            nh[i] = str_hash(nv[i]);
            for (int x = 0; x < t.n_str_props; x++) {
                const size_t o = spoff[i] + x;
                kv[o] = SV(t.str_props[x].key);
                vv[o] = SV(t.str_props[x].value);
                if (bluge_datetime(vv[o], &vdt[o])) vskip[o] = 1;
                else vh[o] = str_hash(vv[o]);
            }
            for (int x = 0; x < t.n_num_props; x++) {
                const size_t o = nsp + npoff[i] + x;
                kv[o] = SV(t.num_props[x].key);
            }
        }
    });
    std::vector<uint32_t> sid(np), pid(m, kNoParty), nid(m), vid(nsp, 0), kid(nsp + nnp);
    bulk_intern(wp, sess_dict_, np, sv.data(), sh.data(), sid.data());
    bulk_intern(wp, party_dict_, m, pv.data(), ph_.data(), pid.data(), nopart.data());
    bulk_intern(wp, node_dict_, m, nv.data(), nh.data(), nid.data());
    bulk_intern(wp, dict_, nsp, vv.data(), vh.data(), vid.data(), vskip.data());
    // property keys -> fields: each chunk lists its distinct keys in order of
    // appearance (a ticket's string keys before its numeric keys), new ones
    // go through prop_field chunk by chunk — the first-appearance order —
    // and every property then reads its field from the (small) key table
    {
        std::vector<std::vector<std::string_view>> ck(nch);
        wp.run(nch, [&](size_t c) {
            std::unordered_map<std::string_view, char> seen;
            for (size_t i = m * c / nch; i < m * (c + 1) / nch; i++) {
                for (uint64_t o = spoff[i]; o < spoff[i + 1]; o++)
                    if (seen.emplace(kv[o], 0).second) ck[c].push_back(kv[o]);
                for (uint64_t o = nsp + npoff[i]; o < nsp + npoff[i + 1]; o++)
                    if (seen.emplace(kv[o], 0).second) ck[c].push_back(kv[o]);
            }
        });
        std::unordered_map<std::string_view, uint32_t> kf;
        for (auto& v : ck)
            for (auto k : v)
                if (!kf.count(k)) kf.emplace(k, prop_field(k));
        wp.run(nch, [&](size_t c) {
            const size_t a = (nsp + nnp) * c / nch, b = (nsp + nnp) * (c + 1) / nch;
            for (size_t o = a; o < b; o++) kid[o] = kf.find(kv[o])->second;
        });
    }
    ph[2] = ms_since(t0);
    t0 = clk::now();
    // ---- 4. the store's columns
    materialize_fields();  // fields the batch's new signatures reference, over the existing slots
    const size_t s0 = nslots(), s1 = s0 + m;
    std::vector<uint64_t> tkoff(m + 1, 0), coff(m + 1, 0);
    wp.run(nch, [&](size_t c) {
        for (size_t i = m * c / nch; i < m * (c + 1) / nch; i++) {
            const mm_ticket& t = ts[keep[i]];
            tkoff[i + 1] = SV(t.ticket).size() + 1;
            size_t r = 12 + rec_str(SV(t.session_id)) + rec_str(SV(t.party_id)) + rec_str(SV(t.query));
            for (int x = 0; x < t.n_presences; x++)
                r += rec_str(SV(t.presences[x].user_id)) + rec_str(SV(t.presences[x].session_id)) +
                     rec_str(SV(t.presences[x].username)) + rec_str(SV(t.presences[x].node));
            for (int x = 0; x < t.n_str_props; x++) r += rec_str(SV(t.str_props[x].key)) + rec_str(SV(t.str_props[x].value));
            for (int x = 0; x < t.n_num_props; x++) r += rec_str(SV(t.num_props[x].key)) + 8;
            coff[i + 1] = r;
        }
    });
    for (size_t i = 0; i < m; i++) {
        tkoff[i + 1] += tkoff[i];
        coff[i + 1] += coff[i];
    }
    char* tkb = tk_arena_.block(tkoff[m]);
    const size_t cb0 = cold_.bytes.size();
    cold_.bytes.resize(cb0 + coff[m]);
    cold_.off.resize(s1);
    tk_ptr_.resize(s1);
    tk_len_.resize(s1);
    tnode_.resize(s1);
    created_.resize(s1);
    ckey_.resize(s1);
    minc_.resize(s1);
    maxc_.resize(s1);
    cm_.resize(s1);
    count_.resize(s1);
    intervals_.resize(s1);
    party_.resize(s1);
    live_.resize(s1, 1);
    indexed_.resize(s1, 1);
    is_active_.resize(s1);
    sig_.resize(s1);
    self_match_.resize(s1);
    squery_.resize(s1);
    hot_.resize(s1);
    if (pres_off_.empty()) pres_off_.push_back(0);
    const uint32_t pbase = pres_off_.back();
    pres_off_.resize(s1 + 1);
    pres_sess_.resize((size_t)pbase + np);
    std::vector<uint16_t> cols;  // fields with a dense host column
    for (size_t f = 0; f < fval_.size(); f++)
        if (!fval_[f].empty() || field_used_[f]) {
            fval_[f].resize(s1, 0);
            fkind_[f].resize(s1, KIND_ABSENT);
            cols.push_back((uint16_t)f);
        }
    std::vector<uint8_t> has_col(fval_.size(), 0);
    for (uint16_t f : cols) has_col[f] = 1;
    const int maxI = cfg_.max_intervals;
    std::vector<int32_t> cmax(nch, 0);
    wp.run(nch, [&](size_t c) {
        int32_t mp = 0;
        for (size_t i = m * c / nch; i < m * (c + 1) / nch; i++) {
            const mm_ticket& t = ts[keep[i]];
            const uint32_t s = (uint32_t)(s0 + i);
            const std::string_view id = SV(t.ticket);
            char* p = tkb + tkoff[i];
            if (!id.empty()) std::memcpy(p, id.data(), id.size());
            p[id.size()] = 0;
            tk_ptr_[s] = p;
            tk_len_[s] = (uint32_t)id.size();
            // cold record (strstore.h ColdStore layout)
            char* w = cold_.bytes.data() + cb0 + coff[i];
            cold_.off[s] = cb0 + coff[i];
            w = put_u32(w, (uint32_t)std::max(t.n_presences, 0));
            w = put_u32(w, (uint32_t)std::max(t.n_str_props, 0));
            w = put_u32(w, (uint32_t)std::max(t.n_num_props, 0));
            w = put_str(w, SV(t.session_id));
            w = put_str(w, SV(t.party_id));
            w = put_str(w, SV(t.query));
            for (int x = 0; x < t.n_presences; x++) {
                w = put_str(w, SV(t.presences[x].user_id));
                w = put_str(w, SV(t.presences[x].session_id));
                w = put_str(w, SV(t.presences[x].username));
                w = put_str(w, SV(t.presences[x].node));
            }
            for (int x = 0; x < t.n_str_props; x++) {
                w = put_str(w, SV(t.str_props[x].key));
                w = put_str(w, SV(t.str_props[x].value));
            }
            for (int x = 0; x < t.n_num_props; x++) {
                w = put_str(w, SV(t.num_props[x].key));
                std::memcpy(w, &t.num_props[x].value, 8);
                w += 8;
            }
            tnode_[s] = nid[i];
            created_[s] = t.created_at;
            ckey_[s] = sortable_i64((double)t.created_at);
            minc_[s] = t.min_count;
            maxc_[s] = t.max_count;
            cm_[s] = t.count_multiple;
            count_[s] = t.n_presences;
            mp = std::max(mp, t.n_presences);
            intervals_[s] = t.intervals;
            party_[s] = nopart[i] ? kNoParty : pid[i];
            is_active_[s] = t.intervals < maxI ? 1 : 0;
            pres_off_[s + 1] = pbase + (uint32_t)poff[i + 1];
            for (int x = 0; x < t.n_presences; x++) pres_sess_[pbase + poff[i] + x] = sid[poff[i] + x];
            const uint32_t sg = tsg[tpos[trep[i]]];
            sig_[s] = sg;
            squery_[s] = DQuery{sigs_[sg].clause_off, sigs_[sg].n_clauses, sigs_[sg].qkind, 0};
            // document columns: builtins, then the properties in order (the
            // last value of a field wins; numeric after string, so numeric
            // wins on a key clash: doc_props)
            if (has_col[F_MIN]) { fkind_[F_MIN][s] = KIND_NUMERIC; fval_[F_MIN][s] = sortable_i64((double)t.min_count); }
            if (has_col[F_MAX]) { fkind_[F_MAX][s] = KIND_NUMERIC; fval_[F_MAX][s] = sortable_i64((double)t.max_count); }
            if (has_col[F_CREATED]) { fkind_[F_CREATED][s] = KIND_NUMERIC; fval_[F_CREATED][s] = ckey_[s]; }
            for (int x = 0; x < t.n_str_props; x++) {
                const size_t o = spoff[i] + x;
                const uint16_t f = (uint16_t)kid[o];
                if (!has_col[f]) continue;
                if (vskip[o]) { fkind_[f][s] = KIND_NUMERIC; fval_[f][s] = vdt[o]; }
                else { fkind_[f][s] = KIND_KEYWORD; fval_[f][s] = (int64_t)vid[o]; }
            }
            for (int x = 0; x < t.n_num_props; x++) {
                const uint16_t f = (uint16_t)kid[nsp + npoff[i] + x];
                if (!has_col[f]) continue;
                fkind_[f][s] = KIND_NUMERIC;
                fval_[f][s] = sortable_i64(t.num_props[x].value);
            }
        }
        cmax[c] = mp;
    });
    for (int32_t x : cmax) max_pres_ = std::max(max_pres_, x);
    wp.run(nch, [&](size_t c) {
        for (size_t s = s0 + m * c / nch; s < s0 + m * (c + 1) / nch; s++) {
            set_hot((uint32_t)s);
            self_match_[s] = self_match_of((uint32_t)s);
        }
    });
    ph[3] = ms_since(t0);
    t0 = clk::now();
    // ---- 5. indexes and orders
    slot_of_.reserve(slot_of_.n + m);
    wp.run(nch, [&](size_t c) {
        for (size_t i = m * c / nch; i < m * (c + 1) / nch; i++) slot_of_.put_new_concurrent(th[keep[i]], (uint32_t)(s0 + i));
    });
    slot_of_.n += m;
    for (size_t s = s0; s < s1; s++) {  // sessionTickets / partyTickets (a session counts a ticket once)
        const uint32_t p0 = pres_off_[s], p1 = pres_off_[s + 1];
        for (uint32_t p = p0; p < p1; p++) {
            bool dup = false;
            for (uint32_t q = p0; q < p; q++) dup |= pres_sess_[q] == pres_sess_[p];
            if (!dup) sess_slots_.add(pres_sess_[p], (uint32_t)s);
        }
        if (party_[s] != kNoParty) party_slots_.add(party_[s], (uint32_t)s);
    }
    // time order of the slots (scan order, active order) across the batch
    std::vector<uint8_t> mono(nch, 1), osort(nch, 1);
    wp.run(nch, [&](size_t c) {
        for (size_t s = std::max<size_t>(s0 + m * c / nch, 1); s < s0 + m * (c + 1) / nch; s++) {
            if (!(created_[s] > created_[s - 1] && ckey_[s] > ckey_[s - 1])) mono[c] = 0;
            if (s > s0 && ckey_[s - 1] > ckey_[s]) osort[c] = 0;
        }
    });
    for (size_t c = 0; c < nch; c++) {
        monotone_ = monotone_ && mono[c];
        order_sorted_ = order_sorted_ && osort[c];
    }
    if (!order_.empty() && ckey_[order_.back()] > ckey_[s0]) order_sorted_ = false;
    const size_t o0 = order_.size();
    order_.resize(o0 + m);
    for (size_t i = 0; i < m; i++) order_[o0 + i] = (uint32_t)(s0 + i);
    const std::vector<uint32_t> act = select(wp, m, [&](size_t i) { return is_active_[s0 + i] != 0; });
    if (!act.empty()) {
        auto before = [&](uint32_t a, uint32_t b) {  // a after b in the pinned (CreatedAt, Ticket) order
            return created_[a] > created_[b] || (created_[a] == created_[b] && tk(a) > tk(b));
        };
        bool sorted = active_sorted_;
        if (sorted && !active_list_.empty() && before(active_list_.back(), (uint32_t)(s0 + act[0]))) sorted = false;
        std::atomic<bool> unsorted{false};
        const size_t na = act.size();
        wp.run(nch, [&](size_t c) {
            for (size_t j = std::max<size_t>(na * c / nch, 1); j < na * (c + 1) / nch; j++)
                if (before((uint32_t)(s0 + act[j - 1]), (uint32_t)(s0 + act[j]))) { unsorted = true; return; }
        });
        active_sorted_ = sorted && !unsorted;
        const size_t a0 = active_list_.size();
        active_list_.resize(a0 + na);
        for (size_t j = 0; j < na; j++) active_list_[a0 + j] = (uint32_t)(s0 + act[j]);
    }
    n_live_ += (uint32_t)m;
    index_dirty_ = true;
    ph[4] = ms_since(t0);
    return true;
}

}  // namespace nkm
