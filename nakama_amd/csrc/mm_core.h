// nakama_amd/csrc/mm_core.h — host side of the MI355X matchmaker.
//
// `Core` mirrors LocalMatchmaker (server/matchmaker.go:185-212): the ticket
// maps become a slot-indexed SoA store whose hot columns live in HBM
// (mm_device.h), each ticket's query is compiled once at Add/Insert into a
// clause list shared by every ticket with the same compiled signature, and
// Process() runs the interval pass as batches of device searches followed by
// an exact replay of processDefault's greedy grouping.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <exception>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <unordered_map>
#include <vector>

#include "../../include/nakama_cluster.h"
#include "../../include/nakama_mm.h"
#include "mm_device.h"
#include "mm_handle.h"
#include "qcompile.h"
#include "termmatch.h"
#include "range_walk.h"
#include "replay_core.h"
#include "strstore.h"

namespace nkm {

hipError_t launch_search(const DStore& st, const DGroup* d_groups, int n_groups, DHit* d_out, uint8_t* d_rev,
                         DGroupResult* d_res, hipStream_t stream, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr,
                         int kinds = 3);
hipError_t launch_rpack(const DStore& st, const DSmallRow* d_rows, uint32_t n_rows, uint8_t* d_obuf, const PackLayout& L,
                        hipStream_t stream, hipEvent_t ev0, hipEvent_t ev1);
hipError_t launch_rsmall(const DStore& st, const DGroup* d_groups, const uint32_t* d_rows, uint32_t n_rows, DHit* d_out,
                         uint8_t* d_rev, uint32_t* d_pm, DGroupResult* d_res, hipStream_t stream, hipEvent_t ev0,
                         hipEvent_t ev1);
int small_src_max();
hipError_t launch_clear_alive(uint8_t* d_alive, const uint32_t* d_slots, uint32_t n, hipStream_t stream,
                              uint8_t value = 0);
hipError_t launch_pairs(const DStore& st, const uint32_t* d_pairs, uint32_t n, uint8_t* d_out, hipStream_t stream);
// enum_kernel: d_base == nullptr -> the count pass (2 words per item into
// d_cnt); else the write pass (entries as word pairs, group ends + e0).
hipError_t launch_enum(const DEnumRow* d_rows, const DEnumHit* d_hits, const DEnumItem* d_items, uint32_t n_items,
                       uint32_t* d_cnt, const uint64_t* d_base, uint32_t e0, uint32_t* d_ents, uint32_t* d_off,
                       hipStream_t stream, bool slots = false);
int var_k_capacity();
hipError_t launch_scan(const DStore& st, const DGroup* d_chunks, int n_chunks, DHit* d_scratch, DGroupResult* d_cres,
                       hipStream_t stream, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// cell_scan_kernel (ranks of every chunk in its search, one workgroup per
// search: d_ranges = [first cell, end cell) pairs) then stitch_kernel.
hipError_t launch_pack_slots(const DHit* d_out, uint64_t n, uint32_t* d_slots, const DGroup* d_groups,
                             const DGroupResult* d_res, int n_whole, DHit* d_last, hipStream_t stream);
hipError_t launch_stitch(const DChunkMap* d_map, int n_chunks, const DGroupResult* d_cres, const uint32_t* d_ranges,
                         int n_searches, uint32_t* d_offs, const DHit* d_scratch, DHit* d_out, hipStream_t stream);
int scan_chunk_len();
// gen: some signature is not term-only (the clause-loop instantiation)
hipError_t launch_mscan(const DStore& st, const DMScan& ms, const DMSig* d_sigs, const DClause* d_mcl, uint32_t* d_scratch,
                        DGroupResult* d_cres, bool gen, hipStream_t stream, hipEvent_t ev0 = nullptr,
                        hipEvent_t ev1 = nullptr);
// hashed multi-signature scan (ms.hmask != 0): d_blob = DMSig[n_sigs], u64
// output word offsets[n_sigs], then at mscan_hash_table_off the cuckoo table
// (DMHashEntry[hmask + 1]); d_work sized by mscan_hash_work_words
// phases: kMHashEval runs mscan_hash_kernel over chunks [c_lo, c_hi) (a
// row-sharded rank's block), kMHashPlace mscan_base + mscan_place over every
// chunk (after the blocks' scratch and counts were all-gathered)
hipError_t launch_mscan_hash(const DStore& st, const DMScan& ms, const void* d_blob, uint32_t* d_work,
                             DGroupResult* d_cres, uint32_t* d_out32, hipStream_t stream, hipEvent_t ev0 = nullptr,
                             hipEvent_t ev1 = nullptr, int phases = kMHashEval | kMHashPlace, uint32_t c_lo = 0,
                             uint32_t c_hi = UINT32_MAX);
// word offset of the counts in d_work (the chunks' scratch comes first: chunk c at c * ms.chunk)
uint64_t mscan_hash_counts_word(const DMScan& ms);
uint64_t mscan_hash_work_words(const DMScan& ms);
size_t mscan_hash_table_off(uint32_t n_sigs);
size_t mscan_hash_blob_bytes(uint32_t n_sigs, uint32_t cap, uint32_t dsize);
int mscan_hash_chunk_len(bool contig);
int mscan_chunk_len(uint32_t n_sigs);
int mscan_max_sigs();
int mscan_max_fields();
int mscan_max_clauses();
// range batches (range_walk.h): the pools' candidates sorted by (value, source
// position), then the bound queries; see mm_kernels.hip
hipError_t launch_rsrc(const DStore& st, const DRangePool* d_pools, uint32_t max_pad, const DRangeTile* d_tiles,
                       uint32_t n_tiles, const uint32_t* d_blk_pool, uint32_t n_elems, int64_t* d_key[2],
                       uint32_t* d_pos[2], const DRangeBound* d_q, uint32_t nq, uint32_t* d_bounds, int* which,
                       hipStream_t stream, hipEvent_t ev_tile0, hipEvent_t ev_tile1, const hipEvent_t* ev_merge,
                       int max_merge, int* n_merge);
hipError_t launch_rsrc_bounds(const DRangePool* d_pools, const int64_t* d_key, const DRangeBound* d_q, uint32_t nq,
                              uint32_t* d_bounds, hipStream_t stream);

struct DeviceError {
    hipError_t err;
    const char* expr;
    int line;
};
#define NKM_HIP(x)                                                        \
    do {                                                                  \
        hipError_t e__ = (x);                                             \
        if (e__ != hipSuccess) throw ::nkm::DeviceError{e__, #x, __LINE__}; \
    } while (0)

// Growable device array.
template <class T>
struct DevArray {
    T* p = nullptr;
    size_t cap = 0;
    void reserve(size_t n, bool keep = true);
    void release();
    ~DevArray() { release(); }
};

// Pinned host staging buffer.
template <class T>
struct PinnedArray {
    T* p = nullptr;
    size_t cap = 0;
    void reserve(size_t n);
    void release();
    ~PinnedArray() { release(); }
};

// Resizes with 25% headroom once the capacity is exceeded: a pass's arrays
// settle at the first pass's size plus a margin instead of reallocating (and
// page-faulting a fresh copy) on a later pass a few percent larger.
template <class V>
inline void grow_to(V& v, size_t n) {
    if (n > v.capacity()) v.reserve(n + n / 4);
    v.resize(n);
}

struct Presence {
    std::string user_id, session_id, username, node;
};

// One compiled signature: clauses + the searching ticket's filters.  Tickets
// whose searches are identical share it (and share one device search).
struct Sig {
    uint32_t clause_off = 0;
    uint16_t n_clauses = 0;
    uint8_t qkind = 0;
    bool var_score = false;
    int32_t tmin = 0, tmax = 0;
    uint32_t tparty = kNoParty;
    int64_t ub_key = INT64_MAX;
    uint16_t n_fields = 0;  // distinct field columns the clauses read
    std::vector<std::pair<uint16_t, uint32_t>> must_terms;  // candidate posting lists
    // the only MUST term's posting key (field << 32 | term) when there is
    // exactly one, else UINT64_MAX: source_of reads no term list then
    uint64_t must_key1 = UINT64_MAX;
    uint64_t must_fmask = 0;  // bit f: a MUST keyword term on field f (f >= 63: bit 63)
    // every clause score is a multiple of 2^-20 below 2^20 in magnitude: any
    // sum of them is exact in double, whatever the order (top-tier lists)
    bool exact_scores = false;
    // a range-source search (range_walk.h): one MUST keyword term (must_terms[0],
    // its pool) and numeric range clauses on this one other field, at least one
    // MUST; kNoRange otherwise
    static constexpr uint16_t kNoRange = 0xFFFF;
    uint16_t rs_field = kNoRange;
    uint8_t rs_nrange = 0;  // its range clauses
};

// Moved on by every failed pass of any handle (Core::reset_pass_scratch).
inline std::atomic<uint64_t> g_scratch_epoch{0};

// A worker thread's per-slot flags for the parallel walks (selected this
// batch, Intervals increment pending): zero between tasks; re-zeroed whole
// when the handle's scratch epoch moved on (a pass threw midway).
struct TlFlags {
    std::vector<uint8_t> sel, proc;
    uint64_t epoch = 0;
    void ready(size_t n, uint64_t cur_epoch) {
        if (epoch != cur_epoch) {
            sel.assign(sel.size(), 0);
            proc.assign(proc.size(), 0);
            epoch = cur_epoch;
        }
        if (sel.size() < n) sel.resize(n, 0);
        if (proc.size() < n) proc.resize(n, 0);
    }
};

// Persistent host workers for the pass's data-parallel host phases (pool
// replay, post-pass bookkeeping): run(n, fn) calls fn(0..n-1) over the
// workers and the caller, and returns when all n tasks are done.
class WorkPool {
public:
    // cpus: optional placement for the workers (worker i -> cpus[i % size]);
    // else `area`: every worker may run on any of those CPUs (none: anywhere).
    explicit WorkPool(unsigned n_threads, const std::vector<int>& cpus = {}, const std::vector<int>& area = {}) {
        for (unsigned i = 0; i + 1 < n_threads; i++) {
            const int cpu = cpus.empty() ? -1 : cpus[i % cpus.size()];
            th_.emplace_back([this, cpu, area] {
                if (cpu >= 0) pin(cpu);
                else if (!area.empty()) pin_set(area);
                loop();
            });
        }
    }
    static void pin(int cpu);
    static void pin_set(const std::vector<int>& cpus);
    ~WorkPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    unsigned size() const { return (unsigned)th_.size() + 1; }
    // A pass issues a few dozen short jobs back to back: after a job a worker
    // spins on the generation word (spin_window) before it sleeps on the condition
    // variable, and the caller spins on the done count before it sleeps, so a
    // job inside a pass starts and ends without futex wake-ups (tens of
    // microseconds each across 15 threads).
    void run(size_t n, const std::function<void(size_t)>& fn) {
        if (n == 0) return;
        if (n == 1 || th_.empty()) {
            for (size_t i = 0; i < n; i++) fn(i);
            return;
        }
        // A job is shared with the workers: one that wakes late only sees an
        // exhausted counter and never touches fn.
        auto job = std::make_shared<Job>(&fn, n);
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = job;
            gen_.fetch_add(1, std::memory_order_release);
        }
        if (sleepers_.load(std::memory_order_acquire) > 0) cv_.notify_all();
        work(*job);
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t k = 0; job->done.load(std::memory_order_acquire) != n; k++) {
            if ((k & 255) == 255 && std::chrono::steady_clock::now() - t0 > spin_window()) {
                std::unique_lock<std::mutex> lk(m_);
                done_cv_.wait(lk, [&] { return job->done.load() == n; });
                break;
            }
            relax();
        }
        {
            std::lock_guard<std::mutex> lk(m_);
            job_.reset();
        }
        // Workers that went to sleep during a long, uneven job (C3's walks
        // leave most of them idle for milliseconds) are woken now to spin for
        // the next job: a pass's next job then starts without a futex wake-up
        // per worker on its critical path.
        if (sleepers_.load(std::memory_order_acquire) > 0) {
            {
                std::lock_guard<std::mutex> lk(m_);
                wake_.fetch_add(1, std::memory_order_release);
            }
            cv_.notify_all();
        }
        // a task's exception, rethrown on the caller once every task is done
        // (no worker is still inside fn, whose captures may be on this stack)
        if (job->failed.load(std::memory_order_acquire)) std::rethrow_exception(job->err);
    }

private:
    // spin window: long enough to bridge the host code between a pass's
    // back-to-back jobs, short enough that idle workers do not steal cycles
    // (SMT siblings) from a long job's busy ones (30 us; 200 us measured
    // slower on C3, profiles r03h)
    static std::chrono::microseconds spin_window() { return std::chrono::microseconds{30}; }
    static inline void relax() { __builtin_ia32_pause(); }
    struct Job {
        Job(const std::function<void(size_t)>* f, size_t count) : fn(f), n(count) {}
        const std::function<void(size_t)>* fn;
        const size_t n;
        std::atomic<size_t> next{0}, done{0};
        std::atomic<bool> failed{false};
        std::mutex err_mu;
        std::exception_ptr err;  // the first task exception (under err_mu)
    };
    void work(Job& j) {
        size_t mine = 0;
        for (;;) {
            const size_t i = j.next.fetch_add(1);
            if (i >= j.n) break;
            try {
                (*j.fn)(i);
            } catch (...) {
                std::lock_guard<std::mutex> lk(j.err_mu);
                if (!j.err) j.err = std::current_exception();
                j.failed.store(true, std::memory_order_release);
            }
            mine++;
        }
        if (mine && j.done.fetch_add(mine) + mine == j.n) {
            std::lock_guard<std::mutex> lk(m_);
            done_cv_.notify_all();
        }
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            // spin for the next job of the same pass, then sleep
            const auto t0 = std::chrono::steady_clock::now();
            for (uint32_t k = 0; gen_.load(std::memory_order_acquire) == seen; k++) {
                if ((k & 255) == 255 && std::chrono::steady_clock::now() - t0 > spin_window()) break;
                relax();
            }
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> lk(m_);
                if (!quit_ && gen_.load() == seen) {
                    const uint64_t w = wake_.load();
                    sleepers_.fetch_add(1);
                    cv_.wait(lk, [&] { return quit_ || gen_.load() != seen || wake_.load() != w; });
                    sleepers_.fetch_sub(1);
                }
                if (quit_) return;
                if (gen_.load() == seen) continue;  // woken ahead of a job: spin for it
                seen = gen_.load();
                j = job_;
            }
            if (j) work(*j);
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::shared_ptr<Job> job_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> sleepers_{0};
    std::atomic<uint64_t> wake_{0};
    bool quit_ = false;
};

// key id -> set of slots, optimised for the common one-slot case
// (sessionTickets / partyTickets, matchmaker.go:201-204).  `first` may hold a
// dead slot (a ticket a pass retired without touching this map: slots are
// never reused before compaction rebuilds it), which counts as absent; `more`
// holds live slots only (erase keeps it exact).
struct SlotSets {
    std::vector<uint32_t> first;
    std::unordered_map<uint32_t, std::vector<uint32_t>> more;
    const std::vector<uint8_t>* live = nullptr;  // the store's live_ (set by Core)
    bool alive(uint32_t s) const { return s != kNoSlot && (*live)[s]; }
    void ensure(uint32_t key) { if (key >= first.size()) first.resize(key + 1, kNoSlot); }
    size_t count(uint32_t key) const {
        if (key >= first.size()) return 0;
        const size_t n = alive(first[key]) ? 1 : 0;
        if (more.empty()) return n;
        auto it = more.find(key);
        return n + (it == more.end() ? 0 : it->second.size());
    }
    void add(uint32_t key, uint32_t slot) {
        ensure(key);
        if (!alive(first[key])) { first[key] = slot; return; }
        more[key].push_back(slot);
    }
    void erase(uint32_t key, uint32_t slot) {
        if (key >= first.size() || first[key] == kNoSlot) return;
        if (more.empty()) {  // common case: every key holds one slot
            if (first[key] == slot) first[key] = kNoSlot;
            return;
        }
        auto it = more.find(key);
        if (first[key] == slot || !alive(first[key])) {
            if (first[key] != slot && it != more.end()) {  // a stale first: the slot may sit in more
                auto& v = it->second;
                for (size_t i = 0; i < v.size(); i++)
                    if (v[i] == slot) { v[i] = v.back(); v.pop_back(); break; }
            }
            if (it == more.end() || it->second.empty()) {
                first[key] = kNoSlot;
            } else {
                first[key] = it->second.back();
                it->second.pop_back();
            }
        } else if (it != more.end()) {
            auto& v = it->second;
            for (size_t i = 0; i < v.size(); i++)
                if (v[i] == slot) { v[i] = v.back(); v.pop_back(); break; }
        } else {
            return;
        }
        if (it != more.end() && it->second.empty()) more.erase(it);
    }
    std::vector<uint32_t> list(uint32_t key) const {
        std::vector<uint32_t> v;
        if (key >= first.size()) return v;
        if (alive(first[key])) v.push_back(first[key]);
        auto it = more.find(key);
        if (it != more.end()) v.insert(v.end(), it->second.begin(), it->second.end());
        return v;
    }
    void clear() { first.clear(); more.clear(); }
};

struct PostingRange {
    uint32_t off = 0, len = 0, head = 0;  // head: first entry possibly alive
};

// The posting-list directory, (field << 32 | term) -> PostingRange: one flat
// open-addressed table (linear probing, power-of-two size, at most half
// full): a lookup reads one slot instead of unordered_map's bucket + node.
// Keys are scrambled in blocks of eight: eight consecutive dictionary ids of
// a field sit in consecutive slots (C5's buckets, interned in arrival order
// and looked up in row order, then read a few lines per 64 rows), the blocks
// spread over the table so no field's ids form one long probe run.  A fully
// scrambling hash measured +0.8 ms on C5's assembly
// (profiles/r05/r05ae_c5_pruns.txt).  Keys never equal kEmpty (fields fit 16
// bits).  Iteration visits the live slots in table order.
struct PostingMap {
    static constexpr uint64_t kEmpty = ~0ull;
    struct Slot {
        uint64_t first = kEmpty;
        PostingRange second;
    };
    std::vector<Slot> slots;
    size_t used = 0;

    static size_t mix(uint64_t k) {
        uint64_t b = k >> 3;
        b ^= b >> 33;
        b *= 0xff51afd7ed558ccdull;
        b ^= b >> 33;
        return (size_t)((b << 3) | (k & 7));
    }
    void clear() {
        for (Slot& s : slots) s = Slot{};
        used = 0;
    }
    PostingRange* find(uint64_t k) {
        if (slots.empty()) return nullptr;
        const size_t m = slots.size() - 1;
        for (size_t i = mix(k) & m;; i = (i + 1) & m) {
            if (slots[i].first == k) return &slots[i].second;
            if (slots[i].first == kEmpty) return nullptr;
        }
    }
    const PostingRange* find(uint64_t k) const { return const_cast<PostingMap*>(this)->find(k); }
    PostingRange& operator[](uint64_t k) {
        if ((used + 1) * 2 > slots.size()) grow();
        const size_t m = slots.size() - 1;
        size_t i = mix(k) & m;
        while (slots[i].first != k && slots[i].first != kEmpty) i = (i + 1) & m;
        if (slots[i].first == kEmpty) {
            slots[i].first = k;
            used++;
        }
        return slots[i].second;
    }
    template <class F> void for_each(F&& f) {
        for (Slot& s : slots)
            if (s.first != kEmpty) f(s.second);
    }

private:
    void grow() {
        std::vector<Slot> old;
        old.swap(slots);
        slots.assign(std::max<size_t>(64, old.size() * 2), Slot{});
        used = 0;
        for (Slot& s : old)
            if (s.first != kEmpty) (*this)[s.first] = s.second;
    }
};

// Identity of a signature (the sig_idx_ hash): query kind, the searching
// ticket's filters and the compiled clauses.
uint64_t sig_clause_hash(const DClause* dc, size_t n);
uint64_t sig_hash(uint64_t clause_hash, uint8_t kind, int32_t mn, int32_t mx, uint32_t party);

// Builtin document fields (MapMatchmakerIndex, matchmaker.go:1026-1040).
enum BuiltinField : uint16_t { F_TICKET = 0, F_MIN = 1, F_MAX = 2, F_PARTY = 3, F_CREATED = 4, F_NBUILTIN = 5 };


// Matched (or candidate) groups of a pass as a flat CSR of (slot, presence
// index) entries: group g = ents[off[g], off[g+1]).
// (DefaultInitAlloc: strstore.h)
template <class T>
using UVec = std::vector<T, DefaultInitAlloc<T>>;

// One group entry: (ticket slot, presence index).  Trivially default
// constructible (see DefaultInitAlloc); converts from the replay's pairs.
struct GroupEntry {
    uint32_t first;
    int second;
    GroupEntry() = default;
    constexpr GroupEntry(uint32_t a, int b) : first(a), second(b) {}
    GroupEntry(const std::pair<uint32_t, int>& p) : first(p.first), second(p.second) {}
};
static_assert(std::is_trivially_default_constructible<GroupEntry>::value, "GroupEntry: no zero-fill on resize");

struct GroupList {
    using Entry = GroupEntry;
    UVec<uint32_t> off{0};
    UVec<Entry> ents;
    size_t size() const { return off.size() - 1; }
    bool empty() const { return off.size() == 1; }
    template <class It>
    void push(It b, It e) {
        ents.insert(ents.end(), b, e);
        off.push_back((uint32_t)ents.size());
    }
    void push(const std::vector<std::pair<uint32_t, int>>& g) { push(g.begin(), g.end()); }
    void clear() {
        off.resize(1);
        ents.clear();
    }
    void reserve_more(size_t groups, size_t entries) {  // geometric, so repeated calls stay linear
        if (off.capacity() < off.size() + groups) off.reserve(std::max(off.size() + groups, 2 * off.capacity()));
        if (ents.capacity() < ents.size() + entries) ents.reserve(std::max(ents.size() + entries, 2 * ents.capacity()));
    }
    const Entry* begin(size_t g) const { return ents.data() + off[g]; }
    const Entry* end(size_t g) const { return ents.data() + off[g + 1]; }
    size_t len(size_t g) const { return off[g + 1] - off[g]; }
};

struct SrcChoice {  // the posting list a search streams, when it has one
    bool has_term = false;
    uint16_t field = 0;
    uint32_t term = 0;
};

// RevThreshold (matchmaker.go:244-248, matchmaker_process.go:31-46): with
// RevPrecision and RevThreshold > 0, an active pass starts a timer of
// IntervalSec * RevThreshold seconds; the rows examined after it fired skip
// every reverse (validateMatch) check.  Pin: the timer counts as fired at the
// first row examined once the duration has elapsed (a zero duration fires at
// the first row; Go's channel select may see it a little later).
struct RevTimer {
    bool armed = false, fired = false;
    double limit_ms = 0;
    std::chrono::steady_clock::time_point t0;
    RevTimer(bool arm, double seconds) : armed(arm), limit_ms(seconds * 1e3), t0(std::chrono::steady_clock::now()) {}
    bool check() {
        if (armed && !fired)
            fired = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() >= limit_ms;
        return fired;
    }
};

struct PassStats {
    int full_lists = 0;  // variable-score searches run as full lists (host-sorted)
    int tier_lists = 0;  // variable-score searches run as top-tier lists (search_kernel path 2)
    // per query-eval kernel: 0 search_kernel, 1 scan_kernel, 2 mscan_kernel, 3 rsmall_kernel,
    // 4 rsrc_merge_kernel, 5 rsrc_tile_kernel (range batches)
    static constexpr int kKernels = 6;
    double k_ms[kKernels] = {};         // HIP-event time of the launches
    bool mhash = false;                 // a batch's mscan ran hashed (mscan_hash_kernel)
    bool rpack = false;                 // kernel 3's launches were packed batches (rpack_kernel)
    int64_t k_bytes[kKernels] = {};     // algorithmic bytes
    int k_launches[kKernels] = {};
    int64_t pair_evals = 0;
    int64_t pairs_decided = 0;  // rows that searched x their search's source (mm_matched.pairs_decided)
    double eval_ms() const {
        double t = 0;
        for (int k = 0; k < kKernels; k++) t += k_ms[k];
        return t;
    }
    int launches() const {
        int t = 0;
        for (int k = 0; k < kKernels; k++) t += k_launches[k];
        return t;
    }
    int dominant() const {  // the kernel with the most algorithmic bytes
        int d = 0;
        for (int k = 1; k < kKernels; k++)
            if (k_bytes[k] > k_bytes[d]) d = k;
        return d;
    }
    int batches = 0;
    int refetches = 0;
    double search_ms = 0;   // host wall time of batch searches incl. H2D/D2H and stitching
    double replay_ms = 0;   // host wall time of the greedy replay
    double assemble_ms = 0; // batch assembly (rows -> searches)
    double apply_ms = 0;    // pushing the batch's selections to the device alive mask
    int parallel_batches = 0;
    double par_bucket_ms = 0, par_work_ms = 0, par_merge_ms = 0;  // parallel replay phases
    double par_task_max_ms = 0;
    // finer split (NKM_PROFILE): run_batch's host prep + launches, the
    // overlapped host work, the wait for the device, result accounting and
    // wiring, the hit-list copies; replay_parallel's gathers and the walk job
    double rb_prep_ms = 0, rb_overlap_ms = 0, rb_wait_ms = 0, rb_post_ms = 0, rb_lists_ms = 0;
    int mhash_respec = 0;  // counts-only hashed scans re-run in full (a list not proven)
    int mscan_lists = 0, lists_proven = 0;  // mscan lists placed / proven equal to their rows (not downloaded)
    double par_gather_ms = 0, par_job_ms = 0, par_clear_ms = 0;
    double asm_count_ms = 0, asm_scatter_ms = 0;  // assemble_parallel's two sweeps over the rows
    double prologue_ms = 0;  // process_default before its first batch (sel / dec, the active rows)
    uint64_t par_rows = 0, par_hits = 0;
};

// Algorithmic HBM bytes of one search (DESIGN.md "Roofline"): every scanned
// candidate reads its 4-B slot id and 1-B alive flag; candidates still in the
// index also read Min/MaxCount (8 B), the party id when the searching ticket
// has a party (4 B), and one 8-B value + 1-B kind per field column the query
// references (plus the candidate's own query descriptor and clauses for the
// RevPrecision reverse check); each emitted hit writes 16 B.
inline int64_t search_bytes(uint16_t n_fields, const DGroup& d, const DGroupResult& r) {
    int64_t per_live = 8 + (d.tparty != kNoParty ? 4 : 0) + 9 * (int64_t)n_fields;
    if (d.rev_slot != kNoSlot) per_live += 8 + 32 * (int64_t)d.n_clauses;
    return (int64_t)r.scanned * 5 + (int64_t)r.live * per_live + (int64_t)r.count * 16 +
           (int64_t)(sizeof(DGroup) + sizeof(DGroupResult));
}

// Set by the multi-device front (mm_multi.cpp) around the creation of its
// sub-handles: the number of Cores that share this process's host cores.
extern thread_local unsigned g_create_share;

class Core : public Handle {
public:
    explicit Core(const mm_config& cfg);
    ~Core() override;

    int add(const mm_ticket& t) override;
    int insert(const mm_ticket* ts, int32_t n) override;
    int extract(mm_extract_list* out) override;
    void free_extract(mm_extract_list* out) override;
    int remove_session(const std::string& sid, const std::string& ticket) override;
    int remove_session_all(const std::string& sid) override;
    int remove_party(const std::string& pid, const std::string& ticket) override;
    int remove_party_all(const std::string& pid) override;
    int remove_all(const std::string& node) override;
    int remove(const char* const* tickets, int32_t n) override;
    int process(mm_matched* out) override;
    int process_commit(const int32_t* offs, const mm_entry_ref* ents, int32_t n_groups, mm_matched* out) override;
    void free_matched(mm_matched* out) override;
    int32_t ticket_count() override;
    int32_t active_count() override;
    int32_t debug_hits(const std::string& ticket, const char** tk, double* sc, int32_t cap) override;
    int32_t session_ticket_count(const std::string& sid) override;
    int32_t party_ticket_count(const std::string& pid) override;
    int32_t find_tickets(const char* const* ids, int32_t n, uint8_t* found) override;

    void pause() override { active_flag_ = false; }
    void resume() override { active_flag_ = true; }
    void stop() override { stopped_ = true; }
    const char* last_error() const override { return last_error_.c_str(); }
    void set_error(const std::string& e) override { last_error_ = e; }
    void set_pass_hook(void (*fn)(void*), void* ctx) override {
        std::lock_guard<std::mutex> lk(mu_);
        pass_hook_ = fn;
        pass_hook_ctx_ = ctx;
    }
    int drain_removed(mm_str_list* out) override;
    void free_str_list(mm_str_list* out) override;
    int set_row_shard(int world, int rank, mm_allgather_fn fn, void* ctx) override;
    int set_row_shard_rccl(int world, int rank, const uint8_t* uid, int len) override;

private:
    friend struct Replay;
    struct Ticket;

    // ---- mutations that arrive while a pass runs ----
    // Process() holds the store lock only to take its snapshot and to finish;
    // a mutator called in between validates against the store plus the
    // mutations already queued (the "effective" state), returns its status,
    // and queues itself; the queue is applied in arrival order when the pass
    // ends, before its completeness re-check (matchmaker.go:309-343), so a
    // group that lost a ticket is dropped exactly as the reference drops it.
    struct OwnedTicket {  // an mm_ticket's strings, owned (callers' memory is not retained)
        std::string ticket, session_id, party_id, query, node;
        int32_t min_count = 0, max_count = 0, count_multiple = 1, intervals = 0;
        int64_t created_at = 0;
        std::vector<Presence> presences;
        std::vector<std::pair<std::string, std::string>> sprops;
        std::vector<std::pair<std::string, double>> nprops;
        explicit OwnedTicket(const mm_ticket& t);
        struct View {  // an mm_ticket over this record (valid while it lives)
            mm_ticket t{};
            std::vector<mm_presence> p;
            std::vector<mm_str_prop> s;
            std::vector<mm_num_prop> n;
        };
        void view(View& v) const;
    };
    enum PendKind { P_ADD, P_INSERT, P_REMOVE_SESSION, P_REMOVE_SESSION_ALL, P_REMOVE_PARTY, P_REMOVE_PARTY_ALL,
                    P_REMOVE_ALL, P_REMOVE };
    struct PendingOp {
        PendKind kind;
        std::vector<OwnedTicket> tickets;  // P_ADD / P_INSERT
        std::vector<CompiledQuery> cqs;
        std::vector<uint8_t> ok;
        std::string a, b;                  // session / party / node, ticket
        std::vector<std::string> ids;      // P_REMOVE
    };
    struct PendTk {  // a ticket's effective state while a pass runs
        bool alive = false;
        std::string session_id, party_id, node;
        std::vector<std::string> sessions;  // distinct, presence order
    };
    bool pass_running_ = false;
    std::vector<PendingOp> pending_;
    std::unordered_map<std::string, PendTk> pend_tk_;
    std::unordered_map<std::string, int> pend_sess_, pend_party_;  // ticket-count deltas
    PendTk* eff_ticket(const std::string& id);
    void eff_remove(PendTk& t);
    void eff_add(const OwnedTicket& t);
    int eff_sess_count(const std::string& sid);
    int eff_party_count(const std::string& pid);
    void apply_pending();  // under mu_, at the end of a pass
    void (*pass_hook_)(void*) = nullptr;  // tests: called once per pass, between the searches and the finish
    void* pass_hook_ctx_ = nullptr;
    // tickets that left the matchmaker since the last drain (Remove*, replaced
    // ids, matched): the Go shim drops its delivery entries with them
    bool track_removed_ = false;
    std::vector<std::string> removed_ids_;
    std::unordered_map<const char* const*, std::vector<std::string>*> str_lists_;  // outstanding drains
    std::mutex pair_mu_;     // Replay::pair_slow from pool workers
    std::mutex process_mu_;  // one pass at a time (the ticker); lock order process_mu_ -> mu_
    int remove_session_locked(const std::string& sid, const std::string& ticket);
    int remove_session_all_locked(const std::string& sid);
    int remove_party_locked(const std::string& pid, const std::string& ticket);
    int remove_party_all_locked(const std::string& pid);
    int remove_all_locked(const std::string& node);
    int remove_locked(const std::vector<std::string>& ids);

    // ---- store ----
    int add_locked(const mm_ticket& t, uint32_t sig, bool from_insert);
    // Signature of a ticket's search, through a cache keyed by (query text,
    // MinCount, MaxCount): a repeated query skips the compile.  -1 - status
    // when the query does not compile.
    int64_t sig_cached(const mm_ticket& t);
    Dict qtext_;                    // cached query texts
    std::vector<int32_t> qstatus_;  // per cached text: compile_query's status
    struct QSig { uint32_t q; int32_t mn, mx; uint32_t sig; };
    std::vector<QSig> qsig_;
    HashIndex qsig_idx_;
    Dict prop_key_;                 // property name -> field ("properties." + name)
    std::vector<uint16_t> prop_field_;
    uint16_t prop_field(std::string_view key);
    uint16_t field_of(const std::string& name);
    uint32_t sig_of(const CompiledQuery& cq, int32_t mn, int32_t mx, uint32_t party);
    static void sig_describe(Sig& s, const std::vector<DClause>& dc, const CompiledQuery& cq, int32_t mn, int32_t mx,
                             uint32_t party);
    template <class Get>
    void commit_new_sigs(WorkPool& wp, size_t nt, const std::vector<int64_t>& tfound, const std::vector<uint64_t>& thash,
                         std::vector<Sig>& tsig, std::vector<uint32_t>& tsg, Get get);
    uint32_t sig_commit(Sig&& s, const DClause* dc, size_t n, uint64_t hash, bool materialize);
    bool sig_eq(uint32_t id, uint8_t kind, int32_t mn, int32_t mx, uint32_t party, const DClause* dc, size_t n) const;
    void materialize_fields();
    // Insert of a large batch on the host workers (mm_insert.cpp); false:
    // the batch takes the per-ticket path (nothing was changed)
    bool insert_bulk(const mm_ticket* ts, int32_t n, double* phase_ms);
    uint32_t termset_of(const HostClause& c);  // interned regexp/wildcard/fuzzy matcher
    void refresh_termsets();                   // extends accepted sets over new dictionary terms, uploads
    void set_field(uint16_t f, uint32_t slot, uint8_t kind, int64_t val);
    // the ticket leaves the index and the maps; quiet: not reported by
    // mm_drain_removed (a replaced id lives on, a matched ticket is in the pass result)
    void kill_slot(uint32_t slot, bool device_cleared = false, bool quiet = false);
    void maybe_compact();
    void compact();
    bool live(uint32_t slot) const { return live_[slot] != 0; }
    int64_t slot_of_ticket(std::string_view t) const;

    // ---- device ----
    void sync_device();     // uploads, index build, pending deletes
    void build_index();     // scan order + posting lists
    void ensure_field_on_device(uint16_t f);
    DStore dstore() const;

    // ---- pass ----
    int process_default(GroupList& groups, UVec<uint32_t>& expired,
                        PassStats& st);
    int process_custom(GroupList& cands, UVec<uint32_t>& expired,
                       PassStats& st);
    void finish_pass(const UVec<uint32_t>& expired, GroupList& groups, bool disjoint);
    // selected: the groups' tickets were deleted from the search index during
    // the pass (processDefault), so members of a dropped group leave it
    void finish_pass_serial(GroupList& groups, bool selected);
    void fill_matched(const GroupList& groups, mm_matched* out, bool cands);
    bool finish_fill_fast(const UVec<uint32_t>& expired, GroupList& groups, mm_matched* out, bool mutated);
    void choose_source(const Sig& s, DGroup& g, SrcChoice* ch = nullptr);
    void source_of(const Sig& s, DGroup& g, SrcChoice* ch = nullptr) const;
    void source_of_key1(uint64_t key1, DGroup& g) const;
    struct ParPlan {  // a batch's pools (plan_parallel), bucketed while its searches run
        bool ok = false;
        size_t ng = 0;
        std::vector<uint32_t> search_pool;  // per search
        std::vector<uint32_t> pool_off;     // CSR: pool p's batch rows are pool_rows[pool_off[p], pool_off[p+1])
        std::vector<uint32_t> pool_rows;    // ascending per pool
        std::vector<uint8_t> self_rows;     // per pool: every row carries its own search's terms
        std::vector<uint32_t> pool_key1;    // one key field: each pool's term
        bool runs = false;                  // every pool is one run of the batch, pools in row order
    };
    // replay_runs: one task's output (its rows' groups in row order)
    struct alignas(128) RunOut {
        std::vector<uint32_t> gend;  // per group: the end of its entries in `ents`
        std::vector<uint32_t> gT;    // per group: its searching ticket
        std::vector<std::pair<uint32_t, int>> ents;
        UVec<uint32_t> expired;
        uint64_t hits = 0, pairs = 0;
        double ms = 0.0;
    };
    std::vector<RunOut> run_outs_;
    bool replay_runs(const ParPlan& P, std::vector<BGroup>& bg, const UVec<uint32_t>& brow,
                     const UVec<uint32_t>& brow_group, std::vector<uint8_t>& sel, GroupList& out_groups,
                     UVec<uint32_t>& expired, UVec<uint32_t>& newly, PassStats& stats, bool rev,
                     uint32_t* min_stop, const std::function<BGroup&(uint32_t)>* view);
    struct RowRec {  // a batch row's outcome in a parallel replay (indexed by batch row)
        uint32_t ent, len, task;  // its group's entries: task_ents_[task][ent, ent + len)
        uint8_t matched, expired, processed, pad;
    };
    std::vector<RowRec> row_recs_;
    std::vector<std::vector<std::pair<uint32_t, int>>> task_ents_;
    std::vector<uint32_t> pool_remap_;  // dictionary id -> pool (one-field pool keys)
    std::unique_ptr<std::atomic<uint32_t>[]> pool_first_;  // dictionary id -> first search with it
    size_t pool_first_cap_ = 0;
    UVec<uint32_t> pool_cuts_;  // pipelined merge: [pool][chunk] the walk's records before the chunk's end
    std::vector<uint32_t> run_terms_;  // plan_packed_runs: per row its pool term | foreign bit
    UVec<uint32_t> pool_cnt_;            // plan_pools: [chunk][pool] row counts, then positions
    UVec<uint8_t> pool_foreign_;         // plan_pools: [chunk][pool] a row not known to self-match
    ParPlan par_plan_;
    bool plan_parallel(const std::vector<BGroup>& bg, const UVec<uint32_t>& brow,
                       const UVec<uint32_t>& brow_group, ParPlan& P, PassStats& stats);
    // plan_parallel when the batch assembly already bucketed the rows per
    // search (P.pool_off / P.pool_rows) and every row carries its own terms:
    // each search its own pool when their pool keys are pairwise distinct
    bool plan_fused(const std::vector<BGroup>& bg, const UVec<uint32_t>& brow, const UVec<uint32_t>& brow_group,
                    ParPlan& P, PassStats& stats);
    template <class SigOf, class GroupOf, class RowOf>
    bool plan_pools(size_t nsearch, SigOf sig_of, GroupOf group_of, RowOf row_of, const UVec<uint32_t>& brow,
                    ParPlan& P, PassStats& stats);
    bool replay_parallel(const ParPlan& P, std::vector<BGroup>& bg, const UVec<uint32_t>& brow,
                         const UVec<uint32_t>& brow_group, std::vector<uint8_t>& sel,
                         GroupList& out_groups,
                         UVec<uint32_t>& expired, UVec<uint32_t>& newly, PassStats& stats,
                         bool rev, uint32_t* min_stop, const std::function<BGroup&(uint32_t)>* view = nullptr);
    // ---- proven mscan lists ----
    // A hashed-scan list (term-only pool signature) always holds every batch
    // row of its search: the row is alive on the device (live, indexed, not
    // selected), carries its signature's key terms (self_match_) and its own
    // counts meet the signature's count musts.  So when the list's count
    // equals the search's batch rows, the list IS those rows; and with slots
    // in time order (monotone_: scan order = slot order = pinned order) it
    // holds them in batch order.  Such a list is not downloaded
    // (BGroup::rows_list).  NKM_LISTPROOF=0: every list is downloaded;
    // 2: downloaded and compared with the proof's claim (throws on a miss).
    int list_proof_mode_ = 1;
    // Counts-only speculation (mode 1, contiguous hashed scans): the scan
    // writes only the per-(signature, chunk) counts — no ranking into scratch,
    // no placement — since a proven list is never read.  A search whose count
    // then differs from its rows needs its list: the full scan runs again for
    // that batch and the speculation pauses for kSpecPause passes.
    // NKM_MHCOUNT=0: always the full scan.
    bool mhash_count_mode_ = true;
    uint32_t mhash_spec_pause_ = 0;
    static constexpr uint32_t kSpecPause = 16;
    // the hashed scan's direct key-grid lookup when the signatures' values
    // span small ranges (DMScan::dsize); NKM_MHGRID=0: the cuckoo table always
    bool mhash_grid_mode_ = true;
    bool row_lists_pending_ = false;  // the last batch flagged some BGroup::rows_list
    // writes every rows_list search's host list from its batch rows (a reader
    // other than the dense identity walk) and clears the flags
    void fill_row_lists(std::vector<BGroup>& bg, const UVec<uint32_t>& brow, const UVec<uint32_t>& brow_group);
    // NKM_LISTPROOF=2: the downloaded lists against the proof's claim
    void check_row_lists(const std::vector<BGroup>& bg, const UVec<uint32_t>& brow, const UVec<uint32_t>& brow_group);
    // ---- packed RevPrecision batches (rpack_kernel) ----
    // A RevPrecision batch whose every row searches a source of <= 64
    // entries: rows go to the device as 12-B DSmallRows, the lists come back
    // fixed-stride in one buffer (pack_layout), and the replay reads each row
    // through a thread-local BGroup view — no per-row search descriptors.
    struct PackBatch {
        size_t n = 0;        // rows in the batch
        size_t end = 0;      // pass rows consumed (rows[pos, end))
        int S = 8;           // list stride: the longest source, rounded up to 8 / 16 / 32 / 64
        uint64_t scanned = 0;
        uint64_t unique = 0; // distinct candidates per wave, summed (the loads a wave issues, once each)
        double live_w = 0;   // sum over rows of src_len x the row's per-live-candidate bytes
    };
    bool tier_mode_ = true;  // NKM_TIER=0: variable-score searches never return top-tier lists
    // ---- range batches (mm_range.cpp, range_walk.h) ----
    // A batch whose every row is a range-source search (Sig::rs_field) of a
    // pool on one keyword field: the pools' candidates sorted by value on the
    // device (rsrc_* kernels), every remaining row decided in one batch by
    // the min-tree walk.  false: the rows do not qualify (nothing changed).
    bool range_mode_ = true;  // NKM_RANGE=0: such batches take the hit-list path
    bool range_batch(const std::vector<uint32_t>& rows, size_t pos, GroupList& out_groups,
                     UVec<uint32_t>& expired, UVec<uint32_t>& newly, PassStats& stats);
    struct RangePoolHost {  // one pool of a range batch (kept across passes: capacity reused)
        uint32_t term = 0;
        uint16_t field = 0;
        DRangePool d{};
        std::vector<uint32_t> slot, rank, leaf_of;
        std::vector<HotRec> lhot;
        std::vector<int32_t> livl;
        RangeSrc src;
    };
    std::vector<RangePoolHost> rs_pools_;
    std::unique_ptr<std::atomic<uint8_t>[]> rs_mark_;  // per signature: claimed by a batch row (all zero between batches)
    size_t rs_mark_cap_ = 0;
    std::vector<uint32_t> rs_sig_loc_;  // signature -> its index in the batch (valid for the batch's signatures)
    std::vector<uint32_t> rs_leaf_;     // slot -> its leaf in its pool during a range batch, else kNoSlot
    // Per-slot scratch that the parallel walks keep all zero (kNoSlot) between
    // tasks — rs_mark_, rs_leaf_, pos_of_ and every worker's thread-local
    // selection / pending-Intervals flags (TlFlags).  A pass that throws
    // midway may leave entries set: reset_pass_scratch() clears the shared
    // arrays and moves g_scratch_epoch on, and each worker re-zeroes its
    // thread-local flags before it uses them again.
    void reset_pass_scratch();
    std::vector<RRange> rs_tiers_;      // the batch's signatures' tier lists
    DevArray<uint8_t> d_rblob_;         // pools, tiles, block -> pool
    PinnedArray<uint8_t> h_rblob_;
    DevArray<uint8_t> d_rq_;            // the bound queries (DRangeBound), uploaded after the sort is issued
    PinnedArray<uint8_t> h_rq_;
    DevArray<int64_t> d_rkey_[2];
    DevArray<uint32_t> d_rpos_[2], d_rbound_;
    PinnedArray<uint32_t> h_rpos_, h_rbound_;
    static constexpr int kRsrcMaxMerge = 20;
    hipEvent_t rs_ev_[2 + 2 * kRsrcMaxMerge] = {};  // the tile launch, then each merge launch
    int bulk_mode_ = 1;      // NKM_BULK: 0 = Insert per ticket, 1 = batches of >= 4096 on the workers, 2 = any batch
    bool pack_mode_ = true;  // NKM_RPACK=0: RevPrecision batches search per row (rsmall / search_kernel)
    UVec<DSmallRow> pk_tmp_;
    PinnedArray<DSmallRow> h_srows_;
    DevArray<DSmallRow> d_srows_;
    DevArray<uint8_t> d_pack_;
    PinnedArray<uint8_t> h_pack_;
    bool assemble_packed(const std::vector<uint32_t>& rows, size_t pos, size_t cap, UVec<uint32_t>& brow, PackBatch& pb);
    PackLayout run_packed(const PackBatch& pb, PassStats& stats, const std::function<void()>& overlap);
    bool plan_packed(size_t n, const UVec<uint32_t>& brow, ParPlan& P, PassStats& stats);
    int plan_packed_runs(size_t n, const UVec<uint32_t>& brow, ParPlan& P, PassStats& stats);
    std::atomic<uint32_t>* pool_first_table(size_t nd);
    std::function<BGroup&(uint32_t)> packed_view(const PackLayout& L, const UVec<uint32_t>& brow);
    // the replay over this store (mm_process.cpp's Replay: device pages and
    // pair checks), for the pool workers of replay_parallel
    ReplayView replay_view() const;
    std::unique_ptr<ReplayCore> make_replay(std::vector<uint8_t>& sel, bool rev, int max_intervals, PassStats& stats);
    std::vector<uint8_t> dec_;  // per pass: rows a parallel replay decided ahead of the pass's row pointer
    void apply_selected_to_device(const uint32_t* slots, size_t n);
    // A batch's selections reach the device alive mask before the next
    // device search (the next batch, a page, a pair check, the next pass's
    // sync_device): deferred here, flushed by flush_apply (a compaction
    // renumbers the slots and drops them: its re-upload carries the flags).
    UVec<uint32_t> apply_defer_;
    void defer_apply(UVec<uint32_t>& newly);
    void flush_apply();

    std::mutex mu_;
    mm_config cfg_;
    std::string node_;
    bool active_flag_ = true;
    bool stopped_ = false;
    std::string last_error_;
    int device_ = 0;
    hipStream_t stream_ = nullptr;
    hipEvent_t ev_[9] = {};  // start/stop of the search / scan / mscan dispatches, a marker before stitch_kernel,
                             // start/stop of the rsmall dispatch
    hipEvent_t apply_ev_ = nullptr;  // after the last asynchronous alive-flag update (h_slots_tmp_ reuse)
    bool apply_pending_ = false;
    std::unique_ptr<WorkPool> workers_;  // created on the first large pass
    unsigned host_share_ = 1;            // Cores sharing the host cores (multi handle: those on this NUMA node)
    int numa_node_ = -1;                 // the device's NUMA node (device_numa_node), -1 unknown
    WorkPool& workers();
    size_t par_min(size_t auto_min) const { return par_mode_ == 2 ? 0 : auto_min; }
    bool big_list(const std::vector<uint32_t>& v) const { return par_mode_ != 0 && v.size() >= par_min(65536); }

public:
    using Props = std::vector<std::pair<uint16_t, std::pair<uint8_t, int64_t>>>;  // (field, (kind, value))
    void doc_props(const ColdView& v, Props& out);
    // ---- host SoA (per slot) ----  (public for the replay helpers)
    Dict dict_;                       // keyword values / terms / parties
    Dict sess_dict_;                  // presence session ids (rebuilt at compaction)
    Dict party_dict_;                 // party ids (rebuilt at compaction)
    // per-pass scratch, kept across passes (no page faults on the hot path)
    std::vector<uint8_t> sel_;
    std::vector<uint32_t> rows_, list_tmp_;
    // The first batch's signature counts, taken by the pass prologue while it
    // copies the rows (nothing is selected or decided yet): per chunk of the
    // workers' split, the signatures in first-appearance order, their counts,
    // the rows and whether every row carries its own search's terms.
    // assemble_parallel uses them instead of its count sweep when its batch
    // is those rows in that split (valid: for this pass's rows).
    struct PreCount {
        bool valid = false;
        size_t n_rows = 0;
        std::vector<std::vector<uint32_t>> first, cnt;
        std::vector<size_t> n;
        std::vector<uint8_t> self;
    };
    PreCount precount_;
    UVec<uint32_t> brow_, brow_group_;  // the batch's rows and their searches (filled in full)
    UVec<uint32_t> newly_;  // slots selected by the batch (filled in full by the merges)
    GroupList pass_groups_;
    UVec<uint32_t> expired_;
    std::vector<BGroup> bg_;              // a pass's batch searches (kept: capacity reused)
    std::vector<DGroup> lg_;              // their device descriptors (Replay::lg)
    std::vector<uint32_t> lg_group_;
    std::vector<DensePool> dense_pools_;  // dense replay per pool (kept: capacity reused)
    std::vector<PoolOut> pool_outs_;      // few-pool replays: each pool's records
    void merge_pools(size_t ng, size_t nch, const UVec<uint32_t>& brow, std::vector<uint8_t>& sel,
                     GroupList& out_groups, UVec<uint32_t>& expired, UVec<uint32_t>& newly);
    void merge_rows(size_t nb, size_t nch, const UVec<uint32_t>& brow, std::vector<uint8_t>& sel,
                    GroupList& out_groups, UVec<uint32_t>& expired, UVec<uint32_t>& newly);
    std::vector<uint32_t> pos_of_;        // slot -> list position during a dense replay, else kNoSlot
    Dict field_dict_;                 // field names -> field id
    std::vector<const char*> tk_ptr_;  // per slot: NUL-terminated ticket id in tk_arena_
    std::vector<uint32_t> tk_len_;
    StrArena tk_arena_;                // ticket ids (blocks never move: results point here)
    std::string_view tk(uint32_t s) const { return {tk_ptr_[s], tk_len_[s]}; }
    size_t nslots() const { return tk_ptr_.size(); }
    std::vector<int64_t> created_;
    std::vector<int64_t> ckey_;       // sortable key of float64(CreatedAt)
    std::vector<int32_t> minc_, maxc_, cm_, count_, intervals_;
    std::vector<uint32_t> party_;     // kNoParty for ""
    std::vector<uint8_t> live_;       // in m.indexes
    // in the search index: 0 for the members of a group the post-pass re-check
    // dropped (processDefault had deleted them from bluge when it selected
    // them; they stay in m.indexes and can search, but are never found)
    std::vector<uint8_t> indexed_;
    std::vector<uint8_t> is_active_;  // in m.activeIndexes
    std::vector<uint32_t> sig_;
    // per slot: the ticket carries every keyword its own query requires (its
    // signature's MUST terms), so it lies in its own pool (plan_parallel)
    std::vector<uint8_t> self_match_;
    // slots in CreatedAt order with strictly increasing created_ and ckey_
    // (tickets inserted in time order): scan order, slot order and the pinned
    // active order agree
    bool monotone_ = true;
    uint8_t self_match_of(uint32_t s) const;
    std::vector<HotRec> hot_;         // per slot: the replay's packed fields
    void set_hot(uint32_t s);
    std::vector<uint32_t> pres_off_;  // CSR over presences: [slot] -> first presence
    std::vector<uint32_t> pres_sess_; // per presence: session dict id
    ColdStore cold_;                  // per slot: session, party, query, presences, properties
    std::vector<uint32_t> tnode_;     // per slot: node_dict_ id
    Dict node_dict_;
    std::vector<std::vector<int64_t>> fval_;
    std::vector<std::vector<uint8_t>> fkind_;
    HashIndex slot_of_;               // ticket id -> latest slot (may be dead: checked with live_)
    std::vector<uint32_t> active_list_;                  // pinned (CreatedAt, Ticket) order, may hold inactive
    // every entry of active_list_ is live and active (set by the filters that
    // end a pass and a compaction, kept by appends, cleared by kill_slot):
    // the next pass's rows are then the list itself, copied, not filtered
    bool active_exact_ = false;
    bool active_sorted_ = true;
    SlotSets sess_slots_;             // session dict id -> slots (sessionTickets)
    SlotSets party_slots_;            // party dict id -> slots (partyTickets)
    uint32_t n_live_ = 0;

    // ---- signatures / clauses ----
    HashIndex sig_idx_;  // signature identity (sig_hash) -> id, compared by sig_eq
    std::vector<Sig> sigs_;
    std::vector<uint64_t> sig_fmask_;  // per signature: its must_fmask (plan_pools reads 8 B, not the Sig)
    // per signature, what a packed batch's assembly reads of it (16 B, not the
    // 88-B Sig over two lines): the single MUST term's posting key and the
    // roofline's field / clause counts
    struct SigLite {
        uint64_t key1;
        uint16_t n_fields, n_clauses;
        uint32_t pad;
    };
    static SigLite lite_of(const Sig& s) { return SigLite{s.must_key1, s.n_fields, s.n_clauses, 0}; }
    std::vector<SigLite> sig_lite_;
    std::vector<DClause> clauses_;
    std::vector<DQuery> squery_;      // per slot
    std::vector<uint8_t> field_used_; // per field: referenced by some clause
    std::vector<uint8_t> field_posting_; // per field: used as a MUST TERM source

    // ---- index (scan order + postings), host mirror ----
    std::vector<uint32_t> order_;
    bool full_var_mode_ = true;  // NKM_FULLVAR=0: variable-score searches always use the LDS top-K
    bool slot_lists_mode_ = true;  // NKM_SLOTLISTS=0: hit lists come back as 16-B DHits, not 4-B slot ids
    bool slot_lists_rev_ = false;  // NKM_SLOTLISTS=2: RevPrecision batches' lists as slot ids too
    bool page_mode_ = true;  // NKM_PAGE=0: only a batch's first row pages a truncated list
    // Batch window after a variable-score list ran out: the next batch takes
    // twice the rows the last one decided (at least kWinMin), not every
    // remaining row, since its lists go stale at about the same depth; a
    // batch that runs to its end doubles the window.
    static constexpr size_t kWinMin = 2048;
    static constexpr uint32_t kVarKMin = 64;  // floor of a variable-score search's hit capacity
    bool batch_profile_ = false;  // NKM_PROFILE=2: one stderr line per serial batch
    bool partial_mode_ = true;    // NKM_PARTIAL=0: a batch with a truncated list replays serially
    bool dev_enum_mode_ = true;   // NKM_DEVENUM=0: processCustom enumerates its subsets on the host
    bool order_sorted_ = true;
    bool index_dirty_ = true;
    uint32_t order_head_ = 0;
    bool order_identity_ = false;  // order_[p] == p for every p (build_index): the hashed mscan's contiguous mode
    bool mcontig_mode_ = true;     // NKM_MCONTIG=0: never the contiguous mode
    PostingMap postings_map_;
    std::vector<uint32_t> postings_;
    std::vector<uint32_t> pending_dead_;  // slots to clear on the device at next sync

    // ---- device mirror ----
    size_t dev_slots_ = 0;  // slots uploaded
    size_t dev_cap_ = 0;
    DevArray<uint8_t> d_alive_;
    DevArray<int32_t> d_minc_, d_maxc_;
    DevArray<uint32_t> d_party_;
    DevArray<DQuery> d_squery_;
    DevArray<DClause> d_clauses_;
    // multi-term matchers (OP_TERMSET): accepted dictionary ids (ascending) and
    // each one's score contribution; device copy = desc (off, len) + ids + scores
    struct TermSet {
        TermMatcher m;
        double b = 1.0;         // query boost of the clause
        uint32_t done = 0;      // dictionary ids [0, done) already tested
        std::vector<uint32_t> ids;
        std::vector<double> sc;
    };
    std::vector<TermSet> tsets_;
    std::unordered_map<std::string, uint32_t> tset_index_;
    bool tsets_dirty_ = false;
    DevArray<uint32_t> d_tset_desc_, d_tset_ids_;
    DevArray<double> d_tset_sc_;
    size_t dev_clauses_ = 0;
    std::vector<DevArray<int64_t>*> d_fval_;
    std::vector<DevArray<uint8_t>*> d_fkind_;
    std::vector<size_t> dev_field_slots_;
    DevArray<int64_t*> d_fval_ptrs_;
    DevArray<uint8_t*> d_fkind_ptrs_;
    DevArray<uint32_t> d_order_, d_postings_;
    DevArray<DGroup> d_groups_;
    DevArray<DHit> d_out_;
    DevArray<DHit> d_scan_;          // scan_kernel chunk outputs (stitch_kernel input)
    DevArray<DChunkMap> d_map_;
    DevArray<uint32_t> d_cranges_, d_coffs_;  // per chunked search: its cell range; per cell: its rank
    PinnedArray<uint32_t> h_cranges_;
    PinnedArray<DChunkMap> h_map_;
    DevArray<DClause> d_mcl_;        // mscan_kernel's clause copies
    PinnedArray<DClause> h_mcl_;
    DevArray<DMSig> d_msig_;         // mscan_kernel's signatures
    PinnedArray<DMSig> h_msig_;
    PinnedArray<uint32_t> h_mx_;     // row-sharded hashed scan: scratch + counts through the host exchange
    DevArray<uint8_t> d_rev_;
    DevArray<uint32_t> d_small_;     // rsmall_kernel's rows (indexes of the batch's whole searches)
    PinnedArray<uint32_t> h_small_;
    PinnedArray<DHit> h_page_;       // fetch_more's page (pinned: one round trip)
    PinnedArray<uint8_t> h_page_rev_;
    DevArray<DGroupResult> d_res_;
    DevArray<uint32_t> d_slots_tmp_;
    DevArray<uint8_t> d_pair_out_;
    PinnedArray<DGroup> h_groups_;
    PinnedArray<DHit> h_out_;
    DevArray<uint32_t> d_slots_;     // hit lists packed to slot ids (pack_slots_kernel)
    PinnedArray<uint32_t> h_slots_;
    DevArray<DHit> d_last_;          // each whole search's last entry (its cursor)
    PinnedArray<DHit> h_last_;
    PinnedArray<uint8_t> h_rev_;
    PinnedArray<DGroupResult> h_res_;
    PinnedArray<uint32_t> h_slots_tmp_;
    PinnedArray<uint8_t> h_pair_out_;

    // ---- row-sharded mode (include/nakama_cluster.h) ----
    int shard_world_ = 1, shard_rank_ = 0;
    mm_allgather_fn shard_fn_ = nullptr;  // host transport
    void* shard_ctx_ = nullptr;
    void* nccl_comm_ = nullptr;           // device transport: an ncclComm_t (RCCL over xGMI)
    // a transport is set (also at world 1: the exchange path runs, trivially)
    bool row_shard() const { return shard_fn_ != nullptr || nccl_comm_ != nullptr; }
    // In-place all-gather-v of the byte ranges [off[q], off[q+1]) of a buffer:
    // a device buffer over RCCL (enqueued on the stream), or a host buffer
    // through the caller's function.
    void shard_gather_device(void* dbuf, const std::vector<int64_t>& off);
    void shard_gather_host(void* hbuf, const std::vector<int64_t>& off);
    bool shard_any(bool v);  // OR over the ranks
    void shard_release();

    // ---- open custom pass ----
    bool custom_open_ = false;
    // NKM_PARALLEL: "0" keeps every host phase serial, "force" takes the
    // parallel paths at any size (tests), unset: parallel above the sizes
    // where it pays.
    int par_mode_ = 1;  // 0 off, 1 auto, 2 force
    // NKM_DENSE=0: single-search pools take the generic walk too (A/B, tests)
    bool dense_mode_ = true;
    bool pipe_mode_ = true;  // NKM_PIPE=0: the pool walks' merge runs after all walks, not beside them
    bool gpipe_mode_ = true; // NKM_GPIPE=0: no identity-pool shortcut (slot -> position map, copies gathered before the walks)
    static constexpr int kMergeMult = 8;  // pipelined merge chunks per worker (the last one is the tail after the slowest walk)
    bool runs_mode_ = true;    // NKM_RUNS=0: pools in contiguous runs take the per-row records + merge_rows
    bool pruns_mode_ = true;   // NKM_PRUNS=0: packed batches always plan through plan_pools
    int32_t max_pres_ = 1;   // most presences of any ticket inserted (an entry bound of the pipelined merge)
    // NKM_FAST=0: every row takes the exact loop body, also when no two live
    // tickets share a session (the fast walk, replay_core.h) (A/B, tests)
    bool fast_mode_ = true;
    // NKM_KERNEL: which query-eval kernel takes a batch's constant-score
    // searches (tests run every path against the oracle at small sizes):
    // "auto" (by size and coverage), "search" (search_kernel only),
    // "scan" (scan_kernel at any size), "mscan" (mscan_kernel whenever eligible)
    enum KernelMode { KM_AUTO = 0, KM_SEARCH = 1, KM_SCAN = 2, KM_MSCAN = 3 };
    int kernel_mode_ = KM_AUTO;
    // NKM_MHASH: 0 (default) the hashed mscan past 16 signatures or when the
    // scan is contiguous, 1 whenever the signatures allow it, 2 never
    int mhash_mode_ = 0;
    UVec<uint32_t> custom_expired_;

    std::vector<std::string> debug_strings_;
    // reusable output arena of mm_process (pages stay mapped across passes)
    std::vector<char> out_chars_;
    std::vector<mm_entry_ref> out_ents_;
    std::vector<int32_t> out_offs_;
    std::vector<int64_t> out_created_;
    std::atomic<bool> out_in_use_{false};
    // The pass has claimed the output arena (out_in_use_ set) to fill its
    // result early: the pipelined merge writes the result entries of its
    // groups beside the pool walks, and groups [0, filled_groups_) of the pass
    // are filled (reset by anything that reorders them).
    bool arena_claimed_ = false;
    size_t filled_groups_ = 0;
    DevArray<uint32_t> d_pm_;      // pair matrices (RevPrecision combos)
    PinnedArray<uint32_t> h_pm_;
    // processCustom's device enumeration (enum_kernel): rows, hits, work items,
    // per-item counts and scanned bases, the candidates' entries and group ends
    DevArray<DEnumRow> d_erows_;
    DevArray<DEnumHit> d_ehits_;
    DevArray<DEnumItem> d_eitems_;
    DevArray<uint32_t> d_ecnt_, d_eents_, d_eoff_;
    DevArray<uint64_t> d_ebase_;
    PinnedArray<DEnumRow> h_erows_;
    PinnedArray<DEnumHit> h_ehits_;
    PinnedArray<DEnumItem> h_eitems_;
    PinnedArray<uint32_t> h_ecnt_;
    PinnedArray<uint64_t> h_ebase_;
    // the candidates straight into the result arena (fill_custom_direct):
    // two pinned chunk buffers of entry word pairs, the group ends, events
    bool custom_direct_mode_ = true;  // NKM_CDIRECT=0: candidate list + fill_matched
    bool custom_filled_ = false;      // this pass's candidates are in the arena
    size_t custom_filled_g_ = 0, custom_filled_e_ = 0;
    PinnedArray<uint32_t> h_ech_[2];
    PinnedArray<uint32_t> h_eoff_;
    hipEvent_t ech_ev_[2] = {nullptr, nullptr};
    void fill_custom_direct(size_t G, size_t E, bool slots);
};

}  // namespace nkm
