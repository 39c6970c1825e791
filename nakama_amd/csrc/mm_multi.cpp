// nakama_amd/csrc/mm_multi.cpp — one mm handle over several devices
// (mm_create_multi, include/nakama_cluster.h).
//
// The reference constructs one LocalMatchmaker per server process
// (main.go:160) and every caller reaches it through server.Matchmaker
// (server/matchmaker.go:169-183).  MultiCore is that one handle for a node's
// GPUs: it drives one sub-handle per device from host threads through the
// nakama_mm.h entry points (this library's, or — in the CPU tests — the
// oracle's), so the Go shim needs nothing beyond the single-handle ABI.
//
// MM_MULTI_POOLS.  processDefault's greedy walk and processCustom's
// candidate enumeration never cross a pool (a search of pool P hits only P's
// documents and only P's searches hit them, matchmaker_process.go:38-330), so
// the reference's pass is the interleaving of independent per-pool passes.
// Pools are placed whole on sub-handles; their passes run concurrently; the
// group (or candidate) lists are merged by the searching ticket — each
// group's last entry (matchmaker_process.go:299-301, :562) — in the pinned
// (CreatedAt, Ticket) order.  What spans pools is answered by the
// sub-handles themselves — no per-ticket state is kept here, so Insert and
// Process cost this front nothing per ticket: MaxTickets per session / party
// (matchmaker.go:508-521) sums mm_session_ticket_count / mm_party_ticket_count
// over the sub-handles, a ticket's sub-handle is found with mm_find_tickets,
// and a targeted Remove* goes to every sub-handle (the holder answers).  The
// post-pass re-check of override-chosen groups (matchmaker.go:326-343) runs
// here in the reference's swap-remove order.
//
// MM_MULTI_ROWS.  Every sub-handle holds every ticket and runs the same pass
// with its batch searches split into one block per sub-handle (the
// row-sharded mode of mm_shard.cpp); the blocks are exchanged over RCCL
// (distinct devices) or host memory (Exchange below) and every sub-handle
// replays the same lists into the same groups; sub-handle 0 answers.
#include <hip/hip_runtime.h>

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "mm_handle.h"
#include "qcompile.h"

namespace nkm {

thread_local unsigned g_create_share = 1;

namespace {

std::string S(const char* p) { return p ? std::string(p) : std::string(); }
int status_of(int cq) { return cq == CQ_UNSUPPORTED ? MM_ERR_UNSUPPORTED : MM_ERR_QUERY_INVALID; }

// In-place all-gather-v over host buffers between the sub-handles of one
// process (mm_allgather_fn of the row-sharded mode): every sub-handle's pass
// calls it at the same points with the same offsets; each copies the other
// sub-handles' segments out of their buffers.  abort() releases every waiter
// with failure (a sub-handle whose pass failed never arrives).
class Exchange {
public:
    explicit Exchange(int n) : n_(n), bufs_((size_t)n, nullptr) {}
    int allgather(int r, void* buf, const int64_t* off) {
        std::unique_lock<std::mutex> lk(m_);
        if (broken_) return 1;
        bufs_[(size_t)r] = static_cast<char*>(buf);
        if (!wait(lk)) return 1;  // every buffer published
        lk.unlock();
        for (int q = 0; q < n_; q++) {
            const int64_t len = off[q + 1] - off[q];
            if (q != r && len > 0) std::memcpy(static_cast<char*>(buf) + off[q], bufs_[(size_t)q] + off[q], (size_t)len);
        }
        lk.lock();
        return wait(lk) ? 0 : 1;  // nobody reuses its buffer before every copy is done
    }
    void abort() {
        std::lock_guard<std::mutex> lk(m_);
        broken_ = true;
        cv_.notify_all();
    }
    void reset() {
        std::lock_guard<std::mutex> lk(m_);
        broken_ = false;
        count_ = 0;
    }

private:
    bool wait(std::unique_lock<std::mutex>& lk) {
        const uint64_t gen = gen_;
        if (++count_ == n_) {
            count_ = 0;
            gen_++;
            cv_.notify_all();
            return !broken_;
        }
        cv_.wait(lk, [&] { return gen_ != gen || broken_; });
        return !broken_;
    }
    const int n_;
    std::vector<char*> bufs_;
    std::mutex m_;
    std::condition_variable cv_;
    int count_ = 0;
    uint64_t gen_ = 0;
    bool broken_ = false;
};

struct ExCtx {
    Exchange* ex;
    int rank;
};
int exchange_fn(void* ctx, void* buf, const int64_t* off) {
    auto* c = static_cast<ExCtx*>(ctx);
    return c->ex->allgather(c->rank, buf, off);
}

mm_sub_api own_api() {
    mm_sub_api a{};
    a.create = mm_create;
    a.destroy = mm_destroy;
    a.pause = mm_pause;
    a.resume = mm_resume;
    a.stop = mm_stop;
    a.last_error = mm_last_error;
    a.add = mm_add;
    a.insert = mm_insert;
    a.extract = mm_extract;
    a.free_extract = mm_free_extract;
    a.remove_session = mm_remove_session;
    a.remove_session_all = mm_remove_session_all;
    a.remove_party = mm_remove_party;
    a.remove_party_all = mm_remove_party_all;
    a.remove_all = mm_remove_all;
    a.remove = mm_remove;
    a.process = mm_process;
    a.process_commit = mm_process_commit;
    a.free_matched = mm_free_matched;
    a.ticket_count = mm_ticket_count;
    a.active_count = mm_active_count;
    a.drain_removed = mm_drain_removed;
    a.free_str_list = mm_free_str_list;
    a.debug_hits = mm_debug_hits;
    a.debug_set_pass_hook = mm_debug_set_pass_hook;
    a.session_ticket_count = mm_session_ticket_count;
    a.party_ticket_count = mm_party_ticket_count;
    a.find_tickets = mm_find_tickets;
    return a;
}

}  // namespace

struct MultiError {
    int status;
    std::string what;
};

class MultiCore final : public Handle {
public:
    MultiCore(const mm_config& cfg, const mm_multi_config& mc);
    ~MultiCore() override;

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
    void pause() override { each_serial([&](int i) { api_.pause(subs_[i]); }); }
    void resume() override { each_serial([&](int i) { api_.resume(subs_[i]); }); }
    void stop() override {
        stopped_ = true;
        each_serial([&](int i) { api_.stop(subs_[i]); });
    }
    const char* last_error() const override { return last_error_.c_str(); }
    void set_error(const std::string& e) override { last_error_ = e; }
    void set_pass_hook(void (*fn)(void*), void* ctx) override {
        // a test hook: installed on sub-handle 0 (whose pass calls it once)
        if (api_.debug_set_pass_hook) api_.debug_set_pass_hook(subs_[0], fn, ctx);
    }
    int drain_removed(mm_str_list* out) override;
    void free_str_list(mm_str_list* out) override;
    int set_row_shard(int, int, mm_allgather_fn, void*) override { return MM_ERR_ARG; }
    int set_row_shard_rccl(int, int, const uint8_t*, int) override { return MM_ERR_ARG; }

    int32_t n_subs() const { return (int32_t)subs_.size(); }
    int32_t sub_tickets(int32_t i) { return i < n_subs() ? api_.ticket_count(subs_[(size_t)i]) : -1; }

private:
    // ---- sub-handles ----
    mm_sub_api api_{};
    bool own_ = false;  // sub-handles are this library's (HIP) handles
    std::vector<void*> subs_;
    std::vector<int> devs_;
    std::vector<std::vector<int>> sub_cpus_;  // per sub-handle: its device node's CPUs (read once)
    int mode_ = MM_MULTI_POOLS;
    bool rows() const { return mode_ == MM_MULTI_ROWS; }
    std::unique_ptr<Exchange> ex_;
    std::vector<ExCtx> ex_ctx_;
    // f(i) for every sub-handle, concurrently (each on its own host thread,
    // with its device current), or one after the other
    template <class F>
    void each(F&& f) {
        const int n = (int)subs_.size();
        if (n == 1) { f(0); return; }
        // every sub-handle on its persistent thread, confined once to its
        // device's node (the caller's thread keeps its placement), its
        // thread_local scratch kept between calls; a call made while another
        // holds those threads (a mutator beside a pass, or from inside f)
        // runs on fresh threads instead of waiting
        std::unique_lock<std::mutex> rl(st_run_mu_, std::try_to_lock);
        if (!rl.owns_lock()) { each_spawn(f); return; }
        if (st_.th.empty())
            for (int i = 0; i < n; i++) st_.th.emplace_back([this, i] { sub_thread(i); });
        const std::function<void(int)> job = [&](int i) { f(i); };
        std::unique_lock<std::mutex> lk(st_.mu);
        st_.job = &job;
        st_.pending = n;
        st_.err = nullptr;
        st_.gen++;
        st_.cv.notify_all();
        st_.done.wait(lk, [&] { return st_.pending == 0; });
        st_.job = nullptr;
        if (st_.err) std::rethrow_exception(std::exchange(st_.err, nullptr));
    }
    struct SubThreads {
        std::mutex mu;
        std::condition_variable cv, done;
        std::vector<std::thread> th;
        const std::function<void(int)>* job = nullptr;
        uint64_t gen = 0;
        int pending = 0;
        bool stop = false;
        std::exception_ptr err;
        void halt() {
            {
                std::lock_guard<std::mutex> lk(mu);
                stop = true;
            }
            cv.notify_all();
            for (auto& t : th) t.join();
            th.clear();
        }
        ~SubThreads() { halt(); }  // also when the constructor throws after a row-shard setup used them
    };
    SubThreads st_;
    std::mutex st_run_mu_;  // one each() at a time on st_'s threads
    void sub_thread(int i) {
        if (own_) {
            (void)hipSetDevice(devs_[(size_t)i]);
            place_thread(i);
        }
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> lk(st_.mu);
                st_.cv.wait(lk, [&] { return st_.stop || st_.gen != seen; });
                if (st_.stop) return;
                seen = st_.gen;
                job = st_.job;
            }
            std::exception_ptr e;
            try {
                (*job)(i);
            } catch (...) {
                e = std::current_exception();
            }
            std::lock_guard<std::mutex> lk(st_.mu);
            if (e && !st_.err) st_.err = e;
            if (--st_.pending == 0) st_.done.notify_all();
        }
    }
    void stop_threads() { st_.halt(); }
    template <class F>
    void each_spawn(F&& f) {
        const int n = (int)subs_.size();
        std::vector<std::thread> th;
        for (int i = 0; i < n; i++)
            th.emplace_back([&, i] {
                if (own_) {
                    (void)hipSetDevice(devs_[(size_t)i]);
                    place_thread(i);
                }
                f(i);
            });
        for (auto& t : th) t.join();
    }
    // Confines the calling (per-sub-handle) thread to the CPUs of sub-handle
    // i's device node, so what it first-touches (Insert's columns and records)
    // lands in that node's memory; nothing on a one-node host.
    void place_thread(int i) {
        const std::vector<int>& cpus = sub_cpus_[(size_t)i];
        if (cpus.empty()) return;
        cpu_set_t cs;
        CPU_ZERO(&cs);
        for (int c : cpus)
            if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &cs);
        (void)pthread_setaffinity_np(pthread_self(), sizeof cs, &cs);
    }
    template <class F>
    void each_serial(F&& f) {
        for (int i = 0; i < (int)subs_.size(); i++) f(i);
    }
    // Rows: one mutator on every replica, one after the other (mu_ held, so
    // never during a pass: process() holds mu_ for the whole pass in rows
    // mode).  The replicas hold the same tickets, so they must answer alike;
    // a different answer means they diverged, which is reported.
    template <class F>
    int rows_apply(F&& f) {
        int rc0 = MM_OK;
        for (int i = 0; i < (int)subs_.size(); i++) {
            const int rc = f(subs_[(size_t)i]);
            if (i == 0) {
                rc0 = sub_status(0, rc);
            } else if (rc != rc0) {
                last_error_ = "replica " + std::to_string(i) + " answered " + std::to_string(rc) + ", replica 0 " +
                              std::to_string(rc0) + " (replicas diverged)";
                return MM_ERR_INDEX;
            }
        }
        return rc0;
    }
    int sub_status(int i, int rc) {  // a sub-handle's failure becomes this handle's
        if (rc != MM_OK) {
            const char* e = api_.last_error(subs_[(size_t)i]);
            last_error_ = "sub-handle " + std::to_string(i) + ": " + (e ? e : "");
        }
        return rc;
    }

    // ---- routing (pools) ----
    std::vector<std::string> fields_;
    std::unordered_map<uint64_t, int> dir_;  // pool key -> sub-handle
    std::vector<int64_t> load_;              // tickets routed to each sub-handle
    struct QC {
        int status;
        CompiledQuery cq;
    };
    std::unordered_map<std::string, QC> qcache_;  // compiled queries by text (routing only)
    const QC& compiled(const char* q);
    int place(const std::vector<std::pair<uint64_t, int64_t>>& new_keys);  // directory update, returns 0

    // ---- cross-pool questions, answered by the sub-handles ----
    int32_t sum_counts(int32_t (*fn)(void*, const char*), const std::string& key);
    // per sub-handle i (concurrently): found[i][k] for tickets[k] (all k)
    std::vector<std::vector<uint8_t>> find_all(const char* const* ids, int32_t n, const std::vector<uint8_t>* only = nullptr);
    // a targeted removal: every sub-handle tries, the holder answers
    template <class F>
    int remove_targeted(F&& f);
    void drain_subs(bool keep);  // the sub-handles' removal logs (onto removed_ when keep)
    int max_tickets_ = 3;
    std::string node_;

    // ---- passes ----
    std::mutex mu_;          // maps, directory, outputs
    std::mutex process_mu_;  // one pass at a time; lock order process_mu_ -> mu_
    bool custom_open_ = false;
    std::vector<uint8_t> open_;  // pools: sub-handles whose processCustom pass waits for a commit
    std::atomic<bool> stopped_{false};
    std::string last_error_;
    struct MatchedHold {  // a merged result and the sub-handle results it points into
        std::vector<mm_matched> subs;
        std::vector<int32_t> offs;
        std::vector<mm_entry_ref> ents;
        std::vector<int64_t> created;
    };
    void free_hold(MatchedHold* h);
    void merge_groups(const std::vector<mm_matched>& outs, MatchedHold* h);
    void fill_stats(const std::vector<mm_matched>& outs, mm_matched* out);
    struct ExtractHold {
        std::vector<mm_extract_list> subs;
        std::vector<mm_ticket> t;
    };
    std::unordered_map<const void*, std::unique_ptr<ExtractHold>> extracts_;
    bool track_removed_ = false;
    std::vector<std::string> removed_;
    std::unordered_map<const void*, std::unique_ptr<std::vector<std::string>>> str_lists_;
};

MultiCore::MultiCore(const mm_config& cfg, const mm_multi_config& mc) {
    if (!mc.devices || mc.n_devices < 1) throw MultiError{MM_ERR_ARG, "no devices"};
    if (mc.mode != MM_MULTI_POOLS && mc.mode != MM_MULTI_ROWS) throw MultiError{MM_ERR_ARG, "mode"};
    mode_ = mc.mode;
    own_ = mc.api == nullptr;
    api_ = own_ ? own_api() : *mc.api;
    if (!api_.create || !api_.destroy || !api_.add || !api_.insert || !api_.process || !api_.process_commit ||
        !api_.free_matched || !api_.extract || !api_.free_extract || !api_.remove || !api_.remove_session ||
        !api_.remove_session_all || !api_.remove_party || !api_.remove_party_all || !api_.remove_all ||
        !api_.ticket_count || !api_.active_count || !api_.drain_removed || !api_.free_str_list || !api_.pause ||
        !api_.resume || !api_.stop || !api_.last_error)
        throw MultiError{MM_ERR_ARG, "incomplete sub-handle api"};
    if (rows() && !own_) throw MultiError{MM_ERR_ARG, "MM_MULTI_ROWS needs this library's sub-handles"};
    if (!rows()) {
        if (!mc.pool_fields || mc.n_pool_fields < 1) throw MultiError{MM_ERR_ARG, "MM_MULTI_POOLS needs pool fields"};
        for (int i = 0; i < mc.n_pool_fields; i++) fields_.push_back(S(mc.pool_fields[i]));
    }
    max_tickets_ = cfg.max_tickets;
    node_ = S(cfg.node);
    const int n = mc.n_devices;
    devs_.assign(mc.devices, mc.devices + n);
    load_.assign((size_t)n, 0);
    // each sub-handle's host share: the sub-handles on its device's NUMA node
    // (every one when the nodes are unknown) split that node's cores
    std::vector<int> nodes((size_t)n, -1);
    sub_cpus_.assign((size_t)n, {});
    if (own_)
        for (int i = 0; i < n; i++) {
            nodes[(size_t)i] = device_numa_node(devs_[(size_t)i]);
            sub_cpus_[(size_t)i] = node_cpus(nodes[(size_t)i]);
        }
    for (int i = 0; i < n; i++) {
        mm_config c = cfg;
        c.device = devs_[(size_t)i];
        unsigned share = 0;
        for (int k = 0; k < n; k++) share += nodes[(size_t)i] < 0 || nodes[(size_t)k] == nodes[(size_t)i];
        g_create_share = nodes[(size_t)i] < 0 ? (unsigned)n : share;
        void* s = api_.create(&c);
        g_create_share = 1;
        if (!s) {
            const std::string e = S(api_.last_error(nullptr));
            for (void* p : subs_) api_.destroy(p);
            subs_.clear();
            throw MultiError{MM_ERR_DEVICE, "sub-handle " + std::to_string(i) + ": " + e};
        }
        subs_.push_back(s);
    }
    if (!api_.session_ticket_count || !api_.party_ticket_count || !api_.find_tickets) {
        for (void* p : subs_) api_.destroy(p);
        subs_.clear();
        throw MultiError{MM_ERR_ARG, "sub-handle api without the ABI 4 lookups"};
    }
    if (rows() && n > 1) {
        int tr = mc.transport;
        if (tr == MM_MULTI_AUTO) {
            std::vector<int> d = devs_;
            std::sort(d.begin(), d.end());
            tr = std::unique(d.begin(), d.end()) == d.end() ? MM_MULTI_RCCL : MM_MULTI_HOST;
        }
        std::vector<int> rc((size_t)n, MM_OK);
        if (tr == MM_MULTI_RCCL) {
            uint8_t uid[128];
            if (mm_rccl_unique_id(uid, sizeof uid) != MM_OK) throw MultiError{MM_ERR_DEVICE, "ncclGetUniqueId"};
            // ncclCommInitRank blocks until every rank joins: one thread per sub-handle
            each([&](int i) { rc[(size_t)i] = mm_shard_rows_rccl(subs_[(size_t)i], n, i, uid, 128); });
        } else {
            ex_.reset(new Exchange(n));
            ex_ctx_.resize((size_t)n);
            for (int i = 0; i < n; i++) {
                ex_ctx_[(size_t)i] = ExCtx{ex_.get(), i};
                rc[(size_t)i] = mm_shard_rows(subs_[(size_t)i], n, i, exchange_fn, &ex_ctx_[(size_t)i]);
            }
        }
        for (int i = 0; i < n; i++)
            if (rc[(size_t)i] != MM_OK) {
                const std::string e = S(api_.last_error(subs_[(size_t)i]));
                for (void* p : subs_) api_.destroy(p);
                subs_.clear();
                throw MultiError{rc[(size_t)i], "row-shard setup of sub-handle " + std::to_string(i) + ": " + e};
            }
    }
}

MultiCore::~MultiCore() {
    stop_threads();
    for (auto& kv : extracts_)
        for (size_t i = 0; i < kv.second->subs.size(); i++) api_.free_extract(subs_[i], &kv.second->subs[i]);
    if (ex_) ex_->abort();
    for (void* s : subs_) api_.destroy(s);
}

// ---- routing ----------------------------------------------------------------

const MultiCore::QC& MultiCore::compiled(const char* q) {
    const std::string key = S(q);
    auto it = qcache_.find(key);
    if (it != qcache_.end()) return it->second;
    if (qcache_.size() >= (1u << 16)) qcache_.clear();  // unique-query workloads gain nothing from it
    QC c;
    c.status = compile_query(key, &c.cq);
    return qcache_.emplace(key, std::move(c)).first->second;
}

// New pools, largest first, each to the least-loaded sub-handle (online LPT,
// as nakama_amd/cluster.py places pools over ranks).
int MultiCore::place(const std::vector<std::pair<uint64_t, int64_t>>& new_keys) {
    std::vector<std::pair<uint64_t, int64_t>> k = new_keys;
    std::sort(k.begin(), k.end(), [](const auto& a, const auto& b) {
        return a.second != b.second ? a.second > b.second : a.first < b.first;
    });
    for (auto& kv : k) {
        int best = 0;
        for (int i = 1; i < (int)load_.size(); i++)
            if (load_[(size_t)i] < load_[(size_t)best]) best = i;
        dir_[kv.first] = best;
        load_[(size_t)best] += kv.second;
    }
    return 0;
}

int32_t MultiCore::sum_counts(int32_t (*fn)(void*, const char*), const std::string& key) {
    int32_t n = 0;
    for (void* sh : subs_) n += std::max(0, fn(sh, key.c_str()));
    return n;
}

std::vector<std::vector<uint8_t>> MultiCore::find_all(const char* const* ids, int32_t n,
                                                      const std::vector<uint8_t>* only) {
    std::vector<std::vector<uint8_t>> f(subs_.size());
    each([&](int i) {
        if (only && !(*only)[(size_t)i]) return;
        f[(size_t)i].assign((size_t)std::max(n, 1), 0);
        if (n > 0 && api_.ticket_count(subs_[(size_t)i]) > 0) api_.find_tickets(subs_[(size_t)i], ids, n, f[(size_t)i].data());
    });
    return f;
}

// RemoveSession / RemoveParty (matchmaker.go:725-767, :830-870) name a
// ticket: the sub-handle holding it decides; the others answer not-found.
template <class F>
int MultiCore::remove_targeted(F&& f) {
    int rc = MM_ERR_TICKET_NOT_FOUND;
    for (int i = 0; i < (int)subs_.size(); i++) {
        const int r = f(subs_[(size_t)i]);
        if (r == MM_OK) rc = MM_OK;
        else if (r != MM_ERR_TICKET_NOT_FOUND && rc != MM_OK) rc = sub_status(i, r);
    }
    return rc;
}

// The sub-handles' removal logs (Remove*, replaced ids: matched tickets are
// in the pass results).  Rows: replicas log alike, sub-handle 0 speaks.
void MultiCore::drain_subs(bool keep) {
    for (int i = 0; i < (int)subs_.size(); i++) {
        mm_str_list l{};
        if (api_.drain_removed(subs_[(size_t)i], &l) != MM_OK) continue;
        if (keep && (!rows() || i == 0))
            for (int k = 0; k < l.n; k++) removed_.emplace_back(S(l.items[k]));
        api_.free_str_list(subs_[(size_t)i], &l);
    }
}

// ---- mutators ---------------------------------------------------------------

// Add (matchmaker.go:443-565): the query, then duplicate sessions, then
// MaxTickets over every sub-handle's tickets, in the reference's order.
int MultiCore::add(const mm_ticket& t) {
    if (stopped_) return MM_ERR_NOT_AVAILABLE;
    std::lock_guard<std::mutex> lk(mu_);
    if (rows()) return rows_apply([&](void* sh) { return api_.add(sh, &t); });
    const QC& q = compiled(t.query);
    if (q.status != CQ_OK) return status_of(q.status);
    {
        std::unordered_set<std::string> seen;
        for (int i = 0; i < t.n_presences; i++)
            if (!seen.insert(S(t.presences[i].session_id)).second) return MM_ERR_DUPLICATE_SESSION;
    }
    const uint64_t key = route_key(t, fields_, q.cq);
    if (!key) {
        last_error_ = "ticket query does not pin every pool field to the ticket's own value (MM_MULTI_POOLS)";
        return MM_ERR_UNSUPPORTED;
    }
    for (int i = 0; i < t.n_presences; i++)
        if (sum_counts(api_.session_ticket_count, S(t.presences[i].session_id)) >= max_tickets_)
            return MM_ERR_TOO_MANY_TICKETS;
    const std::string party = S(t.party_id);
    if (!party.empty() && sum_counts(api_.party_ticket_count, party) >= max_tickets_) return MM_ERR_TOO_MANY_TICKETS;
    if (!dir_.count(key)) place({{key, 1}});
    const int sub = dir_[key];
    const char* id = t.ticket;
    for (int i = 0; i < (int)subs_.size(); i++) {  // the same id on another sub-handle: replaced
        uint8_t f = 0;
        if (i != sub && api_.find_tickets(subs_[(size_t)i], &id, 1, &f) > 0) api_.remove(subs_[(size_t)i], &id, 1);
    }
    const int rc = sub_status(sub, api_.add(subs_[(size_t)sub], &t));
    if (rc == MM_OK) load_[(size_t)sub]++;
    return rc;
}

// Insert (matchmaker.go:567-682): tickets whose query fails to compile are
// skipped (the reference logs and continues); the others go to their pool's
// sub-handle, all sub-handles inserting concurrently.
int MultiCore::insert(const mm_ticket* ts, int32_t n) {
    if (stopped_ || n <= 0) return MM_OK;
    std::lock_guard<std::mutex> lk(mu_);
    const int ns = (int)subs_.size();
    if (rows()) {
        std::vector<int> rc((size_t)ns, MM_OK);
        each([&](int i) { rc[(size_t)i] = api_.insert(subs_[(size_t)i], ts, n); });
        for (int i = 0; i < ns; i++)
            if (rc[(size_t)i] != MM_OK) return sub_status(i, rc[(size_t)i]);
        return MM_OK;
    }
    // pool keys on host threads, each with its own compile cache (a pool's
    // tickets share a query; unique queries compile once either way)
    std::vector<uint64_t> key((size_t)n, 0);
    std::vector<uint8_t> skip((size_t)n, 0);  // the query does not compile: skipped, as the reference's Insert does
    {
        const unsigned W = n >= 16384 ? std::max(1u, std::min(16u, std::thread::hardware_concurrency())) : 1u;
        auto route = [&](unsigned w) {
            std::unordered_map<std::string_view, QC> local;
            for (int32_t k = (int32_t)((int64_t)n * w / W); k < (int32_t)((int64_t)n * (w + 1) / W); k++) {
                const std::string_view q = ts[k].query ? std::string_view(ts[k].query) : std::string_view();
                auto it = local.find(q);
                if (it == local.end()) {
                    if (local.size() >= (1u << 12)) local.clear();
                    QC c;
                    c.status = compile_query(q, &c.cq);
                    it = local.emplace(q, std::move(c)).first;
                }
                if (it->second.status != CQ_OK) { skip[(size_t)k] = 1; continue; }
                key[(size_t)k] = route_key(ts[k], fields_, it->second.cq);
            }
        };
        std::vector<std::thread> th;
        for (unsigned w = 1; w < W; w++) th.emplace_back(route, w);
        route(0);
        for (auto& t : th) t.join();
    }
    int64_t unroutable = 0;
    std::unordered_map<uint64_t, int64_t> fresh;
    for (int32_t k = 0; k < n; k++) {
        if (skip[(size_t)k]) continue;
        if (!key[(size_t)k]) { unroutable++; continue; }
        if (!dir_.count(key[(size_t)k])) fresh[key[(size_t)k]]++;
    }
    if (!fresh.empty()) place(std::vector<std::pair<uint64_t, int64_t>>(fresh.begin(), fresh.end()));
    std::vector<int> sub_of((size_t)n, -1);
    {
        uint64_t last_key = 0;
        int last_sub = -1;
        for (int32_t k = 0; k < n; k++) {
            const uint64_t kk = key[(size_t)k];
            if (!kk) continue;
            if (kk != last_key) {
                last_key = kk;
                last_sub = dir_[kk];
            }
            sub_of[(size_t)k] = last_sub;
            load_[(size_t)last_sub]++;
        }
    }
    // an id already held by another sub-handle is replaced (matchmaker.go:650):
    // each sub-handle looks the batch up itself, concurrently, and drops the
    // ids routed elsewhere (a fresh batch finds nothing)
    std::vector<int> rc((size_t)ns, MM_OK);
    std::vector<const char*> ids((size_t)n);
    for (int32_t k = 0; k < n; k++) ids[(size_t)k] = ts[k].ticket;
    each([&](int i) {
        void* sh = subs_[(size_t)i];
        std::vector<mm_ticket> part;  // this sub-handle's tickets, in batch order
        for (int32_t k = 0; k < n; k++)
            if (sub_of[(size_t)k] == i) part.push_back(ts[k]);
        if (api_.ticket_count(sh) > 0) {
            std::vector<uint8_t> f((size_t)n, 0);
            if (api_.find_tickets(sh, ids.data(), n, f.data()) > 0) {
                std::vector<const char*> moved;
                for (int32_t k = 0; k < n; k++)
                    if (f[(size_t)k] && sub_of[(size_t)k] >= 0 && sub_of[(size_t)k] != i) moved.push_back(ids[(size_t)k]);
                if (!moved.empty()) api_.remove(sh, moved.data(), (int32_t)moved.size());
            }
        }
        if (!part.empty()) rc[(size_t)i] = api_.insert(sh, part.data(), (int32_t)part.size());
    });
    for (int i = 0; i < ns; i++)
        if (rc[(size_t)i] != MM_OK) return sub_status(i, rc[(size_t)i]);
    if (unroutable) {
        last_error_ = std::to_string(unroutable) +
                      " ticket(s) not inserted: query does not pin every pool field to the ticket's own value";
        return MM_ERR_UNSUPPORTED;
    }
    return MM_OK;
}

int MultiCore::remove_session(const std::string& sid, const std::string& ticket) {
    std::lock_guard<std::mutex> lk(mu_);
    if (rows()) return rows_apply([&](void* sh) { return api_.remove_session(sh, sid.c_str(), ticket.c_str()); });
    return remove_targeted([&](void* sh) { return api_.remove_session(sh, sid.c_str(), ticket.c_str()); });
}

int MultiCore::remove_party(const std::string& pid, const std::string& ticket) {
    std::lock_guard<std::mutex> lk(mu_);
    if (rows()) return rows_apply([&](void* sh) { return api_.remove_party(sh, pid.c_str(), ticket.c_str()); });
    return remove_targeted([&](void* sh) { return api_.remove_party(sh, pid.c_str(), ticket.c_str()); });
}

int MultiCore::remove_session_all(const std::string& sid) {
    std::lock_guard<std::mutex> lk(mu_);
    int rc0 = MM_OK;
    each_serial([&](int i) {
        const int rc = api_.remove_session_all(subs_[(size_t)i], sid.c_str());
        if (rc != MM_OK && rc0 == MM_OK) rc0 = sub_status(i, rc);
    });
    return rc0;
}

int MultiCore::remove_party_all(const std::string& pid) {
    std::lock_guard<std::mutex> lk(mu_);
    int rc0 = MM_OK;
    each_serial([&](int i) {
        const int rc = api_.remove_party_all(subs_[(size_t)i], pid.c_str());
        if (rc != MM_OK && rc0 == MM_OK) rc0 = sub_status(i, rc);
    });
    return rc0;
}

int MultiCore::remove_all(const std::string& node) {
    std::lock_guard<std::mutex> lk(mu_);
    int rc0 = MM_OK;
    each_serial([&](int i) {
        const int rc = api_.remove_all(subs_[(size_t)i], node.c_str());
        if (rc != MM_OK && rc0 == MM_OK) rc0 = sub_status(i, rc);
    });
    return rc0;
}

int MultiCore::remove(const char* const* tickets, int32_t n) {
    std::lock_guard<std::mutex> lk(mu_);
    if (rows()) return rows_apply([&](void* sh) { return api_.remove(sh, tickets, n); });
    // every sub-handle drops the ids it holds (unknown ids are ignored,
    // matchmaker.go:972-1024), concurrently
    std::vector<int> rc(subs_.size(), MM_OK);
    each([&](int i) { rc[(size_t)i] = api_.remove(subs_[(size_t)i], tickets, n); });
    for (int i = 0; i < (int)subs_.size(); i++)
        if (rc[(size_t)i] != MM_OK) return sub_status(i, rc[(size_t)i]);
    return MM_OK;
}

// ---- the pass -----------------------------------------------------------------

void MultiCore::fill_stats(const std::vector<mm_matched>& outs, mm_matched* out) {
    int best = 0;
    for (size_t i = 0; i < outs.size(); i++) {
        out->n_expired += outs[i].n_expired;
        out->pair_evals += outs[i].pair_evals;
        out->pairs_decided += outs[i].pairs_decided;
        out->eval_launches += outs[i].eval_launches;
        out->full_lists += outs[i].full_lists;
        out->n_batches = std::max(out->n_batches, outs[i].n_batches);
        out->eval_ms = std::max(out->eval_ms, outs[i].eval_ms);  // the devices run concurrently
        if (outs[i].eval_bytes > outs[(size_t)best].eval_bytes) best = (int)i;
        if (rows()) break;  // replicas: sub-handle 0's pass
    }
    out->eval_kernel = outs[(size_t)best].eval_kernel;
    for (size_t i = 0; i < outs.size(); i++) {
        if (outs[i].eval_kernel == out->eval_kernel) out->eval_bytes += outs[i].eval_bytes;
        if (rows()) break;
    }
}

// The sub-handles' group (or candidate) lists merged into the reference's
// order: by the searching ticket's (CreatedAt, Ticket) — the group's last
// entry.  Each list ascends by CreatedAt, so the merge is cut into key ranges
// at sampled splitter keys (equal keys never straddle a cut: ties are decided
// by ticket id inside one range); each range is k-way merged on its own
// thread straight into the output at offsets from a prefix over the ranges.
// C3 at 8 x 1M tickets: 1.4M groups, 8M entries (128 MB) — a serial merge
// would take tens of milliseconds against a few-millisecond pass.
void MultiCore::merge_groups(const std::vector<mm_matched>& outs, MatchedHold* h) {
    const int ns = (int)outs.size();
    size_t ng = 0, ne = 0;
    for (auto& o : outs) {
        ng += (size_t)o.n_groups;
        ne += (size_t)o.n_entries;
    }
    h->offs.assign(ng + 1, 0);
    h->ents.resize(ne);
    h->created.resize(ng);
    if (!ng) return;
    bool asc = true;
    for (auto& o : outs)
        for (int32_t g = 1; g < o.n_groups && asc; g++) asc = o.group_created[g - 1] <= o.group_created[g];
    unsigned W = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    // the parallel merge's threshold; NKM_PARALLEL=force (the host paths' "at
    // any size" switch, tests) takes it at every size
    const char* par_env = std::getenv("NKM_PARALLEL");
    const size_t kMergeMin = par_env && !std::strcmp(par_env, "force") ? 1 : (size_t)65536;
    if (ng < kMergeMin || !asc) W = 1;  // small (or, defensively, unsorted) lists: one serial merge
    // splitters: every (ng / 64W)-th key of every list, sorted, at the W - 1 quantiles
    std::vector<int64_t> cut;  // W + 1 keys: [cut[p], cut[p + 1]) is range p
    if (W > 1) {
        std::vector<int64_t> sample;
        const size_t step = std::max<size_t>(1, ng / (64 * (size_t)W));
        for (auto& o : outs)
            for (int32_t g = 0; g < o.n_groups; g += (int32_t)step) sample.push_back(o.group_created[g]);
        std::sort(sample.begin(), sample.end());
        cut.push_back(INT64_MIN);
        for (unsigned p = 1; p < W; p++) {
            const int64_t k = sample[sample.size() * p / W];
            if (k > cut.back()) cut.push_back(k);
        }
        W = (unsigned)cut.size();
        cut.push_back(INT64_MAX);
    }
    // per (range, list): its groups [a, b)
    std::vector<int32_t> ga((size_t)W * ns), gb((size_t)W * ns);
    std::vector<size_t> gofs(W + 1, 0), eofs(W + 1, 0);
    for (unsigned p = 0; p < W; p++) {
        for (int i = 0; i < ns; i++) {
            const mm_matched& o = outs[(size_t)i];
            int32_t a = 0, b = o.n_groups;
            if (W > 1) {
                a = (int32_t)(std::lower_bound(o.group_created, o.group_created + o.n_groups, cut[p]) - o.group_created);
                b = p + 1 == W ? o.n_groups
                               : (int32_t)(std::lower_bound(o.group_created, o.group_created + o.n_groups, cut[p + 1]) -
                                           o.group_created);
            }
            ga[(size_t)p * ns + i] = a;
            gb[(size_t)p * ns + i] = b;
            gofs[p + 1] += (size_t)(b - a);
            eofs[p + 1] += (size_t)(o.group_offsets[b] - o.group_offsets[a]);
        }
    }
    for (unsigned p = 0; p < W; p++) {
        gofs[p + 1] += gofs[p];
        eofs[p + 1] += eofs[p];
    }
    auto merge_range = [&](unsigned p) {
        std::vector<int32_t> at(ga.begin() + (size_t)p * ns, ga.begin() + (size_t)(p + 1) * ns);
        const int32_t* end = gb.data() + (size_t)p * ns;
        size_t go = gofs[p], eo = eofs[p];
        for (size_t k = gofs[p]; k < gofs[p + 1]; k++) {
            int best = -1;
            for (int i = 0; i < ns; i++) {
                const mm_matched& o = outs[(size_t)i];
                const int32_t g = at[(size_t)i];
                if (g >= end[i]) continue;
                if (best < 0) { best = i; continue; }
                const mm_matched& b = outs[(size_t)best];
                const int32_t gbst = at[(size_t)best];
                if (o.group_created[g] != b.group_created[gbst]) {
                    if (o.group_created[g] < b.group_created[gbst]) best = i;
                    continue;
                }
                const char* ti = o.entries[o.group_offsets[g + 1] - 1].ticket;
                const char* tb = b.entries[b.group_offsets[gbst + 1] - 1].ticket;
                if (std::strcmp(ti, tb) < 0) best = i;
            }
            const mm_matched& o = outs[(size_t)best];
            const int32_t g = at[(size_t)best]++;
            const int32_t e0 = o.group_offsets[g], e1 = o.group_offsets[g + 1];
            std::memcpy(h->ents.data() + eo, o.entries + e0, (size_t)(e1 - e0) * sizeof(mm_entry_ref));
            eo += (size_t)(e1 - e0);
            h->offs[go + 1] = (int32_t)eo;
            h->created[go] = o.group_created[g];
            go++;
        }
    };
    if (W == 1) {
        merge_range(0);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned p = 1; p < W; p++) th.emplace_back(merge_range, p);
    merge_range(0);
    for (auto& t : th) t.join();
}

void MultiCore::free_hold(MatchedHold* h) {
    for (size_t i = 0; i < h->subs.size(); i++)
        if (h->subs[i].group_offsets || h->subs[i].reserved2) api_.free_matched(subs_[i], &h->subs[i]);
    delete h;
}

int MultiCore::process(mm_matched* out) {
    std::memset(out, 0, sizeof(*out));
    const auto t0 = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> pl(process_mu_);
    if (custom_open_) return MM_ERR_STATE;
    const int ns = (int)subs_.size();
    std::vector<mm_matched> outs((size_t)ns);
    std::vector<int> rc((size_t)ns, MM_OK);
    // Rows: the replicas take their pass snapshots at their own moments, so a
    // mutation must not land between them — mu_ is held across the whole
    // pass and a concurrent mutator waits for its end (the reference allows
    // a mutation anywhere in the pass, matchmaker.go:290-343; this serialises
    // it after the pass).  Pools: each sub-handle queues its own mutations.
    std::unique_lock<std::mutex> lk(mu_, std::defer_lock);
    if (rows()) lk.lock();
    if (ex_) ex_->reset();
    each([&](int i) {
        rc[(size_t)i] = api_.process(subs_[(size_t)i], &outs[(size_t)i]);
        if (rc[(size_t)i] != MM_OK && ex_) ex_->abort();  // the other replicas stop waiting for this one
    });
    if (!rows()) lk.lock();
    int bad = -1;
    for (int i = 0; i < ns; i++)
        if (rc[(size_t)i] != MM_OK && (bad < 0 || rc[(size_t)bad] == MM_ERR_DEVICE)) bad = i;
    if (bad >= 0) {  // close every pass that did open, and report the failure
        const std::string why = S(api_.last_error(subs_[(size_t)bad]));
        for (int i = 0; i < ns; i++) {
            if (rc[(size_t)i] != MM_OK) continue;
            if (outs[(size_t)i].is_candidates) {
                mm_matched none{};
                if (api_.process_commit(subs_[(size_t)i], nullptr, nullptr, 0, &none) == MM_OK)
                    api_.free_matched(subs_[(size_t)i], &none);
            }
            api_.free_matched(subs_[(size_t)i], &outs[(size_t)i]);
        }
        last_error_ = "sub-handle " + std::to_string(bad) + ": " + why;
        return rc[(size_t)bad];
    }
    auto* h = new MatchedHold();
    h->subs = outs;
    bool cands = false;
    for (auto& o : outs) cands |= o.is_candidates != 0;
    if (rows()) {
        const mm_matched& o = outs[0];
        h->offs.assign(o.group_offsets, o.group_offsets + o.n_groups + 1);
        h->ents.assign(o.entries, o.entries + o.n_entries);
        h->created.assign(o.group_created, o.group_created + o.n_groups);
    } else {
        merge_groups(outs, h);
    }
    out->n_groups = (int32_t)h->created.size();
    out->n_entries = (int32_t)h->ents.size();
    out->group_offsets = h->offs.data();
    out->entries = h->ents.data();
    out->group_created = h->created.data();
    out->is_candidates = cands ? 1 : 0;
    fill_stats(outs, out);
    out->reserved2 = (int64_t)(intptr_t)h;
    if (cands) {
        custom_open_ = true;
        open_.assign((size_t)ns, 0);
        for (int i = 0; i < ns; i++) open_[(size_t)i] = outs[(size_t)i].is_candidates ? 1 : 0;
    }
    out->pass_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return MM_OK;
}

// The override's choice (processCustom, matchmaker_process.go:573), then the
// post-pass re-check of matchmaker.go:326-343 over the whole list — a group
// is dropped when one of its tickets is gone (removed meanwhile, or taken by
// an earlier group), with the reference's swap-remove — and each
// sub-handle's share of the kept groups, in their final order, goes to its
// commit (nothing is dropped there any more).  A group may span pools: its
// per-sub-handle parts are reassembled in entry order.
int MultiCore::process_commit(const int32_t* offs, const mm_entry_ref* ents, int32_t n_groups, mm_matched* out) {
    std::memset(out, 0, sizeof(*out));
    const auto t0 = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> pl(process_mu_);
    std::lock_guard<std::mutex> lk(mu_);
    if (!custom_open_) return MM_ERR_STATE;
    for (int g = 0; g < n_groups; g++)
        if (offs[g + 1] < offs[g]) return MM_ERR_ARG;
    const int ns = (int)subs_.size();
    std::vector<mm_matched> couts((size_t)ns);
    std::vector<int> rc((size_t)ns, MM_OK);
    auto* h = new MatchedHold();
    if (rows()) {
        each([&](int i) { rc[(size_t)i] = api_.process_commit(subs_[(size_t)i], offs, ents, n_groups, &couts[(size_t)i]); });
        custom_open_ = false;
        for (int i = 0; i < ns; i++)
            if (rc[(size_t)i] != MM_OK) {
                for (int k = 0; k < ns; k++)
                    if (rc[(size_t)k] == MM_OK) api_.free_matched(subs_[(size_t)k], &couts[(size_t)k]);
                delete h;
                return sub_status(i, rc[(size_t)i]);
            }
        const mm_matched& o = couts[0];
        h->offs.assign(o.group_offsets, o.group_offsets + o.n_groups + 1);
        h->ents.assign(o.entries, o.entries + o.n_entries);
        h->created.assign(o.group_created, o.group_created + o.n_groups);
    } else {
        // owner of each chosen entry, found by the open sub-handles (a ticket
        // on a sub-handle whose pass is not open — it had no candidate —
        // cannot be committed: treated as gone)
        const int32_t e0 = n_groups > 0 ? offs[0] : 0, ne = n_groups > 0 ? offs[n_groups] - e0 : 0;
        std::vector<const char*> ids((size_t)std::max(ne, 1));
        for (int32_t k = 0; k < ne; k++) ids[(size_t)k] = ents[e0 + k].ticket ? ents[e0 + k].ticket : "";
        const auto found = find_all(ids.data(), ne, &open_);
        std::vector<int> sub_of((size_t)(n_groups > 0 ? offs[n_groups] : 0), -1);
        for (int32_t k = 0; k < ne; k++)
            for (int i = 0; i < ns && sub_of[(size_t)(e0 + k)] < 0; i++)
                if (open_[(size_t)i] && found[(size_t)i][(size_t)k]) sub_of[(size_t)(e0 + k)] = i;
        std::vector<int32_t> list((size_t)std::max(n_groups, 0));
        for (int g = 0; g < n_groups; g++) list[(size_t)g] = g;
        std::unordered_set<std::string> taken;
        for (size_t i = 0; i < list.size();) {
            const int g = list[i];
            bool incomplete = false;
            for (int k = offs[g]; k < offs[g + 1] && !incomplete; k++)
                incomplete = sub_of[(size_t)k] < 0 || taken.count(S(ents[k].ticket));
            if (incomplete) {  // matchedEntries[i] = matchedEntries[len-1]; shrink; i--
                list[i] = list.back();
                list.pop_back();
                continue;
            }
            for (int k = offs[g]; k < offs[g + 1]; k++) taken.insert(S(ents[k].ticket));
            i++;
        }
        std::vector<std::vector<int32_t>> po((size_t)ns, std::vector<int32_t>{0});
        std::vector<std::vector<mm_entry_ref>> pe((size_t)ns);
        for (int32_t g : list) {
            std::vector<uint8_t> touched((size_t)ns, 0);
            for (int k = offs[g]; k < offs[g + 1]; k++) {
                const int s = sub_of[(size_t)k];
                pe[(size_t)s].push_back(ents[k]);
                touched[(size_t)s] = 1;
            }
            for (int s = 0; s < ns; s++)
                if (touched[(size_t)s]) po[(size_t)s].push_back((int32_t)pe[(size_t)s].size());
        }
        each([&](int i) {
            if (!open_[(size_t)i]) return;
            const int32_t npart = (int32_t)po[(size_t)i].size() - 1;
            rc[(size_t)i] = api_.process_commit(subs_[(size_t)i], po[(size_t)i].data(), pe[(size_t)i].data(), npart,
                                                &couts[(size_t)i]);
        });
        custom_open_ = false;
        int bad = -1;
        for (int i = 0; i < ns; i++) {
            if (rc[(size_t)i] != MM_OK && bad < 0) bad = i;
            if (open_[(size_t)i] && rc[(size_t)i] == MM_OK &&
                couts[(size_t)i].n_groups != (int32_t)po[(size_t)i].size() - 1 && bad < 0)
                bad = i;
        }
        if (bad >= 0) {
            for (int k = 0; k < ns; k++)
                if (open_[(size_t)k] && rc[(size_t)k] == MM_OK) api_.free_matched(subs_[(size_t)k], &couts[(size_t)k]);
            delete h;
            if (rc[(size_t)bad] != MM_OK) return sub_status(bad, rc[(size_t)bad]);
            last_error_ = "sub-handle " + std::to_string(bad) + " dropped a re-checked group";
            return MM_ERR_INDEX;
        }
        // reassemble: entry k of a kept group is the next entry of its
        // sub-handle's part, which the sub-handle returned in the same order
        std::vector<int32_t> gpos((size_t)ns, 0), epos((size_t)ns, 0);
        h->offs.push_back(0);
        for (int32_t g : list) {
            std::vector<uint8_t> touched((size_t)ns, 0);
            for (int k = offs[g]; k < offs[g + 1]; k++) {
                const int s = sub_of[(size_t)k];
                const mm_matched& o = couts[(size_t)s];
                h->ents.push_back(o.entries[o.group_offsets[gpos[(size_t)s]] + epos[(size_t)s]++]);
                touched[(size_t)s] = 1;
            }
            const int s_last = sub_of[(size_t)offs[g + 1] - 1];
            const mm_matched& ol = couts[(size_t)s_last];
            h->created.push_back(ol.group_created[gpos[(size_t)s_last]]);
            for (int s = 0; s < ns; s++)
                if (touched[(size_t)s]) {
                    gpos[(size_t)s]++;
                    epos[(size_t)s] = 0;
                }
            h->offs.push_back((int32_t)h->ents.size());
        }
    }
    h->subs = couts;
    out->n_groups = (int32_t)h->created.size();
    out->n_entries = (int32_t)h->ents.size();
    out->group_offsets = h->offs.data();
    out->entries = h->ents.data();
    out->group_created = h->created.data();
    fill_stats(couts, out);
    out->reserved2 = (int64_t)(intptr_t)h;
    out->pass_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return MM_OK;
}

void MultiCore::free_matched(mm_matched* out) {
    if (!out) return;
    if (out->reserved2) free_hold(reinterpret_cast<MatchedHold*>((intptr_t)out->reserved2));
    std::memset(out, 0, sizeof(*out));
}

// ---- state ----------------------------------------------------------------------

int MultiCore::extract(mm_extract_list* out) {
    out->n = 0;
    out->tickets = nullptr;
    if (stopped_) return MM_OK;
    std::lock_guard<std::mutex> lk(mu_);
    auto h = std::make_unique<ExtractHold>();
    const int ns = rows() ? 1 : (int)subs_.size();
    h->subs.resize((size_t)ns);
    for (int i = 0; i < ns; i++) {
        const int rc = api_.extract(subs_[(size_t)i], &h->subs[(size_t)i]);
        if (rc != MM_OK) {
            for (int k = 0; k < i; k++) api_.free_extract(subs_[(size_t)k], &h->subs[(size_t)k]);
            return sub_status(i, rc);
        }
        h->t.insert(h->t.end(), h->subs[(size_t)i].tickets, h->subs[(size_t)i].tickets + h->subs[(size_t)i].n);
    }
    const int32_t total = (int32_t)h->t.size();
    if (h->t.empty()) h->t.resize(1);  // a unique, non-null key for the hold
    out->n = total;
    out->tickets = h->t.data();
    extracts_[out->tickets] = std::move(h);
    return MM_OK;
}

void MultiCore::free_extract(mm_extract_list* out) {
    if (!out || !out->tickets) return;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = extracts_.find(out->tickets);
    if (it != extracts_.end()) {
        for (size_t i = 0; i < it->second->subs.size(); i++) api_.free_extract(subs_[i], &it->second->subs[i]);
        extracts_.erase(it);
    }
    out->tickets = nullptr;
    out->n = 0;
}

int32_t MultiCore::ticket_count() {
    if (rows()) return api_.ticket_count(subs_[0]);
    int32_t n = 0;
    for (void* s : subs_) n += api_.ticket_count(s);
    return n;
}

int32_t MultiCore::active_count() {
    if (rows()) return api_.active_count(subs_[0]);
    int32_t n = 0;
    for (void* s : subs_) n += api_.active_count(s);
    return n;
}

int32_t MultiCore::debug_hits(const std::string& ticket, const char** tk, double* sc, int32_t cap) {
    if (!api_.debug_hits) return -1;
    int sub = 0;
    if (!rows()) {
        std::lock_guard<std::mutex> lk(mu_);
        const char* id = ticket.c_str();
        sub = -1;
        for (int i = 0; i < (int)subs_.size() && sub < 0; i++) {
            uint8_t f = 0;
            if (api_.find_tickets(subs_[(size_t)i], &id, 1, &f) > 0) sub = i;
        }
        if (sub < 0) return -1;
    }
    return api_.debug_hits(subs_[(size_t)sub], ticket.c_str(), tk, sc, cap);
}

int32_t MultiCore::session_ticket_count(const std::string& sid) {
    std::lock_guard<std::mutex> lk(mu_);
    if (rows()) return api_.session_ticket_count(subs_[0], sid.c_str());
    return sum_counts(api_.session_ticket_count, sid);
}

int32_t MultiCore::party_ticket_count(const std::string& pid) {
    std::lock_guard<std::mutex> lk(mu_);
    if (rows()) return api_.party_ticket_count(subs_[0], pid.c_str());
    return sum_counts(api_.party_ticket_count, pid);
}

int32_t MultiCore::find_tickets(const char* const* ids, int32_t n, uint8_t* found) {
    std::lock_guard<std::mutex> lk(mu_);
    if (rows()) return api_.find_tickets(subs_[0], ids, n, found);
    const auto f = find_all(ids, n);
    int32_t k = 0;
    for (int32_t j = 0; j < n; j++) {
        uint8_t x = 0;
        for (auto& v : f) x |= v[(size_t)j];
        found[j] = x;
        k += x;
    }
    return k;
}

int MultiCore::drain_removed(mm_str_list* out) {
    std::lock_guard<std::mutex> lk(mu_);
    const bool first = !track_removed_;
    drain_subs(!first);  // the first call starts the sub-handles' logs
    if (!rows() && !removed_.empty()) {
        // a ticket re-inserted into another pool left its old sub-handle but
        // lives on (a replaced id is not reported, as one handle does)
        std::vector<const char*> ids(removed_.size());
        for (size_t k = 0; k < ids.size(); k++) ids[k] = removed_[k].c_str();
        const auto f = find_all(ids.data(), (int32_t)ids.size());
        size_t w = 0;
        for (size_t k = 0; k < removed_.size(); k++) {
            uint8_t alive = 0;
            for (auto& v : f) alive |= v[k];
            if (alive) continue;
            if (w != k) removed_[w] = std::move(removed_[k]);
            w++;
        }
        removed_.resize(w);
    }
    track_removed_ = true;
    auto v = std::make_unique<std::vector<std::string>>(first ? std::vector<std::string>{} : std::move(removed_));
    removed_.clear();
    auto* ptrs = new const char*[v->empty() ? 1 : v->size()];
    for (size_t i = 0; i < v->size(); i++) ptrs[i] = (*v)[i].c_str();
    out->n = (int32_t)v->size();
    out->items = ptrs;
    str_lists_[ptrs] = std::move(v);
    return MM_OK;
}

void MultiCore::free_str_list(mm_str_list* out) {
    if (!out || !out->items) return;
    std::lock_guard<std::mutex> lk(mu_);
    str_lists_.erase(out->items);
    delete[] out->items;
    out->items = nullptr;
    out->n = 0;
}

}  // namespace nkm

extern "C" {

void* mm_create_multi(const mm_config* cfg, const mm_multi_config* mc) {
    if (!cfg || !mc) return nullptr;
    try {
        return static_cast<nkm::Handle*>(new nkm::MultiCore(*cfg, *mc));
    } catch (const nkm::MultiError& e) {
        nkm::set_create_error("mm_create_multi: " + e.what);
    } catch (const std::exception& e) {
        nkm::set_create_error(std::string("mm_create_multi: ") + e.what());
    } catch (...) {
        nkm::set_create_error("mm_create_multi: internal error");
    }
    return nullptr;
}

int32_t mm_device_numa_node(int32_t device) {
    try {
        return nkm::device_numa_node(device);
    } catch (...) {
        return -1;
    }
}

int32_t mm_multi_info(void* h, int32_t sub) {
    if (!h) return -1;
    auto* m = dynamic_cast<nkm::MultiCore*>(static_cast<nkm::Handle*>(h));
    if (!m) return 0;
    return sub < 0 ? m->n_subs() : m->sub_tickets(sub);
}

}  // extern "C"
