// nakama_amd/csrc/mm_capi.cpp — extern "C" entry points of include/nakama_mm.h.
// Every entry converts device failures into MM_ERR_DEVICE with a message in
// mm_last_error; nothing here falls back to a CPU search.
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>

#include "mm_core.h"

using nkm::Core;
using nkm::DeviceError;
using nkm::Handle;

namespace {
thread_local std::string g_create_error;

template <class F>
int guarded(void* h, F&& f) {
    if (!h) return MM_ERR_ARG;
    Handle* c = static_cast<Handle*>(h);
    try {
        return f(*c);
    } catch (const DeviceError& e) {
        char buf[256];
        std::snprintf(buf, sizeof buf, "HIP error %d (%s) at %s:%d", (int)e.err, hipGetErrorString(e.err), e.expr,
                      e.line);
        c->set_error(buf);
        return MM_ERR_DEVICE;
    } catch (const std::bad_alloc&) {
        c->set_error("out of host memory");
        return MM_ERR_INDEX;
    } catch (const std::exception& e) {  // nothing may unwind into the cgo caller
        c->set_error(std::string("internal error: ") + e.what());
        return MM_ERR_INDEX;
    } catch (...) {
        c->set_error("internal error");
        return MM_ERR_INDEX;
    }
}
std::string S(const char* p) { return p ? std::string(p) : std::string(); }

// Pipelined delivery (nakama_mm.h): one thread per handle
// that hands each queued pass result to the caller's callback, in pass order,
// then frees it; the queue holds at most `depth` results (push blocks beyond:
// back-pressure).  The handle itself is untouched — a queued result is an
// ordinary outstanding mm_matched (a second one takes private copies).
struct Delivery {
    Handle* h;
    mm_deliver_fn fn;
    void* ctx;
    size_t depth;
    std::mutex mu;
    std::condition_variable cv_item, cv_space, cv_idle;
    std::deque<std::pair<mm_matched, int64_t>> q;
    bool busy = false, quit = false;
    int64_t seq = 0;
    std::thread th;

    Delivery(Handle* hh, mm_deliver_fn f, void* c, size_t d) : h(hh), fn(f), ctx(c), depth(d) {
        th = std::thread([this] { loop(); });
    }
    ~Delivery() {
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
        }
        cv_item.notify_all();
        th.join();  // the loop delivers what is queued before it exits
    }
    void loop() {
        for (;;) {
            std::unique_lock<std::mutex> lk(mu);
            cv_item.wait(lk, [&] { return quit || !q.empty(); });
            if (q.empty()) return;  // quit, nothing left
            std::pair<mm_matched, int64_t> it = q.front();
            q.pop_front();
            busy = true;
            lk.unlock();
            cv_space.notify_all();
            fn(ctx, &it.first, it.second);
            (void)guarded(h, [&](Handle& c) { c.free_matched(&it.first); return MM_OK; });
            lk.lock();
            busy = false;
            lk.unlock();
            cv_idle.notify_all();
        }
    }
    void push(const mm_matched& m) {
        std::unique_lock<std::mutex> lk(mu);
        cv_space.wait(lk, [&] { return q.size() < depth; });
        q.emplace_back(m, seq++);
        lk.unlock();
        cv_item.notify_one();
    }
    void flush() {
        std::unique_lock<std::mutex> lk(mu);
        cv_idle.wait(lk, [&] { return q.empty() && !busy; });
    }
};
std::mutex g_deliv_mu;
// shared: a caller of push / flush holds its own reference, so a concurrent
// mm_set_delivery / mm_destroy cannot free the Delivery under it (the last
// reference joins the thread)
std::map<void*, std::shared_ptr<Delivery>> g_deliv;

std::shared_ptr<Delivery> delivery_of(void* h) {
    std::lock_guard<std::mutex> lk(g_deliv_mu);
    auto it = g_deliv.find(h);
    return it == g_deliv.end() ? nullptr : it->second;
}
// The calling thread is h's delivery thread (inside the callback): the calls
// that would join or wait for that thread are refused with MM_ERR_STATE.
bool on_delivery_thread(void* h) {
    std::lock_guard<std::mutex> lk(g_deliv_mu);
    auto it = g_deliv.find(h);
    return it != g_deliv.end() && it->second->th.get_id() == std::this_thread::get_id();
}
// the pass's counts and statistics without its arrays (the result is queued)
mm_matched summary_of(const mm_matched& m) {
    mm_matched s = m;
    s.group_offsets = nullptr;
    s.entries = nullptr;
    s.group_created = nullptr;
    s.reserved2 = 0;
    return s;
}
}  // namespace

void nkm::set_create_error(const std::string& e) { g_create_error = e; }

extern "C" {

int mm_abi_version(void) { return MM_ABI_VERSION; }
const char* mm_backend_name(void) { return "hip-gfx950"; }

void* mm_create(const mm_config* cfg) {
    if (!cfg) return nullptr;
    try {
        return static_cast<Handle*>(new Core(*cfg));
    } catch (const DeviceError& e) {
        g_create_error = std::string("mm_create: ") + hipGetErrorString(e.err);
        return nullptr;
    } catch (const std::exception& e) {
        g_create_error = std::string("mm_create: ") + e.what();
        return nullptr;
    } catch (...) {
        g_create_error = "mm_create: internal error";
        return nullptr;
    }
}
void mm_destroy(void* h) {
    try {
        if (on_delivery_thread(h)) return;  // from the callback: refused (the header forbids it)
        std::shared_ptr<Delivery> d;
        {
            std::lock_guard<std::mutex> lk(g_deliv_mu);
            auto it = g_deliv.find(h);
            if (it != g_deliv.end()) {
                d = std::move(it->second);
                g_deliv.erase(it);
            }
        }
        d.reset();  // the queued results are delivered and freed first
        delete static_cast<Handle*>(h);
    } catch (...) {
    }
}
void mm_pause(void* h) { if (h) static_cast<Handle*>(h)->pause(); }
void mm_resume(void* h) { if (h) static_cast<Handle*>(h)->resume(); }
void mm_stop(void* h) { if (h) static_cast<Handle*>(h)->stop(); }
const char* mm_last_error(void* h) { return h ? static_cast<Handle*>(h)->last_error() : g_create_error.c_str(); }

int mm_add(void* h, const mm_ticket* t) {
    if (!t) return MM_ERR_ARG;
    return guarded(h, [&](Handle& c) { return c.add(*t); });
}
int mm_insert(void* h, const mm_ticket* ts, int32_t n) {
    if (n > 0 && !ts) return MM_ERR_ARG;
    return guarded(h, [&](Handle& c) { return c.insert(ts, n); });
}
int mm_extract(void* h, mm_extract_list* out) {
    if (!out) return MM_ERR_ARG;
    return guarded(h, [&](Handle& c) { return c.extract(out); });
}
void mm_free_extract(void* h, mm_extract_list* out) {
    (void)guarded(h, [&](Handle& c) { c.free_extract(out); return MM_OK; });
}
int mm_remove_session(void* h, const char* session_id, const char* ticket) {
    return guarded(h, [&](Handle& c) { return c.remove_session(S(session_id), S(ticket)); });
}
int mm_remove_session_all(void* h, const char* session_id) {
    return guarded(h, [&](Handle& c) { return c.remove_session_all(S(session_id)); });
}
int mm_remove_party(void* h, const char* party_id, const char* ticket) {
    return guarded(h, [&](Handle& c) { return c.remove_party(S(party_id), S(ticket)); });
}
int mm_remove_party_all(void* h, const char* party_id) {
    return guarded(h, [&](Handle& c) { return c.remove_party_all(S(party_id)); });
}
int mm_remove_all(void* h, const char* node) {
    return guarded(h, [&](Handle& c) { return c.remove_all(S(node)); });
}
int mm_remove(void* h, const char* const* tickets, int32_t n) {
    if (n > 0 && !tickets) return MM_ERR_ARG;
    return guarded(h, [&](Handle& c) { return c.remove(tickets, n); });
}
int mm_process(void* h, mm_matched* out) {
    if (!out) return MM_ERR_ARG;
    return guarded(h, [&](Handle& c) { return c.process(out); });
}
int mm_process_commit(void* h, const int32_t* group_offsets, const mm_entry_ref* entries, int32_t n_groups,
                      mm_matched* out) {
    if (!out || (n_groups > 0 && (!group_offsets || !entries))) return MM_ERR_ARG;
    return guarded(h, [&](Handle& c) { return c.process_commit(group_offsets, entries, n_groups, out); });
}
void mm_free_matched(void* h, mm_matched* out) {
    (void)guarded(h, [&](Handle& c) { c.free_matched(out); return MM_OK; });
}
int mm_set_delivery(void* h, mm_deliver_fn fn, void* ctx, int32_t depth) {
    if (!h || (fn && depth < 1)) return MM_ERR_ARG;
    if (on_delivery_thread(h)) return MM_ERR_STATE;  // it would join its own thread
    try {
        std::shared_ptr<Delivery> old;
        {
            std::lock_guard<std::mutex> lk(g_deliv_mu);
            auto it = g_deliv.find(h);
            if (it != g_deliv.end()) {
                old = std::move(it->second);
                g_deliv.erase(it);
            }
        }
        old.reset();  // its queue delivered, its thread joined
        if (fn) {
            std::shared_ptr<Delivery> d = std::make_shared<Delivery>(static_cast<Handle*>(h), fn, ctx, (size_t)depth);
            std::lock_guard<std::mutex> lk(g_deliv_mu);
            g_deliv[h] = std::move(d);
        }
        return MM_OK;
    } catch (...) {
        static_cast<Handle*>(h)->set_error("mm_set_delivery: could not start the delivery thread");
        return MM_ERR_INDEX;
    }
}
int mm_process_deliver(void* h, mm_matched* summary) {
    if (!summary) return MM_ERR_ARG;
    const std::shared_ptr<Delivery> d = delivery_of(h);
    if (!d) return h ? MM_ERR_STATE : MM_ERR_ARG;
    mm_matched m{};
    const int rc = guarded(h, [&](Handle& c) { return c.process(&m); });
    if (rc != MM_OK) return rc;
    if (m.is_candidates) {  // processCustom: the override chooses first (mm_process_commit_deliver)
        *summary = m;
        return MM_OK;
    }
    *summary = summary_of(m);
    d->push(m);
    return MM_OK;
}
int mm_process_commit_deliver(void* h, const int32_t* group_offsets, const mm_entry_ref* entries, int32_t n_groups,
                              mm_matched* summary) {
    if (!summary || (n_groups > 0 && (!group_offsets || !entries))) return MM_ERR_ARG;
    const std::shared_ptr<Delivery> d = delivery_of(h);
    if (!d) return h ? MM_ERR_STATE : MM_ERR_ARG;
    mm_matched m{};
    const int rc = guarded(h, [&](Handle& c) { return c.process_commit(group_offsets, entries, n_groups, &m); });
    if (rc != MM_OK) return rc;
    *summary = summary_of(m);
    d->push(m);
    return MM_OK;
}
int mm_delivery_flush(void* h) {
    if (on_delivery_thread(h)) return MM_ERR_STATE;  // it would wait for itself
    const std::shared_ptr<Delivery> d = delivery_of(h);
    if (!d) return h ? MM_ERR_STATE : MM_ERR_ARG;
    d->flush();
    return MM_OK;
}
int32_t mm_ticket_count(void* h) {
    int32_t n = -1;
    (void)guarded(h, [&](Handle& c) { n = c.ticket_count(); return MM_OK; });
    return n;
}
int32_t mm_active_count(void* h) {
    int32_t n = -1;
    (void)guarded(h, [&](Handle& c) { n = c.active_count(); return MM_OK; });
    return n;
}
int32_t mm_session_ticket_count(void* h, const char* session_id) {
    int32_t n = -1;
    const int rc = guarded(h, [&](Handle& c) { n = c.session_ticket_count(S(session_id)); return MM_OK; });
    return rc == MM_OK ? n : rc;
}
int32_t mm_party_ticket_count(void* h, const char* party_id) {
    int32_t n = -1;
    const int rc = guarded(h, [&](Handle& c) { n = c.party_ticket_count(S(party_id)); return MM_OK; });
    return rc == MM_OK ? n : rc;
}
int32_t mm_find_tickets(void* h, const char* const* tickets, int32_t n, uint8_t* found) {
    if (n < 0 || (n > 0 && (!tickets || !found))) return MM_ERR_ARG;
    int32_t k = 0;
    const int rc = guarded(h, [&](Handle& c) { k = c.find_tickets(tickets, n, found); return MM_OK; });
    return rc == MM_OK ? k : rc;
}
int mm_drain_removed(void* h, mm_str_list* out) {
    if (!out) return MM_ERR_ARG;
    return guarded(h, [&](Handle& c) { return c.drain_removed(out); });
}
void mm_free_str_list(void* h, mm_str_list* out) {
    (void)guarded(h, [&](Handle& c) { c.free_str_list(out); return MM_OK; });
}
void mm_debug_set_pass_hook(void* h, void (*fn)(void*), void* ctx) {
    (void)guarded(h, [&](Handle& c) { c.set_pass_hook(fn, ctx); return MM_OK; });
}
int mm_shard_rows(void* h, int32_t world, int32_t rank, mm_allgather_fn fn, void* ctx) {
    return guarded(h, [&](Handle& c) { return c.set_row_shard(world, rank, fn, ctx); });
}
int mm_shard_rows_rccl(void* h, int32_t world, int32_t rank, const uint8_t* uid, int32_t len) {
    return guarded(h, [&](Handle& c) { return c.set_row_shard_rccl(world, rank, uid, len); });
}
int32_t mm_debug_hits(void* h, const char* ticket, const char** tickets_out, double* scores_out, int32_t cap) {
    int32_t r = -1;
    int rc = guarded(h, [&](Handle& c) {
        r = c.debug_hits(S(ticket), tickets_out, scores_out, cap);
        return MM_OK;
    });
    return rc == MM_OK ? r : rc;
}

}  // extern "C"
