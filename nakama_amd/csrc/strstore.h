// nakama_amd/csrc/strstore.h — allocation-free string storage for the ticket
// store: interned dictionaries, the ticket-id index and the per-ticket cold
// records (presences, properties, query text) kept for Extract and the
// effective-state checks.
//
// LocalMatchmaker keeps its tickets as Go maps of structs of strings
// (server/matchmaker.go:185-212, MatchmakerExtract 106-120); a C++ restatement
// with std::unordered_map<std::string,…> and per-ticket std::string/std::vector
// members costs ~20 heap allocations per ticket on Insert and as many frees at
// compaction, which dominated a 1M-ticket Insert.  Here every string lives in
// a few large byte arenas and every index is an open-addressing table of
// 64-bit words, so adding a ticket touches no allocator in the steady state
// and dropping a million dead tickets frees a handful of blocks.
#pragma once
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <type_traits>
#include <utility>
#include <vector>

namespace nkm {

// std::allocator whose value-less construct() default-initialises, so
// resize() of trivially constructible elements leaves them unwritten: the
// pass's output arrays are filled in full by the parallel merges, and
// std::vector's value-initialisation was a serial zero-fill of the whole
// output ahead of them (C3: 21 MB per pass); the bulk Insert's cold records
// likewise (C3 1M: ~400 MB).
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInitAlloc<U>;
    };
    DefaultInitAlloc() = default;
    template <class U>
    DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};

// 64-bit hash of a byte string (8 bytes per step, multiply-xorshift mixing).
inline uint64_t str_hash(const char* p, size_t n) {
    constexpr uint64_t k = 0x9E3779B97F4A7C15ull;
    uint64_t h = 0x243F6A8885A308D3ull ^ (n * k);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        std::memcpy(&w, p + i, 8);
        h = (h ^ w) * k;
        h ^= h >> 29;
    }
    if (i < n) {
        uint64_t w = 0;
        std::memcpy(&w, p + i, n - i);
        h = (h ^ w) * k;
        h ^= h >> 29;
    }
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 32);
}
inline uint64_t str_hash(std::string_view s) { return str_hash(s.data(), s.size()); }

// Append-only NUL-terminated strings in 1 MiB blocks that never move.
struct StrArena {
    std::vector<std::unique_ptr<char[]>> blocks;
    size_t used = 0, cap = 0;
    const char* put(std::string_view s) {
        const size_t need = s.size() + 1;
        if (blocks.empty() || used + need > cap) {
            cap = std::max<size_t>(size_t(1) << 20, need);
            blocks.emplace_back(new char[cap]);
            used = 0;
        }
        char* p = blocks.back().get() + used;
        if (!s.empty()) std::memcpy(p, s.data(), s.size());
        p[s.size()] = 0;
        used += need;
        return p;
    }
    // A block of exactly `bytes` the caller fills (a bulk append: the
    // Insert workers copy their strings into it in parallel); the next put()
    // starts a new block.
    char* block(size_t bytes) {
        blocks.emplace_back(new char[std::max<size_t>(bytes, 1)]);
        used = cap = std::max<size_t>(bytes, 1);
        return blocks.back().get();
    }
    void clear() {
        blocks.clear();
        used = cap = 0;
    }
};

// Open-addressing index of values (< 2^32 - 1) by a 64-bit key hash; the
// caller resolves collisions of the 32 stored hash bits with `eq(value)`.
// An entry's position derives from its stored tag (the hash's high half), so a
// rehash needs no keys.
struct HashIndex {
    std::vector<uint64_t> tab;  // tag << 32 | (value + 1); 0 = empty
    size_t n = 0;
    template <class Eq>
    int64_t find(uint64_t h, Eq eq) const {
        if (tab.empty()) return -1;
        const size_t mask = tab.size() - 1;
        const uint32_t tag = (uint32_t)(h >> 32);
        for (size_t i = tag & mask;; i = (i + 1) & mask) {
            const uint64_t e = tab[i];
            if (!e) return -1;
            if ((uint32_t)(e >> 32) == tag && eq((uint32_t)e - 1)) return (uint32_t)e - 1;
        }
    }
    // Inserts (h, v), or replaces the value of the entry eq matches.
    template <class Eq>
    void put(uint64_t h, uint32_t v, Eq eq) {
        if (2 * (n + 1) > tab.size()) rehash(tab.empty() ? 16 : tab.size() * 2);
        const size_t mask = tab.size() - 1;
        const uint32_t tag = (uint32_t)(h >> 32);
        const uint64_t word = ((uint64_t)tag << 32) | (uint64_t)(v + 1);
        for (size_t i = tag & mask;; i = (i + 1) & mask) {
            const uint64_t e = tab[i];
            if (!e) {
                tab[i] = word;
                n++;
                return;
            }
            if ((uint32_t)(e >> 32) == tag && eq((uint32_t)e - 1)) {
                tab[i] = word;
                return;
            }
        }
    }
    // Inserts a key the caller knows is absent.
    void put_new(uint64_t h, uint32_t v) {
        put(h, v, [](uint32_t) { return false; });
    }
    // put_new from several threads at once: keys absent and pairwise
    // distinct, capacity reserved beforehand (no rehash); each thread claims
    // an empty word with a compare-exchange.  The caller adds the count to n
    // after the threads are done.
    void put_new_concurrent(uint64_t h, uint32_t v) {
        const size_t mask = tab.size() - 1;
        const uint32_t tag = (uint32_t)(h >> 32);
        const uint64_t word = ((uint64_t)tag << 32) | (uint64_t)(v + 1);
        for (size_t i = tag & mask;; i = (i + 1) & mask) {
            uint64_t expect = 0;
            if (__atomic_load_n(&tab[i], __ATOMIC_RELAXED) == 0 &&
                __atomic_compare_exchange_n(&tab[i], &expect, word, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED))
                return;
        }
    }
    void reserve(size_t count) {
        size_t c = 16;
        while (c < 2 * count) c <<= 1;
        if (c > tab.size()) rehash(c);
    }
    void clear() {
        std::vector<uint64_t>().swap(tab);
        n = 0;
    }

private:
    void rehash(size_t c) {
        std::vector<uint64_t> old;
        old.swap(tab);
        tab.assign(c, 0);
        const size_t mask = c - 1;
        for (uint64_t e : old) {
            if (!e) continue;
            for (size_t i = (uint32_t)(e >> 32) & mask;; i = (i + 1) & mask)
                if (!tab[i]) {
                    tab[i] = e;
                    break;
                }
        }
    }
};

// Interned strings: id -> view (NUL-terminated), view -> id.
struct Dict {
    StrArena arena;
    std::vector<const char*> ptr;
    std::vector<uint32_t> len;
    HashIndex idx;
    size_t size() const { return ptr.size(); }
    std::string_view str(uint32_t id) const { return {ptr[id], len[id]}; }
    int64_t find(std::string_view s) const {
        return idx.find(str_hash(s), [&](uint32_t id) { return str(id) == s; });
    }
    uint32_t intern(std::string_view s) {
        const uint64_t h = str_hash(s);
        const int64_t f = idx.find(h, [&](uint32_t id) { return str(id) == s; });
        if (f >= 0) return (uint32_t)f;
        const uint32_t id = (uint32_t)ptr.size();
        ptr.push_back(arena.put(s));
        len.push_back((uint32_t)s.size());
        idx.put_new(h, id);
        return id;
    }
    void clear() {
        arena.clear();
        ptr.clear();
        len.clear();
        idx.clear();
    }
};

// Per-ticket cold record (session, party, query, presences, properties) as one
// length-prefixed byte record in an append-only buffer; records of dead slots
// are dropped when the store compacts.
//   u32 n_presences, n_str_props, n_num_props
//   str session_id, party_id, query
//   n_presences x (str user_id, session_id, username, node)
//   n_str_props x (str key, value)
//   n_num_props x (str key, f64 value)
// where str = u32 length + bytes + NUL.
struct ColdView {
    std::string_view session_id, party_id, query;
    uint32_t n_pres = 0, n_sp = 0, n_np = 0;
    const char* rest = nullptr;  // the presences, then the properties
    struct Cursor {
        const char* p;
        std::string_view str() {
            uint32_t n;
            std::memcpy(&n, p, 4);
            std::string_view v(p + 4, n);
            p += 4 + n + 1;
            return v;
        }
        double f64() {
            double d;
            std::memcpy(&d, p, 8);
            p += 8;
            return d;
        }
    };
    // fn(user_id, session_id, username, node)
    template <class Fn>
    const char* each_presence(Fn fn) const {
        Cursor c{rest};
        for (uint32_t i = 0; i < n_pres; i++) {
            auto u = c.str(), s = c.str(), n = c.str(), nd = c.str();
            fn(u, s, n, nd);
        }
        return c.p;
    }
    template <class S, class N>
    void each_prop(S fs, N fn) const {
        Cursor c{each_presence([](auto, auto, auto, auto) {})};
        for (uint32_t i = 0; i < n_sp; i++) {
            auto k = c.str(), v = c.str();
            fs(k, v);
        }
        for (uint32_t i = 0; i < n_np; i++) {
            auto k = c.str();
            fn(k, c.f64());
        }
    }
};

struct ColdStore {
    std::vector<char, DefaultInitAlloc<char>> bytes;  // resized then written (bulk Insert): no zero-fill
    std::vector<uint64_t> off;  // per slot
    size_t size() const { return off.size(); }

    struct Writer {
        std::vector<char, DefaultInitAlloc<char>>& b;
        void u32(uint32_t v) {
            const size_t at = b.size();
            b.resize(at + 4);
            std::memcpy(b.data() + at, &v, 4);
        }
        void str(const char* s) { str(std::string_view(s ? s : "")); }
        void str(std::string_view s) {
            const size_t at = b.size();
            b.resize(at + 4 + s.size() + 1);
            const uint32_t n = (uint32_t)s.size();
            std::memcpy(b.data() + at, &n, 4);
            if (n) std::memcpy(b.data() + at + 4, s.data(), n);
            b[at + 4 + n] = 0;
        }
        void f64(double d) {
            const size_t at = b.size();
            b.resize(at + 8);
            std::memcpy(b.data() + at, &d, 8);
        }
    };
    Writer begin() {
        off.push_back(bytes.size());
        return Writer{bytes};
    }
    ColdView view(uint32_t s) const { return parse(bytes.data() + off[s]); }
    static ColdView parse(const char* p) {
        ColdView v;
        std::memcpy(&v.n_pres, p, 4);
        std::memcpy(&v.n_sp, p + 4, 4);
        std::memcpy(&v.n_np, p + 8, 4);
        ColdView::Cursor c{p + 12};
        v.session_id = c.str();
        v.party_id = c.str();
        v.query = c.str();
        v.rest = c.p;
        return v;
    }
    size_t record_bytes(uint32_t s) const {
        return (s + 1 < off.size() ? off[s + 1] : bytes.size()) - off[s];
    }
    // Drops every record, keeping the buffers' capacity (a drained store:
    // the next Insert writes into pages already mapped)
    void clear() {
        bytes.clear();
        off.clear();
    }
    // Keeps the records of the slots where keep[s] (in slot order).
    void compact(const std::vector<uint8_t>& keep) {
        std::vector<char, DefaultInitAlloc<char>> nb;
        std::vector<uint64_t> no;
        size_t total = 0;
        for (uint32_t s = 0; s < off.size(); s++)
            if (keep[s]) total += record_bytes(s);
        nb.reserve(total);
        for (uint32_t s = 0; s < off.size(); s++) {
            if (!keep[s]) continue;
            no.push_back(nb.size());
            const size_t n = record_bytes(s);
            nb.insert(nb.end(), bytes.data() + off[s], bytes.data() + off[s] + n);
        }
        bytes.swap(nb);
        off.swap(no);
    }
};

}  // namespace nkm
