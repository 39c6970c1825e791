// nakama_amd/csrc/mm_finish.cpp — the pass's post-pass (matchmaker.go:
// 320-372): expiry, the completeness re-check with the reference's
// swap-remove, retirement of matched tickets, and the result arena.
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

// Process() post-pass (matchmaker.go:320-372).
// Post-pass bookkeeping (matchmaker.go:320-375).  `disjoint`: no ticket is in
// two groups (the default pass's selection guarantees it; an override's
// groups may overlap and then follow the reference's sequential order, where
// a group meeting an already-retired ticket is dropped).
void Core::finish_pass(const UVec<uint32_t>& expired, GroupList& groups, bool disjoint) {
    using fclk = std::chrono::steady_clock;
    const auto f0 = fclk::now();
    auto f_ms = [](fclk::time_point a, fclk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    fclk::time_point f1 = f0, f2 = f0;
    for (uint32_t s : expired) is_active_[s] = 0;
    const size_t ngr = groups.size();
    if (!disjoint || !par_mode_ || ngr < par_min(16384)) {
        finish_pass_serial(groups, disjoint);
    } else {
        WorkPool& wp = workers();
        const size_t nchunk = wp.size();
        // a group is incomplete when one of its tickets left the index
        std::vector<uint8_t> incomplete(ngr, 0);
        wp.run(nchunk, [&](size_t c) {
            for (size_t g = ngr * c / nchunk; g < ngr * (c + 1) / nchunk; g++)
                for (const auto* e = groups.begin(g); e != groups.end(g); ++e)
                    if (e->first == kNoSlot || !live_[e->first]) { incomplete[g] = 1; break; }
        });
        // group order after the reference's swap-removes (:337-341)
        std::vector<uint32_t> order(ngr);
        for (uint32_t i = 0; i < order.size(); i++) order[i] = i;
        bool removed = false;
        for (size_t i = 0; i < order.size(); i++) {
            if (incomplete[order[i]]) {
                // its members were deleted from the search index when the pass
                // selected them (matchmaker_process.go:306-321) and stay out of
                // it: they remain in m.indexes and may still search
                for (const auto* e = groups.begin(order[i]); e != groups.end(order[i]); ++e)
                    if (e->first != kNoSlot && live_[e->first]) indexed_[e->first] = 0;
                order[i] = order.back();
                order.pop_back();
                removed = true;
                i--;
            }
        }
        if (removed) {
            GroupList kept;
            for (uint32_t g : order) kept.push(groups.begin(g), groups.end(g));
            groups = std::move(kept);
        }
        f1 = fclk::now();
        // Retire the matched tickets.  When no session or party holds more
        // than one ticket, a retired slot left in sessionTickets /
        // partyTickets counts as absent (SlotSets reads live_), so retiring is
        // clearing the flags, in parallel chunks of whole groups.
        if (sess_slots_.more.empty() && party_slots_.more.empty()) {
            const size_t ng2 = groups.size();
            std::vector<uint32_t> killed(nchunk, 0);
            wp.run(nchunk, [&](size_t c) {
                uint32_t k = 0;
                const size_t e0 = groups.off[ng2 * c / nchunk], e1 = groups.off[ng2 * (c + 1) / nchunk];
                for (size_t i = e0; i < e1; i++) {
                    const uint32_t s = groups.ents[i].first;
                    if (!live_[s]) continue;  // a ticket's presence entries repeat its slot
                    live_[s] = 0;
                    is_active_[s] = 0;
                    k++;
                }
                killed[c] = k;
            });
            for (uint32_t k : killed) n_live_ -= k;
        } else {
            for (auto& e : groups.ents) kill_slot(e.first, true, true);  // matched: in the result, not the drain
        }
        f2 = fclk::now();
    }
    filter_slots(big_list(active_list_) ? &workers() : nullptr, active_list_, list_tmp_,
                 [&](uint32_t s) { return live_[s] && is_active_[s]; });
    active_list_.swap(list_tmp_);
    active_exact_ = true;
    if (batch_profile_)
        std::fprintf(stderr, "[nkm]   finish: expired %zu, checks/order %.2f, retire %.2f, active filter %.2f ms\n",
                     expired.size(), f_ms(f0, f1), f_ms(f1, f2), f_ms(f2 > f0 ? f2 : f0, fclk::now()));
}

// finish_pass(expired, groups, true) + fill_matched(groups, out, false) for
// the common large processDefault pass — no group lost a ticket, no session or
// party holds two tickets, the output arena is free — in two parallel sweeps:
// the completeness re-check (matchmaker.go:326-343) over every group, then
// per chunk of groups the result entries and the retirement of their tickets
// (groups are disjoint, so the sweeps see the state the serial loop would).
// Returns false, having changed nothing but the expired tickets' active flags
// (finish_pass sets them again), when a condition fails.
bool Core::finish_fill_fast(const UVec<uint32_t>& expired, GroupList& groups, mm_matched* out, bool mutated) {
    const size_t ng = groups.size(), ne = groups.ents.size();
    if (!par_mode_ || ng < par_min(16384) || !sess_slots_.more.empty() || !party_slots_.more.empty()) return false;
    if (!arena_claimed_ && out_in_use_.exchange(true)) return false;  // a second outstanding result: fill_matched copies
    arena_claimed_ = true;
    const bool filled = filled_groups_ == ng;  // the pipelined merge wrote the result entries
    const auto f0 = std::chrono::steady_clock::now();
    WorkPool& wp = workers();
    const size_t nch = (size_t)wp.size() * 2;
    std::vector<uint8_t> bad(nch, 0);
    const size_t nx = expired.size();
    // Without a mutation queued during the pass no member left the index
    // (groups are formed from live tickets only): every group is complete
    // and the re-check is skipped; the retire sweep clears the expired flags.
    if (mutated) {
        wp.run(nch, [&](size_t c) {
            for (size_t i = nx * c / nch; i < nx * (c + 1) / nch; i++) is_active_[expired[i]] = 0;
            for (size_t g = ng * c / nch; g < ng * (c + 1) / nch && !bad[c]; g++)
                for (const auto* e = groups.begin(g); e != groups.end(g); ++e)
                    if (e->first == kNoSlot || !live_[e->first]) { bad[c] = 1; break; }
        });
        for (uint8_t b : bad)
            if (b) return false;  // fill_matched, on the claimed arena, after finish_pass's re-check
    }
    if (out_offs_.size() < ng + 1) grow_to(out_offs_, ng + 1);
    if (out_ents_.size() < std::max<size_t>(ne, 1)) grow_to(out_ents_, std::max<size_t>(ne, 1));
    if (out_created_.size() < std::max<size_t>(ng, 1)) grow_to(out_created_, std::max<size_t>(ng, 1));
    int32_t* offs = out_offs_.data();
    mm_entry_ref* ents = out_ents_.data();
    int64_t* gc = out_created_.data();
    std::vector<uint32_t> killed(nch, 0);
    std::vector<double> task_us(nch, 0.0), start_us(nch, 0.0);  // NKM_PROFILE=2: the job's own time vs its wall
    // Without a mutation, the matched tickets are exactly the pass's selection
    // (sel_): retired by one sequential sweep over the slots instead of
    // scattered writes per result entry
    const size_t N = nslots();
    const bool by_slot = !mutated && sel_.size() == N;
    wp.run(nch, [&](size_t c) {
        const auto tc0 = std::chrono::steady_clock::now();
        const size_t g0 = ng * c / nch, g1 = ng * (c + 1) / nch;
        uint32_t k = 0;
        if (!mutated)
            for (size_t i = nx * c / nch; i < nx * (c + 1) / nch; i++) is_active_[expired[i]] = 0;
        if (!filled) {
            for (size_t g = g0; g < g1; g++) {
                offs[g] = (int32_t)groups.off[g];
                gc[g] = groups.len(g) ? created_[groups.end(g)[-1].first] : 0;
            }
            if (c + 1 == nch) offs[ng] = (int32_t)groups.off[ng];
            for (size_t i = groups.off[g0]; i < groups.off[g1]; i++) {
                const uint32_t s = groups.ents[i].first;
                ents[i].ticket = tk_ptr_[s];
                ents[i].presence_index = groups.ents[i].second;
                ents[i].reserved = 0;
            }
        }
        if (by_slot) {
            // the arrays in locals: a byte store may alias a member vector's
            // pointer, which would then be reloaded after every store
            const uint8_t* const S = sel_.data();
            uint8_t* const L = live_.data();
            uint8_t* const A = is_active_.data();
            // (conditional stores: another task clears is_active_ of this
            // range's expired slots meanwhile, which a read-modify-write of
            // every byte here could undo)
            for (size_t s = N * c / nch; s < N * (c + 1) / nch; s++)
                if (S[s] & L[s]) {
                    L[s] = 0;  // retired: sessionTickets / partyTickets read live_ (SlotSets)
                    A[s] = 0;
                    k++;
                }
        } else {
            for (size_t i = groups.off[g0]; i < groups.off[g1]; i++) {
                const uint32_t s = groups.ents[i].first;
                if (!live_[s]) continue;  // a ticket's presence entries repeat its slot
                live_[s] = 0;
                is_active_[s] = 0;
                k++;
            }
        }
        killed[c] = k;
        const auto tc1 = std::chrono::steady_clock::now();
        start_us[c] = std::chrono::duration<double, std::micro>(tc0 - f0).count();
        task_us[c] = std::chrono::duration<double, std::micro>(tc1 - tc0).count();
    });
    const auto f1 = std::chrono::steady_clock::now();
    for (uint32_t k : killed) n_live_ -= k;
    filter_slots(big_list(active_list_) ? &workers() : nullptr, active_list_, list_tmp_,
                 [&](uint32_t s) { return live_[s] && is_active_[s]; });
    active_list_.swap(list_tmp_);
    active_exact_ = true;
    if (const char* p = std::getenv("NKM_PROFILE"); p && std::atoi(p) >= 2) {
        auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "[nkm]   finish: retire %.3f ms (%s, %s; its tasks: max %.0f us, last start %.0f us) | "
                     "filter %.3f ms (%zu active)\n", ms(f0, f1),
                     by_slot ? "by slot" : "by entry", filled ? "filled" : "fill",
                     *std::max_element(task_us.begin(), task_us.end()), *std::max_element(start_us.begin(), start_us.end()),
                     ms(f1, std::chrono::steady_clock::now()), active_list_.size());
    }
    out->group_created = gc;
    out->n_groups = (int32_t)ng;
    out->n_entries = (int32_t)ne;
    out->group_offsets = offs;
    out->entries = ents;
    out->is_candidates = 0;
    out->reserved2 = 1;  // the handle's arena (out_in_use_ until mm_free_matched)
    arena_claimed_ = false;
    return true;
}

void Core::finish_pass_serial(GroupList& groups, bool selected) {
    std::vector<uint32_t> order(groups.size());
    for (uint32_t i = 0; i < order.size(); i++) order[i] = i;
    bool removed = false;
    for (size_t i = 0; i < order.size(); i++) {
        bool incomplete = false;
        for (const auto* e = groups.begin(order[i]); e != groups.end(order[i]); ++e)
            if (e->first == kNoSlot || !live_[e->first]) { incomplete = true; break; }
        if (incomplete) {  // swap-remove (:337-341)
            // processDefault deleted the members from the search index when it
            // selected them (matchmaker_process.go:306-321): they stay out of it
            if (selected)
                for (const auto* e = groups.begin(order[i]); e != groups.end(order[i]); ++e)
                    if (e->first != kNoSlot && live_[e->first]) indexed_[e->first] = 0;
            order[i] = order.back();
            order.pop_back();
            removed = true;
            i--;
            continue;
        }
        for (const auto* e = groups.begin(order[i]); e != groups.end(order[i]); ++e) kill_slot(e->first, true, true);
    }
    if (removed) {
        GroupList kept;
        for (uint32_t g : order) kept.push(groups.begin(g), groups.end(g));
        groups = std::move(kept);
    }
}

void Core::fill_matched(const GroupList& groups, mm_matched* out,
                        bool cands) {
    const size_t n = groups.ents.size();
    // The handle's arena (reused: its pages stay mapped) points entries at the
    // store's ticket-string arena, which does not move while the result is
    // outstanding (compaction waits for mm_free_matched).  A second
    // outstanding result gets private copies.
    const bool arena = arena_claimed_ || !out_in_use_.exchange(true);
    arena_claimed_ = false;
    int32_t* offs;
    mm_entry_ref* ents;
    char* buf = nullptr;
    if (arena) {
        if (out_offs_.size() < groups.size() + 1) grow_to(out_offs_, groups.size() + 1);
        if (out_ents_.size() < std::max<size_t>(n, 1)) grow_to(out_ents_, std::max<size_t>(n, 1));
        offs = out_offs_.data();
        ents = out_ents_.data();
    } else {
        size_t bytes = 0;
        for (auto& e : groups.ents) bytes += tk_len_[e.first] + 1;
        offs = new int32_t[groups.size() + 1];
        ents = new mm_entry_ref[n ? n : 1];
        buf = new char[bytes ? bytes : 1];
    }
    int64_t* gc;  // per group: its last entry's CreatedAt (the cluster merge's key)
    if (arena) {
        if (out_created_.size() < std::max<size_t>(groups.size(), 1)) grow_to(out_created_, std::max<size_t>(groups.size(), 1));
        gc = out_created_.data();
    } else {
        gc = new int64_t[groups.size() ? groups.size() : 1];
    }
    auto created_of = [&](size_t g) {
        const uint32_t last = groups.len(g) ? groups.end(g)[-1].first : kNoSlot;
        gc[g] = last == kNoSlot ? 0 : created_[last];
    };
    size_t b = 0;
    if (arena && par_mode_ && n >= par_min(65536)) {  // chunks of the result in parallel
        WorkPool& wp = workers();
        const size_t nch = wp.size(), ng = groups.size() + 1;
        wp.run(nch, [&](size_t c) {
            for (size_t gi = ng * c / nch; gi < ng * (c + 1) / nch; gi++) {
                offs[gi] = (int32_t)groups.off[gi];
                if (gi < ng - 1) created_of(gi);
            }
            for (size_t k = n * c / nch; k < n * (c + 1) / nch; k++) {
                const auto& e = groups.ents[k];
                ents[k].ticket = tk_ptr_[e.first];
                ents[k].presence_index = e.second;
                ents[k].reserved = 0;
            }
        });
    } else {
        for (size_t gi = 0; gi <= groups.size(); gi++) offs[gi] = (int32_t)groups.off[gi];
        for (size_t g = 0; g < groups.size(); g++) created_of(g);
        uint32_t prev = kNoSlot;
        const char* prev_p = nullptr;
        for (size_t k = 0; k < n; k++) {
            const auto& e = groups.ents[k];
            if (e.first != prev) {
                if (arena) {
                    prev_p = tk_ptr_[e.first];
                } else {
                    std::memcpy(buf + b, tk_ptr_[e.first], tk_len_[e.first] + 1);
                    prev_p = buf + b;
                    b += tk_len_[e.first] + 1;
                }
                prev = e.first;
            }
            ents[k].ticket = prev_p;
            ents[k].presence_index = e.second;
            ents[k].reserved = 0;
        }
    }
    out->group_created = gc;
    out->n_groups = (int32_t)groups.size();
    out->n_entries = (int32_t)n;
    out->group_offsets = offs;
    out->entries = ents;
    out->is_candidates = cands ? 1 : 0;
    out->reserved2 = arena ? 1 : (int64_t)(intptr_t)buf;  // 1: the handle's arena
}

// processCustom's candidates (enum_kernel's write pass: entries as (slot,
// presence) word pairs in d_eents_, group ends in d_eoff_) straight into the
// result arena, which the caller claimed: the group ends first, then the
// entries in chunks through two pinned buffers — chunk k + 1 copies while the
// workers turn chunk k into result entries (ticket string, presence) and set
// the CreatedAt of every group that ends in it.  Replaces one pageable copy
// of the whole list (1.12 GB on C5's 35M candidates) plus fill_matched's pass
// over it.  process() then hands the arena out (custom_filled_).
void Core::fill_custom_direct(size_t G, size_t E, bool slots) {
    // slots: the write pass gave slot ids alone (every presence index 0) and
    // a byte of size per group (enum_kernel<false, true>); else (slot,
    // presence) word pairs and group ends
    WorkPool& wp = workers();
    if (!ech_ev_[0])
        for (auto& e : ech_ev_) NKM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (out_offs_.size() < G + 1) grow_to(out_offs_, G + 1);
    if (out_ents_.size() < E) grow_to(out_ents_, E);
    if (out_created_.size() < G) grow_to(out_created_, G);
    int32_t* offs = out_offs_.data();
    mm_entry_ref* ents = out_ents_.data();
    int64_t* gc = out_created_.data();
    const size_t off_bytes = slots ? G : G * sizeof(uint32_t);
    h_eoff_.reserve((off_bytes + 3) / 4);
    NKM_HIP(hipMemcpyAsync(h_eoff_.p, d_eoff_.p, off_bytes, hipMemcpyDeviceToHost, stream_));
    const size_t W = slots ? 1 : 2;  // words per entry
    const size_t kChunk = (size_t)1 << 23;  // entries per chunk (32 / 64 MB)
    const size_t nck = (E + kChunk - 1) / kChunk;
    for (auto& b : h_ech_) b.reserve(W * std::min(kChunk, E));
    auto issue = [&](size_t k) {
        const size_t lo = k * kChunk, n = std::min(kChunk, E - lo);
        NKM_HIP(hipMemcpyAsync(h_ech_[k & 1].p, d_eents_.p + W * lo, n * W * sizeof(uint32_t), hipMemcpyDeviceToHost,
                               stream_));
        NKM_HIP(hipEventRecord(ech_ev_[k & 1], stream_));
    };
    issue(0);
    if (nck > 1) issue(1);
    NKM_HIP(hipStreamSynchronize(stream_));  // the group ends / sizes (and the first chunks) are down
    const size_t nch = (size_t)wp.size() * 2;
    if (slots) {  // sizes -> ends: chunk sums, then every chunk's running ends
        const uint8_t* sz = reinterpret_cast<const uint8_t*>(h_eoff_.p);
        std::vector<uint64_t> at(nch + 1, 0);
        wp.run(nch, [&](size_t c) {
            uint64_t t = 0;
            for (size_t g = G * c / nch; g < G * (c + 1) / nch; g++) t += sz[g];
            at[c + 1] = t;
        });
        for (size_t c = 0; c < nch; c++) at[c + 1] += at[c];
        if (at[nch] != E) throw std::logic_error("processCustom: group sizes do not add up to the entries");
        wp.run(nch, [&](size_t c) {
            uint64_t t = at[c];
            if (c == 0) offs[0] = 0;
            for (size_t g = G * c / nch; g < G * (c + 1) / nch; g++) offs[g + 1] = (int32_t)(t += sz[g]);
        });
    } else {
        wp.run(nch, [&](size_t c) {
            const size_t g0 = G * c / nch, g1 = G * (c + 1) / nch;
            if (c == 0) offs[0] = 0;
            for (size_t g = g0; g < g1; g++) offs[g + 1] = (int32_t)h_eoff_.p[g];
        });
    }
    for (size_t k = 0; k < nck; k++) {
        NKM_HIP(hipEventSynchronize(ech_ev_[k & 1]));
        const uint32_t* w = h_ech_[k & 1].p;
        const size_t lo = k * kChunk, n = std::min(kChunk, E - lo);
        wp.run(nch, [&](size_t c) {
            const size_t a = lo + n * c / nch, b = lo + n * (c + 1) / nch;
            // streaming stores: 2.24 GB of result entries on C5 + override
            // never fit a cache, and a normal store reads each line first
            typedef long long v2i __attribute__((vector_size(16)));
            static_assert(sizeof(mm_entry_ref) == 16 && alignof(mm_entry_ref) <= 16, "16-B result entries");
            v2i* dst = reinterpret_cast<v2i*>(ents);
            for (size_t i = a; i < b; i++) {
                const uint32_t slot = w[W * (i - lo)];
                const long long pi = slots ? 0 : (long long)(uint32_t)w[W * (i - lo) + 1];  // presence_index, reserved = 0
                const v2i v = {(long long)(intptr_t)tk_ptr_[slot], pi};
                __builtin_nontemporal_store(v, dst + i);
            }
            std::atomic_thread_fence(std::memory_order_seq_cst);  // this worker's streaming stores drained
            // groups whose last entry (the searching ticket) lies in [a, b): end in (a, b]
            size_t g = (size_t)(std::upper_bound(offs + 1, offs + 1 + G, (int32_t)a) - (offs + 1));
            for (; g < G && (size_t)offs[g + 1] <= b; g++) gc[g] = created_[w[W * ((size_t)offs[g + 1] - 1 - lo)]];
        });
        if (k + 2 < nck) issue(k + 2);  // into the buffer just converted
    }
    custom_filled_ = true;
    custom_filled_g_ = G;
    custom_filled_e_ = E;
}

void Core::free_matched(mm_matched* out) {
    if (!out) return;
    if (out->reserved2 == 1) {
        out_in_use_.store(false);
    } else if (out->reserved2 != 0 || out->group_offsets) {
        delete[] out->group_offsets;
        delete[] out->entries;
        delete[] out->group_created;
        delete[] reinterpret_cast<char*>((intptr_t)out->reserved2);
    }
    std::memset(out, 0, sizeof(*out));
}


}  // namespace nkm
