// nakama_amd/csrc/mm_pass.h — internal to the pass's translation units
// (mm_process.cpp: batches, searches, the serial replay; mm_pools.cpp: the
// pool-parallel replay and packed RevPrecision batches; mm_finish.cpp: the
// post-pass): batch limits and the order-preserving slot filter.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "mm_core.h"

namespace nkm {

constexpr size_t kMaxBatchRows = 1u << 22;  // a batch may hold C4's 4M rows

// Order-preserving filter of a slot list: on the workers in chunks (counts,
// then every chunk writes at its offset), or serially when wp is null.
template <class Keep>
inline void filter_slots(WorkPool* wp, const std::vector<uint32_t>& in, std::vector<uint32_t>& out, Keep keep) {
    const size_t n = in.size();
    if (!wp || wp->size() < 2) {
        out.clear();
        for (uint32_t s : in)
            if (keep(s)) out.push_back(s);
        return;
    }
    const size_t nch = wp->size();
    std::vector<size_t> at(nch + 1, 0);
    wp->run(nch, [&](size_t c) {
        size_t k = 0;
        for (size_t i = n * c / nch; i < n * (c + 1) / nch; i++) k += keep(in[i]) ? 1 : 0;
        at[c + 1] = k;
    });
    for (size_t c = 0; c < nch; c++) at[c + 1] += at[c];
    out.resize(at[nch]);
    wp->run(nch, [&](size_t c) {
        size_t o = at[c];
        for (size_t i = n * c / nch; i < n * (c + 1) / nch; i++)
            if (keep(in[i])) out[o++] = in[i];
    });
}
constexpr uint64_t kOutCap = 1ull << 24;  // max hit entries per batch (16M x 16 B)
constexpr uint32_t kFullVarMax = 16384;   // max source of a full-list variable-score search
constexpr uint64_t kTierMax = 16384;      // max entries of a top-tier list (search_kernel path 2)


}  // namespace nkm
