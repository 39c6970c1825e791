// nakama_amd/csrc/mm_device.h — HBM layout of the ticket store and the work
// descriptors of the query-eval kernels.  Shared by host code (.cpp) and the
// HIP kernels (.hip); plain structs only.
#pragma once
#include <cstdint>

// Helpers below compile for both sides in the kernels' translation unit and
// as plain host functions elsewhere.
#if defined(__HIPCC__)
#define NKM_HD __host__ __device__
#else
#define NKM_HD
#endif

namespace nkm {

constexpr uint32_t kNoParty = 0xFFFFFFFFu;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
constexpr uint32_t kMaxShardBlocks = 8;  // ranks of a row-sharded hashed scan (one node's GPUs)

// Column value kinds (one byte per (field, slot)).
enum : uint8_t { KIND_ABSENT = 0, KIND_KEYWORD = 1, KIND_NUMERIC = 2 };

// One compiled clause (32 B).  lo/hi: sortable int64 bounds (RANGE) or the
// numeric literal (NUMLIT, lo == hi); term: dictionary id of the keyword form
// (TERMSET: the matcher's set index).
struct DClause {
    int64_t lo;
    int64_t hi;
    double score;
    uint32_t term;
    uint16_t field;
    uint8_t op;     // ClauseOp
    uint8_t occur;  // Occur
};
static_assert(sizeof(DClause) == 32, "DClause is 32 bytes");

// Query of one slot (its ParsedQuery), used by the reverse (RevPrecision) check.
struct DQuery {
    uint32_t clause_off;
    uint16_t n_clauses;
    uint8_t kind;       // QueryKind
    uint8_t n_must_nz;  // 1 if the query has at least one MUST clause
};

// Read-only view of the device-resident SoA store passed to kernels.
struct DStore {
    const uint8_t* alive;       // [cap] 1 = in the index (not deleted / not selected)
    const int32_t* minc;        // [cap] MinCount
    const int32_t* maxc;        // [cap] MaxCount
    const uint32_t* party;      // [cap] dictionary id of PartyId, kNoParty for ""
    const DQuery* squery;       // [cap] per-slot parsed query descriptor
    const DClause* clauses;     // clause table (all signatures)
    const int64_t* const* fval; // [n_fields] -> [cap] keyword id or sortable int64
    const uint8_t* const* fkind;// [n_fields] -> [cap] KIND_*
    const uint32_t* order;      // scan order: slots sorted by (created key, slot)
    const uint32_t* postings;   // concatenated posting lists (slots, scan order)
    const uint32_t* tset_desc;  // [2 * n_sets] (offset, length) of each OP_TERMSET matcher's set
    const uint32_t* tset_ids;   // accepted keyword dictionary ids, ascending per set
    const double* tset_sc;      // the clause's score contribution for each accepted id
    uint32_t n_fields;          // entries of fval / fkind
};

// One search (a group of rows sharing a compiled signature, or one row).
struct DGroup {
    uint32_t clause_off;
    uint16_t n_clauses;
    uint8_t qkind;
    uint8_t var_score;     // 0: every hit scores the same (ordered compaction); 1: top-K by score
    int32_t tmin, tmax;    // searching ticket's Min/MaxCount (count-range musts)
    uint32_t tparty;       // kNoParty or dictionary id (party mustNot)
    uint32_t rev_slot;     // kNoSlot, or the searching ticket for the per-hit reverse check
    uint32_t src_kind;     // 0: order[], 1: postings[]
    uint32_t src_off;
    uint32_t src_len;
    uint32_t k;            // max entries to emit
    uint32_t path;         // 0: search_kernel; 1: rsmall_kernel (a short source, one wave per row);
                           // 2: a variable-score search as a top-tier list: search_kernel<0>
                           //    compacts its hits scoring ub_key in source order, then
                           //    search_kernel<kVarK> appends the top-K of the rest if room is left
    uint64_t out_off;      // first output entry
    int64_t ub_key;        // sortable key of an upper bound of any score (early exit)
    int64_t cur_key;       // pagination cursor: emit only entries after (cur_key, cur_idx)
    uint32_t cur_idx;
    uint32_t has_cursor;
};

static_assert(sizeof(DGroup) == 80, "DGroup layout");

// Per-group result.
struct DGroupResult {
    uint32_t count;     // entries written (<= k)
    uint32_t complete;  // 1: no further hit exists after the written ones
    uint32_t scanned;   // candidates examined
    uint32_t matched;   // candidates that passed the predicate (after the cursor)
    uint32_t live;      // scanned candidates still in the index (their columns were read)
    uint32_t pad;
};

// A multi-signature scan (mscan_kernel): the scan-order range, the fields the
// signatures' clauses read (clause.field indexes this list in the rewritten
// clause copies), and the (signature x chunk) output grid.
struct DMScan {
    uint32_t src_off, src_len;  // range of order[]
    uint32_t n_sigs, n_chunks;
    uint32_t n_fields;
    uint32_t n_clauses;         // of all the signatures
    uint16_t field[4];
    uint32_t chunk;             // candidates per chunk (workgroup): 2, 4 or 8 per lane
    uint32_t hmask;             // hashed lookup (mscan_hash_kernel): table entries - 1; 0: mscan_kernel
    uint32_t contig;            // hashed: order[p] == p over the range, chunks are slot ranges aligned
                                // to `chunk` from src_off rounded down
    uint32_t hseed[2];          // hashed: the two cuckoo hash seeds
    uint32_t pad;
    // hashed, direct lookup (dsize > 0): the key grid over the signatures'
    // values, cell = sum_f (value_f - dlo[f]) * prod_{g > f} drng[g]
    uint32_t dsize;
    uint32_t dlo[4], drng[4];
    // hashed, row-sharded: rank r evaluates chunks [cb[r], cb[r + 1]) and its
    // (n_sigs + 1) count columns are one contiguous block (mhash_cidx), so the
    // ranks' scratch and counts are all-gathered as one segment each.
    // n_blk <= 1: one block, the plain column-major layout.
    uint32_t n_blk;
    uint32_t cb[kMaxShardBlocks + 1];
};

// Index of the (column q, chunk c) count of a hashed scan (see DMScan::cb).
NKM_HD inline uint64_t mhash_cidx(const DMScan& ms, uint32_t q, uint32_t c) {
    if (ms.n_blk <= 1) return (uint64_t)q * ms.n_chunks + c;
    uint32_t r = 0;
    while (r + 1 < ms.n_blk && c >= ms.cb[r + 1]) r++;
    const uint32_t b0 = ms.cb[r], len = ms.cb[r + 1] - b0;
    return (uint64_t)(ms.n_sigs + 1) * b0 + (uint64_t)q * len + (c - b0);
}

// Hashed signature lookup of mscan_hash_kernel: term-only pool signatures that
// all require the same keyword fields, with pairwise distinct required values,
// so a candidate matches at most one — found by its values (dictionary ids,
// 32 bits) in a two-choice cuckoo table: every signature sits at one of its
// two hashed positions, so a candidate reads exactly two entries, independent
// of each other and of the signature count.  The host builds the table.
constexpr uint32_t kMHashSigs = 256;  // signatures of one hashed scan
constexpr uint32_t kMHashCap = 1024;  // table entries (a power of two >= 2 x signatures)
constexpr uint32_t kMHashEmpty = 0xFFFFu;
// launch_mscan_hash phases: kMHashEval the per-chunk scan, kMHashPlace the
// bases + placement; kMHashCount (contiguous chunks) the scan writing counts
// only (no lists: placement reduced to the bases)
constexpr int kMHashEval = 1, kMHashPlace = 2, kMHashCount = 8;
constexpr uint32_t kMHashGrid = 4096;  // key-grid cells (u16 each) of the direct lookup
struct DMHashEntry {                  // 32 B
    uint32_t key[4];                  // required dictionary id per scanned field (0 past n_fields)
    uint32_t q;                       // signature, kMHashEmpty: free
    int32_t tmin, tmax;               // its count-range musts
    uint32_t pad;
};
static_assert(sizeof(DMHashEntry) == 32, "DMHashEntry is 32 bytes");
NKM_HD inline uint32_t msig_mix(uint32_t h, uint32_t k) {  // 32-bit multiplies only
    h = (h ^ k) * 0x9E3779B1u;
    return h ^ (h >> 15);
}
NKM_HD inline uint32_t msig_fin(uint32_t h) {
    h *= 0x85EBCA77u;
    return h ^ (h >> 13);
}

// One signature of a multi-signature scan.  term_only: every clause is a
// MUST keyword TERM, so the match is "field f == req[f] for every f in
// req_mask" and every hit scores `key` (precomputed on the host exactly as
// the device would sum the clause scores); otherwise the clauses at
// clause_off are evaluated.
struct DMSig {
    int64_t req[4];
    int64_t key;
    int32_t tmin, tmax;
    uint32_t clause_off;
    uint16_t n_clauses;
    uint8_t qkind;
    uint8_t term_only;
    uint8_t req_mask;
    uint8_t pad[7];
};
static_assert(sizeof(DMSig) == 64, "DMSig is 64 bytes");

// One row of a packed RevPrecision batch (rpack_kernel): every search of the
// batch is one searching ticket over a short source, so the descriptor is the
// ticket's slot (its query, Min/MaxCount and the reverse-check document are
// store columns) and its source range.
constexpr uint32_t kSrcOrder = 0x80000000u;  // src_len flag: the source is order[], else postings[]
struct DSmallRow {
    uint32_t slot;
    uint32_t src_off;
    uint32_t src_len;  // <= 64 entries, | kSrcOrder
};
static_assert(sizeof(DSmallRow) == 12, "DSmallRow is 12 bytes");

// rpack_kernel's output for n rows of stride S (8, 16, 32 or 64 entries), one
// buffer with 256-B aligned sections: per row its S entries' source positions
// (u8: entry k is source entry pos[k], the host maps it to the slot through
// its mirror of the posting / order list — a quarter of the D2H of slot ids), min(S, 32)
// pair-matrix words of S bits (u8 / u16 / u32), S reverse-check bits in
// entry order (u8 / u16 / u32 / u64) and the entry count (u8); then per
// workgroup its live candidates and its entries (2 x u32: the roofline's bytes).
constexpr int kPackRowsPerBlock(int S) { return 4 * (64 / S); }
struct PackLayout {
    uint64_t pos, pm, rev, cnt, live, total;
    uint32_t blocks;
    int S, pm_w, rev_w;
    // the store's query fields when at most 2 (Core::run_packed; npf = 0
    // otherwise): the square wave loads entry j's values of these columns in
    // the round that loads the row's query, so the clauses that name them need
    // no column round after their own
    uint32_t npf;
    uint16_t pf[2];
    const int64_t* pf_val[2];
    const uint8_t* pf_kind[2];
};
NKM_HD inline PackLayout pack_layout(uint64_t n, int S) {
    auto al = [](uint64_t x) { return (x + 255) & ~(uint64_t)255; };
    PackLayout L{};
    L.S = S;
    L.pm_w = S <= 8 ? 1 : S <= 16 ? 2 : 4;
    L.rev_w = S / 8;
    L.blocks = (uint32_t)((n + kPackRowsPerBlock(S) - 1) / kPackRowsPerBlock(S));
    L.pos = 0;
    L.pm = al(L.pos + n * S);
    L.rev = al(L.pm + n * (S < 32 ? S : 32) * L.pm_w);
    L.cnt = al(L.rev + n * L.rev_w);
    L.live = al(L.cnt + n);
    L.total = al(L.live + (uint64_t)L.blocks * 8);
    return L;
}

// ---- range sources (rsrc_* kernels; range_walk.h) ----------------------------
// A pool of a range batch: the posting range of its term (postings[src_off,
// + src_len), source order) and the numeric field its searches' ranges read.
// Its candidates are sorted by (value, source position) into the elements
// [out_off, out_off + pad_len) of the key / position buffers (pad_len: src_len
// rounded up to 256); a candidate that is not alive or holds no number in
// `field`, and the padding, sort after every valid one (key INT64_MAX,
// position | kRsrcInvalid), so the valid candidates are a prefix.
constexpr uint32_t kRsrcTile = 1024;           // elements sorted in LDS by one workgroup (one per lane)
constexpr uint32_t kRsrcInvalid = 0x80000000u;
struct DRangePool {
    uint32_t src_off, src_len;
    uint32_t out_off, pad_len;
    uint32_t field;
    uint32_t pad;
};
static_assert(sizeof(DRangePool) == 24, "DRangePool is 24 bytes");
// One tile of rsrc_tile_kernel: elements [start, start + len) of a pool.
struct DRangeTile {
    uint32_t pool, start, len, pad;
};
// A bound query of rsrc_bounds_kernel: the first sorted element of `pool`
// whose key is >= key (upper = 0) or > key (upper = 1).
struct DRangeBound {
    int64_t key;
    uint32_t pool, upper;
};
static_assert(sizeof(DRangeBound) == 16, "DRangeBound is 16 bytes");

// Placement of one scan chunk (scan_kernel / mscan_kernel -> stitch_kernel).
struct DChunkMap {
    uint32_t first;    // result index of the search's first chunk
    uint32_t start;    // chunk's first source position within the search
    uint32_t cap;      // the search's output capacity (k)
    uint32_t u32;      // 1: the cell and the output hold 4-B slot ids (mscan), `so` / dst_off in slot words
    uint64_t dst_off;  // the search's first output entry
    uint64_t so;       // the chunk's compacted hits in the scratch buffer
};

// One emitted hit.
struct DHit {
    uint32_t slot;
    uint32_t idx;   // position in the group's source (tie-break / cursor)
    int64_t key;    // sortable score key (tie-break / cursor); bit 0 of flags below
};

// ---- processCustom's combineIndexes on the device (enum_kernel) -------------
// combineIndexes (matchmaker_process.go:578-612) walks the bitmasks of a row's
// L filtered hits in ascending order; every mask with more than
// Max - Count bits is rejected by its first test (each hit holds >= 1 entry),
// so the masks that reach the remaining tests are exactly those with at most
// c = min(Max - Count, L) bits, in ascending order.  Rank r of that sequence
// (mask 0 = rank 0) is found by unrank_mask; a work item takes kEnumSpan
// consecutive ranks of one row.

// One searching row (T) of the pass.
struct DEnumRow {
    uint32_t hit_off;  // its first DEnumHit
    uint32_t T;        // its slot
    int32_t L;         // filtered hits (1..62)
    int32_t tcount;    // T's entries
    int32_t cmin, cmax;  // entries the hits may add: [Min - Count, Max - Count]
    int32_t tmin, tmax, tcm;
    int32_t pad;
};
static_assert(sizeof(DEnumRow) == 40, "DEnumRow is 40 bytes");

// One filtered hit of a row, with what the member checks read (:487-498).
struct DEnumHit {
    uint64_t pm;   // bit b: validateMatch holds both ways with hit b (all ones without RevPrecision)
    uint32_t slot;
    int32_t count, minc, maxc, cm;
    uint8_t wait;     // Intervals <= MaxIntervals (the member waits for a fuller group)
    uint8_t self_ok;  // a hit with >= 2 sessions meets itself in parsedQueries (:509-546): its own query must match it
    uint8_t pad[2];
};
static_assert(sizeof(DEnumHit) == 32, "DEnumHit is 32 bytes");

struct DEnumItem {
    uint64_t rank;  // first rank (>= 1: the empty mask is never a candidate)
    uint32_t row;
    uint32_t n;     // ranks [rank, rank + n), n <= kEnumSpan
};

constexpr uint32_t kEnumSpan = 256;  // masks per work item

// Number of L-bit masks with at most c bits set: sum_{k <= min(c, L)} C(L, k)
// (L <= 62: every partial product fits 64 bits).
NKM_HD inline uint64_t masks_le(int L, int c) {
    uint64_t s = 0, b = 1;
    for (int k = 0; k <= c && k <= L; k++) {
        s += b;
        b = b * (uint64_t)(L - k) / (uint64_t)(k + 1);
    }
    return s;
}

// The mask of rank r among the L-bit masks with at most c bits, ascending.
NKM_HD inline uint64_t unrank_mask(uint64_t r, int L, int c) {
    uint64_t m = 0;
    for (int p = L - 1; p >= 0 && r > 0; p--) {
        const uint64_t below = masks_le(p, c);  // those with bit p clear (the bits above fixed)
        if (r >= below) {
            m |= 1ull << p;
            r -= below;
            c--;
        }
    }
    return m;
}

}  // namespace nkm
