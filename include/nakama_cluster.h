/*
 * nakama_cluster.h — the host side of the pool-sharded multi-GPU front
 * (nakama_amd/cluster.py), exported by libnakama_mm.so next to the
 * single-handle ABI of nakama_mm.h.
 *
 * The reference runs one LocalMatchmaker per node: every Add/Insert/Remove*
 * goes to that instance and one Process() pass covers every ticket
 * (server/matchmaker.go:169-183, constructed once at main.go:160).  On an
 * 8-GPU node the front keeps that contract over one process per GPU: a
 * ticket is routed to the rank that owns its *pool* — the keyword values its
 * query requires on the configured pool fields, which must also be the
 * ticket's own property values — so every search and every document of a
 * pool lives on one rank and each rank's pass equals the reference's pass
 * restricted to its pools (processDefault's greedy walk never crosses a
 * pool).  These entry points compute the routing keys and move tickets
 * between ranks; the collectives run in cluster.py over torch.distributed
 * (RCCL over xGMI on the GPU path, gloo in the CPU tests).
 *
 * All functions are host-only (no device work) and thread-safe.
 */
#ifndef NAKAMA_CLUSTER_H
#define NAKAMA_CLUSTER_H

#include "nakama_mm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Pool key of each ticket over the pool fields (query field names, e.g.
 * "properties.region"): a nonzero 64-bit hash of the values its query requires
 * (MUST keyword terms, one value per field) when they equal the ticket's own
 * keyword property values (blugeProcessProperty, match_common.go:148-212);
 * 0 when the ticket is not partitionable that way (a field the query does not
 * pin, a property that differs, is numeric or parses as a datetime, or a query
 * that does not compile).  Returns the number of partitionable tickets. */
int32_t mm_route_keys(const mm_ticket* ts, int32_t n, const char* const* pool_fields, int32_t n_fields,
                      uint64_t* keys_out);

/* Packs tickets ts[idx[0..n)] into buf (a self-contained byte string); returns
 * the bytes needed — nothing is written when cap is smaller. */
int64_t mm_pack_tickets(const mm_ticket* ts, const int32_t* idx, int32_t n, uint8_t* buf, int64_t cap);

/* Unpacks a buffer of mm_pack_tickets records (several packs may be
 * concatenated); the returned set owns the tickets until mm_free_unpacked.
 * NULL on a malformed buffer. */
void* mm_unpack_tickets(const uint8_t* buf, int64_t len, int32_t* n_out, const mm_ticket** tickets_out);
void mm_free_unpacked(void* set);

/* The reference's group order over the ranks' results: processDefault
 * appends a group when its searching ticket (the group's last entry) is
 * processed, in the pinned (CreatedAt, Ticket) order, so the global list is
 * the merge of the ranks' lists by their mm_matched.group_created keys.
 * keys = every rank's key array concatenated (each ascending), counts[r] =
 * rank r's group count; writes the global position of each of `rank`'s
 * groups (linear in the keys).  Returns 1 when one of them has the same key
 * as a group of another rank (the caller orders those by ticket id), else 0. */
int32_t mm_merge_positions(const int64_t* keys, const int32_t* counts, int32_t world, int32_t rank, int64_t* pos_out);
/* The same over an all-gathered [world][stride] key matrix (rank r's keys at
 * keys + r * stride, padding ignored), with no ascending precondition: when
 * some rank's keys do not ascend (an override's choice may reorder its
 * groups) the positions are the stable order by (key, rank, index) and the
 * return value is 2 — every rank sees the same matrix, so every rank takes
 * the same branch. */
int32_t mm_merge_positions_strided(const int64_t* keys, int64_t stride, const int32_t* counts, int32_t world,
                                   int32_t rank, int64_t* pos_out);
/* mm_merge_positions_strided when the caller already knows whether every
 * rank's keys ascend (sorted != 0: each rank checked its own before the
 * all-gather, and the flags came with the group counts), so no rank re-reads
 * the whole matrix to find out; sorted == 0 is mm_merge_positions_strided.
 * The positions are computed on the library's persistent host threads. */
int32_t mm_merge_positions_ex(const int64_t* keys, int64_t stride, const int32_t* counts, int32_t world, int32_t rank,
                              int32_t sorted, int64_t* pos_out);
/* Matched tickets of a result (its entries with presence index 0: a
 * ticket's presence entries hold index 0 exactly once), counted on host
 * threads — the cluster front's per-pass summary without a Python pass over
 * the entries. */
int64_t mm_count_tickets(const mm_matched* m);

/* ---- Row-sharded mode --------------------------------------------------
 * For queries that cross pools (or a pool larger than one GPU) the pool
 * split above does not hold.  Then every rank keeps the whole ticket set (the
 * caller replicates Insert/Remove*) and runs the same pass, but each batch's
 * searches are cut into `world` contiguous blocks balanced by source length:
 * rank r evaluates block r only, and the blocks' results — per-search result
 * records, hit lists (16 B per hit), RevPrecision flags and pair matrices —
 * are exchanged in place, after which every rank replays the same lists into
 * the same groups (processDefault's single ordered replay, replicated).  A
 * batch's pool signatures on the hashed multi-signature scan (C4's 64 mode x
 * region pools) are split by candidate instead: rank r scans one block of the
 * scan order's chunks for every signature, the blocks' per-chunk hits and
 * counts are exchanged the same way, and every rank places every list.  The
 * RevThreshold timer is read at batch boundaries and OR-ed over the ranks, so
 * the replicas never diverge.  Only mm_process's batch searches are split;
 * a row's extra pages (a truncated list) are searched by every rank alike. */

/* Host transport: fn(ctx, buf, offsets) must fill buf[offsets[q],
 * offsets[q+1]) with rank q's segment for every q != rank (an in-place
 * all-gather-v over host memory, e.g. gloo); offsets has world + 1 entries (bytes).
 * Returns 0 on success. */
typedef int (*mm_allgather_fn)(void* ctx, void* buf, const int64_t* offsets);
int mm_shard_rows(void* h, int32_t world, int32_t rank, mm_allgather_fn fn, void* ctx);

/* Device transport: the exchange runs as RCCL broadcasts over xGMI on the
 * library's stream, between device buffers.  Rank 0 calls mm_rccl_unique_id
 * (128 bytes) and every rank passes the same id to mm_shard_rows_rccl. */
int mm_rccl_unique_id(uint8_t* out, int32_t cap);
int mm_shard_rows_rccl(void* h, int32_t world, int32_t rank, const uint8_t* uid, int32_t len);

/* ---- One handle over several GPUs, in one process ---------------------
 * The reference constructs ONE matchmaker per server process (main.go:160)
 * behind server.Matchmaker (server/matchmaker.go:169-183).  mm_create_multi
 * returns a handle that every entry point of nakama_mm.h accepts, exactly as
 * a single-device handle, and that drives one sub-handle per listed device
 * from host threads (no Python, no torch): a Go server gets a node's GPUs
 * through one cgo Matchmaker.
 *
 * MM_MULTI_POOLS — pools kept whole.  Add/Insert route each ticket by its
 *   pool key (mm_route_keys over pool_fields) to the sub-handle that owns the
 *   pool (a new pool goes to the least-loaded sub-handle, largest first within
 *   a batch); Process runs every sub-handle's pass concurrently and merges
 *   the group lists into the reference's order by the searching ticket's
 *   (CreatedAt, Ticket) — the group's last entry (matchmaker_process.go:
 *   299-301, mm_matched.group_created).  With an override registered the
 *   merged processCustom candidate list goes to the caller in the same order
 *   and mm_process_commit re-checks the chosen groups in the reference's
 *   post-pass order (matchmaker.go:326-343, swap-remove included) before
 *   handing each sub-handle its part.  MaxTickets per session / party
 *   (matchmaker.go:508-521) is checked against the tickets of all
 *   sub-handles.  A ticket whose query does not pin every pool field to its
 *   own property value is refused by Add with MM_ERR_UNSUPPORTED (Insert
 *   inserts the others and returns MM_ERR_UNSUPPORTED); such workloads use
 *   MM_MULTI_ROWS.
 * MM_MULTI_ROWS — any query.  Every sub-handle holds every ticket (mutators
 *   are replicated); each pass's batch searches are split into one block per
 *   sub-handle and exchanged before the replicated ordered replay (the
 *   row-sharded mode above): over RCCL between distinct devices
 *   (transport MM_MULTI_RCCL, ncclCommInitRank per sub-handle thread), or
 *   through host memory (MM_MULTI_HOST: sub-handles may share a device).
 *   A mutator called during a pass waits for the pass to end (the replicas
 *   must see it at the same point); Process itself never waits for one.
 *
 * api: the entry points of the library the sub-handles come from; NULL =
 * this library (HIP sub-handles, cfg->device replaced by devices[i]).  The
 * tests pass the CPU oracle's entry points (MM_MULTI_POOLS only).  Returns
 * NULL on failure (mm_last_error(NULL) says why). */
typedef struct mm_sub_api {
    void* (*create)(const mm_config*);
    void (*destroy)(void*);
    void (*pause)(void*);
    void (*resume)(void*);
    void (*stop)(void*);
    const char* (*last_error)(void*);
    int (*add)(void*, const mm_ticket*);
    int (*insert)(void*, const mm_ticket*, int32_t);
    int (*extract)(void*, mm_extract_list*);
    void (*free_extract)(void*, mm_extract_list*);
    int (*remove_session)(void*, const char*, const char*);
    int (*remove_session_all)(void*, const char*);
    int (*remove_party)(void*, const char*, const char*);
    int (*remove_party_all)(void*, const char*);
    int (*remove_all)(void*, const char*);
    int (*remove)(void*, const char* const*, int32_t);
    int (*process)(void*, mm_matched*);
    int (*process_commit)(void*, const int32_t*, const mm_entry_ref*, int32_t, mm_matched*);
    void (*free_matched)(void*, mm_matched*);
    int32_t (*ticket_count)(void*);
    int32_t (*active_count)(void*);
    int (*drain_removed)(void*, mm_str_list*);
    void (*free_str_list)(void*, mm_str_list*);
    int32_t (*debug_hits)(void*, const char*, const char**, double*, int32_t);
    void (*debug_set_pass_hook)(void*, void (*)(void*), void*);
    int32_t (*session_ticket_count)(void*, const char*);
    int32_t (*party_ticket_count)(void*, const char*);
    int32_t (*find_tickets)(void*, const char* const*, int32_t, uint8_t*);
} mm_sub_api;

#define MM_MULTI_POOLS 0
#define MM_MULTI_ROWS 1
#define MM_MULTI_AUTO 0 /* transport: RCCL when the devices are distinct, else host */
#define MM_MULTI_HOST 1
#define MM_MULTI_RCCL 2

typedef struct mm_multi_config {
    const int32_t* devices;          /* one sub-handle per entry (HIP ordinals; repeats share a device) */
    int32_t n_devices;
    int32_t mode;                    /* MM_MULTI_POOLS / MM_MULTI_ROWS */
    const char* const* pool_fields;  /* MM_MULTI_POOLS: query fields a pool is keyed on, e.g. "properties.region" */
    int32_t n_pool_fields;
    int32_t transport;               /* MM_MULTI_ROWS: MM_MULTI_AUTO / _HOST / _RCCL */
    const mm_sub_api* api;           /* NULL: this library */
} mm_multi_config;

void* mm_create_multi(const mm_config* cfg, const mm_multi_config* mc);
/* Number of sub-handles of a multi handle (0 for a single-device handle);
 * with sub >= 0, that sub-handle's ticket count. */
int32_t mm_multi_info(void* h, int32_t sub);

/* The NUMA node a device hangs off (its PCI device's numa_node), -1 when
 * unknown.  A handle places its host workers on its device's node (and a
 * multi handle each sub-handle's); a one-process-per-GPU launcher binds each
 * rank there (bench.py). */
int32_t mm_device_numa_node(int32_t device);

#ifdef __cplusplus
}
#endif
#endif /* NAKAMA_CLUSTER_H */
