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

/* ---- Row-sharded mode --------------------------------------------------
 * For queries that cross pools (or a pool larger than one GPU) the pool
 * split above does not hold.  Then every rank keeps the whole ticket set (the
 * caller replicates Insert/Remove*) and runs the same pass, but each batch's
 * searches are cut into `world` contiguous blocks balanced by source length:
 * rank r evaluates block r only, and the blocks' results — per-search result
 * records, hit lists (16 B per hit), RevPrecision flags and pair matrices —
 * are exchanged in place, after which every rank replays the same lists into
 * the same groups (processDefault's single ordered replay, replicated).  The
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

#ifdef __cplusplus
}
#endif
#endif /* NAKAMA_CLUSTER_H */
