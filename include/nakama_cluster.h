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

#ifdef __cplusplus
}
#endif
#endif /* NAKAMA_CLUSTER_H */
