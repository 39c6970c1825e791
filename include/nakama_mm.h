/*
 * nakama_mm.h — C ABI of the MI355X-native matchmaker interval pass.
 *
 * This is the drop-in boundary behind Nakama's `server.Matchmaker` interface
 * (reference: server/matchmaker.go:169-183).  A Go cgo shim
 * implements `server.Matchmaker` by forwarding each interface method to the
 * entry point named beside it below.  Presences, properties and query strings
 * cross the boundary as plain C strings / doubles; the library owns the ticket
 * store (device-resident SoA), the query compiler and the interval pass.
 * Delivery (JWT signing, MatchmakerMatched hook, router fan-out,
 * server/matchmaker.go:374-440) stays on the Go side: mm_process returns the
 * matched groups and the shim delivers them.
 *
 * Conventions
 *  - Every function returning int returns MM_OK (0) or a negative MM_ERR_*
 *    status; the Go shim maps these to the nakama-common sentinels
 *    (runtime/runtime.go:180-186) listed next to each code.
 *  - Inputs are caller-owned and are copied before the call returns; the
 *    library never retains a caller pointer (cgo pointer rules).
 *  - Outputs (mm_matched, mm_extract_list) are library-owned and released
 *    with the matching mm_free_* call.
 *  - A handle is internally synchronised: mutators and mm_process may be
 *    called from different threads (server/matchmaker.go:186 mutex).  Like
 *    LocalMatchmaker.Process, mm_process holds the handle's lock only to take
 *    its snapshot and to finish (matchmaker.go:290-343): a mutator called while
 *    a pass runs returns its status at once (validated against the store plus
 *    the mutations already queued) and is applied when the pass ends, before
 *    the completeness re-check, so a group that lost a ticket is dropped.
 *    mm_extract and mm_debug_hits wait for a running pass to end.
 *
 * The CPU oracle under oracle/ exports the same symbols from its own shared
 * object so that one test harness can drive both (tests only).
 */
#ifndef NAKAMA_MM_H
#define NAKAMA_MM_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MM_ABI_VERSION 4

/* Status codes. */
#define MM_OK 0
#define MM_ERR_QUERY_INVALID     (-1) /* runtime.ErrMatchmakerQueryInvalid  (matchmaker.go:451,455) */
#define MM_ERR_DUPLICATE_SESSION (-2) /* runtime.ErrMatchmakerDuplicateSession (matchmaker.go:473) */
#define MM_ERR_INDEX             (-3) /* runtime.ErrMatchmakerIndex (matchmaker.go:527,533,655) */
#define MM_ERR_DELETE            (-4) /* runtime.ErrMatchmakerDelete (matchmaker.go:762,...) */
#define MM_ERR_NOT_AVAILABLE     (-5) /* runtime.ErrMatchmakerNotAvailable (matchmaker.go:446) */
#define MM_ERR_TOO_MANY_TICKETS  (-6) /* runtime.ErrMatchmakerTooManyTickets (matchmaker.go:512,518) */
#define MM_ERR_TICKET_NOT_FOUND  (-7) /* runtime.ErrMatchmakerTicketNotFound (matchmaker.go:732,836) */
#define MM_ERR_UNSUPPORTED       (-8) /* a ticket the call cannot take: mm_create_multi MM_MULTI_POOLS, a query that does not
                                         pin every pool field to the ticket's own value; (reserved for a query feature not
                                         lowered: none remain).  The shim maps it to QueryInvalid */
#define MM_ERR_DEVICE            (-9) /* HIP runtime failure / no usable gfx950 device */
#define MM_ERR_ARG               (-10)/* malformed call (null handle, bad sizes) */
#define MM_ERR_STATE             (-11)/* e.g. mm_process_commit without an open custom pass */

/* MatchmakerConfig (server/config.go:971-989). */
typedef struct mm_config {
    int32_t max_tickets;     /* max_tickets, default 3 */
    int32_t interval_sec;    /* interval_sec (informational: the caller drives Process) */
    int32_t max_intervals;   /* max_intervals, default 2 */
    int32_t rev_precision;   /* rev_precision (bool) */
    int32_t rev_threshold;   /* rev_threshold: reverse checks stop interval_sec * rev_threshold s into a pass
                                (matchmaker_process.go:31-46); bench.py pins it to 0 */
    int32_t override_enabled;/* a MatchmakerOverride is registered -> processCustom path (matchmaker.go:314) */
    int32_t device;          /* HIP device ordinal of this handle (mm_create_multi, include/nakama_cluster.h,
                                drives several devices from one handle) */
    const char* node;        /* this node's name (config.GetName(), matchmaker.go:225) */
} mm_config;

/* MatchmakerPresence (server/matchmaker.go:32-38). */
typedef struct mm_presence {
    const char* user_id;
    const char* session_id;
    const char* username;
    const char* node;
} mm_presence;

typedef struct mm_str_prop { const char* key; const char* value; } mm_str_prop;
typedef struct mm_num_prop { const char* key; double value; } mm_num_prop;

/* One ticket as passed to Add (intervals/node ignored) or Insert
 * (MatchmakerExtract, server/matchmaker.go:110-125). */
typedef struct mm_ticket {
    const char* ticket;
    const char* session_id;
    const char* party_id;
    const char* query;
    int32_t min_count;
    int32_t max_count;
    int32_t count_multiple;
    int32_t intervals;
    int64_t created_at;       /* UnixNano */
    const char* node;
    const mm_presence* presences;
    int32_t n_presences;
    const mm_str_prop* str_props;
    int32_t n_str_props;
    const mm_num_prop* num_props;
    int32_t n_num_props;
} mm_ticket;

/* A matched (or candidate) group: entries reference (ticket, presence index)
 * of tickets known to the handle (MatchmakerEntry, matchmaker.go:65-73). */
typedef struct mm_entry_ref {
    const char* ticket;
    int32_t presence_index;
    int32_t reserved;
} mm_entry_ref;

typedef struct mm_matched {
    int32_t n_groups;
    int32_t n_entries;
    const int32_t* group_offsets;   /* n_groups + 1 */
    const mm_entry_ref* entries;    /* n_entries */
    int32_t is_candidates;          /* 1: processCustom candidates awaiting mm_process_commit */
    int32_t n_expired;              /* tickets dropped from the active set this pass */
    double pass_ms;                 /* wall time of the pass inside the library */
    double eval_ms;                 /* device query-eval time (HIP events), 0 for the oracle */
    int64_t pair_evals;             /* (row, candidate) predicate evaluations issued */
    int64_t reserved2;              /* library-private */
    int64_t eval_bytes;             /* algorithmic bytes of the search launches (DESIGN.md roofline) */
    int32_t eval_launches;          /* search kernel launches in the pass */
    int32_t n_batches;              /* replay batches */
    int32_t eval_kernel;            /* query-eval kernel with the most bytes: 0 search, 1 scan, 2 mscan, 3 rsmall, 4 hashed mscan, 5 rpack, 6 range merge, 7 range tile */
    int32_t full_lists;             /* variable-score searches run as full lists (host-sorted), 0 for the oracle */
    const int64_t* group_created;   /* n_groups: CreatedAt of each group's last entry (its searching ticket) — the
                                       key a pool-sharded cluster merges rank results by (ABI 3) */
    int64_t pairs_decided;          /* (row, candidate) pairs the pass decided: over the rows that searched, the
                                       candidates their search's source holds (the posting list of the
                                       query's most selective MUST term, which bluge's conjunction walks:
                                       C3's region list of 250k, not the 125k mode x region pool) — what
                                       the reference's per-row bluge search evaluates (ABI 4) */
} mm_matched;

typedef struct mm_extract_list {
    int32_t n;
    const mm_ticket* tickets;
} mm_extract_list;

/* A library-owned list of strings (ticket ids), freed with mm_free_str_list. */
typedef struct mm_str_list {
    int32_t n;
    const char* const* items;
} mm_str_list;

/* ---- lifecycle (NewLocalMatchmaker / Pause / Resume / Stop) ---- */
void* mm_create(const mm_config* cfg);                 /* matchmaker.go:214 */
void  mm_destroy(void* h);
void  mm_pause(void* h);                               /* matchmaker.go:265 */
void  mm_resume(void* h);                              /* matchmaker.go:269 */
void  mm_stop(void* h);                                /* matchmaker.go:273 */
const char* mm_last_error(void* h);
int   mm_abi_version(void);
const char* mm_backend_name(void);                     /* "hip-gfx950" or "cpu-oracle" */

/* ---- mutators ---- */
int mm_add(void* h, const mm_ticket* t);               /* Add, matchmaker.go:443 (ticket/created_at supplied by caller) */
int mm_insert(void* h, const mm_ticket* ts, int32_t n);/* Insert, matchmaker.go:567 */
int mm_extract(void* h, mm_extract_list* out);         /* Extract, matchmaker.go:684 */
void mm_free_extract(void* h, mm_extract_list* out);
int mm_remove_session(void* h, const char* session_id, const char* ticket); /* :725 */
int mm_remove_session_all(void* h, const char* session_id);                 /* :769 */
int mm_remove_party(void* h, const char* party_id, const char* ticket);     /* :830 */
int mm_remove_party_all(void* h, const char* party_id);                     /* :872 */
int mm_remove_all(void* h, const char* node);                               /* :919 */
int mm_remove(void* h, const char* const* tickets, int32_t n);              /* :972 */

/* ---- the interval pass ---- */
/* Process (matchmaker.go:282).  Default path: out holds the matched groups
 * (already removed from the pool).  Override path (cfg.override_enabled):
 * out holds the processCustom candidate list (is_candidates=1) and the pass
 * stays open until mm_process_commit hands back the override's choice. */
int  mm_process(void* h, mm_matched* out);
int  mm_process_commit(void* h, const int32_t* group_offsets, const mm_entry_ref* entries,
                       int32_t n_groups, mm_matched* out);
void mm_free_matched(void* h, mm_matched* out);

/* Tickets that left the matchmaker by an explicit removal (Remove*) since the
 * previous call; the first call starts the recording.  A re-inserted ticket id
 * that replaces its old record is not reported (the id stays in the
 * matchmaker).  Tickets matched by a pass are not repeated here: they are the
 * pass's result (mm_matched), delivered and dropped from there.  The Go shim
 * drops its delivery entries with them (ABI 4: before, matched tickets were
 * logged too, a million strings per 1M-ticket pass).  The multi-device handle
 * (mm_create_multi) reports only ids no sub-handle holds at the drain: an id
 * removed and then added again before the drain is live and not reported
 * there, while a single handle reports its removal. */
int  mm_drain_removed(void* h, mm_str_list* out);
void mm_free_str_list(void* h, mm_str_list* out);

/* ---- pipelined delivery (matchmaker.go:374-440) ----
 * The reference delivers a pass's matched groups — a token or the
 * OnMatchedEntries hook per group, and the router fan-out — from Process
 * itself, so the next interval waits for it.  Here delivery runs behind the
 * pass: mm_process_deliver runs the pass (as mm_process) and hands its result
 * to a library-owned delivery thread, which calls fn(ctx, matched, pass_seq)
 * once per pass in pass order (pass_seq counts from 0 per mm_set_delivery)
 * while the caller's next pass may already run, then frees the result.  Up to
 * `depth` (>= 1) results wait for the callback; a further mm_process_deliver
 * blocks until one is delivered (a buffered Go channel's back-pressure).
 * `summary` receives the pass's counts and statistics with the group arrays
 * NULL — except on the override path, where the processCustom candidates
 * (is_candidates = 1) are returned in full exactly as by mm_process, and the
 * chosen groups are queued by mm_process_commit_deliver instead.  fn runs on
 * the delivery thread; it may call the handle's mutators and queries, not
 * mm_process*, mm_set_delivery, mm_delivery_flush or mm_destroy (from the
 * callback mm_set_delivery and mm_delivery_flush return MM_ERR_STATE and
 * mm_destroy does nothing: each would wait for the thread it runs on).  Entry
 * points of this section return MM_ERR_STATE when no delivery is set. */
typedef void (*mm_deliver_fn)(void* ctx, const mm_matched* matched, int64_t pass_seq);
/* fn NULL: deliver what is queued, then stop the thread.  Replaces an earlier
 * setting after delivering its queue. */
int  mm_set_delivery(void* h, mm_deliver_fn fn, void* ctx, int32_t depth);
int  mm_process_deliver(void* h, mm_matched* summary);
int  mm_process_commit_deliver(void* h, const int32_t* group_offsets, const mm_entry_ref* entries,
                               int32_t n_groups, mm_matched* summary);
/* Returns when every result queued so far has been delivered and freed. */
int  mm_delivery_flush(void* h);

/* ---- introspection used by tests and the bench ---- */
/* Test hook: fn(ctx) is called once per pass, on the pass's thread, after the
 * device searches and the replay and before the post-pass finish, with the
 * handle unlocked (mutators called from it are queued as concurrent ones). */
void mm_debug_set_pass_hook(void* h, void (*fn)(void*), void* ctx);
int32_t mm_ticket_count(void* h);
int32_t mm_active_count(void* h);
/* sessionTickets / partyTickets sizes (matchmaker.go:201-204): the tickets
 * one session (a presence's session id) or one party holds, counting the
 * mutations queued during a running pass (the state Add checks MaxTickets
 * against, matchmaker.go:505-520).  The multi-device handle sums them over
 * its sub-handles for a session whose tickets sit in different pools (ABI 4). */
int32_t mm_session_ticket_count(void* h, const char* session_id);
int32_t mm_party_ticket_count(void* h, const char* party_id);
/* found[i] = 1 when tickets[i] is in m.indexes (queued mutations included);
 * returns how many were found.  The multi-device handle finds a ticket's
 * sub-handle with it instead of keeping a per-ticket map (ABI 4). */
int32_t mm_find_tickets(void* h, const char* const* tickets, int32_t n, uint8_t* found);
/* Hit list of one active ticket as processDefault's search would return it
 * right now (sorted, self removed): up to cap ticket strings written as
 * pointers valid until the next call on h; returns the total hit count. */
int32_t mm_debug_hits(void* h, const char* ticket, const char** tickets_out, double* scores_out, int32_t cap);
/* Query-string compile status only (no device work): MM_OK,
 * MM_ERR_QUERY_INVALID or MM_ERR_UNSUPPORTED. */
int mm_debug_compile(const char* query);
/* Term matching of one multi-term clause, as bluge's dictionary enumeration
 * decides it (no device work): kind 1 = RegexpQuery pattern (after the leading
 * '^' trim, bluge/query.go:1264), 3 = WildcardQuery text (query.go:1475-1485),
 * 2 = FuzzyQuery term with `fuzziness` (search_fuzzy.go:43-143).  Returns 1 and
 * the per-term boost in *boost when `term` is accepted, 0 when not, -1 when
 * every search with the pattern fails (Go/vellum parse error, fuzziness outside
 * [0, 2]), -2 for a construct not lowered (MM_ERR_UNSUPPORTED at Add). */
int mm_debug_term_match(int32_t kind, const char* pattern, int32_t fuzziness, const char* term, double* boost);
/* groupIndexes (matchmaker.go:132-167) over n synthetic indexes (count,
 * created_at); writes up to cap groups as member positions (into the input
 * arrays, in the reference's append order) and avgCreatedAt; returns the
 * number of groups.  group_members must hold 8*cap entries. */
int32_t mm_debug_group_indexes(const int32_t* counts, const int64_t* created_at, int32_t n, int32_t required,
                               int32_t* group_offsets, int32_t* group_members, int64_t* avg_created_at, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* NAKAMA_MM_H */
