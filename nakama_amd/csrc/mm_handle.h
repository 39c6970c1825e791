// nakama_amd/csrc/mm_handle.h — what an mm_* handle is.
//
// Every entry point of include/nakama_mm.h takes a `void* h` that is a
// `Handle`: either one device's matchmaker (`Core`, mm_core.h) or the
// in-process multi-GPU front (`MultiCore`, mm_multi.cpp) that keeps the
// single-instance server.Matchmaker contract (server/matchmaker.go:169-183)
// over one Core per device.  The Go shim sees one type either way.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/nakama_cluster.h"
#include "../../include/nakama_mm.h"

namespace nkm {

struct Handle {
    virtual ~Handle() = default;
    virtual int add(const mm_ticket& t) = 0;
    virtual int insert(const mm_ticket* ts, int32_t n) = 0;
    virtual int extract(mm_extract_list* out) = 0;
    virtual void free_extract(mm_extract_list* out) = 0;
    virtual int remove_session(const std::string& sid, const std::string& ticket) = 0;
    virtual int remove_session_all(const std::string& sid) = 0;
    virtual int remove_party(const std::string& pid, const std::string& ticket) = 0;
    virtual int remove_party_all(const std::string& pid) = 0;
    virtual int remove_all(const std::string& node) = 0;
    virtual int remove(const char* const* tickets, int32_t n) = 0;
    virtual int process(mm_matched* out) = 0;
    virtual int process_commit(const int32_t* offs, const mm_entry_ref* ents, int32_t n_groups, mm_matched* out) = 0;
    virtual void free_matched(mm_matched* out) = 0;
    virtual int32_t ticket_count() = 0;
    virtual int32_t active_count() = 0;
    virtual int32_t debug_hits(const std::string& ticket, const char** tk, double* sc, int32_t cap) = 0;
    virtual int32_t session_ticket_count(const std::string& sid) = 0;
    virtual int32_t party_ticket_count(const std::string& pid) = 0;
    virtual int32_t find_tickets(const char* const* ids, int32_t n, uint8_t* found) = 0;
    virtual void pause() = 0;
    virtual void resume() = 0;
    virtual void stop() = 0;
    virtual const char* last_error() const = 0;
    virtual void set_error(const std::string& e) = 0;
    virtual void set_pass_hook(void (*fn)(void*), void* ctx) = 0;
    virtual int drain_removed(mm_str_list* out) = 0;
    virtual void free_str_list(mm_str_list* out) = 0;
    // row-sharded exchange of one device's handle (include/nakama_cluster.h)
    virtual int set_row_shard(int world, int rank, mm_allgather_fn fn, void* ctx) = 0;
    virtual int set_row_shard_rccl(int world, int rank, const uint8_t* uid, int len) = 0;
};

// Pool key of one ticket over the pool fields (mm_route_keys, mm_cluster.cpp):
// nonzero when the ticket's query requires, on every pool field, exactly the
// keyword value the ticket itself carries; 0 otherwise.
// What mm_last_error(NULL) reports after a failed mm_create / mm_create_multi.
void set_create_error(const std::string& e);

struct CompiledQuery;
uint64_t route_key(const mm_ticket& t, const std::vector<std::string>& fields);
uint64_t route_key(const mm_ticket& t, const std::vector<std::string>& fields, const CompiledQuery& cq);

// The NUMA node of a GPU (sysfs numa_node of its PCI device), -1 unknown;
// the usable CPUs of node `prefer` (else of the calling thread's node; none on
// a one-node host).  mm_store.cpp.
int device_numa_node(int device);
std::vector<int> node_cpus(int prefer);

}  // namespace nkm
