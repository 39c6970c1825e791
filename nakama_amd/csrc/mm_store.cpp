// nakama_amd/csrc/mm_store.cpp — ticket store: Add/Insert/Remove*/Extract,
// compaction, and the HBM mirror (SoA columns, scan order, posting lists).
//
// Reference: server/matchmaker.go:443-1040 (mutators, MapMatchmakerIndex),
// server/match_common.go:78-212 (document field mapping).
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <pthread.h>
#include <sched.h>
#include <cstdio>
#include <unordered_set>

#include "gocompat.h"
#include "mm_core.h"

#include <chrono>
#include <cstdio>

namespace nkm {

template <class T>
void DevArray<T>::reserve(size_t n, bool keep) {
    if (n <= cap) return;
    size_t ncap = std::max<size_t>(n, cap ? cap + cap / 2 : 1024);
    T* np = nullptr;
    NKM_HIP(hipMalloc((void**)&np, ncap * sizeof(T)));
    if (keep && p && cap) NKM_HIP(hipMemcpy(np, p, cap * sizeof(T), hipMemcpyDeviceToDevice));
    if (p) (void)hipFree(p);
    p = np;
    cap = ncap;
}
template <class T>
void DevArray<T>::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
}
template <class T>
void PinnedArray<T>::reserve(size_t n) {
    if (n <= cap) return;
    size_t ncap = std::max<size_t>(n, cap ? cap * 2 : 1024);
    T* np = nullptr;
    NKM_HIP(hipHostMalloc((void**)&np, ncap * sizeof(T), hipHostMallocDefault));
    if (p) (void)hipHostFree(p);
    p = np;
    cap = ncap;
}
template <class T>
void PinnedArray<T>::release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
}

template struct DevArray<uint8_t>;
template struct DevArray<int32_t>;
template struct DevArray<uint32_t>;
template struct DevArray<int64_t>;
template struct DevArray<DQuery>;
template struct DevArray<DClause>;
template struct DevArray<DGroup>;
template struct DevArray<DHit>;
template struct DevArray<DChunkMap>;
template struct PinnedArray<DChunkMap>;
template struct PinnedArray<DClause>;
template struct PinnedArray<DMSig>;
template struct DevArray<DMSig>;
template struct DevArray<DGroupResult>;
template struct DevArray<int64_t*>;
template struct DevArray<uint8_t*>;
template struct PinnedArray<DGroup>;
template struct PinnedArray<DHit>;
template struct PinnedArray<uint8_t>;
template struct PinnedArray<DGroupResult>;
template struct PinnedArray<uint32_t>;
template struct DevArray<uint64_t>;
template struct DevArray<DEnumRow>;
template struct DevArray<DSmallRow>;
template struct PinnedArray<DSmallRow>;
template struct DevArray<DEnumHit>;
template struct DevArray<DEnumItem>;
template struct PinnedArray<uint64_t>;
template struct PinnedArray<DEnumRow>;
template struct PinnedArray<DEnumHit>;
template struct PinnedArray<DEnumItem>;

static const char* kBuiltinNames[F_NBUILTIN] = {"ticket", "min_count", "max_count", "party_id", "created_at"};

Core::Core(const mm_config& cfg) : cfg_(cfg) {
    node_ = cfg.node ? cfg.node : "";
    cfg_.node = nullptr;
    device_ = cfg.device;
    host_share_ = g_create_share;
    numa_node_ = device_numa_node(device_);
    sess_slots_.live = &live_;
    party_slots_.live = &live_;
    int ndev = 0;
    NKM_HIP(hipGetDeviceCount(&ndev));
    if (ndev <= 0 || device_ < 0 || device_ >= ndev) throw DeviceError{hipErrorNoDevice, "device ordinal", __LINE__};
    NKM_HIP(hipSetDevice(device_));
    NKM_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    for (auto& e : ev_) NKM_HIP(hipEventCreate(&e));
    NKM_HIP(hipEventCreateWithFlags(&apply_ev_, hipEventDisableTiming));
    if (const char* e = std::getenv("NKM_DENSE")) dense_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_PIPE")) pipe_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_GPIPE")) gpipe_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_RUNS")) runs_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_PRUNS")) pruns_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_CDIRECT")) custom_direct_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_FAST")) fast_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_FULLVAR")) full_var_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_MHASH")) mhash_mode_ = std::atoi(e);
    if (const char* e = std::getenv("NKM_MCONTIG")) mcontig_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_SLOTLISTS")) {
        slot_lists_mode_ = std::strcmp(e, "0") != 0;
        slot_lists_rev_ = std::strcmp(e, "2") == 0;
    }
    if (const char* e = std::getenv("NKM_PAGE")) page_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_PROFILE")) batch_profile_ = std::strcmp(e, "2") == 0;
    if (const char* e = std::getenv("NKM_PARTIAL")) partial_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_DEVENUM")) dev_enum_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_RPACK")) pack_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_TIER")) tier_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_RANGE")) range_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_LISTPROOF")) list_proof_mode_ = std::atoi(e);
    if (const char* e = std::getenv("NKM_MHCOUNT")) mhash_count_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_MHGRID")) mhash_grid_mode_ = std::strcmp(e, "0") != 0;
    if (const char* e = std::getenv("NKM_BULK")) bulk_mode_ = std::strcmp(e, "0") == 0 ? 0 : std::strcmp(e, "force") == 0 ? 2 : 1;
    if (const char* e = std::getenv("NKM_KERNEL"))
        kernel_mode_ = !std::strcmp(e, "search") ? KM_SEARCH : !std::strcmp(e, "scan") ? KM_SCAN
                     : !std::strcmp(e, "mscan") ? KM_MSCAN : KM_AUTO;
    if (const char* e = std::getenv("NKM_PARALLEL")) par_mode_ = !std::strcmp(e, "0") ? 0 : !std::strcmp(e, "force") ? 2 : 1;
    for (int f = 0; f < F_NBUILTIN; f++) field_dict_.intern(kBuiltinNames[f]);
    fval_.resize(F_NBUILTIN);
    fkind_.resize(F_NBUILTIN);
    field_used_.assign(F_NBUILTIN, 0);
    field_posting_.assign(F_NBUILTIN, 0);
    d_fval_.assign(F_NBUILTIN, nullptr);
    d_fkind_.assign(F_NBUILTIN, nullptr);
    dev_field_slots_.assign(F_NBUILTIN, 0);
}

void WorkPool::pin(int cpu) {
    cpu_set_t cs;
    CPU_ZERO(&cs);
    CPU_SET(cpu, &cs);
    (void)pthread_setaffinity_np(pthread_self(), sizeof cs, &cs);
}

void WorkPool::pin_set(const std::vector<int>& cpus) {
    cpu_set_t cs;
    CPU_ZERO(&cs);
    for (int c : cpus)
        if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &cs);
    (void)pthread_setaffinity_np(pthread_self(), sizeof cs, &cs);
}

namespace {
std::vector<int> parse_cpulist(const std::string& path) {  // "0-3,8,10-11"
    std::vector<int> out;
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return out;
    char buf[4096];
    const size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    const char* p = buf;
    while (*p >= '0' && *p <= '9') {
        char* e;
        const long a = std::strtol(p, &e, 10);
        long b = a;
        p = e;
        if (*p == '-') {
            b = std::strtol(p + 1, &e, 10);
            p = e;
        }
        for (long c = a; c <= b; c++) out.push_back((int)c);
        if (*p == ',') p++;
    }
    return out;
}
}  // namespace

// The NUMA node a GPU hangs off (its PCI device's numa_node in sysfs), or -1
// (unknown, or a one-node host).
int device_numa_node(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof bus - 1, device) != hipSuccess || !bus[0]) return -1;
    std::string id(bus);
    for (char& ch : id) ch = (char)std::tolower((unsigned char)ch);
    FILE* f = std::fopen(("/sys/bus/pci/devices/" + id + "/numa_node").c_str(), "r");
    if (!f) return -1;
    int nd = -1;
    if (std::fscanf(f, "%d", &nd) != 1) nd = -1;
    std::fclose(f);
    return nd;
}

// The CPUs (that the process may use) of NUMA node `prefer` — the handle's
// GPU's node — or, when that is unknown or holds none of them, of the calling
// thread's node; none when the host has one node.  Default worker placement:
// every worker may run anywhere on that node, so the OS still moves it off a
// busy core, but it never leaves the socket whose memory the store was
// first-touched on (MI355X boxes: 2 x EPYC 9575F, 2 NUMA nodes; unrestricted
// workers drifting to the other socket made every walk's store access remote:
// C2 p50 5.44 -> 3.31 ms, C3 5.42 -> 4.73 ms with node-local workers,
// profiles/r04n_pin.txt).
std::vector<int> node_cpus(int prefer) {
    std::vector<int> out;
    const int cpu = sched_getcpu();
    cpu_set_t allowed;
    if (cpu < 0 || sched_getaffinity(0, sizeof allowed, &allowed) != 0) return out;
    int nodes = 0;
    std::vector<int> mine, pref;
    for (int nd = 0; nd < 64; nd++) {
        std::vector<int> l = parse_cpulist("/sys/devices/system/node/node" + std::to_string(nd) + "/cpulist");
        if (l.empty()) continue;
        nodes++;
        if (std::find(l.begin(), l.end(), cpu) != l.end()) mine = l;
        if (nd == prefer) pref = l;
    }
    if (nodes < 2) return out;
    for (int c : pref)
        if (c < CPU_SETSIZE && CPU_ISSET(c, &allowed)) out.push_back(c);
    if (!out.empty()) return out;
    for (int c : mine)
        if (c < CPU_SETSIZE && CPU_ISSET(c, &allowed)) out.push_back(c);
    return out;
}

// Host worker count: NKM_THREADS, else the visible cores capped at 16 (the
// per-GPU host share on an 8-GPU node).  Same-box A/B runs on MI355X boxes
// (profiles/r01_ab_threads.txt) put 8 and 16 workers within the boxes'
// run-to-run noise on C3 (8 pools); 16 keeps pools > 8 (C4) parallel.
WorkPool& Core::workers() {
    if (!workers_) {
        unsigned n = std::thread::hardware_concurrency();
        cpu_set_t cs;
        CPU_ZERO(&cs);
        if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = (unsigned)CPU_COUNT(&cs);
        // one process per GPU: the node's cores are shared by the local ranks
        if (const char* lw = std::getenv("LOCAL_WORLD_SIZE")) n /= std::max(1, std::atoi(lw));
        n /= std::max(1u, host_share_);  // sub-handles of one multi handle (mm_multi.cpp) split them too
        n = std::max(1u, std::min(16u, n));
        if (const char* e = std::getenv("NKM_THREADS")) n = std::max(1, std::atoi(e));
        // node-local workers (node_cpus; per-CPU pinning measured no better
        // and cannot move off a core another job keeps busy, profiles/r04n_pin.txt)
        std::vector<int> area = node_cpus(numa_node_);
        // the node's share: its CPUs over the handles placed on it (a multi
        // handle's sub-handles on that node, or the local ranks)
        if (!area.empty() && !std::getenv("NKM_THREADS") && !std::getenv("LOCAL_WORLD_SIZE"))
            n = std::max(1u, std::min(16u, (unsigned)area.size() / std::max(1u, host_share_)));
        workers_.reset(new WorkPool(n, {}, area));
    }
    return *workers_;
}

Core::~Core() {
    workers_.reset();
    shard_release();
    (void)hipSetDevice(device_);
    for (auto* p : d_fval_) delete p;
    for (auto* p : d_fkind_) delete p;
    for (auto& e : ev_)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : rs_ev_)
        if (e) (void)hipEventDestroy(e);
    if (apply_ev_) (void)hipEventDestroy(apply_ev_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

uint16_t Core::field_of(const std::string& name) {
    int64_t f = field_dict_.find(name);
    if (f >= 0) return (uint16_t)f;
    if (field_dict_.size() >= 65535) throw DeviceError{hipErrorOutOfMemory, "too many fields", __LINE__};
    uint16_t id = (uint16_t)field_dict_.intern(name);
    fval_.emplace_back();
    fkind_.emplace_back();
    field_used_.push_back(0);
    field_posting_.push_back(0);
    d_fval_.push_back(nullptr);
    d_fkind_.push_back(nullptr);
    dev_field_slots_.push_back(0);
    return id;
}

int64_t Core::slot_of_ticket(std::string_view t) const {
    const int64_t s = slot_of_.find(str_hash(t), [&](uint32_t v) { return tk(v) == t; });
    if (s < 0 || !live_[s]) return -1;
    return s;
}

// Value of field f in a ticket's document properties (doc_props).
static void field_value(uint16_t f, const Core::Props& props, uint8_t* kind, int64_t* val) {
    *kind = KIND_ABSENT;
    *val = 0;
    for (auto& p : props)
        if (p.first == f) { *kind = p.second.first; *val = p.second.second; }
}

// Field of a property name ("properties." + name, interned on first sight).
uint16_t Core::prop_field(std::string_view key) {
    const int64_t i = prop_key_.find(key);
    if (i >= 0) return prop_field_[i];
    std::string name = "properties.";
    name.append(key);
    const uint16_t f = field_of(name);
    prop_key_.intern(key);
    prop_field_.push_back(f);
    return f;
}

// Builds the property part of the bluge document of a ticket
// (blugeProcessProperty, match_common.go:148-212): string props become keyword
// terms unless they parse as a datetime (then the raw UnixNano numeric term);
// numeric props the sortable int64 of the float64; numeric wins on key clash
// (matchmaker.go:460-466).  Fields in first-seen order, the last value wins.
void Core::doc_props(const ColdView& v, Props& out) {
    out.clear();
    auto put = [&](uint16_t f, uint8_t kind, int64_t val) {
        for (auto& p : out)
            if (p.first == f) {
                p.second = {kind, val};
                return;
            }
        out.push_back({f, {kind, val}});
    };
    v.each_prop(
        [&](std::string_view k, std::string_view val) {
            int64_t ns;
            if (bluge_datetime(val, &ns)) put(prop_field(k), KIND_NUMERIC, ns);
            else put(prop_field(k), KIND_KEYWORD, (int64_t)dict_.intern(val));
        },
        [&](std::string_view k, double d) { put(prop_field(k), KIND_NUMERIC, sortable_i64(d)); });
}

void Core::set_field(uint16_t f, uint32_t slot, uint8_t kind, int64_t val) {
    fkind_[f][slot] = kind;
    fval_[f][slot] = val;
}

// Interns a regexp/wildcard/fuzzy matcher (kind, pattern, fuzziness, boost).
uint32_t Core::termset_of(const HostClause& c) {
    std::string key;
    key.push_back((char)c.mt_kind);
    key.push_back((char)c.fuzziness);
    key.append((const char*)&c.score, sizeof(double));
    key += c.term;
    auto it = tset_index_.find(key);
    if (it != tset_index_.end()) return it->second;
    TermSet ts;
    ts.m.kind = (TermMatcher::Kind)c.mt_kind;
    ts.m.pattern = c.term;
    ts.m.fuzziness = c.fuzziness;
    if (ts.m.kind == TermMatcher::K_REGEXP) ts.m.re.compile(c.term);  // validated by compile_query
    ts.b = c.score;
    const uint32_t id = (uint32_t)tsets_.size();
    tsets_.push_back(std::move(ts));
    tset_index_.emplace(std::move(key), id);
    tsets_dirty_ = true;
    return id;
}

// bluge enumerates the field dictionary through the matcher's automaton at
// every search (search_regexp.go:27-56, search_fuzzy.go:79-113); the keyword
// dictionary here only grows, so each set is extended over the ids interned
// since the last pass.  Ids of strings that are not values of the clause's
// field are harmless: the kernels test the candidate's own value id.
void Core::refresh_termsets() {
    if (tsets_.empty()) return;
    const uint32_t nd = (uint32_t)dict_.size();
    for (auto& ts : tsets_) {
        for (uint32_t id = ts.done; id < nd; id++) {
            double tb;
            if (!ts.m.accept(std::string(dict_.str(id)), &tb)) continue;
            ts.ids.push_back(id);
            // RegexpQuery(b): b.  Fuzzy MatchQuery(b): (0 + b*tb) * b (composite.go:37-43)
            ts.sc.push_back(ts.m.kind == TermMatcher::K_FUZZY ? (0.0 + ts.b * tb) * ts.b : ts.b);
            tsets_dirty_ = true;
        }
        ts.done = nd;
    }
    if (!tsets_dirty_) return;
    std::vector<uint32_t> desc, ids;
    std::vector<double> sc;
    for (auto& ts : tsets_) {
        desc.push_back((uint32_t)ids.size());
        desc.push_back((uint32_t)ts.ids.size());
        ids.insert(ids.end(), ts.ids.begin(), ts.ids.end());
        sc.insert(sc.end(), ts.sc.begin(), ts.sc.end());
    }
    d_tset_desc_.reserve(desc.size(), false);
    d_tset_ids_.reserve(std::max<size_t>(ids.size(), 1), false);
    d_tset_sc_.reserve(std::max<size_t>(sc.size(), 1), false);
    NKM_HIP(hipMemcpyAsync(d_tset_desc_.p, desc.data(), desc.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream_));
    if (!ids.empty()) {
        NKM_HIP(hipMemcpyAsync(d_tset_ids_.p, ids.data(), ids.size() * sizeof(uint32_t), hipMemcpyHostToDevice, stream_));
        NKM_HIP(hipMemcpyAsync(d_tset_sc_.p, sc.data(), sc.size() * sizeof(double), hipMemcpyHostToDevice, stream_));
    }
    NKM_HIP(hipStreamSynchronize(stream_));  // the staging vectors die here
    tsets_dirty_ = false;
}

// Identity of a signature: query kind, the searching ticket's filters and the
// compiled clauses (field / term ids, bounds, boosts) — hashed here, compared
// against the stored signature (sig_eq): the index keeps no key strings.
uint64_t sig_clause_hash(const DClause* dc, size_t n) { return str_hash((const char*)dc, n * sizeof(DClause)); }
uint64_t sig_hash(uint64_t clause_hash, uint8_t kind, int32_t mn, int32_t mx, uint32_t party) {
    uint64_t h = clause_hash ^ ((uint64_t)kind << 56);
    h = (h ^ (uint32_t)mn) * 0x9E3779B97F4A7C15ull;
    h = (h ^ (uint32_t)mx) * 0xBF58476D1CE4E5B9ull;
    h = (h ^ party) * 0x94D049BB133111EBull;
    return h ^ (h >> 31);
}
bool Core::sig_eq(uint32_t id, uint8_t kind, int32_t mn, int32_t mx, uint32_t party, const DClause* dc, size_t n) const {
    const Sig& g = sigs_[id];
    return g.qkind == kind && g.tmin == mn && g.tmax == mx && g.tparty == party && g.n_clauses == n &&
           (n == 0 || std::memcmp(clauses_.data() + g.clause_off, dc, n * sizeof(DClause)) == 0);
}

// A signature's descriptor from its compiled clauses (no store state is
// touched: the bulk Insert runs it on the workers): score bound, variable
// score, MUST terms, fields.  clause_off is set when it is committed.
void Core::sig_describe(Sig& s, const std::vector<DClause>& dc, const CompiledQuery& cq, int32_t mn, int32_t mx,
                        uint32_t party) {
    s = Sig{};
    s.n_clauses = (uint16_t)dc.size();
    s.qkind = cq.kind;
    s.tmin = mn;
    s.tmax = mx;
    s.tparty = party;
    bool has_must = false, has_should = false, any_pos = false;
    int n_should_live = 0;
    double ms = 0.0, ss = 0.0, best_neg = -HUGE_VAL;
    for (auto& d : dc) {
        if (d.occur == OCC_MUST) {
            has_must = true;
            ms += d.score;
            if (d.op == OP_TERM) {
                s.must_terms.push_back({d.field, d.term});
                s.must_fmask |= 1ull << (d.field < 63 ? d.field : 63);
            }
        } else if (d.occur == OCC_SHOULD) {
            has_should = true;
            if (d.op != OP_FALSE) {
                n_should_live++;
                if (d.score > 0) { ss += d.score; any_pos = true; }
                else best_neg = std::max(best_neg, d.score);
            }
        }
    }
    if (s.must_terms.size() == 1) s.must_key1 = ((uint64_t)s.must_terms[0].first << 32) | s.must_terms[0].second;
    // a fuzzy clause scores per accepted term: variable-score search, no score bound
    bool fuzzy = false;
    for (auto& c : cq.clauses)
        if (c.op == OP_TERMSET && c.mt_kind == TermMatcher::K_FUZZY && c.occur != OCC_MUSTNOT) fuzzy = true;
    s.var_score = cq.kind == QK_BOOL && !(n_should_live == 0 || (!has_must && n_should_live == 1));
    double S;
    if (cq.kind != QK_BOOL) S = 1.0;
    else if (!has_must && !has_should) S = 1.0;
    else if (!has_must) S = any_pos ? ss : best_neg;
    else S = any_pos ? ms + ss : ms;
    double ub = (S + 1.0) + 1.0;
    s.ub_key = std::isfinite(ub) ? sortable_i64(ub) : INT64_MAX;
    if (!std::isfinite(ms) || !std::isfinite(ss)) s.ub_key = INT64_MAX;
    if (fuzzy) {
        s.var_score = true;
        s.ub_key = INT64_MAX;
    }
    std::vector<uint16_t> fs;
    for (auto& d : dc)
        if (d.op != OP_FALSE && std::find(fs.begin(), fs.end(), d.field) == fs.end()) fs.push_back(d.field);
    s.n_fields = (uint16_t)fs.size();
    s.exact_scores = dc.size() <= 64;
    for (auto& d : dc) {
        const double x = std::ldexp(d.score, 20);
        s.exact_scores = s.exact_scores && std::isfinite(d.score) && std::fabs(d.score) <= 1048576.0 && x == std::nearbyint(x);
    }
    // range source: exactly one MUST keyword term, every other clause a numeric
    // range on one other field, at least one of them MUST (so every hit holds
    // a number there), at most 32 ranges (range_walk.h: build_tiers)
    if (cq.kind == QK_BOOL && !fuzzy && dc.size() <= 33) {
        int n_term = 0, n_must_range = 0, n_range = 0, rf = -1;
        bool ok = true;
        for (auto& d : dc) {
            if (d.op == OP_TERM && d.occur == OCC_MUST) {
                n_term++;
            } else if (d.op == OP_RANGE) {
                if (rf < 0) rf = d.field;
                ok = ok && d.field == rf;
                n_range++;
                n_must_range += d.occur == OCC_MUST;
            } else {
                ok = false;
            }
        }
        if (ok && n_term == 1 && n_must_range >= 1 && n_range <= 32 && rf != (int)s.must_terms[0].first) {
            s.rs_field = (uint16_t)rf;
            s.rs_nrange = (uint8_t)n_range;
        }
    }
}

// Adds a described signature: its clauses, the fields it references (and
// posting lists of its MUST terms), the index entry.  materialize: build the
// dense host column of a field referenced for the first time now (the bulk
// Insert does it once for the batch: materialize_fields).
uint32_t Core::sig_commit(Sig&& s, const DClause* dc, size_t n, uint64_t hash, bool materialize) {
    s.clause_off = (uint32_t)clauses_.size();
    for (size_t k = 0; k < n; k++) {
        if (dc[k].op != OP_FALSE) field_used_[dc[k].field] = 1;
        clauses_.push_back(dc[k]);
    }
    for (auto& mt : s.must_terms)
        if (!field_posting_[mt.first]) { field_posting_[mt.first] = 1; index_dirty_ = true; }
    const uint32_t id = (uint32_t)sigs_.size();
    sig_fmask_.push_back(s.must_fmask);
    sig_lite_.push_back(lite_of(s));
    sigs_.push_back(std::move(s));
    sig_idx_.put_new(hash, id);
    if (materialize) materialize_fields();
    return id;
}

// Fields referenced for the first time get a dense host column over the
// existing slots.
void Core::materialize_fields() {
    const size_t n = nslots();
    for (size_t f = 0; f < field_used_.size(); f++) {
        if (field_used_[f] && fval_[f].size() != n) {
            fval_[f].assign(n, 0);
            fkind_[f].assign(n, KIND_ABSENT);
            Props props;
            for (uint32_t sl = 0; sl < n; sl++) {
                if (f < F_NBUILTIN) {
                    switch (f) {
                    case F_TICKET: set_field((uint16_t)f, sl, KIND_KEYWORD, dict_.intern(tk(sl))); break;
                    case F_MIN: set_field((uint16_t)f, sl, KIND_NUMERIC, sortable_i64((double)minc_[sl])); break;
                    case F_MAX: set_field((uint16_t)f, sl, KIND_NUMERIC, sortable_i64((double)maxc_[sl])); break;
                    case F_PARTY:
                        set_field((uint16_t)f, sl, KIND_KEYWORD, dict_.intern(cold_.view(sl).party_id));
                        break;
                    case F_CREATED: set_field((uint16_t)f, sl, KIND_NUMERIC, ckey_[sl]); break;
                    }
                } else {
                    doc_props(cold_.view(sl), props);
                    uint8_t k;
                    int64_t v;
                    field_value((uint16_t)f, props, &k, &v);
                    set_field((uint16_t)f, sl, k, v);
                }
            }
            dev_field_slots_[f] = 0;
        }
    }
}

// Assigns (or reuses) the compiled signature of a ticket's search.
uint32_t Core::sig_of(const CompiledQuery& cq, int32_t mn, int32_t mx, uint32_t party) {
    std::vector<DClause> dc;
    dc.reserve(cq.clauses.size());
    for (auto& c : cq.clauses) {
        DClause d{};
        d.op = c.op;
        d.occur = c.occur;
        d.lo = c.lo;
        d.hi = c.hi;
        d.score = c.score;
        d.field = 0;
        d.term = 0;
        if (c.op != OP_FALSE) {
            d.field = field_of(c.field);
            if (c.op == OP_TERM || c.op == OP_NUMLIT) d.term = dict_.intern(c.term);
            else if (c.op == OP_TERMSET) d.term = termset_of(c);
        }
        dc.push_back(d);
    }
    const uint64_t h = sig_hash(sig_clause_hash(dc.data(), dc.size()), cq.kind, mn, mx, party);
    const int64_t f = sig_idx_.find(h, [&](uint32_t id) { return sig_eq(id, cq.kind, mn, mx, party, dc.data(), dc.size()); });
    if (f >= 0) return (uint32_t)f;
    Sig s;
    sig_describe(s, dc, cq, mn, mx, party);
    return sig_commit(std::move(s), dc.data(), dc.size(), h, true);
}

void Core::kill_slot(uint32_t s, bool device_cleared, bool quiet) {
    if (!live_[s]) return;
    if (track_removed_ && !quiet) removed_ids_.emplace_back(tk(s));
    live_[s] = 0;
    is_active_[s] = 0;
    active_exact_ = false;
    n_live_--;
    if (!device_cleared) pending_dead_.push_back(s);
    uint32_t p0 = pres_off_[s], p1 = pres_off_[s + 1];
    // sessionTickets bookkeeping (a ticket counts once per distinct session)
    for (uint32_t p = p0; p < p1; p++) {
        bool dup = false;
        for (uint32_t q = p0; q < p; q++) dup |= pres_sess_[q] == pres_sess_[p];
        if (!dup) sess_slots_.erase(pres_sess_[p], s);
    }
    if (party_[s] != kNoParty) party_slots_.erase(party_[s], s);
}

int Core::add_locked(const mm_ticket& t, uint32_t sg, bool from_insert) {
    auto S = [](const char* p) { return p ? std::string_view(p) : std::string_view(); };
    const std::string_view tkv = S(t.ticket);
    const uint64_t th = str_hash(tkv);
    const int64_t existing = slot_of_.find(th, [&](uint32_t v) { return tk(v) == tkv; });
    if (existing >= 0 && live_[existing]) kill_slot((uint32_t)existing, false, true);  // same id re-inserted: replace
    const uint32_t s = (uint32_t)nslots();
    tk_ptr_.push_back(tk_arena_.put(tkv));
    tk_len_.push_back((uint32_t)tkv.size());
    {
        ColdStore::Writer w = cold_.begin();
        w.u32((uint32_t)std::max(t.n_presences, 0));
        w.u32((uint32_t)std::max(t.n_str_props, 0));
        w.u32((uint32_t)std::max(t.n_num_props, 0));
        w.str(t.session_id);
        w.str(t.party_id);
        w.str(t.query);
        for (int i = 0; i < t.n_presences; i++) {
            const mm_presence& p = t.presences[i];
            w.str(p.user_id);
            w.str(p.session_id);
            w.str(p.username);
            w.str(p.node);
        }
        for (int i = 0; i < t.n_str_props; i++) {
            w.str(t.str_props[i].key);
            w.str(t.str_props[i].value);
        }
        for (int i = 0; i < t.n_num_props; i++) {
            w.str(t.num_props[i].key);
            w.f64(t.num_props[i].value);
        }
    }
    tnode_.push_back(node_dict_.intern(from_insert ? S(t.node) : std::string_view(node_)));
    created_.push_back(t.created_at);
    ckey_.push_back(sortable_i64((double)t.created_at));
    minc_.push_back(t.min_count);
    maxc_.push_back(t.max_count);
    cm_.push_back(t.count_multiple);
    count_.push_back(t.n_presences);
    max_pres_ = std::max(max_pres_, t.n_presences);
    intervals_.push_back(from_insert ? t.intervals : 0);
    const std::string_view pid = S(t.party_id);
    const uint32_t party = pid.empty() ? kNoParty : party_dict_.intern(pid);
    party_.push_back(party);
    live_.push_back(1);
    indexed_.push_back(1);
    bool act = from_insert ? (t.intervals < cfg_.max_intervals) : true;
    is_active_.push_back(act ? 1 : 0);
    if (pres_off_.empty()) pres_off_.push_back(0);
    for (int i = 0; i < t.n_presences; i++) pres_sess_.push_back(sess_dict_.intern(S(t.presences[i].session_id)));
    pres_off_.push_back((uint32_t)pres_sess_.size());
    {
        uint32_t p0 = pres_off_[s], p1 = pres_off_[s + 1];
        for (uint32_t p = p0; p < p1; p++) {
            bool dup = false;
            for (uint32_t q = p0; q < p; q++) dup |= pres_sess_[q] == pres_sess_[p];
            if (!dup) sess_slots_.add(pres_sess_[p], s);
        }
    }
    if (party != kNoParty) party_slots_.add(party, s);
    hot_.emplace_back();
    set_hot(s);
    // dense columns of referenced fields
    for (size_t f = 0; f < fval_.size(); f++) {
        if (!fval_[f].empty() || field_used_[f]) {
            fval_[f].push_back(0);
            fkind_[f].push_back(KIND_ABSENT);
        }
    }
    if (field_used_[F_TICKET]) set_field(F_TICKET, s, KIND_KEYWORD, dict_.intern(tkv));
    if (field_used_[F_MIN]) set_field(F_MIN, s, KIND_NUMERIC, sortable_i64((double)t.min_count));
    if (field_used_[F_MAX]) set_field(F_MAX, s, KIND_NUMERIC, sortable_i64((double)t.max_count));
    if (field_used_[F_PARTY]) set_field(F_PARTY, s, KIND_KEYWORD, dict_.intern(pid));
    if (field_used_[F_CREATED]) set_field(F_CREATED, s, KIND_NUMERIC, ckey_[s]);
    {
        static thread_local Props props;
        doc_props(cold_.view(s), props);
        for (auto& p : props)
            if (p.first < fval_.size() && fval_[p.first].size() == nslots()) set_field(p.first, s, p.second.first, p.second.second);
    }
    // The party mustNot (matchmaker_process.go:80-85) only ever removes the
    // searching ticket's own party (<= MaxTickets tickets), so it is applied
    // while walking the hit list instead of in the shared search: party
    // tickets then share their pool's search (sig: the caller's sig_of with
    // kNoParty).
    sig_.push_back(sg);
    self_match_.push_back(self_match_of(s));
    if (s > 0) monotone_ = monotone_ && created_[s] > created_[s - 1] && ckey_[s] > ckey_[s - 1];
    squery_.push_back(DQuery{sigs_[sg].clause_off, sigs_[sg].n_clauses, sigs_[sg].qkind, 0});
    slot_of_.put(th, s, [&](uint32_t v) { return tk(v) == tkv; });
    n_live_++;
    if (act) {
        if (!active_list_.empty()) {
            uint32_t l = active_list_.back();
            if (created_[l] > t.created_at || (created_[l] == t.created_at && tk(l) > tkv)) active_sorted_ = false;
        }
        active_list_.push_back(s);
    }
    if (!order_.empty()) {
        uint32_t l = order_.back();
        if (ckey_[l] > ckey_[s]) order_sorted_ = false;
    }
    order_.push_back(s);
    index_dirty_ = true;
    return MM_OK;
}

uint8_t Core::self_match_of(uint32_t s) const {
    for (auto& mt : sigs_[sig_[s]].must_terms)
        if (fkind_[mt.first].size() <= s || fkind_[mt.first][s] != KIND_KEYWORD || (uint32_t)fval_[mt.first][s] != mt.second)
            return 0;
    return 1;
}

// sig_of through the (query text, MinCount, MaxCount) cache.  The cache is
// dropped when it reaches 64k texts (a workload of unique queries gains
// nothing from it and must not grow it without bound).
int64_t Core::sig_cached(const mm_ticket& t) {
    const std::string_view q = t.query ? std::string_view(t.query) : std::string_view();
    if (qtext_.size() >= (1u << 16)) {
        qtext_.clear();
        qstatus_.clear();
        qsig_.clear();
        qsig_idx_.clear();
    }
    int64_t qi = qtext_.find(q);
    CompiledQuery cq;
    bool compiled = false;
    if (qi < 0) {
        const int rc = compile_query(q, &cq);
        compiled = true;
        qi = qtext_.intern(q);
        qstatus_.push_back(rc);
    }
    if (qstatus_[qi] != CQ_OK) return -1 - qstatus_[qi];
    uint64_t h = (uint64_t)qi * 0x9E3779B97F4A7C15ull;
    h = (h ^ (uint32_t)t.min_count) * 0xBF58476D1CE4E5B9ull;
    h = (h ^ (uint32_t)t.max_count) * 0x94D049BB133111EBull;
    h ^= h >> 31;
    auto eq = [&](uint32_t i) { return qsig_[i].q == qi && qsig_[i].mn == t.min_count && qsig_[i].mx == t.max_count; };
    const int64_t e = qsig_idx_.find(h, eq);
    if (e >= 0) return qsig_[e].sig;
    if (!compiled) compile_query(q, &cq);
    const uint32_t sg = sig_of(cq, t.min_count, t.max_count, kNoParty);  // may materialise new columns
    qsig_idx_.put_new(h, (uint32_t)qsig_.size());
    qsig_.push_back(QSig{(uint32_t)qi, t.min_count, t.max_count, sg});
    return sg;
}

static int status_of(int cq) { return cq == CQ_UNSUPPORTED ? MM_ERR_UNSUPPORTED : MM_ERR_QUERY_INVALID; }

// Add (matchmaker.go:443-565).
int Core::add(const mm_ticket& t) {
    if (stopped_) return MM_ERR_NOT_AVAILABLE;
    CompiledQuery cq;
    int rc = compile_query(t.query ? t.query : "", &cq);
    if (rc != CQ_OK) { last_error_ = "query"; return status_of(rc); }
    {
        std::unordered_set<std::string> seen;
        for (int i = 0; i < t.n_presences; i++) {
            std::string s = t.presences[i].session_id ? t.presences[i].session_id : "";
            if (!seen.insert(s).second) return MM_ERR_DUPLICATE_SESSION;
        }
    }
    std::lock_guard<std::mutex> lk(mu_);
    // MaxTickets per session / party (matchmaker.go:505-520), against the
    // effective state while a pass runs
    for (int i = 0; i < t.n_presences; i++)
        if (eff_sess_count(t.presences[i].session_id ? t.presences[i].session_id : "") >= cfg_.max_tickets)
            return MM_ERR_TOO_MANY_TICKETS;
    std::string party = t.party_id ? t.party_id : "";
    if (!party.empty() && eff_party_count(party) >= cfg_.max_tickets) return MM_ERR_TOO_MANY_TICKETS;
    if (pass_running_) {
        PendingOp op{P_ADD};
        op.tickets.emplace_back(t);
        op.cqs.push_back(std::move(cq));
        op.ok.push_back(1);
        eff_add(op.tickets.back());
        pending_.push_back(std::move(op));
        return MM_OK;
    }
    maybe_compact();
    return add_locked(t, sig_of(cq, t.min_count, t.max_count, kNoParty), false);
}

// ---- the effective state while a pass runs (see mm_core.h) ----
Core::OwnedTicket::OwnedTicket(const mm_ticket& t) {
    auto S = [](const char* p) { return p ? std::string(p) : std::string(); };
    ticket = S(t.ticket);
    session_id = S(t.session_id);
    party_id = S(t.party_id);
    query = S(t.query);
    node = S(t.node);
    min_count = t.min_count;
    max_count = t.max_count;
    count_multiple = t.count_multiple;
    intervals = t.intervals;
    created_at = t.created_at;
    for (int i = 0; i < t.n_presences; i++)
        presences.push_back({S(t.presences[i].user_id), S(t.presences[i].session_id), S(t.presences[i].username),
                             S(t.presences[i].node)});
    for (int i = 0; i < t.n_str_props; i++) sprops.push_back({S(t.str_props[i].key), S(t.str_props[i].value)});
    for (int i = 0; i < t.n_num_props; i++) nprops.push_back({S(t.num_props[i].key), t.num_props[i].value});
}

void Core::OwnedTicket::view(View& v) const {
    v.p.clear();
    v.s.clear();
    v.n.clear();
    for (auto& p : presences)
        v.p.push_back({p.user_id.c_str(), p.session_id.c_str(), p.username.c_str(), p.node.c_str()});
    for (auto& kv : sprops) v.s.push_back({kv.first.c_str(), kv.second.c_str()});
    for (auto& kv : nprops) v.n.push_back({kv.first.c_str(), kv.second});
    v.t = mm_ticket{ticket.c_str(), session_id.c_str(), party_id.c_str(), query.c_str(), min_count, max_count,
                    count_multiple, intervals, created_at, node.c_str(), v.p.data(), (int32_t)v.p.size(),
                    v.s.data(), (int32_t)v.s.size(), v.n.data(), (int32_t)v.n.size()};
}

Core::PendTk* Core::eff_ticket(const std::string& id) {
    auto it = pend_tk_.find(id);
    if (it != pend_tk_.end()) return &it->second;
    const int64_t s = slot_of_ticket(id);
    if (s < 0) return nullptr;
    PendTk t;
    t.alive = true;
    const ColdView c = cold_.view((uint32_t)s);
    t.session_id = std::string(c.session_id);
    t.party_id = std::string(c.party_id);
    t.node = std::string(node_dict_.str(tnode_[s]));
    c.each_presence([&](std::string_view, std::string_view sid, std::string_view, std::string_view) {
        if (std::find(t.sessions.begin(), t.sessions.end(), sid) == t.sessions.end()) t.sessions.emplace_back(sid);
    });
    return &pend_tk_.emplace(id, std::move(t)).first->second;
}

void Core::eff_remove(PendTk& t) {
    if (!t.alive) return;
    t.alive = false;
    for (auto& s : t.sessions) pend_sess_[s]--;
    if (!t.party_id.empty()) pend_party_[t.party_id]--;
}

void Core::eff_add(const OwnedTicket& ot) {
    if (PendTk* old = eff_ticket(ot.ticket)) eff_remove(*old);  // same id: replaced
    PendTk t;
    t.alive = true;
    t.session_id = ot.session_id;
    t.party_id = ot.party_id;
    t.node = ot.node;
    for (auto& p : ot.presences)
        if (std::find(t.sessions.begin(), t.sessions.end(), p.session_id) == t.sessions.end())
            t.sessions.push_back(p.session_id);
    for (auto& s : t.sessions) pend_sess_[s]++;
    if (!t.party_id.empty()) pend_party_[t.party_id]++;
    pend_tk_[ot.ticket] = std::move(t);
}

int Core::eff_sess_count(const std::string& sid) {
    const int64_t id = sess_dict_.find(sid);
    int n = id >= 0 ? (int)sess_slots_.count((uint32_t)id) : 0;
    if (pass_running_) {
        auto it = pend_sess_.find(sid);
        if (it != pend_sess_.end()) n += it->second;
    }
    return n;
}

int Core::eff_party_count(const std::string& pid) {
    const int64_t id = party_dict_.find(pid);
    int n = id >= 0 ? (int)party_slots_.count((uint32_t)id) : 0;
    if (pass_running_) {
        auto it = pend_party_.find(pid);
        if (it != pend_party_.end()) n += it->second;
    }
    return n;
}

// The queued mutations, in arrival order, against the store as the pass
// found it (their statuses were decided against that same state).
void Core::apply_pending() {
    for (PendingOp& op : pending_) {
        switch (op.kind) {
        case P_ADD:
        case P_INSERT: {
            OwnedTicket::View v;
            for (size_t i = 0; i < op.tickets.size(); i++) {
                if (!op.ok[i]) continue;
                op.tickets[i].view(v);
                add_locked(v.t, sig_of(op.cqs[i], v.t.min_count, v.t.max_count, kNoParty), op.kind == P_INSERT);
            }
            break;
        }
        case P_REMOVE_SESSION: remove_session_locked(op.a, op.b); break;
        case P_REMOVE_SESSION_ALL: remove_session_all_locked(op.a); break;
        case P_REMOVE_PARTY: remove_party_locked(op.a, op.b); break;
        case P_REMOVE_PARTY_ALL: remove_party_all_locked(op.a); break;
        case P_REMOVE_ALL: remove_all_locked(op.a); break;
        case P_REMOVE: remove_locked(op.ids); break;
        }
    }
    pending_.clear();
    pend_tk_.clear();
    pend_sess_.clear();
    pend_party_.clear();
}

int Core::drain_removed(mm_str_list* out) {
    std::lock_guard<std::mutex> lk(mu_);
    track_removed_ = true;
    auto* v = new std::vector<std::string>(std::move(removed_ids_));
    removed_ids_.clear();
    auto* ptrs = new const char*[v->empty() ? 1 : v->size()];
    for (size_t i = 0; i < v->size(); i++) ptrs[i] = (*v)[i].c_str();
    out->n = (int32_t)v->size();
    out->items = ptrs;
    str_lists_[ptrs] = v;
    return MM_OK;
}

void Core::free_str_list(mm_str_list* out) {
    if (!out || !out->items) return;
    std::lock_guard<std::mutex> lk(mu_);
    auto it = str_lists_.find(out->items);
    if (it != str_lists_.end()) {
        delete it->second;
        str_lists_.erase(it);
    }
    delete[] out->items;
    out->items = nullptr;
    out->n = 0;
}

// Insert (matchmaker.go:567-682): queries that fail to parse are skipped.
int Core::insert(const mm_ticket* ts, int32_t n) {
    if (stopped_ || n <= 0) return MM_OK;
    using clk = std::chrono::steady_clock;
    std::lock_guard<std::mutex> lk(mu_);  // also serialises use of the worker pool
    if (pass_running_) {  // queued (the pass owns the workers)
        PendingOp op{P_INSERT};
        op.tickets.reserve((size_t)n);
        op.cqs.resize((size_t)n);
        for (int i = 0; i < n; i++) {
            op.tickets.emplace_back(ts[i]);
            op.ok.push_back(compile_query(ts[i].query ? ts[i].query : "", &op.cqs[i]) == CQ_OK);
            if (op.ok.back()) eff_add(op.tickets.back());
        }
        pending_.push_back(std::move(op));
        return MM_OK;
    }
    // Repeated queries (a pool's tickets share theirs) skip the compile
    // through the signature cache; the rest compile here, under the lock.
    const auto t1 = clk::now();
    maybe_compact();
    const auto t2 = clk::now();
    // a large batch on the host workers (mm_insert.cpp); NKM_BULK=0: always
    // per ticket, =force: at any size (tests)
    double ph[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const bool bulk = bulk_mode_ != 0 && par_mode_ && (bulk_mode_ == 2 || n >= 4096) && insert_bulk(ts, n, ph);
    if (!bulk)
        for (int i = 0; i < n; i++) {
            const int64_t sg = sig_cached(ts[i]);
            if (sg >= 0) add_locked(ts[i], (uint32_t)sg, true);
        }
    const auto t3 = clk::now();
    if (n >= 1024) sync_device();  // index the batch now (bluge indexes synchronously too)
    if (std::getenv("NKM_PROFILE") && n >= 1024) {
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr,
                     "[nkm] insert %d: compact %.1f ms | %s %.1f ms (ids %.1f, sigs %.1f [queries %.1f compile %.1f "
                     "triples %.1f clauses %.1f lookup %.1f commit %.1f], strings %.1f, columns %.1f, "
                     "indexes %.1f) | sync/index/upload %.1f ms\n",
                     n, ms(t1, t2), bulk ? "bulk add" : "add (incl. compiles)", ms(t2, t3), ph[0], ph[1], ph[5], ph[6],
                     ph[7], ph[8], ph[9], ph[10], ph[2], ph[3], ph[4], ms(t3, clk::now()));
    }
    return MM_OK;
}

int Core::extract(mm_extract_list* out) {
    out->n = 0;
    out->tickets = nullptr;
    if (stopped_) return MM_OK;
    std::lock_guard<std::mutex> pl(process_mu_);  // a running pass writes Intervals
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<uint32_t> v;
    const int64_t me = node_dict_.find(node_);
    for (uint32_t s = 0; s < nslots(); s++)
        if (live_[s] && (int64_t)tnode_[s] == me) v.push_back(s);
    // One block owned by the result: the ticket array, the presence and
    // property arrays, then copies of the tickets' records and strings (the
    // store may compact or grow before the caller frees the result).
    size_t np = 0, nsp = 0, nnp = 0, bytes = 0;
    for (uint32_t s : v) {
        const ColdView c = cold_.view(s);
        np += c.n_pres;
        nsp += c.n_sp;
        nnp += c.n_np;
        bytes += cold_.record_bytes(s) + tk_len_[s] + 1 + node_dict_.str(tnode_[s]).size() + 1;
    }
    static_assert(sizeof(mm_ticket) % 8 == 0 && sizeof(mm_presence) % 8 == 0 && sizeof(mm_str_prop) % 8 == 0 &&
                      sizeof(mm_num_prop) % 8 == 0,
                  "extract block layout");
    const size_t head = v.size() * sizeof(mm_ticket) + np * sizeof(mm_presence) + nsp * sizeof(mm_str_prop) +
                        nnp * sizeof(mm_num_prop);
    char* blob = new char[head + bytes + 1];
    mm_ticket* T = reinterpret_cast<mm_ticket*>(blob);
    mm_presence* P = reinterpret_cast<mm_presence*>(T + v.size());
    mm_str_prop* SP = reinterpret_cast<mm_str_prop*>(P + np);
    mm_num_prop* NP = reinterpret_cast<mm_num_prop*>(SP + nsp);
    char* str = reinterpret_cast<char*>(NP + nnp);
    auto copy = [&](std::string_view x) {
        char* at = str;
        if (!x.empty()) std::memcpy(at, x.data(), x.size());
        at[x.size()] = 0;
        str += x.size() + 1;
        return (const char*)at;
    };
    for (size_t i = 0; i < v.size(); i++) {
        const uint32_t s = v[i];
        const size_t rb = cold_.record_bytes(s);
        std::memcpy(str, cold_.bytes.data() + cold_.off[s], rb);
        const ColdView c = ColdStore::parse(str);  // strings in the record are NUL-terminated
        str += rb;
        mm_ticket& t = T[i];
        t.ticket = copy(tk(s));
        t.session_id = c.session_id.data();
        t.party_id = c.party_id.data();
        t.query = c.query.data();
        t.min_count = minc_[s];
        t.max_count = maxc_[s];
        t.count_multiple = cm_[s];
        t.intervals = intervals_[s];
        t.created_at = created_[s];
        t.node = copy(node_dict_.str(tnode_[s]));
        t.presences = P;
        t.n_presences = (int32_t)c.n_pres;
        c.each_presence([&](std::string_view u, std::string_view se, std::string_view un, std::string_view nd) {
            *P++ = mm_presence{u.data(), se.data(), un.data(), nd.data()};
        });
        t.str_props = SP;
        t.n_str_props = (int32_t)c.n_sp;
        t.num_props = NP;
        t.n_num_props = (int32_t)c.n_np;
        c.each_prop([&](std::string_view k, std::string_view val) { *SP++ = mm_str_prop{k.data(), val.data()}; },
                    [&](std::string_view k, double d) { *NP++ = mm_num_prop{k.data(), d}; });
    }
    out->n = (int32_t)v.size();
    out->tickets = T;
    return MM_OK;
}

void Core::free_extract(mm_extract_list* out) {
    if (!out || !out->tickets) return;
    delete[] reinterpret_cast<const char*>(out->tickets);
    out->tickets = nullptr;
    out->n = 0;
}

// RemoveSession (matchmaker.go:725-767)
int Core::remove_session(const std::string& sid, const std::string& ticket) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!pass_running_) return remove_session_locked(sid, ticket);
    PendTk* t = eff_ticket(ticket);
    if (!t || !t->alive || !t->party_id.empty() || t->session_id != sid) return MM_ERR_TICKET_NOT_FOUND;
    eff_remove(*t);
    pending_.push_back(PendingOp{P_REMOVE_SESSION, {}, {}, {}, sid, ticket, {}});
    return MM_OK;
}
int Core::remove_session_locked(const std::string& sid, const std::string& ticket) {
    int64_t s = slot_of_ticket(ticket);
    if (s < 0) return MM_ERR_TICKET_NOT_FOUND;
    const ColdView c = cold_.view((uint32_t)s);
    if (!c.party_id.empty() || c.session_id != sid) return MM_ERR_TICKET_NOT_FOUND;
    kill_slot((uint32_t)s);
    return MM_OK;
}

// RemoveSessionAll (matchmaker.go:769-828)
int Core::remove_session_all(const std::string& sid) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!pass_running_) return remove_session_all_locked(sid);
    const int64_t id = sess_dict_.find(sid);
    if (id >= 0)
        for (uint32_t s : sess_slots_.list((uint32_t)id))
            if (PendTk* t = eff_ticket(std::string(tk(s)))) eff_remove(*t);
    for (auto& kv : pend_tk_)
        if (kv.second.alive && std::find(kv.second.sessions.begin(), kv.second.sessions.end(), sid) != kv.second.sessions.end())
            eff_remove(kv.second);
    pending_.push_back(PendingOp{P_REMOVE_SESSION_ALL, {}, {}, {}, sid, {}, {}});
    return MM_OK;
}
int Core::remove_session_all_locked(const std::string& sid) {
    int64_t id = sess_dict_.find(sid);
    if (id < 0) return MM_OK;
    for (uint32_t s : sess_slots_.list((uint32_t)id)) kill_slot(s);
    return MM_OK;
}

// RemoveParty (matchmaker.go:830-870)
int Core::remove_party(const std::string& pid, const std::string& ticket) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!pass_running_) return remove_party_locked(pid, ticket);
    PendTk* t = eff_ticket(ticket);
    if (!t || !t->alive || !t->session_id.empty() || t->party_id != pid) return MM_ERR_TICKET_NOT_FOUND;
    eff_remove(*t);
    pending_.push_back(PendingOp{P_REMOVE_PARTY, {}, {}, {}, pid, ticket, {}});
    return MM_OK;
}
int Core::remove_party_locked(const std::string& pid, const std::string& ticket) {
    int64_t s = slot_of_ticket(ticket);
    if (s < 0) return MM_ERR_TICKET_NOT_FOUND;
    const ColdView c = cold_.view((uint32_t)s);
    if (!c.session_id.empty() || c.party_id != pid) return MM_ERR_TICKET_NOT_FOUND;
    kill_slot((uint32_t)s);
    return MM_OK;
}

// RemovePartyAll (matchmaker.go:872-917)
int Core::remove_party_all(const std::string& pid) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!pass_running_) return remove_party_all_locked(pid);
    if (pid.empty()) return MM_OK;
    const int64_t id = party_dict_.find(pid);
    if (id >= 0)
        for (uint32_t s : party_slots_.list((uint32_t)id))
            if (PendTk* t = eff_ticket(std::string(tk(s)))) eff_remove(*t);
    for (auto& kv : pend_tk_)
        if (kv.second.alive && kv.second.party_id == pid) eff_remove(kv.second);
    pending_.push_back(PendingOp{P_REMOVE_PARTY_ALL, {}, {}, {}, pid, {}, {}});
    return MM_OK;
}
int Core::remove_party_all_locked(const std::string& pid) {
    int64_t id = party_dict_.find(pid);
    if (id < 0 || pid.empty()) return MM_OK;
    for (uint32_t s : party_slots_.list((uint32_t)id)) kill_slot(s);
    return MM_OK;
}

// RemoveAll (matchmaker.go:919-970)
int Core::remove_all(const std::string& node) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!pass_running_) return remove_all_locked(node);
    const int64_t nid = node_dict_.find(node);
    for (uint32_t s = 0; s < nslots(); s++)
        if (live_[s] && (int64_t)tnode_[s] == nid)
            if (PendTk* t = eff_ticket(std::string(tk(s)))) eff_remove(*t);
    for (auto& kv : pend_tk_)
        if (kv.second.alive && kv.second.node == node) eff_remove(kv.second);
    pending_.push_back(PendingOp{P_REMOVE_ALL, {}, {}, {}, node, {}, {}});
    return MM_OK;
}
int Core::remove_all_locked(const std::string& node) {
    const int64_t nid = node_dict_.find(node);
    for (uint32_t s = 0; s < nslots(); s++)
        if (live_[s] && (int64_t)tnode_[s] == nid) kill_slot(s);
    return MM_OK;
}

// Remove (matchmaker.go:972-1024)
int Core::remove(const char* const* tickets, int32_t n) {
    std::vector<std::string> ids;
    ids.reserve((size_t)std::max(n, 0));
    for (int i = 0; i < n; i++) ids.emplace_back(tickets[i] ? tickets[i] : "");
    std::lock_guard<std::mutex> lk(mu_);
    if (!pass_running_) return remove_locked(ids);
    for (auto& id : ids)
        if (PendTk* t = eff_ticket(id)) eff_remove(*t);
    pending_.push_back(PendingOp{P_REMOVE, {}, {}, {}, {}, {}, std::move(ids)});
    return MM_OK;
}
int Core::remove_locked(const std::vector<std::string>& ids) {
    for (auto& id : ids) {
        int64_t s = slot_of_ticket(id);
        if (s >= 0) kill_slot((uint32_t)s);
    }
    return MM_OK;
}

int32_t Core::session_ticket_count(const std::string& sid) {
    std::lock_guard<std::mutex> lk(mu_);
    return eff_sess_count(sid);
}
int32_t Core::party_ticket_count(const std::string& pid) {
    std::lock_guard<std::mutex> lk(mu_);
    return pid.empty() ? 0 : eff_party_count(pid);
}

// Membership in m.indexes, queued mutations included; large lists on the
// workers (read-only lookups) when no pass owns them.
int32_t Core::find_tickets(const char* const* ids, int32_t n, uint8_t* found) {
    std::lock_guard<std::mutex> lk(mu_);
    auto one = [&](int32_t i) -> uint8_t {
        const std::string_view id = ids[i] ? std::string_view(ids[i]) : std::string_view();
        if (pass_running_ && !pend_tk_.empty()) {
            auto it = pend_tk_.find(std::string(id));
            if (it != pend_tk_.end()) return it->second.alive ? 1 : 0;
        }
        return slot_of_ticket(id) >= 0 ? 1 : 0;
    };
    if (n >= 65536 && par_mode_ && !pass_running_) {
        WorkPool& wp = workers();
        const size_t nch = (size_t)wp.size() * 4;
        std::vector<int32_t> cnt(nch, 0);
        wp.run(nch, [&](size_t c) {
            int32_t k = 0;
            for (int32_t i = (int32_t)((size_t)n * c / nch); i < (int32_t)((size_t)n * (c + 1) / nch); i++) k += found[i] = one(i);
            cnt[c] = k;
        });
        int32_t k = 0;
        for (int32_t x : cnt) k += x;
        return k;
    }
    int32_t k = 0;
    for (int32_t i = 0; i < n; i++) k += found[i] = one(i);
    return k;
}

int32_t Core::ticket_count() {
    std::lock_guard<std::mutex> lk(mu_);
    return (int32_t)n_live_;
}
int32_t Core::active_count() {
    std::lock_guard<std::mutex> lk(mu_);
    int32_t n = 0;
    for (uint32_t s : active_list_) n += is_active_[s] && live_[s];
    return n;
}

void Core::set_hot(uint32_t s) {
    HotRec& h = hot_[s];
    h.party = party_[s];
    h.pres_off = pres_off_[s];
    h.sess0 = pres_off_[s + 1] > pres_off_[s] ? pres_sess_[pres_off_[s]] : kNoSlot;
    h.count = count_[s];
    h.minc = minc_[s];
    h.maxc = maxc_[s];
    h.cm = cm_[s];
    h.smask = 0;
    for (uint32_t p = pres_off_[s]; p < pres_off_[s + 1]; p++) h.smask |= 1u << (pres_sess_[p] & 31);
}

void Core::maybe_compact() {
    size_t n = nslots();
    // a process result still held by the caller points into the string arena
    if (out_in_use_.load()) return;
    if (n >= 65536 && n > 2 * (size_t)n_live_) compact();
}

// Drops dead slots and renumbers the store (preserves relative slot order, so
// the scan order stays sorted and insertion-order tie-breaks are unchanged).
// The work is proportional to the slot count for the fixed-size columns —
// one column per host worker — and to the live tickets for strings and
// dictionaries (a store whose tickets all matched drops its arenas as a few
// blocks, and its columns are simply emptied).
void Core::compact() {
    using cclk = std::chrono::steady_clock;
    const auto c0 = cclk::now();
    double cph[6] = {0, 0, 0, 0, 0, 0};
    auto lap = [&, t = c0](int k) mutable {
        const auto now = cclk::now();
        cph[k] = std::chrono::duration<double, std::milli>(now - t).count();
        t = now;
    };
    const size_t n = nslots();
    std::vector<uint32_t> remap(n, kNoSlot);
    uint32_t m = 0;
    for (uint32_t s = 0; s < n; s++)
        if (live_[s]) remap[s] = m++;
    const bool none = m == 0;  // every ticket left (a drained store)
    auto keep = [&](auto& vec) {
        if (none) {
            vec.clear();
            return;
        }
        size_t w = 0;
        for (uint32_t s = 0; s < n; s++)
            if (live_[s]) vec[w++] = std::move(vec[s]);
        vec.resize(w);
    };
    // presences CSR and sessions (the session dictionary is rebuilt so it
    // holds live sessions only)
    std::vector<uint32_t> npoff{0};
    std::vector<uint32_t> npsess;
    Dict nsess;
    for (uint32_t s = 0; s < n && !none; s++) {
        if (!live_[s]) continue;
        for (uint32_t p = pres_off_[s]; p < pres_off_[s + 1]; p++)
            npsess.push_back(nsess.intern(sess_dict_.str(pres_sess_[p])));
        npoff.push_back((uint32_t)npsess.size());
    }
    lap(0);
    pres_off_ = std::move(npoff);
    pres_sess_ = std::move(npsess);
    sess_dict_ = std::move(nsess);
    // party dictionary: live parties only
    {
        Dict np;
        for (uint32_t s = 0; s < n && !none; s++)
            if (live_[s] && party_[s] != kNoParty) party_[s] = np.intern(party_dict_.str(party_[s]));
        party_dict_ = std::move(np);
    }
    // ticket-id arena: live ids only
    {
        StrArena na;
        for (uint32_t s = 0; s < n && !none; s++)
            if (live_[s]) tk_ptr_[s] = na.put(tk(s));
        tk_arena_ = std::move(na);
    }
    lap(1);
    if (none) cold_.clear();
    else cold_.compact(live_);
    {
        // the columns, one job each on the workers
        std::vector<std::function<void()>> jobs = {
            [&] { keep(tk_ptr_); },   [&] { keep(tk_len_); }, [&] { keep(tnode_); },    [&] { keep(created_); },
            [&] { keep(ckey_); },     [&] { keep(minc_); },   [&] { keep(maxc_); },     [&] { keep(cm_); },
            [&] { keep(count_); },    [&] { keep(intervals_); }, [&] { keep(party_); }, [&] { keep(is_active_); },
            [&] { keep(sig_); },      [&] { keep(squery_); }, [&] { keep(indexed_); }, [&] { keep(self_match_); }};
        for (size_t f = 0; f < fval_.size(); f++)
            if (fval_[f].size() == n) {
                jobs.push_back([&, f] { keep(fval_[f]); });
                jobs.push_back([&, f] { keep(fkind_[f]); });
            }
        if (none || !par_mode_) for (auto& j : jobs) j();
        else workers().run(jobs.size(), [&](size_t k) { jobs[k](); });
    }
    lap(2);
    live_.assign(m, 1);
    hot_.resize(m);
    for (uint32_t s = 0; s < m; s++) set_hot(s);
    // maps
    slot_of_.clear();
    slot_of_.reserve(m);
    for (uint32_t s = 0; s < m; s++) slot_of_.put_new(str_hash(tk(s)), s);
    sess_slots_.clear();
    party_slots_.clear();
    for (uint32_t s = 0; s < m; s++) {
        uint32_t p0 = pres_off_[s], p1 = pres_off_[s + 1];
        for (uint32_t p = p0; p < p1; p++) {
            bool dup = false;
            for (uint32_t q = p0; q < p; q++) dup |= pres_sess_[q] == pres_sess_[p];
            if (!dup) sess_slots_.add(pres_sess_[p], s);
        }
        if (party_[s] != kNoParty) party_slots_.add(party_[s], s);
    }
    lap(3);
    // signatures and clauses: the live tickets' only (a workload of unique
    // queries would grow them without bound); renumbered in slot order
    {
        std::vector<uint32_t> smap(sigs_.size(), UINT32_MAX);
        std::vector<Sig> ns;
        std::vector<DClause> nc;
        for (uint32_t s = 0; s < m; s++) {
            uint32_t& g = sig_[s];
            if (smap[g] == UINT32_MAX) {
                smap[g] = (uint32_t)ns.size();
                Sig x = sigs_[g];
                const uint32_t off = (uint32_t)nc.size();
                nc.insert(nc.end(), clauses_.begin() + x.clause_off, clauses_.begin() + x.clause_off + x.n_clauses);
                x.clause_off = off;
                ns.push_back(std::move(x));
            }
            g = smap[g];
            squery_[s].clause_off = ns[g].clause_off;
        }
        sigs_.swap(ns);
        sig_fmask_.resize(sigs_.size());
        for (size_t g = 0; g < sigs_.size(); g++) sig_fmask_[g] = sigs_[g].must_fmask;
        sig_lite_.resize(sigs_.size());
        for (size_t g = 0; g < sigs_.size(); g++) sig_lite_[g] = lite_of(sigs_[g]);
        clauses_.swap(nc);
        sig_idx_.clear();
        sig_idx_.reserve(sigs_.size());
        for (uint32_t g = 0; g < sigs_.size(); g++) {
            const Sig& x = sigs_[g];
            sig_idx_.put_new(sig_hash(sig_clause_hash(clauses_.data() + x.clause_off, x.n_clauses), x.qkind, x.tmin,
                                      x.tmax, x.tparty),
                             g);
        }
        dev_clauses_ = 0;
        qtext_.clear();  // the (query, counts) -> signature cache holds old ids
        qstatus_.clear();
        qsig_.clear();
        qsig_idx_.clear();
    }
    lap(4);
    std::vector<uint32_t> nact;
    for (uint32_t s : active_list_)
        if (remap[s] != kNoSlot && is_active_[remap[s]]) nact.push_back(remap[s]);
    active_list_ = std::move(nact);
    active_exact_ = true;  // remapped slots are live
    std::vector<uint32_t> nord;
    for (size_t k = 0; k < order_.size() && !none; k++)
        if (remap[order_[k]] != kNoSlot) nord.push_back(remap[order_[k]]);
    order_ = std::move(nord);
    pending_dead_.clear();
    apply_defer_.clear();  // old slot numbers; the re-upload below carries the flags
    monotone_ = true;      // the live slots alone
    for (uint32_t s = 1; s < m && monotone_; s++) monotone_ = created_[s] > created_[s - 1] && ckey_[s] > ckey_[s - 1];
    index_dirty_ = true;
    dev_slots_ = 0;
    for (auto& d : dev_field_slots_) d = 0;
    n_live_ = m;
    lap(5);
    if (std::getenv("NKM_PROFILE"))
        std::fprintf(stderr,
                     "[nkm] compact %zu -> %u slots: remap+sessions %.2f, parties+ids %.2f, cold+columns %.2f, "
                     "hot+maps %.2f, signatures %.2f, lists %.2f ms\n",
                     n, m, cph[0], cph[1], cph[2], cph[3], cph[4], cph[5]);
}

// ---------------------------------------------------------------------------
// HBM mirror
// ---------------------------------------------------------------------------
void Core::ensure_field_on_device(uint16_t f) {
    if (!d_fval_[f]) {
        d_fval_[f] = new DevArray<int64_t>();
        d_fkind_[f] = new DevArray<uint8_t>();
        dev_field_slots_[f] = 0;
    }
}

void Core::build_index() {
    const uint32_t n = (uint32_t)nslots();
    // scan order: slots sorted by (sortable float64(CreatedAt), slot)
    if (!order_sorted_ || order_.size() != n) {
        order_.resize(n);
        for (uint32_t s = 0; s < n; s++) order_[s] = s;
        std::stable_sort(order_.begin(), order_.end(), [&](uint32_t a, uint32_t b) { return ckey_[a] < ckey_[b]; });
        order_sorted_ = true;
    }
    order_identity_ = true;
    for (uint32_t p = 0; p < n && order_identity_; p++) order_identity_ = order_[p] == p;
    // posting lists for fields used as required-term sources
    postings_map_.clear();
    postings_.clear();
    std::vector<uint16_t> pf;
    for (size_t f = 0; f < field_posting_.size(); f++)
        if (field_posting_[f]) pf.push_back((uint16_t)f);
    if (!pf.empty()) {
        for (uint32_t s : order_) {
            if (!live_[s]) continue;
            for (uint16_t f : pf) {
                if (fkind_[f][s] != KIND_KEYWORD) continue;
                uint64_t key = ((uint64_t)f << 32) | (uint64_t)(uint32_t)fval_[f][s];
                postings_map_[key].len++;
            }
        }
        uint32_t off = 0;
        postings_map_.for_each([&](PostingRange& r) { r.off = off; off += r.len; r.head = r.off; });
        postings_.resize(off);
        for (uint32_t s : order_) {
            if (!live_[s]) continue;
            for (uint16_t f : pf) {
                if (fkind_[f][s] != KIND_KEYWORD) continue;
                uint64_t key = ((uint64_t)f << 32) | (uint64_t)(uint32_t)fval_[f][s];
                auto& r = postings_map_[key];
                postings_[r.head++] = s;
            }
        }
        postings_map_.for_each([](PostingRange& r) { r.head = 0; });
    }
    order_head_ = 0;
    d_order_.reserve(std::max<size_t>(n, 1), false);
    if (n) NKM_HIP(hipMemcpyAsync(d_order_.p, order_.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice, stream_));
    d_postings_.reserve(std::max<size_t>(postings_.size(), 1), false);
    if (!postings_.empty())
        NKM_HIP(hipMemcpyAsync(d_postings_.p, postings_.data(), postings_.size() * sizeof(uint32_t),
                               hipMemcpyHostToDevice, stream_));
    index_dirty_ = false;
}

void Core::sync_device() {
    NKM_HIP(hipSetDevice(device_));
    const size_t n = nslots();
    const size_t need = std::max<size_t>(n, 1);
    bool regrow = need > dev_cap_;
    if (regrow) {
        size_t cap = std::max(need, dev_cap_ + dev_cap_ / 2);
        d_alive_.reserve(cap);
        d_minc_.reserve(cap);
        d_maxc_.reserve(cap);
        d_party_.reserve(cap);
        d_squery_.reserve(cap);
        dev_cap_ = cap;
    }
    auto up = [&](auto* dst, const auto* src, size_t from, size_t to) {
        if (to > from)
            NKM_HIP(hipMemcpyAsync(dst + from, src + from, (to - from) * sizeof(*src), hipMemcpyHostToDevice, stream_));
    };
    if (dev_slots_ < n) {
        // device alive = in the search index: in m.indexes and not a dropped
        // group's member (indexed_)
        std::vector<uint8_t> alive(n - dev_slots_);
        for (size_t s = dev_slots_; s < n; s++) alive[s - dev_slots_] = live_[s] & indexed_[s];
        NKM_HIP(hipMemcpyAsync(d_alive_.p + dev_slots_, alive.data(), alive.size(), hipMemcpyHostToDevice, stream_));
        NKM_HIP(hipStreamSynchronize(stream_));  // the staging vector dies here
        up(d_minc_.p, minc_.data(), dev_slots_, n);
        up(d_maxc_.p, maxc_.data(), dev_slots_, n);
        up(d_party_.p, party_.data(), dev_slots_, n);
        up(d_squery_.p, squery_.data(), dev_slots_, n);
    }
    flush_apply();  // the last pass's selections (slots below dev_slots_)
    // dead slots that were already on the device
    if (!pending_dead_.empty()) {
        std::vector<uint32_t> v;
        for (uint32_t s : pending_dead_)
            if (s < dev_slots_) v.push_back(s);
        if (!v.empty()) apply_selected_to_device(v.data(), v.size());
        pending_dead_.clear();
    }
    dev_slots_ = n;
    if (clauses_.size() > dev_clauses_ || !d_clauses_.p) {
        d_clauses_.reserve(std::max<size_t>(clauses_.size(), 1));
        up(d_clauses_.p, clauses_.data(), dev_clauses_, clauses_.size());
        dev_clauses_ = clauses_.size();
    }
    bool ptrs_dirty = d_fval_ptrs_.cap < fval_.size();
    for (size_t f = 0; f < fval_.size(); f++) {
        if (!field_used_[f]) continue;
        ensure_field_on_device((uint16_t)f);
        if (d_fval_[f]->cap < need) {
            d_fval_[f]->reserve(std::max(need, dev_cap_));
            d_fkind_[f]->reserve(std::max(need, dev_cap_));
            ptrs_dirty = true;
        }
        if (dev_field_slots_[f] < n) {
            up(d_fval_[f]->p, fval_[f].data(), dev_field_slots_[f], n);
            up(d_fkind_[f]->p, fkind_[f].data(), dev_field_slots_[f], n);
            dev_field_slots_[f] = n;
        }
    }
    if (ptrs_dirty || d_fval_ptrs_.cap < fval_.size() || true) {
        std::vector<int64_t*> pv(std::max<size_t>(fval_.size(), 1), nullptr);
        std::vector<uint8_t*> pk(std::max<size_t>(fval_.size(), 1), nullptr);
        for (size_t f = 0; f < fval_.size(); f++) {
            if (d_fval_[f]) { pv[f] = d_fval_[f]->p; pk[f] = d_fkind_[f]->p; }
        }
        d_fval_ptrs_.reserve(pv.size(), false);
        d_fkind_ptrs_.reserve(pk.size(), false);
        NKM_HIP(hipMemcpyAsync(d_fval_ptrs_.p, pv.data(), pv.size() * sizeof(int64_t*), hipMemcpyHostToDevice, stream_));
        NKM_HIP(hipMemcpyAsync(d_fkind_ptrs_.p, pk.data(), pk.size() * sizeof(uint8_t*), hipMemcpyHostToDevice, stream_));
    }
    if (index_dirty_) build_index();
    refresh_termsets();
    NKM_HIP(hipStreamSynchronize(stream_));
}

DStore Core::dstore() const {
    DStore st;
    st.alive = d_alive_.p;
    st.minc = d_minc_.p;
    st.maxc = d_maxc_.p;
    st.party = d_party_.p;
    st.squery = d_squery_.p;
    st.clauses = d_clauses_.p;
    st.fval = d_fval_ptrs_.p;
    st.fkind = d_fkind_ptrs_.p;
    st.order = d_order_.p;
    st.postings = d_postings_.p;
    st.tset_desc = d_tset_desc_.p;
    st.tset_ids = d_tset_ids_.p;
    st.tset_sc = d_tset_sc_.p;
    st.n_fields = (uint32_t)std::max<size_t>(fval_.size(), 1);
    return st;
}

void Core::defer_apply(UVec<uint32_t>& newly) {
    if (newly.empty()) return;
    flush_apply();
    apply_defer_.swap(newly);  // newly keeps the other buffer's capacity
    newly.clear();
}

void Core::flush_apply() {
    if (apply_defer_.empty()) return;
    apply_selected_to_device(apply_defer_.data(), apply_defer_.size());
    apply_defer_.clear();
}

// Clears the device alive flags of the given slots.  Asynchronous: the copy
// and kernel are ordered before the next search on the library's stream; the
// pinned staging buffer is reused only after the previous copy completed.
void Core::apply_selected_to_device(const uint32_t* slots, size_t n_slots) {
    if (!n_slots) return;
    if (apply_pending_) {
        NKM_HIP(hipEventSynchronize(apply_ev_));
        apply_pending_ = false;
    }
    h_slots_tmp_.reserve(n_slots);
    if (n_slots >= (1u << 20) && par_mode_) {  // a whole pass's selection (C3: 7 MB) copies on the workers
        WorkPool& wp = workers();
        const size_t nch = wp.size();
        wp.run(nch, [&](size_t c) {
            const size_t lo = n_slots * c / nch, hi = n_slots * (c + 1) / nch;
            std::memcpy(h_slots_tmp_.p + lo, slots + lo, (hi - lo) * sizeof(uint32_t));
        });
    } else {
        std::memcpy(h_slots_tmp_.p, slots, n_slots * sizeof(uint32_t));
    }
    d_slots_tmp_.reserve(n_slots, false);
    NKM_HIP(hipMemcpyAsync(d_slots_tmp_.p, h_slots_tmp_.p, n_slots * sizeof(uint32_t), hipMemcpyHostToDevice,
                           stream_));
    NKM_HIP(launch_clear_alive(d_alive_.p, d_slots_tmp_.p, (uint32_t)n_slots, stream_));
    NKM_HIP(hipEventRecord(apply_ev_, stream_));
    apply_pending_ = true;
}

}  // namespace nkm
