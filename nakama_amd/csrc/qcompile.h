// nakama_amd/csrc/qcompile.h — ticket query string -> predicate/boost bytecode.
//
// Accepts the language of blugelabs/query_string v0.3.0 as used by
// ParseQueryString (server/match_common.go:244-251): "*" = match all, "" =
// match none, otherwise a flat list of [+|-]clause[^boost] parts
// (query_string.y:31-233).  Each part lowers to one Clause with a precomputed
// score contribution reproducing bluge's composite scoring
// (vendor/.../bluge/query.go:198-229, 950-1005, 1146-1156;
// search/similarity/composite.go:37-43).
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace nkm {

enum ClauseOp : uint8_t {
    OP_TERM = 0,    // keyword field value == term                       (MatchQuery, keyword analyzer)
    OP_RANGE = 1,   // numeric/datetime term value in [lo, hi]            (Numeric/DateRangeQuery)
    OP_NUMLIT = 2,  // keyword == term  OR  numeric term value == lo      (queryStringNumberToken)
    OP_FALSE = 3,   // never matches (phrase on untokenised fields, unfielded `_all` clauses)
    OP_TERMSET = 4, // keyword value in the accepted-term set of a regexp/wildcard/fuzzy matcher (termmatch.h)
};
enum Occur : uint8_t { OCC_MUST = 0, OCC_SHOULD = 1, OCC_MUSTNOT = 2 };

struct HostClause {
    ClauseOp op = OP_FALSE;
    Occur occur = OCC_SHOULD;
    std::string field;  // full field name, e.g. "properties.region", "min_count"
    std::string term;   // TERM / NUMLIT keyword form
    int64_t lo = 0, hi = 0;
    double score = 1.0; // contribution when matched (TERMSET: the query boost b)
    uint8_t mt_kind = 0; // TERMSET: TermMatcher::Kind; `term` holds the regexp / fuzzy term
    int fuzziness = 0;
};

enum QueryKind : uint8_t { QK_BOOL = 0, QK_MATCHALL = 1, QK_MATCHNONE = 2 };

struct CompiledQuery {
    QueryKind kind = QK_MATCHNONE;
    std::vector<HostClause> clauses;
};

enum CompileStatus { CQ_OK = 0, CQ_INVALID = -1, CQ_UNSUPPORTED = -8 };

// Compiles `q`; CQ_INVALID mirrors ErrMatchmakerQueryInvalid (parse or Validate
// failure, server/matchmaker.go:449-457).  A regexp that Go's parser (or
// vellum's compiler) rejects, or a fuzziness outside [0, 2], is accepted at Add
// (RegexpQuery.Validate returns nil, query.go:1271-1273) but fails every search:
// such a query compiles to QK_MATCHNONE, the outcome of processDefault's
// `continue` on a search error (matchmaker_process.go:97-101).  CQ_UNSUPPORTED is
// reserved for a construct Go accepts that is not lowered here: none remains
// (Unicode category and script classes, flag groups incl. (?U), POSIX classes
// are all lowered, termmatch.h).
int compile_query(std::string_view q, CompiledQuery* out);

}  // namespace nkm
