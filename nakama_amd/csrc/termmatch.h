// nakama_amd/csrc/termmatch.h — multi-term clauses of the query language:
// regexp (`f:/re/`), wildcard (`f:a*b?`) and fuzzy (`f:term~N`).
//
// bluge evaluates these by enumerating the field's term dictionary through an
// automaton and OR-ing one TermSearcher per accepted term
// (search/searcher/search_regexp.go:27-84, search_fuzzy.go:43-143,
// search_multi_term.go:23-177).  Here the same enumeration runs on the host over
// the store's keyword dictionary (append-only, so each pattern's accepted-id set
// is extended incrementally), and the device evaluates "keyword id in set" with a
// binary search (mm_kernels.hip, OP_TERMSET).
//
// Regexp language: Go regexp/syntax with syntax.Perl flags (the parse of
// parseRegexp, search_regexp.go:61-66), restricted to what
// vellum/regexp/compile.go:56-200 compiles; the automaton accepts a term when
// the whole term matches (anchored both ends).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace nkm {

// Status of a pattern, decided once at compile time.
enum MtStatus {
    MT_OK = 0,
    MT_SEARCH_ERROR = 1,  // bluge accepts the query but every search with it fails (processDefault `continue`)
    MT_UNSUPPORTED = 2,   // reserved: valid in Go, not lowered here (none remain: script classes and (?U) are lowered)
};

class GoRegexp {
public:
    // Parses `pattern` (already stripped of one leading '^', query.go:1264-1265).
    MtStatus compile(const std::string& pattern);
    bool full_match(const std::string& term) const;

private:
    enum Op : uint8_t { I_CLASS, I_SPLIT, I_JMP, I_MATCH };
    struct Inst {
        Op op;
        uint32_t x = 0, y = 0;  // SPLIT targets / JMP target / CLASS index
    };
    std::vector<Inst> prog_;
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> classes_;  // sorted rune ranges
    friend struct RxCompiler;
};

// Restricted Damerau-Levenshtein (optimal string alignment) distance over
// runes, or max+1 when it exceeds `max`: the language of vellum's
// levenshtein automaton built with transpositions (search_fuzzy.go:34-38).
int osa_distance_runes(const std::string& a, const std::string& b, int max);

struct TermMatcher {
    enum Kind : uint8_t { K_REGEXP = 1, K_FUZZY = 2 } kind = K_REGEXP;
    std::string pattern;  // regexp text, or the fuzzy term
    int fuzziness = 0;
    GoRegexp re;
    // Accepts `term`?  *boost: the per-term boost (1 for regexp; for fuzzy
    // 1 - distance/min(rune lengths), search_fuzzy.go:113-126).
    bool accept(const std::string& term, double* boost) const;
};

// wildcardRegexpReplacer (bluge/query.go:1455-1473): a wildcard to its regexp.
std::string wildcard_to_regexp(const std::string& w);

}  // namespace nkm
