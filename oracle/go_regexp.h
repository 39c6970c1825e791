// oracle/go_regexp.h — TEST INFRASTRUCTURE ONLY (part of the CPU oracle; never
// linked into the product).  Restates, for the oracle's per-document query
// evaluation, the term matching of bluge's multi-term queries:
//   * RegexpQuery / WildcardQuery (vendor/.../bluge/query.go:1254-1273,
//     1455-1485; search/searcher/search_regexp.go:27-100): the pattern is parsed
//     by Go regexp/syntax with syntax.Perl flags and compiled by
//     vellum/regexp/compile.go:56-200, which rejects anchors, word boundaries and
//     lazy repetitions; a term matches when the WHOLE term is in the language;
//   * FuzzyQuery (search_fuzzy.go:43-143): terms within restricted
//     Damerau-Levenshtein distance <= fuzziness (vellum levenshtein automaton built
//     with transpositions), per-term boost 1 - d / min(rune lengths).
// Parsing is a direct recursive restatement of the grammar; matching computes
// the set of end positions reachable from each start position over the term's
// runes (no automaton), an independent method from the product's Pike VM.
#pragma once
#include <algorithm>
#include <cstdint>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "unicode_ref.h"  // data only, the oracle's own layout: Unicode 13 category / script runs, SimpleFold

namespace oracle_re {

enum Status { OK = 0, SEARCH_ERROR = 1, UNSUPPORTED = 2 };

// UTF-8 -> runes; invalid bytes -> -1 (a rune no class contains).
inline std::vector<int32_t> runes(const std::string& s, bool bad_as_fffd) {
    std::vector<int32_t> out;
    size_t i = 0;
    while (i < s.size()) {
        unsigned char c = s[i];
        int n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
        int32_t r = -1;
        if (n == 1) r = c;
        else if (n > 1 && i + n <= s.size()) {
            r = c & (0x7F >> n);
            for (int k = 1; k < n; k++) {
                unsigned char d = s[i + k];
                if ((d >> 6) != 2) { r = -1; break; }
                r = (r << 6) | (d & 0x3F);
            }
            static const int32_t kMin[5] = {0, 0, 0x80, 0x800, 0x10000};
            if (r >= 0 && (r < kMin[n] || r > 0x10FFFF || (r >= 0xD800 && r < 0xE000))) r = -1;
        }
        if (r < 0) { i++; out.push_back(bad_as_fffd ? 0xFFFD : -1); }
        else { i += n; out.push_back(r); }
    }
    return out;
}

struct Re {
    enum K { SET, SEQ, OR, REP } k = SEQ;
    std::vector<std::pair<int32_t, int32_t>> set;  // SET: rune ranges
    bool neg = false;
    std::vector<std::shared_ptr<Re>> kids;
    int lo = 0, hi = 0;  // REP: hi < 0 = unbounded
    bool has(int32_t r) const {
        if (r < 0) return false;
        bool in = false;
        for (auto& p : set) in = in || (r >= p.first && r <= p.second);
        return in != neg;
    }
};
using RP = std::shared_ptr<Re>;

using RangeV = std::vector<std::pair<int32_t, int32_t>>;

// unicode.SimpleFold (the next rune of r's orbit; r itself when alone)
inline int32_t simple_fold(int32_t r) {
    int lo = 0, hi = uref::kNFold;
    while (lo < hi) {
        const int mid = (lo + hi) / 2;
        if ((int32_t)uref::kSimpleFold[mid].r < r) lo = mid + 1;
        else hi = mid;
    }
    return lo < uref::kNFold && (int32_t)uref::kSimpleFold[lo].r == r ? (int32_t)uref::kSimpleFold[lo].next : r;
}

// (?i): every rune of the set brings its whole SimpleFold orbit (vellum
// expands FoldCase literals through unicode.SimpleFold; Go's parser folds
// classes the same way).
inline void fold_in(RangeV& rs) {
    RangeV add;
    for (int k = 0; k < uref::kNFold; k++) {
        const int32_t r = (int32_t)uref::kSimpleFold[k].r;
        bool in = false;
        for (auto& q : rs) in = in || (r >= q.first && r <= q.second);
        if (!in) continue;
        for (int32_t x = simple_fold(r); x != r; x = simple_fold(x)) add.push_back({x, x});
    }
    rs.insert(rs.end(), add.begin(), add.end());
}

// The runes of a Go class name: unicode.Categories (two-letter categories
// without Cn, and the one-letter unions, C without Cn), then unicode.Scripts
// (regexp/syntax unicodeTable); false for any other name.
inline bool named_class(const std::string& n, RangeV* out) {
    int want_cat = -1, want_script = -1;
    bool union_of = false;
    if (n.size() == 2 && n != "Cn") {
        for (int k = 0; k < uref::kNCat; k++)
            if (n == uref::kCatName[k]) want_cat = k;
    } else if (n.size() == 1 && std::string("CLMNPSZ").find(n[0]) != std::string::npos) {
        union_of = true;
    }
    if (want_cat < 0 && !union_of)
        for (int k = 1; k < uref::kNScript; k++)
            if (n == uref::kScriptName[k]) want_script = k;
    if (want_cat < 0 && !union_of && want_script < 0) return false;
    out->clear();
    for (int k = 0; k < uref::kNRuns; k++) {
        const uref::Run& r = uref::kRuns[k];
        const char* cn = uref::kCatName[r.cat];
        const bool in = union_of ? (cn[0] == n[0] && std::string(cn) != "Cn")
                                 : want_cat >= 0 ? (int)r.cat == want_cat : (int)r.script == want_script;
        if (!in) continue;
        if (!out->empty() && out->back().second + 1 == (int32_t)r.lo) out->back().second = (int32_t)r.hi;
        else out->push_back({(int32_t)r.lo, (int32_t)r.hi});
    }
    return true;
}

// complement within [0, 0x10FFFF]
inline RangeV complement(RangeV rs) {
    std::sort(rs.begin(), rs.end());
    RangeV out;
    int32_t nx = 0;
    for (auto& q : rs) {
        if (q.first > nx) out.push_back({nx, q.first - 1});
        nx = std::max(nx, q.second + 1);
    }
    if (nx <= 0x10FFFF) out.push_back({nx, 0x10FFFF});
    return out;
}

struct Parse {
    std::vector<int32_t> p;  // pattern runes
    size_t i = 0;
    int nest = 0;
    // (?i) FoldCase, (?s) DotNL, (?U) NonGreedy in effect.  NonGreedy is
    // stamped on every node parsed while it holds (regexp/syntax copies the
    // flags into each literal, class and capture), and vellum rejects any
    // node carrying it (compile.go:57-59, ErrNoLazy): under (?U) every atom
    // is a search error; empty groups and flag groups parse to no node.
    bool fc = false, dn = false, ug = false;
    struct Fail { Status s; };
    [[noreturn]] void fail() { throw Fail{SEARCH_ERROR}; }
    [[noreturn]] void unsup() { throw Fail{UNSUPPORTED}; }
    bool at_end() const { return i >= p.size(); }
    int32_t cur(size_t k = 0) const { return i + k < p.size() ? p[i + k] : -2; }

    static RP single(int32_t a, int32_t b) { auto r = std::make_shared<Re>(); r->k = Re::SET; r->set = {{a, b}}; return r; }
    RP literal(int32_t a) {  // a pattern rune (folded under (?i))
        RP r = single(a, a);
        if (fc) fold_in(r->set);
        return r;
    }
    // a named group's runes (perl / POSIX / Unicode class), folded under (?i),
    // complemented for the negative form
    RangeV group(RangeV g, bool negative) const {
        if (fc) fold_in(g);
        return negative ? complement(g) : g;
    }
    static bool posix(const std::vector<int32_t>& name, RangeV* out) {
        std::string n;
        for (int32_t c : name) { if (c < 0 || c > 0x7e) return false; n.push_back((char)c); }
        if (n == "alnum") *out = {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}};
        else if (n == "alpha") *out = {{'A', 'Z'}, {'a', 'z'}};
        else if (n == "ascii") *out = {{0, 127}};
        else if (n == "blank") *out = {{9, 9}, {32, 32}};
        else if (n == "cntrl") *out = {{0, 31}, {127, 127}};
        else if (n == "digit") *out = {{'0', '9'}};
        else if (n == "graph") *out = {{33, 126}};
        else if (n == "lower") *out = {{'a', 'z'}};
        else if (n == "print") *out = {{32, 126}};
        else if (n == "punct") *out = {{33, 47}, {58, 64}, {91, 96}, {123, 126}};
        else if (n == "space") *out = {{9, 13}, {32, 32}};
        else if (n == "upper") *out = {{'A', 'Z'}};
        else if (n == "word") *out = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
        else if (n == "xdigit") *out = {{'0', '9'}, {'A', 'F'}, {'a', 'f'}};
        else return false;
        return true;
    }
    // at the backslash of \p / \P: the class's runes (an unknown name is
    // ErrInvalidCharRange: a search error)
    RangeV uclass() {
        bool negative = cur(1) == 'P';
        i += 2;
        std::vector<int32_t> name;
        if (cur() == '{') {
            size_t j = i + 1;
            while (j < p.size() && p[j] != '}') j++;
            if (j >= p.size()) fail();
            name.assign(p.begin() + i + 1, p.begin() + j);
            i = j + 1;
        } else {
            if (at_end()) fail();
            if (cur() < 0) fail();
            name.push_back(p[i++]);
        }
        if (!name.empty() && name[0] == '^') { negative = !negative; name.erase(name.begin()); }
        std::string n;
        for (int32_t c : name) { if (c < 0 || c > 0x7e) fail(); n.push_back((char)c); }
        RangeV g;
        if (n == "Any") g = {{0, 0x10FFFF}};
        else if (!named_class(n, &g)) fail();
        return group(g, negative);
    }
    static bool alnum(int32_t c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
    static bool odig(int32_t c) { return c >= '0' && c <= '7'; }
    static int hexd(int32_t c) {
        return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
    }
    // \d \s \w and negations as (ranges, negated)
    bool perl(int32_t c, std::vector<std::pair<int32_t, int32_t>>* rs, bool* neg) {
        int32_t l = c | 0x20;
        if (l == 'd') *rs = {{'0', '9'}};
        else if (l == 's') *rs = {{9, 10}, {12, 13}, {32, 32}};
        else if (l == 'w') *rs = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
        else return false;
        *neg = c != l;
        return true;
    }
    int32_t esc() {  // after the backslash
        if (at_end()) fail();
        int32_t c = p[i++];
        if (c >= '1' && c <= '7' && !odig(cur())) fail();
        if (odig(c)) {
            int32_t v = c - '0';
            for (int k = 0; k < 2 && odig(cur()); k++) v = v * 8 + (p[i++] - '0');
            return v;
        }
        if (c == 'x') {
            if (cur() == '{') {
                i++;
                int64_t v = 0;
                size_t st = i;
                while (hexd(cur()) >= 0) { v = v * 16 + hexd(p[i++]); if (v > 0x10FFFF) fail(); }
                if (i == st || cur() != '}') fail();
                i++;
                return (int32_t)v;
            }
            if (hexd(cur()) < 0 || hexd(cur(1)) < 0) fail();
            int32_t v = hexd(p[i]) * 16 + hexd(p[i + 1]);
            i += 2;
            return v;
        }
        switch (c) {
        case 'a': return 7;
        case 'f': return 12;
        case 'n': return 10;
        case 'r': return 13;
        case 't': return 9;
        case 'v': return 11;
        }
        if (c < 0x80 && !alnum(c)) return c;
        fail();
    }
    RP klass() {  // after '['
        auto r = std::make_shared<Re>();
        r->k = Re::SET;
        if (cur() == '^') { r->neg = true; i++; }
        bool first = true;
        std::vector<std::pair<int32_t, int32_t>> negs;  // negated perl classes inside
        while (first || cur() != ']') {
            if (at_end()) fail();
            first = false;
            if (cur() == '[' && cur(1) == ':') {  // [:name:] / [:^name:] when a ":]" follows
                size_t j = i + 2;
                while (j + 1 < p.size() && !(p[j] == ':' && p[j + 1] == ']')) j++;
                if (j + 1 < p.size()) {
                    std::vector<int32_t> name(p.begin() + i + 2, p.begin() + j);
                    bool negative = !name.empty() && name[0] == '^';
                    if (negative) name.erase(name.begin());
                    RangeV g;
                    if (!posix(name, &g)) fail();
                    RangeV gg = group(g, negative);
                    r->set.insert(r->set.end(), gg.begin(), gg.end());
                    i = j + 2;
                    continue;
                }
            }
            if (cur() == '\\' && (cur(1) == 'p' || cur(1) == 'P')) {
                RangeV gg = uclass();
                r->set.insert(r->set.end(), gg.begin(), gg.end());
                continue;
            }
            std::vector<std::pair<int32_t, int32_t>> rs;
            bool ng;
            if (cur() == '\\' && perl(cur(1), &rs, &ng)) {
                i += 2;
                RangeV gg = group(rs, ng);
                r->set.insert(r->set.end(), gg.begin(), gg.end());
                continue;
            }
            int32_t a;
            if (cur() == '\\') { i++; a = esc(); }
            else { if (cur() < 0) fail(); a = p[i++]; }
            int32_t b = a;
            if (cur() == '-' && i + 1 < p.size() && p[i + 1] != ']') {
                i++;
                if (cur() == '\\') { i++; b = esc(); }
                else { if (cur() < 0) fail(); b = p[i++]; }
                if (b < a) fail();
            }
            RangeV one{{a, b}};
            if (fc) fold_in(one);
            r->set.insert(r->set.end(), one.begin(), one.end());
        }
        i++;
        return r;
    }
    bool bounds(int* lo, int* hi) {  // at '{'
        size_t j = i + 1;
        auto num = [&](int* v) {
            size_t s = j;
            long x = 0;
            while (j < p.size() && p[j] >= '0' && p[j] <= '9') { x = std::min(100000L, x * 10 + (p[j] - '0')); j++; }
            if (j == s || (j - s > 1 && p[s] == '0')) return false;
            *v = (int)x;
            return true;
        };
        if (!num(lo)) return false;
        *hi = *lo;
        if (j < p.size() && p[j] == ',') {
            j++;
            if (j < p.size() && p[j] == '}') *hi = -1;
            else if (!num(hi)) return false;
        }
        if (j >= p.size() || p[j] != '}') return false;
        i = j + 1;
        return true;
    }
    RP atom() {
        int32_t c = cur();
        if (c == -1) fail();  // invalid UTF-8 in the pattern
        if (c == '(') {
            i++;
            const bool fc0 = fc, dn0 = dn, ug0 = ug;
            if (cur() != '?' && ug) fail();  // a capture under (?U)
            if (cur() == '?') {
                if (cur(1) == 'P' && cur(2) == '<') {
                    if (ug) fail();
                    i += 3;
                    size_t s = i;
                    while (i < p.size() && p[i] != '>') {
                        if (!(alnum(p[i]) || p[i] == '_')) fail();
                        i++;
                    }
                    if (at_end() || i == s) fail();
                    i++;
                } else {
                    // flags: [imsU]* ( '-' [imsU]+ )? then ':' (a group) or ')' (the rest of this group)
                    i++;
                    bool on = true, any_after_minus = false, minus = false;
                    bool nfc = fc, ndn = dn, nug = ug;
                    while (true) {
                        int32_t f = cur();
                        if (f < 0 && at_end()) fail();
                        i++;
                        if (f == 'i') { nfc = on; any_after_minus = true; }
                        else if (f == 's') { ndn = on; any_after_minus = true; }
                        else if (f == 'm') { any_after_minus = true; }
                        else if (f == 'U') { nug = on; any_after_minus = true; }
                        else if (f == '-' && !minus) { minus = true; on = false; any_after_minus = false; }
                        else if (f == ':' || f == ')') {
                            if (minus && !any_after_minus) fail();
                            fc = nfc;
                            dn = ndn;
                            ug = nug;
                            if (f == ')') return nullptr;  // no node: the flags hold to the group's end
                            break;
                        } else fail();
                    }
                }
            }
            if (++nest > 1000) fail();
            RP r = alt();
            nest--;
            if (cur() != ')') fail();
            i++;
            fc = fc0;
            dn = dn0;
            ug = ug0;
            return r;
        }
        if (ug) fail();  // any other atom under (?U) carries NonGreedy
        if (c == '^' || c == '$') fail();
        if (c == '.') {
            i++;
            auto r = single(10, 10);
            if (dn) r->set.clear();  // (?s): any rune
            r->neg = true;
            return r;
        }
        if (c == '[') { i++; return klass(); }
        if (c == '\\') {
            int32_t e = cur(1);
            if (e == 'A' || e == 'z' || e == 'b' || e == 'B') fail();
            if (e == 'p' || e == 'P') {
                auto r = std::make_shared<Re>();
                r->k = Re::SET;
                r->set = uclass();
                return r;
            }
            if (e == 'Q') {
                i += 2;
                auto seq = std::make_shared<Re>();
                seq->k = Re::SEQ;
                while (!at_end() && !(cur() == '\\' && cur(1) == 'E')) {
                    if (cur() < 0) fail();
                    seq->kids.push_back(literal(p[i]));
                    i++;
                }
                if (!at_end()) i += 2;
                return seq;
            }
            std::vector<std::pair<int32_t, int32_t>> rs;
            bool ng;
            if (perl(e, &rs, &ng)) {
                i += 2;
                auto r = std::make_shared<Re>();
                r->k = Re::SET;
                r->set = group(rs, ng);
                return r;
            }
            i++;
            int32_t v = esc();
            return literal(v);
        }
        i++;
        return literal(c);
    }
    RP seq() {
        auto s = std::make_shared<Re>();
        s->k = Re::SEQ;
        bool after_rep = false;
        while (!at_end() && cur() != '|' && cur() != ')') {
            int32_t c = cur();
            int lo = -9, hi = -9;
            if (c == '*') { lo = 0; hi = -1; i++; }
            else if (c == '+') { lo = 1; hi = -1; i++; }
            else if (c == '?') { lo = 0; hi = 1; i++; }
            else if (c == '{' && bounds(&lo, &hi)) {
                if (lo > 1000 || hi > 1000 || (hi >= 0 && hi < lo)) fail();
            }
            if (lo != -9) {
                if (s->kids.empty() || after_rep) fail();
                bool lazy = cur() == '?';
                if (lazy) i++;
                lazy = lazy != ug;  // `x*?` under (?U) is greedy again (flags ^= NonGreedy)
                auto r = std::make_shared<Re>();
                r->k = Re::REP;
                r->lo = lo;
                r->hi = hi;
                r->kids = {s->kids.back()};
                s->kids.back() = r;
                after_rep = true;
                if (lazy) fail();
                continue;
            }
            after_rep = false;
            if (RP a = atom()) s->kids.push_back(a);  // null: a (?flags) item
        }
        return s;
    }
    RP alt() {
        auto o = std::make_shared<Re>();
        o->k = Re::OR;
        o->kids.push_back(seq());
        while (cur() == '|') { i++; o->kids.push_back(seq()); }
        return o;
    }
};

// End positions of `r` matched from each position in `from` over runes `t`.
inline std::set<size_t> step(const Re& r, const std::vector<int32_t>& t, const std::set<size_t>& from) {
    std::set<size_t> out;
    switch (r.k) {
    case Re::SET:
        for (size_t s : from)
            if (s < t.size() && r.has(t[s])) out.insert(s + 1);
        return out;
    case Re::SEQ: {
        std::set<size_t> cur = from;
        for (auto& k : r.kids) cur = step(*k, t, cur);
        return cur;
    }
    case Re::OR:
        for (auto& k : r.kids) {
            auto e = step(*k, t, from);
            out.insert(e.begin(), e.end());
        }
        return out;
    case Re::REP: {
        std::set<size_t> cur = from;
        for (int n = 0; n < r.lo; n++) cur = step(*r.kids[0], t, cur);
        out = cur;
        if (r.hi < 0) {  // closure
            std::set<size_t> frontier = cur;
            while (!frontier.empty()) {
                auto e = step(*r.kids[0], t, frontier);
                frontier.clear();
                for (size_t x : e)
                    if (out.insert(x).second) frontier.insert(x);
            }
        } else {
            for (int n = r.lo; n < r.hi && !cur.empty(); n++) {
                cur = step(*r.kids[0], t, cur);
                out.insert(cur.begin(), cur.end());
            }
        }
        return out;
    }
    }
    return out;
}

struct Regexp {
    RP root;
    Status compile(const std::string& pattern) {
        Parse ps;
        ps.p = runes(pattern, false);
        try {
            root = ps.alt();
            if (!ps.at_end()) ps.fail();
        } catch (const Parse::Fail& f) {
            root.reset();
            return f.s;
        }
        return OK;
    }
    bool matches(const std::string& term) const {
        if (!root) return false;
        auto t = runes(term, false);
        auto e = step(*root, t, {0});
        return e.count(t.size()) > 0;
    }
};

// Optimal-string-alignment distance over runes (full table, no cutoff).
inline int osa(const std::string& a, const std::string& b) {
    auto x = runes(a, true), y = runes(b, true);
    const size_t n = x.size(), m = y.size();
    std::vector<std::vector<int>> d(n + 1, std::vector<int>(m + 1));
    for (size_t i = 0; i <= n; i++) d[i][0] = (int)i;
    for (size_t j = 0; j <= m; j++) d[0][j] = (int)j;
    for (size_t i = 1; i <= n; i++)
        for (size_t j = 1; j <= m; j++) {
            int v = std::min(d[i - 1][j] + 1, d[i][j - 1] + 1);
            v = std::min(v, d[i - 1][j - 1] + (x[i - 1] == y[j - 1] ? 0 : 1));
            if (i > 1 && j > 1 && x[i - 1] == y[j - 2] && x[i - 2] == y[j - 1]) v = std::min(v, d[i - 2][j - 2] + 1);
            d[i][j] = v;
        }
    return d[n][m];
}

inline size_t rune_count(const std::string& s) { return runes(s, true).size(); }

}  // namespace oracle_re
