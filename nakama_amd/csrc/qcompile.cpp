// nakama_amd/csrc/qcompile.cpp — query_string -> Clause list (see qcompile.h).
//
// Lexer: vendor/.../query_string/query_string_lex.go (state machine driven by
// runes; a token ends on an unescaped ' ', ':', '^' or '~', the last three
// re-scanned as their own tokens).  Grammar: query_string.y:31-233, whose
// searchBase alternatives are recognised here by a small hand-written LL(2)
// matcher that accepts exactly the LALR(1) language (every conflict in the
// yacc table resolves to the longer production, which is also what the
// matcher tries first).
#include "qcompile.h"
#include "termmatch.h"

#include <cmath>
#include <string_view>

#include "gocompat.h"

namespace nkm {
namespace {

enum TokKind { TK_END, TK_STR, TK_PHRASE, TK_PLUS, TK_MINUS, TK_COLON, TK_BOOST, TK_NUM, TK_GT, TK_LT, TK_EQ, TK_TILDE };
struct Tk { TokKind k; std::string s; };

// One UTF-8 rune as Go's bufio.Reader.ReadRune sees it; invalid input yields
// U+FFFD consuming one byte.
struct Rune { uint32_t cp; std::string_view bytes; };  // bytes: a view into the input (or U+FFFD's encoding)

bool next_rune(std::string_view in, size_t& at, Rune& r) {
    if (at >= in.size()) return false;
    const unsigned char* p = reinterpret_cast<const unsigned char*>(in.data()) + at;
    size_t left = in.size() - at;
    size_t len = p[0] < 0x80 ? 1 : (p[0] >> 5) == 6 ? 2 : (p[0] >> 4) == 14 ? 3 : (p[0] >> 3) == 30 ? 4 : 0;
    bool ok = len != 0 && len <= left;
    uint32_t cp = 0;
    if (ok) {
        cp = len == 1 ? p[0] : len == 2 ? (p[0] & 0x1f) : len == 3 ? (p[0] & 0x0f) : (p[0] & 0x07);
        for (size_t k = 1; k < len && ok; k++) {
            if ((p[k] & 0xc0) != 0x80) ok = false;
            cp = (cp << 6) | (p[k] & 0x3f);
        }
    }
    if (!ok) {
        r.cp = 0xFFFD;
        r.bytes = std::string_view("\xEF\xBF\xBD", 3);
        at += 1;
        return true;
    }
    r.cp = cp;
    r.bytes = std::string_view(in.data() + at, len);
    at += len;
    return true;
}

bool go_is_space(uint32_t c) {  // unicode.IsSpace
    switch (c) {
    case '\t': case '\n': case '\v': case '\f': case '\r': case ' ': case 0x85: case 0xA0: case 0x1680:
    case 0x2028: case 0x2029: case 0x202F: case 0x205F: case 0x3000:
        return true;
    default:
        return c >= 0x2000 && c <= 0x200A;
    }
}
bool is_ascii_digit(uint32_t c) { return c >= '0' && c <= '9'; }

std::string lex_unescape(std::string_view ch) {  // query_string_lex.go:27-34
    static constexpr std::string_view reserved = "+-=&|><!(){}[]^\"~*?:\\/ ";
    if (ch.find_first_of(reserved) != std::string_view::npos) return std::string(ch);
    return "\\" + std::string(ch);
}

class Lexer {
public:
    explicit Lexer(std::string_view in) : in_(in) {}
    bool run(std::vector<Tk>& out);  // false on lexer error (unterminated phrase)

private:
    enum Mode { M_START, M_PHRASE, M_NUM, M_STR, M_BOOST, M_TILDE, M_OP };
    std::string_view in_;
};

bool Lexer::run(std::vector<Tk>& out) {
    size_t at = 0;
    Mode mode = M_START;
    std::string buf;
    bool esc = false, dot = false, eof = false, take = true;
    Rune r{0, {}};
    for (;;) {
        if (take) {
            if (!next_rune(in_, at, r)) { eof = true; r.cp = 0; r.bytes = {}; }
        }
        take = true;
        const bool ender = !esc && (r.cp == ' ' || r.cp == ':' || r.cp == '^' || r.cp == '~');
        switch (mode) {
        case M_START:
            if (eof) return true;
            if (esc) { esc = false; buf += lex_unescape(r.bytes); mode = M_STR; }
            else if (r.cp == '"') mode = M_PHRASE;
            else if (r.cp == '+' || r.cp == '-' || r.cp == ':' || r.cp == '>' || r.cp == '<' || r.cp == '=') {
                buf.assign(r.bytes);
                mode = M_OP;
            } else if (r.cp == '^') mode = M_BOOST;
            else if (r.cp == '~') mode = M_TILDE;
            else if (r.cp == '\\') esc = true;
            else if (is_ascii_digit(r.cp)) { buf += r.bytes; mode = M_NUM; }
            else if (!go_is_space(r.cp)) { buf += r.bytes; mode = M_STR; }
            else { buf.clear(); esc = false; dot = false; }
            break;
        case M_OP: {
            static const char ops[] = "+-:><=";
            static const TokKind kinds[] = {TK_PLUS, TK_MINUS, TK_COLON, TK_GT, TK_LT, TK_EQ};
            for (int k = 0; k < 6; k++)
                if (buf[0] == ops[k]) out.push_back({kinds[k], ""});
            buf.clear(); esc = false; dot = false;
            mode = M_START;
            take = false;  // the current rune is examined again
            break;
        }
        case M_PHRASE:
            if (eof) return false;  // "unterminated quote"
            if (!esc && r.cp == '"') {
                out.push_back({TK_PHRASE, std::move(buf)});
                buf.clear(); esc = false; dot = false;
                mode = M_START;
            } else if (!esc && r.cp == '\\') esc = true;
            else if (esc) { esc = false; buf += lex_unescape(r.bytes); }
            else buf += r.bytes;
            break;
        case M_BOOST:
        case M_TILDE:
            if (eof || (!esc && r.cp == ' ')) {
                out.push_back({mode == M_BOOST ? TK_BOOST : TK_TILDE, buf.empty() ? std::string("1") : std::move(buf)});
                buf.clear(); esc = false; dot = false;
                mode = M_START;
                if (eof) return true;
            } else if (!esc && r.cp == '\\') esc = true;
            else if (esc) { esc = false; buf += lex_unescape(r.bytes); }
            else buf += r.bytes;
            break;
        case M_NUM:
        case M_STR:
            if (eof || ender) {
                out.push_back({mode == M_NUM ? TK_NUM : TK_STR, std::move(buf)});
                buf.clear(); esc = false; dot = false;
                mode = M_START;
                if (eof) return true;
                take = (r.cp == ' ');
            } else if (!esc && r.cp == '\\') esc = true;
            else if (esc) {
                esc = false;
                buf += lex_unescape(r.bytes);
                mode = M_STR;  // an escape never yields a number
            } else if (mode == M_NUM && !dot && r.cp == '.') { dot = true; buf += r.bytes; }
            else if (mode == M_NUM && is_ascii_digit(r.cp)) buf += r.bytes;
            else { buf += r.bytes; mode = M_STR; }
            break;
        }
    }
}

struct Fail { int code; };

class Compiler {
public:
    Compiler(const std::vector<Tk>& t, CompiledQuery* out) : t_(t), out_(out) {}
    void run();

private:
    const std::vector<Tk>& t_;
    CompiledQuery* out_;
    size_t i_ = 0;
    TokKind at(size_t k = 0) const { return i_ + k < t_.size() ? t_[i_ + k].k : TK_END; }
    const std::string& text(size_t k = 0) const { return t_[i_ + k].s; }
    [[noreturn]] void bad() const { throw Fail{CQ_INVALID}; }

    struct Base {
        HostClause c;
        enum { B_MATCH, B_NUMLIT, B_RANGE, B_DATE, B_PHRASE, B_REGEXP, B_FUZZY } kind;
    };
    bool search_error_ = false;
    Base multi_term(const std::string& field, const std::string& pattern, uint8_t kind, int fuzz);
    Base fuzzy_token(const std::string& field, const std::string& s, const std::string& fz);
public:
    bool search_error() const { return search_error_; }
private:
    Base base();
    Base string_token(const std::string& field, const std::string& s);
    Base number_token(const std::string& field, const std::string& s);
    Base range(const std::string& field, bool greater, bool or_equal);
    std::string signed_number();
};

std::string Compiler::signed_number() {  // posOrNegNumber
    if (at() == TK_NUM) return t_[i_++].s;
    if (at() == TK_MINUS && at(1) == TK_NUM) { i_ += 2; return "-" + t_[i_ - 1].s; }
    bad();
}

Compiler::Base Compiler::string_token(const std::string& field, const std::string& s) {
    // queryStringStringToken (query_string_parser.go:171-183)
    if (s.size() >= 2 && s.front() == '/' && s.back() == '/') {
        // RegexpQuery: one leading '^' trimmed (bluge/query.go:1264-1265)
        std::string re = s.substr(1, s.size() - 2);
        if (!re.empty() && re[0] == '^') re.erase(0, 1);
        return multi_term(field, re, TermMatcher::K_REGEXP, 0);
    }
    if (s.find_first_of("*?") != std::string::npos)  // WildcardQuery (query.go:1475-1485)
        return multi_term(field, wildcard_to_regexp(s), TermMatcher::K_REGEXP, 0);
    Base b;
    b.kind = Base::B_MATCH;
    b.c.op = field.empty() ? OP_FALSE : OP_TERM;  // "" -> _all, never indexed
    b.c.field = field;
    b.c.term = s;
    return b;
}

Compiler::Base Compiler::multi_term(const std::string& field, const std::string& pattern, uint8_t kind, int fuzz) {
    Base b;
    b.kind = kind == TermMatcher::K_FUZZY ? Base::B_FUZZY : Base::B_REGEXP;
    b.c.op = field.empty() ? OP_FALSE : OP_TERMSET;
    b.c.field = field;
    b.c.term = pattern;
    b.c.mt_kind = kind;
    b.c.fuzziness = fuzz;
    if (kind == TermMatcher::K_REGEXP) {
        GoRegexp re;
        MtStatus st = re.compile(pattern);
        if (st == MT_UNSUPPORTED) throw Fail{CQ_UNSUPPORTED};
        if (st == MT_SEARCH_ERROR) search_error_ = true;
    }
    return b;
}

// queryStringStringTokenFuzzy (query_string_parser.go:185-196): MatchQuery with
// fuzziness int(ParseFloat(fz)); fuzziness 0 is a plain MatchQuery, outside
// [0, MaxFuzziness=2] the FuzzySearcher fails (search_fuzzy.go:47-53).
Compiler::Base Compiler::fuzzy_token(const std::string& field, const std::string& s, const std::string& fz) {
    double v;
    if (!go_parse_float(fz, &v)) bad();
    if (std::isnan(v) || v <= -1.0 || v >= 3.0) {
        search_error_ = true;
        return multi_term(field, s, TermMatcher::K_FUZZY, 0);
    }
    const int f = (int)v;  // Go int(): truncation toward zero
    if (f == 0) {
        Base b;
        b.kind = Base::B_MATCH;
        b.c.op = field.empty() ? OP_FALSE : OP_TERM;
        b.c.field = field;
        b.c.term = s;
        return b;
    }
    return multi_term(field, s, TermMatcher::K_FUZZY, f);
}

Compiler::Base Compiler::number_token(const std::string& field, const std::string& s) {
    // queryStringNumberToken (query_string_parser.go:198-210): should{Match(s), Range[v,v]}
    double v;
    if (!go_parse_float(s, &v)) bad();
    Base b;
    b.kind = Base::B_NUMLIT;
    b.c.op = field.empty() ? OP_FALSE : OP_NUMLIT;
    b.c.field = field;
    b.c.term = s;
    b.c.lo = b.c.hi = sortable_i64(v);
    return b;
}

Compiler::Base Compiler::range(const std::string& field, bool greater, bool or_equal) {
    Base b;
    b.c.field = field;
    if (at() == TK_PHRASE) {
        // DateRangeQuery via RFC3339 (query_string_parser.go:234-250), validated by
        // DateRangeQuery.Validate (query.go:380-389); scores ConstantScorer(1).
        GoTime tm = go_parse_time(text(), 1);
        i_++;
        if (!tm.ok || tm.zero || !tm.in_range) bad();
        b.kind = Base::B_DATE;
        b.c.op = field.empty() ? OP_FALSE : OP_RANGE;
        int64_t lo = INT64_MIN, hi = INT64_MAX;
        if (greater) { lo = tm.unix_nano; if (!or_equal && lo != INT64_MAX) lo++; }
        else { hi = tm.unix_nano; if (!or_equal && hi != INT64_MIN) hi--; }
        b.c.lo = lo;
        b.c.hi = hi;
        return b;
    }
    std::string num = signed_number();
    double v;
    if (!go_parse_float(num, &v)) bad();
    // NumericRangeInclusiveQuery -> NewNumericRangeSearcher bound adjustment
    // (search_numeric_range.go:26-52)
    b.kind = Base::B_RANGE;
    b.c.op = field.empty() ? OP_FALSE : OP_RANGE;
    int64_t key = sortable_i64(v);
    if (greater) {
        b.c.lo = (std::isinf(v) && v < 0) ? INT64_MIN : key;
        if (!or_equal && b.c.lo != INT64_MAX) b.c.lo++;
        b.c.hi = INT64_MAX;
    } else {
        b.c.lo = INT64_MIN;
        b.c.hi = (std::isinf(v) && v > 0) ? INT64_MAX : key;
        if (!or_equal && b.c.hi != INT64_MIN) b.c.hi--;
    }
    return b;
}

Compiler::Base Compiler::base() {
    if (at() == TK_NUM) { const std::string& s = t_[i_++].s; return number_token("", s); }
    if (at() == TK_PHRASE) { i_++; Base b; b.kind = Base::B_PHRASE; b.c.op = OP_FALSE; return b; }
    if (at() != TK_STR) bad();
    const std::string& first = t_[i_++].s;  // tokens are not modified while compiling: references stay valid
    if (at() == TK_TILDE) { const std::string& fz = t_[i_++].s; return fuzzy_token("", first, fz); }
    if (at() != TK_COLON) return string_token("", first);
    i_++;
    switch (at()) {
    case TK_STR: {
        const std::string& v = t_[i_++].s;
        if (at() == TK_TILDE) { const std::string& fz = t_[i_++].s; return fuzzy_token(first, v, fz); }
        return string_token(first, v);
    }
    case TK_NUM:
    case TK_MINUS: {
        std::string v = signed_number();
        return number_token(first, v);
    }
    case TK_PHRASE: { i_++; Base b; b.kind = Base::B_PHRASE; b.c.op = OP_FALSE; b.c.field = first; return b; }
    case TK_GT:
    case TK_LT: {
        bool greater = at() == TK_GT;
        i_++;
        bool eq = false;
        if (at() == TK_EQ) { eq = true; i_++; }
        return range(first, greater, eq);
    }
    default:
        bad();
    }
}

void Compiler::run() {
    out_->kind = QK_BOOL;
    if (at() == TK_END) bad();
    out_->clauses.reserve(4);
    while (at() != TK_END) {
        Occur occ = OCC_SHOULD;
        if (at() == TK_PLUS) { occ = OCC_MUST; i_++; }
        else if (at() == TK_MINUS) { occ = OCC_MUSTNOT; i_++; }
        Base b = base();
        bool boosted = false;
        double boost = 1.0;
        if (at() == TK_BOOST) {
            if (!go_parse_float(text(), &boost)) bad();
            boosted = true;
            i_++;
        }
        // Score contribution of the clause inside the parsed BooleanQuery, as
        // bluge composes it (CompositeSumScorer: (0 + sum) * boost):
        //  MatchQuery(b):   Bool{should:[Term(b)], boost b} -> (0 + b) * b
        //  number literal:  Bool{should:[Match, Range], boost b} -> (0 + 1) * b
        //  NumericRange(b): ConstantScorer(b) per term      -> b
        //  DateRange:       ConstantScorer(1)                -> 1
        switch (b.kind) {
        case Base::B_MATCH: b.c.score = boosted ? (0.0 + boost) * boost : 1.0; break;
        case Base::B_NUMLIT: b.c.score = boosted ? (0.0 + 1.0) * boost : 1.0; break;
        case Base::B_RANGE: b.c.score = boosted ? boost : 1.0; break;
        case Base::B_DATE: b.c.score = 1.0; break;
        case Base::B_PHRASE: b.c.score = 0.0; break;
        // RegexpQuery(b): term searchers ConstantScorer(b), one term per doc -> b.
        // Fuzzy MatchQuery(b): Bool{should:[Fuzzy(b)], boost b}, term boost
        // b*tb -> (0 + b*tb) * b; the set stores the per-term value, score = b.
        case Base::B_REGEXP:
        case Base::B_FUZZY: b.c.score = boosted ? boost : 1.0; break;
        }
        b.c.occur = occ;
        out_->clauses.push_back(std::move(b.c));
    }
}

}  // namespace

int compile_query(std::string_view q, CompiledQuery* out) {
    out->clauses.clear();
    if (q == "*") { out->kind = QK_MATCHALL; return CQ_OK; }   // match_common.go:246-248
    if (q.empty()) { out->kind = QK_MATCHNONE; return CQ_OK; } // query_string_parser.go:93-95
    std::vector<Tk> toks;
    toks.reserve(16);
    Lexer lx(q);
    if (!lx.run(toks)) return CQ_INVALID;
    try {
        Compiler c(toks, out);
        c.run();
        if (c.search_error()) {  // every search with this query fails
            out->clauses.clear();
            out->kind = QK_MATCHNONE;
        }
    } catch (const Fail& f) {
        out->clauses.clear();
        return f.code;
    }
    return CQ_OK;
}

}  // namespace nkm
