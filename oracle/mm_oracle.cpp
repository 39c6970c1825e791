// oracle/mm_oracle.cpp — CPU restatement of Nakama's matchmaker interval pass.
//
// TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
// product in nakama_amd/: only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it.  It is deliberately written as a direct,
// slow restatement of the reference (quiph/nakama 3.16.0, Go) and shares no
// code with the product: its own query_string lexer/parser, a bluge-shaped
// query tree evaluated per document, a per-row full scan + full sort (the
// same algorithm class as bluge's TopN search), and processDefault /
// processCustom transcribed statement by statement.
//
// Pins: active tickets iterate by (CreatedAt, Ticket);
// RevThreshold's wall-clock cutoff is off; HitNumber = insertion order into the
// index; eligibleIndexesUniq iterates in first-appearance order and the
// CountMultiple trim sorts stably; processCustom candidates follow (T order,
// ascending bitmask); per-ticket session sets iterate in presence order.
//
// Score summation order: bluge sums conjunction constituents ordered by posting
// Count() (search_conjunction.go:40) and disjunction constituents by Count()
// descending (search_disjunction_slice.go:48).  This oracle sums in clause order;
// both orders give identical bits for dyadic boosts (every test/bench input) and
// agree within 1e-15 relative otherwise.
//
// Exports the C ABI of include/nakama_mm.h (backend name "cpu-oracle").

#include "../include/nakama_mm.h"
#include "go_compat.h"
#include "go_regexp.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

using gocompat::f2i;
using std::string;
using std::vector;

namespace oracle {

// ---------------------------------------------------------------------------
// Query tree (vendor/.../bluge/query.go)
// ---------------------------------------------------------------------------
struct Query;
using QP = std::shared_ptr<Query>;

enum QKind { Q_BOOL, Q_TERM, Q_RANGE, Q_MATCHALL, Q_MATCHNONE, Q_PHRASE, Q_UNSUPPORTED, Q_REGEXP, Q_FUZZY };

struct Query {
    QKind kind = Q_MATCHNONE;
    // BooleanQuery (query.go:86-93)
    vector<QP> must, should, mustnot;
    bool has_boost = false;
    double boost = 1.0;
    int min_should = 0;
    // TermQuery / NumericRangeQuery
    string field;
    string term;
    int64_t lo = 0, hi = 0;      // NumericRangeSearcher bounds after ±1 adjustment (search_numeric_range.go:26-52)
    double const_score = 1.0;    // ConstantScorer value of the range's term searchers
    bool is_date = false;        // DateRangeQuery: ConstantScorer(1) whatever the boost
    // RegexpQuery / WildcardQuery (term = pattern) and FuzzyQuery (term, fuzziness)
    std::shared_ptr<oracle_re::Regexp> re;
    int fuzziness = 0;
    uint32_t fid = 0;  // field_id(field), set when the query is parsed (bind_fields)
};

static double boost_value(const Query& q) { return q.has_boost ? q.boost : 1.0; }

// Field names interned to small ids (process-wide: handles share it), so a
// document's fields are a short vector searched by id — the per-document
// evaluation of every search reads no string map.
static uint32_t field_id(const string& name) {
    static std::mutex mu;
    static std::unordered_map<string, uint32_t> ids;
    std::lock_guard<std::mutex> lk(mu);
    auto it = ids.find(name);
    if (it != ids.end()) return it->second;
    const uint32_t id = (uint32_t)ids.size();
    ids.emplace(name, id);
    return id;
}

// Field values of one indexed document (MapMatchmakerIndex, matchmaker.go:1026-1040).
struct FieldVal {
    int kind = 0;  // 1 keyword, 2 numeric term (Float64ToInt64 or raw UnixNano for datetime)
    string kw;
    int64_t num = 0;
};
struct Doc {
    vector<std::pair<uint32_t, FieldVal>> f;  // by field id, each field once
    const FieldVal* find(uint32_t fid) const {
        for (auto& kv : f)
            if (kv.first == fid) return &kv.second;
        return nullptr;
    }
    void set(const string& name, FieldVal v) {
        const uint32_t id = field_id(name);
        for (auto& kv : f)
            if (kv.first == id) { kv.second = std::move(v); return; }
        f.push_back({id, std::move(v)});
    }
};

struct EvalRes { bool match; double score; };

// Per-document evaluation of the searcher tree built by Query.Searcher.
static EvalRes eval(const Query& q, const Doc& d) {
    switch (q.kind) {
    case Q_MATCHALL:  // MatchAllSearcher with ConstantScorer(1) (query.go:709-711)
        return {true, 1.0};
    case Q_MATCHNONE:
    case Q_PHRASE:    // keyword/numeric fields carry no locations: phrase never matches
    case Q_UNSUPPORTED:
        return {false, 0.0};
    case Q_TERM: {    // TermSearcher + ConstantScorer(boost) (search_term.go, match_common.go:259)
        const FieldVal* it = d.find(q.fid);
        if (it && it->kind == 1 && it->kw == q.term) return {true, boost_value(q)};
        return {false, 0.0};
    }
    case Q_REGEXP: {  // multi-term disjunction of TermSearchers(boost), one term per keyword doc
        const FieldVal* it = d.find(q.fid);
        if (it && it->kind == 1 && q.re->matches(it->kw)) return {true, boost_value(q)};
        return {false, 0.0};
    }
    case Q_FUZZY: {   // FuzzySearcher: TermSearcher(boost * boostFromDistance) (search_fuzzy.go:99-126)
        const FieldVal* it = d.find(q.fid);
        if (!it || it->kind != 1) return {false, 0.0};
        const string& t = it->kw;
        int dist = oracle_re::osa(q.term, t);
        if (dist > q.fuzziness) return {false, 0.0};
        double tb = 1.0;
        if (t != q.term) {
            double ml = (double)std::min(oracle_re::rune_count(q.term), oracle_re::rune_count(t));
            tb = 1.0 - ((double)dist / ml);
        }
        return {true, boost_value(q) * tb};
    }
    case Q_RANGE: {   // NumericRangeSearcher: disjoint prefix-coded terms, one hit per doc
        const FieldVal* it = d.find(q.fid);
        if (it && it->kind == 2 && it->num >= q.lo && it->num <= q.hi)
            return {true, q.const_score};
        return {false, 0.0};
    }
    case Q_BOOL: {    // BooleanQuery.Searcher (query.go:198-229) + BooleanSearcher (search_boolean.go)
        bool has_must = !q.must.empty(), has_should = !q.should.empty(), has_not = !q.mustnot.empty();
        if (!has_must && !has_should && !has_not) return {false, 0.0};
        for (auto& n : q.mustnot)
            if (eval(*n, d).match) return {false, 0.0};
        double must_score = 0.0;
        bool must_present = has_must;
        if (has_must) {
            for (auto& m : q.must) {  // ConjunctionSearcher + CompositeSumScorer
                EvalRes r = eval(*m, d);
                if (!r.match) return {false, 0.0};
                must_score += r.score;
            }
        } else if (!has_should) {
            must_present = true;      // only mustNots: MatchAll(1)
            must_score = 1.0;
        }
        double should_score = 0.0;
        int nmatched = 0;
        for (auto& s : q.should) {    // DisjunctionSliceSearcher(min) + CompositeSumScorer
            EvalRes r = eval(*s, d);
            if (r.match) { should_score += r.score; nmatched++; }
        }
        bool should_ok = nmatched > 0 && nmatched >= q.min_should;
        double b = boost_value(q);
        if (must_present) {
            if (has_should && should_ok) return {true, (must_score + should_score) * b};
            if (!has_should || q.min_should == 0) return {true, must_score * b};
            return {false, 0.0};
        }
        if (should_ok) return {true, should_score * b};
        return {false, 0.0};
    }
    }
    return {false, 0.0};
}

// ---------------------------------------------------------------------------
// query_string lexer (vendor/.../query_string/query_string_lex.go)
// ---------------------------------------------------------------------------
enum Tok { T_EOF = 0, T_STRING, T_PHRASE, T_PLUS, T_MINUS, T_COLON, T_BOOST, T_NUMBER, T_GREATER, T_LESS, T_EQUAL, T_TILDE };
struct Token { Tok t; string s; };

struct LexError {};

static const char* kReserved = "+-=&|><!(){}[]^\"~*?:\\/ ";
static string unescape_one(const string& c) {  // query_string_lex.go:27-34
    if (c.find_first_of(kReserved) != string::npos) return c;
    return "\\" + c;
}

// Decodes one UTF-8 rune (bufio.Reader.ReadRune semantics: invalid -> U+FFFD, 1 byte).
static bool read_rune(const string& s, size_t& p, string& out, uint32_t& cp) {
    if (p >= s.size()) return false;
    unsigned char c = (unsigned char)s[p];
    size_t n = 1;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6) { n = 2; cp = c & 0x1f; }
    else if ((c >> 4) == 14) { n = 3; cp = c & 0x0f; }
    else if ((c >> 3) == 30) { n = 4; cp = c & 0x07; }
    else { cp = 0xFFFD; out = "\xEF\xBF\xBD"; p += 1; return true; }
    if (p + n > s.size()) { cp = 0xFFFD; out = "\xEF\xBF\xBD"; p += 1; return true; }
    for (size_t k = 1; k < n; k++) {
        unsigned char cc = (unsigned char)s[p + k];
        if ((cc >> 6) != 2) { cp = 0xFFFD; out = "\xEF\xBF\xBD"; p += 1; return true; }
        cp = (cp << 6) | (cc & 0x3f);
    }
    out = s.substr(p, n);
    p += n;
    return true;
}

static bool rune_is_digit(uint32_t cp) { return cp >= '0' && cp <= '9'; }  // ASCII digits (sufficient for tests)
static bool rune_is_space(uint32_t cp) {
    return cp == ' ' || cp == '\t' || cp == '\n' || cp == '\v' || cp == '\f' || cp == '\r' || cp == 0x85 || cp == 0xA0;
}

static vector<Token> lex(const string& in) {
    enum St { START, PHRASE, NUMSTR, STR, BOOST, TILDE, SINGLE };
    vector<Token> out;
    St st = START;
    string buf;
    bool in_escape = false, seen_dot = false;
    size_t pos = 0;
    string rune;
    uint32_t cp = 0;
    bool eof = false;
    bool consumed = true;
    auto reset = [&]() { buf.clear(); in_escape = false; seen_dot = false; };
    for (;;) {
        if (consumed) {
            if (!read_rune(in, pos, rune, cp)) { eof = true; rune.clear(); cp = 0; }
        }
        switch (st) {
        case START:
            if (eof) return out;
            if (in_escape) { in_escape = false; buf += unescape_one(rune); st = STR; consumed = true; break; }
            if (cp == '"') { st = PHRASE; consumed = true; break; }
            if (cp == '+' || cp == '-' || cp == ':' || cp == '>' || cp == '<' || cp == '=') {
                buf += rune; st = SINGLE; consumed = true; break;
            }
            if (cp == '^') { st = BOOST; consumed = true; break; }
            if (cp == '~') { st = TILDE; consumed = true; break; }
            if (cp == '\\') { in_escape = true; st = START; consumed = true; break; }
            if (rune_is_digit(cp)) { buf += rune; st = NUMSTR; consumed = true; break; }
            if (!rune_is_space(cp)) { buf += rune; st = STR; consumed = true; break; }
            reset();
            st = START;
            consumed = true;
            break;
        case PHRASE:
            if (eof) throw LexError{};  // "unterminated quote"
            if (!in_escape && cp == '"') { out.push_back({T_PHRASE, buf}); reset(); st = START; consumed = true; break; }
            if (!in_escape && cp == '\\') in_escape = true;
            else if (in_escape) { in_escape = false; buf += unescape_one(rune); }
            else buf += rune;
            consumed = true;
            break;
        case SINGLE: {
            Tok t = T_EOF;
            if (buf == "+") t = T_PLUS;
            else if (buf == "-") t = T_MINUS;
            else if (buf == ":") t = T_COLON;
            else if (buf == ">") t = T_GREATER;
            else if (buf == "<") t = T_LESS;
            else if (buf == "=") t = T_EQUAL;
            out.push_back({t, ""});
            reset();
            st = START;
            consumed = false;  // singleCharOpState does not consume
            break;
        }
        case BOOST:
        case TILDE:
            if (eof || (!in_escape && cp == ' ')) {
                if (buf.empty()) buf = "1";
                out.push_back({st == BOOST ? T_BOOST : T_TILDE, buf});
                reset();
                st = START;
                consumed = true;
                if (eof) return out;
                break;
            }
            if (!in_escape && cp == '\\') in_escape = true;
            else if (in_escape) { in_escape = false; buf += unescape_one(rune); }
            else buf += rune;
            consumed = true;
            break;
        case NUMSTR:
            if (eof || (!in_escape && (cp == ' ' || cp == ':' || cp == '^' || cp == '~'))) {
                out.push_back({T_NUMBER, buf});
                reset();
                st = START;
                consumed = !( !eof && (cp == ':' || cp == '^' || cp == '~'));
                if (eof) return out;
                break;
            }
            if (!in_escape && cp == '\\') { in_escape = true; consumed = true; break; }
            if (in_escape) { in_escape = false; buf += unescape_one(rune); st = STR; consumed = true; break; }
            if (!seen_dot && cp == '.') { seen_dot = true; buf += rune; consumed = true; break; }
            if (rune_is_digit(cp)) { buf += rune; consumed = true; break; }
            buf += rune;
            st = STR;
            consumed = true;
            break;
        case STR:
            if (eof || (!in_escape && (cp == ' ' || cp == ':' || cp == '^' || cp == '~'))) {
                out.push_back({T_STRING, buf});
                reset();
                st = START;
                consumed = !(!eof && (cp == ':' || cp == '^' || cp == '~'));
                if (eof) return out;
                break;
            }
            if (!in_escape && cp == '\\') in_escape = true;
            else if (in_escape) { in_escape = false; buf += unescape_one(rune); }
            else buf += rune;
            consumed = true;
            break;
        }
    }
}

// ---------------------------------------------------------------------------
// query_string grammar (query_string.y:31-233) -> bluge queries
// (query_string_parser.go:171-280)
// ---------------------------------------------------------------------------
struct ParseError {};
struct Unsupported {};

static QP make_term(const string& field, const string& term) {
    auto q = std::make_shared<Query>();
    q->kind = Q_TERM;
    q->field = field;
    q->term = term;
    return q;
}
// MatchQuery with the keyword analyzer (query.go:950-1005): one token = whole
// string; Bool{should:[Term(boost b)], minShould 1, boost b}.
static QP make_match(const string& field, const string& str) {
    auto t = make_term(field.empty() ? "_all" : field, str);
    auto b = std::make_shared<Query>();
    b->kind = Q_BOOL;
    b->should.push_back(t);
    b->min_should = 1;
    return b;
}
static void set_match_boost(QP& m, double b) {  // MatchQuery.SetBoost: term and wrapper
    m->has_boost = true;
    m->boost = b;
    m->should[0]->has_boost = true;
    m->should[0]->boost = b;
}
// NumericRangeQuery.Searcher -> NewNumericRangeSearcher (search_numeric_range.go:26-52)
static QP make_range(const string& field, double mn, double mx, bool incl_min, bool incl_max) {
    auto q = std::make_shared<Query>();
    q->kind = Q_RANGE;
    q->field = field.empty() ? "_all" : field;
    int64_t lo = std::isinf(mn) && mn < 0 ? INT64_MIN : f2i(mn);
    int64_t hi = std::isinf(mx) && mx > 0 ? INT64_MAX : f2i(mx);
    if (!incl_min && lo != INT64_MAX) lo++;
    if (!incl_max && hi != INT64_MIN) hi--;
    q->lo = lo;
    q->hi = hi;
    q->const_score = 1.0;
    return q;
}
static QP make_number(const string& field, const string& str) {  // queryStringNumberToken
    double v;
    if (!gocompat::parse_float(str, &v)) throw ParseError{};
    auto b = std::make_shared<Query>();
    b->kind = Q_BOOL;
    b->should.push_back(make_match(field, str));
    b->should.push_back(make_range(field, v, v, true, true));
    return b;
}

struct Parser {
    vector<Token> toks;
    size_t p = 0;
    QP top;
    Tok peek(size_t k = 0) const { return p + k < toks.size() ? toks[p + k].t : T_EOF; }
    const Token& take() { if (p >= toks.size()) throw ParseError{}; return toks[p++]; }

    string pos_or_neg() {
        if (peek() == T_NUMBER) return take().s;
        if (peek() == T_MINUS && peek(1) == T_NUMBER) { take(); return "-" + take().s; }
        throw ParseError{};
    }
    // date range endpoint (query_string_parser.go:234-250, DateRangeQuery.Validate query.go:380-389)
    QP date_range(const string& field, const string& phrase, bool greater, bool or_equal) {
        gocompat::ParsedTime t = gocompat::go_time_parse(phrase, 1);  // dateFormat = time.RFC3339
        if (!t.ok) throw ParseError{};
        // DateRangeQuery with one endpoint zero-valued; a zero time parses as
        // "unbounded" on both sides -> Validate error
        if (t.is_zero) throw ParseError{};
        if (t.overflow) throw ParseError{};   // isDatetimeCompatible
        auto q = std::make_shared<Query>();
        q->kind = Q_RANGE;
        q->field = field.empty() ? "_all" : field;
        int64_t lo = INT64_MIN, hi = INT64_MAX;
        bool incl_min = true, incl_max = true;
        if (greater) { lo = t.unix_nano; incl_min = or_equal; }
        else { hi = t.unix_nano; incl_max = or_equal; }
        // min/max pass through Int64ToFloat64 -> Float64ToInt64 (identity), then ±1
        if (!incl_min && lo != INT64_MAX) lo++;
        if (!incl_max && hi != INT64_MIN) hi--;
        q->lo = lo;
        q->hi = hi;
        q->const_score = 1.0;  // DateRangeQuery.Searcher uses ConstantScorer(1) (query.go:349-351)
        q->is_date = true;
        return q;
    }
    QP search_base() {
        Tok t0 = peek();
        if (t0 == T_NUMBER) {
            return make_number("", take().s);
        }
        if (t0 == T_PHRASE) { take(); auto q = std::make_shared<Query>(); q->kind = Q_PHRASE; return q; }
        if (t0 != T_STRING) throw ParseError{};
        string s1 = take().s;
        if (peek() == T_TILDE) return fuzzy_token("", s1, take().s);
        if (peek() != T_COLON) {  // unfielded string -> _all
            return string_token("", s1);
        }
        take();  // ':'
        Tok t2 = peek();
        if (t2 == T_STRING) {
            string s3 = take().s;
            if (peek() == T_TILDE) return fuzzy_token(s1, s3, take().s);
            return string_token(s1, s3);
        }
        if (t2 == T_NUMBER || t2 == T_MINUS) {
            string n = pos_or_neg();
            return make_number(s1, n);
        }
        if (t2 == T_PHRASE) { take(); auto q = std::make_shared<Query>(); q->kind = Q_PHRASE; return q; }
        if (t2 == T_GREATER || t2 == T_LESS) {
            take();
            bool greater = t2 == T_GREATER;
            bool or_equal = false;
            if (peek() == T_EQUAL) { take(); or_equal = true; }
            if (peek() == T_PHRASE) return date_range(s1, take().s, greater, or_equal);
            string n = pos_or_neg();
            double v;
            if (!gocompat::parse_float(n, &v)) throw ParseError{};
            if (greater) return make_range(s1, v, INFINITY, or_equal, true);
            return make_range(s1, -INFINITY, v, true, or_equal);
        }
        throw ParseError{};
    }
    bool search_error = false;  // accepted by the parser, fails at search time
    QP regexp(const string& field, const string& pattern) {
        auto q = std::make_shared<Query>();
        q->kind = Q_REGEXP;
        q->field = field.empty() ? "_all" : field;
        q->term = pattern;
        q->re = std::make_shared<oracle_re::Regexp>();
        oracle_re::Status st = q->re->compile(pattern);
        if (st == oracle_re::UNSUPPORTED) throw Unsupported{};
        if (st == oracle_re::SEARCH_ERROR) search_error = true;
        return q;
    }
    QP string_token(const string& field, const string& s) {  // queryStringStringToken (query_string_parser.go:171-183)
        if (s.size() >= 2 && s.front() == '/' && s.back() == '/') {
            string re = s.substr(1, s.size() - 2);
            if (re.rfind("^", 0) == 0) re = re.substr(1);  // strings.TrimPrefix(regexp, "^") (query.go:1264-1265)
            return regexp(field, re);
        }
        if (s.find_first_of("*?") != string::npos) {     // WildcardQuery: wildcardRegexpReplacer (query.go:1455-1485)
            string re;
            for (char c : s) {
                if (string("+()^$.{}[]|\\").find(c) != string::npos) { re += '\\'; re += c; }
                else if (c == '*') re += ".*";
                else if (c == '?') re += ".";
                else re += c;
            }
            return regexp(field, re);
        }
        return make_match(field, s);
    }
    // queryStringStringTokenFuzzy (query_string_parser.go:185-196): MatchQuery
    // with fuzziness int(ParseFloat(fz)) -> Bool{should:[Fuzzy]} (query.go:966-975)
    QP fuzzy_token(const string& field, const string& s, const string& fz) {
        double v;
        if (!gocompat::parse_float(fz, &v)) throw ParseError{};
        long f;
        if (std::isnan(v) || v >= 3.0 || v <= -1.0) { search_error = true; f = 3; }  // > MaxFuzziness or negative
        else f = (long)v;
        QP m = make_match(field, s);
        if (f == 0) return m;
        m->should[0]->kind = Q_FUZZY;
        m->should[0]->fuzziness = (int)f;
        return m;
    }
    QP parse() {
        top = std::make_shared<Query>();
        top->kind = Q_BOOL;
        if (peek() == T_EOF) throw ParseError{};  // searchParts needs one part
        while (peek() != T_EOF) {
            int prefix = 0;  // 0 should, 1 must, 2 mustnot
            if (peek() == T_PLUS) { take(); prefix = 1; }
            else if (peek() == T_MINUS) { take(); prefix = 2; }
            QP q = search_base();
            if (peek() == T_BOOST) {
                double b;
                if (!gocompat::parse_float(take().s, &b)) throw ParseError{};
                // queryStringSetBoost (query_string_parser.go:262-280)
                if (q->kind == Q_BOOL && q->min_should == 1 && q->should.size() == 1 &&
                    (q->should[0]->kind == Q_TERM || q->should[0]->kind == Q_FUZZY) &&
                    q->must.empty() && q->mustnot.empty()) {
                    set_match_boost(q, b);               // MatchQuery
                } else if (q->kind == Q_RANGE) {
                    // NumericRangeQuery: ConstantScorer(boost) (query.go:1146-1156)
                    if (!q->is_date) q->const_score = b;
                    q->has_boost = true;
                    q->boost = b;
                } else {
                    q->has_boost = true;                 // number token BooleanQuery / phrase
                    q->boost = b;
                }
            }
            if (prefix == 0) top->should.push_back(q);
            else if (prefix == 1) top->must.push_back(q);
            else top->mustnot.push_back(q);
        }
        return top;
    }
};

static void bind_fields(Query& q) {
    q.fid = field_id(q.field);
    for (auto* v : {&q.must, &q.should, &q.mustnot})
        for (auto& c : *v) bind_fields(*c);
}

// ParseQueryString (server/match_common.go:244-251 + query_string_parser.go:92-103).
// Returns 0 ok, MM_ERR_QUERY_INVALID, MM_ERR_UNSUPPORTED.
static int parse_query(const string& query, QP* out) {
    if (query == "*") {
        auto q = std::make_shared<Query>();
        q->kind = Q_MATCHALL;
        *out = q;
        return 0;
    }
    if (query.empty()) {
        auto q = std::make_shared<Query>();
        q->kind = Q_MATCHNONE;
        *out = q;
        return 0;
    }
    try {
        Parser ps;
        ps.toks = lex(query);
        QP q = ps.parse();
        if (ps.search_error) {  // every search fails: processDefault `continue`s (matchmaker_process.go:97-101)
            q = std::make_shared<Query>();
            q->kind = Q_MATCHNONE;
        }
        bind_fields(*q);
        *out = q;
        return 0;
    } catch (const Unsupported&) {
        return MM_ERR_UNSUPPORTED;
    } catch (const ParseError&) {
        return MM_ERR_QUERY_INVALID;
    } catch (const LexError&) {
        return MM_ERR_QUERY_INVALID;
    }
}

// ---------------------------------------------------------------------------
// Matchmaker state (server/matchmaker.go)
// ---------------------------------------------------------------------------
struct Presence { string user_id, session_id, username, node; };

struct Index {  // MatchmakerIndex (matchmaker.go:88-108)
    string ticket;
    int min_count = 0, max_count = 0, count_multiple = 1, count = 0, intervals = 0;
    string party_id, query, session_id, node;
    int64_t created_at = 0;
    vector<string> session_ids;        // SessionIDs set, presence order
    std::unordered_set<string> session_set;
    vector<std::pair<string, string>> sprops;
    vector<std::pair<string, double>> nprops;
    QP parsed;
    vector<Presence> entries;
    Doc doc;
    uint64_t selected_in = 0;  // processDefault's `selected` set: the pass (process_default's serial) that selected it
};
using IP = std::shared_ptr<Index>;

struct Entry { IP idx; int pi; };  // MatchmakerEntry = (ticket, presence)

struct BlugeDoc { IP idx; bool alive; uint64_t docnum; };

struct Matchmaker {
    std::mutex mu;
    mm_config cfg;
    string node;
    bool active = true, stopped = false;
    // mm_set_delivery: the checker delivers synchronously, in pass order (the
    // contract's observable part; the product's delivery thread pipelines it)
    mm_deliver_fn deliver_fn = nullptr;
    void* deliver_ctx = nullptr;
    int64_t deliver_seq = 0;
    string last_error;
    uint64_t next_docnum = 0;
    vector<BlugeDoc> bluge;                               // the in-memory index, insertion order
    std::unordered_map<string, size_t> bluge_pos;         // ticket -> position of live doc
    std::unordered_map<string, IP> indexes;               // m.indexes
    std::unordered_map<string, IP> active_indexes;        // m.activeIndexes
    std::unordered_map<string, std::map<string, bool>> rev_cache;  // m.revCache
    std::unordered_map<string, std::set<string>> session_tickets, party_tickets;
    // open processCustom pass
    bool custom_open = false;
    vector<string> custom_expired;
    // drained removals (mm_drain_removed): ids that left m.indexes
    bool track_removed = false;
    vector<string> removed;
    void note_removed(const string& t) { if (track_removed) removed.push_back(t); }
    // test hook: between processDefault/processCustom and the post-pass lock
    void (*pass_hook)(void*) = nullptr;
    void* pass_hook_ctx = nullptr;
    // output storage
    vector<string> out_strings;
    // debug hit strings / extract keep-alive
    vector<string> dbg;
    vector<IP> extract_keep;
};

static void bluge_delete(Matchmaker& m, const string& ticket) {
    auto it = m.bluge_pos.find(ticket);
    if (it == m.bluge_pos.end()) return;
    m.bluge[it->second].alive = false;
    m.bluge_pos.erase(it);
}
static void bluge_update(Matchmaker& m, const IP& idx) {  // Writer.Update / Batch.Insert
    bluge_delete(m, idx->ticket);
    m.bluge.push_back({idx, true, m.next_docnum++});
    m.bluge_pos[idx->ticket] = m.bluge.size() - 1;
}

// MapMatchmakerIndex + BlugeWalkDocument/blugeProcessProperty (matchmaker.go:1026-1040,
// match_common.go:78-212).  Numeric props win on key clash (matchmaker.go:460-466).
static void build_doc(Index& ix) {
    Doc d;
    d.set("ticket", FieldVal{1, ix.ticket, 0});
    d.set("min_count", FieldVal{2, "", f2i((double)ix.min_count)});
    d.set("max_count", FieldVal{2, "", f2i((double)ix.max_count)});
    d.set("party_id", FieldVal{1, ix.party_id, 0});
    d.set("created_at", FieldVal{2, "", f2i((double)ix.created_at)});
    std::map<string, FieldVal> props;
    for (auto& kv : ix.sprops) {
        int64_t ns;
        if (gocompat::bluge_parse_datetime(kv.second, &ns)) props[kv.first] = FieldVal{2, "", ns};
        else props[kv.first] = FieldVal{1, kv.second, 0};
    }
    for (auto& kv : ix.nprops) props[kv.first] = FieldVal{2, "", f2i(kv.second)};
    for (auto& kv : props) d.set("properties." + kv.first, kv.second);
    ix.doc = std::move(d);
}

// Matchmaker search of processDefault/processCustom (matchmaker_process.go:65-90).
static bool eval_search(const Index& T, const Index& H, double* score) {
    EvalRes p = eval(*T.parsed, H.doc);
    if (!p.match) return false;
    if (!(H.min_count >= T.min_count)) return false;   // min_count range [T.Min, +Inf]
    if (!(H.max_count <= T.max_count)) return false;   // max_count range [-Inf, T.Max]
    if (!T.party_id.empty() && H.party_id == T.party_id) return false;  // mustNot party_id
    // top-level BooleanQuery: must conjunction [P, minRange, maxRange], boost 1
    *score = p.score + 1.0 + 1.0;
    return true;
}

struct Hit { IP idx; double score; int64_t ckey; uint64_t docnum; };

// TopN search sorted by ["-_score", "created_at"] (search/sort.go:53-76), all hits.
static vector<Hit> search_hits(Matchmaker& m, const Index& T) {
    vector<Hit> hits;
    for (auto& bd : m.bluge) {
        if (!bd.alive) continue;
        double s;
        if (eval_search(T, *bd.idx, &s)) hits.push_back({bd.idx, s, f2i((double)bd.idx->created_at), bd.docnum});
    }
    std::sort(hits.begin(), hits.end(), [](const Hit& a, const Hit& b) {
        int64_t sa = f2i(a.score), sb = f2i(b.score);
        if (sa != sb) return sa > sb;
        if (a.ckey != b.ckey) return a.ckey < b.ckey;
        return a.docnum < b.docnum;
    });
    return hits;
}

// The same hits for processDefault's walk, which reads them in order and
// usually stops after a few: the hits that are not the searching ticket and
// not selected earlier in the pass (matchmaker_process.go:112-126) are kept
// as a heap under the same total order (score desc, created_at asc, doc
// order) and popped one at a time — the sequence std::sort would give, at
// O(n + k log n) for k hits read instead of O(n log n) (a 62,500-ticket C4
// pool pass: 31k searches over 62.5k documents each).
struct LazyHit { Index* idx; int64_t skey; int64_t ckey; uint64_t docnum; };
static bool lazy_before(const LazyHit& a, const LazyHit& b) {
    if (a.skey != b.skey) return a.skey > b.skey;
    if (a.ckey != b.ckey) return a.ckey < b.ckey;
    return a.docnum < b.docnum;
}
struct LazyHits {
    vector<LazyHit> h;
    size_t n = 0, taken = 0;
    static bool heap_less(const LazyHit& a, const LazyHit& b) { return lazy_before(b, a); }
    void build() {
        n = h.size();
        std::make_heap(h.begin(), h.end(), heap_less);
    }
    size_t size() const { return n; }
    // the next hit in sorted order (call at most size() times)
    const LazyHit& next() {
        std::pop_heap(h.begin(), h.begin() + (n - taken), heap_less);
        taken++;
        return h[n - taken];
    }
};
static void search_hits_walk(Matchmaker& m, const Index& T, uint64_t pass, LazyHits& out) {
    out.h.clear();
    out.taken = 0;
    for (auto& bd : m.bluge) {
        if (!bd.alive) continue;
        Index* H = bd.idx.get();
        if (H == &T || H->selected_in == pass) continue;  // self: the same MatchmakerIndex
        double s;
        if (eval_search(T, *H, &s)) out.h.push_back({H, f2i(s), f2i((double)H->created_at), bd.docnum});
    }
    out.build();
}

// validateMatch (matchmaker.go:1042-1068): to's document must match from's parsed query.
static bool validate_match(Matchmaker& m, const Index& from, const string& to_ticket) {
    auto c = m.rev_cache.find(from.ticket);
    if (c == m.rev_cache.end()) return false;
    auto r = c->second.find(to_ticket);
    if (r != c->second.end()) return r->second;
    bool valid = false;
    auto bp = m.bluge_pos.find(to_ticket);
    if (bp != m.bluge_pos.end()) valid = eval(*from.parsed, m.bluge[bp->second].idx->doc).match;
    c->second[to_ticket] = valid;
    return valid;
}

// groupIndexes (matchmaker.go:132-167), Go int64 wrapping arithmetic.
struct IGroup { vector<IP> indexes; int64_t avg; };
static vector<IGroup> group_indexes(const vector<IP>& indexes, size_t from, int required) {
    if (from >= indexes.size() || required <= 0) return {};
    const IP& current = indexes[from];
    if (current->count > required) return group_indexes(indexes, from + 1, required);
    vector<IGroup> results;
    if (current->count == required) {
        results.push_back({{current}, current->created_at});
    } else if (current->count < required) {
        auto fill = group_indexes(indexes, from + 1, required - current->count);
        for (auto& fr : fill) {
            int64_t n = (int64_t)fr.indexes.size();
            uint64_t num = (uint64_t)fr.avg * (uint64_t)n + (uint64_t)current->created_at;  // wraps like Go
            fr.avg = (int64_t)num / (n + 1);
            fr.indexes.push_back(current);
            results.push_back(std::move(fr));
        }
    }
    auto others = group_indexes(indexes, from + 1, required);
    for (auto& o : others) results.push_back(std::move(o));
    return results;
}

// m.revThresholdFn (matchmaker.go:244-248): a timer of IntervalSec*RevThreshold
// seconds, created at the start of an active pass when RevPrecision is on and
// RevThreshold > 0.  Pin: it counts as fired from the first row examined after
// the duration elapsed (zero duration: from the first row).
struct RevThresholdTimer {
    bool armed;
    double limit_s;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit RevThresholdTimer(const Matchmaker& m)
        : armed(m.active && m.cfg.rev_precision && m.cfg.rev_threshold > 0),
          limit_s((double)m.cfg.interval_sec * (double)m.cfg.rev_threshold) {}
    bool fired() const {
        return armed && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >= limit_s;
    }
};

static vector<IP> active_order(Matchmaker& m) {  // pin: (CreatedAt, Ticket)
    vector<IP> v;
    v.reserve(m.active_indexes.size());
    for (auto& kv : m.active_indexes) v.push_back(kv.second);
    std::sort(v.begin(), v.end(), [](const IP& a, const IP& b) {
        if (a->created_at != b->created_at) return a->created_at < b->created_at;
        return a->ticket < b->ticket;
    });
    return v;
}

// processDefault (matchmaker_process.go:27-334)
static void process_default(Matchmaker& m, const vector<IP>& order,
                            const std::unordered_map<string, IP>& indexes_copy,
                            vector<vector<Entry>>& matched, vector<string>& expired, int64_t* pair_evals) {
    // `selected` (a set of ticket ids): Index::selected_in == this pass
    static std::atomic<uint64_t> pass_serial{0};
    const uint64_t pass = ++pass_serial;
    auto selected = [&](const Index* ix) { return ix->selected_in == pass; };
    const int max_intervals = m.cfg.max_intervals;
    // RevThreshold timer (matchmaker.go:244-248, matchmaker_process.go:31-46)
    RevThresholdTimer timer(m);
    bool threshold = false;
    LazyHits h2;
    for (const IP& ai : order) {
        if (!threshold && timer.fired()) threshold = true;
        const bool rev = m.cfg.rev_precision != 0 && !threshold;  // :139, :178
        const string& ticket = ai->ticket;
        if (selected(ai.get())) continue;
        ai->intervals++;
        bool last_interval = ai->intervals >= max_intervals || ai->min_count == ai->max_count;
        if (last_interval) expired.push_back(ticket);
        if (!m.active) continue;

        // the hits, minus self and the already-selected (matchmaker_process.go:112-126)
        search_hits_walk(m, *ai, pass, h2);
        *pair_evals += (int64_t)m.bluge_pos.size();
        vector<vector<Entry>> combos;
        int last_hit_counter = (int)h2.size() - 1;
        for (int hit_counter = 0; hit_counter < (int)h2.size(); hit_counter++) {
            const string& hid = h2.next().idx->ticket;
            auto hi_it = indexes_copy.find(hid);
            if (hi_it == indexes_copy.end()) continue;  // missing index
            const IP& hit = hi_it->second;
            if (rev) {
                if (!validate_match(m, *hit, ticket)) continue;
            }
            if (ai->max_count < hit->max_count && hit->intervals <= max_intervals) continue;  // dead branch
            bool session_conflict = false;
            for (auto& s : ai->session_ids)
                if (hit->session_set.count(s)) { session_conflict = true; break; }
            if (session_conflict) continue;

            int found_idx = -1;
            for (size_t ci = 0; ci < combos.size(); ci++) {
                auto& combo = combos[ci];
                if ((int)combo.size() + (int)hit->entries.size() + ai->count <= ai->max_count) {
                    bool mutual_conflict = false;
                    for (auto& e : combo) {
                        // A nil'd slot of a trimmed combo (below) would be a nil
                        // dereference in Go here; unreachable: such a combo formed
                        // at l == MaxCount and has no room at :170 (or it was
                        // trimmed at the row's last hit).
                        if (!e.idx) {
                            std::fprintf(stderr, "oracle: nil MatchmakerEntry in a combo with room (matchmaker_process.go:174)\n");
                            std::abort();
                        }
                        if (hit->session_set.count(e.idx->entries[e.pi].session_id)) { session_conflict = true; break; }
                        if (rev) {
                            if (!validate_match(m, *hit, e.idx->ticket)) { mutual_conflict = true; break; }
                            auto ee = indexes_copy.find(e.idx->ticket);
                            if (ee != indexes_copy.end()) {
                                if (!validate_match(m, *ee->second, hid)) { mutual_conflict = true; break; }
                            }
                        }
                    }
                    if (session_conflict || mutual_conflict) continue;  // sticky sessionIdConflict (:156,:206)
                    for (int k = 0; k < (int)hit->entries.size(); k++) combo.push_back({hit, k});
                    found_idx = (int)ci;
                    break;
                }
            }
            if (found_idx < 0) {
                vector<Entry> nc;
                for (int k = 0; k < (int)hit->entries.size(); k++) nc.push_back({hit, k});
                combos.push_back(std::move(nc));
                found_idx = (int)combos.size() - 1;
            }
            // foundCombo (:213, :224) is a slice header over the backing array of
            // entryCombos[foundComboIdx]: `stored` is that array, `flen` the
            // header's length.  The trim below shortens the header only; the
            // stored slice keeps its length with nil'd tail slots (:265-267).
            vector<Entry>& stored = combos[found_idx];
            int flen = (int)stored.size();
            int l = flen + ai->count;
            if (l == ai->max_count ||
                (last_interval && l >= ai->min_count && l <= ai->max_count && hit_counter >= last_hit_counter)) {
                int rem = l % ai->count_multiple;
                if (rem != 0) {
                    // eligibleIndexesUniq, pinned to first-appearance order
                    vector<IP> eligible;
                    std::unordered_set<const Index*> seen;
                    for (int i = 0; i < flen; i++) {
                        auto fi = indexes_copy.find(stored[i].idx->ticket);
                        if (fi != indexes_copy.end() && fi->second->count <= rem && !seen.count(fi->second.get())) {
                            seen.insert(fi->second.get());
                            eligible.push_back(fi->second);
                        }
                    }
                    auto groups = group_indexes(eligible, 0, rem);
                    if (groups.empty()) continue;
                    std::stable_sort(groups.begin(), groups.end(),
                                     [](const IGroup& a, const IGroup& b) { return a.avg < b.avg; });
                    for (auto& eg : groups[0].indexes) {
                        for (int i = 0; i < flen; i++) {
                            if (eg->ticket == stored[i].idx->ticket) {
                                stored[i] = stored[flen - 1];       // swap-remove in the shared array (:265)
                                stored[flen - 1] = Entry{nullptr, 0};  // :266
                                flen--;                               // :267 (the header only)
                                i--;
                            }
                        }
                    }
                    l = flen + ai->count;
                    if (l % ai->count_multiple != 0) continue;
                }
                bool cond_failed = false;
                for (int i = 0; i < flen; i++) {
                    auto fi = indexes_copy.find(stored[i].idx->ticket);
                    if (fi != indexes_copy.end() &&
                        (fi->second->min_count > l || fi->second->max_count < l || l % fi->second->count_multiple != 0)) {
                        cond_failed = true;
                        break;
                    }
                }
                if (cond_failed) continue;
                vector<Entry> current(stored.begin(), stored.begin() + flen);
                for (int k = 0; k < (int)ai->entries.size(); k++) current.push_back({ai, k});
                combos.erase(combos.begin() + found_idx);
                for (auto& e : current) {
                    if (selected(e.idx.get())) continue;
                    e.idx->selected_in = pass;
                    bluge_delete(m, e.idx->ticket);   // synchronous batch delete (:306-321)
                }
                matched.push_back(std::move(current));
                break;
            }
        }
    }
}

// processCustom (matchmaker_process.go:336-576) up to the override call.
static void process_custom(Matchmaker& m, const vector<IP>& order,
                           const std::unordered_map<string, IP>& indexes_copy,
                           vector<vector<Entry>>& candidates, vector<string>& expired, int64_t* pair_evals) {
    const int max_intervals = m.cfg.max_intervals;
    RevThresholdTimer timer(m);  // :340-346
    bool threshold = false;
    for (const IP& ix : order) ix->intervals++;
    for (const IP& ix : order) {
        if (!threshold && timer.fired()) threshold = true;  // :353-358
        const bool rev = m.cfg.rev_precision != 0 && !threshold;  // :439, :519
        const string& ticket = ix->ticket;
        bool last_interval = ix->intervals >= max_intervals || ix->min_count == ix->max_count;
        if (last_interval) expired.push_back(ticket);
        if (!m.active) continue;
        vector<Hit> hits = search_hits(m, *ix);
        *pair_evals += (int64_t)m.bluge_pos.size();
        vector<IP> hit_indexes;
        for (auto& h : hits) {
            if (h.idx->ticket == ticket) continue;
            auto hi_it = indexes_copy.find(h.idx->ticket);
            if (hi_it == indexes_copy.end()) continue;
            const IP& hit = hi_it->second;
            if (rev && !validate_match(m, *hit, ticket)) continue;
            if (ix->max_count < hit->max_count && hit->intervals <= max_intervals) continue;
            bool sc = false;
            for (auto& s : ix->session_ids)
                if (hit->session_set.count(s)) { sc = true; break; }
            if (sc) continue;
            hit_indexes.push_back(hit);
        }
        // combineIndexes (:578-612): Go `1 << length` is 0 / negative for length >= 63
        size_t length = hit_indexes.size();
        if (length >= 63) continue;
        int cmin = ix->min_count - ix->count, cmax = ix->max_count - ix->count;
        if (cmax <= 0) continue;  // `count > max` rejects every mask
        uint64_t limit = 1ULL << length;
        for (uint64_t bits = 1; bits < limit; bits++) {
            int cnt = __builtin_popcountll(bits);
            if (cnt > cmax) {
                // `continue` (:590) up to the next mask that can pass: below
                // bits + lowbit(bits) every mask holds all of bits' set bits
                // plus more, so it fails the same test (keeps n <= 62 tractable)
                bits += (bits & (~bits + 1)) - 1;
                continue;
            }
            vector<IP> combo;
            int entry_count = 0;
            bool over = false;
            for (size_t el = 0; el < length; el++) {
                if ((bits >> el) & 1) {
                    entry_count += hit_indexes[el]->count;
                    if (entry_count > cmax) { over = true; break; }
                    combo.push_back(hit_indexes[el]);
                }
            }
            if (over || entry_count < cmin) continue;
            int hit_count = 0;
            for (auto& h : combo) hit_count += h->count;
            hit_count += ix->count;
            if (hit_count > ix->max_count || hit_count < ix->min_count) continue;
            if (hit_count % ix->count_multiple != 0) continue;
            bool reject = false;
            for (auto& h : combo) {
                if (hit_count > h->max_count || hit_count < h->min_count) { reject = true; break; }
                if (hit_count % h->count_multiple != 0) { reject = true; break; }
                if (hit_count < h->max_count && h->intervals <= max_intervals) { reject = true; break; }
            }
            if (reject) continue;
            bool sconf = false, mconf = false;
            std::unordered_set<string> sids;
            vector<std::pair<string, IP>> parsed_queries;  // pinned: insertion order
            for (auto& h : combo) {
                for (auto& sid : h->session_ids) {
                    if (sids.count(sid)) { sconf = true; break; }
                    sids.insert(sid);
                    if (rev) {
                        for (auto& pq : parsed_queries) {
                            if (!validate_match(m, *h, pq.first)) { mconf = true; break; }
                            if (!validate_match(m, *pq.second, h->ticket)) { mconf = true; break; }
                        }
                        if (mconf) break;
                        bool present = false;
                        for (auto& pq : parsed_queries) if (pq.first == h->ticket) { present = true; pq.second = h; }
                        if (!present) parsed_queries.push_back({h->ticket, h});
                    }
                }
                if (sconf || mconf) break;
            }
            if (sconf || mconf) continue;
            vector<Entry> me;
            for (auto& h : combo)
                for (int k = 0; k < (int)h->entries.size(); k++) me.push_back({h, k});
            for (int k = 0; k < (int)ix->entries.size(); k++) me.push_back({ix, k});
            candidates.push_back(std::move(me));
        }
    }
}

// Process() post-pass (matchmaker.go:320-372): expire, completeness re-check with
// swap-remove, bookkeeping deletes.
static void finish_pass(Matchmaker& m, const vector<string>& expired, vector<vector<Entry>>& matched) {
    for (auto& t : expired) m.active_indexes.erase(t);
    for (int i = 0; i < (int)matched.size(); i++) {
        bool incomplete = false;
        for (auto& e : matched[i])
            if (!m.indexes.count(e.idx->ticket)) { incomplete = true; break; }
        if (incomplete) {
            matched[i] = std::move(matched.back());
            matched.pop_back();
            i--;
            continue;
        }
        for (auto& e : matched[i]) {
            const string t = e.idx->ticket;  // matched: reported by the pass result, not the drain (ABI 4)
            m.indexes.erase(t);
            m.active_indexes.erase(t);
            m.rev_cache.erase(t);
            const string& sid = e.idx->entries[e.pi].session_id;
            auto st = m.session_tickets.find(sid);
            if (st != m.session_tickets.end()) {
                if (st->second.size() <= 1) m.session_tickets.erase(st);
                else st->second.erase(t);
            }
            if (!e.idx->party_id.empty()) {
                auto pt = m.party_tickets.find(e.idx->party_id);
                if (pt != m.party_tickets.end()) {
                    if (pt->second.size() <= 1) m.party_tickets.erase(pt);
                    else pt->second.erase(t);
                }
            }
        }
    }
}

static void fill_matched(Matchmaker& m, const vector<vector<Entry>>& groups, mm_matched* out, bool candidates) {
    auto* offs = new int32_t[groups.size() + 1];
    size_t n = 0;
    for (auto& g : groups) n += g.size();
    auto* ents = new mm_entry_ref[n > 0 ? n : 1];
    auto* strs = new vector<string>();
    strs->reserve(n);
    size_t k = 0;
    offs[0] = 0;
    for (size_t gi = 0; gi < groups.size(); gi++) {
        for (auto& e : groups[gi]) {
            strs->push_back(e.idx->ticket);
            ents[k].presence_index = e.pi;
            ents[k].reserved = 0;
            k++;
        }
        offs[gi + 1] = (int32_t)k;
    }
    for (size_t i = 0; i < k; i++) ents[i].ticket = (*strs)[i].c_str();
    auto* gc = new int64_t[groups.size() + 1];
    for (size_t gi = 0; gi < groups.size(); gi++) gc[gi] = groups[gi].empty() ? 0 : groups[gi].back().idx->created_at;
    out->group_created = gc;
    out->n_groups = (int32_t)groups.size();
    out->n_entries = (int32_t)k;
    out->group_offsets = offs;
    out->entries = ents;
    out->is_candidates = candidates ? 1 : 0;
    out->reserved2 = (int64_t)(intptr_t)strs;
}

static IP make_index(Matchmaker& m, const mm_ticket& t, QP parsed, bool from_insert) {
    auto ix = std::make_shared<Index>();
    ix->ticket = t.ticket ? t.ticket : "";
    ix->min_count = t.min_count;
    ix->max_count = t.max_count;
    ix->count_multiple = t.count_multiple;
    ix->party_id = t.party_id ? t.party_id : "";
    ix->created_at = t.created_at;
    ix->query = t.query ? t.query : "";
    ix->count = t.n_presences;
    ix->session_id = t.session_id ? t.session_id : "";
    ix->intervals = from_insert ? t.intervals : 0;
    ix->node = from_insert ? (t.node ? t.node : "") : m.node;
    for (int i = 0; i < t.n_presences; i++) {
        Presence p{t.presences[i].user_id ? t.presences[i].user_id : "",
                   t.presences[i].session_id ? t.presences[i].session_id : "",
                   t.presences[i].username ? t.presences[i].username : "",
                   t.presences[i].node ? t.presences[i].node : ""};
        ix->entries.push_back(p);
        if (!ix->session_set.count(p.session_id)) {
            ix->session_set.insert(p.session_id);
            ix->session_ids.push_back(p.session_id);
        }
    }
    for (int i = 0; i < t.n_str_props; i++) ix->sprops.push_back({t.str_props[i].key, t.str_props[i].value});
    for (int i = 0; i < t.n_num_props; i++) ix->nprops.push_back({t.num_props[i].key, t.num_props[i].value});
    ix->parsed = parsed;
    build_doc(*ix);
    return ix;
}


}  // namespace oracle

using namespace oracle;

extern "C" {

int mm_abi_version(void) { return MM_ABI_VERSION; }
const char* mm_backend_name(void) { return "cpu-oracle"; }

void* mm_create(const mm_config* cfg) {
    if (!cfg) return nullptr;
    auto* m = new Matchmaker();
    m->cfg = *cfg;
    m->node = cfg->node ? cfg->node : "";
    m->cfg.node = nullptr;
    return m;
}
void mm_destroy(void* h) { delete static_cast<Matchmaker*>(h); }
void mm_pause(void* h) { static_cast<Matchmaker*>(h)->active = false; }
void mm_resume(void* h) { static_cast<Matchmaker*>(h)->active = true; }
void mm_stop(void* h) { static_cast<Matchmaker*>(h)->stopped = true; }
const char* mm_last_error(void* h) { return h ? static_cast<Matchmaker*>(h)->last_error.c_str() : "null handle"; }

// Add (matchmaker.go:443-565)
int mm_add(void* h, const mm_ticket* t) {
    auto& m = *static_cast<Matchmaker*>(h);
    if (m.stopped) return MM_ERR_NOT_AVAILABLE;
    QP parsed;
    int rc = parse_query(t->query ? t->query : "", &parsed);
    if (rc != 0) return rc;
    {
        std::unordered_set<string> sids;
        for (int i = 0; i < t->n_presences; i++) {
            string s = t->presences[i].session_id ? t->presences[i].session_id : "";
            if (sids.count(s)) return MM_ERR_DUPLICATE_SESSION;
            sids.insert(s);
        }
    }
    std::lock_guard<std::mutex> lk(m.mu);
    for (int i = 0; i < t->n_presences; i++) {
        auto it = m.session_tickets.find(t->presences[i].session_id ? t->presences[i].session_id : "");
        if (it != m.session_tickets.end() && (int)it->second.size() >= m.cfg.max_tickets) return MM_ERR_TOO_MANY_TICKETS;
    }
    string party = t->party_id ? t->party_id : "";
    if (!party.empty()) {
        auto it = m.party_tickets.find(party);
        if (it != m.party_tickets.end() && (int)it->second.size() >= m.cfg.max_tickets) return MM_ERR_TOO_MANY_TICKETS;
    }
    IP ix = make_index(m, *t, parsed, false);
    bluge_update(m, ix);
    for (auto& p : ix->entries) m.session_tickets[p.session_id].insert(ix->ticket);
    if (!party.empty()) m.party_tickets[party].insert(ix->ticket);
    m.indexes[ix->ticket] = ix;
    m.active_indexes[ix->ticket] = ix;
    m.rev_cache[ix->ticket] = {};
    return MM_OK;
}

// Insert (matchmaker.go:567-682)
int mm_insert(void* h, const mm_ticket* ts, int32_t n) {
    auto& m = *static_cast<Matchmaker*>(h);
    if (m.stopped || n <= 0) return MM_OK;
    vector<IP> batch;
    for (int i = 0; i < n; i++) {
        QP parsed;
        if (parse_query(ts[i].query ? ts[i].query : "", &parsed) != 0) continue;  // logged, skipped
        batch.push_back(make_index(m, ts[i], parsed, true));
    }
    std::lock_guard<std::mutex> lk(m.mu);
    for (auto& ix : batch) bluge_update(m, ix);
    for (auto& ix : batch) {
        m.indexes[ix->ticket] = ix;
        m.rev_cache[ix->ticket] = {};
        if (ix->intervals < m.cfg.max_intervals) m.active_indexes[ix->ticket] = ix;
        if (!ix->party_id.empty()) m.party_tickets[ix->party_id].insert(ix->ticket);
        for (auto& p : ix->entries) m.session_tickets[p.session_id].insert(ix->ticket);
    }
    return MM_OK;
}

int mm_extract(void* h, mm_extract_list* out) {
    auto& m = *static_cast<Matchmaker*>(h);
    out->n = 0;
    out->tickets = nullptr;
    if (m.stopped) return MM_OK;
    std::lock_guard<std::mutex> lk(m.mu);
    vector<IP> v;
    for (auto& kv : m.indexes)
        if (kv.second->node == m.node) v.push_back(kv.second);
    std::sort(v.begin(), v.end(), [](const IP& a, const IP& b) { return a->ticket < b->ticket; });
    auto* arr = new mm_ticket[v.size() > 0 ? v.size() : 1];
    for (size_t i = 0; i < v.size(); i++) {
        const Index& ix = *v[i];
        mm_ticket& t = arr[i];
        t.ticket = ix.ticket.c_str();
        t.session_id = ix.session_id.c_str();
        t.party_id = ix.party_id.c_str();
        t.query = ix.query.c_str();
        t.min_count = ix.min_count;
        t.max_count = ix.max_count;
        t.count_multiple = ix.count_multiple;
        t.intervals = ix.intervals;
        t.created_at = ix.created_at;
        t.node = ix.node.c_str();
        auto* ps = new mm_presence[ix.entries.size() > 0 ? ix.entries.size() : 1];
        for (size_t k = 0; k < ix.entries.size(); k++)
            ps[k] = {ix.entries[k].user_id.c_str(), ix.entries[k].session_id.c_str(), ix.entries[k].username.c_str(),
                     ix.entries[k].node.c_str()};
        t.presences = ps;
        t.n_presences = (int32_t)ix.entries.size();
        auto* sp = new mm_str_prop[ix.sprops.size() > 0 ? ix.sprops.size() : 1];
        for (size_t k = 0; k < ix.sprops.size(); k++) sp[k] = {ix.sprops[k].first.c_str(), ix.sprops[k].second.c_str()};
        t.str_props = sp;
        t.n_str_props = (int32_t)ix.sprops.size();
        auto* np = new mm_num_prop[ix.nprops.size() > 0 ? ix.nprops.size() : 1];
        for (size_t k = 0; k < ix.nprops.size(); k++) np[k] = {ix.nprops[k].first.c_str(), ix.nprops[k].second};
        t.num_props = np;
        t.n_num_props = (int32_t)ix.nprops.size();
    }
    out->n = (int32_t)v.size();
    out->tickets = arr;
    m.extract_keep = v;  // strings stay valid until mm_free_extract / the next extract
    return MM_OK;
}

void mm_free_extract(void* h, mm_extract_list* out) {
    (void)h;
    if (!out || !out->tickets) return;
    for (int i = 0; i < out->n; i++) {
        delete[] out->tickets[i].presences;
        delete[] out->tickets[i].str_props;
        delete[] out->tickets[i].num_props;
    }
    delete[] out->tickets;
    out->tickets = nullptr;
    out->n = 0;
}

static void erase_session_ticket(Matchmaker& m, const string& sid, const string& ticket) {
    auto st = m.session_tickets.find(sid);
    if (st != m.session_tickets.end()) {
        if (st->second.size() <= 1) m.session_tickets.erase(st);
        else st->second.erase(ticket);
    }
}
static void erase_party_ticket(Matchmaker& m, const string& pid, const string& ticket) {
    auto pt = m.party_tickets.find(pid);
    if (pt != m.party_tickets.end()) {
        if (pt->second.size() <= 1) m.party_tickets.erase(pt);
        else pt->second.erase(ticket);
    }
}

int mm_remove_session(void* h, const char* session_id, const char* ticket) {  // :725-767
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    auto it = m.indexes.find(ticket);
    if (it == m.indexes.end() || !it->second->party_id.empty() || it->second->session_id != session_id)
        return MM_ERR_TICKET_NOT_FOUND;
    IP ix = it->second;
    m.note_removed(ix->ticket);
    m.indexes.erase(it);
    for (auto& p : ix->entries) erase_session_ticket(m, p.session_id, ix->ticket);
    if (!ix->party_id.empty()) erase_party_ticket(m, ix->party_id, ix->ticket);
    m.active_indexes.erase(ix->ticket);
    m.rev_cache.erase(ix->ticket);
    bluge_delete(m, ix->ticket);
    return MM_OK;
}

int mm_remove_session_all(void* h, const char* session_id) {  // :769-828
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    auto st = m.session_tickets.find(session_id);
    if (st == m.session_tickets.end()) return MM_OK;
    std::set<string> tickets = st->second;
    m.session_tickets.erase(st);
    for (auto& t : tickets) {
        bluge_delete(m, t);
        auto it = m.indexes.find(t);
        if (it == m.indexes.end()) continue;
        IP ix = it->second;
        m.note_removed(t);
        m.indexes.erase(it);
        m.active_indexes.erase(t);
        m.rev_cache.erase(t);
        for (auto& p : ix->entries) {
            if (p.session_id == session_id) continue;
            erase_session_ticket(m, p.session_id, t);
        }
        if (!ix->party_id.empty()) erase_party_ticket(m, ix->party_id, t);
    }
    return MM_OK;
}

int mm_remove_party(void* h, const char* party_id, const char* ticket) {  // :830-870
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    auto it = m.indexes.find(ticket);
    if (it == m.indexes.end() || !it->second->session_id.empty() || it->second->party_id != party_id)
        return MM_ERR_TICKET_NOT_FOUND;
    IP ix = it->second;
    m.note_removed(ix->ticket);
    m.indexes.erase(it);
    for (auto& p : ix->entries) erase_session_ticket(m, p.session_id, ix->ticket);
    erase_party_ticket(m, party_id, ix->ticket);
    m.active_indexes.erase(ix->ticket);
    m.rev_cache.erase(ix->ticket);
    bluge_delete(m, ix->ticket);
    return MM_OK;
}

int mm_remove_party_all(void* h, const char* party_id) {  // :872-917
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    auto pt = m.party_tickets.find(party_id);
    if (pt == m.party_tickets.end()) return MM_OK;
    std::set<string> tickets = pt->second;
    m.party_tickets.erase(pt);
    for (auto& t : tickets) {
        bluge_delete(m, t);
        auto it = m.indexes.find(t);
        if (it == m.indexes.end()) continue;
        IP ix = it->second;
        m.note_removed(t);
        m.indexes.erase(it);
        m.active_indexes.erase(t);
        m.rev_cache.erase(t);
        for (auto& p : ix->entries) erase_session_ticket(m, p.session_id, t);
    }
    return MM_OK;
}

static void remove_tickets(Matchmaker& m, const vector<IP>& v) {
    for (auto& ix : v) {
        m.note_removed(ix->ticket);
        bluge_delete(m, ix->ticket);
        m.indexes.erase(ix->ticket);
        m.active_indexes.erase(ix->ticket);
        m.rev_cache.erase(ix->ticket);
        if (!ix->party_id.empty()) erase_party_ticket(m, ix->party_id, ix->ticket);
        for (auto& p : ix->entries) erase_session_ticket(m, p.session_id, ix->ticket);
    }
}

int mm_remove_all(void* h, const char* node) {  // :919-970
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    vector<IP> v;
    for (auto& kv : m.indexes)
        if (kv.second->node == node) v.push_back(kv.second);
    remove_tickets(m, v);
    return MM_OK;
}

int mm_remove(void* h, const char* const* tickets, int32_t n) {  // :972-1024
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    vector<IP> v;
    for (int i = 0; i < n; i++) {
        auto it = m.indexes.find(tickets[i]);
        if (it == m.indexes.end()) continue;
        bool dup = false;
        for (auto& x : v) if (x == it->second) dup = true;
        if (!dup) v.push_back(it->second);
    }
    remove_tickets(m, v);
    return MM_OK;
}

// Process (matchmaker.go:282-441), delivery excluded.
int mm_process(void* h, mm_matched* out) {
    auto& m = *static_cast<Matchmaker*>(h);
    std::memset(out, 0, sizeof(*out));
    auto t0 = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(m.mu);
    if (m.custom_open) return MM_ERR_STATE;
    if (m.active_indexes.empty()) { fill_matched(m, {}, out, false); return MM_OK; }
    std::unordered_map<string, IP> indexes_copy = m.indexes;  // snapshot (matchmaker.go:300-307)
    vector<IP> order = active_order(m);
    vector<vector<Entry>> matched;
    vector<string> expired;
    int64_t pe = 0;
    lk.unlock();  // the pass runs unlocked (:309); mutators apply to the live maps meanwhile
    if (m.cfg.override_enabled) {
        process_custom(m, order, indexes_copy, matched, expired, &pe);
        if (m.pass_hook) m.pass_hook(m.pass_hook_ctx);
        lk.lock();
        out->n_expired = (int32_t)expired.size();
        if (matched.empty()) {
            // no candidates: the override is not called (:568-570)
            vector<vector<Entry>> none;
            finish_pass(m, expired, none);
            fill_matched(m, {}, out, false);
        } else {
            m.custom_open = true;
            m.custom_expired = expired;
            fill_matched(m, matched, out, true);
        }
    } else {
        process_default(m, order, indexes_copy, matched, expired, &pe);
        if (m.pass_hook) m.pass_hook(m.pass_hook_ctx);
        lk.lock();  // :320
        out->n_expired = (int32_t)expired.size();
        finish_pass(m, expired, matched);
        fill_matched(m, matched, out, false);
    }
    out->pair_evals = pe;
    out->pairs_decided = pe;  // every row that searched visited every document
    out->pass_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return MM_OK;
}

int mm_process_commit(void* h, const int32_t* group_offsets, const mm_entry_ref* entries, int32_t n_groups,
                      mm_matched* out) {
    auto& m = *static_cast<Matchmaker*>(h);
    std::memset(out, 0, sizeof(*out));
    std::lock_guard<std::mutex> lk(m.mu);
    if (!m.custom_open) return MM_ERR_STATE;
    vector<vector<Entry>> groups;
    for (int g = 0; g < n_groups; g++) {
        vector<Entry> grp;
        for (int k = group_offsets[g]; k < group_offsets[g + 1]; k++) {
            auto it = m.indexes.find(entries[k].ticket);
            IP ix;
            if (it != m.indexes.end()) ix = it->second;
            else {
                // entry for a ticket no longer present: keep a stub so the completeness check drops the group
                ix = std::make_shared<Index>();
                ix->ticket = entries[k].ticket;
                ix->entries.push_back({});
            }
            grp.push_back({ix, std::min<int>(entries[k].presence_index, (int)ix->entries.size() - 1)});
        }
        groups.push_back(std::move(grp));
    }
    finish_pass(m, m.custom_expired, groups);
    m.custom_open = false;
    m.custom_expired.clear();
    fill_matched(m, groups, out, false);
    return MM_OK;
}

void mm_free_matched(void* h, mm_matched* out) {
    (void)h;
    if (!out) return;
    delete[] out->group_offsets;
    delete[] out->entries;
    delete[] out->group_created;
    delete reinterpret_cast<vector<string>*>((intptr_t)out->reserved2);
    std::memset(out, 0, sizeof(*out));
}

// Delivery (nakama_mm.h "pipelined delivery"): the result goes to fn in pass
// order, then is freed; the caller gets the counts (test infrastructure: no
// thread, no queue — depth only validated).
int mm_set_delivery(void* h, mm_deliver_fn fn, void* ctx, int32_t depth) {
    if (!h || (fn && depth < 1)) return MM_ERR_ARG;
    auto& m = *static_cast<Matchmaker*>(h);
    m.deliver_fn = fn;
    m.deliver_ctx = ctx;
    m.deliver_seq = 0;
    return MM_OK;
}
static void deliver_now(Matchmaker& m, void* h, mm_matched& r, mm_matched* summary) {
    *summary = r;
    summary->group_offsets = nullptr;
    summary->entries = nullptr;
    summary->group_created = nullptr;
    summary->reserved2 = 0;
    m.deliver_fn(m.deliver_ctx, &r, m.deliver_seq++);
    mm_free_matched(h, &r);
}
int mm_process_deliver(void* h, mm_matched* summary) {
    if (!h || !summary) return MM_ERR_ARG;
    auto& m = *static_cast<Matchmaker*>(h);
    if (!m.deliver_fn) return MM_ERR_STATE;
    mm_matched r{};
    const int rc = mm_process(h, &r);
    if (rc != MM_OK) return rc;
    if (r.is_candidates) {
        *summary = r;
        return MM_OK;
    }
    deliver_now(m, h, r, summary);
    return MM_OK;
}
int mm_process_commit_deliver(void* h, const int32_t* group_offsets, const mm_entry_ref* entries, int32_t n_groups,
                              mm_matched* summary) {
    if (!h || !summary) return MM_ERR_ARG;
    auto& m = *static_cast<Matchmaker*>(h);
    if (!m.deliver_fn) return MM_ERR_STATE;
    mm_matched r{};
    const int rc = mm_process_commit(h, group_offsets, entries, n_groups, &r);
    if (rc != MM_OK) return rc;
    deliver_now(m, h, r, summary);
    return MM_OK;
}
int mm_delivery_flush(void* h) {
    if (!h) return MM_ERR_ARG;
    return static_cast<Matchmaker*>(h)->deliver_fn ? MM_OK : MM_ERR_STATE;
}

int32_t mm_ticket_count(void* h) { auto& m = *static_cast<Matchmaker*>(h); std::lock_guard<std::mutex> lk(m.mu); return (int32_t)m.indexes.size(); }
// m.sessionTickets / m.partyTickets sizes (matchmaker.go:201-204, read by Add :505-520)
int32_t mm_session_ticket_count(void* h, const char* sid) {
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    auto it = m.session_tickets.find(sid ? sid : "");
    return it == m.session_tickets.end() ? 0 : (int32_t)it->second.size();
}
int32_t mm_party_ticket_count(void* h, const char* pid) {
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    auto it = m.party_tickets.find(pid ? pid : "");
    return it == m.party_tickets.end() ? 0 : (int32_t)it->second.size();
}
// membership in m.indexes
int32_t mm_find_tickets(void* h, const char* const* ids, int32_t n, uint8_t* found) {
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    int32_t k = 0;
    for (int32_t i = 0; i < n; i++) {
        found[i] = m.indexes.count(ids[i] ? ids[i] : "") ? 1 : 0;
        k += found[i];
    }
    return k;
}
int32_t mm_active_count(void* h) { auto& m = *static_cast<Matchmaker*>(h); std::lock_guard<std::mutex> lk(m.mu); return (int32_t)m.active_indexes.size(); }

int32_t mm_debug_hits(void* h, const char* ticket, const char** tickets_out, double* scores_out, int32_t cap) {
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    auto it = m.indexes.find(ticket);
    if (it == m.indexes.end()) return -1;
    vector<Hit> hits = search_hits(m, *it->second);
    m.dbg.clear();
    for (auto& x : hits)
        if (x.idx->ticket != ticket) m.dbg.push_back(x.idx->ticket);
    int32_t n = 0;
    for (auto& x : hits) {
        if (x.idx->ticket == ticket) continue;
        if (n < cap) {
            if (tickets_out) tickets_out[n] = m.dbg[n].c_str();
            if (scores_out) scores_out[n] = x.score;
        }
        n++;
    }
    return n;
}

int mm_debug_term_match(int32_t kind, const char* pattern, int32_t fuzziness, const char* term, double* boost) {
    *boost = 0.0;
    string t = term;
    if (kind == 2) {
        if (fuzziness < 0 || fuzziness > 2) return -1;
        int d = oracle_re::osa(pattern, t);
        if (d > fuzziness) return 0;
        *boost = 1.0;
        if (t != pattern)
            *boost = 1.0 - (double)d / (double)std::min(oracle_re::rune_count(pattern), oracle_re::rune_count(t));
        return 1;
    }
    string re = pattern;
    if (kind == 3) {  // the query parser's wildcard lowering, via a one-clause query
        re.clear();
        for (char c : string(pattern)) {
            if (string("+()^$.{}[]|\\").find(c) != string::npos) { re += '\\'; re += c; }
            else if (c == '*') re += ".*";
            else if (c == '?') re += ".";
            else re += c;
        }
    }
    oracle_re::Regexp rx;
    oracle_re::Status st = rx.compile(re);
    if (st != oracle_re::OK) return st == oracle_re::UNSUPPORTED ? -2 : -1;
    if (!rx.matches(t)) return 0;
    *boost = 1.0;
    return 1;
}

int mm_drain_removed(void* h, mm_str_list* out) {
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    m.track_removed = true;
    auto* v = new vector<string>(std::move(m.removed));
    m.removed.clear();
    auto* ptrs = new const char*[v->size() + 1];
    for (size_t i = 0; i < v->size(); i++) ptrs[i] = (*v)[i].c_str();
    ptrs[v->size()] = reinterpret_cast<const char*>(v);  // owner, after the last item
    out->n = (int32_t)v->size();
    out->items = ptrs;
    return MM_OK;
}

void mm_free_str_list(void* h, mm_str_list* out) {
    (void)h;
    if (!out || !out->items) return;
    delete reinterpret_cast<const vector<string>*>(out->items[out->n]);
    delete[] out->items;
    out->items = nullptr;
    out->n = 0;
}

void mm_debug_set_pass_hook(void* h, void (*fn)(void*), void* ctx) {
    auto& m = *static_cast<Matchmaker*>(h);
    std::lock_guard<std::mutex> lk(m.mu);
    m.pass_hook = fn;
    m.pass_hook_ctx = ctx;
}

int mm_debug_compile(const char* query) {
    QP q;
    return parse_query(query ? query : "", &q);
}

int32_t mm_debug_group_indexes(const int32_t* counts, const int64_t* created_at, int32_t n, int32_t required,
                               int32_t* group_offsets, int32_t* group_members, int64_t* avg_created_at, int32_t cap) {
    vector<IP> v;
    std::unordered_map<const Index*, int> pos;
    for (int i = 0; i < n; i++) {
        auto ix = std::make_shared<Index>();
        ix->count = counts[i];
        ix->created_at = created_at[i];
        pos[ix.get()] = i;
        v.push_back(ix);
    }
    auto groups = group_indexes(v, 0, required);
    int32_t k = 0, g = 0;
    group_offsets[0] = 0;
    for (auto& gr : groups) {
        if (g >= cap) break;
        for (auto& ix : gr.indexes) {
            if (k < 8 * cap) group_members[k++] = pos[ix.get()];
        }
        avg_created_at[g] = gr.avg;
        group_offsets[++g] = k;
    }
    return g;
}

}  // extern "C"
