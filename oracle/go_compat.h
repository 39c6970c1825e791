// oracle/go_compat.h — TEST INFRASTRUCTURE ONLY (CPU oracle).
//
// Small restatements of Go standard-library behaviour the reference path relies
// on: strconv.ParseFloat syntax (used by the query_string parser for numbers and
// ^boost, vendor/.../query_string/query_string_parser.go:198-260), time.Parse for
// the five layouts of blugeParseDateTime (server/match_common.go:221-236) and the
// RFC3339 layout of the date-range grammar (query_string_parser.go:163-169), and
// bluge's Float64ToInt64 (vendor/.../bluge/numeric/float.go:21-27).
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
// anything under oracle/.
#pragma once
#include <cstdint>
#include <cstring>
#include <cstdlib>
#include <cmath>
#include <string>
#include <cerrno>

namespace gocompat {

// bluge numeric/float.go:21-27
inline int64_t f2i(double f) {
    int64_t i;
    std::memcpy(&i, &f, 8);
    if (i < 0) i ^= 0x7fffffffffffffffLL;
    return i;
}
inline double i2f(int64_t i) {
    if (i < 0) i ^= 0x7fffffffffffffffLL;
    double f;
    std::memcpy(&f, &i, 8);
    return f;
}

inline bool ieq(const std::string& a, const char* b) {
    size_t n = std::strlen(b);
    if (a.size() != n) return false;
    for (size_t i = 0; i < n; i++) {
        char c = a[i];
        if (c >= 'A' && c <= 'Z') c = char(c - 'A' + 'a');
        if (c != b[i]) return false;
    }
    return true;
}

// strconv.ParseFloat(s, 64): decimal or hex mantissa, optional exponent, optional
// sign, "inf"/"infinity"/"nan" (case-insensitive), underscores only with a base
// prefix.  Overflow (±Inf from a finite literal) is an error (ErrRange).
inline bool parse_float(const std::string& s, double* out) {
    if (s.empty()) return false;
    size_t i = 0;
    bool neg = false;
    if (s[i] == '+' || s[i] == '-') { neg = s[i] == '-'; i++; }
    std::string rest = s.substr(i);
    if (ieq(rest, "inf") || ieq(rest, "infinity")) { *out = neg ? -INFINITY : INFINITY; return true; }
    if (ieq(rest, "nan") && i == 0) { *out = NAN; return true; }
    if (rest.empty()) return false;
    bool hex = rest.size() >= 2 && rest[0] == '0' && (rest[1] == 'x' || rest[1] == 'X');
    std::string clean;
    size_t j = 0;
    if (hex) { clean = "0x"; j = 2; }
    bool sawdigits = false, sawdot = false, sawexp = false;
    bool underscore_ok = hex;  // base prefix present
    char prev = 0;
    for (; j < rest.size(); j++) {
        char c = rest[j];
        if (c == '_') {
            if (!underscore_ok) return false;
            prev = c;
            continue;
        }
        if (!sawexp && (std::isdigit((unsigned char)c) || (hex && std::isxdigit((unsigned char)c)))) {
            sawdigits = true;
            clean += c;
        } else if (!sawexp && c == '.' && !sawdot) {
            sawdot = true;
            clean += c;
        } else if (!sawexp && ((!hex && (c == 'e' || c == 'E')) || (hex && (c == 'p' || c == 'P')))) {
            if (!sawdigits) return false;
            sawexp = true;
            clean += c;
            if (j + 1 < rest.size() && (rest[j + 1] == '+' || rest[j + 1] == '-')) { clean += rest[j + 1]; j++; }
            if (j + 1 >= rest.size()) return false;
            bool expdig = false;
            for (size_t k = j + 1; k < rest.size(); k++) {
                if (rest[k] == '_') { if (!underscore_ok) return false; continue; }
                if (!std::isdigit((unsigned char)rest[k])) return false;
                expdig = true;
                clean += rest[k];
            }
            if (!expdig) return false;
            j = rest.size();
            break;
        } else {
            return false;
        }
        prev = c;
    }
    (void)prev;
    if (!sawdigits) return false;
    if (hex && !sawexp) return false;  // Go requires a 'p' exponent for hex floats
    errno = 0;
    char* end = nullptr;
    double v = std::strtod(clean.c_str(), &end);
    if (end == nullptr || *end != '\0') return false;
    if (std::isinf(v)) return false;  // ErrRange on overflow
    *out = neg ? -v : v;
    return true;
}

// Days from civil (proleptic Gregorian), Howard Hinnant's algorithm.
inline int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const unsigned yoe = static_cast<unsigned>(y - era * 400);
    const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + static_cast<int64_t>(doe) - 719468;
}
inline bool is_leap(int64_t y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }
inline int days_in(int m, int64_t y) {
    static const int dm[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    if (m == 2 && is_leap(y)) return 29;
    return dm[m - 1];
}

// A tiny restatement of Go time.Parse for the layouts the path uses.
// layout codes: 0 RFC3339Nano, 1 RFC3339, 2 "2006-01-02T15:04:05",
// 3 "2006-01-02 15:04:05", 4 "2006-01-02".  Returns UnixNano in *ns and
// whether the value equals Go's zero time (year 1, Jan 1, 00:00:00 UTC).
struct ParsedTime { int64_t unix_nano; bool is_zero; bool ok; bool overflow; };

inline bool getnum_fixed2(const std::string& v, size_t& p, int* out) {
    if (p + 2 > v.size() || !std::isdigit((unsigned char)v[p]) || !std::isdigit((unsigned char)v[p + 1])) return false;
    *out = (v[p] - '0') * 10 + (v[p + 1] - '0');
    p += 2;
    return true;
}
inline bool getnum_var12(const std::string& v, size_t& p, int* out) {
    // Go getnum(s, false): one digit, optionally a second one.
    if (p >= v.size() || !std::isdigit((unsigned char)v[p])) return false;
    int n = v[p] - '0';
    p++;
    if (p < v.size() && std::isdigit((unsigned char)v[p])) { n = n * 10 + (v[p] - '0'); p++; }
    *out = n;
    return true;
}

inline ParsedTime go_time_parse(const std::string& v, int layout) {
    ParsedTime r{0, false, false, false};
    size_t p = 0;
    // year "2006" (stdLongYear): four characters, the first a digit, Go atoi
    if (v.size() < 4) return r;
    int64_t year = 0;
    for (size_t q = 0; q < 4; q++) {
        if (!std::isdigit((unsigned char)v[q])) return r;
        year = year * 10 + (v[q] - '0');
    }
    p = 4;
    auto expect = [&](char c) { if (p < v.size() && v[p] == c) { p++; return true; } return false; };
    int month = 0, day = 0, hour = 0, minute = 0, sec = 0;
    int64_t nsec = 0;
    if (!expect('-')) return r;
    if (!getnum_fixed2(v, p, &month)) return r;
    if (!expect('-')) return r;
    if (!getnum_fixed2(v, p, &day)) return r;
    int64_t offset_sec = 0;
    if (layout != 4) {
        char sep = (layout == 3) ? ' ' : 'T';
        if (!expect(sep)) return r;
        if (!getnum_var12(v, p, &hour)) return r;  // "15" is stdHour (1-2 digits)
        if (!expect(':')) return r;
        if (!getnum_fixed2(v, p, &minute)) return r;
        if (!expect(':')) return r;
        if (!getnum_fixed2(v, p, &sec)) return r;
        // fractional seconds: accepted after "05" when the layout has none too
        if (p + 1 < v.size() && (v[p] == '.' || v[p] == ',') && std::isdigit((unsigned char)v[p + 1])) {
            size_t q = p + 1;
            int64_t frac = 0;
            int nd = 0;
            while (q < v.size() && std::isdigit((unsigned char)v[q])) {
                if (nd < 9) { frac = frac * 10 + (v[q] - '0'); }  // parseNanoseconds keeps 9 digits
                nd++;
                q++;
            }
            if (nd > 9) nd = 9;
            for (int k = nd; k < 9; k++) frac *= 10;
            nsec = frac;
            p = q;
        }
        if (layout == 0 || layout == 1) {
            if (p < v.size() && v[p] == 'Z') {
                p++;
            } else {
                if (p + 6 > v.size()) return r;
                char sg = v[p];
                if (sg != '+' && sg != '-') return r;
                p++;
                int oh = 0, om = 0;
                if (!getnum_fixed2(v, p, &oh)) return r;
                if (!expect(':')) return r;
                if (!getnum_fixed2(v, p, &om)) return r;
                if (oh > 24 || om > 60) return r;
                offset_sec = (int64_t)(oh * 3600 + om * 60) * (sg == '-' ? -1 : 1);
            }
        }
    }
    if (p != v.size()) return r;  // extra text
    if (month < 1 || month > 12) return r;
    if (day < 1 || day > days_in(month, year)) return r;
    if (hour >= 24 || minute >= 60 || sec >= 60) return r;
    int64_t days = days_from_civil(year, (unsigned)month, (unsigned)day);
    // seconds since epoch; UnixNano overflows outside ~1678..2262
    long double secs = (long double)days * 86400.0L + hour * 3600 + minute * 60 + sec - offset_sec;
    long double ns = secs * 1e9L + nsec;
    r.ok = true;
    {
        // time.Time.IsZero(): the instant 0001-01-01T00:00:00Z
        __int128 since1 = (__int128)(days - days_from_civil(1, 1, 1)) * 86400 + hour * 3600 + minute * 60 + sec -
                          offset_sec;
        r.is_zero = since1 == 0 && nsec == 0;
    }
    if (ns > 9.223372036854775807e18L || ns < -9.223372036854775808e18L) {
        r.overflow = true;
        // Go's UnixNano is undefined (wraps) outside the representable range; the
        // store path never relies on it.
        __int128 full = (__int128)days * 86400 + hour * 3600 + minute * 60 + sec - offset_sec;
        full = full * 1000000000 + nsec;
        r.unix_nano = (int64_t)(uint64_t)(unsigned __int128)full;
    } else {
        __int128 full = (__int128)days * 86400 + hour * 3600 + minute * 60 + sec - offset_sec;
        full = full * 1000000000 + nsec;
        r.unix_nano = (int64_t)full;
    }
    return r;
}

// blugeParseDateTime (server/match_common.go:221-236): first layout that parses.
inline bool bluge_parse_datetime(const std::string& v, int64_t* unix_nano) {
    for (int layout = 0; layout < 5; layout++) {
        ParsedTime t = go_time_parse(v, layout);
        if (t.ok) { *unix_nano = t.unix_nano; return true; }
    }
    return false;
}

}  // namespace gocompat
