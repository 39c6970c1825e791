#!/usr/bin/env python3
"""Generates the Unicode data of the two regexp matchers, as two headers in two
different layouts, so that a wrong table in one is not shared by the other:

  * nakama_amd/csrc/unicode_tables.h (the product, termmatch.cpp): per class
    name a sorted list of rune ranges, and the simple case-folding orbits;
  * oracle/unicode_ref.h (the oracle, go_regexp.h; test infrastructure): one
    sorted run-length table over all runes of (general category, script), and
    Go's unicode.SimpleFold as a (rune -> next rune of its orbit) map.

tests/test_unicode_tables.py recomputes both from unicodedata / regex and
checks every entry of both headers.

The reference builds with Go 1.20 (go.mod), whose unicode package is Unicode
13.0.0 — the same version as this interpreter's unicodedata (checked below).
  * categories: Go's unicode.Categories (`\\pL`, `\\p{Lu}`, ...): the two-letter
    categories and the one-letter unions (C = Cc|Cf|Co|Cs: Go's C table omits
    unassigned Cn), as sorted disjoint rune ranges;
  * scripts: Go's unicode.Scripts (`\\p{Greek}`; regexp/syntax looks a name up
    in Categories first, then Scripts).  unicodedata has no Script property;
    the installed `regex` module's Script data (a later Unicode version) is
    restricted to the runes assigned in Unicode 13.0.0, so scripts added later
    never appear and a rune keeps its later-version script (parity unpinned for
    the few runes whose script changed after 13.0, e.g. none of the ASCII or
    Latin-1 ranges);
  * folding: the orbits unicode.SimpleFold walks — the closure of the simple
    one-to-one lower/upper mappings, with U+0130 and U+0131 kept alone (Go's
    caseOrbit pins them to themselves).
"""
import os
import unicodedata

import regex

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "nakama_amd", "csrc", "unicode_tables.h")
OUT_ORACLE = os.path.join(ROOT, "oracle", "unicode_ref.h")
assert unicodedata.unidata_version == "13.0.0", unicodedata.unidata_version
MAX = 0x10FFFF

# Go 1.20 unicode.Scripts (Unicode 13.0.0 Scripts.txt values)
SCRIPTS = """Adlam Ahom Anatolian_Hieroglyphs Arabic Armenian Avestan Balinese Bamum Bassa_Vah Batak Bengali
Bhaiksuki Bopomofo Brahmi Braille Buginese Buhid Canadian_Aboriginal Carian Caucasian_Albanian Chakma Cham
Cherokee Chorasmian Common Coptic Cuneiform Cypriot Cyrillic Deseret Devanagari Dives_Akuru Dogra Duployan
Egyptian_Hieroglyphs Elbasan Elymaic Ethiopic Georgian Glagolitic Gothic Grantha Greek Gujarati Gunjala_Gondi
Gurmukhi Han Hangul Hanifi_Rohingya Hanunoo Hatran Hebrew Hiragana Imperial_Aramaic Inherited
Inscriptional_Pahlavi Inscriptional_Parthian Javanese Kaithi Kannada Katakana Kayah_Li Kharoshthi
Khitan_Small_Script Khmer Khojki Khudawadi Lao Latin Lepcha Limbu Linear_A Linear_B Lisu Lycian Lydian Mahajani
Makasar Malayalam Mandaic Manichaean Marchen Masaram_Gondi Medefaidrin Meetei_Mayek Mende_Kikakui
Meroitic_Cursive Meroitic_Hieroglyphs Miao Modi Mongolian Mro Multani Myanmar Nabataean Nandinagari New_Tai_Lue
Newa Nko Nushu Nyiakeng_Puachue_Hmong Ogham Ol_Chiki Old_Hungarian Old_Italic Old_North_Arabian Old_Permic
Old_Persian Old_Sogdian Old_South_Arabian Old_Turkic Oriya Osage Osmanya Pahawh_Hmong Palmyrene Pau_Cin_Hau
Phags_Pa Phoenician Psalter_Pahlavi Rejang Runic Samaritan Saurashtra Sharada Shavian Siddham SignWriting
Sinhala Sogdian Sora_Sompeng Soyombo Sundanese Syloti_Nagri Syriac Tagalog Tagbanwa Tai_Le Tai_Tham Tai_Viet
Takri Tamil Tangut Telugu Thaana Thai Tibetan Tifinagh Tirhuta Ugaritic Vai Wancho Warang_Citi Yezidi Yi
Zanabazar_Square""".split()
assert len(SCRIPTS) == 156


def category_of():
    return [unicodedata.category(chr(c)) if not 0xD800 <= c <= 0xDFFF else "Cs" for c in range(MAX + 1)]


def script_of(cat):
    """Script index per rune (-1: none / unassigned in Unicode 13.0)."""
    out = [-1] * (MAX + 1)
    assigned = "".join(chr(c) for c in range(MAX + 1) if cat[c] not in ("Cn", "Cs"))
    for k, name in enumerate(SCRIPTS):
        for m in regex.finditer(r"\p{Script=%s}+" % name, assigned):
            for ch in m.group():
                out[ord(ch)] = k
    for c in range(MAX + 1):
        if cat[c] in ("Cn", "Cs"):
            out[c] = -1
    return out


def fold_orbits():
    parent = list(range(MAX + 1))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x

    for c in range(MAX + 1):
        if 0xD800 <= c <= 0xDFFF or c in (0x130, 0x131):
            continue
        ch = chr(c)
        for m in (ch.lower(), ch.upper()):
            if len(m) == 1 and ord(m) != c and ord(m) not in (0x130, 0x131):
                ra, rb = find(c), find(ord(m))
                if ra != rb:
                    parent[max(ra, rb)] = min(ra, rb)
    orbits = {}
    for c in range(MAX + 1):
        orbits.setdefault(find(c), []).append(c)
    return sorted(v for v in orbits.values() if len(v) > 1)


def ranges(pred):
    out, start = [], None
    for c in range(MAX + 2):
        ok = c <= MAX and pred(c)
        if ok and start is None:
            start = c
        elif not ok and start is not None:
            out.append((start, c - 1))
            start = None
    return out


def write_product(cat, scr, orb):
    two = sorted({c for c in cat if c != "Cn"})
    tables = {c: ranges(lambda r, c=c: cat[r] == c) for c in two}
    for k in "CLMNPSZ":
        s = {c for c in two if c[0] == k}
        tables[k] = ranges(lambda r, s=s: cat[r] in s)
    stables = {n: ranges(lambda r, k=k: scr[r] == k) for k, n in enumerate(SCRIPTS)}
    with open(OUT, "w") as f:
        f.write("// nakama_amd/csrc/unicode_tables.h — GENERATED by tools/gen_unicode_tables.py\n")
        f.write("// (Unicode %s, the version of the reference's Go 1.20 unicode package).\n" % unicodedata.unidata_version)
        f.write("// Data only: general-category and script rune ranges and simple\n")
        f.write("// case-folding orbits for the product's regexp matcher (termmatch.cpp).\n")
        f.write("#pragma once\n#include <cstdint>\n#include <cstring>\n\nnamespace uni {\n\n")
        f.write("struct Range { uint32_t lo, hi; };\n")
        names = sorted(tables)
        for n in names:
            f.write("static const Range k%s[] = {%s};\n" % (n, ",".join("{0x%X,0x%X}" % r for r in tables[n])))
        for n in SCRIPTS:
            f.write("static const Range kS_%s[] = {%s};\n" % (n, ",".join("{0x%X,0x%X}" % r for r in stables[n])))
        f.write("struct Category { const char* name; const Range* r; int n; };\n")
        f.write("static const Category kCategories[] = {\n")
        for n in names:
            f.write('    {"%s", k%s, %d},\n' % (n, n, len(tables[n])))
        f.write("};\n")
        f.write("static const Category kScripts[] = {\n")
        for n in SCRIPTS:
            f.write('    {"%s", kS_%s, %d},\n' % (n, n, len(stables[n])))
        f.write("};\n")
        f.write("// regexp/syntax unicodeTable: unicode.Categories first, then unicode.Scripts\n")
        f.write("inline const Category* category(const char* name, size_t len) {\n")
        f.write("    for (const Category& c : kCategories)\n")
        f.write("        if (std::strlen(c.name) == len && std::memcmp(c.name, name, len) == 0) return &c;\n")
        f.write("    for (const Category& c : kScripts)\n")
        f.write("        if (std::strlen(c.name) == len && std::memcmp(c.name, name, len) == 0) return &c;\n")
        f.write("    return nullptr;\n}\n\n")
        flat, starts = [], []
        for o in orb:
            starts.append(len(flat))
            flat.extend(o)
        starts.append(len(flat))
        idx = sorted((r, i) for i, o in enumerate(orb) for r in o)
        f.write("// orbits of size > 1: members ascending, kOrbitStart[i]..kOrbitStart[i+1]\n")
        f.write("static const uint32_t kOrbitRunes[] = {%s};\n" % ",".join("0x%X" % r for r in flat))
        f.write("static const uint16_t kOrbitStart[] = {%s};\n" % ",".join(str(s) for s in starts))
        f.write("static const uint32_t kFoldRune[] = {%s};  // ascending\n" % ",".join("0x%X" % r for r, _ in idx))
        f.write("static const uint16_t kFoldOrbit[] = {%s};\n" % ",".join(str(i) for _, i in idx))
        f.write("static const int kFoldCount = %d;\n" % len(idx))
        f.write("\n}  // namespace uni\n")


def write_oracle(cat, scr, orb):
    cats = sorted(set(cat))  # two-letter, Cn included (a run's category)
    runs = []
    for c in range(MAX + 1):
        key = (cats.index(cat[c]), scr[c] + 1)
        if runs and runs[-1][2] == key and runs[-1][1] == c - 1:
            runs[-1][1] = c
        else:
            runs.append([c, c, key])
    nxt = []  # SimpleFold: the next rune of the orbit, wrapping to the smallest
    for o in orb:
        for k, r in enumerate(o):
            nxt.append((r, o[(k + 1) % len(o)]))
    nxt.sort()
    with open(OUT_ORACLE, "w") as f:
        f.write("// oracle/unicode_ref.h — TEST INFRASTRUCTURE ONLY; GENERATED by\n")
        f.write("// tools/gen_unicode_tables.py (Unicode %s) in a layout of its own, so the\n" % unicodedata.unidata_version)
        f.write("// oracle shares no table with the product (nakama_amd/csrc/unicode_tables.h):\n")
        f.write("// every rune's (general category, script) as sorted runs, and Go's\n")
        f.write("// unicode.SimpleFold as (rune, next rune of its orbit) pairs.\n")
        f.write("#pragma once\n#include <cstdint>\n\nnamespace uref {\n\n")
        f.write("static const char* const kCatName[] = {%s};\n" % ",".join('"%s"' % c for c in cats))
        f.write("static const int kNCat = %d;\n" % len(cats))
        f.write("// script 0: none (unassigned, private use, surrogates)\n")
        f.write("static const char* const kScriptName[] = {\"\",%s};\n" % ",".join('"%s"' % s for s in SCRIPTS))
        f.write("static const int kNScript = %d;\n" % (len(SCRIPTS) + 1))
        f.write("struct Run { uint32_t lo, hi; uint8_t cat, script; };\n")
        f.write("static const Run kRuns[] = {%s};\n" % ",".join("{0x%X,0x%X,%d,%d}" % (a, b, k[0], k[1]) for a, b, k in runs))
        f.write("static const int kNRuns = %d;\n" % len(runs))
        f.write("struct Fold { uint32_t r, next; };\n")
        f.write("static const Fold kSimpleFold[] = {%s};  // ascending r\n" % ",".join("{0x%X,0x%X}" % p for p in nxt))
        f.write("static const int kNFold = %d;\n" % len(nxt))
        f.write("\n}  // namespace uref\n")


def main():
    cat = category_of()
    scr = script_of(cat)
    orb = fold_orbits()
    write_product(cat, scr, orb)
    write_oracle(cat, scr, orb)
    print("orbits", len(orb), "folded runes", sum(len(o) for o in orb), "scripts", len(SCRIPTS))


if __name__ == "__main__":
    main()
