"""The Unicode data of both regexp matchers, checked entry by entry against
the interpreter's Unicode 13.0.0 database (the version of Go 1.20's unicode
package the reference builds with).

The product (nakama_amd/csrc/unicode_tables.h: per-name range lists, fold
orbits) and the oracle (oracle/unicode_ref.h: category/script runs, a
SimpleFold map) carry the data in different layouts, so the differential
regexp tests cannot pass on a table error both share; this test reads the two
headers as text and recomputes every category, script and case-folding orbit
here, independently of tools/gen_unicode_tables.py's code.
"""
import os
import re
import unicodedata

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRODUCT = os.path.join(ROOT, "nakama_amd", "csrc", "unicode_tables.h")
ORACLE = os.path.join(ROOT, "oracle", "unicode_ref.h")
MAX = 0x10FFFF

regex = pytest.importorskip("regex")


@pytest.fixture(scope="module")
def cats():
    assert unicodedata.unidata_version == "13.0.0"
    return [unicodedata.category(chr(c)) if not 0xD800 <= c <= 0xDFFF else "Cs" for c in range(MAX + 1)]


def _runs(flags):
    """Sorted [lo, hi] runs of the runes whose flag is set."""
    out, start = [], None
    for c, f in enumerate(flags + [False]):
        if f and start is None:
            start = c
        elif not f and start is not None:
            out.append((start, c - 1))
            start = None
    return out


def _ranges(text):
    return [(int(a, 16), int(b, 16)) for a, b in re.findall(r"\{0x([0-9A-F]+),0x([0-9A-F]+)\}", text)]


@pytest.fixture(scope="module")
def product_h():
    return open(PRODUCT).read()


@pytest.fixture(scope="module")
def oracle_h():
    return open(ORACLE).read()


def test_product_categories(cats, product_h):
    tables = dict(re.findall(r"static const Range k([A-Z][a-z]?)\[\] = \{(.*?)\};", product_h))
    two = sorted({c for c in cats if c != "Cn"})
    assert sorted(k for k in tables if len(k) == 2) == two  # Go has no Cn table
    for name, body in tables.items():
        members = {name} if len(name) == 2 else {c for c in two if c[0] == name}
        assert _ranges(body) == _runs([c in members for c in cats]), name


def _script_flags(cats, name):
    assigned = "".join(chr(c) for c in range(MAX + 1) if cats[c] not in ("Cn", "Cs"))
    flags = [False] * (MAX + 1)
    for m in regex.finditer(r"\p{Script=%s}" % name, assigned):
        flags[ord(m.group())] = True
    return flags


def test_product_scripts(cats, product_h):
    tables = dict(re.findall(r"static const Range kS_(\w+)\[\] = \{(.*?)\};", product_h))
    assert len(tables) == 156  # Go 1.20 unicode.Scripts (Unicode 13.0.0)
    for name in ("Greek", "Latin", "Han", "Cyrillic", "Common", "Inherited", "Arabic", "Yezidi", "Khitan_Small_Script"):
        assert _ranges(tables[name]) == _runs(_script_flags(cats, name)), name
    # every assigned, non-private rune has exactly one script
    seen = [0] * (MAX + 1)
    for body in tables.values():
        for a, b in _ranges(body):
            for c in range(a, b + 1):
                seen[c] += 1
    for c in range(MAX + 1):
        want = 0 if cats[c] in ("Cn", "Cs", "Co") else 1
        assert seen[c] == want, hex(c)


def _orbits():
    """Simple case-folding orbits: the closure of one-to-one lower/upper
    mappings, U+0130 / U+0131 alone (Go's caseOrbit)."""
    adj = {}
    for c in range(MAX + 1):
        if 0xD800 <= c <= 0xDFFF or c in (0x130, 0x131):
            continue
        for m in (chr(c).lower(), chr(c).upper()):
            if len(m) == 1 and ord(m) != c and ord(m) not in (0x130, 0x131):
                adj.setdefault(c, set()).add(ord(m))
                adj.setdefault(ord(m), set()).add(c)
    seen, out = set(), []
    for c in sorted(adj):
        if c in seen:
            continue
        stack, orb = [c], set()
        while stack:
            x = stack.pop()
            if x in orb:
                continue
            orb.add(x)
            stack.extend(adj.get(x, ()))
        seen |= orb
        out.append(sorted(orb))
    return sorted(out)


def test_product_fold_orbits(product_h):
    runes = [int(x, 16) for x in re.search(r"kOrbitRunes\[\] = \{(.*?)\};", product_h).group(1).split(",")]
    starts = [int(x) for x in re.search(r"kOrbitStart\[\] = \{(.*?)\};", product_h).group(1).split(",")]
    got = sorted(runes[starts[k]:starts[k + 1]] for k in range(len(starts) - 1))
    assert got == _orbits()
    assert sorted(map(len, got))[-1] >= 3  # e.g. k K U+212A
    assert [0x4B, 0x6B, 0x212A] in got and [0x130] not in got


def test_oracle_runs(cats, oracle_h):
    cat_names = re.findall(r'"(\w\w)"', re.search(r"kCatName\[\] = \{(.*?)\};", oracle_h).group(1))
    scr_names = [""] + re.findall(r'"(\w+)"', re.search(r"kScriptName\[\] = \{\"\",(.*?)\};", oracle_h).group(1))
    runs = [(int(a, 16), int(b, 16), int(c), int(d))
            for a, b, c, d in re.findall(r"\{0x([0-9A-F]+),0x([0-9A-F]+),(\d+),(\d+)\}",
                                         re.search(r"kRuns\[\] = \{(.*?)\};", oracle_h).group(1))]
    assert runs[0][0] == 0 and runs[-1][1] == MAX
    for (a, b, _, _), (c, _, _, _) in zip(runs, runs[1:]):
        assert c == b + 1
    got_cat = [None] * (MAX + 1)
    got_scr = [None] * (MAX + 1)
    for a, b, c, s in runs:
        for r in range(a, b + 1):
            got_cat[r] = cat_names[c]
            got_scr[r] = scr_names[s]
    assert got_cat == cats
    for name in ("Greek", "Latin", "Han", "Common", "Inherited", "Devanagari"):
        flags = _script_flags(cats, name)
        assert [got_scr[r] == name for r in range(MAX + 1)] == flags, name
    assert all(got_scr[r] == "" for r in range(MAX + 1) if cats[r] in ("Cn", "Cs", "Co"))


def test_oracle_simple_fold(oracle_h):
    pairs = [(int(a, 16), int(b, 16)) for a, b in
             re.findall(r"\{0x([0-9A-F]+),0x([0-9A-F]+)\}", re.search(r"kSimpleFold\[\] = \{(.*?)\};", oracle_h).group(1))]
    nxt = dict(pairs)
    for orb in _orbits():
        for k, r in enumerate(orb):  # unicode.SimpleFold: the next larger orbit member, wrapping
            assert nxt[r] == orb[(k + 1) % len(orb)], hex(r)
    assert len(nxt) == sum(len(o) for o in _orbits())
