"""CPU-side checks of the drop-in boundary (no GPU needed).

* the HIP library loads and exports every entry point include/nakama_mm.h
  declares (and the oracle exports the same set);
* the product's query compiler accepts/rejects exactly what the reference
  parser does (the oracle's restatement of query_string, pinned by the
  known-answer fixtures), over the fixture cases and a seeded fuzz corpus;
* the product's groupIndexes restatement reproduces TestGroupIndexes exactly.
"""
import os
import random
import re

import pytest

import harness
from nakama_amd import capi

HEADER = os.path.join(harness.ROOT, "include", "nakama_mm.h")


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mm_[a-z_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def product():
    import __graft_entry__  # noqa: F401
    if not os.path.exists(harness.PRODUCT_SO):
        __graft_entry__.build()
    return capi.load_library(harness.PRODUCT_SO)


def test_cluster_header_symbols_exported(product):
    """include/nakama_cluster.h: the multi-GPU front's host entry points."""
    from nakama_amd import cluster
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(harness.ROOT, "include", "nakama_cluster.h")).read(), flags=re.S)
    syms = sorted(set(re.findall(r"\b(mm_[a-z_]+)\s*\(", txt)))
    assert set(syms) == set(cluster.CLUSTER_SYMBOLS)
    for s in syms:
        assert hasattr(product, s), f"libnakama_mm.so does not export {s}"


def test_header_symbols_exported(product):
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(product, s), f"libnakama_mm.so does not export {s}"
        assert hasattr(harness.oracle_lib(), s), f"oracle does not export {s}"
    assert set(syms) == set(capi.EXPORTED_SYMBOLS)
    assert product.mm_backend_name() == b"hip-gfx950"
    assert product.mm_abi_version() == 4


def test_library_is_gfx950(product):
    # the shared object embeds a gfx950 code object (clang offload bundle)
    blob = open(harness.PRODUCT_SO, "rb").read()
    assert b"gfx950" in blob


def _fuzz_corpus(n=3000, seed=7):
    rnd = random.Random(seed)
    atoms = ["properties.a", "properties.skill", "min_count", "party_id", "a", "5", "-", "+", ":", ">", "<", "=", ">=",
             "<=", "^2", "^", "^0.5", "^x", "~", "~2", "\"x y\"", "\"2021-01-01T00:00:00Z\"", "\\:", "\\ ", "\\x",
             "10", "-3.5", "1.2.3", "foo", "bar*", "/re/", " ", "  ", "\t", "é", "\xff", "/(/", "/a|b/", "/[a-/",
             "/\\pL/", "/(?i)a/", "/x{2}/", "~1.5", "~-1", "~3", "ba?r", "/\\w+/", "/a$/"]
    out = []
    for _ in range(n):
        k = rnd.randint(1, 7)
        out.append("".join(rnd.choice(atoms) for _ in range(k)))
    return out


def test_compile_status_matches_oracle(product):
    orc = harness.oracle_lib()
    # numbers the parser's integer fast path takes (<= 15 digits after a
    # sign) and the forms next to it that go through the general parse
    nums = ["0", "00", "007", "-0", "+0", "-7", "+7", "123456789012345", "1234567890123456", "99999999999999999999",
            "1_000", "0x10", "0x1p3", "1e3", "1.", ".5", "-", "+", "--1", "1-", "12a", "٣"]
    cases = [q for q, _ in harness.load_known_answer()["query_cases"]] + _fuzz_corpus()
    for x in nums:
        cases += [x, "properties.skill:" + x, "properties.skill:>=" + x, "properties.skill:<" + x + "^2",
                  "+properties.a:" + x + " properties.b:>" + x]
    bad = []
    for q in cases:
        b = q.encode("utf-8", "surrogateescape")
        a, o = product.mm_debug_compile(b), orc.mm_debug_compile(b)
        if a != o:
            bad.append((q, a, o))
    assert not bad, bad[:20]


def test_group_indexes_product(product):
    gi = harness.load_known_answer()["group_indexes"]
    names = [x[0] for x in gi["indexes"]]
    got = capi.group_indexes(product, [x[1] for x in gi["indexes"]], [x[2] for x in gi["indexes"]], gi["required"])
    assert [[[names[i] for i in idx], avg] for idx, avg in got] == [[list(g), a] for g, a in gi["expected"]]


def test_group_indexes_random_vs_oracle(product):
    rnd = random.Random(11)
    for _ in range(200):
        n = rnd.randint(0, 9)
        counts = [rnd.randint(1, 4) for _ in range(n)]
        created = [rnd.randint(0, 1 << 62) for _ in range(n)]  # large values exercise int64 wrap
        req = rnd.randint(0, 6)
        assert capi.group_indexes(product, counts, created, req) == \
            capi.group_indexes(harness.oracle_lib(), counts, created, req)


def test_product_fails_loudly_without_device():
    """No CPU fallback: creating a handle without a gfx950 device raises."""
    import nakama_amd
    try:
        import torch  # noqa: F401
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(capi.ErrDevice):
        nakama_amd.LocalMatchmaker()


def test_term_cases_product(product):
    """The product's matchers reproduce the fixture term cases (CPU only)."""
    for kind, pattern, fz, term, want in harness.load_known_answer()["term_cases"]:
        got = harness.term_match(product, kind, pattern, fz, term)
        if isinstance(want, list):
            assert got[0] == want[0] and got[1] == want[1] or abs(got[1] - want[1]) <= 1e-15, (pattern, term, got)
        else:
            assert got == want, (pattern, term, got)


# Go 1.20 regexp/syntax semantics of flags, POSIX and Unicode classes and case
# folding (parse.go parsePerlFlags / parseNamedClass / parseUnicodeClass,
# appendFoldedRange; unicode.SimpleFold orbits, Unicode 13.0), derived by hand:
# (pattern, term, expected) with expected True/False (whole-term match),
# "search_error" or "unsupported".
GO_REGEXP_CASES = [
    ("(?i)k", "k", True), ("(?i)k", "K", True), ("(?i)k", "\u212a", True), ("(?i)k", "x", False),
    ("k", "K", False), ("(?i)ß", "\u1e9e", True), ("(?i)σ+", "Σσς", True), ("(?i)[a-c]+", "AbC", True),
    ("(?i)\\w", "\u212a", True), ("(?i)\\w", "\u017f", True), ("\\w", "\u212a", False), ("(?i)\\W", "\u212a", False),
    ("(?i)[^k]", "\u212a", False), ("(?i)é", "É", True), ("(?i)i", "\u0130", False), ("(?i)i", "\u0131", False),
    ("(?s).", "\n", True), (".", "\n", False), ("a(?i)b", "aB", True), ("a(?i)b", "AB", False),
    ("(?i:a)b", "Ab", True), ("(?i:a)b", "AB", False), ("(?i)a|b", "B", True), ("((?i)a)b", "AB", False),
    ("(?i-s:a.)", "A\n", False), ("(?s-i:A.)", "A\n", True), ("(?)a", "a", True), ("(?m)a", "a", True),
    ("[[:alpha:]]+", "abcXYZ", True), ("[[:alpha:]]+", "ab1", False), ("[[:^digit:]]", "a", True),
    ("[[:^digit:]]", "5", False), ("(?i)[[:upper:]]", "q", True), ("[[:upper:]]", "q", False),
    ("[[:word:][:punct:]]+", "a_!", True), ("[[:foo:]]", "a", "search_error"), ("[[:alpha:]", "a", "search_error"),
    ("\\pL+", "héllo", True), ("\\pL+", "Ωμέγα", True), ("\\pL+", "h3", False), ("\\p{Lu}\\p{Ll}+", "Hello", True),
    ("\\p{Lu}\\p{Ll}+", "hello", False), ("\\PL", "3", True), ("\\p{^L}", "3", True), ("\\P{^L}", "x", True),
    ("\\pN", "\u0663", True), ("\\p{Nd}", "\u2167", False), ("\\p{Nl}", "\u2167", True), ("[\\pL\\d]+", "a1b2", True),
    ("\\p{Any}+", "a\n", True), ("(?i)\\p{Lu}", "a", True), ("\\p{Lu}", "a", False),
    ("(?i-)a", "a", "search_error"),
    # Go's unicode.Scripts after its Categories (unicodeTable); FoldScript under (?i)
    ("\\p{Greek}", "α", True), ("\\p{Greek}", "a", False), ("\\p{Greek}+", "Ωμέγα", True),
    ("\\p{Greek}", "\u00b5", False), ("(?i)\\p{Greek}", "\u00b5", True), ("\\P{Greek}", "\u00b5", True),
    ("\\p{Latin}+", "héllo", True), ("\\p{Han}", "中", True), ("\\p{Cyrillic}\\p{Latin}", "жa", True),
    ("\\p{Common}", "1", True), ("\\p{Inherited}", "\u0301", True), ("[\\p{Greek}\\p{Latin}]+", "aβc", True),
    ("\\p{greek}", "α", "search_error"), ("\\p{Foo}", "a", "search_error"), ("\\p{Cn}", "a", "search_error"),
    ("\\p{Cypro_Minoan}", "a", "search_error"),  # a Unicode 14 script: not in Go 1.20
    # (?U): NonGreedy stamped on every later node; vellum rejects each (ErrNoLazy)
    ("(?U)a", "a", "search_error"), ("(?U)", "", True), ("a(?U)", "a", True), ("(?U:)a", "a", True),
    ("(?U)(?-U)a", "a", True), ("(?U:a)", "a", "search_error"), ("(?U)()", "", "search_error"),
    ("(?U:(?-U:a+))", "aa", True), ("a*?", "a", "search_error"),
    ("(?x)a", "a", "search_error"), ("(?P=n)", "a", "search_error"), ("\\p{", "a", "search_error"),
]


def test_go_regexp_flag_and_class_cases(product):
    """Flags (?i) (?s) (?m), POSIX [:classes:], Unicode \\p classes and case
    folding: hand-derived Go semantics, product and oracle alike."""
    orc = harness.oracle_lib()
    for pat, term, want in GO_REGEXP_CASES:
        for lib in (product, orc):
            got = harness.term_match(lib, 1, pat, 0, term)
            if isinstance(want, bool):
                assert isinstance(got, list) and bool(got[0]) == want, (pat, term, got, want)
            else:
                assert got == want, (pat, term, got, want)


def _rand_regex(rnd, depth=0):
    atoms = ["a", "b", "c", ".", "[ab]", "[^a]", "[a-c]", "\\d", "\\w", "\\s", "\\.", "x", "é", "-", "_", "{", "}",
             "(?i)", "(?s)", "(?-i)", "K", "k", "\u212a", "s", "ſ", "É", "σ", "Σ", "[[:alpha:]]", "[[:^lower:]]",
             "[[:punct:][:digit:]]", "\\pL", "\\PL", "\\p{Lu}", "\\p{^Ll}", "[\\pN_]", "\\W", "[^\\w]", "(?i:k)",
             "(?s:.)", "\\p{Greek}", "\\P{Latin}", "[\\p{Greek}x]", "(?U)", "(?-U)", "(?U:)", "α", "Ω"]
    parts = []
    for _ in range(rnd.randint(0, 4)):
        r = rnd.random()
        if r < 0.15 and depth < 3:
            a = "(" + _rand_regex(rnd, depth + 1) + ")"
        elif r < 0.2 and depth < 3:
            a = "(?:" + _rand_regex(rnd, depth + 1) + "|" + _rand_regex(rnd, depth + 1) + ")"
        else:
            a = rnd.choice(atoms)
        q = rnd.random()
        if q < 0.15: a += "*"
        elif q < 0.25: a += "+"
        elif q < 0.32: a += "?"
        elif q < 0.38: a += rnd.choice(["{2}", "{1,2}", "{0,}", "{3,1}", "{,2}", "*?", "**"])
        parts.append(a)
    s = "".join(parts)
    if rnd.random() < 0.1:
        s += rnd.choice(["|", "(", ")", "[", "\\", "$", "^"])
    return s


def test_regexp_differential_vs_oracle(product):
    """Product Pike VM vs the oracle's end-position-set matcher on random
    patterns and terms: same parse status, same acceptance."""
    rnd = random.Random(5)
    orc = harness.oracle_lib()
    alphabet = ["a", "b", "c", "x", ".", "1", "_", " ", "\n", "é", "-", "A", "K", "k", "\u212a", "ſ", "S", "É", "σ",
                "ς", "Σ", "!", "٣", "α", "Ω", "\u00b5", "ж"]
    bad = []
    for _ in range(1500):
        pat = _rand_regex(rnd)
        for _ in range(6):
            term = "".join(rnd.choice(alphabet) for _ in range(rnd.randint(0, 6)))
            a = harness.term_match(product, 1, pat, 0, term)
            o = harness.term_match(orc, 1, pat, 0, term)
            if a != o:
                bad.append((pat, term, a, o))
    assert not bad, bad[:10]


def test_fuzzy_differential_vs_oracle(product):
    rnd = random.Random(9)
    orc = harness.oracle_lib()
    alphabet = ["a", "b", "c", "é"]
    bad = []
    for _ in range(3000):
        p = "".join(rnd.choice(alphabet) for _ in range(rnd.randint(1, 6)))
        t = "".join(rnd.choice(alphabet) for _ in range(rnd.randint(0, 7)))
        fz = rnd.randint(1, 2)
        a, o = harness.term_match(product, 2, p, fz, t), harness.term_match(orc, 2, p, fz, t)
        if a != o:
            bad.append((p, t, fz, a, o))
    assert not bad, bad[:10]
